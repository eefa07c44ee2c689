# round 3, job c: RCCL AllReduce dispatched as CollNetDirect into the plugin
# (2 ranks on one GPU), then the GPU tests touched by the burst API, the
# packet loop, the xgmi hardening and the acquire/release flags.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03c
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 180 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 3 \
  --algo CollNetDirect --log-dir $OUT/rccl --out $OUT/rccl_collnet.json 2>&1 | tee $OUT/rccl_collnet.stdout
rc=$?
echo "rccl rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_packets_gpu.py tests/test_xgmi_switch.py tests/test_client_gpu.py tests/test_switch_gpu.py \
  > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -15 $OUT/tests.log
