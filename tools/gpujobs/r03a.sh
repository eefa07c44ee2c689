# round 3, job a: RCCL dispatching CollNet all-reduces (2 ranks on one GPU,
# distinct NCCL_HOSTID), then the switch / plugin / bench-contract GPU tests
# after the acquire/release and ABI-2 changes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03a
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 300 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 3 \
  --log-dir $OUT/rccl --out $OUT/rccl_collnet.json 2>&1 | tee $OUT/rccl_collnet.stdout
rc=$?
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_switch_gpu.py tests/test_xgmi_switch.py tests/test_collnet_plugin.py tests/test_bench_contract.py \
  > $OUT/tests.log 2>&1
echo "rccl rc=$rc tests rc=$?"
tail -5 $OUT/tests.log
