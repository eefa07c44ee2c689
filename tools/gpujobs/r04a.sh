# round 4, job a: the switch data path under RCCL on one GPU (2/3/8 ranks, one
# RCCL host each), the per-LTU refusal, the burst-server replay fix, the
# segment-mapping fixes (xgmi / plugin tests); then the N=2 rehearsal over
# RCCL and the N=1 bench (copy ceiling with K1's store policy).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_switch_rccl_gpu.py tests/test_per_ltu_policy.py tests/test_packets_gpu.py tests/test_xgmi_switch.py \
  tests/test_rccl_collnet.py tests/test_collnet_plugin.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 550 python -u bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_2.json 2> $OUT/rehearse_2.err
rc=$?; echo "rehearse 2 rc=$rc"; tail -c 600 $OUT/rehearse_2.err; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rccl-collnet > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"
