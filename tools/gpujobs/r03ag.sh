# round 3, job ag: the push form with the multicast pushed too of the in-node switch — xgmi tests (pull and
# push, W up to 5 on one GPU), then the N>1 rehearsals with the new field.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03ag
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_xgmi_switch.py \
  > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 550 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-rccl-collnet \
  > $OUT/rehearse_2_full.json 2> $OUT/rehearse_2_full.err
rc=$?; echo "rehearse 2 rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 8 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_8.json 2> $OUT/rehearse_8.err
rc=$?; echo "rehearse 8 rc=$rc"
