# round 3, job l: rocprofv3 evidence of the final K1 instance (cycling
# buckets, non-temporal stores from 64 MiB), the N=1 bench with the copy
# ceiling, and the N>1 path rehearsed with 2 and 8 ranks on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03l
mkdir -p $OUT
bash profiles/run_profiles.sh r03 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
for n in 2 8; do
  SML_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus $n --switch-numel 4194304 --steps 20 --warmup 5 \
    > $OUT/rehearse_$n.json 2> $OUT/rehearse_$n.err
  rc=$?; echo "rehearse $n rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
done
