# round 4, job u: the N=2 / N=8 rehearsals over RCCL on the final kernels
# (sc1 nt stores).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04u
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_2.json 2> $OUT/rehearse_2.err
rc=$?; echo "rehearse 2 rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 8 --switch-numel 4194304 --steps 20 --warmup 5 \
  --no-rccl-collnet > $OUT/rehearse_8.json 2> $OUT/rehearse_8.err
rc=$?; echo "rehearse 8 rc=$rc"
