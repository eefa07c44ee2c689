# round 5, job m: the N=1 bench-line contract test after the hipGraph fix,
# and eager vs 20-step graphs with the driver's command (two processes each).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05m
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_bench_multi_gpu.py -k n1 > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
for i in 1 2; do
  for G in 1 20; do
    timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 20 --graph-steps $G --no-cpu-baseline --no-side --no-rccl-collnet > $OUT/bench_g${G}_$i.json 2> $OUT/bench_g${G}_$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_g${G}_$i.json').read().strip().splitlines()[-1]); print('G=$G run $i', d['value'], d['roofline']['frac'], d['self_check'])"
  done
done
