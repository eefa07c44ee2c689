set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bb
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python tools/ab_coalesce.py > $OUT/ab_coalesce.json 2> $OUT/ab_coalesce.err && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1
