set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ay
mkdir -p $OUT
timeout -k 10 120 python -u -m pytest -v --timeout 100 --timeout-method thread -m gpu tests/test_client_gpu.py -k waits_for -p tools.debug.noready > $OUT/noready.log 2>&1
rc=$?; echo "noready rc=$rc" >> $OUT/noready.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
