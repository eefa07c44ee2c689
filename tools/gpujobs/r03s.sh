# round 3, job s: exchange bursts under the dummy backend's random delivery.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03s
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_packets_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 $OUT/tests.log
