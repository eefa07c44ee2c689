# round 5, job d: the adopted default-policy claim loads — frames tests,
# then the frames kernels under rocprofv3 on 4 cycled (cold) frame sets:
# kernel trace + separate FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_frames.py tests/test_frames_rx.py tests/test_nt_store_boundaries.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
FR="$GRAFT_REPO_ROOT/tools/prof_frames.py"
P=$GRAFT_REPO_ROOT/gpurun_out/prof_r05fr
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/fr_kt -o kt --output-format csv -- python3 $FR > $P/fr_kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $P/fr_fetch -o pmc --output-format csv -- python3 $FR > $P/fr_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $P/fr_write -o pmc --output-format csv -- python3 $FR > $P/fr_write.log 2>&1 || exit $?
cat $P/fr_kt.log | tail -2
