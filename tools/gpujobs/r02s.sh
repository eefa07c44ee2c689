set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02s
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_frames.py > $OUT/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/prof_frames.py > $OUT/fetch.log 2>&1
