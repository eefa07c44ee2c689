set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/fr_kt -o kt --output-format csv -- python3 tools/prof_frames.py > $OUT/fr_kt.log 2>&1
