# round 4, job n: frames tx with the first tile's loads before the scale
# table (frames_early1) vs the previous order (frames_early0), cold A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_frames_libs.py p4app-switchml_amd/bin/ab/frames_early0.so \
  p4app-switchml_amd/bin/ab/frames_early1.so > $OUT/ab_frames_early.json 2> $OUT/ab_frames_early.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_frames_early.json; tail -3 $OUT/ab_frames_early.err
