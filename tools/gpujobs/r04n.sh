# round 4, job n: frames tx store policy on cold frame sets: default (nt0), non-temporal payload (nt1),
# non-temporal payload + header dwords (nt2).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 300 python -u tools/ab_frames_libs.py p4app-switchml_amd/bin/ab/frames_nt0.so \
  p4app-switchml_amd/bin/ab/frames_nt1.so p4app-switchml_amd/bin/ab/frames_nt2.so > $OUT/ab_frames_nt.json 2> $OUT/ab_frames_nt.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_frames_nt.json; tail -3 $OUT/ab_frames_nt.err
