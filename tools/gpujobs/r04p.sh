# round 4, job p: nt store cache-policy bits (sc0 sc1 nt / sc1 nt vs nt) in
# K1 / K4 / round trip and frames tx, cold buckets, interleaved builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04p
mkdir -p $OUT
AB=p4app-switchml_amd/bin/ab
AB_KINDS=K1,K4,RT timeout -k 10 400 python -u tools/ab_libs_cold.py $AB/cpol0.so $AB/cpol1.so $AB/cpol2.so \
  > $OUT/ab_cpol.json 2> $OUT/ab_cpol.err
rc=$?; echo "ab libs rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/ab_frames_libs.py $AB/cpol0.so $AB/cpol1.so $AB/cpol2.so \
  > $OUT/ab_frames_cpol.json 2> $OUT/ab_frames_cpol.err
echo "ab frames rc=$?"
