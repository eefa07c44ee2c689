# round 4, job l: K4 and the fused round trip with the first tile's loads
# issued before the scale-table build (SML_LUT_EARLY2=1) vs after, cold A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04l
mkdir -p $OUT
AB_KINDS=K4,RT timeout -k 10 400 python -u tools/ab_libs_cold.py p4app-switchml_amd/bin/ab/early2_0.so \
  p4app-switchml_amd/bin/ab/early2_1.so > $OUT/ab_lut_early2.json 2> $OUT/ab_lut_early2.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_lut_early2.json; tail -3 $OUT/ab_lut_early2.err
