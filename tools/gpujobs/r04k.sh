# round 4, job k: K1/K3/K2 with the first tile's loads issued before the
# workgroup's scale-table build (SML_LUT_EARLY=1) vs after (0), cold A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 400 python -u tools/ab_libs_cold.py p4app-switchml_amd/bin/ab/lut_early0.so \
  p4app-switchml_amd/bin/ab/lut_early1.so > $OUT/ab_lut_early.json 2> $OUT/ab_lut_early.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_lut_early.json; tail -3 $OUT/ab_lut_early.err
