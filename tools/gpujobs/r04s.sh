# round 4, job s: cache-policy bits through compiler-scheduled buffer ops
# (descriptor sign extension fixed): stores sc1 nt (SML_NT_CPOL=3), loads
# nt / sc0 nt (SML_LOAD_CPOL=2 / 3), both; vs the production build. Cold buckets.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04s
mkdir -p $OUT
AB=p4app-switchml_amd/bin/ab
AB_KINDS=K1,K3,K2,K4,RT timeout -k 10 500 python -u tools/ab_libs_cold.py $AB/base.so $AB/cpol3.so $AB/ld2.so $AB/ld3.so $AB/ld3cp3.so \
  > $OUT/ab_bufpol.json 2> $OUT/ab_bufpol.err
rc=$?; echo "ab libs rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/ab_frames_libs.py $AB/base.so $AB/ld2.so $AB/ld3.so \
  > $OUT/ab_frames_bufpol.json 2> $OUT/ab_frames_bufpol.err
echo "ab frames rc=$?"
