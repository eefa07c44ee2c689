# round 4, job r: K1 / K3 / K2 input loads as buffer loads with explicit
# cache-policy bits (nt, sc0 nt, sc1 nt, sc0 sc1 nt) vs global nt loads,
# cold buckets, interleaved builds; frames tx on the same builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04r
mkdir -p $OUT
AB=p4app-switchml_amd/bin/ab
AB_KINDS=K1,K3,K2 timeout -k 10 500 python -u tools/ab_libs_cold.py $AB/ldbase.so $AB/ld2.so $AB/ld3.so $AB/ld18.so $AB/ld19.so \
  > $OUT/ab_ldpol.json 2> $OUT/ab_ldpol.err
rc=$?; echo "ab libs rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/ab_frames_libs.py $AB/ldbase.so $AB/ld2.so $AB/ld3.so $AB/ld18.so $AB/ld19.so \
  > $OUT/ab_frames_ldpol.json 2> $OUT/ab_frames_ldpol.err
echo "ab frames rc=$?"
