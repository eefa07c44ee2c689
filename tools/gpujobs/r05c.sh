# round 5, job c: frames rx on cold frame sets, claim-pass header loads
# non-temporal (base) vs default policy (abv1: header lines kept in the
# caches for the apply pass, which reads the same lines for the payload).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_rx_libs_cold.py p4app-switchml_amd/bin/ab/base.so p4app-switchml_amd/bin/ab/nocount.so > $OUT/ab_rx_counts.json 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_rx_counts.json
