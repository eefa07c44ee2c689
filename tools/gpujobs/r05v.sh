# round 5, job v: frames rx on cold frame sets, the adopted default-policy
# claim loads (cur) vs non-temporal ones (ntclaim), on one box: interleaved
# rounds and bench.py --extra's one-shot timing; then bench --extra's own rx fields.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05v
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_rx_libs_cold.py p4app-switchml_amd/bin/ab/cur.so p4app-switchml_amd/bin/ab/ntclaim.so > $OUT/ab.json 2> $OUT/ab.err || exit $?
cat $OUT/ab.json
