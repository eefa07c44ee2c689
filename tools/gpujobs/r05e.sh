# round 5, job e: frames rx on cold frame sets, the claim pass with
# returning atomics (accepted / discarded counters, base) vs non-returning
# (nocount: counters off) — what counting costs.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/ab_rx_libs_cold.py p4app-switchml_amd/bin/ab/base.so p4app-switchml_amd/bin/ab/nocount.so > $OUT/ab_rx_counts.json 2> $OUT/ab.err
rc=$?; echo "ab rc=$rc"; cat $OUT/ab_rx_counts.json
