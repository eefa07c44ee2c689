# round 4, job c: K1/K3/K2 tile-slice sweep on cold HBM now that 1- and
# 2-slice tiles also take non-temporal payload stores for planes >= 64 MiB
# (round 2's sweep ran them with default-policy stores only).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_per_ltu_policy.py \
  > $OUT/tests_per_ltu.log 2>&1
rc=$?; echo "per-LTU tests rc=$rc"; tail -3 $OUT/tests_per_ltu.log; grep -h "registered ring" -r /tmp 2>/dev/null | head -2
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/sweep_cold.py > $OUT/sweep_p256.json 2> $OUT/sweep_p256.err
rc=$?; echo "sweep rc=$rc"; tail -c 1500 $OUT/sweep_p256.json
