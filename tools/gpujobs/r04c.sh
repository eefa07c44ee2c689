# round 4, job c: K1/K3/K2 tile-slice sweep on cold HBM now that 1- and
# 2-slice tiles also take non-temporal payload stores for planes >= 64 MiB
# (round 2's sweep ran them with default-policy stores only).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 400 python -u tools/sweep_cold.py > $OUT/sweep_p256.json 2> $OUT/sweep_p256.err
rc=$?; echo "sweep rc=$rc"; tail -c 1500 $OUT/sweep_p256.json
