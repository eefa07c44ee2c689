# round 4, job d: K1 tile-size A/B on the bench workload at the N = 8/4/2/1
# slice sizes (tools/ab_slices_nt.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_slices_nt.py > $OUT/ab_slices_nt.json 2> $OUT/ab_slices_nt.err
rc=$?; echo "ab rc=$rc"; tail -c 3000 $OUT/ab_slices_nt.json
