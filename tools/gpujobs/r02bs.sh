set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bs
mkdir -p $OUT
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-side --no-cpu-baseline > $OUT/b$i.json 2> $OUT/b$i.err || exit $?
done
