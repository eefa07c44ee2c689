# round 3, job b: which RCCL algorithm setting dispatches AllReduce into the
# CollNet plugin (2 ranks on one GPU, distinct NCCL_HOSTID).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03b
mkdir -p $OUT
cd p4app-switchml_amd
for algo in CollNetDirect none; do
  a=$algo; [ "$algo" = none ] && a=""
  timeout -k 10 150 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 3 \
    --algo "$a" --log-dir $OUT/$algo --out $OUT/$algo.json 2>&1 | tee $OUT/$algo.stdout
  rc=$?
  echo "algo=$algo rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac   # a timeout / abort ends the GPU work of this call
done
