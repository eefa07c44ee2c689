# round 3, job d: RCCL settings under which AllReduce reaches the CollNet
# plugin's iallreduce (2 ranks on one GPU, distinct NCCL_HOSTID).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03d
mkdir -p $OUT
cd p4app-switchml_amd
run() {
  name=$1; shift
  timeout -k 10 120 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 2 \
    --log-dir $OUT/$name --out $OUT/$name.json "$@" > $OUT/$name.stdout 2>&1
  rc=$?
  echo "$name rc=$rc"; grep -h "^\[rank" $OUT/$name.stdout | head -8
  case $rc in 124|137|134|139) exit $rc;; esac
}
run override --algo "" --env RCCL_OVERRIDE_ALGO=CollNetDirect --env RCCL_OVERRIDE_PROTO=Simple
run direct_simple --algo CollNetDirect --env NCCL_PROTO=Simple
run direct_ring --algo "CollNetDirect,Ring" --env NCCL_PROTO=Simple
