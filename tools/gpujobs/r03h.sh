# round 3, job h: CollNetDirect with GPU-direct collnet buffers (last RCCL
# CollNet experiment: does the proxy post iallreduce then?).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03h
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 80 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 1 --timeout 60 \
  --env SWITCHML_COLLNET_TRACE=1 --env NCCL_NET_GDR_LEVEL=SYS --env RCCL_FORCE_ENABLE_GDRDMA=1 \
  --env NCCL_DEBUG_SUBSYS=INIT,NET,GRAPH,ENV,COLL,PROXY \
  --log-dir $OUT/log --out $OUT/run.json 2>&1 | tee $OUT/run.stdout | grep -v "^ \|^{\|^}"
echo "rc=$?"
