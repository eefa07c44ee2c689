# round 3, job g: RCCL AllReduce as CollNetDirect into the plugin, with the
# switch node added to each one-GPU worker's topology (2 ranks on one GPU).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03g
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 90 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 3 --timeout 70 \
  --env SWITCHML_COLLNET_TRACE=1 --env NCCL_DEBUG_SUBSYS=INIT,NET,GRAPH,ENV,TUNING,COLL,PROXY \
  --log-dir $OUT/log --out $OUT/run.json 2>&1 | tee $OUT/run.stdout | grep -v "^ \|^{\|^}"
echo "rc=$?"
