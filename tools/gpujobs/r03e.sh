# round 3, job e: dump RCCL's detected topology (2 ranks on one GPU, distinct
# NCCL_HOSTID) to see where CollNetDirect's NVSwitch requirement comes from.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03e
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 120 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 65536 --iters 0 \
  --algo Ring --env NCCL_TOPO_DUMP_FILE=$OUT/topo.xml --env NCCL_DEBUG_SUBSYS=INIT,GRAPH,ENV \
  --log-dir $OUT/log --out $OUT/run.json > $OUT/run.stdout 2>&1
echo "rc=$?"
ls -la $OUT
