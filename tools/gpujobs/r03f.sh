# round 3, job f: (1) RCCL's detected topology (2 ranks on one GPU, distinct
# NCCL_HOSTID); (2) packet mode (burst per-LTU calls) vs the CPU reference
# loop on this host.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03f
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 120 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 65536 --iters 0 \
  --algo Ring --env NCCL_TOPO_DUMP_FILE=$OUT/topo.xml --env NCCL_DEBUG_SUBSYS=INIT,GRAPH,ENV \
  --log-dir $OUT/log --out $OUT/run.json > $OUT/run.stdout 2>&1
rc=$?
echo "topo rc=$rc"
case $rc in 124|137|134|139) exit $rc;; esac
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/packet_mode_vs_cpu.py $OUT/packet_mode_vs_cpu.json > $OUT/packet.log 2>&1
echo "packet rc=$?"
tail -30 $OUT/packet.log
