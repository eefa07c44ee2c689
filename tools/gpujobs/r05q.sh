# round 5, job q: where configs[4]'s device iteration goes — bin/collnet_bench
# (the CollNet table driven in RCCL's proxy order, 4 ResNet-50 buckets in
# flight) plain, then under a rocprofv3 kernel trace (launches per iteration,
# kernel time vs the iteration).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05q
mkdir -p $OUT
export SWITCHML_CONFIG_INI="$(printf '[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\nmax_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\n')"
export SWITCHML_COLLNET_LOOPBACK=1
EXE=$GRAFT_REPO_ROOT/p4app-switchml_amd/bin/collnet_bench
PLUG=$GRAFT_REPO_ROOT/p4app-switchml_amd/switchml_amd/librccl-net-switchml.so
timeout -k 10 120 $EXE 50 $PLUG > $OUT/plain.json 2> $OUT/plain.err || exit $?
tail -1 $OUT/plain.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $EXE 50 $PLUG > $OUT/kt.log 2>&1 || exit $?
tail -1 $OUT/kt.log
