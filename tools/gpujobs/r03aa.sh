# round 3, job aa: 16-B packet accesses, op in the doorbell word, 8-B descriptor loads (packets in pinned host memory
# served by one resident workgroup polling a doorbell): packet / client tests,
# then packet mode with the pinned ring through it vs per-burst launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_packets_gpu.py tests/test_client_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u tools/packet_mode_vs_cpu.py $OUT/packet_mode_vs_cpu.json > $OUT/packet.log 2>&1
rc=$?; echo "packet rc=$rc"; grep -A3 '"packet' $OUT/packet_mode_vs_cpu.json | head -30
