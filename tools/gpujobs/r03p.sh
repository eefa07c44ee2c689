# round 3, job p: the exchange burst with ProcessPacket fused for the pinned ring too (post of q + pre of q + b in one launch,
# ProcessPacket fused for the HBM ring): packet / client / plugin tests, then
# the packet-mode rate against the CPU reference loop.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_packets_gpu.py tests/test_client_gpu.py tests/test_capi_gpu.py tests/test_client_property_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 500 python -u tools/packet_mode_vs_cpu.py $OUT/packet_mode_vs_cpu.json > $OUT/packet.log 2>&1
rc=$?; echo "packet rc=$rc"; tail -30 $OUT/packet.log
