set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bd
mkdir -p $OUT
SML_BENCH_REHEARSE=1 timeout -k 10 600 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 5 > $OUT/rehearse2.json 2> $OUT/rehearse2.err || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_collnet_plugin.py tests/test_switchsim_dist.py > $OUT/tests.log 2>&1 || exit $?
SWITCHML_COLLNET_LOOPBACK=1 SWITCHML_CONFIG_INI=$'[general]\nnum_workers = 8\nnum_worker_threads = 4\npacket_numel = 256\nmax_outstanding_packets = 256\n[backend.dummy]\nbandwidth = 0\n[backend.hip]\nmode = fused\n' timeout -k 10 120 ./p4app-switchml_amd/bin/collnet_bench 30 p4app-switchml_amd/switchml_amd/librccl-net-switchml.so > $OUT/collnet_bench.json 2> $OUT/collnet_bench.err
