set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > gpurun_out/r02a_affinity.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_kat_gpu.py tests/test_collnet_plugin.py tests/test_golden_digests.py tests/test_client_gpu.py > gpurun_out/r02a_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02a_bench1.json 2> gpurun_out/r02a_bench1.err && \
SML_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --switch-numel 4194304 --steps 20 --warmup 20 > gpurun_out/r02a_bench2.json 2> gpurun_out/r02a_bench2.err && \
timeout -k 10 240 python tools/rccl_plugin_probe.py 1 > gpurun_out/r02a_probe.json 2>&1
