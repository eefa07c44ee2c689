# K1 vs K3 counters, cold-HBM PMC traffic (item 6),
# the machine's CPU quota, counter list, and the new client GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02b
mkdir -p $OUT
export TMPDIR=/tmp
(cat /sys/fs/cgroup/cpu.max; cat /proc/self/cgroup; nproc) > $OUT/cpu_quota.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_client_gpu.py > $OUT/tests_client.log 2>&1 && \
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 ; \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 tools/prof_k3.py > $OUT/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_SALU -d $OUT/pmc_sq -o pmc --output-format csv -- python3 tools/prof_k3.py > $OUT/pmc_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o pmc --output-format csv -- python3 tools/prof_k3.py > $OUT/pmc_tcc.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 tools/prof_k3.py > $OUT/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- python3 tools/prof_k3.py > $OUT/pmc_write.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_grbm -o pmc --output-format csv -- python3 tools/prof_k3.py > $OUT/pmc_grbm.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cold_fetch -o pmc --output-format csv -- python3 bench.py --buckets 4 --steps 20 --warmup 8 --settle-ms 0 --no-cpu-baseline --no-side > $OUT/cold_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/cold_write -o pmc --output-format csv -- python3 bench.py --buckets 4 --steps 20 --warmup 8 --settle-ms 0 --no-cpu-baseline --no-side > $OUT/cold_write.log 2>&1
