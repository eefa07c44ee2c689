# round 4, job ae: final kernels (batched round trip on 2-slice tiles too) — whole GPU suite, smoke, the driver's N=1 command, rocprofv3 evidence,
# bench --extra.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04ae
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 700 bash profiles/run_profiles.sh r04
rc=$?; echo "profiles rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet > $OUT/bench_extra.json 2> $OUT/bench_extra.err
echo "bench extra rc=$?"
