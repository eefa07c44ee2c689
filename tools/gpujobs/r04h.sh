# round 4, job h: K4 on 2-slice tiles by default and the copy probe in K1's
# tile shape — the kernel tests, the N=1 bench, then the rocprofv3 evidence.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_launch_geometry.py \
  tests/test_gpu_parity.py tests/test_golden_digests.py tests/test_kat_gpu.py tests/test_property_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-rccl-collnet > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
PROBE_SET=nt timeout -k 10 120 p4app-switchml_amd/bin/hbm_probe 1024 7 > $OUT/hbm_probe_nt_1024MiB.json 2> $OUT/hbm_probe.err
rc=$?; echo "probe rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 700 bash profiles/run_profiles.sh r04
rc=$?; echo "profiles rc=$rc"
