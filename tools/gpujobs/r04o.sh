# round 4, job o: frames tx with non-temporal payload stores — frames tests,
# the cold frames A/B on the in-tree library vs the committed default-policy
# build is not repeated; bench --extra (frames resident and 4-set cycling).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_frames.py \
  tests/test_frames_rx.py tests/test_launch_geometry.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet \
  > $OUT/bench_extra.json 2> $OUT/bench_extra.err
rc=$?; echo "bench extra rc=$rc"
PROBE_SET=cpol timeout -k 10 120 p4app-switchml_amd/bin/hbm_probe 1024 7 > $OUT/hbm_probe_cpol_1024MiB.json 2> $OUT/hbm_probe_cpol.err
echo "probe rc=$?"
