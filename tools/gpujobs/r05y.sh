# round 5, job y: the one-pass INT32 rx (k_rx_int32 + fix-up): the INT32
# frames suite, then bench --extra's frames fields and a kernel trace of them
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_frames_int32.py tests/test_frames.py tests/test_frames_rx.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
grep "copies claimed ahead" $OUT/pytest.log | head -8
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet --no-side > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/r05y/bench.json").read().strip().splitlines()[-1])
print({k: v for k, v in b.get("extra", {}).items() if "frames" in k})
PY
