#!/bin/bash
# Collect the rocprofv3 evidence for the bench's dominant kernel on a GPU box.
#   1) kernel trace + stats (durations)      -> gpurun_out/prof_<tag>/kt
#   2) PMC pass FETCH_SIZE (own pass)        -> gpurun_out/prof_<tag>/pmc_fetch
#   3) PMC pass WRITE_SIZE (own pass)        -> gpurun_out/prof_<tag>/pmc_write
# FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950 (TCC slots), and
# --pmc is never combined with sys/runtime/hip traces (gpurun refuses that).
set -uo pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# a step that times out, aborts or faults ends the GPU work of this run
step() { "$@"; rc=$?; case $rc in 124|137|134|139) echo "step failed rc=$rc: $*"; exit $rc;; esac; }
# kernel-trace pass: the bench's own defaults (50 ms settle, 500 warmup steps)
# and 2000 timed steps, so the average is dominated by steady-state launches;
# collect_pmc.py also reports the average over the timed window alone.  The
# strong_1GiB reading runs too (its own grid: collect_pmc.py reports each
# grid's launches apart, so the two readings' K1 launches are never mixed).
KT_ARGS="$ROOT/bench.py --steps 2000 --no-cpu-baseline --no-side --no-rccl-collnet"
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 $KT_ARGS > "$OUT/kt.log" 2>&1
# PMC passes: bytes per launch do not depend on clocks; few launches suffice
ARGS="$ROOT/bench.py --steps 20 --warmup 5 --settle-ms 0 --job-numel 0 --no-cpu-baseline --no-side --no-rccl-collnet"
step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- python3 $ARGS > "$OUT/pmc_fetch.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- python3 $ARGS > "$OUT/pmc_write.log" 2>&1
# the bench's default steps cycle 4 distinct buckets (HBM proper); the
# resident side number re-reads one bucket (HBM + Infinity Cache)
RARGS="$ARGS --buckets 1"
step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/res_fetch" -o pmc --output-format csv -- python3 $RARGS > "$OUT/res_fetch.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/res_write" -o pmc --output-format csv -- python3 $RARGS > "$OUT/res_write.log" 2>&1
# configs[3]'s per-GPU FIFO slices at N = 1, 2 and 8 (1 GiB, 512 and 128 MiB;
# N = 4's slice is the 256 MiB headline bucket): HBM bytes per launch for the
# strong_1GiB reading's roofline.traffic, the steps cycling 4 buckets as it does
for SN in 268435456 134217728 33554432; do
  SARGS="$ROOT/bench.py --numel $SN --steps 20 --warmup 5 --settle-ms 0 --job-numel 0 --no-cpu-baseline --no-side --no-rccl-collnet"
  step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/slice_${SN}_fetch" -o pmc --output-format csv -- python3 $SARGS > "$OUT/slice_${SN}_fetch.log" 2>&1
  step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/slice_${SN}_write" -o pmc --output-format csv -- python3 $SARGS > "$OUT/slice_${SN}_write.log" 2>&1
done
# F3 frames kernels (tx quantize-into-frames, rx claim/apply) on the same bucket
# (SKIP_FRAMES=1: leave them out — the frames kernels are unchanged since r05)
if [ "${SKIP_FRAMES:-0}" = 1 ]; then echo "profiles done (no frames): $OUT"; exit 0; fi
FR="$ROOT/tools/prof_frames.py"
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/fr_kt" -o kt --output-format csv -- python3 $FR > "$OUT/fr_kt.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fr_fetch" -o pmc --output-format csv -- python3 $FR > "$OUT/fr_fetch.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/fr_write" -o pmc --output-format csv -- python3 $FR > "$OUT/fr_write.log" 2>&1
echo "profiles done: $OUT"
