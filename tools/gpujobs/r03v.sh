# round 3, job v: the N = 8 slice (128 MiB of the 1 GiB job) on one GPU under
# grid-stride caps (sml_set_grid_limit): does a grid sized to the chip shorten
# the short launch's ramp-up / tail?
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03v
mkdir -p $OUT
for g in 0 1024 2048 4096 0; do
  timeout -k 10 300 python -u bench.py --numel 33554432 --grid-limit $g --steps 200 --warmup 50 --no-side --no-cpu-baseline --no-rccl-collnet \
    > $OUT/g$g.json 2> $OUT/g$g.err
  rc=$?; echo "grid $g rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
  python -c "
import json; t=open('$OUT/g$g.json').read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1]); print('grid $g', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
