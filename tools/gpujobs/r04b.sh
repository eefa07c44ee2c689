# round 4, job b: (1) RCCL offered the CollNet table with CollNetChain (the
# r03a setting): RCCL's no-op vs the plugin driven by hand on a fresh copy;
# (2) bench --extra on this tree (H<->D-inclusive rates for DESIGN §7);
# (3) the driver's N=8 command rehearsed over RCCL with 8 ranks on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04b
mkdir -p $OUT
cd p4app-switchml_amd
timeout -k 10 200 python -u -m switchml_amd.rccl_collnet --world 2 --same-gpu --numel 4194304 --iters 0 \
  --algo CollNetChain --channels 1 --env SWITCHML_COLLNET_RCCL=1 --timeout 150 \
  --log-dir $OUT/chain --out $OUT/rccl_collnet_chain.json > $OUT/chain.stdout 2>&1
rc=$?; echo "chain rc=$rc"; grep -h "^\[rank" $OUT/chain.stdout | head; case $rc in 0|1) ;; *) exit $rc;; esac
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --extra --no-cpu-baseline --no-rccl-collnet \
  > $OUT/bench_extra.json 2> $OUT/bench_extra.err
rc=$?; echo "bench extra rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
SML_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 8 --switch-numel 4194304 --steps 20 --warmup 5 \
  > $OUT/rehearse_8.json 2> $OUT/rehearse_8.err
rc=$?; echo "rehearse 8 rc=$rc"
