set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02as
mkdir -p $OUT
timeout -k 10 300 python -c "
import sys, json, torch; sys.path[:0]=['.', 'p4app-switchml_amd']
import bench
for i in range(5):
    r = bench.plugin_buckets(torch, torch.device('cuda:0'), iters=20)
    print(json.dumps({'device_ms': r['device']['ms_per_iteration'], 'pinned_ms': r['pinned_host']['ms_per_iteration']}), flush=True)
" > $OUT/plugin5.json 2> $OUT/plugin.err
