set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02j
timeout -k 10 300 python tools/sweep_cold.py > gpurun_out/r02j/sweep_cold.json 2> gpurun_out/r02j/sweep_cold.err
