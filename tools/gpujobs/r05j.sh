# round 5, job j: the rocprofv3 evidence again on the current tree, now with
# K1's PMC passes at configs[3]'s per-GPU slice sizes (N = 2, 8) and the
# frames kernels on 4 cycled frame sets.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash profiles/run_profiles.sh r05
rc=$?; echo "profiles rc=$rc"
