# round 4, job f: rocprofv3 evidence on the final K1 (kernel trace of the
# 2000-step bench + PMC passes; frames kernels) -> gpurun_out/prof_r04
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 bash profiles/run_profiles.sh r04
rc=$?; echo "profiles rc=$rc"
