set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash profiles/run_profiles.sh r02
