# round 4: job g then job e in one box session (see r04g.sh, r04e.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpujobs/r04g.sh && bash tools/gpujobs/r04e.sh
