# round 4: job j then job i in one box session (see r04j.sh, r04i.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpujobs/r04j.sh && bash tools/gpujobs/r04i.sh
