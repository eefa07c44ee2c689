# round 4: jobs c then b in one box session (see r04c.sh, r04b.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpujobs/r04c.sh && bash tools/gpujobs/r04b.sh
