set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_kern.sh alone tools/ssg_alone.py || exit 11
