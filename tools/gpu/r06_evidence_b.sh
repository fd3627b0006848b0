# round-6 evidence, part B: tools/profile_round.sh without the tests (bench lines, rocprof, PMC, voxel, MSG, FPS phases)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh ${1:-r06} notests || exit $?
