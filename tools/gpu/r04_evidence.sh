# round-4 evidence on the in-tree library: tools/profile_round.sh (GPU tests, bench lines, rocprof, PMC,
# voxel passes), then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh ${1:-r04} tests || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${1:-r04}/smoke.log 2>&1 || exit 30
