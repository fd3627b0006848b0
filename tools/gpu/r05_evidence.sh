# round-5 evidence on the in-tree library: tools/profile_round.sh (GPU tests -> gpurun_out/plane_report_gpu.json,
# bench lines, rocprof, PMC, voxel passes), then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh ${1:-r05} ${2:-tests} || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${1:-r05}/smoke.log 2>&1 || exit 30
