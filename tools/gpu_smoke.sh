# __graft_entry__.smoke() on the GPU box, as the driver runs it at round end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke/smoke.log 2>&1 || exit 11
