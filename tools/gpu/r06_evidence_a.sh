# round-6 evidence, part A: every GPU test (-> gpurun_out/plane_report_gpu.json), then smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06}; mkdir -p $O; cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 30
exit 0
