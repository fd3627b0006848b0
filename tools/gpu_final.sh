# final-tree check: the whole GPU suite, then the bench line at the driver's settings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 12
