# round 4, first check: GPU suite, precision probe, bench line at the driver's settings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/precision_probe.py > $O/precision.log 2>&1 || exit 12
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit 13
