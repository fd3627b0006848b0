# Tier N GPU tests + the bench line at the driver's settings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04x}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --no-density --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit 13
