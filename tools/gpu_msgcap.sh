set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mc; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 200 --timeout-method thread -k "msg or bq or backbone" > $O/tests.log 2>&1 || exit 11
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-density --no-cpu-baseline --no-fp32-mfma-leg > $O/bench.json 2> $O/bench.err || exit 12
