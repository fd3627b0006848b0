set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_n.py -x -q -k "dense or backbone or stream" --timeout 120 --timeout-method thread > gpurun_out/t8_tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/micro.py dense > gpurun_out/t8_dense.log 2>&1 || exit 12
timeout -k 10 200 python bench.py --no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg > gpurun_out/t8_bench.json 2> gpurun_out/t8_bench.err || exit 13
