#!/bin/bash
# A/B on the GPU box: GPU tests matching $TESTK on the in-tree lib, micro $MICRO and the headline
# bench (no extras) on ab/base vs the in-tree lib.  Every GPU step has its own limit; && chain.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
TAG=${1:-ab}
B=ab/${BASE:-base}/liblidar_amd.so
BA="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg ${BENCH_ARGS:-}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-fps}" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 11
if [ -n "$MICRO" ]; then
  timeout -k 10 200 python tools/micro.py $MICRO > gpurun_out/${TAG}_microB.log 2>&1 || exit 12
  LIDAR_AMD_LIB=$B timeout -k 10 200 python tools/micro.py $MICRO > gpurun_out/${TAG}_microA.log 2>&1 || exit 13
fi
timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_benchB.json 2> gpurun_out/${TAG}_benchB.err || exit 14
LIDAR_AMD_LIB=$B timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_benchA.json 2> gpurun_out/${TAG}_benchA.err || exit 15
timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_benchB2.json 2> gpurun_out/${TAG}_benchB2.err || exit 16
exit 0
