#!/bin/bash
# A/B of one env knob on the GPU box: GPU tests matching $TESTK, then the bench with
# $KNOB=0 / 1 / 0 / 1 (same library).  Every GPU step has its own limit; && chain.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
TAG=${1:-envab}
BA="--no-density --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "${TESTK:-ball_query}" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 11
for i in 1 2; do
  for v in 0 1; do
    env $KNOB=$v timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_${v}_$i.json 2> gpurun_out/${TAG}_${v}_$i.err || exit 12
  done
done
exit 0
