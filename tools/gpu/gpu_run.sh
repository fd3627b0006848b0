#!/bin/bash
# GPU-box driver for one gpurun call: tests, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-run}
STEPS=${STEPS:-tests,bench,prof}
ok=0
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q -rfE > gpurun_out/${TAG}_tests.log 2>&1 || exit 11
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 12
fi
if [[ $STEPS == *prof* ]]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/${TAG}_prof" -o prof -- python3 "$R/bench.py" --no-extras --no-cpu-baseline --no-density \
      > "$R/gpurun_out/${TAG}_prof_bench.json" 2> "$R/gpurun_out/${TAG}_prof.err") || exit 13
fi
exit 0
