#!/bin/bash
# bench policy sweep (headline only): each config its own time limit, && chain
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
TAG=${1:-sw}; shift
BA="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg"
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $BA $cfg > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || exit $((20+i))
done
exit 0
