#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
BA="--no-density --no-cpu-baseline --no-fp32-mfma-leg --steps 30"
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $BA $cfg > gpurun_out/msg_$i.json 2> gpurun_out/msg_$i.err || exit $((20+i))
done
