#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "dense or split or backbone or stream" --timeout 120 --timeout-method thread > gpurun_out/x3s_tests.log 2>&1 || exit 11
tools/gpu/gpu_sweep.sh x3s "--steps 240" "--steps 240 --x3s 0" "--steps 240"
