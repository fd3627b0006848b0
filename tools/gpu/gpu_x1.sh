#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "bf16 or backbone" --timeout 120 --timeout-method thread > gpurun_out/x1_tests.log 2>&1 || exit 11
tools/gpu/gpu_msg.sh "--msg-batch 32" "--msg-batch 32 --msg-steps 48"
