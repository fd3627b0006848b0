#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "fps" --timeout 120 --timeout-method thread > gpurun_out/pair_tests.log 2>&1 || exit 11
./gpu_sweep.sh pair "" "--fps-pair 1" "--fps-pair 1 --fps-group 4" "--fps-pair 1 --fps-group 5" ""
