#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" && mkdir -p gpurun_out
T=${1:-tr}
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_r.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/micro.py tier_r_batch > gpurun_out/${T}_B.log 2>&1 || exit 12
LIDAR_AMD_LIB=ab/base/liblidar_amd.so timeout -k 10 200 python tools/micro.py tier_r_batch > gpurun_out/${T}_A.log 2>&1 || exit 13
cd /tmp && export TMPDIR=/tmp && R=${GRAFT_REPO_ROOT}
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o p -- python3 $R/tools/micro.py tier_r_batch > $R/gpurun_out/${T}_prof.log 2>&1
