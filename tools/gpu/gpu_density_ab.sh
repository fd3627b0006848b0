#!/bin/bash
# Density-path A/B: GPU tests of Tier R / variant / radius, then the bench's density leg and a
# rocprofv3 kernel-trace of the batch path, on the in-tree lib (B) and ab/base (A).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R" && mkdir -p gpurun_out
TAG=${1:-dab}
B=$R/ab/${BASE:-base}/liblidar_amd.so
BA="--no-extras --no-cpu-baseline --no-fp32-mfma-leg --steps 20"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "tier_r or density or variant or radius or dbscan" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_benchB.json 2> gpurun_out/${TAG}_benchB.err || exit 12
LIDAR_AMD_LIB=$B timeout -k 10 300 python bench.py $BA > gpurun_out/${TAG}_benchA.json 2> gpurun_out/${TAG}_benchA.err || exit 13
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_profB -o p -- python3 $R/tools/tier_r_batch_prof.py > $R/gpurun_out/${TAG}_profB.log 2>&1 || exit 14
exit 0
