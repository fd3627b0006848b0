#!/bin/bash
# A/B: run a micro-benchmark against the in-tree library and against a variant .so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
WHAT=$1; VAR=$2; TAG=$3
timeout -k 10 200 python tools_micro.py $WHAT > gpurun_out/${TAG}_A.log 2>&1 || exit 11
cp lidar_ai_recommendation_software_amd/liblidar_amd.so /tmp/orig.so && cp $VAR lidar_ai_recommendation_software_amd/liblidar_amd.so && \
timeout -k 10 200 python tools_micro.py $WHAT > gpurun_out/${TAG}_B.log 2>&1; rc=$?
cp /tmp/orig.so lidar_ai_recommendation_software_amd/liblidar_amd.so
exit $rc
