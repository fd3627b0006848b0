# preprocess_kernel section stamps (diagnostic build) on one 65 536-point uniform frame
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pre
LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/lidar_ai_recommendation_software_amd/liblidar_amd_diag.so timeout -k 10 120 python tools/micro/pre_phases.py > gpurun_out/pre/phases.log 2>&1 || exit 11
