# the Tier N GPU tests on the LIDAR_SA_E3_BOUND=1 build, then the A/B (head / in-tree / e3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/tools/ablib/liblidar_e3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c/tests_e3.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/r04_ab.sh r04c 2 "head=tools/ablib/liblidar_head.so" "new=-" "e3=tools/ablib/liblidar_e3.so"
