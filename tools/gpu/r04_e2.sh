# the Tier N GPU tests on the LIDAR_SA1_E2_BOUND=1 build, then the A/B (in-tree / e2), 3 reps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04d
LIDAR_AMD_LIB=$GRAFT_REPO_ROOT/tools/ablib/liblidar_e2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/tests_e2.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu/r04_ab.sh r04d 3 "new=-" "e2=tools/ablib/liblidar_e2.so"
