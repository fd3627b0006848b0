# candidate library (tools/ablib/liblidar_cand.so; used for: split LDS buffers in the strict-fp32 sa16_kernel, the fused SA1
# kernel at 80 VGPRs, DENSE_SBK=16 on the double-buffered dense kernels) against the product build: the Tier N tests on the candidate, then the full SSG line
# (with the fp32-MFMA leg and the standalone legs) with both libraries alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab32; mkdir -p $O
CAND=$GRAFT_REPO_ROOT/tools/ablib/liblidar_cand.so
LIDAR_AMD_LIB=$CAND timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
AB_BASE="--no-extras --no-density --no-cpu-baseline" bash tools/ab_args.sh $O 2 "LIDAR_AMD_LIB=$CAND --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
