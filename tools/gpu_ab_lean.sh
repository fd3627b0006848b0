# A/B of a candidate library (tools/ablib/liblidar_cand.so, built from the working tree) against the product build,
# same box: the Tier N tests on the candidate, the SA2 grouped MLP alone (tools/micro/sa2_ablate.py), then the
# SSG line with both libraries alternating. Used for the MFMA kernels' double buffering, pass-epilogue deferral and the FPS batch wait.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abl2; mkdir -p $O
CAND=$GRAFT_REPO_ROOT/tools/ablib/liblidar_cand.so
LIDAR_AMD_LIB=$CAND timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
for rep in 1 2; do
  timeout -k 10 120 python tools/micro/sa2_ablate.py >> $O/alone.log 2>> $O/err.log || exit 12
  LIDAR_AMD_LIB=$CAND timeout -k 10 120 python tools/micro/sa2_ablate.py >> $O/alone.log 2>> $O/err.log || exit 13
done
AB_BASE="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg" bash tools/ab_args.sh $O 2 "LIDAR_AMD_LIB=$CAND --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 14
