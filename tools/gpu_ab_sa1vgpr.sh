# the fused SA1 kernel at its natural 89 VGPRs (candidate) vs the product's 80-VGPR launch bound, 4 alternating
# reps of the SSG line at the driver's settings (standalone legs on)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abv; mkdir -p $O
CAND=$GRAFT_REPO_ROOT/tools/ablib/liblidar_cand.so
AB_BASE="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg" bash tools/ab_args.sh $O 4 "LIDAR_AMD_LIB=$CAND --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
