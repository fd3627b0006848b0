# the main chain's MFMA kernels at s_setprio 1 (ahead of the FPS waves on shared SIMDs) vs the shipped library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abm; mkdir -p $O
A=$GRAFT_REPO_ROOT/tools/ablib/liblidar_mfmaprio.so
bash tools/ab_args.sh $O 3 "LIDAR_AMD_LIB=$A --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
