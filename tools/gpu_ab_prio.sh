# FPS waves at raised issue priority (s_setprio at kernel start) against the shipped library, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abp; mkdir -p $O
A=$GRAFT_REPO_ROOT/tools/ablib/liblidar_fpsprio.so; B=$GRAFT_REPO_ROOT/tools/ablib/liblidar_fpsprio1.so
bash tools/ab_args.sh $O 2 "LIDAR_AMD_LIB=$A --steps 20 --warmup 5" "LIDAR_AMD_LIB=$B --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
