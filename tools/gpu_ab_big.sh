# dense_x3s 256 x 256 tiles for group_all (the shipped library) against 128 x 128 (tools/ablib/liblidar_base.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abb; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 200 --timeout-method thread -k "dense or backbone or bench_shape" > $O/tests.log 2>&1 || exit 11
B=$GRAFT_REPO_ROOT/tools/ablib/liblidar_base.so
AB_BASE="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg" bash tools/ab_args.sh $O 2 "--steps 20 --warmup 5" "LIDAR_AMD_LIB=$B --steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
