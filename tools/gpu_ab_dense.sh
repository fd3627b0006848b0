# dense_x3s K stage 16 (32 KiB of LDS: 4 workgroups per CU) against 32 (64 KiB: 2), same box:
# the x3 dense tests on the candidate library, then the SSG line with both libraries alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abd; mkdir -p $O
CAND=$GRAFT_REPO_ROOT/tools/ablib/liblidar_sbk16.so
LIDAR_AMD_LIB=$CAND timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "dense or backbone_vs_oracle or bench_shape" > $O/tests.log 2>&1 || exit 11
AB_BASE="--no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg" bash tools/ab_args.sh $O 2 "LIDAR_AMD_LIB=$CAND --steps 20 --warmup 5" "--steps 20 --warmup 5" > $O/ab.log 2>&1 || exit 12
