# level 0's fused MLPs for the first k frames of each group on the side stream (StreamingSSG sa1_side)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abs; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 200 --timeout-method thread -k "streaming" > $O/tests.log 2>&1 || exit 11
bash tools/ab_args.sh $O 2 "--steps 20 --warmup 5" "--steps 20 --warmup 5 --sa1-side 32" "--steps 20 --warmup 5 --sa1-side 48" "--steps 20 --warmup 5 --sa1-side 20" > $O/ab.log 2>&1 || exit 12
