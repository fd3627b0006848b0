# one-wave FPS: exactness (FPS tests incl. the pipeline / nested ones), FPS alone per size, and the
# headline A/B of the one-wave kernel (auto) against the 512-thread kernel in the pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "fps or streaming or bench_shape" > $O/tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/fps_scale.py 64,512 1,128,384 > $O/fps_scale.log 2>&1 || exit 12
bash tools/ab_args.sh $O 2 "--steps 20 --warmup 5 --fps-threads 0" "--steps 20 --warmup 5 --fps-threads 512" > $O/ab.log 2>&1 || exit 13
