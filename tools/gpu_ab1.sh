set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab1
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "fps or streaming or bench_shape" > gpurun_out/ab1/tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/fps_scale.py 1024,512,256 128,384 > gpurun_out/ab1/fps_scale.log 2>&1 || exit 12
bash tools/ab_args.sh gpurun_out/ab1 2 "--steps 20 --warmup 5 --fps-threads 512" "--steps 20 --warmup 5 --fps-threads 256" "--steps 20 --warmup 5 --fps-threads 1024" > gpurun_out/ab1/ab.log 2>&1 || exit 13
