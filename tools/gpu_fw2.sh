set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fw2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "fps_bit_exact" > $O/tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/micro/fps_wave_phases.py 1,128,384 > $O/phases.log 2>&1 || exit 12
timeout -k 10 200 python tools/fps_scale.py 64 1,128 > $O/fps_scale.log 2>&1 || exit 13
bash tools/ab_args.sh $O 1 "--steps 20 --warmup 5 --fps-threads 0" "--steps 20 --warmup 5 --fps-threads 512" > $O/ab.log 2>&1 || exit 14
