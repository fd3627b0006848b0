# FPS alone per library build (after its bit-exactness tests on the product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05_fpsalone}; shift
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread \
    -k "fps or nested or streaming or bench_shape" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 11; }
tail -2 $O/tests.log
for lib in "$@"; do
  echo "== $lib alone"
  LIDAR_AMD_LIB=$lib timeout -k 10 120 python tools/fps_scale.py 512 128,384 || exit 12
done
