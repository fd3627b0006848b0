set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tier_n.py -x -q -k "fps_bit_exact" --timeout 120 --timeout-method thread > gpurun_out/t12_tests.log 2>&1 || exit 11
run() { tag=$1; shift 1; timeout -k 10 200 python bench.py --no-extras --no-density --no-cpu-baseline --no-fp32-mfma-leg "$@" > gpurun_out/t12_$tag.json 2> gpurun_out/t12_$tag.err; }
run t256g3d3 --fps-threads 256 && run t256g4d3 --fps-threads 256 --fps-group 4 && run t256g3d4 --fps-threads 256 --depth 4 && run t256g4d4 --fps-threads 256 --fps-group 4 --depth 4 && run t512g4d3 --fps-group 4
