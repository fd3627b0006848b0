# voxel GPU tests, Tier N GPU tests, the full bench line, a kernel trace of the voxel micro
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04v}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_r.py -k voxel -x -q --timeout 300 --timeout-method thread > $O/tests_voxel.log 2>&1 || exit 10
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.log 2> $O/bench.err || exit 13
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/vprof -o v -- \
    python3 $GRAFT_REPO_ROOT/tools/voxel_micro.py > $GRAFT_REPO_ROOT/$O/vprof.log 2>&1 || exit 14
