# voxel GPU tests + a kernel trace of the voxel micro (tools/voxel_micro.py), then the e2 tests and A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_r.py -k voxel -x -q --timeout 120 --timeout-method thread > $O/tests_voxel.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/vprof -o v -- \
    python3 $GRAFT_REPO_ROOT/tools/voxel_micro.py > $GRAFT_REPO_ROOT/$O/vprof.log 2>&1 || exit 14
cd $GRAFT_REPO_ROOT
bash tools/gpu/r04_e2.sh
