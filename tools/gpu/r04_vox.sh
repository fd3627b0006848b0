# voxel GPU tests, then the voxel micro's kernel trace and PMC passes (tools/pmc_voxel.py reduces them)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r04f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_r.py -k voxel -x -q --timeout 120 --timeout-method thread > $O/tests_voxel.log 2>&1 || exit 11
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/vprof -o v -- \
    python3 $R/tools/voxel_micro.py > $R/$O/vprof.log 2>&1 || exit 20
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/$O/vpmc_fetch -o v -- \
    python3 $R/tools/voxel_micro.py > $R/$O/vpmc_fetch.log 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/$O/vpmc_write -o v -- \
    python3 $R/tools/voxel_micro.py > $R/$O/vpmc_write.log 2>&1 || exit 22
