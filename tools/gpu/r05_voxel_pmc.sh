set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05v; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vprof -o v -- python3 $R/tools/voxel_micro.py > $O/vprof.log 2>&1 || exit 20
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/vpmc_fetch -o v -- python3 $R/tools/voxel_micro.py > $O/vpmc_fetch.log 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/vpmc_write -o v -- python3 $R/tools/voxel_micro.py > $O/vpmc_write.log 2>&1 || exit 22
