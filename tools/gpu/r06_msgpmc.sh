set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/mpmc_fetch -o m -- \
    python3 $R/tools/msg_pipe.py 30 0 3,3,0 > $O/mpmc_fetch.log 2>&1 || exit 24
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/mpmc_write -o m -- \
    python3 $R/tools/msg_pipe.py 30 0 3,3,0 > $O/mpmc_write.log 2>&1 || exit 25
cd $R && python3 tools/pmc_msg.py $O/mpmc_fetch $O/mpmc_write $O/pmc_traffic_msg.json 96
