set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread -k "streaming" > $O/t_streaming.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/msg_pipe.py 30 0 3,3,0 3,3,128 3,3,32 3,3,16 3,3,0 3,3,128 3,3,32 3,3,16 > $O/msg_sideq.log 2>&1 || exit 12
exit 0
