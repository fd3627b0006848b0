# configs[4] MSG pipeline settings sweep (tools/msg_pipe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/msg
timeout -k 10 600 python tools/msg_pipe.py 30 > gpurun_out/msg/sweep.log 2>&1 || exit 11
