#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_msg -o t -- python3 $R/tools/trace_pipe.py msg bf16 32 131072 15 3 3 pre 1 0 512 > $R/gpurun_out/tl_msg.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_ssg -o t -- python3 $R/tools/trace_pipe.py ssg f32 32 65536 60 3 3 pre 1 0 512 > $R/gpurun_out/tl_ssg.log 2>&1
