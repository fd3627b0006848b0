set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O; cd $R
timeout -k 10 150 python -u tools/msg_pipe.py 30 0 3,3 3,3 3,3 > $O/msg_pooled.log 2>&1 || exit 11
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/msgtrace -o m -- python3 $R/tools/msg_pipe.py 30 0 3,3 > $O/msgtrace.log 2>&1 || exit 12
f=$(find $O/msgtrace -name '*kernel_trace.csv' | head -1); python3 $R/tools/timeline.py $f > $O/msg_timeline.txt 2>&1; python3 $R/tools/rocprof_by_grid.py $f $O/msg_by_grid.csv > $O/msg_by_grid.txt 2>&1
exit 0
