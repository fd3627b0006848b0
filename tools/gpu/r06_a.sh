set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -k "host_feed or eight_ranks" > $O/t_a.log 2>&1 || exit 11
LIDAR_AMD_LIB=$R/lidar_ai_recommendation_software_amd/liblidar_amd_diag.so timeout -k 10 300 python -u tools/micro/fps_pipe_phases.py 20 4 $O/fps_pipe_phases.json > $O/fps_pipe_phases.log 2>&1 || exit 12
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --detail $O/bench_a_detail.json > $O/bench_a.json 2> $O/bench_a.err || exit 13
MSG_SLEEP=15 timeout -k 10 200 python -u tools/msg_pipe.py 30 0 3,3 3,3 3,3 > $O/msg_sleep.log 2>&1 || exit 14
exit 0
