#!/bin/bash
# One GPU-box call that refreshes a round's evidence, every GPU step under its own time limit and
# the steps chained so that the first failure ends the call:
#   1 the GPU tests               2 the bench line at the driver's settings (bench.json = the driver-readable
#     last line, bench_detail.json = the full record; --steps 20 --warmup 5) and a 240-step SSG-only line
#   3 rocprofv3 --kernel-trace --stats of the SSG bench (kernel durations to compare with the
#     in-bench HIP-event means)
#   4 PMC: a 1 GiB copy calibrating FETCH_SIZE / WRITE_SIZE, then one pass per counter group over
#     the SSG bench at the driver's shape (FETCH_SIZE; WRITE_SIZE; the SQ / GRBM VALU group)
#   5 the voxel leg's kernels (tools/voxel_micro.py: 20 batched launches at the bench's shape): kernel
#     trace, FETCH_SIZE and WRITE_SIZE passes (tools/pmc_voxel.py reduces them)
#   6 (round 6) configs[4]'s MSG pipeline: kernel trace + FETCH_SIZE / WRITE_SIZE passes (tools/pmc_msg.py), the same
#     passes over configs[1]'s pipeline (tools/pmc_msg.py --cfg1), and the SA1 FPS step phases inside the SSG
#     pipeline (tools/micro/fps_pipe_phases.py, diagnostic library)
# reduce afterwards (CPU): tools/pmc_traffic.py and tools/pmc_valu.py with the passes' bench lines
# usage (on the box): bash tools/profile_round.sh TAG [tests|notests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
# the PMC passes run the driver's shape (--steps 20: G = 4, 128-frame launches) with only the pipeline's own
# launches (--no-verify: no one-batch forward() references), so every counted dispatch is a 128-frame launch
SHORT="--no-verify --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err || exit 12
timeout -k 10 600 python bench.py --steps 240 --warmup 3 --no-extras --no-density --no-fp32-mfma-leg \
    --detail $O/bench240_detail.json > $O/bench240.json 2> $O/bench240.err || exit 19
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone \
    --detail $O/prof_bench_detail.json > $O/prof_bench.json 2> $O/prof.err || exit 13
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_f -o c -- \
    python3 $R/tools/pmc_calib.py > $O/pmc_calib.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_w -o c -- \
    python3 $R/tools/pmc_calib.py >> $O/pmc_calib.log 2>&1 || exit 15
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- \
    python3 $R/bench.py $SHORT --detail $O/pmc_fetch_detail.json > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 16
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- \
    python3 $R/bench.py $SHORT --detail $O/pmc_write_detail.json > $O/pmc_write.json 2> $O/pmc_write.err || exit 17
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_valu -o p -- \
    python3 $R/bench.py $SHORT --detail $O/pmc_valu_detail.json > $O/pmc_valu.json 2> $O/pmc_valu.err || exit 18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vprof -o v -- \
    python3 $R/tools/voxel_micro.py > $O/vprof.log 2>&1 || exit 20
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/vpmc_fetch -o v -- \
    python3 $R/tools/voxel_micro.py > $O/vpmc_fetch.log 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/vpmc_write -o v -- \
    python3 $R/tools/voxel_micro.py > $O/vpmc_write.log 2>&1 || exit 22
# configs[4] (round 6): kernel trace of the MSG pipeline alone (tools/msg_pipe.py, the bench's MSG settings), then
# FETCH_SIZE / WRITE_SIZE passes over the same run (tools/pmc_msg.py reduces them)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mprof -o m -- \
    python3 $R/tools/msg_pipe.py 30 0 3,3,0 > $O/mprof.log 2>&1 || exit 23
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/mpmc_fetch -o m -- \
    python3 $R/tools/msg_pipe.py 30 0 3,3,0 > $O/mpmc_fetch.log 2>&1 || exit 24
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/mpmc_write -o m -- \
    python3 $R/tools/msg_pipe.py 30 0 3,3,0 > $O/mpmc_write.log 2>&1 || exit 25
# configs[1] (round 6): FETCH_SIZE / WRITE_SIZE passes over its pipeline at the bench's leg settings (tools/pmc_msg.py --cfg1)
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/cpmc_fetch -o c -- \
    python3 $R/tools/msg_pipe.py --cfg1 40 > $O/cpmc_fetch.log 2>&1 || exit 27
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/cpmc_write -o c -- \
    python3 $R/tools/msg_pipe.py --cfg1 40 > $O/cpmc_write.log 2>&1 || exit 28
# the SA1 FPS step phases in the pipeline and alone (the diagnostic library)
cd $R
LIDAR_AMD_LIB=$R/lidar_ai_recommendation_software_amd/liblidar_amd_diag.so timeout -k 10 300 \
    python3 tools/micro/fps_pipe_phases.py 20 4 $O/fps_pipe_phases.json > $O/fps_pipe_phases.log 2>&1 || exit 26
exit 0
