#!/bin/bash
# One GPU-box call that refreshes a round's evidence, every GPU step under its own time limit and
# the steps chained so that the first failure ends the call:
#   1 the GPU tests               2 the bench line at the driver's settings (bench.json, --steps 20
#     --warmup 5) and a 240-step SSG-only line (bench240.json)
#   3 rocprofv3 --kernel-trace --stats of the SSG bench (kernel durations to compare with the
#     in-bench HIP-event means)
#   4 PMC: a 1 GiB copy calibrating FETCH_SIZE / WRITE_SIZE, then one pass per counter group over
#     the SSG bench at the driver's shape (FETCH_SIZE; WRITE_SIZE; the SQ / GRBM VALU group)
# reduce afterwards (CPU): tools/pmc_traffic.py and tools/pmc_valu.py with the passes' bench lines
# usage (on the box): bash tools/profile_round.sh TAG [tests|notests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
# the PMC passes run the driver's shape (--steps 20: G = 4, 128-frame launches) with only the pipeline's own
# launches (--no-verify: no one-batch forward() references), so every counted dispatch is a 128-frame launch
SHORT="--no-verify --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 11
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 12
timeout -k 10 600 python bench.py --steps 240 --warmup 3 --no-extras --no-density --no-fp32-mfma-leg > $O/bench240.json 2> $O/bench240.err || exit 19
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone > $O/prof_bench.json 2> $O/prof.err || exit 13
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_f -o c -- \
    python3 $R/tools/pmc_calib.py > $O/pmc_calib.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_w -o c -- \
    python3 $R/tools/pmc_calib.py >> $O/pmc_calib.log 2>&1 || exit 15
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- \
    python3 $R/bench.py $SHORT > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 16
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- \
    python3 $R/bench.py $SHORT > $O/pmc_write.json 2> $O/pmc_write.err || exit 17
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_valu -o p -- \
    python3 $R/bench.py $SHORT > $O/pmc_valu.json 2> $O/pmc_valu.err || exit 18
exit 0
