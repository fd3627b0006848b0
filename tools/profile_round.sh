#!/bin/bash
# One GPU-box call that refreshes the round's evidence: GPU tests, the default bench line,
# the rocprofv3 kernel-trace summary of the same bench, and the two PMC traffic passes
# (+ their calibration copy).  Every GPU step has its own time limit; steps chained with &&.
# usage (on the box): bash tools/profile_round.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 11
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 12
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- \
    python3 $R/bench.py --no-extras --no-cpu-baseline --no-density > $O/prof_bench.json 2> $O/prof.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_f -o c -- \
    python3 $R/tools/pmc_calib.py > $O/pmc_calib.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_w -o c -- \
    python3 $R/tools/pmc_calib.py >> $O/pmc_calib.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- \
    python3 $R/bench.py --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --ramp 0 --steps 6 --warmup 1 \
    > $O/pmc_fetch.json 2> $O/pmc_fetch.err || exit 16
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- \
    python3 $R/bench.py --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --ramp 0 --steps 6 --warmup 1 \
    > $O/pmc_write.json 2> $O/pmc_write.err || exit 17
exit 0
