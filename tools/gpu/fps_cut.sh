#!/bin/bash
# FPS layout A/B in one GPU call: the FPS / pipeline GPU tests on the built library, the SSG line
# alternating the built library with a control (tools/ab.sh), then FETCH_SIZE / WRITE_SIZE passes over
# the SSG bench for both libraries plus the copy calibration (reduce with tools/pmc_traffic.py).
#   bash tools/gpu/fps_cut.sh OUTDIR CONTROL.so [REPS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/$1; CTL=$R/$2; REPS=${3:-3}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_tier_n.py -x -q --timeout 120 --timeout-method thread \
    -k "fps or streaming or bench_shape" > $O/tests.log 2>&1 || exit 11
bash tools/ab.sh $1 $REPS "" "LIDAR_AMD_LIB=$CTL" || exit 12
SHORT="--no-verify --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_f -o c -- \
    python3 $R/tools/pmc_calib.py > $O/pmc_calib.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_w -o c -- \
    python3 $R/tools/pmc_calib.py >> $O/pmc_calib.log 2>&1 || exit 15
for arm in cand ctl; do
  if [ $arm = ctl ]; then export LIDAR_AMD_LIB=$CTL; fi
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/${arm}_fetch -o p -- \
      python3 $R/bench.py $SHORT --detail $O/${arm}_fetch_detail.json > $O/${arm}_fetch.json 2> $O/${arm}_fetch.err || exit 16
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/${arm}_write -o p -- \
      python3 $R/bench.py $SHORT --detail $O/${arm}_write_detail.json > $O/${arm}_write.json 2> $O/${arm}_write.err || exit 17
done
