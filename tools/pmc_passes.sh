set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_calib_f -o c -- python3 $R/tools/pmc_calib.py > $R/gpurun_out/pmc_calib.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_calib_w -o c -- python3 $R/tools/pmc_calib.py >> $R/gpurun_out/pmc_calib.log 2>&1 &&
timeout -k 10 500 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o p -- python3 $R/bench.py --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --ramp 0 --steps 6 --warmup 1 > $R/gpurun_out/pmc_fetch.json 2> $R/gpurun_out/pmc_fetch.err &&
timeout -k 10 500 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o p -- python3 $R/bench.py --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --ramp 0 --steps 6 --warmup 1 > $R/gpurun_out/pmc_write.json 2> $R/gpurun_out/pmc_write.err
