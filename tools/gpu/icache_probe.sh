#!/bin/bash
# Instruction-cache counters of the SSG pipeline with and without the SA1 FPS on the side streams
# (tools/skip_probe.py fps): is the FPS's presence an I-cache effect on the MFMA kernels?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i "SQC_ICACHE\|SQC_INST\|SQ_IFETCH" $O/avail.txt | head -20 > $O/avail_icache.txt || true
ARGS="--no-verify --no-extras --no-cpu-baseline --no-density --no-fp32-mfma-leg --no-standalone --steps 20 --warmup 5"
for w in none fps; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH \
      --output-format csv -d $O/$w -o p -- python3 $R/tools/skip_probe.py $w $ARGS > $O/$w.json 2> $O/$w.err || exit 11
done
# the same FPS with one guarded update_batch instance (13 KiB of code instead of 20, 72 VGPRs instead of 64)
if [ -n "$1" ]; then
  cd $R && bash tools/ab.sh -c $1 -t "fps or streaming" gpurun_out/icache_ab 2 "" "LIDAR_AMD_LIB=$1" || exit 12
fi
