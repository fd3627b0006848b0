#!/bin/bash
# PMC passes over one FPS launch (tools/fps_pmc.py); each pass its own run and time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
TAG=${1:-fpspmc}; B=${2:-32}; T=${3:-512}
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o p -- python3 "$R/tools/fps_pmc.py" $B $T > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || exit 20
done
exit 0
