#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, own time limit) over a python command:
#   tools/pmc_kern.sh TAG script.py [args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" && mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o p -- python3 "$R/$@" > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || exit 20
done
exit 0
