#!/bin/bash
# Round 3: why k_wgrad_lds runs at ~30 % MFMA: stall / instruction counters on the c4 grouped
# weight-gradient micro (one pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=gpurun_out/r3_wgpmc; mkdir -p $R
tools/gpu_steps.sh \
  "120 r3_wgpmc/list.log rocprofv3 -L" \
  "200 r3_wgpmc/a.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/a -- python3 tools/wgrad_micro.py c4" \
  "200 r3_wgpmc/b.log rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS --output-format csv -d $R/b -- python3 tools/wgrad_micro.py c4"
grep -i "SQ_WAIT\|SQ_INST\|LDS\|MFMA\|SQ_ACTIVE\|STALL" gpurun_out/r3_wgpmc/list.log | head -80 > $R/sq_counters.txt
