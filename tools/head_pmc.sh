#!/bin/bash
# GPU box: PMC passes over the fused-head shape sweep (k_head_fwd dominates): where the waves wait.
set -o pipefail
mkdir -p gpurun_out/hpmc
cd tools
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d ../gpurun_out/hpmc/a -- python3 head_shapes.py > ../gpurun_out/hpmc/a.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d ../gpurun_out/hpmc/b -- python3 head_shapes.py > ../gpurun_out/hpmc/b.log 2>&1
