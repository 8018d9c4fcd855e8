set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R=gpurun_out/pmc5; mkdir -p $R
export AIMX_HOPU_COL_CAP=1024  # (tuning build: AIMX_LIB_PATH=aimnet-x2d_amd/lib/libaimx_tune.so)
tools/gpu_steps.sh \
 "120 pmc5/a.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/a -- python3 tools/hop_bwd_only.py --config c5" \
 "120 pmc5/b.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_UNALIGNED_STALL --output-format csv -d $R/b -- python3 tools/hop_bwd_only.py --config c5" \
 "120 pmc5/c.log timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/c -- python3 tools/hop_bwd_only.py --config c4" \
 "120 pmc5/k.log timeout -s KILL 100 rocprofv3 --kernel-trace --stats --output-format csv -d $R/k -- python3 tools/hop_bwd_only.py --config c5"
