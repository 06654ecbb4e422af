# Kernel-focused PMC passes (PMC_REGEX, default dad_encode_wp; output gpurun_out/$PMC_OUT, default
# pmce), each pass its own rocprofv3 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=${PMC_OUT:-pmce}
mkdir -p gpurun_out/$O
cd /tmp
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "${PMC_REGEX:-dad_encode_wp}" --output-format csv \
    -d "$R/gpurun_out/$O/$name" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path \
    > "$R/gpurun_out/$O/$name.log" 2>&1
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES && \
pass b SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_MFMA && \
pass c SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES && \
pass d SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT
rc=$?
python "$R/tools/profile_report.py" "${PMC_REGEX:-dad_encode_wp} PMC" "$R/gpurun_out/$O/report.md" "$R/gpurun_out/nonexistent" "$R/gpurun_out/$O" 2>&1 | tail -2
exit $rc
