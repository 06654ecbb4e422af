# PMC passes (counters only with --kernel-trace, never with sys/runtime traces) over a
# short bench run; each pass in its own rocprofv3 process under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc/counters.txt" 2>&1 || true
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "${PMC_REGEX:-dad_}" --output-format csv \
    -d "$R/gpurun_out/pmc/$name" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path \
    > "$R/gpurun_out/pmc/$name.log" 2>&1
}
pass time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES && \
pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
pass write WRITE_SIZE
rc=$?
for f in "$R"/gpurun_out/pmc/*.log; do echo "== $f"; tail -2 "$f"; done
exit $rc
