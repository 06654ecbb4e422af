# PMC passes over the FP32 (parity-mode) step: bench.py's fp32 leg only, counters of the FP32
# encoder / weight-gradient kernels (each pass its own rocprofv3 process and time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc32
cd /tmp
pass() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "${PMC_REGEX:-dad_(encode|wgrad)_f32|dad_wsum}" --output-format csv \
    -d "$R/gpurun_out/pmc32/$name" -o run -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-parity --fp32-steps 6 --bf16-steps 0 --no-data-path \
    > "$R/gpurun_out/pmc32/$name.log" 2>&1 && python "$R/tools/pmc_brief.py" "$R/gpurun_out/pmc32/$name/run_counter_collection.csv"
}
if [ -n "${PMC_SETS:-}" ]; then
  # PMC_SETS="A B C;D E" -> one pass per ';'-separated set
  IFS=';' read -ra SETS <<< "$PMC_SETS"
  n=0
  for set in "${SETS[@]}"; do n=$((n + 1)); pass "set$n" $set || exit 1; done
  exit 0
fi
pass time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU && \
pass mem SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE FETCH_SIZE
