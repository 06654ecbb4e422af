# FP32 (parity-mode) step profile: rocprofv3 kernel trace + stats of a 20-step fp32 bench, and
# PMC passes (time, instruction mix, HBM traffic) of its kernels; one markdown report
# (TITLE names it).  Each GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
TITLE=${TITLE:-fp32}
mkdir -p gpurun_out/p32 gpurun_out/p32pmc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/p32/prof" -o run -- \
  python "$R/bench.py" --precision fp32 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path \
  > "$R/gpurun_out/p32/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$R/gpurun_out/p32/prof.log"; exit 1; }
pass() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "dad_" --output-format csv \
    -d "$R/gpurun_out/p32pmc/$name" -o run -- python "$R/bench.py" --precision fp32 --steps 3 --warmup 1 \
    --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path > "$R/gpurun_out/p32pmc/$name.log" 2>&1
}
pass time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES && \
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
pass write WRITE_SIZE || { echo PMC_FAIL; for f in "$R"/gpurun_out/p32pmc/*.log; do tail -3 "$f"; done; exit 1; }
cd "$R"
python tools/profile_report.py "$TITLE" gpurun_out/p32/profile.md gpurun_out/p32/prof gpurun_out/p32pmc && sed -n 1,30p gpurun_out/p32/profile.md
grep '^{' gpurun_out/p32/prof.log | tail -1 > gpurun_out/p32/bench.json
