# Kernel trace of the loader-fed step loop (tools/host_loader.py): per-kernel durations and the
# GPU's busy fraction of the span, to tell a host-bound loop from a GPU-bound one.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/lprof" -o run -- python "$R/tools/host_loader.py" \
  > "$R/gpurun_out/lprof.log" 2>&1 || { tail -20 "$R/gpurun_out/lprof.log"; exit 1; }
cd "$R"
grep -E "host|wall" gpurun_out/lprof.log
python tools/trace_busy.py gpurun_out/lprof/run_kernel_trace.csv
