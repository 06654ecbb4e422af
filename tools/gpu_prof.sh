# Kernel trace + stats of a short bench run into gpurun_out/prof (summary: tools/profile_report.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 ${PROF_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python tools/profile_report.py "dev profile" gpurun_out/prof_report.md gpurun_out/prof gpurun_out/none > /dev/null && sed -n 1,40p gpurun_out/prof_report.md
