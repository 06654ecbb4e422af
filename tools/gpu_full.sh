# Round profile: PMC passes (HBM traffic per kernel -> profiles/pmc_latest.json, read by
# bench.py as roofline.traffic), the default bench line (with the CPU baseline), and a
# rocprofv3 kernel-trace/stats run of bench.py; one markdown report.  TITLE names the report.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TITLE=${TITLE:-profile}
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc.log; exit 1; }
python tools/profile_report.py "$TITLE" gpurun_out/report_pmc.md gpurun_out/none gpurun_out/pmc gpurun_out/pmc_latest.json || exit 1
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
cat gpurun_out/bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo PROF_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
# the data path's kernels (dad_collate_kernel, dad_collate_index_kernel) in a run of their own
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv --kernel-include-regex dad_collate -d "$GRAFT_REPO_ROOT/gpurun_out/prof_data" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_data.log" 2>&1 || { echo PROF_DATA_FAIL; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_data.log"; exit 1; }
cp "$GRAFT_REPO_ROOT/gpurun_out/prof_data/run_kernel_stats.csv" "$GRAFT_REPO_ROOT/gpurun_out/data_kernel_stats.csv"
cd "$GRAFT_REPO_ROOT"
python tools/profile_report.py "$TITLE" gpurun_out/profile.md gpurun_out/prof gpurun_out/pmc && sed -n 1,14p gpurun_out/profile.md
