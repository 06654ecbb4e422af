# Quick iteration on the GPU box: the step's parity tests, the launch-mode probe (eager / graph,
# us per step), one rocprofv3 kernel trace of a short eager run, and the encoder's FETCH/WRITE
# PMC pass.  Stops at the first crash or time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${QUICK_TESTS:-tests/test_gpu_parity.py tests/test_gpu_throughput_parity.py tests/test_gpu_16bit.py tests/test_gpu_graph.py tests/test_gpu_shadow.py} \
  -q -x --timeout 150 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -2 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/graph_probe.py > gpurun_out/gp.log 2>&1 || exit 1
grep us/step gpurun_out/gp.log
PROF_ARGS="--kernel-steps 0 --no-data-path --no-parity --launch eager" bash tools/gpu_prof.sh > gpurun_out/quick_prof.txt 2>&1 || exit 1
sed -n '/Kernel durations/,/Step period/p' gpurun_out/prof_report.md | grep -E "dad_|Step period"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "dad_(encode|wgrad)" --output-format csv \
  -d "$R/gpurun_out/qpmc" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path --launch eager \
  > "$R/gpurun_out/qpmc.log" 2>&1 || exit 1
cd "$R"
python tools/pmc_brief.py gpurun_out/qpmc/run_counter_collection.csv || true
exit $rc
