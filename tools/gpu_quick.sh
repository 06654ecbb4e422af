# Parity tests of the step (goldens, edge geometries, bf16 replays), the tail/ECDA phase stamps
# and a short bench (per-kernel times): the iteration loop of a kernel change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16_parity.py tests/test_gpu_utils.py ${QUICK_TESTS:-} -q -x \
  --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${STAMPS:-}" ]; then timeout -k 10 120 python tools/tailw_stamps.py > gpurun_out/tailw_stamps.log 2>&1 && tail -6 gpurun_out/tailw_stamps.log; fi
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --no-data-path ${BENCH_ARGS:-} > gpurun_out/bq.log 2>&1 || exit 1
python -c "
import json; d=json.loads([l for l in open('gpurun_out/bq.log') if l.startswith('{')][-1])
print('value %.0f ms %.4f' % (d['value'], d['ms_per_step']), {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v})"
if [ -n "${PMC:-}" ]; then
  R="$GRAFT_REPO_ROOT"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $PMC --kernel-trace --kernel-include-regex "${PMC_REGEX:-dad_}" --output-format csv \
    -d "$R/gpurun_out/qpmc" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 \
    --no-data-path > "$R/gpurun_out/qpmc.log" 2>&1) && python tools/pmc_brief.py gpurun_out/qpmc/run_counter_collection.csv || exit 1
fi
exit $rc
