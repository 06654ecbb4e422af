# Development loop: the step's parity tests (TESTS, default the 16-bit / graph / prefetch / fp32
# parity files), then BENCH_RUNS alternating short benches of the default line and of the
# BENCH_B arguments (default --no-ahead) under the ENV_B variables, one summary line each.  Stops at a crash or limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_prefetch.py tests/test_gpu_16bit.py tests/test_gpu_throughput_parity.py tests/test_gpu_graph.py tests/test_gpu_parity.py"}
timeout -k 10 ${TEST_LIMIT:-400} python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/dev_tests.log 2>&1
rc=$?; tail -3 gpurun_out/dev_tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/dev_tests.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
B="--no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path --kernel-steps 32"
for r in $(seq 1 ${BENCH_RUNS:-2}); do
  for v in A B; do
    extra=""; envv=""; [ $v = B ] && extra="${BENCH_B---no-ahead}" && envv="${ENV_B:-}"
    env $envv timeout -k 10 120 python -u bench.py --steps ${STEPS:-400} --warmup 50 $B $extra > gpurun_out/dev_bench_$v$r.log 2>&1 || { echo "bench $v$r failed"; tail -20 gpurun_out/dev_bench_$v$r.log; exit 1; }
    python - "$v$r" gpurun_out/dev_bench_$v$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d["kernels"]
print(sys.argv[1], "step %.1f us" % (d["ms_per_step"] * 1e3), "%.0fk utt/s" % (d["value"] / 1e3),
      " ".join("%s=%.1f" % (n.replace("dad_", ""), v["avg_ms"] * 1e3) for n, v in sorted(k.items()) if isinstance(v, dict) and "avg_ms" in v))
PY
  done
done
