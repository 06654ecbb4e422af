# A/B/C... of library variants and bench flags on one box.  VARIANTS="name:lib:args ..." (lib empty =
# libdad_hip.so, else lib/libdad_hip_<lib>.so; args with '+' for spaces), ROUNDS alternating 400-step
# benches; TESTS (optional) run first; STAMPS=1 runs tools/wp_stamps.py at the end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abv
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-400} python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/abv_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/abv_tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/abv_tests.log | head -10
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
B="--no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path --kernel-steps 32"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-A::}; do
    name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; args=${rest#*:}; args=${args//+/ }
    DAD_LIB_VARIANT=$lib timeout -k 10 120 python -u bench.py --steps ${STEPS:-400} --warmup 50 $B $args > gpurun_out/abv/$name$r.log 2>&1 || { echo "bench $name$r failed"; tail -20 gpurun_out/abv/$name$r.log; exit 1; }
    python - "$name$r" gpurun_out/abv/$name$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d["kernels"]
print(sys.argv[1], "step %.1f us" % (d["ms_per_step"] * 1e3), "%.0fk utt/s" % (d["value"] / 1e3),
      " ".join("%s=%.1f" % (n.replace("dad_", ""), v["avg_ms"] * 1e3) for n, v in sorted(k.items()) if isinstance(v, dict) and "avg_ms" in v))
PY
  done
done
if [ -n "${STAMPS:-}" ]; then
  timeout -k 10 120 python -u tools/wp_stamps.py > gpurun_out/wp_stamps.txt 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/wp_stamps.txt; exit 1; }
  cat gpurun_out/wp_stamps.txt
fi
