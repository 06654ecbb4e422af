# A/B sweep on one box: SWEEP holds ';'-separated cases "label|VAR=x VAR2=y|lib variant|bench args"
# (empty fields allowed; lib variant "" = libdad_hip.so), run ROUNDS times in alternation as short
# benches (STEPS steps); one summary line per run: step time and the per-kernel event table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
B="--no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path --kernel-steps 32"
IFS=';' read -ra CASES <<< "$SWEEP"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CASES[@]}"; do
    IFS='|' read -r label envs variant args <<< "$c"
    log=gpurun_out/sweep/$label.$r.log
    env $envs DAD_LIB_VARIANT="$variant" timeout -k 10 150 python -u bench.py --steps ${STEPS:-400} --warmup 50 $B $args > $log 2>&1 \
      || { echo "FAIL $label"; tail -20 $log; exit 1; }
    python - "$label r$r" $log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d["kernels"]
print("%-14s step %.1f us %4.0fk utt/s  " % (sys.argv[1], d["ms_per_step"] * 1e3, d["value"] / 1e3) +
      " ".join("%s=%.1f" % (n.replace("dad_", ""), v["avg_ms"] * 1e3) for n, v in sorted(k.items()) if isinstance(v, dict) and "avg_ms" in v))
PY
  done
done
