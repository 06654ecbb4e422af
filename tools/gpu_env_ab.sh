# A/B of environment settings: CONFIGS="name:VAR=val ..." ('-' = none), ROUNDS rounds, 300-step benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
for c in ${CONFIGS}; do
  name=${c%%:*}; envs=${c#*:}
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --no-data-path --fp32-steps 0 --steps 300 --warmup 30 > gpurun_out/envab_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/envab_$name.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/envab_$name.log') if l.startswith('{')][-1]); print('%-10s enc %.1f us  step %.1f us' % ('$name', d['roofline']['avg_launch_ms']*1e3, d['ms_per_step']*1e3))"
done
done
