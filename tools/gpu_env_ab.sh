# A/B of environment switches on one box: AB_ENVS="DAD_WP_SCOST=1.0 DAD_WP_SCOST=1.1" (one token per
# variant; "base" = no change), AB_ROUNDS alternating eager benches each (per-kernel times), then
# one FETCH_SIZE PMC pass per variant for the kernels in PMC_REGEX.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/eab
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in ${AB_ENVS:-base}; do
    if [ "$v" = base ]; then ev=""; else ev="$v"; fi
    env $ev timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path \
      --launch eager --steps ${AB_STEPS:-400} ${BENCH_ARGS:-} > gpurun_out/eab/$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/eab/$r.log; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/eab/$r.log') if l.startswith('{')][-1])
print('$v r$r', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v})"
  done
done
if [ -n "${NO_PMC:-}" ]; then exit 0; fi
cd /tmp
i=0
for v in ${AB_ENVS:-base}; do
  i=$((i+1))
  if [ "$v" = base ]; then ev=""; else ev="$v"; fi
  env $ev timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "${PMC_REGEX:-dad_(encode|wgrad)}" --output-format csv \
    -d "$R/gpurun_out/eab/pmc$i" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --no-data-path --launch eager \
    > "$R/gpurun_out/eab/pmc$i.log" 2>&1 || { echo "PMC FAIL $v"; exit 1; }
  echo "$v"; python "$R/tools/pmc_brief.py" "$R/gpurun_out/eab/pmc$i/run_counter_collection.csv"
done
