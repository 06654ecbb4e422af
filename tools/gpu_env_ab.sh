# A/B of an environment switch on one box: AB_ENV="DAD_PREP_STATIC=1" against the default, AB_ROUNDS
# alternating benches of AB_STEPS; per-kernel times of every run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in default switched; do
    if [ "$v" = default ]; then e=""; else e="${AB_ENV}"; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path \
      --steps ${AB_STEPS:-300} ${BENCH_ARGS:-} > gpurun_out/ab/env_$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab/env_$v.$r.log; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab/env_$v.$r.log') if l.startswith('{')][-1])
print('$v r$r', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v},
      'randlab ms %.4f' % d['random_labels']['ms_per_step'] if 'random_labels' in d else '')"
  done
done
