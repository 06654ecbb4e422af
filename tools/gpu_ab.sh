# A/B of library variants on one box: AB_VARIANTS="base lut1" (base = libdad_hip.so), AB_ROUNDS
# alternating 400-step benches each; prints the per-kernel times of every run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in ${AB_VARIANTS:-base}; do
    if [ "$v" = base ]; then vv=""; else vv="$v"; fi
    DAD_LIB_VARIANT=$vv timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path \
      --steps ${AB_STEPS:-400} ${BENCH_ARGS:-} > gpurun_out/ab/$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab/$v.$r.log; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab/$v.$r.log') if l.startswith('{')][-1])
print('$v r$r', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v},
      'randlab ms %.4f' % d['random_labels']['ms_per_step'] if 'random_labels' in d else '')"
  done
done
