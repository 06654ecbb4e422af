# The driver's short timed region against the long one on one box: bench.py --steps 20 --warmup 5
# (the driver's flags) and --steps 200 --warmup 50, alternating, all side legs on (no CPU baseline).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/region
for r in 1 2; do
  for s in "20 5" "200 50"; do
    set -- $s
    timeout -k 10 300 python bench.py --steps $1 --warmup $2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/region/s$1.$r.log 2>&1 || { echo "FAIL $1"; tail -5 gpurun_out/region/s$1.$r.log; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/region/s$1.$r.log') if l.startswith('{')][-1])
print('steps $1 r$r', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v})"
  done
done
