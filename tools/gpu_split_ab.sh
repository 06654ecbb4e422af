# A/B at N = 1 of the next batch's noisy-row preparation: in the tail launch (default) or on a side
# stream from the end of the backward (--prep-under-exchange on, the DP layout), 2 rounds
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in 1 2; do for v in off on; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path \
    --steps 400 --prep-under-exchange $v > gpurun_out/ab/split_$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab/split_$v.$r.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab/split_$v.$r.log') if l.startswith('{')][-1])
print('$v r$r', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v})"
done; done
