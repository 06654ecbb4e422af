# encoder knockout experiments (diagnostic variants; bench encoder launch time per variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-base xnorng xl2 xnomfma xall}; do
  lib=$v; [ "$v" = base ] && lib=""
  DAD_LIB_VARIANT=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-data-path --fp32-steps 0 --steps 200 --warmup 30 ${BENCH_ARGS:-} > gpurun_out/encexp_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/encexp_$v.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/encexp_$v.log') if l.startswith('{')][-1]); print('%-8s enc %.1f us  step %.1f us' % ('$v', d['roofline']['avg_launch_ms']*1e3, d['ms_per_step']*1e3))"
done
