# encoder split A/B: CONFIGS="name:libvariant:weights ..." (libvariant '-' = product, weights '-' = built-in)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
for c in ${CONFIGS}; do
  IFS=: read -r name lib wts <<< "$c"
  [ "$lib" = "-" ] && lib=""
  if [ "$wts" = "-" ]; then unset DAD_WS_WEIGHTS; else export DAD_WS_WEIGHTS=$wts; fi
  DAD_LIB_VARIANT=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-data-path --fp32-steps 0 --steps 300 --warmup 30 > gpurun_out/sweep_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/sweep_$name.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/sweep_$name.log') if l.startswith('{')][-1]); print('%-10s enc %.1f us  step %.1f us' % ('$name', d['roofline']['avg_launch_ms']*1e3, d['ms_per_step']*1e3))"
done
done
unset DAD_WS_WEIGHTS
