# A/B the product library against diagnostic variants (lib/libdad_hip_<v>.so): parity
# tests on the product build, then a short bench per build.  VARIANTS="norng ..." inline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in "" ${VARIANTS:-}; do
  DAD_LIB_VARIANT="$v" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp32-steps ${FP32_STEPS:-0} > "gpurun_out/bench_${v:-product}.log" 2>&1 || { tail -20 "gpurun_out/bench_${v:-product}.log"; exit 1; }
  echo "== ${v:-product}"; python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('%.0f utt/s  %.3f ms/step  enc %.1f us  %s' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d.get('fp32_mode','')))" "gpurun_out/bench_${v:-product}.log"
done
