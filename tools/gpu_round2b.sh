# round-2 session check: product GPU tests, the driver's bench command, encoder A/B vs VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv.log 2>&1 || { tail -20 gpurun_out/bench_drv.log; exit 1; }
grep '^{' gpurun_out/bench_drv.log | tail -1 | cut -c1-400
for v in ${VARIANTS:-}; do
  DAD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/pytest_$v.log)"
done
VARIANTS="base ${VARIANTS:-}" bash tools/gpu_encexp.sh
VARIANTS="base ${VARIANTS:-}" bash tools/gpu_encexp.sh
