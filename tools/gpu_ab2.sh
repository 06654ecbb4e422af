# A/B of diagnostic library variants: parity of each variant, then alternating 200-step benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-}; do
  DAD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/pytest_$v.log)"
done
for r in ${ROUNDS:-1 2}; do
  VARIANTS="base ${VARIANTS:-}" bash tools/gpu_encexp.sh || exit 1
done
