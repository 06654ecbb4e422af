# Development check: smoke, the bf16 tests, the full GPU suite, one bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1 || { echo BF16_FAIL; grep -v amdgpu.ids gpurun_out/pytest_bf16.log | tail -40; exit 1; }
tail -3 gpurun_out/pytest_bf16.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -40; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench.log') if l.startswith('{')][-1]); print('%.0f utt/s  %.3f ms/step  enc %.1f us  fp32 %s' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms']*1e3, d.get('fp32_mode')))"
