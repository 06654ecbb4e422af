# Iteration loop of a kernel change: the parity tests of the step, the tail/ECDA phase stamps
# (lib variant 'stamps'), an A/B of the product library against variant 'old' (AB_ROUNDS
# alternating 400-step benches), the host-overhead breakdown.  Stops at a crash or time limit.
# Variants are built here, before the call (the box only runs what the snapshot carries), e.g.
#   python -c "import sys; sys.path.insert(0, '<pkg>'); import _build; \
#              _build.build(variant='stamps', extra=['-DDAD_PROBE_STAMPS'])"
# and 'old' from the previous commit's sources (git stash; _build.build(variant='old'); git stash pop).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_throughput_parity.py tests/test_gpu_16bit.py -q -x \
  --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?; tail -2 gpurun_out/iter_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 150 python tools/tailw_stamps.py > gpurun_out/tailw.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/tailw.log | tail -5
AB_VARIANTS="${AB_VARIANTS:-base old}" AB_ROUNDS=${AB_ROUNDS:-2} bash tools/gpu_ab.sh || exit 1
if [ -n "${HOST:-}" ]; then timeout -k 10 120 python tools/host_overhead.py 2>&1 | grep -v amdgpu.ids; fi
exit $rc
