# GPU tests (all -m gpu, measured fp16/bf16 parity errors to gpurun_out/parity16.json), then the
# default bench line.  Test failures (pytest rc 1) still run the bench; a crash, abort or time
# limit stops the script there.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
DAD_PARITY_JSON=gpurun_out/parity16.json timeout -k 10 ${TEST_LIMIT:-420} python -u -m pytest tests -m gpu -v -rf \
  --timeout 120 --timeout-method thread -s ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
if [ -n "${NO_BENCH:-}" ]; then exit $rc; fi
timeout -k 10 ${BENCH_LIMIT:-400} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
grep '^{' gpurun_out/bench.log | tail -1 > gpurun_out/bench.json
tail -c 3000 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
