# The DP step's preparation layouts on one GPU: --exchange-us X stands in for the all-reduce window,
# --prep-under-exchange {off, clean, noisy} moves next-batch rows under it.  Tests first
# (PYTEST_ARGS narrows them).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest ${PYTEST_ARGS:-tests/test_gpu_prefetch.py tests/test_gpu_dp.py} -q -x --timeout 150 --timeout-method thread > gpurun_out/ab/xtests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/xtests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for x in ${XUS:-0 10 20}; do for v in off clean noisy; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --bf16-steps 0 --randlab-steps 0 --no-data-path \
    --steps ${AB_STEPS:-300} --exchange-us $x --prep-under-exchange $v > gpurun_out/ab/x$x.$v.log 2>&1 || { echo "FAIL $x $v"; tail -5 gpurun_out/ab/x$x.$v.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('gpurun_out/ab/x$x.$v.log') if l.startswith('{')][-1])
print('x=$x $v', 'ms %.4f' % d['ms_per_step'], {k: round(v['avg_ms'] * 1e3, 1) for k, v in d['kernels'].items() if 'avg_ms' in v})"
done; done
exit $rc
