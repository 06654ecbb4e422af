set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench.log | tail -5
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
exit $rc
