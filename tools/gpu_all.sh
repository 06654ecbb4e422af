# Round-end style record in one box: every -m gpu test (NO_BENCH), then tools/gpu_full.sh (PMC
# passes, the default bench line, rocprofv3 kernel trace/stats), then the seam gaps of the trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NO_BENCH=1 bash tools/gpu_round.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_full.sh || exit 1
python tools/trace_gaps.py gpurun_out/prof > gpurun_out/gaps.md && cat gpurun_out/gaps.md
exit $rc
