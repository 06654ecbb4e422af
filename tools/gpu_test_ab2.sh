# GPU tests, then the A/B of library variants twice: the default bench (next batch prepared ahead:
# the weight gradient carries the clean-row conversion) and --no-ahead (the weight gradient alone).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NO_BENCH=1 bash tools/gpu_round.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
bash tools/gpu_ab.sh || exit $?
BENCH_ARGS="--no-ahead ${BENCH_ARGS:-}" bash tools/gpu_ab.sh || exit $?
exit $rc
