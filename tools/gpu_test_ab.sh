# GPU tests (all -m gpu unless PYTEST_ARGS narrows them), then an A/B of library variants
# (tools/gpu_ab.sh: AB_VARIANTS, AB_ROUNDS, AB_STEPS).  A crash, abort or time limit in the tests
# stops the script before the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NO_BENCH=1 bash tools/gpu_round.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
bash tools/gpu_ab.sh
arc=$?
exit $(( rc > arc ? rc : arc ))
