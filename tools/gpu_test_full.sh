# GPU tests, then the round profile (tools/gpu_full.sh: PMC passes, bench line, rocprof); a crash,
# abort or time limit in the tests stops the script before the profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NO_BENCH=1 bash tools/gpu_round.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
bash tools/gpu_full.sh
frc=$?
exit $(( rc > frc ? rc : frc ))
