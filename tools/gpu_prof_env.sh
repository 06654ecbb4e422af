# kernel-trace stats of a short bench under extra env settings (ENVS="A=1 B=2"), one table per run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp
export TMPDIR=/tmp
i=0
for e in "${@}"; do
  i=$((i+1))
  env $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_env$i" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 30 --warmup 5 --no-cpu-baseline --fp32-steps 0 --no-data-path > "$GRAFT_REPO_ROOT/gpurun_out/prof_env$i.log" 2>&1 || { echo "FAIL $e"; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof_env$i.log"; exit 1; }
  echo "== $e"
  python - "$GRAFT_REPO_ROOT/gpurun_out/prof_env$i/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "dad_" in r["Name"]:
        print("%-28s calls %4s avg %8.1f us" % (r["Name"].split("(")[0][:28], r["Calls"], float(r["AverageNs"]) / 1000))
PY
done
