# Per-kernel timing of the product library and diagnostic variants (lib/libdad_hip_<v>.so):
# one rocprofv3 --kernel-trace --stats pass per build over a short bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/abprof
cd /tmp
for v in product ${VARIANTS:-}; do
  lv="$v"; [ "$v" = product ] && lv=""
  DAD_LIB_VARIANT="$lv" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/abprof/$v" -o run -- python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 --no-data-path \
    > "$R/gpurun_out/abprof/$v.log" 2>&1 || { tail -20 "$R/gpurun_out/abprof/$v.log"; exit 1; }
  echo "== $v"
  python - "$R/gpurun_out/abprof/$v/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith("dad_"):
        print("  %-22s %8.1f us" % (r["Name"].split("(")[0], float(r["AverageNs"]) / 1e3))
PY
done
