set -o pipefail
cd /tmp
R="$GRAFT_REPO_ROOT"
DAD_LIB_VARIANT=twice timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv --kernel-include-regex dad_ -d "$R/gpurun_out/twice" -o run -- python "$R/bench.py" --steps 40 --warmup 10 --no-cpu-baseline --fp32-steps 0 --no-data-path > "$R/gpurun_out/twice.log" 2>&1 || { tail -20 "$R/gpurun_out/twice.log"; exit 1; }
cd "$R"
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/twice/run_kernel_trace.csv")))
ts = [r for r in rows if "dad_tail_ecda" in r["Kernel_Name"]]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ts]
first, second = d[0::2], d[1::2]
print("pairs", len(second))
print("first  launch us:", " ".join("%.1f" % x for x in first[-12:]))
print("second launch us:", " ".join("%.1f" % x for x in second[-12:]))
PY
