# One default bench line without the CPU baseline: the headline's and every side leg's per-kernel
# times (are the legs measured on settled clocks), then the bench tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_legs.log 2>&1 || { tail -20 gpurun_out/b_legs.log; exit 1; }
grep '^{' gpurun_out/b_legs.log | tail -1 > gpurun_out/b_legs.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/b_legs.json"))
kt = lambda r: {k: round(v["avg_ms"] * 1e3, 1) for k, v in r["kernels"].items() if "avg_ms" in v}
print("head", round(d["ms_per_step"], 4), kt(d))
for leg in ("fp32_mode", "bf16_mode", "random_labels"):
    if leg in d:
        print(leg, round(d[leg]["ms_per_step"], 4), kt(d[leg]))
dp = d.get("data_path")
if dp:
    print("store", round(dp["step_with_store_gather"]["ms_per_step"], 4), "collate",
          round(dp["step_with_device_collate"]["ms_per_step"], 4))
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench.py -q -x --timeout 200 --timeout-method thread 2>&1 | tail -1
