# GPU tests, then the default bench line (tools/gpu_round.sh), and a one-line summary of it.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh > gpurun_out/round_final.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench.json"))
print("ms %.4f utt/s %.0f frac %.3f stale %s | random %.4f store %.4f bf16 %.4f fp32 %.4f cpu %.0f" % (
    d["ms_per_step"], d["value"], d["roofline"]["frac"], d["roofline"]["traffic_stale"],
    d["random_labels"]["ms_per_step"], d["data_path"]["step_with_store_gather"]["ms_per_step"],
    d["bf16_mode"]["ms_per_step"], d["fp32_mode"]["ms_per_step"], d["cpu_baseline"]["value"]))
PY
exit $rc
