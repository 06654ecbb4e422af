# instruction-mix PMC passes for one kernel (KREGEX), each pass its own rocprofv3 run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmci
cd /tmp
pass() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "${KREGEX:-dad_encode_ws}" --output-format csv \
    -d "$R/gpurun_out/pmci/$name" -o run -- python "$R/bench.py" --steps 4 --warmup 2 --no-cpu-baseline --fp32-steps 0 --no-data-path \
    > "$R/gpurun_out/pmci/$name.log" 2>&1
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_SMEM && \
pass b SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM && \
pass c SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16
rc=$?
cd "$R"
python - <<'PY'
import csv, glob, os, collections
R = os.environ["GRAFT_REPO_ROOT"]
for p in sorted(glob.glob(R + "/gpurun_out/pmci/*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(p)))
    agg = collections.defaultdict(float); n = collections.defaultdict(set)
    for r in rows:
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
    for k in sorted(agg):
        print("%-32s per launch %.4g" % (k, agg[k] / max(1, len(n[k]))))
PY
for f in "$R"/gpurun_out/pmci/*.log; do tail -1 "$f"; done
exit $rc
