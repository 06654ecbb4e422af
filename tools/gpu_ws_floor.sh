# Encoder floor microbenchmark: the W-stationary encoder with parts knocked out at compile time
# (csrc/encode_ws.hip WS_FLOOR_*; outputs wrong by design), each timed by a 400-step bench
# (per-kernel HIP events).  Variants are built on the CPU side beforehand (tools/ws_floor_build.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/floor
for r in $(seq 1 ${FLOOR_ROUNDS:-2}); do
  for v in base ${FLOOR_VARIANTS:-fl_norng fl_noxs fl_nomfma fl_nodma fl_skeleton fl_data}; do
    if [ "$v" = base ]; then vv=""; else vv="$v"; fi
    DAD_LIB_VARIANT=$vv timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --fp32-steps 0 --no-data-path \
      --steps 400 > gpurun_out/floor/$v.$r.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/floor/$v.$r.log; exit 1; }
    python -c "
import json; d=json.loads([l for l in open('gpurun_out/floor/$v.$r.log') if l.startswith('{')][-1])
print('$v r$r encoder %.1f us' % (d['kernels']['dad_encode_ws']['avg_ms'] * 1e3))"
  done
done
