# weight-gradient diagnostics: per-phase stamps of library variants (STAMP_VARIANTS, stamps builds)
# with and without the next batch named (STAMP_AHEADS, default "0 1": the GEMM alone, then the _cp
# launch with the next batch's clean-row conversion), then an A/B of AB_VARIANTS (tools/gpu_ab.sh;
# BENCH_ARGS, e.g. --no-ahead for the GEMM alone)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${STAMP_VARIANTS:-stamps}; do for ah in ${STAMP_AHEADS:-0 1}; do
  echo "== $v ahead=$ah"
  STAMP_AHEAD=$ah DAD_LIB_VARIANT=$v timeout -k 10 120 python tools/wgd_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1
done; done
if [ -n "${AB_VARIANTS:-}" ]; then bash tools/gpu_ab.sh || exit $?; fi
