# weight-gradient diagnostics: per-phase stamps of library variants (STAMP_VARIANTS), then A/B of
# AB_VARIANTS with --no-ahead (the weight gradient without the clean-row conversion)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${STAMP_VARIANTS:-stamps}; do echo "== $v"; DAD_LIB_VARIANT=$v timeout -k 10 120 python tools/wgd_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
BENCH_ARGS="--no-ahead ${BENCH_ARGS:-}" bash tools/gpu_ab.sh || exit $?
