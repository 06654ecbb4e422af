# weight-gradient stamps with and without the next batch named (the _cp launch vs GEMM only)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${STAMP_VARIANTS:-stamps}; do for ah in 0 1; do echo "== $v ahead=$ah"; STAMP_AHEAD=$ah DAD_LIB_VARIANT=$v timeout -k 10 120 python tools/wgd_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done; done
