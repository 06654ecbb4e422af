cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in stamps stampsv1; do echo "== $v"; DAD_LIB_VARIANT=$v timeout -k 10 120 python tools/wgd_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
