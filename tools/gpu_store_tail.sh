# Loader-fed step loop (tools/host_loader.py) on the stamps build: host/wall per step, then the
# tail launch's phase timeline and the losses / range flag of the last store-fed steps.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
DAD_LIB_VARIANT=stamps timeout -k 10 180 python tools/host_loader.py 2>&1 | grep -v amdgpu.ids | head -40 || exit 1
