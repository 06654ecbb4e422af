# Host cost of the loader-fed step (tools/host_loader.py), then the tail launch's phase stamps on
# balanced and random-label batches (tools/tailw_stamps.py, stamps build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 180 python tools/host_loader.py 2>&1 | grep -v amdgpu.ids | head -40 || exit 1
for rl in 0 1; do echo "== randlab $rl"; STAMP_RANDLAB=$rl timeout -k 10 120 python tools/tailw_stamps.py 2>&1 | grep -v amdgpu.ids || exit 1; done
