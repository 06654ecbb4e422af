set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
AB_VARIANTS="base ko1 ko3" AB_ROUNDS=1 bash tools/gpu_ab.sh || exit 1
for v in stamps stko1 stko3; do echo "== $v"; DAD_LIB_VARIANT=$v timeout -k 10 120 python -u tools/wp_stamps.py 2>&1 | grep -v amdgpu.ids | tail -4; done
