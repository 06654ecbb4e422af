set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_b64.py iemocap_b64 3 2>&1 | grep -v amdgpu.ids
