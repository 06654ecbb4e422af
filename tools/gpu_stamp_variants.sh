set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${VARIANTS:-stamps}; do
  DAD_LIB_VARIANT=$v timeout -k 10 60 python tools/head_stamps.py > gpurun_out/st_$v.log 2>&1 || exit 1
done
