# Loader-fed loop (tools/host_loader.py): the working tree's library against lib/libdad_hip_prev.so, two rounds, then the loop on the stamps build.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for r in 1 2; do for v in "" prev; do echo "== variant ${v:-base} r$r"; DAD_LIB_VARIANT=$v timeout -k 10 180 python tools/host_loader.py 2>&1 | grep -E "^(collate|store) " || exit 1; done; done
bash tools/gpu_store_tail.sh 2>&1 | grep -E "class ends|\(cand|store"
