cd "$GRAFT_REPO_ROOT"
STAMP_VARIANTS="stampsv2 stampscpd2" bash tools/gpu_wgd_diag2.sh || exit $?
AB_VARIANTS="base cpd2" AB_ROUNDS=2 bash tools/gpu_ab.sh
echo "== pp_mfma_bench"
timeout -k 10 60 tools/bin/pp_mfma_bench
