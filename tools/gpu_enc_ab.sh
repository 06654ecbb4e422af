# Encoder iteration: the encoder's parity tests, then AB_ROUNDS alternating 400-step benches of the
# product library and the variants in AB_VARIANTS, then the stamps timeline.  Stops at a crash or limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_gpu_throughput_parity.py tests/test_gpu_16bit.py tests/test_gpu_prefetch.py"}
timeout -k 10 ${TEST_LIMIT:-300} python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/enc_tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/enc_tests.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
AB_VARIANTS="${AB_VARIANTS:-base old}" AB_ROUNDS=${AB_ROUNDS:-2} bash tools/gpu_ab.sh || exit 1
if [ -n "${STAMPS:-1}" ]; then timeout -k 10 120 python -u tools/wp_stamps.py > gpurun_out/wp_stamps.log 2>&1; cat gpurun_out/wp_stamps.log | tail -8; fi
