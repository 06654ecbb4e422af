// Standalone launch of the 16-bit steps' row preparation (dad_prep.h): augmentation + 16-bit
// conversion of one step's clean, strong and weak rows into a prepared set, ahead of the encoder
// (dad_encode_wp).  Used when the previous step could not prepare this batch in its tail launch
// (first step, a batch the caller did not name in advance, a change of shape or switches).
// HBM-bound streaming: 3072 B read per source row, 1536 B written per prepared row.
#include "dad_prep.h"

__global__ __launch_bounds__(DAD_PREP_THREADS) void dad_prep(DadPrepArgs a) {
  DAD_GUARD_BLOCK(DAD_PREP_THREADS);
  if (!a.x16) return;
  constexpr int kWaves = DAD_PREP_THREADS / 64;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  dad_prep_dispatch<2>(a, (int)blockIdx.x * kWaves + w, (int)gridDim.x * kWaves, (int)threadIdx.x & 63);
}
