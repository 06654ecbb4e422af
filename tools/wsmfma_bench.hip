// Diagnostic: the W-stationary encoder's inner chain in isolation on gfx950.  Every CU runs one
// 512-thread workgroup (8 waves, two per SIMD) with 192 VGPRs of resident B fragments per wave
// (a stand-in for W1) and a 16-row x 768-k 16-bit tile in LDS (XOR-swizzled as the encoder's);
// each iteration is one sub-slab: 24 k-steps x NT=2 v_mfma_f32_16x16x32_f16 per wave.  Variants:
//   lds_bar   A fragments read from LDS one k-step ahead, s_barrier per iteration (the encoder)
//   lds       the same without the barrier
//   lds_pf4   A fragments four k-steps ahead (16 more VGPRs), barrier per iteration
//   reg       A fragments from registers (no LDS), barrier per iteration: the MFMA issue floor
// Prints cycles (s_memtime) per iteration per wave and ns per iteration from events.
//   hipcc --offload-arch=gfx950 -O3 tools/wsmfma_bench.hip -o tools/bin/wsmfma_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 256, KS = 24, NT = 2, ROW = 1536;

__device__ __forceinline__ void mfma(f32x4& acc, const f16x8& a, const f16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

template <int MODE>   // 0 lds_bar, 1 lds, 2 lds_pf4, 3 reg
__global__ __launch_bounds__(512, 1) void chain(float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char tile[16 * ROW];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16 * ROW / 4; i += 512) reinterpret_cast<float*>(tile)[i] = 0.001f * (i & 7);
  __syncthreads();
  f16x8 w[NT][KS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) w[t][k][j] = (_Float16)(0.001f * ((lane + t + k + j) & 15));
  int aoff[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) aoff[m] = (lane & 15) * ROW + 16 * ((4 * m + (lane >> 4)) ^ (lane & 15));
  f32x4 acc[NT] = {};
  f16x8 areg[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) areg[m] = *reinterpret_cast<const f16x8*>(tile + aoff[m]);
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (MODE == 3) {
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int t = 0; t < NT; ++t) mfma(acc[t], areg[k & 3], w[t][k]);
    } else {
      constexpr int PF = MODE == 2 ? 4 : 1;
      f16x8 a[PF + 1];
#pragma unroll
      for (int k = 0; k < PF; ++k) a[k] = *reinterpret_cast<const f16x8*>(tile + aoff[k & 3] + 256 * (k >> 2));
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        if (k + PF < KS)
          a[(k + PF) % (PF + 1)] = *reinterpret_cast<const f16x8*>(tile + aoff[(k + PF) & 3] + 256 * ((k + PF) >> 2));
#pragma unroll
        for (int t = 0; t < NT; ++t) mfma(acc[t], a[k % (PF + 1)], w[t][k]);
      }
    }
    if constexpr (MODE != 1) __syncthreads();
  }
  const unsigned long long c1 = __builtin_readcyclecounter();
  if (lane == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = c1 - c0;
  out[blockIdx.x * 512 + threadIdx.x] = acc[0][0] + acc[1][1];
}

typedef void (*kfn)(float*, unsigned long long*);

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)cus * 512 * 4);
  hipMalloc(&cyc, (size_t)cus * 8 * 8);
  unsigned long long* h = new unsigned long long[cus * 8];
  struct { const char* n; kfn f; } ks[] = {{"lds_bar", chain<0>}, {"lds", chain<1>}, {"lds_pf4", chain<2>}, {"reg", chain<3>}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, cyc);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, (size_t)cus * 8 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < cus * 8; ++i) s += (double)h[i];
    const double cpi = s / (cus * 8) / ITER;
    printf("%-8s %7.0f cycles/iter/wave (48 MFMA/wave, 96/SIMD: floor 1536)  %6.3f us/iter  %.2f GHz\n", k.n, cpi,
           ms * 1e3 / ITER, cpi / (ms * 1e6 / ITER));
  }
  return 0;
}
