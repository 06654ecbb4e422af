// Diagnostic: the ping-pong encoder's MFMA phase in isolation on gfx950 (csrc/encode_ws.hip,
// pp_mfma): ONE wave per SIMD issues one 32-row job = 24 k-steps x 4 v_mfma_f32_16x16x32_f16
// (2 row tiles x 2 hidden tiles) against 192 VGPRs of resident B fragments, its A fragments
// read from an XOR-swizzled LDS tile.  Every CU runs one 256-thread workgroup (4 waves; 100 KB of
// LDS keeps it alone on the CU).  Variants (cycles per job per wave, s_memtime):
//   0 asm    A by inline-asm ds_read_b128 two k-steps ahead, explicit lgkmcnt waits (the kernel)
//   1 reg    A from four registers, no LDS reads: the issue floor of this operand arrangement
//   2 agpr   as 0 with the accumulators in AGPRs
//   3 asm3   as 0, three k-steps ahead
//   4 nowait as 0 without the waits (timing only: the MFMAs read fragments still in flight)
//   5 half   VERDICT r05 item 4's layout: each wave holds HALF the hidden units (one 16-h tile, 96
//            VGPRs of B), so every A fragment read feeds one MFMA instead of two: 24 k-steps x 2
//            MFMAs per job (the same FLOP per CU takes twice the jobs); cycles are reported per MFMA
//   hipcc --offload-arch=gfx950 -O3 tools/pp_mfma_bench.hip -o tools/bin/pp_mfma_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 64, KS = 24, ROW = 1536, TILE = 16 * ROW;

template <bool AG>
__device__ __forceinline__ void mfma(f32x4& acc, const f16x8& a, const f16x8& b) {
  if constexpr (AG) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
template <int OFF>
__device__ __forceinline__ void rd(f16x8& x, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void wt(f16x8& a, f16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}

template <int K, int PF>
__device__ __forceinline__ void rdk(f16x8 (&xa)[PF + 1][2], const uint32_t (&addr)[4]) {
  if constexpr (K < KS) {
    rd<256 * (K >> 2)>(xa[K % (PF + 1)][0], addr[K & 3]);
    rd<TILE + 256 * (K >> 2)>(xa[K % (PF + 1)][1], addr[K & 3]);
  }
}

template <int K, int PF, bool AG, bool WAIT>
__device__ __forceinline__ void kstep(f16x8 (&xa)[PF + 1][2], const uint32_t (&addr)[4], const f16x8 (&w)[2][KS],
                                      f32x4 (&acc)[2][2]) {
  if constexpr (K < KS) {
    rdk<K + PF, PF>(xa, addr);
    constexpr int younger = (K + PF < KS ? PF : KS - 1 - K);
    if constexpr (WAIT) wt<2 * younger>(xa[K % (PF + 1)][0], xa[K % (PF + 1)][1]);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      mfma<AG>(acc[0][t], xa[K % (PF + 1)][0], w[t][K]);
      mfma<AG>(acc[1][t], xa[K % (PF + 1)][1], w[t][K]);
    }
    kstep<K + 1, PF, AG, WAIT>(xa, addr, w, acc);
  }
}

template <int K, int PF>
__device__ __forceinline__ void kstep_half(f16x8 (&xa)[PF + 1][2], const uint32_t (&addr)[4], const f16x8 (&w)[2][KS],
                                           f32x4 (&acc)[2][2]) {
  if constexpr (K < KS) {
    rdk<K + PF, PF>(xa, addr);
    constexpr int younger = (K + PF < KS ? PF : KS - 1 - K);
    wt<2 * younger>(xa[K % (PF + 1)][0], xa[K % (PF + 1)][1]);
    mfma<false>(acc[0][0], xa[K % (PF + 1)][0], w[0][K]);
    mfma<false>(acc[1][0], xa[K % (PF + 1)][1], w[0][K]);
    kstep_half<K + 1, PF>(xa, addr, w, acc);
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void chain(float* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) char lds[100 * 1024];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2 * TILE / 4; i += 256) reinterpret_cast<float*>(lds)[i] = 0.001f * (i & 7);
  __syncthreads();
  f16x8 w[2][KS];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int k = 0; k < KS; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) w[t][k][j] = (_Float16)(0.001f * ((lane + t + k + j) & 15));
  const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  uint32_t addr[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) addr[m] = base + (lane & 15) * ROW + 16 * ((4 * m + (lane >> 4)) ^ (lane & 15));
  f32x4 acc[2][2] = {};
  f16x8 areg[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) areg[m] = *reinterpret_cast<const f16x8*>(lds + (addr[m] - base));
  const unsigned long long c0 = __builtin_readcyclecounter();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (MODE == 1) {
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          mfma<false>(acc[0][t], areg[k & 3], w[t][k]);
          mfma<false>(acc[1][t], areg[(k + 1) & 3], w[t][k]);
        }
    } else {
      constexpr int PF = MODE == 3 ? 3 : 2;
      f16x8 xa[PF + 1][2];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        rd<256 * 0>(xa[k][0], addr[k & 3] + 256 * (k >> 2));
        rd<TILE>(xa[k][1], addr[k & 3] + 256 * (k >> 2));
      }
      if constexpr (MODE == 5) kstep_half<0, PF>(xa, addr, w, acc);
      else kstep<0, PF, MODE == 2, MODE != 4>(xa, addr, w, acc);
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0][0]));
  const unsigned long long c1 = __builtin_readcyclecounter();
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = c1 - c0;
  float s = 0.0f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 2; ++t) s += acc[m][t][0] + acc[m][t][1] + acc[m][t][2] + acc[m][t][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, float* out, unsigned long long* cyc, int nwg) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(chain<MODE>, dim3(nwg), dim3(256), 0, 0, out, cyc);
  hipEventRecord(e0);
  constexpr int REP = 20;
  for (int r = 0; r < REP; ++r) hipLaunchKernelGGL(chain<MODE>, dim3(nwg), dim3(256), 0, 0, out, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.0f;
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[256 * 4];
  hipMemcpy(h, cyc, sizeof(unsigned long long) * nwg * 4, hipMemcpyDeviceToHost);
  double sum = 0.0;
  for (int i = 0; i < nwg * 4; ++i) sum += (double)h[i];
  const double per_job = sum / (nwg * 4) / ITER;
  const double us_job = ms * 1e3 / REP / ITER;
  const double nm = MODE == 5 ? 48.0 : 96.0;   // MFMAs per job per wave
  printf("%-7s cycles/job/wave %7.0f  (%.1f per MFMA)  us/job %.3f  implied clock %.2f GHz\n", name, per_job,
         per_job / nm, us_job, per_job / us_job / 1e3);
}

int main() {
  const int nwg = 256;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(float) * nwg * 256);
  hipMalloc(&cyc, sizeof(unsigned long long) * nwg * 4);
  run<0>("asm", out, cyc, nwg);
  run<1>("reg", out, cyc, nwg);
  run<2>("agpr", out, cyc, nwg);
  run<3>("asm3", out, cyc, nwg);
  run<4>("nowait", out, cyc, nwg);
  run<5>("half", out, cyc, nwg);
  run<0>("asm", out, cyc, nwg);
  return 0;
}
