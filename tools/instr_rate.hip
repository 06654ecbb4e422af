// Diagnostic: issue cost of single VALU instructions on gfx950, relative to v_add_u32.
// Every CU runs 8 waves (2 per SIMD); each wave runs ITER x 8 independent instances of the
// instruction under test (8 accumulator chains, so latency is hidden).  Prints ns per
// wave-instruction per SIMD and the ratio to v_add_u32.
//   hipcc --offload-arch=gfx950 -O3 tools/instr_rate.hip -o tools/bin/instr_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITER = 4096;

#define BODY8(INS)                                                                       \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS     \
                   " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS     \
                   " %6, %6, %8\n\t" INS " %7, %7, %8"                                   \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(k));
#define BODY8U(INS)                                                                       \
  asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS \
                   " %4, %4\n\t" INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"        \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));

#define KERNEL2(NAME, INS)                                                                \
  __global__ __launch_bounds__(512) void NAME(unsigned* out, unsigned k) {                 \
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7;                                                    \
    for (int i = 0; i < ITER; ++i) { BODY8(INS) }                                          \
    out[blockIdx.x * 512 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;           \
  }
#define KERNEL1(NAME, INS)                                                                \
  __global__ __launch_bounds__(512) void NAME(unsigned* out, unsigned k) {                 \
    unsigned a0 = threadIdx.x | 0x3f800000u, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                       \
    for (int i = 0; i < ITER; ++i) { BODY8U(INS) }                                         \
    out[blockIdx.x * 512 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ k;       \
  }

KERNEL2(k_add, "v_add_u32")
KERNEL2(k_xor, "v_xor_b32")
KERNEL2(k_mul_lo, "v_mul_lo_u32")
KERNEL2(k_mul_hi, "v_mul_hi_u32")
KERNEL2(k_mul24, "v_mul_u32_u24")
KERNEL2(k_mulhi24, "v_mul_hi_u32_u24")
KERNEL2(k_fmul, "v_mul_f32")
KERNEL1(k_log, "v_log_f32")
KERNEL1(k_sqrt, "v_sqrt_f32")
KERNEL1(k_sin, "v_sin_f32")
KERNEL1(k_cvtf, "v_cvt_f32_u32")
KERNEL1(k_bcnt, "v_bfrev_b32")

typedef void (*kfn)(unsigned*, unsigned);

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned* out;
  hipMalloc(&out, (size_t)cus * 512 * 4);
  struct { const char* n; kfn f; } ks[] = {
      {"v_add_u32", k_add},       {"v_xor_b32", k_xor},     {"v_mul_lo_u32", k_mul_lo},
      {"v_mul_hi_u32", k_mul_hi}, {"v_mul_u32_u24", k_mul24}, {"v_mul_hi_u32_u24", k_mulhi24},
      {"v_mul_f32", k_fmul},      {"v_log_f32", k_log},
      {"v_sqrt_f32", k_sqrt},     {"v_sin_f32", k_sin},     {"v_cvt_f32_u32", k_cvtf},
      {"v_bfrev_b32", k_bcnt}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float base = 0;
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, 3u);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(cus), dim3(512), 0, 0, out, 3u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // per SIMD: 2 waves x ITER x 8 instructions per launch
    const double ns = ms * 1e6 / 5 / (2.0 * ITER * 8);
    if (!base) base = ns;
    printf("%-20s %7.3f ns/wave-instr/SIMD   x%.2f of v_add_u32\n", k.n, ns, ns / base);
  }
  return 0;
}
