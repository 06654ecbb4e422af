// Diagnostic timestamps for the 'stamps' build variant (-DDAD_PROBE_STAMPS, built into
// lib/libdad_hip_stamps.so and read by tools/{ws,wgd,head}_stamps.py).  Never part of the
// product library: there every macro below expands to nothing, so the kernels carry only
// the named stamp points.
#pragma once
#include <hip/hip_runtime.h>

#ifdef DAD_PROBE_STAMPS
// a device buffer of n u64 stamps and its host reader dad_probe_read_<sym>(host, count)
#define DAD_PROBE_BUFFER(sym, n)                                                                    \
  __device__ unsigned long long sym[n];                                                             \
  extern "C" int dad_probe_read_##sym(void* host, int count) {                                      \
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(sym), sizeof(unsigned long long) * (size_t)count, 0, \
                                    hipMemcpyDeviceToHost);                                         \
  }
#define DAD_PROBE_SET(sym, i, v) (sym[i] = (unsigned long long)(v))
#define DAD_PROBE_ADD(sym, i, v) (sym[i] += (unsigned long long)(v))
#define DAD_PROBE_CLK() __builtin_amdgcn_s_memtime()
#define DAD_PROBE_WALL() wall_clock64()
// make the MFMA results a and b complete before the next stamp
#define DAD_PROBE_FENCE2(a, b) asm volatile("s_nop 0" ::"v"(a), "v"(b))
#define DAD_PROBE_ON 1
#else
#define DAD_PROBE_BUFFER(sym, n)
#define DAD_PROBE_SET(sym, i, v) ((void)0)
#define DAD_PROBE_ADD(sym, i, v) ((void)0)
#define DAD_PROBE_CLK() 0ull
#define DAD_PROBE_WALL() 0ull
#define DAD_PROBE_FENCE2(a, b) ((void)0)
#define DAD_PROBE_ON 0
#endif
