// The weight-independent half of the 16-bit encoder: the reference's augmentation
//   weak_augment   x + weak_std * N                          (I/utils.py:328-331)
//   strong_augment (x + strong_std * N) * (u > p), then frames [start, start + mask_len) zeroed
//                                                            (I/utils.py:333-375)
// and the conversion of every MFMA input row to 16 bits (fp16 or bf16, round to nearest even), for
// the three encoder passes of one step (I/train.py:399,406-410,439).  None of it depends on the
// weights, so it need not sit between the previous step's optimizer and this step's GEMMs: the
// step launches it either standalone before the encoder (dad_prep), or -- when the caller names
// the next batch -- for the NEXT step on the ~250 workgroups the current step's tail launch
// leaves idle (dad_tail_ecda_w blocks > DAD_C), where it overlaps the latency-bound tail/ECDA.
//
// Output: one prepared set [clean Bc*Tc | strong Bn*Tn | weak Bn*Tn][768] of 16-bit rows in the
// padded layout (row b*T + t), whatever the source mode.  The strong and clean parts are also the
// weight gradient's operand.  The step prepares all three parts (a.clean = 1; 206 MB of HBM
// traffic at B=64, T=300: 118 MB of fp32 rows read, 88.5 MB of 16-bit rows written); a.clean = 0
// (noisy rows only) is kept for callers whose clean rows are converted elsewhere.
//
// One wave per row; lane l owns columns 256k + 4l .. +3 (k = 0..2): the element pairs the fused
// encoder converted per lane, so the counter RNG draws the same values (pair (row*768 + d) / 2 of
// the stream, dad_aug_noise_pair) and the bytes equal what the fused encoder multiplied.  Each
// wave loads R rows before converting any (R x 3 KB in flight per wave; rows past the end are
// clamped to the last one and not stored, so no load sits under a condition).  The fp32 source
// rows are read once: non-temporal loads keep them out of the caches, so the prepared rows this
// pass writes stay in the 256 MB Infinity Cache for the encoder and the weight gradient (A/B: step
// 114.1-114.5 -> 110.3-110.6 us, encoder 38.5 -> 36.7 us, weight gradient 26.0 -> 25.0 us).  In
// the tail launch (8 waves per CU) R = 2 measured best: 111.3-112.0 us against 112.7-113.3 (R = 4),
// 113.5 (R = 3), 111.7-113.2 (R = 1), 119 (R = 8).  Loading the next group's rows before converting
// the current one (software pipelining, 2 x R x 12 VGPRs) measured no faster: tail launch 42.7-42.9
// against 41.2 us (R = 2), 45.0 (R = 4), 42.7-42.8 (R = 1): the pass is bound by HBM at ~5 TB/s
// of mixed read/write traffic, not by the loads in flight per wave.
#pragma once
#include "dad_kernels.h"

// Stores of the prepared rows.  WT (dad_prep_rows, the noisy rows in the tail launch and the
// standalone dad_prep): write-through (sc1), so the line leaves the XCD's L2 with the store and the
// launch does not end with megabytes of dirty rows for the kernel-end writeback (MI355X_MICROARCH.md
// "boundary": + dirty bytes / 6 TB/s).  A/B on one box, 3 rounds: tail launch 29.2 -> 28.0-28.6 us,
// step 100.4-101.2 -> 99.7-100.2 us.  Inline asm: an atomic store (__hip_atomic_store) made hipcc
// wait for the memory operations in flight around every store.  Not write-through (measured, round 5):
//  - the clean rows converted inside the weight gradient (dad_prep_clean_store): 34 -> 110 us, since
//    every later vmcnt wait of the GEMM's pipeline then waits for the stores' round trip to memory;
//  - the weight gradient's split-K partials: step +0.8 us (tail launch of the next step +1 us);
//  - 16-B stores (lane pairs swapping 8-B pieces by DPP, 2 instead of 3 stores per row): tail
//    launch +0.4 us;
//  - non-temporal stores: encoder 27.9-28.2 -> 29.2-29.6 us (it then reads the rows from HBM
//    instead of the Infinity Cache), tail launch unchanged.
template <bool WT>
__device__ __forceinline__ void dad_prep_st(char* p, uint2 v) {
  if constexpr (WT) asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v));
  else *reinterpret_cast<uint2*>(p) = v;
}

template <int NOISE>
__device__ __forceinline__ int dad_prep_tstart(const DadPrepArgs& a, int b) {
  if (NOISE) return (int)a.start[b];
  return dad_tstart_at(a.key_tstart, b, a.start_hi);
}

// waves [wave, wave + nwaves, ...) of the prepared set; wave index wave-uniform.
// STOREN (store-mode noisy batch, Bn <= 64): every noisy utterance's store row base and length sit in
// lane b of two registers, loaded once, so a row's source is a readlane instead of two dependent
// global loads per row (dad_src_row): the tail launch's noisy preparation of a store batch took
// 40.2 us against 29.8 for a padded batch (events, one box).
template <int NOISE, bool F16, int R, bool STOREN>
__device__ __forceinline__ void dad_prep_rows(const DadPrepArgs& a, int wave, int nwaves, int lane) {
  const DadGeom& G = a.g;
  const int Nc = G.Bc * G.Tc;
  const int Nn = a.warmup ? 0 : G.Bn * G.Tn;
  const int N = Nc + Nn;
  uint16_t* const oc = a.x16;
  uint16_t* const os = a.x16 + (size_t)Nc * DAD_D;
  uint16_t* const ow = os + (size_t)Nn * DAD_D;
  uint32_t sn_lo = 0, sn_hi = 0;
  int sn_len = 0;
  if constexpr (STOREN) {
    const int b = min(lane, max(G.Bn, 1) - 1);
    const int64_t base = a.src.rown[b];
    sn_lo = (uint32_t)base;
    sn_hi = (uint32_t)((uint64_t)base >> 32);
    sn_len = a.src.lenn[b];
  }
  // feature keep flags of the lane's 12 columns (one [768] mask per step, I/utils.py:343)
  float kp[3][4];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) kp[k][e] = dad_feat_keep(a.u, a.key_feat, 256 * k + 4 * lane + e, a.feat_p);
  for (int base = (a.clean ? 0 : Nc) + wave; base < N; base += R * nwaves) {
    f32x4 v[R][3];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int u = min(base + r * nwaves, N - 1);
      const bool noisy = u >= Nc;
      const int un = noisy ? u - Nc : u;
      const int T = noisy ? G.Tn : G.Tc;
      const int b = un / T, t = un - b * T;
      size_t srow;
      if (STOREN && noisy) {   // (b is wave-uniform: the wave's row is)
        const uint64_t base = (uint64_t)__builtin_amdgcn_readlane(sn_lo, b) |
                              ((uint64_t)__builtin_amdgcn_readlane(sn_hi, b) << 32);
        srow = (size_t)(base + (uint64_t)min(t, max(__builtin_amdgcn_readlane(sn_len, b), 1) - 1));   // dad_src_row's rule
      } else {
        srow = dad_src_row(a.src, noisy, b, T, t);
      }
      const float* x = (noisy ? a.xn : a.xc) + srow * DAD_D + 4 * lane;
#pragma unroll
      for (int k = 0; k < 3; ++k) v[r][k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + 256 * k));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int u = base + r * nwaves;
      if (u >= N) break;
      if (u < Nc) {
        char* o = reinterpret_cast<char*>(oc + (size_t)u * DAD_D + 4 * lane);
#pragma unroll
        for (int k = 0; k < 3; ++k)
          dad_prep_st<true>(o + 512 * k, uint2{dad_pack2<F16>(v[r][k][0], v[r][k][1]), dad_pack2<F16>(v[r][k][2], v[r][k][3])});
        continue;
      }
      const int un = u - Nc;
      const int b = un / G.Tn, t = un - b * G.Tn;
      const int st = a.mask_len > 0 ? dad_prep_tstart<NOISE>(a, b) : -(1 << 30);
      const bool tzero = t >= st && t < st + a.mask_len;      // I/utils.py:365-372 (padded Tmax)
      char* o_w = reinterpret_cast<char*>(ow + (size_t)un * DAD_D + 4 * lane);
      char* o_s = reinterpret_cast<char*>(os + (size_t)un * DAD_D + 4 * lane);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int d = 256 * k + 4 * lane;
        f32x4 nw, ns;
        if constexpr (NOISE) {
          nw = *reinterpret_cast<const f32x4*>(a.nw + (size_t)un * DAD_D + d);
          ns = *reinterpret_cast<const f32x4*>(a.ns + (size_t)un * DAD_D + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) { nw[e] *= a.weak_std; ns[e] *= a.strong_std; }
        } else {
          const uint32_t p = ((uint32_t)un * (uint32_t)DAD_D + (uint32_t)d) >> 1;
          float z[8];
          dad_aug_noise_pair(a.key_weak, p, a.weak_std, z[0], z[1]);
          dad_aug_noise_pair(a.key_weak, p + 1u, a.weak_std, z[2], z[3]);
          dad_aug_noise_pair(a.key_strong, p, a.strong_std, z[4], z[5]);
          dad_aug_noise_pair(a.key_strong, p + 1u, a.strong_std, z[6], z[7]);
          nw = f32x4{z[0], z[1], z[2], z[3]};
          ns = f32x4{z[4], z[5], z[6], z[7]};
        }
        // reference op order: x + std*N, then * feature mask, then temporal zero
        f32x4 w, s;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          w[e] = v[r][k][e] + nw[e];
          s[e] = (v[r][k][e] + ns[e]) * kp[k][e];
        }
        dad_prep_st<true>(o_w + 512 * k, uint2{dad_pack2<F16>(w[0], w[1]), dad_pack2<F16>(w[2], w[3])});
        const uint2 so = uint2{dad_pack2<F16>(s[0], s[1]), dad_pack2<F16>(s[2], s[3])};
        dad_prep_st<true>(o_s + 512 * k, tzero ? uint2{0u, 0u} : so);
      }
    }
  }
}

// runtime dispatch on the set's precision and draw source (wave-uniform)
template <int R, bool STOREN>
__device__ __forceinline__ void dad_prep_dispatch_s(const DadPrepArgs& a, int wave, int nwaves, int lane) {
  const bool noise = a.nw != nullptr;
  if (a.f16) {
    if (noise) dad_prep_rows<1, true, R, STOREN>(a, wave, nwaves, lane);
    else dad_prep_rows<0, true, R, STOREN>(a, wave, nwaves, lane);
  } else {
    if (noise) dad_prep_rows<1, false, R, STOREN>(a, wave, nwaves, lane);
    else dad_prep_rows<0, false, R, STOREN>(a, wave, nwaves, lane);
  }
}
template <int R>
__device__ __forceinline__ void dad_prep_dispatch(const DadPrepArgs& a, int wave, int nwaves, int lane) {
  if (a.src.rown != nullptr && a.g.Bn <= 64 && !a.warmup) dad_prep_dispatch_s<R, true>(a, wave, nwaves, lane);
  else dad_prep_dispatch_s<R, false>(a, wave, nwaves, lane);
}

// One CLEAN row of a prepared set in two halves, for callers that interleave it with other work
// (the weight-gradient launch, dad_wgrad_direct: its loads go out in one round, the conversion and
// stores a few rounds later): row u of [Bc*Tc] (clamped for the load, not stored past the end);
// lane l owns columns 256k + 4l .. +3 as in dad_prep_rows (no RNG on the clean rows).  Padded
// batches: source row u is row u of xc; store batches (STORE, Bc <= 64): the row through the
// utterance table held in registers (StoreRowsW) -- no table lookup in memory (a dependent load
// there would drain the caller's loads in flight).
// Store batches (a.src.rowc set, Bc <= 64): StoreRowsW holds each utterance's store row base and
// length in lane b (loaded once, before the caller's loop), so the source row is a wave-uniform
// readlane, not a dependent global load.
struct StoreRowsW {
  uint32_t lo, hi;   // lane b: rowc[b] (int64) halves
  int len;           // lane b: lenc[b]
  uint32_t tmag;     // fast division by Tc: floor(2^32 / Tc) + 1 (0 for Tc = 1)
};
__device__ __forceinline__ StoreRowsW dad_store_rows_w(const DadPrepArgs& a, int lane) {
  StoreRowsW r;
  const int b = min(lane, a.g.Bc - 1);
  const int64_t base = a.src.rowc[b];
  r.lo = (uint32_t)base;
  r.hi = (uint32_t)((uint64_t)base >> 32);
  r.len = a.src.lenc[b];
  r.tmag = a.g.Tc > 1 ? 0xffffffffu / (uint32_t)a.g.Tc + 1u : 0u;
  return r;
}
template <bool STORE>
__device__ __forceinline__ size_t dad_clean_src_row(const DadPrepArgs& a, int uc, const StoreRowsW& sr) {
  if constexpr (!STORE) return (size_t)uc;
  const int b = sr.tmag ? (int)__umulhi((uint32_t)uc, sr.tmag) : uc;   // uniform (uc is)
  const int t = uc - b * a.g.Tc;
  const uint64_t base = (uint64_t)__builtin_amdgcn_readlane(sr.lo, b) |
                        ((uint64_t)__builtin_amdgcn_readlane(sr.hi, b) << 32);
  const int len = __builtin_amdgcn_readlane(sr.len, b);
  return (size_t)(base + (uint64_t)min(t, max(len, 1) - 1));   // dad_src_row's rule
}
template <bool STORE = false>
__device__ __forceinline__ void dad_prep_clean_load(const DadPrepArgs& a, int u, int lane, f32x4 (&v)[3],
                                                    const StoreRowsW& sr = StoreRowsW{}) {
  const int uc = min(u, a.g.Bc * a.g.Tc - 1);
  const float* x = a.xc + dad_clean_src_row<STORE>(a, uc, sr) * DAD_D + 4 * lane;
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + 256 * k));
}
// (a row past the end was loaded as the last row and is stored there again: the same bytes, so the
// stores need no condition -- a conditional memory operation inside the caller's pipelined loop
// would make hipcc drain the loads in flight where the paths merge)
// F16: the set's precision (a.f16; the caller's compile-time copy, so no branch sits between stores)
template <bool F16>
__device__ __forceinline__ void dad_prep_clean_store(const DadPrepArgs& a, int u, int lane, const f32x4 (&v)[3]) {
  const int uc = min(u, a.g.Bc * a.g.Tc - 1);
  char* o = reinterpret_cast<char*>(a.x16 + (size_t)uc * DAD_D + 4 * lane);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    dad_prep_st<false>(o + 512 * k, uint2{dad_pack2<F16>(v[k][0], v[k][1]), dad_pack2<F16>(v[k][2], v[k][3])});
}
