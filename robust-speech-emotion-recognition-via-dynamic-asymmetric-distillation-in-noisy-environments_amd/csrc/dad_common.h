// Shared device-side definitions for the DAD train-step kernels (gfx950 / CDNA4).
//
// Layout contract (see DESIGN.md "Data layout in HBM"):
//   features   f32 [B][T][768] row-major (the reference collator's padded layout,
//              I/dataload_noisy.py:111-129), padding mask u8 [B][T] (1 = pad)
//   W1         f32 [256][768] (nn.Linear weight, I/model.py:13), 16-bit shadow [256][768]
//              (fp16 or bf16 by the step's precision)
//   rows are processed in 32-row "slabs" that never cross an utterance: slab (b, c)
//   covers frames 32c .. 32c+31 of utterance b (frames >= T are masked).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dad.h"

#define DAD_D 768
#define DAD_H 256
#define DAD_C 4
#define DAD_SLAB 32
#define DAD_HT (DAD_H / 32)      // 32-wide h tiles

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // register-promotable (unlike HIP uint4)

__device__ __forceinline__ int dad_nchunk(int T) { return (T + DAD_SLAB - 1) / DAD_SLAB; }

// 16-bit MFMA operands of the throughput modes: fp16 (DAD_PREC_FP16, 11-bit significand) or
// bf16 (DAD_PREC_BF16, 8-bit), both rounded to nearest even.  Two floats -> one packed word
// (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32 on gfx950).
template <bool F16>
__device__ __forceinline__ uint32_t dad_pack2(float a, float b) {
  if constexpr (F16) return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, f16x2));
  else return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
}
__device__ __forceinline__ uint16_t dad_half_bits(float x, bool f16) {
  return f16 ? __builtin_bit_cast(uint16_t, (_Float16)x) : __builtin_bit_cast(uint16_t, (__bf16)x);
}
static inline __host__ __device__ bool dad_prec16(int precision) {
  return precision == DAD_PREC_BF16 || precision == DAD_PREC_FP16;
}

// ---------------------------------------------------------------------------------
// Counter-based RNG (production mode).  Each random value is a pure function of
// (seed, step counter, stream, element index), so the weight-gradient kernel can
// regenerate the strong augmentation instead of storing it.  Per value: the three-round
// "triple32" integer mixer (three 32-bit multiplies) with the 32-bit stream key injected
// after its first round, so different streams are different bijections of the element
// index (not shifted copies of one sequence) and two full rounds follow the key.  (A
// two-round mixer keyed between its rounds left adjacent elements correlated at ~2x the iid
// spread over 1.5e7 samples: tests/test_gpu_rng.py.)  The stream key is derived on the host
// from (seed, counter, stream) with splitmix64 (dad_stream_key).  Philox4x32-10 costs ~40
// quarter-rate multiplies per 4 outputs, which made the augmentation VALU-bound.
enum DadStream {
  DAD_RNG_WEAK = 1,      // teacher weak-aug noise      (I/utils.py:330)
  DAD_RNG_STRONG = 2,    // student strong-aug noise    (I/utils.py:338)
  DAD_RNG_FEAT = 3,      // feature-dropout uniforms    (I/utils.py:343)
  DAD_RNG_TSTART = 4,    // temporal mask start         (I/utils.py:370)
  DAD_RNG_DROP1 = 5,     // classifier dropout, clean   (I/train.py:400)
  DAD_RNG_DROP2 = 6,     // classifier dropout, strong  (I/train.py:440)
};

__host__ __device__ __forceinline__ uint32_t dad_rng32(uint32_t i, uint32_t key) {
  uint32_t x = i;
  x ^= x >> 17;
  x *= 0xed5ad4bbu;
  x ^= key;
  x ^= x >> 11;
  x *= 0xac4c1b51u;
  x ^= x >> 15;
  x *= 0x31848babu;
  x ^= x >> 14;
  return x;
}

static inline uint32_t dad_stream_key(uint64_t seed, uint64_t counter, uint32_t stream) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + counter * 0xD1B54A32D192ED03ull + (uint64_t)stream * 0xABC98388FB8FAC03ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z ^ (z >> 32));
}

// uniform in [0, 1)  (24-bit resolution)
__device__ __forceinline__ float dad_u01(uint32_t h) { return (float)(h >> 8) * (1.0f / 16777216.0f); }

// Two normals of standard deviation s from ONE hash: Box-Muller on its two 16-bit halves,
// each turned into a float in [1, 2) by bit placement (no int->float convert):
//   f1 = 1 + hi/2^16, u1 = 2 - f1 = 1 - hi/2^16 in [2^-16, 1]  (never 0)
//   f2 = 1 + lo/2^16: v_sin/v_cos take revolutions, so sin(2 pi f2) = sin(2 pi lo/2^16)
//   r = s sqrt(-2 ln u1) = sqrt(c log2 u1) with c = -2 ln2 s^2 folded into one constant
//   z0 = r cos(2 pi u2),  z1 = r sin(2 pi u2);   |z| <= 4.71 s.
// Element i of a stream takes normal (i & 1) of pair i >> 1, so every kernel that needs
// the value of element i regenerates it bit for bit.
#define DAD_NEG2LN2 (-1.38629436112f)
__device__ __forceinline__ void dad_normal_pair_c(uint32_t key, uint32_t pair, float c, float& z0, float& z1) {
  const uint32_t h = dad_rng32(pair, key);
  const float f1 = __uint_as_float(((h >> 9) & 0x007fff80u) | 0x3f800000u);
  const float f2 = __uint_as_float(((h << 7) & 0x007fff80u) | 0x3f800000u);
  const float r = __builtin_amdgcn_sqrtf(c * __builtin_amdgcn_logf(2.0f - f1));
  z0 = r * __builtin_amdgcn_cosf(f2);
  z1 = r * __builtin_amdgcn_sinf(f2);
}
__device__ __forceinline__ void dad_normal_pair(uint32_t key, uint32_t pair, float& z0, float& z1) {
  dad_normal_pair_c(key, pair, DAD_NEG2LN2, z0, z1);
}

// normal of element idx of stream `key`
__device__ __forceinline__ float dad_normal1(uint32_t key, uint32_t idx) {
  float z0, z1;
  dad_normal_pair(key, idx >> 1, z0, z1);
  return (idx & 1u) ? z1 : z0;
}

// 4 normals for elements (row, d..d+3) of a [rows][768] tensor in stream `key` (d % 4 == 0).
__device__ __forceinline__ f32x4 dad_normal4(uint32_t key, uint32_t row, uint32_t d) {
  const uint32_t p = (row * (uint32_t)DAD_D + d) >> 1;
  f32x4 z;
  float a, b, c, e;
  dad_normal_pair(key, p, a, b);
  dad_normal_pair(key, p + 1u, c, e);
  z[0] = a; z[1] = b; z[2] = c; z[3] = e;
  return z;
}

// Source rows of the feature tensors.  Padded mode: frame t of utterance b is row b*T + t of
// the [B][T][768] batch.  Store mode (dad_batch.rowc..lenn set): row base[b] + min(t, len[b]-1)
// of the feature store, so padding frames re-read the utterance's last frame (every consumer
// masks them) and nothing is read past the utterance.  Noise / RNG indices always use the
// padded row b*T + t, so both modes draw the same values.
struct DadStoreRows {
  const int64_t* rowc; const int32_t* lenc;
  const int64_t* rown; const int32_t* lenn;
};
__device__ __forceinline__ size_t dad_src_row(const DadStoreRows& s, bool noisy, int b, int T, int t) {
  const int64_t* base = noisy ? s.rown : s.rowc;
  if (!base) return (size_t)b * T + t;
  const int len = (noisy ? s.lenn : s.lenc)[b];
  return (size_t)(base[b] + min(t, max(len, 1) - 1));
}

// W1 16-bit shadow layout = the B-fragment order of the W-stationary encoder (encode_ws.hip):
// fragment ((w*4 + t)*24 + ks) is 64 lanes x 8 halves, lane l holding
// W1[h = 64w + 16t + (l & 15)][k = 32ks + 8(l >> 4) + j], so each wave loads its resident
// W1 with fully coalesced 1 KB reads.
__host__ __device__ __forceinline__ uint32_t dad_w1frag_index(uint32_t h, uint32_t k) {
  const uint32_t w = h >> 6, t = (h >> 4) & 3u, n = h & 15u, ks = k >> 5, q = (k >> 3) & 3u, j = k & 7u;
  return ((((w * 4u + t) * 24u + ks) * 64u) + n + 16u * q) * 8u + j;
}

__device__ __forceinline__ float dad_uniform_at(uint32_t key, uint32_t idx) {
  return dad_u01(dad_rng32(idx, key));
}

// Augmentation noise std*N of elements 2*pair, 2*pair+1 as the 16-bit encoder adds it: the scale
// folded into the Box-Muller radius constant (c = -2 ln2 std^2).
__device__ __forceinline__ void dad_aug_noise_pair(uint32_t key, uint32_t pair, float sd, float& z0, float& z1) {
  dad_normal_pair_c(key, pair, DAD_NEG2LN2 * sd * sd, z0, z1);
}

// Temporal-mask start of utterance b: uniform in [0, start_hi) (I/utils.py:370,
// randint(0, max(1, Tmax - mask_len + 1))) by a 32x32 -> 64-bit multiply-high.
__device__ __forceinline__ int dad_tstart_at(uint32_t key, int b, int start_hi) {
  const uint32_t h = dad_rng32((uint32_t)b, key);
  return (int)(((uint64_t)h * (uint64_t)start_hi) >> 32);
}

// Strong-augmentation feature keep flag of channel d (I/utils.py:343: rand(D) > dropout_rate,
// one [768] mask per call, no rescale); u = the explicit draw or the counter uniform.
__device__ __forceinline__ float dad_feat_keep(const float* u, uint32_t key, int d, float p) {
  const float v = u ? u[d] : dad_uniform_at(key, (uint32_t)d);
  return v > p ? 1.0f : 0.0f;
}

// classifier dropout keep factor of (utterance b, hidden unit h): nn.Dropout(p) in training
// mode, inverted scaling (I/model.py:54-64); explicit mask (parity) or counter RNG
__device__ __forceinline__ float keep_value(const uint8_t* keep, uint32_t key, int b, int h, float p, float scale) {
  if (p <= 0.0f) return 1.0f;
  bool k;
  if (keep) k = keep[(size_t)b * DAD_H + h] != 0;
  else k = dad_uniform_at(key, (uint32_t)(b * DAD_H + h)) >= p;
  return k ? scale : 0.0f;
}
// The same with the explicit-or-counter choice made by the caller, once, outside its loops
// (EXPLICIT = the mask pointers are set): no load sits inside a branch, so a batch of these
// keeps its loads in flight instead of draining vmcnt at every call.
template <bool EXPLICIT>
__device__ __forceinline__ float keep_value_t(const uint8_t* keep, uint32_t key, int b, int h, float p, float scale) {
  bool k;
  if constexpr (EXPLICIT) k = keep[(size_t)b * DAD_H + h] != 0;
  else k = dad_uniform_at(key, (uint32_t)(b * DAD_H + h)) >= p;
  return p <= 0.0f ? 1.0f : (k ? scale : 0.0f);
}


// LDS-DMA: 16 B per lane of `src` into LDS at lds_dst + 16 * lane (M0 = wave-uniform LDS
// byte address), three consecutive 1-KB pieces (src, src + 1 KB, src + 2 KB -> lds_dst, +1 KB,
// +2 KB) under ONE M0 write: the instruction offset advances the global address and the LDS
// destination alike.  Inline asm: the compiler neither counts it in its vmcnt waits nor drains
// it at barriers; the caller waits for it (s_waitcnt vmcnt) before reading the LDS bytes.
__device__ __forceinline__ void dad_glds16x3(const void* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "global_load_lds_dwordx4 %1, off offset:1024\n\t"
      "global_load_lds_dwordx4 %1, off offset:2048\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}

// ---------------------------------------------------------------------------------
// wave helpers (wave64).  Sums use DPP (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 across rows; lane 63 ends with the total, broadcast by
// v_readlane): six VALU ops per level-free reduction instead of six LDS-routed shuffles.
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dad_dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, 0xf, true);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ float dad_dpp_f(float v) {
  return __int_as_float(dad_dpp_i<CTRL, RM>(__float_as_int(v)));
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dad_dpp_d(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const int lo = dad_dpp_i<CTRL, RM>((int)(uint32_t)u), hi = dad_dpp_i<CTRL, RM>((int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ float dad_wave_sum(float v) {
  v += dad_dpp_f<0x111>(v);
  v += dad_dpp_f<0x112>(v);
  v += dad_dpp_f<0x114>(v);
  v += dad_dpp_f<0x118>(v);
  v += dad_dpp_f<0x142, 0xa>(v);
  v += dad_dpp_f<0x143, 0xc>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ double dad_wave_sum_d(double v) {
  v += dad_dpp_d<0x111>(v);
  v += dad_dpp_d<0x112>(v);
  v += dad_dpp_d<0x114>(v);
  v += dad_dpp_d<0x118>(v);
  v += dad_dpp_d<0x142, 0xa>(v);
  v += dad_dpp_d<0x143, 0xc>(v);
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ float dad_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Row index inside a 32x32 MFMA accumulator tile for (register r, lane half kh):
// C/D layout of v_mfma_f32_32x32x{2f32,16bf16}: col = lane&31, row = (r&3)+8*(r>>2)+4*(lane>>5).
__device__ __forceinline__ int dad_acc_row(int r, int kh) { return (r & 3) + 8 * (r >> 2) + 4 * kh; }

// ---------------------------------------------------------------------------------
// Batch geometry: the clean and noisy batches are collated independently by the reference
// (I/train.py:479-483), so their utterance counts and padded lengths differ in general.
struct DadGeom {
  int Bc, Tc, ncc, tpc;   // clean: utterances, frames, 32-row slabs per utterance, padded frames
  int Bn, Tn, ncn, tpn;   // noisy (Bn = 0 during warm-up when no noisy batch is used)
};

static inline __host__ __device__ DadGeom dad_geom(int Bc, int Tc, int Bn, int Tn) {
  DadGeom g;
  g.Bc = Bc; g.Tc = Tc; g.ncc = (Tc + DAD_SLAB - 1) / DAD_SLAB; g.tpc = g.ncc * DAD_SLAB;
  g.Bn = Bn; g.Tn = Tn > 0 ? Tn : 1; g.ncn = (g.Tn + DAD_SLAB - 1) / DAD_SLAB; g.tpn = g.ncn * DAD_SLAB;
  return g;
}

// live_jobs_at: the 32-row job boundary nearest to x cumulative live 16-row sub-slabs of one
// branch (nc slabs and L live sub-slabs per utterance, J jobs).  The last slab of an utterance
// holds ceil(T/16) - 2(nc-1) live sub-slabs (one at T = 300: rows 304..319 are skipped), so the
// encoder's ranges are priced by the sub-slabs they run, not by their job count.
static inline __host__ __device__ int dad_live_jobs_at(float x, int nc, int L, int J) {
  if (x <= 0.0f) return 0;
  const int b = (int)(x / (float)L);
  const float r = x - (float)b * (float)L;
  const int c0 = (int)(0.5f * r + 0.5f);
  const int c = c0 < nc ? c0 : nc;
  const int j = b * nc + c;
  return j < J ? j : J;
}
// Job ranges of the prepared-row encoder (dad_encode_wp, encode_ws.hip), shared by the kernel and
// the host.  Teachers [0, nt) split the weak slabs, students [nt, nt + ns) the clean slabs then the
// strong slabs, all evenly by live 16-row sub-slabs (every prepared sub-slab costs the same).  Job
// numbers: teacher j = weak slab j; student j < Jc clean slab j, j >= Jc strong slab j - Jc (job_of).
static inline __host__ __device__ void dad_wp_job_range(int wg, int nt, int ns, int Bc, int Tc, int ncc, int Bn,
                                                        int Tn, int ncn, int Js, bool& teacher, int& j0, int& j1) {
  const int Lc = (Tc + 15) / 16, Ln = (Tn + 15) / 16, Jc = Bc * ncc;
  teacher = wg < nt;
  const int k = teacher ? wg : wg - nt, n = teacher ? nt : ns;
  const float tn = Js ? (float)Bn * (float)Ln : 0.0f, tc = (float)Bc * (float)Lc;
  const float tot = teacher ? tn : tc + tn;
  int j[2];
  for (int e = 0; e < 2; ++e) {
    const int kk = k + e;
    if (kk >= n) { j[e] = teacher ? Js : Jc + Js; continue; }
    const float x = tot * (float)kk / (float)n;
    if (teacher) j[e] = dad_live_jobs_at(x, ncn, Ln, Js);
    else j[e] = x <= tc ? dad_live_jobs_at(x, ncc, Lc, Jc) : Jc + dad_live_jobs_at(x - tc, ncn, Ln, Js);
  }
  j0 = j[0];
  j1 = j[1];
}

// Workspace layout (bytes), shared by host and device.  All offsets 256-B aligned.
//   slab-indexed buffers: clean slabs [0, Bc*ncc), noisy slabs after them.
struct DadWs {
  size_t part_sum;   // f32 [Bc*ncc + 2*Bn*ncn][H]  per-slab pooled ReLU sums (clean | teacher-weak | strong)
  size_t part_cnt;   // f32 [Bc*ncc + Bn*ncn][H]    per-slab active-row counts (clean | strong)
  size_t bits;       // u32 [Bc*ncc + Bn*ncn][H]    ReLU'-and-valid row mask per (slab, h): bit r = row r
  size_t vlen;       // f32 [Bc + Bn]               valid lengths (clean | noisy)
  size_t cnt_tot;    // f32 [Bc + Bn][H]            active-row counts per utterance (clean | strong)
  size_t ge;         // f32 [Bc + Bn][H]            dL/de_clean | dL/de_strong (CE/KL part)
  size_t ge_ecda;    // f32 [Bc + Bn][H]            ECDA part of dL/de (rows flagged in eflag)
  size_t gzb;        // f32 [Bc + Bn][C]            dL/dz per utterance (clean | strong), from dad_tail
  size_t eflag;      // u32 [Bc + Bn]               1: ECDA wrote this row of ge_ecda this step
  size_t wpart;      // f32 [S][H][D]               split-K weight-gradient partial slabs
  size_t normpart;   // f32 [DAD_NORM_BLOCKS]       squared-norm partials
  size_t ecda;       // f32 [C][Bc+Bn][Bc+Bn]       ECDA pairwise scratch for large member sets
  size_t xs16;       // 16-bit modes: two prepared sets (dad_prep.h), set s at xs16 + s * x16set, each
                     // f16/bf16 [Bc*Tc clean | Bn*Tn strong | Bn*Tn weak][768] (the encoder's input;
                     // clean + strong are the weight gradient's operand)
  size_t x16set;     // bytes per prepared set
  size_t w1h;        // f16/bf16 [H][D]             modular encoder ops: 16-bit copy of W1
  size_t gflat;      // f32 [DAD_GRAD_FLOATS]       modular encoder backward: scratch grad vector
  size_t ready;      // u32                        fused pooling counter of dad_tail_ecda_w (DAD_POOL_SHARDS lines),
                     //                            then the step's pooling-timeout word (DAD_POOL_ABORT)
  size_t bytes;
  int splits;
};

static inline size_t dad_align(size_t x) { return (x + 255) & ~(size_t)255; }

// weight-gradient split-K factor.  FP32 (dad_wgrad_f32, 6 column blocks per split): 42
// splits -> 252 tiles.  FP16/BF16 (dad_wgrad_direct, 12 column blocks per split): 21 splits -> 252 workgroups,
// one per CU, and never more than WGD_MAXU = 64 slabs per split (its dL/de table in LDS).
// Both are bounded by the number of 32-row slabs.
#ifndef WGD_SPLITS
#define WGD_SPLITS 21   // x 12 column blocks = 252 workgroups (one per CU with 2 slab groups)
#endif
static inline int dad_wgd_min_splits(int total) { return (total + 63) / 64; }
static inline int dad_auto_splits(const DadGeom& g, int precision, int warmup) {
  const int total = g.Bc * g.ncc + (warmup ? 0 : g.Bn * g.ncn);
  // FP32: 42 splits x 6 column blocks = 252 tiles, one per CU
  const int target = dad_prec16(precision) ? WGD_SPLITS : 42;
  int s = total < target ? total : target;
  if (dad_prec16(precision) && s < dad_wgd_min_splits(total)) s = dad_wgd_min_splits(total);
  return s;
}

static inline DadWs dad_ws_layout(const DadGeom& g, int splits, int precision) {
  DadWs w;
  const size_t nsc = (size_t)g.Bc * g.ncc, nsn = (size_t)g.Bn * g.ncn;
  const size_t nb = (size_t)g.Bc + g.Bn;
  size_t off = 0;
  w.splits = splits;
  w.part_sum = off; off = dad_align(off + sizeof(float) * (nsc + 2 * nsn) * DAD_H);
  w.part_cnt = off; off = dad_align(off + sizeof(float) * (nsc + nsn) * DAD_H);
  w.bits = off;     off = dad_align(off + sizeof(uint32_t) * ((size_t)g.Bc * g.tpc + (size_t)g.Bn * g.tpn) * DAD_HT);
  w.vlen = off;     off = dad_align(off + sizeof(float) * nb);
  w.cnt_tot = off;  off = dad_align(off + sizeof(float) * nb * DAD_H);
  w.ge = off;       off = dad_align(off + sizeof(float) * nb * DAD_H);
  w.ge_ecda = off;  off = dad_align(off + sizeof(float) * nb * DAD_H);
  w.gzb = off;      off = dad_align(off + sizeof(float) * nb * DAD_C);
  w.eflag = off;    off = dad_align(off + sizeof(uint32_t) * nb);
  w.wpart = off;    off = dad_align(off + sizeof(float) * (size_t)splits * DAD_H * DAD_D);
  w.normpart = off; off = dad_align(off + sizeof(float) * DAD_NORM_BLOCKS);
  w.ecda = off;     off = dad_align(off + sizeof(float) * DAD_C * nb * nb);
  w.x16set = dad_align(dad_prec16(precision) ? 2 * ((size_t)g.Bc * g.Tc + 2 * (size_t)g.Bn * g.Tn) * DAD_D : 0);
  w.xs16 = off;     off = dad_align(off + 2 * w.x16set);
  w.w1h = off;      off = dad_align(off + 2 * (size_t)DAD_H * DAD_D);
  w.gflat = off;    off = dad_align(off + sizeof(float) * DAD_GRAD_FLOATS);
  w.ready = off;    off = dad_align(off + 128 * 9);   // DAD_POOL_SHARDS counters, 128 B apart, + the abort word
  w.bytes = off;
  return w;
}
