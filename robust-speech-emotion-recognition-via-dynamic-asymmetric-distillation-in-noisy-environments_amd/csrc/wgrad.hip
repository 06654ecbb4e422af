// Encoder weight gradient: dW1 = sum_rows G[row]^T x[row],  G = relu'(pre) * valid * dL/de_b / len_b
// (autograd of pre_net + ReLU + masked mean pool, I/model.py:28-36, for the clean branch
// (I/train.py:399) and the strong-augmented noisy branch (I/train.py:439)).
//
// K = rows (B*T per branch) is long and the output (256x768) small, so the reduction is
// split over `splits` row ranges; each workgroup writes one f32 partial slab, and
// dad_reduce sums them in a fixed order (deterministic, no float atomics).
// G is rebuilt on the fly from the ReLU' bit mask written by the forward and the
// per-(utterance, h) scale dL/de / len.  The strong branch's augmented input is
//   FP32: regenerated exactly (same counter-RNG function, or re-read explicit noise);
//   FP16/BF16: re-read from the 16-bit copy the forward stored (the exact MFMA operand it used).
// Both run after the losses as one direct split-K GEMM with the loss scale folded into G.
#include <type_traits>

#include "dad_common.h"
#include "dad_kernels.h"
#include "dad_prep.h"
#include "dad_probe.h"

namespace {

__device__ __forceinline__ int wg_tstart(const DadWgradArgs& a, int b) {
  if (a.start) return (int)a.start[b];
  return dad_tstart_at(a.key_tstart, b, a.start_hi);
}

__device__ __forceinline__ float wg_featkeep(const DadWgradArgs& a, int d) {
  return dad_feat_keep(a.u, a.key_feat, d, a.feat_p);
}

// slab s of the weight-gradient row list: clean slabs first, then strong (noisy) slabs
struct SlabIdx {
  int br, b, c, T;
  int erow;          // row of ge / vlen (clean b, or Bc + b)
  size_t row0;       // [b][T] row of frame 0
  size_t bits_slab;  // slab index in the ReLU' row-mask buffer (= s)
};
__device__ __forceinline__ SlabIdx wg_slab(const DadWgradArgs& a, int s) {
  const DadGeom& g = a.g;
  const int nsc = g.Bc * g.ncc;
  SlabIdx r;
  r.br = s >= nsc;
  const int rem = r.br ? s - nsc : s;
  const int nc = r.br ? g.ncn : g.ncc;
  r.b = rem / nc;
  r.c = rem - r.b * nc;
  r.T = r.br ? g.Tn : g.Tc;
  r.erow = r.br ? g.Bc + r.b : r.b;
  r.row0 = (size_t)r.b * r.T;
  r.bits_slab = (size_t)s;
  return r;
}

__device__ __forceinline__ int wg_total(const DadWgradArgs& a) {
  return a.g.Bc * a.g.ncc + (a.warmup ? 0 : a.g.Bn * a.g.ncn);
}

// slab range [s0, s1) of a split: a contiguous share of all slabs
__device__ __forceinline__ void wg_range(const DadWgradArgs& a, int split, int& s0, int& s1) {
  const int total = wg_total(a);
  const int per = (total + a.splits - 1) / a.splits;
  s0 = split * per;
  s1 = min(total, s0 + per);
}

// Fused step: dL/de of utterance row u (clean u < Bc, strong Bc + b), hidden unit h: the
// classifier part keep(u,h) * sum_c W2[c][h] dL/dz[u][c] (nn.Linear + nn.Dropout backward,
// I/model.py:62-63) plus the ECDA part where ECDA wrote the row.
// ec = ge_ecda[u][h] as loaded by the caller (read whatever the flag: unflagged rows hold
// stale values and are selected away, so a caller can keep all its loads in flight)
// EX: explicit dropout masks (a.keep1 set), chosen by the caller outside its loops
// (gz = dL/dz[u], ef = eflag[u], ec as loaded by the caller)
template <bool EX>
__device__ __forceinline__ float fused_ge1_v(const DadReduceArgs& a, int Bc, int u, int h, const float (&w2)[4],
                                             const f32x4& gz, uint32_t ef, float ec, float* kv_out = nullptr) {
  const bool strong = u >= Bc;
  const int b = strong ? u - Bc : u;
  const float kv = keep_value_t<EX>(strong ? a.keep2 : a.keep1, strong ? a.key_drop2 : a.key_drop1, b, h, a.p_drop,
                                    a.drop_scale);
  if (kv_out) *kv_out = kv;
  const float z = ((w2[0] * gz[0] + w2[1] * gz[1]) + w2[2] * gz[2]) + w2[3] * gz[3];
  return z * kv + (ef ? ec : 0.0f);
}
template <bool EX>
__device__ __forceinline__ float fused_ge1_ec(const DadReduceArgs& a, int Bc, int u, int h, const float (&w2)[4],
                                              float ec, float* kv_out = nullptr) {
  return fused_ge1_v<EX>(a, Bc, u, h, w2, *reinterpret_cast<const f32x4*>(a.gzb + (size_t)u * DAD_C), a.eflag[u], ec,
                         kv_out);
}
template <bool EX>
__device__ __forceinline__ float fused_ge1(const DadReduceArgs& a, int Bc, int u, int h, const float (&w2)[4],
                                           float* kv_out = nullptr) {
  return fused_ge1_ec<EX>(a, Bc, u, h, w2, a.ge_ecda[(size_t)u * DAD_H + h], kv_out);
}

}  // namespace

// ------------------------------------------------------------------- FP32 (parity mode)
// grid = 6 column blocks x splits; wave = 32 columns x 256 rows of dW1.
// v_mfma_f32_32x32x2_f32: A[i=h][k] = G[row k][h], B[k][j=d] = x[row k][d] (k = 2 rows).
//
// An f32 MFMA holds the SIMD's vector issue for its whole 64 cycles (PMC: zero VALU/MFMA
// co-execution cycles), so every VALU instruction of the loop adds its 4+ cycles to the
// MFMA time: the loop is built to issue as few as possible per MFMA.
//   * G (256 h x 32 rows of the slab, = ReLU' bit ? dL/de_u[h] / len_u : 0) is built ONCE per
//     workgroup into LDS (thread = h, double-buffered, one barrier per slab) and read as MFMA
//     A operands with ds_read_b128 (4 row pairs per read), instead of every wave rebuilding
//     all of it per MFMA (select + scale: 2-3 VALU per MFMA, and the fused dL/de per h).
//   * x (rows 2j + kh at column d) is loaded one slab ahead through a buffer descriptor of the
//     slab's valid rows (rows past the utterance read 0; one add per load for the address).
// The strong branch's augmentation is regenerated per element (counter RNG or explicit noise).
constexpr int F32_GP = 36;   // G tile pitch per h: [kh][16 pairs] + 4 floats (conflict-free b128 reads)

// the scale of G: dL/de / len from a dL/de buffer (modular encoder backward), or rebuilt from
// the tail's dL/dz and the ECDA rows (fused step, fused_ge1)
enum { F32_GE = 1, F32_FUSED = 2 };

struct F32X {
  float x[16], n[16];
};

// this lane's x (and explicit noise) of slab s: rows 2j + kh, column d
template <bool EXPLICIT, bool STORE>
__device__ __forceinline__ void f32_xload(const DadWgradArgs& a, int s, int d, int kh, F32X& r) {
  const SlabIdx q = wg_slab(a, s);
  const int nval = min(DAD_SLAB, q.T - q.c * DAD_SLAB);   // rows of the slab inside the utterance
#ifndef F32_BUFLOAD
#define F32_BUFLOAD 1
#endif
  if constexpr (!STORE && F32_BUFLOAD) {
    const float* X = (q.br ? a.xn : a.xc) + (q.row0 + (size_t)q.c * DAD_SLAB) * DAD_D;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(X), 0, nval * DAD_D * 4, 0x00020000);
    // The row offset goes in voffset, not soffset: the range check compares voffset (+ the
    // instruction offset) with num_records, so rows past the utterance read 0 and nothing is
    // read past the slab.  (The builtin returns the raw bits: __uint_as_float, not a value
    // conversion.)
    const int vo = (kh * DAD_D + d) * 4;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      r.x[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, vo + j * 2 * DAD_D * 4, 0, 0));
    if constexpr (EXPLICIT) {
      const float* N = a.ns + (q.row0 + (size_t)q.c * DAD_SLAB) * DAD_D;
      const auto rn = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(N), 0, nval * DAD_D * 4, 0x00020000);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        r.n[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rn, vo + j * 2 * DAD_D * 4, 0, 0));
    }
  } else {
    const float* X = q.br ? a.xn : a.xc;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int t = min(q.c * DAD_SLAB + 2 * j + kh, q.T - 1);
      r.x[j] = X[dad_src_row(a.src, q.br, q.b, q.T, t) * DAD_D + d];
      if constexpr (EXPLICIT) r.n[j] = a.ns[(q.row0 + t) * DAD_D + d];
    }
  }
}

// G inputs of thread h for slab s: the ReLU' row mask and the ECDA row / dL/de value
struct F32GIn {
  uint32_t mw;
  float ec;
};
template <int MODE>
__device__ __forceinline__ void f32_gload(const DadWgradArgs& a, const DadReduceArgs& ra, int s, int h, F32GIn& r) {
  const SlabIdx q = wg_slab(a, s);
  r.mw = a.bits[q.bits_slab * DAD_H + h];
  r.ec = 0.0f;
  if constexpr (MODE == F32_GE) r.ec = a.ge[(size_t)q.erow * DAD_H + h];
  if constexpr (MODE == F32_FUSED) r.ec = ra.ge_ecda[(size_t)q.erow * DAD_H + h];
}

// G^T of slab s into LDS: thread h writes G[h][kh][j] = bit (2j + kh) of its mask ? scale : 0
template <int MODE, bool KEEPX>
__device__ __forceinline__ void f32_gbuild(const DadWgradArgs& a, const DadReduceArgs& ra, int s, int h,
                                           const float (&w2h)[4], const F32GIn& gi, float* G) {
  const SlabIdx q = wg_slab(a, s);
  float scale = 0.0f;
  if constexpr (MODE == F32_GE) scale = gi.ec / fmaxf(a.vlen[q.erow], 1.0f);
  if constexpr (MODE == F32_FUSED) {
    // dL/de_u[h] / max(1, len_u), as dad_wgrad_direct builds it (16-bit there, f32 here)
    const int u = q.erow;
    const f32x4 gz = *reinterpret_cast<const f32x4*>(ra.gzb + (size_t)u * DAD_C);
    scale = fused_ge1_v<KEEPX>(ra, a.g.Bc, u, h, w2h, gz, ra.eflag[u], gi.ec) / fmaxf(ra.vlen[u], 1.0f);
  }
  const uint32_t sb = __float_as_uint(scale);
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)gi.mw, 2 * (4 * q4 + e) + kh, 1) & sb);
      *reinterpret_cast<f32x4*>(G + h * F32_GP + kh * 16 + 4 * q4) = v;
    }
}

// one slab's 128 MFMAs of this wave: A from the LDS G tile, B = x (strong: augmented here)
template <bool EXPLICIT, bool STRONG>
__device__ __forceinline__ void f32_mma(const DadWgradArgs& a, const SlabIdx& q, int d, int kh, float fkeep, int st,
                                        const float* G, const F32X& r, f32x16 (&acc)[DAD_HT]) {
  const int lane = threadIdx.x & 63;
  const float* gl = G + (lane & 31) * F32_GP + kh * 16;
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    f32x4 gv[DAD_HT];
#pragma unroll
    for (int ht = 0; ht < DAD_HT; ++ht) gv[ht] = *reinterpret_cast<const f32x4*>(gl + ht * 32 * F32_GP + 4 * q4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * q4 + e;
      float x = r.x[j];
      if constexpr (STRONG) {
        const int t = q.c * DAD_SLAB + 2 * j + kh;
        const bool tin = t < q.T;
        const size_t grow = q.row0 + (tin ? t : 0);
        const float n = EXPLICIT ? r.n[j] : dad_normal1(a.key_strong, (uint32_t)(grow * DAD_D + d));
        const float sn = n * a.strong_std;
        x = (x + sn) * fkeep;
        x = (t >= st && t < st + a.mask_len) ? 0.0f : x;   // (st + mask_len <= st when mask_len = 0)
        x = tin ? x : 0.0f;
      }
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht) acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(gv[ht][e], x, acc[ht], 0, 0, 0);
    }
  }
}

template <bool EXPLICIT, int MODE, bool STORE, bool KEEPX>
__device__ __forceinline__ void wgrad_f32_body(const DadWgradArgs& a, const DadReduceArgs& ra, float* Gs) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int i = lane & 31, kh = lane >> 5;
  const int h = tid;   // (256 threads = the 256 hidden units, for the G tile)
  float w2h[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if constexpr (MODE == F32_FUSED)
#pragma unroll
    for (int c = 0; c < 4; ++c) w2h[c] = ra.student[DAD_OFF_W2 + c * DAD_H + h];
  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int dblk = tile % 6, split = tile / 6;
    const int d = (dblk * 4 + wv) * 32 + i;
    int s0, s1;
    wg_range(a, split, s0, s1);
    f32x16 acc[DAD_HT];
#pragma unroll
    for (int ht = 0; ht < DAD_HT; ++ht) acc[ht] = f32x16{};
    const float fkeep = wg_featkeep(a, d);   // (the strong branch's feature mask; clean rows ignore it)
    if (s0 < s1) {
      F32GIn gi, gn;
      F32X cur, nxt;
      f32_gload<MODE>(a, ra, s0, h, gi);
      f32_xload<EXPLICIT, STORE>(a, s0, d, kh, cur);
      f32_gload<MODE>(a, ra, min(s0 + 1, s1 - 1), h, gn);
      f32_gbuild<MODE, KEEPX>(a, ra, s0, h, w2h, gi, Gs);
      f32_xload<EXPLICIT, STORE>(a, min(s0 + 1, s1 - 1), d, kh, nxt);
      __syncthreads();
      for (int s = s0; s < s1; ++s) {
        const int buf = (s - s0) & 1;
        const SlabIdx q = wg_slab(a, s);
        const float* G = Gs + buf * (DAD_H * F32_GP);
        if (q.br) {
          const int st = a.mask_len > 0 ? (EXPLICIT ? (int)a.start[q.b] : dad_tstart_at(a.key_tstart, q.b, a.start_hi)) : 0;
          f32_mma<EXPLICIT, true>(a, q, d, kh, fkeep, st, G, cur, acc);
        } else {
          f32_mma<EXPLICIT, false>(a, q, d, kh, fkeep, 0, G, cur, acc);
        }
        // the next slab's G (its inputs loaded a slab ago), then the loads of slab s + 2
        if (s + 1 < s1) f32_gbuild<MODE, KEEPX>(a, ra, s + 1, h, w2h, gn, Gs + (buf ^ 1) * (DAD_H * F32_GP));
        cur = nxt;
        f32_gload<MODE>(a, ra, min(s + 2, s1 - 1), h, gn);
        f32_xload<EXPLICIT, STORE>(a, min(s + 2, s1 - 1), d, kh, nxt);
        __syncthreads();
      }
    }
    float* out = a.wpart + (size_t)split * DAD_H * DAD_D;
#pragma unroll
    for (int ht = 0; ht < DAD_HT; ++ht)
#pragma unroll
      for (int r = 0; r < 16; ++r) out[(size_t)(ht * 32 + dad_acc_row(r, kh)) * DAD_D + d] = acc[ht][r];
  }
}

// KEEPX: explicit classifier-dropout masks (fused mode only)
template <bool EXPLICIT, int MODE, bool KEEPX>
__device__ __forceinline__ void wgrad_f32_store(const DadWgradArgs& a, const DadReduceArgs& ra, float* Gs) {
  if (a.src.rowc != nullptr) wgrad_f32_body<EXPLICIT, MODE, true, KEEPX>(a, ra, Gs);
  else wgrad_f32_body<EXPLICIT, MODE, false, KEEPX>(a, ra, Gs);
}
template <bool EXPLICIT>
__device__ __forceinline__ void wgrad_f32_mode(const DadWgradArgs& a, const DadReduceArgs& ra, float* Gs) {
  if (ra.gzb == nullptr) wgrad_f32_store<EXPLICIT, F32_GE, false>(a, ra, Gs);
  else if (ra.keep1) wgrad_f32_store<EXPLICIT, F32_FUSED, true>(a, ra, Gs);
  else wgrad_f32_store<EXPLICIT, F32_FUSED, false>(a, ra, Gs);
}

__global__ __launch_bounds__(DAD_WGRAD_THREADS) void dad_wgrad_f32(DadWgradArgs a, DadReduceArgs ra) {
  DAD_GUARD_BLOCK(DAD_WGRAD_THREADS);
  static_assert(DAD_WGRAD_THREADS == DAD_H, "dad_wgrad_f32: thread = hidden unit for the G tile");
  __shared__ __attribute__((aligned(16))) float Gs[2 * DAD_H * F32_GP];
  if (a.ns) wgrad_f32_mode<true>(a, ra, Gs);
  else wgrad_f32_mode<false>(a, ra, Gs);
}

// ------------------------------------------------------- FP16 / BF16 (throughput modes)
// Direct split-K GEMM after the losses: dW1 = sum_rows G[row]^T x[row] with
//   G[row][h] = ReLU'(row, h) * valid(row) * dL/de_u[h] / max(1, len_u)      (u = row's utterance)
// x is the encoder's 16-bit copy of the student's MFMA input (clean rows, then the
// strong-augmented rows), so one loop with one load type covers both branches.
// One workgroup per (column block of WGD_DB d, split of the slab list), two groups of 4 waves
// (two waves per SIMD): the groups take alternate slabs of the split and their accumulators
// are summed through LDS at the end.  Wave w of a group owns h tiles {2w, 2w+1} x both
// 32-wide d tiles.  Per 32-row slab:
//   x -> LDS [32][WGD_DB] (192-B row pitch: the four rows of a transposed read land on
//     disjoint bank quarters), read as k-major B fragments with ds_read_b64_tr_b16;
//   G is never staged: each lane loads the ReLU' row masks (one u32 per h) of its own two
//     hidden units straight into registers, and its A fragment (8 rows of one h) is byte
//     (16 ks + 8 (lane/32)) of that mask, expanded through a 256-entry LDS table into four
//     0xFFFF/0 dword masks and AND-ed with the 16-bit dL/de_u[h] / len_u in both halves: one
//     bitfield extract, one table read and four ANDs per fragment.  (The loop is bound by
//     vector issue, about ten VALU instructions per MFMA, so table reads replace arithmetic.)
// FP16: the per-utterance scales of hidden unit h are stored as fp16(v * 2^s_h), one power of
// two per h (its largest |v| over the split's utterances maps into [2^14, 2^15): 11 significant
// bits and no overflow or subnormals for values within 2^-28 of the largest), and row h of the
// partial is multiplied by 2^-s_h (exact) before it is stored.
// (The encoder's ping-pong schedule -- one group multiplies under s_setprio while the other builds
// operands, one barrier per phase -- measured slower here in round 5: 29.5-30.1 against 23.2-23.8
// us; a phase of 8 MFMAs is 256 cycles, and the barrier per phase cost more than the overlap won:
// stamps per round 250 operand + 412 MFMA cycles and ~880 waiting at the two barriers.)
// Software pipeline, one barrier per TWO rounds: round j computes slab j from LDS buffer j&3
// while it stages slab j+2 into buffer (j+2)&3 and issues the loads of slab j+2+WGD_DEPTH,
// all in one basic block so the staging VALU fills the MFMA gaps.  dL/de_u[h] / len_u of the
// workgroup's utterances is rebuilt in the prologue (fused_ge1) while the first loads are in
// flight.  Output: one f32 partial slab per split, summed in fixed order by dad_reduce_w.
static_assert(WGD_THREADS == 256 * WGD_GROUPS && DAD_H == 256, "dad_wgrad_direct: groups of 256 threads, thread = h");
static_assert(WGD_GROUPS == 1 || WGD_GROUPS == 2, "dad_wgrad_direct: one or two slab groups");
static_assert(WGD_DB == 64 && DAD_D % WGD_DB == 0, "dad_wgrad_direct: 8 threads x 8 columns per row");
// per-workgroup cycles of wave 0 in the stamps build (dad_probe.h): [prologue, loop, epilogue,
// -, sum over rounds of: compute+stage+load, barrier, -, -, rounds]
DAD_PROBE_BUFFER(wgd_stamps, 512 * 10)
#define WGD_CLK() DAD_PROBE_CLK()
#define WGD_ACC(k, v) \
  if (threadIdx.x == 0 && blockIdx.x < 512) DAD_PROBE_ADD(wgd_stamps, blockIdx.x * 10 + (k), (v))
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// B fragment (k-major) of the x tile: 8 x 16-bit in a bf16x8 register container
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* tile, int pitch, int rowbase, int colbase) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = colbase + 16 * (g & 1) + 4 * p;
  const int row = rowbase + 8 * (g >> 1) + q;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + row * pitch + col));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(tile + (row + 4) * pitch + col));
  // one concatenation (a register-pair sequence), not eight element copies
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 c = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

// one slab in flight: group thread t holds 8 consecutive columns of row t/8 (staged to LDS
// for everyone) and the ReLU' row masks of its own A-fragment hidden units (kept in
// registers); the slab's utterance slot and valid row count are wave-uniform
struct WgdSlab {
  u32x4 x;
  uint32_t mw[2];
  int ul, nvalid;
};

// Loop-invariant lane offsets and buffer resources of one tile (WGD_V2): every per-slab address of
// the loop is then a scalar (SGPR) base plus one of these, so the loads, the LDS staging and the
// table reads cost no vector instructions for their addresses (the loop is bound by vector issue).
struct WgdLane {
  uint32_t xoff;     // byte offset of this thread's 16 B of x in a 32-row slab of the prepared set
  uint32_t moff;     // byte offset of this lane's row-mask word in a slab's [H] u32 block (m = 0; m = 1 +128)
  uint32_t lsel[2];  // v_perm selectors of the byte of the mask word an A fragment uses (ks = 0, 1),
                     // merged with the lane's 16-B table slot offset (wgd_amask)
  uint32_t slot;     // (lane & 15) * 16: the lane's table slot
  uint32_t gsoff;    // byte offset of this lane's dL/de value in a utterance's [H] row of gs (m = 0)
  int nrows;         // rows of the clean + strong parts of the prepared set (x reads past them read 0)
};

// Slab table of one group, one slab per lane: lane l describes the group's slab j = l,
// global slab s0 + grp + WGD_GROUPS l (clean slabs first, then strong): its first x row (rows of the
// 16-bit copy: clean [b][Tc], then strong [b][Tn]) and (utterance slot << 8 | valid rows).
// A load reads its slab's entry with v_readlane, so no cursor arithmetic runs per slab.
struct WgdTable {
  int row0, info;
};

__device__ __forceinline__ WgdTable wgd_table(const DadGeom& g, int s, int u0) {
  const int nsc = g.Bc * g.ncc;
  const bool br = s >= nsc;
  const int rem = br ? s - nsc : s;
  const int nc = br ? g.ncn : g.ncc;
  const int b = rem / nc, c = rem - b * nc;
  const int T = br ? g.Tn : g.Tc;
  WgdTable t;
  t.row0 = (br ? g.Bc * g.Tc + b * T : b * T) + c * DAD_SLAB;
  t.info = (((br ? g.Bc + b : b) - u0) << 8) | min(T - c * DAD_SLAB, DAD_SLAB);
  return t;
}


// group slab j: its x rows through a buffer resource of the slab's 32 rows (SGPR base: rows past the
// clean + strong parts read 0, rows past the utterance are the next utterance's prepared rows; both
// are finite and meet mask bits 0, so no clamp runs per slab) and this lane's two row masks
// (buffer loads at the slab's scalar offset)
__device__ __forceinline__ void wgd_load(const DadWgradArgs& a, const WgdTable& tab, int j, int sfirst,
                                          const WgdLane& ln, WgdSlab& r) {
  const int row0 = __builtin_amdgcn_readlane(tab.row0, j);
  const int info = __builtin_amdgcn_readlane(tab.info, j);
  r.ul = info >> 8;
  r.nvalid = 0;
  const int n = min(__builtin_amdgcn_readfirstlane(ln.nrows) - row0, DAD_SLAB);   // (uniform: SGPR rsrc)
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.xs16 + (size_t)row0 * DAD_D), (short)0,
                                                    n * DAD_D * 2, 0x00020000);
  r.x = __builtin_amdgcn_raw_buffer_load_b128(rx, ln.xoff, 0, 0);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(a.bits), (short)0, -1, 0x00020000);
  const int soff = (sfirst + WGD_GROUPS * j) * DAD_H * 4;
  r.mw[0] = __builtin_amdgcn_raw_buffer_load_b32(rb, ln.moff, soff, 0);
  r.mw[1] = __builtin_amdgcn_raw_buffer_load_b32(rb, ln.moff + 128, soff, 0);
}

__device__ __forceinline__ void wgd_stage(const WgdSlab& r, uint16_t* Xt) {
  const int tid = threadIdx.x & 255;
  const int row = tid >> 3;
  // rows past the utterance hold a copy of its last row (finite); their ReLU' mask bits are 0
  *reinterpret_cast<u32x4*>(&Xt[row * WGD_XP + (tid & 7) * 8]) = r.x;
}

// A fragment of h tile ht, k rows 16 ks + 8 (lane/32) + 0..7: bit ? gb : 0 (16-bit pattern).
// lut[b][s] = the 0xFFFF/0 halfword masks of the 8 bits of byte b (16 B), once per 16-B bank
// slot s (64 KB): lane l reads slot l & 15, which is a different slot for every lane of each
// ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and +32), so the
// data-dependent bytes never meet on a bank (one table with one copy: 27 % of the kernel's
// LDS cycles were bank conflicts).  One bitfield extract and one 16-B LDS read per fragment.
constexpr int WGD_LUT_SLOTS = 16;
constexpr int WGD_LUT = 256 * WGD_LUT_SLOTS;
// WGD_V2 table: lut[b][s] holds v_perm SELECTORS instead of halfword masks: dword p of the A fragment
// is v_perm(g, g, sel) with sel taking bytes 0, 1 of g (the 16-bit dL/de_u[h] / len_u) into the
// halfword of each set bit (row 2p: bits 0-15, row 2p + 1: bits 16-31) and the zero byte (0x0c)
// into the others.  One v_perm per dword replaces the AND with a g | g << 16 pair, and the
// table address is one v_perm too: byte (2 ks + lane / 32) of the mask word into bits 8-15, the
// lane's slot offset into bits 0-7 (lsel).
__device__ __forceinline__ uint4 wgd_amask(uint32_t mask, const uint4* lut, uint32_t lsel, uint32_t slot) {
  const uint32_t off = __builtin_amdgcn_perm(mask, slot, lsel);   // (mask byte << 8) | (lane & 15) * 16
  return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(lut) + off);
}

// one slab's operands for one wave: A (G) fragments a[ks][m], B (x) fragments b[ks][n]
struct WgdFrag {
  bf16x8 a[2][2], b[2][2];
};

// the LDS reads of one slab's operands, issued together at the start of a round: B fragments
// (final), the A fragments' table masks and the dL/de pair (combined by wgd_finish at the
// round's end, after the MFMAs have covered the read latency)
struct WgdRaw {
  bf16x8 b[2][2];
  uint4 am[2][2];
  uint32_t gp[2];
};

__device__ __forceinline__ WgdRaw wgd_read(const uint16_t* Xt, const uint32_t (&mk)[2], const uint4* lut,
                                            const uint16_t* gs, int ul, const WgdLane& ln) {
  WgdRaw w;
  const uint16_t* gl = reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(gs) + ln.gsoff) + ul * DAD_H;
#pragma unroll
  for (int m = 0; m < 2; ++m) w.gp[m] = gl[32 * m];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int n = 0; n < 2; ++n) w.b[ks][n] = tr_frag(Xt, WGD_XP, 16 * ks, 32 * n);
#pragma unroll
    for (int m = 0; m < 2; ++m) w.am[ks][m] = wgd_amask(mk[m], lut, ln.lsel[ks], ln.slot);
  }
  return w;
}
__device__ __forceinline__ WgdFrag wgd_finish(const WgdRaw& w) {
  WgdFrag f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint4 s = w.am[ks][m];
      const uint32_t g = w.gp[m];
      f.a[ks][m] = __builtin_bit_cast(bf16x8, uint4{__builtin_amdgcn_perm(g, g, s.x), __builtin_amdgcn_perm(g, g, s.y),
                                                    __builtin_amdgcn_perm(g, g, s.z), __builtin_amdgcn_perm(g, g, s.w)});
    }
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int n = 0; n < 2; ++n) f.b[ks][n] = w.b[ks][n];
  return f;
}

template <bool F16>
__device__ __forceinline__ void wgd_mma(const WgdFrag& f, f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if constexpr (F16)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, f.a[ks][m]),
                                                             __builtin_bit_cast(f16x8, f.b[ks][n]), acc[m][n], 0, 0, 0);
        else
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[ks][m], f.b[ks][n], acc[m][n], 0, 0, 0);
      }
}

__device__ __forceinline__ int wgd_utt(const DadGeom& g, int s) {
  const int nsc = g.Bc * g.ncc;
  return s < nsc ? s / g.ncc : g.Bc + (s - nsc) / g.ncn;
}

// power of two 2^s with max_abs * 2^s in [2^14, 2^15) (1 for 0 or a non-finite max)
__device__ __forceinline__ int wgd_f16_exp(float max_abs) {
  if (!(max_abs > 0.0f) || !__builtin_isfinite(max_abs)) return 0;
  int e = 0;
  (void)frexpf(max_abs, &e);   // max_abs = f 2^e, f in [0.5, 1)
  return min(max(15 - e, -126), 126);
}

}  // namespace

// dad_prep_clean_load / _store with the row's address in SGPRs (u is wave-uniform): a buffer
// resource per row, the lane's column offset a loop-invariant register, the three 16-B / 8-B
// pieces at immediate offsets; non-temporal loads as in dad_prep_clean_load
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <bool STORE>
__device__ __forceinline__ void wgd_cp_load(const DadPrepArgs& a, int u, uint32_t loff, f32x4 (&v)[3],
                                            const StoreRowsW& sr) {
  const int uc = min(u, a.g.Bc * a.g.Tc - 1);
  const size_t srow = dad_clean_src_row<STORE>(a, uc, sr);
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xc + srow * DAD_D), (short)0, DAD_D * 4,
                                                   0x00020000);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, loff + 1024 * k, 0, 2));
}
template <bool F16>
__device__ __forceinline__ void wgd_cp_store(const DadPrepArgs& a, int u, uint32_t soff, const f32x4 (&v)[3]) {
  const int uc = min(u, a.g.Bc * a.g.Tc - 1);
  const auto r = __builtin_amdgcn_make_buffer_rsrc(a.x16 + (size_t)uc * DAD_D, (short)0, DAD_D * 2, 0x00020000);
#pragma unroll
  for (int k = 0; k < 3; ++k)
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{dad_pack2<F16>(v[k][0], v[k][1]), dad_pack2<F16>(v[k][2], v[k][3])}, r,
                                          soff + 512 * k, 0, 0);
}

// x-tile LDS buffers per slab group: a slab is staged two rounds before it is read, one barrier
// per two rounds (eight buffers and a barrier every four rounds measured neutral, round 3)
constexpr int WGD_NBUF = 4;
// one 256 h x WGD_DB d tile over slabs [s0, s1): fp32 partial
// CP: this launch also converts the NEXT step's clean rows into its prepared set (pc, when the
// step names its next batch): wave gw of GW takes rows gw, gw + GW, ...; two rows' loads go out in
// the first round of each block of NB rounds and are converted and stored at the start of the next
// block (an HBM miss under this load takes about as long as NB rounds); the rows left after the
// loop follow it.  CP = 1: padded next batch; CP = 2: store batch (Bc <= 64), source rows through
// the utterance table held in registers (StoreRowsW).
template <bool F16, int CP>
__device__ __forceinline__ void wgd_tile(const DadWgradArgs& a, const DadReduceArgs& ra, int s0, int s1, int dbase,
                                         float* outf, uint16_t* Xt, const uint4* lut, uint16_t* gs, float* red,
                                         const DadPrepArgs& pc, int gw, int GW) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane((tid >> 6) & 3);
  const int grp = __builtin_amdgcn_readfirstlane(tid >> 8);
  const DadGeom& g = a.g;
  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = f32x16{};
  float unscale = 1.0f;   // FP16: 2^-s_h of row h = 64 wv + lane
  const uint32_t cploff = (uint32_t)lane * 16u, cpsoff = (uint32_t)lane * 8u;   // CP: a row's lane columns
  for (int k = 0; DAD_PROBE_ON && k < 10; ++k)
    if (tid == 0 && blockIdx.x < 512) DAD_PROBE_SET(wgd_stamps, blockIdx.x * 10 + k, 0);
  const unsigned long long t0 = WGD_CLK();
  unsigned long long t1 = t0, t2 = t0;
  if (s0 < s1) {
    // group g takes slabs s0 + g, s0 + g + WGD_GROUPS, ...; all groups run nround rounds
    // (barriers); cntmin = the smallest group's slab count
    const int n = s1 - s0;
    const int nround = (n + WGD_GROUPS - 1) / WGD_GROUPS;
    const int mine = (n - grp + WGD_GROUPS - 1) / WGD_GROUPS;   // group 1 may have one slab fewer
    const int cntmin = n / WGD_GROUPS;
    const int u0 = wgd_utt(g, s0), nu = wgd_utt(g, s1 - 1) - u0 + 1;
    uint16_t* Xg = Xt + grp * (WGD_NBUF * DAD_SLAB * WGD_XP);   // this group's WGD_NBUF LDS buffers
    // dL/de_u[h] / max(1, len_u) of this split's utterances (thread = h of each group) as 16-bit;
    // the host bounds a split to WGD_MAXU slabs, hence utterances.  In each batch of eight
    // utterances group g builds entries 4g .. 4g+3 (KG per group).  The first batch's vector
    // loads (dL/dz, ECDA row and flag, length) go out before the slab prefetch, so their math
    // never waits on it.
    // FP16: row h of G is stored as fp16(v * 2^s_h), with 2^s_h putting max_u |v[u][h]| in
    // [2^14, 2^15) (wgd_f16_exp); both groups evaluate all KL = 8 utterances of a batch for that
    // max (the same arithmetic: identical s_h in both), so no barrier is needed, and the row
    // of the partial is multiplied back by 2^-s_h when it is stored.  Thread hh is lane hh & 63
    // of wave (hh >> 6) & 3 of its group: the wave that owns rows 64 wv .. 64 wv + 63.
    constexpr int KG = 8 / WGD_GROUPS;
    constexpr int KL = F16 ? 8 : KG;
    auto slot = [&](int k) { return F16 ? k : grp * KG + k; };   // utterance slot of evaluation k
    const int hh = tid & (DAD_H - 1);
    float w2[4], ec0[KL], vl0[KL];
    f32x4 gz0[KL];
    uint32_t ef0[KL];
#pragma unroll
    for (int c = 0; c < 4; ++c) w2[c] = ra.student[DAD_OFF_W2 + c * DAD_H + hh];
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int u = u0 + min(slot(k), nu - 1);
      ec0[k] = ra.ge_ecda[(size_t)u * DAD_H + hh];
      gz0[k] = *reinterpret_cast<const f32x4*>(ra.gzb + (size_t)u * DAD_C);
      ef0[k] = ra.eflag[u];
      vl0[k] = ra.vlen[u];
    }
    const int sfirst = s0 + grp;
    const WgdTable tab = wgd_table(g, min(sfirst + WGD_GROUPS * lane, s1 - 1), u0);
    WgdLane ln;
    {
      const int t = tid & 255;
      ln.xoff = (uint32_t)(((t >> 3) * DAD_D + dbase + (t & 7) * 8) * 2);
      ln.moff = (uint32_t)(((2 * wv) * 32 + (t & 31)) * 4);
      ln.slot = (uint32_t)(lane & (WGD_LUT_SLOTS - 1)) << 4;
      ln.lsel[0] = 0x0c0c0000u | ((4u + (uint32_t)(lane >> 5)) << 8);   // mask byte 0 / 1 (ks = 0)
      ln.lsel[1] = 0x0c0c0000u | ((6u + (uint32_t)(lane >> 5)) << 8);   // mask byte 2 / 3 (ks = 1)
      ln.gsoff = (uint32_t)(((2 * wv) * 32 + (lane & 31)) * 2);
      ln.nrows = g.Bc * g.Tc + (a.warmup ? 0 : g.Bn * g.Tn);
    }
    const int jlast = max(mine - 1, 0);
    WgdSlab r[WGD_DEPTH];
    // loads are unconditional (slab index clamped at the group's last slab): conditional
    // loads make the compiler merge the paths' pending counts into a vmcnt(0) drain
#pragma unroll
    for (int k = 0; k < WGD_DEPTH; ++k) wgd_load(a, tab, min(k, jlast), sfirst, ln, r[k]);
    const unsigned long long ta = WGD_CLK();
    // the table: the first batch's values stay in registers (v0); FP16 takes the row's largest
    // |v| first (a second pass recomputes later batches), then writes the scaled values
    auto ge_table = [&](auto ex_tag) {
      constexpr bool EX = decltype(ex_tag)::value;
      auto batch = [&](int ul0, float (&v)[KL]) {
#pragma unroll
        for (int k = 0; k < KL; ++k) {   // the batch's loads in flight (index clamped)
          const int u = u0 + min(ul0 + slot(k), nu - 1);
          v[k] = ul0 == 0 ? fused_ge1_v<EX>(ra, g.Bc, u, hh, w2, gz0[k], ef0[k], ec0[k]) / fmaxf(vl0[k], 1.0f)
                          : fused_ge1<EX>(ra, g.Bc, u, hh, w2) / fmaxf(ra.vlen[u], 1.0f);
        }
      };
      auto put = [&](int ul0, const float (&v)[KL], float scale) {
#pragma unroll
        for (int k = 0; k < KG; ++k) {
          const int uk = ul0 + grp * KG + k;
          const float x = v[F16 ? grp * KG + k : k];
          if (uk < nu) gs[uk * DAD_H + hh] = dad_half_bits(F16 ? x * scale : x, F16);
        }
      };
      float v0[KL];
      batch(0, v0);
      float scale = 1.0f;
      if constexpr (F16) {
        float mx = 0.0f;
#pragma unroll
        for (int k = 0; k < KL; ++k) mx = fmaxf(mx, fabsf(v0[k]));   // (clamped slots repeat a real one)
        for (int ul0 = 8; ul0 < nu; ul0 += 8) {
          float v[KL];
          batch(ul0, v);
#pragma unroll
          for (int k = 0; k < KL; ++k) mx = fmaxf(mx, ul0 + k < nu ? fabsf(v[k]) : 0.0f);
        }
        const int s = wgd_f16_exp(mx);
        scale = __builtin_ldexpf(1.0f, s);
        unscale = __builtin_ldexpf(1.0f, -s);
      }
      put(0, v0, scale);
      for (int ul0 = 8; ul0 < nu; ul0 += 8) {
        float v[KL];
        batch(ul0, v);
        put(ul0, v, scale);
      }
    };
    if (ra.keep1) ge_table(std::true_type{});
    else ge_table(std::false_type{});
    const unsigned long long tb = WGD_CLK();
    // slabs 0 .. SD-1 of each group into buffers 0 .. SD-1; their ring slots reload slabs
    // WGD_DEPTH .. WGD_DEPTH + SD - 1
    constexpr int NB = WGD_NBUF, SD = WGD_NBUF / 2;   // LDS buffers, staging distance (rounds)
    static_assert(WGD_DEPTH == 4 && NB == 4, "dad_wgrad_direct: four ring slots, 4 LDS buffers");
    int ulq[SD];   // utterance slot and row masks of slabs j .. j+SD-1 (by j mod SD)
    uint32_t mwq[SD][2];
#pragma unroll
    for (int q = 0; q < SD; ++q) {
      if (mine > q) wgd_stage(r[q], Xg + q * (DAD_SLAB * WGD_XP));
      ulq[q] = r[q].ul;
      mwq[q][0] = r[q].mw[0];
      mwq[q][1] = r[q].mw[1];
    }
#pragma unroll
    for (int q = 0; q < SD; ++q) wgd_load(a, tab, min(WGD_DEPTH + q, jlast), sfirst, ln, r[q]);
    const unsigned long long tc = WGD_CLK();
    __syncthreads();
    t1 = WGD_CLK();
    WGD_ACC(3, ta - t0); WGD_ACC(6, tb - ta); WGD_ACC(7, tc - tb); (void)ta; (void)tb; (void)tc;
    // round j: read slab j's operands from buffer j % NB into registers | MFMAs of slab j-1 from
    // the registers read in round j-1 (so they never wait on LDS) | stage slab j+SD into
    // buffer (j+SD) % NB from ring slot (j+SD) % 4 and reload that slot with slab j+SD+4.  A slab
    // is staged SD = NB/2 rounds before it is read, so one barrier per SD rounds (after rounds
    // j = SD-1 mod SD) orders every staging before its reads and every read before its buffer is
    // restaged.
    WgdFrag F;
    auto round = [&](int jr, int k, bool prev, bool comp, bool stage, bool bar) {
      const unsigned long long c0 = WGD_CLK();
      const int nk = (k + SD) % WGD_DEPTH;
      WgdRaw R;
      if (comp) R = wgd_read(Xg + (k % NB) * (DAD_SLAB * WGD_XP), mwq[k % SD], lut, gs, ulq[k % SD], ln);
      __builtin_amdgcn_sched_barrier(0);   // reads first, their latency under the MFMAs
      if (prev) wgd_mma<F16>(F, acc);
      if (stage) wgd_stage(r[nk], Xg + ((k + SD) % NB) * (DAD_SLAB * WGD_XP));
      ulq[k % SD] = r[nk].ul;
      mwq[k % SD][0] = r[nk].mw[0];
      mwq[k % SD][1] = r[nk].mw[1];
      wgd_load(a, tab, min(jr + SD + WGD_DEPTH, jlast), sfirst, ln, r[nk]);
      __builtin_amdgcn_sched_barrier(0);
      if (comp) F = wgd_finish(R);
      const unsigned long long c1 = WGD_CLK();
      if (bar) __syncthreads();
      WGD_ACC(4, c1 - c0); WGD_ACC(5, WGD_CLK() - c1); WGD_ACC(8, 1);
      (void)c0; (void)c1;
    };
    // round 0, then blocks of NB rounds (NB is a multiple of the 4 ring slots) in which both
    // groups have every step (no early exits: an exit inside the block would reach the loop
    // header with a different load order and force vmcnt(0) there; buffers and ring slots are
    // compile-time: j = 1 mod NB at a block start), then the last rounds with per-group flags and
    // the final MFMAs.  Both groups run the same rounds, so the barriers match.
    round(0, 0, false, mine > 0, SD < mine, false);
    int j = 1;
    int prow = gw;        // CP: this wave's next clean row of the next step
    const StoreRowsW srw = CP == 2 ? dad_store_rows_w(pc, lane) : StoreRowsW{};
    f32x4 pv[2][3];
    bool pending = false; // CP: rows prow - 2 GW, prow - GW loaded, not yet stored
    f32x4 po[2][3];       // CP two blocks ahead: rows prow - 4 GW, prow - 3 GW (loaded two blocks ago)
    bool pend2 = false;
    for (; j + NB - 1 + SD < cntmin; j += NB) {   // every round stages slab j + k + SD < cntmin
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if constexpr (CP) {
          if (k == 0) {
            // the rows loaded two blocks (2 NB rounds) ago, then this block's two
            if (pend2) {
              wgd_cp_store<F16>(pc, prow - 4 * GW, cpsoff, po[0]);
              wgd_cp_store<F16>(pc, prow - 3 * GW, cpsoff, po[1]);
            }
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
              for (int e = 0; e < 3; ++e) po[q][e] = pv[q][e];
            pend2 = pending;
            wgd_cp_load<CP == 2>(pc, prow, cploff, pv[0], srw);
            wgd_cp_load<CP == 2>(pc, prow + GW, cploff, pv[1], srw);
            prow += 2 * GW;
            pending = true;
          }
        }
        round(j + k, (k + 1) % NB, true, true, true, (k + 1) % SD == SD - 1);
      }
    }
#pragma unroll
    for (int k = 0; k < NB + SD + 1; ++k)   // nround - j <= NB + SD
      if (j + k < nround)
        round(j + k, (k + 1) % NB, j + k - 1 < mine, j + k < mine, j + k + SD < mine, (k + 1) % SD == SD - 1);
    if (nround - 1 < mine) wgd_mma<F16>(F, acc);
    if constexpr (CP) {
      if (pend2) {
        wgd_cp_store<F16>(pc, prow - 4 * GW, cpsoff, po[0]);
        wgd_cp_store<F16>(pc, prow - 3 * GW, cpsoff, po[1]);
      }
      if (pending) {
        wgd_cp_store<F16>(pc, prow - 2 * GW, cpsoff, pv[0]);
        wgd_cp_store<F16>(pc, prow - GW, cpsoff, pv[1]);
      }
      for (; prow < pc.g.Bc * pc.g.Tc; prow += GW) {   // the rows the loop left
        wgd_cp_load<CP == 2>(pc, prow, cploff, pv[0], srw);
        wgd_cp_store<F16>(pc, prow, cpsoff, pv[0]);
      }
    }
    t2 = WGD_CLK();
  } else if constexpr (CP != 0) {
    const StoreRowsW srw = CP == 2 ? dad_store_rows_w(pc, lane) : StoreRowsW{};
    for (int prow = gw; prow < pc.g.Bc * pc.g.Tc; prow += GW) {
      f32x4 pv[3];
      wgd_cp_load<CP == 2>(pc, prow, cploff, pv, srw);
      wgd_cp_store<F16>(pc, prow, cpsoff, pv);
    }
  }
  const int kh = lane >> 5;
  if constexpr (WGD_GROUPS == 2) {
    __syncthreads();   // red aliases the x tiles: every group's last reads are done
    // exchange halves: group 0 finishes h tile 2w (+ group 1's partial), group 1 tile 2w+1
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (m != grp)
#pragma unroll
        for (int nn = 0; nn < 2; ++nn)
#pragma unroll
          for (int rr = 0; rr < 16; ++rr)
            red[((2 * wv + m) * 32 + dad_acc_row(rr, kh)) * WGD_DB + 32 * nn + (lane & 31)] = acc[m][nn][rr];
    __syncthreads();
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
    if (WGD_GROUPS == 1 || m == grp)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int h = (2 * wv + m) * 32 + dad_acc_row(rr, kh);
          const int d = 32 * nn + (lane & 31);
          const float v = acc[m][nn][rr] + (WGD_GROUPS == 2 ? red[h * WGD_DB + d] : 0.0f);
          // FP16: 2^-s_h of row h, held by lane h - 64 wv of this wave (ds_bpermute)
          outf[(size_t)h * DAD_D + dbase + d] = F16 ? v * __shfl(unscale, h - 64 * wv, 64) : v;
        }
  if constexpr (WGD_GROUPS == 2) __syncthreads();   // red free for the next tile
  WGD_ACC(0, t1 - t0); WGD_ACC(1, t2 - t1); WGD_ACC(2, WGD_CLK() - t2);
  (void)t0; (void)t1; (void)t2;
}

// the byte table of the A-fragment masks, 16 slot copies per byte (wgd_amask)
__device__ __forceinline__ void wgd_lut(uint4* lut) {
  // consecutive threads store consecutive 16-B slots (conflict-free stores); entry i is byte
  // i / 16, the byte's four dwords by sign-extended bit fields
#pragma unroll
  for (int k = 0; k < (WGD_LUT + WGD_THREADS - 1) / WGD_THREADS; ++k) {
    const int i = k * WGD_THREADS + threadIdx.x;
    if (WGD_LUT < WGD_THREADS && i >= WGD_LUT) break;
    const int t = i / WGD_LUT_SLOTS;
    uint32_t e[4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
      e[p] = (((t >> (2 * p)) & 1) ? 0x00000100u : 0x00000c0cu) | (((t >> (2 * p + 1)) & 1) ? 0x01000000u : 0x0c0c0000u);
    lut[i] = uint4{e[0], e[1], e[2], e[3]};
  }
}

// LDS of the weight-gradient workgroups (160 KB with the dL/de table): the x tiles, then the
// mask table; the end-of-tile exchange (red, 64 KB) reuses the x tiles and the spare space
// after them (the table stays intact for the next tile)
constexpr int WGD_XT = WGD_GROUPS * WGD_NBUF * DAD_SLAB * WGD_XP;   // 16-bit elements
constexpr int WGD_RED = WGD_GROUPS == 2 ? DAD_H * WGD_DB : 1;
struct __attribute__((aligned(16))) WgdSmem {
  uint4 lut[WGD_LUT];   // first: its 64 KB sit at LDS offsets 0 .. 65535, so a table read needs no base add
                        // (the ds_read offset field holds 16 bits)
  union {
    uint16_t xt[WGD_XT];
    float red[WGD_RED];
  } a;
};

__device__ double extra_block(const DadReduceArgs& a, int e, int tid, float (*xs)[16][6]);


template <bool F16, int CP>
__device__ __forceinline__ void wgrad_direct_body(const DadWgradArgs& a, const DadReduceArgs& ra, const DadPrepArgs& pc) {
  __shared__ WgdSmem S;
  __shared__ __attribute__((aligned(16))) uint16_t gs[WGD_MAXU * DAD_H];
  uint16_t* Xt = S.a.xt;
  // XCD-aware tile order (grid is a multiple of 8; workgroups go round-robin over the 8
  // XCDs): each XCD takes a consecutive run of tiles, so the column blocks of one split,
  // which read the same ReLU' row masks, share an L2
  const int per_xcd = gridDim.x >> 3;
  const int tile = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (tile >= a.ntiles) {
    // The first WGD_XWG spare workgroups do dad_reduce's extra blocks (db1, dW2, loss totals):
    // their inputs are ready before this launch and the work then overlaps the GEMM instead of
    // trailing the reduction.  Two extra blocks at a time, one per 256-thread half, combining
    // in the (otherwise unused) x-tile LDS.
    const int xi = tile - a.ntiles;
    if (xi >= WGD_XWG) return;
    static_assert(sizeof(S.a) >= 2 * 16 * 16 * 6 * sizeof(float), "extra-block scratch fits the x tile");
    double* wred = reinterpret_cast<double*>(S.lut);   // (the mask table is not used here)
    const int half = threadIdx.x >> 8, htid = threadIdx.x & 255;
    float (*xs)[16][6] = reinterpret_cast<float (*)[16][6]>(S.a.red) + 16 * half;
    constexpr int per_wg = DAD_REDUCE_XBLK / WGD_XWG;
    constexpr int NB = DAD_REDUCE_BLOCKS - DAD_REDUCE_XBLK;
    for (int r = 0; r < per_wg; r += 2) {
      const int e = xi * per_wg + r + half;
      const double v = dad_wave_sum_d(extra_block(ra, e, htid, xs));
      if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = v;
      __syncthreads();
      if (htid == 0 && ra.want_norm)
        ra.normpart[NB + e] = (float)(((wred[4 * half] + wred[4 * half + 1]) + wred[4 * half + 2]) + wred[4 * half + 3]);
      __syncthreads();
    }
    return;
  }
  const int split = tile / WGD_NDB, dblk = tile - split * WGD_NDB;
  const int total = wg_total(a);
  const int per = (total + a.splits - 1) / a.splits;
  const int s0 = split * per, s1 = min(total, s0 + per);
  wgd_lut(S.lut);   // (the tile's first barrier orders it before the first read)
  const int gw = __builtin_amdgcn_readfirstlane(tile * (WGD_THREADS / 64) + (int)(threadIdx.x >> 6));
  wgd_tile<F16, CP>(a, ra, s0, s1, dblk * WGD_DB, a.wpart + (size_t)split * DAD_H * DAD_D, Xt, S.lut, gs, S.a.red, pc,
                    gw, a.ntiles * (WGD_THREADS / 64));
}

__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct(DadWgradArgs a, DadReduceArgs ra) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<false, 0>(a, ra, DadPrepArgs{});
}
__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct_f16(DadWgradArgs a, DadReduceArgs ra) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<true, 0>(a, ra, DadPrepArgs{});
}
__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct_cp(DadWgradArgs a, DadReduceArgs ra, DadPrepArgs pc) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<false, 1>(a, ra, pc);
}
__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct_f16_cp(DadWgradArgs a, DadReduceArgs ra,
                                                                         DadPrepArgs pc) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<true, 1>(a, ra, pc);
}
__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct_cps(DadWgradArgs a, DadReduceArgs ra, DadPrepArgs pc) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<false, 2>(a, ra, pc);
}
__global__ __launch_bounds__(WGD_THREADS, 1) void dad_wgrad_direct_f16_cps(DadWgradArgs a, DadReduceArgs ra,
                                                                          DadPrepArgs pc) {
  DAD_GUARD_BLOCK(WGD_THREADS);
  wgrad_direct_body<true, 2>(a, ra, pc);
}

// ---------------------------------------------------------------- reduce + squared norms
// blocks [0, NB): DAD_REDUCE_COLS floats of dW1 each (+ squared-norm partial).
// blocks NB + e, e < DAD_REDUCE_XBLK: hidden units 16e .. 16e+15 of
//   db1[h]    = sum_r dL/de[r][h] / max(1, len_r) * active_count[r][h]      (autograd of b1)
//   dW2[c][h] = sum_r dL/dz[r][c] * dropout(e_r)[h]   (fused step; the tail no longer does it)
// their squared-norm share, and (e = 0) the b2 norm share and the loss totals
// (I/train.py:462-466).  Thread = (hidden unit hl, row group rg): rows rg, rg+16, ...;
// the 16 row groups are combined in fixed order (deterministic).
static_assert(DAD_REDUCE_THREADS == 256 && DAD_H == 16 * DAD_REDUCE_XBLK, "extra blocks: 16 h x 16 row groups");

// run by 256 threads (tid = 0..255 of a workgroup or of half of one), combining in xs
template <bool EX>
__device__ double extra_block_t(const DadReduceArgs& a, int e, int tid, float (*xs)[16][6]) {
  const int hl = tid & 15, rg = tid >> 4;
  const int h = 16 * e + hl;
  const DadGeom& g = a.g;
  const int nb = g.Bc + (a.warmup ? 0 : g.Bn);
  const bool fused = a.gzb != nullptr;
  const bool ecda = a.ge_ecda != nullptr;
  float w2[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (fused)
#pragma unroll
    for (int c = 0; c < 4; ++c) w2[c] = a.student[DAD_OFF_W2 + c * DAD_H + h];
  float db = 0.0f, gw[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // rows rg, rg + 16, ... in batches of 8 whose loads are all issued before any is used
  // (index clamped, contribution masked): one memory round trip per batch, not per row
  for (int r0 = rg; r0 < nb; r0 += 16 * 8) {
    float gv[8], kv[8], rl[8], ct[8], em[8];
    f32x4 gzv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int r = min(r0 + 16 * k, nb - 1);
      kv[k] = 1.0f;
      if (fused) {
        gv[k] = fused_ge1<EX>(a, g.Bc, r, h, w2, &kv[k]);
        const int erow = r >= g.Bc ? g.Bn + r : r;   // strong row b lives at Bc + Bn + b
        em[k] = a.emb[(size_t)erow * DAD_H + h];
        gzv[k] = *reinterpret_cast<const f32x4*>(a.gzb + (size_t)r * DAD_C);
      } else {
        gv[k] = a.ge[(size_t)r * DAD_H + h];
        if (ecda) gv[k] += a.ge_ecda[(size_t)r * DAD_H + h];
        em[k] = 0.0f;
        gzv[k] = f32x4{};
      }
      rl[k] = a.vlen[r];
      ct[k] = a.cnt_tot[(size_t)r * DAD_H + h];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (r0 + 16 * k >= nb) break;
      db += gv[k] / fmaxf(rl[k], 1.0f) * ct[k];
      if (fused) {
        // dW2[c][h] = sum_u dL/dz[u][c] * dropout(e_u)[h]  (student clean / strong embeddings)
        const float d = em[k] * kv[k];
#pragma unroll
        for (int c = 0; c < 4; ++c) gw[c] += gzv[k][c] * d;
      }
    }
  }
  xs[rg][hl][0] = db;
#pragma unroll
  for (int c = 0; c < 4; ++c) xs[rg][hl][1 + c] = gw[c];
  __syncthreads();
  double sq = 0.0;
  if (tid < 16 * 5) {
    const int k = tid >> 4, hh = tid & 15;   // k: 0 = db1, 1..4 = dW2 row c = k-1
    float v = xs[0][hh][k];
    for (int q = 1; q < 16; ++q) v += xs[q][hh][k];
    if (k == 0) {
      a.grad[DAD_OFF_B1 + 16 * e + hh] = v;
      sq = (double)v * v;
    } else if (a.tailf) {
      if (fused) a.grad[DAD_OFF_W2 + (k - 1) * DAD_H + 16 * e + hh] = v;
      else v = a.grad[DAD_OFF_W2 + (k - 1) * DAD_H + 16 * e + hh];
      sq = (double)v * v;
    }
  }
  if (e == 0 && a.tailf && tid >= 96 && tid < 100) {
    const float gb = a.grad[DAD_OFF_B2 + tid - 96];
    sq += (double)gb * gb;
  }
  if (e == 0 && a.tailf && tid == 128) {
    const float* tf = a.tailf;
    const float ecda_l = ((tf[DAD_T_ECDA_TERM] + tf[DAD_T_ECDA_TERM + 1]) + tf[DAD_T_ECDA_TERM + 2]) +
                         tf[DAD_T_ECDA_TERM + 3];
    const float ce = tf[DAD_T_CE], kl = tf[DAD_T_KL];
    float* ex = a.grad + DAD_NPARAM;
    // a pooling timeout in the tail launch (DAD_POOL_ABORT): NaN total, so dad_optim (on every DP
    // rank, after the all-reduce) skips this step's update
    const bool abort = a.pool_abort != nullptr && __hip_atomic_load(a.pool_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    ex[12] = abort ? __builtin_nanf("") : ce + a.w_kl * kl + a.w_ecda * ecda_l;
    ex[13] = ce;
    ex[14] = kl;
    ex[15] = ecda_l;
  }
  return sq;
}
__device__ double extra_block(const DadReduceArgs& a, int e, int tid, float (*xs)[16][6]) {
  return a.keep1 ? extra_block_t<true>(a, e, tid, xs) : extra_block_t<false>(a, e, tid, xs);
}

static_assert(DAD_REDUCE_THREADS == 4 * (DAD_REDUCE_COLS / 4), "dad_reduce: 4 split groups x float4 columns");
static_assert(DAD_REDUCE_BLOCKS <= DAD_NORM_BLOCKS, "norm partials must fit the workspace");
static_assert((DAD_NPARAM + 1023) / 1024 <= DAD_NORM_BLOCKS, "dad_norm partials must fit the workspace");
__global__ __launch_bounds__(DAD_REDUCE_THREADS) void dad_reduce(DadReduceArgs a) {
  DAD_GUARD_BLOCK(DAD_REDUCE_THREADS);
  __shared__ double red[DAD_REDUCE_THREADS / 64];
  __shared__ f32x4 part[4][DAD_REDUCE_COLS / 4 > DAD_H / 4 ? DAD_REDUCE_COLS / 4 : DAD_H / 4];
  const int tid = threadIdx.x;
  constexpr int NB = DAD_REDUCE_BLOCKS - DAD_REDUCE_XBLK;
  double sq = 0.0;
  if (blockIdx.x < NB) {
    const int col = tid & (DAD_REDUCE_COLS / 4 - 1), kg = tid / (DAD_REDUCE_COLS / 4);
    const size_t e0 = (size_t)blockIdx.x * DAD_REDUCE_COLS + (size_t)col * 4;
    f32x4 s = f32x4{};
#pragma unroll 4
    for (int k = kg; k < a.splits; k += 4) s += *reinterpret_cast<const f32x4*>(a.wpart + (size_t)k * DAD_H * DAD_D + e0);
    part[kg][col] = s;
    __syncthreads();
    if (kg == 0) {
      const f32x4 t = ((part[0][col] + part[1][col]) + part[2][col]) + part[3][col];
      *reinterpret_cast<f32x4*>(a.grad + DAD_OFF_W1 + e0) = t;
      for (int e = 0; e < 4; ++e) sq += (double)t[e] * t[e];
    }
  } else {
    __shared__ float xsx[16][16][6];
    sq = extra_block(a, blockIdx.x - NB, tid, xsx);
  }
  if (!a.want_norm) return;
  double v = dad_wave_sum_d(sq);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int k = 0; k < DAD_REDUCE_THREADS / 64; ++k) t += red[k];
    a.normpart[blockIdx.x] = (float)t;
  }
}

// FP16/BF16 step (the extra blocks ran on spare dad_wgrad_direct workgroups): one wave per
// DAD_REDUCE_COLS columns, 4 per lane, the splits summed in split order with every partial's
// load issued first (batches of 8, index clamped, +0 past the last split), the squared-norm
// partial a wave reduction: no LDS, no barrier (dad_reduce's 4 row groups met through LDS
// twice).
static_assert(DAD_REDUCE_COLS == 4 * 64, "dad_reduce_w: one wave, 4 columns per lane");
__global__ __launch_bounds__(64) void dad_reduce_w(DadReduceArgs a) {
  DAD_GUARD_BLOCK(64);
  const int lane = threadIdx.x;
  const size_t e0 = (size_t)blockIdx.x * DAD_REDUCE_COLS + 4 * (size_t)lane;
  constexpr int KB = 8;
  f32x4 t = f32x4{};
  for (int k0 = 0; k0 < a.splits; k0 += KB) {
    f32x4 v[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k)
      v[k] = *reinterpret_cast<const f32x4*>(a.wpart + (size_t)min(k0 + k, a.splits - 1) * DAD_H * DAD_D + e0);
#pragma unroll
    for (int k = 0; k < KB; ++k) t += k0 + k < a.splits ? v[k] : f32x4{};
  }
  *reinterpret_cast<f32x4*>(a.grad + DAD_OFF_W1 + e0) = t;
  if (!a.want_norm) return;
  double sq = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) sq += (double)t[e] * t[e];
  sq = dad_wave_sum_d(sq);
  if (lane == 0) a.normpart[blockIdx.x] = (float)sq;
}

// Data-parallel path: after the SUM all-reduce, average (grads, thresholds, losses) and
// recompute the squared-norm partials over the averaged gradient.
__global__ __launch_bounds__(256) void dad_norm(float* grad, float* normpart, float inv) {
  __shared__ double red[4];
  const int tid = threadIdx.x;
  double sq = 0.0;
  const size_t n0 = (size_t)blockIdx.x * 1024;
  for (int k = 0; k < 4; ++k) {
    const size_t e = n0 + (size_t)k * 256 + tid;
    if (e < DAD_NPARAM) {
      const float g = grad[e] * inv;
      grad[e] = g;
      sq += (double)g * g;
    }
  }
  if (blockIdx.x == 0 && tid < DAD_GRAD_EXTRA) {
    float* ex = grad + DAD_NPARAM;
    if (tid < 4 || tid >= 12) ex[tid] *= inv;   // thresholds and losses are means; sums stay sums
  }
  double v = dad_wave_sum_d(sq);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) normpart[blockIdx.x] = (float)(((red[0] + red[1]) + red[2]) + red[3]);
}
