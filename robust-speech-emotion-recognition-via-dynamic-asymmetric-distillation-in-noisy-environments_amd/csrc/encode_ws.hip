// W-stationary 16-bit encoder: the throughput-mode forward of all three encoder passes, with
// fp16 (default throughput mode, 11-bit significand) or bf16 MFMA operands and fp32 accumulation.
//
// Replaces, per step (I/train.py:399,406-410,439):
//   student_encoder(clean)                         Emotion2VecEncoder.forward, I/model.py:18-41
//   teacher_encoder(weak_augment(noisy))           + DataAugmentation.weak_augment, I/utils.py:328-331
//   student_encoder(strong_augment(noisy))         + strong_augment/_apply_temporal_masking, I/utils.py:333-375
// and emits what the rest of the step consumes: per-32-row-slab pooled ReLU sums and active
// counts, the ReLU'-and-valid row masks, and the 16-bit student inputs (clean and strong-augmented
// rows, the weight gradient's operand).
//
// Shape of the work: out[rows][256] = x[rows][768] . W1^T with tens of thousands of rows and
// W1 only 384 KB in 16 bits.  So W1 is STATIONARY: a persistent workgroup holds all 256 hidden
// units of ONE network's W1 in its register file (each wave 256/WAVES hidden units x 768 k,
// read in place as MFMA B operands) and streams 16-row sub-slabs of x through LDS:
//
//   HBM fp32 rows --LDS-DMA (global_load_lds_dwordx4, 2 stages x 48 KB in flight)--> raw ring
//   raw ring --augment (counter-RNG Box-Muller, feature mask, temporal zero) + cvt f16/bf16-->
//      16-bit tile ring (2 x 24 KB; 16-B chunks XOR-swizzled by row: conflict-free A reads)
//   tile --ds_read_b128 A fragments--> v_mfma_f32_16x16x32_{f16,bf16} against the resident W1
//   accumulators --bias, ReLU, valid mask, row sums, ballots--> slab partials + ReLU' bits
//
// Each x element is fetched once per network that consumes it and augmented once.  Roles are
// per workgroup: TEACHER workgroups (teacher W1) run the weak-augmented noisy slabs, STUDENT
// workgroups (student W1) the clean slabs and the strong-augmented noisy slabs.  Jobs (32-row
// slabs) are split into contiguous, cost-weighted ranges (host: ws_split in dad_abi.hip).
//
// Pipeline per wave (iteration q = sub-slab q of the workgroup's range):
//   wait for the wave's own DMA of sub-slab q+1 (counted vmcnt: the stores and the youngest
//   DMA batch stay in flight) -> MFMA(q) with convert(q+1)'s units issued between its k-steps
//   -> epilogue(q) -> DMA of sub-slab q+3 into the raw stage convert(q+1) just freed -> barrier.
// A sub-slab without a valid row (e.g. rows 304..319 of a 300-frame utterance) is neither
// converted nor multiplied.  The first two sub-slabs' DMAs are issued ahead of the resident W1
// load, so sub-slab 0 is converted while W1 streams in.
#include <type_traits>

#include "dad_common.h"
#include "dad_kernels.h"
#include "dad_probe.h"

// per-workgroup wave-0 timeline of the stamps build (dad_probe.h): [start, after prologue, end
// (100 MHz wall clock), role<<16 | sub-slabs, then wave-0 cycles summed over the loop in: DMA
// wait, MFMA, convert, epilogue, DMA issue, barrier]
DAD_PROBE_BUFFER(ws_stamps, 4096 * 10)
#define WS_CLK() DAD_PROBE_CLK()
#define WS_STAMP(k, v) \
  if (threadIdx.x == 0 && blockIdx.x < 4096) DAD_PROBE_SET(ws_stamps, blockIdx.x * 10 + (k), (v))
#define WS_PHASES(c0, c1, c2, c3, c4, c5)                                                    \
  do {                                                                                       \
    const unsigned long long c6_ = WS_CLK();                                                 \
    if (DAD_PROBE_ON && threadIdx.x == 0 && blockIdx.x < 4096) {                             \
      const int i_ = blockIdx.x * 10;                                                        \
      DAD_PROBE_ADD(ws_stamps, i_ + 4, c1 - c0); DAD_PROBE_ADD(ws_stamps, i_ + 5, c2 - c1);  \
      DAD_PROBE_ADD(ws_stamps, i_ + 6, c3 - c2); DAD_PROBE_ADD(ws_stamps, i_ + 7, c4 - c3);  \
      DAD_PROBE_ADD(ws_stamps, i_ + 8, c5 - c4); DAD_PROBE_ADD(ws_stamps, i_ + 9, c6_ - c5); \
    }                                                                                        \
    (void)c0; (void)c1; (void)c2; (void)c3; (void)c4; (void)c5; (void)c6_;                   \
  } while (0)

namespace {

constexpr int kSub = 16;                       // rows per sub-slab (one MFMA M tile)
constexpr int kKS = DAD_D / 32;                // 24 k-steps of v_mfma_f32_16x16x32_{f16,bf16}
constexpr int kRawRow = DAD_D * 4;             // 3072 B
constexpr int kRawStage = kSub * kRawRow;      // 48 KB
constexpr int kTileRow = DAD_D * 2;            // 1536 B
constexpr int kTile = kSub * kTileRow;         // 24 KB
// tiles first: every A-fragment / tile address then fits ds_read/ds_write's 16-bit immediate
constexpr int kOffTile = 0;
constexpr int kOffRaw = 2 * kTile;             // 48 KB
constexpr int kOffFK = kOffRaw + 2 * kRawStage;  // 144 KB: feature keep flags f32[768]
constexpr int kOffVB = kOffFK + DAD_D * 4;     // valid bits u32[DAD_ENC_WS_MAXJ]
constexpr int kLds = kOffVB + 4 * DAD_ENC_WS_MAXJ;
static_assert(kLds <= 160 * 1024, "LDS budget");

enum { KIND_CLEAN = 0, KIND_WEAK = 1, KIND_STRONG = 2 };

// Every scalar the kernel needs, copied out of the kernel arguments once: a select between
// two argument fields must not become a select between their addresses (which drags the
// argument block into scratch and makes every job field a VGPR).
struct Ctx {
  int Bc, Tc, ncc, tpc, Bn, Tn, ncn, tpn;
  uint32_t mcc, mcn;     // division magics for ncc / ncn (fast_div)
  int nsc, nsn, Jc, Js;
  int mask_len, start_hi;
  const float* xc; const float* xn;
  DadStoreRows src;
  const uint8_t* mc; const uint8_t* mn;
  const float* nw; const float* ns; const float* u; const int64_t* start;
  uint32_t key_weak, key_strong, key_feat, key_tstart;
  float wstd, sstd, feat_p;
  float* part_sum; float* part_cnt; uint32_t* bits;
  uint16_t* xs; uint16_t* xsn;   // 16-bit copies of the student's MFMA input: clean rows, strong rows
};

__device__ __forceinline__ Ctx ctx_of(const DadEncodeArgs& a) {
  Ctx c;
  c.Bc = a.g.Bc; c.Tc = a.g.Tc; c.ncc = a.g.ncc; c.tpc = a.g.tpc;
  c.Bn = a.g.Bn; c.Tn = a.g.Tn; c.ncn = a.g.ncn; c.tpn = a.g.tpn;
  c.nsc = c.Bc * c.ncc; c.nsn = c.Bn * c.ncn;
  c.mcc = c.ncc > 1 ? 0xffffffffu / (uint32_t)c.ncc + 1u : 0u;
  c.mcn = c.ncn > 1 ? 0xffffffffu / (uint32_t)c.ncn + 1u : 0u;
  c.Jc = c.nsc; c.Js = a.warmup ? 0 : c.nsn;
  c.mask_len = a.mask_len; c.start_hi = a.start_hi;
  c.xc = a.xc; c.xn = a.xn; c.src = a.src; c.mc = a.mc; c.mn = a.mn;
  c.nw = a.nw; c.ns = a.ns; c.u = a.u; c.start = a.start;
  c.key_weak = a.key_weak; c.key_strong = a.key_strong; c.key_feat = a.key_feat; c.key_tstart = a.key_tstart;
  c.wstd = a.weak_std; c.sstd = a.strong_std; c.feat_p = a.feat_p;
  c.part_sum = a.part_sum; c.part_cnt = a.part_cnt; c.bits = a.bits;
  c.xs = a.xs16; c.xsn = a.xs16 + (size_t)c.Bc * c.Tc * DAD_D;
  return c;
}

// n / d for the slab counts per utterance: m = floor(2^32 / d) + 1 (0 for d = 1) is exact for
// n * d < 2^32; one scalar multiply-high instead of a ~40-instruction scalar division on a
// path every sub-slab takes several times
__device__ __forceinline__ int fast_div(int n, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)n, m) : n;
}

struct Job {
  int kind, b, c, T;
  long row0;        // [b][T] row of frame 0
  long sum_slab;    // part_sum slab
  long cnt_slab;    // part_cnt slab = ReLU' row-mask slab (student only)
  long src0;        // source row of frame 0: row0, or the store row (store mode)
  int srcT;         // source frames: T, or the utterance's length (store mode)
};

// job j of the workgroup's role list: teacher -> weak slab j; student -> clean slab j, then
// strong slab j - Jc.  Slab numbering matches dad_pool / the weight gradient.
__device__ __forceinline__ Job job_of(const Ctx& C, bool teacher, int j) {
  Job J;
  const bool noisy = teacher || j >= C.Jc;
  const int s = (teacher || j < C.Jc) ? j : j - C.Jc;
  const int nc = noisy ? C.ncn : C.ncc;
  J.kind = teacher ? KIND_WEAK : (noisy ? KIND_STRONG : KIND_CLEAN);
  J.b = fast_div(s, noisy ? C.mcn : C.mcc);
  J.c = s - J.b * nc;
  J.T = noisy ? C.Tn : C.Tc;
  J.row0 = (long)J.b * J.T;
  J.sum_slab = teacher ? (long)C.nsc + s : (noisy ? (long)C.nsc + C.nsn + s : (long)s);
  J.cnt_slab = noisy ? (long)C.nsc + s : (long)s;
  const int64_t* base = noisy ? C.src.rown : C.src.rowc;
  J.src0 = base ? base[J.b] : J.row0;
  J.srcT = base ? max((noisy ? C.src.lenn : C.src.lenc)[J.b], 1) : J.T;
  return J;
}

// Contiguous job range of workgroup wg: dad_ws_job_range (dad_common.h), the same function
// the host runs to size the grid (ws_split, dad_abi.hip), so no range exceeds DAD_ENC_WS_MAXJ.
__device__ __forceinline__ void job_range(const Ctx& C, int wg, int nt, int ns, float wstrong, bool& teacher,
                                          int& j0, int& j1) {
  dad_ws_job_range(wg, nt, ns, wstrong, C.Bc, C.Tc, C.ncc, C.Bn, C.Tn, C.ncn, C.Js, teacher, j0, j1);
}

// a workgroup's jobs: local job l is job a0 + l * stride (a contiguous range, or an XCD sweep)
struct JobMap {
  int a0, stride;
  __device__ __forceinline__ int operator()(int l) const { return a0 + l * stride; }
};

template <int NOISE>
__device__ __forceinline__ int tstart_of(const Ctx& C, int b) {
  if (NOISE && C.start) return (int)C.start[b];
  return dad_tstart_at(C.key_tstart, b, C.start_hi);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// a per-lane value the compiler must treat as new: addresses derived from it are computed
// where they are used instead of being hoisted out of the loop as ~30 long-lived VGPRs (the
// resident W1 leaves a wave only 64 registers for everything else)
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-workgroup-shape constants: WAVES waves, each holding NT 16-wide hidden-unit tiles of W1
// (NT * 96 registers) and converting RPW of the 16 rows of each sub-slab.
template <int WAVES>
struct Shape {
  static constexpr int kThreads = 64 * WAVES;
  static constexpr int NT = 16 / WAVES;        // 16-h tiles per wave
  static constexpr int HW = 16 * NT;           // hidden units per wave
  static constexpr int RPW = kSub / WAVES;     // rows converted per wave
  static constexpr int kDma = 3 * RPW;         // LDS-DMA instructions per wave per sub-slab
  static constexpr int kXsRow = 3;             // 16-bit x-copy stores per converted row (student)
  // 4 waves (one per SIMD, 512 registers): 256 of the 384 W1 registers in AGPRs.
  // 8 waves (two per SIMD, 256 registers): all 192 in VGPRs, no AGPRs at all.
  static constexpr bool AGPR_W = WAVES == 4;
  static constexpr bool STAGGER = WAVES == 8;  // two waves per SIMD: opposite MFMA / convert order
};

// DMA the wave's RPW rows of sub-slab (J, half) into a raw stage.  Frames past the
// utterance (padded mode: past T; store mode: past its length) are clamped to its last
// source frame (masked out by the valid bits).
template <class S>
__device__ __forceinline__ void dma_rows(const float* x, const Job& J, int half, int w, uint32_t stage_base,
                                         int lane) {
#pragma unroll
  for (int i = 0; i < S::RPW; ++i) {
    const int r = S::RPW * w + i;
    const int t = min(J.c * DAD_SLAB + half * kSub + r, J.srcT - 1);
    const float* src = x + (size_t)(J.src0 + t) * DAD_D + 4 * lane;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(stage_base + (uint32_t)(r * kRawRow));
    dad_glds16x3(src, dst);   // one M0 write per row (measured 1.7 us per launch faster than one per KB)
  }
}

// rows of sub-slab (J, half) this wave converts that exist in the utterance (the others are
// clamped duplicates: their tile rows are left stale and masked out)
template <class S>
__device__ __forceinline__ int live_rows(const Job& J, int half, int w) {
  const int t0 = J.c * DAD_SLAB + half * kSub + S::RPW * w;
  const int n = J.T - t0;
  return n < 0 ? 0 : (n > S::RPW ? S::RPW : n);
}

// Convert the wave's rows of sub-slab (J, HALF): raw stage -> 16-bit tile; CLEAN / STRONG also
// store the 16-bit row to HBM for the weight gradient (write-through, sc1: no dirty L2 lines are
// left for the kernel-end release, A/B -0.5 us per launch).  Straight-line code per KIND (one
// basic block, so the 3*RPW independent RNG chains interleave): rows past the utterance are
// converted as copies of its last row (identical bytes to the same xs address), temporally
// masked rows are selected to zero after the RNG.  Noise comes pre-scaled (dad_normal_pair_c).
// F16: v_cvt_pk_f16_f32 (round to nearest even; |x| > 65504 becomes inf, which makes the row's
// pre-activations non-finite and is reported by dad_pool's range flag), else v_cvt_pk_bf16_f32.
template <class S, int NOISE, int KIND, int HALF, bool F16>
struct WsConv {
  static constexpr bool strong = KIND == KIND_STRONG;
  static constexpr int kUnits = 3 * S::RPW;   // (row i, 256-column chunk k) units of 4 elements per lane
  const Ctx& C;
  const Job& J;
  int w, lane;
  const float* raw;
  char* tile;
  const float* fk;
  int st;
  uint32_t key;
  float sd;
  const float* nsrc;
  __device__ __forceinline__ WsConv(const Ctx& C_, const Job& J_, int w_, int lane_, const float* raw_, char* tile_,
                                    const float* fk_)
      : C(C_), J(J_), w(w_), lane(opaque(lane_)), raw(raw_), tile(tile_), fk(fk_) {
    st = (strong && C.mask_len > 0) ? tstart_of<NOISE>(C, J.b) : -(1 << 30);
    key = strong ? C.key_strong : C.key_weak;
    sd = strong ? C.sstd : C.wstd;
    nsrc = strong ? C.ns : C.nw;
  }
  // unit U: row i = U / 3 of the wave's rows, chunk k = U % 3 (columns 256k + 4 lane .. +3)
  template <int U>
  __device__ __forceinline__ void unit() const {
    constexpr int i = U / 3, k = U % 3;
    const int r = S::RPW * w + i;                               // row within the sub-slab (w uniform)
    const int t = min(J.c * DAD_SLAB + HALF * kSub + r, J.T - 1);
    const long grow = J.row0 + t;
    const bool tzero = t >= st && t < st + C.mask_len;          // I/utils.py:365-372 (padded Tmax)
    const float* rrow = raw + r * DAD_D + 4 * lane;
    char* trow = tile + r * kTileRow + 16 * ((lane >> 1) ^ (r & 15)) + 8 * (lane & 1);
    const int d = 256 * k + 4 * lane;
    f32x4 v = *reinterpret_cast<const f32x4*>(rrow + 256 * k);
    [[maybe_unused]] f32x4 kp;
    if constexpr (strong) kp = *reinterpret_cast<const f32x4*>(fk + d);
    if constexpr (KIND != KIND_CLEAN) {
      f32x4 n;
      if constexpr (NOISE) {
        n = *reinterpret_cast<const f32x4*>(nsrc + (size_t)grow * DAD_D + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) n[e] *= sd;
      } else {
        const uint32_t p = ((uint32_t)grow * (uint32_t)DAD_D + (uint32_t)d) >> 1;
        float z0, z1, z2, z3;
        dad_aug_noise_pair(key, p, sd, z0, z1);
        dad_aug_noise_pair(key, p + 1u, sd, z2, z3);
        n = f32x4{z0, z1, z2, z3};
      }
      // reference op order: x + std*N, then * feature mask, then temporal zero
      // (I/utils.py:330,338-344,365-372)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] + n[e];
      if constexpr (strong) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] * kp[e];
      }
    }
    // two packed converts per 4 elements; the temporal zero selects the packed words
    uint2 o = uint2{dad_pack2<F16>(v[0], v[1]), dad_pack2<F16>(v[2], v[3])};
    if constexpr (strong) o = tzero ? uint2{0u, 0u} : o;
    *reinterpret_cast<uint2*>(trow + 512 * k) = o;             // chunk 32k + (lane>>1), swizzled by row
    if constexpr (KIND != KIND_WEAK) {
      // 32-bit byte offset from the uniform base (saddr store, no 64-bit address math)
      const uint32_t boff = ((uint32_t)grow * (uint32_t)DAD_D + (uint32_t)d) * 2u;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(strong ? C.xsn : C.xs) + boff),
                         __builtin_bit_cast(uint64_t, o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  template <int U = 0>
  __device__ __forceinline__ void all() const {
    if constexpr (U < kUnits) {
      unit<U>();
      // one unit per scheduling region: the wave's partner on the SIMD covers the rest of the
      // dependent latency, and nothing is hoisted across regions
      __builtin_amdgcn_sched_barrier(0);
      all<U + 1>();
    }
  }
};
// no conversion riding along an MFMA pass
struct WsNoConv {
  static constexpr int kUnits = 0;
  template <int U>
  __device__ __forceinline__ void unit() const {}
};

template <class S, int NOISE, int KIND, int HALF, bool F16>
__device__ __forceinline__ void ws_convert(const Ctx& C, const Job& J, int w, int lane_, const float* raw, char* tile,
                                           const float* fk) {
  WsConv<S, NOISE, KIND, HALF, F16>(C, J, w, lane_, raw, tile, fk).all();
}

// 16-bit copies of an empty sub-slab's rows that lie inside the utterance (padded frames): zeros.
// Rows past the utterance alias its last row's copy and are left alone.
template <class S, int HALF>
__device__ __forceinline__ void ws_zero_xs(const Ctx& C, const Job& J, int w, int lane) {
  uint16_t* xs = J.kind == KIND_STRONG ? C.xsn : C.xs;
#pragma unroll
  for (int i = 0; i < S::RPW; ++i) {
    const int t = J.c * DAD_SLAB + HALF * kSub + S::RPW * w + i;
    if (t >= J.T) break;
    const uint32_t boff = ((uint32_t)(J.row0 + t) * (uint32_t)DAD_D + 4u * (uint32_t)lane) * 2u;
#pragma unroll
    for (int k = 0; k < 3; ++k) *reinterpret_cast<uint2*>(reinterpret_cast<char*>(xs) + boff + 512u * k) = uint2{0u, 0u};
  }
}

// One MFMA against a resident W1 fragment, as inline asm so the fragment is read in place as
// the B operand (the compiler otherwise parks W1 in the accumulator file and copies 4
// registers back per MFMA).  AGPR-resident fragments: "a"; VGPR-resident: "v".  The first
// k-step takes C = 0; a chain on one accumulator needs no wait states.  Operands are 8 x 16-bit
// (bf16x8 is only the register container; F16 selects the fp16 instruction).
#define DAD_WS_MFMA(OP)                                                                            \
  if constexpr (AGPR) {                                                                            \
    if constexpr (FIRST) asm(OP " %0, %1, %2, 0" : "=&v"(acc) : "v"(xa), "a"(wfr));                 \
    else asm(OP " %0, %1, %2, %0" : "+v"(acc) : "v"(xa), "a"(wfr));                                 \
  } else {                                                                                         \
    if constexpr (FIRST) asm(OP " %0, %1, %2, 0" : "=&v"(acc) : "v"(xa), "v"(wfr));                 \
    else asm(OP " %0, %1, %2, %0" : "+v"(acc) : "v"(xa), "v"(wfr));                                 \
  }
template <bool AGPR, bool FIRST, bool F16>
__device__ __forceinline__ void mfma1(f32x4& acc, const bf16x8& xa, const bf16x8& wfr) {
  if constexpr (F16) {
    DAD_WS_MFMA("v_mfma_f32_16x16x32_f16")
  } else {
    DAD_WS_MFMA("v_mfma_f32_16x16x32_bf16")
  }
}
#undef DAD_WS_MFMA

// A fragment of k-step KS: rows lane&15, k = 32KS + 8(lane>>4) .. +7.  The XOR swizzle only
// touches the low 4 bits of the chunk index, so chunk (4KS + g) ^ row = 16(KS>>2) +
// ((4(KS&3) + g) ^ row): four per-lane offsets aoff[KS&3] plus an immediate 256(KS>>2).
template <int KS>
__device__ __forceinline__ bf16x8 afrag(const char* tile, const int (&aoff)[4]) {
  return *reinterpret_cast<const bf16x8*>(tile + aoff[KS & 3] + 256 * (KS >> 2));
}

// acc[t] = x_tile(16 rows) . W1[hw + 16t .. +15]^T over K = 768.  The A fragment of k-step
// KS+1 is read while the MFMAs of k-step KS issue.  CV: conversion units of the next sub-slab
// riding along the MFMA chain: unit u is issued after k-step (u + 1) * kKS / kUnits - 1, between
// scheduling barriers, so the VALU work of the RNG fills the matrix pipe's cycles inside ONE
// wave (measured 0.6-0.8 us per launch faster than the MFMA-then-convert order alone).
template <class S, int KS, bool F16, class CV>
__device__ __forceinline__ void ws_mfma_from(const char* tile, const int (&aoff)[4], const bf16x8 (&wf)[S::NT][kKS],
                                             f32x4 (&acc)[S::NT], bf16x8 x0, const CV& cv) {
  if constexpr (KS < kKS) {
    bf16x8 xn;
    if constexpr (KS + 1 < kKS) xn = afrag<KS + 1>(tile, aoff);
#pragma unroll
    for (int t = 0; t < S::NT; ++t) {
      const bool agpr = S::AGPR_W && (t < 2 || (t == 2 && KS < 16));
      if (agpr) mfma1<true, KS == 0, F16>(acc[t], x0, wf[t][KS]);
      else mfma1<false, KS == 0, F16>(acc[t], x0, wf[t][KS]);
    }
    if constexpr (CV::kUnits > 0) {
      constexpr int U = (KS + 1) * CV::kUnits / kKS;        // units due after this k-step
      constexpr int U0 = KS * CV::kUnits / kKS;
      if constexpr (U > U0) {
        __builtin_amdgcn_sched_barrier(0);
        cv.template unit<U - 1>();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    ws_mfma_from<S, KS + 1, F16>(tile, aoff, wf, acc, xn, cv);
  }
}
template <class S, bool F16, class CV = WsNoConv>
__device__ __forceinline__ void ws_mfma(const char* tile, const int (&aoff)[4], const bf16x8 (&wf)[S::NT][kKS],
                                        f32x4 (&acc)[S::NT], const CV& cv = CV{}) {
  ws_mfma_from<S, 0, F16>(tile, aoff, wf, acc, afrag<0>(tile, aoff), cv);
  // MFMA D -> VALU readers of the epilogue (hipcc pads nothing after an asm MFMA)
  if constexpr (S::NT == 4) asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0]), "v"(acc[1]), "v"(acc[2]), "v"(acc[3]));
  else asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0]), "v"(acc[1]));
}

// sum over the 4 row groups (lane >> 4) of a 16x16 C tile column: v_permlane32_swap and
// v_permlane16_swap (gfx950) with both operands = x give [x_lo, x_lo] + [x_hi, x_hi]
__device__ __forceinline__ float rowgroup_sum(float x) {
  const uint32_t xi = __float_as_uint(x);
  const auto a = __builtin_amdgcn_permlane32_swap(xi, xi, false, false);
  const float s1 = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const uint32_t si = __float_as_uint(s1);
  const auto b = __builtin_amdgcn_permlane16_swap(si, si, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// OR over the 4 row groups, same swaps as rowgroup_sum
__device__ __forceinline__ uint32_t rowgroup_or(uint32_t x) {
  const auto a = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  const uint32_t s1 = a[0] | a[1];
  const auto b = __builtin_amdgcn_permlane16_swap(s1, s1, false, false);
  return b[0] | b[1];
}

// bias + ReLU + valid mask of one sub-slab.  Per-lane partial sums/counts (4 rows of the C
// tile) accumulate over the job's two sub-slabs and are reduced across the 4 row groups only
// at the job's end (HALF 1).  Student: the ReLU'-and-valid row mask of each hidden unit (bit
// r = row r of the 32-row slab): a lane's 4 rows form a nibble, the 4 row groups are OR-ed
// by lane swaps, the two halves meet in bw and one 32-lane store writes the job's words.
// Stores: student 3 at HALF 1 (row masks, sums, counts); teacher 1 at HALF 1 (sums).
template <class S, bool TEACHER, int HALF>
__device__ __forceinline__ void ws_epilogue(const Ctx& C, const Job& J, int w, int lane, uint32_t vmask,
                                            const float (&bh)[S::NT], const f32x4 (&acc)[S::NT], float (&ssum)[S::NT],
                                            float (&scnt)[S::NT], uint32_t (&bw)[S::NT]) {
  const int g = lane >> 4;
#pragma unroll
  for (int t = 0; t < S::NT; ++t) {
    float s = 0.0f, n = 0.0f;
    uint32_t nib = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool v = (vmask >> (4 * g + r)) & 1u;     // C/D layout: row = 4(lane>>4) + r, col = lane&15
      const float pre = acc[t][r] + bh[t];
      const bool act = v && pre > 0.0f;
      s += act ? pre : 0.0f;
      if constexpr (!TEACHER) {
        n += act ? 1.0f : 0.0f;
        nib |= act ? (1u << r) : 0u;
      }
    }
    ssum[t] = HALF ? ssum[t] + s : s;
    if constexpr (!TEACHER) {
      scnt[t] = HALF ? scnt[t] + n : n;
      const uint32_t m16 = rowgroup_or(nib << (4 * g));   // rows 0..15 of the sub-slab, h = hw + 16t + col
      bw[t] = HALF ? bw[t] | (m16 << 16) : m16;
    }
  }
  const int hw = S::HW * w;
  if constexpr (HALF == 1) {
    const int t = lane >> 4;                           // h = hw + lane (lanes < HW)
    float sv = 0.0f, cv = 0.0f;
    uint32_t mv = 0;
#pragma unroll
    for (int k = 0; k < S::NT; ++k) {
      const float a = rowgroup_sum(ssum[k]);
      sv = t == k ? a : sv;
      if constexpr (!TEACHER) {
        const float c = rowgroup_sum(scnt[k]);
        cv = t == k ? c : cv;
        mv = t == k ? bw[k] : mv;
      }
    }
    if (lane < S::HW) {
      C.part_sum[(size_t)J.sum_slab * DAD_H + hw + lane] = sv;
      if constexpr (!TEACHER) {
        C.part_cnt[(size_t)J.cnt_slab * DAD_H + hw + lane] = cv;
        C.bits[(size_t)J.cnt_slab * DAD_H + hw + lane] = mv;
      }
    }
  }
}


// VMEM instructions one wave issues per sub-slab (the counted vmcnt waits depend on them)
template <class S>
__device__ __forceinline__ constexpr int n_xs(int kind) {
  return kind != KIND_WEAK ? S::kXsRow * S::RPW : 0;
}
template <bool TEACHER, int HALF>
__device__ __forceinline__ constexpr int n_epi() { return TEACHER ? HALF : 3 * HALF; }

template <int N>
__device__ __forceinline__ void wait_vm_sw(int n) {
  // n in {0, 1, 3} + {0, 12 (xs)} + {0, kDma}: the handful of counts the pipeline produces
  switch (n) {
    case 0: wait_vm<0>(); break;     case 1: wait_vm<1>(); break;     case 3: wait_vm<3>(); break;
    case N: wait_vm<N>(); break;     case N + 1: wait_vm<N + 1>(); break; case N + 3: wait_vm<N + 3>(); break;
    case 2 * N: wait_vm<2 * N>(); break; case 2 * N + 1: wait_vm<2 * N + 1>(); break;
    case 2 * N + 3: wait_vm<2 * N + 3>(); break;
    default: wait_vm<0>(); break;
  }
}

}  // namespace

template <int WAVES, int NOISE, bool TEACHER, bool F16>
__device__ __forceinline__ void ws_loop(const Ctx& C, const JobMap jm, const int Q, const int w, const int lane,
                                        char* smem, const uint32_t sbase, const bf16x8* W, const float* bias,
                                        const float* fk, const uint32_t* vb) {
  using S = Shape<WAVES>;
  bf16x8 wf[S::NT][kKS];
  float bh[S::NT];
  float ssum[S::NT], scnt[S::NT];
  uint32_t bw[S::NT];
  const float* raw0 = reinterpret_cast<const float*>(smem + kOffRaw);
  const float* raw1 = reinterpret_cast<const float*>(smem + kOffRaw + kRawStage);
  char* tile0 = smem + kOffTile;
  char* tile1 = smem + kOffTile + kTile;
  auto jobq = [&](int q) { return job_of(C, TEACHER, jm(q >> 1)); };
  // valid-row mask of sub-slab q (uniform): an empty one (frames past every utterance's end,
  // e.g. rows 304..319 of a 300-frame utterance) is neither converted nor multiplied -- the
  // epilogue's valid mask zeroes it anyway
  auto vmask_of = [&](int q) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((vb[q >> 1] >> (16 * (q & 1))) & 0xffffu);
  };
  // xs stores convert(q) issued (the counted vmcnt waits depend on them; for an empty sub-slab
  // 0 even where it zeroes padded rows' copies: under-counting younger stores only waits longer)
  auto xs_of = [&](int q) -> int { return vmask_of(q) ? n_xs<S>(jobq(q).kind) : 0; };
  auto dma = [&](int q) {
    if (q < Q) {
      const Job J = jobq(q);
      dma_rows<S>(J.kind == KIND_CLEAN ? C.xc : C.xn, J, q & 1, w, sbase + kOffRaw + (q & 1) * kRawStage, lane);
    }
  };
  // convert sub-slab q (its half HN is a template parameter: raw stage and tile HN)
  auto convert = [&](auto hn_tag, const Job& J, uint32_t vm) {
    constexpr int HN = decltype(hn_tag)::value;
    if (vm == 0) {
      // nothing to multiply; the student's 16-bit copies of padded frames inside the utterance
      // still get finite bytes (the weight gradient multiplies them by a zero mask)
      if constexpr (!TEACHER) ws_zero_xs<S, HN>(C, J, w, lane);
      return;
    }
    const float* rawp = HN ? raw1 : raw0;
    char* tl = HN ? tile1 : tile0;
    if constexpr (TEACHER) ws_convert<S, NOISE, KIND_WEAK, HN, F16>(C, J, w, lane, rawp, tl, fk);
    else if (J.kind == KIND_CLEAN) ws_convert<S, NOISE, KIND_CLEAN, HN, F16>(C, J, w, lane, rawp, tl, fk);
    else ws_convert<S, NOISE, KIND_STRONG, HN, F16>(C, J, w, lane, rawp, tl, fk);
  };
  // sub-slab q (half H): MFMA on tile H, convert sub-slab q+1 (half 1-H), epilogue, DMA q+3
  auto iter = [&](auto h_tag, int q) {
    constexpr int H = decltype(h_tag)::value;
    f32x4 acc[S::NT];
    int aoff[4];
    {
      const int ln = opaque(lane);
#pragma unroll
      for (int m = 0; m < 4; ++m) aoff[m] = (ln & 15) * kTileRow + 16 * ((4 * m + (ln >> 4)) ^ (ln & 15));
    }
    unsigned long long c0 = WS_CLK(), c1 = c0, c2 = c0;
    const uint32_t vmask = vmask_of(q);
    auto mfma = [&]() {
      if (vmask) {
        ws_mfma<S, F16>(H ? tile1 : tile0, aoff, wf, acc);
      } else {
#pragma unroll
        for (int t = 0; t < S::NT; ++t) acc[t] = f32x4{};
      }
    };
    if (q + 1 < Q) {
      const Job Jn = jobq(q + 1);
      const uint32_t vmn = vmask_of(q + 1);
      // this wave's DMA of sub-slab q+1 (issued at the end of iteration q-2) has landed once at
      // most these younger VMEM ops remain: xs stores of convert(q), epilogue(q-1), DMA(q+2)
      wait_vm_sw<S::kDma>(xs_of(q) + (q > 0 ? n_epi<TEACHER, 1 - H>() : 0) + (q + 2 < Q ? S::kDma : 0));
      c1 = WS_CLK();
      if (vmask && vmn) {
        // MFMA(q) with convert(q+1)'s units riding along the chain
        constexpr int HN = 1 - H;
        const float* rawp = HN ? raw1 : raw0;
        char* tl = HN ? tile1 : tile0;
        const char* tm = H ? tile1 : tile0;
        if constexpr (TEACHER) {
          ws_mfma<S, F16>(tm, aoff, wf, acc, WsConv<S, NOISE, KIND_WEAK, HN, F16>(C, Jn, w, lane, rawp, tl, fk));
        } else if (Jn.kind == KIND_CLEAN) {
          ws_mfma<S, F16>(tm, aoff, wf, acc, WsConv<S, NOISE, KIND_CLEAN, HN, F16>(C, Jn, w, lane, rawp, tl, fk));
        } else {
          ws_mfma<S, F16>(tm, aoff, wf, acc, WsConv<S, NOISE, KIND_STRONG, HN, F16>(C, Jn, w, lane, rawp, tl, fk));
        }
        c2 = WS_CLK();
      } else if (S::STAGGER && w >= WAVES / 2) {
        // The two waves sharing a SIMD (w and w + WAVES/2) run the two halves in opposite
        // order, so one's MFMA chain overlaps the other's RNG/convert VALU work between barriers.
        convert(std::integral_constant<int, 1 - H>{}, Jn, vmn);
        c2 = WS_CLK();
        mfma();
      } else {
        mfma();
        DAD_PROBE_FENCE2(acc[0], acc[S::NT - 1]);
        c2 = WS_CLK();
        convert(std::integral_constant<int, 1 - H>{}, Jn, vmn);
      }
    } else {
      mfma();
    }
    const unsigned long long c3 = WS_CLK();
    ws_epilogue<S, TEACHER, H>(C, jobq(q), w, lane, vmask, bh, acc, ssum, scnt, bw);
    const unsigned long long c4 = WS_CLK();
    dma(q + 3);
    const unsigned long long c5 = WS_CLK();
    lds_barrier();
    WS_PHASES(c0, c1, c2, c3, c4, c5);
  };
  // the first two sub-slabs' DMAs go out ahead of the resident W1 (48 KB per wave), so
  // sub-slab 0 is converted while W1 streams in
  dma(0);
  dma(1);
  const int hw = S::HW * w;
#pragma unroll
  for (int t = 0; t < S::NT; ++t)   // fragment-major shadow (dad_w1frag_index): 1 KB coalesced loads
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) wf[t][ks] = W[(size_t)(((hw >> 4) + t) * kKS + ks) * 64 + lane];
#pragma unroll
  for (int t = 0; t < S::NT; ++t) bh[t] = bias[hw + 16 * t + (lane & 15)];
  constexpr int kW1 = S::NT * kKS + S::NT;   // VMEM loads of the resident W1 and the bias
  static_assert(S::kDma + kW1 <= 63, "vmcnt range");
  if (Q > 1) wait_vm<S::kDma + kW1>();        // sub-slab 0 landed (DMA 1 and W1 still in flight)
  else wait_vm<kW1>();
  convert(std::integral_constant<int, 0>{}, jobq(0), vmask_of(0));
  dma(2);
  lds_barrier();
  for (int q = 0; q < Q; q += 2) {   // Q is even: a job is two sub-slabs
    iter(std::integral_constant<int, 0>{}, q);
    iter(std::integral_constant<int, 1>{}, q + 1);
  }
  wait_vm<0>();
}

// NOISE: 0 = counter RNG, 1 = explicit noise tensors (parity mode)
template <int WAVES, int NOISE, bool F16>
__device__ __forceinline__ void encode_ws_body(const DadEncodeArgs& a, char* smem) {
  using S = Shape<WAVES>;
  WS_STAMP(0, DAD_PROBE_WALL());
  for (int k = 4; DAD_PROBE_ON && k < 10; ++k) WS_STAMP(k, 0);
  const Ctx C = ctx_of(a);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  bool teacher;
  JobMap jm;
  int nj;
  if (a.ws_sweep.nt > 0) {
    dad_ws_sweep_jobs(blockIdx.x, a.ws_sweep, C.Bc, C.Tc, C.ncc, C.Jc, C.Js, teacher, jm.a0, jm.stride, nj);
  } else {
    int j0, j1;
    job_range(C, blockIdx.x, a.ws_nt, a.ws_ns, a.ws_wstrong, teacher, j0, j1);
    jm = JobMap{j0, 1};
    nj = j1 - j0;
  }
  if (nj <= 0) return;
  const uint32_t sbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;   // LDS byte address

  // ---- prologue: feature keep flags, valid bits of every job, resident W1, bias
  float* fk = reinterpret_cast<float*>(smem + kOffFK);
  uint32_t* vb = reinterpret_cast<uint32_t*>(smem + kOffVB);
  if (!teacher)
    for (int d = tid; d < DAD_D; d += S::kThreads) {
      fk[d] = dad_feat_keep(C.u, C.key_feat, d, C.feat_p);     // I/utils.py:343 (rand(D) > p)
    }
  for (int p = tid; p < nj * DAD_SLAB; p += S::kThreads) {
    const Job J = job_of(C, teacher, jm(p / DAD_SLAB));
    const int t = J.c * DAD_SLAB + (p & (DAD_SLAB - 1));
    const uint8_t* pad = J.kind == KIND_CLEAN ? C.mc : C.mn;
    const bool v = t < J.T && pad[J.row0 + t] == 0;
    const uint64_t bal = __ballot(v);
    if ((lane & 31) == 0) vb[p / DAD_SLAB] = (uint32_t)(bal >> (lane & 32));
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): the pad / u loads retired (no DMA in flight yet)
  lds_barrier();                        // fk / vb visible
  WS_STAMP(1, DAD_PROBE_WALL());
  const bf16x8* W = reinterpret_cast<const bf16x8*>(teacher ? a.w1h_teacher : a.w1h_student);
  const float* bias = teacher ? a.b1_teacher : a.b1_student;
  if (teacher) ws_loop<WAVES, NOISE, true, F16>(C, jm, 2 * nj, w, lane, smem, sbase, W, bias, fk, vb);
  else ws_loop<WAVES, NOISE, false, F16>(C, jm, 2 * nj, w, lane, smem, sbase, W, bias, fk, vb);
  WS_STAMP(2, DAD_PROBE_WALL());
  WS_STAMP(3, ((unsigned long long)teacher << 16) | (unsigned long long)(2 * nj));
}


// Counter-RNG (throughput) and explicit-noise (parity) kernels are separate so the noise
// loads do not share the register allocation of the throughput kernel; fp16 and bf16 operand
// kernels likewise.
#define DAD_WS_KERNEL(name, NOISE, F16)                                              \
  __global__ __launch_bounds__(DAD_ENC_WS_THREADS, 1) void name(DadEncodeArgs a) {   \
    DAD_GUARD_BLOCK(DAD_ENC_WS_THREADS);                                             \
    __shared__ __attribute__((aligned(16))) char smem[kLds];                         \
    encode_ws_body<DAD_ENC_WS_THREADS / 64, NOISE, F16>(a, smem);                    \
  }
DAD_WS_KERNEL(dad_encode_ws, 0, false)
DAD_WS_KERNEL(dad_encode_ws_explicit, 1, false)
DAD_WS_KERNEL(dad_encode_ws_f16, 0, true)
DAD_WS_KERNEL(dad_encode_ws_f16_explicit, 1, true)
#undef DAD_WS_KERNEL

// ------------------------------------------------------------ prepared-row encoder (wp)
// dad_encode_wp: the same W-stationary GEMM + epilogue on a PREPARED set (dad_prep.h: the
// augmentation and the 16-bit conversion already done, weight-independent, off this launch).
// What is left per 16-row sub-slab is data movement and matrix work only:
//   HBM 16-bit rows --LDS-DMA (3 x 1 KB per wave, straight into the XOR-swizzled tile: lane l of
//   a piece loads the source chunk that lands at its slot)--> one of kPS = 6 tile stages
//   --ds_read_b128 A fragments--> 48 MFMAs per wave against the resident W1 --> epilogue.
// Five sub-slabs are in flight ahead of the one being multiplied (120 KB per CU), one barrier per
// sub-slab, no VALU conversion, no raw stage, no 16-bit copy stores (the set is the copy).
namespace {

constexpr int kPS = 6;                                   // 24-KB tile stages
constexpr int kOffPVB = kPS * kTile;                     // valid bits u32[DAD_ENC_WS_MAXJ]
constexpr int kLdsP = kOffPVB + 4 * DAD_ENC_WS_MAXJ;
static_assert(kLdsP <= 160 * 1024, "LDS budget");

// one 1-KB LDS-DMA piece: 16 B per lane from `src` to lds_dst + 16 * lane (see dad_glds16x3)
__device__ __forceinline__ void dad_glds16(const void* src, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep) : "v"(src), "s"(lds_dst) : "memory");
}

// vmcnt(D + n) for the counts the prepared-row pipeline produces: D = NP (kPS - 2) DMA
// instructions plus n = 0..3 odd iterations' epilogue stores (1 teacher, 3 student)
template <int D>
__device__ __forceinline__ void wp_wait(int n) {
  switch (n) {
    case 1: wait_vm<D + 1>(); break;  case 2: wait_vm<D + 2>(); break;  case 3: wait_vm<D + 3>(); break;
    case 6: wait_vm<D + 6>(); break;  case 9: wait_vm<D + 9>(); break;
    default: wait_vm<D>(); break;
  }
}

}  // namespace

template <int WAVES, bool TEACHER, bool F16>
__device__ __forceinline__ void wp_loop(const Ctx& C, const JobMap jm, const int Q, const int w, const int lane,
                                        char* smem, const uint32_t sbase, const bf16x8* W, const float* bias,
                                        const uint32_t* vb, const DadEncodeArgs& a) {
  using S = Shape<WAVES>;
  constexpr int NP = 24 / WAVES;   // 1-KB DMA pieces per wave per sub-slab
  bf16x8 wf[S::NT][kKS];
  float bh[S::NT];
  float ssum[S::NT], scnt[S::NT];
  uint32_t bw[S::NT];
  // resident W1 and bias before any DMA: every later sub-slab wait covers them too
  const int hw = S::HW * w;
#pragma unroll
  for (int t = 0; t < S::NT; ++t)   // fragment-major shadow (dad_w1frag_index): 1 KB coalesced loads
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) wf[t][ks] = W[(size_t)(((hw >> 4) + t) * kKS + ks) * 64 + lane];
#pragma unroll
  for (int t = 0; t < S::NT; ++t) bh[t] = bias[hw + 16 * t + (lane & 15)];
  // the wave's pieces p = NP w + i of a sub-slab tile: lane slot 1024p + 16 lane = row prow[i],
  // swizzled position P; it loads source chunk P ^ (row & 15) (byte offset pcol[i] in the row)
  int prow[NP], pcol[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int o = 1024 * (NP * w + i) + 16 * lane;
    prow[i] = o / kTileRow;
    pcol[i] = 16 * (((o - kTileRow * prow[i]) >> 4) ^ (prow[i] & 15));
  }
  // DMA of sub-slab q into stage s (sub-slabs past the range re-read the last one's rows, so
  // every iteration issues the same VMEM count; their stages are never read)
  auto dma = [&](int q, int s) {
    const int qq = min(q, Q - 1);
    const Job J = job_of(C, TEACHER, jm(qq >> 1));
    const char* base = reinterpret_cast<const char*>(J.kind == KIND_CLEAN ? a.x16c : (J.kind == KIND_STRONG ? a.x16s : a.x16w));
    const uint32_t dst = sbase + (uint32_t)(s * kTile) + 1024u * NP * (uint32_t)w;
    const int t0 = J.c * DAD_SLAB + (qq & 1) * kSub;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int t = min(t0 + prow[i], J.T - 1);
      dad_glds16(base + (size_t)(J.row0 + t) * (DAD_D * 2) + pcol[i], dst + 1024u * (uint32_t)i);
    }
  };
  auto vmask_of = [&](int q) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((vb[q >> 1] >> (16 * (q & 1))) & 0xffffu);
  };
  constexpr int E = TEACHER ? 1 : 3;   // epilogue stores of an odd (HALF 1) iteration
  int s_cur = 0;                       // stage of sub-slab q
  auto iter = [&](auto h_tag, int q) {
    constexpr int H = decltype(h_tag)::value;
    // DMA(q) has landed once at most these younger VMEM ops remain: DMA(q+1 .. q+kPS-2) and the
    // epilogue stores of iterations max(0, q-kPS+1) .. q-1 (stores only in odd iterations)
    const int lo = max(0, q - (kPS - 1));
    wp_wait<NP * (kPS - 2)>(E * ((q >> 1) - (lo >> 1)));
    lds_barrier();   // every wave's pieces of q visible; stage of q-1 free (its reads retired)
    dma(q + kPS - 1, s_cur == 0 ? kPS - 1 : s_cur - 1);
    f32x4 acc[S::NT];
    const uint32_t vmask = vmask_of(q);
    if (vmask) {
      int aoff[4];
      const int ln = opaque(lane);
#pragma unroll
      for (int m = 0; m < 4; ++m) aoff[m] = (ln & 15) * kTileRow + 16 * ((4 * m + (ln >> 4)) ^ (ln & 15));
      ws_mfma<S, F16>(smem + s_cur * kTile, aoff, wf, acc);
    } else {
#pragma unroll
      for (int t = 0; t < S::NT; ++t) acc[t] = f32x4{};
    }
    ws_epilogue<S, TEACHER, H>(C, job_of(C, TEACHER, jm(q >> 1)), w, lane, vmask, bh, acc, ssum, scnt, bw);
    s_cur = s_cur == kPS - 1 ? 0 : s_cur + 1;
  };
#pragma unroll
  for (int q = 0; q < kPS - 1; ++q) dma(q, q);
  for (int q = 0; q < Q; q += 2) {   // Q is even: a job is two sub-slabs
    iter(std::integral_constant<int, 0>{}, q);
    iter(std::integral_constant<int, 1>{}, q + 1);
  }
  wait_vm<0>();   // no DMA may still target this workgroup's LDS when it exits
}

template <int WAVES, bool F16>
__device__ __forceinline__ void encode_wp_body(const DadEncodeArgs& a, char* smem) {
  const Ctx C = ctx_of(a);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  bool teacher;
  int j0, j1;
  job_range(C, blockIdx.x, a.ws_nt, a.ws_ns, a.ws_wstrong, teacher, j0, j1);
  const JobMap jm{j0, 1};
  const int nj = j1 - j0;
  if (nj <= 0) return;
  const uint32_t sbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // valid bits of every job (bit r = row r of the 32-row slab is a frame of the utterance)
  uint32_t* vb = reinterpret_cast<uint32_t*>(smem + kOffPVB);
  for (int p = tid; p < nj * DAD_SLAB; p += 64 * WAVES) {
    const Job J = job_of(C, teacher, jm(p / DAD_SLAB));
    const int t = J.c * DAD_SLAB + (p & (DAD_SLAB - 1));
    const uint8_t* pad = J.kind == KIND_CLEAN ? C.mc : C.mn;
    const bool v = t < J.T && pad[J.row0 + t] == 0;
    const uint64_t bal = __ballot(v);
    if ((lane & 31) == 0) vb[p / DAD_SLAB] = (uint32_t)(bal >> (lane & 32));
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): the pad loads retired (no DMA in flight yet)
  lds_barrier();                        // vb visible
  const bf16x8* W = reinterpret_cast<const bf16x8*>(teacher ? a.w1h_teacher : a.w1h_student);
  const float* bias = teacher ? a.b1_teacher : a.b1_student;
  if (teacher) wp_loop<WAVES, true, F16>(C, jm, 2 * nj, w, lane, smem, sbase, W, bias, vb, a);
  else wp_loop<WAVES, false, F16>(C, jm, 2 * nj, w, lane, smem, sbase, W, bias, vb, a);
}

#define DAD_WP_KERNEL(name, WAVES, F16)                                        \
  __global__ __launch_bounds__(64 * WAVES, 1) void name(DadEncodeArgs a) {     \
    DAD_GUARD_BLOCK(64 * WAVES);                                               \
    __shared__ __attribute__((aligned(16))) char smem[kLdsP];                  \
    encode_wp_body<WAVES, F16>(a, smem);                                       \
  }
DAD_WP_KERNEL(dad_encode_wp, 8, false)
DAD_WP_KERNEL(dad_encode_wp_f16, 8, true)
DAD_WP_KERNEL(dad_encode_wp4, 4, false)
DAD_WP_KERNEL(dad_encode_wp4_f16, 4, true)
#undef DAD_WP_KERNEL
