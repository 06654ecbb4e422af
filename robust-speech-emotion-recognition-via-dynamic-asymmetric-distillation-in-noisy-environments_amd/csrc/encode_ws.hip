// W-stationary 16-bit encoder GEMM: the throughput-mode forward of all three encoder passes on
// PREPARED rows (dad_prep.h: augmentation + 16-bit conversion, weight-independent, done by the
// previous step's tail launch or a standalone launch), fp16 (default) or bf16 MFMA operands,
// fp32 accumulation.
//
// Replaces, per step (I/train.py:399,406-410,439):
//   student_encoder(clean)                         Emotion2VecEncoder.forward, I/model.py:18-41
//   teacher_encoder(weak_augment(noisy))           (the weak rows prepared by dad_prep)
//   student_encoder(strong_augment(noisy))         (the strong rows prepared by dad_prep)
// and emits what the rest of the step consumes: per-32-row-slab pooled ReLU sums and active
// counts and the ReLU'-and-valid row masks.
//
// Shape of the work: out[rows][256] = x[rows][768] . W1^T with tens of thousands of rows and
// W1 only 384 KB in 16 bits.  So W1 is STATIONARY: a persistent workgroup holds all 256 hidden
// units of ONE network's W1 in its register file (each of 8 waves 32 hidden units x 768 k, 192
// VGPRs, read in place as MFMA B operands) and streams 16-row sub-slabs through LDS:
//
//   HBM 16-bit rows --LDS-DMA (3 x 1 KB per wave, straight into the XOR-swizzled tile: lane l of
//   a piece loads the source chunk that lands at its slot)--> one of 3 job stages (two 16-row
//   tiles each) --ds_read_b128 A fragments (conflict-free)--> 96 v_mfma_f32_16x16x32_{f16,bf16}
//   per wave per 32-row job
//   --bias, ReLU, valid mask, row sums, ballots--> slab partials + ReLU' bits
//
// Roles are per workgroup: TEACHER workgroups (teacher W1) run the weak slabs, STUDENT workgroups
// (student W1) the clean slabs and then the strong slabs, contiguous ranges balanced by live
// sub-slabs (dad_wp_job_range; host: wp_split in dad_abi.hip).  Two jobs are in flight ahead of
// the one being multiplied (96 KB per CU), one barrier per job.
#include <type_traits>

#include "dad_common.h"
#include "dad_kernels.h"
#include "dad_probe.h"

// per-workgroup stamps of the stamps build (dad_probe.h): [start, after the valid-bit prologue,
// end (100 MHz wall clock), role<<16 | sub-slabs, then wave-0 cycles summed over the loop in: DMA
// wait, barrier, DMA issue + valid mask, first phase, second phase]
DAD_PROBE_BUFFER(ws_stamps, 4096 * 10)
#define WS_CLK() DAD_PROBE_CLK()
#define WS_STAMP(k, v) \
  if (threadIdx.x == 0 && blockIdx.x < 4096) DAD_PROBE_SET(ws_stamps, blockIdx.x * 10 + (k), (v))

namespace {

constexpr int kSub = 16;                       // rows per sub-slab (one MFMA M tile)
constexpr int kKS = DAD_D / 32;                // 24 k-steps of v_mfma_f32_16x16x32_{f16,bf16}
constexpr int kTileRow = DAD_D * 2;            // 1536 B
constexpr int kTile = kSub * kTileRow;         // 24 KB

enum { KIND_CLEAN = 0, KIND_WEAK = 1, KIND_STRONG = 2 };

// Every scalar the kernel needs, copied out of the kernel arguments once.
struct Ctx {
  int Bc, Tc, ncc, Bn, Tn, ncn;
  uint32_t mcc, mcn;     // division magics for ncc / ncn (fast_div)
  int nsc, nsn, Jc, Js;
  const uint8_t* mc; const uint8_t* mn;
  float* part_sum; float* part_cnt; uint32_t* bits;
};

__device__ __forceinline__ Ctx ctx_of(const DadEncodeArgs& a) {
  Ctx c;
  c.Bc = a.g.Bc; c.Tc = a.g.Tc; c.ncc = a.g.ncc;
  c.Bn = a.g.Bn; c.Tn = a.g.Tn; c.ncn = a.g.ncn;
  c.nsc = c.Bc * c.ncc; c.nsn = c.Bn * c.ncn;
  c.mcc = c.ncc > 1 ? 0xffffffffu / (uint32_t)c.ncc + 1u : 0u;
  c.mcn = c.ncn > 1 ? 0xffffffffu / (uint32_t)c.ncn + 1u : 0u;
  c.Jc = c.nsc; c.Js = a.warmup ? 0 : c.nsn;
  c.mc = a.mc; c.mn = a.mn;
  c.part_sum = a.part_sum; c.part_cnt = a.part_cnt; c.bits = a.bits;
  return c;
}

// n / d for the slab counts per utterance: m = floor(2^32 / d) + 1 (0 for d = 1) is exact for
// n * d < 2^32; one scalar multiply-high instead of a ~40-instruction scalar division
__device__ __forceinline__ int fast_div(int n, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)n, m) : n;
}

struct Job {
  int kind, b, c, T;
  long row0;        // [b][T] row of frame 0 (the prepared set's padded layout)
  long sum_slab;    // part_sum slab
  long cnt_slab;    // part_cnt slab = ReLU' row-mask slab (student only)
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
  return J;
}

// a workgroup's jobs: local job l is job a0 + l
struct JobMap {
  int a0, stride;
  __device__ __forceinline__ int operator()(int l) const { return a0 + l * stride; }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// a per-lane value the compiler must treat as new: addresses derived from it are computed
// where they are used instead of being hoisted out of the loop as long-lived VGPRs (the
// resident W1 leaves a wave only 64 registers for everything else)
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-workgroup-shape constants: WAVES waves, each holding NT 16-wide hidden-unit tiles of W1
// (NT * 96 registers).
template <int WAVES>
struct Shape {
  static constexpr int NT = 16 / WAVES;        // 16-h tiles per wave
  static constexpr int HW = 16 * NT;           // hidden units per wave
};

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
// KS+1 is read while the MFMAs of k-step KS issue.
template <class S, int KS, bool F16>
__device__ __forceinline__ void ws_mfma_from(const char* tile, const int (&aoff)[4], const bf16x8 (&wf)[S::NT][kKS],
                                             f32x4 (&acc)[S::NT], bf16x8 x0) {
  if constexpr (KS < kKS) {
    bf16x8 xn;
    if constexpr (KS + 1 < kKS) xn = afrag<KS + 1>(tile, aoff);
#pragma unroll
    for (int t = 0; t < S::NT; ++t) mfma1<false, KS == 0, F16>(acc[t], x0, wf[t][KS]);
    ws_mfma_from<S, KS + 1, F16>(tile, aoff, wf, acc, xn);
  }
}
template <class S, bool F16>
__device__ __forceinline__ void ws_mfma(const char* tile, const int (&aoff)[4], const bf16x8 (&wf)[S::NT][kKS],
                                        f32x4 (&acc)[S::NT]) {
  ws_mfma_from<S, 0, F16>(tile, aoff, wf, acc, afrag<0>(tile, aoff));
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


}  // namespace

namespace {

constexpr int kJS = 3;                                   // 48-KB job stages (two 16-row tiles each)
constexpr int kOffPVB = kJS * 2 * kTile;                 // valid bits u32[DAD_ENC_WS_MAXJ]
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

}  // namespace

// One 32-row job per iteration: its two 16-row sub-slab tiles are one 48-KB stage of three (two
// jobs in flight ahead of the one multiplied), one barrier, one wait and one valid-mask read per
// job, and every k-step issues 4 independent MFMAs (2 row tiles x 2 hidden-unit tiles) per A pair.
// (The 16-row iteration, one barrier and one epilogue per sub-slab, measured 42.5 against 37.6-38.6
// us per launch by events, step 118.4-119.2 against 114.6-115.0 us.)
template <bool F16>
__device__ __forceinline__ void wp_mfma2(const char* tile, const int (&aoff)[4], const bf16x8 (&wf)[2][kKS],
                                         f32x4 (&acc)[2][2], uint32_t vm) {
  const bool h0 = (vm & 0xffffu) != 0, h1 = (vm >> 16) != 0;
  bf16x8 x0 = afrag<0>(tile, aoff), x1 = afrag<0>(tile + kTile, aoff);
#pragma unroll
  for (int ks = 0; ks < kKS; ++ks) {
    bf16x8 n0, n1;
    if (ks + 1 < kKS) {
      n0 = *reinterpret_cast<const bf16x8*>(tile + aoff[(ks + 1) & 3] + 256 * ((ks + 1) >> 2));
      n1 = *reinterpret_cast<const bf16x8*>(tile + kTile + aoff[(ks + 1) & 3] + 256 * ((ks + 1) >> 2));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (ks == 0) {
        mfma1<false, true, F16>(acc[0][t], x0, wf[t][0]);
        mfma1<false, true, F16>(acc[1][t], x1, wf[t][0]);
      } else {
        mfma1<false, false, F16>(acc[0][t], x0, wf[t][ks]);
        mfma1<false, false, F16>(acc[1][t], x1, wf[t][ks]);
      }
    }
    x0 = n0;
    x1 = n1;
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0][0]), "v"(acc[0][1]), "v"(acc[1][0]), "v"(acc[1][1]));
  if (!h0) { acc[0][0] = f32x4{}; acc[0][1] = f32x4{}; }
  if (!h1) { acc[1][0] = f32x4{}; acc[1][1] = f32x4{}; }
}

template <bool TEACHER, bool F16>
__device__ __forceinline__ void wp_loop(const Ctx& C, const JobMap jm, const int nj, const int w, const int lane,
                                          char* smem, const uint32_t sbase, const bf16x8* W, const float* bias,
                                          const uint32_t* vb, const DadEncodeArgs& a) {
  using S = Shape<8>;
  constexpr int NP = 6;                  // 1-KB DMA pieces per wave per job (48 per job)
  constexpr int E = TEACHER ? 1 : 3;     // epilogue stores per job
  bf16x8 wf[S::NT][kKS];
  float bh[S::NT];
  float ssum[S::NT], scnt[S::NT];
  uint32_t bw[S::NT];
  const int hw = S::HW * w;
#pragma unroll
  for (int t = 0; t < S::NT; ++t)
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) wf[t][ks] = W[(size_t)(((hw >> 4) + t) * kKS + ks) * 64 + lane];
#pragma unroll
  for (int t = 0; t < S::NT; ++t) bh[t] = bias[hw + 16 * t + (lane & 15)];
  // pieces p = 6w + i of a job stage: tile p / 24 (rows 16 (p/24) ..), 1-KB piece p % 24 of it
  int prow[NP], pcol[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = NP * w + i;
    const int o = 1024 * (p % 24) + 16 * lane;
    const int r = o / kTileRow;
    prow[i] = 16 * (p / 24) + r;
    pcol[i] = 16 * (((o - kTileRow * r) >> 4) ^ (r & 15));
  }
  auto dma = [&](int j, int s) {
    const Job J = job_of(C, TEACHER, jm(min(j, nj - 1)));
    const char* base = reinterpret_cast<const char*>(J.kind == KIND_CLEAN ? a.x16c : (J.kind == KIND_STRONG ? a.x16s : a.x16w));
    const uint32_t dst = sbase + (uint32_t)(s * 2 * kTile) + 1024u * NP * (uint32_t)w;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int t = min(J.c * DAD_SLAB + prow[i], J.T - 1);
      dad_glds16(base + (size_t)(J.row0 + t) * (DAD_D * 2) + pcol[i], dst + 1024u * (uint32_t)i);
    }
  };
  int aoff[4];
  {
    const int ln = opaque(lane);
#pragma unroll
    for (int m = 0; m < 4; ++m) aoff[m] = (ln & 15) * kTileRow + 16 * ((4 * m + (ln >> 4)) ^ (ln & 15));
  }
  unsigned long long ph[5] = {0, 0, 0, 0, 0};
  int s_cur = 0;
  dma(0, 0);
  dma(1, 1);
  for (int j = 0; j < nj; ++j) {
    const unsigned long long c0 = WS_CLK();
    // DMA(j) landed once at most these younger ops remain: DMA(j+1) and the epilogue stores of
    // jobs max(0, j-2) .. j-1
    const int ne = min(j, 2);
    if (ne == 0) wait_vm<NP>();
    else if (ne == 1) wait_vm<NP + E>();
    else wait_vm<NP + 2 * E>();
    const unsigned long long c1 = WS_CLK();
    lds_barrier();
    const unsigned long long c2 = WS_CLK();
    dma(j + 2, s_cur == 0 ? kJS - 1 : s_cur - 1);
    const uint32_t vm = __builtin_amdgcn_readfirstlane(vb[j]);
    const unsigned long long c3 = WS_CLK();
    f32x4 acc[2][S::NT];
    wp_mfma2<F16>(smem + s_cur * 2 * kTile, aoff, wf, acc, vm);
    const unsigned long long c4 = WS_CLK();
    const Job J = job_of(C, TEACHER, jm(j));
    ws_epilogue<S, TEACHER, 0>(C, J, w, lane, vm & 0xffffu, bh, acc[0], ssum, scnt, bw);
    ws_epilogue<S, TEACHER, 1>(C, J, w, lane, vm >> 16, bh, acc[1], ssum, scnt, bw);
    s_cur = s_cur == kJS - 1 ? 0 : s_cur + 1;
    const unsigned long long c5 = WS_CLK();
    if (DAD_PROBE_ON) {
      ph[0] += c1 - c0; ph[1] += c2 - c1; ph[2] += c3 - c2; ph[3] += c4 - c3; ph[4] += c5 - c4;
    }
  }
  for (int k = 0; DAD_PROBE_ON && k < 5; ++k) WS_STAMP(4 + k, ph[k]);
  wait_vm<0>();
}

// Roles (dad_wp_job_range): teacher workgroups run the weak slabs with the teacher's W1, student
// workgroups the clean then the strong slabs with the student's W1, all on prepared rows.
template <bool F16>
__device__ __forceinline__ void encode_wp_body(const DadEncodeArgs& a, char* smem) {
  constexpr int WAVES = DAD_ENC_WS_THREADS / 64;
  const Ctx C = ctx_of(a);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  bool teacher;
  int j0, j1;
  dad_wp_job_range(blockIdx.x, a.ws_nt, a.ws_ns, C.Bc, C.Tc, C.ncc, C.Bn, C.Tn, C.ncn, C.Js, teacher, j0, j1);
  const JobMap jm{j0, 1};
  const int nj = j1 - j0;
  WS_STAMP(0, DAD_PROBE_WALL());
  WS_STAMP(3, ((unsigned long long)(teacher ? 0 : 1) << 16) | (unsigned long long)(2 * nj));
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
  WS_STAMP(1, DAD_PROBE_WALL());
  if (teacher) wp_loop<true, F16>(C, jm, nj, w, lane, smem, sbase, W, bias, vb, a);
  else wp_loop<false, F16>(C, jm, nj, w, lane, smem, sbase, W, bias, vb, a);
  WS_STAMP(2, DAD_PROBE_WALL());
}

#define DAD_WP_KERNEL(name, F16)                                                     \
  __global__ __launch_bounds__(DAD_ENC_WS_THREADS, 1) void name(DadEncodeArgs a) {   \
    DAD_GUARD_BLOCK(DAD_ENC_WS_THREADS);                                             \
    __shared__ __attribute__((aligned(16))) char smem[kLdsP];                        \
    encode_wp_body<F16>(a, smem);                                                    \
  }
DAD_WP_KERNEL(dad_encode_wp, false)
DAD_WP_KERNEL(dad_encode_wp_f16, true)
#undef DAD_WP_KERNEL
