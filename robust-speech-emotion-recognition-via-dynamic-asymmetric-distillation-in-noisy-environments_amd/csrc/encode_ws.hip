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
// VGPRs, read in place as MFMA B operands) and streams 32-row jobs through LDS:
//
//   HBM 16-bit rows --LDS-DMA (6 x 1 KB per wave, straight into the XOR-swizzled tiles: lane l
//   of a piece loads the source chunk that lands at its slot; per-lane offsets from an LDS
//   table)--> one of 3 job stages (two 16-row tiles each) --ds_read_b128 A fragments
//   (conflict-free, two k-steps ahead)--> 96 v_mfma_f32_16x16x32_{f16,bf16} per wave per job,
//   accumulators starting at the bias --ReLU, valid mask, row sums, ReLU' words by lane
//   swaps--> slab partials + ReLU' bits
//
// PING-PONG schedule (wp_loop_pp): the two waves sharing a SIMD alternate between an MFMA phase
// (the SIMD's matrix pipe to themselves, s_setprio) and an overhead phase (the epilogue of the job
// they just multiplied and the LDS-DMA issue two jobs ahead), one workgroup barrier per phase.
// Round 4's loop (every wave: barrier, DMA issue, MFMAs, epilogue, per job) left the matrix pipe
// idle during each wave's overhead: 35.3 -> 28.2 us per launch (A/B on one box, B = 64, T = 300).
//
// Roles are per workgroup: TEACHER workgroups (teacher W1) run the weak slabs, STUDENT workgroups
// (student W1) the clean slabs and then the strong slabs, contiguous ranges balanced by live
// sub-slabs (dad_wp_job_range; host: wp_split in dad_abi.hip); a job whose second 16 rows hold no
// frame multiplies only the first.
#include <type_traits>

#include "dad_common.h"
#include "dad_kernels.h"
#include "dad_probe.h"

// per-workgroup stamps of the stamps build (dad_probe.h): [start, after the valid-bit prologue,
// end (100 MHz wall clock), role<<16 | sub-slabs, then wave-0 cycles summed over the loop in: MFMA
// phase, its end (vmcnt wait + barrier), epilogue + DMA issue, the overhead phase's barrier]
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

}  // namespace

#ifndef WP_PRIO
#define WP_PRIO 2
#endif

namespace {

constexpr int kJS = 3;                                   // 48-KB job stages (two 16-row tiles each)
constexpr int kOffPVB = kJS * 2 * kTile;                 // valid bits u32[DAD_ENC_WS_MAXJ]
constexpr int kOffSimd = kOffPVB + 4 * DAD_ENC_WS_MAXJ;       // SIMD id per wave
constexpr int kOffDMA = kOffSimd + 4 * 8;                      // per-lane DMA source offsets (12 KB)
constexpr int kLdsP = kOffDMA + 8 * 6 * 64 * 4;
static_assert(kLdsP <= 160 * 1024, "LDS budget");

}  // namespace

// ---- Ping-pong schedule -----------------------------------------------------------------------
// The two waves that share a SIMD are in different groups (grp, from the hardware SIMD id).  Time
// is cut into PHASES separated by one workgroup barrier each; a wave of group g multiplies job j in
// phase 2j + g (the MFMA phase: 96 MFMAs, the SIMD's matrix pipe to itself) and runs job j's
// epilogue and the LDS-DMA issue of job j + 2 in phase 2j + g + 1 (the overhead phase), while its
// partner multiplies.  So each SIMD's matrix pipe alternates between its two waves and the
// per-job overhead (epilogue, DMA issue, valid mask) hides under the partner's MFMAs instead of
// stalling both.  Every wave executes 2 nj + 1 barriers (group 1 idles in phase 0, group 0 in
// phase 2 nj).
//
// Stages: job J lives in stage J % 3.  Its pieces are issued by group 0 in phase 2J - 3 and by
// group 1 in phase 2J - 2; the first reader is group 0 in phase 2J.  Every wave waits vmcnt(0) at
// the end of its MFMA phase (it issued no memory op in it), i.e. group 0 at the end of phase
// 2J - 2 and group 1 at the end of 2J - 1, so all pieces of J have landed before the barrier that
// opens phase 2J.  Stage J % 3 last held job J - 3, read in phases 2J - 6 and 2J - 5, before either
// group starts refilling it.
// The fragment reads are inline asm with explicit lgkmcnt waits: left to the compiler, the reads
// of k-step ks sank to right before its MFMAs (register pressure), exposing the LDS latency on
// every k-step.  A wait names the fragments it guards as in/out operands, so no MFMA that reads
// them can be scheduled above it.  addr[m] = this tile's LDS byte address + aoff[m].
template <int OFF>
__device__ __forceinline__ void lds_rd128(bf16x8& x, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void lgkm_wait2(bf16x8& x0, bf16x8& x1) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(x0), "+v"(x1) : "i"(N));
}
template <int KS, bool TWO>
__device__ __forceinline__ void pp_read(bf16x8 (&xa)[3][2], const uint32_t (&addr)[4]) {
  if constexpr (KS < kKS) {
    lds_rd128<256 * (KS >> 2)>(xa[KS % 3][0], addr[KS & 3]);
    if constexpr (TWO) lds_rd128<kTile + 256 * (KS >> 2)>(xa[KS % 3][1], addr[KS & 3]);
  }
}
template <int KS, bool F16, bool TWO>
__device__ __forceinline__ void pp_kstep(bf16x8 (&xa)[3][2], const uint32_t (&addr)[4], const bf16x8 (&wf)[2][kKS],
                                         f32x4 (&acc)[2][2]) {
  if constexpr (KS < kKS) {
    pp_read<KS + 2, TWO>(xa, addr);
    // reads younger than k-step KS's: those of KS + 1 and KS + 2 that exist
    constexpr int younger = (KS + 1 < kKS ? 1 : 0) + (KS + 2 < kKS ? 1 : 0);
    lgkm_wait2<younger * (TWO ? 2 : 1)>(xa[KS % 3][0], xa[KS % 3][1]);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      mfma1<false, false, F16>(acc[0][t], xa[KS % 3][0], wf[t][KS]);
      if constexpr (TWO) mfma1<false, false, F16>(acc[1][t], xa[KS % 3][1], wf[t][KS]);
    }
    pp_kstep<KS + 1, F16, TWO>(xa, addr, wf, acc);
  }
}
// acc = bias + x . W1^T: the accumulators start at the bias (the epilogue adds nothing)
template <bool F16, bool TWO>
__device__ __forceinline__ void pp_mfma(const uint32_t (&addr)[4], const bf16x8 (&wf)[2][kKS], const float (&bh)[2],
                                        f32x4 (&acc)[2][2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    acc[0][t] = f32x4{bh[t], bh[t], bh[t], bh[t]};
    if constexpr (TWO) acc[1][t] = acc[0][t];
  }
  // A fragments two k-steps ahead of the MFMAs that use them (one MFMA wave per SIMD in this
  // phase: the fragment reads' latency is not covered by a partner wave)
  bf16x8 xa[3][2];
  if constexpr (!TWO) xa[0][1] = xa[1][1] = xa[2][1] = bf16x8{};
  pp_read<0, TWO>(xa, addr);
  pp_read<1, TWO>(xa, addr);
  pp_kstep<0, F16, TWO>(xa, addr, wf, acc);
  // MFMA D -> VALU readers of the epilogue (hipcc pads nothing after an asm MFMA)
  if constexpr (TWO) {
    asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0][0]), "v"(acc[0][1]), "v"(acc[1][0]), "v"(acc[1][1]));
  } else {
    asm volatile("s_nop 7\n\ts_nop 7" ::"v"(acc[0][0]), "v"(acc[0][1]));
    acc[1][0] = f32x4{};                           // rows 16..31 hold no frame (valid bits 0)
    acc[1][1] = f32x4{};
  }
}

// Epilogue of one 32-row job on bias-included accumulators: acc[half][t][r] is row 16 half + 4 g + r
// (g = lane >> 4) of hidden unit hw + 16 t + (lane & 15).  Per element (integer ops on the float's
// bits): m = max(bits, 0) = ReLU(pre), the ReLU' bit = min(m, 1) (pre > 0), the row sum += m; a lane's 8 bits of a hidden
// unit sit at 16 half + r, moved to their rows by << 4g and OR-ed over the row groups; the
// active-row count is the popcount of that 32-row word.  FULL: every row of the slab is a frame;
// otherwise the valid bits gate each element.  Stores: lanes 16 t + col -> h = hw + lane.
template <bool TEACHER, bool FULL>
__device__ __forceinline__ void pp_epilogue(const Ctx& C, const Job& J, int hw, int lane, uint32_t vm,
                                            const f32x4 (&acc)[2][2]) {
  const int g = lane >> 4;
  const uint32_t vg = vm >> (4 * g);
  float sv[2];
  uint32_t mv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float s = 0.0f;
    uint32_t word = 0;
#pragma unroll
    for (int half = 0; half < 2; ++half)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // ReLU on the bits: a float's int image is > 0 exactly when the float is > 0 (or a NaN of
        // sign 0, which then reaches the sum and the range flag); no canonicalising v_max pairs
        int mi = max(__float_as_int(acc[half][t][r]), 0);
        if constexpr (!FULL) mi &= __builtin_amdgcn_sbfe((int)vg, 16 * half + r, 1);   // valid: all ones
        s += __int_as_float(mi);
        if constexpr (!TEACHER) word |= min((uint32_t)mi, 1u) << (16 * half + r);
      }
    sv[t] = rowgroup_sum(s);
    if constexpr (!TEACHER) mv[t] = rowgroup_or(word << (4 * g));
  }
  if (lane < 32) {
    // wave-uniform row bases + the lane (no per-lane 64-bit addresses held across the loop)
    const int ln = opaque(lane);
    const bool t1 = ln >= 16;
    (C.part_sum + (size_t)J.sum_slab * DAD_H + hw)[ln] = t1 ? sv[1] : sv[0];
    if constexpr (!TEACHER) {
      const uint32_t m = t1 ? mv[1] : mv[0];
      (C.part_cnt + (size_t)J.cnt_slab * DAD_H + hw)[ln] = (float)__popc(m);
      (C.bits + (size_t)J.cnt_slab * DAD_H + hw)[ln] = m;
    }
  }
}

// six 1-KB LDS-DMA pieces: per lane, source base + off[i], off[i] read from the wave's LDS table
// ([i][lane] u32 at tab = the lane's entry of piece 0) in the same asm block (the compiler would
// otherwise forward the table's stores into six registers held across the loop); LDS destination
// dst + 1024 i (dst: the wave's first piece in the stage); M0 saved and restored around them
__device__ __forceinline__ void dad_glds16x6(const char* base, uint32_t tab, uint32_t dst) {
  uint32_t keep, o0, o1, o2, o3, o4, o5;
  asm volatile(
      "ds_read_b32 %1, %9\n\t"
      "ds_read_b32 %2, %9 offset:256\n\t"
      "ds_read_b32 %3, %9 offset:512\n\t"
      "ds_read_b32 %4, %9 offset:768\n\t"
      "ds_read_b32 %5, %9 offset:1024\n\t"
      "ds_read_b32 %6, %9 offset:1280\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b32 m0, %8\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %7\n\t"
      "s_add_u32 m0, %8, 0x400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %7\n\t"
      "s_add_u32 m0, %8, 0x800\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %7\n\t"
      "s_add_u32 m0, %8, 0xc00\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %7\n\t"
      "s_add_u32 m0, %8, 0x1000\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %5, %7\n\t"
      "s_add_u32 m0, %8, 0x1400\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %6, %7\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep), "=&v"(o0), "=&v"(o1), "=&v"(o2), "=&v"(o3), "=&v"(o4), "=&v"(o5)
      : "s"(base), "s"(dst), "v"(tab)
      : "memory", "scc");
}

template <bool TEACHER, bool F16>
__device__ __forceinline__ void wp_loop_pp(const Ctx& C, const JobMap jm, const int nj, const int w, const int lane,
                                           char* smem, const uint32_t sbase, const bf16x8* W, const float* bias,
                                           uint32_t* vb, const DadEncodeArgs& a, const int grp) {
  using S = Shape<8>;
  constexpr int NP = 6;                  // 1-KB DMA pieces per wave per job (48 per job)
  bf16x8 wf[S::NT][kKS];
  float bh[S::NT];
  const int hw = S::HW * w;
  // W1 into the registers (48 KB per wave: 393 KB per CU, at the ~70 GB/s a CU reads from L2 the
  // longest part of the prologue), and a use of every fragment, so the compiler's waits for them
  // sit in the prologue and not at the first MFMA inside the loop
  auto load_w1 = [&]() {
#pragma unroll
    for (int t = 0; t < S::NT; ++t)
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) wf[t][ks] = W[(size_t)(((hw >> 4) + t) * kKS + ks) * 64 + lane];
#pragma unroll
    for (int t = 0; t < S::NT; ++t) bh[t] = bias[hw + 16 * t + (lane & 15)];
  };
  auto w1_resident = [&]() {
#pragma unroll
    for (int t = 0; t < S::NT; ++t) {
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) asm volatile("" ::"v"(wf[t][ks]));
      asm volatile("" ::"v"(bh[t]));
    }
  };
  // Per-lane source offsets of the wave's pieces relative to the slab's first row: piece p = 6w + i
  // of a stage lands at LDS byte 1024 (p % 24) + 16 lane of tile p / 24, i.e. row r, slot k of the
  // XOR-swizzled tile, and loads source chunk k ^ r of row 16 (p / 24) + r.  Job-independent: kept
  // in LDS ([w][i][lane] u32) and read by dad_glds16x6.  Rows past the utterance's
  // end read the next rows of the prepared set (or the workspace after it): finite or not, they are
  // masked by the valid bits in the epilogue, and a row's output depends on that row only.
  uint32_t* dtab = reinterpret_cast<uint32_t*>(smem + kOffDMA) + w * (NP * 64);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = NP * w + i;
    const int o = 1024 * (p % 24) + 16 * lane;
    const int r = o / kTileRow;
    const int pc = 16 * (((o - kTileRow * r) >> 4) ^ (r & 15));
    dtab[i * 64 + lane] = (uint32_t)((16 * (p / 24) + r) * kTileRow + pc);
  }
  auto dma = [&](int j, int s) {
    const Job J = job_of(C, TEACHER, jm(j));
    const char* base = reinterpret_cast<const char*>(J.kind == KIND_CLEAN ? a.x16c : (J.kind == KIND_STRONG ? a.x16s : a.x16w)) +
                       (size_t)(J.row0 + J.c * DAD_SLAB) * (DAD_D * 2);
    dad_glds16x6(base, sbase + (uint32_t)(kOffDMA + 4 * (w * NP * 64) + 4 * opaque(lane)),
                 sbase + (uint32_t)(s * 2 * kTile) + 1024u * NP * (uint32_t)w);
  };
  unsigned long long ph[4] = {0, 0, 0, 0};
  // Prologue.  Every wave issues its pieces of jobs 0 and 1; group 0 (which multiplies in phase 0)
  // loads its W1 now, group 1 only after the first barrier, while group 0 multiplies job 0: the
  // CU's inbound bytes before phase 0 are jobs 0-1 + half of W1 instead of all of it (stamps: W1
  // and both jobs resident 7.6 us after the launch's start, the loop ~18.5 us).
  dma(0, 0);
  if (nj > 1) dma(1, 1);
  if (!grp) load_w1();
  // valid bits of every job (bit r = row r of the 32-row slab is a frame of the utterance)
  for (int p = w * 64 + lane; p < nj * DAD_SLAB; p += 64 * 8) {
    const Job J = job_of(C, TEACHER, jm(p / DAD_SLAB));
    const int t = J.c * DAD_SLAB + (p & (DAD_SLAB - 1));
    const uint8_t* pad = J.kind == KIND_CLEAN ? C.mc : C.mn;
    const bool v = t < J.T && pad[J.row0 + t] == 0;
    const uint64_t bal = __ballot(v);
    if ((lane & 31) == 0) vb[p / DAD_SLAB] = (uint32_t)(bal >> (lane & 32));
  }
  wait_vm<0>();
  if (!grp) w1_resident();
  lds_barrier();                                     // jobs 0 and 1 landed, valid bits visible
  WS_STAMP(8, DAD_PROBE_WALL());                     // (group 0's W1 resident)
  if (grp) {                                         // group 1: phase 0 (idle) loads its W1
    load_w1();
    wait_vm<0>();
    w1_resident();
    lds_barrier();
  }
  int s_cur = 0;
  for (int j = 0; j < nj; ++j) {
    // MFMA phase of job j
    const unsigned long long c0 = WS_CLK();
    const uint32_t vm = __builtin_amdgcn_readfirstlane(vb[j]);
    f32x4 acc[2][S::NT];
    // A-fragment addresses of k-steps 4q + m (rows lane & 15, k = 32 ks + 8 (lane >> 4) .. +7; the XOR
    // swizzle only touches the low 4 bits of the chunk index, so chunk (4 ks + g) ^ row = 16 (ks >> 2) +
    // ((4 (ks & 3) + g) ^ row): four per-lane addresses plus an immediate 256 (ks >> 2)), rebuilt per
    // job: no registers held across the loop
    uint32_t addr[4];
    {
      const int ln = opaque(lane);
      const uint32_t tb = sbase + (uint32_t)(s_cur * 2 * kTile) + (uint32_t)((ln & 15) * kTileRow);
#pragma unroll
      for (int m = 0; m < 4; ++m) addr[m] = tb + 16u * (uint32_t)((4 * m + (ln >> 4)) ^ (ln & 15));
    }
    // the MFMA wave takes the SIMD's issue first; the partner's overhead fills the gaps
    if (WP_PRIO) __builtin_amdgcn_s_setprio(WP_PRIO);
    if (vm >> 16) pp_mfma<F16, true>(addr, wf, bh, acc);
    else pp_mfma<F16, false>(addr, wf, bh, acc);
    if (WP_PRIO) __builtin_amdgcn_s_setprio(0);
    const unsigned long long c1 = WS_CLK();
    wait_vm<0>();                                    // this wave's pieces of job j + 1 (and j + 2) landed
    lds_barrier();
    const unsigned long long c2 = WS_CLK();
    // overhead phase: epilogue of job j, DMA issue of job j + 2
    const Job J = job_of(C, TEACHER, jm(j));
    if (vm == 0xffffffffu) pp_epilogue<TEACHER, true>(C, J, hw, lane, vm, acc);
    else pp_epilogue<TEACHER, false>(C, J, hw, lane, vm, acc);
    if (j + 2 < nj) dma(j + 2, s_cur == 0 ? kJS - 1 : s_cur - 1);
    s_cur = s_cur == kJS - 1 ? 0 : s_cur + 1;
    const unsigned long long c3 = WS_CLK();
    lds_barrier();
    const unsigned long long c4 = WS_CLK();
    if (DAD_PROBE_ON) {
      ph[0] += c1 - c0; ph[1] += c2 - c1; ph[2] += c3 - c2; ph[3] += c4 - c3;
    }
  }
  if (!grp) lds_barrier();                           // group 0: phase 2 nj idle
  for (int k = 0; DAD_PROBE_ON && k < 4; ++k) WS_STAMP(4 + k, ph[k]);
  // every wave's phase sums (stamps build): [2560 + 40 wg + 5 w] = MFMA, MFMA-end, overhead work,
  // overhead barrier, group | SIMD << 8
  if (DAD_PROBE_ON && lane == 0 && blockIdx.x < 256) {
    for (int k = 0; k < 4; ++k) DAD_PROBE_SET(ws_stamps, 2560 + 40 * blockIdx.x + 5 * w + k, ph[k]);
    DAD_PROBE_SET(ws_stamps, 2560 + 40 * blockIdx.x + 5 * w + 4,
                  grp | ((__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4) & 3u) << 8));
  }
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
  if (blockIdx.x == 0 && tid == 0 && a.pool_ready)   // (the tail launch that counts into it follows this one)
    for (int k = 0; k <= DAD_POOL_SHARDS; ++k) __hip_atomic_store(a.pool_ready + 32 * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (nj <= 0) return;
  const uint32_t sbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // valid bits of every job (bit r = row r of the 32-row slab is a frame of the utterance)
  uint32_t* vb = reinterpret_cast<uint32_t*>(smem + kOffPVB);
  // ping-pong group: 1 for the second wave on this wave's SIMD (hardware SIMD id, HW_ID[5:4])
  int* simd = reinterpret_cast<int*>(smem + kOffSimd);
  if (lane == 0) simd[w] = (int)((__builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4)) & 3u);
  lds_barrier();                        // simd visible (the valid bits follow in wp_loop_pp's prologue)
  int grp = 0;
  for (int v = 0; v < w; ++v) grp += simd[v] == simd[w];
  grp &= 1;
  const bf16x8* W = reinterpret_cast<const bf16x8*>(teacher ? a.w1h_teacher : a.w1h_student);
  const float* bias = teacher ? a.b1_teacher : a.b1_student;
  WS_STAMP(1, DAD_PROBE_WALL());
  if (teacher) wp_loop_pp<true, F16>(C, jm, nj, w, lane, smem, sbase, W, bias, vb, a, grp);
  else wp_loop_pp<false, F16>(C, jm, nj, w, lane, smem, sbase, W, bias, vb, a, grp);
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
