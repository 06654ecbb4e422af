// Fused encoder forward for the DAD step (one launch covers all three encoder passes).
//
// Replaces, per step (I/train.py:399,406-410,439):
//   student_encoder(clean)                         Emotion2VecEncoder.forward, I/model.py:18-41
//   teacher_encoder(weak_augment(noisy))           + DataAugmentation.weak_augment, I/utils.py:328-331
//   student_encoder(strong_augment(noisy))         + strong_augment/_apply_temporal_masking, I/utils.py:333-375
//
// Work unit = one wave = one 32-row slab (utterance b, frames 32c..32c+31) x all 256 hidden
// units.  A noisy slab is read from HBM once and feeds BOTH the teacher (weak aug, teacher W1)
// and the student (strong aug, student W1) GEMMs.  The epilogue adds the bias, applies ReLU
// and the padding mask and reduces over the slab's frames, so the [B,T,256] activation never
// reaches HBM; it emits per-slab pooled sums, per-slab active counts (for d b1) and the
// ReLU'-and-valid bit mask the weight-gradient kernel consumes.
//
// Precision modes:  FP32 -> v_mfma_f32_32x32x2_f32 (exact f32 FMA chain; parity mode)
//                   BF16 -> v_mfma_f32_32x32x16_bf16 on the augmented tile rounded to bf16
//                           and the bf16 shadow of W1 (fp32 accumulate; throughput mode)
#include "dad_common.h"
#include "dad_kernels.h"

#ifdef DAD_PROBE_STAMPS
// diagnostic build only: per-workgroup [start, after-loop, end] wall clocks (100 MHz)
__device__ unsigned long long g_enc_stamps[4096 * 3];
extern "C" int dad_probe_read_stamps(void* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_enc_stamps), sizeof(unsigned long long) * 3 * n, 0,
                                  hipMemcpyDeviceToHost);
}
#define ENC_STAMP(k) \
  if (threadIdx.x == 0 && blockIdx.x < 4096) g_enc_stamps[blockIdx.x * 3 + (k)] = wall_clock64()
#else
#define ENC_STAMP(k)
#endif

namespace {

struct EncodeGeom {
  int b, c, noisy, T, nc;
  size_t sum_slab;     // slab index into part_sum for the (first) branch of this wave
  size_t row0;         // global row of frame 0 of this utterance ([b][T] layout)
};

// waves [0, Bn*ncn) are noisy slabs (when not warming up), the rest clean slabs
__device__ __forceinline__ EncodeGeom encode_geom(const DadEncodeArgs& a, int wid) {
  EncodeGeom e;
  const DadGeom& g = a.g;
  const int nnoisy = a.warmup ? 0 : g.Bn * g.ncn;
  e.noisy = wid < nnoisy;
  const int slab = e.noisy ? wid : wid - nnoisy;
  e.nc = e.noisy ? g.ncn : g.ncc;
  e.T = e.noisy ? g.Tn : g.Tc;
  e.b = slab / e.nc;
  e.c = slab - e.b * e.nc;
  e.sum_slab = e.noisy ? (size_t)g.Bc * g.ncc + slab : (size_t)slab;
  e.row0 = (size_t)e.b * e.T;
  return e;
}

// Temporal-mask start for utterance b (I/utils.py:370: randint(0, max(1, Tmax-mlen+1))).
__device__ __forceinline__ int tmask_start(const DadEncodeArgs& a, int b) {
  if (a.start) return (int)a.start[b];
  uint32_t h = dad_rng32((uint32_t)b, a.key_tstart);
  return (int)(((uint64_t)h * (uint64_t)a.start_hi) >> 32);
}

// Feature-dropout keep flag for channel d (I/utils.py:343: rand(D) > dropout_rate).
__device__ __forceinline__ float feat_keep(const DadEncodeArgs& a, int d) {
  float u = a.u ? a.u[d] : dad_uniform_at(a.key_feat, (uint32_t)d);
  return u > a.feat_p ? 1.0f : 0.0f;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// Augment 4 consecutive channels d..d+3 of row (b, t): weak and strong variants.
// Op order mirrors the reference: noise*std then add; *feature mask; temporal zero.
__device__ __forceinline__ void augment4(const DadEncodeArgs& a, f32x4 x, int grow, int d, bool tzero,
                                         f32x4& xw, f32x4& xs) {
  f32x4 nw, ns;
  if (a.nw) {
    nw = ld4(a.nw + (size_t)grow * DAD_D + d);
    ns = ld4(a.ns + (size_t)grow * DAD_D + d);
  } else {
    nw = dad_normal4(a.key_weak, (uint32_t)grow, (uint32_t)d);
    ns = dad_normal4(a.key_strong, (uint32_t)grow, (uint32_t)d);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float w = nw[e] * a.weak_std;
    xw[e] = x[e] + w;
    float s = ns[e] * a.strong_std;
    float v = (x[e] + s) * feat_keep(a, d + e);
    xs[e] = tzero ? 0.0f : v;
  }
}

// Pool one 32x256 accumulator set: bias + ReLU + padding mask + sum over the slab rows.
// sum_slab / cnt_slab index part_sum / part_cnt; bits_row (< 0: no bits) is the first
// row of this slab in the bits buffer.
__device__ __forceinline__ void encode_epilogue(const DadEncodeArgs& a, const f32x16* acc, const float* bias,
                                                size_t sum_slab, long cnt_slab, long bits_row, uint32_t vbits,
                                                uint32_t* lds_bits) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, kh = lane >> 5;
  const bool want_bits = bits_row >= 0;
  // all bias loads up front: a load between the part_sum stores would wait on each of them
  float bhs[DAD_HT];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) bhs[ht] = bias[ht * 32 + j];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) {
    const int h = ht * 32 + j;
    const float bh = bhs[ht];
    float s = 0.0f, n = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = dad_acc_row(r, kh);
      const bool v = (vbits >> row) & 1u;
      const float pre = acc[ht][r] + bh;
      const bool act = v && pre > 0.0f;
      s += act ? pre : 0.0f;
      n += act ? 1.0f : 0.0f;
      if (want_bits) {
        // the ballot is wave-uniform: every lane writes the same word to the same address
        // (no lane-0 branch per row)
        const uint64_t m = __ballot(act);
        const int row0 = dad_acc_row(r, 0);
        lds_bits[row0 * DAD_HT + ht] = (uint32_t)m;
        lds_bits[(row0 + 4) * DAD_HT + ht] = (uint32_t)(m >> 32);
      }
    }
    s += __shfl_xor(s, 32, 64);
    n += __shfl_xor(n, 32, 64);
    if (kh == 0) {
      a.part_sum[sum_slab * DAD_H + h] = s;
      if (cnt_slab >= 0) a.part_cnt[(size_t)cnt_slab * DAD_H + h] = n;
    }
  }
  if (want_bits) {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): lane 0's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    // 32 rows x 8 words = 1 KB per slab, stored contiguously: 16 B per lane
    const uint4 w = reinterpret_cast<const uint4*>(lds_bits)[lane];
    reinterpret_cast<uint4*>(a.bits + (size_t)bits_row * DAD_HT)[lane] = w;
  }
}

// epilogues of one wave: clean -> (clean sums, clean counts, clean bits);
// noisy -> teacher sums (no grads), then strong sums/counts/bits
__device__ __forceinline__ void encode_finish(const DadEncodeArgs& a, const EncodeGeom& e, const f32x16* acc0,
                                              const f32x16* acc1, uint32_t vbits, uint32_t* lb) {
  const DadGeom& g = a.g;
  if (!e.noisy) {
    encode_epilogue(a, acc0, a.b1_student, e.sum_slab, (long)e.sum_slab,
                    (long)e.b * g.tpc + (long)e.c * DAD_SLAB, vbits, lb);
  } else {
    const size_t nslab_n = (size_t)g.Bn * g.ncn;
    const size_t local = e.sum_slab - (size_t)g.Bc * g.ncc;
    encode_epilogue(a, acc0, a.b1_teacher, e.sum_slab, -1, -1, vbits, lb);
    encode_epilogue(a, acc1, a.b1_student, e.sum_slab + nslab_n, (long)((size_t)g.Bc * g.ncc + local),
                    (long)g.Bc * g.tpc + (long)e.b * g.tpn + (long)e.c * DAD_SLAB, vbits, lb);
  }
}

}  // namespace

// ------------------------------------------------------------------- FP32 (parity mode)
__global__ __launch_bounds__(DAD_ENC_F32_THREADS) void dad_encode_f32(DadEncodeArgs a) {
  DAD_GUARD_BLOCK(DAD_ENC_F32_THREADS);
  __shared__ __attribute__((aligned(16))) uint32_t lds_bits_all[4][DAD_SLAB * DAD_HT];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int wid = blockIdx.x * 4 + wv;
  if (wid >= (a.warmup ? 0 : a.g.Bn * a.g.ncn) + a.g.Bc * a.g.ncc) return;
  const EncodeGeom g = encode_geom(a, wid);
  const int i = lane & 31, kh = lane >> 5;
  const int t = g.c * DAD_SLAB + i;
  const bool tin = t < g.T;
  const int grow = (int)g.row0 + (tin ? t : 0);
  const uint8_t* pad = g.noisy ? a.mn : a.mc;
  const bool valid = tin && pad[g.row0 + t] == 0;
  const uint32_t vbits = (uint32_t)__ballot(valid);
  const float* X = (g.noisy ? a.xn : a.xc) + (size_t)grow * DAD_D;
  bool tzero = false;
  if (g.noisy && a.mask_len > 0) {
    const int st = tmask_start(a, g.b);
    tzero = t >= st && t < st + a.mask_len;
  }
  // B operands: student W1 (clean + strong), teacher W1 (weak)
  const float* Ws = a.w1_student + (size_t)i * DAD_D + 4 * kh;
  const float* Wt = a.w1_teacher + (size_t)i * DAD_D + 4 * kh;

  f32x16 acc0[DAD_HT], acc1[DAD_HT];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) {
    acc0[ht] = f32x16{};
    acc1[ht] = f32x16{};
  }
  // k ordering: step (d0, e, kh) uses channel d0 + 4*kh + e for BOTH operands
  if (!g.noisy) {
    for (int d0 = 0; d0 < DAD_D; d0 += 8) {
      const f32x4 x = tin ? ld4(X + d0 + 4 * kh) : f32x4{};
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht) {
        const f32x4 w = ld4(Ws + (size_t)ht * 32 * DAD_D + d0);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc0[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[e], w[e], acc0[ht], 0, 0, 0);
      }
    }
  } else {
    for (int d0 = 0; d0 < DAD_D; d0 += 8) {
      const int d = d0 + 4 * kh;
      const f32x4 x = tin ? ld4(X + d) : f32x4{};
      f32x4 xw, xs;
      augment4(a, x, grow, d, tzero, xw, xs);
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht) {
        const f32x4 wt = ld4(Wt + (size_t)ht * 32 * DAD_D + d0);
        const f32x4 ws = ld4(Ws + (size_t)ht * 32 * DAD_D + d0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(xw[e], wt[e], acc0[ht], 0, 0, 0);
          acc1[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[e], ws[e], acc1[ht], 0, 0, 0);
        }
      }
    }
  }
  encode_finish(a, g, acc0, acc1, vbits, lds_bits_all[wv]);
}

// ------------------------------------------------------------ BF16 (throughput mode)
// One wave = one GEMM on one 32-row slab: 32 rows x 256 hidden units x K=768 with
// v_mfma_f32_32x32x16_bf16 (8 accumulator tiles = 128 VGPRs -> 2 waves per SIMD).
// Workgroup = 8 waves sharing W1 through LDS:
//   noisy workgroup: 4 slabs; waves 0-3 teacher (weak aug, teacher W1), waves 4-7 student
//                    (strong aug, student W1) on the SAME slabs, so the second read of a
//                    slab's rows hits the CU's L1/L2 instead of HBM;
//   clean workgroup: 8 slabs, student W1.
// W1 streams through a double-buffered LDS ring in 32-column chunks ([256 h][4 x 16 B],
// 16-B chunk position XOR-swizzled by (h>>2)&3 so the ds_read_b128 B-fragment reads of
// 16 consecutive rows are bank-conflict free); x is prefetched two chunks ahead in
// registers (8 KB in flight per wave) and augmented + rounded to bf16 in registers.
#define ENC_WAVES 8
#define ENC_KC 32
#define ENC_NCH (DAD_D / ENC_KC)
static_assert(ENC_NCH % 2 == 0 && ENC_NCH >= 4, "bf16 encoder pipeline assumes an even chunk count");
#define ENC_WCHUNK_BYTES (DAD_H * ENC_KC * 2)   // 16 KB per weight per chunk

struct Bf16Geom {
  int kind;        // 0 clean-student, 1 noisy-teacher (weak), 2 noisy-student (strong), -1 idle
  int b, c, T;
  size_t row0, sum_slab;
  long cnt_slab, bits_row;
};

__device__ __forceinline__ Bf16Geom bf16_geom(const DadEncodeArgs& a, int& noisy_wg) {
  const DadGeom& g = a.g;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar branches
  const int nsn = a.warmup ? 0 : g.Bn * g.ncn;
  const int nwg_n = (nsn + 3) / 4;
  Bf16Geom e;
  noisy_wg = (int)blockIdx.x < nwg_n;
  int slab;
  if (noisy_wg) {
    slab = blockIdx.x * 4 + (wv & 3);
    e.kind = slab < nsn ? (wv < 4 ? 1 : 2) : -1;
  } else {
    slab = (blockIdx.x - nwg_n) * 8 + wv;
    e.kind = slab < g.Bc * g.ncc ? 0 : -1;
  }
  if (e.kind < 0) { e.b = e.c = 0; e.T = 1; e.row0 = 0; e.sum_slab = 0; e.cnt_slab = -1; e.bits_row = -1; return e; }
  const int nc = e.kind == 0 ? g.ncc : g.ncn;
  e.T = e.kind == 0 ? g.Tc : g.Tn;
  e.b = slab / nc;
  e.c = slab - e.b * nc;
  e.row0 = (size_t)e.b * e.T;
  const size_t nsc = (size_t)g.Bc * g.ncc;
  if (e.kind == 0) {
    e.sum_slab = slab; e.cnt_slab = slab; e.bits_row = (long)e.b * g.tpc + (long)e.c * DAD_SLAB;
  } else if (e.kind == 1) {
    e.sum_slab = nsc + slab; e.cnt_slab = -1; e.bits_row = -1;
  } else {
    e.sum_slab = nsc + (size_t)g.Bn * g.ncn + slab; e.cnt_slab = (long)(nsc + slab);
    e.bits_row = (long)g.Bc * g.tpc + (long)e.b * g.tpn + (long)e.c * DAD_SLAB;
  }
  return e;
}

__device__ __forceinline__ bf16x8 to_bf16x8(f32x4 lo, f32x4 hi) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = (__bf16)lo[e];
    r[e + 4] = (__bf16)hi[e];
  }
  return r;
}

// stage one 32-column chunk of (one or two) bf16 W1 matrices: global -> registers
struct WStage {
  u32x4 v[2][2];
};
template <bool TWO>
__device__ __forceinline__ void w_load(WStage& w, const __bf16* W0, const __bf16* W1, int ch) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int item = tid + q * 512;               // 1024 16-B pieces per matrix per chunk
    const int h = item >> 2, c = item & 3;
    const size_t off = (size_t)h * DAD_D + ch * ENC_KC + 8 * c;
    w.v[0][q] = *reinterpret_cast<const u32x4*>(W0 + off);
    if constexpr (TWO) w.v[1][q] = *reinterpret_cast<const u32x4*>(W1 + off);
  }
}
template <bool TWO>
__device__ __forceinline__ void w_store(const WStage& w, char* buf) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int item = tid + q * 512;
    const int h = item >> 2, c = item & 3;
    const int pos = c ^ ((h >> 2) & 3);
    *reinterpret_cast<u32x4*>(buf + h * 64 + pos * 16) = w.v[0][q];
    if constexpr (TWO) *reinterpret_cast<u32x4*>(buf + ENC_WCHUNK_BYTES + h * 64 + pos * 16) = w.v[1][q];
  }
}

struct XChunk {
  f32x4 v[2][2];    // [k-step][lo/hi]: lane (row r, half kh) holds columns 16ks + 8kh .. +7
};
// unconditional: rows past the utterance read its frame 0 (row clamped by the caller) and
// are discarded by the epilogue's valid mask, so no per-lane branch splits the vmcnt chain
__device__ __forceinline__ void x_load(XChunk& x, const float* row, int ch, int kh) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int d = ch * ENC_KC + 16 * ks + 8 * kh;
#ifdef DAD_PROBE_NOX
    x.v[ks][0] = f32x4{(float)d, 1.0f, 2.0f, 3.0f};
    x.v[ks][1] = f32x4{(float)kh, 1.0f, 2.0f, 3.0f};
    (void)row;
#else
    x.v[ks][0] = *reinterpret_cast<const f32x4*>(row + d);
    x.v[ks][1] = *reinterpret_cast<const f32x4*>(row + d + 4);
#endif
  }
}

// NOISE: 0 = counter RNG in-kernel, 1 = explicit noise tensors (parity mode draws)
// TWO: noisy workgroup (teacher + student weights, waves 0-3 weak / 4-7 strong) vs clean
template <int NOISE, bool TWO>
__device__ __forceinline__ void encode_bf16_body(const DadEncodeArgs& a, char (*wbuf)[2 * ENC_WCHUNK_BYTES],
                                                 uint32_t (*lds_bits_all)[DAD_SLAB * DAD_HT], float* featkeep) {
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 31, kh = lane >> 5;
  int noisy_wg;
  Bf16Geom e = bf16_geom(a, noisy_wg);
  e.kind = __builtin_amdgcn_readfirstlane(e.kind);
  const __bf16* W0 = TWO ? a.w1bf_teacher : a.w1bf_student;        // buffer half 0
  const __bf16* W1 = a.w1bf_student;                               // buffer half 1 (noisy only)
  // strong-aug feature keep flags for all 768 channels (I/utils.py:343), once per workgroup
  if constexpr (TWO)
    for (int d = threadIdx.x; d < DAD_D; d += 512) featkeep[d] = feat_keep(a, d);
  // per-wave row state
  const bool active = e.kind >= 0;
  const int t = e.c * DAD_SLAB + i;
  const bool tin = active && t < e.T;
  const int grow = (int)e.row0 + (tin ? t : 0);
  bool valid = false;
  if (tin) valid = (e.kind == 0 ? a.mc : a.mn)[e.row0 + t] == 0;
  const uint32_t vbits = (uint32_t)__ballot(valid);
  const float* xrow = (e.kind == 0 ? a.xc : a.xn) + (size_t)grow * DAD_D;
  const float* nrow = NOISE ? (e.kind == 2 ? a.ns : a.nw) + (size_t)grow * DAD_D : nullptr;
  bool tzero = false;
  if (e.kind == 2 && a.mask_len > 0) {
    const int st = tmask_start(a, e.b);
    tzero = t >= st && t < st + a.mask_len;
  }
  const int wsel = (TWO && wv >= 4) ? ENC_WCHUNK_BYTES : 0;   // student half of a noisy workgroup
  const bool noisy_kind = TWO && (e.kind == 1 || e.kind == 2);
  const bool strong = TWO && e.kind == 2;
  const uint32_t key = strong ? a.key_strong : a.key_weak;
  const float sd = strong ? a.strong_std : a.weak_std;

  f32x16 acc[DAD_HT];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) acc[ht] = f32x16{};

  auto compute = [&](int ch, const XChunk& x) {
    const char* wb = wbuf[ch & 1] + wsel;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int d = ch * ENC_KC + 16 * ks + 8 * kh;
      f32x4 lo = x.v[ks][0], hi = x.v[ks][1];
      if (noisy_kind) {
        f32x4 nlo, nhi;
        if constexpr (NOISE) {
          nlo = *reinterpret_cast<const f32x4*>(nrow + d);
          nhi = *reinterpret_cast<const f32x4*>(nrow + d + 4);
        } else {
#ifdef DAD_PROBE_NORNG
          nlo = f32x4{}; nhi = f32x4{};
#else
          nlo = dad_normal4(key, (uint32_t)grow, (uint32_t)d);
          nhi = dad_normal4(key, (uint32_t)grow, (uint32_t)(d + 4));
#endif
        }
        // feature keep flags read unconditionally (a per-lane tzero guard made them branches)
        f32x4 fk_lo = f32x4{1.0f, 1.0f, 1.0f, 1.0f}, fk_hi = fk_lo;
        if (strong) {
          fk_lo = *reinterpret_cast<const f32x4*>(featkeep + d);
          fk_hi = *reinterpret_cast<const f32x4*>(featkeep + d + 4);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // op order of the reference: noise*std, add; then feature mask; then temporal zero
          float v0 = lo[q] + nlo[q] * sd;
          float v1 = hi[q] + nhi[q] * sd;
          if (strong) {
            v0 = tzero ? 0.0f : v0 * fk_lo[q];
            v1 = tzero ? 0.0f : v1 * fk_hi[q];
          }
          lo[q] = v0;
          hi[q] = v1;
        }
      }
      const bf16x8 xa8 = to_bf16x8(lo, hi);
      if (strong && tin) *reinterpret_cast<bf16x8*>(a.xs_bf16 + (size_t)grow * DAD_D + d) = xa8;
      if (active) {
        const int c16 = ks * 2 + kh;
#pragma unroll
        for (int ht = 0; ht < DAD_HT; ++ht) {
          const int h = ht * 32 + i;
          const bf16x8 w = *reinterpret_cast<const bf16x8*>(wb + h * 64 + ((c16 ^ ((h >> 2) & 3)) * 16));
#ifdef DAD_PROBE_NOMFMA
          acc[ht][0] += (float)xa8[0] * (float)w[0];
#else
          acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa8, w, acc[ht], 0, 0, 0);
#endif
        }
      }
    }
  };

  // prologue: W chunk 0 -> LDS; W chunks 1, 2 and x chunks 0, 1 in flight in registers
  WStage wa, wb_;
  XChunk xa, xb;
  w_load<TWO>(wa, W0, W1, 0);
  w_load<TWO>(wb_, W0, W1, 1);
  x_load(xa, xrow, 0, kh);
  x_load(xb, xrow, 1, kh);
  w_store<TWO>(wa, wbuf[0]);
  w_load<TWO>(wa, W0, W1, 2);
  __syncthreads();

  // chunk ch: x in xa, W in wbuf[0]; W(ch+1) in wb_, W(ch+2) in wa.  ENC_NCH is even.
  // Every prefetch is issued unconditionally (chunk index clamped: the tail re-reads the
  // last, L2-hot chunk): a conditional load leaves the two paths with different pending
  // counts and the compiler then merges them into a full vmcnt(0) drain every chunk.
  const int last = ENC_NCH - 1;
  for (int ch = 0; ch < ENC_NCH; ch += 2) {
    compute(ch, xa);
    x_load(xa, xrow, min(ch + 2, last), kh);
#ifndef DAD_PROBE_NOW
    w_store<TWO>(wb_, wbuf[1]);
    w_load<TWO>(wb_, W0, W1, min(ch + 3, last));
#endif
    __syncthreads();
    compute(ch + 1, xb);
    x_load(xb, xrow, min(ch + 3, last), kh);
#ifndef DAD_PROBE_NOW
    w_store<TWO>(wa, wbuf[0]);            // past the end: overwrites a buffer nobody reads again
    w_load<TWO>(wa, W0, W1, min(ch + 4, last));
#endif
    __syncthreads();
  }
  if (wv == 0) ENC_STAMP(1);
  if (!active) return;
  const float* bias = e.kind == 1 ? a.b1_teacher : a.b1_student;
#ifdef DAD_PROBE_NOEPI
  if (acc[0][0] == 12345.0f && acc[7][15] == 54321.0f)   // keeps the accumulators live
#endif
  encode_epilogue(a, acc, bias, e.sum_slab, e.cnt_slab, e.bits_row, vbits, lds_bits_all[wv]);
  if (wv == 0) ENC_STAMP(2);
}

__global__ __launch_bounds__(DAD_ENC_BF16_THREADS, 1) void dad_encode_bf16(DadEncodeArgs a) {
  DAD_GUARD_BLOCK(DAD_ENC_BF16_THREADS);
  ENC_STAMP(0);
  __shared__ __attribute__((aligned(16))) char wbuf[2][2 * ENC_WCHUNK_BYTES];
  __shared__ __attribute__((aligned(16))) uint32_t lds_bits_all[ENC_WAVES][DAD_SLAB * DAD_HT];
  __shared__ __attribute__((aligned(16))) float featkeep[DAD_D];
  const int nsn = a.warmup ? 0 : a.g.Bn * a.g.ncn;
  if ((int)blockIdx.x >= (nsn + 3) / 4) encode_bf16_body<0, false>(a, wbuf, lds_bits_all, featkeep);
  else if (a.nw) encode_bf16_body<1, true>(a, wbuf, lds_bits_all, featkeep);
  else encode_bf16_body<0, true>(a, wbuf, lds_bits_all, featkeep);
}
