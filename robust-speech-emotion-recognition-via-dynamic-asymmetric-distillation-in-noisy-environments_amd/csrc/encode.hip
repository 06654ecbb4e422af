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
// This file is the FP32 parity mode: v_mfma_f32_32x32x2_f32 (an exact f32 FMA chain).  The
// BF16 throughput mode is the W-stationary encoder in encode_ws.hip.
#include "dad_common.h"
#include "dad_kernels.h"



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
  return dad_tstart_at(a.key_tstart, b, a.start_hi);
}

// Feature-dropout keep flag for channel d (I/utils.py:343: rand(D) > dropout_rate).
__device__ __forceinline__ float feat_keep(const DadEncodeArgs& a, int d) {
  return dad_feat_keep(a.u, a.key_feat, d, a.feat_p);
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
// sum_slab / cnt_slab index part_sum / part_cnt; bits_slab (< 0: no bits) is the slab's
// index in the ReLU' buffer, which holds one 32-bit row mask per (slab, h).
__device__ __forceinline__ void encode_epilogue(const DadEncodeArgs& a, const f32x16* acc, const float* bias,
                                                size_t sum_slab, long cnt_slab, long bits_slab, uint32_t vbits) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, kh = lane >> 5;
  const bool want_bits = bits_slab >= 0;
  // all bias loads up front: a load between the part_sum stores would wait on each of them
  float bhs[DAD_HT];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) bhs[ht] = bias[ht * 32 + j];
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) {
    const int h = ht * 32 + j;
    const float bh = bhs[ht];
    float s = 0.0f, n = 0.0f;
    uint32_t m = 0;   // this lane's rows of h (C layout: rows dad_acc_row(r, kh))
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = dad_acc_row(r, kh);
      const bool v = (vbits >> row) & 1u;
      const float pre = acc[ht][r] + bh;
      const bool act = v && pre > 0.0f;
      s += act ? pre : 0.0f;
      n += act ? 1.0f : 0.0f;
      m |= act ? (1u << row) : 0u;
    }
    s += __shfl_xor(s, 32, 64);
    n += __shfl_xor(n, 32, 64);
    m |= (uint32_t)__shfl_xor((int)m, 32, 64);
    if (kh == 0) {
      a.part_sum[sum_slab * DAD_H + h] = s;
      if (cnt_slab >= 0) a.part_cnt[(size_t)cnt_slab * DAD_H + h] = n;
      if (want_bits) a.bits[(size_t)bits_slab * DAD_H + h] = m;
    }
  }
}

// epilogues of one wave: clean -> (clean sums, clean counts, clean bits);
// noisy -> teacher sums (no grads), then strong sums/counts/bits
__device__ __forceinline__ void encode_finish(const DadEncodeArgs& a, const EncodeGeom& e, const f32x16* acc0,
                                              const f32x16* acc1, uint32_t vbits) {
  const DadGeom& g = a.g;
  if (!e.noisy) {
    encode_epilogue(a, acc0, a.b1_student, e.sum_slab, (long)e.sum_slab, (long)e.sum_slab, vbits);
  } else {
    const size_t nslab_n = (size_t)g.Bn * g.ncn;
    const size_t local = e.sum_slab - (size_t)g.Bc * g.ncc;
    const long strong_slab = (long)((size_t)g.Bc * g.ncc + local);
    encode_epilogue(a, acc0, a.b1_teacher, e.sum_slab, -1, -1, vbits);
    encode_epilogue(a, acc1, a.b1_student, e.sum_slab + nslab_n, strong_slab, strong_slab, vbits);
  }
}

}  // namespace

// ------------------------------------------------------------------- FP32 (parity mode)
// Software-pipelined over the 96 k-steps: the W1 fragments (16 x 16 B per lane, both networks
// on a noisy slab) and the x chunk of k-step n+1 are loaded while the MFMAs of k-step n run
// (unconditional loads, the last step's prefetch clamped), so the L2 round trip of W1 is
// not paid once per k-step.
template <bool NOISY, bool EXPLICIT>
__device__ __forceinline__ void encode_f32_slab(const DadEncodeArgs& a, const float* X, const float* Ws,
                                                const float* Wt, int grow, int kh, bool tin, bool tzero, const float* fk,
                                                f32x16 (&acc0)[DAD_HT], f32x16 (&acc1)[DAD_HT]) {
  constexpr int NW = NOISY ? 2 : 1;
  f32x4 xc = ld4(X + 4 * kh), wc[NW][DAD_HT];
  f32x4 nwc, nsc;
#pragma unroll
  for (int ht = 0; ht < DAD_HT; ++ht) {
    wc[0][ht] = ld4(Ws + (size_t)ht * 32 * DAD_D);
    if constexpr (NOISY) wc[1][ht] = ld4(Wt + (size_t)ht * 32 * DAD_D);
  }
  if constexpr (NOISY && EXPLICIT) {
    nwc = ld4(a.nw + (size_t)grow * DAD_D + 4 * kh);
    nsc = ld4(a.ns + (size_t)grow * DAD_D + 4 * kh);
  }
  for (int d0 = 0; d0 < DAD_D; d0 += 8) {
    const int dn = d0 + 8 < DAD_D ? d0 + 8 : d0;   // next k-step (the last one reloads itself)
    f32x4 xn = ld4(X + dn + 4 * kh), wn[NW][DAD_HT];
    f32x4 nwn, nsn;
#pragma unroll
    for (int ht = 0; ht < DAD_HT; ++ht) {
      wn[0][ht] = ld4(Ws + (size_t)ht * 32 * DAD_D + dn);
      if constexpr (NOISY) wn[1][ht] = ld4(Wt + (size_t)ht * 32 * DAD_D + dn);
    }
    if constexpr (NOISY && EXPLICIT) {
      nwn = ld4(a.nw + (size_t)grow * DAD_D + dn + 4 * kh);
      nsn = ld4(a.ns + (size_t)grow * DAD_D + dn + 4 * kh);
    }
    __builtin_amdgcn_sched_barrier(0);
    const f32x4 x = tin ? xc : f32x4{};
    if constexpr (!NOISY) {
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc0[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[e], wc[0][ht][e], acc0[ht], 0, 0, 0);
    } else {
      const int d = d0 + 4 * kh;
      f32x4 nw, ns;
      if constexpr (EXPLICIT) { nw = nwc; ns = nsc; }
      else {
        nw = dad_normal4(a.key_weak, (uint32_t)grow, (uint32_t)d);
        ns = dad_normal4(a.key_strong, (uint32_t)grow, (uint32_t)d);
      }
      // op order of the reference: noise * std then add; * feature mask; temporal zero
      const f32x4 kp = *reinterpret_cast<const f32x4*>(fk + d);
      f32x4 xw, xs;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xw[e] = x[e] + nw[e] * a.weak_std;
        const float v = (x[e] + ns[e] * a.strong_std) * kp[e];
        xs[e] = tzero ? 0.0f : v;
      }
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc0[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(xw[e], wc[1][ht][e], acc0[ht], 0, 0, 0);
          acc1[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(xs[e], wc[0][ht][e], acc1[ht], 0, 0, 0);
        }
    }
    xc = xn;
#pragma unroll
    for (int k = 0; k < NW; ++k)
#pragma unroll
      for (int ht = 0; ht < DAD_HT; ++ht) wc[k][ht] = wn[k][ht];
    if constexpr (NOISY && EXPLICIT) { nwc = nwn; nsc = nsn; }
  }
}

__global__ __launch_bounds__(DAD_ENC_F32_THREADS) void dad_encode_f32(DadEncodeArgs a) {
  DAD_GUARD_BLOCK(DAD_ENC_F32_THREADS);
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.pool_ready)   // the tail launch's fused pooling counter
    for (int k = 0; k <= DAD_POOL_SHARDS; ++k) __hip_atomic_store(a.pool_ready + 32 * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the strong augmentation's feature keep flags (I/utils.py:343), once per workgroup
  __shared__ __attribute__((aligned(16))) float fk[DAD_D];
  for (int d = threadIdx.x; d < DAD_D; d += DAD_ENC_F32_THREADS) fk[d] = dad_feat_keep(a.u, a.key_feat, d, a.feat_p);
  __syncthreads();
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
  const float* X = (g.noisy ? a.xn : a.xc) + dad_src_row(a.src, g.noisy, g.b, g.T, tin ? t : 0) * DAD_D;
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
  if (!g.noisy) encode_f32_slab<false, false>(a, X, Ws, Wt, grow, kh, tin, tzero, fk, acc0, acc1);
  else if (a.nw) encode_f32_slab<true, true>(a, X, Ws, Wt, grow, kh, tin, tzero, fk, acc0, acc1);
  else encode_f32_slab<true, false>(a, X, Ws, Wt, grow, kh, tin, tzero, fk, acc0, acc1);
  encode_finish(a, g, acc0, acc1, vbits);
}
