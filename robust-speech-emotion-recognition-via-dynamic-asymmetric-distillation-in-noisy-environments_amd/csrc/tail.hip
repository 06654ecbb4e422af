// The small "tail" of the DAD step: pooling finalisation + classifier forward, the losses,
// the DACP mask and the analytic backward down to dL/de (the per-utterance embedding grads).
//
//   dad_pool  (grid B)   : e = sum(slab partials)/max(1,len)       I/model.py:35-36
//                          logits = W2 (dropout(e)) + b2            I/model.py:54-64
//   dad_tail  (1 block)  : CE(label smoothing), softmax, certainty, DACP thresholds and
//                          mask, masked KL, classifier backward     I/train.py:397-471,
//                                                                   I/utils.py:400-507
//   dad_ecda  (grid C)   : ECDALoss forward + backward, one workgroup per class
//                                                                   I/utils.py:510-652
//
// Numerics: float32 with torch's op order where the result feeds a discrete decision
// (softmax -> certainty -> quantile -> EMA threshold -> mask); double accumulators for
// the batch sums.  The per-class set sizes are data dependent; everything is decided on
// device (no host sync), so the step is graph-capturable.
#include <type_traits>

#include "dad_common.h"
#include "dad_kernels.h"
#include "dad_prep.h"
#include "dad_probe.h"

// ECDA per-class phase wall clocks (100 MHz) of the stamps build (dad_probe.h): 16 slots per
// class, then the tail block's phases
#define ECDA_SLOTS 32
DAD_PROBE_BUFFER(ecda_stamps, DAD_C * ECDA_SLOTS + 16)
// dad_tail_ecda_w's preparation waves (spare block xb < 256, wave w): [start, end] wall clocks
DAD_PROBE_BUFFER(prep_stamps, 256 * 8 * 2)
#define ECDA_STAMP(k) \
  if (threadIdx.x == 0) DAD_PROBE_SET(ecda_stamps, (gridDim.x > DAD_C ? blockIdx.x - 1 : blockIdx.x) * ECDA_SLOTS + (k), DAD_PROBE_WALL())
// shader-clock stamp of wave 0 (cycle-level sub-phases of the stamps build), pinned in place
#define ECDA_CYC(k)                                                                          \
  do {                                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                       \
    if (threadIdx.x == 0)                                                                    \
      DAD_PROBE_SET(ecda_stamps, (gridDim.x > DAD_C ? blockIdx.x - 1 : blockIdx.x) * ECDA_SLOTS + (k), DAD_PROBE_CLK()); \
    __builtin_amdgcn_sched_barrier(0);                                                       \
  } while (0)
#define ECDA_STAMP_SIZES(c, n, ns) \
  do { DAD_PROBE_SET(ecda_stamps, (c) * ECDA_SLOTS + 10, (n)); DAD_PROBE_SET(ecda_stamps, (c) * ECDA_SLOTS + 11, (ns)); } while (0)
#define TAIL_STAMP(k) \
  if (threadIdx.x == 0) DAD_PROBE_SET(ecda_stamps, DAD_C * ECDA_SLOTS + (k), DAD_PROBE_WALL())
// shader-clock cycles at the tail block's start / end (slots 12 / 13): with the wall-clock
// stamps 0 / 1 they give the clock the block ran at
#define TAIL_CYCLES(k) \
  if (threadIdx.x == 0) DAD_PROBE_SET(ecda_stamps, DAD_C * ECDA_SLOTS + (k), DAD_PROBE_CLK())

// stamp from wave 1's first lane (the tail block's DACP / KL wave)
#define TAIL_STAMP_W1(k) \
  if (threadIdx.x == 64 && blockIdx.x == 0) DAD_PROBE_SET(ecda_stamps, DAD_C * ECDA_SLOTS + (k), DAD_PROBE_WALL())

#define TAIL_THREADS DAD_TAIL_THREADS

__device__ __forceinline__ float block_sum_f(float v, float* red) {
  v = dad_wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.0f;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) s += red[k];
  return s;
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = dad_wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = blockDim.x >> 6;
  for (int k = 0; k < nw; ++k) s += red[k];
  return s;
}


// ------------------------------------------------------------------------------ pool
// One wave per (utterance, branch): blocks [0, Bc) clean, [Bc, Bc+Bn) teacher (weak),
// [Bc+Bn, Bc+2Bn) student (strong).  Lane l owns hidden units 4l..4l+3, so a slab partial is
// one 16-B load per lane, every load of the block (pad bytes, all slab partials in batches of
// POOL_BATCH, active counts, W2 columns) is issued before the first sum, and the length and
// the four logit dot products are wave reductions: no LDS, no barrier (the 256-thread form
// issued 48 dword loads per thread and joined its 4 waves through LDS twice).  Embeddings sum
// the slab partials in slab order (I/model.py:35-36 masked mean pooling); logits
// W2 . dropout(e) + b2 (I/model.py:54-64; the teacher classifier's dropout is off).
//
// The same item runs in dad_tail_ecda_w's spare workgroups (SC1 = true: the tail and class
// blocks of that launch read the results after a counter hand-off, so every store is
// write-through, MI355X_MICROARCH.md "Valid forms").
static_assert(DAD_POOL_THREADS == 64 && DAD_H == 4 * 64, "dad_pool: one wave, 4 hidden units per lane");

template <bool SC1>
__device__ __forceinline__ void pool_st4(float* p, const f32x4& v) {
  if constexpr (SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  else *reinterpret_cast<f32x4*>(p) = v;
}
template <bool SC1, class T>
__device__ __forceinline__ void pool_st1(T* p, T v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// pool item blk (one wave, lane = 0..63): what one dad_pool workgroup does
template <bool SC1>
__device__ __forceinline__ void pool_item(const DadPoolArgs& a, const int blk, const int lane) {
  const DadGeom& g = a.g;
  const int kind = blk < g.Bc ? 0 : (blk < g.Bc + g.Bn ? 1 : 2);   // clean, teacher (weak), student (strong)
  const int b = kind == 0 ? blk : (kind == 1 ? blk - g.Bc : blk - g.Bc - g.Bn);
  const bool noisy = kind != 0, teacher = kind == 1;
  const int T = noisy ? g.Tn : g.Tc;
  const uint8_t* pad = (noisy ? a.mn : a.mc) + (size_t)b * T;
  const size_t nsc = (size_t)g.Bc * g.ncc, nsn = (size_t)g.Bn * g.ncn;
  const int nc = noisy ? g.ncn : g.ncc;
  const size_t slab0 = kind == 0 ? (size_t)b * g.ncc : (kind == 1 ? nsc + (size_t)b * g.ncn : nsc + nsn + (size_t)b * g.ncn);
  const size_t cslab0 = noisy ? nsc + (size_t)b * g.ncn : (size_t)b * g.ncc;   // active counts (clean / strong)
  const int erow = kind == 0 ? b : (kind == 1 ? g.Bc + b : g.Bc + g.Bn + b);
  const int h0 = 4 * lane;
  // First batch, every load issued before any sum: the pad bytes of frames lane + 64k (k <
  // POOL_PADB: T <= 512), the slab partials and active counts of slabs 0 .. POOL_BATCH-1 (index
  // clamped, contribution masked; summed in slab order).  (A pad loop with the sum inside waited
  // on each byte before the next load: one memory round trip per 64 frames, ahead of the slab
  // loads.)  The teacher also loads the strong counts it does not use: no load under a branch.
  constexpr int POOL_PADB = 8, POOL_BATCH = 16;
  uint8_t pv[POOL_PADB];
#pragma unroll
  for (int k = 0; k < POOL_PADB; ++k) pv[k] = pad[min(lane + 64 * k, T - 1)];
  f32x4 ps[POOL_BATCH], pc[POOL_BATCH];
#pragma unroll
  for (int k = 0; k < POOL_BATCH; ++k) {
    const int c = min(k, nc - 1);
    ps[k] = *reinterpret_cast<const f32x4*>(a.part_sum + (slab0 + c) * DAD_H + h0);
    pc[k] = *reinterpret_cast<const f32x4*>(a.part_cnt + (cslab0 + c) * DAD_H + h0);
  }
  // valid length (I/model.py:35: (1-mask).sum(dim=1)); frames past the first batch in a loop
  float len = 0.0f;
#pragma unroll
  for (int k = 0; k < POOL_PADB; ++k) len += ((lane + 64 * k < T) & (pv[k] == 0)) ? 1.0f : 0.0f;
  for (int t = lane + 64 * POOL_PADB; t < T; t += 64) len += pad[t] == 0 ? 1.0f : 0.0f;
  f32x4 ssum = f32x4{}, cnt = f32x4{};
#pragma unroll
  for (int k = 0; k < POOL_BATCH; ++k) {   // (+0 past the utterance's slabs: the sums are unchanged)
    const bool in = k < nc;
    ssum += in ? ps[k] : f32x4{};
    cnt += in ? pc[k] : f32x4{};
  }
  for (int c0 = POOL_BATCH; c0 < nc; c0 += POOL_BATCH) {   // utterances past 512 frames
#pragma unroll
    for (int k = 0; k < POOL_BATCH; ++k) {
      const int c = min(c0 + k, nc - 1);
      ps[k] = *reinterpret_cast<const f32x4*>(a.part_sum + (slab0 + c) * DAD_H + h0);
      pc[k] = *reinterpret_cast<const f32x4*>(a.part_cnt + (cslab0 + c) * DAD_H + h0);
    }
#pragma unroll
    for (int k = 0; k < POOL_BATCH; ++k) {
      const bool in = c0 + k < nc;
      ssum += in ? ps[k] : f32x4{};
      cnt += in ? pc[k] : f32x4{};
    }
  }
  const float* par = teacher ? a.teacher : a.student;
  f32x4 w2[DAD_C];
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) w2[c] = *reinterpret_cast<const f32x4*>(par + DAD_OFF_W2 + c * DAD_H + h0);
  const float bias = par[DAD_OFF_B2 + (lane & (DAD_C - 1))];
  f32x4 kv;
#pragma unroll
  for (int e = 0; e < 4; ++e)   // teacher classifier: dropout p = 0 (I/model.py:121); students: masks #1 / #2
    kv[e] = teacher ? 1.0f
                    : (kind == 0 ? keep_value(a.keep1, a.key_drop1, b, h0 + e, a.p_drop, a.drop_scale)
                                 : keep_value(a.keep2, a.key_drop2, b, h0 + e, a.p_drop, a.drop_scale));
  len = dad_wave_sum(len);
  f32x4 e;
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = ssum[k] / fmaxf(len, 1.0f);
  pool_st4<SC1>(a.emb + (size_t)erow * DAD_H + h0, e);
  const f32x4 d = teacher ? e : e * kv;
  float zp[DAD_C];
#pragma unroll
  for (int c = 0; c < DAD_C; ++c)
    zp[c] = dad_wave_sum(((w2[c][0] * d[0] + w2[c][1] * d[1]) + w2[c][2] * d[2]) + w2[c][3] * d[3]);
  if (lane < DAD_C)
    pool_st1<SC1>(a.logits + (size_t)erow * DAD_C + lane, (lane == 0 ? zp[0] : (lane == 1 ? zp[1] : (lane == 2 ? zp[2] : zp[3]))) + bias);
  // range check: a non-finite embedding or logit sets the sticky flag.  In FP16 steps an encoder
  // operand beyond +-65504 converts to inf, which turns every pre-activation of its row into
  // +-inf or NaN: the +inf units survive the ReLU into the pooled sum.
  const bool fin = __builtin_isfinite(e[0]) & __builtin_isfinite(e[1]) & __builtin_isfinite(e[2]) &
                   __builtin_isfinite(e[3]) & __builtin_isfinite(((zp[0] + zp[1]) + zp[2]) + zp[3]);
  if (__ballot(!fin) != 0 && lane == 0 && a.range_flag)
    __hip_atomic_fetch_or(a.range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!teacher) {
    // active-row count per (utterance, h) of the branch that gets a gradient (clean / strong);
    // the length, and the ECDA row flag (clean b / noisy Bc + b) starts at zero: the ECDA
    // workgroups write only what they own
    const int urow = noisy ? g.Bc + b : b;
    pool_st4<SC1>(a.cnt_tot + (size_t)urow * DAD_H + h0, cnt);
    if (lane == 0) {
      pool_st1<SC1>(a.vlen + urow, len);
      pool_st1<SC1>(a.eflag + urow, 0u);
    }
  }
  if (blk == 0 && lane < 2 * DAD_C) pool_st1<SC1>(a.tail_terms + lane, 0.0f);   // per-class ECDA terms and gates
}

__global__ __launch_bounds__(DAD_POOL_THREADS) void dad_pool(DadPoolArgs a) {
  DAD_GUARD_BLOCK(DAD_POOL_THREADS);
  pool_item<false>(a, (int)blockIdx.x, (int)threadIdx.x);
}

// Fused pooling hand-off (dad_tail_ecda_w): each pooling wave stores its item write-through (sc1),
// drains (s_waitcnt vmcnt(0)) and adds 1 to the counter; a tail / class block polls the counter
// (one lane, sc1 loads), then ONE agent-scope acquire, a drain and a barrier before any of its
// waves loads (MI355X_MICROARCH.md "Valid forms": producer sc1 stores, consumer poll + acquire).
// The poll is bounded (~0.2 s); on timeout it sets bit 1 of the range flag and the step's abort
// word and goes on (no hung device): the block then computes on partly pooled rows, but the
// weight gradient's loss-total block turns the total loss into NaN and dad_optim leaves the
// parameters, moments, teacher and DACP state of that step untouched.
// The counter is sharded per XCD (DAD_POOL_SHARDS words, each on a 128-B line of its own: the
// arrivals of one XCD serialise on one line only) and a poll sums the shards.
__device__ __forceinline__ void pool_publish(uint32_t* ready, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & (DAD_POOL_SHARDS - 1);   // HW_REG_XCC_ID
    __hip_atomic_fetch_add(ready + 32 * xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void pool_wait(uint32_t* ready, uint32_t n, uint32_t* range_flag) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    uint32_t spins = 0;
    for (;;) {
      const uint32_t v = lane < DAD_POOL_SHARDS ? __hip_atomic_load(ready + 32 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      if ((uint32_t)dad_wave_sum((float)v) >= n) break;   // (exact: at most a few hundred arrivals)
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 23)) {
        if (lane == 0) {   // bit 1 of the sticky flag, and this step's abort word: no update (dad_optim)
          if (range_flag) __hip_atomic_fetch_or(range_flag, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(ready + DAD_POOL_ABORT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
    }
    if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------ tail
// Latency design (one workgroup, ~30 dependent phases): every global input is requested at
// kernel entry -- logits, labels, the DACP state, W2 and the embedding values of the
// classifier backward -- so a single memory round trip is paid; the O(B^2) DACP ranks, the
// per-class epoch statistics and the b2 reduction are spread over the whole block with
// fixed-order (deterministic) combines instead of serial loops.

// fixed-order block reduction of 4 doubles (one per class), result valid in all threads
__device__ __forceinline__ void block_sum4_d(double (&v)[4], double (*red)[4]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = dad_wave_sum_d(v[c]);
  __syncthreads();
  if (l == 0)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[w][c] = v[c];
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    double s = 0.0;
    for (int k = 0; k < TAIL_THREADS / 64; ++k) s += red[k][c];
    v[c] = s;
  }
}

struct TailSmem {
  double dred[16];
  double dred4[TAIL_THREADS / 64][4];
  float fred[16];
  float gz[2][DAD_MAX_BATCH][DAD_C];       // dL/dz clean, strong
  float sq[DAD_MAX_BATCH][DAD_C];          // teacher probs
  float ss[DAD_MAX_BATCH];                 // certainty scores
  int sp[DAD_MAX_BATCH];                   // pseudo labels
  float sm[DAD_MAX_BATCH];                 // mask
  float srt[DAD_C][DAD_MAX_BATCH];         // per-class sorted scores
  int ncls[DAD_C];
  float tau_new[DAD_C];
  float dstate[20];                        // DACP state: tau | Q | (sums) | (counts) | anchors
};

// DACPManager.calculate_certainty_scores (I/utils.py:400-428) of one probability row:
// pseudo-label = first argmax, score = max_prob * (1 - H / log2 C) with
// H = -sum q log2(q + 1e-8) (log2(NUM_CLASSES) = 2), or max_prob without the entropy term
__device__ __forceinline__ void certainty_from_probs(const float (&q)[4], bool entropy, float& s, int& pred) {
  float mx = -1.0f;
  pred = 0;
  for (int c = 0; c < 4; ++c)
    if (q[c] > mx) { mx = q[c]; pred = c; }
  s = mx;
  if (entropy) {
    float ent = 0.0f;
    for (int c = 0; c < 4; ++c) ent += q[c] * log2f(q[c] + 1e-8f);
    ent = -ent;
    s = mx * (1.0f - ent / 2.0f);
  }
}

// teacher probs (I/train.py:409-410), certainty score and pseudo-label (I/utils.py:400-428);
// the fixed-threshold branch (I/train.py:417-420) uses max_prob
__device__ __forceinline__ void teacher_certainty(const float (&z)[4], const dad_config& cfg, float (&q)[4],
                                                  float& s, int& pred) {
  float m = -INFINITY;
  for (int c = 0; c < 4; ++c) m = fmaxf(m, z[c]);
  float e[4], se = 0.0f;
  for (int c = 0; c < 4; ++c) { e[c] = expf(z[c] - m); se += e[c]; }
  for (int c = 0; c < 4; ++c) q[c] = e[c] / se;
  certainty_from_probs(q, cfg.use_dacp && cfg.use_entropy, s, pred);
}

// DACPManager.calculate_mask thresholds (I/utils.py:449-507): per-class ranks of the scores,
// torch.quantile(linear) of each class, sigmoid class weights, floored + EMA-blended tau.
// Entry: ncls[] zeroed and ss/sp visible (barrier done by the caller).  Exit: tau_new[] and
// wc[] valid in all threads.  tf/extras (nullable): the per-step outputs of the tail block.
// Shared by the tail block and the ECDA blocks of dad_tail_ecda, so both derive the same mask.
template <int SRT = DAD_MAX_BATCH>
__device__ __forceinline__ void dacp_thresholds(const dad_config& cfg, int Bn, const float* ss, const int* sp,
                                                float (*srt)[SRT], int* ncls, const float* dstate,
                                                float* tau_new, float* wcs, float* tf, float* extras,
                                                bool stamp = false) {
  const int tid = threadIdx.x;
  // rank of each score inside its pseudo-label class (ties by index): 16 threads per
  // utterance, each counting a strided share of the others, combined by a 16-lane sum
  {
    const int bb = tid >> 4, part = tid & 15;
    for (int b0 = 0; b0 < Bn; b0 += TAIL_THREADS / 16) {
      const int b = b0 + bb;
      int cnt = 0, c = 0;
      float sv = 0.0f;
      if (b < Bn) {
        c = sp[b];
        sv = ss[b];
        int k = part;
        for (; k + 48 < Bn; k += 64) {   // four candidates per LDS round trip
          float o[4];
          int pc[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) { o[u] = ss[k + 16 * u]; pc[u] = sp[k + 16 * u]; }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kk = k + 16 * u;
            cnt += (pc[u] == c && (o[u] < sv || (o[u] == sv && kk < b))) ? 1 : 0;
          }
        }
        for (; k < Bn; k += 16) {
          const float o = ss[k];
          cnt += (sp[k] == c && (o < sv || (o == sv && k < b))) ? 1 : 0;
        }
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 16);
      if (b < Bn && part == 0) {
        srt[c][cnt] = sv;
        atomicAdd(&ncls[c], 1);
      }
    }
  }
  __syncthreads();
  if (stamp) TAIL_STAMP(8);
  if (tid < DAD_C) {
    const int c = tid;
    const float* Qs = dstate + 4;
    const float qmean = (((Qs[0] + Qs[1]) + Qs[2]) + Qs[3]) / 4.0f;
    const float wc = 1.0f / (1.0f + expf(-(cfg.dacp_k * (Qs[c] - qmean))));
    const int n = ncls[c];
    float that;
    if (n > 0) {
      // torch.quantile(linear): rank = q*(n-1) in f32, lerp(below, above, rank-floor)
      const float rank = cfg.dacp_gamma * (float)(n - 1);
      const int lo = (int)rank;
      const int hi = (int)ceilf(rank);
      const float wgt = rank - (float)lo;
      const float vlo = srt[c][lo], vhi = srt[c][hi];
      that = wgt < 0.5f ? vlo + wgt * (vhi - vlo) : vhi - (vhi - vlo) * (1.0f - wgt);
    } else {
      that = dstate[c];
    }
    const float adj = cfg.dacp_lambda * (wc - 0.5f);
    const float fl = fmaxf(that + adj, dstate[16 + c]);
    const float tn = cfg.dacp_alpha * dstate[c] + cfg.dacp_one_m_alpha * fl;
    tau_new[c] = tn;
    wcs[c] = wc;
    if (tf) {
      tf[DAD_T_W + c] = wc;
      tf[DAD_T_TAU_BEFORE + c] = dstate[c];
      tf[DAD_T_TAU_AFTER + c] = tn;
      tf[DAD_T_FLOORED + c] = fl;
      tf[DAD_T_TAU_HAT + c] = that;
      extras[0 + c] = fl;
    }
  }
  __syncthreads();
  if (stamp) TAIL_STAMP(9);
}

__device__ __forceinline__ void tail_block(const DadTailArgs& a, TailSmem& T) {
  TAIL_STAMP(0);
  TAIL_CYCLES(12);
  const dad_config& cfg = a.cfg;
  const int B = cfg.B;                       // clean utterances
  const int Bn = cfg.warmup ? 0 : cfg.Bn;    // noisy utterances
  const int tid = threadIdx.x;
  double* dred = T.dred;
  auto& dred4 = T.dred4;
  float* fred = T.fred;
  auto& gz = T.gz;
  auto& sq = T.sq;
  float* ss = T.ss;
  int* sp = T.sp;
  float* sm = T.sm;
  float* dstate = T.dstate;
  float wc_unused[DAD_C];

  float* tf = a.tailf;
  float* extras = a.grad + DAD_NPARAM;
  const float* z0 = a.logits;
  const float* z1 = a.logits + (size_t)B * DAD_C;
  const float* z2 = a.logits + (size_t)(B + Bn) * DAD_C;
  const float eps = cfg.ls_eps;

  // ---- every global input up front (one round trip; consumed in this order)
  f32x4 zc = f32x4{}, zt = f32x4{}, zs = f32x4{};
  int yb = 0;
  if (tid < B) { zc = reinterpret_cast<const f32x4*>(z0)[tid]; yb = (int)a.yc[tid]; }
  if (tid < Bn) { zt = reinterpret_cast<const f32x4*>(z1)[tid]; zs = reinterpret_cast<const f32x4*>(z2)[tid]; }
  if (tid >= TAIL_THREADS - 20) dstate[tid - (TAIL_THREADS - 20)] = a.dacp[tid - (TAIL_THREADS - 20)];

  // ---- supervised CE with label smoothing on the clean logits (I/train.py:364,400)
  double ce_part = 0.0;
  for (int b = tid; b < B; b += TAIL_THREADS) {
    float z[4], m = -INFINITY;
    if (b == tid) { z[0] = zc[0]; z[1] = zc[1]; z[2] = zc[2]; z[3] = zc[3]; }
    else for (int c = 0; c < 4; ++c) z[c] = z0[b * 4 + c];
    for (int c = 0; c < 4; ++c) m = fmaxf(m, z[c]);
    float se = 0.0f;
    for (int c = 0; c < 4; ++c) se += expf(z[c] - m);
    const float lse = m + logf(se);
    const int y = b == tid ? yb : (int)a.yc[b];
    float lsum = 0.0f;
    for (int c = 0; c < 4; ++c) {
      const float ls = z[c] - lse;
      lsum += ls;
      const float p = expf(ls);
      gz[0][b][c] = (p - (c == y ? 1.0f - eps : 0.0f) - eps * 0.25f) / (float)B;
    }
    ce_part += -(1.0 - (double)eps) * (double)(z[y] - lse) - (double)eps * 0.25 * (double)lsum;
  }
  const double ce = block_sum_d(ce_part, dred) / (double)B;
  TAIL_STAMP(2);

  float kl = 0.0f, msum = 0.0f;
  int kl_on = 0;
  if (!cfg.warmup) {
    // ---- teacher probs (I/train.py:409-410) and certainty (I/utils.py:400-428)
    for (int b = tid; b < Bn; b += TAIL_THREADS) {
      float z[4], q[4], s;
      int pred;
      if (b == tid) { z[0] = zt[0]; z[1] = zt[1]; z[2] = zt[2]; z[3] = zt[3]; }
      else for (int c = 0; c < 4; ++c) z[c] = z1[b * 4 + c];
      teacher_certainty(z, cfg, q, s, pred);
      for (int c = 0; c < 4; ++c) sq[b][c] = q[c];
      ss[b] = s;
      sp[b] = pred;
    }
    if (tid < DAD_C) T.ncls[tid] = 0;
    __syncthreads();
    TAIL_STAMP(3);
    if (cfg.use_dacp) {
      // ---- DACPManager.calculate_mask (I/utils.py:449-507)
      dacp_thresholds(cfg, Bn, ss, sp, T.srt, T.ncls, dstate, T.tau_new, wc_unused, tf, extras, true);
      // mask, and the epoch statistics for update_class_quality_scores_epoch
      // (I/utils.py:503-505): per-class score sums and counts, fixed-order block reduction
      for (int b = tid; b < Bn; b += TAIL_THREADS) sm[b] = ss[b] >= T.tau_new[sp[b]] ? 1.0f : 0.0f;
      double st4[4] = {0.0, 0.0, 0.0, 0.0}, ct4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int b = tid; b < Bn; b += TAIL_THREADS)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          st4[c] += sp[b] == c ? (double)ss[b] : 0.0;
          ct4[c] += sp[b] == c ? 1.0 : 0.0;
        }
      TAIL_STAMP(10);
      block_sum4_d(st4, dred4);
      block_sum4_d(ct4, dred4);
      TAIL_STAMP(11);
      if (tid < DAD_C) {
        extras[4 + tid] = (float)st4[tid];
        extras[8 + tid] = (float)ct4[tid];
      }
    } else {
      // fixed threshold (I/train.py:417-420): mask = float(max prob >= thr), weights = ones
      for (int b = tid; b < Bn; b += TAIL_THREADS) sm[b] = ss[b] >= cfg.fixed_thr ? 1.0f : 0.0f;
      if (tid < DAD_C) {
        tf[DAD_T_W + tid] = 1.0f;
        extras[0 + tid] = 0.0f;
        extras[4 + tid] = 0.0f;
        extras[8 + tid] = 0.0f;
      }
    }
    __syncthreads();
    TAIL_STAMP(4);
  }
  if (!cfg.warmup) {
    float mpart = 0.0f;
    for (int b = tid; b < Bn; b += TAIL_THREADS) mpart += sm[b];
    msum = block_sum_f(mpart, fred);
    kl_on = msum > 1.0f;   // I/train.py:444 (mask.sum().item() > 1)
    // ---- masked consistency KL(q || p_student) (I/train.py:445-447) + its logit grad
    double kl_part = 0.0;
    const float denom = msum + 1e-8f;
    for (int b = tid; b < Bn; b += TAIL_THREADS) {
      float z[4], m = -INFINITY;
      if (b == tid) { z[0] = zs[0]; z[1] = zs[1]; z[2] = zs[2]; z[3] = zs[3]; }
      else for (int c = 0; c < 4; ++c) z[c] = z2[b * 4 + c];
      for (int c = 0; c < 4; ++c) m = fmaxf(m, z[c]);
      float se = 0.0f;
      for (int c = 0; c < 4; ++c) se += expf(z[c] - m);
      const float lse = m + logf(se);
      float klb = 0.0f;
      for (int c = 0; c < 4; ++c) {
        const float q = sq[b][c];
        const float ls = z[c] - lse;
        klb += q > 0.0f ? q * (logf(q) - ls) : 0.0f;
        gz[1][b][c] = kl_on ? cfg.w_kl * sm[b] * (expf(ls) - q) / denom : 0.0f;
      }
      kl_part += (double)(klb * sm[b]);
    }
    const double kls = block_sum_d(kl_part, dred);
    kl = kl_on ? (float)(kls / (double)denom) : 0.0f;
    TAIL_STAMP(5);
  }
  // ---- per-sample outputs (noisy batch) for inspection / ECDA
  for (int b = tid; b < Bn; b += TAIL_THREADS) {
    tf[DAD_TAIL_HDR + b] = ss[b];
    tf[DAD_TAIL_HDR + Bn + b] = (float)sp[b];
    tf[DAD_TAIL_HDR + 2 * Bn + b] = sm[b];
    for (int c = 0; c < 4; ++c) tf[DAD_TAIL_HDR + 3 * Bn + b * 4 + c] = sq[b][c];
  }
  if (tid == 0) {
    tf[DAD_T_CE] = (float)ce;
    tf[DAD_T_KL] = kl;
    tf[DAD_T_SCL] = 0.0f;
    tf[DAD_T_MSUM] = msum;
    tf[DAD_T_KL_ON] = (float)kl_on;
    tf[DAD_T_ECDA_ON] = (kl_on && cfg.ecda_on) ? 1.0f : 0.0f;
  }
  __syncthreads();
  TAIL_STAMP(6);
  // ---- dL/dz of every utterance for the weight-gradient kernels (which rebuild the
  // classifier part of dL/de on the fly, I/model.py:62-63), the b2 grad, ECDA row flags
  for (int b = tid; b < B; b += TAIL_THREADS)
    *reinterpret_cast<f32x4*>(a.gzb + (size_t)b * DAD_C) = f32x4{gz[0][b][0], gz[0][b][1], gz[0][b][2], gz[0][b][3]};
  for (int b = tid; b < Bn; b += TAIL_THREADS)
    *reinterpret_cast<f32x4*>(a.gzb + (size_t)(B + b) * DAD_C) =
        f32x4{gz[1][b][0], gz[1][b][1], gz[1][b][2], gz[1][b][3]};
  double b2s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = tid; b < B; b += TAIL_THREADS)
#pragma unroll
    for (int c = 0; c < 4; ++c) b2s[c] += (double)gz[0][b][c];
  for (int b = tid; b < Bn; b += TAIL_THREADS)
#pragma unroll
    for (int c = 0; c < 4; ++c) b2s[c] += (double)gz[1][b][c];
  block_sum4_d(b2s, dred4);
  TAIL_STAMP(7);
  if (tid < 4) a.grad[DAD_OFF_B2 + tid] = (float)b2s[tid];
  TAIL_CYCLES(13);
  TAIL_STAMP(1);
}

__global__ __launch_bounds__(TAIL_THREADS) void dad_tail(DadTailArgs a) {
  DAD_GUARD_BLOCK(TAIL_THREADS);
  __shared__ TailSmem T;
  tail_block(a, T);
}

// ------------------------------------------------------------------------------ ECDA
// One workgroup per class (I/utils.py:601-632 loop body); the global-MMD ablation
// (I/utils.py:633-650) runs in workgroup 0.  Each workgroup only writes the embedding
// grads of ITS class members (clean: label == c, noisy: masked & pseudo-label == c), so
// no atomics are needed and the result is deterministic.

#define ECDA_THREADS DAD_ECDA_THREADS
static_assert(ECDA_THREADS % DAD_H == 0 && ECDA_THREADS >= DAD_H, "ECDA column groups");
#define ECDA_NZ 80                          // members staged in LDS (n <= 80); larger sets read global
#define ECDA_NG (ECDA_THREADS / 64)         // row groups (one wave each) of the centroid pass
#define ECDA_PRE_U 8                        // rows per group held in registers from kernel entry
#define ECDA_PRE (ECDA_NG * ECDA_PRE_U)     // batches of at most this many rows prefetch every row

struct EcdaSmem {
  float z[ECDA_NZ * DAD_H];       // staged member embeddings (before that: centroid partials)
  float dm[ECDA_NZ * ECDA_NZ];    // pairwise distances, then symmetric MMD coefficients
  int idx[2 * DAD_MAX_BATCH];     // member list: [0,ns) clean rows, [ns,n) noisy rows
  float wt[2 * DAD_MAX_BATCH];    // member weights
  int pos[2 * ECDA_PRE];          // inverse of idx (prefetch path): clean row b -> [b], noisy row b -> [ECDA_PRE + b]
  float cent[DAD_C][DAD_H];
  double dred[ECDA_THREADS / 64][3];
  float fred[ECDA_THREADS / 64];
  int cnt_clean[DAD_C], cnt_noisy[DAD_C];
  int lab[DAD_MAX_BATCH];         // clean labels
  int prd[DAD_MAX_BATCH];         // noisy pseudo-labels, -1 where not masked in
  float scr[DAD_MAX_BATCH];       // noisy certainty scores
  int wcount[ECDA_THREADS / 64];
  float repg[DAD_H];              // repulsion grad of this class's noisy members, per hidden unit
};

// fixed-order block reduction of NV doubles (one barrier pair for all), valid in all threads
template <int NV>
__device__ __forceinline__ void ecda_block_sum_d(EcdaSmem& S, double (&v)[NV]) {
  static_assert(NV <= 3, "dred holds 3 values per wave");
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = dad_wave_sum_d(v[k]);
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) S.dred[threadIdx.x >> 6][k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < ECDA_THREADS / 64; ++w) s += S.dred[w][k];
    v[k] = s;
  }
}

__device__ __forceinline__ float ecda_block_sum_f(EcdaSmem& S, float v) {
  v = dad_wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) S.fred[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < ECDA_THREADS / 64; ++k) s += S.fred[k];
  return s;
}

// Ordered block-wide compaction: appends every i in [0, n) with flag(i) to S.idx (and
// weight(i) to S.wt) after position `base`, in ascending i; inv (nullable) gets i's position.
// Returns the new length.
template <typename Flag, typename Wgt>
__device__ int ecda_compact(EcdaSmem& S, int n, int base, Flag flag, Wgt weight, int* inv) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int c0 = 0; c0 < n; c0 += ECDA_THREADS) {
    const int i = c0 + tid;
    const bool f = i < n && flag(i);
    const float wi = f ? weight(i) : 0.0f;   // in flight across the barrier
    const uint64_t bal = __ballot(f);
    if (lane == 0) S.wcount[w] = __popcll(bal);
    __syncthreads();
    int pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < ECDA_THREADS / 64; ++k) {
      const int ck = S.wcount[k];
      pre += k < w ? ck : 0;
      tot += ck;
    }
    if (f) {
      const int pos = base + pre + __popcll(bal & ((1ull << lane) - 1ull));
      S.idx[pos] = i;
      S.wt[pos] = wi;
      if (inv) inv[i] = pos;
    }
    base += tot;
    __syncthreads();
  }
  return base;
}

// Member embeddings: staged in LDS when n <= ECDA_NZ, read from global otherwise.  The two
// cases are separate instantiations so that every access has a known address space (a
// run-time LDS-or-global select compiles to flat loads with full waits).
template <bool STAGED>
struct EcdaRows {
  const float* emb_c;
  const float* emb_s;
  EcdaSmem& S;
  int ns;
  __device__ __forceinline__ const float* row(int a) const {
    if constexpr (STAGED) return &S.z[a * DAD_H];
    else return (a < ns ? emb_c : emb_s) + (size_t)S.idx[a] * DAD_H;
  }
};

// staging from global rows (no prefetch: batches above ECDA_PRE rows)
__device__ __forceinline__ void ecda_stage_global(EcdaSmem& S, const float* emb_c, const float* emb_s, int ns, int n) {
#pragma unroll 4
  for (int k = threadIdx.x; k < n * (DAD_H / 4); k += ECDA_THREADS) {
    const int a = k / (DAD_H / 4), q = k - a * (DAD_H / 4);
    const float* src = (a < ns ? emb_c : emb_s) + (size_t)S.idx[a] * DAD_H;
    reinterpret_cast<f32x4*>(S.z)[k] = reinterpret_cast<const f32x4*>(src)[q];
  }
  __syncthreads();
}

// upper-triangle index t of an m x m matrix (row-major, diagonal included) -> (i, j), i <= j
__device__ __forceinline__ void ecda_tri(int t, int m, int& i, int& j) {
  const float b = 2.0f * (float)m + 1.0f;
  int r = (int)((b - sqrtf(fmaxf(b * b - 8.0f * (float)t, 0.0f))) * 0.5f);
  r = r < 0 ? 0 : (r >= m ? m - 1 : r);
  while (r > 0 && r * m - r * (r - 1) / 2 > t) --r;               // float rounding fix-ups
  while (r + 1 < m && (r + 1) * m - (r + 1) * r / 2 <= t) ++r;
  i = r;
  j = t - (r * m - r * (r - 1) / 2) + r;
}

// recursive-halving reduce-scatter of 16 per-lane values over KS adjacent slice lanes (KS <= 16):
// afterwards lane sl holds in v[0 .. 16/KS) the slice sums of values [base, base + 16/KS),
// base returned.  Every value is summed by the same tree over the slices (up to operand order
// of each add, which is commutative), so equal inputs give bit-equal sums in any lane.
template <int O, int M>
__device__ __forceinline__ void ecda_rs_level(float (&v)[16], int sl, int& base) {
  if constexpr (O > 0) {
    constexpr int HALF = M / 2;
    const bool up = (sl & O) != 0;
#pragma unroll
    for (int t = 0; t < HALF; ++t) {
      const float send = up ? v[t] : v[HALF + t];
      const float keep = up ? v[HALF + t] : v[t];
      v[t] = keep + __shfl_xor(send, O, 64);
    }
    base += up ? HALF : 0;
    ecda_rs_level<O / 2, HALF>(v, sl, base);
  }
}
template <int KS>
__device__ __forceinline__ int ecda_reduce_scatter(float (&v)[16], int sl) {
  int base = 0;
  ecda_rs_level<KS / 2, 16>(v, sl, base);
  return base;
}

// mmd = t_ss + t_tt - 2 t_st of _gaussian_kernel (I/utils.py:521-563) over members
// [0, ns) (clean embeddings) and [ns, n) (strong embeddings).  Leaves the symmetric
// coefficient matrix Csym = dmmd/dD + (dmmd/dD)^T in D, so that
// dmmd/dz_i = 2 sum_j Csym_ij (z_i - z_j).  Returns mmd (valid in all threads).
template <class RW>
__device__ __forceinline__ float ecda_mmd_coef(EcdaSmem& S, const RW& R, int n, float* D) {
  const int tid = threadIdx.x;
  const int ns = R.ns;
  // pairwise squared distances (I/utils.py:533-537), register-tiled over the upper triangle:
  // a work item is a 4x4 block (bi <= bj) of member pairs over one slice of the 256 hidden
  // units.  Per float4 step a lane loads 8 rows' values and does 16 pairs' differences.  The
  // slices per block (ks, a power of two) are chosen for the least per-SIMD time given the
  // round-robin wave placement; the slice lanes of a block are adjacent and combined by a
  // fixed butterfly.  Each block writes D[i][j] and D[j][i] from one value, and a diagonal
  // block computes (p, r) and (r, p) from exactly negated differences, so D is symmetric.
  const int nb = (n + 3) >> 2, nblk = nb * (nb + 1) / 2;
  // slices per block: least per-SIMD time, in units of 1/32 float4 step (a step: 8 row loads
  // and 64 packed VALU ops per lane; a reduce-scatter shuffle ~1/32 of that; 1/2 step setup)
  int lks = 0, best = 1 << 30;
  for (int l = 0; l <= 4; ++l) {
    const int waves = ((nblk << l) + 63) >> 6;
    const int cost = ((waves + 3) >> 2) * (((DAD_H / 4) >> l) * 32 + (16 - (16 >> l)) + 16);
    if (cost < best) { best = cost; lks = l; }
  }
  const int ks = 1 << lks, qs = (DAD_H / 4) >> lks;   // slices per block, float4 steps per slice
  const int nitem = nblk << lks;
  double part = 0.0;
  for (int it0 = 0; it0 < nitem; it0 += ECDA_THREADS) {   // uniform trip count: every lane shuffles
    const int item = it0 + tid;
    const bool on = item < nitem;
    const int sl = item & (ks - 1);
    int bi = 0, bj = 0;
    if (on) ecda_tri(item >> lks, nb, bi, bj);
    ECDA_STAMP(20);
    // packed accumulators: (sum over even dims, sum over odd dims) of each pair, so the
    // squares accumulate by v_pk_fma_f32 (half the VALU issues of scalar FMAs)
    f32x2 acc2[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc2[p][q] = f32x2{0.0f, 0.0f};
    if (on) {
      const f32x4* zi[4];
      const f32x4* zj[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        zi[p] = reinterpret_cast<const f32x4*>(R.row(min(4 * bi + p, n - 1))) + sl * qs;
        zj[p] = reinterpret_cast<const f32x4*>(R.row(min(4 * bj + p, n - 1))) + sl * qs;
      }
      const int rot = bi + bj + sl;   // spreads the lanes of a wave over the banks
      for (int q = 0; q < qs; ++q) {
        const int qq = (q + rot) & (qs - 1);
        f32x4 xi[4], xj[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          xi[p] = zi[p][qq];
          xj[p] = zj[p][qq];
        }
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const f32x4 df = xi[p] - xj[r];
            const f32x2 lo = f32x2{df[0], df[1]}, hi = f32x2{df[2], df[3]};
            acc2[p][r] = __builtin_elementwise_fma(lo, lo, acc2[p][r]);
            acc2[p][r] = __builtin_elementwise_fma(hi, hi, acc2[p][r]);
          }
      }
    }
    float v[16];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * p + r] = acc2[p][r][0] + acc2[p][r][1];
    DAD_PROBE_FENCE2(v[0], v[15]);
    ECDA_STAMP(21);
    // combine the slices: lane sl ends with pairs [base, base + 16/ks) of the block
    int base = 0;
    switch (lks) {
      case 0: break;
      case 1: base = ecda_reduce_scatter<2>(v, sl); break;
      case 2: base = ecda_reduce_scatter<4>(v, sl); break;
      case 3: base = ecda_reduce_scatter<8>(v, sl); break;
      default: base = ecda_reduce_scatter<16>(v, sl); break;
    }
    DAD_PROBE_FENCE2(v[0], v[1]);
    ECDA_STAMP(22);
    if (on) {
      const int m = 16 >> lks;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        if (t >= m) break;
        const int k = base + t, p = k >> 2, r = k & 3;
        const int i = 4 * bi + p, j = 4 * bj + r;
        if (i < n && j < n && (bi < bj || p <= r)) {
          const float d = i == j ? 0.0f : v[t];
          D[i * n + j] = d;
          D[j * n + i] = d;
          part += i == j ? 0.0 : 2.0 * (double)d;
        }
      }
    }
  }
  ECDA_STAMP(12);
  double sd[1] = {part};
  ecda_block_sum_d<1>(S, sd);
  ECDA_STAMP(13);
  // detached bandwidth (I/utils.py:540-544): sum(D)/(n^2-n) / mul^(num//2), x mul^i
  float bw = (n > 1) ? (float)(sd[0] / (double)(n * n - n)) : 1.0f;
  bw = bw / 4.0f;
  float ibw[5];   // reciprocals: one division per bandwidth instead of ten per pair
#pragma unroll
  for (int m = 0; m < 5; ++m) ibw[m] = 1.0f / (bw * (float)(1 << m) + 1e-8f);
  // weight normalisers (I/utils.py:552-557)
  double wsum_t = 0.0;
  {
    int a = ns;
    for (; a + 8 <= n; a += 8) {   // eight weights per LDS round trip, summed in index order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = S.wt[a + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) wsum_t += v[u];
    }
    for (; a < n; ++a) wsum_t += S.wt[a];
  }
  const float Wss = (float)ns * (float)ns + 1e-8f;
  const float Wtt = (float)(wsum_t * wsum_t) + 1e-8f;
  const float Wst = (float)((double)ns * wsum_t) + 1e-8f;
  // terms and the symmetric coefficients Csym_ij = C_ij + C_ji, C = dmmd/dK * dK/dD, one
  // unordered pair per work item (K and dK computed once for (i, j) and (j, i))
  double t3[3] = {0.0, 0.0, 0.0};   // t_ss, t_tt, t_st numerators
  const int npair = n * (n + 1) / 2;
  for (int t = tid; t < npair; t += ECDA_THREADS) {
    int i, j;
    ecda_tri(t, n, i, j);
    const float d = D[i * n + j];
    float K = 0.0f, dK = 0.0f;
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const float e = __expf(-d * ibw[m]);
      K += e;
      dK -= e * ibw[m];
    }
    const double mult = i == j ? 1.0 : 2.0;   // (i, j) and (j, i) of the sums
    float cs;
    if (j < ns) {                               // both clean
      t3[0] += mult * (double)K;
      cs = (i == j ? 1.0f : 2.0f) / Wss;
    } else if (i >= ns) {                       // both noisy
      const float ww = S.wt[i] * S.wt[j];
      t3[1] += mult * ((double)K * ww);
      cs = (i == j ? 1.0f : 2.0f) * ww / Wtt;
    } else {                                    // (i, j) in S x T; (j, i) in T x S is unused by t_st
      t3[2] += (double)K * S.wt[j];
      cs = -2.0f * S.wt[j] / Wst;
    }
    const float v = cs * dK;
    D[i * n + j] = v;
    D[j * n + i] = v;
  }
  ECDA_STAMP(14);
  ecda_block_sum_d<3>(S, t3);   // its barriers also publish D
  const float mmd = (float)(t3[0] / Wss + t3[1] / Wtt - 2.0 * (t3[2] / Wst));
  ECDA_STAMP(15);
  return mmd;
}

// Embedding grads of the members into the ECDA part of dL/de (plain stores; a row belongs to
// at most one class), register-tiled: a work item is 4 members x 4 hidden units (one float4
// column chunk), so each member row chunk read from LDS serves 4 members' sums:
//   g = mmd_scale * 2 sum_j Csym_ij (z_i - z_j)            (all members, if D)
//     + comp_scale * (z_i - mu_c) + repg                     (noisy members)
// comp_part accumulates sum ||z_i - mu_c||^2 over noisy members (when cent).
template <class RW>
__device__ __forceinline__ void ecda_member_grads(EcdaSmem& S, const RW& R, int n, const float* D,
                                                  float mmd_scale, const float* cent, float comp_scale,
                                                  const float* repg, float* ge_c, float* ge_s, uint32_t* eflag,
                                                  int B_, float& comp_part) {
  const int ns = R.ns;
  const int nb = (n + 3) >> 2;
  for (int item = threadIdx.x; item < nb * (DAD_H / 4); item += ECDA_THREADS) {
    const int ib = item / (DAD_H / 4), hq = item - ib * (DAD_H / 4);
    int m[4];
    f32x4 zi[4], acc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      m[p] = min(4 * ib + p, n - 1);
      zi[p] = reinterpret_cast<const f32x4*>(R.row(m[p]))[hq];
      acc[p] = f32x4{};
    }
    if (D) {
      // four members j per round: every LDS read of the round issued before its FMAs
      int j = 0;
      for (; j + 4 <= n; j += 4) {
        f32x4 zj[4];
        float cj[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          zj[u] = reinterpret_cast<const f32x4*>(R.row(j + u))[hq];
#pragma unroll
          for (int p = 0; p < 4; ++p) cj[u][p] = D[(j + u) * n + m[p]];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int p = 0; p < 4; ++p)   // Csym[j][i] = Csym[i][j]; packed sub + packed FMA
            acc[p] = __builtin_elementwise_fma(f32x4{cj[u][p], cj[u][p], cj[u][p], cj[u][p]}, zi[p] - zj[u], acc[p]);
      }
      for (; j < n; ++j) {
        const f32x4 zj = reinterpret_cast<const f32x4*>(R.row(j))[hq];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float cji = D[j * n + m[p]];
          acc[p] = __builtin_elementwise_fma(f32x4{cji, cji, cji, cji}, zi[p] - zj, acc[p]);
        }
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int mm = 4 * ib + p;
      if (mm >= n) break;
      f32x4 g = D ? mmd_scale * (2.0f * acc[p]) : f32x4{};
      if (mm >= ns) {
        if (cent) {
          const f32x4 df = zi[p] - reinterpret_cast<const f32x4*>(cent)[hq];
          comp_part += ((df[0] * df[0] + df[1] * df[1]) + df[2] * df[2]) + df[3] * df[3];
          g += comp_scale * df;
        }
        g += reinterpret_cast<const f32x4*>(repg)[hq];
      }
      reinterpret_cast<f32x4*>((mm < ns ? ge_c : ge_s) + (size_t)S.idx[mm] * DAD_H)[hq] = g;
      if (hq == 0) eflag[mm < ns ? S.idx[mm] : B_ + S.idx[mm]] = 1u;
    }
  }
}

// DACP state and thresholds of the fused prefix (dad_tail_ecda's ECDA blocks)
struct EcdaPrefix {
  float dstate[20];
  int ncls[DAD_C];
  float tau_new[DAD_C];
  float wc[DAD_C];
  float fred[16];
};

// One class of ECDA.  FUSED: the DACP mask, scores and class weights are derived here from
// the teacher logits by the same code as the tail block (teacher_certainty, dacp_thresholds),
// instead of being read back from the tail's outputs.
// Batches of at most ECDA_PRE rows per side load every embedding row into registers at entry
// (wave g holds rows g, g + 8, ... of column chunk lane), in flight during the metadata phase;
// the centroid pass and the member staging then need no global round trip.
template <bool FUSED>
__device__ __forceinline__ void ecda_block(const DadEcdaArgs& a, const int c, EcdaSmem& S, float (&pdist)[DAD_C][DAD_C],
                                           const DadTailArgs* ta, EcdaPrefix& P) {
  const dad_config& cfg = a.cfg;
  const int B = cfg.B, Bn = cfg.Bn;
  const int tid = threadIdx.x;
  const int g = tid >> 6, lq = tid & 63;
  const float* tf = a.tailf;
  ECDA_STAMP(0);
  const float* emb_c = a.emb;
  const float* emb_s = a.emb + (size_t)(B + Bn) * DAD_H;
  float* ge_c = a.ge;
  float* ge_s = a.ge + (size_t)B * DAD_H;
  float* scratch = a.scratch + (size_t)c * (B + Bn) * (B + Bn);
  const float wscale = cfg.w_ecda;
  float ecda_on;
  const float* w;   // DACP class weights
  const bool pre = B <= ECDA_PRE && Bn <= ECDA_PRE;
  f32x4 pc[ECDA_PRE_U], ps[ECDA_PRE_U];
  if (FUSED) {
    // teacher logits first: the DACP prefix waits on them
    f32x4 zt = f32x4{};
    const float* z1 = ta->logits + (size_t)B * DAD_C;
    if (tid < Bn) zt = reinterpret_cast<const f32x4*>(z1)[tid];
    if (tid >= ECDA_THREADS - 20) P.dstate[tid - (ECDA_THREADS - 20)] = ta->dacp[tid - (ECDA_THREADS - 20)];
    for (int b = tid; b < B; b += ECDA_THREADS) S.lab[b] = (int)a.yc[b];
    if (pre) {
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u) {
        const int b = g + ECDA_NG * u;
        pc[u] = b < B ? reinterpret_cast<const f32x4*>(emb_c + (size_t)b * DAD_H)[lq] : f32x4{};
        ps[u] = b < Bn ? reinterpret_cast<const f32x4*>(emb_s + (size_t)b * DAD_H)[lq] : f32x4{};
      }
    }
    for (int b = tid; b < Bn; b += ECDA_THREADS) {
      float z[4], q[4], sc;
      int pred;
      if (b == tid) { z[0] = zt[0]; z[1] = zt[1]; z[2] = zt[2]; z[3] = zt[3]; }
      else for (int k = 0; k < 4; ++k) z[k] = z1[b * 4 + k];
      teacher_certainty(z, cfg, q, sc, pred);
      S.scr[b] = sc;
      S.prd[b] = pred;
    }
    if (tid < DAD_C) { P.ncls[tid] = 0; S.cnt_clean[tid] = 0; S.cnt_noisy[tid] = 0; }
    __syncthreads();
    // masked-out noisy samples get pseudo-label -1 (noisy_mask>thr re-cast: I/utils.py:573-576)
    if (cfg.use_dacp) {
      dacp_thresholds(cfg, Bn, S.scr, S.prd, reinterpret_cast<float(*)[DAD_MAX_BATCH]>(S.z), P.ncls, P.dstate,
                      P.tau_new, P.wc, nullptr, nullptr);
      for (int b = tid; b < Bn; b += ECDA_THREADS) S.prd[b] = S.scr[b] >= P.tau_new[S.prd[b]] ? S.prd[b] : -1;
    } else {
      for (int b = tid; b < Bn; b += ECDA_THREADS) S.prd[b] = S.scr[b] >= cfg.fixed_thr ? S.prd[b] : -1;
      if (tid < DAD_C) P.wc[tid] = 1.0f;
    }
    float mpart = 0.0f;
    for (int b = tid; b < Bn; b += ECDA_THREADS) mpart += S.prd[b] >= 0 ? 1.0f : 0.0f;
    const float msum = block_sum_f(mpart, P.fred);   // the tail's mask sum (exact: a count)
    ecda_on = (msum > 1.0f && cfg.ecda_on) ? 1.0f : 0.0f;   // I/train.py:444
    w = P.wc;
  } else {
    ecda_on = tf[DAD_T_ECDA_ON];   // branched on after the metadata loads are issued
    w = tf + DAD_T_W;
    const float* score = tf + DAD_TAIL_HDR;
    const float* predf = tf + DAD_TAIL_HDR + Bn;
    const float* mask = tf + DAD_TAIL_HDR + 2 * Bn;
    // stage per-sample metadata (masked-out noisy samples get pseudo-label -1)
    for (int b = tid; b < B; b += ECDA_THREADS) S.lab[b] = (int)a.yc[b];
    for (int b = tid; b < Bn; b += ECDA_THREADS) {
      S.prd[b] = mask[b] > 0.0f ? (int)predf[b] : -1;   // noisy_mask>thr re-cast: I/utils.py:573-576
      S.scr[b] = score[b];
    }
    if (pre) {
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u) {
        const int b = g + ECDA_NG * u;
        pc[u] = b < B ? reinterpret_cast<const f32x4*>(emb_c + (size_t)b * DAD_H)[lq] : f32x4{};
        ps[u] = b < Bn ? reinterpret_cast<const f32x4*>(emb_s + (size_t)b * DAD_H)[lq] : f32x4{};
      }
    }
    if (tid < DAD_C) { S.cnt_clean[tid] = 0; S.cnt_noisy[tid] = 0; }
  }
  __syncthreads();
  ECDA_STAMP(1);
  if (ecda_on == 0.0f) return;   // no row flagged: the ECDA part of dL/de is zero

  // member rows into S.z at their compacted positions: from the registers (prefetch), or
  // from global rows through S.idx
  auto stage = [&](int ns, int n) {
    ECDA_STAMP(19);
    if (pre) {
      // every position read before the first store (one LDS round trip); -1: not a member
      int pcl[ECDA_PRE_U], pno[ECDA_PRE_U];
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u) {
        const int b = g + ECDA_NG * u;   // < ECDA_PRE: S.pos rows past B / Bn stay -1
        pcl[u] = S.pos[b];
        pno[u] = S.pos[ECDA_PRE + b];
      }
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u) {
        if (pcl[u] >= 0) reinterpret_cast<f32x4*>(&S.z[pcl[u] * DAD_H])[lq] = pc[u];
        if (pno[u] >= 0) reinterpret_cast<f32x4*>(&S.z[pno[u] * DAD_H])[lq] = ps[u];
      }
      __syncthreads();
    } else {
      ecda_stage_global(S, emb_c, emb_s, ns, n);
    }
  };
  int* inv = pre ? S.pos : nullptr;

  if (!cfg.class_aware) {
    // global MMD ablation: all clean vs all masked noisy, unit weights (I/utils.py:633-650)
    if (c != 0) return;
    if (tid < DAD_H) S.repg[tid] = 0.0f;   // no repulsion term (read after the compaction's barriers)
    if (pre && tid < 2 * ECDA_PRE) S.pos[tid] = -1;
    int n = ecda_compact(S, B, 0, [](int) { return true; }, [](int) { return 1.0f; }, inv);
    const int ns = n;
    n = ecda_compact(S, Bn, n, [&](int i) { return S.prd[i] >= 0; }, [](int) { return 1.0f; },
                     inv ? inv + ECDA_PRE : nullptr);
    const int nt = n - ns;
    if (ns >= 2 && nt >= 2) {
      auto run = [&](auto staged_tag) {
        constexpr bool ST = decltype(staged_tag)::value;
        const EcdaRows<ST> R{emb_c, emb_s, S, ns};
        float* D = ST ? S.dm : scratch;
        if constexpr (ST) stage(ns, n);
        const float mmd = ecda_mmd_coef(S, R, n, D);
        float unused = 0.0f;
        ecda_member_grads(S, R, n, D, wscale, nullptr, 0.0f, S.repg, ge_c, ge_s, a.eflag, B, unused);
        if (tid == 0) { a.tail_terms[0] = mmd; a.tail_terms[DAD_T_ECDA_GATE - DAD_T_ECDA_TERM] = 1.0f; }
      };
      if (n <= ECDA_NZ) run(std::true_type{});
      else run(std::false_type{});
    }
    return;
  }

  // class-aware path.  In fixed-threshold mode class_weights_wce = ones(Bn) (I/train.py:420)
  // so the loop runs over range(Bn): only classes < min(Bn, C) can have members.
  const int ncls = cfg.use_dacp ? DAD_C : (Bn < DAD_C ? Bn : DAD_C);
  if (c >= ncls) return;
  for (int b = tid; b < B; b += ECDA_THREADS)
    if (S.lab[b] >= 0 && S.lab[b] < ncls) atomicAdd(&S.cnt_clean[S.lab[b]], 1);
  for (int b = tid; b < Bn; b += ECDA_THREADS)
    if (S.prd[b] >= 0 && S.prd[b] < ncls) atomicAdd(&S.cnt_noisy[S.prd[b]], 1);
  if (pre && tid < 2 * ECDA_PRE) S.pos[tid] = -1;
  ECDA_STAMP(16);
  // noisy centroids of every class (needed for the repulsion term): row group g (one wave) x
  // 64 float4 columns, partials combined in fixed group order
  {
    float* part = S.z;   // [NG groups][C][H], before the members are staged
    static_assert(ECDA_NG * DAD_C * DAD_H <= ECDA_NZ * DAD_H, "centroid partials must fit in S.z");
    f32x4 cs[DAD_C];
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) cs[k] = f32x4{};
    if (pre) {
      int pk[ECDA_PRE_U];
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u) {   // all pseudo-labels first (one LDS round trip)
        const int b = g + ECDA_NG * u;
        pk[u] = S.prd[b < Bn ? b : 0];
        pk[u] = b < Bn ? pk[u] : -1;
      }
#pragma unroll
      for (int u = 0; u < ECDA_PRE_U; ++u)
#pragma unroll
        for (int k = 0; k < DAD_C; ++k) cs[k] += pk[u] == k ? ps[u] : f32x4{};
    } else {
#pragma unroll 4
      for (int b = g; b < Bn; b += ECDA_NG) {
        const int pk = S.prd[b];
        const f32x4 e = reinterpret_cast<const f32x4*>(emb_s + (size_t)b * DAD_H)[lq];
#pragma unroll
        for (int k = 0; k < DAD_C; ++k) cs[k] += pk == k ? e : f32x4{};
      }
    }
    ECDA_STAMP(17);
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) reinterpret_cast<f32x4*>(part + (g * DAD_C + k) * DAD_H)[lq] = cs[k];
    __syncthreads();
    ECDA_STAMP(18);
    for (int e = tid; e < DAD_C * DAD_H; e += ECDA_THREADS) {
      const int k = e / DAD_H, hh = e & (DAD_H - 1);
      float sk = 0.0f;
#pragma unroll
      for (int gg = 0; gg < ECDA_NG; ++gg) sk += part[(gg * DAD_C + k) * DAD_H + hh];
      S.cent[k][hh] = S.cnt_noisy[k] > 0 ? sk / (float)S.cnt_noisy[k] : 0.0f;
    }
  }
  __syncthreads();
  ECDA_STAMP(2);
  // per-class counts into registers (one LDS round trip for all of them)
  int cn[DAD_C], cc[DAD_C];
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) { cn[k] = S.cnt_noisy[k]; cc[k] = S.cnt_clean[k]; }
  // class attention (I/utils.py:597-599)
  float att[DAD_C];
  if (cfg.use_dacp) {
    float wk[DAD_C];
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) wk[k] = w[k];
    const float wmean = (((wk[0] + wk[1]) + wk[2]) + wk[3]) / 4.0f;
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) att[k] = expf(cfg.ecda_att_lambda * (wmean - wk[k]));
  } else {
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) att[k] = 1.0f;
  }
  const float att_c = att[c];
  // repulsion over valid centroids (I/utils.py:582-595)
  int nvalid = 0;
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) nvalid += (k < ncls && cn[k] > 0) ? 1 : 0;
  const int npairs = nvalid * (nvalid - 1) / 2;
  {
    // 16 (p, q) pairs x 256 dims over all threads: 32 threads per pair, 8 dims each,
    // combined by a 32-lane reduction (pair-symmetric order, so pdist stays symmetric)
    const int pair = tid / 32, l32 = tid & 31;
    float d = 0.0f;
    if (pair < DAD_C * DAD_C) {
      const int p = pair / DAD_C, q = pair % DAD_C;
      const int lo = p < q ? p : q, hi = p < q ? q : p;
      if (p < ncls && q < ncls && S.cnt_noisy[p] > 0 && S.cnt_noisy[q] > 0 && p != q) {
        const f32x4* a0 = reinterpret_cast<const f32x4*>(&S.cent[lo][l32 * (DAD_H / 32)]);
        const f32x4* a1 = reinterpret_cast<const f32x4*>(&S.cent[hi][l32 * (DAD_H / 32)]);
        const f32x4 x0 = a0[0], x1 = a0[1], y0 = a1[0], y1 = a1[1];
        const float v[8] = {x0[0] - y0[0], x0[1] - y0[1], x0[2] - y0[2], x0[3] - y0[3],
                            x1[0] - y1[0], x1[1] - y1[1], x1[2] - y1[2], x1[3] - y1[3]};
#pragma unroll
        for (int k = 0; k < 8; ++k) d += v[k] * v[k];
      }
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 32);
    if (pair < DAD_C * DAD_C && l32 == 0) pdist[pair / DAD_C][pair % DAD_C] = sqrtf(d);
  }
  __syncthreads();
  ECDA_STAMP(4);
  float pd[DAD_C][DAD_C];
#pragma unroll
  for (int p = 0; p < DAD_C; ++p)
#pragma unroll
    for (int q = 0; q < DAD_C; ++q) pd[p][q] = pdist[p][q];
  float rep = 0.0f;
  if (nvalid > 1) {
    float sp = 0.0f;
#pragma unroll
    for (int p = 0; p < DAD_C; ++p)
#pragma unroll
      for (int q = p + 1; q < DAD_C; ++q)
        if (q < ncls && cn[p] > 0 && cn[q] > 0) sp += pd[p][q];
    rep = -sp / (float)npairs;
  }
  bool gated[DAD_C];
  float rep_coef = 0.0f;
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) {
    gated[k] = k < ncls && cc[k] >= 2 && cn[k] >= 2;   // I/utils.py:609-610
    if (gated[k]) rep_coef += att[k] * cfg.ecda_delta;
  }
  // repulsion grad of this class's noisy members (d rep / d mu_c, then 1/n_c per member)
  const bool rep_on = nvalid > 1 && cn[c] > 0 && rep_coef != 0.0f;
  if (tid < DAD_H) {
    const int hh = tid;
    float rep_g = 0.0f;
    if (rep_on) {
      float ce[DAD_C];
#pragma unroll
      for (int q = 0; q < DAD_C; ++q) ce[q] = S.cent[q][hh];
      float gsum = 0.0f;
#pragma unroll
      for (int q = 0; q < DAD_C; ++q) {
        if (q == c || q >= ncls || cn[q] == 0) continue;
        const float nd = pd[c][q];
        if (nd > 0.0f) gsum += (ce[c] - ce[q]) / nd;
      }
      rep_g = wscale * rep_coef * (-gsum / (float)npairs / (float)cn[c]);
    }
    S.repg[hh] = rep_g;   // read after the member compaction's barriers
  }
  if (!gated[c] && !rep_on) return;
  ECDA_STAMP(3);
  // members of class c: clean (label c, weight 1) then masked noisy (pseudo-label c, weight = score);
  // a class below the gate only needs its noisy members (repulsion)
  int n = gated[c] ? ecda_compact(S, B, 0, [&](int i) { return S.lab[i] == c; }, [](int) { return 1.0f; }, inv) : 0;
  ECDA_STAMP(5);
  const int ns = n;
  n = ecda_compact(S, Bn, n, [&](int i) { return S.prd[i] == c; }, [&](int i) { return S.scr[i]; },
                   inv ? inv + ECDA_PRE : nullptr);
  const int nt = n - ns;
  float mmd = 0.0f;
  float cpart = 0.0f;
  auto run = [&](auto R, float* Dbuf) {
    constexpr bool ST = std::is_same_v<decltype(R), EcdaRows<true>>;
    float* D = nullptr;
    if (gated[c]) {
      D = Dbuf;
      if constexpr (ST) stage(ns, n);
      ECDA_STAMP(6);
      mmd = ecda_mmd_coef(S, R, n, D);
      ECDA_STAMP(7);
    }   // (a repulsion-only class needs no member rows: g = repg)
    // compactness (I/utils.py:614-616): mean_j ||z_j - mu||^2, grad (2/nt)(z_j - mu)
    ecda_member_grads(S, R, n, D, wscale * att_c, gated[c] ? S.cent[c] : nullptr,
                      wscale * att_c * cfg.ecda_gamma * (2.0f / (float)nt), S.repg, ge_c, ge_s, a.eflag, B, cpart);
  };
  if (n <= ECDA_NZ) run(EcdaRows<true>{emb_c, emb_s, S, ns}, S.dm);
  else run(EcdaRows<false>{emb_c, emb_s, S, ns}, scratch);
  if (!gated[c]) return;
  ECDA_STAMP(8);
  const float comp = ecda_block_sum_f(S, cpart) / (float)nt;
  if (tid == 0) {
    a.tail_terms[c] = att_c * (mmd + cfg.ecda_gamma * comp + cfg.ecda_delta * rep);
    ECDA_STAMP_SIZES(c, n, ns);
    a.tail_terms[DAD_T_ECDA_GATE - DAD_T_ECDA_TERM + c] = 1.0f;
  }
}

__global__ __launch_bounds__(ECDA_THREADS) void dad_ecda(DadEcdaArgs a) {
  DAD_GUARD_BLOCK(ECDA_THREADS);
  __shared__ struct { EcdaSmem s; float pdist[DAD_C][DAD_C]; EcdaPrefix p; } u;
  ecda_block<false>(a, blockIdx.x, u.s, u.pdist, nullptr, u.p);
}

// block 0: the tail (losses, DACP outputs, dL/dz); blocks 1..C: ECDA class blockIdx.x - 1,
// which re-derives the DACP mask itself and so does not wait for block 0.  The two roles
// write disjoint outputs (dad_pool zeroed the ECDA flags and terms).  LDS: one union.
static_assert(DAD_TAIL_THREADS == DAD_ECDA_THREADS, "dad_tail_ecda: one block size for both roles");
__global__ __launch_bounds__(TAIL_THREADS) void dad_tail_ecda(DadTailArgs ta, DadEcdaArgs ca) {
  DAD_GUARD_BLOCK(TAIL_THREADS);
  __shared__ union U {
    TailSmem t;
    struct E { EcdaSmem s; float pdist[DAD_C][DAD_C]; EcdaPrefix p; } e;
  } u;
  if (blockIdx.x == 0) tail_block(ta, u.t);
  else {
    ecda_block<true>(ca, (int)blockIdx.x - 1, u.e.s, u.e.pdist, &ta, u.e.p);
  }
}

// =====================================================================================
// Wave-centric tail + ECDA for batches of at most 64 utterances per side (the bench
// geometry): dad_tail_ecda_w.  Same outputs as dad_tail_ecda, far fewer barrier-separated
// phases:
//  * DACP (I/utils.py:449-507) inside ONE wave: lane i = noisy row i; ranks by an LDS
//    broadcast sweep, the per-class quantile by lanes 0..3, thresholds broadcast by readlane
//    (dacp_wave; the arithmetic of dacp_thresholds, so the masks are bit-identical).  Every
//    wave of an ECDA block derives the mask itself: no barrier before the class work.
//  * the tail block: CE in wave 0 (lane = clean row), teacher certainty + DACP + KL in wave 1
//    (lane = noisy row), wave reductions by DPP, one barrier to combine.
//  * an ECDA class block stages its CANDIDATE rows (clean label c, noisy pseudo-label c: known
//    before the mask) from the registers they were prefetched into; the pairwise distances
//    come from a Gram matrix on the fp32 matrix cores (v_mfma_f32_32x32x2_f32, K split over
//    the 8 waves), D_ij = |z_i|^2 + |z_j|^2 - 2 z_i.z_j; the member gradients
//    2 sum_j C_ij (z_i - z_j) = 2 (rowsum(C)_i z_i - (C Z)_i) are a second MFMA GEMM.
//    Four workgroup barriers in all.  A class with more than 64 candidates falls back to
//    ecda_block (the general path) inside the same launch.
// =====================================================================================
#define TW_MAXB 64
// Pitches (floats) of the staged rows and the coefficient matrix: multiples of 4 (16-B rows) with
// pitch/4 odd, so the MFMA operand reads -- one ds_read_b128 of 4 consecutive k per lane, the
// 32 lanes of a half on 32 different rows -- fall on 16 different 16-B bank slots per lane group
// (conflict-free; scalar reads of one column over rows at pitch 260 were 4-way conflicts)
#define EW_ZP 260          // staged row pitch
#define EW_CP 68           // coefficient matrix pitch (narrow)
#define EW_CPW 132         // coefficient matrix pitch (wide, 128 candidates)
#define EW_GP 33           // Gram tile row pitch: the distance pass reads tiles transposed too

// DACP scratch of a workgroup: per-wave partial ranks and per-wave sorted-score tables
struct DacpBlockScratch {
  int rk[ECDA_THREADS / 64][TW_MAXB];   // [wave][row]: each wave's store is 64 consecutive ints
  float srt[ECDA_THREADS / 64][DAD_C][TW_MAXB];
};

// The DACP state a wave reads (uniform): tau, Q and the calibrated anchors.  Loaded by ONE
// unconditional load per lane (lane k < 20 holds dacp[k]) issued with the kernel's other entry
// loads, then broadcast by readlane: a load under a lane condition would be waited for on the
// spot (the compiler drains vmcnt where the paths merge), one memory round trip per value.
__device__ __forceinline__ float sel4(const float (&v)[DAD_C], int k) {
  return k == 0 ? v[0] : (k == 1 ? v[1] : (k == 2 ? v[2] : v[3]));
}
__device__ __forceinline__ int sel4i(const int (&v)[DAD_C], int k) {
  return k == 0 ? v[0] : (k == 1 ? v[1] : (k == 2 ? v[2] : v[3]));
}

struct DacpState {
  float tau[DAD_C], Q[DAD_C], anc[DAD_C];
};

// segmented sums by DPP (no LDS-routed shuffles): the sum of each aligned group of N lanes lands
// in the group's LAST lane (N = 4, 8, 16 inside a 16-lane row; 32 adds row_bcast:15)
template <int N>
__device__ __forceinline__ float dpp_seg_sum(float v) {
  static_assert(N == 4 || N == 8 || N == 16 || N == 32, "segment");
  v += dad_dpp_f<0x111>(v);
  v += dad_dpp_f<0x112>(v);
  if constexpr (N >= 8) v += dad_dpp_f<0x114>(v);
  if constexpr (N >= 16) v += dad_dpp_f<0x118>(v);
  if constexpr (N == 32) v += dad_dpp_f<0x142, 0xa>(v);
  return v;
}
__device__ __forceinline__ DacpState dacp_state_of(float dv) {
  DacpState d;
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) {
    d.tau[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), k));
    d.Q[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), 4 + k));
    d.anc[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dv), 16 + k));
  }
  return d;
}

// DACP thresholds (I/utils.py:449-507) by all 8 waves of a workgroup, every wave holding the
// scores s and pseudo-labels p of every noisy row (lane i = row i < Bn; p = -1 past Bn).  Wave g
// counts, for every row, the rows j in [8g, 8g + 8) of its class below it (ties by index:
// readlane sweep, bitwise so nothing branches); one barrier; the rank is the sum of the 8
// partials.  Then every wave sorts into its own table and lanes 0..3 take torch.quantile(linear)
// of their class; outputs uniform.  The arithmetic is dacp_thresholds', so the thresholds and
// masks are bit-identical to the general path's.
__device__ __forceinline__ void dacp_block8(const dad_config& cfg, int Bn, float s, int p, const DacpState& D,
                                            DacpBlockScratch& W, float (&tau)[DAD_C], float (&wc)[DAD_C],
                                            float (&that)[DAD_C], float (&fl)[DAD_C]) {
  const int lane = threadIdx.x & 63;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  TAIL_STAMP_W1(7);
  int part = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int j = 8 * g + u;
    const float sj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), j));
    const int pj = __builtin_amdgcn_readlane(p, j);
    part += (int)((pj == p) & ((sj < s) | ((sj == s) & (j < lane))));
  }
  W.rk[g][lane] = part;   // ([row][wave] put 8 rows of a store on one bank: 8-way conflicts)
  __syncthreads();
  int r[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = W.rk[k][lane];
  const int cnt = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  TAIL_STAMP_W1(8);
  int ncls[DAD_C];
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) ncls[c] = (int)__popcll(__ballot(lane < Bn && p == c));
  float (*srt)[TW_MAXB] = W.srt[g];
  if (lane < Bn) srt[p][cnt] = s;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float tn = 0.0f, w = 0.0f, th = 0.0f, f = 0.0f;
  if (lane < DAD_C) {
    const int c = lane;
    const float q0 = D.Q[0], q1 = D.Q[1], q2 = D.Q[2], q3 = D.Q[3];
    const float qc = sel4(D.Q, c), tc = sel4(D.tau, c), ac = sel4(D.anc, c);
    const float qmean = (((q0 + q1) + q2) + q3) / 4.0f;
    w = 1.0f / (1.0f + expf(-(cfg.dacp_k * (qc - qmean))));
    const int n = sel4i(ncls, c);
    // torch.quantile(linear): rank = q*(n-1) in f32, lerp(below, above, rank-floor)
    const float rank = cfg.dacp_gamma * (float)(n - 1);
    const int lo = (int)rank;
    const int hi = (int)ceilf(rank);
    const float wgt = rank - (float)lo;
    const float vlo = srt[c][lo < 0 ? 0 : lo], vhi = srt[c][hi < 0 ? 0 : hi];
    const float q = wgt < 0.5f ? vlo + wgt * (vhi - vlo) : vhi - (vhi - vlo) * (1.0f - wgt);
    th = n > 0 ? q : tc;
    const float adj = cfg.dacp_lambda * (w - 0.5f);
    f = fmaxf(th + adj, ac);
    tn = cfg.dacp_alpha * tc + cfg.dacp_one_m_alpha * f;
  }
  DAD_PROBE_FENCE2(tn, f);
  TAIL_STAMP_W1(9);
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) {
    tau[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tn), c));
    wc[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w), c));
    that[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(th), c));
    fl[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(f), c));
  }
  DAD_PROBE_FENCE2(tau[3], fl[3]);
  TAIL_STAMP_W1(10);
}

// the DACP / fixed-threshold mask of noisy row `lane` (I/train.py:413-420), score s, pseudo-label
// p; called by all 8 waves of a workgroup (one barrier inside when DACP is on)
struct WaveMask {
  float s, q[DAD_C];
  int p;                 // pseudo-label, -1 on lanes >= Bn
  bool m;                // masked in (confident)
  float tau[DAD_C], wc[DAD_C], that[DAD_C], fl[DAD_C];
};
__device__ __forceinline__ void block_mask(const dad_config& cfg, int Bn, const f32x4& zt, const DacpState& D,
                                           DacpBlockScratch& W, WaveMask& M) {
  const int lane = threadIdx.x & 63;
  {
    const float z[4] = {zt[0], zt[1], zt[2], zt[3]};
    teacher_certainty(z, cfg, M.q, M.s, M.p);   // every lane (rows past Bn are clamped copies)
  }
  if (lane >= Bn) {
    M.s = 0.0f;
    M.p = -1;
  }
  if (cfg.use_dacp) {
    dacp_block8(cfg, Bn, M.s, M.p, D, W, M.tau, M.wc, M.that, M.fl);
    M.m = (lane < Bn) & (M.s >= sel4(M.tau, M.p < 0 ? 0 : M.p));
  } else {
#pragma unroll
    for (int c = 0; c < DAD_C; ++c) { M.tau[c] = 0.0f; M.wc[c] = 1.0f; M.that[c] = 0.0f; M.fl[c] = 0.0f; }
    M.m = (lane < Bn) & (M.s >= cfg.fixed_thr);
  }
}

struct TailW {
  DacpBlockScratch dw;
  double d[2][8];
  float f[2][4];
};

// The tail (block 0) for B, Bn <= 64: see tail_block for the reference lines of each step.
// Every wave: entry loads, teacher certainty and the DACP mask (block_mask: one barrier);
// wave 0: CE on the clean logits (lane = clean row); wave 1: DACP outputs, epoch statistics and
// the masked KL (lane = noisy row); one barrier to combine.
__device__ __forceinline__ void tail_block_w(const DadTailArgs& a, TailW& T) {
  const dad_config& cfg = a.cfg;
  const int B = cfg.B, Bn = cfg.Bn;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* tf = a.tailf;
  float* extras = a.grad + DAD_NPARAM;
  const float eps = cfg.ls_eps;
  TAIL_STAMP(0);
  TAIL_CYCLES(12);
  // entry loads, unconditional (rows clamped): clean logits + labels, teacher and strong logits,
  // the DACP state
  const int rc = lane < B ? lane : B - 1, rn = lane < Bn ? lane : Bn - 1;
  const f32x4 zv = reinterpret_cast<const f32x4*>(a.logits)[rc];
  const int yv = (int)a.yc[rc];
  const f32x4 zt = reinterpret_cast<const f32x4*>(a.logits + (size_t)B * DAD_C)[rn];
  const f32x4 zs = reinterpret_cast<const f32x4*>(a.logits + (size_t)(B + Bn) * DAD_C)[rn];
  const float dv = a.dacp[lane < DAD_DACP_FLOATS ? lane : 0];
  // teacher probs + certainty + DACP mask (I/train.py:408-420, I/utils.py:400-507), lane = noisy row
  const DacpState D = dacp_state_of(dv);
  WaveMask M;
  block_mask(cfg, Bn, zt, D, T.dw, M);
  TAIL_STAMP_W1(4);
  if (w == 0) {
    // supervised CE with label smoothing on the clean logits (I/train.py:364,400), lane = row
    double ce_part = 0.0, b2p[4] = {0.0, 0.0, 0.0, 0.0};
    {
      const int y = yv;
      const float z[4] = {zv[0], zv[1], zv[2], zv[3]};
      float m = -INFINITY;
      for (int c = 0; c < 4; ++c) m = fmaxf(m, z[c]);
      float se = 0.0f;
      for (int c = 0; c < 4; ++c) se += expf(z[c] - m);
      const float lse = m + logf(se);
      float lsum = 0.0f, g[4];
      for (int c = 0; c < 4; ++c) {
        const float ls = z[c] - lse;
        lsum += ls;
        const float pr = expf(ls);
        g[c] = (pr - (c == y ? 1.0f - eps : 0.0f) - eps * 0.25f) / (float)B;
        b2p[c] = lane < B ? (double)g[c] : 0.0;
      }
      const float zy = y == 0 ? z[0] : (y == 1 ? z[1] : (y == 2 ? z[2] : z[3]));
      ce_part = lane < B ? -(1.0 - (double)eps) * (double)(zy - lse) - (double)eps * 0.25 * (double)lsum : 0.0;
      if (lane < B) *reinterpret_cast<f32x4*>(a.gzb + (size_t)lane * DAD_C) = f32x4{g[0], g[1], g[2], g[3]};
    }
    const double ce = dad_wave_sum_d(ce_part) / (double)B;
    double b2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) b2[c] = dad_wave_sum_d(b2p[c]);
    TAIL_STAMP(2);
    if (lane == 0) {
      T.d[0][0] = ce;
#pragma unroll
      for (int c = 0; c < 4; ++c) T.d[0][1 + c] = b2[c];
    }
  } else if (w == 1) {
    if (cfg.use_dacp) {
      if (lane < DAD_C) {
        const int c = lane;
        tf[DAD_T_W + c] = sel4(M.wc, c);
        tf[DAD_T_TAU_BEFORE + c] = sel4(D.tau, c);
        tf[DAD_T_TAU_AFTER + c] = sel4(M.tau, c);
        tf[DAD_T_FLOORED + c] = sel4(M.fl, c);
        tf[DAD_T_TAU_HAT + c] = sel4(M.that, c);
        extras[c] = sel4(M.fl, c);
      }
      // epoch statistics of update_class_quality_scores_epoch (I/utils.py:503-505)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double st = dad_wave_sum_d(M.p == c ? (double)M.s : 0.0);
        const double ct = dad_wave_sum_d(M.p == c ? 1.0 : 0.0);
        if (lane == 0) {
          extras[4 + c] = (float)st;
          extras[8 + c] = (float)ct;
        }
      }
    } else if (lane < DAD_C) {
      tf[DAD_T_W + lane] = 1.0f;
      extras[0 + lane] = 0.0f;
      extras[4 + lane] = 0.0f;
      extras[8 + lane] = 0.0f;
    }
    const float mk = M.m ? 1.0f : 0.0f;
    const float msum = (float)__popcll(__ballot(M.m));   // the mask sum (an exact count)
    const bool kl_on = msum > 1.0f;                      // I/train.py:444
    // masked consistency KL(q || p_student) (I/train.py:445-447) and its logit grad
    const float denom = msum + 1e-8f;
    double kl_part = 0.0, b2p[4] = {0.0, 0.0, 0.0, 0.0};
    {
      const float z[4] = {zs[0], zs[1], zs[2], zs[3]};
      float m = -INFINITY;
      for (int c = 0; c < 4; ++c) m = fmaxf(m, z[c]);
      float se = 0.0f;
      for (int c = 0; c < 4; ++c) se += expf(z[c] - m);
      const float lse = m + logf(se);
      float klb = 0.0f, g[4];
      for (int c = 0; c < 4; ++c) {
        const float q = M.q[c];
        const float ls = z[c] - lse;
        const float t = q * (logf(q) - ls);
        klb += q > 0.0f ? t : 0.0f;
        g[c] = kl_on ? cfg.w_kl * mk * (expf(ls) - q) / denom : 0.0f;
        b2p[c] = lane < Bn ? (double)g[c] : 0.0;
      }
      kl_part = lane < Bn ? (double)(klb * mk) : 0.0;
      if (lane < Bn) {
        *reinterpret_cast<f32x4*>(a.gzb + (size_t)(B + lane) * DAD_C) = f32x4{g[0], g[1], g[2], g[3]};
        // per-sample outputs (noisy batch) for inspection / ECDA
        tf[DAD_TAIL_HDR + lane] = M.s;
        tf[DAD_TAIL_HDR + Bn + lane] = (float)M.p;
        tf[DAD_TAIL_HDR + 2 * Bn + lane] = mk;
        *reinterpret_cast<f32x4*>(tf + DAD_TAIL_HDR + 3 * Bn + lane * 4) = f32x4{M.q[0], M.q[1], M.q[2], M.q[3]};
      }
    }
    TAIL_STAMP_W1(5);
    const double kls = dad_wave_sum_d(kl_part);
    double b2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) b2[c] = dad_wave_sum_d(b2p[c]);
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) T.d[1][1 + c] = b2[c];
      T.f[1][0] = kl_on ? (float)(kls / (double)denom) : 0.0f;
      T.f[1][1] = msum;
      T.f[1][2] = kl_on ? 1.0f : 0.0f;
    }
    TAIL_STAMP_W1(6);
  }
  __syncthreads();
  if (tid == 0) {
    const float kl_on = T.f[1][2];
    tf[DAD_T_CE] = (float)T.d[0][0];
    tf[DAD_T_KL] = T.f[1][0];
    tf[DAD_T_SCL] = 0.0f;
    tf[DAD_T_MSUM] = T.f[1][1];
    tf[DAD_T_KL_ON] = kl_on;
    tf[DAD_T_ECDA_ON] = (kl_on != 0.0f && cfg.ecda_on) ? 1.0f : 0.0f;
  }
  if (tid < 4) a.grad[DAD_OFF_B2 + tid] = (float)(T.d[0][1 + tid] + T.d[1][1 + tid]);
  TAIL_CYCLES(13);
  TAIL_STAMP(1);
}

struct __attribute__((aligned(16))) EcdaW {
  union {
    float zc[(TW_MAXB + 1) * EW_ZP];    // narrow (<= 64 candidates): staged candidate rows + a spare row
    float dbw[2 * TW_MAXB * EW_CPW];    // wide (65..128): D, then the MMD coefficients
  } a;
  union {
    DacpBlockScratch dw;                     // DACP scratch (before barrier 1)
    float gp[10][32 * EW_GP];                // Gram partial tiles (after barrier 1)
  } b;
  union {
    float cp[ECDA_THREADS / 64][DAD_C][DAD_H];   // per-wave centroid partial sums (until barrier 2)
    float dbn[TW_MAXB * EW_CP];                  // narrow: D, then the MMD coefficients (after barrier 2)
  } c;
  float cent[DAD_C][DAD_H];
  float nz[2 * TW_MAXB], wz[2 * TW_MAXB], rs[2 * TW_MAXB];
  int rowz[2 * TW_MAXB], mem[2 * TW_MAXB];
  int cnt[DAD_C];                       // masked noisy rows per class (pseudo-label)
  float pd[DAD_C][DAD_C];
  float msp[ECDA_THREADS / 64][DAD_H];   // per-wave sums of the member rows minus candidate row 0
  double nsp[ECDA_THREADS / 64];        // per-wave sums of |member row - candidate row 0|^2
  double t3p[ECDA_THREADS / 64][3];
  float cmp[ECDA_THREADS / 64];
};

// upper-triangle tile pair index of (ti <= tj) among nt tiles, and its inverse
__device__ __forceinline__ int ew_pair(int ti, int tj, int nt) { return ti * nt - ti * (ti - 1) / 2 + (tj - ti); }
__device__ __forceinline__ void ew_pair_inv(int pr, int nt, int& ti, int& tj) {
  ti = 0;
  while (pr >= nt - ti) { pr -= nt - ti; ++ti; }
  tj = ti + pr;
}

// Member gradients of a narrow class (NP = 32 or 64 padded candidates, rows and coefficients in
// LDS): 2 (rs_i z_i - (Csym Z)_i) scaled, plus the compactness and repulsion parts of the noisy
// members, per item of 32 candidates x 32 hidden units.  Every LDS operand of an item -- the
// NP/8 coefficient reads and 4 NP/8 row reads of the MFMA chain and the 16 rows' epilogue values
// -- is issued before its first MFMA.  The 32 x 32 result goes out through the wave's own LDS
// tile (the dead Gram partials, pitch EW_TP: the two lane halves' rows 32 banks apart), read back
// as 4 consecutive hidden units per lane: 4 dwordx4 stores per lane instead of 16 dword stores
// (the phase was bound by issuing the 32 KB of stores, not by the MFMA chain).
#define EW_TP 40
static_assert(ECDA_NG * 32 * EW_TP <= sizeof(EcdaW::b) / sizeof(float), "ew_member_grads: a 32 x EW_TP tile per wave in S.b");
// NK: the 8-candidate blocks of the (Csym Z) chain, ceil(ncand_all / 8) (the coefficients and rows
// past the candidates are zero, so the blocks they fill add nothing): a 33-candidate class runs 5
// blocks of its 64-row tiling's 8
// 64-row tiling: the 8-candidate column blocks of the coefficient matrix that the member-gradient
// chain reads (ew_member_grads<64, NK> reads columns [0, 8 NK) of db) and that the coefficient pass
// therefore writes: ONE helper for both, so the pass never leaves a read column stale
__device__ __forceinline__ int ew_nk64(int ncand_all) { return max((ncand_all + 7) >> 3, 5); }

template <int NP, int NK, class RG>
__device__ __forceinline__ void ew_member_grads(EcdaW& S, const float* db, int dp, int c, int ncs, int ncand_all,
                                                float mmd_scale, float comp_scale, float* ge_c, float* ge_s,
                                                float* sink, const RG& repg_at) {
  static_assert(NK >= 1 && NK <= NP / 8, "ew_member_grads: NK 8-candidate blocks of NP");
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = lane >> 5, l32 = lane & 31;
  for (int item = g; item < (NP / 32) * (DAD_H / 32); item += ECDA_NG) {
    const int ti = item >> 3, tc = item & 7;
    const int d = 32 * tc + l32;
    const float* ra = &db[(32 * ti + l32) * dp + 4 * kh];
    f32x4 av[NK];
    float bv[NK][4];
#pragma unroll
    for (int q = 0; q < NK; ++q) {
      av[q] = *reinterpret_cast<const f32x4*>(ra + 8 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[q][e] = S.a.zc[(8 * q + 4 * kh + e) * EW_ZP + d];
    }
    float zi[16], rsv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * ti + dad_acc_row(r, kh);   // (< NP <= TW_MAXB: staged or zero row)
      const int ic = i < ncand_all ? i : 0;
      zi[r] = S.a.zc[i * EW_ZP + d];
      rsv[r] = S.rs[ic];
    }
    const float mu = S.cent[c][d], rg = repg_at(d);
    f32x16 acc = f32x16{};
#pragma unroll
    for (int q = 0; q < NK; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q][e], bv[q][e], acc, 0, 0, 0);
    ECDA_CYC(25);
    float* stg = &S.b.gp[0][0] + g * (32 * EW_TP);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = 32 * ti + dad_acc_row(r, kh);
      const bool noisy = i >= ncs;
      stg[dad_acc_row(r, kh) * EW_TP + l32] =
          mmd_scale * (2.0f * (rsv[r] * zi[r] - acc[r])) + (noisy ? comp_scale * (zi[r] - mu) + rg : 0.0f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (the wave's own tile: LDS ops are in order)
    ECDA_CYC(26);
    // every row stored: members to their ge row, the rest to the sink (no branch)
    const int rl = lane >> 3, c4 = 4 * (lane & 7);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = rl + 8 * k, i = 32 * ti + row;
      const int ic = i < ncand_all ? i : 0;
      const bool mem = (i < ncand_all) & (S.mem[ic] != 0);
      const f32x4 v = *reinterpret_cast<const f32x4*>(stg + row * EW_TP + c4);
      float* dst = mem ? (i >= ncs ? ge_s : ge_c) + (size_t)S.rowz[ic] * DAD_H + 32 * tc + c4 : sink + 32 * tc + c4;
      *reinterpret_cast<f32x4*>(dst) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tile reads done before the next item's writes
    ECDA_CYC(27);
  }
}

// The class work after the candidates are known.  WIDE = more than 64 candidates: rows are read
// from the embedding buffer (global, through the candidate -> row table) instead of LDS.
template <bool WIDE>
__device__ __forceinline__ void ecda_class_w(const DadEcdaArgs& a, const int c, EcdaW& S, const WaveMask& M,
                                             const f32x4 (&ps)[ECDA_PRE_U], const int prd,
                                             const int ncls, const int nvalid, const int npairs, const bool gc,
                                             const bool rep_on, const float rep_coef, const float att_c, const int ncs,
                                             const int ncand_all, const double wsum_t) {
  const dad_config& cfg = a.cfg;
  const int B = cfg.B, Bn = cfg.Bn;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = lane >> 5, l32 = lane & 31;
  const float* emb_c = a.emb;
  const float* emb_s = a.emb + (size_t)(B + Bn) * DAD_H;
  const int npad = ncand_all <= 32 ? 32 : (ncand_all <= 64 ? 64 : 128);
  const int nt = npad / 32;                       // 32-row tiles
  const int npt = nt * (nt + 1) / 2;              // upper-triangle tile pairs: 1, 3 or 10
  const int ks = npt == 1 ? 8 : (npt == 3 ? 2 : 1);   // K splits per pair
  float* db = WIDE ? S.a.dbw : S.c.dbn;
  const int dp = WIDE ? EW_CPW : EW_CP;
  const int cnc = S.cnt[c];
  const int nmem = ncs + cnc;   // members: clean candidates + masked noisy candidates
  // candidate row i: LDS (narrow) or the embedding buffer (wide; rows past the candidates: zero)
  auto rowp = [&](int i) -> const float* {
    if constexpr (WIDE) return (i < ncs ? emb_c : emb_s) + (size_t)S.rowz[i < ncand_all ? i : 0] * DAD_H;
    else return &S.a.zc[i * EW_ZP];
  };
  auto rowv = [&](int i, int col) -> float {
    if constexpr (WIDE) return i < ncand_all ? rowp(i)[col] : 0.0f;
    else return S.a.zc[i * EW_ZP + col];
  };
  if (gc) {
    // squared norms of the candidate rows (a runtime loop: only the candidates are summed), and
    // for the bandwidth this wave's sums over its member rows of d = z - z0 and |d|^2, z0 =
    // candidate row 0 (lane = 4 hidden units).  Post-ReLU embeddings share a large positive mean;
    // centred on a row of the class, the identity below sums no large cancelling terms.
    f32x4 ms = f32x4{};
    double ns = 0.0;
    const f32x4 z0 = *reinterpret_cast<const f32x4*>(rowp(0) + 4 * lane);
    for (int r = g; r < ncand_all; r += ECDA_NG) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(rowp(r) + 4 * lane);
      const float nr = dad_wave_sum(((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]) + v[3] * v[3]);
      if (lane == 0) S.nz[r] = nr;
      if (S.mem[r]) {
        const f32x4 d = v - z0;
        ms += d;
        ns += (double)dad_wave_sum(((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) + d[3] * d[3]);
      }
    }
    *reinterpret_cast<f32x4*>(&S.msp[g][4 * lane]) = ms;
    if (lane == 0) S.nsp[g] = ns;
    // Gram partials: tile pair (ti, tj) over a K slice, fp32 matrix cores.  The 64-row tiling
    // (3 pairs) cuts pairs (0,0) and (0,1) into 4 slices and (1,1) into 2: 10 items in the 10
    // partial slots, dealt so that the waves w and w + 4 (one SIMD's pair) hold 6 slices' MFMAs
    // each (3 x 64 or 128 + 64 of K) instead of two 128-K items on two SIMDs and one on the others
    for (int item = g; item < (npt == 3 ? 10 : npt * ks); item += ECDA_NG) {
      int pr, sl, nsl;
      if (npt == 3) {
        // item -> pair (2 bits) | slice (2 bits): 0:(0,2) 1:(1,1) 2:(2,0) 3:(2,1) 4:(0,3) 5:(1,2)
        // 6:(0,0) 7:(0,1) 8:(1,0) 9:(1,3)
        constexpr uint64_t kDeal = 0x2ull | (0x5ull << 4) | (0x8ull << 8) | (0x9ull << 12) | (0x3ull << 16) |
                                   (0x6ull << 20) | (0x0ull << 24) | (0x1ull << 28) | (0x4ull << 32) | (0x7ull << 36);
        const int v = (int)((kDeal >> (4 * item)) & 15u);
        pr = v >> 2;
        sl = v & 3;
        nsl = pr < 2 ? 4 : 2;
      } else {
        pr = item / ks;
        sl = item - pr * ks;
        nsl = ks;
      }
      const int slot = npt == 3 ? (pr < 2 ? 4 * pr : 8) + sl : item;
      int ti, tj;
      ew_pair_inv(pr, nt, ti, tj);
      const int kw = DAD_H / nsl, k0 = sl * kw;
      const int ia = 32 * ti + l32, ib = 32 * tj + l32;
      // MFMA step e of a k-block of 8 takes k-index k + 4 kh + e on both operands (any k order
      // sums the same dot products): each lane reads 4 consecutive floats per operand
      const float* ra = rowp(ia) + 4 * kh;
      const float* rb = rowp(ib) + 4 * kh;
      const bool za = WIDE && ia >= ncand_all, zb = WIDE && ib >= ncand_all;
      f32x16 acc = f32x16{};
      for (int k = k0; k < k0 + kw; k += 8) {
        f32x4 av = *reinterpret_cast<const f32x4*>(ra + k), bv = *reinterpret_cast<const f32x4*>(rb + k);
        if (za) av = f32x4{};
        if (zb) bv = f32x4{};
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bv[e], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) S.b.gp[slot][dad_acc_row(r, kh) * EW_GP + l32] = acc[r];
    }
  }
  // centroids of every class over its masked noisy rows, partials combined in wave order
  for (int e = tid; e < DAD_C * DAD_H; e += ECDA_THREADS) {
    const int k = e >> 8, hh = e & (DAD_H - 1);
    float sk = 0.0f;
#pragma unroll
    for (int gg = 0; gg < ECDA_NG; ++gg) sk += S.c.cp[gg][k][hh];
    const int nk = S.cnt[k];
    S.cent[k][hh] = nk > 0 ? sk / (float)nk : 0.0f;
  }
  ECDA_STAMP(4);
  __syncthreads();   // ---------------------------------------------------------------- 2
  ECDA_STAMP(5);
  ECDA_CYC(6);
  // element ownership of the [npad x npad] matrices: row ei, columns ej0 .. ej0 + ept - 1
  const int ept = npad * npad / ECDA_THREADS;     // 2, 8 or 32
  const int tpr = npad / ept;                     // threads per row: 16, 8 or 4
  const int ei = tid / tpr, ej0 = (tid - ei * tpr) * ept;
  // centroid distances (I/utils.py:582-595): 32 threads per (p, q) pair, pair-symmetric order
  {
    const int pair = tid / 32, t32 = tid & 31;
    float d = 0.0f;
    if (pair < DAD_C * DAD_C) {
      const int p = pair / DAD_C, q = pair % DAD_C;
      const int lo = p < q ? p : q, hi = p < q ? q : p;
      const int np = S.cnt[p];
      const int nq = S.cnt[q];
      if (p < ncls && q < ncls && np > 0 && nq > 0 && p != q) {
        const f32x4* a0 = reinterpret_cast<const f32x4*>(&S.cent[lo][t32 * (DAD_H / 32)]);
        const f32x4* a1 = reinterpret_cast<const f32x4*>(&S.cent[hi][t32 * (DAD_H / 32)]);
        const f32x4 x0 = a0[0], x1 = a0[1], y0 = a1[0], y1 = a1[1];
        const float v[8] = {x0[0] - y0[0], x0[1] - y0[1], x0[2] - y0[2], x0[3] - y0[3],
                            x1[0] - y1[0], x1[1] - y1[1], x1[2] - y1[2], x1[3] - y1[3]};
#pragma unroll
        for (int k = 0; k < 8; ++k) d += v[k] * v[k];
      }
    }
    d = dpp_seg_sum<32>(d);
    if (pair < DAD_C * DAD_C && t32 == 31) S.pd[pair / DAD_C][pair % DAD_C] = sqrtf(d);
  }
  ECDA_CYC(20);
  const float Wss = (float)ncs * (float)ncs + 1e-8f;
  const float Wtt = (float)(wsum_t * wsum_t) + 1e-8f;
  const float Wst = (float)((double)ncs * wsum_t) + 1e-8f;
  if (gc) {
    // compactness partial (I/utils.py:614-616): this wave's masked noisy rows of class c
    float cpart = 0.0f;
    const f32x4 mu = *reinterpret_cast<const f32x4*>(&S.cent[c][4 * lane]);
#pragma unroll
    for (int u = 0; u < ECDA_PRE_U; ++u) {
      const int b = g + ECDA_NG * u;
      const int pk = __builtin_amdgcn_readlane(prd, b < 64 ? b : 0);
      if (b < Bn && pk == c) {
        const f32x4 df = ps[u] - mu;
        cpart += ((df[0] * df[0] + df[1] * df[1]) + df[2] * df[2]) + df[3] * df[3];
      }
    }
    cpart = dad_wave_sum(cpart);
    // detached bandwidth (I/utils.py:538-544) without the distance matrix: over the nmem member
    // rows, with d_i = z_i - z0 for any fixed z0, sum_ij |z_i - z_j|^2 = 2 nmem sum_i |d_i|^2 -
    // 2 |sum_i d_i|^2, from the waves' partial sums (every wave alike, combined in double), so the
    // kernel values and coefficients follow the distances in the same pass (the distance matrix
    // no longer makes a round trip through LDS and a barrier before them)
    f32x4 m = f32x4{};
#pragma unroll
    for (int gg = 0; gg < ECDA_NG; ++gg) m += *reinterpret_cast<const f32x4*>(&S.msp[gg][4 * lane]);
    const double msq = dad_wave_sum_d(((double)m[0] * m[0] + (double)m[1] * m[1]) + ((double)m[2] * m[2] + (double)m[3] * m[3]));
    double nsq = 0.0;
#pragma unroll
    for (int gg = 0; gg < ECDA_NG; ++gg) nsq += S.nsp[gg];
    const double bws = fmax(2.0 * (double)nmem * nsq - 2.0 * msq, 0.0);
    float bw = nmem > 1 ? (float)(bws / (double)(nmem * nmem - nmem)) : 1.0f;
    bw = bw / 4.0f;
    float ibw[5];
#pragma unroll
    for (int mm = 0; mm < 5; ++mm) ibw[mm] = 1.0f / (bw * (float)(1 << mm) + 1e-8f);
    ECDA_CYC(21);
    // the weighted kernel terms (I/utils.py:546-563): every ordered member pair (i, j); the
    // symmetric coefficients Csym_ij = dmmd/dD_ij + dmmd/dD_ji; branch-free, invalid elements 0
    double t3[3] = {0.0, 0.0, 0.0};
    float rsp = 0.0f;
    const int ic = ei < ncand_all ? ei : 0;
    const bool mi = (ei < ncand_all) & (S.mem[ic] != 0);
    const float wi = S.wz[ic];
    const bool si = ei < ncs;
    const float css = 2.0f / Wss, ctt = 2.0f / Wtt, cst = -2.0f / Wst;
    auto coef = [&](const int j) {
      const int i = ei;
      // G_ij read at (min, max) in the upper-triangle tiles: D is symmetric bit for bit
      const int lo = i < j ? i : j, hi = i < j ? j : i;
      const int pr = ew_pair(lo >> 5, hi >> 5, nt);
      float gsum = 0.0f;
      const int sb = npt == 3 ? (pr < 2 ? 4 * pr : 8) : pr * ks, sn = npt == 3 ? (pr < 2 ? 4 : 2) : ks;
      for (int s2 = 0; s2 < sn; ++s2) gsum += S.b.gp[sb + s2][(lo & 31) * EW_GP + (hi & 31)];
      const bool ok = (i < ncand_all) & (j < ncand_all) & (i != j);
      const float d = ok ? fmaxf((S.nz[lo] + S.nz[hi]) - 2.0f * gsum, 0.0f) : 0.0f;
      const int jc = j < ncand_all ? j : 0;
      const bool on = mi & (j < ncand_all) & (S.mem[jc] != 0);
      const float wj = S.wz[jc];
      float K = 0.0f, dK = 0.0f;
#pragma unroll
      for (int mm = 0; mm < 5; ++mm) {
        const float ex = __expf(-d * ibw[mm]);
        K += ex;
        dK -= ex * ibw[mm];
      }
      const bool sj = j < ncs;
      const bool ss = on & si & sj, tt = on & !si & !sj, st = on & si & !sj, ts = on & !si & sj;
      const float ww = wi * wj;
      t3[0] += ss ? (double)K : 0.0;
      t3[1] += tt ? (double)K * ww : 0.0;
      t3[2] += st ? (double)K * wj : 0.0;
      // Csym: SS 2/Wss dK, TT 2 w_i w_j/Wtt dK, ST -2 w_j/Wst dK, TS -2 w_i/Wst dK
      const float vss = css * dK, vtt = (ctt * ww) * dK, vst = (cst * wj) * dK, vts = (cst * wi) * dK;
      float v = ss ? vss : (tt ? vtt : (st ? vst : (ts ? vts : 0.0f)));
      v = i == j ? 0.0f : v;
      rsp += v;
      return v;
    };
    // 64-row tiling: the thread's 8 elements unrolled, their stores after the last one (a store
    // to db inside the loop kept the next element's LDS reads behind it: pairs 9.7k -> 8.9k
    // cycles for a 38-41 member class; the 32-row case, 2 elements, measured no better so)
    if (!WIDE && npad == 64) {
      // the 64-row tiling: thread column jt + tpr e, only the columns the member-gradient chain
      // reads (8 ceil(ncand / 8), ew_member_grads' NK blocks), so a 40-candidate class runs 5 of
      // the 8 elements per thread; rows past the candidates get their zeros without the kernel math
      const int jt = ej0 / ept, kz = 8 * ew_nk64(ncand_all);   // = ew_member_grads' 8 NK columns
      float v8[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = jt + 8 * e;
        v8[e] = (j < kz && ei < ncand_all) ? coef(j) : 0.0f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (jt + 8 * e < kz) db[ei * dp + jt + 8 * e] = v8[e];
    } else {
      for (int e = 0; e < ept; ++e) db[ei * dp + ej0 + e] = coef(ej0 + e);
    }
    ECDA_CYC(22);
    // row sums of the coefficients: the tpr threads of a row are adjacent lanes
    rsp = tpr == 16 ? dpp_seg_sum<16>(rsp) : (tpr == 8 ? dpp_seg_sum<8>(rsp) : dpp_seg_sum<4>(rsp));
    if ((tid & (tpr - 1)) == tpr - 1) S.rs[ei] = rsp;
#pragma unroll
    for (int k = 0; k < 3; ++k) t3[k] = dad_wave_sum_d(t3[k]);
    if (lane == 0) { S.t3p[g][0] = t3[0]; S.t3p[g][1] = t3[1]; S.t3p[g][2] = t3[2]; S.cmp[g] = cpart; }
    ECDA_CYC(23);
  }
  __syncthreads();   // ---------------------------------------------------------------- 3
  ECDA_STAMP(7);
  const float wscale = cfg.w_ecda;
  float pd[DAD_C][DAD_C];
#pragma unroll
  for (int p = 0; p < DAD_C; ++p)
#pragma unroll
    for (int q = 0; q < DAD_C; ++q) pd[p][q] = S.pd[p][q];
  float rep = 0.0f;
  if (nvalid > 1) {
    float sp = 0.0f;
#pragma unroll
    for (int p = 0; p < DAD_C; ++p)
#pragma unroll
      for (int q = p + 1; q < DAD_C; ++q) {
        const int np = S.cnt[p];
        const int nq = S.cnt[q];
        if (q < ncls && np > 0 && nq > 0) sp += pd[p][q];
      }
    rep = -sp / (float)npairs;
  }
  // repulsion grad of the class's noisy members at hidden unit d (d rep / d mu_c / n_c), each
  // lane for its own columns: rk * sum_q (cent_c[d] - cent_q[d]) / pd_cq over the valid other
  // classes in the reference's class order; the reciprocals are wave-uniform, taken once
  float rq[DAD_C];
#pragma unroll
  for (int q = 0; q < DAD_C; ++q) {
    const int nq = S.cnt[q];
    const float nd = S.pd[c][q];
    rq[q] = (rep_on && q != c && q < ncls && nq > 0 && nd > 0.0f) ? 1.0f / nd : 0.0f;
  }
  const float rk = rep_on ? -wscale * rep_coef / (float)npairs / (float)cnc : 0.0f;
  auto repg_at = [&](int d) -> float {
    if (!rep_on) return 0.0f;
    const float cc0 = S.cent[c][d];
    float gsum = 0.0f;
#pragma unroll
    for (int q = 0; q < DAD_C; ++q) gsum += rq[q] != 0.0f ? (cc0 - S.cent[q][d]) * rq[q] : 0.0f;
    return rk * gsum;
  };
  float* ge_c = a.ge;
  float* ge_s = a.ge + (size_t)B * DAD_H;
  if (gc) {
    double t3[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int gg = 0; gg < ECDA_NG; ++gg) {
      t3[0] += S.t3p[gg][0];
      t3[1] += S.t3p[gg][1];
      t3[2] += S.t3p[gg][2];
    }
    // t_ss, t_tt, t_st as the reference forms them in float32 (I/utils.py:558-563)
    const float mmd = (float)t3[0] / Wss + (float)t3[1] / Wtt - 2.0f * ((float)t3[2] / Wst);
    float csum = 0.0f;
#pragma unroll
    for (int gg = 0; gg < ECDA_NG; ++gg) csum += S.cmp[gg];
    const float comp = csum / (float)cnc;
    if (tid == 0) {
      a.tail_terms[c] = att_c * (mmd + cfg.ecda_gamma * comp + cfg.ecda_delta * rep);
      a.tail_terms[DAD_T_ECDA_GATE - DAD_T_ECDA_TERM + c] = 1.0f;
    }
    ECDA_CYC(24);
    const float mmd_scale = wscale * att_c;
    const float comp_scale = wscale * att_c * cfg.ecda_gamma * (2.0f / (float)cnc);
    // member grads 2 sum_j Csym_ij (z_i - z_j) = 2 (rs_i z_i - (Csym Z)_i): (Csym Z) on the
    // matrix cores, 32 candidates x 32 hidden units per item
    if constexpr (!WIDE) {
      if (npad == 32) {
        ew_member_grads<32, 4>(S, db, dp, c, ncs, ncand_all, mmd_scale, comp_scale, ge_c, ge_s, a.sink, repg_at);
      } else {
        const int nk = ew_nk64(ncand_all);   // 5 .. 8 (33 .. 64 candidates): the columns the pass wrote
        if (nk <= 5) ew_member_grads<64, 5>(S, db, dp, c, ncs, ncand_all, mmd_scale, comp_scale, ge_c, ge_s, a.sink, repg_at);
        else if (nk == 6) ew_member_grads<64, 6>(S, db, dp, c, ncs, ncand_all, mmd_scale, comp_scale, ge_c, ge_s, a.sink, repg_at);
        else if (nk == 7) ew_member_grads<64, 7>(S, db, dp, c, ncs, ncand_all, mmd_scale, comp_scale, ge_c, ge_s, a.sink, repg_at);
        else ew_member_grads<64, 8>(S, db, dp, c, ncs, ncand_all, mmd_scale, comp_scale, ge_c, ge_s, a.sink, repg_at);
      }
    }
    for (int item = g; WIDE && item < nt * (DAD_H / 32); item += ECDA_NG) {
      const int ti = item >> 3, tc = item & 7;
      const int d = 32 * tc + l32;
      f32x16 acc = f32x16{};
      const float* ra = &db[(32 * ti + l32) * dp + 4 * kh];
      for (int k = 0; k < npad; k += 8) {
        // step e: candidate k + 4 kh + e (one b128 read of the coefficient row per lane)
        const f32x4 av = *reinterpret_cast<const f32x4*>(ra + k);
        float bv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = rowv(k + 4 * kh + e, d);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[e], bv[e], acc, 0, 0, 0);
      }
      const float mu = S.cent[c][d], rg = repg_at(d);
      // every accumulator row stored: members to their ge row, the rest to the sink (no branch)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * ti + dad_acc_row(r, kh);
        const int ic = i < ncand_all ? i : 0;
        const bool ok = (i < ncand_all) & (S.mem[ic] != 0);
        const float zi = rowv(i, d);
        const bool noisy = i >= ncs;
        const float gv = mmd_scale * (2.0f * (S.rs[ic] * zi - acc[r])) + (noisy ? comp_scale * (zi - mu) + rg : 0.0f);
        float* dst = ok ? (noisy ? ge_s : ge_c) + (size_t)S.rowz[ic] * DAD_H + d : a.sink + d;
        *dst = gv;
      }
    }
  } else {
    // a class below the gate only feeds the repulsion: its noisy members get repg
    const int nct = ncand_all - ncs;
    for (int e = tid; e < nct * (DAD_H / 4); e += ECDA_THREADS) {
      const int i = ncs + e / (DAD_H / 4), q = e % (DAD_H / 4);
      if (S.mem[i]) {
        const f32x4 v = f32x4{repg_at(4 * q), repg_at(4 * q + 1), repg_at(4 * q + 2), repg_at(4 * q + 3)};
        reinterpret_cast<f32x4*>(ge_s + (size_t)S.rowz[i] * DAD_H)[q] = v;
      }
    }
  }
  for (int i = tid; i < ncand_all; i += ECDA_THREADS)
    if (S.mem[i]) a.eflag[i < ncs ? S.rowz[i] : B + S.rowz[i]] = 1u;
  ECDA_STAMP(8);
  if (tid == 0) ECDA_STAMP_SIZES(c, ncand_all, ncs);
}

// One ECDA class (I/utils.py:565-632, class-aware) for B, Bn <= 64.
__device__ __forceinline__ void ecda_block_w(const DadEcdaArgs& a, const DadTailArgs& ta, const int c, EcdaW& S) {
  const dad_config& cfg = a.cfg;
  const int B = cfg.B, Bn = cfg.Bn;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* emb_c = a.emb;
  const float* emb_s = a.emb + (size_t)(B + Bn) * DAD_H;
  ECDA_STAMP(0);
  // ---- entry: teacher logits (lane = noisy row), labels (lane = clean row), and the embedding
  // rows this wave handles (rows g, g + 8, ...; lane = 16-B column chunk), all in flight
  // every load unconditional (rows clamped; the clamped duplicates are never used): a load
  // under a condition is waited for where the paths merge, one round trip each
  const int rc = lane < B ? lane : B - 1, rn = lane < Bn ? lane : Bn - 1;
  const f32x4 zt = reinterpret_cast<const f32x4*>(ta.logits + (size_t)B * DAD_C)[rn];
  const int yv = (int)a.yc[rc];
  const float dv = ta.dacp[lane < DAD_DACP_FLOATS ? lane : 0];
  // the rows are issued after the DACP inputs, so the DACP waits for those alone (counted
  // vmcnt) while the rows are still in flight
  __builtin_amdgcn_sched_barrier(0);
  // strong rows: all (the centroids of every class need the masked ones)
  f32x4 pc[ECDA_PRE_U], ps[ECDA_PRE_U];
#pragma unroll
  for (int u = 0; u < ECDA_PRE_U; ++u) {
    const int b = g + ECDA_NG * u;
    ps[u] = reinterpret_cast<const f32x4*>(emb_s + (size_t)(b < Bn ? b : Bn - 1) * DAD_H)[lane];
  }
  const int y = lane < B ? yv : -1;
  // clean rows: only this class's candidates (label c), compacted; wave g loads candidates
  // g, g + 8, ... (row 0 past the last), in flight during the DACP.  Per-CU load bandwidth from
  // another XCD's writes is the limit here, so rows nobody stages are not fetched.
  const uint64_t bcl = __ballot(y == c);
  const int ncl = (int)__popcll(bcl);
  const int posl = (int)__popcll(bcl & ((1ull << lane) - 1ull));
#pragma unroll
  for (int u = 0; u < ECDA_PRE_U; ++u) {
    const int j = g + ECDA_NG * u;
    const uint64_t hit = __ballot((y == c) & (posl == j));
    const int row = hit ? (int)__builtin_ctzll(hit) : 0;
    pc[u] = reinterpret_cast<const f32x4*>(emb_c + (size_t)row * DAD_H)[lane];
  }
  // ---- the DACP mask, in this wave (every wave computes the same one)
  WaveMask M;
  block_mask(cfg, Bn, zt, dacp_state_of(dv), S.b.dw, M);
  ECDA_STAMP(1);
  const int prd = M.m ? M.p : -1;                                // I/utils.py:573-576
  const float msum = (float)__popcll(__ballot(M.m));
  if (!(msum > 1.0f && cfg.ecda_on)) return;                     // I/train.py:444,450
  const int ncls = cfg.use_dacp ? DAD_C : (Bn < DAD_C ? Bn : DAD_C);
  if (c >= ncls) return;
  // per-class counts, attention, gates, repulsion coefficient (uniform; I/utils.py:582-610)
  int cc[DAD_C], cn[DAD_C];
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) {
    cc[k] = k < ncls ? (int)__popcll(__ballot(y == k)) : 0;
    cn[k] = k < ncls ? (int)__popcll(__ballot(prd == k)) : 0;
  }
  float att[DAD_C];
  if (cfg.use_dacp) {
    const float wmean = (((M.wc[0] + M.wc[1]) + M.wc[2]) + M.wc[3]) / 4.0f;
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) att[k] = expf(cfg.ecda_att_lambda * (wmean - M.wc[k]));
  } else {
#pragma unroll
    for (int k = 0; k < DAD_C; ++k) att[k] = 1.0f;
  }
  int nvalid = 0;
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) nvalid += (k < ncls && cn[k] > 0) ? 1 : 0;
  const int npairs = nvalid * (nvalid - 1) / 2;
#if DAD_PROBE_ON
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stamps build: when the prefetched rows have landed
  ECDA_STAMP(9);
  ECDA_CYC(19);
#endif
  bool gated[DAD_C];
  float rep_coef = 0.0f;
#pragma unroll
  for (int k = 0; k < DAD_C; ++k) {
    gated[k] = k < ncls && cc[k] >= 2 && cn[k] >= 2;   // I/utils.py:609-610
    if (gated[k]) rep_coef += att[k] * cfg.ecda_delta;
  }
  const int cnc = c == 0 ? cn[0] : (c == 1 ? cn[1] : (c == 2 ? cn[2] : cn[3]));
  const int ccc = c == 0 ? cc[0] : (c == 1 ? cc[1] : (c == 2 ? cc[2] : cc[3]));
  const bool gc = c == 0 ? gated[0] : (c == 1 ? gated[1] : (c == 2 ? gated[2] : gated[3]));
  const float att_c = sel4(att, c);
  const bool rep_on = nvalid > 1 && cnc > 0 && rep_coef != 0.0f;
  ECDA_CYC(13);
  if (!gc && !rep_on) return;
  // candidates: clean rows of label c (members when gated), then the noisy rows of pseudo-label c
  // that the mask takes in (I/utils.py:573-576, the reference's target set); positions by ballot
  // prefix counts, every wave alike.  Noisy rows of pseudo-label c left out by the mask take no part
  // in any term (kernel pairs, bandwidth, centroids, gradients), so they are not staged: a teacher
  // that sends most of the noisy batch to one class with half of it masked out no longer pushes
  // that class past 64 candidates into the wide path
  const bool ccand = gc && y == c;
  const bool ncand = lane < Bn && M.p == c && M.m;
  const uint64_t bc = __ballot(ccand), bn = __ballot(ncand);
  const int ncs = gc ? ccc : 0;
  const int ncand_all = ncs + (int)__popcll(bn);
  const bool wide = ncand_all > TW_MAXB;
  const uint64_t below = (1ull << lane) - 1ull;
  const int posc = (int)__popcll(bc & below);
  const int posn = ncs + (int)__popcll(bn & below);
  // ---- stage: candidate norms (and, narrow, rows), weights, rows and member flags; the
  // per-wave centroid partial sums of every class
  // a wave's candidate rows: their candidate positions (uniform), the others go to the spare
  // row TW_MAXB (narrow) -- unconditional stores, no branches; norms by one batched butterfly
  int npos[2 * ECDA_PRE_U];
#pragma unroll
  for (int u = 0; u < ECDA_PRE_U; ++u) {
    const int b = g + ECDA_NG * u;                 // noisy row b; clean candidate b (compacted)
    const bool okc = gc & (b < ncl);
    const bool okn = (b < Bn) & (((bn >> b) & 1ull) != 0);
    npos[2 * u] = __builtin_amdgcn_readfirstlane(okc ? b : -1);
    npos[2 * u + 1] = __builtin_amdgcn_readfirstlane(okn ? __builtin_amdgcn_readlane(posn, b) : -1);
    // candidate rows only, under uniform (scalar) branches: storing every row (the others to a
    // spare row) had all 8 waves queue 128 KB of LDS writes at once (~2500 cycles per wave)
    if (!wide & okc) *reinterpret_cast<f32x4*>(&S.a.zc[npos[2 * u] * EW_ZP + 4 * lane]) = pc[u];
    if (!wide & okn) *reinterpret_cast<f32x4*>(&S.a.zc[npos[2 * u + 1] * EW_ZP + 4 * lane]) = ps[u];
  }
  ECDA_CYC(14);
  // (the candidates' squared norms are taken from the staged rows after barrier 1: here the
  // compiler computed the wave sums of all 16 rows, candidate or not, ~2000 cycles)
  ECDA_STAMP(12);
  ECDA_CYC(15);
  if (!wide) {
    const int npad = ncand_all <= 32 ? 32 : 64;
    for (int r = ncand_all + g; r < npad; r += ECDA_NG) *reinterpret_cast<f32x4*>(&S.a.zc[r * EW_ZP + 4 * lane]) = f32x4{};
  }
  if (g == 0) {
    if (lane < DAD_C) S.cnt[lane] = sel4i(cn, lane);
    if (ccand) { S.rowz[posc] = lane; S.wz[posc] = 1.0f; S.mem[posc] = 1; }
    if (ncand) { S.rowz[posn] = lane; S.wz[posn] = M.s; S.mem[posn] = 1; }
  }
  ECDA_CYC(16);
  {
    // the class of each row is wave-uniform: one add per row into its class's sum (a uniform
    // branch), not a select per class
    // branch-free: each row added to every class sum times a uniform 0/1 factor (adding
    // zeros leaves each sum bit-identical); a switch on the class made a branch per row and
    // register copies at every join (~2000 cycles)
    f32x4 cs0 = f32x4{}, cs1 = f32x4{}, cs2 = f32x4{}, cs3 = f32x4{};
#pragma unroll
    for (int u = 0; u < ECDA_PRE_U; ++u) {
      const int b = g + ECDA_NG * u;
      const int pk = __builtin_amdgcn_readfirstlane(b < Bn ? __builtin_amdgcn_readlane(prd, b < 64 ? b : 0) : -1);
      cs0 += ps[u] * (pk == 0 ? 1.0f : 0.0f);
      cs1 += ps[u] * (pk == 1 ? 1.0f : 0.0f);
      cs2 += ps[u] * (pk == 2 ? 1.0f : 0.0f);
      cs3 += ps[u] * (pk == 3 ? 1.0f : 0.0f);
    }
    *reinterpret_cast<f32x4*>(&S.c.cp[g][0][4 * lane]) = cs0;
    *reinterpret_cast<f32x4*>(&S.c.cp[g][1][4 * lane]) = cs1;
    *reinterpret_cast<f32x4*>(&S.c.cp[g][2][4 * lane]) = cs2;
    *reinterpret_cast<f32x4*>(&S.c.cp[g][3][4 * lane]) = cs3;
  }
  ECDA_CYC(17);
  // weight sum of the noisy members (I/utils.py:552-557), in every wave
  const double wsum_t = dad_wave_sum_d(ncand ? (double)M.s : 0.0);
  (void)cc;
  ECDA_CYC(18);
  ECDA_STAMP(2);
  __syncthreads();   // ---------------------------------------------------------------- 1
  ECDA_STAMP(3);
  if (wide)
    ecda_class_w<true>(a, c, S, M, ps, prd, ncls, nvalid, npairs, gc, rep_on, rep_coef, att_c, ncs, ncand_all, wsum_t);
  else
    ecda_class_w<false>(a, c, S, M, ps, prd, ncls, nvalid, npairs, gc, rep_on, rep_coef, att_c, ncs, ncand_all, wsum_t);
}

// block 0: the wave-centric tail; blocks 1..C: ECDA class blockIdx.x - 1.  Host contract:
// B <= 64, Bn <= 64, class-aware MMD (dad_tail_ecda otherwise).  Blocks > C pool the step's
// embeddings and logits first (pl.ready set; the tail and class blocks wait for them: pool_wait),
// which saves the separate dad_pool launch and its boundary.  Then (when pa.x16 is set):
// the NEXT step's row preparation (dad_prep.h) on the CUs the tail and the class blocks leave
// idle; it reads only the next batch and writes only the other prepared set, so it overlaps this
// step's latency-bound tail and ECDA.  The tail and class blocks have the lowest block ids, so
// they are dispatched first and never wait for a CU behind the preparation blocks.
__global__ __launch_bounds__(TAIL_THREADS) void dad_tail_ecda_w(DadTailArgs ta, DadEcdaArgs ca, DadPrepArgs pa,
                                                                  DadPoolArgs pl) {
  DAD_GUARD_BLOCK(TAIL_THREADS);
  __shared__ union UW {
    TailW t;
    EcdaW e;
  } u;
  // fused pooling (pl.ready): the Bc + 2 Bn pool items (dad_pool's workgroups) on the spare
  // blocks' waves, item i on block i mod nx, wave i / nx (one item per CU first)
  const int nitems = pl.ready ? pl.g.Bc + 2 * pl.g.Bn : 0;
  if ((int)blockIdx.x > DAD_C) {
    constexpr int kWaves = TAIL_THREADS / 64;
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int nx = (int)gridDim.x - 1 - DAD_C, xb = (int)blockIdx.x - 1 - DAD_C;
    for (int i = xb + nx * w; i < nitems; i += nx * kWaves) {
      pool_item<true>(pl, i, (int)threadIdx.x & 63);
      pool_publish(pl.ready, (int)threadIdx.x & 63);
    }
    if (!pa.x16) return;
#ifdef DAD_PROBE_STAMPS
    if ((threadIdx.x & 63) == 0 && xb < 256) prep_stamps[2 * (xb * kWaves + w)] = DAD_PROBE_WALL();
#endif
    dad_prep_dispatch<2>(pa, xb * kWaves + w, nx * kWaves, (int)threadIdx.x & 63);
#ifdef DAD_PROBE_STAMPS
    if (threadIdx.x == 0) atomicMax(&ecda_stamps[DAD_C * ECDA_SLOTS + 15], (unsigned long long)DAD_PROBE_WALL());
    if ((threadIdx.x & 63) == 0 && xb < 256) prep_stamps[2 * (xb * kWaves + w) + 1] = DAD_PROBE_WALL();
#endif
    return;
  }
  if (ta.cfg.B > TW_MAXB || ta.cfg.Bn > TW_MAXB) return;
  if (blockIdx.x == 0) TAIL_STAMP(14);   // launch entry (slot 15: the last preparation block's end)
  if (nitems) pool_wait(pl.ready, (uint32_t)nitems, pl.range_flag);
  if (blockIdx.x == 0) tail_block_w(ta, u.t);
  else ecda_block_w(ca, ta, (int)blockIdx.x - 1, u.e);
}

// ------------------------------------------------------------- helper-type drop-ins
// DACPManager.calculate_certainty_scores (I/utils.py:400-428): one thread per row of probs.
__global__ __launch_bounds__(256) void dad_certainty_kernel(const float* probs, int B, int use_entropy, float* score,
                                                            int64_t* pred) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  const f32x4 v = reinterpret_cast<const f32x4*>(probs)[b];
  const float q[4] = {v[0], v[1], v[2], v[3]};
  float s;
  int p;
  certainty_from_probs(q, use_entropy != 0, s, p);
  if (score) score[b] = s;
  if (pred) pred[b] = p;
}

// DACPManager.calculate_mask (I/utils.py:449-507) on teacher probabilities, one workgroup:
// the tail block's own thresholds (dacp_thresholds) and mask, then the state update the fused
// step commits in dad_optim (tau EMA, epoch score sums and counts).  dacp = the 20-float state
// (tau | Q | sums | counts | anchors).
__global__ __launch_bounds__(TAIL_THREADS) void dad_dacp_mask_kernel(dad_config cfg, const float* probs, int Bn,
                                                                      float* dacp, uint8_t* mask, float* score,
                                                                      int64_t* pred, float* wout) {
  DAD_GUARD_BLOCK(TAIL_THREADS);
  __shared__ TailSmem T;
  const int tid = threadIdx.x;
  if (tid < 20) T.dstate[tid] = dacp[tid];
  for (int b = tid; b < Bn; b += TAIL_THREADS) {
    const f32x4 v = reinterpret_cast<const f32x4*>(probs)[b];
    const float q[4] = {v[0], v[1], v[2], v[3]};
    certainty_from_probs(q, cfg.use_entropy != 0, T.ss[b], T.sp[b]);
  }
  if (tid < DAD_C) T.ncls[tid] = 0;
  __syncthreads();
  float wc[DAD_C];
  dacp_thresholds(cfg, Bn, T.ss, T.sp, T.srt, T.ncls, T.dstate, T.tau_new, wc, nullptr, nullptr);
  double st4[4] = {0.0, 0.0, 0.0, 0.0}, ct4[4] = {0.0, 0.0, 0.0, 0.0};
  for (int b = tid; b < Bn; b += TAIL_THREADS) {
    const int p = T.sp[b];
    mask[b] = T.ss[b] >= T.tau_new[p] ? 1 : 0;
    if (score) score[b] = T.ss[b];
    if (pred) pred[b] = p;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      st4[c] += p == c ? (double)T.ss[b] : 0.0;
      ct4[c] += p == c ? 1.0 : 0.0;
    }
  }
  block_sum4_d(st4, T.dred4);
  block_sum4_d(ct4, T.dred4);
  if (tid < DAD_C) {
    dacp[tid] = T.tau_new[tid];
    dacp[8 + tid] += (float)st4[tid];
    dacp[12 + tid] += (float)ct4[tid];
    if (wout) wout[tid] = wc[tid];
  }
}

// ECDALoss.forward (I/utils.py:565-652) on caller embeddings: stage them in the step's layout
// (emb rows [clean | - | noisy], tail header + per-sample score / pred / mask) for dad_ecda.
__global__ __launch_bounds__(256) void dad_ecda_prep_kernel(const float* clean, int B, const float* noisy, int Bn,
                                                            const int64_t* noisy_labels, const uint8_t* noisy_mask,
                                                            const float* noisy_scores, const float* class_weights,
                                                            int nw, float* emb, float* tailf, uint32_t* eflag) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t nc = (size_t)B * DAD_H, nn = (size_t)Bn * DAD_H;
  if (i < nc) emb[i] = clean[i];
  if (i < nn) emb[(size_t)(B + Bn) * DAD_H + i] = noisy[i];
  if (i < DAD_TAIL_HDR) {
    float v = 0.0f;
    if (i >= DAD_T_W && i < DAD_T_W + DAD_C) v = (int)(i - DAD_T_W) < nw ? class_weights[i - DAD_T_W] : 1.0f;
    if (i == DAD_T_ECDA_ON) v = 1.0f;
    tailf[i] = v;
  }
  if (i < (size_t)Bn) {
    tailf[DAD_TAIL_HDR + i] = noisy_scores[i];
    tailf[DAD_TAIL_HDR + Bn + i] = (float)noisy_labels[i];
    tailf[DAD_TAIL_HDR + 2 * Bn + i] = noisy_mask[i] ? 1.0f : 0.0f;
  }
  if (i < (size_t)(B + Bn)) eflag[i] = 0u;
}

// loss = sum of the per-class terms (class-aware: ((t0 + t1) + t2) + t3, the reference's
// accumulation order; global MMD: t0), grads = the member rows dad_ecda wrote, zero elsewhere
__global__ __launch_bounds__(256) void dad_ecda_finish_kernel(int B, int Bn, const float* tailf, const float* ge,
                                                              const uint32_t* eflag, float* loss, float* gclean,
                                                              float* gnoisy) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t nc = (size_t)B * DAD_H, nn = (size_t)Bn * DAD_H;
  if (i == 0 && loss) {
    const float* t = tailf + DAD_T_ECDA_TERM;
    *loss = ((t[0] + t[1]) + t[2]) + t[3];
  }
  if (gclean && i < nc) gclean[i] = eflag[i / DAD_H] ? ge[i] : 0.0f;
  if (gnoisy && i < nn) gnoisy[i] = eflag[B + i / DAD_H] ? ge[nc + i] : 0.0f;
}
