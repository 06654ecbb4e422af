// Parameter update: global-norm clip + Adam (L2 weight decay) + teacher EMA + DACP commit.
//
//   torch.nn.utils.clip_grad_norm_(model.parameters(), MAX_GRAD_NORM)   I/train.py:487-488
//   optim.Adam(weight_decay=1e-5).step()  (single-tensor algorithm)       I/train.py:362,489
//   SSRLModel.update_teacher_ema()         (post-warm-up only)           I/model.py:211-223
//   DACPManager state: ema_thresholds EMA + epoch score collection        I/utils.py:485-505
//
// One elementwise pass over the flat [W1|b1|W2|b2] vectors; every block re-derives the
// clip coefficient from the same squared-norm partials in the same order, so the result
// is identical across blocks (and across data-parallel ranks).  The 16-bit shadows of W1
// used by the FP16/BF16 forward (fp16 when the step's precision is FP16, else bf16) are
// refreshed in the same pass.
#include "dad_common.h"
#include "dad_kernels.h"

// DACP state commit (thresholds were computed against the pre-step state by dad_tail;
// with data parallelism the floored thresholds are the rank mean): tau EMA and the epoch
// score collection of calculate_mask (I/utils.py:485-505).  Threads 0..C-1.
__device__ __forceinline__ void dacp_commit(const dad_config& cfg, const float* grad, float* d, int tid) {
  if (tid < DAD_C && !cfg.warmup && cfg.use_dacp) {
    const float* ex = grad + DAD_NPARAM;
    d[tid] = cfg.dacp_alpha * d[tid] + cfg.dacp_one_m_alpha * ex[tid];
    d[8 + tid] += ex[4 + tid];
    d[12 + tid] += ex[8 + tid];
  }
}

// train_step without the update (the caller runs clip / optimizer.step / EMA itself,
// I/train.py:486-492): commit the DACP state and publish this step's losses.
__global__ void dad_commit_kernel(dad_config cfg, const float* grad, float* dacp, float* tailf, float* losses_out) {
  const int tid = threadIdx.x;
  const float* ex = grad + DAD_NPARAM;
  if (tid == 0) tailf[DAD_T_TOTAL] = ex[12];
  if (losses_out && tid < 4) losses_out[tid] = ex[12 + tid];
  dacp_commit(cfg, grad, dacp, tid);
}

// Elementwise clip + Adam + EMA over this block's 1024 parameters, 4 per thread
// (i = n0 + 256k + tid).  The operands are loaded before the clip coefficient is known, so
// the loads overlap the global-norm reduction; the stores follow once it is.
struct AdamOperands {
  float g[4], p[4], m[4], v[4], t[4];
};

__device__ __forceinline__ void adam_load(size_t n0, const float* __restrict__ grad, const float* __restrict__ student,
                                          const float* __restrict__ teacher, const float* __restrict__ exp_avg,
                                          const float* __restrict__ exp_avg_sq, AdamOperands& o) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t i = n0 + (size_t)k * 256 + tid;
    if (i >= DAD_NPARAM) break;
    o.g[k] = grad[i];
    o.p[k] = student[i];
    o.m[k] = exp_avg[i];
    o.v[k] = exp_avg_sq[i];
    o.t[k] = teacher[i];
  }
}

__device__ __forceinline__ void adam_ema_apply(const dad_config& cfg, float coef, size_t n0, const AdamOperands& o,
                                               float* __restrict__ student,
                                                float* __restrict__ teacher, float* __restrict__ exp_avg,
                                                float* __restrict__ exp_avg_sq, uint16_t* __restrict__ w1bf_s,
                                                uint16_t* __restrict__ w1bf_t, bool f16) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t i = n0 + (size_t)k * 256 + tid;
    if (i >= DAD_NPARAM) break;
    float g = o.g[k] * coef;
    float p = o.p[k];
    g = g + cfg.weight_decay * p;                               // grad.add(param, alpha=wd)
    float m = o.m[k];
    m = m + cfg.one_m_beta1 * (g - m);                          // exp_avg.lerp_(grad, 1-beta1)
    float v = o.v[k];
    v = v * cfg.beta2 + cfg.one_m_beta2 * g * g;                // mul_(beta2).addcmul_(g, g, 1-beta2)
    const float denom = sqrtf(v) / cfg.bc2_sqrt + cfg.adam_eps;
    p = p + (-cfg.lr_step_size) * (m / denom);                  // addcdiv_(m, denom, -step_size)
    exp_avg[i] = m;
    exp_avg_sq[i] = v;
    student[i] = p;
    float t = o.t[k];
    if (!cfg.warmup) {
      t = t * cfg.ema_m + p * cfg.ema_one_m;
      teacher[i] = t;
    }
    if (i < (size_t)DAD_H * DAD_D) {
      const uint32_t f = dad_w1frag_index((uint32_t)(i / DAD_D), (uint32_t)(i % DAD_D));
      w1bf_s[f] = dad_half_bits(p, f16);
      w1bf_t[f] = dad_half_bits(t, f16);
    }
  }
}

// The same update with 4 CONSECUTIVE parameters per thread (i = n0 + 4 tid .. +3; DAD_NPARAM and
// the W1 size are multiples of 4): one 16-B load per stream and one 16-B store per written stream,
// and the 4 16-bit shadow values of a thread are 4 consecutive k of one h, i.e. 8 contiguous bytes
// of the fragment-major shadow (dad_w1frag_index: k & 7 is the innermost index).  The scalar
// form issued 20 loads and 24 stores per thread, 8 of them 2-byte stores to scattered shadow
// slots; the kernel's length was set by issuing them.  Used when every stream is 16-B aligned.
static_assert(DAD_OPTIM_THREADS * 4 == 1024 && DAD_NPARAM % 4 == 0 && (DAD_H * DAD_D) % 1024 == 0,
              "dad_optim: 1024 parameters per block, 4 per thread, whole blocks of W1");
struct AdamOperands4 {
  f32x4 g, p, m, v, t;
};

__device__ __forceinline__ void adam_load4(size_t i0, const float* __restrict__ grad, const float* __restrict__ student,
                                           const float* __restrict__ teacher, const float* __restrict__ exp_avg,
                                           const float* __restrict__ exp_avg_sq, AdamOperands4& o) {
  const size_t i = i0 < DAD_NPARAM ? i0 : 0;   // (clamped: the tail block's spare threads load a valid row)
  o.g = *reinterpret_cast<const f32x4*>(grad + i);
  o.p = *reinterpret_cast<const f32x4*>(student + i);
  o.m = *reinterpret_cast<const f32x4*>(exp_avg + i);
  o.v = *reinterpret_cast<const f32x4*>(exp_avg_sq + i);
  o.t = *reinterpret_cast<const f32x4*>(teacher + i);
}

__device__ __forceinline__ void adam_ema_apply4(const dad_config& cfg, float coef, size_t i0, uint32_t f,
                                                const AdamOperands4& o, float* __restrict__ student,
                                                float* __restrict__ teacher, float* __restrict__ exp_avg,
                                                float* __restrict__ exp_avg_sq, uint16_t* __restrict__ w1bf_s,
                                                uint16_t* __restrict__ w1bf_t, bool f16) {
  if (i0 >= DAD_NPARAM) return;
  f32x4 mo, vo, po, to;
#pragma unroll
  for (int e = 0; e < 4; ++e) {   // adam_ema_apply's arithmetic, element by element
    float g = o.g[e] * coef;
    float p = o.p[e];
    g = g + cfg.weight_decay * p;
    float m = o.m[e];
    m = m + cfg.one_m_beta1 * (g - m);
    float v = o.v[e];
    v = v * cfg.beta2 + cfg.one_m_beta2 * g * g;
    const float denom = sqrtf(v) / cfg.bc2_sqrt + cfg.adam_eps;
    p = p + (-cfg.lr_step_size) * (m / denom);
    mo[e] = m;
    vo[e] = v;
    po[e] = p;
    to[e] = o.t[e] * cfg.ema_m + p * cfg.ema_one_m;
  }
  *reinterpret_cast<f32x4*>(exp_avg + i0) = mo;
  *reinterpret_cast<f32x4*>(exp_avg_sq + i0) = vo;
  *reinterpret_cast<f32x4*>(student + i0) = po;
  if (!cfg.warmup) *reinterpret_cast<f32x4*>(teacher + i0) = to;
  const f32x4 tt = cfg.warmup ? o.t : to;
  if (i0 < (size_t)DAD_H * DAD_D) {
    const uint2 bs = f16 ? uint2{dad_pack2<true>(po[0], po[1]), dad_pack2<true>(po[2], po[3])}
                         : uint2{dad_pack2<false>(po[0], po[1]), dad_pack2<false>(po[2], po[3])};
    const uint2 bt = f16 ? uint2{dad_pack2<true>(tt[0], tt[1]), dad_pack2<true>(tt[2], tt[3])}
                         : uint2{dad_pack2<false>(tt[0], tt[1]), dad_pack2<false>(tt[2], tt[3])};
    *reinterpret_cast<uint2*>(w1bf_s + f) = bs;
    *reinterpret_cast<uint2*>(w1bf_t + f) = bt;
  }
}

// W1 parameter of shadow position f (f % 4 == 0: 4 consecutive k of one h), the inverse of
// dad_w1frag_index: f = ((((h>>4)*24 + ks)*64) + (h & 15) + 16q)*8 + j, k = 32ks + 8q + j.
// The 4-per-thread W1 blocks walk the SHADOW in order: a wave writes 512 contiguous shadow bytes
// and a block 1024 consecutive fragment slots = 16 h x 64 k, i.e. whole 128-B lines of every
// fp32 stream too.  (Walking the parameters in order wrote each shadow line as 16-B pieces from 8
// blocks, partial lines left dirty in several XCD L2s: the optimizer's kernel-end writeback then
// held the next launch ~5 us, measured as the optim -> encoder gap.)
__device__ __forceinline__ size_t w1_param_of_frag(uint32_t f) {
  const uint32_t j = f & 7u, lane = (f >> 3) & 63u, r2 = f >> 9;
  const uint32_t n = lane & 15u, q = lane >> 4, ks = r2 % 24u, ht = r2 / 24u;
  return (size_t)(16u * ht + n) * DAD_D + 32u * ks + 8u * q + j;
}

__global__ __launch_bounds__(DAD_OPTIM_THREADS) void dad_optim(DadOptimArgs a) {
  DAD_GUARD_BLOCK(DAD_OPTIM_THREADS);
  const dad_config& cfg = a.cfg;
  const int tid = threadIdx.x;
  const size_t n0 = (size_t)blockIdx.x * 1024;
  // 16-B aligned streams (the step's flat buffers): 4 consecutive parameters per thread
  const bool vec = ((reinterpret_cast<uintptr_t>(a.grad) | reinterpret_cast<uintptr_t>(a.student) |
                     reinterpret_cast<uintptr_t>(a.teacher) | reinterpret_cast<uintptr_t>(a.exp_avg) |
                     reinterpret_cast<uintptr_t>(a.exp_avg_sq)) & 15u) == 0;
  AdamOperands o;
  AdamOperands4 o4;
  // vector path: W1 blocks walk the shadow's fragment order (w1_param_of_frag), the rest linearly
  const uint32_t f4 = (uint32_t)(n0 + 4 * (size_t)tid);
  const size_t i4 = n0 < (size_t)DAD_H * DAD_D ? w1_param_of_frag(f4) : n0 + 4 * (size_t)tid;
  if (vec) adam_load4(i4, a.grad, a.student, a.teacher, a.exp_avg, a.exp_avg_sq, o4);
  else adam_load(n0, a.grad, a.student, a.teacher, a.exp_avg, a.exp_avg_sq, o);
  // global norm from the squared-norm partials: EVERY wave sums all of them in the same fixed
  // order (lane-strided, then the wave reduction), so every wave of every block derives the
  // same clip coefficient with no LDS round trip or barrier
  const int lane = tid & 63;
  constexpr int NJ = (DAD_REDUCE_BLOCKS + 63) / 64;   // (nnorm <= DAD_REDUCE_BLOCKS: one batch of loads)
  float pv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) pv[j] = a.normpart[min(lane + 64 * j, a.nnorm - 1)];
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) s += lane + 64 * j < a.nnorm ? (double)pv[j] : 0.0;
  for (int k = lane + 64 * NJ; k < a.nnorm; k += 64) s += (double)a.normpart[k];
  s = dad_wave_sum_d(s);
  const float norm = (float)sqrt(s);
  float coef = 1.0f;
  if (cfg.clip) coef = fminf(cfg.max_norm / (norm + 1e-6f), 1.0f);
  if (blockIdx.x == 0 && tid == 0) {
    a.tailf[DAD_T_CLIPNORM] = norm;
    a.tailf[DAD_T_CLIPCOEF] = coef;
    const float* ex = a.grad + DAD_NPARAM;
    a.tailf[DAD_T_TOTAL] = ex[12];
    if (a.losses_out)
      for (int k = 0; k < 4; ++k) a.losses_out[k] = ex[12 + k];
  }
  // a non-finite total loss (NaN from a pooling timeout in the tail launch, DAD_POOL_ABORT; or an
  // FP16 operand overflow / non-finite inputs) leaves this step's parameters, moments, teacher,
  // shadows and DACP state untouched; the losses and the clip fields above still report it (the
  // reference would write NaN into all of them)
  const float total = a.grad[DAD_NPARAM + 12];
  if (!(fabsf(total) <= 3.402823466e38f)) return;
  if (blockIdx.x == 0) dacp_commit(cfg, a.grad, a.dacp, tid);
  const bool f16 = cfg.precision == DAD_PREC_FP16;
  if (vec)
    adam_ema_apply4(cfg, coef, i4, f4, o4, a.student, a.teacher, a.exp_avg, a.exp_avg_sq, a.w1h_student,
                    a.w1h_teacher, f16);
  else
    adam_ema_apply(cfg, coef, n0, o, a.student, a.teacher, a.exp_avg, a.exp_avg_sq, a.w1h_student, a.w1h_teacher,
                   f16);
}

// DACPManager.update_class_quality_scores_epoch (I/utils.py:430-447)
__global__ void dad_epoch_end_kernel(float* dacp, float beta, float one_m_beta) {
  const int c = threadIdx.x;
  if (c >= DAD_C) return;
  const float n = dacp[12 + c];
  const float cur = n > 0.0f ? dacp[8 + c] / n : dacp[4 + c];
  dacp[4 + c] = beta * dacp[4 + c] + one_m_beta * cur;
  dacp[8 + c] = 0.0f;
  dacp[12 + c] = 0.0f;
}

__global__ __launch_bounds__(256) void dad_shadow_kernel(const float* student, const float* teacher, uint16_t* ws,
                                                         uint16_t* wt, int f16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (size_t)DAD_H * DAD_D) {
    const uint32_t f = dad_w1frag_index((uint32_t)(i / DAD_D), (uint32_t)(i % DAD_D));
    ws[f] = dad_half_bits(student[i], f16 != 0);
    wt[f] = dad_half_bits(teacher[i], f16 != 0);
  }
}

__global__ __launch_bounds__(256) void dad_ema_kernel(const float* student, float* teacher, size_t n, float m,
                                                      float one_m) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) teacher[i] = teacher[i] * m + student[i] * one_m;
}

extern "C" int dad_teacher_ema(const float* student, float* teacher, size_t n, float ema_m, float ema_one_m,
                               void* stream) {
  if (!student || !teacher) return DAD_E_ARG;
  if (n == 0) return DAD_OK;
  hipLaunchKernelGGL(dad_ema_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, student,
                     teacher, n, ema_m, ema_one_m);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DAD_OK : (int)e;
}
