// The reference's DAD helper types as C-ABI operators (I/utils.py:317-652), for trainer code
// that drives them directly instead of the fused step:
//
//   DataAugmentation.weak_augment / strong_augment     dad_augment           I/utils.py:317-375
//   DACPManager.calculate_certainty_scores              dad_certainty_scores  I/utils.py:400-428
//   DACPManager.calculate_mask (+ its state update)     dad_dacp_mask         I/utils.py:449-507
//   ECDALoss.forward (+ its embedding gradients)        dad_ecda_loss         I/utils.py:510-652
//
// Each runs the device functions of the fused step (dad_common.h's augmentation draws,
// tail.hip's certainty / thresholds / ECDA class blocks), so the helpers and the step agree.
#include <string.h>

#include <algorithm>

#include "dad_common.h"
#include "dad_kernels.h"

namespace {

#define DAD_TRY(expr)                           \
  do {                                          \
    hipError_t e_ = (expr);                     \
    if (e_ != hipSuccess) return (int)e_;       \
  } while (0)

struct AugArgs {
  const float* x; float* out;
  uint64_t n;                 // B * T * D elements
  int T, D, strong, mask_len, start_hi;
  float sd, feat_p;
  uint32_t key_noise, key_feat, key_tstart;
  const float* noise; const float* u; const int64_t* start;
};

// One thread per element pair (2i, 2i+1): the pair shares one Box-Muller hash, as in the
// encoders, so element e of the [B][T][D] tensor draws normal (e & 1) of pair e >> 1 -- with
// D = 768 exactly the values the fused step adds to row b*T + t.
__global__ __launch_bounds__(256) void dad_augment_kernel(AugArgs a) {
  const uint64_t pair = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t e0 = 2 * pair;
  if (e0 >= a.n) return;
  float z[2];
  if (!a.noise) dad_aug_noise_pair(a.key_noise, (uint32_t)pair, a.sd, z[0], z[1]);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t e = e0 + k;
    if (e >= a.n) break;
    const float nz = a.noise ? a.noise[e] * a.sd : z[k];     // randn_like(x) * std (I/utils.py:330,338)
    float v = a.x[e] + nz;
    if (a.strong) {
      const int d = (int)(e % (uint64_t)a.D);
      const uint64_t row = e / (uint64_t)a.D;
      if (a.feat_p > 0.0f) v = v * dad_feat_keep(a.u, a.key_feat, d, a.feat_p);   // I/utils.py:342-344
      if (a.mask_len > 0) {                                                         // I/utils.py:352-375
        const int b = (int)(row / (uint64_t)a.T), t = (int)(row % (uint64_t)a.T);
        const int st = a.start ? (int)a.start[b] : dad_tstart_at(a.key_tstart, b, a.start_hi);
        if (t >= st && t < st + a.mask_len) v = 0.0f;
      }
    }
    a.out[e] = v;
  }
}

}  // namespace

extern "C" {

int dad_augment(const float* x, int B, int T, int D, int strong, float noise_std, float feat_p, int mask_len,
                uint64_t seed, uint64_t counter, const float* noise, const float* u, const int64_t* start, float* out,
                void* stream) {
  if (!x || !out || B < 0 || T < 1 || D < 1 || mask_len < 0 || mask_len > T) return DAD_E_ARG;
  const uint64_t n = (uint64_t)B * (uint64_t)T * (uint64_t)D;
  if (n == 0) return DAD_OK;
  if (n / 2 + 1 > 0xffffffffull) return DAD_E_SHAPE;   // 32-bit pair index of the counter stream
  AugArgs a;
  memset(&a, 0, sizeof(a));
  a.x = x; a.out = out; a.n = n; a.T = T; a.D = D; a.strong = strong ? 1 : 0;
  a.mask_len = strong ? mask_len : 0;
  a.start_hi = T - mask_len + 1 > 1 ? T - mask_len + 1 : 1;      // randint(0, max(1, T - mlen + 1))
  a.sd = noise_std; a.feat_p = strong ? feat_p : 0.0f;
  a.key_noise = dad_stream_key(seed, counter, strong ? DAD_RNG_STRONG : DAD_RNG_WEAK);
  a.key_feat = dad_stream_key(seed, counter, DAD_RNG_FEAT);
  a.key_tstart = dad_stream_key(seed, counter, DAD_RNG_TSTART);
  a.noise = noise; a.u = u; a.start = start;
  const uint64_t pairs = (n + 1) / 2;
  hipLaunchKernelGGL(dad_augment_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

int dad_certainty_scores(const float* probs, int B, int use_entropy, float* score, int64_t* pred, void* stream) {
  if (!probs || B < 0 || B > DAD_MAX_BATCH * 1024) return DAD_E_ARG;
  if (B == 0) return DAD_OK;
  hipLaunchKernelGGL(dad_certainty_kernel, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, probs, B,
                     use_entropy, score, pred);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

int dad_dacp_mask(const dad_config* cfg, const float* probs, int Bn, float* dacp, uint8_t* mask, float* score,
                  int64_t* pred, float* class_weights, void* stream) {
  if (!cfg || !probs || !dacp || !mask) return DAD_E_ARG;
  if (Bn < 1 || Bn > DAD_MAX_BATCH) return DAD_E_SHAPE;
  hipLaunchKernelGGL(dad_dacp_mask_kernel, dim3(1), dim3(DAD_TAIL_THREADS), 0, (hipStream_t)stream, *cfg, probs, Bn,
                     dacp, mask, score, pred, class_weights);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

size_t dad_ecda_workspace_bytes(int B, int Bn) {
  if (B < 0 || Bn < 0) return 0;
  const size_t nb = (size_t)B + Bn;
  size_t off = 0;
  off = dad_align(off + sizeof(float) * ((size_t)B + 2 * (size_t)Bn) * DAD_H);   // emb
  off = dad_align(off + sizeof(float) * DAD_TAIL_FLOATS((size_t)Bn));            // tail
  off = dad_align(off + sizeof(float) * nb * DAD_H);                             // ge
  off = dad_align(off + sizeof(uint32_t) * nb);                                  // eflag
  off = dad_align(off + sizeof(float) * DAD_C * nb * nb);                        // scratch
  return off;
}

int dad_ecda_loss(const dad_config* cfg, const float* clean, int B, const float* noisy, int Bn,
                  const int64_t* clean_labels, const int64_t* noisy_labels, const uint8_t* noisy_mask,
                  const float* noisy_scores, const float* class_weights, int n_weights, float* loss,
                  float* grad_clean, float* grad_noisy, void* workspace, void* stream_) {
  if (!cfg || !clean || !noisy || !clean_labels || !noisy_labels || !noisy_mask || !noisy_scores || !class_weights ||
      !loss || !workspace)
    return DAD_E_ARG;
  if (B < 1 || Bn < 1 || B > DAD_MAX_BATCH || Bn > DAD_MAX_BATCH) return DAD_E_SHAPE;
  // class_weights: DACP's [C] weights, or the fixed-threshold branch's ones(Bn) (I/train.py:420)
  if (n_weights != DAD_C && n_weights != Bn) return DAD_E_ARG;
  hipStream_t stream = (hipStream_t)stream_;
  const size_t nb = (size_t)B + Bn;
  char* ws = reinterpret_cast<char*>(workspace);
  size_t off = 0;
  float* emb = reinterpret_cast<float*>(ws + off); off = dad_align(off + sizeof(float) * ((size_t)B + 2 * (size_t)Bn) * DAD_H);
  float* tailf = reinterpret_cast<float*>(ws + off); off = dad_align(off + sizeof(float) * DAD_TAIL_FLOATS((size_t)Bn));
  float* ge = reinterpret_cast<float*>(ws + off); off = dad_align(off + sizeof(float) * nb * DAD_H);
  uint32_t* eflag = reinterpret_cast<uint32_t*>(ws + off); off = dad_align(off + sizeof(uint32_t) * nb);
  float* scratch = reinterpret_cast<float*>(ws + off);
  const size_t nprep = std::max((size_t)std::max(B, Bn) * DAD_H, (size_t)DAD_TAIL_HDR);
  hipLaunchKernelGGL(dad_ecda_prep_kernel, dim3((unsigned)((nprep + 255) / 256)), dim3(256), 0, stream, clean, B, noisy,
                     Bn, noisy_labels, noisy_mask, noisy_scores, class_weights, n_weights, emb, tailf, eflag);
  DAD_TRY(hipGetLastError());
  DadEcdaArgs ca;
  memset(&ca, 0, sizeof(ca));
  ca.cfg = *cfg;
  ca.cfg.B = B; ca.cfg.Bn = Bn; ca.cfg.warmup = 0; ca.cfg.ecda_on = 1;
  ca.cfg.w_ecda = 1.0f;                             // grads of the unweighted loss
  // ones(Bn) weights: the class loop of the fixed-threshold branch (unit attention, classes < Bn)
  ca.cfg.use_dacp = n_weights == DAD_C ? 1 : 0;
  ca.yc = clean_labels; ca.emb = emb; ca.tailf = tailf; ca.tail_terms = tailf + DAD_T_ECDA_TERM;
  ca.ge = ge; ca.eflag = eflag; ca.scratch = scratch;
  hipLaunchKernelGGL(dad_ecda, dim3(DAD_C), dim3(DAD_ECDA_THREADS), 0, stream, ca);
  DAD_TRY(hipGetLastError());
  const size_t nfin = std::max((size_t)std::max(B, Bn) * DAD_H, (size_t)1);
  hipLaunchKernelGGL(dad_ecda_finish_kernel, dim3((unsigned)((nfin + 255) / 256)), dim3(256), 0, stream, B, Bn, tailf,
                     ge, eflag, loss, grad_clean, grad_noisy);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

}  // extern "C"
