// Eval path head: the classifier of SSRLModel.predict in eval mode and
// the per-utterance quantities validation and anchor calibration read from it.
//
// Replaces, per batch:
//   logits = classifier(embedding)                     I/model.py:225-245 (eval: dropout off)
//   probs  = F.softmax(logits, dim=1)                  I/train.py:333,340
//   scores, preds = DACPManager.calculate_certainty_scores(probs)   I/utils.py:401-430
//   _, predicted = torch.max(outputs, 1)               I/train.py:530
// The embeddings come from the encoder forward (dad_encoder_forward); this kernel is one wave
// per utterance: 256 hidden units x 4 classes as 4 floats per lane, a DPP wave reduction per
// class, then the softmax / entropy / argmax of 4 values on lane 0.  Latency-bound, ~0 bytes.
#include "dad_common.h"
#include "dad_kernels.h"

namespace {

constexpr int kEvalWaves = 4;

__global__ __launch_bounds__(64 * kEvalWaves) void dad_predict_head_kernel(const float* e, int B, const float* w2,
                                                                            const float* b2, int use_entropy,
                                                                            float* logits, float* probs, float* score,
                                                                            int64_t* pred) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * kEvalWaves + (int)(threadIdx.x >> 6);
  if (b >= B) return;
  const f32x4 x = *reinterpret_cast<const f32x4*>(e + (size_t)b * DAD_H + 4 * lane);
  float z[DAD_C];
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) {
    const f32x4 w = *reinterpret_cast<const f32x4*>(w2 + (size_t)c * DAD_H + 4 * lane);
    float p = x[0] * w[0];
    p = fmaf(x[1], w[1], p);
    p = fmaf(x[2], w[2], p);
    p = fmaf(x[3], w[3], p);
    z[c] = dad_wave_sum(p) + b2[c];
  }
  if (lane != 0) return;
  // softmax (max-subtracted, as torch) and torch.max's first maximal index
  float m = z[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < DAD_C; ++c)
    if (z[c] > m) { m = z[c]; am = c; }
  float ex[DAD_C], s = 0.0f;
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) { ex[c] = expf(z[c] - m); s += ex[c]; }
  float p[DAD_C], pmax = 0.0f, ent = 0.0f;
#pragma unroll
  for (int c = 0; c < DAD_C; ++c) {
    p[c] = ex[c] / s;
    pmax = fmaxf(pmax, p[c]);
    ent -= p[c] * log2f(p[c] + 1e-8f);            // I/utils.py:417
  }
  if (logits) {
#pragma unroll
    for (int c = 0; c < DAD_C; ++c) logits[(size_t)b * DAD_C + c] = z[c];
  }
  if (probs) {
#pragma unroll
    for (int c = 0; c < DAD_C; ++c) probs[(size_t)b * DAD_C + c] = p[c];
  }
  // I/utils.py:420-427: max_prob * (1 - H / log2(C)), or max_prob alone
  if (score) score[b] = use_entropy ? pmax * (1.0f - ent / 2.0f) : pmax;
  if (pred) pred[b] = am;
}

}  // namespace

extern "C" int dad_predict_head(const float* e, int B, const float* w2, const float* b2, int use_entropy,
                                float* logits, float* probs, float* score, int64_t* pred, void* stream) {
  if (!e || !w2 || !b2) return DAD_E_ARG;
  if (B <= 0) return DAD_E_SHAPE;
  hipLaunchKernelGGL(dad_predict_head_kernel, dim3((unsigned)((B + kEvalWaves - 1) / kEvalWaves)),
                     dim3(64 * kEvalWaves), 0, (hipStream_t)stream, e, B, w2, b2, use_entropy, logits, probs, score,
                     pred);
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? DAD_OK : (int)err;
}
