// Kernel argument blocks and entry points (internal to libdad_hip.so).
#pragma once
#include "dad_common.h"

// Block sizes: kernels index with these, launches use them; every kernel whose indexing
// depends on its block size exits uniformly if launched with another one.
#define DAD_ENC_F32_THREADS 256
#define DAD_ENC_WS_THREADS 512                               // W-stationary 16-bit encoder (8 waves, two per SIMD)
#define DAD_ENC_WS_MAXJ 256                                  // max 32-row jobs per encoder workgroup
#define DAD_POOL_THREADS 64
#define DAD_TAIL_THREADS 512
#define DAD_ECDA_THREADS 512
// 1: the tail and ECDA run as one launch (dad_tail_ecda): block 0 is the tail, blocks 1..C
// re-derive the DACP mask themselves and go straight on to ECDA (no kernel boundary and no
// round trip of the mask through HBM).  0: dad_tail then dad_ecda (A/B builds).
#ifndef DAD_FUSED_TAIL
#define DAD_FUSED_TAIL 1
#endif
#define DAD_WGRAD_THREADS 256
// dad_wgrad_direct (FP16/BF16): 64-column blocks, slab-range splits of at most WGD_MAXU slabs,
// WGD_DEPTH slabs in flight per group, x tile row pitch WGD_XP halves (192 B)
#define WGD_DB 64
#define WGD_NDB (DAD_D / WGD_DB)
#define WGD_MAXU 64
#ifndef WGD_DEPTH
#define WGD_DEPTH 4       // slabs whose loads are in flight per group
#endif
#define WGD_XP 96
#ifndef WGD_GROUPS
#define WGD_GROUPS 2      // slab groups of 4 waves per workgroup (2: two waves per SIMD)
#endif
#define WGD_THREADS (256 * WGD_GROUPS)
#define WGD_XWG 4         // spare dad_wgrad_direct workgroups that run dad_reduce's extra blocks
#define DAD_REDUCE_THREADS 256
#define DAD_REDUCE_COLS 256                                  // dW1 floats per reduce block
#define DAD_REDUCE_XBLK 16                                   // db1 / dW2 / totals blocks (16 hidden units each)
#define DAD_REDUCE_BLOCKS (DAD_H * DAD_D / DAD_REDUCE_COLS + DAD_REDUCE_XBLK)
#define DAD_OPTIM_THREADS 256
#define DAD_COLLATE_THREADS 256                              // device collate (4 waves, 2 rows each)
#define DAD_GUARD_BLOCK(n) \
  if (blockDim.x != (n) || blockDim.y != 1 || blockDim.z != 1) return

#define DAD_POOL_SHARDS 8   // fused-pooling arrival counters, one per XCD (128 B apart)
// the word after them (ready + 32 * DAD_POOL_SHARDS): 1 when a tail / class block of this step gave up
// waiting for the pooling (pool_wait); zeroed with the counters by the step's encoder.  The weight
// gradient's loss-total block then writes a NaN total loss, and dad_optim skips the update.
#define DAD_POOL_ABORT (32 * DAD_POOL_SHARDS)

struct DadPoolArgs {
  DadGeom g;
  int warmup;
  const uint8_t* mc; const uint8_t* mn;
  const float* part_sum;
  const float* student; const float* teacher;     // flat params (W2/b2 used)
  const uint8_t* keep1; const uint8_t* keep2;     // explicit dropout masks or NULL
  uint32_t key_drop1, key_drop2;
  float p_drop, drop_scale;
  float* emb; float* vlen; float* logits;
  const float* part_cnt; float* cnt_tot;
  uint32_t* eflag;        // [Bc+Bn] ECDA row flags, zeroed here (ECDA flags the rows it writes)
  float* tail_terms;      // per-class ECDA terms + gates, zeroed here (block 0)
  uint32_t* range_flag;   // sticky: set when a pooled embedding is not finite (tail header DAD_T_RANGE)
  uint32_t* ready;        // pooling fused into dad_tail_ecda_w: pool items done, DAD_POOL_SHARDS
                          // counters 128 B apart (zeroed by the step's encoder); NULL: the
                          // separate dad_pool launch
};

struct DadEncodeArgs {
  DadGeom g;
  int warmup, mask_len, start_hi;
  const float* xc; const uint8_t* mc;
  const float* xn; const uint8_t* mn;
  DadStoreRows src;         // store mode (dad_batch.rowc..lenn) or all NULL
  const float* w1_student; const float* b1_student;
  const float* w1_teacher; const float* b1_teacher;
  const uint16_t* w1h_student; const uint16_t* w1h_teacher;   // 16-bit W1 shadows (fragment-major)
  // explicit draws (parity mode) or NULL -> counter RNG
  const float* nw; const float* ns; const float* u; const int64_t* start;
  uint32_t key_weak, key_strong, key_feat, key_tstart;
  float weak_std, strong_std, feat_p;
  float* part_sum; float* part_cnt; uint32_t* bits;
  // dad_encode_wp roles (dad_wp_job_range): ws_nt teacher and ws_ns student workgroups
  int ws_nt, ws_ns;
  // the prepared 16-bit rows (dad_prep) of the clean, strong and weak branches, [B][T][768] each
  // (padded layout whatever the source mode)
  const uint16_t* x16c; const uint16_t* x16s; const uint16_t* x16w;
  uint32_t* pool_ready;     // workgroup 0 zeroes it: the counter of the tail launch's fused pooling
};

// The weight-independent half of the 16-bit encoder (prep.hip, dad_prep.h): augmentation
// (I/utils.py:328-375) and the 16-bit conversion of every row of one step, written as one
// "prepared set" [clean Bc*Tc | strong Bn*Tn | weak Bn*Tn][768] of 16-bit rows (padded layout).
// Runs standalone before the encoder, or -- for the NEXT step -- on the spare workgroups of the
// current step's tail launch (dad_tail_ecda_w blocks > DAD_C).
struct DadPrepArgs {
  DadGeom g;
  int warmup, mask_len, start_hi, f16;
  int clean;                // 1: also the clean rows (else the encoder converts them itself)
  const float* xc; const float* xn;
  DadStoreRows src;
  const float* nw; const float* ns; const float* u; const int64_t* start;   // explicit draws, or NULL
  uint32_t key_weak, key_strong, key_feat, key_tstart;
  float weak_std, strong_std, feat_p;
  uint16_t* x16;            // the set; NULL: nothing to prepare (tail launch without a next batch)
};


struct DadTailArgs {
  dad_config cfg;
  const int64_t* yc;
  const float* logits; const float* emb;
  const float* student;
  const uint8_t* keep1; const uint8_t* keep2;
  uint32_t key_drop1, key_drop2;
  float* dacp;            // persistent DACP state (read; committed by the optimizer kernel)
  float* tailf;           // per-step outputs (see DAD_TAIL_* in dad.h)
  float* ge;              // [Bc+Bn][H] dL/de (CE/KL part)
  float* ge_ecda;         // [Bc+Bn][H] modular path only (fused step: ge_ecda rows are flagged)
  float* gzb;             // [Bc+Bn][C] dL/dz per utterance (clean | strong)
  uint32_t* eflag;        // [Bc+Bn]    (zeroed by dad_pool; ECDA flags the rows it writes)
  float* grad;            // flat grads (W2, b2 written here) + extras
};

struct DadEcdaArgs {
  dad_config cfg;
  const int64_t* yc;
  const float* emb;
  const float* tailf;
  float* tail_terms;      // per-class loss terms
  float* ge;              // ECDA part of dL/de: member rows written (and flagged in eflag)
  uint32_t* eflag;
  float* scratch;         // global fallback for large member sets
  float* sink;            // dad_tail_ecda_w: [DAD_H] floats its unselected lanes store to
};

struct DadWgradArgs {
  DadGeom g;
  int warmup, splits, mask_len, start_hi;
  const float* xc; const float* xn;
  DadStoreRows src;
  const float* ns; const float* u; const int64_t* start;
  uint32_t key_strong, key_feat, key_tstart;
  float strong_std, feat_p;
  const uint32_t* bits; const float* ge; const float* vlen;
  const uint16_t* xs16;    // the encoder's 16-bit copies of the student's MFMA input
  float* wpart;
  int ntiles;          // column blocks x splits; workgroups stride over them (grid may be smaller)
};

struct DadReduceArgs {
  DadGeom g;
  int splits, warmup, want_norm;
  float w_kl, w_ecda;
  const float* wpart; const float* ge; const float* vlen; const float* cnt_tot;
  const float* ge_ecda;       // ECDA part of dL/de, added where eflag is set
  // fused step: dL/de is not materialised; the classifier part is rebuilt per (utterance, h)
  // as keep(u,h) * sum_c W2[c][h] gzb[u][c] (nn.Linear + dropout backward, I/model.py:62-63)
  const float* gzb; const uint32_t* eflag;
  const float* student; const float* emb;
  const uint8_t* keep1; const uint8_t* keep2;
  uint32_t key_drop1, key_drop2;
  float p_drop, drop_scale;
  const float* tailf;
  float* grad; float* normpart;
  const uint32_t* pool_abort;   // fused pooling: this step's abort word (DAD_POOL_ABORT), else NULL
};

struct DadOptimArgs {
  dad_config cfg;
  float* student; float* teacher; float* exp_avg; float* exp_avg_sq;
  float* grad; uint16_t* w1h_student; uint16_t* w1h_teacher;   // shadows: fp16 if cfg.precision is FP16, else bf16
  float* dacp; float* tailf; const float* normpart; int nnorm;
  float* losses_out;
};

// device-resident data path (collate.hip)
struct DadCollateArgs {
  const void* store; int dtype;
  const int64_t* offsets; const int32_t* sizes; long n_samples;
  const int64_t* index; int B, T;
  float* feats; uint8_t* pad;
  const int64_t* labels_in; int64_t* labels_out;
};

__global__ void dad_collate_kernel(DadCollateArgs a);
int dad_collate_grid(long B, long T);
__global__ void dad_encode_f32(DadEncodeArgs a);
__global__ void dad_encode_wp(DadEncodeArgs a);                // bf16 operands from a prepared set
__global__ void dad_encode_wp_f16(DadEncodeArgs a);            // fp16 operands from a prepared set
#define DAD_PREP_THREADS 256
__global__ void dad_prep(DadPrepArgs a);                       // one prepared set, standalone
__global__ void dad_pool(DadPoolArgs a);
__global__ void dad_tail(DadTailArgs a);
__global__ void dad_ecda(DadEcdaArgs a);
__global__ void dad_tail_ecda(DadTailArgs ta, DadEcdaArgs ca);
// B, Bn <= 64, class-aware; blocks > DAD_C pool the step's embeddings first (pl.ready != NULL)
// and then prepare the next step's set (pa.x16 != NULL)
__global__ void dad_tail_ecda_w(DadTailArgs ta, DadEcdaArgs ca, DadPrepArgs pa, DadPoolArgs pl);
__global__ void dad_wgrad_f32(DadWgradArgs a, DadReduceArgs r);   // r: the fused step's dL/de sources (gzb) or zeroed
__global__ void dad_wgrad_direct(DadWgradArgs a, DadReduceArgs r);       // bf16 operands
__global__ void dad_wgrad_direct_f16(DadWgradArgs a, DadReduceArgs r);   // fp16 operands
// the same, also converting the NEXT step's clean rows into its prepared set (dad_prep.h, pc.clean)
__global__ void dad_wgrad_direct_cp(DadWgradArgs a, DadReduceArgs r, DadPrepArgs pc);
__global__ void dad_wgrad_direct_f16_cp(DadWgradArgs a, DadReduceArgs r, DadPrepArgs pc);
// store-batch variants (the next batch's clean rows gathered from a FeatureStore, Bc <= 64)
__global__ void dad_wgrad_direct_cps(DadWgradArgs a, DadReduceArgs r, DadPrepArgs pc);
__global__ void dad_wgrad_direct_f16_cps(DadWgradArgs a, DadReduceArgs r, DadPrepArgs pc);
__global__ void dad_reduce(DadReduceArgs a);
__global__ void dad_reduce_w(DadReduceArgs a);
__global__ void dad_norm(float* grad, float* normpart, float inv_world);
__global__ void dad_optim(DadOptimArgs a);
__global__ void dad_commit_kernel(dad_config cfg, const float* grad, float* dacp, float* tailf, float* losses_out);
__global__ void dad_epoch_end_kernel(float* dacp, float beta, float one_m_beta);
__global__ void dad_shadow_kernel(const float* student, const float* teacher, uint16_t* ws, uint16_t* wt, int f16);
// helper-type drop-ins (DACPManager / ECDALoss, tail.hip; DataAugmentation, utils_abi.hip)
__global__ void dad_certainty_kernel(const float* probs, int B, int use_entropy, float* score, int64_t* pred);
__global__ void dad_dacp_mask_kernel(dad_config cfg, const float* probs, int Bn, float* dacp, uint8_t* mask,
                                     float* score, int64_t* pred, float* wout);
__global__ void dad_ecda_prep_kernel(const float* clean, int B, const float* noisy, int Bn, const int64_t* noisy_labels,
                                     const uint8_t* noisy_mask, const float* noisy_scores, const float* class_weights,
                                     int nw, float* emb, float* tailf, uint32_t* eflag);
__global__ void dad_ecda_finish_kernel(int B, int Bn, const float* tailf, const float* ge, const uint32_t* eflag,
                                       float* loss, float* gclean, float* gnoisy);

// offsets inside the flat parameter vector [W1 | b1 | W2 | b2]
#define DAD_OFF_W1 0
#define DAD_OFF_B1 (DAD_H * DAD_D)
#define DAD_OFF_W2 (DAD_OFF_B1 + DAD_H)
#define DAD_OFF_B2 (DAD_OFF_W2 + DAD_C * DAD_H)
