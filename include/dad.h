/*
 * dad.h — C ABI of the MI355X-native DAD (Dynamic Asymmetric Distillation) train step.
 *
 * The reference (TMZZ22331/Robust-Speech-Emotion-Recognition-via-Dynamic-Asymmetric-
 * Distillation-in-Noisy-Environments) is pure Python/PyTorch with no FFI; its operator
 * surface for the hot path is the Python object API listed in SURVEY.md §8(b).  Each
 * entry point below names the reference interface it replaces (I/ = IEMOCAP/DAD-train-
 * IEMOCAP/, identical in CASIA/ and EMODB/ up to the differences resolved by dad_config).
 *
 * Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller (PyTorch tensors in the
 *     Python host layer); sizes are explicit; no allocation, no host synchronisation,
 *     enqueue-only on `stream` (a hipStream_t), graph-capturable;
 *   - return 0 on success, a hipError_t value, or a DAD_E_* code; no exceptions cross;
 *   - reentrant across streams; not thread-safe on one shared state.
 *   - fixed model dims: INPUT_DIM 768, HIDDEN_DIM 256, NUM_CLASSES 4 (I/config.py:54-56).
 */
#ifndef DAD_ABI_H_
#define DAD_ABI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAD_ABI_VERSION 7

/* error codes (besides hipError_t values) */
#define DAD_OK 0
#define DAD_E_ARG 1001        /* null pointer / invalid scalar */
#define DAD_E_SHAPE 1002      /* B/T out of the supported range */
#define DAD_E_COMM 1003       /* RCCL failure */
#define DAD_E_UNSUPPORTED 1004

#define DAD_INPUT_DIM 768
#define DAD_HIDDEN_DIM 256
#define DAD_NUM_CLASSES 4
#define DAD_MAX_BATCH 1024
/* flat parameter vector [W1 (256x768) | b1 (256) | W2 (4x256) | b2 (4)] — the student
 * (or teacher) half of SSRLModel.parameters() (I/model.py:101-122) */
#define DAD_NPARAM (256 * 768 + 256 + 4 * 256 + 4)
/* per-step extras appended to the gradient buffer so ONE all-reduce carries them:
 * [0,4) DACP floored thresholds tau' (mean over ranks), [4,8) per-class certainty
 * sums, [8,12) per-class counts, [12,16) losses (total, ce, kl, ecda) */
#define DAD_GRAD_EXTRA 16
#define DAD_GRAD_FLOATS (DAD_NPARAM + DAD_GRAD_EXTRA)
/* persistent DACPManager state (I/utils.py:384-398): [0,4) tau (ema_thresholds),
 * [4,8) Q (class_quality_scores), [8,12) epoch score sums, [12,16) epoch counts,
 * [16,20) calibrated anchors */
#define DAD_DACP_FLOATS 20
#define DAD_NORM_BLOCKS 1024

/* per-step outputs ("tail" buffer): header then per-sample arrays */
#define DAD_TAIL_HDR 64
#define DAD_T_TOTAL 0
#define DAD_T_CE 1
#define DAD_T_KL 2
#define DAD_T_ECDA 3
#define DAD_T_SCL 4           /* always 0: C/train_CASIA.py:442, E/train_emodb.py:404 */
#define DAD_T_MSUM 5
#define DAD_T_CLIPNORM 6
#define DAD_T_CLIPCOEF 7
#define DAD_T_W 8             /* [4] DACP class weights W_c */
#define DAD_T_TAU_BEFORE 12   /* [4] */
#define DAD_T_TAU_AFTER 16    /* [4] */
#define DAD_T_FLOORED 20      /* [4] */
#define DAD_T_ECDA_TERM 24    /* [4] att_c * (mmd_c + gamma comp_c + delta rep) */
#define DAD_T_ECDA_GATE 28    /* [4] */
#define DAD_T_KL_ON 32
#define DAD_T_ECDA_ON 33
#define DAD_T_RANGE 34        /* u32 bits, sticky (only the caller clears them; the buffer starts zero-filled):
                                 DAD_RANGE_NONFINITE: a step's pooled embedding or logit was not finite (FP16: an
                                 encoder operand beyond +-65504; any mode: non-finite features);
                                 DAD_RANGE_POOL_TIMEOUT: a tail / class block gave up waiting for the tail
                                 launch's fused pooling (~0.2 s); that step's update was skipped (its total loss
                                 is NaN).  dad_step_apply skips the update of any step whose total loss is not finite. */
#define DAD_RANGE_NONFINITE 1u
#define DAD_RANGE_POOL_TIMEOUT 2u
#define DAD_T_TAU_HAT 40      /* [4] batch quantile thresholds */
/* after the header (noisy batch, Bn rows): score[Bn], pred[Bn] (as float), mask[Bn], q[Bn][4] */
#define DAD_TAIL_FLOATS(Bn) (DAD_TAIL_HDR + (Bn) * (3 + DAD_NUM_CLASSES))

/* FP32: exact-f32 MFMA (the reference's arithmetic, parity mode).  FP16 / BF16: the encoder and
 * weight-gradient GEMMs on 16-bit operands (fp16: 11-bit significand, the throughput mode that
 * meets the 1e-4 loss/logit bound; bf16: 8-bit) with fp32 accumulation; everything else fp32. */
enum dad_precision { DAD_PREC_FP32 = 0, DAD_PREC_BF16 = 1, DAD_PREC_FP16 = 2 };
enum dad_rng_mode { DAD_RNG_EXPLICIT = 0, DAD_RNG_COUNTER = 1 };

/* Every scalar the step reads from the reference's config module, resolved by the host
 * at CALL time (the reference re-reads config inside the functions, I/utils.py:410,567,
 * and the ablation runners mutate it between runs, I/run_granular_ablations.py:25-30).
 * Float scalars are the float32 values torch would use for the python-float operands. */
typedef struct dad_config {
  int32_t B, T;                 /* clean batch: utterances, padded frames (batch max length) */
  int32_t Bn, Tn;               /* noisy batch (collated independently, I/train.py:479-483) */
  int32_t precision;            /* dad_precision */
  int32_t rng_mode;             /* dad_rng_mode */
  uint64_t seed, counter;       /* counter-RNG key material (counter = global step) */
  int32_t warmup;               /* epoch < WARMUP_EPOCHS: CE only, no EMA (I/train.py:402,491) */
  int32_t use_dacp;             /* DACP vs fixed threshold (I/train.py:414-420) */
  int32_t ecda_on;              /* USE_ECDA && weight_ecda > 0 (I/train.py:450) */
  int32_t use_entropy;          /* USE_ENTROPY_IN_SCORE (I/utils.py:415) */
  int32_t class_aware;          /* USE_CLASS_AWARE_MMD (I/utils.py:579) */
  int32_t dp_world;             /* ranks whose grads are all-reduced (1 = single GPU) */
  float w_kl, w_ecda;           /* update_loss_weights (I/train.py:380-395) */
  float dacp_gamma;             /* quantile level gamma_e (I/utils.py:471-473) */
  float dacp_k, dacp_lambda, dacp_alpha, dacp_one_m_alpha;
  float fixed_thr;              /* FIXED_CONFIDENCE_THRESHOLD */
  float ecda_att_lambda, ecda_gamma, ecda_delta;
  float ls_eps;                 /* label smoothing (I/train.py:364) */
  float p_drop, drop_scale;     /* classifier dropout p, float32(1)/float32(1-p) */
  float feat_p;                 /* strong-aug feature dropout rate (I/utils.py:325,343) */
  float weak_std, strong_std;
  int32_t mask_len, start_hi;   /* int(Tn*ratio), max(1, Tn-mask_len+1) (I/utils.py:365,370) */
  int32_t clip;                 /* GRADIENT_CLIPPING */
  float max_norm;
  float lr_step_size;           /* lr / (1 - beta1^t)      (torch Adam single-tensor) */
  float bc2_sqrt;               /* sqrt(1 - beta2^t) */
  float beta1, one_m_beta1, beta2, one_m_beta2, adam_eps, weight_decay;
  float ema_m, ema_one_m;       /* EMA_MOMENTUM, 1-EMA_MOMENTUM (I/model.py:219) */
  float dacp_beta, dacp_one_m_beta;   /* epoch-end quality smoothing (I/utils.py:433-436) */
  int32_t splits;               /* weight-gradient split-K factor (0 = auto) */
  int32_t prepped;              /* FP16/BF16: 1 = the previous step's dad_step_backward_ahead prepared this
                                   batch's 16-bit rows (it reported *prepped = 1 for this cfg and batch), so
                                   the encoder skips the preparation; 0 = prepare them in this step */
  int32_t reserved[4];
} dad_config;

/* One clean + one noisy collated batch (I/dataload_noisy.py:124-129 format). */
typedef struct dad_batch {
  const float* xc;              /* [B][T][768] clean features */
  const uint8_t* mc;            /* [B][T] padding mask, 1 = pad */
  const int64_t* yc;            /* [B] clean labels */
  const float* xn;              /* [Bn][Tn][768] noisy features */
  const uint8_t* mn;            /* [Bn][Tn] */
  /* DAD_RNG_EXPLICIT only (parity mode; NULL otherwise): the reference's six draws */
  const float* nw;              /* [Bn][Tn][768] randn for weak aug */
  const float* ns;              /* [Bn][Tn][768] randn for strong aug */
  const float* u;               /* [768] rand for feature dropout */
  const int64_t* start;         /* [Bn] temporal-mask starts */
  const uint8_t* keep1;         /* [B][256] classifier dropout keep mask, clean pass */
  const uint8_t* keep2;         /* [Bn][256] classifier dropout keep mask, strong pass */
  /* STORE MODE, per batch (rowc+lenc for the clean one, rown+lenn for the noisy one; NULL =
   * padded): xc / xn point at a feature store [frames][768] (FeatureStore, the device-
   * resident data path) instead of a padded [B][T][768] batch, and
   * frame t < T of utterance b is store row rowc[b] + min(t, lenc[b] - 1) (rown/lenn for the
   * noisy batch).  The encoder's LDS-DMA reads the rows in place: collation never copies the
   * features.  mc / mn / yc keep their [B][T] / [B] meaning (dad_collate_index builds them
   * together with rowc / lenc). */
  const int64_t* rowc;          /* [B] store row of frame 0 of each clean utterance */
  const int32_t* lenc;          /* [B] its frame count (rows >= it are padding) */
  const int64_t* rown;          /* [Bn] */
  const int32_t* lenn;          /* [Bn] */
} dad_batch;

/* Persistent training state, all caller-owned device buffers. */
typedef struct dad_state {
  float* student;               /* [DAD_NPARAM] */
  float* teacher;               /* [DAD_NPARAM] */
  float* exp_avg;               /* [DAD_NPARAM] Adam m */
  float* exp_avg_sq;            /* [DAD_NPARAM] Adam v */
  float* grad;                  /* [DAD_GRAD_FLOATS] grads (+extras); the DP all-reduce buffer */
  uint16_t* w1bf_student;       /* [256*768] 16-bit shadow of student W1 (fp16 in FP16 steps, else bf16) */
  uint16_t* w1bf_teacher;       /* [256*768] 16-bit shadow of teacher W1 */
  float* dacp;                  /* [DAD_DACP_FLOATS] */
  float* tail;                  /* [DAD_TAIL_FLOATS(Bn)] per-step outputs */
  float* emb;                   /* [B+2*Bn][256] e_clean [B], e_teacher [Bn], e_strong [Bn] */
  float* logits;                /* [B+2*Bn][4]   z_clean, z_teacher, z_strong */
  float* losses;                /* [4] (optional) total, ce, kl, ecda of this step (rank mean) */
} dad_state;

/* --- sizing ------------------------------------------------------------------------ */
/* DAD_ABI_VERSION the library was built with (ABI 7; 6 lacked dad_timing_reset): a binding compares it with the header's
 * value when it loads the library, so a stale build fails at load instead of at a call. */
int dad_abi_version(void);
size_t dad_param_count(void);
/* Step workspace bytes for cfg's geometry and precision (no initialisation needed). */
int dad_workspace_bytes(const dad_config* cfg, size_t* bytes);
const char* dad_error_string(int code);
/* Host-only planning of the 16-bit (FP16/BF16) encoder grid (no device call): teacher / student workgroups
 * for a device of `cus` compute units and the most 32-row jobs any workgroup's range holds
 * (always <= 256, the kernel's per-workgroup table).  Diagnostics and tests. */
int dad_encoder_ws_plan(const dad_config* cfg, int cus, int* nt, int* ns, int* max_jobs);
/* Host-only: the 16-bit encoder's job assignment for a device of `cus` CUs: for every workgroup
 * wg of the grid, jobs[4wg..4wg+3] = (teacher 1/0, first job, job stride, job count); student jobs
 * j < B*ceil(T/32) are clean slabs, the rest strong slabs.  `capacity` = ints available at jobs.
 * The grid is nt + ns of dad_encoder_ws_plan: usually `cus`, more when a range would exceed the
 * kernel's 256-job table (very long batches), so size jobs as 4 * (nt + ns).  Returns the grid
 * size (> 0), DAD_E_ARG when 4 * grid > capacity (nothing written), or another DAD_E_* code.
 * Diagnostics and tests.  (ABI 5: `capacity` added.) */
int dad_encoder_ws_jobs(const dad_config* cfg, int cus, int* jobs, int capacity);

/* --- fused train step ---------------------------------------------------------------
 * Replaces the body of Trainer.train_epoch's loop (I/train.py:484-492):
 *   train_step (I/train.py:397-471) + backward + clip_grad_norm_ + Adam.step + update_teacher_ema.
 * dad_step_compute: encoder passes, losses, DACP mask, analytic backward -> state->grad.
 * dad_step_apply:   global-norm clip, Adam (L2 decay), teacher EMA, DACP state commit,
 *                   16-bit W1 shadow refresh.  A DP caller all-reduces state->grad in between.
 * dad_step = compute + apply (single GPU). */
int dad_step_compute(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
                     void* workspace, void* stream);
/* dad_step_compute = dad_step_encode (the fused augmentation + three encoder GEMMs +
 * pooling partials, one launch) followed by dad_step_backward (pool, losses, DACP,
 * ECDA, analytic backward, weight gradient, reduction); split so callers can time the
 * encoder launch on their stream. */
int dad_step_encode(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
                    void* workspace, void* stream);
int dad_step_backward(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
                      void* workspace, void* stream);
/* dad_step_backward + the NEXT step's row preparation (FP16/BF16: the augmentation and 16-bit
 * conversion of next_batch under next_cfg, weight-independent) on the CUs this step's tail launch
 * leaves idle.  *prepped = 1 when it was enqueued: the next step then passes cfg->prepped = 1 with
 * the same next_cfg scalars and next_batch pointers, whose contents must not change in between.
 * *prepped = 0 (and nothing extra enqueued) unless: 16-bit precision, the tail runs as the
 * wave-centric launch (B, Bn <= 64, class-aware MMD), next_cfg has this cfg's geometry and
 * precision and the other counter parity.  Replaces nothing in the reference: its loop draws the
 * augmentation inside train_step (I/train.py:406-410,439); the draws are the same streams. */
int dad_step_backward_ahead(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
                            void* workspace, void* stream, const dad_config* next_cfg,
                            const dad_batch* next_batch, int* prepped);
/* dad_step_backward_ahead with parts of the next batch's rows left to the caller, for the data-parallel
 * step (ABI 6): `defer` (DAD_PREP_CLEAN and/or DAD_PREP_NOISY) names the parts this step's launches skip
 * (deferred clean rows: the weight gradient runs as the plain GEMM; deferred noisy rows: the tail launch
 * ends with its tail and class blocks); *pending = the parts the caller must prepare with
 * dad_step_prepare_rows(next_cfg, next_batch, workspace, any stream, *pending) before the next step's
 * dad_step_encode (order the streams with events).  A DP caller issues it on a second stream under the
 * gradient all-reduce, where the CUs would idle.  *prepped as for dad_step_backward_ahead (*pending = 0
 * when *prepped = 0). */
#define DAD_PREP_CLEAN 1
#define DAD_PREP_NOISY 2
int dad_step_backward_ahead_split(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
                                  void* workspace, void* stream, const dad_config* next_cfg,
                                  const dad_batch* next_batch, int defer, int* prepped, int* pending);
/* FP16/BF16: the augmentation and 16-bit conversion of (cfg, batch)'s rows (parts: DAD_PREP_CLEAN and/or
 * DAD_PREP_NOISY) into the workspace's prepared set of cfg->counter's parity -- the set the step with this
 * cfg reads (dad_prep; the draws of cfg's counter).  DAD_E_UNSUPPORTED in FP32. */
int dad_step_prepare_rows(const dad_config* cfg, const dad_batch* batch, void* workspace, void* stream, int parts);
int dad_step_apply(const dad_config* cfg, const dad_state* st, void* workspace, void* stream);
int dad_step(const dad_config* cfg, const dad_batch* batch, const dad_state* st,
             void* workspace, void* stream);
/* Trainer.train_step alone (I/train.py:397-471) for callers that keep their own
 * backward/clip/optimizer/EMA (I/train.py:486-492): after dad_step_compute, commits the
 * DACP state update of calculate_mask (I/utils.py:485-505) and writes st->losses; the
 * pre-clip gradient of total_loss stays in st->grad (rank mean when dp_world > 1). */
int dad_step_commit(const dad_config* cfg, const dad_state* st, void* workspace, void* stream);

/* DACPManager.update_class_quality_scores_epoch (I/utils.py:430-447) */
int dad_epoch_end(const dad_config* cfg, const dad_state* st, void* stream);
/* refresh the 16-bit shadows of W1 after the caller changed student/teacher params
 * (e.g. load_complete_pretrained_weights, I/model.py:143-198): fp16 for precision
 * DAD_PREC_FP16, bf16 otherwise (the format the next step of that precision reads) */
int dad_refresh_shadow(const dad_state* st, int precision, void* stream);

/* SSRLModel.update_teacher_ema (I/model.py:211-223) over flat [W1|b1|W2|b2] vectors:
 * teacher = teacher*ema_m + student*ema_one_m (n floats) */
int dad_teacher_ema(const float* student, float* teacher, size_t n, float ema_m, float ema_one_m, void* stream);

/* --- modular operators (the SSRLModel / utils.py surface) --------------------------
 * Emotion2VecEncoder.forward (I/model.py:18-41): e[B][256] = masked mean of ReLU(x W1^T + b1).
 * workspace: dad_encoder_workspace_bytes(B, T). */
size_t dad_encoder_workspace_bytes(int B, int T);
int dad_encoder_forward(const float* x, const uint8_t* pad, int B, int T, const float* w1,
                        const float* b1, float* e_out, int precision, void* workspace, void* stream);
/* backward of the above w.r.t. W1, b1 given de[B][256] (autograd of I/model.py:28-36);
 * recomputes the ReLU pattern; dw1 [256][768], db1 [256] are overwritten. */
int dad_encoder_backward(const float* x, const uint8_t* pad, int B, int T, const float* w1,
                         const float* b1, const float* de, float* dw1, float* db1,
                         void* workspace, void* stream);

/* --- device-resident data path ---------------------------
 * One padded batch gathered from a feature store resident in HBM.  Replaces the DataLoader's
 * per-sample row slice + .float() (NoisyEmotionDatasetFromArrays.__getitem__,
 * I/dataload_noisy.py:104-115; CleanEmotionDatasetFromArrays.__getitem__, I/dataload_clean.py:
 * 170-176) and its collator (I/dataload_noisy.py:116-129, I/dataload_clean.py:177-193,
 * C/dataload_casia_noisy.py:68-99):
 *   store     [frames][768] features of the whole split, dtype DAD_STORE_*
 *   offsets   [n_samples] int64 first frame of each sample; sizes [n_samples] int32 frames
 *   index     [B] int64 sample indices of this batch (the sampler's order)
 *   T         padded length, >= max(sizes[index]) (the collator's target_size)
 *   feats     [B][T][768] f32 out: sample rows, zeros past each size
 *   pad       [B][T] u8 out: 1 = padding (padding_mask[i, size:] = True)
 *   labels_in [n_samples] int64, labels_out [B] int64: both null for an unlabeled loader
 * An index outside [0, n_samples) yields an all-padding row and label -1 (no read). */
#define DAD_STORE_F32 0
#define DAD_STORE_F16 1
#define DAD_STORE_BF16 2
int dad_collate(const void* store, int store_dtype, const int64_t* offsets, const int32_t* sizes,
                int64_t n_samples, const int64_t* index, int B, int T, float* feats, uint8_t* pad,
                const int64_t* labels_in, int64_t* labels_out, void* stream);

/* Store-mode batch index (see dad_batch): for each b, row_out[b] = offsets[index[b]],
 * len_out[b] = sizes[index[b]] (0 and row 0 for an index outside [0, n_samples)),
 * pad [B][T] and labels exactly as dad_collate writes them -- the collator's outputs without
 * the feature copy. */
int dad_collate_index(const int64_t* offsets, const int32_t* sizes, int64_t n_samples, const int64_t* index,
                      int B, int T, int64_t* row_out, int32_t* len_out, uint8_t* pad,
                      const int64_t* labels_in, int64_t* labels_out, void* stream);
/* dad_collate_index for every batch of an epoch in one launch (the store-mode loader's epoch start):
 * n samples in batch order, sample i of a batch padded to T_i = pad_T[i] (its batch's T) with its
 * pad row at pad + pad_off[i] (T_i bytes); row_out / len_out / labels_out [n].  Per sample the same
 * values dad_collate_index writes. */
int dad_collate_index_epoch(const int64_t* offsets, const int32_t* sizes, int64_t n_samples, const int64_t* index,
                            int64_t n, const int64_t* pad_off, const int64_t* pad_T, int64_t* row_out,
                            int32_t* len_out, uint8_t* pad, const int64_t* labels_in, int64_t* labels_out,
                            void* stream);

/* --- eval path ------------------------------------------------
 * SSRLModel.predict's classifier in eval mode (I/model.py:225-245) on embeddings e [B][256]
 * from dad_encoder_forward, with what validation (I/train.py:522-564) and anchor calibration
 * (I/train.py:317-357) read from it: logits [B][4], softmax probs [B][4], the DACP certainty
 * score [B] (DACPManager.calculate_certainty_scores, I/utils.py:401-430; use_entropy selects
 * max_prob * (1 - H/log2 C) or max_prob) and the argmax pred [B].  Outputs may be NULL. */
int dad_predict_head(const float* e, int B, const float* w2, const float* b2, int use_entropy,
                     float* logits, float* probs, float* score, int64_t* pred, void* stream);

/* --- the reference's helper types as operators (I/utils.py:317-652) -------------------
 * For trainer code that drives DataAugmentation / DACPManager / ECDALoss itself (the
 * train_step shim's callers, anchor calibration, I/train.py:334,341).  Same device functions
 * as the fused step.
 *
 * DataAugmentation.weak_augment (strong = 0, I/utils.py:328-331) / strong_augment (strong = 1,
 * I/utils.py:333-375) of x [B][T][D] (a [T][D] input is B = 1; 1-D or > 3-D inputs are
 * passed with mask_len 0, as the reference masks only 2-D / 3-D data):
 *   out = x + std * N;  strong: * (u[d] > feat_p) (one [D] mask, no rescale; skipped when
 *   feat_p <= 0), then frames [start_b, start_b + mask_len) of utterance b zeroed, start_b
 *   uniform in [0, max(1, T - mask_len + 1)).
 * Draws: explicit (noise [B][T][D] standard normals, u [D] uniforms, start [B]) or, for NULL,
 * the counter streams of (seed, counter) -- with D = 768 the values the fused step draws. */
int dad_augment(const float* x, int B, int T, int D, int strong, float noise_std, float feat_p, int mask_len,
                uint64_t seed, uint64_t counter, const float* noise, const float* u, const int64_t* start,
                float* out, void* stream);
/* DACPManager.calculate_certainty_scores (I/utils.py:400-428): probs [B][4] -> score [B],
 * pred [B] (first argmax); use_entropy = USE_ENTROPY_IN_SCORE.  Outputs may be NULL. */
int dad_certainty_scores(const float* probs, int B, int use_entropy, float* score, int64_t* pred, void* stream);
/* DACPManager.calculate_mask (I/utils.py:449-507): teacher probs [Bn][4] and the 20-float
 * DACP state (tau | Q | epoch score sums | counts | calibrated anchors, DAD_DACP_FLOATS) ->
 * mask [Bn] (1 = confident), score [Bn], pred [Bn], class_weights [4] (W_c); updates tau
 * (EMA of the floored thresholds) and the epoch sums / counts in place, as the reference
 * updates its fields.  Reads cfg: dacp_gamma (from the epoch), dacp_k, dacp_lambda,
 * dacp_alpha / one_m_alpha, use_entropy.  score / pred / class_weights may be NULL. */
int dad_dacp_mask(const dad_config* cfg, const float* probs, int Bn, float* dacp, uint8_t* mask, float* score,
                  int64_t* pred, float* class_weights, void* stream);
/* ECDALoss.forward (I/utils.py:565-652) + its gradients: clean [B][256], noisy [Bn][256]
 * embeddings, clean_labels [B], noisy_labels [Bn] (teacher pseudo-labels), noisy_mask [Bn]
 * (1 = confident), noisy_scores [Bn], class_weights [n_weights] (DACP's [4] W_c, or the
 * fixed-threshold branch's ones(Bn), I/train.py:420).  loss [1] (device) = the class-aware sum
 * (or the global-MMD ablation when cfg->class_aware = 0); grad_clean [B][256] / grad_noisy
 * [Bn][256] = d loss / d embeddings (rows outside every member set are 0; may be NULL).
 * Reads cfg: class_aware, ecda_att_lambda, ecda_gamma, ecda_delta.
 * workspace: dad_ecda_workspace_bytes(B, Bn). */
size_t dad_ecda_workspace_bytes(int B, int Bn);
int dad_ecda_loss(const dad_config* cfg, const float* clean, int B, const float* noisy, int Bn,
                  const int64_t* clean_labels, const int64_t* noisy_labels, const uint8_t* noisy_mask,
                  const float* noisy_scores, const float* class_weights, int n_weights, float* loss,
                  float* grad_clean, float* grad_noisy, void* workspace, void* stream);

/* --- counter-RNG draws (diagnostics, distribution tests) ------------------------------
 * The random draws the throughput mode (DAD_RNG_COUNTER) makes inside the step kernels for
 * the step described by cfg (seed, counter = global step, B / Bn / Tn, stds, p, mask
 * geometry), computed by the same device functions the kernels call.  Elements
 * [first, first + n) of one stream, as float:
 *   DAD_DRAW_WEAK       weak-aug noise std*N of element i of the [Bn][Tn][768] tensor
 *                       (DataAugmentation.weak_augment's randn_like * std, I/utils.py:330)
 *   DAD_DRAW_STRONG     strong-aug noise (I/utils.py:338)
 *   DAD_DRAW_FEAT_KEEP  feature keep flag 1/0 of channel d < 768 (rand(D) > p, I/utils.py:343)
 *   DAD_DRAW_TSTART     temporal-mask start of utterance b < Bn (randint, I/utils.py:370)
 *   DAD_DRAW_KEEP1      classifier dropout factor (0 or 1/(1-p)) of element b*256+h, b < B
 *                       (student_classifier dropout, clean pass, I/train.py:400)
 *   DAD_DRAW_KEEP2      same, strong pass, b < Bn (I/train.py:440) */
#define DAD_DRAW_WEAK 1
#define DAD_DRAW_STRONG 2
#define DAD_DRAW_FEAT_KEEP 3
#define DAD_DRAW_TSTART 4
#define DAD_DRAW_KEEP1 5
#define DAD_DRAW_KEEP2 6
int dad_rng_draws(const dad_config* cfg, int which, uint64_t first, size_t n, float* out, void* stream);

/* --- per-kernel timing of the fused step (diagnostics; not inside graph capture) ------
 * dad_timing_start(every, max_steps): from now on every `every`-th step (counted at its
 * dad_step_encode / dad_step_compute call) records hip events at the boundaries of its kernels
 * on the caller's stream, up to max_steps timed steps; all events are created here, so a timed
 * region only records them.  dad_timing_stop: waits for the recorded events and returns, per
 * kernel k < n (DAD_TK_*), the summed milliseconds ms_sum[k] over count[k] timed steps, then
 * frees the events and turns timing off.  dad_timing_start fails (DAD_E_ARG) while a timing
 * session is active: stop the first before starting another. */
#define DAD_TK_ENCODE 0       /* dad_encode_ws[_f16] / dad_encode_f32 */
#define DAD_TK_POOL 1         /* dad_pool */
#define DAD_TK_TAIL 2         /* dad_tail_ecda_w / dad_tail_ecda (or dad_tail + dad_ecda) */
#define DAD_TK_WGRAD 3        /* dad_wgrad_direct (FP16/BF16) / dad_wgrad_f32 (FP32) */
#define DAD_TK_REDUCE 4       /* dad_reduce_w (FP16/BF16) / dad_reduce (FP32) */
#define DAD_TK_OPTIM 5        /* dad_optim */
#define DAD_TK_KERNELS 6
int dad_timing_start(int every, int max_steps);
/* dad_timing_kernels(mask): after dad_timing_start, record only the boundaries of the kernels
 * whose bit (1 << DAD_TK_*) is set (default: all).  Each recorded event costs the stream a few
 * microseconds, so a timed region that needs one kernel's duration records only its two. */
int dad_timing_kernels(unsigned mask);
/* dad_timing_reset (ABI 7): forget the steps counted and recorded so far in the active session (its
 * events stay created); the next step is the session's step 0.  A timed region can then follow its
 * warm-up with no gap: dad_timing_start's event set-up (milliseconds of host time with the GPU idle)
 * runs before the warm-up, the reset between them. */
int dad_timing_reset(void);
int dad_timing_stop(double* ms_sum, int* count, int n);

/* --- data-parallel gradient exchange (RCCL over xGMI) ------------------------------ */
int dad_comm_unique_id_bytes(void);
int dad_comm_get_unique_id(void* id_out);
int dad_comm_init(void** comm, int nranks, const void* id, int rank);
/* in-place SUM all-reduce of state->grad (DAD_GRAD_FLOATS floats) on `stream` */
int dad_comm_allreduce_grad(void* comm, const dad_state* st, void* stream);
/* ranks in the communicator (ncclCommCount) */
int dad_comm_count(void* comm, int* nranks);
/* in-place SUM all-reduce of n floats on `stream` (bench/test probe: a buffer of ones
 * all-reduced gives the number of ranks the transport actually connected) */
int dad_comm_allreduce_f32(void* comm, float* buf, size_t n, void* stream);
int dad_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* DAD_ABI_H_ */
