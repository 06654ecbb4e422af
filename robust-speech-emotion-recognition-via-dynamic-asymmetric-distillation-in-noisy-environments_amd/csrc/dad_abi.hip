// Host side of the C ABI (include/dad.h): argument validation, workspace carving and the
// kernel sequence of one DAD step.  Enqueue-only: no allocation, no synchronisation.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "dad_common.h"
#include "dad_kernels.h"

namespace {

#define DAD_TRY(expr)                           \
  do {                                          \
    hipError_t e_ = (expr);                     \
    if (e_ != hipSuccess) return (int)e_;       \
  } while (0)

inline int check_cfg(const dad_config* c) {
  if (!c) return DAD_E_ARG;
  if (c->B < 1 || c->B > DAD_MAX_BATCH || c->T < 1) return DAD_E_SHAPE;
  if (c->Bn < 0 || c->Bn > DAD_MAX_BATCH || c->Tn < 0) return DAD_E_SHAPE;
  if (!c->warmup && (c->Bn < 1 || c->Tn < 1)) return DAD_E_SHAPE;
  if (c->precision != DAD_PREC_FP32 && !dad_prec16(c->precision)) return DAD_E_ARG;
  if (c->rng_mode != DAD_RNG_EXPLICIT && c->rng_mode != DAD_RNG_COUNTER) return DAD_E_ARG;
  if (c->dp_world < 1) return DAD_E_ARG;
  return DAD_OK;
}

inline DadGeom geom_of(const dad_config* c) { return dad_geom(c->B, c->T, c->Bn, c->Tn); }

inline int splits_of(const dad_config* c) {
  const DadGeom g = geom_of(c);
  if (c->splits <= 0) return dad_auto_splits(g, c->precision, c->warmup);
  if (!dad_prec16(c->precision)) return c->splits;
  // dad_wgrad_direct holds at most WGD_MAXU slabs' utterances per split
  const int total = g.Bc * g.ncc + (c->warmup ? 0 : g.Bn * g.ncn);
  return std::max(c->splits, dad_wgd_min_splits(total));
}

inline int max_splits_of(const dad_config* c) {
  // the workspace is sized for the largest split count any step with this geometry may use
  dad_config post = *c;
  post.warmup = 0;
  return std::max(splits_of(c), splits_of(&post));
}

template <typename T>
inline T* ws_ptr(void* ws, size_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(ws) + off);
}

struct Keys {
  uint32_t weak, strong, feat, tstart, drop1, drop2;
};

inline Keys keys_of(const dad_config* c) {
  Keys k;
  k.weak = dad_stream_key(c->seed, c->counter, DAD_RNG_WEAK);
  k.strong = dad_stream_key(c->seed, c->counter, DAD_RNG_STRONG);
  k.feat = dad_stream_key(c->seed, c->counter, DAD_RNG_FEAT);
  k.tstart = dad_stream_key(c->seed, c->counter, DAD_RNG_TSTART);
  k.drop1 = dad_stream_key(c->seed, c->counter, DAD_RNG_DROP1);
  k.drop2 = dad_stream_key(c->seed, c->counter, DAD_RNG_DROP2);
  return k;
}

// DAD_TAIL_W=0 selects the general tail + ECDA launch for every batch (A/B runs; read once)
#ifndef DAD_CLEAN_IN_WGRAD
#define DAD_CLEAN_IN_WGRAD 1  // 0: the next batch's clean rows also prepared in the tail launch (A/B builds)
#endif
#ifndef DAD_POOL_IN_TAIL
#define DAD_POOL_IN_TAIL 1   // 0: the separate dad_pool launch also before the wave-centric tail (A/B builds)
#endif
bool tail_w_on() {
  static const bool on = [] { const char* e = getenv("DAD_TAIL_W"); return !(e && strcmp(e, "0") == 0); }();
  return on;
}

constexpr int kMaxDevices = 64;

int device_cus(int* out) {
  static int cache[kMaxDevices];
  int dev = 0;
  DAD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return DAD_E_ARG;
  if (!cache[dev]) DAD_TRY(hipDeviceGetAttribute(&cache[dev], hipDeviceAttributeMultiprocessorCount, dev));
  *out = cache[dev];
  return DAD_OK;
}

// Roles of the prepared-row encoder (dad_encode_wp, dad_wp_job_range): nt teacher and ns student
// workgroups, one per CU, in proportion to their live 16-row sub-slabs (every prepared sub-slab
// costs the same); more workgroups than CUs only when a range would exceed the kernel's
// DAD_ENC_WS_MAXJ-job table.
int wp_max_range(const DadGeom& G, int Bn, int nt, int ns) {
  int worst = 0;
  for (int wg = 0; wg < nt + ns; ++wg) {
    bool t = false;
    int j0 = 0, j1 = 0;
    dad_wp_job_range(wg, nt, ns, G.Bc, G.Tc, G.ncc, Bn, G.Tn, G.ncn, Bn * G.ncn, t, j0, j1);
    worst = std::max(worst, j1 - j0);
  }
  return worst;
}
int wp_split(const DadGeom& G, int Bn, int cus, int& nt, int& ns) {
  struct Entry { int Bc, Tc, Bn, Tn, cus, rc, nt, ns; };
  static thread_local Entry last{-1, -1, -1, -1, -1, 0, 0, 0};
  if (!(last.Bc == G.Bc && last.Tc == G.Tc && last.Bn == Bn && last.Tn == G.Tn && last.cus == cus)) {
    Entry e{G.Bc, G.Tc, Bn, G.Tn, cus, 0, 0, 0};
    const int Js = Bn * G.ncn, Jc = G.Bc * G.ncc;
    const double ln = (double)Bn * ((G.Tn + 15) / 16), lc = (double)G.Bc * ((G.Tc + 15) / 16);
    if (Js == 0) {
      e.ns = std::min(cus, Jc);
    } else {
      e.nt = std::max(1, std::min(std::min(Js, cus - 1), (int)(cus * ln / (2.0 * ln + lc) + 0.5)));
      e.ns = std::min(cus - e.nt, Jc + Js);
    }
    while (e.rc == DAD_OK && wp_max_range(G, Bn, e.nt, e.ns) > DAD_ENC_WS_MAXJ) {
      if (e.nt > 0 && e.nt < Js) ++e.nt;
      if (e.ns < Jc + Js) ++e.ns;
      if (e.nt + e.ns > Js + Jc + 2) e.rc = DAD_E_SHAPE;
    }
    last = e;
  }
  nt = last.nt;
  ns = last.ns;
  return last.rc;
}

// Row-preparation arguments (dad_prep.h) of the step described by (cfg, bt) into set x16.
DadPrepArgs prep_args(const dad_config* cfg, const dad_batch* bt, uint16_t* x16) {
  DadPrepArgs p;
  memset(&p, 0, sizeof(p));
  const Keys k = keys_of(cfg);
  p.g = geom_of(cfg);
  p.warmup = cfg->warmup; p.mask_len = cfg->mask_len; p.start_hi = cfg->start_hi;
  p.f16 = cfg->precision == DAD_PREC_FP16 ? 1 : 0;
  p.clean = 1;
  p.xc = bt->xc; p.xn = bt->xn;
  p.src = DadStoreRows{bt->rowc, bt->lenc, bt->rown, bt->lenn};
  if (cfg->rng_mode == DAD_RNG_EXPLICIT) { p.nw = bt->nw; p.ns = bt->ns; p.u = bt->u; p.start = bt->start; }
  p.key_weak = k.weak; p.key_strong = k.strong; p.key_feat = k.feat; p.key_tstart = k.tstart;
  p.weak_std = cfg->weak_std; p.strong_std = cfg->strong_std; p.feat_p = cfg->feat_p;
  p.x16 = x16;
  return p;
}

// standalone preparation of one set: ~4 workgroups of 4 waves per CU, two rows in flight per wave
int launch_prep(const DadPrepArgs& p, hipStream_t stream) {
  int cus = 0;
  const int rc = device_cus(&cus);
  if (rc) return rc;
  hipLaunchKernelGGL(dad_prep, dim3(4 * cus), dim3(DAD_PREP_THREADS), 0, stream, p);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

// Per-kernel timing of the fused step (dad_timing_start / dad_timing_stop): every `every`-th
// step (counted at its encoder call) records hip events at the kernel boundaries of the
// caller's stream.  Events are created up front by dad_timing_start, so a timed region only
// records them.  Not for graph capture.
enum { TK_E0, TK_E1, TK_POOL, TK_TAIL, TK_WGRAD, TK_RED, TK_OPT0, TK_OPT1, TK_N };
// (event-pair points of each DAD_TK_* kernel: dad_timing_stop's pairs)
const int kTkPairs[DAD_TK_KERNELS][2] = {{TK_E0, TK_E1}, {TK_E1, TK_POOL}, {TK_POOL, TK_TAIL}, {TK_TAIL, TK_WGRAD},
                                         {TK_WGRAD, TK_RED}, {TK_OPT0, TK_OPT1}};
struct Timing {
  unsigned points = ~0u;               // TK points recorded (dad_timing_kernels)
  int every = 0;
  long calls = 0;
  int cur = -1;                        // event set of the step being timed, -1: none
  std::vector<hipEvent_t> ev;          // nset * TK_N
  std::vector<uint8_t> rec;            // recorded flags
  int nset = 0, used = 0;
};
Timing g_tk;
std::mutex g_tk_mu;

void tk_begin() {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  g_tk.cur = -1;
  if (g_tk.every <= 0) return;
  if (g_tk.calls++ % g_tk.every == g_tk.every - 1 && g_tk.used < g_tk.nset) g_tk.cur = g_tk.used++;
}
void tk_mark(int point, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  if (g_tk.cur < 0 || !((g_tk.points >> point) & 1u)) return;
  const size_t i = (size_t)g_tk.cur * TK_N + point;
  if (hipEventRecord(g_tk.ev[i], s) == hipSuccess) g_tk.rec[i] = 1;
}
void tk_end() {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  g_tk.cur = -1;
}

}  // namespace

extern "C" {

int dad_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  if (g_tk.nset <= 0) return DAD_E_ARG;   // no active session
  g_tk.calls = 0;
  g_tk.used = 0;
  g_tk.cur = -1;
  std::fill(g_tk.rec.begin(), g_tk.rec.end(), (uint8_t)0);
  return DAD_OK;
}

int dad_timing_start(int every, int max_steps) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  if (every < 1 || max_steps < 1) return DAD_E_ARG;
  if (g_tk.nset > 0) return DAD_E_ARG;   // a session is active: dad_timing_stop it first
  for (hipEvent_t e : g_tk.ev) (void)hipEventDestroy(e);
  g_tk = Timing();
  g_tk.ev.assign((size_t)max_steps * TK_N, nullptr);
  g_tk.rec.assign((size_t)max_steps * TK_N, 0);
  // on any failure: the events created so far are destroyed and no session is left half set up
  auto fail = [](hipError_t e, hipStream_t s) {
    for (hipEvent_t x : g_tk.ev)
      if (x) (void)hipEventDestroy(x);
    if (s) (void)hipStreamDestroy(s);
    g_tk = Timing();
    return (int)e;
  };
  // timing-only events: no system-scope fence (no L2 writeback / invalidate at each record, which had
  // cost the stream ~3 us per event and slowed the kernel after it); dad_timing_stop reads them after
  // a device synchronize
  for (auto& e : g_tk.ev) {
    const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (r != hipSuccess) return fail(r, nullptr);
  }
  // first use outside the timed region: a HIP event's first record sets it up (host time the
  // first recorded steps would otherwise pay).  Recorded on a private non-blocking stream and
  // synchronised there only: no other stream waits, and a stream capturing a graph is untouched.
  hipStream_t ws = nullptr;
  hipError_t r = hipStreamCreateWithFlags(&ws, hipStreamNonBlocking);
  if (r != hipSuccess) return fail(r, nullptr);
  for (auto& e : g_tk.ev)
    if ((r = hipEventRecord(e, ws)) != hipSuccess) return fail(r, ws);
  if ((r = hipStreamSynchronize(ws)) != hipSuccess) return fail(r, ws);
  (void)hipStreamDestroy(ws);
  g_tk.every = every;
  g_tk.nset = max_steps;
  return DAD_OK;
}

int dad_timing_kernels(unsigned mask) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  unsigned pts = 0;
  for (int k = 0; k < DAD_TK_KERNELS; ++k)
    if ((mask >> k) & 1u) pts |= (1u << kTkPairs[k][0]) | (1u << kTkPairs[k][1]);
  if (pts & (1u << TK_POOL)) pts |= 1u << TK_E1;   // the tail's start when pooling is fused into it
  g_tk.points = pts;
  return DAD_OK;
}

int dad_timing_stop(double* ms_sum, int* count, int n) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  const auto& pairs = kTkPairs;
  if (n < 0 || (n > 0 && (!ms_sum || !count))) return DAD_E_ARG;
  for (int k = 0; k < n; ++k) { ms_sum[k] = 0.0; count[k] = 0; }
  int rc = DAD_OK;
  for (int s = 0; s < g_tk.used && rc == DAD_OK; ++s) {
    const size_t b = (size_t)s * TK_N;
    for (int k = 0; k < n && k < DAD_TK_KERNELS; ++k) {
      int a = pairs[k][0];
      const int z = pairs[k][1];
      // pooling fused into the tail launch: no pool point; the tail launch runs from the encoder's end
      if (a == TK_POOL && !g_tk.rec[b + a] && z != TK_POOL) a = TK_E1;
      if (!g_tk.rec[b + a] || !g_tk.rec[b + z]) continue;
      float ms = 0.0f;
      hipError_t e = hipEventSynchronize(g_tk.ev[b + z]);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, g_tk.ev[b + a], g_tk.ev[b + z]);
      if (e != hipSuccess) { rc = (int)e; break; }
      ms_sum[k] += ms;
      count[k] += 1;
    }
  }
  for (hipEvent_t e : g_tk.ev) (void)hipEventDestroy(e);
  g_tk = Timing();
  return rc;
}

int dad_abi_version(void) { return DAD_ABI_VERSION; }
size_t dad_param_count(void) { return DAD_NPARAM; }

const char* dad_error_string(int code) {
  switch (code) {
    case DAD_OK: return "ok";
    case DAD_E_ARG: return "DAD_E_ARG: invalid argument";
    case DAD_E_SHAPE: return "DAD_E_SHAPE: unsupported batch/sequence shape";
    case DAD_E_COMM: return "DAD_E_COMM: RCCL failure";
    case DAD_E_UNSUPPORTED: return "DAD_E_UNSUPPORTED";
    default: return hipGetErrorString((hipError_t)code);
  }
}

int dad_encoder_ws_plan(const dad_config* cfg, int cus, int* nt, int* ns, int* max_jobs) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (cus < 2 || !nt || !ns || !max_jobs) return DAD_E_ARG;
  const DadGeom G = geom_of(cfg);
  const int Bn = cfg->warmup ? 0 : G.Bn;
  rc = wp_split(G, Bn, cus, *nt, *ns);
  if (rc) return rc;
  *max_jobs = wp_max_range(G, Bn, *nt, *ns);
  return DAD_OK;
}

int dad_encoder_ws_jobs(const dad_config* cfg, int cus, int* jobs, int capacity) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (cus < 2 || !jobs) return DAD_E_ARG;
  const DadGeom G = geom_of(cfg);
  const int Bn = cfg->warmup ? 0 : G.Bn;
  int nt = 0, ns = 0;
  rc = wp_split(G, Bn, cus, nt, ns);
  if (rc) return rc;
  if (capacity < 4 * (nt + ns)) return DAD_E_ARG;   // the grid outgrew the caller's table
  for (int wg = 0; wg < nt + ns; ++wg) {
    bool t = false;
    int j0 = 0, j1 = 0;
    dad_wp_job_range(wg, nt, ns, G.Bc, G.Tc, G.ncc, Bn, G.Tn, G.ncn, Bn * G.ncn, t, j0, j1);
    jobs[4 * wg] = t ? 1 : 0;
    jobs[4 * wg + 1] = j0;
    jobs[4 * wg + 2] = 1;
    jobs[4 * wg + 3] = j1 - j0;
  }
  return nt + ns;
}

int dad_workspace_bytes(const dad_config* cfg, size_t* bytes) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!bytes) return DAD_E_ARG;
  *bytes = dad_ws_layout(geom_of(cfg), max_splits_of(cfg), cfg->precision).bytes;
  return DAD_OK;
}

}  // extern "C"

// The next step's batch may be prepared in this step's tail launch when the tail runs as
// dad_tail_ecda_w and the next step has this step's workspace layout (so its prepared set sits
// where the next step will look) and the other set parity.
static bool can_prepare_ahead(const dad_config* cfg, const dad_config* ncfg, const dad_batch* nbt) {
  if (!ncfg || !nbt || check_cfg(ncfg) != DAD_OK) return false;
  if (!dad_prec16(cfg->precision) || ncfg->precision != cfg->precision) return false;
  if (ncfg->B != cfg->B || ncfg->T != cfg->T || ncfg->Bn != cfg->Bn || ncfg->Tn != cfg->Tn) return false;
  if (((ncfg->counter ^ cfg->counter) & 1u) == 0) return false;
  if (max_splits_of(ncfg) != max_splits_of(cfg)) return false;
  if (!nbt->xc || !nbt->mc) return false;
  if (!ncfg->warmup && (!nbt->xn || !nbt->mn)) return false;
  if (ncfg->rng_mode == DAD_RNG_EXPLICIT && !ncfg->warmup && (!nbt->nw || !nbt->ns || !nbt->u || !nbt->start))
    return false;
  if ((nbt->rowc == nullptr) != (nbt->lenc == nullptr) || (nbt->rown == nullptr) != (nbt->lenn == nullptr)) return false;
  return true;
}

// defer (dad_step_backward_ahead_split): the DAD_PREP_* parts of the next batch's rows this step's
// launches leave to the caller (dad_step_prepare_rows); *pending = the parts actually left
static int step_compute_phases(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                               void* stream_, bool do_encode, bool do_backward, const dad_config* ncfg = nullptr,
                               const dad_batch* nbt = nullptr, int* prepped = nullptr, int defer = 0,
                               int* pending = nullptr) {
  if (prepped) *prepped = 0;
  if (pending) *pending = 0;
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!bt || !st || !workspace) return DAD_E_ARG;
  if (!bt->xc || !bt->mc || !bt->yc || !st->student || !st->teacher || !st->grad || !st->dacp || !st->tail ||
      !st->emb || !st->logits || !st->w1bf_student || !st->w1bf_teacher)
    return DAD_E_ARG;
  if (!cfg->warmup && (!bt->xn || !bt->mn)) return DAD_E_ARG;
  const bool explicit_rng = cfg->rng_mode == DAD_RNG_EXPLICIT;
  if (explicit_rng && cfg->p_drop > 0.0f && (!bt->keep1 || (!cfg->warmup && !bt->keep2))) return DAD_E_ARG;
  if (explicit_rng && !cfg->warmup && (!bt->nw || !bt->ns || !bt->u || !bt->start)) return DAD_E_ARG;
  // store mode, per batch (clean and noisy independently): rows and lengths together
  if ((bt->rowc == nullptr) != (bt->lenc == nullptr) || (bt->rown == nullptr) != (bt->lenn == nullptr))
    return DAD_E_ARG;
  const DadStoreRows src = {bt->rowc, bt->lenc, bt->rown, bt->lenn};
  hipStream_t stream = (hipStream_t)stream_;
  const DadGeom G = geom_of(cfg);
  const int Bn = cfg->warmup ? 0 : G.Bn;
  const int splits = splits_of(cfg);
  if (splits > max_splits_of(cfg)) return DAD_E_ARG;
  const DadWs L = dad_ws_layout(G, max_splits_of(cfg), cfg->precision);
  const Keys k = keys_of(cfg);
  float* part_sum = ws_ptr<float>(workspace, L.part_sum);
  float* part_cnt = ws_ptr<float>(workspace, L.part_cnt);
  uint32_t* bits = ws_ptr<uint32_t>(workspace, L.bits);
  float* vlen = ws_ptr<float>(workspace, L.vlen);
  float* cnt_tot = ws_ptr<float>(workspace, L.cnt_tot);
  float* ge = ws_ptr<float>(workspace, L.ge);
  float* ge_ecda = ws_ptr<float>(workspace, L.ge_ecda);
  float* normpart = ws_ptr<float>(workspace, L.normpart);
  float* ecda_scratch = ws_ptr<float>(workspace, L.ecda);
  float* gzb = ws_ptr<float>(workspace, L.gzb);
  uint32_t* eflag = ws_ptr<uint32_t>(workspace, L.eflag);
  uint32_t* pool_ready = ws_ptr<uint32_t>(workspace, L.ready);
  // the wave-centric tail launch (B, Bn <= 64, class-aware MMD, after the warm-up) also pools the
  // embeddings (dad_tail_ecda_w's spare blocks) instead of a separate dad_pool launch
  const bool tail_w = !cfg->warmup && DAD_FUSED_TAIL && G.Bc <= 64 && Bn <= 64 && cfg->class_aware && tail_w_on();
  const bool pool_in_tail = tail_w && DAD_POOL_IN_TAIL;
  const bool h16 = dad_prec16(cfg->precision);
  const bool f16 = cfg->precision == DAD_PREC_FP16;
  // 16-bit modes: this step's prepared set (parity of the step counter; the next step's set is
  // the other one, so preparing it in this step's tail launch leaves this one intact for wgrad)
  uint16_t* xs16 = ws_ptr<uint16_t>(workspace, L.xs16 + (cfg->counter & 1u) * L.x16set);
  const size_t nrc = (size_t)G.Bc * G.Tc, nrn = (size_t)G.Bn * G.Tn;

  // 1. fused augmentation + encoder GEMMs + pooling partials
  DadEncodeArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.g = G; ea.warmup = cfg->warmup;
  ea.mask_len = cfg->mask_len; ea.start_hi = cfg->start_hi;
  ea.xc = bt->xc; ea.mc = bt->mc; ea.xn = bt->xn; ea.mn = bt->mn; ea.src = src;
  ea.w1_student = st->student + DAD_OFF_W1; ea.b1_student = st->student + DAD_OFF_B1;
  ea.w1_teacher = st->teacher + DAD_OFF_W1; ea.b1_teacher = st->teacher + DAD_OFF_B1;
  ea.w1h_student = st->w1bf_student;
  ea.w1h_teacher = st->w1bf_teacher;
  ea.pool_ready = pool_ready;
  if (explicit_rng) { ea.nw = bt->nw; ea.ns = bt->ns; ea.u = bt->u; ea.start = bt->start; }
  ea.key_weak = k.weak; ea.key_strong = k.strong; ea.key_feat = k.feat; ea.key_tstart = k.tstart;
  ea.weak_std = cfg->weak_std; ea.strong_std = cfg->strong_std; ea.feat_p = cfg->feat_p;
  ea.part_sum = part_sum; ea.part_cnt = part_cnt; ea.bits = bits;
  const int nwaves = G.Bc * G.ncc + Bn * G.ncn;
  const dim3 egrid((nwaves + 3) / 4);
  if (do_encode) {
    tk_begin();
    tk_mark(TK_E0, stream);
    if (h16) {
      // augmentation + 16-bit conversion (unless the previous step's tail launch prepared this
      // batch: cfg->prepped), then the W-stationary GEMM on the prepared set
      if (!cfg->prepped) {
        const int rp = launch_prep(prep_args(cfg, bt, xs16), stream);
        if (rp) return rp;
      }
      int cus = 0;
      const int rc = device_cus(&cus);
      if (rc) return rc;
      const int rs = wp_split(G, Bn, cus, ea.ws_nt, ea.ws_ns);
      if (rs) return rs;
      ea.x16c = xs16; ea.x16s = xs16 + nrc * DAD_D; ea.x16w = ea.x16s + (cfg->warmup ? 0 : nrn) * DAD_D;
      const dim3 grid(ea.ws_nt + ea.ws_ns);
      if (f16) hipLaunchKernelGGL(dad_encode_wp_f16, grid, dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
      else hipLaunchKernelGGL(dad_encode_wp, grid, dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
    } else {
      hipLaunchKernelGGL(dad_encode_f32, egrid, dim3(DAD_ENC_F32_THREADS), 0, stream, ea);
    }
    DAD_TRY(hipGetLastError());
    tk_mark(TK_E1, stream);
  }
  if (!do_backward) return DAD_OK;

  // 2. pooled embeddings + classifier logits
  DadPoolArgs pa;
  memset(&pa, 0, sizeof(pa));
  pa.g = G; pa.warmup = cfg->warmup;
  pa.mc = bt->mc; pa.mn = bt->mn; pa.part_sum = part_sum;
  pa.student = st->student; pa.teacher = st->teacher;
  if (explicit_rng) { pa.keep1 = bt->keep1; pa.keep2 = bt->keep2; }
  pa.key_drop1 = k.drop1; pa.key_drop2 = k.drop2;
  pa.p_drop = cfg->p_drop; pa.drop_scale = cfg->drop_scale;
  pa.emb = st->emb; pa.vlen = vlen; pa.logits = st->logits;
  pa.part_cnt = part_cnt; pa.cnt_tot = cnt_tot;
  pa.eflag = eflag; pa.tail_terms = st->tail + DAD_T_ECDA_TERM;
  pa.range_flag = reinterpret_cast<uint32_t*>(st->tail + DAD_T_RANGE);
  if (pool_in_tail) {
    pa.ready = pool_ready;   // pooled by the tail launch (zeroed by this step's encoder); no pool
                             // timing point: the tail launch is timed from the encoder's end
  } else {
    hipLaunchKernelGGL(dad_pool, dim3(G.Bc + 2 * Bn), dim3(DAD_POOL_THREADS), 0, stream, pa);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_POOL, stream);
  }

  // 3. losses, DACP mask, analytic backward to dL/de and the classifier grads
  DadTailArgs ta;
  memset(&ta, 0, sizeof(ta));
  ta.cfg = *cfg; ta.yc = bt->yc; ta.logits = st->logits; ta.emb = st->emb; ta.student = st->student;
  if (explicit_rng) { ta.keep1 = bt->keep1; ta.keep2 = bt->keep2; }
  ta.key_drop1 = k.drop1; ta.key_drop2 = k.drop2;
  ta.dacp = st->dacp; ta.tailf = st->tail; ta.ge = ge; ta.ge_ecda = ge_ecda; ta.grad = st->grad;
  ta.gzb = gzb; ta.eflag = eflag;
  // 4. ECDA (class-aware MMD + compactness + repulsion) and its embedding grads: after the
  //    warm-up, in the same launch as the tail (block 0 = tail, blocks 1..C = classes)
  DadEcdaArgs ca;
  memset(&ca, 0, sizeof(ca));
  ca.cfg = *cfg; ca.yc = bt->yc; ca.emb = st->emb; ca.tailf = st->tail;
  ca.tail_terms = st->tail + DAD_T_ECDA_TERM; ca.ge = ge_ecda; ca.scratch = ecda_scratch; ca.eflag = eflag;
  ca.sink = ws_ptr<float>(workspace, L.gflat);
  // next-batch preparation split (padded next batch): its noisy rows in the tail launch, its clean
  // rows in the weight-gradient launch (dad_wgrad_direct*_cp, interleaved with the GEMM)
  DadPrepArgs pcw;
  memset(&pcw, 0, sizeof(pcw));
  bool clean_in_wgrad = false, clean_store = false;
  if (!cfg->warmup && DAD_FUSED_TAIL) {
    // batches of at most 64 utterances per side, class-aware MMD: the wave-centric launch, whose
    // spare blocks pool the embeddings (one item per wave: Bc + 2 Bn items) and then run
    if (tail_w) {
      // the next step's row preparation on the CUs the tail and class blocks leave idle
      DadPrepArgs pp;
      memset(&pp, 0, sizeof(pp));
      int nblk = 1 + DAD_C + (pool_in_tail ? (G.Bc + 2 * Bn + DAD_TAIL_THREADS / 64 - 1) / (DAD_TAIL_THREADS / 64) : 0);
      if (can_prepare_ahead(cfg, ncfg, nbt)) {
        int cus = 0;
        const int rc = device_cus(&cus);
        if (rc) return rc;
        pp = prep_args(ncfg, nbt, ws_ptr<uint16_t>(workspace, L.xs16 + (ncfg->counter & 1u) * L.x16set));
        if (prepped) *prepped = 1;
        if (!(defer & DAD_PREP_CLEAN) && DAD_CLEAN_IN_WGRAD && h16 && (nbt->rowc == nullptr || ncfg->B <= 64)) {
          clean_in_wgrad = true;
          clean_store = nbt->rowc != nullptr;   // store batch: rows through its utterance table
          pcw = pp;        // clean rows only (dad_prep_clean_load / _store)
          pp.clean = 0;    // noisy rows only
        }
        if (defer & DAD_PREP_CLEAN) pp.clean = 0;   // the caller's (under the DP exchange)
        const bool noisy_here = !(defer & DAD_PREP_NOISY);
        if (pending) *pending = defer & (DAD_PREP_CLEAN | DAD_PREP_NOISY);
        if (!noisy_here && !pp.clean) memset(&pp, 0, sizeof(pp));   // nothing left for the tail launch
        // spare blocks for whatever the tail launch prepares (noisy rows, and clean ones when the weight
        // gradient cannot take them)
        if (pp.x16) nblk = std::max(nblk, std::max(cus, 2 * (1 + DAD_C)));
        if (pp.x16 && !noisy_here) pp.warmup = 1;   // (dad_prep_rows: clean rows only)
      }
      hipLaunchKernelGGL(dad_tail_ecda_w, dim3(nblk), dim3(DAD_TAIL_THREADS), 0, stream, ta, ca, pp, pa);
    } else
      hipLaunchKernelGGL(dad_tail_ecda, dim3(1 + DAD_C), dim3(DAD_TAIL_THREADS), 0, stream, ta, ca);
    DAD_TRY(hipGetLastError());
  } else {
    hipLaunchKernelGGL(dad_tail, dim3(1), dim3(DAD_TAIL_THREADS), 0, stream, ta);
    DAD_TRY(hipGetLastError());
    if (!cfg->warmup) {
      hipLaunchKernelGGL(dad_ecda, dim3(DAD_C), dim3(DAD_ECDA_THREADS), 0, stream, ca);
      DAD_TRY(hipGetLastError());
    }
  }
  tk_mark(TK_TAIL, stream);

  // 5. dW1 as one direct split-K GEMM (G = ReLU' * dL/de / len rebuilt from the tail's dL/dz
  //    and the ECDA rows), then the split sums with db1, dW2, loss totals, squared-norm partials
  DadWgradArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.g = G; wa.warmup = cfg->warmup;
  wa.mask_len = cfg->mask_len; wa.start_hi = cfg->start_hi;
  wa.xc = bt->xc; wa.xn = bt->xn; wa.src = src;
  if (explicit_rng) { wa.ns = bt->ns; wa.u = bt->u; wa.start = bt->start; }
  wa.key_strong = k.strong; wa.key_feat = k.feat; wa.key_tstart = k.tstart;
  wa.strong_std = cfg->strong_std; wa.feat_p = cfg->feat_p;
  wa.bits = bits; wa.ge = ge; wa.vlen = vlen; wa.xs16 = xs16;
  wa.splits = splits;
  wa.wpart = ws_ptr<float>(workspace, L.wpart);
  DadReduceArgs ra;
  memset(&ra, 0, sizeof(ra));
  ra.g = G; ra.warmup = cfg->warmup;
  ra.want_norm = cfg->dp_world == 1;
  ra.w_kl = cfg->w_kl; ra.w_ecda = cfg->w_ecda;
  ra.ge_ecda = ge_ecda;
  ra.gzb = gzb; ra.eflag = eflag; ra.student = st->student; ra.emb = st->emb;
  if (explicit_rng) { ra.keep1 = bt->keep1; ra.keep2 = bt->keep2; }
  ra.key_drop1 = k.drop1; ra.key_drop2 = k.drop2; ra.p_drop = cfg->p_drop; ra.drop_scale = cfg->drop_scale;
  ra.ge = ge; ra.vlen = vlen; ra.cnt_tot = cnt_tot; ra.tailf = st->tail;
  ra.grad = st->grad; ra.normpart = normpart;
  ra.pool_abort = pool_in_tail ? pool_ready + DAD_POOL_ABORT : nullptr;
  ra.splits = splits; ra.wpart = wa.wpart;
  if (!h16) {
    // FP32: one tile = (split, 128 columns); then every reduce block (dW1 sums and the
    // db1 / dW2 / totals blocks)
    wa.ntiles = 6 * splits;
    hipLaunchKernelGGL(dad_wgrad_f32, dim3(wa.ntiles), dim3(DAD_WGRAD_THREADS), 0, stream, wa, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_WGRAD, stream);
    hipLaunchKernelGGL(dad_reduce, dim3(DAD_REDUCE_BLOCKS), dim3(DAD_REDUCE_THREADS), 0, stream, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_RED, stream);
  } else {
    wa.ntiles = WGD_NDB * splits;
    // multiple of 8 (XCD-aware tile order) with WGD_XWG spare workgroups for the extra blocks
    const dim3 grid((wa.ntiles + WGD_XWG + 7) / 8 * 8);
    if (clean_in_wgrad && clean_store) {
      if (f16) hipLaunchKernelGGL(dad_wgrad_direct_f16_cps, grid, dim3(WGD_THREADS), 0, stream, wa, ra, pcw);
      else hipLaunchKernelGGL(dad_wgrad_direct_cps, grid, dim3(WGD_THREADS), 0, stream, wa, ra, pcw);
    } else if (clean_in_wgrad) {
      if (f16) hipLaunchKernelGGL(dad_wgrad_direct_f16_cp, grid, dim3(WGD_THREADS), 0, stream, wa, ra, pcw);
      else hipLaunchKernelGGL(dad_wgrad_direct_cp, grid, dim3(WGD_THREADS), 0, stream, wa, ra, pcw);
    } else {
      if (f16) hipLaunchKernelGGL(dad_wgrad_direct_f16, grid, dim3(WGD_THREADS), 0, stream, wa, ra);
      else hipLaunchKernelGGL(dad_wgrad_direct, grid, dim3(WGD_THREADS), 0, stream, wa, ra);
    }
    DAD_TRY(hipGetLastError());
    tk_mark(TK_WGRAD, stream);
    hipLaunchKernelGGL(dad_reduce_w, dim3(DAD_REDUCE_BLOCKS - DAD_REDUCE_XBLK), dim3(64), 0, stream, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_RED, stream);
  }
  return DAD_OK;
}

extern "C" {

int dad_step_compute(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                     void* stream) {
  return step_compute_phases(cfg, bt, st, workspace, stream, true, true);
}

int dad_step_encode(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                    void* stream) {
  return step_compute_phases(cfg, bt, st, workspace, stream, true, false);
}

int dad_step_backward(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                      void* stream) {
  return step_compute_phases(cfg, bt, st, workspace, stream, false, true);
}

int dad_step_backward_ahead(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                            void* stream, const dad_config* next_cfg, const dad_batch* next_batch, int* prepped) {
  return step_compute_phases(cfg, bt, st, workspace, stream, false, true, next_cfg, next_batch, prepped);
}

int dad_step_backward_ahead_split(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                                  void* stream, const dad_config* next_cfg, const dad_batch* next_batch, int defer,
                                  int* prepped, int* pending) {
  if (!pending || (defer & ~(DAD_PREP_CLEAN | DAD_PREP_NOISY)) != 0) return DAD_E_ARG;
  return step_compute_phases(cfg, bt, st, workspace, stream, false, true, next_cfg, next_batch, prepped, defer,
                             pending);
}

int dad_step_prepare_rows(const dad_config* cfg, const dad_batch* bt, void* workspace, void* stream, int parts) {
  const int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!bt || !workspace || (parts & ~(DAD_PREP_CLEAN | DAD_PREP_NOISY)) != 0) return DAD_E_ARG;
  if (!dad_prec16(cfg->precision)) return DAD_E_UNSUPPORTED;
  if (parts == 0) return DAD_OK;
  if ((parts & DAD_PREP_CLEAN) && !bt->xc) return DAD_E_ARG;
  const bool noisy = (parts & DAD_PREP_NOISY) && !cfg->warmup;
  if (noisy && (!bt->xn || (cfg->rng_mode == DAD_RNG_EXPLICIT && (!bt->nw || !bt->ns || !bt->u || !bt->start))))
    return DAD_E_ARG;
  if ((bt->rowc == nullptr) != (bt->lenc == nullptr) || (bt->rown == nullptr) != (bt->lenn == nullptr)) return DAD_E_ARG;
  const DadWs L = dad_ws_layout(geom_of(cfg), max_splits_of(cfg), cfg->precision);
  DadPrepArgs p = prep_args(cfg, bt, ws_ptr<uint16_t>(workspace, L.xs16 + (cfg->counter & 1u) * L.x16set));
  p.clean = (parts & DAD_PREP_CLEAN) ? 1 : 0;
  if (!p.clean && !noisy) return DAD_OK;
  if (!noisy) p.warmup = 1;   // (dad_prep_rows: no noisy rows in a warm-up set)
  return launch_prep(p, (hipStream_t)stream);
}

int dad_step_apply(const dad_config* cfg, const dad_state* st, void* workspace, void* stream_) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!st || !workspace) return DAD_E_ARG;
  hipStream_t stream = (hipStream_t)stream_;
  const DadWs L = dad_ws_layout(geom_of(cfg), max_splits_of(cfg), cfg->precision);
  float* normpart = ws_ptr<float>(workspace, L.normpart);
  const int nblk = (DAD_NPARAM + 1023) / 1024;
  int nnorm = DAD_REDUCE_BLOCKS;
  if (cfg->dp_world > 1) {
    hipLaunchKernelGGL(dad_norm, dim3(nblk), dim3(256), 0, stream, st->grad, normpart, 1.0f / (float)cfg->dp_world);
    DAD_TRY(hipGetLastError());
    nnorm = nblk;
  }
  DadOptimArgs oa;
  memset(&oa, 0, sizeof(oa));
  oa.cfg = *cfg;
  oa.student = st->student; oa.teacher = st->teacher; oa.exp_avg = st->exp_avg; oa.exp_avg_sq = st->exp_avg_sq;
  oa.grad = st->grad;
  oa.w1h_student = st->w1bf_student;
  oa.w1h_teacher = st->w1bf_teacher;
  oa.dacp = st->dacp; oa.tailf = st->tail; oa.normpart = normpart; oa.nnorm = nnorm;
  oa.losses_out = st->losses;
  tk_mark(TK_OPT0, stream);
  hipLaunchKernelGGL(dad_optim, dim3(nblk), dim3(DAD_OPTIM_THREADS), 0, stream, oa);
  DAD_TRY(hipGetLastError());
  tk_mark(TK_OPT1, stream);
  tk_end();
  return DAD_OK;
}

int dad_step_commit(const dad_config* cfg, const dad_state* st, void* workspace, void* stream_) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!st || !st->grad || !st->dacp || !st->tail || !workspace) return DAD_E_ARG;
  hipStream_t stream = (hipStream_t)stream_;
  if (cfg->dp_world > 1) {
    const DadWs L = dad_ws_layout(geom_of(cfg), max_splits_of(cfg), cfg->precision);
    const int nblk = (DAD_NPARAM + 1023) / 1024;
    hipLaunchKernelGGL(dad_norm, dim3(nblk), dim3(256), 0, stream, st->grad, ws_ptr<float>(workspace, L.normpart),
                       1.0f / (float)cfg->dp_world);
    DAD_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(dad_commit_kernel, dim3(1), dim3(64), 0, stream, *cfg, st->grad, st->dacp, st->tail, st->losses);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

int dad_step(const dad_config* cfg, const dad_batch* batch, const dad_state* st, void* workspace, void* stream) {
  int rc = dad_step_compute(cfg, batch, st, workspace, stream);
  if (rc) return rc;
  return dad_step_apply(cfg, st, workspace, stream);
}

int dad_epoch_end(const dad_config* cfg, const dad_state* st, void* stream_) {
  if (!cfg || !st || !st->dacp) return DAD_E_ARG;
  hipLaunchKernelGGL(dad_epoch_end_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream_, st->dacp, cfg->dacp_beta,
                     cfg->dacp_one_m_beta);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

int dad_refresh_shadow(const dad_state* st, int precision, void* stream_) {
  if (!st || !st->student || !st->teacher || !st->w1bf_student || !st->w1bf_teacher) return DAD_E_ARG;
  if (precision != DAD_PREC_FP32 && !dad_prec16(precision)) return DAD_E_ARG;
  hipLaunchKernelGGL(dad_shadow_kernel, dim3((DAD_H * DAD_D + 255) / 256), dim3(256), 0, (hipStream_t)stream_,
                     st->student, st->teacher, st->w1bf_student, st->w1bf_teacher, precision == DAD_PREC_FP16 ? 1 : 0);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

// ------------------------------------------------------------------ counter-RNG draws
}  // extern "C"

namespace {

// The throughput mode's random draws, by the device functions the step kernels call
// (dad_common.h): elements [first, first + n) of stream `which`.
__global__ __launch_bounds__(256) void dad_draws_kernel(int which, uint32_t key, uint64_t first, size_t n, float sd,
                                                        float p, float scale, int start_hi, float* out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t e = first + i;
  float v = 0.0f;
  switch (which) {
    case DAD_DRAW_WEAK:
    case DAD_DRAW_STRONG: {
      float z0, z1;
      dad_aug_noise_pair(key, (uint32_t)(e >> 1), sd, z0, z1);
      v = (e & 1) ? z1 : z0;
      break;
    }
    case DAD_DRAW_FEAT_KEEP: v = dad_feat_keep(nullptr, key, (int)e, p); break;
    case DAD_DRAW_TSTART: v = (float)dad_tstart_at(key, (int)e, start_hi); break;
    default:   // DAD_DRAW_KEEP1 / KEEP2: element b * 256 + h
      v = keep_value(nullptr, key, (int)(e / DAD_H), (int)(e % DAD_H), p, scale);
      break;
  }
  out[i] = v;
}

}  // namespace

extern "C" {

int dad_rng_draws(const dad_config* cfg, int which, uint64_t first, size_t n, float* out, void* stream) {
  if (!cfg || (!out && n)) return DAD_E_ARG;
  const Keys k = keys_of(cfg);
  uint32_t key = 0;
  float sd = 0.0f, p = 0.0f;
  uint64_t limit = 0;
  const uint64_t noise = (uint64_t)cfg->Bn * (uint64_t)cfg->Tn * DAD_D;
  switch (which) {
    case DAD_DRAW_WEAK: key = k.weak; sd = cfg->weak_std; limit = noise; break;
    case DAD_DRAW_STRONG: key = k.strong; sd = cfg->strong_std; limit = noise; break;
    case DAD_DRAW_FEAT_KEEP: key = k.feat; p = cfg->feat_p; limit = DAD_D; break;
    case DAD_DRAW_TSTART: key = k.tstart; limit = (uint64_t)cfg->Bn; break;
    case DAD_DRAW_KEEP1: key = k.drop1; p = cfg->p_drop; limit = (uint64_t)cfg->B * DAD_H; break;
    case DAD_DRAW_KEEP2: key = k.drop2; p = cfg->p_drop; limit = (uint64_t)cfg->Bn * DAD_H; break;
    default: return DAD_E_ARG;
  }
  if (first + n > limit || limit > 0xffffffffull * 2) return DAD_E_SHAPE;
  if (n == 0) return DAD_OK;
  hipLaunchKernelGGL(dad_draws_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, which,
                     key, first, n, sd, p, cfg->drop_scale, cfg->start_hi, out);
  DAD_TRY(hipGetLastError());
  return DAD_OK;
}

// ----------------------------------------------------------------- modular encoder ops
}  // extern "C"

// The modular encoder ops' workspace: the FP32 layout plus a prepared-row region (the 16-bit
// encoder's input: x converted by dad_prep).
static DadWs enc_layout(const DadGeom& G) {
  return dad_ws_layout(G, dad_auto_splits(G, DAD_PREC_FP32, 1), DAD_PREC_BF16);
}

extern "C" {
size_t dad_encoder_workspace_bytes(int B, int T) {
  if (B < 1 || T < 1) return 0;
  return enc_layout(dad_geom(B, T, 0, 0)).bytes;
}

}  // extern "C"

namespace {

__global__ __launch_bounds__(256) void dad_embed_kernel(const float* part_sum, const uint8_t* pad, int B, int T,
                                                        int nchunk, float* vlen, float* e_out) {
  (void)B;
  __shared__ float red[4];
  const int b = blockIdx.x, h = threadIdx.x;
  float l = 0.0f;
  for (int t = h; t < T; t += 256) l += pad[(size_t)b * T + t] == 0 ? 1.0f : 0.0f;
  l = dad_wave_sum(l);
  if ((h & 63) == 0) red[h >> 6] = l;
  __syncthreads();
  const float len = ((red[0] + red[1]) + red[2]) + red[3];
  float s = 0.0f;
  for (int c = 0; c < nchunk; ++c) s += part_sum[((size_t)b * nchunk + c) * DAD_H + h];
  e_out[(size_t)b * DAD_H + h] = s / fmaxf(len, 1.0f);
  if (h == 0 && vlen) vlen[b] = len;
}

// 16-bit copy of W1 in the W-stationary encoder's fragment order (dad_w1frag_index)
__global__ __launch_bounds__(256) void dad_w1h_kernel(const float* w, uint16_t* out, int f16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (size_t)DAD_H * DAD_D)
    out[dad_w1frag_index((uint32_t)(i / DAD_D), (uint32_t)(i % DAD_D))] = dad_half_bits(w[i], f16 != 0);
}

int encoder_forward_impl(const float* x, const uint8_t* pad, int B, int T, const float* w1, const float* b1,
                         int precision, void* workspace, hipStream_t stream, const DadWs& L, float* vlen_out,
                         float* e_out) {
  uint16_t* w1h = ws_ptr<uint16_t>(workspace, L.w1h);
  const bool f16 = precision == DAD_PREC_FP16;
  if (dad_prec16(precision)) {
    hipLaunchKernelGGL(dad_w1h_kernel, dim3((DAD_H * DAD_D + 255) / 256), dim3(256), 0, stream, w1, w1h, f16 ? 1 : 0);
    DAD_TRY(hipGetLastError());
  }
  const DadGeom G = dad_geom(B, T, 0, 0);
  DadEncodeArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.g = G; ea.warmup = 1;
  ea.xc = x; ea.mc = pad; ea.w1_student = w1; ea.b1_student = b1; ea.w1h_student = w1h;
  ea.part_sum = ws_ptr<float>(workspace, L.part_sum);
  ea.part_cnt = ws_ptr<float>(workspace, L.part_cnt);
  ea.bits = ws_ptr<uint32_t>(workspace, L.bits);
  const dim3 egrid((B * G.ncc + 3) / 4);
  if (dad_prec16(precision)) {
    // the rows of x prepared (16-bit conversion: a clean-only set), then the GEMM on them
    DadPrepArgs pp;
    memset(&pp, 0, sizeof(pp));
    pp.g = G; pp.warmup = 1; pp.clean = 1; pp.f16 = f16 ? 1 : 0; pp.xc = x;
    pp.x16 = ws_ptr<uint16_t>(workspace, L.xs16);
    const int rp = launch_prep(pp, stream);
    if (rp) return rp;
    ea.x16c = pp.x16;
    int cus = 0;
    const int rc = device_cus(&cus);
    if (rc) return rc;
    const int rs = wp_split(G, 0, cus, ea.ws_nt, ea.ws_ns);
    if (rs) return rs;
    const dim3 grid(ea.ws_nt + ea.ws_ns);
    if (f16) hipLaunchKernelGGL(dad_encode_wp_f16, grid, dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
    else hipLaunchKernelGGL(dad_encode_wp, grid, dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
  } else {
    hipLaunchKernelGGL(dad_encode_f32, egrid, dim3(DAD_ENC_F32_THREADS), 0, stream, ea);
  }
  DAD_TRY(hipGetLastError());
  if (e_out) {
    hipLaunchKernelGGL(dad_embed_kernel, dim3(B), dim3(256), 0, stream, ea.part_sum, pad, B, T, G.ncc, vlen_out,
                       e_out);
    DAD_TRY(hipGetLastError());
  }
  return DAD_OK;
}

__global__ __launch_bounds__(256) void dad_embed_len_kernel(const uint8_t* pad, int B, int T, int nchunk,
                                                            const float* part_cnt, float* vlen, float* cnt_tot) {
  __shared__ float red[4];
  const int b = blockIdx.x, h = threadIdx.x;
  float l = 0.0f;
  for (int t = h; t < T; t += 256) l += pad[(size_t)b * T + t] == 0 ? 1.0f : 0.0f;
  l = dad_wave_sum(l);
  if ((h & 63) == 0) red[h >> 6] = l;
  __syncthreads();
  if (h == 0) vlen[b] = ((red[0] + red[1]) + red[2]) + red[3];
  float cnt = 0.0f;
  for (int c = 0; c < nchunk; ++c) cnt += part_cnt[((size_t)b * nchunk + c) * DAD_H + h];
  cnt_tot[(size_t)b * DAD_H + h] = cnt;
}

}  // namespace

extern "C" {

int dad_encoder_forward(const float* x, const uint8_t* pad, int B, int T, const float* w1, const float* b1,
                        float* e_out, int precision, void* workspace, void* stream) {
  if (!x || !pad || !w1 || !b1 || !e_out || !workspace) return DAD_E_ARG;
  if (B < 1 || B > DAD_MAX_BATCH || T < 1) return DAD_E_SHAPE;
  if (precision != DAD_PREC_FP32 && !dad_prec16(precision)) return DAD_E_ARG;
  const DadGeom G = dad_geom(B, T, 0, 0);
  const DadWs L = enc_layout(G);
  return encoder_forward_impl(x, pad, B, T, w1, b1, precision, workspace, (hipStream_t)stream, L,
                              ws_ptr<float>(workspace, L.vlen), e_out);
}

int dad_encoder_backward(const float* x, const uint8_t* pad, int B, int T, const float* w1, const float* b1,
                         const float* de, float* dw1, float* db1, void* workspace, void* stream_) {
  if (!x || !pad || !w1 || !b1 || !de || !dw1 || !db1 || !workspace) return DAD_E_ARG;
  if (B < 1 || B > DAD_MAX_BATCH || T < 1) return DAD_E_SHAPE;
  hipStream_t stream = (hipStream_t)stream_;
  const DadGeom G = dad_geom(B, T, 0, 0);
  const DadWs L = enc_layout(G);
  const int splits = L.splits;
  float* vlen = ws_ptr<float>(workspace, L.vlen);
  // recompute the ReLU'/valid bits and per-slab active counts (FP32 forward)
  int rc = encoder_forward_impl(x, pad, B, T, w1, b1, DAD_PREC_FP32, workspace, stream, L, nullptr, nullptr);
  if (rc) return rc;
  float* cnt_tot = ws_ptr<float>(workspace, L.cnt_tot);
  hipLaunchKernelGGL(dad_embed_len_kernel, dim3(B), dim3(256), 0, stream, pad, B, T, G.ncc,
                     ws_ptr<float>(workspace, L.part_cnt), vlen, cnt_tot);
  DAD_TRY(hipGetLastError());
  DadWgradArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.g = G; wa.warmup = 1; wa.splits = splits; wa.ntiles = 6 * splits;
  wa.xc = x; wa.bits = ws_ptr<uint32_t>(workspace, L.bits); wa.ge = de; wa.vlen = vlen;
  wa.wpart = ws_ptr<float>(workspace, L.wpart);
  DadReduceArgs none;
  memset(&none, 0, sizeof(none));
  hipLaunchKernelGGL(dad_wgrad_f32, dim3(6 * splits), dim3(DAD_WGRAD_THREADS), 0, stream, wa, none);
  DAD_TRY(hipGetLastError());
  float* gflat = ws_ptr<float>(workspace, L.gflat);
  DadReduceArgs ra;
  memset(&ra, 0, sizeof(ra));
  ra.g = G; ra.splits = splits; ra.warmup = 1; ra.want_norm = 0;
  ra.wpart = wa.wpart; ra.ge = de; ra.vlen = vlen; ra.cnt_tot = cnt_tot;
  ra.tailf = nullptr; ra.grad = gflat; ra.normpart = ws_ptr<float>(workspace, L.normpart);
  hipLaunchKernelGGL(dad_reduce, dim3(DAD_REDUCE_BLOCKS), dim3(DAD_REDUCE_THREADS), 0, stream, ra);
  DAD_TRY(hipGetLastError());
  DAD_TRY(hipMemcpyAsync(dw1, gflat + DAD_OFF_W1, sizeof(float) * DAD_H * DAD_D, hipMemcpyDeviceToDevice, stream));
  DAD_TRY(hipMemcpyAsync(db1, gflat + DAD_OFF_B1, sizeof(float) * DAD_H, hipMemcpyDeviceToDevice, stream));
  return DAD_OK;
}

}  // extern "C"
