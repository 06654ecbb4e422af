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
  if (c->precision != DAD_PREC_FP32 && c->precision != DAD_PREC_BF16) return DAD_E_ARG;
  if (c->rng_mode != DAD_RNG_EXPLICIT && c->rng_mode != DAD_RNG_COUNTER) return DAD_E_ARG;
  if (c->dp_world < 1) return DAD_E_ARG;
  return DAD_OK;
}

inline DadGeom geom_of(const dad_config* c) { return dad_geom(c->B, c->T, c->Bn, c->Tn); }

inline int splits_of(const dad_config* c) {
  const DadGeom g = geom_of(c);
  if (c->splits <= 0) return dad_auto_splits(g, c->precision, c->warmup);
  if (c->precision != DAD_PREC_BF16) return c->splits;
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

// Second stream per device for work that only depends on the forward: the
// loss-independent factor S_u of the weight gradient runs there while pool/tail/ECDA
// (a handful of workgroups) run on the caller's stream.  Fork/join by events, so the
// step stays enqueue-only and graph-capturable.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  int cus = 0;   // compute units of the device
};
// CUs the side-stream GEMM leaves free, so the caller-stream kernels that run meanwhile
// (pool, the one-workgroup tail, ECDA's per-class workgroups) are dispatched at once
// instead of waiting for a register file to drain
constexpr int kReservedCUs = 32;   // 4 per XCD (workgroups are spread round-robin over the 8 XCDs)
constexpr int kMaxDevices = 64;
SideStream g_side[kMaxDevices];
std::mutex g_side_mu;

int side_stream(SideStream** out) {
  int dev = 0;
  DAD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return DAD_E_ARG;
  std::lock_guard<std::mutex> lk(g_side_mu);
  SideStream& ss = g_side[dev];
  if (!ss.s) {
    DAD_TRY(hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking));
    DAD_TRY(hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming));
    DAD_TRY(hipEventCreateWithFlags(&ss.join, hipEventDisableTiming));
    DAD_TRY(hipDeviceGetAttribute(&ss.cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  *out = &ss;
  return DAD_OK;
}

// BF16 weight-gradient strategy: the direct GEMM after the losses (default), or the factorised
// S_u GEMM on the side stream (DAD_WGRAD=su, read per step).  Measured on MI355X the
// side-stream fork/join latency (~7 + ~12 us) cancels the overlap, so direct is the default.
bool wgrad_direct() {
  const char* e = getenv("DAD_WGRAD");
  return !(e && strcmp(e, "su") == 0);
}
// FP32: likewise the direct split-K GEMM after the losses (default), or S_u per utterance on
// the side stream (DAD_WGRAD_F32=su).  S_u costs 98 MB written and read again and its 768
// per-utterance tiles do not divide evenly over the CUs: measured 254 + 15 us against ~130 +
// 8 us for the direct form, which only loses the ~40 us of pool/tail overlap.
bool wgrad_f32_direct() {
  const char* e = getenv("DAD_WGRAD_F32");
  return !(e && strcmp(e, "su") == 0);
}

// DAD_POOL_FUSE=1: the BF16 encoder pools the slab partials in its own launch (last arriver per
// utterance) instead of a dad_pool launch.  Off by default: measured 2.7 us per step slower
// (encode_ws.hip, ws_pool_arrive).  Read once.
bool pool_fuse_on() {
  static const bool on = [] { const char* e = getenv("DAD_POOL_FUSE"); return e && strcmp(e, "1") == 0; }();
  return on;
}

// DAD_TAIL_W=0 selects the general tail + ECDA launch for every batch (A/B runs; read once)
bool tail_w_on() {
  static const bool on = [] { const char* e = getenv("DAD_TAIL_W"); return !(e && strcmp(e, "0") == 0); }();
  return on;
}

int device_cus(int* out) {
  static int cache[kMaxDevices];
  int dev = 0;
  DAD_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) return DAD_E_ARG;
  if (!cache[dev]) DAD_TRY(hipDeviceGetAttribute(&cache[dev], hipDeviceAttributeMultiprocessorCount, dev));
  *out = cache[dev];
  return DAD_OK;
}

// Workgroup split of the W-stationary encoder (encode_ws.hip): one persistent workgroup per
// CU, teacher : student in proportion to their work (32-row slab costs: clean 1, weak
// kWsWeak, strong kWsStrong -- the augmentation RNG dominates a noisy slab), more
// workgroups than CUs only when a range would exceed DAD_ENC_WS_MAXJ jobs.
constexpr float kWsWeak = 1.03f, kWsStrong = 1.55f;   // sweeps of 300-step benches (tools/gpu_ws_sweep.sh)
// DAD_WS_WEIGHTS="weak,strong" overrides the two costs (tuning runs; read once per process)
struct WsWeights { float weak, strong; };
WsWeights ws_weights() {
  static const WsWeights w = [] {
    WsWeights v{kWsWeak, kWsStrong};
    if (const char* e = getenv("DAD_WS_WEIGHTS")) {
      float a = 0.0f, b = 0.0f;
      if (sscanf(e, "%f,%f", &a, &b) == 2 && a > 0.0f && b > 0.0f) v = WsWeights{a, b};
    }
    return v;
  }();
  return w;
}
// DAD_WS_TABLE=1 turns the student range table on (off by default: at B=64, T=300 it brings the
// modelled slowest student range from 18.6 to 17.5 clean-sub-slab units, but the launch measured
// unchanged (62.7 vs 63.0 us) in A/B runs; read once per process)
bool ws_table_on() {
  static const bool on = [] { const char* e = getenv("DAD_WS_TABLE"); return e && strcmp(e, "1") == 0; }();
  return on;
}
// the largest job range of the teacher (or student) workgroups of a split, by the kernel's own
// range function (dad_ws_job_range)
int ws_max_range(const DadGeom& G, int Bn, int nt, int ns, float wstrong, bool teacher_side) {
  const int Js = Bn * G.ncn;
  int worst = 0;
  const int lo = teacher_side ? 0 : nt, hi = teacher_side ? nt : nt + ns;
  for (int wg = lo; wg < hi; ++wg) {
    bool t = false;
    int j0 = 0, j1 = 0;
    dad_ws_job_range(wg, nt, ns, wstrong, G.Bc, G.Tc, G.ncc, Bn, G.Tn, G.ncn, Js, t, j0, j1);
    worst = std::max(worst, j1 - j0);
  }
  return worst;
}
// Returns DAD_E_SHAPE if no split keeps every range within DAD_ENC_WS_MAXJ jobs (cannot happen
// for B <= DAD_MAX_BATCH: one job per workgroup always fits).
int ws_split(const DadGeom& G, int Bn, int cus, int& nt, int& ns) {
  const float kWsWeak = ws_weights().weak, kWsStrong = ws_weights().strong;
  const int Jt = Bn * G.ncn, Jc = G.Bc * G.ncc, Js = Jt;
  if (Jt == 0) {
    nt = 0;
    ns = std::min(cus, Jc);
  } else {
    const double tot = Jt * (double)kWsWeak + Jc + Js * (double)kWsStrong;
    nt = (int)(cus * (Jt * (double)kWsWeak) / tot + 0.5);
    nt = std::max(1, std::min(cus - 1, nt));
    ns = cus - nt;
    nt = std::min(nt, Jt);
    ns = std::min(ns, Jc + Js);
  }
  // every range within DAD_ENC_WS_MAXJ jobs (the kernel's valid-bit table), checked with the
  // kernel's range function: ranges are priced by live sub-slabs, so a job-count bound is not
  // enough when clean and strong jobs hold different numbers of live sub-slabs (Tc != Tn)
  nt = std::max(nt, (Jt + DAD_ENC_WS_MAXJ - 1) / DAD_ENC_WS_MAXJ);
  ns = std::max(ns, (Jc + Js + DAD_ENC_WS_MAXJ - 1) / DAD_ENC_WS_MAXJ);
  while (nt > 0 && ws_max_range(G, Bn, nt, ns, kWsStrong, true) > DAD_ENC_WS_MAXJ) {
    if (++nt > Jt) return DAD_E_SHAPE;
  }
  while (ws_max_range(G, Bn, nt, ns, kWsStrong, false) > DAD_ENC_WS_MAXJ) {
    if (++ns > Jc + Js) return DAD_E_SHAPE;
  }
  return DAD_OK;
}

// Student ranges of the W-stationary encoder by a min-max assignment: every student workgroup
// takes a contiguous run of strong jobs, then a contiguous run of clean jobs, filled up to a
// common cost bound T (jobs priced by live 16-row sub-slabs: clean 1, strong wstrong); the
// smallest T that places every job in ns workgroups (bisection).  The clean jobs (cost 2 or 1)
// fill what the coarser strong jobs (2 wstrong) leave, so the slowest range sits about half a
// clean job above the mean instead of up to a strong job (ws_split's contiguous ranges).
// Cached per geometry: computed once, then copied into each launch's arguments.
bool ws_student_table(const DadGeom& G, int Bn, int ns, float wstrong, DadEncodeArgs& ea) {
  const int Jc = G.Bc * G.ncc, Js = Bn * G.ncn;
  ea.ws_tab_n = 0;
  if (ns <= 0 || ns > DAD_WS_TAB || Jc + Js == 0 || Jc > 65535 || Js > 65535) return false;
  struct Key { int Bc, Tc, Bn, Tn, ns; float w; };
  static thread_local Key key{-1, -1, -1, -1, -1, 0.0f};
  static thread_local uint16_t tab[DAD_WS_TAB][4];
  const Key k{G.Bc, G.Tc, Bn, G.Tn, ns, wstrong};
  if (!(key.Bc == k.Bc && key.Tc == k.Tc && key.Bn == k.Bn && key.Tn == k.Tn && key.ns == k.ns && key.w == k.w)) {
    auto live = [](int c, int T) { return (c * DAD_SLAB + 16 < T) ? 2 : 1; };   // live sub-slabs of slab c
    auto cs = [&](int j) { return wstrong * (float)live(j % G.ncn, G.Tn); };
    auto cc = [&](int j) { return (float)live(j % G.ncc, G.Tc); };
    // greedy fill to T; returns the workgroups used (ns + 1 when T is too small)
    auto fill = [&](float T, bool write) {
      int sp = 0, cp = 0, k = 0;
      for (; k < ns && (sp < Js || cp < Jc); ++k) {
        float cost = 0.0f;
        const int s0 = sp, c0 = cp;
        while (sp < Js && sp - s0 < DAD_ENC_WS_MAXJ - 2 && cost + cs(sp) <= T) cost += cs(sp++);
        while (cp < Jc && (sp - s0) + (cp - c0) < DAD_ENC_WS_MAXJ - 2 && cost + cc(cp) <= T) cost += cc(cp++);
        if (sp == s0 && cp == c0) return ns + 1;   // a single job above T
        if (write) { tab[k][0] = (uint16_t)s0; tab[k][1] = (uint16_t)sp; tab[k][2] = (uint16_t)c0; tab[k][3] = (uint16_t)cp; }
      }
      if (sp < Js || cp < Jc) return ns + 1;
      if (write)
        for (int r = k; r < ns; ++r) { tab[r][0] = tab[r][1] = (uint16_t)Js; tab[r][2] = tab[r][3] = (uint16_t)Jc; }
      return k;
    };
    float tot = 0.0f, jmax = 0.0f;
    for (int j = 0; j < Js; ++j) { tot += cs(j); jmax = std::max(jmax, cs(j)); }
    for (int j = 0; j < Jc; ++j) { tot += cc(j); jmax = std::max(jmax, cc(j)); }
    float lo = tot / (float)ns, hi = lo + 2.0f * jmax + 1.0f;
    if (fill(hi, false) > ns) return false;
    for (int it = 0; it < 24; ++it) {
      const float mid = 0.5f * (lo + hi);
      if (fill(mid, false) <= ns) hi = mid; else lo = mid;
    }
    fill(hi, true);
    key = k;
  }
  memcpy(ea.ws_tab, tab, sizeof(uint16_t) * 4 * (size_t)ns);
  ea.ws_tab_n = ns;
  return true;
}

// Per-kernel timing of the fused step (dad_timing_start / dad_timing_stop): every `every`-th
// step (counted at its encoder call) records hip events at the kernel boundaries of the
// caller's stream (and around the side-stream GEMM of the FP32 step).  Events are created up
// front by dad_timing_start, so a timed region only records them.  Not for graph capture.
enum { TK_E0, TK_E1, TK_POOL, TK_TAIL, TK_WGRAD, TK_RED, TK_OPT0, TK_OPT1, TK_S0, TK_S1, TK_N };
// (event-pair points of each DAD_TK_* kernel: dad_timing_stop's pairs)
const int kTkPairs[DAD_TK_KERNELS][2] = {{TK_E0, TK_E1}, {TK_E1, TK_POOL}, {TK_POOL, TK_TAIL}, {TK_TAIL, TK_WGRAD},
                                         {TK_WGRAD, TK_RED}, {TK_OPT0, TK_OPT1}, {TK_S0, TK_S1}};
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

int dad_timing_start(int every, int max_steps) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  if (every < 1 || max_steps < 1) return DAD_E_ARG;
  for (hipEvent_t e : g_tk.ev) (void)hipEventDestroy(e);
  g_tk = Timing();
  g_tk.ev.assign((size_t)max_steps * TK_N, nullptr);
  g_tk.rec.assign((size_t)max_steps * TK_N, 0);
  for (auto& e : g_tk.ev) DAD_TRY(hipEventCreate(&e));
  g_tk.every = every;
  g_tk.nset = max_steps;
  return DAD_OK;
}

int dad_timing_kernels(unsigned mask) {
  std::lock_guard<std::mutex> lk(g_tk_mu);
  unsigned pts = 0;
  for (int k = 0; k < DAD_TK_KERNELS; ++k)
    if ((mask >> k) & 1u) pts |= (1u << kTkPairs[k][0]) | (1u << kTkPairs[k][1]);
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
      const int a = pairs[k][0], z = pairs[k][1];
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
  rc = ws_split(G, Bn, cus, *nt, *ns);
  if (rc) return rc;
  const float ws = ws_weights().strong;
  *max_jobs = std::max(ws_max_range(G, Bn, *nt, *ns, ws, true), ws_max_range(G, Bn, *nt, *ns, ws, false));
  return DAD_OK;
}

int dad_workspace_bytes(const dad_config* cfg, size_t* bytes) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!bytes) return DAD_E_ARG;
  *bytes = dad_ws_layout(geom_of(cfg), max_splits_of(cfg), cfg->precision).bytes;
  return DAD_OK;
}

}  // extern "C"

static int step_compute_phases(const dad_config* cfg, const dad_batch* bt, const dad_state* st, void* workspace,
                               void* stream_, bool do_encode, bool do_backward) {
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
  __bf16* xs_bf16 = ws_ptr<__bf16>(workspace, L.xs_bf16);
  const bool bf16 = cfg->precision == DAD_PREC_BF16;

  // pooling arguments (dad_pool, or the BF16 encoder's in-launch pooling)
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
  // (split calls: the encode call pooled, so the backward call launches no dad_pool)
  const bool pool_fused = bf16 && pool_fuse_on();

  // 1. fused augmentation + encoder GEMMs + pooling partials
  DadEncodeArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.g = G; ea.warmup = cfg->warmup;
  ea.mask_len = cfg->mask_len; ea.start_hi = cfg->start_hi;
  ea.xc = bt->xc; ea.mc = bt->mc; ea.xn = bt->xn; ea.mn = bt->mn; ea.src = src;
  ea.w1_student = st->student + DAD_OFF_W1; ea.b1_student = st->student + DAD_OFF_B1;
  ea.w1_teacher = st->teacher + DAD_OFF_W1; ea.b1_teacher = st->teacher + DAD_OFF_B1;
  ea.w1bf_student = reinterpret_cast<const __bf16*>(st->w1bf_student);
  ea.w1bf_teacher = reinterpret_cast<const __bf16*>(st->w1bf_teacher);
  if (explicit_rng) { ea.nw = bt->nw; ea.ns = bt->ns; ea.u = bt->u; ea.start = bt->start; }
  ea.key_weak = k.weak; ea.key_strong = k.strong; ea.key_feat = k.feat; ea.key_tstart = k.tstart;
  ea.weak_std = cfg->weak_std; ea.strong_std = cfg->strong_std; ea.feat_p = cfg->feat_p;
  ea.part_sum = part_sum; ea.part_cnt = part_cnt; ea.bits = bits; ea.xs_bf16 = xs_bf16;
  if (pool_fused) { ea.pool = pa; ea.pool_cnt = ws_ptr<uint32_t>(workspace, L.pool_cnt); }
  const int nwaves = G.Bc * G.ncc + Bn * G.ncn;
  const dim3 egrid((nwaves + 3) / 4);
  if (do_encode) {
    tk_begin();
    tk_mark(TK_E0, stream);
    if (bf16) {
      int cus = 0;
      const int rc = device_cus(&cus);
      if (rc) return rc;
      const int rs = ws_split(G, Bn, cus, ea.ws_nt, ea.ws_ns);
      if (rs) return rs;
      ea.ws_wstrong = ws_weights().strong;
      if (ws_table_on()) ws_student_table(G, Bn, ea.ws_ns, ea.ws_wstrong, ea);
      if (ea.ws_nt + ea.ws_ns > 0) {
        if (explicit_rng) hipLaunchKernelGGL(dad_encode_ws_explicit, dim3(ea.ws_nt + ea.ws_ns), dim3(DAD_ENC_WS_THREADS), 0,
                                             stream, ea);
        else hipLaunchKernelGGL(dad_encode_ws, dim3(ea.ws_nt + ea.ws_ns), dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
      }
    } else {
      hipLaunchKernelGGL(dad_encode_f32, egrid, dim3(DAD_ENC_F32_THREADS), 0, stream, ea);
    }
    DAD_TRY(hipGetLastError());
    tk_mark(TK_E1, stream);
  }
  if (!do_backward) return DAD_OK;

  // 2. The loss-independent factor of dW1 on the side stream, S_u = bits_u^T X_u per
  //    utterance (clean rows, then the strong-augmented noisy rows; BF16: the encoder's bf16
  //    copies, S_u stored in bf16), concurrent with 3-5, for FP32 and for BF16 with DAD_WGRAD=su.
  //    BF16 default: one direct GEMM after ECDA (6) with dL/de folded into its A operand.
  const int nutt = G.Bc + Bn;
  float* sbuf = ws_ptr<float>(workspace, L.sbuf);
  DadWgradArgs wa;
  memset(&wa, 0, sizeof(wa));
  wa.g = G; wa.warmup = cfg->warmup;
  wa.mask_len = cfg->mask_len; wa.start_hi = cfg->start_hi;
  wa.xc = bt->xc; wa.xn = bt->xn; wa.src = src;
  if (explicit_rng) { wa.ns = bt->ns; wa.u = bt->u; wa.start = bt->start; }
  wa.key_strong = k.strong; wa.key_feat = k.feat; wa.key_tstart = k.tstart;
  wa.strong_std = cfg->strong_std; wa.feat_p = cfg->feat_p;
  wa.bits = bits; wa.ge = ge; wa.vlen = vlen; wa.xs_bf16 = xs_bf16;
  SideStream* side = nullptr;
  const bool factorised = bf16 ? !wgrad_direct() : !wgrad_f32_direct();
  if (factorised) {
    const int rc = side_stream(&side);
    if (rc) return rc;
    wa.splits = nutt; wa.per_utt = 1; wa.wpart = sbuf;
    DAD_TRY(hipEventRecord(side->fork, stream));
    DAD_TRY(hipStreamWaitEvent(side->s, side->fork, 0));
    tk_mark(TK_S0, side->s);
    if (bf16) {
      wa.su = reinterpret_cast<__bf16*>(sbuf);
      wa.ntiles = WGD_NDB * nutt;
      const int sgrid = std::max(1, std::min(wa.ntiles, side->cus - kReservedCUs));
      hipLaunchKernelGGL(dad_wgrad_su, dim3(sgrid), dim3(WGD_THREADS), 0, side->s, wa);
    } else {
      wa.ntiles = 6 * nutt;
      const int sgrid = std::max(1, std::min(wa.ntiles, side->cus - kReservedCUs));
      DadReduceArgs none;
      memset(&none, 0, sizeof(none));
      hipLaunchKernelGGL(dad_wgrad_f32, dim3(sgrid), dim3(DAD_WGRAD_THREADS), 0, side->s, wa, none);
    }
    DAD_TRY(hipGetLastError());
    tk_mark(TK_S1, side->s);
    DAD_TRY(hipEventRecord(side->join, side->s));
  }

  // 3. pooled embeddings + classifier logits (BF16: pooled inside the encoder launch)
  if (!pool_fused) {
    hipLaunchKernelGGL(dad_pool, dim3(G.Bc + 2 * Bn), dim3(DAD_POOL_THREADS), 0, stream, pa);
    DAD_TRY(hipGetLastError());
  }
  tk_mark(TK_POOL, stream);

  // 4. losses, DACP mask, analytic backward to dL/de and the classifier grads
  DadTailArgs ta;
  memset(&ta, 0, sizeof(ta));
  ta.cfg = *cfg; ta.yc = bt->yc; ta.logits = st->logits; ta.emb = st->emb; ta.student = st->student;
  if (explicit_rng) { ta.keep1 = bt->keep1; ta.keep2 = bt->keep2; }
  ta.key_drop1 = k.drop1; ta.key_drop2 = k.drop2;
  ta.dacp = st->dacp; ta.tailf = st->tail; ta.ge = ge; ta.ge_ecda = ge_ecda; ta.grad = st->grad;
  ta.gzb = gzb; ta.eflag = eflag;
  // 5. ECDA (class-aware MMD + compactness + repulsion) and its embedding grads: after the
  //    warm-up, in the same launch as the tail (block 0 = tail, blocks 1..C = classes)
  DadEcdaArgs ca;
  memset(&ca, 0, sizeof(ca));
  ca.cfg = *cfg; ca.yc = bt->yc; ca.emb = st->emb; ca.tailf = st->tail;
  ca.tail_terms = st->tail + DAD_T_ECDA_TERM; ca.ge = ge_ecda; ca.scratch = ecda_scratch; ca.eflag = eflag;
  ca.sink = ws_ptr<float>(workspace, L.gflat);
  if (!cfg->warmup && DAD_FUSED_TAIL) {
    // batches of at most 64 utterances per side, class-aware MMD: the wave-centric launch
    if (G.Bc <= 64 && Bn <= 64 && cfg->class_aware && tail_w_on())
      hipLaunchKernelGGL(dad_tail_ecda_w, dim3(1 + DAD_C), dim3(DAD_TAIL_THREADS), 0, stream, ta, ca);
    else
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
  // 6. dW1 (join, then sum_u (dL/de_u / len_u) * S_u; or the direct split-K GEMM), db1,
  //    dW2, loss totals, squared-norm partials
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
  if (!factorised && !bf16) {
    // FP32 direct: G = ReLU' * dL/de / len rebuilt per slab from the tail's dL/dz and the
    // ECDA rows; one tile = (split, 128 columns); then every reduce block (dW1 sums and the
    // db1 / dW2 / totals blocks)
    wa.splits = splits; wa.per_utt = 0;
    wa.wpart = ws_ptr<float>(workspace, L.wpart);
    wa.ntiles = 6 * splits;
    hipLaunchKernelGGL(dad_wgrad_f32, dim3(wa.ntiles), dim3(DAD_WGRAD_THREADS), 0, stream, wa, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_WGRAD, stream);
    ra.splits = splits; ra.wpart = wa.wpart;
    hipLaunchKernelGGL(dad_reduce, dim3(DAD_REDUCE_BLOCKS), dim3(DAD_REDUCE_THREADS), 0, stream, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_RED, stream);
  } else if (!factorised) {
    wa.splits = splits; wa.per_utt = 0;
    wa.wpart = ws_ptr<float>(workspace, L.wpart);
    wa.ntiles = WGD_NDB * splits;
    // multiple of 8 (XCD-aware tile order) with WGD_XWG spare workgroups for the extra blocks
    const int grid = (wa.ntiles + WGD_XWG + 7) / 8 * 8;
    hipLaunchKernelGGL(dad_wgrad_direct, dim3(grid), dim3(WGD_THREADS), 0, stream, wa, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_WGRAD, stream);
    ra.splits = splits; ra.wpart = wa.wpart;
    hipLaunchKernelGGL(dad_reduce_w, dim3(DAD_REDUCE_BLOCKS - DAD_REDUCE_XBLK), dim3(64), 0, stream, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_RED, stream);
  } else {
    DAD_TRY(hipStreamWaitEvent(stream, side->join, 0));
    ra.splits = nutt; ra.wpart = sbuf;
    if (bf16) ra.su = wa.su;
    hipLaunchKernelGGL(dad_wsum, dim3(DAD_REDUCE_BLOCKS), dim3(DAD_REDUCE_THREADS), 0, stream, ra);
    DAD_TRY(hipGetLastError());
    tk_mark(TK_WGRAD, stream);
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
  oa.w1bf_student = reinterpret_cast<__bf16*>(st->w1bf_student);
  oa.w1bf_teacher = reinterpret_cast<__bf16*>(st->w1bf_teacher);
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

int dad_refresh_shadow(const dad_state* st, void* stream_) {
  if (!st || !st->student || !st->teacher || !st->w1bf_student || !st->w1bf_teacher) return DAD_E_ARG;
  hipLaunchKernelGGL(dad_shadow_kernel, dim3((DAD_H * DAD_D + 255) / 256), dim3(256), 0, (hipStream_t)stream_,
                     st->student, st->teacher, reinterpret_cast<__bf16*>(st->w1bf_student),
                     reinterpret_cast<__bf16*>(st->w1bf_teacher));
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

// The modular encoder ops' workspace: the FP32 layout plus the bf16 row-copy region, so the
// BF16 encoder writes its copies to scratch instead of testing for a missing buffer in the
// conversion units it interleaves with the MFMA k-steps (a branch there splits the schedule).
static DadWs enc_layout(const DadGeom& G) {
  return dad_ws_layout(G, dad_auto_splits(G, DAD_PREC_FP32, 1), DAD_PREC_BF16, false);
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

// bf16 copy of W1 in the W-stationary encoder's fragment order (dad_w1frag_index)
__global__ __launch_bounds__(256) void dad_w1bf_kernel(const float* w, __bf16* out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (size_t)DAD_H * DAD_D) out[dad_w1frag_index((uint32_t)(i / DAD_D), (uint32_t)(i % DAD_D))] = (__bf16)w[i];
}

int encoder_forward_impl(const float* x, const uint8_t* pad, int B, int T, const float* w1, const float* b1,
                         int precision, void* workspace, hipStream_t stream, const DadWs& L, float* vlen_out,
                         float* e_out) {
  __bf16* w1bf = ws_ptr<__bf16>(workspace, L.w1bf);
  if (precision == DAD_PREC_BF16) {
    hipLaunchKernelGGL(dad_w1bf_kernel, dim3((DAD_H * DAD_D + 255) / 256), dim3(256), 0, stream, w1, w1bf);
    DAD_TRY(hipGetLastError());
  }
  const DadGeom G = dad_geom(B, T, 0, 0);
  DadEncodeArgs ea;
  memset(&ea, 0, sizeof(ea));
  ea.g = G; ea.warmup = 1;
  ea.xc = x; ea.mc = pad; ea.w1_student = w1; ea.b1_student = b1; ea.w1bf_student = w1bf;
  ea.part_sum = ws_ptr<float>(workspace, L.part_sum);
  ea.part_cnt = ws_ptr<float>(workspace, L.part_cnt);
  ea.bits = ws_ptr<uint32_t>(workspace, L.bits);
  ea.xs_bf16 = ws_ptr<__bf16>(workspace, L.xs_bf16);
  const dim3 egrid((B * G.ncc + 3) / 4);
  if (precision == DAD_PREC_BF16) {
    int cus = 0;
    const int rc = device_cus(&cus);
    if (rc) return rc;
    const int rs = ws_split(G, 0, cus, ea.ws_nt, ea.ws_ns);
    if (rs) return rs;
    ea.ws_wstrong = ws_weights().strong;
    hipLaunchKernelGGL(dad_encode_ws, dim3(ea.ws_nt + ea.ws_ns), dim3(DAD_ENC_WS_THREADS), 0, stream, ea);
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
  if (precision != DAD_PREC_FP32 && precision != DAD_PREC_BF16) return DAD_E_ARG;
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
