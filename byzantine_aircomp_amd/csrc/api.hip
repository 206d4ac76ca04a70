// C ABI of libgmagg.so (include/gmagg.h): contexts, workspace, the Weiszfeld
// host loop, OMA and the synthetic fills.
//
// The host loop mirrors the reference's control flow (MNIST_Air_weight.py:145-160
// for gm, 173-184 for gm2) but keeps every decision on the device: the
// K-space kernel sets a `done` word that makes later launches no-ops, and the
// host only polls it every `check_every` iterations.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gmagg.h"
#include "gmagg_internal.h"

using namespace gmk;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(GM_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                  __FILE__, __LINE__);                                                  \
  } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace


struct gm_ctx {
  int device = 0;
  int num_cu = 256;
  int64_t d_total = -1;   // -1: unsharded
  int64_t d_offset = 0;
  gm_allreduce_cb ar_fn = nullptr;
  void* ar_user = nullptr;
  ncclComm_t comm = nullptr;
  char* ws = nullptr;
  size_t ws_bytes = 0;
  char* host = nullptr;   // pinned: KState mirror + host-noise staging
  size_t host_bytes = 0;
  bool timing = false;
  hipEvent_t poll_ev[2] = {nullptr, nullptr};   // lagged convergence polls
  std::vector<hipEvent_t> ev_free;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_used;
  // Workspace ordering across streams: every call that touches ws / host records
  // ws_ev on its stream when it returns (work may still be queued: the lagged
  // poll returns before the no-op tail drains); a call on ANOTHER stream waits
  // for it before zeroing or overwriting the workspace.
  hipEvent_t ws_ev = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_pending = false;
  float* stage = nullptr;   // panel copy of a row-major client matrix (gm_weiszfeld_f32)
  size_t stage_bytes = 0;
  // A register-resident grid that failed its co-residency check-in (device_util.h
  // grid_checkin: a shared GPU, CUs held by another stream) makes the next calls stream
  // straight away instead of paying the check-in's 100 ms again; retried after this many.
  int res_skip = 0;
  // the last Krum call (gm_krum_last_info): {algorithm, candidates, reason}
  int64_t krum_info[3] = {GM_KRUM_EXACT, 0, GM_KRUM_REASON_NOT_CHOSEN};
};

namespace {

constexpr int kResSkipAfterCheckinFail = 64;

// Resident paths are tried unless a recent call's grid failed its check-in.  Called ONCE
// per public call (gm_weiszfeld_f32, gm_weiszfeld_batched_f32), so the skip window lasts
// kResSkipAfterCheckinFail calls however many resident paths a call considers.
bool resident_allowed(gm_ctx* c) {
  if (c->res_skip <= 0) return true;
  --c->res_skip;
  return false;
}

// GMAGG_RES_CHECKIN_FAIL=1: the check-in waits for one slot nobody writes, so it fails
// (tests of the fallback; read per call).
unsigned checkin_need(unsigned blocks) {
  const char* e = getenv("GMAGG_RES_CHECKIN_FAIL");
  return blocks + ((e && atoi(e) != 0) ? 1u : 0u);
}

// XCD placement of the resident grids (read per call).  The single-problem kernel's blocks
// all on one XCD when they fit its CUs (stride 8: only blocks b % 8 == 0 work), its
// granules stored so that they stay in that XCD's L2 (GMAGG_RES_XCD=2, the default):
// C2 178.4 -> 227.3 aggregations/s (profiles/r4s2_xcd_local_ab.jsonl).  GMAGG_RES_XCD=1:
// the same placement with agent-scope (L2-dropping) stores, 172.9; 0: neither.  The batched
// kernel's groups are numbered XCD by XCD (GMAGG_RB_XCD=0 turns it off): a group of 49
// blocks spans 2-3 XCDs instead of 8, the AirComp exchange's traffic 259 -> 110 GB per
// 1024-problem launch, the prenoise sweep 70.5k -> 71.6k problems/s.
// (local stores only when the check-in confirms from XCC_ID that every block is on one XCD:
// resident.hip put_value; otherwise agent-scope stores, as for any placement)
int res_xcd_mode() {
  const char* e = getenv("GMAGG_RES_XCD");
  return e ? atoi(e) : 2;
}
// GMAGG_RB_HIER=1 (read per call): the batched resident kernel's groups gather by XCD
// (sub-group leaders, then the <= 3 sub-group sums) instead of flat over the group's 49
// blocks.  It cuts the C5 AirComp launch's HBM traffic 109.7 -> 33.8 GB (5.3x -> 1.65x the
// tile read) but measured slower — 818 -> 787 problems/s (AirComp), 70.3k -> 69.1k
// (prenoise): the exchange is latency-bound, not traffic-bound, and the leader's hop adds
// latency (profiles/r5s1_c5_rb_hier_ab.jsonl, r5s1_pmc_c5air_hier.txt).  Off by default.
int rb_hier_mode() {
  const char* e = getenv("GMAGG_RB_HIER");
  return e ? atoi(e) : 0;
}
// GMAGG_RES_SPLIT (read per call): 1 (default) the split-scope exchange for resident grids
// beyond one XCD that do not take the hierarchical gather (results bit-identical to the
// flat gather's; 50 x 20,000 6.03 -> 5.95 µs per iteration, 50 x 30,000 6.75 -> 6.62,
// 30 x 48,670 6.95 -> 6.77; profiles/r5s1_resident_split_ab.jsonl), 0 the flat gather
int res_split_mode() {
  const char* e = getenv("GMAGG_RES_SPLIT");
  return e ? atoi(e) : 1;
}
// GMAGG_RES_HIER (read per call): 1 (default) the XCD-hierarchical gather for resident grids
// beyond one XCD where it measured faster (>= 90 blocks, K > 32), 2 for every grid beyond
// one XCD, 0 never (the flat gather over every block)
int res_hier_mode() {
  const char* e = getenv("GMAGG_RES_HIER");
  return e ? atoi(e) : 1;
}
unsigned res_xcd_stride(int nb, int num_cu) {
  // GMAGG_RES_XCD_BPC=n (A/B): up to n blocks per CU of the one XCD
  static const int bpc = getenv("GMAGG_RES_XCD_BPC") ? std::max(1, atoi(getenv("GMAGG_RES_XCD_BPC"))) : 1;
  return (res_xcd_mode() != 0 && nb <= num_cu / 8 * bpc) ? 8u : 1u;
}
// GMAGG_RB_XCD: 0 round-robin numbering, 1 XCD-major (default), 2 XCD-major with whole
// groups per XCD whose granules stay in the XCD's L2 (resident_batched.hip rb_put)
// The single-problem resident kernel's tile (round 4 session 2): at 32 < K <= 64, 8 waves
// of 8 rows per lane (512-thread blocks) instead of the streaming tile's 16 waves of 4 —
// half the waves in every cross-wave reduction and block barrier of the iteration, the
// same 256 columns per block: C2 238.0 -> 281.2 aggregations/s (profiles/r4s2_c2_tile_ab.jsonl).
// GMAGG_RES_CFG="NW,R" forces a tile (LPR 64; NW * R >= K), e.g. "16,4" the previous one.
void resident_tile(PassCfg* cfg, int64_t K) {
  if (cfg->LPR != 64) return;
  int nw = 0, r = 0;
  if (const char* e = getenv("GMAGG_RES_CFG")) {
    if (sscanf(e, "%d,%d", &nw, &r) != 2 || (int64_t)nw * r < K) nw = 0;
  } else if (K > 32 && K <= 64 && cfg->NW == 16 && cfg->R == 4) {
    nw = 8;
    r = 8;
  }
  if (nw > 0) {
    cfg->NW = nw;
    cfg->R = r;
  }
}
int rb_xcd_major() {
  const char* e = getenv("GMAGG_RB_XCD");
  return e ? atoi(e) : 1;                 // 1 by default (round 4 A/B)
}

// Stream-orders the context's workspace between calls (see gm_ctx::ws_ev): the
// constructor makes `s` wait for the previous call's tail when that call ran on
// another stream; the destructor marks the end of this call's work on `s`.
struct WsOrder {
  gm_ctx* c;
  hipStream_t s;
  hipError_t err = hipSuccess;
  WsOrder(gm_ctx* c_, hipStream_t s_) : c(c_), s(s_) {
    if (!c->ws_ev) err = hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming);
    if (err == hipSuccess && c->ws_pending && c->ws_stream != s)
      err = hipStreamWaitEvent(s, c->ws_ev, 0);
  }
  ~WsOrder() {
    if (c->ws_ev && hipEventRecord(c->ws_ev, s) == hipSuccess) {
      c->ws_stream = s;
      c->ws_pending = true;
    }
  }
};

// The context's panel copy of a row-major client matrix (gm_weiszfeld_f32 /
// gm_weiszfeld_batched_f32 stage row-major AirComp inputs into it).  GMAGG_STAGE_PANELS=0
// turns staging off.  Returns false (and streams the rows) when the buffer cannot be had.
bool stage_enabled() {
  static const bool on = [] {
    const char* e = getenv("GMAGG_STAGE_PANELS");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

bool ensure_stage(gm_ctx* c, size_t bytes) {
  if (bytes <= c->stage_bytes) return true;
  if (c->stage) (void)hipFree(c->stage);   // (hipFree waits for queued work)
  c->stage = nullptr;
  c->stage_bytes = 0;
  if (hipMalloc(&c->stage, bytes) != hipSuccess) {
    (void)hipGetLastError();
    c->stage = nullptr;
    return false;
  }
  c->stage_bytes = bytes;
  return true;
}

struct Workspace {
  KState* st;
  double* sums;
  double* r;
  float* coef;
  double* slab;
  float* g[2];
  float* h_re;   // host-noise device copies
  float* h_im;
  float* hnoise; // d local + 1
  // Gram variant
  float* gslab;  // [blocks][tiles][1024] fp32 partial Grams
  double* G;     // [KP][KP]
  double* alpha;
  double* u;
};

int ensure_ws(gm_ctx* c, int64_t K, int64_t d, int nb, Workspace* w, size_t gram_slab_n = 0,
              int KP = 0) {
  const int64_t S = 2 * K + 2;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, 256); return o; };
  const size_t o_st = take(sizeof(KState));
  const size_t o_sums = take(sizeof(double) * S);
  const size_t o_r = take(sizeof(double) * K);
  const size_t o_coef = take(sizeof(float) * K);
  const size_t o_slab = take(sizeof(double) * S * (size_t)nb);
  const size_t o_g0 = take(sizeof(float) * d);
  const size_t o_g1 = take(sizeof(float) * d);
  const size_t o_hr = take(sizeof(float) * K);
  const size_t o_hi = take(sizeof(float) * K);
  const size_t o_hn = take(sizeof(float) * (d + 1));
  const size_t o_gs = take(sizeof(float) * gram_slab_n);
  const size_t o_G = take(sizeof(double) * (size_t)KP * KP);
  const size_t o_al = take(sizeof(double) * K);
  const size_t o_u = take(sizeof(double) * K);
  w->gslab = nullptr;
  if (off > c->ws_bytes) {
    if (c->ws) HIPCHK(hipFree(c->ws));
    c->ws = nullptr;
    c->ws_bytes = 0;
    HIPCHK(hipMalloc(&c->ws, off));
    c->ws_bytes = off;
  }
  char* b = c->ws;
  w->st = reinterpret_cast<KState*>(b + o_st);
  w->sums = reinterpret_cast<double*>(b + o_sums);
  w->r = reinterpret_cast<double*>(b + o_r);
  w->coef = reinterpret_cast<float*>(b + o_coef);
  w->slab = reinterpret_cast<double*>(b + o_slab);
  w->g[0] = reinterpret_cast<float*>(b + o_g0);
  w->g[1] = reinterpret_cast<float*>(b + o_g1);
  w->h_re = reinterpret_cast<float*>(b + o_hr);
  w->h_im = reinterpret_cast<float*>(b + o_hi);
  w->hnoise = reinterpret_cast<float*>(b + o_hn);
  w->gslab = reinterpret_cast<float*>(b + o_gs);
  w->G = reinterpret_cast<double*>(b + o_G);
  w->alpha = reinterpret_cast<double*>(b + o_al);
  w->u = reinterpret_cast<double*>(b + o_u);
  return GM_OK;
}

int ensure_host(gm_ctx* c, size_t bytes) {
  if (bytes <= c->host_bytes) return GM_OK;
  if (c->host) HIPCHK(hipHostFree(c->host));
  c->host = nullptr;
  c->host_bytes = 0;
  HIPCHK(hipHostMalloc(&c->host, bytes, hipHostMallocDefault));
  c->host_bytes = bytes;
  return GM_OK;
}

int allreduce(gm_ctx* c, double* buf, int64_t n, hipStream_t s) {
  if (c->comm) {
    ncclResult_t r = ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, c->comm, s);
    if (r != ncclSuccess) return fail(GM_ERR_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    return GM_OK;
  }
  if (c->ar_fn) {
    if (c->ar_fn(c->ar_user, buf, n, (void*)s) != 0)
      return fail(GM_ERR_CALLBACK, "all-reduce callback failed");
  }
  return GM_OK;
}

// Streaming-pass tile for K rows.
// The tile is K_pad x J with J = LPR*V columns; NRG = 16*64/LPR row groups of
// R rows each cover K.  Bigger K -> narrower chunk, so a block's tile (and the
// bytes it has in flight) stays ~64-128 KiB.
// panel: the tile of a panel-layout call (its chunk width is the panel width W).
bool pick_cfg(int64_t K, int V, int64_t ldx, PassCfg* cfg, bool panel = false) {
  int nw = 16, lpr, r, occ = 1;
  if (K <= 16) { lpr = 64; r = 1; }
  else if (K <= 32) { lpr = 64; r = 2; }
  // 32 < K <= 64 on panels (C5's K = 50 batched problems): 512-thread blocks of 64 x 128
  // chunks, 5.41-5.49 vs 5.07-5.13 TB/s per C5 STEP pass (profiles/history/r2_c5_panels.txt); rows
  // keep (16,64,4), whose 256-column chunks let C1/C2 stay register-resident
  else if (K <= 64) { if (panel) { nw = 8; lpr = 32; r = 4; } else { lpr = 64; r = 4; } }
  else if (K <= 128) { lpr = 64; r = 8; }
  // 128 < K <= 256 on panels: 256 x 64 chunks (W = 64, each chunk 64 KB contiguous),
  // STEP 2.38 vs 2.54 ms and the C4-shard Gram closing pass 2.58 vs 2.80 ms against the
  // 256 x 128 tile (profiles/history/r2_k256_tiles.txt); rows keep the 512-B row segments
  else if (K <= 256) { if (panel) { lpr = 16; r = 4; } else { lpr = 32; r = 8; } }
  else if (K <= 512) { lpr = 16; r = 8; }
  // K <= 1024: two 512-thread blocks per CU, each with a 1024 x 32 tile (128 B row
  // segments): 6.29 vs 6.05 TB/s for one 1024-thread block (profiles/history/r01_occ_sweep.txt)
  else if (K <= 1024) { nw = 8; lpr = 8; r = 16; occ = 2; }
  else if (K <= 2048) { lpr = 4; r = 8; }
  else return false;
  // GMAGG_PASS_CFG="NW,LPR,R[,OCC]" forces a tile (tuning runs); it must cover K.
  if (const char* e = getenv("GMAGG_PASS_CFG")) {
    int a = 0, b = 0, c2 = 0, o = 1;
    const int n = sscanf(e, "%d,%d,%d,%d", &a, &b, &c2, &o);
    if (n >= 3 && b > 0 && (int64_t)a * (64 / b) * c2 >= K) {
      nw = a; lpr = b; r = c2; occ = n == 4 ? o : 1;
    }
  }
  // lane offsets are 32-bit: (rows per wave - 1) * ldx + ldx must fit in bytes
  if ((uint64_t)(64 / lpr) * (uint64_t)ldx * 4u >= (1ull << 31)) return false;   // buffer offsets
  *cfg = PassCfg{V, nw, lpr, r, occ};
  return pass_cfg_supported(*cfg);
}

// Tile of the passes without phase A's weighted sum feeding phase B (INIT) or
// without phase B (the Gram closing pass): at 128 < K <= 256 the 1-KiB row
// segments of (16,64,16) beat the STEP tile (16,32,8): 2.81 / 2.76 vs 3.00 /
// 2.99 ms at K=256 x d=15.6M (profiles/history/r02_sweep_close.txt).
PassCfg light_cfg(int64_t K, const PassCfg& step) {
  if (getenv("GMAGG_PASS_CFG") || step.V != 4 || K <= 128 || K > 256) return step;
  const PassCfg c{4, 16, 64, 16, 1};
  return pass_cfg_supported(c) ? c : step;
}

int pick_vec(const float* X, int64_t d, int64_t ldx) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(X);
  if (d % 4 == 0 && ldx % 4 == 0 && p % 16 == 0) return 4;
  if (d % 2 == 0 && ldx % 2 == 0 && p % 8 == 0) return 2;
  return 1;
}

// PassArgs.chunk_pair for a row-major pass of `grid` blocks on tile `cfg`: the CU count when
// the grid is exactly two blocks per CU (GMAGG_CHUNK_PAIR=0: off, for A/B).  Only the 32-wave
// rows kernel reads it (the generic tile's chunk order, and so its sums, stay as they were)
int chunk_pair(const gm_ctx* c, const PassCfg& cfg, int64_t grid) {
  static const bool off = [] {
    const char* e = getenv("GMAGG_CHUNK_PAIR");
    return e && atoi(e) == 0;
  }();
  return !off && cfg.OCC == 2 && grid == 2 * (int64_t)c->num_cu ? c->num_cu : 0;
}

int record_pass_begin(gm_ctx* c, hipStream_t s, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!c->timing) return GM_OK;
  for (int i = 0; i < 2; ++i) {
    hipEvent_t e;
    if (!c->ev_free.empty()) {
      e = c->ev_free.back();
      c->ev_free.pop_back();
    } else {
      HIPCHK(hipEventCreate(&e));
    }
    (i == 0 ? *e0 : *e1) = e;
  }
  HIPCHK(hipEventRecord(*e0, s));
  return GM_OK;
}

int record_pass_end(gm_ctx* c, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (!c->timing) return GM_OK;
  HIPCHK(hipEventRecord(e1, s));
  c->ev_used.emplace_back(e0, e1);
  return GM_OK;
}

// Small problems (resident.hip): one cooperative launch, X in VGPRs, every
// iteration on the device.
int run_resident(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx,
                 const float* guess0, float* out, const gm_opts* o, gm_result* res,
                 const PassCfg& cfg, int cpb, int nb, hipStream_t s, bool* timed_out,
                 int64_t pstride = 0, int wshift = 0) {
  *timed_out = false;
  // granules [2][nb][2 values] in the slab region, + the timeout word in sums
  const size_t words = resident_gran_words(K, cfg, nb);
  const int64_t S = 2 * K + 2;
  Workspace w;
  int rc = ensure_ws(c, K, d, (int)((words + S - 1) / S), &w);
  if (rc) return rc;
  rc = ensure_host(c, sizeof(KState));
  if (rc) return rc;
  unsigned* bar = reinterpret_cast<unsigned*>(w.sums);  // reuse: timeout word, zeroed per call
  HIPCHK(hipMemsetAsync(w.st, 0, sizeof(KState), s));
  HIPCHK(hipMemsetAsync(bar, 0, 16, s));
  HIPCHK(hipMemsetAsync(w.slab, 0, align_up(words * 8, 16), s));   // every tag = 0
  ResArgs a{};
  a.X = X; a.K = K; a.d = d; a.ldx = ldx; a.guess0 = guess0; a.out = out;
  a.pstride = pstride; a.wshift = wshift;
  a.maxiter = o->maxiter; a.tol = (float)o->tol; a.eps = (float)o->eps;
  a.mode = o->mode; a.has_noise = o->mode == GM_MODE_AIRCOMP && o->has_noise;
  a.P_max = o->P_max; a.noise_sd = std::sqrt(std::max(0.0, o->noise_var) / 2.0);
  a.seed = o->seed;
  a.gran = reinterpret_cast<unsigned long long*>(w.slab);
  a.checkin = a.gran + (size_t)2 * nb * S;      // (resident_gran_words: + nb + 1 slots)
  a.need = checkin_need((unsigned)nb);
  a.stride = res_xcd_stride(nb, c->num_cu);
  // beyond one XCD: the XCD-hierarchical gather (members -> group leader -> every block),
  // its member granules L2-kept where the check-in confirms a group on one XCD
  // (where it pays, measured: K = 50 × d = 48,670 (96 blocks of 512 columns) 8.45 -> 7.47 µs
  // per iteration, 50 × 60,000 (118 blocks) 8.78 -> 7.38; but 50 × 30,000 (59) 6.72 -> 7.32,
  // 50 × 20,000 (40) 5.99 -> 7.16 and K <= 32 slower at every size: the leader's extra hop
  // costs more than the polls it saves on smaller grids or fewer values;
  // profiles/r5s1_resident_hier_shapes_ab.jsonl, r5s1_resident_hier2_ab.jsonl)
  const int hm = res_hier_mode();
  a.hier = a.stride == 1 && nb > 8 && 2 * K + 2 <= cfg.NW * 64 &&
           (hm == 2 || (hm == 1 && nb >= 90 && K > 32)) && resident_has_exchange(cfg, cpb, 1);
  a.local = (a.stride == 8 || a.hier) && res_xcd_mode() == 2;
  a.lvl2 = a.checkin + nb + 1;
  // below the hierarchical gather's range: the split-scope exchange (one hop, as the flat
  // gather, but each reader polls its own XCD's blocks from L2-kept copies)
  a.split = a.stride == 1 && !a.hier && nb > 8 && res_xcd_mode() == 2 && res_split_mode() != 0 &&
            resident_has_exchange(cfg, cpb, 2);
  a.granL = a.lvl2 + (size_t)32 * (2 * K + 2);
  a.bar = bar; a.st = w.st;
  hipEvent_t e0, e1;
  rc = record_pass_begin(c, s, &e0, &e1);
  if (rc) return rc;
  HIPCHK(launch_resident(cfg, cpb, nb * (int)a.stride, a, s));
  rc = record_pass_end(c, s, e0, e1);
  if (rc) return rc;
  KState* hst = reinterpret_cast<KState*>(c->host);
  HIPCHK(hipMemcpyAsync(hst, w.st, sizeof(KState), hipMemcpyDeviceToHost, s));
  unsigned hbar[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(hbar, bar, 16, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  static const bool verbose = getenv("GMAGG_RES_VERBOSE") != nullptr;
  if (verbose)
    fprintf(stderr, "gmagg resident: nb=%d stride=%u local=%d (requested %d) timed_out=%u\n", nb,
            a.stride, hbar[0] ? (int)hbar[0] - 1 : -1, a.local, hbar[2]);
  if (hbar[2]) {   // the grid was not co-resident long enough: caller reruns on streaming
    *timed_out = true;
    if (!hbar[3]) c->res_skip = kResSkipAfterCheckinFail;   // failed at the check-in
    if (c->timing && !c->ev_used.empty()) {
      c->ev_free.push_back(c->ev_used.back().first);
      c->ev_free.push_back(c->ev_used.back().second);
      c->ev_used.pop_back();
    }
    return GM_OK;
  }
  gm_result r{};
  r.iters = hst->iters;
  r.last_movement = hst->last_movement;
  r.converged = hst->converged;
  r.algo_used = GM_ALGO_RESIDENT;
  // The hierarchical gather ran whenever a.hier is set (its member granules are L2-kept
  // only where the check-in confirmed a group on one XCD; ADVICE r5: report the gather that
  // ran, as run_resident_batched does).  Otherwise bar[0] = 1 + local.
  r.exchange = a.hier ? GM_EXCHANGE_XCD_HIER
               : hbar[0] != 2 ? GM_EXCHANGE_AGENT
               : a.split ? GM_EXCHANGE_XCD_SPLIT : GM_EXCHANGE_XCD_LOCAL;
  if (res) *res = r;
  return GM_OK;
}

// Batched problems that fit on chip (resident_batched.hip, BASELINE C5): every problem's
// X is read once and held in VGPRs (+ LDS) for all its iterations, instead of once per
// pass.  Returns kRbNotTaken when the shape is not eligible, or when the kernel timed out
// (blocks not co-resident) before touching X: the caller streams.  GMAGG_BATCH_RESIDENT=0
// turns it off (A/B).
constexpr int kRbNotTaken = 1;
int run_resident_batched(gm_ctx* c, const float* X, int64_t P, int64_t K, int64_t d,
                         int64_t ldx, int64_t ldp, bool panels, int64_t Wp, const float* guess0,
                         int64_t ldg, float* out, int64_t ldo, const gm_opts* o,
                         gm_result* results, hipStream_t s, bool res_ok) {
  static const bool on = [] {
    const char* e = getenv("GMAGG_BATCH_RESIDENT");
    return !(e && atoi(e) == 0);
  }();
  if (!on || c->d_total > 0) return kRbNotTaken;
  if (o->mode == GM_MODE_AIRCOMP && o->noise_source != GM_NOISE_PHILOX) return kRbNotTaken;
  if (!res_ok) return kRbNotTaken;   // (resident_allowed, taken once by the caller)
  // float4 tile rows: 16-byte aligned problems, rows and panels
  if ((reinterpret_cast<uintptr_t>(X) & 15) || ldp % 4 || ldx % 4 || (panels && Wp % 4))
    return kRbNotTaken;
  const int64_t pbytes = panels ? (d + Wp - 1) / Wp * ldx * 4 : K * ldx * 4;
  if (pbytes >= ((int64_t)1 << 31)) return kRbNotTaken;
  RbPlan plan{};
  const int xcd = rb_xcd_major();
  if (!rb_plan(K, d, P, o->mode, c->num_cu, &plan, xcd == 2)) return kRbNotTaken;

  size_t off = 0;
  auto take = [&](size_t bytes) { size_t r0 = off; off = align_up(off + bytes, 256); return r0; };
  const size_t o_st = take(sizeof(KState) * P), o_flag = take(16);
  const size_t o_gran = take(sizeof(unsigned long long) * rb_gran_words(K, plan));
  const unsigned nblocks = (unsigned)(plan.ng * plan.nb);
  const size_t o_ci = take(sizeof(unsigned long long) * (nblocks + 1));
  if (off > c->ws_bytes) {
    if (c->ws) HIPCHK(hipFree(c->ws));
    c->ws = nullptr;
    c->ws_bytes = 0;
    HIPCHK(hipMalloc(&c->ws, off));
    c->ws_bytes = off;
  }
  int rc = ensure_host(c, sizeof(KState) * P + 256);
  if (rc) return rc;
  char* b = c->ws;
  KState* st = reinterpret_cast<KState*>(b + o_st);
  unsigned* flag = reinterpret_cast<unsigned*>(b + o_flag);
  HIPCHK(hipMemsetAsync(b, 0, off, s));          // states, the timeout word, every tag = 0

  ResBArgs a{};
  a.X = X; a.P = P; a.K = K; a.d = d; a.ldx = ldx; a.x_ps = ldp;
  a.pstride = panels ? ldx : 0;
  int ws = 0;
  while (panels && ((int64_t)1 << ws) < Wp) ++ws;
  a.wshift = ws;
  a.prob_bytes = (int)pbytes;
  a.nb = plan.nb;
  a.guess0 = guess0; a.ldg = ldg; a.out = out; a.ldo = ldo;
  a.maxiter = o->maxiter; a.tol = (float)o->tol; a.eps = (float)o->eps;
  a.mode = o->mode; a.has_noise = o->mode == GM_MODE_AIRCOMP && o->has_noise;
  a.P_max = o->P_max; a.noise_sd = std::sqrt(std::max(0.0, o->noise_var) / 2.0);
  a.seed = o->seed;
  a.pre_oma = o->pre_oma ? 1 : 0;
  a.oma_sd = (float)std::sqrt(std::max(0.0, o->pre_oma_var));
  a.oma_seed = o->pre_oma_seed;
  a.gran = reinterpret_cast<unsigned long long*>(b + o_gran);
  a.flag = flag;
  a.checkin = reinterpret_cast<unsigned long long*>(b + o_ci);
  a.need = checkin_need(nblocks);
  a.xcd_major = xcd != 0;
  // the hierarchical gather: sub-group granules L2-kept where the check-in confirms them
  a.hier = xcd != 0 && rb_hier_mode() == 1;
  a.local = xcd == 2 || a.hier != 0;
  a.lvl2 = a.gran + (size_t)plan.ng * 2 * plan.nb * (size_t)(2 * K + 2);
  a.st = st;
  hipEvent_t e0, e1;
  rc = record_pass_begin(c, s, &e0, &e1);
  if (rc) return rc;
  HIPCHK(launch_resident_batched(plan, a, res_coop_launch(), s));
  rc = record_pass_end(c, s, e0, e1);
  if (rc) return rc;
  KState* hst = reinterpret_cast<KState*>(c->host);
  unsigned* hflag = reinterpret_cast<unsigned*>(c->host + sizeof(KState) * P);
  HIPCHK(hipMemcpyAsync(hst, st, sizeof(KState) * P, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hflag, flag, 16, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  static const bool verbose = getenv("GMAGG_RES_VERBOSE") != nullptr;
  if (verbose)
    fprintf(stderr, "gmagg resident_batched: ng=%d nb=%d xcd=%d local_groups=%u timed_out=%u\n",
            plan.ng, plan.nb, xcd, hflag[1], hflag[0]);
  if (hflag[0]) {
    if (c->timing && !c->ev_used.empty()) {
      c->ev_free.push_back(c->ev_used.back().first);
      c->ev_free.push_back(c->ev_used.back().second);
      c->ev_used.pop_back();
    }
    // The grid was not co-resident.  Failed at the check-in (hflag[2] == 0): no block
    // read or wrote X, the caller streams (the pre-noise fused into its INIT pass) and
    // the next calls skip the resident kernels for a while.  Timed out after the
    // check-in (a block descheduled for 2 s mid-call): with the fused pre-noise some
    // problems may already carry their noise, so that call cannot be streamed again.
    if (!hflag[2]) {
      c->res_skip = kResSkipAfterCheckinFail;
      return kRbNotTaken;
    }
    if (o->pre_oma)
      return fail(GM_ERR_HIP, "batched resident kernel timed out after its check-in, with "
                  "the fused pre-noise begun (a block descheduled for 2 s?); X is partly noised");
    return kRbNotTaken;
  }
  if (results)
    for (int64_t p = 0; p < P; ++p)
      results[p] = gm_result{hst[p].iters, hst[p].last_movement, hst[p].converged,
                             GM_ALGO_RESIDENT, GM_GUARD_NONE, 0,
                             a.hier == 1 ? GM_EXCHANGE_XCD_HIER
                             : hflag[1] == (unsigned)plan.ng ? GM_EXCHANGE_XCD_LOCAL
                                                             : GM_EXCHANGE_AGENT};
  return GM_OK;
}

// Gram-space gm2 (gram.hip): G = X'X'^T once (MFMA), the Weiszfeld loop in K-space
// (one launch, fp64), one closing pass g = sum_k a_k x_k.  Two reads of X.
//
// AUTO guard (guarded = true).  The K-space loop is exact up to the error of G
// (fp32 accumulation; for the bf16 split also the bits of x' beyond h + m), and
// it has none of the reference's fp32 rounding of the iterate.  The closing pass
// is then a full streaming STEP pass at the returned weights, which also yields
// the exact distances ||x_k - g||^2; gram_verify compares the next weights from
// those with the K-space map's and measures the one-step error e = ||X'^T b||.
// The result is kept only if (1) e / (1 - rho) <= 1e-6 ||g|| (rho = the last
// K-space contraction ratio, clamped to [0.5, 0.95]), and (2) the reference's own
// fp32 movement noise floor, measured at 0.4-1.8 x 2^-24 ||g|| and
// taken as 2^-23 ||g||, is at most tol, so that the reference's loop does stop.
// Otherwise *rejected is set and the caller runs the streaming path.  With the floor
// below tol/3 the reference stops within +-1 iteration of the exact loop (guard
// ACCEPTED); between tol/3 and tol its count is decided by rounding — the streaming
// path's too — and the Gram's exact count lies in that window of legitimate stopping
// points (guard ACCEPTED_FLOOR; round 4: the whole C4 job, ||g|| = 74, is here).
int run_gram(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, const float* guess0,
             float* out, const gm_opts* o, gm_result* res, const PassCfg& cfg, hipStream_t s,
             bool split, bool guarded, bool* rejected, int64_t pstride = 0) {
  *rejected = false;
  // panels (pstride > 0): X is [ceil(d/W)][K][W] with W = the STEP tile's chunk width
  // (cfg), a multiple of the Gram kernel's 64-column stage; the f16 kernel only
  int wshift = 0;
  if (pstride) {
    const int W = cfg.LPR * cfg.V;
    while ((1 << wshift) < W) ++wshift;
    if ((1 << wshift) != W || W % 64 || !split) return fail(GM_ERR_UNSUPPORTED, "Gram on panels: W=%d", W);
  }
  const int KT = gram_kt(K), KP = 32 * KT;
  // split: the scaled f16 kernel (3 products), rerun as the bf16 split (4 products,
  // the full fp32 exponent range) if its G came out non-finite (GMAGG_GRAM_KIND=bf16
  // forces the bf16 kernel: A/B)
  const char* kind_env = getenv("GMAGG_GRAM_KIND");
  const bool force_bf16 = kind_env && strcmp(kind_env, "bf16") == 0;
  GramKind kind = !split ? GramKind::F32 : (force_bf16 && !pstride) ? GramKind::BF16 : GramKind::H16;
  GramGrid gg = gram_grid(d, kind, c->num_cu);
  const GramGrid gb = gram_grid(d, GramKind::BF16, c->num_cu);
  const size_t slab_n = std::max(gram_slab_floats(KT, gg),
                                 kind == GramKind::H16 ? gram_slab_floats(KT, gb) : 0);
  // closing pass: the STEP tile when it also yields the distances (guarded), else
  // the lighter sum-only tile
  const PassCfg ccfg = (guarded || pstride) ? cfg : light_cfg(K, cfg);
  const int J = ccfg.LPR * ccfg.V;
  const int nb_p = (int)std::max<int64_t>(
      1, std::min<int64_t>((d + J - 1) / J,
                           (int64_t)c->num_cu * pass_blocks_per_cu(ccfg, guarded ? 0 : 3)));
  Workspace w;
  int rc = ensure_ws(c, K, d, nb_p, &w, slab_n, KP);
  if (rc) return rc;
  rc = ensure_host(c, sizeof(KState) + 4 * sizeof(double));
  if (rc) return rc;
  KState* hst = reinterpret_cast<KState*>(c->host);
  double* hsums = reinterpret_cast<double*>(c->host + sizeof(KState));
  // centre p = guess0, staged to an aligned workspace copy (float4 loads)
  float* p = w.g[1];
  HIPCHK(hipMemcpyAsync(p, guess0, sizeof(float) * d, hipMemcpyDeviceToDevice, s));
again:
  HIPCHK(hipMemsetAsync(w.st, 0, sizeof(KState), s));
  hipEvent_t e0, e1;
  rc = record_pass_begin(c, s, &e0, &e1);
  if (rc) return rc;
  HIPCHK(launch_gram(X, K, d, ldx, p, kind, gg, w.gslab, w.G, w.st, s, pstride, wshift));
  rc = record_pass_end(c, s, e0, e1);
  if (rc) return rc;
  rc = allreduce(c, w.G, (int64_t)KP * KP, s);
  if (rc) return rc;
  // a non-finite G (f16 overflow on any rank, or a non-finite input) sets
  // gram_bad; checked after the all-reduce, so every rank takes the same branch
  HIPCHK(launch_gram_check(w.G, KP, w.st, s));
  HIPCHK(launch_gram_solve(w.G, KP, K, o->maxiter, (float)o->tol, (float)o->eps, w.alpha, w.u,
                           w.coef, w.st, s));
  // closing pass: g = sum_k a_k x_k (+ the exact distances to g when guarded)
  const int64_t S = guarded ? K + 2 : 2;
  PassArgs a{};
  a.X = X; a.K = K; a.d = d; a.ldx = pstride ? pstride : ldx;
  a.g_old = p; a.g_new = out; a.coef = w.coef; a.st = w.st;
  a.slab = w.slab; a.slab_stride = S;
  a.panel_stride = pstride;
  HIPCHK(launch_pass(ccfg, guarded ? 0 : 3, nb_p, a, s));
  HIPCHK(launch_slab_reduce(w.slab, nb_p, S, w.sums, w.st, s));   // [D (K)] [||p-g||^2, ||g||^2]
  rc = allreduce(c, w.sums, S, s);
  if (rc) return rc;
  if (guarded)
    HIPCHK(launch_gram_verify(w.G, KP, K, (float)o->eps, w.u, w.alpha, w.sums, w.r, w.st, s));
  HIPCHK(hipMemcpyAsync(hst, w.st, sizeof(KState), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(hsums, w.sums + (S - 2), 2 * sizeof(double), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (hst->gram_bad && kind == GramKind::H16) {   // rare: the f16 range was exceeded
    if (pstride) {                                 // no bf16 panel kernel: streaming path
      *rejected = true;
      return GM_OK;
    }
    kind = GramKind::BF16;
    gg = gb;
    goto again;
  }
  bool floor_band = false;
  if (guarded) {
    const double u = std::ldexp(1.0, -24);
    const double gn = std::sqrt(std::max(0.0, hsums[1]));
    double rho = hst->guard_r;
    rho = rho != rho ? 0.5 : std::min(0.95, std::max(0.5, rho));
    const double pred = hst->guard_q / (1.0 - rho) / gn;
    const bool accurate = pred <= 1e-6;                     // NaN fails
    const double floor = kFloorUlps * u * gn;        // (oracle FLOOR_ULPS, the count window)
    const bool floor_ok = !hst->converged || floor <= o->tol;
    floor_band = hst->converged && floor > o->tol / 3.0;
    static const bool dbg = getenv("GMAGG_GUARD_DEBUG") != nullptr;
    if (dbg)
      fprintf(stderr, "[gram guard] K=%lld d=%lld q=%.3e rho=%.3f |g|=%.4e pred=%.3e converged=%d "
              "iters=%d floor_ok=%d band=%d accurate=%d\n", (long long)K, (long long)d, hst->guard_q,
              rho, gn, pred, (int)hst->converged, (int)hst->iters, (int)floor_ok, (int)floor_band,
              (int)accurate);
    if (!accurate || !floor_ok) {
      *rejected = true;
      return GM_OK;
    }
  }
  gm_result r{};
  r.iters = hst->iters;
  r.last_movement = hst->last_movement;
  r.converged = hst->converged;
  r.algo_used = split ? GM_ALGO_GRAM : GM_ALGO_GRAM_F32;
  r.gram_kind = kind == GramKind::H16 ? 1 : kind == GramKind::BF16 ? 2 : 3;
  r.guard = !guarded ? GM_GUARD_NONE : floor_band ? GM_GUARD_ACCEPTED_FLOOR : GM_GUARD_ACCEPTED;
  if (res) *res = r;
  return GM_OK;
}

}  // namespace

extern "C" {

const char* gm_last_error(void) { return g_err.c_str(); }
int gm_abi_version(void) { return GMAGG_ABI_VERSION; }

int64_t gm_panel_width(int64_t K) {
  PassCfg cfg{};
  return K >= 1 && pick_cfg(K, 4, 1, &cfg, true) ? (int64_t)cfg.LPR * cfg.V : 0;
}

int gm_ctx_create(int device, gm_ctx** out) {
  if (!out) return fail(GM_ERR_INVALID, "gm_ctx_create: out is NULL");
  *out = nullptr;
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n)
    return fail(GM_ERR_INVALID, "gm_ctx_create: device %d of %d", device, n);
  gm_ctx* c = new gm_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cu = prop.multiProcessorCount;
  *out = c;
  return GM_OK;
}

int gm_ctx_destroy(gm_ctx* c) {
  if (!c) return GM_OK;
  (void)hipSetDevice(c->device);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->ws) (void)hipFree(c->ws);
  if (c->stage) (void)hipFree(c->stage);
  if (c->host) (void)hipHostFree(c->host);
  for (auto e : c->poll_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->ev_free) (void)hipEventDestroy(e);
  for (auto& p : c->ev_used) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  delete c;
  return GM_OK;
}

int gm_ctx_set_shard(gm_ctx* c, int64_t d_total, int64_t d_offset) {
  if (!c || d_total < -1 || d_offset < 0) return fail(GM_ERR_INVALID, "gm_ctx_set_shard: bad args");
  c->d_total = d_total;
  c->d_offset = d_offset;
  return GM_OK;
}

int gm_ctx_set_allreduce(gm_ctx* c, gm_allreduce_cb fn, void* user) {
  if (!c) return fail(GM_ERR_INVALID, "gm_ctx_set_allreduce: ctx is NULL");
  c->ar_fn = fn;
  c->ar_user = user;
  return GM_OK;
}

int gm_rccl_get_unique_id(void* uid) {
  if (!uid) return fail(GM_ERR_INVALID, "gm_rccl_get_unique_id: NULL");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(GM_ERR_COMM, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(uid, &id, sizeof id);
  return GM_OK;
}

int gm_ctx_init_rccl(gm_ctx* c, const void* uid, int nranks, int rank) {
  if (!c || !uid || nranks < 1 || rank < 0 || rank >= nranks)
    return fail(GM_ERR_INVALID, "gm_ctx_init_rccl: bad args");
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId id;
  memcpy(&id, uid, sizeof id);
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    c->comm = nullptr;
    return fail(GM_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  return GM_OK;
}

int gm_ctx_pass_timing(gm_ctx* c, int enable, double* total_ms, int64_t* launches) {
  if (!c) return fail(GM_ERR_INVALID, "gm_ctx_pass_timing: ctx is NULL");
  double tot = 0.0;
  int64_t n = 0;
  for (auto& p : c->ev_used) {
    HIPCHK(hipEventSynchronize(p.second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p.first, p.second));
    tot += ms;
    ++n;
    c->ev_free.push_back(p.first);
    c->ev_free.push_back(p.second);
  }
  c->ev_used.clear();
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  c->timing = enable != 0;
  return GM_OK;
}

int gm_weiszfeld_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx,
                     const float* guess0, float* out, const gm_opts* o, gm_result* res,
                     void* stream) {
  if (!c || !o || !out || !guess0) return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: NULL argument");
  if (K < 1 || d < 1 || (ldx < d && o && o->layout == GM_LAYOUT_ROWS) || (!X)) return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: bad shape K=%lld d=%lld ldx=%lld", (long long)K, (long long)d, (long long)ldx);
  if (o->maxiter < 0) return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: maxiter < 0");
  if (o->mode != GM_MODE_IDEAL && o->mode != GM_MODE_AIRCOMP)
    return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: unknown mode %d", o->mode);
  if (o->mode == GM_MODE_AIRCOMP && o->noise_source == GM_NOISE_HOST && !o->noise_cb)
    return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: GM_NOISE_HOST needs noise_cb");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WsOrder order(c, s);
  HIPCHK(order.err);
  // d-sharding: every decision that changes the sequence of collectives (Gram or
  // streaming, the poll interval and with it the passes queued after the stop) is
  // taken from GLOBAL quantities (K, d_total, options), so all ranks issue the same
  // all-reduces even when the last shard is shorter or ragged.  Local properties
  // (vector width, tile) only pick kernels.
  const bool sharded = c->d_total > 0;
  const int64_t d_total = sharded ? c->d_total : d;
  const int64_t col_off = sharded ? c->d_offset : 0;
  gm_result r{};
  // pre_oma: the reference's OMA(weight_f, var) before a non-gm aggregator (M:351-352),
  // applied to X in place.  The streaming path fuses it into its INIT pass (MODE 4: one
  // read + write of X instead of OMA's read + write and INIT's read); every other path
  // runs the standalone kernel first.  Draws as gm_oma_philox_f32 / _panels_f32.
  if (o->pre_oma && (o->mode != GM_MODE_IDEAL || !(o->pre_oma_var >= 0)))
    return fail(GM_ERR_INVALID, "pre_oma: gm2 only (the reference applies OMA before non-gm "
                "aggregators, M:351), noise variance >= 0");
  bool oma_pending = o->pre_oma != 0;
  auto apply_oma = [&]() -> int {
    if (!oma_pending) return GM_OK;
    oma_pending = false;
    int wshift = 0;
    if (o->layout == GM_LAYOUT_PANELS) {
      const int64_t W = gm_panel_width(K);
      while ((int64_t)1 << wshift < W) ++wshift;
    }
    HIPCHK(launch_oma_philox(const_cast<float*>(X), K, d, ldx, d_total, col_off,
                             (float)std::sqrt(o->pre_oma_var), o->pre_oma_seed, s, wshift));
    return GM_OK;
  };
  if (o->maxiter == 0) {
    int rco = apply_oma();
    if (rco) return rco;
    HIPCHK(hipMemcpyAsync(out, guess0, sizeof(float) * d, hipMemcpyDeviceToDevice, s));
    r.last_movement = NAN;
    if (res) *res = r;
    return GM_OK;
  }

  // Algorithm and tile.
  PassCfg cfg{};
  int algo = o->algo;
  // (a recursive call on the staged panel copy is the same call: no second turn)
  const bool res_ok = o->algo == GM_ALGO_STREAM || resident_allowed(c);
  bool panel_gram_rejected = false;
  const bool panels = o->layout == GM_LAYOUT_PANELS;
  if (o->layout != GM_LAYOUT_ROWS && !panels)
    return fail(GM_ERR_INVALID, "gm_weiszfeld_f32: unknown layout %d", o->layout);
  if (panels) {
    // [ceil(d/W)][K][W] panels: the streaming pass only, with the tile whose chunk
    // width is W (pick_cfg's tile for K; light_cfg's wider INIT tile is not used).
    const int64_t W = gm_panel_width(K);
    if (W == 0 || !pick_cfg(K, 4, W, &cfg, true) || cfg.LPR * cfg.V != W)
      return fail(GM_ERR_UNSUPPORTED, "panel layout: no streaming tile of width %lld for K=%lld",
                  (long long)W, (long long)K);
    if (ldx < K * W || (reinterpret_cast<uintptr_t>(X) & 15) || K * W * 4 > 0x7fffffff)
      return fail(GM_ERR_INVALID, "panel layout: need panel stride >= K*W (%lld), 16-byte aligned "
                  "X, K*W*4 < 2^31 (ldx=%lld)", (long long)(K * W), (long long)ldx);
    // gm2 at K <= 256: the scaled-f16 Gram reads panels too (AUTO on large d, as
    // for rows, guarded; explicit algo="gram" guarded likewise); streaming otherwise
    const bool gram_ok = o->mode == GM_MODE_IDEAL && gram_kt(K) > 0 && W % 64 == 0 &&
                         (W & (W - 1)) == 0;
    if ((algo == GM_ALGO_AUTO && gram_ok && d_total >= (int64_t)1 << 18) ||
        (algo == GM_ALGO_GRAM && gram_ok)) {
      static const bool unguarded = getenv("GMAGG_GRAM_UNGUARDED") != nullptr;
      bool rejected = false;
      int rco = apply_oma();
      if (rco) return rco;
      const int rc0 = run_gram(c, X, K, d, W, guess0, out, o, res, cfg, s, true,
                               algo == GM_ALGO_AUTO || !unguarded, &rejected, ldx);
      if (rc0 || !rejected) return rc0;
      panel_gram_rejected = true;
      algo = GM_ALGO_STREAM;
    }
    // One problem that fits on chip: the single-problem resident kernel (C2's, reading the
    // panels with its rows tile: V = 2 columns per lane, within one panel) when its grid
    // fits one XCD (the L2-kept exchange, §3.3: C2's shape 4.3 ms there against 6.7 ms on
    // the batched kernel's 4 blocks), else the batched kernel with P = 1 (K <= 52; gm at
    // K <= 50; the fused pre-noise included).  Either reads the panels once for all
    // iterations.
    const bool host_noise = o->mode == GM_MODE_AIRCOMP && o->noise_source == GM_NOISE_HOST;
    if ((algo == GM_ALGO_AUTO || algo == GM_ALGO_RESIDENT) && !sharded && !c->comm && !c->ar_fn &&
        !host_noise && K <= 64 && res_ok) {
      PassCfg rcfg{};
      int cpb = 0, nbr = 0;
      int ws = 0;
      while (((int64_t)1 << ws) < W) ++ws;
      if (pick_cfg(K, 2, W, &rcfg) && W % rcfg.V == 0 && (resident_tile(&rcfg, K), true) &&
          resident_plan(rcfg, (d + rcfg.LPR * rcfg.V - 1) / (rcfg.LPR * rcfg.V), c->num_cu, &cpb,
                        &nbr) &&
          res_xcd_stride(nbr, c->num_cu) == 8) {
        bool timed_out = false;
        int rco = apply_oma();
        if (rco) return rco;
        const int rc0 = run_resident(c, X, K, d, K * W, guess0, out, o, res, rcfg, cpb, nbr, s,
                                     &timed_out, ldx, ws);
        if (rc0 || !timed_out) return rc0;
        algo = GM_ALGO_STREAM;   // the X noised above: stream (no second pre-noise)
      }
    }
    if ((algo == GM_ALGO_AUTO || algo == GM_ALGO_RESIDENT) && !sharded && !c->comm && !c->ar_fn) {
      const int rc0 = run_resident_batched(c, X, 1, K, d, ldx, (d + W - 1) / W * ldx, true, W,
                                           guess0, d, out, d, o, res, s, res_ok);
      if (rc0 != kRbNotTaken) return rc0;
    }
    if (algo == GM_ALGO_AUTO) algo = GM_ALGO_STREAM;
    if (algo != GM_ALGO_STREAM)
      return fail(GM_ERR_UNSUPPORTED, "panel layout: streaming, (gm2, K <= 256) Gram or (K <= 52 "
                  "gm2 / K <= 50 gm, unsharded) resident only (algo %d)", algo);
  }
  const int V = panels ? 4 : pick_vec(X, d, ldx);
  // AUTO: Gram-space (split bf16) for gm2 at K <= 256 on large d, kept if its
  // accuracy guard passes (run_gram); streaming otherwise.  X is read twice
  // instead of n+1 times (profiles/history/r01_cmp_algos.txt, r02_gram_split.txt).
  // Sharded: the choice is made on d_total (every rank the same); each rank's
  // shard must then meet the kernel's local needs, which shard_range-aligned,
  // contiguous shards of a d_total % 4 == 0 update always do.
  // (panels never take this path, and their tile in cfg must stay: it sets the chunk
  // width the panel layout was built for)
  const bool gram_local_ok = !panels && gram_kt(K) > 0 && V == 4 && ldx < ((int64_t)1 << 26) &&
                             pick_cfg(K, V, ldx, &cfg);
  bool guard_rejected = panel_gram_rejected;   // a Gram result was computed and refused
  const bool gram_auto = algo == GM_ALGO_AUTO && o->mode == GM_MODE_IDEAL && !panels &&
                         gram_kt(K) > 0 && d_total >= (int64_t)1 << 18 &&
                         (sharded ? d_total % 4 == 0 : gram_local_ok);
  if (gram_auto) {
    if (!gram_local_ok)
      return fail(GM_ERR_INVALID, "sharded gm2 (AUTO -> Gram, d_total=%lld): this rank's shard "
                  "must be 16-byte aligned with d_local %% 4 == 0 and ldx %% 4 == 0 like every "
                  "other rank's (use sharded.shard_range + contiguous shards)",
                  (long long)d_total);
    bool rejected = false;
    int rco = apply_oma();
    if (rco) return rco;
    const int rc0 = run_gram(c, X, K, d, ldx, guess0, out, o, res, cfg, s, true, true, &rejected);
    if (rc0 || !rejected) return rc0;
    guard_rejected = true;
  }
  // Small problems: the register-resident single launch when every chunk fits one
  // co-resident block (unsharded, Philox or no noise).
  const bool host_noise_req = o->mode == GM_MODE_AIRCOMP && o->noise_source == GM_NOISE_HOST;
  if ((algo == GM_ALGO_AUTO || algo == GM_ALGO_RESIDENT) && !host_noise_req &&
      c->d_total <= 0 && !c->comm && !c->ar_fn && pick_cfg(K, V, ldx, &cfg)) {
    resident_tile(&cfg, K);
    const int J = cfg.LPR * cfg.V;
    const int64_t nch = (d + J - 1) / J;
    int cpb = 0, nbr = 0;
    if (res_ok && resident_plan(cfg, nch, c->num_cu, &cpb, &nbr)) {
      bool timed_out = false;
      int rco = apply_oma();
      if (rco) return rco;
      const int rc0 = run_resident(c, X, K, d, ldx, guess0, out, o, res, cfg, cpb, nbr, s,
                                   &timed_out);
      if (rc0 || !timed_out) return rc0;
      // barrier timeout (e.g. a time-sliced GPU): the same problem, same draw keys,
      // on the launch-per-pass streaming path below
      if (algo == GM_ALGO_RESIDENT) algo = GM_ALGO_AUTO;
    }
  }
  if (algo == GM_ALGO_RESIDENT)
    return fail(GM_ERR_UNSUPPORTED, "resident kernel: problem too large, sharded or host noise");
  // Row-major AirComp gm over many passes (the reference's `gm`: 1000 iterations, never
  // meeting tol; M:131-160) on a large client matrix: pack the panel layout once into a
  // context-owned buffer (one read + one write of X) and stream every pass from it.  Rows
  // stream at 79-80 % of HBM against 85-87 % on panels (C3 STEP 6.87-6.99 vs 6.35-6.47 ms),
  // so the copy pays for itself after ~35 passes.  Results equal the row-major passes' bit
  // for bit where both run the same tile (K outside 32 < K <= 64 and 128 < K <= 256, V = 4).
  // If the buffer cannot be allocated the rows are streamed (ensure_stage).
  // d-sharded calls too: the layout changes no collective (one all-reduce per pass either
  // way), so a rank may decide it from its own shard.
  if (!panels && algo == GM_ALGO_AUTO && o->mode == GM_MODE_AIRCOMP && o->has_noise &&
      !host_noise_req && o->maxiter >= 64 && K * d >= ((int64_t)1 << 24)) {
    const int64_t W = gm_panel_width(K);
    if (stage_enabled() && W > 0 && K * W * 4 <= 0x7fffffff) {
      if (ensure_stage(c, sizeof(float) * (size_t)((d + W - 1) / W) * (size_t)(K * W))) {
        HIPCHK(launch_rows_to_panels(X, K, d, ldx, c->stage, W, K * W, s));
        gm_opts o2 = *o;
        o2.layout = GM_LAYOUT_PANELS;
        o2.algo = GM_ALGO_STREAM;
        return gm_weiszfeld_f32(c, c->stage, K, d, K * W, guess0, out, &o2, res, stream);
      }
    }
  }
  if (panels) {
    // cfg fixed above
  } else if (algo == GM_ALGO_AUTO || algo == GM_ALGO_STREAM) {
    if (pick_cfg(K, V, ldx, &cfg)) algo = GM_ALGO_STREAM;
    else if (algo == GM_ALGO_STREAM)
      return fail(GM_ERR_UNSUPPORTED, "streaming pass supports K <= 2048 (K=%lld)", (long long)K);
    else algo = GM_ALGO_TWOPASS;
  }
  if (algo == GM_ALGO_GRAM || algo == GM_ALGO_GRAM_F32) {
    if (o->mode != GM_MODE_IDEAL)
      return fail(GM_ERR_UNSUPPORTED, "Gram variant is gm2 only (AirComp noise leaves span(X))");
    if (gram_kt(K) == 0 || V != 4 || !pick_cfg(K, V, ldx, &cfg))
      return fail(GM_ERR_UNSUPPORTED, "Gram variant needs K <= 256, d and ldx multiples of 4, "
                  "16-byte aligned X (K=%lld d=%lld ldx=%lld)", (long long)K, (long long)d,
                  (long long)ldx);
    // the split kernel addresses a 16-row group with 32-bit lane offsets
    const bool split = algo == GM_ALGO_GRAM && ldx < ((int64_t)1 << 26);
    // Explicit Gram runs the same a-posteriori guard as AUTO: a result the guard
    // refuses is never returned; the call then runs the streaming path and
    // reports guard = GM_GUARD_REJECTED.  (GMAGG_GRAM_UNGUARDED=1: A/B timing of
    // the bare Gram path, whose closing pass is the lighter sum-only tile.)
    static const bool unguarded = getenv("GMAGG_GRAM_UNGUARDED") != nullptr;
    bool rejected = false;
    int rco = apply_oma();
    if (rco) return rco;
    const int rc0 = run_gram(c, X, K, d, ldx, guess0, out, o, res, cfg, s, split, !unguarded,
                             &rejected);
    if (rc0 || !rejected) return rc0;
    guard_rejected = true;
    algo = GM_ALGO_STREAM;   // pick_cfg(K, V, ldx) succeeded above
  }
  if (algo != GM_ALGO_STREAM && algo != GM_ALGO_TWOPASS)
    return fail(GM_ERR_INVALID, "unknown algo %d", o->algo);
  const int init_mode = o->mode == GM_MODE_AIRCOMP ? 2 : 1;   // ||x_k||^2 only for AirComp

  int nb_step, nb_init;
  const PassCfg cfg_i = panels ? cfg : light_cfg(K, cfg);
  if (algo == GM_ALGO_STREAM) {
    const int J = cfg.LPR * cfg.V, Ji = cfg_i.LPR * cfg_i.V;
    const int64_t nch = (d + J - 1) / J, nchi = (d + Ji - 1) / Ji;
    const int64_t cap_s = (int64_t)c->num_cu * pass_blocks_per_cu(cfg, 0);
    const int64_t cap_i = (int64_t)c->num_cu * pass_blocks_per_cu(cfg_i, init_mode);
    nb_step = (int)std::max<int64_t>(1, std::min(nch, cap_s));
    nb_init = (int)std::max<int64_t>(1, std::min(nchi, cap_i));
  } else {
    nb_step = nb_init = twopass_blocks(K, d, c->num_cu);
  }
  const int nb = std::max(nb_step, nb_init);
  Workspace w;
  int rc = ensure_ws(c, K, d, nb, &w);
  if (rc) return rc;
  const bool host_noise = o->mode == GM_MODE_AIRCOMP && o->noise_source == GM_NOISE_HOST;
  const size_t host_ks = align_up(3 * sizeof(KState), 256);   // final + two lagged slots
  rc = ensure_host(c, host_ks + sizeof(float) * (2 * K + d_total + 1) + 256);
  if (rc) return rc;
  KState* hst = reinterpret_cast<KState*>(c->host);
  KState* hslot = hst + 1;
  float* h_hr = reinterpret_cast<float*>(c->host + host_ks);
  float* h_hi = h_hr + K;
  float* h_n = h_hi + K;   // d_total + 1
  HIPCHK(hipMemsetAsync(w.st, 0, sizeof(KState), s));

  const int noise_kind = o->mode != GM_MODE_AIRCOMP || !o->has_noise ? 0 : (host_noise ? 2 : 1);
  const double noise_sd = std::sqrt(std::max(0.0, o->noise_var) / 2.0);
  KspaceArgs ka{};
  ka.K = K;
  ka.d_total = d_total;
  ka.mode = o->mode;
  ka.has_noise = o->mode == GM_MODE_AIRCOMP && o->has_noise;
  ka.noise_src = host_noise ? 1 : 0;
  ka.tol = (float)o->tol;
  ka.eps = (float)o->eps;
  ka.P_max = o->P_max;
  ka.noise_sd = noise_sd;
  ka.seed = o->seed;
  ka.sums = w.sums;
  ka.r = w.r;
  ka.h_re = w.h_re;
  ka.h_im = w.h_im;
  ka.n_last = w.hnoise + d;
  ka.coef = w.coef;
  ka.st = w.st;

  auto upload_draws = [&](int64_t it) -> int {
    // The reference's draws of iteration `it` (OMA2, M:401-402, M:411).
    if (o->noise_cb(o->noise_user, it, h_hr, h_hi, o->has_noise ? h_n : nullptr) != 0)
      return fail(GM_ERR_CALLBACK, "noise callback failed at iteration %lld", (long long)it);
    HIPCHK(hipMemcpyAsync(w.h_re, h_hr, sizeof(float) * K, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(w.h_im, h_hi, sizeof(float) * K, hipMemcpyHostToDevice, s));
    if (o->has_noise) {
      HIPCHK(hipMemcpyAsync(w.hnoise, h_n + col_off, sizeof(float) * d, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(w.hnoise + d, h_n + d_total, sizeof(float), hipMemcpyHostToDevice, s));
    }
    return GM_OK;
  };
  auto poll = [&](KState* dst) -> int {
    HIPCHK(hipMemcpyAsync(dst, w.st, sizeof(KState), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return GM_OK;
  };

  // Pass over X: INIT (t = -1) or STEP t; leaves the reduced partials in w.sums.
  auto do_pass = [&](int64_t t) -> int {
    const bool init = t < 0;
    const float* g_old = init ? guess0 : (t == 0 ? guess0 : w.g[(t - 1) & 1]);
    float* g_new = init ? nullptr : w.g[t & 1];
    const int64_t S = init ? 2 * K + 2 : K + 2;
    hipEvent_t e0, e1;
    int rc2 = init ? GM_OK : record_pass_begin(c, s, &e0, &e1);
    if (rc2) return rc2;
    if (algo == GM_ALGO_STREAM) {
      PassArgs a{};
      a.X = X; a.K = K; a.d = d; a.ldx = ldx;
      a.g_old = g_old; a.g_new = g_new; a.coef = w.coef; a.st = w.st;
      a.slab = w.slab; a.slab_stride = S;
      a.noise = noise_kind; a.hnoise = w.hnoise; a.seed = o->seed; a.iter = t; a.col_off = col_off;
      a.panel_stride = panels ? ldx : 0;
      a.chunk_pair = panels ? 0 : chunk_pair(c, init ? cfg_i : cfg, init ? nb_init : nb_step);
      int mode = init ? init_mode : 0;
      if (init && oma_pending) {
        // the fused OMA needs float4 groups = Philox blocks: V = 4, 4-aligned shards
        if (cfg_i.V == 4 && col_off % 4 == 0 && init_mode == 1) {
          mode = 4;
          a.oma_sd = (float)std::sqrt(o->pre_oma_var);
          a.oma_seed = o->pre_oma_seed;
          oma_pending = false;
        } else {
          int rco = apply_oma();
          if (rco) return rco;
        }
      }
      HIPCHK(launch_pass(init ? cfg_i : cfg, mode, init ? nb_init : nb_step, a, s));
      if (!init) { rc2 = record_pass_end(c, s, e0, e1); if (rc2) return rc2; }
      HIPCHK(launch_slab_reduce(w.slab, init ? nb_init : nb_step, S, w.sums, w.st, s));
    } else {
      if (init) { int rco = apply_oma(); if (rco) return rco; }
      HIPCHK(launch_twopass(init, X, K, d, ldx, g_old, g_new, w.coef, w.st, noise_kind, w.hnoise,
                            o->seed, t, col_off, w.slab, nb, w.sums, s));
      if (!init) { rc2 = record_pass_end(c, s, e0, e1); if (rc2) return rc2; }
    }
    return allreduce(c, w.sums, S, s);
  };

  // Initial distances (and ||x_k||^2, ||g0||^2), then iteration-0 coefficients.
  rc = do_pass(-1);
  if (rc) return rc;
  ka.t = -1;
  ka.do_check = 0;
  if (host_noise) { rc = upload_draws(0); if (rc) return rc; }
  ka.do_coef = 1;
  HIPCHK(launch_kspace(ka, s));

  int check_every = o->check_every;
  if (check_every <= 0) check_every = (K * d_total >= (int64_t)1 << 24) ? 1 : 16;   // global
  if (host_noise) check_every = 1;
  // Polling every iteration (large passes): read iteration t-1's state while
  // iteration t is already queued, so the device never waits for the host.  If
  // t-1 stopped the loop, iteration t's launches see `done` and exit at once.
  static const bool no_lag = getenv("GMAGG_NO_LAG") != nullptr;   // A/B switch
  const bool lagged = check_every == 1 && !host_noise && !no_lag;
  if (lagged)
    for (auto& e : c->poll_ev)
      if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int64_t pending = -1;   // iteration whose KState copy is in flight (lagged)

  int64_t t = 0, enqueued = 0;
  const KState* final_st = nullptr;   // set when a lagged poll already saw the stop
  for (; t < o->maxiter; ++t) {
    rc = do_pass(t);
    if (rc) return rc;
    enqueued = t + 1;
    const bool last = t + 1 == o->maxiter;
    ka.t = t;
    if (host_noise) {
      // tol test first; draw the next iteration only if the loop goes on (M:145-159)
      ka.do_check = 1;
      ka.do_coef = 0;
      HIPCHK(launch_kspace(ka, s));
      rc = poll(hst);
      if (rc) return rc;
      if (hst->done || last) break;
      rc = upload_draws(t + 1);
      if (rc) return rc;
      ka.do_check = 0;
      ka.do_coef = 1;
      HIPCHK(launch_kspace(ka, s));
      continue;
    }
    ka.do_check = 1;
    ka.do_coef = last ? 0 : 1;
    // lagged poll: the K-space step itself leaves its KState in the host-mapped slot
    ka.mirror = lagged && !last ? &hslot[t & 1] : nullptr;
    HIPCHK(launch_kspace(ka, s));
    ka.mirror = nullptr;
    if (lagged && !last) {
      HIPCHK(hipEventRecord(c->poll_ev[t & 1], s));
      if (pending >= 0) {
        HIPCHK(hipEventSynchronize(c->poll_ev[pending & 1]));
        if (hslot[pending & 1].done) {
          final_st = &hslot[pending & 1];
          break;
        }
      }
      pending = t;
      continue;
    }
    if (last || (t + 1) % check_every == 0) {
      rc = poll(hst);
      if (rc) return rc;
      if (hst->done) break;
    }
  }
  // The state the lagged poll saw is final (launches after the stop are no-ops and
  // leave it alone), so no second copy + sync: the host returns while the device
  // drains the queued no-op iteration, and the next call's work queues behind it.
  if (!final_st) {
    rc = poll(hst);
    if (rc) return rc;
    final_st = hst;
  }
  r.iters = final_st->iters;
  r.last_movement = final_st->last_movement;
  r.converged = final_st->converged;
  r.algo_used = algo;
  r.guard = guard_rejected ? GM_GUARD_REJECTED : GM_GUARD_NONE;
  if (r.iters < 1) return fail(GM_ERR_HIP, "Weiszfeld loop recorded no iteration");
  // passes queued after the stop (lagged poll) exited at once: not timed as passes
  for (int64_t k = r.iters; k < enqueued && c->timing && !c->ev_used.empty(); ++k) {
    c->ev_free.push_back(c->ev_used.back().first);
    c->ev_free.push_back(c->ev_used.back().second);
    c->ev_used.pop_back();
  }
  HIPCHK(hipMemcpyAsync(out, w.g[(r.iters - 1) & 1], sizeof(float) * d, hipMemcpyDeviceToDevice, s));
  if (res) *res = r;
  return GM_OK;
}

int gm_weiszfeld_batched_f32(gm_ctx* c, const float* X, int64_t P, int64_t K, int64_t d,
                             int64_t ldx, int64_t ldp, const float* guess0, int64_t ldg,
                             float* out, int64_t ldo, const gm_opts* o, gm_result* results,
                             void* stream) {
  if (!c || !o || !X || !guess0 || !out)
    return fail(GM_ERR_INVALID, "gm_weiszfeld_batched_f32: NULL argument");
  // GM_LAYOUT_PANELS: problem p is [ceil(d/W)][K][W] at X + p*ldp, ldx = its panel stride
  const bool panels = o->layout == GM_LAYOUT_PANELS;
  if (o->layout != GM_LAYOUT_ROWS && !panels)
    return fail(GM_ERR_INVALID, "gm_weiszfeld_batched_f32: unknown layout %d", o->layout);
  const int64_t Wp = panels ? gm_panel_width(K) : 0;
  const int64_t rows_per_problem = panels ? (Wp > 0 ? (d + Wp - 1) / Wp : 0) : K;
  if (P < 1 || P > 65535 || K < 1 || d < 1 || ldx < (panels ? K * Wp : d) ||
      ldp < rows_per_problem * ldx || ldg < d || ldo < d || o->maxiter < 0 || (panels && Wp == 0))
    return fail(GM_ERR_INVALID, "gm_weiszfeld_batched_f32: bad shape P=%lld K=%lld d=%lld",
                (long long)P, (long long)K, (long long)d);
  if (panels && ((reinterpret_cast<uintptr_t>(X) & 15) || ldp % 4 || K * Wp * 4 > 0x7fffffff))
    return fail(GM_ERR_INVALID, "gm_weiszfeld_batched_f32 (panels): 16-byte aligned X and "
                "problem stride, K*W*4 < 2^31");
  if (o->mode == GM_MODE_AIRCOMP && o->noise_source != GM_NOISE_PHILOX)
    return fail(GM_ERR_UNSUPPORTED, "batched AirComp uses Philox noise only");
  if (c->d_total > 0) return fail(GM_ERR_UNSUPPORTED, "batched problems are not d-sharded");
  if (o->pre_oma && (o->mode != GM_MODE_IDEAL || !(o->pre_oma_var >= 0)))
    return fail(GM_ERR_INVALID, "pre_oma: gm2 only, noise variance >= 0");
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WsOrder order(c, s);
  HIPCHK(order.err);
  // Problems that fit on chip (K <= 52, d <= ~500k): the register-resident batched kernel
  // reads each problem's X once (resident_batched.hip); AUTO or GM_ALGO_RESIDENT
  if (o->maxiter > 0 && (o->algo == GM_ALGO_AUTO || o->algo == GM_ALGO_RESIDENT)) {
    const int rcr = run_resident_batched(c, X, P, K, d, ldx, ldp, panels, Wp, guess0, ldg, out,
                                         ldo, o, results, s, resident_allowed(c));
    if (rcr != kRbNotTaken) return rcr;
  }
  if (o->algo == GM_ALGO_RESIDENT)
    return fail(GM_ERR_UNSUPPORTED, "batched resident kernel: K <= 52 (gm2) / K <= 50 (gm), "
                "d <= %lld, 16-byte aligned problems", (long long)c->num_cu * 2048);
  // Row-major AirComp problems over >= 64 passes: pack them once into the context's panel
  // buffer and stream every pass from it, as gm_weiszfeld_f32 does (C5 AirComp reading on
  // rows: every problem runs all 1000 iterations).
  if (!panels && o->mode == GM_MODE_AIRCOMP && o->maxiter >= 64 &&
      P * K * d >= ((int64_t)1 << 24)) {
    const int64_t W = gm_panel_width(K);
    if (stage_enabled() && W > 0 && K * W * 4 <= 0x7fffffff) {
      const int64_t pst = (d + W - 1) / W * K * W;   // problem stride (floats)
      if (ensure_stage(c, sizeof(float) * (size_t)(P * pst))) {
        for (int64_t p = 0; p < P; ++p)
          HIPCHK(launch_rows_to_panels(X + p * ldp, K, d, ldx, c->stage + p * pst, W, K * W, s));
        gm_opts o2 = *o;
        o2.layout = GM_LAYOUT_PANELS;
        return gm_weiszfeld_batched_f32(c, c->stage, P, K, d, K * W, pst, guess0, ldg, out, ldo,
                                        &o2, results, stream);
      }
    }
  }
  // pre_oma (the reference's `--agg gm2 --var v` pre-noise, M:351-352): fused into the
  // INIT pass when the tile takes float4 groups, else the standalone batched OMA first;
  // problem p keyed pre_oma_seed + p * kSeedStride either way
  const float oma_sd = (float)std::sqrt(std::max(0.0, o->pre_oma_var));
  auto oma_standalone = [&]() -> int {
    int wshift = 0;
    while (panels && ((int64_t)1 << wshift) < Wp) ++wshift;
    HIPCHK(launch_oma_philox(const_cast<float*>(X), K, d, ldx, d, 0, oma_sd, o->pre_oma_seed, s,
                             wshift, P, P > 1 ? ldp : 0));
    return GM_OK;
  };
  if (o->maxiter == 0) {
    if (o->pre_oma) {
      const int rco = oma_standalone();
      if (rco) return rco;
    }
    HIPCHK(hipMemcpy2DAsync(out, ldo * 4, guess0, ldg * 4, d * 4, P, hipMemcpyDeviceToDevice, s));
    if (results)
      for (int64_t p = 0; p < P; ++p) results[p] = gm_result{0, NAN, 0, GM_ALGO_STREAM, GM_GUARD_NONE, 0};
    return GM_OK;
  }
  PassCfg cfg{};
  int V = panels ? 4 : pick_vec(X, d, ldx);
  if (ldp % V) V = 1;
  if (!pick_cfg(K, V, ldx, &cfg, panels) || (panels && cfg.LPR * cfg.V != Wp))
    return fail(GM_ERR_UNSUPPORTED, "batched streaming pass supports K <= 2048");
  const int init_mode = o->mode == GM_MODE_AIRCOMP ? 2 : 1;
  const int J = cfg.LPR * cfg.V;
  const int64_t nch = (d + J - 1) / J;
  // blocks per problem: the grid is OVERSUB rounds of co-resident blocks, so that the
  // iterations where only the slowest problems are still active (the others exit at
  // their `done` flag) still spread over the chip.  C5 on ProblemPanels: 8 rounds
  // 40.7-41.7k vs 2 rounds 39.7-39.9k problems/s (profiles/history/r2_c5_oversub.txt;
  // GMAGG_BATCH_OVERSUB: A/B)
  static const int oversub = [] {
    const char* e = getenv("GMAGG_BATCH_OVERSUB");
    return e && atoi(e) > 0 ? atoi(e) : 8;
  }();
  const int64_t target = (int64_t)c->num_cu * pass_blocks_per_cu(cfg, 0) * oversub;
  const int nbp = (int)std::max<int64_t>(1, std::min<int64_t>(nch, (target + P - 1) / P));
  const int64_t S = 2 * K + 2;

  // workspace: per problem KState, sums, r, coef, slab[nbp][S], g[2][d]; + a done counter
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t r0 = off; off = align_up(off + bytes, 256); return r0; };
  const size_t o_st = take(sizeof(KState) * P), o_cnt = take(sizeof(int) * 4);
  const size_t o_sums = take(sizeof(double) * S * P), o_r = take(sizeof(double) * K * P);
  const size_t o_coef = take(sizeof(float) * K * P), o_slab = take(sizeof(double) * S * nbp * P);
  const size_t o_g0 = take(sizeof(float) * d * P), o_g1 = take(sizeof(float) * d * P);
  if (off > c->ws_bytes) {
    if (c->ws) HIPCHK(hipFree(c->ws));
    c->ws = nullptr;
    c->ws_bytes = 0;
    HIPCHK(hipMalloc(&c->ws, off));
    c->ws_bytes = off;
  }
  char* b = c->ws;
  KState* st = reinterpret_cast<KState*>(b + o_st);
  int* cnt = reinterpret_cast<int*>(b + o_cnt);
  double* sums = reinterpret_cast<double*>(b + o_sums);
  double* rr = reinterpret_cast<double*>(b + o_r);
  float* coef = reinterpret_cast<float*>(b + o_coef);
  double* slab = reinterpret_cast<double*>(b + o_slab);
  float* g[2] = {reinterpret_cast<float*>(b + o_g0), reinterpret_cast<float*>(b + o_g1)};
  int rc = ensure_host(c, sizeof(KState) * P + 256);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(b, 0, o_sums, s));          // KStates + counter

  KspaceArgs ka{};
  ka.K = K;
  ka.d_total = d;
  ka.mode = o->mode;
  ka.has_noise = o->mode == GM_MODE_AIRCOMP && o->has_noise;
  ka.noise_src = 0;
  ka.tol = (float)o->tol;
  ka.eps = (float)o->eps;
  ka.P_max = o->P_max;
  ka.noise_sd = std::sqrt(std::max(0.0, o->noise_var) / 2.0);
  ka.seed = o->seed;
  ka.sums = sums;
  ka.r = rr;
  ka.coef = coef;
  ka.st = st;
  ka.sums_ps = S;
  ka.n_done = cnt;
  const int noise_kind = ka.has_noise ? 1 : 0;

  auto do_pass = [&](int64_t t) -> int {
    const bool init = t < 0;
    PassArgs a{};
    a.X = X; a.K = K; a.d = d; a.ldx = ldx; a.x_ps = ldp;
    if (init || t == 0) { a.g_old = guess0; a.gold_ps = ldg; }
    else { a.g_old = g[(t - 1) & 1]; a.gold_ps = d; }
    a.g_new = init ? nullptr : g[t & 1];
    a.gnew_ps = d;
    a.coef = coef; a.st = st; a.slab = slab; a.slab_stride = init ? S : K + 2;
    a.noise = noise_kind; a.seed = o->seed; a.iter = t;
    a.panel_stride = panels ? ldx : 0;
    int mode = init ? init_mode : 0;
    if (init && o->pre_oma) {
      if (cfg.V == 4 && init_mode == 1) {
        mode = 4;
        a.oma_sd = oma_sd;
        a.oma_seed = o->pre_oma_seed;
      } else {
        const int rco = oma_standalone();
        if (rco) return rco;
      }
    }
    hipEvent_t e0, e1;
    int rc2 = init ? GM_OK : record_pass_begin(c, s, &e0, &e1);
    if (rc2) return rc2;
    HIPCHK(launch_pass(cfg, mode, nbp, a, s, (int)P));
    if (!init) { rc2 = record_pass_end(c, s, e0, e1); if (rc2) return rc2; }
    HIPCHK(launch_slab_reduce(slab, nbp, init ? S : K + 2, sums, st, s, (int)P, S));
    return GM_OK;
  };
  int* hcnt = reinterpret_cast<int*>(c->host);
  auto poll_done = [&]() -> int {
    HIPCHK(hipMemcpyAsync(hcnt, cnt, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return *hcnt;
  };

  rc = do_pass(-1);
  if (rc) return rc;
  ka.t = -1;
  ka.do_check = 0;
  ka.do_coef = 1;
  HIPCHK(launch_kspace(ka, s, (int)P));
  static const int batch_check = [] {
    const char* e = getenv("GMAGG_BATCH_CHECK");
    return e && atoi(e) > 0 ? atoi(e) : 16;
  }();
  int check_every = o->check_every > 0 ? o->check_every : batch_check;
  for (int64_t t = 0; t < o->maxiter; ++t) {
    rc = do_pass(t);
    if (rc) return rc;
    const bool last = t + 1 == o->maxiter;
    ka.t = t;
    ka.do_check = 1;
    ka.do_coef = last ? 0 : 1;
    HIPCHK(launch_kspace(ka, s, (int)P));
    if (!last && (t + 1) % check_every == 0) {
      const int nd = poll_done();
      if (nd < 0) return nd;
      if (nd >= P) break;
    }
  }
  HIPCHK(launch_batched_finalize(g[0], g[1], d, (int)P, st, out, ldo, s));
  KState* hst = reinterpret_cast<KState*>(c->host);
  HIPCHK(hipMemcpyAsync(hst, st, sizeof(KState) * P, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (results)
    for (int64_t p = 0; p < P; ++p)
      results[p] = gm_result{hst[p].iters, hst[p].last_movement, hst[p].converged, GM_ALGO_STREAM,
                             GM_GUARD_NONE, 0};
  return GM_OK;
}

int gm_mean_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                void* stream) {
  if (!c || !X || !out || K < 1 || d < 0 || ldx < d) return fail(GM_ERR_INVALID, "gm_mean_f32: bad args");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_mean(X, K, d, ldx, out, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

// The coordinate-wise aggregators on client updates in the panel layout: the same
// kernels with panel addressing (W = gm_panel_width(K) = 2^ws, ldx = panel_stride);
// results identical to the row-major calls (same per-column reductions).
static int panel_shift(int64_t K, int64_t panel_stride, int* ws) {
  const int64_t W = gm_panel_width(K);
  if (W == 0 || panel_stride < K * W) return GM_ERR_INVALID;
  int s = 0;
  while (((int64_t)1 << s) < W) ++s;
  *ws = s;
  return GM_OK;
}

int gm_mean_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                       float* out, void* stream) {
  int ws = 0;
  if (!c || !X || !out || K < 1 || d < 0 || panel_shift(K, panel_stride, &ws))
    return fail(GM_ERR_INVALID, "gm_mean_panels_f32: bad args");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_mean(X, K, d, panel_stride, out, reinterpret_cast<hipStream_t>(stream), ws));
  return GM_OK;
}

int gm_median_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                         float* out, void* stream) {
  int ws = 0;
  if (!c || !X || !out || K < 1 || d < 0 || panel_shift(K, panel_stride, &ws))
    return fail(GM_ERR_INVALID, "gm_median_panels_f32: bad args");
  if (K > 2048) return fail(GM_ERR_UNSUPPORTED, "gm_median_panels_f32: K <= 2048");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_select(X, K, d, panel_stride, 0, 0, out, reinterpret_cast<hipStream_t>(stream),
                           ws));
  return GM_OK;
}

int gm_trimmed_mean_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t d,
                               int64_t panel_stride, int64_t trim, float* out, void* stream) {
  int ws = 0;
  if (!c || !X || !out || K < 1 || d < 0 || trim < 0 || 2 * trim >= K ||
      panel_shift(K, panel_stride, &ws))
    return fail(GM_ERR_INVALID, "gm_trimmed_mean_panels_f32: bad args");
  if (K > 2048) return fail(GM_ERR_UNSUPPORTED, "gm_trimmed_mean_panels_f32: K <= 2048");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_select(X, K, d, panel_stride, 1, trim, out,
                           reinterpret_cast<hipStream_t>(stream), ws));
  return GM_OK;
}

int gm_honest_variance_f32(gm_ctx* c, const float* X, int64_t honest, int64_t d, int64_t ldx,
                           float* out, void* stream) {
  if (!c || !X || !out || honest < 1 || d < 1 || ldx < d)
    return fail(GM_ERR_INVALID, "gm_honest_variance_f32: bad args");
  const int wshift = 0;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WsOrder order(c, s);
  HIPCHK(order.err);
  const int nb = honest_var_blocks(d, c->num_cu);
  Workspace w;
  const int rc = ensure_ws(c, 1, 1, nb, &w);
  if (rc) return rc;
  HIPCHK(launch_honest_var(X, honest, d, ldx, wshift, nb, w.slab, out, s));
  return GM_OK;
}

int gm_honest_variance_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t honest, int64_t d,
                                  int64_t panel_stride, float* out, void* stream) {
  const int64_t W = gm_panel_width(K);
  if (!c || !X || !out || honest < 1 || honest > K || d < 1 || W == 0 || panel_stride < K * W)
    return fail(GM_ERR_INVALID, "gm_honest_variance_panels_f32: bad args");
  int wshift = 0;
  while ((int64_t)1 << wshift < W) ++wshift;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WsOrder order(c, s);
  HIPCHK(order.err);
  const int nb = honest_var_blocks(d, c->num_cu);
  Workspace w;
  const int rc = ensure_ws(c, 1, 1, nb, &w);
  if (rc) return rc;
  HIPCHK(launch_honest_var(X, honest, d, panel_stride, wshift, nb, w.slab, out, s));
  return GM_OK;
}

int gm_median_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, float* out,
                  void* stream) {
  if (!c || !X || !out || K < 1 || d < 0 || ldx < d) return fail(GM_ERR_INVALID, "gm_median_f32: bad args");
  if (K > 2048) return fail(GM_ERR_UNSUPPORTED, "gm_median_f32: K <= 2048");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_select(X, K, d, ldx, 0, 0, out, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_trimmed_mean_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx,
                        int64_t trim, float* out, void* stream) {
  if (!c || !X || !out || K < 1 || d < 0 || ldx < d || trim < 0 || 2 * trim >= K)
    return fail(GM_ERR_INVALID, "gm_trimmed_mean_f32: bad args");
  if (K > 2048) return fail(GM_ERR_UNSUPPORTED, "gm_trimmed_mean_f32: K <= 2048");
  if (d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_col_select(X, K, d, ldx, 1, trim, out, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

static int krum_impl(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, int ws,
                     int64_t honest, float* out, int64_t* index, void* stream);

int gm_krum_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, int64_t honest,
                float* out, int64_t* index, void* stream) {
  if (!c || !X || !out || K < 1 || d < 0 || ldx < d || honest < 2 || honest - 1 > K)
    return fail(GM_ERR_INVALID, "gm_krum_f32: bad args (needs 2 <= honestSize <= K+1)");
  if (K > 4096) return fail(GM_ERR_UNSUPPORTED, "gm_krum_f32: K <= 4096");
  return krum_impl(c, X, K, d, ldx, 0, honest, out, index, stream);
}

int gm_krum_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t panel_stride,
                       int64_t honest, float* out, int64_t* index, void* stream) {
  int ws = 0;
  if (!c || !X || !out || K < 1 || d < 0 || honest < 2 || honest - 1 > K ||
      panel_shift(K, panel_stride, &ws))
    return fail(GM_ERR_INVALID, "gm_krum_panels_f32: bad args (needs 2 <= honestSize <= K+1)");
  if (K > 4096) return fail(GM_ERR_UNSUPPORTED, "gm_krum_panels_f32: K <= 4096");
  return krum_impl(c, X, K, d, panel_stride, ws, honest, out, index, stream);
}

// Krum through the Gram MFMA kernel (coordinate.hip krum_gram_bounds: the bounds, the
// candidates, the exact recomputation).  epsg bounds the relative error |G~_ij - G_ij| /
// (n_i n_j) of the scaled-f16 split (gram.hip): the split's dropped terms (<= 3 * 2^-22),
// the fp32 chain of one flush period (kH16Flush stages x 64 columns = 8192 columns, 3
// products: <= 768 accumulator roundings + the 32-term MFMA sums + the fp32 partial,
// <= 800 * 2^-24) and the centring rounding (2^-24 each side), rounded up to 6e-5.  The f16
// subnormal floor is an ABSOLUTE error set by each column block's shared scale (one large
// row raises it for every row of the block): krum_gram_bounds adds it from the exponents
// the Gram kernel exports (a per-row bound was assumed here before).
static double krum_gram_eps() { return 6e-5; }

// GMAGG_KRUM: 0 exact pair distances only, 1 the Gram path wherever it is eligible, 2
// (default) AUTO: the Gram path at K >= 64 and K^2 d >= 2^29 (it measured faster on every
// shape from 64 x 131,072 up, profiles/r5s2_krum_ab.jsonl).  Read per call (the tests
// switch it).
static int krum_mode() {
  const char* e = getenv("GMAGG_KRUM");
  return e ? atoi(e) : 2;
}

// Returns GM_OK with *done = false when the exact path must run (not eligible, a
// non-finite Gram, too many candidates), c->krum_info saying why.
static int krum_gram(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, int ws,
                     int64_t honest, float* out, int64_t* index, hipStream_t s, bool* done) {
  *done = false;
  const int KT = gram_kt(K), KP = 32 * KT;
  const int64_t kk = honest - 1;
  const GramGrid gg = gram_grid(d, GramKind::H16, c->num_cu);
  const int64_t S = krum_slices(K, d);
  const int64_t RC = krum_refine_max();
  const int64_t maxc = 4 * RC;
  // slab: the Gram partials, then (after gram_reduce has consumed them) the refinement's
  // [S][RC][K] fp64 partials + Dc [RC][K]; behind both the candidate list (int64)
  size_t body = std::max(gram_slab_floats(KT, gg), (size_t)2 * (size_t)(S * RC * K + RC * K));
  body = (body + 1) / 2 * 2;
  Workspace w;
  int rc = ensure_ws(c, K, d, 1, &w, body + 2 * (size_t)(maxc + 2), KP);
  if (rc) return rc;
  rc = ensure_host(c, sizeof(KState) + 2 * sizeof(int64_t));
  if (rc) return rc;
  double* part = reinterpret_cast<double*>(w.gslab);
  double* Dc = part + (size_t)S * RC * K;
  int64_t* cand = reinterpret_cast<int64_t*>(w.gslab + body);
  int64_t* didx = reinterpret_cast<int64_t*>(w.r);
  KState* hst = reinterpret_cast<KState*>(c->host);
  int64_t* hcand = reinterpret_cast<int64_t*>(c->host + sizeof(KState));
  const int64_t W = ws ? (int64_t)1 << ws : 0;
  // The bounds scale with the rows' distances from the centre p: row 0 first (honest in
  // the reference's layout, M:292); when it leaves too many candidates (a Byzantine row 0,
  // far from the honest cluster) once more from the row of the smallest upper bound.
  int64_t n = 0, centre = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    float* p = w.g[1];
    HIPCHK(launch_copy_row_k(X, d, ldx, ws, centre, p, s));
    HIPCHK(hipMemsetAsync(w.st, 0, sizeof(KState), s));
    HIPCHK(launch_gram(X, K, d, ws ? W : ldx, p, GramKind::H16, gg, w.gslab, w.G, w.st, s,
                       ws ? ldx : 0, ws));
    HIPCHK(launch_gram_check(w.G, KP, w.st, s));
    HIPCHK(launch_krum_gram_select(w.G, KP, K, kk, krum_gram_eps(),
                                   gram_block_exp(w.gslab, KT, gg), gg.nb, d, w.alpha, w.u, maxc,
                                   cand, s));
    HIPCHK(hipMemcpyAsync(hst, w.st, sizeof(KState), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hcand, cand, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hcand + 1, cand + maxc + 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (hst->gram_bad) {
      c->krum_info[2] = GM_KRUM_REASON_GRAM_NONFINITE;
      return GM_OK;
    }
    n = hcand[0];
    if (n != -2 || hcand[1] == centre) break;
    centre = hcand[1];
  }
  if (n < 1) {
    c->krum_info[2] = GM_KRUM_REASON_CANDIDATES;
    return GM_OK;
  }
  for (int64_t q = 0; q < n; q += RC) {
    const int m = (int)std::min<int64_t>(RC, n - q);
    HIPCHK(launch_krum_refine(X, K, d, ldx, ws, cand + 1 + q, m, kk, part, Dc, w.sums + q, s));
  }
  HIPCHK(launch_krum_pick(w.sums, cand + 1, n, X, d, ldx, ws, didx, out, s));
  if (index) {
    HIPCHK(hipMemcpyAsync(index, didx, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  c->krum_info[0] = GM_KRUM_GRAM;
  c->krum_info[1] = n;
  c->krum_info[2] = GM_KRUM_REASON_OK;
  *done = true;
  return GM_OK;
}

int gm_krum_last_info(gm_ctx* c, int64_t* info) {
  if (!c || !info) return fail(GM_ERR_INVALID, "gm_krum_last_info: bad args");
  for (int i = 0; i < 3; ++i) info[i] = c->krum_info[i];
  return GM_OK;
}

static int krum_impl(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx, int ws,
                     int64_t honest, float* out, int64_t* index, void* stream) {
  HIPCHK(hipSetDevice(c->device));
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  WsOrder order(c, s);
  HIPCHK(order.err);
  c->krum_info[0] = GM_KRUM_EXACT;
  c->krum_info[1] = 0;
  c->krum_info[2] = GM_KRUM_REASON_NOT_CHOSEN;
  // the Gram kernel's inputs: K <= 256; rows 16-byte aligned with d, ldx multiples of 4
  // (float4 stages); panels of width 64 / 128 / 256 (a power of two, multiple of 64)
  const bool eligible =
      gram_kt(K) > 0 && d > 0 && honest - 1 <= K &&
      (ws ? (ws >= 6 && ws <= 8 && K * ((int64_t)1 << ws) * 4 <= 0x7fffffff)
          : (d % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 &&
             ldx < ((int64_t)1 << 26)));
  const int mode = krum_mode();
  const bool want = mode == 1 || (mode == 2 && K >= 64 && (double)K * K * d >= 536870912.0);
  if (want && !eligible) c->krum_info[2] = GM_KRUM_REASON_NOT_ELIGIBLE;
  if (want && eligible) {
    bool done = false;
    const int rc = krum_gram(c, X, K, d, ldx, ws, honest, out, index, s, &done);
    if (rc || done) return rc;
  }
  Workspace w;
  // G area holds the K x K distances; the float slab holds the per-slice fp64 partials
  const size_t part_doubles = (size_t)krum_slices(K, d) * (size_t)(K * K);
  int rc = ensure_ws(c, K, 1, 1, &w, 2 * part_doubles, (int)K);
  if (rc) return rc;
  int64_t* didx = reinterpret_cast<int64_t*>(w.u);
  HIPCHK(launch_krum(X, K, d, ldx, honest - 1, w.G, reinterpret_cast<double*>(w.gslab), w.alpha,
                     out, didx, reinterpret_cast<hipStream_t>(stream), ws));
  if (index) {
    HIPCHK(hipMemcpyAsync(index, didx, sizeof(int64_t), hipMemcpyDeviceToHost,
                          reinterpret_cast<hipStream_t>(stream)));
    HIPCHK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  }
  return GM_OK;
}

int gm_oma_philox_f32(gm_ctx* c, float* X, int64_t K, int64_t d, int64_t ldx, double noise_var,
                      uint64_t seed, void* stream) {
  if (!c || !X || K < 0 || d < 0 || ldx < d || noise_var < 0)
    return fail(GM_ERR_INVALID, "gm_oma_philox_f32: bad args");
  if (K == 0 || d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  const int64_t d_total = c->d_total > 0 ? c->d_total : d;
  const int64_t col_off = c->d_total > 0 ? c->d_offset : 0;
  HIPCHK(launch_oma_philox(X, K, d, ldx, d_total, col_off, (float)std::sqrt(noise_var), seed,
                           reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_oma_philox_batched_f32(gm_ctx* c, float* X, int64_t P, int64_t K, int64_t d, int64_t ldx,
                              int64_t pstride, double noise_var, uint64_t seed, void* stream) {
  if (!c || !X || P < 0 || K < 0 || d < 0 || ldx < d || noise_var < 0 ||
      (P > 1 && pstride < K * ldx))
    return fail(GM_ERR_INVALID, "gm_oma_philox_batched_f32: bad args");
  if (P == 0 || K == 0 || d == 0) return GM_OK;
  if (c->d_total > 0)
    return fail(GM_ERR_UNSUPPORTED, "gm_oma_philox_batched_f32: not on a d-sharded context");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_oma_philox(X, K, d, ldx, d, 0, (float)std::sqrt(noise_var), seed,
                           reinterpret_cast<hipStream_t>(stream), 0, P, P > 1 ? pstride : 0));
  return GM_OK;
}

int gm_oma_philox_batched_panels_f32(gm_ctx* c, float* X, int64_t P, int64_t K, int64_t d,
                                     int64_t panel_stride, int64_t pstride, double noise_var,
                                     uint64_t seed, void* stream) {
  const int64_t W = gm_panel_width(K);
  if (!c || !X || P < 0 || K < 0 || d < 0 || noise_var < 0 || (K > 0 && W == 0) ||
      panel_stride < K * W || (P > 1 && pstride < (d + W - 1) / W * panel_stride))
    return fail(GM_ERR_INVALID, "gm_oma_philox_batched_panels_f32: bad args");
  if (P == 0 || K == 0 || d == 0) return GM_OK;
  if (c->d_total > 0)
    return fail(GM_ERR_UNSUPPORTED, "gm_oma_philox_batched_panels_f32: not on a d-sharded context");
  HIPCHK(hipSetDevice(c->device));
  int wshift = 0;
  while ((int64_t)1 << wshift < W) ++wshift;
  HIPCHK(launch_oma_philox(X, K, d, panel_stride, d, 0, (float)std::sqrt(noise_var), seed,
                           reinterpret_cast<hipStream_t>(stream), wshift, P, P > 1 ? pstride : 0));
  return GM_OK;
}

int gm_oma_philox_panels_f32(gm_ctx* c, float* X, int64_t K, int64_t d, int64_t panel_stride,
                             double noise_var, uint64_t seed, void* stream) {
  const int64_t W = gm_panel_width(K);
  if (!c || !X || K < 0 || d < 0 || noise_var < 0 || (K > 0 && W == 0) || panel_stride < K * W)
    return fail(GM_ERR_INVALID, "gm_oma_philox_panels_f32: bad args");
  if (K == 0 || d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  const int64_t d_total = c->d_total > 0 ? c->d_total : d;
  const int64_t col_off = c->d_total > 0 ? c->d_offset : 0;
  int wshift = 0;
  while ((int64_t)1 << wshift < W) ++wshift;
  HIPCHK(launch_oma_philox(X, K, d, panel_stride, d_total, col_off, (float)std::sqrt(noise_var),
                           seed, reinterpret_cast<hipStream_t>(stream), wshift));
  return GM_OK;
}

int gm_rows_to_panels_f32(gm_ctx* c, const float* X, int64_t K, int64_t d, int64_t ldx,
                          float* P, int64_t W, int64_t panel_stride, void* stream) {
  if (!c || !X || !P || K < 0 || d < 0 || ldx < d || W < 1 || panel_stride < K * W)
    return fail(GM_ERR_INVALID, "gm_rows_to_panels_f32: bad args");
  if (K == 0 || d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_rows_to_panels(X, K, d, ldx, P, W, panel_stride,
                               reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_client_chain_f32(gm_ctx* c, const float* data, int64_t ldd, const int64_t* labels,
                        int64_t F, int64_t C, const int32_t* idx, int64_t K, int64_t B,
                        int64_t honest, int32_t attack, float gamma, float weight_decay,
                        float* W, float* b, float* X, int64_t ldx, int32_t layout, void* stream) {
  if (!c || !data || !labels || !idx || !W || !b || !X || K < 0 || honest < 0 || ldd < F ||
      attack < 0 || attack > 2 || (layout != GM_LAYOUT_ROWS && layout != GM_LAYOUT_PANELS))
    return fail(GM_ERR_INVALID, "gm_client_chain_f32: bad args");
  if (!client_chain_supported(F, C, B))
    return fail(GM_ERR_UNSUPPORTED, "gm_client_chain_f32: needs F <= 832, C <= 64, B <= 64 "
                "(F=%lld C=%lld B=%lld)", (long long)F, (long long)C, (long long)B);
  const int64_t d = C * F + C;
  ClientChainArgs a{};
  a.data = data; a.ldd = ldd; a.labels = labels; a.F = F; a.C = C; a.idx = idx;
  a.K = K; a.B = B; a.honest = honest; a.attack = attack; a.gamma = gamma; a.wd = weight_decay;
  a.W = W; a.b = b; a.X = X;
  if (layout == GM_LAYOUT_PANELS) {
    const int64_t Wp = gm_panel_width(K);
    if (Wp == 0 || ldx < K * Wp) return fail(GM_ERR_INVALID, "gm_client_chain_f32: panel stride");
    int ws = 0;
    while (((int64_t)1 << ws) < Wp) ++ws;
    a.pstride = ldx;
    a.wshift = ws;
  } else {
    if (ldx < d) return fail(GM_ERR_INVALID, "gm_client_chain_f32: ldx < C*F + C");
    a.ldx = ldx;
  }
  if (K == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_client_chain(a, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_oma_apply_f32(gm_ctx* c, float* X, int64_t K, int64_t d, int64_t ldx, const float* hr,
                     const float* hi, const float* nr, const float* ni, void* stream) {
  if (!c || !X || !hr || !hi || !nr || !ni || K < 0 || d < 0 || ldx < d)
    return fail(GM_ERR_INVALID, "gm_oma_apply_f32: bad args");
  if (K == 0 || d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(launch_oma_apply(X, K, d, ldx, hr, hi, nr, ni, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_fill_clients_f32(gm_ctx* c, float* X, int64_t K, int64_t d, int64_t ldx, int64_t B,
                        float mu_h, float sd_h, float mu_b, float sd_b, uint64_t seed,
                        void* stream) {
  if (!c || !X || K < 0 || d < 0 || ldx < d || B < 0 || B > K)
    return fail(GM_ERR_INVALID, "gm_fill_clients_f32: bad args");
  if (K == 0 || d == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  const int64_t d_total = c->d_total > 0 ? c->d_total : d;
  const int64_t col_off = c->d_total > 0 ? c->d_offset : 0;
  HIPCHK(launch_fill_clients(X, K, d, ldx, B, mu_h, sd_h, mu_b, sd_b, d_total, col_off, seed,
                             reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

int gm_fill_normal_f32(gm_ctx* c, float* v, int64_t n, float mu, float sd, uint64_t seed,
                       void* stream) {
  if (!c || !v || n < 0) return fail(GM_ERR_INVALID, "gm_fill_normal_f32: bad args");
  if (n == 0) return GM_OK;
  HIPCHK(hipSetDevice(c->device));
  const int64_t col_off = c->d_total > 0 ? c->d_offset : 0;
  HIPCHK(launch_fill_normal(v, n, mu, sd, col_off, seed, reinterpret_cast<hipStream_t>(stream)));
  return GM_OK;
}

}  // extern "C"
