// libdcnr C ABI: the native runtime that sequences the DCN-R forward/backward
// kernels on one HIP stream over caller-owned memory (include/dcnr.h).
//
// Forward  = DCN_RecSys.forward (train.py:155-170):
//   gather+x0+cross (1 kernel) -> initial Linear (MFMA GEMM) ->
//   per ResBlock: L1 GEMM -> BN1 stats/finalize -> BN1+ReLU+dropout ->
//                 L2 GEMM -> BN2 stats/finalize -> BN2 + residual + ReLU
//   -> deep head dot -> logits
// Backward = loss.backward() (train.py:225), reverse order, BN backward with
// deterministic fp64 column reductions, dW by split-K MFMA GEMMs over the batch,
// cross backward + dense embedding-grad scatter in one kernel.
#include "dcnr_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace dcnr {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

dcnr_status set_max_dyn_lds(const void* kernel, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  int dev = 0;
  DCNR_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  size_t& cur = done[{kernel, dev}];
  if (bytes > cur) {
    DCNR_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    cur = bytes;
  }
  return DCNR_OK;
}

// ------------------------------------------------------------ profiling
// Optional per-launch HIP-event timing by kernel class (dcnr_profile_*).
// Each record carries the launch's ALGORITHMIC bytes (the operands the
// function must move: inputs read once, outputs written once; 0 = not
// accounted) so the bench prices every kernel class against HBM.
struct ProfRec { int cat; double bytes; hipEvent_t a, b; };
static std::mutex g_pm;
static bool g_prof = false;
static int g_prof_mode = 0;   // 1: every class, each launch alone; 2: gemm_dw only, concurrent
static std::vector<ProfRec> g_recs;
static std::vector<hipEvent_t> g_pool;

static hipEvent_t prof_event() {
  if (!g_pool.empty()) { hipEvent_t e = g_pool.back(); g_pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

struct ProfScope {
  int cat; hipStream_t s; double bytes; hipEvent_t a = nullptr;
  ProfScope(int c, hipStream_t st, double nbytes = 0.0) : cat(c), s(st), bytes(nbytes) {
    if (!g_prof || (g_prof_mode == 2 && c != DCNR_K_GEMM_DW)) return;
    std::lock_guard<std::mutex> lk(g_pm);
    a = prof_event();
    (void)hipEventRecord(a, s);
  }
  ~ProfScope() {
    if (!a) return;
    std::lock_guard<std::mutex> lk(g_pm);
    hipEvent_t b = prof_event();
    (void)hipEventRecord(b, s);
    g_recs.push_back(ProfRec{cat, bytes, a, b});
  }
};

namespace {

#define TRY(x)                       \
  do {                               \
    dcnr_status st_ = (x);           \
    if (st_ != DCNR_OK) return st_;  \
  } while (0)
// TRY with the launch attributed to a kernel class (stream `s` in scope)
#define TRYP(cat, x)                 \
  do {                               \
    ProfScope ps_(cat, s);           \
    dcnr_status st_ = (x);           \
    if (st_ != DCNR_OK) return st_;  \
  } while (0)
// ... and its algorithmic bytes
#define TRYB(cat, nbytes, x)                 \
  do {                                       \
    ProfScope ps_(cat, s, (double)(nbytes)); \
    dcnr_status st_ = (x);                   \
    if (st_ != DCNR_OK) return st_;          \
  } while (0)

// Flags of the fork/join events between the caller's stream and the side
// stream (both on this device: a device-scope release/acquire orders them;
// without the system-scope fence the step measured 4.019 vs 4.051 ms,
// alternating A/B x3 on one box, profiles/lab/r03x_event_fence_ab.txt).
constexpr unsigned SYNC_EV = hipEventDisableTiming | hipEventDisableSystemFence;

// Measured and rejected side-stream pipe variants:
// the apply pass's own completion event as the dependency (+1.4 %), the
// weight-gradient call after the dX GEMM (+3.5 %), fewer workgroups for the
// overlapped weight-gradient GEMMs, BN statistics reduced by the producing
// GEMM's last workgroup (+2.3-3.7 %).

// One side stream per device (created on first use, never destroyed) for the
// backward's work that does not depend on the deep tower; fork/join events
// per call.
dcnr_status side_stream(hipStream_t* out) {
  static std::mutex mu;
  static hipStream_t streams[64] = {};
  int dev = 0;
  DCNR_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) {
    set_error("side stream: device %d out of range", dev);
    return DCNR_BAD_ARG;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (!streams[dev]) DCNR_HIP(hipStreamCreateWithFlags(&streams[dev], hipStreamNonBlocking));
  *out = streams[dev];
  return DCNR_OK;
}
// Every exit path orders the side stream's work before the caller's stream:
// an error return between fork() and join() (a failed hook, a too-small
// scratch) must not let the caller free buffers the side stream still
// writes, so the destructor joins whatever was not joined.
struct SideJoin {
  hipStream_t side = nullptr, main = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr, mark_ev = nullptr;
  bool recorded = false, joined = false;
  dcnr_status fork(hipStream_t s) {
    TRY(side_stream(&side));
    DCNR_HIP(hipEventCreateWithFlags(&fork_ev, SYNC_EV));
    DCNR_HIP(hipEventCreateWithFlags(&join_ev, SYNC_EV));
    DCNR_HIP(hipEventRecord(fork_ev, s));
    DCNR_HIP(hipStreamWaitEvent(side, fork_ev, 0));
    main = s;
    return DCNR_OK;
  }
  dcnr_status record() {
    DCNR_HIP(hipEventRecord(join_ev, side));
    recorded = true;
    return DCNR_OK;
  }
  dcnr_status join(hipStream_t s) {
    DCNR_HIP(hipStreamWaitEvent(s, join_ev, 0));
    joined = true;
    return DCNR_OK;
  }
  // an intermediate point of the side stream's work that `s` waits for alone
  dcnr_status mark() {
    DCNR_HIP(hipEventCreateWithFlags(&mark_ev, SYNC_EV));
    DCNR_HIP(hipEventRecord(mark_ev, side));
    return DCNR_OK;
  }
  dcnr_status wait_mark(hipStream_t s) {
    DCNR_HIP(hipStreamWaitEvent(s, mark_ev, 0));
    return DCNR_OK;
  }
  ~SideJoin() {
    if (main && join_ev && !joined) {   // error path: join everything enqueued so far
      (void)hipEventRecord(join_ev, side);
      (void)hipStreamWaitEvent(main, join_ev, 0);
    }
    if (mark_ev) (void)hipEventDestroy(mark_ev);
    if (fork_ev) (void)hipEventDestroy(fork_ev);
    if (join_ev) (void)hipEventDestroy(join_ev);
  }
};

// dcnr_grad_ready_fn of the model desc, if any
dcnr_status grads_ready(const dcnr_model_desc* desc, int group, hipStream_t s) {
  if (!desc->grad_ready) return DCNR_OK;
  const int rc = desc->grad_ready(desc->grad_ready_ctx, group, (void*)s);
  if (rc != 0) {
    set_error("grad_ready hook failed (%d) for gradient group %d", rc, group);
    return DCNR_HIP_ERROR;
  }
  return DCNR_OK;
}

constexpr int MAX_CAT = 64;
constexpr int MAX_RES = 8;
constexpr int MAX_CROSS = 7;
constexpr int64_t PART_CHUNKS = 2100;  // >= rowcol chunk count (2048 target + rounding)

struct Dims {
  int K, D, Dp, H, Hp, L, R, prec, es;
  int widths[2 + MAX_CAT];
  int64_t rows[2 + MAX_CAT];
  float dropout;
};

dcnr_status make_dims(const dcnr_model_desc* d, Dims* o) {
  if (!d) { set_error("null desc"); return DCNR_BAD_ARG; }
  if (d->n_cat < 0 || d->n_cat > MAX_CAT || (d->n_cat > 0 && !d->cat_rows)) {
    set_error("n_cat=%d unsupported (max %d)", d->n_cat, MAX_CAT);
    return DCNR_BAD_ARG;
  }
  if (d->n_res < 1 || d->n_res > MAX_RES) {
    set_error("n_res_blocks=%d unsupported (1..%d)", d->n_res, MAX_RES);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (d->n_cross < 0 || d->n_cross > MAX_CROSS) {
    set_error("n_cross_layers=%d unsupported (0..%d)", d->n_cross, MAX_CROSS);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  if (d->emb_dim < 1 || d->hidden < 1 || d->n_num < 0 || d->n_users < 1 || d->n_items < 1) {
    set_error("bad model dims");
    return DCNR_BAD_ARG;
  }
  if (d->precision != DCNR_PREC_FP32 && d->precision != DCNR_PREC_BF16) {
    set_error("bad precision %d", d->precision);
    return DCNR_BAD_ARG;
  }
  o->K = d->n_cat;
  o->widths[0] = o->widths[1] = d->emb_dim;
  o->rows[0] = d->n_users;
  o->rows[1] = d->n_items;
  int D = 2 * d->emb_dim;
  for (int k = 0; k < d->n_cat; ++k) {
    int64_t n = d->cat_rows[k];
    if (n < 1) { set_error("cat table %d has %lld rows", k, (long long)n); return DCNR_BAD_ARG; }
    int w = (int)std::sqrt((double)n) + 1;  // train.py:139 int(np.sqrt(n_cat)) + 1
    while ((int64_t)(w - 1) * (w - 1) > n) --w;        // guard fp rounding of sqrt
    while ((int64_t)w * w <= n) ++w;
    o->widths[2 + k] = w;
    o->rows[2 + k] = n;
    D += w;
  }
  D += d->n_num;
  o->D = D;
  o->Dp = (int)rup(D, 8);
  o->H = d->hidden;
  o->Hp = (int)rup(d->hidden, 8);
  o->L = d->n_cross;
  o->R = d->n_res;
  o->prec = d->precision;
  o->es = d->precision == DCNR_PREC_BF16 ? 2 : 4;
  o->dropout = d->dropout;
  if (o->Hp > 2048 || o->D > 1024) {
    set_error("hidden_dim=%d / input_dim=%d unsupported", o->H, o->D);
    return DCNR_UNSUPPORTED_SHAPE;
  }
  return DCNR_OK;
}

// ------------------------------------------------- algorithmic byte counts
// (profiling only): one [B][Hp] activation, its 1-bit mask, one gathered
// input row (ids + embedding rows + dense features), a weight
double act_b(const Dims& d, int64_t B) { return (double)B * d.Hp * d.es; }
double mask_b(const Dims& d, int64_t B) { return (double)B * d.Hp / 8.0; }
double gather_row_b(const Dims& d, int n_num) {
  double w = 0;
  for (int t = 0; t < 2 + d.K; ++t) w += d.widths[t];
  return 8.0 * (2 + d.K) + 4.0 * w + 4.0 * n_num;
}
double w_b(const Dims& d, int K) { return (double)d.Hp * K * d.es; }

// ------------------------------------------------------------- workspace
struct Bump {
  char* base; size_t off = 0;
  explicit Bump(void* b) : base((char*)b) {}
  void* take(size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    void* p = base ? base + off : nullptr;
    off += bytes;
    return p;
  }
};

struct BnBufs { float *scale, *shift, *mean, *invstd; };

struct Layout {
  int* err;
  void* W0p; void* W0t; float* b0p;
  void* W1p[MAX_RES]; void* W1t[MAX_RES]; float* b1p[MAX_RES];
  void* W2p[MAX_RES]; void* W2t[MAX_RES]; float* b2p[MAX_RES];
  void* x0;
  void* h[MAX_RES + 1];
  void* t1[MAX_RES]; void* t2[MAX_RES];
  void* a1;                 // eval: BN1/ReLU output scratch; train: backward scratch (dt1)
  void* a1s[MAX_RES];       // train: each block's dropout(relu(BN1(t1))), saved for dW2
  float* zc; float* zdeep;
  float* headp;             // eval: [head parts][B] deep-head partial dots (null: row_dot)
  char* twp;                // eval, fused tower: the packed weight slices (null: layer by layer)
  BnBufs bn[2 * MAX_RES];
  float* part; double* sums; float* coef;
  double* red2; int* red_cnt;   // reduce_fused scratch (counters zeroed by pack_all)
  // backward
  void* G; void* dt2; void* du; void* da;
  void* dt2b; void* dt1b;   // second dt2 / dt1 set (bf16 train, odd blocks); null: one set
  // per-block backward buffers: all alias G/dt2/du/da/a1 unless
  // DCNR_FLAG_KEEP_INTERMEDIATES gives each block its own
  void* duk[MAX_RES]; void* dt2k[MAX_RES]; void* dak[MAX_RES]; void* dt1k[MAX_RES];
  float* dx0;                 // deep part of dL/dx0, [B][Dq] (Dq = Dp rounded up to 32)
  float* slab; int64_t slab_elems;
  float* slab2;   // the side stream's weight gradients alternate slabs (DwPipe)
  float* sc;                 // forward -> backward cross scalars [B][2L+1]
  float* xcoef; float* xalpha;  // [B][L+1] each (cross_bwd.hip)
  void* cscratch; size_t cscratch_bytes;
  // 1-bit keep masks for the backward GEMM epilogues (bf16, Hp % 32 == 0):
  // mask_a1[j] = [a1_j != 0], mask_h[j] = [h_j > 0] (j >= 1)
  uint8_t* mask_a1[MAX_RES]; uint8_t* mask_h[MAX_RES + 1];
  EmbSortBufs emb;                              // deterministic embedding backward
  double* bce_part;
  uint8_t* rowmap; size_t rowmap_bytes;   // DCNR_FLAG_ROW_MAP: byte per table row (last in ws)
  size_t total;
};

// the backward GEMM epilogues read 1-bit keep masks (bf16 path, mask rows of
// whole 32-bit words) instead of the bf16 activations
bool masks_ok(const Dims& d) { return d.prec == DCNR_PREC_BF16 && d.Hp % 32 == 0; }
// leading dimension of the deep dx0: 32-float (128-B) rows so that each
// embedding table's segment of a row is line-aligned for embed_bwd.hip
int dq_of(const Dims& d) { return (int)rup(d.Dp, 32); }
bool keep_of(const dcnr_model_desc* desc) { return (desc->flags & DCNR_FLAG_KEEP_INTERMEDIATES) != 0; }

// bf16 train: the last block's head pass does not store h_R; the backward's
// BN2 statistics pass rebuilds it from t2, h_{R-1} and the BN2 affine
// (KEEP_INTERMEDIATES still stores it for the stage tests)
bool head_rebuild(const Dims& d, bool train) {
  return train && d.prec == DCNR_PREC_BF16 && bn_add_relu_head_supported(d.prec, d.Hp);
}
bool eval_fuse_ok(const Dims& d) { return d.prec == DCNR_PREC_BF16 && gemm_ws_supported(d.Hp, d.Hp); }

// The eval forward's deep tower as one persistent launch (tower.hip): bf16,
// the shapes it covers (input width <= 512, hidden <= 512), not when the
// stage tests ask for every intermediate, and from TOWER_MIN_B samples (or
// with DCNR_FLAG_FUSED_TOWER): one 128-sample tile per CU walks all 2R+1
// layers in sequence, ~150 us however few tiles there are, while the
// layer-by-layer path spreads each layer over the chip (bench model: 179 vs
// 139 us at 4096 samples, 622 vs 806 us at 131072).
constexpr int64_t TOWER_MIN_B = 16384;
bool tower_ok(const Dims& d, bool train, uint32_t flags, int64_t B) {
  const bool size_ok = B >= TOWER_MIN_B || (flags & DCNR_FLAG_FUSED_TOWER);
  return !train && !(flags & DCNR_FLAG_KEEP_INTERMEDIATES) && size_ok && d.prec == DCNR_PREC_BF16 &&
         tower_supported(d.Dp, d.H, d.R);
}

Layout make_layout(const Dims& d, int64_t B, int mode, void* ws, uint32_t flags = 0) {
  const bool keep = (flags & DCNR_FLAG_KEEP_INTERMEDIATES) != 0;
  Layout L;
  memset(&L, 0, sizeof(L));
  Bump b(ws);
  const bool train = mode == DCNR_TRAIN;
  const size_t es = d.es;
  const size_t act = (size_t)B * d.Hp * es;
  L.err = (int*)b.take(256);
  if (tower_ok(d, train, flags, B)) {   // x0, zc, the packed slices: nothing of the tower in HBM
    L.x0 = b.take((size_t)B * d.Dp * es);
    L.zc = (float*)b.take(B * 4);
    L.twp = (char*)b.take((size_t)tower_ws_bytes(d.H, d.R));
    L.total = b.off + 256;
    return L;
  }
  L.W0p = b.take((size_t)d.Hp * d.Dp * es);
  L.W0t = train ? b.take((size_t)d.Dp * d.Hp * es) : nullptr;
  L.b0p = (float*)b.take(d.Hp * 4);
  for (int j = 0; j < d.R; ++j) {
    L.W1p[j] = b.take((size_t)d.Hp * d.Hp * es);
    L.W2p[j] = b.take((size_t)d.Hp * d.Hp * es);
    L.W1t[j] = train ? b.take((size_t)d.Hp * d.Hp * es) : nullptr;
    L.W2t[j] = train ? b.take((size_t)d.Hp * d.Hp * es) : nullptr;
    L.b1p[j] = (float*)b.take(d.Hp * 4);
    L.b2p[j] = (float*)b.take(d.Hp * 4);
  }
  L.x0 = b.take((size_t)B * d.Dp * es);
  if (train) {
    for (int j = 0; j <= d.R; ++j) L.h[j] = b.take(act);
    for (int j = 0; j < d.R; ++j) { L.t1[j] = b.take(act); L.t2[j] = b.take(act); }
  } else {
    void* h0 = b.take(act);
    void* h1 = b.take(act);
    for (int j = 0; j <= d.R; ++j) L.h[j] = (j & 1) ? h1 : h0;
    void* t = b.take(act);
    for (int j = 0; j < d.R; ++j) L.t1[j] = L.t2[j] = t;
  }
  L.a1 = b.take(act);
  if (train)
    for (int j = 0; j < d.R; ++j) L.a1s[j] = b.take(act);
  if (train && masks_ok(d)) {
    const size_t mb = (size_t)B * d.Hp / 8;
    for (int j = 0; j < d.R; ++j) L.mask_a1[j] = (uint8_t*)b.take(mb);
    for (int j = 1; j < d.R; ++j) L.mask_h[j] = (uint8_t*)b.take(mb);
    if (bn_add_relu_head_supported(d.prec, d.Hp))   // [h_R > 0] for the last block's BN2 apply
      L.mask_h[d.R] = (uint8_t*)b.take(mb);
  }
  L.zc = (float*)b.take(B * 4);
  L.zdeep = (float*)b.take(B * 4);
  // the last eval GEMM's head partials (32-bit buffer offsets: at Hp = 512
  // up to ~33M rows; larger batches take the unfused, M-chunked tail)
  if (!train && !keep && eval_fuse_ok(d) && d.R >= 1 &&
      (int64_t)B * gemm_ws_head_parts(d.Hp) * 4 < (int64_t(1) << 31))
    L.headp = (float*)b.take((size_t)B * gemm_ws_head_parts(d.Hp) * 4);
  for (int i = 0; i < 2 * d.R; ++i) {
    L.bn[i].scale = (float*)b.take(d.Hp * 4);
    L.bn[i].shift = (float*)b.take(d.Hp * 4);
    L.bn[i].mean = (float*)b.take(d.Hp * 4);
    L.bn[i].invstd = (float*)b.take(d.Hp * 4);
  }
  L.part = (float*)b.take((size_t)PART_CHUNKS * 3 * d.Hp * 4);
  L.sums = (double*)b.take((size_t)(3 * d.Hp + 1) * 8);
  L.coef = (float*)b.take((size_t)3 * d.Hp * 4);
  L.red2 = (double*)b.take((size_t)RED_G * 3 * d.Hp * 8);
  L.red_cnt = (int*)b.take(CNT_SLOTS * 4);
  if (train) {
    L.G = b.take(act);
    L.dt2 = b.take(act);
    L.du = b.take(act);
    L.da = b.take(act);
    L.dx0 = (float*)b.take((size_t)B * dq_of(d) * 4);
    // split-K slabs: the fp32 path adapts its splits to 64; the bf16 kernel's
    // split count depends on the tile count (narrow H -> more splits)
    L.slab_elems = std::max<int64_t>({(int64_t)64 * d.Hp * std::max(d.Hp, d.Dp),
                                      (int64_t)gemm_dw_splits(d.Hp, d.Hp, B) * d.Hp * d.Hp,
                                      (int64_t)gemm_dw_splits(d.Hp, d.Dp, B) * d.Hp * d.Dp});
    L.slab = (float*)b.take((size_t)L.slab_elems * 4);
    L.slab2 = (float*)b.take((size_t)L.slab_elems * 4);
    L.sc = (float*)b.take((size_t)B * (2 * d.L + 1) * 4);
    L.xcoef = (float*)b.take((size_t)B * (d.L + 1) * 4);
    L.xalpha = (float*)b.take((size_t)B * (d.L + 1) * 4);
    L.cscratch_bytes = cross_bwd_scratch_bytes(d.D, d.L, B);
    L.cscratch = b.take(L.cscratch_bytes);
    {
      const int64_t n = (int64_t)(2 + d.K) * B;
      L.emb.ids = (uint32_t*)b.take((size_t)n * 4);
      L.emb.keys = (uint32_t*)b.take((size_t)n * 4);
      L.emb.vals = (uint32_t*)b.take((size_t)n * 4);
      L.emb.keys_s = (uint32_t*)b.take((size_t)n * 4);
      L.emb.vals_s = (uint32_t*)b.take((size_t)n * 4);
      L.emb.tmp_bytes = emb_sort_tmp_bytes(d.rows, d.widths, 2 + d.K, B);
      L.emb.tmp = b.take(L.emb.tmp_bytes);
    }
    // bf16: every residual block has its own dt2 / dt1 buffers (blocks 0
    // and 1 take the shared set and dt2b / dt1b): the side stream's
    // weight-gradient GEMMs read them while the main stream goes on, and the
    // main stream never waits for the side stream inside the backward
    // (4.029-4.044 vs 4.068-4.075 ms per step with two sets alternating by
    // block parity and a wait for call n-3, same box, profiles/lab/r04s_dt_per_block_ab.txt;
    // +0.54 GB of workspace at the bench shape)
    const bool own_dt = !keep && d.prec == DCNR_PREC_BF16 && d.R > 1;
    if (own_dt) {
      L.dt2b = b.take(act);
      L.dt1b = b.take(act);
    }
    for (int j = 0; j < d.R; ++j) {
      const bool fresh = own_dt && j > 1;
      L.duk[j] = keep ? b.take(act) : L.du;
      L.dt2k[j] = keep || fresh ? b.take(act) : own_dt && j == 1 ? L.dt2b : L.dt2;
      L.dak[j] = keep ? b.take(act) : L.da;
      L.dt1k[j] = keep || fresh ? b.take(act) : own_dt && j == 1 ? L.dt1b : L.a1;
    }

  }
  L.bce_part = (double*)b.take(bce_ws_bytes());
  if (train && (flags & DCNR_FLAG_ROW_MAP)) {   // last: every other offset as without the flag
    int64_t rows = 0;
    for (int t = 0; t < 2 + d.K; ++t) rows += d.rows[t];
    L.rowmap_bytes = (size_t)rup(rows, 256);
    L.rowmap = (uint8_t*)b.take(L.rowmap_bytes);
  }
  L.total = b.off + 256;
  return L;
}

// ------------------------------------------------------------- params
struct Params {
  const float* tab[2 + MAX_CAT];
  const float *W0, *b0;
  struct Blk {
    const float *w1, *b1, *g1, *be1; float *rm1, *rv1; int64_t* nbt1;
    const float *w2, *b2, *g2, *be2; float *rm2, *rv2; int64_t* nbt2;
  } blk[MAX_RES];
  const float* cb[MAX_CROSS]; const float* cw[MAX_CROSS];
  const float *wf, *bf;
};

Params map_params(const Dims& d, void* const* p) {
  Params P;
  int i = 0;
  for (int t = 0; t < 2 + d.K; ++t) P.tab[t] = (const float*)p[i++];
  P.W0 = (const float*)p[i++];
  P.b0 = (const float*)p[i++];
  for (int j = 0; j < d.R; ++j) {
    auto& B = P.blk[j];
    B.w1 = (const float*)p[i++]; B.b1 = (const float*)p[i++];
    B.g1 = (const float*)p[i++]; B.be1 = (const float*)p[i++];
    B.rm1 = (float*)p[i++]; B.rv1 = (float*)p[i++]; B.nbt1 = (int64_t*)p[i++];
    B.w2 = (const float*)p[i++]; B.b2 = (const float*)p[i++];
    B.g2 = (const float*)p[i++]; B.be2 = (const float*)p[i++];
    B.rm2 = (float*)p[i++]; B.rv2 = (float*)p[i++]; B.nbt2 = (int64_t*)p[i++];
  }
  for (int l = 0; l < d.L; ++l) { P.cb[l] = (const float*)p[i++]; P.cw[l] = (const float*)p[i++]; }
  P.wf = (const float*)p[i++];
  P.bf = (const float*)p[i++];
  return P;
}

struct Grads {
  float* tab[2 + MAX_CAT];
  float *W0, *b0;
  struct Blk { float *w1, *b1, *g1, *be1, *w2, *b2, *g2, *be2; } blk[MAX_RES];
  float* cb[MAX_CROSS]; float* cw[MAX_CROSS];
  float *wf, *bf;
};

Grads map_grads(const Dims& d, void* const* g) {
  Grads G;
  int i = 0;
  for (int t = 0; t < 2 + d.K; ++t) G.tab[t] = (float*)g[i++];
  G.W0 = (float*)g[i++];
  G.b0 = (float*)g[i++];
  for (int j = 0; j < d.R; ++j) {
    auto& B = G.blk[j];
    B.w1 = (float*)g[i++]; B.b1 = (float*)g[i++]; B.g1 = (float*)g[i++]; B.be1 = (float*)g[i++];
    B.w2 = (float*)g[i++]; B.b2 = (float*)g[i++]; B.g2 = (float*)g[i++]; B.be2 = (float*)g[i++];
  }
  for (int l = 0; l < d.L; ++l) { G.cb[l] = (float*)g[i++]; G.cw[l] = (float*)g[i++]; }
  G.wf = (float*)g[i++];
  G.bf = (float*)g[i++];
  return G;
}

GatherDesc make_gather(const Dims& d, const Params& P, int n_num) {
  GatherDesc g;
  memset(&g, 0, sizeof(g));
  g.n_tab = 2 + d.K;
  int off = 0;
  for (int t = 0; t < g.n_tab; ++t) {
    g.tab[t] = P.tab[t];
    g.rows[t] = d.rows[t];
    g.width[t] = d.widths[t];
    g.off[t] = off;
    off += d.widths[t];
  }
  g.n_num = n_num;
  g.D = d.D;
  return g;
}

CrossParams make_cross(const Dims& d, const Params& P) {
  CrossParams c;
  memset(&c, 0, sizeof(c));
  c.L = d.L;
  for (int l = 0; l < d.L; ++l) { c.w[l] = P.cw[l]; c.b[l] = P.cb[l]; }
  c.wf_cross = P.wf + d.H;
  return c;
}

dcnr_status pack_all(const Dims& d, const Params& P, const Layout& L, bool train, hipStream_t s,
                     bool zero_err = false) {
  // weights -> padded T copies (+ transposes for backward); biases -> padded
  // f32; one launch per MAX_PACK descriptors
  std::vector<PackDesc> v;
  auto add = [&](const float* src, void* dst, void* dst_t, int rows, int cols, int ld, int ld_t,
                 int rows_p, int cols_p) {
    PackDesc p{src, dst, dst_t, rows, cols, ld, ld_t, rows_p, cols_p, 0};   // T = the precision
    v.push_back(p);
  };
  add(P.W0, L.W0p, train ? L.W0t : nullptr, d.H, d.D, d.Dp, d.Hp, d.Hp, d.Dp);
  for (int j = 0; j < d.R; ++j) {
    add(P.blk[j].w1, L.W1p[j], train ? L.W1t[j] : nullptr, d.H, d.H, d.Hp, d.Hp, d.Hp, d.Hp);
    add(P.blk[j].w2, L.W2p[j], train ? L.W2t[j] : nullptr, d.H, d.H, d.Hp, d.Hp, d.Hp, d.Hp);
  }
  auto addb = [&](const float* src, float* dst) {
    PackDesc p{src, dst, nullptr, 1, d.H, d.Hp, 0, 1, 0, 1};
    v.push_back(p);
  };
  addb(P.b0, L.b0p);
  // reduce_fused's column-group counters start at zero (a 1-row pack of 0 columns)
  v.push_back(PackDesc{P.b0, L.red_cnt, nullptr, 0, 0, CNT_SLOTS, 0, 1, 0, 1});
  // (eval, index check on: the gather's error word, in the same launch)
  if (zero_err) v.push_back(PackDesc{P.b0, L.err, nullptr, 0, 0, 8, 0, 1, 0, 1});
  for (int j = 0; j < d.R; ++j) { addb(P.blk[j].b1, L.b1p[j]); addb(P.blk[j].b2, L.b2p[j]); }
  for (size_t o = 0; o < v.size(); o += MAX_PACK) {
    PackBatch pb;
    pb.n = (int)std::min<size_t>(MAX_PACK, v.size() - o);
    for (int i = 0; i < pb.n; ++i) pb.d[i] = v[o + i];
    TRYP(DCNR_K_PACK, pack_weights(d.prec, pb, s));
  }
  return DCNR_OK;
}

// C = A . B^T with k-contiguous operands: bf16 -> the weight-stationary
// streaming kernel (gemm_ws.hip) when the weight fits its registers (K <= 512);
// otherwise the generic tiled MFMA kernel (fp32 parity path, K > 512).
dcnr_status gemm_nn(int prec, int epi, const GemmArgs& g, int splits, hipStream_t s) {
  if (prec == DCNR_PREC_BF16 && splits == 1 && gemm_ws_supported(g.K, g.N)) {
    NtArgs a;
    memset(&a, 0, sizeof(a));
    a.X = (const bf16*)g.A; a.ldx = g.lda; a.M = g.M; a.K = (int)g.K;
    a.W = (const bf16*)g.B; a.ldw = g.ldb; a.N = (int)g.N;
    a.C = g.C; a.ldc = g.ldc; a.bias = g.bias;
    a.R = g.resid; a.ldr = g.ldr;
    int ne = epi == EPI_STORE_RESID ? NT_EPI_RESID : (g.out_f32 ? NT_EPI_F32 : NT_EPI_BIAS);
    return gemm_ws(ne, a, s);
  }
  return gemm(prec, false, false, epi, g, splits, s);
}

dcnr_status linear_fwd(const Dims& d, const void* A, int lda, const void* W, int K,
                       const float* bias, void* out, int64_t B, hipStream_t s) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.A = A; g.lda = lda; g.B = W; g.ldb = K;
  g.C = out; g.ldc = d.Hp; g.bias = bias;
  g.M = B; g.N = d.Hp; g.K = K; g.k_per_split = K;
  return gemm_nn(d.prec, EPI_STORE, g, 1, s);
}

// Stats epilogues of the streaming GEMM (BN column partials produced by the
// GEMM that writes the BN input / the BN output gradient) -- bf16 only.
bool epi_stats_ok(const Dims& d) { return masks_ok(d) && gemm_ws_supported(d.Hp, d.Hp); }

// Eval forward with BatchNorm (running statistics) + ReLU (+ residual) in the
// streaming GEMM's epilogue: no t1/t2 round trip through HBM and no rowwise
// passes (bf16, gemm_ws shapes).

// out = relu((A W^T + b) * bn.scale + bn.shift [+ R]); with rs (the layer's
// gamma, beta, running mean, running var) the kernel makes scale / shift
// itself; with headp (needs R) no out: the deep head's partial dots with wf
dcnr_status linear_bn_relu(const Dims& d, const void* A, const void* W, const float* bias,
                           const BnBufs& bn, const void* R, void* out, int64_t B, hipStream_t s,
                           const float* const* rs = nullptr, const float* wf = nullptr,
                           float* headp = nullptr) {
  NtArgs a;
  memset(&a, 0, sizeof(a));
  a.X = (const bf16*)A; a.ldx = d.Hp; a.M = B; a.K = d.Hp;
  a.W = (const bf16*)W; a.ldw = d.Hp; a.N = d.Hp; a.Nr = d.H;
  a.C = out; a.ldc = d.Hp; a.bias = bias;
  a.R = R; a.ldr = d.Hp;
  a.bn_scale = bn.scale; a.bn_shift = bn.shift;
  if (rs) { a.bn_g = rs[0]; a.bn_b = rs[1]; a.bn_rm = rs[2]; a.bn_rv = rs[3]; }
  a.wf = wf; a.headp = headp; a.ldh = B;
  return gemm_ws(headp ? NT_EPI_BN_RESID_RELU_HEAD : R ? NT_EPI_BN_RESID_RELU : NT_EPI_BN_RELU, a, s);
}

// t = A W^T + b  and  part = BN column partials of t, shifted by b (nc rows)
dcnr_status linear_fwd_stats(const Dims& d, const Layout& L, const void* A, int lda, const void* W,
                             int K, const float* bias, void* out, int64_t B, int* nc,
                             hipStream_t s) {
  NtArgs a;
  memset(&a, 0, sizeof(a));
  a.X = (const bf16*)A; a.ldx = lda; a.M = B; a.K = K;
  a.W = (const bf16*)W; a.ldw = K; a.N = d.Hp;
  a.C = out; a.ldc = d.Hp; a.bias = bias;
  a.part = L.part;
  return gemm_ws(NT_EPI_BIAS_STATS, a, s, nc);
}

// C = mask(H) * (X W^T [+ R]) and part = [sum C, sum C*xhat(T)] (BN backward)
// xbn (optional): X is a BatchNorm backward's du; the GEMM's operand is its
// dt = bn_bwd_dt(du, xt, xbn mean / invstd, L.coef), also written to dt_out
// (the row pass folded into this GEMM, gemm_ws.hip XBN)
struct XbnOperand { const void* xt; const BnBufs* bn; void* dt_out; };
dcnr_status linear_dx_bn(const Dims& d, const Layout& L, int epi, const void* X, const void* Wt,
                         const void* R, void* C, const uint8_t* Hbits, float hscale,
                         const void* T, const BnBufs& bn, int64_t B, int* nc, hipStream_t s,
                         const XbnOperand* xbn = nullptr) {
  NtArgs a;
  memset(&a, 0, sizeof(a));
  if (xbn) {
    a.Tx = (const bf16*)xbn->xt;
    a.xmean = xbn->bn->mean; a.xinvstd = xbn->bn->invstd; a.xcoef = L.coef;
    a.dt = (bf16*)xbn->dt_out;
  }
  a.X = (const bf16*)X; a.ldx = d.Hp; a.M = B; a.K = d.Hp;
  a.W = (const bf16*)Wt; a.ldw = d.Hp; a.N = d.Hp;
  a.C = C; a.ldc = d.Hp;
  a.R = R; a.ldr = d.Hp;
  a.hscale = hscale;
  a.Hb = (const uint32_t*)Hbits; a.ldhb = d.Hp / 32;
  a.T = (const bf16*)T; a.ldt = d.Hp;
  a.mean = bn.mean; a.invstd = bn.invstd;
  a.part = L.part;
  return gemm_ws(epi, a, s, nc);
}

// dW[N][Kc] = sum_b dY[b][n] X[b][k]   (real extents Nr x Kr written to out)
// bf16: the 256x256 LDS-DMA weight-gradient kernel (gemm_dw.hip), S batch
// splits, fp32 slabs summed by splitk_reduce
dcnr_status wgrad_bf16(const void* dY, int64_t ldy, int N, const void* X, int64_t ldx, int Kc,
                       int64_t B, float* slab, int64_t slab_elems, float* out, int Nr, int Kr,
                       int accumulate, hipStream_t s) {
  const int S = gemm_dw_splits(N, Kc, B);
  if ((int64_t)S * N * Kc > slab_elems) {
    set_error("wgrad: slab too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  DwArgs a;
  memset(&a, 0, sizeof(a));
  a.A = (const bf16*)dY; a.lda = ldy; a.B = (const bf16*)X; a.ldb = ldx;
  a.C = slab; a.ldc = N; a.slab_stride = (int64_t)N * Kc;   // transposed slab [Kc][N]
  a.Btot = B; a.k_per_split = rup(cdiv(B, S), 64);
  a.N = N; a.K = Kc; a.splits = S;
  TRYB(DCNR_K_GEMM_DW, 2.0 * B * (N + Kc) + 4.0 * Nr * Kr * (accumulate ? 2 : 1), gemm_dw(a, s));
  TRYB(DCNR_K_REDUCE, 4.0 * S * N * Kc + 4.0 * Nr * Kr * (accumulate ? 2 : 1),
       splitk_reduce_t(slab, S, (int64_t)N * Kc, N, Nr, Kr, out, accumulate, s));
  return DCNR_OK;
}

// The backward's bf16 weight gradients run on the side stream: each call's
// gemm_dw + split-K reduce are ordered after the main stream's work so far
// (its dY is complete) and overlap the main stream's next dX GEMM and BN
// passes. The operands stay alive: with a dt2 / dt1 set per block nothing
// writes a call's dY again before the join (lag: never); with one shared set
// (a single residual block) call n's enter() orders the main stream after
// call n-1's GEMM. The reduces share one slab because they are serialised
// on the side stream. join() orders the main stream after all of it. Same kernels, same order per
// output: the gradients are unchanged.
// Round 6: each call's split-K combine runs in the NEXT call's gemm_dw
// launch (its tail, over the workgroups already resident) instead of as a
// launch of its own, which beside the dX GEMMs waited for CUs (150-240 us
// for a 12 us kernel): the calls alternate slabs (L.slab, L.slab2), and the
// last call's combine is launched by join().  Same tiles, same order: the
// gradients are unchanged.
struct DwPipe {
  static constexpr int RING = 4;
  hipStream_t side = nullptr, main = nullptr;
  hipEvent_t in_ev = nullptr, done_ev = nullptr;
  hipEvent_t dw_ev[RING] = {};
  int calls = 0, lag = 1;
  bool pending = false;   // side work enqueued since the last join
  struct Combine { const float* slab; int S; int64_t stride; int ld, Nr, Kr; float* out; int acc; };
  Combine pend{};          // the last call's combine, not yet enqueued (slab != null)
  dcnr_status flush() {
    if (!pend.slab) return DCNR_OK;
    const Combine c = pend;
    pend = Combine{};
    hipStream_t s = side;   // TRYB launches and times on the side stream
    TRYB(DCNR_K_REDUCE, 4.0 * c.S * c.stride + 4.0 * c.Nr * c.Kr * (c.acc ? 2 : 1),
         splitk_reduce_t(c.slab, c.S, c.stride, c.ld, c.Nr, c.Kr, c.out, c.acc, s));
    return DCNR_OK;
  }
  dcnr_status init(hipStream_t side_stream, int lag_calls) {
    side = side_stream;
    lag = lag_calls;
    DCNR_HIP(hipEventCreateWithFlags(&in_ev, SYNC_EV));
    DCNR_HIP(hipEventCreateWithFlags(&done_ev, SYNC_EV));
    for (auto& e : dw_ev) DCNR_HIP(hipEventCreateWithFlags(&e, SYNC_EV));
    return DCNR_OK;
  }
  // order the side stream after the main stream's work so far (and the main
  // stream after call (calls - lag)'s GEMM, see above)
  dcnr_status enter(hipStream_t main_s) {
    if (calls >= lag) DCNR_HIP(hipStreamWaitEvent(main_s, dw_ev[(calls - lag) % RING], 0));
    DCNR_HIP(hipEventRecord(in_ev, main_s));
    DCNR_HIP(hipStreamWaitEvent(side, in_ev, 0));
    main = main_s;
    pending = true;
    return DCNR_OK;
  }
  dcnr_status wgrad(const Layout& L, const void* dY, int64_t ldy, int N, const void* X, int64_t ldx,
                    int Kc, int64_t B, float* out, int Nr, int Kr, int accumulate, hipStream_t main_s) {
    TRY(enter(main_s));
    const int call = calls++;
    hipStream_t s = side;   // TRYB launches and times on the side stream
    // (the full-chip split count: 32 / 16 splits, leaving CUs to the main
    // stream and halving the slab, measured 2 % / 21 % slower per step)
    const int S = gemm_dw_splits(N, Kc, B);
    if ((int64_t)S * N * Kc > L.slab_elems) {
      set_error("wgrad: slab too small");
      return DCNR_WORKSPACE_TOO_SMALL;
    }
    float* slab = (call & 1) ? L.slab2 : L.slab;
    DwArgs a;
    memset(&a, 0, sizeof(a));
    a.A = (const bf16*)dY; a.lda = ldy; a.B = (const bf16*)X; a.ldb = ldx;
    a.C = slab; a.ldc = N; a.slab_stride = (int64_t)N * Kc;   // transposed slab [Kc][N]
    a.Btot = B; a.k_per_split = rup(cdiv(B, S), 64);
    a.N = N; a.K = Kc; a.splits = S;
    double rbytes = 0;
    if (pend.slab) {   // the previous call's combine, in this launch's tail
      a.rslab = pend.slab; a.rsplits = pend.S; a.rstride = pend.stride; a.rld = pend.ld;
      a.rN = pend.Nr; a.rK = pend.Kr; a.rout = pend.out;
      const int vec = pend.Kr % 4 == 0 && (uintptr_t)pend.out % 16 == 0;
      a.racc = (pend.acc ? 1 : 0) | (vec << 1);
      rbytes = 4.0 * pend.S * pend.stride + 4.0 * pend.Nr * pend.Kr * (pend.acc ? 2 : 1);
      if (pend.ld % 4 || pend.stride % 4 || (uintptr_t)pend.slab % 16) {
        set_error("wgrad: slab not 16-B aligned");
        return DCNR_UNSUPPORTED_SHAPE;
      }
    }
    TRYB(DCNR_K_GEMM_DW, 2.0 * B * (N + Kc) + 4.0 * Nr * Kr * (accumulate ? 2 : 1) + rbytes, gemm_dw(a, s));
    DCNR_HIP(hipEventRecord(dw_ev[call % RING], s));
    pend = Combine{slab, S, (int64_t)N * Kc, N, Nr, Kr, out, accumulate};
    return DCNR_OK;
  }
  dcnr_status join(hipStream_t main_s) {
    if (!pending) return DCNR_OK;
    TRY(flush());
    DCNR_HIP(hipEventRecord(done_ev, side));
    DCNR_HIP(hipStreamWaitEvent(main_s, done_ev, 0));
    pending = false;
    return DCNR_OK;
  }
  ~DwPipe() {
    if (pend.slab && side) (void)flush();   // error path: the last combine too
    if (pending && main) {   // error path: order the side work before the caller's stream
      (void)hipEventRecord(done_ev, side);
      (void)hipStreamWaitEvent(main, done_ev, 0);
    }
    for (auto e : {in_ev, done_ev})
      if (e) (void)hipEventDestroy(e);
    for (auto e : dw_ev)
      if (e) (void)hipEventDestroy(e);
  }
};

dcnr_status linear_dw(const Dims& d, const Layout& L, const void* dY, int ldy, int N,
                      const void* X, int ldx, int Kc, int64_t B, float* out, int Nr, int Kr,
                      int accumulate, hipStream_t s, DwPipe* pipe = nullptr) {
  if (d.prec == DCNR_PREC_BF16 && gemm_dw_supported(N, Kc, ldy, ldx, B)) {
    if (pipe) return pipe->wgrad(L, dY, ldy, N, X, ldx, Kc, B, out, Nr, Kr, accumulate, s);
    return wgrad_bf16(dY, ldy, N, X, ldx, Kc, B, L.slab, L.slab_elems, out, Nr, Kr, accumulate, s);
  }
  // the generic path below writes the slab on this stream: the side stream's
  // split-K reduces of earlier calls may still be reading it
  if (pipe) TRY(pipe->join(s));
  int64_t tiles = cdiv(N, 128) * cdiv(Kc, 128);
  int64_t S = std::max<int64_t>(1, std::min<int64_t>(512 / tiles, cdiv(B, 256)));
  int64_t kps = rup(cdiv(B, S), 64);
  S = cdiv(B, kps);
  if (S * (int64_t)N * Kc > L.slab_elems) {
    S = std::max<int64_t>(1, L.slab_elems / ((int64_t)N * Kc));
    kps = rup(cdiv(B, S), 64);
    S = cdiv(B, kps);
  }
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.A = dY; g.lda = ldy; g.B = X; g.ldb = ldx;
  g.C = L.slab; g.ldc = Kc;
  g.M = N; g.N = Kc; g.K = B; g.k_per_split = kps; g.slab_stride = (int64_t)N * Kc;
  TRYB(DCNR_K_GEMM_DW, (double)d.es * B * (N + Kc) + 4.0 * Nr * Kr, gemm(d.prec, true, true, EPI_SPLITK, g, (int)S, s));
  TRYB(DCNR_K_REDUCE, 4.0 * S * N * Kc + 4.0 * Nr * Kr * (accumulate ? 2 : 1),
       splitk_reduce(L.slab, (int)S, (int64_t)N * Kc, Kc, Nr, Kr, out, accumulate, s));
  return DCNR_OK;
}

dcnr_status hook(const dcnr_model_desc* desc, const Dims& d, const Layout& L, hipStream_t s) {
  if (!desc->bn_allreduce) return DCNR_OK;
  int rc = desc->bn_allreduce(desc->bn_allreduce_ctx, L.sums, 3 * (int64_t)d.Hp + 1, (void*)s);
  if (rc != 0) {
    set_error("bn_allreduce hook failed (%d)", rc);
    return DCNR_HIP_ERROR;
  }
  return DCNR_OK;
}

RedFinal red_init(const Layout& L, int mode, double count, int accumulate) {
  RedFinal rf;
  memset(&rf, 0, sizeof(rf));
  rf.mode = mode; rf.count = count; rf.accumulate = accumulate;
  rf.red2 = L.red2; rf.counter = L.red_cnt; rf.sums = L.sums;
  return rf;
}


RedFinal bn_bwd_rf(const Layout& L, int64_t B, const float* gamma, const float* invstd,
                   float* dgamma, float* dbeta, float* dwf, float* dbias_pre, int accumulate) {
  RedFinal rf = red_init(L, RED_BN_BWD, (double)B, accumulate);
  rf.gamma = gamma; rf.invstd = invstd; rf.dgamma = dgamma; rf.dbeta = dbeta; rf.dwf = dwf;
  rf.coef = L.coef;
  rf.dbias_pre = dbias_pre;
  return rf;
}

// nc_pre > 0: the partials of t are already in L.part (from the GEMM epilogue),
// shifted by shiftf (the Linear bias); otherwise a stats pass over t makes them.
dcnr_status bn_layer_fwd(const dcnr_model_desc* desc, const Dims& d, const Layout& L,
                         const void* t, int64_t B, bool train, const float* gamma,
                         const float* beta, float* rm, float* rv, int64_t* nbt,
                         const BnBufs& bb, hipStream_t s, int nc_pre = 0,
                         const float* shiftf = nullptr) {
  BnFinal f{gamma, beta, rm, rv, nbt, bb.scale, bb.shift, bb.mean, bb.invstd};
  if (train) {
    int nc = nc_pre;
    const void* shift = nc_pre ? nullptr : t;
    if (!nc_pre) TRYB(DCNR_K_ROWWISE, act_b(d, B), col_stats(d.prec, t, B, d.Hp, d.Hp, L.part, &nc, s));
    if (!desc->bn_allreduce) {  // local BN: reduce + finalize in one launch
      RedFinal rf = red_init(L, RED_BN_FWD, (double)B, 0);
      rf.f = f;
      rf.shiftf = shiftf;
      TRYP(DCNR_K_REDUCE, reduce_fused(d.prec, L.part, nc, 2, d.Hp, d.H, shift, rf, s));
      return DCNR_OK;
    }
    RedFinal rf = red_init(L, RED_SUMS, (double)B, 0);
    rf.shiftf = shiftf;
    TRYP(DCNR_K_REDUCE, reduce_fused(d.prec, L.part, nc, 2, d.Hp, d.H, shift, rf, s));
    TRY(hook(desc, d, L, s));
  }
  TRYP(DCNR_K_REDUCE, bn_finalize2(L.sums, d.Hp, d.H, train ? 1 : 0, f, s));
  return DCNR_OK;
}

// BN backward reductions: part [nc][NK][Hp] -> dgamma, dbeta (+ dW_f deep half
// when dwf != null) and coef.  Fused into one launch unless SyncBN must sum
// the statistics across ranks first.
dcnr_status bn_bwd_reduce(const dcnr_model_desc* desc, const Dims& d, const Layout& L, int nc,
                          int NK, int64_t B, const float* gamma, const float* invstd,
                          float* dgamma, float* dbeta, float* dwf, float* dbias_pre,
                          int accumulate, hipStream_t s) {
  const int Hp = d.Hp, H = d.H;
  if (!desc->bn_allreduce) {
    RedFinal rf = bn_bwd_rf(L, B, gamma, invstd, dgamma, dbeta, dwf, dbias_pre, accumulate);
    TRYP(DCNR_K_REDUCE, reduce_fused(DCNR_PREC_FP32, L.part, nc, NK, Hp, H, nullptr, rf, s));
    return DCNR_OK;
  }
  RedFinal rf = red_init(L, RED_SUMS, (double)B, 0);
  TRYP(DCNR_K_REDUCE, reduce_fused(DCNR_PREC_FP32, L.part, nc, NK, Hp, H, nullptr, rf, s));
  if (dwf) TRYP(DCNR_K_REDUCE, sums_to_grad(L.sums + 2 * Hp, H, dwf, accumulate, s));
  TRYP(DCNR_K_REDUCE, sums_to_grad(L.sums + Hp, H, dgamma, accumulate, s));
  TRYP(DCNR_K_REDUCE, sums_to_grad(L.sums, H, dbeta, accumulate, s));
  TRY(hook(desc, d, L, s));
  TRYP(DCNR_K_REDUCE, bn_bwd_coef(L.sums, Hp, H, gamma, invstd, L.coef, 1, s));
  if (!accumulate) TRYP(DCNR_K_PACK, fill_zero(dbias_pre, (size_t)H * 4, s));   // exactly 0 (see finalize)
  return DCNR_OK;
}

// Bias gradient: part [nc][NK][Hp], component 0 -> grad[H] (never needs the hook).
dcnr_status bias_reduce(const Dims& d, const Layout& L, int nc, float* grad, int accumulate,
                        hipStream_t s, int NK = 1) {
  RedFinal rf = red_init(L, RED_BIAS, 0.0, accumulate);
  rf.grad = grad;
  TRYP(DCNR_K_REDUCE, reduce_fused(DCNR_PREC_FP32, L.part, nc, NK, d.Hp, d.H, nullptr, rf, s));
  return DCNR_OK;
}

}  // namespace
}  // namespace dcnr

using namespace dcnr;

extern "C" {

int dcnr_abi_version(void) { return DCNR_ABI_VERSION; }
const char* dcnr_last_error(void) { return g_err; }

int64_t dcnr_input_dim(const dcnr_model_desc* desc) {
  Dims d;
  if (make_dims(desc, &d) != DCNR_OK) return -1;
  return d.D;
}

dcnr_status dcnr_workspace_size(const dcnr_model_desc* desc, int64_t B, int mode, size_t* bytes) {
  Dims d;
  TRY(make_dims(desc, &d));
  if (!bytes || B < 0) { set_error("bad args"); return DCNR_BAD_ARG; }
  *bytes = make_layout(d, B, mode, nullptr, desc->flags).total;
  return DCNR_OK;
}

dcnr_status dcnr_workspace_offset(const dcnr_model_desc* desc, int64_t B, int mode, int kind,
                                  int index, int64_t* offset) {
  Dims d;
  TRY(make_dims(desc, &d));
  if (!offset || B < 0 || kind < 0 || kind >= DCNR_WS_KINDS) { set_error("bad args"); return DCNR_BAD_ARG; }
  // a null base yields offsets as pointers from 0 (Bump takes nullptr -> nullptr),
  // so lay out against a fake non-null base
  char* base = (char*)(uintptr_t)4096;
  Layout L = make_layout(d, B, mode, base, desc->flags);
  const bool train = mode == DCNR_TRAIN;
  const int R = d.R;
  auto blk = [&](int n) { return index >= 0 && index < n; };
  const void* p = nullptr;
  switch (kind) {
    case DCNR_WS_X0: p = L.x0; break;
    case DCNR_WS_H: if (blk(R + 1)) p = L.h[index]; break;
    case DCNR_WS_T1: if (blk(R)) p = L.t1[index]; break;
    case DCNR_WS_T2: if (blk(R)) p = L.t2[index]; break;
    case DCNR_WS_A1: if (blk(R) && train) p = L.a1s[index]; break;
    case DCNR_WS_MASK_A1: if (blk(R)) p = L.mask_a1[index]; break;
    case DCNR_WS_MASK_H: if (blk(R)) p = L.mask_h[index]; break;
    case DCNR_WS_BN_MEAN: if (blk(2 * R)) p = L.bn[index].mean; break;
    case DCNR_WS_BN_INVSTD: if (blk(2 * R)) p = L.bn[index].invstd; break;
    case DCNR_WS_BN_SCALE: if (blk(2 * R)) p = L.bn[index].scale; break;
    case DCNR_WS_BN_SHIFT: if (blk(2 * R)) p = L.bn[index].shift; break;
    case DCNR_WS_DU: if (blk(R) && train) p = L.duk[index]; break;
    case DCNR_WS_DT2: if (blk(R) && train) p = L.dt2k[index]; break;
    case DCNR_WS_DA: if (blk(R) && train) p = L.dak[index]; break;
    case DCNR_WS_DT1: if (blk(R) && train) p = L.dt1k[index]; break;
    case DCNR_WS_G: if (train) p = L.G; break;
    case DCNR_WS_DX0: if (train) p = L.dx0; break;
    case DCNR_WS_ZC: p = L.zc; break;
    case DCNR_WS_XCOEF: if (train) p = L.xcoef; break;
    case DCNR_WS_SC: if (train) p = L.sc; break;
    case DCNR_WS_ROW_MAP: p = L.rowmap; break;
  }
  *offset = p ? (int64_t)((const char*)p - base) : -1;
  return DCNR_OK;
}

dcnr_status dcnr_gather_cross(const dcnr_model_desc* desc, void* const* params,
                              const int64_t* user_ids, const int64_t* item_ids,
                              const int64_t* cat_features, const float* num_features, int64_t B,
                              float* x0, int64_t ld_x0, float* cross_out, int64_t ld_cross,
                              int32_t* oob_flag, dcnr_stream_t stream) {
  Dims d;
  TRY(make_dims(desc, &d));
  hipStream_t s = (hipStream_t)stream;
  if (!params || B < 0 || (B > 0 && (!user_ids || !item_ids)) ||
      (d.K > 0 && B > 0 && !cat_features) || (desc->n_num > 0 && B > 0 && !num_features)) {
    set_error("dcnr_gather_cross: null argument");
    return DCNR_BAD_ARG;
  }
  if ((x0 && (ld_x0 < d.D || ld_x0 > INT32_MAX)) ||
      (cross_out && (ld_cross < d.D || ld_cross > INT32_MAX))) {
    set_error("dcnr_gather_cross: row stride below D=%d", d.D);
    return DCNR_BAD_ARG;
  }
  if (B == 0 || (!x0 && !cross_out)) return DCNR_OK;
  Params P = map_params(d, params);
  GatherDesc g = make_gather(d, P, desc->n_num);
  CrossParams cp = make_cross(d, P);
  const GcOut o{cross_out, x0, nullptr, (int)ld_cross, (int)ld_x0};
  const int check = oob_flag != nullptr;
  TRYB(DCNR_K_GATHER_CROSS, (double)B * (gather_row_b(d, desc->n_num) + 4.0 * d.D * ((x0 ? 1 : 0) + (cross_out ? 1 : 0))),
       gather_cross_out(g, cp, user_ids, item_ids, cat_features, num_features, B, o, 0, oob_flag, check, s));
  return DCNR_OK;
}

static dcnr_status forward_body(const dcnr_model_desc* desc, void* const* params,
                                const int64_t* user_ids, const int64_t* item_ids,
                                const int64_t* cat_features, const float* num_features, int64_t B,
                                int mode, uint64_t dropout_seed, float* logits, void* ws,
                                size_t ws_bytes, dcnr_stream_t stream, bool* mirrored);

dcnr_status dcnr_forward(const dcnr_model_desc* desc, void* const* params,
                         const int64_t* user_ids, const int64_t* item_ids,
                         const int64_t* cat_features, const float* num_features, int64_t B,
                         int mode, uint64_t dropout_seed, float* logits, void* ws,
                         size_t ws_bytes, dcnr_stream_t stream) {
  bool mirrored = false;
  TRY(forward_body(desc, params, user_ids, item_ids, cat_features, num_features, B, mode, dropout_seed,
                   logits, ws, ws_bytes, stream, &mirrored));
  // the id-check word to the caller's mirror (the fused eval tower stores it
  // itself); after the forward's last kernel on the stream
  if (B > 0 && !mirrored && desc->error_mirror && (desc->flags & DCNR_FLAG_CHECK_INDICES)) {
    hipStream_t s = (hipStream_t)stream;
    TRYP(DCNR_K_PACK, mirror_word((const int*)ws, desc->error_mirror, s));
  }
  return DCNR_OK;
}

static dcnr_status forward_body(const dcnr_model_desc* desc, void* const* params,
                                const int64_t* user_ids, const int64_t* item_ids,
                                const int64_t* cat_features, const float* num_features, int64_t B,
                                int mode, uint64_t dropout_seed, float* logits, void* ws,
                                size_t ws_bytes, dcnr_stream_t stream, bool* mirrored) {
  Dims d;
  TRY(make_dims(desc, &d));
  hipStream_t s = (hipStream_t)stream;
  const bool train = mode == DCNR_TRAIN;
  if (!params || !logits || !ws || B < 0 || (B > 0 && (!user_ids || !item_ids)) ||
      (d.K > 0 && B > 0 && !cat_features) || (desc->n_num > 0 && B > 0 && !num_features)) {
    set_error("dcnr_forward: null argument");
    return DCNR_BAD_ARG;
  }
  if (train && B < 2) {
    set_error("Expected more than 1 value per channel when training");
    return DCNR_BAD_ARG;
  }
  Layout L = make_layout(d, B, mode, ws, desc->flags);
  if (ws_bytes < L.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, L.total);
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  if (B == 0) return DCNR_OK;
  Params P = map_params(d, params);
  const int check = (desc->flags & DCNR_FLAG_CHECK_INDICES) ? 1 : 0;
  GatherDesc g = make_gather(d, P, desc->n_num);
  CrossParams cp = make_cross(d, P);
  // Train: the weight packing (bf16 copies + transposes of the deep tower's
  // weights) is not read by the gather/cross kernel, so it runs on the side
  // stream under it and the first GEMM waits for it alone (same box, two
  // runs each: 4.033 / 4.045 vs 4.071 / 4.055 ms/step; eval keeps it on the
  // stream: its fork/join cost ~1 % of the eval forward). The embedding
  // backward's id sort needs the ids alone, so it follows there, under this
  // forward (joined before returning, so the caller's id tensors are free to
  // go once the forward's work is done).
  if (L.twp) {
    // eval: gather + cross (x0 bf16, zc) -> the fused deep tower + head
    TowerPack tp;
    memset(&tp, 0, sizeof(tp));
    tp.W0 = P.W0; tp.D = d.D; tp.b0 = P.b0;
    for (int j = 0; j < d.R; ++j) {
      const auto& Bk = P.blk[j];
      tp.w1[j] = Bk.w1; tp.b1[j] = Bk.b1; tp.g1[j] = Bk.g1; tp.be1[j] = Bk.be1; tp.rm1[j] = Bk.rm1; tp.rv1[j] = Bk.rv1;
      tp.w2[j] = Bk.w2; tp.b2[j] = Bk.b2; tp.g2[j] = Bk.g2; tp.be2[j] = Bk.be2; tp.rm2[j] = Bk.rm2; tp.rv2[j] = Bk.rv2;
    }
    tp.wf = P.wf; tp.H = d.H; tp.R = d.R; tp.out = L.twp; tp.err = check ? L.err : nullptr;
    TRYP(DCNR_K_PACK, tower_pack(tp, s));
    const GcOut o{nullptr, L.x0, L.zc, 0, d.Dp, nullptr};
    TRYB(DCNR_K_GATHER_CROSS, (double)B * (gather_row_b(d, desc->n_num) + (double)d.Dp * d.es + 4.0),
         gather_cross_out(g, cp, user_ids, item_ids, cat_features, num_features, B, o, 1, L.err, check, s));
    TowerArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.x0 = (const bf16*)L.x0; ta.ldx = d.Dp; ta.M = B; ta.Dp = d.Dp; ta.H = d.H; ta.R = d.R;
    ta.wp = L.twp; ta.zc = L.zc; ta.bias = P.bf; ta.logits = logits;
    ta.err = L.err;
    ta.err_mirror = check ? desc->error_mirror : nullptr;
    *mirrored = true;
    // algorithmic bytes: the x0 rows + zc in, the logits out (the packed
    // weights are L2-resident: every CU streams the same 4.7 MB)
    TRYB(DCNR_K_TOWER, (double)B * (d.Dp * d.es + 8.0), eval_tower(ta, s));
    return DCNR_OK;
  }
  SideJoin sj;
  if (train) {
    TRY(sj.fork(s));
    hipStream_t s = sj.side;
    TRY(pack_all(d, P, L, train, s));
    TRY(sj.mark());
  } else {
    TRY(pack_all(d, P, L, train, s, check != 0));
  }
  // (train: the pack runs on the side stream beside the gather, so the
  // error word is zeroed here, before it)
  if (check && train) TRYP(DCNR_K_PACK, fill_zero(L.err, 4, s));
  if (train) {
    EmbBwdDesc eb;
    memset(&eb, 0, sizeof(eb));
    eb.n_tab = g.n_tab;
    for (int t = 0; t < g.n_tab; ++t) { eb.rows[t] = g.rows[t]; eb.width[t] = g.width[t]; }
    hipStream_t s = sj.side;   // TRYB launches and times on the side stream
    TRYB(DCNR_K_EMB_SORT, 2.0 * 8.0 * g.n_tab * B + 8.0 * B * (2 + d.K) + 4.0 * B * 2,
         emb_sort(eb, user_ids, item_ids, cat_features, B, L.emb, s));
    TRY(sj.record());
  }
  {
    const GcOut o{nullptr, L.x0, L.zc, 0, d.Dp, train ? L.sc : nullptr};
    TRYB(DCNR_K_GATHER_CROSS, (double)B * (gather_row_b(d, desc->n_num) + (double)d.Dp * d.es + 4.0),
         gather_cross_out(g, cp, user_ids, item_ids, cat_features, num_features, B, o,
                          d.prec == DCNR_PREC_BF16, L.err, check, s));
  }
  if (train) TRY(sj.wait_mark(s));   // packed weights, biases, zeroed reduction counters
  TRYB(DCNR_K_GEMM_FWD, (double)B * d.Dp * d.es + act_b(d, B) + w_b(d, d.Dp),
       linear_fwd(d, L.x0, d.Dp, L.W0p, d.Dp, L.b0p, L.h[0], B, s));
  if (!train && eval_fuse_ok(d)) {
    if (L.headp) {
      // each GEMM makes its layer's running-stat affine itself; the last
      // block's GEMM ends in the deep head dot (no h_R), summed with zc + bf
      for (int j = 0; j < d.R; ++j) {
        const auto& Bk = P.blk[j];
        const float* rs1[4] = {Bk.g1, Bk.be1, Bk.rm1, Bk.rv1};
        const float* rs2[4] = {Bk.g2, Bk.be2, Bk.rm2, Bk.rv2};
        const bool last = j == d.R - 1;
        TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
             linear_bn_relu(d, L.h[j], L.W1p[j], L.b1p[j], L.bn[2 * j], nullptr, L.a1, B, s, rs1));
        TRYB(DCNR_K_GEMM_FWD, (last ? 2 * act_b(d, B) + 4.0 * B * gemm_ws_head_parts(d.Hp) : 3 * act_b(d, B)) + w_b(d, d.Hp),
             linear_bn_relu(d, L.a1, L.W2p[j], L.b2p[j], L.bn[2 * j + 1], L.h[j], last ? nullptr : L.h[j + 1],
                            B, s, rs2, last ? P.wf : nullptr, last ? L.headp : nullptr));
      }
      const int np = gemm_ws_head_parts(d.Hp);
      TRYB(DCNR_K_HEAD, (4.0 * np + 8.0) * B, head_parts(L.headp, np, L.zc, P.bf, B, logits, s));
      return DCNR_OK;
    }
    // every layer's running-stat affine in one launch
    BnEvalBatch eb;
    memset(&eb, 0, sizeof(eb));
    eb.n = 2 * d.R; eb.N = d.Hp; eb.Nr = d.H;
    for (int j = 0; j < d.R; ++j) {
      const auto& Bk = P.blk[j];
      const BnBufs& b1 = L.bn[2 * j];
      const BnBufs& b2 = L.bn[2 * j + 1];
      eb.f[2 * j] = BnFinal{Bk.g1, Bk.be1, Bk.rm1, Bk.rv1, Bk.nbt1, b1.scale, b1.shift, b1.mean, b1.invstd};
      eb.f[2 * j + 1] = BnFinal{Bk.g2, Bk.be2, Bk.rm2, Bk.rv2, Bk.nbt2, b2.scale, b2.shift, b2.mean, b2.invstd};
    }
    TRYP(DCNR_K_REDUCE, bn_eval_finalize(eb, s));
    for (int j = 0; j < d.R; ++j) {
      TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
           linear_bn_relu(d, L.h[j], L.W1p[j], L.b1p[j], L.bn[2 * j], nullptr, L.a1, B, s));
      TRYB(DCNR_K_GEMM_FWD, 3 * act_b(d, B) + w_b(d, d.Hp),
           linear_bn_relu(d, L.a1, L.W2p[j], L.b2p[j], L.bn[2 * j + 1], L.h[j], L.h[j + 1], B, s));
    }
    TRYB(DCNR_K_HEAD, act_b(d, B) + 4.0 * B, row_dot(d.prec, L.h[d.R], d.Hp, d.H, P.wf, B, L.zdeep, s));
    TRYB(DCNR_K_HEAD, 12.0 * B, head_logits(L.zdeep, L.zc, P.bf, B, logits, s));
    return DCNR_OK;   // (eval: nothing forked)
  }
  const float p = train ? d.dropout : 0.f;
  for (int j = 0; j < d.R; ++j) {
    const auto& Bk = P.blk[j];
    const bool fuse = train && epi_stats_ok(d);   // BN partials from the GEMM epilogue
    int nc = 0;
    if (fuse)
      TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
           linear_fwd_stats(d, L, L.h[j], d.Hp, L.W1p[j], d.Hp, L.b1p[j], L.t1[j], B, &nc, s));
    else
      TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
           linear_fwd(d, L.h[j], d.Hp, L.W1p[j], d.Hp, L.b1p[j], L.t1[j], B, s));
    TRY(bn_layer_fwd(desc, d, L, L.t1[j], B, train, Bk.g1, Bk.be1, Bk.rm1, Bk.rv1, Bk.nbt1,
                     L.bn[2 * j], s, nc, fuse ? L.b1p[j] : nullptr));
    void* a1 = train ? L.a1s[j] : L.a1;
    TRYB(DCNR_K_ROWWISE, 2 * act_b(d, B) + (train ? mask_b(d, B) : 0), bn_relu_drop(d.prec, L.t1[j], a1, B, d.Hp, d.Hp, L.bn[2 * j].scale, L.bn[2 * j].shift, p,
                     dropout_seed, j, s, train ? L.mask_a1[j] : nullptr));
    if (fuse)
      TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
           linear_fwd_stats(d, L, a1, d.Hp, L.W2p[j], d.Hp, L.b2p[j], L.t2[j], B, &nc, s));
    else
      TRYB(DCNR_K_GEMM_FWD, 2 * act_b(d, B) + w_b(d, d.Hp),
           linear_fwd(d, a1, d.Hp, L.W2p[j], d.Hp, L.b2p[j], L.t2[j], B, s));
    TRY(bn_layer_fwd(desc, d, L, L.t2[j], B, train, Bk.g2, Bk.be2, Bk.rm2, Bk.rv2, Bk.nbt2,
                     L.bn[2 * j + 1], s, nc, fuse ? L.b2p[j] : nullptr));
    const bool head = j == d.R - 1 && bn_add_relu_head_supported(d.prec, d.Hp);
    if (head)   // last block: residual + ReLU + deep head dot + logits in one pass
      TRYB(DCNR_K_ROWWISE, (head_rebuild(d, train) && !keep_of(desc) ? 2 : 3) * act_b(d, B) + 12.0 * B,
           bn_add_relu_head(d.prec, L.t2[j], L.h[j],
                            head_rebuild(d, train) && !keep_of(desc) ? nullptr : L.h[j + 1], B, d.Hp, d.Hp,
                                            L.bn[2 * j + 1].scale, L.bn[2 * j + 1].shift, P.wf,
                                            d.H, L.zc, P.bf, logits, s, train ? L.mask_h[d.R] : nullptr));
    else
      TRYB(DCNR_K_ROWWISE, 3 * act_b(d, B) + (train && j + 1 < d.R ? mask_b(d, B) : 0), bn_add_relu2(d.prec, L.t2[j], L.h[j], L.h[j + 1], B, d.Hp, d.Hp,
                                        L.bn[2 * j + 1].scale, L.bn[2 * j + 1].shift, s,
                                        train && j + 1 < d.R ? L.mask_h[j + 1] : nullptr));
  }
  if (!bn_add_relu_head_supported(d.prec, d.Hp)) {
    TRYB(DCNR_K_HEAD, act_b(d, B) + 4.0 * B, row_dot(d.prec, L.h[d.R], d.Hp, d.H, P.wf, B, L.zdeep, s));
    TRYB(DCNR_K_HEAD, 12.0 * B, head_logits(L.zdeep, L.zc, P.bf, B, logits, s));
  }
  if (train) TRY(sj.join(s));   // the sorted ids (workspace) for dcnr_backward
  return DCNR_OK;
}

dcnr_status dcnr_backward(const dcnr_model_desc* desc, void* const* params, void* const* grads,
                          const int64_t* user_ids, const int64_t* item_ids,
                          const int64_t* cat_features, const float* num_features, int64_t B,
                          const float* dlogits, uint64_t dropout_seed, int accumulate, void* ws, size_t ws_bytes,
                          dcnr_stream_t stream) {
  Dims d;
  TRY(make_dims(desc, &d));
  hipStream_t s = (hipStream_t)stream;
  if (!params || !grads || !dlogits || !ws || B < 2) {
    set_error("dcnr_backward: bad argument");
    return DCNR_BAD_ARG;
  }
  Layout L = make_layout(d, B, DCNR_TRAIN, ws, desc->flags);
  if (ws_bytes < L.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, L.total);
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  Params P = map_params(d, params);
  Grads Gr = map_grads(d, grads);
  const float* dz = dlogits;
  const int Hp = d.Hp, H = d.H;
  const float p = d.dropout;
  const bool rowmap = (desc->flags & DCNR_FLAG_ROW_MAP) != 0;
  if (rowmap && (accumulate || !L.rowmap)) {
    set_error("dcnr_backward: DCNR_FLAG_ROW_MAP needs accumulate = 0");
    return DCNR_BAD_ARG;
  }
  // dense embedding grads: zeroed; the per-row sums (emb_segment_sum) then
  // write every row an id references.  (On the side stream under the deep
  // tower instead: 3.99-4.00 vs 3.98-3.99 ms/step, same box; kept here.)
  // DCNR_FLAG_ROW_MAP: only the row map is zeroed; the sums mark the rows
  // they write and the optimizer reads unmarked rows as 0.
  if (rowmap) {
    TRYB(DCNR_K_PACK, (double)L.rowmap_bytes, fill_zero(L.rowmap, L.rowmap_bytes, s));
  } else if (!accumulate) {
    void* zp[2 + MAX_CAT];
    int64_t zn[2 + MAX_CAT];
    for (int t = 0; t < 2 + d.K; ++t) { zp[t] = Gr.tab[t]; zn[t] = d.rows[t] * d.widths[t] * 4; }
    double zb = 0;
    for (int t = 0; t < 2 + d.K; ++t) zb += (double)zn[t];
    TRYB(DCNR_K_PACK, zb, fill_zero_multi(2 + d.K, zp, zn, s));
  }

  // embedding backward, part 1 (the stable sort of the (table row, sample)
  // pairs) ran under the train forward (dcnr_forward); its result is in ws
  GatherDesc g = make_gather(d, P, desc->n_num);
  EmbBwdDesc eb;
  memset(&eb, 0, sizeof(eb));
  eb.n_tab = g.n_tab;
  eb.touched = rowmap ? L.rowmap : nullptr;
  for (int t = 0; t < g.n_tab; ++t) {
    eb.grad[t] = Gr.tab[t]; eb.rows[t] = g.rows[t]; eb.width[t] = g.width[t]; eb.off[t] = g.off[t];
  }
  // The cross backward depends on dz and the forward's outputs alone: it
  // runs on a side stream under the deep-tower backward and joins before the
  // dense-gradient hook.
  SideJoin sj;
  TRY(sj.fork(s));
  const CrossParams cpx = make_cross(d, P);
  {
  hipStream_t s = sj.side;   // TRYB launches and times on the side stream
  // ---- cross network + head bias (low-rank form, from the forward's
  // per-sample scalars, dz and the stored x0 alone; cross_bwd.hip)
  CrossGrads cg;
  memset(&cg, 0, sizeof(cg));
  for (int l = 0; l < d.L; ++l) { cg.dw[l] = Gr.cw[l]; cg.db[l] = Gr.cb[l]; }
  cg.dwf_cross = Gr.wf + H;
  cg.dbf = Gr.bf;
  TRYB(DCNR_K_CROSS_BWD, (double)B * (4.0 * (2 * d.L + 1) + 4.0 + 8.0 * (d.L + 1)) +
                             (double)B * d.Dp * d.es,
       cross_backward(cpx, d.D, L.sc, dz, L.x0, d.prec == DCNR_PREC_BF16, d.Dp, B, cg, L.xcoef,
                      L.xalpha, L.cscratch, L.cscratch_bytes, accumulate, s));
  }
  TRY(sj.record());
  DwPipe dwp;
  DwPipe* pipe = nullptr;
  // (not while kernel classes are being timed: there every launch is priced
  // alone, on the main stream, as before the overlap -- except in profile
  // mode 2, which times the side stream's gemm_dw launches in place)
  if (d.prec == DCNR_PREC_BF16 && (!g_prof || g_prof_mode == 2)) {
    // with a dt2 / dt1 set per block the main stream never waits for the
    // side stream before the join (one shared set: after the previous call)
    TRY(dwp.init(sj.side, keep_of(desc) || L.dt2b ? 1 << 30 : 1));
    pipe = &dwp;
  }

  const void* Gin = nullptr;  // gradient wrt the current block output (null: rank-1 dz*wf)
  const bool fuse = epi_stats_ok(d);   // BN partials from the dX GEMM epilogues
  // the BN backward's row passes folded into those GEMMs (bf16, K = Hp in (256, 512])
  const bool xbn_ok = fuse && d.prec == DCNR_PREC_BF16 && gemm_ws_xbn_supported(NT_EPI_DROP_BN, d.Hp, d.Hp);
  int nc_du = 0;   // > 0: L.du and its BN2 partials were made by the previous dX GEMM
  bool b0_done = false;   // the initial layer's bias gradient came with G (NT_EPI_RESID_SUM)
  for (int j = d.R - 1; j >= 0; --j) {
    const auto& Bk = P.blk[j];
    auto& Gk = Gr.blk[j];
    const BnBufs& bn1 = L.bn[2 * j];
    const BnBufs& bn2 = L.bn[2 * j + 1];
    int nc = 0;
    // this block's backward buffers (one shared set unless KEEP_INTERMEDIATES)
    void* du = L.duk[j];
    void* dt2 = L.dt2k[j];
    void* da = L.dak[j];
    void* dt1 = L.dt1k[j];
    // ---- out = relu(BN2(t2) + h_j):  du, BN2 backward
    if (nc_du) {
      TRY(bn_bwd_reduce(desc, d, L, nc_du, 2, B, Bk.g2, bn2.invstd, Gk.g2, Gk.be2, nullptr,
                        Gk.b2, accumulate, s));
    } else {
      const bool rebuild = !Gin && j == d.R - 1 && head_rebuild(d, true);
      TRYB(DCNR_K_ROWWISE, 3 * act_b(d, B) + (Gin ? act_b(d, B) : 4.0 * B), bwd_bn2_stats3(d.prec, Gin, dz, P.wf, L.h[j + 1], L.t2[j], bn2.mean,
                                          bn2.invstd, B, Hp, Hp, du, L.part, &nc, s,
                                          rebuild ? L.h[j] : nullptr, bn2.scale, bn2.shift));
      // dbeta2, dgamma2 and (last block only) dW_f[:H]
      TRY(bn_bwd_reduce(desc, d, L, nc, 3, B, Bk.g2, bn2.invstd, Gk.g2, Gk.be2,
                        Gin ? nullptr : Gr.wf, Gk.b2, accumulate, s));
    }
    const bool rank1 = !Gin && j == d.R - 1 && L.mask_h[d.R] && d.prec == DCNR_PREC_BF16;
    // the BN2 backward's row pass folded into the DROP_BN dX GEMM (du and t2
    // in, dt2 out for dW2) where that GEMM runs the fused epilogue
    const bool xbn2 = fuse && !rank1 && xbn_ok;
    if (rank1)
      TRYB(DCNR_K_ROWWISE, 2 * act_b(d, B) + mask_b(d, B) + 4.0 * B,
           bwd_bn2_apply_rank1(L.mask_h[d.R], dz, P.wf, L.t2[j], bn2.mean, bn2.invstd, L.coef, B, Hp, Hp,
                               dt2, s));
    else if (!xbn2)
      TRYB(DCNR_K_ROWWISE, 3 * act_b(d, B), bwd_bn2_apply2(d.prec, du, L.t2[j], bn2.mean, bn2.invstd, L.coef, B, Hp, Hp,
                         dt2, L.part, &nc, s));
    // ---- layer2: dW2 = dt2^T a1 ; da = dt2 W2 (the weight gradient after
    // the GEMM that makes dt2 when the row pass is folded in)
    if (!xbn2) TRY(linear_dw(d, L, dt2, Hp, Hp, L.a1s[j], Hp, Hp, B, Gk.w2, H, H, accumulate, s, pipe));
    if (fuse) {
      // dy1 = (dt2 W2) * [a1 != 0] / (1-p): relu and dropout masks from the
      // saved activation, BN1 partials in the same pass
      const XbnOperand xo{L.t2[j], &bn2, dt2};
      TRYB(DCNR_K_GEMM_DX, (xbn2 ? 5 : 3) * act_b(d, B) + mask_b(d, B) + w_b(d, d.Hp),
           linear_dx_bn(d, L, NT_EPI_DROP_BN, xbn2 ? du : dt2, L.W2t[j], nullptr, da, L.mask_a1[j],
                        p > 0.f ? 1.f / (1.f - p) : 1.f, L.t1[j], bn1, B, &nc, s, xbn2 ? &xo : nullptr));
      if (xbn2) TRY(linear_dw(d, L, dt2, Hp, Hp, L.a1s[j], Hp, Hp, B, Gk.w2, H, H, accumulate, s, pipe));
    } else {
      GemmArgs g;
      memset(&g, 0, sizeof(g));
      g.A = dt2; g.lda = Hp; g.B = L.W2t[j]; g.ldb = Hp; g.C = da; g.ldc = Hp;
      g.M = B; g.N = Hp; g.K = Hp; g.k_per_split = Hp;
      TRYB(DCNR_K_GEMM_DX, 2 * act_b(d, B) + w_b(d, d.Hp), gemm_nn(d.prec, EPI_STORE, g, 1, s));
      // ---- relu/dropout + BN1 backward
      TRYB(DCNR_K_ROWWISE, 3 * act_b(d, B), bwd_bn1_stats(d.prec, da, L.t1[j], bn1.scale, bn1.shift, bn1.mean,
                                         bn1.invstd, B, Hp, Hp, p, dropout_seed, j, L.part, &nc, s));
    }
    TRY(bn_bwd_reduce(desc, d, L, nc, 2, B, Bk.g1, bn1.invstd, Gk.g1, Gk.be1, nullptr, Gk.b1,
                        accumulate, s));
    // the BN1 backward's row pass folded into the RESID_BN dX GEMM likewise
    // (block 0: into the RESID GEMM that makes G)
    const bool xbn1 = fuse && xbn_ok;
    if (!xbn1) {
      TRYB(DCNR_K_ROWWISE, 3 * act_b(d, B), bwd_bn1_apply2(d.prec, da, L.t1[j], bn1.mean, bn1.invstd, L.coef, B, Hp, Hp, dt1,
                         L.part, &nc, s));
      // ---- layer1: dW1 = dt1^T h_j ; G = dt1 W1 + du
      TRY(linear_dw(d, L, dt1, Hp, Hp, L.h[j], Hp, Hp, B, Gk.w1, H, H, accumulate, s, pipe));
    }
    if (fuse && j > 0) {
      // G is only consumed by block j-1's BN2 backward: emit its du = G * [h_j > 0]
      // (in place over this block's du, the residual operand, unless
      // KEEP_INTERMEDIATES) and the partials
      const BnBufs& bp = L.bn[2 * (j - 1) + 1];
      const XbnOperand xo{L.t1[j], &bn1, dt1};
      TRYB(DCNR_K_GEMM_DX, (xbn1 ? 6 : 4) * act_b(d, B) + mask_b(d, B) + w_b(d, d.Hp),
           linear_dx_bn(d, L, NT_EPI_RESID_BN, xbn1 ? da : dt1, L.W1t[j], du, L.duk[j - 1], L.mask_h[j], 1.f,
                        L.t2[j - 1], bp, B, &nc_du, s, xbn1 ? &xo : nullptr));
      if (xbn1) TRY(linear_dw(d, L, dt1, Hp, Hp, L.h[j], Hp, Hp, B, Gk.w1, H, H, accumulate, s, pipe));
      Gin = L.duk[j - 1];
    } else if (xbn1) {   // G = dt1 W1 + du, dt1 made from da and t1 in the GEMM,
                         // G's column sums (the initial layer's bias gradient) in its epilogue
      NtArgs a;
      memset(&a, 0, sizeof(a));
      a.Tx = (const bf16*)L.t1[j];
      a.xmean = bn1.mean; a.xinvstd = bn1.invstd; a.xcoef = L.coef;
      a.dt = (bf16*)dt1;
      a.X = (const bf16*)da; a.ldx = Hp; a.M = B; a.K = Hp;
      a.W = (const bf16*)L.W1t[j]; a.ldw = Hp; a.N = Hp;
      a.C = L.G; a.ldc = Hp;
      a.R = du; a.ldr = Hp;
      a.part = L.part;
      int ncg = 0;
      TRYB(DCNR_K_GEMM_DX, 5 * act_b(d, B) + w_b(d, d.Hp), gemm_ws(NT_EPI_RESID_SUM, a, s, &ncg));
      TRY(linear_dw(d, L, dt1, Hp, Hp, L.h[j], Hp, Hp, B, Gk.w1, H, H, accumulate, s, pipe));
      TRY(bias_reduce(d, L, ncg, Gr.b0, accumulate, s, 2));
      b0_done = true;
      Gin = L.G;
      nc_du = 0;
    } else {
      GemmArgs g;
      memset(&g, 0, sizeof(g));
      g.A = dt1; g.lda = Hp; g.B = L.W1t[j]; g.ldb = Hp; g.C = L.G; g.ldc = Hp;
      g.resid = du; g.ldr = Hp;
      g.M = B; g.N = Hp; g.K = Hp; g.k_per_split = Hp;
      TRYB(DCNR_K_GEMM_DX, 3 * act_b(d, B) + w_b(d, d.Hp), gemm_nn(d.prec, EPI_STORE_RESID, g, 1, s));
      Gin = L.G;
      nc_du = 0;
    }
  }
  // ---- initial layer: the weight gradient on the side stream (after block
  // 0's); the bias gradient came with G (b0_done) or is a column-sum pass
  // here on the main stream, ahead of the dx0 GEMM.  The side stream's queue
  // sets the backward's tail: with the column sums on it, the optimizer
  // waited 135 us for it while the main stream was done
  // (profiles/r06fin_step_timeline.txt)
  TRY(linear_dw(d, L, L.G, Hp, Hp, L.x0, d.Dp, d.Dp, B, Gr.W0, H, d.D, accumulate, s, pipe));
  if (!b0_done) {
    int nc = 0;
    TRYB(DCNR_K_ROWWISE, act_b(d, B), col_sum(d.prec, L.G, B, Hp, Hp, L.part, &nc, s));
    TRY(bias_reduce(d, L, nc, Gr.b0, accumulate, s));
  }
  TRY(sj.join(s));   // the side stream's cross gradients, coefficients and sorted ids
  // and the weight gradients; without a hook nothing reads them before the
  // optimizer, so they join at the end (under the dx0 GEMM and embedding sums)
  if (desc->grad_ready) TRY(dwp.join(s));
  TRY(grads_ready(desc, DCNR_GRADS_DENSE, s));   // every non-embedding gradient is enqueued
  {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = L.G; g.lda = Hp; g.B = L.W0t; g.ldb = Hp; g.C = L.dx0; g.ldc = dq_of(d); g.out_f32 = 1;
    g.M = B; g.N = d.Dp; g.K = Hp; g.k_per_split = Hp;
    TRYB(DCNR_K_GEMM_DX, act_b(d, B) + 4.0 * B * d.Dp + w_b(d, d.Dp), gemm_nn(d.prec, EPI_STORE, g, 1, s));
  }
  // ---- embedding backward part 2: sorted (table row, sample) pairs -> per row
  // sum of the deep dx0 segments + sum of the cross coefficients
  double ew = 0;
  for (int t = 0; t < 2 + d.K; ++t) ew += d.widths[t];
  eb.nv = d.L + 1;
  for (int l = 0; l < d.L; ++l) eb.V[l] = cpx.w[l];
  eb.V[d.L] = cpx.wf_cross;
  TRYB(DCNR_K_EMB_SUM, (double)B * (4.0 * ew + (8.0 + 4.0 * (d.L + 1)) * g.n_tab),
       emb_segment_sum(eb, L.emb, B, L.dx0, dq_of(d), L.xcoef, accumulate, s));
  if (!desc->grad_ready) TRY(dwp.join(s));
  TRY(grads_ready(desc, DCNR_GRADS_EMBEDDING, s));
  return DCNR_OK;
}

dcnr_status dcnr_gather_rows(const int64_t* idx, int64_t n, int64_t n_src, int32_t n_arrays,
                             const void* const* src, void* const* dst, const int64_t* row_bytes,
                             dcnr_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!src || !dst || !row_bytes || (n > 0 && !idx)) {
    set_error("dcnr_gather_rows: null argument");
    return DCNR_BAD_ARG;
  }
  TRYP(DCNR_K_SERVE, gather_rows(idx, n, n_src, n_arrays, src, dst, row_bytes, s));
  return DCNR_OK;
}

dcnr_status dcnr_candidate_union(const int64_t* positives, int64_t Q, const int64_t* knn_idx,
                                 int32_t k, int64_t* out_rows, int32_t* out_count,
                                 dcnr_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (Q < 0 || (Q > 0 && (!positives || !knn_idx || !out_rows || !out_count))) {
    set_error("dcnr_candidate_union: bad argument");
    return DCNR_BAD_ARG;
  }
  if (Q == 0) return DCNR_OK;
  TRYP(DCNR_K_SERVE, candidate_union(positives, Q, knn_idx, k, out_rows, out_count, s));
  return DCNR_OK;
}

dcnr_status dcnr_ranking_batch(const int64_t* item_rows, int64_t n, int64_t user_row,
                               const int64_t* item_cat, int32_t n_cat, const float* item_num,
                               int32_t n_num, int64_t n_items, int64_t* user_ids,
                               int64_t* item_ids, int64_t* cat_features, float* num_features,
                               dcnr_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n < 0 || n_items < 1 || n_cat < 0 || n_num < 0 ||
      (n > 0 && (!item_rows || !user_ids || !item_ids || (n_cat && (!item_cat || !cat_features)) ||
                 (n_num && (!item_num || !num_features))))) {
    set_error("dcnr_ranking_batch: bad argument");
    return DCNR_BAD_ARG;
  }
  TRYP(DCNR_K_SERVE, ranking_batch(item_rows, n, user_row, item_cat, n_cat, item_num, n_num,
                                   n_items, user_ids, item_ids, cat_features, num_features, s));
  return DCNR_OK;
}

dcnr_status dcnr_rank_by_score(const float* scores, int64_t n, int64_t* order,
                               dcnr_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n < 0 || (n > 0 && (!scores || !order))) {
    set_error("dcnr_rank_by_score: bad argument");
    return DCNR_BAD_ARG;
  }
  TRYP(DCNR_K_SERVE, rank_desc(scores, n, order, s));
  return DCNR_OK;
}

dcnr_status dcnr_mmr_rerank(const float* table, const float* inv_norms, int32_t d,
                            const int64_t* rows, const float* scores, int64_t n,
                            float lambda_param, int32_t top_k, int64_t* out_pos,
                            int32_t* out_count, dcnr_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n < 0 || top_k < 1 || (n > 0 && (!table || !inv_norms || !rows || !scores || !out_pos ||
                                       !out_count))) {
    set_error("dcnr_mmr_rerank: bad argument");
    return DCNR_BAD_ARG;
  }
  TRYP(DCNR_K_SERVE, mmr_rerank(table, inv_norms, d, rows, scores, n, lambda_param, top_k,
                                out_pos, out_count, s));
  return DCNR_OK;
}

size_t dcnr_bce_workspace_size(void) { return bce_ws_bytes() + 256; }

dcnr_status dcnr_emb_touched_rows(const dcnr_model_desc* desc, const void* ws, size_t ws_bytes,
                                  int64_t B, int32_t n_tables, const int32_t* tables,
                                  const int64_t* elem_off, int64_t shard_elems, int32_t world,
                                  int64_t* out_offsets, int64_t* table_counts,
                                  int64_t* owner_counts, dcnr_stream_t stream) {
  Dims d;
  TRY(make_dims(desc, &d));
  if (!ws || B < 0 || n_tables < 1 || n_tables > 2 + d.K || !tables || !elem_off ||
      !out_offsets || !table_counts || !owner_counts) {
    set_error("dcnr_emb_touched_rows: bad argument");
    return DCNR_BAD_ARG;
  }
  Layout L = make_layout(d, B, DCNR_TRAIN, (void*)ws, desc->flags);
  if (ws_bytes < L.total) {
    set_error("workspace too small: %zu < %zu", ws_bytes, L.total);
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  TouchedArgs a;
  memset(&a, 0, sizeof(a));
  a.n = n_tables;
  a.shard = shard_elems;
  a.world = world;
  for (int i = 0; i < n_tables; ++i) {
    const int t = tables[i];
    if (t < 0 || t >= 2 + d.K) {
      set_error("dcnr_emb_touched_rows: table %d out of range", t);
      return DCNR_BAD_ARG;
    }
    uint32_t base = 0;
    for (int u = 0; u < t; ++u) base += (uint32_t)d.rows[u];
    a.tab[i] = t;
    a.base[i] = base;
    a.width[i] = d.widths[t];
    a.elem_off[i] = elem_off[i];
  }
  return emb_touched_rows(a, L.emb, B, out_offsets, table_counts, owner_counts,
                          (hipStream_t)stream);
}

dcnr_status dcnr_sparse_pack(const float* grad, const int64_t* offsets, int64_t ld,
                             const int64_t* table_counts, int32_t n_tables, int32_t width,
                             int64_t* out_offsets, float* out_rows, dcnr_stream_t stream) {
  if (!grad || !offsets || !table_counts || !out_offsets || !out_rows || ld < 0 || n_tables < 1 ||
      width < 1) {
    set_error("dcnr_sparse_pack: bad argument");
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  TRYP(DCNR_K_SERVE, sparse_pack(grad, offsets, ld, table_counts, n_tables, width, out_offsets, out_rows, s));
  return DCNR_OK;
}

dcnr_status dcnr_sparse_accumulate(float* shard, int64_t shard_lo, int64_t shard_elems, int32_t width,
                                   const int64_t* offsets, const float* rows,
                                   const int64_t* source_counts, int32_t n_sources,
                                   dcnr_stream_t stream) {
  if (!shard || shard_lo < 0 || shard_elems < 0 || width < 1 || n_sources < 0 ||
      (n_sources > 0 && !source_counts)) {
    set_error("dcnr_sparse_accumulate: bad argument");
    return DCNR_BAD_ARG;
  }
  int64_t n = 0;
  for (int r = 0; r < n_sources; ++r) {
    if (source_counts[r] < 0) { set_error("dcnr_sparse_accumulate: negative count"); return DCNR_BAD_ARG; }
    n += source_counts[r];
  }
  if (n > 0 && (!offsets || !rows)) {
    set_error("dcnr_sparse_accumulate: null rows");
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  TRYP(DCNR_K_SERVE, sparse_accumulate(shard, shard_lo, shard_elems, width, offsets, rows, source_counts,
                                       n_sources, s));
  return DCNR_OK;
}

dcnr_status dcnr_bce_with_logits(const float* logits, const float* labels, int64_t B, float* loss,
                                 float* dlogits, float grad_scale, void* ws, size_t ws_bytes,
                                 dcnr_stream_t stream) {
  if (!logits || !labels || !loss || !ws || B < 1) {
    set_error("dcnr_bce_with_logits: bad argument");
    return DCNR_BAD_ARG;
  }
  if (ws_bytes < bce_ws_bytes()) {
    set_error("dcnr_bce_with_logits: workspace too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  hipStream_t s = (hipStream_t)stream;
  TRYP(DCNR_K_HEAD, bce(logits, labels, B, loss, dlogits, grad_scale, (double*)ws, s));
  return DCNR_OK;
}

dcnr_status dcnr_adam_step(int32_t n_tensors, float* const* params, const float* const* grads,
                           float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                           float lr, float beta1, float beta2, float eps, float weight_decay,
                           int64_t step, int decoupled, dcnr_stream_t stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel)) ||
      step < 1) {
    set_error("dcnr_adam_step: bad argument");
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  double nparam = 0;
  for (int i = 0; i < n_tensors; ++i) nparam += (double)numel[i];
  TRYB(DCNR_K_ADAM, 28.0 * nparam, adam(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, lr, beta1, beta2,
                         eps, weight_decay, step, decoupled, s));
  return DCNR_OK;
}

dcnr_status dcnr_adam_step_rows(int32_t n_tensors, float* const* params, const float* const* grads,
                                float* const* exp_avg, float* const* exp_avg_sq, const int64_t* numel,
                                const uint8_t* const* row_map, const int32_t* row_width,
                                float lr, float beta1, float beta2, float eps, float weight_decay,
                                int64_t step, int decoupled, dcnr_stream_t stream) {
  if (n_tensors < 0 || (n_tensors > 0 && (!params || !grads || !exp_avg || !exp_avg_sq || !numel ||
                                          !row_map || !row_width)) || step < 1) {
    set_error("dcnr_adam_step_rows: bad argument");
    return DCNR_BAD_ARG;
  }
  double nbytes = 0;
  for (int i = 0; i < n_tensors; ++i) {
    if (row_map[i] && (row_width[i] < 1 || numel[i] % row_width[i])) {
      set_error("dcnr_adam_step_rows: tensor %d: %lld elements in rows of %d", i, (long long)numel[i],
                row_width[i]);
      return DCNR_BAD_ARG;
    }
    // p, m, v read and written, the map byte per row; the gradient of a
    // mapped tensor only where marked (a share the library does not know:
    // not counted, so the figure is a floor)
    nbytes += (row_map[i] ? 24.0 : 28.0) * (double)numel[i] +
              (row_map[i] ? (double)numel[i] / row_width[i] : 0.0);
  }
  hipStream_t s = (hipStream_t)stream;
  TRYB(DCNR_K_ADAM, nbytes, adam(n_tensors, params, grads, exp_avg, exp_avg_sq, numel, lr, beta1, beta2,
                                 eps, weight_decay, step, decoupled, s, row_map, row_width));
  return DCNR_OK;
}

dcnr_status dcnr_row_inv_norms(const float* table, int64_t N, int32_t d, float* inv_norms,
                               dcnr_stream_t stream) {
  if (!table || !inv_norms || d < 1 || N < 0) {
    set_error("dcnr_row_inv_norms: bad argument");
    return DCNR_BAD_ARG;
  }
  return row_inv_norms(table, N, d, inv_norms, (hipStream_t)stream);
}

size_t dcnr_cosine_topk_workspace_size(int64_t N, int64_t Q, int32_t k) {
  if (N < 1 || Q < 1 || k < 1) return 256;   // nothing to plan (cosine_topk returns or rejects)
  return topk_ws(N, Q, k) + 256;
}

dcnr_status dcnr_cosine_pack_rows(const float* table, const float* inv_norms, int64_t N, int32_t d,
                                  uint16_t* packed, dcnr_stream_t stream) {
  if (!table || !inv_norms || !packed || d < 1 || N < 0) {
    set_error("dcnr_cosine_pack_rows: bad argument");
    return DCNR_BAD_ARG;
  }
  return cosine_pack_rows(table, inv_norms, N, d, (bf16*)packed, (hipStream_t)stream);
}

dcnr_status dcnr_cosine_topk_packed(const float* table, const float* inv_norms, const uint16_t* packed,
                                    int64_t N, int32_t d, const float* queries, int64_t Q, int32_t k,
                                    int64_t* idx, float* dist, void* ws, size_t ws_bytes,
                                    dcnr_stream_t stream) {
  // (no queries: the query and output pointers may be null)
  if (!table || !inv_norms || (Q > 0 && (!queries || !idx || !dist || !ws))) {
    set_error("dcnr_cosine_topk: null argument");
    return DCNR_BAD_ARG;
  }
  if (k > N) {
    set_error("Expected n_neighbors <= n_samples_fit, but n_neighbors = %d, n_samples_fit = %lld",
              k, (long long)N);
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  TRYB(DCNR_K_KNN, (double)N * (4.0 * d + 4.0),
       cosine_topk(table, inv_norms, (const bf16*)packed, N, d, queries, Q, k, idx, dist, ws, ws_bytes, s));
  return DCNR_OK;
}

dcnr_status dcnr_cosine_topk(const float* table, const float* inv_norms, int64_t N, int32_t d,
                             const float* queries, int64_t Q, int32_t k, int64_t* idx, float* dist,
                             void* ws, size_t ws_bytes, dcnr_stream_t stream) {
  return dcnr_cosine_topk_packed(table, inv_norms, nullptr, N, d, queries, Q, k, idx, dist, ws, ws_bytes,
                                 stream);
}

dcnr_status dcnr_topk_merge(const float* dist, const int64_t* idx, int32_t lists, int64_t Q,
                            int32_t k, int64_t* out_idx, float* out_dist, dcnr_stream_t stream) {
  if (!dist || !idx || !out_idx || !out_dist || Q < 0) {
    set_error("dcnr_topk_merge: bad argument");
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  TRYB(DCNR_K_KNN, (double)lists * Q * k * 12.0 + Q * k * 12.0,
       topk_merge(dist, idx, lists, Q, k, out_idx, out_dist, s));
  return DCNR_OK;
}

dcnr_status dcnr_linear_bf16(const void* X, int64_t ldx, int64_t M, int32_t K, const void* W,
                             int64_t ldw, int32_t N, const float* bias, void* C, int64_t ldc,
                             int out_f32, dcnr_stream_t stream) {
  if (!X || !W || !C || M < 0 || K < 1 || N < 1) {
    set_error("dcnr_linear_bf16: bad argument");
    return DCNR_BAD_ARG;
  }
  hipStream_t s = (hipStream_t)stream;
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.A = X; g.lda = ldx; g.B = W; g.ldb = ldw; g.C = C; g.ldc = ldc; g.bias = bias;
  g.M = M; g.N = N; g.K = K; g.k_per_split = K; g.out_f32 = out_f32 ? 1 : 0;
  TRYP(DCNR_K_GEMM_FWD, gemm_nn(DCNR_PREC_BF16, EPI_STORE, g, 1, s));
  return DCNR_OK;
}

size_t dcnr_linear_wgrad_workspace_size(int32_t N, int32_t K, int64_t B) {
  if (N < 1 || K < 1 || B < 1) return 0;   // (dcnr_linear_wgrad_bf16 rejects these shapes)
  return (size_t)gemm_dw_splits(N, K, B) * (size_t)N * (size_t)K * sizeof(float);
}

dcnr_status dcnr_linear_wgrad_bf16(const void* dY, int64_t ldy, const void* X, int64_t ldx,
                                   int64_t B, int32_t N, int32_t K, float* dW, int accumulate,
                                   void* ws, size_t ws_bytes, dcnr_stream_t stream) {
  if (!dY || !X || !dW || !ws || B < 1 || N < 1 || K < 1 || !gemm_dw_supported(N, K, ldy, ldx, B)) {
    set_error("dcnr_linear_wgrad_bf16: bad or unsupported arguments");
    return DCNR_BAD_ARG;
  }
  if (ws_bytes < dcnr_linear_wgrad_workspace_size(N, K, B)) {
    set_error("workspace too small");
    return DCNR_WORKSPACE_TOO_SMALL;
  }
  return wgrad_bf16(dY, ldy, N, X, ldx, K, B, (float*)ws, (int64_t)(ws_bytes / 4), dW, N, K,
                    accumulate, (hipStream_t)stream);
}

void dcnr_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_pm);
  g_prof = on != 0;
  g_prof_mode = on;
}

dcnr_status dcnr_profile_collect(double* ms, int64_t* launches, int32_t n) {
  return dcnr_profile_collect_bytes(ms, launches, nullptr, n);
}

dcnr_status dcnr_profile_collect_bytes(double* ms, int64_t* launches, double* bytes, int32_t n) {
  std::vector<ProfRec> recs;
  {
    std::lock_guard<std::mutex> lk(g_pm);
    recs.swap(g_recs);
  }
  for (int i = 0; i < n; ++i) {
    if (ms) ms[i] = 0.0;
    if (launches) launches[i] = 0;
    if (bytes) bytes[i] = 0.0;
  }
  dcnr_status st = DCNR_OK;
  for (auto& r : recs) {
    float t = 0.f;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) {
      set_error("profile: event query failed");
      st = DCNR_HIP_ERROR;
    }
    if (r.cat >= 0 && r.cat < n) {
      if (ms) ms[r.cat] += t;
      if (launches) launches[r.cat] += 1;
      if (bytes) bytes[r.cat] += r.bytes;
    }
  }
  std::lock_guard<std::mutex> lk(g_pm);
  for (auto& r : recs) { g_pool.push_back(r.a); g_pool.push_back(r.b); }
  return st;
}

dcnr_status dcnr_check_errors(void* ws, size_t ws_bytes, dcnr_stream_t stream) {
  if (!ws || ws_bytes < 4) { set_error("bad workspace"); return DCNR_BAD_ARG; }
  int flag = 0;
  DCNR_HIP(hipMemcpyAsync(&flag, ws, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  DCNR_HIP(hipStreamSynchronize((hipStream_t)stream));
  if (flag) {
    set_error("index out of range in self");
    return DCNR_INDEX_OOB;
  }
  return DCNR_OK;
}

}  // extern "C"
