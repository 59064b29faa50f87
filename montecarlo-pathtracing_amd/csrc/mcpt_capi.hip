// mcpt_capi.hip — C ABI, device half: context, scene upload (repack to device records),
// framebuffer / row-band sharding, render launches, accumulator read-back.
//
// Replaces the GL state of the reference's render path: Texture2D uploads
// (bvh_gpu/gpu_bvh_scene.cpp:143-160), the RGB32F FBO + blend (MontecarloGPU/montecarlo.cpp:
// 384-386, 420-467), the uniform ABI (montecarlo.cpp:439-453) and the corner-ray vertex
// shader (shaders/raytracer.vert:9-22, evaluated here once per launch on the host).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/mcpt.h"
#include "mcpt_internal.h"
#include "mcpt_math.h"

// The detail of the calling thread's last failed call (set_err), with its status.  "fresh"
// until mcpt_error_string hands it out once or a later call fails without a detail (every bare
// error return goes through mcpt_err_bare, which drops it), so a detail is never attached to a
// later error that did not set one (HIP errors keep theirs: mcpt_error_string(MCPT_ERR_HIP)
// always returns it).
static thread_local char g_last_error[256] = "";
static thread_local char g_detail[320] = "";
static thread_local int g_last_status = 0;
static thread_local bool g_fresh = false;

static int set_err(int status, const char* what, hipError_t e = hipSuccess) {
  if (e != hipSuccess)
    std::snprintf(g_last_error, sizeof(g_last_error), "%s: %s", what, hipGetErrorString(e));
  else
    std::snprintf(g_last_error, sizeof(g_last_error), "%s", what);
  g_last_status = status;
  g_fresh = true;
  return status;
}

int mcpt_err_bare(int status) {
  g_fresh = false;
  return status;
}

#define HIP_OR_RETURN(call)                                         \
  do {                                                              \
    hipError_t e_ = (call);                                         \
    if (e_ != hipSuccess) return set_err(MCPT_ERR_HIP, #call, e_);  \
  } while (0)

// default bound of the segment-sum buffer of one sub-launch (4 GiB of the 288 GB of HBM: 172
// segments = 5,504 passes per launch at 1080p, 43 = 1,376 at 4K, so a C5 step of 1,024 passes
// is one launch: +0.7 % against four launches under a 1 GiB bound, whose grid tails add up,
// profiles/r03_ab_partial_budget_c5.jsonl; mcpt_set_partial_budget / MCPT_PARTIAL_BYTES)
constexpr size_t kDefaultPartialBudget = size_t(4) << 30;
// per-pass value store of pass stealing (mesh launches), per render lane
constexpr size_t kStealBudget = size_t(8) << 30;
// render calls whose events a context keeps (mcpt_kernel_ms_back)
constexpr int kTimingRing = 64;
// work-item order (mcpt_order.hip): launches with at least this many work items run in the
// order sorted from an earlier launch of their shape; the order is re-sorted every
// kOrderRefresh launches of the shape (costs drift little: the same tiles and pass counts)
constexpr long long kOrderMinItems = 4096;
constexpr int kOrderRefresh = 16;
// split items (mesh launches): at most this many of the costliest items run in
// mcpt::kSplitPieces pass ranges each (RenderParams::split_n; 100 MB of per-pass values)
constexpr int kSplitMax = 1024;

struct mcpt_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // scene (device records)
  float4* d_nodes = nullptr;
  int* d_leaves = nullptr;
  int* d_ptype = nullptr;
  float4* d_prims = nullptr;
  int n_prims = 0, depth = 0, nb_emissive = 0;
  bool has_scene = false;
  // triangle meshes
  int4* d_minfo = nullptr;
  float4* d_mpairs = nullptr;      // mesh BVH child-pair records (SceneT::mpairs)
  float4* d_mleaftris = nullptr;   // mesh leaf triangle records (SceneT::mleaftris)
  int4* d_mtris = nullptr;
  float4* d_mverts = nullptr;
  float4* d_mnorms = nullptr;
  int n_meshes = 0, flat_face = 0;
  std::vector<int> mesh_ids;     // per primitive: mesh id of a CODE_MESH record, else -1
  // framebuffer
  float* d_accum = nullptr;
  size_t accum_bytes = 0;
  int W = 0, H = 0, band_rows = 1, world = 1, rank = 0, n_local_rows = 0;
  int* d_rows = nullptr;            // global row of each local row (n_local_rows)
  std::vector<int> rows;
  int pass_count = 0;
  bool has_target = false;
  unsigned long long* d_events = nullptr;
  // per sub-launch of a render call: (start, after the path-tracing kernel, after the combine
  // kernel); a call is split into sub-launches at chunk boundaries (partial_budget).  The last
  // kTimingRing calls keep their events (mcpt_kernel_ms_back), so a caller can time a run of
  // calls without waiting after each; ring_pos = the last call's slot.
  std::vector<hipEvent_t> evs[kTimingRing];
  int ring_n_sub[kTimingRing] = {};
  std::vector<char> ring_lane[kTimingRing];   // per sub-launch: a lane launch
  int ring_pos = 0;
  long long n_timed = 0;            // render calls timed so far
  int n_sub = 0;                    // sub-launches of the last render call
  int pass_split = 0;               // the last render call ran one segment per pass (launch())
  bool timed = false;
  size_t partial_budget = kDefaultPartialBudget;
  int traversal = MCPT_TRAVERSAL_AUTO;
  // AUTO schedule: the first sizeable launches after a scene upload run each candidate twice
  // (kernel time per sample from the launch events), later launches use the fastest (results
  // are identical either way).  Candidates: 1 = per-lane walk, 2 = wave-coherent walk (BVH depth
  // < 8), per-lane walks with 2 (4, on launches of >= 2 pass segments) or 4 (5, >= 4 segments)
  // pass segments per work item, and for BVH depth >= 8 per-lane walks with the deep knobs (leaf
  // batch 16, walk exit 40) and 4 (6) or 8 (7, >= 8 segments) segments per item.  (3, the stream
  // schedule, is only run when selected explicitly.)
  // trial launches whose timing is not collected yet, oldest first: a trial's time is read when the
  // call after the next one starts, so that consecutive trials overlap on the render lanes as the
  // settled launches do (its period is then measured as the settled launches' is)
  struct TunePending {
    int cand = 0;                   // its candidate
    double samples = 0.0;           // its samples
    long long shape[2] = {0, 0};    // its (local pixels, passes)
    int slot = 0;                   // its timing-ring slot
  };
  TunePending pend[2];
  int n_pend = 0;
  long long meas_shape[2] = {0, 0};      // shape the measurements below were taken on
  int meas_segs = 0;                // pass segments of that shape (which candidates apply)
  double tune_ns[8] = {0.0};       // best ns per sample measured, by candidate (same shape)
  int tune_cnt[8] = {0};            // trials of each candidate so far
  bool deep_auto = false;           // the deep-knob candidates apply (BVH depth >= 8, per-lane kernel)
  int tune_choice = 0;              // resolved candidate once all are measured
  int walk_exit = -1;               // mcpt_set_walk_exit; -1: by BVH depth
  int leaf_batch = -1;              // MCPT_LEAF_BATCH env (tuning); -1: default
  // stream schedule (MCPT_TRAVERSAL_STREAM): slot pool, payload queues, counters
  int n_cu = 0;                     // compute units of the device (persistent grids)
  float* d_slots = nullptr;         // SF_COUNT x slot capacity
  float* d_queue = nullptr;         // 2 x QF_COUNT x slot capacity
  unsigned* d_sctr = nullptr;       // SC_COUNT counters per pool
  long long slot_cap = 0;           // slots of d_slots / d_queue
  unsigned* h_sctr = nullptr;       // pinned: each pool's counters read back after each batch (2 x pools x SC_COUNT)
  hipEvent_t batch_ev[2] = {nullptr, nullptr};
  hipStream_t pool_stream[2] = {nullptr, nullptr};   // the pools' iterations overlap on two streams
  hipEvent_t pool_ev[3] = {nullptr, nullptr, nullptr};   // fork / join of the pool streams
  int stream_slots = 0;             // MCPT_STREAM_SLOTS env / mcpt_set_stream_pool (0: default)
  int stream_refill = -1;           // MCPT_STREAM_REFILL env / mcpt_set_stream_pool (-1: default)
  long long stream_iters = 0;       // iterations of the last stream render (diagnostics)
  // Render lanes (round 6): the sub-launches of render calls alternate between two lanes, each with
  // its own HIP stream, segment-sum buffer and work-item order state, so that a launch's render
  // kernel can start while the previous launch's last workgroups still run (its tail).  The
  // combines stay in call order on `stream`; a lane's next render waits for the lane's previous
  // combine (its buffers free).  Lane launches are only used once AUTO has settled, for launches
  // of several pass segments (a one-segment launch adds into the accumulator itself).
  struct Lane {
    hipStream_t stream = nullptr;
    hipEvent_t freed = nullptr;     // on `stream` after the lane's last combine: its buffers are free
    bool freed_stale = false;       // launches in order on `stream` used the lane since (not recorded:
                                    // launch-bound calls skip the record; the next waiter records it)
    hipEvent_t tail = nullptr;      // on the lane's stream after its last operation
    float* d_partial = nullptr;     // pass-segment sums (launches spanning > 1 chunk)
    size_t partial_bytes = 0;
    // work-item order (mcpt_order.hip): item costs of the lane's last ordered launch, the order
    // sorted from them (costliest first) and the launch shape it belongs to
    unsigned* d_item_cost = nullptr;
    unsigned* d_cost_sorted = nullptr;
    int* d_item_iota = nullptr;
    int* d_item_perm = nullptr;
    int* d_split_of = nullptr;      // split items: item -> split index (-1: whole)
    float* d_split_pass = nullptr;  // split items: the later pieces' per-pass values
    float* d_steal = nullptr;       // pass stealing: every pass's value (RenderParams::steal_vals)
    size_t steal_bytes = 0;
    int* d_split_n = nullptr;       // split items: how many (from the last sort)
    void* d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    long long item_cap = 0;
    long long order_key[8] = {};
    bool order_valid = false;
    int order_age = 0;              // launches since the order was last sorted
  };
  Lane lanes[2];
  int next_lane = 0;                // the lane of the next sub-launch
  int overlap = 1;                  // MCPT_OVERLAP (0: every launch in order on `stream`)
  int prev_lane = -1;               // the lane of the previous sub-launch if it was a lane launch, else -1
};

// events of sub-launch k of the last call: start / mid / stop
// (4 per sub-launch: 0 the timed interval's start — for a lane launch that follows one on the
// other lane, that launch's render end —, 1 the render's end, 2 the combine's end, 3 the render's
// own start on its stream: 3 -> 1 is the kernel's whole span, overlapped tails included)
constexpr int kEvPerSub = 4;
static hipEvent_t ev_start(const mcpt_ctx* c, int k) { return c->evs[c->ring_pos][kEvPerSub * k]; }
static hipEvent_t ev_stop(const mcpt_ctx* c, int k) { return c->evs[c->ring_pos][kEvPerSub * k + 2]; }
// event i of sub-launch k in ring slot `slot` (0 start, 1 mid, 2 stop)
static hipEvent_t ev_at(const mcpt_ctx* c, int slot, int k, int i) { return c->evs[slot][kEvPerSub * k + i]; }
static hipError_t ensure_events(mcpt_ctx* c, int slot, int n_sub) {
  if ((int)c->ring_lane[slot].size() < n_sub) c->ring_lane[slot].resize(n_sub, 0);
  while ((int)c->evs[slot].size() < kEvPerSub * n_sub) {
    hipEvent_t e = nullptr;
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) return r;
    c->evs[slot].push_back(e);
  }
  return hipSuccess;
}
// (path-tracing kernel ms, combine kernel ms) summed over the sub-launches of the call in ring
// slot `slot` (waits for it)
static hipError_t slot_launch_ms(const mcpt_ctx* c, int slot, float* trace_ms, float* combine_ms) {
  *trace_ms = 0.0f; *combine_ms = 0.0f;
  const std::vector<hipEvent_t>& v = c->evs[slot];
  for (int k = 0; k < c->ring_n_sub[slot]; ++k) {
    float a = 0.0f, b = 0.0f;
    hipError_t e = hipEventSynchronize(v[kEvPerSub * k + 2]);
    if (e == hipSuccess) e = hipEventElapsedTime(&a, v[kEvPerSub * k], v[kEvPerSub * k + 1]);
    if (e == hipSuccess) e = hipEventElapsedTime(&b, v[kEvPerSub * k + 1], v[kEvPerSub * k + 2]);
    if (e != hipSuccess) return e;
    *trace_ms += a; *combine_ms += b;
  }
  return hipSuccess;
}
// the same for the last call
static hipError_t sub_launch_ms(const mcpt_ctx* c, float* trace_ms, float* combine_ms) {
  return slot_launch_ms(c, c->ring_pos, trace_ms, combine_ms);
}

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}

// Deep-BVH walk (walk_run's SUSPEND kernel): suspend the walk loop at <= walk_exit walking
// lanes and batch leaf visits (>= leaf_batch waiting lanes).  Both pay off when traversals
// are long (depth >= 8: scenes 3/7/8 +63-76 % over v6, profiles/r01_ab21_leaf_batch.jsonl)
// and cost extra rounds when they are short (scenes 1/2/6: -10-30 %), so they are off there.
static int resolve_walk_exit(const mcpt_ctx* c) {
  if (c->walk_exit >= 0) return c->walk_exit;
  // mesh scenes: a lane's walk includes its instances' mesh DFSs (walk_run_mesh), long and
  // very unequal across lanes: leaving the loop once 24 lanes are done more than doubled
  // throughput in round 1 (1 M-triangle meshes 173 -> 381 Msamples/s, walk exit 40); with the
  // one-fetch mesh records of round 5, exit 24 (40 lanes done) measures best (24 / 32 / 40 / 48:
  // 840 / 784 / 760 / 691 Msamples/s, profiles/r05_ab_mesh_walk_exit.jsonl)
  if (c->n_meshes > 0) return 24;
  return c->depth >= 8 ? 16 : 0;
}
static int resolve_leaf_batch(const mcpt_ctx* c) {
  if (c->leaf_batch >= 0) return c->leaf_batch;
  return c->depth >= 8 ? 8 : 0;
}

constexpr int kCandStream = MCPT_TRAVERSAL_STREAM, kCandLaneSeg2 = 4, kCandLaneSeg4 = 5;
// deep-BVH candidates (BVH depth >= 8): per-lane walks with the deep knobs at leaf batch 16 and
// walk exit 40 (instead of 8 / 16), four or eight segments per item.  Scene 8 (C4 workload):
// 539 / 544 Msamples/s at walk exit 32 against 515 for the defaults at four segments; walk exit
// 40 another +2..3 % at eight segments (552 / 540; with the node rows loaded together 574 / 558);
// scene 3 prefers the defaults (profiles/r03_ab_deep_knobs.jsonl, r03_ab_deep_walk_exit.jsonl,
// r02_deep_knobs_sweep.jsonl): timed, not guessed
constexpr int kCandDeepSeg4 = 6, kCandDeepSeg8 = 7, kCandLast = kCandDeepSeg8;
constexpr int kDeepLeafBatch = 16, kDeepWalkExit = 40;
// ... and they leave the walk loop only once at least 8 walks of the call have ended (shading
// rounds with more lanes): C4 shape 593 -> 608 Msamples/s; 4 / 12 / 16: 603 / 605 / 604
// (profiles/r04_ab_walk_min_done.jsonl)
constexpr int kDeepMinDone = 8;
// pass split (launch()): launches with fewer than this many work items per CU, of at most
// kPassSplitMaxPasses passes
constexpr int kPassSplitItemsPerCu = 4, kPassSplitMaxPasses = 256;
// AUTO does not time the wave-coherent walk on BVHs at least this deep: the union of a wave's
// incoherent secondary rays visits nearly the whole tree, and on scene 8 (C4) one trial launch
// took 8.36 s against 1.81 s for the per-lane walk (profiles/r03_r03s_c4_kernel_stats.csv).  The
// stream schedule (candidate 3) is never timed by AUTO: it was 5 % behind the megakernel on
// scene 8 and 4-7x slower on shallow scenes; mcpt_set_traversal selects it.
constexpr int kWaveAutoMaxDepth = 7;
// the candidates that apply to a launch of `segs` pass segments
static bool cand_applies(const mcpt_ctx* c, int cand, long long segs) {
  return cand == 1 || (cand == 2 && c->depth <= kWaveAutoMaxDepth) || (cand == kCandLaneSeg2 && segs >= 2) ||
         (cand == kCandLaneSeg4 && segs >= 4) || (cand == kCandDeepSeg4 && c->deep_auto && segs >= 4) ||
         (cand == kCandDeepSeg8 && c->deep_auto && segs >= 8);
}
static int cand_seg_per_item(int cand) {
  return cand == kCandLaneSeg2 ? 2 : (cand == kCandLaneSeg4 || cand == kCandDeepSeg4) ? 4 : cand == kCandDeepSeg8 ? 8 : 1;
}
static bool cand_deep_knobs(int cand) { return cand == kCandDeepSeg4 || cand == kCandDeepSeg8; }

// AUTO times every applicable candidate kTuneRounds times and keeps each one's best time:
// round 1 in candidate order, round 2 in reverse, so that the clock ramp and cache warm-up of
// the first launches after an upload do not favour the candidates tried last (one trial each
// picked two- or four-segment items run to run on scene 6, 1-2.5 % apart)
constexpr int kTuneRounds = 2;

// The decision's one tie-break: the per-lane walk with two segments per item gives way to four
// when the four-segment trials are within kSegMargin of it (render lanes on).  The trials run in
// order, the settled schedule on the render lanes, where an item of four segments overlaps the
// previous launch's tail better: on the lanes four are 3.1 % (C2) and 3.4 % (C5) faster than two
// (profiles/r06_seg_ab.jsonl), while the in-order trials put the two within ~1-2 % of each other
// either way, so AUTO settled on two in some runs (the r06w bench: 14,585 against 14,814
// Msamples/s with four).
constexpr double kSegMargin = 0.02;
static int prefer_longer_items(const mcpt_ctx* c, int best, long long segs) {
  if (c->overlap && best == kCandLaneSeg2 && cand_applies(c, kCandLaneSeg4, segs) && c->tune_cnt[kCandLaneSeg4] > 0 &&
      c->tune_ns[kCandLaneSeg4] <= c->tune_ns[kCandLaneSeg2] * (1.0 + kSegMargin))
    return kCandLaneSeg4;
  return best;
}

// trials of candidate k issued so far on the measured shape (collected + pending)
static int tune_issued(const mcpt_ctx* c, int k) {
  int n = c->tune_cnt[k];
  for (int i = 0; i < c->n_pend; ++i) n += c->pend[i].cand == k ? 1 : 0;
  return n;
}

// schedule candidate of the next launch (`segs`: its pass segments)
static int resolve_candidate(const mcpt_ctx* c, long long segs) {
  if (c->traversal != MCPT_TRAVERSAL_AUTO) return c->traversal;
  if (c->tune_choice) return c->tune_choice;
  // next trial: in the current round (the fewest issued trials of any applicable candidate), the
  // first candidate of the round's order not yet tried that often on the measured shape
  int round = kTuneRounds;
  for (int k = 1; k <= kCandLast; ++k)
    if (cand_applies(c, k, segs)) round = std::min(round, tune_issued(c, k));
  if (round >= kTuneRounds) {   // every trial issued, the last ones not collected yet: the best so far
    int best = MCPT_TRAVERSAL_LANE;
    for (int k = 1; k <= kCandLast; ++k)
      if (cand_applies(c, k, segs) && c->tune_cnt[k] > 0 && (c->tune_cnt[best] == 0 || c->tune_ns[k] < c->tune_ns[best]))
        best = k;
    return prefer_longer_items(c, best, segs);
  }
  for (int i = 0; i < kCandLast; ++i) {
    const int k = (round % 2 == 0) ? 1 + i : kCandLast - i;
    if (cand_applies(c, k, segs) && tune_issued(c, k) == round) return k;
  }
  return MCPT_TRAVERSAL_LANE;
}
static int cand_traversal(int cand) { return cand >= kCandLaneSeg2 ? MCPT_TRAVERSAL_LANE : cand; }
static int resolve_traversal(const mcpt_ctx* c) { return cand_traversal(resolve_candidate(c, c->meas_segs)); }

static void reset_tuning(mcpt_ctx* c) {
  for (auto& L : c->lanes) L.order_valid = false;   // a new scene / target: item costs start over
  c->n_pend = 0;
  c->meas_shape[0] = c->meas_shape[1] = 0;
  c->meas_segs = 0;
  for (double& t : c->tune_ns) t = 0.0;
  for (int& n : c->tune_cnt) n = 0;
  c->tune_choice = 0;
}

// collect the timing of the oldest pending trial (waits for it) while more than `keep` are
// pending; decide once every applicable candidate is measured kTuneRounds times
static hipError_t collect_tuning(mcpt_ctx* c, int keep) {
  while (c->n_pend > keep) {
    const mcpt_ctx::TunePending t0 = c->pend[0];
    for (int i = 1; i < c->n_pend; ++i) c->pend[i - 1] = c->pend[i];
    c->n_pend--;
    float ms = 0.0f, ms_combine = 0.0f;
    hipError_t e = slot_launch_ms(c, t0.slot, &ms, &ms_combine);
    if (e != hipSuccess) return e;
    // per-sample times are compared only between launches of the same shape (pixels, passes):
    // a launch of another shape restarts the comparison
    if (t0.shape[0] != c->meas_shape[0] || t0.shape[1] != c->meas_shape[1]) {
      for (double& t : c->tune_ns) t = 0.0;
      for (int& n : c->tune_cnt) n = 0;
      c->meas_shape[0] = t0.shape[0];
      c->meas_shape[1] = t0.shape[1];
    }
    const double ns = (double)ms * 1e6 / t0.samples;
    const int k0 = t0.cand;
    c->tune_ns[k0] = (c->tune_cnt[k0] == 0) ? ns : std::min(c->tune_ns[k0], ns);
    c->tune_cnt[k0]++;
    const double* t = c->tune_ns;
    bool all = true;
    int best = MCPT_TRAVERSAL_LANE;
    for (int k = 1; k <= kCandLast; ++k) {
      if (!cand_applies(c, k, c->meas_segs)) continue;
      if (c->tune_cnt[k] < kTuneRounds) all = false;
      else if (t[k] < t[best]) best = k;
    }
    if (all) {
      c->tune_choice = prefer_longer_items(c, best, c->meas_segs);
      c->n_pend = 0;   // (trials of another shape still pending are dropped with the decision)
    }
  }
  return hipSuccess;
}
constexpr double kTuneMinSamples = 1 << 24;   // launches smaller than this are not timed

extern "C" {

const char* mcpt_error_string(int status) {
  if (status != MCPT_ERR_HIP && status != MCPT_OK && g_fresh && g_last_status == status) {
    g_fresh = false;
    const char* base = status == MCPT_ERR_INVALID_ARG ? "invalid argument"
                       : status == MCPT_ERR_NO_SCENE  ? "no scene uploaded"
                       : status == MCPT_ERR_NO_TARGET ? "no render target"
                       : status == MCPT_ERR_BAD_SCENE ? "malformed scene buffers"
                                                      : "error";
    std::snprintf(g_detail, sizeof(g_detail), "%s (%s)", base, g_last_error);
    return g_detail;
  }
  switch (status) {
    case MCPT_OK: return "ok";
    case MCPT_ERR_INVALID_ARG: return "invalid argument";
    case MCPT_ERR_NO_SCENE: return "no scene uploaded";
    case MCPT_ERR_NO_TARGET: return "no render target (call mcpt_set_target)";
    case MCPT_ERR_HIP: return g_last_error[0] ? g_last_error : "HIP runtime error";
    case MCPT_ERR_NOT_FINALIZED: return "scene not finalized";
    case MCPT_ERR_BAD_SCENE: return "malformed scene buffers";
    default: return "unknown status";
  }
}

int mcpt_version(void) { return 2; }

int mcpt_build_flags(void) {
  int f = 0;
#ifdef MCPT_CHECKED
  f |= MCPT_BUILD_CHECKED;
#endif
#ifdef MCPT_STAMPS
  f |= MCPT_BUILD_STAMPS;
#endif
#ifdef MCPT_LANESTATS
  f |= MCPT_BUILD_LANESTATS;
#endif
#ifdef MCPT_BLOCKTIMES
  f |= MCPT_BUILD_BLOCKTIMES;
#endif
#if MCPT_DRIVER_MATH   // (mcpt_math.h: 0 in the shipped build)
  f |= MCPT_BUILD_DRIVER_MATH;
#endif
  return f;
}

int mcpt_create(int device_ordinal, mcpt_ctx** out) {
  if (!out) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *out = nullptr;
  int n = 0;
  HIP_OR_RETURN(hipGetDeviceCount(&n));
  if (device_ordinal < 0 || device_ordinal >= n) return set_err(MCPT_ERR_INVALID_ARG, "device ordinal out of range");
  HIP_OR_RETURN(hipSetDevice(device_ordinal));
  mcpt_ctx* c = new (std::nothrow) mcpt_ctx();
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  c->leaf_batch = env_int("MCPT_LEAF_BATCH", -1);   // tuning hook (same results for any value)
  c->stream_slots = env_int("MCPT_STREAM_SLOTS", 0);
  c->stream_refill = env_int("MCPT_STREAM_REFILL", -1);
  c->device = device_ordinal;
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device_ordinal) != hipSuccess ||
      c->n_cu <= 0)
    c->n_cu = 256;
  // the context's own stream (combines, copies) at the device's greatest priority: with render
  // lanes its short kernels are dispatched ahead of the next render's waiting workgroups
  int prio_least = 0, prio_greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) prio_greatest = 0;
  hipError_t e = hipStreamCreateWithPriority(&c->own_stream, hipStreamNonBlocking, prio_greatest);
  for (auto& L : c->lanes) {
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L.freed, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&L.tail, hipEventDisableTiming);
  }
  // (recorded once, so that the first waits on them are satisfied)
  for (auto& L : c->lanes) {
    if (e == hipSuccess) e = hipEventRecord(L.freed, c->own_stream);
    if (e == hipSuccess) e = hipEventRecord(L.tail, L.stream);
  }
  c->overlap = env_int("MCPT_OVERLAP", 1);
  if (e == hipSuccess) e = ensure_events(c, 0, 1);
  if (const char* pb = std::getenv("MCPT_PARTIAL_BYTES")) c->partial_budget = (size_t)std::strtoull(pb, nullptr, 10);
#ifdef MCPT_BLOCKTIMES
  // diagnostic build: per-wave (start, end) clock pairs after the debug slots
  static_assert(mcpt::kBlockTimeBase == MCPT_DEBUG_SLOTS, "block times follow the debug slots");
  constexpr size_t kEventSlots = MCPT_DEBUG_SLOTS + mcpt::kBlockTimeSlots;
#else
  constexpr size_t kEventSlots = MCPT_DEBUG_SLOTS;
#endif
  if (e == hipSuccess) e = hipMalloc(&c->d_events, sizeof(unsigned long long) * kEventSlots);
  if (e == hipSuccess) e = hipMemset(c->d_events, 0, sizeof(unsigned long long) * kEventSlots);
  if (e != hipSuccess) { mcpt_destroy(c); return set_err(MCPT_ERR_HIP, "mcpt_create", e); }
  c->stream = c->own_stream;
  *out = c;
  return MCPT_OK;
}

static void free_meshes(mcpt_ctx* c) {
  (void)hipFree(c->d_minfo); (void)hipFree(c->d_mpairs);   // (d_mleaftris points into d_mpairs)
  (void)hipFree(c->d_mtris); (void)hipFree(c->d_mverts); (void)hipFree(c->d_mnorms);
  c->d_minfo = nullptr; c->d_mpairs = nullptr; c->d_mleaftris = nullptr;
  c->d_mtris = nullptr; c->d_mverts = nullptr; c->d_mnorms = nullptr;
  c->n_meshes = 0;
}

static void free_scene(mcpt_ctx* c) {
  (void)hipFree(c->d_nodes); (void)hipFree(c->d_leaves); (void)hipFree(c->d_ptype); (void)hipFree(c->d_prims);
  c->d_nodes = nullptr; c->d_leaves = nullptr; c->d_ptype = nullptr; c->d_prims = nullptr;
  c->has_scene = false;
}

int mcpt_destroy(mcpt_ctx* c) {
  if (!c) return MCPT_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_scene(c);
  free_meshes(c);
  (void)hipFree(c->d_accum);
  (void)hipFree(c->d_rows);
  (void)hipFree(c->d_events);
  for (auto& L : c->lanes) {
    if (L.stream) (void)hipStreamSynchronize(L.stream);
    (void)hipFree(L.d_partial);
    (void)hipFree(L.d_item_cost);
    (void)hipFree(L.d_cost_sorted);
    (void)hipFree(L.d_item_iota);
    (void)hipFree(L.d_item_perm);
    (void)hipFree(L.d_split_of);
    (void)hipFree(L.d_split_pass);
    (void)hipFree(L.d_steal);
    (void)hipFree(L.d_split_n);
    (void)hipFree(L.d_sort_tmp);
    if (L.freed) (void)hipEventDestroy(L.freed);
    if (L.tail) (void)hipEventDestroy(L.tail);
    if (L.stream) (void)hipStreamDestroy(L.stream);
  }
  (void)hipFree(c->d_slots);
  (void)hipFree(c->d_queue);
  (void)hipFree(c->d_sctr);
  if (c->h_sctr) (void)hipHostFree(c->h_sctr);
  for (hipEvent_t e : c->batch_ev) if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->pool_ev) if (e) (void)hipEventDestroy(e);
  for (hipStream_t st : c->pool_stream) if (st) (void)hipStreamDestroy(st);
  for (const std::vector<hipEvent_t>& v : c->evs)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return MCPT_OK;
}

int mcpt_upload_scene(mcpt_ctx* c, const float* prims, int n_prims, const float* nodes, const int* leaves,
                      int depth, int nb_emissives) {
  // n_prims < 2^24: the kernel packs a hit's primitive index, shape and face in one word
  if (!c || !prims || !nodes || !leaves || n_prims <= 0 || n_prims >= (1 << 24) || depth < 0 || depth > 24)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_upload_scene: bad arguments");
  const int n_leaf = 1 << depth, n_node = 2 * n_leaf - 1;
  for (int i = 0; i < n_leaf; ++i)
    if (leaves[i] < -1 || leaves[i] >= n_prims) return set_err(MCPT_ERR_BAD_SCENE, "leaf id out of range");
  // subtree-holds-a-primitive flags (bottom-up over the implicit heap): empty subtrees
  // are never visited by the kernel (they cannot change the closest hit)
  std::vector<char> has(n_node, 0);
  for (int i = n_node - 1; i >= 0; --i)
    has[i] = (i >= n_leaf - 1) ? (leaves[i - (n_leaf - 1)] >= 0) : (has[2 * i + 1] || has[2 * i + 2]);
  // nodes → (centre, has-prim flag) (half-width, 0) (1/half-width, 0): raytracer_func.frag:319-320
  // hoisted to upload
  std::vector<float4> hn((size_t)n_node * mcpt::kNodeF4);
  for (int i = 0; i < n_node; ++i) {
    const float* b = nodes + (size_t)i * 6;
    float cx = (b[0] + b[3]) / 2.0f, cy = (b[1] + b[4]) / 2.0f, cz = (b[2] + b[5]) / 2.0f;
    float wx = 0.5f * (b[3] - b[0]), wy = 0.5f * (b[4] - b[1]), wz = 0.5f * (b[5] - b[2]);
    hn[(size_t)i * 3 + 0] = make_float4(cx, cy, cz, has[i] ? 1.0f : 0.0f);
    hn[(size_t)i * 3 + 1] = make_float4(wx, wy, wz, 0.0f);
    hn[(size_t)i * 3 + 2] = make_float4(1.0f / wx, 1.0f / wy, 1.0f / wz, 0.0f);
  }
  // prims → rows of the inverse and of the transform (the shader uses .xyz of mat4·v).  A
  // CODE_MESH record's transform rows are its mesh transform (texel 8-11, read_mesh_transfo:
  // the only transform Mesh_intersect / mesh_inter_geom_info use); its mesh id (texel 12 .y,
  // "mesh_line") goes into ptype's high bits.
  std::vector<int> ht(n_prims), mesh_ids(n_prims, -1);
  std::vector<float4> hp((size_t)n_prims * mcpt::kPrimF4);
  for (int i = 0; i < n_prims; ++i) {
    const float* r = prims + (size_t)i * 64;
    float tcode = r[48];
    if (!(tcode >= 0.0f && tcode <= 5.0f) || tcode != (float)(int)tcode)
      return set_err(MCPT_ERR_BAD_SCENE, "primitive type code not in 0..5");
    ht[i] = (int)tcode;
    const float* trf = r;
    if (ht[i] == 0) {
      const float ml = r[49];
      if (!(ml >= 0.0f && ml < (float)(1 << 26)) || ml != (float)(int)ml)
        return set_err(MCPT_ERR_BAD_SCENE, "mesh primitive without a valid mesh id");
      mesh_ids[i] = (int)ml;
      ht[i] |= mesh_ids[i] << 4;
      trf = r + 32;
    }
    float4* o = &hp[(size_t)i * mcpt::kPrimF4];
    for (int row = 0; row < 3; ++row) {
      const float* inv = r + 16;
      o[row] = make_float4(inv[row], inv[4 + row], inv[8 + row], inv[12 + row]);
      o[3 + row] = make_float4(trf[row], trf[4 + row], trf[8 + row], trf[12 + row]);
    }
    o[6] = make_float4(r[52], r[53], r[54], r[55]);
    o[7] = make_float4(r[56], r[57], r[58], r[59]);
  }
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  free_scene(c);
  HIP_OR_RETURN(hipMalloc(&c->d_nodes, hn.size() * sizeof(float4)));
  HIP_OR_RETURN(hipMalloc(&c->d_leaves, (size_t)n_leaf * sizeof(int)));
  HIP_OR_RETURN(hipMalloc(&c->d_ptype, (size_t)n_prims * sizeof(int)));
  HIP_OR_RETURN(hipMalloc(&c->d_prims, hp.size() * sizeof(float4)));
  HIP_OR_RETURN(hipMemcpy(c->d_nodes, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_leaves, leaves, (size_t)n_leaf * sizeof(int), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_ptype, ht.data(), (size_t)n_prims * sizeof(int), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_prims, hp.data(), hp.size() * sizeof(float4), hipMemcpyHostToDevice));
  c->n_prims = n_prims; c->depth = depth; c->nb_emissive = nb_emissives;
  c->mesh_ids = mesh_ids;
  free_meshes(c);                 // a new scene drops the previous meshes (upload them again)
  c->has_scene = true;
  reset_tuning(c);
  return MCPT_OK;
}

// nodes (bbmin, bbmax) → device node records with the subtree-holds-an-item flag
static void pack_nodes(const float* nodes, const int* leaves, int depth, float4* out) {
  const int n_leaf = 1 << depth, n_node = 2 * n_leaf - 1;
  std::vector<char> has(n_node, 0);
  for (int i = n_node - 1; i >= 0; --i)
    has[i] = (i >= n_leaf - 1) ? (leaves[i - (n_leaf - 1)] >= 0) : (has[2 * i + 1] || has[2 * i + 2]);
  for (int i = 0; i < n_node; ++i) {
    const float* b = nodes + (size_t)i * 6;
    float cx = (b[0] + b[3]) / 2.0f, cy = (b[1] + b[4]) / 2.0f, cz = (b[2] + b[5]) / 2.0f;
    float wx = 0.5f * (b[3] - b[0]), wy = 0.5f * (b[4] - b[1]), wz = 0.5f * (b[5] - b[2]);
    out[(size_t)i * 3 + 0] = make_float4(cx, cy, cz, has[i] ? 1.0f : 0.0f);
    out[(size_t)i * 3 + 1] = make_float4(wx, wy, wz, 0.0f);
    out[(size_t)i * 3 + 2] = make_float4(1.0f / wx, 1.0f / wy, 1.0f / wz, 0.0f);
  }
}

static float int_bits_f(int v) {
  float f;
  std::memcpy(&f, &v, sizeof f);
  return f;
}

// A mesh BVH's child-pair records: internal node i -> 4 rows (the device's one 64-byte fetch per
// visit): (c_left, has_left) (w_left, 0) (c_right, has_right) (w_right, 0), c and w computed as
// pack_nodes does; 1/w is recomputed on the device (rcp_rn, correctly rounded: the bits of the
// host's 1/w)
static void pack_mesh_pairs(const float* nodes, const int* leaves, int depth, float4* out) {
  const int n_leaf = 1 << depth, n_node = 2 * n_leaf - 1;
  std::vector<float4> rec((size_t)n_node * 3);
  pack_nodes(nodes, leaves, depth, rec.data());
  for (int i = 0; i + 1 < n_leaf; ++i) {   // internal nodes 0 .. n_leaf - 2
    const float4* l = &rec[(size_t)(2 * i + 1) * 3];
    const float4* r = &rec[(size_t)(2 * i + 2) * 3];
    float4* o = out + (size_t)mcpt::mesh_pair_slot((unsigned)i) * 4;
    // row 1's w: 1 when all six half-widths lie in rcp_core's exact range (rcp6_rn then skips
    // its six range tests), else 0
    bool in_range = true;
    for (float v : {l[1].x, l[1].y, l[1].z, r[1].x, r[1].y, r[1].z}) {
      const float a = std::fabs(v);
      in_range = in_range && a >= 0x1p-126f && a < 0x1p126f;
    }
    o[0] = l[0];
    o[1] = make_float4(l[1].x, l[1].y, l[1].z, in_range ? 1.0f : 0.0f);
    o[2] = r[0];
    o[3] = make_float4(r[1].x, r[1].y, r[1].z, 0.0f);
  }
}

int mcpt_upload_meshes(mcpt_ctx* c, int n_meshes, const int* info, int n_nodes, const float* nodes, int n_leaves,
                       const int* leaves, int n_tris, const int* tris, int n_verts, const float* verts,
                       const float* normals) {
  if (!c || n_meshes < 0) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_upload_meshes: bad arguments");
  if (!c->has_scene) return set_err(MCPT_ERR_NO_SCENE, "upload the scene before its meshes");
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  free_meshes(c);
  if (n_meshes == 0) {
    for (int id : c->mesh_ids)
      if (id >= 0) return set_err(MCPT_ERR_BAD_SCENE, "the scene has mesh instances but no meshes were uploaded");
    return MCPT_OK;
  }
  if (!info || !nodes || !leaves || !tris || !verts || !normals || n_nodes <= 0 || n_leaves <= 0 || n_tris <= 0 ||
      n_verts <= 0)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_upload_meshes: bad arguments");
  // validate the layout: each mesh's BVH within the node / leaf arrays, leaf triangle ids
  // within the mesh's triangles, vertex ids within the vertex array
  // pair records: each mesh's in its own run of slots (mesh_pair_slot), the run starting at an
  // even slot so that two-slot lines are 128-byte aligned; leaf triangle records indexed by the
  // global leaf index
  std::vector<unsigned> pair_base(n_meshes);
  size_t n_slots = 0;
  for (int m = 0; m < n_meshes; ++m) {
    const int d = info[4 * m + 2];
    if (d < 0 || d > 24) return set_err(MCPT_ERR_BAD_SCENE, "bad mesh info");
    pair_base[m] = (unsigned)n_slots;
    n_slots = (n_slots + mcpt::mesh_pair_slots(d) + 1) & ~(size_t)1;
  }
  if (n_slots * 4 >= (size_t(1) << 31)) return set_err(MCPT_ERR_BAD_SCENE, "mesh BVHs too large");
  std::vector<float4> hn(std::max<size_t>(n_slots, 2) * 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  for (int m = 0; m < n_meshes; ++m) {
    const int no = info[4 * m], lo = info[4 * m + 1], d = info[4 * m + 2], to = info[4 * m + 3];
    if (d < 0 || d > 24 || no < 0 || lo < 0 || to < 0) return set_err(MCPT_ERR_BAD_SCENE, "bad mesh info");
    const int nl = 1 << d, nn = 2 * nl - 1;
    if (no + nn > n_nodes || lo + nl > n_leaves) return set_err(MCPT_ERR_BAD_SCENE, "mesh BVH out of range");
    const int nt = (m + 1 < n_meshes ? info[4 * (m + 1) + 3] : n_tris) - to;
    if (nt <= 0 || to + nt > n_tris) return set_err(MCPT_ERR_BAD_SCENE, "mesh triangles out of range");
    for (int k = 0; k < nl; ++k)
      if (leaves[lo + k] < -1 || leaves[lo + k] >= nt) return set_err(MCPT_ERR_BAD_SCENE, "mesh leaf id out of range");
    pack_mesh_pairs(nodes + (size_t)no * 6, leaves + lo, d, &hn[(size_t)pair_base[m] * 4]);
  }
  for (int id : c->mesh_ids)
    if (id >= n_meshes) return set_err(MCPT_ERR_BAD_SCENE, "mesh instance refers to a missing mesh");
  std::vector<int4> hi(n_meshes), ht(n_tris);
  // device mesh info: (first pair slot, first leaf, depth, first triangle)
  for (int m = 0; m < n_meshes; ++m) hi[m] = make_int4((int)pair_base[m], info[4 * m + 1], info[4 * m + 2], info[4 * m + 3]);
  for (int t = 0; t < n_tris; ++t) {
    const int* v = tris + (size_t)t * 3;
    for (int k = 0; k < 3; ++k)
      if (v[k] < 0 || v[k] >= n_verts) return set_err(MCPT_ERR_BAD_SCENE, "vertex id out of range");
    ht[t] = make_int4(v[0], v[1], v[2], 0);
  }
  std::vector<float4> hv(n_verts), hm(n_verts);
  for (int i = 0; i < n_verts; ++i) {
    hv[i] = make_float4(verts[3 * i], verts[3 * i + 1], verts[3 * i + 2], 0.0f);
    hm[i] = make_float4(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2], 0.0f);
  }
  // leaf triangle records (one 64-byte fetch per leaf visit, no index -> vertex indirection):
  // (A, t) (B - A, 0) (C - A, 0) (0): Triangle_intersect's vertex A and its two edges, computed
  // with the binary32 subtractions the device did (same bits), and the mesh-local triangle id t
  // (-1: an empty leaf) as int bits
  std::vector<float4> hl((size_t)n_leaves * 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
  for (int k = 0; k < n_leaves; ++k) hl[(size_t)k * 4].w = int_bits_f(-1);
  for (int m = 0; m < n_meshes; ++m) {
    const int lo = info[4 * m + 1], d = info[4 * m + 2], to = info[4 * m + 3];
    for (int k = 0; k < (1 << d); ++k) {
      const int t = leaves[lo + k];
      if (t < 0) continue;
      const int4 vi = ht[to + t];
      const float4 A = hv[vi.x], B = hv[vi.y], C = hv[vi.z];
      float4* r = &hl[(size_t)(lo + k) * 4];
      r[0] = make_float4(A.x, A.y, A.z, int_bits_f(t));
      r[1] = make_float4(B.x - A.x, B.y - A.y, B.z - A.z, 0.0f);
      r[2] = make_float4(C.x - A.x, C.y - A.y, C.z - A.z, 0.0f);
    }
  }
  HIP_OR_RETURN(hipMalloc(&c->d_minfo, hi.size() * sizeof(int4)));
  // one allocation: the pair slots, then the leaf records (walk_run_mesh addresses both by 32-bit
  // byte offsets from d_mpairs)
  if ((hn.size() + hl.size()) * sizeof(float4) > (size_t(1) << 32))
    return set_err(MCPT_ERR_BAD_SCENE, "mesh BVH records exceed 4 GiB");
  HIP_OR_RETURN(hipMalloc(&c->d_mpairs, (hn.size() + hl.size()) * sizeof(float4)));
  c->d_mleaftris = c->d_mpairs + hn.size();
  HIP_OR_RETURN(hipMalloc(&c->d_mtris, ht.size() * sizeof(int4)));
  HIP_OR_RETURN(hipMalloc(&c->d_mverts, hv.size() * sizeof(float4)));
  HIP_OR_RETURN(hipMalloc(&c->d_mnorms, hm.size() * sizeof(float4)));
  HIP_OR_RETURN(hipMemcpy(c->d_minfo, hi.data(), hi.size() * sizeof(int4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_mpairs, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_mleaftris, hl.data(), hl.size() * sizeof(float4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_mtris, ht.data(), ht.size() * sizeof(int4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_mverts, hv.data(), hv.size() * sizeof(float4), hipMemcpyHostToDevice));
  HIP_OR_RETURN(hipMemcpy(c->d_mnorms, hm.data(), hm.size() * sizeof(float4), hipMemcpyHostToDevice));
  c->n_meshes = n_meshes;
  return MCPT_OK;
}

int mcpt_set_flat_face(mcpt_ctx* c, int flat_face) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  c->flat_face = flat_face ? 1 : 0;
  return MCPT_OK;
}

// Shard the frame by explicit row lists: `rows` = the global rows this context renders, in
// local-row order.  mcpt_set_target (interleaved bands) and mcpt_balanced_rows are row lists.
static int set_target_rows(mcpt_ctx* c, int W, int H, const int* rows, int n_rows, int band_rows, int world,
                           int rank) {
  // the kernels index a shard's pixels with 32-bit ints (render_kernel's local pixel index)
  if ((long long)n_rows * W >= (1LL << 31))
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_target: a shard of 2^31 pixels or more");
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  size_t bytes = (size_t)n_rows * W * 3 * sizeof(float);
  if (bytes != c->accum_bytes) {
    (void)hipFree(c->d_accum);
    c->d_accum = nullptr;
    c->accum_bytes = 0;
    if (bytes) HIP_OR_RETURN(hipMalloc(&c->d_accum, bytes));
    c->accum_bytes = bytes;
  }
  if ((size_t)n_rows != c->rows.size() || !c->d_rows) {
    (void)hipFree(c->d_rows);
    c->d_rows = nullptr;
    HIP_OR_RETURN(hipMalloc(&c->d_rows, sizeof(int) * (size_t)std::max(n_rows, 1)));
  }
  c->rows.assign(rows, rows + n_rows);
  if (n_rows) HIP_OR_RETURN(hipMemcpy(c->d_rows, rows, sizeof(int) * (size_t)n_rows, hipMemcpyHostToDevice));
  c->W = W; c->H = H; c->band_rows = band_rows; c->world = world; c->rank = rank; c->n_local_rows = n_rows;
  c->has_target = true;
  for (auto& L : c->lanes) L.order_valid = false;   // other pixels: the item costs start over
  return mcpt_clear_accum(c);
}

int mcpt_set_target(mcpt_ctx* c, int W, int H, int band_rows, int world, int rank) {
  if (!c || W <= 0 || H <= 0 || band_rows <= 0 || world <= 0 || rank < 0 || rank >= world)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_target: bad arguments");
  std::vector<int> rows;
  for (int y = 0; y < H; ++y)
    if ((y / band_rows) % world == rank) rows.push_back(y);
  return set_target_rows(c, W, H, rows.data(), (int)rows.size(), band_rows, world, rank);
}

int mcpt_set_target_rows(mcpt_ctx* c, int W, int H, const int* rows, int n_rows) {
  if (!c || W <= 0 || H <= 0 || n_rows < 0 || n_rows > H || (n_rows > 0 && !rows))
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_target_rows: bad arguments");
  std::vector<char> seen((size_t)H, 0);
  for (int i = 0; i < n_rows; ++i) {
    if (rows[i] < 0 || rows[i] >= H || seen[(size_t)rows[i]])
      return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_target_rows: rows must be distinct and in [0, H)");
    seen[(size_t)rows[i]] = 1;
  }
  return set_target_rows(c, W, H, rows, n_rows, 0, 0, 0);
}

int mcpt_balanced_rows(int H, int world, int rank, int band_rows, int* rows_out, int* n_out) {
  if (H <= 0 || world <= 0 || rank < 0 || rank >= world || band_rows <= 0 || !n_out)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_balanced_rows: bad arguments");
  // whole periods of `world` bands: in period j, rank r takes band j·world + (r + j) mod world
  // (each rank gets every band position of a period equally often); the rows after the last
  // whole period are dealt one at a time, rotated the same way
  const int periods = (H / band_rows) / world;
  const int rest0 = periods * world * band_rows;
  int n = 0;
  for (int y = 0; y < H; ++y) {
    int owner;
    if (y < rest0) {
      const int b = y / band_rows, j = b / world;
      owner = ((b % world) - j % world + world) % world;
    } else {
      owner = ((y - rest0) + periods) % world;
    }
    if (owner == rank) {
      if (rows_out) rows_out[n] = y;
      ++n;
    }
  }
  *n_out = n;
  return MCPT_OK;
}

int mcpt_local_row_ids(mcpt_ctx* c, int* rows_out) {
  if (!c || !rows_out) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  std::copy(c->rows.begin(), c->rows.end(), rows_out);
  return MCPT_OK;
}

int mcpt_local_rows(mcpt_ctx* c, int* n) {
  if (!c || !n) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  *n = c->n_local_rows;
  return MCPT_OK;
}

int mcpt_clear_accum(mcpt_ctx* c) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  HIP_OR_RETURN(hipSetDevice(c->device));
  if (c->accum_bytes) HIP_OR_RETURN(hipMemsetAsync(c->d_accum, 0, c->accum_bytes, c->stream));
  c->pass_count = 0;
  return MCPT_OK;
}

// raytracer.vert:9-22 for the 4 strip corners: Ori = invV·(0,0,0,1), Dir = normalize(Q.xyz/Q.w − Ori)
static void corner_rays(const float* invPV, const float* invV, mcpt::RenderParams& p) {
  auto matvec = [](const float* m, const float v[4], float o[4]) {
    for (int r = 0; r < 4; ++r)
      o[r] = std::fma(m[12 + r], v[3], std::fma(m[8 + r], v[2], std::fma(m[4 + r], v[1], m[r] * v[0])));
  };
  const float origin[4] = {0.0f, 0.0f, 0.0f, 1.0f};
  float o4[4];
  matvec(invV, origin, o4);
  p.ox = o4[0]; p.oy = o4[1]; p.oz = o4[2];
  for (int v = 0; v < 4; ++v) {
    float tcx = (float)(v % 2), tcy = (float)(v / 2);
    float cv[4] = {2.0f * tcx - 1.0f, 2.0f * tcy - 1.0f, 1.0f, 1.0f};
    float q[4];
    matvec(invPV, cv, q);
    float dx = q[0] / q[3] - o4[0], dy = q[1] / q[3] - o4[1], dz = q[2] / q[3] - o4[2];
    float len2 = std::fma(dz, dz, std::fma(dy, dy, dx * dx));
    float rn = 1.0f / std::sqrt(len2);
    p.cd[3 * v + 0] = dx * rn; p.cd[3 * v + 1] = dy * rn; p.cd[3 * v + 2] = dz * rn;
  }
}

// stream schedule defaults: 16 Mi path slots (2 x 92 B of queue payload + 64 B of unit data
// each: 4 GB) keep the iterations few and every trace kernel long against its tail (the last
// walks of the iteration): scene 8, 512 spp, 1080p (33 M units): 4 Mi slots 1,344 iterations
// 447 Msamples/s, 8 Mi 792 / 472, 12 Mi 624 / 482, 16 Mi 512 / 484, 32 Mi 352 / 478 (the
// units' own tail grows); a wave refills its idle lanes once 8 of them have finished their walks
constexpr int kStreamSlotsDefault = 1 << 24;
constexpr int kStreamRefillDefault = 56;
constexpr int kStreamBatch = 8;   // iterations issued between two reads of the counters
// the shade kernel compacts its output (drops dead entries) once fewer than this share of the
// queue is live
constexpr double kStreamCompactBelow = 0.6;

static bool stream_applies(const mcpt_ctx* c, int variant, int bounces, bool count) {
  (void)c;
  return !count && variant == 0 && bounces > 0;
}

// path-slot pools of a launch: each runs its own iterations on its own stream, so one pool's
// shade kernel and trace-kernel tail overlap the other pool's trace kernel
constexpr int kStreamPools = 2;

// One sub-launch (one pass range of <= max_seg segments) with the stream schedule: the slots of
// every pool set up, then iterations (trace + shade) in batches until every slot has run out of
// units.  The host reads the counters of batch b-1 while batch b runs, so the device never waits
// for the host.
static int stream_run(mcpt_ctx* c, const mcpt::RenderParams& p) {
  const unsigned long long n_units = (unsigned long long)p.n_local_px * (unsigned long long)p.n_segments;
  if (n_units == 0) return MCPT_OK;
  if (n_units >= (1ULL << 31) || p.n_local_px >= (1LL << 31))
    return set_err(MCPT_ERR_INVALID_ARG, "stream schedule: too many units in one launch");
  // the kernels address a pool's queue / slot data through one buffer resource: below 2 GiB each
  const int max_pool = (int)(((1ULL << 31) - 1) / (mcpt::QF_COUNT * sizeof(float)));
  const int n_pools = (int)std::max(1, std::min(env_int("MCPT_STREAM_POOLS", kStreamPools), kStreamPools));
  const long long want = c->stream_slots > 0 ? c->stream_slots : kStreamSlotsDefault;
  const long long n_slots = std::min<long long>((long long)n_units, std::min<long long>(want, (long long)max_pool * n_pools));
  int pool_n[kStreamPools] = {0, 0};
  int np = 0;
  for (int k = 0; k < n_pools; ++k) {
    pool_n[k] = (int)(n_slots / n_pools + (k < n_slots % n_pools ? 1 : 0));
    if (pool_n[k] > 0) np = k + 1;
  }
  if (n_slots > c->slot_cap) {
    HIP_OR_RETURN(hipStreamSynchronize(c->stream));
    (void)hipFree(c->d_slots); (void)hipFree(c->d_queue);
    c->d_slots = nullptr; c->d_queue = nullptr; c->slot_cap = 0;
    HIP_OR_RETURN(hipMalloc(&c->d_slots, (size_t)mcpt::SF_COUNT * n_slots * sizeof(float)));
    HIP_OR_RETURN(hipMalloc(&c->d_queue, (size_t)2 * mcpt::QF_COUNT * n_slots * sizeof(float)));
    c->slot_cap = n_slots;
  }
  if (!c->d_sctr) HIP_OR_RETURN(hipMalloc(&c->d_sctr, kStreamPools * mcpt::SC_COUNT * sizeof(unsigned)));
  if (!c->h_sctr)
    HIP_OR_RETURN(hipHostMalloc(&c->h_sctr, 2 * kStreamPools * mcpt::SC_COUNT * sizeof(unsigned), hipHostMallocDefault));
  for (hipEvent_t& e : c->batch_ev)
    if (!e) HIP_OR_RETURN(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t& e : c->pool_ev)
    if (!e) HIP_OR_RETURN(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipStream_t& st : c->pool_stream)
    if (!st) HIP_OR_RETURN(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // BVH nodes in the trace kernel's LDS where they fit (MCPT_STREAM_LDS_NODES=1): off by default,
  // no faster on scenes 3/7/8 (random lanes' node reads conflict in the LDS banks, 11 conflict
  // cycles per LDS instruction; gpurun_out r03e/r03f)
  const bool lds_nodes = env_int("MCPT_STREAM_LDS_NODES", 0) != 0 && p.n_meshes == 0 && mcpt_stream_lds_nodes_fit(p.depth);
  mcpt::StreamParams q[kStreamPools];
  unsigned* unit_ctr = c->d_sctr + mcpt::SC_UNIT;   // pool 0's slot: shared
  {
    const unsigned first_free = (unsigned)n_slots;   // units 0 .. n_slots-1 start in the pools' slots
    HIP_OR_RETURN(hipMemcpyAsync(unit_ctr, &first_free, sizeof(unsigned), hipMemcpyHostToDevice, c->stream));
  }
  size_t slot_off = 0, queue_off = 0;
  int unit_base = 0;
  for (int k = 0; k < np; ++k) {
    mcpt::StreamParams& s = q[k];
    s.r = p;
    // leaf batching of the trace kernel's walks: 16 lanes (8 for the megakernel; scene 8: 16 is
    // +4 % over 8 and 32, 4 is -8 %)
    if (c->leaf_batch < 0) s.r.leaf_batch = 16;
    // field f of pool entry i at queue[par][f * n + i], slot data likewise: laid out per pool
    s.slots = c->d_slots + slot_off;
    s.queue[0] = c->d_queue + queue_off;
    s.queue[1] = s.queue[0] + (size_t)mcpt::QF_COUNT * pool_n[k];
    s.ctr = c->d_sctr + k * mcpt::SC_COUNT;
    s.unit_ctr = unit_ctr;
    s.n_slots = pool_n[k];
    s.unit_base = unit_base;
    s.n_units = (unsigned)n_units;
    s.parity = 0;
    s.refill = c->stream_refill >= 0 ? c->stream_refill : kStreamRefillDefault;
    s.compact = 0;
    slot_off += (size_t)mcpt::SF_COUNT * pool_n[k];
    queue_off += (size_t)2 * mcpt::QF_COUNT * pool_n[k];
    unit_base += pool_n[k];
    HIP_OR_RETURN(mcpt_launch_stream_init(s, c->stream));
  }
  // fork: the pool streams start after the set-up (and everything before it) on the context's stream
  HIP_OR_RETURN(hipEventRecord(c->pool_ev[2], c->stream));
  for (int k = 0; k < np; ++k) HIP_OR_RETURN(hipStreamWaitEvent(c->pool_stream[k], c->pool_ev[2], 0));
  // every iteration advances each live slot by one traversal; a unit needs at most
  // (passes) x (2 B + 1) + 1 of them, and a slot runs ceil(units / slots) units
  const long long per_unit = (long long)mcpt::kPassChunk * (2LL * p.bounces + 1) + 1;
  const long long min_pool = pool_n[np - 1];
  const long long cap = ((long long)(n_units / min_pool) + 2) * per_unit + 4 * kStreamBatch;
  long long it = 0;
  bool compact[kStreamPools] = {false, false}, done[kStreamPools] = {false, false};
  const int st = [&]() -> int {
  for (int b = 0;; ++b) {
    for (int k = 0; k < kStreamBatch; ++k, ++it)
      for (int j = 0; j < np; ++j) {
        if (done[j]) continue;
        q[j].parity = (int)(it & 1);
        q[j].compact = (k == 0 && compact[j]) ? 1 : 0;
        HIP_OR_RETURN(mcpt_launch_stream_iter(q[j], c->n_cu, lds_nodes, c->pool_stream[j]));
      }
    // every pool's counters after the batch, read on pool 0's stream once all pools are there
    for (int j = 1; j < np; ++j) {
      HIP_OR_RETURN(hipEventRecord(c->pool_ev[j], c->pool_stream[j]));
      HIP_OR_RETURN(hipStreamWaitEvent(c->pool_stream[0], c->pool_ev[j], 0));
    }
    unsigned* h = c->h_sctr + (b & 1) * kStreamPools * mcpt::SC_COUNT;
    HIP_OR_RETURN(hipMemcpyAsync(h, c->d_sctr, (size_t)np * mcpt::SC_COUNT * sizeof(unsigned), hipMemcpyDeviceToHost,
                                 c->pool_stream[0]));
    HIP_OR_RETURN(hipEventRecord(c->batch_ev[b & 1], c->pool_stream[0]));
    if (b >= 1) {
      HIP_OR_RETURN(hipEventSynchronize(c->batch_ev[(b - 1) & 1]));
      bool all = true;
      for (int j = 0; j < np; ++j) {
        const unsigned* hp = c->h_sctr + ((b - 1) & 1) * kStreamPools * mcpt::SC_COUNT + j * mcpt::SC_COUNT;
        const unsigned dead = hp[mcpt::SC_DEAD];
        done[j] = dead >= (unsigned)pool_n[j];   // every slot of the pool was done by the end of batch b-1
        all = all && done[j];
        // the queue length the iteration after batch b-1 read (in place: unchanged until compacted)
        const unsigned len = hp[mcpt::SC_CNT + (int)((it - kStreamBatch) & 1)];
        compact[j] = !done[j] && (double)(pool_n[j] - dead) < kStreamCompactBelow * (double)len;
      }
      if (all) break;
    }
    if (it > cap) return set_err(MCPT_ERR_HIP, "stream schedule did not drain its queue");
  }
  return MCPT_OK;
  }();
  // join: the context's stream (the combine kernel, the caller's next work) waits for every
  // pool stream.  Also after an error: kernels already queued on a pool stream still read and
  // write d_slots / d_queue / d_partial, which the context frees or reallocates only after
  // synchronizing its own stream, so that stream must not run ahead of them.
  bool joined = true;
  for (int j = 0; j < np; ++j)
    joined = joined && hipEventRecord(c->pool_ev[j], c->pool_stream[j]) == hipSuccess &&
             hipStreamWaitEvent(c->stream, c->pool_ev[j], 0) == hipSuccess;
  if (!joined)   // cannot order them: wait for them here
    for (int j = 0; j < np; ++j) (void)hipStreamSynchronize(c->pool_stream[j]);
  if (st != MCPT_OK) return st;
  if (!joined) return set_err(MCPT_ERR_HIP, "stream schedule: joining the pool streams failed");
  c->stream_iters += it;
  return MCPT_OK;
}

// the stream schedule's pools (4 GB at the default 16 Mi slots), once no longer selected
static int free_stream_pools(mcpt_ctx* c) {
  if (!c->d_slots && !c->d_queue) return MCPT_OK;
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  (void)hipFree(c->d_slots); (void)hipFree(c->d_queue);
  c->d_slots = nullptr; c->d_queue = nullptr; c->slot_cap = 0;
  return MCPT_OK;
}

// Buffers of the work-item order for `items` items (grown on demand, with the identity values
// the sort permutes and its temporary storage)
static hipError_t ensure_item_order(mcpt_ctx* c, mcpt_ctx::Lane& L, long long items) {
  if (items <= L.item_cap) return hipSuccess;
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(L.stream);
  if (e != hipSuccess) return e;
  (void)hipFree(L.d_item_cost); (void)hipFree(L.d_cost_sorted); (void)hipFree(L.d_item_iota);
  (void)hipFree(L.d_item_perm); (void)hipFree(L.d_sort_tmp); (void)hipFree(L.d_split_of);
  L.d_item_cost = L.d_cost_sorted = nullptr; L.d_item_iota = L.d_item_perm = nullptr; L.d_sort_tmp = nullptr;
  L.d_split_of = nullptr;
  L.item_cap = 0; L.sort_tmp_bytes = 0; L.order_valid = false;
  const size_t n = (size_t)items;
  size_t tmp = 0;
  if ((e = hipMalloc(&L.d_item_cost, sizeof(unsigned) * n)) != hipSuccess) return e;
  if ((e = hipMalloc(&L.d_cost_sorted, sizeof(unsigned) * n)) != hipSuccess) return e;
  if ((e = hipMalloc(&L.d_item_iota, sizeof(int) * n)) != hipSuccess) return e;
  if ((e = hipMalloc(&L.d_item_perm, sizeof(int) * n)) != hipSuccess) return e;
  if ((e = hipMalloc(&L.d_split_of, sizeof(int) * n)) != hipSuccess) return e;
  if (!L.d_split_n && (e = hipMalloc(&L.d_split_n, sizeof(int))) != hipSuccess) return e;
  if ((e = hipMemset(L.d_split_n, 0, sizeof(int))) != hipSuccess) return e;
  if ((e = mcpt_order_items(nullptr, nullptr, nullptr, nullptr, (int)items, nullptr, &tmp, c->stream)) != hipSuccess)
    return e;
  if ((e = hipMalloc(&L.d_sort_tmp, std::max<size_t>(tmp, 1))) != hipSuccess) return e;
  if ((e = mcpt_iota(L.d_item_iota, (int)items, c->stream)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return e;
  L.sort_tmp_bytes = tmp;
  L.item_cap = items;
  return hipSuccess;
}

#ifdef MCPT_CHECKED
// checked build (mcpt_internal.h, kCheckedCountSlot): wait for sub-launch k of n_sub and report a
// HIP fault or an out-of-range index the kernels counted, naming the sub-launch and its shape
static int checked_sub_launch(mcpt_ctx* c, int k, int n_sub, const mcpt::RenderParams& p) {
  char what[200];
  std::snprintf(what, sizeof(what),
                "checked build: sub-launch %d of %d (passes %d+%d, %d segments, %d items, K %d, tail %d, split max %d)",
                k, n_sub, p.first_pass, p.n_passes, p.n_segments, p.n_items, p.seg_per_item, p.tail_m, p.split_max);
  hipError_t e = hipStreamSynchronize(c->stream);   // (ordered after the sub-launch's lane work)
  if (e != hipSuccess) return set_err(MCPT_ERR_HIP, what, e);
  unsigned long long v[2] = {0, 0};
  e = hipMemcpy(v, c->d_events + mcpt::kCheckedCountSlot, sizeof(v), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return set_err(MCPT_ERR_HIP, what, e);
  if (v[0] != 0) {
    char msg[256];
    std::snprintf(msg, sizeof(msg), "%s: %llu out-of-range indices, first at site %llu index %lld", what, v[0],
                  v[1] >> 48, (long long)(v[1] & 0xffffffffffffull));
    (void)hipMemset(c->d_events + mcpt::kCheckedCountSlot, 0, sizeof(v));
    return set_err(MCPT_ERR_HIP, msg);
  }
  return MCPT_OK;
}
#endif

static int launch(mcpt_ctx* c, const float* invPV, const float* invV, int first_pass, int n_passes, float date,
                  int bounces, float refract_ind, int variant, bool count, unsigned long long* events) {
  if (!c || !invPV || !invV || n_passes < 0 || variant < 0 || variant > 2)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_render: bad arguments");
  if (!c->has_scene) return set_err(MCPT_ERR_NO_SCENE, "no scene uploaded");
  if (!c->has_target) return set_err(MCPT_ERR_NO_TARGET, "no render target");
  if (c->n_meshes == 0)
    for (int id : c->mesh_ids)
      if (id >= 0) return set_err(MCPT_ERR_BAD_SCENE, "mesh instances present: call mcpt_upload_meshes");
  HIP_OR_RETURN(hipSetDevice(c->device));
  mcpt::RenderParams p;
  std::memset(&p, 0, sizeof(p));
  p.nodes = c->d_nodes; p.leaves = c->d_leaves; p.ptype = c->d_ptype; p.prims = c->d_prims;
  p.accum = c->d_accum; p.events = c->d_events;
  corner_rays(invPV, invV, p);
  p.W = c->W; p.H = c->H; p.rows = c->d_rows;
  p.n_local_rows = c->n_local_rows; p.depth = c->depth; p.n_prims = c->n_prims;
  {
    const long long lds = ((3LL * ((2LL << c->depth) - 1) + (long long)mcpt::kPrimF4 * c->n_prims) * 16) +
                          (((1LL << c->depth) + c->n_prims) * 4);
    p.lds_scene_bytes = lds <= mcpt::kLdsSceneBytes ? (int)lds : 0;
  }
  p.minfo = c->d_minfo; p.mpairs = c->d_mpairs; p.mleaftris = c->d_mleaftris; p.mtris = c->d_mtris;
  p.mverts = c->d_mverts; p.mnorms = c->d_mnorms; p.n_meshes = c->n_meshes; p.flat_face = c->flat_face;
  {
    // AUTO: the trial before the last call is collected now (its render has ended while the last
    // call's runs); all of them first when this call's shape differs from theirs
    const long long px = (long long)c->n_local_rows * c->W;
    bool other = false;
    for (int i = 0; i < c->n_pend; ++i) other |= c->pend[i].shape[0] != px || c->pend[i].shape[1] != n_passes;
    HIP_OR_RETURN(collect_tuning(c, (other || count) ? 0 : 1));
  }
  // (the counting build is not timed: AUTO counts with the per-lane walk)
  p.tile_w = mcpt::tile_w_for(c->n_meshes > 0, p.lds_scene_bytes);
  p.n_tiles = ((c->W + p.tile_w - 1) / p.tile_w) * ((c->n_local_rows + mcpt::kTileH - 1) / mcpt::kTileH);
  auto fdiv = [](int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); };
  const long long total_seg = n_passes > 0 ? fdiv(first_pass + n_passes - 2, mcpt::kPassChunk) -
                                                 fdiv(first_pass - 1, mcpt::kPassChunk) + 1
                                           : 0;
  // segment groups need segments to group; whether longer items pay (the lanes' pass-count
  // tails average out) or cost (longer grid tail) depends on the scene and the launch: timed,
  // not guessed (profiles/r01_ab44_seg_per_item.jsonl, r01_ab49_seg_groups_tail.jsonl)
  c->deep_auto = c->depth >= 8;
  const int cand = count ? (c->traversal == MCPT_TRAVERSAL_AUTO ? MCPT_TRAVERSAL_LANE : c->traversal)
                         : resolve_candidate(c, total_seg);
  const bool stream = cand == kCandStream && stream_applies(c, variant, bounces, count);
  c->stream_iters = 0;
  const int mode = (cand >= kCandLaneSeg2 || cand == kCandStream) ? MCPT_TRAVERSAL_LANE : cand;
  p.wave_traversal = (mode == MCPT_TRAVERSAL_WAVE) ? 1 : 0;
  p.walk_exit = resolve_walk_exit(c);
  p.leaf_batch = resolve_leaf_batch(c);
  p.walk_min_done = 1;
  if (cand_deep_knobs(cand)) {   // the deep candidates' knobs, unless set explicitly
    if (c->walk_exit < 0) p.walk_exit = kDeepWalkExit;
    if (c->leaf_batch < 0) p.leaf_batch = kDeepLeafBatch;
    p.walk_min_done = kDeepMinDone;
  }
  // MCPT_WALK_MIN_DONE overrides (tuning hook; same bits for any value)
  if (const int md = env_int("MCPT_WALK_MIN_DONE", 0); md > 0) p.walk_min_done = md;
  // pass segments per work item: candidate 3 of AUTO runs two; MCPT_SEG_PER_ITEM overrides
  const int env_seg = env_int("MCPT_SEG_PER_ITEM", 0);
  p.seg_per_item = env_seg > 0 ? env_seg : cand_seg_per_item(cand);
  p.first_pass = first_pass; p.n_passes = n_passes; p.bounces = bounces; p.variant = variant;
  p.date = date; p.ior = refract_ind;
  p.inv_ior = 1.0f / refract_ind;
  {
    float r0 = (refract_ind - 1.0f) / (refract_ind + 1.0f);   // schlick tp/montecarlo.frag:93-94
    p.schlick_r0 = r0 * r0;
    p.schlick_1mr0 = 1.0f - p.schlick_r0;
    p.ior_sq = refract_ind * refract_ind;
    p.inv_ior_sq = p.inv_ior * p.inv_ior;
    const float fmax = mcpt::kFLTMAX, nx = std::nextafter(fmax, INFINITY);   // cull_bound_sq(FLT_MAX)
    const double m = ((double)fmax + (double)nx) * 0.5;
    p.cull2_max = m * m;
  }
  p.n_local_px = (long long)c->n_local_rows * c->W;
  // The call's pass range is cut at accumulation-chunk boundaries into sub-launches of at
  // most max_seg segments, so that the segment-sum buffer stays within partial_budget and
  // the grid within 2^32 work-items (an 84,000-pass 4K call is ~2,600 segments: 261 GB of
  // segment sums in one launch).  Chunk sums still reach the accumulator in chunk order, so
  // the result is bit-identical to one launch.
  const long long seg_bytes = p.n_local_px * 3 * (long long)sizeof(float);
  // (the grid's spare workgroups — split pieces of mesh launches, tail pieces: mcpt_launch_render —
  // are reserved: tail_m <= 4 x 7 workgroups per CU (tile_w >= 16 outside the mesh kernels))
  const long long kseg_max = std::max(1, p.seg_per_item);
  const long long spare = (long long)kSplitMax * (mcpt::kSplitPieces - 1) + 28LL * c->n_cu * (kseg_max - 1);
  const long long max_items = (1LL << 32) / (p.tile_w * mcpt::kTileH) - 1 - spare;
  if (p.n_tiles > max_items) return set_err(MCPT_ERR_INVALID_ARG, "render target too large for one launch");
  long long max_seg = seg_bytes > 0 ? (long long)(c->partial_budget / (size_t)seg_bytes) : (1LL << 30);
  // mesh launches that may steal passes also store every pass's value (kPassChunk per segment and
  // pixel): at most kStealBudget of them per render lane, but two segments at least, so that
  // split items and stealing still apply (1080p: 10 segments per sub-launch; 4K: 2, 6.4 GB)
  const bool may_steal = c->n_meshes > 0 && !p.wave_traversal && kseg_max == 1 && env_int("MCPT_STEAL", 1) != 0;
  if (may_steal && seg_bytes > 0)
    max_seg = std::min(max_seg, std::max(2LL, (long long)(kStealBudget / ((size_t)seg_bytes * mcpt::kPassChunk))));
  max_seg = std::max(1LL, std::min(max_seg, p.n_tiles > 0 ? max_items / p.n_tiles : max_items));
  // Pass split: a launch with too few work items to fill the chip (C1: 256 tiles x 1 segment
  // on 256 CUs, one wave per SIMD running every pass of its pixels in turn) runs one segment per
  // pass instead, so the passes of a pixel run side by side in different work items; the split
  // combine sums each chunk's passes from 0 in pass order (the bits of the unsplit launch).
  // MCPT_PASS_SPLIT=0/1 forces it off/on (tests, A/B).
  const int env_split = env_int("MCPT_PASS_SPLIT", -1);
  const bool split_fits = !stream && n_passes > 1 && n_passes <= max_seg && n_passes <= kPassSplitMaxPasses &&
                          p.n_tiles * (long long)n_passes <= max_items;
  const bool split = split_fits && (env_split >= 0 ? env_split > 0
                                                   : p.n_tiles * total_seg < (long long)kPassSplitItemsPerCu * c->n_cu);
  p.pass_split = split ? 1 : 0;
  if (split) p.seg_per_item = 1;
  int n_sub = 0;
  for (long long lo = first_pass, end = (long long)first_pass + n_passes; lo < end; ++n_sub) {
    const long long c0 = fdiv((int)(lo - 1), mcpt::kPassChunk);
    lo = split ? end : std::min(end, (c0 + max_seg) * mcpt::kPassChunk + 1);
  }
  const int slot = (c->ring_pos + 1) % kTimingRing;   // this call's events (ring of calls)
  HIP_OR_RETURN(ensure_events(c, slot, std::max(n_sub, 1)));
  // lane launches (mcpt_ctx::Lane) once AUTO has settled.  (AUTO's trials run in order on
  // `stream`: on the lanes a trial's period would be charged its own tail and discounted the
  // previous trial's, which favours the candidates with short items — C2 / C5 picked two segments
  // per item where four are 3 % faster on the lanes, tools/seg_ab.py, profiles/r06_seg_ab.jsonl)
  const bool lanes_ok = c->overlap != 0 && !count && !stream &&
                        (c->traversal != MCPT_TRAVERSAL_AUTO || c->tune_choice != 0);
  if (count) HIP_OR_RETURN(hipMemsetAsync(c->d_events, 0, sizeof(unsigned long long) * mcpt::EV_COUNT, c->stream));
  const double samples = (double)p.n_local_px * n_passes;
  // The call's events go to ring slot `slot`; the ring position (what mcpt_last_render_ms and
  // the AUTO timing read) moves there only once every event of the call has been recorded, so a
  // call that fails part-way leaves the previous call's complete timings in place.
  if (n_sub == 0) {   // no passes: an empty timed interval
    for (int i = 0; i < kEvPerSub; ++i) HIP_OR_RETURN(hipEventRecord(ev_at(c, slot, 0, i), c->stream));
    c->ring_lane[slot][0] = 0;
  }
  for (long long lo = first_pass, end = (long long)first_pass + n_passes, k = 0; lo < end; ++k) {
    const long long c0 = fdiv((int)(lo - 1), mcpt::kPassChunk);
    const long long hi = split ? end : std::min(end, (c0 + max_seg) * mcpt::kPassChunk + 1);
    p.first_pass = (int)lo;
    p.n_passes = (int)(hi - lo);
    p.n_segments = split ? p.n_passes : fdiv((int)(hi - 2), mcpt::kPassChunk) - (int)c0 + 1;
    // work-item order (mcpt_order.hip): launches of >= kOrderMinItems items run the order
    // sorted from an earlier launch of the same shape and measure their items for the next sort
    const int kseg = p.seg_per_item > 1 ? p.seg_per_item : 1;
    const long long items = (long long)p.n_tiles * ((p.n_segments + kseg - 1) / kseg);
    const long long key[8] = {items, p.n_segments, kseg, p.wave_traversal, p.walk_exit, bounces, variant,
                              (long long)p.pass_split};
    // (MCPT_ITEM_ORDER=0: dispatch order b = item, tests and A/B; the same bits either way)
    const bool order = !count && !stream && items >= kOrderMinItems && env_int("MCPT_ITEM_ORDER", 1) != 0;
    p.item_perm = nullptr;
    p.item_cost = nullptr;
    p.split_n = nullptr; p.split_of = nullptr; p.split_pass = nullptr; p.split_max = 0;
    p.steal_vals = nullptr;
    p.n_items = (int)items;
    p.tail_m = 0;
#ifdef MCPT_CHECKED
    p.check_inject = env_int("MCPT_CHECKED_INJECT", 0);
#endif
    // split items: mesh launches of whole 32-pass segments, one per item (MCPT_SPLIT_ITEMS=0: off)
    const bool split_items = order && c->n_meshes > 0 && !p.wave_traversal && kseg == 1 && !p.pass_split &&
                             p.n_segments > 1 && (p.first_pass - 1) % mcpt::kPassChunk == 0 &&
                             p.n_passes % mcpt::kPassChunk == 0 && env_int("MCPT_SPLIT_ITEMS", 1) != 0;
    // the sub-launch's lane: its segment-sum buffer and work-item order state.  A lane launch
    // (several segments: the render writes only the lane's buffers) runs its set-up and render on
    // the lane's stream once the lane's previous combine is done, so it can start while the
    // previous launch's last workgroups still run; the combine follows on `stream` in call order.
    const int li = c->next_lane;
    c->next_lane ^= 1;
    mcpt_ctx::Lane& L = c->lanes[li];
    const bool lane = lanes_ok && p.n_segments > 1;
    hipStream_t ws = lane ? L.stream : c->stream;   // the stream of the render and its set-up
    if (p.n_segments > 1 && (size_t)p.n_segments * (size_t)seg_bytes > L.partial_bytes) {
      const size_t need = (size_t)p.n_segments * (size_t)seg_bytes;
      HIP_OR_RETURN(hipStreamSynchronize(c->stream));   // (ordered after every lane's work)
      (void)hipFree(L.d_partial);
      L.d_partial = nullptr;
      L.partial_bytes = 0;
      HIP_OR_RETURN(hipMalloc(&L.d_partial, need));
      L.partial_bytes = need;
    }
    p.partial = L.d_partial;
    if (order) HIP_OR_RETURN(ensure_item_order(c, L, items));
    // (a lane whose last launches ran in order on `stream` is free once `stream`'s work so far is)
    auto freed = [&](mcpt_ctx::Lane& X) -> hipEvent_t {
      if (X.freed_stale && hipEventRecord(X.freed, c->stream) == hipSuccess) X.freed_stale = false;
      return X.freed;
    };
    if (lane) HIP_OR_RETURN(hipStreamWaitEvent(L.stream, freed(L), 0));
    if (order && !(L.order_valid && std::equal(key, key + 8, L.order_key))) {
      // the other lane holds this shape's order (AUTO's trials alternate candidates between the
      // lanes; a new shape's first launches): copied once its last sort is done, so that a trial
      // runs the order a settled launch of its candidate would
      mcpt_ctx::Lane& O = c->lanes[li ^ 1];
      if (O.order_valid && std::equal(key, key + 8, O.order_key) && O.item_cap >= items) {
        HIP_OR_RETURN(hipStreamWaitEvent(ws, O.tail, 0));
        HIP_OR_RETURN(hipStreamWaitEvent(ws, freed(O), 0));
        HIP_OR_RETURN(hipMemcpyAsync(L.d_item_perm, O.d_item_perm, sizeof(int) * (size_t)items, hipMemcpyDeviceToDevice, ws));
        HIP_OR_RETURN(hipMemcpyAsync(L.d_split_n, O.d_split_n, sizeof(int), hipMemcpyDeviceToDevice, ws));
        // (the other lane's next sort, which rewrites its order, waits for the copy)
        HIP_OR_RETURN(hipEventRecord(L.tail, ws));
        HIP_OR_RETURN(hipStreamWaitEvent(O.stream, L.tail, 0));
        std::copy(key, key + 8, L.order_key);
        L.order_valid = true;
        L.order_age = O.order_age;
      }
    }
    if (order) {
      if (L.order_valid && std::equal(key, key + 8, L.order_key)) {
        p.item_perm = L.d_item_perm;
        // items of several segments: the cheapest (last) one workgroup-generation of the order
        // runs one segment per workgroup, so the launch does not end on whole long items
        if (kseg > 1 && !p.pass_split && c->n_meshes == 0 && env_int("MCPT_TAIL_PIECES", 1) != 0) {   // (the mesh kernels split items their own way)
          const int waves_simd = c->n_meshes > 0 ? 5 : 7;
          const long long per_cu = 4LL * waves_simd / (p.tile_w / 8);
          // (one generation: C4 +2.0 %, C2 +0.3 %; 0.5 / 2 / 3 generations no better on C4:
          // profiles/r05_ab_tail_pieces.jsonl)
          p.tail_m = (int)std::min(items / 2, per_cu * c->n_cu);
        }
      }
      HIP_OR_RETURN(hipMemsetAsync(L.d_item_cost, 0, sizeof(unsigned) * (size_t)items, ws));
      p.item_cost = L.d_item_cost;
    }
    if (split_items) {
      if (!L.d_split_pass) {
        HIP_OR_RETURN(hipMalloc(&L.d_split_pass, sizeof(float) * 3 * (size_t)kSplitMax * mcpt::kPassChunk *
                                                     mcpt::kTileThreads));
      }
      HIP_OR_RETURN(hipMemsetAsync(L.d_split_of, 0xff, sizeof(int) * (size_t)items, ws));
      p.split_of = L.d_split_of;
      p.split_pass = L.d_split_pass;
      p.split_max = kSplitMax;
      if (p.item_perm) p.split_n = L.d_split_n;
      // pass stealing (kernel: steal_next; MCPT_STEAL=0: off, tests and A/B; the same bits either way)
      if (env_int("MCPT_STEAL", 1) != 0) {
        const size_t need = sizeof(float) * 3 * (size_t)items * mcpt::kPassChunk * mcpt::kTileThreads;
        if (need > L.steal_bytes) {
          HIP_OR_RETURN(hipStreamSynchronize(c->stream));   // (ordered after every lane's work)
          (void)hipFree(L.d_steal);
          L.d_steal = nullptr;
          L.steal_bytes = 0;
          HIP_OR_RETURN(hipMalloc(&L.d_steal, need));
          L.steal_bytes = need;
        }
        p.steal_vals = L.d_steal;
      }
    }
    // The timed interval of a lane launch that follows one on the other lane starts where that
    // launch's render ended (recorded on its stream): the launches overlap, and each is charged
    // its period, not its whole span (which would count the overlapped tails twice)
    const bool period = lane && c->prev_lane >= 0 && c->prev_lane != li;
    HIP_OR_RETURN(hipEventRecord(ev_at(c, slot, (int)k, 0), period ? c->lanes[c->prev_lane].stream : ws));
    if (lane) HIP_OR_RETURN(hipEventRecord(ev_at(c, slot, (int)k, 3), ws));   // (in order: the span is 0 -> 1)
    c->ring_lane[slot][k] = lane;
    if (stream) {
      const int st = stream_run(c, p);
      if (st != MCPT_OK) return st;
    } else {
      HIP_OR_RETURN(mcpt_launch_render(p, count, ws));
    }
    HIP_OR_RETURN(hipEventRecord(ev_at(c, slot, (int)k, 1), ws));
    if (lane) {   // the combine after the render; (the period's start too, so that the events a
                  // caller reads once the combine's end has completed are all complete)
      HIP_OR_RETURN(hipStreamWaitEvent(c->stream, ev_at(c, slot, (int)k, 1), 0));
      if (period) HIP_OR_RETURN(hipStreamWaitEvent(c->stream, ev_at(c, slot, (int)k, 0), 0));
    }
    HIP_OR_RETURN(mcpt_launch_combine(p, c->stream));
    HIP_OR_RETURN(hipEventRecord(ev_at(c, slot, (int)k, 2), c->stream));
    if (order && (!p.item_perm || ++L.order_age >= kOrderRefresh)) {
      // sorted after this launch's render (outside its timed events); the lane's next launch of
      // this shape reads the order in stream order, so no host wait
      size_t tmp = L.sort_tmp_bytes;
      HIP_OR_RETURN(mcpt_order_items(L.d_item_cost, L.d_cost_sorted, L.d_item_iota, L.d_item_perm, (int)items,
                                     L.d_sort_tmp, &tmp, ws));
      // mesh scenes: how many of the costliest to split next time (the mesh kernels run 5
      // waves per SIMD: 20 per CU, in workgroups of tile_w / 8 waves)
      if (c->n_meshes > 0)
        HIP_OR_RETURN(mcpt_split_count(L.d_cost_sorted, (int)items, 20 / (p.tile_w / 8) * c->n_cu, kSplitMax, L.d_split_n,
                                       c->d_events + kDebugSplitSlot, ws));
      std::copy(key, key + 8, L.order_key);
      L.order_valid = true;
      L.order_age = 0;
    }
    if (lane) {   // `stream` stays ordered after all of the lane's work
      HIP_OR_RETURN(hipEventRecord(L.tail, L.stream));
      HIP_OR_RETURN(hipStreamWaitEvent(c->stream, L.tail, 0));
    }
    if (lane) {
      HIP_OR_RETURN(hipEventRecord(L.freed, c->stream));
      L.freed_stale = false;
    } else {
      L.freed_stale = true;
    }
    c->prev_lane = lane ? li : -1;
#ifdef MCPT_CHECKED
    {
      // checked build: the sub-launch (render, combine, order sort) is waited for here, so a fault
      // is reported with the sub-launch that caused it, and the kernels' bounds tests are read
      const int st = checked_sub_launch(c, (int)k, n_sub, p);
      if (st != MCPT_OK) return st;
    }
#endif
    lo = hi;
  }
  if (!count && c->traversal == MCPT_TRAVERSAL_AUTO && !c->tune_choice && samples >= kTuneMinSamples && c->n_pend < 2) {
    if (p.n_local_px != c->meas_shape[0] || n_passes != c->meas_shape[1]) c->meas_segs = (int)total_seg;
    mcpt_ctx::TunePending& t = c->pend[c->n_pend++];
    t.cand = cand;
    t.samples = samples;
    t.shape[0] = p.n_local_px;
    t.shape[1] = n_passes;
    t.slot = slot;
  }
  c->n_sub = std::max(n_sub, 1);
  c->ring_pos = slot;
  c->ring_n_sub[slot] = c->n_sub;
  c->n_timed++;
  c->pass_split = split ? 1 : 0;
  c->timed = true;
  c->pass_count += n_passes;
  if (count) {
    unsigned long long h[mcpt::EV_COUNT];
    HIP_OR_RETURN(hipMemcpyAsync(h, c->d_events, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIP_OR_RETURN(hipStreamSynchronize(c->stream));
    for (int e = 0; e < mcpt::EV_COUNT; ++e) events[e] += h[e];
  }
  return MCPT_OK;
}

int mcpt_render(mcpt_ctx* c, const float* invPV, const float* invV, int first_pass, int n_passes, float date,
                int bounces, float refract_ind, int variant) {
  return launch(c, invPV, invV, first_pass, n_passes, date, bounces, refract_ind, variant, false, nullptr);
}

int mcpt_render_counted(mcpt_ctx* c, const float* invPV, const float* invV, int first_pass, int n_passes,
                        float date, int bounces, float refract_ind, int variant, unsigned long long* events) {
  if (!events) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  return launch(c, invPV, invV, first_pass, n_passes, date, bounces, refract_ind, variant, true, events);
}

int mcpt_debug_counters(mcpt_ctx* c, unsigned long long* out, int n_slots, int reset) {
  if (!c || n_slots < 0 || (!out && n_slots > 0)) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  HIP_OR_RETURN(hipSetDevice(c->device));
  const int n = n_slots < MCPT_DEBUG_SLOTS ? n_slots : MCPT_DEBUG_SLOTS;   // never past the caller's buffer
  if (n > 0)
    HIP_OR_RETURN(hipMemcpyAsync(out, c->d_events, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost, c->stream));
  if (reset) HIP_OR_RETURN(hipMemsetAsync(c->d_events, 0, sizeof(unsigned long long) * MCPT_DEBUG_SLOTS, c->stream));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  return MCPT_OK;
}

#ifdef MCPT_BLOCKTIMES
// diagnostic build only: the per-wave (start, end) clock pairs of the last render launch
// (wave w of workgroup b at 2 (b * waves per workgroup + w)), zeroed after the copy
extern "C" int mcpt_debug_blocktimes(mcpt_ctx* c, unsigned long long* out, long long n) {
  if (!c || !out || n < 0 || (size_t)n > mcpt::kBlockTimeSlots) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipMemcpyAsync(out, c->d_events + MCPT_DEBUG_SLOTS, sizeof(unsigned long long) * n,
                               hipMemcpyDeviceToHost, c->stream));
  HIP_OR_RETURN(hipMemsetAsync(c->d_events + MCPT_DEBUG_SLOTS, 0, sizeof(unsigned long long) * mcpt::kBlockTimeSlots, c->stream));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  return MCPT_OK;
}
#endif

int mcpt_event_bytes(int e) {
  if (e < 0 || e >= mcpt::EV_COUNT) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  return mcpt::kEventBytes[e];
}

int mcpt_read_accum(mcpt_ctx* c, float* rgb_out, int* pass_count) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  HIP_OR_RETURN(hipSetDevice(c->device));
  if (rgb_out && c->accum_bytes)
    HIP_OR_RETURN(hipMemcpyAsync(rgb_out, c->d_accum, c->accum_bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  if (pass_count) *pass_count = c->pass_count;
  return MCPT_OK;
}

int mcpt_write_accum(mcpt_ctx* c, const float* rgb, int pass_count) {
  if (!c || !rgb || pass_count < 0) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  HIP_OR_RETURN(hipSetDevice(c->device));
  if (c->accum_bytes)
    HIP_OR_RETURN(hipMemcpyAsync(c->d_accum, rgb, c->accum_bytes, hipMemcpyHostToDevice, c->stream));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  c->pass_count = pass_count;
  return MCPT_OK;
}

namespace mcpt {
namespace host {
int checkpoint_write_ex(const char* path, const float* rgb, int W, int rows, int pass_count, int next_pass,
                        const char* tag, int H, unsigned long long rows_hash);
int checkpoint_read_ex(const char* path, float* rgb_out, long long capacity, int* W, int* rows, int* pass_count,
                       int* next_pass, char* tag_out, int* H, unsigned long long* rows_hash);
}  // namespace host
}  // namespace mcpt

// identity of a context's target for its checkpoints: FNV-1a (64 bit) over its image row ids
static unsigned long long rows_hash(const mcpt_ctx* c) {
  unsigned long long h = 1469598103934665603ULL;
  for (int y : c->rows)
    for (int b = 0; b < 4; ++b) {
      h ^= (unsigned long long)(((uint32_t)y >> (8 * b)) & 0xFFu);
      h *= 1099511628211ULL;
    }
  return h ? h : 1;   // 0 means "no identity" in the file
}

int mcpt_checkpoint_save(mcpt_ctx* c, const char* path, int next_pass, const char* tag) {
  if (!c || !path) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  std::vector<float> acc((size_t)c->n_local_rows * c->W * 3);
  int n = 0;
  const int st = mcpt_read_accum(c, acc.data(), &n);
  if (st != MCPT_OK) return st;
  if (mcpt::host::checkpoint_write_ex(path, acc.data(), c->W, c->n_local_rows, n, next_pass, tag, c->H, rows_hash(c)) !=
      MCPT_OK)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_checkpoint_save: cannot write the file");
  return MCPT_OK;
}

int mcpt_checkpoint_load(mcpt_ctx* c, const char* path, const char* tag, int* next_pass) {
  if (!c || !path) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  int w = 0, rows = 0, n = 0, nxt = 0, h = 0;
  unsigned long long hash = 0;
  std::vector<char> t(MCPT_CHECKPOINT_TAG_MAX);
  std::vector<float> acc((size_t)c->n_local_rows * c->W * 3);
  if (mcpt::host::checkpoint_read_ex(path, acc.data(), (long long)acc.size(), &w, &rows, &n, &nxt, t.data(), &h,
                                     &hash) != MCPT_OK)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_checkpoint_load: missing, foreign or truncated file, or not this target's size");
  if (h == 0 || hash == 0)
    return set_err(MCPT_ERR_INVALID_ARG,
                   "mcpt_checkpoint_load: the file carries no target identity (mcpt_checkpoint_write); "
                   "read it with mcpt_checkpoint_read and load it with mcpt_write_accum");
  if (w != c->W || rows != c->n_local_rows || h != c->H || hash != rows_hash(c))
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_checkpoint_load: the checkpoint belongs to another target or shard");
  if (tag && std::strcmp(tag, t.data()) != 0)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_checkpoint_load: the render parameters differ (tag)");
  const int st = mcpt_write_accum(c, acc.data(), n);
  if (st != MCPT_OK) return st;
  if (next_pass) *next_pass = nxt;
  return MCPT_OK;
}

int mcpt_accum_device_ptr(mcpt_ctx* c, void** dev_ptr, size_t* bytes) {
  if (!c || !dev_ptr) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  *dev_ptr = c->d_accum;
  if (bytes) *bytes = c->accum_bytes;
  return MCPT_OK;
}

int mcpt_copy_accum_device(mcpt_ctx* c, void* dst, size_t bytes) {
  if (!c || (!dst && bytes)) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->has_target) return mcpt_err_bare(MCPT_ERR_NO_TARGET);
  if (bytes < c->accum_bytes) return set_err(MCPT_ERR_INVALID_ARG, "destination smaller than the accumulator");
  HIP_OR_RETURN(hipSetDevice(c->device));
  if (c->accum_bytes)
    HIP_OR_RETURN(hipMemcpyAsync(dst, c->d_accum, c->accum_bytes, hipMemcpyDeviceToDevice, c->stream));
  return MCPT_OK;
}

int mcpt_gather_rows(mcpt_ctx* frame, mcpt_ctx* const* shards, int n_shards) {
  if (!frame || n_shards < 0 || (n_shards > 0 && !shards)) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_gather_rows: bad arguments");
  if (!frame->has_target) return set_err(MCPT_ERR_NO_TARGET, "mcpt_gather_rows: frame has no target");
  if (frame->n_local_rows != frame->H) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_gather_rows: frame target is a shard");
  for (int k = 0; k < n_shards; ++k) {
    const mcpt_ctx* s = shards[k];
    if (!s || s == frame) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_gather_rows: bad shard context");
    if (!s->has_target) return set_err(MCPT_ERR_NO_TARGET, "mcpt_gather_rows: shard has no target");
    if (s->W != frame->W || s->H != frame->H) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_gather_rows: shard size differs");
    if (s->pass_count != shards[0]->pass_count)
      return set_err(MCPT_ERR_INVALID_ARG, "mcpt_gather_rows: shards hold different pass counts");
  }
  // the calling thread's current device is restored on every return path
  struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
  } device_guard;
  // an event created here is destroyed on every return path (it is released by HIP once the
  // waits recorded against it have been satisfied)
  struct EventGuard {
    hipEvent_t e = nullptr;
    ~EventGuard() { if (e) (void)hipEventDestroy(e); }
  };
  const size_t row_bytes = (size_t)frame->W * 3 * sizeof(float);
  for (int k = 0; k < n_shards; ++k) {
    mcpt_ctx* s = shards[k];
    if (s->device != frame->device) {
      int ok = 0;
      HIP_OR_RETURN(hipDeviceCanAccessPeer(&ok, frame->device, s->device));
      if (ok) {   // direct xGMI reads/writes between the two devices (once per process)
        HIP_OR_RETURN(hipSetDevice(frame->device));
        const hipError_t e = hipDeviceEnablePeerAccess(s->device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return set_err(MCPT_ERR_HIP, "hipDeviceEnablePeerAccess", e);
        (void)hipGetLastError();
      }
    }
    // (1) the frame's stream waits for the shard's queued work (its renders and combines)
    EventGuard done;
    HIP_OR_RETURN(hipSetDevice(s->device));
    HIP_OR_RETURN(hipEventCreateWithFlags(&done.e, hipEventDisableTiming));
    HIP_OR_RETURN(hipEventRecord(done.e, s->stream));
    HIP_OR_RETURN(hipSetDevice(frame->device));
    HIP_OR_RETURN(hipStreamWaitEvent(frame->stream, done.e, 0));
    hipError_t e = hipSuccess;
    for (int i = 0; e == hipSuccess && i < s->n_local_rows;) {
      int j = i + 1;   // run of consecutive global rows: one contiguous copy
      while (j < s->n_local_rows && s->rows[(size_t)j] == s->rows[(size_t)j - 1] + 1) ++j;
      e = hipMemcpyPeerAsync((char*)frame->d_accum + (size_t)s->rows[(size_t)i] * row_bytes, frame->device,
                             (const char*)s->d_accum + (size_t)i * row_bytes, s->device, (size_t)(j - i) * row_bytes,
                             frame->stream);
      i = j;
    }
    if (e != hipSuccess) return set_err(MCPT_ERR_HIP, "mcpt_gather_rows: peer copy", e);
    // (2) the shard's later work (a progressive caller's next render adds into d_accum in
    // place) waits for the copies that read its accumulator
    EventGuard copied;
    HIP_OR_RETURN(hipEventCreateWithFlags(&copied.e, hipEventDisableTiming));
    HIP_OR_RETURN(hipEventRecord(copied.e, frame->stream));
    HIP_OR_RETURN(hipSetDevice(s->device));
    HIP_OR_RETURN(hipStreamWaitEvent(s->stream, copied.e, 0));
  }
  if (n_shards > 0) frame->pass_count = shards[0]->pass_count;
  return MCPT_OK;
}

int mcpt_trace(mcpt_ctx* c, const float* origins, const float* dirs, int n, int any_hit, int prim, mcpt_hit* out) {
  if (!c || n < 0 || (n > 0 && (!origins || !dirs || !out))) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_trace: bad arguments");
  if (!c->has_scene) return set_err(MCPT_ERR_NO_SCENE, "no scene uploaded");
  if (prim >= c->n_prims) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_trace: primitive index out of range");
  if (c->n_meshes == 0)
    for (int id : c->mesh_ids)
      if (id >= 0) return set_err(MCPT_ERR_BAD_SCENE, "mesh instances present: call mcpt_upload_meshes");
  if (n == 0) return MCPT_OK;
  HIP_OR_RETURN(hipSetDevice(c->device));
  const size_t n3 = (size_t)n * 3 * sizeof(float), ni = (size_t)n * 3 * sizeof(int);
  const size_t nf = (size_t)n * mcpt::kTraceFloats * sizeof(float);
  char* buf = nullptr;
  HIP_OR_RETURN(hipMalloc(&buf, 2 * n3 + ni + nf));
  mcpt::TraceParams q;
  q.nodes = c->d_nodes; q.leaves = c->d_leaves; q.ptype = c->d_ptype; q.prims = c->d_prims; q.depth = c->depth;
  q.prim = prim < 0 ? -1 : prim;
  q.minfo = c->d_minfo; q.mpairs = c->d_mpairs; q.mleaftris = c->d_mleaftris; q.mtris = c->d_mtris;
  q.mverts = c->d_mverts; q.mnorms = c->d_mnorms; q.n_meshes = c->n_meshes; q.flat_face = c->flat_face;
  q.orig = (const float*)buf; q.dir = (const float*)(buf + n3);
  q.out_i = (int*)(buf + 2 * n3); q.out = (float*)(buf + 2 * n3 + ni); q.n = n;
  std::vector<int> hi((size_t)n * 3);
  std::vector<float> hf((size_t)n * mcpt::kTraceFloats);
  hipError_t e = hipMemcpyAsync(buf, origins, n3, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(buf + n3, dirs, n3, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = mcpt_launch_trace(q, any_hit != 0, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hi.data(), q.out_i, ni, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hf.data(), q.out, nf, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(buf);
  if (e != hipSuccess) return set_err(MCPT_ERR_HIP, "mcpt_trace", e);
  for (int i = 0; i < n; ++i) {
    mcpt_hit& h = out[i];
    const int* a = &hi[(size_t)i * 3];
    const float* f = &hf[(size_t)i * mcpt::kTraceFloats];
    h.shape = a[0]; h.prim = a[1]; h.dir = a[2];
    h.dist = f[0];
    std::memcpy(h.pl, f + 1, 12); std::memcpy(h.pg, f + 4, 12);
    std::memcpy(h.N, f + 7, 12); std::memcpy(h.P, f + 10, 12);
    std::memcpy(h.color, f + 13, 16); std::memcpy(h.material, f + 17, 16);
  }
  return MCPT_OK;
}

int mcpt_sample_hemisphere(mcpt_ctx* c, const float* normal3, const float* fseed3, float roughness, int nb_used,
                           int n, float* out_xyz) {
  if (!c || !normal3 || !fseed3 || n < 0 || nb_used < 0 || (n > 0 && !out_xyz))
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_sample_hemisphere: bad arguments");
  if (n == 0) return MCPT_OK;
  HIP_OR_RETURN(hipSetDevice(c->device));
  mcpt::SampleParams q;
  for (int k = 0; k < 3; ++k) { q.normal[k] = normal3[k]; q.fseed[k] = fseed3[k]; }
  q.roughness = roughness; q.nb_used = (uint32_t)nb_used; q.n = n;
  HIP_OR_RETURN(hipMalloc(&q.out, (size_t)n * 3 * sizeof(float)));
  hipError_t e = mcpt_launch_sample(q, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(out_xyz, q.out, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(q.out);
  if (e != hipSuccess) return set_err(MCPT_ERR_HIP, "mcpt_sample_hemisphere", e);
  return MCPT_OK;
}

int mcpt_set_traversal(mcpt_ctx* c, int mode) {
  if (!c || mode < MCPT_TRAVERSAL_AUTO || mode > MCPT_TRAVERSAL_STREAM)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_traversal: bad mode");
  c->traversal = mode;
  reset_tuning(c);
  if (mode != MCPT_TRAVERSAL_STREAM) return free_stream_pools(c);
  return MCPT_OK;
}

int mcpt_set_walk_exit(mcpt_ctx* c, int lanes) {
  if (!c || lanes < -1 || lanes > 64) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_walk_exit: bad lane count");
  c->walk_exit = lanes;
  return MCPT_OK;
}

int mcpt_set_stream_pool(mcpt_ctx* c, int slots, int refill) {
  if (!c || slots < 0 || refill < -1 || refill > 64) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_stream_pool: bad arguments");
  c->stream_slots = slots;
  c->stream_refill = refill;
  return MCPT_OK;
}

int mcpt_stream_iterations(mcpt_ctx* c, long long* iterations) {
  if (!c || !iterations) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *iterations = c->stream_iters;
  return MCPT_OK;
}

int mcpt_set_render_lanes(mcpt_ctx* c, int on) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));   // (ordered after every lane's work)
  c->overlap = on ? 1 : 0;
  c->prev_lane = -1;
  return MCPT_OK;
}

int mcpt_set_partial_budget(mcpt_ctx* c, size_t bytes) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  c->partial_budget = bytes;
  return MCPT_OK;
}

int mcpt_last_launch_count(mcpt_ctx* c, int* n_launches) {
  if (!c || !n_launches) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *n_launches = c->timed ? c->n_sub : 0;
  return MCPT_OK;
}

int mcpt_last_pass_split(mcpt_ctx* c, int* split) {
  if (!c || !split) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *split = c->timed ? c->pass_split : 0;
  return MCPT_OK;
}

int mcpt_set_leaf_batch(mcpt_ctx* c, int lanes) {
  if (!c || lanes < -1 || lanes > 64) return set_err(MCPT_ERR_INVALID_ARG, "mcpt_set_leaf_batch: bad lane count");
  c->leaf_batch = lanes;
  return MCPT_OK;
}

int mcpt_get_leaf_batch(mcpt_ctx* c, int* resolved) {
  if (!c || !resolved) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  // the value the next launch of the last launch shape uses (an AUTO deep candidate sets its own)
  const int cand = resolve_candidate(c, c->meas_segs);
  *resolved = (cand_deep_knobs(cand) && c->leaf_batch < 0) ? kDeepLeafBatch : resolve_leaf_batch(c);
  return MCPT_OK;
}

int mcpt_get_walk_exit(mcpt_ctx* c, int* resolved) {
  if (!c || !resolved) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const int cand = resolve_candidate(c, c->meas_segs);
  *resolved = (cand_deep_knobs(cand) && c->walk_exit < 0) ? kDeepWalkExit : resolve_walk_exit(c);
  return MCPT_OK;
}

int mcpt_get_traversal(mcpt_ctx* c, int* resolved) {
  if (!c || !resolved) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  *resolved = resolve_traversal(c);
  return MCPT_OK;
}

int mcpt_get_schedule(mcpt_ctx* c, int* traversal, int* seg_per_item, int* settled) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  const int cand = resolve_candidate(c, c->meas_segs);
  if (traversal) *traversal = cand_traversal(cand);
  const int env_seg = env_int("MCPT_SEG_PER_ITEM", 0);
  if (seg_per_item) *seg_per_item = env_seg > 0 ? env_seg : cand_seg_per_item(cand);
  if (settled) *settled = (c->traversal != MCPT_TRAVERSAL_AUTO || c->tune_choice != 0) ? 1 : 0;
  return MCPT_OK;
}

int mcpt_set_stream(mcpt_ctx* c, void* s) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return MCPT_OK;
}

int mcpt_synchronize(mcpt_ctx* c) {
  if (!c) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipStreamSynchronize(c->stream));
  return MCPT_OK;
}

int mcpt_last_render_ms(mcpt_ctx* c, float* ms) {
  if (!c || !ms) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->timed) return set_err(MCPT_ERR_INVALID_ARG, "no render timed yet");
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(hipEventSynchronize(ev_stop(c, c->n_sub - 1)));
  HIP_OR_RETURN(hipEventElapsedTime(ms, ev_start(c, 0), ev_stop(c, c->n_sub - 1)));
  return MCPT_OK;
}

int mcpt_kernel_ms_back(mcpt_ctx* c, int back, float* trace_ms, float* combine_ms) {
  if (!c || !trace_ms || !combine_ms) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (back < 0 || back >= kTimingRing || back >= c->n_timed)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_kernel_ms_back: no such call in the timing ring");
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(slot_launch_ms(c, (c->ring_pos - back + kTimingRing) % kTimingRing, trace_ms, combine_ms));
  return MCPT_OK;
}

int mcpt_kernel_span_ms_back(mcpt_ctx* c, int back, float* span_ms) {
  if (!c || !span_ms) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (back < 0 || back >= kTimingRing || back >= c->n_timed)
    return set_err(MCPT_ERR_INVALID_ARG, "mcpt_kernel_span_ms_back: no such call in the timing ring");
  HIP_OR_RETURN(hipSetDevice(c->device));
  const int slot = (c->ring_pos - back + kTimingRing) % kTimingRing;
  const std::vector<hipEvent_t>& v = c->evs[slot];
  float tot = 0.0f;
  for (int k = 0; k < c->ring_n_sub[slot]; ++k) {
    float a = 0.0f;
    HIP_OR_RETURN(hipEventSynchronize(v[kEvPerSub * k + 1]));
    HIP_OR_RETURN(hipEventElapsedTime(&a, v[kEvPerSub * k + (c->ring_lane[slot][k] ? 3 : 0)], v[kEvPerSub * k + 1]));
    tot += a;
  }
  *span_ms = tot;
  return MCPT_OK;
}

int mcpt_last_kernel_ms(mcpt_ctx* c, float* trace_ms, float* combine_ms) {
  if (!c || !trace_ms || !combine_ms) return mcpt_err_bare(MCPT_ERR_INVALID_ARG);
  if (!c->timed) return set_err(MCPT_ERR_INVALID_ARG, "no render timed yet");
  HIP_OR_RETURN(hipSetDevice(c->device));
  HIP_OR_RETURN(sub_launch_ms(c, trace_ms, combine_ms));
  return MCPT_OK;
}

}  // extern "C"
