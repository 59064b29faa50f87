// mcpt_internal.h — shared between the C-ABI host code and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// an error return without a detail (mcpt_capi.hip): drops the calling thread's unread detail of an
// earlier failure, so mcpt_error_string never attaches it to this one
int mcpt_err_bare(int status);

namespace mcpt {

// algorithmic-byte events; same order as the oracle's counters
enum { EV_NODE = 0, EV_LEAF, EV_PRIM, EV_CAND, EV_GEOM, EV_COLMAT, EV_SAMPLE, EV_TRAV, EV_MESH, EV_TRI, EV_MGEOM,
       EV_COUNT };

// bytes per event in the reference's texel model
constexpr int kEventBytes[EV_COUNT] = {
    48,   // internal node visit: 2 child boxes × 2 RGB32F texels  (raytracer_func.frag:249-255)
    4,    // leaf id R32I                                          (:243-247)
    16 + 64,  // prim header texel + inverse transform (4 texels)  (:171-178, :199-207)
    64,   // transform per accepted candidate                       (:409/426/457/498/563)
    64,   // intersection_info transform                            (:816/825/837/867)
    32,   // colour + material texels                               (:899-907)
    24,   // accumulate: RGB32F read + write (blend)                (montecarlo.cpp:450-452)
    0,    // traversal count (no bytes of its own)
    12 + 64 + 64,  // mesh instance entry: mesh info + mesh transform + transform   (:652-656)
    12 + 36,       // triangle test: index triplet + 3 positions (RGB32I/RGB32F)   (:145-153)
    12 + 72 + 64,  // mesh hit info: triplet + 3 × (position, normal) + mesh transform (:156-169, :792)
};

// device record layout (built by mcpt_upload_scene from the reference texture layout)
//   node  : 3 × float4  (centre.xyz,0) (halfwidth.xyz,0) (1/halfwidth.xyz,0)
//   prim  : 8 × float4  inverse rows 0..2, transform rows 0..2, colour, material
constexpr int kNodeF4 = 3;
// accumulation chunk of the arithmetic contract: passes are summed from 0
// inside each chunk of kPassChunk consecutive absolute pass numbers, chunk sums added to
// the accumulator in chunk order
constexpr int kPassChunk = 32;
constexpr int kSplitPieces = 4;   // pass ranges of a split work item (RenderParams::split_n)
constexpr size_t kBlockTimeSlots = size_t(8) << 20;   // diagnostic build: per-wave clock pairs
constexpr size_t kBlockTimeBase = 64;                   // after the debug slots (= MCPT_DEBUG_SLOTS)
// largest scene render_kernel stages into LDS: 160 KB / 7 workgroups - 19 KB of per-pixel rows
constexpr int kLdsSceneBytes = 3584;
constexpr int kPrimF4 = 8;
// work-item tile (pixels): a work item is a kTileW x kTileH pixel tile for one pass chunk, one
// lane per pixel, made of 8x8-pixel waves side by side: 32x8 = four waves in one 8-row strip, so
// in a row-band shard (8-row bands) all waves of a workgroup lie in one band of the image (16x16
// tiles: the slowest 8-GPU shard 2.4-4.1 % slower, profiles/r01_ab33_tile_shape.jsonl)
constexpr int kTileW = 32, kTileH = 8;
constexpr int kTileThreads = kTileW * kTileH;   // the widest tile (LDS-scene kernels)
static_assert(kTileW % 8 == 0 && kTileH % 8 == 0 && kTileThreads <= 1024, "tiles are made of 8x8 waves");
// Tile width of a render launch: a workgroup holds its LDS (per-pixel rows, staged scene) until
// its LAST wave ends, so the waves that end early leave their slots idle when no further
// workgroup fits the LDS.  Launches whose LDS allows it run narrower workgroups (round 5,
// profiles/r05_ab_tile_width.jsonl): the L1/L2 walk kernels two waves (16x8; C4 +0.7 % over
// 32x8, scene 3 +7 %; one wave: C4 -1.5 %), the mesh kernels one wave (8x8; the mesh workload
// +7 % over 32x8, +1.7 % over 16x8).  The LDS-scene kernel (7 waves/SIMD = 14 two-wave
// workgroups per CU, 9.5 KB of per-pixel rows each) runs 16x8 when the staged scene fits the
// rest of the 160 KB (kLdsScene16: scene 6, i.e. C2 / C3 / C5: +0.3..0.9 %), else 32x8.
constexpr int kLdsScene16 = (163840 / 14 - 16 * kTileH * 76) / 16 * 16;
__host__ __device__ constexpr int tile_w_for(bool mesh, int lds_scene_bytes) {
  return mesh ? 8 : (lds_scene_bytes > 0 ? (lds_scene_bytes <= kLdsScene16 ? 16 : kTileW) : 16);
}
// Slot of a mesh BVH internal node's child-pair record (64 B) from its mesh's first slot
// (mcpt_upload_meshes; SceneT::mpairs): node i -> slot i + 1, so the records of two siblings
// (2i+1, 2i+2: the left child's pending pop follows the right child's subtree) share one
// 128-byte line.  Measured interleaved on the mesh workload (tools/ab_interleave.py,
// profiles/r05_ab_mesh_layouts.jsonl): heap order (slot i) within noise of it, two-level
// treelets (a node and its right child, the reference's first descent, in one line) 2-8 %
// slower.
__host__ __device__ inline unsigned mesh_pair_slot(unsigned i) { return i + 1u; }
__host__ __device__ inline unsigned mesh_pair_slots(int depth) { return 1u << depth; }   // slots one mesh spans

struct RenderParams {
  const float4* nodes;
  const int* leaves;
  const int* ptype;
  const float4* prims;
  float* accum;                 // n_local_rows × W × 3 (local rows of this shard)
  float* partial;               // n_segments × n_local_px × 3 (segment sums; n_segments > 1)
  unsigned long long* events;   // EV_COUNT counters (counting build only)
  float ox, oy, oz;             // camera origin (invV · (0,0,0,1))
  float cd[12];                 // 4 normalized corner directions (raytracer.vert:19)
  int W, H;
  const int* rows;               // global row of each local row (n_local_rows)
  int n_local_rows;
  long long n_local_px;         // n_local_rows × W
  int n_tiles, n_segments;      // tile_w x 8 tiles of the local rows; pass segments of this launch
  int seg_per_item;             // consecutive segments one work item runs (>= 1)
  int pass_split;               // 1: one segment per pass (n_segments = n_passes; small launches)
  int depth, n_prims;
  int lds_scene_bytes;          // > 0: stage the scene into LDS (<= kLdsSceneBytes)
  // triangle meshes (mcpt_upload_meshes; layouts: SceneT); n_meshes == 0: none
  const int4* minfo;
  const float4* mpairs;
  const float4* mleaftris;
  const int4* mtris;
  const float4* mverts;
  const float4* mnorms;
  int n_meshes, flat_face;
  int wave_traversal;           // 1: wave-coherent BVH walk (traverse_wave), 0: per lane
  int walk_exit;                // per-lane walks: leave the loop at <= this many walking lanes
  int leaf_batch;               // deep-BVH walk: run the leaf block once >= this many lanes wait
  int walk_min_done;            // per-lane walks: ... and once >= this many lanes finished in the call (>= 1)
  int first_pass, n_passes, bounces, variant;
  float date, ior;
  // wave-uniform constants computed on the host (same binary32/binary64 operations as the
  // kernel would do) so that they live in SGPRs, not in spilled VGPRs: 1/ior (grefract of the
  // inner exit), Schlick's ((ior-1)/(ior+1))^2, and cull_bound_sq(FLT_MAX) (walk start).
  // ior², (1/ior)² and 1 - r0 too: computed in the kernel, the compiler hoisted them out of the
  // render loop into VGPRs and spilled them (12 B of scratch written per lane and work item:
  // ~0.4 GB of HBM writes per C4 launch, round 5)
  float inv_ior, schlick_r0;
  float ior_sq, inv_ior_sq, schlick_1mr0;
  // work-item order (mcpt_order.hip): workgroup b runs item item_perm[b] (null: item b), the
  // items sorted costliest first from an earlier launch of the same shape; item_cost[i] gets
  // item i's longest wave time of this launch (100 MHz clock ticks; null: not measured)
  const int* item_perm;
  unsigned* item_cost;
  // split items (mesh kernels, mcpt_order.hip): the first (*split_n) x kSplitPieces workgroups
  // run the (*split_n) costliest items of item_perm in kSplitPieces pass ranges each; the rest
  // run item_perm[split_n ..] whole.  Piece 0 sums its passes from 0 into the segment's slot
  // and marks split_of[item] = its split index; the later pieces store every pass's value in
  // split_pass (kPassChunk x kTileThreads x 3 floats per split index), which the combine adds
  // after piece 0's sum in pass order: the bits of the whole item.  split_n null: no split.
  const int* split_n;
  int* split_of;
  float* split_pass;
  // pass stealing (mesh kernels with split items; null: off): every pass's value of the launch goes
  // to steal_vals (n_items x kPassChunk x kTileThreads x 3 floats, by the pass's offset in its
  // segment and its pixel's thread), a lane done with its own pixel takes the next unstarted pass
  // of any pixel of its workgroup, and combine_steal_kernel sums each segment's passes from 0 in
  // pass order: the bits of the per-lane sums
  float* steal_vals;
  int n_items;                  // work items of the launch (its grid may hold spare workgroups)
  int tail_m;                   // seg_per_item > 1: the last tail_m items of item_perm run one segment per workgroup
  int tile_w;                   // the launch's tile width (tile_w_for)
  int split_max;                // most split items (grid = n_items + split_max x (kSplitPieces - 1))
  int check_inject;             // checked build only (MCPT_CHECKED_INJECT=1): test every workgroup id
                                // against n_items as round 5's tail-piece form read item_perm[b]
  double cull2_max;
};

// Stream schedule (MCPT_TRAVERSAL_STREAM): wavefront path tracing in two
// kernels per iteration.  Rays travel in a queue of payloads (SoA, field f of entry i at
// queue[par][f * n_slots + i]): the ray, the path state and, once traced, the hit record, so
// both kernels read and write them contiguously; the data of a (pixel, pass segment) unit
// that outlives one ray (its sum, cached primary hit, N/P across an inner walk) stays in the
// slot that runs the unit (slots[f * n_slots + slot]).
enum QueueField {
  QF_OX, QF_OY, QF_OZ, QF_DX, QF_DY, QF_DZ,   // the ray
  QF_AX, QF_AY, QF_AZ, QF_TX, QF_TY, QF_TZ,   // att, total
  QF_RX, QF_RY, QF_RZ,                        // RNG state (u32 bits)
  QF_STATE,                                   // bounce | phase << 8 (u32 bits)
  QF_PASS, QF_UNIT,                           // current pass; unit = segment * n_local_px + px
  QF_SLOT,                                    // the slot running the unit (-1: a dead entry)
  QF_HX, QF_HY, QF_HZ, QF_HCODE,              // the traversal's hit record (pl, code)
  QF_HTRI,                                    // ... and a mesh hit's triangle (mesh scenes)
  QF_COUNT
};
enum SlotField {
  SF_SX, SF_SY, SF_SZ,                        // the unit's sum (passes in order, from 0)
  SF_N0X, SF_N0Y, SF_N0Z, SF_P0X, SF_P0Y, SF_P0Z, SF_KEY0,   // the unit's cached primary hit
  SF_NSX, SF_NSY, SF_NSZ, SF_PSX, SF_PSY, SF_PSZ,            // N, P kept across an inner walk
  SF_COUNT
};
// ctr[]: queue lengths [0..1], trace-kernel fetch counters [2..3], dead slots [5] of one pool;
// the next unit [4] of the first pool's counters is shared by all pools (StreamParams::unit_ctr)
enum { SC_CNT = 0, SC_FETCH = 2, SC_UNIT = 4, SC_DEAD = 5, SC_COUNT = 8 };
struct StreamParams {
  RenderParams r;               // scene, target, the sub-launch's pass range and constants
  float* slots;                 // SF_COUNT x n_slots
  float* queue[2];              // QF_COUNT x n_slots each (ping-pong by parity)
  unsigned* ctr;                // SC_* counters of this pool
  unsigned* unit_ctr;           // next unit, shared by the pools of a launch
  int n_slots;                  // this pool's slots
  int unit_base;                // this pool's slots start with units unit_base, unit_base + 1, ...
  unsigned n_units;             // n_segments x n_local_px
  int parity;                   // iteration & 1: queue[parity] is this iteration's input
  int refill;                   // trace kernel: refill a wave's idle lanes once <= this many still walk
  int compact;                  // this iteration's shade kernel drops dead entries (atomic append)
};

// ray-query batch (mcpt_trace): per ray 3 ints (shape, prim, dir) and kTraceFloats floats
// (dist, pl.xyz, pg.xyz, N.xyz, P.xyz, colour rgba, material rgba) — the mcpt_hit layout
constexpr int kTraceFloats = 21;
struct TraceParams {
  const float4* nodes;
  const int* leaves;
  const int* ptype;
  const float4* prims;
  int depth;
  // triangle meshes (mcpt_upload_meshes; layouts: SceneT); n_meshes == 0: none
  const int4* minfo;
  const float4* mpairs;
  const float4* mleaftris;
  const int4* mtris;
  const float4* mverts;
  const float4* mnorms;
  int n_meshes, flat_face;
  int prim;                     // -1: whole BVH, >= 0: this primitive only
  const float* orig;            // n × 3
  const float* dir;             // n × 3
  long long n;
  int* out_i;                   // n × 3
  float* out;                   // n × kTraceFloats
};

struct SampleParams {
  float normal[3], fseed[3];
  float roughness;
  uint32_t nb_used;
  long long n;
  float* out;                   // n × 3
};

}  // namespace mcpt

hipError_t mcpt_launch_trace(const mcpt::TraceParams& q, bool any_hit, hipStream_t stream);
hipError_t mcpt_launch_sample(const mcpt::SampleParams& q, hipStream_t stream);
hipError_t mcpt_launch_render(const mcpt::RenderParams& p, bool count, hipStream_t stream);
hipError_t mcpt_launch_combine(const mcpt::RenderParams& p, hipStream_t stream);
hipError_t mcpt_iota(int* a, int n, hipStream_t stream);
hipError_t mcpt_split_count(const unsigned* cost_sorted, int n, int capacity, int split_max, int* out,
                            unsigned long long* dbg, hipStream_t stream);
constexpr int kDebugSplitSlot = 63;   // debug counter slot: items split by the last sort (mesh scenes)
constexpr int kDebugStealSlot = 62;   // debug counter slot: passes rendered by pass stealing (summed)

// Checked diagnostic build (make checked: -DMCPT_CHECKED; never timed).  Every index the render
// and combine kernels derive from the work-item order, the split items and the segment slots is
// tested against its array's length before the access; a violation is counted in debug slot
// kCheckedCountSlot, the first one's site and index kept in kCheckedSiteSlot (site << 48 | index),
// and the access is skipped — a bounds bug shows as a count, not as a memory fault that the next
// HIP call reports.  launch() synchronises after every sub-launch in this build and fails with the
// sub-launch's number and the site (mcpt_error_string).  Round 6: the tail-piece over-read of round
// 5 (item_perm read at workgroups >= n_items) would have been site CK_PERM_HEAD.
namespace mcpt {
constexpr int kCheckedCountSlot = 60, kCheckedSiteSlot = 61;
enum CheckSite {
  CK_SPLIT_N = 1,     // *split_n <= split_max
  CK_PERM_SPLIT,      // item_perm[sj], a split item's index (sj < n_items)
  CK_PERM_TAIL,       // item_perm[head + j], a tail piece's item (< n_items)
  CK_PERM_HEAD,       // item_perm[b] / item b, a whole item's workgroup (b < n_items)
  CK_ITEM,            // the item a workgroup runs (< n_items)
  CK_SPLIT_OF,        // split_of[item] (< n_items)
  CK_SPLIT_PASS,      // split_pass slot: split index < split_max, pass within the chunk
  CK_SEGMENT,         // segment slot of partial (< n_segments)
  CK_PIXEL,           // local pixel of accum / partial (< n_local_px)
  CK_COMBINE_SPLIT,   // combine_items_kernel: split index read from split_of (< split_max)
  CK_COUNT
};
#ifdef MCPT_CHECKED
constexpr bool kChecked = true;
__device__ inline bool idx_ok(unsigned long long* ev, int site, long long i, long long n) {
  if (i >= 0 && i < n) return true;
  if (ev) {
    atomicAdd(ev + kCheckedCountSlot, 1ull);
    atomicCAS(ev + kCheckedSiteSlot, 0ull, ((unsigned long long)site << 48) | ((unsigned long long)i & 0xffffffffffffull));
  }
  return false;
}
#else
constexpr bool kChecked = false;
__device__ __forceinline__ bool idx_ok(unsigned long long*, int, long long, long long) { return true; }
#endif
}  // namespace mcpt
hipError_t mcpt_order_items(const unsigned* cost, unsigned* cost_sorted, const int* iota, int* perm, int n,
                            void* tmp, size_t* tmp_bytes, hipStream_t stream);
// stream schedule: slot set-up (queue[0] = every slot with a unit), then one iteration = the
// trace kernel over queue[parity] + the shade kernel appending to queue[parity ^ 1]
hipError_t mcpt_launch_stream_init(const mcpt::StreamParams& q, hipStream_t stream);
hipError_t mcpt_launch_stream_iter(const mcpt::StreamParams& q, int n_cu, bool lds_nodes, hipStream_t stream);
// (q.r.n_meshes > 0: the mesh instantiations, walk_run_mesh in the trace kernel)
// the trace kernel can hold a BVH of this depth in LDS (nodes + leaf ids)
bool mcpt_stream_lds_nodes_fit(int depth);
