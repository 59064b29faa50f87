// mcpt_kernel.hip — the per-pixel Monte Carlo sampling loop for CDNA4 (gfx950).
//
// Replaces the reference's fragment program prg_ray = raytracer.vert +
// raytracer_func.frag + tp/<variant>.frag + main.frag (MontecarloGPU/montecarlo.cpp:345-347)
// and its additive ONE/ONE blend into the RGB32F FBO (montecarlo.cpp:450-466).
//
// Design:
//  * one lane = one pixel for a segment of up to 32 passes (one accumulation chunk);
//    a lane whose path terminates immediately regenerates the next pass's path
//    (persistent-lane regeneration), so a wave runs until its lanes' *sums* of path
//    lengths are exhausted, not the max path per pass — the 4 material branches and
//    the 0..B bounce lengths average out.  Work items = (pixel tile, pass segment), so
//    a shard has enough items to fill the chip even at 8-way row-band sharding;
//  * the bounce loop and the mixed/refraction branch's inner traversal are folded into
//    ONE traversal site per loop iteration (a 2-phase state machine), so lanes doing an
//    inner traversal and lanes doing their next bounce run the same instructions;
//  * BVH traversal is the reference's DFS (raytracer_func.frag:734-769, right child
//    popped first, cull test at push time) but stackless: the implicit-heap stack is
//    encoded as a bitmask of levels holding a pending left sibling — registers only.
//    Per lane (walk_run, resumable: deep BVHs suspend the walk loop when few lanes still
//    walk and batch leaf visits) or wave-coherent (traverse_wave, scalar loads);
//  * the primary hit of a pixel is cached per segment (no jitter: same camera ray every
//    pass); square roots and reciprocals outside the walk loop use short sequences proven
//    correctly rounded on all 2^32 inputs (mcpt_math.h, tools/mathcheck);
//  * the scene is repacked at upload into 16-byte records (node: centre / half-width /
//    1/half-width; prim: inverse rows, transform rows, colour, material) so every fetch
//    is a dwordx4; scenes up to kLdsSceneBytes are staged once per workgroup into LDS;
//  * each lane sums its segment from 0 in pass order; segment sums are added to the
//    accumulator in chunk order (combine_kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mcpt_device.h"

// minimum waves per SIMD the register allocator must allow (occupancy vs spills):
// the LDS-scene and wave-coherent kernels (72 VGPRs, no spills: 7 waves)
constexpr int kMinWaves = 7;


namespace mcpt {

// ------------------------------------------------------------------------------------
// the kernel
// ------------------------------------------------------------------------------------
// Work item = (TW x 8 pixel tile of TW/8 8x8 waves, group of seg_per_item pass segments; TW per
// launch, tile_w_for).  A
// segment is the part of the launch's pass range inside one accumulation chunk of kPassChunk
// absolute passes: segments of one pixel are independent (strong-scaling
// parallelism beyond one lane per pixel); their sums are combined in chunk order by
// combine_kernel.  Lanes: one pixel each; a lane whose path ends starts the pixel's next pass
// in the same loop iteration (sky / end folds below).
// LDSS: the scene (nodes, primitive records, leaves, type codes: RenderParams::lds_scene_bytes
// <= kLdsSceneBytes) is copied into the workgroup's LDS first, so the traversal's dependent
// node loads are LDS reads instead of L1/L2 gathers.
// SUSPEND: the deep-BVH walk (suspendable walks, batched leaf visits: RenderParams::walk_exit,
// leaf_batch; walk_run)
// per-lane walks of mesh scenes (walk_run_mesh keeps the mesh walk state and the ray in mesh
// space in registers; the instance transform is re-read per step): 5 waves/SIMD, 96 VGPRs and
// 48 B of scratch, against 113 VGPRs without spills at 4 waves: the mesh workload +5..8 %
// (round 5, profiles/r05_ab_mesh_layouts.jsonl, r05_ab_mesh_trf_reload_waves.jsonl; 7 waves
// with that state spill and run at a third of the speed, round 1)
constexpr int kMinWavesMesh = 5;
// per-lane walks over scenes read through L1/L2 (not LDS-staged: scenes 3, 5, 7, 8): 6 waves/SIMD
// while their state spilled at 7 (profiles/r01_ab35_occupancy_v12.jsonl); with the packed hit
// record they fit 72 VGPRs and 7 waves hide more of the dependent node loads (scene 8 +4 %,
// scene 3 +5 %: profiles/r02_ab4_spill_free.jsonl; 6 / 8 waves re-measured in round 4: -1.9 / -6.1 %)
constexpr int kMinWavesL2 = 7;
template <bool COUNT, bool WAVE, bool MESH, bool LDSS, bool SUSPEND, int TW>
__global__ __launch_bounds__(TW * kTileH, MESH && !WAVE ? kMinWavesMesh
                                           : (!WAVE && !LDSS ? kMinWavesL2 : kMinWaves)) void render_kernel(
    RenderParams p) {
  constexpr int TT = TW * kTileH;   // this kernel's tile (tile_w_for)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  // (XCD-aware remaps of the item order measured slower or within noise: giving each XCD one
  // contiguous 1/8 of the items unbalances the XCDs — C2 -39 %, mesh -10..18 %, C4 -4 % —
  // and chunks of 4 / 32 items per XCD change nothing; profiles/r05_ab_xcd_item_order.jsonl)
  // the launch's work-item order (mcpt_order.hip): costliest items of an earlier launch first;
  // in the mesh kernels the costliest of them split in kSplitPieces pass ranges (piece >= 0)
  constexpr bool kSplit = MESH && !WAVE && !COUNT;
  int item, piece = -1, sj = -1;
  // (idx_ok: the checked build's bounds tests, mcpt_internal.h; true in the shipped build.  The
  // workgroup-uniform ones return the whole workgroup before the LDS staging barrier.)
  if constexpr (kChecked) {   // the checker's own test: round 5's form read item_perm[blockIdx.x] first
    if (p.check_inject) (void)idx_ok(p.events, CK_PERM_HEAD, blockIdx.x, p.n_items);
  }
  if constexpr (kSplit) {
    const int b = blockIdx.x;
    int sn = (p.item_perm && p.split_n) ? *p.split_n : 0;
    if (!idx_ok(p.events, CK_SPLIT_N, sn, (long long)p.split_max + 1)) sn = 0;
    if (b < sn * kSplitPieces) {
      sj = b / kSplitPieces;
      piece = b - sj * kSplitPieces;
      if (!idx_ok(p.events, CK_PERM_SPLIT, sj, p.n_items)) return;
      item = p.item_perm[sj];
    } else {
      const int r = sn + (b - sn * kSplitPieces);
      if (r >= p.n_items) return;   // a spare workgroup (the grid holds the most pieces)
      item = p.item_perm ? p.item_perm[r] : r;
    }
  }
  // tail pieces (launches of several segments per item, mcpt_order.hip): the last tail_m items of
  // the order — the cheapest — run one segment per workgroup, so the launch ends on short pieces.
  // (The grid holds n_items + tail_m (K - 1) workgroups: item_perm is read at b < n_items only.)
  int seg_only = -1;
  if constexpr (!kSplit) {
    const int b = blockIdx.x;
    const int head = p.tail_m > 0 ? p.n_items - p.tail_m : p.n_items;
    if (b >= head && p.tail_m > 0) {
      const int q = b - head, j = q / p.seg_per_item;
      if (!idx_ok(p.events, CK_PERM_TAIL, head + j, p.n_items)) return;
      item = p.item_perm[head + j];
      seg_only = q - j * p.seg_per_item;
    } else {
      if (!idx_ok(p.events, CK_PERM_HEAD, b, p.n_items)) return;
      item = p.item_perm ? p.item_perm[b] : b;
    }
  }
  if (!idx_ok(p.events, CK_ITEM, item, p.n_items)) return;
  const unsigned long long t_item0 = __builtin_amdgcn_s_memrealtime();
#ifdef MCPT_BLOCKTIMES
  // diagnostic build only (tools/blocktimes.py; never timed): each wave's start and end on the
  // 100 MHz real-time clock, for the launch's occupancy over time (tail, XCD balance)
  const unsigned long long bt0 = __builtin_amdgcn_s_memrealtime();
#endif

  // segment-fastest item order: the pass segments of one tile are consecutive workgroups
  // (tile-fastest order was 1-12 % slower on one GPU and 7 % on a 1/8-row shard's launch:
  // profiles/r01_ab42_item_order.jsonl)
  // A work item runs K = seg_per_item consecutive segments of its tile; a lane runs its pixel's
  // segments one after another (each summed from 0 in pass order, written when it ends).
  const int K = p.seg_per_item > 1 ? p.seg_per_item : 1;
  const int n_groups = (p.n_segments + K - 1) / K;
  const int tile = item / n_groups;
  int seg_lo = (item % n_groups) * K;
  int seg_n = min(K, p.n_segments - seg_lo);
  if (seg_only >= 0) {   // a tail piece: one segment of its item
    if (seg_only >= seg_n) return;   // (the item has fewer segments: an empty piece)
    seg_lo += seg_only;
    seg_n = 1;
  }
  int seg = seg_lo;
  const int tiles_x = (p.W + TW - 1) / TW;
  const int bx0 = (tile % tiles_x) * TW + (wave % (TW / 8)) * 8;   // this wave's 8x8 block
  const int by0 = (tile / tiles_x) * kTileH + (wave / (TW / 8)) * 8;
  const int x = bx0 + (lane & 7);
  const int lr = by0 + (lane >> 3);
  const bool live = x < p.W && lr < p.n_local_rows;   // (no early return: LDS staging barrier)
  const int cbase = floordiv(p.first_pass - 1, kPassChunk);   // chunk of the launch's first pass
  const int c0 = cbase + seg_lo;
  int pass_begin = max(p.first_pass, c0 * kPassChunk + 1);
  int pass_end = min(p.first_pass + p.n_passes, (c0 + 1) * kPassChunk + 1);   // this unit's end
  if (p.pass_split) {   // one segment per pass (small launches; combine_split_kernel sums them)
    pass_begin = p.first_pass + seg_lo;
    pass_end = pass_begin + 1;
  }
  const int seg_first = pass_begin;   // the segment's first pass (pass stealing: value slots)
  int b1 = 0;   // a split item's first pass of piece 1 (its later pieces store per-pass values)
  if (kSplit && piece >= 0) {   // (split launches: full 32-pass segments, one per item)
    const int n = pass_end - pass_begin;
    b1 = pass_begin + n / kSplitPieces;
    const int lo = pass_begin + (piece * n) / kSplitPieces, hi = pass_begin + ((piece + 1) * n) / kSplitPieces;
    pass_begin = lo;
    pass_end = hi;
    if (piece == 0 && tid == 0 && idx_ok(p.events, CK_SPLIT_OF, item, p.n_items)) p.split_of[item] = sj;
  }
  const int y = live ? p.rows[lr] : 0;   // this shard's local row -> image row (mcpt_set_target*)

  SceneT<MESH, LDSS> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mpairs, p.mleaftris, p.mtris,
                       p.mverts, p.mnorms, p.flat_face};
  if constexpr (LDSS) {
    // staged layout: nodes (3 float4 each), prims (8 float4 each), leaves, type codes
    extern __shared__ float4 s_scene[];
    const int n_nodes = (2 << p.depth) - 1, n_leaves = 1 << p.depth;
    const int n4 = 3 * n_nodes + 8 * p.n_prims;
    for (int i = tid; i < n4; i += TT) s_scene[i] = i < 3 * n_nodes ? p.nodes[i] : p.prims[i - 3 * n_nodes];
    int* s_int = (int*)(s_scene + n4);
    for (int i = tid; i < n_leaves + p.n_prims; i += TT)
      s_int[i] = i < n_leaves ? p.leaves[i] : p.ptype[i - n_leaves];
    __syncthreads();
    s.nodes = s_scene;
    s.prims = s_scene + 3 * n_nodes;
    s.leaves = s_int;
    s.ptype = s_int + n_leaves;
  }
  // pass stealing (mesh kernels, steal_vals set): the workgroup's units are (pass offset, thread)
  // = (u / TT, u % TT) for u < TT x (pass_end - pass_begin); thread t starts with unit t (its own
  // pixel's first pass) and every lane claims the next one when its pass ends (s_claim)
  static_assert(!kSplit || TT == 64, "pass stealing: one wave per workgroup (LDS order, unit mapping)");
  const bool steal = kSplit && p.steal_vals != nullptr;
  __shared__ int s_claim;
  __shared__ unsigned s_stolen;   // passes this workgroup's lanes rendered for other lanes' pixels
  if constexpr (kSplit) {
    if (steal) {
      if (tid == 0) { s_claim = TT; s_stolen = 0u; }
      __syncthreads();
    }
  }
  Ev<COUNT> ev;
  ev.init();
#ifdef MCPT_LANESTATS
  for (int k = lane; k < LS_COUNT; k += 64) ls_row()[k] = 0u;
  __builtin_amdgcn_wave_barrier();
  if (!live) return;   // (diagnostic build: frames of whole tiles only)
#else
  if (!live) return;
#endif

  const float u = ((float)x + 0.5f) / (float)p.W;
  const float v = ((float)y + 0.5f) / (float)p.H;
  // Per-pixel constants live in LDS (SoA by thread: conflict-free), not in VGPRs: the
  // camera direction and the cached primary hit are read once per pass, and keeping them
  // out of the register file is what lets 7 waves/SIMD fit.  rows: 0-2 Dcam, 3-5 N0, 6-8 P0
  // (primary hit), 9-11 N / 15-17 P saved across the inner traversal, 12-14 this segment's
  // sum (from 0 in pass order); s_hit0 = primary hit shape << 28 | index (-1: miss).
  // 76 B per thread (19 KB per 32x8 workgroup), + the staged scene (LDSS, <= kLdsSceneBytes).
  // Kernels without a staged scene also keep the pixel's (u, v) there (rows 18-19), the mesh
  // kernels its local index too (row 20): held in VGPRs across the render loop they were
  // spilled registers, written to scratch once per lane and work item (C4: 1.16 -> 0.50 GB of
  // HBM writes per launch, round 5, profiles/r05_ab_c4_spills.jsonl).  The LDS-scene kernel
  // at 7 waves/SIMD has no room for them (7 x (22 + 3) KB > 160 KB) and does not spill them;
  // the per-lane mesh kernels run 5 workgroups per CU, which leaves room.  (The local index in
  // LDS cost C4 0.5 %: there it is recomputed.)
  constexpr bool kPixLds = !LDSS || (MESH && !WAVE);
  constexpr bool kPxLds = kPixLds && MESH;
  // the refraction constants ior², (1/ior)², 1 - r0 from the host (RenderParams) in the same
  // kernels: in the LDS-scene kernel they do not spill, and the in-kernel products are 0.8 %
  // faster on C2 (same file)
  constexpr bool kIorConst = kPixLds;
  __shared__ float s_pix[kPxLds ? 21 : (kPixLds ? 20 : 18)][TT];
  __shared__ int s_hit0[TT];
  const f3 Dcam0 = camera_dir(p, u, v);
  s_pix[0][tid] = Dcam0.x; s_pix[1][tid] = Dcam0.y; s_pix[2][tid] = Dcam0.z;
  if constexpr (kPixLds) {
    s_pix[18][tid] = u; s_pix[19][tid] = v;
    if constexpr (kPxLds) s_pix[20][tid] = __int_as_float(lr * p.W + x);   // < n_local_px <= 2^31 - 1 (mcpt_set_target*)
  }
  // the thread whose pixel this lane renders: its own, except for passes taken by pass stealing
  int pj = tid;
  // (u, v) of this pixel for the seed of a new pass (seed_for): the same values as u, v above
  auto pix_seed = [&](int ps) {
    if constexpr (kPixLds) return seed_for(s_pix[18][pj], s_pix[19][pj], ps, p.date);
    else return seed_for(((float)x + 0.5f) / (float)p.W, ((float)y + 0.5f) / (float)p.H, ps, p.date);
  };
  s_pix[12][tid] = 0.0f; s_pix[13][tid] = 0.0f; s_pix[14][tid] = 0.0f;   // this segment's sum
  const f3 Ocam = mk(p.ox, p.oy, p.oz);


  const float ior = p.ior;
  const int B = p.bounces;
  int pass = pass_begin;
  // path state
  Rng rng = seed_for(u, v, pass, p.date);
  f3 O = Ocam, D = Dcam0, att = mk(0.8f, 0.8f, 0.8f), total = mk(0.0f, 0.0f, 0.0f);
  f3 N = mk(0.0f, 0.0f, 0.0f), P = mk(0.0f, 0.0f, 0.0f);
  int bounce = 0, phase = 0;
  Hit h;
  h.pl = mk(0.0f, 0.0f, 0.0f); h.dist = kFLTMAX; h.clear(); h.tri = 0;
  h.cull2 = 0.0;

  // Primary-ray cache.  The camera ray of a pixel is the same in every pass (fixed
  // interpolated direction, fixed origin: raytracer.vert has no jitter) and the
  // traversal, the hit record and intersection_info consume no RNG, so the first
  // traversal of every pass has one result per pixel: compute it once per segment.
  // Exact (same values); the counting build keeps the reference's per-pass traversal so
  // its events stay the reference's algorithmic model.
  int key0 = -1;
  f3 N0 = N, P0 = P;   // only live until stored to LDS
  const bool run = !(p.variant == 0 && B <= 0);
#ifdef MCPT_STAMPS
  // diagnostic build only (never timed): wave-cycle shares of the kernel's sections
  unsigned long long st_k0 = __builtin_amdgcn_s_memtime(), st_t = 0, st_s = 0, st_it = 0;
#endif
  if (!COUNT && run) {
    traverse<COUNT, WAVE, SUSPEND && !LDSS && !MESH>(s, Ocam, Dcam0, h, ev);
    key0 = hit_key(h);
    if (h.hit()) geom_info<COUNT>(s, h, N0, P0, ev);
  }
  s_pix[3][tid] = N0.x; s_pix[4][tid] = N0.y; s_pix[5][tid] = N0.z;
  s_pix[6][tid] = P0.x; s_pix[7][tid] = P0.y; s_pix[8][tid] = P0.z;
  s_hit0[tid] = key0;   // shape << 28 | index, -1: miss

#ifdef MCPT_STAMPS
  const unsigned long long st_p = __builtin_amdgcn_s_memtime() - st_k0;
#endif
  // this segment's sum -> accumulator (one-segment launch) or its segment slot
  auto flush_sum = [&]() {
    if (kSplit && (piece > 0 || steal)) return;   // passes stored one by one (add_pass)
    // the pixel's address is recomputed at each flush (an empty asm makes the row opaque):
    // hoisted out of the render loop, its 64-bit index and pointer were 4 spilled VGPRs
    size_t px;
    if constexpr (kPxLds) {
      px = (size_t)(unsigned)__float_as_int(s_pix[20][tid]);
    } else {
      int lrow = lr, col = x;
      asm volatile("" : "+v"(lrow), "+v"(col));
      px = (size_t)lrow * p.W + col;
    }
    if (!idx_ok(p.events, CK_PIXEL, (long long)px, p.n_local_px)) return;
    if (p.n_segments == 1) {
      float* accp = p.accum + px * 3;
      accp[0] = accp[0] + s_pix[12][tid]; accp[1] = accp[1] + s_pix[13][tid]; accp[2] = accp[2] + s_pix[14][tid];
    } else {
      if (!idx_ok(p.events, CK_SEGMENT, seg, p.n_segments)) return;
      float* part = p.partial + ((size_t)seg * p.n_local_px + px) * 3;
      part[0] = s_pix[12][tid]; part[1] = s_pix[13][tid]; part[2] = s_pix[14][tid];
    }
  };
  // after pass++: the segment's last pass closes it (its sum to the segment slot) and the lane
  // goes on with its pixel's next segment of the work item.  With none left, pass stays at
  // pass_end and the lane leaves the loop.
  // a finished pass's value: into this segment's sum, or (a split item's later pieces) stored
  // for the combine, which adds it after piece 0's sum in pass order
  auto add_pass = [&](f3 v) {
    if (kSplit && steal) {
      if constexpr (kChecked) {
        if (!idx_ok(p.events, CK_SPLIT_PASS, pass - seg_first, kPassChunk) || !idx_ok(p.events, CK_SPLIT_PASS, pj, kTileThreads))
          return;
      }
      float* q = p.steal_vals + (((size_t)item * kPassChunk + (pass - seg_first)) * kTileThreads + pj) * 3;
      q[0] = v.x; q[1] = v.y; q[2] = v.z;
      return;
    }
    if (kSplit && piece > 0) {
      if constexpr (kChecked) {
        if (!idx_ok(p.events, CK_SPLIT_PASS, sj, p.split_max) || !idx_ok(p.events, CK_SPLIT_PASS, pass - b1, kPassChunk) ||
            !idx_ok(p.events, CK_SPLIT_PASS, tid, kTileThreads))
          return;
      }
      float* q = p.split_pass + (((size_t)sj * kPassChunk + (pass - b1)) * kTileThreads + tid) * 3;
      q[0] = v.x; q[1] = v.y; q[2] = v.z;
    } else {
      s_pix[12][tid] = s_pix[12][tid] + v.x;
      s_pix[13][tid] = s_pix[13][tid] + v.y;
      s_pix[14][tid] = s_pix[14][tid] + v.z;
    }
  };
  // pass stealing: after a pass (pass++ done by the caller), the lane's next unit.  Units whose
  // pixel lies outside the frame are skipped; none left: pass = pass_end, the lane is done.
  const int steal_n = pass_end - pass_begin;
  auto steal_next = [&]() {
    for (;;) {
      const int u = atomicAdd(&s_claim, 1);
      if (u >= TT * steal_n) { pass = pass_end; return; }
      const int t = u % TT;
      const int xt = bx0 + (t & 7), lt = by0 + (t >> 3);   // (one 8x8 wave per workgroup: TW = 8)
      if (xt < p.W && lt < p.n_local_rows) {
        pj = t; pass = pass_begin + u / TT;
        if (t != tid) atomicAdd(&s_stolen, 1u);
        return;
      }
    }
  };
  auto next_chunk = [&]() {
    if (kSplit && steal) {
      steal_next();
      return;
    }
    if (pass >= pass_end) {
      flush_sum();
      if (seg + 1 < seg_lo + seg_n) {
        seg++;
        const int c = c0 + (seg - seg_lo);
        pass = c * kPassChunk + 1;
        pass_end = min(p.first_pass + p.n_passes, (c + 1) * kPassChunk + 1);
        s_pix[12][tid] = 0.0f; s_pix[13][tid] = 0.0f; s_pix[14][tid] = 0.0f;
      }
    }
  };
  Walk walk;
  walk.invD = mk(0.0f, 0.0f, 0.0f); walk.node = 0; walk.level = 0; walk.pending = 0; walk.mpf = 0;
  bool walking = false;   // a suspended per-lane walk is waiting to be continued
#ifdef MCPT_LANESTATS
  ls_add(LS_WAVES, 1u);
#endif
  while (pass < pass_end) {
#ifdef MCPT_STAMPS
    const unsigned long long st_a = __builtin_amdgcn_s_memtime();
    st_it++;
#endif
#ifdef MCPT_LANESTATS
    ls_add(LS_ROUNDS, 1u);
    ls_add(LS_ROUND_LN, ls_pop(true));
#endif
    bool done = false;
    f3 res = mk(0.0f, 0.0f, 0.0f);
    bool first = !COUNT && bounce == 0 && phase == 0;   // camera ray of this pass
    bool ready = true;   // this lane's hit record is complete
    if (!run) {
      done = true;   // for(i=0; i<NB_BOUNCES ...) never runs: black
    } else {
      if (first) {
        h.code = s_hit0[pj];
      } else if (WAVE) {
        traverse<COUNT, WAVE>(s, O, D, h, ev);
      } else {
        if (!walking) { walk_begin<COUNT>(s, D, h, walk, ev, p.cull2_max); walking = true; }
        if constexpr (MESH) {
          walking = !walk_run_mesh<COUNT, SUSPEND>(s, O, D, h, walk, ev, p.walk_exit);
        } else {
          walking = !walk_run<COUNT, SUSPEND>(s, O, D, h, walk, ev, p.walk_exit, p.leaf_batch, p.walk_min_done);
        }
        ready = !walking;
      }
    }
#ifdef MCPT_STAMPS
    const unsigned long long st_b = __builtin_amdgcn_s_memtime();
    st_t += st_b - st_a;
    st_s -= st_b;
#endif
    // Sky fold: a bounce ray that left the scene ends its pass here, before the shading
    // block, and the lane starts its next pass at once with the cached primary hit, so
    // that one shading block serves both (the pass's camera-ray round, in which this
    // lane would otherwise only shade while the others traverse, disappears).  Same
    // per-lane sequence of values: the sky term, the segment sum in pass order, then the
    // next pass from its seed.
    //
    // End fold: the other two path ends known before shading fold the same
    // way.  An emissive hit (material .z > 0.5) ends the pass with total + its emission
    // term (montecarlo.frag's `else` branch: no RNG draw, no new ray), and a non-emissive
    // hit at bounce B-1 ends it black whatever the branch (reflect / diffuse reach bounce
    // B in this shading, the refraction branch after its inner walk), so neither needs
    // the shading block.
    bool fold_end = !COUNT && ready && run && p.variant == 0 && phase == 0 && !first;
    f3 fres = mk(0.0f, 0.0f, 0.0f);
    if (fold_end) {
      if (!h.hit()) {
        const float a = gmax(0.0f, D.z);
        fres = add(total, mulv(att, gmix3(mk(0.5f, 0.5f, 0.9f), mk(1.0f, 1.0f, 0.8f), a)));
      } else {
        const float4 m4 = s.prims[(size_t)h.index() * 8 + 7];
        if (!(m4.z <= 0.5f)) {   // the shading block's emissive `else`, NaN included
          const float4 c4 = s.prims[(size_t)h.index() * 8 + 6];
          fres = add(total, add(muls(mk(c4.x, c4.y, c4.z), 0.1f), muls(muls(muls(att, m4.z), 1.0f - m4.x), c4.w)));
        } else if (bounce < B - 1) {
          fold_end = false;
        }
      }
    }
    if (fold_end) {
      add_pass(fres);
      ev.inc(EV_SAMPLE);
      pass++;
      next_chunk();
      if (pass < pass_end) {
        rng = pix_seed(pass);
        O = Ocam; D = mk(s_pix[0][pj], s_pix[1][pj], s_pix[2][pj]);
        att = mk(0.8f, 0.8f, 0.8f); total = mk(0.0f, 0.0f, 0.0f);
        bounce = 0;
        h.code = s_hit0[pj];
        first = true;
      } else {
        ready = false;   // unit finished: the lane claims another at the end of the round
      }
    }
    if (ready && run) {
      if (p.variant != 0) {
        // tp/montecarlo_mat.frag:5-20 / montecarlo_mat_tr.frag:5-20
        if (!h.hit()) {
          res = mk(0.0f, 0.0f, 0.2f);
        } else {
          if (first) {
            N = mk(s_pix[3][pj], s_pix[4][pj], s_pix[5][pj]);
            P = mk(s_pix[6][pj], s_pix[7][pj], s_pix[8][pj]);
          }
          else geom_info<COUNT>(s, h, N, P, ev);
          ev.inc(EV_COLMAT);
          if (p.variant == 1) {
            float rx = rnd(rng), ry = rnd(rng), rz = rnd(rng);
            res = mk(__builtin_fabsf(N.x) * rx, __builtin_fabsf(N.y) * ry, __builtin_fabsf(N.z) * rz);
          } else {
            float4 col = s.prims[(size_t)h.index() * 8 + 6];
            float r = rnd(rng);
            res = mk(col.x * r, col.y * r, col.z * r);
          }
        }
        done = true;
      } else if (phase == 0) {
        // tp/montecarlo.frag:100-179, one bounce
        if (!h.hit()) {
          float a = gmax(0.0f, D.z);
          res = add(total, mulv(att, gmix3(mk(0.5f, 0.5f, 0.9f), mk(1.0f, 1.0f, 0.8f), a)));
          done = true;
        } else {
          if (first) {
            N = mk(s_pix[3][pj], s_pix[4][pj], s_pix[5][pj]);
            P = mk(s_pix[6][pj], s_pix[7][pj], s_pix[8][pj]);
          }
          else geom_info<COUNT>(s, h, N, P, ev);
          ev.inc(EV_COLMAT);
          const float4 c4 = s.prims[(size_t)h.index() * 8 + 6];
          const float4 m4 = s.prims[(size_t)h.index() * 8 + 7];
#ifdef MCPT_LANESTATS
          ls_cond(LS_SHADE_WV, LS_SHADE_LN, true);
#endif
          f3 ray = random_ray(rng, N, 1.0f - m4.y);
          const f3 col = mk(c4.x, c4.y, c4.z);
          const float alpha = c4.w;
          float rs = schlick(p.schlick_r0, kIorConst ? p.schlick_1mr0 : 1.0f - p.schlick_r0, D, N);
          f3 R = greflect(neg(ray), N);
          f3 E = normalize3(sub(O, P));
          float se = gmix(100.0f, 2.0f, m4.y);
          float spec = mc_pow_le1(gmax(0.0f, dot3(E, R)), se);   // E, R unit: dot <= 1 + ulps
          total = add(total, add(muls(col, 0.1f), muls(muls(muls(att, m4.z), 1.0f - m4.x), alpha)));
          if (m4.z <= 0.5f) {
            const f3 mx = gmix3(att, col, m4.x);
            const f3 base = mulv(col, att);
            bool reflect_push = false, inner = false;
            if (m4.x > 0.0f && alpha == 1.0f) {
              reflect_push = true;
            } else if (alpha < 1.0f && m4.x == 0.0f) {
              inner = true;
              // new_attenu of the pushed ray (att is not read again before the push)
              att = add(base, mulv(muls(muls(muls(att, 1.0f - alpha), 1.0f - rs), spec), mx));
              O = sub(P, muls(N, kBIAS));
              D = grefract(D, N, ior, kIorConst ? p.ior_sq : ior * ior);
            } else if (alpha < 1.0f && m4.x > 0.0f) {
              float r = rnd(rng);
              if (r > 0.5f) {
                reflect_push = true;
              } else {
                inner = true;
                att = add(base, mulv(muls(muls(muls(att, 1.0f - alpha), 1.0f - rs), spec), mx));
                O = sub(P, muls(N, kBIAS));
              }
            } else {   // diffuse
              att = add(base, mulv(muls(att, spec), mx));
              O = add(P, muls(N, kBIAS));
              D = ray;
              bounce++;
            }
            if (reflect_push) {
              f3 na = add(base, mulv(muls(muls(muls(att, alpha), rs), spec), mx));
#ifdef MCPT_LANESTATS
              ls_cond(LS_RR2_WV, LS_RR2_LN, true);
#endif
              f3 rd = random_ray(rng, greflect(D, N), 1.0f - m4.x * m4.y);
              att = na;
              O = add(P, muls(N, kBIAS));
              D = rd;
              bounce++;
            }
            if (inner) {
              // intersection_info leaves N,P untouched on a miss: keep them for the
              // inner hit in LDS rather than across the traversal in registers
              phase = 1;
              s_pix[9][tid] = N.x; s_pix[10][tid] = N.y; s_pix[11][tid] = N.z;
              s_pix[15][tid] = P.x; s_pix[16][tid] = P.y; s_pix[17][tid] = P.z;
            }
            else if (bounce >= B) done = true;   // budget exhausted: black (res = 0)
          } else {
            res = total;                          // emissive: end of path
            done = true;
          }
        }
      } else {
        // inner traversal of the refraction branches (montecarlo.frag:148-152 / 162-165)
        if (h.hit()) {
          geom_info<COUNT>(s, h, N, P, ev);
        } else {
          N = mk(s_pix[9][tid], s_pix[10][tid], s_pix[11][tid]);
          P = mk(s_pix[15][tid], s_pix[16][tid], s_pix[17][tid]);
        }
        O = add(P, muls(N, kBIAS));
        D = grefract(D, neg(N), p.inv_ior, kIorConst ? p.inv_ior_sq : p.inv_ior * p.inv_ior);
        phase = 0;
        bounce++;
        if (bounce >= B) done = true;
      }
    }
    if (done) {
      add_pass(res);
      ev.inc(EV_SAMPLE);
      pass++;
      next_chunk();
      rng = pix_seed(pass);   // = (u, v)
      O = Ocam; D = mk(s_pix[0][pj], s_pix[1][pj], s_pix[2][pj]);
      att = mk(0.8f, 0.8f, 0.8f); total = mk(0.0f, 0.0f, 0.0f);
      bounce = 0; phase = 0;
    }
#ifdef MCPT_STAMPS
    st_s += __builtin_amdgcn_s_memtime();
#endif
  }
#ifdef MCPT_STAMPS
  {
    // diagnostic build (tools/stamps.py; frames whose tiles are all inside the image): wave
    // totals = the last-finishing lane's sums (max over lanes), lane-iterations summed
    unsigned long long vals[6] = {__builtin_amdgcn_s_memtime() - st_k0, st_p, st_t, st_s, st_it, ev.st_leaf};
    unsigned long long it_sum = st_it, lit = ev.st_lit, wit = ev.st_wit;
    unsigned long long nl = ev.st_nl, nw = ev.st_nw, ll = ev.st_ll, lw = ev.st_lw;
    for (int off = 32; off > 0; off >>= 1) {
      for (int k = 0; k < 6; ++k) { unsigned long long o = __shfl_xor(vals[k], off); vals[k] = vals[k] > o ? vals[k] : o; }
      it_sum += __shfl_xor(it_sum, off);
      lit += __shfl_xor(lit, off);
      wit += __shfl_xor(wit, off);
      nl += __shfl_xor(nl, off);
      nw += __shfl_xor(nw, off);
      ll += __shfl_xor(ll, off);
      lw += __shfl_xor(lw, off);
    }
    if ((int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1 && p.events) {
      for (int k = 0; k < 5; ++k) atomicAdd(p.events + k, vals[k]);
      atomicAdd(p.events + 5, it_sum);
      atomicAdd(p.events + 6, 1ull);
      atomicAdd(p.events + 7, vals[5]);
      atomicAdd(p.events + 9, lit);
      atomicAdd(p.events + 10, wit);
      atomicAdd(p.events + 11, nl);
      atomicAdd(p.events + 12, nw);
      atomicAdd(p.events + 13, ll);
      atomicAdd(p.events + 14, lw);
    }
  }
#endif

  if constexpr (kSplit) {   // (one wave: its LDS operations are in order)
    if (steal && p.events && (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1 && s_stolen)
      atomicAdd(p.events + kDebugStealSlot, (unsigned long long)s_stolen);
  }
  if (p.item_cost && (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1) {
    // this item's cost for the next launch's order: its longest wave (100 MHz ticks)
    unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_item0;
    if (kSplit && piece >= 0) dt *= kSplitPieces;   // a piece stands for its whole item
    if (seg_only >= 0) dt *= (unsigned)p.seg_per_item;
    atomicMax(p.item_cost + item, dt < 0xffffffffull ? (unsigned)dt : 0xffffffffu);
  }
#ifdef MCPT_BLOCKTIMES
  {
    const unsigned long long bt1 = __builtin_amdgcn_s_memrealtime();
    const int lead = __builtin_ffsll((long long)__ballot(1)) - 1, k = (int)__lane_id() - lead;
    // (launches of more waves than the buffer holds drop the later waves' pairs)
    const unsigned long long slot = 2ull * ((unsigned long long)blockIdx.x * (TT / 64) + wave) + k;
    if ((k == 0 || k == 1) && p.events && slot < kBlockTimeSlots)   // two lanes, one value each (vector stores)
      p.events[kBlockTimeBase + slot] = k ? bt1 : bt0;
  }
#endif
#ifdef MCPT_LANESTATS
  if (ls_lead() && p.events)
    for (int k = 0; k < LS_COUNT; ++k) atomicAdd(p.events + 16 + k, (unsigned long long)ls_row()[k]);
#endif
  if (COUNT) {
#pragma unroll
    for (int e = 0; e < EV_COUNT; ++e) {
      unsigned long long vsum = ev.c.v[e];
      for (int off = 32; off > 0; off >>= 1) vsum += __shfl_xor(vsum, off);
      if (lane == 0) atomicAdd(p.events + e, vsum);
    }
  }
}

// accum += seg_0 + seg_1 + ... in chunk order (one thread per pixel channel triple)
// pass-split launches (RenderParams::pass_split): slot k holds pass first_pass + k's value
// (0 + v, as a lane's segment sum starts); each accumulation chunk's passes are summed from 0 in
// pass order, as one lane would have, and the chunk sum is added to the accumulator in chunk
// order: the bits of an unsplit launch
__global__ __launch_bounds__(256) void combine_split_kernel(float* __restrict__ accum, const float* __restrict__ partial,
                                                            long long n_px, int first_pass, int n_passes) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_px) return;
  float a0 = accum[i * 3], a1 = accum[i * 3 + 1], a2 = accum[i * 3 + 2];
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
  for (int k = 0; k < n_passes; ++k) {
    const float* q = partial + ((size_t)k * n_px + i) * 3;
    s0 = s0 + q[0]; s1 = s1 + q[1]; s2 = s2 + q[2];
    const int pass = first_pass + k;
    if (k + 1 == n_passes || floordiv(pass - 1, kPassChunk) != floordiv(pass, kPassChunk)) {   // chunk ends
      a0 = a0 + s0; a1 = a1 + s1; a2 = a2 + s2;
      s0 = 0.0f; s1 = 0.0f; s2 = 0.0f;
    }
  }
  accum[i * 3] = a0; accum[i * 3 + 1] = a1; accum[i * 3 + 2] = a2;
}

__global__ __launch_bounds__(256) void combine_kernel(float* __restrict__ accum, const float* __restrict__ partial,
                                                      long long n_px, int n_seg) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_px) return;
  float a0 = accum[i * 3], a1 = accum[i * 3 + 1], a2 = accum[i * 3 + 2];
  for (int s = 0; s < n_seg; ++s) {
    const float* q = partial + ((size_t)s * n_px + i) * 3;
    a0 = a0 + q[0]; a1 = a1 + q[1]; a2 = a2 + q[2];
  }
  accum[i * 3] = a0; accum[i * 3 + 1] = a1; accum[i * 3 + 2] = a2;
}

// combine_kernel for launches with split items (mesh kernels; one segment per item, full
// 32-pass segments): a split segment's sum is piece 0's sum, then the later pieces' stored
// pass values added in pass order (the sequence one lane would have summed)
__global__ __launch_bounds__(256) void combine_items_kernel(float* __restrict__ accum, const float* __restrict__ partial,
                                                            long long n_px, int n_seg, int W, int TW,
                                                            const int* __restrict__ split_of,
                                                            const float* __restrict__ split_pass, int split_max,
                                                            unsigned long long* ev) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_px) return;
  const int lr = (int)(i / W), x = (int)(i - (long long)lr * W);
  const int tiles_x = (W + TW - 1) / TW;
  const int tile = (lr / kTileH) * tiles_x + x / TW;
  const int t = (((lr % kTileH) / 8) * (TW / 8) + (x % TW) / 8) * 64 + (lr % 8) * 8 + (x % 8);   // its thread
  constexpr int p1 = kPassChunk / kSplitPieces;   // piece 1's first pass within the segment
  float a0 = accum[i * 3], a1 = accum[i * 3 + 1], a2 = accum[i * 3 + 2];
  for (int s = 0; s < n_seg; ++s) {
    const float* q = partial + ((size_t)s * n_px + i) * 3;
    float s0 = q[0], s1 = q[1], s2 = q[2];
    const int j = split_of[(size_t)tile * n_seg + s];
    if (j >= 0 && idx_ok(ev, CK_COMBINE_SPLIT, j, split_max)) {
      for (int k = 0; k < kPassChunk - p1; ++k) {
        const float* v = split_pass + (((size_t)j * kPassChunk + k) * kTileThreads + t) * 3;
        s0 = s0 + v[0]; s1 = s1 + v[1]; s2 = s2 + v[2];
      }
    }
    a0 = a0 + s0; a1 = a1 + s1; a2 = a2 + s2;
  }
  accum[i * 3] = a0; accum[i * 3 + 1] = a1; accum[i * 3 + 2] = a2;
}

// launches with pass stealing (RenderParams::steal_vals): every pass's value is stored; per pixel
// and segment the passes are summed from 0 in pass order (as the lane's segment sum was), and the
// segment sums are added to the accumulator in segment order — the bits of combine_items_kernel's
// launches (one segment per item, full 32-pass segments)
__global__ __launch_bounds__(256) void combine_steal_kernel(float* __restrict__ accum, long long n_px, int n_seg,
                                                            int W, int TW, const float* __restrict__ vals) {
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n_px) return;
  const int lr = (int)(i / W), x = (int)(i - (long long)lr * W);
  const int tiles_x = (W + TW - 1) / TW;
  const int tile = (lr / kTileH) * tiles_x + x / TW;
  const int t = (((lr % kTileH) / 8) * (TW / 8) + (x % TW) / 8) * 64 + (lr % 8) * 8 + (x % 8);   // its thread
  float a0 = accum[i * 3], a1 = accum[i * 3 + 1], a2 = accum[i * 3 + 2];
  for (int s = 0; s < n_seg; ++s) {
    const size_t item = (size_t)tile * n_seg + s;
    float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
    for (int k = 0; k < kPassChunk; ++k) {
      const float* v = vals + ((item * kPassChunk + k) * kTileThreads + t) * 3;
      s0 = s0 + v[0]; s1 = s1 + v[1]; s2 = s2 + v[2];
    }
    a0 = a0 + s0; a1 = a1 + s1; a2 = a2 + s2;
  }
  accum[i * 3] = a0; accum[i * 3 + 1] = a1; accum[i * 3 + 2] = a2;
}

// ------------------------------------------------------------------------------------
// ray queries: the shader library's traverse_all_bvh / just_hit_bvh / intersect_one_prim /
// hit_one_prim + intersection_info + intersection_color_info / _mat_info
// (raytracer_func.frag:718-781, 874-907) for caller-supplied rays, one lane per ray
// ------------------------------------------------------------------------------------
template <bool ANY, bool MESH>
__global__ __launch_bounds__(256) void trace_kernel(TraceParams q) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= q.n) return;
  SceneT<MESH> s{q.nodes, q.leaves, q.ptype, q.prims, q.depth, q.minfo, q.mpairs, q.mleaftris, q.mtris, q.mverts,
                 q.mnorms, q.flat_face};
  Ev<false> ev;
  const f3 O = mk(q.orig[3 * i], q.orig[3 * i + 1], q.orig[3 * i + 2]);
  const f3 D = mk(q.dir[3 * i], q.dir[3 * i + 1], q.dir[3 * i + 2]);
  Hit h;
  h.pl = mk(0.0f, 0.0f, 0.0f); h.cull2 = 0.0;
  if (q.prim < 0) {
    traverse_lane<false, ANY>(s, O, D, h, ev);
  } else {                                       // intersect_one_prim / hit_one_prim
    h.clear(); h.dist = kFLTMAX; h.cull2 = cull_bound_sq(kFLTMAX);
    prim_test<false, false, ANY>(s, q.prim, O, D, h, ev);
  }
  float* o = q.out + i * kTraceFloats;
  int* oi = q.out_i + i * 3;
  oi[0] = h.hit() ? h.shape() : -1;
  oi[1] = h.hit() ? h.index() : -1;
  oi[2] = !h.hit() ? -1 : (h.shape() == CODE_MESH ? h.tri : h.face());
  f3 N = mk(0.0f, 0.0f, 0.0f), P = N;
  float4 col = make_float4(0.0f, 0.0f, 0.0f, 0.0f), mat = col;
  f3 pg = h.pl;   // (0,0,0) on a miss
  if (h.hit()) {
    const size_t b = (size_t)h.index() * 8;
    pg = xpoint(s.prims[b + 3], s.prims[b + 4], s.prims[b + 5], h.pl);
    geom_info<false>(s, h, N, P, ev);
    col = s.prims[(size_t)h.index() * 8 + 6];
    mat = s.prims[(size_t)h.index() * 8 + 7];
  }
  const float v[kTraceFloats] = {h.hit() ? h.dist : kFLTMAX, h.pl.x, h.pl.y, h.pl.z, pg.x, pg.y, pg.z,
                                 N.x, N.y, N.z, P.x, P.y, P.z, col.x, col.y, col.z, col.w, mat.x, mat.y, mat.z, mat.w};
#pragma unroll
  for (int k = 0; k < kTraceFloats; ++k) o[k] = v[k];
}

// DrawSampling's point cloud (tp/sampling_base.vert:23-26 seeding + tp/hsphere.vert
// random_ray): point k = random_ray(normalize(normal), roughness) with the RNG seeded at
// floatBitsToUint(fseed) + k * nb_used * (11, 43, 67)
__global__ __launch_bounds__(256) void sample_kernel(SampleParams q) {
  const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
  if (k >= q.n) return;
  const uint32_t step = (uint32_t)k * q.nb_used;
  Rng rng;
  rng.x = fbits(q.fseed[0]) + step * 11u;
  rng.y = fbits(q.fseed[1]) + step * 43u;
  rng.z = fbits(q.fseed[2]) + step * 67u;
  const f3 n = normalize3(mk(q.normal[0], q.normal[1], q.normal[2]));
  const f3 r = random_ray(rng, n, q.roughness);
  q.out[3 * k] = r.x; q.out[3 * k + 1] = r.y; q.out[3 * k + 2] = r.z;
}

}  // namespace mcpt


hipError_t mcpt_launch_trace(const mcpt::TraceParams& q, bool any_hit, hipStream_t stream) {
  if (q.n <= 0) return hipSuccess;
  dim3 block(256), grid((unsigned)((q.n + 255) / 256));
  if (q.n_meshes > 0) {
    if (any_hit) hipLaunchKernelGGL((mcpt::trace_kernel<true, true>), grid, block, 0, stream, q);
    else hipLaunchKernelGGL((mcpt::trace_kernel<false, true>), grid, block, 0, stream, q);
  } else {
    if (any_hit) hipLaunchKernelGGL((mcpt::trace_kernel<true, false>), grid, block, 0, stream, q);
    else hipLaunchKernelGGL((mcpt::trace_kernel<false, false>), grid, block, 0, stream, q);
  }
  return hipGetLastError();
}

hipError_t mcpt_launch_sample(const mcpt::SampleParams& q, hipStream_t stream) {
  if (q.n <= 0) return hipSuccess;
  dim3 block(256), grid((unsigned)((q.n + 255) / 256));
  hipLaunchKernelGGL(mcpt::sample_kernel, grid, block, 0, stream, q);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------
// launch wrapper (host)
// ------------------------------------------------------------------------------------
hipError_t mcpt_launch_render(const mcpt::RenderParams& p, bool count, hipStream_t stream) {
  const int K = p.seg_per_item > 1 ? p.seg_per_item : 1;
  const long long items = (long long)p.n_tiles * ((p.n_segments + K - 1) / K);
  if (items <= 0) return hipSuccess;
  // split items: spare workgroups for the most pieces (the kernel skips the unused ones)
  const long long blocks = items + (p.split_of ? (long long)p.split_max * (mcpt::kSplitPieces - 1) : 0) +
                           (long long)p.tail_m * (K - 1);
  dim3 block(p.tile_w * mcpt::kTileH), grid((unsigned)blocks);
  const bool wave = p.wave_traversal != 0, mesh = p.n_meshes > 0;
  const bool lds = p.lds_scene_bytes > 0;
  if (p.tile_w != mcpt::tile_w_for(mesh, p.lds_scene_bytes)) return hipErrorInvalidValue;   // (launch() sets it)
  // deep-BVH walk kernel: suspendable walks and/or batched leaf visits (walk_run)
  const bool susp = !count && !wave && (p.walk_exit > 0 || p.leaf_batch > 0);
  const size_t shm = lds ? (size_t)p.lds_scene_bytes : 0;
#define MCPT_RENDER(C, W, M, L, S, T) \
  hipLaunchKernelGGL((mcpt::render_kernel<C, W, M, L, S, T>), grid, block, shm, stream, p)
#define MCPT_RENDER_CW(C, W, S)                                          \
  if (mesh && lds) MCPT_RENDER(C, W, true, true, S, 8);                  \
  else if (mesh) MCPT_RENDER(C, W, true, false, S, 8);                   \
  else if (lds && p.tile_w == 16) MCPT_RENDER(C, W, false, true, S, 16); \
  else if (lds) MCPT_RENDER(C, W, false, true, S, 32);                   \
  else MCPT_RENDER(C, W, false, false, S, 16)
  if (count) {
    if (wave) { MCPT_RENDER_CW(true, true, false); } else { MCPT_RENDER_CW(true, false, false); }
  } else if (wave) {
    MCPT_RENDER_CW(false, true, false);
  } else if (susp) {
    MCPT_RENDER_CW(false, false, true);
  } else {
    MCPT_RENDER_CW(false, false, false);
  }
#undef MCPT_RENDER_CW
#undef MCPT_RENDER
  return hipGetLastError();
}

hipError_t mcpt_launch_combine(const mcpt::RenderParams& p, hipStream_t stream) {
  if (p.n_local_px <= 0) return hipSuccess;
  dim3 block(256), grid((unsigned)((p.n_local_px + 255) / 256));
  if (p.steal_vals) {   // (also for one segment: the render stored passes, no sums)
    hipLaunchKernelGGL(mcpt::combine_steal_kernel, grid, block, 0, stream, p.accum, p.n_local_px, p.n_segments, p.W,
                       p.tile_w, p.steal_vals);
    return hipGetLastError();
  }
  if (p.n_segments <= 1) return hipSuccess;
  if (p.pass_split)
    hipLaunchKernelGGL(mcpt::combine_split_kernel, grid, block, 0, stream, p.accum, p.partial, p.n_local_px,
                       p.first_pass, p.n_passes);
  else if (p.split_of)
    hipLaunchKernelGGL(mcpt::combine_items_kernel, grid, block, 0, stream, p.accum, p.partial, p.n_local_px,
                       p.n_segments, p.W, p.tile_w, p.split_of, p.split_pass, p.split_max, p.events);
  else
    hipLaunchKernelGGL(mcpt::combine_kernel, grid, block, 0, stream, p.accum, p.partial, p.n_local_px, p.n_segments);
  return hipGetLastError();
}
