// mcpt_stream.hip — the stream (wavefront) schedule of the integrator, MCPT_TRAVERSAL_STREAM
// (DESIGN.md §4.3): a second, complete schedule of tp/montecarlo.frag:100-179 with the rays
// compacted into a queue, idle lanes refilled by ballot + mbcnt from an LDS stage and the rays
// ordered by direction octant (the north star's "ray compaction / sort").  Bit-exact against the
// oracle (tests/test_gpu_stream.py); selected only explicitly (mcpt_set_traversal): it measured
// 5 % behind the megakernel on the deepest BVH (scene 8) and 4-7x behind on shallow scenes, so
// AUTO does not time it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mcpt_device.h"

namespace mcpt {

// ------------------------------------------------------------------------------------
// stream schedule (MCPT_TRAVERSAL_STREAM): wavefront path tracing for deep
// BVHs.  A pool of path slots each runs one (pixel, pass segment) unit at a time, its passes
// in order (the unit's sum is the megakernel's segment sum, so the bits are the same).  The
// rays travel through a queue of payloads (ray, path state, then hit record); an iteration is
//   stream_trace_kernel: persistent waves claim chunks of the queue, stage their live rays in
//     LDS and walk them with the per-lane DFS; a lane whose walk ends takes the next staged ray
//     at the wave's next refill point (no lane waits for the wave's longest walk);
//   stream_shade_kernel: one lane per queue entry shades the hit (tp/montecarlo.frag:100-179),
//     ends passes and units, takes new units, and writes the entry's next payload (in place,
//     or appended when the host asks for compaction).
// Each path's sequence of operations is the megakernel's (same traversal, same shading, same
// RNG draws, same sums): only the interleaving across paths changes.
// ------------------------------------------------------------------------------------
constexpr uint32_t kPhaseInner = 1, kPhasePrimary = 2;
constexpr int kStreamBlock = 256, kStreamWaves = kStreamBlock / 64;   // stream kernels' workgroups
constexpr int kMinWavesStream = 8;
// the mesh trace kernel (walk_run_mesh: the mesh walk state and mesh-space ray): as the mesh
// megakernel, 5 waves/SIMD
constexpr int kMinWavesStreamMesh = 5;
// the shade kernel streams payloads from HBM: occupancy over registers
constexpr int kMinWavesShade = 5;
// queue entries a trace wave claims (one atomic) and stages in LDS at once
constexpr int kStreamChunk = 128;
// trace waves stage each claimed chunk in order of the rays' direction octants (+2-4 %)
static_assert(kStreamChunk % 64 == 0, "chunks are staged 64 entries per step");

// Field columns through a buffer resource: the column offset f * n * 4 is a wave-uniform
// scalar (soffset) and the entry offset i * 4 one 32-bit VGPR shared by every field, so no
// 64-bit per-lane address is formed or kept per field (with plain pointers the compiler
// strength-reduced ~40 columns into live 64-bit addresses and spilled them).  Buffers stay
// below 2 GiB (host check).  0x00020000: the gfx9 raw-buffer descriptor word 3.
// Queue payloads are streamed once per iteration: their loads and stores carry the
// non-temporal hint (aux bit 1: nt on gfx950) so that they do not evict the
// BVH records the walks read through L2.
constexpr int kQueueAux = 2;
template <int AUX>
struct ColsT {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t col_bytes;   // one column: n * 4 bytes
  __device__ __forceinline__ uint32_t ldu(int f, uint32_t i) const {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(i * 4u), (int)((uint32_t)f * col_bytes), AUX);
  }
  __device__ __forceinline__ float ld(int f, uint32_t i) const { return __uint_as_float(ldu(f, i)); }
  __device__ __forceinline__ void setu(int f, uint32_t i, uint32_t v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, rs, (int)(i * 4u), (int)((uint32_t)f * col_bytes), AUX);
  }
  __device__ __forceinline__ void set(int f, uint32_t i, float v) const { setu(f, i, __float_as_uint(v)); }
  __device__ __forceinline__ f3 ld3(int f, uint32_t i) const { return mk(ld(f, i), ld(f + 1, i), ld(f + 2, i)); }
  __device__ __forceinline__ void set3(int f, uint32_t i, f3 v) const {
    set(f, i, v.x); set(f + 1, i, v.y); set(f + 2, i, v.z);
  }
};
typedef ColsT<kQueueAux> Cols;   // queue payloads
typedef ColsT<0> SlotCols;       // per-unit slot data (read and written at pass ends: cached)
template <int AUX = kQueueAux>
__device__ __forceinline__ ColsT<AUX> cols(float* base, int n, int n_fields) {
  ColsT<AUX> c;
  c.col_bytes = (uint32_t)n * 4u;
  c.rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)((uint32_t)n_fields * c.col_bytes), 0x00020000);
  return c;
}

// a unit = (pass segment, local pixel): its pixel and its pass range in this launch
struct UnitGeom { int x, y, px, seg, pass_begin, pass_end; };
__device__ __forceinline__ UnitGeom unit_geom(const RenderParams& p, uint32_t unit) {
  UnitGeom g;
  const uint32_t npx = (uint32_t)p.n_local_px;
  g.seg = (int)(unit / npx);
  g.px = (int)(unit - (uint32_t)g.seg * npx);
  const int lr = g.px / p.W;
  g.x = g.px - lr * p.W;
  g.y = p.rows[lr];
  const int c = floordiv(p.first_pass - 1, kPassChunk) + g.seg;
  g.pass_begin = max(p.first_pass, c * kPassChunk + 1);
  g.pass_end = min(p.first_pass + p.n_passes, (c + 1) * kPassChunk + 1);
  return g;
}

// a queue entry's path state besides the ray and the hit
struct Payload {
  f3 O, D, att, total;
  Rng rng;
  uint32_t state, pass, unit;
};
__device__ __forceinline__ void put_payload(const Cols& Q, uint32_t i, const Payload& pl, int slot) {
  Q.set3(QF_OX, i, pl.O); Q.set3(QF_DX, i, pl.D); Q.set3(QF_AX, i, pl.att); Q.set3(QF_TX, i, pl.total);
  Q.setu(QF_RX, i, pl.rng.x); Q.setu(QF_RY, i, pl.rng.y); Q.setu(QF_RZ, i, pl.rng.z);
  Q.setu(QF_STATE, i, pl.state); Q.setu(QF_PASS, i, pl.pass); Q.setu(QF_UNIT, i, pl.unit);
  Q.setu(QF_SLOT, i, (uint32_t)slot);
}
// a slot starts `unit`: its camera ray goes to the primary traversal, its sum to 0
__device__ __forceinline__ void start_unit(const RenderParams& p, const SlotCols& S, int slot, uint32_t unit,
                                           Payload& pl) {
  const UnitGeom g = unit_geom(p, unit);
  pl.O = mk(p.ox, p.oy, p.oz);
  pl.D = camera_dir(p, ((float)g.x + 0.5f) / (float)p.W, ((float)g.y + 0.5f) / (float)p.H);
  pl.att = mk(0.0f, 0.0f, 0.0f); pl.total = pl.att;
  pl.rng.x = pl.rng.y = pl.rng.z = 0u;
  pl.state = kPhasePrimary << 8;
  pl.pass = (uint32_t)g.pass_begin;
  pl.unit = unit;
  S.set3(SF_SX, (uint32_t)slot, mk(0.0f, 0.0f, 0.0f));
}

// the pool's slot i starts unit unit_base + i (the host sizes the pools so that every slot has one)
__global__ __launch_bounds__(256) void stream_init_kernel(StreamParams q) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {
    q.ctr[SC_CNT] = (unsigned)q.n_slots;
    q.ctr[SC_CNT + 1] = 0u;
    q.ctr[SC_FETCH] = 0u;
    q.ctr[SC_FETCH + 1] = 0u;
    q.ctr[SC_DEAD] = 0u;
  }
  if (i >= q.n_slots) return;
  const Cols Q = cols(q.queue[0], q.n_slots, QF_COUNT);
  const SlotCols S = cols<0>(q.slots, q.n_slots, SF_COUNT);
  Payload pl;
  start_unit(q.r, S, i, (uint32_t)(q.unit_base + i), pl);
  put_payload(Q, (uint32_t)i, pl, i);
}

// The traversal half of an iteration: every live entry's ray walked with the per-lane DFS of
// walk_run (right child first, cull at push time, batched leaf visits), its hit record stored
// in the entry.  Persistent waves: a wave claims kStreamChunk entries with one atomic, stages
// their rays in LDS (dead entries dropped), and whenever it leaves walk_run (at <= q.refill
// walking lanes) its idle lanes take the next staged rays — LDS reads, so a refill waits on
// no memory load.
// LDSN: the BVH nodes and leaf ids live in the workgroup's LDS (copied once per persistent
// workgroup; one 1024-thread workgroup per CU, 4 waves/SIMD), so the walk's dependent node
// loads are LDS reads; primitive records stay in global memory.
template <bool LDSN> struct TraceCfg {
  static constexpr int kBlock = 256, kWaves = 4, kChunk = kStreamChunk, kMinWaves = kMinWavesStream;
};
template <> struct TraceCfg<true> {
  static constexpr int kBlock = 1024, kWaves = 16, kChunk = 64, kMinWaves = 4;
};
// LDS of the LDSN trace kernel besides its scene copy: the waves' staged rays
constexpr int kTraceLdsStaging = TraceCfg<true>::kWaves * TraceCfg<true>::kChunk * 32;

// MESH: scenes with triangle-mesh instances, the walk of walk_run_mesh (suspended at <= refill
// walking lanes like walk_run), the hit's triangle kept in the entry
template <bool LDSN, bool MESH>
__global__ __launch_bounds__(TraceCfg<LDSN>::kBlock, MESH ? kMinWavesStreamMesh : TraceCfg<LDSN>::kMinWaves)
void stream_trace_kernel(StreamParams q) {
  typedef TraceCfg<LDSN> C;
  constexpr int kChunkT = C::kChunk;
  const RenderParams& p = q.r;
  SceneT<MESH, false> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mpairs, p.mleaftris,
                        p.mtris, p.mverts, p.mnorms, p.flat_face};
  if constexpr (LDSN) {
    extern __shared__ float4 s_bvh[];
    const int n_nodes = (2 << p.depth) - 1, n_leaves = 1 << p.depth;
    for (int k = threadIdx.x; k < 3 * n_nodes; k += C::kBlock) s_bvh[k] = p.nodes[k];
    int* s_leaf = (int*)(s_bvh + 3 * n_nodes);
    for (int k = threadIdx.x; k < n_leaves; k += C::kBlock) s_leaf[k] = p.leaves[k];
    __syncthreads();
    s.nodes = s_bvh;
    s.leaves = s_leaf;
  }
  const int par = q.parity;
  const unsigned n = q.ctr[SC_CNT + par];
  if (blockIdx.x == 0 && threadIdx.x == 0) q.ctr[SC_CNT + (par ^ 1)] = 0u;   // the shade kernel's output length
  unsigned* fetch = q.ctr + SC_FETCH + par;
  const Cols Q = cols(q.queue[par], q.n_slots, QF_COUNT);
  __shared__ float4 s_ro[C::kWaves][kChunkT], s_rd[C::kWaves][kChunkT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4* ro = s_ro[wave];   // staged rays: (O, queue index bits), (D, 0)
  float4* rd = s_rd[wave];
  int live = 0, cc = 0;      // wave-uniform: staged rays of the current chunk, first unserved
  bool more = true;          // wave-uniform: the queue may hold unclaimed entries
  Ev<false> ev;
  ev.init();
  // idle lanes take staged rays into slot (r, O, D, h, w); an empty stage claims and stages
  // the next chunk
  auto take = [&](int& r, f3& O, f3& D, Hit& h, Walk& w) {
    for (;;) {
      const uint64_t need = __ballot(r < 0);
      if (!need) break;
      if (cc == live) {
        if (!more) break;
        unsigned b = 0;
        if (lane == 0) b = atomicAdd(fetch, (unsigned)kChunkT);
        b = (unsigned)__shfl((int)b, 0);
        if (b >= n) {
          more = false;
          break;
        }
        const unsigned e = min(b + (unsigned)kChunkT, n);
        live = 0;
        cc = 0;
        // the chunk's live entries (neighbouring pixels' rays), staged in order of the
        // direction octant: lanes that take consecutive staged rays then
        // walk rays of one octant from nearby origins, which visit the same nodes and take the
        // same branches
        constexpr int G = kChunkT / 64;
        float4 eo[G], ed[G];
        int key[G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const unsigned idx = b + (unsigned)(g * 64) + (unsigned)lane;
          const int slot = idx < e ? (int)Q.ldu(QF_SLOT, idx) : -1;
          eo[g] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(idx));
          ed[g] = eo[g];
          key[g] = 8;   // dead / beyond the queue: not staged
          if (slot >= 0) {
            eo[g].x = Q.ld(QF_OX, idx); eo[g].y = Q.ld(QF_OY, idx); eo[g].z = Q.ld(QF_OZ, idx);
            ed[g].x = Q.ld(QF_DX, idx); ed[g].y = Q.ld(QF_DY, idx); ed[g].z = Q.ld(QF_DZ, idx);
            key[g] = (ed[g].x < 0.0f) | ((ed[g].y < 0.0f) << 1) | ((ed[g].z < 0.0f) << 2);
          }
        }
#pragma unroll
        for (int o = 0; o < 8; ++o) {
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const bool mine = key[g] == o;
            const uint64_t m = __ballot(mine);
            if (mine) {
              const int pos = live + mbcnt64(m);
              ro[pos] = eo[g];
              rd[pos] = ed[g];
            }
            live += __builtin_popcountll(m);
          }
        }
        __builtin_amdgcn_wave_barrier();
        continue;
      }
      const int k = mbcnt64(need);
      const int avail = live - cc;
      if (r < 0 && k < avail) {
        const float4 a = ro[cc + k], d = rd[cc + k];
        r = (int)__float_as_uint(a.w);
        O = mk(a.x, a.y, a.z);
        D = mk(d.x, d.y, d.z);
        walk_begin<false>(s, D, h, w, ev, p.cull2_max);
      }
      cc += min(__builtin_popcountll(need), avail);
    }
  };
  auto put_hit = [&](int r, const Hit& h) {
    Q.set3(QF_HX, (uint32_t)r, h.pl);
    Q.setu(QF_HCODE, (uint32_t)r, (uint32_t)h.code);
    if constexpr (MESH) Q.setu(QF_HTRI, (uint32_t)r, (uint32_t)h.tri);
  };
  int r = -1;                // queue index of this lane's ray
  f3 O = mk(0.0f, 0.0f, 0.0f), D = O;
  Hit h;
  h.pl = O; h.dist = kFLTMAX; h.clear(); h.tri = 0; h.cull2 = 0.0;
  Walk w;
  w.invD = O; w.node = 0; w.level = 0; w.pending = 0; w.mpf = 0;
  for (;;) {
    take(r, O, D, h, w);
    if (__ballot(r >= 0) == 0) break;   // nothing staged and nothing left to claim
    if (r >= 0) {
      bool ended;
      if constexpr (MESH) ended = walk_run_mesh<false, true>(s, O, D, h, w, ev, q.refill);
      else ended = walk_run<false, true>(s, O, D, h, w, ev, q.refill, p.leaf_batch);
      if (ended) {
        put_hit(r, h);
        r = -1;
      }
    }
  }
#ifdef MCPT_STAMPS
  // diagnostic build (tools/stamps.py --stream): the walk loop's iterations and lane counts of
  // this wave's whole life, summed over the wave's lanes (walk_run's counters), into the debug slots
  {
    unsigned long long v[7] = {ev.st_lit, ev.st_wit, ev.st_nl, ev.st_nw, ev.st_ll, ev.st_lw, ev.st_leaf};
    for (int off = 32; off > 0; off >>= 1)
      for (int k = 0; k < 6; ++k) v[k] += __shfl_xor(v[k], off);
    for (int off = 32; off > 0; off >>= 1) { const unsigned long long o = __shfl_xor(v[6], off); v[6] = v[6] > o ? v[6] : o; }
    if (lane == 0 && p.events) {
      for (int k = 0; k < 6; ++k) atomicAdd(p.events + 9 + k, v[k]);
      atomicAdd(p.events + 7, v[6]);
      atomicAdd(p.events + 6, 1ull);
    }
  }
#endif
}

// The shading half for queue entry i (slot `slot`): the hit through tp/montecarlo.frag:100-179
// (the megakernel's shading block, variant montecarlo.frag).  A path that ends adds its result
// to the unit's sum in pass order and the slot goes on with the unit's next pass, whose camera
// ray is the cached primary hit (shaded at once, no traversal); a unit that ends writes its
// sum and the slot takes the next unit.  Returns true with the next payload in `out` when the
// slot's next ray must be traversed, false when the slot has no unit left.
template <bool MESH>
__device__ __forceinline__ bool stream_shade(const StreamParams& q, const Cols& Qi, uint32_t i, const SlotCols& Sl,
                                             int slot, Payload& out) {
  const RenderParams& p = q.r;
  const SceneT<MESH, false> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mpairs, p.mleaftris,
                              p.mtris, p.mverts, p.mnorms, p.flat_face};
  Ev<false> ev;
  ev.init();
  const uint32_t sidx = (uint32_t)slot;
  uint32_t unit = Qi.ldu(QF_UNIT, i);
  const UnitGeom g = unit_geom(p, unit);
  const uint32_t sw = Qi.ldu(QF_STATE, i);
  int bounce = (int)(sw & 255u);
  uint32_t phase = sw >> 8;
  int pass = (int)Qi.ldu(QF_PASS, i);
  const int B = p.bounces;
  const f3 Ocam = mk(p.ox, p.oy, p.oz);
  Hit h;
  h.pl = Qi.ld3(QF_HX, i); h.code = (int)Qi.ldu(QF_HCODE, i); h.dist = 0.0f; h.cull2 = 0.0;
  h.tri = MESH ? (int)Qi.ldu(QF_HTRI, i) : 0;
  f3 O = Qi.ld3(QF_OX, i), D = Qi.ld3(QF_DX, i), att, total, N = mk(0.0f, 0.0f, 0.0f), P = N;
  Rng rng;
  bool first = false;
  const float u = ((float)g.x + 0.5f) / (float)p.W, v = ((float)g.y + 0.5f) / (float)p.H;
  if (phase == kPhasePrimary) {
    // the unit's camera-ray hit, computed once and reused by all its passes (exact: the camera
    // ray has no jitter and traversal / intersection_info draw no random numbers)
    const int key0 = hit_key(h);
    f3 N0 = mk(0.0f, 0.0f, 0.0f), P0 = N0;
    if (h.hit()) geom_info<false>(s, h, N0, P0, ev);
    Sl.set3(SF_N0X, sidx, N0); Sl.set3(SF_P0X, sidx, P0); Sl.setu(SF_KEY0, sidx, (uint32_t)key0);
    phase = 0;
    first = true;
    N = N0; P = P0;
    h.code = key0;
    rng = seed_for(u, v, pass, p.date);   // pass `pass` of the unit starts (O, D: the camera ray)
    att = mk(0.8f, 0.8f, 0.8f); total = mk(0.0f, 0.0f, 0.0f);
    bounce = 0;
  } else {
    att = Qi.ld3(QF_AX, i); total = Qi.ld3(QF_TX, i);
    rng.x = Qi.ldu(QF_RX, i); rng.y = Qi.ldu(QF_RY, i); rng.z = Qi.ldu(QF_RZ, i);
  }
  for (;;) {
    bool done = false;
    f3 res = mk(0.0f, 0.0f, 0.0f);
    if (phase == 0) {
      if (!h.hit()) {
        const float a = gmax(0.0f, D.z);
        res = add(total, mulv(att, gmix3(mk(0.5f, 0.5f, 0.9f), mk(1.0f, 1.0f, 0.8f), a)));
        done = true;
      } else {
        if (!first) geom_info<false>(s, h, N, P, ev);
        const float4 c4 = s.prims[(size_t)h.index() * 8 + 6];
        const float4 m4 = s.prims[(size_t)h.index() * 8 + 7];
        if (!(m4.z <= 0.5f)) {   // emissive: the path ends with its emission (no draw, no ray)
          res = add(total, add(muls(mk(c4.x, c4.y, c4.z), 0.1f), muls(muls(muls(att, m4.z), 1.0f - m4.x), c4.w)));
          done = true;
        } else if (bounce >= B - 1) {   // every branch reaches the budget: black (MCPT_FOLD_END)
          done = true;
        } else {
          f3 ray = random_ray(rng, N, 1.0f - m4.y);
          const f3 col = mk(c4.x, c4.y, c4.z);
          const float alpha = c4.w;
          const float rs = schlick(p.schlick_r0, D, N);
          const f3 R = greflect(neg(ray), N);
          const f3 E = normalize3(sub(O, P));
          const float se = gmix(100.0f, 2.0f, m4.y);
          const float spec = mc_pow_le1(gmax(0.0f, dot3(E, R)), se);
          total = add(total, add(muls(col, 0.1f), muls(muls(muls(att, m4.z), 1.0f - m4.x), alpha)));
          const f3 mx = gmix3(att, col, m4.x);
          const f3 base = mulv(col, att);
          bool reflect_push = false, inner = false;
          if (m4.x > 0.0f && alpha == 1.0f) {
            reflect_push = true;
          } else if (alpha < 1.0f && m4.x == 0.0f) {
            inner = true;
            att = add(base, mulv(muls(muls(muls(att, 1.0f - alpha), 1.0f - rs), spec), mx));
            O = sub(P, muls(N, kBIAS));
            D = grefract(D, N, p.ior);
          } else if (alpha < 1.0f && m4.x > 0.0f) {
            const float rc = rnd(rng);
            if (rc > 0.5f) {
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
            const f3 na = add(base, mulv(muls(muls(muls(att, alpha), rs), spec), mx));
            const f3 rd = random_ray(rng, greflect(D, N), 1.0f - m4.x * m4.y);
            att = na;
            O = add(P, muls(N, kBIAS));
            D = rd;
            bounce++;
          }
          if (inner) {   // intersection_info leaves N, P untouched on a miss: kept for the inner hit
            phase = kPhaseInner;
            Sl.set3(SF_NSX, sidx, N); Sl.set3(SF_PSX, sidx, P);
          }
        }
      }
    } else {
      // inner traversal of the refraction branches (montecarlo.frag:148-152 / 162-165)
      if (h.hit()) {
        geom_info<false>(s, h, N, P, ev);
      } else {
        N = Sl.ld3(SF_NSX, sidx); P = Sl.ld3(SF_PSX, sidx);
      }
      O = add(P, muls(N, kBIAS));
      D = grefract(D, neg(N), p.inv_ior);
      phase = 0;
      bounce++;
      if (bounce >= B) done = true;   // budget exhausted: black
    }
    if (!done) {   // the path goes on: its next ray is queued
      out.O = O; out.D = D; out.att = att; out.total = total; out.rng = rng;
      out.state = (uint32_t)bounce | (phase << 8);
      out.pass = (uint32_t)pass;
      out.unit = unit;
      return true;
    }
    f3 sum = Sl.ld3(SF_SX, sidx);
    sum = mk(sum.x + res.x, sum.y + res.y, sum.z + res.z);
    pass++;
    if (pass >= g.pass_end) {   // the unit's sum: accumulator (one-segment launch) or its segment slot
      if (p.n_segments == 1) {
        float* accp = p.accum + (size_t)g.px * 3;
        accp[0] = accp[0] + sum.x; accp[1] = accp[1] + sum.y; accp[2] = accp[2] + sum.z;
      } else {
        float* part = p.partial + ((size_t)g.seg * p.n_local_px + g.px) * 3;
        part[0] = sum.x; part[1] = sum.y; part[2] = sum.z;
      }
      unit = atomicAdd(q.unit_ctr, 1u);
      if (unit >= q.n_units) {
        atomicAdd(q.ctr + SC_DEAD, 1u);
        return false;
      }
      start_unit(p, Sl, slot, unit, out);
      return true;
    }
    Sl.set3(SF_SX, sidx, sum);
    // the unit's next pass starts with the cached primary hit
    h.code = (int)Sl.ldu(SF_KEY0, sidx);
    N = Sl.ld3(SF_N0X, sidx); P = Sl.ld3(SF_P0X, sidx);
    first = true;
    phase = 0;
    rng = seed_for(u, v, pass, p.date);
    O = Ocam; D = camera_dir(p, u, v);
    att = mk(0.8f, 0.8f, 0.8f); total = mk(0.0f, 0.0f, 0.0f);
    bounce = 0;
  }
}

template <bool MESH>
__global__ __launch_bounds__(kStreamBlock, kMinWavesShade) void stream_shade_kernel(StreamParams q) {
  const int par = q.parity;
  const unsigned n = q.ctr[SC_CNT + par];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    q.ctr[SC_FETCH + (par ^ 1)] = 0u;                // the next trace kernel's fetch counter
    if (!q.compact) q.ctr[SC_CNT + (par ^ 1)] = n;   // in place: the same length
  }
  const Cols Qi = cols(q.queue[par], q.n_slots, QF_COUNT), Qo = cols(q.queue[par ^ 1], q.n_slots, QF_COUNT);
  const SlotCols Sl = cols<0>(q.slots, q.n_slots, SF_COUNT);
  __shared__ unsigned s_wc[kStreamWaves + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (unsigned base = blockIdx.x * (unsigned)kStreamBlock; base < n; base += gridDim.x * (unsigned)kStreamBlock) {   // block-uniform
    const unsigned i = base + threadIdx.x;
    const int slot = i < n ? (int)Qi.ldu(QF_SLOT, i) : -1;
    Payload pl;
    const bool cont = slot >= 0 && stream_shade<MESH>(q, Qi, i, Sl, slot, pl);
    if (!q.compact) {   // in place: entry i of the next queue (dead entries marked)
      if (cont) put_payload(Qo, i, pl, slot);
      else if (i < n) Qo.setu(QF_SLOT, i, 0xFFFFFFFFu);
    } else {            // compaction: live entries appended (one atomic per block)
      const uint64_t m = __ballot(cont);
      if (lane == 0) s_wc[wave] = (unsigned)__builtin_popcountll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned t = 0;
        for (int k = 0; k < kStreamWaves; ++k) { const unsigned c = s_wc[k]; s_wc[k] = t; t += c; }
        s_wc[kStreamWaves] = t ? atomicAdd(q.ctr + SC_CNT + (par ^ 1), t) : 0u;
      }
      __syncthreads();
      if (cont) put_payload(Qo, s_wc[kStreamWaves] + s_wc[wave] + (unsigned)mbcnt64(m), pl, slot);
      __syncthreads();
    }
  }
}

}  // namespace mcpt

hipError_t mcpt_launch_stream_init(const mcpt::StreamParams& q, hipStream_t stream) {
  if (q.n_slots <= 0) return hipSuccess;
  dim3 block(256), grid((unsigned)((q.n_slots + 255) / 256));
  hipLaunchKernelGGL(mcpt::stream_init_kernel, grid, block, 0, stream, q);
  return hipGetLastError();
}

int mcpt_stream_lds_nodes_bytes(int depth) {
  return (3 * ((2 << depth) - 1)) * 16 + (1 << depth) * 4;
}
bool mcpt_stream_lds_nodes_fit(int depth) {
  return depth <= 12 && mcpt_stream_lds_nodes_bytes(depth) + mcpt::kTraceLdsStaging <= 160 * 1024;
}

hipError_t mcpt_launch_stream_iter(const mcpt::StreamParams& q, int n_cu, bool lds_nodes, hipStream_t stream) {
  hipError_t e;
  const bool mesh = q.r.n_meshes > 0;
  if (mesh) {
    hipLaunchKernelGGL((mcpt::stream_trace_kernel<false, true>), dim3((unsigned)n_cu * 8), dim3(mcpt::kStreamBlock), 0,
                       stream, q);
  } else if (lds_nodes) {
    const size_t shm = (size_t)mcpt_stream_lds_nodes_bytes(q.r.depth);
    // above the default 64 KiB of dynamic LDS (set on the calling thread's current device)
    e = hipFuncSetAttribute((const void*)mcpt::stream_trace_kernel<true, false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - mcpt::kTraceLdsStaging);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mcpt::stream_trace_kernel<true, false>), dim3((unsigned)n_cu),
                       dim3(mcpt::TraceCfg<true>::kBlock), shm, stream, q);
  } else {
    hipLaunchKernelGGL((mcpt::stream_trace_kernel<false, false>), dim3((unsigned)n_cu * 8), dim3(mcpt::kStreamBlock), 0,
                       stream, q);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned persistent_blocks = (unsigned)n_cu * 8;
  if (mesh) hipLaunchKernelGGL(mcpt::stream_shade_kernel<true>, dim3(persistent_blocks), dim3(mcpt::kStreamBlock), 0, stream, q);
  else hipLaunchKernelGGL(mcpt::stream_shade_kernel<false>, dim3(persistent_blocks), dim3(mcpt::kStreamBlock), 0, stream, q);
  return hipGetLastError();
}
