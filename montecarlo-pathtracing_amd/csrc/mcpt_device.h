// mcpt_device.h — the device-side building blocks of the path tracer for CDNA4 (gfx950),
// shared by the per-pixel megakernel (mcpt_kernel.hip) and the stream schedule
// (mcpt_stream.hip): scene views, the box / primitive intersections, the stackless per-lane
// and wave-coherent BVH walks (raytracer_func.frag), intersection_info, the roughness-lobe
// sampler and Schlick term (tp/montecarlo.frag), the camera ray (raytracer.vert).  Design notes
// in mcpt_kernel.hip's header and DESIGN.md §4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mcpt_math.h"
#include "mcpt_internal.h"

namespace mcpt {

// math inside the BVH walk loop (primitive tests): the short exact sequences of mcpt_math.h or
// the generic IEEE expansions — same results either way.  The LDS-scene kernels (shallow BVHs)
// take all four short sequences (+2.4 % scene 6, +2 % scenes 1/2/4:
// profiles/r02_ab10_walk_fast_math.jsonl); the L2-read deep-BVH kernels only the normalize
// (+1.2..+5 % on scenes 3/5/7/8; sqrt alone +-0, normalize + sqrt -9..-15 % through register
// allocation: profiles/r02_ab12_l2_fast_math.jsonl).  Bits: 1 normalize, 2 length, 4 sqrt, 8 rcp.
constexpr int kL2Fast = 1;
template <bool FAST>
__device__ __forceinline__ f3 wnormalize3(f3 a) {
  if constexpr (FAST) return normalize3(a); else return normalize3_g(a);
}
template <bool FAST>
__device__ __forceinline__ float wlength3(f3 a) {
  if constexpr (FAST) return length3(a); else return length3_g(a);
}
template <bool FAST>
__device__ __forceinline__ float wsqrt(float x) {
  if constexpr (FAST || kDriverRoots) return sqrt_rn(x); else return __builtin_sqrtf(x);
}
template <bool FAST>
__device__ __forceinline__ float wrcp(float x) {
  if constexpr (FAST || kDriverRoots) return rcp_rn(x); else return 1.0f / x;
}

// Closest-hit record.  The world-space hit point is not kept: it is xpoint(transform of
// `index`, pl), recomputed by geom_info with the same operations accept_cand used (same bits),
// which keeps 3 VGPRs out of the traversal's live state.
//
// The hit's primitive, shape and face are one word, `code` = shape << 28 | face << 24 | index
// (-1: no hit; index < 2^24, mcpt_upload_scene), so the record a walk carries is 7 VGPRs
// (pl, dist, code, cull2).  A mesh hit's face is its mesh-local triangle (`tri`, mesh kernels
// only; the reference's tri_index).
struct Hit {
  f3 pl;
  float dist;
  int code;
  int tri;
  double cull2;   // (midpoint between dist and the next float above)^2, exact in binary64
  __device__ __forceinline__ int shape() const { return code >> 28; }
  __device__ __forceinline__ int index() const { return code & 0x00FFFFFF; }
  __device__ __forceinline__ int face() const { return (code >> 24) & 15; }
  __device__ __forceinline__ bool hit() const { return code >= 0; }
  __device__ __forceinline__ void clear() { code = -1; }
  __device__ __forceinline__ void set(int index, int shape, int face) { code = (shape << 28) | (face << 24) | index; }
};
// (shape, index) of the primary-hit cache: the same word with the face dropped (the cached
// N, P make the face unnecessary)
__device__ __forceinline__ int hit_key(const Hit& h) { return h.hit() ? (h.code & ~0x0F000000) : -1; }

// The BVH cull `length(O - Pg) <= dist` (raytracer_func.frag:351) without the sqrt: for
// binary32 d2 >= 0 and c >= 0, RN(sqrt(d2)) <= c  <=>  sqrt(d2) < m, m = the midpoint
// between c and the next float (sqrt of a binary32 is never exactly such a 25-bit
// midpoint), <=> d2 < m*m, and m*m (<= 52 significant bits) is exact in binary64.
// NaN and +inf d2 compare false on both sides.  Bit-identical decisions, 2 VALU ops
// instead of the ~16-op correctly rounded sqrt.
__device__ __forceinline__ double cull_bound_sq(float c) {
  const float nx = __uint_as_float(__float_as_uint(c) + 1u);
  const double m = ((double)c + (double)nx) * 0.5;
  return m * m;
}

enum { CODE_MESH = 0, CODE_SPHERE = 1, CODE_CUBE = 2, CODE_CYLINDER = 3, CODE_CONE = 4, CODE_QUAD = 5 };

// ------------------------------------------------------------------------------------
// scene views: global memory or LDS-staged copy (same record layout)
// ------------------------------------------------------------------------------------
// MESH: the scene has triangle-mesh instances (CODE_MESH); a compile-time switch so scenes
// without meshes do not pay the mesh code's registers.
// LDS: the node / leaf / primitive arrays were staged into the workgroup's LDS (small
// scenes; render_kernel): plain loads (ds_read), no constant-address-space casts.
template <bool MESH, bool LDS = false>
struct SceneT {
  static constexpr bool kMesh = MESH;
  static constexpr bool kLds = LDS;
  // walk-loop math (wnormalize3, wlength3, wsqrt, wrcp): short exact sequences or generic
  static constexpr int kFast = LDS ? 15 : kL2Fast;
  static constexpr bool kFastNorm = kFast & 1, kFastLen = kFast & 2, kFastSqrt = kFast & 4, kFastRcp = kFast & 8;
  const float4* __restrict__ nodes;   // 3 per node: (c, has-prim) (w, 0) (1/w, 0)
  const int* __restrict__ leaves;
  const int* __restrict__ ptype;      // type code | mesh id << 4
  const float4* __restrict__ prims;   // 8 per prim: inv r0..r2, trf r0..r2, colour, material
  int depth;
  // meshes (mcpt_upload_meshes): per mesh (first pair slot, first leaf, depth, first triangle)
  const int4* __restrict__ minfo;
  // mesh BVHs, mesh space: one 64-byte slot of 4 rows per internal node (slot: mesh_pair_slot,
  // from the mesh's first slot), both children's boxes, (c_left, has_left) (w_left, 0)
  // (c_right, has_right) (w_right, 0)
  const float4* __restrict__ mpairs;
  // 4 rows per mesh leaf at its global leaf index: (A, t) (B - A, 0) (C - A, 0) (0) of the
  // leaf's triangle, t = the mesh-local triangle id as int bits (-1: empty leaf).  In the same
  // allocation as mpairs, after its slots (walk_run_mesh addresses both from mpairs)
  const float4* __restrict__ mleaftris;
  const int4* __restrict__ mtris;     // global vertex ids (a, b, c, 0) (intersection_info)
  const float4* __restrict__ mverts;  // (x, y, z, 0)
  const float4* __restrict__ mnorms;
  int flat_face;                      // uniform flat_face (raytracer_func.frag:26; never set: 0)
};

// Wave-uniform records are read through the constant address space so the compiler emits
// scalar loads (s_load_dwordx4/x8 into SGPRs, scalar cache) instead of per-lane gathers.
typedef float v4f __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) v4f* cv4p;
typedef const __attribute__((address_space(4))) int* cip;

template <bool UNIFORM>
__device__ __forceinline__ float4 ld4(const float4* p, size_t i) {
  if (UNIFORM) {
    v4f v = ((cv4p)(const void*)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return p[i];
}
template <bool UNIFORM>
__device__ __forceinline__ int ld1(const int* p, size_t i) {
  if (UNIFORM) return ((cip)(const void*)p)[i];
  return p[i];
}

__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct Counters {
  uint32_t v[EV_COUNT];
  __device__ __forceinline__ void inc(int e) { v[e]++; }
};

template <bool COUNT>
struct Ev {
  Counters c;
#ifdef MCPT_STAMPS
  unsigned long long st_leaf = 0;   // diagnostic: wave-cycles in the traversal's leaf blocks
  unsigned long long st_lit = 0, st_wit = 0;   // traversal loop: lane iterations, wave iterations
  unsigned long long st_nl = 0, st_ll = 0, st_nw = 0, st_lw = 0;   // node / leaf block lanes, iterations
#endif
  __device__ __forceinline__ void init() { if (COUNT) for (int i = 0; i < EV_COUNT; ++i) c.v[i] = 0; }
  __device__ __forceinline__ void inc(int e) { if (COUNT) c.v[e]++; }
};

#ifdef MCPT_LANESTATS
// Diagnostic build only (tools/lanestats.py; never timed): per-wave lane accounting of the deep
// walk.  The wave's first active lane adds wave-level values (ballot popcounts, iteration counts)
// to its wave's LDS row; render_kernel flushes the rows to the debug slots at its end.
enum {
  LS_NODE_IT, LS_NODE_LN, LS_NE_WV, LS_NE_LN, LS_OUT_WV, LS_OUT_LN, LS_VAL_WV, LS_VAL_LN,
  LS_LEAF_IT, LS_LEAF_LN, LS_PRIM_LN, LS_SPH_WV, LS_SPH_LN, LS_CUBE_WV, LS_CUBE_LN, LS_CYL_WV,
  LS_CYL_LN, LS_QUAD_WV, LS_QUAD_LN, LS_WALK_IT, LS_WALK_LN, LS_WALK_CALLS, LS_ROUNDS, LS_ROUND_LN,
  LS_SHADE_WV, LS_SHADE_LN, LS_RR2_WV, LS_RR2_LN, LS_WAVES, LS_FIT_IT, LS_TWO_IT,
  // walk_run_mesh: the scene-node and scene-leaf blocks (LS_NODE / LS_LEAF count the mesh-node and
  // mesh-leaf blocks there), and the lanes still walking when the wave leaves the walk
  LS_SNODE_IT, LS_SNODE_LN, LS_SLEAF_IT, LS_SLEAF_LN, LS_EXIT_LN, LS_COUNT
};
__device__ __forceinline__ unsigned* ls_row() {
  __shared__ unsigned s_ls[16][LS_COUNT];
  return s_ls[threadIdx.x >> 6];
}
__device__ __forceinline__ bool ls_lead() { return (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1; }
__device__ __forceinline__ void ls_add(int k, unsigned v) { if (ls_lead()) ls_row()[k] += v; }
__device__ __forceinline__ unsigned ls_pop(bool b) { return (unsigned)__builtin_popcountll(__ballot(b)); }
// (lanes, waves) of a per-lane condition: popcount and whether any lane holds it
__device__ __forceinline__ void ls_cond(int k_wv, int k_ln, bool b) {
  const unsigned n = ls_pop(b);
  ls_add(k_wv, n ? 1u : 0u);
  ls_add(k_ln, n);
}
// which stage of box_test a child reaches: 0 empty (not tested), 1 inside, 2 faces (no valid
// face), 3 a valid face (cull compare)
__device__ __forceinline__ int box_stage(float4 a0, float4 a1, float4 a2, f3 O, f3 D, f3 invD) {
  if (a0.w == 0.0f) return 0;
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  if (__builtin_fabsf(Oi.x) < 1.0f && __builtin_fabsf(Oi.y) < 1.0f && __builtin_fabsf(Oi.z) < 1.0f) return 1;
  f3 rD = mulv(invD, w);
  const bool dv[3] = {__builtin_fabsf(Di.x) > kEPS, __builtin_fabsf(Di.y) > kEPS, __builtin_fabsf(Di.z) > kEPS};
  const float o[3] = {Oi.x, Oi.y, Oi.z}, d[3] = {Di.x, Di.y, Di.z}, r[3] = {rD.x, rD.y, rD.z};
  for (int f = 0; f < 6; ++f) {
    const int c0 = f / 2, c1 = (c0 + 1) % 3, c2 = (c0 + 2) % 3;
    const float a = ((f % 2 ? 1.0f : -1.0f) - o[c0]) * r[c0];
    if (dv[c0] && a > kEPS && __builtin_fabsf(o[c1] + a * d[c1]) <= 1.0f && __builtin_fabsf(o[c2] + a * d[c2]) <= 1.0f)
      return 3;
  }
  return 2;
}
#endif

// one face of intersect_bv's loop (raytracer_func.frag:322-345) folded into the running minimum
// al: a = (cd - oa) / da as (cd - oa) * ra (hoisted reciprocal, contract), valid when the axis
// divides (dv), a > EPSILON and the hit lies in the face (|ob + a db| <= 1, |oc + a dc| <= 1).
// `if (a < al) al = a` == min(al, valid ? a : FLT_MAX) for the non-NaN a a valid face has;
// bitwise & keeps the compares in SGPR masks instead of exec-mask branches (+5 %, r01_ab4).
// The two in-face bounds are one compare of their NaN-propagating maximum (v_maximum3_f32):
// maximum(|p|, |q|) <= 1 == (|p| <= 1) & (|q| <= 1) for every p, q, NaN included.  One SGPR
// mask op fewer per face, same VALU count: C4 shape +2.3 %, C2 +1.2..1.7 %, scene 3 +0.5 %
// (profiles/r04_ab_face_max3.jsonl).
template <bool FIRST = false>
__device__ __forceinline__ float box_face(float al, float cd, float oa, bool dv, float ra, float ob, float db,
                                          float oc, float dc) {
  const float a = (cd - oa) * ra;
  const bool ok = dv & (a > kEPS) &
                  (__builtin_elementwise_maximum(__builtin_fabsf(ob + a * db), __builtin_fabsf(oc + a * dc)) <= 1.0f);
  // FIRST: the first face's candidate is al itself, without the min against the starting
  // kFLTMAX.  Only a candidate above kFLTMAX (3.402823e38 < a <= +inf) differs, and either way
  // al stays >= kFLTMAX until a smaller valid face: the box's result (al < kFLTMAX, then the
  // entry point from al) is the same (tests/test_box_face_forms.py).
  if constexpr (FIRST) return ok ? a : kFLTMAX;
  return __builtin_fminf(al, ok ? a : kFLTMAX);
}

// intersect_bv raytracer_func.frag:314-352; divisions as hoisted reciprocals (contract).
// WAVE: the all-lanes-inside early out is taken wave-uniformly (big boxes such as the
// ground's contain every ray origin).
// FLAT (the L1/L2 kernels' per-lane walks): no exec-mask branches inside the test.  A wave
// almost always holds lanes outside the box and lanes that reach the cull compare, so the
// inside early-out and the cull branch only add scalar mask work; the result is the same
// boolean.  L2 kernels: C4 shape +4.1 % (with node_tests' flat empty-child test), scenes 3 / 7
// +2.6 / +5 %; the LDS kernels lose 6-8 % (their spill-free 72-VGPR budget), so they keep the
// branches (profiles/r04_ab_box_flat.jsonl).
template <bool WAVE, bool FLAT = false>
__device__ __forceinline__ bool box_test(float4 a0, float4 a1, float4 a2, f3 O, f3 D, f3 invD, double cull2) {
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  // all |Oi| < 1 as one compare of the NaN-propagating maximum (exact, as in box_face)
  const bool inside = __builtin_elementwise_maximum(__builtin_elementwise_maximum(__builtin_fabsf(Oi.x), __builtin_fabsf(Oi.y)),
                                                    __builtin_fabsf(Oi.z)) < 1.0f;
  if (WAVE && __ballot(!inside) == 0) return true;
  constexpr bool kFlat = FLAT && !WAVE;
  if (!kFlat && inside) return true;
  f3 rD = mulv(invD, w);
  // faces in reference order: (x,-1) (x,+1) (y,-1) (y,+1) (z,-1) (z,+1), branch-free (box_face)
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
  al = box_face<true>(al, -1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z);
  al = box_face(al, 1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z);
  al = box_face(al, -1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x);
  al = box_face(al, 1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x);
  al = box_face(al, -1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y);
  al = box_face(al, 1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y);
  if constexpr (kFlat) {
    f3 Pg = add(mulv(add(muls(Di, al), Oi), w), c);
    f3 v = sub(O, Pg);
    return inside | ((al < kFLTMAX) & ((double)dot3(v, v) < cull2));
  }
  if (al < kFLTMAX) {
    f3 Pg = add(mulv(add(muls(Di, al), Oi), w), c);
    f3 v = sub(O, Pg);
    return (double)dot3(v, v) < cull2;
  }
  return false;
}


// A node visit's two child records (rows: centre + has-prim flag, half-width, 1/half-width)
// and their box tests: (hl, hr) = the reference's push decisions for the left and right child.
// A child whose subtree holds no primitive (flag 0) cannot change the hit and is never tested
// (COUNT keeps the reference's visits for its event model).
// In the source a row is first used behind a test (the child-empty flag, the box test's inside
// early-out, the left child's whole test before the right's), and LLVM sinks each load to its
// first use, so one node visit of the L1/L2-read kernels was a chain of up to five dependent
// cache round trips (flag -> centre + 1/w -> w -> right 1/w -> right w, read off the ISA).
// So in those kernels every row is issued at once and an empty asm consumes them at that
// point: a visit waits for one round trip (scene 8 +4..5 %, scenes 3/5/7 +1..3 %:
// profiles/r03_ab_node_loads_together.jsonl).  Same values, same bits.  The asm takes the rows
// as inputs only: it defines no new values, so the register allocator keeps the rows in their
// load tuples (in-out operands made it copy 11 rows per visit: -1.4..-1.7 % on scene 8,
// profiles/r03_ab_node_loads_inputs.jsonl).  The LDS-scene kernels (ds_read latency is short:
// -0.2..-1 % with the rows together, profiles/r03_ab_lds_rows_together.jsonl) and the mesh
// kernels (128-VGPR walk state: they spill) keep the lazy form.
#define MCPT_ROWS_IN(...) asm volatile("" ::__VA_ARGS__)
// Row k of a per-lane record array at a 32-bit byte offset from the array's wave-uniform base
// (n_prims < 2^24 keeps every node and primitive row below 2^31 bytes): the load takes the
// base from SGPRs with a 32-bit lane offset (global_load ... saddr) instead of a 64-bit VALU
// address per visit (+0.9..1.3 %: profiles/r03_ab_row_offset32.jsonl).
__device__ __forceinline__ const float4* row_ptr(const float4* __restrict__ base, size_t k) {
  return (const float4*)((const char*)base + (uint32_t)k * 16u);
}
// the two child records of a node pair j (rows 3j .. 3j+5): byte offset 48 j, with j * 3 as
// one full-rate shift-add (LLVM turns * 48 into v_mul_lo_u32, a quarter-rate instruction)
__device__ __forceinline__ const float4* node_rows(const float4* __restrict__ nodes, size_t j) {
  uint32_t t;
  asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(t) : "v"((uint32_t)j));
  return (const float4*)((const char*)nodes + (t << 4));
}
template <bool COUNT, bool FLAT = false, class SR>
__device__ __forceinline__ void node_tests(const SR& s, const float4* __restrict__ nodes, size_t j, f3 O, f3 D,
                                           f3 invD, double cull2, bool& hl, bool& hr) {
  if constexpr (!SR::kLds && !SR::kMesh) {
    const float4* q = node_rows(nodes, j);
    float4 l0 = q[0], l1 = q[1], l2 = q[2], r0 = q[3], r1 = q[4], r2 = q[5];
    MCPT_ROWS_IN("v"(l0.x), "v"(l0.y), "v"(l0.z), "v"(l0.w), "v"(l1.x), "v"(l1.y), "v"(l1.z), "v"(l2.x),
                 "v"(l2.y), "v"(l2.z));
    MCPT_ROWS_IN("v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z), "v"(r2.x),
                 "v"(r2.y), "v"(r2.z));
    if constexpr (FLAT && !COUNT) {   // an empty child's test runs and is dropped (see box_test)
      hl = (l0.w != 0.0f) & box_test<false, true>(l0, l1, l2, O, D, invD, cull2);
      hr = (r0.w != 0.0f) & box_test<false, true>(r0, r1, r2, O, D, invD, cull2);
    } else {
      hl = (COUNT || l0.w != 0.0f) && box_test<false>(l0, l1, l2, O, D, invD, cull2);
      hr = (COUNT || r0.w != 0.0f) && box_test<false>(r0, r1, r2, O, D, invD, cull2);
    }
#ifdef MCPT_LANESTATS
    const int sl = box_stage(l0, l1, l2, O, D, invD), sr = box_stage(r0, r1, r2, O, D, invD);
    ls_cond(LS_NE_WV, LS_NE_LN, sl >= 1); ls_cond(LS_NE_WV, LS_NE_LN, sr >= 1);
    ls_cond(LS_OUT_WV, LS_OUT_LN, sl >= 2); ls_cond(LS_OUT_WV, LS_OUT_LN, sr >= 2);
    ls_cond(LS_VAL_WV, LS_VAL_LN, sl >= 3); ls_cond(LS_VAL_WV, LS_VAL_LN, sr >= 3);
#endif
  } else {
    const float4 l0 = nodes[j * 3], r0 = nodes[j * 3 + 3];
    hl = (COUNT || l0.w != 0.0f) && box_test<false>(l0, nodes[j * 3 + 1], nodes[j * 3 + 2], O, D, invD, cull2);
    hr = (COUNT || r0.w != 0.0f) && box_test<false>(r0, nodes[j * 3 + 4], nodes[j * 3 + 5], O, D, invD, cull2);
  }
}

// intersect_bvm raytracer_func.frag:273-311: the mesh BVH's box test, in mesh space (O, D),
// with the entry point taken to world space through the mesh transform (rows t0..t2) and
// compared with the world distance from Ol.  Same face loop as box_test.
// FLAT (default): no exec-mask branches, as box_test's FLAT form; the mesh workload +0.8..4 %
// (profiles/r05_ab_mesh_flat_lds.jsonl)
template <bool FLAT = true>
__device__ __forceinline__ bool box_test_mesh(float4 a0, float4 a1, f3 iw, f3 O, f3 D, f3 invD, f3 Ol,
                                              float4 t0, float4 t1, float4 t2, double cull2) {
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  // all |Oi| < 1 as one compare of the NaN-propagating maximum (exact, as in box_test)
  const bool inside = __builtin_elementwise_maximum(__builtin_elementwise_maximum(__builtin_fabsf(Oi.x),
                                                    __builtin_fabsf(Oi.y)), __builtin_fabsf(Oi.z)) < 1.0f;
  if (!FLAT && inside) return true;
  f3 rD = mulv(invD, w);
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
  al = box_face<true>(al, -1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z);
  al = box_face(al, 1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z);
  al = box_face(al, -1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x);
  al = box_face(al, 1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x);
  al = box_face(al, -1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y);
  al = box_face(al, 1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y);
  if constexpr (FLAT) {   // no exec-mask branches: the entry point's cull computed and selected
    f3 Pl = add(Oi, muls(Di, al));
    f3 Pg = xpoint(t0, t1, t2, add(mulv(Pl, w), c));
    f3 v = sub(Ol, Pg);
    return inside | ((al < kFLTMAX) & ((double)dot3(v, v) < cull2));
  }
  if (al < kFLTMAX) {
    f3 Pl = add(Oi, muls(Di, al));
    f3 Pg = xpoint(t0, t1, t2, add(mulv(Pl, w), c));
    f3 v = sub(Ol, Pg);
    return (double)dot3(v, v) < cull2;
  }
  return false;
}

// a candidate hit at local point Pl of primitive `index` (transform rows t0..t2): world
// distance from Ol, kept if closer
template <bool COUNT>
__device__ __forceinline__ void accept_rows(int index, int shape, int dir, f3 Pl, f3 Ol, float4 t0, float4 t1,
                                            float4 t2, Hit& h, Ev<COUNT>& ev, bool fast_len) {
  ev.inc(EV_CAND);
  f3 Pg = xpoint(t0, t1, t2, Pl);
  float dist = fast_len ? length3(sub(Ol, Pg)) : length3_g(sub(Ol, Pg));
  if (dist < h.dist) {
    h.dist = dist; h.pl = Pl; h.set(index, shape, dir);
    h.cull2 = cull_bound_sq(dist);
  }
}
template <bool COUNT, bool UNI, class SR>
__device__ __forceinline__ void accept_cand(const SR& s, int index, int shape, int dir, f3 Pl, f3 Ol,
                                            Hit& h, Ev<COUNT>& ev) {
  const size_t b = (size_t)index * 8;
  constexpr bool U = UNI && !SR::kLds;
  accept_rows<COUNT>(index, shape, dir, Pl, Ol, ld4<U>(s.prims, b + 3), ld4<U>(s.prims, b + 4),
                     ld4<U>(s.prims, b + 5), h, ev, SR::kFastLen);
}

// Triangle_intersect raytracer_func.frag:354-396 (Möller–Trumbore, mesh space) on a leaf record
// (vertex A, edges B - A and C - A: the same binary32 values the test computed from the vertices);
// a hit keeps the mesh-local triangle index in Hit::tri (the reference's tri_index; its dir is 0)
template <bool COUNT, class SR>
__device__ __forceinline__ void tri_test(int t, float4 r0, float4 r1, float4 r2, int index, f3 O, f3 D, f3 Ol,
                                         float4 t0, float4 t1, float4 t2, Hit& h, Ev<COUNT>& ev) {
  ev.inc(EV_TRI);
  const f3 vA = mk(r0.x, r0.y, r0.z), edge1 = mk(r1.x, r1.y, r1.z), edge2 = mk(r2.x, r2.y, r2.z);
  const f3 hv = cross3(D, edge2);
  const float det = dot3(edge1, hv);
  if (__builtin_fabsf(det) < kEPS) return;
  const float invdet = wrcp<SR::kFastRcp>(det);
  const f3 sv = sub(O, vA);
  const float u = dot3(sv, hv) * invdet;
  if (u < 0.0f || u > 1.0f) return;
  const f3 q = cross3(sv, edge1);
  const float v = dot3(D, q) * invdet;
  if (v < 0.0f || (u + v) > 1.0f) return;
  const float a = dot3(edge2, q) * invdet;
  if (a > kEPS) {
    const f3 Pl = add(O, muls(D, a));
    const f3 Pg = xpoint(t0, t1, t2, Pl);
    const float dist = wlength3<SR::kFastLen>(sub(Ol, Pg));
    if (dist < h.dist) {
      h.dist = dist; h.pl = Pl; h.set(index, CODE_MESH, 0); h.tri = t;
      h.cull2 = cull_bound_sq(dist);
    }
  }
}

// a mesh leaf visit: the leaf's triangle record in one round trip, then its test (t >= 0)
template <bool COUNT, class SR>
__device__ __forceinline__ void mesh_leaf(const SR& s, size_t leaf, int index, f3 O, f3 D, f3 Ol, float4 t0,
                                          float4 t1, float4 t2, Hit& h, Ev<COUNT>& ev) {
  const float4* q = s.mleaftris + leaf * 4;
  const float4 r0 = q[0], r1 = q[1], r2 = q[2];
  MCPT_ROWS_IN("v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z), "v"(r2.x),
               "v"(r2.y), "v"(r2.z));
  MCPT_ROWS_IN("v"(t0.x), "v"(t0.y), "v"(t0.z), "v"(t0.w), "v"(t1.x), "v"(t1.y), "v"(t1.z), "v"(t1.w),
               "v"(t2.x), "v"(t2.y), "v"(t2.z), "v"(t2.w));
  const int t = __float_as_int(r0.w);
  if (t >= 0) tri_test<COUNT, SR>(t, r0, r1, r2, index, O, D, Ol, t0, t1, t2, h, ev);
}

// 1/w of a mesh child box, correctly rounded (= the host's 1.0f / w of pack_nodes): rcp_core on
// all six lanes' values, the IEEE reciprocal where some operand leaves its exact range.  Whether
// all six lie in that range is the record's own flag (wl.w, set by pack_mesh_pairs with the same
// test as rcp_core_ok): one compare instead of twelve per node step (mesh workload +2.8 %,
// mesh_big +2.1 %, with the scalar suspension compare: profiles/r06_ab_mesh_rcp_flag.jsonl)
__device__ __forceinline__ void rcp6_rn(float4 wl, float4 wr, f3& il, f3& ir) {
  il = mk(rcp_core(wl.x), rcp_core(wl.y), rcp_core(wl.z));
  ir = mk(rcp_core(wr.x), rcp_core(wr.y), rcp_core(wr.z));
  const bool ok = wl.w != 0.0f;
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) {
      il = mk(rcp_ieee(wl.x), rcp_ieee(wl.y), rcp_ieee(wl.z));
      ir = mk(rcp_ieee(wr.x), rcp_ieee(wr.y), rcp_ieee(wr.z));
    }
  }
}

// a mesh node visit (intersect_bvm for both children, :273-311): the child-pair record in one
// round trip (all four rows issued together: a visit waits for one fetch), 1/w recomputed
template <bool COUNT, class SR>
__device__ __forceinline__ void mesh_pair_tests(const SR& s, size_t node, f3 O, f3 D, f3 invD, f3 Ol, float4 t0,
                                                float4 t1, float4 t2, double cull2, bool& hl, bool& hr) {
  const float4* q = s.mpairs + node * 4;
  const float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
  MCPT_ROWS_IN("v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z));
  MCPT_ROWS_IN("v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z));
  MCPT_ROWS_IN("v"(t0.x), "v"(t0.y), "v"(t0.z), "v"(t0.w), "v"(t1.x), "v"(t1.y), "v"(t1.z), "v"(t1.w),
               "v"(t2.x), "v"(t2.y), "v"(t2.z), "v"(t2.w));
  f3 il, ir;
  rcp6_rn(a1, a3, il, ir);
  hl = (COUNT || a0.w != 0.0f) && box_test_mesh(a0, a1, il, O, D, invD, Ol, t0, t1, t2, cull2);
  hr = (COUNT || a2.w != 0.0f) && box_test_mesh(a2, a3, ir, O, D, invD, Ol, t0, t1, t2, cull2);
}

// Mesh_intersect raytracer_func.frag:642-678: the instance's own BVH, same DFS as
// intersect_bvh (right child first, cull at push with intersect_bvm), stackless per lane
template <bool COUNT, bool ANY, class SR>
__device__ __forceinline__ void mesh_test(const SR& s, int mesh, int index, f3 O, f3 D, f3 Ol, Hit& h,
                                          Ev<COUNT>& ev) {
  ev.inc(EV_MESH);
  const int4 mi = s.minfo[mesh];   // first node, first leaf, depth, first triangle
  const size_t b = (size_t)index * 8;
  const float4 t0 = s.prims[b + 3], t1 = s.prims[b + 4], t2 = s.prims[b + 5];   // read_mesh_transfo
  const f3 invD = mk(rcp_rn(D.x), rcp_rn(D.y), rcp_rn(D.z));
  const int leaf0 = (1 << mi.z) - 1;
  int node = 0, level = 0;
  uint32_t pending = 0;
  for (;;) {
    bool pop = true;
    if (node >= leaf0) {
      ev.inc(EV_LEAF);
      mesh_leaf<COUNT>(s, (size_t)mi.y + (node - leaf0), index, O, D, Ol, t0, t1, t2, h, ev);
      if (ANY && h.hit()) return;   // hit_only (:664-665): only a triangle can have set it
    } else {
      ev.inc(EV_NODE);
      const size_t j = 2 * (size_t)node + 1;
      bool hl, hr;
      mesh_pair_tests<COUNT>(s, (size_t)mi.x + mesh_pair_slot(node), O, D, invD, Ol, t0, t1, t2,
                             h.cull2, hl, hr);
      pop = !(hl || hr);
      if (hr) {
        if (hl) pending |= 1u << (level + 1);
        node = (int)j + 1; level++;
      } else if (hl) {
        node = (int)j; level++;
      }
    }
    if (pop) {
      if (pending == 0) break;
      int L = 31 - __builtin_clz(pending);
      pending &= ~(1u << L);
      node = ((node + 1) >> (level - L)) - 2;
      level = L;
    }
  }
}

// num / den from den's reciprocal y = rcp_core(den) by div_core (mcpt_math.h; exhaustively
// checked), the IEEE division for the lanes whose operands leave div_core's exact range (ok false;
// a wave-uniform branch, taken only when some lane is out of range).  Same bits as num / den;
// C2 +1.6 % over the IEEE division everywhere (profiles/r04_ab_short_div.jsonl).
__device__ __forceinline__ float quot(float num, float den, float y, bool ok) {
  if constexpr (kDriverDiv) return fdiv(num, den);
  float q = div_core(num, den, y);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) q = div_ieee(num, den);
  }
  return q;
}

// intersect_prim raytracer_func.frag:681-705 + Sphere/Cube/Cylinder/Cone/OrientedQuad :398-640
// NOMESH: the caller handles CODE_MESH leaves itself (walk_run_mesh), so the nested mesh DFS is not
// compiled in here
template <bool COUNT, bool UNI, bool ANY = false, bool NOMESH = false, class SR>
__device__ __forceinline__ void prim_test(const SR& s, int i, f3 Ow, f3 Dw, Hit& h, Ev<COUNT>& ev) {
  ev.inc(EV_PRIM);
  constexpr bool U = UNI && !SR::kLds;
  // per-lane L1/L2 reads (node_tests): the type code and the inverse rows in one round trip,
  // else the rows' loads wait behind the type test
  constexpr bool kTogether = !U && !SR::kLds && !SR::kMesh;
  int pt = kTogether ? s.ptype[(uint32_t)i] : ld1<U>(s.ptype, i);
  if constexpr (!kTogether) {
    if (pt < 0) return;
  }
  const size_t b = (size_t)i * 8;
  float4 r0, r1, r2;
  if constexpr (kTogether) {
    const float4* q = row_ptr(s.prims, b);
    r0 = q[0]; r1 = q[1]; r2 = q[2];
    MCPT_ROWS_IN("v"(pt), "v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z),
                 "v"(r1.w), "v"(r2.x), "v"(r2.y), "v"(r2.z), "v"(r2.w));
  } else {
    r0 = ld4<U>(s.prims, b); r1 = ld4<U>(s.prims, b + 1); r2 = ld4<U>(s.prims, b + 2);
  }
  // kOne (the L1/L2-read kernels: scene 8, C4 shape +2.1 %, profiles/r04_ab_deep_walk.jsonl; the
  // LDS-scene C2 kernel -0.6 % with it, so not there): the type branches only record their
  // candidate (the sphere's near and far
  // roots: two) and one accept site after the switch tests it against the hit record, so a leaf
  // block whose lanes hold several primitive types runs the candidate code (transform rows,
  // world point, length, compare, record update) once instead of once per type.  Each lane's
  // candidates reach the hit record in the same order (same bits).
  constexpr bool kOne = !SR::kLds;
  bool has1 = false, has2 = false;
  int shape1 = 0, dir1 = 0;
  f3 P1 = mk(0.0f, 0.0f, 0.0f), P2 = P1;
  auto accept = [&](int shape, int dir, f3 Pl) {
    if constexpr (kOne) { has1 = true; shape1 = shape; dir1 = dir; P1 = Pl; }
    else accept_cand<COUNT, UNI>(s, i, shape, dir, Pl, Ow, h, ev);
  };
  auto accept_far = [&](f3 Pl) {   // the sphere's far root, after its near root
    if constexpr (kOne) { has2 = true; P2 = Pl; }
    else accept_cand<COUNT, UNI>(s, i, CODE_SPHERE, 0, Pl, Ow, h, ev);
  };
  if (pt < 0) return;
  const int t = pt & 15;
  f3 O = xpoint(r0, r1, r2, Ow);
  f3 D = wnormalize3<SR::kFastNorm>(xdir(r0, r1, r2, Dw));
  if (t == CODE_SPHERE) {
    float OO = dot3(O, O), OD = dot3(O, D), D2 = dot3(D, D);
    float delta4 = OD * OD - D2 * (OO - 1.0f);
    if (delta4 > 0.0f) {
      float sq = wsqrt<SR::kFastSqrt>(delta4);
      // D2 = |D|^2 of a normalized D: within div_core's range
      const float y = rcp_core(D2), n1 = -(OD + sq), n2 = -(OD - sq);
      float a = quot(n1, D2, y, div_a_ok(n1));
      if (a > kEPS) accept(CODE_SPHERE, 0, add(O, muls(D, a)));
      a = quot(n2, D2, y, div_a_ok(n2));
      if (a > kEPS) accept_far(add(O, muls(D, a)));
    }
  } else if (t == CODE_QUAD) {
    if (!(D.z > -kEPS)) {
      float a = quot(-O.z, D.z, rcp_core(D.z), div_a_ok(-O.z));   // D.z <= -kEPS
      f3 Pl = add(O, muls(D, a));
      if (!(__builtin_fabsf(Pl.x) > 1.0f || __builtin_fabsf(Pl.y) > 1.0f)) accept(CODE_QUAD, 0, Pl);
    }
  } else if (t == CODE_CUBE) {
    float al = kFLTMAX; int cl = 0;
    float o[3] = {O.x, O.y, O.z}, d[3] = {D.x, D.y, D.z};
    // the two faces of an axis divide by the same d (one reciprocal); |d| > kEPS of a normalized
    // D and, for |o| <= 2^59, the numerators cd - o (+0, never -0, or >= 2^-24 in magnitude) are
    // in range
    const bool o_ok = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(O.x), __builtin_fabsf(O.y)), __builtin_fabsf(O.z)) <= 0x1p59f;
    const float yd[3] = {rcp_core(D.x), rcp_core(D.y), rcp_core(D.z)};
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const int c0 = f / 2, c1 = (c0 + 1) % 3, c2 = (c0 + 2) % 3;
      // branch-free: every face's quotient, the axis flag and the in-face bounds (one compare
      // of their NaN-propagating maximum, as in box_face) in one mask; the strict a < al keeps
      // the reference's first-minimum face.  A face of a non-dividing axis (|d| <= kEPS) gets a
      // meaningless quotient that the mask drops.  C4 shape +0.5 %, scene 3 +4.4 % over the
      // branching form (profiles/r04_ab_masks.jsonl).
      const bool dv = __builtin_fabsf(d[c0]) > kEPS;
      const float cd = (f % 2) ? 1.0f : -1.0f;
      const float a = quot(cd - o[c0], d[c0], yd[c0], o_ok);
      if (dv & (a > kEPS) & (a < al) &
          (__builtin_elementwise_maximum(__builtin_fabsf(o[c1] + a * d[c1]), __builtin_fabsf(o[c2] + a * d[c2])) <= 1.0f)) {
        al = a; cl = f;
      }
    }
    if (al < kFLTMAX) accept(CODE_CUBE, cl, add(O, muls(D, al)));
  } else if (t == CODE_CYLINDER) {
    int cl = -1; float al = kFLTMAX;
    if (__builtin_fabsf(D.z) > kEPS) {
      // the caps divide by D.z (one reciprocal; numerators as in the cube test); each
      // candidate's conditions in one mask
      const float yz = rcp_core(D.z);
      const bool z_ok = __builtin_fabsf(O.z) <= 0x1p59f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const float a = quot((k ? 1.0f : -1.0f) - O.z, D.z, yz, z_ok);
        const float rx = O.x + a * D.x, ry = O.y + a * D.y;
        if ((a > kEPS) & (__builtin_fmaf(ry, ry, rx * rx) < 1.0f) & (a < al)) { cl = k; al = a; }
      }
    }
    float O2 = __builtin_fmaf(O.y, O.y, O.x * O.x);
    float OD = __builtin_fmaf(O.y, D.y, O.x * D.x);
    float D2 = __builtin_fmaf(D.y, D.y, D.x * D.x);
    float delta4 = OD * OD - D2 * (O2 - 1.0f);
    if (delta4 > 0.0f) {
      const float n = -(OD + wsqrt<SR::kFastSqrt>(delta4));
      float a = quot(n, D2, rcp_core(D2), div_a_ok(n) && div_b_ok(D2));
      if ((a > kEPS) & (a < al) & (__builtin_fabsf(O.z + a * D.z) < 1.0f)) { cl = 2; al = a; }
    }
    if (al < kFLTMAX) accept(CODE_CYLINDER, cl, add(O, muls(D, al)));
  } else if (t == CODE_CONE) {
    int cl = -1; float tl = kFLTMAX;
    if (__builtin_fabsf(D.z) > kEPS) {
      float t0 = fdiv(-1.0f - O.z, D.z);
      if (t0 > kEPS) {
        float rx = O.x + t0 * D.x, ry = O.y + t0 * D.y;
        if ((__builtin_fmaf(ry, ry, rx * rx) < 1.0f) && (t0 < tl)) { cl = 0; tl = t0; }
      }
    }
    f3 co = O; co.z -= 1.0f;
    float a = D.z * D.z - 0.8f;
    float b = 2.0f * (D.z * co.z - dot3(D, co) * 0.8f);
    float cc = co.z * co.z - dot3(co, co) * 0.8f;
    float det = b * b - (4.0f * a) * cc;
    if (det > 0.0f) {
      det = wsqrt<SR::kFastSqrt>(det);
      float t1 = fdiv(-b - det, 2.0f * a);
      if (__builtin_fabsf(O.z + t1 * D.z) > 1.0f) t1 = kFLTMAX;
      float t2 = fdiv(-b + det, 2.0f * a);
      if (__builtin_fabsf(O.z + t2 * D.z) > 1.0f) t2 = kFLTMAX;
      float tt = gmin(t1, t2);
      if (tt < tl) { cl = 2; tl = tt; }
    }
    if (tl < kFLTMAX) accept(CODE_CONE, cl, add(O, muls(D, tl)));
  } else if (t == CODE_MESH) {
    if constexpr (SR::kMesh && !NOMESH) mesh_test<COUNT, ANY>(s, pt >> 4, i, O, D, Ow, h, ev);
  }
  if constexpr (kOne) {
    if (has1) accept_cand<COUNT, UNI>(s, i, shape1, dir1, P1, Ow, h, ev);
    if (has2) accept_cand<COUNT, UNI>(s, i, CODE_SPHERE, 0, P2, Ow, h, ev);
  }
}

// intersect_bvh raytracer_func.frag:734-769, per lane, stackless.  pending bit L = "a left
// sibling at level L waits on the reference's stack"; popping the deepest pending bit is
// exactly the reference's LIFO order (right child first, cull decided at push time).
// ANY: just_hit_bvh (raytracer_func.frag:771-775) — stop at the first leaf whose primitive
// produced a hit (hit_only, :756-757); the render path always uses traverse_all_bvh.
template <bool COUNT, bool ANY = false, bool FLAT = false, class SR>
__device__ __forceinline__ void traverse_lane(const SR& s, f3 O, f3 D, Hit& h, Ev<COUNT>& ev) {
  ev.inc(EV_TRAV);
  h.clear(); h.dist = kFLTMAX; h.cull2 = cull_bound_sq(kFLTMAX);
  const f3 invD = mk(rcp_rn(D.x), rcp_rn(D.y), rcp_rn(D.z));
  const int leaf0 = (1 << s.depth) - 1;
  int node = 0, level = 0;
  uint32_t pending = 0;
  for (;;) {
    bool pop = true;
    const bool is_leaf = node >= leaf0;
#ifdef MCPT_STAMPS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();   // wave-uniform stamps
#endif
    if (is_leaf) {
      ev.inc(EV_LEAF);
      int p = s.leaves[node - leaf0];
      if (p >= 0) prim_test<COUNT, false, ANY>(s, p, O, D, h, ev);
      if (ANY && h.hit()) break;
    }
#ifdef MCPT_STAMPS
    ev.st_leaf += __builtin_amdgcn_s_memtime() - t0;
    ev.st_lit++;
    ev.st_wit += (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1;
#endif
    if (!is_leaf) {
      ev.inc(EV_NODE);
      const size_t j = 2 * (size_t)node + 1;
      bool hl, hr;
      node_tests<COUNT, FLAT>(s, s.nodes, j, O, D, invD, h.cull2, hl, hr);
      pop = !(hl || hr);
      if (hr) {
        if (hl) pending |= 1u << (level + 1);
        node = (int)j + 1; level++;
      } else if (hl) {
        node = (int)j; level++;
      }
    }
    if (pop) {
      if (pending == 0) break;
      int L = 31 - __builtin_clz(pending);
      pending &= ~(1u << L);
      node = ((node + 1) >> (level - L)) - 2;
      level = L;
    }
  }
}

// Resumable form of traverse_lane for the render loop.  The wave leaves the traversal loop
// once at most `exit` lanes are still walking (and at least one lane finished in this call):
// the finished lanes shade and start their next ray while the stragglers keep their walk
// state (node, level, pending, invD, hit record) and continue in the next round.  Each
// lane's own sequence of visits is traverse_lane's; only the interleaving changes.
struct Walk {
  f3 invD;
  int node, level;
  uint32_t pending;
  // mesh kernels (walk_run_mesh): the instance whose mesh BVH this lane is walking (-1: none),
  // its mesh id, the mesh walk's node / level / pending mask, and the ray in mesh space
  int mprim, mnode, mlevel;
  int mpf;                 // mesh kernels: the last prefetch's dummy value (walk_run_mesh)
  uint32_t mpending;
  f3 Om, Dm, invDm;
  int4 mi;                 // the mesh's (first pair slot, first leaf, depth, first triangle)
};

template <bool COUNT, class SR>
__device__ __forceinline__ void walk_begin(const SR& s, f3 D, Hit& h, Walk& w, Ev<COUNT>& ev, double cull2_max) {
  ev.inc(EV_TRAV);
  // cull2_max = cull_bound_sq(kFLTMAX), a kernel argument (SGPRs) rather than a constant the
  // register allocator keeps in (spilled) VGPRs across the render loop
  h.clear(); h.dist = kFLTMAX; h.cull2 = cull2_max;
  w.invD = mk(rcp_rn(D.x), rcp_rn(D.y), rcp_rn(D.z));
  w.node = 0; w.level = 0; w.pending = 0;
  if constexpr (SR::kMesh) w.mprim = -1;
}

// true: this lane's walk is complete; false: suspended (wave-level early exit).
// SUSPEND (deep-BVH kernel) also batches leaf visits: an iteration runs either the leaf
// block (for the lanes sitting on a leaf) or the node block (for the others), and the leaf
// block only once at least `leaf_batch` lanes wait on a leaf or no lane can take a node step.
// In the if/if loop nearly every iteration of a deep walk pays for both blocks (some lane
// is always on a leaf); here a lane waits a few node iterations instead.  Each lane's own
// visit sequence is unchanged (the cull reads its own hit record only).
template <bool COUNT, bool SUSPEND, class SR>
__device__ __forceinline__ bool walk_run(const SR& s, f3 O, f3 D, Hit& h, Walk& w, Ev<COUNT>& ev, int exit,
                                         int leaf_batch, int min_done = 1) {
  // the suspendable L1/L2 walk (the deep-BVH kernel) runs its box tests and its push / pop
  // without exec-mask branches (box_test FLAT): C4 shape +4.1 % and +2.5 %; the LDS, mesh and
  // non-suspending kernels lose with it (-6..11 %: profiles/r04_ab_box_flat.jsonl,
  // r04_ab_walk_flat.jsonl), so they keep the branches
  constexpr bool kFlat = SUSPEND && !SR::kLds && !SR::kMesh;
  const int leaf0 = (1 << s.depth) - 1;
  const int n0 = SUSPEND ? __builtin_popcountll(__ballot(1)) : 0;
#ifdef MCPT_LANESTATS
  ls_add(LS_WALK_CALLS, 1u);
#endif
  for (;;) {
    bool pop = true;
    bool is_leaf = w.node >= leaf0;
    bool do_leaf = is_leaf, do_node = !is_leaf;
    if (SUSPEND) {   // wave-uniform choice of the block; the ballot taken where is_leaf is computed
      // (computed under `leaf_batch > 0`, the compiler rebuilt the lane mask from a VGPR and
      // chained ~18 scalar ops per iteration: C4 shape +0.7 %, profiles/r04_ab_masks.jsonl)
      const uint64_t on_leaf = __ballot(is_leaf);
      const bool leaves = leaf_batch <= 0 || __builtin_popcountll(on_leaf) >= leaf_batch ||
                          on_leaf == __builtin_amdgcn_read_exec();
      if (leaf_batch > 0) {
        do_leaf = leaves && is_leaf;
        do_node = !leaves && !is_leaf;
      }
    }
#ifdef MCPT_STAMPS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();   // wave-uniform stamps
#endif
#ifdef MCPT_LANESTATS
    ls_add(LS_WALK_IT, 1u);
    ls_add(LS_WALK_LN, ls_pop(true));
    if (__ballot(do_node)) {   // face jobs of this node iteration (both children's face stages)
      int jobs = 0;
      if (do_node) {
        const float4* q = node_rows(s.nodes, 2 * (size_t)w.node + 1);
        jobs = (box_stage(q[0], q[1], q[2], O, D, w.invD) >= 2) + (box_stage(q[3], q[4], q[5], O, D, w.invD) >= 2);
      }
      unsigned tot = 0;
      for (int k = 1; k <= 2; ++k) tot += (unsigned)k * ls_pop(jobs == k);
      ls_add(LS_FIT_IT, tot <= ls_pop(true) ? 1u : 0u);   // one round of the walking lanes would do
      ls_add(LS_TWO_IT, ls_pop(jobs == 2) ? 1u : 0u);     // some lane needs both children's faces
    }
    {
      const unsigned nn = ls_pop(do_node), nl = ls_pop(do_leaf);
      ls_add(LS_NODE_IT, nn ? 1u : 0u); ls_add(LS_NODE_LN, nn);
      ls_add(LS_LEAF_IT, nl ? 1u : 0u); ls_add(LS_LEAF_LN, nl);
      int pp = do_leaf ? s.leaves[(uint32_t)(w.node - leaf0)] : -1;
      const int ty = pp >= 0 ? (s.ptype[pp] & 15) : -1;
      ls_add(LS_PRIM_LN, ls_pop(pp >= 0 && s.ptype[pp] >= 0));
      ls_cond(LS_SPH_WV, LS_SPH_LN, ty == CODE_SPHERE);
      ls_cond(LS_CUBE_WV, LS_CUBE_LN, ty == CODE_CUBE);
      ls_cond(LS_CYL_WV, LS_CYL_LN, ty == CODE_CYLINDER);
      ls_cond(LS_QUAD_WV, LS_QUAD_LN, ty == CODE_QUAD);
    }
#endif
    if (do_leaf) {
      ev.inc(EV_LEAF);
      int p = s.leaves[(uint32_t)(w.node - leaf0)];
      if (p >= 0) prim_test<COUNT, false, false>(s, p, O, D, h, ev);
    }
#ifdef MCPT_STAMPS
    ev.st_leaf += __builtin_amdgcn_s_memtime() - t0;
    ev.st_lit += do_leaf || do_node;
    {
      const bool lead = (int)__lane_id() == __builtin_ffsll((long long)__ballot(1)) - 1;
      ev.st_wit += lead;
      ev.st_nl += do_node;   // lanes in the node block / leaf block, and iterations running each
      ev.st_ll += do_leaf;
      ev.st_nw += lead && __ballot(do_node) != 0;
      ev.st_lw += lead && __ballot(do_leaf) != 0;
    }
#endif
    if (do_node) {
      ev.inc(EV_NODE);
      const size_t j = 2 * (size_t)w.node + 1;
      bool hl, hr;
      node_tests<COUNT, kFlat>(s, s.nodes, j, O, D, w.invD, h.cull2, hl, hr);
      if constexpr (kFlat) {   // the push as selects instead of exec-mask branches
        const bool any = hl | hr;
        w.pending |= (hl & hr) ? 1u << (w.level + 1) : 0u;
        w.node = any ? (int)j + (hr ? 1 : 0) : w.node;
        w.level += any ? 1 : 0;
        pop = !any;
      } else {
        pop = !(hl || hr);
        if (hr) {
          if (hl) w.pending |= 1u << (w.level + 1);
          w.node = (int)j + 1; w.level++;
        } else if (hl) {
          w.node = (int)j; w.level++;
        }
      }
    }
    if constexpr (kFlat) {   // the pop as selects; only the walk's end leaves the loop per lane
      if (pop & (do_leaf | do_node)) {
        if (w.pending == 0) return true;
      }
      const bool p2 = pop & (do_leaf | do_node);
      const int L = 31 - __builtin_clz(w.pending | 1u);
      w.pending = p2 ? w.pending & ~(1u << L) : w.pending;
      w.node = p2 ? ((w.node + 1) >> (w.level - L)) - 2 : w.node;
      w.level = p2 ? L : w.level;
    } else if (pop && (do_leaf || do_node)) {
      if (w.pending == 0) return true;
      int L = 31 - __builtin_clz(w.pending);
      w.pending &= ~(1u << L);
      w.node = ((w.node + 1) >> (w.level - L)) - 2;
      w.level = L;
    }
    if (SUSPEND) {   // wave-uniform
      const int n = __builtin_popcountll(__ballot(1));
      if (n <= exit && n0 - n >= min_done) return false;
    }
  }
}



// walk_run for scenes with mesh instances.  The reference runs an instance's whole mesh DFS
// (Mesh_intersect raytracer_func.frag:642-678) inside the scene DFS's leaf visit; nested that
// way on the GPU, only the lanes sitting on a mesh leaf walk their (long, divergent) mesh
// BVHs while the rest of the wave waits (5 % VALU lane utilisation on a 1 M-triangle scene).
// Here a lane's mesh walk is part of the same loop: each iteration is one scene node, scene
// leaf, mesh node or mesh leaf step of that lane; a lane reaching a mesh leaf sets up its
// mesh-space ray (intersect_prim :681-705) and continues in the mesh until its pending mask
// is empty, then pops the scene stack.  Each lane's sequence of box / primitive / triangle
// tests is the reference's, in the reference's order (same bits, same event counts).
template <bool COUNT, bool SUSPEND, class SR>
__device__ __forceinline__ bool walk_run_mesh(const SR& s, f3 O, f3 D, Hit& h, Walk& w, Ev<COUNT>& ev, int exit) {
  const int leaf0 = (1 << s.depth) - 1;
  const int n0 = SUSPEND ? __builtin_popcountll(__ballot(1)) : 0;
#ifdef MCPT_LANESTATS
  ls_add(LS_WALK_CALLS, 1u);
#endif
  for (;;) {
    // the suspension test at the loop head rather than its tail (the same test between the same
    // iterations: lanes whose walk ended have returned): the compiler's copies of the walk state
    // at the back edge shrink (mesh workload +3.7 %, profiles/r06_ab_mesh_walk_copies.jsonl).
    // (n != n0 is n < n0: lanes only leave; a 32-bit scalar compare, where n < n0 became a 64-bit
    // vector one)
    if (SUSPEND) {   // wave-uniform
      const int n = __builtin_popcountll(__ballot(1));
      if (n <= exit && n != n0) {
#ifdef MCPT_LANESTATS
        ls_add(LS_EXIT_LN, (unsigned)n);
#endif
        return false;
      }
    }
#ifdef MCPT_LANESTATS
    {   // which block each walking lane takes this iteration
      const bool inm = w.mprim >= 0, ml = inm && w.mnode >= (1 << w.mi.z) - 1, sl = !inm && w.node >= leaf0;
      ls_add(LS_WALK_IT, 1u);
      ls_add(LS_WALK_LN, ls_pop(true));
      ls_cond(LS_NODE_IT, LS_NODE_LN, inm && !ml);
      ls_cond(LS_LEAF_IT, LS_LEAF_LN, ml);
      ls_cond(LS_SNODE_IT, LS_SNODE_LN, !inm && !sl);
      ls_cond(LS_SLEAF_IT, LS_SLEAF_LN, sl);
    }
#endif
    bool pop = false;   // the scene walk pops its stack this iteration
    int enter_p = -1;   // this lane starts the mesh walk of instance enter_p (set up below)
    if (w.mprim >= 0) {
      // one step of the instance's mesh walk (mesh_test's loop body)
      const int4 mi = w.mi;
      // the instance's transform rows are read again at every mesh step (LDS for small scenes,
      // else L1/L2 hits issued with the step's record) rather than held in the walk state: the
      // mesh workload +6 % (profiles/r05_ab_mesh_trf_reload_waves.jsonl: main vs trf0)
      const float4* tp = s.prims + (size_t)w.mprim * 8 + 3;
      const float4 t0 = tp[0], t1 = tp[1], t2 = tp[2];
      const int mleaf0 = (1 << mi.z) - 1;
      bool mpop = true;
      // one record per lane and step, node or leaf alike (64 B: a child-pair record, or a leaf's
      // triangle record), issued before the lanes split into the node and leaf blocks: the wave
      // waits once per iteration instead of once per block (measured neutral on the mesh
      // workload, r05_ab_mesh_prefetch.jsonl session r05x; kept as the simpler form)
      // Both kinds of record live in one allocation, the leaf records after the pair slots
      // (mcpt_upload_meshes), so a record is a 32-bit byte offset from the wave-uniform base: the
      // load takes the base from SGPRs (global_load ... saddr) and the step computes one 32-bit
      // offset instead of two 64-bit addresses and a select of the bases.  The mesh workload
      // +3.4 %, mesh_big +3.2 % (profiles/r06_ab_mesh_rec32.jsonl: ro vs main); records < 4 GiB.
      const bool mleaf = w.mnode >= mleaf0;
      const unsigned j = 2u * (unsigned)w.mnode + 1u;
      const unsigned lslot0 = (unsigned)(s.mleaftris - s.mpairs) >> 2;   // first leaf record (uniform)
      const unsigned rec = mleaf ? lslot0 + (unsigned)(mi.y + (w.mnode - mleaf0))
                                 : (unsigned)mi.x + mesh_pair_slot((unsigned)w.mnode);
      // node lanes also request their children's line (both pair records, or the two leaf
      // records of the last level), consumed one step later: +0.9..1.4 % on the mesh workload;
      // the grandchildren's two lines as well: -5..8 % (profiles/r05_ab_mesh_prefetch.jsonl)
      const unsigned recc = mleaf ? rec
                                  : ((w.mlevel + 1 < mi.z) ? (unsigned)mi.x + mesh_pair_slot(j)
                                                           : lslot0 + (unsigned)mi.y + (j - (unsigned)mleaf0));
      const float4* q = (const float4*)((const char*)s.mpairs + rec * 64u);
      const float4* qc = (const float4*)((const char*)s.mpairs + recc * 64u);
      const float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
      asm volatile("" ::"v"(w.mpf));
      w.mpf = *(const int*)qc;
      MCPT_ROWS_IN("v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z));
      MCPT_ROWS_IN("v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z));
      MCPT_ROWS_IN("v"(t0.x), "v"(t0.y), "v"(t0.z), "v"(t0.w), "v"(t1.x), "v"(t1.y), "v"(t1.z), "v"(t1.w),
                   "v"(t2.x), "v"(t2.y), "v"(t2.z), "v"(t2.w));
      if (mleaf) {
        ev.inc(EV_LEAF);
        const int t = __float_as_int(a0.w);
        if (t >= 0) tri_test<COUNT, SR>(t, a0, a1, a2, w.mprim, w.Om, w.Dm, O, t0, t1, t2, h, ev);
      } else {
        ev.inc(EV_NODE);
        f3 il, ir;
        rcp6_rn(a1, a3, il, ir);
        const bool hl = (COUNT || a0.w != 0.0f) && box_test_mesh(a0, a1, il, w.Om, w.Dm, w.invDm, O, t0, t1, t2, h.cull2);
        const bool hr = (COUNT || a2.w != 0.0f) && box_test_mesh(a2, a3, ir, w.Om, w.Dm, w.invDm, O, t0, t1, t2, h.cull2);
        mpop = !(hl || hr);
        if (hr) {
          if (hl) w.mpending |= 1u << (w.mlevel + 1);
          w.mnode = (int)j + 1; w.mlevel++;
        } else if (hl) {
          w.mnode = (int)j; w.mlevel++;
        }
      }
      if (mpop) {
        if (w.mpending == 0) {
          w.mprim = -1;   // Mesh_intersect done: back to the scene DFS
          pop = true;
        } else {
          const int L = 31 - __builtin_clz(w.mpending);
          w.mpending &= ~(1u << L);
          w.mnode = ((w.mnode + 1) >> (w.mlevel - L)) - 2;
          w.mlevel = L;
        }
      }
    } else if (w.node >= leaf0) {
      ev.inc(EV_LEAF);
      pop = true;
      const int p = s.leaves[w.node - leaf0];
      if (p >= 0) {
        const int pt = s.ptype[p];
        if (pt >= 0 && (pt & 15) == CODE_MESH) {
          // the mesh walk starts with the next iteration; its set-up (intersect_prim's
          // transforms) runs after the step blocks, below
          ev.inc(EV_PRIM);
          ev.inc(EV_MESH);
          enter_p = p;
          w.mprim = p;
          w.mnode = 0; w.mlevel = 0; w.mpending = 0;
          pop = false;
        } else {
          prim_test<COUNT, false, false, true>(s, p, O, D, h, ev);
        }
      }
    } else {
      ev.inc(EV_NODE);
      const size_t j = 2 * (size_t)w.node + 1;
      const float4 l0 = s.nodes[j * 3], r0 = s.nodes[j * 3 + 3];   // (mesh kernels: see node_tests)
      const bool hl = (COUNT || l0.w != 0.0f) &&
                      box_test<false>(l0, s.nodes[j * 3 + 1], s.nodes[j * 3 + 2], O, D, w.invD, h.cull2);
      const bool hr = (COUNT || r0.w != 0.0f) &&
                      box_test<false>(r0, s.nodes[j * 3 + 4], s.nodes[j * 3 + 5], O, D, w.invD, h.cull2);
      pop = !(hl || hr);
      if (hr) {
        if (hl) w.pending |= 1u << (w.level + 1);
        w.node = (int)j + 1; w.level++;
      } else if (hl) {
        w.node = (int)j; w.level++;
      }
    }
    // The mesh entry's set-up (intersect_prim's transforms, :681-705) in a wave-uniform block
    // where every path of the iteration meets: each walking lane computes it (from its own
    // instance, else from prim 0's records) and keeps it by a select.  Assigned inside the
    // scene-leaf block, the twelve values of the mesh-space ray and mesh info were joined there
    // and the compiler copied all twelve into other registers and back on every iteration (24
    // v_mov per iteration); as selects they stay in place.  The entering lanes compute the same
    // values as before (same bits).  Mesh workload +6.3 %, mesh_big +6.7 % with the head test
    // above (r06_ab_mesh_walk_copies.jsonl: t13 vs main).
    if (__ballot(enter_p >= 0)) {
      const bool e = enter_p >= 0;
      const int pe = e ? enter_p : w.mprim >= 0 ? w.mprim : 0;
      const size_t b = (size_t)pe * 8;
      const float4 r0 = s.prims[b], r1 = s.prims[b + 1], r2 = s.prims[b + 2];
      const f3 nOm = xpoint(r0, r1, r2, O);
      const f3 nDm = wnormalize3<SR::kFastNorm>(xdir(r0, r1, r2, D));
      const f3 niD = mk(rcp_rn(nDm.x), rcp_rn(nDm.y), rcp_rn(nDm.z));
      const int4 nmi = s.minfo[e ? (s.ptype[pe] >> 4) : 0];
      w.Om.x = e ? nOm.x : w.Om.x; w.Om.y = e ? nOm.y : w.Om.y; w.Om.z = e ? nOm.z : w.Om.z;
      w.Dm.x = e ? nDm.x : w.Dm.x; w.Dm.y = e ? nDm.y : w.Dm.y; w.Dm.z = e ? nDm.z : w.Dm.z;
      w.invDm.x = e ? niD.x : w.invDm.x; w.invDm.y = e ? niD.y : w.invDm.y; w.invDm.z = e ? niD.z : w.invDm.z;
      w.mi.x = e ? nmi.x : w.mi.x; w.mi.y = e ? nmi.y : w.mi.y; w.mi.z = e ? nmi.z : w.mi.z; w.mi.w = e ? nmi.w : w.mi.w;
    }
    if (pop) {
      if (w.pending == 0) return true;
      const int L = 31 - __builtin_clz(w.pending);
      w.pending &= ~(1u << L);
      w.node = ((w.node + 1) >> (w.level - L)) - 2;
      w.level = L;
    }
  }
}

// intersect_bvh, wave-coherent.  Every lane's DFS visits a subsequence of ONE fixed order:
// the right-child-first pre-order of the implicit heap, with the subtrees its push-time
// box tests culled.  The wave walks that order once with a wave-uniform cursor (node,
// level) and skips a subtree only when NO lane pushed it (ballot); a lane works at a
// node only if it pushed it ("act").  Per lane this is the reference's visit sequence, so
// every box test sees the same h.dist and every prim test happens in the same order.
// Gains: node records, leaf ids and prim records are wave-uniform (scalar loads into
// SGPRs), the primitive-type switch is a uniform branch, and leaf and internal-node
// work never diverge inside a wave.  Per lane: 1 bit per level for a pushed left child.
template <bool COUNT, class SR>
__device__ __forceinline__ void traverse_wave(const SR& s, f3 O, f3 D, Hit& h, Ev<COUNT>& ev) {
  ev.inc(EV_TRAV);
  h.clear(); h.dist = kFLTMAX; h.cull2 = cull_bound_sq(kFLTMAX);
  const f3 invD = mk(rcp_rn(D.x), rcp_rn(D.y), rcp_rn(D.z));
  const int leaf0 = (1 << s.depth) - 1;
  uint32_t lpend = 0;    // bit L: this lane pushed the left child at level L of the cursor path
  bool act = true;       // this lane visits the cursor node
  int node = 0, level = 0;   // wave-uniform cursor
  for (;;) {
    bool descend = false;
    if (node >= leaf0) {
      if (act) {
        ev.inc(EV_LEAF);
        int p = ld1<!SR::kLds>(s.leaves, node - leaf0);
        if (p >= 0) prim_test<COUNT, true>(s, p, O, D, h, ev);
      }
    } else {
      const size_t j = 2 * (size_t)node + 1;
      bool hl = false, hr = false;
      if (act) {
        ev.inc(EV_NODE);
        constexpr bool U = !SR::kLds;
        const float4 l0 = ld4<U>(s.nodes, j * 3), r0 = ld4<U>(s.nodes, j * 3 + 3);
        // empty subtrees (c.w == 0) are never visited (wave-uniform skip; see traverse_lane)
        if (COUNT || l0.w != 0.0f)
          hl = box_test<true>(l0, ld4<U>(s.nodes, j * 3 + 1), ld4<U>(s.nodes, j * 3 + 2), O, D, invD, h.cull2);
        if (COUNT || r0.w != 0.0f)
          hr = box_test<true>(r0, ld4<U>(s.nodes, j * 3 + 4), ld4<U>(s.nodes, j * 3 + 5), O, D, invD, h.cull2);
      }
      const uint32_t bit = 1u << (level + 1);
      lpend = hl ? (lpend | bit) : (lpend & ~bit);
      if (__ballot(hr)) {
        node = (int)j + 1; level++; act = hr; descend = true;
      } else if (__ballot(hl)) {
        node = (int)j; level++; act = hl; descend = true;
      }
    }
    if (descend) continue;
    // subtree(node) done: next pushed node in right-first pre-order, climbing
    bool found = false;
    while (level > 0) {
      if ((node & 1) == 0) {                       // a right child: its left sibling next
        const bool a = (lpend >> level) & 1u;
        if (__ballot(a)) { node = node - 1; act = a; found = true; break; }
      }
      node = (node - 1) >> 1; level--;
    }
    if (!found) break;
  }
}

// FLAT: the box tests without exec-mask branches (box_test), as the walk of the same kernel
template <bool COUNT, bool WAVE, bool FLAT = false, class SR>
__device__ __forceinline__ void traverse(const SR& s, f3 O, f3 D, Hit& h, Ev<COUNT>& ev) {
  if (WAVE) traverse_wave<COUNT>(s, O, D, h, ev);
  else traverse_lane<COUNT, false, FLAT>(s, O, D, h, ev);
}

// intersection_info raytracer_func.frag:812-897 (hit only; misses leave N,P untouched)
template <bool COUNT, class SR>
__device__ __forceinline__ void geom_info(const SR& s, const Hit& h, f3& N, f3& P, Ev<COUNT>& ev) {
  ev.inc(EV_GEOM);
  const int shape = h.shape(), dir = h.face();
  const float4* pr = s.prims + (size_t)h.index() * 8;
  float4 t0 = pr[3], t1 = pr[4], t2 = pr[5];
  P = xpoint(t0, t1, t2, h.pl);   // = the candidate's Pg (accept_cand / tri_test)
  f3 q;
  if (shape == CODE_SPHERE) {
    q = muls(h.pl, 2.0f);
  } else if (shape == CODE_CUBE) {
    float sg = (dir % 2 != 0) ? 1.0f : -1.0f;
    int ax = dir / 2;
    q = add(h.pl, mk(ax == 0 ? sg : 0.0f, ax == 1 ? sg : 0.0f, ax == 2 ? sg : 0.0f));
  } else if (shape == CODE_CYLINDER) {
    f3 No = (dir < 2) ? mk(0.0f, 0.0f, (dir % 2 != 0) ? 1.0f : -1.0f) : mk(h.pl.x, h.pl.y, 0.0f);
    q = add(h.pl, No);
  } else if (shape == CODE_CONE) {
    if (dir == 1) { N = mk(0.0f, 0.0f, 0.0f); return; }
    if (dir == 0) q = mk(h.pl.x, h.pl.y, h.pl.z - 1.0f);
    else {
      float lxy = sqrt_rn(__builtin_fmaf(h.pl.y, h.pl.y, h.pl.x * h.pl.x));
      q = add(h.pl, mk(h.pl.x, h.pl.y, lxy / 2.0f));
    }
  } else if (shape == CODE_QUAD) {
    q = add(h.pl, mk(0.0f, 0.0f, 1.0f));
  } else {   // CODE_MESH: mesh_inter_geom_info :783-810 (smooth unless flat_face)
    if constexpr (SR::kMesh) {
      ev.inc(EV_MGEOM);
      const int4 mi = s.minfo[s.ptype[h.index()] >> 4];
      const int4 vi = s.mtris[mi.w + h.tri];
      const float4 a4 = s.mverts[vi.x], b4 = s.mverts[vi.y], c4 = s.mverts[vi.z];
      const f3 A = mk(a4.x, a4.y, a4.z), Bv = mk(b4.x, b4.y, b4.z), C = mk(c4.x, c4.y, c4.z);
      if (s.flat_face) {
        q = add(h.pl, cross3(sub(Bv, A), sub(C, A)));
      } else {
        const float4 na = s.mnorms[vi.x], nb = s.mnorms[vi.y], nc = s.mnorms[vi.z];
        const f3 PA = sub(A, h.pl), PB = sub(Bv, h.pl), PC = sub(C, h.pl);
        const float tA = length3(cross3(PB, PC)), tB = length3(cross3(PA, PC)), tC = length3(cross3(PA, PB));
        const f3 No = add(add(muls(mk(na.x, na.y, na.z), tA), muls(mk(nb.x, nb.y, nb.z), tB)),
                          muls(mk(nc.x, nc.y, nc.z), tC));
        q = add(h.pl, No);
      }
    } else {
      return;
    }
  }
  N = normalize3(sub(xpoint(t0, t1, t2, q), P));
}

// sample_hemisphere + random_ray tp/montecarlo.frag:49-89
//
// Range checks the sampler's operands never fail are dropped (same bits):
//  * log(1 - u): 1 - u in [2^-23, 1] (mc_log_unit);
//  * 1/sqrt(1 + tanTheta2): one range test for the pair (rsqrt_rn = RN(1/RN(sqrt)));
//  * sqrt(max(0, 1 - c^2)): the operand is 0 or >= 2^-24 (1 - RN(c^2) with RN(c^2) <= 1 is
//    exact), where sqrt_core is exact;
//  * the local sample's normalize: |(cos b sin t, sin b sin t, cos t)|^2 is 1 within a few
//    ulp for every finite angle pair (NaN stays NaN either way), where rcp_core(sqrt_core)
//    is exact.
// Scene 6 +1.4..+1.9 %, scene 3 +2.5 %, scenes 1 / 8 +0.4..+0.8 % over the checked sequences
// (profiles/r02_ab19_rr_short.jsonl).
__device__ __forceinline__ f3 random_ray(Rng& rng, f3 D, float roughness) {
  f3 W = normalize3(mk(D.x, D.y + 5.0f, D.z + 3.0f));
  f3 U = normalize3(cross3(D, W));
  f3 V = normalize3(cross3(D, U));
  float alpha = roughness * roughness;
  float beta = (2.0f * kPI) * rnd(rng);
  float tanTheta2 = ((-alpha) * alpha) * mc_log_unit(1.0f - rnd(rng));
  float cosTheta = rsqrt_rn(1.0f + tanTheta2);
  const float s2 = gmax(0.0f, 1.0f - cosTheta * cosTheta);
  float sinTheta = sqrt_core(s2);
  float sb, cb;
  mc_sincos(beta, sb, cb);
  const f3 sl = mk(cb * sinTheta, sb * sinTheta, cosTheta);
  f3 sm = muls(sl, rcp_core(sqrt_core(dot3(sl, sl))));
  f3 m = mk(__builtin_fmaf(D.x, sm.z, __builtin_fmaf(V.x, sm.y, U.x * sm.x)),
            __builtin_fmaf(D.y, sm.z, __builtin_fmaf(V.y, sm.y, U.y * sm.x)),
            __builtin_fmaf(D.z, sm.z, __builtin_fmaf(V.z, sm.y, U.z * sm.x)));
  return normalize3(m);
}

// r0 = ((ior-1)/(ior+1))^2 (:93-94), computed once on the host (RenderParams::schlick_r0)
// one_m_r0 = 1 - r0 (binary32; RenderParams::schlick_1mr0)
__device__ __forceinline__ float schlick(float r0, float one_m_r0, f3 I, f3 N) {   // :91-98
  float x = 1.0f - dot3(N, I);
  return gclamp(r0 + ((((one_m_r0) * x) * x * x) * x) * x, 0.0f, 1.0f);
}
__device__ __forceinline__ float schlick(float r0, f3 I, f3 N) { return schlick(r0, 1.0f - r0, I, N); }

__device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// raytracer.vert:9-22: the camera ray of screen position (u, v) — the 4 corner rays
// interpolated over the strip triangles (v0,v1,v2) / (v1,v3,v2), normalized
__device__ __forceinline__ f3 camera_dir(const RenderParams& p, float u, float v) {
  const f3 d0 = mk(p.cd[0], p.cd[1], p.cd[2]), d1 = mk(p.cd[3], p.cd[4], p.cd[5]);
  const f3 d2 = mk(p.cd[6], p.cd[7], p.cd[8]), d3 = mk(p.cd[9], p.cd[10], p.cd[11]);
  f3 dir;
  if (u + v <= 1.0f) {
    float w0 = (1.0f - u) - v;
    dir = add(add(muls(d0, w0), muls(d1, u)), muls(d2, v));
  } else {
    float w1 = 1.0f - v, w3 = (u + v) - 1.0f, w2 = 1.0f - u;
    dir = add(add(muls(d1, w1), muls(d3, w3)), muls(d2, w2));
  }
  return normalize3(dir);
}

}  // namespace mcpt
