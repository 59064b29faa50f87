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
//    the 0..B bounce lengths average out.  Work items = (32x8 tile, pass segment), so
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
#include "mcpt_math.h"
#include "mcpt_internal.h"

// minimum waves per SIMD the register allocator must allow (occupancy vs spills)
#ifndef MCPT_MIN_WAVES
#define MCPT_MIN_WAVES 7
#endif
// sky fold (render_kernel): a bounce ray that misses the scene starts the lane's next pass in
// the same round
#ifndef MCPT_FOLD_SKY
#define MCPT_FOLD_SKY 1
#endif
// end fold: emissive hits and hits at bounce B-1 (black) end the pass before the shading block
#ifndef MCPT_FOLD_END
#define MCPT_FOLD_END 1
#endif


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
  // meshes (mcpt_upload_meshes): per mesh (first node, first leaf, depth, first triangle)
  const int4* __restrict__ minfo;
  const float4* __restrict__ mnodes;  // 3 per node, mesh space
  const int* __restrict__ mleaves;    // mesh-local triangle ids or -1
  const int4* __restrict__ mtris;     // global vertex ids (a, b, c, 0)
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
__device__ __forceinline__ uint32_t bperm(int lane, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(lane << 2, (int)v);
}
__device__ __forceinline__ float bpermf(int lane, float v) { return __uint_as_float(bperm(lane, __float_as_uint(v))); }

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
  LS_SHADE_WV, LS_SHADE_LN, LS_RR2_WV, LS_RR2_LN, LS_WAVES, LS_FIT_IT, LS_TWO_IT, LS_COUNT
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

// intersect_bv raytracer_func.frag:314-352; divisions as hoisted reciprocals (contract).
// WAVE: the all-lanes-inside early out is taken wave-uniformly (big boxes such as the
// ground's contain every ray origin).
template <bool WAVE>
__device__ __forceinline__ bool box_test(float4 a0, float4 a1, float4 a2, f3 O, f3 D, f3 invD, double cull2) {
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  const bool inside = __builtin_fabsf(Oi.x) < 1.0f && __builtin_fabsf(Oi.y) < 1.0f && __builtin_fabsf(Oi.z) < 1.0f;
  if (WAVE && __ballot(!inside) == 0) return true;
  if (inside) return true;
  f3 rD = mulv(invD, w);
  // faces in reference order: (x,-1) (x,+1) (y,-1) (y,+1) (z,-1) (z,+1).  Branch-free:
  // every face is evaluated and the valid minimum kept with a select (`if (a < al) al = a`
  // == min(al, valid ? a : FLT_MAX) for the non-NaN a a valid face has); bitwise & keeps
  // the compares in SGPR masks instead of exec-mask branches (+5 % Msamples/s, r01_ab4).
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
#define MCPT_FACE(CD, OA, DV, RA, OB, DB, OC, DC)                                              \
  {                                                                                            \
    const float a = ((CD) - (OA)) * (RA);                                                      \
    const bool ok = (DV) & (a > kEPS) & (__builtin_fabsf(OB + a * DB) <= 1.0f) &               \
                    (__builtin_fabsf(OC + a * DC) <= 1.0f);                                    \
    al = __builtin_fminf(al, ok ? a : kFLTMAX);                                                \
  }
  MCPT_FACE(-1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(-1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(-1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
  MCPT_FACE(1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
#undef MCPT_FACE
  if (al < kFLTMAX) {
    f3 Pg = add(mulv(add(muls(Di, al), Oi), w), c);
    f3 v = sub(O, Pg);
    return (double)dot3(v, v) < cull2;
  }
  return false;
}

// box_test without branches (MCPT_BOX_SELECT): the same operations for every lane, the outcome
// chosen by selects.  Returns the key the cull compares: -1 when the origin is inside the box
// (always pushed), the squared distance to the entry point when a face is valid, +inf when
// none is; (double)key < cull2 is box_test's result bit for bit (same operations on the lanes
// box_test runs them on; cull2 > 0).  No exec-mask branches: the deep walk's node block keeps
// every lane in one instruction stream (SALU / branch bookkeeping, verdict r03).
__device__ __forceinline__ float box_key(float4 a0, float4 a1, float4 a2, f3 O, f3 D, f3 invD) {
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  const bool inside = (__builtin_fabsf(Oi.x) < 1.0f) & (__builtin_fabsf(Oi.y) < 1.0f) & (__builtin_fabsf(Oi.z) < 1.0f);
  f3 rD = mulv(invD, w);
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
#define MCPT_FACE(CD, OA, DV, RA, OB, DB, OC, DC)                                              \
  {                                                                                            \
    const float a = ((CD) - (OA)) * (RA);                                                      \
    const bool ok = (DV) & (a > kEPS) & (__builtin_fabsf(OB + a * DB) <= 1.0f) &               \
                    (__builtin_fabsf(OC + a * DC) <= 1.0f);                                    \
    al = __builtin_fminf(al, ok ? a : kFLTMAX);                                                \
  }
  MCPT_FACE(-1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(-1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(-1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
  MCPT_FACE(1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
#undef MCPT_FACE
  f3 Pg = add(mulv(add(muls(Di, al), Oi), w), c);
  f3 v = sub(O, Pg);
  const float d2 = dot3(v, v);
  return inside ? -1.0f : (al < kFLTMAX ? d2 : __builtin_inff());
}
#ifndef MCPT_BOX_SELECT
#define MCPT_BOX_SELECT 0
#endif
#ifndef MCPT_FACE_PAIR
#define MCPT_FACE_PAIR 0
#endif
#ifndef MCPT_FACE_JOBS
#define MCPT_FACE_JOBS 0
#endif

// The face loop of intersect_bv (raytracer_func.frag:330-343) on a box-local ray: the smallest
// valid face parameter, kFLTMAX when no face is valid (box_test's operations).
__device__ __forceinline__ float face_min(f3 Oi, f3 Di, f3 rD) {
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
#define MCPT_FACE(CD, OA, DV, RA, OB, DB, OC, DC)                                              \
  {                                                                                            \
    const float a = ((CD) - (OA)) * (RA);                                                      \
    const bool ok = (DV) & (a > kEPS) & (__builtin_fabsf(OB + a * DB) <= 1.0f) &               \
                    (__builtin_fabsf(OC + a * DC) <= 1.0f);                                    \
    al = __builtin_fminf(al, ok ? a : kFLTMAX);                                                \
  }
  MCPT_FACE(-1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(-1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(-1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
  MCPT_FACE(1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
#undef MCPT_FACE
  return al;
}
__device__ __forceinline__ f3 sel3(bool c, f3 a, f3 b) { return mk(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

// MCPT_FACE_PAIR: a node visit's two box tests with their face loops paired up per lane.  A lane
// needs the face loop for a child that holds a primitive and whose box does not contain the ray
// origin; the wave ran the left child's loop for the lanes that need it and then the right
// child's, whenever any lane needed either.  Here every lane runs its first needed loop (left,
// else right) in one pass, and a second pass runs only when some lane needs both.  Each child's
// decision uses box_test's operations on the same values (same bits).
__device__ __forceinline__ void node_tests_paired(float4 l0, float4 l1, float4 l2, float4 r0, float4 r1, float4 r2,
                                                  f3 O, f3 D, f3 invD, double cull2, bool& hl, bool& hr) {
  const f3 cl = mk(l0.x, l0.y, l0.z), wl = mk(l1.x, l1.y, l1.z), iwl = mk(l2.x, l2.y, l2.z);
  const f3 cr = mk(r0.x, r0.y, r0.z), wr = mk(r1.x, r1.y, r1.z), iwr = mk(r2.x, r2.y, r2.z);
  const f3 Oil = mulv(sub(O, cl), iwl), Dil = mulv(D, iwl);
  const f3 Oir = mulv(sub(O, cr), iwr), Dir = mulv(D, iwr);
  const bool in_l = (__builtin_fabsf(Oil.x) < 1.0f) & (__builtin_fabsf(Oil.y) < 1.0f) & (__builtin_fabsf(Oil.z) < 1.0f);
  const bool in_r = (__builtin_fabsf(Oir.x) < 1.0f) & (__builtin_fabsf(Oir.y) < 1.0f) & (__builtin_fabsf(Oir.z) < 1.0f);
  const bool ne_l = l0.w != 0.0f, ne_r = r0.w != 0.0f;
  const bool need_l = ne_l & !in_l, need_r = ne_r & !in_r;
  float al_l = kFLTMAX, al_r = kFLTMAX;
  if (__ballot(need_l | need_r)) {
    const f3 rDl = mulv(invD, wl), rDr = mulv(invD, wr);
    const float a1 = face_min(sel3(need_l, Oil, Oir), sel3(need_l, Dil, Dir), sel3(need_l, rDl, rDr));
    al_l = need_l ? a1 : kFLTMAX;
    al_r = (!need_l & need_r) ? a1 : kFLTMAX;
    if (__ballot(need_l & need_r)) {
      const float a2 = face_min(Oir, Dir, rDr);
      if (need_l & need_r) al_r = a2;
    }
  }
  auto cull = [&](float al, f3 Oi, f3 Di, f3 w, f3 c) {
    f3 Pg = add(mulv(add(muls(Di, al), Oi), w), c);
    f3 v = sub(O, Pg);
    return (al < kFLTMAX) & ((double)dot3(v, v) < cull2);
  };
  hl = ne_l & (in_l | cull(al_l, Oil, Dil, wl, cl));
  hr = ne_r & (in_r | cull(al_r, Oir, Dir, wr, cr));
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
template <bool COUNT, class SR>
__device__ __forceinline__ void node_tests(const SR& s, const float4* __restrict__ nodes, size_t j, f3 O, f3 D,
                                           f3 invD, double cull2, bool& hl, bool& hr) {
  if constexpr (!SR::kLds && !SR::kMesh) {
    const float4* q = node_rows(nodes, j);
    float4 l0 = q[0], l1 = q[1], l2 = q[2], r0 = q[3], r1 = q[4], r2 = q[5];
    MCPT_ROWS_IN("v"(l0.x), "v"(l0.y), "v"(l0.z), "v"(l0.w), "v"(l1.x), "v"(l1.y), "v"(l1.z), "v"(l2.x),
                 "v"(l2.y), "v"(l2.z));
    MCPT_ROWS_IN("v"(r0.x), "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z), "v"(r2.x),
                 "v"(r2.y), "v"(r2.z));
    if constexpr (MCPT_FACE_PAIR && !COUNT) {
      node_tests_paired(l0, l1, l2, r0, r1, r2, O, D, invD, cull2, hl, hr);
    } else if constexpr (MCPT_BOX_SELECT && !COUNT) {
      const float kl = box_key(l0, l1, l2, O, D, invD), kr = box_key(r0, r1, r2, O, D, invD);
      hl = (l0.w != 0.0f) & ((double)kl < cull2);
      hr = (r0.w != 0.0f) & ((double)kr < cull2);
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
__device__ __forceinline__ bool box_test_mesh(float4 a0, float4 a1, float4 a2, f3 O, f3 D, f3 invD, f3 Ol,
                                              float4 t0, float4 t1, float4 t2, double cull2) {
  f3 c = mk(a0.x, a0.y, a0.z), w = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
  f3 Oi = mulv(sub(O, c), iw);
  f3 Di = mulv(D, iw);
  if (__builtin_fabsf(Oi.x) < 1.0f && __builtin_fabsf(Oi.y) < 1.0f && __builtin_fabsf(Oi.z) < 1.0f) return true;
  f3 rD = mulv(invD, w);
  const bool dx = __builtin_fabsf(Di.x) > kEPS, dy = __builtin_fabsf(Di.y) > kEPS, dz = __builtin_fabsf(Di.z) > kEPS;
  float al = kFLTMAX;
#define MCPT_FACE(CD, OA, DV, RA, OB, DB, OC, DC)                                              \
  {                                                                                            \
    const float a = ((CD) - (OA)) * (RA);                                                      \
    const bool ok = (DV) & (a > kEPS) & (__builtin_fabsf(OB + a * DB) <= 1.0f) &               \
                    (__builtin_fabsf(OC + a * DC) <= 1.0f);                                    \
    al = __builtin_fminf(al, ok ? a : kFLTMAX);                                                \
  }
  MCPT_FACE(-1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(1.0f, Oi.x, dx, rD.x, Oi.y, Di.y, Oi.z, Di.z)
  MCPT_FACE(-1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(1.0f, Oi.y, dy, rD.y, Oi.z, Di.z, Oi.x, Di.x)
  MCPT_FACE(-1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
  MCPT_FACE(1.0f, Oi.z, dz, rD.z, Oi.x, Di.x, Oi.y, Di.y)
#undef MCPT_FACE
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

// Triangle_intersect raytracer_func.frag:354-396 (Möller–Trumbore, mesh space); a hit keeps
// the mesh-local triangle index in Hit::dir (the reference's tri_index; its dir is 0)
template <bool COUNT, class SR>
__device__ __forceinline__ void tri_test(const SR& s, int tri_base, int t, int index, f3 O, f3 D, f3 Ol,
                                         float4 t0, float4 t1, float4 t2, Hit& h, Ev<COUNT>& ev) {
  ev.inc(EV_TRI);
  const int4 vi = s.mtris[tri_base + t];
  const float4 a4 = s.mverts[vi.x], b4 = s.mverts[vi.y], c4 = s.mverts[vi.z];
  const f3 vA = mk(a4.x, a4.y, a4.z), vB = mk(b4.x, b4.y, b4.z), vC = mk(c4.x, c4.y, c4.z);
  const f3 edge1 = sub(vB, vA), edge2 = sub(vC, vA);
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

// Mesh_intersect raytracer_func.frag:642-678: the instance's own BVH, same DFS as
// intersect_bvh (right child first, cull at push with intersect_bvm), stackless per lane
template <bool COUNT, bool ANY, class SR>
__device__ __forceinline__ void mesh_test(const SR& s, int mesh, int index, f3 O, f3 D, f3 Ol, Hit& h,
                                          Ev<COUNT>& ev) {
  ev.inc(EV_MESH);
  const int4 mi = s.minfo[mesh];   // first node, first leaf, depth, first triangle
  const size_t b = (size_t)index * 8;
  const float4 t0 = s.prims[b + 3], t1 = s.prims[b + 4], t2 = s.prims[b + 5];   // read_mesh_transfo
  const float4* nodes = s.mnodes + (size_t)mi.x * 3;
  const f3 invD = mk(rcp_rn(D.x), rcp_rn(D.y), rcp_rn(D.z));
  const int leaf0 = (1 << mi.z) - 1;
  int node = 0, level = 0;
  uint32_t pending = 0;
  for (;;) {
    bool pop = true;
    if (node >= leaf0) {
      ev.inc(EV_LEAF);
      const int t = s.mleaves[mi.y + node - leaf0];
      if (t >= 0) {
        tri_test<COUNT>(s, mi.w, t, index, O, D, Ol, t0, t1, t2, h, ev);
        if (ANY && h.hit()) return;   // hit_only (:664-665)
      }
    } else {
      ev.inc(EV_NODE);
      const size_t j = 2 * (size_t)node + 1;
      const float4 l0 = nodes[j * 3], r0 = nodes[j * 3 + 3];   // (mesh kernels: see node_tests)
      bool hl = (COUNT || l0.w != 0.0f) &&
                box_test_mesh(l0, nodes[j * 3 + 1], nodes[j * 3 + 2], O, D, invD, Ol, t0, t1, t2, h.cull2);
      bool hr = (COUNT || r0.w != 0.0f) &&
                box_test_mesh(r0, nodes[j * 3 + 4], nodes[j * 3 + 5], O, D, invD, Ol, t0, t1, t2, h.cull2);
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

#ifndef MCPT_ONE_ACCEPT
#define MCPT_ONE_ACCEPT 0
#endif
// intersect_prim raytracer_func.frag:681-705 + Sphere/Cube/Cylinder/Cone/OrientedQuad :398-640
template <bool COUNT, bool UNI, bool ANY = false, class SR>
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
  // MCPT_ONE_ACCEPT: the type branches only record their candidate (the sphere's near and far
  // roots: two) and one accept site after the switch tests it against the hit record, so a leaf
  // block whose lanes hold several primitive types runs the candidate code (transform rows,
  // world point, length, compare, record update) once instead of once per type.  Each lane's
  // candidates reach the hit record in the same order (same bits).
  bool has1 = false, has2 = false;
  int shape1 = 0, dir1 = 0;
  f3 P1 = mk(0.0f, 0.0f, 0.0f), P2 = P1;
  auto accept = [&](int shape, int dir, f3 Pl) {
    if constexpr (MCPT_ONE_ACCEPT) { has1 = true; shape1 = shape; dir1 = dir; P1 = Pl; }
    else accept_cand<COUNT, UNI>(s, i, shape, dir, Pl, Ow, h, ev);
  };
  auto accept_far = [&](f3 Pl) {   // the sphere's far root, after its near root
    if constexpr (MCPT_ONE_ACCEPT) { has2 = true; P2 = Pl; }
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
      float a = fdiv(-(OD + sq), D2);
      if (a > kEPS) accept(CODE_SPHERE, 0, add(O, muls(D, a)));
      a = fdiv(-(OD - sq), D2);
      if (a > kEPS) accept_far(add(O, muls(D, a)));
    }
  } else if (t == CODE_QUAD) {
    if (!(D.z > -kEPS)) {
      float a = fdiv(-O.z, D.z);
      f3 Pl = add(O, muls(D, a));
      if (!(__builtin_fabsf(Pl.x) > 1.0f || __builtin_fabsf(Pl.y) > 1.0f)) accept(CODE_QUAD, 0, Pl);
    }
  } else if (t == CODE_CUBE) {
    float al = kFLTMAX; int cl = 0;
    float o[3] = {O.x, O.y, O.z}, d[3] = {D.x, D.y, D.z};
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const int c0 = f / 2, c1 = (c0 + 1) % 3, c2 = (c0 + 2) % 3;
      if (__builtin_fabsf(d[c0]) > kEPS) {
        const float cd = (f % 2) ? 1.0f : -1.0f;
        float a = fdiv(cd - o[c0], d[c0]);
        if ((a > kEPS) && (__builtin_fabsf(o[c1] + a * d[c1]) <= 1.0f) && (__builtin_fabsf(o[c2] + a * d[c2]) <= 1.0f))
          if (a < al) { al = a; cl = f; }
      }
    }
    if (al < kFLTMAX) accept(CODE_CUBE, cl, add(O, muls(D, al)));
  } else if (t == CODE_CYLINDER) {
    int cl = -1; float al = kFLTMAX;
    if (__builtin_fabsf(D.z) > kEPS) {
      float a = fdiv(-1.0f - O.z, D.z);
      if (a > kEPS) {
        float rx = O.x + a * D.x, ry = O.y + a * D.y;
        if ((__builtin_fmaf(ry, ry, rx * rx) < 1.0f) && (a < al)) { cl = 0; al = a; }
      }
      a = fdiv(1.0f - O.z, D.z);
      if (a > kEPS) {
        float rx = O.x + a * D.x, ry = O.y + a * D.y;
        if ((__builtin_fmaf(ry, ry, rx * rx) < 1.0f) && (a < al)) { cl = 1; al = a; }
      }
    }
    float O2 = __builtin_fmaf(O.y, O.y, O.x * O.x);
    float OD = __builtin_fmaf(O.y, D.y, O.x * D.x);
    float D2 = __builtin_fmaf(D.y, D.y, D.x * D.x);
    float delta4 = OD * OD - D2 * (O2 - 1.0f);
    if (delta4 > 0.0f) {
      float a = fdiv(-(OD + wsqrt<SR::kFastSqrt>(delta4)), D2);
      if ((a > kEPS) && (a < al)) {
        float z = O.z + a * D.z;
        if (__builtin_fabsf(z) < 1.0f) { cl = 2; al = a; }
      }
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
    if constexpr (SR::kMesh) mesh_test<COUNT, ANY>(s, pt >> 4, i, O, D, Ow, h, ev);
  }
  if constexpr (MCPT_ONE_ACCEPT) {
    if (has1) accept_cand<COUNT, UNI>(s, i, shape1, dir1, P1, Ow, h, ev);
    if (has2) accept_cand<COUNT, UNI>(s, i, CODE_SPHERE, 0, P2, Ow, h, ev);
  }
}

// intersect_bvh raytracer_func.frag:734-769, per lane, stackless.  pending bit L = "a left
// sibling at level L waits on the reference's stack"; popping the deepest pending bit is
// exactly the reference's LIFO order (right child first, cull decided at push time).
// ANY: just_hit_bvh (raytracer_func.frag:771-775) — stop at the first leaf whose primitive
// produced a hit (hit_only, :756-757); the render path always uses traverse_all_bvh.
template <bool COUNT, bool ANY = false, class SR>
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
      node_tests<COUNT>(s, s.nodes, j, O, D, invD, h.cull2, hl, hr);
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
  uint32_t mpending;
  f3 Om, Dm, invDm;
  int4 mi;                 // the mesh's (first node, first leaf, depth, first triangle)
  float4 t0, t1, t2;       // the instance's mesh transform rows
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
  const int leaf0 = (1 << s.depth) - 1;
  const int n0 = SUSPEND ? __builtin_popcountll(__ballot(1)) : 0;
#ifdef MCPT_LANESTATS
  ls_add(LS_WALK_CALLS, 1u);
#endif
  for (;;) {
    bool pop = true;
    bool is_leaf = w.node >= leaf0;
    bool do_leaf = is_leaf, do_node = !is_leaf;
    if (SUSPEND && leaf_batch > 0) {   // wave-uniform choice of the block
      const uint64_t on_leaf = __ballot(is_leaf), act = __ballot(1);
      const bool leaves = __builtin_popcountll(on_leaf) >= leaf_batch || on_leaf == act;
      do_leaf = leaves && is_leaf;
      do_node = !leaves && !is_leaf;
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
      node_tests<COUNT>(s, s.nodes, j, O, D, w.invD, h.cull2, hl, hr);
      pop = !(hl || hr);
      if (hr) {
        if (hl) w.pending |= 1u << (w.level + 1);
        w.node = (int)j + 1; w.level++;
      } else if (hl) {
        w.node = (int)j; w.level++;
      }
    }
    if (pop && (do_leaf || do_node)) {
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


// MCPT_FACE_JOBS: walk_run for the deep kernel with the box tests' face loops compacted across
// the wave (north star: ray compaction through wavefront primitives).  In a node iteration a
// lane needs the face loop of a child that holds a primitive and whose box does not contain the
// ray origin (lane accounting, scene 8: 28.7 lanes per face block, 1.97 face blocks per node
// iteration).  Here those (lane, child) face jobs are numbered by ballot + mbcnt and run by
// ALL lanes of the call -- the lanes waiting on a leaf and the lanes whose walk has ended stay in
// the loop as workers -- in ceil(jobs / lanes) passes instead of one pass per child.  A worker
// pulls its job owner's ray (O, D, 1/D), node pair and cull bound with ds_bpermute, loads the
// child's rows itself, runs intersect_bv's face loop and cull, and the owner pulls the push
// decision back.  Every decision is box_test's, on the same values, at the same point of the
// owner's walk (same bits).  LDS: rank -> lane and job -> owner tables, 192 B per wave.
__device__ __forceinline__ unsigned char* jobs_lds() {
  __shared__ unsigned char s_jobs[kTileThreads / 64][192];
  return s_jobs[threadIdx.x >> 6];
}
template <class SR>
__device__ __forceinline__ bool walk_run_jobs(const SR& s, f3 O, f3 D, Hit& h, Walk& w, int exit, int leaf_batch,
                                              int min_done) {
  Ev<false> ev;
  const int leaf0 = (1 << s.depth) - 1;
  const int lane = (int)__lane_id();
  const uint64_t A = __ballot(1);
  const int n0 = __builtin_popcountll(A), rank = mbcnt64(A);
  unsigned char* wl = jobs_lds();        // [0, 64): rank -> lane
  unsigned char* own = jobs_lds() + 64;  // [64, 192): job -> owner lane
  wl[rank] = (unsigned char)lane;
  __builtin_amdgcn_wave_barrier();
  bool alive = true;
  for (;;) {
    const bool is_leaf = alive && w.node >= leaf0;
    const uint64_t on_leaf = __ballot(is_leaf), walking = __ballot(alive);
    const bool leaves = __builtin_popcountll(on_leaf) >= leaf_batch || on_leaf == walking;   // wave-uniform
    bool pop = false;
    if (leaves) {
      if (is_leaf) {
        const int p = s.leaves[(uint32_t)(w.node - leaf0)];
        if (p >= 0) prim_test<false, false, false>(s, p, O, D, h, ev);
        pop = true;
      }
    } else {
      const bool do_node = alive && !is_leaf;
      const uint32_t jn = 2u * (uint32_t)(do_node ? w.node : 0) + 1u;
      const float4* q = node_rows(s.nodes, jn);
      const float4 l0 = q[0], l1 = q[2], r0 = q[3], r1 = q[5];   // centre + flag, 1/half-width
      MCPT_ROWS_IN("v"(l0.x), "v"(l0.y), "v"(l0.z), "v"(l0.w), "v"(l1.x), "v"(l1.y), "v"(l1.z), "v"(r0.x),
                   "v"(r0.y), "v"(r0.z), "v"(r0.w), "v"(r1.x), "v"(r1.y), "v"(r1.z));
      const f3 Oil = mulv(sub(O, mk(l0.x, l0.y, l0.z)), mk(l1.x, l1.y, l1.z));
      const f3 Oir = mulv(sub(O, mk(r0.x, r0.y, r0.z)), mk(r1.x, r1.y, r1.z));
      const bool in_l = (__builtin_fabsf(Oil.x) < 1.0f) & (__builtin_fabsf(Oil.y) < 1.0f) & (__builtin_fabsf(Oil.z) < 1.0f);
      const bool in_r = (__builtin_fabsf(Oir.x) < 1.0f) & (__builtin_fabsf(Oir.y) < 1.0f) & (__builtin_fabsf(Oir.z) < 1.0f);
      const bool ne_l = l0.w != 0.0f, ne_r = r0.w != 0.0f;
      const bool need_l = do_node & ne_l & !in_l, need_r = do_node & ne_r & !in_r;
      const uint64_t mL = __ballot(need_l), mR = __ballot(need_r);
      const int nL = __builtin_popcountll(mL), nJ = nL + __builtin_popcountll(mR);
      const int sL = mbcnt64(mL), sR = nL + mbcnt64(mR);
      if (need_l) own[sL] = (unsigned char)lane;
      if (need_r) own[sR] = (unsigned char)lane;
      __builtin_amdgcn_wave_barrier();
      bool pass_l = false, pass_r = false;
      for (int base = 0; base < nJ; base += n0) {   // wave-uniform
        const int jj = base + rank;
        const bool has = jj < nJ;
        const int o = has ? (int)own[jj] : lane;
        const bool right = jj >= nL;
        const f3 Oo = mk(bpermf(o, O.x), bpermf(o, O.y), bpermf(o, O.z));
        const f3 Do = mk(bpermf(o, D.x), bpermf(o, D.y), bpermf(o, D.z));
        const f3 iDo = mk(bpermf(o, w.invD.x), bpermf(o, w.invD.y), bpermf(o, w.invD.z));
        const uint32_t jo = bperm(o, jn) + (right ? 1u : 0u);   // the child's row triple
        const uint64_t cb = __double_as_longlong(h.cull2);
        const double c2o = __longlong_as_double((long long)(((uint64_t)bperm(o, (uint32_t)(cb >> 32)) << 32) |
                                                            (uint64_t)bperm(o, (uint32_t)cb)));
        const float4* qc = node_rows(s.nodes, jo);
        const float4 a0 = qc[0], a1 = qc[1], a2 = qc[2];
        MCPT_ROWS_IN("v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a2.x), "v"(a2.y),
                     "v"(a2.z));
        const f3 c = mk(a0.x, a0.y, a0.z), wd = mk(a1.x, a1.y, a1.z), iw = mk(a2.x, a2.y, a2.z);
        const f3 Oi = mulv(sub(Oo, c), iw), Di = mulv(Do, iw), rD = mulv(iDo, wd);
        const float al = face_min(Oi, Di, rD);
        const f3 Pg = add(mulv(add(muls(Di, al), Oi), wd), c);
        const f3 v = sub(Oo, Pg);
        const bool ok = has & (al < kFLTMAX) & ((double)dot3(v, v) < c2o);
        // owners pull their jobs' decisions from the workers of this pass
        const bool gl = need_l & (sL >= base) & (sL < base + n0), gr = need_r & (sR >= base) & (sR < base + n0);
        const int wkl = gl ? (int)wl[sL - base] : lane, wkr = gr ? (int)wl[sR - base] : lane;
        const uint32_t okl = bperm(wkl, ok ? 1u : 0u), okr = bperm(wkr, ok ? 1u : 0u);
        if (gl) pass_l = okl != 0u;
        if (gr) pass_r = okr != 0u;
      }
      __builtin_amdgcn_wave_barrier();   // own[] is rewritten next iteration
      if (do_node) {
        const bool hl = ne_l & (in_l | pass_l), hr = ne_r & (in_r | pass_r);
        pop = !(hl || hr);
        if (hr) {
          if (hl) w.pending |= 1u << (w.level + 1);
          w.node = (int)jn + 1; w.level++;
        } else if (hl) {
          w.node = (int)jn; w.level++;
        }
      }
    }
    if (pop) {
      if (w.pending == 0) {
        alive = false;
      } else {
        const int L = 31 - __builtin_clz(w.pending);
        w.pending &= ~(1u << L);
        w.node = ((w.node + 1) >> (w.level - L)) - 2;
        w.level = L;
      }
    }
    const int n = __builtin_popcountll(__ballot(alive));   // wave-uniform
    if (n == 0 || (n <= exit && n0 - n >= min_done)) return !alive;
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
  for (;;) {
    bool pop = false;   // the scene walk pops its stack this iteration
    if (w.mprim >= 0) {
      // one step of the instance's mesh walk (mesh_test's loop body)
      const int4 mi = w.mi;
      const float4 t0 = w.t0, t1 = w.t1, t2 = w.t2;
      const int mleaf0 = (1 << mi.z) - 1;
      bool mpop = true;
      if (w.mnode >= mleaf0) {
        ev.inc(EV_LEAF);
        const int t = s.mleaves[mi.y + w.mnode - mleaf0];
        if (t >= 0) tri_test<COUNT>(s, mi.w, t, w.mprim, w.Om, w.Dm, O, t0, t1, t2, h, ev);
      } else {
        ev.inc(EV_NODE);
        const float4* nodes = s.mnodes + (size_t)mi.x * 3;
        const size_t j = 2 * (size_t)w.mnode + 1;
        const float4 l0 = nodes[j * 3], r0 = nodes[j * 3 + 3];   // (mesh kernels: see node_tests)
        const bool hl = (COUNT || l0.w != 0.0f) &&
                        box_test_mesh(l0, nodes[j * 3 + 1], nodes[j * 3 + 2], w.Om, w.Dm, w.invDm, O, t0, t1, t2, h.cull2);
        const bool hr = (COUNT || r0.w != 0.0f) &&
                        box_test_mesh(r0, nodes[j * 3 + 4], nodes[j * 3 + 5], w.Om, w.Dm, w.invDm, O, t0, t1, t2, h.cull2);
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
          // intersect_prim's transforms, then the mesh walk starts with the next iteration
          ev.inc(EV_PRIM);
          ev.inc(EV_MESH);
          const size_t b = (size_t)p * 8;
          const float4 r0 = s.prims[b], r1 = s.prims[b + 1], r2 = s.prims[b + 2];
          w.Om = xpoint(r0, r1, r2, O);
          w.Dm = wnormalize3<SR::kFastNorm>(xdir(r0, r1, r2, D));
          w.invDm = mk(rcp_rn(w.Dm.x), rcp_rn(w.Dm.y), rcp_rn(w.Dm.z));
          w.mprim = p; w.mi = s.minfo[pt >> 4];
          w.t0 = s.prims[b + 3]; w.t1 = s.prims[b + 4]; w.t2 = s.prims[b + 5];
          w.mnode = 0; w.mlevel = 0; w.mpending = 0;
          pop = false;
        } else {
          prim_test<COUNT, false, false>(s, p, O, D, h, ev);
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
    if (pop) {
      if (w.pending == 0) return true;
      const int L = 31 - __builtin_clz(w.pending);
      w.pending &= ~(1u << L);
      w.node = ((w.node + 1) >> (w.level - L)) - 2;
      w.level = L;
    }
    if (SUSPEND) {   // wave-uniform
      const int n = __builtin_popcountll(__ballot(1));
      if (n <= exit && n < n0) return false;
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

template <bool COUNT, bool WAVE, class SR>
__device__ __forceinline__ void traverse(const SR& s, f3 O, f3 D, Hit& h, Ev<COUNT>& ev) {
  if (WAVE) traverse_wave<COUNT>(s, O, D, h, ev);
  else traverse_lane<COUNT>(s, O, D, h, ev);
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
// MCPT_RR_SHORT drops range checks the sampler's operands never fail (same bits):
//  * log(1 - u): 1 - u in [2^-23, 1] (mc_log_unit);
//  * 1/sqrt(1 + tanTheta2): one range test for the pair (rsqrt_rn = RN(1/RN(sqrt)));
//  * sqrt(max(0, 1 - c^2)): the operand is 0 or >= 2^-24 (1 - RN(c^2) with RN(c^2) <= 1 is
//    exact), where sqrt_core is exact;
//  * the local sample's normalize: |(cos b sin t, sin b sin t, cos t)|^2 is 1 within a few
//    ulp for every finite angle pair (NaN stays NaN either way), where rcp_core(sqrt_core)
//    is exact.
// Bits 1 / 2 / 4 / 8 select the four in that order.  All four: scene 6 +1.4..+1.9 %, scene 3
// +2.5 %, scenes 1 / 8 +0.4..+0.8 % (profiles/r02_ab19_rr_short.jsonl); the C2 kernel then keeps
// 12 B of scratch, stored once in the prologue and reloaded only on the segment flush.
#ifndef MCPT_RR_SHORT
#define MCPT_RR_SHORT 15
#endif
__device__ __forceinline__ f3 random_ray(Rng& rng, f3 D, float roughness) {
  f3 W = normalize3(mk(D.x, D.y + 5.0f, D.z + 3.0f));
  f3 U = normalize3(cross3(D, W));
  f3 V = normalize3(cross3(D, U));
  float alpha = roughness * roughness;
  float beta = (2.0f * kPI) * rnd(rng);
  float tanTheta2 = ((-alpha) * alpha) * ((MCPT_RR_SHORT & 1) ? mc_log_unit(1.0f - rnd(rng)) : mc_log(1.0f - rnd(rng)));
  float cosTheta = (MCPT_RR_SHORT & 2) ? rsqrt_rn(1.0f + tanTheta2) : rcp_rn(sqrt_rn(1.0f + tanTheta2));
  const float s2 = gmax(0.0f, 1.0f - cosTheta * cosTheta);
  float sinTheta = (MCPT_RR_SHORT & 4) ? sqrt_core(s2) : sqrt_rn(s2);
  float sb, cb;
  mc_sincos(beta, sb, cb);
#if MCPT_RR_SHORT & 8
  const f3 sl = mk(cb * sinTheta, sb * sinTheta, cosTheta);
  f3 sm = muls(sl, rcp_core(sqrt_core(dot3(sl, sl))));
#else
  f3 sm = normalize3(mk(cb * sinTheta, sb * sinTheta, cosTheta));
#endif
  f3 m = mk(__builtin_fmaf(D.x, sm.z, __builtin_fmaf(V.x, sm.y, U.x * sm.x)),
            __builtin_fmaf(D.y, sm.z, __builtin_fmaf(V.y, sm.y, U.y * sm.x)),
            __builtin_fmaf(D.z, sm.z, __builtin_fmaf(V.z, sm.y, U.z * sm.x)));
  return normalize3(m);
}

// r0 = ((ior-1)/(ior+1))^2 (:93-94), computed once on the host (RenderParams::schlick_r0)
__device__ __forceinline__ float schlick(float r0, f3 I, f3 N) {   // :91-98
  float x = 1.0f - dot3(N, I);
  return gclamp(r0 + ((((1.0f - r0) * x) * x * x) * x) * x, 0.0f, 1.0f);
}


// ------------------------------------------------------------------------------------
// the kernel
// ------------------------------------------------------------------------------------
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

// Work item = (32x8 pixel tile of four 8x8 waves, group of seg_per_item pass segments).  A
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
template <bool COUNT, bool WAVE, bool MESH, bool LDSS, bool SUSPEND>
// per-lane walks of mesh scenes (walk_run_mesh keeps the mesh walk state, ray in mesh space
// and instance transform in registers): 4 waves/SIMD, 128 VGPRs (tools/big_mesh_bench.py:
// 7 waves with that state spills and runs at a third of the speed)
#ifndef MCPT_MIN_WAVES_MESH
#define MCPT_MIN_WAVES_MESH 4
#endif
// per-lane walks over scenes read through L1/L2 (not LDS-staged: scenes 3, 5, 7, 8): 6 waves/SIMD
// while their state spilled at 7 (profiles/r01_ab35_occupancy_v12.jsonl); with the packed hit
// record they fit 72 VGPRs and 7 waves hide more of the dependent node loads (scene 8 +4 %,
// scene 3 +5 %: profiles/r02_ab4_spill_free.jsonl)
#ifndef MCPT_MIN_WAVES_L2
#define MCPT_MIN_WAVES_L2 7
#endif
__global__ __launch_bounds__(kTileThreads, MESH && !WAVE ? MCPT_MIN_WAVES_MESH
                                           : (!WAVE && !LDSS ? MCPT_MIN_WAVES_L2 : MCPT_MIN_WAVES)) void render_kernel(
    RenderParams p) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int item = blockIdx.x;
  // segment-fastest item order: the pass segments of one tile are consecutive workgroups
  // (tile-fastest order was 1-12 % slower on one GPU and 7 % on a 1/8-row shard's launch:
  // profiles/r01_ab42_item_order.jsonl)
  // A work item runs K = seg_per_item consecutive segments of its tile; a lane runs its pixel's
  // segments one after another (each summed from 0 in pass order, written when it ends).
  const int K = p.seg_per_item > 1 ? p.seg_per_item : 1;
  const int n_groups = (p.n_segments + K - 1) / K;
  const int tile = item / n_groups, seg_lo = (item % n_groups) * K;
  const int seg_n = min(K, p.n_segments - seg_lo);
  int seg = seg_lo;
  const int tiles_x = (p.W + kTileW - 1) / kTileW;
  const int bx0 = (tile % tiles_x) * kTileW + (wave % (kTileW / 8)) * 8;   // this wave's 8x8 block
  const int by0 = (tile / tiles_x) * kTileH + (wave / (kTileW / 8)) * 8;
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
  const int y = live ? p.rows[lr] : 0;   // this shard's local row -> image row (mcpt_set_target*)

  SceneT<MESH, LDSS> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mnodes, p.mleaves, p.mtris,
                       p.mverts, p.mnorms, p.flat_face};
  if constexpr (LDSS) {
    // staged layout: nodes (3 float4 each), prims (8 float4 each), leaves, type codes
    extern __shared__ float4 s_scene[];
    const int n_nodes = (2 << p.depth) - 1, n_leaves = 1 << p.depth;
    const int n4 = 3 * n_nodes + 8 * p.n_prims;
    for (int i = tid; i < n4; i += kTileThreads) s_scene[i] = i < 3 * n_nodes ? p.nodes[i] : p.prims[i - 3 * n_nodes];
    int* s_int = (int*)(s_scene + n4);
    for (int i = tid; i < n_leaves + p.n_prims; i += kTileThreads)
      s_int[i] = i < n_leaves ? p.leaves[i] : p.ptype[i - n_leaves];
    __syncthreads();
    s.nodes = s_scene;
    s.prims = s_scene + 3 * n_nodes;
    s.leaves = s_int;
    s.ptype = s_int + n_leaves;
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
  // 19 KB per workgroup, + the staged scene (LDSS, <= kLdsSceneBytes): 7 workgroups/CU.
  __shared__ float s_pix[18][kTileThreads];
  __shared__ int s_hit0[kTileThreads];
  const f3 Dcam0 = camera_dir(p, u, v);
  s_pix[0][tid] = Dcam0.x; s_pix[1][tid] = Dcam0.y; s_pix[2][tid] = Dcam0.z;
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
    traverse<COUNT, WAVE>(s, Ocam, Dcam0, h, ev);
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
    // the pixel's address is recomputed at each flush (an empty asm makes the row opaque):
    // hoisted out of the render loop, its 64-bit index and pointer were 4 spilled VGPRs
    int lrow = lr, col = x;
    asm volatile("" : "+v"(lrow), "+v"(col));
    const size_t px = (size_t)lrow * p.W + col;
    if (p.n_segments == 1) {
      float* accp = p.accum + px * 3;
      accp[0] = accp[0] + s_pix[12][tid]; accp[1] = accp[1] + s_pix[13][tid]; accp[2] = accp[2] + s_pix[14][tid];
    } else {
      float* part = p.partial + ((size_t)seg * p.n_local_px + px) * 3;
      part[0] = s_pix[12][tid]; part[1] = s_pix[13][tid]; part[2] = s_pix[14][tid];
    }
  };
  // after pass++: the segment's last pass closes it (its sum to the segment slot) and the lane
  // goes on with its pixel's next segment of the work item.  With none left, pass stays at
  // pass_end and the lane leaves the loop.
  auto next_chunk = [&]() {
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
  walk.invD = mk(0.0f, 0.0f, 0.0f); walk.node = 0; walk.level = 0; walk.pending = 0;
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
        h.code = s_hit0[tid];
      } else if (WAVE) {
        traverse<COUNT, WAVE>(s, O, D, h, ev);
      } else {
        if (!walking) { walk_begin<COUNT>(s, D, h, walk, ev, p.cull2_max); walking = true; }
        if constexpr (MESH) walking = !walk_run_mesh<COUNT, SUSPEND>(s, O, D, h, walk, ev, p.walk_exit);
        else if constexpr (MCPT_FACE_JOBS && SUSPEND && !COUNT && !LDSS) {
          if (p.leaf_batch > 0) walking = !walk_run_jobs(s, O, D, h, walk, p.walk_exit, p.leaf_batch, p.walk_min_done);
          else walking = !walk_run<COUNT, SUSPEND>(s, O, D, h, walk, ev, p.walk_exit, p.leaf_batch, p.walk_min_done);
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
#if MCPT_FOLD_SKY
    // Sky fold: a bounce ray that left the scene ends its pass here, before the shading
    // block, and the lane starts its next pass at once with the cached primary hit, so
    // that one shading block serves both (the pass's camera-ray round, in which this
    // lane would otherwise only shade while the others traverse, disappears).  Same
    // per-lane sequence of values: the sky term, the segment sum in pass order, then the
    // next pass from its seed.
    //
    // End fold (MCPT_FOLD_END): the other two path ends known before shading fold the same
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
#if MCPT_FOLD_END
        const float4 m4 = s.prims[(size_t)h.index() * 8 + 7];
        if (!(m4.z <= 0.5f)) {   // the shading block's emissive `else`, NaN included
          const float4 c4 = s.prims[(size_t)h.index() * 8 + 6];
          fres = add(total, add(muls(mk(c4.x, c4.y, c4.z), 0.1f), muls(muls(muls(att, m4.z), 1.0f - m4.x), c4.w)));
        } else if (bounce < B - 1) {
          fold_end = false;
        }
#else
        fold_end = false;
#endif
      }
    }
    if (fold_end) {
      s_pix[12][tid] = s_pix[12][tid] + fres.x;
      s_pix[13][tid] = s_pix[13][tid] + fres.y;
      s_pix[14][tid] = s_pix[14][tid] + fres.z;
      ev.inc(EV_SAMPLE);
      pass++;
      next_chunk();
      if (pass < pass_end) {
        rng = seed_for(((float)x + 0.5f) / (float)p.W, ((float)y + 0.5f) / (float)p.H, pass, p.date);
        O = Ocam; D = mk(s_pix[0][tid], s_pix[1][tid], s_pix[2][tid]);
        att = mk(0.8f, 0.8f, 0.8f); total = mk(0.0f, 0.0f, 0.0f);
        bounce = 0;
        h.code = s_hit0[tid];
        first = true;
      } else {
        ready = false;   // unit finished: the lane claims another at the end of the round
      }
    }
#endif
    if (ready && run) {
      if (p.variant != 0) {
        // tp/montecarlo_mat.frag:5-20 / montecarlo_mat_tr.frag:5-20
        if (!h.hit()) {
          res = mk(0.0f, 0.0f, 0.2f);
        } else {
          if (first) {
            N = mk(s_pix[3][tid], s_pix[4][tid], s_pix[5][tid]);
            P = mk(s_pix[6][tid], s_pix[7][tid], s_pix[8][tid]);
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
            N = mk(s_pix[3][tid], s_pix[4][tid], s_pix[5][tid]);
            P = mk(s_pix[6][tid], s_pix[7][tid], s_pix[8][tid]);
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
          float rs = schlick(p.schlick_r0, D, N);
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
              D = grefract(D, N, ior);
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
        D = grefract(D, neg(N), p.inv_ior);
        phase = 0;
        bounce++;
        if (bounce >= B) done = true;
      }
    }
    if (done) {
      s_pix[12][tid] = s_pix[12][tid] + res.x;
      s_pix[13][tid] = s_pix[13][tid] + res.y;
      s_pix[14][tid] = s_pix[14][tid] + res.z;
      ev.inc(EV_SAMPLE);
      pass++;
      next_chunk();
      rng = seed_for(((float)x + 0.5f) / (float)p.W, ((float)y + 0.5f) / (float)p.H, pass, p.date);   // = (u, v)
      O = Ocam; D = mk(s_pix[0][tid], s_pix[1][tid], s_pix[2][tid]);
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
#ifndef MCPT_MIN_WAVES_STREAM
#define MCPT_MIN_WAVES_STREAM 8
#endif
// the shade kernel streams payloads from HBM: occupancy over registers
#ifndef MCPT_MIN_WAVES_SHADE
#define MCPT_MIN_WAVES_SHADE 5
#endif
// queue entries a trace wave claims (one atomic) and stages in LDS at once
#ifndef MCPT_STREAM_CHUNK
#define MCPT_STREAM_CHUNK 128
#endif
constexpr int kStreamChunk = MCPT_STREAM_CHUNK;
// trace waves stage each claimed chunk in order of the rays' direction octants
#ifndef MCPT_STREAM_SORT
#define MCPT_STREAM_SORT 1
#endif
static_assert(kStreamChunk % 64 == 0, "chunks are staged 64 entries per step");

// Field columns through a buffer resource: the column offset f * n * 4 is a wave-uniform
// scalar (soffset) and the entry offset i * 4 one 32-bit VGPR shared by every field, so no
// 64-bit per-lane address is formed or kept per field (with plain pointers the compiler
// strength-reduced ~40 columns into live 64-bit addresses and spilled them).  Buffers stay
// below 2 GiB (host check).  0x00020000: the gfx9 raw-buffer descriptor word 3.
// Queue payloads are streamed once per iteration: their loads and stores carry the
// non-temporal hint (MCPT_STREAM_NT, aux bit 1: nt on gfx950) so that they do not evict the
// BVH records the walks read through L2.
#ifndef MCPT_STREAM_NT
#define MCPT_STREAM_NT 1
#endif
constexpr int kQueueAux = MCPT_STREAM_NT ? 2 : 0;
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
  static constexpr int kBlock = 256, kWaves = 4, kChunk = kStreamChunk, kMinWaves = MCPT_MIN_WAVES_STREAM;
};
template <> struct TraceCfg<true> {
  static constexpr int kBlock = 1024, kWaves = 16, kChunk = 64, kMinWaves = 4;
};
// LDS of the LDSN trace kernel besides its scene copy: the waves' staged rays
constexpr int kTraceLdsStaging = TraceCfg<true>::kWaves * TraceCfg<true>::kChunk * 32;

template <bool LDSN>
__global__ __launch_bounds__(TraceCfg<LDSN>::kBlock, TraceCfg<LDSN>::kMinWaves) void stream_trace_kernel(StreamParams q) {
  typedef TraceCfg<LDSN> C;
  constexpr int kChunkT = C::kChunk;
  const RenderParams& p = q.r;
  SceneT<false, false> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mnodes, p.mleaves,
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
        // direction octant (MCPT_STREAM_SORT): lanes that take consecutive staged rays then
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
            key[g] = MCPT_STREAM_SORT ? ((ed[g].x < 0.0f) | ((ed[g].y < 0.0f) << 1) | ((ed[g].z < 0.0f) << 2)) : 0;
          }
        }
#pragma unroll
        for (int o = 0; o < (MCPT_STREAM_SORT ? 8 : 1); ++o) {
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
  };
  int r = -1;                // queue index of this lane's ray
  f3 O = mk(0.0f, 0.0f, 0.0f), D = O;
  Hit h;
  h.pl = O; h.dist = kFLTMAX; h.clear(); h.tri = 0; h.cull2 = 0.0;
  Walk w;
  w.invD = O; w.node = 0; w.level = 0; w.pending = 0;
  for (;;) {
    take(r, O, D, h, w);
    if (__ballot(r >= 0) == 0) break;   // nothing staged and nothing left to claim
    if (r >= 0) {
      if (walk_run<false, true>(s, O, D, h, w, ev, q.refill, p.leaf_batch)) {
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
__device__ __forceinline__ bool stream_shade(const StreamParams& q, const Cols& Qi, uint32_t i, const SlotCols& Sl,
                                             int slot, Payload& out) {
  const RenderParams& p = q.r;
  const SceneT<false, false> s{p.nodes, p.leaves, p.ptype, p.prims, p.depth, p.minfo, p.mnodes, p.mleaves,
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
  h.pl = Qi.ld3(QF_HX, i); h.code = (int)Qi.ldu(QF_HCODE, i); h.dist = 0.0f; h.tri = 0; h.cull2 = 0.0;
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

__global__ __launch_bounds__(kStreamBlock, MCPT_MIN_WAVES_SHADE) void stream_shade_kernel(StreamParams q) {
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
    const bool cont = slot >= 0 && stream_shade(q, Qi, i, Sl, slot, pl);
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

// ------------------------------------------------------------------------------------
// ray queries: the shader library's traverse_all_bvh / just_hit_bvh / intersect_one_prim /
// hit_one_prim + intersection_info + intersection_color_info / _mat_info
// (raytracer_func.frag:718-781, 874-907) for caller-supplied rays, one lane per ray
// ------------------------------------------------------------------------------------
template <bool ANY, bool MESH>
__global__ __launch_bounds__(256) void trace_kernel(TraceParams q) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= q.n) return;
  SceneT<MESH> s{q.nodes, q.leaves, q.ptype, q.prims, q.depth, q.minfo, q.mnodes, q.mleaves, q.mtris, q.mverts,
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
  dim3 block(mcpt::kTileThreads), grid((unsigned)items);
  const bool wave = p.wave_traversal != 0, mesh = p.n_meshes > 0;
  const bool lds = !mesh && p.lds_scene_bytes > 0;
  // deep-BVH walk kernel: suspendable walks and/or batched leaf visits (walk_run)
  const bool susp = !count && !wave && (p.walk_exit > 0 || p.leaf_batch > 0);
  const size_t shm = lds ? (size_t)p.lds_scene_bytes : 0;
#define MCPT_RENDER(C, W, M, L, S) \
  hipLaunchKernelGGL((mcpt::render_kernel<C, W, M, L, S>), grid, block, shm, stream, p)
#define MCPT_RENDER_CW(C, W, S)                       \
  if (mesh) MCPT_RENDER(C, W, true, false, S);        \
  else if (lds) MCPT_RENDER(C, W, false, true, S);    \
  else MCPT_RENDER(C, W, false, false, S)
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
  if (p.n_segments <= 1 || p.n_local_px <= 0) return hipSuccess;
  dim3 block(256), grid((unsigned)((p.n_local_px + 255) / 256));
  if (p.pass_split)
    hipLaunchKernelGGL(mcpt::combine_split_kernel, grid, block, 0, stream, p.accum, p.partial, p.n_local_px,
                       p.first_pass, p.n_passes);
  else
    hipLaunchKernelGGL(mcpt::combine_kernel, grid, block, 0, stream, p.accum, p.partial, p.n_local_px, p.n_segments);
  return hipGetLastError();
}

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
  if (lds_nodes) {
    const size_t shm = (size_t)mcpt_stream_lds_nodes_bytes(q.r.depth);
    // above the default 64 KiB of dynamic LDS (set on the calling thread's current device)
    e = hipFuncSetAttribute((const void*)mcpt::stream_trace_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024 - mcpt::kTraceLdsStaging);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mcpt::stream_trace_kernel<true>, dim3((unsigned)n_cu), dim3(mcpt::TraceCfg<true>::kBlock), shm,
                       stream, q);
  } else {
    hipLaunchKernelGGL(mcpt::stream_trace_kernel<false>, dim3((unsigned)n_cu * 8), dim3(mcpt::kStreamBlock), 0, stream,
                       q);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned persistent_blocks = (unsigned)n_cu * 8;
  hipLaunchKernelGGL(mcpt::stream_shade_kernel, dim3(persistent_blocks), dim3(mcpt::kStreamBlock), 0, stream, q);
  return hipGetLastError();
}
