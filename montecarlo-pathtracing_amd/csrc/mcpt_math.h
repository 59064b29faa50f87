// mcpt_math.h — binary32 arithmetic contract of the path tracer.
//
// Everything the integrator computes goes through these helpers so that the
// HIP kernel reproduces, bit for bit, the CPU restatement in oracle/ (which
// implements the same contract independently).  Rules:
//   * IEEE-754 binary32, round-to-nearest, built with -ffp-contract=off;
//   * dot products and matrix·vector products are explicit fmaf chains in
//     component order (x, then y, then z, then the translation column);
//   * sqrt and '/' are correctly rounded: '/' the HIP default expansion, sqrt and the
//     reciprocals 1/x through sqrt_rn / rcp_rn below, shorter sequences proven equal to the
//     correctly rounded results by an exhaustive check of all 2^32 inputs on gfx950
//     (tools/mathcheck, tests/test_gpu_mathcheck.py);
//   * normalize(v) = v * (1/sqrt(dot(v,v)));
//   * sin/cos/log/exp2/pow are the fixed polynomial algorithms below (GLSL leaves
//     their precision to the driver; ours are ≤ a few ulp and reproducible);
//   * GLSL min/max/clamp keep the GLSL definitions (max(x,y) = x<y ? y : x).
// Reference semantics: shaders/raytracer_func.frag, tp/montecarlo.frag (GLSL 4.30).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// MCPT_DRIVER_MATH (diagnostic builds only, never shipped: results differ from the oracle):
// the arithmetic a GL driver's shader compiler emits for the pieces GLSL leaves
// implementation-defined, so that the deviation of an *executed* GLSL render from the shipped
// contract can be measured at equal RNG seeds (tests/test_gpu_driver_math.py).
// Bits: 1 = raw v_sqrt_f32 / v_rcp_f32 / v_rsq_f32 for sqrt, 1/x, inversesqrt (normalize,
// length); 2 = hardware v_sin_f32 / v_cos_f32 / v_log_f32 / v_exp_f32 for sin, cos, log, exp2
// and pow = exp2(y log2 x); 4 = a / b as a * v_rcp_f32(b) in the primitive tests.
#ifndef MCPT_DRIVER_MATH
#define MCPT_DRIVER_MATH 0
#endif

namespace mcpt {

constexpr bool kDriverRoots = (MCPT_DRIVER_MATH & 1) != 0;
constexpr bool kDriverTrans = (MCPT_DRIVER_MATH & 2) != 0;
constexpr bool kDriverDiv = (MCPT_DRIVER_MATH & 4) != 0;

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }

// generic IEEE expansions, out of line: the rare slow paths of the short sequences below stay
// out of the register allocation of the hot code
__device__ __attribute__((noinline)) inline float sqrt_ieee(float x) { return __builtin_sqrtf(x); }
__device__ __attribute__((noinline)) inline float rcp_ieee(float x) { return 1.0f / x; }

// Short sequences for RN(sqrt(x)) and RN(1/x), checked against the correctly rounded results
// on all 2^32 inputs (tools/mathcheck/exhaustive.hip, tests/test_gpu_mathcheck.py):
//  * sqrt_core: the hardware root (~1 ulp) corrected by the signs of the exact residuals
//    x - s'·s of its two neighbours (7 VALU vs 16): exact except for 0 < |x| < 2^-96;
//  * rcp_core: the hardware reciprocal + one Newton step on the exact residual (3 VALU vs
//    11): exact for 2^-126 <= |x| < 2^126.
// The *_rn wrappers route the other inputs to the generic expansions, wave-uniformly.
__device__ __forceinline__ float sqrt_core(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  if constexpr (kDriverRoots) return s;
  const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
  float r = s;
  if (__builtin_fmaf(-sd, s, x) <= 0.0f) r = sd;
  if (__builtin_fmaf(-su, s, x) > 0.0f) r = su;
  return r;
}
__device__ __forceinline__ float rcp_core(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  if constexpr (kDriverRoots) return y;
  return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
}
__device__ __forceinline__ bool sqrt_core_ok(float x) { return !(__builtin_fabsf(x) < 0x1p-96f) || x == 0.0f; }
__device__ __forceinline__ bool rcp_core_ok(float x) {
  const float ax = __builtin_fabsf(x);
  return ax >= 0x1p-126f && ax < 0x1p126f;
}
__device__ __forceinline__ float sqrt_rn(float x) {
  if constexpr (kDriverRoots) return __builtin_amdgcn_sqrtf(x);
  float r = sqrt_core(x);
  const bool ok = sqrt_core_ok(x);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) r = sqrt_ieee(x);
  }
  return r;
}
__device__ __forceinline__ float rcp_rn(float x) {
  if constexpr (kDriverRoots) return __builtin_amdgcn_rcpf(x);
  float r = rcp_core(x);
  const bool ok = rcp_core_ok(x);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) r = rcp_ieee(x);
  }
  return r;
}
// RN(1/RN(sqrt(x))), the factor of normalize: for 2^-96 <= x < 2^126 both cores are exact
// (the root lies in [2^-48, 2^63)): one range test for the pair
__device__ __forceinline__ float rsqrt_rn(float x) {
  if constexpr (kDriverRoots) return __builtin_amdgcn_rsqf(x);
  float r = rcp_core(sqrt_core(x));
  const bool ok = x >= 0x1p-96f && x < 0x1p126f;
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) r = rcp_ieee(sqrt_ieee(x));
  }
  return r;
}

// RN(a / b) from b's correctly rounded reciprocal y = RN(1/b) (rcp_core): q0 = RN(a y) is within
// an ulp of a / b, so r = a - b q0 is exact in one fma and q1 = RN(q0 + r y) is the correctly
// rounded quotient (Markstein's correction step; checked on all 2^46 significand pairs on gfx950,
// tools/mathcheck/div_exhaustive.hip, tests/test_gpu_mathcheck.py).  5 VALU against the 11 of the
// IEEE expansion, 3 of them shared by every division by the same b.  Exact for
// 2^-60 <= |a|, |b| <= 2^60 and for a == +0 (div_core_ok): there y, q0, q1 are normal and r is 0
// or at least |a| 2^-47; div_rn routes other operands to the IEEE expansion, wave-uniformly.
__device__ __forceinline__ float div_core(float a, float b, float y) {
  const float q = a * y;
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), y, q);
}
__device__ __forceinline__ bool div_b_ok(float b) {
  const float ab = __builtin_fabsf(b);
  return ab >= 0x1p-60f && ab <= 0x1p60f;
}
__device__ __forceinline__ bool div_a_ok(float a) {   // (+0 only: div_core turns -0 / b into +0)
  const float aa = __builtin_fabsf(a);
  return (aa >= 0x1p-60f && aa <= 0x1p60f) || __float_as_uint(a) == 0u;
}
__device__ __forceinline__ bool div_core_ok(float a, float b) { return div_a_ok(a) && div_b_ok(b); }
__device__ __attribute__((noinline)) inline float div_ieee(float a, float b) { return a / b; }
__device__ __forceinline__ float div_rn(float a, float b) {
  float q = div_core(a, b, rcp_core(b));
  const bool ok = div_core_ok(a, b);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) {
    if (!ok) q = div_ieee(a, b);
  }
  return q;
}

__device__ __forceinline__ float dot3(f3 a, f3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ f3 normalize3(f3 a) { return muls(a, rsqrt_rn(dot3(a, a))); }
__device__ __forceinline__ float length3(f3 a) { return sqrt_rn(dot3(a, a)); }
// the same with the generic expansions inline (for code inside the BVH walk loop, where the
// short sequences' fallback branches cost more registers than they save instructions)
__device__ __forceinline__ f3 normalize3_g(f3 a) {
  if constexpr (kDriverRoots) return muls(a, __builtin_amdgcn_rsqf(dot3(a, a)));
  float r = 1.0f / __builtin_sqrtf(dot3(a, a));
  return muls(a, r);
}
__device__ __forceinline__ float length3_g(f3 a) {
  if constexpr (kDriverRoots) return __builtin_amdgcn_sqrtf(dot3(a, a));
  return __builtin_sqrtf(dot3(a, a));
}
// the primitive tests' divisions (correctly rounded; MCPT_DRIVER_MATH & 4: a * rcp(b))
__device__ __forceinline__ float fdiv(float a, float b) {
  if constexpr (kDriverDiv) return a * __builtin_amdgcn_rcpf(b);
  return a / b;
}
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }
__device__ __forceinline__ float gclamp(float x, float a, float b) { return gmin(gmax(x, a), b); }
__device__ __forceinline__ float gmix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
__device__ __forceinline__ f3 gmix3(f3 x, f3 y, float a) { return mk(gmix(x.x, y.x, a), gmix(x.y, y.y, a), gmix(x.z, y.z, a)); }
__device__ __forceinline__ f3 greflect(f3 I, f3 N) { return sub(I, muls(N, 2.0f * dot3(N, I))); }
// eta_sq = eta * eta (binary32), passed in when the caller has it as a host-computed constant
__device__ __forceinline__ f3 grefract(f3 I, f3 N, float eta, float eta_sq) {
  float d = dot3(N, I);
  float k = 1.0f - eta_sq * (1.0f - d * d);
  if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
  // k >= 0 here is 0 or >= 2^-24 (1 - y for a float y < 1 is exact: y <= 1 - 2^-24, or
  // k > 0.5 when y < 0.5), or +inf / NaN: never in sqrt_core's inexact range (0, 2^-96)
  return sub(muls(I, eta), muls(N, eta * d + sqrt_core(k)));
}
__device__ __forceinline__ f3 grefract(f3 I, f3 N, float eta) { return grefract(I, N, eta, eta * eta); }

// 3x4 affine rows (row r = (m[r], m[4+r], m[8+r], m[12+r]) of a column-major mat4)
__device__ __forceinline__ f3 xpoint(float4 r0, float4 r1, float4 r2, f3 p) {
  return mk(__builtin_fmaf(r0.z, p.z, __builtin_fmaf(r0.y, p.y, r0.x * p.x)) + r0.w,
            __builtin_fmaf(r1.z, p.z, __builtin_fmaf(r1.y, p.y, r1.x * p.x)) + r1.w,
            __builtin_fmaf(r2.z, p.z, __builtin_fmaf(r2.y, p.y, r2.x * p.x)) + r2.w);
}
__device__ __forceinline__ f3 xdir(float4 r0, float4 r1, float4 r2, f3 d) {
  return mk(__builtin_fmaf(r0.z, d.z, __builtin_fmaf(r0.y, d.y, r0.x * d.x)),
            __builtin_fmaf(r1.z, d.z, __builtin_fmaf(r1.y, d.y, r1.x * d.x)),
            __builtin_fmaf(r2.z, d.z, __builtin_fmaf(r2.y, d.y, r2.x * d.x)));
}

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }

constexpr float kPI = 3.14159274101257324f;   // 2*acos(0) in binary32 (raytracer_func.frag:9)
constexpr float kEPS = 1e-10f;                // EPSILON raytracer_func.frag:13
constexpr float kBIAS = 1e-2f;                // BIAS raytracer_func.frag:14
constexpr float kFLTMAX = 3.402823e38f;       // FLT_MAX raytracer_func.frag:8

// sin/cos: Cody-Waite reduction by pi/2, minimax polynomials on [-pi/4, pi/4]
__device__ __forceinline__ void mc_sincos(float x, float& s_out, float& c_out) {
  if constexpr (kDriverTrans) {   // v_sin / v_cos take revolutions
    const float rev = x * 0.159154943091895336f;
    s_out = __builtin_amdgcn_sinf(rev);
    c_out = __builtin_amdgcn_cosf(rev);
    return;
  }
  float t = x * 0.636619746685028076f;
  float qf = __builtin_floorf(t + 0.5f);
  int q = (int)qf;
  float r = __builtin_fmaf(-qf, 1.57079637050628662f, x);
  r = __builtin_fmaf(-qf, -4.37113900018624283e-8f, r);
  r = __builtin_fmaf(-qf, -1.71512451e-15f, r);
  float s = r * r;
  float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, s, 8.3321608736e-3f), s, -1.6666654611e-1f);
  float sn = __builtin_fmaf(r * s, sp, r);
  float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, s, -1.388731625493765e-3f), s, 4.166664568298827e-2f);
  float cs = __builtin_fmaf(s * s, cp, __builtin_fmaf(-0.5f, s, 1.0f));
  int qq = q & 3;
  float a = (qq & 1) ? cs : sn;      // sin candidate
  float b = (qq & 1) ? sn : cs;      // cos candidate
  s_out = (qq & 2) ? -a : a;
  c_out = ((qq + 1) & 2) ? -b : b;
}

// natural log, normal positive finite x with bits b and exponent offset e (the polynomial
// shared by mc_log and its domain-restricted forms below)
__device__ __forceinline__ float mc_log_core(uint32_t b, int e) {
  e += (int)(b >> 23) - 127;
  float m = bitsf((b & 0x007FFFFFu) | 0x3F800000u);
  if (m > 1.41421353816986084f) { m = m * 0.5f; e += 1; }
  float f = m - 1.0f;
  float z = f * f;
  float p = 7.0376836292e-2f;
  p = __builtin_fmaf(p, f, -1.1514610310e-1f);
  p = __builtin_fmaf(p, f, 1.1676998740e-1f);
  p = __builtin_fmaf(p, f, -1.2420140846e-1f);
  p = __builtin_fmaf(p, f, 1.4249322787e-1f);
  p = __builtin_fmaf(p, f, -1.6668057665e-1f);
  p = __builtin_fmaf(p, f, 2.0000714765e-1f);
  p = __builtin_fmaf(p, f, -2.4999993993e-1f);
  p = __builtin_fmaf(p, f, 3.3333331174e-1f);
  float ef = (float)e;
  float y = (f * z) * p;
  y = __builtin_fmaf(ef, -2.12194440e-4f, y);
  y = __builtin_fmaf(-0.5f, z, y);
  float r = f + y;
  return __builtin_fmaf(ef, 0.693359375f, r);
}
// natural log (x > 0 finite expected; 0 -> -inf, <0/NaN -> NaN)
__device__ __forceinline__ float mc_log(float x) {
  if constexpr (kDriverTrans) return __builtin_amdgcn_logf(x) * 0.693147182464599609f;
  if (!(x > 0.0f)) return (x == 0.0f) ? -__builtin_inff() : __builtin_nanf("");
  if (x == __builtin_inff()) return x;
  uint32_t b = fbits(x);
  int e = 0;
  if (b < 0x00800000u) { x = x * 8388608.0f; b = fbits(x); e = -23; }
  return mc_log_core(b, e);
}
// mc_log for x in [2^-23, 1] (sample_hemisphere's log(1 - random_float()): random_float is a
// multiple of 2^-23 in [0, 1 - 2^-23], so 1 - u is exact, normal and positive): mc_log with
// its zero / negative / inf / subnormal cases dropped, none of which that domain reaches —
// same bits
__device__ __forceinline__ float mc_log_unit(float x) {
  if constexpr (kDriverTrans) return __builtin_amdgcn_logf(x) * 0.693147182464599609f;
  return mc_log_core(fbits(x), 0);
}

__device__ __forceinline__ float mc_exp2(float x) {
  if constexpr (kDriverTrans) return __builtin_amdgcn_exp2f(x);
  if (x != x) return x;
  if (x >= 128.0f) return __builtin_inff();
  if (x < -150.0f) return 0.0f;
  float kf = __builtin_floorf(x + 0.5f);
  float f = x - kf;
  float p = 1.535336188319500e-4f;
  p = __builtin_fmaf(p, f, 1.339887440266574e-3f);
  p = __builtin_fmaf(p, f, 9.618437357674640e-3f);
  p = __builtin_fmaf(p, f, 5.550332471162809e-2f);
  p = __builtin_fmaf(p, f, 2.402264791363012e-1f);
  p = __builtin_fmaf(p, f, 6.931472028550421e-1f);
  float r = __builtin_fmaf(p, f, 1.0f);
  int k = (int)kf;
  if (k >= -126) return r * bitsf((uint32_t)(k + 127) << 23);
  return (r * bitsf((uint32_t)(k + 127 + 64) << 23)) * 5.42101086242752217e-20f;
}

// pow for x in [0, 1 + a few ulp] (the specular term: max(0, dot) of unit vectors, NaN -> 0):
// mc_log's inf test is unreachable there; same bits as mc_pow
__device__ __forceinline__ float mc_pow_le1(float x, float y) {
  if constexpr (kDriverTrans) return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
  float l;
  if (!(x > 0.0f)) l = (x == 0.0f) ? -__builtin_inff() : __builtin_nanf("");
  else {
    uint32_t b = fbits(x);
    int e = 0;
    if (b < 0x00800000u) { x = x * 8388608.0f; b = fbits(x); e = -23; }
    l = mc_log_core(b, e);
  }
  return mc_exp2(y * (l * 1.44269502162933350f));
}
__device__ __forceinline__ float mc_pow(float x, float y) {
  if constexpr (kDriverTrans) return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
  return mc_exp2(y * (mc_log(x) * 1.44269502162933350f));
}

// xxhash32 RNG — raytracer_func.frag:90-124
__device__ __forceinline__ uint32_t xxhash32(uint32_t px, uint32_t py, uint32_t pz) {
  uint32_t h = pz + 374761393u + px * 3266489917u;
  h = 668265263u * ((h << 17) | (h >> 15));
  h += py * 3266489917u;
  h = 668265263u * ((h << 17) | (h >> 15));
  h = 2246822519u * (h ^ (h >> 15));
  h = 3266489917u * (h ^ (h >> 13));
  return h ^ (h >> 16);
}

struct Rng { uint32_t x, y, z; };
__device__ __forceinline__ float rnd(Rng& s) {
  uint32_t m = xxhash32(s.x, s.y, s.z);
  float f = bitsf((m & 0x007FFFFFu) | 0x3F800000u);
  s.x += 11u; s.y += 43u; s.z += 67u;
  return f - 1.0f;
}
// the state after k draws: random_float only adds (11, 43, 67) to the seed per draw, so a
// draw sequence can be entered at any position without computing the draws before it
__device__ __forceinline__ void rng_skip(Rng& s, uint32_t k) { s.x += 11u * k; s.y += 43u * k; s.z += 67u * k; }
// srand raytracer_func.frag:105-110
__device__ __forceinline__ Rng seed_for(float tcx, float tcy, int np, float date) {
  float f = (float)(1 + np);
  float mid = (float)np * 3.14f + date;
  Rng r;
  r.x = fbits((tcx * f) * 1.125f);
  r.y = fbits((mid * f) * 1.125f);
  r.z = fbits((tcy * f) * 1.125f);
  return r;
}

}  // namespace mcpt
