// Exhaustive proof, on the device, that the short division sequence of the arithmetic contract
// (csrc/mcpt_math.h div_core: y = rcp_core(b) = RN(1/b), q0 = RN(a y), r = a - b q0 (one fma,
// exact), q1 = RN(q0 + r y)) equals the correctly rounded quotient RN(a / b) -- the compiler's
// IEEE expansion, -fno-fast-math -- for every pair of binary32 significands: a, b in [1, 2),
// 2^23 x 2^23 = 2^46 pairs.  Signs and exponents scale every step exactly (RN is symmetric and
// commutes with powers of two) while no intermediate leaves the normal range, which
// div_core_ok's bounds (2^-60 <= |a|, |b| <= 2^60, or a == +0) guarantee: there y, q0 and q1 are
// normal and r is 0 or at least |a| 2^-47.  A randomized pass over signs and exponents inside
// those bounds (and around them) checks the wrapper div_rn, fallback included.
// Prints one JSON object; exit status 0 iff no mismatch.
//   make -C montecarlo-pathtracing_amd/csrc mathcheck   (-> tools/mathcheck/div_exhaustive)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../../montecarlo-pathtracing_amd/csrc/mcpt_math.h"

constexpr int kPerThread = 1 << 12;   // a significands per thread (one b each)

__global__ void check_pairs(unsigned long long base, unsigned long long* bad, unsigned long long* first) {
  const unsigned long long t = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t mb = (uint32_t)(t >> 11) | 0x800000u;            // divisor significand
  const uint32_t ma0 = ((uint32_t)(t & 2047u) << 12) | 0x800000u;  // first dividend significand
  const float b = __uint_as_float(0x3F800000u | (mb & 0x7FFFFFu));
  const float y = mcpt::rcp_core(b);
  unsigned long long n_bad = 0;
  uint32_t first_a = 0;
  for (int k = 0; k < kPerThread; ++k) {
    const float a = __uint_as_float(0x3F800000u | ((ma0 + (uint32_t)k) & 0x7FFFFFu));
    const float got = mcpt::div_core(a, b, y);
    const float want = a / b;
    if (__float_as_uint(got) != __float_as_uint(want)) {
      if (!n_bad) first_a = ma0 + (uint32_t)k;
      ++n_bad;
    }
  }
  if (n_bad) {
    atomicAdd(bad, n_bad);
    atomicMin(first, ((unsigned long long)mb << 32) | first_a);
  }
}

// xorshift64* stream per thread: random signs, exponents in [-70, 70], significands
__device__ __forceinline__ uint64_t next(uint64_t& s) {
  s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
  return s * 2685821657736338717ull;
}
__global__ void check_random(unsigned long long seed, unsigned long long* bad, unsigned long long* in_range) {
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(blockIdx.x * blockDim.x + threadIdx.x + 1));
  unsigned long long n_bad = 0, n_in = 0;
  for (int k = 0; k < 256; ++k) {
    const uint64_t r = next(s);
    const int ea = (int)((r >> 48) % 141) - 70, eb = (int)((r >> 56) % 141) - 70;
    const uint32_t ua = ((uint32_t)(r & 0x7FFFFFu)) | ((uint32_t)(ea + 127) << 23) | ((r >> 23) & 1u ? 0x80000000u : 0u);
    const uint32_t ub = ((uint32_t)((r >> 24) & 0x7FFFFFu)) | ((uint32_t)(eb + 127) << 23) | ((r >> 47) & 1u ? 0x80000000u : 0u);
    float a = __uint_as_float(ua), b = __uint_as_float(ub);
    if ((r & 0xFFu) == 0u) a = 0.0f;    // zero dividends too, both signs
    if ((r & 0xFFu) == 1u) a = -0.0f;
    n_in += mcpt::div_core_ok(a, b) ? 1u : 0u;
    const float got = mcpt::div_rn(a, b), want = a / b;
    if (__float_as_uint(got) != __float_as_uint(want)) ++n_bad;
  }
  atomicAdd(bad, n_bad);
  atomicAdd(in_range, n_in);
}

int main() {
  unsigned long long *bad = nullptr, *first = nullptr, *rbad = nullptr, *rin = nullptr;
  if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess || hipMalloc(&rbad, 8) != hipSuccess ||
      hipMalloc(&rin, 8) != hipSuccess || hipMemset(bad, 0, 8) != hipSuccess || hipMemset(first, 0xFF, 8) != hipSuccess ||
      hipMemset(rbad, 0, 8) != hipSuccess || hipMemset(rin, 0, 8) != hipSuccess) {
    std::printf("{\"error\": \"hip allocation failed\"}\n");
    return 2;
  }
  const unsigned long long threads = 1ull << 34, chunk = 1ull << 26;   // 2^34 threads x 2^12 pairs
  for (unsigned long long b0 = 0; b0 < threads; b0 += chunk) {
    hipLaunchKernelGGL(check_pairs, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b0, bad, first);
    if (((b0 / chunk) & 15u) == 15u) {   // progress on stderr (a long run must not look hung)
      if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("{\"error\": \"kernel failed\"}\n");
        return 2;
      }
      std::fprintf(stderr, "div_exhaustive: %llu / %llu divisor significands\n", (b0 + chunk) >> 11, threads >> 11);
    }
  }
  const unsigned rand_blocks = 1u << 16;   // 2^16 x 256 threads x 256 draws = 2^32 random pairs
  hipLaunchKernelGGL(check_random, dim3(rand_blocks), dim3(256), 0, 0, 12345ull, rbad, rin);
  unsigned long long h_bad = 0, h_first = 0, h_rbad = 0, h_rin = 0;
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&h_bad, bad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&h_first, first, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&h_rbad, rbad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&h_rin, rin, 8, hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("{\"error\": \"kernel failed\"}\n");
    return 2;
  }
  std::printf("{\"significand_pairs\": %llu, \"div_core_mismatches\": %llu", threads * kPerThread, h_bad);
  if (h_bad) std::printf(", \"first_mismatch\": {\"b_significand\": \"0x%06llx\", \"a_significand\": \"0x%06llx\"}",
                         h_first >> 32, h_first & 0xFFFFFFFFull);
  std::printf(", \"random_pairs\": %llu, \"random_in_range\": %llu, \"div_rn_mismatches\": %llu",
              (unsigned long long)rand_blocks * 256ull * 256ull, h_rin, h_rbad);
  std::printf(", \"exact\": %s}\n", (h_bad == 0 && h_rbad == 0) ? "true" : "false");
  return (h_bad == 0 && h_rbad == 0) ? 0 : 1;
}
