// Exhaustive proof, on the device, that the short square-root / reciprocal sequences of the
// arithmetic contract (csrc/mcpt_math.h: sqrt_rn, rcp_rn, and normalize's rsqrt_rn(x))
// equal the correctly rounded results (the compiler's IEEE expansions, -fno-fast-math) for
// every one of the 2^32 binary32 inputs.  Also reports how far the raw hardware
// instructions (v_sqrt_f32, v_rcp_f32, v_rsq_f32) are from correct rounding, for DESIGN.md.
// Prints one JSON object; exit status 0 iff the contract's sequences have no mismatch.
//   make -C montecarlo-pathtracing_amd/csrc mathcheck   (-> tools/mathcheck/exhaustive)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../../montecarlo-pathtracing_amd/csrc/mcpt_math.h"

constexpr int K = 6;

__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first) {
  const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t u = (uint32_t)i;
  const float x = __uint_as_float(u);
  const int e = (u >> 23) & 0xFF;
  const float s_cr = __builtin_sqrtf(x), r_cr = 1.0f / x, q_cr = 1.0f / s_cr;
  const float got[K] = {mcpt::sqrt_rn(x), mcpt::rcp_rn(x), mcpt::rsqrt_rn(x),
                        __builtin_amdgcn_sqrtf(x), __builtin_amdgcn_rcpf(x), __builtin_amdgcn_rsqf(x)};
  const float want[K] = {s_cr, r_cr, q_cr, s_cr, r_cr, q_cr};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const bool same = __float_as_uint(got[k]) == __float_as_uint(want[k]) || (got[k] != got[k] && want[k] != want[k]);
    if (!same) {
      atomicAdd(&bad[k * 256 + e], 1ull);
      atomicMin(&first[k * 256 + e], u);
    }
  }
}

int main() {
  unsigned long long* bad = nullptr;
  unsigned* first = nullptr;
  if (hipMalloc(&bad, K * 256 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&first, K * 256 * sizeof(unsigned)) != hipSuccess ||
      hipMemset(bad, 0, K * 256 * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(first, 0xFF, K * 256 * sizeof(unsigned)) != hipSuccess) {
    std::printf("{\"error\": \"hip allocation failed\"}\n");
    return 2;
  }
  const unsigned long long total = 1ull << 32, chunk = 1ull << 28;
  for (unsigned long long b = 0; b < total; b += chunk)
    hipLaunchKernelGGL(check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, b, bad, first);
  unsigned long long h[K * 256];
  unsigned f[K * 256];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("{\"error\": \"kernel failed\"}\n");
    return 2;
  }
  const char* names[K] = {"sqrt_rn", "rcp_rn", "rsqrt_rn", "hw v_sqrt_f32", "hw v_rcp_f32", "hw v_rsq_f32"};
  unsigned long long contract_bad = 0;
  std::printf("{\"inputs\": %llu", total);
  for (int k = 0; k < K; ++k) {
    unsigned long long tot = 0;
    int worst = -1;
    for (int e = 0; e < 256; ++e) {
      tot += h[k * 256 + e];
      if (h[k * 256 + e] && worst < 0) worst = e;
    }
    if (k < 3) contract_bad += tot;
    std::printf(", \"%s\": {\"mismatches\": %llu", names[k], tot);
    if (worst >= 0) std::printf(", \"first_exponent\": %d, \"first_input\": \"0x%08x\"", worst, f[k * 256 + worst]);
    // input exponents (biased) with mismatches, as [lo, hi] ranges
    std::printf(", \"exponent_ranges\": [");
    bool any = false;
    for (int e = 0; e < 256; ++e) {
      if (!h[k * 256 + e]) continue;
      int e2 = e;
      while (e2 + 1 < 256 && h[k * 256 + e2 + 1]) ++e2;
      std::printf("%s[%d, %d]", any ? ", " : "", e, e2);
      any = true;
      e = e2;
    }
    std::printf("]}");
  }
  std::printf(", \"contract_exact\": %s}\n", contract_bad == 0 ? "true" : "false");
  return contract_bad == 0 ? 0 : 1;
}
