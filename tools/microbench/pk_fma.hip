// Issue cost of packed vs scalar f32 VALU on gfx950: chains of independent v_fma_f32 /
// v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (inline asm, 8 independent accumulators),
// 7 waves per SIMD like the render kernel.  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, float a, float b) {
  f2 x[8];
  const f2 va = {a, a}, vb = {b, b};
  for (int i = 0; i < 8; ++i) x[i] = (f2){threadIdx.x * 0.001f + i, 1.0f * i};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(va), "v"(vb));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkmul(float* out, float a, float b) {
  f2 x[8];
  const f2 va = {a, a};
  for (int i = 0; i < 8; ++i) x[i] = (f2){threadIdx.x * 0.001f + i, 1.0f * i};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(va));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mul(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
float run(K kern, float* out, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 7;   // 7 workgroups (of 4 waves) per CU = 7 waves per SIMD
  float* out;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  const double waves_per_simd = 7.0, instr = (double)ITERS * 8;
  const char* names[4] = {"v_fma_f32", "v_mul_f32", "v_pk_fma_f32", "v_pk_mul_f32"};
  float ms[4] = {run(k_scalar, out, blocks), run(k_mul, out, blocks), run(k_pkfma, out, blocks), run(k_pkmul, out, blocks)};
  printf("{");
  for (int k = 0; k < 4; ++k) {
    // cycles per wave-instruction per SIMD at 2.4 GHz
    const double cyc = ms[k] * 1e-3 * 2.4e9 / (waves_per_simd * instr);
    printf("%s\"%s\": {\"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.3f}", k ? ", " : "", names[k], ms[k], cyc);
  }
  printf("}\n");
  return 0;
}
