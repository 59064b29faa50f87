// Calibration of rocprofv3's VALU lane-utilisation counters on gfx950: the same chain of
// v_fma_f32 executed with 64, 32, 16 and 1 active lanes per wave (exec mask from a lane-id
// branch).  Run under `rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
// --kernel-trace`: SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU) should read 1, 1/2, 1/4,
// 1/64 if the counter ratio is the active-lane fraction (DESIGN.md §4.2 reads 0.34 for the
// render kernel from it).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;

template <int LANES>
__global__ __launch_bounds__(256) void k_lanes(float* out, float a, float b) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 0.001f + i;
  if ((int)(threadIdx.x & 63) < LANES) {
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(a), "v"(b));
    }
  }
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 8;
  float* out;
  if (hipMalloc(&out, sizeof(float) * blocks * 256) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_lanes<64>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
  hipLaunchKernelGGL(k_lanes<32>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
  hipLaunchKernelGGL(k_lanes<16>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
  hipLaunchKernelGGL(k_lanes<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("lane_util kernels done\n");
  hipFree(out);
  return 0;
}
