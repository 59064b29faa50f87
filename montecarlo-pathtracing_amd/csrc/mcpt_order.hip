// Work-item order of the render kernel (round 5): after a launch, its work items are sorted by
// the time each took (RenderParams::item_cost, the longest wave of the item on the 100 MHz
// real-time clock), costliest first; the next launch of the same shape deals its workgroups in
// that order (RenderParams::item_perm).  A launch ends when its last workgroup does: started
// late, a costly item (a tile whose paths run long — e.g. through the mesh instances) leaves
// the rest of the chip idle (longest-processing-time-first scheduling).  The order changes
// which workgroup runs an item, never what it computes: the results are the same bits.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include "mcpt_internal.h"

namespace mcpt {

__global__ void iota_kernel(int* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = i;
}

// How many of the costliest items to split (mesh launches): those costing more than half the
// launch's ideal span, sum(costs) / capacity (the concurrent workgroups), at most split_max.
// A launch cannot end before its longest item does; split in kSplitPieces pass ranges, a costly
// item's pieces run side by side instead of one after another.
__global__ __launch_bounds__(1024) void split_count_kernel(const unsigned* cost_sorted, int n, int capacity,
                                                           int split_max, int* out, unsigned long long* dbg) {
  __shared__ double s_sum[1024];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc += (double)cost_sorted[i];
  s_sum[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double lim = 0.5 * s_sum[0] / (double)(capacity > 0 ? capacity : 1);
  int lo = 0, hi = n < split_max ? n : split_max;   // first index whose cost <= lim
  while (lo < hi) {
    const int mid = (lo + hi) / 2;
    if ((double)cost_sorted[mid] > lim) lo = mid + 1; else hi = mid;
  }
  *out = lo;
  if (dbg) *dbg = (unsigned long long)lo;   // debug slot kDebugSplitSlot (mcpt_debug_counters)
}

}  // namespace mcpt

hipError_t mcpt_split_count(const unsigned* cost_sorted, int n, int capacity, int split_max, int* out,
                            unsigned long long* dbg, hipStream_t stream) {
  hipLaunchKernelGGL(mcpt::split_count_kernel, dim3(1), dim3(1024), 0, stream, cost_sorted, n, capacity, split_max, out,
                     dbg);
  return hipGetLastError();
}

hipError_t mcpt_iota(int* a, int n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mcpt::iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a, n);
  return hipGetLastError();
}

// temporary storage the sort of n items needs (tmp == nullptr: query)
hipError_t mcpt_order_items(const unsigned* cost, unsigned* cost_sorted, const int* iota, int* perm, int n,
                            void* tmp, size_t* tmp_bytes, hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortPairsDescending(tmp, *tmp_bytes, cost, cost_sorted, iota, perm, n, 0, 32,
                                                      stream);
}
