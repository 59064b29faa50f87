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

}  // namespace mcpt

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
