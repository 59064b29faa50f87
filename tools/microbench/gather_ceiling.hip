// Random-record gather ceiling on gfx950: the memory rate the mesh walk's access pattern allows.
// The mesh walk (mcpt_device.h walk_run_mesh) is, per lane, a chain of dependent 64-byte record
// reads at random places of a 128 MB (mesh) / 400 MB (mesh_big) record array.  This program
// measures, on the same chip, what such reads can reach without the walk's arithmetic:
//   chain    each lane reads one 64-B record per step; the next record's index comes from the
//            record just read (a dependent chain, like a walk step)
//   chain2   as chain, plus one more 64-B record per step whose index is known one step ahead
//            (the walk's request of its children's line)
//   indep    each lane reads 4 independent random 64-B records per step (no dependence: the
//            throughput ceiling of random 64-B reads)
//   line     as indep with whole 128-B lines (8 x 16 B per lane)
//   stream   consecutive 16-B words, coalesced (the streaming ceiling, for comparison)
// over working sets of 64 MB .. 4 GB and 2 / 4 / 5 / 8 waves per SIMD (the grid holds exactly
// that many one-wave workgroups per SIMD: 1,024 SIMDs).  Prints one JSON line per case: the
// record bytes read per second (GB/s) and the fraction of 8 TB/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/gather_ceiling tools/microbench/gather_ceiling.hip
//   tools/microbench/gather_ceiling [working sets in MB, comma-separated] [waves per SIMD, comma-separated]
//
// Every index is scaled into the array (high half of index x count); every loop has a fixed
// trip count; the only stores are one vector store per lane at the end.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

// a uniform index in [0, n) from a 32-bit value
__device__ __forceinline__ uint32_t below(uint32_t v, uint32_t n) { return (uint32_t)(((uint64_t)v * n) >> 32); }

__global__ void fill(uint4* buf, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t k = (uint32_t)(i * 4);
    buf[i] = make_uint4(mix(k), mix(k + 1), mix(k + 2), mix(k + 3));
  }
}

__device__ __forceinline__ uint32_t rec_word(const uint4* r) {
  // every word of the record is used, so each 16-B piece is a full dwordx4 load as in the walk
  const uint4 a = r[0], b = r[1], c = r[2], d = r[3];
  return (a.x ^ a.y ^ a.z ^ a.w) + (b.x ^ b.y ^ b.z ^ b.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w);
}

// MODE 0 chain, 1 chain2, 2 indep, 3 line, 4 stream
template <int MODE>
__global__ __launch_bounds__(64) void gather(const uint4* __restrict__ buf, uint32_t n_rec, int steps,
                                             uint32_t* __restrict__ out) {
  const uint32_t tid = blockIdx.x * 64u + threadIdx.x;
  uint32_t acc = 0;
  if constexpr (MODE == 0 || MODE == 1) {
    uint32_t i = below(mix(tid * 2654435761u), n_rec);
    uint32_t nxt = below(mix(tid + 0x51ed27u), n_rec);   // chain2: the record known one step ahead
    // (the lane id enters every step, so two lanes reaching one record do not merge their chains)
    const uint32_t salt = mix(tid ^ 0x2545f491u);
    for (int s = 0; s < steps; ++s) {
      const uint32_t v = rec_word(buf + (size_t)i * 4);
      if constexpr (MODE == 1) {
        acc += rec_word(buf + (size_t)nxt * 4);
        nxt = below(mix(v ^ salt), n_rec);
      }
      acc += v;
      i = below(mix((v ^ salt) + (uint32_t)s), n_rec);
    }
  } else if constexpr (MODE == 2) {
    uint32_t h = mix(tid * 2654435761u);
    for (int s = 0; s < steps; ++s) {
      uint32_t j[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) { h = mix(h + k + 1); j[k] = below(h, n_rec); }
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += rec_word(buf + (size_t)j[k] * 4);
    }
  } else if constexpr (MODE == 3) {
    uint32_t h = mix(tid * 2654435761u);
    for (int s = 0; s < steps; ++s) {
      uint32_t j[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) { h = mix(h + k + 1); j[k] = below(h, n_rec >> 1); }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const uint4* r = buf + (size_t)j[k] * 8;
        acc += rec_word(r) ^ rec_word(r + 4);
      }
    }
  } else {
    // stream: the grid reads the array front to back, 16 B per lane per step, coalesced
    const size_t n16 = (size_t)n_rec * 4;
    const size_t stride = (size_t)gridDim.x * 64;
    size_t i = tid;
    for (int s = 0; s < steps; ++s) {
      const uint4 a = buf[i];
      acc += a.x ^ a.y ^ a.z ^ a.w;
      i += stride;
      if (i >= n16) i -= n16;
    }
  }
  out[tid] = acc;
}

template <class T>
static std::vector<T> parse_list(const char* s) {
  std::vector<T> v;
  for (const char* p = s; *p;) {
    char* e;
    v.push_back((T)strtoull(p, &e, 10));
    p = *e == ',' ? e + 1 : e;
    if (e == p && *p) break;
  }
  return v;
}

struct Mode { const char* name; int id; int bytes_per_step; };

int main(int argc, char** argv) {
  std::vector<size_t> sizes_mb = {64, 128, 400, 1024, 4096};
  std::vector<int> waves_per_simd = {2, 4, 5, 8};
  if (argc > 1) sizes_mb = parse_list<size_t>(argv[1]);
  if (argc > 2) waves_per_simd = parse_list<int>(argv[2]);
  size_t max_mb = 0;
  for (size_t m : sizes_mb) max_mb = m > max_mb ? m : max_mb;
  for (int w : waves_per_simd) if (w < 1 || w > 8) { fprintf(stderr, "waves per SIMD in 1..8\n"); return 1; }
  const size_t max_bytes = max_mb << 20;
  uint4* buf;
  CK(hipMalloc(&buf, max_bytes));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, buf, max_bytes / 16);
  const int max_waves = 1024 * 8;
  uint32_t* out;
  CK(hipMalloc(&out, sizeof(uint32_t) * 64 * max_waves));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const Mode modes[] = {{"chain", 0, 64}, {"chain2", 1, 128}, {"indep", 2, 256}, {"line", 3, 256}, {"stream", 4, 16}};
  for (size_t ws_mb : sizes_mb) {
    const uint32_t n_rec = (uint32_t)((ws_mb << 20) / 64);   // 64-B records
    for (const Mode& m : modes) {
      for (int w : waves_per_simd) {
        const int blocks = 1024 * w;
        const double lanes = 64.0 * blocks;
        // about 8 GB of record bytes per launch (at least 16 steps)
        int steps = (int)(8e9 / (lanes * m.bytes_per_step));
        if (steps < 16) steps = 16;
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {   // rep 0 warms up; the best of the other two
          CK(hipEventRecord(e0, 0));
          switch (m.id) {
            case 0: hipLaunchKernelGGL(gather<0>, dim3(blocks), dim3(64), 0, 0, buf, n_rec, steps, out); break;
            case 1: hipLaunchKernelGGL(gather<1>, dim3(blocks), dim3(64), 0, 0, buf, n_rec, steps, out); break;
            case 2: hipLaunchKernelGGL(gather<2>, dim3(blocks), dim3(64), 0, 0, buf, n_rec, steps, out); break;
            case 3: hipLaunchKernelGGL(gather<3>, dim3(blocks), dim3(64), 0, 0, buf, n_rec, steps, out); break;
            default: hipLaunchKernelGGL(gather<4>, dim3(blocks), dim3(64), 0, 0, buf, n_rec, steps, out); break;
          }
          CK(hipGetLastError());
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (rep > 0 && ms < best) best = ms;
        }
        const double bytes = lanes * steps * m.bytes_per_step;
        const double gbs = bytes / (best * 1e-3) / 1e9;
        printf("{\"mode\": \"%s\", \"working_set_mb\": %zu, \"records\": %u, \"waves_per_simd\": %d, \"steps\": %d, "
               "\"ms\": %.3f, \"record_GBs\": %.1f, \"frac_of_8TBs\": %.4f}\n",
               m.name, ws_mb, n_rec, w, steps, best, gbs, gbs / 8000.0);
        fflush(stdout);
      }
    }
  }
  CK(hipFree(out));
  CK(hipFree(buf));
  return 0;
}
