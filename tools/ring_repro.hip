// Standalone reproducer of the round-4 post-free corruption (profiles/r4_ring):
// uncached device memory (hipExtMallocWithFlags(hipDeviceMallocUncached), the
// xGMI ring's memory type) carries tagged-granule traffic from a kernel
// (relaxed system-scope 8-byte stores and loads, the fused step's ring
// protocol), is released with hipFree after a device synchronise, and fresh
// ordinary allocations made afterwards are filled and read back (by a kernel
// and through the host).  A session-long buffer is checked every iteration.
// No torch, no library of ours: if this reports mismatches, the defect is below
// our kernels; if it stays clean, the suspects are our kernels' addressing.
//
//   hipcc --offload-arch=gfx950 -O2 tools/ring_repro.hip -o tools/ring_repro
//   ./tools/ring_repro [iterations] [ring MiB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("{\"status\": \"hip error\", \"at\": \"%s\", \"err\": %d}\n", #x, (int)e_); \
      return 2;                                                                    \
    }                                                                              \
  } while (0)

typedef __attribute__((address_space(1))) unsigned long long gu64;

// every thread stores granules {tag, index} into its slice, then re-reads them
// until every tag matches (bounded), the fused step's consumer loop
__global__ void ring_traffic(unsigned long long* ring, size_t n, unsigned tag, unsigned* bad) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __hip_atomic_store((gu64*)(ring + i), ((unsigned long long)tag << 32) | (unsigned)i, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    unsigned long long v = 0;
    for (int spin = 0; spin < 1000; ++spin) {
      v = __hip_atomic_load((gu64*)(ring + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((unsigned)(v >> 32) == tag) break;
    }
    if (v != (((unsigned long long)tag << 32) | (unsigned)i)) atomicAdd(bad, 1u);
  }
}

__global__ void fill(double* p, size_t n, double v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void check(const double* p, size_t n, double v, unsigned* bad) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != v) atomicAdd(bad, 1u);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
  const size_t ring_mib = argc > 2 ? (size_t)std::atoll(argv[2]) : 4;
  const int nbuf = 48;
  CK(hipSetDevice(0));
  unsigned* dbad = nullptr;
  CK(hipMalloc(&dbad, 4 * sizeof(unsigned)));
  double* keep = nullptr;
  const size_t nkeep = (size_t)1 << 22;
  CK(hipMalloc(&keep, nkeep * sizeof(double)));
  hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, 0, keep, nkeep, 7.0);
  CK(hipDeviceSynchronize());
  long long ring_bad = 0, fresh_bad = 0, host_bad = 0, keep_bad = 0, first_iter = -1;
  std::vector<double> hbuf;
  for (int it = 0; it < iters; ++it) {
    // 1. an uncached ring with tagged-granule traffic, then hipFree
    void* ring = nullptr;
    const size_t rb = ring_mib << 20;
    CK(hipExtMallocWithFlags(&ring, rb, hipDeviceMallocUncached));
    CK(hipMemset(ring, 0, rb));
    CK(hipMemset(dbad, 0, 4 * sizeof(unsigned)));
    for (int rep = 0; rep < 4; ++rep)
      hipLaunchKernelGGL(ring_traffic, dim3(216), dim3(768), 0, 0, (unsigned long long*)ring, rb / 8,
                         (unsigned)(it * 4 + rep + 1), dbad);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipFree(ring));
    // 2. fresh ordinary allocations of many sizes, each filled with its own value
    std::vector<double*> bufs(nbuf, nullptr);
    std::vector<size_t> ns(nbuf);
    for (int k = 0; k < nbuf; ++k) {
      ns[k] = ((size_t)1 << (10 + k % 12)) + 64 * k;
      CK(hipMalloc(&bufs[k], ns[k] * sizeof(double)));
      hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, bufs[k], ns[k], (double)(k + 1) + 0.5 * it);
    }
    CK(hipDeviceSynchronize());
    for (int k = 0; k < nbuf; ++k)
      hipLaunchKernelGGL(check, dim3(64), dim3(256), 0, 0, bufs[k], ns[k], (double)(k + 1) + 0.5 * it, dbad + 1);
    hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, 0, keep, nkeep, 7.0, dbad + 2);
    unsigned hb[4] = {0, 0, 0, 0};
    CK(hipMemcpy(hb, dbad, sizeof(hb), hipMemcpyDeviceToHost));
    // 3. the same through the host
    long long hbad = 0;
    for (int k = 0; k < nbuf; k += 5) {
      hbuf.resize(ns[k]);
      CK(hipMemcpy(hbuf.data(), bufs[k], ns[k] * sizeof(double), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < ns[k]; ++i) hbad += hbuf[i] != (double)(k + 1) + 0.5 * it;
    }
    ring_bad += hb[0];
    fresh_bad += hb[1];
    keep_bad += hb[2];
    host_bad += hbad;
    if (first_iter < 0 && (hb[0] || hb[1] || hb[2] || hbad)) first_iter = it;
    for (int k = 0; k < nbuf; ++k) CK(hipFree(bufs[k]));
  }
  std::printf("{\"status\": \"ok\", \"iterations\": %d, \"ring_mib\": %zu, \"ring_granules_bad\": %lld, "
              "\"fresh_alloc_words_bad\": %lld, \"fresh_alloc_host_words_bad\": %lld, \"keep_words_bad\": %lld, "
              "\"first_bad_iteration\": %lld}\n",
              iters, ring_mib, ring_bad, fresh_bad, host_bad, keep_bad, first_iter);
  hipFree(keep);
  hipFree(dbad);
  return (ring_bad || fresh_bad || host_bad || keep_bad) ? 1 : 0;
}
