// Can kernels of several processes run at the same time on one GPU?  (The
// shared-GPU rehearsals of the multi-rank fused step need every rank's
// multi-step kernel resident together: a block waits for producer blocks of
// other ranks.)  Independent of the framework: R processes share one uncached
// counter (IPC handle through a file), each launches `blocks` workgroups of
// `threads` threads holding `lds` bytes of LDS; every workgroup adds 1 per
// round and spins until all R x blocks workgroups of all processes have added
// theirs (bounded: 2 s).  Prints one JSON line per process: rounds completed,
// the longest wait, and whether a wait timed out.
//
//   hipcc --offload-arch=gfx950 -O2 tools/coresident_probe.hip -o tools/coresident_probe
//   for r in 0 1 2; do ./tools/coresident_probe $r 3 /tmp/cr 72 768 65536 20 & done; wait
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::printf("{\"rank\": %d, \"status\": \"hip error\", \"at\": \"%s\", \"err\": %d}\n", rank, #x, (int)e_); \
      return 2;                                                                                 \
    }                                                                                           \
  } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;

__global__ void rounds_kernel(unsigned* counter, unsigned total, int rounds, long long timeout_ticks,
                              unsigned long long* out) {
  extern __shared__ unsigned char lds[];
  if (threadIdx.x == 0) lds[0] = 1;
  __syncthreads();
  unsigned long long worst = 0;
  int done = 0, timed_out = 0;
  if (threadIdx.x == 0) {
    for (int r = 0; r < rounds; ++r) {
      __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const unsigned want = total * (unsigned)(r + 1);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        if (__hip_atomic_load((gu32*)counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= want) break;
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout_ticks) { timed_out = 1; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      const unsigned long long w = __builtin_amdgcn_s_memrealtime() - t0;
      worst = w > worst ? w : worst;
      if (timed_out) break;
      ++done;
    }
    out[blockIdx.x * 3 + 0] = worst;
    out[blockIdx.x * 3 + 1] = (unsigned long long)done;
    out[blockIdx.x * 3 + 2] = (unsigned long long)timed_out;
  }
  __syncthreads();
  if (threadIdx.x == 1) lds[1] = lds[0];
}

static bool exists(const std::string& p) { std::ifstream f(p); return f.good(); }

int main(int argc, char** argv) {
  if (argc < 8) {
    std::printf("usage: coresident_probe rank nranks dir blocks threads lds_bytes rounds\n");
    return 2;
  }
  const int rank = std::atoi(argv[1]), nranks = std::atoi(argv[2]);
  const std::string dir = argv[3];
  const int blocks = std::atoi(argv[4]), threads = std::atoi(argv[5]), lds = std::atoi(argv[6]);
  const int rounds = std::atoi(argv[7]);
  if (nranks < 1 || nranks > 16 || blocks < 1 || blocks > 1024 || threads < 64 || threads > 1024 || lds < 2 ||
      lds > 160 * 1024 || rounds < 1 || rounds > 1000) {
    std::printf("{\"rank\": %d, \"status\": \"bad arguments\"}\n", rank);
    return 2;
  }
  CK(hipSetDevice(0));
  unsigned* counter = nullptr;
  const std::string hfile = dir + "/handle.bin";
  if (rank == 0) {
    CK(hipExtMallocWithFlags((void**)&counter, 256, hipDeviceMallocUncached));
    CK(hipMemset(counter, 0, 256));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, counter));
    {
      std::ofstream f(hfile + ".tmp", std::ios::binary);
      f.write(reinterpret_cast<const char*>(&h), sizeof(h));
    }
    std::rename((hfile + ".tmp").c_str(), hfile.c_str());
  } else {
    for (int k = 0; k < 3000 && !exists(hfile); ++k) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    hipIpcMemHandle_t h;
    std::ifstream f(hfile, std::ios::binary);
    f.read(reinterpret_cast<char*>(&h), sizeof(h));
    if (!f) { std::printf("{\"rank\": %d, \"status\": \"no handle\"}\n", rank); return 2; }
    CK(hipIpcOpenMemHandle((void**)&counter, h, hipIpcMemLazyEnablePeerAccess));
  }
  unsigned long long* dout = nullptr;
  CK(hipMalloc(&dout, (size_t)blocks * 3 * sizeof(unsigned long long)));
  CK(hipMemset(dout, 0, (size_t)blocks * 3 * sizeof(unsigned long long)));
  CK(hipFuncSetAttribute((const void*)rounds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipDeviceSynchronize());
  // every process ready before any launches
  { std::ofstream f(dir + "/ready." + std::to_string(rank)); f << 1; }
  for (int k = 0; k < 3000; ++k) {
    int n = 0;
    for (int r = 0; r < nranks; ++r) n += exists(dir + "/ready." + std::to_string(r));
    if (n == nranks) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(rounds_kernel, dim3(blocks), dim3(threads), lds, 0, counter, (unsigned)(nranks * blocks), rounds,
                     200000000LL, dout);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const double wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  unsigned long long* h = (unsigned long long*)std::malloc((size_t)blocks * 3 * sizeof(unsigned long long));
  CK(hipMemcpy(h, dout, (size_t)blocks * 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  unsigned long long worst = 0, mind = ~0ull;
  int tos = 0;
  for (int b = 0; b < blocks; ++b) {
    worst = h[3 * b] > worst ? h[3 * b] : worst;
    mind = h[3 * b + 1] < mind ? h[3 * b + 1] : mind;
    tos += (int)h[3 * b + 2];
  }
  std::printf("{\"rank\": %d, \"nranks\": %d, \"blocks\": %d, \"threads\": %d, \"lds\": %d, \"rounds\": %d, "
              "\"rounds_done_min\": %llu, \"worst_wait_us\": %.1f, \"blocks_timed_out\": %d, \"wall_ms\": %.1f}\n",
              rank, nranks, blocks, threads, lds, rounds, mind, worst / 100.0, tos, wall_ms);
  std::free(h);
  hipFree(dout);
  if (rank != 0) hipIpcCloseMemHandle(counter);
  else {
    std::this_thread::sleep_for(std::chrono::milliseconds(500));   // peers close their mappings first
    hipFree(counter);
  }
  return tos ? 1 : 0;
}
