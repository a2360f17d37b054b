// Kernel-argument preload probe (gfx950): per-launch time of dependent
// launches in a hipGraph, 216 blocks x 640 threads (the C96 stage grid), for
//   A: every argument in a by-value struct (read with s_load from the kernarg
//      segment once the wave runs, as the stage kernel does today), and
//   B: the first arguments as scalars, preloaded into SGPRs by the dispatcher
//      (-mllvm -amdgpu-kernarg-preload-count=16).
// Each block does one dependent global load -> store through the arguments.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Big {
  const double* x; double* y; const int* p[16]; int n, m, k, l; double c[9]; unsigned u[4];
};

__global__ __launch_bounds__(640) void ka(Big a) {
  const int i = blockIdx.x;
  if (threadIdx.x == 0 && i < a.n) a.y[i] = a.x[(i * a.m) % a.n] * a.c[0] + (double)a.u[0];
}

__global__ __launch_bounds__(640) void kb(const double* __restrict__ x, double* __restrict__ y, int n, int m, double c0,
                                          unsigned u0) {
  const int i = blockIdx.x;
  if (threadIdx.x == 0 && i < n) y[i] = x[(i * m) % n] * c0 + (double)u0;
}

// C: the same scalar arguments, not preloaded (kernarg-preload attribute off)
__global__ __launch_bounds__(640) __attribute__((amdgpu_max_num_work_groups(65535, 1, 1))) void kc(const double* __restrict__ x, double* __restrict__ y, int n, int m, double c0,
                                          unsigned u0, int pad0, int pad1, int pad2, int pad3, int pad4, int pad5, int pad6, int pad7, int pad8, int pad9, int pad10, int pad11, int pad12, int pad13, int pad14, int pad15) {
  const int i = blockIdx.x;
  if (threadIdx.x == 0 && i < n) y[i] = x[(i * m) % n] * c0 + (double)u0 + (double)pad15;
}

int main() {
  const int NB = 216, R = 300;
  double *x, *y;
  CK(hipMalloc(&x, 4096 * sizeof(double)));
  CK(hipMalloc(&y, 4096 * sizeof(double)));
  CK(hipMemset(x, 0, 4096 * sizeof(double)));
  Big a{};
  a.x = x; a.y = y; a.n = NB; a.m = 7; a.k = 0; a.c[0] = 1.0;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 3; ++round) {
    for (int v = 0; v < 3; ++v) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int r = 0; r < R; ++r) {
        if (v == 0) hipLaunchKernelGGL(ka, dim3(NB), dim3(640), 0, s, a);
        else if (v == 1) hipLaunchKernelGGL(kb, dim3(NB), dim3(640), 0, s, (const double*)x, y, NB, 7, 1.0, 0u);
        else hipLaunchKernelGGL(kc, dim3(NB), dim3(640), 0, s, (const double*)x, y, NB, 7, 1.0, 0u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int k = 0; k < 3; ++k) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("round %d %s: %.3f us per launch\n", round, v == 0 ? "A struct (s_load)" : v == 1 ? "B preloaded scalars" : "C scalars, last one past the preload limit", ms * 1e3 / (3 * R));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
