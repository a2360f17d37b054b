// Shared declarations of the gfx950 kernels and their C ABI descriptors.
//
// The descriptors are plain C structs mirrored by ctypes (ops/native.py) and
// by the C++ runtime (runtime.cpp).  Pointers are device pointers; scalars are
// carried as double and converted to the kernel's element type at launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// One fused finite-volume RK stage (see stage_kernel.hip).
typedef struct StageDesc {
  const void* X;        // [F][S]  RK combination input, read at own cell (padded layout)
  const void* Q;        // [F][S]  stage input, read with halos (padded layout)
  const void* acc_in;   // [F][S]  RK4 accumulator in (nullable)
  void* out;            // [F][S]
  void* acc_out;        // [F][S]  (nullable)
  const void* recv;     // [R][F]  remote ghost slots (nullable when R == 0)
  const int* gmap;      // [T][4][mg][n]  ghost map (remote slots < 0)
  const int* push;      // [T][4][mg][n]  push map (same-rank ghost slot fed by a strip cell, or -1)
  const int* blocks;    // work list of linear block ids (nullable -> all blocks)
  const void* invA;     // [T][n][n]
  const void* ex;       // [T][n][n+1]  per x-edge coefficient (L, U*L or kappa L/d)
  const void* ey;       // [T][n+1][n]
  const void* mx;       // [T][3][n+1]  x-edge unit normals (SWE)
  const void* my;       // [T][3][n+1]
  const void* cgeo;     // [T][n][n][8] per-cell record (1/A, centre xyz, grad b xyz, 0) (SWE)
  int ntile, n, S, mg, pw;  // pw = n + 2 mg (padded tile width), S = ntile pw^2
  int nblocks;          // number of entries in `blocks` (or total blocks)
  int limiter;
  int remote;           // 1: read remote ghost slots from recv via gmap (boundary blocks)
  double a0, a1, a2, c0, c1, c2, dt;
  double g, omega2;
  void* stamps;         // diagnostic builds only (-DSTSP_STAMPS): [nblocks][8] s_memtime per phase
} StageDesc;

int stsp_stage_launch(int phys, int dtype, int bx, int by, const StageDesc* d, hipStream_t stream);
// Persistent multi-step kernel (single rank, small grids): nsteps x nstages
// stages in one cooperative launch with neighbour-only flag hand-offs.
int stsp_persistent_launch(int phys, int dtype, int bx, int by, const StageDesc* stages, int nstages, int nsteps,
                           unsigned* flags, const int* nbr, int maxnbr, int* err, double timeout_s,
                           hipStream_t stream);
int stsp_pack_launch(int dtype, const void* q, int S, int F, const int* idx, int ns, void* send, hipStream_t stream);
int stsp_copy_index_launch(int dtype, const void* src, const int* sidx, void* dst, const int* didx, int k,
                           int batch, long src_stride, long dst_stride, hipStream_t stream);
}
