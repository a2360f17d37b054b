// Persistent factored diffusion step (fp64, gfx950): the whole CholeskyQR3
// recompression of LowRankDiffusion (models/tt.py) -- and as many of those
// steps as asked -- in ONE launch of two workgroups, no host round trip.
//
// Round 4's native step (tt_kernels.hip, stsp_tt_lr_step3) is a chain of ~36
// dependent kernels per step (2 expansions, per factor and pass a Gram partial,
// a Gram reduce, a shifted Cholesky + inverse and a product, then the core and
// two products) plus a 4-byte read-back of the new rank: at N = 1024 every
// kernel is 1.5-8 us of mostly idle GPU (profiles/r4_tt/tt_step_trace_N1024_r3.txt).
// Here workgroup s (s = 0: the row factor A, s = 1: the column factor B) keeps
// its N x k factor in LDS for the whole launch (N k <= 12288 doubles, 96 KiB)
// and runs, per step:
//
//   expand    nsub explicit substeps on the factors, [A, c D A] [B + c D B, B]
//   3 passes  G = X^T X (MFMA f64 16x16x4, one 4-row group per MFMA, the 16
//             waves' tiles summed in a fixed order), shifted Cholesky and R^-1
//             (wave 0), X <- X R^-1 (one row per thread), R <- R_p R
//   core      B's R to A (sc1 stores, drained flag), C = R_A R_B^T and its
//             one-sided Jacobi SVD on workgroup 0 (round-robin pairs, 16 lanes
//             per pair), truncation, B's core map back (drained flag)
//   product   X <- X M (k x rn), the new factor, still in LDS
//
// and writes the factors once, after the last step.  Hand-offs between the two
// workgroups: write-through (sc1) payload stores, every storing wave drained,
// a workgroup barrier, one relaxed agent-scope flag store; the consumer polls
// the flag (bounded, s_sleep) and loads the payload with sc1 loads
// (cdna_hip_programming.md Guideline 16, R1).  The flags are zeroed by the
// launcher before every launch.  Numerics: the same CholeskyQR3 (shift
// 11 (N k + k (k + 1)) u, passes 2-3 shifted only where a pivot fails) and core
// as stsp_tt_lr_step3; tests/test_tt_kernels.py compares the two.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tt_common.h"

namespace {

// 512 threads (8 waves, 2 per SIMD): a 256-VGPR budget, so the k x k
// Cholesky and R^-1 run from registers (at 1024 threads the 128-VGPR budget
// forced them through LDS: ~39k cycles per CholeskyQR pass at k = 12)
constexpr int TP_T = 512, TP_W = 8, TP_KP = 16, TP_NK = 12288, TP_RPT = 2;
typedef double d4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned long long tp_gu64;
typedef __attribute__((address_space(1))) unsigned tp_gu32;

struct TPArgs {
  const double* A;
  const double* B;
  int lda, ldb, N, r0, ncalls, nsub, periodic, max_rank;
  double c, ih2, eps;
  double* xch;              // [0, 256): R of B; [256, 512): B's core map (k x rn)
  unsigned* flags;          // [0] R_B ready = step + 1, [1] core ready (step + 1) << 8 | rn, [3] error
  double* outA;
  double* outB;
  int ldo;
  int* rn_out;              // final rank (<= 0: failure)
  unsigned long long* stamps;   // [ncalls][2][16] shader clocks, or null
  long long timeout_ticks;
};

__device__ __forceinline__ void wsync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void st_wt(double* p, double v) {   // write-through (sc1)
  __hip_atomic_store((tp_gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {    // L1 bypass (sc1)
  return __builtin_bit_cast(double, __hip_atomic_load((tp_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// wait until *f >= want (one lane), bounded; false on timeout (sets flags[3])
__device__ bool tp_wait(unsigned* f, unsigned want, unsigned* err, long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (__hip_atomic_load((tp_gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want) return true;
    if (__hip_atomic_load((tp_gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
    if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) {
      __hip_atomic_store((tp_gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// X (N x k, row stride k, LDS) times M (k x m, M[l][j] in an LDS array of
// TP_KP + 1 columns) on the matrix cores: 16-row blocks of X, v_mfma_f64_16x16x4
// over k in steps of 4 (operands beyond k / m read as 0).  Returns each wave's
// TP_XB output blocks in registers: the caller
// synchronises before xmul_store overwrites X (the product is in place).
// Layouts (checked by the Gram above and tests/test_tt_kernels.py): A 16x4,
// lane l holds A[l % 16][l / 16]; B 4x16, lane l holds B[l / 16][l % 16];
// D 16x16, lane l, register i holds D[l / 16 + 4 i][l % 16].
constexpr int TP_XB = 1024 / 16 / TP_W;           // 16-row blocks per wave at N = 1024
__device__ __forceinline__ void xmul(const double* X, int N, int k, const double (*M)[TP_KP + 1], int m, int wv,
                                     int lane, d4 (&acc)[TP_XB]) {
  const int nb = (N + 15) >> 4;
#pragma unroll
  for (int q = 0; q < TP_XB; ++q) {
    const int b = wv + q * TP_W;
    d4 c = {0, 0, 0, 0};
    if (b < nb) {
      for (int c0 = 0; c0 < k; c0 += 4) {
        const int row = 16 * b + (lane & 15), kk = c0 + (lane >> 4), col = lane & 15;
        const double av = (row < N && kk < k) ? X[row * k + kk] : 0.0;
        const double bv = (kk < k && col < m) ? M[kk][col] : 0.0;
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c, 0, 0, 0);
      }
    }
    acc[q] = c;
  }
}
__device__ __forceinline__ void xmul_store(double* X, int N, int m, int wv, int lane, const d4 (&acc)[TP_XB]) {
  const int nb = (N + 15) >> 4;
#pragma unroll
  for (int q = 0; q < TP_XB; ++q) {
    const int b = wv + q * TP_W;
    if (b >= nb) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * b + (lane >> 4) + 4 * i, col = lane & 15;
      if (row < N && col < m) X[row * m + col] = acc[q][i];
    }
  }
}

#define TP_STAMP(k)                                                                           \
  do {                                                                                        \
    if (a.stamps && tid == 0) a.stamps[((long)call * 2 + side) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

__global__ __launch_bounds__(TP_T) void tt_persist_kernel(TPArgs a) {
  __shared__ double X[TP_NK];                     // the factor, row-major, row stride k
  __shared__ double red[TP_W][TP_KP * TP_KP];     // per-wave Gram tiles
  __shared__ double Gm[TP_KP][TP_KP + 1];         // Gram -> Cholesky factor (upper)
  __shared__ double Ri[TP_KP][TP_KP + 1];         // its inverse
  __shared__ double Rt[TP_KP][TP_KP + 1];         // R3 R2 R1
  __shared__ double Tm[TP_KP][TP_KP + 1];         // scratch
  __shared__ double sC[TP_KP][TP_KP + 1];         // core: C -> U S (columns), then this side's map
  __shared__ double sW[TP_KP][TP_KP + 1];         // core: right singular vectors
  __shared__ double sig[TP_KP];
  __shared__ int s_ord[TP_KP];
  __shared__ int s_i[5];                          // pivot flag, rotation flag, rank, wait failed, core rank
  __shared__ double s_d[2];
  const int side = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = a.N;
  int r = a.r0;
  {
    const double* src = side ? a.B : a.A;
    const int ld = side ? a.ldb : a.lda;
    for (int e = tid; e < N * r; e += TP_T) {
      const int i = e / r, j = e - i * r;
      X[i * r + j] = src[(long)i * ld + j];
    }
  }
  __syncthreads();
  int call = 0;
  for (; call < a.ncalls; ++call) {
    TP_STAMP(0);
    // ---- expansion: nsub explicit substeps, the rank doubles each ----------
    for (int sub = 0; sub < a.nsub; ++sub) {
      // cell value and second difference of each column (static indices: the
      // new layout [x, y] is written after every thread has read its rows)
      double xv[TP_RPT][TP_KP / 2], dv[TP_RPT][TP_KP / 2];
#pragma unroll
      for (int q = 0; q < TP_RPT; ++q) {
        const int i = tid + q * TP_T;
        int im = i - 1, ip = i + 1;
        if (a.periodic) { im = im < 0 ? N - 1 : im; ip = ip >= N ? 0 : ip; }
#pragma unroll
        for (int j = 0; j < TP_KP / 2; ++j) {
          xv[q][j] = dv[q][j] = 0.0;
          if (i < N && j < r) {
            const double xc = X[i * r + j];
            const double xl = im >= 0 ? X[im * r + j] : 0.0, xh = ip < N ? X[ip * r + j] : 0.0;
            xv[q][j] = xc;
            dv[q][j] = ((xl + xh) - 2.0 * xc) * a.ih2;
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < TP_RPT; ++q) {
        const int i = tid + q * TP_T;
        if (i >= N) continue;
#pragma unroll
        for (int j = 0; j < TP_KP / 2; ++j) {
          if (j < r) {
            const double xc = xv[q][j], cd = a.c * dv[q][j];
            X[i * 2 * r + j] = side == 0 ? xc : xc + cd;          // [A, c D A] / [B + c D B, B]
            X[i * 2 * r + r + j] = side == 0 ? cd : xc;
          }
        }
      }
      r *= 2;
      __syncthreads();
    }
    const int k = r;
    // CholeskyQR shift of this step's width (models/tt.py::cholqr3_shift)
    const double shc = 11.0 * ((double)N * k + (double)k * (k + 1)) * 1.1102230246251565e-16;
    TP_STAMP(1);
    // ---- CholeskyQR3 of the LDS factor ----------------------------------------
    if (tid < TP_KP * TP_KP) Rt[tid / TP_KP][tid % TP_KP] = (tid / TP_KP == tid % TP_KP) ? 1.0 : 0.0;
    for (int pass = 0; pass < 3; ++pass) {
      // G = X^T X: one MFMA per 4-row group, both operands X[row][col]
      // (four independent accumulator chains per wave: one chain of 16
      // dependent MFMAs was ~9k cycles)
      d4 acc = {0, 0, 0, 0}, acc1 = acc, acc2 = acc, acc3 = acc;
      const int ng = (N + 3) >> 2;
      const int col = lane & 15;
      for (int g = wv; g < ng; g += 4 * TP_W) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int row = 4 * (g + u * TP_W) + (lane >> 4);
          v[u] = (row < N && col < k) ? X[row * k + col] : 0.0;
        }
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v[0], v[0], acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(v[1], v[1], acc1, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(v[2], v[2], acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(v[3], v[3], acc3, 0, 0, 0);
      }
      acc = (acc + acc1) + (acc2 + acc3);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) red[wv][((lane >> 4) + 4 * rr) * TP_KP + col] = acc[rr];
      __syncthreads();
      if (pass == 0) TP_STAMP(8);
      if (tid < k * k) {
        const int i = tid / k, j = tid - i * k;
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < TP_W; ++w) s += red[w][i * TP_KP + j];
        Gm[i][j] = s;
      }
      __syncthreads();
      if (pass == 0) TP_STAMP(9);
      if (wv == 0) {
        // shifted Cholesky G + s I = R^T R (pass 0 always shifted; passes 1, 2
        // plain unless a pivot fails), then R^-1, in registers: lane c holds
        // column c (g[i] = entry (i, c)), padded to TP_KP with an identity
        // block (R = diag(R_k, I)) so every loop has static bounds; entries
        // of other columns arrive by lane shuffles
        const bool adaptive = pass > 0;
        double trace = 0.0;
        for (int i = 0; i < k; ++i) trace += Gm[i][i];
        double g[TP_KP];
        int fail = 0;
        for (int attempt = adaptive ? 0 : 1; attempt < 2; ++attempt) {
#pragma unroll
          for (int i = 0; i < TP_KP; ++i) {
            g[i] = (i < k && lane < k) ? Gm[i][lane] : (i == lane ? 1.0 : 0.0);
            if (attempt == 1 && i == lane && lane < k) g[i] += shc * trace;
          }
          fail = 0;
#pragma unroll
          for (int j = 0; j < TP_KP; ++j) {
            double d = tt::lane_bcast(g[j], j);
            if (!(d > 0.0)) { if (!fail) fail = j + 1; d = 1.0; }
            const double sq = sqrt(d);
            if (lane == j) g[j] = sq;
            if (lane > j) g[j] /= sq;
            const double rt = g[j];
#pragma unroll
            for (int i = j + 1; i < TP_KP; ++i) {
              const double rji = tt::lane_bcast(g[j], i);     // R[j][i]: lane i's column
              if (i <= lane) g[i] -= rji * rt;
            }
          }
          if (!fail) break;
        }
        double ri[TP_KP];
#pragma unroll
        for (int i = TP_KP - 1; i >= 0; --i) {
          const double rii = tt::lane_bcast(g[i], i);
          double sum = 0.0;
#pragma unroll
          for (int l = i + 1; l < TP_KP; ++l) sum += tt::lane_bcast(g[i], l) * ri[l];
          ri[i] = i == lane ? 1.0 / rii : (i < lane ? -sum / rii : 0.0);
        }
        if (lane < k) {
#pragma unroll
          for (int i = 0; i < TP_KP; ++i)
            if (i < k) { Tm[i][lane] = g[i]; Ri[i][lane] = ri[i]; }
        }
        if (lane == 0 && fail) __hip_atomic_store((tp_gu32*)(a.flags + 3), 2u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (pass == 0) TP_STAMP(10);
      // X <- X R^-1 on the matrix cores (round 5's first version: one row per
      // thread, k trips of 16 LDS broadcasts and FMAs: ~21k cycles per pass)
      d4 xacc[TP_XB];
      xmul(X, N, k, Ri, k, wv, lane, xacc);
      double rv = 0.0;
      if (tid < k * k) {
        const int i = tid / k, j = tid - i * k;
        for (int l = i; l < k; ++l) rv += Tm[i][l] * Rt[l][j];
      }
      __syncthreads();
      xmul_store(X, N, k, wv, lane, xacc);
      if (tid < k * k) Rt[tid / k][tid - (tid / k) * k] = rv;
      __syncthreads();
      TP_STAMP(2 + pass);
    }
    // ---- core ----------------------------------------------------------------
    int rn = 0;
    if (side == 1) {
      if (tid < k * k) st_wt(a.xch + tid, Rt[tid / k][tid - (tid / k) * k]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store((tp_gu32*)a.flags, (unsigned)call + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      TP_STAMP(5);
      // flags[1] = (step + 1) << 8 | rn: one single-copy-atomic word, so the rank
      // can never be read from an older step than the ready count
      if (tid == 0) {
        const bool ok = tp_wait(a.flags + 1, ((unsigned)call + 1u) << 8, a.flags + 3, a.timeout_ticks);
        s_i[3] = ok ? 0 : 1;
        s_i[4] = ok ? (int)(__hip_atomic_load((tp_gu32*)(a.flags + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                            255u) : 0;
      }
      __syncthreads();
      if (s_i[3]) break;
      rn = s_i[4];
      if (rn <= 0 || rn > k) break;
      if (tid < k * rn) sC[tid / rn][tid - (tid / rn) * rn] = ld_wt(a.xch + 256 + tid);
      __syncthreads();
      TP_STAMP(6);
    } else {
      if (tid == 0) s_i[3] = tp_wait(a.flags, (unsigned)call + 1u, a.flags + 3, a.timeout_ticks) ? 0 : 1;
      __syncthreads();
      if (s_i[3]) break;
      TP_STAMP(5);
      // C = R_A R_B^T (R_B from B's workgroup), W = I
      if (tid < k * k) Tm[tid / k][tid - (tid / k) * k] = ld_wt(a.xch + tid);
      __syncthreads();
      if (tid < k * k) {
        const int i = tid / k, j = tid - i * k;
        double s = 0.0;
        for (int l = 0; l < k; ++l) s += Rt[i][l] * Tm[j][l];
        sC[i][j] = s;
        sW[i][j] = i == j ? 1.0 : 0.0;
      }
      __syncthreads();
      if (tid == 0) {
        double t = 0.0;
        for (int i = 0; i < k; ++i)
          for (int j = 0; j < k; ++j) t += sC[i][j] * sC[i][j];
        s_d[1] = t;
      }
      __syncthreads();
      const double tiny = 1e-30 * s_d[1];
      const int m = (k + 1) & ~1;
      // one-sided Jacobi on wave 0 alone (round-robin pairs, 8 lanes per pair,
      // two rows per lane): the rounds synchronise the wave, not the 16-wave
      // workgroup (round 5's first version: two workgroup barriers per round,
      // ~47k cycles per core)
      if (wv == 0) {
        const int pr = lane >> 3, ln = lane & 7;
        for (int sweep = 0; sweep < 60; ++sweep) {
          bool rotated = false;
          for (int rd = 0; rd < m - 1; ++rd) {
            if (pr < m / 2) {
              const int qa = pr, qb = m - 1 - pr;
              int p = qa == 0 ? 0 : 1 + (qa - 1 + rd) % (m - 1);
              int q = qb == 0 ? 0 : 1 + (qb - 1 + rd) % (m - 1);
              if (p > q) { const int x = p; p = q; q = x; }
              if (q < k) {
                double al = 0, be = 0, ga = 0;
                for (int rr = ln; rr < k; rr += 8) {
                  const double x = sC[rr][p], y = sC[rr][q];
                  al += x * x;
                  be += y * y;
                  ga += x * y;
                }
                al = tt::sum8(al);        // 8-lane sums through DPP
                be = tt::sum8(be);
                ga = tt::sum8(ga);
                if (!(al <= tiny || be <= tiny || fabs(ga) <= 1e-15 * sqrt(al * be))) {
                  const double ze = (be - al) / (2.0 * ga);
                  const double t = (ze >= 0 ? 1.0 : -1.0) / (fabs(ze) + sqrt(1.0 + ze * ze));
                  const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
                  for (int rr = ln; rr < k; rr += 8) {
                    const double x = sC[rr][p], y = sC[rr][q];
                    sC[rr][p] = cs * x - sn * y;
                    sC[rr][q] = sn * x + cs * y;
                    const double u = sW[rr][p], w = sW[rr][q];
                    sW[rr][p] = cs * u - sn * w;
                    sW[rr][q] = sn * u + cs * w;
                  }
                  rotated = true;
                }
              }
            }
            wsync();
          }
          if (__builtin_amdgcn_ballot_w64(rotated) == 0) break;
        }
      }
      __syncthreads();
      if (tid < k) {
        double s2 = 0;
        for (int rr = 0; rr < k; ++rr) s2 += sC[rr][tid] * sC[rr][tid];
        sig[tid] = sqrt(s2);
      }
      __syncthreads();
      if (tid == 0) {
        for (int j = 0; j < k; ++j) s_ord[j] = j;
        for (int x = 1; x < k; ++x) {               // insertion sort, descending
          const int v = s_ord[x];
          int y = x - 1;
          while (y >= 0 && sig[s_ord[y]] < sig[v]) { s_ord[y + 1] = s_ord[y]; --y; }
          s_ord[y + 1] = v;
        }
        double tot = 0;
        for (int j = 0; j < k; ++j) tot += sig[j] * sig[j];
        int rr = k;
        double tail = 0;
        for (int jj = k - 1; jj >= 1; --jj) {
          tail += sig[s_ord[jj]] * sig[s_ord[jj]];
          if (tail <= a.eps * a.eps * tot) rr = jj;
          else break;
        }
        if (a.max_rank > 0 && rr > a.max_rank) rr = a.max_rank;
        if (rr < 1) rr = 1;
        s_i[2] = tot > 0 ? rr : -22;
      }
      __syncthreads();
      rn = s_i[2];
      if (rn > 0) {
        // B's map W_r to B's workgroup, A's map (U S)_r kept (in Tm)
        if (tid < k * rn) {
          const int i = tid / rn, jj = tid - i * rn, j = s_ord[jj];
          st_wt(a.xch + 256 + tid, sW[i][j]);
          Tm[i][jj] = sC[i][j];
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __hip_atomic_store((tp_gu32*)(a.flags + 1), (((unsigned)call + 1u) << 8) | ((unsigned)rn & 255u),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (rn <= 0) break;
      if (tid < k * rn) sC[tid / rn][tid - (tid / rn) * rn] = Tm[tid / rn][tid - (tid / rn) * rn];
      __syncthreads();
      TP_STAMP(6);
    }
    // ---- the new factor X <- X M (k x rn), still in LDS (matrix cores) ---------
    {
      d4 xacc[TP_XB];
      xmul(X, N, k, sC, rn, wv, lane, xacc);
      __syncthreads();
      xmul_store(X, N, rn, wv, lane, xacc);
    }
    r = rn;
    __syncthreads();
    TP_STAMP(7);
  }
  // ---- the factors after the last step ------------------------------------------
  const bool ok = call == a.ncalls;
  if (ok) {
    double* dst = side ? a.outB : a.outA;
    for (int e = tid; e < N * r; e += TP_T) {
      const int i = e / r, j = e - i * r;
      dst[(long)i * a.ldo + j] = X[i * r + j];
    }
  }
  if (side == 0 && tid == 0) a.rn_out[0] = ok ? r : -1;
}

}  // namespace

extern "C" {

// Largest N x k factor the persistent step holds in LDS (doubles) and its
// widest factor (columns after the expansion).
int stsp_tt_persist_limits(int* nk_max, int* k_max) {
  *nk_max = TP_NK;
  *k_max = TP_KP;
  return 0;
}

// ncalls factored diffusion steps (each: nsub explicit substeps + one
// CholeskyQR3 recompression) of U = A B^T in one launch.  fp64.  xch: 512
// doubles, flags: 4 unsigned (zeroed here, before the launch).  The final
// rank goes to rn_out[0] (device); outA / outB hold N x rn (ld ldo).
int stsp_tt_persist(const double* A, int lda, const double* B, int ldb, int N, int r, int ncalls, int nsub, double c,
                    double ih2, int periodic, double eps, int max_rank, double* xch, unsigned* flags, double* outA,
                    double* outB, int ldo, int* rn_out, unsigned long long* stamps, double timeout_s,
                    hipStream_t st) {
  if (N < 4 || r < 1 || nsub < 0 || ncalls < 1) return -1;
  const int k = r << nsub;
  if (k > TP_KP || (long)N * k > TP_NK || N > TP_T * TP_RPT) return -2;
  if (max_rank > 0 && (max_rank << nsub) > TP_KP) return -3;
  if (max_rank <= 0) max_rank = TP_KP >> nsub;     // the next step's expansion must fit too
  TPArgs a;
  a.A = A; a.B = B; a.lda = lda; a.ldb = ldb; a.N = N; a.r0 = r; a.ncalls = ncalls; a.nsub = nsub;
  a.periodic = periodic; a.max_rank = max_rank; a.c = c; a.ih2 = ih2; a.eps = eps;
  a.xch = xch; a.flags = flags; a.outA = outA; a.outB = outB; a.ldo = ldo; a.rn_out = rn_out; a.stamps = stamps;
  a.timeout_ticks = (long long)(timeout_s * 1e8);
  if (hipMemsetAsync(flags, 0, 4 * sizeof(unsigned), st) != hipSuccess) return -4;
  hipLaunchKernelGGL(tt_persist_kernel, dim3(2), dim3(TP_T), 0, st, a);
  return (int)hipGetLastError();
}

}  // extern "C"
