// Low-rank / Tensor-Train kernels on the gfx950 matrix cores (MFMA).
//
// The reference's research direction (PDF s.3, s.5, s.19) is to
// carry a panel field U (N x N) in factored form U = A B^T (the d = 2 TT) so the
// FV update becomes "r x r x r multiplies" (PDF s.19) instead of a memory-bound
// stencil.  One explicit diffusion step in factored form (models/tt.py,
// LowRankDiffusion) is:
//
//   expand    A^ = [A, c D A],  B^ = [B + c D B, B]        (k = 2r columns)
//   gram      Ga = A^T A^,  Gb = B^T B^                    (k x k, reduction over N)
//   (host)    eigh(Ga), eigh(Gb), SVD of the k x k core    (microseconds)
//   mm        A' = A^ Xa,  B' = B^ Xb                      (N x k times k x r')
//
// `gram` and `mm` are the tall-skinny GEMMs: MFMA 16x16x4 (f64 or f32 inputs,
// both exact at the vector rate on CDNA4) with one wave per 16-row strip; the
// k x m result of `gram` is reduced over blocks in a fixed order (bitwise
// reproducible, no float atomics).  `expand` is the tridiagonal second
// difference applied to the factors (VALU, memory-bound) and `dense_diffusion`
// is the N x N five-point step the factored form replaces (the comparison
// point, tools/tt_bench.py).
//
// Lane maps of v_mfma_{f64,f32}_16x16x4 (cdna_hip_programming.md section 3):
//   A operand: lane l holds A[row l&15][k l>>4];  B operand: B[k l>>4][col l&15]
//   D, f64:   col = l&15, row = (l>>4) + 4 r     (r = accumulator register 0..3)
//   D, f32:   col = l&15, row = 4 (l>>4) + r
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tt_common.h"

#include <algorithm>
#include <cmath>
#include <vector>

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <typename T> struct Mfma;
template <> struct Mfma<double> {
  typedef d4 acc_t;
  static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct Mfma<float> {
  typedef f4 acc_t;
  static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

constexpr int GRAM_UNROLL = 4;   // 4-row chunks per wave per loop trip (all loads issued first)

// Partial Gram matrices: block b sums rows of the chunks it owns into
// part[b][KT*16][MT*16].  Chunk c (rows 4c..4c+3) belongs to wave
// (c mod (4 * gridDim.x)); each wave keeps KT*MT accumulator tiles.
template <typename T, int KT, int MT>
__global__ __launch_bounds__(256) void gram_partial(const T* __restrict__ A, int lda, const T* __restrict__ B, int ldb,
                                                   int N, int k, int m, T* __restrict__ part) {
  using M = Mfma<T>;
  constexpr int W = MT * 16;
  __shared__ T red[KT * 16 * W];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  typename M::acc_t acc[KT][MT];
#pragma unroll
  for (int i = 0; i < KT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = typename M::acc_t{0, 0, 0, 0};
  const int nchunk = (N + 3) >> 2;
  const int stride = gridDim.x * 4;
  for (int c0 = blockIdx.x * 4 + wave; c0 < nchunk; c0 += stride * GRAM_UNROLL) {
    T a[GRAM_UNROLL][KT], b[GRAM_UNROLL][MT];
#pragma unroll
    for (int u = 0; u < GRAM_UNROLL; ++u) {
      const int row = (c0 + u * stride) * 4 + kq;
      const bool rv = (c0 + u * stride) < nchunk && row < N;
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        const int cc = i * 16 + col;
        a[u][i] = (rv && cc < k) ? A[(size_t)row * lda + cc] : T(0);
      }
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int cc = j * 16 + col;
        b[u][j] = (rv && cc < m) ? B[(size_t)row * ldb + cc] : T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < GRAM_UNROLL; ++u)
#pragma unroll
      for (int i = 0; i < KT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = M::op(a[u][i], b[u][j], acc[i][j]);
  }
  // waves add their tiles into LDS one after the other (fixed order)
  for (int w = 0; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int i = 0; i < KT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int idx = (i * 16 + M::row(lane, r)) * W + j * 16 + col;
            red[idx] = (w == 0 ? T(0) : red[idx]) + acc[i][j][r];
          }
    }
    __syncthreads();
  }
  T* out = part + (size_t)blockIdx.x * (KT * 16 * W);
  for (int e = threadIdx.x; e < KT * 16 * W; e += 256) out[e] = red[e];
}

// C[i][j] = alpha * sum_b part[b][i][j] (fixed order over b), i < k, j < m.
// One lane per entry, the 4 waves of a block split the partials; LDS combine.
template <typename T>
__global__ __launch_bounds__(256) void gram_reduce(const T* __restrict__ part, int P, int E, int W, int k, int m,
                                                  T* __restrict__ C, int ldc, T alpha) {
  __shared__ T s[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int q = (P + 3) >> 2, b0 = wave * q, b1 = min(P, b0 + q);
  T sum = 0;
  if (e < E) {
#pragma unroll 8
    for (int b = b0; b < b1; ++b) sum += part[(size_t)b * E + e];
  }
  s[wave][lane] = sum;
  __syncthreads();
  if (wave == 0 && e < E) {
    const T t = ((s[0][lane] + s[1][lane]) + s[2][lane]) + s[3][lane];
    const int i = e / W, j = e - i * W;
    if (i < k && j < m) C[(size_t)i * ldc + j] = alpha * t;
  }
}

// C = alpha * A X + beta * C;  A [N][k] (lda), X [k][m] (ldx), C [N][m] (ldc).
// A block = 4 waves = 64 rows; X is staged zero-padded in LDS.
template <typename T, int KT, int MT>
__global__ __launch_bounds__(256) void tsmm_kernel(const T* __restrict__ A, int lda, const T* __restrict__ X, int ldx,
                                                  T* __restrict__ C, int ldc, int N, int k, int m, T alpha, T beta) {
  using M = Mfma<T>;
  constexpr int W = MT * 16;
  __shared__ T xs[KT * 16 * W];
  for (int e = threadIdx.x; e < KT * 16 * W; e += 256) {
    const int i = e / W, j = e - i * W;
    xs[e] = (i < k && j < m) ? X[(size_t)i * ldx + j] : T(0);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16;
  const int arow = r0 + col;
  // every A element of the strip is loaded before the first MFMA
  T a[KT * 4];
#pragma unroll
  for (int s = 0; s < KT * 4; ++s) {
    const int kk = s * 4 + kq;
    a[s] = (arow < N && kk < k) ? A[(size_t)arow * lda + kk] : T(0);
  }
  __syncthreads();
  typename M::acc_t acc[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) acc[j] = typename M::acc_t{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < KT * 4; ++s)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[j] = M::op(a[s], xs[(s * 4 + kq) * W + j * 16 + col], acc[j]);
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int cc = j * 16 + col;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + M::row(lane, r);
      if (row < N && cc < m) {
        T* p = C + (size_t)row * ldc + cc;
        *p = beta == T(0) ? alpha * acc[j][r] : alpha * acc[j][r] + beta * *p;
      }
    }
  }
}

// out[:, 0:r] = x0 X + x1 (D X),  out[:, r:2r] = y0 X + y1 (D X), with
// (D X)[i] = (X[i-1] - 2 X[i] + X[i+1]) * ih2 (zero outside, or periodic).
template <typename T>
__global__ __launch_bounds__(256) void expand_kernel(const T* __restrict__ X, int ldx, T* __restrict__ out, int ldo,
                                                    int N, int r, T x0, T x1, T y0, T y1, T ih2, int periodic) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)N * r) return;
  const int i = (int)(e / r), j = (int)(e - (long)i * r);
  const T c = X[(size_t)i * ldx + j];
  int im = i - 1, ip = i + 1;
  if (periodic) {
    im = im < 0 ? N - 1 : im;
    ip = ip >= N ? 0 : ip;
  }
  const T l = im >= 0 ? X[(size_t)im * ldx + j] : T(0);
  const T h = ip < N ? X[(size_t)ip * ldx + j] : T(0);
  const T d = ((l + h) - T(2) * c) * ih2;
  out[(size_t)i * ldo + j] = x0 * c + x1 * d;
  out[(size_t)i * ldo + r + j] = y0 * c + y1 * d;
}

// V = U + c (U_{i-1,j} + U_{i+1,j} + U_{i,j-1} + U_{i,j+1} - 4 U_ij), zero
// Dirichlet outside; 64 x 4 threads per block along contiguous j.
template <typename T>
__global__ __launch_bounds__(256) void dense_diffusion_kernel(const T* __restrict__ U, T* __restrict__ V, int N,
                                                             int Mc, T c) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= N || j >= Mc) return;
  const size_t o = (size_t)i * Mc + j;
  const T u = U[o];
  const T n = i > 0 ? U[o - Mc] : T(0);
  const T s = i + 1 < N ? U[o + Mc] : T(0);
  const T w = j > 0 ? U[o - 1] : T(0);
  const T e = j + 1 < Mc ? U[o + 1] : T(0);
  V[o] = u + c * (((n + s) + (w + e)) - T(4) * u);
}

template <typename T, int KT, int MT>
int gram_launch(const T* A, int lda, const T* B, int ldb, int N, int k, int m, T* work, int P, T* C, int ldc, T alpha,
                hipStream_t st) {
  const int E = KT * 16 * MT * 16;
  hipLaunchKernelGGL((gram_partial<T, KT, MT>), dim3(P), dim3(256), 0, st, A, lda, B, ldb, N, k, m, work);
  hipLaunchKernelGGL(gram_reduce<T>, dim3((E + 63) / 64), dim3(256), 0, st, (const T*)work, P, E, MT * 16, k, m, C,
                     ldc, alpha);
  return (int)hipGetLastError();
}

template <typename T, int KT>
int gram_m(int mt, const T* A, int lda, const T* B, int ldb, int N, int k, int m, T* work, int P, T* C, int ldc,
           T alpha, hipStream_t st) {
  switch (mt) {
    case 1: return gram_launch<T, KT, 1>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, st);
    case 2: return gram_launch<T, KT, 2>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, st);
    case 3: return gram_launch<T, KT, 3>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, st);
    case 4: return gram_launch<T, KT, 4>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, st);
  }
  return -2;
}

template <typename T>
int gram_t(const void* A, int lda, const void* B, int ldb, int N, int k, int m, void* work, int P, void* C, int ldc,
           double alpha, hipStream_t st) {
  const int kt = (k + 15) / 16, mt = (m + 15) / 16;
  const T* a = (const T*)A;
  const T* b = (const T*)B;
  T* w = (T*)work;
  T* c = (T*)C;
  switch (kt) {
    case 1: return gram_m<T, 1>(mt, a, lda, b, ldb, N, k, m, w, P, c, ldc, (T)alpha, st);
    case 2: return gram_m<T, 2>(mt, a, lda, b, ldb, N, k, m, w, P, c, ldc, (T)alpha, st);
    case 3: return gram_m<T, 3>(mt, a, lda, b, ldb, N, k, m, w, P, c, ldc, (T)alpha, st);
    case 4: return gram_m<T, 4>(mt, a, lda, b, ldb, N, k, m, w, P, c, ldc, (T)alpha, st);
  }
  return -2;
}

template <typename T, int KT, int MT>
int tsmm_launch(const T* A, int lda, const T* X, int ldx, T* C, int ldc, int N, int k, int m, T alpha, T beta,
                hipStream_t st) {
  hipLaunchKernelGGL((tsmm_kernel<T, KT, MT>), dim3((N + 63) / 64), dim3(256), 0, st, A, lda, X, ldx, C, ldc, N, k, m,
                     alpha, beta);
  return (int)hipGetLastError();
}

template <typename T, int KT>
int tsmm_m(int mt, const T* A, int lda, const T* X, int ldx, T* C, int ldc, int N, int k, int m, T alpha, T beta,
           hipStream_t st) {
  switch (mt) {
    case 1: return tsmm_launch<T, KT, 1>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, st);
    case 2: return tsmm_launch<T, KT, 2>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, st);
    case 3: return tsmm_launch<T, KT, 3>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, st);
    case 4: return tsmm_launch<T, KT, 4>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, st);
  }
  return -2;
}

template <typename T>
int tsmm_t(const void* A, int lda, const void* X, int ldx, void* C, int ldc, int N, int k, int m, double alpha,
           double beta, hipStream_t st) {
  const int kt = (k + 15) / 16, mt = (m + 15) / 16;
  const T* a = (const T*)A;
  const T* x = (const T*)X;
  T* c = (T*)C;
  switch (kt) {
    case 1: return tsmm_m<T, 1>(mt, a, lda, x, ldx, c, ldc, N, k, m, (T)alpha, (T)beta, st);
    case 2: return tsmm_m<T, 2>(mt, a, lda, x, ldx, c, ldc, N, k, m, (T)alpha, (T)beta, st);
    case 3: return tsmm_m<T, 3>(mt, a, lda, x, ldx, c, ldc, N, k, m, (T)alpha, (T)beta, st);
    case 4: return tsmm_m<T, 4>(mt, a, lda, x, ldx, c, ldc, N, k, m, (T)alpha, (T)beta, st);
  }
  return -2;
}

// ---------------------------------------------------------------------------
// Host side of the factored step: the 2r x 2r "core" (microseconds of scalar
// work; a BLAS call or a Python round trip costs more than the arithmetic).
// ---------------------------------------------------------------------------

// Cyclic Jacobi eigen-decomposition of the symmetric n x n matrix a (row-major,
// destroyed): eigenvalues w[j], eigenvectors in the columns of v.
void jacobi_eigh(int n, double* a, double* w, double* v) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) v[i * n + j] = i == j ? 1.0 : 0.0;
  double nrm = 0;
  for (int i = 0; i < n * n; ++i) nrm += a[i] * a[i];
  // entries below 1e-15 |a|_F only move eigenvalues far under the 1e-13 max
  // cut of gram_factor; rotating them would chase rounding noise forever
  const double tiny = 1e-15 * std::sqrt(nrm);
  for (int sweep = 0; sweep < 64; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = a[p * n + q];
        if (std::fabs(apq) <= tiny ||
            std::fabs(apq) <= 1e-16 * std::sqrt(std::fabs(a[p * n + p] * a[q * n + q]))) {
          a[p * n + q] = a[q * n + p] = 0.0;
          continue;
        }
        rotated = true;
        const double th = (a[q * n + q] - a[p * n + p]) / (2.0 * apq);
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double kp = a[k * n + p], kq = a[k * n + q];
          a[k * n + p] = c * kp - s * kq;
          a[k * n + q] = s * kp + c * kq;
        }
        for (int k = 0; k < n; ++k) {
          const double pk = a[p * n + k], qk = a[q * n + k];
          a[p * n + k] = c * pk - s * qk;
          a[q * n + k] = s * pk + c * qk;
        }
        for (int k = 0; k < n; ++k) {
          const double kp = v[k * n + p], kq = v[k * n + q];
          v[k * n + p] = c * kp - s * kq;
          v[k * n + q] = s * kp + c * kq;
        }
      }
    if (!rotated) break;
  }
  for (int i = 0; i < n; ++i) w[i] = a[i * n + i];
}

// One-sided (Hestenes) Jacobi SVD of m (rows x cols, row-major, overwritten by
// U Sigma): on return the columns of m are mutually orthogonal, sig[j] = |col j|
// and m = (m_out) W^T with W (cols x cols) in w.
void jacobi_svd(int rows, int cols, double* m, double* sig, double* w) {
  for (int i = 0; i < cols; ++i)
    for (int j = 0; j < cols; ++j) w[i * cols + j] = i == j ? 1.0 : 0.0;
  double tot = 0;
  for (int i = 0; i < rows * cols; ++i) tot += m[i] * m[i];
  const double tiny = 1e-30 * tot;   // columns this small are rounding noise
  for (int sweep = 0; sweep < 64; ++sweep) {
    bool rotated = false;
    for (int p = 0; p < cols; ++p)
      for (int q = p + 1; q < cols; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int k = 0; k < rows; ++k) {
          const double x = m[k * cols + p], y = m[k * cols + q];
          al += x * x;
          be += y * y;
          ga += x * y;
        }
        if (al <= tiny || be <= tiny || std::fabs(ga) <= 1e-15 * std::sqrt(al * be)) continue;
        rotated = true;
        const double ze = (be - al) / (2.0 * ga);
        const double t = (ze >= 0 ? 1.0 : -1.0) / (std::fabs(ze) + std::sqrt(1.0 + ze * ze));
        const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
        for (int k = 0; k < rows; ++k) {
          const double x = m[k * cols + p], y = m[k * cols + q];
          m[k * cols + p] = c * x - s * y;
          m[k * cols + q] = s * x + c * y;
        }
        for (int k = 0; k < cols; ++k) {
          const double x = w[k * cols + p], y = w[k * cols + q];
          w[k * cols + p] = c * x - s * y;
          w[k * cols + q] = s * x + c * y;
        }
      }
    if (!rotated) break;
  }
  for (int j = 0; j < cols; ++j) {
    double s2 = 0;
    for (int k = 0; k < rows; ++k) s2 += m[k * cols + j] * m[k * cols + j];
    sig[j] = std::sqrt(s2);
  }
}

// Factor G = R^T R of a PSD Gram matrix through its eigenvectors, dropping
// eigenvalues below 1e-13 max: R = sqrt(L) V^T (rho x k) and I = V L^-1/2 (k x rho).
int gram_factor(int k, const double* g, double* R, double* I) {
  std::vector<double> a(k * k), w(k), v(k * k);
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) a[i * k + j] = 0.5 * (g[i * k + j] + g[j * k + i]);
  jacobi_eigh(k, a.data(), w.data(), v.data());
  double wmax = 0;
  for (int i = 0; i < k; ++i) wmax = std::max(wmax, w[i]);
  int rho = 0;
  for (int j = 0; j < k; ++j) {
    if (!(w[j] > 1e-13 * std::max(wmax, 1e-300))) continue;
    const double sq = std::sqrt(w[j]);
    for (int i = 0; i < k; ++i) {
      R[rho * k + i] = sq * v[i * k + j];
      I[i * k + rho] = v[i * k + j] / sq;   // I has row stride k
    }
    ++rho;
  }
  return rho;
}

// Core maps of the recompression: Xa (k x rn), Xb (k x rn), written as
// X[i * ldx + j] and X[i * ldx + rn + j].  Returns rn (0 on a zero field).
int lr_core(int k, const double* Ga, const double* Gb, double eps, int max_rank, double* X, int ldx) {
  std::vector<double> Ra(k * k), Ia(k * k), Rb(k * k), Ib(k * k);
  const int ra = gram_factor(k, Ga, Ra.data(), Ia.data());
  const int rb = gram_factor(k, Gb, Rb.data(), Ib.data());
  if (ra == 0 || rb == 0) return 0;
  std::vector<double> M(ra * rb), sig(rb), W(rb * rb);
  for (int i = 0; i < ra; ++i)
    for (int j = 0; j < rb; ++j) {
      double t = 0;
      for (int l = 0; l < k; ++l) t += Ra[i * k + l] * Rb[j * k + l];
      M[i * rb + j] = t;
    }
  jacobi_svd(ra, rb, M.data(), sig.data(), W.data());
  std::vector<int> ord(rb);
  for (int j = 0; j < rb; ++j) ord[j] = j;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return sig[x] > sig[y]; });
  double tot = 0;
  for (int j = 0; j < rb; ++j) tot += sig[j] * sig[j];
  int rn = std::min(ra, rb);
  double tail = 0;   // smallest rank whose discarded tail is <= eps^2 * total
  for (int j = std::min(ra, rb) - 1; j >= 1; --j) {
    tail += sig[ord[j]] * sig[ord[j]];
    if (tail <= eps * eps * tot) rn = j;
    else break;
  }
  if (max_rank > 0) rn = std::min(rn, max_rank);
  rn = std::max(rn, 1);
  // Xa = Ia (U Sigma)_r, where U Sigma = M's columns (ra x rb after rotation);
  // Xb = Ib W_r
  for (int i = 0; i < k; ++i)
    for (int jj = 0; jj < rn; ++jj) {
      const int j = ord[jj];
      double ta = 0, tb = 0;
      for (int l = 0; l < ra; ++l) ta += Ia[i * k + l] * M[l * rb + j];
      for (int l = 0; l < rb; ++l) tb += Ib[i * k + l] * W[l * rb + j];
      X[i * ldx + jj] = ta;
      X[i * ldx + rn + jj] = tb;
    }
  return rn;
}


// ---------------------------------------------------------------------------
// Shifted CholeskyQR (Fukaya et al. 2020) for the factored step's tall-skinny
// factors: X = Q R with Q orthonormal to working precision.  One pass is
//   G = X^T X (gram, MFMA),  G + s I = R^T R,  Q = X R^-1 (tsmm, MFMA)
// with s = shift_c * trace(G); three passes (CholeskyQR3) give Q to machine
// precision where the Gram/eigen route stopped at sqrt(eps), and the shift in
// every pass keeps the Cholesky defined when X is (numerically) rank deficient
// (the duplicated columns of the expanded factors): X = Q R still holds, and
// Q's near-null directions carry no weight in the product, so the truncation
// bound of the core SVD is unchanged.
//
// This kernel is the k x k part of one pass: one wave per matrix (batch =
// blockIdx.x).  Lane c holds column c of G in registers (padded to KP = 16,
// 32 or 64 with an identity block, R = diag(R_k, I), so every loop has static
// bounds); the right-looking Cholesky and then R^-1 by back substitution take
// the other columns' entries by lane shuffles (ds_bpermute), no LDS round
// trip and no barrier per column.  The round-5 form (thread per column through
// LDS, three barriers per column) took 54 us per k ~ 30 matrix in the six-panel
// SWE's roundings (profiles/r6_tt).  info[b] = j + 1 if pivot j was not
// positive (left for the host to report; the factor is then unusable).
template <typename T, int KP>
__device__ __forceinline__ void chol_inv_wave(const T* __restrict__ G, int ldg, T* __restrict__ R,
                                              T* __restrict__ Ri, int ldr, int k, double shift_c, T tr,
                                              int* __restrict__ info, int istride) {
  const int lane = threadIdx.x;
  // shift_c < 0: try the plain Cholesky first and shift (by |shift_c|) only
  // if a pivot fails (CholeskyQR passes 2 and 3: orthonormal to eps when the
  // factor is well conditioned, defined when it is rank deficient)
  const bool adaptive = shift_c < 0;
  const T sc = T(adaptive ? -shift_c : shift_c);
  T g[KP];
  int fail = 0;
  for (int attempt = adaptive ? 0 : 1; attempt < 2; ++attempt) {
#pragma unroll
    for (int i = 0; i < KP; ++i) {
      g[i] = (i < k && lane < k) ? G[(long)i * ldg + lane] : (i == lane ? T(1) : T(0));
      if (attempt == 1 && i == lane && lane < k) g[i] += sc * tr;
    }
    fail = 0;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      T d = tt::lane_bcast(g[j], j);
      if (!(d > T(0))) { if (!fail) fail = j + 1; d = T(1); }
      const T sq = sqrt(d);
      if (lane == j) g[j] = sq;
      if (lane > j) g[j] /= sq;
      const T rt = g[j];
#pragma unroll
      for (int i = j + 1; i < KP; ++i) {
        const T rji = tt::lane_bcast(g[j], i);     // R[j][i]: lane i's column
        if (i <= lane) g[i] -= rji * rt;
      }
    }
    if (!fail) break;
  }
  // column c of R^-1: x[c][c] = 1 / R[c][c], x[i][c] = -(sum_{i<l<=c} R[i][l] x[l][c]) / R[i][i]
  T ri[KP];
#pragma unroll
  for (int i = KP - 1; i >= 0; --i) {
    const T rii = tt::lane_bcast(g[i], i);
    T sum = T(0);
#pragma unroll
    for (int l = i + 1; l < KP; ++l) sum += tt::lane_bcast(g[i], l) * ri[l];
    ri[i] = i == lane ? T(1) / rii : (i < lane ? -sum / rii : T(0));
  }
  if (lane < k) {
#pragma unroll
    for (int i = 0; i < KP; ++i)
      if (i < k) {
        R[(long)i * ldr + lane] = i <= lane ? g[i] : T(0);
        Ri[(long)i * ldr + lane] = ri[i];
      }
  }
  if (lane == 0) info[blockIdx.x * istride] = fail;
}

template <typename T>
__global__ __launch_bounds__(64) void chol_inv_kernel(const T* __restrict__ G, int ldg, long sg, T* __restrict__ R,
                                                      T* __restrict__ Ri, int ldr, long sr, int k, double shift_c,
                                                      int* __restrict__ info, int istride) {
  const int b = blockIdx.x, t = threadIdx.x;
  G += b * sg;
  R += b * sr;
  Ri += b * sr;
  T tr = t < k ? G[(long)t * ldg + t] : T(0);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) tr += __shfl_xor(tr, o);
  // an exactly zero factor (G = 0: a field at rest times a coefficient) is
  // X = Q R with Q = X, R = 0: R^-1 := I, no failure; its core is zero and the
  // recompression reports the zero product (-22) for the caller to map to the
  // rank-1 zero field
  if (tr == T(0)) {
    if (t < k)
      for (int i = 0; i < k; ++i) {
        R[(long)i * ldr + t] = T(0);
        Ri[(long)i * ldr + t] = i == t ? T(1) : T(0);
      }
    if (t == 0) info[b * istride] = 0;
    return;
  }
  if (k <= 16) chol_inv_wave<T, 16>(G, ldg, R, Ri, ldr, k, shift_c, tr, info, istride);
  else if (k <= 32) chol_inv_wave<T, 32>(G, ldg, R, Ri, ldr, k, shift_c, tr, info, istride);
  else chol_inv_wave<T, 64>(G, ldg, R, Ri, ldr, k, shift_c, tr, info, istride);
}


// The k x k core of the CholeskyQR3 recompression on the device (k <= 32, one
// workgroup, fp64 arithmetic for either element type): Rt = R3 R2 R1 per
// factor, C = Rt_A Rt_B^T, one-sided (Hestenes) Jacobi SVD of C with the
// round-robin pair order (16 lanes per column pair, one barrier per round),
// singular values sorted, the eps / max_rank truncation, and the core maps
// X = [U S | W] (k x 2k, row stride 2k, rn columns each) of the final
// products; out[0] = rn (<= 0: failure code).  Replaces the host round trip
// of stsp_tt_lr_step3 (six R factors down, jacobi_svd on the host, X up).
constexpr int CORE_K = 32;

template <typename T>
__global__ __launch_bounds__(256) void tt_core_kernel(const T* __restrict__ Rs, const int* __restrict__ dinfo, int k,
                                                      double eps, int max_rank, T* __restrict__ X,
                                                      int* __restrict__ out) {
  constexpr int K = CORE_K, KS = CORE_K + 1;
  __shared__ double sR[2][3][K * K];        // R factors [side][pass]
  __shared__ double sP[2][K * K];           // R2 R1
  __shared__ double sC[K * KS], sW[K * KS];
  __shared__ double sig[K];
  __shared__ int s_ord[K];
  __shared__ int s_flag, s_rot, s_rn;
  __shared__ double s_tot;
  const int tid = threadIdx.x;
  const int kk = k * k;
  if (tid == 0) {
    int bad = 0;
    for (int i = 0; i < 6; ++i) bad |= dinfo[i] != 0;
    s_flag = bad;
  }
  for (int e = tid; e < 6 * kk; e += blockDim.x) {
    const int sp = e / kk, r = e - sp * kk;
    sR[sp / 3][sp % 3][r] = (double)Rs[(size_t)(sp * 2) * kk + r];     // [side][pass][R, Ri]: the R block
  }
  __syncthreads();
  if (s_flag) {
    if (tid == 0) out[0] = -24;
    return;
  }
  // P = R2 R1, then R3 P (into sR[side][0]); upper-triangular left factors
  for (int e = tid; e < 2 * kk; e += blockDim.x) {
    const int sd = e / kk, r = e - sd * kk, i = r / k, j = r - i * k;
    double acc = 0;
    for (int l = i; l < k; ++l) acc += sR[sd][1][i * k + l] * sR[sd][0][l * k + j];
    sP[sd][r] = acc;
  }
  __syncthreads();
  for (int e = tid; e < 2 * kk; e += blockDim.x) {
    const int sd = e / kk, r = e - sd * kk, i = r / k, j = r - i * k;
    double acc = 0;
    for (int l = i; l < k; ++l) acc += sR[sd][2][i * k + l] * sP[sd][l * k + j];
    sR[sd][0][r] = acc;
  }
  __syncthreads();
  // C = Rt_A Rt_B^T, W = I
  for (int e = tid; e < kk; e += blockDim.x) {
    const int i = e / k, j = e - i * k;
    double acc = 0;
    for (int l = 0; l < k; ++l) acc += sR[0][0][i * k + l] * sR[1][0][j * k + l];
    sC[i * KS + j] = acc;
    sW[i * KS + j] = i == j ? 1.0 : 0.0;
  }
  __syncthreads();
  {   // ||C||_F^2: strided partial sums, wave reduction, one add per wave
    double t = 0;
    for (int e = tid; e < kk; e += blockDim.x) {
      const double x = sC[(e / k) * KS + e % k];
      t += x * x;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
    if ((tid & 63) == 0) sig[tid >> 6] = t;     // sig[] is free until the sweeps end
    __syncthreads();
    if (tid == 0) s_tot = (sig[0] + sig[1]) + (sig[2] + sig[3]);   // fixed order: reproducible
  }
  __syncthreads();
  // only rounding noise (below 1e-15 of ||C||) is left unrotated.  Skipping
  // every column below 1 % of the truncation tolerance saved ~20 % of the
  // sweeps on the six-panel SWE's fp64 cores but changed the rank of an fp32
  // core (eps 1e-6: 3 vs the host's 7; tests/test_tt_kernels.py): a column
  // small early in the sweeps can still gain weight from a large one
  const double tiny = 1e-30 * s_tot;
  // round-robin: m = k rounded up to even, position 0 fixed, the rest rotate;
  // pair p joins positions p and m - 1 - p (index k: the dummy of odd k)
  const int m = (k + 1) & ~1;
  const int pr = tid >> 4, ln = tid & 15;
  for (int sweep = 0; sweep < 60; ++sweep) {
    if (tid == 0) s_rot = 0;
    __syncthreads();
    for (int rd = 0; rd < m - 1; ++rd) {
      if (pr < m / 2) {
        const int qa = pr, qb = m - 1 - pr;
        int p = qa == 0 ? 0 : 1 + (qa - 1 + rd) % (m - 1);
        int q = qb == 0 ? 0 : 1 + (qb - 1 + rd) % (m - 1);
        if (p > q) { const int x = p; p = q; q = x; }
        if (q < k) {
          double al = 0, be = 0, ga = 0;
          for (int r = ln; r < k; r += 16) {
            const double x = sC[r * KS + p], y = sC[r * KS + q];
            al += x * x;
            be += y * y;
            ga += x * y;
          }
          // 16-lane sums through DPP; every lane of the wave runs them (the
          // pair guard above is lane-group uniform and DPP needs no exec gaps
          // inside a row)
          al = tt::sum16(al);
          be = tt::sum16(be);
          ga = tt::sum16(ga);
          if (!(al <= tiny || be <= tiny || fabs(ga) <= 1e-15 * sqrt(al * be))) {
            const double ze = (be - al) / (2.0 * ga);
            const double t = (ze >= 0 ? 1.0 : -1.0) / (fabs(ze) + sqrt(1.0 + ze * ze));
            const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
            for (int r = ln; r < k; r += 16) {
              const double x = sC[r * KS + p], y = sC[r * KS + q];
              sC[r * KS + p] = c * x - s * y;
              sC[r * KS + q] = s * x + c * y;
              const double u = sW[r * KS + p], w = sW[r * KS + q];
              sW[r * KS + p] = c * u - s * w;
              sW[r * KS + q] = s * u + c * w;
            }
            if (ln == 0) s_rot = 1;
          }
        }
      }
      __syncthreads();
    }
    const int rot = s_rot;
    __syncthreads();
    if (!rot) break;
  }
  if (tid < k) {
    double s2 = 0;
    for (int r = 0; r < k; ++r) s2 += sC[r * KS + tid] * sC[r * KS + tid];
    sig[tid] = sqrt(s2);
  }
  __syncthreads();
  if (tid < k) {   // descending order by rank (ties by index): thread j places column j
    const double v = sig[tid];
    int r = 0;
    for (int i = 0; i < k; ++i) r += sig[i] > v || (sig[i] == v && i < tid);
    s_ord[r] = tid;
  }
  __syncthreads();
  if (tid == 0) {
    double tot = 0;
    for (int j = 0; j < k; ++j) tot += sig[j] * sig[j];
    int rn = k;
    double tail = 0;
    for (int jj = k - 1; jj >= 1; --jj) {
      tail += sig[s_ord[jj]] * sig[s_ord[jj]];
      if (tail <= eps * eps * tot) rn = jj;
      else break;
    }
    if (max_rank > 0 && rn > max_rank) rn = max_rank;
    if (rn < 1) rn = 1;
    s_rn = tot > 0 ? rn : -22;
  }
  __syncthreads();
  const int rn = s_rn;
  if (rn > 0) {
    for (int e = tid; e < k * rn; e += blockDim.x) {
      const int i = e / rn, jj = e - i * rn, j = s_ord[jj];
      X[(size_t)i * 2 * k + jj] = (T)sC[i * KS + j];
      X[(size_t)i * 2 * k + rn + jj] = (T)sW[i * KS + j];
    }
  }
  if (tid == 0) out[0] = rn;
}

}  // namespace

extern "C" {

// Blocks `gram` uses for N rows (the partial-workspace size is
// stsp_tt_gram_blocks(N) * ceil16(k) * ceil16(m) elements).
int stsp_tt_gram_blocks(int N) {
  const int chunks = (N + 3) / 4;
  int p = (chunks + 4 * 4 * GRAM_UNROLL - 1) / (4 * 4 * GRAM_UNROLL);   // >= 4 loop trips per wave
  return p < 1 ? 1 : (p > 256 ? 256 : p);
}

// C[k][m] (ldc) = alpha * A^T B,  A [N][k] (lda), B [N][m] (ldb), k, m <= 64.
int stsp_tt_gram(int dtype, const void* A, int lda, const void* B, int ldb, int N, int k, int m, void* work, int P,
                 void* C, int ldc, double alpha, hipStream_t stream) {
  if (k < 1 || m < 1 || k > 64 || m > 64 || N < 1 || P < 1) return -1;
  if (dtype == 1) return gram_t<double>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, stream);
  if (dtype == 0) return gram_t<float>(A, lda, B, ldb, N, k, m, work, P, C, ldc, alpha, stream);
  return -4;
}

// Batched shifted Cholesky + factor inverse (chol_inv_kernel): for b < batch,
// G_b + shift_c trace(G_b) I = R_b^T R_b, Ri_b = R_b^-1 (k <= 64, row-major;
// shift_c < 0: unshifted unless a pivot fails, then shifted by |shift_c|,
// batch strides sg / sr in elements), info[b] = 0 or the failing pivot + 1.
static int chol_inv_launch(int dtype, const void* G, int ldg, long sg, void* R, void* Ri, int ldr, long sr, int k,
                           int batch, double shift_c, int* info, int istride, hipStream_t stream) {
  if (k < 1 || k > 64 || batch < 1) return -1;
  if (dtype == 1)
    hipLaunchKernelGGL(chol_inv_kernel<double>, dim3(batch), dim3(64), 0, stream, (const double*)G, ldg, sg,
                       (double*)R, (double*)Ri, ldr, sr, k, shift_c, info, istride);
  else if (dtype == 0)
    hipLaunchKernelGGL(chol_inv_kernel<float>, dim3(batch), dim3(64), 0, stream, (const float*)G, ldg, sg, (float*)R,
                       (float*)Ri, ldr, sr, k, shift_c, info, istride);
  else
    return -4;
  return (int)hipGetLastError();
}

int stsp_tt_chol_inv(int dtype, const void* G, int ldg, long sg, void* R, void* Ri, int ldr, long sr, int k,
                     int batch, double shift_c, int* info, hipStream_t stream) {
  return chol_inv_launch(dtype, G, ldg, sg, R, Ri, ldr, sr, k, batch, shift_c, info, 1, stream);
}

// C[N][m] (ldc) = alpha * A X + beta * C,  A [N][k] (lda), X [k][m] (ldx), k, m <= 64.
int stsp_tt_mm(int dtype, const void* A, int lda, const void* X, int ldx, void* C, int ldc, int N, int k, int m,
               double alpha, double beta, hipStream_t stream) {
  if (k < 1 || m < 1 || k > 64 || m > 64 || N < 1) return -1;
  if (dtype == 1) return tsmm_t<double>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, stream);
  if (dtype == 0) return tsmm_t<float>(A, lda, X, ldx, C, ldc, N, k, m, alpha, beta, stream);
  return -4;
}

int stsp_tt_expand(int dtype, const void* X, int ldx, void* out, int ldo, int N, int r, double x0, double x1,
                   double y0, double y1, double ih2, int periodic, hipStream_t stream) {
  if (N < 1 || r < 1 || ldo < 2 * r) return -1;
  const long n = (long)N * r;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == 1)
    hipLaunchKernelGGL(expand_kernel<double>, grid, dim3(256), 0, stream, (const double*)X, ldx, (double*)out, ldo, N,
                       r, x0, x1, y0, y1, ih2, periodic);
  else if (dtype == 0)
    hipLaunchKernelGGL(expand_kernel<float>, grid, dim3(256), 0, stream, (const float*)X, ldx, (float*)out, ldo, N, r,
                       (float)x0, (float)x1, (float)y0, (float)y1, (float)ih2, periodic);
  else
    return -4;
  return (int)hipGetLastError();
}

int stsp_tt_dense_diffusion(int dtype, const void* U, void* V, int N, int M, double c, hipStream_t stream) {
  if (N < 1 || M < 1) return -1;
  const dim3 grid((M + 63) / 64, (N + 3) / 4);
  if (dtype == 1)
    hipLaunchKernelGGL(dense_diffusion_kernel<double>, grid, dim3(256), 0, stream, (const double*)U, (double*)V, N, M,
                       c);
  else if (dtype == 0)
    hipLaunchKernelGGL(dense_diffusion_kernel<float>, grid, dim3(256), 0, stream, (const float*)U, (float*)V, N, M,
                       (float)c);
  else
    return -4;
  return (int)hipGetLastError();
}

// Host only: core maps of the factored step from the two k x k Gram matrices
// (G = [Ga, Gb], doubles).  X (k x ldx, ldx >= 2 k) receives [Xa | Xb].
int stsp_tt_core(int k, const double* G, double eps, int max_rank, double* X, int ldx) {
  if (k < 1 || k > 64 || ldx < 2 * k) return -1;
  return lr_core(k, G, G + k * k, eps, max_rank, X, ldx);
}

// nsub explicit factored diffusion steps U' = U + c (D U + U D^T) for U = A B^T
// (A, B: N x r, row strides lda / ldb), then ONE recompression to rank
// rn <= max_rank: expand nsub times (2 launches each; the rank doubles every
// step, k = 2^nsub r <= 64, exact: no truncation in between) -> MFMA Gram
// (2 x 2 launches) -> Gram to pinned host -> host core -> maps to the device
// -> MFMA products into Aout / Bout (N x rn, row stride ldo).  The sync and the
// host core are paid once per nsub steps: the step is latency-bound (~70 us at
// every N with nsub = 1, profiles/r1_tt_bench.log), so rounding every second
// step halves its cost per step.  ws = device workspace
// (stsp_tt_step_workspace2 elements), hbuf = pinned host buffer of 4 k^2
// doubles.  Returns rn (> 0) or an error (< 0).
size_t stsp_tt_step_workspace2(int N, int r, int nsub) {
  const int k = r << nsub, kp = (k + 15) / 16 * 16;
  return (size_t)2 * 2 * N * k + 2 * (size_t)k * k + (size_t)stsp_tt_gram_blocks(N) * kp * kp + (size_t)k * 2 * k;
}
size_t stsp_tt_step_workspace(int N, int r) { return stsp_tt_step_workspace2(N, r, 1); }

int stsp_tt_lr_step2(int dtype, const void* A, int lda, const void* B, int ldb, int N, int r, int nsub, double c,
                     double ih2, int periodic, double eps, int max_rank, void* ws, double* hbuf, void* Aout,
                     void* Bout, int ldo, hipStream_t st) {
  if (N < 1 || r < 1 || nsub < 1 || nsub > 6) return -1;
  const int k = r << nsub;
  if (k > 64) return -1;
  const size_t es = dtype == 1 ? 8 : 4;
  char* w = (char*)ws;
  // ping-pong expansion buffers: [A-side, B-side] x 2, each N x k (row stride k)
  void* buf[2][2] = {{w, w + es * (size_t)N * k}, {w + es * 2 * (size_t)N * k, w + es * 3 * (size_t)N * k}};
  void* G = w + es * 4 * (size_t)N * k;
  void* part = (char*)G + es * 2 * (size_t)k * k;
  const int P = stsp_tt_gram_blocks(N);
  const int kp = (k + 15) / 16 * 16;
  void* dX = (char*)part + es * (size_t)P * kp * kp;
  int rc;
  const void* srcA = A;
  const void* srcB = B;
  int sa = lda, sb = ldb, rr = r, cur = 0;
  for (int s = 0; s < nsub; ++s, rr *= 2) {
    void* dA = buf[cur][0];
    void* dB = buf[cur][1];
    if ((rc = stsp_tt_expand(dtype, srcA, sa, dA, 2 * rr, N, rr, 1.0, 0.0, 0.0, c, ih2, periodic, st))) return rc;
    if ((rc = stsp_tt_expand(dtype, srcB, sb, dB, 2 * rr, N, rr, 1.0, c, 1.0, 0.0, ih2, periodic, st))) return rc;
    srcA = dA;
    srcB = dB;
    sa = sb = 2 * rr;
    cur ^= 1;
  }
  void* Ah = (void*)srcA;
  void* Bh = (void*)srcB;
  if ((rc = stsp_tt_gram(dtype, Ah, k, Ah, k, N, k, k, part, P, G, k, 1.0, st))) return rc;
  if ((rc = stsp_tt_gram(dtype, Bh, k, Bh, k, N, k, k, part, P, (char*)G + es * k * k, k, 1.0, st))) return rc;
  double* hG = hbuf;
  double* hX = hbuf + 2 * k * k;
  if (hipMemcpyAsync(hG, G, es * 2 * k * k, hipMemcpyDeviceToHost, st) != hipSuccess) return -20;
  if (hipStreamSynchronize(st) != hipSuccess) return -21;
  if (dtype == 0) {   // widen in place (back to front)
    const float* f = (const float*)hG;
    for (int i = 2 * k * k - 1; i >= 0; --i) hG[i] = (double)f[i];
  }
  const int rn = lr_core(k, hG, hG + k * k, eps, max_rank, hX, 2 * k);
  if (rn <= 0) return -22;
  if (dtype == 0) {   // narrow in place (front to back)
    float* f = (float*)hX;
    for (int i = 0; i < 2 * k * k; ++i) f[i] = (float)hX[i];
  }
  if (hipMemcpyAsync(dX, hX, es * 2 * k * k, hipMemcpyHostToDevice, st) != hipSuccess) return -23;
  if ((rc = stsp_tt_mm(dtype, Ah, k, dX, 2 * k, Aout, ldo, N, k, rn, 1.0, 0.0, st))) return rc;
  if ((rc = stsp_tt_mm(dtype, Bh, k, (char*)dX + es * rn, 2 * k, Bout, ldo, N, k, rn, 1.0, 0.0, st))) return rc;
  return rn;
}

// The same step with the CholeskyQR3 recompression (models/tt.py::cholqr3) in
// one native call: expansion, three passes per factor of {MFMA Gram, shifted
// Cholesky + inverse (chol_inv_kernel), MFMA product}, one device-to-host copy
// of the six k x k R factors and pivot flags, the core C = Ra Rb^T and its
// one-sided Jacobi SVD on the host, one host-to-device copy, two MFMA products.
// Workspace: stsp_tt_step_workspace3 elements; hbuf: 8 k^2 + 8 doubles.
size_t stsp_tt_step_workspace3(int N, int r, int nsub) {
  const int k = r << nsub, kp = (k + 15) / 16 * 16;
  return (size_t)2 * 2 * N * k + 2 * (size_t)k * k + (size_t)stsp_tt_gram_blocks(N) * kp * kp + (size_t)k * 2 * k +
         (size_t)12 * k * k + 16;
}

// stsp_tt_set_core: 1 (default) forms the k x k core of stsp_tt_lr_step3 /
// stsp_tt_recompress on the device when k <= 32 (tt_core_kernel); 0: on the
// host (jacobi_svd), for comparison.

// CholeskyQR3 of the two factors X[side] [N[side]][k] (row stride ldx[side])
// side by side on the device (models/tt.py::cholqr3): per pass one MFMA Gram
// per factor, ONE batched shifted Cholesky + inverse for both (two waves in
// parallel: the single-wave latency chain is paid once per pass, not twice),
// one MFMA product per factor.  Passes write s0, s1, s0 (row stride k), so Q
// ends in s0[side] and s1[side] may alias X[side].  G: 2 k^2; Rs: [side][pass]
// [R, Ri] k x k; dinfo[side * 3 + pass].  The shift uses the taller factor.
static int cholqr3_pair(int dtype, const void* const X[2], const int ldx[2], const int N[2], int k,
                        void* const s0[2], void* const s1[2], void* part, void* G, char* Rs, int* dinfo,
                        hipStream_t st) {
  const size_t es = dtype == 1 ? 8 : 4;
  const size_t kk = (size_t)k * k;
  // shift coefficient 11 (N k + k (k + 1)) u (models/tt.py::cholqr3_shift)
  const double u = dtype == 1 ? 1.1102230246251565e-16 : 5.960464477539063e-08;
  const int Nmax = N[0] > N[1] ? N[0] : N[1];
  const double shc = 11.0 * ((double)Nmax * k + (double)k * (k + 1)) * u;
  const void* in[2] = {X[0], X[1]};
  int ldin[2] = {ldx[0], ldx[1]};
  int rc;
  for (int pass = 0; pass < 3; ++pass) {
    for (int side = 0; side < 2; ++side)
      if ((rc = stsp_tt_gram(dtype, in[side], ldin[side], in[side], ldin[side], N[side], k, k, part,
                             stsp_tt_gram_blocks(N[side]), (char*)G + es * side * kk, k, 1.0, st)))
        return rc;
    char* R0 = Rs + es * (size_t)(pass * 2) * kk;          // side 0's R of this pass; side 1 at + 6 k^2
    if ((rc = chol_inv_launch(dtype, G, k, (long)kk, R0, R0 + es * kk, k, (long)(6 * kk), k, 2,
                              pass == 0 ? shc : -shc, dinfo + pass, 3, st)))
      return rc;
    for (int side = 0; side < 2; ++side) {
      void* out = pass == 1 ? s1[side] : s0[side];
      const char* Ri = R0 + es * (size_t)side * 6 * kk + es * kk;
      if ((rc = stsp_tt_mm(dtype, in[side], ldin[side], Ri, k, out, k, N[side], k, k, 1.0, 0.0, st))) return rc;
      in[side] = out;
      ldin[side] = k;
    }
  }
  return 0;
}

// The k x k core of a recompression after CholeskyQR3 of both factors (Rs:
// [side][pass][R, Ri], dinfo[side * 3 + pass], Q[side] with row stride k) and
// the two final MFMA products Aout = QA (U S)_rn, Bout = QB W_rn.  k <= 32 and
// tt_core_mode: tt_core_kernel on the device, one 4-byte read-back (the rank
// sizes the products); else the six R factors to the host, jacobi_svd there,
// the maps back.  dX: 2 k^2 elements; dinfo needs 9 ints.  Returns rn or < 0.
static int tt_core_mode = 1;
static int core_and_products(int dtype, void* const Q[2], const int Nq[2], int k, double eps, int max_rank, char* Rs,
                             int* dinfo, void* dX, double* hbuf, void* Aout, int ldao, void* Bout, int ldbo,
                             hipStream_t st) {
  const size_t es = dtype == 1 ? 8 : 4;
  auto Rp = [&](int side, int pass) { return (void*)(Rs + es * (size_t)((side * 3 + pass) * 2) * k * k); };
  double* hR = hbuf;                 // [side][pass] k x k
  int* hinfo = (int*)(hbuf + 6 * k * k);
  double* hX = hbuf + 6 * k * k + 8;
  int rc, rn;
  if (k <= CORE_K && tt_core_mode != 0) {
    int* drn = dinfo + 8;
    if (dtype == 1)
      hipLaunchKernelGGL(tt_core_kernel<double>, dim3(1), dim3(256), 0, st, (const double*)Rs, dinfo, k, eps,
                         max_rank, (double*)dX, drn);
    else
      hipLaunchKernelGGL(tt_core_kernel<float>, dim3(1), dim3(256), 0, st, (const float*)Rs, dinfo, k, eps,
                         max_rank, (float*)dX, drn);
    if (hipGetLastError() != hipSuccess) return -25;
    if (hipMemcpyAsync(hinfo, drn, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) return -20;
    if (hipStreamSynchronize(st) != hipSuccess) return -21;
    rn = hinfo[0];
    if (rn <= 0) return rn;
  } else {
    for (int side = 0; side < 2; ++side)
      for (int pass = 0; pass < 3; ++pass)
        if (hipMemcpyAsync((char*)hR + es * (size_t)(side * 3 + pass) * k * k, Rp(side, pass), es * (size_t)k * k,
                           hipMemcpyDeviceToHost, st) != hipSuccess)
          return -20;
    if (hipMemcpyAsync(hinfo, dinfo, sizeof(int) * 6, hipMemcpyDeviceToHost, st) != hipSuccess) return -20;
    if (hipStreamSynchronize(st) != hipSuccess) return -21;
    for (int i = 0; i < 6; ++i)
      if (hinfo[i] != 0) return -24;
    if (dtype == 0) {
      const float* f = (const float*)hR;
      for (int i = 6 * k * k - 1; i >= 0; --i) hR[i] = (double)f[i];
    }
    // R = R3 R2 R1 per side, core C = Ra Rb^T
    std::vector<double> Rt[2], tmp(k * k), C(k * k), sig(k), W(k * k);
    for (int side = 0; side < 2; ++side) {
      Rt[side].assign(hR + (size_t)(side * 3) * k * k, hR + (size_t)(side * 3 + 1) * k * k);
      for (int pass = 1; pass < 3; ++pass) {
        const double* Rk = hR + (size_t)(side * 3 + pass) * k * k;
        for (int i = 0; i < k; ++i)
          for (int j = 0; j < k; ++j) {
            double acc = 0;
            for (int l = i; l < k; ++l) acc += Rk[i * k + l] * Rt[side][l * k + j];   // Rk upper triangular
            tmp[i * k + j] = acc;
          }
        Rt[side] = tmp;
      }
    }
    for (int i = 0; i < k; ++i)
      for (int j = 0; j < k; ++j) {
        double acc = 0;
        for (int l = 0; l < k; ++l) acc += Rt[0][i * k + l] * Rt[1][j * k + l];
        C[i * k + j] = acc;
      }
    jacobi_svd(k, k, C.data(), sig.data(), W.data());       // C = (U S) W^T, U S in C's columns
    std::vector<int> ord(k);
    for (int j = 0; j < k; ++j) ord[j] = j;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return sig[a] > sig[b]; });
    double tot = 0;
    for (int j = 0; j < k; ++j) tot += sig[j] * sig[j];
    rn = k;
    double tail = 0;
    for (int jj = k - 1; jj >= 1; --jj) {
      tail += sig[ord[jj]] * sig[ord[jj]];
      if (tail <= eps * eps * tot) rn = jj;
      else break;
    }
    if (max_rank > 0) rn = std::min(rn, max_rank);
    rn = std::max(rn, 1);
    if (!(tot > 0)) return -22;
    for (int i = 0; i < k; ++i)
      for (int jj = 0; jj < rn; ++jj) {
        const int j = ord[jj];
        hX[i * 2 * k + jj] = C[i * k + j];
        hX[i * 2 * k + rn + jj] = W[i * k + j];
      }
    if (dtype == 0) {
      float* f = (float*)hX;
      for (int i = 0; i < 2 * k * k; ++i) f[i] = (float)hX[i];
    }
    if (hipMemcpyAsync(dX, hX, es * 2 * k * k, hipMemcpyHostToDevice, st) != hipSuccess) return -23;
  }
  if ((rc = stsp_tt_mm(dtype, Q[0], k, dX, 2 * k, Aout, ldao, Nq[0], k, rn, 1.0, 0.0, st))) return rc;
  if ((rc = stsp_tt_mm(dtype, Q[1], k, (char*)dX + es * rn, 2 * k, Bout, ldbo, Nq[1], k, rn, 1.0, 0.0, st))) return rc;
  return rn;
}

int stsp_tt_set_core(int mode) {
  const int old = tt_core_mode;
  tt_core_mode = mode;
  return old;
}

int stsp_tt_lr_step3(int dtype, const void* A, int lda, const void* B, int ldb, int N, int r, int nsub, double c,
                     double ih2, int periodic, double eps, int max_rank, void* ws, double* hbuf, void* Aout,
                     void* Bout, int ldo, hipStream_t st) {
  if (N < 1 || r < 1 || nsub < 1 || nsub > 6) return -1;
  const int k = r << nsub;
  if (k > 64) return -1;
  const size_t es = dtype == 1 ? 8 : 4;
  char* w = (char*)ws;
  void* buf[2][2] = {{w, w + es * (size_t)N * k}, {w + es * 2 * (size_t)N * k, w + es * 3 * (size_t)N * k}};
  void* G = w + es * 4 * (size_t)N * k;
  void* part = (char*)G + es * 2 * (size_t)k * k;
  const int P = stsp_tt_gram_blocks(N);
  const int kp = (k + 15) / 16 * 16;
  void* dX = (char*)part + es * (size_t)P * kp * kp;
  char* Rs = (char*)dX + es * (size_t)2 * k * k;          // [side][pass][R, Ri] k x k
  int* dinfo = (int*)(Rs + es * (size_t)12 * k * k);       // [side][pass]
  int rc;
  const void* srcA = A;
  const void* srcB = B;
  int sa = lda, sb = ldb, rr = r, cur = 0;
  for (int s = 0; s < nsub; ++s, rr *= 2) {
    void* dA = buf[cur][0];
    void* dB = buf[cur][1];
    if ((rc = stsp_tt_expand(dtype, srcA, sa, dA, 2 * rr, N, rr, 1.0, 0.0, 0.0, c, ih2, periodic, st))) return rc;
    if ((rc = stsp_tt_expand(dtype, srcB, sb, dB, 2 * rr, N, rr, 1.0, c, 1.0, 0.0, ih2, periodic, st))) return rc;
    srcA = dA;
    srcB = dB;
    sa = sb = 2 * rr;
    cur ^= 1;
  }
  // CholeskyQR3 per factor: scratch = the free buffer and the expansion output
  // itself (no longer read after pass 1's Gram + product)
  const void* src[2] = {srcA, srcB};
  const int lds[2] = {k, k}, Nq[2] = {N, N};
  void* const s0[2] = {buf[cur][0], buf[cur][1]};
  void* const s1[2] = {(void*)srcA, (void*)srcB};
  if ((rc = cholqr3_pair(dtype, src, lds, Nq, k, s0, s1, part, G, Rs, dinfo, st))) return rc;
  void* Q[2] = {s0[0], s0[1]};
  return core_and_products(dtype, Q, Nq, k, eps, max_rank, Rs, dinfo, dX, hbuf, Aout, ldo, Bout, ldo, st);
}

// Rounding of one product A B^T (A [NA][k], B [NB][k], k <= 64) to the rank
// rn <= max_rank of relative accuracy eps, in one native call: CholeskyQR3 of
// both factors on the device (MFMA Gram + shifted Cholesky + MFMA product, x 3),
// the k x k core (device when k <= 32, else host), Aout = QA (U S)_rn,
// Bout = QB W_rn.  The inputs are not written.  The recompression that every
// operation of the six-panel factored SWE ends with (models/tt.py::
// CubedSphereLowRankShallowWater, backend "hip").  ws: stsp_tt_recompress_
// workspace elements; hbuf: 8 k^2 + 8 doubles (pinned).  Returns rn or < 0.
size_t stsp_tt_recompress_workspace(int NA, int NB, int k) {
  const int kp = (k + 15) / 16 * 16;
  return (size_t)2 * ((size_t)NA + NB) * k + (size_t)2 * k * k +
         (size_t)stsp_tt_gram_blocks(NA > NB ? NA : NB) * kp * kp + (size_t)2 * k * k + (size_t)12 * k * k + 16;
}

int stsp_tt_recompress(int dtype, const void* A, int lda, int NA, const void* B, int ldb, int NB, int k, double eps,
                       int max_rank, void* ws, double* hbuf, void* Aout, int ldao, void* Bout, int ldbo,
                       hipStream_t st) {
  if (NA < 1 || NB < 1 || k < 1 || k > 64 || lda < k || ldb < k) return -1;
  if (dtype != 0 && dtype != 1) return -4;
  const size_t es = dtype == 1 ? 8 : 4;
  const int kp = (k + 15) / 16 * 16;
  char* w = (char*)ws;
  void* sA[2] = {w, w + es * (size_t)NA * k};
  void* sB[2] = {w + es * 2 * (size_t)NA * k, w + es * (2 * (size_t)NA * k + (size_t)NB * k)};
  void* G = w + es * 2 * ((size_t)NA + NB) * k;
  void* part = (char*)G + es * (size_t)2 * k * k;
  void* dX = (char*)part + es * (size_t)stsp_tt_gram_blocks(NA > NB ? NA : NB) * kp * kp;
  char* Rs = (char*)dX + es * (size_t)2 * k * k;
  int* dinfo = (int*)(Rs + es * (size_t)12 * k * k);
  int rc;
  const void* X[2] = {A, B};
  const int ldx[2] = {lda, ldb}, Nq[2] = {NA, NB};
  void* const s0[2] = {sA[0], sB[0]};
  void* const s1[2] = {sA[1], sB[1]};
  if ((rc = cholqr3_pair(dtype, X, ldx, Nq, k, s0, s1, part, G, Rs, dinfo, st))) return rc;
  void* Q[2] = {sA[0], sB[0]};
  return core_and_products(dtype, Q, Nq, k, eps, max_rank, Rs, dinfo, dX, hbuf, Aout, ldao, Bout, ldbo, st);
}

int stsp_tt_lr_step(int dtype, const void* A, int lda, const void* B, int ldb, int N, int r, double c, double ih2,
                    int periodic, double eps, int max_rank, void* ws, double* hbuf, void* Aout, void* Bout, int ldo,
                    hipStream_t st) {
  return stsp_tt_lr_step2(dtype, A, lda, B, ldb, N, r, 1, c, ih2, periodic, eps, max_rank, ws, hbuf, Aout, Bout, ldo,
                          st);
}

}  // extern "C"
