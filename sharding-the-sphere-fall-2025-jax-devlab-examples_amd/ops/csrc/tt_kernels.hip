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

}  // extern "C"
