// Fused SSP-RK step for the cubed-sphere shallow-water equations, gfx950.
//
// One launch = one whole time step (temporal blocking).  The launch-per-stage
// kernel (stage_kernel.hip) pays a dependent kernel boundary (~1.5 us) and a
// window round trip per RK stage; at C96 that is most of a 5 us stage.  Here a
// workgroup loads its 16 x 16 block plus a ring R = 2 NS cells wide once, then
// advances the ring through the earlier stages by redundant recompute (stage s
// updates the square [R - 2 (NS - s), W - R + 2 (NS - s)) of the W x W window),
// so no workgroup waits for another inside the step.  This is the
// MI355X-native counterpart of the reference's single composed compiled program
// (PY:238-246; PDF s.10 "Why two JITs?").
//
// Ring cells beyond a cube edge belong to another panel and are updated in
// that panel's frame (ops/fused.py explains the tables, all host-built):
//   * the window cell's region (P inside the block's panel; W, E, S, N across
//     one panel edge; none beyond a cube corner) comes from its panel
//     coordinates; a stencil neighbour in another region is replaced by the
//     ghost-strip value of (reader region, side, along position): the two
//     window cells and the weight of the Putman-Lin interpolation onto the
//     reader's grid line (models/base.py::reconstruct);
//   * faces that point into a cube corner's empty quadrant are the third cube
//     edge: a short list pairs each with its real partner cell;
//   * line normals per (region, window line) and face lengths per face are
//     per-block tables; cell records (1/A, centre, grad b) are gathered through
//     the padded layout.
// ops/fused.py::FusedTorch is the same algorithm in PyTorch; both are checked
// against the stage-by-stage oracle (tests/test_fused.py).
//
// Work split (1024 threads): thread t < W^2 owns window cell t for the whole
// step (its step-start and stage states stay in registers, primitives in LDS);
// face tasks (x-faces, then y-faces, then corner faces) are spread over all
// threads.  Per stage: faces -> barrier -> cell updates -> barrier.
#include "stage_common.h"


namespace {

template <int NS, int B>
struct FD {
  static constexpr int R = 2 * NS;
  static constexpr int W = B + 2 * R;
  static constexpr int WS = W + 1;                 // LDS row stride of the window
  static constexpr int WW = W * WS;                // LDS field stride
  static constexpr int L1 = R - 2 * (NS - 1);
  static constexpr int H1 = B + 4 * (NS - 1);
  static constexpr int NFX = H1 * (H1 + 1);
  static constexpr int NFL = 2 * NFX;
  static constexpr int NT = 1024;
  static constexpr int GMAX = 256;
  static constexpr int CMAX = 32;
};

// region of extended-panel coordinates: 0 P, 1 W, 2 E, 3 S, 4 N, -1 none
__device__ __forceinline__ int fregion(int X, int Y, int N) {
  const bool inx = (unsigned)X < (unsigned)N, iny = (unsigned)Y < (unsigned)N;
  if (inx) return iny ? 0 : (Y < 0 ? 3 : 4);
  return iny ? (X < 0 ? 1 : 2) : -1;
}

template <typename T>
struct FArgs {
  const T* Q;
  T* out;
  const T* cgeo;
  const int* src;
  const int* org;
  const T* len;
  const T* nrm;
  const short* gidx;
  const int* gtab;
  const T* gw;
  const int* ctab;
  const T* cgf;
  const int* ccnt;
  const int* push;
  int G, C, nblocks, n, N, S, mg, pw;
  T a0[4], a1[4], a2[4];
  T dt, g, omega2;
};

template <typename T, int LIM, int NS, int B>
__global__ __launch_bounds__(1024) void fused_step_kernel(FArgs<T> a) {
  using D = FD<NS, B>;
  constexpr int W = D::W, WS = D::WS, WW = D::WW, R = D::R, L1 = D::L1, H1 = D::H1;
  constexpr int NFX = D::NFX, NFL = D::NFL, NT = D::NT;
  __shared__ T s_w[5][W][WS];            // primitives h, vx, vy, vz and sound speed
  __shared__ T s_fl[4][NFL];             // face fluxes (stage-1 face set, compact)
  __shared__ T s_len[NFL];               // face lengths
  __shared__ T s_nrm[2][5][W + 1][3];    // line normals per region (oriented +u / +v)
  __shared__ short s_gi[20 * W];         // ghost entry per (strip, pos)
  __shared__ short s_gs[D::GMAX][2];     // interpolation pair (LDS window index)
  __shared__ T s_gt[D::GMAX];
  __shared__ int s_ct[D::CMAX][4];
  __shared__ T s_cg[D::CMAX][4];

  const int tid = threadIdx.x;
  const int bid = xcd_remap(blockIdx.x, a.nblocks);
  const int N = a.N;
  const int* og = a.org + bid * 4;
  const int X0 = og[0], Y0 = og[1], tile = og[2], ow = og[3];
  const int xo = ow & 0xFFF, yo = (ow >> 12) & 0xFFF, flags = (ow >> 24) & 0x1F;
  const bool edge = (flags & 0x1E) != 0;                 // a side region is present (block-uniform)
  const T* wf = &s_w[0][0][0];

  // ---- 0. prologue: tables -> LDS, window state + cell records -> registers ----
  const int u = tid % W, v = tid / W;
  const bool owner = tid < W * W;
  int src = -1;
  if (owner) src = a.src[(long)bid * W * W + tid];
  {
    const T* ln = a.len + (long)bid * NFL;
    for (int k = tid; k < NFL; k += NT) s_len[k] = ln[k];
    const T* nr = a.nrm + (long)bid * (2 * 5 * (W + 1) * 3);
    T* sn = &s_nrm[0][0][0][0];
    constexpr int NN = 2 * 5 * (W + 1) * 3;
    for (int k = tid; k < NN; k += NT) {
      const int r_ = (k / ((W + 1) * 3)) % 5;
      if (r_ == 0 || ((flags >> r_) & 1)) sn[k] = nr[k];
    }
    if (edge) {
      const short* gi = a.gidx + (long)bid * 20 * W;
      for (int k = tid; k < 20 * W; k += NT) s_gi[k] = gi[k];
      const int* gt = a.gtab + (long)bid * a.G * 2;
      const T* gw = a.gw + (long)bid * a.G;
      for (int k = tid; k < a.G; k += NT) {
        s_gs[k][0] = (short)gt[2 * k];
        s_gs[k][1] = (short)gt[2 * k + 1];
        s_gt[k] = gw[k];
      }
    }
  }
  const int ncor = edge ? a.ccnt[bid] : 0;
  if (tid < ncor) {
    const int* ct = a.ctab + ((long)bid * a.C + tid) * 8;
    const T* cg = a.cgf + ((long)bid * a.C + tid) * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) { s_ct[tid][k] = ct[k]; s_cg[tid][k] = cg[k]; }
  }
  // own window cell
  T X[4], Q[4];
  T iA = T(0), r0 = T(0), r1 = T(0), r2 = T(0), gb0 = T(0), gb1 = T(0), gb2 = T(0);
  const bool loaded = src >= 0;
  const bool in1 = (u >= L1) & (u < L1 + H1) & (v >= L1) & (v < L1 + H1);
  if (loaded) {
    const unsigned S = (unsigned)a.S;
#pragma unroll
    for (int f = 0; f < 4; ++f) Q[f] = *o32(a.Q, (unsigned)src + f * S);
    if (in1) {
      T rec[8];
      load_rec8<T>(o32(a.cgeo, (unsigned)src * 8u), rec);
      iA = rec[0]; r0 = rec[1]; r1 = rec[2]; r2 = rec[3];
      gb0 = rec[4]; gb1 = rec[5]; gb2 = rec[6];
    }
  } else {
#pragma unroll
    for (int f = 0; f < 4; ++f) Q[f] = T(0);
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) X[f] = Q[f];
  auto put = [&](const T (&q)[4]) {
    const T inv = q[0] != T(0) ? trcp(q[0]) : T(0);
    T* p = &s_w[0][v][u];
    p[0] = q[0];
    p[WW] = q[1] * inv;
    p[2 * WW] = q[2] * inv;
    p[3 * WW] = q[3] * inv;
    p[4 * WW] = tsqrt(a.g * tmax(q[0], T(0)));
  };
  if (owner) put(Q);
  __syncthreads();

  // ghost-strip value of field f for (strip, pos), or `dflt` when untabulated
  auto ghost = [&](int strip, int pos, int f, T dflt) -> T {
    const int e = s_gi[strip * W + pos];
    if (e < 0) return dflt;
    const T x0 = wf[f * WW + s_gs[e][0]], x1 = wf[f * WW + s_gs[e][1]];
    return x0 + s_gt[e] * (x1 - x0);
  };

#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int lo = R - 2 * (NS - 1 - s), hi = W - lo;
    const int nr = hi - lo, nl = nr + 1, nx = nr * nl;
    const int ntask = 2 * nx + ncor;
    // ---- faces ---------------------------------------------------------------
    for (int task = tid; task < ntask; task += NT) {
      if (task < 2 * nx) {
        const bool ax = task >= nx;                          // false: x-face, true: y-face
        const int t2 = ax ? task - nx : task;
        int fu, fv, k, fslot, st;
        if (!ax) {
          const int r = t2 / nl, c = t2 - r * nl;
          fv = lo + r; k = lo + c; fu = k;                   // b = (k, fv), a = (k - 1, fv)
          fslot = (fv - L1) * (H1 + 1) + (k - L1);
          st = 1;
        } else {
          const int r = t2 / nr, c = t2 - r * nr;
          k = lo + r; fu = lo + c; fv = k;                   // b = (fu, k), a = (fu, k - 1)
          fslot = NFX + (k - L1) * H1 + (fu - L1);
          st = WS;
        }
        const int ib = fv * WS + fu, ia = ib - st;
        int ra = 0, rb = 0, ram = 0, rbp = 0;
        if (edge) {
          const int X = X0 + fu, Y = Y0 + fv;
          const int dx = ax ? 0 : 1, dy = ax ? 1 : 0;
          rb = fregion(X, Y, N);
          ra = fregion(X - dx, Y - dy, N);
          ram = fregion(X - 2 * dx, Y - 2 * dy, N);
          rbp = fregion(X + dx, Y + dy, N);
        }
        if (ra >= 0 && rb >= 0) {
          const int pos = ax ? fu : fv;
          const int sm = ax ? 2 : 0;                         // side index of -axis; +axis = sm + 1
          T wl[4], wr[4], cl[5], cr[5];
#pragma unroll
          for (int f = 0; f < 5; ++f) { cl[f] = wf[f * WW + ia]; cr[f] = wf[f * WW + ib]; }
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            T am = wf[f * WW + ia - st], bp = wf[f * WW + ib + st];
            T ap = cr[f], bm = cl[f];
            if (edge) {
              if (ram != ra) am = ghost(ra * 4 + sm, pos, f, am);
              if (rb != ra) {
                ap = ghost(ra * 4 + sm + 1, pos, f, ap);
                bm = ghost(rb * 4 + sm, pos, f, bm);
              }
              if (rbp != rb) bp = ghost(rb * 4 + sm + 1, pos, f, bp);
            }
            wl[f] = cl[f] + half_slope<LIM>(cl[f] - am, ap - cl[f]);
            wr[f] = cr[f] - half_slope<LIM>(cr[f] - bm, bp - cr[f]);
          }
          const T* m = &s_nrm[ax ? 1 : 0][ra][k][0];
          T fl[4];
          swe_flux<T>(wl, wr, cl, cr, m[0], m[1], m[2], s_len[fslot], a.g, fl);
#pragma unroll
          for (int f = 0; f < 4; ++f) s_fl[f][fslot] = fl[f];
        }
      } else {
        // cube-corner face j: cell c's face on side_c meets cell d's face on side_d
        const int j = task - 2 * nx;
        const int ec = s_ct[j][0], ed = s_ct[j][1];
        T fv2[2][4], cc[2][5];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int e = q ? ed : ec;
          const int cu = e & 0xFF, cv = (e >> 8) & 0xFF, side = (e >> 16) & 3;
          const int axs = side >> 1, plus = side & 1;
          const int st = axs ? WS : 1;
          const int ic = cv * WS + cu;
          const int rc = fregion(X0 + cu, Y0 + cv, N);
          const int du = axs ? 0 : 1, dv = axs ? 1 : 0;
          const int rin = plus ? fregion(X0 + cu - du, Y0 + cv - dv, N) : fregion(X0 + cu + du, Y0 + cv + dv, N);
          const int pos = axs ? cu : cv;
#pragma unroll
          for (int f = 0; f < 5; ++f) cc[q][f] = wf[f * WW + ic];
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const T c0 = cc[q][f];
            const T across = ghost(rc * 4 + side, pos, f, c0);
            T inward = wf[f * WW + (plus ? ic - st : ic + st)];
            if (rin != rc) inward = ghost(rc * 4 + (side ^ 1), pos, f, inward);
            fv2[q][f] = plus ? c0 + half_slope<LIM>(c0 - inward, across - c0)
                             : c0 - half_slope<LIM>(c0 - across, inward - c0);
          }
        }
        T fl[4];
        swe_flux<T>(fv2[0], fv2[1], cc[0], cc[1], s_cg[j][0], s_cg[j][1], s_cg[j][2], s_cg[j][3], a.g, fl);
        const int fc = s_ct[j][2], fd = s_ct[j][3];
        const bool pc = ((ec >> 16) & 1) != 0, pd = ((ed >> 16) & 1) != 0;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          if (fc >= 0) s_fl[f][fc] = pc ? fl[f] : -fl[f];
          if (fd >= 0) s_fl[f][fd] = pd ? -fl[f] : fl[f];
        }
      }
    }
    __syncthreads();
    // ---- cell updates ------------------------------------------------------------
    const bool upd = loaded & (u >= lo) & (u < hi) & (v >= lo) & (v < hi);
    if (upd) {
      const int xw = (v - L1) * (H1 + 1) + (u - L1), xe = xw + 1;
      const int ys = NFX + (v - L1) * H1 + (u - L1), yn = ys + H1;
      T dq[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) dq[f] = -((s_fl[f][xe] - s_fl[f][xw]) + (s_fl[f][yn] - s_fl[f][ys])) * iA;
      int rc = 0, rw = 0, rs = 0;
      if (edge) {
        rc = fregion(X0 + u, Y0 + v, N);
        rw = fregion(X0 + u - 1, Y0 + v, N);
        rs = fregion(X0 + u, Y0 + v - 1, N);
        if (rw < 0) rw = rc;
        if (rs < 0) rs = rc;
      }
      const T Lw = s_len[xw], Le = s_len[xe], Ls = s_len[ys], Ln = s_len[yn];
      const T* mw = &s_nrm[0][rw][u][0];
      const T* me = &s_nrm[0][rc][u + 1][0];
      const T* ms = &s_nrm[1][rs][v][0];
      const T* mn = &s_nrm[1][rc][v + 1][0];
      const T h = Q[0];
      const T fcor = a.omega2 * r2;
      const T cor[3] = {r1 * Q[3] - r2 * Q[2], r2 * Q[1] - r0 * Q[3], r0 * Q[2] - r1 * Q[1]};
      const T pb = T(0.5) * a.g * h * h * iA, gh = a.g * h;
      const T gbv[3] = {gb0, gb1, gb2};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const T Sk = Le * me[k] - Lw * mw[k] + Ln * mn[k] - Ls * ms[k];
        dq[1 + k] += -fcor * cor[k] + pb * Sk - gh * gbv[k];
      }
      const T c0 = a.a0[s], c1 = a.a1[s], c2 = a.a2[s] * a.dt;
      T o[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        T base = c1 * Q[f];
        if (c0 != T(0)) base += c0 * X[f];
        o[f] = c2 * dq[f] + base;
      }
      const T dd = o[1] * r0 + o[2] * r1 + o[3] * r2;
      o[1] -= dd * r0; o[2] -= dd * r1; o[3] -= dd * r2;
#pragma unroll
      for (int f = 0; f < 4; ++f) Q[f] = o[f];
      if (s + 1 < NS) put(Q);
    }
    if (s + 1 < NS) __syncthreads();
  }

  // ---- 4. the block's cells -> output, plus same-rank ghost pushes -----------
  if (owner && (u >= R) & (u < R + B) & (v >= R) & (v < R + B)) {
    const unsigned S = (unsigned)a.S;
#pragma unroll
    for (int f = 0; f < 4; ++f) *o32(a.out, (unsigned)src + f * S) = Q[f];
    const int n = a.n, mg = a.mg;
    const int x = xo + u - R, y = yo + v - R;              // tile-local
    const int* pm = a.push + (long)tile * 4 * mg * n;
    int pt[4] = {-1, -1, -1, -1};
    if (x < mg) pt[0] = pm[(0 * mg + x) * n + y];
    if (x >= n - mg) pt[1] = pm[(1 * mg + (n - 1 - x)) * n + y];
    if (y < mg) pt[2] = pm[(2 * mg + y) * n + x];
    if (y >= n - mg) pt[3] = pm[(3 * mg + (n - 1 - y)) * n + x];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (pt[k] >= 0) {
#pragma unroll
        for (int f = 0; f < 4; ++f) *o32(a.out, (unsigned)pt[k] + f * S) = Q[f];
      }
    }
  }
}

template <typename T, int NS, int B>
int launch_fused(const FusedDesc* d, hipStream_t s) {
  using D = FD<NS, B>;
  if (d->G > D::GMAX || d->C > D::CMAX || d->nblocks <= 0) return -2;
  if (d->pw != d->n + 2 * d->mg || d->mg < 2 || d->n % B) return -3;
  FArgs<T> a;
  a.Q = (const T*)d->Q; a.out = (T*)d->out; a.cgeo = (const T*)d->cgeo; a.src = d->src; a.org = d->org;
  a.len = (const T*)d->len; a.nrm = (const T*)d->nrm; a.gidx = d->gidx; a.gtab = d->gtab; a.gw = (const T*)d->gw;
  a.ctab = d->ctab; a.cgf = (const T*)d->cgf; a.ccnt = d->ccnt; a.push = d->push;
  a.G = d->G; a.C = d->C; a.nblocks = d->nblocks; a.n = d->n; a.N = d->N; a.S = d->S; a.mg = d->mg; a.pw = d->pw;
  for (int k = 0; k < 4; ++k) {
    a.a0[k] = (T)d->a0[k]; a.a1[k] = (T)d->a1[k]; a.a2[k] = (T)d->a2[k];
  }
  a.dt = (T)d->dt; a.g = (T)d->g; a.omega2 = (T)d->omega2;
  const dim3 grid(d->nblocks), block(D::NT);
  switch (d->limiter) {
    case 0: hipLaunchKernelGGL((fused_step_kernel<T, 0, NS, B>), grid, block, 0, s, a); break;
    case 1: hipLaunchKernelGGL((fused_step_kernel<T, 1, NS, B>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((fused_step_kernel<T, 2, NS, B>), grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL((fused_step_kernel<T, 3, NS, B>), grid, block, 0, s, a); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int stsp_fused_launch(int dtype, const FusedDesc* d, hipStream_t stream) {
  if (d->B != 16 || d->ns != 3) return -1;
  if (dtype == 1) return launch_fused<double, 3, 16>(d, stream);
  if (dtype == 0) return launch_fused<float, 3, 16>(d, stream);
  return -5;
}

// Compile-time sizes of the fused kernel (host checks): ghost entries and corner faces per block.
extern "C" int stsp_fused_limits(int* gmax, int* cmax) {
  *gmax = FD<3, 16>::GMAX;
  *cmax = FD<3, 16>::CMAX;
  return 0;
}
