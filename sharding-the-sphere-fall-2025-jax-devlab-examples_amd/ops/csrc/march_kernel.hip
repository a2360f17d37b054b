// Streaming ("march") RK stage of the shallow-water solver for large grids,
// gfx950 (CDNA4).
//
// The block stage kernel (stage_kernel.hip) is built for C96-class grids where
// every launch is latency-bound: one thread per edge, the window and the fluxes
// in LDS, two barriers.  On C360 / C720 that shape pays its index arithmetic,
// its LDS traffic and its barriers for every cell: the fp32 C720 stage was 85 %
// VALU-busy with only 31 % of the VALU instructions doing floating-point math
// (docs/ARCHITECTURE.md, profiles/r2_roofline).  Here one wave marches a strip
// of 60 columns up the tile, one row per iteration:
//
//   * lane l owns column x = 60 cs + l - 2 (lanes 0, 1, 62, 63 are the x-halo);
//     x-neighbours come from the adjacent lanes through DPP wave shifts
//     (v_mov_b32_dpp wave_shr / wave_shl: no LDS, no barrier);
//   * y-neighbours stay in registers: the march keeps rows j and j+1 as
//     primitives (h, v, sqrt(g h)), the half slope of row j and the flux through
//     the face below row j, and loads one new row per step (prefetched a row
//     ahead), so every face flux is evaluated exactly once;
//   * the waves of a workgroup are independent jobs (no LDS, no barrier), so a
//     CU holds as many marches as its VGPRs allow and hides their loads behind
//     each other's arithmetic;
//   * panel edges (models/base.py::reconstruct) are the same treatment as the
//     block kernel: the ghost strip used for slopes is interpolated along the
//     neighbour's grid lines, the neighbour's edge state is reconstructed in its
//     own frame, the wave speeds use the raw cells.  W/E strips are per-row
//     gathers in the edge waves, S/N strips per-lane gathers at the first and
//     last rows of the tile.
//
// Same inputs and outputs as one stage_kernel launch (StageDesc), same push map
// for the same-rank ghost strips; PLR limiters only (PPM keeps the block kernel).
// Several ranks (XG): the direct xGMI exchange of the block kernel, tagged
// granules (ops/xgmi.py): a ghost cell that belongs to another rank is read
// from this rank's receive ring (spin until its granules carry this stage's
// tag), and a cell that is another rank's ghost is stored into that rank's
// ring (push-map entries <= -2); each wave (job) keeps its own stage count.
// Compared with the fp64 PyTorch oracle in tests/test_march.py.
#include "march_common.h"

namespace {

constexpr int MO = MW - 4;      // output columns per wave

// panel-local components (e_i, e_j, n) -> Cartesian for a panel whose frame
// vectors are signed coordinate axes (frame code of ops/fused.py::frame_code)
template <typename T>
__device__ __forceinline__ void frame_to_global(int fr, T xi, T xj, T xn, T& o0, T& o1, T& o2) {
  const int ai = fr & 3, aj = (fr >> 2) & 3;
  if (fr & 64) xi = -xi;
  if (fr & 128) xj = -xj;
  if (fr & 256) xn = -xn;
  o0 = ai == 0 ? xi : (aj == 0 ? xj : xn);
  o1 = ai == 1 ? xi : (aj == 1 ? xj : xn);
  o2 = ai == 2 ? xi : (aj == 2 ? xj : xn);
}

// Waves per SIMD the register allocation must allow: fp32 fits 4 (<= 128
// VGPRs); fp64 needs ~225 VGPRs, 2 waves (asking for 3 spills to scratch).
#ifndef STSP_MARCH_WPE64
#define STSP_MARCH_WPE64 2
#endif
#ifndef STSP_MARCH_WPE32
#define STSP_MARCH_WPE32 4
#endif
// ACC: the RK4 accumulator operands (acc_in / acc_out); the SSP-RK3 and Euler
// stages run the instantiation without them (4 fewer live values per lane).
// CG: compact geometry: the panel-shared tables of the fused step (1/A,
// curvature sum and centre by panel-local index, rotated by the panel frame;
// edge lengths by panel-local index) instead of the per-tile records, and the
// topography gradient formed from b itself (104 instead of 176 B per fp64 cell
// through HBM; the shared tables are read by all six panels)
template <typename T, int LIM, int R, bool ACC, bool CG, bool XG>
__global__ __launch_bounds__(MW * MWPB) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 8 ? STSP_MARCH_WPE64 : STSP_MARCH_WPE32)))
void march_kernel(Args<T> a, int ncs, int nrs, int njobs) {
  pin_args(a);
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // job = (tile, column strip cs, row segment rs), rs fastest: the four waves of
  // a workgroup march stacked segments of one strip (their halo rows are each
  // other's rows), and consecutive workgroups share an XCD (xcd_remap)
  const int gw = xcd_remap(blockIdx.x, gridDim.x) * MWPB + wv;
  if (gw >= njobs) return;
  const int rs = gw % nrs, rest = gw / nrs;
  const int cs = rest % ncs, tile = rest / ncs;
  const int n = a.n, S = a.S, mg = a.mg, pw = a.pw;
  const int x = cs * MO + lane - 2;
  const int xc = x < n + 1 ? x : n + 1;            // lanes past the padded tile load column n + 1
  const bool outl = (lane >= 2) & (lane < MW - 2) & (x < n);
  const bool inx = (x >= 0) & (x < n);
  const int y0 = rs * R;
  const int y1 = y0 + R < n ? y0 + R : n;
  constexpr unsigned ES = sizeof(T);
  const unsigned tb = (unsigned)(tile * pw * pw);
  const __amdgpu_buffer_rsrc_t rQ = brsrc(a.Q), rX = brsrc(a.X), rO = brsrc(a.out),
                               rG = brsrc(CG ? (const T*)a.crec : a.cgeo);
  const unsigned fs = (unsigned)S * ES;              // field stride in bytes (soffset)
  const T g = a.g;

  auto cell = [&](int cx, int y) -> unsigned { return tb + (unsigned)((y + mg) * pw + (cx + mg)); };
  auto ldq = [&](unsigned pa, T (&q)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) q[f] = bld<T>(rQ, pa * ES, f * fs);
  };
  // XG: this job's stage count (tags), and the cell load that takes a remote
  // ghost from the receive ring
  int xe = 0;
  if constexpr (XG) xe = a.epoch[gw];
  auto ldc = [&](int cx, int y, T (&q)[4]) {
    if constexpr (XG) {
      const bool gx = (unsigned)cx >= (unsigned)n, gy = (unsigned)y >= (unsigned)n;
      if (gx || gy) {                              // an edge ghost, or a tile-corner ghost (carried ones may be remote)
        int m = 0;
        if (gx != gy) {
          const int side = gx ? (cx < 0 ? 0 : 1) : (y < 0 ? 2 : 3);
          const int layer = gx ? (cx < 0 ? -1 - cx : cx - n) : (y < 0 ? -1 - y : y - n);
          const int pos = gx ? y : cx;
          if (layer < mg) m = a.gmap[((tile * 4 + side) * mg + layer) * n + pos];
        } else if (a.cgmap) {
          const int ca = y < 0 ? -1 - y : y - n, cb = cx < 0 ? -1 - cx : cx - n;
          if (ca < mg && cb < mg) m = a.cgmap[((tile * 4 + (cx >= n ? 1 : 0) + (y >= n ? 2 : 0)) * mg + ca) * mg + cb];
        }
        if (m < 0) {                               // remote slot -1 - m: spin on its granules
          constexpr int G = sizeof(T) / 4;
          const gu64* rp = ((const gu64*)(a.recv)) + (long)(xe % STSP_XG_SLOTS) * a.ring;
          const int nrec = a.ring / (4 * G), rec = -1 - m;
          const unsigned want = (unsigned)xe + 1u;
          unsigned long long gr[4 * G];
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < 4 * G; ++k) {
              gr[k] = __hip_atomic_load(rp + ring_word(nrec, 4 * G, rec, k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              ok &= (unsigned)(gr[k] >> 32) == want;
            }
            if (ok) break;
            if (__hip_atomic_load((gu32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
            if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
              __hip_atomic_store((gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            if constexpr (G == 2)
              q[f] = __builtin_bit_cast(T, (gr[2 * f + 1] << 32) | (gr[2 * f] & 0xFFFFFFFFull));
            else
              q[f] = __builtin_bit_cast(T, (unsigned)gr[f]);
          }
          return;
        }
      }
    }
    ldq(cell(cx, y), q);
  };
  // primitive (h, v) + sound speed, as the block kernel's put()
  auto prim = [&](const T (&q)[4], T (&w)[5]) {
    const T inv = q[0] != T(0) ? trcp(q[0]) : T(0);
    w[0] = q[0];
    w[1] = q[1] * inv;
    w[2] = q[2] * inv;
    w[3] = q[3] * inv;
    w[4] = tsqrt(g * tmax(q[0], T(0)));
  };
  // linear interpolation between the primitives of two cells
  auto interp2 = [&](int x0_, int y0_, int x1_, int y1_, T t, T (&o)[4]) {
    T q0[4], q1[4], w0[5], w1[5];
    ldc(x0_, y0_, q0);
    ldc(x1_, y1_, q1);
    prim(q0, w0);
    prim(q1, w1);
#pragma unroll
    for (int f = 0; f < 4; ++f) o[f] = w0[f] + t * (w1[f] - w0[f]);
  };

  // ---- panel edges of this wave's part of the tile (wave-uniform) -------------
  const int pe = a.pedge[tile];
  const int lnE = n - cs * MO + 2;                   // lane of column n
  const bool peW = (pe & 1) && cs == 0;
  const bool peE = (pe & 2) && lnE >= 0 && lnE < MW;
  // a segment reads rows y0 - 2 .. y1 + 1: the S ghost row -1 when y0 <= 1 and
  // the N ghost row n when y1 >= n - 1 (a segment ending one row short of the
  // tile still takes the slope of row n - 1 across the panel edge)
  const bool peS = (pe & 4) && y0 <= 1;
  const bool peN = (pe & 8) && y1 >= n - 1;
  auto tab = [&](int side, int pos) -> unsigned { return (unsigned)(((tile * 4 + side) * 3 + 0) * n + pos); };
  // S / N strips (along x, per lane): interpolation of row y at this lane's table pair
  auto interp_row = [&](int side, int y, T (&o)[4]) {
    const unsigned ti = tab(side, inx ? x : 0);
    const int b = a.pe_base[ti];
    const T t = a.pe_t[ti];
    interp2(b, y, b + 1, y, t, o);
  };
  // W / E strips (along y, one table entry per row): every lane interpolates its
  // own column between rows b and b + 1
  auto interp_col = [&](int side, int j, T (&o)[4]) {
    const unsigned ti = tab(side, j);
    const int b = a.pe_base[ti];
    const T t = a.pe_t[ti];
    interp2(xc, b, xc, b + 1, t, o);
  };

  // the primitives a row offers to its y-neighbours' slopes: the raw cells,
  // except a panel-edge ghost row (interpolated)
  auto wsrow = [&](int y, const T (&c)[5], T (&ws)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) ws[f] = c[f];
    if ((peS && y == -1) || (peN && y == n)) {
      if (inx) {
        T o[4];
        interp_row(y < 0 ? 2 : 3, y, o);
#pragma unroll
        for (int f = 0; f < 4; ++f) ws[f] = o[f];
      }
    }
  };
  // the neighbour's state at a S / N panel-edge face, reconstructed in its own
  // frame from [our edge row interpolated at its grid line | its raw rows]
  auto nf_row = [&](int side, const T (&c)[5], const T (&r)[5], T (&nf)[4]) {
    T l[4];
    interp_row(side, side == 2 ? 0 : n - 1, l);
#pragma unroll
    for (int f = 0; f < 4; ++f) nf[f] = c[f] - half_slope<LIM>(c[f] - l[f], r[f] - c[f]);
  };

  // ---- per-lane constants ------------------------------------------------------
  const bool xe_ok = (x >= 0) & (x <= n);            // the lane's west face is a tile face
  T mxc[3], mxe[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    mxc[k] = xe_ok ? *o32(a.mx, (unsigned)((tile * 3 + k) * (n + 1) + x)) : T(0);
    mxe[k] = shl(mxc[k]);
  }
  const T* myt = a.my + (long)tile * 3 * (n + 1);
  const T* ext = a.ex + (long)tile * n * (n + 1);
  const T* eyt = a.ey + (long)tile * (n + 1) * n;
  const int* pm = a.push + (long)tile * 4 * mg * n;
  // compact geometry: panel-local cell (I0 + x, J0 + y) of this tile's face
  int I0 = 0, J0 = 0, fr = 0, Nf = n, Nf1 = n + 1;
  if constexpr (CG) {
    const int face = a.torg[3 * tile];
    I0 = a.torg[3 * tile + 1];
    J0 = a.torg[3 * tile + 2];
    fr = (int)(a.frames >> (9 * face)) & 511;
    Nf = a.Nf;
    Nf1 = a.Nf + 1;
  }
  const int xg = I0 + (inx ? x : 0);                  // panel column of the lane (clamped)
  const bool topo = CG && a.bpad != nullptr;
  const __amdgpu_buffer_rsrc_t rB = brsrc(topo ? a.bpad : a.Q);
  // edge lengths: x-face (j, x) and y-face (j', x) of this tile
  auto len_x = [&](int j) -> T { return CG ? a.lxt[(J0 + j) * Nf1 + I0 + x] : ext[(long)j * (n + 1) + x]; };
  auto len_y = [&](int jp) -> T { return CG ? a.lxt[xg * Nf1 + J0 + jp] : eyt[(long)jp * n + x]; };
  const bool need_x = (a.a0 != T(0)) || (ACC && a.c1 != T(0));
  const bool need_acc = ACC && a.acc_in && (a.c0 != T(0));

  // ---- prologue: rows y0-2 .. y0+1, the flux through the face below row y0 -----
  T cA[5], cB[5], hsA[4], Gs[4];
  T Ls;                                              // length of the face below row j
  {
    T q[4], cm2[5], cm1[5];
    ldc(xc, y0 - 2, q); prim(q, cm2);
    ldc(xc, y0 - 1, q); prim(q, cm1);
    ldc(xc, y0, q);     prim(q, cA);
    ldc(xc, y0 + 1, q); prim(q, cB);
    T wsm2[4], wsm1[4], ws0[4], ws1[4];
    wsrow(y0 - 2, cm2, wsm2);
    wsrow(y0 - 1, cm1, wsm1);
    wsrow(y0, cA, ws0);
    wsrow(y0 + 1, cB, ws1);
    T wl[4], wr[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      hsA[f] = half_slope<LIM>(cA[f] - wsm1[f], ws1[f] - cA[f]);
      wl[f] = cm1[f] + half_slope<LIM>(cm1[f] - wsm2[f], ws0[f] - cm1[f]);
      wr[f] = cA[f] - hsA[f];
    }
    if (peS && y0 == 0) nf_row(2, cm1, cm2, wl);     // the face below row 0 is a panel edge
    if (peN && y0 + 1 == n) { /* row y0 + 1 == n: its state enters only the loop's face */ }
    Ls = inx ? len_y(y0) : T(0);
    swe_flux<T>(wl, wr, cm1, cA, myt[0 * (n + 1) + y0], myt[1 * (n + 1) + y0], myt[2 * (n + 1) + y0], Ls, g, Gs);
  }
  T qn[4];                                           // raw row j + 2, loaded one step ahead
  ldc(xc, y0 + 2, qn);
  T bS = T(0), bA = T(0), bB = T(0), bn = T(0);       // topography of rows j - 1 .. j + 2 (CG)
  if (topo) {
    bS = bld<T>(rB, cell(xc, y0 - 1) * ES, 0);
    bA = bld<T>(rB, cell(xc, y0) * ES, 0);
    bB = bld<T>(rB, cell(xc, y0 + 1) * ES, 0);
    bn = bld<T>(rB, cell(xc, y0 + 2) * ES, 0);
  }

  for (int j = y0; j < y1; ++j) {
    T cC[5];
    prim(qn, cC);
    const T bC = bn;
    if (j + 1 < y1) {                                // prefetch (row j + 3 <= n + 1)
      ldc(xc, j + 3, qn);
      if (topo) bn = bld<T>(rB, cell(xc, j + 3) * ES, 0);
    }
    // own-row operands of row j (needed after the fluxes)
    const unsigned pc = cell(xc, j);
    T qo[4], xs[4], acs[ACC ? 4 : 1], rec[8];
    ldc(xc, j, qo);
#pragma unroll
    for (int f = 0; f < 4; ++f) xs[f] = T(0);
    if (need_x) {
#pragma unroll
      for (int f = 0; f < 4; ++f) xs[f] = bld<T>(rX, pc * ES, f * fs);
    }
    if constexpr (ACC) {
#pragma unroll
      for (int f = 0; f < 4; ++f) acs[f] = need_acc ? *o32(a.acc_in + f * S, pc) : T(0);
    }
    const unsigned gc = CG ? (unsigned)((J0 + j) * Nf + xg) : (unsigned)((tile * n + j) * n + (inx ? x : 0));
    bld_rec8<T>(rG, gc * 8u * ES, rec);
    const T Lw = xe_ok ? len_x(j) : T(0);
    const T Ln = inx ? len_y(j + 1) : T(0);
    const T my0 = myt[0 * (n + 1) + j + 1], my1 = myt[1 * (n + 1) + j + 1], my2 = myt[2 * (n + 1) + j + 1];
    const T ms0 = myt[0 * (n + 1) + j], ms1 = myt[1 * (n + 1) + j], ms2 = myt[2 * (n + 1) + j];

    // ---- y: slope of row j + 1, flux through the face above row j --------------
    T hsB[4], Gn[4];
    {
      T wsC[4];
      wsrow(j + 2, cC, wsC);
      T wl[4], wr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        hsB[f] = half_slope<LIM>(cB[f] - cA[f], wsC[f] - cB[f]);
        wl[f] = cA[f] + hsA[f];
        wr[f] = cB[f] - hsB[f];
      }
      if (peN && j + 1 == n) nf_row(3, cB, cC, wr);
      swe_flux<T>(wl, wr, cA, cB, my0, my1, my2, Ln, g, Gn);
    }

    // ---- x: faces of row j across the lanes ------------------------------------
    T Fw[4], Fe[4];
    {
      T ws[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) ws[f] = cA[f];
      T giW[4] = {T(0), T(0), T(0), T(0)}, giE[4] = {T(0), T(0), T(0), T(0)};
      if (peW) {
        if (x == -1 || x == 0) interp_col(0, j, giW);   // lane x = -1: the ghost; x = 0: own column 0
        if (x == -1) {
#pragma unroll
          for (int f = 0; f < 4; ++f) ws[f] = giW[f];
        }
      }
      if (peE) {
        if (x == n || x == n - 1) interp_col(1, j, giE);
        if (x == n) {
#pragma unroll
          for (int f = 0; f < 4; ++f) ws[f] = giE[f];
        }
      }
      T fP[4], fM[4], wm[4], wp[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        wm[f] = shr(ws[f]);
        wp[f] = shl(ws[f]);
        const T hs = half_slope<LIM>(cA[f] - wm[f], wp[f] - cA[f]);
        fP[f] = cA[f] + hs;
        fM[f] = cA[f] - hs;
      }
      if (peW) {
        T gp[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) gp[f] = shl(giW[f]);   // column 0 at the ghost's grid line
        if (x == -1) {
#pragma unroll
          for (int f = 0; f < 4; ++f) fP[f] = cA[f] - half_slope<LIM>(cA[f] - gp[f], wm[f] - cA[f]);
        }
      }
      if (peE) {
        T gp[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) gp[f] = shr(giE[f]);   // column n - 1
        if (x == n) {
#pragma unroll
          for (int f = 0; f < 4; ++f) fM[f] = cA[f] - half_slope<LIM>(cA[f] - gp[f], wp[f] - cA[f]);
        }
      }
      T wl[4], cl[5];
#pragma unroll
      for (int f = 0; f < 4; ++f) wl[f] = shr(fP[f]);
#pragma unroll
      for (int f = 0; f < 5; ++f) cl[f] = shr(cA[f]);
      swe_flux<T>(wl, fM, cl, cA, mxc[0], mxc[1], mxc[2], Lw, g, Fw);
#pragma unroll
      for (int f = 0; f < 4; ++f) Fe[f] = shl(Fw[f]);
    }
    const T Le = shl(Lw);
    const T bW = shr(bA), bE = shl(bA);               // (every lane: DPP reads the neighbours' registers)

    // ---- divergence, sources, RK combination, tangent projection, stores --------
    if (outl) {
      const T iA = rec[0];
      T r0 = rec[1], r1 = rec[2], r2 = rec[3], Sg[3] = {T(0), T(0), T(0)};
      if constexpr (CG) {
        frame_to_global(fr, rec[1], rec[2], rec[3], Sg[0], Sg[1], Sg[2]);   // curvature sum S = sum(L m)
        frame_to_global(fr, rec[4], rec[5], rec[6], r0, r1, r2);            // cell centre
      }
      T dq[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) dq[f] = -((Fe[f] - Fw[f]) + (Gn[f] - Gs[f])) * iA;
      const T fc = a.omega2 * r2;
      const T h = qo[0];
      const T cor[3] = {r1 * qo[3] - r2 * qo[2], r2 * qo[1] - r0 * qo[3], r0 * qo[2] - r1 * qo[1]};
      const T pb = T(0.5) * g * h * h * iA, gh = g * h;
      const T mn[3] = {my0, my1, my2}, ms[3] = {ms0, ms1, ms2};
      T gb[3] = {rec[4], rec[5], rec[6]};
      if constexpr (CG) {
        gb[0] = gb[1] = gb[2] = T(0);
        if (topo) {
          // grad b = (sum_e b_e L_e m_e - b S) / A with face averages b_e, projected
          // onto the tangent plane (models/base.py::fv_gradient)
          const T fE = T(0.5) * (bA + bE) * Le, fW = T(0.5) * (bW + bA) * Lw;
          const T fN = T(0.5) * (bA + bB) * Ln, fS = T(0.5) * (bS + bA) * Ls;
#pragma unroll
          for (int k = 0; k < 3; ++k)
            gb[k] = (((fE * mxe[k] - fW * mxc[k]) + (fN * mn[k] - fS * ms[k])) - bA * Sg[k]) * iA;
          const T d = gb[0] * r0 + gb[1] * r1 + gb[2] * r2;
          gb[0] -= d * r0; gb[1] -= d * r1; gb[2] -= d * r2;
        }
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const T Sk = CG ? Sg[k] : Le * mxe[k] - Lw * mxc[k] + Ln * mn[k] - Ls * ms[k];
        const T src = -fc * cor[k] + pb * Sk - gh * gb[k];
        dq[1 + k] += src;
      }
      T o[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        T base = T(0);
        if (a.a1 != T(0)) base = a.a1 * qo[f];
        if (a.a0 != T(0)) base += a.a0 * xs[f];
        o[f] = a.a2 * a.dt * dq[f] + base;
      }
      {
        const T d = o[1] * r0 + o[2] * r1 + o[3] * r2;
        o[1] -= d * r0; o[2] -= d * r1; o[3] -= d * r2;
      }
      if constexpr (ACC) {
        T p[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) p[f] = a.c2 * a.dt * dq[f];
        if (a.c1 != T(0)) {
#pragma unroll
          for (int f = 0; f < 4; ++f) p[f] += a.c1 * xs[f];
        }
        if (need_acc) {
#pragma unroll
          for (int f = 0; f < 4; ++f) p[f] += a.c0 * acs[f];
        }
        const T d = p[1] * r0 + p[2] * r1 + p[3] * r2;
        p[1] -= d * r0; p[2] -= d * r1; p[3] -= d * r2;
#pragma unroll
        for (int f = 0; f < 4; ++f) *o32(a.acc_out + f * S, pc) = p[f];
      }
#pragma unroll
      for (int f = 0; f < 4; ++f) bst<0>(o[f], rO, pc * ES, f * fs);
      // same-rank ghost pushes (push map, as the block kernel)
      int pt[4] = {-1, -1, -1, -1};
      if (x < mg) pt[0] = pm[(0 * mg + x) * n + j];
      if (x >= n - mg) pt[1] = pm[(1 * mg + (n - 1 - x)) * n + j];
      if (j < mg) pt[2] = pm[(2 * mg + j) * n + x];
      if (j >= n - mg) pt[3] = pm[(3 * mg + (n - 1 - j)) * n + x];
      if (a.cpush && (x < mg || x >= n - mg) && (j < mg || j >= n - mg)) {   // carried corner ghost (block kernel)
        const int qx = x < mg ? 0 : 1, qy = j < mg ? 0 : 1;
        const int v = a.cpush[((tile * 4 + (qx | (qy << 1))) * mg + (qy ? n - 1 - j : j)) * mg + (qx ? n - 1 - x : x)];
        if (v != -1) pt[qx ^ 1] = v;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (pt[k] >= 0) {
#pragma unroll
          for (int f = 0; f < 4; ++f) bst<0>(o[f], rO, (unsigned)pt[k] * ES, f * fs);
        } else if (XG && pt[k] <= -2) {
          // another rank's ghost: its ring slot (xe + 1) % SLOTS, tag xe + 2
          constexpr int G = sizeof(T) / 4;
          const int code = -2 - pt[k];
          gu64* dst = ((gu64*)(a.peer_ring[code >> 24])) + (long)((xe + 1) % STSP_XG_SLOTS) * a.ring;
          const int nrec = a.ring / (4 * G), rec = code & 0xFFFFFF;
          const unsigned long long tag = (unsigned long long)((unsigned)xe + 2u) << 32;
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            if constexpr (G == 2) {
              const unsigned long long bits = __builtin_bit_cast(unsigned long long, o[f]);
              __hip_atomic_store(dst + ring_word(nrec, 8, rec, 2 * f), tag | (bits & 0xFFFFFFFFull), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
              __hip_atomic_store(dst + ring_word(nrec, 8, rec, 2 * f + 1), tag | (bits >> 32), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
              __hip_atomic_store(dst + ring_word(nrec, 4, rec, f), tag | __builtin_bit_cast(unsigned, o[f]),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
        }
      }
    }
    // ---- advance the march -----------------------------------------------------
#pragma unroll
    for (int f = 0; f < 5; ++f) { cA[f] = cB[f]; cB[f] = cC[f]; }
#pragma unroll
    for (int f = 0; f < 4; ++f) { hsA[f] = hsB[f]; Gs[f] = Gn[f]; }
    Ls = Ln;
    bS = bA; bA = bB; bB = bC;
  }
  if constexpr (XG) {
    if (lane == 0) a.epoch[gw] = xe + 1;           // read again at the next stage's launch
  }
}

template <typename T, int LIM, int R>
int march_l(const StageDesc* d, hipStream_t s) {
  Args<T> a = make_args<T>(d);
  const int ncs = (d->n + MO - 1) / MO, nrs = (d->n + R - 1) / R;
  const int njobs = d->ntile * ncs * nrs;
  const int nb = (njobs + MWPB - 1) / MWPB;
  const bool cg = d->crec && d->lxt && d->torg;
  if (d->xg) {      // several ranks, direct xGMI exchange (SSP-RK3 / Euler stages, rows R = 4)
    if constexpr (R == 4) {
      if (d->acc_out) return -13;
      if (cg) hipLaunchKernelGGL((march_kernel<T, LIM, R, false, true, true>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
      else hipLaunchKernelGGL((march_kernel<T, LIM, R, false, false, true>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
      return (int)hipGetLastError();
    }
    return -13;
  }
  if (d->acc_out) {
    if (cg) hipLaunchKernelGGL((march_kernel<T, LIM, R, true, true, false>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
    else hipLaunchKernelGGL((march_kernel<T, LIM, R, true, false, false>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
  } else {
    if (cg) hipLaunchKernelGGL((march_kernel<T, LIM, R, false, true, false>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
    else hipLaunchKernelGGL((march_kernel<T, LIM, R, false, false, false>), dim3(nb), dim3(MW * MWPB), 0, s, a, ncs, nrs, njobs);
  }
  return (int)hipGetLastError();
}

template <typename T, int R>
int march_r(const StageDesc* d, hipStream_t s) {
  switch (d->limiter) {
    case 0: return march_l<T, 0, R>(d, s);
    case 1: return march_l<T, 1, R>(d, s);
    case 2: return march_l<T, 2, R>(d, s);
    case 3: return march_l<T, 3, R>(d, s);
  }
  return -11;      // PPM: the block kernel
}

template <typename T>
int march_t(int rows, const StageDesc* d, hipStream_t s) {
  switch (rows) {
    case 4: return march_r<T, 4>(d, s);
    case 8: return march_r<T, 8>(d, s);
    case 16: return march_r<T, 16>(d, s);
    case 32: return march_r<T, 32>(d, s);
  }
  return -2;
}

// DPP lane-shift probe (tests/test_march.py): out[0][i] = lane i-1's value,
// out[1][i] = lane i+1's, for one wave of doubles and one of floats
__global__ void dpp_probe_kernel(const double* in, double* out, float* outf) {
  const int i = threadIdx.x;
  out[i] = shr(in[i]);
  out[64 + i] = shl(in[i]);
  outf[i] = shr((float)in[i]);
  outf[64 + i] = shl((float)in[i]);
}

}  // namespace

// Rows per wave `rows` (4, 8, 16, 32).  Shallow water, PLR; remote ghosts only
// through the direct xGMI exchange with tagged granules (d->xg, rows 4; the
// epoch array has one count per job), never through a receive buffer or a
// block list.
extern "C" int stsp_march_launch(int dtype, int rows, const StageDesc* d, hipStream_t stream) {
  if (d->remote || d->blocks) return -13;
  if (d->xg && (!STSP_XG_TAG || !d->recv || !d->peer_ring || !d->epoch || !d->err || !d->gmap || d->ring <= 0))
    return -13;
  if (d->pw != d->n + 2 * d->mg || d->mg < 2 || d->n < 2) return -5;
  if (!d->pedge || !d->pe_base || !d->pe_t || !d->push || !d->mx || !d->my) return -12;
  const bool cg = d->crec && d->lxt && d->torg;
  if (cg ? d->Nf < d->n : (!d->cgeo || !d->ex || !d->ey)) return -12;
  if (dtype == 1) return march_t<double>(rows, d, stream);
  if (dtype == 0) return march_t<float>(rows, d, stream);
  return -4;
}

extern "C" int stsp_dpp_probe(const double* in, double* out, float* outf, hipStream_t stream) {
  hipLaunchKernelGGL(dpp_probe_kernel, dim3(1), dim3(64), 0, stream, in, out, outf);
  return (int)hipGetLastError();
}
