// Pipelined streaming SSP-RK3 step of the shallow-water solver for large
// grids, gfx950 (CDNA4).
//
// The streaming stage (march_kernel.hip) is one launch per RK stage, so a step
// reads and writes the state three times (C720 fp64: ~440 MB per stage at
// ~3.1 TB/s, profiles/r4_pmc).  Here ONE launch per step marches all three
// SSP-RK3 stages up a strip of a tile together:
//
//   * a wave owns 64 lanes = columns 52 cs - 2 .. 52 cs + 61 of the tile.
//     Stage 1 is valid on lanes 2..61, stage 2 on 4..59, stage 3 on 6..57:
//     each stage loses the two columns its PLR stencil reaches, so 52 columns
//     per wave come out of stage 3.  x-neighbours come through DPP lane shifts;
//   * per iteration the wave loads one new row of the step input (row j + 2,
//     prefetched a row ahead); stage 1 produces row j, stage 2 consumes it as
//     its own new row and produces row j - 2, and stage 3 consumes that and
//     produces row j - 4.  Each stage keeps its own rolling rows (primitives of
//     two rows, the half slope of the lower one, the flux below it) in
//     registers, so every face flux of every stage is evaluated once per strip;
//   * the conserved stage results that the next stage needs at its own row two
//     iterations later wait in a 3-row LDS ring per wave (no other wave reads
//     it: no barrier);
//   * a segment of R stage-3 rows starts stage 1 four rows lower and ends it
//     four rows higher: (3 R + 12) row steps per 3 R, and the step input is read
//     once (R + 12 rows per R), where the streaming stage reads R + 4 rows per R
//     rows in every one of three launches.
//
// Tile edges.  Stage 1 needs only the step input, whose ghost ring the
// previous step pushed: it runs everywhere in the tile, with the streaming
// stage's panel-edge treatment (models/base.py::reconstruct).  Stages 2 and 3
// of the cells within 2 / 4 of a tile edge would need the neighbouring tiles'
// stage results: they are NOT computed here.  The march stores its stage-1 and
// stage-2 results within D of a tile edge into q1 / q2 (stage 1 also pushes its
// same-rank ghost copies into q1), and two launches of the block stage kernel
// over the blocks along the tile edges finish stages 2 and 3 there
// (ops/march3.py).  So stages 2 and 3 of the march never see a ghost cell or a
// panel edge: they run the plain interior body.
//
// Same state layout, geometry (per-tile records cgeo / ex / ey / mx / my) and
// arithmetic as the streaming stage; compared with the fp64 PyTorch oracle in
// tests/test_march3.py.
#include "march_common.h"

namespace {

constexpr int M3O = MW - 12;    // stage-3 columns per wave

// Waves per SIMD the register allocation must allow.  The per-wave LDS rings
// (fp64 104 KB per 4-wave workgroup) allow one workgroup per CU in fp64, two in
// fp32; asking for more only spills (profiles/r6_march3).
#ifndef STSP_M3_WPE64
#define STSP_M3_WPE64 1
#endif
#ifndef STSP_M3_WPE32
#define STSP_M3_WPE32 2
#endif

template <typename T>
struct P3 {
  T* q1;
  T* q2;
  int D, ncs, nrs, njobs;
};

// SSP-RK3 (models/integrators.py::ssp_rk3): stage s computes
// b0 X + b1 Q + b2 dt L(Q).  Compile-time constants, the same values the stage
// kernel receives as (T) of the host doubles (the host checks the integrator).
template <typename T, int S> struct RK3;
template <typename T> struct RK3<T, 1> { static constexpr T b0 = T(0.0), b1 = T(1.0), b2 = T(1.0); };
template <typename T> struct RK3<T, 2> { static constexpr T b0 = T(0.75), b1 = T(0.25), b2 = T(0.25); };
template <typename T> struct RK3<T, 3> { static constexpr T b0 = T(1.0 / 3.0), b1 = T(2.0 / 3.0), b2 = T(2.0 / 3.0); };

// rolling rows of one interior march stage: primitives (h, v, sqrt(g h)) of
// rows j and j + 1, the half slope of row j, the flux through the face below j
template <typename T>
struct MRows {
  T cA[5], cB[5], hsA[4], Gs[4];
};

template <typename T>
__device__ __forceinline__ void prim5(const T (&q)[4], T g, T (&w)[5]) {
  const T inv = q[0] != T(0) ? trcp(q[0]) : T(0);
  w[0] = q[0];
  w[1] = q[1] * inv;
  w[2] = q[2] * inv;
  w[3] = q[3] * inv;
  w[4] = tsqrt(g * tmax(q[0], T(0)));
}

// interior x-faces of row c: flux through every lane's west face, and (one
// lane shift) through its east face
template <typename T, int LIM>
__device__ __forceinline__ void xfaces(const T (&c)[5], const T (&mxc)[3], T Lw, T g, T (&Fw)[4], T (&Fe)[4]) {
  T fP[4], fM[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const T wm = shr(c[f]), wp = shl(c[f]);
    const T hs = half_slope<LIM>(c[f] - wm, wp - c[f]);
    fP[f] = c[f] + hs;
    fM[f] = c[f] - hs;
  }
  T wl[4], cl[5];
#pragma unroll
  for (int f = 0; f < 4; ++f) wl[f] = shr(fP[f]);
#pragma unroll
  for (int f = 0; f < 5; ++f) cl[f] = shr(c[f]);
  swe_flux<T>(wl, fM, cl, c, mxc[0], mxc[1], mxc[2], Lw, g, Fw);
#pragma unroll
  for (int f = 0; f < 4; ++f) Fe[f] = shl(Fw[f]);
}

// divergence, sources, RK combination and tangent projection of one cell, as
// the streaming stage (rec = 1/A, centre xyz, grad b xyz, 0)
template <typename T, int STG>
__device__ __forceinline__ void update_cell(const T (&Fw)[4], const T (&Fe)[4], const T (&Gs)[4], const T (&Gn)[4],
                                            const T (&rec)[8], const T (&qo)[4], const T (&xs)[4], const T (&mxc)[3],
                                            const T (&mxe)[3], const T (&mn)[3], const T (&ms)[3], T Lw, T Le, T Ln,
                                            T Ls, T g, T omega2, T dt, T (&o)[4]) {
  constexpr T c0 = RK3<T, STG>::b0, c1 = RK3<T, STG>::b1, c2 = RK3<T, STG>::b2;
  const T iA = rec[0];
  const T r0 = rec[1], r1 = rec[2], r2 = rec[3];
  T dq[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) dq[f] = -((Fe[f] - Fw[f]) + (Gn[f] - Gs[f])) * iA;
  const T fc = omega2 * r2;
  const T h = qo[0];
  const T cor[3] = {r1 * qo[3] - r2 * qo[2], r2 * qo[1] - r0 * qo[3], r0 * qo[2] - r1 * qo[1]};
  const T pb = T(0.5) * g * h * h * iA, gh = g * h;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T Sk = Le * mxe[k] - Lw * mxc[k] + Ln * mn[k] - Ls * ms[k];
    const T src = -fc * cor[k] + pb * Sk - gh * rec[4 + k];
    dq[1 + k] += src;
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    T base = T(0);
    if constexpr (c1 != T(0)) base = c1 * qo[f];
    if constexpr (c0 != T(0)) base += c0 * xs[f];
    o[f] = c2 * dt * dq[f] + base;
  }
  const T d = o[1] * r0 + o[2] * r1 + o[3] * r2;
  o[1] -= d * r0; o[2] -= d * r1; o[3] -= d * r2;
}

// geometry of one output row of one stage, loaded an iteration ahead
template <typename T>
struct RowGeo {
  T rec[8];     // 1/A, centre xyz, grad b xyz, 0
  T Lw, Ln, Ls; // west face of the lane's cell, faces above and below it
};

template <typename T, int LIM, int R>
__global__ __launch_bounds__(MW * MWPB) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 8 ? STSP_M3_WPE64 : STSP_M3_WPE32)))
void march3_kernel(Args<T> a, P3<T> m) {
  // (no pin_args: a long-running march needs few of the arguments, and pinned
  // SGPRs spilled into VGPR lanes inside the loop)
  // per wave: the stage-1 and stage-2 results [row % 3], and the raw step
  // input rows j - 4 .. j + 2 [row % 7] (stage 1's own cell, the RK base of
  // stages 2 and 3): read once from memory, never again
  __shared__ T ring[MWPB][2][3][4][MW];
  __shared__ T qring[MWPB][7][4][MW];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // job = (tile, strip cs, segment rs), rs fastest: the four waves of a
  // workgroup march stacked segments of one strip (shared input rows in L2)
  const int gw = xcd_remap(blockIdx.x, gridDim.x) * MWPB + wv;
  if (gw >= m.njobs) return;
  const int rs = gw % m.nrs, rest = gw / m.nrs;
  const int cs = rest % m.ncs, tile = rest / m.ncs;
  const int n = a.n, S = a.S, mg = a.mg, pw = a.pw;
  const int x = cs * M3O + lane - 2;
  const int xc = x < n + 1 ? x : n + 1;            // lanes past the padded tile load column n + 1
  const bool inx = (x >= 0) & (x < n);
  const int xr = x < 0 ? 0 : (x > n - 1 ? n - 1 : x);   // clamped cell / edge indices (lanes outside
  const int xe = x < 0 ? 0 : (x > n ? n : x);           // the tile compute values nobody stores)
  const int ys = 4 + rs * R;                        // stage-3 rows [ys, ye)
  const int ye = ys + R < n - 4 ? ys + R : n - 4;
  const int y0 = ys - 4, y1 = ye + 4;               // stage-1 rows [y0, y1)
  constexpr unsigned ES = sizeof(T);
  const unsigned tb = (unsigned)(tile * pw * pw);
  const __amdgpu_buffer_rsrc_t rQ = brsrc(a.Q), rO = brsrc(a.out), r1 = brsrc(m.q1), r2 = brsrc(m.q2),
                               rG = brsrc(a.cgeo), rEX = brsrc(a.ex), rEY = brsrc(a.ey);
  const unsigned fs = (unsigned)S * ES;              // field stride in bytes (soffset)
  const T g = a.g;
  // cells this wave stores: columns [olo, ohi) (strips partition the tile),
  // rows [rlo, rhi) (segments partition it); the band of stage-1 / stage-2
  // results within D of a tile edge
  const int olo = cs == 0 ? 0 : cs * M3O + 4;
  const int ohi = cs == m.ncs - 1 ? n : cs * M3O + 4 + M3O;
  const bool own = (x >= olo) & (x < ohi);
  const int rlo = rs == 0 ? 0 : ys, rhi = rs == m.nrs - 1 ? n : ye;
  const bool xband = (x < m.D) | (x >= n - m.D);
  auto yband = [&](int y) -> bool { return (y < m.D) | (y >= n - m.D); };

  auto cell = [&](int cx, int y) -> unsigned { return tb + (unsigned)((y + mg) * pw + (cx + mg)); };
  auto ldq = [&](int cx, int y, T (&q)[4]) {
    const unsigned pa = cell(cx, y);
#pragma unroll
    for (int f = 0; f < 4; ++f) q[f] = bld<T>(rQ, pa * ES, f * fs);
  };
  auto prim = [&](const T (&q)[4], T (&w)[5]) { prim5(q, g, w); };
  auto interp2 = [&](int x0_, int y0_, int x1_, int y1_, T t, T (&o)[4]) {
    T q0[4], q1[4], w0[5], w1[5];
    ldq(x0_, y0_, q0);
    ldq(x1_, y1_, q1);
    prim(q0, w0);
    prim(q1, w1);
#pragma unroll
    for (int f = 0; f < 4; ++f) o[f] = w0[f] + t * (w1[f] - w0[f]);
  };

  // ---- panel edges met by stage 1 (wave-uniform), as the streaming stage -----
  const int pe = a.pedge[tile];
  const int lnE = n - cs * M3O + 2;                  // lane of column n
  const bool peW = (pe & 1) && cs == 0;
  const bool peE = (pe & 2) && lnE >= 0 && lnE < MW;
  const bool peS = (pe & 4) && y0 <= 1;
  const bool peN = (pe & 8) && y1 >= n - 1;
  auto tab = [&](int side, int pos) -> unsigned { return (unsigned)(((tile * 4 + side) * 3 + 0) * n + pos); };
  auto interp_row = [&](int side, int y, T (&o)[4]) {
    const unsigned ti = tab(side, inx ? x : 0);
    const int b = a.pe_base[ti];
    const T t = a.pe_t[ti];
    interp2(b, y, b + 1, y, t, o);
  };
  auto interp_col = [&](int side, int j, T (&o)[4]) {
    const unsigned ti = tab(side, j);
    const int b = a.pe_base[ti];
    const T t = a.pe_t[ti];
    interp2(xc, b, xc, b + 1, t, o);
  };
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
  auto nf_row = [&](int side, const T (&c)[5], const T (&r)[5], T (&nf)[4]) {
    T l[4];
    interp_row(side, side == 2 ? 0 : n - 1, l);
#pragma unroll
    for (int f = 0; f < 4; ++f) nf[f] = c[f] - half_slope<LIM>(c[f] - l[f], r[f] - c[f]);
  };

  // ---- per-lane geometry --------------------------------------------------------
  T mxc[3], mxe[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    mxc[k] = *o32(a.mx, (unsigned)((tile * 3 + k) * (n + 1) + xe));
    mxe[k] = shl(mxc[k]);
  }
  const T* myt = a.my + (long)tile * 3 * (n + 1);
  const int* pm = a.push + (long)tile * 4 * mg * n;
  // row geometry by 32-bit buffer offsets (rows outside the tile clamp: they
  // are loaded only ahead of pipeline steps that do not use them)
  auto ld_geo = [&](int j, RowGeo<T>& G) {
    const int jc = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
    bld_rec8<T>(rG, (unsigned)((tile * n + jc) * n + xr) * 8u * ES, G.rec);
    G.Lw = bld<T>(rEX, (unsigned)((tile * n + jc) * (n + 1) + xe) * ES, 0);
    G.Ln = bld<T>(rEY, (unsigned)((tile * (n + 1) + jc + 1) * n + xr) * ES, 0);
    G.Ls = bld<T>(rEY, (unsigned)((tile * (n + 1) + jc) * n + xr) * ES, 0);
  };
  T* rg = &ring[wv][0][0][0][0];
  T* qg = &qring[wv][0][0][0];
  auto ring_st = [&](int which, int y, const T (&v)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) rg[((which * 3 + y % 3) * 4 + f) * MW + lane] = v[f];
  };
  auto ring_ld = [&](int which, int y, T (&v)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] = rg[((which * 3 + y % 3) * 4 + f) * MW + lane];
  };
  auto qring_st = [&](int y, const T (&v)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) qg[((y % 7) * 4 + f) * MW + lane] = v[f];
  };
  auto qring_ld = [&](int y, T (&v)[4]) {
#pragma unroll
    for (int f = 0; f < 4; ++f) v[f] = qg[((y % 7) * 4 + f) * MW + lane];
  };
  auto mrow = [&](int jp, T (&v)[3]) {               // face-line normals of y-face jp (clamped)
    const int jc = jp < 0 ? 0 : (jp > n ? n : jp);
#pragma unroll
    for (int k = 0; k < 3; ++k) v[k] = myt[k * (n + 1) + jc];
  };

  // one consumed row r of interior stage STG (2 or 3): slope of row r - 1, flux
  // through the face below it (k = rows consumed before r), then, from the
  // fifth row on, the update of row r - 2 into o (returns true when it did).
  // G: geometry of row r - 2 (its Ln is the face r - 1); mn / ms: normals of
  // the faces above / below row r - 2
  auto stage_row = [&](auto stg, MRows<T>& st, const T (&C)[5], int r, int k, const RowGeo<T>& G,
                       const T (&mn)[3], const T (&ms)[3], T (&o)[4]) -> bool {
    constexpr int STG = decltype(stg)::value;
    T hsB[4], Gn[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
    for (int f = 0; f < 4; ++f) hsB[f] = half_slope<LIM>(st.cB[f] - st.cA[f], C[f] - st.cB[f]);
    if (k >= 3) {
      T wl[4], wr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        wl[f] = st.cA[f] + st.hsA[f];
        wr[f] = st.cB[f] - hsB[f];
      }
      swe_flux<T>(wl, wr, st.cA, st.cB, mn[0], mn[1], mn[2], G.Ln, g, Gn);
    }
    bool out = false;
    if (k >= 4) {
      const int j = r - 2;
      T xs[4], qo[4];
      qring_ld(j, xs);
      ring_ld(STG - 2, j, qo);
      T Fw[4], Fe[4];
      xfaces<T, LIM>(st.cA, mxc, G.Lw, g, Fw, Fe);
      const T Le = shl(G.Lw);
      update_cell<T, STG>(Fw, Fe, st.Gs, Gn, G.rec, qo, xs, mxc, mxe, mn, ms, G.Lw, Le, G.Ln, G.Ls, g, a.omega2,
                          a.dt, o);
      out = true;
    }
#pragma unroll
    for (int f = 0; f < 5; ++f) { st.cA[f] = st.cB[f]; st.cB[f] = C[f]; }
#pragma unroll
    for (int f = 0; f < 4; ++f) { st.hsA[f] = hsB[f]; st.Gs[f] = Gn[f]; }
    return out;
  };

  MRows<T> st2, st3;
#pragma unroll
  for (int f = 0; f < 5; ++f) st2.cA[f] = st2.cB[f] = st3.cA[f] = st3.cB[f] = T(0);
#pragma unroll
  for (int f = 0; f < 4; ++f) st2.hsA[f] = st2.Gs[f] = st3.hsA[f] = st3.Gs[f] = T(0);
  // geometry of each stage's row in the first iteration; afterwards each
  // stage loads its next row's geometry right after using the current one
  RowGeo<T> G1, G2, G3;
  ld_geo(y0, G1);
  ld_geo(y0 - 2, G2);
  ld_geo(y0 - 4, G3);

  // ---- stage 1 prologue: rows y0-2 .. y0+1, the flux through the face below y0
  T cA[5], cB[5], hsA[4], Gs[4];
  {
    T q[4], cm2[5], cm1[5];
    ldq(xc, y0 - 2, q); prim(q, cm2);
    ldq(xc, y0 - 1, q); prim(q, cm1);
    ldq(xc, y0, q);     prim(q, cA); qring_st(y0, q);
    ldq(xc, y0 + 1, q); prim(q, cB); qring_st(y0 + 1, q);
    T wsm2[4], wsm1[4], ws0[4], ws1[4];
    wsrow(y0 - 2, cm2, wsm2);
    wsrow(y0 - 1, cm1, wsm1);
    wsrow(y0, cA, ws0);
    wsrow(y0 + 1, cB, ws1);
    T wl[4], wr[4], mf[3];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      hsA[f] = half_slope<LIM>(cA[f] - wsm1[f], ws1[f] - cA[f]);
      wl[f] = cm1[f] + half_slope<LIM>(cm1[f] - wsm2[f], ws0[f] - cm1[f]);
      wr[f] = cA[f] - hsA[f];
    }
    if (peS && y0 == 0) nf_row(2, cm1, cm2, wl);     // the face below row 0 is a panel edge
    mrow(y0, mf);
    swe_flux<T>(wl, wr, cm1, cA, mf[0], mf[1], mf[2], G1.Ls, g, Gs);
  }
  // normals of the face below each stage's row (the face above it is the next
  // row's face below: one load of three values per stage and row)
  T ms1[3], ms2[3], ms3[3];
  mrow(y0, ms1);
  mrow(y0 - 2, ms2);
  mrow(y0 - 4, ms3);
  T qn[4];                                           // raw row j + 2, loaded one step ahead
  ldq(xc, y0 + 2, qn);

  for (int j = y0; j < y1; ++j) {
    T cC[5];
    prim(qn, cC);
    qring_st(j + 2, qn);
    if (j + 1 < y1) ldq(xc, j + 3, qn);              // prefetch (row j + 3 <= n + 1)
    T qo[4], mn[3];
    qring_ld(j, qo);
    mrow(j + 1, mn);

    // ---- stage 1, y: slope of row j + 1, flux through the face above row j ---
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
      swe_flux<T>(wl, wr, cA, cB, mn[0], mn[1], mn[2], G1.Ln, g, Gn);
    }

    // ---- stage 1, x: faces of row j across the lanes (panel edges W / E) -------
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
      swe_flux<T>(wl, fM, cl, cA, mxc[0], mxc[1], mxc[2], G1.Lw, g, Fw);
#pragma unroll
      for (int f = 0; f < 4; ++f) Fe[f] = shl(Fw[f]);
    }

    // ---- stage 1 update of row j (every lane; valid on lanes 2..61) ------------
    T o1[4];
    {
      const T xz[4] = {T(0), T(0), T(0), T(0)};
      const T Le = shl(G1.Lw);
      update_cell<T, 1>(Fw, Fe, Gs, Gn, G1.rec, qo, xz, mxc, mxe, mn, ms1, G1.Lw, Le, G1.Ln, G1.Ls, g, a.omega2,
                        a.dt, o1);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) ms1[k] = mn[k];
    ld_geo(j + 1, G1);                               // stage 1's next row, an iteration ahead
    ring_st(0, j, o1);
    if (own & (j >= rlo) & (j < rhi)) {
      const unsigned pc = cell(x, j);
      if (xband | yband(j)) {
#pragma unroll
        for (int f = 0; f < 4; ++f) bst<0>(o1[f], r1, pc * ES, f * fs);
      }
      // same-rank ghost copies of the stage-1 result (push map, as the stage kernels)
      int pt[4] = {-1, -1, -1, -1};
      if (x < mg) pt[0] = pm[(0 * mg + x) * n + j];
      if (x >= n - mg) pt[1] = pm[(1 * mg + (n - 1 - x)) * n + j];
      if (j < mg) pt[2] = pm[(2 * mg + j) * n + x];
      if (j >= n - mg) pt[3] = pm[(3 * mg + (n - 1 - j)) * n + x];
      if (a.cpush && (x < mg || x >= n - mg) && (j < mg || j >= n - mg)) {   // carried corner ghost
        const int qx = x < mg ? 0 : 1, qy = j < mg ? 0 : 1;
        const int v = a.cpush[((tile * 4 + (qx | (qy << 1))) * mg + (qy ? n - 1 - j : j)) * mg + (qx ? n - 1 - x : x)];
        if (v != -1) pt[qx ^ 1] = v;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (pt[k] >= 0) {
#pragma unroll
          for (int f = 0; f < 4; ++f) bst<0>(o1[f], r1, (unsigned)pt[k] * ES, f * fs);
        }
      }
    }

    // ---- stage 2 consumes row j, stage 3 consumes stage 2's row j - 2 ----------
    {
      T C2[5], o2[4];
      prim(o1, C2);
      T mn2[3];
      mrow(j - 1, mn2);
      const bool out2 = stage_row(std::integral_constant<int, 2>(), st2, C2, j, j - y0, G2, mn2, ms2, o2);
#pragma unroll
      for (int k = 0; k < 3; ++k) ms2[k] = mn2[k];
      ld_geo(j - 1, G2);
      if (out2) {
        const int j2 = j - 2;
        ring_st(1, j2, o2);
        if (own & (x >= 2) & (x < n - 2) & (j2 >= rlo) & (j2 < rhi) & (xband | yband(j2))) {
          const unsigned pc = cell(x, j2);
#pragma unroll
          for (int f = 0; f < 4; ++f) bst<0>(o2[f], r2, pc * ES, f * fs);
        }
        T C3[5], o3[4];
        prim(o2, C3);
        T mn3[3];
        mrow(j - 3, mn3);
        const bool out3 = stage_row(std::integral_constant<int, 3>(), st3, C3, j2, j2 - (ys - 2), G3, mn3, ms3, o3);
#pragma unroll
        for (int k = 0; k < 3; ++k) ms3[k] = mn3[k];
        if (out3) {
          const int j3 = j2 - 2;
          if (own & (x >= 4) & (x < n - 4)) {
            const unsigned pc = cell(x, j3);
#pragma unroll
            for (int f = 0; f < 4; ++f) bst<0>(o3[f], rO, pc * ES, f * fs);
          }
        }
      }
      ld_geo(j - 3, G3);
    }

    // ---- advance stage 1 -----------------------------------------------------------
#pragma unroll
    for (int f = 0; f < 5; ++f) { cA[f] = cB[f]; cB[f] = cC[f]; }
#pragma unroll
    for (int f = 0; f < 4; ++f) { hsA[f] = hsB[f]; Gs[f] = Gn[f]; }
  }
}

template <typename T, int LIM, int R>
int march3_l(const StageDesc* d, const March3Desc* md, hipStream_t s) {
  Args<T> a = make_args<T>(d);
  P3<T> m;
  m.q1 = (T*)md->q1;
  m.q2 = (T*)md->q2;
  // the kernel's SSP-RK3 coefficients are compile-time (RK3<T, s>): refuse others
  const double b[3][3] = {{0.0, 1.0, 1.0}, {0.75, 0.25, 0.25}, {1.0 / 3.0, 2.0 / 3.0, 2.0 / 3.0}};
  for (int k = 0; k < 3; ++k)
    if (md->b0[k] != b[k][0] || md->b1[k] != b[k][1] || md->b2[k] != b[k][2]) return -14;
  m.D = md->D;
  m.ncs = (d->n - 8 + M3O - 1) / M3O;
  m.nrs = (d->n - 8 + R - 1) / R;
  m.njobs = d->ntile * m.ncs * m.nrs;
  const int nb = (m.njobs + MWPB - 1) / MWPB;
  hipLaunchKernelGGL((march3_kernel<T, LIM, R>), dim3(nb), dim3(MW * MWPB), 0, s, a, m);
  return (int)hipGetLastError();
}

template <typename T, int R>
int march3_r(const StageDesc* d, const March3Desc* m, hipStream_t s) {
  switch (d->limiter) {
    case 0: return march3_l<T, 0, R>(d, m, s);
    case 1: return march3_l<T, 1, R>(d, m, s);
    case 2: return march3_l<T, 2, R>(d, m, s);
    case 3: return march3_l<T, 3, R>(d, m, s);
  }
  return -11;      // PPM: the block kernel
}

template <typename T>
int march3_t(int rows, const StageDesc* d, const March3Desc* m, hipStream_t s) {
  switch (rows) {
    case 16: return march3_r<T, 16>(d, m, s);
    case 32: return march3_r<T, 32>(d, m, s);
    case 64: return march3_r<T, 64>(d, m, s);
  }
  return -2;
}

}  // namespace

// One pipelined SSP-RK3 step over the tile interiors (see the header comment);
// the band launches of the stage kernel complete it (ops/march3.py).  One rank
// (no remote ghosts), PLR limiters, per-tile geometry records.
extern "C" int stsp_march3_launch(int dtype, int rows, const StageDesc* d, const March3Desc* m, hipStream_t stream) {
  if (!m || !m->q1 || !m->q2 || !d->Q || !d->out) return -12;
  if (d->remote || d->blocks || d->xg) return -13;
  if (d->pw != d->n + 2 * d->mg || d->mg != 2 || d->n < 24) return -5;
  // the band must reach what the edge blocks read (<= D - 1) and stay inside
  // the first / last strip's stage-1 columns
  if (m->D < 6 || m->D > 48 || 2 * m->D > d->n) return -5;
  if (!d->pedge || !d->pe_base || !d->pe_t || !d->push || !d->mx || !d->my || !d->cgeo || !d->ex || !d->ey)
    return -12;
  if (dtype == 1) return march3_t<double>(rows, d, m, stream);
  if (dtype == 0) return march3_t<float>(rows, d, m, stream);
  return -4;
}
