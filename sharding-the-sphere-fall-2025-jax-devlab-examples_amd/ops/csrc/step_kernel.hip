// Persistent step kernel for the cubed sphere, gfx950 (CDNA4).
//
// ONE launch runs `nsteps` whole time steps (every RK stage) for a rank.  Each
// workgroup keeps one BX x BY block for the whole launch:
//
//   * the block's own state (the step-start state X and the current stage
//     input Q) lives in registers across stages and steps; its geometry (cell
//     record, edge lengths, normals, push targets) is loaded once;
//   * a stage boundary is a hand-off of the halo ring only: every cell that a
//     neighbouring block's window reads (the NG-wide band along each interior
//     block side, and the tile-edge cells pushed into neighbouring tiles' ghost
//     slots, with the cube-edge T/R/TR orientation folded into the push map)
//     is stored as 8-byte {tag, 32-bit payload} granules into an exchange
//     buffer laid out like the padded state, one plane per field
//     ([slot][F][S], see xoff: lanes holding consecutive cells touch
//     consecutive bytes, so a wave's store or poll is a few whole lines, not
//     one line per lane); the reading thread re-reads its
//     window cell's granules until every tag equals the stage epoch.  The data
//     is the flag: no drain, no flag, no fence, no grid barrier
//     (cdna_hip_programming.md Guideline 16, R2; MI355X_MICROARCH.md price list,
//     handoff-1to1 ~0.8-1.0 us against a ~1.5-1.9 us dependent kernel boundary
//     plus the window round trip every launch pays);
//   * window corners (never read by the dimension-split stencils) are not
//     loaded, so a block depends on its four side neighbours only.
//
// Why two slots are enough.  Stage s reads tag E = e0 + s from slot E % 2 and
// writes tag E + 1 into slot (E + 1) % 2.  A producer P overwrites slot E % 2
// with tag E + 2 only in ITS stage s + 1, which first waits for OUR stage-s
// output, which we store only after our stage-s window loads returned.  This
// needs the read relation to be symmetric (P reads from us whenever we read
// from P); the host checks that for every block before it launches
// (ops/persistent.py: producer_blocks + symmetry check).
//
// Launch contract (checked on the host and in stsp_step_launch): all blocks
// co-resident (the grid is at most the occupancy-API bound), every wait bounded
// by a wall-clock timeout that sets *err and lets every block drain, tags only
// grow (per-block epochs persist in device memory across launches, so a
// replayed or repeated launch never needs the buffer cleared).
//
// The first stage of a launch reads its ring from the state buffer (written by
// the previous launch or the host); the last stage writes its cells and pushes
// to the state buffer with plain stores.  Arithmetic is that of stage_body
// (stage_kernel.hip), statement for statement, so the result is bitwise equal
// to launch-per-stage stepping.
#include "stage_common.h"

#ifndef STSP_STEP_BAND_PLAIN
#define STSP_STEP_BAND_PLAIN 0
#endif

namespace {

template <typename T>
struct SArgs {
  Args<T> a;            // a.Q = a.X = a.out = the state buffer
  int nst, nsteps;
  T a0[4], a1[4], a2[4];
  unsigned long long* xb;
  int* epoch;
  int* err;
  long long timeout_ticks;
#ifdef STSP_STEP_DEBUG
  long long* dbg;       // nullable: [0] count, then records of 8 (timeout diagnostics)
#endif
};

// Debug build (STSP_STEP_DEBUG): lane 0 of wave 0 records s_memrealtime (100 MHz)
// at 4 points of the first 16 stages: window start, after the window barrier,
// after the flux barrier, after the hand-off stores; dbg[4096 + (bid * 16 + s) * 4 + k].
#ifdef STSP_STEP_DEBUG
#define SSTAMP_T(k, who)                                                                           \
  do {                                                                                             \
    if (sa.dbg && tid == (who) && s < 16) sa.dbg[4096 + ((long)bid * 16 + s) * 8 + (k)] =           \
        (long long)__builtin_amdgcn_s_memrealtime();                                               \
  } while (0)
#else
#define SSTAMP_T(k, who) do {} while (0)
#endif
#define SSTAMP(k) SSTAMP_T(k, 0)

// Exchange-buffer layout: [slot][F][S] cells of 8 * G bytes, G = esize / 4.
// fp32: one 8-byte {tag, payload} granule per field; fp64: a 16-byte pair of
// granules {tag | low word, tag | high word} per field, written by ONE
// dwordx4 store and read by one dwordx4 load (each 8-byte half is single-copy
// atomic, so the reader checks both tags).  Stores are write-through (sc1);
// lanes holding consecutive cells touch consecutive bytes.
template <typename T>
__device__ __forceinline__ unsigned xoff(unsigned slot, int F, int f, unsigned S, unsigned cell) {
  return ((slot * (unsigned)F + (unsigned)f) * S + cell) * (unsigned)(2 * sizeof(T));
}

template <typename T, int F, int AUX = 16>
__device__ __forceinline__ void store_granules(__amdgpu_buffer_rsrc_t xr, unsigned slot, unsigned S, unsigned cell,
                                               unsigned tag, const T (&o)[F]) {
#pragma unroll
  for (int f = 0; f < F; ++f) {
    if constexpr (sizeof(T) == 8) {
      const unsigned long long b = __builtin_bit_cast(unsigned long long, o[f]);
      const v4u32 g = {(unsigned)b, tag, (unsigned)(b >> 32), tag};
      __builtin_amdgcn_raw_buffer_store_b128(g, xr, (int)xoff<T>(slot, F, f, S, cell), 0, AUX);
    } else {
      const v2u32 g = {__builtin_bit_cast(unsigned, o[f]), tag};
      __builtin_amdgcn_raw_buffer_store_b64(g, xr, (int)xoff<T>(slot, F, f, S, cell), 0, AUX);
    }
  }
}

// Re-read one cell's granules until every tag equals `want`; false on
// timeout / after another block's timeout (values then undefined).
template <typename T, int F>
__device__ __forceinline__ bool wait_granules(__amdgpu_buffer_rsrc_t xr, unsigned slot, unsigned S, unsigned cell,
                                              unsigned want, T (&v)[F], int* err, long long timeout_ticks,
                                              unsigned* seen = nullptr) {
  unsigned lo[F], hi[F], t0_[F], t1_[F];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool ok;
  for (;;) {
    ok = true;
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if constexpr (sizeof(T) == 8) {
        const v4u32 g = __builtin_amdgcn_raw_buffer_load_b128(xr, (int)xoff<T>(slot, F, f, S, cell), 0, 16);
        lo[f] = g.x; t0_[f] = g.y; hi[f] = g.z; t1_[f] = g.w;
        ok &= (t0_[f] == want) & (t1_[f] == want);
      } else {
        const v2u32 g = __builtin_amdgcn_raw_buffer_load_b64(xr, (int)xoff<T>(slot, F, f, S, cell), 0, 16);
        lo[f] = g.x; t0_[f] = g.y; hi[f] = 0; t1_[f] = want;
        ok &= t0_[f] == want;
      }
    }
    if (ok) break;
    if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
    if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout_ticks) {
      __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (seen) {
        unsigned bad = want;
#pragma unroll
        for (int f = 0; f < F; ++f) {
          if (t0_[f] != want) bad = t0_[f];
          if (t1_[f] != want) bad = t1_[f];
        }
        *seen = bad;
      }
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");   // the buffer loads above are re-issued every pass
  }
#pragma unroll
  for (int f = 0; f < F; ++f) {
    if constexpr (sizeof(T) == 8)
      v[f] = __builtin_bit_cast(T, ((unsigned long long)hi[f] << 32) | lo[f]);
    else
      v[f] = __builtin_bit_cast(T, lo[f]);
  }
  return ok;
}

template <typename T, int P, int BX, int BY, int LIM>
__global__ __launch_bounds__((Geom<BX, BY>::NT)) void step_kernel(SArgs<T> sa) {
  const Args<T>& a = sa.a;
  pin_args(a);
  constexpr int F = Phys<P>::F;
  constexpr int NG = (LIM == 4) ? 3 : Phys<P>::NG;
  constexpr int FL = Phys<P>::FL;
  constexpr bool RECON = (P != 1);
  constexpr bool FUSED = RECON && (LIM != 4) && STSP_FUSE_FACES;
  constexpr bool FACES = RECON && !FUSED;
  constexpr int NT = Geom<BX, BY>::NT;
  constexpr int NX = Geom<BX, BY>::NX;
  constexpr int NY = Geom<BX, BY>::NY;
  constexpr int EX = BX + 2 * NG;
  constexpr int EY = BY + 2 * NG;
  constexpr int NFX = (BX + 2) * BY;
  constexpr int NFY = BX * (BY + 2);
  static_assert(EX * EY <= NT, "window load assumes one cell per thread");
  constexpr int WS = EX + 1;
  constexpr int WF = EY * WS;
  constexpr int NE = NX + NY;
  constexpr int NFT = NFX + NFY;
  constexpr bool SW = (P == 2);
  __shared__ T s_w[FL][EY][EX + 1];
  __shared__ T s_fm[FACES ? F : 1][FACES ? NFT : 1];
  __shared__ T s_fp[FACES ? F : 1][FACES ? NFT : 1];
  __shared__ T s_fl[F][NE];
  __shared__ T s_nrm[SW ? 3 : 1][SW ? BX + BY + 2 : 1];
  __shared__ T s_len[SW ? NE : 1];

  const int bid = xcd_remap(blockIdx.x, a.nblocks);
  const int n = a.n, S = a.S, nn = n * n, mg = a.mg, pw = a.pw;
  const int nbx = (n + BX - 1) / BX, nby = (n + BY - 1) / BY;
  const int tile = a.mdiv_t ? (int)__umulhi((unsigned)bid, a.mdiv_t) : bid / (nbx * nby);
  const int rem = bid - tile * nbx * nby;
  const int yb = a.mdiv_r ? (int)__umulhi((unsigned)rem, a.mdiv_r) : rem / nbx;
  const int xb = rem - yb * nbx;
  const int x0 = xb * BX, y0 = yb * BY;
  const int tid = threadIdx.x;
  const unsigned tb = (unsigned)(tile * pw * pw);
  const int gbase = tile * nn;
  const int e0 = sa.epoch[bid];

  // ---- thread roles (as stage_body) -------------------------------------------
  constexpr int NIN = BX * BY, RING = EX * EY - NIN, NOWN = NIN / 64;
  static_assert(NIN % 64 == 0, "own cells fill whole waves");
  static_assert(RING <= NT - NIN, "one ring cell per thread without an own cell");
  const int wv = tid >> 6;
  int oid, rid, eid;
  if constexpr (Geom<BX, BY>::W10) {
    const int lane = tid & 63;
    const unsigned os = (unsigned)(Geom<BX, BY>::OWN_TAB >> (4 * wv)) & 15u;
    const unsigned fs = (unsigned)(Geom<BX, BY>::FLUX_TAB >> (4 * wv)) & 15u;
    const unsigned rs = (unsigned)(Geom<BX, BY>::RING_TAB >> (4 * wv)) & 15u;
    oid = os != 15u ? (int)os * 64 + lane : -1;
    eid = fs != 15u ? (int)fs * 64 + lane : NE;
    rid = rs != 15u ? (int)rs * 64 + lane : RING;
  } else {
#if STSP_OWN_SKIP0
    const int below = wv - (wv + 3) / 4;
    oid = ((wv & 3) != 0 && below < NOWN) ? below * 64 + (tid & 63) : -1;
#else
    const int below = wv;
    oid = wv < NOWN ? tid : -1;
#endif
    rid = oid >= 0 ? RING : tid - 64 * (below < NOWN ? below : NOWN);
    eid = tid;
  }
  int wly = -1, wlx = 0;
  if (oid >= 0) {
    wly = NG + oid / BX;
    wlx = NG + oid % BX;
  } else {
    const int r = rid;
    if (r < 2 * NG * EX) {
      const int rr = r / EX;
      wlx = r - rr * EX;
      wly = rr < NG ? rr : EY - 2 * NG + rr;
    } else if (r < RING) {
      const int r2 = r - 2 * NG * EX, rr = r2 / (2 * NG), c = r2 - rr * (2 * NG);
      wly = NG + rr;
      wlx = c < NG ? c : EX - 2 * NG + c;
    }
  }
  const int ox = oid % BX, oy = oid / BX;
  const int cx = x0 + ox, cy = y0 + oy;
  const bool own = (oid >= 0) && (cx < n) && (cy < n);
  // window cell of a thread without an own cell (a ring cell, or an own slot
  // past the tile edge of a partial block): 0 = zero / not needed, 1 = a real
  // cell (from the state at a launch's first stage, then from granules)
  int ring_kind = 0;
  unsigned ring_pa = 0;
  if (!own && wly >= 0) {
    // read iff within NG of the block's real cells along one of their rows or
    // columns (ops/persistent.py::producer_blocks): window corners, tile
    // corner ghosts and, in a partial block, the rows / columns past the tile
    // edge are never read by the dimension-split stencils
    const int x = x0 + wlx - NG, y = y0 + wly - NG;
    const int xe = x0 + BX < n ? x0 + BX : n, ye = y0 + BY < n ? y0 + BY : n;
    const bool inx = (x >= x0) & (x < xe), iny = (y >= y0) & (y < ye);
    const bool nx = (x >= x0 - NG) & (x < xe + NG), ny = (y >= y0 - NG) & (y < ye + NG);
    const bool oxx = (x < 0) | (x >= n), oyy = (y < 0) | (y >= n);
    if (((inx & ny) | (iny & nx)) && !(oxx & oyy)) {
      ring_kind = 1;
      ring_pa = tb + (unsigned)((y + mg) * pw + (x + mg));
    }
  }

  // ---- loaded once: own-cell geometry, push targets, edge coefficient, normals
  const unsigned pc = tb + (unsigned)((cy + mg) * pw + (cx + mg));
  const unsigned gc = (unsigned)(gbase + cy * n + cx);
  T xs[F], qc[F];
  T iA = T(0), r0 = T(0), r1 = T(0), r2 = T(0);
  T gb[3] = {T(0), T(0), T(0)};
  int pt[4] = {-1, -1, -1, -1};
  bool exp_own = false;
  if (own) {
#pragma unroll
    for (int f = 0; f < F; ++f) qc[f] = *o32(a.Q + f * S, pc);
    if constexpr (P == 2) {
      T rec[8];
      load_rec8<T>(o32(a.cgeo, gc * 8u), rec);
      iA = rec[0]; r0 = rec[1]; r1 = rec[2]; r2 = rec[3];
      gb[0] = rec[4]; gb[1] = rec[5]; gb[2] = rec[6];
    } else {
      iA = *o32(a.invA, gc);
    }
    const int* pm = a.push + (long)tile * 4 * mg * n;
    if (cx < mg) pt[0] = *o32(pm, (unsigned)((0 * mg + cx) * n + cy));
    if (cx >= n - mg) pt[1] = *o32(pm, (unsigned)((1 * mg + (n - 1 - cx)) * n + cy));
    if (cy < mg) pt[2] = *o32(pm, (unsigned)((2 * mg + cy) * n + cx));
    if (cy >= n - mg) pt[3] = *o32(pm, (unsigned)((3 * mg + (n - 1 - cy)) * n + cx));
    // band cells read by the side-neighbour block of the same tile
    exp_own = (ox < NG && x0 > 0) || (ox >= BX - NG && x0 + BX < n) || (oy < NG && y0 > 0) ||
              (oy >= BY - NG && y0 + BY < n);
  }
  T nrm = T(0);
  if constexpr (P == 2) {
    if (tid < 3 * (BX + 1)) {
      const int k = tid / (BX + 1), c = tid - k * (BX + 1);
      if (x0 + c <= n) nrm = *o32(a.mx, (unsigned)((tile * 3 + k) * (n + 1) + x0 + c));
    } else if (tid < 3 * (BX + 1) + 3 * (BY + 1)) {
      const int u = tid - 3 * (BX + 1);
      const int k = u / (BY + 1), c = u - k * (BY + 1);
      if (y0 + c <= n) nrm = *o32(a.my, (unsigned)((tile * 3 + k) * (n + 1) + y0 + c));
    }
  }
  const bool is_x = eid < NX;
  const int ete = is_x ? eid : eid - NX;
  const int e_r = is_x ? ete / (BX + 1) : ete / BX;
  const int e_c = is_x ? ete - e_r * (BX + 1) : ete - e_r * BX;
  const int ex_ = x0 + e_c, ey_ = y0 + e_r;
  const bool edge_ok = is_x ? (ex_ <= n && ey_ < n) : (eid < NX + NY && ex_ < n && ey_ <= n);
  T coef = T(0);
  if (edge_ok) {
    coef = is_x ? *o32(a.ex, (unsigned)(tile * n * (n + 1) + ey_ * (n + 1) + ex_))
                : *o32(a.ey, (unsigned)(tile * (n + 1) * n + ey_ * n + ex_));
  }
  const int pe = (LIM == 4) ? a.pedge[tile] : 0;
  if constexpr (P == 2) {
    if (tid < 3 * (BX + 1)) {
      const int k = tid / (BX + 1), c = tid - k * (BX + 1);
      s_nrm[k][c] = nrm;
    } else if (tid < 3 * (BX + 1) + 3 * (BY + 1)) {
      const int u = tid - 3 * (BX + 1);
      const int k = u / (BY + 1), c = u - k * (BY + 1);
      s_nrm[k][BX + 1 + c] = nrm;
    }
    if (edge_ok) s_len[eid] = coef;
  }
  if (own) {
#pragma unroll
    for (int f = 0; f < F; ++f) xs[f] = qc[f];
  }
  const __amdgpu_buffer_rsrc_t xr = brsrc(sa.xb);
  const int total = sa.nst * sa.nsteps;

  auto put = [&](int ly, int lx, const T (&v)[F]) {
    if constexpr (P == 2) {
      const T inv = v[0] != T(0) ? trcp(v[0]) : T(0);
      s_w[0][ly][lx] = v[0];
      s_w[1][ly][lx] = v[1] * inv;
      s_w[2][ly][lx] = v[2] * inv;
      s_w[3][ly][lx] = v[3] * inv;
      s_w[4][ly][lx] = tsqrt(a.g * tmax(v[0], T(0)));
    } else {
      s_w[0][ly][lx] = v[0];
    }
  };

  for (int s = 0; s < total; ++s) {
    SSTAMP(0);
    const int k = s % sa.nst;
    const unsigned E = (unsigned)(e0 + s);
    // ---- 1. window ---------------------------------------------------------------
    if (own) {
      put(wly, wlx, qc);
    } else if (ring_kind && s > 0) {
      T v[F];
#ifdef STSP_STEP_DEBUG
      unsigned seen = E;
      const bool ok = wait_granules<T, F>(xr, E & 1u, (unsigned)S, ring_pa, E, v, sa.err, sa.timeout_ticks,
                                          sa.dbg ? &seen : nullptr);
      if (!ok && sa.dbg && seen != E) {   // diagnostics: who timed out waiting for what
        const long long i = __hip_atomic_fetch_add((gu64*)sa.dbg, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (i < 64) {
          long long* r = sa.dbg + 8 + 8 * i;
          r[0] = bid; r[1] = s; r[2] = ring_pa; r[3] = E; r[4] = seen; r[5] = wly; r[6] = wlx;
          r[7] = (long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_ID
        }
      }
#else
      wait_granules<T, F>(xr, E & 1u, (unsigned)S, ring_pa, E, v, sa.err, sa.timeout_ticks);
#endif
      put(wly, wlx, v);
    } else if (ring_kind) {
      T v[F];
#pragma unroll
      for (int f = 0; f < F; ++f) v[f] = *o32(a.Q + f * S, ring_pa);
      put(wly, wlx, v);
    } else if (wly >= 0) {
      const T z[F] = {};
      put(wly, wlx, z);
    }
    SSTAMP(6);
    __syncthreads();
    SSTAMP(1);

    // ---- 1b. face values (PPM / unfused PLR) ------------------------------------------
    if constexpr (FACES) {
      const T* w0 = &s_w[0][0][0];
      for (int t = tid; t < NFT; t += NT) {
        const bool tx = t < NFX;
        const int u = tx ? t : t - NFX;
        const int r = tx ? u / (BX + 2) : u / BX;
        const int c = u - r * (tx ? BX + 2 : BX);
        const int x = x0 + (tx ? c - 1 : c), y = y0 + (tx ? r : r - 1);
        if (x <= n && y <= n) {
          const int ci = (tx ? NG + r : NG - 1 + r) * WS + (tx ? NG - 1 + c : NG + c);
          const int st = tx ? 1 : WS;
#pragma unroll
          for (int f = 0; f < F; ++f) {
            const T m1 = w0[f * WF + ci - st], c0 = w0[f * WF + ci], p1 = w0[f * WF + ci + st];
            const int xc = tx ? x : y;
            const bool edge_cell = (LIM == 4) && (((pe & (tx ? 1 : 4)) && xc <= 1) || ((pe & (tx ? 2 : 8)) && xc >= n - 2));
            if (LIM == 4 && edge_cell) {
              const T hs = T(0.5) * slope<2>(c0 - m1, p1 - c0);
              s_fm[f][t] = c0 - hs;
              s_fp[f][t] = c0 + hs;
            } else if constexpr (LIM == 4) {
              const T m2 = w0[f * WF + ci - 2 * st], p2 = w0[f * WF + ci + 2 * st];
              T aL = T(7.0 / 12.0) * (m1 + c0) - T(1.0 / 12.0) * (m2 + p1);
              T aR = T(7.0 / 12.0) * (c0 + p1) - T(1.0 / 12.0) * (m1 + p2);
              const bool flat = (aR - c0) * (c0 - aL) <= T(0);
              const T d = aR - aL;
              const T m6 = T(6) * (c0 - T(0.5) * (aL + aR));
              const bool ovl = d * m6 > d * d;
              const bool ovr = -(d * d) > d * m6;
              const T nL = flat ? c0 : (ovl ? T(3) * c0 - T(2) * aR : aL);
              const T nR = flat ? c0 : ((!ovl && ovr) ? T(3) * c0 - T(2) * aL : aR);
              s_fm[f][t] = nL;
              s_fp[f][t] = nR;
            } else {
              const T hs = T(0.5) * slope<LIM>(c0 - m1, p1 - c0);
              s_fm[f][t] = c0 - hs;
              s_fp[f][t] = c0 + hs;
            }
          }
        }
      }
      __syncthreads();
    }

    // ---- 2. one edge flux per thread ---------------------------------------------------
    if (edge_ok) {
      const int fl_ = is_x ? e_r * (BX + 2) + e_c : NFX + e_r * BX + e_c;
      const int fst = is_x ? 1 : BX;
      const int cl_ = is_x ? (NG + e_r) * WS + NG - 1 + e_c : (NG - 1 + e_r) * WS + NG + e_c;
      const int cst = is_x ? 1 : WS;
      const T* w0 = &s_w[0][0][0];
      if constexpr (P == 1) {
        s_fl[0][eid] = -coef * (w0[cl_ + cst] - w0[cl_]);
      } else if constexpr (P == 0) {
        T wl, wr;
        if constexpr (FUSED) {
          const T m1 = w0[cl_ - cst], c0 = w0[cl_], p1 = w0[cl_ + cst], p2 = w0[cl_ + 2 * cst];
          wl = c0 + half_slope<LIM>(c0 - m1, p1 - c0);
          wr = p1 - half_slope<LIM>(p1 - c0, p2 - p1);
        } else {
          wl = s_fp[0][fl_];
          wr = s_fm[0][fl_ + fst];
        }
        s_fl[0][eid] = coef * (coef > T(0) ? wl : wr);
      } else {
        T wl[4], wr[4], cl[5], cr[5];
#pragma unroll
        for (int f = 0; f < 5; ++f) { cl[f] = w0[f * WF + cl_]; cr[f] = w0[f * WF + cl_ + cst]; }
        if constexpr (FUSED) {
#pragma unroll
          for (int f = 0; f < 4; ++f) {
            const T m1 = w0[f * WF + cl_ - cst], p2 = w0[f * WF + cl_ + 2 * cst];
            const T d1 = cr[f] - cl[f];
            wl[f] = cl[f] + half_slope<LIM>(cl[f] - m1, d1);
            wr[f] = cr[f] - half_slope<LIM>(d1, p2 - cr[f]);
          }
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) { wl[f] = s_fp[f][fl_]; wr[f] = s_fm[f][fl_ + fst]; }
        }
        const int ni = is_x ? e_c : BX + 1 + e_r;
        T fl[4];
        swe_flux<T>(wl, wr, cl, cr, s_nrm[0][ni], s_nrm[1][ni], s_nrm[2][ni], coef, a.g, fl);
#pragma unroll
        for (int f = 0; f < 4; ++f) s_fl[f][eid] = fl[f];
      }
    }
    // ---- 2b. sources and the RK base (before the barrier, as stage_body) --------------
    const int ew = oy * (BX + 1) + ox;
    const int es = NX + oy * BX + ox;
    const T ca0 = sa.a0[k], ca1 = sa.a1[k], ca2 = sa.a2[k];
    T qs[F], base[F];
    T src[3] = {T(0), T(0), T(0)};
    if (own) {
      if constexpr (P == 2) {
#pragma unroll
        for (int f = 0; f < 4; ++f) qs[f] = qc[f];
        const T fc = a.omega2 * r2;
        const T h = qs[0];
        const T cor[3] = {r1 * qs[3] - r2 * qs[2], r2 * qs[1] - r0 * qs[3], r0 * qs[2] - r1 * qs[1]};
        const T Lw = s_len[ew], Le = s_len[ew + 1], Ls = s_len[es], Ln = s_len[es + BX];
        const T pb = T(0.5) * a.g * h * h * iA, gh = a.g * h;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const T Sk = Le * s_nrm[q][ox + 1] - Lw * s_nrm[q][ox] + Ln * s_nrm[q][BX + 2 + oy] - Ls * s_nrm[q][BX + 1 + oy];
          src[q] = -fc * cor[q] + pb * Sk - gh * gb[q];
        }
      } else {
        qs[0] = s_w[0][NG + oy][NG + ox];
      }
#pragma unroll
      for (int f = 0; f < F; ++f) {
        base[f] = T(0);
        if (ca1 != T(0)) base[f] = ca1 * qs[f];
        if (ca0 != T(0)) base[f] += ca0 * xs[f];
      }
    }
    __syncthreads();
    SSTAMP(2);

    // ---- 3. divergence + RK combination, then the hand-off ----------------------------
    if (own) {
      T dq[F];
#pragma unroll
      for (int f = 0; f < F; ++f)
        dq[f] = -((s_fl[f][ew + 1] - s_fl[f][ew]) + (s_fl[f][es + BX] - s_fl[f][es])) * iA;
      if constexpr (P == 2) {
#pragma unroll
        for (int q = 0; q < 3; ++q) dq[1 + q] += src[q];
      }
      T o[F];
#pragma unroll
      for (int f = 0; f < F; ++f) o[f] = ca2 * a.dt * dq[f] + base[f];
      if constexpr (P == 2) {
        const T d = o[1] * r0 + o[2] * r1 + o[3] * r2;
        o[1] -= d * r0; o[2] -= d * r1; o[3] -= d * r2;
      }
      SSTAMP_T(4, 64);
      if (s + 1 < total) {
        const unsigned tag = E + 1u;
        // band cells go to side neighbours of the same tile, which the XCD-aware
        // block remap places on this XCD: STSP_STEP_BAND_PLAIN stores them
        // without write-through (they stay in the shared L2)
        if (exp_own) store_granules<T, F, STSP_STEP_BAND_PLAIN ? 0 : 16>(xr, tag & 1u, (unsigned)S, pc, tag, o);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (pt[q] >= 0) store_granules<T, F>(xr, tag & 1u, (unsigned)S, (unsigned)pt[q], tag, o);
        }
        SSTAMP_T(5, 64);
#ifdef STSP_STEP_DEBUG
        if (sa.dbg && tid == 64) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          SSTAMP_T(7, 64);
        }
#endif
      } else {
#pragma unroll
        for (int f = 0; f < F; ++f) st_out<false>(a.wt, o32(a.out + f * S, pc), o[f]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (pt[q] >= 0) {
#pragma unroll
            for (int f = 0; f < F; ++f) st_out<false>(a.wt, o32(a.out + f * S, (unsigned)pt[q]), o[f]);
          }
        }
      }
#pragma unroll
      for (int f = 0; f < F; ++f) qc[f] = o[f];
      if (k == sa.nst - 1) {
#pragma unroll
        for (int f = 0; f < F; ++f) xs[f] = o[f];
      }
    }
    SSTAMP(3);
  }
  if (tid == 0) sa.epoch[bid] = e0 + total;
}

// Blocks of this instantiation that are guaranteed co-resident on the device.
// The occupancy API counts wave slots per CU; a block's waves are spread over
// the CU's 4 SIMDs, and with k blocks per CU some SIMD may have to host
// k * ceil(W / 4) of them (W waves per block).  Only k with that worst case
// within the VGPR-limited waves per SIMD are counted (a 5-wave block at 3
// waves/SIMD: the API says 2 per CU, but the second one did not always fit,
// and blocks waiting for a slot deadlock a persistent grid).
template <typename T, int P, int BX, int BY, int LIM>
int occupancy() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, step_kernel<T, P, BX, BY, LIM>, Geom<BX, BY>::NT, 0) !=
      hipSuccess)
    return -1;
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, (const void*)step_kernel<T, P, BX, BY, LIM>) != hipSuccess) return -1;
  const int vg = fa.numRegs > 0 ? ((fa.numRegs + 7) / 8) * 8 : 512;
  int per_simd = 512 / vg;
  if (per_simd > 8) per_simd = 8;
  constexpr int W = Geom<BX, BY>::NT / 64;
  const int k = per_simd / ((W + 3) / 4);
  if (k < nb) nb = k;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  return nb * cus;
}

template <typename T, int P, int BX, int BY, int LIM>
int launch_s(const StepDesc* d, hipStream_t s, bool query) {
  static const int maxb = occupancy<T, P, BX, BY, LIM>();
  if (query) return maxb;
  const StageDesc* st = &d->st;
  if (st->nblocks <= 0 || st->nblocks > maxb) return -12;     // all blocks must be co-resident
  SArgs<T> sa;
  sa.a = make_args<T>(st);
  set_magic<T, BX, BY>(sa.a);
  sa.a.wt = want_wt((long)st->nblocks * BX * BY) ? 1 : 0;
  sa.nst = d->nst;
  sa.nsteps = d->nsteps;
  for (int k = 0; k < 4; ++k) {
    sa.a0[k] = (T)d->a0[k];
    sa.a1[k] = (T)d->a1[k];
    sa.a2[k] = (T)d->a2[k];
  }
  sa.xb = (unsigned long long*)d->xb;
  sa.epoch = d->epoch;
  sa.err = d->err;
  sa.timeout_ticks = d->timeout_ticks;
#ifdef STSP_STEP_DEBUG
  sa.dbg = (long long*)d->dbg;
#endif
  hipLaunchKernelGGL((step_kernel<T, P, BX, BY, LIM>), dim3(st->nblocks), dim3(Geom<BX, BY>::NT), 0, s, sa);
  return (int)hipGetLastError();
}

template <typename T, int P, int BX, int BY>
int launch_st(const StepDesc* d, int limiter, hipStream_t s, bool query) {
  if constexpr (P == 1) return launch_s<T, P, BX, BY, 0>(d, s, query);
  switch (limiter) {
    case 0: return launch_s<T, P, BX, BY, 0>(d, s, query);
    case 1: return launch_s<T, P, BX, BY, 1>(d, s, query);
    case 2: return launch_s<T, P, BX, BY, 2>(d, s, query);
    case 3: return launch_s<T, P, BX, BY, 3>(d, s, query);
    case 4:
      if constexpr ((BX + 6) * (BY + 6) <= Geom<BX, BY>::NT) return launch_s<T, P, BX, BY, 4>(d, s, query);
      else return -11;
  }
  return -7;
}

template <typename T, int P>
int launch_sp(int bx, int by, const StepDesc* d, int limiter, hipStream_t s, bool query) {
  if (bx == 16 && by == 16) return launch_st<T, P, 16, 16>(d, limiter, s, query);
  if (bx == 16 && by == 8) return launch_st<T, P, 16, 8>(d, limiter, s, query);
  if (bx == 8 && by == 8) return launch_st<T, P, 8, 8>(d, limiter, s, query);
  return -2;
}

template <typename T>
int launch_sd(int phys, int bx, int by, const StepDesc* d, int limiter, hipStream_t s, bool query) {
  switch (phys) {
    case 0: return launch_sp<T, 0>(bx, by, d, limiter, s, query);
    case 1: return launch_sp<T, 1>(bx, by, d, limiter, s, query);
    case 2: return launch_sp<T, 2>(bx, by, d, limiter, s, query);
  }
  return -3;
}

}  // namespace

extern "C" int stsp_step_launch(int phys, int dtype, int bx, int by, const StepDesc* d, hipStream_t stream) {
  const StageDesc* st = &d->st;
  if (d->nst < 1 || d->nst > 4 || d->nsteps < 1 || d->nst * d->nsteps < 2) return -8;
  if (!d->xb || !d->epoch || !d->err) return -10;
  if (st->blocks || st->remote || st->xg || !st->push || st->pw != st->n + 2 * st->mg) return -6;
  if (st->X != st->Q || st->out != (void*)st->Q) return -9;
  if (st->limiter == 4 && (st->mg < 3 || !st->pedge)) return -5;
  if (dtype == 1) return launch_sd<double>(phys, bx, by, d, st->limiter, stream, false);
  if (dtype == 0) return launch_sd<float>(phys, bx, by, d, st->limiter, stream, false);
  return -4;
}

extern "C" int stsp_step_max_blocks(int phys, int dtype, int bx, int by, int limiter) {
  if (dtype == 1) return launch_sd<double>(phys, bx, by, nullptr, limiter, nullptr, true);
  if (dtype == 0) return launch_sd<float>(phys, bx, by, nullptr, limiter, nullptr, true);
  return -4;
}
