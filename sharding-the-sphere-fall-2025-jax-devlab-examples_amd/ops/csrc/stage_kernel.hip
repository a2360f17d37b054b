// Fused finite-volume Runge-Kutta stage for the cubed sphere, gfx950 (CDNA4).
//
// One launch = one RK stage of one rank: halo load + PLR reconstruction + edge
// fluxes + flux divergence + sources + RK combination + tangent projection +
// halo push, for every cell.  It replaces the reference's XLA-generated chain
// K1-K9 (boundary-strip slices, reversal, dynamic-update-slice
// scatter, then the numerics) with a single kernel, built for the regime the
// headline case lives in (C96: 55k cells = ~1 wave per SIMD on 256 CUs, so every
// dependent memory round trip and every serial flux evaluation is exposed):
//
//   * storage is tile-major with a ghost ring (padded width pw = n + 2 mg); a
//     stage writes each cell and also PUSHES cells near a tile edge into the
//     neighbour tile's ghost slots (same rank), so the next stage loads its
//     whole window with plain, regular loads: one memory round trip, no index
//     indirection.  Cross-panel orientation (the reference's T/R/TR ops,
//     PY:143-163) lives in the precomputed push map.  Remote ghosts (other
//     GPUs) are read from the RCCL receive buffer through the ghost map, only
//     in the REMOTE (boundary-block) variant;
//   * a workgroup owns a BX x BY block and runs one thread per edge
//     (576 threads for 16x16: 272 x-edges + 272 y-edges), so the flux phase is
//     a single pass; the block + NG halo and the edge fluxes live in LDS;
//   * every own-cell operand (RK inputs, metric terms, push targets) is issued
//     before the first barrier, so its latency hides under the window load;
//   * the linear block id is remapped so consecutive logical blocks (which
//     share halo cells) land on one XCD and its L2 (bijective remap).
//
// Physics (compile-time):  0 = tracer advection (PDF s.13), 1 = diffusion
// (PDF s.12), 2 = shallow water with Cartesian momentum (PY:2).
#include "stage_common.h"

namespace {

// One RK stage of one BX x BY block (all phases).  SYNC: every access to state
// written by other workgroups in this launch is an agent-scope sc1 access (L1
// bypass, write-through); the launch-per-stage kernels use SYNC = false (the
// persistent step kernel, step_kernel.hip, hands its halos off as granules).
// XG = direct xGMI halo: a block reads its remote ghosts from this rank's
// receive ring (slot epoch % STSP_XG_SLOTS) once they have arrived (tags match,
// or the peers' arrival counters are complete), and every block stores the cells
// its peers need into their rings (slot (epoch + 1) % STSP_XG_SLOTS).  Why four
// slots and no reset: see STSP_XG_SLOTS; tags and counters only grow.
template <typename T, int P, int BX, int BY, int LIM, bool REMOTE, bool SYNC, bool XG = false>
__device__ __forceinline__ void stage_body(const Args<T>& a, const int bid) {
  constexpr int F = Phys<P>::F;
  constexpr int NG = (LIM == 4) ? 3 : Phys<P>::NG;   // PPM reads 3 ghost layers
  constexpr int FL = Phys<P>::FL;              // primitive fields (+ sound speed) in LDS
  constexpr bool RECON = (P != 1);             // PLR reconstruction (not for diffusion)
  // FUSED: each edge thread reconstructs the two faces it needs straight from
  // the window (PLR only; PPM keeps the separate face phase, its stencil is wider)
  constexpr bool FUSED = RECON && (LIM != 4) && STSP_FUSE_FACES;
  constexpr bool FACES = RECON && !FUSED;
  // PEW: panel-edge fix-up inside the two border-edge waves (PLR, ten-wave
  // 256-cell blocks): flux slot 0 holds the x-edges at columns 0, 1, BX-1, BX
  // of every row and slot 1 the y-edges at rows 0, 1, BY-1, BY (edge_of_slot),
  // so the only readers of an interpolated ghost or of the neighbour's edge
  // state are the lanes of the wave that computes them: no barrier, and the
  // other seven flux waves never wait for the fix-up
  // (a partial block's panel edge is not at border column BX, so grids with
  // n % 16 != 0 take the block-wide fix-up: pew below)
  constexpr bool PEW = FUSED && Geom<BX, BY>::W10 && STSP_PE_WAVE;
  const bool pew = PEW && a.pew != 0;            // block-uniform
  constexpr int NT = Geom<BX, BY>::NT;
  constexpr int NX = Geom<BX, BY>::NX;
  constexpr int NY = Geom<BX, BY>::NY;
  constexpr int EX = BX + 2 * NG;
  constexpr int EY = BY + 2 * NG;
  constexpr int NFX = (BX + 2) * BY;           // x-direction face tasks
  constexpr int NFY = BX * (BY + 2);           // y-direction face tasks
  static_assert(EX * EY <= NT, "window load assumes one cell per thread");
  // LDS.  Face values, fluxes, normals and lengths are stored flat, x part then
  // y part, indexed by task / edge id, so the x- and y-direction work of the
  // face and flux phases is ONE code path (a wave that holds both kinds of
  // task would otherwise execute both paths back to back).
  constexpr int WS = EX + 1;                   // LDS row stride of the window
  constexpr int WF = EY * WS;                  // LDS field stride of the window
  constexpr int NE = NX + NY;                  // edges
  constexpr int NFT = NFX + NFY;               // face tasks
  constexpr bool SW = (P == 2);
  __shared__ T s_w[FL][EY][EX + 1];
  __shared__ T s_fm[FACES ? F : 1][FACES ? NFT : 1];   // face value on the cell's minus side
  __shared__ T s_fp[FACES ? F : 1][FACES ? NFT : 1];   // ... and plus side
  __shared__ T s_fl[F][NE];                            // edge fluxes
  __shared__ T s_nrm[SW ? 3 : 1][SW ? BX + BY + 2 : 1];  // edge normals: x columns, then y rows
  __shared__ T s_len[SW ? NE : 1];                     // edge lengths (for the curvature balance)
  // panel edges: the neighbour's state at each panel-edge edge of the block,
  // reconstructed in the neighbour's frame, and its raw cell (wave speeds)
  constexpr int BM = BX > BY ? BX : BY;
  constexpr int KG = (LIM == 4) ? 2 : 1;             // interpolated ghost layers the faces read
  __shared__ T s_pf[RECON ? F : 1][RECON ? 4 * BM : 1];
  __shared__ T s_pr[SW ? FL : 1][SW ? 4 * BM : 1];
  // raw (index-space copied) ghost layers k < KG of the panel-edge strips, by
  // window position along the side: the interpolation reads these, so the
  // interpolated ghosts can replace the raw ones in the window without a
  // barrier between the reads and the writes
  constexpr int EM = EX > EY ? EX : EY;
  // It lives in the flux array, which nothing writes before the flux phase
  // (LDS per block decides how many blocks share a CU on the large grids:
  // 16x8 fp64 SWE 29 -> 26.6 KB, six blocks per CU instead of five).
  static_assert(4 * KG * F * EM <= F * NE, "the raw strip copy fits in the flux array");
  T (&s_raw)[4][KG][F][EM] = *reinterpret_cast<T (*)[4][KG][F][EM]>(&s_fl[0][0]);

  const int n = a.n, S = a.S, nn = n * n, mg = a.mg, pw = a.pw;
  const int nbx = (n + BX - 1) / BX, nby = (n + BY - 1) / BY;
  // bid -> (tile, yb, xb) by multiply-high with host-checked magic numbers
  // (one s_mul_hi each; the generic division is a ~50-op float-reciprocal chain)
  const int tile = a.mdiv_t ? (int)__umulhi((unsigned)bid, a.mdiv_t) : bid / (nbx * nby);
  const int rem = bid - tile * nbx * nby;
  const int yb = a.mdiv_r ? (int)__umulhi((unsigned)rem, a.mdiv_r) : rem / nbx;
  const int xb = rem - yb * nbx;
  const int x0 = xb * BX, y0 = yb * BY;
  const int tid = threadIdx.x;
  const unsigned tb = (unsigned)(tile * pw * pw);   // padded tile base
  // buffer resources of the state / geometry arrays (plain launches only; the
  // persistent kernel keeps its agent-scope atomic accesses)
  // Measured (profiles/r1_buffer_ops_ab.txt): a win for the 5- and 3-wave blocks
  // (16x8 4.76 -> 4.62 us, 8x8 4.84 -> 4.78 us per C96 stage), a 1-2 % loss for
  // 16x16 (4.64 -> 4.72 us), which keeps its global loads.
  constexpr bool BUF = !SYNC && (BX * BY < 256);
  const __amdgpu_buffer_rsrc_t rX = brsrc(a.X), rQ = brsrc(a.Q), rO = brsrc(a.out), rG = brsrc(a.cgeo);
  constexpr unsigned ES = sizeof(T);
  const int gbase = tile * nn;                 // compact geometry base
  STAMP(0);
  // direct xGMI: the block's epoch and peer masks are issued before every other
  // load, so waiting for them (vmcnt counts in issue order) never waits for the
  // prefetch below and the poll can start one round trip into the kernel
  int xe = 0, need = 0, feed = 0;
  if constexpr (XG) {
    xe = a.epoch[bid];
    need = a.bmask[2 * bid];
    feed = a.bmask[2 * bid + 1];
  }
  // panel-edge bits of the tile: a vector load (the compiler cannot prove the
  // array unwritten, so no s_load), issued before the prefetch and first used
  // after the window is loaded, so waiting for it never waits for anything
  // else.  (Read in the prologue, its vmcnt(0) held every wave for a whole
  // memory round trip before the window loads: +0.3 us per C96 stage.)
  // The lane-dependent zero (mbcnt of an empty mask) keeps the compiler from
  // treating the word as uniform: a uniform load result is moved to an SGPR
  // with v_readfirstlane right at the load, i.e. a vmcnt(0) in the prologue.
  int pe_word = 0;
  if constexpr (P != 1) pe_word = a.pedge[tile + (int)__builtin_amdgcn_mbcnt_lo(0u, 0u)];
  // Thread roles.  Waves run on SIMD (wave % 4).  256-cell blocks use the
  // ten-wave map of Geom (STSP_W10).  Otherwise edge e is thread e, and since
  // SIMD 0 carries the extra waves, the own-cell waves (prefetch, sources,
  // update, stores) are the first BX*BY/64 waves NOT on SIMD 0.  An own-cell thread puts its own cell's state
  // (which it loads anyway) into the window; every other thread loads at most
  // one cell of the NG-wide ring around the block.  Measured on C96 fp64
  // (profiles/r1_c96_stage_ab.txt): splitting the window this way instead of
  // row-major 16-byte pairs in waves 0-3 took the stage from 5.52 to 5.22 us.
  constexpr int NIN = BX * BY, RING = EX * EY - NIN, NOWN = NIN / 64;
  constexpr int NE_ = Geom<BX, BY>::NX + Geom<BX, BY>::NY;
  static_assert(NIN % 64 == 0, "own cells fill whole waves");
  static_assert(RING <= NT - NIN, "one ring cell per thread without an own cell");
  const int wv = tid >> 6;
  int oid, rid, eid;    // own-cell slot, ring slot (RING: none), edge (NE_: none)
  int eslot = -1;       // flux slot of this wave (ten-wave map)
  if constexpr (Geom<BX, BY>::W10) {
    const int lane = tid & 63;
    const unsigned os = (unsigned)(Geom<BX, BY>::OWN_TAB >> (4 * wv)) & 15u;
    const unsigned fs = (unsigned)(Geom<BX, BY>::FLUX_TAB >> (4 * wv)) & 15u;
    const unsigned rs = (unsigned)(Geom<BX, BY>::RING_TAB >> (4 * wv)) & 15u;
    oid = os != 15u ? (int)os * 64 + lane : -1;
    eid = fs != 15u ? (int)fs * 64 + lane : NE_;
    if constexpr (PEW) {
      if (pew) eid = fs != 15u ? edge_of_slot<BX, BY>((int)fs, lane) : NE_;
    }
    rid = rs != 15u ? (int)rs * 64 + lane : RING;
    eslot = (int)fs;
  } else {
    static_assert(Geom<BX, BY>::W10 || NOWN <= NT / 64 - (NT / 64 + 3) / 4, "enough waves off SIMD 0");
#if STSP_OWN_SKIP0
    const int below = wv - (wv + 3) / 4;          // waves < wv that are not on SIMD 0
    oid = ((wv & 3) != 0 && below < NOWN) ? below * 64 + (tid & 63) : -1;
#else
    const int below = wv;                         // own cells in waves 0 .. NOWN-1
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
    if (r < 2 * NG * EX) {          // NG rows above and below
      const int rr = r / EX;
      wlx = r - rr * EX;
      wly = rr < NG ? rr : EY - 2 * NG + rr;
    } else if (r < RING) {          // NG columns left and right
      const int r2 = r - 2 * NG * EX, rr = r2 / (2 * NG), c = r2 - rr * (2 * NG);
      wly = NG + rr;
      wlx = c < NG ? c : EX - 2 * NG + c;
    }
  }
  // ghost-map entry of this thread's window cell when it lies in a ghost strip
  // (the map is static: issued now, it is back by the time the poll is done
  // instead of costing its own round trip in the window phase)
  int wgm = 0;
  if constexpr (REMOTE || XG) {
    if (wly >= 0) {
      const int ly = wly, lx = wlx;
      const int x = x0 + lx - NG, y = y0 + ly - NG;
      const bool oxx = (x < 0) | (x >= n), oyy = (y < 0) | (y >= n);
      if (x < n + NG && y < n + NG && oxx != oyy) {
        int side, layer, pos;
        if (x < 0) { side = 0; layer = -1 - x; pos = y; }
        else if (x >= n) { side = 1; layer = x - n; pos = y; }
        else if (y < 0) { side = 2; layer = -1 - y; pos = x; }
        else { side = 3; layer = y - n; pos = x; }
        wgm = a.gmap[((tile * 4 + side) * mg + layer) * n + pos];
      } else if (x < n + NG && y < n + NG && oxx && a.cgmap) {   // a tile-corner ghost: carried ones may be remote
        const int ca = y < 0 ? -1 - y : y - n, cb = x < 0 ? -1 - x : x - n;
        if (ca < mg && cb < mg)
          wgm = a.cgmap[(((tile * 4 + (x >= n ? 1 : 0) + (y >= n ? 2 : 0)) * mg + ca) * mg + cb)];
      }
    }
  }

  // ---- 0. issue every per-thread operand load up front ------------------------
  // (a) own cell (threads < BX*BY)
  const int ox = oid % BX, oy = oid / BX;
  const int cx = x0 + ox, cy = y0 + oy;
  const bool own = (oid >= 0) && (cx < n) && (cy < n);
  const unsigned pc = tb + (unsigned)((cy + mg) * pw + (cx + mg));
  const unsigned gc = (unsigned)(gbase + cy * n + cx);
  T xs[F], acs[F];
  T qo[F];                // own conserved state: from global, not kept in LDS
  T iA = T(0), r0 = T(0), r1 = T(0), r2 = T(0);
  T gb[3] = {T(0), T(0), T(0)};
  int pt[4] = {-1, -1, -1, -1};
  const bool need_x = (a.a0 != T(0)) || (a.acc_out && a.c1 != T(0));
  const bool need_acc = a.acc_out && a.acc_in && (a.c0 != T(0));
  if (own) {
    if (need_x) {
#pragma unroll
      for (int f = 0; f < F; ++f) {
        if constexpr (!BUF) xs[f] = ld_state<SYNC>(o32(a.X + f * S, pc));
        else xs[f] = bld<T>(rX, pc * ES, (unsigned)(f * S) * ES);
      }
    }
#pragma unroll
    for (int f = 0; f < F; ++f) {
      if constexpr (!BUF) qo[f] = ld_state<SYNC>(o32(a.Q + f * S, pc));
      else qo[f] = bld<T>(rQ, pc * ES, (unsigned)(f * S) * ES);
    }
    if (need_acc) {
#pragma unroll
      for (int f = 0; f < F; ++f) acs[f] = ld_state<SYNC>(o32(a.acc_in + f * S, pc));
    }
    if constexpr (P == 2) {
      T rec[8];
      if constexpr (BUF) bld_rec8<T>(rG, gc * 8u * ES, rec);
      else load_rec8<T>(o32(a.cgeo, gc * 8u), rec);
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
    // a cell of a tile-corner block may also feed a carried corner ghost
    // (layout: only when n >= 2 mg, so its x push on the far side is unused)
    if (a.cpush && (cx < mg || cx >= n - mg) && (cy < mg || cy >= n - mg)) {
      const int qx = cx < mg ? 0 : 1, qy = cy < mg ? 0 : 1;
      const int cb = qx ? n - 1 - cx : cx, ca = qy ? n - 1 - cy : cy;
      const int v = *o32(a.cpush, (unsigned)(((tile * 4 + (qx | (qy << 1))) * mg + ca) * mg + cb));
      if (v != -1) pt[qx ^ 1] = v;
    }
  }
  // edge normals of this block's columns / rows: into a register now, into LDS
  // only after the window loads are issued (an LDS store of a global load makes
  // the wave wait for it, and vmcnt waits are in order: storing here would put a
  // whole memory round trip in front of the window load)
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
  // (b) this thread's edge (threads < NX: x-edge, NX <= tid < NX+NY: y-edge)
  const bool is_x = eid < NX;
  const int ete = is_x ? eid : eid - NX;
  const int e_r = is_x ? ete / (BX + 1) : ete / BX;       // edge row (x) / row index (y)
  const int e_c = is_x ? ete - e_r * (BX + 1) : ete - e_r * BX;
  const int ex_ = x0 + e_c, ey_ = y0 + e_r;
  const bool edge_ok = is_x ? (ex_ <= n && ey_ < n) : (eid < NX + NY && ex_ < n && ey_ <= n);
  T coef = T(0);
  if (edge_ok) {
    coef = is_x ? *o32(a.ex, (unsigned)(tile * n * (n + 1) + ey_ * (n + 1) + ex_))
                : *o32(a.ey, (unsigned)(tile * (n + 1) * n + ey_ * n + ex_));
  }
  // (c) panel edges (models/base.py::reconstruct).  bsides: the sides of this
  // block that lie on a cube edge (block-uniform).  Fix-up thread tid < 4 BM F
  // owns field pf of strip cell pjl of side pside: it interpolates that cell's
  // ghost layers along the neighbour's grid lines and reconstructs the
  // neighbour's edge state in the neighbour's frame (one field per thread, so
  // the F fields run on F waves / SIMDs side by side).  Its table entries are
  // issued here.
  // sides of this block on a cube edge; evaluated where first needed (after the window).
  // A side counts as soon as the block's window reaches that side's ghost strip:
  // also the last-but-one block of a tile whose last block is 1 (PLR) or 1-2
  // (PPM) cells wide, whose outer faces reconstruct a cell next to the ghost
  // (found by the streaming stage's odd-size tests: C25 with 8 x 8 blocks was
  // 4.8e-2 off the oracle)
  auto block_sides = [&]() {
    if constexpr (RECON)
      return (x0 == 0 ? (pe_word & 1) : 0) | (x0 + BX + NG > n ? (pe_word & 2) : 0) | (y0 == 0 ? (pe_word & 4) : 0) |
             (y0 + BY + NG > n ? (pe_word & 8) : 0);
    else
      return 0;
  };
  constexpr int NPF = RECON ? 4 * BM * F : 0;
  static_assert(NPF <= NT, "one fix-up thread per (side, strip cell, field)");
  int pf, pslt, pside, pjl;
  bool pown;
  if (pew) {
    // border wave of slot PEW_SX: sides W, E; of slot PEW_SY: sides S, N.
    // lane = side bit (5) | strip cell (4..1) | field pair (0): fields pf, pf + 1
    const int lane = tid & 63;
    pside = (eslot == PEW_SY ? 2 : 0) + (lane >> 5);
    pjl = (lane >> 1) & (BM - 1);
    pf = F == 4 ? 2 * (lane & 1) : 0;
    pown = (eslot == PEW_SX || eslot == PEW_SY) && (F == 4 || (lane & 1) == 0);
  } else {
    pf = tid / (4 * BM);
    pown = tid < NPF;
    pside = (tid - pf * (4 * BM)) / BM;
    pjl = tid - pf * (4 * BM) - pside * BM;
  }
  pslt = pside * BM + pjl;
  const int pj = (pside < 2 ? y0 : x0) + pjl;           // strip cell (tile-local, along the side)
  const bool pin = RECON && pown && pjl < (pside < 2 ? BY : BX) && pj < n;   // a strip cell of this tile
  int pb[KG];
  T pt_[KG];
  // (issued for every tile side, not only panel edges: the tables cover all
  // four sides, and the loads then need not wait for the pedge word).  The
  // blocks that run several per CU (all but the 640-thread 16x16 map) load
  // them after the window instead: held across the window phase they cost
  // three VGPRs there, which is what decides the waves per SIMD.
  constexpr bool LATE_TAB = !Geom<BX, BY>::W10;
  auto load_tab = [&]() {
    if (pin) {
#pragma unroll
      for (int k = 0; k < KG; ++k) {
        const unsigned ti = (unsigned)(((tile * 4 + pside) * 3 + k) * n + pj);
        pb[k] = *o32(a.pe_base, ti);
        pt_[k] = *o32(a.pe_t, ti);
      }
    }
  };
  if constexpr (!LATE_TAB) load_tab();
  STAMP(1);

  // ---- 0b. direct xGMI: wait for the peers whose ghosts this block reads ------
  bool rblk = REMOTE;
  const T* rring = a.recv;
  if constexpr (XG) {
    rblk = need != 0;
    rring = a.recv + (long)(xe % STSP_XG_SLOTS) * a.ring;   // tags: a.ring counts 8-byte granules, see below
    if (!STSP_XG_TAG && rblk) {
      if (tid < 32 && ((need >> tid) & 1)) {
        const unsigned long long want = (unsigned long long)xe * a.nprod[tid];
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load((gu64*)(a.cnt + tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
          if (__hip_atomic_load((gu32*)a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
          if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
            __hip_atomic_store((gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
    }
  }

  // ---- 1. window (block + NG halo) -> LDS --------------------------------------
  // Own-cell threads store the state they prefetched, the ring threads load one
  // cell each (a remote ghost from the receive ring).
  auto put = [&](int ly, int lx, const T (&v)[F]) {
    if constexpr (P == 2) {  // primitive (h, v) + sqrt(g h)
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
  // one window cell: zero past a partial block, a remote ghost from the
  // receive ring, anything else from the padded state
  auto load_win = [&](int ly, int lx, T (&v)[F]) {
    const int x = x0 + lx - NG, y = y0 + ly - NG;
#pragma unroll
    for (int f = 0; f < F; ++f) v[f] = T(0);
    if (x < n + NG && y < n + NG) {          // false only past a partial block
      const unsigned pa = tb + (unsigned)((y + mg) * pw + (x + mg));
      bool from_recv = false;
      if constexpr (REMOTE || XG) {
        if (rblk) {
          const int m = wgm;   // < 0: remote slot -1 - m (0 outside the ghost strips)
          if (m < 0) {
            from_recv = true;
            if constexpr (XG && STSP_XG_TAG) {
              // spin on this cell's granules until all carry this stage's tag
              constexpr int G = sizeof(T) / 4;
              const gu64* rp = ((const gu64*)(a.recv)) + (long)(xe % STSP_XG_SLOTS) * a.ring;
              const int nrec = a.ring / (F * G), rec = -1 - m;
              const unsigned want = (unsigned)xe + 1u;
              unsigned long long gr[F * G];
              const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
              for (;;) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < F * G; ++k) {
                  gr[k] = __hip_atomic_load(rp + ring_word(nrec, F * G, rec, k), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
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
              for (int f = 0; f < F; ++f) {
                if constexpr (G == 2)
                  v[f] = __builtin_bit_cast(T, (gr[2 * f + 1] << 32) | (gr[2 * f] & 0xFFFFFFFFull));
                else
                  v[f] = __builtin_bit_cast(T, (unsigned)gr[f]);
              }
            } else if constexpr (XG) {
              const int nrec = a.ring / F;
#pragma unroll
              for (int f = 0; f < F; ++f) v[f] = ld_sys(rring + ring_word(nrec, F, -1 - m, f));
            } else {
              const T* rp = rring + (long)(-1 - m) * F;
#pragma unroll
              for (int f = 0; f < F; ++f) v[f] = ld_state<SYNC>(rp + f);
            }
          }
        }
      }
      if (!from_recv) {
#pragma unroll
        for (int f = 0; f < F; ++f) {
          if constexpr (!BUF) v[f] = ld_state<SYNC>(o32(a.Q + f * S, pa));
          else v[f] = bld<T>(rQ, pa * ES, (unsigned)(f * S) * ES);
        }
      }
    }
  };
  if (wly >= 0) {
    T v[F];
    if (own) {
#pragma unroll
      for (int f = 0; f < F; ++f) v[f] = qo[f];
    } else {
      load_win(wly, wlx, v);
    }
    put(wly, wlx, v);
    if constexpr (RECON) {
      const int bsides = block_sides();
      if (bsides && !own && !pew) {  // a raw panel-edge ghost the fix-up interpolates from
        const int x = x0 + wlx - NG, y = y0 + wly - NG;
        const bool inx = (x >= 0) & (x < n), iny = (y >= 0) & (y < n);
        // strip cells, and the tile-corner cells beyond the strip ends (carried
        // corner ghosts, read by the interpolation pairs of the end cells):
        // filed under the side that is a panel edge
        int side = -1, k = 0, al = 0;
        if (!inx) {
          side = x < 0 ? 0 : 1; k = x < 0 ? -1 - x : x - n; al = wly;
          if (!(k < KG && ((bsides >> side) & 1))) side = -1;
        }
        if (side < 0 && !iny) { side = y < 0 ? 2 : 3; k = y < 0 ? -1 - y : y - n; al = wlx; }
        if (side >= 0 && k < KG && ((bsides >> side) & 1)) {
#pragma unroll
          for (int f = 0; f < F; ++f) s_raw[side][k][f][al] = s_w[f][wly][wlx];   // primitives, as put() stored them
        }
      }
    }
  }
  if constexpr (P == 2) {
    if (tid < 3 * (BX + 1)) {
      const int k = tid / (BX + 1), c = tid - k * (BX + 1);
      s_nrm[k][c] = nrm;
    } else if (tid < 3 * (BX + 1) + 3 * (BY + 1)) {
      const int u = tid - 3 * (BX + 1);
      const int k = u / (BY + 1), c = u - k * (BY + 1);
      s_nrm[k][BX + 1 + c] = nrm;
    }
    if (edge_ok) s_len[eid] = coef;   // edge lengths for the curvature balance (phase 2b)
  }
  STAMP(2);
  __syncthreads();
  STAMP(3);

  // ---- 1a. panel edges: interpolated ghosts + the neighbour's edge state ------
  // Ghost layer k of a panel-edge strip holds the neighbour's cells on ITS grid
  // lines (index-space copy); this panel's grid lines cross into the neighbour
  // elsewhere (beta' = atan(tan beta / tan(pi/4 + delta_k)), pulled toward the
  // edge middle).  The ghosts the faces read are replaced by x[b] + t (x[b+1] -
  // x[b]) along the strip; the neighbour's state at the edge is reconstructed
  // from [our cells interpolated at its grid line | its raw cells], exactly as
  // the neighbour block computes it, so the edge flux is single-valued.
  // fix-up of field f for strip cell pj of side pside.  PEW reads the raw
  // ghosts straight from the window (the lanes that replace them are the
  // lanes of this wave, and all reads come first); the block-wide path reads
  // them from s_raw
  const bool plow = (pside & 1) == 0;
  auto widx = [&](int cn, int al) {  // window index of (normal coord, along coord), tile-local
    const int x = pside < 2 ? cn : al, y = pside < 2 ? al : cn;
    return (y - y0 + NG) * WS + (x - x0 + NG);
  };
  const int pab = (pside < 2 ? y0 : x0) - NG;           // tile-local coordinate of window position 0
  auto fix_read = [&](int f, T (&gk)[KG], T& nf, T& c) {
    const T* wf = &s_w[f][0][0];
    T gp[KG];
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int cg = plow ? -1 - k : n + k;
      T g0, g1;
      if (pew) {
        g0 = wf[widx(cg, pb[k])];
        g1 = wf[widx(cg, pb[k] + 1)];
      } else {
        g0 = s_raw[pside][k][f][pb[k] - pab];
        g1 = s_raw[pside][k][f][pb[k] + 1 - pab];
      }
      gk[k] = g0 + pt_[k] * (g1 - g0);
      const int co = plow ? k : n - 1 - k;
      const T o0 = wf[widx(co, pb[k])], o1 = wf[widx(co, pb[k] + 1)];
      gp[k] = o0 + pt_[k] * (o1 - o0);
    }
    if (pew) c = wf[widx(plow ? -1 : n, pj)];
    else c = s_raw[pside][0][f][pj - pab];
    T r;
    if constexpr (KG > 1) r = s_raw[pside][KG - 1][f][pj - pab];   // raw layer 1 (replaced in the window)
    else r = wf[widx(plow ? -2 : n + 1, pj)];
    const T l = gp[0];
    if constexpr (LIM == 4) {
      const T l2 = gp[KG - 1], r2 = wf[widx(plow ? -3 : n + 2, pj)];
      const T aL = T(7.0 / 12.0) * (l + c) - T(1.0 / 12.0) * (l2 + r);
      const T aR = T(7.0 / 12.0) * (c + r) - T(1.0 / 12.0) * (l + r2);
      const bool flat = (aR - c) * (c - aL) <= T(0);
      const T d = aR - aL;
      const T m6 = T(6) * (c - T(0.5) * (aL + aR));
      const bool ovl = d * m6 > d * d;
      nf = flat ? c : (ovl ? T(3) * c - T(2) * aR : aL);
    } else {
      nf = c - half_slope<LIM>(c - l, r - c);
    }
  };
  auto fix_write = [&](int f, const T (&gk)[KG], T nf, T c) {
    T* wm = &s_w[f][0][0];
    const int wend = (pside < 2 ? x0 + BX : y0 + BY) + NG;   // first coordinate past the window
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      if (plow || n + k < wend) wm[widx(plow ? -1 - k : n + k, pj)] = gk[k];
    }
    s_pf[f][pslt] = nf;
    if constexpr (SW) s_pr[f][pslt] = c;
  };
  auto fix_sound = [&]() {   // raw sound speed of the neighbour cell (never replaced)
    if constexpr (SW) s_pr[FL - 1][pslt] = (&s_w[FL - 1][0][0])[widx(plow ? -1 : n, pj)];
  };
  const int bsides = block_sides();
  const bool pact = pin && ((bsides >> pside) & 1);
  if constexpr (RECON) {
    if (bsides && !pew) {              // block-uniform
      if constexpr (LATE_TAB) {
        if (pact) load_tab();
      }
      if (pact) {
        T gk[KG], nf, c;
        fix_read(pf, gk, nf, c);
        fix_write(pf, gk, nf, c);
        if (pf == 0) fix_sound();
      }
      STAMP(11);
      __syncthreads();
    }
  }

  // ---- 1b. PLR face values, one (cell, direction) per thread -------------------
  // task t < NFX: x-direction, cell (x0 + c - 1, y0 + r), t = r (BX + 2) + c;
  // else y-direction, cell (x0 + c, y0 + r - 1), t - NFX = r BX + c.
  if constexpr (FACES) {
    const T* w0 = &s_w[0][0][0];
    // (panel-edge ghosts are already interpolated in the window: no fallback)
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
          if constexpr (LIM == 4) {
            // PPM (models/base.py::ppm_faces): 4th-order interface values,
            // Colella-Woodward monotonicity limiter
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
  STAMP(4);

  // ---- 2. one edge flux per thread (edge id eid: x-edges, then y-edges) --------
  // x-edge (e_r, e_c) lies between cells e_c - 1 and e_c of row e_r (face tasks
  // e_r (BX + 2) + e_c and + 1); y-edge (e_r, e_c) between rows e_r - 1 and e_r
  // (face tasks NFX + e_r BX + e_c and + BX).
  if constexpr (PEW) {
    if (pew && bsides && (eslot == PEW_SX || eslot == PEW_SY)) {   // the border-edge waves (wave-uniform)
      if (pact) {
        constexpr int NF = F == 4 ? 2 : 1;
        T gk[NF][KG], nf[NF], c[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) fix_read(pf + i, gk[i], nf[i], c[i]);   // every read first
#pragma unroll
        for (int i = 0; i < NF; ++i) fix_write(pf + i, gk[i], nf[i], c[i]);
        if (pf == 0) fix_sound();
      }
      // LDS operations of one wave complete in order: the flux reads below see
      // the writes above (the wave barrier only keeps the compiler from moving
      // them across)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      STAMP(11);
    }
  }
  // the edge thread of a panel-edge edge takes the neighbour's state from the
  // fix-up slot pslot (the neighbour is on the left of the edge when plo)
  int pslot = -1;
  bool plo = false;
  if (RECON && bsides && edge_ok) {
    if (is_x && ex_ == 0 && (bsides & 1)) { pslot = 0 * BM + ey_ - y0; plo = true; }
    else if (is_x && ex_ == n && (bsides & 2)) { pslot = 1 * BM + ey_ - y0; }
    else if (!is_x && ey_ == 0 && (bsides & 4)) { pslot = 2 * BM + ex_ - x0; plo = true; }
    else if (!is_x && ey_ == n && (bsides & 8)) { pslot = 3 * BM + ex_ - x0; }
  }
  if (edge_ok) {
    const int fl_ = is_x ? e_r * (BX + 2) + e_c : NFX + e_r * BX + e_c;   // face task of the left cell
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
      if (pslot >= 0) {
        if (plo) wl = s_pf[0][pslot];
        else wr = s_pf[0][pslot];
      }
      s_fl[0][eid] = coef * (coef > T(0) ? wl : wr);
    } else {
      T wl[4], wr[4], cl[5], cr[5];
#pragma unroll
      for (int f = 0; f < 5; ++f) { cl[f] = w0[f * WF + cl_]; cr[f] = w0[f * WF + cl_ + cst]; }
      if constexpr (FUSED) {
        // + face of the left cell and - face of the right cell (same arithmetic
        // as the face phase: c0 +- 0.5 slope)
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
      if (pslot >= 0) {   // panel edge: the neighbour's state and raw cell
        if (plo) {
#pragma unroll
          for (int f = 0; f < 4; ++f) wl[f] = s_pf[f][pslot];
#pragma unroll
          for (int f = 0; f < 5; ++f) cl[f] = s_pr[f][pslot];
        } else {
#pragma unroll
          for (int f = 0; f < 4; ++f) wr[f] = s_pf[f][pslot];
#pragma unroll
          for (int f = 0; f < 5; ++f) cr[f] = s_pr[f][pslot];
        }
      }
      const int ni = is_x ? e_c : BX + 1 + e_r;
      T fl[4];
      swe_flux<T>(wl, wr, cl, cr, s_nrm[0][ni], s_nrm[1][ni], s_nrm[2][ni], coef, a.g, fl);
#pragma unroll
      for (int f = 0; f < 4; ++f) s_fl[f][eid] = fl[f];
    }
  }
  // ---- 2b. own-cell terms that need no flux: sources and the RK base ----------
  // Done before the barrier: the own-cell waves finish their edges well before
  // the SIMD that runs the ninth (partial) flux wave, so this is off the
  // critical path instead of in front of the stores.
  const int ew = oy * (BX + 1) + ox;            // west x-edge of the cell
  const int es = NX + oy * BX + ox;             // south y-edge
  T qs[F], base[F];
  T src[3] = {T(0), T(0), T(0)};
  if (own) {
    if constexpr (P == 2) {
#pragma unroll
      for (int f = 0; f < 4; ++f) qs[f] = qo[f];
      const T fc = a.omega2 * r2;
      const T h = qs[0];
      const T cor[3] = {r1 * qs[3] - r2 * qs[2], r2 * qs[1] - r0 * qs[3], r0 * qs[2] - r1 * qs[1]};
      // curvature balance g/2 h^2 sum(+-L m)/A: a constant depth is force-free
      const T Lw = s_len[ew], Le = s_len[ew + 1], Ls = s_len[es], Ln = s_len[es + BX];
      const T pb = T(0.5) * a.g * h * h * iA, gh = a.g * h;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const T Sk = Le * s_nrm[k][ox + 1] - Lw * s_nrm[k][ox] + Ln * s_nrm[k][BX + 2 + oy] - Ls * s_nrm[k][BX + 1 + oy];
        src[k] = -fc * cor[k] + pb * Sk - gh * gb[k];
      }
    } else {
      qs[0] = s_w[0][NG + oy][NG + ox];
    }
#pragma unroll
    for (int f = 0; f < F; ++f) {
      base[f] = T(0);
      if (a.a1 != T(0)) base[f] = a.a1 * qs[f];
      if (a.a0 != T(0)) base[f] += a.a0 * xs[f];
    }
  }
  STAMP(5);
  __syncthreads();
  STAMP(7);

  // ---- 3. divergence + RK combination + push -----------------------------------
  if (own) {
    T dq[F];
#pragma unroll
    for (int f = 0; f < F; ++f)
      dq[f] = -((s_fl[f][ew + 1] - s_fl[f][ew]) + (s_fl[f][es + BX] - s_fl[f][es])) * iA;
    if constexpr (P == 2) {
#pragma unroll
      for (int k = 0; k < 3; ++k) dq[1 + k] += src[k];
    }
    T o[F];
#pragma unroll
    for (int f = 0; f < F; ++f) o[f] = a.a2 * a.dt * dq[f] + base[f];
    if constexpr (P == 2) {
      const T d = o[1] * r0 + o[2] * r1 + o[3] * r2;
      o[1] -= d * r0; o[2] -= d * r1; o[3] -= d * r2;
    }
    if (a.acc_out) {
      T p[F];
#pragma unroll
      for (int f = 0; f < F; ++f) p[f] = a.c2 * a.dt * dq[f];
      if (a.c1 != T(0)) {
#pragma unroll
        for (int f = 0; f < F; ++f) p[f] += a.c1 * xs[f];
      }
      if (need_acc) {
#pragma unroll
        for (int f = 0; f < F; ++f) p[f] += a.c0 * acs[f];
      }
      if constexpr (P == 2) {
        const T d = p[1] * r0 + p[2] * r1 + p[3] * r2;
        p[1] -= d * r0; p[2] -= d * r1; p[3] -= d * r2;
      }
#pragma unroll
      for (int f = 0; f < F; ++f) st_out<SYNC>(a.wt, o32(a.acc_out + f * S, pc), p[f]);
    }
    // state stores (write-through when a.wt, see st_out)
    auto put_out = [&](unsigned idx, const T (&v)[F]) {
      if constexpr (!BUF) {
#pragma unroll
        for (int f = 0; f < F; ++f) st_out<SYNC>(a.wt, o32(a.out + f * S, idx), v[f]);
      } else if (a.wt) {
#pragma unroll
        for (int f = 0; f < F; ++f) bst<16>(v[f], rO, idx * ES, (unsigned)(f * S) * ES);
      } else {
#pragma unroll
        for (int f = 0; f < F; ++f) bst<0>(v[f], rO, idx * ES, (unsigned)(f * S) * ES);
      }
    };
    STAMP(8);
    put_out(pc, o);
    STAMP(9);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (pt[k] >= 0) put_out((unsigned)pt[k], o);
    }
    STAMP(10);
    if constexpr (XG) {   // remote ghosts: straight into the consumer's ring
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (pt[k] < -1) {
          const int code = -2 - pt[k];
          if constexpr (STSP_XG_TAG) {
            constexpr int G = sizeof(T) / 4;
            gu64* dst = ((gu64*)(a.peer_ring[code >> 24])) + (long)((xe + 1) % STSP_XG_SLOTS) * a.ring;
            const int nrec = a.ring / (F * G), rec = code & 0xFFFFFF;
            const unsigned long long tag = (unsigned long long)((unsigned)xe + 2u) << 32;
#pragma unroll
            for (int f = 0; f < F; ++f) {
              if constexpr (G == 2) {
                const unsigned long long b = __builtin_bit_cast(unsigned long long, o[f]);
                __hip_atomic_store(dst + ring_word(nrec, F * G, rec, 2 * f), tag | (b & 0xFFFFFFFFull),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(dst + ring_word(nrec, F * G, rec, 2 * f + 1), tag | (b >> 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
              } else {
                __hip_atomic_store(dst + ring_word(nrec, F, rec, f), tag | __builtin_bit_cast(unsigned, o[f]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              }
            }
          } else {
            T* dst = a.peer_ring[code >> 24] + (long)((xe + 1) % STSP_XG_SLOTS) * a.ring;
            const int nrec = a.ring / F, rec = code & 0xFFFFFF;
#pragma unroll
            for (int f = 0; f < F; ++f) st_sys(dst + ring_word(nrec, F, rec, f), o[f]);
          }
        }
      }
    }
  }
  if constexpr (XG) {
    if (!STSP_XG_TAG && feed) {   // publish: every storing wave drains, then one lane per peer counts
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid < 32 && ((feed >> tid) & 1))
        __hip_atomic_fetch_add((gu64*)a.peer_cnt[tid], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tid == 0) a.epoch[bid] = xe + 1;
  }
  STAMP(6);
}


// Waves per SIMD: the large grids run several blocks per CU, and the VGPR
// count decides how many (512 / ceil8(vgprs) waves per SIMD).  The panel-edge
// treatment took the fp64 16x8 / 8x8 bodies from 93 to 100 VGPRs, i.e. from 5
// to 4 waves per SIMD (C180 stage 11.0 -> 15.1 us even without panel edges,
// C720 143 -> 169 us); asking for 5 keeps them at <= 96.  The 640-thread
// 16x16 blocks run one per CU at C96 and are left alone.
#ifndef STSP_WPE
#define STSP_WPE 5
#endif
template <int BX, int BY> struct StageOcc { static constexpr int WPE = Geom<BX, BY>::W10 ? 1 : STSP_WPE; };

template <typename T, int P, int BX, int BY, int LIM, bool REMOTE, bool LIST, bool XG>
__global__ __launch_bounds__((Geom<BX, BY>::NT)) __attribute__((amdgpu_waves_per_eu(StageOcc<BX, BY>::WPE)))
void stage_kernel(Args<T> a) {
  pin_args(a);
  const int bid = LIST ? a.blocks[blockIdx.x] : xcd_remap(blockIdx.x, a.nblocks);
  stage_body<T, P, BX, BY, LIM, REMOTE, false, XG>(a, bid);
#ifdef STSP_STAMPS
  // warm-instruction-cache experiment: repeat the (idempotent, for stages
  // without an in-place accumulator) body; the stamps keep the last pass
  for (int r = 0; r < a.diag_repeat; ++r) {
    __syncthreads();
    stage_body<T, P, BX, BY, LIM, REMOTE, false, XG>(a, bid);
  }
#endif
}

template <typename T, int P, int BX, int BY, int LIM>
int launch_l(const StageDesc* d, hipStream_t s) {
  Args<T> a = make_args<T>(d);
  set_magic<T, BX, BY>(a);
  a.wt = want_wt((long)d->nblocks * BX * BY) ? 1 : 0;
  a.pew = (d->n % BX == 0 && d->n % BY == 0) ? 1 : 0;   // partial blocks: the block-wide fix-up
#ifdef STSP_STAMPS
  const char* rp = std::getenv("STSP_DIAG_REPEAT");
  a.diag_repeat = rp ? std::atoi(rp) : 0;
#endif
  constexpr int NT = Geom<BX, BY>::NT;
  const dim3 grid(d->nblocks), block(NT);
  if (d->xg)
    hipLaunchKernelGGL((stage_kernel<T, P, BX, BY, LIM, false, false, true>), grid, block, 0, s, a);
  else if (d->remote)
    hipLaunchKernelGGL((stage_kernel<T, P, BX, BY, LIM, true, true, false>), grid, block, 0, s, a);
  else if (d->blocks)
    hipLaunchKernelGGL((stage_kernel<T, P, BX, BY, LIM, false, true, false>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((stage_kernel<T, P, BX, BY, LIM, false, false, false>), grid, block, 0, s, a);
  return (int)hipGetLastError();
}

template <typename T, int P, int BX, int BY>
int launch_t(const StageDesc* d, hipStream_t s) {
  if (d->nblocks <= 0) return 0;
  if (d->pw != d->n + 2 * d->mg || d->mg < Phys<P>::NG || (d->limiter == 4 && d->mg < 3)) return -5;
  if (P != 1 && (!d->pedge || !d->pe_base || !d->pe_t || d->n < 2)) return -12;   // panel-edge tables
  if (!d->push || (d->remote && (!d->gmap || !d->blocks))) return -6;
  if (d->xg && (d->remote || d->blocks || !d->gmap || !d->recv || !d->peer_ring || !d->peer_cnt || !d->cnt ||
                !d->nprod || !d->bmask || !d->epoch || !d->err || d->ring <= 0))
    return -10;
  if constexpr (P == 1) return launch_l<T, P, BX, BY, 0>(d, s);  // diffusion: no reconstruction
  switch (d->limiter) {
    case 0: return launch_l<T, P, BX, BY, 0>(d, s);
    case 1: return launch_l<T, P, BX, BY, 1>(d, s);
    case 2: return launch_l<T, P, BX, BY, 2>(d, s);
    case 3: return launch_l<T, P, BX, BY, 3>(d, s);
    case 4:   // PPM: the 3-layer window must fit one cell per thread
      if constexpr ((BX + 6) * (BY + 6) <= Geom<BX, BY>::NT) return launch_l<T, P, BX, BY, 4>(d, s);
      else return -11;
  }
  return -7;
}

template <typename T, int P>
int launch_p(int bx, int by, const StageDesc* d, hipStream_t s) {
  if (bx == 16 && by == 16) return launch_t<T, P, 16, 16>(d, s);
  if (bx == 32 && by == 8) return launch_t<T, P, 32, 8>(d, s);
  if (bx == 16 && by == 8) return launch_t<T, P, 16, 8>(d, s);
  if (bx == 8 && by == 16) return launch_t<T, P, 8, 16>(d, s);
  if (bx == 8 && by == 8) return launch_t<T, P, 8, 8>(d, s);
  return -2;
}

template <typename T>
int launch_d(int phys, int bx, int by, const StageDesc* d, hipStream_t s) {
  switch (phys) {
    case 0: return launch_p<T, 0>(bx, by, d, s);
    case 1: return launch_p<T, 1>(bx, by, d, s);
    case 2: return launch_p<T, 2>(bx, by, d, s);
  }
  return -3;
}

// ---- pack: send[k][f] = q[f][idx[k]] ----------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(const T* __restrict__ q, int S, int F, const int* __restrict__ idx,
                                                   int ns, T* __restrict__ send) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ns) return;
  const int src = idx[k];
  for (int f = 0; f < F; ++f) send[(long)k * F + f] = q[(long)f * S + src];
}

// ---- direct xGMI halo: initial ghost delivery (no counter bump) -------------
// Writes the ghosts of stage `epoch`'s input: slot epoch % SLOTS, tag epoch + 1.
template <typename T>
__global__ __launch_bounds__(256) void xg_prime_kernel(const T* __restrict__ q, int S, int F,
                                                       const int* __restrict__ src, const int* __restrict__ code,
                                                       int nent, T* const* peer_ring, int ring, int epoch) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int slot = epoch % STSP_XG_SLOTS;
  if (i < nent) {
    const int c = code[i];
    if constexpr (STSP_XG_TAG) {
      constexpr int G = sizeof(T) / 4;
      gu64* dst = ((gu64*)(peer_ring[c >> 24])) + (long)slot * ring;
      const int nrec = ring / (F * G), rec = c & 0xFFFFFF;
      const unsigned long long tag = (unsigned long long)((unsigned)epoch + 1u) << 32;
      for (int f = 0; f < F; ++f) {
        const T v = q[(long)f * S + src[i]];
        if constexpr (G == 2) {
          const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
          __hip_atomic_store(dst + ring_word(nrec, F * G, rec, 2 * f), tag | (b & 0xFFFFFFFFull), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(dst + ring_word(nrec, F * G, rec, 2 * f + 1), tag | (b >> 32), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
          __hip_atomic_store(dst + ring_word(nrec, F, rec, f), tag | __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    } else {
      T* dst = peer_ring[c >> 24] + (long)slot * ring;
      const int nrec = ring / F, rec = c & 0xFFFFFF;
      for (int f = 0; f < F; ++f) st_sys(dst + ring_word(nrec, F, rec, f), q[(long)f * S + src[i]]);
    }
  }
  __threadfence_system();
}

// ---- generic indexed copy: dst[b][didx[k]] = src[b][sidx[k]] ------------------
template <typename T>
__global__ __launch_bounds__(256) void copy_index_kernel(const T* __restrict__ src, const int* __restrict__ sidx,
                                                         T* __restrict__ dst, const int* __restrict__ didx, int k,
                                                         long ss, long ds) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const int b = blockIdx.y;
  dst[b * ds + didx[i]] = src[b * ss + sidx[i]];
}

}  // namespace

extern "C" int stsp_march_launch(int dtype, int rows, const StageDesc* d, hipStream_t stream);

// bx == 64: the streaming shallow-water stage (march_kernel.hip), by = rows per wave
extern "C" int stsp_stage_launch(int phys, int dtype, int bx, int by, const StageDesc* d, hipStream_t stream) {
  if (bx == 64) return phys == 2 ? stsp_march_launch(dtype, by, d, stream) : -2;
  if (dtype == 1) return launch_d<double>(phys, bx, by, d, stream);
  if (dtype == 0) return launch_d<float>(phys, bx, by, d, stream);
  return -4;
}

extern "C" int stsp_pack_launch(int dtype, const void* q, int S, int F, const int* idx, int ns, void* send,
                                hipStream_t stream) {
  if (ns <= 0) return 0;
  const int nb = (ns + 255) / 256;
  if (dtype == 1)
    hipLaunchKernelGGL(pack_kernel<double>, dim3(nb), dim3(256), 0, stream, (const double*)q, S, F, idx, ns,
                       (double*)send);
  else
    hipLaunchKernelGGL(pack_kernel<float>, dim3(nb), dim3(256), 0, stream, (const float*)q, S, F, idx, ns,
                       (float*)send);
  return (int)hipGetLastError();
}

extern "C" int stsp_copy_index_launch(int dtype, const void* src, const int* sidx, void* dst, const int* didx, int k,
                                      int batch, long src_stride, long dst_stride, hipStream_t stream) {
  if (k <= 0 || batch <= 0) return 0;
  const dim3 grid((k + 255) / 256, batch);
  if (dtype == 1)
    hipLaunchKernelGGL(copy_index_kernel<double>, grid, dim3(256), 0, stream, (const double*)src, sidx,
                       (double*)dst, didx, k, src_stride, dst_stride);
  else
    hipLaunchKernelGGL(copy_index_kernel<float>, grid, dim3(256), 0, stream, (const float*)src, sidx, (float*)dst,
                       didx, k, src_stride, dst_stride);
  return (int)hipGetLastError();
}

extern "C" int stsp_xg_prime_launch(int dtype, const void* q, int S, int F, const int* src, const int* code, int nent,
                                    void* const* peer_ring, int ring, int epoch, hipStream_t stream) {
  if (nent <= 0) return 0;
  if (epoch < 0 || ring <= 0) return -6;
  const int nb = (nent + 255) / 256;
  if (dtype == 1)
    hipLaunchKernelGGL(xg_prime_kernel<double>, dim3(nb), dim3(256), 0, stream, (const double*)q, S, F, src, code,
                       nent, (double* const*)peer_ring, ring, epoch);
  else
    hipLaunchKernelGGL(xg_prime_kernel<float>, dim3(nb), dim3(256), 0, stream, (const float*)q, S, F, src, code,
                       nent, (float* const*)peer_ring, ring, epoch);
  return (int)hipGetLastError();
}

extern "C" int stsp_xg_protocol(void) { return STSP_XG_TAG; }
extern "C" int stsp_xg_slots(void) { return STSP_XG_SLOTS; }

// Threads per stage block as compiled (Geom<BX, BY>::NT; depends on the
// STSP_W10 build flag), so the host's block_threads() / PPM window check
// describe the kernel that actually runs.  -1: unsupported shape.
extern "C" int stsp_block_threads(int bx, int by) {
  if (bx == 16 && by == 16) return Geom<16, 16>::NT;
  if (bx == 32 && by == 8) return Geom<32, 8>::NT;
  if (bx == 16 && by == 8) return Geom<16, 8>::NT;
  if (bx == 8 && by == 16) return Geom<8, 16>::NT;
  if (bx == 8 && by == 8) return Geom<8, 8>::NT;
  return -1;
}
