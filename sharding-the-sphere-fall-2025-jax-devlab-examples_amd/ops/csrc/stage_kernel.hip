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
#include "stsp_kernels.h"

// Publish protocol of the arrival-counter hand-off (STSP_XG_TAG=0 below; probe
// variants, tools/xg_fence_probe.py, profiles/r1_xg_fence_probe.jsonl; loopback
// C96 µs/step, plain step 17.1):
//   0 = __threadfence_system() + release add: 117.5 (the fence is seq_cst, so
//       every wave also invalidates L2 and the whole grid re-reads from HBM)
//   1 = release add only (one L2 write-back per producing block): 28.6  <- default
//   2 = relaxed add after the storing waves drain: 26.8 (relies on the ring
//       stores being system-scope write-through; not a release in the model)
#ifndef STSP_XG_FENCE
#define STSP_XG_FENCE 1
#endif
// Halo hand-off form (stsp_kernels.h, xg fields):
//   0 = arrival counters (drain + release add per producing block, block-level poll)
//   1 = tagged granules: the data is the flag.  Each 32-bit word of a ghost cell
//       travels as ONE 8-byte {tag = stage epoch + 1, payload} relaxed system-scope
//       atomic store (single-copy atomic, so never torn); the consumer thread
//       re-reads its cell's granules until every tag matches.  The producer
//       neither drains nor signals, and the consumer skips the separate poll
//       round trip (cdna_hip_programming.md Guideline 16, R2).
//   Measured (tools/xg_tag_round.sh, profiles/r1_xg_tag_probe.jsonl, C96 fp64 µs/step):
//   loopback 28.9 (counters) -> 24.9 (tags); two ranks sharing one GPU 26.9 -> 21.8.
#ifndef STSP_XG_TAG
#define STSP_XG_TAG 1
#endif
// Ring slots.  A rank reads slot e % S during its stage e while a peer writes
// slot (e_p + 1) % S during its stage e_p.  A peer can have STARTED at most two
// stages past us: its stage e + 2 needs its stage e + 1 complete, which waited
// for our stage-e output, i.e. our stage e started and e - 1 completed.  So the
// peer writes slot (e + 1 .. e + 3) % S, never e % S, iff S does not divide 1,
// 2 or 3: S = 4 (three slots left a window where a peer two stages ahead
// overwrote the slot a slow block of ours was still reading).
#define STSP_XG_SLOTS 4
// Own-cell waves: 1 = the first waves not on SIMD 0, 0 = waves 0 .. n-1.
#ifndef STSP_OWN_SKIP0
#define STSP_OWN_SKIP0 1
#endif
// Face reconstruction fused into the flux phase for PLR (stage_body phase 2):
// 1 = each edge thread computes its two faces from the window; 0 = separate
// face phase through LDS (always for PPM).
#ifndef STSP_FUSE_FACES
#define STSP_FUSE_FACES 1
#endif

#include <cstdlib>
#include <type_traits>

namespace {

template <int P> struct Phys;
template <> struct Phys<0> { static constexpr int F = 1, NG = 2, FL = 1; };
template <> struct Phys<1> { static constexpr int F = 1, NG = 1, FL = 1; };
template <> struct Phys<2> { static constexpr int F = 4, NG = 2, FL = 5; };  // + sound speed

// Ten-wave role map for 256-cell blocks (STSP_W10): SIMD s runs waves
// {s, s+4, s+8}.  Nine waves (one per edge) left SIMD 1 with two own-cell waves
// that also carried full flux waves, while SIMD 0 had three flux waves: the
// slowest SIMD set both barriers.  With a tenth wave:
//   SIMD 0: W0 flux+ring, W4 flux+ring, W8 flux
//   SIMD 1: W1 own+flux,  W5 own,       W9 32 edges
//   SIMD 2: W2 own+flux,  W6 flux+ring
//   SIMD 3: W3 own+flux,  W7 flux
// (ring = the window cells around the block, 144 for 16x16).
// Tables: one nibble per wave (wave w at bits 4w), 0xF = no role.
#ifndef STSP_W10
#define STSP_W10 1
#endif
// Branch-free minmod / MC slopes through a sign factor (slope()).
#ifndef STSP_SIGN_SLOPE
#define STSP_SIGN_SLOPE 1
#endif
template <int BX, int BY> struct Geom {
  static constexpr int NX = (BX + 1) * BY;   // x-edges
  static constexpr int NY = BX * (BY + 1);   // y-edges
  static constexpr bool W10 = STSP_W10 && (BX * BY == 256) && (NX + NY <= 9 * 64 - 32);
  static constexpr int NT = W10 ? 640 : ((NX + NY + 63) / 64) * 64;
  static constexpr unsigned long long OWN_TAB = 0xffff1f320fULL;    // own-cell slot
  static constexpr unsigned long long FLUX_TAB = 0x8275f16430ULL;   // flux slot: edges slot*64 + lane
  static constexpr unsigned long long RING_TAB = 0x5432f1fff0ULL;   // ring slot (non-own waves)
};

// Hardware min/max/abs/copysign (v_max_f64, |x| source modifier, v_bfi):
// one VALU op each where compare + select pairs cost three (wave64 fp64 and
// integer VALU ops issue at the same 4 cycles, so every instruction counts).
__device__ __forceinline__ double tabs(double x) { return __builtin_fabs(x); }
__device__ __forceinline__ float tabs(float x) { return __builtin_fabsf(x); }
__device__ __forceinline__ double tmin(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ float tmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double tmax(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float tmax(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ double tsign(double m, double s) { return __builtin_copysign(m, s); }
__device__ __forceinline__ float tsign(float m, float s) { return __builtin_copysignf(m, s); }
// Sound speed sqrt(g h) for g h in [0, ~1e7]: v_rsq_f64 + one Goldschmidt
// step + a final correction (~1 ulp, like the library expansion) without the
// library's range scaling for denormal / huge arguments (~15 VALU ops -> ~9).
// The bare v_sqrt_f64 is not enough: 3.6e-9 relative error in the state after
// a few steps against the fp64 reference.
#ifndef STSP_HW_SQRT
#define STSP_HW_SQRT 1
#endif
#if STSP_HW_SQRT
__device__ __forceinline__ double tsqrt(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = 0.5 * r;
  const double e = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  const double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return x > 0.0 ? g : 0.0;
}
__device__ __forceinline__ float tsqrt(float x) { return sqrtf(x); }
#else
__device__ __forceinline__ double tsqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float tsqrt(float x) { return sqrtf(x); }
#endif
// 1/x: hardware reciprocal + two Newton steps (within an ulp of IEEE division,
// 5 VALU ops instead of the 12-op div_scale/div_fmas/div_fixup sequence)
__device__ __forceinline__ double trcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ float trcp(float x) {
  float r = __builtin_amdgcn_rcpf(x);
  return __builtin_fmaf(r, __builtin_fmaf(-x, r, 1.0f), r);
}

// Limited slope, identical to models/base.py::limited_slope; LIM is a
// compile-time constant and every form is branch-free (selects only).
template <int LIM, typename T>
__device__ __forceinline__ T slope(T dl, T dr) {
  if constexpr (LIM == 0) {
    return T(0.5) * (dl + dr);
  } else if constexpr ((LIM == 1 || LIM == 2) && STSP_SIGN_SLOPE) {
    // sign factor instead of the dl * dr > 0 test and two selects: sg is +-1
    // when dl and dr agree in sign and 0 otherwise; the magnitude is 0 when
    // either difference is 0, so the result equals the select form
    const T sg = tsign(T(0.5), dl) + tsign(T(0.5), dr);
    T m = tmin(tabs(dl), tabs(dr));
    if constexpr (LIM == 2) m = tmin(T(2) * m, tabs(T(0.5) * (dl + dr)));
    return sg * m;
  } else {
    const bool same = dl * dr > T(0);
    T s;
    if constexpr (LIM == 1) {
      s = tsign(tmin(tabs(dl), tabs(dr)), dl);
    } else if constexpr (LIM == 2) {
      const T c = T(0.5) * (dl + dr);
      s = tsign(tmin(T(2) * tmin(tabs(dl), tabs(dr)), tabs(c)), c);
    } else {
      const T den = same ? dl + dr : T(1);
      s = T(2) * dl * dr / den;
    }
    return same ? s : T(0);
  }
}

// Half slope 0.5 * slope<LIM>(dl, dr), the offset from a cell average to its
// face value, with the powers of two folded into the sign factor and the
// limiter bound (exact: every folded factor is a power of two), so a face value
// is one fma on top: c0 +- half_slope.
template <int LIM, typename T>
__device__ __forceinline__ T half_slope(T dl, T dr) {
  if constexpr (LIM == 1 && STSP_SIGN_SLOPE) {
    const T sg = tsign(T(0.25), dl) + tsign(T(0.25), dr);   // +-0.5 or 0
    return sg * tmin(tabs(dl), tabs(dr));
  } else if constexpr (LIM == 2 && STSP_SIGN_SLOPE) {
    const T sg = tsign(T(0.5), dl) + tsign(T(0.5), dr);     // +-1 or 0
    return sg * tmin(tmin(tabs(dl), tabs(dr)), T(0.25) * tabs(dl + dr));
  } else if constexpr (LIM == 0) {
    return T(0.25) * (dl + dr);
  } else {
    return T(0.5) * slope<LIM>(dl, dr);
  }
}

// 16-byte vector loads (the CU's load path moves 16 B/lane at about twice the
// byte rate of 8 B/lane).
template <typename T> struct V16;
template <> struct V16<double> { using type = double2; static constexpr int W = 2; };
template <> struct V16<float> { using type = float4; static constexpr int W = 4; };

// base + i with a 32-bit byte offset: keeps the address in the global_load
// saddr + voffset form (uniform 64-bit base in SGPRs, one 32-bit VGPR offset)
// instead of a 64-bit VALU add per access.  Every buffer here is < 4 GiB.
template <typename T>
__device__ __forceinline__ const T* o32(const T* base, unsigned i) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + (unsigned)(i * (unsigned)sizeof(T)));
}
template <typename T>
__device__ __forceinline__ T* o32(T* base, unsigned i) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (unsigned)(i * (unsigned)sizeof(T)));
}

template <typename T>
__device__ __forceinline__ void load_rec8(const T* __restrict__ p, T (&r)[8]) {
  using V = typename V16<T>::type;
  constexpr int W = V16<T>::W;
  const V* vp = reinterpret_cast<const V*>(p);
#pragma unroll
  for (int k = 0; k < 8 / W; ++k) {
    const V v = vp[k];
    if constexpr (W == 2) { r[2 * k] = v.x; r[2 * k + 1] = v.y; }
    else { r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w; }
  }
}

// Raw buffer access to the state and geometry arrays: one uniform resource per
// array (4 SGPRs), the per-lane byte offset in one VGPR and the field offset
// f * S in an SGPR (soffset).  A field costs no VALU address arithmetic: with
// plain global pointers the compiler materialised a 64-bit VGPR address per
// field (v_lshl_add_u64 chains, 42 in the SWE kernel) in front of every load
// and store.  Stores take the cache policy as aux (16 = sc1, write-through).
typedef unsigned int v2u32 __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, -1, 0x00020000);
}
template <typename T>
__device__ __forceinline__ T bld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  if constexpr (sizeof(T) == 8)
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
  else
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
template <int AUX, typename T>
__device__ __forceinline__ void bst(T v, __amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  if constexpr (sizeof(T) == 8)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32, v), r, (int)voff, (int)soff, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)voff, (int)soff, AUX);
}
// 8-value cell record (64 B fp64 / 32 B fp32) as 16-byte buffer loads
template <typename T>
__device__ __forceinline__ void bld_rec8(__amdgpu_buffer_rsrc_t r, unsigned voff, T (&out)[8]) {
  constexpr int W = 16 / sizeof(T);
#pragma unroll
  for (int k = 0; k < 8 / W; ++k) {
    const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(voff + 16u * k), 0, 0);
    if constexpr (W == 2) {
      const double2 d = __builtin_bit_cast(double2, v);
      out[2 * k] = (T)d.x; out[2 * k + 1] = (T)d.y;
    } else {
      const float4 f = __builtin_bit_cast(float4, v);
      out[4 * k] = (T)f.x; out[4 * k + 1] = (T)f.y; out[4 * k + 2] = (T)f.z; out[4 * k + 3] = (T)f.w;
    }
  }
}

template <typename T>
struct Args {
  const T* X;
  const T* Q;
  const T* acc_in;
  T* out;
  T* acc_out;
  const T* recv;
  const int* gmap;
  const int* push;
  const int* blocks;
  const T* invA;
  const T* ex;
  const T* ey;
  const T* mx;
  const T* my;
  const T* cgeo;
  int ntile, n, S, mg, pw, nblocks, limiter;
  T a0, a1, a2, c0, c1, c2, dt, g, omega2;
  unsigned long long* stamps;
  unsigned mdiv_t, mdiv_r;   // ceil(2^32 / (nbx nby)), ceil(2^32 / nbx); 0 = divide
  int diag_repeat;           // diag build only: run the block body this many extra times
  int wt;                    // write-through output stores (st_out)
  // direct xGMI halo (XG kernels only, see stsp_kernels.h)
  int ring;
  T* const* peer_ring;
  unsigned long long* const* peer_cnt;
  const unsigned long long* cnt;
  const unsigned long long* nprod;
  const int* bmask;
  int* epoch;
  int* err;
  long long timeout_ticks;
  const int* pedge;
};

#ifdef STSP_STAMPS
// Diagnostic build: lane 0 of every wave records the shader clock at phase
// boundaries into stamps[block][wave < 16][16] (shares only; never quote a
// stamped build's run time).
#define STAMP(k)                                                                        \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if ((threadIdx.x & 63) == 0 && a.stamps)                                            \
      a.stamps[((long)blockIdx.x * 16 + (threadIdx.x >> 6)) * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

// Rusanov flux of the SWE along unit normal (m0,m1,m2); L = edge length.
// wl/wr: reconstructed primitive (h, v); cl/cr: cell-average primitive + sound speed.
template <typename T>
__device__ __forceinline__ void swe_flux(const T (&wl)[4], const T (&wr)[4], const T (&cl)[5], const T (&cr)[5],
                                         T m0, T m1, T m2, T L, T g, T (&f)[4]) {
  const T hL = wl[0], hR = wr[0];
  const T vnL = wl[1] * m0 + wl[2] * m1 + wl[3] * m2;
  const T vnR = wr[1] * m0 + wr[2] * m1 + wr[3] * m2;
  const T sL = tabs(cl[1] * m0 + cl[2] * m1 + cl[3] * m2) + cl[4];
  const T sR = tabs(cr[1] * m0 + cr[2] * m1 + cr[3] * m2) + cr[4];
  const T hc = T(0.5) * tmax(sL, sR);
  const T pL = hL * vnL, pR = hR * vnR;
  f[0] = (T(0.5) * (pL + pR) - hc * (hR - hL)) * L;
  const T pr = T(0.25) * g * (hL * hL + hR * hR);
  const T mm[3] = {m0, m1, m2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const T uL = hL * wl[1 + k], uR = hR * wr[1 + k];
    f[1 + k] = (T(0.5) * (uL * vnL + uR * vnR) + pr * mm[k] - hc * (uR - uL)) * L;
  }
}

// State access: plain in launch-per-stage kernels; in the persistent kernel,
// agent-scope relaxed atomics, which gfx950 lowers to global_load/store ... sc1
// (L1 bypass / write-through), the hand-off form of cdna_hip_programming.md
// Guideline 16 (R1) measured valid for one workgroup per CU.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

template <bool SYNC, typename T>
__device__ __forceinline__ T ld_state(const T* p) {
  if constexpr (!SYNC) {
    return *p;
  } else if constexpr (sizeof(T) == 8) {
    return __builtin_bit_cast(T, __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  } else {
    return __builtin_bit_cast(T, __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  }
}

// System-scope (cross-GPU) accesses of the direct xGMI halo: sc0 sc1, i.e.
// no GPU cache keeps a copy, so a peer's store is seen by the next poll/load.
template <typename T>
__device__ __forceinline__ T ld_sys(const T* p) {
  if constexpr (sizeof(T) == 8)
    return __builtin_bit_cast(T, __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  else
    return __builtin_bit_cast(T, __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

template <typename T>
__device__ __forceinline__ void st_sys(T* p, T v) {
  if constexpr (sizeof(T) == 8)
    __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else
    __hip_atomic_store((gu32*)p, __builtin_bit_cast(unsigned int, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stage output stores.  wt (block-uniform): write-through (agent-scope relaxed
// atomic store, global_store ... sc1), so the kernel-end release has no dirty
// L2 lines of the state to write back.  That shortens the kernel boundary on
// latency-bound grids (C96: 15.2 -> 14.9 us/step) but costs HBM efficiency on
// grids that stream (C360: 120 -> 221 us/step); launch_l decides per launch.
template <bool SYNC, typename T>
__device__ __forceinline__ void st_state(T* p, T v);
template <bool SYNC, typename T>
__device__ __forceinline__ void st_out(int wt, T* p, T v) {
  if (wt) st_state<true>(p, v);
  else st_state<SYNC>(p, v);
}

template <bool SYNC, typename T>
__device__ __forceinline__ void st_state(T* p, T v) {
  if constexpr (!SYNC) {
    *p = v;
  } else if constexpr (sizeof(T) == 8) {
    __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store((gu32*)p, __builtin_bit_cast(unsigned int, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One RK stage of one BX x BY block (all phases).  SYNC = persistent-kernel
// mode: every access to state written by other workgroups in this launch is an
// agent-scope sc1 access (L1 bypass, write-through), see persistent_kernel.
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
  if constexpr (Geom<BX, BY>::W10) {
    const int lane = tid & 63;
    const unsigned os = (unsigned)(Geom<BX, BY>::OWN_TAB >> (4 * wv)) & 15u;
    const unsigned fs = (unsigned)(Geom<BX, BY>::FLUX_TAB >> (4 * wv)) & 15u;
    const unsigned rs = (unsigned)(Geom<BX, BY>::RING_TAB >> (4 * wv)) & 15u;
    oid = os != 15u ? (int)os * 64 + lane : -1;
    eid = fs != 15u ? (int)fs * 64 + lane : NE_;
    rid = rs != 15u ? (int)rs * 64 + lane : RING;
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
              const gu64* rp = ((const gu64*)(a.recv)) + (long)(xe % STSP_XG_SLOTS) * a.ring +
                               (long)(-1 - m) * (F * G);
              const unsigned want = (unsigned)xe + 1u;
              unsigned long long gr[F * G];
              const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
              for (;;) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < F * G; ++k) {
                  gr[k] = __hip_atomic_load(rp + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
              const T* rp = rring + (long)(-1 - m) * F;
#pragma unroll
              for (int f = 0; f < F; ++f) v[f] = ld_sys(rp + f);
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

  // ---- 1b. PLR face values, one (cell, direction) per thread -------------------
  // task t < NFX: x-direction, cell (x0 + c - 1, y0 + r), t = r (BX + 2) + c;
  // else y-direction, cell (x0 + c, y0 + r - 1), t - NFX = r BX + c.
  if constexpr (FACES) {
    const T* w0 = &s_w[0][0][0];
    // PPM: tile sides on a cube (panel) edge; cells whose 5-cell stencil
    // crosses one use MC-limited PLR faces (models/base.py::ppm_faces)
    const int pe = (LIM == 4) ? a.pedge[tile] : 0;
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
          const int xc = tx ? x : y;                  // cell index along the task direction
          const bool edge_cell = (LIM == 4) && (((pe & (tx ? 1 : 4)) && xc <= 1) || ((pe & (tx ? 2 : 8)) && xc >= n - 2));
          if (LIM == 4 && edge_cell) {
            const T hs = T(0.5) * slope<2>(c0 - m1, p1 - c0);
            s_fm[f][t] = c0 - hs;
            s_fp[f][t] = c0 + hs;
          } else if constexpr (LIM == 4) {
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
            gu64* dst = ((gu64*)(a.peer_ring[code >> 24])) + (long)((xe + 1) % STSP_XG_SLOTS) * a.ring +
                        (long)(code & 0xFFFFFF) * (F * G);
            const unsigned long long tag = (unsigned long long)((unsigned)xe + 2u) << 32;
#pragma unroll
            for (int f = 0; f < F; ++f) {
              if constexpr (G == 2) {
                const unsigned long long b = __builtin_bit_cast(unsigned long long, o[f]);
                __hip_atomic_store(dst + 2 * f, tag | (b & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(dst + 2 * f + 1, tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              } else {
                __hip_atomic_store(dst + f, tag | __builtin_bit_cast(unsigned, o[f]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
              }
            }
          } else {
            T* dst = a.peer_ring[code >> 24] + (long)((xe + 1) % STSP_XG_SLOTS) * a.ring + (long)(code & 0xFFFFFF) * F;
#pragma unroll
            for (int f = 0; f < F; ++f) st_sys(dst + f, o[f]);
          }
        }
      }
    }
  }
  if constexpr (XG) {
    if (!STSP_XG_TAG && feed) {   // publish: every storing wave drains, then one lane per peer counts
#if STSP_XG_FENCE == 0
      __threadfence_system();
#endif
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid < 32 && ((feed >> tid) & 1))
#if STSP_XG_FENCE == 2
        __hip_atomic_fetch_add((gu64*)a.peer_cnt[tid], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
        __hip_atomic_fetch_add((gu64*)a.peer_cnt[tid], 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    }
    if (tid == 0) a.epoch[bid] = xe + 1;
  }
  STAMP(6);
}


// XCD-aware bijective remap: logical blocks [k*nb/8, ...) share one XCD
// (blocks b and b+8 are dealt to the same XCD), so neighbouring blocks, which
// share halo cells, share an L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nb) {
  const int xcd = orig & 7, q = nb >> 3, r = nb & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

template <typename T>
__device__ __forceinline__ void pin_args(const Args<T>& a) {
  // Pin every kernel argument in SGPRs here: hipcc otherwise issues the
  // kernarg scalar loads lazily, each behind its own lgkmcnt(0) (3-4 serial
  // round trips in the prologue, seen with in-kernel stamps).
  asm volatile("" ::"s"(a.X), "s"(a.Q), "s"(a.acc_in), "s"(a.out), "s"(a.acc_out), "s"(a.recv), "s"(a.gmap),
               "s"(a.push), "s"(a.blocks));
  asm volatile("" ::"s"(a.invA), "s"(a.ex), "s"(a.ey), "s"(a.mx), "s"(a.my), "s"(a.cgeo));
  asm volatile("" ::"s"(a.ntile), "s"(a.n), "s"(a.S), "s"(a.mg), "s"(a.pw), "s"(a.nblocks));
  asm volatile("" ::"s"(a.a0), "s"(a.a1), "s"(a.a2), "s"(a.c0), "s"(a.c1), "s"(a.c2), "s"(a.dt), "s"(a.g),
               "s"(a.omega2));
}

template <typename T, int P, int BX, int BY, int LIM, bool REMOTE, bool LIST, bool XG>
__global__ __launch_bounds__((Geom<BX, BY>::NT)) void stage_kernel(Args<T> a) {
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

// ---- persistent multi-step kernel (small grids) --------------------------------
// One workgroup per CU, all co-resident (checked by the cooperative launch).
// Each workgroup runs every stage of `nsteps` steps for its block; a stage
// boundary is a neighbour-only hand-off instead of a kernel boundary:
//   publish: all state stores are sc1 (write-through) -> every wave
//            s_waitcnt vmcnt(0) -> barrier -> lane 0 stores flag[bid] = epoch (sc1)
//   consume: lanes 0..nn-1 poll the flags of the blocks whose output this block
//            reads (sc1 loads, s_sleep, bounded by a wall-clock timeout) -> barrier
// so no block ever waits on the whole grid.  Any timeout sets *err and every
// block drains out (no hang).
template <typename T>
struct PArgs {
  Args<T> st[4];        // stage descriptors of one step (buffer-invariant period)
  int nstages;
  int nsteps;
  unsigned* flags;      // [nblocks] epochs, zeroed before the launch
  const int* nbr;       // [nblocks][maxnbr] producer blocks (-1 padded)
  int maxnbr;
  int* err;             // 0 ok; 1 timeout
  unsigned long long timeout_ticks;   // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ unsigned flag_load(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T, int P, int BX, int BY, int LIM>
__global__ __launch_bounds__((Geom<BX, BY>::NT)) void persistent_kernel(PArgs<T> pa) {
  pin_args(pa.st[0]);
  const int bid = xcd_remap(blockIdx.x, pa.st[0].nblocks);
  const int tid = threadIdx.x;
  __shared__ int s_abort;
  if (tid == 0) s_abort = 0;
  __syncthreads();
  unsigned epoch = 0;
#ifdef STSP_STAMPS
  unsigned long long acc_body = 0, acc_drain = 0, acc_wait = 0, tA = 0, tB = 0, tC = 0;
#endif
  for (int step = 0; step < pa.nsteps; ++step) {
    for (int s = 0; s < pa.nstages; ++s) {
#ifdef STSP_STAMPS
      if (tid == 0) tA = __builtin_amdgcn_s_memtime();
#endif
      stage_body<T, P, BX, BY, LIM, false, true>(pa.st[s], bid);
#ifdef STSP_STAMPS
      if (tid == 0) tB = __builtin_amdgcn_s_memtime();
#endif
      // -- publish this block's stage output
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#ifdef STSP_STAMPS
      if (tid == 0) tC = __builtin_amdgcn_s_memtime();
#endif
      ++epoch;
      if (tid == 0) __hip_atomic_store((gu32*)&pa.flags[bid], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // -- wait for every producer of the next stage's window
      if (tid < pa.maxnbr) {
        const int nb = pa.nbr[bid * pa.maxnbr + tid];
        if (nb >= 0) {
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          while (flag_load(&pa.flags[nb]) < epoch) {
            if (__hip_atomic_load((gu32*)pa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
              s_abort = 1;
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > pa.timeout_ticks) {
              __hip_atomic_store((gu32*)pa.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              s_abort = 1;
              break;
            }
            __builtin_amdgcn_s_sleep(2);
          }
        }
      }
      __syncthreads();
#ifdef STSP_STAMPS
      if (tid == 0) {
        const unsigned long long tD = __builtin_amdgcn_s_memtime();
        acc_body += tB - tA; acc_drain += tC - tB; acc_wait += tD - tC;
      }
#endif
      if (s_abort) return;
    }
  }
#ifdef STSP_STAMPS
  if (tid == 0 && pa.st[0].stamps) {
    pa.st[0].stamps[(long)blockIdx.x * 256 + 0] = acc_body;
    pa.st[0].stamps[(long)blockIdx.x * 256 + 1] = acc_drain;
    pa.st[0].stamps[(long)blockIdx.x * 256 + 2] = acc_wait;
  }
#endif
}

template <typename T>
Args<T> make_args(const StageDesc* d) {
  Args<T> a;
  a.X = (const T*)d->X; a.Q = (const T*)d->Q; a.acc_in = (const T*)d->acc_in;
  a.out = (T*)d->out; a.acc_out = (T*)d->acc_out; a.recv = (const T*)d->recv;
  a.gmap = d->gmap; a.push = d->push; a.blocks = d->blocks;
  a.invA = (const T*)d->invA; a.ex = (const T*)d->ex; a.ey = (const T*)d->ey;
  a.mx = (const T*)d->mx; a.my = (const T*)d->my; a.cgeo = (const T*)d->cgeo;
  a.ntile = d->ntile; a.n = d->n; a.S = d->S; a.mg = d->mg; a.pw = d->pw; a.nblocks = d->nblocks;
  a.limiter = d->limiter;
  a.a0 = (T)d->a0; a.a1 = (T)d->a1; a.a2 = (T)d->a2; a.c0 = (T)d->c0; a.c1 = (T)d->c1; a.c2 = (T)d->c2;
  a.dt = (T)d->dt; a.g = (T)d->g; a.omega2 = (T)d->omega2;
  a.stamps = (unsigned long long*)d->stamps;
  a.diag_repeat = 0;
  a.wt = 0;
  a.ring = d->ring;
  a.peer_ring = (T* const*)d->peer_ring;
  a.peer_cnt = d->peer_cnt;
  a.cnt = d->cnt;
  a.nprod = d->nprod;
  a.bmask = d->bmask;
  a.epoch = d->epoch;
  a.err = d->err;
  a.timeout_ticks = d->timeout_ticks;
  a.pedge = d->pedge;
  return a;
}

// ceil(2^32 / dv) if floor(x * M / 2^32) == x / dv for every x < xmax (holds
// when xmax * dv <= 2^32: the rounding excess x (M dv - 2^32) / 2^32 < 1), else 0.
inline unsigned magic_div(unsigned dv, unsigned long long xmax) {
  if (dv <= 1 || xmax * dv > (1ull << 32)) return 0;
  return (unsigned)(((1ull << 32) + dv - 1) / dv);
}

template <typename T, int BX, int BY>
void set_magic(Args<T>& a) {
  const unsigned nbx = (a.n + BX - 1) / BX, nby = (a.n + BY - 1) / BY;
  const unsigned long long total = (unsigned long long)a.ntile * nbx * nby;
  a.mdiv_t = magic_div(nbx * nby, total);
  a.mdiv_r = magic_div(nbx, (unsigned long long)nbx * nby);
}

// Write-through output stores pay off while the launch is latency-bound: up to
// about 1024 cells per CU (C180 on one GPU, every multi-GPU C96 rank).
// STSP_WT_STORES=0/1 overrides (A/B runs).
inline bool want_wt(long cells) {
  static const int cus = [] {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 256;
    return c > 0 ? c : 256;
  }();
  static const int force = [] {
    const char* e = std::getenv("STSP_WT_STORES");
    return e ? std::atoi(e) : -1;
  }();
  if (force >= 0) return force != 0;
  return cells <= 1024L * cus;
}

template <typename T, int P, int BX, int BY, int LIM>
int launch_l(const StageDesc* d, hipStream_t s) {
  Args<T> a = make_args<T>(d);
  set_magic<T, BX, BY>(a);
  a.wt = want_wt((long)d->nblocks * BX * BY) ? 1 : 0;
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
  if (d->pw != d->n + 2 * d->mg || d->mg < Phys<P>::NG || (d->limiter == 4 && (d->mg < 3 || !d->pedge))) return -5;
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
      gu64* dst = ((gu64*)(peer_ring[c >> 24])) + (long)slot * ring + (long)(c & 0xFFFFFF) * F * G;
      const unsigned long long tag = (unsigned long long)((unsigned)epoch + 1u) << 32;
      for (int f = 0; f < F; ++f) {
        const T v = q[(long)f * S + src[i]];
        if constexpr (G == 2) {
          const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
          __hip_atomic_store(dst + 2 * f, tag | (b & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(dst + 2 * f + 1, tag | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
          __hip_atomic_store(dst + f, tag | __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    } else {
      T* dst = peer_ring[c >> 24] + (long)slot * ring + (long)(c & 0xFFFFFF) * F;
      for (int f = 0; f < F; ++f) st_sys(dst + f, q[(long)f * S + src[i]]);
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

template <typename T, int P, int BX, int BY, int LIM>
int launch_persist(const StageDesc* st, int nstages, int nsteps, unsigned* flags, const int* nbr, int maxnbr,
                   int* err, double timeout_s, hipStream_t s) {
  PArgs<T> pa;
  for (int k = 0; k < nstages; ++k) {
    pa.st[k] = make_args<T>(&st[k]);
    set_magic<T, BX, BY>(pa.st[k]);
  }
  pa.nstages = nstages;
  pa.nsteps = nsteps;
  pa.flags = flags;
  pa.nbr = nbr;
  pa.maxnbr = maxnbr;
  pa.err = err;
  pa.timeout_ticks = (unsigned long long)(timeout_s * 1e8);
  const int nb = st[0].nblocks;
  hipError_t e = hipMemsetAsync(flags, 0, sizeof(unsigned) * ((nb + 3) & ~3), s);
  if (e != hipSuccess) return (int)e;
  void* args[] = {&pa};
  e = hipLaunchCooperativeKernel((const void*)persistent_kernel<T, P, BX, BY, LIM>, dim3(nb),
                                 dim3(Geom<BX, BY>::NT), args, 0, s);
  return (int)e;
}

template <typename T, int P>
int persist_p(int bx, int by, const StageDesc* st, int nstages, int nsteps, unsigned* flags, const int* nbr,
              int maxnbr, int* err, double timeout_s, hipStream_t s) {
  if (bx != 16 || by != 16) return -2;
  if (P == 1) return launch_persist<T, P, 16, 16, 0>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
  switch (st[0].limiter) {
    case 0: return launch_persist<T, P, 16, 16, 0>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
    case 1: return launch_persist<T, P, 16, 16, 1>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
    case 2: return launch_persist<T, P, 16, 16, 2>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
    case 3: return launch_persist<T, P, 16, 16, 3>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
    case 4: return launch_persist<T, P, 16, 16, 4>(st, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, s);
  }
  return -7;
}

}  // namespace

extern "C" int stsp_persistent_launch(int phys, int dtype, int bx, int by, const StageDesc* stages, int nstages,
                                      int nsteps, unsigned* flags, const int* nbr, int maxnbr, int* err,
                                      double timeout_s, hipStream_t stream) {
  if (nstages < 1 || nstages > 4 || nsteps < 1) return -8;
  for (int k = 0; k < nstages; ++k) {
    const StageDesc* d = &stages[k];
    if (d->blocks || d->remote || !d->push || d->pw != d->n + 2 * d->mg) return -6;
    if (d->limiter == 4 && (d->mg < 3 || !d->pedge)) return -5;
    if (d->nblocks != stages[0].nblocks) return -9;
  }
  if (dtype == 1) {
    switch (phys) {
      case 0: return persist_p<double, 0>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
      case 1: return persist_p<double, 1>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
      case 2: return persist_p<double, 2>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
    }
  } else if (dtype == 0) {
    switch (phys) {
      case 0: return persist_p<float, 0>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
      case 1: return persist_p<float, 1>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
      case 2: return persist_p<float, 2>(bx, by, stages, nstages, nsteps, flags, nbr, maxnbr, err, timeout_s, stream);
    }
  }
  return -3;
}

extern "C" int stsp_stage_launch(int phys, int dtype, int bx, int by, const StageDesc* d, hipStream_t stream) {
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
