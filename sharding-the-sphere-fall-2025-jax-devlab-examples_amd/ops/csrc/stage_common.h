// Device helpers shared by the fused stage kernel (stage_kernel.hip) and the
// persistent step kernel (step_kernel.hip): physics constants, the block
// role geometry, branch-free math, buffer access, the SWE Rusanov flux and
// the launch-argument record.  Everything lives in an anonymous namespace:
// each translation unit gets its own copy of these inline templates.
#pragma once
#include "stsp_kernels.h"

// Publish protocol of the arrival-counter hand-off (STSP_XG_TAG=0 below):
// every storing wave drains, then a release add per peer (one L2 write-back
// per producing block).  Measured alternatives (profiles/r1_xg_fence_probe.jsonl,
// loopback C96 us/step, plain step 17.1): a __threadfence_system() before the
// add 117.5 (the fence is seq_cst: every wave also invalidates L2), the
// release add 28.6, a relaxed add after the drain 26.8 (not a release in the
// model); the probes are gone, the release add stays.
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
// Ring record layout.  A slot holds nrec = ring / NW records of NW words (NW =
// F G tagged 8-byte granules, or F values under STSP_XG_TAG=0).
// STSP_XG_SOA=1 (default): word-major, word w of record r at w nrec + r.  The
// host numbers a consumer's records by owner rank, then cell id (row order),
// so the lanes of one store or poll instruction touch consecutive 8-byte words
// (up to 512 contiguous bytes per wave) instead of words NW x 8 bytes apart
// (record-major, r NW + w: STSP_XG_SOA=0, the round-5 layout, kept for the A/B
// in profiles/r6_ring).
#ifndef STSP_XG_SOA
#define STSP_XG_SOA 1
#endif
__device__ __forceinline__ long ring_word(int nrec, int nw, int rec, int w) {
  return STSP_XG_SOA ? (long)w * nrec + rec : (long)rec * nw + w;
}
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

// Border-edge flux slots for the panel-edge fix-up (stage_kernel.hip, PEW):
// slot PEW_SX = x-edges at columns {0, 1, BX-1, BX} of every row (lane = row * 4 + q),
// slot PEW_SY = y-edges at rows {0, 1, BY-1, BY} of every column, the other
// seven slots (in slot order) = the interior x-edges (columns 2 .. BX-2) then
// the interior y-edges (rows 2 .. BY-2), 64 per slot.  The border slots sit on
// waves 7 (SIMD 3) and 6 (SIMD 2), the SIMDs with the most slack before the
// flux barrier (SIMD 0 already runs three flux waves; profiles/r2_pe_stamps).
// Returns the canonical edge id (x-edge r (BX+1) + c, y-edge NX + r BX + c) or
// NX + NY past the last edge.  A bijection onto the edges for 16 x 16 blocks
// (tests/test_kernel_contracts.py mirrors it).
#ifndef STSP_PE_WAVE
#define STSP_PE_WAVE 1
#endif
constexpr int PEW_SX = 7, PEW_SY = 5;
template <int BX, int BY>
__device__ __forceinline__ int edge_of_slot(int slot, int lane) {
  constexpr int NX = (BX + 1) * BY, NY = BX * (BY + 1);
  constexpr int IX = BX - 3, IY = BY - 3;         // interior columns / rows per line
  static_assert(BX == 16 && BY == 16, "border slots are laid out for 16 x 16 blocks");
  const int q = lane & 3, u4 = lane >> 2;
  const int b = q < 2 ? q : q + (BX - 3);         // 0, 1, B-1, B
  if (slot == PEW_SX) return u4 * (BX + 1) + b;
  if (slot == PEW_SY) return NX + b * BX + u4;
  const int u = (slot - (slot > PEW_SY) - (slot > PEW_SX)) * 64 + lane;
  if (u < BY * IX) {
    const int r = u / IX;
    return r * (BX + 1) + 2 + (u - r * IX);
  }
  const int v = u - BY * IX;
  if (v < IY * BX) {
    const int r = v / BX;
    return NX + (2 + r) * BX + (v - r * BX);
  }
  return NX + NY;
}

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
  int pew;                   // border-wave panel-edge fix-up allowed (full blocks: n % BX == n % BY == 0)
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
  const int* pe_base;
  const T* pe_t;
  // streaming stage (march_kernel.hip)
  const int* torg;
  const T* crec;
  const T* lxt;
  const T* bpad;
  int Nf;
  unsigned long long frames;   // 9 bits per panel (ops/fused.py::frame_code)
  const int* cgmap;            // carried corner ghosts (stsp_kernels.h)
  const int* cpush;
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
  // F = L [ hL (vnL/2 + hc) (1, vL) + hR (vnR/2 - hc) (1, vR) + (0, pr m) ]: the
  // Rusanov average and jump folded into one weight per side (fewer fp64 ops)
  const T bL = L * hL * (T(0.5) * vnL + hc), bR = L * hR * (T(0.5) * vnR - hc);
  const T prL = T(0.25) * g * L * (hL * hL + hR * hR);
  f[0] = bL + bR;
  f[1] = bL * wl[1] + (bR * wr[1] + prL * m0);
  f[2] = bL * wl[2] + (bR * wr[2] + prL * m1);
  f[3] = bL * wl[3] + (bR * wr[3] + prL * m2);
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
  a.pew = 0;
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
  a.pe_base = d->pe_base;
  a.pe_t = (const T*)d->pe_t;
  a.torg = d->torg;
  a.crec = (const T*)d->crec;
  a.lxt = (const T*)d->lxt;
  a.bpad = (const T*)d->bpad;
  a.Nf = d->Nf;
  a.cgmap = d->cgmap;
  a.cpush = d->cpush;
  a.frames = 0;
  for (int k = 0; k < 6; ++k) a.frames |= (unsigned long long)(d->frames[k] & 511) << (9 * k);
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

}  // namespace
