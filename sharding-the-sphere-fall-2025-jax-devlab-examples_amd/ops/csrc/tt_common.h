// Wave-level helpers shared by the low-rank kernels (tt_kernels.hip,
// tt_persist.hip): a lane broadcast through v_readlane and 8 / 16-lane sums
// through DPP, instead of __shfl / __shfl_xor (each a ds_bpermute round trip
// through the LDS crossbar).
#pragma once
#include <hip/hip_runtime.h>

namespace tt {

// value of lane l (wave-uniform: a constant once the caller's loop is
// unrolled) in every lane, through v_readlane (scalar result, no LDS)
template <typename T>
__device__ __forceinline__ T lane_bcast(T v, int l) {
  if constexpr (sizeof(T) == 8) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  }
}

// DPP move of a 64-bit value (two 32-bit moves, every lane active)
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

constexpr int DPP_QP_1032 = 0xB1;       // quad_perm [1, 0, 3, 2]: lane xor 1
constexpr int DPP_QP_2301 = 0x4E;       // quad_perm [2, 3, 0, 1]: lane xor 2
constexpr int DPP_ROW_HALF_MIRROR = 0x141;   // i <-> 7 - i within 8 lanes
constexpr int DPP_ROW_MIRROR = 0x140;        // i <-> 15 - i within 16 lanes

// sum over the aligned group of 8 lanes, in every lane of the group
__device__ __forceinline__ double sum8(double x) {
  x += dpp64<DPP_QP_1032>(x);
  x += dpp64<DPP_QP_2301>(x);
  x += dpp64<DPP_ROW_HALF_MIRROR>(x);   // the other quad holds the other half
  return x;
}
// sum over the aligned group of 16 lanes (a DPP row), in every lane of the row
__device__ __forceinline__ double sum16(double x) {
  x = sum8(x);
  return x + dpp64<DPP_ROW_MIRROR>(x);
}

}  // namespace tt
