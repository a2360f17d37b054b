// Wave-level helpers shared by the streaming stage (march_kernel.hip) and the
// pipelined streaming step (march3_kernel.hip): one wave of 64 lanes marches a
// strip of columns up a tile, x-neighbours come from the adjacent lanes.
#pragma once
#include "stage_common.h"

namespace {

constexpr int MW = 64;          // lanes per wave
constexpr int MWPB = 4;         // independent waves (jobs) per workgroup

// Wave-wide lane shifts.  wave_shr:1: lane i <- lane i-1; wave_shl:1: lane i
// <- lane i+1 (lanes without a source read 0).  DPP moves are 32-bit, so a
// double is two moves.
constexpr int DPP_SHR = 0x138, DPP_SHL = 0x130;
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  int2 p = __builtin_bit_cast(int2, v);
  p.x = __builtin_amdgcn_update_dpp(0, p.x, CTRL, 0xf, 0xf, false);
  p.y = __builtin_amdgcn_update_dpp(0, p.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, p);
}
template <typename T> __device__ __forceinline__ T shr(T v) { return dpp<DPP_SHR>(v); }
template <typename T> __device__ __forceinline__ T shl(T v) { return dpp<DPP_SHL>(v); }

}  // namespace
