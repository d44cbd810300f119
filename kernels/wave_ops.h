// wave_ops.h — 64-lane wave reductions on CDNA4 (gfx950) without LDS.
//
// __shfl_xor lowers to ds_bpermute_b32: an LDS round trip (issue + lgkmcnt(0) wait) per step, six
// dependent steps per 64-lane reduction. Here the steps stay in the VALU:
//   * within a 16-lane row: DPP quad_perm [1,0,3,2] and [2,3,0,1] (lane ^ 1, lane ^ 2), then
//     row_ror:4 and row_ror:8 (rotations: after the quad step every lane of a quad holds the quad's
//     value, so adding the row rotated by 4 and then by 8 sums the row's four quads in every lane);
//   * across rows: v_permlane16_swap (rows 0<->1, 2<->3) and v_permlane32_swap (halves), gfx950's
//     cross-row swaps (cdna_hip_programming.md T21), each one VALU op.
// The rotations add in a lane-dependent order, so the sum is taken from the first lane
// (v_readfirstlane): wave-uniform and bit-identical in every lane, as the xor butterfly's is. The max
// is order-independent.
#pragma once
#include <hip/hip_runtime.h>

namespace kfw {

namespace dpp {
constexpr int kQuadXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kRowRor4 = 0x124;  // row_ror:4
constexpr int kRowRor8 = 0x128;  // row_ror:8
constexpr int kRowMirror = 0x140;      // lane i <- 15 - i within each 16-lane row
constexpr int kRowHalfMirror = 0x141;  // lane i <- 7 - i within each 8-lane half row
}  // namespace dpp

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// value of lane ^ 16 (row pairs 0<->1, 2<->3) and of lane ^ 32 (wave halves)
__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ float xor16(float v) {
  const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  // s[0]: odd rows took the even rows' values; s[1]: even rows took the odd rows' values
  const unsigned lane = lane_id();
  return __uint_as_float((lane & 16) ? s[0] : s[1]);
}
__device__ __forceinline__ float xor32(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const unsigned lane = lane_id();
  return __uint_as_float((lane & 32) ? s[0] : s[1]);
}

// lane i combined with lane i ^ 32: one v_permlane32_swap (both halves get the pair in the same order)
__device__ __forceinline__ float sum_halves(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
__device__ __forceinline__ float max_halves(float v) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

// sum over aligned groups of N = 8 or 16 lanes (every lane of a group gets its group's sum; the
// mirrors pair each quad with the other quad(s) of its group)
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 8 || N == 16, "group_sum: 8 or 16 lanes");
  v += dpp_mov<dpp::kQuadXor1>(v);
  v += dpp_mov<dpp::kQuadXor2>(v);
  v += dpp_mov<dpp::kRowHalfMirror>(v);
  if constexpr (N == 16) v += dpp_mov<dpp::kRowMirror>(v);
  return v;
}

// sum / max over the 64 lanes, result in every lane
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_mov<dpp::kQuadXor1>(v);
  v += dpp_mov<dpp::kQuadXor2>(v);
  v += dpp_mov<dpp::kRowRor4>(v);
  v += dpp_mov<dpp::kRowRor8>(v);
  auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(s[0]) + __uint_as_float(s[1]);
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<dpp::kQuadXor1>(v));
  v = fmaxf(v, dpp_mov<dpp::kQuadXor2>(v));
  v = fmaxf(v, dpp_mov<dpp::kRowRor4>(v));
  v = fmaxf(v, dpp_mov<dpp::kRowRor8>(v));
  auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
  s = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}

}  // namespace kfw
