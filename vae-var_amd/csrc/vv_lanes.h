// Lane permutes for wave64 reductions (r05): exact replacements of __shfl_xor(v, O) for the compile-time offsets the
// kernels reduce over, as VALU lane permutes instead of ds_bpermute_b32 (an LDS round trip per step).
// Callers keep the reduced lanes' group fully active (whole L-lane groups, whole waves).
#pragma once
#include <hip/hip_runtime.h>

namespace vv {

// __shfl_xor(v, O) without the LDS crossbar (r05): ds_bpermute_b32 (what __shfl_xor compiles to here) costs an LDS
// round trip per step; these are VALU lane permutes with the same result bit for bit. O = 1, 2: DPP quad_perm; 4, 8:
// two DPP steps (row_half_mirror is l ^ 7 within 8 lanes, row_mirror l ^ 15 within 16); 16, 32: gfx950's
// v_permlane16/32_swap, whose two outputs hold lane l's value and its partner's (the partner picked by the lane's row).
template <int O>
__device__ __forceinline__ int xshfl_i(int v) {
  static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor offset");
  if constexpr (O == 1) {
    return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (O == 2) {
    return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (O == 4) {
    const int t = __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false);  // row_half_mirror: l ^ 7
    return __builtin_amdgcn_mov_dpp(t, 0x1B, 0xF, 0xF, false);           // quad_perm [3,2,1,0]: l ^ 3
  } else if constexpr (O == 8) {
    const int t = __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false);  // row_mirror: l ^ 15
    return __builtin_amdgcn_mov_dpp(t, 0x141, 0xF, 0xF, false);          // row_half_mirror: l ^ 7
  } else if constexpr (O == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)(((threadIdx.x >> 4) & 1) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)(((threadIdx.x >> 5) & 1) ? r[0] : r[1]);
  }
}
template <int O>
__device__ __forceinline__ float xshfl(float v) { return __int_as_float(xshfl_i<O>(__float_as_int(v))); }
template <int O>
__device__ __forceinline__ int xshfl(int v) { return xshfl_i<O>(v); }

// all-reduce over aligned groups of L lanes in the order L / 2, L / 4, .., 1 (the order of the __shfl_xor loops
// they replace: bit-identical results)
template <int L>
__device__ __forceinline__ float lane_sum(float v) {
  static_assert(L == 1 || L == 2 || L == 4 || L == 8 || L == 16 || L == 32 || L == 64, "group");
  if constexpr (L >= 64) v += xshfl<32>(v);
  if constexpr (L >= 32) v += xshfl<16>(v);
  if constexpr (L >= 16) v += xshfl<8>(v);
  if constexpr (L >= 8) v += xshfl<4>(v);
  if constexpr (L >= 4) v += xshfl<2>(v);
  if constexpr (L >= 2) v += xshfl<1>(v);
  return v;
}
template <int O>
__device__ __forceinline__ double xshfl(double x) {  // the two 32-bit halves: the value __shfl_xor exchanges
  const long long b = __double_as_longlong(x);
  const int lo = xshfl_i<O>((int)(b & 0xffffffff)), hi = xshfl_i<O>((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int L>
__device__ __forceinline__ double lane_sum(double v) {
  if constexpr (L >= 64) v += xshfl<32>(v);
  if constexpr (L >= 32) v += xshfl<16>(v);
  if constexpr (L >= 16) v += xshfl<8>(v);
  if constexpr (L >= 8) v += xshfl<4>(v);
  if constexpr (L >= 4) v += xshfl<2>(v);
  if constexpr (L >= 2) v += xshfl<1>(v);
  return v;
}
template <int L>
__device__ __forceinline__ float lane_max(float v) {
  if constexpr (L >= 64) v = fmaxf(v, xshfl<32>(v));
  if constexpr (L >= 32) v = fmaxf(v, xshfl<16>(v));
  if constexpr (L >= 16) v = fmaxf(v, xshfl<8>(v));
  if constexpr (L >= 8) v = fmaxf(v, xshfl<4>(v));
  if constexpr (L >= 4) v = fmaxf(v, xshfl<2>(v));
  if constexpr (L >= 2) v = fmaxf(v, xshfl<1>(v));
  return v;
}
template <int L>
__device__ __forceinline__ unsigned lane_max(unsigned v) {
  if constexpr (L >= 64) v = max(v, (unsigned)xshfl<32>((int)v));
  if constexpr (L >= 32) v = max(v, (unsigned)xshfl<16>((int)v));
  if constexpr (L >= 16) v = max(v, (unsigned)xshfl<8>((int)v));
  if constexpr (L >= 8) v = max(v, (unsigned)xshfl<4>((int)v));
  if constexpr (L >= 4) v = max(v, (unsigned)xshfl<2>((int)v));
  if constexpr (L >= 2) v = max(v, (unsigned)xshfl<1>((int)v));
  return v;
}

// the same over 16-lane rows in the ascending order 1, 2, 4, 8 (the softmax loops `for (o = 1; o < 16; o <<= 1)`)
__device__ __forceinline__ float lane_sum16_up(float v) {
  v += xshfl<1>(v);
  v += xshfl<2>(v);
  v += xshfl<4>(v);
  v += xshfl<8>(v);
  return v;
}
__device__ __forceinline__ float lane_max16_up(float v) {
  v = fmaxf(v, xshfl<1>(v));
  v = fmaxf(v, xshfl<2>(v));
  v = fmaxf(v, xshfl<4>(v));
  v = fmaxf(v, xshfl<8>(v));
  return v;
}

}  // namespace vv
