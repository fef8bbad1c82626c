// osc_wave_sum.hpp -- 64-lane butterfly reductions (sum, max, (value, index) min) of the assembly,
// fallback and dual kernels, in the shuffle butterfly's exact order (xor 32, 16, 8, 4, 2, 1;
// every lane ends with the same bits) but with each level's partner fetched by a VALU lane
// crossing instead of a ds_bpermute round trip: v_permlane32_swap / v_permlane16_swap (gfx950)
// for xor 32 / 16, DPP for the rest.  Checked bit for bit against the shuffle form by
// tools/mb_wave_sum.hip (596 -> 231 clocks per 64-lane double sum).
#pragma once
#include "osc_device.hpp"

namespace osc {

// lane ^ O's 32-bit value
template <int O>
__device__ __forceinline__ unsigned xor_partner_u32(unsigned x, int lane) {
  if constexpr (O == 32) {
    // the swap pair: the lane keeps its own value in one result and finds its partner's in the other
    const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return lane >= 32 ? p[0] : p[1];
  } else if constexpr (O == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane & 16) ? p[0] : p[1];
  } else if constexpr (O == 8) {
    return static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x128, 0xf, 0xf,
                                                          false));   // row_ror:8
  } else if constexpr (O == 4) {
    const int up = __builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x104, 0xf, 0xf, false);  // shl:4
    const int dn = __builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x114, 0xf, 0xf, false);  // shr:4
    return static_cast<unsigned>((lane & 4) ? dn : up);
  } else if constexpr (O == 2) {
    return static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x4E, 0xf, 0xf,
                                                          false));   // quad_perm [2,3,0,1]
  } else {
    static_assert(O == 1, "xor level");
    return static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xB1, 0xf, 0xf,
                                                          false));   // quad_perm [1,0,3,2]
  }
}

template <int O>
__device__ __forceinline__ double xor_partner(double v, int lane) {
  const long long x = __double_as_longlong(v);
  const unsigned lo = xor_partner_u32<O>(static_cast<unsigned>(x), lane);
  const unsigned hi = xor_partner_u32<O>(static_cast<unsigned>(x >> 32), lane);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | lo);
}

__device__ __forceinline__ int wave_lane() { return static_cast<int>(threadIdx.x) & 63; }

// sum over the 64 lanes, the same bits on every lane
__device__ __forceinline__ double wave_sum_fast(double v) {
  const int lane = wave_lane();
  v += xor_partner<32>(v, lane);
  v += xor_partner<16>(v, lane);
  v += xor_partner<8>(v, lane);
  v += xor_partner<4>(v, lane);
  v += xor_partner<2>(v, lane);
  v += xor_partner<1>(v, lane);
  return v;
}

__device__ __forceinline__ double wave_max_fast(double v) {
  const int lane = wave_lane();
  v = fmax(v, xor_partner<32>(v, lane));
  v = fmax(v, xor_partner<16>(v, lane));
  v = fmax(v, xor_partner<8>(v, lane));
  v = fmax(v, xor_partner<4>(v, lane));
  v = fmax(v, xor_partner<2>(v, lane));
  v = fmax(v, xor_partner<1>(v, lane));
  return v;
}

// (value, index) minimum, the lowest index among ties
template <int O>
__device__ __forceinline__ void argmin_level(double& v, int& idx, int lane) {
  const double ov = xor_partner<O>(v, lane);
  const int oi = static_cast<int>(xor_partner_u32<O>(static_cast<unsigned>(idx), lane));
  if (ov < v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}
__device__ __forceinline__ void wave_argmin_fast(double& v, int& idx) {
  const int lane = wave_lane();
  argmin_level<32>(v, idx, lane);
  argmin_level<16>(v, idx, lane);
  argmin_level<8>(v, idx, lane);
  argmin_level<4>(v, idx, lane);
  argmin_level<2>(v, idx, lane);
  argmin_level<1>(v, idx, lane);
}

// (value, index) maximum with the lowest index among ties (the dual kernel's column pivoting)
template <int O>
__device__ __forceinline__ void argmax_level(double& v, int& idx, int lane) {
  const double ov = xor_partner<O>(v, lane);
  const int oi = static_cast<int>(xor_partner_u32<O>(static_cast<unsigned>(idx), lane));
  if (ov > v || (ov == v && oi < idx)) {
    v = ov;
    idx = oi;
  }
}
__device__ __forceinline__ void wave_argmax_fast(double& v, int& idx) {
  const int lane = wave_lane();
  argmax_level<32>(v, idx, lane);
  argmax_level<16>(v, idx, lane);
  argmax_level<8>(v, idx, lane);
  argmax_level<4>(v, idx, lane);
  argmax_level<2>(v, idx, lane);
  argmax_level<1>(v, idx, lane);
}

}  // namespace osc
