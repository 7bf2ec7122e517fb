// cfp_lane.h -- cross-lane moves of complex values inside a wave64 (gfx950), used by the lane
// DFTs of the 3-sweep kernels (cfp_three_pass.hip, cfp_wave_three.hip).  DPP moves run on the
// VALU; lane ^ 16 has no DPP form on gfx9 and takes ds_swizzle (LDS pipe, no LDS memory).
#pragma once
#include "cfp_fft_device.h"

namespace cfp {
namespace {

// DPP controls: quad_perm lane ^ 1, ^ 2, ^ 3; row_half_mirror (lane ^ 7 within 8 lanes);
// row_ror:8 (lane ^ 8 within a row of 16)
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_XOR3 = 0x1B, DPP_HALF_MIRROR = 0x141, DPP_ROW_ROR8 = 0x128;
// whole-wave shifts by one lane (gfx9 DPP): wave_shr:1 gives lane L the value of lane L - 1,
// wave_shl:1 that of lane L + 1 (lanes 0 / 63 get nothing defined)
constexpr int DPP_WAVE_SHR1 = 0x138, DPP_WAVE_SHL1 = 0x130;
// ds_swizzle bit mode: and 0x1f, or 0, xor 0x10 (lane ^ 16 within 32 lanes)
constexpr int SWZ_XOR16 = (0x10 << 10) | 0x1f;

template <int M>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), M, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), M, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int M>
__device__ __forceinline__ cd dpp_c(cd v) { return make_cd(dpp_d<M>(v.x), dpp_d<M>(v.y)); }
// lane ^ 4: mirror within 8 lanes (7 - j), then reverse within the quad (^ 3)
__device__ __forceinline__ cd lane_xor4(cd v) { return dpp_c<DPP_XOR3>(dpp_c<DPP_HALF_MIRROR>(v)); }
__device__ __forceinline__ cd lane_xor8(cd v) { return dpp_c<DPP_ROW_ROR8>(v); }
__device__ __forceinline__ double swz_xor16(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(b & 0xffffffffll), SWZ_XOR16);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), SWZ_XOR16);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ cd lane_xor16(cd v) { return make_cd(swz_xor16(v.x), swz_xor16(v.y)); }
__device__ __forceinline__ cd mul_mi(cd v) { return make_cd(v.y, -v.x); }  // x W_4 = x (-i)

// register <-> lane-bit transposes (v_permlane32_swap: lane bit 5, v_permlane16_swap: bit 4)
// (a, b) -> lanes with bit B clear: (a[L], a[L ^ 2^B]); set: (b[L ^ 2^B], b[L])
template <int B>
__device__ __forceinline__ void swap32(unsigned& a, unsigned& b) {
  if constexpr (B == 5) {
    const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    a = r[0];
    b = r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    a = r[0];
    b = r[1];
  }
}
template <int B>
__device__ __forceinline__ void swap_d(double& a, double& b) {
  unsigned long long ua = (unsigned long long)__double_as_longlong(a),
                     ub = (unsigned long long)__double_as_longlong(b);
  unsigned al = (unsigned)ua, ah = (unsigned)(ua >> 32), bl = (unsigned)ub, bh = (unsigned)(ub >> 32);
  swap32<B>(al, bl);
  swap32<B>(ah, bh);
  a = __longlong_as_double((long long)(((unsigned long long)ah << 32) | al));
  b = __longlong_as_double((long long)(((unsigned long long)bh << 32) | bl));
}
template <int B>
__device__ __forceinline__ void swap_c(cd& a, cd& b) {
  swap_d<B>(a.x, b.x);
  swap_d<B>(a.y, b.y);
}

}  // namespace
// sum over the wave's 64 lanes (every lane gets it): DPP within rows, swizzle across 16, permlane32
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<DPP_XOR1>(v);
  v += dpp_d<DPP_XOR2>(v);
  v += dpp_d<DPP_XOR3>(dpp_d<DPP_HALF_MIRROR>(v));  // lane ^ 4
  v += dpp_d<DPP_ROW_ROR8>(v);
  v += swz_xor16(v);
  double w = v;
  swap_d<5>(v, w);  // lanes < 32 get (v, v[L + 32]) pairs' partner in w
  return v + w;
}

}  // namespace cfp
