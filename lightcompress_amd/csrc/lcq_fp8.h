// FP8 (OCP E4M3FN / E5M2) scalar encoders and decoders shared by the FP8 quant kernels
// (fp8.hip), the float-quant auto-clip search (awq.hip) and the float-quant GPTQ column loop
// (gptq.hip). Encoders reproduce c10's Float8_e4m3fn / Float8_e5m2 conversion bit for bit;
// fp8_sat<FMT> is the saturation of FloatQuantizer's float_quantize stand-in.
#pragma once

#include "lcq_common.h"

namespace lcq {

// ---------------------------------------------------------------------------------------
// fp32 -> fp8 encoders with c10's exact rounding, and exact decoders
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t enc_e4m3(float f) {
  uint32_t b = __float_as_uint(f);
  const uint32_t sign = b & 0x80000000u;
  b ^= sign;
  uint32_t r;
  if (b >= (1087u << 20)) {
    r = 0x7f;
  } else if (b < (121u << 23)) {
    const float t = __uint_as_float(b) + __uint_as_float(141u << 23);
    r = (__float_as_uint(t) - (141u << 23)) & 0xffu;
  } else {
    const uint32_t odd = (b >> 20) & 1u;
    b += ((uint32_t)(7 - 127) << 23) + 0x7ffffu;
    b += odd;
    r = (b >> 20) & 0xffu;
  }
  return r | (sign >> 24);
}

__device__ __forceinline__ uint32_t enc_e5m2(float f) {
  uint32_t b = __float_as_uint(f);
  const uint32_t sign = b & 0x80000000u;
  b ^= sign;
  uint32_t r;
  if (b >= (143u << 23)) {
    r = b > 0x7f800000u ? 0x7fu : 0x7cu;
  } else if (b < (113u << 23)) {
    const float t = __uint_as_float(b) + __uint_as_float(134u << 23);
    r = (__float_as_uint(t) - (134u << 23)) & 0xffu;
  } else {
    const uint32_t odd = (b >> 21) & 1u;
    b += ((uint32_t)(15 - 127) << 23) + 0xfffffu;
    b += odd;
    r = (b >> 21) & 0xffu;
  }
  return r | (sign >> 24);
}

__device__ __forceinline__ float dec_e4m3(uint32_t u) {
  const uint32_t sign = (u & 0x80u) << 24;
  const uint32_t e = (u >> 3) & 15u, m = u & 7u;
  if (e == 15u && m == 7u) return __uint_as_float(0x7fc00000u | sign);
  if (e == 0u) return __uint_as_float(__float_as_uint((float)m * 0.001953125f) | sign);
  return __uint_as_float(sign | ((e + 120u) << 23) | (m << 20));
}

__device__ __forceinline__ float dec_e5m2(uint32_t u) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(u << 8));
}

template <int FMT>
__device__ __forceinline__ uint32_t enc(float f) {
  if constexpr (FMT == LCQ_FP8E4M3) return enc_e4m3(f);
  else return enc_e5m2(f);
}
template <int FMT>
__device__ __forceinline__ float dec(uint32_t u) {
  if constexpr (FMT == LCQ_FP8E4M3) return dec_e4m3(u);
  else return dec_e5m2(u);
}

// largest finite value of the format (torch.finfo(float8_*).max)
template <int FMT>
__device__ __forceinline__ constexpr float fp8_fmax() {
  if constexpr (FMT == LCQ_FP8E4M3) return 448.0f;
  else return 57344.0f;
}

// clamp to +-finfo.max keeping NaN (comparisons with NaN are false): the float_quantize
// stand-in saturates, as the reference's Triton casts (cvt ... satfinite) and vLLM do
template <int FMT>
__device__ __forceinline__ float fp8_sat(float v) {
  const float m = fp8_fmax<FMT>();
  return v > m ? m : (v < -m ? -m : v);
}

// float_quantize(v) -> the fp8 value as fp32 (saturating RNE)
template <int FMT>
__device__ __forceinline__ float fp8_round(float v) {
  return dec<FMT>(enc<FMT>(fp8_sat<FMT>(v)));
}

}  // namespace lcq
