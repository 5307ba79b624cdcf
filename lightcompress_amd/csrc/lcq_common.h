// Shared device/host helpers for the lcq HIP library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "lcq.h"

namespace lcq {

// ----------------------------------------------------------------------------------------
// error plumbing (thread-local message, negative status codes)
// ----------------------------------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

#define LCQ_REQUIRE(cond, msg)                                                       \
  do {                                                                               \
    if (!(cond)) return ::lcq::fail(LCQ_EINVAL, std::string(__func__) + ": " + (msg)); \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// C[M, N] (ldc) = C - A B with A given k-major (element (m, k) at A[k lda + m]) and B [K, N]
// (ldb) row-major, on the LDS-DMA fp32 MFMA GEMM of chol.hip (tiled, no stream-K): every
// element is the k-ordered fmaf chain over k = 0 .. K-1 (bit-identical to lcq_gptq_trailing's
// register-staged kernel). LCQ_EUNSUP (nothing launched) when the operands are not 16-byte
// aligned row by row or K % 32 != 0. Used by lcq_gptq_trailing.
int gemm_f32_sub_akn(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                     const float* B, int64_t ldb, float* C, int64_t ldc, hipStream_t st);

inline int dtype_size(int dt) {
  switch (dt) {
    case LCQ_F32: return 4;
    case LCQ_F16: return 2;
    case LCQ_BF16: return 2;
    case LCQ_I8: return 1;
    case LCQ_U8: return 1;
    case LCQ_I32: return 4;
    case LCQ_FP8E4M3: return 1;
    case LCQ_F64: return 8;
    default: return 0;
  }
}
inline bool is_float_dt(int dt) { return dt == LCQ_F32 || dt == LCQ_F16 || dt == LCQ_BF16; }
inline bool is_code_dt(int dt) { return dt == LCQ_I8 || dt == LCQ_U8 || dt == LCQ_I32; }

// ----------------------------------------------------------------------------------------
// rounding to the compute dtype: every reference torch op on a bf16/fp16 tensor computes in
// fp32 and rounds its result (RNE) to the tensor dtype; we apply the same after each op.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ float bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return __uint_as_float((u | 0x00400000u) & 0xffff0000u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return __uint_as_float(u & 0xffff0000u);
}
// the same rounding on v_cvt_pk_bf16_f32 (gfx950; a NaN stays a NaN, payload not kept).
// Faster in the streaming quant kernels (14336x4096 fake quant 3.4 -> 4.3 TB/s); the auto-clip
// search keeps the integer form above (measured: 8 % slower with the conversion instruction).
__device__ __forceinline__ float bf16_rne_hw(float f) {
  const __bf16 h = (__bf16)f;
  return __uint_as_float((uint32_t)__builtin_bit_cast(uint16_t, h) << 16);
}

// IEEE quotient a / b from rb = RN(1 / b) (Markstein: the residual a - b*q0 is exact in one
// fma, the second fma rounds once). Equal to a / b whenever a, b and the quotient are finite
// and the quotient is not subnormal; callers guarantee finite inputs and bounded quotients.
__device__ __forceinline__ float div_mk(float a, float b, float rb) {
  const float q0 = a * rb;
  const float e = __fmaf_rn(-b, q0, a);
  return __fmaf_rn(e, rb, q0);
}
// a / b exactly as IEEE division, from rb = RN(1 / b): the Markstein quotient where the
// residual and the correction stay clear of the subnormal range (|a|, |q| >= 2^-100, q finite,
// rb normal), the IEEE division otherwise (zero, tiny, inf, NaN). Checked bit for bit against
// __fdiv_rn (tests/test_awq_gpu.py scale-broadcast exhaustive test, gptq in-block tests).
__device__ __forceinline__ float div_exact(float a, float b, float rb) {
  const float q = div_mk(a, b, rb);
  const float aq = fabsf(q);
  return (aq >= 0x1p-100f && aq <= 3.40282347e38f && fabsf(a) >= 0x1p-100f &&
          fabsf(rb) >= 0x1p-126f)
             ? q
             : __fdiv_rn(a, b);
}
__device__ __forceinline__ float f16_rne(float f) { return (float)(_Float16)f; }

// Translation units that define LCQ_BF16_HW before including this header (the streaming
// quant kernels) round on the conversion instruction everywhere (rnd, st8); the rest keep
// the integer form. Both are RNE; device code is per translation unit (no -fgpu-rdc).
#ifdef LCQ_BF16_HW
#define LCQ_BF16_ROUND bf16_rne_hw
#else
#define LCQ_BF16_ROUND bf16_rne
#endif

template <int CT>
__device__ __forceinline__ float rnd(float v) {
  if constexpr (CT == LCQ_BF16) return LCQ_BF16_ROUND(v);
  else if constexpr (CT == LCQ_F16) return f16_rne(v);
  else return v;
}

// quant.py:545-559 (get_qparams) with every op rounded to the compute dtype CT.
template <int CT>
__device__ __forceinline__ void qparams_ct(float mn, float mx, float qmin, float qmax, int sym,
                                           float& s, float& z) {
  const float lo = rnd<CT>(1e-5f);
  if (sym) {
    float am = fmaxf(fabsf(mx), fabsf(mn));
    am = fmaxf(am, lo);           // .clamp(min=1e-5)
    s = rnd<CT>(am / qmax);       // abs_max / qmax
    z = 0.f;
  } else {
    float r = rnd<CT>(mx - mn);
    r = fmaxf(r, lo);
    s = rnd<CT>(r / (qmax - qmin));
    float t = rnd<CT>(rintf(rnd<CT>(mn / s)));  // torch.round(min_val / scales)
    t = rnd<CT>(qmin - t);
    z = fminf(fmaxf(t, qmin), qmax);              // .clamp(qmin, qmax)
  }
}
__device__ __forceinline__ void qparams_f32(float mn, float mx, float qmin, float qmax, int sym,
                                            float& s, float& z) {
  qparams_ct<LCQ_F32>(mn, mx, qmin, qmax, sym, s, z);
}

// Learnable clip range (clip_version v2): torch.nn.Sigmoid, auto_clip.py:41 logit
// log(x / (1 - x)) and quant.py:205-219 get_learnable_range, every tensor op rounded to CT as
// the reference's CT tensors are. Sigmoid and log evaluate in fp32 and round once, like
// torch-CPU's reduced-float kernels; expf / logf and torch-CPU's vectorised exp / log may
// differ in the last fp32 ulp, which moves the CT result only at a rounding tie.
template <int CT>
__device__ __forceinline__ float sigmoid_ct(float f) {
  return rnd<CT>(1.0f / (1.0f + expf(-f)));
}
template <int CT>
__device__ __forceinline__ float logit_ct(float x) {
  return rnd<CT>(logf(rnd<CT>(x / rnd<CT>(1.0f - x))));
}
// (mn, mx): the group's min / max on entry, the learnable range on exit. sym: only the upper
// factor is used; asym: both, and the range is left alone without a lower factor.
template <int CT>
__device__ __forceinline__ void learnable_range(float& mn, float& mx, float up, float low,
                                                bool has_low, int sym) {
  if (sym) {
    float am = fmaxf(fmaxf(fabsf(mx), fabsf(mn)), rnd<CT>(1e-5f));  // .clamp(min=1e-5)
    am = rnd<CT>(sigmoid_ct<CT>(up) * am);
    mn = -am;
    mx = am;
  } else if (has_low) {
    mn = rnd<CT>(sigmoid_ct<CT>(low) * mn);
    mx = rnd<CT>(sigmoid_ct<CT>(up) * mx);
  }
}

// load/store one element of dtype DT as float
template <int DT>
__device__ __forceinline__ float ld1(const void* p, int64_t i) {
  if constexpr (DT == LCQ_F32) return reinterpret_cast<const float*>(p)[i];
  else if constexpr (DT == LCQ_BF16)
    return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(p)[i] << 16);
  else if constexpr (DT == LCQ_F16) return (float)reinterpret_cast<const _Float16*>(p)[i];
  else if constexpr (DT == LCQ_I32) return (float)reinterpret_cast<const int32_t*>(p)[i];
  else if constexpr (DT == LCQ_I8) return (float)reinterpret_cast<const int8_t*>(p)[i];
  else if constexpr (DT == LCQ_U8) return (float)reinterpret_cast<const uint8_t*>(p)[i];
  else return 0.f;
}

// store a float that is already exactly representable in DT (or round it RNE)
template <int DT>
__device__ __forceinline__ void st1(void* p, int64_t i, float v) {
  if constexpr (DT == LCQ_F32) reinterpret_cast<float*>(p)[i] = v;
  else if constexpr (DT == LCQ_BF16)
    reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)(__float_as_uint(LCQ_BF16_ROUND(v)) >> 16);
  else if constexpr (DT == LCQ_F16) reinterpret_cast<_Float16*>(p)[i] = (_Float16)v;
}

// 8 consecutive elements <-> float[8] with 16-byte vector accesses (Guideline 13)
template <int DT>
__device__ __forceinline__ void ld8(const void* base, int64_t e0, float (&v)[8]) {
  if constexpr (DT == LCQ_F32) {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + e0);
    float4 a = p[0], b = p[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + e0);
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (DT == LCQ_BF16) {
        v[2 * k] = __uint_as_float(w[k] << 16);
        v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      } else {
        v[2 * k] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[k] & 0xffffu));
        v[2 * k + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[k] >> 16));
      }
    }
  }
}

template <int DT>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (DT == LCQ_BF16) {
    return (__float_as_uint(LCQ_BF16_ROUND(a)) >> 16) |
           (__float_as_uint(LCQ_BF16_ROUND(b)) & 0xffff0000u);
  } else {
    uint16_t lo = __builtin_bit_cast(uint16_t, (_Float16)a);
    uint16_t hi = __builtin_bit_cast(uint16_t, (_Float16)b);
    return (uint32_t)lo | ((uint32_t)hi << 16);
  }
}

template <int DT>
__device__ __forceinline__ void st8(void* base, int64_t e0, const float (&v)[8]) {
  if constexpr (DT == LCQ_F32) {
    float4* p = reinterpret_cast<float4*>(reinterpret_cast<float*>(base) + e0);
    p[0] = make_float4(v[0], v[1], v[2], v[3]);
    p[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    uint4 r;
    r.x = pack2<DT>(v[0], v[1]);
    r.y = pack2<DT>(v[2], v[3]);
    r.z = pack2<DT>(v[4], v[5]);
    r.w = pack2<DT>(v[6], v[7]);
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(base) + e0) = r;
  }
}

// grid sizing for streaming kernels (Guideline 11): cap and grid-stride
inline unsigned stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > 65535LL * 16) g = 65535LL * 16;
  return (unsigned)g;
}

}  // namespace lcq
