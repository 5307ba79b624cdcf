// FP8 (E4M3FN / E5M2) quantization for gfx950 -- FloatQuantizer and the block-fp8 casts.
//
// Reference semantics:
//   FloatQuantizer (llmc/compression/quantization/quant.py:963-1229):
//     use_qtorch=True : s = clamp(absmax, 1e-5) / finfo.max (0-dim fp32) in the tensor dtype,
//                       q = float_quantize(x / s + 0, e, m, 'nearest'), x^ = (q - 0) * s
//                       (:982-996, :545-559, :1061-1076).  qtorch is not available anywhere in
//                       this build, so the rounding step is the native OCP cast that torch's
//                       `.to(torch.float8_*)` performs (c10 Float8_e4m3fn / Float8_e5m2:
//                       round-to-nearest-even, e4m3fn |v| >= 480 -> NaN, e5m2 >= 65536 -> inf).
//     use_qtorch=False: get_float_qparams (:1005-1027) -- per-element power-of-two scales,
//                       round(x / scale) (lcq_fp_emul_quant below).
//   per_block 128x128 (:132-143 amax over .float(), :636-641 zero padding).
//   weight_cast_to_fp8 / weight_cast_to_bf16 / act_quant (kernel.py:7-138, quant.py:18-43).
//
// Design: HBM-bound streaming, 16-byte loads (8 elements per lane), scales reduced with
// wave butterflies / one LDS hop; the 128x128 block kernel keeps its block in VGPRs between
// the amax and the cast (one HBM read). No MFMA: this is byte work, not a GEMM.
#define LCQ_BF16_HW 1  // bf16 rounding on v_cvt_pk_bf16_f32 (see lcq_common.h)
#include "lcq_common.h"
#include "lcq_fp8.h"

namespace lcq {

__device__ __forceinline__ void st_codes8(void* p, int64_t e0, const uint32_t (&c)[8]) {
  const uint32_t lo = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
  const uint32_t hi = c[4] | (c[5] << 8) | (c[6] << 16) | (c[7] << 24);
  *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(p) + e0) = make_uint2(lo, hi);
}

__device__ __forceinline__ void st_any8(void* p, int dt, int64_t e0, const float (&v)[8]) {
  switch (dt) {
    case LCQ_F32: st8<LCQ_F32>(p, e0, v); break;
    case LCQ_BF16: st8<LCQ_BF16>(p, e0, v); break;
    case LCQ_F16: st8<LCQ_F16>(p, e0, v); break;
    default: break;
  }
}

struct Fp8Args {
  const void* x;
  int64_t rows, cols, group;
  float qmax, clamp_min;
  int add_zero;              // quant.py quant(): scales 0 -> 1, `+ zeros` (0.0) after the division
  int saturate;              // float_quantize stand-in: clamp to +-finfo.max before the cast
  const float* tensor_amax;  // per-tensor mode: device scalar from lcq_absmax
  void* codes;
  void* fq;
  int fq_dt;
  void* s_out;
};

// scale for one group (quant.py:545-559 with a 0-dim fp32 qmax): the clamp compares in the
// tensor dtype CT, the division rounds to SCT -- CT for [rows, 1] scales, fp32 for per-tensor
// (0-dim / 0-dim promotes to fp32). quant() then maps a zero scale to 1 (quant.py:1062).
template <int CT, int SCT = CT>
__device__ __forceinline__ float fp8_scale(float amax, float qmax, float clamp_min,
                                           int quant_py) {
  float am = amax;
  if (clamp_min > 0.f) am = fmaxf(am, rnd<CT>(clamp_min));
  float s = rnd<SCT>(am / qmax);
  if (quant_py && s == 0.f) s = 1.f;
  return s;
}

// x -> code / fake-quant for 8 elements sharing scale s
template <int CT, int FMT>
__device__ __forceinline__ void fp8_qdq8(const float (&w)[8], float s, int add_zero,
                                         int saturate, uint32_t (&c)[8], float (&dq)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = rnd<CT>(w[j] / s);
    if (add_zero) v = rnd<CT>(v + 0.0f);  // `+ zeros`: -0 -> +0
    if (saturate) v = fp8_sat<FMT>(v);
    c[j] = enc<FMT>(v);
    dq[j] = dec<FMT>(c[j]) * s;  // fp32 q times the scale (promotes to fp32), exact
  }
}

template <int CT, int FMT>
__device__ __forceinline__ void fp8_emit(const Fp8Args& a, int64_t e0, const float (&w)[8],
                                         float s) {
  uint32_t c[8];
  float dq[8];
  fp8_qdq8<CT, FMT>(w, s, a.add_zero, a.saturate, c, dq);
  if (a.codes) st_codes8(a.codes, e0, c);
  if (a.fq) st_any8(a.fq, a.fq_dt, e0, dq);
}

// ---- groups of L*8 elements (L adjacent lanes) -----------------------------------------
template <int XT, int CT, int FMT, int L>
__global__ void __launch_bounds__(256) k_fp8_lanes(Fp8Args a) {
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8;
    float w[8];
    ld8<XT>(a.x, e0, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j]);
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(w[j]));
#pragma unroll
    for (int m = L / 2; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
    const float s = fp8_scale<CT>(am, a.qmax, a.clamp_min, a.add_zero);
    fp8_emit<CT, FMT>(a, e0, w, s);
    if (a.s_out && (e0 % a.group) == 0) st1<CT>(a.s_out, e0 / a.group, s);
  }
}

// ---- one 256-thread workgroup per wide group (per-channel / per-token rows) ------------
template <int XT, int CT, int FMT>
__global__ void __launch_bounds__(256) k_fp8_rows(Fp8Args a) {
  __shared__ float red[4];
  const int64_t gi = blockIdx.x;
  const int64_t base = gi * a.group;
  const int64_t n8 = a.group / 8;
  float am = 0.f;
  for (int64_t c = threadIdx.x; c < n8; c += 256) {
    float w[8];
    ld8<XT>(a.x, base + c * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(rnd<CT>(w[j])));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = fp8_scale<CT>(am, a.qmax, a.clamp_min, a.add_zero);
  for (int64_t c = threadIdx.x; c < n8; c += 256) {
    float w[8];
    ld8<XT>(a.x, base + c * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j]);
    fp8_emit<CT, FMT>(a, base + c * 8, w, s);
  }
  if (threadIdx.x == 0 && a.s_out) st1<CT>(a.s_out, gi, s);
}

// ---- per-tensor: scale from a device amax (lcq_absmax), element-parallel ----------------
// the scale is a 0-dim fp32 tensor; torch divides the CT tensor by it in fp32 (the CPU scalar
// operand is not rounded to CT) and rounds the quotient to CT.
template <int XT, int CT, int FMT>
__global__ void __launch_bounds__(256) k_fp8_tensor(Fp8Args a) {
  const float s = fp8_scale<CT, LCQ_F32>(*a.tensor_amax, a.qmax, a.clamp_min, a.add_zero);
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    float w[8];
    ld8<XT>(a.x, t * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j]);
    fp8_emit<CT, FMT>(a, t * 8, w, s);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.s_out) st1<LCQ_F32>(a.s_out, 0, s);
}

// ---- static scales (quant.py:1061-1076 with given scales): s = scales[e / group] ---------
__device__ __forceinline__ float ld_scale(const void* p, int dt, int64_t i) {
  switch (dt) {
    case LCQ_F32: return ld1<LCQ_F32>(p, i);
    case LCQ_BF16: return ld1<LCQ_BF16>(p, i);
    default: return ld1<LCQ_F16>(p, i);
  }
}

template <int XT, int CT, int FMT>
__global__ void __launch_bounds__(256) k_fp8_static(Fp8Args a, const void* s_in, int s_dt) {
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8;
    // the scale keeps its own dtype: a 0-dim scale is a CPU scalar to torch (opmath), and a
    // dim scale is promoted with x, so CT is never narrower than it
    float s = ld_scale(s_in, s_dt, e0 / a.group);
    if (s == 0.f) s = 1.f;  // scales[scales == 0] = 1 (quant.py:1062)
    float w[8];
    ld8<XT>(a.x, e0, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j]);
    fp8_emit<CT, FMT>(a, e0, w, s);
  }
}

// ---- max |x| over a whole tensor (values are >= 0, so float order == uint order) -------
template <int XT>
__global__ void __launch_bounds__(256) k_absmax(const void* x, int64_t n, uint32_t* partials) {
  __shared__ float red[4];
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  float am = 0.f;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    float w[8];
    ld8<XT>(x, t * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(w[j]));
  }
  const int64_t tail = n8 * 8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tail < n) am = fmaxf(am, fabsf(ld1<XT>(x, tail)));
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0)
    partials[blockIdx.x] = __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// ---- 128x128 (BS x BS) blocks: amax over the block in fp32, block held in VGPRs ----------
// quant.py per_block: amax of |x|.float() over the block, s = clamp(amax, 1e-5) / 448 (fp32),
// q = cast(x.float() / s + 0); kernel.py weight_cast_to_fp8: same without the clamp / +0.
template <int XT, int FMT>
__global__ void __launch_bounds__(256) k_fp8_blocks(Fp8Args a, int64_t M, int64_t N) {
  constexpr int BS = 128, RPI = 256 / (BS / 8), IT = BS / RPI;  // 16 rows per pass, 8 passes
  __shared__ float red[4];
  const int64_t r0 = (int64_t)blockIdx.y * BS, c0 = (int64_t)blockIdx.x * BS;
  const int lr = threadIdx.x / (BS / 8), lc = (threadIdx.x % (BS / 8)) * 8;
  const int64_t col = c0 + lc;
  const bool cok = col < N;  // N % 8 == 0, so a lane's 8 columns are all in or all out
  float w[IT][8];
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int64_t row = r0 + i * RPI + lr;
    if (cok && row < M) {
      ld8<XT>(a.x, row * N + col, w[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) w[i][j] = 0.f;  // quant.py zero padding
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(w[i][j]));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = fp8_scale<LCQ_F32>(am, a.qmax, a.clamp_min, a.add_zero);
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int64_t row = r0 + i * RPI + lr;
    if (cok && row < M) fp8_emit<LCQ_F32, FMT>(a, row * N + col, w[i], s);
  }
  if (threadIdx.x == 0 && a.s_out)
    reinterpret_cast<float*>(a.s_out)[blockIdx.y * gridDim.x + blockIdx.x] = s;
}

// ---- block-fp8 -> per-tensor fp8, bf16 intermediate kept in registers ------------------
// The reference deploy of an fp8 checkpoint weight (module_utils.py:917-922 + quant.py:
// 1191-1221): w = bf16(float(code) * s_inv[block]) (weight_cast_to_bf16), then per-tensor
// FloatQuantizer real quant of w. Pass 1 = max|w| over the dequantized values, pass 2 =
// dequantize again and quantize: 1 + 1 B read, 1 B written per element (the composed chain
// moves 8 B per element).
template <int FIN>
__device__ __forceinline__ void deq8_row(const uint8_t* crow, float sc, int c, float (&w)[8]) {
  const uint2 u = *reinterpret_cast<const uint2*>(crow + c);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w[j] = bf16_rne(dec<FIN>((u.x >> (8 * j)) & 0xffu) * sc);
    w[4 + j] = bf16_rne(dec<FIN>((u.y >> (8 * j)) & 0xffu) * sc);
  }
}

// Row-walking traversal shared by the block-fp8 kernels: workgroup b takes rows b, b+G, ...;
// its 256 threads stride the row in 8-element chunks. Index math is 32-bit and per row (no
// per-element 64-bit division).
#define LCQ_ROWS_BEGIN(M, N, bs, ROWVAR)                                               \
  for (int64_t ROWVAR = blockIdx.x; ROWVAR < (M); ROWVAR += gridDim.x) {               \
    const int nb_ = (int)(((N) + (bs)-1) / (bs));                                      \
    const int rb_ = (int)(ROWVAR / (bs));                                              \
    for (int c = threadIdx.x * 8; c < (int)(N); c += 256 * 8) {                        \
      const int cbk_ = c / (bs);
#define LCQ_ROWS_END \
  }                  \
  }

// ---- batched form: blockIdx.y = tensor; descriptors in device memory ------------------
struct Fp8Desc {
  const uint8_t* codes;
  const float* s_inv;
  uint8_t* out;
  int64_t M, N;
};

// max over the np partials of one tensor (float bits of values >= 0 / NaN order as uints)
__device__ __forceinline__ float fold_partials(const uint32_t* p, int np) {
  __shared__ uint32_t red[4];
  uint32_t m = 0;
  for (int i = threadIdx.x; i < np; i += 256) m = max(m, p[i]);
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, k, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  return __uint_as_float(max(max(red[0], red[1]), max(red[2], red[3])));
}

template <int FIN>
__global__ void __launch_bounds__(256) k_absmax_blockfp8_many(const Fp8Desc* d, Fp8Desc one,
                                                              int bs, uint32_t* partials) {
  __shared__ float red[4];
  const Fp8Desc t = d ? d[blockIdx.y] : one;
  float am = 0.f;
  LCQ_ROWS_BEGIN(t.M, t.N, bs, r)
    float w[8];
    deq8_row<FIN>(t.codes + r * t.N, t.s_inv[rb_ * nb_ + cbk_], c, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(w[j]));
  LCQ_ROWS_END
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0)
    partials[(int64_t)blockIdx.y * LCQ_FP8_PARTIALS + blockIdx.x] =
        __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

template <int FIN, int FOUT>
__global__ void __launch_bounds__(256) k_requant_blockfp8_many(const Fp8Desc* d, Fp8Desc one,
                                                               int bs, const uint32_t* partials,
                                                               float qmax, float clamp_min,
                                                               int add_zero, float* s_out) {
  const Fp8Desc t = d ? d[blockIdx.y] : one;
  const float am = fold_partials(partials + (int64_t)blockIdx.y * LCQ_FP8_PARTIALS, gridDim.x);
  const float sc = fp8_scale<LCQ_BF16, LCQ_F32>(am, qmax, clamp_min, add_zero);
  LCQ_ROWS_BEGIN(t.M, t.N, bs, r)
    float w[8], dq[8];
    uint32_t cc[8];
    deq8_row<FIN>(t.codes + r * t.N, t.s_inv[rb_ * nb_ + cbk_], c, w);
    fp8_qdq8<LCQ_BF16, FOUT>(w, sc, add_zero, 0, cc, dq);
    st_codes8(t.out, r * t.N + c, cc);
  LCQ_ROWS_END
  if (blockIdx.x == 0 && threadIdx.x == 0) s_out[blockIdx.y] = sc;
}

__global__ void __launch_bounds__(256) k_fold_partials(const uint32_t* partials, int np,
                                                       float* out) {
  const float m = fold_partials(partials, np);
  if (threadIdx.x == 0) *out = m;
}

// ---- fast path (block 128, N % 16 == 0): 16 codes per lane, hardware OCP conversions -----
// Pass 1 never dequantizes element-wise: w = bf16(float(code) * s_inv) is monotonic in
// |code| for a fixed block scale, so max|w| over a 16-code chunk is bf16(dec(max|code|) *
// |s_inv|) with the byte max taken on the sign-stripped codes (sign-magnitude order == value
// order for e4m3fn and e5m2; NaN/inf codes sort above every finite one, and float bits of
// non-negative values compare like uints, so NaN propagates into the amax as torch's
// abs().amax() does). Pass 2 decodes with v_cvt_pk_f32_{fp8,bf8} (exact), rounds with
// v_cvt_pk_bf16_f32 (RNE), divides by the per-tensor scale with a Markstein quotient (IEEE
// quotient given RN(1/s)) and encodes with v_cvt_pk_{fp8,bf8}_f32 (RNE); a chunk whose
// |quotient| reaches c10's overflow band (e4m3fn > 464, e5m2 >= 61440, or NaN) takes the
// software encoder (enc_e4m3/enc_e5m2), so the codes are c10's for every input.
typedef float v2f_t __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
typedef unsigned short v2u16_t __attribute__((ext_vector_type(2)));

template <int FMT, bool HI>
__device__ __forceinline__ v2f_t hw_dec2(uint32_t u) {
  if constexpr (FMT == LCQ_FP8E4M3) return __builtin_amdgcn_cvt_pk_f32_fp8((int)u, HI);
  else return __builtin_amdgcn_cvt_pk_f32_bf8((int)u, HI);
}
template <int FMT>
__device__ __forceinline__ uint32_t hw_enc4(v2f_t a, v2f_t b) {
  int r;
  if constexpr (FMT == LCQ_FP8E4M3) {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a.x, a.y, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(b.x, b.y, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a.x, a.y, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(b.x, b.y, r, true);
  }
  return (uint32_t)r;
}
// first |v| bit pattern where c10's encoder leaves the RNE-in-range regime
template <int FMT>
__device__ __forceinline__ uint32_t enc_hw_limit() {
  if constexpr (FMT == LCQ_FP8E4M3) return 0x43e80000u;  // 464.0f: (464, 480) -> NaN code
  else return 0x476fffffu;                               // just below 61440.0f (rounds to inf)
}

__device__ __forceinline__ v2f_t bf16r_pk(v2f_t p) {  // RNE to bf16 and back, a pair
  const v2bf_t h = __builtin_convertvector(p, v2bf_t);
  const uint32_t u = __builtin_bit_cast(uint32_t, h);
  v2f_t r;
  r.x = __uint_as_float(u << 16);
  r.y = __uint_as_float(u & 0xffff0000u);
  return r;
}

__device__ __forceinline__ uint32_t absbyte_max16(const uint4 u) {
  const uint32_t m0 = u.x & 0x7f7f7f7fu, m1 = u.y & 0x7f7f7f7fu, m2 = u.z & 0x7f7f7f7fu,
                 m3 = u.w & 0x7f7f7f7fu;
  v2u16_t lo = __builtin_bit_cast(v2u16_t, m0 & 0x00ff00ffu);
  v2u16_t hi = __builtin_bit_cast(v2u16_t, m0 & 0xff00ff00u);
  lo = __builtin_elementwise_max(lo, __builtin_bit_cast(v2u16_t, m1 & 0x00ff00ffu));
  hi = __builtin_elementwise_max(hi, __builtin_bit_cast(v2u16_t, m1 & 0xff00ff00u));
  lo = __builtin_elementwise_max(lo, __builtin_bit_cast(v2u16_t, m2 & 0x00ff00ffu));
  hi = __builtin_elementwise_max(hi, __builtin_bit_cast(v2u16_t, m2 & 0xff00ff00u));
  lo = __builtin_elementwise_max(lo, __builtin_bit_cast(v2u16_t, m3 & 0x00ff00ffu));
  hi = __builtin_elementwise_max(hi, __builtin_bit_cast(v2u16_t, m3 & 0xff00ff00u));
  const uint32_t l = max((uint32_t)lo.x, (uint32_t)lo.y);
  const uint32_t h = max((uint32_t)hi.x, (uint32_t)hi.y) >> 8;
  return max(l, h);
}

// chunk k (16 codes) of an M x N tensor -> (row, 16-column index); valid while k < 2^24
__device__ __forceinline__ void chunk_rc(int k, int nc, float fr, int& row, int& c16) {
  row = (int)((float)k * fr);
  c16 = k - row * nc;
  if (c16 < 0) { --row; c16 += nc; }
  else if (c16 >= nc) { ++row; c16 -= nc; }
}

constexpr int F16_UNROLL = 2;  // 16-byte chunks per lane per iteration (loads in flight)

// the 16-code path needs whole 16-byte chunks, 16-byte aligned rows and k < 2^24
__device__ __forceinline__ bool fast16(const Fp8Desc& t) {
  return (t.N & 15) == 0 && t.M * t.N < (int64_t(1) << 28) &&
         ((reinterpret_cast<uintptr_t>(t.codes) | reinterpret_cast<uintptr_t>(t.out)) & 15) == 0;
}

// Pass 1 writes one partial max per workgroup (partials[tensor * LCQ_FP8_PARTIALS + bx]);
// pass 2's workgroups each fold the gridDim.x partials of their tensor. No device-scope
// atomics: thousands of workgroups hitting one address serialise at the memory side
// (measured: 172 us for 132 MB with one atomicMax per workgroup).
template <int FIN, int BU>
__global__ void __launch_bounds__(256) k_bmax16_many(const Fp8Desc* d, Fp8Desc one,
                                                     uint32_t* partials) {
  __shared__ uint32_t red[4];
  const Fp8Desc t = d ? d[blockIdx.y] : one;
  uint32_t am = 0;
  if (!fast16(t)) {  // ragged / unaligned / huge tensor: row walk, one element at a time
    for (int64_t r = blockIdx.x; r < t.M; r += gridDim.x) {
      const int nbc = (int)((t.N + 127) >> 7);
      for (int64_t c = threadIdx.x; c < t.N; c += 256) {
        const float w = bf16_rne(dec<FIN>(t.codes[r * t.N + c] & 0x7fu) *
                                 fabsf(t.s_inv[(r >> 7) * nbc + (c >> 7)]));
        am = max(am, __float_as_uint(w) & 0x7fffffffu);
      }
    }
  } else {
  const int nc = (int)(t.N >> 4), nbc = (int)((t.N + 127) >> 7);
  const int nk = (int)(t.M * t.N >> 4);
  const float fr = 1.0f / (float)nc;
  const int step = gridDim.x * 256 * BU;
  for (int k0 = blockIdx.x * 256 * BU + threadIdx.x; k0 < nk; k0 += step) {
    uint4 u[BU];
#pragma unroll
    for (int j = 0; j < BU; ++j) {
      const int k = k0 + j * 256;
      if (k < nk) u[j] = reinterpret_cast<const uint4*>(t.codes)[k];
    }
#pragma unroll
    for (int j = 0; j < BU; ++j) {
      const int k = k0 + j * 256;
      if (k < nk) {
        int row, c16;
        chunk_rc(k, nc, fr, row, c16);
        const float sc = fabsf(t.s_inv[(row >> 7) * nbc + (c16 >> 3)]);
        const float w = bf16_rne(dec<FIN>(absbyte_max16(u[j])) * sc);
        am = max(am, __float_as_uint(w) & 0x7fffffffu);
      }
    }
  }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) am = max(am, (uint32_t)__shfl_xor((int)am, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0)
    partials[(int64_t)blockIdx.y * LCQ_FP8_PARTIALS + blockIdx.x] =
        max(max(red[0], red[1]), max(red[2], red[3]));
}


template <int FIN, int FOUT, bool ADD_ZERO>
__global__ void __launch_bounds__(256) k_requant16_many(const Fp8Desc* d, Fp8Desc one,
                                                        const uint32_t* partials, int np,
                                                        float qmax, float clamp_min,
                                                        float* s_out) {
  const Fp8Desc t = d ? d[blockIdx.y] : one;
  const float am = fold_partials(partials + (int64_t)blockIdx.y * LCQ_FP8_PARTIALS, np);
  const float sc = fp8_scale<LCQ_BF16, LCQ_F32>(am, qmax, clamp_min, ADD_ZERO);
  const float rs = 1.0f / sc;  // RN(1/s): Markstein's reciprocal
  const int nc = (int)(t.N >> 4), nbc = (int)((t.N + 127) >> 7);
  const int nk = (int)(t.M * t.N >> 4);
  const float fr = 1.0f / (float)nc;
  const v2f_t s2 = {sc, sc}, r2 = {rs, rs};
  if (blockIdx.x == 0 && threadIdx.x == 0) s_out[blockIdx.y] = sc;
  if (!fast16(t)) {
    for (int64_t r = blockIdx.x; r < t.M; r += gridDim.x) {
      const int nbc = (int)((t.N + 127) >> 7);
      for (int64_t c = threadIdx.x; c < t.N; c += 256) {
        const float w = bf16_rne(dec<FIN>(t.codes[r * t.N + c]) * t.s_inv[(r >> 7) * nbc + (c >> 7)]);
        float v = bf16_rne(w / sc);
        if constexpr (ADD_ZERO) v = v + 0.0f;
        t.out[r * t.N + c] = (uint8_t)enc<FOUT>(v);
      }
    }
    return;
  }
  const int step = gridDim.x * 256 * F16_UNROLL;
  for (int k0 = blockIdx.x * 256 * F16_UNROLL + threadIdx.x; k0 < nk; k0 += step) {
    uint4 u[F16_UNROLL];
#pragma unroll
    for (int j = 0; j < F16_UNROLL; ++j) {
      const int k = k0 + j * 256;
      if (k < nk) u[j] = reinterpret_cast<const uint4*>(t.codes)[k];
    }
#pragma unroll
    for (int j = 0; j < F16_UNROLL; ++j) {
      const int k = k0 + j * 256;
      if (k >= nk) continue;
      int row, c16;
      chunk_rc(k, nc, fr, row, c16);
      const float si = t.s_inv[(row >> 7) * nbc + (c16 >> 3)];
      const v2f_t si2 = {si, si};
      const uint32_t in[4] = {u[j].x, u[j].y, u[j].z, u[j].w};
      v2f_t q[8];
      uint32_t big = 0;
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const v2f_t d2 = (p & 1) ? hw_dec2<FIN, true>(in[p >> 1]) : hw_dec2<FIN, false>(in[p >> 1]);
        const v2f_t w = bf16r_pk(d2 * si2);                                // weight_cast_to_bf16
        const v2f_t q0 = w * r2;
        const v2f_t e = __builtin_elementwise_fma(-s2, q0, w);
        v2f_t v = bf16r_pk(__builtin_elementwise_fma(e, r2, q0));        // bf16(w / s)
        if constexpr (ADD_ZERO) v = v + (v2f_t){0.0f, 0.0f};             // `+ zeros`: -0 -> +0
        q[p] = v;
        big = max(big, max(__float_as_uint(v.x) & 0x7fffffffu, __float_as_uint(v.y) & 0x7fffffffu));
      }
      uint4 o;
      uint32_t* op = reinterpret_cast<uint32_t*>(&o);
      if (big <= enc_hw_limit<FOUT>()) {
#pragma unroll
        for (int p = 0; p < 4; ++p) op[p] = hw_enc4<FOUT>(q[2 * p], q[2 * p + 1]);
      } else {
#pragma unroll
        for (int p = 0; p < 4; ++p)
          op[p] = enc<FOUT>(q[2 * p].x) | (enc<FOUT>(q[2 * p].y) << 8) |
                  (enc<FOUT>(q[2 * p + 1].x) << 16) | (enc<FOUT>(q[2 * p + 1].y) << 24);
      }
      reinterpret_cast<uint4*>(t.out)[k] = o;
    }
  }
}

// ---- block dequant: out = rnd_out(float(code) * s[block])  (weight_cast_to_bf16) --------
template <int FMT, int OT>
__global__ void __launch_bounds__(256) k_fp8_dequant_blocks(const uint8_t* codes,
                                                            const float* s, int64_t M,
                                                            int64_t N, int bs, void* out) {
  LCQ_ROWS_BEGIN(M, N, bs, r)
    const float sc = s[rb_ * nb_ + cbk_];
    const uint2 u = *reinterpret_cast<const uint2*>(codes + r * N + c);
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = dec<FMT>((u.x >> (8 * j)) & 0xffu) * sc;
      v[4 + j] = dec<FMT>((u.y >> (8 * j)) & 0xffu) * sc;
    }
    st8<OT>(out, r * N + c, v);
  LCQ_ROWS_END
}

// ---- use_qtorch=False: get_float_qparams emulation (quant.py:1005-1027, 1061-1076) ------
// Per group: maxval = max(max, -min); bias = 2^e - log2(maxval) + log2(2 - 2^-m) - 1;
// per element: xc = clamp(x, -maxval, maxval); ls = max(floor(log2|xc| + bias), 1);
// scale = 2^(ls - m - bias); x^ = round(xc / scale) * scale. Every op rounds to CT (the
// tensor dtype; fp32 when e >= 5). log2 / exp2 are evaluated in fp64 and rounded once, which
// equals torch-CPU's bf16/fp16 results for every input (checked exhaustively).
template <int CT>
__device__ __forceinline__ float emul_bias(float maxval, int e, int m) {
  const float l = rnd<CT>((float)log2((double)maxval));
  const float c = rnd<CT>((float)log2(2.0 - exp2(-(double)m)));
  float b = rnd<CT>((float)(1 << e) - l);
  b = rnd<CT>(b + c);
  return rnd<CT>(b - 1.0f);
}

template <int CT>
__device__ __forceinline__ float emul_qdq(float x, float maxval, float bias, int m) {
  const float xc = fminf(fmaxf(x, -maxval), maxval);
  const float lg = rnd<CT>((float)log2((double)fabsf(xc)));
  float ls = floorf(rnd<CT>(lg + bias));
  ls = (ls != ls) ? ls : fmaxf(ls, 1.0f);  // torch.clamp(min=1.0) keeps NaN; -inf -> 1
  float ex = rnd<CT>(ls - (float)m);
  ex = rnd<CT>(ex - bias);
  float sc = rnd<CT>((float)exp2((double)ex));
  if (sc == 0.f) sc = 1.f;  // scales[scales == 0] = 1
  float q = rnd<CT>(xc / sc);
  q = rintf(rnd<CT>(q + 0.0f));
  return rnd<CT>(q * sc);
}

template <int XT, int CT>
__global__ void __launch_bounds__(256) k_fp_emul_rows(const void* x, int64_t group, int e,
                                                      int m, void* out, int out_dt) {
  __shared__ float red[2][4];
  const int64_t gi = blockIdx.x;
  const int64_t base = gi * group;
  const int64_t n8 = group / 8;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t c = threadIdx.x; c < n8; c += 256) {
    float w[8];
    ld8<XT>(x, base + c * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mn = fminf(mn, w[j]);
      mx = fmaxf(mx, w[j]);
    }
  }
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, k, 64));
    mx = fmaxf(mx, __shfl_xor(mx, k, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = mn;
    red[1][threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  mn = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
  mx = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  const float maxval = rnd<CT>(fmaxf(mx, -mn));
  const float bias = emul_bias<CT>(maxval, e, m);
  for (int64_t c = threadIdx.x; c < n8; c += 256) {
    float w[8], o[8];
    ld8<XT>(x, base + c * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = emul_qdq<CT>(rnd<CT>(w[j]), maxval, bias, m);
    st_any8(out, out_dt, base + c * 8, o);
  }
}

static bool pow2_lanes(int64_t v) { return v >= 1 && v <= 64 && (v & (v - 1)) == 0; }

template <int XT, int CT, int FMT>
static void launch_groups(const Fp8Args& a, hipStream_t st) {
  const int64_t lanes = a.group / 8;
  const unsigned grid = stream_grid(a.rows * a.cols / 8, 256);
  if (a.tensor_amax) {
    hipLaunchKernelGGL((k_fp8_tensor<XT, CT, FMT>), grid, 256, 0, st, a);
    return;
  }
  switch (pow2_lanes(lanes) ? lanes : 0) {
    case 1: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 1>), grid, 256, 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 2>), grid, 256, 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 4>), grid, 256, 0, st, a); break;
    case 8: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 8>), grid, 256, 0, st, a); break;
    case 16: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 16>), grid, 256, 0, st, a); break;
    case 32: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 32>), grid, 256, 0, st, a); break;
    case 64: hipLaunchKernelGGL((k_fp8_lanes<XT, CT, FMT, 64>), grid, 256, 0, st, a); break;
    default:
      hipLaunchKernelGGL((k_fp8_rows<XT, CT, FMT>), dim3((unsigned)(a.rows * a.cols / a.group)),
                         256, 0, st, a);
  }
}

// x dtype == compute dtype (quant.py computes in the tensor dtype) or fp32 compute (kernel.py
// casts to fp32 first; per_block .float())
template <int XT, int FMT>
static int dispatch_ct(const Fp8Args& a, int ct, hipStream_t st) {
  if (ct == LCQ_F32) launch_groups<XT, LCQ_F32, FMT>(a, st);
  else if (ct == XT && XT == LCQ_BF16) launch_groups<XT, LCQ_BF16, FMT>(a, st);
  else if (ct == XT && XT == LCQ_F16) launch_groups<XT, LCQ_F16, FMT>(a, st);
  else return fail(LCQ_EINVAL, "lcq_fp8_quant: compute dtype must be fp32 or the x dtype");
  return check_launch("lcq_fp8_quant");
}

template <int FMT>
static int dispatch_x(const Fp8Args& a, int x_dtype, int ct, hipStream_t st) {
  switch (x_dtype) {
    case LCQ_F32: return dispatch_ct<LCQ_F32, FMT>(a, ct, st);
    case LCQ_BF16: return dispatch_ct<LCQ_BF16, FMT>(a, ct, st);
    default: return dispatch_ct<LCQ_F16, FMT>(a, ct, st);
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_absmax(const void* x, int x_dtype, int64_t n, void* out, void* workspace,
                          void* stream) {
  LCQ_REQUIRE(is_float_dt(x_dtype), "x dtype must be f32/f16/bf16");
  LCQ_REQUIRE(n > 0 && x != nullptr && out != nullptr && workspace != nullptr, "empty tensor");
  hipStream_t st = as_stream(stream);
  // one partial per workgroup, folded by a one-workgroup kernel (no contended atomics)
  const unsigned grid = std::min<unsigned>(stream_grid(n / 8 + 1, 256), LCQ_FP8_PARTIALS);
  uint32_t* p = reinterpret_cast<uint32_t*>(workspace);
  switch (x_dtype) {
    case LCQ_F32: hipLaunchKernelGGL(k_absmax<LCQ_F32>, grid, 256, 0, st, x, n, p); break;
    case LCQ_BF16: hipLaunchKernelGGL(k_absmax<LCQ_BF16>, grid, 256, 0, st, x, n, p); break;
    default: hipLaunchKernelGGL(k_absmax<LCQ_F16>, grid, 256, 0, st, x, n, p); break;
  }
  hipLaunchKernelGGL(k_fold_partials, 1, 256, 0, st, p, (int)grid, reinterpret_cast<float*>(out));
  return check_launch("lcq_absmax");
}

extern "C" int lcq_fp8_quant(const void* x, int x_dtype, int64_t rows, int64_t cols,
                             int64_t group, int fmt, int ct_dtype, float qmax,
                             float clamp_min, int add_zero, const void* tensor_amax,
                             void* codes_out,
                             void* fq_out, int fq_dtype, void* scales_out, void* stream) {
  LCQ_REQUIRE(is_float_dt(x_dtype), "x dtype must be f32/f16/bf16");
  LCQ_REQUIRE(fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2, "fmt must be e4m3fn or e5m2");
  LCQ_REQUIRE(rows > 0 && cols > 0, "empty tensor");
  if (group <= 0) group = cols;
  LCQ_REQUIRE(cols % group == 0, "cols not divisible by group size");
  LCQ_REQUIRE(group % 8 == 0, "group size must be a multiple of 8");
  LCQ_REQUIRE(fq_out == nullptr || is_float_dt(fq_dtype), "bad fq dtype");
  LCQ_REQUIRE(rows * cols / group <= 0x7fffffffLL, "too many groups");
  LCQ_REQUIRE(qmax > 0.f, "qmax must be positive");
  Fp8Args a{};
  a.x = x; a.rows = rows; a.cols = cols; a.group = group;
  a.qmax = qmax; a.clamp_min = clamp_min; a.add_zero = add_zero;
  a.tensor_amax = reinterpret_cast<const float*>(tensor_amax);
  a.codes = codes_out; a.fq = fq_out; a.fq_dt = fq_dtype; a.s_out = scales_out;
  hipStream_t st = as_stream(stream);
  return fmt == LCQ_FP8E4M3 ? dispatch_x<LCQ_FP8E4M3>(a, x_dtype, ct_dtype, st)
                            : dispatch_x<LCQ_FP8E5M2>(a, x_dtype, ct_dtype, st);
}

extern "C" int lcq_fp8_quant_static(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                    int64_t group, int fmt, int ct_dtype, const void* scales,
                                    int s_dtype, int add_zero, int saturate, void* codes_out,
                                    void* fq_out, int fq_dtype, void* stream) {
  LCQ_REQUIRE(is_float_dt(x_dtype) && is_float_dt(ct_dtype) && is_float_dt(s_dtype),
              "x / compute / scale dtypes must be f32/f16/bf16");
  LCQ_REQUIRE(fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2, "fmt must be e4m3fn or e5m2");
  LCQ_REQUIRE(rows > 0 && cols > 0 && scales != nullptr, "empty tensor or no scales");
  LCQ_REQUIRE(group > 0 && group % 8 == 0 && (rows * cols) % group == 0,
              "group must be a multiple of 8 that tiles the tensor");
  LCQ_REQUIRE(fq_out == nullptr || is_float_dt(fq_dtype), "bad fq dtype");
  Fp8Args a{};
  a.x = x; a.rows = rows; a.cols = cols; a.group = group;
  a.add_zero = add_zero; a.saturate = saturate;
  a.codes = codes_out; a.fq = fq_out; a.fq_dt = fq_dtype;
  const unsigned grid = stream_grid(rows * cols / 8, 256);
  hipStream_t st = as_stream(stream);
#define LCQ_ST(XT, CT, FMT) \
  hipLaunchKernelGGL((k_fp8_static<XT, CT, FMT>), grid, 256, 0, st, a, scales, s_dtype)
#define LCQ_ST_CT(XT, FMT)                                      \
  switch (ct_dtype) {                                           \
    case LCQ_F32: LCQ_ST(XT, LCQ_F32, FMT); break;              \
    case LCQ_BF16: LCQ_ST(XT, LCQ_BF16, FMT); break;            \
    default: LCQ_ST(XT, LCQ_F16, FMT); break;                   \
  }
#define LCQ_ST_X(FMT)                                           \
  switch (x_dtype) {                                            \
    case LCQ_F32: LCQ_ST_CT(LCQ_F32, FMT); break;               \
    case LCQ_BF16: LCQ_ST_CT(LCQ_BF16, FMT); break;             \
    default: LCQ_ST_CT(LCQ_F16, FMT); break;                    \
  }
  if (fmt == LCQ_FP8E4M3) {
    LCQ_ST_X(LCQ_FP8E4M3)
  } else {
    LCQ_ST_X(LCQ_FP8E5M2)
  }
#undef LCQ_ST_X
#undef LCQ_ST_CT
#undef LCQ_ST
  return check_launch("lcq_fp8_quant_static");
}

extern "C" int lcq_fp8_quant_blocks(const void* x, int x_dtype, int64_t M, int64_t N,
                                    int block, int fmt, float qmax, float clamp_min,
                                    int add_zero,
                                    void* codes_out, void* fq_out, int fq_dtype,
                                    void* scales_out, void* stream) {
  LCQ_REQUIRE(is_float_dt(x_dtype), "x dtype must be f32/f16/bf16");
  LCQ_REQUIRE(fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2, "fmt must be e4m3fn or e5m2");
  LCQ_REQUIRE(block == 128, "block size must be 128");
  LCQ_REQUIRE(M > 0 && N > 0 && N % 8 == 0, "N must be a positive multiple of 8");
  LCQ_REQUIRE(fq_out == nullptr || is_float_dt(fq_dtype), "bad fq dtype");
  LCQ_REQUIRE(qmax > 0.f, "qmax must be positive");
  Fp8Args a{};
  a.x = x; a.rows = M; a.cols = N; a.group = 0;
  a.qmax = qmax; a.clamp_min = clamp_min; a.add_zero = add_zero;
  a.codes = codes_out; a.fq = fq_out; a.fq_dt = fq_dtype; a.s_out = scales_out;
  const dim3 grid((unsigned)((N + block - 1) / block), (unsigned)((M + block - 1) / block));
  hipStream_t st = as_stream(stream);
#define LCQ_BLK(XT, FMT) hipLaunchKernelGGL((k_fp8_blocks<XT, FMT>), grid, 256, 0, st, a, M, N)
  if (fmt == LCQ_FP8E4M3) {
    switch (x_dtype) {
      case LCQ_F32: LCQ_BLK(LCQ_F32, LCQ_FP8E4M3); break;
      case LCQ_BF16: LCQ_BLK(LCQ_BF16, LCQ_FP8E4M3); break;
      default: LCQ_BLK(LCQ_F16, LCQ_FP8E4M3); break;
    }
  } else {
    switch (x_dtype) {
      case LCQ_F32: LCQ_BLK(LCQ_F32, LCQ_FP8E5M2); break;
      case LCQ_BF16: LCQ_BLK(LCQ_BF16, LCQ_FP8E5M2); break;
      default: LCQ_BLK(LCQ_F16, LCQ_FP8E5M2); break;
    }
  }
#undef LCQ_BLK
  return check_launch("lcq_fp8_quant_blocks");
}

extern "C" int lcq_fp8_dequant_blocks(const void* codes, int fmt, int64_t M, int64_t N,
                                      int block, const void* scales, void* out, int out_dtype,
                                      void* stream) {
  LCQ_REQUIRE(fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2, "fmt must be e4m3fn or e5m2");
  LCQ_REQUIRE(block > 0 && M > 0 && N > 0 && N % 8 == 0, "N must be a positive multiple of 8");
  LCQ_REQUIRE(N < 0x7fffffffLL, "rows longer than 2^31 elements");
  LCQ_REQUIRE(is_float_dt(out_dtype), "out dtype must be f32/f16/bf16");
  const unsigned grid = (unsigned)std::min<int64_t>(M, 65535);
  hipStream_t st = as_stream(stream);
  const uint8_t* c = reinterpret_cast<const uint8_t*>(codes);
  const float* s = reinterpret_cast<const float*>(scales);
#define LCQ_DQ(FMT, OT) \
  hipLaunchKernelGGL((k_fp8_dequant_blocks<FMT, OT>), grid, 256, 0, st, c, s, M, N, block, out)
  if (fmt == LCQ_FP8E4M3) {
    switch (out_dtype) {
      case LCQ_F32: LCQ_DQ(LCQ_FP8E4M3, LCQ_F32); break;
      case LCQ_BF16: LCQ_DQ(LCQ_FP8E4M3, LCQ_BF16); break;
      default: LCQ_DQ(LCQ_FP8E4M3, LCQ_F16); break;
    }
  } else {
    switch (out_dtype) {
      case LCQ_F32: LCQ_DQ(LCQ_FP8E5M2, LCQ_F32); break;
      case LCQ_BF16: LCQ_DQ(LCQ_FP8E5M2, LCQ_BF16); break;
      default: LCQ_DQ(LCQ_FP8E5M2, LCQ_F16); break;
    }
  }
#undef LCQ_DQ
  return check_launch("lcq_fp8_dequant_blocks");
}

// Both passes of the block-fp8 -> per-tensor deploy over n tensors (descriptors in device
// memory, or `one` by value when d == nullptr). Pass 1 writes LCQ_FP8_PARTIALS partial maxima
// per tensor into ws, pass 2 folds them: no device-scope atomics (thousands of workgroups
// hitting one address serialise at the memory side: 172 us vs 37 us for 132 MB of codes).
static int block_to_tensor(int n, const Fp8Desc* d, const Fp8Desc& one, int64_t max_elems,
                           int fmt_in, int block, int fmt_out, float qmax, float clamp_min,
                           int add_zero, void* ws, float* so, hipStream_t st) {
  uint32_t* part = reinterpret_cast<uint32_t*>(ws);
  if (block == 128) {
    // all tensors in one launch pair (grid.y = tensor): measured on MI355X, fewer launches
    // beat grouping for Infinity-Cache reuse of the re-read (96 DSv3 expert linears: 0.96 ms
    // in one group vs 1.08 ms in 128 MiB groups; 771 linears: 7.0 vs 7.6 ms)
    const int64_t chunks = (max_elems + 15) / 16;
    const unsigned gx =
        (unsigned)std::max<int64_t>(1, std::min<int64_t>((chunks + 256 * F16_UNROLL - 1) /
                                                             (256 * F16_UNROLL), 8192));
    const int np = (int)std::min<unsigned>(gx, LCQ_FP8_PARTIALS);  // pass-1 workgroups/tensor
    const dim3 grid(gx, (unsigned)n), grid1((unsigned)np, (unsigned)n);
    if (fmt_in == LCQ_FP8E4M3)
      hipLaunchKernelGGL((k_bmax16_many<LCQ_FP8E4M3, 2>), grid1, 256, 0, st, d, one, part);
    else
      hipLaunchKernelGGL((k_bmax16_many<LCQ_FP8E5M2, 2>), grid1, 256, 0, st, d, one, part);
#define LCQ_RQ16(FI, FO)                                                                    \
  do {                                                                                       \
    if (add_zero)                                                                            \
      hipLaunchKernelGGL((k_requant16_many<FI, FO, true>), grid, 256, 0, st, d, one, part,   \
                         np, qmax, clamp_min, so);                                           \
    else                                                                                     \
      hipLaunchKernelGGL((k_requant16_many<FI, FO, false>), grid, 256, 0, st, d, one, part,  \
                         np, qmax, clamp_min, so);                                           \
  } while (0)
    if (fmt_in == LCQ_FP8E4M3) {
      if (fmt_out == LCQ_FP8E4M3) LCQ_RQ16(LCQ_FP8E4M3, LCQ_FP8E4M3);
      else LCQ_RQ16(LCQ_FP8E4M3, LCQ_FP8E5M2);
    } else {
      if (fmt_out == LCQ_FP8E4M3) LCQ_RQ16(LCQ_FP8E5M2, LCQ_FP8E4M3);
      else LCQ_RQ16(LCQ_FP8E5M2, LCQ_FP8E5M2);
    }
#undef LCQ_RQ16
    return check_launch("lcq_fp8_block_to_tensor");
  }
  // any other block size: row-walking workgroups per tensor (blockIdx.y = tensor)
  const unsigned gx = (unsigned)std::max<int64_t>(
      1, std::min<int64_t>(max_elems / 65536, LCQ_FP8_PARTIALS));
  const dim3 grid(gx, (unsigned)n);
  if (fmt_in == LCQ_FP8E4M3)
    hipLaunchKernelGGL(k_absmax_blockfp8_many<LCQ_FP8E4M3>, grid, 256, 0, st, d, one, block, part);
  else
    hipLaunchKernelGGL(k_absmax_blockfp8_many<LCQ_FP8E5M2>, grid, 256, 0, st, d, one, block, part);
  int rc = check_launch("lcq_fp8_block_to_tensor: amax");
  if (rc) return rc;
#define LCQ_RQM(FI, FO)                                                                        \
  hipLaunchKernelGGL((k_requant_blockfp8_many<FI, FO>), grid, 256, 0, st, d, one, block, part, \
                     qmax, clamp_min, add_zero, so)
  if (fmt_in == LCQ_FP8E4M3) {
    if (fmt_out == LCQ_FP8E4M3) LCQ_RQM(LCQ_FP8E4M3, LCQ_FP8E4M3); else LCQ_RQM(LCQ_FP8E4M3, LCQ_FP8E5M2);
  } else {
    if (fmt_out == LCQ_FP8E4M3) LCQ_RQM(LCQ_FP8E5M2, LCQ_FP8E4M3); else LCQ_RQM(LCQ_FP8E5M2, LCQ_FP8E5M2);
  }
#undef LCQ_RQM
  return check_launch("lcq_fp8_block_to_tensor: requant");
}

extern "C" int lcq_fp8_block_to_tensor(const void* codes, int fmt_in, int64_t M, int64_t N,
                                       int block, const void* scales_inv, int fmt_out,
                                       float qmax, float clamp_min, int add_zero,
                                       void* amax_ws, void* codes_out, void* scale_out,
                                       void* stream) {
  LCQ_REQUIRE(fmt_in == LCQ_FP8E4M3 || fmt_in == LCQ_FP8E5M2, "bad input format");
  LCQ_REQUIRE(fmt_out == LCQ_FP8E4M3 || fmt_out == LCQ_FP8E5M2, "bad output format");
  LCQ_REQUIRE(block > 0 && M > 0 && N > 0 && N % 8 == 0, "N must be a positive multiple of 8");
  LCQ_REQUIRE(amax_ws != nullptr && codes_out != nullptr && scale_out != nullptr && qmax > 0.f,
              "missing buffers");
  Fp8Desc one{reinterpret_cast<const uint8_t*>(codes), reinterpret_cast<const float*>(scales_inv),
              reinterpret_cast<uint8_t*>(codes_out), M, N};
  return block_to_tensor(1, nullptr, one, M * N, fmt_in, block, fmt_out, qmax, clamp_min,
                         add_zero, amax_ws, reinterpret_cast<float*>(scale_out),
                         as_stream(stream));
}

extern "C" int lcq_fp8_block_to_tensor_many(int n, const void* descs, int64_t max_elems,
                                            int fmt_in, int block, int fmt_out, float qmax,
                                            float clamp_min, int add_zero, void* amax_ws,
                                            void* scales_out, void* stream) {
  LCQ_REQUIRE(n > 0 && n <= 65535 && descs && amax_ws && scales_out, "bad batch");
  LCQ_REQUIRE(fmt_in == LCQ_FP8E4M3 || fmt_in == LCQ_FP8E5M2, "bad input format");
  LCQ_REQUIRE(fmt_out == LCQ_FP8E4M3 || fmt_out == LCQ_FP8E5M2, "bad output format");
  LCQ_REQUIRE(block > 0 && max_elems > 0 && qmax > 0.f, "bad block / sizes");
  return block_to_tensor(n, reinterpret_cast<const Fp8Desc*>(descs), Fp8Desc{}, max_elems,
                         fmt_in, block, fmt_out, qmax, clamp_min, add_zero, amax_ws,
                         reinterpret_cast<float*>(scales_out), as_stream(stream));
}

extern "C" int lcq_fp_emul_quant(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                 int64_t group, int e_bits, int m_bits, void* fq_out,
                                 int fq_dtype, void* stream) {
  LCQ_REQUIRE(is_float_dt(x_dtype) && is_float_dt(fq_dtype), "dtypes must be f32/f16/bf16");
  LCQ_REQUIRE(e_bits >= 1 && e_bits <= 8 && m_bits >= 0 && m_bits <= 10, "bad e/m bits");
  LCQ_REQUIRE(rows > 0 && cols > 0, "empty tensor");
  if (group <= 0) group = cols;
  LCQ_REQUIRE(cols % group == 0 && group % 8 == 0, "group must divide cols, multiple of 8");
  const int64_t ng = rows * cols / group;
  LCQ_REQUIRE(ng <= 0x7fffffffLL, "too many groups");
  hipStream_t st = as_stream(stream);
  // quant.py:1014: maxval goes to fp32 when e_bits >= 5 -> the whole chain computes in fp32
  const bool f32 = e_bits >= 5 || x_dtype == LCQ_F32;
#define LCQ_EM(XT, CT)                                                                      \
  hipLaunchKernelGGL((k_fp_emul_rows<XT, CT>), dim3((unsigned)ng), 256, 0, st, x, group,   \
                     e_bits, m_bits, fq_out, fq_dtype)
  switch (x_dtype) {
    case LCQ_F32: LCQ_EM(LCQ_F32, LCQ_F32); break;
    case LCQ_BF16:
      if (f32) LCQ_EM(LCQ_BF16, LCQ_F32); else LCQ_EM(LCQ_BF16, LCQ_BF16);
      break;
    default:
      if (f32) LCQ_EM(LCQ_F16, LCQ_F32); else LCQ_EM(LCQ_F16, LCQ_F16);
      break;
  }
#undef LCQ_EM
  return check_launch("lcq_fp_emul_quant");
}
