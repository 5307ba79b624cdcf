// Fused elementwise ops of the calibration forward (the inspect-module and block forwards that
// AWQ's scale search and GPTQ's Hessian capture run ~20x per block).
//
// Rotary embedding (transformers modeling_llama.apply_rotary_pos_emb, used by the reference's
// Llama blocks, llmc/models/llama.py): q' = q*cos + rotate_half(q)*sin, same for k. The torch
// form runs cat / neg / 2 mul / add as five launches over q and k; here one pass reads each
// head row once. Rounding is per op in the tensor dtype exactly as torch does (products and
// the sum each rounded), so the result is bit-identical to the unfused ops.
//
// SiLU-gated product (LlamaMLP.forward: act_fn(gate) * up): silu(g) = g / (1 + exp(-g)) in
// fp32, rounded to the dtype, times up, rounded -- one pass instead of two.
#include "lcq_common.h"

namespace lcq {

// one thread: 8 consecutive dims d0..d0+7 of the first half and the partner 8 of the second
// half of one head row (D = head dim, even, D/2 a multiple of 8)
template <int DT>
__global__ void __launch_bounds__(256) k_rotary(const void* __restrict__ q, const void* __restrict__ k,
                                                const void* __restrict__ cs, const void* __restrict__ sn,
                                                int64_t B, int64_t S, int Hq, int Hk, int D,
                                                int64_t cs_bstride, void* __restrict__ oq,
                                                void* __restrict__ ok) {
  const int per_row = D / 16;  // threads per head row
  const int64_t rows_q = B * S * Hq, rows = rows_q + B * S * Hk;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < rows * per_row; t += stride) {
    const int64_t row = t / per_row;
    const int d0 = (int)(t % per_row) * 8;
    const bool isq = row < rows_q;
    const int64_t r = isq ? row : row - rows_q;
    const int H = isq ? Hq : Hk;
    const int64_t bs = r / H;               // (b, s) flat
    const int64_t b = bs / S, s = bs % S;
    const void* src = isq ? q : k;
    void* dst = isq ? oq : ok;
    const int64_t base = r * D;
    const int64_t cbase = b * cs_bstride + s * D;
    float x1[8], x2[8], c1[8], c2[8], s1[8], s2[8], o1[8], o2[8];
    ld8<DT>(src, base + d0, x1);
    ld8<DT>(src, base + D / 2 + d0, x2);
    ld8<DT>(cs, cbase + d0, c1);
    ld8<DT>(cs, cbase + D / 2 + d0, c2);
    ld8<DT>(sn, cbase + d0, s1);
    ld8<DT>(sn, cbase + D / 2 + d0, s2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // first half: q*cos + (-q2)*sin ; second half: q2*cos + q1*sin
      o1[j] = rnd<DT>(rnd<DT>(x1[j] * c1[j]) + rnd<DT>(-x2[j] * s1[j]));
      o2[j] = rnd<DT>(rnd<DT>(x2[j] * c2[j]) + rnd<DT>(x1[j] * s2[j]));
    }
    st8<DT>(dst, base + d0, o1);
    st8<DT>(dst, base + D / 2 + d0, o2);
  }
}

template <int DT>
__global__ void __launch_bounds__(256) k_silu_mul(const void* __restrict__ g, const void* __restrict__ u,
                                                  int64_t n8, void* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    float a[8], b[8], o[8];
    ld8<DT>(g, t * 8, a);
    ld8<DT>(u, t * 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sl = rnd<DT>(a[j] / (1.0f + expf(-a[j])));
      o[j] = rnd<DT>(sl * b[j]);
    }
    st8<DT>(out, t * 8, o);
  }
}

// RMSNorm (modeling_llama.LlamaRMSNorm.forward): v = mean(x_f32^2); y = x_f32 * rsqrt(v + eps)
// rounded to the dtype; out = weight * y rounded. One workgroup per row, the row read once
// (the torch chain makes 6 passes: cast, pow, mean, rsqrt-mul, cast, weight-mul). The sum of
// squares uses a fixed per-lane + tree order (deterministic; not torch's reduction order, so
// outputs can differ from the unfused chain by one rounding of the variance).
template <int DT, int CH>
__global__ void __launch_bounds__(256) k_rmsnorm(const void* __restrict__ x,
                                                 const void* __restrict__ w, int64_t H,
                                                 float eps, void* __restrict__ out) {
  // the row's CH 2048-element slices stay in registers between the sum and the scaling (one
  // HBM read of x); all loads are issued before the first FMA
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const int64_t base = row * H;
  float v[CH][8];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = threadIdx.x * 8 + (int64_t)k * 2048;
    if (c < H) ld8<DT>(x, base + c, v[k]);
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = threadIdx.x * 8 + (int64_t)k * 2048;
    if (c < H) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ss = __fadd_rn(ss, __fmul_rn(v[k][j], v[k][j]));
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) ss = __fadd_rn(ss, __shfl_xor(ss, m, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float var = __fdiv_rn(__fadd_rn(__fadd_rn(red[0], red[1]), __fadd_rn(red[2], red[3])),
                              (float)H);
  const float r = rsqrtf(__fadd_rn(var, eps));
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int64_t c = threadIdx.x * 8 + (int64_t)k * 2048;
    if (c < H) {
      float g[8], o[8];
      ld8<DT>(w, c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rnd<DT>(g[j] * rnd<DT>(v[k][j] * r));
      st8<DT>(out, base + c, o);
    }
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_rmsnorm(const void* x, const void* weight, int dtype, int64_t rows,
                           int64_t H, float eps, void* out, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "dtype must be bf16 or fp16");
  LCQ_REQUIRE(rows > 0 && rows <= 0x7fffffffLL && H > 0 && H % 8 == 0,
              "H must be a positive multiple of 8");
  LCQ_REQUIRE(H <= 8 * 2048, "H must be <= 16384");
  hipStream_t st = as_stream(stream);
  const int ch = (int)((H + 2047) / 2048);
#define LCQ_RMS(DT, CH) \
  hipLaunchKernelGGL((k_rmsnorm<DT, CH>), dim3((unsigned)rows), 256, 0, st, x, weight, H, eps, out)
#define LCQ_RMS_CH(DT)                             \
  switch (ch) {                                    \
    case 1: LCQ_RMS(DT, 1); break;                 \
    case 2: LCQ_RMS(DT, 2); break;                 \
    case 3: LCQ_RMS(DT, 3); break;                 \
    case 4: LCQ_RMS(DT, 4); break;                 \
    case 5: LCQ_RMS(DT, 5); break;                 \
    case 6: LCQ_RMS(DT, 6); break;                 \
    case 7: LCQ_RMS(DT, 7); break;                 \
    default: LCQ_RMS(DT, 8); break;                \
  }
  if (dtype == LCQ_BF16) {
    LCQ_RMS_CH(LCQ_BF16)
  } else {
    LCQ_RMS_CH(LCQ_F16)
  }
#undef LCQ_RMS_CH
#undef LCQ_RMS
  return check_launch("lcq_rmsnorm");
}

extern "C" int lcq_rotary(const void* q, const void* k, const void* cos, const void* sin,
                          int dtype, int64_t B, int64_t S, int Hq, int Hk, int D,
                          int64_t cos_bstride, void* out_q, void* out_k, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "dtype must be bf16 or fp16");
  LCQ_REQUIRE(B > 0 && S > 0 && Hq > 0 && Hk >= 0 && D > 0 && D % 16 == 0,
              "head dim must be a positive multiple of 16");
  const int64_t work = (B * S * (Hq + Hk)) * (D / 16);
  const unsigned grid = stream_grid(work, 256);
  hipStream_t st = as_stream(stream);
  if (dtype == LCQ_BF16)
    hipLaunchKernelGGL(k_rotary<LCQ_BF16>, grid, 256, 0, st, q, k, cos, sin, B, S, Hq, Hk, D,
                       cos_bstride, out_q, out_k);
  else
    hipLaunchKernelGGL(k_rotary<LCQ_F16>, grid, 256, 0, st, q, k, cos, sin, B, S, Hq, Hk, D,
                       cos_bstride, out_q, out_k);
  return check_launch("lcq_rotary");
}

extern "C" int lcq_silu_mul(const void* gate, const void* up, int dtype, int64_t n, void* out,
                            void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "dtype must be bf16 or fp16");
  LCQ_REQUIRE(n > 0 && n % 8 == 0, "n must be a positive multiple of 8");
  const unsigned grid = stream_grid(n / 8, 256);
  hipStream_t st = as_stream(stream);
  if (dtype == LCQ_BF16)
    hipLaunchKernelGGL(k_silu_mul<LCQ_BF16>, grid, 256, 0, st, gate, up, n / 8, out);
  else
    hipLaunchKernelGGL(k_silu_mul<LCQ_F16>, grid, 256, 0, st, gate, up, n / 8, out);
  return check_launch("lcq_silu_mul");
}
