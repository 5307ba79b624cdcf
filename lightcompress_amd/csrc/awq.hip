// AWQ scale search + auto-clip device kernels (gfx950).
//
// Reference: llmc/compression/quantization/awq.py and auto_clip.py. Every op rounds to the
// weight/activation dtype like the reference's torch-bf16 expressions:
//   get_act_scale      awq.py:74-85     mean_t |x|                        -> lcq_absmean_cols
//   get_weight_scale   awq.py:48-72     mean_rows |w| / group max          -> lcq_awq_weight_scale
//   get_scales (v2)    awq.py:87-108    s = x^r ; clamp 1e-4 ; s/sqrt(max*min) -> lcq_awq_scales
//   get_scales (v1)    awq.py:87-108    s = x^r / w^(1-r) ; ...            -> lcq_awq_scales_v1
//   scaling_input / update_input_feat / scale_ln_fcs / scale_fc_fc
//                      base_blockwise_quantization.py:631-778, 880-897  -> lcq_scale_bcast
//   calculate_loss     awq.py:134-145   mean((org-out).float()^2)        -> lcq_sq_diff_mean
//   auto_clip_layer    auto_clip.py:83-191 (10-step shrink grid)          -> lcq_auto_clip_search
//   apply_clip (v1)    auto_clip.py:193-212                               -> lcq_clip_apply
#include "lcq_common.h"
#include "lcq_fp8.h"
#include <stdlib.h>

namespace lcq {

// ----------------------------------------------------------------------------------------
// Column means in torch-CPU's exact summation order.
//
// x.abs().view(-1, H).mean(0) (get_act_scale, awq.py:74-85) and layer_scale.mean(0)
// (get_weight_scale, awq.py:48-72) are fp32 sums over rows then / rows (bf16/fp16 inputs:
// mean_out sums in fp32). torch-CPU's outer-dimension sum (SumKernel.cpp multi_row_sum, per
// column lane, independent of the SIMD width when cols % 64 == 0) is a 4-level cascade with
// blocks of LS = 2^lp rows, lp = max(4, ceil_log2(rows) / 4):
//   acc0 = sequential sum of a block; acc1 += acc0 at every block end; at every LS^2-row
//   boundary acc2 += acc1 (acc1 = 0); at every LS^3-row boundary acc3 += acc2 (acc2 = 0);
//   tail rows -> acc0; result = ((acc0 + acc1) + acc2) + acc3.
// Pass 1: one thread per (8 columns, LS^2-row superblock) -> acc1 of the superblock (and the
// tail's acc0); pass 2: one thread per column folds the superblocks in the same order.
// ----------------------------------------------------------------------------------------
__host__ __device__ inline int colsum_lp(int64_t rows) {
  int cl = 0;
  while (((int64_t)1 << cl) < rows) ++cl;  // ceil_log2
  return cl / 4 > 4 ? cl / 4 : 4;
}

// MODE 0: value = |x| ; MODE 1: value = rnd(|w| / max|w| over its group of G columns)
// (get_weight_scale's abs_weights.div_(max_vals)); G / 8 lanes, a power of two <= 64.
template <int DT, int MODE>
__global__ void __launch_bounds__(256) k_colsum_l1(const void* x, int64_t rows, int64_t c,
                                                  int lp, int glanes, float* part,
                                                  float* tail) {
  const int64_t c8 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = c8 * 8 < c;
  const int64_t LS = (int64_t)1 << lp, SB = LS * LS;
  const int64_t r0 = (int64_t)blockIdx.y * SB;
  const int64_t r1 = min(rows, r0 + SB);
  const int64_t nfull = r0 + (r1 - r0) / LS * LS;  // end of the full blocks
  float acc1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, acc0[8];
  int64_t r = r0;
  for (; r < r1; r += LS) {
    const int64_t re = min(r1, r + LS);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc0[j] = 0.f;
    for (int64_t rr = r; rr < re; ++rr) {
      float v[8];
      if (live) ld8<DT>(x, rr * c + c8 * 8, v);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fabsf(v[j]);
      if constexpr (MODE == 1) {
        float m = v[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) m = fmaxf(m, v[j]);
        for (int o = 1; o < glanes; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rnd<DT>(v[j] / m);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc0[j] += v[j];
    }
    if (re - r == LS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc1[j] += acc0[j];
    }
  }
  if (!live) return;
  float* p = part + (int64_t)blockIdx.y * c + c8 * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = acc1[j];
  if (r1 == rows) {  // last superblock: the tail rows' sequential sum (0 if none)
    const bool has_tail = nfull < rows;
#pragma unroll
    for (int j = 0; j < 8; ++j) tail[c8 * 8 + j] = has_tail ? acc0[j] : 0.f;
  }
}

// fold -> column sum, / rows, rounded to DT. MODE 0: out = mean. MODE 1 (get_weight_scale
// over the subset's layers): layer 0 out = mean, then out = rnd(out + mean), and after the
// last layer out = rnd(out / nlayers).
template <int DT, int MODE>
__global__ void __launch_bounds__(256) k_colsum_fold(const float* part, const float* tail,
                                                    int64_t rows, int64_t c, int lp, int layer,
                                                    int nlayers, void* out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= c) return;
  const int64_t LS = (int64_t)1 << lp, SB = LS * LS;
  const int64_t mask = LS - 1;
  const int64_t nsb = (rows + SB - 1) / SB;
  const int64_t nfull_sb = rows / SB;
  float acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  for (int64_t sb = 0; sb < nfull_sb; ++sb) {
    const int64_t i = (sb + 1) * SB;
    acc2 += part[sb * c + j];
    if ((i & (mask << (2 * lp))) == 0) {
      acc3 += acc2;
      acc2 = 0.f;
    }
  }
  if (nsb > nfull_sb) acc1 = part[nfull_sb * c + j];  // the partial superblock's full blocks
  float acc0 = tail[j];
  acc0 += acc1;
  acc0 += acc2;
  acc0 += acc3;
  const float mean = rnd<DT>(acc0 / (float)rows);
  if constexpr (MODE == 0) {
    st1<DT>(out, j, mean);
  } else {
    float t = layer == 0 ? mean : rnd<DT>(ld1<DT>(out, j) + mean);
    if (layer == nlayers - 1) t = rnd<DT>(t / (float)nlayers);
    st1<DT>(out, j, t);
  }
}

// ----------------------------------------------------------------------------------------
// AWQ v2 scales for one ratio. s = round_dt(pow(x, r_dt)) where the exponent is first rounded
// to the tensor dtype and pow is correctly rounded (torch-CPU bf16 semantics, verified
// exhaustively over all positive bf16 inputs x 20 ratios); clamp(min=1e-4);
// s / sqrt(max(s)*min(s)) with each op rounded to DT. One workgroup.
// ----------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(1024) k_awq_scales(const void* xmean, int64_t c, float r,
                                                    void* out, const void* wmax, float r1) {
  __shared__ float red[2][16];
  const float lo = rnd<DT>(1e-4f);
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t j = threadIdx.x; j < c; j += blockDim.x) {
    const float xv = ld1<DT>(xmean, j);
    float s = rnd<DT>((float)pow((double)xv, (double)r));
    if (wmax) {  // v1: x^r / w^(1 - r), the second exponent also rounded to DT by the caller
      const float wv = rnd<DT>((float)pow((double)ld1<DT>(wmax, j), (double)r1));
      s = rnd<DT>(s / wv);
    }
    s = fmaxf(s, lo);
    mx = fmaxf(mx, s);
    mn = fminf(mn, s);
    st1<DT>(out, j, s);  // s is a DT value: parked losslessly in out for the second pass
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    mn = fminf(mn, __shfl_xor(mn, m, 64));
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = mx;
    red[1][w] = mn;
  }
  __syncthreads();
  mx = red[0][0];
  mn = red[1][0];
  for (int i = 1; i < nw; ++i) {
    mx = fmaxf(mx, red[0][i]);
    mn = fminf(mn, red[1][i]);
  }
  const float d = rnd<DT>(sqrtf(rnd<DT>(mx * mn)));
  for (int64_t j = threadIdx.x; j < c; j += blockDim.x) st1<DT>(out, j, ld1<DT>(out, j) / d);
}

// ----------------------------------------------------------------------------------------
// out[r, c] = round_dt(x[r, c] (op) s[axis index]), op 0 = mul, 1 = div; axis 0 = per column
// (s has cols entries), 1 = per row (s has rows entries). In place allowed.
// 2-D grid: a thread owns one 8-column chunk and walks rb (>= SB_ROWS) rows, so a column scale and its
// reciprocal are loaded / formed once (no per-element index arithmetic). The division is the
// correctly rounded quotient: Markstein's from RN(1/s) (3 VALU), which equals x / s while the
// residual x - s q0 and the correction r / s stay clear of the subnormal range (|x| and |q| >=
// 2^-100) and q is finite; anything else (zero, tiny, inf, NaN) takes the IEEE division.
// ----------------------------------------------------------------------------------------
constexpr int SB_ROWS = 32;

// div_exact: lcq_common.h

// st8 with the bf16 rounding on v_cvt_pk_bf16_f32 (RNE like bf16_rne; a NaN stays a NaN with
// its payload dropped): this streaming kernel is VALU-heavy enough for the integer form to show
template <int DT>
__device__ __forceinline__ void st8_cvt(void* base, int64_t e0, const float (&v)[8]) {
  if constexpr (DT == LCQ_BF16) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (__float_as_uint(bf16_rne_hw(v[2 * i])) >> 16) |
             (__float_as_uint(bf16_rne_hw(v[2 * i + 1])) & 0xffff0000u);
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(base) + e0) =
        make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    st8<DT>(base, e0, v);
  }
}

template <int DT, int OP, int AXIS>
__global__ void __launch_bounds__(256) k_scale_bcast(const void* x, int64_t rows, int64_t cols,
                                                    const void* s, void* out, int64_t rb) {
  const int64_t c8 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c8 * 8 >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.y * rb;
  const int64_t r1 = r0 + rb < rows ? r0 + rb : rows;
  float sv[8], rs[8];
  if constexpr (AXIS == 0) {
    ld8<DT>(s, c8 * 8, sv);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = 1.0f / sv[j];
  }
  // 4 rows per step: their loads are issued together (memory-level parallelism per thread)
  for (int64_t rb4 = r0; rb4 < r1; rb4 += 4) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (rb4 + u < r1) ld8<DT>(x, (rb4 + u) * cols + c8 * 8, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rb4 + u >= r1) break;
      if constexpr (AXIS == 1) {
        const float q = ld1<DT>(s, rb4 + u);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sv[j] = q;
          rs[j] = 1.0f / q;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[u][j] = (OP == 0) ? v[u][j] * sv[j] : div_exact(v[u][j], sv[j], rs[j]);
      st8_cvt<DT>(out, (rb4 + u) * cols + c8 * 8, v[u]);
    }
  }
}

// ----------------------------------------------------------------------------------------
// loss = mean(((a - b) in DT).float()^2): fp64 partial sums per block, fixed-order final sum,
// result stored as fp32(sum) / n (the reference's fp32 mean) into out[slot].
// ----------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) k_sqdiff_p1(const void* a, const void* b, int64_t n,
                                                  double* part) {
  __shared__ double red[4];
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    float va[8], vb[8];
    ld8<DT>(a, t * 8, va);
    ld8<DT>(b, t * 8, vb);
    float s = 0.f;
    double d8 = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = rnd<DT>(va[j] - vb[j]);
      d8 += (double)(d * d);
    }
    (void)s;
    acc += d8;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// one wave: lane l sums parts l, l+64, ... in order, then a fixed xor tree (deterministic)
__global__ void __launch_bounds__(64) k_sqdiff_p2(const double* part, int nparts, int64_t n,
                                                  float* out, int slot) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) s += part[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (threadIdx.x == 0) out[slot] = (float)s / (float)n;
}

// ----------------------------------------------------------------------------------------
// auto_clip search (auto_clip.py:83-191). A workgroup = 128 output rows (one per lane, two
// waves) x one G-wide group (G = 32 / 64 / 128 / 256); the group's sampled-token tiles are
// shared through LDS. Model dtype DT = bf16 or fp16 (every rounding below is to DT).
// For every (row o, group g):
//   org[t]  = DT( sum_k DT(x[t,g,k] * w[o,g,k]) )              (t over the T sampled tokens)
//   step i: max_i = DT(org_max * (1 - i/n_grid)), min_i = -max_i | DT(org_min * (..))
//           q = fake_quant(clamp(w, min_i, max_i)) (DT, per-group min/max qparams)
//           cur[t] = DT( sum_k DT(x * q) );  err_i = DT(mean_t DT(DT(cur-org)^2))
//   keep the first strictly smaller err (min_errs starts at DT(1e9)).
// The reference materialises the DT broadcast product, so every product is rounded to DT
// before the fp32 sum: that rules out MFMA (exact products). VALU design: the candidate
// weights live unpacked in VGPRs, x tiles are fp32 in LDS and read as wave-uniform broadcasts,
// products go through v_pk_mul_f32 + v_cvt_pk_bf16_f32 (RNE) and v_pk_add_f32 into 8 partial
// sums (k mod 8) reduced by a halving tree (torch-CPU's vectorised order), the per-step
// squared-error sums and the original outputs sit in LDS so the token loop stays rolled.
// ----------------------------------------------------------------------------------------
constexpr int CROWS = 128;     // lane pairs per workgroup (2 lanes per row -> 256 threads)
constexpr int CMAXSTEPS = 16;
constexpr int CGMAX = 256;     // largest group (xs tile = CT x G fp32)

typedef float v2f __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
typedef _Float16 v2h __attribute__((ext_vector_type(2)));

// fp16 RNE (subnormals and overflow to inf included) in integer / fp32 arithmetic. Written
// out rather than as (float)(_Float16)f: with the conversion pair the compiler re-forms the
// surrounding fp32 ops into native f16 / mixed-precision instructions (v_mul_f16,
// v_fma_mixlo_f16), which measured 1.5 % of clip bounds off the reference's on fp16 models.
__device__ __forceinline__ float f16r_soft(float f) {
  const uint32_t u = __float_as_uint(f), a = u & 0x7fffffffu, s = u & 0x80000000u;
  if (a > 0x7f800000u) return f;                                    // NaN
  if (a >= 0x477ff000u) return __uint_as_float(s | 0x7f800000u);   // >= 65520 -> inf
  if (a < 0x38800000u) {  // below 2^-14: the fp16 subnormal grid, multiples of 2^-24
    const float t = rintf(__uint_as_float(a) * 16777216.0f) * 5.9604644775390625e-08f;
    return __uint_as_float(__float_as_uint(t) | s);
  }
  const uint32_t r = a + 0xfffu + ((a >> 13) & 1u);
  return __uint_as_float((r & 0xffffe000u) | s);
}

// RNE to the model dtype DT (bf16: v_cvt_pk_bf16_f32; fp16: f16r_soft) and back to fp32
template <int DT>
__device__ __forceinline__ float dtr(float f) {
  if constexpr (DT == LCQ_BF16) {
    // v_cvt_pk_bf16_f32 with a zero low half: the result register is the widened value (one
    // VALU instead of convert + shift)
    const v2bf h = __builtin_convertvector(v2f{0.f, f}, v2bf);
    return __builtin_bit_cast(float, h);
  } else {
    return f16r_soft(f);
  }
}

// products of a pair rounded to DT and widened back to fp32. bf16: one v_cvt_pk_bf16_f32 per
// product with a zero low half, so the result register IS the widened fp32 value (2 VALU per
// pair instead of convert + shift + mask: 3)
template <int DT, bool CVT2 = true>
__device__ __forceinline__ v2f dtr2(v2f p) {
  if constexpr (DT == LCQ_BF16 && CVT2) {
    const v2bf lo = __builtin_convertvector(v2f{0.f, p.x}, v2bf);
    const v2bf hi = __builtin_convertvector(v2f{0.f, p.y}, v2bf);
    return v2f{__builtin_bit_cast(float, lo), __builtin_bit_cast(float, hi)};
  } else if constexpr (DT == LCQ_BF16) {
    const v2bf h = __builtin_convertvector(p, v2bf);
    const uint32_t u = __builtin_bit_cast(uint32_t, h);
    v2f r;
    r.x = __uint_as_float(u << 16);
    r.y = __uint_as_float(u & 0xffff0000u);
    return r;
  } else {
    return v2f{f16r_soft(p.x), f16r_soft(p.y)};
  }
}

// 4 consecutive DT elements (8 bytes) widened to fp32
template <int DT>
__device__ __forceinline__ void widen4(uint2 v, float* q) {
  if constexpr (DT == LCQ_BF16) {
    q[0] = __uint_as_float(v.x << 16);
    q[1] = __uint_as_float(v.x & 0xffff0000u);
    q[2] = __uint_as_float(v.y << 16);
    q[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
    const v2h a = __builtin_bit_cast(v2h, v.x), b = __builtin_bit_cast(v2h, v.y);
    q[0] = (float)a.x; q[1] = (float)a.y; q[2] = (float)b.x; q[3] = (float)b.y;
  }
}

__device__ __forceinline__ float xor1(float v) {  // value of the partner lane (lane ^ 1)
  // DPP quad_perm [1, 0, 3, 2]: a VALU operand modifier, no LDS round trip (ds_bpermute)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               0xB1, 0xF, 0xF, true));
}

// sum_k DT(x[k] * q[k]) over one G-wide group for each of this lane's R rows, split over a
// lane pair: this lane owns k = 8i + 4h + j (j = 0..3) i.e. partial sums acc_{4h+j} of the
// 8-way (k mod 8) order that torch-CPU's vectorised reduction uses for every group size and for
// bf16 and fp16 alike; the pair exchange forms l_j = acc_j + acc_{j+4} and both lanes finish
// the halving tree. One broadcast LDS read of x feeds R rows (R = 2: the ds_read_b128 per 8
// products of R = 1 kept the LDS array busy every cycle; at 2 it is half busy, VALU-bound).
template <int DT, int G, int R>
__device__ __forceinline__ void dot_rows(const float* __restrict__ xr,
                                         const float (&q)[R][G / 2], int h, float (&out)[R]) {
  // packed fp32 products and sums (v_pk_mul_f32 / v_pk_add_f32): measured 1.26x faster than
  // the same work as scalar v_mul_f32 / v_add_f32 (49 % more instructions)
  v2f a0[R], a1[R];
#pragma unroll
  for (int j = 0; j < R; ++j) a0[j] = a1[j] = v2f{0.f, 0.f};
#pragma unroll
  for (int i = 0; i < G / 8; ++i) {
    const float4 xv = *reinterpret_cast<const float4*>(xr + 8 * i + 4 * h);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      a0[j] += dtr2<DT>(v2f{xv.x, xv.y} * v2f{q[j][4 * i], q[j][4 * i + 1]});
      a1[j] += dtr2<DT>(v2f{xv.z, xv.w} * v2f{q[j][4 * i + 2], q[j][4 * i + 3]});
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    // lane h=0 holds acc0..3, h=1 holds acc4..7: l_j = acc_j + acc_{j+4}. The partner values
    // are read in uniform control flow (a cross-lane read inside a divergent branch would see
    // inactive lanes); the operand order is then fixed with selects so both lanes agree.
    const float c[4] = {a0[j].x, a0[j].y, a1[j].x, a1[j].y};
    float l[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float pm = xor1(c[m]);
      l[m] = (h ? pm : c[m]) + (h ? c[m] : pm);
    }
    out[j] = dtr<DT>((l[0] + l[2]) + (l[1] + l[3]));
  }
}

// this lane's half of a row's group (k = 8i + 4h + j), raw DT bits: loaded once per kernel and
// kept in registers across the 1 + nsteps passes (re-reading it from global memory every pass
// cost 11x the weight bytes -- the L2 does not hold a workgroup's 64 KB between passes -- and
// a vmcnt stall at the head of each pass)
template <int G>
__device__ __forceinline__ void fetch_half(const uint16_t* __restrict__ wrow, int h,
                                           uint2 (&raw)[G / 8]) {
#pragma unroll
  for (int i = 0; i < G / 8; ++i) raw[i] = *reinterpret_cast<const uint2*>(wrow + 8 * i + 4 * h);
}

template <int DT, int G>
__device__ __forceinline__ void widen_half(const uint2 (&raw)[G / 8], float (&q)[G / 2]) {
#pragma unroll
  for (int i = 0; i < G / 8; ++i) widen4<DT>(raw[i], &q[4 * i]);
}

// get_qparams in fp32 (quant.py:545-559) for the calib_algo mse search
__device__ __forceinline__ void qparams_f32_mse(float mn, float mx, float qmin, float qmax,
                                                int sym, float& s, float& z) {
  if (sym) {
    float am = fmaxf(fabsf(mx), fabsf(mn));
    am = am < 1e-5f ? 1e-5f : am;
    s = am / qmax;
    z = 0.f;
  } else {
    float r = mx - mn;
    r = r < 1e-5f ? 1e-5f : r;
    s = r / (qmax - qmin);
    z = fminf(fmaxf(qmin - rintf(mn / s), qmin), qmax);
  }
}

// MSE: the weight quantizer's calib_algo is mse (quant.py:145-203): each shrink step's fake
// quant searches its range on the clamped group in fp32 (mse_p[i] = fp32(1 - i / grid),
// |qdq(v) - v|^norm summed, strict improvements shrink the base), then quantizes in fp32 with
// the fp32 qparams and rounds to DT once (the DT tensor is promoted by the fp32 scales).
// R rows per lane pair (R = 2 for G <= 128 without mse: 256 rows per workgroup; R = 1 for
// G = 256, whose 128 weights per lane per row leave no room for a second row, and for mse).
// LDS of one workgroup: x tile [CT][G] fp32, original outputs [CT][rows] as DT bits (they are
// DT values), per-step error sums [CMAXSTEPS][rows] fp32
template <int G, int R>
struct ClipTile {
  static constexpr int CT = R == 2 ? 64 : 32;  // sampled tokens per x tile
  static constexpr int RW = CROWS * R;
  static constexpr int bytes = CT * G * 4 + CT * RW * 2 + CMAXSTEPS * RW * 4;
};

template <int DT>
__device__ __forceinline__ uint16_t dt_bits(float v) {  // v is a DT value
  if constexpr (DT == LCQ_BF16) return (uint16_t)(__float_as_uint(v) >> 16);
  else return __builtin_bit_cast(uint16_t, (_Float16)v);
}
template <int DT>
__device__ __forceinline__ float dt_val(uint16_t b) {
  if constexpr (DT == LCQ_BF16) return __uint_as_float((uint32_t)b << 16);
  else return (float)__builtin_bit_cast(_Float16, b);
}

// One shrink step's candidate weights (auto_clip.py:160-172 with fake_quantize, quant.py
// get_qparams + quant_dequant in DT): q <- fq(clamp(q, smin, smax)) with the qparams of the
// clamped group range [cmn, cmx].
template <int DT, int N>
__device__ __forceinline__ void clip_candidates(float (&q)[N], float smin, float smax, float cmn,
                                                float cmx, float qmin, float qmax, int sym) {
  float qs, qz;
  qparams_ct<DT>(cmn, cmx, qmin, qmax, sym, qs, qz);
  const float rqs = 1.0f / qs;  // RN(1/s): qs >= DT(1e-5) / qmax, so it is normal
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const float v = fminf(fmaxf(q[k], smin), smax);
    // correctly rounded fp32 quotient (Markstein's from RN(1/s), 3 VALU: |v / s| <= qmax + 1,
    // normal or rounding to zero either way, as mk_safe in quant_group.hip), then rounded to
    // DT. A plain v * RN(1/s) can miss by an ulp, which fp16's extra mantissa bits expose.
    float tq = rintf(dtr<DT>(div_mk(v, qs, rqs)));
    if (!sym) tq = dtr<DT>(tq + qz);
    tq = fminf(fmaxf(tq, qmin), qmax);
    q[k] = dtr<DT>((sym ? tq : dtr<DT>(tq - qz)) * qs);
  }
}

template <int DT, int G, int R, bool MSE>
__global__ void __launch_bounds__(2 * CROWS, G >= 256 ? 1 : 2)
    k_auto_clip(const uint16_t* __restrict__ w, const uint16_t* __restrict__ x, int64_t oc,
                int64_t ic, int T, int nsteps, const float* __restrict__ factors, float qmin,
                float qmax, int sym, int clip_sym, uint16_t* best_max, uint16_t* best_min,
                int mse_steps, const float* __restrict__ mse_p, float norm,
                const uint16_t* __restrict__ qx) {
  static_assert(!MSE || R == 1, "the mse search keeps one row per lane pair");
  constexpr int CH = G / 2;    // weights per lane per row: k = 8i + 4h + j, h = lane parity
  constexpr int CHUNKS = G / 8;
  constexpr int RW = CROWS * R;  // rows per workgroup
  constexpr int CT = ClipTile<G, R>::CT;
  extern __shared__ __attribute__((aligned(16))) float clip_lds[];
  float* xs = clip_lds;                                                    // [CT][G]
  uint16_t* orgs = reinterpret_cast<uint16_t*>(clip_lds + CT * G);         // [CT][RW]
  float* es = reinterpret_cast<float*>(orgs + CT * RW);                    // [steps][RW]
  const int tid = threadIdx.x;
  const int r = tid >> 1, h = tid & 1;
  const int64_t g = blockIdx.y;
  const int64_t ng = ic / G;
  int64_t o[R];
  bool live[R];
  const uint16_t* wrow[R];
  float mxs[R], mn[R], org_max[R], org_min[R];
  uint2 wraw[R][CHUNKS];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    o[j] = (int64_t)blockIdx.x * RW + j * CROWS + r;
    live[j] = o[j] < oc;
    wrow[j] = w + (live[j] ? o[j] : 0) * ic + g * G;
    fetch_half<G>(wrow[j], h, wraw[j]);
    float q[CH];
    widen_half<DT, G>(wraw[j], q);
    float mx = -INFINITY, mi = INFINITY, am = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      mx = fmaxf(mx, q[k]);
      mi = fminf(mi, q[k]);
      am = fmaxf(am, fabsf(q[k]));
    }
    mxs[j] = fmaxf(mx, xor1(mx));
    mn[j] = fminf(mi, xor1(mi));
    am = fmaxf(am, xor1(am));
    org_max[j] = clip_sym ? am : mxs[j];
    org_min[j] = mn[j];
  }
  if (h == 0)
    for (int s = 0; s < nsteps; ++s)
#pragma unroll
      for (int j = 0; j < R; ++j) es[s * RW + j * CROWS + r] = 0.f;

  // stage CT token rows of this group as fp32, 8 elements (16 B) per chunk
  auto stage = [&](const uint16_t* __restrict__ src, int t0) {
    for (int idx = tid; idx < CT * CHUNKS; idx += 2 * CROWS) {
      const int row = idx / CHUNKS, ch = idx % CHUNKS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t0 + row < T)
        v = *reinterpret_cast<const uint4*>(src + (int64_t)(t0 + row) * ic + g * G + ch * 8);
      float a[8];
      widen4<DT>(make_uint2(v.x, v.y), a);
      widen4<DT>(make_uint2(v.z, v.w), a + 4);
      *reinterpret_cast<float4*>(&xs[row * G + ch * 8]) = make_float4(a[0], a[1], a[2], a[3]);
      *reinterpret_cast<float4*>(&xs[row * G + ch * 8 + 4]) = make_float4(a[4], a[5], a[6], a[7]);
    }
  };
  for (int t0 = 0; t0 < T; t0 += CT) {
    __syncthreads();  // previous tile fully consumed
    stage(x, t0);
    __syncthreads();
    const int tn = min(CT, T - t0);
    // pass p = 0: original outputs; p = s + 1: shrink step s
    for (int p = 0; p <= nsteps; ++p) {
      if (qx != nullptr && p == 1) {  // w8a8: shrink steps see fake-quantized activations
        __syncthreads();              // (auto_clip.py:177, fake_quantize_input)
        stage(qx, t0);
        __syncthreads();
      }
      float q[R][CH];
#pragma unroll
      for (int j = 0; j < R; ++j) widen_half<DT, G>(wraw[j], q[j]);
      if (p > 0) {
        const float f = factors[p - 1];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const float smax = dtr<DT>(org_max[j] * f);
          const float smin = clip_sym ? -smax : dtr<DT>(org_min[j] * f);
          const float cmn = fminf(fmaxf(mn[j], smin), smax);
          const float cmx = fminf(fmaxf(mxs[j], smin), smax);
          float qs, qz;
          if constexpr (MSE) {
#pragma unroll
            for (int k = 0; k < CH; ++k) q[j][k] = fminf(fmaxf(q[j][k], smin), smax);
            float rmn = cmn, rmx = cmx, best_e = INFINITY;
            for (int i = 0; i < mse_steps; ++i) {
              const float pp = mse_p[i];
              const float xmn = pp * rmn, xmx = pp * rmx;
              float s2, z2;
              qparams_f32_mse(xmn, xmx, qmin, qmax, sym, s2, z2);
              float err = 0.f;
#pragma unroll
              for (int k = 0; k < CH; ++k) {
                float qq = rintf(q[j][k] / s2) + z2;
                qq = fminf(fmaxf(qq, qmin), qmax);
                err += powf(fabsf((qq - z2) * s2 - q[j][k]), norm);
              }
              const float pe = xor1(err);
              err = h ? pe + err : err + pe;  // same operand order on both lanes
              if (err < best_e) {
                best_e = err;
                rmn = xmn;
                rmx = xmx;
              }
            }
            qparams_f32_mse(rmn, rmx, qmin, qmax, sym, qs, qz);
#pragma unroll
            for (int k = 0; k < CH; ++k) {
              float tq = fminf(fmaxf(rintf(q[j][k] / qs) + qz, qmin), qmax);
              q[j][k] = dtr<DT>((tq - qz) * qs);
            }
          } else {
            clip_candidates<DT, CH>(q[j], smin, smax, cmn, cmx, qmin, qmax, sym);
          }
        }
      }
      float e[R];
#pragma unroll
      for (int j = 0; j < R; ++j) e[j] = (p > 0) ? es[(p - 1) * RW + j * CROWS + r] : 0.f;
      for (int t = 0; t < tn; ++t) {
        float d[R];
        dot_rows<DT, G, R>(&xs[t * G], q, h, d);
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if (p == 0) {
            if (h == 0) orgs[t * RW + j * CROWS + r] = dt_bits<DT>(d[j]);
          } else {
            const float dd = dtr<DT>(d[j] - dt_val<DT>(orgs[t * RW + j * CROWS + r]));
            e[j] += dtr<DT>(dd * dd);
          }
        }
      }
      if (p > 0 && h == 0)
#pragma unroll
        for (int j = 0; j < R; ++j) es[(p - 1) * RW + j * CROWS + r] = e[j];
      if (p == 0) __syncthreads();  // orgs written by the even lanes, read by both
    }
  }
  if (h) return;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (!live[j]) continue;
    float bmax = org_max[j], bmin = org_min[j], best = dtr<DT>(1e9f);
    for (int s = 0; s < nsteps; ++s) {
      const float em = dtr<DT>(es[s * RW + j * CROWS + r] / (float)T);
      if (em < best) {
        best = em;
        const float f = factors[s];
        bmax = dtr<DT>(org_max[j] * f);
        bmin = clip_sym ? -bmax : dtr<DT>(org_min[j] * f);
      }
    }
    const int64_t oi = o[j] * ng + g;
    if constexpr (DT == LCQ_BF16) {
      best_max[oi] = (uint16_t)(__float_as_uint(bmax) >> 16);
      best_min[oi] = (uint16_t)(__float_as_uint(bmin) >> 16);
    } else {
      best_max[oi] = __builtin_bit_cast(uint16_t, (_Float16)bmax);
      best_min[oi] = __builtin_bit_cast(uint16_t, (_Float16)bmin);
    }
  }
}

// ----------------------------------------------------------------------------------------
// Token-lane form of the same search (G = 128, minmax qparams, weight-only: the AWQ headline's
// auto-clip). k_auto_clip puts a row on a lane pair and broadcasts x from LDS: one LDS read per
// 16 products and a pair exchange per output kept the VALU issue at ~45 % of its peak
// (profiles/r3b_clip_pmc.json). Here a lane is a token and keeps that token's 128 x values
// of the group in VGPRs for all of a wave's rows; the candidate weights of every (row, step)
// are precomputed once (k_clip_qtable, the same arithmetic) and read as wave-uniform scalar
// loads, so the inner loop is VALU only: per product pair one v_pk_mul_f32, two
// v_cvt_pk_bf16_f32 and one v_pk_add_f32, in the same 8 partial sums and halving tree as
// dot_rows. A wave walks ALL tokens of its rows in order (64 per chunk), so each step's
// squared-error sum is accumulated in token order exactly as in k_auto_clip: the per-token
// errors of three rows go through a small per-wave LDS transpose and one lane per
// (row, step) adds them sequentially. Bit-identical to k_auto_clip (tests/test_awq_gpu.py).
// ----------------------------------------------------------------------------------------
constexpr int TL_G = 128;
constexpr int TL_RB = 6;        // rows per wave: two error flushes of three rows
constexpr int TL_WAVES = 4;     // waves per workgroup (independent; no block barrier)
constexpr int TL_EPAD = 66;     // u16 per (row, step) error row: 64 tokens + pad (no conflicts)

// candidate table of one (row, group): [nsteps + 1][G] fp32 -- pass 0 the weights themselves,
// pass s + 1 shrink step s -- and the group's (org_max, org_min)
template <int DT, int G>
__global__ void __launch_bounds__(2 * CROWS)
    k_clip_qtable(const uint16_t* __restrict__ w, int64_t ic, int64_t row0, int64_t nrows,
                  int nsteps, const float* __restrict__ factors, float qmin, float qmax, int sym,
                  int clip_sym, float* __restrict__ qt, float* __restrict__ om) {
  constexpr int CH = G / 2, CHUNKS = G / 8;
  const int tid = threadIdx.x, r = tid >> 1, h = tid & 1;
  const int64_t g = blockIdx.y, ng = ic / G;
  const int64_t lr = (int64_t)blockIdx.x * CROWS + r;
  const bool live = lr < nrows;
  uint2 raw[CHUNKS];
  fetch_half<G>(w + (row0 + (live ? lr : 0)) * ic + g * G, h, raw);
  float q0[CH];
  widen_half<DT, G>(raw, q0);
  float mx = -INFINITY, mi = INFINITY, am = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    mx = fmaxf(mx, q0[k]);
    mi = fminf(mi, q0[k]);
    am = fmaxf(am, fabsf(q0[k]));
  }
  const float mxs = fmaxf(mx, xor1(mx)), mn = fminf(mi, xor1(mi));
  am = fmaxf(am, xor1(am));
  const float org_max = clip_sym ? am : mxs, org_min = mn;
  if (!live) return;
  float* dst = qt + (lr * ng + g) * (int64_t)(nsteps + 1) * G;
  auto put = [&](const float (&q)[CH], int p) {
#pragma unroll
    for (int i = 0; i < CHUNKS; ++i)
      *reinterpret_cast<float4*>(dst + p * G + 8 * i + 4 * h) =
          make_float4(q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]);
  };
  put(q0, 0);
  for (int p = 1; p <= nsteps; ++p) {
    float q[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) q[k] = q0[k];
    const float f = factors[p - 1];
    const float smax = dtr<DT>(org_max * f);
    const float smin = clip_sym ? -smax : dtr<DT>(org_min * f);
    const float cmn = fminf(fmaxf(mn, smin), smax);
    const float cmx = fminf(fmaxf(mxs, smin), smax);
    clip_candidates<DT, CH>(q, smin, smax, cmn, cmx, qmin, qmax, sym);
    put(q, p);
  }
  if (h == 0) {
    om[(lr * ng + g) * 2] = org_max;
    om[(lr * ng + g) * 2 + 1] = org_min;
  }
}

// Candidate rows reach the VALU as scalar operands: 16 floats per s_load_dwordx16, issued one
// sub-chunk ahead. Scalar loads may return out of order, so a wait is always lgkmcnt(0); the
// next load is therefore issued right AFTER the wait for the current one and runs under the
// current sub-chunk's 32 VALU. Written as inline asm because the compiler's own scalar loads
// wait immediately (one 16-float buffer, the L2 latency exposed per 16 products: 0.65x the
// lane-pair kernel's rate). The "+s" operands order the asm statements against the compute
// that reads the buffers.
typedef uint32_t sv16 __attribute__((ext_vector_type(16)));

template <int V>
struct ic_t {
  static constexpr int value = V;
};
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(ic_t<I>{});
    static_for<I + 1, N>(f);
  }
}

// s_load_dwordx16 of base[OFF .. OFF + 16) with the offset as the instruction's immediate (one
// base pointer in SGPRs for a whole candidate row); `pin` orders the compute that reads the
// previous buffer after this issue
template <int OFF>
__device__ __forceinline__ sv16 sload16(const float* base, sv16& pin) {
  sv16 r;
  asm volatile("s_load_dwordx16 %0, %2, %3" : "=s"(r), "+s"(pin) : "s"(base), "n"(OFF * 4));
  return r;
}
// wait for the outstanding scalar load; the accumulators tie the previous sub-chunk's compute
// before the wait (else the compiler hoists the wait and exposes the load latency)
__device__ __forceinline__ void swait(sv16& r, v2f& a0, v2f& a1, v2f& a2, v2f& a3) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(r), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
}

// 16 products of this lane's token with a 16-float candidate sub-chunk, into the partial sums
// acc_{k mod 8} (a0 = (acc0, acc1) .. a3 = (acc6, acc7)) exactly as dot_rows forms them
template <int DT>
__device__ __forceinline__ void mac16(const float (&xf)[TL_G], int k0, const sv16& q, v2f& a0,
                                      v2f& a1, v2f& a2, v2f& a3) {
#pragma unroll
  for (int o = 0; o < 16; o += 8) {
    const int k = k0 + o;
    // the four products first, then their roundings, then the sums: independent instructions
    // between each result and its use (no hazard nops in the chain)
    v2f p0 = v2f{xf[k], xf[k + 1]} * v2f{__uint_as_float(q[o]), __uint_as_float(q[o + 1])};
    v2f p1 = v2f{xf[k + 2], xf[k + 3]} *
             v2f{__uint_as_float(q[o + 2]), __uint_as_float(q[o + 3])};
    v2f p2 = v2f{xf[k + 4], xf[k + 5]} *
             v2f{__uint_as_float(q[o + 4]), __uint_as_float(q[o + 5])};
    v2f p3 = v2f{xf[k + 6], xf[k + 7]} *
             v2f{__uint_as_float(q[o + 6]), __uint_as_float(q[o + 7])};
    p0 = dtr2<DT>(p0);
    p1 = dtr2<DT>(p1);
    p2 = dtr2<DT>(p2);
    p3 = dtr2<DT>(p3);
    a0 += p0;
    a1 += p1;
    a2 += p2;
    a3 += p3;
  }
}

// one weight row against this lane's token: pass 0 (the original output, org) and the NS
// shrink steps, each dot product summed as dot_rows does (8 partial sums, halving tree, one
// DT rounding); the step errors DT(DT(d - org)^2) go to er[step * TL_EPAD] (DT bits). The
// (NS + 1) x 8 sub-chunk loads form one chain, each issued one sub-chunk ahead.
template <int DT, int NS>
__device__ __forceinline__ void clip_row_tl(const float (&xf)[TL_G], const float* qr,
                                            uint16_t* er) {
  constexpr int SUB = TL_G / 16;
  sv16 cur = {}, nxt;
  cur = sload16<0>(qr, nxt);
  float org = 0.f;
  static_for<0, NS + 1>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    v2f a0 = v2f{0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    static_for<0, SUB>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      swait(cur, a0, a1, a2, a3);
      if constexpr (p == NS && c == SUB - 1) {
        mac16<DT>(xf, 16 * c, cur, a0, a1, a2, a3);
      } else {
        constexpr int off = c < SUB - 1 ? p * TL_G + 16 * (c + 1) : (p + 1) * TL_G;
        nxt = sload16<off>(qr, cur);
        mac16<DT>(xf, 16 * c, cur, a0, a1, a2, a3);
        cur = nxt;
      }
    });
    const v2f l01 = a0 + a2, l23 = a1 + a3;   // (l0, l1), (l2, l3): l_m = acc_m + acc_{m+4}
    const v2f s2 = l01 + l23;                 // (l0 + l2, l1 + l3)
    const float d = dtr<DT>(s2.x + s2.y);
    if constexpr (p == 0) {
      org = d;
    } else {
      const float dd = dtr<DT>(d - org);
      er[(p - 1) * TL_EPAD] = dt_bits<DT>(dtr<DT>(dd * dd));
    }
  });
}

// NS = 10 shrink steps (max_shrink 0.5 x n_grid 20, every shipped AWQ config)
template <int DT, int NS>
__global__ void __launch_bounds__(64 * TL_WAVES)
    k_auto_clip_tl(const uint16_t* __restrict__ x, int64_t ic, int T,
                   const float* __restrict__ qt, const float* __restrict__ om, int64_t row0,
                   int64_t nrows, const float* __restrict__ factors, int clip_sym,
                   uint16_t* __restrict__ best_max, uint16_t* __restrict__ best_min) {
  constexpr int G = TL_G, P = NS + 1, NP = 3 * NS;
  static_assert(NP <= 64, "one lane per (row, step) pair of a row triple");
  __shared__ uint16_t ebuf[TL_WAVES][NP * TL_EPAD];   // [pair][token] error bits
  __shared__ float sums[TL_WAVES][2 * NP];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t g = blockIdx.y, ng = ic / G;
  const int64_t rb = ((int64_t)blockIdx.x * TL_WAVES + w) * TL_RB;  // this wave's first row
  if (rb >= nrows) return;
  uint16_t* eb = ebuf[w];
  float* sm = sums[w];
  // row triples outermost: a triple's 3 x 11 candidate rows (17 KB) are re-read once per
  // 64-token chunk while they are still in L2
  for (int tr = 0; tr < TL_RB / 3; ++tr) {
    float run = 0.f;   // lane < NP: the error sum of pair `lane`, in token order
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + lane, tn = min(64, T - t0);
      float xf[G];
      {
        const uint16_t* xr = x + (int64_t)(t < T ? t : 0) * ic + g * G;
#pragma unroll
        for (int i = 0; i < G / 8; ++i) {
          const uint4 v = t < T ? *reinterpret_cast<const uint4*>(xr + 8 * i)
                                : make_uint4(0, 0, 0, 0);
          widen4<DT>(make_uint2(v.x, v.y), &xf[8 * i]);
          widen4<DT>(make_uint2(v.z, v.w), &xf[8 * i + 4]);
        }
      }
      for (int rr = 0; rr < 3; ++rr) {
        const int64_t lr = min(rb + 3 * tr + rr, nrows - 1);
        clip_row_tl<DT, NS>(xf, qt + (lr * ng + g) * (int64_t)P * G,
                            eb + rr * NS * TL_EPAD + lane);
      }
      // the wave's LDS requests complete in order: the other lanes' error bits written above
      // are visible to the reads below; keep the compiler from moving them across
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
      if (lane < NP) {
        const uint16_t* src = eb + lane * TL_EPAD;
        for (int u = 0; u < tn; ++u) run += dt_val<DT>(src[u]);   // token order
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
    if (lane < NP) sm[tr * NP + lane] = run;
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
  if (lane < TL_RB && rb + lane < nrows) {
    const int64_t lr = rb + lane;
    const float omax = om[(lr * ng + g) * 2], omin = om[(lr * ng + g) * 2 + 1];
    float bmax = omax, bmin = omin, best = dtr<DT>(1e9f);
    const float* e = sm + (lane / 3) * NP + (lane % 3) * NS;
    for (int s = 0; s < NS; ++s) {
      const float em = dtr<DT>(e[s] / (float)T);
      if (em < best) {
        best = em;
        const float f = factors[s];
        bmax = dtr<DT>(omax * f);
        bmin = clip_sym ? -bmax : dtr<DT>(omin * f);
      }
    }
    const int64_t oi = (row0 + lr) * ng + g;
    best_max[oi] = dt_bits<DT>(bmax);
    best_min[oi] = dt_bits<DT>(bmin);
  }
}

// Row-lane form with the activations as scalar operands (k_auto_clip_rl): a lane owns one
// weight row (64 rows per one-wave workgroup) and holds the row's candidates for the current
// pass in VGPRs (read from the k_clip_qtable table); the sampled tokens stream through SGPRs
// from an fp32 copy of x, 16 values per s_load_dwordx16, issued one sub-chunk ahead. Every
// wave of a CU on the same group reads the same token stream, so the scalar loads hit the
// scalar cache; a lane accumulates its row's step errors itself in token order (no cross-lane
// sum), the original outputs of a 128-token tile kept in LDS as DT bits.
constexpr int RL_CT = 128;   // tokens per tile

// sum_k DT(x[k] * q[k]) for this lane's candidates q (VGPRs) and the wave-uniform token row
// xr (fp32, scalar loads), in dot_rows' 8 partial sums and halving tree
template <int DT>
__device__ __forceinline__ float dot_rl(const float (&q)[TL_G], const float* xr) {
  constexpr int SUB = TL_G / 16;
  v2f a0 = v2f{0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
  sv16 cur = {}, nxt;
  cur = sload16<0>(xr, nxt);
  static_for<0, SUB>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    swait(cur, a0, a1, a2, a3);
    if constexpr (c == SUB - 1) {
      mac16<DT>(q, 16 * c, cur, a0, a1, a2, a3);
    } else {
      nxt = sload16<16 * (c + 1)>(xr, cur);
      mac16<DT>(q, 16 * c, cur, a0, a1, a2, a3);
      cur = nxt;
    }
  });
  const v2f l01 = a0 + a2, l23 = a1 + a3;
  const v2f s2 = l01 + l23;
  return dtr<DT>(s2.x + s2.y);
}

template <int DT, int NS>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))   // <= 168 VGPRs
    k_auto_clip_rl(const float* __restrict__ xt, int64_t ic, int T, const float* __restrict__ qt,
                   const float* __restrict__ om, int64_t row0, int64_t nrows,
                   const float* __restrict__ factors, int clip_sym,
                   uint16_t* __restrict__ best_max, uint16_t* __restrict__ best_min) {
  constexpr int G = TL_G, P = NS + 1;
  __shared__ uint16_t orgs[RL_CT * 64];   // [token][lane] original outputs (DT bits)
  const int lane = threadIdx.x;
  const int64_t g = blockIdx.y, ng = ic / G;
  const int64_t lr = (int64_t)blockIdx.x * 64 + lane;
  const bool live = lr < nrows;
  const float* qrow = qt + ((live ? lr : 0) * ng + g) * (int64_t)P * G;
  const float* xg = xt + g * G;
  float e[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) e[s] = 0.f;
  for (int t0 = 0; t0 < T; t0 += RL_CT) {
    const int tn = min(RL_CT, T - t0);
    static_for<0, P>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      float q[G];
      // re-read per tile (an opaque pointer: hoisting every pass's candidates out of the tile
      // loop would hold 11 x 128 values per lane)
      int poff = p * G;
      asm volatile("" : "+s"(poff));
      const float* qp = qrow + poff;
#pragma unroll
      for (int i = 0; i < G / 4; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(qp + 4 * i);
        q[4 * i] = v.x; q[4 * i + 1] = v.y; q[4 * i + 2] = v.z; q[4 * i + 3] = v.w;
      }
      float acc = p > 0 ? e[p > 0 ? p - 1 : 0] : 0.f;
      for (int t = 0; t < tn; ++t) {
        const float d = dot_rl<DT>(q, xg + (int64_t)(t0 + t) * ic);
        if constexpr (p == 0) {
          orgs[t * 64 + lane] = dt_bits<DT>(d);
        } else {
          const float dd = dtr<DT>(d - dt_val<DT>(orgs[t * 64 + lane]));
          acc += dtr<DT>(dd * dd);   // token order
        }
      }
      if constexpr (p > 0) e[p - 1] = acc;
    });
  }
  if (!live) return;
  const float omax = om[(lr * ng + g) * 2], omin = om[(lr * ng + g) * 2 + 1];
  float bmax = omax, bmin = omin, best = dtr<DT>(1e9f);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const float em = dtr<DT>(e[s] / (float)T);
    if (em < best) {
      best = em;
      const float f = factors[s];
      bmax = dtr<DT>(omax * f);
      bmin = clip_sym ? -bmax : dtr<DT>(omin * f);
    }
  }
  const int64_t oi = (row0 + lr) * ng + g;
  best_max[oi] = dt_bits<DT>(bmax);
  best_min[oi] = dt_bits<DT>(bmin);
}

// ----------------------------------------------------------------------------------------
// Token-lane form with the candidates staged in LDS (k_auto_clip_tw): the AWQ headline's
// auto-clip (G = 128, minmax qparams, weight-only, T <= 512 sampled tokens).
// k_auto_clip_tl fed the candidates through scalar loads, whose latency (one lgkmcnt(0) per
// 16 products: scalar loads return out of order) left the VALU issuing 1 instruction per ~7
// cycles, and each of its 64-token waves re-read every candidate row (8x the table at 512
// tokens). Here one workgroup of 8 waves holds ALL T tokens (lane = token, its 128 x values
// of the group widened in VGPRs) and walks TW_RPW rows of one group in sets of TW_R rows:
//  * a set's candidate rows ([TW_R][11][128] fp32, the k_clip_qtable table) come into one of
//    two LDS buffers by LDS-DMA, issued one set ahead (no VGPRs, no wait inside the compute);
//  * the compute reads them as wave-uniform ds_read_b128 broadcasts (4 per 16 products, the
//    next 16 in flight under the current 16's 32 VALU): per product pair one v_pk_mul_f32,
//    two v_cvt_pk_bf16_f32, one v_pk_add_f32, the 8 partial sums and halving tree of dot_rows;
//  * each (row, step)'s per-token errors (DT bits) go to an LDS row [pair][token]; one set
//    later one wave (rotating) sums each pair's T errors sequentially in token order -- the
//    order k_auto_clip and k_auto_clip_tl use -- and picks the first strict minimum.
// LDS: 2 x 22.5 KB candidates + 2 x 40.6 KB error rows = 126 KB: one workgroup per CU.
// Bit-identical to k_auto_clip (tests/test_awq_gpu.py).
// ----------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) char lds_char_t;
constexpr int TW_WAVES = 8;             // 512 lanes = up to 512 sampled tokens
constexpr int TW_R = 4;                  // rows per LDS set
constexpr int TW_RPW = 64;               // rows per workgroup
constexpr int TW_EPAD = 520;             // u16 per (row, step) error row: 512 tokens + pad
constexpr int TW_NS = 10;
constexpr int TW_P = TW_NS + 1;
constexpr int TW_CAND = TW_R * TW_P * TL_G;           // floats per candidate buffer
constexpr int TW_PAIRS = TW_R * TW_NS;                // (row, step) pairs per set
constexpr int TW_LDS = 2 * TW_CAND * 4 + 2 * TW_PAIRS * TW_EPAD * 2 + TW_PAIRS * 4;
static_assert(TW_CAND * 4 % 1024 == 0, "candidate buffer = whole 1 KB DMA pieces");
static_assert(TW_PAIRS <= 64, "one summing lane per (row, step) pair");

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tw_rsrc(const void* p, uint32_t bytes) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)bytes, 0x00020000);
}

// 16 products of this lane's token with 16 candidates (4 float4 from LDS), into the partial
// sums acc_{k mod 8} exactly as mac16 / dot_rows form them
template <int DT>
__device__ __forceinline__ void mac16v(const float (&xf)[TL_G], int k0, const float4 (&q)[4],
                                       v2f& a0, v2f& a1, v2f& a2, v2f& a3) {
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int k = k0 + 8 * o;
    const float4 u = q[2 * o], v = q[2 * o + 1];
    v2f p0 = v2f{xf[k], xf[k + 1]} * v2f{u.x, u.y};
    v2f p1 = v2f{xf[k + 2], xf[k + 3]} * v2f{u.z, u.w};
    v2f p2 = v2f{xf[k + 4], xf[k + 5]} * v2f{v.x, v.y};
    v2f p3 = v2f{xf[k + 6], xf[k + 7]} * v2f{v.z, v.w};
    p0 = dtr2<DT>(p0);
    p1 = dtr2<DT>(p1);
    p2 = dtr2<DT>(p2);
    p3 = dtr2<DT>(p3);
    a0 += p0;
    a1 += p1;
    a2 += p2;
    a3 += p3;
  }
}

template <int DT>
__global__ void __launch_bounds__(64 * TW_WAVES)
    k_auto_clip_tw(const uint16_t* __restrict__ x, int64_t ic, int T,
                   const float* __restrict__ qt, uint32_t qt_bytes, const float* __restrict__ om,
                   int64_t row0, int64_t nrows, const float* __restrict__ factors, int clip_sym,
                   uint16_t* __restrict__ best_max, uint16_t* __restrict__ best_min) {
  constexpr int G = TL_G, NS = TW_NS, P = TW_P;
  extern __shared__ __attribute__((aligned(16))) float tw_lds[];
  float* cand = tw_lds;                                                     // [2][R][P][G]
  uint16_t* ebuf = reinterpret_cast<uint16_t*>(tw_lds + 2 * TW_CAND);       // [2][pairs][EPAD]
  float* sums = reinterpret_cast<float*>(ebuf + 2 * TW_PAIRS * TW_EPAD);    // [pairs]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int t = w * 64 + lane;
  const int64_t g = blockIdx.y, ng = ic / G;
  const int64_t rw0 = (int64_t)blockIdx.x * TW_RPW;
  const int64_t nr = nrows - rw0 < TW_RPW ? nrows - rw0 : TW_RPW;
  const int nsets = (int)((nr + TW_R - 1) / TW_R);
  const __amdgpu_buffer_rsrc_t rs = tw_rsrc(qt, qt_bytes);

  // set s's candidate rows -> cand[s & 1]: 1 KB pieces m = w, w + 8, ... of the 22 per set;
  // 16-B chunk c = 64 m + lane is float4 `c % 352` of the set's row `c / 352`. Issued as
  // inline asm: with the builtin the compiler's waitcnt pass puts a vmcnt(0) before the next
  // ds_read (it cannot tell the DMA's LDS range from the reads'), exposing the whole DMA
  // latency once per set; the kernel waits for its DMA itself before each set's barrier.
  // M0 (the wave's LDS destination) is saved and restored inside the statement.
  auto dma_set = [&](int s) {
    const uint32_t base = (uint32_t)(size_t)(lds_char_t*)(cand + (s & 1) * TW_CAND);
    for (int m = w; m < TW_CAND * 4 / 1024; m += TW_WAVES) {
      const int c = m * 64 + lane;
      const int rr = c / (P * G / 4), within = c % (P * G / 4);
      int64_t lr = rw0 + (int64_t)s * TW_R + rr;
      if (lr > nrows - 1) lr = nrows - 1;
      const uint32_t off = (uint32_t)(((lr * ng + g) * P * G) * 4 + within * 16);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(base + m * 1024);
      uint32_t sv;
      asm volatile(
          "s_mov_b32 %0, m0\n\t"
          "s_mov_b32 m0, %1\n\t"
          "s_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
          "s_mov_b32 m0, %0"
          : "=&s"(sv)
          : "s"(dst), "v"(off), "s"(rs)
          : "memory");
    }
  };

  // one set's error rows: token-order sums, then the first strict minimum per row
  auto sum_pick = [&](int s) {
    const uint16_t* eb = ebuf + (s & 1) * TW_PAIRS * TW_EPAD;
    if (lane < TW_PAIRS) {
      const uint16_t* src = eb + lane * TW_EPAD;
      float run = 0.f;
      int u = 0;
      for (; u + 8 <= T; u += 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + u);
        const uint32_t a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          run += dt_val<DT>((uint16_t)(a[j] & 0xffffu));
          run += dt_val<DT>((uint16_t)(a[j] >> 16));
        }
      }
      for (; u < T; ++u) run += dt_val<DT>(src[u]);
      sums[lane] = run;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const int64_t lr = rw0 + (int64_t)s * TW_R + lane;
    if (lane < TW_R && lr < nrows) {
      const float omax = om[(lr * ng + g) * 2], omin = om[(lr * ng + g) * 2 + 1];
      float bmax = omax, bmin = omin, best = dtr<DT>(1e9f);
      for (int st = 0; st < NS; ++st) {
        const float em = dtr<DT>(sums[lane * NS + st] / (float)T);
        if (em < best) {
          best = em;
          const float f = factors[st];
          bmax = dtr<DT>(omax * f);
          bmin = clip_sym ? -bmax : dtr<DT>(omin * f);
        }
      }
      const int64_t oi = (row0 + lr) * ng + g;
      best_max[oi] = dt_bits<DT>(bmax);
      best_min[oi] = dt_bits<DT>(bmin);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  };

  dma_set(0);
  float xf[G];
  {
    const uint16_t* xr = x + (int64_t)(t < T ? t : 0) * ic + g * G;
#pragma unroll
    for (int i = 0; i < G / 8; ++i) {
      const uint4 v = t < T ? *reinterpret_cast<const uint4*>(xr + 8 * i) : make_uint4(0, 0, 0, 0);
      widen4<DT>(make_uint2(v.x, v.y), &xf[8 * i]);
      widen4<DT>(make_uint2(v.z, v.w), &xf[8 * i + 4]);
    }
  }
  for (int s = 0; s < nsets; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // cand[s & 1] landed; set s - 1's error rows complete
    if (s >= 1 && w == (s - 1) % TW_WAVES) sum_pick(s - 1);
    if (s + 1 < nsets) dma_set(s + 1);
    const float* cs = cand + (s & 1) * TW_CAND;
    uint16_t* eb = ebuf + (s & 1) * TW_PAIRS * TW_EPAD + t;
    // the set's R x P candidate rows are one contiguous walk: chunk c + 2's reads are issued
    // under chunk c's products, across pass boundaries too (the walk's last two prefetches
    // read the 32 floats after the buffer: LDS in bounds, unused)
    float4 q0[4], q1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q0[j] = reinterpret_cast<const float4*>(cs)[j];
      q1[j] = reinterpret_cast<const float4*>(cs + 16)[j];
    }
    float org = 0.f;
#pragma unroll 1
    for (int rp = 0; rp < TW_R * P; ++rp) {
      const float* qp = cs + rp * G;
      v2f a0 = v2f{0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
#pragma unroll
      for (int c = 0; c < G / 16; c += 2) {
        float4 q2[4], q3[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q2[j] = reinterpret_cast<const float4*>(qp + 16 * (c + 2))[j];
        mac16v<DT>(xf, 16 * c, q0, a0, a1, a2, a3);
#pragma unroll
        for (int j = 0; j < 4; ++j) q3[j] = reinterpret_cast<const float4*>(qp + 16 * (c + 3))[j];
        mac16v<DT>(xf, 16 * (c + 1), q1, a0, a1, a2, a3);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          q0[j] = q2[j];
          q1[j] = q3[j];
        }
      }
      const v2f l01 = a0 + a2, l23 = a1 + a3;   // l_m = acc_m + acc_{m+4}
      const v2f s2 = l01 + l23;                 // (l0 + l2, l1 + l3)
      const float d = dtr<DT>(s2.x + s2.y);
      const int r = rp / P, p = rp - r * P;
      if (p == 0) {
        org = d;
      } else {
        const float dd = dtr<DT>(d - org);
        eb[(r * NS + p - 1) * TW_EPAD] = dt_bits<DT>(dtr<DT>(dd * dd));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (w == (nsets - 1) % TW_WAVES) sum_pick(nsets - 1);
}

// x [T, ic] in DT -> fp32 (the scalar-operand token stream of k_auto_clip_rl)
template <int DT>
__global__ void __launch_bounds__(256) k_widen_f32(const uint16_t* __restrict__ x, int64_t n8,
                                                   float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const uint4 v = reinterpret_cast<const uint4*>(x)[i];
    float a[8];
    widen4<DT>(make_uint2(v.x, v.y), a);
    widen4<DT>(make_uint2(v.z, v.w), a + 4);
    reinterpret_cast<float4*>(out)[2 * i] = make_float4(a[0], a[1], a[2], a[3]);
    reinterpret_cast<float4*>(out)[2 * i + 1] = make_float4(a[4], a[5], a[6], a[7]);
  }
}

template <int DT>
__global__ void __launch_bounds__(256) k_clip_apply(const void* x, int64_t rows, int64_t cols,
                                                   int64_t group, const void* cmax,
                                                   const void* cmin, void* out) {
  const int64_t n8 = rows * cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8, gi = e0 / group;
    float v[8];
    ld8<DT>(x, e0, v);
    const float mx = ld1<DT>(cmax, gi);
    const float mn = cmin ? ld1<DT>(cmin, gi) : -mx;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fminf(fmaxf(v[j], mn), mx);
    st8<DT>(out, e0, v);
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int64_t lcq_colmean_workspace_bytes(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int lp = colsum_lp(rows);
  const int64_t SB = (int64_t)1 << (2 * lp);
  return (((rows + SB - 1) / SB) + 1) * cols * (int64_t)sizeof(float);
}

template <int DT, int MODE>
static void launch_colmean(const void* x, int64_t rows, int64_t c, int glanes, int layer,
                           int nlayers, void* out, void* workspace, hipStream_t st) {
  const int lp = colsum_lp(rows);
  const int64_t SB = (int64_t)1 << (2 * lp);
  const int64_t nsb = (rows + SB - 1) / SB;
  float* part = reinterpret_cast<float*>(workspace);
  float* tail = part + nsb * c;
  dim3 g1((unsigned)((c / 8 + 255) / 256), (unsigned)nsb);
  hipLaunchKernelGGL((k_colsum_l1<DT, MODE>), g1, 256, 0, st, x, rows, c, lp, glanes, part, tail);
  hipLaunchKernelGGL((k_colsum_fold<DT, MODE>), dim3((unsigned)((c + 255) / 256)), 256, 0, st,
                     part, tail, rows, c, lp, layer, nlayers, out);
}

extern "C" int lcq_absmean_cols(const void* x, int dtype, int64_t n, int64_t c, void* out,
                                void* workspace, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(n > 0 && c > 0 && c % 8 == 0, "c must be a positive multiple of 8");
  LCQ_REQUIRE(workspace, "workspace of lcq_colmean_workspace_bytes(n, c) required");
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case LCQ_BF16: launch_colmean<LCQ_BF16, 0>(x, n, c, 1, 0, 1, out, workspace, st); break;
    case LCQ_F16: launch_colmean<LCQ_F16, 0>(x, n, c, 1, 0, 1, out, workspace, st); break;
    default: launch_colmean<LCQ_F32, 0>(x, n, c, 1, 0, 1, out, workspace, st);
  }
  return check_launch("lcq_absmean_cols");
}

extern "C" int lcq_awq_weight_scale(const void* w, int dtype, int64_t rows, int64_t cols,
                                    int64_t group, int layer, int nlayers, void* total,
                                    void* workspace, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(rows > 0 && cols > 0, "empty weight");
  LCQ_REQUIRE(group >= 8 && group % 8 == 0 && cols % group == 0,
              "group must be a multiple of 8 dividing cols");
  const int64_t gl = group / 8;
  LCQ_REQUIRE(gl <= 64 && (gl & (gl - 1)) == 0, "group / 8 must be a power of two <= 64");
  LCQ_REQUIRE(layer >= 0 && layer < nlayers, "layer index out of range");
  LCQ_REQUIRE(workspace && total, "null pointer");
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case LCQ_BF16: launch_colmean<LCQ_BF16, 1>(w, rows, cols, (int)gl, layer, nlayers, total, workspace, st); break;
    case LCQ_F16: launch_colmean<LCQ_F16, 1>(w, rows, cols, (int)gl, layer, nlayers, total, workspace, st); break;
    default: launch_colmean<LCQ_F32, 1>(w, rows, cols, (int)gl, layer, nlayers, total, workspace, st);
  }
  return check_launch("lcq_awq_weight_scale");
}

static int awq_scales_impl(const void* xmean, const void* wmax, int dtype, int64_t c,
                           float ratio_dt, float wexp_dt, void* out, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(c > 0, "empty");
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case LCQ_BF16: hipLaunchKernelGGL((k_awq_scales<LCQ_BF16>), 1, 1024, 0, st, xmean, c, ratio_dt, out, wmax, wexp_dt); break;
    case LCQ_F16: hipLaunchKernelGGL((k_awq_scales<LCQ_F16>), 1, 1024, 0, st, xmean, c, ratio_dt, out, wmax, wexp_dt); break;
    default: hipLaunchKernelGGL((k_awq_scales<LCQ_F32>), 1, 1024, 0, st, xmean, c, ratio_dt, out, wmax, wexp_dt);
  }
  return check_launch("lcq_awq_scales");
}

extern "C" int lcq_awq_scales(const void* xmean, int dtype, int64_t c, float ratio_dt,
                              void* out, void* stream) {
  return awq_scales_impl(xmean, nullptr, dtype, c, ratio_dt, 0.f, out, stream);
}

extern "C" int lcq_awq_scales_v1(const void* xmean, const void* wmax, int dtype, int64_t c,
                                 float ratio_dt, float wexp_dt, void* out, void* stream) {
  LCQ_REQUIRE(wmax != nullptr, "wmax required");
  return awq_scales_impl(xmean, wmax, dtype, c, ratio_dt, wexp_dt, out, stream);
}

template <int DT>
static void launch_scale(const void* x, int64_t rows, int64_t cols, const void* s, int op,
                         int axis, void* out, hipStream_t st) {
  int64_t rb = SB_ROWS;
  if ((rows + rb - 1) / rb > 65535) rb = (rows + 65534) / 65535;
  const dim3 grid((unsigned)((cols / 8 + 255) / 256), (unsigned)((rows + rb - 1) / rb));
  if (op == 0 && axis == 0) hipLaunchKernelGGL((k_scale_bcast<DT, 0, 0>), grid, 256, 0, st, x, rows, cols, s, out, rb);
  if (op == 1 && axis == 0) hipLaunchKernelGGL((k_scale_bcast<DT, 1, 0>), grid, 256, 0, st, x, rows, cols, s, out, rb);
  if (op == 0 && axis == 1) hipLaunchKernelGGL((k_scale_bcast<DT, 0, 1>), grid, 256, 0, st, x, rows, cols, s, out, rb);
  if (op == 1 && axis == 1) hipLaunchKernelGGL((k_scale_bcast<DT, 1, 1>), grid, 256, 0, st, x, rows, cols, s, out, rb);
}

extern "C" int lcq_scale_bcast(const void* x, int dtype, int64_t rows, int64_t cols,
                               const void* s, int op, int axis, void* out, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(rows > 0 && cols > 0 && cols % 8 == 0, "cols must be a positive multiple of 8");
  LCQ_REQUIRE((op == 0 || op == 1) && (axis == 0 || axis == 1), "bad op/axis");
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case LCQ_BF16: launch_scale<LCQ_BF16>(x, rows, cols, s, op, axis, out, st); break;
    case LCQ_F16: launch_scale<LCQ_F16>(x, rows, cols, s, op, axis, out, st); break;
    default: launch_scale<LCQ_F32>(x, rows, cols, s, op, axis, out, st);
  }
  return check_launch("lcq_scale_bcast");
}

extern "C" int lcq_sq_diff_mean(const void* a, const void* b, int dtype, int64_t n,
                                void* workspace, int nparts, void* out_f32, int slot,
                                void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(n > 0 && n % 8 == 0, "n must be a positive multiple of 8");
  LCQ_REQUIRE(nparts >= 1 && workspace, "workspace of nparts fp64 required");
  hipStream_t st = as_stream(stream);
  double* part = reinterpret_cast<double*>(workspace);
  switch (dtype) {
    case LCQ_BF16: hipLaunchKernelGGL((k_sqdiff_p1<LCQ_BF16>), nparts, 256, 0, st, a, b, n, part); break;
    case LCQ_F16: hipLaunchKernelGGL((k_sqdiff_p1<LCQ_F16>), nparts, 256, 0, st, a, b, n, part); break;
    default: hipLaunchKernelGGL((k_sqdiff_p1<LCQ_F32>), nparts, 256, 0, st, a, b, n, part);
  }
  hipLaunchKernelGGL(k_sqdiff_p2, 1, 64, 0, st, part, nparts, n,
                     reinterpret_cast<float*>(out_f32), slot);
  return check_launch("lcq_sq_diff_mean");
}

struct ClipLaunch {
  const void* w;
  const void* x;
  int64_t oc, ic, T;
  int nsteps;
  const void* factors;
  int qmin, qmax, sym, clip_sym;
  void* bmax;
  void* bmin;
  int mse_steps;
  const void* mse_p;
  float norm;
  const void* qx;
};

template <int DT, int G, int R, bool MSE>
static void launch_auto_clip_r(const ClipLaunch& c, hipStream_t st) {
  constexpr int lds = ClipTile<G, R>::bytes;
  auto k = k_auto_clip<DT, G, R, MSE>;
  // dynamic LDS beyond 64 KB needs the attribute (per device: set on every launch, cheap)
  hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  dim3 grid((unsigned)((c.oc + CROWS * R - 1) / (CROWS * R)), (unsigned)(c.ic / G));
  hipLaunchKernelGGL(k, grid, 2 * CROWS, lds, st,
                     reinterpret_cast<const uint16_t*>(c.w), reinterpret_cast<const uint16_t*>(c.x),
                     c.oc, c.ic, (int)c.T, c.nsteps, reinterpret_cast<const float*>(c.factors),
                     (float)c.qmin, (float)c.qmax, c.sym, c.clip_sym,
                     reinterpret_cast<uint16_t*>(c.bmax), reinterpret_cast<uint16_t*>(c.bmin),
                     c.mse_steps, reinterpret_cast<const float*>(c.mse_p), c.norm,
                     reinterpret_cast<const uint16_t*>(c.qx));
}

// two rows per lane pair where the grid still fills the chip twice over (512 workgroups at
// 2 per CU); below that (v_proj 1024 x 4096: 128 workgroups) one row per lane pair
template <int DT, int G, bool MSE>
static void launch_auto_clip(const ClipLaunch& c, hipStream_t st) {
  constexpr bool two = G <= 128 && !MSE;
  const int64_t wg2 = (c.oc + 2 * CROWS - 1) / (2 * CROWS) * (c.ic / G);
  if (two && wg2 >= 512) launch_auto_clip_r<DT, G, two ? 2 : 1, MSE>(c, st);
  else launch_auto_clip_r<DT, G, 1, MSE>(c, st);
}

template <int DT, bool MSE>
static void auto_clip_group(int group, const ClipLaunch& c, hipStream_t st) {
  switch (group) {
    case 32: launch_auto_clip<DT, 32, MSE>(c, st); break;
    case 64: launch_auto_clip<DT, 64, MSE>(c, st); break;
    case 128: launch_auto_clip<DT, 128, MSE>(c, st); break;
    default: launch_auto_clip<DT, 256, MSE>(c, st);
  }
}

extern "C" int lcq_auto_clip_search(const void* w, const void* x, int dtype, int64_t oc,
                                    int64_t ic, int64_t T, int group, int nsteps,
                                    const void* factors, int qmin, int qmax, int sym,
                                    int clip_sym, int mse_steps, const void* mse_p, float norm,
                                    void* best_max, void* best_min, void* stream) {
  return lcq_auto_clip_search_act(w, x, nullptr, dtype, oc, ic, T, group, nsteps, factors, qmin,
                                  qmax, sym, clip_sym, mse_steps, mse_p, norm, best_max,
                                  best_min, stream);
}

extern "C" int lcq_auto_clip_search_act(const void* w, const void* x, const void* qx, int dtype,
                                        int64_t oc, int64_t ic, int64_t T, int group,
                                        int nsteps, const void* factors, int qmin, int qmax,
                                        int sym, int clip_sym, int mse_steps, const void* mse_p,
                                        float norm, void* best_max, void* best_min,
                                        void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "auto-clip: bf16 or fp16 model dtype");
  LCQ_REQUIRE(group == 32 || group == 64 || group == 128 || group == CGMAX,
              "auto-clip kernel supports group_size 32 / 64 / 128 / 256");
  LCQ_REQUIRE(oc > 0 && ic > 0 && ic % group == 0, "ic must be a multiple of the group size");
  LCQ_REQUIRE(T > 0 && nsteps >= 1 && nsteps <= CMAXSTEPS, "bad T / nsteps (<= 16)");
  LCQ_REQUIRE(qmax > qmin, "qmax <= qmin");
  LCQ_REQUIRE(mse_steps == 0 || (mse_steps > 0 && mse_p != nullptr && norm > 0.f),
              "mse: steps > 0 need the shrink factors and a positive norm");
  hipStream_t st = as_stream(stream);
  const ClipLaunch c{w, x, oc, ic, T, nsteps, factors, qmin, qmax, sym, clip_sym, best_max,
                     best_min, mse_steps, mse_p, norm, qx};
  if (dtype == LCQ_BF16) {
    if (mse_steps) auto_clip_group<LCQ_BF16, true>(group, c, st);
    else auto_clip_group<LCQ_BF16, false>(group, c, st);
  } else {
    if (mse_steps) auto_clip_group<LCQ_F16, true>(group, c, st);
    else auto_clip_group<LCQ_F16, false>(group, c, st);
  }
  return check_launch("lcq_auto_clip_search");
}

// scalar-operand paths: candidate-table bytes per weight row (fp32 [ng][nsteps + 1][128] + the
// group ranges), the row chunk one table covers (tables of at most 1 GiB), and the fp32 copy
// of x the row-lane kernel streams
static int64_t tl_row_bytes(int64_t ic, int nsteps) {
  return ic / TL_G * ((int64_t)(nsteps + 1) * TL_G + 2) * 4;
}
static constexpr int64_t TL_ROWS_PER_WG = TL_WAVES * TL_RB;   // token-lane rows per workgroup
static constexpr int64_t CL_ROW_UNIT = 192;   // chunk rows: whole workgroups of both kernels
static constexpr int TL_NS = 10;   // the kernels' shrink-step count
static constexpr int64_t CL_PAIR_MIN_ROWGROUPS = 65536;   // automatic choice, see below

// A/B probe hook (scripts/clip_rate.py): 0 = automatic, 1 = token-lane (scalar candidates),
// 2 = row-lane, 3 = token-lane with LDS candidates (k_auto_clip_tw). Process-wide; not for
// production use. Automatic: k_auto_clip_tw whenever the sampled tokens fit its 512 lanes (it
// wins at every Llama-3-8B shape: v / o / gate,up / down 1.80 / 6.63 / 24.9 / 24.1 ms against
// 2.44 / 10.4 / 34.5 / 35.5 for the scalar-candidate token-lane kernel and 3.25 / 8.22 / 27.1 /
// 27.1 for k_auto_clip, profiles/r6_clip_rate_tw.txt); above 512 tokens the round-6 rule: the
// scalar-candidate kernel below 65536 row-groups, k_auto_clip (lcq_auto_clip_search_act) from
// there. All four give the same bits.
static int g_clip_variant = 0;
extern "C" int lcq_auto_clip_force_variant(int v) {
  LCQ_REQUIRE(v >= 0 && v <= 3, "variant: 0, 1, 2 or 3");
  g_clip_variant = v;
  return LCQ_OK;
}

extern "C" int64_t lcq_auto_clip_workspace_bytes(int64_t oc, int64_t ic, int64_t T, int group,
                                                 int nsteps) {
  if (group != TL_G || oc <= 0 || ic <= 0 || T <= 0 || ic % TL_G || nsteps != TL_NS) return 0;
  if (g_clip_variant == 0 && T > 64 * TW_WAVES && oc * (ic / TL_G) >= CL_PAIR_MIN_ROWGROUPS)
    return 0;  // k_auto_clip
  const int64_t per = tl_row_bytes(ic, nsteps);
  int64_t rows = ((int64_t)1 << 30) / per / CL_ROW_UNIT * CL_ROW_UNIT;
  if (rows < CL_ROW_UNIT) rows = CL_ROW_UNIT;
  const int64_t need = (oc + CL_ROW_UNIT - 1) / CL_ROW_UNIT * CL_ROW_UNIT;
  return (rows < need ? rows : need) * per + T * ic * 4;
}

extern "C" int lcq_auto_clip_search_ws(const void* w, const void* x, const void* qx, int dtype,
                                       int64_t oc, int64_t ic, int64_t T, int group,
                                       int nsteps, const void* factors, int qmin, int qmax,
                                       int sym, int clip_sym, int mse_steps, const void* mse_p,
                                       float norm, void* best_max, void* best_min,
                                       void* workspace, int64_t ws_bytes, void* stream) {
  const bool shape_ok = group == TL_G && ic > 0 && ic % TL_G == 0 && nsteps == TL_NS && T > 0 &&
                        T < ((int64_t)1 << 31) && oc > 0;
  const int64_t per = shape_ok ? tl_row_bytes(ic, nsteps) : 0;
  const int64_t xbytes = shape_ok ? T * ic * 4 : 0;
  int64_t chunk =
      per && ws_bytes > xbytes ? (ws_bytes - xbytes) / per / CL_ROW_UNIT * CL_ROW_UNIT : 0;
  // a chunk's table stays below 2 GiB (32-bit DMA offsets of k_auto_clip_tw)
  if (per && chunk * per >= ((int64_t)1 << 31))
    chunk = (((int64_t)1 << 31) - 1) / per / CL_ROW_UNIT * CL_ROW_UNIT;
  const bool al16 = ((reinterpret_cast<uintptr_t>(workspace) | reinterpret_cast<uintptr_t>(x)) &
                     15) == 0;
  const bool tw_fits = T <= 64 * TW_WAVES;
  const bool pair_wins =
      g_clip_variant == 0 && !tw_fits && oc * (ic / TL_G) >= CL_PAIR_MIN_ROWGROUPS;
  if (qx != nullptr || mse_steps != 0 || chunk < CL_ROW_UNIT || workspace == nullptr || !al16 ||
      (dtype != LCQ_BF16 && dtype != LCQ_F16) || qmax <= qmin || pair_wins)
    return lcq_auto_clip_search_act(w, x, qx, dtype, oc, ic, T, group, nsteps, factors, qmin,
                                    qmax, sym, clip_sym, mse_steps, mse_p, norm, best_max,
                                    best_min, stream);
  hipStream_t st = as_stream(stream);
  const int64_t ng = ic / TL_G;
  const bool rl = g_clip_variant == 2;
  const bool tw = (g_clip_variant == 0 || g_clip_variant == 3) && tw_fits;
  if (tw) {
    auto kb = k_auto_clip_tw<LCQ_BF16>;
    auto kh = k_auto_clip_tw<LCQ_F16>;
    hipFuncSetAttribute(reinterpret_cast<const void*>(kb),
                        hipFuncAttributeMaxDynamicSharedMemorySize, TW_LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(kh),
                        hipFuncAttributeMaxDynamicSharedMemorySize, TW_LDS);
  }
  float* xt =reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + chunk * per);
  float* qt = reinterpret_cast<float*>(workspace);
  const auto* wp = reinterpret_cast<const uint16_t*>(w);
  const auto* xp = reinterpret_cast<const uint16_t*>(x);
  const auto* fp = reinterpret_cast<const float*>(factors);
  auto* bx = reinterpret_cast<uint16_t*>(best_max);
  auto* bn = reinterpret_cast<uint16_t*>(best_min);
  if (rl) {
    const int64_t n8 = T * ic / 8;
    if (dtype == LCQ_BF16)
      hipLaunchKernelGGL(k_widen_f32<LCQ_BF16>, stream_grid(n8, 256), 256, 0, st, xp, n8, xt);
    else
      hipLaunchKernelGGL(k_widen_f32<LCQ_F16>, stream_grid(n8, 256), 256, 0, st, xp, n8, xt);
  }
  for (int64_t r0 = 0; r0 < oc; r0 += chunk) {
    const int64_t nr = oc - r0 < chunk ? oc - r0 : chunk;
    float* om = qt + nr * ng * (int64_t)(nsteps + 1) * TL_G;
    const dim3 g1((unsigned)((nr + CROWS - 1) / CROWS), (unsigned)ng);
    const dim3 g2((unsigned)((nr + TL_ROWS_PER_WG - 1) / TL_ROWS_PER_WG), (unsigned)ng);
    const dim3 g3((unsigned)((nr + 63) / 64), (unsigned)ng);
    const dim3 g4((unsigned)((nr + TW_RPW - 1) / TW_RPW), (unsigned)ng);
    const uint32_t qtb = (uint32_t)(nr * ng * (int64_t)(nsteps + 1) * TL_G * 4);
    if (dtype == LCQ_BF16) {
      hipLaunchKernelGGL((k_clip_qtable<LCQ_BF16, TL_G>), g1, 2 * CROWS, 0, st, wp, ic, r0, nr,
                         nsteps, fp, (float)qmin, (float)qmax, sym, clip_sym, qt, om);
      if (tw)
        hipLaunchKernelGGL((k_auto_clip_tw<LCQ_BF16>), g4, 64 * TW_WAVES, TW_LDS, st, xp, ic,
                           (int)T, qt, qtb, om, r0, nr, fp, clip_sym, bx, bn);
      else if (rl)
        hipLaunchKernelGGL((k_auto_clip_rl<LCQ_BF16, TL_NS>), g3, 64, 0, st, xt, ic, (int)T, qt,
                           om, r0, nr, fp, clip_sym, bx, bn);
      else
        hipLaunchKernelGGL((k_auto_clip_tl<LCQ_BF16, TL_NS>), g2, 64 * TL_WAVES, 0, st, xp, ic,
                           (int)T, qt, om, r0, nr, fp, clip_sym, bx, bn);
    } else {
      hipLaunchKernelGGL((k_clip_qtable<LCQ_F16, TL_G>), g1, 2 * CROWS, 0, st, wp, ic, r0, nr,
                         nsteps, fp, (float)qmin, (float)qmax, sym, clip_sym, qt, om);
      if (tw)
        hipLaunchKernelGGL((k_auto_clip_tw<LCQ_F16>), g4, 64 * TW_WAVES, TW_LDS, st, xp, ic,
                           (int)T, qt, qtb, om, r0, nr, fp, clip_sym, bx, bn);
      else if (rl)
        hipLaunchKernelGGL((k_auto_clip_rl<LCQ_F16, TL_NS>), g3, 64, 0, st, xt, ic, (int)T, qt,
                           om, r0, nr, fp, clip_sym, bx, bn);
      else
        hipLaunchKernelGGL((k_auto_clip_tl<LCQ_F16, TL_NS>), g2, 64 * TL_WAVES, 0, st, xp, ic,
                           (int)T, qt, om, r0, nr, fp, clip_sym, bx, bn);
    }
    const int rc = check_launch("lcq_auto_clip_search_ws");
    if (rc) return rc;
  }
  return LCQ_OK;
}

extern "C" int lcq_clip_apply(const void* x, int dtype, int64_t rows, int64_t cols,
                              int64_t group, const void* cmax, const void* cmin, void* out,
                              void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(rows > 0 && cols > 0 && group > 0 && cols % group == 0 && group % 8 == 0,
              "bad shape / group");
  hipStream_t st = as_stream(stream);
  const unsigned grid = stream_grid(rows * cols / 8, 256);
  switch (dtype) {
    case LCQ_BF16: hipLaunchKernelGGL((k_clip_apply<LCQ_BF16>), grid, 256, 0, st, x, rows, cols, group, cmax, cmin, out); break;
    case LCQ_F16: hipLaunchKernelGGL((k_clip_apply<LCQ_F16>), grid, 256, 0, st, x, rows, cols, group, cmax, cmin, out); break;
    default: hipLaunchKernelGGL((k_clip_apply<LCQ_F32>), grid, 256, 0, st, x, rows, cols, group, cmax, cmin, out);
  }
  return check_launch("lcq_clip_apply");
}

// get_clip_factor (auto_clip.py:213-256): one wave per group -> the group's min / max
// (get_minmax_range of the reshaped weight), then the logit of the bound ratios in DT.
template <int DT>
__global__ void __launch_bounds__(256) k_clip_factors(const uint16_t* __restrict__ x,
                                                     int64_t ng, int64_t group,
                                                     const uint16_t* __restrict__ cmax,
                                                     const uint16_t* __restrict__ cmin,
                                                     int clip_sym, uint16_t* __restrict__ up,
                                                     uint16_t* __restrict__ low) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= ng) return;
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t k = (int64_t)lane * 8; k < group; k += 64 * 8) {
    float v[8];
    ld8<DT>(x, g * group + k, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mx = fmaxf(mx, v[j]);
      mn = fminf(mn, v[j]);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    mn = fminf(mn, __shfl_xor(mn, m, 64));
  }
  if (lane != 0) return;
  const float bmax = ld1<DT>(cmax, g);
  if (clip_sym) {
    const float am = fmaxf(fmaxf(fabsf(mx), fabsf(mn)), dtr<DT>(1e-5f));
    st1<DT>(up, g, logit_ct<DT>(dtr<DT>(bmax / am)));
  } else {
    st1<DT>(up, g, logit_ct<DT>(dtr<DT>(bmax / mx)));
    st1<DT>(low, g, logit_ct<DT>(dtr<DT>(ld1<DT>(cmin, g) / mn)));
  }
}

extern "C" int lcq_clip_factors(const void* x, int dtype, int64_t rows, int64_t cols,
                                int64_t group, const void* cmax, const void* cmin, int clip_sym,
                                void* up_out, void* low_out, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "clip factors: bf16 / fp16");
  LCQ_REQUIRE(rows > 0 && cols > 0 && group > 0 && cols % group == 0 && group % 8 == 0,
              "group must divide cols and be a multiple of 8");
  LCQ_REQUIRE(x && cmax && up_out && (clip_sym || (cmin && low_out)), "null pointers");
  const int64_t ng = rows * cols / group;
  const dim3 grid((unsigned)((ng + 3) / 4));
  hipStream_t st = as_stream(stream);
  auto* xp = reinterpret_cast<const uint16_t*>(x);
  auto* mxp = reinterpret_cast<const uint16_t*>(cmax);
  auto* mnp = reinterpret_cast<const uint16_t*>(cmin);
  auto* up = reinterpret_cast<uint16_t*>(up_out);
  auto* lo = reinterpret_cast<uint16_t*>(low_out);
  if (dtype == LCQ_BF16)
    hipLaunchKernelGGL(k_clip_factors<LCQ_BF16>, grid, 256, 0, st, xp, ng, group, mxp, mnp,
                       clip_sym, up, lo);
  else
    hipLaunchKernelGGL(k_clip_factors<LCQ_F16>, grid, 256, 0, st, xp, ng, group, mxp, mnp,
                       clip_sym, up, lo);
  return check_launch("lcq_clip_factors");
}

// ----------------------------------------------------------------------------------------
// auto_clip search for per_channel weights (group = the whole row, auto_clip.py:96-99; the
// w8a8 vLLM / SGLang AWQ configs, awq_w8a8.yml). The per-group kernel's lane-pair-per-row
// layout cannot hold an IC-long row, so:
//  * k_clip_pc_stats: one wave per row -> org max / min and every shrink step's clamp bounds
//    and min/max qparams (the reference's fake_quant_weight_dynamic of the clamped row).
//  * k_auto_clip_pc: a workgroup = 256 rows (lane = row) x PC_TT sampled tokens (16; 8 for
//    fp16 asym), k walked in
//    PC_KC-wide chunks whose x / fake-quantized x tiles sit transposed in LDS (wave-uniform
//    broadcast reads); each k regenerates the 10 candidate weights in registers (Markstein
//    quotient, as the quant kernels) and accumulates the DT-rounded products of the original
//    output (x) and of every step (qx, = x for weight-only) in fp32. Partial squared-error
//    sums per token tile go to a workspace [ntt][nsteps][oc].
//  * k_clip_pc_pick: fixed-order sum of the tiles, DT mean, first strict minimum.
// Products are rounded to DT exactly as the reference's materialised broadcast product; the
// IC-long fp32 sum runs in k order, not torch-CPU's vectorised cascade, so a sum can round
// to a neighbouring DT value -> parity tier T2 (tests/test_awq_gpu.py: bounds equal on
// >= 98 % of rows, chosen errors within a few DT ulps).
// ----------------------------------------------------------------------------------------
constexpr int PC_TT_BF16 = 16;  // sampled tokens per workgroup (bf16: no VGPR spill)
constexpr int PC_TT_MIN = 8;    // fp16 asym (the software RNE needs registers): 8 tokens
constexpr int PC_KC = 128;      // k per LDS chunk
constexpr int PC_NS = 10;       // shrink steps (max_shrink 0.5 x n_grid 20)
constexpr int PC_QP = 5;        // per step: smin, smax, s, 1/s, z

// FQ (float-quant weights, FloatQuantizer use_qtorch, quant.py:545-553 / 1061-1080):
//   0 integer; 1 FP8 per_channel: s = rnd_DT(max(|cmax|, |cmin|).clamp(1e-5) / qmax) per row;
//   2 FP8 per_tensor: the clamped row's max(|cmax|, |cmin|) is left in slot 2 for
//     k_clip_pc_tensor_qp, which forms the scale of the whole 256 (or 64)-row batch the
//     reference fake-quantizes at once (auto_clip.py:108-114, 161-163).
//   3 integer, clip_version v2 (auto_clip.py:258-267): no clamp of the weight; the step's
//     bounds become logit factors of the row's own min / max and the qparams come from
//     get_learnable_range of the unclamped row (slots 0 / 1 = -inf / +inf: fq_pc's clamp is
//     the identity).
template <int DT, int FQ>
__global__ void __launch_bounds__(256) k_clip_pc_stats(const uint16_t* __restrict__ w,
                                                      int64_t oc, int64_t ic, int nsteps,
                                                      const float* __restrict__ factors,
                                                      float qmin, float qmax, int sym,
                                                      int clip_sym, float* __restrict__ qp,
                                                      float* __restrict__ orgmm) {
  const int lane = threadIdx.x & 63;
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= oc) return;
  float mx = -INFINITY, mn = INFINITY, am = 0.f;
  for (int64_t k = (int64_t)lane * 8; k < ic; k += 64 * 8) {
    float v[8];
    ld8<DT>(w, o * ic + k, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mx = fmaxf(mx, v[j]);
      mn = fminf(mn, v[j]);
      am = fmaxf(am, fabsf(v[j]));
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    mn = fminf(mn, __shfl_xor(mn, m, 64));
    am = fmaxf(am, __shfl_xor(am, m, 64));
  }
  const float org_max = clip_sym ? am : mx, org_min = mn;
  if (lane == 0) {
    orgmm[2 * o] = org_max;
    orgmm[2 * o + 1] = org_min;
  }
  if (lane < nsteps) {
    const float f = factors[lane];
    const float smax = dtr<DT>(org_max * f);
    const float smin = clip_sym ? -smax : dtr<DT>(org_min * f);
    const float cmn = fminf(fmaxf(mn, smin), smax), cmx = fminf(fmaxf(mx, smin), smax);
    float qs, qz;
    if constexpr (FQ == 0) {
      qparams_ct<DT>(cmn, cmx, qmin, qmax, sym, qs, qz);
    } else if constexpr (FQ == 3) {
      const float low = logit_ct<DT>(dtr<DT>(smin / org_min));  // logit(min_val / org_min)
      const float up = logit_ct<DT>(dtr<DT>(smax / org_max));
      float lmn = mn, lmx = mx;  // get_learnable_range(w, ...): the unclamped row's range
      learnable_range<DT>(lmn, lmx, up, low, true, sym);
      qparams_ct<DT>(lmn, lmx, qmin, qmax, sym, qs, qz);
    } else {
      const float am = fmaxf(fmaxf(fabsf(cmx), fabsf(cmn)), dtr<DT>(1e-5f));  // .clamp(1e-5)
      qs = FQ == 1 ? dtr<DT>(am / qmax) : am;
      qz = 0.f;
    }
    float* d = qp + ((int64_t)o * PC_NS + lane) * PC_QP;
    d[0] = FQ == 3 ? -INFINITY : smin;
    d[1] = FQ == 3 ? INFINITY : smax;
    d[2] = qs;
    d[3] = 1.0f / qs;
    d[4] = qz;
  }
}

// fake_quant of one clamped weight with step qparams (the per-group kernel's sequence, with
// the quotient from RN(1/s): |v / s| <= qmax-ish, so it is normal or rounds to zero either way)
template <int DT, bool SYM>
__device__ __forceinline__ float fq_pc(float v, float smin, float smax, float qs, float rs,
                                       float qz, float qmin, float qmax) {
  v = fminf(fmaxf(v, smin), smax);
  float tq = rintf(dtr<DT>(div_mk(v, qs, rs)));
  if constexpr (!SYM) tq = dtr<DT>(tq + qz);
  tq = fminf(fmaxf(tq, qmin), qmax);
  return dtr<DT>((SYM ? tq : dtr<DT>(tq - qz)) * qs);
}

// FP8 per_tensor: every step's scale over the rows of one reference batch (get_minmax_range
// of the whole clamped [rows, 1, 1, ic] batch -> 0-dim DT values; their clamp stays DT; the
// division by the 0-dim fp32 qmax promotes to fp32, so the batch scale is fp32).
__global__ void __launch_bounds__(256) k_clip_pc_tensor_qp(float* __restrict__ qp, int64_t oc,
                                                          int nsteps, int batch, float qmax) {
  __shared__ float red[4];
  const int64_t o = (int64_t)blockIdx.x * batch + threadIdx.x;
  const bool live = threadIdx.x < batch && o < oc;
  for (int i = 0; i < nsteps; ++i) {
    float am = live ? qp[((int64_t)o * PC_NS + i) * PC_QP + 2] : 0.f;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) am = fmaxf(am, __shfl_xor(am, m, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
    __syncthreads();
    const float s = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) / qmax;
    __syncthreads();
    if (live) {
      float* d = qp + ((int64_t)o * PC_NS + i) * PC_QP;
      d[2] = s;
      d[3] = 1.0f / s;
    }
  }
}

// FloatQuantizer fake quant of one clamped weight (quant.py:1061-1080 through
// fake_quant_weight_dynamic): DT quotient (a per-tensor fp32 scale is a CPU scalar to torch:
// full precision), `+ zeros`, float_quantize (saturating native cast), fp32 (q - 0) * s, DT.
template <int DT, int FMT>
__device__ __forceinline__ float fq_pc_fp8(float v, float smin, float smax, float qs) {
  v = fminf(fmaxf(v, smin), smax);
  const float t = dtr<DT>(dtr<DT>(v / qs) + 0.0f);
  return dtr<DT>(fp8_round<FMT>(t) * qs);
}

template <int DT, bool SYM, int PC_TT, int FMT = 0>
__global__ void __launch_bounds__(256, 1) k_auto_clip_pc(const uint16_t* __restrict__ w,
                                                        const uint16_t* __restrict__ x,
                                                        const uint16_t* __restrict__ qx,
                                                        int64_t oc, int64_t ic, int T,
                                                        int nsteps, const float* __restrict__ qp,
                                                        float qmin, float qmax,
                                                        float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float xs[PC_KC * PC_TT];   // [k][t], 8 KB
  __shared__ __attribute__((aligned(16))) float qxs[PC_KC * PC_TT];  // 8 KB
  const int tid = threadIdx.x;
  const int64_t o = (int64_t)blockIdx.x * 256 + tid;
  const bool live = o < oc;
  const int t0 = blockIdx.y * PC_TT;
  const int tn = min(PC_TT, T - t0);
  const uint16_t* wrow = w + (live ? o : 0) * ic;
  float q[PC_NS][PC_QP];
#pragma unroll
  for (int i = 0; i < PC_NS; ++i)
#pragma unroll
    for (int j = 0; j < PC_QP; ++j)
      q[i][j] = (live && i < nsteps) ? qp[((int64_t)o * PC_NS + i) * PC_QP + j] : 1.f;
  v2f org[PC_TT / 2], cur[PC_NS][PC_TT / 2];
#pragma unroll
  for (int t = 0; t < PC_TT / 2; ++t) {
    org[t] = v2f{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PC_NS; ++i) cur[i][t] = v2f{0.f, 0.f};
  }
  const uint16_t* qsrc = qx ? qx : x;
  for (int64_t k0 = 0; k0 < ic; k0 += PC_KC) {
    __syncthreads();
    // stage PC_TT tokens x PC_KC k of x and qx transposed: thread -> (token, 8 k); 256
    // threads cover 16 tokens, so with PC_TT 8 the upper half idles
    static_assert(PC_TT * (PC_KC / 8) <= 256, "staging covers at most 256 threads");
    if (tid < PC_TT * (PC_KC / 8)) {
      const int t = tid / (PC_KC / 8), c8 = (tid % (PC_KC / 8)) * 8;
      float a[8], b[8];
      if (t < tn) {
        const uint4 v = *reinterpret_cast<const uint4*>(x + (int64_t)(t0 + t) * ic + k0 + c8);
        const uint4 u = *reinterpret_cast<const uint4*>(qsrc + (int64_t)(t0 + t) * ic + k0 + c8);
        widen4<DT>(make_uint2(v.x, v.y), a);
        widen4<DT>(make_uint2(v.z, v.w), a + 4);
        widen4<DT>(make_uint2(u.x, u.y), b);
        widen4<DT>(make_uint2(u.z, u.w), b + 4);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = b[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xs[(c8 + j) * PC_TT + t] = a[j];
        qxs[(c8 + j) * PC_TT + t] = b[j];
      }
    }
    __syncthreads();
    for (int kk = 0; kk < PC_KC; kk += 8) {
      float wv[8];
      widen4<DT>(*reinterpret_cast<const uint2*>(wrow + k0 + kk), wv);
      widen4<DT>(*reinterpret_cast<const uint2*>(wrow + k0 + kk + 4), wv + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* xk = &xs[(kk + j) * PC_TT];
        const float* qk = &qxs[(kk + j) * PC_TT];
        const v2f wp = {wv[j], wv[j]};
#pragma unroll
        for (int t = 0; t < PC_TT / 4; ++t) {
          const float4 xv = *reinterpret_cast<const float4*>(xk + 4 * t);
          org[2 * t] += dtr2<DT>(v2f{xv.x, xv.y} * wp);
          org[2 * t + 1] += dtr2<DT>(v2f{xv.z, xv.w} * wp);
        }
        float qv[PC_TT];
#pragma unroll
        for (int t = 0; t < PC_TT / 4; ++t) {
          const float4 v = *reinterpret_cast<const float4*>(qk + 4 * t);
          qv[4 * t] = v.x; qv[4 * t + 1] = v.y; qv[4 * t + 2] = v.z; qv[4 * t + 3] = v.w;
        }
#pragma unroll
        for (int i = 0; i < PC_NS; ++i) {
          float c;
          if constexpr (FMT == 0)
            c = fq_pc<DT, SYM>(wv[j], q[i][0], q[i][1], q[i][2], q[i][3], q[i][4], qmin, qmax);
          else
            c = fq_pc_fp8<DT, FMT>(wv[j], q[i][0], q[i][1], q[i][2]);
          const v2f cp = {c, c};
#pragma unroll
          for (int t = 0; t < PC_TT / 2; ++t)
            cur[i][t] += dtr2<DT>(v2f{qv[2 * t], qv[2 * t + 1]} * cp);
        }
      }
    }
  }
  if (!live) return;
  float og[PC_TT];
#pragma unroll
  for (int t = 0; t < PC_TT / 2; ++t) {
    og[2 * t] = dtr<DT>(org[t].x);
    og[2 * t + 1] = dtr<DT>(org[t].y);
  }
  // static indices only (a dynamic one would move the accumulators to scratch)
#pragma unroll
  for (int i = 0; i < PC_NS; ++i) {
    float e = 0.f;
#pragma unroll
    for (int t = 0; t < PC_TT; ++t) {
      const float cu = dtr<DT>((t & 1) ? cur[i][t >> 1].y : cur[i][t >> 1].x);
      const float dd = dtr<DT>(cu - og[t]);
      if (t < tn) e += dtr<DT>(dd * dd);
    }
    if (i < nsteps) part[((int64_t)blockIdx.y * nsteps + i) * oc + o] = e;
  }
}

template <int DT>
__global__ void __launch_bounds__(256) k_clip_pc_pick(const float* __restrict__ part, int ntt,
                                                     int64_t oc, int T, int nsteps,
                                                     const float* __restrict__ factors,
                                                     int clip_sym,
                                                     const float* __restrict__ orgmm,
                                                     uint16_t* best_max, uint16_t* best_min) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= oc) return;
  const float org_max = orgmm[2 * o], org_min = orgmm[2 * o + 1];
  float bmax = org_max, bmin = org_min, best = dtr<DT>(1e9f);
  for (int i = 0; i < nsteps; ++i) {
    float e = 0.f;
    for (int y = 0; y < ntt; ++y) e += part[((int64_t)y * nsteps + i) * oc + o];
    const float em = dtr<DT>(e / (float)T);
    if (em < best) {
      best = em;
      bmax = dtr<DT>(org_max * factors[i]);
      bmin = clip_sym ? -bmax : dtr<DT>(org_min * factors[i]);
    }
  }
  if constexpr (DT == LCQ_BF16) {
    best_max[o] = (uint16_t)(__float_as_uint(bmax) >> 16);
    best_min[o] = (uint16_t)(__float_as_uint(bmin) >> 16);
  } else {
    best_max[o] = __builtin_bit_cast(uint16_t, (_Float16)bmax);
    best_min[o] = __builtin_bit_cast(uint16_t, (_Float16)bmin);
  }
}

extern "C" int64_t lcq_auto_clip_pc_workspace_bytes(int64_t oc, int64_t T, int nsteps) {
  const int64_t ntt = (T + PC_TT_MIN - 1) / PC_TT_MIN;  // the larger tile count (fp16)
  return oc * PC_NS * PC_QP * 4 + oc * 2 * 4 + ntt * nsteps * oc * 4;
}

template <int DT>
static void launch_clip_pc(const void* w, const void* x, const void* qx, int64_t oc, int64_t ic,
                           int64_t T, int nsteps, const void* factors, int qmin, int qmax,
                           int sym, int clip_sym, int fmt, int tensor_batch, int version,
                           char* ws, void* best_max, void* best_min, hipStream_t st) {
  float* qp = reinterpret_cast<float*>(ws);
  float* orgmm = qp + oc * PC_NS * PC_QP;
  float* part = orgmm + oc * 2;
  // fp16: asym spills nothing at 8 tokens (200 spilled VGPRs at 16), sym spills less at 16
  const int TT = (DT == LCQ_BF16 || sym || fmt != 0) ? PC_TT_BF16 : PC_TT_MIN;
  const int ntt = (int)((T + TT - 1) / TT);
  const auto* wp = reinterpret_cast<const uint16_t*>(w);
  const auto* fp = reinterpret_cast<const float*>(factors);
  const dim3 gs((unsigned)((oc + 3) / 4));
  if (fmt == 0 && version == 2)
    hipLaunchKernelGGL((k_clip_pc_stats<DT, 3>), gs, 256, 0, st, wp, oc, ic, nsteps, fp,
                       (float)qmin, (float)qmax, sym, clip_sym, qp, orgmm);
  else if (fmt == 0)
    hipLaunchKernelGGL((k_clip_pc_stats<DT, 0>), gs, 256, 0, st, wp, oc, ic, nsteps, fp,
                       (float)qmin, (float)qmax, sym, clip_sym, qp, orgmm);
  else if (tensor_batch == 0)
    hipLaunchKernelGGL((k_clip_pc_stats<DT, 1>), gs, 256, 0, st, wp, oc, ic, nsteps, fp,
                       (float)qmin, (float)qmax, sym, clip_sym, qp, orgmm);
  else {
    hipLaunchKernelGGL((k_clip_pc_stats<DT, 2>), gs, 256, 0, st, wp, oc, ic, nsteps, fp,
                       (float)qmin, (float)qmax, sym, clip_sym, qp, orgmm);
    hipLaunchKernelGGL(k_clip_pc_tensor_qp, dim3((unsigned)((oc + tensor_batch - 1) / tensor_batch)),
                       256, 0, st, qp, oc, nsteps, tensor_batch, (float)qmax);
  }
  const dim3 g((unsigned)((oc + 255) / 256), (unsigned)ntt);
  auto k = fmt == LCQ_FP8E4M3 ? k_auto_clip_pc<DT, true, PC_TT_BF16, LCQ_FP8E4M3>
         : fmt == LCQ_FP8E5M2 ? k_auto_clip_pc<DT, true, PC_TT_BF16, LCQ_FP8E5M2>
         : sym ? k_auto_clip_pc<DT, true, PC_TT_BF16>
               : (DT == LCQ_BF16 ? k_auto_clip_pc<DT, false, PC_TT_BF16>
                                 : k_auto_clip_pc<DT, false, PC_TT_MIN>);
  hipLaunchKernelGGL(k, g, 256, 0, st, wp, reinterpret_cast<const uint16_t*>(x),
                     reinterpret_cast<const uint16_t*>(qx), oc, ic, (int)T, nsteps, qp,
                     (float)qmin, (float)qmax, part);
  hipLaunchKernelGGL(k_clip_pc_pick<DT>, dim3((unsigned)((oc + 255) / 256)), 256, 0, st, part,
                     ntt, oc, (int)T, nsteps, fp, clip_sym, orgmm,
                     reinterpret_cast<uint16_t*>(best_max), reinterpret_cast<uint16_t*>(best_min));
}

extern "C" int lcq_auto_clip_search_pc(const void* w, const void* x, const void* qx, int dtype,
                                       int64_t oc, int64_t ic, int64_t T, int nsteps,
                                       const void* factors, int qmin, int qmax, int sym,
                                       int clip_sym, int fmt, int tensor_batch, int version,
                                       void* workspace, int64_t ws_bytes, void* best_max,
                                       void* best_min, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "auto-clip: bf16 or fp16 model dtype");
  LCQ_REQUIRE(oc > 0 && ic > 0 && ic % PC_KC == 0, "per-channel auto-clip: ic % 128 == 0");
  LCQ_REQUIRE(T > 0 && nsteps >= 1 && nsteps <= PC_NS, "bad T / nsteps (<= 10)");
  LCQ_REQUIRE(fmt == 0 || fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2,
              "fmt must be 0 (integer) or an fp8 format");
  LCQ_REQUIRE(tensor_batch == 0 || (fmt != 0 && tensor_batch > 0 && tensor_batch <= 256),
              "tensor_batch (per-tensor fp8 scale rows) must be 1..256, fp8 only");
  LCQ_REQUIRE(version == 1 || (version == 2 && fmt == 0),
              "version must be 1, or 2 (learnable clip factors) for integer weights");
  if (fmt != 0) {  // FloatQuantizer: symmetric, qmax = finfo.max
    qmax = fmt == LCQ_FP8E4M3 ? 448 : 57344;
    qmin = -qmax;
    sym = 1;
  }
  LCQ_REQUIRE(qmax > qmin, "qmax <= qmin");
  LCQ_REQUIRE(workspace != nullptr &&
                  ws_bytes >= lcq_auto_clip_pc_workspace_bytes(oc, T, nsteps),
              "workspace smaller than lcq_auto_clip_pc_workspace_bytes");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  if (dtype == LCQ_BF16)
    launch_clip_pc<LCQ_BF16>(w, x, qx, oc, ic, T, nsteps, factors, qmin, qmax, sym, clip_sym,
                             fmt, tensor_batch, version, ws, best_max, best_min, st);
  else
    launch_clip_pc<LCQ_F16>(w, x, qx, oc, ic, T, nsteps, factors, qmin, qmax, sym, clip_sym,
                            fmt, tensor_batch, version, ws, best_max, best_min, st);
  return check_launch("lcq_auto_clip_search_pc");
}
