// AWQ scale search + auto-clip device kernels (gfx950).
//
// Reference: llmc/compression/quantization/awq.py and auto_clip.py. Every op rounds to the
// weight/activation dtype like the reference's torch-bf16 expressions:
//   get_act_scale      awq.py:74-85     mean_t |x|                        -> lcq_absmean_cols
//   get_scales (v2)    awq.py:87-108    s = x^r ; clamp 1e-4 ; s/sqrt(max*min) -> lcq_awq_scales
//   scaling_input / update_input_feat / scale_ln_fcs / scale_fc_fc
//                      base_blockwise_quantization.py:631-778, 880-897  -> lcq_scale_bcast
//   calculate_loss     awq.py:134-145   mean((org-out).float()^2)        -> lcq_sq_diff_mean
//   auto_clip_layer    auto_clip.py:83-191 (10-step shrink grid)          -> lcq_auto_clip_search
//   apply_clip (v1)    auto_clip.py:193-212                               -> lcq_clip_apply
#include "lcq_common.h"

namespace lcq {

// ----------------------------------------------------------------------------------------
// mean over rows of |x| per column: pass 1 writes fp32 partial sums for row slices,
// pass 2 sums the slices in fixed order (deterministic), divides by n, rounds to DT.
// ----------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) k_absmean_p1(const void* x, int64_t n, int64_t c,
                                                   int64_t rows_per_split, double* part) {
  const int64_t c8 = (int64_t)blockIdx.x * 256 + threadIdx.x;  // 8-column chunk
  if (c8 * 8 >= c) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t r1 = min(n, r0 + rows_per_split);
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = r0; r < r1; ++r) {
    float v[8];
    ld8<DT>(x, r * c + c8 * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (double)fabsf(v[j]);
  }
  double* p = part + (int64_t)blockIdx.y * c + c8 * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = acc[j];
}

template <int DT>
__global__ void __launch_bounds__(256) k_absmean_p2(const double* part, int splits, int64_t n,
                                                   int64_t c, void* out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= c) return;
  double s = 0.0;
  for (int i = 0; i < splits; ++i) s += part[(int64_t)i * c + j];
  // the reference's fp32 sum is an approximation of this (near-)exact sum; its bf16 mean is
  // the correctly rounded fp32(sum) / n (parity tier T3)
  st1<DT>(out, j, (float)s / (float)n);
}

// ----------------------------------------------------------------------------------------
// AWQ v2 scales for one ratio. s = round_dt(pow(x, r_dt)) where the exponent is first rounded
// to the tensor dtype and pow is correctly rounded (torch-CPU bf16 semantics, verified
// exhaustively over all positive bf16 inputs x 20 ratios); clamp(min=1e-4);
// s / sqrt(max(s)*min(s)) with each op rounded to DT. One workgroup.
// ----------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(1024) k_awq_scales(const void* xmean, int64_t c, float r,
                                                    void* out) {
  __shared__ float red[2][16];
  const float lo = rnd<DT>(1e-4f);
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t j = threadIdx.x; j < c; j += blockDim.x) {
    const float xv = ld1<DT>(xmean, j);
    float s = rnd<DT>((float)pow((double)xv, (double)r));
    s = fmaxf(s, lo);
    mx = fmaxf(mx, s);
    mn = fminf(mn, s);
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
  for (int64_t j = threadIdx.x; j < c; j += blockDim.x) {
    const float xv = ld1<DT>(xmean, j);
    float s = rnd<DT>((float)pow((double)xv, (double)r));
    s = fmaxf(s, lo);
    st1<DT>(out, j, s / d);
  }
}

// ----------------------------------------------------------------------------------------
// out[r, c] = round_dt(x[r, c] (op) s[axis index]), op 0 = mul, 1 = div; axis 0 = per column
// (s has cols entries), 1 = per row (s has rows entries). In place allowed.
// ----------------------------------------------------------------------------------------
template <int DT, int OP, int AXIS>
__global__ void __launch_bounds__(256) k_scale_bcast(const void* x, int64_t rows, int64_t cols,
                                                    const void* s, void* out) {
  const int64_t n8 = rows * cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8;
    float v[8], sv[8];
    ld8<DT>(x, e0, v);
    if constexpr (AXIS == 0) {
      ld8<DT>(s, e0 % cols, sv);
    } else {
      const float r = ld1<DT>(s, e0 / cols);
#pragma unroll
      for (int j = 0; j < 8; ++j) sv[j] = r;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (OP == 0) ? v[j] * sv[j] : v[j] / sv[j];
    st8<DT>(out, e0, v);
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

__global__ void k_sqdiff_p2(const double* part, int nparts, int64_t n, float* out, int slot) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nparts; ++i) s += part[i];
  out[slot] = (float)s / (float)n;
}

// ----------------------------------------------------------------------------------------
// auto_clip search (auto_clip.py:83-191), one wave = 64 output rows x one 128-wide group.
// For every (row o, group g):
//   org[t]  = bf16( sum_k bf16(x[t,g,k] * w[o,g,k]) )          (t over the T sampled tokens)
//   step i: max_i = bf16(org_max * (1 - i/n_grid)), min_i = -max_i | bf16(org_min * (..))
//           q = fake_quant(clamp(w, min_i, max_i)) (bf16, per-group min/max qparams)
//           cur[t] = bf16( sum_k bf16(x * q) );  err_i = bf16(mean_t bf16(bf16(cur-org)^2))
//   keep the first strictly smaller err (min_errs starts at bf16(1e9)).
// The per-product bf16 rounding of the reference's materialised broadcast product rules out
// MFMA (which accumulates exact products), so this is a VALU kernel: weights stay in VGPRs,
// token tiles of x are staged in LDS and read as wave-uniform broadcasts. Sums over k use 16
// partial accumulators + a halving tree (torch-CPU's vectorised reduction order).
// ----------------------------------------------------------------------------------------
constexpr int CG = 128;  // group size
constexpr int CT = 32;   // tokens per LDS tile
constexpr int CMAXSTEPS = 16;

__device__ __forceinline__ float bf(uint32_t u, int hi) {
  return __uint_as_float(hi ? (u & 0xffff0000u) : (u << 16));
}

__device__ __forceinline__ float bf16r(float f) {  // finite-only RNE
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return __uint_as_float(u & 0xffff0000u);
}

// dot of one LDS token row (64 packed dwords) with 64 packed weight dwords
__device__ __forceinline__ float dot_bf16(const uint32_t* xr, const uint32_t (&wp)[64]) {
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
  for (int c = 0; c < 128; c += 16) {
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const uint32_t xv = xr[(c + j) >> 1];
      const uint32_t wv = wp[(c + j) >> 1];
      acc[j] += bf16r(bf(xv, 0) * bf(wv, 0));
      acc[j + 1] += bf16r(bf(xv, 1) * bf(wv, 1));
    }
  }
#pragma unroll
  for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
    for (int j = 0; j < h; ++j) acc[j] += acc[j + h];
  return bf16r(acc[0]);
}

__global__ void __launch_bounds__(64)
    k_auto_clip(const uint16_t* __restrict__ w, const uint16_t* __restrict__ x, int64_t oc,
                int64_t ic, int T, int nsteps, const float* __restrict__ factors, float qmin,
                float qmax, int sym, int clip_sym, uint16_t* best_max, uint16_t* best_min) {
  __shared__ __attribute__((aligned(16))) uint32_t xs[CT * 64];
  const int lane = threadIdx.x;
  const int64_t o = (int64_t)blockIdx.x * 64 + lane;
  const int64_t g = blockIdx.y;
  const int64_t ng = ic / CG;
  const bool live = o < oc;
  uint32_t wp[64];
  {
    const uint4* src = reinterpret_cast<const uint4*>(w + (live ? o : 0) * ic + g * CG);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint4 v = src[i];
      wp[4 * i] = v.x; wp[4 * i + 1] = v.y; wp[4 * i + 2] = v.z; wp[4 * i + 3] = v.w;
    }
  }
  float mxs = -INFINITY, mn = INFINITY, amax = 0.f;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float v = bf(wp[i], h);
      mxs = fmaxf(mxs, v);
      mn = fminf(mn, v);
      amax = fmaxf(amax, fabsf(v));
    }
  }
  const float org_max = clip_sym ? amax : mxs;
  const float org_min = mn;
  float smax[CMAXSTEPS], smin[CMAXSTEPS], qs[CMAXSTEPS], qz[CMAXSTEPS], err[CMAXSTEPS];
#pragma unroll
  for (int s = 0; s < CMAXSTEPS; ++s) {
    if (s < nsteps) {
      const float f = factors[s];
      smax[s] = bf16r(org_max * f);
      smin[s] = clip_sym ? -smax[s] : bf16r(org_min * f);
      // min/max of clamp(w, min, max) = clamp of the group's min/max (clamp is monotone)
      const float cmn = fminf(fmaxf(mn, smin[s]), smax[s]);
      const float cmx = fminf(fmaxf(mxs, smin[s]), smax[s]);
      qparams_ct<LCQ_BF16>(cmn, cmx, qmin, qmax, sym, qs[s], qz[s]);
    }
    err[s] = 0.f;
  }

  for (int t0 = 0; t0 < T; t0 += CT) {
    __syncthreads();
    // stage CT token rows of this group (CT x 256 B) into LDS: 8 x 16 B per lane
#pragma unroll
    for (int i = 0; i < (CT * 16) / 64; ++i) {
      const int idx = i * 64 + lane;
      const int row = idx >> 4, ch = idx & 15;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (t0 + row < T)
        v = *reinterpret_cast<const uint4*>(x + (int64_t)(t0 + row) * ic + g * CG + ch * 8);
      *reinterpret_cast<uint4*>(&xs[row * 64 + ch * 4]) = v;
    }
    __syncthreads();
    const int tn = min(CT, T - t0);
    float org[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) org[t] = (t < tn) ? dot_bf16(&xs[t * 64], wp) : 0.f;
    for (int s = 0; s < nsteps; ++s) {
      uint32_t qp[64];
      const float lo = smin[0], hi = smax[0];
      float a_lo = lo, a_hi = hi, a_s = qs[0], a_z = qz[0];
#pragma unroll
      for (int k = 1; k < CMAXSTEPS; ++k)
        if (k == s) {
          a_lo = smin[k]; a_hi = smax[k]; a_s = qs[k]; a_z = qz[k];
        }
      (void)lo; (void)hi;
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        float q2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float v = fminf(fmaxf(bf(wp[i], h), a_lo), a_hi);
          float tq = rintf(bf16r(v / a_s));
          tq = bf16r(tq + a_z);
          tq = fminf(fmaxf(tq, qmin), qmax);
          q2[h] = bf16r(bf16r(tq - a_z) * a_s);
        }
        qp[i] = (__float_as_uint(q2[0]) >> 16) | (__float_as_uint(q2[1]) & 0xffff0000u);
      }
      // running fp32 sum over t in token order (sum of the bf16 squares, then / T)
      float e = err[0];
#pragma unroll
      for (int k = 1; k < CMAXSTEPS; ++k)
        if (k == s) e = err[k];
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        if (t < tn) {
          const float cur = dot_bf16(&xs[t * 64], qp);
          const float d = bf16r(cur - org[t]);
          e += bf16r(d * d);
        }
      }
#pragma unroll
      for (int k = 0; k < CMAXSTEPS; ++k)
        if (k == s) err[k] = e;
    }
  }
  if (!live) return;
  float bmax = org_max, bmin = org_min, best = bf16r(1e9f);
#pragma unroll
  for (int s = 0; s < CMAXSTEPS; ++s) {
    if (s < nsteps) {
      const float em = bf16r(err[s] / (float)T);
      if (em < best) {
        best = em;
        bmax = smax[s];
        bmin = smin[s];
      }
    }
  }
  best_max[o * ng + g] = (uint16_t)(__float_as_uint(bmax) >> 16);
  best_min[o * ng + g] = (uint16_t)(__float_as_uint(bmin) >> 16);
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

extern "C" int lcq_absmean_cols(const void* x, int dtype, int64_t n, int64_t c, void* out,
                                void* workspace, int splits, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(n > 0 && c > 0 && c % 8 == 0, "c must be a positive multiple of 8");
  LCQ_REQUIRE(splits >= 1 && workspace, "workspace of splits*c fp64 required");
  hipStream_t st = as_stream(stream);
  const int64_t rps = (n + splits - 1) / splits;
  dim3 g1((unsigned)((c / 8 + 255) / 256), (unsigned)splits);
  double* part = reinterpret_cast<double*>(workspace);
  switch (dtype) {
    case LCQ_BF16:
      hipLaunchKernelGGL((k_absmean_p1<LCQ_BF16>), g1, 256, 0, st, x, n, c, rps, part);
      hipLaunchKernelGGL((k_absmean_p2<LCQ_BF16>), dim3((unsigned)((c + 255) / 256)), 256, 0, st,
                         part, splits, n, c, out);
      break;
    case LCQ_F16:
      hipLaunchKernelGGL((k_absmean_p1<LCQ_F16>), g1, 256, 0, st, x, n, c, rps, part);
      hipLaunchKernelGGL((k_absmean_p2<LCQ_F16>), dim3((unsigned)((c + 255) / 256)), 256, 0, st,
                         part, splits, n, c, out);
      break;
    default:
      hipLaunchKernelGGL((k_absmean_p1<LCQ_F32>), g1, 256, 0, st, x, n, c, rps, part);
      hipLaunchKernelGGL((k_absmean_p2<LCQ_F32>), dim3((unsigned)((c + 255) / 256)), 256, 0, st,
                         part, splits, n, c, out);
  }
  return check_launch("lcq_absmean_cols");
}

extern "C" int lcq_awq_scales(const void* xmean, int dtype, int64_t c, float ratio_dt,
                              void* out, void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16 || dtype == LCQ_F32, "bad dtype");
  LCQ_REQUIRE(c > 0, "empty");
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case LCQ_BF16: hipLaunchKernelGGL((k_awq_scales<LCQ_BF16>), 1, 1024, 0, st, xmean, c, ratio_dt, out); break;
    case LCQ_F16: hipLaunchKernelGGL((k_awq_scales<LCQ_F16>), 1, 1024, 0, st, xmean, c, ratio_dt, out); break;
    default: hipLaunchKernelGGL((k_awq_scales<LCQ_F32>), 1, 1024, 0, st, xmean, c, ratio_dt, out);
  }
  return check_launch("lcq_awq_scales");
}

template <int DT>
static void launch_scale(const void* x, int64_t rows, int64_t cols, const void* s, int op,
                         int axis, void* out, hipStream_t st) {
  const unsigned grid = stream_grid(rows * cols / 8, 256);
  if (op == 0 && axis == 0) hipLaunchKernelGGL((k_scale_bcast<DT, 0, 0>), grid, 256, 0, st, x, rows, cols, s, out);
  if (op == 0 && axis == 1) hipLaunchKernelGGL((k_scale_bcast<DT, 0, 1>), grid, 256, 0, st, x, rows, cols, s, out);
  if (op == 1 && axis == 0) hipLaunchKernelGGL((k_scale_bcast<DT, 1, 0>), grid, 256, 0, st, x, rows, cols, s, out);
  if (op == 1 && axis == 1) hipLaunchKernelGGL((k_scale_bcast<DT, 1, 1>), grid, 256, 0, st, x, rows, cols, s, out);
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

extern "C" int lcq_auto_clip_search(const void* w, const void* x, int64_t oc, int64_t ic,
                                    int64_t T, int group, int nsteps, const void* factors,
                                    int qmin, int qmax, int sym, int clip_sym, void* best_max,
                                    void* best_min, void* stream) {
  LCQ_REQUIRE(group == CG, "auto-clip kernel supports group_size 128");
  LCQ_REQUIRE(oc > 0 && ic > 0 && ic % CG == 0, "ic must be a multiple of 128");
  LCQ_REQUIRE(T > 0 && nsteps >= 1 && nsteps <= CMAXSTEPS, "bad T / nsteps (<= 16)");
  LCQ_REQUIRE(qmax > qmin, "qmax <= qmin");
  dim3 grid((unsigned)((oc + 63) / 64), (unsigned)(ic / CG));
  hipLaunchKernelGGL(k_auto_clip, grid, 64, 0, as_stream(stream),
                     reinterpret_cast<const uint16_t*>(w), reinterpret_cast<const uint16_t*>(x),
                     oc, ic, (int)T, nsteps, reinterpret_cast<const float*>(factors),
                     (float)qmin, (float)qmax, sym, clip_sym,
                     reinterpret_cast<uint16_t*>(best_max), reinterpret_cast<uint16_t*>(best_min));
  return check_launch("lcq_auto_clip_search");
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
