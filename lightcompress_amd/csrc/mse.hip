// MSE range search for weight qparams (calib_algo 'mse'; quant.py:145-203, get_mse_range) on
// gfx950: one wavefront per group row, the reference's shrink grid (p = 1 - i / grid for
// i < maxshrink * grid) evaluated on the fp32 copy of the row, |qdq(x) - x|^norm summed per
// candidate, strict improvements accepted (and, as in the reference, shrinking the base of the
// later candidates); then get_qparams (quant.py:545-559) on the final range, in fp32 like the
// reference (the search works on tensor.float()).
//
// Every op of the candidate's quant_dequant is the reference's fp32 op (IEEE division, rint,
// no contraction). The error sum of a candidate is taken in a fixed wave order and pow is the
// device powf (<= 1 ulp): the reference's vectorised powf (Sleef u10) and its SIMD-width
// dependent row sums make near-tie choices order dependent there too (parity tier T2).
#include <math.h>

#include "lcq_common.h"

namespace lcq {
namespace {

__device__ inline void qparams_f32_ref(float mn, float mx, float qmin, float qmax, int sym,
                                       float& s, float& z) {
  if (sym) {
    float am = fmaxf(fabsf(mx), fabsf(mn));
    am = am < 1e-5f ? 1e-5f : am;
    s = am / qmax;
    z = 0.f;
  } else {
    float r = mx - mn;
    r = r < 1e-5f ? 1e-5f : r;
    s = r / (qmax - qmin);
    const float t = rintf(mn / s);
    z = fminf(fmaxf(qmin - t, qmin), qmax);
  }
}

// rows groups of `group` contiguous elements; 4 waves per workgroup, one row per wave
template <int DT>
__global__ __launch_bounds__(256) void k_mse_range(const void* x, int64_t rows, int64_t group,
                                                   int sym, float qmin, float qmax, int nsteps,
                                                   float grid, float norm, float* out_min,
                                                   float* out_max, float* s_out,
                                                   float* z_out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;  // whole wave exits together
  const int64_t base = row * group;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t j = lane; j < group; j += 64) {
    const float v = ld1<DT>(x, base + j);
    mn = fminf(mn, v);
    mx = fmaxf(mx, v);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  // the reference's best_min_val / best_max_val are views of the running min / max, updated
  // in place: an accepted candidate becomes the base the later p's shrink
  float best = INFINITY;
  for (int i = 0; i < nsteps; ++i) {
    const float p = (float)(1.0 - (double)i / (double)grid);  // python double -> fp32 scalar
    const float xmn = p * mn, xmx = p * mx;
    float s, z;
    qparams_f32_ref(xmn, xmx, qmin, qmax, sym, s, z);
    float err = 0.f;
    for (int64_t j = lane; j < group; j += 64) {
      const float v = ld1<DT>(x, base + j);
      float q = rintf(v / s) + z;
      q = fminf(fmaxf(q, qmin), qmax);
      const float d = (q - z) * s - v;
      err += powf(fabsf(d), norm);
    }
    for (int o = 32; o >= 1; o >>= 1) err += __shfl_xor(err, o, 64);
    if (err < best) {  // tmp = err < best (strict)
      best = err;
      mn = xmn;
      mx = xmx;
    }
  }
  if (lane == 0) {
    out_min[row] = mn;
    out_max[row] = mx;
    float s, z;
    qparams_f32_ref(mn, mx, qmin, qmax, sym, s, z);
    s_out[row] = s;
    if (z_out) z_out[row] = z;
  }
}

}  // namespace
}  // namespace lcq

using namespace lcq;

extern "C" int lcq_mse_qparams(const void* x, int dtype, int64_t rows, int64_t group, int sym,
                               int qmin, int qmax, int nsteps, float grid, float norm,
                               void* range_min, void* range_max, void* scales, void* zeros,
                               void* stream) {
  LCQ_REQUIRE(dtype == LCQ_F32 || dtype == LCQ_F16 || dtype == LCQ_BF16, "bad dtype");
  LCQ_REQUIRE(rows > 0 && group > 0, "empty tensor");
  LCQ_REQUIRE(nsteps >= 1 && grid > 0.f, "bad shrink grid");
  LCQ_REQUIRE(qmax > qmin, "qmax must exceed qmin");
  LCQ_REQUIRE(range_min && range_max && scales && (sym || zeros), "null pointer");
  hipStream_t st = as_stream(stream);
  const dim3 g((unsigned)((rows + 3) / 4));
  float* mn = reinterpret_cast<float*>(range_min);
  float* mx = reinterpret_cast<float*>(range_max);
  float* s = reinterpret_cast<float*>(scales);
  float* z = sym ? nullptr : reinterpret_cast<float*>(zeros);
  switch (dtype) {
    case LCQ_BF16:
      k_mse_range<LCQ_BF16><<<g, 256, 0, st>>>(x, rows, group, sym, (float)qmin, (float)qmax,
                                              nsteps, grid, norm, mn, mx, s, z);
      break;
    case LCQ_F16:
      k_mse_range<LCQ_F16><<<g, 256, 0, st>>>(x, rows, group, sym, (float)qmin, (float)qmax,
                                             nsteps, grid, norm, mn, mx, s, z);
      break;
    default:
      k_mse_range<LCQ_F32><<<g, 256, 0, st>>>(x, rows, group, sym, (float)qmin, (float)qmax,
                                             nsteps, grid, norm, mn, mx, s, z);
  }
  return check_launch("lcq_mse_qparams");
}
