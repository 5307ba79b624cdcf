// HQQ half-quadratic qparam search and round_zp=False qparams on gfx950.
//
// Reference: llmc/compression/quantization/quant.py
//   get_qparams :545-559 (round_zp False: zeros = qmin - min_val / scales, no round / clamp)
//   get_hqq_qparams :680-689 (tensor.float(), minmax qparams, optimize_weights_proximal)
//   optimize_weights_proximal :588-610 (and the HQQ algorithm's own copy, hqq.py:36-61)
//   shrink_op :92-101 (lp_norm 1: soft threshold; else sign(x) relu(|x| - |x|^(p-1) / beta),
//   with the quantizer's own beta, not the per-iteration current_beta)
//
// One proximal iteration over W [ng, gs] (fp32, s_inv = 1 / scales, z per group):
//   W_q = clamp(round(W * s_inv + z), qmin, qmax); W_r = (W_q - z) / s_inv
//   W_e = shrink(W - W_r); z <- mean_g(W_q - (W - W_e) * s_inv); err = mean(|W - W_r|)
//   stop when err >= best (the z of that iteration is kept, as in the reference loop).
// Design: each group is one team of L lanes (8 elements per lane per pass) -- a single HBM
// pass per iteration (4 B read per element, ng * 8 B written), the per-group error sums go to
// fp64 partials and a one-workgroup check kernel turns them into the global mean, compares it
// with the running best and raises a device stop flag. The host enqueues `iters` (step,
// check) pairs without synchronising; steps after the stop return at once.
#include "lcq_common.h"

namespace lcq {

struct HqqState {
  float best;
  int stop;
  int iters_run;
  int pad;
};

template <int CT>
__global__ void __launch_bounds__(256) k_minmax_qparams(const void* x, int64_t ng, int64_t gs,
                                                        float qmin, float qmax, int sym,
                                                        int round_zp, void* s_out, void* z_out) {
  // one wave per group: lanes stride over the group 8 elements at a time
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= ng) return;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t c = lane; c < gs / 8; c += 64) {
    float w[8];
    ld8<CT>(x, g * gs + c * 8, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mn = fminf(mn, w[j]);
      mx = fmaxf(mx, w[j]);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, m, 64));
    mx = fmaxf(mx, __shfl_xor(mx, m, 64));
  }
  float s, z;
  if (round_zp || sym) {
    qparams_ct<CT>(mn, mx, qmin, qmax, sym, s, z);
  } else {  // quant.py:557-558
    float r = rnd<CT>(mx - mn);
    r = fmaxf(r, rnd<CT>(1e-5f));
    s = rnd<CT>(r / (qmax - qmin));
    z = rnd<CT>(qmin - rnd<CT>(mn / s));
  }
  if (lane == 0) {
    st1<CT>(s_out, g, s);
    if (z_out) st1<CT>(z_out, g, z);
  }
}

__global__ void k_hqq_init(const float* s, int64_t ng, float* s_inv, HqqState* st) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ng) s_inv[i] = 1.0f / s[i];  // scales = 1 / scales
  if (i == 0) {
    st->best = 1e4f;
    st->stop = 0;
    st->iters_run = 0;
  }
}

__device__ __forceinline__ float shrink(float x, float inv_beta, float pm1, int l1) {
  const float ax = fabsf(x);
  float t;
  if (l1) t = ax - inv_beta;
  else t = ax - inv_beta * powf(ax, pm1);
  const float r = t > 0.f ? t : 0.f;                       // relu
  const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);  // torch.sign
  return sg * r;
}

// team of L lanes per group (L | 64); lanes stride the group 8 elements at a time
template <int L>
__global__ void __launch_bounds__(256) k_hqq_step(const float* w, int64_t ng, int64_t gs,
                                                  const float* s_inv, float* z, float qmin,
                                                  float qmax, float inv_beta, float pm1, int l1,
                                                  double* part, HqqState* st) {
  if (*reinterpret_cast<volatile int*>(&st->stop)) return;
  const int64_t team = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int tl = threadIdx.x & (L - 1);
  const bool live = team < ng;
  const int64_t g = live ? team : ng - 1;
  const float si = s_inv[g], zz = z[g];
  float acc = 0.f;
  double err = 0.0;
  for (int64_t c = tl; c < gs / 8; c += L) {
    float v[8];
    ld8<LCQ_F32>(w, g * gs + c * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float q = rintf(__fadd_rn(__fmul_rn(v[j], si), zz));
      q = fminf(fmaxf(q, qmin), qmax);
      const float r = __fsub_rn(q, zz) / si;
      const float d = __fsub_rn(v[j], r);
      err += (double)fabsf(d);
      const float e = shrink(d, inv_beta, pm1, l1);
      acc += __fsub_rn(q, __fmul_rn(__fsub_rn(v[j], e), si));
    }
  }
#pragma unroll
  for (int m = L / 2; m >= 1; m >>= 1) {
    acc += __shfl_xor(acc, m, 64);
    err += __shfl_xor(err, m, 64);
  }
  if (live && tl == 0) {
    z[g] = acc / (float)gs;  // torch.mean(..., axis=-1)
    part[g] = err;
  }
}

// global mean of |W - W_r| from the per-group partials (fixed order), compare, stop flag
__global__ void __launch_bounds__(256) k_hqq_check(const double* part, int64_t ng, int64_t numel,
                                                   HqqState* st) {
  if (st->stop) return;
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < ng; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k >= 1; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float e = (float)(red[0] / (double)numel);
    st->iters_run += 1;
    if (e < st->best) st->best = e;
    else st->stop = 1;
  }
}

__global__ void k_hqq_final(const float* s_inv, int64_t ng, float* s_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ng) s_out[i] = 1.0f / s_inv[i];  // scales = 1 / scales
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_minmax_qparams(const void* x, int dtype, int64_t ng, int64_t gs, int qmin,
                                  int qmax, int sym, int round_zp, void* scales, void* zeros,
                                  void* stream) {
  LCQ_REQUIRE(is_float_dt(dtype), "x dtype must be f32/f16/bf16");
  LCQ_REQUIRE(ng > 0 && gs > 0 && gs % 8 == 0, "groups must be non-empty multiples of 8");
  LCQ_REQUIRE(x && scales && (sym || zeros), "null pointer");
  LCQ_REQUIRE(qmin < qmax, "qmin must be < qmax");
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)((ng + 3) / 4));
  switch (dtype) {
    case LCQ_F32:
      hipLaunchKernelGGL((k_minmax_qparams<LCQ_F32>), grid, 256, 0, st, x, ng, gs, (float)qmin,
                         (float)qmax, sym, round_zp, scales, zeros);
      break;
    case LCQ_BF16:
      hipLaunchKernelGGL((k_minmax_qparams<LCQ_BF16>), grid, 256, 0, st, x, ng, gs, (float)qmin,
                         (float)qmax, sym, round_zp, scales, zeros);
      break;
    default:
      hipLaunchKernelGGL((k_minmax_qparams<LCQ_F16>), grid, 256, 0, st, x, ng, gs, (float)qmin,
                         (float)qmax, sym, round_zp, scales, zeros);
      break;
  }
  return check_launch("lcq_minmax_qparams");
}

extern "C" int64_t lcq_hqq_workspace_bytes(int64_t ng) {
  if (ng <= 0) return 0;
  return (int64_t)sizeof(HqqState) + ng * (int64_t)(sizeof(double) + sizeof(float));
}

extern "C" int lcq_hqq_proximal(const void* w, int64_t ng, int64_t gs, void* scales,
                                void* zeros, int qmin, int qmax, float lp_norm, float beta,
                                int iters, void* workspace, int64_t ws_bytes, void* state_out,
                                void* stream) {
  LCQ_REQUIRE(ng > 0 && gs > 0 && gs % 8 == 0, "groups must be non-empty multiples of 8");
  LCQ_REQUIRE(w && scales && zeros && workspace, "null pointer");
  LCQ_REQUIRE(ws_bytes >= lcq_hqq_workspace_bytes(ng), "workspace smaller than "
              "lcq_hqq_workspace_bytes");
  LCQ_REQUIRE(iters >= 0 && beta != 0.f, "iters >= 0, beta != 0");
  hipStream_t st = as_stream(stream);
  char* ws = reinterpret_cast<char*>(workspace);
  HqqState* state = reinterpret_cast<HqqState*>(ws);
  double* part = reinterpret_cast<double*>(ws + sizeof(HqqState));
  float* s_inv = reinterpret_cast<float*>(ws + sizeof(HqqState) + ng * sizeof(double));
  float* s = reinterpret_cast<float*>(scales);
  float* z = reinterpret_cast<float*>(zeros);
  const unsigned g1 = (unsigned)((ng + 255) / 256);
  hipLaunchKernelGGL(k_hqq_init, g1, 256, 0, st, s, ng, s_inv, state);
  int rc = check_launch("lcq_hqq_proximal: init");
  if (rc) return rc;
  int64_t lanes = gs / 8;
  int L = 64;
  while (L > lanes) L >>= 1;  // largest power of two <= gs / 8, at most a wave
  const int64_t threads = ng * L;
  const unsigned gridx = (unsigned)((threads + 255) / 256);
  const float inv_beta = (float)(1.0 / (double)beta);
  const float pm1 = (float)((double)lp_norm - 1.0);
  const int l1 = lp_norm == 1.f;
  for (int it = 0; it < iters; ++it) {
#define LCQ_HQQ_STEP(LL)                                                                    \
  hipLaunchKernelGGL((k_hqq_step<LL>), gridx, 256, 0, st, reinterpret_cast<const float*>(w), \
                     ng, gs, s_inv, z, (float)qmin, (float)qmax, inv_beta, pm1, l1, part, state)
    switch (L) {
      case 1: LCQ_HQQ_STEP(1); break;
      case 2: LCQ_HQQ_STEP(2); break;
      case 4: LCQ_HQQ_STEP(4); break;
      case 8: LCQ_HQQ_STEP(8); break;
      case 16: LCQ_HQQ_STEP(16); break;
      case 32: LCQ_HQQ_STEP(32); break;
      default: LCQ_HQQ_STEP(64); break;
    }
#undef LCQ_HQQ_STEP
    hipLaunchKernelGGL(k_hqq_check, 1, 256, 0, st, part, ng, ng * gs, state);
    rc = check_launch("lcq_hqq_proximal: step");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_hqq_final, g1, 256, 0, st, s_inv, ng, s);
  if (state_out)
    (void)hipMemcpyAsync(state_out, state, sizeof(HqqState), hipMemcpyDeviceToDevice, st);
  return check_launch("lcq_hqq_proximal: final");
}
