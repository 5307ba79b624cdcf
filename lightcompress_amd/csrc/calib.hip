// Static per-tensor activation calibration (gfx950): the range statistics and qparams of
// register_act_qparams (base_blockwise_quantization.py:567-588) -> get_batch_tensors_qparams
// (quant.py:561-586), static_minmax (quant.py:253-262) and static_moving_minmax (:431-450).
//
// The work is one HBM pass over every calibration activation of a linear's input (Llama-3-8B,
// 128 x 2048 tokens: 2 GB per 4096-wide input, 7.5 GB for down_proj's): k_seg_minmax streams
// each segment (= one calibration entry of the reference's act_tensors list) with 16-byte
// loads, many workgroups per segment (per-workgroup partials, no atomics), then two tiny
// kernels fold the partials and evaluate the reference's scalar chain on the device.
#include <math.h>

#include "lcq_common.h"

namespace lcq {
namespace {

constexpr int kBlock = 256;

struct SegArgs {
  const void* p[LCQ_MINMAX_SEGS];
  int64_t n[LCQ_MINMAX_SEGS];
};

__device__ __forceinline__ void upd(float v, float& mn, float& mx, bool& nan) {
  mn = fminf(mn, v);
  mx = fmaxf(mx, v);
  nan |= (v != v);
}

// torch.min / torch.max of one segment (NaN-propagating: any NaN -> both NaN). grid =
// (parts, segments of this launch); partial (min, max) per workgroup -> ws[seg * parts + part].
template <int DT>
__global__ __launch_bounds__(kBlock) void k_seg_minmax(SegArgs a, int parts, float2* ws) {
  const int seg = blockIdx.y;
  const void* x = a.p[seg];
  const int64_t n = a.n[seg];
  const int64_t nvec = n / 8;
  float mn = INFINITY, mx = -INFINITY;
  bool nan = false;
  const int64_t stride = (int64_t)parts * kBlock;
  int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  // four independent 16-byte (bf16/f16) or 32-byte (f32) loads in flight per lane
  for (; v + 3 * stride < nvec; v += 4 * stride) {
    float e0[8], e1[8], e2[8], e3[8];
    ld8<DT>(x, v * 8, e0);
    ld8<DT>(x, (v + stride) * 8, e1);
    ld8<DT>(x, (v + 2 * stride) * 8, e2);
    ld8<DT>(x, (v + 3 * stride) * 8, e3);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      upd(e0[k], mn, mx, nan);
      upd(e1[k], mn, mx, nan);
      upd(e2[k], mn, mx, nan);
      upd(e3[k], mn, mx, nan);
    }
  }
  for (; v < nvec; v += stride) {
    float e0[8];
    ld8<DT>(x, v * 8, e0);
#pragma unroll
    for (int k = 0; k < 8; ++k) upd(e0[k], mn, mx, nan);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nvec * 8 + threadIdx.x; i < n; i += kBlock) upd(ld1<DT>(x, i), mn, mx, nan);
  }
  // wave reduction, then across the 4 waves through LDS
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, o, 64));
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  }
  nan = __any(nan);
  __shared__ float smn[kBlock / 64], smx[kBlock / 64];
  __shared__ int snan[kBlock / 64];
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    smn[w] = mn;
    smx[w] = mx;
    snan[w] = nan ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    bool bn = false;
    for (int i = 0; i < kBlock / 64; ++i) {
      mn = fminf(mn, smn[i]);
      mx = fmaxf(mx, smx[i]);
      bn |= snan[i] != 0;
    }
    ws[(int64_t)seg * parts + blockIdx.x] = bn ? make_float2(NAN, NAN) : make_float2(mn, mx);
  }
}

// fold each segment's partials (fixed order) -> minmax[2 * (seg0 + i) + {0, 1}]
__global__ void k_fold_minmax(const float2* ws, int nseg, int parts, float* minmax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  float mn = INFINITY, mx = -INFINITY;
  bool nan = false;
  for (int p = 0; p < parts; ++p) {
    const float2 t = ws[(int64_t)i * parts + p];
    nan |= (t.x != t.x);
    mn = fminf(mn, t.x);
    mx = fmaxf(mx, t.y);
  }
  minmax[2 * i] = nan ? NAN : mn;
  minmax[2 * i + 1] = nan ? NAN : mx;
}

__device__ __forceinline__ float rnd_rt(int dt, float v) {
  if (dt == LCQ_BF16) return bf16_rne(v);
  if (dt == LCQ_F16) return f16_rne(v);
  return v;
}
__device__ __forceinline__ float max_nan(float a, float b) {  // torch.max(a, b): NaN wins
  return (a != a || b != b) ? NAN : fmaxf(a, b);
}
__device__ __forceinline__ float clamp_min_t(float a, float lo) {  // std::max(a, lo)
  return (a < lo) ? lo : a;
}

// the range, then get_qparams (quant.py:545-559). One workgroup.
__global__ __launch_bounds__(kBlock) void k_act_qparams(const float* minmax, int64_t nseg,
                                                        int algo, float alpha, int rdt, int sdt,
                                                        int sym, float qmin, float qmax,
                                                        float* out) {
  __shared__ double smn[kBlock], smx[kBlock];
  float mn = 0.f, mx = 0.f;
  if (algo == LCQ_CALIB_STATIC_MINMAX) {
    // torch: stats (fp32) .mean() = fp32 sum, then / n. The sum is taken in fp64 here (torch's
    // fp32 cascade order is SIMD-width dependent) and rounded once: T2, within an ulp.
    double a = 0.0, b = 0.0;
    for (int64_t i = threadIdx.x; i < nseg; i += kBlock) {
      a += (double)minmax[2 * i];
      b += (double)minmax[2 * i + 1];
    }
    smn[threadIdx.x] = a;
    smx[threadIdx.x] = b;
    __syncthreads();
    for (int o = kBlock / 2; o >= 1; o >>= 1) {
      if (threadIdx.x < o) {
        smn[threadIdx.x] += smn[threadIdx.x + o];
        smx[threadIdx.x] += smx[threadIdx.x + o];
      }
      __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const float fn = (float)nseg;
    mn = (float)smn[0] / fn;
    mx = (float)smx[0] / fn;
  } else {
    if (threadIdx.x != 0) return;
    // moving = moving + alpha * (v - moving), each op rounded to the range dtype
    mn = minmax[0];
    mx = minmax[1];
    for (int64_t i = 1; i < nseg; ++i) {
      mn = rnd_rt(rdt, mn + rnd_rt(rdt, alpha * rnd_rt(rdt, minmax[2 * i] - mn)));
      mx = rnd_rt(rdt, mx + rnd_rt(rdt, alpha * rnd_rt(rdt, minmax[2 * i + 1] - mx)));
    }
  }
  const float lo = rnd_rt(rdt, 1e-5f);  // .clamp(min=1e-5) in the range dtype
  float s, z = 0.f;
  if (sym) {
    float am = max_nan(fabsf(mx), fabsf(mn));
    am = clamp_min_t(am, lo);
    s = rnd_rt(sdt, am / rnd_rt(sdt, qmax));
  } else {
    float r = clamp_min_t(rnd_rt(rdt, mx - mn), lo);
    s = rnd_rt(sdt, r / (qmax - qmin));
    const float t = rintf(rnd_rt(sdt, mn / s));  // torch.round(min_val / scales)
    z = rnd_rt(sdt, qmin - t);
    z = (z != z) ? z : fminf(fmaxf(z, qmin), qmax);  // .clamp(qmin, qmax)
  }
  out[0] = s;
  out[1] = z;
  out[2] = mn;
  out[3] = mx;
}

}  // namespace
}  // namespace lcq

using namespace lcq;

extern "C" int lcq_minmax_segments(const void* const* segs, const int64_t* seg_lens,
                                   int64_t nseg, int dtype, void* minmax, void* workspace,
                                   void* stream) {
  LCQ_REQUIRE(segs && seg_lens && minmax && workspace, "null pointer");
  LCQ_REQUIRE(nseg > 0, "no calibration tensors (the reference asserts len(act_tensors) > 0)");
  LCQ_REQUIRE(dtype == LCQ_F32 || dtype == LCQ_F16 || dtype == LCQ_BF16,
              "dtype must be F32, F16 or BF16");
  int64_t longest = 0;
  for (int64_t i = 0; i < nseg; ++i) {
    LCQ_REQUIRE(segs[i] != nullptr, "null segment");
    LCQ_REQUIRE(seg_lens[i] > 0, "empty segment (torch.max of an empty tensor raises)");
    LCQ_REQUIRE((reinterpret_cast<uintptr_t>(segs[i]) & 15) == 0, "segments must be 16-byte aligned");
    longest = seg_lens[i] > longest ? seg_lens[i] : longest;
  }
  // enough workgroups per segment that a launch of LCQ_MINMAX_SEGS segments fills the chip,
  // each lane still streaming >= 4 vectors
  int64_t parts = (longest / 8 + 4 * kBlock - 1) / (4 * kBlock);
  parts = parts < 1 ? 1 : (parts > LCQ_MINMAX_PARTS ? LCQ_MINMAX_PARTS : parts);
  hipStream_t st = as_stream(stream);
  float2* ws = reinterpret_cast<float2*>(workspace);
  float* mm = reinterpret_cast<float*>(minmax);
  for (int64_t s0 = 0; s0 < nseg; s0 += LCQ_MINMAX_SEGS) {
    const int cnt = (int)((nseg - s0) < LCQ_MINMAX_SEGS ? (nseg - s0) : LCQ_MINMAX_SEGS);
    SegArgs a{};
    for (int i = 0; i < cnt; ++i) {
      a.p[i] = segs[s0 + i];
      a.n[i] = seg_lens[s0 + i];
    }
    dim3 grid((unsigned)parts, (unsigned)cnt);
    switch (dtype) {
      case LCQ_BF16: k_seg_minmax<LCQ_BF16><<<grid, kBlock, 0, st>>>(a, (int)parts, ws); break;
      case LCQ_F16: k_seg_minmax<LCQ_F16><<<grid, kBlock, 0, st>>>(a, (int)parts, ws); break;
      default: k_seg_minmax<LCQ_F32><<<grid, kBlock, 0, st>>>(a, (int)parts, ws); break;
    }
    k_fold_minmax<<<1, LCQ_MINMAX_SEGS, 0, st>>>(ws, cnt, (int)parts, mm + 2 * s0);
  }
  return check_launch("lcq_minmax_segments");
}

extern "C" int lcq_act_static_qparams(const void* minmax, int64_t nseg, int algo, float alpha,
                                      int range_dtype, int scale_dtype, int sym, float qmin,
                                      float qmax, void* out, void* stream) {
  LCQ_REQUIRE(minmax && out, "null pointer");
  LCQ_REQUIRE(nseg > 0, "no calibration ranges");
  LCQ_REQUIRE(algo == LCQ_CALIB_STATIC_MINMAX || algo == LCQ_CALIB_STATIC_MOVING_MINMAX,
              "algo must be LCQ_CALIB_STATIC_MINMAX or LCQ_CALIB_STATIC_MOVING_MINMAX");
  LCQ_REQUIRE(is_float_dt(range_dtype) && is_float_dt(scale_dtype),
              "range / scale dtype must be F32, F16 or BF16");
  LCQ_REQUIRE(algo != LCQ_CALIB_STATIC_MINMAX || range_dtype == LCQ_F32,
              "static_minmax ranges are fp32 means");
  LCQ_REQUIRE(qmax > qmin, "qmax must exceed qmin");
  k_act_qparams<<<1, kBlock, 0, as_stream(stream)>>>(
      reinterpret_cast<const float*>(minmax), nseg, algo, alpha, range_dtype, scale_dtype, sym,
      qmin, qmax, reinterpret_cast<float*>(out));
  return check_launch("lcq_act_static_qparams");
}
