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

// ---------------------------------------------------------------------------------------
// static_hist (quant.py:264-529, get_static_hist_range): per-segment histograms, their
// sequential combination, the L2 threshold search and get_qparams.
// ---------------------------------------------------------------------------------------
constexpr int kBins = 2048;  // BaseQuantizer bins (quant.py:83)
constexpr int kUp = 16;      // upsample_rate (quant.py:84)

// histc bounds of segment i: the running (min, max) over segments 0..i (the reference's
// new_min / new_max), histc_select_outer_bin_edges' degenerate-range rules
__device__ inline void hist_bounds(const float* mm, int64_t i, float& lo, float& hi) {
  float a = mm[0], b = mm[1];
  for (int64_t j = 1; j <= i; ++j) {
    a = fminf(a, mm[2 * j]);
    b = fmaxf(b, mm[2 * j + 1]);
  }
  if (a == b) {  // aminmax of the input itself, then +-1
    a = mm[2 * i];
    b = mm[2 * i + 1];
  }
  if (a == b) {
    a = (float)((double)a - 1.0);
    b = (float)((double)b + 1.0);
  }
  lo = a;
  hi = b;
}

// torch.histc(x.float(), 2048, lo, hi) on CPU (histogramdd LINEAR_INTERPOLATION): pos =
// int((x - lo) * bins / (hi - lo)) in fp32, the right edge in the last bin, NaN / out of range
// skipped. Exact integer counts (LDS then global atomics).
template <int DT>
__global__ __launch_bounds__(kBlock) void k_histc_segs(SegArgs a, int64_t seg0, int parts,
                                                       const float* minmax, uint32_t* hist) {
  __shared__ uint32_t h[kBins];
  for (int i = threadIdx.x; i < kBins; i += kBlock) h[i] = 0;
  const int seg = blockIdx.y;
  float lo, hi;
  hist_bounds(minmax, seg0 + seg, lo, hi);
  const float span = hi - lo;
  __syncthreads();
  const void* x = a.p[seg];
  const int64_t n = a.n[seg];
  auto add = [&](float v) {
    if (!(v >= lo && v <= hi)) return;
    int64_t pos = (int64_t)(((v - lo) * (float)kBins) / span);
    if (pos == kBins) pos = kBins - 1;
    atomicAdd(&h[pos], 1u);
  };
  const int64_t nvec = n / 8;
  const int64_t stride = (int64_t)parts * kBlock;
  for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < nvec; v += stride) {
    float e[8];
    ld8<DT>(x, v * 8, e);
#pragma unroll
    for (int k = 0; k < 8; ++k) add(e[k]);
  }
  if (blockIdx.x == 0)
    for (int64_t i = nvec * 8 + threadIdx.x; i < n; i += kBlock) add(ld1<DT>(x, i));
  __syncthreads();
  uint32_t* g = hist + (seg0 + seg) * kBins;
  for (int i = threadIdx.x; i < kBins; i += kBlock)
    if (h[i]) atomicAdd(&g[i], h[i]);
}

// torch.linspace(start, end, steps)[k] on CPU, scalar path (float): step = (end - start) /
// (steps - 1); first half start + step * k, second half end - step * (steps - 1 - k)
__device__ inline float linspace_at(float start, float end, int64_t steps, int64_t k) {
  const float step = (end - start) / (float)(steps - 1);
  if (k < steps / 2) return start + step * (float)k;
  return end - step * (float)(steps - 1 - k);
}

// torch.div(a, b, rounding_mode='floor') for float (c10 div_floor_floating)
__device__ inline float div_floor_f(float a, float b) {
  if (b == 0.f) return a / b;
  const float mod = fmodf(a, b);
  float div = (a - mod) / b;
  if (mod != 0.f && ((b < 0.f) != (mod < 0.f))) div -= 1.f;
  float fd;
  if (div != 0.f) {
    fd = floorf(div);
    if (div - fd > 0.5f) fd += 1.f;
  } else {
    fd = copysignf(0.f, a / b);
  }
  return fd;
}

// BaseQuantizer.get_norm: density * ((e^3 - b^3) / 3), every op in fp32
__device__ inline float l2norm_term(float b, float e, float dens) {
  const float n = ((e * e) * e - (b * b) * b) / 3.f;
  return dens * n;
}

constexpr int kHT = 1024;  // threads of the threshold kernel

__device__ inline double block_sum_d(double v, double* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x / 64;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < kHT / 64; ++i) t += red[i];
  return t;
}

// One workgroup: combine the per-segment histograms in order (quant.py:462-512,
// _combine_histograms / _upscale_histogram :332-401), search the threshold (get_hist_threshold
// :403-451 with get_quantization_error :275-330), then get_qparams (sym). out fp32 [4] =
// scale, 0, new_min, new_max.
__global__ __launch_bounds__(kHT) void k_hist_threshold(const uint32_t* hist, const float* mm,
                                                       int64_t nseg, int dst_nbins, float qmax,
                                                       float* out) {
  __shared__ float H[kBins], U[kBins];
  __shared__ float bnd[kBins + 1];
  __shared__ double red[kHT / 64];
  __shared__ float cs[kBins];
  __shared__ int ctl[4];
  float cur_min = 0.f, cur_max = 0.f;
  for (int64_t i = 0; i < nseg; ++i) {
    float lo, hi;
    hist_bounds(mm, i, lo, hi);  // the bounds its histc used == (new_min, new_max)
    const uint32_t* g = hist + i * kBins;
    if (i == 0) {
      for (int b = threadIdx.x; b < kBins; b += kHT) H[b] = (float)g[b];
      cur_min = mm[0];
      cur_max = mm[1];
      __syncthreads();
      continue;
    }
    const float new_min = fminf(cur_min, mm[2 * i]);
    const float new_max = fmaxf(cur_max, mm[2 * i + 1]);
    if (new_min == cur_min && new_max == cur_max) {
      for (int b = threadIdx.x; b < kBins; b += kHT) H[b] = H[b] + (float)g[b];
    } else if (cur_min == cur_max) {
      // orig_min == orig_max: histc(orig_min, new range) * sum(update) + update
      double t = 0.0;
      for (int b = threadIdx.x; b < kBins; b += kHT) t += (double)g[b];
      const float bin_value = (float)block_sum_d(t, red);
      int64_t pos = (int64_t)(((cur_min - new_min) * (float)kBins) / (new_max - new_min));
      if (pos == kBins) pos = kBins - 1;
      for (int b = threadIdx.x; b < kBins; b += kHT)
        H[b] = (b == pos ? bin_value : 0.f) + (float)g[b];
    } else {
      // upscale: 2048*16 midpoints of the old range, bucketized into the new bins
      const float bin_size = (cur_max - cur_min) / (float)(kBins * kUp);
      const float half = 0.5f * bin_size;
      for (int b = threadIdx.x; b <= kBins; b += kHT)
        bnd[b] = linspace_at(new_min, new_max, kBins + 1, b);
      for (int b = threadIdx.x; b < kBins; b += kHT) U[b] = H[b];
      __syncthreads();
      auto bucket = [&](int64_t k) -> int {
        const float mid = linspace_at(cur_min, cur_max, (int64_t)kBins * kUp + 1, k) + half;
        int l = 0, r = kBins + 1;  // count of boundaries <= mid (bucketize right=True)
        while (l < r) {
          const int m = (l + r) >> 1;
          if (bnd[m] <= mid) l = m + 1;
          else r = m;
        }
        int bi = l - 1;
        return bi < 0 ? 0 : (bi >= kBins ? kBins - 1 : bi);
      };
      for (int b = threadIdx.x; b < kBins; b += kHT) {
        // first midpoint with bucket >= b (buckets are non-decreasing in k)
        int64_t l = 0, r = (int64_t)kBins * kUp;
        while (l < r) {
          const int64_t m = (l + r) >> 1;
          if (bucket(m) < b) l = m + 1;
          else r = m;
        }
        float acc = 0.f;  // bincount: sequential in midpoint order
        for (int64_t k = l; k < (int64_t)kBins * kUp && bucket(k) == b; ++k)
          acc += U[k / kUp] / (float)kUp;
        H[b] = (float)g[b] + acc;
      }
    }
    cur_min = new_min;
    cur_max = new_max;
    __syncthreads();
  }
  // ---- get_hist_threshold ----
  double t = 0.0;
  for (int b = threadIdx.x; b < kBins; b += kHT) t += (double)H[b];
  const double total = (double)(float)block_sum_d(t, red);  // torch.sum(histogram).item()
  if (threadIdx.x == 0) {
    double c = 0.0;  // cumsum: double accumulation, float results
    for (int b = 0; b < kBins; ++b) {
      c += (double)H[b];
      cs[b] = (float)c;
    }
  }
  __syncthreads();
  const double bw_d = ((double)cur_max - (double)cur_min) / kBins;
  double alpha = 0.0, beta = 1.0, norm_min = INFINITY;
  int start_bin = 0, end_bin = kBins - 1;
  // thread 0 walks the quantile bounds; the whole block evaluates each candidate's error
  while (true) {
    if (threadIdx.x == 0) {
      int go = 0;
      while (alpha < beta) {
        const double na = alpha + 1e-8, nb = beta - 1e-8;
        int left = start_bin, right = end_bin;
        while (left < end_bin && cs[left] < (float)(na * total)) ++left;
        while (right > start_bin && cs[right] > (float)(nb * total)) --right;
        int ns = start_bin, ne = end_bin;
        if ((left - start_bin) > (end_bin - right)) {
          ns = left;
          alpha = na;
        } else {
          ne = right;
          beta = nb;
        }
        if (ns == start_bin && ne == end_bin) continue;
        ctl[0] = ns;
        ctl[1] = ne;
        go = 1;
        break;
      }
      ctl[2] = go;
    }
    __syncthreads();
    if (!ctl[2]) break;
    const int ns = ctl[0], ne = ctl[1];
    const double dbw_d = bw_d * (double)(ne - ns + 1) / (double)dst_nbins;
    double part = 0.0;
    if (dbw_d != 0.0) {
      const float bw = (float)bw_d, dbw = (float)dbw_d, hdbw = (float)(dbw_d / 2);
      const float v0 = l2norm_term((float)(-dbw_d / 2), hdbw, 1.f);  // (e^3 - b^3) / 3
      float sumf = 0.f;
      for (int b = threadIdx.x; b < kBins; b += kHT) {
        const float sbb = (float)(b - ns) * bw;
        const float sbe = sbb + bw;
        const float db = fminf(fmaxf(div_floor_f(sbb, dbw), 0.f), (float)(dst_nbins - 1));
        const float dbc = (db + 0.5f) * dbw;
        const float de = fminf(fmaxf(div_floor_f(sbe, dbw), 0.f), (float)(dst_nbins - 1));
        const float dens = H[b] / bw;
        float nrm = 0.f;
        nrm = nrm + l2norm_term(sbb - dbc, hdbw * 1.f, dens);
        nrm = nrm + ((de - db) - 1.f) * (dens * v0);
        const float dec = de * dbw + hdbw;
        nrm = nrm + l2norm_term((float)(-dbw_d / 2), sbe - dec, dens);
        part += (double)nrm;
        (void)sumf;
      }
      part = block_sum_d(part, red);
    }
    if (threadIdx.x == 0) {
      const double norm = dbw_d == 0.0 ? 0.0 : (double)(float)part;
      if (norm > norm_min) {
        ctl[3] = 1;
      } else {
        ctl[3] = 0;
        norm_min = norm;
        start_bin = ns;
        end_bin = ne;
      }
    }
    __syncthreads();
    if (ctl[3]) break;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float bwt = (cur_max - cur_min) / (float)kBins;  // tensor op in get_hist_threshold
    const float nmin = cur_min + bwt * (float)start_bin;
    const float nmax = cur_min + bwt * (float)(end_bin + 1);
    float am = fmaxf(fabsf(nmax), fabsf(nmin));
    am = am < 1e-5f ? 1e-5f : am;
    out[0] = am / qmax;
    out[1] = 0.f;
    out[2] = nmin;
    out[3] = nmax;
  }
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

extern "C" int64_t lcq_act_hist_workspace_bytes(int64_t nseg) {
  return nseg > 0 ? nseg * kBins * (int64_t)sizeof(uint32_t) : 0;
}

extern "C" int lcq_act_static_hist_qparams(const void* const* segs, const int64_t* seg_lens,
                                           int64_t nseg, int dtype, const void* minmax,
                                           int dst_nbins, float qmax, void* out,
                                           void* workspace, void* stream) {
  LCQ_REQUIRE(segs && seg_lens && minmax && out && workspace, "null pointer");
  LCQ_REQUIRE(nseg > 0, "no calibration tensors");
  LCQ_REQUIRE(dtype == LCQ_F32 || dtype == LCQ_F16 || dtype == LCQ_BF16,
              "dtype must be F32, F16 or BF16");
  LCQ_REQUIRE(dst_nbins >= 2 && qmax > 0.f, "bad dst_nbins / qmax");
  int64_t longest = 0;
  for (int64_t i = 0; i < nseg; ++i) {
    LCQ_REQUIRE(segs[i] != nullptr && seg_lens[i] > 0, "empty segment");
    LCQ_REQUIRE((reinterpret_cast<uintptr_t>(segs[i]) & 15) == 0, "segments must be 16-byte aligned");
    longest = seg_lens[i] > longest ? seg_lens[i] : longest;
  }
  int64_t parts = (longest / 8 + 4 * kBlock - 1) / (4 * kBlock);
  parts = parts < 1 ? 1 : (parts > LCQ_MINMAX_PARTS ? LCQ_MINMAX_PARTS : parts);
  hipStream_t st = as_stream(stream);
  uint32_t* hist = reinterpret_cast<uint32_t*>(workspace);
  if (hipMemsetAsync(hist, 0, (size_t)nseg * kBins * sizeof(uint32_t), st) != hipSuccess)
    return fail(LCQ_ELAUNCH, "lcq_act_static_hist_qparams: memset failed");
  const float* mm = reinterpret_cast<const float*>(minmax);
  for (int64_t s0 = 0; s0 < nseg; s0 += LCQ_MINMAX_SEGS) {
    const int cnt = (int)((nseg - s0) < LCQ_MINMAX_SEGS ? (nseg - s0) : LCQ_MINMAX_SEGS);
    SegArgs a{};
    for (int i = 0; i < cnt; ++i) {
      a.p[i] = segs[s0 + i];
      a.n[i] = seg_lens[s0 + i];
    }
    dim3 grid((unsigned)parts, (unsigned)cnt);
    switch (dtype) {
      case LCQ_BF16: k_histc_segs<LCQ_BF16><<<grid, kBlock, 0, st>>>(a, s0, (int)parts, mm, hist); break;
      case LCQ_F16: k_histc_segs<LCQ_F16><<<grid, kBlock, 0, st>>>(a, s0, (int)parts, mm, hist); break;
      default: k_histc_segs<LCQ_F32><<<grid, kBlock, 0, st>>>(a, s0, (int)parts, mm, hist); break;
    }
  }
  k_hist_threshold<<<1, kHT, 0, st>>>(hist, mm, nseg, dst_nbins, qmax,
                                      reinterpret_cast<float*>(out));
  return check_launch("lcq_act_static_hist_qparams");
}
