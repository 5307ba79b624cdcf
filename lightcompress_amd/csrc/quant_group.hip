// Grouped integer quantization (fake quant / real quant / vLLM pack) for gfx950.
//
// Reference semantics: llmc/compression/quantization/quant.py
//   get_minmax_range  :132-143   get_qparams :545-559   quant/dequant :699-717
//   fake_quant_weight_dynamic :833-869   real_quant_weight_dynamic :916-953
//   fake/real_quant_weight_static :785-831, 871-914
// and VllmRealQuantLinear.pack (module_utils.py:929-955).
//
// Design (HBM-bound streaming, no MFMA): one lane owns 8 consecutive elements (one 16-byte
// load for bf16/fp16), a group of G elements is G/8 adjacent lanes of one wave, and the group
// min/max is a butterfly over those lanes (__shfl_xor) -- no LDS, one pass over HBM:
// read 2 B/elem, write 2 B (fake quant) or 0.5 B (int4 packed) per element.
// Groups wider than 512 (per-channel rows) use one 256-thread workgroup per group.
#define LCQ_BF16_HW 1  // bf16 rounding on v_cvt_pk_bf16_f32 (see lcq_common.h)
#include "lcq_common.h"

namespace lcq {

struct QuantArgs {
  const void* x;
  const void* pre;   // optional [cols] pre-scale (x dtype)
  const void* cmax;  // optional [ngroups] clip max (x dtype)
  const void* cmin;  // optional [ngroups] clip min (x dtype); NULL + cmax => -cmax
  const void* s_in;  // static: scales
  const void* z_in;  // static: zeros (nullable)
  int s_dt, z_dt;
  int64_t rows, cols, group;
  float qmin, qmax;
  int sym;
  void* fq;
  int fq_dt;
  void* codes;
  int codes_dt;
  void* packed;
  int pack_bits;
  void* s_out;
  void* z_out;
  int qp_scalar;  // static: one fp32 scale / zero used at full precision (0-dim CPU operands)
  int nozp;       // static: round_zp False (quant.py:701-707): round(x / s.clamp_min(1e-9) + z)
  const void* up;   // dynamic, calib_algo learnable: [ngroups] clip factors (x dtype)
  const void* low;  // nullable
};

// calib_algo learnable: the group's range through get_learnable_range (quant.py:205-219)
template <int CT>
__device__ __forceinline__ void learnable(const QuantArgs& a, int64_t gi, float& mn, float& mx) {
  if (a.up)
    learnable_range<CT>(mn, mx, ld1<CT>(a.up, gi), a.low ? ld1<CT>(a.low, gi) : 0.f,
                        a.low != nullptr, a.sym);
}

__device__ __forceinline__ float ld_rt(const void* p, int dt, int64_t i) {
  switch (dt) {
    case LCQ_F32: return ld1<LCQ_F32>(p, i);
    case LCQ_BF16: return ld1<LCQ_BF16>(p, i);
    case LCQ_F16: return ld1<LCQ_F16>(p, i);
    case LCQ_I32: return ld1<LCQ_I32>(p, i);
    case LCQ_I8: return ld1<LCQ_I8>(p, i);
    case LCQ_U8: return ld1<LCQ_U8>(p, i);
    default: return 0.f;
  }
}

// quant.py:699-717: q = clamp(round(x/s) + z, qmin, qmax); x^ = (q - z) * s
template <int CT>
__device__ __forceinline__ void qdq8(const float (&w)[8], float s, float z, float qmin,
                                     float qmax, float (&q)[8], float (&dq)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = rintf(rnd<CT>(w[j] / s));
    t = rnd<CT>(t + z);
    t = fminf(fmaxf(t, qmin), qmax);
    q[j] = t;
    dq[j] = rnd<CT>(rnd<CT>(t - z) * s);
  }
}

// qdq8 with the Markstein quotient (div_mk, 3 ops instead of the ~10-op IEEE division) for a
// group where it is provably the IEEE quotient: see mk_safe.
// The group's values lie in [mn, mx]; with s and 1/s finite and every |x| * (1/s) far from
// overflow, each x / s is finite and either normal (Markstein's theorem: exact) or below
// 2^-126 in magnitude, where both quotients round to a signed zero of x's sign after rint.
// Asym groups of huge, nearly equal values (range floored at 1e-5) or ranges that overflow
// the compute dtype take the IEEE path.
__device__ __forceinline__ bool mk_safe(float mn, float mx, float s, float rs) {
  return isfinite(s) && fmaxf(fabsf(mn), fabsf(mx)) * rs < 1e30f;  // NaN -> false
}

template <int CT>
__device__ __forceinline__ void qdq8_mk(const float (&w)[8], float s, float rs, float z,
                                        float qmin, float qmax, float (&q)[8], float (&dq)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = rintf(rnd<CT>(div_mk(w[j], s, rs)));
    t = rnd<CT>(t + z);
    t = fminf(fmaxf(t, qmin), qmax);
    q[j] = t;
    dq[j] = rnd<CT>(rnd<CT>(t - z) * s);
  }
}

__device__ __forceinline__ float round_dt(float v, int dt) {
  if (dt == LCQ_BF16) return rnd<LCQ_BF16>(v);
  if (dt == LCQ_F16) return rnd<LCQ_F16>(v);
  return v;
}

__device__ __forceinline__ void store_fq8(void* fq, int dt, int64_t e0, const float (&v)[8]) {
  switch (dt) {
    case LCQ_F32: st8<LCQ_F32>(fq, e0, v); break;
    case LCQ_BF16: st8<LCQ_BF16>(fq, e0, v); break;
    case LCQ_F16: st8<LCQ_F16>(fq, e0, v); break;
    default: break;
  }
}

__device__ __forceinline__ void store_codes8(void* codes, int dt, int64_t e0,
                                             const float (&q)[8]) {
  if (dt == LCQ_I32) {
    int4* p = reinterpret_cast<int4*>(reinterpret_cast<int32_t*>(codes) + e0);
    p[0] = make_int4((int)q[0], (int)q[1], (int)q[2], (int)q[3]);
    p[1] = make_int4((int)q[4], (int)q[5], (int)q[6], (int)q[7]);
  } else {
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo |= ((uint32_t)((int)q[j]) & 0xffu) << (8 * j);
      hi |= ((uint32_t)((int)q[4 + j]) & 0xffu) << (8 * j);
    }
    *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(codes) + e0) = make_uint2(lo, hi);
  }
}

// module_utils.py:929-955: u = uint8(code + 2^(b-1)); packed |= u << (b*i) (uint32)
__device__ __forceinline__ void store_packed8(void* packed, int bits, int64_t e0,
                                              const float (&q)[8]) {
  const uint32_t off = 1u << (bits - 1);
  uint32_t* p = reinterpret_cast<uint32_t*>(packed);
  if (bits == 4) {
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) w |= (((uint32_t)((int)q[j]) + off) & 0xffu) << (4 * j);
    p[e0 >> 3] = w;
  } else {  // 8
    uint32_t w0 = 0, w1 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w0 |= (((uint32_t)((int)q[j]) + off) & 0xffu) << (8 * j);
      w1 |= (((uint32_t)((int)q[4 + j]) + off) & 0xffu) << (8 * j);
    }
    *reinterpret_cast<uint2*>(p + (e0 >> 2)) = make_uint2(w0, w1);
  }
}

template <int CT>
__device__ __forceinline__ void load_pre_clip(const QuantArgs& a, int64_t e0, int64_t gi,
                                              float (&w)[8], bool small = false) {
  ld8<CT>(a.x, e0, w);
  if (a.pre) {  // awq.py:39-46 w.mul_(scales.view(1,-1)) in the weight dtype
    float s[8];
    ld8<CT>(a.pre, small ? (int64_t)((uint32_t)e0 % (uint32_t)a.cols) : e0 % a.cols, s);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j] * s[j]);
  }
  if (a.cmax) {  // auto_clip.py:206 torch.clamp(w, min_val, max_val)
    float mx = ld1<CT>(a.cmax, gi);
    float mn = a.cmin ? ld1<CT>(a.cmin, gi) : -mx;
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = fminf(fmaxf(w[j], mn), mx);
  }
}

template <int CT>
__device__ __forceinline__ void emit(const QuantArgs& a, int64_t e0, const float (&q)[8],
                                     const float (&dq)[8]) {
  if (a.fq) store_fq8(a.fq, a.fq_dt, e0, dq);
  if (a.codes) store_codes8(a.codes, a.codes_dt, e0, q);
  if (a.packed) store_packed8(a.packed, a.pack_bits, e0, q);
}

// ---------------------------------------------------------------------------------------
// dynamic, group of L*8 elements = L adjacent lanes (L in {1..64}, power of two)
// ---------------------------------------------------------------------------------------
template <int CT, int L>
__global__ void __launch_bounds__(256) k_quant_dyn_lanes(QuantArgs a) {
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool small = a.rows * a.cols < (int64_t(1) << 32);  // 32-bit column index math
  // all lanes of a group stay in the loop together: n8 is a multiple of L (group = 8 L)
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8;
    const int64_t gi = t / L;  // L is a power of two: a shift
    float w[8];
    load_pre_clip<CT>(a, e0, gi, w, small);
    float mn = w[0], mx = w[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      mn = fminf(mn, w[j]);
      mx = fmaxf(mx, w[j]);
    }
#pragma unroll
    for (int m = L / 2; m >= 1; m >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, m, 64));
      mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    }
    const float gmn = mn, gmx = mx;  // the group's values lie in [gmn, gmx] (mk_safe)
    learnable<CT>(a, gi, mn, mx);
    float s, z;
    qparams_ct<CT>(mn, mx, a.qmin, a.qmax, a.sym, s, z);
    float q[8], dq[8];
    const float rs = 1.0f / s;
    if (mk_safe(gmn, gmx, s, rs)) qdq8_mk<CT>(w, s, rs, z, a.qmin, a.qmax, q, dq);
    else qdq8<CT>(w, s, z, a.qmin, a.qmax, q, dq);
    emit<CT>(a, e0, q, dq);
    if ((t & (L - 1)) == 0) {
      if (a.s_out) st1<CT>(a.s_out, gi, s);
      if (a.z_out && !a.sym) st1<CT>(a.z_out, gi, z);
    }
  }
}

// ---------------------------------------------------------------------------------------
// dynamic, one 256-thread workgroup per (wide) group, e.g. per-channel rows of 4096..28672
// ---------------------------------------------------------------------------------------
template <int CT>
__global__ void __launch_bounds__(256) k_quant_dyn_rows(QuantArgs a) {
  __shared__ float red[2][4];
  const int64_t gi = blockIdx.x;
  const int64_t base = gi * a.group;
  const int64_t n8 = a.group / 8;
  float mn = INFINITY, mx = -INFINITY;
  for (int64_t c = threadIdx.x; c < n8; c += blockDim.x) {
    float w[8];
    load_pre_clip<CT>(a, base + c * 8, gi, w);
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
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wid] = mn;
    red[1][wid] = mx;
  }
  __syncthreads();
  mn = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
  mx = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  const float gmn = mn, gmx = mx;
  learnable<CT>(a, gi, mn, mx);
  float s, z;
  qparams_ct<CT>(mn, mx, a.qmin, a.qmax, a.sym, s, z);
  const float rs = 1.0f / s;
  const bool fin = mk_safe(gmn, gmx, s, rs);
  for (int64_t c = threadIdx.x; c < n8; c += blockDim.x) {
    float w[8], q[8], dq[8];
    load_pre_clip<CT>(a, base + c * 8, gi, w);
    if (fin) qdq8_mk<CT>(w, s, rs, z, a.qmin, a.qmax, q, dq);
    else qdq8<CT>(w, s, z, a.qmin, a.qmax, q, dq);
    emit<CT>(a, base + c * 8, q, dq);
  }
  if (threadIdx.x == 0) {
    if (a.s_out) st1<CT>(a.s_out, gi, s);
    if (a.z_out && !a.sym) st1<CT>(a.z_out, gi, z);
  }
}

// ---------------------------------------------------------------------------------------
// static qparams: element-parallel, compute dtype CT, input dtype XT
// ---------------------------------------------------------------------------------------
template <int XT, int CT>
__global__ void __launch_bounds__(256) k_quant_static(QuantArgs a) {
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t e0 = t * 8;
    const int64_t gi = a.qp_scalar ? 0 : e0 / a.group;
    float w[8];
    ld8<XT>(a.x, e0, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = rnd<CT>(w[j]);  // .to(compute dtype)
    float s = ld_rt(a.s_in, a.s_dt, gi);
    float z = a.z_in ? ld_rt(a.z_in, a.z_dt, gi) : 0.f;
    if (!a.qp_scalar) {  // tensor operands are converted to the compute dtype
      s = rnd<CT>(s);
      z = rnd<CT>(z);
    }
    float q[8], dq[8];
    if (a.nozp) {
      // scales.clamp_min(1e-9) in the scales' dtype, then the quotient + zeros rounded once
      // more before torch.round; dequant is the same (q - z) * s
      const float sc = rnd<CT>(round_dt(fmaxf(s, 1e-9f), a.s_dt));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = rintf(rnd<CT>(rnd<CT>(w[j] / sc) + z));
        t = fminf(fmaxf(t, a.qmin), a.qmax);
        q[j] = t;
        dq[j] = rnd<CT>(rnd<CT>(t - z) * s);
      }
    } else {
      qdq8<CT>(w, s, z, a.qmin, a.qmax, q, dq);
    }
    emit<CT>(a, e0, q, dq);
  }
}

// ---------------------------------------------------------------------------------------
// static qparams with a column -> group map (GPTQ act-order deploy, gptq.py:411-459):
// element (r, c) uses group r * ngc + cgroup[c]. With cgroup[c] = invperm[c] / group this is
// fake_quant_static(W[:, perm])[:, invperm] without the two column gathers (the same
// per-element arithmetic, so bit-identical). cols % 8 == 0.
// ---------------------------------------------------------------------------------------
template <int XT, int CT>
__global__ void __launch_bounds__(256) k_quant_static_cols(QuantArgs a, const int32_t* cgroup,
                                                           int64_t ngc) {
  const int64_t n8 = a.rows * a.cols / 8;
  const int64_t c8 = a.cols / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t r = t / c8, c0 = (t - r * c8) * 8;
    const int64_t e0 = t * 8;
    float w[8], q[8], dq[8];
    ld8<XT>(a.x, e0, w);
    const int4 ga = *reinterpret_cast<const int4*>(cgroup + c0);
    const int4 gb = *reinterpret_cast<const int4*>(cgroup + c0 + 4);
    const int g[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t gi = r * ngc + g[j];
      const float x = rnd<CT>(w[j]);  // .to(compute dtype)
      const float sc = rnd<CT>(ld_rt(a.s_in, a.s_dt, gi));
      const float z = a.z_in ? rnd<CT>(ld_rt(a.z_in, a.z_dt, gi)) : 0.f;
      float t1 = rintf(rnd<CT>(x / sc));
      t1 = rnd<CT>(t1 + z);
      t1 = fminf(fmaxf(t1, a.qmin), a.qmax);
      q[j] = t1;
      dq[j] = rnd<CT>(rnd<CT>(t1 - z) * sc);
    }
    emit<CT>(a, e0, q, dq);
  }
}

// ---------------------------------------------------------------------------------------
// standalone vLLM pack of integer codes (module_utils.py:929-955), incl. zero padding
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_pack_vllm(const void* codes, int dt, int64_t rows,
                                                   int64_t cols, int bits, uint32_t* out) {
  const int pf = 32 / bits;
  const int64_t pcols = (cols + pf - 1) / pf;
  const int64_t n = rows * pcols;
  const uint32_t off = 1u << (bits - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
    const int64_t r = t / pcols, pc = t % pcols;
    uint32_t w = 0;
    for (int i = 0; i < pf; ++i) {
      const int64_t c = pc * pf + i;
      uint32_t u = 0;  // np.pad(..., constant_values=0) pads AFTER the offset/uint8 step
      if (c < cols) u = ((uint32_t)(int)ld_rt(codes, dt, r * cols + c) + off) & 0xffu;
      w |= u << (bits * i);
    }
    out[t] = w;
  }
}

static bool pow2_le64(int64_t v) { return v >= 1 && v <= 64 && (v & (v - 1)) == 0; }

template <int CT>
static int launch_dyn(const QuantArgs& a, hipStream_t st) {
  const int64_t lanes = a.group / 8;
  const int64_t n8 = a.rows * a.cols / 8;
  if (pow2_le64(lanes)) {
    const unsigned grid = stream_grid(n8, 256);
    switch (lanes) {
      case 1: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 1>), grid, 256, 0, st, a); break;
      case 2: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 2>), grid, 256, 0, st, a); break;
      case 4: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 4>), grid, 256, 0, st, a); break;
      case 8: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 8>), grid, 256, 0, st, a); break;
      case 16: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 16>), grid, 256, 0, st, a); break;
      case 32: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 32>), grid, 256, 0, st, a); break;
      case 64: hipLaunchKernelGGL((k_quant_dyn_lanes<CT, 64>), grid, 256, 0, st, a); break;
    }
  } else {
    const int64_t ng = a.rows * a.cols / a.group;
    LCQ_REQUIRE(ng <= 0x7fffffffLL, "too many groups for the row kernel");
    hipLaunchKernelGGL((k_quant_dyn_rows<CT>), dim3((unsigned)ng), 256, 0, st, a);
  }
  return check_launch("lcq_int_quant_dynamic");
}

template <int XT>
static int launch_static_x(const QuantArgs& a, int ct, hipStream_t st) {
  const unsigned grid = stream_grid(a.rows * a.cols / 8, 256);
  switch (ct) {
    case LCQ_F32: hipLaunchKernelGGL((k_quant_static<XT, LCQ_F32>), grid, 256, 0, st, a); break;
    case LCQ_BF16: hipLaunchKernelGGL((k_quant_static<XT, LCQ_BF16>), grid, 256, 0, st, a); break;
    case LCQ_F16: hipLaunchKernelGGL((k_quant_static<XT, LCQ_F16>), grid, 256, 0, st, a); break;
    default: return fail(LCQ_EINVAL, "lcq_int_quant_static: bad compute dtype");
  }
  return check_launch("lcq_int_quant_static");
}

static int common_checks(const char* fn, int x_dtype, int64_t rows, int64_t cols,
                         int64_t& group, int qmin, int qmax, void* fq_out, int fq_dtype,
                         void* codes_out, int codes_dtype, void* packed_out, int pack_bits) {
  std::string f(fn);
  if (!is_float_dt(x_dtype)) return fail(LCQ_EINVAL, f + ": x dtype must be f32/f16/bf16");
  if (rows <= 0 || cols <= 0) return fail(LCQ_EINVAL, f + ": empty tensor");
  if (group <= 0) group = cols;
  if (cols % group != 0) return fail(LCQ_EINVAL, f + ": cols not divisible by group size");
  if (group % 8 != 0) return fail(LCQ_EINVAL, f + ": group size must be a multiple of 8");
  if (qmax <= qmin) return fail(LCQ_EINVAL, f + ": qmax <= qmin");
  if (fq_out && !is_float_dt(fq_dtype)) return fail(LCQ_EINVAL, f + ": bad fq dtype");
  if (codes_out && !is_code_dt(codes_dtype)) return fail(LCQ_EINVAL, f + ": bad codes dtype");
  if (packed_out && pack_bits != 4 && pack_bits != 8)
    return fail(LCQ_EUNSUP, f + ": pack_bits must be 4 or 8");
  return 0;
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_int_quant_dynamic(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                     int64_t group, const void* pre_scale, const void* clip_max,
                                     const void* clip_min, int qmin, int qmax, int sym,
                                     void* fq_out, int fq_dtype, void* codes_out,
                                     int codes_dtype, void* packed_out, int pack_bits,
                                     void* scales_out, void* zeros_out, void* stream) {
  int rc = common_checks("lcq_int_quant_dynamic", x_dtype, rows, cols, group, qmin, qmax,
                         fq_out, fq_dtype, codes_out, codes_dtype, packed_out, pack_bits);
  if (rc) return rc;
  QuantArgs a{};
  a.x = x; a.pre = pre_scale; a.cmax = clip_max; a.cmin = clip_min;
  a.rows = rows; a.cols = cols; a.group = group;
  a.qmin = (float)qmin; a.qmax = (float)qmax; a.sym = sym;
  a.fq = fq_out; a.fq_dt = fq_dtype; a.codes = codes_out; a.codes_dt = codes_dtype;
  a.packed = packed_out; a.pack_bits = pack_bits; a.s_out = scales_out; a.z_out = zeros_out;
  hipStream_t st = as_stream(stream);
  switch (x_dtype) {
    case LCQ_F32: return launch_dyn<LCQ_F32>(a, st);
    case LCQ_BF16: return launch_dyn<LCQ_BF16>(a, st);
    default: return launch_dyn<LCQ_F16>(a, st);
  }
}

extern "C" int lcq_int_quant_learnable(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                       int64_t group, const void* up, const void* low, int qmin,
                                       int qmax, int sym, void* fq_out, int fq_dtype,
                                       void* codes_out, int codes_dtype, void* scales_out,
                                       void* zeros_out, void* stream) {
  int rc = common_checks("lcq_int_quant_learnable", x_dtype, rows, cols, group, qmin, qmax,
                         fq_out, fq_dtype, codes_out, codes_dtype, nullptr, 0);
  if (rc) return rc;
  LCQ_REQUIRE(x_dtype == LCQ_BF16 || x_dtype == LCQ_F16, "learnable: bf16 / fp16 tensors");
  LCQ_REQUIRE(up != nullptr, "up factors required");
  QuantArgs a{};
  a.x = x; a.up = up; a.low = sym ? nullptr : low;
  a.rows = rows; a.cols = cols; a.group = group;
  a.qmin = (float)qmin; a.qmax = (float)qmax; a.sym = sym;
  a.fq = fq_out; a.fq_dt = fq_dtype; a.codes = codes_out; a.codes_dt = codes_dtype;
  a.s_out = scales_out; a.z_out = zeros_out;
  hipStream_t st = as_stream(stream);
  return x_dtype == LCQ_BF16 ? launch_dyn<LCQ_BF16>(a, st) : launch_dyn<LCQ_F16>(a, st);
}

static int int_quant_static(const char* fn, int nozp, const void* x, int x_dtype, int64_t rows,
                            int64_t cols, int64_t group, const void* scales, int s_dtype,
                            const void* zeros, int z_dtype, int ct_dtype, int qmin, int qmax,
                            void* fq_out, int fq_dtype, void* codes_out, int codes_dtype,
                            void* packed_out, int pack_bits, void* stream) {
  int rc = common_checks(fn, x_dtype, rows, cols, group, qmin, qmax,
                         fq_out, fq_dtype, codes_out, codes_dtype, packed_out, pack_bits);
  if (rc) return rc;
  LCQ_REQUIRE(scales != nullptr, "scales required");
  LCQ_REQUIRE(is_float_dt(s_dtype), "scales dtype must be float");
  LCQ_REQUIRE(zeros == nullptr || is_float_dt(z_dtype) || is_code_dt(z_dtype),
              "bad zeros dtype");
  LCQ_REQUIRE(is_float_dt(ct_dtype), "compute dtype must be float");
  QuantArgs a{};
  a.x = x; a.s_in = scales; a.s_dt = s_dtype; a.z_in = zeros; a.z_dt = z_dtype;
  a.rows = rows; a.cols = cols; a.group = group;
  a.qmin = (float)qmin; a.qmax = (float)qmax; a.sym = zeros == nullptr;
  a.fq = fq_out; a.fq_dt = fq_dtype; a.codes = codes_out; a.codes_dt = codes_dtype;
  a.packed = packed_out; a.pack_bits = pack_bits; a.nozp = nozp;
  hipStream_t st = as_stream(stream);
  switch (x_dtype) {
    case LCQ_F32: return launch_static_x<LCQ_F32>(a, ct_dtype, st);
    case LCQ_BF16: return launch_static_x<LCQ_BF16>(a, ct_dtype, st);
    default: return launch_static_x<LCQ_F16>(a, ct_dtype, st);
  }
}

extern "C" int lcq_int_quant_static(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                    int64_t group, const void* scales, int s_dtype,
                                    const void* zeros, int z_dtype, int ct_dtype, int qmin,
                                    int qmax, void* fq_out, int fq_dtype, void* codes_out,
                                    int codes_dtype, void* packed_out, int pack_bits,
                                    void* stream) {
  return int_quant_static("lcq_int_quant_static", 0, x, x_dtype, rows, cols, group, scales,
                          s_dtype, zeros, z_dtype, ct_dtype, qmin, qmax, fq_out, fq_dtype,
                          codes_out, codes_dtype, packed_out, pack_bits, stream);
}

extern "C" int lcq_int_quant_static_nozp(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                         int64_t group, const void* scales, int s_dtype,
                                         const void* zeros, int z_dtype, int ct_dtype, int qmin,
                                         int qmax, void* fq_out, int fq_dtype, void* codes_out,
                                         int codes_dtype, void* stream) {
  return int_quant_static("lcq_int_quant_static_nozp", 1, x, x_dtype, rows, cols, group, scales,
                          s_dtype, zeros, z_dtype, ct_dtype, qmin, qmax, fq_out, fq_dtype,
                          codes_out, codes_dtype, nullptr, 0, stream);
}

extern "C" int lcq_int_quant_static_scalar(const void* x, int x_dtype, int64_t rows,
                                           int64_t cols, const void* scale, const void* zero,
                                           int ct_dtype, int qmin, int qmax, void* fq_out,
                                           int fq_dtype, void* codes_out, int codes_dtype,
                                           void* stream) {
  int64_t group = cols;
  int rc = common_checks("lcq_int_quant_static_scalar", x_dtype, rows, cols, group, qmin, qmax,
                         fq_out, fq_dtype, codes_out, codes_dtype, nullptr, 0);
  if (rc) return rc;
  LCQ_REQUIRE(scale != nullptr, "scale required");
  LCQ_REQUIRE(is_float_dt(ct_dtype), "compute dtype must be float");
  QuantArgs a{};
  a.x = x; a.s_in = scale; a.s_dt = LCQ_F32; a.z_in = zero; a.z_dt = LCQ_F32;
  a.rows = rows; a.cols = cols; a.group = group; a.qp_scalar = 1;
  a.qmin = (float)qmin; a.qmax = (float)qmax; a.sym = zero == nullptr;
  a.fq = fq_out; a.fq_dt = fq_dtype; a.codes = codes_out; a.codes_dt = codes_dtype;
  hipStream_t st = as_stream(stream);
  switch (x_dtype) {
    case LCQ_F32: return launch_static_x<LCQ_F32>(a, ct_dtype, st);
    case LCQ_BF16: return launch_static_x<LCQ_BF16>(a, ct_dtype, st);
    default: return launch_static_x<LCQ_F16>(a, ct_dtype, st);
  }
}

extern "C" int lcq_pack_vllm(const void* codes, int codes_dtype, int64_t rows, int64_t cols,
                             int bits, void* packed_out, void* stream) {
  LCQ_REQUIRE(is_code_dt(codes_dtype), "codes dtype must be int8/uint8/int32");
  LCQ_REQUIRE(bits >= 1 && bits <= 8 && 32 % bits == 0, "bits must divide 32 and be <= 8");
  LCQ_REQUIRE(rows > 0 && cols > 0, "empty tensor");
  const int pf = 32 / bits;
  const int64_t n = rows * ((cols + pf - 1) / pf);
  hipLaunchKernelGGL(k_pack_vllm, stream_grid(n, 256), 256, 0, as_stream(stream), codes,
                     codes_dtype, rows, cols, bits, reinterpret_cast<uint32_t*>(packed_out));
  return check_launch("lcq_pack_vllm");
}

extern "C" int lcq_int_quant_static_cols(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                         const int32_t* col_group, int64_t ngc,
                                         const void* scales, int s_dtype, const void* zeros,
                                         int z_dtype, int ct_dtype, int qmin, int qmax,
                                         void* fq_out, int fq_dtype, void* codes_out,
                                         int codes_dtype, void* stream) {
  int64_t group = 8;  // only the shared shape / dtype checks apply here
  int rc = common_checks("lcq_int_quant_static_cols", x_dtype, rows, cols, group, qmin, qmax,
                         fq_out, fq_dtype, codes_out, codes_dtype, nullptr, 0);
  if (rc) return rc;
  LCQ_REQUIRE(cols % 8 == 0, "cols must be a multiple of 8");
  LCQ_REQUIRE(col_group != nullptr && ngc > 0 && scales != nullptr, "col_group / scales required");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(col_group) & 15) == 0, "col_group must be 16-byte aligned");
  LCQ_REQUIRE(is_float_dt(s_dtype), "scales dtype must be float");
  QuantArgs a{};
  a.x = x; a.s_in = scales; a.s_dt = s_dtype; a.z_in = zeros; a.z_dt = z_dtype;
  a.rows = rows; a.cols = cols; a.group = 0;
  a.qmin = (float)qmin; a.qmax = (float)qmax;
  a.fq = fq_out; a.fq_dt = fq_dtype; a.codes = codes_out; a.codes_dt = codes_dtype;
  hipStream_t st = as_stream(stream);
  const unsigned grid = stream_grid(rows * cols / 8, 256);
#define LCQ_SC(XT, CT) \
  hipLaunchKernelGGL((k_quant_static_cols<XT, CT>), grid, 256, 0, st, a, col_group, ngc)
#define LCQ_SC_X(XT)                                                         \
  switch (ct_dtype) {                                                        \
    case LCQ_F32: LCQ_SC(XT, LCQ_F32); break;                                \
    case LCQ_BF16: LCQ_SC(XT, LCQ_BF16); break;                              \
    case LCQ_F16: LCQ_SC(XT, LCQ_F16); break;                                \
    default: return fail(LCQ_EINVAL, "lcq_int_quant_static_cols: bad compute dtype"); \
  }
  switch (x_dtype) {
    case LCQ_F32: LCQ_SC_X(LCQ_F32); break;
    case LCQ_BF16: LCQ_SC_X(LCQ_BF16); break;
    default: LCQ_SC_X(LCQ_F16);
  }
#undef LCQ_SC_X
#undef LCQ_SC
  return check_launch("lcq_int_quant_static_cols");
}
