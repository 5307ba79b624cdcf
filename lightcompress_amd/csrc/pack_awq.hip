// AutoAWQ "gemm" pack (AutoawqRealQuantLinear.gemm_pack, module_utils.py:1097-1158).
//
// The reference re-quantises every weight in fp32 from bf16 W and fp16 scales:
//   s16 = fp16(scales^T); sz = fp16(zeros^T * s16); iw[o,c] = int(round((W[o,c] + sz)/s16))
// WITHOUT a clamp, transposes to [IC, OC] and ORs nibbles `iw << 4i` (int32, raw bits) into
// words along OC in the order [0,2,4,6,1,3,5,7]. Out-of-range iw (e.g. -1, 16) therefore
// spill into neighbouring nibbles; that behaviour is reproduced bit for bit.
//
// Kernel: a 256-thread workgroup owns a 256(OC) x 64(IC) tile; the load phase reads 16-byte
// row segments (coalesced along IC), re-quantises and parks int32 codes in LDS; the store
// phase ORs 8 codes down the OC axis (the transpose) and writes 128-byte runs of qweight.
#include "lcq_common.h"

namespace lcq {

constexpr int kTileO = 256;
constexpr int kTileC = 64;
constexpr int kLdsStride = kTileC + 1;
__constant__ int kOrder[8] = {0, 2, 4, 6, 1, 3, 5, 7};

template <int WT>
__global__ void __launch_bounds__(256)
    k_awq_gemm_pack(const void* w, int64_t oc, int64_t ic, int64_t group, const void* scales,
                    int s_dt, const int32_t* zeros, uint32_t* qweight) {
  __shared__ int32_t tile[kTileO * kLdsStride];
  const int64_t ng = ic / group;
  const int64_t o0 = (int64_t)blockIdx.y * kTileO;
  const int64_t c0 = (int64_t)blockIdx.x * kTileC;
  const int tid = threadIdx.x;
  for (int it = 0; it < (kTileO * kTileC / 8) / 256; ++it) {
    const int chunk = it * 256 + tid;
    const int r = chunk / (kTileC / 8);
    const int c8 = chunk % (kTileC / 8);
    const int64_t o = o0 + r;
    const int64_t c = c0 + c8 * 8;
    if (o < oc && c < ic) {
      float v[8];
      ld8<WT>(w, o * ic + c, v);
      const int64_t g = c / group;
      float sraw = (s_dt == LCQ_BF16) ? ld1<LCQ_BF16>(scales, o * ng + g)
                   : (s_dt == LCQ_F16) ? ld1<LCQ_F16>(scales, o * ng + g)
                                       : ld1<LCQ_F32>(scales, o * ng + g);
      const float s16 = f16_rne(sraw);                          // scales.t().to(fp16)
      const float sz = f16_rne((float)zeros[o * ng + g] * s16);  // zeros * scales (fp16)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = rintf((v[j] + sz) / s16);  // fp32 (bf16 + fp16 promotes to fp32)
        tile[r * kLdsStride + c8 * 8 + j] = (int32_t)t;
      }
    }
  }
  __syncthreads();
  const int64_t pw_total = oc / 8;
  for (int it = 0; it < (kTileC * (kTileO / 8)) / 256; ++it) {
    const int wid = it * 256 + tid;
    const int cl = wid / (kTileO / 8);
    const int pw = wid % (kTileO / 8);
    const int64_t c = c0 + cl;
    const int64_t gpw = o0 / 8 + pw;
    if (c < ic && gpw < pw_total) {
      uint32_t word = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        word |= (uint32_t)tile[(pw * 8 + kOrder[i]) * kLdsStride + cl] << (4 * i);
      qweight[c * pw_total + gpw] = word;
    }
  }
}

// scales^T -> fp16 and qzeros pack (same nibble order), one thread per (group, packed word)
__global__ void __launch_bounds__(256)
    k_awq_pack_qparams(int64_t oc, int64_t ng, const void* scales, int s_dt,
                       const int32_t* zeros, _Float16* scales_t, uint32_t* qzeros) {
  const int64_t pw_total = oc / 8;
  const int64_t n = ng * pw_total;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
    const int64_t g = t / pw_total, pw = t % pw_total;
    uint32_t word = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t o = pw * 8 + kOrder[i];
      word |= (uint32_t)zeros[o * ng + g] << (4 * i);
    }
    qzeros[t] = word;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t o = pw * 8 + i;
      float sraw = (s_dt == LCQ_BF16) ? ld1<LCQ_BF16>(scales, o * ng + g)
                   : (s_dt == LCQ_F16) ? ld1<LCQ_F16>(scales, o * ng + g)
                                       : ld1<LCQ_F32>(scales, o * ng + g);
      scales_t[g * oc + o] = (_Float16)sraw;
    }
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_pack_autoawq_gemm(const void* w, int w_dtype, int64_t oc, int64_t ic,
                                     int64_t group, const void* scales, int s_dtype,
                                     const void* zeros, int bits, void* qweight_out,
                                     void* scales_t_out, void* qzeros_out, void* stream) {
  LCQ_REQUIRE(bits == 4, "Only 4-bit are supported for now.");
  LCQ_REQUIRE(is_float_dt(w_dtype) && is_float_dt(s_dtype), "float weight/scales required");
  LCQ_REQUIRE(oc > 0 && ic > 0 && oc % 8 == 0, "oc must be a positive multiple of 8");
  LCQ_REQUIRE(group > 0 && ic % group == 0 && group % 8 == 0, "bad group size");
  LCQ_REQUIRE(scales && zeros && qweight_out && scales_t_out && qzeros_out, "null buffer");
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)((ic + kTileC - 1) / kTileC), (unsigned)((oc + kTileO - 1) / kTileO));
  const int32_t* z = reinterpret_cast<const int32_t*>(zeros);
  uint32_t* qw = reinterpret_cast<uint32_t*>(qweight_out);
  switch (w_dtype) {
    case LCQ_BF16:
      hipLaunchKernelGGL((k_awq_gemm_pack<LCQ_BF16>), grid, 256, 0, st, w, oc, ic, group,
                         scales, s_dtype, z, qw);
      break;
    case LCQ_F16:
      hipLaunchKernelGGL((k_awq_gemm_pack<LCQ_F16>), grid, 256, 0, st, w, oc, ic, group,
                         scales, s_dtype, z, qw);
      break;
    default:
      hipLaunchKernelGGL((k_awq_gemm_pack<LCQ_F32>), grid, 256, 0, st, w, oc, ic, group,
                         scales, s_dtype, z, qw);
  }
  int rc = check_launch("lcq_pack_autoawq_gemm");
  if (rc) return rc;
  const int64_t ng = ic / group;
  hipLaunchKernelGGL(k_awq_pack_qparams, stream_grid(ng * (oc / 8), 256), 256, 0, st, oc, ng,
                     scales, s_dtype, z, reinterpret_cast<_Float16*>(scales_t_out),
                     reinterpret_cast<uint32_t*>(qzeros_out));
  return check_launch("lcq_pack_autoawq_gemm");
}
