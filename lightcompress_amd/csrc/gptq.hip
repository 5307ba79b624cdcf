// GPTQ blocked OBS column loop for one 128-column block (gfx950, fp32 VALU).
//
// Reference: GPTQ.weight_transform (llmc/compression/quantization/gptq.py:198-244) with
// per-group qparams from search_column_qparams (:358-366 -> quant.py:545-559, fp32) and the
// fp32 quant_dequant (quant.py:699-717):
//   for i in block: if (i1+i) % g == 0: qparams <- minmax(W[:, i1+i : i1+i+g])  (block-start W)
//                   q = qdq(w_i); err = (w_i - q)/U[i,i]; W1[:, i:] -= err * U[i, i:]
//                   tmp[:, i] = w_i ; Losses[:, i] = (w_i - q)^2 / (2 U[i,i]^2)
// Every row is independent given U, so one lane owns one weight row and keeps the block's 128
// columns in registers; the 128x128 U block is staged once in LDS and read as wave-uniform
// broadcasts. The rank-1 updates use a separate multiply and subtract (no FMA contraction),
// which is exactly the reference's outer-product-then-subtract rounding, so the in-block loop
// is bit-exact given the same block-start W and U. The trailing update
// W[:, i2:] -= Err @ U[i1:i2, i2:] is a GEMM done by the caller.
#include "lcq_common.h"

namespace lcq {

constexpr int GB = 128;  // GPTQ blocksize (gptq.yml `blocksize: 128`)

struct GptqArgs {
  float* W;           // [rows, ld] fp32, permuted column space; block columns updated in place
  int64_t rows, ld, col0;
  int count;          // columns in this block (<= 128)
  const float* U;     // [ldu, ldu] upper Cholesky factor of H^-1 (permuted)
  int64_t ldu;
  float qmin, qmax;
  int sym;
  const float* s_in;  // per-row fixed qparams (per_channel) or NULL (per-group search)
  const float* z_in;
  float* s_out;       // [rows, ng_total] fp32 (group order = permuted column order)
  float* z_out;
  int64_t ng_total;
  float* err;         // [rows, 128]
  float* losses;      // optional [rows, ld]
};

template <int GS>
__global__ void __launch_bounds__(256) k_gptq_block(GptqArgs a) {
  __shared__ float u[GB * GB];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < GB * GB; idx += 256) {
    const int i = idx / GB, j = idx % GB;
    u[idx] = (i < a.count && j < a.count) ? a.U[(a.col0 + i) * a.ldu + a.col0 + j] : 0.f;
  }
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * 256 + tid;
  if (r >= a.rows) return;  // no barriers below
  float* wrow = a.W + r * a.ld + a.col0;
  float w[GB];
#pragma unroll
  for (int j = 0; j < GB; j += 4) {
    if (j + 3 < a.count) {
      float4 v = *reinterpret_cast<const float4*>(wrow + j);
      w[j] = v.x; w[j + 1] = v.y; w[j + 2] = v.z; w[j + 3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[j + k] = (j + k < a.count) ? wrow[j + k] : 0.f;
    }
  }
  // group qparams from the block-start weights (gptq.py:215-223 reads W, not W1)
  constexpr int NG = (GS > 0) ? GB / GS : 1;
  float qs[NG], qz[NG];
  if constexpr (GS > 0) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      float mn = w[g * GS], mx = w[g * GS];
#pragma unroll
      for (int j = 1; j < GS; ++j) {
        // a group truncated by the end of the quantized columns uses only its valid part
        if (g * GS + j < a.count) {
          mn = fminf(mn, w[g * GS + j]);
          mx = fmaxf(mx, w[g * GS + j]);
        }
      }
      qparams_f32(mn, mx, a.qmin, a.qmax, a.sym, qs[g], qz[g]);
      if (g * GS < a.count) {
        const int64_t gi = (a.col0 + g * GS) / GS;
        a.s_out[r * a.ng_total + gi] = qs[g];
        if (a.z_out && !a.sym) a.z_out[r * a.ng_total + gi] = qz[g];
      }
    }
  } else {
    qs[0] = a.s_in[r];
    qz[0] = a.z_in ? a.z_in[r] : 0.f;
  }
  float* erow = a.err + r * GB;
#pragma unroll
  for (int c = 0; c < GB; ++c) {
    if (c < a.count) {
      const float s = qs[(GS > 0) ? c / (GS > 0 ? GS : 1) : 0];
      const float z = qz[(GS > 0) ? c / (GS > 0 ? GS : 1) : 0];
      const float d = u[c * GB + c];
      const float wc = w[c];
      float t = rintf(wc / s);
      t = t + z;
      t = fminf(fmaxf(t, a.qmin), a.qmax);
      const float q = (t - z) * s;
      const float diff = wc - q;
      const float e = diff / d;
      wrow[c] = wc;  // tmp1[:, i] = w
      erow[c] = e;
      if (a.losses) a.losses[r * a.ld + a.col0 + c] = (diff * diff) / (2.f * (d * d));
#pragma unroll
      for (int j = c + 1; j < GB; ++j) w[j] = w[j] - e * u[c * GB + j];
    } else {
      erow[c] = 0.f;
    }
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_gptq_block(void* W, int64_t rows, int64_t ld, int64_t col0, int count,
                              const void* U, int64_t ldu, int64_t group, int qmin, int qmax,
                              int sym, const void* s_in, const void* z_in, void* s_out,
                              void* z_out, int64_t ng_total, void* err, void* losses,
                              void* stream) {
  LCQ_REQUIRE(rows > 0 && ld > 0 && count > 0 && count <= GB, "bad block shape");
  LCQ_REQUIRE(col0 >= 0 && col0 + count <= ld && col0 + count <= ldu, "block out of range");
  LCQ_REQUIRE(col0 % GB == 0, "col0 must be a multiple of the 128-column blocksize");
  LCQ_REQUIRE(qmax > qmin, "qmax <= qmin");
  GptqArgs a{};
  a.W = reinterpret_cast<float*>(W);
  a.rows = rows; a.ld = ld; a.col0 = col0; a.count = count;
  a.U = reinterpret_cast<const float*>(U); a.ldu = ldu;
  a.qmin = (float)qmin; a.qmax = (float)qmax; a.sym = sym;
  a.s_in = reinterpret_cast<const float*>(s_in);
  a.z_in = reinterpret_cast<const float*>(z_in);
  a.s_out = reinterpret_cast<float*>(s_out);
  a.z_out = reinterpret_cast<float*>(z_out);
  a.ng_total = ng_total;
  a.err = reinterpret_cast<float*>(err);
  a.losses = reinterpret_cast<float*>(losses);
  const dim3 grid((unsigned)((rows + 255) / 256));
  hipStream_t st = as_stream(stream);
  switch (group) {
    case 32: hipLaunchKernelGGL((k_gptq_block<32>), grid, 256, 0, st, a); break;
    case 64: hipLaunchKernelGGL((k_gptq_block<64>), grid, 256, 0, st, a); break;
    case 128: hipLaunchKernelGGL((k_gptq_block<128>), grid, 256, 0, st, a); break;
    case 0:
      LCQ_REQUIRE(s_in != nullptr, "fixed-qparams mode needs s_in");
      hipLaunchKernelGGL((k_gptq_block<0>), grid, 256, 0, st, a);
      break;
    default: return fail(LCQ_EUNSUP, "lcq_gptq_block: group size must be 32, 64 or 128");
  }
  return check_launch("lcq_gptq_block");
}

// ---------------------------------------------------------------------------------------
// GPTQ trailing update  W[:, c1:] -= E[:, :cnt] @ U[c0:c0+cnt, c1:]   (gptq.py:244)
// fp32 MFMA v_mfma_f32_32x32x2_f32: bit-for-bit a k-ordered fmaf chain, so every output
// element's value is independent of the tiling / row range (row-sharded GPTQ on N GPUs is
// bit-identical to one GPU). The product is rounded to fp32 and then subtracted, like the
// reference's `W -= Err @ Hinv` (two roundings). 128x128 tile per 256-thread workgroup,
// 2x2 waves of 64x64 = 2x2 MFMA 32x32 tiles, K staged through LDS 32 at a time.
// ---------------------------------------------------------------------------------------
namespace lcq {

typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int TT = 128;   // output tile
constexpr int TK = 32;    // k chunk

__global__ void __launch_bounds__(256)
    k_gptq_trailing(float* __restrict__ W, int64_t rows, int64_t ld, int64_t c0, int cnt,
                    int64_t c1, const float* __restrict__ E, const float* __restrict__ U,
                    int64_t ldu) {
  __shared__ float As[TK][TT];  // As[k][row]
  __shared__ float Bs[TK][TT];  // Bs[k][col]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t r0 = (int64_t)blockIdx.y * TT;
  const int64_t j0 = c1 + (int64_t)blockIdx.x * TT;
  v16f acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  for (int k0 = 0; k0 < GB; k0 += TK) {
    __syncthreads();
    // E tile: 128 rows x 32 k, float4 along k, stored transposed As[k][row]
#pragma unroll
    for (int it = 0; it < (TT * TK / 4) / 256; ++it) {
      const int idx = it * 256 + tid;
      const int row = idx / (TK / 4), k4 = (idx % (TK / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r0 + row < rows) v = *reinterpret_cast<const float4*>(E + (r0 + row) * GB + k0 + k4);
      As[k4 + 0][row] = (k0 + k4 + 0 < cnt) ? v.x : 0.f;
      As[k4 + 1][row] = (k0 + k4 + 1 < cnt) ? v.y : 0.f;
      As[k4 + 2][row] = (k0 + k4 + 2 < cnt) ? v.z : 0.f;
      As[k4 + 3][row] = (k0 + k4 + 3 < cnt) ? v.w : 0.f;
    }
    // U tile: 32 k x 128 cols, float4 along cols
#pragma unroll
    for (int it = 0; it < (TT * TK / 4) / 256; ++it) {
      const int idx = it * 256 + tid;
      const int k = idx / (TT / 4), c4 = (idx % (TT / 4)) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k0 + k < cnt) {
        const float* src = U + (c0 + k0 + k) * ldu + j0 + c4;
        if (j0 + c4 + 3 < ld) {
          v = *reinterpret_cast<const float4*>(src);
        } else {
          if (j0 + c4 + 0 < ld) v.x = src[0];
          if (j0 + c4 + 1 < ld) v.y = src[1];
          if (j0 + c4 + 2 < ld) v.z = src[2];
        }
      }
      *reinterpret_cast<float4*>(&Bs[k][c4]) = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; kk += 2) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = As[kk + (lane >> 5)][wr * 64 + t * 32 + (lane & 31)];
        b[t] = Bs[kk + (lane >> 5)][wc * 64 + t * 32 + (lane & 31)];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb)
          acc[ta][tb] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
  }
  // epilogue (C layout: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5))
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int64_t r = r0 + wr * 64 + ta * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        const int64_t c = j0 + wc * 64 + tb * 32 + (lane & 31);
        if (r < rows && c < ld) W[r * ld + c] = W[r * ld + c] - acc[ta][tb][reg];
      }
}

}  // namespace lcq

extern "C" int lcq_gptq_trailing(void* W, int64_t rows, int64_t ld, int64_t c0, int cnt,
                                 int64_t c1, const void* err, const void* U, int64_t ldu,
                                 void* stream) {
  LCQ_REQUIRE(rows > 0 && ld > 0 && cnt > 0 && cnt <= GB, "bad shape");
  LCQ_REQUIRE(c0 >= 0 && c0 + cnt <= ldu && c1 >= c0 + cnt && c1 <= ld && ld <= ldu,
              "bad column ranges");
  if (c1 == ld) return LCQ_OK;
  const dim3 grid((unsigned)((ld - c1 + TT - 1) / TT), (unsigned)((rows + TT - 1) / TT));
  hipLaunchKernelGGL(k_gptq_trailing, grid, 256, 0, as_stream(stream),
                     reinterpret_cast<float*>(W), rows, ld, c0, cnt, c1,
                     reinterpret_cast<const float*>(err), reinterpret_cast<const float*>(U),
                     ldu);
  return check_launch("lcq_gptq_trailing");
}
