// GPTQ Hessian accumulation H = beta*H + alpha * X^T X on CDNA4 bf16/fp16 MFMA.
//
// Reference: GPTQ.add_batch (llmc/compression/quantization/gptq.py:253-295):
//   H *= n/(n+b); n += b; x = sqrt(2/n) * x.float(); H += x @ x.T
// Here x (bf16/fp16 calibration activations, token-major [n_tok, ic]) is consumed directly by
// v_mfma_f32_16x16x32_{bf16,f16} with fp32 accumulation (products of 16-bit inputs are exact
// in fp32); the sqrt(2/n)^2 factor is applied once as `alpha` in the epilogue. Only the upper
// triangle of 128x128 output tiles is computed (a symmetric rank-k update does half the
// FLOPs of the reference's full GEMM); each tile is written to H[i][j] and mirrored to H[j][i].
//
// Operand staging: both MFMA operands want 8 consecutive tokens (k) per lane, but x is
// token-major, so tiles are stored to LDS row-wise (coalesced 16-B global loads along the
// channel axis) and fragments are read with ds_read_b64_tr_b16 (hardware transpose, T10).
// The LDS image XOR-swizzles 8-byte chunks so the 32 lanes of a transposed read hit 64
// distinct banks.
#include "lcq_common.h"

namespace lcq {

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int HT = 128;  // output tile (rows = channels i, cols = channels j)
constexpr int HK = 32;   // tokens per k-step (one 16x16x32 MFMA deep)
constexpr int kRowBytes = HT * 2;

// byte offset of element (token row r, channel c) in a [HK][HT] 16-bit tile image
__device__ __forceinline__ int swz(int r, int c) {
  const int chunk = (c >> 2) ^ (((r & 3) << 2) | (((r >> 3) & 1) << 4));
  return r * kRowBytes + chunk * 8 + (c & 3) * 2;
}

// Operands are assembled with one whole-vector shuffle + bitcast: an element-wise
// bit_cast repack of the two transposed reads was mis-scheduled by hipcc (ROCm 7.2) into a
// duplicated first dword (observed in the .s), so keep this form.
template <bool FP16>
__device__ __forceinline__ v4f mfma(const v4s (&a)[2], const v4s (&b)[2], v4f c) {
  const v8s as = __builtin_shufflevector(a[0], a[1], 0, 1, 2, 3, 4, 5, 6, 7);
  const v8s bs = __builtin_shufflevector(b[0], b[1], 0, 1, 2, 3, 4, 5, 6, 7);
  if constexpr (FP16) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, as),
                                                  __builtin_bit_cast(v8h, bs), c, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, as),
                                                   __builtin_bit_cast(v8bf, bs), c, 0, 0, 0);
  }
}

// fragment of 16 channels x 32 tokens: lane (g = l>>4, i = l&15) gets channel c0+i at tokens
// 8g..8g+7 (two transposed reads of 4 tokens each)
__device__ __forceinline__ void load_frag(const char* tile, int c0, int lane, v4s (&f)[2]) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 8 * g + 4 * h + q;
    const char* a = tile + swz(r, c0 + 4 * p);
    f[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)(a));
  }
}

// global [HK tokens][HT channels] panel -> registers (2 x 16 B per thread, zero padded)
__device__ __forceinline__ void gload(const uint16_t* x, int64_t n, int64_t ic, int64_t t0,
                                      int64_t c0, int tid, uint4 (&r)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int idx = s * 256 + tid;      // 512 chunks of 8 channels
    const int row = idx >> 4, ch = (idx & 15) * 8;
    const int64_t t = t0 + row, c = c0 + ch;
    if (t < n && c < ic)
      r[s] = *reinterpret_cast<const uint4*>(x + t * ic + c);
    else
      r[s] = make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void lstore(char* tile, int tid, const uint4 (&r)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int idx = s * 256 + tid;
    const int row = idx >> 4, ch = (idx & 15) * 8;
    // 16 B = two 8-byte chunks (ch/4, ch/4+1); the XOR keeps the pair adjacent & ordered
    *reinterpret_cast<uint4*>(tile + swz(row, ch)) = r[s];
  }
}

template <bool FP16>
__global__ void __launch_bounds__(256)
    k_hessian_syrk(const uint16_t* __restrict__ x, int64_t n, int64_t ic, float* __restrict__ H,
                   float alpha, float beta, int nt) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][HK * kRowBytes];  // [buf][A/B]
  // upper-triangle tile (ti <= tj) of the nt x nt tile grid
  int b = blockIdx.x, ti = 0;
  while (b >= nt - ti) {
    b -= nt - ti;
    ++ti;
  }
  const int tj = ti + b;
  const bool diag = ti == tj;
  const int64_t i0 = (int64_t)ti * HT, j0 = (int64_t)tj * HT;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  v4f acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = v4f{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = (n + HK - 1) / HK;
  uint4 ra[2], rb[2];
  gload(x, n, ic, 0, i0, tid, ra);
  if (!diag) gload(x, n, ic, 0, j0, tid, rb);
  lstore(lds[0][0], tid, ra);
  if (!diag) lstore(lds[0][1], tid, rb);
  __syncthreads();

  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      gload(x, n, ic, (kt + 1) * HK, i0, tid, ra);
      if (!diag) gload(x, n, ic, (kt + 1) * HK, j0, tid, rb);
    }
    const char* ta = lds[cur][0];
    const char* tb = diag ? lds[cur][0] : lds[cur][1];
    v4s fa[4][2], fb[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) load_frag(ta, wr * 64 + m * 16, lane, fa[m]);
#pragma unroll
    for (int q = 0; q < 4; ++q) load_frag(tb, wc * 64 + q * 16, lane, fb[q]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[m][q] = mfma<FP16>(fa[m], fb[q], acc[m][q]);
    if (more) {
      lstore(lds[cur ^ 1][0], tid, ra);
      if (!diag) lstore(lds[cur ^ 1][1], tid, rb);
    }
    __syncthreads();
  }

  // epilogue: C/D layout of 16x16x32: col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t gi = i0 + wr * 64 + m * 16 + (lane >> 4) * 4;
      const int64_t gj = j0 + wc * 64 + q * 16 + (lane & 15);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t ii = gi + r;
        float a = __fmul_rn(alpha, acc[m][q][r]);
        if (ii < ic && gj < ic) {
          if (beta != 0.f) a = __fadd_rn(__fmul_rn(beta, H[ii * ic + gj]), a);
          H[ii * ic + gj] = a;
        }
        v[r] = a;
      }
      if (!diag && gj < ic) {  // mirror: H[gj][gi..gi+3] contiguous
        if (gi + 3 < ic) {
          *reinterpret_cast<float4*>(H + gj * ic + gi) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          for (int r = 0; r < 4; ++r)
            if (gi + r < ic) H[gj * ic + gi + r] = v[r];
        }
      }
    }
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_hessian_accum(const void* x, int x_dtype, int64_t n, int64_t ic, void* H,
                                 float alpha, float beta, void* stream) {
  LCQ_REQUIRE(x_dtype == LCQ_BF16 || x_dtype == LCQ_F16, "x must be bf16 or fp16");
  LCQ_REQUIRE(n > 0 && ic > 0, "empty input");
  LCQ_REQUIRE(ic % 8 == 0, "ic must be a multiple of 8");
  const int nt = (int)((ic + HT - 1) / HT);
  const unsigned tiles = (unsigned)(nt * (nt + 1) / 2);
  hipStream_t st = as_stream(stream);
  const uint16_t* xp = reinterpret_cast<const uint16_t*>(x);
  float* h = reinterpret_cast<float*>(H);
  if (x_dtype == LCQ_F16)
    hipLaunchKernelGGL((k_hessian_syrk<true>), dim3(tiles), 256, 0, st, xp, n, ic, h, alpha,
                       beta, nt);
  else
    hipLaunchKernelGGL((k_hessian_syrk<false>), dim3(tiles), 256, 0, st, xp, n, ic, h, alpha,
                       beta, nt);
  return check_launch("lcq_hessian_accum");
}
