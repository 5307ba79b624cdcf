// Block-scaled FP8 GEMM for FP8-weight (DeepSeek-V3-style) linears on gfx950 — the
// calibration forward of an fp8 checkpoint without a bf16 round trip of the weight.
//
// Replaces llmc/compression/quantization/kernel.py:141-242 (fp8_gemm, a Triton kernel) as
// called by block_wise_fp8_forward_func (module_utils.py:41-46):
//   C[m, n] = sum_kb ( sum_{k in block kb} A[m, k] B[n, k] ) * a_s[m, kb] * b_s[n / 128, kb]
// A [M, K] e4m3 (act_quant output, per-token 128-column scales a_s [M, K/128]); B [N, K] e4m3
// with 128x128 block scales b_s [ceil(N/128), K/128]; fp32 accumulation; C fp32 or bf16.
//
// Tile 128x128 per workgroup (4 waves, each 64x64 = 2x2 MFMA 32x32x16 fp8 tiles), one K block
// of 128 per step staged through LDS (16-byte global loads, padded rows); the block's partial
// dot products are scaled ((dot * a_s) * b_s, the reference's order) and accumulated in fp32.
#include "lcq_common.h"

namespace lcq {
namespace {

typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 128;
constexpr int LDA = BK + 16;  // padded LDS row (bytes): 16-byte aligned, offsets the banks

struct GemmArgs {
  const uint8_t* a;
  const float* as;
  const uint8_t* b;
  const float* bs;
  void* c;
  int64_t M, N, K;
  int c_dt;
};

__global__ __launch_bounds__(256) void k_fp8_gemm(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) uint8_t sa[BM * LDA];
  __shared__ __attribute__((aligned(16))) uint8_t sb[BN * LDA];
  __shared__ float sas[BM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const int64_t nkb = g.K / BK;
  const float* bsrow = g.bs + (n0 / 128) * nkb;
  v16f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int r_hi = lane >> 5, r_lo = lane & 31;
  for (int64_t kb = 0; kb < nkb; ++kb) {
    // stage A / B K-block tiles (128 rows x 128 bytes each; rows past M / N read as zeros)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int idx = p * 256 + tid;
      const int row = idx >> 3, ch = idx & 7;
      uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
      if (m0 + row < g.M)
        va = *reinterpret_cast<const uint4*>(g.a + (m0 + row) * g.K + kb * BK + ch * 16);
      if (n0 + row < g.N)
        vb = *reinterpret_cast<const uint4*>(g.b + (n0 + row) * g.K + kb * BK + ch * 16);
      *reinterpret_cast<uint4*>(sa + row * LDA + ch * 16) = va;
      *reinterpret_cast<uint4*>(sb + row * LDA + ch * 16) = vb;
    }
    if (tid < BM) sas[tid] = (m0 + tid < g.M) ? g.as[(m0 + tid) * nkb + kb] : 0.f;
    __syncthreads();
    v16f t[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      long fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        fa[i] = *reinterpret_cast<const long*>(sa + (64 * wm + 32 * i + r_lo) * LDA + 16 * ks +
                                               8 * r_hi);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[j] = *reinterpret_cast<const long*>(sb + (64 * wn + 32 * j + r_lo) * LDA + 16 * ks +
                                               8 * r_hi);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          t[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(fa[i], fb[j], t[i][j], 0, 0, 0);
    }
    // acc += (dot * a_s[m]) * b_s[n / 128]   (kernel.py: tl.dot(a, b) * a_s[:, None] * b_s)
    const float bsv = bsrow[kb];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float asv = sas[64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * r_hi];
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j][r] = acc[i][j][r] + (t[i][j][r] * asv) * bsv;
      }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + 64 * wn + 32 * j + r_lo;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * r_hi;
        if (m >= g.M) continue;
        if (g.c_dt == LCQ_F32) reinterpret_cast<float*>(g.c)[m * g.N + n] = acc[i][j][r];
        else st1<LCQ_BF16>(g.c, m * g.N + n, acc[i][j][r]);
      }
    }
}

}  // namespace
}  // namespace lcq

using namespace lcq;

extern "C" int lcq_fp8_gemm(const void* a, const void* a_s, const void* b, const void* b_s,
                            int64_t M, int64_t N, int64_t K, void* c, int c_dtype,
                            void* stream) {
  LCQ_REQUIRE(a && a_s && b && b_s && c, "null pointer");
  LCQ_REQUIRE(M > 0 && N > 0 && K > 0, "empty GEMM");
  LCQ_REQUIRE(K % 128 == 0, "K must be a multiple of 128 (the scale block)");
  LCQ_REQUIRE(c_dtype == LCQ_F32 || c_dtype == LCQ_BF16, "C dtype must be F32 or BF16");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(b) & 15) == 0,
              "A / B must be 16-byte aligned");
  GemmArgs g{static_cast<const uint8_t*>(a), static_cast<const float*>(a_s),
             static_cast<const uint8_t*>(b), static_cast<const float*>(b_s), c, M, N, K, c_dtype};
  dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM));
  k_fp8_gemm<<<grid, 256, 0, as_stream(stream)>>>(g);
  return check_launch("lcq_fp8_gemm");
}
