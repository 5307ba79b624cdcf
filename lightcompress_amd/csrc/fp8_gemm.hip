// Block-scaled FP8 GEMM for FP8-weight (DeepSeek-V3-style) linears on gfx950 — the
// calibration forward of an fp8 checkpoint without a bf16 round trip of the weight.
//
// Replaces llmc/compression/quantization/kernel.py:141-242 (fp8_gemm, a Triton kernel) as
// called by block_wise_fp8_forward_func (module_utils.py:41-46):
//   C[m, n] = sum_kb ( sum_{k in block kb} A[m, k] B[n, k] ) * a_s[m, kb] * b_s[n / 128, kb]
// A [M, K] e4m3 (act_quant output, per-token 128-column scales a_s [M, K/128]); B [N, K] e4m3
// with 128x128 block scales b_s [ceil(N/128), K/128]; fp32 accumulation; C fp32 or bf16.
//
// Tile 128x128 (or 64x128 when the grid would be small) per workgroup, 4 waves on gfx950's
// 32x32x64 f8f6f4 MFMA, one K block of 128 per step double-buffered through LDS (16-byte global
// loads into registers one block ahead, padded rows); the block's partial dot products are
// scaled ((dot * a_s) * b_s, the reference's order) and accumulated in fp32. Grids of fewer
// than 256 64-row tiles (short MoE / calibration batches) split K over blockIdx.z into fp32
// partials that a second kernel sums in split order (deterministic).
#include "lcq_common.h"

namespace lcq {
namespace {

typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v8i __attribute__((ext_vector_type(8)));

constexpr int BN = 128, BK = 128;
constexpr int LDA = BK + 16;  // padded LDS row (bytes): 16-byte aligned, offsets the banks

struct GemmArgs {
  const uint8_t* a;
  const float* as;
  const uint8_t* b;
  const float* bs;
  void* c;
  float* ws;  // split-K partials [splits, M, N] fp32, or null (one split, C written directly)
  int64_t M, N, K;
  int64_t kb_per_split;
  int c_dt;
};

// BM x 128 output tile per workgroup, 4 waves in a 2 x 2 grid, each (BM/2) x 64 of 32x32 MFMA
// tiles. K advances one 128-wide scale block at a time through two LDS buffers: the global
// loads of block kb+1 are issued into registers before block kb's MFMAs and written to the
// other buffer after them (one barrier per block). The MFMA is gfx950's 32x32x64 f8f6f4 form
// (e4m3 x e4m3, no block scale: twice the fp8 rate of 32x32x16); each lane feeds 32 consecutive
// k of its row to both operands, so the k order inside the instruction is the same for A and B.
template <int BM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_fp8_gemm(GemmArgs g) {
  constexpr int TI = BM / 64;          // 32-row MFMA tiles per wave
  constexpr int ACH = BM * 8 / 256;    // 16-byte A chunks per thread per block
  constexpr int BCH = BN * 8 / 256;
  __shared__ __attribute__((aligned(16))) uint8_t sa[2][BM * LDA];
  __shared__ __attribute__((aligned(16))) uint8_t sb[2][BN * LDA];
  __shared__ float sas[2][BM];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  // XCD-aware tile order: workgroup L runs on XCD L % 8, so hand each XCD a contiguous run of
  // tiles, walked in groups of 8 M-tiles (column-major inside a group) to share A / B in its L2
  const unsigned nx = gridDim.x, my = gridDim.y, total = nx * my;
  unsigned L = blockIdx.x + nx * blockIdx.y;
  if ((total & 7u) == 0) L = (L & 7u) * (total >> 3) + (L >> 3);
  const unsigned grp = L / (8u * nx), first = grp * 8u;
  const unsigned gsz = (my - first) < 8u ? (my - first) : 8u;
  const unsigned in = L - grp * 8u * nx;
  const int64_t m0 = (int64_t)(first + in % gsz) * BM, n0 = (int64_t)(in / gsz) * BN;
  const int64_t nkb = g.K / BK;
  const int64_t kb_begin = (int64_t)blockIdx.z * g.kb_per_split;
  const int64_t kb_end = kb_begin + g.kb_per_split < nkb ? kb_begin + g.kb_per_split : nkb;
  const float* bsrow = g.bs + (n0 / 128) * nkb;
  const int r_hi = lane >> 5, r_lo = lane & 31;

  uint4 ra[ACH], rb[BCH];
  float ras = 0.f;
  auto load = [&](int64_t kb) {
#pragma unroll
    for (int p = 0; p < ACH; ++p) {
      const int idx = p * 256 + tid, row = idx >> 3, ch = idx & 7;
      ra[p] = make_uint4(0, 0, 0, 0);
      if (m0 + row < g.M)
        ra[p] = *reinterpret_cast<const uint4*>(g.a + (m0 + row) * g.K + kb * BK + ch * 16);
    }
#pragma unroll
    for (int p = 0; p < BCH; ++p) {
      const int idx = p * 256 + tid, row = idx >> 3, ch = idx & 7;
      rb[p] = make_uint4(0, 0, 0, 0);
      if (n0 + row < g.N)
        rb[p] = *reinterpret_cast<const uint4*>(g.b + (n0 + row) * g.K + kb * BK + ch * 16);
    }
    if (tid < BM) ras = (m0 + tid < g.M) ? g.as[(m0 + tid) * nkb + kb] : 0.f;
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int p = 0; p < ACH; ++p) {
      const int idx = p * 256 + tid, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4*>(&sa[buf][row * LDA + ch * 16]) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < BCH; ++p) {
      const int idx = p * 256 + tid, row = idx >> 3, ch = idx & 7;
      *reinterpret_cast<uint4*>(&sb[buf][row * LDA + ch * 16]) = rb[p];
    }
    if (tid < BM) sas[buf][tid] = ras;
  };

  v16f acc[TI][2];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load(kb_begin);
  store(0);
  __syncthreads();
  for (int64_t kb = kb_begin; kb < kb_end; ++kb) {
    const int buf = (int)((kb - kb_begin) & 1);
    if (kb + 1 < kb_end) load(kb + 1);
    v16f t[TI][2];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t[i][j][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < BK / 64; ++ks) {
      v8i fa[TI], fb[2];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const uint8_t* p = &sa[buf][((BM / 2) * wm + 32 * i + r_lo) * LDA + 64 * ks + 32 * r_hi];
        const uint4 lo = *reinterpret_cast<const uint4*>(p);
        const uint4 hi = *reinterpret_cast<const uint4*>(p + 16);
        fa[i] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w,
                    (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint8_t* p = &sb[buf][(64 * wn + 32 * j + r_lo) * LDA + 64 * ks + 32 * r_hi];
        const uint4 lo = *reinterpret_cast<const uint4*>(p);
        const uint4 hi = *reinterpret_cast<const uint4*>(p + 16);
        fb[j] = v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w,
                    (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          t[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[i], fb[j], t[i][j], 0, 0,
                                                                    0, 0, 0, 0);
    }
    // acc += (dot * a_s[m]) * b_s[n / 128]   (kernel.py: tl.dot(a, b) * a_s[:, None] * b_s)
    const float bsv = bsrow[kb];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float asv = sas[buf][(BM / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * r_hi];
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j][r] = acc[i][j][r] + (t[i][j][r] * asv) * bsv;
      }
    if (kb + 1 < kb_end) store(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + 64 * wn + 32 * j + r_lo;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + (BM / 2) * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * r_hi;
        if (m >= g.M) continue;
        if (g.ws) g.ws[((int64_t)blockIdx.z * g.M + m) * g.N + n] = acc[i][j][r];
        else if (g.c_dt == LCQ_F32) reinterpret_cast<float*>(g.c)[m * g.N + n] = acc[i][j][r];
        else st1<LCQ_BF16>(g.c, m * g.N + n, acc[i][j][r]);
      }
    }
}

// Split-K epilogue: c = sum over splits in split order (deterministic), then the C dtype.
__global__ __launch_bounds__(256) void k_fp8_gemm_reduce(const float* __restrict__ ws,
                                                         int splits, int64_t mn, void* c,
                                                         int c_dt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < mn;
       i += (int64_t)gridDim.x * 256) {
    float v = ws[i];
    for (int z = 1; z < splits; ++z) v += ws[(int64_t)z * mn + i];
    if (c_dt == LCQ_F32) reinterpret_cast<float*>(c)[i] = v;
    else st1<LCQ_BF16>(c, i, v);
  }
}

// K splits for a short batch: a 64-row grid of fewer than 256 tiles is split along K until
// ~512 workgroups (two per CU at this kernel's occupancy) are in flight, keeping at least 4 K
// blocks per split.
int64_t gemm_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t nt = (N + BN - 1) / BN;
  if (((M + 127) / 128) * nt >= 512) return 1;
  const int64_t tiles = ((M + 63) / 64) * nt, nkb = K / BK;
  if (tiles >= 256) return 1;  // one workgroup per CU already: the partials' traffic costs more
  int64_t s = (512 + tiles - 1) / tiles;
  if (s > nkb / 4) s = nkb / 4;
  if (s < 2) return 1;
  const int64_t per = (nkb + s - 1) / s;
  return (nkb + per - 1) / per;  // no empty split
}

}  // namespace
}  // namespace lcq

using namespace lcq;

extern "C" int64_t lcq_fp8_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0) return 0;
  const int64_t s = gemm_splits(M, N, K);
  return s > 1 ? s * M * N * (int64_t)sizeof(float) : 0;
}

extern "C" int lcq_fp8_gemm(const void* a, const void* a_s, const void* b, const void* b_s,
                            int64_t M, int64_t N, int64_t K, void* c, int c_dtype,
                            void* workspace, int64_t ws_bytes, void* stream) {
  LCQ_REQUIRE(a && a_s && b && b_s && c, "null pointer");
  LCQ_REQUIRE(M > 0 && N > 0 && K > 0, "empty GEMM");
  LCQ_REQUIRE(K % 128 == 0, "K must be a multiple of 128 (the scale block)");
  LCQ_REQUIRE(c_dtype == LCQ_F32 || c_dtype == LCQ_BF16, "C dtype must be F32 or BF16");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(b) & 15) == 0,
              "A / B must be 16-byte aligned");
  const int64_t nkb = K / BK;
  int64_t splits = gemm_splits(M, N, K);
  if (!workspace || ws_bytes < splits * M * N * (int64_t)sizeof(float)) splits = 1;
  const int64_t per = (nkb + splits - 1) / splits;
  GemmArgs g{static_cast<const uint8_t*>(a), static_cast<const float*>(a_s),
             static_cast<const uint8_t*>(b), static_cast<const float*>(b_s), c,
             splits > 1 ? static_cast<float*>(workspace) : nullptr, M, N, K, per, c_dtype};
  // 128-row tiles unless that leaves most of the 256 CUs idle (short calibration batches)
  const int64_t nt = (N + BN - 1) / BN;
  if (splits == 1 && ((M + 127) / 128) * nt >= 512) {
    dim3 grid((unsigned)nt, (unsigned)((M + 127) / 128));
    k_fp8_gemm<128><<<grid, 256, 0, as_stream(stream)>>>(g);
  } else {
    dim3 grid((unsigned)nt, (unsigned)((M + 63) / 64), (unsigned)splits);
    k_fp8_gemm<64><<<grid, 256, 0, as_stream(stream)>>>(g);
  }
  if (splits > 1) {
    const int rc = check_launch("lcq_fp8_gemm");
    if (rc) return rc;
    const int64_t mn = M * N;
    int64_t blocks = (mn + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    k_fp8_gemm_reduce<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(
        static_cast<const float*>(workspace), (int)splits, mn, c, c_dtype);
  }
  return check_launch("lcq_fp8_gemm");
}
