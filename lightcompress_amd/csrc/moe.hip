// MoE routed-expert combine of the grouped block-fp8 expert forward (deepseekv3.ExpertList).
//
// Replaces the combine of the per-expert loop (reference models/deepseekv3.py MoE forward on
// the checkpoint's modeling code; transformers' DeepseekV3 expert loop): for every hit expert
// in ascending index, `out.index_add_(0, tok, (h_e * w[tok, pos]).to(out.dtype))`. Per token t
// and output column, that is
//   acc = 0; for the token's k slots in ascending expert id: acc = rnd(acc + rnd(y * w))
// with rnd = round to bf16 (nearest even), y the slot's expert output row (bf16) and w its
// routing weight (fp32 or bf16, the product in fp32). The expert outputs arrive in the grouped
// GEMM's expert-sorted row order: slot (t, j) is row slot_row[t k + j].
// One 256-thread workgroup per (token, 2048-column chunk), 8 columns per thread (16-byte
// loads and stores); the token's k slots are ordered once per workgroup (k <= 16, uniform).
// HBM-bound: reads the k expert rows once, writes the token's row once.
#define LCQ_BF16_HW 1  // conversion-instruction RNE (a NaN stays a NaN)
#include "lcq_common.h"

namespace lcq {
namespace {

constexpr int MAXK = 16;

template <int WDT>
__global__ __launch_bounds__(256) void k_moe_combine(const uint16_t* __restrict__ y,
                                                     const int64_t* __restrict__ slot_row,
                                                     const int64_t* __restrict__ expert,
                                                     const void* __restrict__ w, int64_t T,
                                                     int k, int64_t H,
                                                     uint16_t* __restrict__ out) {
  const int64_t t = blockIdx.x;
  const int64_t h0 = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 8;
  // the token's slots in ascending (expert id, slot) order: the loop adds the experts in
  // ascending index, and a repeated expert's slots in slot order (torch.where over its mask)
  int64_t rows[MAXK];
  float ws[MAXK];
  int cnt = 0;
  int64_t last_e = -1;
  int last_j = -1;
  for (int p = 0; p < k; ++p) {
    int best = -1;
    int64_t bid = 0;
    for (int j = 0; j < k; ++j) {
      const int64_t e = expert[t * k + j];
      const bool after = e > last_e || (e == last_e && j > last_j);
      if (after && (best < 0 || e < bid)) {
        best = j;
        bid = e;
      }
    }
    if (best < 0) break;
    last_e = bid;
    last_j = best;
    rows[cnt] = slot_row[t * k + best];
    if constexpr (WDT == LCQ_F32) ws[cnt] = reinterpret_cast<const float*>(w)[t * k + best];
    else ws[cnt] = __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(w)[t * k + best]
                                   << 16);
    ++cnt;
  }
  if (h0 >= H) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < cnt; ++s) {
    float v[8];
    ld8<LCQ_BF16>(y, rows[s] * H + h0, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = rnd<LCQ_BF16>(acc[i] + rnd<LCQ_BF16>(v[i] * ws[s]));
    }
  }
  st8<LCQ_BF16>(out, t * H + h0, acc);
}

}  // namespace
}  // namespace lcq

using namespace lcq;

extern "C" int lcq_moe_combine(const void* y, const int64_t* slot_row, const int64_t* expert,
                               const void* w, int w_dtype, int64_t T, int k, int64_t H,
                               void* out, void* stream) {
  LCQ_REQUIRE(T >= 0 && k > 0 && k <= MAXK && H > 0, "bad combine shape (k <= 16)");
  LCQ_REQUIRE(H % 8 == 0, "H must be a multiple of 8");
  LCQ_REQUIRE(w_dtype == LCQ_F32 || w_dtype == LCQ_BF16, "weights must be fp32 or bf16");
  if (T == 0) return LCQ_OK;
  LCQ_REQUIRE(y && slot_row && expert && w && out, "null pointer");
  LCQ_REQUIRE(T < ((int64_t)1 << 31) && H / 8 < 256 * 65535LL, "too many tokens / columns");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(out) & 15) == 0,
              "y / out must be 16-byte aligned");
  const dim3 grid((unsigned)T, (unsigned)((H / 8 + 255) / 256));
  hipStream_t st = as_stream(stream);
  if (w_dtype == LCQ_F32)
    hipLaunchKernelGGL(k_moe_combine<LCQ_F32>, grid, 256, 0, st,
                       static_cast<const uint16_t*>(y), slot_row, expert, w, T, k, H,
                       static_cast<uint16_t*>(out));
  else
    hipLaunchKernelGGL(k_moe_combine<LCQ_BF16>, grid, 256, 0, st,
                       static_cast<const uint16_t*>(y), slot_row, expert, w, T, k, H,
                       static_cast<uint16_t*>(out));
  return check_launch("lcq_moe_combine");
}
