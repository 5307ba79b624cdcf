// Deterministic pairwise (tree) sum of fp32 partials: out = alpha * tree(p_0 .. p_{np-1}).
//
// Used by the grouped GPTQ Hessian (gptq_core.HessianAccumulator): the calibration samples are
// cut into a fixed number of groups whose X^T X partials are summed in one fixed binary tree,
// ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)), so that N ranks holding contiguous
// power-of-two blocks of the groups (their local subtrees) and one GPU holding all of them
// produce the same fp32 bits (token-sharded GPTQ bit-identical to one GPU).
// Streaming, HBM-bound: np loads + 1 store of 16 B per lane per step.
#include "lcq_common.h"

namespace lcq {

constexpr int TREE_MAX = 8;

struct TreeArgs {
  const float* p[TREE_MAX];
  int np;
  int64_t n;
  float alpha;
  float* out;
};

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y), __fadd_rn(a.z, b.z),
                     __fadd_rn(a.w, b.w));
}

// the tree order of NP (1, 2, 4, 8) values, level by level (no recursion: a recursive helper
// is not inlined and spills v[] to scratch)
template <int NP>
__global__ void __launch_bounds__(256) k_tree_sum(TreeArgs a) {
  const int64_t n4 = a.n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) v[k] = reinterpret_cast<const float4*>(a.p[k])[i];
#pragma unroll
    for (int w = 1; w < NP; w *= 2)
#pragma unroll
      for (int k = 0; k < NP; k += 2 * w) v[k] = add4(v[k], v[k + w]);
    float4 s = v[0];
    if (a.alpha != 1.0f)
      s = make_float4(__fmul_rn(a.alpha, s.x), __fmul_rn(a.alpha, s.y),
                      __fmul_rn(a.alpha, s.z), __fmul_rn(a.alpha, s.w));
    reinterpret_cast<float4*>(a.out)[i] = s;
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_tree_sum(const void* const* parts, int np, int64_t n, float alpha, void* out,
                            void* stream) {
  LCQ_REQUIRE(parts != nullptr && out != nullptr, "null pointers");
  LCQ_REQUIRE(np == 1 || np == 2 || np == 4 || np == 8, "np must be 1, 2, 4 or 8");
  LCQ_REQUIRE(n > 0 && n % 4 == 0, "n must be a positive multiple of 4");
  TreeArgs a{};
  for (int k = 0; k < np; ++k) {
    LCQ_REQUIRE(parts[k] != nullptr && (reinterpret_cast<uintptr_t>(parts[k]) & 15) == 0,
                "partials must be 16-byte aligned");
    a.p[k] = reinterpret_cast<const float*>(parts[k]);
  }
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(out) & 15) == 0, "out must be 16-byte aligned");
  a.np = np;
  a.n = n;
  a.alpha = alpha;
  a.out = reinterpret_cast<float*>(out);
  const unsigned grid = stream_grid(n / 4, 256);
  hipStream_t st = as_stream(stream);
  switch (np) {
    case 1: hipLaunchKernelGGL(k_tree_sum<1>, grid, 256, 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_tree_sum<2>, grid, 256, 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_tree_sum<4>, grid, 256, 0, st, a); break;
    default: hipLaunchKernelGGL(k_tree_sum<8>, grid, 256, 0, st, a); break;
  }
  return check_launch("lcq_tree_sum");
}
