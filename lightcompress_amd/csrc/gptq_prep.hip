// GPTQ act-order preparation without the ATen gathers (gptq.py:58-64, 128-176):
//
//   reference:  H[dead, dead] = 1; H = H[perm][:, perm]; H[d, d] += damp   (then the chain)
//               W[:, dead] = 0; W = W[:, perm]                (fp32 copy of the weight)
//   after:      W = W[:, invperm]
//
// One kernel, k_gather_rc: out[i][j] = f(A[rsrc[i]][csrc[j]]) with f = widen to fp32, zero a
// dead column (csrc[j] dead, the weight side), or on the diagonal (i == j) the dead fix (1)
// then + damp (the Hessian side). A workgroup stages the source row in LDS with coalesced loads
// and writes the output row in order (coalesced), the column gather served from LDS: one read
// and one write of the matrix, where the torch path runs a row gather, a column gather, a flip
// copy and a diagonal add (four reads and writes of the n^2 fp32 Hessian). The chain factors
// the reversed matrix J H J (gptq_core.prepare_hessian, reversal identity), so the Hessian
// call passes rsrc = csrc = perm reversed. Every output element is the same fp32 value as the
// torch path's (a copy, or the same single fp32 add on the diagonal). Rows wider than one LDS
// image (> 40960 fp32 columns: the 53248-wide down_proj of Llama-3.1-405B) take the same
// kernel with the column gather read straight from the source row (STAGED = false; the row,
// <= 46336 x 4 B, stays in L2 while the workgroup writes it).
#include "lcq_common.h"

namespace lcq {
namespace prep {

template <typename T>
__device__ __forceinline__ float widen(T v);
template <>
__device__ __forceinline__ float widen<float>(float v) { return v; }
template <>
__device__ __forceinline__ float widen<uint16_t>(uint16_t v) {  // bf16
  return __uint_as_float((uint32_t)v << 16);
}

template <typename T, bool STAGED>
__global__ void __launch_bounds__(256) k_gather_rc(const T* __restrict__ A, int64_t rows,
                                                   int64_t cols, int64_t lda,
                                                   const int64_t* __restrict__ rsrc,
                                                   const int64_t* __restrict__ csrc,
                                                   const uint8_t* __restrict__ dead_col,
                                                   const uint8_t* __restrict__ dead_diag,
                                                   const float* __restrict__ damp,
                                                   float* __restrict__ out, int64_t ldo) {
  extern __shared__ float row[];
  const float dv = damp ? *damp : 0.f;
  for (int64_t i = blockIdx.x; i < rows; i += gridDim.x) {
    const int64_t si = rsrc ? rsrc[i] : i;
    const T* a = A + si * lda;
    if constexpr (STAGED) {
      for (int64_t c = threadIdx.x; c < cols; c += blockDim.x) row[c] = widen<T>(a[c]);
      __syncthreads();
    }
    float* o = out + i * ldo;
    for (int64_t j = threadIdx.x; j < cols; j += blockDim.x) {
      const int64_t sj = csrc ? csrc[j] : j;
      float v = STAGED ? row[sj] : widen<T>(a[sj]);
      if (dead_col && dead_col[sj]) v = 0.f;
      if (i == j) {
        if (dead_diag && dead_diag[sj]) v = 1.f;
        if (damp) v = __fadd_rn(v, dv);
      }
      o[j] = v;
    }
    if constexpr (STAGED) __syncthreads();
  }
}

template <typename T>
static void launch_gather(const T* A, int64_t rows, int64_t cols, int64_t lda,
                          const int64_t* rsrc, const int64_t* csrc, const uint8_t* dead_col,
                          const uint8_t* dead_diag, const float* damp, float* out, int64_t ldo,
                          hipStream_t st) {
  const unsigned grid = (unsigned)(rows < 8192 ? rows : 8192);
  if (cols * 4 <= 160 * 1024) {
    const size_t lds = (size_t)cols * 4;
    auto k = k_gather_rc<T, true>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    hipLaunchKernelGGL(k, dim3(grid), 256, lds, st, A, rows, cols, lda, rsrc, csrc, dead_col,
                       dead_diag, damp, out, ldo);
  } else {
    hipLaunchKernelGGL((k_gather_rc<T, false>), dim3(grid), 256, 0, st, A, rows, cols, lda,
                       rsrc, csrc, dead_col, dead_diag, damp, out, ldo);
  }
}

}  // namespace prep
}  // namespace lcq

using namespace lcq;
using namespace lcq::prep;

extern "C" int lcq_gather_rc(const void* A, int a_dtype, int64_t rows, int64_t cols,
                             int64_t lda, const int64_t* rsrc, const int64_t* csrc,
                             const uint8_t* dead_col, const uint8_t* dead_diag,
                             const float* damp, void* out, int64_t ldo, void* stream) {
  LCQ_REQUIRE(a_dtype == LCQ_BF16 || a_dtype == LCQ_F32, "A must be bf16 or fp32");
  LCQ_REQUIRE(rows >= 0 && cols > 0 && lda >= cols && ldo >= cols, "bad shape");
  LCQ_REQUIRE(A != nullptr && out != nullptr && A != out, "A, out: distinct device buffers");
  if (rows == 0) return 0;
  hipStream_t st = as_stream(stream);
  if (a_dtype == LCQ_BF16)
    launch_gather(reinterpret_cast<const uint16_t*>(A), rows, cols, lda, rsrc, csrc, dead_col,
                  dead_diag, damp, reinterpret_cast<float*>(out), ldo, st);
  else
    launch_gather(reinterpret_cast<const float*>(A), rows, cols, lda, rsrc, csrc, dead_col,
                  dead_diag, damp, reinterpret_cast<float*>(out), ldo, st);
  return check_launch("lcq_gather_rc");
}
