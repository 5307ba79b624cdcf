// Diagonal-tile kernel of the recursive fp32 Cholesky / triangular inverse behind GPTQ's
// U = chol(H^-1, upper) (gptq.py:169-174; computed as J chol(J H J)^-1 J, see gptq_core).
// The recursion (host side) does the large updates as fp32 GEMMs; this kernel factors a
// <= 128 x 128 diagonal tile and inverts its factor, in one workgroup with both in LDS.
//
// Right-looking over PW-column panels on the augmented [A | R], R = I initially; after panel P
// R's rows P hold X_P = L_PP^-1 R_P, the rows of L^-1 (blocked forward substitution of L X = I):
//   S1 (one wave, registers): every lane factors the whole PW x PW diagonal block redundantly
//      in its own registers (no cross-lane traffic, no barriers), then lane j computes column
//      j of Z = L_PP^-1;
//   S2 (threads 0-127) X_P = Z R_P, one thread per column; (threads 128-255)
//      L_below = A_below Z^T, one thread per row;
//   S3 (all threads, two tile loops): A22 -= L_below L_below^T (lower) and
//      R_below -= L_below X_P, 4x4 register tiles with every LDS read issued before the FMAs.
// Two barriers per panel; nothing leaves LDS until the end. Only X = L^-1 is needed by the
// recursion (gptq_core._chol_inv_rec); L is written back only when asked for (L may alias A:
// every read of A precedes the first barrier, every write of L follows the last).
// Measured (scripts/probes/chol_tile_prof.py, one 128-tile): PW 16 / 256 threads 70 us, PW 8 /
// 256 threads 60 us, PW 8 / 1024 threads 51 us (PW 4 / 1024 threads in the n 14336 chain: 84 us
// against 64 per tile, twice the barriers; profiles/r4_chain_breakdown.txt) -- S1 is VALU-bound
// in one wave at ~PW^3/6 FMAs
// per panel, S3 is LDS-latency-bound; what remains is the S1 -> S2 -> S3 chain per panel.
#include "lcq_common.h"

namespace lcq {

constexpr int CTILE = 128;
constexpr int CLD = CTILE + 4;  // LDS row pitch: 16-byte aligned rows (ds_read_b128 of row
                                // segments); 132 = 4 mod 64 banks, 16 rows per bank sweep
#ifndef LCQ_CHOL_PW
#define LCQ_CHOL_PW 8
#endif
constexpr int PW = LCQ_CHOL_PW;  // panel width
#ifndef LCQ_CHOL_NT
#define LCQ_CHOL_NT 1024
#endif
constexpr int NT = LCQ_CHOL_NT;  // threads; > 256 hides the LDS latency of the S3 tiles
constexpr int VEC_PER_THREAD = CTILE * CTILE / 4 / NT;

#ifdef LCQ_CHOL_PROF  // probe builds only (scripts/probes/chol_tile_prof.py): stage timestamps
#define PROF_STAMP(k)                                                                 \
  if (threadIdx.x == 0)                                                               \
    reinterpret_cast<unsigned long long*>(info)[1 + (k)] = __builtin_amdgcn_s_memtime();
#else
#define PROF_STAMP(k)
#endif

// lower-triangle 4x4 tile index t -> (ti, tk), tk <= ti
__device__ __forceinline__ void tri_tile(int t, int& ti, int& tk) {
  ti = (int)((__builtin_amdgcn_sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);  // corrected below
  while (ti * (ti + 1) / 2 > t) --ti;
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  tk = t - ti * (ti + 1) / 2;
}

// S1: factor a[c0:c0+cw, c0:c0+cw] (lower) in every lane's registers; lane 0 writes L_PP back,
// lanes < PW write column `lane` of Z = L_PP^-1 to zs[r*PW+lane]. Returns the first bad pivot
// (1-based within the block) or 0 -- uniform.
__device__ __forceinline__ int factor_diag(float* a, float* zs, int c0, int cw, int lane) {
  float l[PW][PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const float4* row = reinterpret_cast<const float4*>(a + (c0 + i) * CLD + c0);
#pragma unroll
    for (int q = 0; q < PW / 4; ++q) {
      if (4 * q <= i) {
        const float4 v = row[q];  // broadcast: every lane reads the same address
        l[i][4 * q] = v.x;
        l[i][4 * q + 1] = v.y;
        l[i][4 * q + 2] = v.z;
        l[i][4 * q + 3] = v.w;
      }
    }
    if (i >= cw) {  // rows past the tile edge: identity, keeps the unrolled code finite
#pragma unroll
      for (int k = 0; k < PW; ++k) l[i][k] = (k == i) ? 1.f : 0.f;
    }
  }
  float rinv[PW];
  int bad = 0;
#pragma unroll
  for (int c = 0; c < PW; ++c) {
    const float d = l[c][c];
    const bool nb = !(d > 0.f);
    if (nb && bad == 0) bad = c + 1;
    const float sq = nb ? 1.f : sqrtf(d);
    rinv[c] = 1.f / sq;
    l[c][c] = sq;
#pragma unroll
    for (int i = c + 1; i < PW; ++i) l[i][c] *= rinv[c];
#pragma unroll
    for (int i = c + 1; i < PW; ++i)
#pragma unroll
      for (int k = c + 1; k <= i; ++k) l[i][k] = fmaf(-l[i][c], l[k][c], l[i][k]);
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < PW; ++i)
      if (i < cw)
#pragma unroll
        for (int k = 0; k <= i; ++k) a[(c0 + i) * CLD + c0 + k] = l[i][k];
  }
  // Z column `lane`: z[r] = (e_lane[r] - sum_{q<r} L[r][q] z[q]) / L[r][r]
  float z[PW];
#pragma unroll
  for (int r = 0; r < PW; ++r) {
    float sacc = (lane == r) ? 1.f : 0.f;
#pragma unroll
    for (int q = 0; q < r; ++q) sacc = fmaf(-l[r][q], z[q], sacc);
    z[r] = sacc * rinv[r];
  }
  if (lane < PW) {
#pragma unroll
    for (int r = 0; r < PW; ++r) zs[r * PW + lane] = (r < cw && lane < cw) ? z[r] : 0.f;
  }
  return bad;
}

// S3 tile: rows i0..i0+3 of L_below (panel columns c0..c0+PW-1) times either rows k0..k0+3 of
// the panel (LOWER: A22 tile, lower part only) or X_P[:, k0..k0+3] (R tile); all b128
// reads are issued before any FMA
template <bool LOWER>
__device__ __forceinline__ void rank_tile(float* a, float* x, int c0, int i0, int k0, int n) {
  float4 pi[4][PW / 4], pk[4][PW / 4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int q = 0; q < PW / 4; ++q)
      pi[u][q] = *reinterpret_cast<const float4*>(a + (i0 + u) * CLD + c0 + 4 * q);
  if (LOWER) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < PW / 4; ++q)
        pk[u][q] = *reinterpret_cast<const float4*>(a + (k0 + u) * CLD + c0 + 4 * q);
  } else {
    // pk[v][q].{x,y,z,w} = X[c0+4q+{0..3}][k0+v], from X rows (k0..k0+3 contiguous)
#pragma unroll
    for (int q = 0; q < PW / 4; ++q) {
      const float4 r0 = *reinterpret_cast<const float4*>(x + (c0 + 4 * q) * CLD + k0);
      const float4 r1 = *reinterpret_cast<const float4*>(x + (c0 + 4 * q + 1) * CLD + k0);
      const float4 r2 = *reinterpret_cast<const float4*>(x + (c0 + 4 * q + 2) * CLD + k0);
      const float4 r3 = *reinterpret_cast<const float4*>(x + (c0 + 4 * q + 3) * CLD + k0);
      pk[0][q] = make_float4(r0.x, r1.x, r2.x, r3.x);
      pk[1][q] = make_float4(r0.y, r1.y, r2.y, r3.y);
      pk[2][q] = make_float4(r0.z, r1.z, r2.z, r3.z);
      pk[3][q] = make_float4(r0.w, r1.w, r2.w, r3.w);
    }
  }
  float acc[4][4] = {};
#pragma unroll
  for (int q = 0; q < PW / 4; ++q)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        acc[u][v] = fmaf(pi[u][q].x, pk[v][q].x, acc[u][v]);
        acc[u][v] = fmaf(pi[u][q].y, pk[v][q].y, acc[u][v]);
        acc[u][v] = fmaf(pi[u][q].z, pk[v][q].z, acc[u][v]);
        acc[u][v] = fmaf(pi[u][q].w, pk[v][q].w, acc[u][v]);
      }
  float* dst = LOWER ? a : x;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = i0 + u, k = k0 + v;
      if (i < n && (!LOWER || k <= i)) dst[i * CLD + k] -= acc[u][v];
    }
}

__global__ void __launch_bounds__(NT) k_chol_inv_tile(const float* A, int64_t lda,
                                                       int n, float* Lout,
                                                       int64_t ldl, float* __restrict__ X,
                                                       int64_t ldx, int* __restrict__ info,
                                                       int64_t row0, int vec) {
  __shared__ __attribute__((aligned(16))) float a[CTILE * CLD];
  __shared__ __attribute__((aligned(16))) float x[CTILE * CLD];
  __shared__ __attribute__((aligned(16))) float zs[PW * PW];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  PROF_STAMP(0)
  if (vec) {  // n == 128, lda % 4 == 0, 16-byte aligned: one batch of float4 loads per thread
    float4 v[VEC_PER_THREAD];
#pragma unroll
    for (int u = 0; u < VEC_PER_THREAD; ++u) {
      const int e = tid + NT * u, i = e >> 5, j = (e & 31) * 4;
      v[u] = *reinterpret_cast<const float4*>(A + (int64_t)i * lda + j);
    }
#pragma unroll
    for (int u = 0; u < VEC_PER_THREAD; ++u) {
      const int e = tid + NT * u, i = e >> 5, j = (e & 31) * 4;
      *reinterpret_cast<float4*>(a + i * CLD + j) = v[u];
    }
  } else {
#pragma unroll
    for (int it0 = 0; it0 < CTILE * CTILE / NT; it0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int idx = tid + NT * (it0 + u), i = idx >> 7, j = idx & 127;
        v[u] = (i < n && j < n) ? A[(int64_t)i * lda + j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int idx = tid + NT * (it0 + u), i = idx >> 7, j = idx & 127;
        a[i * CLD + j] = v[u];
      }
    }
  }
  for (int idx = tid; idx < CTILE * CTILE; idx += NT) {
    const int i = idx >> 7, j = idx & 127;
    x[i * CLD + j] = (i == j) ? 1.f : 0.f;
  }
  __syncthreads();
  PROF_STAMP(1)

  for (int c0 = 0; c0 < n; c0 += PW) {
    const int cw = min(PW, n - c0);
    const int b0 = c0 + PW, m2 = n - b0;
    if (wave == 0) {
      const int bad = factor_diag(a, zs, c0, cw, lane);
      if (bad && lane == 0 && info) atomicCAS(info, 0, (int)(row0 + c0 + bad));
    }
    PROF_STAMP(2 + 4 * (c0 / PW))
    __syncthreads();
    if (tid < 128) {
      // X_P = Z R_P for column j (columns >= c0 + cw of R_P are zero)
      const int j = tid;
      if (j < c0 + cw) {
        float rp[PW], t[PW];
#pragma unroll
        for (int q = 0; q < PW; ++q) rp[q] = (q < cw) ? x[(c0 + q) * CLD + j] : 0.f;
#pragma unroll
        for (int r = 0; r < PW; ++r) {
          const float4* z4 = reinterpret_cast<const float4*>(zs + r * PW);
          float sacc = 0.f;
#pragma unroll
          for (int q4 = 0; q4 < PW / 4; ++q4) {
            const float4 zz = z4[q4];
            sacc = fmaf(zz.x, rp[4 * q4], sacc);
            sacc = fmaf(zz.y, rp[4 * q4 + 1], sacc);
            sacc = fmaf(zz.z, rp[4 * q4 + 2], sacc);
            sacc = fmaf(zz.w, rp[4 * q4 + 3], sacc);
          }
          t[r] = sacc;
        }
#pragma unroll
        for (int r = 0; r < PW; ++r)
          if (r < cw) x[(c0 + r) * CLD + j] = t[r];
      }
    } else if (m2 > 0) {
      // L_below row i = A row i (panel columns) Z^T
      const int i = b0 + tid - 128;
      if (i < n) {
        float ar[PW];
#pragma unroll
        for (int q = 0; q < PW / 4; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(a + i * CLD + c0 + 4 * q);
          ar[4 * q] = v.x;
          ar[4 * q + 1] = v.y;
          ar[4 * q + 2] = v.z;
          ar[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int c = 0; c < PW; ++c) {
          const float4* z4 = reinterpret_cast<const float4*>(zs + c * PW);
          float sacc = 0.f;
#pragma unroll
          for (int q4 = 0; q4 < PW / 4; ++q4) {
            const float4 zz = z4[q4];
            sacc = fmaf(zz.x, ar[4 * q4], sacc);
            sacc = fmaf(zz.y, ar[4 * q4 + 1], sacc);
            sacc = fmaf(zz.z, ar[4 * q4 + 2], sacc);
            sacc = fmaf(zz.w, ar[4 * q4 + 3], sacc);
          }
          a[i * CLD + c0 + c] = sacc;
        }
      }
    }
    PROF_STAMP(3 + 4 * (c0 / PW))
    __syncthreads();
    PROF_STAMP(4 + 4 * (c0 / PW))
    if (m2 > 0) {
      // S3: tiles of A22 (lower) then tiles of R_below (columns < c0 + PW); rows stay < 128
      const int nt = (m2 + 3) >> 2, T = nt * (nt + 1) / 2, nc = (c0 + PW) >> 2;
      int t = tid;
      for (; t < T; t += NT) {
        int ti, tk;
        tri_tile(t, ti, tk);
        rank_tile<true>(a, x, c0, b0 + 4 * ti, b0 + 4 * tk, n);
      }
      for (; t < T + nt * nc; t += NT) {
        const int t2 = t - T;
        rank_tile<false>(a, x, c0, b0 + 4 * (t2 / nc), 4 * (t2 % nc), n);
      }
    }
    PROF_STAMP(5 + 4 * (c0 / PW))
    __syncthreads();
  }
  PROF_STAMP(70)

  if (vec) {
#pragma unroll
    for (int u = 0; u < VEC_PER_THREAD; ++u) {
      const int e = tid + NT * u, i = e >> 5, j = (e & 31) * 4;
      float4 o = *reinterpret_cast<const float4*>(x + i * CLD + j);
      if (j > i) o.x = 0.f;
      if (j + 1 > i) o.y = 0.f;
      if (j + 2 > i) o.z = 0.f;
      if (j + 3 > i) o.w = 0.f;
      *reinterpret_cast<float4*>(X + (int64_t)i * ldx + j) = o;
      if (Lout) {
        o = *reinterpret_cast<const float4*>(a + i * CLD + j);
        if (j > i) o.x = 0.f;
        if (j + 1 > i) o.y = 0.f;
        if (j + 2 > i) o.z = 0.f;
        if (j + 3 > i) o.w = 0.f;
        *reinterpret_cast<float4*>(Lout + (int64_t)i * ldl + j) = o;
      }
    }
  } else {
#pragma unroll 8
    for (int it = 0; it < CTILE * CTILE / NT; ++it) {
      const int idx = tid + NT * it, i = idx >> 7, j = idx & 127;
      if (i < n && j < n) {
        X[(int64_t)i * ldx + j] = (j <= i) ? x[i * CLD + j] : 0.f;
        if (Lout) Lout[(int64_t)i * ldl + j] = (j <= i) ? a[i * CLD + j] : 0.f;
      }
    }
  }
  PROF_STAMP(71)
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_chol_inv_tile(const void* A, int64_t lda, int n, void* L, int64_t ldl,
                                 void* X, int64_t ldx, void* info, int64_t row0, void* stream) {
  LCQ_REQUIRE(n > 0 && n <= CTILE && lda >= n && ldx >= n && (!L || ldl >= n),
              "tile must be 1..128 wide");
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec = n == CTILE && lda % 4 == 0 && ldx % 4 == 0 && al(A) && al(X) &&
                  (!L || (ldl % 4 == 0 && al(L)));
  hipLaunchKernelGGL(k_chol_inv_tile, dim3(1), NT, 0, as_stream(stream),
                     reinterpret_cast<const float*>(A), lda, n, reinterpret_cast<float*>(L), ldl,
                     reinterpret_cast<float*>(X), ldx, reinterpret_cast<int*>(info), row0, vec);
  return check_launch("lcq_chol_inv_tile");
}

// ---------------------------------------------------------------------------------------
// fp32 GEMM for the recursion's updates (gptq_core._mm_lowT / _mm_low_right / _mm_low_left /
// _syrk_lower; torch `out.addmm_(A, B, beta=, alpha=)` in the reference-equivalent chain of
// gptq.py:161-170): C = beta C + alpha A B, all row-major strided views; A [M, K] (k
// contiguous), B [K, N] (bt 0) or given as its transpose [N, K] (bt 1). beta 0 never reads C
// (the recursion's outputs start uninitialised). fp32 MFMA v_mfma_f32_32x32x2_f32 (the
// trailing-update core of gptq.hip): 128x128 output tile per 256-thread workgroup (2x2 waves
// of 64x64), K in 32-deep chunks double-buffered through LDS with register staging. Operands
// whose k runs along the row (A, B^T) are transposed into [k][row] LDS panels while staged
// (pitch 129: the 8 rows x 8 k-quads a wave writes land <= 2 per bank); B [K, N] copies
// straight into [k][col] (pitch 128, 16-byte writes).
// ---------------------------------------------------------------------------------------
namespace lcq {
namespace f32g {

typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int KC = 32;   // K chunk

struct Args {
  const float* A;
  const float* B;
  float* C;
  int64_t M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int vec;  // every row start 16-byte aligned: float4 loads
};

// T x T output tile per 256-thread workgroup, 2 x 2 waves of (T/2)^2 = (T/64)^2 MFMA 32x32
// tiles each; T = 128 for grids that fill the chip, 64 below that (the recursion's many
// mid-size products: a 1024^2 output is 64 tiles of 128 but 256 of 64).
template <int T>
struct Tile {
  static constexpr int PT = T + 1;      // pitch of a transposed [k][row] panel
  static constexpr int PK = T;          // pitch of a k-major [k][col] panel
  static constexpr int SLOTS = T * KC / 4 / 256;  // float4 slots per thread per operand chunk
  static constexpr int MT = T / 64;     // MFMA tiles per wave side
};

// a k-contiguous operand tile: rows r0.., k0..k0+31
template <int T>
__device__ __forceinline__ void load_kc(const float* __restrict__ P, int64_t rows, int64_t K,
                                        int64_t ld, int64_t r0, int64_t k0, int tid, int vec,
                                        float4 (&v)[Tile<T>::SLOTS]) {
#pragma unroll
  for (int it = 0; it < Tile<T>::SLOTS; ++it) {
    const int idx = it * 256 + tid;
    const int64_t r = r0 + idx / 8, k = k0 + (idx % 8) * 4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < rows) {
      const float* p = P + r * ld + k;
      if (vec && k + 3 < K) {
        x = *reinterpret_cast<const float4*>(p);
      } else {
        if (k + 0 < K) x.x = p[0];
        if (k + 1 < K) x.y = p[1];
        if (k + 2 < K) x.z = p[2];
        if (k + 3 < K) x.w = p[3];
      }
    }
    v[it] = x;
  }
}
template <int T>
__device__ __forceinline__ void store_kc(float* __restrict__ S, int tid,
                                         const float4 (&v)[Tile<T>::SLOTS]) {
  constexpr int PT = Tile<T>::PT;
#pragma unroll
  for (int it = 0; it < Tile<T>::SLOTS; ++it) {
    const int idx = it * 256 + tid;
    const int r = idx / 8, k = (idx % 8) * 4;
    S[(k + 0) * PT + r] = v[it].x;
    S[(k + 1) * PT + r] = v[it].y;
    S[(k + 2) * PT + r] = v[it].z;
    S[(k + 3) * PT + r] = v[it].w;
  }
}
// a k-major operand tile (B [K, N]): k0..k0+31, cols c0..c0+T-1
template <int T>
__device__ __forceinline__ void load_km(const float* __restrict__ P, int64_t K, int64_t cols,
                                        int64_t ld, int64_t k0, int64_t c0, int tid, int vec,
                                        float4 (&v)[Tile<T>::SLOTS]) {
#pragma unroll
  for (int it = 0; it < Tile<T>::SLOTS; ++it) {
    const int idx = it * 256 + tid;
    const int64_t k = k0 + idx / (T / 4), c = c0 + (idx % (T / 4)) * 4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (k < K) {
      const float* p = P + k * ld + c;
      if (vec && c + 3 < cols) {
        x = *reinterpret_cast<const float4*>(p);
      } else {
        if (c + 0 < cols) x.x = p[0];
        if (c + 1 < cols) x.y = p[1];
        if (c + 2 < cols) x.z = p[2];
        if (c + 3 < cols) x.w = p[3];
      }
    }
    v[it] = x;
  }
}
template <int T>
__device__ __forceinline__ void store_km(float* __restrict__ S, int tid,
                                         const float4 (&v)[Tile<T>::SLOTS]) {
#pragma unroll
  for (int it = 0; it < Tile<T>::SLOTS; ++it) {
    const int idx = it * 256 + tid;
    *reinterpret_cast<float4*>(&S[(idx / (T / 4)) * Tile<T>::PK + (idx % (T / 4)) * 4]) = v[it];
  }
}

template <int BT, int T>
__global__ void __launch_bounds__(256, 2) k_gemm_f32(Args a) {
  using TL = Tile<T>;
  constexpr int PT = TL::PT, PB = BT ? TL::PT : TL::PK, MT = TL::MT, HW = T / 2;
  __shared__ __attribute__((aligned(16))) float As[2][KC * PT];
  __shared__ __attribute__((aligned(16))) float Bs[2][KC * PB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int64_t r0 = (int64_t)blockIdx.y * T, c0 = (int64_t)blockIdx.x * T;
  v16f acc[MT][MT];
#pragma unroll
  for (int x = 0; x < MT; ++x)
#pragma unroll
    for (int y = 0; y < MT; ++y)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[x][y][i] = 0.f;
  float4 ra[TL::SLOTS], rb[TL::SLOTS];
  auto load = [&](int64_t k0) {
    load_kc<T>(a.A, a.M, a.K, a.lda, r0, k0, tid, a.vec, ra);
    if constexpr (BT) load_kc<T>(a.B, a.N, a.K, a.ldb, c0, k0, tid, a.vec, rb);
    else load_km<T>(a.B, a.K, a.N, a.ldb, k0, c0, tid, a.vec, rb);
  };
  auto store = [&](int buf) {
    store_kc<T>(As[buf], tid, ra);
    if constexpr (BT) store_kc<T>(Bs[buf], tid, rb);
    else store_km<T>(Bs[buf], tid, rb);
  };
  load(0);
  store(0);
  __syncthreads();
  const int64_t nch = (a.K + KC - 1) / KC;
  for (int64_t ch = 0; ch < nch; ++ch) {
    const int cur = (int)(ch & 1);
    if (ch + 1 < nch) load((ch + 1) * KC);
    // all of this chunk's operand values first (the reads overlap the MFMAs that follow)
    float av[KC / 2][MT], bv[KC / 2][MT];
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      const int k = kk + (lane >> 5);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        av[kk / 2][t] = As[cur][k * PT + wr * HW + t * 32 + (lane & 31)];
        bv[kk / 2][t] = Bs[cur][k * PB + wc * HW + t * 32 + (lane & 31)];
      }
    }
#pragma unroll
    for (int kk = 0; kk < KC / 2; ++kk)
#pragma unroll
      for (int x = 0; x < MT; ++x)
#pragma unroll
        for (int y = 0; y < MT; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk][x], bv[kk][y], acc[x][y], 0,
                                                           0, 0);
    if (ch + 1 < nch) store(cur ^ 1);
    __syncthreads();
  }
  // C layout of a 32x32 MFMA tile: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int x = 0; x < MT; ++x)
#pragma unroll
    for (int y = 0; y < MT; ++y)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int64_t r = r0 + wr * HW + x * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        const int64_t c = c0 + wc * HW + y * 32 + (lane & 31);
        if (r < a.M && c < a.N) {
          float* p = a.C + r * a.ldc + c;
          const float v = a.alpha * acc[x][y][reg];
          *p = a.beta == 0.f ? v : __fmaf_rn(a.beta, *p, v);
        }
      }
}


// ---------------------------------------------------------------------------------------
// k_gemm_f32d_*: the same product with LDS-DMA staging, for 16-byte aligned rows and K % 32 == 0
// (every product of the recursion on 128-multiple Hessians). k_gemm_f32 above stages through
// registers (per-element bounds checks, transposing scalar LDS stores) and measured 55-80 TF/s
// (MFMA busy ~55 %, profiles/r3c_gemm_pmc.txt). Here:
//  * 32-float K chunks of T rows land in LDS by buffer_load ... lds (16 B per lane, 8 rows x
//    128 B per wave-instruction; rows / columns past the operand's end read as zero through
//    the buffer descriptor's range) in an NS-stage ring (2: one chunk in flight while the
//    other is multiplied), one barrier per chunk;
//  * v_mfma_f32_16x16x4_f32 with the chunk's k permuted: lane group g = lane >> 4 supplies k =
//    8g + s at step s (0..7) for both operands, so a lane's 8 values of a k-contiguous row are
//    two ds_read_b128 (16-B chunks 2g, 2g + 1 of the row, swizzled by swz32 so that every
//    16-lane group of the read hits 16 distinct bank slots). The k order of each output element
//    is fixed (deterministic), not the sequential one: the recursion is checked at T2;
//  * a k-major B [K, N] (bt = 0) is staged as [k][col] rows (T floats) with the 16-B chunks of
//    row k XOR-ed by ((k >> 3) & 1) * 4 (lane groups g and g + 1 of one 32-lane half land 64 B
//    apart) and read with ds_read_b32.
// T x T tile per 256-thread workgroup (2 x 2 waves of T/2 x T/2, (T/32)^2 16x16 MFMA tiles
// each): T = 128 where the grid fills the chip, 64 below.
// ---------------------------------------------------------------------------------------
typedef float v4f32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int DKC = 32;  // K chunk (floats): 128 B per k-contiguous row

__device__ __forceinline__ int swz32(int row) { return ((row >> 1) & 1) | ((row >> 1) & 4); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t f32_rsrc(const float* p, int64_t bytes) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  const int nb = __builtin_amdgcn_readfirstlane(
      (int)(bytes > 0x7fffffff ? 0x7fffffff : (bytes < 0 ? 0 : bytes)));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, nb, 0x00020000);
}

// One output tile (rows r0.., columns c0..) over K chunks [ch0, ch1): `part` null -> the
// alpha / beta epilogue into C, else the raw fp32 accumulators into the T x T partial tile
// `part` (stream-K segments, summed in k order by k_gemm_f32_sk_fixup).
// AK: A given k-major (element (m, k) at A[k lda + m], the GPTQ trailing update's stacked
// errors), staged and read like a k-major B.
template <int BT, int T, int NS, int AK = 0>
__device__ __forceinline__ void gemm_f32d_body(const Args& a, char* f32lds, int64_t r0,
                                               int64_t c0, int64_t ch0, int64_t ch1,
                                               float* part) {
  constexpr int OPB = T * DKC * 4;        // one operand chunk image (bytes)
  constexpr int STG = 2 * OPB;
  constexpr int PA = T / 32;              // A pieces (8 rows x 128 B) per wave
  constexpr int PB = T / 32;              // B pieces per wave (k-major: 1 KB of [k][col] rows)
  constexpr int WT = T / 2, MT = WT / 16; // wave tile, 16x16 MFMA tiles per side
  constexpr int LPS = PA + PB;            // DMA instructions per wave per stage
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int64_t nch = ch1;

  const __amdgpu_buffer_rsrc_t ra =
      AK ? f32_rsrc(a.A + r0, ((a.K - 1) * a.lda + (a.M - r0)) * 4)
         : f32_rsrc(a.A + r0 * a.lda, (a.M - r0) * a.lda * 4);
  __amdgpu_buffer_rsrc_t rb;
  if constexpr (BT) rb = f32_rsrc(a.B + c0 * a.ldb, (a.N - c0) * a.ldb * 4);
  else rb = f32_rsrc(a.B + c0, ((a.K - 1) * a.ldb + (a.N - c0)) * 4);
  uint32_t aoff[PA], boff[PB];
#pragma unroll
  for (int j = 0; j < PA; ++j) {  // piece j of wave w: rows (j * 4 + w) * 8 .. + 7
    if constexpr (AK) {  // [k][row] rows of T floats, as a k-major B
      constexpr int CPR = T / 4;
      const int k = (j * 4 + w) * (256 / T) + lane / CPR, pc = lane % CPR;
      const int lc = pc ^ (((k >> 3) & 1) * 4);
      aoff[j] = (uint32_t)((k * a.lda + lc * 4) * 4);
    } else {
      const int row = (j * 4 + w) * 8 + (lane >> 3);
      aoff[j] = (uint32_t)((row * a.lda + (((lane & 7) ^ swz32(row)) * 4)) * 4);
    }
  }
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    if constexpr (BT) {
      const int row = (j * 4 + w) * 8 + (lane >> 3);
      boff[j] = (uint32_t)((row * a.ldb + (((lane & 7) ^ swz32(row)) * 4)) * 4);
    } else {  // [k][col] rows of T floats: a piece = 1024 / (4 T) k-rows
      constexpr int CPR = T / 4;           // 16-B chunks per k-row
      const int k = (j * 4 + w) * (256 / T) + lane / CPR, pc = lane % CPR;
      const int lc = pc ^ (((k >> 3) & 1) * 4);
      boff[j] = (uint32_t)((k * a.ldb + lc * 4) * 4);
    }
  }
  auto stage = [&](int buf, int64_t ch) {
    const int64_t cc = ch < nch ? ch : nch - 1;  // past the end: re-fetch (unused)
    char* dst = f32lds + buf * STG;
    // the chunk offset goes into voffset (not soffset), so the descriptor's range check covers
    // every byte: past-the-end rows / columns read as zero and never leave the allocation
    const uint32_t ka = (uint32_t)(cc * DKC * 4);
    const uint32_t kao = AK ? (uint32_t)(cc * DKC * a.lda * 4) : ka;
    const uint32_t kbo = BT ? ka : (uint32_t)(cc * DKC * a.ldb * 4);
#pragma unroll
    for (int j = 0; j < PA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(dst + (j * 4 + w) * 1024), 16,
                                               aoff[j] + kao, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < PB; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (lds_void_t*)(dst + OPB + (j * 4 + w) * 1024), 16, boff[j] + kbo, 0, 0, 0);
  };

  v4f32 acc[MT][MT];
#pragma unroll
  for (int x = 0; x < MT; ++x)
#pragma unroll
    for (int y = 0; y < MT; ++y) acc[x][y] = v4f32{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, g = lane >> 4;

  __syncthreads();  // a previous segment of this workgroup may still read the ring
#pragma unroll
  for (int j = 0; j + 1 < NS; ++j) stage(j, ch0 + j);
  for (int64_t ch = ch0; ch < nch; ++ch) {
    const int buf = (int)((ch - ch0) % NS);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * LPS) : "memory");
    __builtin_amdgcn_s_barrier();
    stage((int)((ch - ch0 + NS - 1) % NS), ch + NS - 1);
    const char* As = f32lds + buf * STG;
    const char* Bs = As + OPB;
    float av[MT][8], bv[MT][8];
#pragma unroll
    for (int x = 0; x < MT; ++x) {
      const int row = wr * WT + x * 16 + r16;
      if constexpr (AK) {
        // both operands k-major: lane group g supplies k = 4 s + g at step s, so every
        // output element accumulates k = 0, 1, 2, ... in order -- the same fmaf chain as the
        // register-staged 32x32x2 kernel, bit for bit
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int k = 4 * s + g;
          const int pc = (row >> 2) ^ (((k >> 3) & 1) * 4);
          av[x][s] = *reinterpret_cast<const float*>(As + (k * T + pc * 4 + (row & 3)) * 4);
        }
      } else {
        const char* rp = As + row * 128;
        const float4 lo = *reinterpret_cast<const float4*>(rp + ((2 * g) ^ swz32(row)) * 16);
        const float4 hi = *reinterpret_cast<const float4*>(rp + ((2 * g + 1) ^ swz32(row)) * 16);
        av[x][0] = lo.x; av[x][1] = lo.y; av[x][2] = lo.z; av[x][3] = lo.w;
        av[x][4] = hi.x; av[x][5] = hi.y; av[x][6] = hi.z; av[x][7] = hi.w;
      }
    }
#pragma unroll
    for (int y = 0; y < MT; ++y) {
      if constexpr (BT) {
        const int row = wc * WT + y * 16 + r16;
        const char* rp = Bs + row * 128;
        const float4 lo = *reinterpret_cast<const float4*>(rp + ((2 * g) ^ swz32(row)) * 16);
        const float4 hi = *reinterpret_cast<const float4*>(rp + ((2 * g + 1) ^ swz32(row)) * 16);
        bv[y][0] = lo.x; bv[y][1] = lo.y; bv[y][2] = lo.z; bv[y][3] = lo.w;
        bv[y][4] = hi.x; bv[y][5] = hi.y; bv[y][6] = hi.z; bv[y][7] = hi.w;
      } else {
        const int col = wc * WT + y * 16 + r16;
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const int k = AK ? 4 * s + g : 8 * g + s;
          const int pc = (col >> 2) ^ (((k >> 3) & 1) * 4);
          bv[y][s] = *reinterpret_cast<const float*>(Bs + (k * T + pc * 4 + (col & 3)) * 4);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int x = 0; x < MT; ++x)
#pragma unroll
        for (int y = 0; y < MT; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[x][s], bv[y][s], acc[x][y], 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // 16x16 MFMA tile: lane holds column lane & 15, rows 4 (lane >> 4) + v
  if (part != nullptr) {
#pragma unroll
    for (int x = 0; x < MT; ++x)
#pragma unroll
      for (int y = 0; y < MT; ++y)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          part[(wr * WT + x * 16 + 4 * g + v) * T + wc * WT + y * 16 + r16] = acc[x][y][v];
    return;
  }
#pragma unroll
  for (int x = 0; x < MT; ++x)
#pragma unroll
    for (int y = 0; y < MT; ++y) {
      const int64_t c = c0 + wc * WT + y * 16 + r16;
      if (c >= a.N) continue;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t r = r0 + wr * WT + x * 16 + 4 * g + v;
        if (r < a.M) {
          float* p = a.C + r * a.ldc + c;
          const float val = a.alpha * acc[x][y][v];
          *p = a.beta == 0.f ? val : __fmaf_rn(a.beta, *p, val);
        }
      }
    }
}

#ifndef LCQ_F32D_NS
#define LCQ_F32D_NS 2  // measured against 3 on the chain's shapes: 77-93 -> 96-114 TF/s,
                       // 4096^3 110 -> 136 (profiles/r4_f32_variants.txt)
#endif
#ifndef LCQ_F32D_OCC
#define LCQ_F32D_OCC 1
#endif
constexpr int NS_F32D = LCQ_F32D_NS;  // (probe builds vary the ring depth / occupancy)
template <int T>
constexpr int f32d_lds() { return NS_F32D * 2 * T * DKC * 4; }

// fixed kernels around the body (a templated __global__ with device builtins inside its
// lambda loses its host stub under hipcc)
#define LCQ_F32D_KERNEL(NAME, BT, T)                                                   \
  __global__ void __launch_bounds__(256, LCQ_F32D_OCC) NAME(Args a) {                             \
    extern __shared__ __attribute__((aligned(16))) char f32lds[];                      \
    gemm_f32d_body<BT, T, NS_F32D>(a, f32lds, (int64_t)blockIdx.y * T,                 \
                                   (int64_t)blockIdx.x * T, 0, a.K / DKC, nullptr);    \
  }
#define LCQ_F32D_AK_KERNEL(NAME, T)                                                    \
  __global__ void __launch_bounds__(256, LCQ_F32D_OCC) NAME(Args a) {                  \
    extern __shared__ __attribute__((aligned(16))) char f32lds[];                      \
    gemm_f32d_body<0, T, NS_F32D, 1>(a, f32lds, (int64_t)blockIdx.y * T,               \
                                     (int64_t)blockIdx.x * T, 0, a.K / DKC, nullptr);  \
  }
LCQ_F32D_AK_KERNEL(k_gemm_f32d_kn128, 128)
LCQ_F32D_AK_KERNEL(k_gemm_f32d_kn64, 64)
#undef LCQ_F32D_AK_KERNEL
LCQ_F32D_KERNEL(k_gemm_f32d_n128, 0, 128)
LCQ_F32D_KERNEL(k_gemm_f32d_t128, 1, 128)
LCQ_F32D_KERNEL(k_gemm_f32d_n64, 0, 64)
LCQ_F32D_KERNEL(k_gemm_f32d_t64, 1, 64)
#undef LCQ_F32D_KERNEL

// Stream-K over 128^2 tiles: the tiles x K-chunks work units split evenly over SK_WG
// workgroups (one per CU: SK_WG = 256 on MI355X), so a grid of e.g. 784 tiles (3.06 rounds of
// 256, 76 % of the last round idle) runs as one full round. Workgroup w takes units
// [b(w), b(w + 1)), b(w) = w U / SK_WG, tile-major (t = u / nch): a whole tile goes straight
// to C with the normal epilogue (the same k order as k_gemm_f32d_*128); a tile cut by a
// workgroup boundary leaves its k segments as raw partial tiles in fixed slots (the segment
// that starts the workgroup's range -> slot 2w, the one that ends it -> slot 2w + 1) and
// k_gemm_f32_sk_fixup sums them in k order (deterministic: no atomics, no spin-waits).
constexpr int SK_WG = 256;
struct SkArgs {
  int64_t tiles, ntn, nch, units;
  float* part;   // 2 * SK_WG slots of 128 x 128 fp32
};
__device__ __forceinline__ int64_t sk_bound(const SkArgs& s, int64_t w) {
  return w * s.units / SK_WG;
}

#define LCQ_F32D_SK_KERNEL(NAME, BT)                                                  \
  __global__ void __launch_bounds__(256, 1) NAME(Args a, SkArgs sk) {                 \
    extern __shared__ __attribute__((aligned(16))) char f32lds[];                     \
    const int64_t w = blockIdx.x, u0 = sk_bound(sk, w), u1 = sk_bound(sk, w + 1);     \
    for (int64_t u = u0; u < u1;) {                                                   \
      const int64_t t = u / sk.nch, ts = t * sk.nch, te = ts + sk.nch;                \
      const int64_t e = te < u1 ? te : u1;                                            \
      float* part = nullptr;                                                          \
      if (u != ts || e != te)                                                         \
        part = sk.part + (u == u0 && u != ts ? 2 * w : 2 * w + 1) * (128 * 128);      \
      gemm_f32d_body<BT, 128, NS_F32D>(a, f32lds, (t / sk.ntn) * 128,                 \
                                       (t % sk.ntn) * 128, u - ts, e - ts, part);      \
      u = e;                                                                          \
    }                                                                                 \
  }
LCQ_F32D_SK_KERNEL(k_gemm_f32d_sk_n128, 0)
LCQ_F32D_SK_KERNEL(k_gemm_f32d_sk_t128, 1)
#undef LCQ_F32D_SK_KERNEL

// C tile t = beta C + alpha * (((seg_0 + seg_1) + ...) in k order) for every tile cut by a
// workgroup boundary; a workgroup per (tile, 16-row piece), whole tiles exit at once
__global__ void __launch_bounds__(256) k_gemm_f32_sk_fixup(Args a, SkArgs sk) {
  const int64_t t = blockIdx.x;
  const int64_t ts = t * sk.nch, tl = ts + sk.nch - 1;
  // the workgroups holding the tile's first and last unit (b(w) = w U / SK_WG)
  int64_t wa = (ts * SK_WG) / sk.units, wb = (tl * SK_WG) / sk.units;
  while (sk_bound(sk, wa + 1) <= ts) ++wa;
  while (wa > 0 && sk_bound(sk, wa) > ts) --wa;
  while (sk_bound(sk, wb + 1) <= tl) ++wb;
  while (wb > 0 && sk_bound(sk, wb) > tl) --wb;
  if (wa == wb) return;  // one workgroup: written by the main kernel
  const int64_t r0 = (t / sk.ntn) * 128, c0 = (t % sk.ntn) * 128;
  const int cx = threadIdx.x & 127, rr0 = blockIdx.y * 16 + (threadIdx.x >> 7);
  for (int rr = rr0; rr < blockIdx.y * 16 + 16; rr += 2) {
    const int64_t r = r0 + rr, c = c0 + cx;
    if (r >= a.M || c >= a.N) continue;
    float v = sk.part[(2 * wa + 1) * (128 * 128) + rr * 128 + cx];
    for (int64_t w = wa + 1; w <= wb; ++w)
      if (sk_bound(sk, w + 1) > sk_bound(sk, w))  // (an empty range holds no segment)
        v = __fadd_rn(v, sk.part[(2 * w) * (128 * 128) + rr * 128 + cx]);
    float* p = a.C + r * a.ldc + c;
    const float val = a.alpha * v;
    *p = a.beta == 0.f ? val : __fmaf_rn(a.beta, *p, val);
  }
}

}  // namespace f32g
}  // namespace lcq

static int64_t sk_ws_bytes() { return (int64_t)2 * f32g::SK_WG * 128 * 128 * 4; }

// Stream-K (k_gemm_f32d_sk_*) where a 128^2-tile grid leaves more than 10 % of its last round
// of 256 workgroups idle and every workgroup still gets >= 32 K chunks of work
static bool use_stream_k(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((N + 127) / 128) * ((M + 127) / 128);
  if (tiles < 128 || K % f32g::DKC) return false;
  const int64_t rounds = (tiles + f32g::SK_WG - 1) / f32g::SK_WG;
  const bool ragged = tiles * 10 < rounds * f32g::SK_WG * 9;
  return ragged && tiles * (K / f32g::DKC) >= (int64_t)32 * f32g::SK_WG;
}

extern "C" int64_t lcq_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  return use_stream_k(M, N, K) ? sk_ws_bytes() : 0;
}

static int gemm_f32_impl(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                         int64_t lda, const void* B, int64_t ldb, int bt, float beta, void* C,
                         int64_t ldc, void* ws, int64_t ws_bytes, void* stream) {

  LCQ_REQUIRE(M >= 0 && N >= 0 && K >= 0, "negative size");
  if (M == 0 || N == 0) return LCQ_OK;
  LCQ_REQUIRE(A != nullptr && B != nullptr && C != nullptr, "null pointers");
  LCQ_REQUIRE(lda >= K && ldc >= N && ldb >= (bt ? K : N), "leading dimensions too small");
  LCQ_REQUIRE(M / 64 < 65535, "M too large");
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  f32g::Args a{};
  a.A = reinterpret_cast<const float*>(A);
  a.B = reinterpret_cast<const float*>(B);
  a.C = reinterpret_cast<float*>(C);
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.alpha = alpha; a.beta = beta;
  a.vec = al(A) && al(B) && lda % 4 == 0 && ldb % 4 == 0;
  if (K == 0) a.alpha = 0.f;  // C = beta C
  hipStream_t st = as_stream(stream);
  // 128^2 tiles where they fill the chip, 64^2 below (4x the workgroups)
  const int64_t t128 = ((N + 127) / 128) * ((M + 127) / 128);
  const bool big = t128 >= 256;
  // LDS-DMA kernel: K % 32 == 0, 16-byte aligned rows, 32-bit byte offsets
  const bool dma = K % f32g::DKC == 0 && a.vec && al(C) &&
                   M * lda < ((int64_t)1 << 29) && (bt ? N * ldb : K * ldb) < ((int64_t)1 << 29);
  if (dma && ws != nullptr && ws_bytes >= sk_ws_bytes() && use_stream_k(M, N, K)) {
    f32g::SkArgs sk{};
    sk.ntn = (N + 127) / 128;
    sk.tiles = sk.ntn * ((M + 127) / 128);
    sk.nch = K / f32g::DKC;
    sk.units = sk.tiles * sk.nch;
    sk.part = reinterpret_cast<float*>(ws);
    constexpr int L = f32g::f32d_lds<128>();
    auto k = bt ? f32g::k_gemm_f32d_sk_t128 : f32g::k_gemm_f32d_sk_n128;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, L);
    hipLaunchKernelGGL(k, dim3(f32g::SK_WG), 256, L, st, a, sk);
    int rc = check_launch("lcq_gemm_f32: stream-k");
    if (rc) return rc;
    hipLaunchKernelGGL(f32g::k_gemm_f32_sk_fixup, dim3((unsigned)sk.tiles, 8), 256, 0, st, a,
                       sk);
  } else if (dma) {
    if (big) {
      const dim3 grid((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128));
      constexpr int L = f32g::f32d_lds<128>();
      if (bt) {
        (void)hipFuncSetAttribute((const void*)f32g::k_gemm_f32d_t128,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, L);
        hipLaunchKernelGGL(f32g::k_gemm_f32d_t128, grid, 256, L, st, a);
      } else {
        (void)hipFuncSetAttribute((const void*)f32g::k_gemm_f32d_n128,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, L);
        hipLaunchKernelGGL(f32g::k_gemm_f32d_n128, grid, 256, L, st, a);
      }
    } else {
      const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
      constexpr int L = f32g::f32d_lds<64>();
      if (bt) hipLaunchKernelGGL(f32g::k_gemm_f32d_t64, grid, 256, L, st, a);
      else hipLaunchKernelGGL(f32g::k_gemm_f32d_n64, grid, 256, L, st, a);
    }
  } else if (big) {
    const dim3 grid((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128));
    if (bt) hipLaunchKernelGGL((f32g::k_gemm_f32<1, 128>), grid, 256, 0, st, a);
    else hipLaunchKernelGGL((f32g::k_gemm_f32<0, 128>), grid, 256, 0, st, a);
  } else {
    const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
    if (bt) hipLaunchKernelGGL((f32g::k_gemm_f32<1, 64>), grid, 256, 0, st, a);
    else hipLaunchKernelGGL((f32g::k_gemm_f32<0, 64>), grid, 256, 0, st, a);
  }
  return check_launch("lcq_gemm_f32");
}

namespace lcq {
int gemm_f32_sub_akn(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                     const float* B, int64_t ldb, float* C, int64_t ldc, hipStream_t st) {
  if (M <= 0 || N <= 0) return LCQ_OK;
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (K <= 0 || K % f32g::DKC != 0 || !al(A) || !al(B) || !al(C) || lda % 4 != 0 ||
      ldb % 4 != 0 || ldc % 4 != 0 || lda < M || ldb < N ||
      K * lda >= ((int64_t)1 << 29) || K * ldb >= ((int64_t)1 << 29) || M / 64 >= 65535)
    return LCQ_EUNSUP;
  f32g::Args a{};
  a.A = A;
  a.B = B;
  a.C = C;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.alpha = -1.f; a.beta = 1.f;   // C = fma(1, C, -acc): the product rounded, then subtracted
  a.vec = 1;
  const int64_t t128 = ((N + 127) / 128) * ((M + 127) / 128);
  if (t128 >= 256) {
    constexpr int L = f32g::f32d_lds<128>();
    (void)hipFuncSetAttribute((const void*)f32g::k_gemm_f32d_kn128,
                              hipFuncAttributeMaxDynamicSharedMemorySize, L);
    hipLaunchKernelGGL(f32g::k_gemm_f32d_kn128,
                       dim3((unsigned)((N + 127) / 128), (unsigned)((M + 127) / 128)), 256, L,
                       st, a);
  } else {
    constexpr int L = f32g::f32d_lds<64>();
    (void)hipFuncSetAttribute((const void*)f32g::k_gemm_f32d_kn64,
                              hipFuncAttributeMaxDynamicSharedMemorySize, L);
    hipLaunchKernelGGL(f32g::k_gemm_f32d_kn64,
                       dim3((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64)), 256, L, st,
                       a);
  }
  return check_launch("gemm_f32_sub_akn");
}
}  // namespace lcq

extern "C" int lcq_gemm_f32(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                            int64_t lda, const void* B, int64_t ldb, int bt, float beta, void* C,
                            int64_t ldc, void* stream) {
  return gemm_f32_impl(M, N, K, alpha, A, lda, B, ldb, bt, beta, C, ldc, nullptr, 0, stream);
}

extern "C" int lcq_gemm_f32_ws(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                               int64_t lda, const void* B, int64_t ldb, int bt, float beta,
                               void* C, int64_t ldc, void* workspace, int64_t ws_bytes,
                               void* stream) {
  return gemm_f32_impl(M, N, K, alpha, A, lda, B, ldb, bt, beta, C, ldc, workspace, ws_bytes,
                       stream);
}
