// Diagonal-tile kernel of the recursive fp32 Cholesky / triangular inverse behind GPTQ's
// U = chol(H^-1, upper) (gptq.py:169-174; computed as J chol(J H J)^-1 J, see gptq_core).
// The recursion (host side) does the large updates as fp32 GEMMs; this kernel factors a
// <= 128 x 128 diagonal tile and inverts its factor, in one 256-thread workgroup.
//
// Blocked right-looking over 16-column panels on the augmented [A | R], R = I initially
// (after panel p, R's rows p hold X_p = L_pp^-1 R_p: the rows of X = L^-1, blocked forward
// substitution of L X = I). The tile is 8 x 8 blocks of 16 x 16, each block kept in LDS in the
// accumulator layout of v_mfma_f32_16x16x4_f32 (lane l, register j: row 4 (l >> 4) + j,
// column l & 15; one ds_read_b128 / ds_write_b128 per lane per block, conflict-free):
//   At(i, j), i >= j: the block A_ij^T (its transpose: see below); after panel j it holds L_ij^T
//   Rt(i, k), i >= k: R_ik; after panel i, X_ik
// With both operands' k permuted as k = 4 (l >> 4) + s at MFMA step s, the accumulator layout
// of M^T is exactly M's A-operand fragment and the accumulator layout of N is N's B-operand
// fragment, so every product below reads its operands straight from the stored blocks:
//   S1 (wave 0): factor the 16 x 16 diagonal block -- lane r holds row r of A_pp in registers,
//      column c's pivot and the L[k][c] it needs are taken by v_readlane (no LDS, no barrier);
//      the same fmas run the forward substitution of Z = L_pp^-1 in lanes 16 + j (column j)
//   S2 (all waves, 8 blocks): L_i^T = Z A_ip^T (i > p) and X_pk = Z R_pk (k <= p)
//   S3: A_ij^T -= L_j L_i^T (p < j <= i), R_ik -= L_i X_pk (i > p, k <= p). Look-ahead: wave 0
//      updates the next diagonal block first and runs S1 of panel p + 1 while waves 1-3 do the
//      rest of S3, so the serial factorisation overlaps the trailing update (two barriers per
//      panel).
// Rows / columns past n are an identity pad (chol of [A 0; 0 I] is [L 0; 0 I]); only the n x n
// corner is written. Only X = L^-1 is needed by the recursion (gptq_core._chol_inv_rec); L is
// written back only when asked for (L may alias A: every read of A precedes the first barrier,
// every write of L follows the last). fp32 throughout (the fp32 MFMA sums its products exactly
// like an fmaf chain, in the permuted k order); checked against fp64 (tests/test_gptq_gpu.py).
// Round 4's kernel (8-column panels, LDS-resident 4 x 4 register tiles, one wave redundantly
// factoring each 8 x 8 block) took ~64 us per 128-tile in the GPTQ chain.
#include "lcq_common.h"

namespace lcq {
namespace ctile {

constexpr int CTILE = 128;
constexpr int TT = 16;                       // MFMA block side
constexpr int NTL = CTILE / TT;              // 8 block rows / columns
constexpr int NLOW = NTL * (NTL + 1) / 2;    // 36 lower blocks
constexpr int TF = TT * TT;                  // floats per block
constexpr int NT = 256;                      // 4 waves
constexpr int OFF_A = 0, OFF_R = NLOW * TF, OFF_Z = 2 * NLOW * TF, OFF_L = OFF_Z + TF;
constexpr int OFF_SCR = OFF_L + NTL * TF;            // one scratch block (padding jobs)
constexpr int OFF_Z2 = OFF_SCR + TF;                 // Z of odd panels (Zs double-buffered)
constexpr int OFF_SYNC = OFF_Z2 + TF;                // per panel: S2 arrivals of waves 1-3,
                                                     // and wave 0's "L_{p+1} written" flag
constexpr int OFF_JOB = OFF_SYNC + 2 * NTL;          // the S3 job table (kJobs), copied in
constexpr int JOB_WORDS = (NTL - 1) * 3 * (12 * 2 + 4);  // 21 rows of 24 entries + count, 16-B rows
constexpr int LDS_BYTES = (OFF_JOB + JOB_WORDS) * 4;   // 87408 B

typedef float v4f __attribute__((ext_vector_type(4)));

#ifdef LCQ_CHOL_PROF  // probe builds only (scripts/probes/chol_tile_prof2.py): s_memtime stamps
#define PROF_STAMP(k, who)                                                              \
  if (w == (who) && lane == 0)                                                          \
    reinterpret_cast<unsigned long long*>(info)[1 + (k)] = __builtin_amdgcn_s_memtime();
#define PROF_REAL(k)                                                                     \
  if (w == 0 && lane == 0)                                                              \
    reinterpret_cast<unsigned long long*>(info)[1 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define PROF_STAMP(k, who)
#define PROF_REAL(k)
#endif

__host__ __device__ constexpr int tix(int i, int j) { return i * (i + 1) / 2 + j; }

__device__ __forceinline__ void tri_ij(int t, int& i, int& j) {
  i = 0;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  j = t - i * (i + 1) / 2;
}

__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ v4f ld4(const float* blk, int lane) {
  return *reinterpret_cast<const v4f*>(blk + 4 * lane);
}
__device__ __forceinline__ void st4(float* blk, int lane, v4f v) {
  *reinterpret_cast<v4f*>(blk + 4 * lane) = v;
}

// acc += A B over one block's 16 k: `at` = accumulator-layout block of A^T, `b` = of B
__device__ __forceinline__ v4f mma16(v4f acc, v4f at, v4f b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(at.w, b.w, acc, 0, 0, 0);
  return acc;
}

#ifndef LCQ_PROBE_CHOL_IEEE_RSQ
#define LCQ_PROBE_CHOL_IEEE_RSQ 0   // probe builds: IEEE sqrtf / division in S1
#endif

// S1 on wave 0: factor the (symmetric) diagonal block At(q, q); L_qq rows -> Ld[q] (row-major,
// zero above the diagonal), Z = L_qq^-1 -> Zs column-major (Zs[j * 16 + r] = Z[r][j]; Zs of
// panel q at OFF_Z (q even) or OFF_Z2 (q odd): S1 of panel q + 1 runs while the other waves
// still read panel q's).
// Lanes 0-15 hold row r of the block (right-looking: A[r][k] -= L[r][c] L[k][c]), lanes 16-31
// column j of W = I (forward substitution: W[k][j] -= L[k][c] Z[c][j]); both updates are
// v[k] -= m * L[k][c] with the lane's own multiplier m = v[c] / L[c][c] (L[r][c], or Z[c][j]),
// so ONE fma per (c, k) serves the factorisation and the inverse, and the L[k][c] come from
// v_readlane of the row lanes' m. LAPACK's spotf2 step (ajj = sqrt(ajj), column scaled by
// 1 / ajj) on the hardware v_sqrt_f32 / v_rcp_f32 (1 ulp; the IEEE forms, a probe build, cost
// 1.5x the S1 chain -- 5.5k against 3.7k cycles per panel -- and move U by ~1e-7 relative,
// below the chain's GEMM rounding; profiles/r5_chol_tile.md). The trailing updates subtract
// the summed product once (BLAS's C - A B), which keeps GPTQ's codes >= 99.9 % equal to the
// reference with either. Non-positive pivots: recorded (first one, 1-based row
// row0 + 16 q + c + 1), replaced by 1.
__device__ __forceinline__ void factor_block(float* sm, int q, int lane, int* info, int64_t row0) {
  const float* blk = sm + OFF_A + tix(q, q) * TF;
  const int r = lane & 15;
  const bool rowlane = lane < TT;
  float v[TT];
#pragma unroll
  for (int c = 0; c < TT; ++c)   // row lanes: element (r, c); column lanes: identity column
    v[c] = rowlane ? blk[4 * (c + 16 * (r >> 2)) + (r & 3)] : (c == r ? 1.f : 0.f);
  int bad = 0;
#pragma unroll
  for (int c = 0; c < TT; ++c) {
    const float piv = rl(v[c], c);
    const bool nb = !(piv > 0.f);
    if (nb && bad == 0) bad = c + 1;
#if LCQ_PROBE_CHOL_IEEE_RSQ   // probe builds only: correctly rounded sqrt and reciprocal
    const float sq = nb ? 1.f : sqrtf(piv);
    const float rinv = 1.f / sq;
#else
    const float sq = nb ? 1.f : __builtin_amdgcn_sqrtf(piv);
    const float rinv = __builtin_amdgcn_rcpf(sq);
#endif
    const float m = v[c] * rinv;   // row lane r: L[r][c]; column lane j: Z[c][j]
#pragma unroll
    for (int k = c + 1; k < TT; ++k) v[k] = fmaf(-m, rl(m, k), v[k]);
    v[c] = lane == c ? sq : m;
  }
  if (lane < 2 * TT) {
    float* dst = lane < TT ? sm + OFF_L + q * TF + TT * lane
                           : sm + ((q & 1) ? OFF_Z2 : OFF_Z) + TT * (lane - TT);
#pragma unroll
    for (int c = 0; c < TT; c += 4)
      *reinterpret_cast<v4f*>(dst + c) =
          rowlane ? v4f{c <= r ? v[c] : 0.f, c + 1 <= r ? v[c + 1] : 0.f,
                        c + 2 <= r ? v[c + 2] : 0.f, c + 3 <= r ? v[c + 3] : 0.f}
                  : v4f{v[c], v[c + 1], v[c + 2], v[c + 3]};
  }
  if (bad && lane == 0 && info) atomicCAS(info, 0, (int)(row0 + TT * q + bad));
}

// Trailing-update jobs: dst -= A B, the product summed first (from 0, in the MFMA k order) and
// subtracted once (BLAS's C - A B^T of the reference's blocked factorisation), four jobs per
// call so that their LDS reads and MFMA chains overlap. A job whose dst is the scratch block
// (Tail) is a no-op padding the last group.
struct Job {
  float* dst;
  const float* at;
  const float* b;
};

__device__ __forceinline__ void run4(const Job& j0, const Job& j1, const Job& j2, const Job& j3,
                                     int lane) {
  const Job* j[4] = {&j0, &j1, &j2, &j3};
  v4f c[4], a[4], b[4], o[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    c[u] = ld4(j[u]->dst, lane);
    a[u] = ld4(j[u]->at, lane);
    b[u] = ld4(j[u]->b, lane);
    o[u] = v4f{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      o[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][s], b[u][s], o[u], 0, 0, 0);
#pragma unroll
  for (int u = 0; u < 4; ++u) st4(j[u]->dst, lane, c[u] - o[u]);
}

// lower 16-block (i, j) of the load phase's block t = w + 4 u (row-major over the triangle)
__device__ constexpr int kTi[NLOW] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5,
                                      5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 7, 7, 7, 7, 7, 7, 7};

// S3 job lists of a full 128-tile (ntl 8), panel p, wave 1 + w3: job n of the panel's list
// (blocks A_{i,jc}, q <= jc <= i but (q, q), then R_{i,k}, k <= p, row by row) goes to
// wave 1 + n % 3. Row pw = 3 p + w3: job u = {dst | A-operand << 16, B-operand} as LDS float
// offsets, padded to a multiple of 4 with no-op jobs on the scratch block, then the padded
// count. The table is copied into LDS in the load phase; a wave reads its row with uniform-
// address LDS reads at the start of the panel (hidden behind S2).
constexpr int JMAX = 12;
constexpr int JROW = JMAX * 2 + 4;   // words per row: 12 jobs x {dst | A << 16, B}, n4, pad
struct JobTab {
  uint32_t w[(NTL - 1) * 3][JROW];
};

constexpr JobTab make_jobs() {
  JobTab t{};
  int cnt[(NTL - 1) * 3] = {};
  for (int p = 0; p < NTL - 1; ++p) {
    const int q = p + 1;
    int jn = 0;
    auto add = [&](int d, int a, int b) {
      const int pw = 3 * p + jn++ % 3, u = cnt[pw]++;
      t.w[pw][2 * u] = (uint32_t)d | ((uint32_t)a << 16);
      t.w[pw][2 * u + 1] = (uint32_t)b;
    };
    for (int i = q; i < NTL; ++i) {
      for (int jc = q; jc <= i; ++jc) {
        if (jc == q && i == q) continue;
        add(OFF_A + tix(i, jc) * TF, OFF_A + tix(jc, p) * TF, OFF_A + tix(i, p) * TF);
      }
      for (int k = 0; k <= p; ++k)
        add(OFF_R + tix(i, k) * TF, OFF_A + tix(i, p) * TF, OFF_R + tix(p, k) * TF);
    }
  }
  for (int pw = 0; pw < (NTL - 1) * 3; ++pw) {
    t.w[pw][2 * JMAX] = (uint32_t)((cnt[pw] + 3) & ~3);
    for (int u = cnt[pw]; u < JMAX; ++u) {
      t.w[pw][2 * u] = (uint32_t)OFF_SCR | ((uint32_t)OFF_SCR << 16);
      t.w[pw][2 * u + 1] = (uint32_t)OFF_SCR;
    }
  }
  return t;
}
static_assert(sizeof(JobTab) == JOB_WORDS * 4, "job table size");
__constant__ constexpr JobTab kJobs = make_jobs();

__global__ void __launch_bounds__(NT) k_chol_inv_tile(const float* A, int64_t lda, int n,
                                                       float* Lout, int64_t ldl,
                                                       float* __restrict__ X, int64_t ldx,
                                                       int* __restrict__ info, int64_t row0,
                                                       int vec) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = (lane >> 4) * 4;
  const int ntl = (n + TT - 1) / TT;
  float* const scratch = sm + OFF_SCR;
  PROF_STAMP(0, 0)
  PROF_REAL(42)

  // load: At(i, j) lane l register jj = A_ij^T[g4 + jj][r16] = A[16 i + r16][16 j + g4 + jj]
  // (one float4 per lane and block when the tile is a full, aligned 128^2; the lower triangle
  // only: a diagonal block's upper half is then taken from its mirror in LDS by the same wave;
  // identity pad past n); Rt = I. Wave 0 loads block (0, 0) and factors it (S1 of panel 0)
  // while waves 1-3 load the other 35 blocks (12 each, every load issued before the stores).
  auto load_blk = [&](int t) {
    const int i = kTi[t], j = t - i * (i + 1) / 2;
    const int gr = TT * i + r16, gc0 = TT * j + g4;
    v4f v;
    if (vec) {
      v = *reinterpret_cast<const v4f*>(A + (int64_t)gr * lda + gc0);
    } else {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int gc = gc0 + jj;
        v[jj] = gr < n && gc < n && gc <= gr ? A[(int64_t)gr * lda + gc] : (gr == gc ? 1.f : 0.f);
      }
    }
    return v;
  };
  auto store_blk = [&](int t, v4f v) {
    const int i = kTi[t], j = t - i * (i + 1) / 2;
    float* blk = sm + OFF_A + t * TF;
    st4(blk, lane, v);
    v4f e = {0.f, 0.f, 0.f, 0.f};
    if (i == j) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) e[jj] = g4 + jj == r16 ? 1.f : 0.f;
      // diagonal block: element (a, b) = A_ii[b][a] with a = g4 + jj > b = r16 lies above the
      // diagonal (not read); take its mirror A_ii[a][b] = element (b, a), stored at lane
      // a + 16 (b >> 2), register b & 3 (this wave's own store: LDS is in order per wave)
      v4f x = ld4(blk, lane);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int a = g4 + jj;
        if (a > r16) x[jj] = blk[4 * (a + 16 * (r16 >> 2)) + (r16 & 3)];
      }
      st4(blk, lane, x);
    }
    st4(sm + OFF_R + t * TF, lane, e);
  };
  if (w == 0) {
    store_blk(0, load_blk(0));
    if (lane < 2 * NTL) reinterpret_cast<int*>(sm + OFF_SYNC)[lane] = 0;
    PROF_STAMP(1, 0)
    factor_block(sm, 0, lane, info, row0);
    PROF_STAMP(2, 0)
  } else {
    // the S3 job table into LDS (full tiles only use it)
    for (int e = tid - 64; e < JOB_WORDS; e += NT - 64)
      reinterpret_cast<uint32_t*>(sm + OFF_JOB)[e] = (&kJobs.w[0][0])[e];
    constexpr int PER = (NLOW - 1 + 2) / 3;   // 12
    v4f v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = 1 + (w - 1) + 3 * u;
      if (t < NLOW) v[u] = load_blk(t);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int t = 1 + (w - 1) + 3 * u;
      if (t < NLOW) store_blk(t, v[u]);
    }
  }
  __syncthreads();

  // X output. A full tile (vec) keeps X in LDS and writes it after the last panel, all four
  // waves in parallel (per panel it sat on the critical S2 -> S3 path). A partial tile stores
  // block row p once S2 of panel p wrote it, from its writers (row 16 p + r16, columns
  // 16 k + g4 .. + 3 per lane, read back from the accumulator layout -- element (r, c) at lane
  // c + 16 (r >> 2), register r & 3), the zero blocks above the diagonal from the waves with
  // spare S2 slots.
  const bool xvec = vec;   // the host checks X's alignment and ldx into vec
  auto store_x = [&](int i, int k, const float* blk) {
    const int row = TT * i + r16, c0 = TT * k + g4;
    v4f x = {0.f, 0.f, 0.f, 0.f};
    if (blk != nullptr) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float e = blk[4 * (g4 + jj + 16 * (r16 >> 2)) + (r16 & 3)];
        x[jj] = i > k || g4 + jj <= r16 ? e : 0.f;
      }
    }
    if (xvec) {
      *reinterpret_cast<v4f*>(X + (int64_t)row * ldx + c0) = x;
    } else {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        if (row < n && c0 + jj < n) X[(int64_t)row * ldx + c0 + jj] = x[jj];
    }
  };

  // Panel p. S2 (<= 8 blocks): L_i^T = Z A_ip^T (i = p+1 .. ntl-1) and X_pk = Z R_pk
  // (k = 0 .. p). Wave 0 takes the first (L_{p+1}), updates the next diagonal block with it
  // (A_{p+1,p+1} -= L_{p+1} L_{p+1}^T: it needs no other wave's result), flags L_{p+1} and runs
  // S1 of panel p + 1 at once; waves 1-3 take the other S2 blocks, meet in an LDS counter (the
  // blocks they wrote, and wave 0's flag), then run S3 of panel p. One workgroup barrier per
  // panel: the S1 chain on wave 0 overlaps both S2 and S3 of the other waves.
  int* const arrive = reinterpret_cast<int*>(sm + OFF_SYNC);
  int* const lflag = arrive + NTL;
  for (int p = 0; p < ntl; ++p) {
    PROF_STAMP(30 + p, 0)
    const int nL = ntl - 1 - p, njobs = nL + p + 1;
    v4f zt;  // accumulator-layout block of Z^T: Z[r16][g4 + jj]
    {
      const float* zs = sm + ((p & 1) ? OFF_Z2 : OFF_Z);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) zt[jj] = zs[(g4 + jj) * TT + r16];
    }
    if (w == 0) {
      float* blk = nL > 0 ? sm + OFF_A + tix(p + 1, p) * TF : sm + OFF_R + tix(p, 0) * TF;
      const v4f o = mma16(v4f{0.f, 0.f, 0.f, 0.f}, zt, ld4(blk, lane));
      st4(blk, lane, o);
      if (nL == 0 && !vec) store_x(p, 0, blk);
      if (nL > 0) {
        float* d = sm + OFF_A + tix(p + 1, p + 1) * TF;
        st4(d, lane, ld4(d, lane) - mma16(v4f{0.f, 0.f, 0.f, 0.f}, o, o));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(lflag + p, 1, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        PROF_STAMP(3 + 4 * p, 0)
        factor_block(sm, p + 1, lane, info, row0);   // look-ahead: S1 of the next panel
        PROF_STAMP(5 + 4 * p, 0)
      }
    } else {
      // this wave's S3 job row (full tiles): uniform-address LDS reads, in flight during S2
      v4f jrow[JROW / 4];
      if (ntl == NTL && nL > 0) {
        const v4f* jr = reinterpret_cast<const v4f*>(sm + OFF_JOB + (3 * p + w - 1) * JROW);
#pragma unroll
        for (int c = 0; c < JROW / 4; ++c) jrow[c] = jr[c];
      }
      // S2 jobs t = w, w + 3, w + 6 (njobs <= 8, wave 0 has t = 0): all operands read first,
      // the three 4-MFMA chains interleaved, then the stores
      {
        float* blk[3];
        v4f b[3], o[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int t = w + 3 * u;
          blk[u] = t >= njobs ? sm + OFF_SCR
                   : t < nL   ? sm + OFF_A + tix(p + 1 + t, p) * TF
                              : sm + OFF_R + tix(p, t - nL) * TF;
          b[u] = ld4(blk[u], lane);
          o[u] = v4f{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int u = 0; u < 3; ++u)
            o[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(zt[st], b[u][st], o[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          const int t = w + 3 * u;
          if (t < njobs) {
            st4(blk[u], lane, o[u]);
            if (t >= nL && !vec) store_x(p, t - nL, blk[u]);
          }
        }
      }
      if (!vec)
        for (int k = p + w; k < ntl; k += 3)   // X_pk = 0 above the diagonal (k = p+1 ..)
          if (k > p) store_x(p, k, nullptr);
      PROF_STAMP(52 + p, 1)
      if (nL > 0) {
        // waves 1-3 meet: every S2 block written (LDS requests of a wave complete in order,
        // so a block is visible once its writer's arrival is), and L_{p+1} from wave 0
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(arrive + p, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);

        while (__hip_atomic_load(arrive + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 3 ||
               __hip_atomic_load(lflag + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
          __builtin_amdgcn_s_sleep(1);
        // acquire side: no LDS read of the S2 blocks / L_{p+1} may move above the spin (LDS
        // requests of the CU are coherent and in order; only the compiler can reorder them)
        asm volatile("" ::: "memory");
        PROF_STAMP(4 + 4 * p, 1)
        // S3 of panel p: A_{i,j} (q <= j <= i, but the diagonal block q done by wave 0) then
        // R_{i,k} (i >= q, k <= p), job n to wave 1 + n % 3, four at a time
        const int q = p + 1;
        const Job pad = {scratch, scratch, scratch};
        if (ntl == NTL) {   // the full tile: the precomputed job list (jrow, read above)
          auto word = [&](int e) { return __float_as_uint(jrow[e >> 2][e & 3]); };
          auto job = [&](int u) {
            const uint32_t da = word(2 * u);
            return Job{sm + (da & 0xffffu), sm + (da >> 16), sm + word(2 * u + 1)};
          };
          const uint32_t jn4 = word(2 * JMAX);
#pragma unroll
          for (int u = 0; u < JMAX; u += 4)
            if (u < (int)jn4) run4(job(u), job(u + 1), job(u + 2), job(u + 3), lane);
        } else {
          Job j0 = pad, j1 = pad, j2 = pad, j3 = pad;   // a shift register (no indexed array)
          int cnt = 0, jn = 0;
          auto push = [&](const Job& jb) {
            j3 = j2;
            j2 = j1;
            j1 = j0;
            j0 = jb;
            if (++cnt == 4) {
              run4(j0, j1, j2, j3, lane);
              cnt = 0;
            }
          };
          for (int i = q; i < ntl; ++i) {
            const float* li = sm + OFF_A + tix(i, p) * TF;           // L_i^T
            for (int jc = q; jc <= i; ++jc) {
              if (jc == q && i == q) continue;
              if (jn++ % 3 != w - 1) continue;
              // At(i, jc) = A_{i,jc}^T -= L_jc L_i^T: A operand L_jc (block L_jc^T), B L_i^T
              push(Job{sm + OFF_A + tix(i, jc) * TF, sm + OFF_A + tix(jc, p) * TF, li});
            }
            for (int k = 0; k <= p; ++k) {
              if (jn++ % 3 != w - 1) continue;
              // Rt(i, k) -= L_i X_pk: A operand L_i (block L_i^T), B operand X_pk
              push(Job{sm + OFF_R + tix(i, k) * TF, li, sm + OFF_R + tix(p, k) * TF});
            }
          }
          while (cnt) push(pad);   // the remainder, padded with no-op jobs
        }
        PROF_STAMP(6 + 4 * p, 1)
      }
    }
    __syncthreads();
  }
  PROF_STAMP(40, 0)

  // X of a full tile: every block row-major from LDS (store_x), the four waves in parallel;
  // the blocks above the diagonal are zeros
  if (vec) {
    // wave w: block rows w and w + 4; a row's LDS reads all issued before its stores
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = w + 4 * h;
      const float* rrow = sm + OFF_R + tix(i, 0) * TF + 4 * (g4 + 16 * (r16 >> 2)) + (r16 & 3);
      v4f xb[NTL];
#pragma unroll
      for (int k = 0; k < NTL; ++k) {
        xb[k] = v4f{0.f, 0.f, 0.f, 0.f};
        if (k <= i) {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            xb[k][jj] = k < i || g4 + jj <= r16 ? rrow[k * TF + 4 * jj] : 0.f;
        }
      }
      float* xr = X + (int64_t)(TT * i + r16) * ldx + g4;
#pragma unroll
      for (int k = 0; k < NTL; ++k) *reinterpret_cast<v4f*>(xr + TT * k) = xb[k];
    }
  }
  // L when asked for
  if (Lout) {
    for (int t = w; t < NTL * NTL; t += 4) {
      const int i = t >> 3, k = t & 7;
      if (i >= ntl || k >= ntl) continue;
      const int row = TT * i + r16, c0 = TT * k + g4;
      // L_ik = (block of L_ik^T)^T: lane l holds L[16 i + r16][16 k + g4 + jj]
      v4f l4 = {0.f, 0.f, 0.f, 0.f};
      if (i > k) {
        l4 = ld4(sm + OFF_A + tix(i, k) * TF, lane);
      } else if (i == k) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) l4[jj] = sm[OFF_L + i * TF + r16 * TT + g4 + jj];
      }
      if (vec) {
        *reinterpret_cast<v4f*>(Lout + (int64_t)row * ldl + c0) = l4;
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (row < n && c0 + jj < n) Lout[(int64_t)row * ldl + c0 + jj] = l4[jj];
      }
    }
  }
  PROF_STAMP(41, 0)
  PROF_REAL(43)
}

}  // namespace ctile
}  // namespace lcq

using namespace lcq;

extern "C" int lcq_chol_inv_tile(const void* A, int64_t lda, int n, void* L, int64_t ldl,
                                 void* X, int64_t ldx, void* info, int64_t row0, void* stream) {
  using namespace lcq::ctile;
  LCQ_REQUIRE(n > 0 && n <= CTILE && lda >= n && ldx >= n && (!L || ldl >= n),
              "tile must be 1..128 wide");
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec = n == CTILE && lda % 4 == 0 && al(A) && (!L || (ldl % 4 == 0 && al(L))) &&
                  ldx % 4 == 0 && al(X);
  // the dynamic-LDS attribute is per device: set it on every launch (cheap, thread-safe)
  (void)hipFuncSetAttribute((const void*)k_chol_inv_tile,
                            hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
  hipLaunchKernelGGL(k_chol_inv_tile, dim3(1), NT, LDS_BYTES, as_stream(stream),
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

// ---------------------------------------------------------------------------------------
// k_gemm_f32_small: the recursion's small products (M, N <= 512, K <= 1024, all multiples of
// 32 / 128: the 128- to 512-level updates of the chain), which as one to sixteen 64^2 LDS-DMA
// workgroups ran at 0.4-13 TF/s (~10 us for a 128^3 product, profiles/r6_chain_small.txt):
// latency of four dependent 32-k chunks on four CUs. Here one 32 x 32 output tile per
// 256-thread workgroup (4 x more workgroups), a 16 x 16 v_mfma_f32_16x16x4_f32 tile per wave,
// both operands straight from global memory (L2) into registers, four 32-k chunks per load
// batch with the next batch in flight under the current one's 32 MFMAs. The k order is the
// LDS-DMA kernels' (k_gemm_f32d_*: in 32-k chunk c, lane group g supplies k = 32 c + 8 g + s at
// step s), so every element gets the same fmaf chain and the products are bit-identical to
// the kernel they replace; epilogue C = beta C + alpha acc as there.
template <int BT>
__global__ void __launch_bounds__(256) k_gemm_f32_small(Args a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int64_t row = (int64_t)blockIdx.y * 32 + (w >> 1) * 16 + r16;
  const int64_t col = (int64_t)blockIdx.x * 32 + (w & 1) * 16 + r16;
  const float* ap = a.A + row * a.lda + 8 * g;
  const float* bp = BT ? a.B + col * a.ldb + 8 * g : a.B + (int64_t)(8 * g) * a.ldb + col;
  const int nb = (int)(a.K / 128);   // load batches of four 32-k chunks
  auto load = [&](int bt_, float (&av)[32], float (&bv)[32]) {
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int k0 = 128 * bt_ + 32 * cc;   // this lane's 8 k: k0 + 8 g + 0..7
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 v = *reinterpret_cast<const float4*>(ap + k0 + 4 * h);
        av[8 * cc + 4 * h] = v.x; av[8 * cc + 4 * h + 1] = v.y;
        av[8 * cc + 4 * h + 2] = v.z; av[8 * cc + 4 * h + 3] = v.w;
      }
      if constexpr (BT) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 v = *reinterpret_cast<const float4*>(bp + k0 + 4 * h);
          bv[8 * cc + 4 * h] = v.x; bv[8 * cc + 4 * h + 1] = v.y;
          bv[8 * cc + 4 * h + 2] = v.z; bv[8 * cc + 4 * h + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) bv[8 * cc + s] = bp[(int64_t)(k0 + s) * a.ldb];
      }
    }
  };
  v4f32 acc = {0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const float (&av)[32], const float (&bv)[32]) {
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
  };
  float a0[32], b0[32], a1[32], b1[32];
  load(0, a0, b0);
  for (int c = 0; c < nb; c += 2) {
    if (c + 1 < nb) load(c + 1, a1, b1);
    mma(a0, b0);
    if (c + 1 < nb) {
      if (c + 2 < nb) load(c + 2, a0, b0);
      mma(a1, b1);
    }
  }
  // 16x16 MFMA tile: lane holds column r16, rows 4 g + v
  const int64_t c_out = (int64_t)blockIdx.x * 32 + (w & 1) * 16 + r16;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int64_t r = (int64_t)blockIdx.y * 32 + (w >> 1) * 16 + 4 * g + v;
    float* p = a.C + r * a.ldc + c_out;
    const float val = a.alpha * acc[v];
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

// plan_m: the row count the kernel variant (tile size, LDS-DMA or register staging) is chosen
// for -- M itself, or the full product's rows when this launch computes a row range of it
// (lcq_gemm_f32_rows: the same variant, hence the same per-element k order, on every rank)
// k_gemm_f32_small's range (probe builds vary it: -DLCQ_PROBE_SMALL_MN / _K)
#ifndef LCQ_PROBE_SMALL_MN
#define LCQ_PROBE_SMALL_MN 512
#endif
#ifndef LCQ_PROBE_SMALL_K
#define LCQ_PROBE_SMALL_K 1024
#endif
constexpr int64_t SMALL_MN = LCQ_PROBE_SMALL_MN, SMALL_K = LCQ_PROBE_SMALL_K;

static int gemm_f32_impl(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                         int64_t lda, const void* B, int64_t ldb, int bt, float beta, void* C,
                         int64_t ldc, void* ws, int64_t ws_bytes, void* stream,
                         int64_t plan_m = -1) {
  if (plan_m < 0) plan_m = M;
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
  // the small products of the chain: 32 x 32 tiles from registers (k_gemm_f32_small); a
  // whole-product launch only (plan_m == M), so row-range launches never change kernel
  if (plan_m == M && M <= SMALL_MN && N <= SMALL_MN && K >= 128 && K <= SMALL_K && M % 32 == 0 &&
      N % 32 == 0 && K % 128 == 0 && a.vec) {
    const dim3 grid((unsigned)(N / 32), (unsigned)(M / 32));
    if (bt) hipLaunchKernelGGL(f32g::k_gemm_f32_small<1>, grid, 256, 0, st, a);
    else hipLaunchKernelGGL(f32g::k_gemm_f32_small<0>, grid, 256, 0, st, a);
    return check_launch("lcq_gemm_f32: small");
  }
  // 128^2 tiles where they fill the chip, 64^2 below (4x the workgroups)
  const int64_t t128 = ((N + 127) / 128) * ((plan_m + 127) / 128);
  const bool big = t128 >= 256;
  // LDS-DMA kernel: K % 32 == 0, 16-byte aligned rows, 32-bit byte offsets
  // ldc % 4 == 0 with al(C): the choice is the same for every row range of C (a shifted C of
  // lcq_gemm_f32_rows stays aligned), so the ranks of a row split run one kernel
  const bool dma = K % f32g::DKC == 0 && a.vec && al(C) && ldc % 4 == 0 &&
                   plan_m * lda < ((int64_t)1 << 29) &&
                   (bt ? N * ldb : K * ldb) < ((int64_t)1 << 29);
  if (dma && ws != nullptr && ws_bytes >= sk_ws_bytes() && plan_m == M &&
      use_stream_k(M, N, K)) {
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

extern "C" int64_t lcq_gemm_f32_row_unit(int64_t M, int64_t N) {
  return ((N + 127) / 128) * ((M + 127) / 128) >= 256 ? 128 : 64;
}

extern "C" int lcq_gemm_f32_rows(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                                 int64_t lda, const void* B, int64_t ldb, int bt, float beta,
                                 void* C, int64_t ldc, int64_t row0, int64_t row1,
                                 void* stream) {
  const int64_t unit = lcq_gemm_f32_row_unit(M, N);
  LCQ_REQUIRE(0 <= row0 && row0 <= row1 && row1 <= M, "row range outside [0, M]");
  LCQ_REQUIRE(row0 % unit == 0 && (row1 % unit == 0 || row1 == M),
              "row range must be cut on the plan's tile rows (lcq_gemm_f32_row_unit)");
  if (row1 == row0) return LCQ_OK;
  LCQ_REQUIRE(A != nullptr && C != nullptr, "null pointers");
  const float* Ar = reinterpret_cast<const float*>(A) + row0 * lda;
  float* Cr = reinterpret_cast<float*>(C) + row0 * ldc;
  return gemm_f32_impl(row1 - row0, N, K, alpha, Ar, lda, B, ldb, bt, beta, Cr, ldc, nullptr, 0,
                       stream, M);
}

extern "C" int lcq_gemm_f32_ws(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                               int64_t lda, const void* B, int64_t ldb, int bt, float beta,
                               void* C, int64_t ldc, void* workspace, int64_t ws_bytes,
                               void* stream) {
  return gemm_f32_impl(M, N, K, alpha, A, lda, B, ldb, bt, beta, C, ldc, workspace, ws_bytes,
                       stream);
}
