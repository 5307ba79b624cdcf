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
#include "lcq_fp8.h"

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
  float* err;         // k-major [128][ld_err]: err[k ld_err + row]
  int64_t ld_err;
  float* losses;      // optional [rows, ld]
  const int32_t* cgroup;  // static groups: group of every (permuted) column, [ld]
  int64_t ngc;            // static groups: groups per row of s_in / z_in
  // left-looking near updates: the k-major errors [nprev * 128][ld_err] of the nprev full
  // blocks right before col0 (columns col0 - 128 nprev .. col0 - 1 of the superblock)
  const float* err_prev;
  int nprev;
};

// 16 lanes per row, 8 consecutive block columns per lane (16 rows per 256-thread workgroup:
// a 4096-row linear is 256 workgroups; with 8 lanes x 16 columns it was 128, half the chip,
// each lane carrying twice the updates per column). Column c's owner lane (c / 8) quantizes
// it; its error is broadcast to the row's other 15 lanes with one shuffle; every lane applies
// the rank-1 update to its own columns > c -- the same per-element operations in any layout,
// so the result is unchanged bit for bit. W, err and losses are written once at the end with
// 16-byte stores (a row's 16 lanes cover 512 contiguous bytes). err is written k-major
// ([128][rows]) for the trailing GEMM's staging.
constexpr int LPR = 16, CPL = GB / LPR;

// FMT = 0: IntegerQuantizer (quant.py:699-717); FMT = LCQ_FP8E4M3 / LCQ_FP8E5M2: FloatQuantizer
// use_qtorch (quant.py:1061-1080): q = float_quantize(w / s + 0) * s in fp32, sym qparams with
// qmax = finfo.max (per-group: the same fp32 formula as the int sym case).
// The U block lives in LDS as its upper triangle, row c from column ustart(c) = c & ~3 (so
// every row segment stays 16-byte aligned): 8448 floats, 33 KB instead of 64, so four
// workgroups share a CU (the 28672-row gate / up blocks: 1792 workgroups) instead of two. A
// lane's float4 of columns below ustart(c) reads the previous row's tail: those columns are
// < c and never updated.
constexpr int ustart(int c) { return c & ~3; }
constexpr int ubase(int c) {  // sum over rows i < c of (GB - ustart(i))
  return GB * c - 8 * (c >> 2) * ((c >> 2) - 1) - 4 * (c >> 2) * (c & 3);
}
constexpr int UPACK = ubase(GB);
static_assert(UPACK >= 64 * 132, "a staged U half of the near updates fits the U block's LDS");

typedef float v4f __attribute__((ext_vector_type(4)));

// The near updates of the superblock, left-looking (gptq.py:244 restricted to this block's
// columns): for every earlier block j of the superblock, in order,
//   W[:, block] -= Err_j @ U[rows of j, block]
// each product an fp32 MFMA chain over k = 0 .. 127 in order (v_mfma_f32_16x16x4_f32, lane
// group g supplying k = 4 s + g at step s: the k-ordered fmaf chain of lcq_gptq_trailing's
// kernels, bit for bit), rounded, then subtracted -- the same per-element operations, in the
// same order, as one lcq_gptq_trailing launch after each earlier block, without those launches
// and their dependent-kernel gaps. U_j goes through LDS (the U block's area, staged only
// afterwards) in halves of 64 k-rows x 128 columns, rows padded to 132 floats (the four lane
// groups of a B read hit distinct banks), the next half prefetched into registers while the
// current one is multiplied; each wave computes 16 rows x 32 columns; the product tile goes
// back through LDS to the row-per-16-lanes layout of the loop.
constexpr int NU_LD = 132;   // padded row of a staged U half (64 x 132 floats = UPACK)

__device__ __forceinline__ void nu_fetch(const GptqArgs& a, int j, int half, int tid,
                                         float4 (&pf)[8]) {
  const float* src = a.U + (a.col0 - (int64_t)(a.nprev - j) * GB + 64 * half) * a.ldu + a.col0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {   // 2048 float4 of 64 rows x 32 float4
    const int idx = q * 256 + tid, row = idx >> 5, c4 = (idx & 31) * 4;
    pf[q] = c4 < a.count ? *reinterpret_cast<const float4*>(src + (int64_t)row * a.ldu + c4)
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

__device__ __forceinline__ void near_updates(const GptqArgs& a, float (&w)[8], float* lds,
                                             int tid, int64_t rbase, int cb) {
  const int lane = tid & 63, wv = tid >> 6, r16 = lane & 15, g = lane >> 4;
  const int64_t arow = rbase + r16;
  const bool arow_ok = arow < a.rows;
  const int c0 = 32 * wv + r16, c1 = c0 + 16;
  const int rloc = tid >> 4;
  float4 pf[8];
  nu_fetch(a, 0, 0, tid, pf);
  for (int j = 0; j < a.nprev; ++j) {
    const float* ej = a.err_prev + (int64_t)j * GB * a.ld_err + (arow_ok ? arow : 0);
    v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float av[16];
#pragma unroll
      for (int st = 0; st < 16; ++st)
        av[st] = arow_ok ? ej[(int64_t)(64 * half + 4 * st + g) * a.ld_err] : 0.f;
      __syncthreads();   // the previous half / product tile has been read
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int idx = q * 256 + tid, row = idx >> 5, c4 = (idx & 31) * 4;
        *reinterpret_cast<float4*>(lds + row * NU_LD + c4) = pf[q];
      }
      __syncthreads();
      if (half == 0) nu_fetch(a, j, 1, tid, pf);
      else if (j + 1 < a.nprev) nu_fetch(a, j + 1, 0, tid, pf);
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const float* br = lds + (4 * st + g) * NU_LD;
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[st], br[c0], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[st], br[c1], acc1, 0, 0, 0);
      }
    }
    __syncthreads();   // the second half has been read
#pragma unroll
    for (int v = 0; v < 4; ++v) {   // lane: column r16 of its tile, rows 4 g + v
      lds[(4 * g + v) * NU_LD + c0] = acc0[v];
      lds[(4 * g + v) * NU_LD + c1] = acc1[v];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CPL; ++k)
      if (cb + k < a.count) w[k] = w[k] - lds[rloc * NU_LD + cb + k];
  }
  __syncthreads();   // LDS free for the U block
}

template <int GS, int FMT>
__global__ void __launch_bounds__(256) k_gptq_block(GptqArgs a) {
  __shared__ __attribute__((aligned(16))) float u[UPACK];
  const int tid = threadIdx.x;
  const int sub = tid & (LPR - 1);
  const int64_t r = (int64_t)blockIdx.x * (256 / LPR) + (tid / LPR);
  const bool valid = r < a.rows;  // invalid lanes still run (shuffles), never store
  const int cb = sub * CPL;       // first block column of this lane
  float* wrow = a.W + (valid ? r : 0) * a.ld + a.col0;
  float w[CPL];
#pragma unroll
  for (int k = 0; k < CPL; k += 4) {
    if (valid && cb + k + 3 < a.count) {
      const float4 v = *reinterpret_cast<const float4*>(wrow + cb + k);
      w[k] = v.x; w[k + 1] = v.y; w[k + 2] = v.z; w[k + 3] = v.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) w[k + q] = (valid && cb + k + q < a.count) ? wrow[cb + k + q] : 0.f;
    }
  }
  if (a.nprev > 0) near_updates(a, w, u, tid, (int64_t)blockIdx.x * (256 / LPR), cb);
  for (int i = tid >> 1; i < GB; i += 128) {   // two threads per row, 16-B pieces
    for (int j4 = (i >> 2) + (tid & 1); j4 < GB / 4; j4 += 2) {
      const int j = 4 * j4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < a.count) {
        const float* src = a.U + (a.col0 + i) * a.ldu + a.col0 + j;
        if (j + 3 < a.count) {
          v = *reinterpret_cast<const float4*>(src);
        } else {
          if (j + 0 < a.count) v.x = src[0];
          if (j + 1 < a.count) v.y = src[1];
          if (j + 2 < a.count) v.z = src[2];
        }
      }
      *reinterpret_cast<float4*>(&u[ubase(i) + j - ustart(i)]) = v;
    }
  }
  __syncthreads();
  // group qparams from the block-start weights (gptq.py:215-223 reads W, not W1); GS >= 32
  // so a lane's 8 columns lie in one group of GS / 8 adjacent lanes
  float qs, qz;
  if constexpr (GS > 0) {
    constexpr int LG = GS / CPL;  // lanes per group (4, 8, 16)
    float mn = INFINITY, mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < CPL; ++k)
      if (cb + k < a.count) {  // a group cut by the end of the columns uses its valid part
        mn = fminf(mn, w[k]);
        mx = fmaxf(mx, w[k]);
      }
#pragma unroll
    for (int m = LG / 2; m >= 1; m >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, m, 64));
      mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    }
    qparams_f32(mn, mx, a.qmin, a.qmax, a.sym, qs, qz);
    if (valid && (sub % LG) == 0 && cb < a.count) {
      const int64_t gi = (a.col0 + cb) / GS;
      a.s_out[r * a.ng_total + gi] = qs;
      if (a.z_out && !a.sym) a.z_out[r * a.ng_total + gi] = qz;
    }
  } else {
    qs = valid ? a.s_in[r] : 1.f;
    qz = (valid && a.z_in) ? a.z_in[r] : 0.f;
  }
  // static groups (GS < 0, gptq.py:224-227): column c takes the precomputed qparams of its
  // ORIGINAL group, groups[perm[c] // group_size] -- per column, held per lane
  float qsk[GS < 0 ? CPL : 1], qzk[GS < 0 ? CPL : 1];
  if constexpr (GS < 0) {
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int g = (cb + k < a.count) ? a.cgroup[a.col0 + cb + k] : 0;
      qsk[k] = valid ? a.s_in[r * a.ngc + g] : 1.f;
      qzk[k] = (valid && a.z_in) ? a.z_in[r * a.ngc + g] : 0.f;
    }
  }
  float ek[CPL], lk[CPL];
  const int rowlane = tid & ~(LPR - 1);
#pragma unroll
  for (int c = 0; c < GB; ++c) {
    if (c < a.count) {
      const int owner = c / CPL, jl = c % CPL;
      // every lane evaluates its own column jl; only the owner's value is used
      const float d = u[ubase(c) + c - ustart(c)];
      const float wc = w[jl];
      const float cs = (GS < 0) ? qsk[jl] : qs, cz = (GS < 0) ? qzk[jl] : qz;
      float q;
      if constexpr (FMT == 0) {
        float t = rintf(wc / cs);
        t = t + cz;
        t = fminf(fmaxf(t, a.qmin), a.qmax);
        q = (t - cz) * cs;
      } else {
        q = fp8_round<FMT>(wc / cs + 0.0f) * cs;
      }
      const float diff = wc - q;
      const float e = __shfl(diff / d, rowlane | owner, 64);
      if (sub == owner) {
        ek[jl] = e;
        lk[jl] = (diff * diff) / (2.f * (d * d));
      }
      const bool ge = sub >= owner, gt = sub > owner;
      const float* urow = u + ubase(c) - ustart(c) + cb;
#pragma unroll
      for (int k = 0; k < CPL; k += 4) {
        const float4 uv = *reinterpret_cast<const float4*>(urow + k);
        const float uu[4] = {uv.x, uv.y, uv.z, uv.w};
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const bool upd = (k + q4 > jl) ? ge : gt;  // block column cb + k + q4 > c
          const float nw = w[k + q4] - e * uu[q4];
          w[k + q4] = upd ? nw : w[k + q4];
        }
      }
    } else {
      const int jl = c % CPL;
      if (sub == c / CPL) {
        ek[jl] = 0.f;
        lk[jl] = 0.f;
      }
    }
  }
  if (!valid) return;
  // tmp1 / Err1 / Losses1 (gptq.py:234-238): w[k] is final once its column was processed
#pragma unroll
  for (int k = 0; k < CPL; k += 4) {
    if (cb + k + 3 < a.count) {
      *reinterpret_cast<float4*>(wrow + cb + k) = make_float4(w[k], w[k + 1], w[k + 2], w[k + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (cb + k + q < a.count) wrow[cb + k + q] = w[k + q];
    }
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) a.err[(int64_t)(cb + k) * a.ld_err + r] = ek[k];
  if (a.losses) {
#pragma unroll
    for (int k = 0; k < CPL; k += 4)
      if (cb + k + 3 < a.count) {
        *reinterpret_cast<float4*>(a.losses + r * a.ld + a.col0 + cb + k) =
            make_float4(lk[k], lk[k + 1], lk[k + 2], lk[k + 3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (cb + k + q < a.count) a.losses[r * a.ld + a.col0 + cb + k + q] = lk[k + q];
      }
  }
}

}  // namespace lcq

using namespace lcq;

template <int FMT>
static void launch_gptq_block(const GptqArgs& a, int64_t group, dim3 grid, hipStream_t st) {
  switch (group) {
    case 32: hipLaunchKernelGGL((k_gptq_block<32, FMT>), grid, 256, 0, st, a); break;
    case 64: hipLaunchKernelGGL((k_gptq_block<64, FMT>), grid, 256, 0, st, a); break;
    case 128: hipLaunchKernelGGL((k_gptq_block<128, FMT>), grid, 256, 0, st, a); break;
    default: hipLaunchKernelGGL((k_gptq_block<0, FMT>), grid, 256, 0, st, a); break;
  }
}

extern "C" int lcq_gptq_block(void* W, int64_t rows, int64_t ld, int64_t col0, int count,
                              const void* U, int64_t ldu, int64_t group, int qmin, int qmax,
                              int sym, int fmt, const void* s_in, const void* z_in, void* s_out,
                              void* z_out, int64_t ng_total, void* err, int64_t ld_err,
                              void* losses, const void* err_prev, int nprev, void* stream) {
  LCQ_REQUIRE(rows > 0 && ld > 0 && count > 0 && count <= GB, "bad block shape");
  LCQ_REQUIRE(nprev >= 0 && (nprev == 0 || err_prev != nullptr) && col0 >= (int64_t)nprev * GB,
              "nprev earlier blocks need err_prev and col0 >= 128 nprev");
  LCQ_REQUIRE(col0 >= 0 && col0 + count <= ld && col0 + count <= ldu, "block out of range");
  LCQ_REQUIRE(col0 % GB == 0, "col0 must be a multiple of the 128-column blocksize");
  LCQ_REQUIRE(ld % 4 == 0 && ldu % 4 == 0, "row lengths must be multiples of 4 (16-B rows)");
  LCQ_REQUIRE(fmt == 0 || fmt == LCQ_FP8E4M3 || fmt == LCQ_FP8E5M2,
              "fmt must be 0 (integer) or an fp8 format");
  if (fmt != 0) {  // FloatQuantizer: symmetric, qmax = finfo.max, no zero point
    qmin = fmt == LCQ_FP8E4M3 ? -448 : -57344;
    qmax = -qmin;
    sym = 1;
    z_in = nullptr;
    z_out = nullptr;
  }
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
  a.ld_err = ld_err;
  a.losses = reinterpret_cast<float*>(losses);
  a.err_prev = reinterpret_cast<const float*>(err_prev);
  a.nprev = nprev;
  LCQ_REQUIRE(ld_err >= rows, "ld_err < rows");
  LCQ_REQUIRE(group == 0 || group == 32 || group == 64 || group == 128,
              "group must be 0 (per-row qparams), 32, 64 or 128");
  LCQ_REQUIRE(group != 0 || s_in != nullptr, "fixed-qparams mode needs s_in");
  const dim3 grid((unsigned)((rows + (256 / LPR) - 1) / (256 / LPR)));
  hipStream_t st = as_stream(stream);
  if (fmt == LCQ_FP8E4M3) launch_gptq_block<LCQ_FP8E4M3>(a, group, grid, st);
  else if (fmt == LCQ_FP8E5M2) launch_gptq_block<LCQ_FP8E5M2>(a, group, grid, st);
  else launch_gptq_block<0>(a, group, grid, st);
  return check_launch("lcq_gptq_block");
}

// ---------------------------------------------------------------------------------------
// GPTQ trailing update  W[:, c1:] -= E[:, :cnt] @ U[c0:c0+cnt, c1:]   (gptq.py:244)
// fp32 MFMA v_mfma_f32_32x32x2_f32: bit-for-bit a k-ordered fmaf chain, so every output
// element's value is independent of the tiling / row range (row-sharded GPTQ on N GPUs is
// bit-identical to one GPU). The product is rounded to fp32 and then subtracted, like the
// reference's `W -= Err @ Hinv` (two roundings). 128x128 output tile per 256-thread
// workgroup (2x2 waves of 64x64 = 2x2 MFMA 32x32 tiles); K in 32-deep chunks, double-
// buffered through 64 KB of LDS with register staging (the next chunk's loads overlap the
// current chunk's MFMAs; 2 workgroups per CU). err arrives k-major [128][rows] from
// lcq_gptq_block and U rows are k-major, so both stage with conflict-free 16-byte copies.
// ---------------------------------------------------------------------------------------
namespace lcq {

typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int TT = 128;   // output tile

constexpr int KC = 32;     // K chunk (double-buffered through LDS)

__device__ __forceinline__ void trail_load(const float* __restrict__ ET, const float* __restrict__ U,
                                           int64_t rows, int64_t ld, int64_t ldu, int64_t c0,
                                           int cnt, int64_t r0, int64_t j0, int k0, int tid,
                                           float4 (&ra)[4], float4 (&rb)[4], int64_t lde) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = it * 256 + tid;           // 0..1023 float4 of a 32 x 128 chunk
    const int k = k0 + idx / (TT / 4), c4 = (idx % (TT / 4)) * 4;
    float4 ea = make_float4(0.f, 0.f, 0.f, 0.f), ub = ea;
    if (k < cnt) {
      const float* es = ET + (int64_t)k * lde + r0 + c4;
      if (r0 + c4 + 3 < rows && (lde & 3) == 0) {
        ea = *reinterpret_cast<const float4*>(es);
      } else {
        if (r0 + c4 + 0 < rows) ea.x = es[0];
        if (r0 + c4 + 1 < rows) ea.y = es[1];
        if (r0 + c4 + 2 < rows) ea.z = es[2];
        if (r0 + c4 + 3 < rows) ea.w = es[3];
      }
      const float* us = U + (c0 + k) * ldu + j0 + c4;
      if (j0 + c4 + 3 < ld) {
        ub = *reinterpret_cast<const float4*>(us);
      } else {
        if (j0 + c4 + 0 < ld) ub.x = us[0];
        if (j0 + c4 + 1 < ld) ub.y = us[1];
        if (j0 + c4 + 2 < ld) ub.z = us[2];
      }
    }
    ra[it] = ea;
    rb[it] = ub;
  }
}

__global__ void __launch_bounds__(256, 2)
    k_gptq_trailing(float* __restrict__ W, int64_t rows, int64_t ld, int64_t c0, int cnt,
                    int64_t c1, int64_t c2, const float* __restrict__ ET, int64_t lde,
                    const float* __restrict__ U, int64_t ldu) {
  __shared__ __attribute__((aligned(16))) float As[2][KC * TT];  // [k][row]
  __shared__ __attribute__((aligned(16))) float Bs[2][KC * TT];  // [k][col]
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
  float4 ra[4], rb[4];
  trail_load(ET, U, rows, c2, ldu, c0, cnt, r0, j0, 0, tid, ra, rb, lde);
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = it * 256 + tid;
    *reinterpret_cast<float4*>(&As[0][idx * 4]) = ra[it];
    *reinterpret_cast<float4*>(&Bs[0][idx * 4]) = rb[it];
  }
  __syncthreads();
  const int nch = (cnt + KC - 1) / KC;
  for (int ch = 0; ch < nch; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < nch)
      trail_load(ET, U, rows, c2, ldu, c0, cnt, r0, j0, (ch + 1) * KC, tid, ra, rb, lde);
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      const int k = kk + (lane >> 5);
      float av[2], bv[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        av[t] = As[cur][k * TT + wr * 64 + t * 32 + (lane & 31)];
        bv[t] = Bs[cur][k * TT + wc * 64 + t * 32 + (lane & 31)];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb)
          acc[ta][tb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[ta], bv[tb], acc[ta][tb], 0, 0, 0);
    }
    if (ch + 1 < nch) {
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int idx = it * 256 + tid;
        *reinterpret_cast<float4*>(&As[cur ^ 1][idx * 4]) = ra[it];
        *reinterpret_cast<float4*>(&Bs[cur ^ 1][idx * 4]) = rb[it];
      }
    }
    __syncthreads();
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
        if (r < rows && c < c2) W[r * ld + c] = W[r * ld + c] - acc[ta][tb][reg];
      }
}

}  // namespace lcq

extern "C" int lcq_gptq_trailing(void* W, int64_t rows, int64_t ld, int64_t c0, int cnt,
                                 int64_t c1, int64_t c2, const void* err, int64_t ld_err,
                                 const void* U, int64_t ldu, void* stream) {
  LCQ_REQUIRE(rows > 0 && ld > 0 && cnt > 0 && cnt <= 8192, "bad shape");
  LCQ_REQUIRE(ld_err >= rows, "ld_err < rows");
  LCQ_REQUIRE(c0 >= 0 && c0 + cnt <= ldu && c1 >= c0 + cnt && c2 >= c1 && c2 <= ld &&
                  ld <= ldu,
              "bad column ranges");
  if (c2 == c1) return LCQ_OK;
  // the recursion's LDS-DMA fp32 GEMM (A k-major) where the operands are 16-byte aligned and
  // cnt % 32 == 0 -- decided by the column window and the strides only, never by the row count,
  // so a row shard takes the same kernel (and the same k order) as the whole matrix
  const float* Up = reinterpret_cast<const float*>(U) + c0 * ldu + c1;
  float* Wp = reinterpret_cast<float*>(W) + c1;
  const int rc = lcq::gemm_f32_sub_akn(rows, c2 - c1, cnt, reinterpret_cast<const float*>(err),
                                       ld_err, Up, ldu, Wp, ld, as_stream(stream));
  if (rc != LCQ_EUNSUP) return rc;
  const dim3 grid((unsigned)((c2 - c1 + TT - 1) / TT), (unsigned)((rows + TT - 1) / TT));
  hipLaunchKernelGGL(k_gptq_trailing, grid, 256, 0, as_stream(stream),
                     reinterpret_cast<float*>(W), rows, ld, c0, cnt, c1, c2,
                     reinterpret_cast<const float*>(err), ld_err,
                     reinterpret_cast<const float*>(U), ldu);
  return check_launch("lcq_gptq_trailing");
}

extern "C" int lcq_gptq_block_cols(void* W, int64_t rows, int64_t ld, int64_t col0, int count,
                                   const void* U, int64_t ldu, int qmin, int qmax,
                                   const void* s_in, const void* z_in, const int32_t* col_group,
                                   int64_t ngc, void* err, int64_t ld_err, void* losses,
                                   const void* err_prev, int nprev, void* stream) {
  LCQ_REQUIRE(rows > 0 && ld > 0 && count > 0 && count <= GB, "bad block shape");
  LCQ_REQUIRE(nprev >= 0 && (nprev == 0 || err_prev != nullptr) && col0 >= (int64_t)nprev * GB,
              "nprev earlier blocks need err_prev and col0 >= 128 nprev");
  LCQ_REQUIRE(col0 >= 0 && col0 + count <= ld && col0 + count <= ldu, "block out of range");
  LCQ_REQUIRE(col0 % GB == 0, "col0 must be a multiple of the 128-column blocksize");
  LCQ_REQUIRE(ld % 4 == 0 && ldu % 4 == 0, "row lengths must be multiples of 4 (16-B rows)");
  LCQ_REQUIRE(qmax > qmin, "qmax <= qmin");
  LCQ_REQUIRE(s_in != nullptr && col_group != nullptr && ngc > 0, "static groups need qparams");
  GptqArgs a{};
  a.W = reinterpret_cast<float*>(W);
  a.rows = rows; a.ld = ld; a.col0 = col0; a.count = count;
  a.U = reinterpret_cast<const float*>(U); a.ldu = ldu;
  a.qmin = (float)qmin; a.qmax = (float)qmax;
  a.s_in = reinterpret_cast<const float*>(s_in);
  a.z_in = reinterpret_cast<const float*>(z_in);
  a.cgroup = col_group; a.ngc = ngc;
  LCQ_REQUIRE(ld_err >= rows, "ld_err < rows");
  a.err = reinterpret_cast<float*>(err);
  a.ld_err = ld_err;
  a.losses = reinterpret_cast<float*>(losses);
  a.err_prev = reinterpret_cast<const float*>(err_prev);
  a.nprev = nprev;
  const dim3 grid((unsigned)((rows + (256 / LPR) - 1) / (256 / LPR)));
  hipLaunchKernelGGL((k_gptq_block<-1, 0>), grid, 256, 0, as_stream(stream), a);
  return check_launch("lcq_gptq_block_cols");
}

