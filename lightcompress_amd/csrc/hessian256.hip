// GPTQ Hessian H <- beta*H + alpha * X^T X on gfx950 MFMA: 256x256-tile SYRK.
//
// Reference: GPTQ.add_batch (llmc/compression/quantization/gptq.py:253-295):
//   H *= n/(n+b); n += b; x = sqrt(2/n) * x.float(); H += x @ x.T   (full fp32 GEMM)
// Here: one bf16 MFMA pass over the upper-triangle tiles only (half the reference's flops),
// exact bf16 products accumulated in fp32, epilogue beta*H + alpha*acc, mirrored.
//
// Structure (cdna_hip_programming.md §5 "256^2 8-phase template"):
//  * Pass 1 (k_xt_pack): X [n][ic] (token-major, as the forward hook hands it over) is
//    transposed into a zero-padded workspace XT [icp][kp] (icp = ceil256(ic), kp = ceil64(n)),
//    so both MFMA operands are k-contiguous rows (A = B = XT panels).
//  * Pass 2 (k_syrk256): one 512-thread workgroup (8 waves, 2(M) x 4(N)) per 256x256 output
//    tile of the upper triangle; each wave owns 128x64 = 8x4 accumulators of
//    mfma_f32_16x16x32_bf16. K-tile = 64. The A and B tiles of a K-tile are split into four
//    16 KB half-tiles in the order the four phases consume them (A_lo, B_lo | B_hi | A_hi | B_lo)
//    and staged by global_load_lds_dwordx4 (LDS image lane-linear, swizzle st_16x32 applied on
//    the global source address) into two LDS buffers (128 KB, one __shared__ array). The two
//    wave rows run one barrier apart (MFMA of one overlaps ds_reads of the other on each
//    SIMD); loads stay ~4 phases in flight across barriers, counted `s_waitcnt vmcnt(8)`,
//    raw s_barrier, never vmcnt(0) in the loop.
//  * Tile order is XCD-aware: each XCD's 32 concurrent workgroups take a 4x8 block of tiles
//    (bijective blockIdx remap + slot_tile), so 12 operand panels feed 32 tiles from L2.
//  * Split-K over `ns` slabs (count from a round-filling cost model, plan()) written to the
//    workspace and combined in a fixed order by k_syrk_reduce (deterministic: no float atomics).
#include "lcq_common.h"

#include <stdlib.h>

namespace lcq {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int ST = 256;          // output tile
constexpr int SKT = 64;          // K-tile (bf16 elements)
constexpr int HALF_B = 16384;    // bytes per half-tile: 128 rows x 64 k x 2 B
constexpr int BUF_B = 4 * HALF_B;  // one K-tile: A_lo, A_hi, B_lo, B_hi
enum { H_ALO = 0, H_AHI = 1, H_BLO = 2, H_BHI = 3 };

// ---------------------------------------------------------------------------------------
// pass 1: XT[c][k] = X[k][c] (bf16 / f16 bits), zero padded to [icp][kp]
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_xt_pack(const uint16_t* __restrict__ X, int64_t n,
                                                 int64_t ic, uint16_t* __restrict__ XT,
                                                 int64_t icp, int64_t kp) {
  // 64 tokens x 128 channels through LDS with a 65-dword row stride: the load phase stores 16 B
  // per chunk as 4 dwords, the store phase reads one dword = 2 channels of a token, so a lane
  // builds 8 tokens of 2 channels (two 16-B row pieces) from 8 dword reads; lanes (k8 = lane
  // & 7, channel pair = lane >> 3) hit 64 distinct banks and 8 lanes write 128 contiguous
  // bytes of an XT row (was: 16-bit reads, 16 per 16-B piece)
  __shared__ uint32_t t[64][65];
  const int64_t k0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 128;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int idx = it * 256 + tid;     // 0..1023: token r, channels c8 .. c8 + 7
    const int r = idx >> 4, c8 = (idx & 15) * 8;
    const int64_t k = k0 + r, c = c0 + c8;
    uint4 q = make_uint4(0, 0, 0, 0);
    if (k < n) {
      if (c + 7 < ic && (ic & 7) == 0) {
        q = *reinterpret_cast<const uint4*>(X + k * ic + c);
      } else {
        uint16_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c + j < ic) v[j] = X[k * ic + c + j];
        q.x = v[0] | ((uint32_t)v[1] << 16); q.y = v[2] | ((uint32_t)v[3] << 16);
        q.z = v[4] | ((uint32_t)v[5] << 16); q.w = v[6] | ((uint32_t)v[7] << 16);
      }
    }
    t[r][c8 / 2 + 0] = q.x;
    t[r][c8 / 2 + 1] = q.y;
    t[r][c8 / 2 + 2] = q.z;
    t[r][c8 / 2 + 3] = q.w;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k8 = (tid & 7) * 8, cp = (tid >> 3) + 32 * h;  // channels 2cp, 2cp + 1
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = t[k8 + j][cp];
    uint4 lo, hi;
    lo.x = (w[0] & 0xffffu) | (w[1] << 16); hi.x = (w[0] >> 16) | (w[1] & 0xffff0000u);
    lo.y = (w[2] & 0xffffu) | (w[3] << 16); hi.y = (w[2] >> 16) | (w[3] & 0xffff0000u);
    lo.z = (w[4] & 0xffffu) | (w[5] << 16); hi.z = (w[4] >> 16) | (w[5] & 0xffff0000u);
    lo.w = (w[6] & 0xffffu) | (w[7] << 16); hi.w = (w[6] >> 16) | (w[7] & 0xffff0000u);
    *reinterpret_cast<uint4*>(XT + (c0 + 2 * cp) * kp + k0 + k8) = lo;
    *reinterpret_cast<uint4*>(XT + (c0 + 2 * cp + 1) * kp + k0 + k8) = hi;
  }
}

// upper-triangle tile index -> (ti, tj), row-major over ti
__device__ __forceinline__ void tri_tile(int idx, int nt, int& ti, int& tj) {
  int i = 0, rem = idx;
  while (rem >= nt - i) {
    rem -= nt - i;
    ++i;
  }
  ti = i;
  tj = i + rem;
}

// work slot -> tile. Slots come in chunks of 32 = a 4 (tile rows) x 8 (tile cols) block of the
// upper triangle, walked band by band (4 tile rows per band). With the XCD remap the 32 CUs of
// one XCD run one chunk at a time: 4 A panels + 8 B panels feed 32 tiles from that XCD's L2
// (a 1 x 32 row strip would stream 32 B panels from HBM). Slots below the diagonal or past
// the edge return false (their workgroup exits at once).
__device__ __forceinline__ bool slot_tile(int slot, int nt, int& ti, int& tj) {
  int b = 0, rem = slot >> 5;
  while (true) {
    const int nch = (nt - 4 * b + 7) / 8;
    if (rem < nch) break;
    rem -= nch;
    ++b;
  }
  const int s = slot & 31;
  ti = 4 * b + (s >> 3);
  tj = 4 * b + rem * 8 + (s & 7);
  return ti < nt && tj < nt && tj >= ti;
}

static int n_slots(int nt) {
  int chunks = 0;
  for (int b = 0; 4 * b < nt; ++b) chunks += (nt - 4 * b + 7) / 8;
  return 32 * chunks;
}

// half-row hr (0..127) of half-tile h -> row of the 256-row operand tile
__device__ __forceinline__ int half_row(int h, int hr) {
  if (h == H_ALO) return (hr >> 6) * 128 + (hr & 63);
  if (h == H_AHI) return (hr >> 6) * 128 + 64 + (hr & 63);
  if (h == H_BLO) return (hr >> 5) * 64 + (hr & 31);
  return (hr >> 5) * 64 + 32 + (hr & 31);
}

struct SyrkArgs {
  const uint16_t* xt;
  int64_t kp;        // row length of XT (elements), multiple of 64
  int64_t ic;        // true size of H
  float* H;
  float* part;       // split-K slabs [ns][icp][icp] or null
  int64_t icp;
  float alpha, beta;
  int nt, ntiles, ns, nslots;
  int64_t kt_per_split;  // K-tiles per split
};

// stage one half-tile h of K-tile kt into LDS buffer `buf` (2 glds per lane)
__device__ __forceinline__ void stage_half(const SyrkArgs& a, char* lds, int buf, int h,
                                           int64_t kt, int64_t row_a0, int64_t row_b0,
                                           int wid, int lane) {
  const int64_t row0 = (h <= H_AHI) ? row_a0 : row_b0;
  char* base = lds + buf * BUF_B + h * HALF_B;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int sub = wid * 2 + q;           // subtile 0..15: (row block rb, k block kb)
    const int rb = sub >> 1, kb = sub & 1;
    const int r = lane >> 2;               // row within the 16-row subtile
    const int pc = (lane & 3) * 16;        // physical byte in the 64-byte row
    const int lc = pc ^ (((r >> 3) & 1) << 5);  // st_16x32: logical byte
    const int hr = rb * 16 + r;
    const int64_t grow = row0 + half_row(h, hr);
    const uint16_t* src = a.xt + grow * a.kp + kt * SKT + kb * 32 + (lc >> 1);
    __builtin_amdgcn_global_load_lds((g_void_t*)src, (lds_void_t*)(base + sub * 1024), 16, 0,
                                     0);
  }
}

// read one 16x32 operand fragment (8 x 16-bit) for MFMA 16x16x32: rows rb*16.., k block kb
__device__ __forceinline__ v8s read_frag(const char* half_base, int rb, int kb, int lane) {
  const int r = lane & 15;
  const int lc = (lane >> 4) * 16;
  const int pc = lc ^ (((r >> 3) & 1) << 5);
  return *reinterpret_cast<const v8s*>(half_base + (rb * 2 + kb) * 1024 + r * 64 + pc);
}

template <bool FP16>
__device__ __forceinline__ void mfma16(v4f& acc, v8s a, v8s b) {
  if constexpr (FP16)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, a),
                                                 __builtin_bit_cast(v8h, b), acc, 0, 0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a),
                                                  __builtin_bit_cast(v8bf, b), acc, 0, 0, 0);
}
#define LCQ_MFMA(acc, a, b) mfma16<FP16>(acc, a, b)

template <bool FP16>
__global__ void __launch_bounds__(512, 1) k_syrk256(SyrkArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  // XCD-aware bijective remap: blocks that share an XCD (bid % 8) get consecutive work ids
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int slot = wgid % a.nslots, split = wgid / a.nslots;
  int ti, tj;
  if (!slot_tile(slot, a.nt, ti, tj)) return;
  const int64_t row_a0 = (int64_t)ti * ST, row_b0 = (int64_t)tj * ST;
  const int64_t kt0 = (int64_t)split * a.kt_per_split;
  const int64_t nkt_total = a.kp / SKT;
  int64_t nk = nkt_total - kt0;
  if (nk > a.kt_per_split) nk = a.kt_per_split;

  v4f acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};

  // K-tile index clamped into this split's range (tail prefetches reload the last tile so the
  // vmcnt count stays constant; nobody reads them)
  auto ktile = [&](int64_t t) { return kt0 + (t < nk ? t : nk - 1); };

  // Schedule (global phase P = 4t + p, p = 1..4). Phase p of K-tile t reads: p1 A_lo + B_lo,
  // p2 B_hi, p3 A_hi, p4 nothing (B_lo fragments stay in VGPRs). The wave rows are staggered
  // by one barrier (wr == 1 waits at one extra barrier first), so on every SIMD one wave's
  // MFMA cluster overlaps the other wave's ds_reads and load issue. Staging (2 glds/lane per
  // half-tile) keeps >= 2 phases after a half-tile's last read (WAR across the stagger) and
  // ~4 phases of load latency before its first read:
  //   p1: A_hi(t+1)   p3: A_lo(t+2), B_lo(t+2)   p4: B_hi(t+2)
  // and `s_waitcnt vmcnt(8)` (4 half-tiles left in flight) at the end of p1, p3, p4 retires
  // exactly what phase p+2 reads, one barrier before the staggered wave group reads it.
  // Prologue = the state a K-tile "-1" would leave: K-tile 0 resident, A_lo/B_lo/B_hi(1) in
  // flight.
  stage_half(a, lds, 0, H_ALO, ktile(0), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 0, H_BLO, ktile(0), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 0, H_BHI, ktile(0), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 0, H_AHI, ktile(0), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 1, H_ALO, ktile(1), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 1, H_BLO, ktile(1), row_a0, row_b0, wid, lane);
  stage_half(a, lds, 1, H_BHI, ktile(1), row_a0, row_b0, wid, lane);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (__builtin_amdgcn_readfirstlane(wr) == 1) __builtin_amdgcn_s_barrier();  // stagger

  v8s fa[4][2], fbl[2][2], fbh[2][2];
  for (int64_t t = 0; t < nk; ++t) {
    const int cur = (int)(t & 1), nxt = cur ^ 1;
    const char* bA_lo = lds + cur * BUF_B + H_ALO * HALF_B;
    const char* bA_hi = lds + cur * BUF_B + H_AHI * HALF_B;
    const char* bB_lo = lds + cur * BUF_B + H_BLO * HALF_B;
    const char* bB_hi = lds + cur * BUF_B + H_BHI * HALF_B;
    // ---- phase 1: wave rows 0-63 x cols 0-31; stage A_hi(t+1)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fbl[n][kb] = read_frag(bB_lo, wc * 2 + n, kb, lane);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fa[m][kb] = read_frag(bA_lo, wr * 4 + m, kb, lane);
    stage_half(a, lds, nxt, H_AHI, ktile(t + 1), row_a0, row_b0, wid, lane);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) LCQ_MFMA(acc[m][n], fa[m][kb], fbl[n][kb]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: rows 0-63 x cols 32-63
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fbh[n][kb] = read_frag(bB_hi, wc * 2 + n, kb, lane);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) LCQ_MFMA(acc[m][2 + n], fa[m][kb], fbh[n][kb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: rows 64-127 x cols 32-63; stage A_lo(t+2), B_lo(t+2)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fa[m][kb] = read_frag(bA_hi, wr * 4 + m, kb, lane);
    stage_half(a, lds, cur, H_ALO, ktile(t + 2), row_a0, row_b0, wid, lane);
    stage_half(a, lds, cur, H_BLO, ktile(t + 2), row_a0, row_b0, wid, lane);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) LCQ_MFMA(acc[4 + m][2 + n], fa[m][kb], fbh[n][kb]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: rows 64-127 x cols 0-31 (no LDS reads); stage B_hi(t+2)
    stage_half(a, lds, cur, H_BHI, ktile(t + 2), row_a0, row_b0, wid, lane);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) LCQ_MFMA(acc[4 + m][n], fa[m][kb], fbl[n][kb]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();  // un-stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped tail prefetches

  // ---- epilogue: wave tile rows wr*128 + m*16 + (lane>>4)*4 + j, cols wc*64 + n*16 + lane&15
  const int fr = lane & 15, fq = lane >> 4;
  if (a.ns > 1) {
    float* P = a.part + (int64_t)split * a.icp * a.icp;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int64_t col = row_b0 + wc * 64 + n * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t row = row_a0 + wr * 128 + m * 16 + fq * 4 + j;
          P[row * a.icp + col] = acc[m][n][j];
        }
      }
    return;
  }
  const bool diag = ti == tj;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int64_t col = row_b0 + wc * 64 + n * 16 + fr;
      const int64_t r0 = row_a0 + wr * 128 + m * 16 + fq * 4;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t row = r0 + j;
        float v = __fmul_rn(a.alpha, acc[m][n][j]);
        if (a.beta != 0.f && row < a.ic && col < a.ic)
          v = __fadd_rn(__fmul_rn(a.beta, a.H[row * a.ic + col]), v);
        o[j] = v;
        if (row < a.ic && col < a.ic) a.H[row * a.ic + col] = v;
      }
      if (!diag && col < a.ic) {  // mirror: H[col][r0..r0+3]
        if (r0 + 3 < a.ic && (a.ic & 3) == 0) {
          *reinterpret_cast<float4*>(a.H + col * a.ic + r0) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + j < a.ic) a.H[col * a.ic + r0 + j] = o[j];
        }
      }
    }
}

// split-K combine: H = beta*H + alpha * sum_s P[s] (fixed order), upper tiles + mirror. A
// workgroup = one 64 x 64 piece of an upper tile: the row-major store and the mirrored store
// both go out coalesced (the mirror through an LDS transpose)
__global__ void __launch_bounds__(256) k_syrk_reduce(SyrkArgs a) {
  __shared__ float tp[64][65];
  int ti, tj;
  tri_tile(blockIdx.x, a.nt, ti, tj);
  const bool diag = ti == tj;
  const int pr = blockIdx.y >> 2, pc = blockIdx.y & 3;  // 4 x 4 pieces of the 256^2 tile
  const int64_t r0 = (int64_t)ti * ST + pr * 64, c0 = (int64_t)tj * ST + pc * 64;
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  for (int rr = ry; rr < 64; rr += 4) {
    const int64_t r = r0 + rr, c = c0 + cx;
    float v = 0.f;
    if (r < a.ic && c < a.ic) {
      float s = 0.f;
      for (int k = 0; k < a.ns; ++k)
        s = __fadd_rn(s, a.part[(int64_t)k * a.icp * a.icp + r * a.icp + c]);
      v = __fmul_rn(a.alpha, s);
      if (a.beta != 0.f) v = __fadd_rn(__fmul_rn(a.beta, a.H[r * a.ic + c]), v);
      a.H[r * a.ic + c] = v;
    }
    tp[rr][cx] = v;
  }
  if (diag) return;  // a diagonal tile's mirror is its own transpose: written above
  __syncthreads();
  for (int cc = ry; cc < 64; cc += 4) {  // H[c0 + cc][r0 + cx] = tile[cx][cc]
    const int64_t c = c0 + cc, r = r0 + cx;
    if (r < a.ic && c < a.ic) a.H[c * a.ic + r] = tp[cx][cc];
  }
}

static int64_t ceil_to(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Split-K count. The k_syrk16 grid is ntiles x ns workgroups, one per CU (128 KB LDS), in
// contiguous wgid ranges per XCD (8 XCDs x 32 CUs), so a launch takes
// rounds = ceil(ceil(ntiles * ns / 8) / 32) waves of workgroups, each ~(ktps + 6) K-tile
// times long (6 ~ prologue + the 256 KB fp32 tile store); every split adds a 256 KB partial
// tile written and re-read by k_syrk_reduce (~0.034 K-tile times at HBM rate). Pick the ns
// with the least modelled time: at n = 262144 ic 4096 (136 tiles) ns 15 fills 8 rounds to
// 99.6 % where ns 8 left a 5th round a quarter full; ic 8192 (528 tiles) ns 8 instead of 1.
// At least 8 K-tiles per split; partial slabs capped at 8 GiB. LCQ_SYRK_NS forces a count
// (A/B probes: scripts/probes/syrk_ns_sweep.py).
static void plan(int64_t n, int64_t ic, int& nt, int& ntiles, int& ns, int64_t& ktps,
                 int64_t& kp, int64_t& icp) {
  icp = ceil_to(ic, ST);
  kp = ceil_to(n, SKT);
  nt = (int)(icp / ST);
  ntiles = nt * (nt + 1) / 2;
  const int64_t nkt = kp / SKT;
  const char* force = getenv("LCQ_SYRK_NS");
  int64_t best_ns = 1;
  if (force && atoi(force) > 0) {
    best_ns = atoi(force);
  } else {
    double best = 1e300;
    for (int64_t c = 1; c <= 256; ++c) {
      if (c > 1 && (nkt / c < 8 || c * icp * icp * 4 > (int64_t(8) << 30))) break;
      const int64_t per = (nkt + c - 1) / c, cc = (nkt + per - 1) / per;
      const int64_t per_xcd = (ntiles * cc + 7) / 8, rounds = (per_xcd + 31) / 32;
      const double cost = (double)rounds * (double)(per + 6) +
                          (cc > 1 ? 0.034 * (double)(cc * ntiles) + 0.07 * ntiles : 0.0);
      if (cost < best * 0.995) {
        best = cost;
        best_ns = cc;
      }
    }
  }
  if (best_ns > nkt) best_ns = nkt;
  ktps = (nkt + best_ns - 1) / best_ns;
  ns = (int)((nkt + ktps - 1) / ktps);
}

}  // namespace lcq

using namespace lcq;

extern "C" int64_t lcq_hessian_workspace_bytes(int64_t n, int64_t ic) {
  if (n <= 0 || ic <= 0) return 0;
  int nt, ntiles, ns;
  int64_t ktps, kp, icp;
  plan(n, ic, nt, ntiles, ns, ktps, kp, icp);
  int64_t b = icp * kp * 2;
  if (ns > 1) b += (int64_t)ns * icp * icp * 4;
  return b;
}

extern "C" int lcq_hessian_accum(const void* x, int x_dtype, int64_t n, int64_t ic, void* H,
                                 float alpha, float beta, void* workspace, int64_t ws_bytes,
                                 void* stream) {
  LCQ_REQUIRE(x_dtype == LCQ_BF16 || x_dtype == LCQ_F16, "x must be bf16 or fp16");
  LCQ_REQUIRE(n > 0 && ic > 0, "empty input");
  LCQ_REQUIRE(workspace != nullptr && ws_bytes >= lcq_hessian_workspace_bytes(n, ic),
              "workspace smaller than lcq_hessian_workspace_bytes(n, ic)");
  int nt, ntiles, ns;
  int64_t ktps, kp, icp;
  plan(n, ic, nt, ntiles, ns, ktps, kp, icp);
  hipStream_t st = as_stream(stream);
  uint16_t* xt = reinterpret_cast<uint16_t*>(workspace);
  hipLaunchKernelGGL(k_xt_pack, dim3((unsigned)(kp / 64), (unsigned)(icp / 128)), 256, 0, st,
                     reinterpret_cast<const uint16_t*>(x), n, ic, xt, icp, kp);
  int rc = check_launch("lcq_hessian_accum: transpose");
  if (rc) return rc;
  SyrkArgs a{};
  a.xt = xt; a.kp = kp; a.ic = ic; a.H = reinterpret_cast<float*>(H); a.icp = icp;
  a.part = ns > 1 ? reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + icp * kp * 2)
                  : nullptr;
  a.alpha = alpha; a.beta = beta; a.nt = nt; a.ntiles = ntiles; a.ns = ns; a.kt_per_split = ktps;
  a.nslots = n_slots(nt);
  const char* sk = getenv("LCQ_SYRK");  // 256: the 8-wave k_syrk256 (previous default)
  if (!(sk && sk[0] == '2')) {
    // default: the 4-wave projection-GEMM core (gemm256.hip k_gemm16b schedule)
    rc = syrk16_launch(xt, kp, ic, icp, a.H, a.part, alpha, beta, nt, ns, ntiles, ktps,
                       x_dtype == LCQ_F16, st);
    if (rc) return rc;
    if (ns > 1) {
      hipLaunchKernelGGL(k_syrk_reduce, dim3((unsigned)ntiles, 16), 256, 0, st, a);
      rc = check_launch("lcq_hessian_accum: reduce");
    }
    return rc;
  }
  // the dynamic-LDS attribute is per device: set it on every launch (cheap, thread-safe)
  (void)hipFuncSetAttribute((const void*)k_syrk256<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF_B);
  (void)hipFuncSetAttribute((const void*)k_syrk256<true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF_B);
  if (x_dtype == LCQ_F16)
    hipLaunchKernelGGL(k_syrk256<true>, dim3((unsigned)(a.nslots * ns)), 512, 2 * BUF_B, st, a);
  else
    hipLaunchKernelGGL(k_syrk256<false>, dim3((unsigned)(a.nslots * ns)), 512, 2 * BUF_B, st, a);
  rc = check_launch("lcq_hessian_accum: syrk");
  if (rc) return rc;
  if (ns > 1) {
    hipLaunchKernelGGL(k_syrk_reduce, dim3((unsigned)ntiles, 16), 256, 0, st, a);
    rc = check_launch("lcq_hessian_accum: reduce");
  }
  return rc;
}
