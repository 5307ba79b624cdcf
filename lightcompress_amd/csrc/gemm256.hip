// Projection GEMMs of the calibration and AWQ loss-search forwards on gfx950 bf16/fp16 MFMA,
// with the elementwise work around them fused into the epilogue.
//
// Reference: every `inspect_module(x)` of Awq.search_scale_subset (llmc/compression/
// quantization/awq.py:110-126, 178-278) is an nn.Linear stack: q/k/v -> attention -> o_proj,
// gate/up -> act_fn(gate) * up -> down_proj, or down_proj alone; calculate_loss (awq.py:134-145)
// then takes mean((org_out - out)^2). The same linears run the block forwards that capture the
// calibration inputs (base_blockwise_quantization.py block_forward).
//
//   C = A . B^T    A [M, K] token-major activations (k-contiguous), B [N, K] nn.Linear weights
//                  (k-contiguous): both MFMA operands stream k-contiguous rows, no transposes.
//
// Epilogues (EPI):
//   EPI_STORE   C_s[t, c] = rnd(acc + bias)   up to 3 column segments with their own weight
//               and output pointers (q / k / v from one launch: one A read for the three)
//   EPI_SILU    pair mode: B_lo = gate rows, B_hi = up rows of the same 128 output columns;
//               h = rnd(rnd(g / (1 + exp(-g))) * u) with g = rnd(acc_gate), u = rnd(acc_up)
//               (LlamaMLP act_fn(gate_proj(x)) * up_proj(x), the two [M, I] projections are
//               never written)
//   EPI_SQDIFF  out = rnd(acc + bias) is never written: d = rnd(ref - out), the tile's
//               sum of fp32 d*d goes to an fp64 partial per tile; k_loss_reduce sums the
//               partials in tile order (deterministic) and writes sum / numel to a device slot
//               (calculate_loss without materialising `out`)
//
// Structure (cdna_hip_programming.md §5, the 256^2 template; the same schedule as the Hessian
// SYRK in hessian256.hip): one 512-thread workgroup (8 waves, 2(M) x 4(N)) per 256x256 output
// tile, each wave 128x64 = 8x4 accumulators of mfma_f32_16x16x32. K-tile 64; A and B tiles
// split into four 16 KB half-tiles staged by global_load_lds_dwordx4 into two LDS buffers
// (128 KB, one __shared__ array; st_16x32 swizzle applied on the global source address),
// 4 phases per K-tile with the two wave rows one barrier apart, counted `s_waitcnt vmcnt(8)`,
// raw s_barrier (never vmcnt(0) in the loop). The MFMA runs swapped (B fragment as the A
// operand), so each lane's accumulator holds 4 consecutive output columns of one token row:
// 8-byte stores / loads in the epilogues. Tile order is XCD-aware: consecutive work ids go to
// one XCD and a chunk of 32 = a 4 (M) x 8 (N) block of tiles shares 12 operand panels in L2.
#define LCQ_BF16_HW 1  // conversion-instruction RNE in the epilogues
#include "lcq_common.h"

#include <stdlib.h>

namespace lcq {
namespace g256 {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int ST = 256;            // output tile (rows of A, rows of B)
constexpr int SKT = 64;            // K-tile
constexpr int HALF_B = 16384;      // 128 rows x 64 k x 2 B
constexpr int BUF_B = 4 * HALF_B;  // A_lo, A_hi, B_lo, B_hi
enum { H_ALO = 0, H_AHI = 1, H_BLO = 2, H_BHI = 3 };
enum { EPI_STORE = 0, EPI_SILU = 1, EPI_SQDIFF = 2 };
constexpr int MAXSEG = 3;

struct Args {
  const uint16_t* a;
  int64_t lda, m, k;
  // B segments (EPI_STORE / EPI_SQDIFF: rows [bend[s-1], bend[s]) of the virtual [N, K]
  // weight come from b[s]; EPI_SILU: b[0] = gate, b[1] = up, each [N, K])
  const uint16_t* b[MAXSEG];
  int64_t bend[MAXSEG];
  int64_t ldb, n;  // n = output columns
  const uint16_t* bias[MAXSEG];
  uint16_t* c[MAXSEG];
  int64_t ldc[MAXSEG];
  const uint16_t* ref;
  int64_t ldr;
  double* part;
  int nseg;
  int n_mt, n_nt, cpb, nslots;
  int order;  // tile order of k_gemm16: 0 = per-XCD bands (slot_tile), 1 = N-band-major (tile_nb)
  int wide;   // every output pointer 16-B aligned and every ldc % 8 == 0: 16-B epilogue stores
};

// half-row hr (0..127) of half-tile h -> row of the 256-row operand tile
__device__ __forceinline__ int half_row(int h, int hr) {
  if (h == H_ALO) return (hr >> 6) * 128 + (hr & 63);
  if (h == H_AHI) return (hr >> 6) * 128 + 64 + (hr & 63);
  if (h == H_BLO) return (hr >> 5) * 64 + (hr & 31);
  return (hr >> 5) * 64 + 32 + (hr & 31);
}

// work slot -> tile (4 x 8 blocks of tiles, bands of 4 tile rows walked along N)
__device__ __forceinline__ bool slot_tile(const Args& a, int slot, int& tm, int& tn) {
  const int chunk = slot >> 5, s = slot & 31;
  const int band = chunk / a.cpb, c = chunk - band * a.cpb;
  tm = band * 4 + (s >> 3);
  tn = c * 8 + (s & 7);
  return tm < a.n_mt && tn < a.n_nt;
}

// N-band-major order: launch step T = bid >> 8 (the 256 workgroups resident at once, one per
// CU) covers a region of 32 (M) x 8 (N) tiles; XCD x = bid & 7 takes its 4 x 8 chunk (tile rows
// 4x..4x+3, 12 operand panels shared in its L2). Regions walk M first inside one band of 8
// N-tiles, so every XCD streams the same B band while the A panels pass once per band:
// beyond-L2 reads of B come from the MALL, HBM reads ~ A x (N / 2048) + B once.
__device__ __forceinline__ bool tile_nb(const Args& a, int bid, int& tm, int& tn) {
  const int xcd = bid & 7, s = (bid >> 3) & 31, T = bid >> 8;
  const int mreg = (a.n_mt + 31) >> 5;
  const int nb = T / mreg, mr = T - nb * mreg;
  tm = mr * 32 + xcd * 4 + (s >> 3);
  tn = nb * 8 + (s & 7);
  return tm < a.n_mt && tn < a.n_nt;
}

// Per-lane staging addresses, computed once per tile: each half-tile h has a wave-uniform
// base (panel start) and per-lane 32-bit byte offsets for the lane's two glds pieces (row
// clamped into the operand, st_16x32 swizzle applied). The K loop only adds kt * 128 bytes:
// no per-K-tile row / segment arithmetic (and no scalar loads + lgkmcnt(0) inside a phase).
struct Stage {
  const char* base[4];
  uint32_t off[4][2];
};

template <int EPI>
__device__ __forceinline__ void make_stage(const Args& a, int tm, int tn, int wid, int lane,
                                           Stage& st) {
  const int64_t arow0 = (int64_t)tm * ST;
  st.base[H_ALO] = st.base[H_AHI] = reinterpret_cast<const char*>(a.a + arow0 * a.lda);
  int64_t brow0, blast;  // first row of this tile in its B source, last valid row there
  const uint16_t* b_lo;
  const uint16_t* b_hi;
  if constexpr (EPI == EPI_SILU) {
    brow0 = (int64_t)tn * 128;
    blast = a.n - 1;
    b_lo = a.b[0];
    b_hi = a.b[1];
  } else {
    const int64_t row0 = (int64_t)tn * ST;
    int s = 0;
    int64_t segbase = 0;
    if (a.nseg > 1 && row0 >= a.bend[0]) { s = 1; segbase = a.bend[0]; }
    if (a.nseg > 2 && row0 >= a.bend[1]) { s = 2; segbase = a.bend[1]; }
    brow0 = row0 - segbase;
    blast = a.bend[s] - segbase - 1;
    b_lo = b_hi = a.b[s];
  }
  st.base[H_BLO] = reinterpret_cast<const char*>(b_lo + brow0 * a.ldb);
  st.base[H_BHI] = reinterpret_cast<const char*>(b_hi + brow0 * a.ldb);
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int sub = wid * 2 + q;           // subtile 0..15: (row block rb, k block kb)
      const int rb = sub >> 1, kb = sub & 1;
      const int r = lane >> 2;               // row within the 16-row subtile
      const int pc = (lane & 3) * 16;        // physical byte in the 64-byte row
      const int lc = pc ^ (((r >> 3) & 1) << 5);  // st_16x32: logical byte
      const int hr = rb * 16 + r;
      int64_t row;
      int64_t ld;
      if (h <= H_AHI) {
        row = half_row(h, hr);
        if (arow0 + row > a.m - 1) row = a.m - 1 - arow0;
        ld = a.lda;
      } else {
        row = (EPI == EPI_SILU) ? hr : half_row(h, hr);
        if (brow0 + row > blast) row = blast - brow0;
        ld = a.ldb;
      }
      st.off[h][q] = (uint32_t)(row * ld * 2 + kb * 64 + lc);
    }
}

// stage one half-tile h of K-tile kt into LDS buffer `buf` (2 glds per lane)
__device__ __forceinline__ void stage_half(const Stage& st, char* lds, int buf, int h,
                                           int64_t kt, int wid) {
  char* base = lds + buf * BUF_B + h * HALF_B;
  const char* g = st.base[h] + kt * (SKT * 2);
#pragma unroll
  for (int q = 0; q < 2; ++q)
    __builtin_amdgcn_global_load_lds((g_void_t*)(g + st.off[h][q]),
                                     (lds_void_t*)(base + (wid * 2 + q) * 1024), 16, 0, 0);
}

__device__ __forceinline__ v8s read_frag(const char* half_base, int rb, int kb, int lane) {
  const int r = lane & 15;
  const int lc = (lane >> 4) * 16;
  const int pc = lc ^ (((r >> 3) & 1) << 5);
  return *reinterpret_cast<const v8s*>(half_base + (rb * 2 + kb) * 1024 + r * 64 + pc);
}

// swapped operands: D[i][j] = sum_k B[i][k] A[j][k]; lane (fr = lane & 15, fq = lane >> 4)
// holds output columns fq*4 + 0..3 of token row fr
template <bool FP16>
__device__ __forceinline__ void mfma16(v4f& acc, v8s bfrag, v8s afrag) {
  if constexpr (FP16)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(v8h, bfrag),
                                                 __builtin_bit_cast(v8h, afrag), acc, 0, 0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, bfrag),
                                                  __builtin_bit_cast(v8bf, afrag), acc, 0, 0, 0);
}

template <int DT>
__device__ __forceinline__ float ld_h(const uint16_t* p) {
  if constexpr (DT == LCQ_BF16) return __uint_as_float((uint32_t)(*p) << 16);
  else return (float)__builtin_bit_cast(_Float16, *p);
}

template <int DT>
__device__ __forceinline__ void unpack4(uint2 w, float (&v)[4]) {
  const uint32_t x[2] = {w.x, w.y};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (DT == LCQ_BF16) {
      v[2 * i] = __uint_as_float(x[i] << 16);
      v[2 * i + 1] = __uint_as_float(x[i] & 0xffff0000u);
    } else {
      v[2 * i] = (float)__builtin_bit_cast(_Float16, (uint16_t)(x[i] & 0xffffu));
      v[2 * i + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(x[i] >> 16));
    }
  }
}

template <int DT, int EPI>
__global__ void __launch_bounds__(512, 1) k_gemm256(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm, tn;
  if (!slot_tile(a, wgid, tm, tn)) return;
  const int64_t nk = a.k / SKT;
  Stage st;
  make_stage<EPI>(a, tm, tn, wid, lane, st);

  v4f acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};

  auto ktile = [&](int64_t t) { return t < nk ? t : nk - 1; };

  // schedule: see hessian256.hip (phase p of K-tile t reads p1 A_lo + B_lo, p2 B_hi, p3 A_hi,
  // p4 nothing; staging p1 A_hi(t+1), p3 A_lo/B_lo(t+2), p4 B_hi(t+2); vmcnt(8) after p1, p3,
  // p4 retires what phase p+2 reads)
  stage_half(st, lds, 0, H_ALO, ktile(0), wid);
  stage_half(st, lds, 0, H_BLO, ktile(0), wid);
  stage_half(st, lds, 0, H_BHI, ktile(0), wid);
  stage_half(st, lds, 0, H_AHI, ktile(0), wid);
  stage_half(st, lds, 1, H_ALO, ktile(1), wid);
  stage_half(st, lds, 1, H_BLO, ktile(1), wid);
  stage_half(st, lds, 1, H_BHI, ktile(1), wid);
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
    // ---- phase 1: rows 0-63 x cols 0-31 of the wave tile; stage A_hi(t+1)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fbl[n][kb] = read_frag(bB_lo, wc * 2 + n, kb, lane);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fa[m][kb] = read_frag(bA_lo, wr * 4 + m, kb, lane);
    stage_half(st, lds, nxt, H_AHI, ktile(t + 1), wid);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) mfma16<FP16>(acc[m][n], fbl[n][kb], fa[m][kb]);
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
        for (int kb = 0; kb < 2; ++kb) mfma16<FP16>(acc[m][2 + n], fbh[n][kb], fa[m][kb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: rows 64-127 x cols 32-63; stage A_lo(t+2), B_lo(t+2)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) fa[m][kb] = read_frag(bA_hi, wr * 4 + m, kb, lane);
    stage_half(st, lds, cur, H_ALO, ktile(t + 2), wid);
    stage_half(st, lds, cur, H_BLO, ktile(t + 2), wid);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) mfma16<FP16>(acc[4 + m][2 + n], fbh[n][kb], fa[m][kb]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: rows 64-127 x cols 0-31 (no LDS reads); stage B_hi(t+2)
    stage_half(st, lds, cur, H_BHI, ktile(t + 2), wid);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) mfma16<FP16>(acc[4 + m][n], fbl[n][kb], fa[m][kb]);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  if (__builtin_amdgcn_readfirstlane(wr) == 0) __builtin_amdgcn_s_barrier();  // un-stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the clamped tail prefetches

  // ---- epilogue. acc[m][n][j]: token row tm*256 + wr*128 + (m & 4 ? 64 : 0) + (m & 3)*16 + fr,
  // tile column wc*64 + n*16 + fq*4 + j (EPI_SILU: n < 2 gate / n >= 2 up of output column
  // tn*128 + wc*32 + (n & 1)*16 + fq*4 + j)
  const int fr = lane & 15, fq = lane >> 4;
  double dsum = 0.0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int64_t trow = (int64_t)tm * ST + wr * 128 + (m >> 2) * 64 + (m & 3) * 16 + fr;
    if (trow >= a.m) continue;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int64_t col = (int64_t)tn * 128 + wc * 32 + n * 16 + fq * 4;
        if (col >= a.n) continue;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g = rnd<DT>(acc[m][n][j]);
          const float u = rnd<DT>(acc[m][n + 2][j]);
          const float sl = rnd<DT>(g / (1.0f + expf(-g)));
          o[j] = rnd<DT>(sl * u);
        }
        uint2 w;
        w.x = pack2<DT>(o[0], o[1]);
        w.y = pack2<DT>(o[2], o[3]);
        *reinterpret_cast<uint2*>(a.c[0] + trow * a.ldc[0] + col) = w;
      }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int64_t col = (int64_t)tn * ST + wc * 64 + n * 16 + fq * 4;
        if (col >= a.n) continue;
        int s = 0;
        int64_t base = 0;
        if (a.nseg > 1 && col >= a.bend[0]) { s = 1; base = a.bend[0]; }
        if (a.nseg > 2 && col >= a.bend[1]) { s = 2; base = a.bend[1]; }
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[m][n][j];
          if (a.bias[s] != nullptr) v = __fadd_rn(v, ld_h<DT>(a.bias[s] + (col - base) + j));
          o[j] = rnd<DT>(v);
        }
        if constexpr (EPI == EPI_STORE) {
          uint2 w;
          w.x = pack2<DT>(o[0], o[1]);
          w.y = pack2<DT>(o[2], o[3]);
          *reinterpret_cast<uint2*>(a.c[s] + trow * a.ldc[s] + (col - base)) = w;
        } else {
          float r[4];
          unpack4<DT>(*reinterpret_cast<const uint2*>(a.ref + trow * a.ldr + col), r);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = rnd<DT>(r[j] - o[j]);
            dsum += (double)(d * d);
          }
        }
      }
    }
  }
  if constexpr (EPI == EPI_SQDIFF) {
#pragma unroll
    for (int msk = 32; msk >= 1; msk >>= 1) dsum += __shfl_xor(dsum, msk, 64);
    __syncthreads();  // every wave past its last LDS read / DMA before reusing the array
    double* red = reinterpret_cast<double*>(lds);
    if (lane == 0) red[wid] = dsum;
    __syncthreads();
    if (tid == 0) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < 8; ++w) s += red[w];
      double* pp = a.part + ((int64_t)tm * a.n_nt + tn) * 4;  // 4 slots per tile (k_gemm16p)
      pp[0] = s;
      pp[1] = pp[2] = pp[3] = 0.0;
    }
  }
}

// ---------------------------------------------------------------------------------------
// 4-wave kernel (the default): one 256-thread workgroup per 256x256 tile, 2 x 2 waves, each
// wave a 128 x 128 sub-tile = 4 x 4 accumulators of mfma_f32_32x32x16_bf16 (256 registers;
// one wave per SIMD, so the accumulators take the AGPR half of the 512-entry file -- with the
// 16x16x32 shape the same 256 accumulators make hipcc shuffle AGPRs every MFMA). Per wave and
// K-tile: 16 B-fragment reads held in registers, A fragments streamed one 32-row block ahead
// (0.5 LDS reads per 32x32x16 MFMA), 64 MFMAs. One barrier per K-tile, placed after the tile's
// last LDS read: behind it the wave issues the loads of K-tile t+2 into the buffer just
// released and refills the B fragments with K-tile t+1's behind its last MFMAs of K-tile t.
//
// LDS image of one operand tile (256 rows x 64 k, 32 KB): blocks of 32 rows x 32 k (2 KB),
// block (rb32, kb) at (rb32 * 2 + kb) * 2048, row r at r * 64, 16-byte piece p (k 8p..8p+7)
// at (p ^ ((r >> 2) & 3)) * 16: a 32x32x16 fragment read (lane -> row lane & 31, piece
// 2 (s & 1) + (lane >> 5)) is bank-conflict-free in every ds_read_b128 lane group.
// ---------------------------------------------------------------------------------------
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int TILE_B = ST * SKT * 2;   // one operand tile: 256 rows x 64 k x 2 B = 32 KB
constexpr int BUF4 = 2 * TILE_B;       // A + B

// Staging through buffer descriptors (cdna_hip_programming.md T8): one wave-uniform
// descriptor per operand panel (built from kernarg / blockIdx values only), per-lane 32-bit
// byte offsets (one VGPR per piece), the K-tile step in the scalar soffset: no 64-bit address
// arithmetic and no per-piece pointer registers in the K loop.
struct Stage4 {
  __amdgpu_buffer_rsrc_t ra;
  __amdgpu_buffer_rsrc_t rb[2];
  uint32_t aoff[8];
  uint32_t boff[8];
  int bsel;  // bit j: B piece j reads rb[1] (EPI_SILU: up rows); wave-uniform
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t panel_rsrc(const void* p) {
  // readfirstlane the base so the compiler can prove the descriptor wave-uniform (T20): no
  // waterfall loop around the loads
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, 0x7fffffff, 0x00020000);
}

// piece j of wave w = LDS piece P = w + 4j of the tile image: block P >> 1 (rb32 = P >> 2,
// kb = (P >> 1) & 1), rows 16 (P & 1) .. +15 of the block
template <int EPI>
__device__ __forceinline__ void make_stage4(const Args& a, int tm, int tn, int w, int lane,
                                            Stage4& st) {
  const int64_t arow0 = (int64_t)tm * ST;
  st.ra = panel_rsrc(a.a + arow0 * a.lda);
  int64_t brow0 = 0, blast = 0;
  if constexpr (EPI == EPI_SILU) {
    st.rb[0] = panel_rsrc(a.b[0]);
    st.rb[1] = panel_rsrc(a.b[1]);
    blast = a.n - 1;
    brow0 = (int64_t)tn * 128;
  } else {
    const int64_t row0 = (int64_t)tn * ST;
    int s = 0;
    int64_t segbase = 0;
    if (a.nseg > 1 && row0 >= a.bend[0]) { s = 1; segbase = a.bend[0]; }
    if (a.nseg > 2 && row0 >= a.bend[1]) { s = 2; segbase = a.bend[1]; }
    brow0 = row0 - segbase;
    blast = a.bend[s] - segbase - 1;
    st.rb[0] = st.rb[1] = panel_rsrc(a.b[s] + brow0 * a.ldb);
  }
  st.bsel = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int P = w + 4 * j;
    const int rb32 = P >> 2, kb = (P >> 1) & 1;
    const int rin = 16 * (P & 1) + (lane >> 2);            // row within the 32-row block
    const int lp = (lane & 3) ^ ((rin >> 2) & 3);           // logical 16-byte piece
    const int kbyte = kb * 64 + lp * 16;
    const int row = rb32 * 32 + rin;                        // tile-local row 0..255
    int64_t ar = row;
    if (arow0 + ar > a.m - 1) ar = a.m - 1 - arow0;
    st.aoff[j] = (uint32_t)(ar * a.lda * 2 + kbyte);
    int64_t br;
    if constexpr (EPI == EPI_SILU) {
      // rows [128 wc, 128 wc + 64) gate, [128 wc + 64, 128 wc + 128) up of the same 64
      // output columns; offsets from the start of gate / up
      if (((rb32 * 32) & 127) >= 64) st.bsel |= 1 << j;  // uniform: whole 32-row block
      br = brow0 + (row >> 7) * 64 + (row & 63);
      if (br > blast) br = blast;
    } else {
      br = row;
      if (brow0 + br > blast) br = blast - brow0;
    }
    st.boff[j] = (uint32_t)(br * a.ldb * 2 + kbyte);
  }
}

__device__ __forceinline__ void stage4(const Stage4& st, char* lds, int buf, int64_t kt, int wu) {
  char* dA = lds + buf * BUF4;
  char* dB = dA + TILE_B;
  const int kofs = (int)(kt * (SKT * 2));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(st.ra, (lds_void_t*)(dA + (wu + 4 * j) * 1024), 16,
                                             st.aoff[j], kofs, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(((st.bsel >> j) & 1) ? st.rb[1] : st.rb[0],
                                             (lds_void_t*)(dB + (wu + 4 * j) * 1024), 16,
                                             st.boff[j], kofs, 0, 0);
  }
}

// 32x32x16 fragment of 32-row block rb32, K-step s (k 16s..16s+15 of the K-tile)
__device__ __forceinline__ v8s read_frag32(const char* tile, int rb32, int s, int lane) {
  const int r = lane & 31;
  const int p = 2 * (s & 1) + (lane >> 5);
  return *reinterpret_cast<const v8s*>(tile + (rb32 * 2 + (s >> 1)) * 2048 + r * 64 +
                                       ((p ^ ((r >> 2) & 3)) << 4));
}

template <bool FP16>
__device__ __forceinline__ void mfma32(v16f& acc, v8s bfrag, v8s afrag) {
  if constexpr (FP16)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, bfrag),
                                                 __builtin_bit_cast(v8h, afrag), acc, 0, 0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf, bfrag),
                                                  __builtin_bit_cast(v8bf, afrag), acc, 0, 0, 0);
}

// Load order of one K-tile's 16 pieces per wave (the vmcnt counts below depend on it):
//   block 0: B pieces 0..7, A pieces 0 and 4 | block 1: A 1, 5 | block 2: A 2, 6 | block 3: A 3, 7
// (A piece j of wave w holds 32-row block j of the A tile.)
__device__ __forceinline__ void load_piece(const Stage4& st, char* lds, int buf, int kofs, int wu,
                                           int idx) {
  char* dA = lds + buf * BUF4;
  if (idx < 8) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(((st.bsel >> idx) & 1) ? st.rb[1] : st.rb[0],
                                             (lds_void_t*)(dA + TILE_B + (wu + 4 * idx) * 1024),
                                             16, st.boff[idx], kofs, 0, 0);
  } else {
    const int q = idx - 8;                       // 0..7 -> A piece 0,4,1,5,2,6,3,7
    const int j = (q >> 1) + 4 * (q & 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(st.ra, (lds_void_t*)(dA + (wu + 4 * j) * 1024), 16,
                                             st.aoff[j], kofs, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
}

// One K-tile in four 32-row blocks of A, one barrier per block. Block m opens with 4 MFMAs
// on registers only (the pipe stays busy while the wave's last LDS reads retire), then
// barrier m: every wave has read A block m of this tile (A blocks m, m+4 of the buffer are
// free; at m = 0 the B region too) and the pieces read next have landed (counted vmcnt).
// Behind it, the block's other 12 MFMAs carry its loads of K-tile t+2 into the regions just
// released and the reads of the next A block (early, so they retire before the next
// barrier); block 3 reads K-tile t+1's A block 0 early and refills each B fragment right
// after its last MFMA. Loads of a K-tile are consumed ~1.75 K-tiles after issue.
// Straight-line code: past the last K-tile the loads re-fetch K-tile nk-1 into released
// regions and the reads fill registers nobody uses.
template <bool FP16>
__device__ __forceinline__ void ktile4(v16f (&acc)[4][4], v8s (&bf)[4][4], v8s (&af)[2][4],
                                       const Stage4& st, char* lds, int64_t t, int64_t nk,
                                       int w, int wr, int wc, int lane) {
  const int cur = (int)(t & 1);
  const char* At = lds + cur * BUF4;
  const char* An = lds + (cur ^ 1) * BUF4;
  const char* Bn = An + TILE_B;
  const int64_t kt2 = t + 2 < nk ? t + 2 : nk - 1;
  const int kofs = (int)(kt2 * (SKT * 2));
#pragma unroll
  for (int m = 0; m < 4; ++m) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = n * 4 + k;  // MFMA index within the block
        mfma32<FP16>(acc[m][n], bf[n][k], af[m & 1][k]);
        if (i == 3) {
          if (m == 0 || m == 3) wait_barrier<20>();
          else wait_barrier<28>();
        }
        if (m == 0 && i >= 4 && i < 14) load_piece(st, lds, cur, kofs, w, i - 4);  // B 0..7, A 0, 4
        if (m > 0 && (i == 4 || i == 10)) load_piece(st, lds, cur, kofs, w, 8 + 2 * m + (i == 10));
        if (i >= 4 && i < 8) {
          if (m < 3) af[(m + 1) & 1][i - 4] = read_frag32(At, wr * 4 + m + 1, i - 4, lane);
          else af[0][i - 4] = read_frag32(An, wr * 4, i - 4, lane);  // K-tile t+1, block 0
        }
        if (m == 3 && k == 3) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) bf[n][kk] = read_frag32(Bn, wc * 4 + n, kk, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
}

template <int DT, int EPI>
__global__ void __launch_bounds__(256, 1) k_gemm4w(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm, tn;
  if (!slot_tile(a, wgid, tm, tn)) return;
  const int64_t nk = a.k / SKT;
  Stage4 st;
  make_stage4<EPI>(a, tm, tn, w, lane, st);

  v16f acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[m][n][j] = 0.f;
  v8s af[2][4], bf[4][4];

  // prologue: K-tiles 0 and 1 in flight (16 pieces each, in the per-tile load order), then
  // K-tile 0's B fragments and A block 0 (its first 10 pieces) into registers
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 0, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 1, nk > 1 ? SKT * 2 : 0, w, i);
  wait_barrier<22>();
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int k = 0; k < 4; ++k) bf[n][k] = read_frag32(lds + TILE_B, wc * 4 + n, k, lane);
#pragma unroll
  for (int k = 0; k < 4; ++k) af[0][k] = read_frag32(lds, wr * 4, k, lane);

  for (int64_t t = 0; t < nk; ++t) ktile4<FP16>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // tail re-fetches landed

  // ---- epilogue. acc[m][n][4q + i]: token row tm*256 + wr*128 + m*32 + (lane & 31), tile
  // column wc*128 + n*32 + 8q + 4*(lane >> 5) + i (EPI_SILU: n < 2 gate / n >= 2 up of output
  // column tn*128 + wc*64 + (n & 1)*32 + 8q + 4*(lane >> 5) + i)
  const int fr = lane & 31, fh = lane >> 5;
  double dsum = 0.0;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 32 + fr;
    if (trow >= a.m) continue;
    if constexpr (EPI == EPI_SILU) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t col = (int64_t)tn * 128 + wc * 64 + n * 32 + 8 * q + 4 * fh;
          if (col >= a.n) continue;
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float g = rnd<DT>(acc[m][n][4 * q + i]);
            const float u = rnd<DT>(acc[m][n + 2][4 * q + i]);
            const float sl = rnd<DT>(g / (1.0f + expf(-g)));
            o[i] = rnd<DT>(sl * u);
          }
          uint2 wv;
          wv.x = pack2<DT>(o[0], o[1]);
          wv.y = pack2<DT>(o[2], o[3]);
          *reinterpret_cast<uint2*>(a.c[0] + trow * a.ldc[0] + col) = wv;
        }
    } else {
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t col = (int64_t)tn * ST + wc * 128 + n * 32 + 8 * q + 4 * fh;
          if (col >= a.n) continue;
          int s = 0;
          int64_t base = 0;
          if (a.nseg > 1 && col >= a.bend[0]) { s = 1; base = a.bend[0]; }
          if (a.nseg > 2 && col >= a.bend[1]) { s = 2; base = a.bend[1]; }
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = acc[m][n][4 * q + i];
            if (a.bias[s] != nullptr) v = __fadd_rn(v, ld_h<DT>(a.bias[s] + (col - base) + i));
            o[i] = rnd<DT>(v);
          }
          if constexpr (EPI == EPI_STORE) {
            uint2 wv;
            wv.x = pack2<DT>(o[0], o[1]);
            wv.y = pack2<DT>(o[2], o[3]);
            *reinterpret_cast<uint2*>(a.c[s] + trow * a.ldc[s] + (col - base)) = wv;
          } else {
            float r[4];
            unpack4<DT>(*reinterpret_cast<const uint2*>(a.ref + trow * a.ldr + col), r);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float d = rnd<DT>(r[i] - o[i]);
              dsum += (double)(d * d);
            }
          }
        }
    }
  }
  if constexpr (EPI == EPI_SQDIFF) {
#pragma unroll
    for (int msk = 32; msk >= 1; msk >>= 1) dsum += __shfl_xor(dsum, msk, 64);
    __syncthreads();  // every wave past its last LDS read / DMA before reusing the array
    double* red = reinterpret_cast<double*>(lds);
    if (lane == 0) red[w] = dsum;
    __syncthreads();
    if (tid < 4) a.part[((int64_t)tm * a.n_nt + tn) * 4 + tid] = red[tid];
  }
}

// ---------------------------------------------------------------------------------------
// 16x16x32 variant of the 4-wave kernel (the default): 8 x 8 accumulators per wave
// kept in AGPRs by an inline-asm MFMA ("+a": hipcc's allocator shuffles AGPRs around the
// builtin with 256 accumulators). LDS image: 16-row x 32-k subtiles (st_16x32 swizzle, as
// the 8-wave kernel); same per-tile load order / vmcnt counts as k_gemm4w.
// ---------------------------------------------------------------------------------------
template <bool FP16>
__device__ __forceinline__ void mfma16a(v4f& acc, v8s bfrag, v8s afrag) {
  if constexpr (FP16)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfrag), "v"(afrag));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfrag), "v"(afrag));
}

template <int EPI>
__device__ __forceinline__ void make_stage16(const Args& a, int tm, int tn, int w, int lane,
                                             Stage4& st) {
  const int64_t arow0 = (int64_t)tm * ST;
  st.ra = panel_rsrc(a.a + arow0 * a.lda);
  int64_t brow0 = 0, blast = 0;
  if constexpr (EPI == EPI_SILU) {
    st.rb[0] = panel_rsrc(a.b[0]);
    st.rb[1] = panel_rsrc(a.b[1]);
    blast = a.n - 1;
    brow0 = (int64_t)tn * 128;
  } else {
    const int64_t row0 = (int64_t)tn * ST;
    int s = 0;
    int64_t segbase = 0;
    if (a.nseg > 1 && row0 >= a.bend[0]) { s = 1; segbase = a.bend[0]; }
    if (a.nseg > 2 && row0 >= a.bend[1]) { s = 2; segbase = a.bend[1]; }
    brow0 = row0 - segbase;
    blast = a.bend[s] - segbase - 1;
    st.rb[0] = st.rb[1] = panel_rsrc(a.b[s] + brow0 * a.ldb);
  }
  st.bsel = 0;
  const int r = lane >> 2;
  const int pc = (lane & 3) * 16;
  const int lc = pc ^ (((r >> 3) & 1) << 5);
  const int kbyte = (w & 1) * 64 + lc;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int rb = (w >> 1) + 2 * j;                   // 16-row subtile row block 0..15
    const int row = rb * 16 + r;
    int64_t ar = row;
    if (arow0 + ar > a.m - 1) ar = a.m - 1 - arow0;
    st.aoff[j] = (uint32_t)(ar * a.lda * 2 + kbyte);
    int64_t br;
    if constexpr (EPI == EPI_SILU) {
      if (((rb * 16) & 127) >= 64) st.bsel |= 1 << j;
      br = brow0 + (row >> 7) * 64 + (row & 63);
      if (br > blast) br = blast;
    } else {
      br = row;
      if (brow0 + br > blast) br = blast - brow0;
    }
    st.boff[j] = (uint32_t)(br * a.ldb * 2 + kbyte);
  }
}

template <bool FP16, int DIAG = 0>
__device__ __forceinline__ void ktile16(v4f (&acc)[8][8], v8s (&bf)[8][2], v8s (&af)[2][2][2],
                                        const Stage4& st, char* lds, int64_t t, int64_t nk,
                                        int w, int wr, int wc, int lane) {
  const int cur = (int)(t & 1);
  const char* At = lds + cur * BUF4;
  const char* An = lds + (cur ^ 1) * BUF4;
  const char* Bn = An + TILE_B;
  const int64_t kt2 = t + 2 < nk ? t + 2 : nk - 1;
  const int kofs = (int)(kt2 * (SKT * 2));
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {     // 32-row A block: m = 2 mb, 2 mb + 1
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int i = mm * 16 + n * 2 + kb;  // MFMA index within the block (0..31)
          mfma16a<FP16>(acc[2 * mb + mm][n], bf[n][kb], af[mb & 1][mm][kb]);
          if (i == 7) {
            if constexpr (DIAG & 2) {  // diagnostic: the counted waits without the barrier
              if (mb == 0 || mb == 3) asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(28) lgkmcnt(0)" ::: "memory");
            } else {
              if (mb == 0 || mb == 3) wait_barrier<20>();
              else wait_barrier<28>();
            }
          }
          if (mb == 0 && i >= 8 && i < 28 && (i & 1) == 0) load_piece(st, lds, cur, kofs, w, (i - 8) >> 1);
          if (mb > 0 && (i == 8 || i == 20)) load_piece(st, lds, cur, kofs, w, 8 + 2 * mb + (i == 20));
          if (i >= 8 && i < 12) {
            const int q = i - 8, m2 = q >> 1, k2 = q & 1;
            if (mb < 3) af[(mb + 1) & 1][m2][k2] = read_frag(At, wr * 8 + 2 * (mb + 1) + m2, k2, lane);
            else af[0][m2][k2] = read_frag(An, wr * 8 + m2, k2, lane);  // K-tile t+1, block 0
          }
          if (mb == 3 && mm == 1 && kb == 1) {
#pragma unroll
            for (int k3 = 0; k3 < 2; ++k3) bf[n][k3] = read_frag(Bn + TILE_B * 0, wc * 8 + n, k3, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
}

// k_gemm16 with the B fragments double-buffered in registers (LCQ_GEMM_KERNEL=b): the B
// fragments of K-tile t+1 are read during blocks 1 and 2 of K-tile t (8 per block, one per MFMA
// gap after that block's 4 A-fragment reads) into the other register set, instead of 16 reads
// in the last 16 MFMA gaps whose lgkmcnt the next K-tile's first MFMAs wait on. Block 1's
// barrier therefore retires K-tile t+1's B pieces (vmcnt 18: the 8 A pieces of K-tile t+1 and
// the 10 pieces of K-tile t+2 issued in block 0 are younger), ~1.3 K-tiles after their issue.
// P = register set of K-tile t (t & 1).
template <bool FP16, int P, int DIAG = 0>
__device__ __forceinline__ void ktile16b(v4f (&acc)[8][8], v8s (&bf)[2][8][2],
                                         v8s (&af)[2][2][2], const Stage4& st, char* lds,
                                         int64_t t, int64_t nk, int w, int wr, int wc,
                                         int lane) {
  const int cur = (int)(t & 1);
  const char* At = lds + cur * BUF4;
  const char* An = lds + (cur ^ 1) * BUF4;
  const char* Bn = An + TILE_B;
  const int64_t kt2 = t + 2 < nk ? t + 2 : nk - 1;
  const int kofs = (int)(kt2 * (SKT * 2));
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int i = mm * 16 + n * 2 + kb;
          mfma16a<FP16>(acc[2 * mb + mm][n], bf[P][n][kb], af[mb & 1][mm][kb]);
          if (i == 7) {
            if constexpr (DIAG & 2) {
              if (mb == 1) asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
            } else {
              if (mb == 1) wait_barrier<18>();
              else wait_barrier<20>();
            }
          }
          if (mb == 0 && i >= 8 && i < 28 && (i & 1) == 0) load_piece(st, lds, cur, kofs, w, (i - 8) >> 1);
          if (mb > 0 && (i == 8 || i == 20)) load_piece(st, lds, cur, kofs, w, 8 + 2 * mb + (i == 20));
          if (i >= 8 && i < 12) {
            const int q = i - 8, m2 = q >> 1, k2 = q & 1;
            if (mb < 3) af[(mb + 1) & 1][m2][k2] = read_frag(At, wr * 8 + 2 * (mb + 1) + m2, k2, lane);
            else af[0][m2][k2] = read_frag(An, wr * 8 + m2, k2, lane);  // K-tile t+1, block 0
          }
          if ((mb == 1 || mb == 2) && i >= 12 && i < 20) {  // B fragments of K-tile t+1
            const int f = (mb - 1) * 8 + (i - 12), nn = f >> 1, k3 = f & 1;
            bf[P ^ 1][nn][k3] = read_frag(Bn, wc * 8 + nn, k3, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
}

// Two column groups of one row (this lane's packed x4 of group n: cols n*16 + fq*4.., and of
// group n+1) -> 8 contiguous columns per lane for ONE 16-B store (T21 for the 16x16 swapped
// layout): v_permlane16_swap exchanges lanes 16-31 of `a` with lanes 0-15 of `b` (and 48-63
// with 32-47), so lane fq holds columns (fq & 1) * 16 + (fq >> 1) * 8 + 0..7 of the pair.
__device__ __forceinline__ uint4 pair16(uint2 a, uint2 b) {
  const auto rx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return make_uint4(rx[0], ry[0], rx[1], ry[1]);
}

// Epilogue of the 4-wave 16x16x32 kernels (swapped layout, see k_gemm16).
template <int DT, int EPI>
__device__ __forceinline__ void epi16(const Args& a, v4f (&acc)[8][8], int tm, int tn, int w,
                                      int wr, int wc, int lane, int tid, char* lds) {
  // epilogue (swapped 16x16 layout): acc[m][n][j] = token tm*256 + wr*128 + m*16 + fr, tile
  // column wc*128 + n*16 + fq*4 + j (EPI_SILU: n < 4 gate, n + 4 up of output column
  // tn*128 + wc*64 + n*16 + fq*4 + j). Segment, bias and row pointers are resolved once per
  // tile / row (a tile never straddles a segment), loads are batched per row.
  const int fr = lane & 15, fq = lane >> 4;
  const int poff = (fq & 1) * 16 + (fq >> 1) * 8;  // pair16 column offset of this lane
  if constexpr (EPI == EPI_SILU) {
    const int64_t col0 = (int64_t)tn * 128 + wc * 64 + fq * 4;
    const bool wide = a.wide && (int64_t)tn * 128 + 128 <= a.n;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      if (trow >= a.m) break;
      uint16_t* crow = a.c[0] + trow * a.ldc[0] + col0;
      if (wide) {  // partner lanes (lane ^ 16) share the row: same branch
        uint2 wv[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float gg = rnd<DT>(acc[m][n][j]);
            const float u = rnd<DT>(acc[m][n + 4][j]);
            const float sl = rnd<DT>(gg / (1.0f + expf(-gg)));
            o[j] = rnd<DT>(sl * u);
          }
          wv[n].x = pack2<DT>(o[0], o[1]);
          wv[n].y = pack2<DT>(o[2], o[3]);
        }
        uint16_t* cpair = crow - fq * 4 + poff;
#pragma unroll
        for (int n = 0; n < 4; n += 2)
          *reinterpret_cast<uint4*>(cpair + n * 16) = pair16(wv[n], wv[n + 1]);
        continue;
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        if (col0 + n * 16 >= a.n) break;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gg = rnd<DT>(acc[m][n][j]);
          const float u = rnd<DT>(acc[m][n + 4][j]);
          const float sl = rnd<DT>(gg / (1.0f + expf(-gg)));
          o[j] = rnd<DT>(sl * u);
        }
        uint2 wv;
        wv.x = pack2<DT>(o[0], o[1]);
        wv.y = pack2<DT>(o[2], o[3]);
        *reinterpret_cast<uint2*>(crow + n * 16) = wv;
      }
    }
  } else {
    const int64_t tcol = (int64_t)tn * ST;
    int s = 0;
    int64_t base = 0;
    if (a.nseg > 1 && tcol >= a.bend[0]) { s = 1; base = a.bend[0]; }
    if (a.nseg > 2 && tcol >= a.bend[1]) { s = 2; base = a.bend[1]; }
    const int64_t col0 = tcol + wc * 128 + fq * 4;  // + n * 16
    const int64_t lcol0 = col0 - base;              // column within segment s
    const bool full_n = tcol + ST <= a.n;
    // bias (uniform presence): 4 values per n, read once
    float bias[8][4];
    const uint16_t* bp = a.bias[s];
    if (bp != nullptr) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        if (full_n || col0 + n * 16 < a.n) {
          float b4[4];
          unpack4<DT>(*reinterpret_cast<const uint2*>(bp + lcol0 + n * 16), b4);
#pragma unroll
          for (int j = 0; j < 4; ++j) bias[n][j] = b4[j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) bias[n][j] = 0.f;
        }
      }
    }
    double dsum = 0.0;
    // EPI_SQDIFF: the reference rows are loaded one row block ahead (16 loads in flight)
    uint2 rv[2][8];
    auto load_ref = [&](int m, uint2 (&dst)[8]) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      const uint16_t* rrow = a.ref + (trow < a.m ? trow : a.m - 1) * a.ldr + col0;
#pragma unroll
      for (int n = 0; n < 8; ++n)
        dst[n] = (full_n || col0 + n * 16 < a.n) ? *reinterpret_cast<const uint2*>(rrow + n * 16)
                                                 : make_uint2(0u, 0u);
    };
    if constexpr (EPI == EPI_SQDIFF) load_ref(0, rv[0]);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      if constexpr (EPI == EPI_SQDIFF) {
        if (m + 1 < 8) load_ref(m + 1, rv[(m + 1) & 1]);
      }
      if (trow >= a.m) continue;
      float o[8][4];
#pragma unroll
      for (int n = 0; n < 8; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[n][j] = rnd<DT>(bp != nullptr ? __fadd_rn(acc[m][n][j], bias[n][j]) : acc[m][n][j]);
      if constexpr (EPI == EPI_STORE) {
        uint16_t* crow = a.c[s] + trow * a.ldc[s] + lcol0;
        if (a.wide && full_n) {
          uint16_t* cpair = crow - fq * 4 + poff;
#pragma unroll
          for (int n = 0; n < 8; n += 2) {
            uint2 w0, w1;
            w0.x = pack2<DT>(o[n][0], o[n][1]);
            w0.y = pack2<DT>(o[n][2], o[n][3]);
            w1.x = pack2<DT>(o[n + 1][0], o[n + 1][1]);
            w1.y = pack2<DT>(o[n + 1][2], o[n + 1][3]);
            *reinterpret_cast<uint4*>(cpair + n * 16) = pair16(w0, w1);
          }
          continue;
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          if (!full_n && col0 + n * 16 >= a.n) break;
          uint2 wv;
          wv.x = pack2<DT>(o[n][0], o[n][1]);
          wv.y = pack2<DT>(o[n][2], o[n][3]);
          *reinterpret_cast<uint2*>(crow + n * 16) = wv;
        }
      } else {
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          if (!full_n && col0 + n * 16 >= a.n) break;
          float r[4];
          unpack4<DT>(rv[m & 1][n], r);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = rnd<DT>(r[j] - o[n][j]);
            dsum += (double)(d * d);
          }
        }
      }
    }
    if constexpr (EPI == EPI_SQDIFF) {
#pragma unroll
      for (int msk = 32; msk >= 1; msk >>= 1) dsum += __shfl_xor(dsum, msk, 64);
      __syncthreads();
      double* red = reinterpret_cast<double*>(lds);
      if (lane == 0) red[w] = dsum;
      __syncthreads();
      if (tid < 4) a.part[((int64_t)tm * a.n_nt + tn) * 4 + tid] = red[tid];
    }
  }
}

// DIAG (timing-only builds, LCQ_GEMM_DIAG; outputs wrong): bit 0 = operand descriptors with
// zero records (every LDS-DMA load dropped: no memory traffic, same instruction stream), bit 1
// = no s_barrier in the K loop (the counted waits stay)
template <int DT, int EPI, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) k_gemm16(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  int tm, tn;
  if (a.order == 1) {
    if (!tile_nb(a, bid, tm, tn)) return;
  } else {
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (!slot_tile(a, wgid, tm, tn)) return;
  }
  const int64_t nk = a.k / SKT;
  Stage4 st;
  make_stage16<EPI>(a, tm, tn, w, lane, st);
  if constexpr (DIAG & 1) {
    st.ra = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, (short)0, 0, 0x00020000);
    st.rb[0] = st.rb[1] = st.ra;
  }

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[2][2][2], bf[8][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 0, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 1, nk > 1 ? SKT * 2 : 0, w, i);
  wait_barrier<22>();
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int k = 0; k < 2; ++k) bf[n][k] = read_frag(lds + TILE_B, wc * 8 + n, k, lane);
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int k = 0; k < 2; ++k) af[0][m2][k] = read_frag(lds, wr * 8 + m2, k, lane);
  asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC

  for (int64_t t = 0; t < nk; ++t)
    ktile16<FP16, DIAG>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  epi16<DT, EPI>(a, acc, tm, tn, w, wr, wc, lane, tid, lds);
}

template <int DT, int EPI, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) k_gemm16b(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  int tm, tn;
  if (a.order == 1) {
    if (!tile_nb(a, bid, tm, tn)) return;
  } else {
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (!slot_tile(a, wgid, tm, tn)) return;
  }
  const int64_t nk = a.k / SKT;
  Stage4 st;
  make_stage16<EPI>(a, tm, tn, w, lane, st);
  if constexpr (DIAG & 1) {
    st.ra = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, (short)0, 0, 0x00020000);
    st.rb[0] = st.rb[1] = st.ra;
  }

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[2][2][2], bf[2][8][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 0, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 1, nk > 1 ? SKT * 2 : 0, w, i);
  wait_barrier<22>();
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int k = 0; k < 2; ++k) bf[0][n][k] = read_frag(lds + TILE_B, wc * 8 + n, k, lane);
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int k = 0; k < 2; ++k) af[0][m2][k] = read_frag(lds, wr * 8 + m2, k, lane);
  asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC

  int64_t t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile16b<FP16, 0, DIAG>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
    ktile16b<FP16, 1, DIAG>(acc, bf, af, st, lds, t + 1, nk, w, wr, wc, lane);
  }
  if (t < nk) ktile16b<FP16, 0, DIAG>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  epi16<DT, EPI>(a, acc, tm, tn, w, wr, wc, lane, tid, lds);
}

// ---------------------------------------------------------------------------------------
// Ring-buffer form of k_gemm16 (LCQ_GEMM_KERNEL=r): K-tile 32, NBR = 4 LDS buffers of 32 KB
// (A 16 KB + B 16 KB, sixteen 16-row x 32-k st_16x32 subtiles each), ONE barrier per K-tile.
// Iteration t: barrier (tile t+1 landed everywhere: counted vmcnt(16) = the 2 younger tiles'
// 8 pieces each; every wave is past iteration t-1, so tile t's buffer -- its fragments were
// read during t-1 -- is free), then 64 MFMAs on tile t's fragments (register set t & 1) with
// the 16 fragment reads of tile t+1 (other set) and the 8 LDS-DMA pieces of tile t+4 (into
// tile t's buffer) interleaved. A load is consumed three iterations after issue.
// ---------------------------------------------------------------------------------------
constexpr int SKR = 32;                 // K-tile
constexpr int NBR = 4;                  // ring depth (5: measured no faster)
constexpr int TILE_R = ST * SKR * 2;    // 16 KB: one operand tile
constexpr int BUFR = 2 * TILE_R;        // A + B

struct StageR {
  __amdgpu_buffer_rsrc_t ra;
  __amdgpu_buffer_rsrc_t rb[2];
  uint32_t aoff[4];
  uint32_t boff[4];
  int bsel;
};

// piece j (0..3) of wave w = subtile rb = w + 4 j of the A / B tile image
template <int EPI>
__device__ __forceinline__ void make_stage_r(const Args& a, int tm, int tn, int w, int lane,
                                             StageR& st) {
  const int64_t arow0 = (int64_t)tm * ST;
  st.ra = panel_rsrc(a.a + arow0 * a.lda);
  int64_t brow0 = 0, blast = 0;
  if constexpr (EPI == EPI_SILU) {
    st.rb[0] = panel_rsrc(a.b[0]);
    st.rb[1] = panel_rsrc(a.b[1]);
    blast = a.n - 1;
    brow0 = (int64_t)tn * 128;
  } else {
    const int64_t row0 = (int64_t)tn * ST;
    int s = 0;
    int64_t segbase = 0;
    if (a.nseg > 1 && row0 >= a.bend[0]) { s = 1; segbase = a.bend[0]; }
    if (a.nseg > 2 && row0 >= a.bend[1]) { s = 2; segbase = a.bend[1]; }
    brow0 = row0 - segbase;
    blast = a.bend[s] - segbase - 1;
    st.rb[0] = st.rb[1] = panel_rsrc(a.b[s] + brow0 * a.ldb);
  }
  st.bsel = 0;
  const int r = lane >> 2;
  const int pc = (lane & 3) * 16;
  const int lc = pc ^ (((r >> 3) & 1) << 5);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int rb = w + 4 * j;
    const int row = rb * 16 + r;
    int64_t ar = row;
    if (arow0 + ar > a.m - 1) ar = a.m - 1 - arow0;
    st.aoff[j] = (uint32_t)(ar * a.lda * 2 + lc);
    int64_t br;
    if constexpr (EPI == EPI_SILU) {
      if (((rb * 16) & 127) >= 64) st.bsel |= 1 << j;  // uniform: whole 16-row subtile
      br = brow0 + (row >> 7) * 64 + (row & 63);
      if (br > blast) br = blast;
    } else {
      br = row;
      if (brow0 + br > blast) br = blast - brow0;
    }
    st.boff[j] = (uint32_t)(br * a.ldb * 2 + lc);
  }
}

// piece idx (0..7) of one K-tile: 0..3 B subtiles, 4..7 A subtiles
__device__ __forceinline__ void load_r(const StageR& st, char* lds, int buf, int kofs, int w,
                                       int idx) {
  char* dA = lds + buf * BUFR;
  if (idx < 4) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(((st.bsel >> idx) & 1) ? st.rb[1] : st.rb[0],
                                             (lds_void_t*)(dA + TILE_R + (w + 4 * idx) * 1024),
                                             16, st.boff[idx], kofs, 0, 0);
  } else {
    const int j = idx - 4;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(st.ra, (lds_void_t*)(dA + (w + 4 * j) * 1024), 16,
                                             st.aoff[j], kofs, 0, 0);
  }
}

// 16x32 fragment of subtile rb (st_16x32 swizzle)
__device__ __forceinline__ v8s frag_r(const char* tile, int rb, int lane) {
  const int r = lane & 15;
  const int lc = (lane >> 4) * 16;
  const int pc = lc ^ (((r >> 3) & 1) << 5);
  return *reinterpret_cast<const v8s*>(tile + rb * 1024 + r * 64 + pc);
}

template <bool FP16, int P>
__device__ __forceinline__ void ring_iter(v4f (&acc)[8][8], v8s (&af)[2][8], v8s (&bf)[2][8],
                                          const StageR& st, char* lds, int64_t t, int64_t nk,
                                          int w, int wr, int wc, int lane) {
  wait_barrier<8 * (NBR - 2)>();
  const int64_t tl = t + NBR < nk ? t + NBR : nk - 1;  // past the end: re-fetch the last tile
  const int kofs = (int)(tl * (SKR * 2));
  const int lbuf = (int)(t % NBR);
  const char* nA = lds + ((t + 1) % NBR) * BUFR;
  const char* nB = nA + TILE_R;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const int m = i >> 3, n = i & 7;
    mfma16a<FP16>(acc[m][n], bf[P][n], af[P][m]);
    if ((i & 3) == 1) {
      const int q = i >> 2;
      if (q < 8) af[P ^ 1][q] = frag_r(nA, wr * 8 + q, lane);
      else bf[P ^ 1][q - 8] = frag_r(nB, wc * 8 + q - 8, lane);
    }
    if ((i & 7) == 3) load_r(st, lds, lbuf, kofs, w, i >> 3);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int DT, int EPI>
__global__ void __launch_bounds__(256, 1) k_gemm16r(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm, tn;
  if (!slot_tile(a, wgid, tm, tn)) return;
  const int64_t nk = a.k / SKR;  // even: K % 64 == 0
  StageR st;
  make_stage_r<EPI>(a, tm, tn, w, lane, st);

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[2][8], bf[2][8];
#pragma unroll
  for (int j = 0; j < NBR; ++j) {
    const int kofs = (int)((j < nk ? j : nk - 1) * (SKR * 2));
#pragma unroll
    for (int i = 0; i < 8; ++i) load_r(st, lds, j, kofs, w, i);
  }
  wait_barrier<8 * (NBR - 1)>();  // tile 0 landed
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    af[0][q] = frag_r(lds, wr * 8 + q, lane);
    bf[0][q] = frag_r(lds + TILE_R, wc * 8 + q, lane);
  }
  asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC

  for (int64_t t = 0; t < nk; t += 2) {
    ring_iter<FP16, 0>(acc, af, bf, st, lds, t, nk, w, wr, wc, lane);
    ring_iter<FP16, 1>(acc, af, bf, st, lds, t + 1, nk, w, wr, wc, lane);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  __syncthreads();  // every wave's DMA landed before the epilogue may reuse LDS
  epi16<DT, EPI>(a, acc, tm, tn, w, wr, wc, lane, tid, lds);
}

// ---------------------------------------------------------------------------------------
// Persistent form of k_gemm16 (probe, LCQ_GEMM_KERNEL=p). One workgroup per CU walks the tile
// slots wgid, wgid + G, ... (consecutive wgids share an XCD: each XCD's workgroups take one
// 4 x 8 tile block per round). The per-lane load offsets are the same for every tile: a tile
// only changes the three buffer descriptors (panel base + the bytes of valid rows, so rows
// past M / N / a segment end read as zeros instead of being clamped). The last two K-tiles
// of a tile load the NEXT tile's first two, so its prologue runs behind this tile's
// epilogue and the matrix pipe restarts without a memory wait.
// ---------------------------------------------------------------------------------------
struct Desc {
  __amdgpu_buffer_rsrc_t ra, rb0, rb1;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_n(const void* p, int64_t bytes) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7fffffff ? 0x7fffffff : bytes));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, nb, 0x00020000);
}

template <int EPI>
__device__ __forceinline__ Desc make_desc(const Args& a, int tm, int tn) {
  Desc d;
  const int64_t arow0 = (int64_t)tm * ST;
  int64_t arows = a.m - arow0;
  if (arows > ST) arows = ST;
  d.ra = rsrc_n(a.a + arow0 * a.lda, arows * a.lda * 2);
  if constexpr (EPI == EPI_SILU) {
    const int64_t brow0 = (int64_t)tn * 128;
    int64_t brows = a.n - brow0;
    if (brows > 128) brows = 128;
    d.rb0 = rsrc_n(a.b[0] + brow0 * a.ldb, brows * a.ldb * 2);
    d.rb1 = rsrc_n(a.b[1] + brow0 * a.ldb, brows * a.ldb * 2);
  } else {
    const int64_t row0 = (int64_t)tn * ST;
    int s = 0;
    int64_t segbase = 0;
    if (a.nseg > 1 && row0 >= a.bend[0]) { s = 1; segbase = a.bend[0]; }
    if (a.nseg > 2 && row0 >= a.bend[1]) { s = 2; segbase = a.bend[1]; }
    int64_t brows = a.bend[s] - row0;
    if (brows > ST) brows = ST;
    d.rb0 = d.rb1 = rsrc_n(a.b[s] + (row0 - segbase) * a.ldb, brows * a.ldb * 2);
  }
  return d;
}

// B piece j of wave w -> LDS subtile (row block rb, k half kb) = index rb * 2 + kb. Plain:
// subtile w + 4j. EPI_SILU: waves 0, 1 stage the 16 gate subtiles (row blocks 0-3, 8-11),
// waves 2, 3 the 16 up subtiles (4-7, 12-15), so every wave reads ONE B descriptor.
template <int EPI>
__device__ __forceinline__ int bsub(int w, int j) {
  if constexpr (EPI == EPI_SILU) {
    const int g = (w & 1) * 8 + j;
    const int rbi = g >> 1;
    const int rb = (rbi < 4 ? rbi : rbi + 4) + (w >= 2 ? 4 : 0);
    return rb * 2 + (g & 1);
  } else {
    return w + 4 * j;
  }
}

// tile-independent per-lane offsets of the 8 A and 8 B pieces (16-row subtiles, st_16x32)
template <int EPI>
__device__ __forceinline__ void make_offsets(const Args& a, int w, int lane, uint32_t (&aoff)[8],
                                             uint32_t (&boff)[8]) {
  const int r = lane >> 2;
  const int pc = (lane & 3) * 16;
  const int lc = pc ^ (((r >> 3) & 1) << 5);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int rb = (w >> 1) + 2 * j;
    aoff[j] = (uint32_t)((int64_t)(rb * 16 + r) * a.lda * 2 + (w & 1) * 64 + lc);
    const int sb = bsub<EPI>(w, j);
    const int row = (sb >> 1) * 16 + r;           // tile-local B row
    int brow = row;
    if constexpr (EPI == EPI_SILU) brow = (row >> 7) * 64 + (row & 63);  // row in gate / up
    boff[j] = (uint32_t)((int64_t)brow * a.ldb * 2 + (sb & 1) * 64 + lc);
  }
}

template <int EPI>
__device__ __forceinline__ void load_piece_d(const Desc& d, const uint32_t (&aoff)[8],
                                             const uint32_t (&boff)[8], char* lds, int buf,
                                             int kofs, int wu, int idx) {
  char* dA = lds + buf * BUF4;
  if (idx < 8) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        (EPI == EPI_SILU && wu >= 2) ? d.rb1 : d.rb0,
        (lds_void_t*)(dA + TILE_B + bsub<EPI>(wu, idx) * 1024), 16, boff[idx], kofs, 0, 0);
  } else {
    const int q = idx - 8;                       // 0..7 -> A piece 0,4,1,5,2,6,3,7
    const int j = (q >> 1) + 4 * (q & 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(d.ra, (lds_void_t*)(dA + (wu + 4 * j) * 1024), 16,
                                             aoff[j], kofs, 0, 0);
  }
}

template <bool FP16>
__device__ __forceinline__ void mfma16z(v4f& acc, v8s bfrag, v8s afrag) {  // C = 0
  if constexpr (FP16)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(bfrag), "v"(afrag));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(bfrag), "v"(afrag));
}

// one K-tile of k_gemm16p (schedule of ktile16); FIRST: kb = 0 MFMAs start from C = 0;
// LAST: no fragment reads of the next K-tile (the next tile's are read after the epilogue,
// so no fragment registers stay live across it)
template <bool FP16, bool FIRST, bool LAST, int EPI>
__device__ __forceinline__ void ktile16p(v4f (&acc)[8][8], v8s (&bf)[8][2], v8s (&af)[2][2][2],
                                         const Desc& d, const uint32_t (&aoff)[8],
                                         const uint32_t (&boff)[8], char* lds, int buf,
                                         int kofs, int w, int wr, int wc, int lane) {
  const char* At = lds + buf * BUF4;
  const char* An = lds + (buf ^ 1) * BUF4;
  const char* Bn = An + TILE_B;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int i = mm * 16 + n * 2 + kb;
          if (FIRST && kb == 0) mfma16z<FP16>(acc[2 * mb + mm][n], bf[n][kb], af[mb & 1][mm][kb]);
          else mfma16a<FP16>(acc[2 * mb + mm][n], bf[n][kb], af[mb & 1][mm][kb]);
          if (i == 7) {
            if (mb == 0 || mb == 3) wait_barrier<20>();
            else wait_barrier<28>();
          }
          if (mb == 0 && i >= 8 && i < 28 && (i & 1) == 0)
            load_piece_d<EPI>(d, aoff, boff, lds, buf, kofs, w, (i - 8) >> 1);
          if (mb > 0 && (i == 8 || i == 20))
            load_piece_d<EPI>(d, aoff, boff, lds, buf, kofs, w, 8 + 2 * mb + (i == 20));
          if (i >= 8 && i < 12) {
            const int q = i - 8, m2 = q >> 1, k2 = q & 1;
            if (mb < 3) af[(mb + 1) & 1][m2][k2] = read_frag(At, wr * 8 + 2 * (mb + 1) + m2, k2, lane);
            else if (!LAST) af[0][m2][k2] = read_frag(An, wr * 8 + m2, k2, lane);
          }
          if (!LAST && mb == 3 && mm == 1 && kb == 1) {
#pragma unroll
            for (int k3 = 0; k3 < 2; ++k3) bf[n][k3] = read_frag(Bn, wc * 8 + n, k3, lane);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
}

// K-tile fragments a workgroup starts a tile with: all B fragments, A block 0
__device__ __forceinline__ void first_frags(v8s (&bf)[8][2], v8s (&af)[2][2][2], const char* lds,
                                            int buf, int wr, int wc, int lane) {
  const char* A0 = lds + buf * BUF4;
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int k = 0; k < 2; ++k) bf[n][k] = read_frag(A0 + TILE_B, wc * 8 + n, k, lane);
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int k = 0; k < 2; ++k) af[0][m2][k] = read_frag(A0, wr * 8 + m2, k, lane);
}

__device__ __forceinline__ bool next_tile(const Args& a, int& slot, int stride, int& tm, int& tn) {
  while (slot < a.nslots) {
    if (slot_tile(a, slot, tm, tn)) return true;
    slot += stride;
  }
  return false;
}

template <int DT, int EPI>
__global__ void __launch_bounds__(256, 1) k_gemm16p(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  int slot = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  int tm, tn;
  if (!next_tile(a, slot, G, tm, tn)) return;
  const int64_t nk = a.k / SKT;  // >= 2 (host)
  uint32_t aoff[8], boff[8];
  make_offsets<EPI>(a, w, lane, aoff, boff);
  Desc d = make_desc<EPI>(a, tm, tn);

  v4f acc[8][8];
  v8s af[2][2][2], bf[8][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece_d<EPI>(d, aoff, boff, lds, 0, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece_d<EPI>(d, aoff, boff, lds, 1, SKT * 2, w, i);
  wait_barrier<22>();

  int buf = 0;  // LDS buffer of the current K-tile (parity of K-tiles run so far)
  for (;;) {
    int nslot = slot + G, ntm = 0, ntn = 0;
    const bool has_next = next_tile(a, nslot, G, ntm, ntn);
    const Desc dn = has_next ? make_desc<EPI>(a, ntm, ntn) : d;
    first_frags(bf, af, lds, buf, wr, wc, lane);
    // K-tile 0 (C = 0), K-tiles 1 .. nk-2, K-tile nk-1 (no next-fragment reads); loads of
    // step t fetch K-tile t+2 of this tile, or K-tile t+2-nk of the next one
    ktile16p<FP16, true, false, EPI>(acc, bf, af, nk > 2 ? d : dn, aoff, boff, lds, buf,
                                (int)((nk > 2 ? 2 : (has_next ? 0 : nk - 1)) * (SKT * 2)), w,
                                wr, wc, lane);
    buf ^= 1;
    for (int64_t t = 1; t < nk - 1; ++t) {
      const bool nx = t + 2 >= nk;
      const int64_t kl = !nx ? t + 2 : (has_next ? t + 2 - nk : nk - 1);
      ktile16p<FP16, false, false, EPI>(acc, bf, af, nx ? dn : d, aoff, boff, lds, buf,
                                   (int)(kl * (SKT * 2)), w, wr, wc, lane);
      buf ^= 1;
    }
    ktile16p<FP16, false, true, EPI>(acc, bf, af, dn, aoff, boff, lds, buf,
                                (int)((has_next ? 1 : nk - 1) * (SKT * 2)), w, wr, wc, lane);
    buf ^= 1;
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");  // last MFMA's D -> epilogue reads

    const int fr = lane & 15, fq = lane >> 4;
    if constexpr (EPI == EPI_SILU) {
      const int64_t col0 = (int64_t)tn * 128 + wc * 64 + fq * 4;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
        if (trow >= a.m) break;
        uint16_t* crow = a.c[0] + trow * a.ldc[0] + col0;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          if (col0 + n * 16 >= a.n) break;
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float gg = rnd<DT>(acc[m][n][j]);
            const float u = rnd<DT>(acc[m][n + 4][j]);
            const float sl = rnd<DT>(gg / (1.0f + expf(-gg)));
            o[j] = rnd<DT>(sl * u);
          }
          uint2 wv;
          wv.x = pack2<DT>(o[0], o[1]);
          wv.y = pack2<DT>(o[2], o[3]);
          *reinterpret_cast<uint2*>(crow + n * 16) = wv;
        }
      }
    } else {
      const int64_t tcol = (int64_t)tn * ST;
      int s = 0;
      int64_t base = 0;
      if (a.nseg > 1 && tcol >= a.bend[0]) { s = 1; base = a.bend[0]; }
      if (a.nseg > 2 && tcol >= a.bend[1]) { s = 2; base = a.bend[1]; }
      const int64_t col0 = tcol + wc * 128 + fq * 4;
      const int64_t lcol0 = col0 - base;
      const bool full_n = tcol + ST <= a.n;
      const uint16_t* bp = a.bias[s];
      double dsum = 0.0;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
        if (trow >= a.m) break;
        uint2 rv[8];
        if constexpr (EPI == EPI_SQDIFF) {
          const uint16_t* rrow = a.ref + trow * a.ldr + col0;
#pragma unroll
          for (int n = 0; n < 8; ++n)
            rv[n] = (full_n || col0 + n * 16 < a.n) ? *reinterpret_cast<const uint2*>(rrow + n * 16)
                                                    : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          if (!full_n && col0 + n * 16 >= a.n) break;
          float o[4];
          if (bp != nullptr) {
            float b4[4];
            unpack4<DT>(*reinterpret_cast<const uint2*>(bp + lcol0 + n * 16), b4);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = rnd<DT>(__fadd_rn(acc[m][n][j], b4[j]));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = rnd<DT>(acc[m][n][j]);
          }
          if constexpr (EPI == EPI_STORE) {
            uint2 wv;
            wv.x = pack2<DT>(o[0], o[1]);
            wv.y = pack2<DT>(o[2], o[3]);
            *reinterpret_cast<uint2*>(a.c[s] + trow * a.ldc[s] + lcol0 + n * 16) = wv;
          } else {
            float r[4];
            unpack4<DT>(rv[n], r);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float dd = rnd<DT>(r[j] - o[j]);
              dsum += (double)(dd * dd);
            }
          }
        }
      }
      if constexpr (EPI == EPI_SQDIFF) {
        // per-wave partial straight to memory (the LDS holds the next tile's K-tiles)
#pragma unroll
        for (int msk = 32; msk >= 1; msk >>= 1) dsum += __shfl_xor(dsum, msk, 64);
        if (lane == 0) a.part[((int64_t)tm * a.n_nt + tn) * 4 + w] = dsum;
      }
    }
    if (!has_next) break;
    slot = nslot;
    tm = ntm;
    tn = ntn;
    d = dn;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // tail re-fetches landed
}

// one wave: lane l sums partials l, l+64, ... in order, then a fixed xor tree (deterministic)
__global__ void __launch_bounds__(64) k_loss_reduce(const double* part, int64_t nparts,
                                                    int64_t numel, float* out, int slot) {
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < nparts; i += 64) s += part[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (threadIdx.x == 0) out[slot] = (float)s / (float)numel;
}

static void plan(Args& a, int64_t tile_n) {
  a.n_mt = (int)((a.m + ST - 1) / ST);
  a.n_nt = (int)((a.n + tile_n - 1) / tile_n);
  a.cpb = (a.n_nt + 7) / 8;
  const int bands = (a.n_mt + 3) / 4;
  a.nslots = 32 * bands * a.cpb;
  // N-band-major order when the M extent fills whole 32-tile regions (every XCD busy);
  // LCQ_GEMM_ORDER=0/1 forces one (read per launch: A/B probes flip it between calls)
  const char* e = getenv("LCQ_GEMM_ORDER");
  a.order = e ? (e[0] == '1') : 0;
  if (a.order == 1) a.nslots = 256 * ((a.n_mt + 31) / 32) * a.cpb;
}

template <int DT, int EPI>
static int launch(Args& a, hipStream_t st) {
  // the dynamic-LDS attribute is per device: set it on every launch (cheap, thread-safe)
  // default: k_gemm16b (4-wave 16x16x32, B fragments double-buffered, one tile per
  // workgroup); LCQ_GEMM_KERNEL=a (k_gemm16) | p (persistent) | r (ring) | w4 | w8 select probes
  const char* sel = getenv("LCQ_GEMM_KERNEL");  // per launch: A/B probes flip it
  if (sel && sel[0] == 'w' && sel[1] == '8') {
    (void)hipFuncSetAttribute((const void*)k_gemm256<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF_B);
    hipLaunchKernelGGL((k_gemm256<DT, EPI>), dim3((unsigned)a.nslots), 512, 2 * BUF_B, st, a);
  } else if (sel && sel[0] == 'w' && sel[1] == '4') {
    (void)hipFuncSetAttribute((const void*)k_gemm4w<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
    hipLaunchKernelGGL((k_gemm4w<DT, EPI>), dim3((unsigned)a.nslots), 256, 2 * BUF4, st, a);
  } else if (sel && sel[0] == 'r') {  // ring-buffer probe (K-tile 32, 4 buffers)
    (void)hipFuncSetAttribute((const void*)k_gemm16r<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, NBR * BUFR);
    hipLaunchKernelGGL((k_gemm16r<DT, EPI>), dim3((unsigned)a.nslots), 256, NBR * BUFR, st, a);
  } else if (const char* dg = (EPI == EPI_STORE && DT == LCQ_BF16) ? getenv("LCQ_GEMM_DIAG")
                                                                   : nullptr) {
    const int d = dg[0] - '0';  // timing-only diagnostic builds (outputs wrong)
    const bool b = !(sel && sel[0] == 'a');
    auto k = d == 1 ? (b ? k_gemm16b<DT, EPI, 1> : k_gemm16<DT, EPI, 1>)
           : d == 2 ? (b ? k_gemm16b<DT, EPI, 2> : k_gemm16<DT, EPI, 2>)
           : d == 3 ? (b ? k_gemm16b<DT, EPI, 3> : k_gemm16<DT, EPI, 3>)
                    : (b ? k_gemm16b<DT, EPI, 0> : k_gemm16<DT, EPI, 0>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * BUF4);
    hipLaunchKernelGGL(k, dim3((unsigned)a.nslots), 256, 2 * BUF4, st, a);
  } else if (!sel || sel[0] == 'b' || (sel[0] == 'p' && a.k < 2 * SKT)) {
    // the default: B fragments double-buffered in registers, one tile per workgroup
    (void)hipFuncSetAttribute((const void*)k_gemm16b<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
    hipLaunchKernelGGL((k_gemm16b<DT, EPI>), dim3((unsigned)a.nslots), 256, 2 * BUF4, st, a);
  } else if (sel[0] != 'p') {  // LCQ_GEMM_KERNEL=a: single B register set (previous default)
    (void)hipFuncSetAttribute((const void*)k_gemm16<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
    hipLaunchKernelGGL((k_gemm16<DT, EPI>), dim3((unsigned)a.nslots), 256, 2 * BUF4, st, a);
  } else {  // LCQ_GEMM_KERNEL=p: persistent probe (SGPR pressure still costs it; see DESIGN)
    (void)hipFuncSetAttribute((const void*)k_gemm16p<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
    int dev = 0, ncu = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int grid = a.nslots < ncu ? a.nslots : ncu;  // persistent: one workgroup per CU
    hipLaunchKernelGGL((k_gemm16p<DT, EPI>), dim3((unsigned)grid), 256, 2 * BUF4, st, a);
  }
  return check_launch("lcq_gemm: k_gemm");
}

template <int EPI>
static int dispatch(int dtype, Args& a, hipStream_t st) {
  if (dtype == LCQ_F16) return launch<LCQ_F16, EPI>(a, st);
  return launch<LCQ_BF16, EPI>(a, st);
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

static int check_common(int dtype, const void* x, int64_t lda, int64_t m, int64_t k,
                        int64_t ldb) {
  LCQ_REQUIRE(dtype == LCQ_BF16 || dtype == LCQ_F16, "dtype must be bf16 or fp16");
  LCQ_REQUIRE(m > 0 && k > 0, "empty GEMM");
  LCQ_REQUIRE(k % SKT == 0, "K must be a multiple of 64");
  LCQ_REQUIRE(lda >= k && lda % 8 == 0 && ldb >= k && ldb % 8 == 0,
              "row strides must be >= K and multiples of 8 elements");
  LCQ_REQUIRE(x != nullptr && aligned16(x), "A must be 16-byte aligned");
  LCQ_REQUIRE(lda < (int64_t)1 << 21 && ldb < (int64_t)1 << 21 && k < (int64_t)1 << 21,
              "row strides and K must be < 2^21 elements (32-bit panel offsets)");
  return 0;
}

// ---------------------------------------------------------------------------------------
// GPTQ Hessian SYRK on the k_gemm16b core (hessian256.hip's lcq_hessian_accum, LCQ_SYRK=16):
// H = beta*H + alpha * X^T X over the upper-triangle 256^2 tiles of the transposed, zero
// padded X^T panels (A = B = XT rows, k-contiguous), split-K over `ns` slabs when the
// triangle has few tiles. Tile order: slot -> (ti, tj) in chunks of 4 x 8 tiles walked band
// by band (12 panels per 32 tiles of one XCD), as k_syrk256.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool syrk_slot_tile(int slot, int nt, int& ti, int& tj) {
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

// v-th upper-triangle tile in the same 4 x 8 chunk order, counting valid tiles only: the grid
// is exactly ntiles x ns workgroups, so every XCD's contiguous wgid range holds the same number
// of live tiles (+-1) and the last round is as full as the tile count allows (no exiting slots
// that leave one XCD a round longer than the others)
__device__ __forceinline__ void syrk_valid_tile(int v, int nt, int& ti, int& tj) {
  for (int b = 0; 4 * b < nt; ++b) {
    const int nch = (nt - 4 * b + 7) / 8;
    for (int rem = 0; rem < nch; ++rem) {
      const int c0 = 4 * b + rem * 8, c1 = min(nt - 1, c0 + 7);
      for (int r = 0; r < 4; ++r) {
        const int i = 4 * b + r;
        if (i >= nt) break;
        const int lo = max(i, c0), cnt = c1 >= lo ? c1 - lo + 1 : 0;
        if (v < cnt) {
          ti = i;
          tj = lo + v;
          return;
        }
        v -= cnt;
      }
    }
  }
  ti = tj = 0;  // not reached for v < nt (nt + 1) / 2
}

struct SyrkArgs16 {
  const uint16_t* xt;
  int64_t kp, ic, icp;
  float* H;
  float* part;
  float alpha, beta;
  int nt, ns, ntiles;
  int64_t ktps;
};

template <bool FP16>
__global__ void __launch_bounds__(256, 1) k_syrk16(SyrkArgs16 s) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = wgid / s.ntiles;
  int ti, tj;
  syrk_valid_tile(wgid - split * s.ntiles, s.nt, ti, tj);
  const int64_t kt0 = (int64_t)split * s.ktps;
  int64_t nk = s.kp / SKT - kt0;
  if (nk > s.ktps) nk = s.ktps;
  Args a{};  // the GEMM view of this split: A = B = XT (k from column kt0 * 64 on)
  a.a = s.xt + kt0 * SKT;
  a.lda = s.kp;
  a.m = s.icp;
  a.k = nk * SKT;
  a.b[0] = a.a;
  a.bend[0] = s.icp;
  a.ldb = s.kp;
  a.n = s.icp;
  a.nseg = 1;
  Stage4 st;
  make_stage16<EPI_STORE>(a, ti, tj, w, lane, st);

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[2][2][2], bf[2][8][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 0, 0, w, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) load_piece(st, lds, 1, nk > 1 ? SKT * 2 : 0, w, i);
  wait_barrier<22>();
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int k = 0; k < 2; ++k) bf[0][n][k] = read_frag(lds + TILE_B, wc * 8 + n, k, lane);
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int k = 0; k < 2; ++k) af[0][m2][k] = read_frag(lds, wr * 8 + m2, k, lane);
  asm volatile("s_nop 4" ::: "memory");

  int64_t t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile16b<FP16, 0>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
    ktile16b<FP16, 1>(acc, bf, af, st, lds, t + 1, nk, w, wr, wc, lane);
  }
  if (t < nk) ktile16b<FP16, 0>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");

  // acc[m][n][jj] (swapped layout): H row i = ti*256 + wr*128 + m*16 + fr, columns
  // tj*256 + wc*128 + n*16 + fq*4 + jj
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t i0 = (int64_t)ti * ST + wr * 128 + fr;
  const int64_t j0 = (int64_t)tj * ST + wc * 128 + fq * 4;
  if (s.ns > 1) {
    float* P = s.part + (int64_t)split * s.icp * s.icp;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n)
        *reinterpret_cast<float4*>(P + (i0 + m * 16) * s.icp + j0 + n * 16) =
            make_float4(acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]);
    return;
  }
  const bool diag = ti == tj;
  const bool vec = (s.ic & 3) == 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int64_t i = i0 + m * 16;
    if (i >= s.ic) break;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int64_t j = j0 + n * 16;
      if (j >= s.ic) break;
      float o[4];
      const bool full = vec && j + 3 < s.ic;
      float h[4] = {0.f, 0.f, 0.f, 0.f};
      if (s.beta != 0.f) {
        if (full) {
          const float4 hv = *reinterpret_cast<const float4*>(s.H + i * s.ic + j);
          h[0] = hv.x; h[1] = hv.y; h[2] = hv.z; h[3] = hv.w;
        } else {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (j + jj < s.ic) h[jj] = s.H[i * s.ic + j + jj];
        }
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        float v = __fmul_rn(s.alpha, acc[m][n][jj]);
        if (s.beta != 0.f) v = __fadd_rn(__fmul_rn(s.beta, h[jj]), v);
        o[jj] = v;
      }
      if (full) {
        *reinterpret_cast<float4*>(s.H + i * s.ic + j) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (j + jj < s.ic) s.H[i * s.ic + j + jj] = o[jj];
      }
      if (!diag) {  // mirror H[j + jj][i]
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (j + jj < s.ic) s.H[(j + jj) * s.ic + i] = o[jj];
      }
    }
  }
}

}  // namespace g256

// host launcher used by lcq_hessian_accum (hessian256.hip) for LCQ_SYRK=16
int syrk16_launch(const uint16_t* xt, int64_t kp, int64_t ic, int64_t icp, float* H,
                  float* part, float alpha, float beta, int nt, int ns, int ntiles,
                  int64_t ktps, bool fp16, hipStream_t st) {
  g256::SyrkArgs16 s{xt, kp, ic, icp, H, part, alpha, beta, nt, ns, ntiles, ktps};
  auto k = fp16 ? g256::k_syrk16<true> : g256::k_syrk16<false>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * g256::BUF4);
  hipLaunchKernelGGL(k, dim3((unsigned)(ntiles * ns)), 256, 2 * g256::BUF4, st, s);
  return check_launch("lcq_hessian_accum: syrk16");
}
}  // namespace lcq

using namespace lcq;
using namespace lcq::g256;

extern "C" int lcq_gemm(const void* a, int dtype, int64_t lda, int64_t m, int64_t k, int nseg,
                        const void* const* b, const int64_t* b_rows, int64_t ldb,
                        const void* const* bias, void* const* c, const int64_t* ldc,
                        void* stream) {
  int rc = check_common(dtype, a, lda, m, k, ldb);
  if (rc) return rc;
  LCQ_REQUIRE(nseg >= 1 && nseg <= MAXSEG && b && b_rows && c && ldc, "1..3 segments");
  Args g{};
  g.a = reinterpret_cast<const uint16_t*>(a);
  g.lda = lda; g.m = m; g.k = k; g.ldb = ldb; g.nseg = nseg;
  int64_t end = 0;
  for (int s = 0; s < nseg; ++s) {
    LCQ_REQUIRE(b_rows[s] > 0 && b_rows[s] % 16 == 0, "segment rows must be multiples of 16");
    LCQ_REQUIRE(s == nseg - 1 || b_rows[s] % ST == 0,
                "all but the last segment must be multiples of 256 rows");
    LCQ_REQUIRE(b[s] && aligned16(b[s]) && c[s] && aligned8(c[s]), "segment pointers");
    LCQ_REQUIRE(ldc[s] >= b_rows[s] && ldc[s] % 4 == 0, "ldc must be >= rows, multiple of 4");
    end += b_rows[s];
    g.b[s] = reinterpret_cast<const uint16_t*>(b[s]);
    g.bend[s] = end;
    g.bias[s] = bias ? reinterpret_cast<const uint16_t*>(bias[s]) : nullptr;
    g.c[s] = reinterpret_cast<uint16_t*>(c[s]);
    g.ldc[s] = ldc[s];
  }
  g.n = end;
  g.wide = 1;
  for (int s = 0; s < nseg; ++s)
    if (!aligned16(c[s]) || ldc[s] % 8 != 0) g.wide = 0;
  plan(g, ST);
  return dispatch<EPI_STORE>(dtype, g, as_stream(stream));
}

extern "C" int lcq_gemm_silu_mul(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                                 const void* gate, const void* up, int64_t ldb, int64_t n,
                                 void* h, int64_t ldh, void* stream) {
  int rc = check_common(dtype, a, lda, m, k, ldb);
  if (rc) return rc;
  LCQ_REQUIRE(n > 0 && n % 16 == 0, "intermediate size must be a multiple of 16");
  LCQ_REQUIRE(gate && up && aligned16(gate) && aligned16(up) && h && aligned8(h),
              "gate / up / h pointers");
  LCQ_REQUIRE(ldh >= n && ldh % 4 == 0, "ldh must be >= n, multiple of 4");
  Args g{};
  g.a = reinterpret_cast<const uint16_t*>(a);
  g.lda = lda; g.m = m; g.k = k; g.ldb = ldb; g.n = n; g.nseg = 1;
  g.b[0] = reinterpret_cast<const uint16_t*>(gate);
  g.b[1] = reinterpret_cast<const uint16_t*>(up);
  g.c[0] = reinterpret_cast<uint16_t*>(h);
  g.ldc[0] = ldh;
  g.wide = aligned16(h) && ldh % 8 == 0;
  plan(g, 128);
  return dispatch<EPI_SILU>(dtype, g, as_stream(stream));
}

extern "C" int64_t lcq_gemm_sq_diff_workspace_bytes(int64_t m, int64_t n) {
  if (m <= 0 || n <= 0) return 0;
  return ((m + ST - 1) / ST) * ((n + ST - 1) / ST) * 4 * (int64_t)sizeof(double);
}

extern "C" int lcq_gemm_sq_diff(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                                const void* b, int64_t ldb, int64_t n, const void* bias,
                                const void* ref, int64_t ldr, void* workspace, int64_t ws_bytes,
                                void* out_f32, int slot, void* stream) {
  int rc = check_common(dtype, a, lda, m, k, ldb);
  if (rc) return rc;
  LCQ_REQUIRE(n > 0 && n % 16 == 0, "N must be a multiple of 16");
  LCQ_REQUIRE(b && aligned16(b) && ref && aligned8(ref) && ldr >= n && ldr % 4 == 0,
              "weight / ref pointers, ldr >= N multiple of 4");
  LCQ_REQUIRE(workspace && ws_bytes >= lcq_gemm_sq_diff_workspace_bytes(m, n),
              "workspace smaller than lcq_gemm_sq_diff_workspace_bytes");
  LCQ_REQUIRE(out_f32 != nullptr && slot >= 0, "loss slot");
  Args g{};
  g.a = reinterpret_cast<const uint16_t*>(a);
  g.lda = lda; g.m = m; g.k = k; g.ldb = ldb; g.n = n; g.nseg = 1;
  g.b[0] = reinterpret_cast<const uint16_t*>(b);
  g.bend[0] = n;
  g.bias[0] = reinterpret_cast<const uint16_t*>(bias);
  g.ref = reinterpret_cast<const uint16_t*>(ref);
  g.ldr = ldr;
  g.part = reinterpret_cast<double*>(workspace);
  plan(g, ST);
  hipStream_t st = as_stream(stream);
  rc = dispatch<EPI_SQDIFF>(dtype, g, st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_loss_reduce, 1, 64, 0, st, g.part, (int64_t)g.n_mt * g.n_nt * 4, m * n,
                     reinterpret_cast<float*>(out_f32), slot);
  return check_launch("lcq_gemm_sq_diff: reduce");
}
