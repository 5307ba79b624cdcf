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
//   EPI_RESID   C[t, c] = rnd(res[t, c] + rnd(acc + bias)): a block's `residual + o_proj(x)` /
//               `h + down_proj(m)` (the residual read through the ref pointer, one segment)
//   EPI_ROPE    EPI_STORE + the rotary embedding of the leading segments (q, k) on the rounded
//               outputs: transformers' apply_rotary_pos_emb, out = rnd(rnd(x cos) + rnd(rh(x) sin))
//               with rh(x) = cat(-x2, x1) -- a head (128 columns) is one wave's tile columns,
//               column c and its partner c +- 64 sit in the same lane (blocks n and n + 4)
//   EPI_SQDIFF  out = rnd(acc + bias) is never written: d = rnd(ref - out), the tile's
//               sum of fp32 d*d goes to an fp64 partial per tile; k_loss_reduce sums the
//               partials in tile order (deterministic) and writes sum / numel to a device slot
//               (calculate_loss without materialising `out`)
//
// Structure (k_gemm16h, the product; k_gemm16b is its round-4 predecessor, kept as a probe
// build): one 256-thread workgroup (4 waves, 2 x 2) per 256x256 output tile, each wave
// 128x128 = 8x8 accumulators of mfma_f32_16x16x32 in AGPRs. K-tile 64; A and B tiles staged by
// buffer-descriptor LDS-DMA (raw_ptr_buffer_load_lds) into two 64 KB LDS buffers; k_gemm16h
// double-buffers the fragments by k half and needs 3 barriers and one counted vmcnt per K-tile
// (k_gemm16b: 4 barriers, B fragments double-buffered across K-tiles). The MFMA runs swapped (B fragment as the A operand), so each
// lane's accumulator holds 4 consecutive output columns of one token row: 8 / 16-byte stores in
// the epilogues. Tile order is XCD-aware: consecutive work ids go to one XCD and a chunk of
// 32 = a 4 (M) x 8 (N) block of tiles shares 12 operand panels in L2.
#define LCQ_BF16_HW 1  // conversion-instruction RNE in the epilogues
#ifndef LCQ_PROBE_GEMM_PP
#define LCQ_PROBE_GEMM_PP 2
#endif
#include "lcq_common.h"

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
enum { EPI_STORE = 0, EPI_SILU = 1, EPI_SQDIFF = 2, EPI_RESID = 3, EPI_ROPE = 4, EPI_F32 = 5 };
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
  // EPI_ROPE: segments s < rope_segs are rotated (head dim 128 = one wave's 128 columns);
  // token row t = b * seq + p reads cos / sin [.., seq, 128] at b * cs_bstride + p * 128
  const uint16_t* cos;
  const uint16_t* sin;
  int64_t seq, cs_bstride;
  int rope_segs;
  // EPI_F32: c[0] is fp32, c = beta c + alpha acc (beta 0 never reads c); the K loop walks 6
  // segments of x6_kt K-tiles, segment s reading plane (x6_roles_* >> 2 s) & 3 of the
  // [rows][3][x6_kp] split operands (lcq_gemm_f32x6)
  float alpha, beta;
  int x6_kt, x6_kp;
  uint32_t x6_roles_a, x6_roles_b;
  // split K (grid y = x6_splits): split y sums K-tiles [y nk / S, (y + 1) nk / S) into the fp32
  // partial y of x6_part ([S][m][n]), folded in split order by k_x6_reduce
  int x6_splits;
  float* x6_part;
};

// chunk shape (probe build -DLCQ_PROBE_GEMM_CM=<tile rows per 32-tile chunk>; default 4 x 8)
#ifndef LCQ_PROBE_GEMM_CM
#define LCQ_PROBE_GEMM_CM 4
#endif
constexpr int CH_M = LCQ_PROBE_GEMM_CM, CH_N = 32 / CH_M;

// work slot -> tile (CH_M x CH_N blocks of tiles, bands of CH_M tile rows walked along N)
__device__ __forceinline__ bool slot_tile(const Args& a, int slot, int& tm, int& tn) {
  const int chunk = slot >> 5, s = slot & 31;
  const int band = chunk / a.cpb, c = chunk - band * a.cpb;
  tm = band * CH_M + s / CH_N;
  tn = c * CH_N + s % CH_N;
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

__device__ __forceinline__ v8s read_frag(const char* half_base, int rb, int kb, int lane) {
  const int r = lane & 15;
  const int lc = (lane >> 4) * 16;
  const int pc = lc ^ (((r >> 3) & 1) << 5);
  return *reinterpret_cast<const v8s*>(half_base + (rb * 2 + kb) * 1024 + r * 64 + pc);
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

// ---------------------------------------------------------------------------------------
// Operand staging: one 256-thread workgroup per 256x256 tile, 2 x 2 waves of 128 x 128; an
// operand tile (256 rows x 64 k, 32 KB) lands in LDS as 16 pieces of 1 KB per wave (16-row x
// 32-k subtiles, st_16x32 swizzle), double-buffered (A + B = 64 KB per buffer).
// ---------------------------------------------------------------------------------------
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

// ---------------------------------------------------------------------------------------
// k_gemm16b: 8 x 8 mfma_f32_16x16x32 accumulators per wave kept in AGPRs by an inline-asm
// MFMA ("+a": hipcc's allocator shuffles AGPRs around the builtin with 256 accumulators).
// (The 8-wave 256^2 kernel, the 32x32x16 4-wave kernel, the single-B-set, ring-buffer and
// persistent variants and the timing-only diagnostic builds were A/B probes of rounds 1-2;
// they were removed from the product library in round 3 -- see git history and DESIGN.md.)
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

// K-tile loop with the B fragments double-buffered in registers: the B
// fragments of K-tile t+1 are read during blocks 1 and 2 of K-tile t (8 per block, one per MFMA
// gap after that block's 4 A-fragment reads) into the other register set, instead of 16 reads
// in the last 16 MFMA gaps whose lgkmcnt the next K-tile's first MFMAs wait on. Block 1's
// barrier therefore retires K-tile t+1's B pieces (vmcnt 18: the 8 A pieces of K-tile t+1 and
// the 10 pieces of K-tile t+2 issued in block 0 are younger), ~1.3 K-tiles after their issue.
// P = register set of K-tile t (t & 1).
template <bool FP16, int P>
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
            if (mb == 1) wait_barrier<18>();
            else wait_barrier<20>();
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

// Epilogue of the 16x16x32 kernels (swapped layout): NB = 16-column blocks per wave (8 in the
// 4-wave kernels: wave columns of 128; 4 was the 8-wave ping-pong probe's 64, round 5).
template <int DT, int EPI, int NB>
__device__ __forceinline__ void epi16(const Args& a, v4f (&acc)[8][NB], int tm, int tn, int w,
                                      int wr, int wc, int lane, int tid, char* lds) {
  // epilogue (swapped 16x16 layout): acc[m][n][j] = token tm*256 + wr*128 + m*16 + fr, tile
  // column wc*NB*16 + n*16 + fq*4 + j (EPI_SILU: n < NB/2 gate, n + NB/2 up of output column
  // tn*128 + wc*NB*8 + n*16 + fq*4 + j). Segment, bias and row pointers are resolved once per
  // tile / row (a tile never straddles a segment), loads are batched per row.
  constexpr int NH = NB / 2;
  const int fr = lane & 15, fq = lane >> 4;
  const int poff = (fq & 1) * 16 + (fq >> 1) * 8;  // pair16 column offset of this lane
  if constexpr (EPI == EPI_F32) {
    // 4 consecutive fp32 columns per lane and block: one 16-B store (n % 4 == 0, ldc % 4 == 0)
    const int64_t col0 = (int64_t)tn * ST + wc * (NB * 16) + fq * 4;
    const bool full_n = (int64_t)tn * ST + ST <= a.n;
    const bool part = a.x6_splits > 1;
    float* cb = part ? a.x6_part + (int64_t)blockIdx.y * a.m * a.n : reinterpret_cast<float*>(a.c[0]);
    const int64_t ldc = part ? a.n : a.ldc[0];
    const float alpha = part ? 1.f : a.alpha, beta = part ? 0.f : a.beta;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      if (trow >= a.m) break;
      float* crow = cb + trow * ldc + col0;
      float4 cv[NB];
      if (beta != 0.f) {
#pragma unroll
        for (int n = 0; n < NB; ++n)
          cv[n] = (full_n || col0 + n * 16 < a.n) ? *reinterpret_cast<const float4*>(crow + n * 16)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        if (!full_n && col0 + n * 16 >= a.n) break;
        float4 o = make_float4(alpha * acc[m][n][0], alpha * acc[m][n][1],
                               alpha * acc[m][n][2], alpha * acc[m][n][3]);
        if (beta != 0.f) {
          o.x = __fadd_rn(beta * cv[n].x, o.x);
          o.y = __fadd_rn(beta * cv[n].y, o.y);
          o.z = __fadd_rn(beta * cv[n].z, o.z);
          o.w = __fadd_rn(beta * cv[n].w, o.w);
        }
        *reinterpret_cast<float4*>(crow + n * 16) = o;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_SILU) {
    const int64_t col0 = (int64_t)tn * 128 + wc * (NB * 8) + fq * 4;
    const bool wide = a.wide && (int64_t)tn * 128 + 128 <= a.n;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      if (trow >= a.m) break;
      uint16_t* crow = a.c[0] + trow * a.ldc[0] + col0;
      if (wide) {  // partner lanes (lane ^ 16) share the row: same branch
        uint2 wv[NH];
#pragma unroll
        for (int n = 0; n < NH; ++n) {
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float gg = rnd<DT>(acc[m][n][j]);
            const float u = rnd<DT>(acc[m][n + NH][j]);
            const float sl = rnd<DT>(gg / (1.0f + expf(-gg)));
            o[j] = rnd<DT>(sl * u);
          }
          wv[n].x = pack2<DT>(o[0], o[1]);
          wv[n].y = pack2<DT>(o[2], o[3]);
        }
        uint16_t* cpair = crow - fq * 4 + poff;
#pragma unroll
        for (int n = 0; n < NH; n += 2)
          *reinterpret_cast<uint4*>(cpair + n * 16) = pair16(wv[n], wv[n + 1]);
        continue;
      }
#pragma unroll
      for (int n = 0; n < NH; ++n) {
        if (col0 + n * 16 >= a.n) break;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gg = rnd<DT>(acc[m][n][j]);
          const float u = rnd<DT>(acc[m][n + NH][j]);
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
    const int64_t col0 = tcol + wc * (NB * 16) + fq * 4;  // + n * 16
    const int64_t lcol0 = col0 - base;              // column within segment s
    const bool full_n = tcol + ST <= a.n;
    // bias (uniform presence): 4 values per n, read once
    float bias[NB][4];
    const uint16_t* bp = a.bias[s];
    if (bp != nullptr) {
#pragma unroll
      for (int n = 0; n < NB; ++n) {
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
    uint2 rv[2][NB];
    auto load_ref = [&](int m, uint2 (&dst)[NB]) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      const uint16_t* rrow = a.ref + (trow < a.m ? trow : a.m - 1) * a.ldr + col0;
#pragma unroll
      for (int n = 0; n < NB; ++n)
        dst[n] = (full_n || col0 + n * 16 < a.n) ? *reinterpret_cast<const uint2*>(rrow + n * 16)
                                                 : make_uint2(0u, 0u);
    };
    if constexpr (EPI == EPI_SQDIFF || EPI == EPI_RESID) load_ref(0, rv[0]);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t trow = (int64_t)tm * ST + wr * 128 + m * 16 + fr;
      if constexpr (EPI == EPI_SQDIFF || EPI == EPI_RESID) {
        if (m + 1 < 8) load_ref(m + 1, rv[(m + 1) & 1]);
      }
      if (trow >= a.m) continue;
      float o[NB][4];
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[n][j] = rnd<DT>(bp != nullptr ? __fadd_rn(acc[m][n][j], bias[n][j]) : acc[m][n][j]);
      if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          float r[4];
          unpack4<DT>(rv[m & 1][n], r);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[n][j] = rnd<DT>(__fadd_rn(r[j], o[n][j]));
        }
      }
      if constexpr (EPI == EPI_ROPE) {
        static_assert(NB == 8, "rotary epilogue: one head per wave column");
        if (s < a.rope_segs) {
          const int64_t b = trow / a.seq, p = trow - b * a.seq;
          const uint16_t* cr = a.cos + b * a.cs_bstride + p * 128 + fq * 4;
          const uint16_t* sr = a.sin + b * a.cs_bstride + p * 128 + fq * 4;
          float cs[NB][4], sn[NB][4];
#pragma unroll
          for (int n = 0; n < NB; ++n) {
            unpack4<DT>(*reinterpret_cast<const uint2*>(cr + n * 16), cs[n]);
            unpack4<DT>(*reinterpret_cast<const uint2*>(sr + n * 16), sn[n]);
          }
#pragma unroll
          for (int n = 0; n < NB / 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float x1 = o[n][j], x2 = o[n + NB / 2][j];
              o[n][j] = rnd<DT>(rnd<DT>(x1 * cs[n][j]) + rnd<DT>(-x2 * sn[n][j]));
              o[n + NB / 2][j] =
                  rnd<DT>(rnd<DT>(x2 * cs[n + NB / 2][j]) + rnd<DT>(x1 * sn[n + NB / 2][j]));
            }
        }
      }
      if constexpr (EPI == EPI_STORE || EPI == EPI_RESID || EPI == EPI_ROPE) {
        uint16_t* crow = a.c[s] + trow * a.ldc[s] + lcol0;
        if (a.wide && full_n) {
          uint16_t* cpair = crow - fq * 4 + poff;
#pragma unroll
          for (int n = 0; n < NB; n += 2) {
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
        for (int n = 0; n < NB; ++n) {
          if (!full_n && col0 + n * 16 >= a.n) break;
          uint2 wv;
          wv.x = pack2<DT>(o[n][0], o[n][1]);
          wv.y = pack2<DT>(o[n][2], o[n][3]);
          *reinterpret_cast<uint2*>(crow + n * 16) = wv;
        }
      } else {
#pragma unroll
        for (int n = 0; n < NB; ++n) {
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
      // 4 partials per tile (an 8-wave NB = 4 layout folds waves q and q + 4: the same 64
      // columns, rows 0-127 and 128-255)
      if (tid < 4)
        a.part[((int64_t)tm * a.n_nt + tn) * 4 + tid] = NB == 8 ? red[tid] : red[tid] + red[tid + 4];
    }
  }
}

template <int DT, int EPI>
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
    ktile16b<FP16, 0>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
    ktile16b<FP16, 1>(acc, bf, af, st, lds, t + 1, nk, w, wr, wc, lane);
  }
  if (t < nk) ktile16b<FP16, 0>(acc, bf, af, st, lds, t, nk, w, wr, wc, lane);
  // The nops carry the last block's accumulators as operands: an epilogue read of them cannot
  // be scheduled above the wait (the asm MFMAs are opaque to the hazard recognizer; the earlier
  // blocks' results are >= 16 MFMAs old by now)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 7"
               : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                 "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7])
               :
               : "memory");

  epi16<DT, EPI, 8>(a, acc, tm, tn, w, wr, wc, lane, tid, lds);
}

// ---------------------------------------------------------------------------------------
// k_gemm16h: k_gemm16b's tile, waves, LDS image and staging with a three-barrier K-tile:
// the fragments are double-buffered by k half instead (set X0 = k 0-31 of the A and B
// fragments, X1 = k 32-63; 128 VGPRs), so every fragment read of a K-tile overlaps the other
// half's 64 MFMAs and the loop needs one vmcnt wait per K-tile:
//   MFMA  0-63  (X0): read X1.A of K-tile t | barrier 1 | DMA A of t+2, read X1.B | barrier 2 |
//                     DMA A, DMA B of t+2
//   MFMA 64-127 (X1): DMA B of t+2 | vmcnt(13) + barrier 3 (K-tile t+1 landed) |
//                     read X0 of K-tile t+1, DMA B of t+2
// K-tile t+2 goes into K-tile t's buffer: its A region after barrier 1 (every wave has read
// t's A halves), its B region after barrier 2. Each accumulator sees k 0-31 then 32-63 per
// K-tile, as in k_gemm16b: identical outputs.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void load_a(const Stage4& st, char* buf, int kofs, int w, int j) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(st.ra, (lds_void_t*)(buf + (w + 4 * j) * 1024), 16,
                                           st.aoff[j], kofs, 0, 0);
}

__device__ __forceinline__ void load_b(const Stage4& st, char* buf, int kofs, int w, int j) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(((st.bsel >> j) & 1) ? st.rb[1] : st.rb[0],
                                           (lds_void_t*)(buf + TILE_B + (w + 4 * j) * 1024), 16,
                                           st.boff[j], kofs, 0, 0);
}

__device__ __forceinline__ void lgkm_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// bc: the buffer of the current K-tile (DMA target of the K-tile two ahead, `st` at `kofs`),
// bn: the next K-tile's buffer
template <bool FP16>
__device__ __forceinline__ void ktile16h(v4f (&acc)[8][8], v8s (&x0a)[8], v8s (&x0b)[8],
                                         v8s (&x1a)[8], v8s (&x1b)[8], const Stage4& st,
                                         int kofs, int kofs_b, char* bc, const char* bn, int w,
                                         int wr, int wc, int lane) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int i = h * 64 + m * 8 + n;
    if (h == 0) mfma16a<FP16>(acc[m][n], x0b[n], x0a[m]);
    else mfma16a<FP16>(acc[m][n], x1b[n], x1a[m]);
    if (i < 16 && (i & 1) == 0) x1a[i >> 1] = read_frag(bc, wr * 8 + (i >> 1), 1, lane);
    if (i == 20) lgkm_barrier();
    if (i >= 22 && i <= 34 && (i - 22) % 3 == 0) load_a(st, bc, kofs, w, (i - 22) / 3);
    if (i == 24 || i == 27 || i == 30 || i == 33 || i == 36 || i == 38 || i == 40 || i == 42) {
      const int f = i <= 36 ? (i - 24) / 3 : 5 + (i - 38) / 2;
      x1b[f] = read_frag(bc + TILE_B, wc * 8 + f, 1, lane);
    }
    if (i == 50) lgkm_barrier();
    if (i == 52 || i == 55 || i == 58) load_a(st, bc, kofs, w, 5 + (i - 52) / 3);
    if (i == 61 || i == 64) load_b(st, bc, kofs_b, w, (i - 61) / 3);
    if (i == 85 || i == 87 || i == 89) load_b(st, bc, kofs_b, w, 2 + (i - 85) / 2);
    if (i == 91) {
      asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    if (i >= 93 && i <= 100) x0a[i - 93] = read_frag(bn, wr * 8 + (i - 93), 0, lane);
    if (i >= 101 && i <= 115 && ((i - 101) & 1) == 0)
      x0b[(i - 101) >> 1] = read_frag(bn + TILE_B, wc * 8 + ((i - 101) >> 1), 0, lane);
    if (i == 96 || i == 100) load_b(st, bc, kofs_b, w, 5 + (i - 96) / 4);
    if (i == 124) load_b(st, bc, kofs_b, w, 7);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int DT, int EPI>
__global__ void __launch_bounds__(256, 1) k_gemm16h(Args a) {
  constexpr bool FP16 = DT == LCQ_F16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nwg = gridDim.x, bid = blockIdx.x;
  int tm, tn;
  {
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (!slot_tile(a, wgid, tm, tn)) return;
  }
  int64_t nk = a.k / SKT;
  int kt0 = 0;  // first K-tile of this workgroup's split (EPI_F32 split K)
  if constexpr (EPI == EPI_F32) {
    if (a.x6_splits > 1) {
      const int y = blockIdx.y;
      kt0 = (int)(nk * y / a.x6_splits);
      nk = nk * (y + 1) / a.x6_splits - kt0;
    }
  }
  Stage4 st;
  make_stage16<EPI>(a, tm, tn, w, lane, st);

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s x0a[8], x0b[8], x1a[8], x1b[8];
  // byte offset of K-tile kt in the A / B rows (EPI_F32: its segment's plane)
  auto kofs_of = [&](int kt, uint32_t roles) -> int {
    if constexpr (EPI == EPI_F32) {
      kt += kt0;
      const int sgm = kt / a.x6_kt;
      const int p = (int)((roles >> (2 * sgm)) & 3u);
      return (p * a.x6_kp + (kt - sgm * a.x6_kt) * SKT) * 2;
    } else {
      (void)roles;
      return kt * (SKT * 2);
    }
  };
  const int k1 = nk > 1 ? 1 : 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) load_a(st, lds, kofs_of(0, a.x6_roles_a), w, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) load_b(st, lds, kofs_of(0, a.x6_roles_b), w, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) load_a(st, lds + BUF4, kofs_of(k1, a.x6_roles_a), w, j);
#pragma unroll
  for (int j = 0; j < 8; ++j) load_b(st, lds + BUF4, kofs_of(k1, a.x6_roles_b), w, j);
  wait_barrier<16>();  // K-tile 0 landed (K-tile 1's 16 pieces may be in flight)
#pragma unroll
  for (int m = 0; m < 8; ++m) x0a[m] = read_frag(lds, wr * 8 + m, 0, lane);
#pragma unroll
  for (int n = 0; n < 8; ++n) x0b[n] = read_frag(lds + TILE_B, wc * 8 + n, 0, lane);
  asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC
  for (int64_t t = 0; t < nk; ++t) {
    const int cur = (int)(t & 1);
    const int kt2 = (int)(t + 2 < nk ? t + 2 : nk - 1);
    ktile16h<FP16>(acc, x0a, x0b, x1a, x1b, st, kofs_of(kt2, a.x6_roles_a),
                   kofs_of(kt2, a.x6_roles_b), lds + cur * BUF4, lds + (cur ^ 1) * BUF4, w, wr,
                   wc, lane);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 7"
               : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                 "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7])
               :
               : "memory");
  epi16<DT, EPI, 8>(a, acc, tm, tn, w, wr, wc, lane, tid, lds);
}

// one 1024-thread workgroup: thread l sums partials l, l + 1024, ... in order, then a fixed
// xor tree per wave and the 16 wave sums in wave order (deterministic; 16 K partials at the
// down_proj shape: one wave took ~0.1 ms, 240 launches per AWQ block step)
__global__ void __launch_bounds__(1024) k_loss_reduce(const double* part, int64_t nparts,
                                                      int64_t numel, float* out, int slot) {
  __shared__ double ws[16];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < nparts; i += 1024) s += part[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += ws[w];
    out[slot] = (float)t / (float)numel;
  }
}

// tile order: 0 = per-XCD 4 x 8 chunks (slot_tile, the default), 1 = N-band-major (tile_nb,
// measured neutral; probe build -DLCQ_PROBE_GEMM_ORDER=1, scripts/probe_build.py)
#ifndef LCQ_PROBE_GEMM_ORDER
#define LCQ_PROBE_GEMM_ORDER 0
#endif
static constexpr int tile_order() { return LCQ_PROBE_GEMM_ORDER; }

static void plan(Args& a, int64_t tile_n) {
  a.n_mt = (int)((a.m + ST - 1) / ST);
  a.n_nt = (int)((a.n + tile_n - 1) / tile_n);
  a.cpb = (a.n_nt + CH_N - 1) / CH_N;
  const int bands = (a.n_mt + CH_M - 1) / CH_M;
  a.nslots = 32 * bands * a.cpb;
  a.order = tile_order();
  if (a.order == 1) a.nslots = 256 * ((a.n_mt + 31) / 32) * a.cpb;
}

// kernel: 2 = k_gemm16h (the product), 0 = k_gemm16b (probe build -DLCQ_PROBE_GEMM_PP=0, for
// A/B runs: 1.5-3 % slower on the AWQ shapes, profiles/r5_gemm_variants.md). Round 6 probes,
// measured and removed (profiles/r6_gemm_vs_hipblaslt.txt): a B ring three K-tiles deep
// (160 KB LDS) and a two-barrier K-tile (both k-half-1 fragment sets read first).
static constexpr int gemm_kernel() { return LCQ_PROBE_GEMM_PP; }

template <int DT, int EPI>
static int launch(Args& a, hipStream_t st) {
  // the dynamic-LDS attribute is per device: set it on every launch (cheap, thread-safe)
  if (gemm_kernel() == 2 && a.order == 0) {
    (void)hipFuncSetAttribute((const void*)k_gemm16h<DT, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
    const unsigned gy = (EPI == EPI_F32 && a.x6_splits > 1) ? (unsigned)a.x6_splits : 1u;
    hipLaunchKernelGGL((k_gemm16h<DT, EPI>), dim3((unsigned)a.nslots, gy), 256, 2 * BUF4, st, a);
    return check_launch("lcq_gemm: k_gemm16h");
  }
  (void)hipFuncSetAttribute((const void*)k_gemm16b<DT, EPI>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF4);
  hipLaunchKernelGGL((k_gemm16b<DT, EPI>), dim3((unsigned)a.nslots), 256, 2 * BUF4, st, a);
  return check_launch("lcq_gemm: k_gemm16b");
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
// fp32 products as bf16 MFMA (the factorisation chain's large updates, lcq_gemm_f32x6):
// fp32 MFMA runs at 1/16 of the bf16 rate on gfx950. Each fp32 operand value is split into
// three bf16 planes x = x0 + x1 + x2 (x0 = RN(x), x1 = RN(x - x0), x2 = RN(x - x0 - x1): ~24
// significant bits), and the six plane products down to the 2^-16 level,
//   a2 b0 + a1 b1 + a0 b2 + a1 b0 + a0 b1 + a0 b0   (small terms first),
// are ONE k_gemm16h GEMM over K' = 6 Kp with fp32 accumulation: its K loop walks six segments,
// reading planes (2 1 0 1 0 0) of A and (0 1 2 0 1 0) of B, stored once per row as
// [plane][Kp] (Kp = K rounded up to 64, zero padded; ROLES_*). Dropped terms are
// O(2^-24) relative, like fp32 rounding (scripts/chain_split_study.py: the chain's inverse
// factor is as accurate as with the fp32 GEMM).
// ---------------------------------------------------------------------------------------
constexpr uint32_t ROLES_A = 2u | 1u << 2 | 0u << 4 | 1u << 6 | 0u << 8 | 0u << 10;
constexpr uint32_t ROLES_B = 0u | 1u << 2 | 2u << 4 | 0u << 6 | 1u << 8 | 0u << 10;

__device__ __forceinline__ void split3(float x, uint16_t& p0, uint16_t& p1, uint16_t& p2) {
  const float h0 = bf16_rne_hw(x);
  const float r1 = x - h0;            // exact
  const float h1 = bf16_rne_hw(r1);
  const float h2 = bf16_rne_hw(r1 - h1);
  p0 = (uint16_t)(__float_as_uint(h0) >> 16);
  p1 = (uint16_t)(__float_as_uint(h1) >> 16);
  p2 = (uint16_t)(__float_as_uint(h2) >> 16);
}

// 8 consecutive k of one row -> its three planes in dst (16 B each, kp apart)
__device__ __forceinline__ void put_split8(const float (&v)[8], uint16_t* drow, int64_t kp) {
  uint16_t p[3][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split3(v[j], p[0][j], p[1][j], p[2][j]);
  uint4 q[3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
    q[i] = make_uint4((uint32_t)p[i][0] | (uint32_t)p[i][1] << 16,
                      (uint32_t)p[i][2] | (uint32_t)p[i][3] << 16,
                      (uint32_t)p[i][4] | (uint32_t)p[i][5] << 16,
                      (uint32_t)p[i][6] | (uint32_t)p[i][7] << 16);
#pragma unroll
  for (int i = 0; i < 3; ++i) *reinterpret_cast<uint4*>(drow + i * kp) = q[i];
}

// row-major source: element (r, k) at src[r * ld + k]; one thread per (row, 8 k)
__global__ void __launch_bounds__(256) k_split3(const float* src, int64_t ld, int64_t rows,
                                                int64_t k, int64_t kp, uint16_t* dst,
                                                int64_t ldd) {
  const int64_t g8 = kp / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * g8) return;
  const int64_t r = i / g8, k0 = (i - r * g8) * 8;
  const float* s = src + r * ld + k0;
  float v[8];
  if (k0 + 8 <= k && (ld & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
    const float4 a = *reinterpret_cast<const float4*>(s);
    const float4 b = *reinterpret_cast<const float4*>(s + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = k0 + j < k ? s[j] : 0.f;
  }
  put_split8(v, dst + r * ldd + k0, kp);
}

// transposed source: element (r, k) at src[k * ld + r]; a 64 (r) x 64 (k) tile per workgroup
// through LDS (coalesced reads along r, 16-B segment writes along k)
__global__ void __launch_bounds__(256) k_split3_t(const float* src, int64_t ld, int64_t rows,
                                                  int64_t k, int64_t kp, uint16_t* dst,
                                                  int64_t ldd) {
  __shared__ float t[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64, k0 = (int64_t)blockIdx.y * 64;
  const int tid = threadIdx.x;
  // reads: 16 k-rows of 64 r per pass, all 16 loads issued before the LDS writes
  float ld16[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int kk = i * 4 + (tid >> 6), rr = tid & 63;
    const int64_t gk = k0 + kk, gr = r0 + rr;
    ld16[i] = (gk < k && gr < rows) ? src[gk * ld + gr] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) t[i * 4 + (tid >> 6)][tid & 63] = ld16[i];
  __syncthreads();
  // writes: 8 lanes per row cover its 64 k (128 B per plane contiguous); LDS bank of
  // (kg, rr) = 8 kg + rr + 65 j mod 64: conflict-free over a wave
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int task = h * 256 + tid;
    const int kg = task & 7, rr = task >> 3;  // kg 0..7: k 8 kg .. 8 kg + 7
    const int64_t gr = r0 + rr, gk = k0 + kg * 8;
    if (gr >= rows || gk >= kp) continue;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[kg * 8 + j][rr];
    put_split8(v, dst + gr * ldd + gk, kp);
  }
}


// out = beta out + alpha (part_0 + part_1 + ...) in split order (4 columns per thread)
__global__ void __launch_bounds__(256) k_x6_reduce(const float* part, int splits, int64_t rows,
                                                   int64_t n, float* c, int64_t ldc,
                                                   float alpha, float beta) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, n4 = n / 4;
  if (i >= rows * n4) return;
  const int64_t r = i / n4, c4 = (i - r * n4) * 4;
  float4 acc = *reinterpret_cast<const float4*>(part + r * n + c4);
  for (int sp = 1; sp < splits; ++sp) {
    const float4 v = *reinterpret_cast<const float4*>(part + (sp * rows + r) * n + c4);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  float4 o = make_float4(alpha * acc.x, alpha * acc.y, alpha * acc.z, alpha * acc.w);
  float* cp = c + r * ldc + c4;
  if (beta != 0.f) {
    const float4 cv = *reinterpret_cast<const float4*>(cp);
    o.x = __fadd_rn(beta * cv.x, o.x);
    o.y = __fadd_rn(beta * cv.y, o.y);
    o.z = __fadd_rn(beta * cv.z, o.z);
    o.w = __fadd_rn(beta * cv.w, o.w);
  }
  *reinterpret_cast<float4*>(cp) = o;
}

}  // namespace g256

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

extern "C" int lcq_gemm_rope(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                             int nseg, const void* const* b, const int64_t* b_rows, int64_t ldb,
                             const void* const* bias, void* const* c, const int64_t* ldc,
                             int rope_segs, const void* cos, const void* sin, int64_t seq,
                             int64_t cs_bstride, int64_t head_dim, void* stream) {
  int rc = check_common(dtype, a, lda, m, k, ldb);
  if (rc) return rc;
  LCQ_REQUIRE(nseg >= 1 && nseg <= MAXSEG && b && b_rows && c && ldc, "1..3 segments");
  LCQ_REQUIRE(head_dim == 128, "the rotary epilogue takes head_dim 128 (one wave column)");
  LCQ_REQUIRE(rope_segs >= 0 && rope_segs <= nseg, "rope_segs must be 0..nseg");
  LCQ_REQUIRE(seq > 0 && m % seq == 0, "m must be a whole number of sequences");
  LCQ_REQUIRE(cos && sin && aligned8(cos) && aligned8(sin) && cs_bstride >= 0 &&
                  cs_bstride % 4 == 0, "cos / sin [1 or B, seq, 128], 8-byte aligned");
  Args g{};
  g.a = reinterpret_cast<const uint16_t*>(a);
  g.lda = lda; g.m = m; g.k = k; g.ldb = ldb; g.nseg = nseg;
  int64_t end = 0;
  for (int s = 0; s < nseg; ++s) {
    LCQ_REQUIRE(b_rows[s] > 0 && b_rows[s] % 16 == 0, "segment rows must be multiples of 16");
    LCQ_REQUIRE(s == nseg - 1 || b_rows[s] % ST == 0,
                "all but the last segment must be multiples of 256 rows");
    LCQ_REQUIRE(s >= rope_segs || b_rows[s] % ST == 0, "rotated segments: multiples of 256");
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
  g.cos = reinterpret_cast<const uint16_t*>(cos);
  g.sin = reinterpret_cast<const uint16_t*>(sin);
  g.seq = seq;
  g.cs_bstride = cs_bstride;
  g.rope_segs = rope_segs;
  plan(g, ST);
  return dispatch<EPI_ROPE>(dtype, g, as_stream(stream));
}

extern "C" int lcq_gemm_residual(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                                 const void* b, int64_t ldb, int64_t n, const void* bias,
                                 const void* res, int64_t ldr, void* c, int64_t ldc,
                                 void* stream) {
  int rc = check_common(dtype, a, lda, m, k, ldb);
  if (rc) return rc;
  LCQ_REQUIRE(n > 0 && n % 16 == 0, "N must be a multiple of 16");
  LCQ_REQUIRE(b && aligned16(b) && res && aligned8(res) && ldr >= n && ldr % 4 == 0,
              "weight / residual pointers, ldr >= N multiple of 4");
  LCQ_REQUIRE(c && aligned8(c) && ldc >= n && ldc % 4 == 0, "c pointer, ldc >= N multiple of 4");
  Args g{};
  g.a = reinterpret_cast<const uint16_t*>(a);
  g.lda = lda; g.m = m; g.k = k; g.ldb = ldb; g.n = n; g.nseg = 1;
  g.b[0] = reinterpret_cast<const uint16_t*>(b);
  g.bend[0] = n;
  g.bias[0] = reinterpret_cast<const uint16_t*>(bias);
  g.c[0] = reinterpret_cast<uint16_t*>(c);
  g.ldc[0] = ldc;
  g.ref = reinterpret_cast<const uint16_t*>(res);
  g.ldr = ldr;
  g.wide = aligned16(c) && ldc % 8 == 0;
  plan(g, ST);
  return dispatch<EPI_RESID>(dtype, g, as_stream(stream));
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
  hipLaunchKernelGGL(k_loss_reduce, 1, 1024, 0, st, g.part, (int64_t)g.n_mt * g.n_nt * 4, m * n,
                     reinterpret_cast<float*>(out_f32), slot);
  return check_launch("lcq_gemm_sq_diff: reduce");
}

// ---- fp32 GEMM on bf16 MFMA (split planes; see k_split3) ---------------------------------
static int64_t x6_kp(int64_t k) { return (k + SKT - 1) / SKT * SKT; }

// K splits of the FULL M x N x K product (so every row range of it sums the same K-tile
// groups): enough workgroups for the 256 CUs, >= 16 K-tiles per split
static int x6_splits(int64_t M, int64_t n, int64_t k, int max_splits) {
  const int64_t tiles = ((M + ST - 1) / ST) * ((n + ST - 1) / ST);
  int64_t sp = tiles >= 256 ? 1 : 256 / tiles;
  const int64_t nk = 6 * x6_kp(k) / SKT;
  if (sp > max_splits) sp = max_splits;
  if (sp > 8) sp = 8;
  while (sp > 1 && nk / sp < 16) --sp;
  return (int)sp;
}

extern "C" int64_t lcq_gemm_f32x6_workspace_bytes(int64_t M, int64_t rows, int64_t n,
                                                  int64_t k, int max_splits) {
  if (M <= 0 || rows <= 0 || n <= 0 || k <= 0 || max_splits < 1) return 0;
  const int sp = x6_splits(M, n, k, max_splits);
  return (rows + n) * 3 * x6_kp(k) * 2 + (sp > 1 ? sp * rows * n * 4 : 0) + 512;
}

extern "C" int lcq_gemm_f32x6(int64_t M, int64_t N, int64_t K, float alpha, const void* A,
                              int64_t lda, int at, const void* B, int64_t ldb, int bt,
                              float beta, void* C, int64_t ldc, int64_t row0, int64_t row1,
                              int max_splits, void* workspace, int64_t ws_bytes, void* stream) {
  LCQ_REQUIRE(M > 0 && N > 0 && K > 0 && 0 <= row0 && row0 <= row1 && row1 <= M,
              "shape / row range");
  if (row0 == row1) return LCQ_OK;   // an empty rank share of a row split (as lcq_gemm_f32_rows)
  LCQ_REQUIRE(N % 16 == 0 && ldc % 4 == 0 && ldc >= N, "N % 16 == 0, ldc % 4 == 0");
  LCQ_REQUIRE(A && B && C && aligned16(C), "pointers (C 16-byte aligned)");
  LCQ_REQUIRE((at ? lda >= M : lda >= K) && (bt ? ldb >= K : ldb >= N), "leading dimensions");
  LCQ_REQUIRE(max_splits >= 1, "max_splits >= 1");
  const int64_t kp = x6_kp(K), rows = row1 - row0;
  LCQ_REQUIRE(6 * kp < ((int64_t)1 << 21), "K too large for 32-bit panel offsets");
  LCQ_REQUIRE(workspace && aligned16(workspace) &&
                  ws_bytes >= lcq_gemm_f32x6_workspace_bytes(M, rows, N, K, max_splits),
              "workspace smaller than lcq_gemm_f32x6_workspace_bytes");
  hipStream_t st = as_stream(stream);
  const int64_t ldd = 3 * kp;  // [rows][3 planes][kp]
  uint16_t* ap = reinterpret_cast<uint16_t*>(workspace);
  uint16_t* bp = ap + rows * ldd;
  const float* a32 = reinterpret_cast<const float*>(A) + (at ? row0 : row0 * lda);
  const float* b32 = reinterpret_cast<const float*>(B);
  if (at) {  // A stored k-major [K, lda]: row r of A is column r
    hipLaunchKernelGGL(k_split3_t, dim3((unsigned)((rows + 63) / 64), (unsigned)((kp + 63) / 64)),
                       256, 0, st, a32, lda, rows, K, kp, ap, ldd);
  } else {
    const int64_t items = rows * (kp / 8);
    hipLaunchKernelGGL(k_split3, dim3((unsigned)((items + 255) / 256)), 256, 0, st, a32, lda,
                       rows, K, kp, ap, ldd);
  }
  if (bt) {
    const int64_t items = N * (kp / 8);
    hipLaunchKernelGGL(k_split3, dim3((unsigned)((items + 255) / 256)), 256, 0, st, b32, ldb, N,
                       K, kp, bp, ldd);
  } else {
    hipLaunchKernelGGL(k_split3_t, dim3((unsigned)((N + 63) / 64), (unsigned)((kp + 63) / 64)),
                       256, 0, st, b32, ldb, N, K, kp, bp, ldd);
  }
  int rc = check_launch("lcq_gemm_f32x6: split");
  if (rc) return rc;
  Args g{};
  g.a = ap;
  g.lda = ldd; g.m = rows; g.k = 6 * kp; g.ldb = ldd; g.n = N; g.nseg = 1;
  g.b[0] = bp;
  g.bend[0] = N;
  g.c[0] = reinterpret_cast<uint16_t*>(reinterpret_cast<float*>(C) + row0 * ldc);
  g.ldc[0] = ldc;
  g.alpha = alpha;
  g.beta = beta;
  g.x6_kt = (int)(kp / SKT);
  g.x6_kp = (int)kp;
  g.x6_roles_a = ROLES_A;
  g.x6_roles_b = ROLES_B;
  g.x6_splits = x6_splits(M, N, K, max_splits);
  if (g.x6_splits > 1) {
    const uintptr_t pp = reinterpret_cast<uintptr_t>(bp + N * ldd);
    g.x6_part = reinterpret_cast<float*>((pp + 255) & ~(uintptr_t)255);
  }
  plan(g, ST);
  rc = launch<LCQ_BF16, EPI_F32>(g, st);
  if (rc || g.x6_splits == 1) return rc;
  const int64_t items = rows * (N / 4);
  hipLaunchKernelGGL(k_x6_reduce, dim3((unsigned)((items + 255) / 256)), 256, 0, st, g.x6_part,
                     g.x6_splits, rows, N, reinterpret_cast<float*>(C) + row0 * ldc, ldc, alpha,
                     beta);
  return check_launch("lcq_gemm_f32x6: reduce");
}
