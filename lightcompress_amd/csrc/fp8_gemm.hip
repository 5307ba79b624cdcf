// Block-scaled FP8 GEMM for FP8-weight (DeepSeek-V3-style) linears on gfx950 — the
// calibration forward of an fp8 checkpoint without a bf16 round trip of the weight.
//
// Replaces llmc/compression/quantization/kernel.py:141-242 (fp8_gemm, a Triton kernel) as
// called by block_wise_fp8_forward_func (module_utils.py:41-46):
//   C[m, n] = sum_kb ( sum_{k in block kb} A[m, k] B[n, k] ) * a_s[m, kb] * b_s[n / 128, kb]
// A [M, K] e4m3 (act_quant output, per-token 128-column scales a_s [M, K/128]); B [N, K] e4m3
// with 128x128 block scales b_s [ceil(N/128), K/128]; fp32 accumulation; C fp32 / bf16 / fp16.
//
// Kernels: k_fp8_gemm2 (256x256 tiles on the 16x16x128 MFMA, split-K on grids under 224
// tiles) for batches of more than 64 rows whose 256^2 grid has >= 64 tiles (gemm2_plan), its
// 128x128 sibling k_fp8_gemm2_128 (L2-fill-bound for fp8, reached through the probe hook
// only), and k_fp8_gemm for everything else:
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
        else if (g.c_dt == LCQ_F16) st1<LCQ_F16>(g.c, m * g.N + n, acc[i][j][r]);
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
    else if (c_dt == LCQ_F16) st1<LCQ_F16>(c, i, v);
    else st1<LCQ_BF16>(c, i, v);
  }
}

// ---------------------------------------------------------------------------------------
// gemm2_body<TM, WR, WC>: TM x TM tile, WR x WC waves of (TM/WR) x (TM/WC) each, gfx950's
// 16x16x128 f8f6f4 MFMA: ONE instruction is the whole 128-wide scale block's dot product of a
// 16 x 16 sub-tile, so the block scaling needs no second accumulator set: dot (4 VGPRs, C = 0)
// then acc = fma(dot, a_s[m, kb] * b_s[n / 128, kb], acc) (4 FMAs, the lane's 4 values share
// one row m in the swapped layout). The reference rounds (dot * a_s) * b_s + acc three times;
// this rounds the scale product and one fma: <= 2 ulp of each block term (tested against the
// oracle at 1e-5 of |a||b|).
//   256^2, 8 waves (2 per SIMD, 2 (M) x 4 (N), 128 x 64 each): 128 accumulator VGPRs per wave,
//     ~200 VGPRs; for grids that fill the chip.
//   128^2, 4 waves (one per SIMD, 64 x 64 each): 4x the tiles of the same problem, so a
//     2048 x 2048 output (DSv3 expert gate / up at 2048 calibration tokens) is 256 workgroups
//     instead of 64; smaller grids split K on top (fp32 partials summed in split order).
// Operands stream through LDS by LDS-DMA (buffer_load ... lds, 16 B per lane; 8 rows of 128 B
// per wave-instruction, 4 A and 4 B pieces per wave per K block in both instances) into two
// stage buffers (A TM x 128 B + B TM x 128 B, 16-B chunks XOR-swizzled per row, swz), plus the K
// block's TM a_s values (kb-major copy made by k_as_transpose; 4 B per lane from the first
// TM / 64 waves: an LDS-DMA lane writes a whole dword). One barrier per K block: after it the
// next K block's loads go into the buffer every wave finished reading.
// ---------------------------------------------------------------------------------------
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

template <int TM>
constexpr int stage_bytes() { return 2 * TM * BK + TM * 4; }  // A + B + TM fp32 a_s

struct Gemm2Args {
  const uint8_t* a;
  const uint8_t* b;
  const float* ast;   // a_s transposed, [nkb][mp] (mp = M rounded up to 256)
  const float* bs;    // [ceil(N/128), nkb]
  void* c;
  float* ws;          // split-K partials or null
  int64_t M, N, K, mp;
  int64_t kb_per_split;
  int c_dt;
  int nmt, nnt;
  int64_t ast_elems;  // a_s floats readable from ast (the grouped kernel shifts ast per group)
  const int64_t* arows;  // grouped, gathered A: tile row i reads A row arows[i] (null: a + i)
  int64_t a_bytes;       // bytes of A behind `a` when gathered
  const uint8_t* b2;     // SILU pair mode: the up weight (b = gate) and its block-scales
  const float* bs2;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  const int nb = __builtin_amdgcn_readfirstlane(
      (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo),
                                           (short)0, nb, 0x00020000);
}

// 16-B chunk c (0..7) of row r of an operand tile lives at physical chunk c ^ swz(r). A
// fragment read (lane l: row l & 15 of a 16-row block, chunks 2q and 2q + 1, q = l >> 4) puts
// each ds_read_b128 lane group of 16 on 16 distinct 16-byte bank slots with this swizzle (found
// by exhaustive search over per-row tables; XOR by r & 7 gave every lane a 2-way conflict:
// 47 % of the LDS cycles, profiles/r3c_gemm_pmc.txt)
__device__ __forceinline__ int swz(int row) { return ((row >> 1) & 1) | ((row >> 1) & 4); }

__device__ __forceinline__ v8i frag2(const uint8_t* tile, int row, int q) {
  const uint8_t* rp = tile + row * BK;
  const int c0 = (2 * q) ^ swz(row), c1 = (2 * q + 1) ^ swz(row);
  const uint4 lo = *reinterpret_cast<const uint4*>(rp + c0 * 16);
  const uint4 hi = *reinterpret_cast<const uint4*>(rp + c1 * 16);
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z,
             (int)hi.w};
}

// XCD-aware order of one GEMM's tiles: the 32 workgroups an XCD runs at once take a 4 (M) x 8
// (N) block (sharing 4 A row bands and 8 B column bands in that XCD's L2)
__device__ __forceinline__ bool tile_of_slot(const Gemm2Args& g, int& tm, int& tn) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int cpb = (g.nnt + 7) / 8;
  const int chunk = wg >> 5, sl = wg & 31, band = chunk / cpb, cc = chunk - band * cpb;
  tm = band * 4 + (sl >> 3);
  tn = cc * 8 + (sl & 7);
  return tm < g.nmt && tn < g.nnt;
}

// SILU (256^2, 8 waves only): the pair mode of the grouped MoE gate / up projection. The tile
// covers 128 output columns n0h = 128 tn of BOTH weights: virtual B row v (0..255) is gate
// (bit 5 of v clear) or up (set) column n0h + 32 (v >> 6) + (v & 31), so each wave's 64 tile
// columns hold 32 gate and the same 32 up columns (its accumulator blocks nb 0-1 and 2-3) and
// the epilogue writes h = rnd(rnd(silu(rnd(g))) * rnd(u)) (LlamaMLP / DeepseekV3MLP
// act_fn(gate_proj(x)) * up_proj(x) on the bf16 projections) -- neither projection is
// stored. A staging wave loads only gate (waves 0-3) or only up (4-7) rows.
template <int TM, int WR, int WC, int NS, bool SILU = false>
__device__ __forceinline__ void gemm2_body(const Gemm2Args& g, uint8_t* lds, int tm, int tn,
                                           int kz) {
  static_assert(!SILU || (TM == 256 && WR == 2 && WC == 4), "pair mode: 256^2, 2 x 4 waves");
  constexpr int NW = WR * WC;                 // waves
  constexpr int OPB = TM * BK;                // one operand tile
  constexpr int STG = stage_bytes<TM>();
  constexpr int WM = TM / WR, WN = TM / WC;   // wave tile
  constexpr int MB = WM / 16, NB = WN / 16;
  constexpr int PIECES = TM / (8 * NW);       // 8-row pieces per wave and operand
  constexpr int LPS = 2 * PIECES + 1;         // loads per wave per stage (vmcnt units)
  static_assert(PIECES * 8 * NW == TM && WN <= 128 && TM % 64 == 0, "tile shape");
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / WC, wc = w % WC;
  const int64_t m0 = (int64_t)tm * TM, n0 = SILU ? (int64_t)tn * (TM / 2) : (int64_t)tn * TM;
  const int64_t nkb = g.K / BK;
  const int64_t kb0 = (int64_t)kz * g.kb_per_split;
  int64_t nk = nkb - kb0;
  if (nk > g.kb_per_split) nk = g.kb_per_split;

  // staging: piece j of wave w = rows j * 8 NW + w * 8 .. + 7 of A and of B; 8 rows x 128 B =
  // 64 lanes x 16 B; lane l -> row l / 8, physical chunk l % 8 = logical chunk (l % 8) ^ swz(row)
  const __amdgpu_buffer_rsrc_t ra =
      g.arows ? rsrc(g.a, g.a_bytes) : rsrc(g.a + m0 * g.K, (g.M - m0) * g.K);
  const __amdgpu_buffer_rsrc_t rb =
      rsrc((SILU && w >= 4 ? g.b2 : g.b) + n0 * g.K, (g.N - n0) * g.K);
  const __amdgpu_buffer_rsrc_t rs = rsrc(g.ast + m0, (g.ast_elems - m0) * 4);
  uint32_t off[PIECES], aoff[PIECES], boff[PIECES];
#pragma unroll
  for (int j = 0; j < PIECES; ++j) {
    const int row = j * 8 * NW + w * 8 + (lane >> 3);
    off[j] = (uint32_t)(row * g.K + (((lane & 7) ^ swz(row)) * 16));
    aoff[j] = off[j];
    boff[j] = off[j];
    if (SILU) {  // virtual row -> column of the gate / up weight
      const int r = (row >> 6) * 32 + (row & 31);
      boff[j] = (uint32_t)(r * g.K + (((lane & 7) ^ swz(row)) * 16));
    }
    if (g.arows) {  // gathered rows; rows past M read past the descriptor's range: zeros
      const int64_t m = m0 + row;
      aoff[j] = m < g.M ? (uint32_t)(g.arows[m] * g.K + (((lane & 7) ^ swz(row)) * 16))
                        : 0x80000000u;
    }
  }
  auto stage = [&](int buf, int64_t kbl) {  // kbl: K block index within the split
    const int64_t kb = kb0 + (kbl < nk ? kbl : nk - 1);
    uint8_t* dst = lds + buf * STG;
    const int kofs = (int)(kb * BK);
#pragma unroll
    for (int j = 0; j < PIECES; ++j) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(dst + (j * 8 * NW + w * 8) * BK),
                                               16, aoff[j], kofs, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)(dst + OPB +
                                                                 (j * 8 * NW + w * 8) * BK),
                                               16, boff[j], kofs, 0, 0);
    }
    // a_s of this K block: TM floats = TM / 64 pieces of 64 lanes x 4 B; wave w loads piece
    // w % (TM / 64) (the waves past TM / 64 write the same bytes again) so that every wave
    // issues LPS loads per stage and the K loop can wait with one counted vmcnt
    const int sp = w % (TM / 64);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(dst + 2 * OPB + sp * 256), 4,
                                             (uint32_t)(sp * 256 + lane * 4),
                                             (int)(kb * g.mp * 4), 0, 0);
  };

  v4f acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const v4f zero = {0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, q = lane >> 4;
  // the split's weight block-scales of the tile's TM / 128 column blocks, staged in LDS once (a
  // global load per K block sat on every block's accumulation path: ~5x the MFMA time at
  // 128^2, profiles/r3c_gemm_pmc.txt)
  float* bsl = reinterpret_cast<float*>(lds + NS * STG);
  for (int i = tid; i < (TM / 128) * nk; i += 64 * NW) {
    const int cb = i / (int)nk, t = i - cb * (int)nk;
    int64_t nb = (n0 >> 7) + (SILU ? 0 : cb);   // SILU: cb 0 = gate's block, 1 = up's
    if (nb > (g.N - 1) >> 7) nb = (g.N - 1) >> 7;  // clamped past N (columns never stored)
    bsl[i] = (SILU && cb ? g.bs2 : g.bs)[nb * nkb + kb0 + t];
  }
  __syncthreads();
  const float* bsrow = bsl + (SILU ? 0 : ((wc * WN) >> 7) * nk);  // the wave's scale block

  // NS-stage ring: NS - 1 K blocks in flight ahead of the one being multiplied. (Round 4
  // measured two reschedulings of this loop slower on every shape, 1.64 -> 1.45 PF at
  // 2048 x 7168 x 7168: all of a K block's LDS reads issued first with the scaled
  // accumulation software-pipelined one row block behind the MFMAs, and a buffer's B half
  // refilled after a second barrier so that B streams two K blocks ahead;
  // profiles/r4_fp8_gemm_rate_resched.txt against r3d_fp8_gemm_rate.txt.)
#pragma unroll
  for (int j = 0; j + 1 < NS; ++j) stage(j, j);
  for (int64_t t = 0; t < nk; ++t) {
    const int buf = (int)(t % NS);
    // this K block's pieces landed (the NS - 2 younger stages may still be in flight) ...
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * LPS) : "memory");
    __builtin_amdgcn_s_barrier();  // ... for every wave; buffer (t - 1) % NS is free
    stage((int)((t + NS - 1) % NS), t + NS - 1);  // past the end: re-fetch (unused)
    const uint8_t* At = lds + buf * STG;
    const uint8_t* Bt = At + OPB;
    const float* Sa = reinterpret_cast<const float*>(At + 2 * OPB);
    const float bsv = bsrow[t];
    const float bsv2 = SILU ? bsrow[nk + t] : bsv;  // up's block-scale (nb >= NB / 2)
    v8i bfr[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bfr[nb] = frag2(Bt, wc * WN + nb * 16 + r16, q);
    float sc[MB], sc2[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      sc[mb] = Sa[wr * WM + mb * 16 + r16] * bsv;
      sc2[mb] = SILU ? Sa[wr * WM + mb * 16 + r16] * bsv2 : sc[mb];
    }
    v8i afr = frag2(At, wr * WM + r16, q);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      v8i anext = afr;
      if (mb < MB - 1) anext = frag2(At, wr * WM + (mb + 1) * 16 + r16, q);
      v4f d[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        d[nb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bfr[nb], afr, zero, 0, 0, 0, 0,
                                                                  0, 0);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[mb][nb][j] = __builtin_fmaf(d[nb][j], (SILU && nb >= NB / 2) ? sc2[mb] : sc[mb],
                                          acc[mb][nb][j]);
      afr = anext;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (SILU) {  // h[m][n0 + 32 wc + 16 nb + 4q + j] from acc[mb][nb] (gate), [nb + 2] (up)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int64_t m = m0 + wr * WM + mb * 16 + r16;
      if (m >= g.M) continue;
#pragma unroll
      for (int nb = 0; nb < NB / 2; ++nb) {
        const int64_t n = n0 + wc * 32 + nb * 16 + 4 * q;
        if (n >= g.N) continue;
        float h[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gg = rnd<LCQ_BF16>(acc[mb][nb][j]);
          const float u = rnd<LCQ_BF16>(acc[mb][nb + NB / 2][j]);
          h[j] = rnd<LCQ_BF16>(rnd<LCQ_BF16>(gg / (1.0f + expf(-gg))) * u);
        }
        uint2 o;
        o.x = pack2<LCQ_BF16>(h[0], h[1]);
        o.y = pack2<LCQ_BF16>(h[2], h[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(g.c) + m * g.N + n) = o;
      }
    }
    return;
  }
  // acc[mb][nb][j] (swapped layout): C[m0 + wr*WM + mb*16 + r16][n0 + wc*WN + nb*16 + 4q + j]
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int64_t m = m0 + wr * WM + mb * 16 + r16;
    if (m >= g.M) continue;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int64_t n = n0 + wc * WN + nb * 16 + 4 * q;
      if (n >= g.N) continue;
      const v4f v = acc[mb][nb];
      if (g.ws) {
        *reinterpret_cast<float4*>(g.ws + ((int64_t)kz * g.M + m) * g.N + n) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else if (g.c_dt == LCQ_F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.c) + m * g.N + n) =
            make_float4(v[0], v[1], v[2], v[3]);
      } else if (g.c_dt == LCQ_F16) {
        uint2 o;
        o.x = pack2<LCQ_F16>(v[0], v[1]);
        o.y = pack2<LCQ_F16>(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(g.c) + m * g.N + n) = o;
      } else {
        uint2 o;
        o.x = pack2<LCQ_BF16>(v[0], v[1]);
        o.y = pack2<LCQ_BF16>(v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(g.c) + m * g.N + n) = o;
      }
    }
  }
}

// 256^2: 2 stages (133 KB; ~2000 MFMA cycles per K block cover the load latency); 128^2: 4
// stages (133 KB; a K block is only ~500 MFMA cycles, measured 1.4 us per K block with 2)
constexpr int NS256 = 2, NS128 = 4;

__global__ __launch_bounds__(512, 1) void k_fp8_gemm2(Gemm2Args g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int tm, tn;
  if (!tile_of_slot(g, tm, tn)) return;
  gemm2_body<256, 2, 4, NS256>(g, lds, tm, tn, blockIdx.z);
}

__global__ __launch_bounds__(256, 1) void k_fp8_gemm2_128(Gemm2Args g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  int tm, tn;
  if (!tile_of_slot(g, tm, tn)) return;
  gemm2_body<128, 2, 2, NS128>(g, lds, tm, tn, blockIdx.z);
}

// ---------------------------------------------------------------------------------------
// Grouped GEMM: G independent problems C_g = A_g B_g^T (the routed experts of one MoE layer,
// one launch per projection). A is the tokens sorted by expert, [rows, K] e4m3 with rows
// [row_off[g], row_off[g + 1]) for group g (row_off on the device: the routing never visits the
// host); group g's weight and block-scales are wtab[2 g], wtab[2 g + 1] (device pointers, all
// [N, K] / [ceil(N/128), K/128]); C is [rows, N] in the same row order. Each output row is
// computed exactly as the single-problem k_fp8_gemm2 computes it unsplit (same body, same K
// order), so grouping changes which rows share a launch, not a row's value.
//   k_group_tiles (one workgroup per group) lays the groups' 256^2 tile slots end to end: group
//   g owns slots [tile0[g], tile0[g + 1]), nmt_g x 8 ceil(nnt / 8) of them, and writes its
//   group index into tmap for each; the last group also writes the total.
//   k_fp8_gemm2_grouped runs on an upper bound of the slot count: XCD x takes slots
//   [x q, (x + 1) q), q = ceil(total / 8), so one XCD walks consecutive tiles of one or two
//   experts (their A bands and B columns stay in its L2); inside a group, 4 (M) x 8 (N) tile
//   blocks (a last band of nmt % 4 rows) so that the 32 concurrent workgroups of an XCD share
//   operands as in the single-problem order. Slots past N's tile count return at once.
// ---------------------------------------------------------------------------------------
struct GroupedArgs {
  const uint8_t* a;
  const float* ast;      // [nkb][mp] (k_as_transpose of the act_quant scales, sorted rows)
  const int64_t* row_off;
  const int64_t* wtab;   // [nsets][G][2]: weight, block-scales
  const int* tile0;      // [G + 1]
  const int* tmap;       // [slots]: group of each slot
  const int64_t* arows;  // sorted row -> A row, or null (A already sorted)
  int64_t a_bytes;
  void* c;               // [nsets][rows][N], or [rows][N] (silu)
  int64_t N, K, mp, rows;
  int G, c_dt, nnt, nsets;
  int silu;              // nsets 2 as gate / up, h = act(gate) * up stored (the pair mode)
};

__global__ __launch_bounds__(256) void k_group_tiles(const int64_t* __restrict__ row_off, int G,
                                                     int nnt, int* __restrict__ tile0,
                                                     int* __restrict__ tmap) {
  __shared__ int part[256];
  const int g = blockIdx.x, tid = threadIdx.x;
  const int row8 = 8 * ((nnt + 7) / 8);
  int s = 0;  // slots of the groups before g
  for (int j = tid; j < g; j += 256)
    s += (int)((row_off[j + 1] - row_off[j] + 255) / 256) * row8;
  part[tid] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) part[tid] += part[tid + w];
    __syncthreads();
  }
  const int base = part[0];
  const int mine = (int)((row_off[g + 1] - row_off[g] + 255) / 256) * row8;
  if (tid == 0) {
    tile0[g] = base;
    if (g == G - 1) tile0[G] = base + mine;
  }
  for (int i = tid; i < mine; i += 256) tmap[base + i] = g;
}

__device__ __forceinline__ void grouped_body(const GroupedArgs& ga, uint8_t* lds,
                                             const bool SILU) {
  const int bid = blockIdx.x;
  const int sets = SILU ? 1 : ga.nsets;   // the pair mode's tile holds both weights
  const int total = __builtin_amdgcn_readfirstlane(ga.tile0[ga.G]) * sets;
  const int q = (total + 7) >> 3;
  const int j = bid >> 3, vs = (bid & 7) * q + j;
  if (j >= q || vs >= total) return;  // the grid covers 8 q slots (host bound)
  // the weight sets of one tile are consecutive slots (they read the same A rows)
  const int slot = vs / sets, set = vs - slot * sets;
  const int grp = __builtin_amdgcn_readfirstlane(ga.tmap[slot]);
  const int64_t r0 = ga.row_off[grp], M = ga.row_off[grp + 1] - r0;
  const int l = slot - ga.tile0[grp];
  const int nmt = (int)((M + 255) / 256), cpb = (ga.nnt + 7) / 8;
  // 4 x 8 blocks over full 4-row bands, then the last band's (nmt % 4) x 8 blocks
  const int full = nmt / 4, fslots = full * 32 * cpb;
  int tm, tn;
  if (l < fslots) {
    const int chunk = l >> 5, sl = l & 31, band = chunk / cpb, cc = chunk - band * cpb;
    tm = band * 4 + (sl >> 3);
    tn = cc * 8 + (sl & 7);
  } else {
    const int bh = nmt - full * 4, ll = l - fslots, cs = bh * 8;
    const int cc = ll / cs, sl = ll - cc * cs;
    tm = full * 4 + sl / 8;
    tn = cc * 8 + (sl & 7);
  }
  if (tn >= ga.nnt) return;
  const int64_t nkb = ga.K / BK;
  const int64_t wi = 2 * ((int64_t)set * ga.G + grp);
  Gemm2Args g{ga.arows ? ga.a : ga.a + r0 * ga.K,
              reinterpret_cast<const uint8_t*>(ga.wtab[wi]),
              ga.ast + r0,
              reinterpret_cast<const float*>(ga.wtab[wi + 1]),
              static_cast<uint8_t*>(ga.c) +
                  ((int64_t)set * ga.rows + r0) * ga.N * (ga.c_dt == LCQ_F32 ? 4 : 2),
              nullptr, M, ga.N, ga.K, ga.mp, nkb, ga.c_dt, nmt, ga.nnt,
              ga.mp * nkb - r0, ga.arows ? ga.arows + r0 : nullptr, ga.a_bytes,
              SILU ? reinterpret_cast<const uint8_t*>(ga.wtab[2 * ((int64_t)ga.G + grp)])
                   : nullptr,
              SILU ? reinterpret_cast<const float*>(ga.wtab[2 * ((int64_t)ga.G + grp) + 1])
                   : nullptr};
  if (SILU) gemm2_body<256, 2, 4, NS256, true>(g, lds, tm, tn, 0);
  else gemm2_body<256, 2, 4, NS256, false>(g, lds, tm, tn, 0);
}

__global__ __launch_bounds__(512, 1) void k_fp8_gemm2_grouped(GroupedArgs ga) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  grouped_body(ga, lds, false);
}

__global__ __launch_bounds__(512, 1) void k_fp8_gemm2_grouped_silu(GroupedArgs ga) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  grouped_body(ga, lds, true);
}

// a_s [M, nkb] -> [nkb, mp] (rows past M zero)
__global__ __launch_bounds__(256) void k_as_transpose(const float* __restrict__ as, int64_t M,
                                                      int64_t nkb, int64_t mp,
                                                      float* __restrict__ out,
                                                      const int64_t* __restrict__ rows) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nkb * mp) return;
  const int64_t kb = i / mp, m = i - kb * mp;
  out[i] = m < M ? as[(rows ? rows[m] : m) * nkb + kb] : 0.f;
}

// Tile plan. An fp8 K block of a 128^2 tile is 4.2 MFLOP per 32 KB staged (128 flop/B): at the
// CU's 8192 fp8 flop/cycle that needs ~64 B/cycle of L2 -> LDS fill, about twice what a CU
// gets (profiles/r3c_gemm_pmc.txt, r3c_fp8_gemm_rate.txt: 78-83 us at 2048 x 2048 x 7168 with
// the MFMAs ~17 % busy), so the 16x16x128 body runs 256^2 tiles (256 flop/B): unsplit when they
// fill >= 7/8 of the chip, split along K (>= 4 K blocks per split, ~256 workgroups) from 64
// tiles up; smaller grids take the 32x32x64 kernel with its 64-row tiles (tm = 0). 128^2 is
// kept for the probe hook only.
struct Plan2 {
  int tm;          // 256, 128 (probe), or 0: the <= 64-row-tile kernel
  int64_t splits;  // K splits (1: C written directly)
};

static int64_t split_count(int64_t tiles, int64_t nkb, int64_t full) {
  if (tiles >= full) return 1;
  int64_t s = (256 + tiles - 1) / tiles;
  if (s > nkb / 4) s = nkb / 4;
  if (s < 2) return 1;
  const int64_t per = (nkb + s - 1) / s;
  return (nkb + per - 1) / per;  // no empty split
}

Plan2 gemm2_plan(int64_t M, int64_t N, int64_t K) {
  const int64_t t256 = ((M + 255) / 256) * ((N + 255) / 256), nkb = K / BK;
  if (M <= 64 || t256 < 64) return {0, 1};
  return {256, split_count(t256, nkb, 224)};
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

// plan override for A/B probes (lcq_fp8_gemm_force_plan): 0 = auto, 1 = the <= 64-row kernel,
// 128 / 256 = that tile (split-K as gemm2_plan computes for it)
static int g_force_plan = 0;

static Plan2 pick_plan(int64_t M, int64_t N, int64_t K) {
  if (g_force_plan == 1) return {0, 1};
  if (g_force_plan == 128 || g_force_plan == 256) {
    const int tm = g_force_plan;
    const int64_t tiles = ((M + tm - 1) / tm) * ((N + tm - 1) / tm);
    return {tm, split_count(tiles, K / BK, tm == 256 ? 224 : 192)};
  }
  return gemm2_plan(M, N, K);
}

// workspace of the 16x16x128 kernels: the kb-major a_s copy, then the split-K partials
static int64_t ws2_bytes(int64_t M, int64_t N, int64_t K) {
  const int64_t mp = (M + 255) / 256 * 256, nkb = K / BK;
  // the largest split count any plan takes (a forced plan fits the queried workspace too)
  int64_t s = 1;
  for (int tm : {128, 256}) {
    const int64_t tiles = ((M + tm - 1) / tm) * ((N + tm - 1) / tm);
    const int64_t c = split_count(tiles, nkb, tm == 256 ? 224 : 192);
    if (c > s) s = c;
  }
  return nkb * mp * 4 + (s > 1 ? s * M * N * 4 : 0);
}

extern "C" int64_t lcq_fp8_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || K % BK != 0) return 0;
  const int64_t s = gemm_splits(M, N, K);
  const int64_t old = s > 1 ? s * M * N * (int64_t)sizeof(float) : 0;
  const int64_t w2 = ws2_bytes(M, N, K);
  return old > w2 ? old : w2;
}

extern "C" int lcq_fp8_gemm_force_plan(int plan) {
  LCQ_REQUIRE(plan == 0 || plan == 1 || plan == 128 || plan == 256, "plan: 0, 1, 128 or 256");
  g_force_plan = plan;
  return LCQ_OK;
}

extern "C" int lcq_fp8_gemm(const void* a, const void* a_s, const void* b, const void* b_s,
                            int64_t M, int64_t N, int64_t K, void* c, int c_dtype,
                            void* workspace, int64_t ws_bytes, void* stream) {
  LCQ_REQUIRE(a && a_s && b && b_s && c, "null pointer");
  LCQ_REQUIRE(M > 0 && N > 0 && K > 0, "empty GEMM");
  LCQ_REQUIRE(K % 128 == 0, "K must be a multiple of 128 (the scale block)");
  LCQ_REQUIRE(c_dtype == LCQ_F32 || c_dtype == LCQ_BF16 || c_dtype == LCQ_F16,
              "C dtype must be F32, BF16 or F16");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(b) & 15) == 0,
              "A / B must be 16-byte aligned");
  const int64_t nkb = K / BK;
  // the 16x16x128 body where the plan picks it (gemm2_plan), else the 32x32x64 kernel below
  const Plan2 pl = pick_plan(M, N, K);
  if (pl.tm != 0 && M > 64 && workspace && ws_bytes >= ws2_bytes(M, N, K) && N % 4 == 0 &&
      M * K < ((int64_t)1 << 31) && N * K < ((int64_t)1 << 31)) {
    hipStream_t st = as_stream(stream);
    const int64_t mp = (M + 255) / 256 * 256;
    const int64_t s2 = pl.splits;
    float* ast = static_cast<float*>(workspace);
    float* part = s2 > 1 ? ast + nkb * mp : nullptr;
    hipLaunchKernelGGL(k_as_transpose, dim3((unsigned)((nkb * mp + 255) / 256)), 256, 0, st,
                       static_cast<const float*>(a_s), M, nkb, mp, ast, nullptr);
    Gemm2Args g2{static_cast<const uint8_t*>(a), static_cast<const uint8_t*>(b), ast,
                 static_cast<const float*>(b_s), c, part, M, N, K, mp,
                 (nkb + s2 - 1) / s2, c_dtype, (int)((M + pl.tm - 1) / pl.tm),
                 (int)((N + pl.tm - 1) / pl.tm), nkb * mp, nullptr, 0, nullptr, nullptr};
    const int nslots = 32 * ((g2.nmt + 3) / 4) * ((g2.nnt + 7) / 8);
    // stage ring + the split's block-scales (TM / 128 column blocks x K blocks per split)
    const int bsb = (int)(((pl.tm / 128) * g2.kb_per_split * 4 + 15) / 16 * 16);
    if (pl.tm == 256) {
      const int L = NS256 * stage_bytes<256>() + bsb;
      LCQ_REQUIRE(L <= 160 * 1024, "K too large for the staged block-scales");
      (void)hipFuncSetAttribute((const void*)k_fp8_gemm2,
                                hipFuncAttributeMaxDynamicSharedMemorySize, L);
      hipLaunchKernelGGL(k_fp8_gemm2, dim3((unsigned)nslots, 1, (unsigned)s2), 512, L, st, g2);
    } else {
      const int L = NS128 * stage_bytes<128>() + bsb;
      LCQ_REQUIRE(L <= 160 * 1024, "K too large for the staged block-scales");
      (void)hipFuncSetAttribute((const void*)k_fp8_gemm2_128,
                                hipFuncAttributeMaxDynamicSharedMemorySize, L);
      hipLaunchKernelGGL(k_fp8_gemm2_128, dim3((unsigned)nslots, 1, (unsigned)s2), 256, L, st,
                         g2);
    }
    if (s2 > 1) {
      const int rc = check_launch("lcq_fp8_gemm");
      if (rc) return rc;
      const int64_t mn = M * N;
      int64_t blocks = (mn + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      k_fp8_gemm_reduce<<<(unsigned)blocks, 256, 0, st>>>(part, (int)s2, mn, c, c_dtype);
    }
    return check_launch("lcq_fp8_gemm");
  }
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

// grouped workspace: the kb-major a_s copy, tile0 [G + 1], tmap [slot bound]
static int64_t grouped_slot_bound(int64_t rows, int64_t G, int64_t N) {
  const int64_t nnt = (N + 255) / 256;
  return ((rows + 255) / 256 + G) * 8 * ((nnt + 7) / 8);
}

extern "C" int64_t lcq_fp8_gemm_grouped_workspace_bytes(int64_t rows, int64_t G, int64_t N,
                                                        int64_t K) {
  if (rows < 0 || G <= 0 || N <= 0 || K <= 0 || K % BK != 0) return 0;
  const int64_t mp = (rows + 255) / 256 * 256, nkb = K / BK;
  return nkb * mp * 4 + (G + 1) * 4 + grouped_slot_bound(rows, G, N) * 4 + 64;
}

extern "C" int lcq_fp8_gemm_grouped(const void* a, const void* a_s, int64_t a_rows_total,
                                    const int64_t* a_rows, int64_t rows,
                                    const int64_t* row_off, const int64_t* wtab, int64_t G,
                                    int nsets, int silu_mul, int64_t N, int64_t K, void* c,
                                    int c_dtype, void* workspace, int64_t ws_bytes,
                                    void* stream) {
  LCQ_REQUIRE(a && a_s && row_off && wtab && c && workspace, "null pointer");
  LCQ_REQUIRE(rows >= 0 && G > 0 && G <= (1 << 20) && N > 0 && K > 0, "bad grouped shape");
  LCQ_REQUIRE(nsets == 1 || nsets == 2, "nsets must be 1 or 2");
  LCQ_REQUIRE(!silu_mul || (nsets == 2 && c_dtype == LCQ_BF16),
              "silu_mul pairs two weight sets (gate, up) into a bf16 output");
  LCQ_REQUIRE(a_rows ? (a_rows_total >= 0 && a_rows_total * K < ((int64_t)1 << 31))
                     : a_rows_total == rows,
              "gathered A must be < 2 GiB; ungathered A has `rows` rows");
  LCQ_REQUIRE(K % BK == 0, "K must be a multiple of 128 (the scale block)");
  LCQ_REQUIRE(N % 4 == 0, "N must be a multiple of 4");
  LCQ_REQUIRE(256 * K < ((int64_t)1 << 31) && N * K < ((int64_t)1 << 31),
              "K / N too large for the 32-bit tile offsets");
  LCQ_REQUIRE(c_dtype == LCQ_F32 || c_dtype == LCQ_BF16 || c_dtype == LCQ_F16,
              "C dtype must be F32, BF16 or F16");
  LCQ_REQUIRE((reinterpret_cast<uintptr_t>(a) & 15) == 0, "A must be 16-byte aligned");
  // the pair mode's tiles are 128 output columns of two weights: the slot count of 2 N
  const int64_t NT = silu_mul ? 2 * N : N;
  LCQ_REQUIRE(ws_bytes >= lcq_fp8_gemm_grouped_workspace_bytes(rows, G, NT, K),
              "workspace too small");
  if (rows == 0) return LCQ_OK;
  hipStream_t st = as_stream(stream);
  const int64_t mp = (rows + 255) / 256 * 256, nkb = K / BK;
  float* ast = static_cast<float*>(workspace);
  int* tile0 = reinterpret_cast<int*>(ast + nkb * mp);
  int* tmap = tile0 + (G + 1);
  const int64_t bound = grouped_slot_bound(rows, G, NT);
  const int sets = silu_mul ? 1 : nsets;
  LCQ_REQUIRE(bound * sets < ((int64_t)1 << 30), "too many tiles");
  hipLaunchKernelGGL(k_as_transpose, dim3((unsigned)((nkb * mp + 255) / 256)), 256, 0, st,
                     static_cast<const float*>(a_s), rows, nkb, mp, ast, a_rows);
  const int nnt = (int)((NT + 255) / 256);
  hipLaunchKernelGGL(k_group_tiles, dim3((unsigned)G), 256, 0, st, row_off, (int)G, nnt, tile0,
                     tmap);
  GroupedArgs ga{static_cast<const uint8_t*>(a), ast, row_off, wtab, tile0, tmap, a_rows,
                 a_rows_total * K, c, N, K, mp, rows, (int)G, c_dtype, nnt, nsets, silu_mul};
  const int bsb = (int)((2 * nkb * 4 + 15) / 16 * 16);
  const int L = NS256 * stage_bytes<256>() + bsb;
  LCQ_REQUIRE(L <= 160 * 1024, "K too large for the staged block-scales");
  // the slot bound rounded to 8 XCD lanes (the kernel's q never exceeds bound / 8 rounded up)
  const int64_t grid = (bound * sets + 7) / 8 * 8;
  if (silu_mul) {
    (void)hipFuncSetAttribute((const void*)k_fp8_gemm2_grouped_silu,
                              hipFuncAttributeMaxDynamicSharedMemorySize, L);
    hipLaunchKernelGGL(k_fp8_gemm2_grouped_silu, dim3((unsigned)grid), 512, L, st, ga);
  } else {
    (void)hipFuncSetAttribute((const void*)k_fp8_gemm2_grouped,
                              hipFuncAttributeMaxDynamicSharedMemorySize, L);
    hipLaunchKernelGGL(k_fp8_gemm2_grouped, dim3((unsigned)grid), 512, L, st, ga);
  }
  return check_launch("lcq_fp8_gemm_grouped");
}
