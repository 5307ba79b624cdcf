// GPTQ Hessian H <- beta*H + alpha * X^T X on gfx950 bf16/fp16 MFMA, read from the token-major
// activations as the forward hook hands them over (no transposed copy).
//
// Reference: GPTQ.add_batch (llmc/compression/quantization/gptq.py:253-295):
//   H *= n/(n+b); n += b; x = sqrt(2/n) * x.float(); H += x @ x.T   (full fp32 GEMM)
// Here: one MFMA pass over the upper-triangle 256x256 tiles only (half the reference's flops),
// exact bf16 products accumulated in fp32, epilogue beta*H + alpha*acc, mirrored.
//
// Structure (k_syrk_x): one 256-thread workgroup (2 x 2 waves of 128 x 128, 8 x 8
// mfma_f32_16x16x32 accumulators each, in AGPRs) per upper tile (ti, tj). The contraction runs
// over tokens in K-tiles of 64: the A operand is X[t0 : t0+64, 256 ti : 256 ti + 256] and B the
// same rows at columns 256 tj -- rows of X are channel-contiguous, so both are staged with
// coalesced 64-byte row segments by buffer-descriptor LDS-DMA, and the MFMA's k-contiguous
// fragments (8 consecutive tokens of one channel per lane) come out of LDS through the gfx950
// transposed read ds_read_b64_tr_b16 (cdna_hip_programming.md T10): two reads of 4 tokens x 16
// channels per fragment.
//
// LDS image of one operand K-tile (64 tokens x 256 channels, 32 KB): 32 pieces of 1 KB, piece
// (cb, tg) = channels 32 cb .. 32 cb + 31 of tokens 16 tg .. 16 tg + 15 at (4 cb + tg) KB, row r
// (token) at r * 64 B, 16-B chunk c (8 channels) at physical chunk c ^ (2 ((r >> 3) & 1)). A
// transposed fragment read then covers 8 token rows x 2 chunks per 32-lane half on 16 distinct
// 16-B bank slots: conflict-free. Piece (cb, *) holds the 32 channels that MFMA block cb & 3 of
// wave row cb >> 2 consumes, so the per-block release / reload schedule of the projection
// GEMM (gemm256.hip k_gemm16b: 4 barriers per K-tile, counted vmcnt, B fragments double
// buffered in registers, loads two K-tiles ahead) carries over unchanged.
//
// Tokens past the last whole K-tile come from a zero-padded 64-row tail copy in the
// workspace; channels past ic are clamped reads whose outputs are discarded. Split-K over `ns`
// token slabs (count from a round-filling cost model, plan()) goes to fp32 partials in the
// workspace, combined in a fixed order by k_syrk_reduce (deterministic: no float atomics).
#include "lcq_common.h"


namespace lcq {
namespace hx {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int ST = 256;                // output tile
constexpr int SKT = 64;                // K-tile (tokens)
constexpr int TILE_B = SKT * ST * 2;   // one operand K-tile image: 32 KB
constexpr int BUF = 2 * TILE_B;        // A + B

struct Args {
  const uint16_t* x;     // [n, ld] token-major
  const uint16_t* tail;  // [64, ld] zero-padded copy of the last partial K-tile (or null)
  int64_t ld, ic, icp;
  int64_t nk_main, nk;   // whole K-tiles read from x; all K-tiles (nk_main + tail)
  float* H;
  float* part;           // split partials, upper tiles packed: [ns][ntiles][256 * 256], or null
  float alpha, beta;
  int nt, ns, ntiles;
  int64_t ktps;          // K-tiles per split
};

// Token groups of one launch (the grouped GPTQ Hessian, gptq_core.HessianAccumulator): group g
// holds tokens [row0[g], row0[g] + 64 nk_main[g]) of x plus an optional zero-padded tail
// K-tile, split into splits split0[g] .. split0[g + 1] - 1 of ktps[g] K-tiles each. Every
// split writes its own partial; k_syrk_reduce folds each group's splits in order, then sums
// the groups in the fixed pairwise tree. ng = 1 describes a plain (ungrouped) launch.
constexpr int GMAX = 8;
struct GArgs {
  int64_t row0[GMAX], nk_main[GMAX], nk[GMAX], ktps[GMAX];
  const uint16_t* tail[GMAX];
  int split0[GMAX + 1];
  int ng;
};

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

// v-th upper-triangle tile in chunks of 4 x 8 tiles walked band by band (4 tile rows per band):
// one XCD's 32 concurrent workgroups share 12 operand panels in its L2. The grid is exactly
// ntiles x ns workgroups (valid tiles only), so every XCD's contiguous wgid range holds the
// same number of live tiles (+-1).
__device__ __forceinline__ void valid_tile(int v, int nt, int& ti, int& tj) {
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  // readfirstlane the base so the descriptor is provably wave-uniform (no waterfall loop)
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, 0x7fffffff, 0x00020000);
}

// token rows of K-tile kt (absolute): from x, or from the zero-padded tail copy
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ktile_rsrc(const Args& a, int64_t kt) {
  const uint16_t* p = kt < a.nk_main ? a.x + kt * SKT * a.ld : a.tail;
  return rsrc_of(p);
}

// per-lane byte offsets of the 16 pieces a wave stages per K-tile: B pieces cb = 0..7 and A
// pieces cb = 0..7, all of token group tg = wave (16 tokens); lane -> (row lane >> 2, physical
// chunk lane & 3) of the piece, loading logical chunk (lane & 3) ^ (2 ((row >> 3) & 1))
struct Stage {
  uint32_t aoff[8], boff[8];
};

__device__ __forceinline__ void make_stage(const Args& a, int ti, int tj, int w, int lane,
                                           Stage& st) {
  const int r = lane >> 2;
  const int c = (lane & 3) ^ (((r >> 3) & 1) << 1);
  const int64_t trow = (int64_t)w * 16 + r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int64_t ca = (int64_t)ti * ST + j * 32 + c * 8, cb = (int64_t)tj * ST + j * 32 + c * 8;
    if (ca > a.ic - 8) ca = a.ic - 8;  // past ic: a valid address, the outputs are dropped
    if (cb > a.ic - 8) cb = a.ic - 8;
    st.aoff[j] = (uint32_t)((trow * a.ld + ca) * 2);
    st.boff[j] = (uint32_t)((trow * a.ld + cb) * 2);
  }
}

// Load order of one K-tile's 16 pieces per wave (the vmcnt counts of ktile() depend on it):
//   block 0: B pieces 0..7, A pieces 0 and 4 | block 1: A 1, 5 | block 2: A 2, 6 | block 3: A 3, 7
// (A piece cb holds the 32 channels of MFMA block cb & 3 of wave row cb >> 2.)
__device__ __forceinline__ void load_piece(const Stage& st, __amdgpu_buffer_rsrc_t rs, char* lds,
                                           int buf, int w, int idx) {
  char* d = lds + buf * BUF;
  if (idx < 8) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(d + TILE_B + (idx * 4 + w) * 1024),
                                             16, st.boff[idx], 0, 0, 0);
  } else {
    const int q = idx - 8;  // 0..7 -> A piece 0,4,1,5,2,6,3,7
    const int j = (q >> 1) + 4 * (q & 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(d + (j * 4 + w) * 1024), 16,
                                             st.aoff[j], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
}

// The transposed reads are issued as inline asm: with the builtin, the waitcnt pass cannot
// tell them apart from the in-flight LDS-DMA stores and drains vmcnt(0) before each one (the
// whole load pipeline, 14 drains per K-tile pair measured in the ISA). As asm their completion
// is ours to wait for: every block starts with lgkmcnt(0) (block_wait below), and a fragment
// is always read at least one block before the MFMA that consumes it; the data they read is
// ordered by the counted vmcnt barriers, as for the projection GEMM.
template <int OFF>
__device__ __forceinline__ v4s tr_read(uint32_t addr) {
  v4s v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

__device__ __forceinline__ void block_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Per-lane part of a fragment read: MFMA 16x16x32 operand lane l = channel row l & 15, tokens
// 8 (l >> 4) .. +7. Lane 4q + p of 16-lane group g supplies token row 8 (g & 1) + 4 h + q of
// token group 2 kb + (g >> 1), channels 4p .. 4p + 3 of the fragment's 16 (rb & 1 selects the
// upper 16 of the piece's 32); the XOR term depends on (rb & 1) ^ (g & 1).
__device__ __forceinline__ uint32_t frag_lane_off(int lane, int rbodd, int h) {
  const int g = lane >> 4, l16 = lane & 15, q = l16 >> 2, p = l16 & 3;
  const int r = 8 * (g & 1) + 4 * h + q;
  const int pc = ((rbodd ^ (g & 1)) << 1) + (p >> 1);
  return (uint32_t)((g >> 1) * 1024 + r * 64 + pc * 16 + (p & 1) * 8);
}

// LDS byte addresses of this lane's fragment reads: [operand A / B][parity of the 16-channel
// row block], for the wave's 128-channel half (wave row wr for A, wave column wc for B) of
// buffer 0, h = 0 (h = 1 is 4 token rows = 256 B further)
struct FragOff {
  uint32_t o[2][2][2];  // [buffer][A / B][parity]: offsets within a buffer fit 16 bits
};

// fragment X (16 channels, X = 0..7 within the wave's 128) x k block KB (32 tokens) of the
// operand image at byte TILE of a buffer: everything but the lane base in the offset field
template <int TILE, int X, int KB>
__device__ __forceinline__ v8s read_frag(const uint32_t (&base)[2]) {
  constexpr int off = TILE + ((X >> 1) * 4 + KB * 2) * 1024;
  const v4s lo = tr_read<off>(base[X & 1]);
  const v4s hi = tr_read<off + 256>(base[X & 1]);
  return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int TILE>
__device__ __forceinline__ v8s frag_at(const FragOff& fo, int op, int x, int kb) {
  const uint32_t (&base)[2] = fo.o[TILE / BUF][op];
  constexpr int T = TILE % BUF;
  // x, kb are constants after unrolling: the switch folds to one read pair
  switch (x * 2 + kb) {
    case 0: return read_frag<T, 0, 0>(base);
    case 1: return read_frag<T, 0, 1>(base);
    case 2: return read_frag<T, 1, 0>(base);
    case 3: return read_frag<T, 1, 1>(base);
    case 4: return read_frag<T, 2, 0>(base);
    case 5: return read_frag<T, 2, 1>(base);
    case 6: return read_frag<T, 3, 0>(base);
    case 7: return read_frag<T, 3, 1>(base);
    case 8: return read_frag<T, 4, 0>(base);
    case 9: return read_frag<T, 4, 1>(base);
    case 10: return read_frag<T, 5, 0>(base);
    case 11: return read_frag<T, 5, 1>(base);
    case 12: return read_frag<T, 6, 0>(base);
    case 13: return read_frag<T, 6, 1>(base);
    case 14: return read_frag<T, 7, 0>(base);
    default: return read_frag<T, 7, 1>(base);
  }
}

template <bool FP16>
__device__ __forceinline__ void mfma16a(v4f& acc, v8s bfrag, v8s afrag) {
  if constexpr (FP16)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfrag), "v"(afrag));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(bfrag), "v"(afrag));
}

// One K-tile t (split-relative; kt0 + t absolute) in four blocks of 32 MFMAs, one barrier per
// block: block mb works on A channel rows 2 mb, 2 mb + 1 (16-row fragments) of the wave row.
// Block 0 issues the B pieces and A pieces 0 / 4 of K-tile t + 2 into the buffer being read
// (its B fragments and block-0 A fragments were read before the barrier), blocks 1..3 the A
// pieces of their rows. A fragments are read one block ahead; the B fragments of K-tile t + 1
// are read during blocks 1 and 2 into the other register set (P = t & 1).
template <bool FP16, int P>
__device__ __forceinline__ void ktile(v4f (&acc)[8][8], v8s (&bf)[2][8][2], v8s (&af)[2][2][2],
                                      const Stage& st, const FragOff& fo, const Args& a,
                                      char* lds, int64_t kt0, int64_t t, int64_t nk, int w,
                                      int wr, int wc) {
  constexpr int cur = P;  // t & 1: the caller runs even K-tiles with P = 0, odd with P = 1
  constexpr int At = cur * BUF;
  constexpr int An = (cur ^ 1) * BUF;
  constexpr int Bn = An + TILE_B;
  (void)wr;
  (void)wc;
  const int64_t t2 = t + 2 < nk ? t + 2 : nk - 1;
  const __amdgpu_buffer_rsrc_t rs = ktile_rsrc(a, kt0 + t2);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
#pragma unroll
      for (int n = 0; n < 8; ++n) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int i = mm * 16 + n * 2 + kb;
          if (i == 0) block_wait();  // the fragments read during the previous block
          mfma16a<FP16>(acc[2 * mb + mm][n], bf[P][n][kb], af[mb & 1][mm][kb]);
          if (i == 7) {
            if (mb == 1) wait_barrier<18>();
            else wait_barrier<20>();
          }
          if (mb == 0 && i >= 8 && i < 28 && (i & 1) == 0) load_piece(st, rs, lds, cur, w, (i - 8) >> 1);
          if (mb > 0 && (i == 8 || i == 20)) load_piece(st, rs, lds, cur, w, 8 + 2 * mb + (i == 20));
          if (i >= 8 && i < 12) {
            const int q = i - 8, m2 = q >> 1, k2 = q & 1;
            if (mb < 3) af[(mb + 1) & 1][m2][k2] = frag_at<At>(fo, 0, 2 * (mb + 1) + m2, k2);
            else af[0][m2][k2] = frag_at<An>(fo, 0, m2, k2);  // K-tile t+1, block 0
          }
          if ((mb == 1 || mb == 2) && i >= 12 && i < 20) {  // B fragments of K-tile t+1
            const int f = (mb - 1) * 8 + (i - 12), nn = f >> 1, k3 = f & 1;
            bf[P ^ 1][nn][k3] = frag_at<Bn>(fo, 1, nn, k3);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }
}

// The three-barrier K-tile of the projection GEMM's k_gemm16h (gemm256.hip), on this kernel's
// token-major image: fragments double-buffered by k half (X0 = tokens 0-31 of the K-tile,
// X1 = tokens 32-63), K-tile t + 2 loaded into K-tile t's buffer -- its A pieces after barrier 1,
// its B pieces after barrier 2 -- and one counted vmcnt per K-tile (barrier 3: K-tile t + 1
// landed, its X0 is read during the last 32 MFMAs). The transposed reads are asm: their
// completion is waited for explicitly (barriers 1 and 2 for X1, the end of the K-tile for X0).
// Same k order per accumulator as ktile(): identical sums, so the host picks either per launch
// (profiles/r5_hessian_schedule_ab.txt: faster for the per-input accumulation at every IC and
// for the grouped launch at IC 4096, 5 % slower for the grouped launch at IC 14336).
template <bool FP16, int P>
__device__ __forceinline__ void ktile3(v4f (&acc)[8][8], v8s (&x0a)[8], v8s (&x0b)[8],
                                       v8s (&x1a)[8], v8s (&x1b)[8], const Stage& st,
                                       const FragOff& fo, const Args& a, char* lds, int64_t kt0,
                                       int64_t t, int64_t nk, int w) {
  constexpr int cur = P;  // t & 1
  constexpr int At = cur * BUF;
  constexpr int An = (cur ^ 1) * BUF;
  const int64_t t2 = t + 2 < nk ? t + 2 : nk - 1;
  const __amdgpu_buffer_rsrc_t rs = ktile_rsrc(a, kt0 + t2);
  char* d = lds + cur * BUF;
  auto load_a = [&](int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(d + (j * 4 + w) * 1024), 16,
                                             st.aoff[j], 0, 0, 0);
  };
  auto load_b = [&](int j) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(d + TILE_B + (j * 4 + w) * 1024),
                                             16, st.boff[j], 0, 0, 0);
  };
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const int i = h * 64 + m * 8 + n;
    if (h == 0) mfma16a<FP16>(acc[m][n], x0b[n], x0a[m]);
    else mfma16a<FP16>(acc[m][n], x1b[n], x1a[m]);
    if (i < 16 && (i & 1) == 0) x1a[i >> 1] = frag_at<At>(fo, 0, i >> 1, 1);
    if (i == 20) {                     // X1.A landed; every wave is past t's A
      block_wait();
      __builtin_amdgcn_s_barrier();
    }
    if (i >= 22 && i <= 34 && (i - 22) % 3 == 0) load_a((i - 22) / 3);
    if (i == 24 || i == 27 || i == 30 || i == 33 || i == 36 || i == 38 || i == 40 || i == 42) {
      const int f = i <= 36 ? (i - 24) / 3 : 5 + (i - 38) / 2;
      x1b[f] = frag_at<At + TILE_B>(fo, 1, f, 1);
    }
    if (i == 50) {                     // X1.B landed; every wave is past t's B
      block_wait();
      __builtin_amdgcn_s_barrier();
    }
    if (i == 52 || i == 55 || i == 58) load_a(5 + (i - 52) / 3);
    if (i == 61 || i == 64) load_b((i - 61) / 3);
    if (i == 85 || i == 87 || i == 89) load_b(2 + (i - 85) / 2);
    if (i == 91) {
      asm volatile("s_waitcnt vmcnt(13)" ::: "memory");   // K-tile t + 1 landed
      __builtin_amdgcn_s_barrier();
    }
    if (i >= 93 && i <= 100) x0a[i - 93] = frag_at<An>(fo, 0, i - 93, 0);
    if (i >= 101 && i <= 115 && ((i - 101) & 1) == 0)
      x0b[(i - 101) >> 1] = frag_at<An + TILE_B>(fo, 1, (i - 101) >> 1, 0);
    if (i == 96 || i == 100) load_b(5 + (i - 96) / 4);
    if (i == 124) load_b(7);
    if (i == 127) block_wait();        // X0 of K-tile t + 1 landed
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool FP16, bool S3>
__global__ void __launch_bounds__(256, 1) k_syrk_x(Args a, GArgs ga) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  // Splits run one after another in launch order, each spread over all 8 XCDs: XCD x (bid & 7)
  // takes the contiguous valid-tile range [x q, x q + q) of every split (q = ceil(ntiles / 8)),
  // so the 8 XCDs stream the SAME token slab at a time (its panels shared through the MALL)
  // while each XCD's 32 CUs share 12 operand panels in its L2 (valid_tile chunks).
  const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
  const int q = (a.ntiles + 7) >> 3;
  const int split = j / q;
  const int v = xcd * q + (j - split * q);
  if (v >= a.ntiles || split >= a.ns) return;   // padding workgroups: before any barrier
  int ti, tj;
  valid_tile(v, a.nt, ti, tj);
  // this split's token group: its rows of x, tail and K-tile range
  int g = 0;
  while (g + 1 < ga.ng && split >= ga.split0[g + 1]) ++g;
  a.x += ga.row0[g] * a.ld;
  a.tail = ga.tail[g];
  a.nk_main = ga.nk_main[g];
  a.nk = ga.nk[g];
  a.ktps = ga.ktps[g];
  const int64_t kt0 = (int64_t)(split - ga.split0[g]) * a.ktps;
  int64_t nk = a.nk - kt0;
  if (nk > a.ktps) nk = a.ktps;
  Stage st;
  make_stage(a, ti, tj, w, lane, st);
  FragOff fo;
  {
    const uint32_t l0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        fo.o[b][0][par] = l0 + b * BUF + wr * 16384 + frag_lane_off(lane, par, 0);  // A: 128 wr..
        fo.o[b][1][par] = l0 + b * BUF + wc * 16384 + frag_lane_off(lane, par, 0);  // B: 128 wc..
      }
  }

  v4f acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = v4f{0.f, 0.f, 0.f, 0.f};
  {
    const __amdgpu_buffer_rsrc_t r0 = ktile_rsrc(a, kt0);
    const __amdgpu_buffer_rsrc_t r1 = ktile_rsrc(a, kt0 + (nk > 1 ? 1 : 0));
#pragma unroll
    for (int i = 0; i < 16; ++i) load_piece(st, r0, lds, 0, w, i);
#pragma unroll
    for (int i = 0; i < 16; ++i) load_piece(st, r1, lds, 1, w, i);
  }
  if constexpr (S3) {
    wait_barrier<16>();  // K-tile 0 landed (K-tile 1's 16 pieces may be in flight)
    v8s x0a[8], x0b[8], x1a[8], x1b[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) x0a[m] = frag_at<0>(fo, 0, m, 0);
#pragma unroll
    for (int n = 0; n < 8; ++n) x0b[n] = frag_at<TILE_B>(fo, 1, n, 0);
    block_wait();
    asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC
    int64_t t = 0;
    for (; t + 1 < nk; t += 2) {
      ktile3<FP16, 0>(acc, x0a, x0b, x1a, x1b, st, fo, a, lds, kt0, t, nk, w);
      ktile3<FP16, 1>(acc, x0a, x0b, x1a, x1b, st, fo, a, lds, kt0, t + 1, nk, w);
    }
    if (t < nk) ktile3<FP16, 0>(acc, x0a, x0b, x1a, x1b, st, fo, a, lds, kt0, t, nk, w);
  } else {
  v8s af[2][2][2], bf[2][8][2];
  wait_barrier<22>();
#pragma unroll
  for (int n = 0; n < 8; ++n)
#pragma unroll
    for (int k = 0; k < 2; ++k) bf[0][n][k] = frag_at<TILE_B>(fo, 1, n, k);
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int k = 0; k < 2; ++k) af[0][m2][k] = frag_at<0>(fo, 0, m2, k);
  asm volatile("s_nop 4" ::: "memory");  // accumulator init (VALU) -> first MFMA srcC

  int64_t t = 0;
  for (; t + 1 < nk; t += 2) {
    ktile<FP16, 0>(acc, bf, af, st, fo, a, lds, kt0, t, nk, w, wr, wc);
    ktile<FP16, 1>(acc, bf, af, st, fo, a, lds, kt0, t + 1, nk, w, wr, wc);
  }
  if (t < nk) ktile<FP16, 0>(acc, bf, af, st, fo, a, lds, kt0, t, nk, w, wr, wc);
  }
  // drain, and cover the last MFMA's result latency before the accumulators are read (the asm
  // MFMA is opaque to the hazard recognizer: 16x16x32 = 8 passes -> 4 * 8 + 2 wait states)
  // The nops carry the last block's accumulators as operands: an epilogue read of them cannot
  // be scheduled above the wait (the asm MFMAs are opaque to the hazard recognizer; the earlier
  // blocks' results are >= 16 MFMAs old by now)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 7"
               : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                 "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7])
               :
               : "memory");

  // acc[m][n][jj] (swapped layout): H row i = ti*256 + wr*128 + m*16 + fr, columns
  // tj*256 + wc*128 + n*16 + fq*4 + jj. 32-bit element offsets (ic, icp <= 46336: checked
  // on the host) keep the 64-bit address math out of the unrolled epilogue.
  const int fr = lane & 15, fq = lane >> 4;
  const int i0 = ti * ST + wr * 128 + fr;
  const int j0 = tj * ST + wc * 128 + fq * 4;
  const int ic = (int)a.ic, icp = (int)a.icp;
  if (a.part != nullptr) {  // the split's partial tile, packed (tile-contiguous 256 KB)
    const int tri = ti * a.nt - ti * (ti - 1) / 2 + (tj - ti);
    float* Pp = a.part + ((int64_t)split * a.ntiles + tri) * (ST * ST);
    const int li = wr * 128 + fr, lj = wc * 128 + fq * 4;
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n)
        *reinterpret_cast<float4*>(Pp + (uint32_t)((li + m * 16) * ST + lj + n * 16)) =
            make_float4(acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]);
    return;
  }
  const bool diag = ti == tj;
  const bool vec = (ic & 3) == 0;
  float* H = a.H;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int i = i0 + m * 16;
    if (i >= ic) break;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const int j = j0 + n * 16;
      if (j >= ic) break;
      const uint32_t e = (uint32_t)(i * ic + j);
      float o[4];
      const bool full = vec && j + 3 < ic;
      float h[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.beta != 0.f) {
        if (full) {
          const float4 hv = *reinterpret_cast<const float4*>(H + e);
          h[0] = hv.x; h[1] = hv.y; h[2] = hv.z; h[3] = hv.w;
        } else {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (j + jj < ic) h[jj] = H[e + jj];
        }
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        float v = __fmul_rn(a.alpha, acc[m][n][jj]);
        if (a.beta != 0.f) v = __fadd_rn(__fmul_rn(a.beta, h[jj]), v);
        o[jj] = v;
      }
      if (full) {
        *reinterpret_cast<float4*>(H + e) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (j + jj < ic) H[e + jj] = o[jj];
      }
      if (!diag) {  // mirror H[j + jj][i]
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          if (j + jj < ic) H[(uint32_t)((j + jj) * ic + i)] = o[jj];
      }
    }
  }
}

// the last partial K-tile's tokens, zero padded to 64 rows (same row stride as x)
__global__ void __launch_bounds__(256) k_tail_copy(const uint16_t* __restrict__ x,
                                                  int64_t row0, int64_t n, int64_t ld,
                                                  uint16_t* __restrict__ tail) {
  const int64_t total = SKT * ld / 8;  // 16-B chunks (ld % 8 == 0)
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / (ld / 8);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (row0 + r < n) v = reinterpret_cast<const uint4*>(x + (row0 + r) * ld)[e - r * (ld / 8)];
    reinterpret_cast<uint4*>(tail)[e] = v;
  }
}

// split combine: per group the fold of its splits in order (the first partial, + the next,
// ...), the groups in the fixed pairwise tree ((g0 + g1) + (g2 + g3)) + ((g4 + g5) + (g6 + g7))
// (ng = 1, 2, 4, 8; a group without tokens counts 0), then H = beta*H + alpha * sum, upper tiles
// + mirror. A workgroup = one 64 x 64 piece of an upper tile: the row-major store and the
// mirrored store both go out coalesced (the mirror through an LDS transpose)
__global__ void __launch_bounds__(256) k_syrk_reduce(Args a, GArgs ga) {
  __shared__ float tp[64][65];
  int ti, tj;
  tri_tile(blockIdx.x, a.nt, ti, tj);
  const bool diag = ti == tj;
  const int pr = blockIdx.y >> 2, pc = blockIdx.y & 3;  // 4 x 4 pieces of the 256^2 tile
  const int64_t r0 = (int64_t)ti * ST + pr * 64, c0 = (int64_t)tj * ST + pc * 64;
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int64_t tstride = (int64_t)a.ntiles * (ST * ST);
  const float* tbase = a.part + (int64_t)blockIdx.x * (ST * ST);
  for (int rr = ry; rr < 64; rr += 4) {
    const int64_t r = r0 + rr, c = c0 + cx;
    float v = 0.f;
    if (r < a.ic && c < a.ic) {
      const int64_t e = (int64_t)(pr * 64 + rr) * ST + pc * 64 + cx;
      float gs[GMAX];
#pragma unroll
      for (int g = 0; g < GMAX; ++g) {
        gs[g] = 0.f;
        if (g < ga.ng) {
          const int s0 = ga.split0[g], s1 = ga.split0[g + 1];
          if (s1 > s0) {
            float s = tbase[s0 * tstride + e];
            for (int k = s0 + 1; k < s1; ++k) s = __fadd_rn(s, tbase[k * tstride + e]);
            gs[g] = s;
          }
        }
      }
#pragma unroll
      for (int wdt = 1; wdt < GMAX; wdt *= 2)
#pragma unroll
        for (int g = 0; g < GMAX; g += 2 * wdt)
          if (g + wdt < ga.ng) gs[g] = __fadd_rn(gs[g], gs[g + wdt]);
      v = a.alpha != 1.0f ? __fmul_rn(a.alpha, gs[0]) : gs[0];
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

// Split-K count. The grid is ntiles x ns workgroups, one per CU (128 KB LDS), in contiguous
// wgid ranges per XCD (8 XCDs x 32 CUs), so a launch takes rounds =
// ceil(ceil(ntiles * ns / 8) / 32) waves of workgroups, each ~(ktps + 6) K-tile times long
// (6 ~ prologue + the 256 KB fp32 tile store); every split adds a 256 KB partial tile written
// and re-read by k_syrk_reduce (~0.034 K-tile times at HBM rate). Pick the ns with the least
// modelled time (n = 262144: ic 4096 -> 15, ic 8192 -> 8, ic 14336 -> 4). At least 8 K-tiles
// per split; partial slabs capped at 8 GiB. A probe build (-DLCQ_PROBE_SYRK_NS=<n>, see
// scripts/probe_build.py) forces a count; the product library has no run-time override.
#ifndef LCQ_PROBE_SYRK_NS
#define LCQ_PROBE_SYRK_NS 0
#endif
static constexpr int forced_ns() { return LCQ_PROBE_SYRK_NS; }

static void plan(int64_t n, int64_t ic, int& nt, int& ntiles, int& ns, int64_t& ktps,
                 int64_t& nkt, int64_t& icp) {
  icp = ceil_to(ic, ST);
  nkt = ceil_to(n, SKT) / SKT;
  nt = (int)(icp / ST);
  ntiles = nt * (nt + 1) / 2;
  int64_t best_ns = 1;
  if (forced_ns() > 0) {
    best_ns = forced_ns();
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

}  // namespace hx
}  // namespace lcq

using namespace lcq;
using namespace lcq::hx;

// Per-group split count of the grouped launch: the same cost model with the grid taken as
// GMAX groups launched together. It depends only on (group tokens, ic) -- never on how many
// groups this process launches -- so a token-sharded rank splits its groups exactly as one GPU
// does (the fp32 fold order per group is world-independent). The split count changes the fp32
// fold order, so it is never a run-time knob: only a probe build (-DLCQ_PROBE_SYRK_GNS=<n>,
// scripts/probe_build.py) forces it.
#ifndef LCQ_PROBE_SYRK_GNS
#define LCQ_PROBE_SYRK_GNS 0
#endif
static constexpr int forced_gns() { return LCQ_PROBE_SYRK_GNS; }

static void plan_group(int64_t n, int64_t ic, int64_t& ns, int64_t& ktps, int64_t& nkt) {
  const int64_t icp = ceil_to(ic, ST);
  const int64_t nt = icp / ST, ntiles = nt * (nt + 1) / 2;
  nkt = ceil_to(n, SKT) / SKT;
  int64_t best_ns = 1;
  double best = 1e300;
  for (int64_t c = 1; c <= 64 && forced_gns() <= 0; ++c) {
    if (c > 1 && nkt / c < 8) break;
    const int64_t per = (nkt + c - 1) / c, cc = (nkt + per - 1) / per;
    const int64_t per_xcd = (ntiles * cc * GMAX + 7) / 8, rounds = (per_xcd + 31) / 32;
    const double cost = (double)rounds * (double)(per + 6) + 0.034 * (double)(cc * ntiles * GMAX);
    if (cost < best * 0.995) {
      best = cost;
      best_ns = cc;
    }
  }
  if (forced_gns() > 0) best_ns = forced_gns() < nkt ? forced_gns() : nkt;
  ktps = (nkt + best_ns - 1) / best_ns;
  ns = nkt ? (nkt + ktps - 1) / ktps : 0;
}

struct GroupedPlan {
  GArgs ga;
  int64_t splits, tail_bytes, part_bytes;
};

static int grouped_plan(const int64_t* bounds, int ng, int64_t ic, GroupedPlan& p) {
  p = GroupedPlan{};
  const int64_t icp = ceil_to(ic, ST), nt = icp / ST, ntiles = nt * (nt + 1) / 2;
  p.ga.ng = ng;
  int64_t sp = 0;
  for (int g = 0; g < ng; ++g) {
    const int64_t n = bounds[g + 1] - bounds[g];
    if (n < 0) return -1;
    int64_t ns = 0, ktps = 1, nkt = 0;
    if (n > 0) plan_group(n, ic, ns, ktps, nkt);
    p.ga.row0[g] = bounds[g];
    p.ga.nk_main[g] = n / SKT;
    p.ga.nk[g] = nkt;
    p.ga.ktps[g] = ktps;
    p.ga.split0[g] = (int)sp;
    if (n % SKT) p.tail_bytes += ceil_to(SKT * ic * 2, 256);
    sp += ns;
  }
  p.ga.split0[ng] = (int)sp;
  p.splits = sp;
  p.part_bytes = sp * ntiles * ST * ST * 4;
  return 0;
}

extern "C" int64_t lcq_hessian_workspace_bytes(int64_t n, int64_t ic) {
  if (n <= 0 || ic <= 0) return 0;
  int nt, ntiles, ns;
  int64_t ktps, nkt, icp;
  plan(n, ic, nt, ntiles, ns, ktps, nkt, icp);
  int64_t b = (n % SKT) ? SKT * ceil_to(ic, 8) * 2 : 0;  // tail copy
  b = ceil_to(b, 256);
  if (ns > 1) b += (int64_t)ns * ntiles * ST * ST * 4;
  return b;
}

extern "C" int lcq_hessian_accum(const void* x, int x_dtype, int64_t n, int64_t ic, void* H,
                                 float alpha, float beta, void* workspace, int64_t ws_bytes,
                                 void* stream) {
  LCQ_REQUIRE(x_dtype == LCQ_BF16 || x_dtype == LCQ_F16, "x must be bf16 or fp16");
  LCQ_REQUIRE(n > 0 && ic > 0, "empty input");
  LCQ_REQUIRE(ic % 8 == 0, "ic must be a multiple of 8 (16-byte token rows)");
  LCQ_REQUIRE(ic <= 46336, "ic must be <= 46336 (32-bit H offsets)");
  LCQ_REQUIRE(x != nullptr && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
              "x must be 16-byte aligned");
  const int64_t need = lcq_hessian_workspace_bytes(n, ic);
  LCQ_REQUIRE(need == 0 || (workspace != nullptr && ws_bytes >= need),
              "workspace smaller than lcq_hessian_workspace_bytes(n, ic)");
  Args a{};
  int64_t nkt;
  plan(n, ic, a.nt, a.ntiles, a.ns, a.ktps, nkt, a.icp);
  hipStream_t st = as_stream(stream);
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.ld = ic;
  a.ic = ic;
  a.nk_main = n / SKT;
  a.nk = nkt;
  char* ws = reinterpret_cast<char*>(workspace);
  int64_t off = 0;
  if (n % SKT) {
    uint16_t* tail = reinterpret_cast<uint16_t*>(ws);
    hipLaunchKernelGGL(k_tail_copy, dim3((unsigned)((SKT * ic / 8 + 255) / 256)), 256, 0, st,
                       a.x, a.nk_main * SKT, n, ic, tail);
    int rc = check_launch("lcq_hessian_accum: tail");
    if (rc) return rc;
    a.tail = tail;
    off = ceil_to(SKT * ic * 2, 256);
  }
  a.H = reinterpret_cast<float*>(H);
  a.part = a.ns > 1 ? reinterpret_cast<float*>(ws + off) : nullptr;
  a.alpha = alpha;
  a.beta = beta;
  GArgs ga{};
  ga.ng = 1;
  ga.row0[0] = 0;
  ga.nk_main[0] = a.nk_main;
  ga.nk[0] = a.nk;
  ga.ktps[0] = a.ktps;
  ga.tail[0] = a.tail;
  ga.split0[0] = 0;
  ga.split0[1] = a.ns;
  // ktile3: the faster schedule for this launch at every IC measured
  auto k = x_dtype == LCQ_F16 ? k_syrk_x<true, true> : k_syrk_x<false, true>;
  // the dynamic-LDS attribute is per device: set it on every launch (cheap, thread-safe)
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF);
  hipLaunchKernelGGL(k, dim3((unsigned)(8 * ((a.ntiles + 7) / 8) * a.ns)), 256, 2 * BUF, st, a,
                     ga);
  int rc = check_launch("lcq_hessian_accum: syrk");
  if (rc) return rc;
  if (a.ns > 1) {
    hipLaunchKernelGGL(k_syrk_reduce, dim3((unsigned)a.ntiles, 16), 256, 0, st, a, ga);
    rc = check_launch("lcq_hessian_accum: reduce");
  }
  return rc;
}

extern "C" int64_t lcq_hessian_grouped_workspace_bytes(const int64_t* bounds, int ng,
                                                       int64_t ic) {
  if (bounds == nullptr || ng < 1 || ng > GMAX || ic <= 0) return 0;
  GroupedPlan p;
  if (grouped_plan(bounds, ng, ic, p)) return 0;
  return p.tail_bytes + p.part_bytes;
}

extern "C" int lcq_hessian_grouped(const void* x, int x_dtype, int64_t ic,
                                   const int64_t* bounds, int ng, void* H, float alpha,
                                   void* workspace, int64_t ws_bytes, void* stream) {
  LCQ_REQUIRE(x_dtype == LCQ_BF16 || x_dtype == LCQ_F16, "x must be bf16 or fp16");
  LCQ_REQUIRE(ng == 1 || ng == 2 || ng == 4 || ng == 8, "ng must be 1, 2, 4 or 8");
  LCQ_REQUIRE(bounds != nullptr && bounds[0] == 0, "bounds: host token offsets from 0");
  LCQ_REQUIRE(ic > 0 && ic % 8 == 0, "ic must be a positive multiple of 8");
  LCQ_REQUIRE(ic <= 46336, "ic must be <= 46336 (32-bit H offsets)");
  LCQ_REQUIRE(x != nullptr && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
              "x must be 16-byte aligned");
  GroupedPlan p;
  LCQ_REQUIRE(grouped_plan(bounds, ng, ic, p) == 0, "bounds must not decrease");
  const int64_t need = p.tail_bytes + p.part_bytes;
  LCQ_REQUIRE(workspace != nullptr && ws_bytes >= need,
              "workspace smaller than lcq_hessian_grouped_workspace_bytes");
  hipStream_t st = as_stream(stream);
  Args a{};
  a.x = reinterpret_cast<const uint16_t*>(x);
  a.ld = ic;
  a.ic = ic;
  a.icp = ceil_to(ic, ST);
  a.nt = (int)(a.icp / ST);
  a.ntiles = a.nt * (a.nt + 1) / 2;
  a.ns = (int)p.splits;
  a.H = reinterpret_cast<float*>(H);
  a.alpha = alpha;
  a.beta = 0.f;
  char* ws = reinterpret_cast<char*>(workspace);
  int64_t off = 0;
  for (int g = 0; g < ng; ++g) {
    const int64_t n = bounds[g + 1] - bounds[g];
    p.ga.tail[g] = nullptr;
    if (n % SKT) {  // this group's last partial K-tile, zero padded
      uint16_t* tail = reinterpret_cast<uint16_t*>(ws + off);
      hipLaunchKernelGGL(k_tail_copy, dim3((unsigned)((SKT * ic / 8 + 255) / 256)), 256, 0, st,
                         a.x + bounds[g] * ic, p.ga.nk_main[g] * SKT, n, ic, tail);
      int rc = check_launch("lcq_hessian_grouped: tail");
      if (rc) return rc;
      p.ga.tail[g] = tail;
      off += ceil_to(SKT * ic * 2, 256);
    }
  }
  a.part = reinterpret_cast<float*>(ws + off);
  if (p.splits > 0) {
    const bool s3 = ic <= 8192;   // the schedule measured faster at this IC (ktile3)
    auto k = x_dtype == LCQ_F16 ? (s3 ? k_syrk_x<true, true> : k_syrk_x<true, false>)
                                : (s3 ? k_syrk_x<false, true> : k_syrk_x<false, false>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * BUF);
    hipLaunchKernelGGL(k, dim3((unsigned)(8 * ((a.ntiles + 7) / 8) * p.splits)), 256, 2 * BUF,
                       st, a, p.ga);
    int rc = check_launch("lcq_hessian_grouped: syrk");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(k_syrk_reduce, dim3((unsigned)a.ntiles, 16), 256, 0, st, a, p.ga);
  return check_launch("lcq_hessian_grouped: reduce");
}
