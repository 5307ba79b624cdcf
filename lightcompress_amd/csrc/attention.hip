// Causal flash-attention forward for the calibration forwards of the AWQ loss search and the
// GPTQ re-forwards (gfx950, bf16 MFMA).
//
// Replaces the sdpa call inside LlamaAttention.forward (transformers sdpa_attention_forward ->
// torch scaled_dot_product_attention(is_causal=True), which on this image is aotriton's
// attn_fwd: 160 TFLOP/s at the AWQ shape B 128, H 32, S 512, D 128). Reference call sites:
// the AWQ inspect forward of self_attn (llmc/compression/quantization/awq.py:110-126) and every
// block forward (base_blockwise_quantization.py:367-381).
//
// softmax(Q K^T * scale + causal mask) V per (batch, query head); GQA: key/value head =
// query head / (H / KVH). fp32 scores, online softmax in the exp2 domain, P rounded to bf16 for
// the P.V product (fp32 accumulate), output rounded once to bf16 -- a flash kernel's numerics
// (the reference's GPU path is a flash kernel too; parity is at the loss level and
// tests/test_attention_gpu.py bounds the error against an fp32 reference).
//
// Structure: a workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32
// rows. Key/value tiles of 64 rows are staged in LDS (image (b) of cdna_hip_programming.md T10:
// 256-byte rows with XOR-swizzled 16-byte chunks, conflict-free for the row reads of K and the
// ds_read_b64_tr_b16 transposed reads of V). Swapped QK^T (mfma(K, Q^T)): each lane holds the
// scores of ONE query row (lane & 31) for 16 of every 32 keys, so the row max / sum is local
// plus one cross-half exchange (v_permlane32_swap), and the score accumulator converts in
// place to the B operand of the swapped P.V, O^T += V^T P^T (cdna_hip_programming.md §3 "An
// accumulator tile as the next MFMA's operand"): O is held transposed, so the softmax
// rescale and the final 1 / l are lane-local too. The next K/V tile's LDS-DMA overlaps the
// current tile (counted vmcnt + raw s_barrier).
#include "lcq_common.h"

namespace lcq {

typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));

constexpr int AQT = 128;  // query rows per workgroup
constexpr int AKT = 64;   // keys per tile
constexpr int AHD = 128;  // head dim

struct AttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  uint16_t* out;          // [B, S, H, D]
  int64_t qsb, qsh, qss;  // element strides of q viewed as [B, H, S, D]; d contiguous
  int64_t ksb, ksh, kss;
  int64_t vsb, vsh, vss;
  int S, H, KVH;
  int nqt;                // query tiles per (batch, head)
  float sl2;              // scale * log2(e)
};

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [rows][128 x bf16] LDS image
__device__ __forceinline__ int img_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

// Transposed 8-byte LDS read as inline asm: the builtin form makes the compiler put a
// vmcnt(0) before it (it cannot tell the read from the K / V stage being filled by LDS-DMA for
// the next tile), which serialised every tile behind the next tile's loads. The asm reads are
// invisible to the compiler's lgkmcnt tracking: tr_wait() below waits for them explicitly and
// ties their results, so no consumer is scheduled above the wait.
__device__ __forceinline__ v4s_t tr_read(const char* lds, int byte_off) {
  v4s_t r;
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(lds + byte_off);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}

__device__ __forceinline__ void tr_wait(v4s_t (&lo)[4], v4s_t (&hi)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(hi[0]), "+v"(hi[1]),
                 "+v"(hi[2]), "+v"(hi[3])
               :
               : "memory");
}

__device__ __forceinline__ v16f_t mfma32(v8s_t a, v8s_t b, v16f_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(v8bf_t, a),
                                                 __builtin_bit_cast(v8bf_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
  typedef float v2f_t __attribute__((ext_vector_type(2)));
  const v2bf_t hv = __builtin_convertvector((v2f_t){a, b}, v2bf_t);
  return __builtin_bit_cast(uint32_t, hv);
}

// value of lane ^ 32 (the other half of a 32-lane query block): v_permlane32_swap, a VALU op,
// where __shfl_xor lowers to ds_bpermute (an LDS round trip and an lgkmcnt wait per call)
__device__ __forceinline__ float other_half(float v, int h) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(h ? r[0] : r[1]);
}

typedef __attribute__((address_space(3))) void lds_void_t;

// Stage one 64-key tile of K and V into LDS by buffer-descriptor LDS-DMA (16 B per lane; a
// wave instruction fills 1 KB = 4 rows lane-linearly, so the image's XOR swizzle is applied to
// the global source chunk). Keys past S re-read row S-1 (finite data; masked later). Buffer
// loads (not global_load_lds): the compiler then leaves the tile's vmcnt to the counted waits
// in the loop instead of a vmcnt(0) before every LDS read of the stage.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const uint16_t* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ void stage_kv(char* kst, char* vst, __amdgpu_buffer_rsrc_t kr,
                                         __amdgpu_buffer_rsrc_t vr, int64_t kss, int64_t vss,
                                         int k0, int S, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 4 * (4 * w + j) + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const int key = min(k0 + row, S - 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(kr, (lds_void_t*)(kst + 1024 * (4 * w + j)), 16,
                                             (uint32_t)(key * kss * 2 + ch * 16), 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vr, (lds_void_t*)(vst + 1024 * (4 * w + j)), 16,
                                             (uint32_t)(key * vss * 2 + ch * 16), 0, 0, 0);
  }
}

// QB query blocks of 32 rows per wave (a workgroup covers 128 QB rows): every K / V fragment
// read from LDS feeds QB MFMAs. QB 2 halves the LDS traffic per flop but needs 492 VGPRs, so
// one wave per SIMD: without a hand-pipelined schedule its MFMA, softmax and LDS phases
// serialise (measured in round 3: 164 vs 277 TFLOP/s at S 512, 194 vs 379 at S 2048). QB 1
// (two workgroups per CU, MFMA of one wave under the softmax of the other) is the one launched;
// the QB 2 launch and its environment switch were removed.
template <int QB>
__global__ void __launch_bounds__(256, QB == 1 ? 2 : 1) k_attn_fwd_causal(AttnArgs a) {
  constexpr int QT = AQT * QB;
  // two stages of [K image | V image], 16 KB each: 64 KB (reused to stage the output tile);
  // dynamic LDS: the compiler then tracks the K reads of a stage apart from the LDS-DMA
  // filling the other one (with a static array it waited vmcnt(0) before them)
  extern __shared__ __attribute__((aligned(1024))) char attn_lds[];
  typedef char stage_t[2][AKT * 256];
  stage_t* smem = reinterpret_cast<stage_t*>(attn_lds);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  // XCD-aware work order: the dispatcher places workgroup p on XCD p % 8, so work id L is
  // taken from contiguous ranges per XCD (L = xcd's base + p / 8). Consecutive ids are the
  // query tiles of the H / KVH query heads sharing one key/value head, i.e. the workgroups
  // that stream the same K / V rows run together on one XCD and share them in its L2 (with
  // the hardware order every XCD fetched every (b, kv head)'s K / V from HBM).
  const int nqt = a.nqt;
  int L;
  {
    const int nwg = (int)gridDim.x, p = (int)blockIdx.x;
    const int xcd = p & 7, q8 = nwg >> 3, r8 = nwg & 7;
    L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (p >> 3);
  }
  const int qt = nqt - 1 - L % nqt;  // longest (last) query tiles first within a group
  const int hq = (L / nqt) % a.H, b = L / (nqt * a.H);
  const int hk = hq / (a.H / a.KVH);
  const int q0 = qt * QT;
  const uint16_t* qp = a.q + b * a.qsb + hq * a.qsh;
  const uint16_t* kp = a.k + b * a.ksb + hk * a.ksh;
  const uint16_t* vp = a.v + b * a.vsb + hk * a.vsh;
  const int kend = min(a.S, q0 + QT);
  const __amdgpu_buffer_rsrc_t kr = head_rsrc(kp), vr = head_rsrc(vp);
  stage_kv(smem[0][0], smem[0][1], kr, vr, a.kss, a.vss, 0, a.S, w, lane);

  int qrow[QB];  // this lane's query row in block qb (both lane halves)
  // Q^T as the B operand of mfma(K, Q^T): lane holds Q[qrow][16 kk + 8 h + j]
  v8s_t qf[QB][8];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    qrow[qb] = q0 + 32 * (QB * w + qb) + c;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (qrow[qb] < a.S)
        qf[qb][kk] = *reinterpret_cast<const v8s_t*>(qp + (int64_t)qrow[qb] * a.qss + 16 * kk +
                                                     8 * h);
      else
        qf[qb][kk] = (v8s_t){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  float m[QB], l[QB];
  v16f_t o[QB][4];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    m[qb] = -INFINITY;
    l[qb] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[qb][dt][r] = 0.f;
  }
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;

  int it = 0;
  for (int k0 = 0; k0 < kend; k0 += AKT, ++it) {
    const int cur = it & 1;
    // Raw s_barrier with counted waits (not __syncthreads, whose release fence waits for
    // vmcnt(0), i.e. for the NEXT tile's loads issued just before it: no prefetch at all).
    // every wave is done with the stage the next tile overwrites (its reads were consumed)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (k0 + AKT < kend) {
      stage_kv(smem[cur ^ 1][0], smem[cur ^ 1][1], kr, vr, a.kss, a.vss, k0 + AKT, a.S, w, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this tile's loads, not the next's
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // this tile is in LDS for every wave
    const char* kimg = smem[cur][0];
    const char* vimg = smem[cur][1];

    // S^T tiles t = 0, 1: register r holds key k0 + 32 t + (r & 3) + 8 (r >> 2) + 4 h of the
    // lane's query row
    v16f_t s[QB][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int qb = 0; qb < QB; ++qb)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[qb][t][r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const v8s_t kf = *reinterpret_cast<const v8s_t*>(kimg + img_off(32 * t + c, 2 * kk + h));
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) s[qb][t] = mfma32(kf, qf[qb][kk], s[qb][t]);
      }
    }
    // causal mask, online softmax in the exp2 domain (scores scaled by scale * log2 e inside
    // the exponent's fma; v_exp_f32 directly: results below 2^-126 flush to 0), per block
    float alpha[QB];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      const bool diag = k0 + AKT - 1 > q0 + 32 * (QB * w + qb);  // a key can exceed a row
      float mx = -INFINITY;
      if (diag) {  // wave-uniform; the per-key mask is an added 0 / -inf (no branches)
        const int lim = min(qrow[qb], a.S - 1) - k0 - 4 * h;  // largest visible key offset
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kofs = 32 * t + (r & 3) + 8 * (r >> 2);
            s[qb][t][r] += (kofs > lim) ? -INFINITY : 0.f;
          }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[qb][t][r]);
      mx = fmaxf(mx, other_half(mx, h)) * a.sl2;  // sl2 > 0: max commutes with the scale
      const float mn = fmaxf(m[qb], mx);
      alpha[qb] = (mn == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m[qb] - mn);
      const float msub = (mn == -INFINITY) ? 0.f : mn;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(__fmaf_rn(s[qb][t][r], a.sl2, -msub));
          s[qb][t][r] = p;
          rs += p;
        }
      rs += other_half(rs, h);
      l[qb] = l[qb] * alpha[qb] + rs;
      m[qb] = mn;
    }
    // rescale O^T (skipped where no row's max moved: a multiply by 1 is exact). O is held
    // transposed (see P.V below), so a lane's registers all belong to its own query row and
    // alpha is lane-local: no exchange through LDS
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      if (alpha[qb] != 1.f) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[qb][dt][r] *= alpha[qb];
      }
    }
    // O^T += V^T P^T: mfma(V^T, P^T), so the accumulator's columns are query rows (lane & 31)
    // and its registers head dims 32 dt + (r & 3) + 8 (r >> 2) + 4 h. k-step (t, s2) takes
    // score registers 8 s2 .. 8 s2 + 7 of tile t; element j is key 32 t + 16 s2 + 8 (j >> 2) +
    // 4 h + (j & 3); V^T fragments by transposed reads of those rows
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        v8s_t pf[QB];
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) {
          uint32_t* pw = reinterpret_cast<uint32_t*>(&pf[qb]);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            pw[j] = pack_bf16(s[qb][t][8 * s2 + 2 * j], s[qb][t][8 * s2 + 2 * j + 1]);
        }
        const int r0 = 32 * t + 16 * s2 + 4 * (g >> 1);  // this 16-lane group's first key row
        v4s_t lo[4], hi[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int ch = 4 * dt + 2 * (g & 1) + (pp >> 1);
          lo[dt] = tr_read(vimg, img_off(r0 + qq, ch) + 8 * (pp & 1));
          hi[dt] = tr_read(vimg, img_off(r0 + 8 + qq, ch) + 8 * (pp & 1));
        }
        tr_wait(lo, hi);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const v8s_t vf = {lo[dt].x, lo[dt].y, lo[dt].z, lo[dt].w,
                            hi[dt].x, hi[dt].y, hi[dt].z, hi[dt].w};
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) o[qb][dt] = mfma32(vf, pf[qb], o[qb][dt]);
        }
      }
  }
  __syncthreads();  // every wave is past its last read of the K / V images
  // normalise (1 / l of the lane's own query row) and stage the QT x 128 bf16 output tile
  // (QT rows of 256 B = 32 KB per 128 rows) in the stage buffers: registers 4 i .. 4 i + 3 of
  // block dt are 4 consecutive head dims (8 bytes), then whole 256-byte rows of out[b, q, hq, :]
  char* ost = &smem[0][0][0];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const float il = 1.f / l[qb];
    const int row = 32 * (QB * w + qb) + c;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint2 pk;
        pk.x = pack_bf16(o[qb][dt][4 * i] * il, o[qb][dt][4 * i + 1] * il);
        pk.y = pack_bf16(o[qb][dt][4 * i + 2] * il, o[qb][dt][4 * i + 3] * il);
        *reinterpret_cast<uint2*>(ost + img_off(row, 4 * dt + i) + 8 * h) = pk;
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 8 * QB; ++i) {  // QT rows x 16 chunks
    const int idx = i * 256 + tid, row = idx >> 4, ch = idx & 15;
    const int qr = q0 + row;
    if (qr < a.S) {
      const uint4 val = *reinterpret_cast<const uint4*>(ost + img_off(row, ch));
      *reinterpret_cast<uint4*>(a.out + (((int64_t)b * a.S + qr) * a.H + hq) * AHD + ch * 8) = val;
    }
  }
}

}  // namespace lcq

using namespace lcq;

extern "C" int lcq_attn_fwd_causal(const void* q, const void* k, const void* v, int dtype,
                                   int64_t B, int64_t S, int H, int KVH, int D,
                                   const int64_t* q_strides, const int64_t* k_strides,
                                   const int64_t* v_strides, float scale, void* out,
                                   void* stream) {
  LCQ_REQUIRE(dtype == LCQ_BF16, "attention kernel: bf16 only");
  LCQ_REQUIRE(D == AHD, "attention kernel: head dim 128 only");
  LCQ_REQUIRE(B > 0 && S > 0 && H > 0 && KVH > 0 && H % KVH == 0, "bad shape / GQA grouping");
  LCQ_REQUIRE(B * H * ((S + AQT - 1) / AQT) < (int64_t(1) << 31) && S < (int64_t(1) << 30),
              "shape too large");
  LCQ_REQUIRE(q && k && v && out && q_strides && k_strides && v_strides, "null pointer");
  AttnArgs a{};
  a.q = reinterpret_cast<const uint16_t*>(q);
  a.k = reinterpret_cast<const uint16_t*>(k);
  a.v = reinterpret_cast<const uint16_t*>(v);
  a.out = reinterpret_cast<uint16_t*>(out);
  a.qsb = q_strides[0]; a.qsh = q_strides[1]; a.qss = q_strides[2];
  a.ksb = k_strides[0]; a.ksh = k_strides[1]; a.kss = k_strides[2];
  a.vsb = v_strides[0]; a.vsh = v_strides[1]; a.vss = v_strides[2];
  // 16-byte loads of 8 head-dim elements: every row start must be 16-byte aligned
  const int64_t all = a.qsb | a.qsh | a.qss | a.ksb | a.ksh | a.kss | a.vsb | a.vsh | a.vss;
  LCQ_REQUIRE((all & 7) == 0, "attention kernel: row strides must be multiples of 8 elements");
  LCQ_REQUIRE(((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(out)) & 15) == 0,
              "attention kernel: 16-byte aligned tensors required");
  LCQ_REQUIRE(S * a.kss < (int64_t(1) << 30) && S * a.vss < (int64_t(1) << 30),
              "attention kernel: one head's K / V span must stay below 2 GB (32-bit offsets)");
  a.S = (int)S; a.H = H; a.KVH = KVH;
  a.sl2 = scale * 1.44269504088896340736f;
  constexpr int kLds = 2 * 2 * AKT * 256;
  (void)hipFuncSetAttribute((const void*)k_attn_fwd_causal<1>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  a.nqt = (int)((S + AQT - 1) / AQT);
  hipLaunchKernelGGL(k_attn_fwd_causal<1>, dim3((unsigned)(a.nqt * H * B)), 256, kLds,
                     as_stream(stream), a);
  return check_launch("lcq_attn_fwd_causal");
}
