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
// plus one cross-half exchange, and the score accumulator converts in place to the A operand
// of P.V (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
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
  float sl2;              // scale * log2(e)
};

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [rows][128 x bf16] LDS image
__device__ __forceinline__ int img_off(int row, int ch) {
  return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__device__ __forceinline__ v4s_t tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s_t*)(lds + byte_off));
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

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void g_void_t;

// Stage one 64-key tile of K and V into LDS with global_load_lds (16 B per lane; a wave
// instruction fills 1 KB = 4 rows lane-linearly, so the image's XOR swizzle is applied to the
// global source chunk). Keys past S re-read row S-1 (finite data; masked later).
__device__ __forceinline__ void stage_kv(char* kst, char* vst, const uint16_t* kp,
                                         const uint16_t* vp, int64_t kss, int64_t vss, int k0,
                                         int S, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 4 * (4 * w + j) + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ (((row & 3) << 2) | ((row >> 2) & 3));
    const int key = min(k0 + row, S - 1);
    __builtin_amdgcn_global_load_lds((g_void_t*)(kp + (int64_t)key * kss + ch * 8),
                                     (lds_void_t*)(kst + 1024 * (4 * w + j)), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((g_void_t*)(vp + (int64_t)key * vss + ch * 8),
                                     (lds_void_t*)(vst + 1024 * (4 * w + j)), 16, 0, 0);
  }
}

// QB query blocks of 32 rows per wave (a workgroup covers 128 QB rows): every K / V fragment
// read from LDS feeds QB MFMAs. QB 2 halves the LDS traffic per flop but needs 492 VGPRs, so
// one wave per SIMD: without a hand-pipelined schedule its MFMA, softmax and LDS phases
// serialise (measured: 164 vs 277 TFLOP/s at S 512, 194 vs 379 at S 2048). QB 1 (two
// workgroups per CU, MFMA of one wave under the softmax of the other) is the default;
// LCQ_ATTN_QB=2 selects the other for probes.
template <int QB>
__global__ void __launch_bounds__(256, QB == 1 ? 2 : 1) k_attn_fwd_causal(AttnArgs a) {
  constexpr int QT = AQT * QB;
  // two stages of [K image | V image], 16 KB each: 64 KB (reused to stage the output tile)
  __shared__ __attribute__((aligned(1024))) char smem[2][2][AKT * 256];
  __shared__ float xch[4][32 * QB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int qt = (int)gridDim.x - 1 - (int)blockIdx.x;  // longest (last) query tiles first
  const int hq = blockIdx.y, b = blockIdx.z;
  const int hk = hq / (a.H / a.KVH);
  const int q0 = qt * QT;
  const uint16_t* qp = a.q + b * a.qsb + hq * a.qsh;
  const uint16_t* kp = a.k + b * a.ksb + hk * a.ksh;
  const uint16_t* vp = a.v + b * a.vsb + hk * a.vsh;
  const int kend = min(a.S, q0 + QT);
  stage_kv(smem[0][0], smem[0][1], kp, vp, a.kss, a.vss, 0, a.S, w, lane);

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
    __syncthreads();  // every wave is done with the stage the next tile overwrites
    if (k0 + AKT < kend) {
      stage_kv(smem[cur ^ 1][0], smem[cur ^ 1][1], kp, vp, a.kss, a.vss, k0 + AKT, a.S, w, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this tile's loads, not the next's
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // this tile is in LDS for every wave
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
    bool rescale = false;
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
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * a.sl2;  // sl2 > 0: max commutes with the scale
      const float mn = fmaxf(m[qb], mx);
      const float alpha = (mn == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m[qb] - mn);
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
      rs += __shfl_xor(rs, 32, 64);
      l[qb] = l[qb] * alpha + rs;
      m[qb] = mn;
      rescale |= alpha != 1.f;
      if (h == 0) xch[w][32 * qb + c] = alpha;
    }
    // rescale O (skipped when no row's max moved: a multiply by 1 is exact): its registers
    // hold rows (r & 3) + 8 (r >> 2) + 4 h of each 32-row block
    __builtin_amdgcn_wave_barrier();
    if (__builtin_amdgcn_read_exec() && __any(rescale)) {
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        float ar[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) ar[r] = xch[w][32 * qb + (r & 3) + 8 * (r >> 2) + 4 * h];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[qb][dt][r] *= ar[r];
      }
    }
    __builtin_amdgcn_wave_barrier();
    // P.V: k-step (t, s2) takes score registers 8 s2 .. 8 s2 + 7 of tile t; element j is key
    // 32 t + 16 s2 + 8 (j >> 2) + 4 h + (j & 3); V^T fragments by transposed reads of those rows
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
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const int ch = 4 * dt + 2 * (g & 1) + (pp >> 1);
          const v4s_t lo = tr_read(vimg, img_off(r0 + qq, ch) + 8 * (pp & 1));
          const v4s_t hi = tr_read(vimg, img_off(r0 + 8 + qq, ch) + 8 * (pp & 1));
          const v8s_t vf = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) o[qb][dt] = mfma32(pf[qb], vf, o[qb][dt]);
        }
      }
  }
  // normalise: rows of O take 1 / l of their query row
#pragma unroll
  for (int qb = 0; qb < QB; ++qb)
    if (h == 0) xch[w][32 * qb + c] = 1.f / l[qb];
  __syncthreads();  // also: every wave is past its last read of the K / V images
  // stage the QT x 128 bf16 output tile (QT rows of 256 B = 32 KB per 128 rows) in the stage
  // buffers, then store whole 256-byte rows of out[b, q, hq, :]
  char* ost = &smem[0][0][0];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    float il[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) il[r] = xch[w][32 * qb + (r & 3) + 8 * (r >> 2) + 4 * h];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * (QB * w + qb) + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = 32 * dt + c;
        *reinterpret_cast<__bf16*>(ost + img_off(row, col >> 3) + 2 * (col & 7)) =
            (__bf16)(o[qb][dt][r] * il[r]);
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
  LCQ_REQUIRE(B <= 65535 && H <= 65535 && S < (int64_t(1) << 30), "shape too large");
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
  a.S = (int)S; a.H = H; a.KVH = KVH;
  a.sl2 = scale * 1.44269504088896340736f;
  static const int qb_env = [] {
    const char* e = getenv("LCQ_ATTN_QB");  // probe override
    return e ? atoi(e) : 1;
  }();
  if (qb_env != 2) {
    const dim3 grid((unsigned)((S + AQT - 1) / AQT), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL(k_attn_fwd_causal<1>, grid, 256, 0, as_stream(stream), a);
  } else {
    const dim3 grid((unsigned)((S + 2 * AQT - 1) / (2 * AQT)), (unsigned)H, (unsigned)B);
    hipLaunchKernelGGL(k_attn_fwd_causal<2>, grid, 256, 0, as_stream(stream), a);
  }
  return check_launch("lcq_attn_fwd_causal");
}
