/*
 * lcq.h — C ABI of the MI355X-native LightCompress weight-quantization hot path.
 *
 * The reference (zhangbilang/LightCompress, package `llmc`) is pure Python/torch and has no
 * FFI of its own; every entry point below replaces one reference function (cited file:line,
 * paths relative to the reference root) and is what a ctypes / cffi binding of that function
 * binds.
 *
 * Conventions
 *   - All tensor arguments are raw DEVICE pointers (hipMalloc'd / torch CUDA storage),
 *     row-major, contiguous, with explicit sizes. No torch types cross this boundary.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream). Launches are
 *     asynchronous on that stream; the caller synchronises.
 *   - The caller owns every buffer; the library never allocates device memory.
 *   - Return value: 0 on success, negative LCQ_E* code on error; lcq_last_error() returns a
 *     thread-local message for the last failing call.
 *   - Numerics follow the reference op by op: every intermediate is rounded to the compute
 *     dtype (the dtype torch's type promotion gives the reference expression), divisions
 *     are IEEE true divisions, torch.round is round-half-to-even.
 */
#ifndef LCQ_H_
#define LCQ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype codes (mirror the torch dtypes the reference uses on this path) */
enum lcq_dtype {
  LCQ_F32 = 0,
  LCQ_F16 = 1,
  LCQ_BF16 = 2,
  LCQ_I8 = 3,
  LCQ_U8 = 4,
  LCQ_I32 = 5,
  LCQ_FP8E4M3 = 6,
  LCQ_F64 = 7,
  LCQ_FP8E5M2 = 8,
};

enum lcq_status {
  LCQ_OK = 0,
  LCQ_EINVAL = -1,  /* bad argument (shape, dtype, divisibility) */
  LCQ_ELAUNCH = -2, /* HIP launch / runtime error */
  LCQ_EUNSUP = -3,  /* combination not supported */
};

int lcq_version(void);
const char* lcq_last_error(void);

/* ---------------------------------------------------------------------------------------
 * Grouped integer quantization, dynamic (min/max) qparams.
 * Replaces IntegerQuantizer.get_tensor_qparams + quant/dequant/quant_dequant +
 * fake_quant_weight_dynamic / real_quant_weight_dynamic
 *   (llmc/compression/quantization/quant.py:132-143, 545-559, 690-717, 833-869, 916-953)
 * optionally fused with:
 *   - the AWQ column pre-scale W * s (awq.py:39-46, 147-164)            [pre_scale != NULL]
 *   - the AWQ clip v1 clamp(W, min, max) per group (auto_clip.py:193-212)  [clip_max != NULL]
 *   - VllmRealQuantLinear.pack (module_utils.py:929-955)                  [packed_out != NULL]
 *
 * x        [rows, cols] dtype x_dtype (F32/F16/BF16); the compute dtype is x_dtype.
 * group    elements per group along cols; 0 or == cols means per-channel (reduce over a row).
 *          cols % group == 0; group % 8 == 0.
 * pre_scale  optional [cols] in x_dtype: x <- round_ct(x * pre_scale[col]) before anything.
 * clip_max/clip_min optional [rows*cols/group] in x_dtype: x <- clamp(x, clip_min, clip_max)
 *          (clip_min may be NULL with clip_max set: symmetric clip, min = -max).
 * qmin, qmax  integer range (IntegerQuantizer.__init__, quant.py:662-678); sym selects the
 *          symmetric qparams formula (zeros = 0).
 * fq_out   optional [rows, cols] fake-quant output, dtype fq_dtype (F32/F16/BF16: final .to()).
 * codes_out optional [rows, cols] integer codes, dtype codes_dtype (I8/U8/I32).
 * packed_out optional [rows, ceil(cols / (32/pack_bits))] int32, vLLM little-endian pack of
 *          (code + 2^(pack_bits-1)) & 0xFF; pack_bits in {4, 8}.
 * scales_out / zeros_out optional [rows*cols/group] in x_dtype (zeros_out unused when sym).
 * ------------------------------------------------------------------------------------- */
int lcq_int_quant_dynamic(const void* x, int x_dtype, int64_t rows, int64_t cols,
                          int64_t group, const void* pre_scale, const void* clip_max,
                          const void* clip_min, int qmin, int qmax, int sym,
                          void* fq_out, int fq_dtype, void* codes_out, int codes_dtype,
                          void* packed_out, int pack_bits, void* scales_out, void* zeros_out,
                          void* stream);

/* lcq_int_quant_dynamic with calib_algo learnable and clip factors (v2 clip buffers
 * buf_upbound_factor / buf_lowbound_factor, passed by BaseBlockwiseQuantization.w_qdq,
 * base_blockwise_quantization.py:46-66): each group's min / max becomes
 * get_learnable_range(group, low, up) (quant.py:205-219) before get_qparams. up / low:
 * [rows*cols/group] in x_dtype (f16 / bf16); sym uses up only; asym with low NULL leaves the
 * range alone, as the reference does. */
int lcq_int_quant_learnable(const void* x, int x_dtype, int64_t rows, int64_t cols,
                            int64_t group, const void* up, const void* low, int qmin, int qmax,
                            int sym, void* fq_out, int fq_dtype, void* codes_out,
                            int codes_dtype, void* scales_out, void* zeros_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Grouped integer quantization with GIVEN qparams.
 * Replaces IntegerQuantizer.fake_quant_weight_static / real_quant_weight_static
 *   (quant.py:699-717, 785-831, 871-914); used by GPTQ deploy (gptq.py:411-452).
 * scales [rows*cols/group] dtype s_dtype; zeros [rows*cols/group] dtype z_dtype or NULL (= 0).
 * ct_dtype is the compute dtype (torch result_type of x, scales, zeros); every input is
 * converted (exactly) to ct_dtype and every op is rounded to ct_dtype.
 * ------------------------------------------------------------------------------------- */
int lcq_int_quant_static(const void* x, int x_dtype, int64_t rows, int64_t cols,
                         int64_t group, const void* scales, int s_dtype, const void* zeros,
                         int z_dtype, int ct_dtype, int qmin, int qmax, void* fq_out,
                         int fq_dtype, void* codes_out, int codes_dtype, void* packed_out,
                         int pack_bits, void* stream);

/* lcq_int_quant_static with round_zp False (quant.py:701-707, the HQQ configs):
 * q = clamp(round(x / s.clamp_min(1e-9) + z), qmin, qmax), x^ = (q - z) * s, every op
 * rounded to ct_dtype; zeros stay float (real quant keeps them unrounded). */
int lcq_int_quant_static_nozp(const void* x, int x_dtype, int64_t rows, int64_t cols,
                              int64_t group, const void* scales, int s_dtype, const void* zeros,
                              int z_dtype, int ct_dtype, int qmin, int qmax, void* fq_out,
                              int fq_dtype, void* codes_out, int codes_dtype, void* stream);

/* get_minmax_range + get_qparams (quant.py:132-143, 545-559) of x [ng, gs] (gs % 8 == 0) in
 * the x dtype, incl. round_zp False (zeros = qmin - min / scales, unrounded, unclamped).
 * scales / zeros [ng] in the x dtype; zeros may be NULL when sym. */
int lcq_minmax_qparams(const void* x, int dtype, int64_t ng, int64_t gs, int qmin, int qmax,
                       int sym, int round_zp, void* scales, void* zeros, void* stream);

/* Workspace bytes of lcq_hqq_proximal for ng groups. */
int64_t lcq_hqq_workspace_bytes(int64_t ng);

/* optimize_weights_proximal (quant.py:588-610; hqq.py:36-61) on w [ng, gs] fp32 (gs % 8 == 0):
 * scales / zeros fp32 [ng] in (get_qparams of the same groups) and out (best scales =
 * 1 / (1 / s), the zeros of the last iteration run). Up to `iters` half-quadratic steps,
 * shrink_op with lp_norm and the quantizer's beta, stopping at the first step whose mean
 * |w - w_r| is not below the best so far; enqueued without a host sync. state_out (nullable,
 * device, 16 B): {float best_error, int stopped, int iters_run, int pad}. */
int lcq_hqq_proximal(const void* w, int64_t ng, int64_t gs, void* scales, void* zeros, int qmin,
                     int qmax, float lp_norm, float beta, int iters, void* workspace,
                     int64_t ws_bytes, void* state_out, void* stream);

/* Per-tensor static qparams given as 0-dim tensors on the reference's CPU path
 * (fake_quant_act_static with register_act_qparams' scale / zero, quant.py:699-743): torch-CPU
 * takes a 0-dim operand as a scalar of the op's opmath type, so the fp32 scale / zero (device
 * fp32, one element each; zero NULL = 0) enter every op at full precision while each result is
 * rounded to ct_dtype. x [rows, cols], cols % 8 == 0. */
int lcq_int_quant_static_scalar(const void* x, int x_dtype, int64_t rows, int64_t cols,
                                const void* scale, const void* zero, int ct_dtype, int qmin,
                                int qmax, void* fq_out, int fq_dtype, void* codes_out,
                                int codes_dtype, void* stream);

/* Static quant with a column -> group map: element (r, c) uses scales/zeros group
 * r * ngc + col_group[c] (int32 [cols], 16-byte aligned). GPTQ's act-order deploy
 * (gptq.py:411-459 w_qdq: fake_quant_static(W[:, perm])[:, invperm]) with
 * col_group[c] = invperm[c] / group, without the two column gathers. cols % 8 == 0. */
int lcq_int_quant_static_cols(const void* x, int x_dtype, int64_t rows, int64_t cols,
                              const int32_t* col_group, int64_t ngc, const void* scales,
                              int s_dtype, const void* zeros, int z_dtype, int ct_dtype,
                              int qmin, int qmax, void* fq_out, int fq_dtype, void* codes_out,
                              int codes_dtype, void* stream);

/* vLLM pack of existing integer codes (module_utils.py:929-955).
 * codes [rows, cols] I8/U8/I32 -> packed [rows, ceil(cols*bits/32)] int32. */
int lcq_pack_vllm(const void* codes, int codes_dtype, int64_t rows, int64_t cols, int bits,
                  void* packed_out, void* stream);

/* AutoAWQ GEMM pack (AutoawqRealQuantLinear.gemm_pack, module_utils.py:1097-1158), incl. its
 * un-clamped fp32 re-quantisation round((W + z*s16)/s16) and raw int32 shift-or packing.
 * w [oc, ic] (BF16/F16/F32), scales [oc, ic/group] s_dtype, zeros [oc, ic/group] I32.
 * qweight_out [ic, oc/8] int32, scales_t_out [ic/group, oc] fp16, qzeros_out [ic/group, oc/8].
 * Only bits == 4 (as the reference). */
int lcq_pack_autoawq_gemm(const void* w, int w_dtype, int64_t oc, int64_t ic, int64_t group,
                          const void* scales, int s_dtype, const void* zeros, int bits,
                          void* qweight_out, void* scales_t_out, void* qzeros_out,
                          void* stream);

/* ---------------------------------------------------------------------------------------
 * GPTQ Hessian: H = beta*H + alpha * X^T X   (GPTQ.add_batch, gptq.py:253-295)
 * x [n, ic] BF16/F16 token-major activations; H [ic, ic] fp32 (kept symmetric).
 * The reference's per-sample running average maps to beta = n/(n+b),
 * alpha = fp32(sqrt(2/(n+b)))^2. 256x256-tile MFMA SYRK (bf16/fp16 products, fp32
 * accumulation) over the upper triangle, mirrored, read from x as it is (transposed LDS
 * reads; ic % 8 == 0). workspace >= lcq_hessian_workspace_bytes (a zero-padded copy of the
 * last partial 64-token tile + split-K slabs when ic is small); caller-owned, device memory.
 * ------------------------------------------------------------------------------------- */
int64_t lcq_hessian_workspace_bytes(int64_t n, int64_t ic);
int lcq_hessian_accum(const void* x, int x_dtype, int64_t n, int64_t ic, void* H, float alpha,
                      float beta, void* workspace, int64_t ws_bytes, void* stream);

/* The grouped GPTQ Hessian (gptq_core.HessianAccumulator) in ONE launch: x [n, ic] token-major,
 * bounds (host int64 [ng + 1], bounds[0] = 0) cut it into ng = 1 / 2 / 4 / 8 token groups;
 * every group's X^T X is split over K-tile slabs by a plan that depends only on the group's
 * token count and ic (world-independent), each slab's upper-tile partial goes to the workspace,
 * and one reduce folds each group's slabs in order, sums the groups in the fixed tree
 * ((g0 + g1) + (g2 + g3)) + ((g4 + g5) + (g6 + g7)) and writes H = alpha * tree, mirrored
 * (gptq.py:253-295 accumulates the same samples as a running average). Bit-identical to one
 * lcq_hessian_accum per group + lcq_tree_sum. */
int64_t lcq_hessian_grouped_workspace_bytes(const int64_t* bounds, int ng, int64_t ic);
int lcq_hessian_grouped(const void* x, int x_dtype, int64_t ic, const int64_t* bounds, int ng,
                        void* H, float alpha, void* workspace, int64_t ws_bytes, void* stream);

/* Deterministic reduction of Hessian partials (the grouped GPTQ Hessian: the calibration
 * samples of add_batch, gptq.py:253-295, cut into 8 fixed groups, so that token-sharded ranks
 * and one GPU sum them in the same order): out[i] = alpha * tree(parts[0..np)[i]) with the
 * fixed pairwise tree ((p0 + p1) + (p2 + p3)) + ...; parts is a HOST array of np in {1, 2, 4, 8}
 * device pointers to fp32 [n] (n % 4 == 0, 16-byte aligned); out may alias none of them. */
int lcq_tree_sum(const void* const* parts, int np, int64_t n, float alpha, void* out,
                 void* stream);

/* ---------------------------------------------------------------------------------------
 * GPTQ in-block column loop for one 128-column block (GPTQ.weight_transform, gptq.py:198-244,
 * group qparams gptq.py:358-366). W [rows, ld] fp32 in (act-order permuted) column space:
 * columns [col0, col0+count) are replaced by the error-compensated weights (`tmp`);
 * err (k-major [128, ld_err], ld_err >= rows: err[k * ld_err + r]) receives Err1 for the caller's trailing update
 * W[:, col0+count:] -= err @ U[col0:col0+count, col0+count:].
 * U [ldu, ldu] fp32 upper Cholesky factor of H^-1. group in {32, 64, 128}: per-group minmax
 * qparams from the block-start weights written to s_out/z_out [rows, ng_total] (fp32);
 * group == 0: fixed per-row qparams s_in/z_in [rows] (per-channel).
 * losses optional [rows, ld] fp32: (w-q)^2 / (2 d^2).
 * fmt 0: IntegerQuantizer qdq (quant.py:699-717). fmt LCQ_FP8E4M3 / LCQ_FP8E5M2: FloatQuantizer
 * (use_qtorch, quant.py:1061-1080): q = float_quantize(w / s + 0) * s in fp32 with the
 * saturating native cast, symmetric qparams with qmax = finfo.max (qmin, qmax,
 * sym, z_in, z_out are ignored); the per-channel form is gptq_fp8.yml's column loop.
 * nprev > 0 (left-looking near updates, gptq.py:244 restricted to this block's columns):
 * before its loop the kernel applies, for each of the nprev full 128-column blocks right
 * before col0 in order, W[:, col0 : col0 + count] -= Err_j @ U[rows of block j, same columns],
 * Err_j being rows [128 j, 128 j + 128) of the k-major err_prev (row stride ld_err) -- each
 * product the k-ordered fp32 fmaf chain of lcq_gptq_trailing, rounded, then subtracted: the
 * same bits as one lcq_gptq_trailing(c1 = col0, c2 >= col0 + count) after each earlier block.
 * ------------------------------------------------------------------------------------- */
int lcq_gptq_block(void* W, int64_t rows, int64_t ld, int64_t col0, int count, const void* U,
                   int64_t ldu, int64_t group, int qmin, int qmax, int sym, int fmt,
                   const void* s_in, const void* z_in, void* s_out, void* z_out,
                   int64_t ng_total, void* err, int64_t ld_err, void* losses,
                   const void* err_prev, int nprev, void* stream);

/* GPTQ static groups (gptq.py:224-227, static_groups: True): the same block loop with fixed
 * qparams per (row, ORIGINAL group): permuted column c uses s_in / z_in [rows, ngc] at group
 * col_group[c] = perm[c] / group_size (int32 [ld]). z_in NULL for symmetric. */
int lcq_gptq_block_cols(void* W, int64_t rows, int64_t ld, int64_t col0, int count,
                        const void* U, int64_t ldu, int qmin, int qmax, const void* s_in,
                        const void* z_in, const int32_t* col_group, int64_t ngc, void* err,
                        int64_t ld_err, void* losses, const void* err_prev, int nprev,
                        void* stream);

/* C = beta C + alpha A op(B) on row-major fp32 views (the fp32 updates of the recursive
 * factorisation behind U, gptq_core._chol_inv_rec: `addmm_` of the reference-equivalent
 * cholesky -> cholesky_inverse -> cholesky chain, gptq.py:161-170). A [M, K] (lda), B [K, N]
 * (bt 0) or its transpose stored [N, K] (bt 1; ldb), C [M, N] (ldc); beta 0 never reads C.
 * fp32 MFMA (32x32x2), 128x128 tiles. */
int lcq_gemm_f32(int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                 const void* B, int64_t ldb, int bt, float beta, void* C, int64_t ldc,
                 void* stream);

/* lcq_gemm_f32 with a caller workspace (lcq_gemm_f32_workspace_bytes(M, N, K) bytes, 0 when
 * not needed): grids whose last round of 256 workgroups would run more than 10 % empty go
 * stream-K -- the tiles x K-chunks work split evenly over 256 workgroups, k segments of cut
 * tiles summed in k order by a fixup pass (deterministic). */
int64_t lcq_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K);
int lcq_gemm_f32_ws(int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                    const void* B, int64_t ldb, int bt, float beta, void* C, int64_t ldc,
                    void* workspace, int64_t ws_bytes, void* stream);

/* Rows [row0, row1) of the lcq_gemm_f32 product C = beta C + alpha A op(B) (A, C the FULL
 * [M, *] operands): the kernel variant and tile size are those the full M x N product gets
 * (never stream-K), so every output element is computed with the same k order whichever rank
 * computes it -- the factorisation's large products row-split over the ranks of a
 * token-sharded GPTQ run (gptq.py:161-170; gptq_core.chain_sharding) are bit-identical to one
 * GPU's. row0 / row1 on multiples of lcq_gemm_f32_row_unit(M, N) (64 or 128; row1 may be M). */
int64_t lcq_gemm_f32_row_unit(int64_t M, int64_t N);
int lcq_gemm_f32_rows(int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                      const void* B, int64_t ldb, int bt, float beta, void* C, int64_t ldc,
                      int64_t row0, int64_t row1, void* stream);

/* Rows [row0, row1) of C = beta C + alpha A op(B) (A, C the FULL [M, *] fp32 operands, B as in
 * lcq_gemm_f32; N % 16 == 0, ldc % 4 == 0, C 16-byte aligned) on bf16 MFMA: every operand
 * value split into three bf16 planes, the six plane products above the 2^-24 level summed by
 * one k_gemm16h GEMM over K' = 6 * roundup(K, 64) with fp32 accumulation (the three dropped
 * plane products are below 2^-24 relative: close to, not identical with, an fp32 GEMM's error;
 * ~2x its rate on gfx950, where fp32 MFMA runs at 1/16 of bf16). The recursion's large
 * products (gptq_core._gemm; gptq.py:161-170). Each output element's k order is independent of
 * the row range, so a row-split product is bit-identical to the whole one. at 1: A stored
 * k-major [K, lda] (GPTQ's stacked Err1). Products with fewer than 256 output tiles split K (by
 * the FULL shape, at most max_splits) into fp32 partials folded in split order. Workspace:
 * lcq_gemm_f32x6_workspace_bytes(M, row1 - row0, N, K, max_splits) bytes, 16-byte aligned.
 * row0 == row1 (an empty rank share) is a no-op, as for lcq_gemm_f32_rows. */
int64_t lcq_gemm_f32x6_workspace_bytes(int64_t M, int64_t rows, int64_t n, int64_t k,
                                       int max_splits);
int lcq_gemm_f32x6(int64_t M, int64_t N, int64_t K, float alpha, const void* A, int64_t lda,
                   int at, const void* B, int64_t ldb, int bt, float beta, void* C, int64_t ldc,
                   int64_t row0, int64_t row1, int max_splits, void* workspace, int64_t ws_bytes,
                   void* stream);

/* Diagonal tile of the recursive fp32 factorisation behind U = chol(H^-1, upper)
 * (gptq.py:169-174): for SPD A (n x n, n <= 128, row-major fp32, leading dim lda), X <- L^-1
 * and, if L is not NULL, L <- the lower Cholesky factor (upper parts zeroed). A is only read.
 * info (int32): row0 + the first non-positive pivot of the tile (1-based), written only on
 * failure and only if still 0 (the order of the leading minor torch.linalg.cholesky reports). */
int lcq_chol_inv_tile(const void* A, int64_t lda, int n, void* L, int64_t ldl, void* X,
                      int64_t ldx, void* info, int64_t row0, void* stream);

/* GPTQ act-order preparation (gptq.py:58-64, 128-176) as one gather pass: out[i][j] =
 * f(A[rsrc[i]][csrc[j]]) (rsrc / csrc int64 index arrays, NULL = identity), A bf16 or fp32
 * [rows, lda], out fp32 [rows, ldo]; f widens to fp32, zeroes dead_col[csrc[j]] columns
 * (prepare_weight: W[:, dead] = 0; W[:, perm]), and on the diagonal i == j sets
 * dead_diag[csrc[j]] entries to 1 then adds *damp (prepare_hessian: H[dead, dead] = 1;
 * H[perm][:, perm]; H[d, d] += damp, with rsrc = csrc = perm reversed for the chain's J H J).
 * uint8 masks / damp may be NULL. Any width: rows of <= 40960 columns are staged in LDS,
 * wider ones gathered straight from the (L2-resident) source row. */
int lcq_gather_rc(const void* A, int a_dtype, int64_t rows, int64_t cols, int64_t lda,
                  const int64_t* rsrc, const int64_t* csrc, const uint8_t* dead_col,
                  const uint8_t* dead_diag, const float* damp, void* out, int64_t ldo,
                  void* stream);

/* GPTQ trailing update W[:, c1:c2] -= err^T[:, :cnt] @ U[c0:c0+cnt, c1:c2] (gptq.py:244) on
 * fp32 MFMA, the product rounded to fp32 then subtracted (the reference's two roundings).
 * err k-major [cnt, ld_err] fp32 (ld_err >= rows, cnt <= 8192): one block's Err1 from
 * lcq_gptq_block, or the stacked Err1 of several blocks (the host's two-level lazy update
 * applies a 1024-column superblock's errors to the far columns at once). With 16-byte aligned
 * operands (ld_err, ld, ldu % 4 == 0) and cnt % 32 == 0 it runs on lcq_gemm_f32's LDS-DMA
 * kernel (A read k-major), else on a register-staged 32x32x2 kernel; both compute every
 * element as the k-ordered fmaf chain (bit-identical to each other and independent of the row
 * range, so row-sharded GPTQ is bit-identical to one GPU). */
int lcq_gptq_trailing(void* W, int64_t rows, int64_t ld, int64_t c0, int cnt, int64_t c1,
                      int64_t c2, const void* err, int64_t ld_err, const void* U, int64_t ldu,
                      void* stream);

/* ---------------------------------------------------------------------------------------
 * AWQ (awq.py) and auto-clip (auto_clip.py) building blocks. dtype = BF16/F16/F32; each op
 * rounds to dtype like the reference's torch expressions.
 * ------------------------------------------------------------------------------------- */
/* calib_algo 'mse' (quant.py:145-203 get_mse_range, then get_qparams :545-559): per group of
 * `group` contiguous elements of x (rows groups), the shrink grid p = 1 - i / grid for
 * i < nsteps (= int(maxshrink * grid)) on the fp32 values, err = sum |qdq(x) - x|^norm, the
 * first strict minimum kept. Outputs fp32 [rows]: range_min, range_max, scales, zeros (asym;
 * may be NULL when sym). */
int lcq_mse_qparams(const void* x, int dtype, int64_t rows, int64_t group, int sym, int qmin,
                    int qmax, int nsteps, float grid, float norm, void* range_min,
                    void* range_max, void* scales, void* zeros, void* stream);

/* Workspace bytes of lcq_absmean_cols / lcq_awq_weight_scale for a [rows, cols] input. */
int64_t lcq_colmean_workspace_bytes(int64_t rows, int64_t cols);

/* Awq.get_act_scale (awq.py:74-85): out[c] = mean_t |x[t, c]| (x [n, c], c % 8 == 0), summed in
 * torch-CPU's exact order (its fp32 4-level cascade over rows, SumKernel.cpp; exact for
 * c % 64 == 0) and rounded like mean_out (fp32 sum / n -> dtype). */
int lcq_absmean_cols(const void* x, int dtype, int64_t n, int64_t c, void* out,
                     void* workspace, void* stream);

/* Awq.get_weight_scale (awq.py:48-72), one linear of the subset per call (layer = 0 ..
 * nlayers - 1, in the subset's order): |w| / max|w| per group of `group` columns (rounded to
 * dtype), mean over rows (same cascade as lcq_absmean_cols), accumulated into total [cols]
 * (dtype): layer 0 writes, later layers add (rounded), the last divides by nlayers.
 * group / 8 must be a power of two <= 64. */
int lcq_awq_weight_scale(const void* w, int dtype, int64_t rows, int64_t cols, int64_t group,
                         int layer, int nlayers, void* total, void* workspace, void* stream);

/* Awq.get_scales, trans_version v2 (awq.py:87-108): s = pow(x, ratio_dt) (exponent already
 * rounded to dtype by the caller, correctly rounded pow) ; clamp(min=1e-4) ;
 * s / sqrt(max(s) * min(s)). xmean, out [c]. */
int lcq_awq_scales(const void* xmean, int dtype, int64_t c, float ratio_dt, void* out,
                   void* stream);

/* Awq.get_scales, trans_version v1 (awq.py:87-108): s = pow(x, ratio_dt) / pow(wmax,
 * wexp_dt) (both exponents rounded to dtype by the caller: ratio and 1 - ratio), then as
 * lcq_awq_scales. wmax [c] from lcq_awq_weight_scale. */
int lcq_awq_scales_v1(const void* xmean, const void* wmax, int dtype, int64_t c,
                      float ratio_dt, float wexp_dt, void* out, void* stream);

/* Broadcast scale: out = x * s (op 0) or x / s (op 1), s per column (axis 0, [cols]) or per
 * row (axis 1, [rows]); in place allowed. Replaces scaling_input / update_input_feat /
 * scale_ln_fcs / scale_fc_fc / scaling_weight (base_blockwise_quantization.py:631-778,
 * 880-897; awq.py:39-46). */
int lcq_scale_bcast(const void* x, int dtype, int64_t rows, int64_t cols, const void* s,
                    int op, int axis, void* out, void* stream);

/* Awq.calculate_loss (awq.py:134-145): out_f32[slot] = fp32(sum((a-b)_dtype^2)) / n, fp64
 * partial sums in workspace (nparts doubles). Losses stay on device (no per-ratio sync). */
int lcq_sq_diff_mean(const void* a, const void* b, int dtype, int64_t n, void* workspace,
                     int nparts, void* out_f32, int slot, void* stream);

/* AutoClipper.auto_clip_layer, clip v1 (auto_clip.py:83-191) for bf16 / fp16 weights:
 * w [oc, ic], x [T, ic] (already token-subsampled), group 32 / 64 / 128 / 256, nsteps shrink
 * steps with factors[nsteps] = fp32(1 - i/n_grid) (device array). best_max / best_min
 * [oc, ic/group] in dtype. Exact emulation of the reference's dtype products and sums (VALU,
 * not MFMA). mse_steps > 0: the weight quantizer's calib_algo is mse -- every step's fake
 * quant searches its range (quant.py:145-203) with mse_p[mse_steps] = fp32(1 - i/mse_grid)
 * (device array) and the norm (2.4); mse_steps = 0: min/max qparams. */
int lcq_auto_clip_search(const void* w, const void* x, int dtype, int64_t oc, int64_t ic,
                         int64_t T, int group, int nsteps, const void* factors, int qmin,
                         int qmax, int sym, int clip_sym, int mse_steps, const void* mse_p,
                         float norm, void* best_max, void* best_min, void* stream);

/* lcq_auto_clip_search with activation fake-quant (w_only False: auto_clip.py:176-177,
 * fake_quantize_input at :269-274): the shrink steps multiply the weights with qx [T, ic] (the
 * aquantizer's fake_quant_act_dynamic of x viewed [1, T, ic/group, group]), the original
 * outputs with x. qx NULL == lcq_auto_clip_search. */
int lcq_auto_clip_search_act(const void* w, const void* x, const void* qx, int dtype, int64_t oc,
                             int64_t ic, int64_t T, int group, int nsteps, const void* factors,
                             int qmin, int qmax, int sym, int clip_sym, int mse_steps,
                             const void* mse_p, float norm, void* best_max, void* best_min,
                             void* stream);

/* lcq_auto_clip_search_act with a caller workspace of lcq_auto_clip_workspace_bytes(oc, ic, T,
 * group, nsteps) bytes (16-byte aligned; 0 = not applicable). Weight-only searches (qx NULL)
 * with group 128, min/max qparams and nsteps 10 tabulate the candidate weights of every
 * (row, step) once in the workspace (row chunks of at most 1 GiB) and then run: with T <= 512
 * sampled tokens, one lane per token, all T tokens in one workgroup, the candidate rows staged
 * in LDS (k_auto_clip_tw); above 512 tokens, below 65536 row-groups, one lane per token with the
 * candidates as scalar operands. Results are bit-identical to lcq_auto_clip_search_act, which
 * every other case (larger layers above 512 tokens, a workspace too small for 192 rows) runs. */
int64_t lcq_auto_clip_workspace_bytes(int64_t oc, int64_t ic, int64_t T, int group, int nsteps);
int lcq_auto_clip_search_ws(const void* w, const void* x, const void* qx, int dtype, int64_t oc,
                            int64_t ic, int64_t T, int group, int nsteps, const void* factors,
                            int qmin, int qmax, int sym, int clip_sym, int mse_steps,
                            const void* mse_p, float norm, void* best_max, void* best_min,
                            void* workspace, int64_t ws_bytes, void* stream);

/* A/B probe hook of lcq_auto_clip_search_ws (scripts/clip_rate.py): 0 = automatic, 1 = the
 * token-lane kernel with scalar-operand candidates at every size, 2 = the row-lane kernel (one
 * lane per weight row, tokens as scalar operands), 3 = k_auto_clip_tw (LDS candidates; T <= 512).
 * Process-wide; not for production use. */
int lcq_auto_clip_force_variant(int variant);

/* AutoClipper.auto_clip_layer for per_channel integer weights (group = ic, auto_clip.py:96-99;
 * awq_w8a8.yml): w [oc, ic] (ic % 128 == 0), x [T, ic] sampled tokens, qx [T, ic] their
 * activation fake-quant or NULL (weight-only), nsteps <= 10 with factors[nsteps] =
 * fp32(1 - i/n_grid) on device; best_max / best_min [oc] in dtype. Products rounded to dtype
 * like the reference's broadcast product; the ic-long fp32 sum runs in k order (parity tier
 * T2). workspace >= lcq_auto_clip_pc_workspace_bytes(oc, T, nsteps).
 * fmt 0: integer weights. fmt LCQ_FP8E4M3 / LCQ_FP8E5M2: FloatQuantizer weights (use_qtorch;
 * awq_fp8.yml / awq_fp8_static.yml): the candidates are fake_quant_weight_dynamic of the
 * clamped weights with the saturating float_quantize stand-in (quant.py:545-553, 1061-1080;
 * qmin / qmax / sym ignored). tensor_batch 0: per_channel scales (one per row); > 0:
 * per_tensor scale over each batch of tensor_batch rows, the reference's oc_batch_size
 * (auto_clip.py:108). version 1: clip_version v1 (the candidate is the clamped weight's
 * dynamic fake quant); 2 (integer only; awq_comb_omni w6a6 / w8a8 step_1_awq.yml, calib_algo
 * learnable): the candidate is the unclamped weight's static fake quant with the qparams of
 * get_learnable_range(w, logit(min_val / org_min), logit(max_val / org_max))
 * (auto_clip.py:258-267, quant.py:205-219). The returned bounds are the same kind in both. */
int64_t lcq_auto_clip_pc_workspace_bytes(int64_t oc, int64_t T, int nsteps);
int lcq_auto_clip_search_pc(const void* w, const void* x, const void* qx, int dtype, int64_t oc,
                            int64_t ic, int64_t T, int nsteps, const void* factors, int qmin,
                            int qmax, int sym, int clip_sym, int fmt, int tensor_batch,
                            int version, void* workspace, int64_t ws_bytes, void* best_max,
                            void* best_min, void* stream);

/* AutoClipper.apply_clip, v1 (auto_clip.py:193-212): out = clamp(x, cmin, cmax) per group;
 * cmin NULL -> -cmax. In place allowed. */
int lcq_clip_apply(const void* x, int dtype, int64_t rows, int64_t cols, int64_t group,
                   const void* cmax, const void* cmin, void* out, void* stream);

/* AutoClipper.get_clip_factor, v2 (auto_clip.py:213-256): per group of x [rows, cols] (group
 * | cols, group % 8 == 0) the logit factors of the searched bounds against the group's own
 * range, in dtype: clip_sym: up = logit(cmax / max(|max|, |min|).clamp(1e-5)), low not
 * written (the reference stores None); else up = logit(cmax / max), low = logit(cmin / min).
 * cmax / cmin / up / low: [rows * cols / group] in dtype (bf16 / fp16). */
int lcq_clip_factors(const void* x, int dtype, int64_t rows, int64_t cols, int64_t group,
                     const void* cmax, const void* cmin, int clip_sym, void* up_out,
                     void* low_out, void* stream);

/* ---------------------------------------------------------------------------------------
 * FP8 (FloatQuantizer, quant.py:963-1229; kernel.py:7-138; quant.py:18-43).
 * fmt = LCQ_FP8E4M3 (float8_e4m3fn) or LCQ_FP8E5M2. The fp8 rounding is
 * torch's native cast (c10 Float8_e4m3fn / Float8_e5m2, RNE); the reference's qtorch
 * float_quantize step is absent from this image, so that step is parity-unpinned.
 * ------------------------------------------------------------------------------------- */
/* Scratch (fp32 count) the per-tensor max reductions take: one partial per workgroup. */
#define LCQ_FP8_PARTIALS 256

/* max |x| over n elements -> out (one fp32 on device). Per-tensor get_minmax_range
 * (quant.py:133-135): max(|torch.max|, |torch.min|) == max|x|. workspace: LCQ_FP8_PARTIALS
 * device fp32 of scratch. */
int lcq_absmax(const void* x, int x_dtype, int64_t n, void* out, void* workspace, void* stream);

/* Dynamic FP8 quant over groups of `group` consecutive elements of x [rows, cols]
 * (per_group / per_channel / per_token; kernel.py act_quant = group 128, ct F32, clamp 0,
 * add_zero 0), or per tensor when tensor_amax (device fp32 from lcq_absmax) is given.
 * s = rnd_ct(max(amax, clamp_min) / qmax) (clamp skipped when clamp_min == 0; qmax = finfo.max
 * of the format, 448 / 57344, or the config's float_range; per tensor the division is fp32);
 * add_zero (quant.py quant()): s == 0 -> 1 and `+ 0` after the division;
 * code = cast(rnd_ct(x / s) [+ 0]); fq = rnd_fq(float(code) * s).
 * ct_dtype = x dtype (quant.py) or F32 (kernel.py). Any of codes_out (uint8 [rows, cols]),
 * fq_out, scales_out (ct dtype per group; one fp32 per tensor) may be NULL. */
int lcq_fp8_quant(const void* x, int x_dtype, int64_t rows, int64_t cols, int64_t group,
                  int fmt, int ct_dtype, float qmax, float clamp_min, int add_zero,
                  const void* tensor_amax, void* codes_out, void* fq_out, int fq_dtype,
                  void* scales_out, void* stream);

/* FP8 quant with given scales (fake/real_quant_*_static, quant.py:1061-1076, 1119-1159):
 * s = rnd_ct(scales[e / group]) (0 -> 1); same cast / fake-quant rules as lcq_fp8_quant.
 * ct_dtype = torch.promote_types(x, scales). saturate != 0 clamps the quotient to
 * +-finfo.max before the cast (FloatQuantizer's float_quantize stand-in: with given scales a
 * quotient can leave the format's range -- GPTQ's error-compensated columns, static act
 * scales -- where c10's cast would give NaN); 0 = torch's `.to()` exactly. */
int lcq_fp8_quant_static(const void* x, int x_dtype, int64_t rows, int64_t cols, int64_t group,
                         int fmt, int ct_dtype, const void* scales, int s_dtype, int add_zero,
                         int saturate, void* codes_out, void* fq_out, int fq_dtype,
                         void* stream);

/* 128x128-block FP8 quant of x [M, N] (N % 8 == 0): per_block FloatQuantizer (clamp_min 1e-5,
 * add_zero 1; quant.py:132-143, 636-641) and weight_cast_to_fp8 (kernel.py:57-81: clamp 0,
 * add_zero 0). scales_out fp32 [ceil(M/128), ceil(N/128)]; codes uint8 [M, N]. */
int lcq_fp8_quant_blocks(const void* x, int x_dtype, int64_t M, int64_t N, int block, int fmt,
                         float qmax, float clamp_min, int add_zero, void* codes_out, void* fq_out,
                         int fq_dtype, void* scales_out, void* stream);

/* weight_cast_to_bf16 (kernel.py:84-138, quant.py:18-31): out = rnd_out(float(code) *
 * scales[r / block][c / block]); codes uint8 [M, N], scales fp32 [ceil(M/b), ceil(N/b)]. */
int lcq_fp8_dequant_blocks(const void* codes, int fmt, int64_t M, int64_t N, int block,
                           const void* scales, void* out, int out_dtype, void* stream);

/* Deploy of a block-fp8 checkpoint weight to per-tensor fp8 (module_utils.py:917-922 +
 * quant.py:1191-1221): w = bf16(float(code) * scales_inv[block]) (weight_cast_to_bf16) kept in
 * registers, then per-tensor FloatQuantizer real quant of w (bf16 compute, fp32 scale).
 * amax_ws: LCQ_FP8_PARTIALS device fp32 of scratch. scale_out: one fp32. Bit-identical to the composed
 * lcq_fp8_dequant_blocks -> lcq_absmax -> lcq_fp8_quant chain at 3 instead of 8 B/element. */
int lcq_fp8_block_to_tensor(const void* codes, int fmt_in, int64_t M, int64_t N, int block,
                            const void* scales_inv, int fmt_out, float qmax, float clamp_min,
                            int add_zero, void* amax_ws, void* codes_out, void* scale_out,
                            void* stream);

/* Batched lcq_fp8_block_to_tensor over n weights (e.g. the 257 x 3 expert linears of a
 * DeepSeek-V3 MoE layer) in one launch pair. descs: device array of n records
 * {const uint8_t* codes; const float* scales_inv; uint8_t* codes_out; int64_t M, N} (40 B);
 * max_elems = the largest M*N; amax_ws: n * LCQ_FP8_PARTIALS device fp32 of scratch
 * (per-workgroup partial maxima, no atomics); scales_out: n fp32. */
int lcq_fp8_block_to_tensor_many(int n, const void* descs, int64_t max_elems, int fmt_in,
                                 int block, int fmt_out, float qmax, float clamp_min,
                                 int add_zero, void* amax_ws, void* scales_out, void* stream);

/* A/B probe hook of lcq_fp8_gemm's tile plan (scripts/fp8_gemm_rate.py): 0 = automatic (the
 * default), 1 = the <= 64-row 32x32x64 kernel, 128 / 256 = that 16x16x128 tile with the split-K
 * count the plan computes for it. Process-wide; not for production use. */
int lcq_fp8_gemm_force_plan(int plan);

/* Block-scaled FP8 GEMM (fp8_gemm, kernel.py:141-242, called by block_wise_fp8_forward_func,
 * module_utils.py:41-46, for LlmcFp8Linear / fp8_forward linears): a [M, K] e4m3 codes with
 * per-token 128-column scales a_s fp32 [M, K/128] (act_quant); b [N, K] e4m3 codes with
 * 128x128 block scales b_s fp32 [ceil(N/128), K/128]. c[m, n] = sum_kb (dot_kb(a[m], b[n]) *
 * a_s[m, kb]) * b_s[n/128, kb], fp32 accumulation, stored as c_dtype (LCQ_F32 / LCQ_BF16 /
 * LCQ_F16). K % 128 == 0; a / b 16-byte aligned. Short batches split K across workgroups when
 * `workspace` holds lcq_fp8_gemm_workspace_bytes(M, N, K) bytes of device memory (fp32
 * partials summed in split order: deterministic for a given M; the split count depends on M,
 * so a row's fp32 sum order -- not its value up to rounding -- can differ between batch
 * sizes); null / smaller workspace = no split. */
int64_t lcq_fp8_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);
int lcq_fp8_gemm(const void* a, const void* a_s, const void* b, const void* b_s, int64_t M,
                 int64_t N, int64_t K, void* c, int c_dtype, void* workspace, int64_t ws_bytes,
                 void* stream);

/* Grouped block-scaled FP8 GEMM: one launch for the G routed experts of an MoE projection
 * (replaces the per-expert block_wise_fp8_forward_func calls of the expert loop, reference
 * models/deepseekv3.py MoE forward -> module_utils.py:41-46 per expert; kernel.py:141-242 per
 * call). The `rows` GEMM rows are the token slots sorted by expert, group g's rows
 * [row_off[g], row_off[g + 1]) (row_off: DEVICE int64 [G + 1], so the routing is never read on
 * the host). a: e4m3 with a_s fp32 [.., K/128] (act_quant) -- `a_rows_total` rows, and sorted
 * row i is a row a_rows[i] (DEVICE int64 [rows]: the token gather happens inside the kernel,
 * act_quant runs once per token), or a_rows null and a already sorted (a_rows_total == rows).
 * wtab: DEVICE int64 [nsets][G][2] = (weight [N, K] e4m3 16-byte aligned, block scales fp32
 * [ceil(N/128), K/128]) addresses; nsets 1 or 2 (gate and up of the same rows in one launch).
 * c [nsets][rows][N] (c_dtype). Every row equals what lcq_fp8_gemm computes for it on an
 * unsplit 256^2 plan. silu_mul (nsets 2, c_dtype BF16): set 0 = gate, set 1 = up, and c
 * [rows][N] receives h = rnd(rnd(silu(rnd(gate))) * rnd(up)) (the expert MLP's
 * act_fn(gate_proj(x)) * up_proj(x) on its bf16 projections, which are never stored).
 * `workspace`: lcq_fp8_gemm_grouped_workspace_bytes(rows, G, silu_mul ? 2 N : N, K). */
int64_t lcq_fp8_gemm_grouped_workspace_bytes(int64_t rows, int64_t G, int64_t N, int64_t K);
int lcq_fp8_gemm_grouped(const void* a, const void* a_s, int64_t a_rows_total,
                         const int64_t* a_rows, int64_t rows, const int64_t* row_off,
                         const int64_t* wtab, int64_t G, int nsets, int silu_mul, int64_t N,
                         int64_t K, void* c, int c_dtype, void* workspace, int64_t ws_bytes,
                         void* stream);

/* MoE combine (the expert loop's `out.index_add_(0, tok, (h_e * w).to(out.dtype))` over hit
 * experts in ascending index; reference models/deepseekv3.py MoE forward): out [T, H] bf16,
 * out[t] = fold over token t's k slots in ascending expert[t k + j] of
 * acc = rnd(acc + rnd(y[slot_row[t k + j]] * w[t k + j])), acc from 0, rnd = bf16 RNE; y bf16
 * [.., H] (the grouped GEMM's sorted rows), w fp32 / bf16 (w_dtype) [T, k]; k <= 16,
 * H % 8 == 0, y / out 16-byte aligned. */
int lcq_moe_combine(const void* y, const int64_t* slot_row, const int64_t* expert,
                    const void* w, int w_dtype, int64_t T, int k, int64_t H, void* out,
                    void* stream);

/* Causal flash-attention forward of the calibration forwards (the sdpa call inside
 * LlamaAttention.forward, reached from awq.py:110-126 inspect forwards and the block forwards
 * of base_blockwise_quantization.py:367-381): out[b, s, h, :] = softmax(q k^T * scale, causal)
 * v with GQA (kv head = h / (H / KVH)). q/k/v bf16 viewed as [B, heads, S, 128] with element
 * strides {batch, head, seq} (host int64[3] each; head dim contiguous, strides multiples of 8,
 * 16-byte aligned); out bf16 [B, S, H, 128] contiguous. fp32 scores and online softmax,
 * bf16 P.V. One (batch, kv head)'s K / V rows must span < 2 GB (S * seq stride < 2^30
 * elements: 32-bit buffer offsets), else LCQ_EINVAL. */
int lcq_attn_fwd_causal(const void* q, const void* k, const void* v, int dtype, int64_t B,
                        int64_t S, int H, int KVH, int D, const int64_t* q_strides,
                        const int64_t* k_strides, const int64_t* v_strides, float scale,
                        void* out, void* stream);

/* FloatQuantizer use_qtorch=False fake quant (get_float_qparams, quant.py:1005-1027, and
 * quant/dequant :1061-1076): per group of `group` elements, power-of-two per-element scales
 * for an e_bits/m_bits float format; every op rounds to the tensor dtype (fp32 when
 * e_bits >= 5, quant.py:1014). */
int lcq_fp_emul_quant(const void* x, int x_dtype, int64_t rows, int64_t cols, int64_t group,
                      int e_bits, int m_bits, void* fq_out, int fq_dtype, void* stream);

/* ---------------------------------------------------------------------------------------
 * Calibration-forward fusions (the Llama block forward the reference runs through
 * transformers: modeling_llama.apply_rotary_pos_emb / LlamaMLP.forward, llmc/models/llama.py).
 * ------------------------------------------------------------------------------------- */
/* q' = q*cos + rotate_half(q)*sin and the same for k, per-op rounding in dtype (bit-identical
 * to the unfused torch ops). q [B, S, Hq, D], k [B, S, Hk, D] contiguous (the projection
 * outputs before the head transpose); cos / sin [*, S, D] with batch stride cos_bstride
 * (0 = broadcast). D % 16 == 0. Outputs have the q / k layout. */
int lcq_rotary(const void* q, const void* k, const void* cos, const void* sin, int dtype,
               int64_t B, int64_t S, int Hq, int Hk, int D, int64_t cos_bstride, void* out_q,
               void* out_k, void* stream);

/* out = rnd(rnd(g / (1 + exp(-g))) * u): act_fn(gate_proj(x)) * up_proj(x) with SiLU. */
int lcq_silu_mul(const void* gate, const void* up, int dtype, int64_t n, void* out,
                 void* stream);

/* LlamaRMSNorm.forward: out = weight * rnd(x_f32 * rsqrt(mean(x_f32^2) + eps)), one pass per
 * row (the row read once, held in registers); x, out [rows, H] contiguous, weight [H] (same
 * dtype), H % 8 == 0, H <= 16384. */
int lcq_rmsnorm(const void* x, const void* weight, int dtype, int64_t rows, int64_t H,
                float eps, void* out, void* stream);

/* ---------------------------------------------------------------------------------------
 * Static activation calibration (per-tensor, `act: {static: True}`): register_act_qparams
 * (base_blockwise_quantization.py:567-588) -> get_batch_tensors_qparams (quant.py:561-586).
 * ------------------------------------------------------------------------------------- */
/* Scratch (float2 count) per launch of lcq_minmax_segments: LCQ_MINMAX_SEGS segments at a time,
 * at most LCQ_MINMAX_PARTS workgroups each. */
#define LCQ_MINMAX_PARTS 32
#define LCQ_MINMAX_SEGS 64
#define LCQ_MINMAX_WORKSPACE (LCQ_MINMAX_PARTS * LCQ_MINMAX_SEGS)

/* torch.min / torch.max of each of nseg device tensors (segs[i]: host array of device pointers,
 * 16-byte aligned, seg_lens[i] > 0 elements, dtype F32 / F16 / BF16), NaN-propagating like torch:
 * get_minmax_stats (quant.py:221-251) on per_tensor ranges (quant.py:132-135). minmax: device
 * fp32 [2 * nseg] = (min, max) per segment, exact. workspace: LCQ_MINMAX_WORKSPACE device
 * float2. */
int lcq_minmax_segments(const void* const* segs, const int64_t* seg_lens, int64_t nseg,
                        int dtype, void* minmax, void* workspace, void* stream);

#define LCQ_CALIB_STATIC_MINMAX 0        /* quant.py:253-262: mean of the per-segment ranges */
#define LCQ_CALIB_STATIC_MOVING_MINMAX 1 /* quant.py:431-450: EMA (alpha) in the range dtype */

/* Static per-tensor qparams from lcq_minmax_segments' ranges: the range (static_minmax: fp32
 * means, sum then / nseg; static_moving_minmax: m += alpha * (v - m) with every op rounded to
 * range_dtype), then get_qparams (quant.py:545-559) with torch's 0-dim type promotion: the
 * scale (and zero) computed in / rounded to scale_dtype (the caller's promote(range dtype,
 * qmax [- qmin] dtype)). out: device fp32 [4] = scale, zero, min, max (each exactly
 * representable in its dtype). */
int lcq_act_static_qparams(const void* minmax, int64_t nseg, int algo, float alpha,
                           int range_dtype, int scale_dtype, int sym, float qmin, float qmax,
                           void* out, void* stream);

/* static_hist (quant.py:264-529, get_static_hist_range + get_qparams, sym per-tensor int):
 * per-segment torch.histc(x.float(), 2048, running min, running max) (exact counts), the
 * reference's sequential histogram combination (upscale x16 + bucketize + bincount), the
 * quantile-walk / L2-error threshold search, then scale = max(|min|, |max|) / qmax. segs as
 * for lcq_minmax_segments; minmax: its output for the same segments; dst_nbins = 2^bit.
 * out: device fp32 [4] = scale, 0, new_min, new_max. workspace: lcq_act_hist_workspace_bytes. */
int64_t lcq_act_hist_workspace_bytes(int64_t nseg);
int lcq_act_static_hist_qparams(const void* const* segs, const int64_t* seg_lens, int64_t nseg,
                                int dtype, const void* minmax, int dst_nbins, float qmax,
                                void* out, void* workspace, void* stream);

/* ---------------------------------------------------------------------------------------
 * Projection GEMMs of the calibration / AWQ loss-search forwards (awq.py:110-145, 178-278:
 * the nn.Linear calls inside inspect_module, and calculate_loss) on bf16/fp16 MFMA
 * (csrc/gemm256.hip). A [m, k] (row stride lda), weights [rows, k] (row stride ldb, the
 * nn.Linear layout); k % 64 == 0; strides multiples of 8 elements; fp32 accumulation, each
 * output rounded once to dtype (bias added in fp32 first).
 *
 * lcq_gemm: C_s = A . B_s^T (+ bias_s) for nseg (1..3) weight segments B_s [b_rows[s], k]
 * written to c[s] [m, b_rows[s]] (row stride ldc[s]) -- q / k / v of one input in one launch.
 * All segments but the last are multiples of 256 rows; bias may be NULL or hold NULLs.
 * ------------------------------------------------------------------------------------- */
int lcq_gemm(const void* a, int dtype, int64_t lda, int64_t m, int64_t k, int nseg,
             const void* const* b, const int64_t* b_rows, int64_t ldb, const void* const* bias,
             void* const* c, const int64_t* ldc, void* stream);

/* lcq_gemm with transformers' apply_rotary_pos_emb (models/llama/modeling_llama.py; the
 * calibration forward of LlamaAttention, base_blockwise_quantization.py:367-381, and the AWQ
 * inspect forward of the q/k/v subset, awq.py:110-126) fused into the epilogue: the first
 * rope_segs segments (q, k: multiples of 256 rows, heads of head_dim 128) are written as
 * rnd(rnd(x cos) + rnd(rotate_half(x) sin)) of their rounded outputs x -- bit-identical to
 * lcq_gemm followed by lcq_rotary. cos / sin [1 or B, seq, 128] in dtype, batch stride
 * cs_bstride (0: shared); m = B * seq rows, token row t at position t % seq. */
int lcq_gemm_rope(const void* a, int dtype, int64_t lda, int64_t m, int64_t k, int nseg,
                  const void* const* b, const int64_t* b_rows, int64_t ldb,
                  const void* const* bias, void* const* c, const int64_t* ldc, int rope_segs,
                  const void* cos, const void* sin, int64_t seq, int64_t cs_bstride,
                  int64_t head_dim, void* stream);

/* C = rnd(res + rnd(A B^T + bias)) (one segment): the decoder block's `residual + o_proj(x)`
 * and `h + down_proj(m)` (transformers LlamaDecoderLayer.forward, the calibration forwards of
 * base_blockwise_quantization.py:367-381) with the add in the GEMM epilogue. res [M, N] (ldr),
 * c [M, N] (ldc). */
int lcq_gemm_residual(const void* a, int dtype, int64_t lda, int64_t m, int64_t k, const void* b,
                      int64_t ldb, int64_t n, const void* bias, const void* res, int64_t ldr,
                      void* c, int64_t ldc, void* stream);

/* LlamaMLP's act_fn(gate_proj(x)) * up_proj(x) (SiLU) in one GEMM: h [m, n] =
 * rnd(rnd(silu(rnd(A . gate^T))) * rnd(A . up^T)); gate / up [n, k]; the two [m, n]
 * projections are never written. */
int lcq_gemm_silu_mul(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                      const void* gate, const void* up, int64_t ldb, int64_t n, void* h,
                      int64_t ldh, void* stream);

/* Awq.calculate_loss fused into the last projection of inspect_module: out = rnd(A . B^T +
 * bias) is not written; out_f32[slot] = fp32(sum((ref - out)_dtype^2)) / (m * n), fp64 partial
 * per 256x256 tile summed in tile order (deterministic). ref [m, n] (row stride ldr) = the
 * original module output. workspace >= lcq_gemm_sq_diff_workspace_bytes(m, n). */
int64_t lcq_gemm_sq_diff_workspace_bytes(int64_t m, int64_t n);
int lcq_gemm_sq_diff(const void* a, int dtype, int64_t lda, int64_t m, int64_t k,
                     const void* b, int64_t ldb, int64_t n, const void* bias, const void* ref,
                     int64_t ldr, void* workspace, int64_t ws_bytes, void* out_f32, int slot,
                     void* stream);

#ifdef __cplusplus
}
#endif

#endif /* LCQ_H_ */
