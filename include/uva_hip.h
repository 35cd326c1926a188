/*
 * libuva_hip.so -- C ABI of the MI355X (gfx950) kernels behind the UVA training step.
 *
 * Drop-in boundary: the reference has no native code; every entry point below
 * replaces an implicit PyTorch/cuBLAS/cuDNN/SDPA kernel on the path
 * TrainUnifiedVideoActionWorkspace.run -> UnifiedVideoActionPolicy.compute_loss ->
 * get_vae_latent / MAR.forward -> backward -> AdamW/EMA.  The reference call site each
 * one replaces is cited per function (paths relative to the reference repo root).
 *
 * Conventions (all entry points):
 *  - plain device pointers + sizes; the caller owns every allocation (no allocation on
 *    the hot path); workspaces are sized by the matching *_workspace() query.
 *  - dtype codes: 0 = fp32, 1 = bf16.  Accumulation is always fp32.
 *  - launches go to `stream` (the caller's current HIP stream); no host sync inside.
 *  - return value: 0 or a hipError_t code (the Python host layer raises on non-zero).
 */
#ifndef UVA_HIP_H
#define UVA_HIP_H
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UVA_DT_F32 0
#define UVA_DT_BF16 1
#define UVA_ACT_NONE 0
#define UVA_ACT_GELU 1
#define UVA_ACT_SILU 2
#define UVA_ACT_RELU 3

/* ---- dense contractions ------------------------------------------------------------
 * C[z] = epi(alpha * opA[z] (MxK) . opB[z]^T (NxK)) ; ta/tb select stored layouts
 * (ta=0: A[M][K], ta=1: A[K][M]; tb=0: B[N][K], tb=1: B[K][N]).  Batch z = zo*inner+zi
 * with outer/inner strides.  Epilogue order: +bias[n] -> aux=pre-act -> act -> dropout
 * (counter hash, p, seed) -> +residual -> +beta*C_old.  act = 16 + ACT kind selects the
 * activation BACKWARD: no forward activation and the residual operand is the saved
 * pre-activation, multiplied in as act'(pre) instead of added (GELU/dropout backward of
 * timm Mlp fused into the fc2 dX product, mar_con_unified.py:201-249).
 * Replaces: every nn.Linear fwd/bwd (timm Block qkv/proj/fc1/fc2
 * mar_con_unified.py:201-249; z_proj/z_proj_cond/proj_cond_x_layer/decoder_embed
 * :92-95,185-187,218; SimpleMLPAdaLN diffusion_loss.py:219-283; DiffActLoss fc/refine
 * diffusion_action_loss.py:49-61), torch.bmm of vae/vaekl.py:143-157, and the fp32
 * materialised form of F.scaled_dot_product_attention. */
int uva_gemm(int in_dtype, int out_dtype, int ta, int tb, const void* A, const void* B, void* C, int M, int N,
             int K, long long lda, long long ldb, long long ldc, int batch, int batch_inner, long long sAo,
             long long sAi, long long sBo, long long sBi, long long sCo, long long sCi, const float* bias,
             const void* residual, long long ldr, long long sRo, long long sRi, void* aux, int act, float alpha,
             float beta, float drop_p, unsigned long long drop_seed, int res_dtype, const void* gate,
             long long ldg, int gate_dtype, int force_generic, float* workspace, long long ws_floats,
             hipStream_t stream);
/* res_dtype: dtype of `residual`; gate (dtype gate_dtype, ld ldg) multiplies the value after
 * dropout and before the residual add (adaLN: x + gate * mlp(h), diffusion_loss.py:163-167). */
/* workspace (fp32, ws_floats) enables deterministic split-K for few-tile / long-K products
 * (the dW GEMMs, K = tokens); pass NULL/0 to disable.  Every product runs on this library's own
 * kernels (no vendor BLAS is linked). */

/* ---- convolution as implicit GEMM over NHWC (bf16: MFMA, fp32: VALU) -----------------
 * out[n,oh,ow,co] = bias[co] + residual + sum_{kh,kw,ci} act(in[n,ih,iw,ci]) w[co][kh][kw][ci]
 * with ih = oh*stride + kh - pad_t (zero outside), act = GroupNorm-apply + SiLU when
 * gn_scale/gn_shift ([Nimg][Ci] fp32) are given (SiLU only if gn_silu); `act` applies to the
 * output before the residual add.  Ci % 8 == 0 for the MFMA path.
 * Replaces nn.Conv2d (+ the preceding Normalize/nonlinearity) of the KL-VAE encoder
 * (vae/vaekl.py:36-113,116-159,162-273,469) and DiffActLoss.conv (diffusion_action_loss.py:42-46). */
/* Which kernel a bf16 GEMM of this shape runs on (test / tuning introspection; no device work):
 * kernel | BN << 4 | splits << 16; kernel 0 = VALU, 1 = MFMA register-staged 128x128,
 * 2 = MFMA LDS-DMA 128x128, 3 = MFMA 8-phase (256x256 or 128x384 tiles), splits = split-K slices. */
long long uva_gemm_plan(int in_dtype, int ta, int tb, int M, int N, int K, int batch, int gn_prologue,
                        long long ws_floats);
/* Persistent 8-phase form (gemm_8pp: one workgroup per CU walks full tiles; the next tile's first
 * K-tiles are in flight under this tile's register epilogue) for eligible plain / bias / activation /
 * dropout products: 1 on, 0 off (default: measured 1-4 % slower than gemm_8ph),
 * -1 query.  Returns the previous setting. */
int uva_gemm_set_persist(int on);
/* Persistent 4-wave GEMM (gemm4.hip: one workgroup of 4 waves per CU, 256 x 192 block tiles, 128 x 96
 * per wave with AGPR accumulators, a 2-region LDS-DMA ring of 64-deep K-tiles read as two 32-deep
 * substeps, register epilogue through buffer stores).  uva_gemm routes to it
 *   - the K-contiguous (ta = tb = 0) products with a bias-only epilogue, batch 1, K % 128 == 0: the timm
 *     Block qkv / fc1 / fc2 forwards and the dX products through transposed weight copies
 *     (mar_con_unified.py:201-249);
 *   - the fp32 dW products (ta = tb = 1, plain epilogue incl. beta, K = tokens % 128 == 0): (tile,
 *     K-slice) work items writing fp32 partial slabs into the split-K workspace, reduced in slice order
 *     (deterministic) by the same reduce as the other split-K paths.
 * uva_gemm4_set(on, force): measurement switch (tests / tools): on = 0 sends those products back to the
 * 8-phase kernel; force = tile configuration (1: 256x192; -1 automatic); -2 leaves a value unchanged;
 * returns the previous (on | (force + 1) << 1).
 * uva_gemm4_plan: cfg | grid << 8 the dispatcher would launch for a K-contiguous product, -1 = not
 * eligible; uva_gemm4_plan_tt: splits | grid << 8 for a dW product with ws_floats of workspace, -1 = not
 * eligible (no device work). */
int uva_gemm4_set(int on, int force);
/* Persistent 8-wave GEMM (gemm8w.hip: two waves per SIMD, 64 x 96 or 64 x 64 per wave, the gemm_4w ring /
 * DMA / substep schedule, column-major MFMA order with single-buffered B fragments) whose epilogue can be
 * DEFERRED into the next tile's first substeps (outputs packed to bf16, one fragment row per even substep,
 * beside the partner wave's MFMAs).
 * uva_linear_gelu_drop: the timm Mlp fc1 forward (mar_con_unified.py:236-249, Mlp.fc1 -> GELU -> drop) in
 *      one launch: pre_out = bf16(X W^T + b) (the GELU input the backward keeps), out = bf16(drop(gelu(pre)))
 *      -- bit-identical to the bias-only GEMM + uva_act_drop_fwd (same counter-hash mask on the flat index).
 * uva_linear_drop_res: Mlp.fc2 -> drop (+ the Block's residual add, :247-249): out (fp32) = R +
 *      drop(bf16(X W^T + b)) -- bit-identical to the bias-only GEMM + uva_act_drop_fwd(residual).
 *      Both: X [M][K], W [N][K] bf16 (K-contiguous), bias fp32 [N], contiguous outputs; 1 = launched,
 *      0 = shape not eligible (M >= 256, N >= 192, K % 128 == 0, K >= 256, 16-B aligned), < 0 = -hipError.
 * uva_gemm8w_try: a plain (bias) product on this kernel when switched on by uva_gemm8w_set(on, mode)
 *      (measurement: mode bit 0 deferred epilogue, bit 1 64 x 64 wave tiles); uva_gemm routes its plain
 *      K-contiguous products here first while on.  Returns the previous on | mode << 1; -2 keeps a value. */
int uva_gemm8w_set(int on, int mode);
int uva_linear_gelu_drop(const void* X, const void* W, const float* bias, void* pre_out, void* out, int M, int N, int K,
                         float drop_p, unsigned long long seed, const void* plane, hipStream_t stream);
int uva_linear_drop_res(const void* X, const void* W, const float* bias, const float* R, float* out, int M, int N,
                        int K, float drop_p, unsigned long long seed, const void* plane, hipStream_t stream);
/* uva_linear_dgelu_drop: the timm Mlp backward through fc2 -> dropout -> GELU in fc2's dX product:
 *      dpre = bf16(gelu'(pre) * drop(bf16(dY Wt^T))) -- bit-identical to the dX GEMM + uva_act_bwd_bias --
 *      and dbias (+)= the column sums of dpre (fc1's bias gradient: per-64-row partials in `part`,
 *      ((M + 255) / 256) * 4 * N floats, reduced by a second launch; the sums of the same stored values in
 *      another order than uva_act_bwd_bias).  dY [M][K], Wt [N][K] (fc2's transposed weight), pre / dpre
 *      [M][N] bf16 (replaces autograd of mar_con_unified.py:236-249 Mlp fc1 -> GELU -> drop -> fc2). */
int uva_linear_dgelu_drop(const void* dY, const void* Wt, const void* pre, void* dpre, float* dbias, int accum_bias,
                          float* part, int M, int N, int K, float drop_p, unsigned long long seed, const void* plane,
                          hipStream_t stream);
/* Dropout keep-bit planes: bit (i & 31) of u32 word i >> 5 = keep decision of flat element i under (drop_p,
 * seed) -- the same counter-hash mask every dropout kernel here evaluates (common.h dropout_keep).  The
 * fused Mlp GEMMs above take one as `plane` (non-null: test a bit instead of hashing per element in the
 * epilogue; N % 32 == 0, drop_p > 0), so the mask of a Block's fc1 / fc2 / proj dropout is computed once per
 * step, off the GEMMs (mar_con_unified.py:236-249 Mlp.drop, :201-215 proj_drop).  words = ceil(n / 32). */
/* LayerNorm backward of the timm Block's norm2 (mar_con_unified.py:236-249; fp32 x / dx, bf16 dy, D = 768,
 * affine, dx = dx_base + LN'(dy)) that also writes drop_out = bf16(drop(dx)) and adds the column sums of those
 * stored values to dbias: the backward of proj_drop and the attention proj's bias gradient (:201-215) in
 * the same pass, instead of a second pass (uva_act_bwd_bias, act none) over the fp32 dx.  workspace: 3 *
 * ceil(rows / 64) * D floats.  Other shapes / forms: hipErrorInvalidValue. */
int uva_layernorm_bwd_drop(const float* x, const float* w, const void* dy, const float* mean, const float* rstd,
                           const float* dx_base, float* dx, float* dw, float* db, int accum_wb, void* drop_out,
                           float drop_p, unsigned long long seed, float* dbias, int accum_dbias, float* workspace,
                           int rows, int D, hipStream_t stream);
long long uva_dropout_plane_words(long long n);
int uva_dropout_plane(void* plane, long long n, float drop_p, unsigned long long seed, hipStream_t stream);
long long uva_gemm4_plan(int M, int N, int K);
long long uva_gemm4_plan_tt(int M, int N, int K, long long ws_floats);
int uva_conv2d(int dtype, const void* in, const void* w, void* out, const float* bias, const void* residual, int Nimg,
               int Hin, int Win, int Ci, int Co, int ks, int stride, int pad_t, int pad_l, int Hout, int Wout,
               const float* gn_scale, const float* gn_shift, int gn_silu, int act, float* gn_part,
               int force_generic, hipStream_t stream);
/* Direct 3x3/s1/p1 conv with the input halo staged once per 64-channel chunk in LDS and the
 * GroupNorm-apply(+SiLU) prologue fused into that staging (ResnetBlock conv1/conv2,
 * vaekl.py:56-113 incl. Normalize+swish :94-104).  uva_conv2d routes eligible shapes here;
 * _bn returns the output-channel tile (0 = shape not eligible: H, W % 16, Ci % 64, Co % 128). */
/* ---- conv_fc action trunk row kernels (action_head.hip; diffusion_action_loss.py:42-61) -----
 * uva_pool4x4_cwh: AdaptiveAvgPool2d((4,4)) of NHWC [n][16][16][C] + flatten (c w h) -> [n][16 C].
 * uva_pool4x4_relu_bwd: dpre[n][16][16][C] = (post > 0) * gpool[n][16 c + cell] / 16 (the backward
 *      of ReLU -> mean-pool; post = the forward's post-ReLU conv output, gpool any of bf16 / fp32).
 * uva_im2col3x3: cols[n H W][9 Ci] with column ci*9 + kh*3 + kw (nn.Conv2d weight order), zero pad 1.
 * uva_im2col3x3_tc: the same columns in tap-major order, tap*Ci + ci (16-B vector moves; Ci % 8 for
 *      bf16, % 4 for fp32; 16-B aligned).  Both im2col forms stay exported for hosts that want the
 *      materialised columns; the training step's trunk dW uses uva_pad_nhwc below (no 9x tensor).
 *      The tap-major dW partial [Co][9][Ci] is added into the nn.Conv2d-layout fp32 gradient
 *      [Co][Ci][3][3] by uva_conv3x3_dw_scatter_add.
 * uva_conv3x3_weight_layout: fp32 [Co][Ci][3][3] -> mode 0 [Co][3][3][Ci] (forward conv operand),
 *      mode 1 [Ci][3][3][Co] flipped (the dX conv), out_dtype bf16 / fp32. */
int uva_pool4x4_cwh(int dtype, const void* in, void* out, int n, int C, hipStream_t stream);
int uva_pool4x4_relu_bwd(int dtype, const void* post, int gdtype, const void* gpool, void* dpre, int n, int C,
                         hipStream_t stream);
int uva_im2col3x3(int dtype, const void* in, void* cols, int n, int H, int W, int Ci, hipStream_t stream);
int uva_im2col3x3_tc(int dtype, const void* in, void* cols, int n, int H, int W, int Ci, hipStream_t stream);
/* uva_pad_nhwc: [n][H][W][C] -> [G + n (H+2) (W+2) + G][C], zero 1-pixel border and G zero guard rows
 *      at each end: with dY and X both padded, the weight gradient of a 3x3 / p1 conv is 9 plain GEMMs
 *      dW[:, tap, :] = dYp^T Xp(shifted by (kh-1)(W+2) + (kw-1) rows), G >= W + 3 (no im2col). */
int uva_pad_nhwc(int dtype, const void* in, void* out, int n, int H, int W, int C, int G, hipStream_t stream);
int uva_conv3x3_dw_scatter_add(const float* part, float* grad, int Co, int Ci, hipStream_t stream);
int uva_conv3x3_weight_layout(const float* w, int out_dtype, void* out, int Co, int Ci, int mode, hipStream_t stream);
int uva_conv3x3_halo_bn(int Nimg, int H, int W, int Ci, int Co);
int uva_conv3x3_halo(const void* in, const void* w, void* out, const float* bias, const void* residual, int Nimg,
                     int H, int W, int Ci, int Co, const float* gn_scale, const float* gn_shift, int gn_silu,
                     float* gn_part, hipStream_t stream);
/* Downsample (vaekl.py Downsample with_conv: F.pad(x, (0, 1, 0, 1)) then 3x3 / stride 2 / pad 0) as a
 * halo-tile kernel: NHWC bf16 [Nimg][Hin][Win][Ci] -> [Nimg][Hin/2][Win/2][Co], bias, optional fused
 * GN partials of the output.  uva_conv3x3s2_ok: Hin % 16, Win % 32, Ci % 64, Co % 128 == 0.
 * uva_conv2d routes 3x3/s2/p0 with Hout == Hin/2 (the implicit bottom/right zero pad) here. */
int uva_conv3x3s2_ok(int Nimg, int Hin, int Win, int Ci, int Co);
int uva_conv3x3s2_halo(const void* in, const void* w, void* out, const float* bias, int Nimg, int Hin, int Win,
                       int Ci, int Co, float* gn_part, hipStream_t stream);
/* Encoder.conv_in (vaekl.py:246-249) on the 8-channel padded frame -> 128 channels, bf16, bias, optional
 * fused GN partials; H, W % 16 == 0.  uva_conv2d routes Ci == 8, Co == 128 3x3/s1/p1 here. */
int uva_conv_in8(const void* in, const void* w, void* out, const float* bias, int Nimg, int H, int W,
                 float* gn_part, hipStream_t stream);
/* gn_part (bf16 MFMA path): the epilogue also writes per-(128-row tile, group) (sum, sumsq) of
 * the stored output for the NEXT GroupNorm(32) -> uva_groupnorm_finalize_tiles.  Needs
 * (Hout*Wout) % 128 == 0, Co % 32 == 0; buffer [M/128][32][2] floats. */

/* ---- LayerNorm (affine or adaLN-modulated) --------------------------------------------
 * Replaces nn.LayerNorm(eps=1e-6) (mar_con_unified.py:198,215,252; timm norm1/norm2)
 * and modulate(LN(x), shift, scale) (diffusion_loss.py:93-94,163-189). */
int uva_layernorm_fwd(int in_dtype, int out_dtype, const void* x, const float* w, const float* b, const void* scale,
                      const void* shift, long long ldm, void* y, float* mean, float* rstd, int rows, int D, float eps,
                      hipStream_t stream);
/* dy: dy_dtype fp32 or bf16 (the consuming GEMM's bf16 dX, autocast semantics) */
int uva_layernorm_bwd(int in_dtype, int out_dtype, const void* x, const float* w, const float* b, const void* scale,
                      long long ldm,
                      const void* dy, int dy_dtype, const float* mean, const float* rstd, const float* dx_base, float* dx,
                      int accum, void* dscale,
                      void* dshift, float* dw, float* db, int accum_wb, float* workspace, int rows, int D,
                      hipStream_t stream);
long long uva_layernorm_bwd_workspace(int rows, int D); /* floats */

/* column sums (bias gradients) */
int uva_colsum(int dtype, const void* in, long long ld, float* out, int rows, int cols, int accum, float* workspace,
               hipStream_t stream);
long long uva_colsum_workspace(int rows, int cols); /* floats */

/* ---- softmax rows (materialised attention: fp32 parity path, VAE AttnBlock) ----------
 * Replaces softmax inside F.scaled_dot_product_attention (timm Attention) and
 * torch.nn.functional.softmax of vaekl.py:150. */
int uva_softmax_fwd(int dtype, const void* S, void* P, void* Pd, long long rows, int L, float scale, float drop_p,
                    unsigned long long seed, hipStream_t stream);
int uva_softmax_bwd(int dtype, const void* P, const void* dPd, void* dS, long long rows, int L, float scale,
                    float drop_p, unsigned long long seed, hipStream_t stream);

/* ---- elementwise ----------------------------------------------------------------------- */
int uva_cast(int sdt, const void* src, long long lds, int ddt, void* dst, long long ldd, long long rows, int cols,
             hipStream_t stream);
int uva_act_fwd(int xdt, const void* x, int ydt, void* y, long long n, int act, hipStream_t stream);
/* dst[c][r] = src[r][c], bf16 [rows][cols] (rows, cols % 8 == 0, 16-B aligned): the transposed bf16
 * weight copies of the Block's width-768 dX products (functional.py compute_weight_t). */
int uva_transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t stream);
/* y = residual + dropout(act(x)) over n contiguous elements (n % 8 == 0, 16-B aligned), dropout
 * index = flat element index (the GEMM epilogue's / uva_act_bwd's mask).  timm Mlp forward
 * (mar_con_unified.py:201-249: fc1 -> GELU -> drop, fc2 -> drop -> + residual) when fc1 / fc2 run
 * as bias-only GEMMs.  (xdt, ydt, rdt) in {(bf16, bf16, bf16), (bf16, f32, f32), (f32, f32, f32)}. */
int uva_act_drop_fwd(int xdt, const void* x, int ydt, void* y, int rdt, const void* residual, long long n, int act,
                     float drop_p, unsigned long long seed, hipStream_t stream);
int uva_act_bwd(int pdt, const void* pre, int gdt, const void* dy, long long ld_dy, int xdt, void* dx,
                long long ld_dx, long long rows, int cols, int act, float drop_p, unsigned long long seed, int accum,
                hipStream_t stream);
/* act_bwd fused with the bias gradient: dbias[c] (+)= sum_r dx[r][c] (the values as stored);
 * the nn.Linear bias grad of timm Mlp fc1/fc2 and Attention proj (mar_con_unified.py:201-249),
 * SimpleMLPAdaLN res-block linears (diffusion_loss.py:142-167).  cols % 8 == 0, 16-B aligned
 * operands; workspace: uva_act_bwd_bias_workspace(rows, cols) floats. */
int uva_act_bwd_bias(int pdt, const void* pre, int gdt, const void* dy, long long ld_dy, int xdt, void* dx,
                     long long ld_dx, long long rows, int cols, int act, float drop_p, unsigned long long seed,
                     int accum, float* dbias, int accum_bias, float* workspace, hipStream_t stream);
long long uva_act_bwd_bias_workspace(long long rows, int cols); /* floats */
int uva_gate_bwd(const float* dout, int hdt, const void* h, int gtdt, const void* gate, long long ldg, int dhdt,
                 void* dh, void* dgate, long long rows, int cols, hipStream_t stream);
int uva_fill(float* p, long long n, float v, hipStream_t stream);

/* ---- diffusion loss (gaussian_diffusion.py:220-236, 713-818; diffusion_utils.py:10-73;
 *      diffusion_loss.py:44-66, 111-134; diffusion_action_loss.py:147-166) ---------------
 * tables: 8 device fp32 arrays [T]: sqrt_ac, sqrt_1mac, coef1, coef2, plvc, log_betas,
 * sqrt_recip_ac, sqrt_recipm1_ac (host array of device pointers). */
int uva_q_sample(const float* x0, const float* noise, const long long* t, const float* const* tables, int xdt,
                 void* xt, int rows, int C, hipStream_t stream);
int uva_timestep_features(const long long* t, const float* freqs, int odt, void* out, int rows, int half,
                          hipStream_t stream);
int uva_diffusion_loss(const float* x0, const float* noise, const long long* t, int odt, const void* out,
                       long long ld_out, const float* const* tables, float* loss_row, float* dl, int rows, int C,
                       hipStream_t stream);
int uva_weighted_mean(const float* l, const float* w, int n, float* res, hipStream_t stream);
int uva_loss_grad(const float* dl, const float* w, const float* wsum, const float* g_up, int ddt, void* dout,
                  long long ld, int rows, int C2, hipStream_t stream);

/* ---- diffusion sampler step (gaussian_diffusion.py:260-346,395-440; respace.py:65-130;
 *      diffusion_action_loss.py:168-232 DiffActLoss.sample) --------------------------------
 * out: net output [rows, ld_out] (eps | var_values, 2C columns), x/noise/x_new: fp32 [rows, C]
 * (x_new may alias x), coef: HOST array of 8 floats {sqrt_recip_ac, sqrt_recipm1_ac, coef1,
 * coef2, min_log (posterior_log_variance_clipped), max_log (log beta), nonzero (t != 0),
 * temperature} of the step's spaced timestep; x_net (nullable): x_new in dtype xdt; clip: clip_denoised
 * (1 for the action head, diffusion_action_loss.py:218; 0 for the video head, diffusion_loss.py:84). */
int uva_p_sample_step(int odt, const void* out, long long ld_out, const float* x, const float* noise,
                      const float* coef, float* x_new, int xdt, void* x_net, int clip, int rows, int C,
                      hipStream_t stream);

/* ---- few-row fused linear of the action sampler (inference, bf16; diffusion_loss.py:142-189)
 * out[R,N] = epi(A' W^T + bias), W bf16 [N,K] (K in {256, 512, 1024}), R any.
 * ln = 1: A = fp32 residual rows x [R, lda]; A' = (LN(x)[*lnw + lnb]) * (1 + scale) + shift
 *         (lnw/lnb nullable; shift/scale bf16 columns of the adaLN modulation, row stride ldm).
 * ln = 0: A' = A bf16 [R, lda].  act: 0 or 2 (SiLU).  gate/res (both or neither, fp32 out):
 * out = res + gate * v.  Supported: (ln, SiLU, bf16 out), (ln, none, fp32 out),
 * (plain, gate, fp32 out), (plain, SiLU, bf16 out). */
int uva_sampler_linear(int ln, const void* A, long long lda, const float* lnw, const float* lnb, const void* shift,
                       const void* scale, long long ldm, float eps, const void* W, const float* bias, int act,
                       const void* gate, long long ldg, const float* res, long long ldr, int odt, void* out,
                       long long ldo, int R, int N, int K, hipStream_t stream);

/* ---- persistent action sampler (inference, bf16, R <= 16 rows: B = 1): the whole S-step
 *      p_sample_loop of SimpleMLPAdaLN in one launch (replaces, per step: input_proj, depth x
 *      (uva_sampler_linear LN+SiLU, uva_sampler_linear gate+residual), the final LN linear and
 *      uva_p_sample_step -- diffusion_loss.py:142-189,261-283; gaussian_diffusion.py:395-440).
 * Weights stacked per kind: w1/w2 bf16 [depth, W, W], b1/b2/lnw/lnb fp32 [depth, W]; win bf16 [W, C],
 * bin [W]; wf bf16 [2C, W], bfin [2C].  mod: bf16 [S, R, ldmod] adaLN table (block i shift | scale |
 * gate at 3Wi, final shift | scale at 3W depth); coef fp32 [S, 8] (uva_p_sample_step's order);
 * noise fp32 [S, R, C]; x0 fp32 [R, C] (x_T) -> x_out [R, C].  work: uva_sampler_persistent_workspace
 * bytes, 256-B aligned (the call zeroes its counters with a memset node).  W == 1024, depth == 6,
 * C <= 16.  A run in which any hand-off wait hit its spin bound writes NaN to every x_out element and
 * sets the give-up flag; uva_sampler_persistent_status reads that flag (0 = clean; syncs the stream).
 * The 64 workgroups must be co-resident (one per CU): callers check the CU count first.
 * uva_sampler_persistent_test_hook(1): the NEXT launch publishes no phase (tests of the give-up path). */
long long uva_sampler_persistent_workspace(int W);
int uva_sampler_persistent(int R, int C, int W, int depth, int S, int clip, float eps, const void* w1, const float* b1,
                           const void* w2, const float* b2, const float* lnw, const float* lnb, const void* win,
                           const float* bin, const void* wf, const float* bfin, const void* mod, long long ldmod,
                           const float* coef, const float* noise, const float* x0, float* x_out, void* work,
                           long long work_bytes, hipStream_t stream);
int uva_sampler_persistent_status(const void* work, unsigned* flag, hipStream_t stream);
int uva_sampler_persistent_test_hook(int no_publish);

/* ---- optimizer + EMA (policy:343-360 torch AdamW; ema_model.py:57-89) ----------------- */
/* One launch per parameter group region (16-B aligned p/g/m/v/ema): n_decay = n applies the
 * group's weight decay wd, n_decay = 0 none.  ema (nullable) gets the fused EMA update with
 * ema_decay; p_bf16 (nullable) the refreshed bf16 shadow. */
int uva_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, void* p_bf16, long long n,
                  long long n_decay, float lr, float b1, float b2, float eps, float wd, int step, float grad_scale,
                  float ema_decay, hipStream_t stream);
/* EMAModel.step over the flat buffer (ema_model.py:78-85): ema = d*ema + (1-d)*p (16-B aligned). */
int uva_ema_update(float* ema, const float* p, long long n, float decay, hipStream_t stream);

/* ---- fp8 (OCP e4m3) attention forward, head_dim 64 (BASELINE config 5 "fp8 MFMA attention";
 *      same call site as uva_attn_fwd: timm Attention / SDPA, mar_con_unified.py:201-249).
 * uva_attn_quant_fp8: per (batch, head, q|k|v, 64-row tile) power-of-two scales; rounds the bf16
 *      qkv [B,N,3,H,64] IN PLACE to the fp8 grid (the backward then runs uva_attn_bwd on it:
 *      straight-through rounding) and fills `workspace` (uva_attn_fp8_workspace bytes, 256-B
 *      aligned) with the fp8 Q/K rows, the key-permuted fp8 V^T and the scales.
 * uva_attn_fwd_fp8: Q.K^T and P.V on the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3
 *      operands, per-tile E8M0 scales as MFMA operands), fp32 online softmax; out / lse2
 *      / mask as uva_attn_fwd.  N % 64 == 0. */
long long uva_attn_fp8_workspace(int B, int N, int H);
int uva_attn_quant_fp8(void* qkv, void* workspace, int B, int N, int H, hipStream_t stream);
int uva_attn_fwd_fp8(const void* workspace, void* out, float* lse2, const void* mask, int B, int N, int H, float scale,
                     float drop_p, hipStream_t stream);

/* ---- fused attention, head_dim 64, bf16 (timm Attention / SDPA with attn dropout,
 *      mar_con_unified.py:201-249 -> timm 0.9.7 Attention.forward, F.scaled_dot_product_attention).
 *      qkv: [B,N,3,H,64] (the qkv GEMM output), out/dout: [B,N,H,64], lse2: [B,H,N] log2-domain
 *      row log-sum-exp, Dvec: [B,H,N] scratch (D' = rowsum(dO*O)/(1-p), written by the dQ pass and read
 *      by the dK/dV pass of uva_attn_bwd), dqkv: [B,N,3,H,64].  N % 64 == 0.
 * uva_attn_dropmask: keep-mask bit planes (uva_attn_mask_bytes bytes) of the counter-hash
 *      dropout (p, seed) -- generated once per step, consumed by fwd and bwd (drop_p > 0).
 * uva_attn_bwd: workspace of uva_attn_bwd_workspace bytes (0 in this build: the loops run on the unscaled dO;
 * the query stays for ABI stability). */
long long uva_attn_mask_bytes(int B, int N, int H);
long long uva_attn_bwd_workspace(int B, int N, int H, float drop_p);
int uva_attn_dropmask(void* mask, int B, int N, int H, float drop_p, unsigned long long seed, hipStream_t stream);
int uva_attn_fwd(const void* qkv, void* out, float* lse2, const void* mask, int B, int N, int H, float scale,
                 float drop_p, hipStream_t stream);
int uva_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, const void* mask, float* Dvec,
                 void* dqkv, void* workspace, int B, int N, int H, float scale, float drop_p, hipStream_t stream);
/* uva_attn_bwd + the qkv Linear's bias gradient, dbias[3 H 64] (+)= column sums of dqkv as stored (bf16):
 * per-(batch, 128-row block) partials from the dQ / dK-dV kernels' epilogues in `part`
 * (B * ceil(N / 128) * 3 H 64 floats), then one column reduce -- no separate pass over dqkv
 * (replaces autograd's sum of the qkv output gradient for nn.Linear.bias, mar_con_unified.py:201-215). */
int uva_attn_bwd_bias(const void* qkv, const void* out, const void* dout, const float* lse2, const void* mask,
                      float* Dvec, void* dqkv, float* dbias, int accum, float* part, int B, int N, int H, float scale,
                      float drop_p, hipStream_t stream);

/* ---- KL-VAE encoder plumbing (vae/vaekl.py, utils/data_utils.py) ---------------------
 * uva_resize_select: obs image [B,T,3,Hin,Win] fp32 in [0,1] -> NHWC [B*nsel,256,256,Cpad]
 *   frames sel[] (select_frames, data_utils.py:140-158), bilinear align_corners=False
 *   (data_utils.py:72-81), x*255/127.5-1 (:210,226); images ordered future-half first,
 *   then history-half (get_vae_latent encodes x then c, :405-424).
 * uva_groupnorm_stats: GroupNorm(32, eps) of NHWC x -> scale/shift [Nimg][C] consumed by
 *   uva_conv2d's GN+SiLU A-loader (vaekl.py:14-17).  workspace: uva_groupnorm_workspace floats.
 * uva_posterior_sample: moments NHWC [Nimg,256,32] -> z tokens [Nimg,256,16] fp32,
 *   eps NCHW [Nimg,16,16,16] (DiagonalGaussianDistribution.sample, vaekl.py:400-417, x0.2325). */
int uva_resize_select(const float* img, int B, int T, int Hin, int Win, const int* sel, int nsel, int odt, void* out,
                      int Cpad, hipStream_t stream);
long long uva_groupnorm_workspace(int Nimg, int HW);
int uva_groupnorm_stats(int dtype, const void* x, int Nimg, int HW, int C, const float* gamma, const float* beta,
                        float eps, float* scale, float* shift, float* workspace, hipStream_t stream);
int uva_groupnorm_finalize_tiles(const float* part, int Nimg, int HW, int C, int tile_rows, const float* gamma,
                                 const float* beta, float eps, float* scale, float* shift, hipStream_t stream);
/* y = [SiLU](x*scale + shift) over NHWC bf16 (GroupNorm apply, once per element) */
int uva_groupnorm_apply(const void* x, const float* scale, const float* shift, void* y, int Nimg, int HW, int C,
                        int do_silu, hipStream_t stream);
/* y [n, 2H, 2W, C] = nearest x2 upsample of NHWC x [n, H, W, C] (decoder Upsample,
 * vaekl.py:20-33); C * sizeof(dtype) % 16 == 0. */
int uva_upsample_nearest2x(int dtype, const void* x, void* y, int n, int H, int W, int C, hipStream_t stream);
/* PushT training augmentation (dataset/pusht_image_dataset.py:93-130): per video b, params[b][9] =
 * {crop (0/1), top, left, blur (0/1), k0..k4 (normalised 1-D Gaussian)}; img/out [B,T,C,S,S] fp32,
 * crop window crop_size^2 resized back to S^2 (bilinear), then the 5x5 reflect-padded blur. */
int uva_pusht_augment(const float* img, float* out, const float* params, int B, int T, int C, int S, int crop_size,
                      hipStream_t stream);
/* Video training augmentation: the UMI chain of config/task/umi_lazy.yaml:50-72 (kornia 0.8
 * VideoSequential: RandomCrop -> Resize -> ColorJitter -> RandomSharpness -> RandomAutoContrast ->
 * RandomGrayscale -> RandomGaussianBlur, dataset/base_lazy_dataset.py:365-411) and the Libero ColorJitter of
 * dataset/libero_replay_image_dataset.py:229-247 (torchvision).  img/out [B,T,3,S,S] fp32 in [0,1];
 * params [B][24] per video (utils/augment.py); scratch >= B*T*(6*S*S + 7*ceil(S/8)) floats; S % 4 == 0, S <= 256.
 * Three launches over (frame, 8-row band) workgroups. */
int uva_video_augment(const float* img, float* out, float* scratch, const float* params, int B, int T, int S,
                      hipStream_t stream);
int uva_posterior_sample(int mdt, const void* moments, const float* eps, float* z, int Nimg, float scale,
                         hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UVA_HIP_H */
