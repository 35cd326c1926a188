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
 * (counter hash, p, seed) -> +residual -> +beta*C_old.
 * Replaces: every nn.Linear fwd/bwd (timm Block qkv/proj/fc1/fc2
 * mar_con_unified.py:201-249; z_proj/z_proj_cond/proj_cond_x_layer/decoder_embed
 * :92-95,185-187,218; SimpleMLPAdaLN diffusion_loss.py:219-283; DiffActLoss fc/refine
 * diffusion_action_loss.py:49-61), torch.bmm of vae/vaekl.py:143-157, and the fp32
 * materialised form of F.scaled_dot_product_attention. */
int uva_gemm(int in_dtype, int out_dtype, int ta, int tb, const void* A, const void* B, void* C, int M, int N,
             int K, long long lda, long long ldb, long long ldc, int batch, int batch_inner, long long sAo,
             long long sAi, long long sBo, long long sBi, long long sCo, long long sCi, const float* bias,
             const void* residual, long long ldr, long long sRo, long long sRi, void* aux, int act, float alpha,
             float beta, float drop_p, unsigned long long drop_seed, int force_generic, hipStream_t stream);

/* ---- LayerNorm (affine or adaLN-modulated) --------------------------------------------
 * Replaces nn.LayerNorm(eps=1e-6) (mar_con_unified.py:198,215,252; timm norm1/norm2)
 * and modulate(LN(x), shift, scale) (diffusion_loss.py:93-94,163-189). */
int uva_layernorm_fwd(int in_dtype, int out_dtype, const void* x, const float* w, const float* b, const void* scale,
                      const void* shift, long long ldm, void* y, float* mean, float* rstd, int rows, int D, float eps,
                      hipStream_t stream);
int uva_layernorm_bwd(int in_dtype, int out_dtype, const void* x, const float* w, const void* scale, long long ldm,
                      const float* dy, const float* mean, const float* rstd, float* dx, int accum, void* dscale,
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
int uva_act_bwd(int pdt, const void* pre, int gdt, const void* dy, long long ld_dy, int xdt, void* dx,
                long long ld_dx, long long rows, int cols, int act, float drop_p, unsigned long long seed, int accum,
                hipStream_t stream);
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

/* ---- optimizer + EMA (policy:343-360 torch AdamW; ema_model.py:57-89) ----------------- */
int uva_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, void* p_bf16, long long n,
                  long long n_decay, float lr, float b1, float b2, float eps, float wd, int step, float grad_scale,
                  float ema_decay, hipStream_t stream);

/* ---- fused attention, head_dim 64, bf16 (timm Attention / SDPA with attn dropout,
 *      mar_con_unified.py:201-249).  qkv: [B,N,3,H,64] (the qkv GEMM output), out/dout:
 *      [B,N,H,64], lse2: [B,H,N] log2-domain row log-sum-exp, Dvec: [B,H,N] workspace,
 *      dqkv: [B,N,3,H,64].  N % 64 == 0.  dropout = counter hash (p, seed). */
int uva_attn_fwd(const void* qkv, void* out, float* lse2, int B, int N, int H, float scale, float drop_p,
                 unsigned long long seed, hipStream_t stream);
int uva_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, float* Dvec, void* dqkv,
                 int B, int N, int H, float scale, float drop_p, unsigned long long seed, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UVA_HIP_H */
