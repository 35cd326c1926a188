// Fused optimizer step over the flat fp32 parameter buffer (one pass, HBM-bound):
//   torch.optim.AdamW semantics (decoupled weight decay, bias correction; policy:343-360,
//   two param groups: [0, n_decay) decayed, [n_decay, n) not -- policy:326-341)
//   + gradient averaging over DP ranks (grad_scale = 1/world)
//   + EMA update ema = d*ema + (1-d)*p (ema_model.py:57-89)
//   + bf16 shadow copy of the new weights for the next step's MFMA GEMMs.
// Algorithmic bytes per parameter: p rw 8 + g r 4 + m rw 8 + v rw 8 + ema rw 8 + bf16 w 2 = 38 B.
#include "common.h"

__global__ __launch_bounds__(256) void adamw_ema_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ ema, bf16* __restrict__ pbf, long long n,
                                                        long long n_decay, float lr, float b1, float b2, float eps,
                                                        float wd, float step_size, float bc2_sqrt, float grad_scale,
                                                        float ema_decay) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float gi = g[i] * grad_scale;
    float pi = p[i];
    if (i < n_decay) pi = pi * (1.0f - lr * wd);
    float mi = m[i];
    mi = mi + (1.0f - b1) * (gi - mi);  // lerp
    float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
    if (ema) ema[i] = ema[i] * ema_decay + pi * (1.0f - ema_decay);
    if (pbf) pbf[i] = (bf16)pi;
  }
}

extern "C" int uva_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, void* p_bf16, long long n,
                             long long n_decay, float lr, float b1, float b2, float eps, float wd, int step,
                             float grad_scale, float ema_decay, hipStream_t s) {
  if (n <= 0) return 0;
  double bc1 = 1.0 - pow((double)b1, (double)step);
  double bc2 = 1.0 - pow((double)b2, (double)step);
  float step_size = (float)(lr / bc1);
  float bc2_sqrt = (float)sqrt(bc2);
  long long blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  adamw_ema_kernel<<<dim3((unsigned)blocks), 256, 0, s>>>(p, g, m, v, ema, (bf16*)p_bf16, n, n_decay, lr, b1, b2,
                                                          eps, wd, step_size, bc2_sqrt, grad_scale, ema_decay);
  UVA_LAUNCH_CHECK();
  return 0;
}
