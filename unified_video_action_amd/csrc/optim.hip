// Fused optimizer step over the flat fp32 parameter buffer (one pass, HBM-bound):
//   torch.optim.AdamW semantics (decoupled weight decay, bias correction; policy:343-360)
//   over one parameter group region [p, p+n) (the host launches once per group with that
//   group's lr / weight_decay -- policy:326-341 no-decay / decay groups)
//   + gradient averaging over DP ranks (grad_scale = 1/world)
//   + optional fused EMA update ema = d*ema + (1-d)*p_new (ema_model.py:57-89)
//   + optional bf16 shadow copy of the new weights for the next step's MFMA GEMMs.
// Algorithmic bytes per parameter: p rw 8 + g r 4 + m rw 8 + v rw 8 (+ ema rw 8) (+ bf16 w 2) = 28..38 B.
// Group regions start 16-B aligned (ParamStore pads them), so the body runs on float4 and
// only a < 4-element tail is scalar.
#include "common.h"

namespace {

struct AdamArgs {
  float lr, b1, b2, eps, wd, step_size, bc2_sqrt, grad_scale, ema_decay;
};

__device__ __forceinline__ float adam_one(float pi, float gi, float& mi, float& vi, const AdamArgs& a) {
  gi *= a.grad_scale;
  pi = pi * (1.0f - a.lr * a.wd);
  mi = mi + (1.0f - a.b1) * (gi - mi);  // lerp, as torch's foreach AdamW
  vi = vi * a.b2 + (1.0f - a.b2) * gi * gi;
  float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
  return pi - a.step_size * (mi / denom);
}

__global__ __launch_bounds__(256) void adamw_ema_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ ema, bf16* __restrict__ pbf, long long n,
                                                        AdamArgs a) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<const float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<const float4*>(m)[i];
    float4 vv = reinterpret_cast<const float4*>(v)[i];
    pv.x = adam_one(pv.x, gv.x, mv.x, vv.x, a);
    pv.y = adam_one(pv.y, gv.y, mv.y, vv.y, a);
    pv.z = adam_one(pv.z, gv.z, mv.z, vv.z, a);
    pv.w = adam_one(pv.w, gv.w, mv.w, vv.w, a);
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (ema) {
      float4 ev = reinterpret_cast<const float4*>(ema)[i];
      const float d = a.ema_decay, e = 1.0f - a.ema_decay;
      ev.x = ev.x * d + pv.x * e;
      ev.y = ev.y * d + pv.y * e;
      ev.z = ev.z * d + pv.z * e;
      ev.w = ev.w * d + pv.w * e;
      reinterpret_cast<float4*>(ema)[i] = ev;
    }
    if (pbf) {
      bf16x4 b;
      b[0] = (bf16)(pv.x);
      b[1] = (bf16)(pv.y);
      b[2] = (bf16)(pv.z);
      b[3] = (bf16)(pv.w);
      reinterpret_cast<bf16x4*>(pbf)[i] = b;
    }
  }
  // scalar tail (< 4 elements)
  const long long t = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) {
    float mi = m[t], vi = v[t];
    float pi = adam_one(p[t], g[t], mi, vi, a);
    p[t] = pi;
    m[t] = mi;
    v[t] = vi;
    if (ema) ema[t] = ema[t] * a.ema_decay + pi * (1.0f - a.ema_decay);
    if (pbf) pbf[t] = (bf16)pi;
  }
}

__global__ __launch_bounds__(256) void ema_update_kernel(float* __restrict__ ema, const float* __restrict__ p,
                                                         long long n, float d) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float e = 1.0f - d;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 ev = reinterpret_cast<const float4*>(ema)[i];
    const float4 pv = reinterpret_cast<const float4*>(p)[i];
    ev.x = ev.x * d + pv.x * e;
    ev.y = ev.y * d + pv.y * e;
    ev.z = ev.z * d + pv.z * e;
    ev.w = ev.w * d + pv.w * e;
    reinterpret_cast<float4*>(ema)[i] = ev;
  }
  const long long t = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) ema[t] = ema[t] * d + p[t] * e;
}

inline unsigned grid_for(long long n4) {
  long long blocks = (n4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 8192) blocks = 8192;  // 32 waves/CU resident; grid-stride beyond
  return (unsigned)blocks;
}

inline bool aligned16(const void* q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

extern "C" int uva_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, void* p_bf16, long long n,
                             long long n_decay, float lr, float b1, float b2, float eps, float wd, int step,
                             float grad_scale, float ema_decay, hipStream_t s) {
  if (n <= 0) return 0;
  if (!aligned16(p) || !aligned16(g) || !aligned16(m) || !aligned16(v) || !aligned16(ema) ||
      (p_bf16 && (reinterpret_cast<uintptr_t>(p_bf16) & 7)))
    return (int)hipErrorInvalidValue;  // group regions are 16-B aligned by construction
  if (n_decay != 0 && n_decay != n) return (int)hipErrorInvalidValue;  // one launch = one group
  double bc1 = 1.0 - pow((double)b1, (double)step);
  double bc2 = 1.0 - pow((double)b2, (double)step);
  AdamArgs a;
  a.lr = lr;
  a.b1 = b1;
  a.b2 = b2;
  a.eps = eps;
  a.wd = n_decay ? wd : 0.0f;
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)sqrt(bc2);
  a.grad_scale = grad_scale;
  a.ema_decay = ema_decay;
  adamw_ema_kernel<<<dim3(grid_for(n >> 2)), 256, 0, s>>>(p, g, m, v, ema, (bf16*)p_bf16, n, a);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_ema_update(float* ema, const float* p, long long n, float decay, hipStream_t s) {
  if (n <= 0) return 0;
  if (!aligned16(ema) || !aligned16(p)) return (int)hipErrorInvalidValue;
  ema_update_kernel<<<dim3(grid_for(n >> 2)), 256, 0, s>>>(ema, p, n, decay);
  UVA_LAUNCH_CHECK();
  return 0;
}
