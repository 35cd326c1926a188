// Gaussian-diffusion training loss of the DiffLoss / DiffActLoss heads, fused:
//   q_sample                  gaussian_diffusion.py:220-236
//   eps-MSE + learned-range VB gaussian_diffusion.py:713-818, diffusion_utils.py:10-73
//   timestep features          diffusion_loss.py:111-134
// The schedule tables (float64 in the reference, gathered then cast to fp32,
// gaussian_diffusion.py:892-904) are uploaded once as fp32 arrays.
// The loss kernel also emits d(loss_row)/d(model_out) so the backward is a row scaling.
#include "common.h"

struct DiffTables {
  const float* sqrt_ac;
  const float* sqrt_1mac;
  const float* coef1;
  const float* coef2;
  const float* plvc;
  const float* log_betas;
  const float* sqrt_recip_ac;
  const float* sqrt_recipm1_ac;
};

__device__ __forceinline__ float ldx2(const void* p, int dt, long long i) {
  return dt == UVA_DT_BF16 ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void stx2(void* p, int dt, long long i, float v) {
  if (dt == UVA_DT_BF16) ((bf16*)p)[i] = (bf16)v;
  else ((float*)p)[i] = v;
}

// x_t = sqrt(abar_t) x0 + sqrt(1 - abar_t) noise   (written in the net's input dtype)
__global__ void q_sample_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                const long long* __restrict__ t, DiffTables tb, void* xt, int xdt, int rows, int C) {
  long long n = (long long)rows * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    long long r = i / C;
    long long ti = t[r];
    float a = tb.sqrt_ac[ti] * x0[i];
    float b = tb.sqrt_1mac[ti] * noise[i];
    stx2(xt, xdt, i, a + b);
  }
}

// sinusoidal features [cos(t f_i), sin(t f_i)], f precomputed on host exactly as the reference
__global__ void timestep_feat_kernel(const long long* __restrict__ t, const float* __restrict__ freqs, void* out,
                                     int odt, int rows, int half) {
  long long n = (long long)rows * 2 * half;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    long long r = i / (2 * half);
    int c = (int)(i % (2 * half));
    float a = (float)t[r] * freqs[c % half];
    stx2(out, odt, i, c < half ? cosf(a) : sinf(a));
  }
}

__device__ __forceinline__ float approx_cdf(float x, float* dcdf) {
  const float k = 0.7978845608028654f;  // sqrt(2/pi)
  float u = k * (x + 0.044715f * x * x * x);
  float th = tanhf(u);
  *dcdf = 0.5f * (1.0f - th * th) * k * (1.0f + 3.0f * 0.044715f * x * x);
  return 0.5f * (1.0f + th);
}

// one thread per row.  out: model output [rows, 2C] (dtype odt).  Writes
//   loss_row[r]          = mse + vb
//   dl[r][0..2C)         = d loss_row / d out  (fp32)
__global__ void diff_loss_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                 const long long* __restrict__ t, const void* __restrict__ out, int odt,
                                 long long ld_out, DiffTables tb, float* __restrict__ loss_row, float* __restrict__ dl,
                                 int rows, int C) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const long long ti = t[r];
  const float sa = tb.sqrt_ac[ti], s1 = tb.sqrt_1mac[ti];
  const float c1 = tb.coef1[ti], c2 = tb.coef2[ti];
  const float tlv = tb.plvc[ti], maxlog = tb.log_betas[ti], minlog = tb.plvc[ti];
  const float sr = tb.sqrt_recip_ac[ti], srm1 = tb.sqrt_recipm1_ac[ti];
  const float inv_ln2 = 1.0f / 0.6931471805599453f;
  const float invC = 1.0f / C;
  float mse = 0.f, vbsum = 0.f;
  for (int c = 0; c < C; ++c) {
    const long long i = (long long)r * C + c;
    const float x0v = x0[i], nz = noise[i];
    const float xt = sa * x0v + s1 * nz;
    const float eps = ldx2(out, odt, (long long)r * ld_out + c);
    const float v = ldx2(out, odt, (long long)r * ld_out + C + c);
    const float de = nz - eps;
    mse += de * de;
    const float frac = (v + 1.0f) * 0.5f;
    const float mlv = frac * maxlog + (1.0f - frac) * minlog;
    const float dmlv_dv = 0.5f * (maxlog - minlog);
    const float tm = c1 * x0v + c2 * xt;
    const float x0h = sr * xt - srm1 * eps;
    const float mm = c1 * x0h + c2 * xt;
    float term, dterm_dmlv;
    if (ti > 0) {
      const float e1 = expf(tlv - mlv), e2 = expf(-mlv);
      const float dm = tm - mm;
      term = 0.5f * (-1.0f + mlv - tlv + e1 + dm * dm * e2);
      dterm_dmlv = 0.5f * (1.0f - e1 - dm * dm * e2);
    } else {
      // -log p(x0) of the discretised gaussian, log_scale = 0.5 mlv
      const float inv_std = expf(-0.5f * mlv);
      const float cen = x0v - mm;
      const float pin = inv_std * (cen + 1.0f / 255.0f), min_ = inv_std * (cen - 1.0f / 255.0f);
      float dp, dmn;
      const float cdf_p = approx_cdf(pin, &dp), cdf_m = approx_cdf(min_, &dmn);
      const float dpin = -0.5f * pin, dmin = -0.5f * min_;  // d(in)/d(mlv)
      float lp, dlp;
      if (x0v < -0.999f) {
        float a = fmaxf(cdf_p, 1e-12f);
        lp = logf(a);
        dlp = cdf_p >= 1e-12f ? dp * dpin / cdf_p : 0.f;
      } else if (x0v > 0.999f) {
        float om = 1.0f - cdf_m;
        lp = logf(fmaxf(om, 1e-12f));
        dlp = om >= 1e-12f ? -dmn * dmin / om : 0.f;
      } else {
        float d = cdf_p - cdf_m;
        lp = logf(fmaxf(d, 1e-12f));
        dlp = d >= 1e-12f ? (dp * dpin - dmn * dmin) / d : 0.f;
      }
      term = -lp;
      dterm_dmlv = -dlp;
    }
    vbsum += term;
    dl[(long long)r * 2 * C + c] = -2.0f * de * invC;
    dl[(long long)r * 2 * C + C + c] = dterm_dmlv * dmlv_dv * invC * inv_ln2;
  }
  loss_row[r] = mse * invC + vbsum * invC * inv_ln2;
}

// single-block weighted reduction: res[0] = sum(l*w)/sum(w), res[1] = sum(w)   (w null -> 1)
__global__ __launch_bounds__(1024) void weighted_mean_kernel(const float* __restrict__ l, const float* __restrict__ w,
                                                             int n, float* __restrict__ res) {
  __shared__ float sa[16], sb[16];
  float a = 0.f, b = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float wi = w ? w[i] : 1.0f;
    a += l[i] * wi;
    b += wi;
  }
  a = wave_sum(a);
  b = wave_sum(b);
  int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sa[wid] = a; sb[wid] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float A = 0.f, Bv = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { A += sa[k]; Bv += sb[k]; }
    res[0] = A / Bv;
    res[1] = Bv;
  }
}

// dout[r][c] = g_up[0] * w[r] / wsum[0] * dl[r][c]      (w null -> 1)
__global__ void loss_grad_kernel(const float* __restrict__ dl, const float* __restrict__ w,
                                 const float* __restrict__ wsum, const float* __restrict__ g_up, void* dout, int ddt,
                                 long long ld, int rows, int C2) {
  long long n = (long long)rows * C2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    long long r = i / C2;
    int c = (int)(i % C2);
    float s = g_up[0] * (w ? w[r] : 1.0f) / wsum[0];
    stx2(dout, ddt, r * ld + c, s * dl[i]);
  }
}

// One reverse step of GaussianDiffusion.p_sample for the learned-range eps model
// (gaussian_diffusion.py:260-346 p_mean_variance, :395-440 p_sample):
//   log_var = f*max_log + (1-f)*min_log,  f = (v+1)/2
//   x0      = sqrt_recip_ac*x - sqrt_recipm1_ac*eps   [clamped to [-1, 1] when clip_denoised]
//   mean    = coef1*x0 + coef2*x
//   x_new   = mean + nonzero*exp(log_var/2)*noise*temperature
// Every row shares the step's timestep, so the eight schedule coefficients (float64 tables cast
// to fp32, :892-904) arrive as kernel arguments -- each captured graph node carries its own.
// x_new may alias x; x_net (optional) receives x_new in the net's input dtype for the next step.
struct PStepCoef {
  float sqrt_recip_ac, sqrt_recipm1_ac, coef1, coef2, min_log, max_log, nonzero, temperature;
};

__global__ void p_sample_step_kernel(const void* __restrict__ out, int odt, long long ld_out, const float* x,
                                     const float* __restrict__ noise, PStepCoef k, float* x_new, void* x_net,
                                     int xdt, int clip, int rows, int C) {
  long long n = (long long)rows * C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    long long r = i / C;
    int c = (int)(i % C);
    float eps = ldx2(out, odt, r * ld_out + c);
    float v = ldx2(out, odt, r * ld_out + C + c);
    float xi = x[i];
    float f = (v + 1.0f) / 2.0f;
    float log_var = f * k.max_log + (1.0f - f) * k.min_log;
    float x0 = k.sqrt_recip_ac * xi - k.sqrt_recipm1_ac * eps;
    if (clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
    float mean = k.coef1 * x0 + k.coef2 * xi;
    float xn = mean + k.nonzero * expf(0.5f * log_var) * noise[i] * k.temperature;
    x_new[i] = xn;
    if (x_net) stx2(x_net, xdt, i, xn);
  }
}

static inline dim3 grid_for(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

extern "C" int uva_q_sample(const float* x0, const float* noise, const long long* t, const float* const* tables,
                            int xdt, void* xt, int rows, int C, hipStream_t s) {
  DiffTables tb{tables[0], tables[1], tables[2], tables[3], tables[4], tables[5], tables[6], tables[7]};
  q_sample_kernel<<<grid_for((long long)rows * C), 256, 0, s>>>(x0, noise, t, tb, xt, xdt, rows, C);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_timestep_features(const long long* t, const float* freqs, int odt, void* out, int rows, int half,
                                     hipStream_t s) {
  timestep_feat_kernel<<<grid_for((long long)rows * 2 * half), 256, 0, s>>>(t, freqs, out, odt, rows, half);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_diffusion_loss(const float* x0, const float* noise, const long long* t, int odt, const void* out,
                                  long long ld_out, const float* const* tables, float* loss_row, float* dl, int rows,
                                  int C, hipStream_t s) {
  DiffTables tb{tables[0], tables[1], tables[2], tables[3], tables[4], tables[5], tables[6], tables[7]};
  diff_loss_kernel<<<dim3((rows + 255) / 256), 256, 0, s>>>(x0, noise, t, out, odt, ld_out, tb, loss_row, dl, rows, C);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_weighted_mean(const float* l, const float* w, int n, float* res, hipStream_t s) {
  weighted_mean_kernel<<<1, 1024, 0, s>>>(l, w, n, res);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_loss_grad(const float* dl, const float* w, const float* wsum, const float* g_up, int ddt, void* dout,
                             long long ld, int rows, int C2, hipStream_t s) {
  loss_grad_kernel<<<grid_for((long long)rows * C2), 256, 0, s>>>(dl, w, wsum, g_up, dout, ddt, ld, rows, C2);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_p_sample_step(int odt, const void* out, long long ld_out, const float* x, const float* noise,
                                 const float* coef, float* x_new, int xdt, void* x_net, int clip, int rows, int C,
                                 hipStream_t s) {
  if (rows <= 0 || C <= 0 || ld_out < 2 * C) return (int)hipErrorInvalidValue;
  PStepCoef k{coef[0], coef[1], coef[2], coef[3], coef[4], coef[5], coef[6], coef[7]};
  p_sample_step_kernel<<<grid_for((long long)rows * C), 256, 0, s>>>(out, odt, ld_out, x, noise, k, x_new, x_net,
                                                                      xdt, clip, rows, C);
  UVA_LAUNCH_CHECK();
  return 0;
}
