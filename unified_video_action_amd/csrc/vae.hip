// KL-VAE encoder plumbing around the implicit-GEMM convolutions (gemm.hip uva_conv2d):
//   frame select + bilinear resize + pixel normalisation  (data_utils.py:19-83,140-158,206-226)
//   GroupNorm(32, eps 1e-6) statistics -> per-(image, channel) scale/shift consumed by the
//     next convolution's A-loader (vaekl.py:14-17)
//   posterior sample  z = (mean + exp(0.5*clamp(logvar,-30,20)) * eps) * 0.2325
//     (vaekl.py:400-417, data_utils.py:391-399), written directly as MAR tokens.
#include "common.h"

// obs image [B, T, 3, Hin, Win] fp32 in [0,1] -> NHWC [B*nsel, 256, 256, Cpad] (dtype odt)
// image order: first every sample's future frames (sel[half..]), then the history frames
// (get_vae_latent encodes x = future first, then c = history: data_utils.py:405-424).
__global__ void resize_select_kernel(const float* __restrict__ img, int B, int T, int Hin, int Win,
                                     const int* __restrict__ sel, int nsel, void* out, int odt, int Cpad) {
  const int HO = 256, WO = 256;
  const long long total = (long long)B * nsel * HO * WO;
  const float sh = (float)Hin / HO, sw = (float)Win / WO;
  const int half = nsel / 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int ox = i % WO;
    const int oy = (i / WO) % HO;
    const long long img_id = i / (HO * WO);  // output image index
    const int part = img_id / ((long long)B * half);  // 0: future, 1: history
    const int rem = img_id % ((long long)B * half);
    const int b = rem / half, f = rem % half;
    const int frame = sel[(part == 0 ? half : 0) + f];
    float sy = sh * (oy + 0.5f) - 0.5f;
    float sx = sw * (ox + 0.5f) - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    sx = sx < 0.f ? 0.f : sx;
    int y0 = (int)sy, x0 = (int)sx;
    int y1 = y0 + (y0 < Hin - 1 ? 1 : 0), x1 = x0 + (x0 < Win - 1 ? 1 : 0);
    float ly = sy - y0, lx = sx - x0;
    float hy = 1.f - ly, hx = 1.f - lx;
    const float* base = img + ((long long)b * T + frame) * 3 * Hin * Win;
    for (int c = 0; c < Cpad; ++c) {
      float v = 0.f;
      if (c < 3) {
        const float* p = base + (long long)c * Hin * Win;
        float r = hy * (hx * p[y0 * Win + x0] + lx * p[y0 * Win + x1]) + ly * (hx * p[y1 * Win + x0] + lx * p[y1 * Win + x1]);
        v = (r * 255.0f) / 127.5f - 1.0f;
      }
      long long o = i * Cpad + c;
      if (odt == UVA_DT_BF16) ((bf16*)out)[o] = (bf16)v;
      else ((float*)out)[o] = v;
    }
  }
}

// GroupNorm partial sums: grid (Nimg, chunks).  x NHWC [Nimg, HW, C].
// part[n][chunk][g][0..1] = (sum, sumsq) of the chunk's pixels for group g (32 groups)
template <typename T>
__global__ __launch_bounds__(256) void gn_partial_kernel(const T* __restrict__ x, int HW, int C, int pix_per_chunk,
                                                         float* __restrict__ part) {
  __shared__ float red[2][512];
  const int n = blockIdx.x, chunk = blockIdx.y, nch = gridDim.y;
  const int p0 = chunk * pix_per_chunk, p1 = min(HW, p0 + pix_per_chunk);
  // each thread: fixed channel c, pixels strided by (256 / C) lanes
  for (int i = threadIdx.x; i < 2 * C; i += 256) red[i / C][i % C] = 0.f;
  __syncthreads();
  const int tpc = 256 / C >= 1 ? 256 / C : 1;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int c = c0 + (threadIdx.x % min(C, 256));
    const int pl = threadIdx.x / min(C, 256);
    float s = 0.f, q = 0.f;
    if (c < C)
      for (int p = p0 + pl; p < p1; p += tpc) {
        float v = to_f32(x[((long long)n * HW + p) * C + c]);
        s += v;
        q += v * v;
      }
    if (c < C) {
      atomicAdd(&red[0][c], s);
      atomicAdd(&red[1][c], q);
    }
  }
  __syncthreads();
  const int gs = C / 32;
  if (threadIdx.x < 32) {
    float s = 0.f, q = 0.f;
    for (int j = 0; j < gs; ++j) {
      s += red[0][threadIdx.x * gs + j];
      q += red[1][threadIdx.x * gs + j];
    }
    float* o = part + (((long long)n * nch + chunk) * 32 + threadIdx.x) * 2;
    o[0] = s;
    o[1] = q;
  }
}

// finalize: per (n, c) scale = gamma*rstd, shift = beta - mean*scale
__global__ void gn_finalize_kernel(const float* __restrict__ part, int nch, int HW, int C, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float* __restrict__ scale,
                                   float* __restrict__ shift, int Nimg) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)Nimg * C) return;
  const int n = i / C, c = i % C, gs = C / 32, g = c / gs;
  double s = 0.0, q = 0.0;
  for (int k = 0; k < nch; ++k) {
    const float* o = part + (((long long)n * nch + k) * 32 + g) * 2;
    s += o[0];
    q += o[1];
  }
  const double cnt = (double)HW * gs;
  const double mean = s / cnt;
  double var = q / cnt - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * rstd;
  scale[i] = sc;
  shift[i] = beta[c] - (float)mean * sc;
}

// moments NHWC [Nimg, 256, 32] -> tokens [Nimg, 256, 16] (fp32); eps given NCHW [Nimg,16,16,16]
__global__ void posterior_kernel(const void* __restrict__ mom, int mdt, const float* __restrict__ eps,
                                 float* __restrict__ z, int Nimg, float scale) {
  const long long total = (long long)Nimg * 256 * 16;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = i % 16;
    const long long pix = i / 16;
    const int s = pix % 256;
    const long long n = pix / 256;
    float mean = mdt == UVA_DT_BF16 ? (float)((const bf16*)mom)[pix * 32 + c] : ((const float*)mom)[pix * 32 + c];
    float lv = mdt == UVA_DT_BF16 ? (float)((const bf16*)mom)[pix * 32 + 16 + c] : ((const float*)mom)[pix * 32 + 16 + c];
    lv = fminf(fmaxf(lv, -30.0f), 20.0f);
    const float e = eps[(n * 16 + c) * 256 + s];
    z[i] = (mean + expf(0.5f * lv) * e) * scale;
  }
}

// finalize fused (conv-epilogue) GroupNorm partials: part[tile][32][2], tiles_per_img tiles per image.
// One wave per (image, group): lanes stride over the image's tiles (fp64 sums: E[x^2] - mean^2
// cancels), a wave reduction, then the group's C/32 channels get scale/shift.  (One thread per
// channel, each summing all tiles serially, took 40 us per call at the level-0 shape.)
__global__ __launch_bounds__(256) void gn_finalize_tiles_kernel(const float* __restrict__ part, int tiles_per_img,
                                                                long long cnt_per_group, int C,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps,
                                                                float* __restrict__ scale, float* __restrict__ shift,
                                                                int Nimg) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= Nimg * 32) return;
  const int n = w >> 5, g = w & 31, gs = C / 32;
  const float2* p = (const float2*)part + (long long)n * tiles_per_img * 32 + g;
  double s = 0.0, q = 0.0;
  for (int t = lane; t < tiles_per_img; t += 64) {
    const float2 v = p[(long long)t * 32];
    s += v.x;
    q += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  const double mean = s / cnt_per_group;
  double var = q / cnt_per_group - mean * mean;
  if (var < 0) var = 0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int j = lane; j < gs; j += 64) {
    const int c = g * gs + j;
    const float sc = gamma[c] * rstd;
    scale[(long long)n * C + c] = sc;
    shift[(long long)n * C + c] = beta[c] - (float)mean * sc;
  }
}

// y = act(x * scale[n][c] + shift[n][c]), NHWC bf16, 8 channels per thread
__global__ void gn_apply_kernel(const bf16* __restrict__ x, const float* __restrict__ scale,
                                const float* __restrict__ shift, bf16* __restrict__ y, long long n8, int HW, int C,
                                int do_silu) {
  const int c8 = C / 8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8) * 8;
    const long long n = (i / c8) / HW;
    const float* sc = scale + n * C + c;
    const float* sh = shift + n * C + c;
    float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
    float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
    float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float hh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    bf16x8 v = ((const bf16x8*)x)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float u = (float)v[j] * ss[j] + hh[j];
      v[j] = (bf16)(do_silu ? silu(u) : u);
    }
    ((bf16x8*)y)[i] = v;
  }
}

static inline dim3 gridn(long long n) {
  long long b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  return dim3((unsigned)(b < 1 ? 1 : b));
}

extern "C" int uva_resize_select(const float* img, int B, int T, int Hin, int Win, const int* sel, int nsel, int odt,
                                 void* out, int Cpad, hipStream_t s) {
  resize_select_kernel<<<gridn((long long)B * nsel * 256 * 256), 256, 0, s>>>(img, B, T, Hin, Win, sel, nsel, out, odt,
                                                                              Cpad);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" long long uva_groupnorm_workspace(int Nimg, int HW) {
  int nch = (HW + 1023) / 1024;
  return (long long)Nimg * nch * 32 * 2;
}

extern "C" int uva_groupnorm_stats(int dtype, const void* x, int Nimg, int HW, int C, const float* gamma,
                                   const float* beta, float eps, float* scale, float* shift, float* workspace,
                                   hipStream_t s) {
  if (C % 32 != 0 || C > 512) return (int)hipErrorInvalidValue;
  const int ppc = 1024;
  const int nch = (HW + ppc - 1) / ppc;
  dim3 g1(Nimg, nch);
  if (dtype == UVA_DT_BF16) gn_partial_kernel<bf16><<<g1, 256, 0, s>>>((const bf16*)x, HW, C, ppc, workspace);
  else gn_partial_kernel<float><<<g1, 256, 0, s>>>((const float*)x, HW, C, ppc, workspace);
  gn_finalize_kernel<<<gridn((long long)Nimg * C), 256, 0, s>>>(workspace, nch, HW, C, gamma, beta, eps, scale, shift,
                                                                 Nimg);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_posterior_sample(int mdt, const void* moments, const float* eps, float* z, int Nimg, float scale,
                                    hipStream_t s) {
  posterior_kernel<<<gridn((long long)Nimg * 4096), 256, 0, s>>>(moments, mdt, eps, z, Nimg, scale);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_groupnorm_finalize_tiles(const float* part, int Nimg, int HW, int C, int tile_rows,
                                            const float* gamma, const float* beta, float eps, float* scale,
                                            float* shift, hipStream_t s) {
  if (HW % tile_rows != 0 || C % 32 != 0) return (int)hipErrorInvalidValue;
  gn_finalize_tiles_kernel<<<dim3((unsigned)((Nimg * 32 + 3) / 4)), 256, 0, s>>>(
      part, HW / tile_rows, (long long)HW * (C / 32), C, gamma, beta, eps, scale, shift, Nimg);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_groupnorm_apply(const void* x, const float* scale, const float* shift, void* y, int Nimg, int HW,
                                   int C, int do_silu, hipStream_t s) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  long long n8 = (long long)Nimg * HW * C / 8;
  gn_apply_kernel<<<gridn(n8), 256, 0, s>>>((const bf16*)x, scale, shift, (bf16*)y, n8, HW, C, do_silu);
  UVA_LAUNCH_CHECK();
  return 0;
}

// Nearest x2 upsampling of NHWC maps (Upsample, vae/vaekl.py:20-33: F.interpolate(scale_factor=2,
// mode="nearest")): one 16-byte channel chunk per thread, read once, written to the 4 children.
__global__ void upsample2x_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int n, int H, int W, int chunks) {
  const long long total = (long long)n * H * W * chunks;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % chunks);
    long long p = i / chunks;
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const long long img = p / H;
    const uint4 v = x[i];
    const long long W2 = 2LL * W;
    const long long base = ((img * 2 * H + 2 * h) * W2 + 2 * w) * chunks + c;
    y[base] = v;
    y[base + chunks] = v;
    y[base + W2 * chunks] = v;
    y[base + W2 * chunks + chunks] = v;
  }
}

extern "C" int uva_upsample_nearest2x(int dtype, const void* x, void* y, int n, int H, int W, int C, hipStream_t s) {
  const int esz = dtype == UVA_DT_BF16 ? 2 : 4;
  if (n <= 0 || H <= 0 || W <= 0 || (C * esz) % 16) return (int)hipErrorInvalidValue;
  const int chunks = C * esz / 16;
  const long long total = (long long)n * H * W * chunks;
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  upsample2x_kernel<<<dim3((unsigned)blocks), 256, 0, s>>>((const uint4*)x, (uint4*)y, n, H, W, chunks);
  UVA_LAUNCH_CHECK();
  return 0;
}

// PushT training augmentation on the device (dataset/pusht_image_dataset.py:93-130; the reference
// runs it per video in the CPU dataloader with one seed for all frames):
//   RandomApply(RandomCrop(91), p=0.5) -> Resize(96, antialias) -> RandomApply(GaussianBlur(5), p=0.5)
// img/out: [B, T, C, S, S] fp32 in [0, 1].  prm: [B][9] floats per video
//   {crop, top, left, blur, k0..k4}: k = the normalised 1-D Gaussian (torchvision
//   _get_gaussian_kernel1d, computed on the host).  Upscaling 91 -> 96 with antialias reduces to
//   bilinear with align_corners=False (triangle filter of support 1; edge taps clamp).  The blur
//   is the separable 5x5 product kernel over the reflect-padded resized image, evaluated per
//   output pixel from the source (the 96x96 intermediate never exists).
__device__ __forceinline__ int reflect_idx(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

__device__ __forceinline__ float aug_resized(const float* __restrict__ plane, int S, bool crop, int top, int left,
                                             int cs, int y, int x) {
  if (!crop) return plane[y * S + x];
  const float sc = (float)cs / (float)S;
  float sy = ((float)y + 0.5f) * sc - 0.5f, sx = ((float)x + 0.5f) * sc - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + 1 < cs ? y0 + 1 : cs - 1, x1 = x0 + 1 < cs ? x0 + 1 : cs - 1;
  const float ly = sy - (float)y0, lx = sx - (float)x0;
  const float* r0 = plane + (top + y0) * S + left;
  const float* r1 = plane + (top + y1) * S + left;
  const float a = r0[x0] * (1.f - lx) + r0[x1] * lx;
  const float b = r1[x0] * (1.f - lx) + r1[x1] * lx;
  return a * (1.f - ly) + b * ly;
}

__global__ void pusht_augment_kernel(const float* __restrict__ img, float* __restrict__ out, const float* __restrict__ prm,
                                     int B, int TC, int S, int cs) {
  const long long total = (long long)B * TC * S * S;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(i % S);
    const int y = (int)((i / S) % S);
    const long long plane_id = i / ((long long)S * S);
    const int b = (int)(plane_id / TC);
    const float* p = prm + b * 9;
    const bool crop = p[0] != 0.f, blur = p[3] != 0.f;
    const int top = (int)p[1], left = (int)p[2];
    const float* plane = img + plane_id * S * S;
    float v;
    if (!blur) {
      v = aug_resized(plane, S, crop, top, left, cs, y, x);
    } else {
      v = 0.f;
#pragma unroll
      for (int dy = -2; dy <= 2; ++dy) {
        const int yy = reflect_idx(y + dy, S);
        float row = 0.f;
#pragma unroll
        for (int dx = -2; dx <= 2; ++dx) row += p[6 + dx] * aug_resized(plane, S, crop, top, left, cs, yy, reflect_idx(x + dx, S));
        v += p[6 + dy] * row;
      }
    }
    out[i] = v;
  }
}

extern "C" int uva_pusht_augment(const float* img, float* out, const float* params, int B, int T, int C, int S,
                                 int crop_size, hipStream_t s) {
  if (B <= 0 || T <= 0 || C <= 0 || S < 3 || crop_size <= 0 || crop_size > S || img == out) {
    return (int)hipErrorInvalidValue;
  }
  const long long total = (long long)B * T * C * S * S;
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  pusht_augment_kernel<<<dim3((unsigned)blocks), 256, 0, s>>>(img, out, params, B, T * C, S, crop_size);
  UVA_LAUNCH_CHECK();
  return 0;
}
