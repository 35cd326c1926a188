// Row kernels of the conv_fc action trunk (diffusion_action_loss.py:42-61: Conv2d(D, D, 3, p=1) +
// ReLU + AdaptiveAvgPool2d((4, 4)) + flatten (c w h)), so that its forward and backward run without
// ATen copies: the pooled features come out already flattened in (c, w, h) order, the pool's
// backward is fused with the ReLU mask, the conv weight changes layout in one pass, and the
// weight gradient is an implicit GEMM per tap over spatially padded dY / X (uva_pad_nhwc; the im2col
// builders below remain for tests and external callers).
// Tensors: activations NHWC [n][16][16][C] (first spatial axis = the reference's w).
#include "common.h"

template <typename T>
__device__ __forceinline__ T cvt_out(float v);
template <>
__device__ __forceinline__ float cvt_out<float>(float v) { return v; }
template <>
__device__ __forceinline__ bf16 cvt_out<bf16>(float v) { return (bf16)v; }

// out[n][c*16 + w4*4 + h4] = mean of the 4x4 block (w4, h4) of channel c; one thread per (n, c):
// the lanes of a wave take consecutive channels, so every input read is one coalesced row segment
template <typename T>
__global__ __launch_bounds__(256) void pool4x4_cwh_kernel(const T* __restrict__ in, T* __restrict__ out, int n,
                                                          int C) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n * C) return;
  const int c = (int)(t % C);
  const long long img = t / C;
  const T* src = in + img * 256 * C + c;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll 4
  for (int w = 0; w < 16; ++w)
#pragma unroll
    for (int h = 0; h < 16; ++h) acc[(w >> 2) * 4 + (h >> 2)] += to_f32(src[(w * 16 + h) * (long long)C]);
  T* dst = out + img * 16 * C + (long long)c * 16;
#pragma unroll
  for (int i = 0; i < 16; ++i) dst[i] = cvt_out<T>(acc[i] * 0.0625f);
}

// dpre[n][w][h][c] = (post[n][w][h][c] > 0) * gpool[n][c*16 + (w/4)*4 + h/4] / 16
// (the backward of mean-pool -> ReLU); one thread per (n, c, w4, h4) cell, lanes along c
template <typename T, typename TG>
__global__ __launch_bounds__(256) void pool4x4_relu_bwd_kernel(const T* __restrict__ post, const TG* __restrict__ gpool,
                                                               T* __restrict__ dpre, int n, int C) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n * 16 * C) return;
  const int c = (int)(t % C);
  const long long r = t / C;
  const int cell = (int)(r % 16);
  const long long img = r / 16;
  const int w4 = cell >> 2, h4 = cell & 3;
  const float g = to_f32(gpool[img * 16 * C + (long long)c * 16 + cell]) * 0.0625f;
  const long long base = img * 256 * C + c;
#pragma unroll
  for (int dw = 0; dw < 4; ++dw)
#pragma unroll
    for (int dh = 0; dh < 4; ++dh) {
      const long long o = base + (long long)((w4 * 4 + dw) * 16 + h4 * 4 + dh) * C;
      dpre[o] = cvt_out<T>(to_f32(post[o]) > 0.f ? g : 0.f);
    }
}

// cols[(img, y, x)][ci*9 + kh*3 + kw] = in[img][y + kh - 1][x + kw - 1][ci] (zero outside): one thread
// per (pixel, ci) writes its 9 contiguous columns
template <typename T>
__global__ __launch_bounds__(256) void im2col3x3_kernel(const T* __restrict__ in, T* __restrict__ cols, int n, int H,
                                                        int W, int Ci) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n * H * W * Ci) return;
  const int ci = (int)(t % Ci);
  const long long p = t / Ci;
  const int x = (int)(p % W);
  const long long q = p / W;
  const int y = (int)(q % H);
  const long long img = q / H;
  T* dst = cols + p * 9LL * Ci + (long long)ci * 9;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int yy = y + kh - 1, xx = x + kw - 1;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      dst[kh * 3 + kw] = ok ? in[((img * H + yy) * W + xx) * Ci + ci] : cvt_out<T>(0.f);
    }
}

// cols[(img, y, x)][tap * Ci + ci] = in[img][y + kh - 1][x + kw - 1][ci] (tap = kh * 3 + kw; zero
// outside): one thread per (pixel, tap, 8-channel chunk) moves 16 B, so both the gather reads and the
// 9x-sized column stream are full-width vector accesses (the (ci, tap) order above writes 9
// interleaved 2-B columns per thread: 0.59 ms at the PushT-joint B = 64 shape).  The dW product over
// these columns comes out as [Co][9][Ci] and is added into the nn.Conv2d-layout gradient by
// conv3x3_dw_scatter_add below.
template <typename T>
__global__ __launch_bounds__(256) void im2col3x3_tc_kernel(const T* __restrict__ in, T* __restrict__ cols, int n,
                                                           int H, int W, int Ci) {
  constexpr int V = 16 / sizeof(T);  // elements per 16-B chunk
  const int nc = Ci / V;
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)n * H * W * 9 * nc) return;
  const int c = (int)(t % nc);
  const long long r = t / nc;
  const int tap = (int)(r % 9);
  const long long p = r / 9;
  const int x = (int)(p % W);
  const long long q = p / W;
  const int y = (int)(q % H);
  const long long img = q / H;
  const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
  int4 v = {0, 0, 0, 0};
  if (yy >= 0 && yy < H && xx >= 0 && xx < W) v = *(const int4*)(in + ((img * H + yy) * W + xx) * Ci + c * V);
  *(int4*)(cols + (p * 9 + tap) * Ci + c * V) = v;
}

// grad[co][ci][kh][kw] += part[co][kh * 3 + kw][ci] (fp32): one thread per (co, ci) reads its 9 taps
// (coalesced over ci) and adds them to its 9 contiguous gradient words
__global__ __launch_bounds__(256) void conv3x3_dw_scatter_add_kernel(const float* __restrict__ part,
                                                                     float* __restrict__ grad, int Co, int Ci) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)Co * Ci) return;
  const int ci = (int)(t % Ci);
  const long long co = t / Ci;
  const float* src = part + co * 9 * Ci + ci;
  float* dst = grad + t * 9;
#pragma unroll
  for (int k = 0; k < 9; ++k) dst[k] += src[(long long)k * Ci];
}

// nn.Conv2d weight [Co][Ci][3][3] (fp32 master) -> the implicit-GEMM conv's [Co][kh][kw][Ci]
// (mode 0) or the dX conv's flipped transpose [Ci][kh][kw][Co] = w[co][ci][2-kh][2-kw] (mode 1)
template <typename T>
__global__ __launch_bounds__(256) void conv3x3_weight_layout_kernel(const float* __restrict__ w, T* __restrict__ out,
                                                                    int Co, int Ci, int mode) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long long)Co * Ci * 9) return;
  const int tap = (int)(t % 9);  // source index (co, ci, kh, kw): coalesced reads
  const long long r = t / 9;
  const int ci = (int)(r % Ci), co = (int)(r / Ci);
  const int kh = tap / 3, kw = tap % 3;
  const T v = cvt_out<T>(w[t]);
  if (mode == 0) out[(((long long)co * 3 + kh) * 3 + kw) * Ci + ci] = v;
  else out[(((long long)ci * 3 + (2 - kh)) * 3 + (2 - kw)) * Co + co] = v;
}

static inline unsigned nblocks(long long n) { return (unsigned)((n + 255) / 256); }

extern "C" int uva_pool4x4_cwh(int dtype, const void* in, void* out, int n, int C, hipStream_t s) {
  if (n <= 0) return 0;
  const long long work = (long long)n * C;
  if (dtype == UVA_DT_BF16)
    pool4x4_cwh_kernel<bf16><<<nblocks(work), 256, 0, s>>>((const bf16*)in, (bf16*)out, n, C);
  else
    pool4x4_cwh_kernel<float><<<nblocks(work), 256, 0, s>>>((const float*)in, (float*)out, n, C);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_pool4x4_relu_bwd(int dtype, const void* post, int gdtype, const void* gpool, void* dpre, int n,
                                    int C, hipStream_t s) {
  if (n <= 0) return 0;
  const long long work = (long long)n * 16 * C;
#define PRB(T, TG) pool4x4_relu_bwd_kernel<T, TG><<<nblocks(work), 256, 0, s>>>((const T*)post, (const TG*)gpool, \
                                                                                 (T*)dpre, n, C)
  if (dtype == UVA_DT_BF16 && gdtype == UVA_DT_BF16) PRB(bf16, bf16);
  else if (dtype == UVA_DT_BF16) PRB(bf16, float);
  else if (gdtype == UVA_DT_BF16) PRB(float, bf16);
  else PRB(float, float);
#undef PRB
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_im2col3x3(int dtype, const void* in, void* cols, int n, int H, int W, int Ci, hipStream_t s) {
  if (n <= 0) return 0;
  const long long work = (long long)n * H * W * Ci;
  if (dtype == UVA_DT_BF16)
    im2col3x3_kernel<bf16><<<nblocks(work), 256, 0, s>>>((const bf16*)in, (bf16*)cols, n, H, W, Ci);
  else
    im2col3x3_kernel<float><<<nblocks(work), 256, 0, s>>>((const float*)in, (float*)cols, n, H, W, Ci);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_im2col3x3_tc(int dtype, const void* in, void* cols, int n, int H, int W, int Ci, hipStream_t s) {
  if (n <= 0) return 0;
  const int V = dtype == UVA_DT_BF16 ? 8 : 4;
  if (Ci % V || (((uintptr_t)in | (uintptr_t)cols) % 16)) return (int)hipErrorInvalidValue;
  const long long work = (long long)n * H * W * 9 * (Ci / V);
  if (dtype == UVA_DT_BF16)
    im2col3x3_tc_kernel<bf16><<<nblocks(work), 256, 0, s>>>((const bf16*)in, (bf16*)cols, n, H, W, Ci);
  else
    im2col3x3_tc_kernel<float><<<nblocks(work), 256, 0, s>>>((const float*)in, (float*)cols, n, H, W, Ci);
  UVA_LAUNCH_CHECK();
  return 0;
}

// out[G + (img (H+2) + y) (W+2) + x][c] = in[img][y - 1][x - 1][c] inside, 0 on the 1-pixel border and in
// the G guard rows before / after (the padded operands of the implicit-GEMM weight gradient: with both
// dY and X padded, tap (kh, kw) is the constant row shift (kh - 1)(W + 2) + (kw - 1)); 16 B per thread
template <typename T>
__global__ __launch_bounds__(256) void pad_nhwc_kernel(const T* __restrict__ in, T* __restrict__ out, int n, int H,
                                                       int W, int C, int G) {
  constexpr int V = 16 / sizeof(T);
  const int cv = C / V;
  const long long rows = 2LL * G + (long long)n * (H + 2) * (W + 2);
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * cv) return;
  const long long r = t / cv;
  const int c = (int)(t - r * cv) * V;
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  const long long q = r - G;
  if (q >= 0 && q < (long long)n * (H + 2) * (W + 2)) {
    const int x = (int)(q % (W + 2));
    const long long q2 = q / (W + 2);
    const int y = (int)(q2 % (H + 2));
    const long long img = q2 / (H + 2);
    if (y >= 1 && y <= H && x >= 1 && x <= W)
      v = *(const uint4*)(in + ((img * H + (y - 1)) * W + (x - 1)) * C + c);
  }
  *(uint4*)(out + r * C + c) = v;
}

extern "C" int uva_pad_nhwc(int dtype, const void* in, void* out, int n, int H, int W, int C, int G, hipStream_t s) {
  if (n <= 0) return 0;
  const int V = dtype == UVA_DT_BF16 ? 8 : 4;
  if (C % V || G < 0 || (((uintptr_t)in | (uintptr_t)out) % 16)) return (int)hipErrorInvalidValue;
  const long long work = (2LL * G + (long long)n * (H + 2) * (W + 2)) * (C / V);
  if (dtype == UVA_DT_BF16)
    pad_nhwc_kernel<bf16><<<nblocks(work), 256, 0, s>>>((const bf16*)in, (bf16*)out, n, H, W, C, G);
  else
    pad_nhwc_kernel<float><<<nblocks(work), 256, 0, s>>>((const float*)in, (float*)out, n, H, W, C, G);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_conv3x3_dw_scatter_add(const float* part, float* grad, int Co, int Ci, hipStream_t s) {
  if (Co <= 0 || Ci <= 0) return 0;
  conv3x3_dw_scatter_add_kernel<<<nblocks((long long)Co * Ci), 256, 0, s>>>(part, grad, Co, Ci);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_conv3x3_weight_layout(const float* w, int out_dtype, void* out, int Co, int Ci, int mode,
                                         hipStream_t s) {
  if (mode != 0 && mode != 1) return (int)hipErrorInvalidValue;
  const long long work = (long long)Co * Ci * 9;
  if (out_dtype == UVA_DT_BF16)
    conv3x3_weight_layout_kernel<bf16><<<nblocks(work), 256, 0, s>>>(w, (bf16*)out, Co, Ci, mode);
  else
    conv3x3_weight_layout_kernel<float><<<nblocks(work), 256, 0, s>>>(w, (float*)out, Co, Ci, mode);
  UVA_LAUNCH_CHECK();
  return 0;
}
