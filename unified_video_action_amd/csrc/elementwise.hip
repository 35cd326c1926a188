// Elementwise kernels around the fused GEMMs (all HBM-bound, grid-stride, fp32 math):
//   cast, activation forward, activation/dropout backward (timm Mlp GELU+drop1,
//   proj_drop/drop2, DiffLoss SiLU, DiffActLoss ReLU), adaLN gated-residual backward
//   (diffusion_loss.py:163-167).  Mixed dtypes are resolved per call with a uniform
//   branch (ld/st helpers); the per-element cost is one predictable branch.
#include "common.h"

__device__ __forceinline__ float ldx(const void* p, int dt, long long i) {
  return dt == UVA_DT_BF16 ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void stx(void* p, int dt, long long i, float v) {
  if (dt == UVA_DT_BF16) ((bf16*)p)[i] = (bf16)v;
  else ((float*)p)[i] = v;
}

#define GRID_STRIDE(i, n) for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (long long)gridDim.x * blockDim.x)

static inline dim3 ew_grid(long long n) {
  long long b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

// 2-D strided view helper: element (r, c) of a [rows, cols] view with leading dim ld
__global__ void cast_kernel(const void* src, int sdt, long long lds, void* dst, int ddt, long long ldd, long long rows,
                            int cols) {
  GRID_STRIDE(i, rows * cols) {
    long long r = i / cols, c = i % cols;
    stx(dst, ddt, r * ldd + c, ldx(src, sdt, r * lds + c));
  }
}

// fast contiguous fp32 -> bf16 (8 per thread)
__global__ void cast_f32_bf16_vec(const float* __restrict__ src, bf16* __restrict__ dst, long long n8) {
  GRID_STRIDE(i, n8) {
    float4 a = ((const float4*)src)[2 * i], b = ((const float4*)src)[2 * i + 1];
    bf16x8 o = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
    ((bf16x8*)dst)[i] = o;
  }
}

__global__ void act_fwd_kernel(const void* x, int xdt, void* y, int ydt, long long n, int act) {
  GRID_STRIDE(i, n) stx(y, ydt, i, apply_act(act, ldx(x, xdt, i)));
}

// dx (+)= dy * keep/(1-p) * act'(pre)      (act = NONE -> pure dropout backward)
__global__ void act_bwd_kernel(const void* pre, int pdt, const void* dy, int gdt, void* dx, int xdt, long long rows,
                               int cols, long long ld_dy, long long ld_dx, int act, uint32_t thresh, float dscale,
                               uint64_t seed, int accum) {
  GRID_STRIDE(i, rows * (long long)cols) {
    long long r = i / cols, c = i % cols;
    float g = ldx(dy, gdt, r * ld_dy + c);
    if (thresh) g = dropout_keep(seed, (uint64_t)i, thresh) ? g * dscale : 0.f;
    if (act != ACT_NONE) g *= act_grad(act, ldx(pre, pdt, i));
    long long o = r * ld_dx + c;
    if (accum) g += ldx(dx, xdt, o);
    stx(dx, xdt, o, g);
  }
}

// out = x + gate*h  backward:  dgate = dout*h ; dh = dout*gate   (gate/dgate strided by ldg)
__global__ void gate_bwd_kernel(const float* dout, const void* h, int hdt, const void* gate, int gtdt, long long ldg,
                                void* dh, int dhdt, void* dgate, long long rows, int cols) {
  GRID_STRIDE(i, rows * (long long)cols) {
    long long r = i / cols, c = i % cols;
    float d = dout[i];
    float g = ldx(gate, gtdt, r * ldg + c);
    stx(dgate, gtdt, r * ldg + c, d * ldx(h, hdt, i));
    stx(dh, dhdt, i, d * g);
  }
}

__global__ void fill_kernel(float* p, long long n, float v) {
  GRID_STRIDE(i, n) p[i] = v;
}

extern "C" int uva_cast(int sdt, const void* src, long long lds, int ddt, void* dst, long long ldd, long long rows,
                        int cols, hipStream_t s) {
  long long n = rows * cols;
  if (n <= 0) return 0;
  if (sdt == UVA_DT_F32 && ddt == UVA_DT_BF16 && lds == cols && ldd == cols && n % 8 == 0 &&
      ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0)) {
    cast_f32_bf16_vec<<<ew_grid(n / 8), 256, 0, s>>>((const float*)src, (bf16*)dst, n / 8);
  } else {
    cast_kernel<<<ew_grid(n), 256, 0, s>>>(src, sdt, lds, dst, ddt, ldd, rows, cols);
  }
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_act_fwd(int xdt, const void* x, int ydt, void* y, long long n, int act, hipStream_t s) {
  if (n <= 0) return 0;
  act_fwd_kernel<<<ew_grid(n), 256, 0, s>>>(x, xdt, y, ydt, n, act);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_act_bwd(int pdt, const void* pre, int gdt, const void* dy, long long ld_dy, int xdt, void* dx,
                           long long ld_dx, long long rows, int cols, int act, float drop_p, unsigned long long seed,
                           int accum, hipStream_t s) {
  long long n = rows * cols;
  if (n <= 0) return 0;
  uint32_t th = drop_p > 0.f ? (uint32_t)fminf(drop_p * 4294967296.0f, 4294967295.0f) : 0u;
  float ds = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
  act_bwd_kernel<<<ew_grid(n), 256, 0, s>>>(pre, pdt, dy, gdt, dx, xdt, rows, cols, ld_dy, ld_dx, act, th, ds, seed,
                                            accum);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_gate_bwd(const float* dout, int hdt, const void* h, int gtdt, const void* gate, long long ldg,
                            int dhdt, void* dh, void* dgate, long long rows, int cols, hipStream_t s) {
  long long n = rows * cols;
  if (n <= 0) return 0;
  gate_bwd_kernel<<<ew_grid(n), 256, 0, s>>>(dout, h, hdt, gate, gtdt, ldg, dh, dhdt, dgate, rows, cols);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_fill(float* p, long long n, float v, hipStream_t s) {
  if (n <= 0) return 0;
  fill_kernel<<<ew_grid(n), 256, 0, s>>>(p, n, v);
  UVA_LAUNCH_CHECK();
  return 0;
}
