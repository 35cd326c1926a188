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

// vectorized form: 8 consecutive columns per thread (16-B loads/stores), one mask hash per pair
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
  } else {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
    *(bf16x8*)p = x;
  } else {
    *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
    *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename GT, typename XT>
__global__ void act_bwd_vec_kernel(const void* pre, int pdt, const GT* __restrict__ dy, XT* __restrict__ dx, int rows,
                                   int cols, long long ld_dy, long long ld_dx, int act, uint32_t thresh, float dscale,
                                   uint64_t seed, int accum) {
  const unsigned c8n = (unsigned)cols >> 3;
  const unsigned n8 = (unsigned)rows * c8n;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const unsigned r = i / c8n, c0 = (i - r * c8n) * 8;
    float g[8];
    ld8<GT>(dy + (long long)r * ld_dy + c0, g);
    if (thresh) {
      const uint64_t e0 = (uint64_t)r * cols + c0;  // even: cols % 8 == 0
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        bool k0, k1;
        dropout_keep2(seed, e0 + e, thresh, k0, k1);
        g[e] = k0 ? g[e] * dscale : 0.f;
        g[e + 1] = k1 ? g[e + 1] * dscale : 0.f;
      }
    }
    if (act != ACT_NONE) {
      float pv[8];
      const long long pi = (long long)r * cols + c0;
      if (pdt == UVA_DT_BF16) ld8<bf16>((const bf16*)pre + pi, pv);
      else ld8<float>((const float*)pre + pi, pv);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] *= act_grad(act, pv[e]);
    }
    XT* o = dx + (long long)r * ld_dx + c0;
    if (accum) {
      float prev[8];
      ld8<XT>(o, prev);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += prev[e];
    }
    st8<XT>(o, g);
  }
}

// Activation/dropout backward fused with the bias gradient (nn.Linear bias grad = column sum
// of the pre-activation gradient, the tensor the dW GEMM consumes): block = 32 column groups
// (8 columns, 16-B loads) x 8 row lanes over a chunk of COLSUM_RPB rows; the LDS-reduced chunk
// sums go to part[chunk][cols] (fp32, sums of the values as stored), reduced by colsum_final.
// STORE = false: plain column-sum partials of dy (no act, no store) -- uva_colsum's tall path.
#define COLSUM_RPB 128
template <typename GT, typename XT, bool STORE>
__global__ __launch_bounds__(256) void act_bwd_colsum_kernel(const void* pre, int pdt, const GT* __restrict__ dy,
                                                             XT* __restrict__ dx, int rows, int cols, long long ld_dy,
                                                             long long ld_dx, int act, uint32_t thresh, float dscale,
                                                             uint64_t seed, int accum, float* __restrict__ part) {
  __shared__ float red[8][32 * 8 + 4];
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  const int r0 = blockIdx.y * COLSUM_RPB, r1 = min(rows, r0 + COLSUM_RPB);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < cols) {
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += 8) {
      float g[8];
      ld8<GT>(dy + (long long)r * ld_dy + c0, g);
      if (STORE) {
        if (thresh) {
          const uint64_t e0 = (uint64_t)r * cols + c0;
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            bool k0, k1;
            dropout_keep2(seed, e0 + e, thresh, k0, k1);
            g[e] = k0 ? g[e] * dscale : 0.f;
            g[e + 1] = k1 ? g[e + 1] * dscale : 0.f;
          }
        }
        if (act != ACT_NONE) {
          float pv[8];
          const long long pi = (long long)r * cols + c0;
          if (pdt == UVA_DT_BF16) ld8<bf16>((const bf16*)pre + pi, pv);
          else ld8<float>((const float*)pre + pi, pv);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] *= act_grad(act, pv[e]);
        }
        XT* o = dx + (long long)r * ld_dx + c0;
        if (accum) {
          float prev[8];
          ld8<XT>(o, prev);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] += prev[e];
        }
        st8<XT>(o, g);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += to_f32(from_f32<XT>(g[e]));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += g[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][cg * 8 + e] = s[e];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < cols) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += red[j][threadIdx.x];
    part[(long long)blockIdx.y * cols + c] = t;
  }
}

// out[c] (+)= sum_j part[j][c]: 32 columns x 8 row lanes per block
__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nrows, int cols,
                                                           float* __restrict__ out, int accum) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (c < cols) {
#pragma unroll 8
    for (int j = rl; j < nrows; j += 8) s += part[(long long)j * cols + c];
  }
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += red[j][cl];
    out[c] = accum ? out[c] + t : t;
  }
}

extern "C" long long uva_act_bwd_bias_workspace(long long rows, int cols) {
  return (rows + COLSUM_RPB - 1) / COLSUM_RPB * (long long)cols;
}

// uva_act_bwd + dbias (+)= column sums of dx (as stored); bf16/fp32, cols % 8 == 0, 16-B aligned
extern "C" int uva_act_bwd_bias(int pdt, const void* pre, int gdt, const void* dy, long long ld_dy, int xdt, void* dx,
                                long long ld_dx, long long rows, int cols, int act, float drop_p,
                                unsigned long long seed, int accum, float* dbias, int accum_bias, float* workspace,
                                hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  if (cols % 8 || ld_dy % 8 || ld_dx % 8 || rows >= (1ll << 31) ||
      (((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)pre) % 16) || !dbias || !workspace)
    return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const int nch = (int)((rows + COLSUM_RPB - 1) / COLSUM_RPB);
  dim3 g1((cols / 8 + 31) / 32, nch);
#define AB(GT, XT)                                                                                               \
  act_bwd_colsum_kernel<GT, XT, true><<<g1, 256, 0, s>>>(pre, pdt, (const GT*)dy, (XT*)dx, (int)rows, cols, ld_dy, \
                                                         ld_dx, act, th, ds, seed, accum, workspace)
  if (gdt == UVA_DT_BF16 && xdt == UVA_DT_BF16) AB(bf16, bf16);
  else if (gdt == UVA_DT_BF16) AB(bf16, float);
  else if (xdt == UVA_DT_BF16) AB(float, bf16);
  else AB(float, float);
#undef AB
  UVA_LAUNCH_CHECK();
  colsum_final_kernel<<<dim3((cols + 31) / 32), 256, 0, s>>>(workspace, nch, cols, dbias, accum_bias);
  UVA_LAUNCH_CHECK();
  return 0;
}

// out[c] (+)= sum_j part[j][c] (C++ linkage, library-internal): the column-partial reduce of the fused
// GEMM epilogues (gemm8w.hip EPI 3)
int uva_colsum_final_launch(const float* part, int nrows, int cols, float* out, int accum, hipStream_t s) {
  colsum_final_kernel<<<dim3((cols + 31) / 32), 256, 0, s>>>(part, nrows, cols, out, accum);
  return (int)hipGetLastError();
}

// vectorized tall column sum (uva_colsum fast path): returns 1 if handled
int uva_colsum_vec(int dtype, const void* in, long long ld, float* out, int rows, int cols, int accum,
                   float* workspace, hipStream_t s) {
  if (cols % 8 || ld % 8 || ((uintptr_t)in % 16) || !workspace || rows < 2 * COLSUM_RPB) return 0;
  const int nch = (rows + COLSUM_RPB - 1) / COLSUM_RPB;
  dim3 g1((cols / 8 + 31) / 32, nch);
  if (dtype == UVA_DT_BF16)
    act_bwd_colsum_kernel<bf16, bf16, false><<<g1, 256, 0, s>>>(nullptr, 0, (const bf16*)in, nullptr, rows, cols, ld,
                                                                0, 0, 0, 1.f, 0, 0, workspace);
  else
    act_bwd_colsum_kernel<float, float, false><<<g1, 256, 0, s>>>(nullptr, 0, (const float*)in, nullptr, rows, cols,
                                                                  ld, 0, 0, 0, 1.f, 0, 0, workspace);
  if (hipGetLastError() != hipSuccess) return -1;
  colsum_final_kernel<<<dim3((cols + 31) / 32), 256, 0, s>>>(workspace, nch, cols, out, accum);
  if (hipGetLastError() != hipSuccess) return -1;
  return 1;
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

// dst[c][r] = src[r][c] for a bf16 [rows][cols] matrix: 64 x 64 tiles through LDS (16-B loads and
// stores, 8 consecutive elements per thread each way).  The transposed bf16 weight copies that
// turn the Block's width-768 dX products (x @ W -> x @ (W^T)^T) into the forward GEMM layout
// (K-contiguous B), 17-27 % faster on the 128 x 384 tile than the transposed-B read path.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                             int rows, int cols) {
  __shared__ bf16 t[64][64 + 8];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + i * 256, rr = id >> 3, cc = (id & 7) * 8;
    const int r = r0 + rr, c = c0 + cc;
    bf16x8 v;
    if (r < rows && c + 8 <= cols) {
      v = *(const bf16x8*)(src + (long long)r * cols + c);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (r < rows && c + e < cols) ? src[(long long)r * cols + c + e] : (bf16)0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) t[rr][cc + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + i * 256, cc = id >> 3, rr = (id & 7) * 8;  // output row = src column
    const int c = c0 + cc, r = r0 + rr;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[rr + e][cc];
    if (c < cols && r + 8 <= rows) {
      *(bf16x8*)(dst + (long long)c * rows + r) = v;
    } else if (c < cols) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (r + e < rows) dst[(long long)c * rows + r + e] = v[e];
    }
  }
}

extern "C" int uva_transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return 0;
  if ((rows % 8) || (cols % 8) || (((uintptr_t)src | (uintptr_t)dst) % 16)) return (int)hipErrorInvalidValue;
  transpose_bf16_kernel<<<dim3((cols + 63) / 64, (rows + 63) / 64), 256, 0, s>>>((const bf16*)src, (bf16*)dst, rows,
                                                                                 cols);
  UVA_LAUNCH_CHECK();
  return 0;
}

// y = residual + drop(act(x)), 8 consecutive elements per thread (16-B bf16 / 2 x 16-B fp32
// accesses), dropout index = flat element index (= row * cols + col of a contiguous [rows][cols]:
// the GEMM epilogue's and act_bwd's mask).  The forward of timm Mlp when its GEMMs run bias-only
// on the library: fc1 -> a = drop(GELU(pre)), fc2 -> x2 = x1 + drop(fc2 out).
template <typename TX, typename TY, typename TR>
__global__ __launch_bounds__(256) void act_drop_fwd_kernel(const TX* __restrict__ x, TY* __restrict__ y,
                                                           const TR* __restrict__ res, long long n8, int act,
                                                           uint32_t thresh, float dscale, uint64_t seed) {
  GRID_STRIDE(i, n8) {
    float v[8], r[8];
    ld8<TX>(x + i * 8, v);
    if (res) ld8<TR>(res + i * 8, r);
    switch (act) {
      case ACT_GELU:
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
        break;
      case ACT_SILU:
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = silu(v[e]);
        break;
      case ACT_RELU:
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        break;
      default:
        break;
    }
    if (thresh) {
      bool keep[8];
#pragma unroll
      for (int e = 0; e < 8; e += 2) dropout_keep2(seed, (uint64_t)(i * 8 + e), thresh, keep[e], keep[e + 1]);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = keep[e] ? v[e] * dscale : 0.f;
    }
    if (res) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    st8<TY>(y + i * 8, v);
  }
}

extern "C" int uva_act_drop_fwd(int xdt, const void* x, int ydt, void* y, int rdt, const void* residual, long long n,
                                int act, float drop_p, unsigned long long seed, hipStream_t s) {
  if (n <= 0) return 0;
  if (n % 8 || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)residual) % 16)) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const long long n8 = n / 8;
#define ADF(TX, TY, TR) \
  act_drop_fwd_kernel<TX, TY, TR><<<ew_grid(n8), 256, 0, s>>>((const TX*)x, (TY*)y, (const TR*)residual, n8, act, th, ds, seed)
  if (xdt == UVA_DT_BF16 && ydt == UVA_DT_BF16 && (!residual || rdt == UVA_DT_BF16)) ADF(bf16, bf16, bf16);
  else if (xdt == UVA_DT_BF16 && ydt == UVA_DT_F32 && (!residual || rdt == UVA_DT_F32)) ADF(bf16, float, float);
  else if (xdt == UVA_DT_F32 && ydt == UVA_DT_F32 && (!residual || rdt == UVA_DT_F32)) ADF(float, float, float);
  else return (int)hipErrorInvalidValue;
#undef ADF
  UVA_LAUNCH_CHECK();
  return 0;
}

// ---- dropout keep-bit planes --------------------------------------------------------------
// bit (i & 31) of word i >> 5 = the keep decision of flat element i (dropout_keep: the counter hash of pair
// i >> 1, low half for even i, high half for odd): the mask every dropout kernel of this library derives
// from (seed, flat index), precomputed once so that the GEMM epilogues that apply it (gemm8w.hip: fc1 GELU +
// dropout forward, the fused GELU'-backward, fc2 / proj dropout + residual) test a bit instead of hashing.
// One word per thread: 16 pair hashes whose first words differ only in their low 4 bits (drop_first of a
// 16-aligned pair base, xor j)
__global__ __launch_bounds__(256) void drop_plane_kernel(uint32_t* __restrict__ plane, long long nwords, uint32_t key,
                                                         uint32_t thresh) {
  GRID_STRIDE(w, nwords) {
    const uint32_t f0 = drop_first(key, (uint64_t)w * 16);
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t h = drop_mix(f0 ^ (uint32_t)j);
      bits |= ((h & 0xFFFFu) >= thresh ? 1u : 0u) << (2 * j);
      bits |= ((h >> 16) >= thresh ? 1u : 0u) << (2 * j + 1);
    }
    plane[w] = bits;
  }
}

extern "C" long long uva_dropout_plane_words(long long n) { return (n + 31) / 32; }

extern "C" int uva_dropout_plane(void* plane, long long n, float drop_p, unsigned long long seed, hipStream_t s) {
  if (n <= 0) return 0;
  if (!plane || ((uintptr_t)plane % 4)) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const long long nw = (n + 31) / 32;
  drop_plane_kernel<<<ew_grid(nw), 256, 0, s>>>((uint32_t*)plane, nw, drop_key(seed), th);
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
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const bool vec = cols % 8 == 0 && ld_dy % 8 == 0 && ld_dx % 8 == 0 && n / 8 < (1ll << 31) &&
                   (((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)pre) % 16 == 0);
  if (vec) {
    const long long n8 = n / 8;
#define AB(GT, XT)                                                                                              \
  act_bwd_vec_kernel<GT, XT><<<ew_grid(n8), 256, 0, s>>>(pre, pdt, (const GT*)dy, (XT*)dx, (int)rows, cols, ld_dy, \
                                                         ld_dx, act, th, ds, seed, accum)
    if (gdt == UVA_DT_BF16 && xdt == UVA_DT_BF16) AB(bf16, bf16);
    else if (gdt == UVA_DT_BF16) AB(bf16, float);
    else if (xdt == UVA_DT_BF16) AB(float, bf16);
    else AB(float, float);
#undef AB
  } else {
    act_bwd_kernel<<<ew_grid(n), 256, 0, s>>>(pre, pdt, dy, gdt, dx, xdt, rows, cols, ld_dy, ld_dx, act, th, ds, seed,
                                              accum);
  }
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
