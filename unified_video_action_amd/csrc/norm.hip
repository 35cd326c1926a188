// Row-wise kernels: LayerNorm / adaLN-modulated LayerNorm forward+backward
// (timm Block norm1/norm2, z_proj_ln, encoder/decoder norms: mar_con_unified.py:198,215,252;
//  DiffLoss ResBlock in_ln + modulate and FinalLayer norm_final: diffusion_loss.py:93-94,152,177),
// and the row softmax of the materialised attention path.
//
// One wave per row, each lane owning D/64 elements in registers (VEC contiguous per
// access when D % 256 == 0); statistics in fp32, two passes over registers.
// HBM-bound: algorithmic bytes per row = D*(sizeof(in)+sizeof(out)) (+ modulation).
#include "common.h"

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* out, int n) {
#pragma unroll
  for (int i = 0; i < n; ++i) out[i] = to_f32(p[i]);
}

template <int VEC, typename T>
__device__ __forceinline__ void ldv(const T* p, float (&o)[VEC]) {
  if constexpr (VEC == 4 && sizeof(T) == 4) {
    float4 v = *(const float4*)p;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else if constexpr (VEC == 4 && sizeof(T) == 2) {
    bf16x4 v = *(const bf16x4*)p;
    o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) o[i] = to_f32(p[i]);
  }
}

template <int VEC, typename T>
__device__ __forceinline__ void stv(T* p, const float (&o)[VEC]) {
  if constexpr (VEC == 4 && sizeof(T) == 4) {
    *(float4*)p = make_float4(o[0], o[1], o[2], o[3]);
  } else if constexpr (VEC == 4 && sizeof(T) == 2) {
    bf16x4 v = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
    *(bf16x4*)p = v;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) p[i] = from_f32<T>(o[i]);
  }
}

// element index of slot (c, v) of lane
template <int VEC>
__device__ __forceinline__ int col_of(int c, int lane, int v) { return (c * 64 + lane) * VEC + v; }

// ------------------------------------------------------------------------------------
// forward: y = LN(x) * w + b                    (w, b fp32, nullable)
//          y = LN(x) * (1 + scale) + shift      (scale/shift rows of TO, ld = ldm) if scale
// ------------------------------------------------------------------------------------
template <typename TI, typename TO, int VEC, int NC>
__global__ __launch_bounds__(256) void ln_fwd(const TI* __restrict__ x, const float* __restrict__ w,
                                              const float* __restrict__ b, const TO* __restrict__ scale,
                                              const TO* __restrict__ shift, long long ldm, TO* __restrict__ y,
                                              float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows,
                                              int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const TI* xr = x + (long long)row * D;
  float v[NC][VEC];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int col = col_of<VEC>(c, lane, 0);
    if (col < D) {
      ldv<VEC>(xr + col, v[c]);
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[c][i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) s += v[c][i];
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      int col = col_of<VEC>(c, lane, i);
      float d = (col < D) ? v[c][i] - mean : 0.f;
      q += d * d;
    }
  const float var = wave_sum(q) / D;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  TO* yr = y + (long long)row * D;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    int col0 = col_of<VEC>(c, lane, 0);
    if (col0 >= D) continue;
    float o[VEC];
    float sc[VEC], sh[VEC], wv[VEC], bv[VEC];
    if (scale) {
      ldv<VEC>(scale + (long long)row * ldm + col0, sc);
      ldv<VEC>(shift + (long long)row * ldm + col0, sh);
    }
    if (w) ldv<VEC>(w + col0, wv);  // vector loads: per-element scalar loads were issue-bound
    if (b) ldv<VEC>(b + col0, bv);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float h = (v[c][i] - mean) * rstd;
      if (w) h = h * wv[i];
      if (b) h = h + bv[i];
      if (scale) h = h * (1.0f + sc[i]) + sh[i];
      o[i] = h;
    }
    stv<VEC>(yr + col0, o);
  }
}

// ------------------------------------------------------------------------------------
// backward.  dy fp32 or bf16 (the bf16 dX of the consuming GEMM: autocast semantics, half the
// bytes of the dominant read).  g = dy*w (affine) or dy*(1+scale) (modulated)
//   dx (+)= rstd * (g - mean(g) - xhat*mean(g*xhat))           fp32, accumulate if accum
//   modulated: dscale = dy*xhat, dshift = dy  (TO, ld = ldm)
//   affine: per-block partial sums dw_part[blk][D] = sum dy*xhat, db_part = sum dy
// ------------------------------------------------------------------------------------
// raw (unconverted) VEC-element vector of T: loads are issued into these and converted at first use,
// so a row's loads can be in flight while the previous row is computed
template <int VEC, typename T>
struct RawVec {
  T v[VEC];
};
template <int VEC, typename T>
__device__ __forceinline__ RawVec<VEC, T> ldraw(const T* p) {
  RawVec<VEC, T> r;
  if constexpr (VEC == 4 && sizeof(T) == 4) {
    *(float4*)r.v = *(const float4*)p;
  } else if constexpr (VEC == 4 && sizeof(T) == 2) {
    *(bf16x4*)r.v = *(const bf16x4*)p;
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) r.v[i] = p[i];
  }
  return r;
}

// One wave per row, rows r0 + wid, r0 + wid + 4, ... of the block.  Software-pipelined: the next
// row's x / dy / dx-base loads (and its mean / rstd) are issued before the current row's reductions,
// so a wave keeps two rows of loads in flight and each row costs one memory latency, not two (the
// dx-base read used to wait for the row's reductions).  HBM-bound: per row D * (sizeof(TI) +
// sizeof(TD) + 4 [+ 4 dx base]) bytes read, D * 4 written.
// DROPO: the dx rows also leave as bf16(drop(dx)) (the next op's input: the timm Block's proj_drop backward,
// mar_con_unified.py:201-215, i.e. what act_bwd_bias(none) computed from dx in a second pass) with the column
// sums of those stored values (the proj bias gradient) as per-block partials dd_part
struct LnDrop {
  bf16* out;
  float* part;
  uint32_t key, thresh;
  float dscale;
};

template <typename TI, typename TO, int VEC, int NC, typename TD, bool DROPO = false>
__global__ __launch_bounds__(256) void ln_bwd(const TI* __restrict__ x, const float* __restrict__ w,
                                              const float* __restrict__ b, const TO* __restrict__ scale, long long ldm,
                                              const TD* __restrict__ dy, const float* __restrict__ mean_in,
                                              const float* __restrict__ rstd_in, const float* dx_base,
                                              float* dx, int accum,
                                              TO* __restrict__ dscale, TO* __restrict__ dshift,
                                              float* __restrict__ dw_part, float* __restrict__ db_part, int rows,
                                              int D, int rows_per_block, LnDrop ldrop = LnDrop{}) {
  __shared__ float red_w[4][1024];
  __shared__ float red_b[4][1024];
  __shared__ float red_d[DROPO ? 4 : 1][DROPO ? 1024 : 1];
  float pd[NC][VEC];
  if constexpr (DROPO) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < VEC; ++i) pd[c][i] = 0.f;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float pw[NC][VEC], pb[NC][VEC];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < VEC; ++i) pw[c][i] = pb[c][i] = 0.f;
  // per-column constants of the lane (w, b) once per block
  float wv[NC][VEC], bv[NC][VEC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col0 = col_of<VEC>(c, lane, 0);
#pragma unroll
    for (int i = 0; i < VEC; ++i) wv[c][i] = bv[c][i] = 0.f;
    if (col0 < D) {
      if (w) ldv<VEC>(w + col0, wv[c]);
      if (b) ldv<VEC>(b + col0, bv[c]);
    }
  }
  const float* addsrc = dx_base ? dx_base : (accum ? dx : nullptr);  // row source added to the result
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  struct Row {
    RawVec<VEC, TI> x[NC];
    RawVec<VEC, TD> d[NC];
    RawVec<VEC, float> a[NC];
    float mean, rstd;
  };
  auto load_row = [&](int row, Row& R) __attribute__((always_inline)) {
    R.mean = mean_in[row];
    R.rstd = rstd_in[row];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int col0 = col_of<VEC>(c, lane, 0);
      if (col0 < D) {
        R.x[c] = ldraw<VEC>(x + (long long)row * D + col0);
        R.d[c] = ldraw<VEC>(dy + (long long)row * D + col0);
        if (addsrc) R.a[c] = ldraw<VEC>(addsrc + (long long)row * D + col0);
      }
    }
  };
  // one row: its loads were issued one row earlier into R; the row after next is loaded into L
  auto process = [&](int row, const Row& R, Row& L, bool pf) __attribute__((always_inline)) {
    if (pf && row + 4 < r1) load_row(row + 4, L);
    const float mean = R.mean, rstd = R.rstd;
    float xh[NC][VEC], g[NC][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      int col0 = col_of<VEC>(c, lane, 0);
      if (col0 >= D) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) xh[c][i] = g[c][i] = 0.f;
        continue;
      }
      float sc[VEC];
      if (scale) ldv<VEC>(scale + (long long)row * ldm + col0, sc);
      float ds[VEC], dsh[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        xh[c][i] = (to_f32(R.x[c].v[i]) - mean) * rstd;
        const float dv = to_f32(R.d[c].v[i]);
        // y_aff = xhat*w + b ; h = y_aff*(1+scale) + shift (modulated) or h = y_aff
        float da = dv;
        if (scale) {
          float ya = w ? xh[c][i] * wv[c][i] + (b ? bv[c][i] : 0.f) : xh[c][i];
          da = dv * (1.0f + sc[i]);
          ds[i] = dv * ya;
          dsh[i] = dv;
        }
        if (w) {
          pw[c][i] += da * xh[c][i];
          pb[c][i] += da;
          g[c][i] = da * wv[c][i];
        } else {
          g[c][i] = da;
        }
        s1 += g[c][i];
        s2 += g[c][i] * xh[c][i];
      }
      if (scale) {
        stv<VEC>(dscale + (long long)row * ldm + col0, ds);
        stv<VEC>(dshift + (long long)row * ldm + col0, dsh);
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      int col0 = col_of<VEC>(c, lane, 0);
      if (col0 >= D) continue;
      float o[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float d = rstd * (g[c][i] - m1 - xh[c][i] * m2);
        o[i] = addsrc ? R.a[c].v[i] + d : d;
      }
      stv<VEC>(dx + (long long)row * D + col0, o);
      if constexpr (DROPO) {
        static_assert(VEC % 2 == 0, "pairs");
        const unsigned long long e0 = (unsigned long long)row * (unsigned)D + (unsigned)col0;  // even
        float q[VEC];
#pragma unroll
        for (int i = 0; i < VEC; i += 2) {
          const uint32_t h = drop_hash(ldrop.key, (e0 + i) >> 1);
          q[i] = (h & 0xFFFFu) >= ldrop.thresh ? o[i] * ldrop.dscale : 0.f;
          q[i + 1] = (h >> 16) >= ldrop.thresh ? o[i + 1] * ldrop.dscale : 0.f;
        }
        bf16 qb[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          qb[i] = (bf16)q[i];
          pd[c][i] += (float)qb[i];
        }
        if constexpr (VEC == 4) {
          bf16x4 v4 = {qb[0], qb[1], qb[2], qb[3]};
          *(bf16x4*)(ldrop.out + (long long)row * D + col0) = v4;
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) ldrop.out[(long long)row * D + col0 + i] = qb[i];
        }
      }
    }
  };
  Row ra, rb;
  int row = r0 + wid;
  if constexpr (NC <= 3) {
    // two register sets used in turn (no copies between rows)
    if (row < r1) load_row(row, ra);
    for (; row < r1; row += 8) {
      process(row, ra, rb, true);
      if (row + 4 < r1) process(row + 4, rb, ra, true);
    }
  } else {
    // D = 1024 (adaLN trunk): two row sets do not fit beside the modulated path's state (276
    // VGPRs, one wave per SIMD: 199 -> 283 us), so rows are loaded one at a time
    for (; row < r1; row += 4) {
      load_row(row, ra);
      process(row, ra, rb, false);
    }
  }
  if (dw_part) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        int col = col_of<VEC>(c, lane, i);
        if (col < D) {
          red_w[wid][col] = pw[c][i];
          red_b[wid][col] = pb[c][i];
        }
      }
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += 256) {
      dw_part[(long long)blockIdx.x * D + col] = red_w[0][col] + red_w[1][col] + red_w[2][col] + red_w[3][col];
      db_part[(long long)blockIdx.x * D + col] = red_b[0][col] + red_b[1][col] + red_b[2][col] + red_b[3][col];
    }
  }
  if constexpr (DROPO) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const int col = col_of<VEC>(c, lane, i);
        if (col < D) red_d[wid][col] = pd[c][i];
      }
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += 256)
      ldrop.part[(long long)blockIdx.x * D + col] = red_d[0][col] + red_d[1][col] + red_d[2][col] + red_d[3][col];
  }
}

// column sum: out[c] (+)= sum_r in[r][c]  (in: dtype dt, fp32 out).  Deterministic two-level.
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ in, long long ld, float* __restrict__ out,
                                                     int rows, int cols, int accum) {
  // block = 256 threads over 64 columns x 4 row-lanes
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (col < cols)
    for (int r = rl; r < rows; r += 4) s += to_f32(in[(long long)r * ld + col]);
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && col < cols) {
    float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    out[col] = accum ? out[col] + t : t;
  }
}

// second stage of the two-level column sums: out[c] (+)= sum_r part[r][c] over a short, wide fp32
// partial matrix (rows = #row blocks of the first stage).  256 threads = 8 float4 column groups x
// 32 row lanes per block; grid (cols/32, 2) reduces two matrices (dw, db) in one launch.  (The
// 64-column scalar form ran 12 blocks for D = 768 with a 128-deep dependent chain each: 34 us.)
__global__ __launch_bounds__(256) void colsum_partials_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                              float* __restrict__ o0, float* __restrict__ o1, int rows,
                                                              int cols, int accum) {
  const float* in = blockIdx.y ? p1 : p0;
  float* out = blockIdx.y ? o1 : o0;
  __shared__ float4 red[32][8];
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.x * 32 + cg * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < cols) {
#pragma unroll 4
    for (int r = rl; r < rows; r += 32) {
      const float4 v = *(const float4*)(in + (long long)r * cols + c);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[rl][cg] = acc;
  __syncthreads();
  if (rl < 4 && c < cols) {  // 4 x 8 threads: one column each, fixed summation order
    const int cc = c + rl;
    float t = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) {
      const float4 v = red[k][cg];
      t += rl == 0 ? v.x : (rl == 1 ? v.y : (rl == 2 ? v.z : v.w));
    }
    out[cc] = accum ? out[cc] + t : t;
  }
}

static void colsum_partials(const float* p0, const float* p1, float* o0, float* o1, int rows, int cols, int accum,
                            hipStream_t stream) {
  if (cols % 4 == 0) {
    colsum_partials_kernel<<<dim3((cols + 31) / 32, p1 ? 2 : 1), 256, 0, stream>>>(p0, p1, o0, o1, rows, cols, accum);
  } else {
    colsum_kernel<float><<<dim3((cols + 63) / 64), 256, 0, stream>>>(p0, cols, o0, rows, cols, accum);
    if (p1) colsum_kernel<float><<<dim3((cols + 63) / 64), 256, 0, stream>>>(p1, cols, o1, rows, cols, accum);
  }
}

// row-partitioned column sum for tall inputs: part[blk][c] = sum over blk's rows
template <typename T>
__global__ __launch_bounds__(256) void colsum_part_kernel(const T* __restrict__ in, long long ld,
                                                          float* __restrict__ part, int rows, int cols,
                                                          int rows_per_block) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float s = 0.f;
  if (col < cols)
    for (int r = r0 + rl; r < r1; r += 4) s += to_f32(in[(long long)r * ld + col]);
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && col < cols) part[(long long)blockIdx.y * cols + col] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// ------------------------------------------------------------------------------------
// softmax over rows of length L (materialised attention, fp32 parity path and VAE attn)
//   P = softmax(scale * S);  Pd = P * keep/(1-p) if dropout (else Pd may alias nothing)
// ------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ S, T* __restrict__ P,
                                                          T* __restrict__ Pd, long long rows, int L, float scale,
                                                          uint32_t thresh, float dscale, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* s = S + row * L;
  float m = -INFINITY;
  for (int j = lane; j < L; j += 64) m = fmaxf(m, to_f32(s[j]) * scale);
  m = wave_max(m);
  float sum = 0.f;
  for (int j = lane; j < L; j += 64) sum += __expf(to_f32(s[j]) * scale - m);
  sum = wave_sum(sum);
  const float inv = 1.0f / sum;
  for (int j = lane; j < L; j += 64) {
    float p = __expf(to_f32(s[j]) * scale - m) * inv;
    P[row * L + j] = from_f32<T>(p);
    if (Pd) {
      float pd = dropout_keep(seed, (uint64_t)(row * L + j), thresh) ? p * dscale : 0.f;
      Pd[row * L + j] = from_f32<T>(pd);
    }
  }
}

// dS = scale * P * (dP' - sum_j P*dP'),  dP' = dPd * keep/(1-p)
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ P, const T* __restrict__ dPd,
                                                          T* __restrict__ dS, long long rows, int L, float scale,
                                                          uint32_t thresh, float dscale, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float dot = 0.f;
  for (int j = lane; j < L; j += 64) {
    float dp = to_f32(dPd[row * L + j]);
    if (thresh) dp = dropout_keep(seed, (uint64_t)(row * L + j), thresh) ? dp * dscale : 0.f;
    dot += dp * to_f32(P[row * L + j]);
  }
  dot = wave_sum(dot);
  for (int j = lane; j < L; j += 64) {
    float dp = to_f32(dPd[row * L + j]);
    if (thresh) dp = dropout_keep(seed, (uint64_t)(row * L + j), thresh) ? dp * dscale : 0.f;
    dS[row * L + j] = from_f32<T>(scale * to_f32(P[row * L + j]) * (dp - dot));
  }
}

// =====================================================================================
// C ABI
// =====================================================================================
#define DISPATCH_LNB(TI, TO, TD, ...)                                                       \
  do {                                                                                       \
    if (D == 768) {                                                                          \
      ln_bwd<TI, TO, 4, 3, TD><<<grid, 256, 0, stream>>>(__VA_ARGS__);                       \
    } else if (D % 256 == 0 && D <= 1024) {                                                  \
      ln_bwd<TI, TO, 4, 4, TD><<<grid, 256, 0, stream>>>(__VA_ARGS__);                       \
    } else if (D <= 1024) {                                                                  \
      ln_bwd<TI, TO, 1, 16, TD><<<grid, 256, 0, stream>>>(__VA_ARGS__);                      \
    } else {                                                                                 \
      return (int)hipErrorInvalidValue;                                                      \
    }                                                                                        \
  } while (0)

#define DISPATCH_LN(KERNEL, TI, TO, ...)                                                    \
  do {                                                                                       \
    if (D == 768) { /* the Block width: three 4-wide chunks per lane, no idle fourth chunk */ \
      KERNEL<TI, TO, 4, 3><<<grid, 256, 0, stream>>>(__VA_ARGS__);                           \
    } else if (D % 256 == 0 && D <= 1024) {                                                  \
      KERNEL<TI, TO, 4, 4><<<grid, 256, 0, stream>>>(__VA_ARGS__);                           \
    } else if (D <= 1024) {                                                                  \
      KERNEL<TI, TO, 1, 16><<<grid, 256, 0, stream>>>(__VA_ARGS__);                          \
    } else {                                                                                 \
      return (int)hipErrorInvalidValue;                                                      \
    }                                                                                        \
  } while (0)

extern "C" int uva_layernorm_fwd(int in_dtype, int out_dtype, const void* x, const float* w, const float* b,
                                 const void* scale, const void* shift, long long ldm, void* y, float* mean,
                                 float* rstd, int rows, int D, float eps, hipStream_t stream) {
  if (rows <= 0) return 0;
  dim3 grid((rows + 3) / 4);
  if (in_dtype == UVA_DT_F32 && out_dtype == UVA_DT_F32)
    DISPATCH_LN(ln_fwd, float, float, (const float*)x, w, b, (const float*)scale, (const float*)shift, ldm,
                (float*)y, mean, rstd, rows, D, eps);
  else if (in_dtype == UVA_DT_F32 && out_dtype == UVA_DT_BF16)
    DISPATCH_LN(ln_fwd, float, bf16, (const float*)x, w, b, (const bf16*)scale, (const bf16*)shift, ldm, (bf16*)y,
                mean, rstd, rows, D, eps);
  else if (in_dtype == UVA_DT_BF16 && out_dtype == UVA_DT_BF16)
    DISPATCH_LN(ln_fwd, bf16, bf16, (const bf16*)x, w, b, (const bf16*)scale, (const bf16*)shift, ldm, (bf16*)y,
                mean, rstd, rows, D, eps);
  else
    return (int)hipErrorInvalidValue;
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_layernorm_bwd(int in_dtype, int out_dtype, const void* x, const float* w, const float* b,
                                 const void* scale,
                                 long long ldm, const void* dy, int dy_dtype, const float* mean, const float* rstd,
                                 const float* dx_base, float* dx, int accum, void* dscale, void* dshift, float* dw, float* db, int accum_wb,
                                 float* workspace, int rows, int D, hipStream_t stream) {
  if (rows <= 0) return 0;
  // dw/db via per-block partials in `workspace` (nblk * D * 2 floats), then a column sum
  const int rpb = 64;
  const int nblk = (rows + rpb - 1) / rpb;
  dim3 grid(nblk);
  float* pw = dw ? workspace : nullptr;
  float* pb = dw ? workspace + (long long)nblk * D : nullptr;
#define LNB_DY(TI, TO)                                                                                          \
  do {                                                                                                          \
    if (dy_dtype == UVA_DT_BF16)                                                                                \
      DISPATCH_LNB(TI, TO, bf16, (const TI*)x, w, b, (const TO*)scale, ldm, (const bf16*)dy, mean, rstd, dx_base, \
                   dx, accum, (TO*)dscale, (TO*)dshift, pw, pb, rows, D, rpb);                                  \
    else                                                                                                        \
      DISPATCH_LNB(TI, TO, float, (const TI*)x, w, b, (const TO*)scale, ldm, (const float*)dy, mean, rstd,        \
                   dx_base, dx, accum, (TO*)dscale, (TO*)dshift, pw, pb, rows, D, rpb);                         \
  } while (0)
  if (in_dtype == UVA_DT_F32 && out_dtype == UVA_DT_F32)
    LNB_DY(float, float);
  else if (in_dtype == UVA_DT_F32 && out_dtype == UVA_DT_BF16)
    LNB_DY(float, bf16);
  else if (in_dtype == UVA_DT_BF16 && out_dtype == UVA_DT_BF16)
    LNB_DY(bf16, bf16);
  else
    return (int)hipErrorInvalidValue;
#undef LNB_DY
  UVA_LAUNCH_CHECK();
  if (dw) {
    colsum_partials(pw, db ? pb : nullptr, dw, db, nblk, D, accum_wb, stream);
    UVA_LAUNCH_CHECK();
  }
  return 0;
}

// uva_layernorm_bwd for the timm Block's norm2 (fp32 x / dx, bf16 dy, D = 768, affine, dx_base) that also
// emits bf16(drop(dx)) -> drop_out and adds its column sums to dbias (proj_drop backward + the proj bias
// gradient, one pass instead of a second read of dx).  workspace: 3 * ceil(rows / 64) * D floats.
// Other shapes return hipErrorInvalidValue (callers use the two-pass route).
extern "C" int uva_layernorm_bwd_drop(const float* x, const float* w, const void* dy, const float* mean,
                                      const float* rstd, const float* dx_base, float* dx, float* dw, float* db,
                                      int accum_wb, void* drop_out, float drop_p, unsigned long long seed,
                                      float* dbias, int accum_dbias, float* workspace, int rows, int D,
                                      hipStream_t stream) {
  if (rows <= 0) return 0;
  if (D != 768 || !w || !dw || !db || !drop_out || !dbias || !workspace || ((uintptr_t)drop_out % 8))
    return (int)hipErrorInvalidValue;
  const int rpb = 64;
  const int nblk = (rows + rpb - 1) / rpb;
  float* pw = workspace;
  float* pb = workspace + (long long)nblk * D;
  float* pd = workspace + 2LL * nblk * D;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  LnDrop ld{(bf16*)drop_out, pd, drop_key(seed), th, ds};
  ln_bwd<float, float, 4, 3, bf16, true><<<dim3(nblk), 256, 0, stream>>>(
      x, w, nullptr, (const float*)nullptr, 0, (const bf16*)dy, mean, rstd, dx_base, dx, 0, (float*)nullptr,
      (float*)nullptr, pw, pb, rows, D, rpb, ld);
  UVA_LAUNCH_CHECK();
  colsum_partials(pw, pb, dw, db, nblk, D, accum_wb, stream);
  UVA_LAUNCH_CHECK();
  colsum_partials(pd, nullptr, dbias, nullptr, nblk, D, accum_dbias, stream);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" long long uva_layernorm_bwd_workspace(int rows, int D) {
  const int rpb = 64;
  return (long long)((rows + rpb - 1) / rpb) * D * 2;  // floats
}

// out[c] (+)= sum_r in[r*ld + c]; tall inputs go through a partial buffer (floats: ceil(rows/512)*cols)
int uva_colsum_vec(int dtype, const void* in, long long ld, float* out, int rows, int cols, int accum,
                   float* workspace, hipStream_t s);  // elementwise.hip

extern "C" int uva_colsum(int dtype, const void* in, long long ld, float* out, int rows, int cols, int accum,
                          float* workspace, hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return 0;
  {
    const int r = uva_colsum_vec(dtype, in, ld, out, rows, cols, accum, workspace, stream);
    if (r < 0) return (int)hipErrorLaunchFailure;
    if (r > 0) return 0;
  }
  const int rpb = 512;
  int nb = (rows + rpb - 1) / rpb;
  dim3 g1((cols + 63) / 64, nb);
  if (nb > 1 && workspace) {
    if (dtype == UVA_DT_BF16) colsum_part_kernel<bf16><<<g1, 256, 0, stream>>>((const bf16*)in, ld, workspace, rows, cols, rpb);
    else colsum_part_kernel<float><<<g1, 256, 0, stream>>>((const float*)in, ld, workspace, rows, cols, rpb);
    colsum_partials(workspace, nullptr, out, nullptr, nb, cols, accum, stream);
  } else {
    if (dtype == UVA_DT_BF16) colsum_kernel<bf16><<<dim3((cols + 63) / 64), 256, 0, stream>>>((const bf16*)in, ld, out, rows, cols, accum);
    else colsum_kernel<float><<<dim3((cols + 63) / 64), 256, 0, stream>>>((const float*)in, ld, out, rows, cols, accum);
  }
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" long long uva_colsum_workspace(int rows, int cols) {
  // max of the 512-row scalar path and the 128-row vectorized path (elementwise.hip COLSUM_RPB)
  return (long long)((rows + 127) / 128) * cols;
}

extern "C" int uva_softmax_fwd(int dtype, const void* S, void* P, void* Pd, long long rows, int L, float scale,
                               float drop_p, unsigned long long seed, hipStream_t stream) {
  if (rows <= 0) return 0;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == UVA_DT_BF16)
    softmax_fwd_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)S, (bf16*)P, th ? (bf16*)Pd : nullptr, rows, L, scale, th, ds, seed);
  else
    softmax_fwd_kernel<float><<<grid, 256, 0, stream>>>((const float*)S, (float*)P, th ? (float*)Pd : nullptr, rows, L, scale, th, ds, seed);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_softmax_bwd(int dtype, const void* P, const void* dPd, void* dS, long long rows, int L, float scale,
                               float drop_p, unsigned long long seed, hipStream_t stream) {
  if (rows <= 0) return 0;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == UVA_DT_BF16)
    softmax_bwd_kernel<bf16><<<grid, 256, 0, stream>>>((const bf16*)P, (const bf16*)dPd, (bf16*)dS, rows, L, scale, th, ds, seed);
  else
    softmax_bwd_kernel<float><<<grid, 256, 0, stream>>>((const float*)P, (const float*)dPd, (float*)dS, rows, L, scale, th, ds, seed);
  UVA_LAUNCH_CHECK();
  return 0;
}
