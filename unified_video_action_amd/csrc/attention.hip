// Fused multi-head attention (non-causal, head_dim 64, bf16 in/out, fp32 softmax) for the
// 24 timm Blocks of the MAR (mar_con_unified.py:201-249; timm Attention = SDPA with
// dropout_p = attn_drop while training).  Reads Q/K/V straight from the qkv GEMM output
// [B, N, 3, H, 64] and writes O as [B, N, H, 64] (the proj GEMM input) -- no permutes.
//
// Layout trick (CDNA4 v_mfma_f32_16x16x32_bf16, 64-lane waves): scores are computed
// transposed, S^T = K Q^T, so each lane owns one query column (lane & 15) and 16 keys in
// registers.  P^T then feeds O^T = V^T P^T directly as the B operand (no LDS round trip):
// the k order inside each 32-deep step is the permutation pi(8g+j) = tileA*16+4g+j (j<4),
// tileB*16+4g+j-4 (j>=4), matched on the V side by choosing the row bases of the two
// ds_read_b64_tr_b16 transposed reads.  Softmax statistics are per lane (query), so the
// O^T rescale needs no shuffles.  K/V tiles (64 keys) are register-staged into
// double-buffered LDS ([row][72] bf16 images serve both row and transposed reads).
//
// Backward (FA2 recompute, two kernels, no atomics):
//   attn_bwd_dkdv : block = 128 keys, sweeps all query tiles -> dK, dV
//   attn_bwd_dq   : block = 128 queries, sweeps all key tiles -> dQ
// Dropout keep-mask = counter hash of ((b*H+h)*N + q)*N + key, identical in all kernels
// and in the materialised fp32 path (norm.hip softmax kernels).
#include "common.h"

#define AT_LD 72
#define AT_TILE (64 * AT_LD)

__device__ __forceinline__ bf16x8 lds_row_frag(const bf16* lds, int row0, int ks) {
  const int l = threadIdx.x & 63;
  return *(const bf16x8*)(lds + (row0 + (l & 15)) * AT_LD + ks * 32 + 8 * (l >> 4));
}

__device__ __forceinline__ bf16x8 lds_tr_frag(const bf16* lds, int rowA, int rowB, int col0) {
  const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const bf16* a0 = lds + (rowA + 4 * g + q) * AT_LD + col0 + 4 * p;
  const bf16* a1 = lds + (rowB + 4 * g + q) * AT_LD + col0 + 4 * p;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_pi(const f32x4& a, const f32x4& b) {
  bf16x8 r = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)b[0], (bf16)b[1], (bf16)b[2], (bf16)b[3]};
  return r;
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 64 rows x 64 cols of a strided bf16 matrix -> 2 chunks (16 B) per thread
__device__ __forceinline__ void stage_load(const bf16* __restrict__ g, long long ld, int row0, int nrows,
                                           bf16x8 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int id = t + i * 256, row = id >> 3, c = (id & 7) * 8;
    r[i] = (row0 + row < nrows) ? *(const bf16x8*)(g + (long long)(row0 + row) * ld + c) : (bf16x8){};
  }
}
__device__ __forceinline__ void stage_store(bf16* lds, const bf16x8 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int id = t + i * 256, row = id >> 3, c = (id & 7) * 8;
    *(bf16x8*)(lds + row * AT_LD + c) = r[i];
  }
}

__device__ __forceinline__ float drop_apply(float v, bool on, uint64_t seed, uint64_t idx, uint32_t th, float ds) {
  if (!on) return v;
  return dropout_keep(seed, idx, th) ? v * ds : 0.f;
}

// =====================================================================================
// forward
// =====================================================================================
__global__ __launch_bounds__(256) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                       float* __restrict__ lse2, int N, int H, float scale_log2,
                                                       uint32_t th, float dsc, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) bf16 sK[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][AT_TILE];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int q0 = blockIdx.x * 128 + w * 32;
  const bool drop = th != 0;

  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      int row = q0 + qt * 16 + li;
      qf[qt][ks] = row < N ? *(const bf16x8*)(Qg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
    }
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};
  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rk[2], rv[2];
  stage_load(Kg, ld, 0, N, rk);
  stage_load(Vg, ld, 0, N, rv);
  stage_store(sK[0], rk);
  stage_store(sV[0], rv);
  __syncthreads();
  const int nkv = N / 64;
  int cur = 0;
  for (int kv = 0; kv < nkv; ++kv) {
    const bool more = kv + 1 < nkv;
    if (more) {
      stage_load(Kg, ld, (kv + 1) * 64, N, rk);
      stage_load(Vg, ld, (kv + 1) * 64, N, rv);
    }
    f32x4 s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 kf[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) kf[kt] = lds_row_frag(sK[cur], kt * 16, ks);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s[kt][qt] = mfma16(kf[kt], qf[qt][ks], s[kt][qt]);
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m[qt], mx * scale_log2);
      const float alpha = exp2f(m[qt] - mnew);
      float rs = 0.f;
      const long long qrow = (long long)bh * N + (q0 + qt * 16 + li);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = exp2f(s[kt][qt][r] * scale_log2 - mnew);
          rs += p;
          s[kt][qt][r] = p;
        }
        if (drop) {  // lane owns 4 consecutive keys: two mask pairs
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            bool k0, k1;
            dropout_keep2(seed, (uint64_t)(qrow * N + kv * 64 + kt * 16 + 4 * g + r), th, k0, k1);
            s[kt][qt][r] = k0 ? s[kt][qt][r] * dsc : 0.f;
            s[kt][qt][r + 1] = k1 ? s[kt][qt][r + 1] * dsc : 0.f;
          }
        }
      }
      rs += __shfl_xor(rs, 16, 64);
      rs += __shfl_xor(rs, 32, 64);
      lsum[qt] = lsum[qt] * alpha + rs;
      m[qt] = mnew;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) pf[qt] = pack_pi(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 vf = lds_tr_frag(sV[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma16(vf, pf[qt], o[qt][dt]);
      }
    }
    if (more) {
      stage_store(sK[cur ^ 1], rk);
      stage_store(sV[cur ^ 1], rv);
    }
    __syncthreads();
    cur ^= 1;
  }
  const long long ldo = (long long)H * 64;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + li;
    if (q >= N) continue;
    const float inv = 1.0f / lsum[qt];
    bf16* orow = out + ((long long)b * N + q) * ldo + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v = {(bf16)(o[qt][dt][0] * inv), (bf16)(o[qt][dt][1] * inv), (bf16)(o[qt][dt][2] * inv),
                  (bf16)(o[qt][dt][3] * inv)};
      *(bf16x4*)(orow + dt * 16 + 4 * g) = v;
    }
    if (g == 0) lse2[(long long)bh * N + q] = m[qt] + __log2f(lsum[qt]);
  }
}

// Dvec[bh][q] = sum_d dO[q][d] * O[q][d]
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const bf16* __restrict__ out, const bf16* __restrict__ dout,
                                                           float* __restrict__ Dvec, int B, int N, int H) {
  const long long idx = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);  // (b, q, h)
  const int l = threadIdx.x & 63;
  if (idx >= (long long)B * N * H) return;
  const int h = idx % H;
  const long long bq = idx / H;
  const int b = bq / N, q = bq % N;
  float v = (float)out[idx * 64 + l] * (float)dout[idx * 64 + l];
  v = wave_sum(v);
  if (l == 0) Dvec[((long long)b * H + h) * N + q] = v;
}

// =====================================================================================
// backward: dK, dV  (block = 4 waves x 32 keys)
// =====================================================================================
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                            const float* __restrict__ lse2,
                                                            const float* __restrict__ Dvec, bf16* __restrict__ dqkv,
                                                            int N, int H, float scale, float scale_log2, uint32_t th,
                                                            float dsc, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) bf16 sQ[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sO[2][AT_TILE];
  __shared__ float sL[2][64], sD[2][64];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64, ldo = (long long)H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const bf16* dOg = dout + (long long)b * N * ldo + h * 64;
  const float* Lg = lse2 + (long long)bh * N;
  const float* Dg = Dvec + (long long)bh * N;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int k0 = blockIdx.x * 128 + w * 32;
  const bool drop = th != 0;

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      int row = k0 + kt * 16 + li;
      bool ok = row < N;
      kf[kt][ks] = ok ? *(const bf16x8*)(Kg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
      vf[kt][ks] = ok ? *(const bf16x8*)(Vg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
    }
  f32x4 dv[4][2], dk[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dv[dt][kt] = dk[dt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rq[2], ro[2];
  stage_load(Qg, ld, 0, N, rq);
  stage_load(dOg, ldo, 0, N, ro);
  stage_store(sQ[0], rq);
  stage_store(sO[0], ro);
  if (threadIdx.x < 64) { sL[0][threadIdx.x] = Lg[threadIdx.x]; sD[0][threadIdx.x] = Dg[threadIdx.x]; }
  __syncthreads();
  const int nq = N / 64;
  int cur = 0;
  for (int qi = 0; qi < nq; ++qi) {
    const bool more = qi + 1 < nq;
    float nl = 0.f, nd = 0.f;
    if (more) {
      stage_load(Qg, ld, (qi + 1) * 64, N, rq);
      stage_load(dOg, ldo, (qi + 1) * 64, N, ro);
      if (threadIdx.x < 64) { nl = Lg[(qi + 1) * 64 + threadIdx.x]; nd = Dg[(qi + 1) * 64 + threadIdx.x]; }
    }
    // S[q][key] = Q K^T ; dP[q][key] = dO V^T   (lane: q = qt*16+4g+r, key = kt*16+li)
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) s[qt][kt] = dp[qt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        bf16x8 a = lds_row_frag(sQ[cur], qt * 16, ks);
        bf16x8 c = lds_row_frag(sO[cur], qt * 16, ks);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qt][kt] = mfma16(a, kf[kt][ks], s[qt][kt]);
          dp[qt][kt] = mfma16(c, vf[kt][ks], dp[qt][kt]);
        }
      }
    // P, dropout, dS   (s <- Pd, dp <- dS)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = qt * 16 + 4 * g + r;
        const float L = sL[cur][ql], Dq = sD[cur][ql];
        const long long qrow = (long long)bh * N + qi * 64 + ql;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const float p = exp2f(s[qt][kt][r] * scale_log2 - L);
          float pd = p, dpt = dp[qt][kt][r];
          if (drop) {
            bool keep = dropout_keep(seed, (uint64_t)(qrow * N + k0 + kt * 16 + li), th);
            pd = keep ? p * dsc : 0.f;
            dpt = keep ? dpt * dsc : 0.f;
          }
          s[qt][kt][r] = pd;
          dp[qt][kt][r] = p * (dpt - Dq);
        }
      }
    // dV^T[d][key] += dO^T Pd ; dK^T[d][key] += Q^T dS      (k = q, permuted by pi)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        pb[kt] = pack_pi(s[2 * ks][kt], s[2 * ks + 1][kt]);
        sb[kt] = pack_pi(dp[2 * ks][kt], dp[2 * ks + 1][kt]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 oa = lds_tr_frag(sO[cur], 32 * ks, 32 * ks + 16, dt * 16);
        bf16x8 qa = lds_tr_frag(sQ[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[dt][kt] = mfma16(oa, pb[kt], dv[dt][kt]);
          dk[dt][kt] = mfma16(qa, sb[kt], dk[dt][kt]);
        }
      }
    }
    if (more) {
      stage_store(sQ[cur ^ 1], rq);
      stage_store(sO[cur ^ 1], ro);
      if (threadIdx.x < 64) { sL[cur ^ 1][threadIdx.x] = nl; sD[cur ^ 1][threadIdx.x] = nd; }
    }
    __syncthreads();
    cur ^= 1;
  }
  // lane holds [d = dt*16+4g+r][key = kt*16+li]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + kt * 16 + li;
    if (key >= N) continue;
    bf16* krow = dqkv + ((long long)b * N + key) * ld + H * 64 + h * 64;
    bf16* vrow = krow + H * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 a = {(bf16)(dk[dt][kt][0] * scale), (bf16)(dk[dt][kt][1] * scale), (bf16)(dk[dt][kt][2] * scale),
                  (bf16)(dk[dt][kt][3] * scale)};
      bf16x4 c = {(bf16)dv[dt][kt][0], (bf16)dv[dt][kt][1], (bf16)dv[dt][kt][2], (bf16)dv[dt][kt][3]};
      *(bf16x4*)(krow + dt * 16 + 4 * g) = a;
      *(bf16x4*)(vrow + dt * 16 + 4 * g) = c;
    }
  }
}

// =====================================================================================
// backward: dQ (block = 4 waves x 32 queries)
// =====================================================================================
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse2,
                                                          const float* __restrict__ Dvec, bf16* __restrict__ dqkv,
                                                          int N, int H, float scale, float scale_log2, uint32_t th,
                                                          float dsc, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) bf16 sK[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][AT_TILE];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64, ldo = (long long)H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const bf16* dOg = dout + (long long)b * N * ldo + h * 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int q0 = blockIdx.x * 128 + w * 32;
  const bool drop = th != 0;

  bf16x8 qf[2][2], of[2][2];
  float L[2], Dq[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    int row = q0 + qt * 16 + li;
    bool ok = row < N;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = ok ? *(const bf16x8*)(Qg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
      of[qt][ks] = ok ? *(const bf16x8*)(dOg + (long long)row * ldo + ks * 32 + 8 * g) : (bf16x8){};
    }
    L[qt] = ok ? lse2[(long long)bh * N + row] : 0.f;
    Dq[qt] = ok ? Dvec[(long long)bh * N + row] : 0.f;
  }
  f32x4 dq[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rk[2], rv[2];
  stage_load(Kg, ld, 0, N, rk);
  stage_load(Vg, ld, 0, N, rv);
  stage_store(sK[0], rk);
  stage_store(sV[0], rv);
  __syncthreads();
  const int nkv = N / 64;
  int cur = 0;
  for (int kv = 0; kv < nkv; ++kv) {
    const bool more = kv + 1 < nkv;
    if (more) {
      stage_load(Kg, ld, (kv + 1) * 64, N, rk);
      stage_load(Vg, ld, (kv + 1) * 64, N, rv);
    }
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = dp[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        bf16x8 ka = lds_row_frag(sK[cur], kt * 16, ks);
        bf16x8 va = lds_row_frag(sV[cur], kt * 16, ks);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          s[kt][qt] = mfma16(ka, qf[qt][ks], s[kt][qt]);
          dp[kt][qt] = mfma16(va, of[qt][ks], dp[kt][qt]);
        }
      }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const long long qrow = (long long)bh * N + (q0 + qt * 16 + li);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        bool keep[4] = {true, true, true, true};
        if (drop) {
#pragma unroll
          for (int r = 0; r < 4; r += 2)
            dropout_keep2(seed, (uint64_t)(qrow * N + kv * 64 + kt * 16 + 4 * g + r), th, keep[r], keep[r + 1]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2f(s[kt][qt][r] * scale_log2 - L[qt]);
          float dpt = dp[kt][qt][r];
          if (drop) dpt = keep[r] ? dpt * dsc : 0.f;
          s[kt][qt][r] = p * (dpt - Dq[qt]);
        }
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 sb[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) sb[qt] = pack_pi(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 ka = lds_tr_frag(sK[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = mfma16(ka, sb[qt], dq[dt][qt]);
      }
    }
    if (more) {
      stage_store(sK[cur ^ 1], rk);
      stage_store(sV[cur ^ 1], rv);
    }
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + li;
    if (q >= N) continue;
    bf16* qrow = dqkv + ((long long)b * N + q) * ld + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 a = {(bf16)(dq[dt][qt][0] * scale), (bf16)(dq[dt][qt][1] * scale), (bf16)(dq[dt][qt][2] * scale),
                  (bf16)(dq[dt][qt][3] * scale)};
      *(bf16x4*)(qrow + dt * 16 + 4 * g) = a;
    }
  }
}

static inline void drop_params(float p, uint32_t* th, float* ds) {
  uva_drop_params(p, th, ds);
}

extern "C" int uva_attn_fwd(const void* qkv, void* out, float* lse2, int B, int N, int H, float scale, float drop_p,
                            unsigned long long seed, hipStream_t s) {
  if (N % 64 != 0) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  drop_params(drop_p, &th, &ds);
  dim3 grid((N + 127) / 128, B * H);
  attn_fwd_kernel<<<grid, 256, 0, s>>>((const bf16*)qkv, (bf16*)out, lse2, N, H, scale * 1.4426950408889634f, th, ds,
                                       seed);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, float* Dvec,
                            void* dqkv, int B, int N, int H, float scale, float drop_p, unsigned long long seed,
                            hipStream_t s) {
  if (N % 64 != 0) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  drop_params(drop_p, &th, &ds);
  long long rows = (long long)B * N * H;
  attn_bwd_pre_kernel<<<dim3((unsigned)((rows + 3) / 4)), 256, 0, s>>>((const bf16*)out, (const bf16*)dout, Dvec, B, N,
                                                                        H);
  dim3 grid((N + 127) / 128, B * H);
  const float sl2 = scale * 1.4426950408889634f;
  attn_bwd_dkdv_kernel<<<grid, 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, lse2, Dvec, (bf16*)dqkv, N, H, scale,
                                            sl2, th, ds, seed);
  attn_bwd_dq_kernel<<<grid, 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, lse2, Dvec, (bf16*)dqkv, N, H, scale,
                                          sl2, th, ds, seed);
  UVA_LAUNCH_CHECK();
  return 0;
}
