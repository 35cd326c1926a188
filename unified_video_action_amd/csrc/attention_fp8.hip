// FP8 (OCP e4m3) attention forward for the "fp8_attn" precision (BASELINE config 5, UMI-multi):
// the same timm Attention / SDPA (mar_con_unified.py:201-249) with Q.K^T and P.V as
// v_mfma_f32_16x16x32_fp8_fp8 products, fp32 accumulation and fp32 online softmax.
//
// Scaling: per (batch, head, q|k|v, 64-row tile) power-of-two scales 2^e with amax * 2^-e <= 448
// (uva_attn_quant_fp8, one pass over the qkv GEMM output).  The same pass rounds the bf16 qkv
// IN PLACE to the fp8 grid (x~ = fp8(x * 2^-e) * 2^e, exact in bf16), so the backward -- the bf16
// FA2 kernels of attention.hip run on x~ with this forward's log-sum-exp -- differentiates the
// function the forward evaluated (straight-through estimator for the rounding), and writes
//   qk8 [B, N, 2, H, 64]  fp8 Q / K (row-major, the MFMA A / B fragments are 8 contiguous bytes)
//   v8t [B, H, 64, N]     fp8 V^T, keys permuted inside every 32-key group so the P.V A-fragment
//                         (8 keys of one d row, in the order the S accumulators pack them) is 8
//                         contiguous bytes: position 8g + j holds key j < 4 ? 4g + j : 16 + 4g + j - 4
//   sc   [B, 3, H, N/64]  the fp32 scales 2^e.
// Forward (same lane layout as attention.hip: S^T = K Q^T, so each lane owns one query and P^T is
// already the B operand of O^T = V^T P^T): the Q.K scales fold into the softmax constant per
// 64-key sub-tile (c' = c * sq * sk); P (<= 2^8 with the lazy max rescale) is converted to e4m3
// unscaled after multiplying by 2^(ev - E), E = the largest V scale seen so far for the row
// block (O is rescaled by the exact power of two when E grows), and O is multiplied by E at the end.
// The row sums use the unrounded fp32 P, so the log-sum-exp matches an fp32 softmax of x~.
#include "common.h"

#define A8_MAX 448.0f

typedef long fp8x8;  // 8 e4m3 values (one 16x16x32 MFMA operand fragment)

__device__ __forceinline__ f32x4 mfma8(fp8x8 a, fp8x8 b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
}

// 4 floats -> 4 e4m3 bytes (round to nearest even, saturating)
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, p, true);
}

// position of key r (0..31) inside its permuted 32-key group (inverse of 8g + j -> key)
__host__ __device__ constexpr int v8_pos(int r) {
  return r < 16 ? 8 * (r >> 2) + (r & 3) : 8 * ((r - 16) >> 2) + 4 + ((r - 16) & 3);
}

// =====================================================================================
// quantisation: one workgroup per (64-row tile, q|k|v, batch*head)
// =====================================================================================
__global__ __launch_bounds__(256) void attn_quant_fp8_kernel(bf16* __restrict__ qkv, uint8_t* __restrict__ qk8,
                                                             uint8_t* __restrict__ v8t, float* __restrict__ sc, int N,
                                                             int H) {
  __shared__ float red[4];
  __shared__ __attribute__((aligned(16))) uint8_t tr[64 * 64];
  const int tile = blockIdx.x, t = blockIdx.y, bh = blockIdx.z, b = bh / H, h = bh % H;
  const int tid = threadIdx.x, row = tid >> 2, col = (tid & 3) * 16;
  const int q = tile * 64 + row;
  const long long ld = 3LL * H * 64;
  bf16* src = qkv + ((long long)b * N + q) * ld + (long long)t * H * 64 + h * 64 + col;
  bf16x8 x0 = *(const bf16x8*)src, x1 = *(const bf16x8*)(src + 8);
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fmaxf(fabsf((float)x0[j]), fabsf((float)x1[j])));
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  // smallest e with amax * 2^-e <= 448 (e = 0 for an all-zero tile)
  int e = 0;
  if (amax > 0.f) {
    e = (int)ceilf(log2f(amax / A8_MAX));
    while (ldexpf(amax, -e) > A8_MAX) ++e;
    while (ldexpf(amax, -(e - 1)) <= A8_MAX) --e;
  }
  const float inv = ldexpf(1.f, -e), s = ldexpf(1.f, e);
  int w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bf16x8& xv = k < 2 ? x0 : x1;
    const int o = (k & 1) * 4;
    w[k] = pack4_fp8((float)xv[o] * inv, (float)xv[o + 1] * inv, (float)xv[o + 2] * inv, (float)xv[o + 3] * inv);
  }
  // x~ = fp8 value * 2^e, written back in place (exact in bf16)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bf16x8& xv = k < 2 ? x0 : x1;
    const int o = (k & 1) * 4;
    xv[o + 0] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w[k], 0) * s);
    xv[o + 1] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w[k], 1) * s);
    xv[o + 2] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w[k], 2) * s);
    xv[o + 3] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w[k], 3) * s);
  }
  *(bf16x8*)src = x0;
  *(bf16x8*)(src + 8) = x1;
  if (t < 2) {
    uint8_t* dst = qk8 + (((long long)b * N + q) * 2 + t) * (H * 64) + h * 64 + col;
    *(int4*)dst = (int4){w[0], w[1], w[2], w[3]};
  } else {
    // V^T: this thread holds V[q][col .. col + 15]; scatter the bytes to [d][permuted key] in LDS
    const int pos = (row & ~31) + v8_pos(row & 31);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) tr[(col + 4 * k + j) * 64 + pos] = (uint8_t)((unsigned)w[k] >> (8 * j));
    __syncthreads();
    const int d = tid >> 2, c16 = (tid & 3) * 16;
    uint8_t* dst = v8t + ((long long)bh * 64 + d) * N + tile * 64 + c16;
    *(int4*)dst = *(const int4*)(tr + d * 64 + c16);
  }
  if (tid == 0) sc[((long long)(b * 3 + t) * H + h) * (N / 64) + tile] = s;
}

// LDS images (no padding: LDS-DMA writes 1 KiB lane-linear pieces), 16-B chunk c of row r stored
// at slot c ^ f(r): 64-B rows f = (r >> 2) & 3, 128-B rows f = (r >> 1) & 7 -- the 16 rows x one
// 16-B chunk that a 32-lane half of a fragment read touches then cover all 64 banks once.
template <int RB>
__device__ __forceinline__ int a8_swz(int r) {
  return RB == 64 ? ((r >> 2) & 3) : ((r >> 1) & 7);
}

// K tile [KT keys][64 B] and V^T tile [64 d][KT B] of key tile kv -> LDS by global_load_lds
// (16 B per lane; the swizzle is applied on the per-lane source address)
template <int KT>
__device__ __forceinline__ void a8_dma(const uint8_t* __restrict__ Kg, const uint8_t* __restrict__ Vg, long long ldq,
                                       int N, int kv, uint8_t* sK, uint8_t* sV) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  constexpr int NI = KT * 64 / 1024 / 4;  // 1-KiB wave instructions per wave, per image
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = ((w * NI + i) * 64 + l) * 16;
    const int r = e >> 6, c = ((e >> 4) & 3) ^ a8_swz<64>(r);
    __builtin_amdgcn_global_load_lds((const void*)(Kg + (long long)(kv * KT + r) * ldq + c * 16),
                                     (__attribute__((address_space(3))) void*)(sK + (w * NI + i) * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = ((w * NI + i) * 64 + l) * 16;
    const int r = e / KT, c = ((e % KT) >> 4) ^ a8_swz<KT>(r);
    __builtin_amdgcn_global_load_lds((const void*)(Vg + (long long)r * N + kv * KT + c * 16),
                                     (__attribute__((address_space(3))) void*)(sV + (w * NI + i) * 1024), 16, 0, 0);
  }
}

// 8-byte fragment of row r, byte columns [32 s + 8 g, +8) of an image with RB-byte rows
template <int RB>
__device__ __forceinline__ fp8x8 a8_frag(const uint8_t* img, int r, int s, int g) {
  const int c = (2 * s + (g >> 1)) ^ a8_swz<RB>(r);
  return *(const fp8x8*)(img + r * RB + c * 16 + 8 * (g & 1));
}

// =====================================================================================
// forward: 4 waves x 32 queries per workgroup, KT keys per LDS tile (64 or 128)
// =====================================================================================
template <bool DROP, int KT>
__global__ __launch_bounds__(256, 2) void attn_fwd_fp8_kernel(const uint8_t* __restrict__ qk8,
                                                           const uint8_t* __restrict__ v8t,
                                                           const float* __restrict__ sc, bf16* __restrict__ out,
                                                           float* __restrict__ lse2, const uint64_t* __restrict__ MQ,
                                                           int N, int H, float c, float dsc) {
  constexpr int NKT = KT / 16;   // 16-key MFMA tiles per LDS tile
  constexpr int NH = KT / 64;    // 64-key sub-tiles (scale / mask-word granules) per LDS tile
  // one LDS array (a second __shared__ object beside LDS-DMA targets can cost vmcnt(0) waits)
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * 2 * KT * 64];
  auto sK = [&](int b) { return smem + b * 2 * KT * 64; };
  auto sV = [&](int b) { return smem + b * 2 * KT * 64 + KT * 64; };
  int bx, bh;
  xcd_grid2(bx, bh);
  const int b = bh / H, h = bh % H;
  const int nt64 = N / 64;
  const long long ldq = 2LL * H * 64;
  const uint8_t* Qg = qk8 + (long long)b * N * ldq + h * 64;
  const uint8_t* Kg = Qg + H * 64;
  const uint8_t* Vg = v8t + (long long)bh * 64 * N;
  const float* sq_ = sc + ((long long)(b * 3 + 0) * H + h) * nt64;
  const float* sk_ = sc + ((long long)(b * 3 + 1) * H + h) * nt64;
  const float* sv_ = sc + ((long long)(b * 3 + 2) * H + h) * nt64;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, g = l >> 4, li = l & 15;
  const int q0 = bx * 128 + w * 32;
  const int nkv = N / KT;
  const uint16_t* mq = DROP ? (const uint16_t*)(MQ + (long long)bh * nt64 * N) : nullptr;

  fp8x8 qf[2][2];
  uint32_t mw[2][NH], mwn[2][NH];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int row = q0 + qt * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = row < N ? *(const fp8x8*)(Qg + (long long)row * ldq + ks * 32 + 8 * g) : 0;
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      mw[qt][hh] = (DROP && row < N) ? mq[((long long)hh * N + row) * 4 + g] : 0u;
      mwn[qt][hh] = 0u;
    }
  }
  const float cq = c * (q0 < N ? sq_[q0 >> 6] : 1.f);  // the wave's 32 queries share one 64-row tile
  float m[2] = {-INFINITY, -INFINITY}, rs[2] = {0.f, 0.f};
  float E = 0.f;  // largest V scale folded into O so far (0 = none yet)
  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  a8_dma<KT>(Kg, Vg, ldq, N, 0, sK(0), sV(0));
  __syncthreads();
  int cur = 0;
  for (int kv = 0; kv < nkv; ++kv) {
    const bool more = kv + 1 < nkv;
    if (more) {
      a8_dma<KT>(Kg, Vg, ldq, N, kv + 1, sK(cur ^ 1), sV(cur ^ 1));
      if (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const int row = q0 + qt * 16 + li;
#pragma unroll
          for (int hh = 0; hh < NH; ++hh)
            mwn[qt][hh] = row < N ? mq[((long long)((kv + 1) * NH + hh) * N + row) * 4 + g] : 0u;
        }
      }
    }
    const uint8_t* cK = sK(cur);
    const uint8_t* cV = sV(cur);
    float ck[NH], sv[NH];
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      ck[hh] = cq * sk_[kv * NH + hh];
      sv[hh] = sv_[kv * NH + hh];
    }
    f32x4 s[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const fp8x8 kf = a8_frag<64>(cK, kt * 16 + li, ks, g);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s[kt][qt] = mfma8(kf, qf[qt][ks], s[kt][qt]);
      }
    }
    // row max of the scaled scores: the scales are positive, so max(s * ck) = max over sub-tiles of
    // ck * max(s) -- no per-element multiply (it folds into the exp's fma below)
    float mx[2];
    bool need = false;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float a = -INFINITY;
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        float t = __builtin_amdgcn_fmed3f(s[hh * 4][qt][0], s[hh * 4][qt][1], INFINITY);
#pragma unroll
        for (int kt = hh * 4; kt < hh * 4 + 4; ++kt)
#pragma unroll
          for (int r = (kt == hh * 4 ? 2 : 0); r < 4; ++r) t = __builtin_amdgcn_fmed3f(t, s[kt][qt][r], INFINITY);
        a = fmaxf(a, t * ck[hh]);
      }
      a = fmaxf(a, __shfl_xor(a, 16, 64));
      a = fmaxf(a, __shfl_xor(a, 32, 64));
      mx[qt] = a;
      need |= mx[qt] > m[qt] + 8.0f;
    }
    if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const float mnew = fmaxf(m[qt], mx[qt]);
        const float alpha = __builtin_amdgcn_exp2f(m[qt] - mnew);
        rs[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] = mnew;
      }
    }
    // V scale: fold the tile's 2^ev relative to the running largest E into P (exact powers of two)
    float vmax = sv[0];
#pragma unroll
    for (int hh = 1; hh < NH; ++hh) vmax = fmaxf(vmax, sv[hh]);
    if (vmax > E) {
      if (E > 0.f) {
        const float r = E / vmax;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= r;
      }
      E = vmax;
    }
    // p' = exp2(s * ck - m + log2(sv / E)) in one fma + exp; the row sum is kept per sub-tile in
    // those units and brought back by E / sv once per sub-tile
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        const float lp = __builtin_amdgcn_logf(sv[hh] / E);  // log2 of a power of two <= 1: exact
        const float nm = lp - m[qt];
        float part = 0.f;
#pragma unroll
        for (int kt = hh * 4; kt < hh * 4 + 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[kt][qt][r], ck[hh], nm));
            part += p;
            s[kt][qt][r] = DROP ? __int_as_float(__float_as_int(p) & __builtin_amdgcn_sbfe(mw[qt][hh], (kt & 3) * 4 + r, 1))
                                : p;
          }
        rs[qt] += part * (E / sv[hh]);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KT / 32; ++ks) {
      fp8x8 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const f32x4& a = s[2 * ks][qt];
        const f32x4& e = s[2 * ks + 1][qt];
        const unsigned lo = (unsigned)pack4_fp8(a[0], a[1], a[2], a[3]);
        const unsigned hi = (unsigned)pack4_fp8(e[0], e[1], e[2], e[3]);
        pf[qt] = (fp8x8)(((unsigned long long)hi << 32) | lo);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const fp8x8 vf = a8_frag<KT>(cV, dt * 16 + li, ks, g);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma8(vf, pf[qt], o[qt][dt]);
      }
    }
    if (more) {
      if (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int hh = 0; hh < NH; ++hh) mw[qt][hh] = mwn[qt][hh];
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  const long long ldo = (long long)H * 64;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float lsum = rs[qt];
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const int q = q0 + qt * 16 + li;
    if (q >= N) continue;
    const float inv = dsc * E / lsum;
    bf16* orow = out + ((long long)b * N + q) * ldo + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v = {(bf16)(o[qt][dt][0] * inv), (bf16)(o[qt][dt][1] * inv), (bf16)(o[qt][dt][2] * inv),
                  (bf16)(o[qt][dt][3] * inv)};
      *(bf16x4*)(orow + dt * 16 + 4 * g) = v;
    }
    if (g == 0) lse2[(long long)bh * N + q] = m[qt] + __log2f(lsum);
  }
}

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" long long uva_attn_fp8_workspace(int B, int N, int H) {
  // qk8 (2 B N H 64) + v8t (B H 64 N) bytes, then the scales (B 3 H N/64 floats), 256-B aligned
  const long long a = 3LL * B * N * H * 64;
  return ((a + 255) / 256) * 256 + 4LL * B * 3 * H * (N / 64);
}

extern "C" int uva_attn_quant_fp8(void* qkv, void* workspace, int B, int N, int H, hipStream_t s) {
  if (N % 64 != 0 || workspace == nullptr || ((uintptr_t)qkv % 16) || ((uintptr_t)workspace % 256))
    return (int)hipErrorInvalidValue;
  uint8_t* qk8 = (uint8_t*)workspace;
  uint8_t* v8t = qk8 + 2LL * B * N * H * 64;
  float* sc = (float*)((uint8_t*)workspace + (3LL * B * N * H * 64 + 255) / 256 * 256);
  attn_quant_fp8_kernel<<<dim3(N / 64, 3, B * H), 256, 0, s>>>((bf16*)qkv, qk8, v8t, sc, N, H);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_attn_fwd_fp8(const void* workspace, void* out, float* lse2, const void* mask, int B, int N, int H,
                                float scale, float drop_p, hipStream_t s) {
  if (N % 64 != 0 || workspace == nullptr) return (int)hipErrorInvalidValue;
  const bool drop = drop_p > 0.f;
  if (drop && mask == nullptr) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const uint8_t* qk8 = (const uint8_t*)workspace;
  const uint8_t* v8t = qk8 + 2LL * B * N * H * 64;
  const float* sc = (const float*)((const uint8_t*)workspace + (3LL * B * N * H * 64 + 255) / 256 * 256);
  dim3 grid((N + 127) / 128, B * H);
  const float c = scale * 1.4426950408889634f;
  const uint64_t* MQ = drop ? (const uint64_t*)mask : nullptr;
  const bool k128 = N % 128 == 0;
#define A8L(D, K) attn_fwd_fp8_kernel<D, K><<<grid, 256, 0, s>>>(qk8, v8t, sc, (bf16*)out, lse2, MQ, N, H, c, D ? ds : 1.0f)
  if (drop && k128) A8L(true, 128);
  else if (drop) A8L(true, 64);
  else if (k128) A8L(false, 128);
  else A8L(false, 64);
#undef A8L
  UVA_LAUNCH_CHECK();
  return 0;
}
