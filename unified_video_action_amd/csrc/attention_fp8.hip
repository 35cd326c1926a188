// FP8 (OCP e4m3) attention forward for the "fp8_attn" precision (BASELINE config 5, UMI-multi):
// the same timm Attention / SDPA (mar_con_unified.py:201-249) with Q.K^T and P.V on the
// block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 operands: twice the bf16 MFMA rate; the
// non-scaled fp8 MFMAs run at the bf16 rate, MI355X_MICROARCH.md 'Matrix cores'), fp32
// accumulation and fp32 online softmax.
//
// Scaling: per (batch, head, q|k|v, 64-row tile) power-of-two scales 2^e with amax * 2^-e <= 448
// (uva_attn_quant_fp8, one pass over the qkv GEMM output).  The same pass rounds the bf16 qkv
// IN PLACE to the fp8 grid (x~ = fp8(x * 2^-e) * 2^e, exact in bf16), so the backward -- the bf16
// FA2 kernels of attention.hip run on x~ with this forward's log-sum-exp -- differentiates the
// function the forward evaluated (straight-through estimator for the rounding), and writes
//   qk8 [B, N, 2, H, 64]  fp8 Q / K (row-major: a lane's 32-byte operand is half a row)
//   v8t [B, H, 64, N]     fp8 V^T, keys permuted inside every 64-key tile so the P.V A operand
//                         (32 keys of one d row, in the order the S accumulators pack them) is 32
//                         contiguous bytes: position 32h + 16s + i holds key 32s + (i&3) + 8(i>>2) + 4h
//   sc   [B, 3, H, N/64]  the fp32 scales 2^e.
// The scales are the MFMAs' own e8m0 block scales (uniform per 64-row tile = per operand block),
// so S and O come out of the matrix core already scaled: no per-element multiplies, no running
// V-scale bookkeeping.
// Forward lane view (32x32 C/D map): S^T = K Q^T, a lane owns one query (lane & 31) and 16 keys
// of each 32-key subtile; its 32 probabilities of a 64-key tile, packed to e4m3 in place, are the
// B operand of O^T = V^T P^T.  Dropout reads the bf16 kernels' MQ bit plane (attention.hip): the
// u64 word of (query, 64-key tile) holds key k at bit ((k>>2)&3)*16 + (k>>4)*4 + (k&3), which for
// this lane view is a compile-time position + 16 (lane >> 5).
// The row sums use the unrounded fp32 P, so the log-sum-exp matches an fp32 softmax of x~.
#include "common.h"

#define A8_MAX 448.0f
// quantisation pass in its row form for H = 12 (attn_quant_fp8_rows_kernel): measured level at
// B32/N1024 (0.058 ms) and slower at B56/N1088 (0.176 vs 0.158 ms), profiles/r04/ab_blas_noslp_quantrows.txt
#ifndef UVA_A8_QUANT_ROWS
#define UVA_A8_QUANT_ROWS 0
#endif

typedef __attribute__((ext_vector_type(8))) int i32x8;  // 32 e4m3 values: one lane's 32x32x64 operand

// D = A B + C over K = 64 with e8m0 block scales sa / sb (2^(s - 127)) on A / B: lane l supplies
// row (A) or column (B) l & 31, k block l >> 5, and its scale covers exactly those 32 elements
__device__ __forceinline__ f32x16 mfma8s(const i32x8& a, const i32x8& b, const f32x16& c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// 4 floats -> 4 e4m3 bytes (round to nearest even, saturating)
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, p, true);
}

// position of key r (0..63) inside its permuted 64-key tile (inverse of 32h + 16s + i -> key)
__host__ __device__ constexpr int v8_pos(int r) {
  return 32 * ((r >> 2) & 1) + 16 * (r >> 5) + ((r & 3) + 4 * ((r & 31) >> 3));
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
    const int pos = v8_pos(row);
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

// smallest e with amax * 2^-e <= 448 (e = 0 for an all-zero tile)
__device__ __forceinline__ int a8_exponent(float amax) {
  int e = 0;
  if (amax > 0.f) {
    e = (int)ceilf(log2f(amax / A8_MAX));
    while (ldexpf(amax, -e) > A8_MAX) ++e;
    while (ldexpf(amax, -(e - 1)) <= A8_MAX) --e;
  }
  return e;
}

typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}

// Row form of the same pass for H heads known at compile time (mar_base: 12): one workgroup per
// (64-row tile, q|k|v, batch) walks all H heads of the tile.  The per-(tile, head) workgroups of
// attn_quant_fp8_kernel each move only 8 KiB behind one load round trip and a barrier; here every
// thread issues its 2H 16-B loads up front (8 lanes cover one 128-B head row, a wave-instruction 8
// rows), the H block maxima come out of one cross-wave exchange (|x| as bf16 bit patterns, two
// heads per dword, v_pk_max_u16), and the V^T transposes of all heads share one barrier.  Outputs
// are bit-identical to attn_quant_fp8_kernel.
template <int H>
__global__ __launch_bounds__(256) void attn_quant_fp8_rows_kernel(bf16* __restrict__ qkv, uint8_t* __restrict__ qk8,
                                                                  uint8_t* __restrict__ v8t, float* __restrict__ sc,
                                                                  int N) {
  static_assert(H % 2 == 0, "two heads per reduction word");
  __shared__ uint32_t red[4][H / 2];
  __shared__ __attribute__((aligned(16))) uint8_t tr[H][64 * 64];
  const int tile = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int r0 = w * 16 + (l >> 3), c = (l & 7) * 8;  // rows r0, r0 + 8; columns c .. c + 7 of every head
  const long long ld = 3LL * H * 64;
  bf16* base = qkv + ((long long)b * N + tile * 64 + r0) * ld + (long long)t * H * 64 + c;
  uint4 x[H][2];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int k = 0; k < 2; ++k) x[h][k] = *(const uint4*)(base + k * 8 * ld + h * 64);
  uint32_t m2[H / 2];
#pragma unroll
  for (int i = 0; i < H / 2; ++i) {
    uint32_t a = 0, bb = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      a = pk_max_u16(a, pk_max_u16(x[2 * i][k].x & 0x7FFF7FFFu, x[2 * i][k].y & 0x7FFF7FFFu));
      a = pk_max_u16(a, pk_max_u16(x[2 * i][k].z & 0x7FFF7FFFu, x[2 * i][k].w & 0x7FFF7FFFu));
      bb = pk_max_u16(bb, pk_max_u16(x[2 * i + 1][k].x & 0x7FFF7FFFu, x[2 * i + 1][k].y & 0x7FFF7FFFu));
      bb = pk_max_u16(bb, pk_max_u16(x[2 * i + 1][k].z & 0x7FFF7FFFu, x[2 * i + 1][k].w & 0x7FFF7FFFu));
    }
    a = max(a & 0xFFFFu, a >> 16);
    bb = max(bb & 0xFFFFu, bb >> 16);
    uint32_t v = a | (bb << 16);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = pk_max_u16(v, (uint32_t)__shfl_xor((int)v, o, 64));
    m2[i] = v;
  }
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < H / 2; ++i) red[w][i] = m2[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < H / 2; ++i) m2[i] = pk_max_u16(pk_max_u16(red[0][i], red[1][i]), pk_max_u16(red[2][i], red[3][i]));
  const long long q0 = (long long)b * N + tile * 64 + r0;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const uint32_t bits = (h & 1) ? (m2[h >> 1] >> 16) : (m2[h >> 1] & 0xFFFFu);
    const int e = a8_exponent(__uint_as_float(bits << 16));
    const float inv = ldexpf(1.f, -e), s = ldexpf(1.f, e);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bf16x8 xv = __builtin_bit_cast(bf16x8, x[h][k]);
      const int w0 = pack4_fp8((float)xv[0] * inv, (float)xv[1] * inv, (float)xv[2] * inv, (float)xv[3] * inv);
      const int w1 = pack4_fp8((float)xv[4] * inv, (float)xv[5] * inv, (float)xv[6] * inv, (float)xv[7] * inv);
      bf16x8 yv;
      yv[0] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w0, 0) * s);
      yv[1] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w0, 1) * s);
      yv[2] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w0, 2) * s);
      yv[3] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w0, 3) * s);
      yv[4] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w1, 0) * s);
      yv[5] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w1, 1) * s);
      yv[6] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w1, 2) * s);
      yv[7] = (bf16)(__builtin_amdgcn_cvt_f32_fp8(w1, 3) * s);
      *(bf16x8*)(base + k * 8 * ld + h * 64) = yv;
      if (t < 2) {
        *(int2*)(qk8 + ((q0 + 8 * k) * 2 + t) * (H * 64) + h * 64 + c) = (int2){w0, w1};
      } else {
        const int pos = v8_pos(r0 + 8 * k);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          tr[h][(c + j) * 64 + pos] = (uint8_t)((unsigned)w0 >> (8 * j));
          tr[h][(c + 4 + j) * 64 + pos] = (uint8_t)((unsigned)w1 >> (8 * j));
        }
      }
    }
    if (tid == h) sc[((long long)(b * 3 + t) * H + h) * (N / 64) + tile] = s;
  }
  if (t == 2) {  // workgroup-uniform
    __syncthreads();
    const int d = tid >> 2, c16 = (tid & 3) * 16;
#pragma unroll
    for (int h = 0; h < H; ++h)
      *(int4*)(v8t + (((long long)b * H + h) * 64 + d) * N + tile * 64 + c16) = *(const int4*)(&tr[h][d * 64 + c16]);
  }
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

// 32-byte operand of row r, byte columns [32 h, +32) of a 64-byte-row image (chunks 2h, 2h + 1)
__device__ __forceinline__ i32x8 a8_frag32(const uint8_t* img, int r, int h) {
  const int f = a8_swz<64>(r);
  const int4 lo = *(const int4*)(img + r * 64 + (((2 * h) ^ f) << 4));
  const int4 hi = *(const int4*)(img + r * 64 + (((2 * h + 1) ^ f) << 4));
  return (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}

__device__ __forceinline__ int e8m0_of(float pow2) { return 127 + (int)__builtin_amdgcn_frexp_expf(pow2) - 1; }

// =====================================================================================
// forward: 4 waves x 32 queries per workgroup, 64-key tiles (one 32x32x64 MFMA per 32x32 score
// tile, one per 32 d x 32 queries of P.V)
// =====================================================================================
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_fp8_kernel(const uint8_t* __restrict__ qk8,
                                                           const uint8_t* __restrict__ v8t,
                                                           const float* __restrict__ sc, bf16* __restrict__ out,
                                                           float* __restrict__ lse2, const uint64_t* __restrict__ MQ,
                                                           int N, int H, float c, float dsc) {
  constexpr int KT = 64;
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
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, lq = l & 31, hh = l >> 5;
  const int q0 = bx * 128 + w * 32;
  const int qrow = q0 + lq;
  const uint64_t* mq = DROP ? MQ + (long long)bh * nt64 * N : nullptr;  // [kv][q] words

  // Q^T fragment (B operand of S^T = K Q^T): query qrow, d bytes [32 hh, +32)
  i32x8 qf = {};
  if (qrow < N) {
    const int4 lo = *(const int4*)(Qg + (long long)qrow * ldq + 32 * hh);
    const int4 hi = *(const int4*)(Qg + (long long)qrow * ldq + 32 * hh + 16);
    qf = (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  }
  const int sq = e8m0_of(q0 < N ? sq_[q0 >> 6] : 1.f);  // the wave's 32 queries share one 64-row tile
  float m = -INFINITY, rs = 0.f;
  f32x16 o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;

  uint64_t mw = (DROP && qrow < N) ? mq[qrow] : 0ull;
  a8_dma<KT>(Kg, Vg, ldq, N, 0, sK(0), sV(0));
  __syncthreads();
  int cur = 0;
  for (int kv = 0; kv < nt64; ++kv) {
    const bool more = kv + 1 < nt64;
    uint64_t mwn = 0ull;
    if (more) {
      a8_dma<KT>(Kg, Vg, ldq, N, kv + 1, sK(cur ^ 1), sV(cur ^ 1));
      if (DROP && qrow < N) mwn = mq[(long long)(kv + 1) * N + qrow];
    }
    const uint8_t* cK = sK(cur);
    const uint8_t* cV = sV(cur);
    const int sk = e8m0_of(sk_[kv]), sv = e8m0_of(sv_[kv]);
    // S^T (32 keys x 32 queries) of the tile's two subtiles, already scaled by 2^(eq + ek)
    f32x16 s[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const f32x16 z = {};
      s[st] = mfma8s(a8_frag32(cK, st * 32 + lq, hh), qf, z, sk, sq);
    }
    float mx = __builtin_amdgcn_fmed3f(s[0][0], s[0][1], INFINITY);
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = (st == 0 ? 2 : 0); i < 16; ++i) mx = __builtin_amdgcn_fmed3f(mx, s[st][i], INFINITY);
    {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])) * c;
    }
    const bool need = mx > m + 8.0f;  // lazy rescale (m = -inf at first)
    if (__builtin_amdgcn_ballot_w64(need)) {
      const float mn = need ? mx : m;
      const float a = __builtin_amdgcn_exp2f(m - mn);
      rs *= a;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) o[dt] *= a;
      m = mn;
    }
    // this lane's keep bits: the MQ word of its query, shifted by 16 for the upper half of lanes
    const uint32_t wlo = hh ? __builtin_amdgcn_alignbit((uint32_t)(mw >> 32), (uint32_t)mw, 16) : (uint32_t)mw;
    const uint32_t whi = hh ? (uint32_t)(mw >> 48) : (uint32_t)(mw >> 32);
    const float nm = -m;
    float ps[4] = {0.f, 0.f, 0.f, 0.f};
    int pk[8];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        float p2[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int ii = i + u;
          const float p = __builtin_amdgcn_exp2f(fmaf(s[st][ii], c, nm));
          ps[ii & 3] += p;
          // key 32 st + (ii&3) + 8 (ii>>2) + 4 hh  ->  MQ bit 16 hh + BIT
          const int bit = 32 * ((ii >> 2) & 1) + 4 * (2 * st + (ii >> 3)) + (ii & 3);
          p2[u] = DROP ? __int_as_float(__float_as_int(p) &
                                        __builtin_amdgcn_sbfe(bit < 32 ? wlo : whi, bit & 31, 1))
                       : p;
        }
        // byte 16 st + i (, + 1) of the operand: two e4m3 in the half-word (i & 2) of dword (16 st + i) / 4
        const int word = (16 * st + i) >> 2;
        if ((i & 2) == 0) pk[word] = __builtin_amdgcn_cvt_pk_fp8_f32(p2[0], p2[1], 0, false);
        else pk[word] = __builtin_amdgcn_cvt_pk_fp8_f32(p2[0], p2[1], pk[word], true);
      }
    rs += (ps[0] + ps[1]) + (ps[2] + ps[3]);
    const i32x8 pf = {pk[0], pk[1], pk[2], pk[3], pk[4], pk[5], pk[6], pk[7]};
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) o[dt] = mfma8s(a8_frag32(cV, dt * 32 + lq, hh), pf, o[dt], sv, 127);
    mw = mwn;
    __syncthreads();
    cur ^= 1;
  }
  // lane: query qrow; o[dt][i] <-> d = 32 dt + (i&3) + 8(i>>2) + 4hh
  float lsum;
  {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(rs), __float_as_uint(rs), false, false);
    lsum = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if (qrow < N) {
    const float inv = dsc / lsum;
    bf16* orow = out + ((long long)b * N + qrow) * ((long long)H * 64) + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x4 v = {(bf16)(o[dt][4 * j] * inv), (bf16)(o[dt][4 * j + 1] * inv), (bf16)(o[dt][4 * j + 2] * inv),
                          (bf16)(o[dt][4 * j + 3] * inv)};
        *(bf16x4*)(orow + 32 * dt + 8 * j + 4 * hh) = v;
      }
    if (hh == 0) lse2[(long long)bh * N + qrow] = m + __log2f(lsum);
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
  if (H == 12 && UVA_A8_QUANT_ROWS)
    attn_quant_fp8_rows_kernel<12><<<dim3(N / 64, 3, B), 256, 0, s>>>((bf16*)qkv, qk8, v8t, sc, N);
  else
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
  if (drop)
    attn_fwd_fp8_kernel<true><<<grid, 256, 0, s>>>(qk8, v8t, sc, (bf16*)out, lse2, MQ, N, H, c, ds);
  else
    attn_fwd_fp8_kernel<false><<<grid, 256, 0, s>>>(qk8, v8t, sc, (bf16*)out, lse2, nullptr, N, H, c, 1.0f);
  UVA_LAUNCH_CHECK();
  return 0;
}
