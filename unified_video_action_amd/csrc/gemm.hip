// Dense contractions for the UVA training step: every nn.Linear forward/backward,
// the materialised attention products of the fp32 parity path and of the VAE
// mid-block attention, and im2col convolutions.
//
//   C[z][m][n] = epilogue( alpha * sum_k opA[z][m][k] * opB[z][n][k] )
//   ta = 0: A stored [M][K] (lda)       ta = 1: A stored [K][M]
//   tb = 0: B stored [N][K] (ldb)       tb = 1: B stored [K][N]
// so Linear fwd = (ta0,tb0), dX = (ta0,tb1), dW = (ta1,tb1).
//
// Two kernels:
//  * gemm_mfma_bf16  -- bf16 in, fp32 accumulate on v_mfma_f32_16x16x32_bf16;
//    128x128x64 block tile, 4 waves of 64x64, register-staged double-buffered LDS
//    (loads for tile k+1 issued before the MFMAs of tile k, written after), XOR
//    swizzled K-major images read with ds_read_b128 and M-major images read with
//    ds_read_b64_tr_b16 (hardware transpose) so no operand is ever transposed in HBM.
//  * gemm_generic    -- fp32 FMA on the VALU, any shape / dtype; the fp32 parity
//    path and the tiny-K/N projections (K = 2, 4, 10 ...).
#include "common.h"
#include <stdio.h>
#include <stdlib.h>

struct EpiParams {
  const float* bias;      // [N] fp32 or null
  const void* residual;   // same dtype/layout as C (ldr) or null
  void* aux;              // pre-activation copy (dtype of C, ldc) or null
  int act;
  float alpha, beta;
  uint32_t drop_thresh;   // 0 => no dropout
  float drop_scale;
  uint64_t drop_seed;
  long long ldr;
  long long sRo, sRi;     // residual batch strides
  const void* gate;       // adaLN gate (row-major, ld = ldg, dtype gate_dt) or null
  long long ldg;
  int gate_dt, res_dt;    // runtime dtypes of gate / residual (UVA_DT_*)
  int res_grad;           // ACT_* kind: "residual" is a pre-activation and the output is multiplied by
                          // act'(pre) instead of added (activation backward fused into the dX GEMM)
};

struct BatchStrides {
  long long sAo, sAi, sBo, sBi, sCo, sCi;
  int binner;
};

// implicit-GEMM convolution view of operand A (ta == 2): A[m][k] with
//   m = (n, oh, ow) over the NHWC output,  k = (kh, kw, ci)
//   A[m][k] = act(in[n][oh*stride+kh-pad_t][ow*stride+kw-pad_l][ci])   (0 outside the image)
// act = GroupNorm-apply + SiLU (per-(n, ci) scale/shift, fp32) when gn_scale != null.
// Replaces torch.nn.Conv2d of vae/vaekl.py:73-91,122-133,188,238,469 and the
// GroupNorm+swish that precedes them (vaekl.py:9-17,94-104,270-271).
struct ConvParams {
  int Hin, Win, Ci, Hout, Wout, ks, stride, pad_t, pad_l;
  const float* gn_scale;
  const float* gn_shift;
  int gn_silu;
  float* gn_part;     // if set: per-(row tile, group) (sum, sumsq) of the stored output, 32 groups
};

template <typename TC>
__device__ __forceinline__ float epi_store(TC* C, long long ldc, long long coff, const EpiParams& ep,
                                           long long roff, int row, int col, int N, long long didx, float acc) {
  float v = ep.alpha * acc;
  if (ep.bias) v += ep.bias[col];
  long long ci = coff + (long long)row * ldc + col;
  if (ep.aux) ((TC*)ep.aux)[ci] = from_f32<TC>(v);
  v = apply_act(ep.act, v);
  if (ep.drop_thresh) v = dropout_keep(ep.drop_seed, (uint64_t)didx, ep.drop_thresh) ? v * ep.drop_scale : 0.f;
  if (ep.gate) {
    long long gi = (long long)row * ep.ldg + col;
    v *= ep.gate_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.gate)[gi] : ((const float*)ep.gate)[gi];
  }
  if (ep.residual) {
    long long ri = roff + (long long)row * ep.ldr + col;
    const float r = ep.res_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.residual)[ri] : ((const float*)ep.residual)[ri];
    v = ep.res_grad ? v * act_grad(ep.res_grad, r) : v + r;
  }
  if (ep.beta != 0.f) v += ep.beta * to_f32(C[ci]);
  const TC o = from_f32<TC>(v);
  C[ci] = o;
  return to_f32(o);
}

// =====================================================================================
// generic VALU kernel: 64x64 tile, BK=16, 256 threads x (4x4) outputs
// =====================================================================================
template <typename TI>
__device__ __forceinline__ float conv_gather(const TI* __restrict__ in, const ConvParams& cp, int m, int k) {
  const int hw = cp.Hout * cp.Wout;
  const int n = m / hw, r = m % hw, oh = r / cp.Wout, ow = r % cp.Wout;
  const int tap = k / cp.Ci, ci = k % cp.Ci;
  const int ih = oh * cp.stride + tap / cp.ks - cp.pad_t, iw = ow * cp.stride + tap % cp.ks - cp.pad_l;
  if (ih < 0 || ih >= cp.Hin || iw < 0 || iw >= cp.Win) return 0.f;
  float v = to_f32(in[(((long long)n * cp.Hin + ih) * cp.Win + iw) * cp.Ci + ci]);
  if (cp.gn_scale) {
    v = v * cp.gn_scale[(long long)n * cp.Ci + ci] + cp.gn_shift[(long long)n * cp.Ci + ci];
    if (cp.gn_silu) v = silu(v);
  }
  return v;
}

// SPLIT: blockIdx.z is a K-slice of k_per_split (batch 1); raw fp32 partial sums go to part[z][M][N]
// and splitk_reduce applies the epilogue in slice order (deterministic).  For the tiny-output,
// long-K products (the action head's Linear(4 -> 16) frame-interpolation dW, 16 x 4 over K = B x 768
// tokens; the diffusion heads' input_proj dW over K = rows) one 64x64 block would otherwise walk K alone.
template <typename TI, typename TC, int TA, int TB, bool SPLIT = false>
__global__ __launch_bounds__(256) void gemm_generic(const TI* __restrict__ A, const TI* __restrict__ B,
                                                    TC* __restrict__ C, int M, int N, int K, long long lda,
                                                    long long ldb, long long ldc, BatchStrides bs, EpiParams ep,
                                                    ConvParams cp, float* __restrict__ part = nullptr,
                                                    int k_per_split = 0) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int z = SPLIT ? 0 : blockIdx.z, zo = z / bs.binner, zi = z % bs.binner;
  A += zo * bs.sAo + zi * bs.sAi;
  B += zo * bs.sBo + zi * bs.sBi;
  const long long coff = zo * bs.sCo + zi * bs.sCi;
  const long long roff = zo * ep.sRo + zi * ep.sRi;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const int kb = SPLIT ? blockIdx.z * k_per_split : 0;
  const int ke = SPLIT ? min(K, kb + k_per_split) : K;
  float acc[4][4] = {};
  for (int k0 = kb; k0 < ke; k0 += 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int e = t + i * 256;  // 0..1023 over a 64x16 tile
      int mm, kk;
      if (TA != 1) { mm = e >> 4; kk = e & 15; } else { kk = e >> 6; mm = e & 63; }
      int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < M && gk < ke) {
        if (TA == 2) v = conv_gather(A, cp, gm, gk);
        else v = to_f32(TA == 0 ? A[(long long)gm * lda + gk] : A[(long long)gk * lda + gm]);
      }
      As[kk][mm] = v;
      int nn;
      if (TB == 0) { nn = e >> 4; kk = e & 15; } else { kk = e >> 6; nn = e & 63; }
      int gn = n0 + nn;
      gk = k0 + kk;
      v = 0.f;
      if (gn < N && gk < ke) v = to_f32(TB == 0 ? B[(long long)gn * ldb + gk] : B[(long long)gk * ldb + gn]);
      Bs[kk][nn] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[kk][ty * 4 + i]; b[i] = Bs[kk][tx * 4 + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int r = m0 + ty * 4 + i, c = n0 + tx * 4 + j;
      if (r < M && c < N) {
        if (SPLIT) part[((long long)blockIdx.z * M + r) * N + c] = acc[i][j];
        else epi_store<TC>(C, ldc, coff, ep, roff, r, c, N, (long long)z * M * N + (long long)r * N + c, acc[i][j]);
      }
    }
}

// =====================================================================================
// MFMA bf16 kernel
// =====================================================================================
#define MB_M 128
#define MB_N 128
#define MB_K 64
#define LDK_ROW 64    // K-major image: [rows][64] bf16, 16-B chunks XOR-swizzled by row
#define LDM_ROW 144   // M-major image: [64 k][128 rows + 16 pad] bf16, column XOR 64 by k bit 3
#define STAGE_K_ELEMS (MB_M * LDK_ROW)
#define STAGE_M_ELEMS (MB_K * LDM_ROW)

template <int T>
struct OperandImage {
  static constexpr int elems = (T == 1) ? STAGE_M_ELEMS : STAGE_K_ELEMS;
};

// per-thread decode of the 4 output rows a conv A-tile chunk belongs to (fixed over k)
struct ConvRows {
  int n[4], ih0[4], iw0[4];
  bool ok[4];
};

__device__ __forceinline__ void conv_rows_init(const ConvParams& cp, int row0, int M, ConvRows& cr) {
  const int t = threadIdx.x, hw = cp.Hout * cp.Wout;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = row0 + ((t + i * 256) >> 3);
    cr.ok[i] = m < M;
    int mm = cr.ok[i] ? m : 0;
    int n = mm / hw, r = mm % hw;
    cr.n[i] = n;
    cr.ih0[i] = (r / cp.Wout) * cp.stride - cp.pad_t;
    cr.iw0[i] = (r % cp.Wout) * cp.stride - cp.pad_l;
  }
}

// global -> registers for one 128x64 operand tile (4 chunks of 8 bf16 per thread)
template <int T>
__device__ __forceinline__ void tile_load(const bf16* __restrict__ P, long long ld, int row0, int nrows, int k0, int K,
                                          bf16x8 (&r)[4], const ConvParams& cp, const ConvRows& cr) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int id = t + i * 256;
    if (T == 2) {
      const int k = k0 + (id & 7) * 8;
      bf16x8 v = (bf16x8){};
      if (cr.ok[i] && k < K) {
        int tap, ci;
        if ((cp.Ci & 63) == 0) {  // a 64-deep k tile never straddles two taps: wave-uniform tap
          tap = __builtin_amdgcn_readfirstlane(k0 / cp.Ci);
          ci = k - tap * cp.Ci;
        } else {
          tap = k / cp.Ci;
          ci = k - tap * cp.Ci;
        }
        const int kh = cp.ks == 3 ? (tap >= 6 ? 2 : (tap >= 3 ? 1 : 0)) : 0;
        const int ih = cr.ih0[i] + kh, iw = cr.iw0[i] + (tap - kh * cp.ks);
        if (ih >= 0 && ih < cp.Hin && iw >= 0 && iw < cp.Win) {
          v = *(const bf16x8*)(P + (((long long)cr.n[i] * cp.Hin + ih) * cp.Win + iw) * cp.Ci + ci);
          if (cp.gn_scale) {
            const float* sc = cp.gn_scale + (long long)cr.n[i] * cp.Ci + ci;
            const float* sh = cp.gn_shift + (long long)cr.n[i] * cp.Ci + ci;
            float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
            float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
            float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            float hh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float u = (float)v[j] * ss[j] + hh[j];
              v[j] = (bf16)(cp.gn_silu ? silu(u) : u);
            }
          }
        }
      }
      r[i] = v;
      continue;
    }
    int row, k;
    if (T == 0) { row = id >> 3; k = (id & 7) * 8; } else { k = id >> 4; row = (id & 15) * 8; }
    int gr = row0 + row, gk = k0 + k;
    if (gr < nrows && gk < K) {
      const bf16* src = (T == 0) ? P + (long long)gr * ld + gk : P + (long long)gk * ld + gr;
      r[i] = *(const bf16x8*)src;
    } else {
      r[i] = (bf16x8){};
    }
  }
}

template <int T>
__device__ __forceinline__ void tile_store(bf16* lds, const bf16x8 (&r)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int id = t + i * 256;
    if (T != 1) {
      int row = id >> 3, c = id & 7;
      *(bf16x8*)(lds + row * LDK_ROW + ((c ^ (row & 7)) * 8)) = r[i];
    } else {
      int k = id >> 4, col = (id & 15) * 8;
      *(bf16x8*)(lds + k * LDM_ROW + (col ^ ((k & 8) << 3))) = r[i];
    }
  }
}

// MFMA 16x16x32 operand fragment: rows row0..row0+15 (lane&15), k = ks*32 + 8*(lane>>4) + j
template <int T>
__device__ __forceinline__ bf16x8 frag_load(const bf16* lds, int row0, int ks) {
  const int l = threadIdx.x & 63;
  if (T != 1) {
    int row = row0 + (l & 15);
    int c = ks * 4 + (l >> 4);
    return *(const bf16x8*)(lds + row * LDK_ROW + ((c ^ (row & 7)) * 8));
  } else {
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    int k = ks * 32 + g * 8 + q;
    int col = row0 + 4 * p;
    const bf16* a0 = lds + k * LDM_ROW + (col ^ ((k & 8) << 3));
    const bf16* a1 = lds + (k + 4) * LDM_ROW + (col ^ (((k + 4) & 8) << 3));
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  // bijective: blocks that share an XCD (bid % 8) get a contiguous range of logical ids
  int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// one row segment of 8 consecutive columns (16-B aligned in C): the row-wise epilogue inputs (C for
// beta, residual, gate) are loaded by epi_load_row8 and consumed by epi_apply_row8, so a caller can
// issue the next row's loads before this row's store -- a load issued after a store waits for that
// store on the in-order vector-memory counter, which serialised the epilogue on the store latency
struct EpiRow {
  float prev[8], res[8], gate[8];
};

__device__ __forceinline__ void epi_load_bias8(const EpiParams& ep, int col0, float (&bv)[8]) {
  if (ep.bias) {
    const float4 b0 = *(const float4*)(ep.bias + col0), b1 = *(const float4*)(ep.bias + col0 + 4);
    bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  }
}

template <typename TC>
__device__ __forceinline__ void epi_load_row8(const TC* __restrict__ C, long long cbase, const EpiParams& ep,
                                              long long roff, int row, int col0, EpiRow& in) {
  if (ep.beta != 0.f) {
    if constexpr (sizeof(TC) == 2) {
      bf16x8 pv = *(const bf16x8*)(C + cbase);
#pragma unroll
      for (int e = 0; e < 8; ++e) in.prev[e] = (float)pv[e];
    } else {
      float4 p0 = *(const float4*)(C + cbase), p1 = *(const float4*)(C + cbase + 4);
      in.prev[0] = p0.x; in.prev[1] = p0.y; in.prev[2] = p0.z; in.prev[3] = p0.w;
      in.prev[4] = p1.x; in.prev[5] = p1.y; in.prev[6] = p1.z; in.prev[7] = p1.w;
    }
  }
  if (ep.residual) {
    const long long ri = roff + (long long)row * ep.ldr + col0;
    if (ep.res_dt == UVA_DT_BF16 && (ri % 8 == 0)) {
      bf16x8 rv = *(const bf16x8*)((const bf16*)ep.residual + ri);
#pragma unroll
      for (int e = 0; e < 8; ++e) in.res[e] = (float)rv[e];
    } else if (ep.res_dt != UVA_DT_BF16 && (ri % 4 == 0)) {
      float4 r0 = *(const float4*)((const float*)ep.residual + ri);
      float4 r1 = *(const float4*)((const float*)ep.residual + ri + 4);
      in.res[0] = r0.x; in.res[1] = r0.y; in.res[2] = r0.z; in.res[3] = r0.w;
      in.res[4] = r1.x; in.res[5] = r1.y; in.res[6] = r1.z; in.res[7] = r1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        in.res[e] = ep.res_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.residual)[ri + e]
                                             : ((const float*)ep.residual)[ri + e];
    }
  }
  if (ep.gate) {
    const long long gi = (long long)row * ep.ldg + col0;
    if (ep.gate_dt == UVA_DT_BF16 && gi % 8 == 0) {
      const bf16x8 g8 = *(const bf16x8*)((const bf16*)ep.gate + gi);
#pragma unroll
      for (int e = 0; e < 8; ++e) in.gate[e] = (float)g8[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        in.gate[e] = ep.gate_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.gate)[gi + e] : ((const float*)ep.gate)[gi + e];
    }
  }
}

// o = the values as stored (for fused statistics)
template <typename TC, bool NT = false>
__device__ __forceinline__ void epi_apply_row8(TC* __restrict__ C, long long cbase, const EpiParams& ep,
                                               const float (&bv)[8], const EpiRow& in, int row, int col0, int z,
                                               int M, int N, const float (&v)[8], float (&o)[8]) {
  bool keep[8] = {true, true, true, true, true, true, true, true};
  if (ep.drop_thresh) {
    const uint64_t d0 = (uint64_t)((long long)z * M * N + (long long)row * N + col0);
    if ((d0 & 1) == 0) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) dropout_keep2(ep.drop_seed, d0 + e, ep.drop_thresh, keep[e], keep[e + 1]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) keep[e] = dropout_keep(ep.drop_seed, d0 + e, ep.drop_thresh);
    }
  }
  float x[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = ep.alpha * v[e] + bv[e];
  if (ep.aux) {  // pre-activation copy, one 16-B (bf16) / 2 x 16-B (fp32) store
    if constexpr (sizeof(TC) == 2) {
      bf16x8 av;
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = (bf16)x[e];
      *(bf16x8*)((TC*)ep.aux + cbase) = av;
    } else {
      *(float4*)((TC*)ep.aux + cbase) = make_float4(x[0], x[1], x[2], x[3]);
      *(float4*)((TC*)ep.aux + cbase + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
  }
  // activation: one uniform branch per row segment, not per element
  switch (ep.act) {
    case ACT_GELU:
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = gelu_erf(x[e]);
      break;
    case ACT_SILU:
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = silu(x[e]);
      break;
    case ACT_RELU:
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = x[e] > 0.f ? x[e] : 0.f;
      break;
    default:
      break;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float t = x[e];
    if (ep.drop_thresh) t = keep[e] ? t * ep.drop_scale : 0.f;
    if (ep.gate) t *= in.gate[e];
    if (ep.residual) t = ep.res_grad ? t * act_grad(ep.res_grad, in.res[e]) : t + in.res[e];
    if (ep.beta != 0.f) t += ep.beta * in.prev[e];
    o[e] = t;
  }
  if constexpr (sizeof(TC) == 2) {
    bf16x8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov[e] = (bf16)o[e];
    if constexpr (NT) {
      typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(__builtin_bit_cast(u32x4_nt, ov), (u32x4_nt*)(C + cbase));
    } else {
      *(bf16x8*)(C + cbase) = ov;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (float)ov[e];
  } else {
    *(float4*)(C + cbase) = make_float4(o[0], o[1], o[2], o[3]);
    *(float4*)(C + cbase + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
}

template <typename TC, bool NT = false>
__device__ __forceinline__ void epi_row8(TC* __restrict__ C, long long cbase, const EpiParams& ep, long long roff,
                                         int row, int col0, int z, int M, int N, const float (&v)[8], float (&o)[8]) {
  float bv[8];
  EpiRow in;
  epi_load_bias8(ep, col0, bv);
  epi_load_row8<TC>(C, cbase, ep, roff, row, col0, in);
  epi_apply_row8<TC, NT>(C, cbase, ep, bv, in, row, col0, z, M, N, v, o);
}

// Epilogue staged through LDS: the 128x128 fp32 accumulator tile is written to LDS with
// compile-time indices (no register-array indexing -> no scratch), then every thread finishes
// 8 consecutive columns x 8 rows with 16-B vector loads/stores (coalesced, issue-light).
#define EPI_TP 132  // fp32 row pitch of the staged tile (+4 floats: conflict-free column writes)
#define EPI_LDS_BYTES (128 * EPI_TP * 4 + 4 * 16 * 8 * 2 * 4)

// epilogue barrier that orders LDS only: the chunk's global stores stay in flight across it
__device__ __forceinline__ void epi_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename TC>
__device__ __forceinline__ void epilogue_tile(const f32x4 (&acc)[4][4], char* smem, TC* __restrict__ C, int M, int N,
                                              long long ldc, long long coff, const EpiParams& ep, long long roff,
                                              int m0, int n0, int z, float* __restrict__ pslab,
                                              float* __restrict__ gn_part, int bm) {
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, wm = wid >> 1, wn = wid & 1;
  float* T = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        T[(wm * 64 + i * 16 + (lane >> 4) * 4 + r) * EPI_TP + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  const int c8 = tid & 15, rsub = tid >> 4;
  const int col0 = n0 + c8 * 8;
  const bool full = (col0 + 8 <= N) && (ldc % 8 == 0) && ((coff + col0) % 8 == 0);
  float gs_s[8], gs_q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) gs_s[e] = gs_q[e] = 0.f;
  const bool plain = !ep.residual && !ep.gate && !ep.aux && ep.act == 0 && ep.drop_thresh == 0 && ep.beta == 0.f;
  if (!pslab && full && !gn_part) {
    float bv[8];
    epi_load_bias8(ep, col0, bv);
    if (plain) {  // no loads inside the loop: no store waits for an earlier one (see EpiRow)
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int rl = it * 16 + rsub, row = m0 + rl;
        if (row < M) {
          const float4 a = *(const float4*)(T + rl * EPI_TP + c8 * 8);
          const float4 b = *(const float4*)(T + rl * EPI_TP + c8 * 8 + 4);
          const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          TC* dst = C + coff + (long long)row * ldc + col0;
          if constexpr (sizeof(TC) == 2) {
            bf16x8 ov;
#pragma unroll
            for (int e = 0; e < 8; ++e) ov[e] = (bf16)(ep.alpha * v[e] + bv[e]);
            *(bf16x8*)dst = ov;
          } else {
            *(float4*)dst = make_float4(ep.alpha * v[0] + bv[0], ep.alpha * v[1] + bv[1], ep.alpha * v[2] + bv[2],
                                        ep.alpha * v[3] + bv[3]);
            *(float4*)(dst + 4) = make_float4(ep.alpha * v[4] + bv[4], ep.alpha * v[5] + bv[5],
                                              ep.alpha * v[6] + bv[6], ep.alpha * v[7] + bv[7]);
          }
        }
      }
    } else {  // the next row's inputs are loaded before this row's store
      EpiRow cur, nxt;
      if (m0 + rsub < M) epi_load_row8<TC>(C, coff + (long long)(m0 + rsub) * ldc + col0, ep, roff, m0 + rsub, col0, cur);
#pragma unroll 1
      for (int it = 0; it < 8; ++it) {
        const int rl = it * 16 + rsub, row = m0 + rl;
        if (it + 1 < 8 && row + 16 < M)
          epi_load_row8<TC>(C, coff + (long long)(row + 16) * ldc + col0, ep, roff, row + 16, col0, nxt);
        if (row < M) {
          const float4 a = *(const float4*)(T + rl * EPI_TP + c8 * 8);
          const float4 b = *(const float4*)(T + rl * EPI_TP + c8 * 8 + 4);
          const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          float o[8];
          epi_apply_row8<TC>(C, coff + (long long)row * ldc + col0, ep, bv, cur, row, col0, z, M, N, v, o);
        }
        cur = nxt;
      }
    }
  } else
  for (int it = 0; it < 8; ++it) {
    const int rl = it * 16 + rsub;
    const int row = m0 + rl;
    if (row >= M || col0 >= N) break;
    float v[8];
    const float4 a = *(const float4*)(T + rl * EPI_TP + c8 * 8);
    const float4 b = *(const float4*)(T + rl * EPI_TP + c8 * 8 + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    if (pslab) {
      float* dst = pslab + (long long)row * N + col0;
      if (col0 + 8 <= N && N % 4 == 0) {
        *(float4*)dst = a;
        *(float4*)(dst + 4) = b;
      } else {
        for (int e = 0; e < 8 && col0 + e < N; ++e) dst[e] = v[e];
      }
      continue;
    }
    const long long cbase = coff + (long long)row * ldc + col0;
    if (full) {
      float o[8];
      epi_row8<TC>(C, cbase, ep, roff, row, col0, z, M, N, v, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        gs_s[e] += o[e];
        gs_q[e] += o[e] * o[e];
      }
    } else {
      for (int e = 0; e < 8 && col0 + e < N; ++e) {
        const int col = col0 + e;
        float o = epi_store<TC>(C, ldc, coff, ep, roff, row, col, N,
                                (long long)z * M * N + (long long)row * N + col, v[e]);
        gs_s[e] += o;
        gs_q[e] += o * o;
      }
    }
  }
  if (gn_part) {
    // per-column sums over the tile's 128 rows in a fixed order (deterministic), then 32 groups
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gs_s[e] += __shfl_xor(gs_s[e], 16, 64);
      gs_s[e] += __shfl_xor(gs_s[e], 32, 64);
      gs_q[e] += __shfl_xor(gs_q[e], 16, 64);
      gs_q[e] += __shfl_xor(gs_q[e], 32, 64);
    }
    float* red = T + 128 * EPI_TP;  // [4 waves][16 c8][8][2]
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[((wid * 16 + lane) * 8 + e) * 2 + 0] = gs_s[e];
        red[((wid * 16 + lane) * 8 + e) * 2 + 1] = gs_q[e];
      }
    }
    __syncthreads();
    const int gsz = N / 32;
    const int ngroups = min(MB_N, N - n0) / gsz;
    if (tid < ngroups) {
      float s = 0.f, q = 0.f;
      for (int c = tid * gsz; c < (tid + 1) * gsz; ++c)
        for (int w = 0; w < 4; ++w) {
          s += red[((w * 16 + (c >> 3)) * 8 + (c & 7)) * 2 + 0];
          q += red[((w * 16 + (c >> 3)) * 8 + (c & 7)) * 2 + 1];
        }
      const int g = n0 / gsz + tid;
      gn_part[((long long)bm * 32 + g) * 2 + 0] = s;
      gn_part[((long long)bm * 32 + g) * 2 + 1] = q;
    }
  }
}

// splits > 1: blockIdx.y = K-slice; raw fp32 partials go to `part` (+ slice * M * N),
// the epilogue runs in splitk_reduce.
template <int TA, int TB, typename TC>
__global__ __launch_bounds__(256, 2) void gemm_mfma_bf16(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         TC* __restrict__ C, int M, int N, int K, long long lda,
                                                         long long ldb, long long ldc, BatchStrides bs,
                                                         EpiParams ep, ConvParams cp, float* __restrict__ part,
                                                         int k_per_split) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sA = (bf16*)smem;
  bf16* sB = sA + 2 * OperandImage<TA>::elems;
  const int z = blockIdx.z, zo = z / bs.binner, zi = z % bs.binner;
  A += zo * bs.sAo + zi * bs.sAi;
  B += zo * bs.sBo + zi * bs.sBi;
  const long long coff = zo * bs.sCo + zi * bs.sCi;
  const long long roff = zo * ep.sRo + zi * ep.sRi;

  // tile order: XCD-contiguous logical ids, then groups of 8 row-tiles share B panels
  const int tm = (M + MB_M - 1) / MB_M, tn = (N + MB_N - 1) / MB_N;
  const int nblk = tm * tn;
  int pid = xcd_remap(blockIdx.x, nblk);
  const int GROUP = 8;
  int group = pid / (GROUP * tn), first_m = group * GROUP;
  int gsz = min(tm - first_m, GROUP);
  int bm = first_m + (pid % (GROUP * tn)) % gsz;
  int bn = (pid % (GROUP * tn)) / gsz;
  const int m0 = bm * MB_M, n0 = bn * MB_N;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);

  ConvRows cr;
  if (TA == 2) conv_rows_init(cp, m0, M, cr);

  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[4], rb[4];
  const int nk = (kend - kbeg + MB_K - 1) / MB_K;
  tile_load<TA>(A, lda, m0, M, kbeg, kend, ra, cp, cr);
  tile_load<TB>(B, ldb, n0, N, kbeg, kend, rb, cp, cr);
  tile_store<TA>(sA, ra);
  tile_store<TB>(sB, rb);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {
      tile_load<TA>(A, lda, m0, M, kbeg + (kt + 1) * MB_K, kend, ra, cp, cr);
      tile_load<TB>(B, ldb, n0, N, kbeg + (kt + 1) * MB_K, kend, rb, cp, cr);
    }
    const bf16* cA = sA + cur * OperandImage<TA>::elems;
    const bf16* cB = sB + cur * OperandImage<TB>::elems;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_load<TA>(cA, wm * 64 + i * 16, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_load<TB>(cB, wn * 64 + j * 16, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      tile_store<TA>(sA + (cur ^ 1) * OperandImage<TA>::elems, ra);
      tile_store<TB>(sB + (cur ^ 1) * OperandImage<TB>::elems, rb);
    }
    __syncthreads();
    cur ^= 1;
  }
  epilogue_tile<TC>(acc, smem, C, M, N, ldc, coff, ep, roff, m0, n0, z,
                    part ? part + (long long)blockIdx.y * M * N : nullptr, (TA == 2) ? cp.gn_part : nullptr, bm);
}

// =====================================================================================
// MFMA bf16 kernel v2: LDS-DMA staging (global_load_lds, 16 B/lane, no register pass)
//   K-major image [128 rows][64 k]  (128-B rows), 16-B chunk c of row r stored at c ^ (r & 7)
//   M-major image [64 k][128 rows]  (256-B rows), 16-B chunk c of row k stored at c ^ s(k),
//       s(k) = ((k & 3) << 1) | (((k >> 3) & 1) << 3)  -> the ds_read_b64_tr_b16 fragment
//       reads of one 32-lane half hit 16 distinct chunks (conflict-free), no padding.
// Both images are lane-linear per 1-KiB wave instruction, so the swizzle moves to the
// per-lane SOURCE address (cdna_hip_programming.md rule 21).  OOB lanes read a zero page.
// =====================================================================================
__device__ __attribute__((aligned(16))) bf16 g_uva_zero_page[64];

__device__ __forceinline__ int mswz(int k) { return ((k & 3) << 1) | (((k >> 3) & 1) << 3); }

template <int T>
__device__ __forceinline__ bf16x8 frag_load_v2(const bf16* lds, int row0, int ks) {
  const int l = threadIdx.x & 63;
  if (T != 1) {
    int row = row0 + (l & 15);
    int c = ks * 4 + (l >> 4);
    return *(const bf16x8*)(lds + row * 64 + ((c ^ (row & 7)) * 8));
  } else {
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int k = ks * 32 + g * 8 + q;
    const int col = row0 + 4 * p;  // element column, 4 elements (8 B) inside one 16-B chunk
    const int c = col >> 3, w = col & 7;
    const bf16* a0 = lds + k * 128 + ((c ^ mswz(k)) << 3) + w;
    const bf16* a1 = lds + (k + 4) * 128 + ((c ^ mswz(k + 4)) << 3) + w;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// per-lane source pointers of the 4 wave-instructions (1 KiB each) this wave issues per tile
template <int T>
struct DmaSrc {
  const bf16* p[4];
};

// element position of wave-instruction i, lane l inside the 16-KiB image: e = (w*4+i)*512 + l*8
template <int T>
__device__ __forceinline__ const bf16* dma_addr(const bf16* __restrict__ P, long long ld, int row0, int nrows, int k0,
                                                int K, int i, const ConvParams& cp, const ConvRows& cr) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int e = (w * 4 + i) * 512 + l * 8;
  if (T == 0) {
    const int row = e >> 6, cl = (e & 63) >> 3;
    const int k = k0 + ((cl ^ (row & 7)) << 3);
    const int gr = row0 + row;
    return (gr < nrows && k < K) ? P + (long long)gr * ld + k : g_uva_zero_page;
  } else if (T == 1) {
    const int kr = e >> 7, cl = (e & 127) >> 3;
    const int m = (cl ^ mswz(kr)) << 3;
    const int gk = k0 + kr, gr = row0 + m;
    return (gr < nrows && gk < K) ? P + (long long)gk * ld + gr : g_uva_zero_page;
  } else {
    // implicit-GEMM conv gather; row decode cached in cr (row = (w*4+i)*8 + l/8)
    const int cl = (e & 63) >> 3;
    const int row = e >> 6;
    const int k = k0 + ((cl ^ (row & 7)) << 3);
    if (!cr.ok[i] || k >= K) return g_uva_zero_page;
    const int tap = ((cp.Ci & 63) == 0) ? __builtin_amdgcn_readfirstlane(k0 / cp.Ci) : k / cp.Ci;
    const int ci = k - tap * cp.Ci;
    const int kh = cp.ks == 3 ? (tap >= 6 ? 2 : (tap >= 3 ? 1 : 0)) : 0;
    const int ih = cr.ih0[i] + kh, iw = cr.iw0[i] + (tap - kh * cp.ks);
    if (ih < 0 || ih >= cp.Hin || iw < 0 || iw >= cp.Win) return g_uva_zero_page;
    return P + (((long long)cr.n[i] * cp.Hin + ih) * cp.Win + iw) * cp.Ci + ci;
  }
}

__device__ __forceinline__ void conv_rows_init_v2(const ConvParams& cp, int row0, int M, ConvRows& cr) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, hw = cp.Hout * cp.Wout;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = row0 + ((w * 4 + i) * 512 + l * 8) / 64;
    cr.ok[i] = m < M;
    int mm = cr.ok[i] ? m : 0;
    int n = mm / hw, r = mm % hw;
    cr.n[i] = n;
    cr.ih0[i] = (r / cp.Wout) * cp.stride - cp.pad_t;
    cr.iw0[i] = (r % cp.Wout) * cp.stride - cp.pad_l;
  }
}

template <int T>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ P, long long ld, int row0, int nrows, int k0, int K,
                                         bf16* lds, const ConvParams& cp, const ConvRows& cr) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16* src = dma_addr<T>(P, ld, row0, nrows, k0, K, i, cp, cr);
    bf16* dst = lds + (w * 4 + i) * 512;  // wave-uniform base; hardware adds lane * 16 B
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  }
}

template <int TA, int TB, typename TC>
__global__ __launch_bounds__(256, 2) void gemm_mfma_v2(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       TC* __restrict__ C, int M, int N, int K, long long lda,
                                                       long long ldb, long long ldc, BatchStrides bs, EpiParams ep,
                                                       ConvParams cp, float* __restrict__ part, int k_per_split) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* sA = (bf16*)smem;            // 2 x 8192 elements
  bf16* sB = sA + 2 * 8192;          // 2 x 8192 elements
  const int z = blockIdx.z, zo = z / bs.binner, zi = z % bs.binner;
  A += zo * bs.sAo + zi * bs.sAi;
  B += zo * bs.sBo + zi * bs.sBi;
  const long long coff = zo * bs.sCo + zi * bs.sCi;
  const long long roff = zo * ep.sRo + zi * ep.sRi;
  const int tm = (M + MB_M - 1) / MB_M, tn = (N + MB_N - 1) / MB_N;
  const int nblk = tm * tn;
  int pid = xcd_remap(blockIdx.x, nblk);
  const int GROUP = 8;
  int group = pid / (GROUP * tn), first_m = group * GROUP;
  int gsz = min(tm - first_m, GROUP);
  int bm = first_m + (pid % (GROUP * tn)) % gsz;
  int bn = (pid % (GROUP * tn)) / gsz;
  const int m0 = bm * MB_M, n0 = bn * MB_N;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  ConvRows cr;
  if (TA == 2) conv_rows_init_v2(cp, m0, M, cr);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nk = (kend - kbeg + MB_K - 1) / MB_K;
  dma_tile<TA>(A, lda, m0, M, kbeg, kend, sA, cp, cr);
  dma_tile<TB>(B, ldb, n0, N, kbeg, kend, sB, cp, cr);
  __syncthreads();  // waits vmcnt(0): the LDS-DMA of tile 0 has landed
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      dma_tile<TA>(A, lda, m0, M, kbeg + (kt + 1) * MB_K, kend, sA + (cur ^ 1) * 8192, cp, cr);
      dma_tile<TB>(B, ldb, n0, N, kbeg + (kt + 1) * MB_K, kend, sB + (cur ^ 1) * 8192, cp, cr);
    }
    const bf16* cA = sA + cur * 8192;
    const bf16* cB = sB + cur * 8192;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_load_v2<TA>(cA, wm * 64 + i * 16, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_load_v2<TB>(cB, wn * 64 + j * 16, ks);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    cur ^= 1;
  }
  epilogue_tile<TC>(acc, smem, C, M, N, ldc, coff, ep, roff, m0, n0, z,
                    part ? part + (long long)blockIdx.y * M * N : nullptr, (TA == 2) ? cp.gn_part : nullptr, bm);
}

// =====================================================================================
// gemm_8ph -- 256-row block tile, 8 waves, BK = 64, LDS-DMA staging with an 8-phase
// (2 K-tiles) schedule (cdna_hip_programming.md §5 "256² 8-phase template", T1-T5):
//   * each K-tile is split into 4 half-tiles: A-h0/A-h1 = the first/second half of every
//     wave-row's A rows, B-h0/B-h1 likewise for columns; the LDS image of each half is
//     lane-linear (global_load_lds) with the XOR swizzle applied on the source address;
//   * phase j of K-tile t reads one operand half into registers -- A-h0, B-h1, A-h1 and (in
//     phase 3) B-h0 of tile t+1, i.e. 8/4/8/4 ds_read_b128 -- issues one half-tile of DMA for
//     tile t+2 (B-h0, A-h0, B-h1, A-h1: each ~7 phases ahead of its first read), and runs one
//     16x16x32 MFMA quadrant (A0B0, A0B1, A1B0, A1B1) between two raw s_barriers;
//   * the only vmcnt wait is in phase 2 (counted: GA + 2*GB loads stay in flight) and it
//     retires exactly tile t+1; a half is restaged one phase after the phase whose
//     lgkmcnt(0) -- issued before that phase's first barrier -- retired its last ds_read;
//   * waves 4-7 run one barrier behind waves 0-3 (ping-pong: per SIMD one wave's MFMAs overlap
//     the other's LDS reads); the retire-before-barrier rule keeps the WAR order valid for
//     both wave groups.
// BN = 256: waves 2(M) x 4(N) of 128x64;  BN = 128: waves 4(M) x 2(N) of 64x64.
// =====================================================================================
template <int W>
__device__ __forceinline__ int mswz_w(int k) {
  if constexpr (W == 128) return ((k & 3) << 1) | (((k >> 3) & 1) << 3);   // 256-B rows, 16 chunks
  else return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2);                // 128-B rows, 8 chunks
}

// global row (inside the block tile) of row r of half h: rows are grouped per wave-row
template <int RW>
__device__ __forceinline__ int half_row(int r, int h) {
  constexpr int RH = RW / 2;
  return (r / RH) * RW + h * RH + (r % RH);
}

// per-lane source of wave-instruction i of half h (G instructions per wave per half)
template <int T, int RW, int W, int G>
__device__ __forceinline__ const bf16* dma8_addr(const bf16* __restrict__ P, long long ld, int row0, int nrows, int k0,
                                                 int K, int h, int i, const ConvParams& cp, const ConvRows& cr) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int e = (w * G + i) * 512 + l * 8;
  if constexpr (T == 1) {
    const int kr = e / W, cl = (e % W) >> 3;
    const int m = half_row<RW>((cl ^ mswz_w<W>(kr)) << 3, h);
    const int gk = k0 + kr, gr = row0 + m;
    return (gr < nrows && gk < K) ? P + (long long)gk * ld + gr : g_uva_zero_page;
  } else {
    const int r = e >> 6, cl = (e & 63) >> 3;
    const int k = k0 + ((cl ^ (r & 7)) << 3);
    if constexpr (T == 0) {
      const int gr = row0 + half_row<RW>(r, h);
      return (gr < nrows && k < K) ? P + (long long)gr * ld + k : g_uva_zero_page;
    } else {
      const int ci_ = h * G + i;
      if (!cr.ok[ci_] || k >= K) return g_uva_zero_page;
      const int tap = ((cp.Ci & 63) == 0) ? __builtin_amdgcn_readfirstlane(k0 / cp.Ci) : k / cp.Ci;
      const int ci = k - tap * cp.Ci;
      const int kh = cp.ks == 3 ? (tap >= 6 ? 2 : (tap >= 3 ? 1 : 0)) : 0;
      const int ih = cr.ih0[ci_] + kh, iw = cr.iw0[ci_] + (tap - kh * cp.ks);
      if (ih < 0 || ih >= cp.Hin || iw < 0 || iw >= cp.Win) return g_uva_zero_page;
      return P + (((long long)cr.n[ci_] * cp.Hin + ih) * cp.Win + iw) * cp.Ci + ci;
    }
  }
}

template <int T, int RW, int W, int G>
__device__ __forceinline__ void dma8_half(const bf16* __restrict__ P, long long ld, int row0, int nrows, int k0, int K,
                                          int h, bf16* img, const ConvParams& cp, const ConvRows& cr) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const bf16* src = dma8_addr<T, RW, W, G>(P, ld, row0, nrows, k0, K, h, i, cp, cr);
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(img + (w * G + i) * 512),
                                     16, 0, 0);
  }
}

// fragment (16 rows x 32 k) from a half image; r0 = first image row / column of the fragment
template <int T, int W>
__device__ __forceinline__ bf16x8 frag8(const bf16* img, int r0, int ks) {
  const int l = threadIdx.x & 63;
  if constexpr (T != 1) {
    const int row = r0 + (l & 15);
    const int c = ks * 4 + (l >> 4);
    return *(const bf16x8*)(img + row * 64 + ((c ^ (row & 7)) << 3));
  } else {
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int k = ks * 32 + g * 8 + q;
    const int col = r0 + 4 * p;
    const int c = col >> 3, w = col & 7;
    const bf16* a0 = img + k * W + ((c ^ mswz_w<W>(k)) << 3) + w;
    const bf16* a1 = img + (k + 4) * W + ((c ^ mswz_w<W>(k + 4)) << 3) + w;
    // inline asm: the intrinsic form makes hipcc wait vmcnt(0) (LDS-DMA alias) before every read;
    // completion is ordered by the explicit lgkmcnt(0) + sched_barrier before the MFMAs
    s16x4 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"((unsigned)(size_t)LDS_PTR(char, a0)) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"((unsigned)(size_t)LDS_PTR(char, a1)) : "memory");
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <int RW>
__device__ __forceinline__ void conv_rows_init_8(const ConvParams& cp, int row0, int M, ConvRows& cr) {
  // A halves: 2 x 2 wave-instructions per thread; image row r = ((w*2+i)*512 + l*8) >> 6
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, hw = cp.Hout * cp.Wout;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = ((w * 2 + i) * 512 + l * 8) >> 6;
      const int m = row0 + half_row<RW>(r, h);
      const int c = h * 2 + i;
      cr.ok[c] = m < M;
      const int mm = cr.ok[c] ? m : 0;
      const int n = mm / hw, rr = mm % hw;
      cr.n[c] = n;
      cr.ih0[c] = (rr / cp.Wout) * cp.stride - cp.pad_t;
      cr.iw0[c] = (rr % cp.Wout) * cp.stride - cp.pad_l;
    }
}

// BN = 384 is the 128 x 384 tile (N = 768 outputs: 2 x 256 row tiles fill exactly two rounds of 256
// CUs, where 256 x 256 tiles leave the second round half empty)
template <int BN>
struct Gemm8Cfg {
  static constexpr int BM = (BN == 384) ? 128 : 256, WM = (BN == 128) ? 4 : 2, WN = 8 / WM;
  static constexpr int ER = (BN == 384) ? 64 : 128;      // epilogue rows per LDS chunk
  static constexpr int NCH = BM / ER;                    // epilogue chunks
  static constexpr int RWA = BM / WM, RWB = BN / WN;      // rows (cols) per wave
  static constexpr int FM = RWA / 16, FN = RWB / 16;      // fragments per wave
  static constexpr int HA = FM / 2, HB = FN / 2;          // fragments per half
  static constexpr int A_HALF = (BM / 2) * 64, B_HALF = (BN / 2) * 64;   // elements
  static constexpr int GA = A_HALF / 4096, GB = B_HALF / 4096;          // DMA instrs per thread per half
  static constexpr int WA = BM / 2, WB = BN / 2;          // M-major image row widths (elements)
  static constexpr int STAGE = 2 * A_HALF + 2 * B_HALF;   // elements per K-tile stage
  static constexpr int TP = BN + 4;                       // epilogue fp32 pitch
  static constexpr int EPI_BYTES = ER * TP * 4 + 8 * 32 * 8 * 2 * 4;
  static constexpr int LDS_BYTES = (2 * STAGE * 2 > EPI_BYTES) ? 2 * STAGE * 2 : EPI_BYTES;
};

// VAR: 0 = the general path, 256 = the fast path (full tiles, K a multiple of 64: per-lane DMA
// sources precomputed once).  Only these two are built into the library.  The other bits name
// the structural alternatives that were measured against them and lost (same-box A/B, DESIGN.md
// §5); they stay as compile-time switches of this template for re-measurement, never selected at
// run time: 2 no wave-group stagger, 4 no compiler memory fences around barriers, 8 lgkmcnt after
// the barrier (timing only: breaks the WAR order), 16 no s_setprio, 64 __syncthreads() epilogue
// barriers, 512 no output stores (timing only), 1024 non-temporal output stores.
#define GEMM8_SYNC()                                     \
  do {                                                   \
    if constexpr (!(VAR & 4)) asm volatile("" ::: "memory"); \
  } while (0)

template <int TA, int TB, int BN, typename TC, int VAR = 0>
__global__ __launch_bounds__(512, 1) void gemm_8ph(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                   TC* __restrict__ C, int M, int N, int K, long long lda,
                                                   long long ldb, long long ldc, BatchStrides bs, EpiParams ep,
                                                   ConvParams cp, float* __restrict__ part, int k_per_split) {
  using G = Gemm8Cfg<BN>;
  static_assert(BN != 384 || TA != 2, "the 128x384 tile has no conv / GN-statistics epilogue");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* lds = (bf16*)smem;
  const int z = blockIdx.z, zo = z / bs.binner, zi = z % bs.binner;
  A += zo * bs.sAo + zi * bs.sAi;
  B += zo * bs.sBo + zi * bs.sBi;
  const long long coff = zo * bs.sCo + zi * bs.sCi;
  const long long roff = zo * ep.sRo + zi * ep.sRi;
  const int tm = (M + G::BM - 1) / G::BM, tn = (N + BN - 1) / BN;
  const int nblk = tm * tn;
  const int pid = xcd_remap(blockIdx.x, nblk);
  const int GROUP = 8;
  const int group = pid / (GROUP * tn), first_m = group * GROUP;
  const int gsz = min(tm - first_m, GROUP);
  const int bm = first_m + (pid % (GROUP * tn)) % gsz;
  const int bn = (pid % (GROUP * tn)) / gsz;
  const int m0 = bm * G::BM, n0 = bn * BN;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nt = (kend - kbeg + 63) / 64;
  ConvRows cr;
  if constexpr (TA == 2) conv_rows_init_8<G::RWA>(cp, m0, M, cr);
  const int wid = threadIdx.x >> 6;
  const int wr = wid / G::WN, wc = wid % G::WN;

  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int i = 0; i < G::FM; ++i)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // stage layout: [A-h0][A-h1][B-h0][B-h1]
  auto img_a = [&](int buf, int h) { return lds + buf * G::STAGE + h * G::A_HALF; };
  auto img_b = [&](int buf, int h) { return lds + buf * G::STAGE + 2 * G::A_HALF + h * G::B_HALF; };
  // VAR & 256 (fast path; full tiles, K range a multiple of 64, TA != 2): the per-lane DMA sources of
  // K-tile 0 are computed once and advanced by one uniform stride per K-tile -- the general path
  // re-derives them (swizzle, bounds, zero page) for every half-tile, ~25 VALU per DMA instruction
  // per-lane 32-bit byte offsets from the (uniform) operand base, so every DMA is SGPR base + VGPR
  // offset with no per-tile vector address arithmetic (operands < 4 GiB: checked by the launcher)
  unsigned offA[2][G::GA], offB[2][G::GB];
  const long long stepA = (TA == 1 ? 64 * lda : 64) * 2, stepB = (TB == 1 ? 64 * ldb : 64) * 2;  // bytes
  if constexpr ((VAR & 256) != 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < G::GA; ++i)
        offA[h][i] = (unsigned)((const char*)dma8_addr<TA, G::RWA, G::WA, G::GA>(A, lda, m0, M, kbeg, kend, h, i, cp, cr) -
                                (const char*)A);
#pragma unroll
      for (int i = 0; i < G::GB; ++i)
        offB[h][i] = (unsigned)((const char*)dma8_addr<TB, G::RWB, G::WB, G::GB>(B, ldb, n0, N, kbeg, kend, h, i, cp, cr) -
                                (const char*)B);
    }
  }
  const int w8 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // buffer descriptors built from kernargs only (wave-uniform by construction): the per-tile step is
  // the SGPR soffset, so the DMA issue needs no vector address arithmetic at all
  const int nrA = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)min(2ull * (unsigned long long)(TA == 1 ? K : M) * (unsigned long long)lda, 0xffffffffull));
  const int nrB = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)min(2ull * (unsigned long long)(TB == 1 ? K : N) * (unsigned long long)ldb, 0xffffffffull));
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, nrA, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, nrB, 0x00020000);
  // issue half-tile q of K-tile t (q order A-h0, B-h0, B-h1, A-h1; global sequence S = 4t + q)
  auto stage = [&](auto qc, int t) {
    constexpr int q = decltype(qc)::value;
    const int buf = t & 1, k0 = kbeg + t * 64;
    if constexpr ((VAR & 256) != 0) {
      if constexpr (q == 0 || q == 3) {
        constexpr int h = q == 0 ? 0 : 1;
        bf16* img = img_a(buf, h);
        const int so = (int)(unsigned)(t * stepA);
#pragma unroll
        for (int i = 0; i < G::GA; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(img + (w8 * G::GA + i) * 512),
                                                   16, (int)offA[h][i], so, 0, 0);
      } else {
        constexpr int h = q - 1;
        bf16* img = img_b(buf, h);
        const int so = (int)(unsigned)(t * stepB);
#pragma unroll
        for (int i = 0; i < G::GB; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(img + (w8 * G::GB + i) * 512),
                                                   16, (int)offB[h][i], so, 0, 0);
      }
    } else if constexpr (q == 0 || q == 3) {
      constexpr int h = q == 0 ? 0 : 1;
      dma8_half<TA, G::RWA, G::WA, G::GA>(A, lda, m0, M, k0, kend, h, img_a(buf, h), cp, cr);
    } else {
      constexpr int h = q - 1;
      dma8_half<TB, G::RWB, G::WB, G::GB>(B, ldb, n0, N, k0, kend, h, img_b(buf, h), cp, cr);
    }
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  using Q2 = std::integral_constant<int, 2>;
  using Q3 = std::integral_constant<int, 3>;
  // DMA order inside a K-tile: B-h0, A-h0, B-h1, A-h1 (the order in which their last reads end)
  stage(Q1{}, 0);
  stage(Q0{}, 0);
  stage(Q2{}, 0);
  stage(Q3{}, 0);
  if (nt >= 2) {
    stage(Q1{}, 1);
    stage(Q0{}, 1);
    stage(Q2{}, 1);
    stage(Q3{}, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::GA + 2 * G::GB) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  GEMM8_SYNC();
  __builtin_amdgcn_s_barrier();
  GEMM8_SYNC();
  bf16x8 fa[G::HA][2], fb0[G::HB][2], fb1[G::HB][2];
  // B-h0 fragments of tile 0 (afterwards prefetched in phase 3 of the previous tile); every wave
  // retires them before the common barrier below: phase 0 restages B-h0 of this buffer
#pragma unroll
  for (int g = 0; g < G::HB; ++g)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) fb0[g][ks] = frag8<TB, G::WB>(img_b(0, 0), wc * (G::RWB / 2) + g * 16, ks);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  GEMM8_SYNC();
  __builtin_amdgcn_s_barrier();
  GEMM8_SYNC();
  // stagger: waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave's MFMA
  // cluster overlaps the other wave's LDS reads / DMA issue
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2);
  if (!(VAR & 2) && grp == 1) __builtin_amdgcn_s_barrier();
  GEMM8_SYNC();

#define GEMM8_QUAD(AH, BH, FB)                                                                            \
  if constexpr (!(VAR & 16)) __builtin_amdgcn_s_setprio(1);                                               \
  _Pragma("unroll") for (int f = 0; f < G::HA; ++f)                                                       \
  _Pragma("unroll") for (int g = 0; g < G::HB; ++g)                                                       \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                        \
    acc[AH * G::HA + f][BH * G::HB + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                       \
        fa[f][ks], FB[g][ks], acc[AH * G::HA + f][BH * G::HB + g], 0, 0, 0);                              \
  if constexpr (!(VAR & 16)) __builtin_amdgcn_s_setprio(0)

#define GEMM8_SYNC_MFMA_BEGIN()                                                                           \
  if constexpr (!(VAR & 8)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* retire reads BEFORE the barrier */ \
  GEMM8_SYNC();                                                                                           \
  __builtin_amdgcn_s_barrier();                                                                           \
  if constexpr (VAR & 8) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                              \
  __builtin_amdgcn_sched_barrier(0)

#define GEMM8_SYNC_MFMA_END()                                                                             \
  __builtin_amdgcn_s_barrier();                                                                           \
  GEMM8_SYNC()

  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    const bool pf = t + 2 < nt;  // tile t+2 exists: stage it into this buffer, one half per phase
    // ---- phase 0: read A-h0 ; DMA B-h0(t+2) ; MFMA (A0, B0)
#pragma unroll
    for (int f = 0; f < G::HA; ++f)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[f][ks] = frag8<TA, G::WA>(img_a(buf, 0), wr * (G::RWA / 2) + f * 16, ks);
    if (pf) stage(Q1{}, t + 2);
    GEMM8_SYNC_MFMA_BEGIN();
    GEMM8_QUAD(0, 0, fb0);
    GEMM8_SYNC_MFMA_END();
    // ---- phase 1: read B-h1 ; DMA A-h0(t+2) ; MFMA (A0, B1)
#pragma unroll
    for (int g = 0; g < G::HB; ++g)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb1[g][ks] = frag8<TB, G::WB>(img_b(buf, 1), wc * (G::RWB / 2) + g * 16, ks);
    if (pf) stage(Q0{}, t + 2);
    GEMM8_SYNC_MFMA_BEGIN();
    GEMM8_QUAD(0, 1, fb1);
    GEMM8_SYNC_MFMA_END();
    // ---- phase 2: read A-h1 ; DMA B-h1(t+2) ; retire tile t+1 ; MFMA (A1, B0)
#pragma unroll
    for (int f = 0; f < G::HA; ++f)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[f][ks] = frag8<TA, G::WA>(img_a(buf, 1), wr * (G::RWA / 2) + f * 16, ks);
    if (pf) {
      stage(Q2{}, t + 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::GA + 2 * G::GB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    GEMM8_SYNC_MFMA_BEGIN();
    GEMM8_QUAD(1, 0, fb0);
    GEMM8_SYNC_MFMA_END();
    // ---- phase 3: read B-h0 of tile t+1 (retired in phase 2) ; DMA A-h1(t+2) ; MFMA (A1, B1)
    if (t + 1 < nt) {
#pragma unroll
      for (int g = 0; g < G::HB; ++g)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          fb0[g][ks] = frag8<TB, G::WB>(img_b(buf ^ 1, 0), wc * (G::RWB / 2) + g * 16, ks);
    }
    if (pf) stage(Q3{}, t + 2);
    GEMM8_SYNC_MFMA_BEGIN();
    GEMM8_QUAD(1, 1, fb1);
    GEMM8_SYNC_MFMA_END();
  }
#undef GEMM8_QUAD
#undef GEMM8_SYNC_MFMA_BEGIN
#undef GEMM8_SYNC_MFMA_END
  if (!(VAR & 2) && grp == 0) __builtin_amdgcn_s_barrier();  // re-align barrier counts: every wave is past its last MFMA
  GEMM8_SYNC();

  // ---------------- epilogue: 128-row chunks staged through LDS as fp32
  float* T = (float*)smem;
  float* pslab = part ? part + (long long)blockIdx.y * M * N : nullptr;
  float* gn_part = (TA == 2) ? cp.gn_part : nullptr;
  const int lane = threadIdx.x & 63;
  constexpr int C8 = BN / 8;             // 8-column chunks per row
  constexpr int RPP = 512 / C8;          // rows per pass (BN = 384: 10 rows, the last 32 threads idle)
  constexpr int ER = G::ER;
  const int c8 = threadIdx.x % C8, rsub = (threadIdx.x / C8 < RPP) ? (int)threadIdx.x / C8 : ER;
  const int col0 = n0 + c8 * 8;
  const bool full = (col0 + 8 <= N) && (ldc % 8 == 0) && ((coff + col0) % 8 == 0);
  float bv[8];
  if (!pslab && full) epi_load_bias8(ep, col0, bv);
  const bool plain = !ep.residual && !ep.gate && !ep.aux && ep.act == 0 && ep.drop_thresh == 0 && ep.beta == 0.f;
  // residual-only epilogues (attention proj / fc2 forward: bias + dropout + fp32 residual) stream
  // the residual rows through a ring RQ deep (RQ 32-B loads in flight per thread instead of the
  // general path's one row ahead): the N = 768 products were bound by that stream (404 TFLOP/s
  // at M32768 N768 K768 with the 128 x 384 tile)
  // (128 x 384 tile only: with the 256 x 256 tile's 128 accumulator registers still live in the
  // second chunk's waves, the ring spilled)
  const bool resonly = BN == 384 && TA != 2 && !pslab && full && ep.residual && !ep.gate && !ep.aux && ep.beta == 0.f &&
                       ep.res_grad == 0 && ep.res_dt == UVA_DT_F32 && (ep.ldr % 4 == 0) && (roff % 4 == 0);
#pragma unroll
  for (int chunk = 0; chunk < G::NCH; ++chunk) {
    float gs_s[8], gs_q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gs_s[e] = gs_q[e] = 0.f;
    // waves whose rows fall in [chunk*128, chunk*128+128) write their accumulators
    if ((wr * G::RWA) / ER == chunk) {
      const int rbase = wr * G::RWA - chunk * ER;
#pragma unroll
      for (int i = 0; i < G::FM; ++i)
#pragma unroll
        for (int j = 0; j < G::FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            T[(rbase + i * 16 + (lane >> 4) * 4 + r) * G::TP + wc * G::RWB + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    if constexpr (VAR & 64) __syncthreads(); else epi_lds_barrier();
    constexpr int NIT = (ER + RPP - 1) / RPP;
    const int rowb = m0 + chunk * ER + rsub;
    const int rowe = min(M, m0 + chunk * ER + ER);  // rows of this chunk (rl < ER)
    // (the conv variant keeps the general loop: the GN statistics leave no registers for these)
    if (TA != 2 && !pslab && full && plain && !(VAR & 512)) {
      // alpha * acc (+ bias): no loads inside the loop, so no store ever waits for an earlier one
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int row = rowb + it * RPP;
        if (row < rowe) {
          const int rl = it * RPP + rsub;
          const float4 a = *(const float4*)(T + rl * G::TP + c8 * 8);
          const float4 b = *(const float4*)(T + rl * G::TP + c8 * 8 + 4);
          const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = ep.alpha * v[e] + bv[e];
          TC* dst = C + coff + (long long)row * ldc + col0;
          if constexpr (sizeof(TC) == 2) {
            bf16x8 ov;
#pragma unroll
            for (int e = 0; e < 8; ++e) ov[e] = (bf16)o[e];
            *(bf16x8*)dst = ov;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (float)ov[e];
          } else {
            *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
            *(float4*)(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
          }
          if constexpr (TA == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              gs_s[e] += o[e];
              gs_q[e] += o[e] * o[e];
            }
          }
        }
      }
    } else if (BN == 384 && (VAR & 2048) == 0 && resonly && !(VAR & 512)) {
      constexpr int RQ = NIT < 4 ? NIT : 4;
      float4 rr[RQ][2];
      auto rload = [&](int it, int slot) __attribute__((always_inline)) {
        const int row = rowb + it * RPP;
        if (it < NIT && row < rowe) {
          const float* rp = (const float*)ep.residual + roff + (long long)row * ep.ldr + col0;
          rr[slot][0] = *(const float4*)rp;
          rr[slot][1] = *(const float4*)(rp + 4);
        }
      };
#pragma unroll
      for (int u = 0; u < RQ; ++u) rload(u, u);
      // rolled over groups of RQ rows (a fully unrolled loop hoisted every row's 64-bit addresses and
      // spilled them), static ring slots inside a group
#pragma unroll 1
      for (int it0 = 0; it0 < NIT; it0 += RQ) {
#pragma unroll
        for (int u = 0; u < RQ; ++u) {
          const int it = it0 + u;
          const int row = rowb + it * RPP;
          if (it < NIT && row < rowe) {
            const int rl = it * RPP + rsub;
            const float4 a = *(const float4*)(T + rl * G::TP + c8 * 8);
            const float4 b = *(const float4*)(T + rl * G::TP + c8 * 8 + 4);
            const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            const float4 r0 = rr[u][0], r1 = rr[u][1];
            const float res[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
            bool keep[8] = {true, true, true, true, true, true, true, true};
            if (ep.drop_thresh) {
              const uint64_t d0 = (uint64_t)((long long)z * M * N + (long long)row * N + col0);  // even
#pragma unroll
              for (int e = 0; e < 8; e += 2) dropout_keep2(ep.drop_seed, d0 + e, ep.drop_thresh, keep[e], keep[e + 1]);
            }
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float t = apply_act(ep.act, ep.alpha * v[e] + bv[e]);
              if (ep.drop_thresh) t = keep[e] ? t * ep.drop_scale : 0.f;
              o[e] = t + res[e];
            }
            TC* dst = C + coff + (long long)row * ldc + col0;
            if constexpr (sizeof(TC) == 2) {
              bf16x8 ov;
#pragma unroll
              for (int e = 0; e < 8; ++e) ov[e] = (bf16)o[e];
              *(bf16x8*)dst = ov;
            } else {
              *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
              *(float4*)(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
            }
          }
          rload(it + RQ, u);
        }
      }
    } else if (TA != 2 && !pslab && full && !(VAR & 512)) {
      // row it+1's inputs are loaded before row it's store (see EpiRow)
      EpiRow cur, nxt;
      if (rowb < rowe) epi_load_row8<TC>(C, coff + (long long)rowb * ldc + col0, ep, roff, rowb, col0, cur);
#pragma unroll 1
      for (int it = 0; it < NIT; ++it) {
        const int row = rowb + it * RPP;
        if (it + 1 < NIT && row + RPP < rowe)
          epi_load_row8<TC>(C, coff + (long long)(row + RPP) * ldc + col0, ep, roff, row + RPP, col0, nxt);
        if (row < rowe) {
          const int rl = it * RPP + rsub;
          const float4 a = *(const float4*)(T + rl * G::TP + c8 * 8);
          const float4 b = *(const float4*)(T + rl * G::TP + c8 * 8 + 4);
          const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
          float o[8];
          epi_apply_row8<TC, (VAR & 1024) != 0>(C, coff + (long long)row * ldc + col0, ep, bv, cur, row, col0, z, M,
                                                 N, v, o);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            gs_s[e] += o[e];
            gs_q[e] += o[e] * o[e];
          }
        }
        cur = nxt;
      }
    } else
    for (int it = 0; it < NIT; ++it) {
      const int rl = it * RPP + rsub;
      const int row = m0 + chunk * ER + rl;
      if (row >= rowe || col0 >= N) break;
      float v[8];
      const float4 a = *(const float4*)(T + rl * G::TP + c8 * 8);
      const float4 b = *(const float4*)(T + rl * G::TP + c8 * 8 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      if constexpr ((VAR & 512) != 0) {  // timing only: no output stores
        if (v[0] == 1234.5f && v[7] == -1234.5f) C[0] = (TC)0.f;
        continue;
      }
      if (pslab) {
        float* dst = pslab + (long long)row * N + col0;
        if (col0 + 8 <= N && N % 4 == 0) {
          *(float4*)dst = a;
          *(float4*)(dst + 4) = b;
        } else {
          for (int e = 0; e < 8 && col0 + e < N; ++e) dst[e] = v[e];
        }
        continue;
      }
      const long long cbase = coff + (long long)row * ldc + col0;
      if (full) {
        float o[8];
        epi_row8<TC, (VAR & 1024) != 0>(C, cbase, ep, roff, row, col0, z, M, N, v, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          gs_s[e] += o[e];
          gs_q[e] += o[e] * o[e];
        }
      } else {
        for (int e = 0; e < 8 && col0 + e < N; ++e) {
          const int col = col0 + e;
          float o = epi_store<TC>(C, ldc, coff, ep, roff, row, col, N,
                                  (long long)z * M * N + (long long)row * N + col, v[e]);
          gs_s[e] += o;
          gs_q[e] += o * o;
        }
      }
    }
    if constexpr (TA == 2) {
      if (gn_part) {
        // per-(128-row chunk, group) sums: lanes sharing c8 inside a wave, then the 8 waves via LDS
#pragma unroll
        for (int e = 0; e < 8; ++e) {
#pragma unroll
          for (int o = C8; o < 64; o <<= 1) {
            gs_s[e] += __shfl_xor(gs_s[e], o, 64);
            gs_q[e] += __shfl_xor(gs_q[e], o, 64);
          }
        }
        float* red = T + ER * G::TP;  // [8 waves][C8][8][2]
        if (lane < C8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[((wid * C8 + lane) * 8 + e) * 2 + 0] = gs_s[e];
            red[((wid * C8 + lane) * 8 + e) * 2 + 1] = gs_q[e];
          }
        }
        if constexpr (VAR & 64) __syncthreads(); else epi_lds_barrier();
        const int gsz = N / 32;
        const int ngroups = min(BN, N - n0) / gsz;
        if ((int)threadIdx.x < ngroups && m0 + chunk * ER < M) {
          float sum = 0.f, sq = 0.f;
          for (int c = threadIdx.x * gsz; c < ((int)threadIdx.x + 1) * gsz; ++c)
            for (int w = 0; w < 8; ++w) {
              sum += red[((w * C8 + (c >> 3)) * 8 + (c & 7)) * 2 + 0];
              sq += red[((w * C8 + (c >> 3)) * 8 + (c & 7)) * 2 + 1];
            }
          const int g = n0 / gsz + threadIdx.x;
          const long long tile = (long long)bm * 2 + chunk;
          gn_part[(tile * 32 + g) * 2 + 0] = sum;
          gn_part[(tile * 32 + g) * 2 + 1] = sq;
        }
      }
    }
    // LDS-only: the stores of this chunk stay in flight (a __syncthreads() would drain them), and
    // after the last chunk nothing reads T again
    if constexpr (VAR & 64) __syncthreads(); else if (chunk == 0) epi_lds_barrier();
  }
}

// UVA_GEMM_PERSIST: the default of the run-time switch uva_gemm_set_persist (0: gemm_8ph only, measured
// faster; 1: gemm_8pp where eligible); diagnostic bits 2 (one tile per workgroup) and 4 (next tile's DMA
// after the epilogue)
#ifndef UVA_GEMM_PERSIST
#define UVA_GEMM_PERSIST 0
#endif
static int g_gemm_persist = UVA_GEMM_PERSIST & 1;
extern "C" int uva_gemm_set_persist(int on) {
  const int prev = g_gemm_persist;
  if (on >= 0) g_gemm_persist = on ? 1 : 0;
  return prev;
}
// =====================================================================================
// gemm_8pp -- persistent form of gemm_8ph (full tiles, K a multiple of 64 and >= 128, batch 1, no
// K split; epilogue: alpha, bias, activation, dropout, pre-activation copy).  One workgroup per CU
// walks tiles pid = i * grid + xcd_remap(block) (the GROUP-8 raster of gemm_8ph inside each round),
// and at the end of a tile's K loop it
//   1. issues the NEXT tile's first two K-tiles of LDS-DMA (the LDS images are free: the epilogue
//      below runs from registers), then
//   2. finishes this tile from registers: the MFMAs are issued with the operands swapped (B as the
//      A operand), so a lane holds 4 consecutive output columns of one row, and one
//      v_permlane16_swap per accumulator word pairs two fragments into 8 consecutive columns:
//      16-B (bf16) / 2 x 16-B (fp32) row-segment stores, 64 contiguous bytes per row per instruction
//      across a 16-lane row group.
// The next tile then waits with a COUNTED vmcnt: its K-tile 0 DMAs are older than the E epilogue
// stores, so vmcnt(2GA + 2GB + E) retires exactly K-tile 0 and leaves the stores draining under the
// next K loop (E is the same in every wave: full tiles, unconditional stores).  gemm_8ph instead
// serialises prologue DMA latency, the LDS-staged epilogue and its store drain with the MFMAs at one
// workgroup per CU; hipBLASLt's fastest kernels at these shapes are persistent too (rocprofv3 names,
// profiles/r04/ab_gemm_persist.txt).
// =====================================================================================
template <int TA, int TB, int BN, typename TC>
__global__ __launch_bounds__(512, 1) void gemm_8pp(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                   TC* __restrict__ C, int M, int N, int K, long long lda,
                                                   long long ldb, long long ldc, EpiParams ep) {
  using G = Gemm8Cfg<BN>;
  static_assert(TA != 2 && TB != 2, "plain products only");
  static_assert(G::FN % 2 == 0, "the permlane16 pairing joins two 16-column fragments");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* lds = (bf16*)smem;
  const int tm = M / G::BM, tn = N / BN, ntiles = tm * tn;
  const int nt = K / 64;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wid / G::WN, wc = wid % G::WN;
  const int w8 = __builtin_amdgcn_readfirstlane(wid);
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2);
  const int G_ = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, G_);
  constexpr int GROUP = 8;
  auto tile_of = [&](int pid, int& m0, int& n0) __attribute__((always_inline)) {
    const int group = pid / (GROUP * tn), first_m = group * GROUP;
    const int gsz = min(tm - first_m, GROUP);
    m0 = (first_m + (pid % (GROUP * tn)) % gsz) * G::BM;
    n0 = ((pid % (GROUP * tn)) / gsz) * BN;
  };
  ConvParams cp0{};
  ConvRows cr0{};
  unsigned offA[2][G::GA], offB[2][G::GB];
  auto offsets = [&](int m0, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = 0; i < G::GA; ++i)
        offA[h][i] = (unsigned)((const char*)dma8_addr<TA, G::RWA, G::WA, G::GA>(A, lda, m0, M, 0, K, h, i, cp0, cr0) -
                                (const char*)A);
#pragma unroll
      for (int i = 0; i < G::GB; ++i)
        offB[h][i] = (unsigned)((const char*)dma8_addr<TB, G::RWB, G::WB, G::GB>(B, ldb, n0, N, 0, K, h, i, cp0, cr0) -
                                (const char*)B);
    }
  };
  const long long stepA = (TA == 1 ? 64 * lda : 64) * 2, stepB = (TB == 1 ? 64 * ldb : 64) * 2;  // bytes
  const int nrA = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)min(2ull * (unsigned long long)(TA == 1 ? K : M) * (unsigned long long)lda, 0xffffffffull));
  const int nrB = __builtin_amdgcn_readfirstlane(
      (int)(unsigned)min(2ull * (unsigned long long)(TB == 1 ? K : N) * (unsigned long long)ldb, 0xffffffffull));
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, nrA, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, nrB, 0x00020000);
  auto img_a = [&](int buf, int h) { return lds + buf * G::STAGE + h * G::A_HALF; };
  auto img_b = [&](int buf, int h) { return lds + buf * G::STAGE + 2 * G::A_HALF + h * G::B_HALF; };
  auto stage = [&](auto qc, int t) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    const int buf = t & 1;
    if constexpr (q == 0 || q == 3) {
      constexpr int h = q == 0 ? 0 : 1;
      bf16* img = img_a(buf, h);
      const int so = (int)(unsigned)(t * stepA);
#pragma unroll
      for (int i = 0; i < G::GA; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(img + (w8 * G::GA + i) * 512),
                                                 16, (int)offA[h][i], so, 0, 0);
    } else {
      constexpr int h = q - 1;
      bf16* img = img_b(buf, h);
      const int so = (int)(unsigned)(t * stepB);
#pragma unroll
      for (int i = 0; i < G::GB; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(img + (w8 * G::GB + i) * 512),
                                                 16, (int)offB[h][i], so, 0, 0);
    }
  };
  using Q0 = std::integral_constant<int, 0>;
  using Q1 = std::integral_constant<int, 1>;
  using Q2 = std::integral_constant<int, 2>;
  using Q3 = std::integral_constant<int, 3>;
  auto stage01 = [&]() __attribute__((always_inline)) {
    stage(Q1{}, 0);
    stage(Q0{}, 0);
    stage(Q2{}, 0);
    stage(Q3{}, 0);
    stage(Q1{}, 1);
    stage(Q0{}, 1);
    stage(Q2{}, 1);
    stage(Q3{}, 1);
  };
  // epilogue vector-memory instructions per wave (every one unconditional), for the counted wait
  constexpr int E1 = G::FM * (G::FN / 2) * (sizeof(TC) == 2 ? 1 : 2);
  constexpr int W0 = 2 * G::GA + 2 * G::GB;
  constexpr int WE = (W0 + E1) > 63 ? 63 : (W0 + E1), WEA = (W0 + 2 * E1) > 63 ? 63 : (W0 + 2 * E1);
  const bool has_aux = ep.aux != nullptr;

  int pid = slot;
  if (pid >= ntiles) return;
  int m0, n0;
  tile_of(pid, m0, n0);
  offsets(m0, n0);
  stage01();
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W0) : "memory");
  bool first = true;
  const int li = lane & 15, g4 = lane >> 4;
  const int csub = (g4 & 1) * 16 + (g4 >> 1) * 8;  // the lane's 8 columns inside a 32-column fragment pair
  for (;;) {
    if (!first) {
      // K-tile 0 of this tile was issued before the previous tile's E epilogue stores
      if constexpr ((UVA_GEMM_PERSIST & 4) != 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W0) : "memory");
      else if (has_aux) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WEA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WE) : "memory");
    }
    first = false;
    f32x4 acc[G::FM][G::FN];
#pragma unroll
    for (int i = 0; i < G::FM; ++i)
#pragma unroll
      for (int j = 0; j < G::FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    bf16x8 fa[G::HA][2], fb0[G::HB][2], fb1[G::HB][2];
#pragma unroll
    for (int g = 0; g < G::HB; ++g)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb0[g][ks] = frag8<TB, G::WB>(img_b(0, 0), wc * (G::RWB / 2) + g * 16, ks);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (grp == 1) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

#define GEMM8P_QUAD(AH, BH, FB)                                                                           \
  __builtin_amdgcn_s_setprio(1);                                                                          \
  _Pragma("unroll") for (int f = 0; f < G::HA; ++f)                                                       \
  _Pragma("unroll") for (int g = 0; g < G::HB; ++g)                                                       \
  _Pragma("unroll") for (int ks = 0; ks < 2; ++ks)                                                        \
    acc[AH * G::HA + f][BH * G::HB + g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                       \
        FB[g][ks], fa[f][ks], acc[AH * G::HA + f][BH * G::HB + g], 0, 0, 0);                              \
  __builtin_amdgcn_s_setprio(0)
#define GEMM8P_BEGIN()                                  \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
  asm volatile("" ::: "memory");                        \
  __builtin_amdgcn_s_barrier();                         \
  __builtin_amdgcn_sched_barrier(0)
#define GEMM8P_END()            \
  __builtin_amdgcn_s_barrier(); \
  asm volatile("" ::: "memory")

    float bv[G::FN / 2][8];
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool pf = t + 2 < nt;
      // phase 0: read A-h0 ; DMA B-h0(t+2) ; MFMA (A0, B0)
#pragma unroll
      for (int f = 0; f < G::HA; ++f)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[f][ks] = frag8<TA, G::WA>(img_a(buf, 0), wr * (G::RWA / 2) + f * 16, ks);
      if (pf) stage(Q1{}, t + 2);
      if (t == nt - 1) {
        // the epilogue's bias columns, a K-tile ahead of their use (retired by phase 2's vmcnt(0))
#pragma unroll
        for (int p = 0; p < G::FN / 2; ++p) epi_load_bias8(ep, n0 + wc * G::RWB + p * 32 + csub, bv[p]);
      }
      GEMM8P_BEGIN();
      GEMM8P_QUAD(0, 0, fb0);
      GEMM8P_END();
      // phase 1: read B-h1 ; DMA A-h0(t+2) ; MFMA (A0, B1)
#pragma unroll
      for (int g = 0; g < G::HB; ++g)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fb1[g][ks] = frag8<TB, G::WB>(img_b(buf, 1), wc * (G::RWB / 2) + g * 16, ks);
      if (pf) stage(Q0{}, t + 2);
      GEMM8P_BEGIN();
      GEMM8P_QUAD(0, 1, fb1);
      GEMM8P_END();
      // phase 2: read A-h1 ; DMA B-h1(t+2) ; retire tile t+1 ; MFMA (A1, B0)
#pragma unroll
      for (int f = 0; f < G::HA; ++f)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[f][ks] = frag8<TA, G::WA>(img_a(buf, 1), wr * (G::RWA / 2) + f * 16, ks);
      if (pf) {
        stage(Q2{}, t + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::GA + 2 * G::GB) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      GEMM8P_BEGIN();
      GEMM8P_QUAD(1, 0, fb0);
      GEMM8P_END();
      // phase 3: read B-h0 of tile t+1 ; DMA A-h1(t+2) ; MFMA (A1, B1)
      if (t + 1 < nt) {
#pragma unroll
        for (int g = 0; g < G::HB; ++g)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            fb0[g][ks] = frag8<TB, G::WB>(img_b(buf ^ 1, 0), wc * (G::RWB / 2) + g * 16, ks);
      }
      if (pf) stage(Q3{}, t + 2);
      GEMM8P_BEGIN();
      GEMM8P_QUAD(1, 1, fb1);
      GEMM8P_END();
    }
#undef GEMM8P_QUAD
#undef GEMM8P_BEGIN
#undef GEMM8P_END
    if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align: every wave has retired its last LDS read
    asm volatile("" ::: "memory");

    const int cm0 = m0, cn0 = n0;
    // ---- next tile: its first two K-tiles go out now, under this tile's epilogue.  After the last
    //      tile the current one is restaged instead (drained before the exit): an issue that depends on
    //      a branch leaves a join in front of the epilogue, where hipcc's wait-count merge would make
    //      the bias wait drain the DMAs too
    pid += G_;
    const bool more = pid < ntiles;
    if (more) {
      tile_of(pid, m0, n0);
      offsets(m0, n0);
    }
    if constexpr (!(UVA_GEMM_PERSIST & 4)) stage01();
    asm volatile("" ::: "memory");
    // ---- register epilogue (no LDS): 8 consecutive columns per lane per fragment pair
    EpiRow none;
#pragma unroll
    for (int i = 0; i < G::FM; ++i) {
      const int row = cm0 + wr * G::RWA + i * 16 + li;
#pragma unroll
      for (int p = 0; p < G::FN / 2; ++p) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * p][r]),
                                                          __float_as_uint(acc[i][2 * p + 1][r]), false, false);
          v[r] = __uint_as_float(x[0]);
          v[4 + r] = __uint_as_float(x[1]);
        }
        const int col = cn0 + wc * G::RWB + p * 32 + csub;
        float o[8];
        epi_apply_row8<TC>(C, (long long)row * ldc + col, ep, bv[p], none, row, col, 0, M, N, v, o);
      }
    }
    if constexpr ((UVA_GEMM_PERSIST & 4) != 0) {  // diagnostic: next tile's DMA after the epilogue
      asm volatile("" ::: "memory");
      stage01();
    }
    if (!more) break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the restaged DMAs land before the LDS is released
}

// number of compute units of the current device (persistent grids)
static int device_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <typename TC>
__global__ __launch_bounds__(256) void splitk_reduce(const float* __restrict__ part, int splits, TC* __restrict__ C,
                                                     int M, int N, long long ldc, EpiParams ep) {
  const long long n = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += part[k * n + i];
    int row = (int)(i / N), col = (int)(i % N);
    epi_store<TC>(C, ldc, 0, ep, 0, row, col, N, i, s);
  }
}

// Plain-epilogue fp32 reduce (the dW products: C = alpha * sum + beta * C), 16-byte lanes: the
// scalar kernel above spends its time on 4-byte loads and a 64-bit divide per element.
// The slab loads go out four at a time ahead of their (slice-ordered) adds, so a thread keeps four
// 16-B reads in flight instead of one; a contiguous C (ldc == N: every gradient buffer) skips the
// per-element 64-bit row division.
__global__ __launch_bounds__(256) void splitk_reduce_f32x4(const float4* __restrict__ part, int splits,
                                                           float* __restrict__ C, int N, long long n4, long long ldc,
                                                           float alpha, float beta) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 a = part[i];
    int k = 1;
    for (; k + 4 <= splits; k += 4) {
      const float4 b0 = part[k * n4 + i], b1 = part[(k + 1) * n4 + i];
      const float4 b2 = part[(k + 2) * n4 + i], b3 = part[(k + 3) * n4 + i];
      a.x += b0.x; a.y += b0.y; a.z += b0.z; a.w += b0.w;  // slice order kept: bitwise as one at a time
      a.x += b1.x; a.y += b1.y; a.z += b1.z; a.w += b1.w;
      a.x += b2.x; a.y += b2.y; a.z += b2.z; a.w += b2.w;
      a.x += b3.x; a.y += b3.y; a.z += b3.z; a.w += b3.w;
    }
    for (; k < splits; ++k) {
      const float4 b = part[k * n4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    const long long e = 4 * i;
    long long off = e;
    if (ldc != N) {
      const long long row = e / N;
      off = row * ldc + (e - row * N);
    }
    float4* c = (float4*)(C + off);
    float4 v = make_float4(alpha * a.x, alpha * a.y, alpha * a.z, alpha * a.w);
    if (beta != 0.f) {
      const float4 o = *c;
      v.x += beta * o.x; v.y += beta * o.y; v.z += beta * o.z; v.w += beta * o.w;
    }
    *c = v;
  }
}

template <typename TC>
static void launch_splitk_reduce(const float* part, int splits, void* C, int M, int N, long long ldc,
                                 const EpiParams& ep, hipStream_t s) {
  const long long n = (long long)M * N;
  const bool plain = !ep.bias && !ep.aux && !ep.residual && !ep.gate && ep.act == 0 && ep.drop_thresh == 0;
  if (sizeof(TC) == 4 && plain && N % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)C & 15) == 0 &&
      ((uintptr_t)part & 15) == 0) {
    const long long n4 = n / 4;
    long long blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    splitk_reduce_f32x4<<<dim3((unsigned)blocks), 256, 0, s>>>((const float4*)part, splits, (float*)C, N, n4, ldc,
                                                                ep.alpha, ep.beta);
    return;
  }
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  splitk_reduce<TC><<<dim3((unsigned)blocks), 256, 0, s>>>(part, splits, (TC*)C, M, N, ldc, ep);
}

// =====================================================================================
// host launchers
// =====================================================================================
template <typename TI, typename TC>
static int launch_generic(int ta, int tb, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                          long long ldb, long long ldc, int batch, const BatchStrides& bs, const EpiParams& ep,
                          const ConvParams& cp, hipStream_t s, float* ws = nullptr, long long ws_floats = 0) {
  const long long nblk = (long long)((N + 63) / 64) * ((M + 63) / 64);
  if (batch == 1 && ws && ta != 2 && nblk < 64 && K >= 4096) {
    // split K into slices of >= 256 so that ~512 blocks walk it; partial slabs in the workspace
    int splits = (int)((512 + nblk - 1) / nblk);
    if (splits > K / 256) splits = K / 256;
    while (splits > 1 && (long long)splits * M * N > ws_floats) --splits;
    if (splits > 1) {
      const int kps = ((K + splits - 1) / splits + 15) / 16 * 16;
      splits = (K + kps - 1) / kps;
      dim3 sgrid((N + 63) / 64, (M + 63) / 64, splits);
#define GS(a, b) gemm_generic<TI, TC, a, b, true><<<sgrid, 256, 0, s>>>((const TI*)A, (const TI*)B, (TC*)C, M, N, K, \
                                                                        lda, ldb, ldc, bs, ep, cp, ws, kps)
      if (ta == 0 && tb == 0) GS(0, 0);
      else if (ta == 0 && tb == 1) GS(0, 1);
      else if (ta == 1 && tb == 0) GS(1, 0);
      else if (ta == 1 && tb == 1) GS(1, 1);
      else return (int)hipErrorInvalidValue;
#undef GS
      UVA_LAUNCH_CHECK();
      launch_splitk_reduce<TC>(ws, splits, C, M, N, ldc, ep, s);
      UVA_LAUNCH_CHECK();
      return 0;
    }
  }
  dim3 grid((N + 63) / 64, (M + 63) / 64, batch);
#define GG(a, b) gemm_generic<TI, TC, a, b><<<grid, 256, 0, s>>>((const TI*)A, (const TI*)B, (TC*)C, M, N, K, lda, ldb, ldc, bs, ep, cp)
  if (ta == 2 && tb == 0) GG(2, 0);
  else if (ta == 0 && tb == 0) GG(0, 0);
  else if (ta == 0 && tb == 1) GG(0, 1);
  else if (ta == 1 && tb == 0) GG(1, 0);
  else if (ta == 1 && tb == 1) GG(1, 1);
  else return (int)hipErrorInvalidValue;
#undef GG
  UVA_LAUNCH_CHECK();
  return 0;
}

struct Plan8 {
  int bn, splits, kps;
  long long nblk;
};

// shape -> 8-phase configuration (bn = 0: not for this kernel)
static Plan8 plan_8ph(int ta, int M, int N, int K, int batch, bool gn_prologue, bool have_ws, long long ws_floats) {
  constexpr int f128 = 90;  // relative per-CU efficiency of BN=128 (measured, % of the 256x256 tile)
  constexpr int f384 = 85;  // ... of the 128x384 tile
  Plan8 p{0, 1, K, 0};
  if (M < 256 || N < 128 || (ta == 2 && gn_prologue)) return p;
  auto bm_of = [](int bn) { return bn == 384 ? 128 : 256; };
  auto tiles = [&](int bn) { return (long long)((M + bm_of(bn) - 1) / bm_of(bn)) * ((N + bn - 1) / bn); };
  // work per CU-round, relative: tile occupancy of the last round x useful fraction of each tile
  auto score = [&](int bn) {
    long long t = tiles(bn) * batch;
    long long rounds = (t + 255) / 256;
    double occ = (double)t / (double)(rounds * 256);
    double useful = (double)M * N / ((double)tiles(bn) * bm_of(bn) * bn);
    return occ * useful * (bn == 128 ? f128 / 100.0 : bn == 384 ? f384 / 100.0 : 1.0);
  };
  const bool splitk_regime = batch == 1 && have_ws && tiles(128) < 128 && K >= 8 * 64;
  // measured (tools_kbench.py): BN=256 beats the 128x128 LDS-DMA kernel on every UVA shape it is
  // chosen for, the 128x384 tile beats the 128x128 fallback on every N = 768 shape; a BN=128 form
  // of this kernel measured slower than the fallback kernel and is not built
  int bn;
  // the 128x384 tile: plain products (no conv view), N a multiple of 384, off the split-K regime
  const bool ok384 = ta != 2 && N % 384 == 0 && !splitk_regime;
  if (ok384 && score(384) > score(256)) bn = 384;
  else if (N < 256 || !(splitk_regime || score(256) >= score(128))) return p;
  else bn = 256;
  const long long nblk = tiles(bn);
  int splits = 1;
  if (batch == 1 && have_ws && nblk < 128 && K >= 8 * 64) {
    splits = (int)((256 + nblk / 2) / nblk);
    int kmax = K / (4 * 64);
    if (splits > kmax) splits = kmax;
    while (splits > 1 && (long long)splits * M * N > ws_floats) --splits;
  }
  if (nblk * splits * batch < 96) return p;  // too small to fill the chip with 1 block/CU
  int kps = K;
  if (splits > 1) {
    kps = ((K + splits - 1) / splits + 63) / 64 * 64;
    splits = (K + kps - 1) / kps;
  }
  p.bn = bn;
  p.splits = splits;
  p.kps = kps;
  p.nblk = nblk;
  return p;
}

// 8-phase 256-row kernel: returns 1 if launched, 0 if the shape is not for it, <0 on error
template <typename TC>
static int launch_8ph(int ta, int tb, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                      long long ldb, long long ldc, int batch, const BatchStrides& bs, const EpiParams& ep,
                      const ConvParams& cp, float* ws, long long ws_floats, hipStream_t s) {
  const Plan8 pl = plan_8ph(ta, M, N, K, batch, cp.gn_scale != nullptr, ws != nullptr, ws_floats);
  if (pl.bn == 0) return 0;
  const int bn = pl.bn, splits = pl.splits, kps = pl.kps;
  const long long nblk = pl.nblk;
  float* part = splits > 1 ? ws : nullptr;
  dim3 grid((unsigned)nblk, splits, batch);
#define G8X(a, b, BNV, VV)                                                                                  \
  do {                                                                                                      \
    static bool attr = false;                                                                               \
    const int lb = Gemm8Cfg<BNV>::LDS_BYTES;                                                                \
    if (!attr) {                                                                                            \
      (void)hipFuncSetAttribute((const void*)gemm_8ph<a, b, BNV, TC, VV>, hipFuncAttributeMaxDynamicSharedMemorySize, lb); \
      attr = true;                                                                                          \
    }                                                                                                       \
    gemm_8ph<a, b, BNV, TC, VV><<<grid, 512, lb, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, lda, ldb, ldc, \
                                                      bs, ep, cp, part, kps);                               \
  } while (0)
  // full tiles + K a multiple of 64 (every K-slice then is one too): the precomputed-source fast path
  auto span = [](int t, int rows, int cols, long long ld) {  // bytes an operand's offsets can reach
    return 2.0 * ((t == 1 ? (double)cols : (double)rows) * (double)ld);
  };
  const bool fast = ta != 2 && M % (bn == 384 ? 128 : 256) == 0 && N % bn == 0 && K % 64 == 0 && batch == 1 &&
                    span(ta, M, K, lda) < 4.0e9 && span(tb, N, K, ldb) < 4.0e9;
  // persistent form (gemm_8pp): full tiles, one K range, an epilogue without row inputs
  const bool persist = g_gemm_persist && fast && splits == 1 && K >= 128 && ep.residual == nullptr &&
                       ep.gate == nullptr && ep.beta == 0.f && ep.res_grad == 0 && ldc % 8 == 0 &&
                       (((uintptr_t)C | (uintptr_t)ep.aux | (uintptr_t)ep.bias) % 16) == 0;
  if (persist) {
    // (UVA_GEMM_PERSIST & 2: diagnostic, one tile per workgroup)
    const unsigned g = (UVA_GEMM_PERSIST & 2) ? (unsigned)nblk : (unsigned)std::min<long long>(nblk, (long long)device_cus());
#define G8P(a, b, BNV)                                                                                        do {                                                                                                          static bool attr = false;                                                                                   const int lb = Gemm8Cfg<BNV>::LDS_BYTES;                                                                    if (!attr) {                                                                                                  (void)hipFuncSetAttribute((const void*)gemm_8pp<a, b, BNV, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, lb);       attr = true;                                                                                              }                                                                                                           gemm_8pp<a, b, BNV, TC><<<dim3(g), 512, lb, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, lda, ldb, ldc, ep);   } while (0)
#define G8PC(a, b) do { if (bn == 384) G8P(a, b, 384); else G8P(a, b, 256); } while (0)
    if (ta == 0 && tb == 0) G8PC(0, 0);
    else if (ta == 0 && tb == 1) G8PC(0, 1);
    else if (ta == 1 && tb == 0) G8PC(1, 0);
    else if (ta == 1 && tb == 1) G8PC(1, 1);
    else return -(int)hipErrorInvalidValue;
#undef G8PC
#undef G8P
    UVA_LAUNCH_CHECK();
    return 1;
  }
#define G8(a, b, BNV) do { if (fast) G8X(a, b, BNV, 256); else G8X(a, b, BNV, 0); } while (0)
#define G8B(a, b) G8(a, b, 256)
#define G8C(a, b) do { if (bn == 384) G8(a, b, 384); else G8B(a, b); } while (0)
  if (ta == 2 && tb == 0) G8B(2, 0);
  else if (ta == 0 && tb == 0) G8C(0, 0);
  else if (ta == 0 && tb == 1) G8C(0, 1);
  else if (ta == 1 && tb == 0) G8C(1, 0);
  else if (ta == 1 && tb == 1) G8C(1, 1);
  else return -(int)hipErrorInvalidValue;
#undef G8C
#undef G8B
#undef G8
#undef G8X
  UVA_LAUNCH_CHECK();
  if (part) {
    launch_splitk_reduce<TC>(part, splits, C, M, N, ldc, ep, s);
    UVA_LAUNCH_CHECK();
  }
  return 1;
}

extern "C" int uva_gemm4_try(int out_dtype, const void* A, const void* B, void* C, int M, int N, int K,
                             long long lda, long long ldb, long long ldc, const float* bias, float alpha,
                             hipStream_t s);
extern "C" int uva_gemm8w_try(int out_dtype, const void* A, const void* B, void* C, int M, int N, int K,
                              long long lda, long long ldb, long long ldc, const float* bias, float alpha,
                              hipStream_t s);
extern "C" int uva_gemm8w_tt_try(const void* A, const void* B, float* C, int M, int N, int K, long long lda,
                                 long long ldb, long long ldc, float alpha, float beta, float* ws, long long ws_floats,
                                 int* reduce, hipStream_t s);
extern "C" int uva_gemm4_tt_try(const void* A, const void* B, float* C, int M, int N, int K, long long lda,
                                long long ldb, long long ldc, float alpha, float beta, float* ws, long long ws_floats,
                                int* reduce, hipStream_t s);

template <typename TC>
static int launch_mfma(int ta, int tb, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                       long long ldb, long long ldc, int batch, const BatchStrides& bs, const EpiParams& ep,
                       const ConvParams& cp, float* ws, long long ws_floats, hipStream_t s) {
  // K-contiguous products with a bias-only epilogue: the persistent 4-wave kernel (gemm4.hip)
  if (ta == 0 && tb == 0 && batch == 1 && !ep.residual && !ep.aux && !ep.gate && ep.act == 0 &&
      ep.drop_thresh == 0 && ep.beta == 0.f && ep.res_grad == 0) {
    // (the 8-wave kernel first when a measurement switch routes plain products to it)
    int r = uva_gemm8w_try(sizeof(TC) == 2 ? UVA_DT_BF16 : UVA_DT_F32, A, B, C, M, N, K, lda, ldb, ldc, ep.bias,
                           ep.alpha, s);
    if (r < 0) return -r;
    if (r > 0) return 0;
    r = uva_gemm4_try(sizeof(TC) == 2 ? UVA_DT_BF16 : UVA_DT_F32, A, B, C, M, N, K, lda, ldb, ldc, ep.bias,
                      ep.alpha, s);
    if (r < 0) return -r;
    if (r > 0) return 0;
  }
  // the dW products (M- / N-contiguous operands, fp32 gradients): the same kernel over split-K items
  if (sizeof(TC) == 4 && ta == 1 && tb == 1 && batch == 1 && !ep.bias && !ep.residual && !ep.aux && !ep.gate &&
      ep.act == 0 && ep.drop_thresh == 0 && ep.res_grad == 0) {
    int red = 0;
    int r = uva_gemm8w_tt_try(A, B, (float*)C, M, N, K, lda, ldb, ldc, ep.alpha, ep.beta, ws, ws_floats, &red, s);
    if (r == 0) r = uva_gemm4_tt_try(A, B, (float*)C, M, N, K, lda, ldb, ldc, ep.alpha, ep.beta, ws, ws_floats, &red, s);
    if (r < 0) return -r;
    if (r > 0) {
      if (red > 0) {
        launch_splitk_reduce<TC>(ws, red, C, M, N, ldc, ep, s);
        UVA_LAUNCH_CHECK();
      }
      return 0;
    }
  }
  {
    int r = launch_8ph<TC>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, ws, ws_floats, s);
    if (r < 0) return -r;
    if (r > 0) return 0;
  }
  const int nblk = ((M + MB_M - 1) / MB_M) * ((N + MB_N - 1) / MB_N);
  // split-K when the output tiling cannot fill the chip (dW GEMMs: few tiles, K = tokens)
  int splits = 1;
  // K steps (x MB_K) per split, at least: 2 for the long-K training products; 4 for few-row GEMMs
  // (M <= 1024: the inference sampler's 1024x1024 layers, 41 -> 34 ms per 100-step loop at B=32)
  const int minks = M <= 1024 ? 4 : 2;
  if (batch == 1 && ws && nblk < 256 && K >= 2 * minks * MB_K) {
    splits = (512 + nblk - 1) / nblk;
    int kmax = K / (minks * MB_K);
    if (splits > kmax) splits = kmax;
    // skinny outputs (the z_proj / DiffLoss input_proj dW, [768 | 1024] x 16 over K = tokens): the
    // few 128x128 tiles need many more K slices to fill the chip (16 slices: 96 workgroups, 96 us for
    // 100 MB of dY; the partial slabs stay small)
    const int scap = (N <= 64 || M <= 64) ? 128 : 16;
    if (splits > scap) splits = scap;
    while (splits > 1 && (long long)splits * M * N > ws_floats) --splits;
  }
  int kps = K;
  if (splits > 1) {
    kps = ((K + splits - 1) / splits + MB_K - 1) / MB_K * MB_K;
    splits = (K + kps - 1) / kps;
  }
  float* part = splits > 1 ? ws : nullptr;
  dim3 grid(nblk, splits, batch);
  // LDS-DMA needs 16-B aligned sources for every lane: K-contiguous lds/ld multiples of 8 (checked by
  // the dispatcher) -- and no register-side prologue (GN apply) on the A operand
  const bool v2 = !(ta == 2 && cp.gn_scale);
  if (v2) {
    size_t lds2 = EPI_LDS_BYTES;  // >= 4 x 8192 bf16 staging images
    static bool attr2 = false;
    if (!attr2) {
      hipFuncSetAttribute((const void*)gemm_mfma_v2<0, 0, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      hipFuncSetAttribute((const void*)gemm_mfma_v2<0, 1, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      hipFuncSetAttribute((const void*)gemm_mfma_v2<1, 0, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      hipFuncSetAttribute((const void*)gemm_mfma_v2<1, 1, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      hipFuncSetAttribute((const void*)gemm_mfma_v2<2, 0, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
      attr2 = true;
    }
#define GV(a, b)                                                                                        \
  gemm_mfma_v2<a, b, TC><<<grid, 256, lds2, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, lda, ldb, ldc, \
                                                 bs, ep, cp, part, kps)
    if (ta == 2 && tb == 0) GV(2, 0);
    else if (ta == 0 && tb == 0) GV(0, 0);
    else if (ta == 0 && tb == 1) GV(0, 1);
    else if (ta == 1 && tb == 0) GV(1, 0);
    else if (ta == 1 && tb == 1) GV(1, 1);
    else return (int)hipErrorInvalidValue;
#undef GV
    UVA_LAUNCH_CHECK();
  } else {
  size_t lds = 2 * sizeof(bf16) * ((ta == 1 ? STAGE_M_ELEMS : STAGE_K_ELEMS) + (tb == 1 ? STAGE_M_ELEMS : STAGE_K_ELEMS));
  if (lds < EPI_LDS_BYTES) lds = EPI_LDS_BYTES;
#define GM(a, b)                                                                                          \
  do {                                                                                                    \
    static bool attr = false;                                                                             \
    if (!attr) {                                                                                          \
      hipFuncSetAttribute((const void*)gemm_mfma_bf16<a, b, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                          (int)lds);                                                                      \
      attr = true;                                                                                        \
    }                                                                                                     \
    gemm_mfma_bf16<a, b, TC><<<grid, 256, lds, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, lda, ldb, \
                                                    ldc, bs, ep, cp, part, kps);                          \
  } while (0)
  if (ta == 2 && tb == 0) GM(2, 0);
  else if (ta == 0 && tb == 0) GM(0, 0);
  else if (ta == 0 && tb == 1) GM(0, 1);
  else if (ta == 1 && tb == 0) GM(1, 0);
  else if (ta == 1 && tb == 1) GM(1, 1);
  else return (int)hipErrorInvalidValue;
#undef GM
  UVA_LAUNCH_CHECK();
  }
  if (part) {
    launch_splitk_reduce<TC>(part, splits, C, M, N, ldc, ep, s);
    UVA_LAUNCH_CHECK();
  }
  return 0;
}

static EpiParams make_epi(const float* bias, const void* residual, long long ldr, long long sRo, long long sRi,
                          void* aux, int act, float alpha, float beta, float drop_p, unsigned long long drop_seed) {
  EpiParams ep{};
  ep.bias = bias;
  ep.residual = residual;
  ep.aux = aux;
  ep.act = act;
  if (act >= 16) {  // activation backward: no forward activation, residual = pre-activation
    ep.res_grad = act - 16;
    ep.act = 0;
  }
  ep.alpha = alpha;
  ep.beta = beta;
  uva_drop_params(drop_p, &ep.drop_thresh, &ep.drop_scale);
  ep.drop_seed = drop_seed;
  ep.ldr = ldr;
  ep.sRo = sRo;
  ep.sRi = sRi;
  return ep;
}

static int gemm_dispatch(int in_dtype, int out_dtype, int ta, int tb, const void* A, const void* B, void* C, int M,
                         int N, int K, long long lda, long long ldb, long long ldc, int batch, const BatchStrides& bs,
                         const EpiParams& ep, const ConvParams& cp, int force_generic, float* ws, long long ws_floats,
                         hipStream_t stream) {
  if (in_dtype == UVA_DT_BF16) {
    // MFMA path needs 16-B chunks: K-contiguous dims and M/N-contiguous dims multiple of 8, aligned lds
    bool ok = !force_generic && (K % 8 == 0) && (((uintptr_t)A | (uintptr_t)B) % 16 == 0) &&
              (bs.sAo % 8 == 0) && (bs.sAi % 8 == 0) && (bs.sBo % 8 == 0) && (bs.sBi % 8 == 0) && (ldb % 8 == 0) &&
              (!tb || N % 8 == 0);
    if (ta == 2) ok = ok && (cp.Ci % 8 == 0);
    else ok = ok && (lda % 8 == 0) && (!ta || M % 8 == 0);
    if (ok) {
      if (out_dtype == UVA_DT_BF16)
        return launch_mfma<bf16>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, ws, ws_floats, stream);
      return launch_mfma<float>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, ws, ws_floats, stream);
    }
    if (out_dtype == UVA_DT_BF16)
      return launch_generic<bf16, bf16>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream, ws,
                                        ws_floats);
    return launch_generic<bf16, float>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream, ws,
                                       ws_floats);
  }
  if (out_dtype == UVA_DT_F32)
    return launch_generic<float, float>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream, ws,
                                        ws_floats);
  return launch_generic<float, bf16>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream, ws,
                                     ws_floats);
}

extern "C" int uva_gemm(int in_dtype, int out_dtype, int ta, int tb, const void* A, const void* B, void* C, int M,
                        int N, int K, long long lda, long long ldb, long long ldc, int batch, int batch_inner,
                        long long sAo, long long sAi, long long sBo, long long sBi, long long sCo, long long sCi,
                        const float* bias, const void* residual, long long ldr, long long sRo, long long sRi,
                        void* aux, int act, float alpha, float beta, float drop_p, unsigned long long drop_seed,
                        int res_dtype, const void* gate, long long ldg, int gate_dtype, int force_generic,
                        float* workspace, long long ws_floats, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0 || K <= 0) return 0;
  if (ta == 2) return (int)hipErrorInvalidValue;  // conv view only through uva_conv2d
  BatchStrides bs{sAo, sAi, sBo, sBi, sCo, sCi, batch_inner > 0 ? batch_inner : 1};
  EpiParams ep = make_epi(bias, residual, ldr, sRo, sRi, aux, act, alpha, beta, drop_p, drop_seed);
  ep.res_dt = res_dtype;
  ep.gate = gate;
  ep.ldg = ldg;
  ep.gate_dt = gate_dtype;
  ConvParams cp{};
  return gemm_dispatch(in_dtype, out_dtype, ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, force_generic,
                       workspace, ws_floats, stream);
}

extern "C" long long uva_gemm_plan(int in_dtype, int ta, int tb, int M, int N, int K, int batch, int gn_prologue,
                                   long long ws_floats) {
  // kernel | BN << 4 | splits << 16   (kernel: 0 generic VALU, 1 mfma register-staged, 2 mfma LDS-DMA 128x128,
  // 3 mfma 8-phase 256-row); assumes 16-B aligned operands
  if (in_dtype != UVA_DT_BF16 || K % 8 != 0 || (tb == 1 && N % 8 != 0) || (ta == 1 && M % 8 != 0)) return 0;
  const Plan8 p = plan_8ph(ta, M, N, K, batch, gn_prologue != 0, ws_floats > 0, ws_floats);
  if (p.bn) return 3 | ((long long)p.bn << 4) | ((long long)p.splits << 16);
  return (ta == 2 && gn_prologue) ? 1 : 2;
}

extern "C" int uva_conv3x3_halo_bn(int Nimg, int H, int W, int Ci, int Co);
extern "C" int uva_conv3x3_halo(const void* in, const void* w, void* out, const float* bias, const void* residual,
                                int Nimg, int H, int W, int Ci, int Co, const float* gn_scale, const float* gn_shift,
                                int gn_silu, float* gn_part, hipStream_t stream);

extern "C" int uva_conv3x3s2_ok(int Nimg, int Hin, int Win, int Ci, int Co);
extern "C" int uva_conv3x3s2_halo(const void* in, const void* w, void* out, const float* bias, int Nimg, int Hin,
                                  int Win, int Ci, int Co, float* gn_part, hipStream_t stream);
extern "C" int uva_conv_in8(const void* in, const void* w, void* out, const float* bias, int Nimg, int H, int W,
                            float* gn_part, hipStream_t stream);

extern "C" int uva_conv2d(int dtype, const void* in, const void* w, void* out, const float* bias, const void* residual,
                          int Nimg, int Hin, int Win, int Ci, int Co, int ks, int stride, int pad_t, int pad_l,
                          int Hout, int Wout, const float* gn_scale, const float* gn_shift, int gn_silu, int act,
                          float* gn_part, int force_generic, hipStream_t stream) {
  const int M = Nimg * Hout * Wout, K = ks * ks * Ci;
  if (M <= 0) return 0;
  // 3x3 / s1 / p1 with 16x16-tileable maps and 64 | Ci, 128 | Co: direct halo-tile kernel (conv.hip)
  if (!force_generic && dtype == UVA_DT_BF16 && ks == 3 && stride == 1 && pad_t == 1 && pad_l == 1 &&
      Hout == Hin && Wout == Win && act == ACT_NONE && uva_conv3x3_halo_bn(Nimg, Hin, Win, Ci, Co) > 0)
    return uva_conv3x3_halo(in, w, out, bias, residual, Nimg, Hin, Win, Ci, Co, gn_scale, gn_shift, gn_silu, gn_part,
                            stream);
  // Downsample: F.pad(0, 1, 0, 1) + 3x3 / s2 / p0 with 8x16-tileable outputs: halo-tile kernel (conv.hip)
  if (!force_generic && dtype == UVA_DT_BF16 && ks == 3 && stride == 2 && pad_t == 0 && pad_l == 0 &&
      Hout * 2 == Hin && Wout * 2 == Win && act == ACT_NONE && !residual && !gn_scale &&
      uva_conv3x3s2_ok(Nimg, Hin, Win, Ci, Co))
    return uva_conv3x3s2_halo(in, w, out, bias, Nimg, Hin, Win, Ci, Co, gn_part, stream);
  // the 8-channel (padded RGB) input conv: store-bound special form (conv.hip)
  if (!force_generic && dtype == UVA_DT_BF16 && ks == 3 && stride == 1 && pad_t == 1 && pad_l == 1 &&
      Hout == Hin && Wout == Win && act == ACT_NONE && Ci == 8 && Co == 128 && !residual && !gn_scale &&
      Hin % 16 == 0 && Win % 16 == 0)
    return uva_conv_in8(in, w, out, bias, Nimg, Hin, Win, gn_part, stream);
  BatchStrides bs{0, 0, 0, 0, 0, 0, 1};
  EpiParams ep = make_epi(bias, residual, Co, 0, 0, nullptr, act, 1.0f, 0.0f, 0.0f, 0);
  ep.res_dt = dtype;
  ConvParams cp{Hin, Win, Ci, Hout, Wout, ks, stride, pad_t, pad_l, gn_scale, gn_shift, gn_silu, gn_part};
  if (gn_part) {
    // fused GN statistics need whole 128-row tiles inside one image and 32 | Co
    if ((Hout * Wout) % MB_M != 0 || Co % 32 != 0 || dtype != UVA_DT_BF16) return (int)hipErrorInvalidValue;
  }
  return gemm_dispatch(dtype, dtype, 2, 0, in, w, out, M, Co, K, 0, K, Co, 1, bs, ep, cp, force_generic, nullptr, 0,
                       stream);
}
