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
    v += ep.res_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.residual)[ri] : ((const float*)ep.residual)[ri];
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

template <typename TI, typename TC, int TA, int TB>
__global__ __launch_bounds__(256) void gemm_generic(const TI* __restrict__ A, const TI* __restrict__ B,
                                                    TC* __restrict__ C, int M, int N, int K, long long lda,
                                                    long long ldb, long long ldc, BatchStrides bs, EpiParams ep,
                                                    ConvParams cp) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int z = blockIdx.z, zo = z / bs.binner, zi = z % bs.binner;
  A += zo * bs.sAo + zi * bs.sAi;
  B += zo * bs.sBo + zi * bs.sBi;
  const long long coff = zo * bs.sCo + zi * bs.sCi;
  const long long roff = zo * ep.sRo + zi * ep.sRi;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int e = t + i * 256;  // 0..1023 over a 64x16 tile
      int mm, kk;
      if (TA != 1) { mm = e >> 4; kk = e & 15; } else { kk = e >> 6; mm = e & 63; }
      int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < M && gk < K) {
        if (TA == 2) v = conv_gather(A, cp, gm, gk);
        else v = to_f32(TA == 0 ? A[(long long)gm * lda + gk] : A[(long long)gk * lda + gm]);
      }
      As[kk][mm] = v;
      int nn;
      if (TB == 0) { nn = e >> 4; kk = e & 15; } else { kk = e >> 6; nn = e & 63; }
      int gn = n0 + nn;
      gk = k0 + kk;
      v = 0.f;
      if (gn < N && gk < K) v = to_f32(TB == 0 ? B[(long long)gn * ldb + gk] : B[(long long)gk * ldb + gn]);
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
      if (r < M && c < N)
        epi_store<TC>(C, ldc, coff, ep, roff, r, c, N, (long long)z * M * N + (long long)r * N + c, acc[i][j]);
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

// Epilogue staged through LDS: the 128x128 fp32 accumulator tile is written to LDS with
// compile-time indices (no register-array indexing -> no scratch), then every thread finishes
// 8 consecutive columns x 8 rows with 16-B vector loads/stores (coalesced, issue-light).
#define EPI_TP 132  // fp32 row pitch of the staged tile (+4 floats: conflict-free column writes)
#define EPI_LDS_BYTES (128 * EPI_TP * 4 + 4 * 16 * 8 * 2 * 4)

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
      float prev[8];
      if (ep.beta != 0.f) {
        if constexpr (sizeof(TC) == 2) {
          bf16x8 pv = *(const bf16x8*)(C + cbase);
#pragma unroll
          for (int e = 0; e < 8; ++e) prev[e] = (float)pv[e];
        } else {
          float4 p0 = *(const float4*)(C + cbase), p1 = *(const float4*)(C + cbase + 4);
          prev[0] = p0.x; prev[1] = p0.y; prev[2] = p0.z; prev[3] = p0.w;
          prev[4] = p1.x; prev[5] = p1.y; prev[6] = p1.z; prev[7] = p1.w;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = col0 + e;
        float x = ep.alpha * v[e];
        if (ep.bias) x += ep.bias[col];
        if (ep.aux) ((TC*)ep.aux)[cbase + e] = from_f32<TC>(x);
        x = apply_act(ep.act, x);
        if (ep.drop_thresh)
          x = dropout_keep(ep.drop_seed, (uint64_t)((long long)z * M * N + (long long)row * N + col), ep.drop_thresh)
                  ? x * ep.drop_scale : 0.f;
        if (ep.gate) {
          long long gi = (long long)row * ep.ldg + col;
          x *= ep.gate_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.gate)[gi] : ((const float*)ep.gate)[gi];
        }
        if (ep.residual) {
          long long ri = roff + (long long)row * ep.ldr + col;
          x += ep.res_dt == UVA_DT_BF16 ? (float)((const bf16*)ep.residual)[ri] : ((const float*)ep.residual)[ri];
        }
        if (ep.beta != 0.f) x += ep.beta * prev[e];
        o[e] = x;
      }
      if constexpr (sizeof(TC) == 2) {
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = (bf16)o[e];
        *(bf16x8*)(C + cbase) = ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (float)ov[e];
      } else {
        *(float4*)(C + cbase) = make_float4(o[0], o[1], o[2], o[3]);
        *(float4*)(C + cbase + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
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

// =====================================================================================
// host launchers
// =====================================================================================
template <typename TI, typename TC>
static int launch_generic(int ta, int tb, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                          long long ldb, long long ldc, int batch, const BatchStrides& bs, const EpiParams& ep,
                          const ConvParams& cp, hipStream_t s) {
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

template <typename TC>
static int launch_mfma(int ta, int tb, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                       long long ldb, long long ldc, int batch, const BatchStrides& bs, const EpiParams& ep,
                       const ConvParams& cp, float* ws, long long ws_floats, hipStream_t s) {
  const int nblk = ((M + MB_M - 1) / MB_M) * ((N + MB_N - 1) / MB_N);
  // split-K when the output tiling cannot fill the chip (dW GEMMs: few tiles, K = tokens)
  int splits = 1;
  if (batch == 1 && ws && nblk < 256 && K >= 4 * MB_K) {
    splits = (512 + nblk - 1) / nblk;
    int kmax = K / (2 * MB_K);
    if (splits > kmax) splits = kmax;
    if (splits > 16) splits = 16;
    while (splits > 1 && (long long)splits * M * N > ws_floats) --splits;
  }
  int kps = K;
  if (splits > 1) {
    kps = ((K + splits - 1) / splits + MB_K - 1) / MB_K * MB_K;
    splits = (K + kps - 1) / kps;
  }
  float* part = splits > 1 ? ws : nullptr;
  dim3 grid(nblk, splits, batch);
  static int use_v1 = -1;
  if (use_v1 < 0) {
    const char* e = getenv("UVA_GEMM_V1");
    use_v1 = (e && e[0] == '1') ? 1 : 0;
  }
  // LDS-DMA needs 16-B aligned sources for every lane: K-contiguous lds/ld multiples of 8 (checked by
  // the dispatcher) -- and no register-side prologue (GN apply) on the A operand
  const bool v2 = !use_v1 && !(ta == 2 && cp.gn_scale);
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
    long long n = (long long)M * N;
    long long blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    splitk_reduce<TC><<<dim3((unsigned)blocks), 256, 0, s>>>(part, splits, (TC*)C, M, N, ldc, ep);
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
  ep.alpha = alpha;
  ep.beta = beta;
  ep.drop_thresh = drop_p > 0.f ? (uint32_t)fminf(drop_p * 4294967296.0f, 4294967295.0f) : 0u;
  ep.drop_scale = drop_p > 0.f ? 1.0f / (1.0f - drop_p) : 1.0f;
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
      return launch_generic<bf16, bf16>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream);
    return launch_generic<bf16, float>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream);
  }
  if (out_dtype == UVA_DT_F32)
    return launch_generic<float, float>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream);
  return launch_generic<float, bf16>(ta, tb, A, B, C, M, N, K, lda, ldb, ldc, batch, bs, ep, cp, stream);
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

extern "C" int uva_conv2d(int dtype, const void* in, const void* w, void* out, const float* bias, const void* residual,
                          int Nimg, int Hin, int Win, int Ci, int Co, int ks, int stride, int pad_t, int pad_l,
                          int Hout, int Wout, const float* gn_scale, const float* gn_shift, int gn_silu, int act,
                          float* gn_part, int force_generic, hipStream_t stream) {
  const int M = Nimg * Hout * Wout, K = ks * ks * Ci;
  if (M <= 0) return 0;
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
