// Few-row fused linear for the action sampler's per-step res blocks (inference, bf16).
//
// Reference per step (diffusion_loss.py:142-189, SimpleMLPAdaLN.forward :261-283):
//   h = modulate(LN(x) [* w + b], shift, scale)      (ResBlock.in_ln / FinalLayer.norm_final)
//   a = SiLU(h W1^T + b1);  x' = x + gate * (a W2^T + b2)
// Rows R = B*16 are few (16..1024), so the general 128x128 / 256x256 tiles leave the chip idle
// and split K.  Here one workgroup owns a 32-row x 64-column output tile over the FULL K
// (<= 1024): each wave preloads its 16 columns of W (16 x K bf16 = 128 VGPRs per lane) before
// anything else, so the weight stream from L2/HBM overlaps the A staging; the 32 x K A tile is
// staged once in LDS -- for the LN variant as the modulated LayerNorm of the fp32 residual rows
// (row statistics by wave shuffles, so the separate LN kernel disappears).  MFMA
// v_mfma_f32_16x16x32_bf16, fp32 accumulation; epilogue bias [+SiLU] [gate*v + residual].
#include "common.h"

namespace {
constexpr int SL_BM = 32, SL_BN = 64, SL_KMAX = 1024, SL_LDA = SL_KMAX + 8;  // K in {256, 512, 1024}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// NARROW = false: 4 waves x 16 columns, every wave over the full K (a 32 x 64 tile per workgroup).
// NARROW = true (few rows: the 32 x 64 grid would leave most CUs idle, e.g. 16 workgroups for
// R = 16, N = 1024): a 32 x 16 tile per workgroup, its 8 waves split K (each streams K/8 x 16 of
// W), partial tiles summed through LDS in wave order (deterministic) -- 4x the workgroups, 1/8 of
// each wave's weight stream.
template <int LN, int ACT, int GATE, typename TC, int KS, bool NARROW>
__global__ __launch_bounds__(NARROW ? 512 : 256) void sampler_linear_kernel(
    const void* __restrict__ A, long long lda, const float* __restrict__ lnw, const float* __restrict__ lnb,
    const bf16* __restrict__ shift, const bf16* __restrict__ scale, long long ldm, float eps,
    const bf16* __restrict__ W, const float* __restrict__ bias, const bf16* __restrict__ gate, long long ldg,
    const float* __restrict__ res, long long ldr, TC* __restrict__ out, long long ldo, int R, int N) {
  // K = 32 * KS is a compile-time constant: every load / MFMA below sits in one straight-line
  // block, so the 32 weight loads issue back to back instead of one memory latency each
  constexpr int K = 32 * KS;
  constexpr int NW = NARROW ? 8 : 4, NT = NW * 64;
  constexpr int KSW = NARROW ? KS / NW : KS;  // k-steps of 32 per wave
  static_assert(!NARROW || KS % NW == 0, "K slices of whole k-steps");
  __shared__ bf16 sA[SL_BM * SL_LDA];
  __shared__ f32x4 sRed[NARROW ? NW * 2 * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * SL_BM;
  const int n0 = NARROW ? blockIdx.y * 16 : blockIdx.y * SL_BN + wave * 16;
  const int kw0 = NARROW ? wave * KSW * 32 : 0;  // this wave's K slice
  // 1. this wave's weight fragments: column n0 + (lane & 15), k = kw0 + 32 s + 8 (lane >> 4) .. +8
  //    (columns >= N read row 0: their accumulators are never stored)
  bf16x8 bw[KSW];
  {
    const int n = n0 + (lane & 15);
    const bf16* wp = W + (long long)(n < N ? n : 0) * K + kw0 + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < KSW; ++s) bw[s] = *(const bf16x8*)(wp + 32 * s);
  }
  // 2. A tile -> LDS (bf16), rows >= R zero
  if (LN) {
    // two rows per wave iteration (independent load/reduce chains overlap); a lane owns 4
    // consecutive columns per 256-column slice, so every operand load is a vector load
    const float* X = (const float*)A;
    for (int r0 = 2 * wave; r0 < SL_BM; r0 += 2 * NW) {
      float4 v[2][K / 256];
      float mean[2], rstd[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int m = m0 + r0 + u;
        const float* xr = X + (long long)(m < R ? m : 0) * lda;
#pragma unroll
        for (int i = 0; i < K / 256; ++i) v[u][i] = *(const float4*)(xr + i * 256 + lane * 4);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < K / 256; ++i) s += (v[u][i].x + v[u][i].y) + (v[u][i].z + v[u][i].w);
        mean[u] = wave_sum(s) / (float)K;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < K / 256; ++i) {
          const float a = v[u][i].x - mean[u], b = v[u][i].y - mean[u], c = v[u][i].z - mean[u],
                      d = v[u][i].w - mean[u];
          q += (a * a + b * b) + (c * c + d * d);
        }
        rstd[u] = rsqrtf(wave_sum(q) / (float)K + eps);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int m = m0 + r0 + u;
        bf16* dst = sA + (r0 + u) * SL_LDA;
        const long long mo = (long long)(m < R ? m : 0) * ldm;
#pragma unroll
        for (int i = 0; i < K / 256; ++i) {
          const int k = i * 256 + lane * 4;
          bf16x4 o = bf16x4{};
          if (m < R) {
            const bf16x4 sh = *(const bf16x4*)(shift + mo + k);
            const bf16x4 sc = *(const bf16x4*)(scale + mo + k);
            float4 w4 = make_float4(1.f, 1.f, 1.f, 1.f), b4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (lnw) {
              w4 = *(const float4*)(lnw + k);
              b4 = *(const float4*)(lnb + k);
            }
            const float e[4] = {v[u][i].x, v[u][i].y, v[u][i].z, v[u][i].w};
            const float ww[4] = {w4.x, w4.y, w4.z, w4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float h = (e[j] - mean[u]) * rstd[u];
              if (lnw) h = h * ww[j] + bb[j];
              o[j] = (bf16)(h * (1.0f + (float)sc[j]) + (float)sh[j]);
            }
          }
          *(bf16x4*)(dst + k) = o;
        }
      }
    }
  } else {
    const bf16* Ab = (const bf16*)A;
    const int kv = K / 8;
    for (int i = tid; i < SL_BM * kv; i += NT) {
      const int r = i / kv, k = (i % kv) * 8;
      const int m = m0 + r;
      bf16x8 v = m < R ? *(const bf16x8*)(Ab + (long long)m * lda + k) : bf16x8{};
      *(bf16x8*)(sA + r * SL_LDA + k) = v;
    }
  }
  __syncthreads();
  // 3. 2 (rows) x 1 (cols) 16x16 tiles per wave over the full K
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const bf16* a0 = sA + (lane & 15) * SL_LDA + kw0 + 8 * (lane >> 4);
  const bf16* a1 = a0 + 16 * SL_LDA;
#pragma unroll
  for (int s = 0; s < KSW; ++s) {
    const bf16x8 fa0 = *(const bf16x8*)(a0 + 32 * s);
    const bf16x8 fa1 = *(const bf16x8*)(a1 + 32 * s);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0, bw[s], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1, bw[s], acc1, 0, 0, 0);
  }
  if constexpr (NARROW) {
    // K-slice partials -> LDS; wave 0 sums them in wave order and runs the epilogue
    sRed[(wave * 2 + 0) * 64 + lane] = acc0;
    sRed[(wave * 2 + 1) * 64 + lane] = acc1;
    __syncthreads();
    if (wave != 0) return;
    acc0 = sRed[lane];
    acc1 = sRed[64 + lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      acc0 += sRed[(w * 2 + 0) * 64 + lane];
      acc1 += sRed[(w * 2 + 1) * 64 + lane];
    }
  }
  // 4. epilogue: lane holds rows 4 (lane >> 4) + j (+16), column lane & 15
  const int n = n0 + (lane & 15);
  if (n >= N) return;
  const float bn = bias ? bias[n] : 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x4 acc = t ? acc1 : acc0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + 16 * t + 4 * (lane >> 4) + j;
      if (m >= R) continue;
      float v = acc[j] + bn;
      if (ACT == ACT_SILU) v = silu(v);
      if (GATE) v = res[(long long)m * ldr + n] + (float)gate[(long long)m * ldg + n] * v;
      out[(long long)m * ldo + n] = (TC)v;
    }
  }
}
}  // namespace

extern "C" int uva_sampler_linear(int ln, const void* A, long long lda, const float* lnw, const float* lnb,
                                  const void* shift, const void* scale, long long ldm, float eps, const void* W,
                                  const float* bias, int act, const void* gate, long long ldg, const float* res,
                                  long long ldr, int odt, void* out, long long ldo, int R, int N, int K,
                                  hipStream_t s) {
  if (R <= 0 || N <= 0 || (K != 1024 && K != 512 && K != 256) || (ln && (lda % 4 || ldm % 4)) || (!ln && lda % 8)) {
    return (int)hipErrorInvalidValue;
  }
  if ((gate == nullptr) != (res == nullptr) || (ln && (!shift || !scale)) || (act != 0 && act != ACT_SILU)) {
    return (int)hipErrorInvalidValue;
  }
  // the 32 x 64 tile grid, or (under 64 workgroups) the narrow 32 x 16 tiles with K split over 8 waves
  const unsigned mb = (unsigned)((R + SL_BM - 1) / SL_BM);
  const bool narrow = (long long)mb * ((N + SL_BN - 1) / SL_BN) < 64;
  const dim3 grid(mb, (unsigned)(narrow ? (N + 15) / 16 : (N + SL_BN - 1) / SL_BN));
#define SLKK(L, AC, G, T, KSV)                                                                                    \
  do {                                                                                                            \
    if (narrow)                                                                                                   \
      sampler_linear_kernel<L, AC, G, T, KSV, true><<<grid, 512, 0, s>>>(                                         \
          A, lda, lnw, lnb, (const bf16*)shift, (const bf16*)scale, ldm, eps, (const bf16*)W, bias,                \
          (const bf16*)gate, ldg, res, ldr, (T*)out, ldo, R, N);                                                  \
    else                                                                                                          \
      sampler_linear_kernel<L, AC, G, T, KSV, false><<<grid, 256, 0, s>>>(                                        \
          A, lda, lnw, lnb, (const bf16*)shift, (const bf16*)scale, ldm, eps, (const bf16*)W, bias,                \
          (const bf16*)gate, ldg, res, ldr, (T*)out, ldo, R, N);                                                  \
  } while (0)
#define SLK(L, AC, G, T)                                                                                  \
  do {                                                                                                    \
    if (K == 1024) SLKK(L, AC, G, T, 32);                                                                 \
    else if (K == 512) SLKK(L, AC, G, T, 16);                                                             \
    else SLKK(L, AC, G, T, 8);                                                                            \
  } while (0)
  const bool g = gate != nullptr, f32 = odt == UVA_DT_F32;
  if (ln && act == ACT_SILU && !g && !f32) SLK(1, ACT_SILU, 0, bf16);
  else if (ln && act == 0 && !g && f32) SLK(1, 0, 0, float);
  else if (!ln && act == 0 && g && f32) SLK(0, 0, 1, float);
  else if (!ln && act == ACT_SILU && !g && !f32) SLK(0, ACT_SILU, 0, bf16);
  else return (int)hipErrorInvalidValue;
#undef SLK
#undef SLKK
  UVA_LAUNCH_CHECK();
  return 0;
}
