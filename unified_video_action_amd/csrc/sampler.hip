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

// =====================================================================================
// Persistent sampler for few rows (R <= 16: action sampling at B = 1).  The whole S-step reverse
// diffusion loop -- input_proj, depth x (adaLN-LN + fc1 + SiLU, fc2 + gate + residual), final
// adaLN-LN + linear, p_sample (diffusion_loss.py:142-189, 261-283; gaussian_diffusion.py:395-440)
// -- runs in ONE launch instead of ~15 launches per step (each 4-9 us of latency chain at 16 rows).
//
// 64 workgroups (one per CU: > 80 KB of LDS), workgroup g owns output columns [16 g, 16 g + 16) of
// every fc1 / fc2 (its weight slices, 2 x 32 KB per block, stay L2-resident across the steps).  Per
// block the rows are exchanged twice through global memory: fc1 output a [16, W] bf16 and the
// residual stream h [16, W] fp32 (ping-pong).  What needs no exchange runs redundantly in every
// workgroup: input_proj (K = C <= 16: every workgroup forms the full h0 rows), the final layer
// (N = 2C <= 32) and the p_sample update, so each workgroup carries its own copy of x_t and the
// step boundary costs no hand-off: 2 x depth hand-offs per step.
//
// Hand-off (cdna_hip_programming.md Guideline 16, R1 with one counter per phase; MI355X_MICROARCH
// 'Hand-offs measured with sc1 loads', row 1): the ONE storing wave writes its slice with sc1
// (write-through) 16-B stores, drains vmcnt, then lane 0 adds 1 to the phase's counter (agent
// scope, relaxed); a consumer's wave 0 polls the counter with relaxed agent loads until it reaches
// 64 x (step + 1), the workgroup barrier releases the other waves, and EVERY load of exchanged
// bytes is an sc1 buffer load.  Counters and the give-up flag are zeroed by a memset node ahead of
// every launch; every spin is bounded (give-up flag, then every wait falls through).  (The tagged-
// granule form, Guideline 16 R2 -- payload and epoch in one 8-B granule, no drain, no counter --
// measured 8.4 vs 7.9 ms per 100-step loop on one box: the doubled bytes of every exchanged row
// cost more than the counter round trip it saves.)  Measured (B = 1, pusht joint, 100 steps): the
// loop 11.5 ms as a captured graph of ~15 launches per step -> 7.9 ms here; the per-block phases
// are bound by their latency chains (exchange loads, LDS round trips, the store drain), not by the
// hand-off (all waits removed: 7.75 ms).
// =====================================================================================
namespace {
constexpr int PS_W = 1024, PS_R = 16, PS_C = 16, PS_G = PS_W / 16, PS_LDA = PS_W + 8;
constexpr int PS_SC1 = 16;  // buffer-op aux: sc1
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;
typedef __attribute__((address_space(1))) unsigned gu32;  // shared words: global (never flat) accesses

// block weights stacked per kind (few base pointers: a per-block pointer array in the parameter
// struct held ~70 SGPRs live across the step loop and spilled)
struct PSParams {
  const bf16* w1;    // [depth, W, W]
  const float* b1;   // [depth, W]
  const bf16* w2;    // [depth, W, W]
  const float* b2;   // [depth, W]
  const float* lnw;  // [depth, W]
  const float* lnb;  // [depth, W]
  const bf16* win;    // [W, C]
  const float* bin;   // [W]
  const bf16* wf;     // [2C, W]
  const float* bfin;  // [2C]
  const bf16* mod;    // [S, R, ldmod]: block i shift | scale | gate at 3 W i, final shift | scale at 3 W depth
  long long ldmod;
  const float* coef;   // [S, 8] (PStepCoef order)
  const float* noise;  // [S, R, C]
  const float* x0;     // [R, C]
  float* x_out;        // [R, C]
  float* hx;           // [2, 16, W] exchange: residual stream
  bf16* ha;            // [16, W] exchange: fc1 output
  unsigned* cnt;       // [2 depth] arrival counters
  unsigned* err;       // give-up flag
  int R, C, depth, S, clip;
  float eps;
  int no_publish;  // test hook only (uva_sampler_persistent_test_hook): no phase is ever published
};

// wave sum by DPP (quad perms, row rotates) and two lane swaps: six VALU steps of a few cycles each,
// instead of six dependent ds_bpermute round trips through the LDS crossbar (__shfl_xor); the LN
// statistics of the row pass (two sums per row) sit on every phase's critical path
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ void ps_publish(unsigned* cnt, int no_publish) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the storing wave's sc1 stores have left
  if ((threadIdx.x & 63) == 0 && !no_publish)
    __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void ps_wait(unsigned* cnt, unsigned target, unsigned* err) {
  if (threadIdx.x < 64) {
    for (unsigned spins = 0;; ++spins) {
      if (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if ((spins & 255) == 255) {
        if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
        if (spins > (1u << 21)) {
          __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
}

template <int DEPTH>
__global__ __launch_bounds__(256, 1) void sampler_persistent_kernel(PSParams p) {
  extern __shared__ __attribute__((aligned(16))) char ps_smem[];
  bf16* sA = (bf16*)ps_smem;                                   // [16][PS_LDA] MFMA A tile
  f32x4* sPart = (f32x4*)(ps_smem + PS_R * PS_LDA * 2);        // [4 waves][2 tiles][64 lanes]
  float* sRes = (float*)(sPart + 4 * 2 * 64);                  // [16][16] block input, my columns
  float* sT = sRes + 256;                                      // [16][16] store transpose
  float* sOut = sT + 256;                                      // [16][32] final layer output
  float* sX = sOut + 512;                                      // [16][16] x_t
  float* sXn = sX + 256;                                       // [16][16] bf16(x_t) as float
  bf16* sWinT = (bf16*)(sXn + 256);                            // [C][W] input_proj weight, transposed
  const int tid = threadIdx.x, l = tid & 63, g = l >> 4, li = l & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int R = p.R, C = p.C, W = PS_W;
  constexpr int D = DEPTH;
  const int col0 = blockIdx.x * 16;
  const float invW = 1.0f / (float)W;
  const __amdgpu_buffer_rsrc_t rs_hx = __builtin_amdgcn_make_buffer_rsrc(p.hx, 0, 2 * PS_R * W * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_ha = __builtin_amdgcn_make_buffer_rsrc(p.ha, 0, PS_R * W * 2, 0x00020000);

  for (int i = tid; i < W * C; i += 256) sWinT[(i % C) * W + i / C] = p.win[i];
  {
    const int r = tid >> 4, c = tid & 15;
    const float x = (r < R && c < C) ? p.x0[r * C + c] : 0.f;
    sX[tid] = x;
    sXn[tid] = (float)(bf16)x;
  }
  float binr[4][4];  // input_proj bias of the row-pass columns i*256 + 4l + j
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 b = *(const float4*)(p.bin + i * 256 + 4 * l);
    binr[i][0] = b.x; binr[i][1] = b.y; binr[i][2] = b.z; binr[i][3] = b.w;
  }
  __syncthreads();

  // row pass: wave w owns rows 4w + u, lane l columns i*256 + 4l + j
  float h[4][4][4];

  auto load_h = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * w + u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (r < R)
          v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs_hx, (((buf * PS_R + r) * W) + i * 256 + 4 * l) * 4, 0, PS_SC1));
#pragma unroll
        for (int j = 0; j < 4; ++j) h[u][i][j] = v[j];
      }
    }
  };
  // modulation rows (shift / scale) and LN affine of the row pass, loaded BEFORE the hand-off wait
  // (they do not depend on the other workgroups)
  bf16x4 msh[4][4], msc[4][4];
  float4 mlw[4], mlb[4];
  auto ln_prefetch = [&](const float* lnw, const float* lnb, const bf16* shift, const bf16* scale)
      __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * w + u;
      const long long mo = (long long)(r < R ? r : 0) * p.ldmod;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        msh[u][i] = *(const bf16x4*)(shift + mo + i * 256 + 4 * l);
        msc[u][i] = *(const bf16x4*)(scale + mo + i * 256 + 4 * l);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mlw[i] = lnw ? *(const float4*)(lnw + i * 256 + 4 * l) : make_float4(1.f, 1.f, 1.f, 1.f);
      mlb[i] = lnb ? *(const float4*)(lnb + i * 256 + 4 * l) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // LayerNorm (+ affine) + adaLN modulate of the row pass -> sA (bf16)
  auto ln_mod = [&](bool affine) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * w + u;
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) s += (h[u][i][0] + h[u][i][1]) + (h[u][i][2] + h[u][i][3]);
      const float mean = wave_sum_dpp(s) * invW;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = h[u][i][j] - mean;
          q += d * d;
        }
      const float rstd = rsqrtf(wave_sum_dpp(q) * invW + p.eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = i * 256 + 4 * l;
        const bf16x4 sh = msh[u][i], sc = msc[u][i];
        const float ww[4] = {mlw[i].x, mlw[i].y, mlw[i].z, mlw[i].w}, bb[4] = {mlb[i].x, mlb[i].y, mlb[i].z, mlb[i].w};
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float y = (h[u][i][j] - mean) * rstd;
          if (affine) y = y * ww[j] + bb[j];
          o[j] = r < R ? (bf16)(y * (1.0f + (float)sc[j]) + (float)sh[j]) : (bf16)0.f;
        }
        *(bf16x4*)(sA + r * PS_LDA + k) = o;
      }
    }
  };
  // the block input's fp32 values at my 16 columns (fc2's residual) -> sRes: from the exchange buffer
  // (wave 0, one 16-B sc1 load per lane), or for block 0 from x_net (every thread, K = C)
  auto res_from_hx = [&](int buf) __attribute__((always_inline)) {
    if (w == 0) {
      const int row = l >> 2, c4 = (l & 3) * 4;
      u32x4v v = {0u, 0u, 0u, 0u};
      if (row < R) v = __builtin_amdgcn_raw_buffer_load_b128(rs_hx, ((buf * PS_R + row) * W + col0 + c4) * 4, 0, PS_SC1);
      *(u32x4v*)(sRes + row * 16 + c4) = v;
    }
  };
  auto res_from_input = [&]() __attribute__((always_inline)) {
    const int r = tid >> 4, c = tid & 15;
    float a = p.bin[col0 + c];
    for (int cc = 0; cc < C; ++cc) a = fmaf(sXn[r * 16 + cc], (float)sWinT[cc * W + col0 + c], a);
    sRes[tid] = r < R ? a : 0.f;
  };
  // this wave's K quarter [256 w, 256 w + 256) of sA x the weight fragments -> sPart[w][t]
  auto mma = [&](const bf16x8 (&bw)[8], int t) __attribute__((always_inline)) {
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
    const bf16* ap = sA + li * PS_LDA + 256 * w + 8 * g;
#pragma unroll
    for (int s = 0; s < 8; s += 2) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(ap + 32 * s), bw[s], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)(ap + 32 * s + 32), bw[s + 1], a1, 0, 0, 0);
    }
    sPart[(w * 2 + t) * 64 + l] = a0 + a1;
  };
  auto wload = [&](const bf16* Wl, int n, int N, bf16x8 (&bw)[8]) __attribute__((always_inline)) {
    const bf16* wp = Wl + (long long)(n < N ? n : 0) * W + 256 * w + 8 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) bw[s] = *(const bf16x8*)(wp + 32 * s);
  };
  // wave 0: the four K-quarter partials of tile t summed in wave order
  auto reduce = [&](int t) __attribute__((always_inline)) {
    f32x4 acc = sPart[t * 64 + l];
#pragma unroll
    for (int v = 1; v < 4; ++v) acc += sPart[(v * 2 + t) * 64 + l];
    return acc;
  };

  // every phase's operands that do not depend on other workgroups (weight fragments, modulation rows,
  // LN affine) are loaded one phase AHEAD: bw holds the next phase's fragments, bw2 the final layer's
  // second column tile; msh / msc / mlw / mlb the next fc1 / final LN's rows
  bf16x8 bw[8], bw2[8];
  wload(p.w1, col0 + li, W, bw);
  ln_prefetch(p.lnw, p.lnb, p.mod, p.mod + W);
  for (int k = 0; k < p.S; ++k) {
    const unsigned target = (unsigned)PS_G * (unsigned)(k + 1);
    const bf16* modk = p.mod + (long long)k * R * p.ldmod;
    // input_proj, every row and column in every workgroup: h0 = x_net Win^T + bin (K = C)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = 4 * w + u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a[4] = {binr[i][0], binr[i][1], binr[i][2], binr[i][3]};
        for (int c = 0; c < C; ++c) {
          const float xv = sXn[r * 16 + c];
          const bf16x4 wv = *(const bf16x4*)(sWinT + c * W + i * 256 + 4 * l);
#pragma unroll
          for (int j = 0; j < 4; ++j) a[j] = fmaf(xv, (float)wv[j], a[j]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) h[u][i][j] = r < R ? a[j] : 0.f;
      }
    }
#pragma unroll 1
    for (int blk = 0; blk < D; ++blk) {
      const bf16* mb = modk + 3LL * W * blk;
      // ---- fc1: a = SiLU(modulate(LN(h)) W1^T + b1), my 16 columns
      if (blk > 0) {
        ps_wait(p.cnt + 2 * blk - 1, target, p.err);
        load_h((blk - 1) & 1);
        res_from_hx((blk - 1) & 1);
      } else {
        res_from_input();
      }
      ln_mod(true);
      __syncthreads();
      mma(bw, 0);
      wload(p.w2 + (long long)blk * W * W, col0 + li, W, bw);  // fc2's fragments
      __syncthreads();
      if (w == 0) {
        const f32x4 acc = reduce(0);
        const float bn = p.b1[blk * W + col0 + li];
#pragma unroll
        for (int j = 0; j < 4; ++j) sT[(4 * g + j) * 16 + li] = silu(acc[j] + bn);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (l < 32) {
          const int row = l >> 1, c8 = (l & 1) * 8;
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16)sT[row * 16 + c8 + e];
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, o), rs_ha, (row * W + col0 + c8) * 2, 0,
                                                 PS_SC1);
        }
        ps_publish(p.cnt + 2 * blk, p.no_publish);
      }
      // ---- fc2: h' = h + gate * (a W2^T + b2), my 16 columns
      if (blk + 1 < D) {
        const bf16* mn = mb + 3LL * W;
        ln_prefetch(p.lnw + (blk + 1) * W, p.lnb + (blk + 1) * W, mn, mn + W);
      } else {
        const bf16* mf = modk + 3LL * W * D;
        ln_prefetch(nullptr, nullptr, mf, mf + W);
      }
      float gt[4] = {0.f, 0.f, 0.f, 0.f}, bn2 = 0.f;
      if (w == 0) {
        bn2 = p.b2[blk * W + col0 + li];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          gt[j] = r < R ? (float)mb[(long long)r * p.ldmod + 2 * W + col0 + li] : 0.f;
        }
      }
      ps_wait(p.cnt + 2 * blk, target, p.err);
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int q = tid + 256 * m, row = q >> 7, c8 = (q & 127) * 8;
        const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(rs_ha, (row * W + c8) * 2, 0, PS_SC1);
        *(u32x4v*)(sA + row * PS_LDA + c8) = v;
      }
      __syncthreads();
      mma(bw, 0);
      if (blk + 1 < D) {
        wload(p.w1 + (long long)(blk + 1) * W * W, col0 + li, W, bw);
      } else {
        wload(p.wf, li, 2 * C, bw);
        wload(p.wf, 16 + li, 2 * C, bw2);
      }
      __syncthreads();
      if (w == 0) {
        const f32x4 acc = reduce(0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          sT[r * 16 + li] = sRes[r * 16 + li] + gt[j] * (acc[j] + bn2);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int row = l >> 2, c4 = (l & 3) * 4;
        const u32x4v o = *(const u32x4v*)(sT + row * 16 + c4);
        __builtin_amdgcn_raw_buffer_store_b128(o, rs_hx, (((blk & 1) * PS_R + row) * W + col0 + c4) * 4, 0, PS_SC1);
        ps_publish(p.cnt + 2 * blk + 1, p.no_publish);
      }
    }
    // ---- final layer (every workgroup): out = modulate(LN(h)) Wf^T + bf, N = 2C <= 32
    {
      const int N2 = 2 * C;
      ps_wait(p.cnt + 2 * D - 1, target, p.err);
      load_h((D - 1) & 1);
      ln_mod(false);
      __syncthreads();
      mma(bw, 0);
      if (N2 > 16) mma(bw2, 1);
      if (k + 1 < p.S) {  // the next step's fc1_0 operands
        const bf16* mn = modk + (long long)R * p.ldmod;
        wload(p.w1, col0 + li, W, bw);
        ln_prefetch(p.lnw, p.lnb, mn, mn + W);
      }
      __syncthreads();
      if (w == 0) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (t == 1 && N2 <= 16) break;
          const f32x4 acc = reduce(t);
          const int n = 16 * t + li;
          const float bn = n < N2 ? p.bfin[n] : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) sOut[(4 * g + j) * 32 + n] = acc[j] + bn;
        }
      }
      __syncthreads();
      // p_sample (gaussian_diffusion.py:395-440), one element per thread
      {
        const int r = tid >> 4, c = tid & 15;
        if (r < R && c < C) {
          const float* kc = p.coef + 8LL * k;
          const float eps = sOut[r * 32 + c], v = sOut[r * 32 + C + c], xi = sX[tid];
          const float f = (v + 1.0f) * 0.5f;
          const float log_var = f * kc[5] + (1.0f - f) * kc[4];
          float x0 = kc[0] * xi - kc[1] * eps;
          if (p.clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
          const float mean = kc[2] * x0 + kc[3] * xi;
          const float xn = mean + kc[6] * expf(0.5f * log_var) * p.noise[((long long)k * R + r) * C + c] * kc[7];
          sX[tid] = xn;
          sXn[tid] = (float)(bf16)xn;
        }
      }
      __syncthreads();
    }
  }
  if (blockIdx.x == 0) {
    // a run in which any wait gave up (some workgroup computed on a stale exchange buffer) returns
    // NaN, never plausible-looking actions; the host also reads the flag (sampler.py)
    const bool bad = __hip_atomic_load((gu32*)p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
    const int r = tid >> 4, c = tid & 15;
    if (r < R && c < C) p.x_out[r * C + c] = bad ? __builtin_nanf("") : sX[tid];
  }
}
}  // namespace

// test hook: the NEXT uva_sampler_persistent launch publishes no phase, so every hand-off wait runs
// into its spin bound -> the give-up path (flag set, NaN output) is exercised deterministically
static int ps_test_no_publish = 0;
extern "C" int uva_sampler_persistent_test_hook(int no_publish) {
  ps_test_no_publish = no_publish ? 1 : 0;
  return 0;
}

extern "C" long long uva_sampler_persistent_workspace(int W) {
  return 256 + 2LL * PS_R * W * 4 + (long long)PS_R * W * 2;
}

extern "C" int uva_sampler_persistent(int R, int C, int W, int depth, int S, int clip, float eps, const void* w1,
                                      const float* b1, const void* w2, const float* b2, const float* lnw,
                                      const float* lnb,
                                      const void* win, const float* bin, const void* wf, const float* bfin,
                                      const void* mod, long long ldmod, const float* coef, const float* noise,
                                      const float* x0, float* x_out, void* work, long long work_bytes, hipStream_t s) {
  // built for the action head's depth (diffloss_act_d = 6, config/model/uva.yaml)
  if (R < 1 || R > PS_R || C < 1 || C > PS_C || W != PS_W || depth != 6 || S < 1 || !work ||
      work_bytes < uva_sampler_persistent_workspace(W) || ldmod < (3LL * depth + 2) * W || (ldmod & 3) ||
      ((uintptr_t)work & 255) || ((uintptr_t)mod & 7))
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)w1 | (uintptr_t)w2 | (uintptr_t)lnw | (uintptr_t)lnb | (uintptr_t)wf | (uintptr_t)bin) & 15)
    return (int)hipErrorInvalidValue;
  PSParams p{};
  p.w1 = (const bf16*)w1;
  p.b1 = b1;
  p.w2 = (const bf16*)w2;
  p.b2 = b2;
  p.lnw = lnw;
  p.lnb = lnb;
  p.win = (const bf16*)win;
  p.bin = bin;
  p.wf = (const bf16*)wf;
  p.bfin = bfin;
  p.mod = (const bf16*)mod;
  p.ldmod = ldmod;
  p.coef = coef;
  p.noise = noise;
  p.x0 = x0;
  p.x_out = x_out;
  p.cnt = (unsigned*)work;
  p.err = (unsigned*)work + 32;
  p.hx = (float*)((char*)work + 256);
  p.ha = (bf16*)((char*)work + 256 + 2LL * PS_R * W * 4);
  p.R = R;
  p.C = C;
  p.depth = depth;
  p.S = S;
  p.clip = clip;
  p.eps = eps;
  p.no_publish = ps_test_no_publish;
  ps_test_no_publish = 0;  // one launch only
  // > 80 KB of LDS: one workgroup per CU (the hand-off's measured form), 64 of 256 CUs
  constexpr int kLds = 96 * 1024;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)sampler_persistent_kernel<6>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kLds);
    attr = true;
  }
  hipError_t e = hipMemsetAsync(work, 0, 256, s);  // counters + give-up flag, every call
  if (e != hipSuccess) return (int)e;
  sampler_persistent_kernel<6><<<PS_G, 256, kLds, s>>>(p);
  UVA_LAUNCH_CHECK();
  return 0;
}

// give-up flag of the last persistent sampler run on `work` (debug / tests; host copy)
extern "C" int uva_sampler_persistent_status(const void* work, unsigned* flag, hipStream_t s) {
  hipError_t e = hipMemcpyAsync(flag, (const unsigned*)work + 32, 4, hipMemcpyDeviceToHost, s);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamSynchronize(s);
}
