// Shared device helpers for the UVA MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

#define UVA_DT_F32 0
#define UVA_DT_BF16 1

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// ---- wave (64-lane) reductions --------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// reduce across the 16 lanes that share (lane >> 4) -- the column lanes of an MFMA 16x16 tile
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- counter-based dropout mask (identical in forward and backward kernels) ------------
// ---- dropout mask ----------------------------------------------------------------------
// Stateless counter-based mask shared by every kernel that drops (GEMM epilogues, attention
// fwd/bwd, softmax, activation backward), so forward and backward regenerate identical masks.
// Element idx belongs to pair idx >> 1; one 32-bit hash per pair (the keyed counter through the
// lowbias32 finalizer: 2 x v_mul_lo_u32, no 64-bit multiplies) yields two 16-bit uniforms:
// low half -> even idx, high half -> odd idx.
// keep iff u16 >= thresh, thresh = round(p * 65536); kept values scale by 65536 / (65536 - thresh).
__host__ __device__ __forceinline__ uint32_t drop_key(uint64_t seed) {
  uint32_t k = (uint32_t)seed ^ (((uint32_t)(seed >> 32)) * 0x9E3779B1u);
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  return k;
}
// drop_hash = drop_mix(first word); split so a caller hashing pairs base..base+31 of a 32-aligned
// base can form the first word as (base's first word) ^ j
__device__ __forceinline__ uint32_t drop_first(uint32_t key, uint64_t pair) {
  return (uint32_t)pair ^ (key + __builtin_rotateleft32((uint32_t)(pair >> 32), 11));
}
__device__ __forceinline__ uint32_t drop_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t key, uint64_t pair) {
  uint32_t x = drop_first(key, pair);
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  const uint32_t h = drop_hash(drop_key(seed), idx >> 1);
  return ((idx & 1) ? (h >> 16) : (h & 0xFFFFu)) >= thresh;
}
// both elements of the pair (idx_even, idx_even + 1); idx_even must be even
__device__ __forceinline__ void dropout_keep2(uint64_t seed, uint64_t idx_even, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = drop_hash(drop_key(seed), idx_even >> 1);
  k0 = (h & 0xFFFFu) >= thresh;
  k1 = (h >> 16) >= thresh;
}

// host: p -> (16-bit threshold, keep scale); thresh 0 = no dropout
static inline void uva_drop_params(float p, uint32_t* thresh, float* scale) {
  if (!(p > 0.f)) {
    *thresh = 0;
    *scale = 1.0f;
    return;
  }
  long t = lrintf(p * 65536.0f);
  if (t < 1) t = 1;
  if (t > 65535) t = 65535;
  *thresh = (uint32_t)t;
  *scale = 65536.0f / (float)(65536 - t);
}

// ---- activations ---------------------------------------------------------------------
#define ACT_NONE 0
#define ACT_GELU 1
#define ACT_SILU 2
#define ACT_RELU 3

// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 rounding of every GELU
// output here): one v_rcp_f32 + one v_exp_f32 + 8 FMA-class ops, branch-free.  The library erff is
// a branchy polynomial ~3x the VALU work; in the fc1 GEMM epilogue (32768 x 3072 GELUs per block)
// it cost +85 us over the bias-only epilogue (313 vs 227 us).
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * ax * ax);
  return copysignf(fmaf(-p, e, 1.0f), x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// GELU'(x) = Phi(x) + x phi(x).  erf_fast(x / sqrt 2) evaluates exp(-x^2 / 2) -- phi(x) up to its constant --
// so the two share one v_exp_f32 (three transcendentals per element -> two: the act backward pass is
// VALU-bound at 4.3 TB/s)
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float e = __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);  // exp(-x^2 / 2)
  const float ax = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float erf_ = copysignf(fmaf(-p, e, 1.0f), x);
  // one explicit fma: left to the compiler, the contraction of `a + x * b` depended on the inlining
  // context, and the fused GEMM epilogue (gemm8w.hip EPI 3) and act_bwd_colsum must give the same bits
  return fmaf(x, 0.39894228040143268f * e, fmaf(0.5f, erf_, 0.5f));
}
// sigmoid as v_exp_f32 + v_rcp_f32 (1 ulp each): a plain `x / (1 + e)` compiles to the IEEE division
// sequence (2 x v_div_scale, v_div_fmas, v_div_fixup, v_rcp + 4 FMAs) -- 3x the VALU work of the
// GroupNorm+SiLU staging in the halo conv
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float silu(float x) { return x * sigmoid_fast(x); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = sigmoid_fast(x);
  return s * (1.0f + x * (1.0f - s));
}
__device__ __forceinline__ float apply_act(int act, float x) {
  switch (act) {
    case ACT_GELU: return gelu_erf(x);
    case ACT_SILU: return silu(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case ACT_GELU: return gelu_erf_grad(x);
    case ACT_SILU: return silu_grad(x);
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

// ---- launch error plumbing -----------------------------------------------------------
// XCD-aware (x, y) of a 2-D grid.  The hardware deals linear workgroup ids (x fastest) round-robin
// over the 8 XCDs, so the gridDim.x blocks of one y (one attention head: its K/V or Q/dO rows are
// re-read by every one of them) would land on 8 different L2s.  The remap gives each XCD a
// contiguous range of logical ids, so one head's blocks run back to back on one XCD's L2.
__device__ __forceinline__ void xcd_grid2(int& bx, int& by) {
  const int gx = gridDim.x, T = gx * gridDim.y;
  const int L = blockIdx.y * gx + blockIdx.x;
  const int q = T / 8, r = T % 8, x = L % 8;
  const int Lp = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + L / 8;
  bx = Lp % gx;
  by = Lp / gx;
}

// sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15), result in every lane: quad_perm xor 1,
// xor 2, then row_ror 4 and 8 -- four VALU adds with DPP operands instead of four dependent
// ds_bpermute round trips through the LDS crossbar (what __shfl_xor lowers to)
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  return v;
}

#define UVA_LAUNCH_CHECK() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
