// Shared device helpers for the UVA MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
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
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}
// keep with probability 1-p: threshold = p * 2^32 (host computes, passed as uint32)
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  return mix32(seed ^ (idx * 0x9E3779B97F4A7C15ULL)) >= thresh;
}

// ---- activations ---------------------------------------------------------------------
#define ACT_NONE 0
#define ACT_GELU 1
#define ACT_SILU 2
#define ACT_RELU 3

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  float s = 1.0f / (1.0f + __expf(-x));
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
#define UVA_LAUNCH_CHECK() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
