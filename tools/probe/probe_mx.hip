// Probe of the v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3, unit scales) operand lane maps: one wave,
// A/B given as the raw 32-byte per-lane operand registers, C/D written per lane.  Tool only (not
// part of libuva_hip.so); tools/probe/probe_mx.py compares the result with candidate maps.
#include <hip/hip_runtime.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
__global__ void probe_kernel(const i32x8* a, const i32x8* b, f32x16* c) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[l], b[l], acc, 0, 0, 0, 127, 0, 127);
  c[l] = acc;
}
extern "C" int probe_mx(const void* a, const void* b, void* c) {
  probe_kernel<<<1, 64>>>((const i32x8*)a, (const i32x8*)b, (f32x16*)c);
  return (int)hipDeviceSynchronize();
}
