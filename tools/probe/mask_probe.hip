// Dropout bit-plane kernel variants vs attn_mask_kernel (tools only): bit-identical planes required.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I unified_video_action_amd/csrc tools/probe/mask_probe.hip -o tools/probe/mask_probe
#include "../../unified_video_action_amd/csrc/attention.hip"
// (attn_mask_kernel there is now the v2 / TPW 4 form measured here against the original)

#include <cstdio>
#include <vector>

// the DROP bit of element (pair j, half) enters the plane word by v_alignbit shift-in: positions
// 63..0 in descending order; pair j covers positions mask_pos(2j) (even) and +1
__device__ __forceinline__ uint32_t shin(uint32_t acc, uint32_t t) { return __builtin_amdgcn_alignbit(acc, t, 31); }

template <int TPW>
__global__ __launch_bounds__(256) void mask_v2(uint64_t* __restrict__ MQ, uint64_t* __restrict__ MK, int N, int nt,
                                               long long tasks, uint32_t th, uint64_t seed) {
  const long long task0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * TPW;
  if (task0 >= tasks) return;
  const int L = threadIdx.x & 63;
  const int kv0 = (int)(task0 % nt);
  const long long t2 = task0 / nt;
  const int qb = (int)(t2 % nt);
  const long long bh = t2 / nt;
  const int q = qb * 64 + mask_pos(L);
  const uint32_t key = drop_key(seed);
  const uint64_t rowpair = (((uint64_t)bh * N + q) * (uint64_t)N) >> 1;
#pragma unroll 1
  for (int u = 0; u < TPW; ++u) {
    const int kv = kv0 + u;
    const uint32_t x0 = drop_first(key, rowpair + (uint64_t)kv * 32);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int P = 31; P >= 0; --P) {
      const int j = mask_pos(2 * P) >> 1;
      uint32_t x = x0 ^ (uint32_t)j;
      x ^= x >> 16;
      x *= 0x7feb352du;
      x ^= x >> 15;
      x *= 0x846ca68bu;
      const uint32_t xh = x >> 16;
      const uint32_t t0 = ((x ^ xh) & 0xFFFFu) - th;  // drop iff negative
      const uint32_t t1 = xh - th;
      if (P >= 16) {
        hi = shin(hi, t1);
        hi = shin(hi, t0);
      } else {
        lo = shin(lo, t1);
        lo = shin(lo, t0);
      }
    }
    lo = ~lo;
    hi = ~hi;
    MQ[((long long)bh * nt + kv) * N + q] = ((uint64_t)hi << 32) | lo;
    {
      const bool up = L & 32;
      const auto r = __builtin_amdgcn_permlane32_swap(up ? lo : hi, up ? lo : hi, false, false);
      const uint32_t o = up ? r[0] : r[1];
      if (up) lo = o; else hi = o;
    }
#define UVA_TSTAGE(J, M)                                                                    \
  {                                                                                         \
    const bool up = L & (J);                                                                \
    const uint32_t sr = up ? 0u : (uint32_t)(J);                                            \
    const uint32_t km = up ? ~(M) : (M);                                                    \
    const uint32_t rl = (uint32_t)__builtin_amdgcn_ds_swizzle((int)((lo >> sr) & (M)), 0x1F | ((J) << 10)); \
    const uint32_t rh = (uint32_t)__builtin_amdgcn_ds_swizzle((int)((hi >> sr) & (M)), 0x1F | ((J) << 10)); \
    lo = (lo & km) | (rl << sr);                                                            \
    hi = (hi & km) | (rh << sr);                                                            \
  }
    UVA_TSTAGE(16, 0x0000FFFFu)
    UVA_TSTAGE(8, 0x00FF00FFu)
    UVA_TSTAGE(4, 0x0F0F0F0Fu)
    UVA_TSTAGE(2, 0x33333333u)
    UVA_TSTAGE(1, 0x55555555u)
#undef UVA_TSTAGE
    MK[((long long)bh * nt + qb) * N + (long long)kv * 64 + mask_pos(L)] = ((uint64_t)hi << 32) | lo;
  }
}

// hash-only (no plane stores beyond one word): the VALU floor
__global__ __launch_bounds__(256) void mask_hashonly(uint64_t* __restrict__ MQ, int N, int nt, long long tasks,
                                                     uint32_t th, uint64_t seed) {
  const long long task = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= tasks) return;
  const int L = threadIdx.x & 63;
  const uint32_t key = drop_key(seed);
  const uint32_t x0 = drop_first(key, ((uint64_t)task * 64 + L) * 32);
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int P = 31; P >= 0; --P) {
    uint32_t x = x0 ^ (uint32_t)P;
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    const uint32_t xh = x >> 16;
    const uint32_t t0 = ((x ^ xh) & 0xFFFFu) - th;
    const uint32_t t1 = xh - th;
    if (P >= 16) { hi = shin(hi, t1); hi = shin(hi, t0); } else { lo = shin(lo, t1); lo = shin(lo, t0); }
  }
  if ((lo ^ hi) == 0x12345678u) MQ[task] = lo;
}

// store-only (constant planes): the write floor
__global__ __launch_bounds__(256) void mask_storeonly(uint64_t* __restrict__ MQ, uint64_t* __restrict__ MK, int N,
                                                      int nt, long long tasks) {
  const long long task = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (task >= tasks) return;
  const int L = threadIdx.x & 63;
  const int kv = (int)(task % nt);
  const long long t2 = task / nt;
  const int qb = (int)(t2 % nt);
  const long long bh = t2 / nt;
  const int q = qb * 64 + mask_pos(L);
  MQ[((long long)bh * nt + kv) * N + q] = (uint64_t)task;
  MK[((long long)bh * nt + qb) * N + (long long)kv * 64 + mask_pos(L)] = (uint64_t)task;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const int B = 32, N = 1024, H = 12;
  const float p = 0.1f;
  const unsigned long long seed = 20240;
  const int nt = N / 64;
  const long long words = (long long)B * H * N * nt;  // per plane
  const long long tasks = (long long)B * H * nt * nt;
  uint32_t th;
  float ds;
  uva_drop_params(p, &th, &ds);
  uint64_t *ref, *got;
  CK(hipMalloc(&ref, 2 * words * 8));
  CK(hipMalloc(&got, 2 * words * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int IT = 20;
  auto timeit = [&](auto fn) -> float {
    fn();
    hipEventRecord(e0, 0);
    for (int i = 0; i < IT; ++i) fn();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return 1000.f * ms / IT;
  };
  std::vector<uint64_t> h0(2 * words), h1(2 * words);
  float t = timeit([&] { uva_attn_dropmask(ref, B, N, H, p, seed, 0); });
  CK(hipDeviceSynchronize());
  printf("orig      %8.1f us\n", t);
  CK(hipMemcpy(h0.data(), ref, 2 * words * 8, hipMemcpyDeviceToHost));
  auto check = [&](const char* name, float us) {
    hipDeviceSynchronize();
    hipMemcpy(h1.data(), got, 2 * words * 8, hipMemcpyDeviceToHost);
    long long bad = 0;
    for (long long i = 0; i < 2 * words; ++i) bad += h0[i] != h1[i];
    printf("%-9s %8.1f us  mismatched words %lld\n", name, us, bad);
  };
  CK(hipMemset(got, 0, 2 * words * 8));
  t = timeit([&] { mask_v2<1><<<dim3((unsigned)((tasks + 3) / 4)), 256>>>(got, got + words, N, nt, tasks, th, seed); });
  check("v2", t);
  CK(hipMemset(got, 0, 2 * words * 8));
  t = timeit([&] { mask_v2<2><<<dim3((unsigned)((tasks / 2 + 3) / 4)), 256>>>(got, got + words, N, nt, tasks, th, seed); });
  check("v2 tpw2", t);
  CK(hipMemset(got, 0, 2 * words * 8));
  t = timeit([&] { mask_v2<4><<<dim3((unsigned)((tasks / 4 + 3) / 4)), 256>>>(got, got + words, N, nt, tasks, th, seed); });
  check("v2 tpw4", t);
  t = timeit([&] { mask_hashonly<<<dim3((unsigned)((tasks + 3) / 4)), 256>>>(got, N, nt, tasks, th, seed); });
  printf("hashonly  %8.1f us\n", t);
  t = timeit([&] { mask_storeonly<<<dim3((unsigned)((tasks + 3) / 4)), 256>>>(got, got + words, N, nt, tasks); });
  printf("storeonly %8.1f us\n", t);
  CK(hipDeviceSynchronize());
  return 0;
}
