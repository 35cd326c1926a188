// gemm_4w -- persistent 4-wave bf16 GEMM for the K-contiguous products of the timm Block
// (mar_con_unified.py:201-215 Attention.qkv, :236-249 Mlp.fc1 / fc2 forwards, and every dX product
// through the transposed weight copies): C[m][n] = alpha * sum_k A[m][k] B[n][k] (+ bias[n]),
// A [M][K] (lda), B [N][K] (ldb), both K-contiguous, fp32 accumulation, bf16 / fp32 output.
//
// Structure (one wave per SIMD, accumulators in AGPRs):
//   * workgroup = 4 waves as 2 (M) x 2 (N); a wave owns 16*FM x 16*FN of the 32*FM x 32*FN block tile
//     (FM = 8, FN = 6: 128 x 96 per wave, 192 accumulator registers); v_mfma_f32_16x16x32_bf16 with the
//     operands SWAPPED (B fragment as the MFMA A operand), so a lane holds 4 consecutive output columns
//     of one row and the epilogue runs from registers;
//   * K runs in 64-deep K-tiles; a 2-region LDS ring holds the A [BM][64] and B [BN][64] images of two
//     K-tiles, 128-B rows with the 16-B chunk index XOR-ed by (row & 7) (conflict-free ds_read_b128
//     fragments).  A region is filled by LDS-DMA (buffer_load ... lds, 16 B per lane, 8 rows x 128 B --
//     whole lines -- per wave-instruction: 16 rows x 64 B per instruction measured 13 % slower on the
//     K = 3072 product, profiles/r05/gemm4_diag.txt), per-lane sources computed once per tile and the K
//     step in the SGPR soffset;
//   * each K-tile is two 32-deep substeps.  Even substep: MFMAs on fragments in registers while the
//     odd substep's fragments are read from the same region.  Odd substep: wait until the NEXT K-tile's
//     DMA has landed (vmcnt(0) -- or the epilogue stores' count right after an epilogue -- then ONE
//     s_barrier: every wave is past its reads of this region and can see the next), refill this region
//     with K-tile t+2 (its DMAs among the first MFMAs), read the next K-tile's first fragments among the
//     rest.  The issue order inside a substep is pinned by sched_barrier fences;
//   * persistent: a workgroup per CU walks tiles pid = slot + i * grid (XCD-contiguous slots, GROUP-8
//     raster); the K-tile stream runs across tile boundaries (the last two K-tiles' refills load the next
//     tile's first two), so the next tile's data is in flight while this tile's register epilogue
//     (v_permlane16_swap pairs -> 16-B row segments, + bias from an LDS copy, cvt) issues its stores.
// Tails: rows / columns past M / N read zeros through the buffer descriptors' range check and are
// masked at the store.  The hipBLASLt kernels this replaces use the same 4-wave / 256-thread /
// AGPR-accumulator geometry (profiles/r04/ab_gemm_persist.txt).
#include "common.h"

// diagnostic builds only (tools/build_variant.py gemm4.hip -DUVA_G4_DIAG=n; results are WRONG): bit 1 no
// DMA inside the K loop, 2 no wait / barrier, 4 no epilogue stores, 8 no fragment reads inside the K loop
#ifndef UVA_G4_DIAG
#define UVA_G4_DIAG 0
#endif


namespace {

template <int FM_, int FN_>
struct G4Cfg {
  static constexpr int FM = FM_, FN = FN_;
  static constexpr int BM = 32 * FM, BN = 32 * FN;               // block tile
  static constexpr int GA = BM / 32, GB = BN / 32, G = GA + GB;  // DMA instructions per thread per K-tile
  static constexpr int A_BYTES = BM * 128, REGION = (BM + BN) * 128, RING = 2 * REGION;
};

__device__ __forceinline__ int g4_xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

}  // namespace

template <int FM, int FN, typename TC>
__global__ __launch_bounds__(256, 1) void gemm_4w(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  TC* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                  long long ldc, const float* __restrict__ bias, float alpha,
                                                  int w1ok) {
  using G = G4Cfg<FM, FN>;
  constexpr int E = FM * (FN / 2) * (sizeof(TC) == 2 ? 1 : 2);  // epilogue stores per thread per tile
  constexpr int WE = E > 63 ? 63 : E;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wr = w >> 1, wc = w & 1;
  const int tm = (M + G::BM - 1) / G::BM, tn = (N + G::BN - 1) / G::BN, ntiles = tm * tn;
  const int KT = K / 64;  // K-tiles per tile (even: checked by the launcher)
  const int grid = gridDim.x;
  const int slot = g4_xcd_remap(blockIdx.x, grid);
  if (slot >= ntiles) return;
  const int my_tiles = (ntiles - slot + grid - 1) / grid;

  // bias -> LDS (fp32, tn * BN entries, zero past N), before any DMA is in flight
  float* sbias = (float*)(smem + G::RING);
  const bool has_bias = bias != nullptr;
  if (has_bias) {
    for (int i = threadIdx.x; i < tn * G::BN; i += 256) sbias[i] = i < N ? bias[i] : 0.f;
    __syncthreads();
  }

  constexpr int GROUP = 8;
  auto tile_of = [&](int pid, int& m0, int& n0) __attribute__((always_inline)) {
    const int group = pid / (GROUP * tn), first_m = group * GROUP;
    const int gsz = min(tm - first_m, GROUP);
    m0 = (first_m + (pid % (GROUP * tn)) % gsz) * G::BM;
    n0 = ((pid % (GROUP * tn)) / gsz) * G::BN;
  };

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0,
                                                     (int)(unsigned)min(2ull * (unsigned long long)M * (unsigned)lda,
                                                                        0xffffffffull), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0,
                                                     (int)(unsigned)min(2ull * (unsigned long long)N * (unsigned)ldb,
                                                                        0xffffffffull), 0x00020000);
  // per-lane source offsets of the DMA target tile: instruction i of wave w covers image rows
  // 8 (w GA + i) .. +7; lane l: row (l >> 3), LDS chunk (l & 7) <- global chunk (l & 7) ^ (row & 7)
  const unsigned cofs = (unsigned)((((lane & 7) ^ ((lane >> 3) & 7))) * 16);
  const unsigned laneA = (unsigned)(lane >> 3) * (unsigned)lda * 2u + cofs;
  const unsigned laneB = (unsigned)(lane >> 3) * (unsigned)ldb * 2u + cofs;
  const unsigned rowA8 = 8u * (unsigned)lda * 2u, rowB8 = 8u * (unsigned)ldb * 2u;
  unsigned offA[G::GA], offB[G::GB];
  auto dma_offsets = [&](int pid) __attribute__((always_inline)) {
    int m0, n0;
    tile_of(pid, m0, n0);
    const unsigned a0 = laneA + (unsigned)__builtin_amdgcn_readfirstlane((m0 + 8 * w * G::GA) * lda * 2);
    const unsigned b0 = laneB + (unsigned)__builtin_amdgcn_readfirstlane((n0 + 8 * w * G::GB) * ldb * 2);
#pragma unroll
    for (int i = 0; i < G::GA; ++i) offA[i] = a0 + (unsigned)i * rowA8;
#pragma unroll
    for (int i = 0; i < G::GB; ++i) offB[i] = b0 + (unsigned)i * rowB8;
  };
  // DMA instruction i (A first) of K-tile kt of the offsets' tile into region r
  auto dma_one = [&](int r, int i, int so) __attribute__((always_inline)) {
    if (i < G::GA)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + (w * G::GA + i) * 1024), 16,
          (int)offA[i < G::GA ? i : 0], so, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + G::A_BYTES + (w * G::GB + i - G::GA) * 1024),
          16, (int)offB[i < G::GA ? 0 : i - G::GA], so, 0, 0);
  };
  dma_offsets(slot);

  // fragment reads: row (lane & 15), 16-B chunk h*4 + (lane >> 4) of a 128-B row (XOR row & 7)
  const int lrow = lane & 15;
  const int lofs0 = lrow * 128 + ((((lane >> 4)) ^ (lrow & 7)) << 4);
  const int lofs1 = lrow * 128 + (((4 + (lane >> 4)) ^ (lrow & 7)) << 4);
  const int a0o = wr * (FM * 16 * 128), b0o = G::A_BYTES + wc * (FN * 16 * 128);
  auto frag = [&](int byteofs) __attribute__((always_inline)) { return *(const bf16x8*)(smem + byteofs); };

  f32x4 acc[FM][FN];
  bf16x8 fa[2][FM], fb[2][FN];

  // prologue: K-tiles 0 and 1 into regions 0 and 1, wait for region 0, read substep 0's fragments
#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(0, i, 0);
#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(1, i, 128);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::G) : "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int f = 0; f < FM; ++f) fa[0][f] = frag(lofs0 + a0o + f * 1024 * 2);
#pragma unroll
  for (int g = 0; g < FN; ++g) fb[0][g] = frag(lofs0 + b0o + g * 1024 * 2);

  // one substep.  U: 0 / 2 even (regions 0 / 1), 1 / 3 odd; ZERO: first substep of a tile (MFMAs start
  // from the inline constant 0); post: first odd barrier after an epilogue (its stores are younger than
  // the awaited DMA); so: soffset of the K-tile an odd substep refills its region with
  auto substep = [&](auto UC, auto ZC, bool post, int so) __attribute__((always_inline)) {
    constexpr int u = decltype(UC)::value;
    constexpr bool ZERO = decltype(ZC)::value;
    constexpr bool ODD = (u & 1) != 0;
    constexpr int r = u >> 1, b = u & 1;
    // the fragments read during this substep: odd substep of this region (even) / even substep of the
    // other region (odd)
    constexpr int rn = ODD ? (r ^ 1) : r;
    const int lofs = ODD ? lofs0 : lofs1;
    if constexpr (ODD) {
      if constexpr (!(UVA_G4_DIAG & 2)) {
        if (post) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WE) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int NM = FM * FN, NR = FM + FN;
    // odd: one DMA after each of the first G MFMAs, then one read after every second MFMA;
    // even: one read after every third MFMA
    constexpr int RS = ODD ? G::G : 0, RP = ODD ? 2 : 3;
    static_assert(!ODD || G::G + 2 * NR <= NM + 1, "schedule");
#pragma unroll
    for (int mi = 0; mi < NM; ++mi) {
      const int f = mi / FN, g = mi % FN;
      if constexpr (ZERO)
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b][g], fa[b][f], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      else
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b][g], fa[b][f], acc[f][g], 0, 0, 0);
      if constexpr (ODD && !(UVA_G4_DIAG & 1)) {
        if (mi < G::G) dma_one(r, mi, so);
      }
      if (mi >= RS && (mi - RS) % RP == 0 && (mi - RS) / RP < NR) {
        const int ri = (mi - RS) / RP;
        if constexpr (!(UVA_G4_DIAG & 8)) {
          if (ri < FM) fa[b ^ 1][ri < FM ? ri : 0] = frag(rn * G::REGION + lofs + a0o + (ri < FM ? ri : 0) * 2048);
          else fb[b ^ 1][ri < FM ? 0 : ri - FM] = frag(rn * G::REGION + lofs + b0o + (ri < FM ? 0 : ri - FM) * 2048);
        } else {
          if (ri < FM) fa[b ^ 1][ri < FM ? ri : 0] = fa[b][ri < FM ? ri : 0];
          else fb[b ^ 1][ri < FM ? 0 : ri - FM] = fb[b][ri < FM ? 0 : ri - FM];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using U0 = std::integral_constant<int, 0>;
  using U1 = std::integral_constant<int, 1>;
  using U2 = std::integral_constant<int, 2>;
  using U3 = std::integral_constant<int, 3>;
  using ZT = std::integral_constant<bool, true>;
  using ZF = std::integral_constant<bool, false>;
  // two K-tiles (regions 0, 1); their odd substeps refill with K-tiles kt0 and kt0 + 1 of the offsets' tile
  auto group = [&](auto ZC, bool post, int kt0) __attribute__((always_inline)) {
    const int so0 = __builtin_amdgcn_readfirstlane(kt0 * 128), so1 = so0 + 128;
    substep(U0{}, ZC, false, so0);
    substep(U1{}, ZF{}, post, so0);
    substep(U2{}, ZF{}, false, so1);
    substep(U3{}, ZF{}, false, so1);
  };

  const int csub = ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;  // the lane's 8 columns in a 32-col pair
  const int ngroups = KT / 2;
  for (int ti = 0; ti < my_tiles; ++ti) {
    int m0, n0;
    tile_of(slot + ti * grid, m0, n0);
    const bool post = ti > 0 && w1ok;
    // the K-tile stream is two ahead: the last group's refills load the NEXT tile's K-tiles 0 and 1
    // (past the last tile: this tile's again -- valid addresses, never read)
    const int nxt = ti + 1 < my_tiles ? slot + (ti + 1) * grid : slot + ti * grid;
    group(ZT{}, post, 2);  // (K >= 256: checked by the launcher)
    for (int it = 1; it < ngroups - 1; ++it) group(ZF{}, false, 2 * it + 2);
    dma_offsets(nxt);
    group(ZF{}, false, 0);

    // ---- register epilogue: 8 consecutive columns per lane per fragment pair
    float bv[FN / 2][8];
#pragma unroll
    for (int p = 0; p < FN / 2; ++p) {
      if (has_bias) {
        const float4 x0 = *(const float4*)(sbias + n0 + wc * (FN * 16) + p * 32 + csub);
        const float4 x1 = *(const float4*)(sbias + n0 + wc * (FN * 16) + p * 32 + csub + 4);
        bv[p][0] = x0.x; bv[p][1] = x0.y; bv[p][2] = x0.z; bv[p][3] = x0.w;
        bv[p][4] = x1.x; bv[p][5] = x1.y; bv[p][6] = x1.z; bv[p][7] = x1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[p][e] = 0.f;
      }
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      __builtin_amdgcn_sched_barrier(0);  // one fragment row at a time (bounds the AGPR -> VGPR reads in flight)
      const int row = m0 + wr * (FM * 16) + f * 16 + lrow;
#pragma unroll
      for (int p = 0; p < FN / 2; ++p) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][2 * p][q]),
                                                          __float_as_uint(acc[f][2 * p + 1][q]), false, false);
          v[q] = __uint_as_float(x[0]);
          v[4 + q] = __uint_as_float(x[1]);
        }
        const int col = n0 + wc * (FN * 16) + p * 32 + csub;
        TC* dst = C + (long long)row * ldc + col;
        const bool ok = (UVA_G4_DIAG & 4) ? alpha == 12345.f : (row < M && col < N);
        if constexpr (sizeof(TC) == 2) {
          bf16x8 ov;
#pragma unroll
          for (int e = 0; e < 8; ++e) ov[e] = (bf16)fmaf(alpha, v[e], bv[p][e]);
          if (ok) *(bf16x8*)dst = ov;
        } else {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = fmaf(alpha, v[e], bv[p][e]);
          if (ok) {
            *(float4*)dst = make_float4(o[0], o[1], o[2], o[3]);
            *(float4*)(dst + 4) = make_float4(o[4], o[5], o[6], o[7]);
          }
        }
      }
    }
  }
  // the refills past the end land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int g4_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// -1 = automatic; otherwise the configuration index of g4_cfgs (measurement / tests)
static int g_gemm4_force = -1;
static int g_gemm4_on = 1;

struct G4Choice {
  int cfg;  // 0: 256x256 NS4, 1: 256x192 NS4 ; -1 none
  int grid;
};

static G4Choice g4_plan(int M, int N, int K) {
  G4Choice c{-1, 0};
  const int cus = g4_cus();
  if (K % 128 != 0 || K < 256 || M < 256 || N < 128) return c;
  // 256 x 256 (FN = 8: 256 accumulator AGPRs) is not built: with every AGPR holding an accumulator
  // hipcc shuffles accumulators through VGPRs inside the K loop (644 v_accvgpr_read / 480 _write per
  // tile body vs 192 / 0 for FN = 6); 256 x 192 tiles also divide the Block's N = 768 / 2304 / 3072
  // into whole rounds of 256 CUs at M = 32768
  const int BNs[2] = {256, 192};
  double best = -1.0;
  for (int i = 1; i < 2; ++i) {
    if (g_gemm4_force >= 0 && g_gemm4_force != i) continue;
    const int bn = BNs[i];
    if ((long long)((N + bn - 1) / bn) * bn * 4 + (i == 0 ? 131072 : 114688) > 163840) continue;  // bias in LDS
    const long long tiles = (long long)((M + 255) / 256) * ((N + bn - 1) / bn);
    const long long rounds = (tiles + cus - 1) / cus;
    const double occ = (double)tiles / (double)(rounds * cus);
    const double useful = (double)M * N / ((double)tiles * 256 * bn);
    // per-CU efficiency of the 256 x 192 tile relative to 256 x 256 (fewer MFMAs per staged byte)
    const double eff = occ * useful * (bn == 192 ? 0.97 : 1.0);
    if (eff > best + 1e-9) {
      best = eff;
      c.cfg = i;
      c.grid = (int)(tiles < cus ? tiles : cus);
    }
  }
  return c;
}

template <int FM, int FN, typename TC>
static int g4_launch(const void* A, const void* B, void* C, int M, int N, int K, long long lda, long long ldb,
                     long long ldc, const float* bias, float alpha, int grid, hipStream_t s) {
  using G = G4Cfg<FM, FN>;
  const int tn = (N + G::BN - 1) / G::BN;
  const int lds = G::RING + (bias ? tn * G::BN * 4 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_4w<FM, FN, TC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              163840);
    attr = true;
  }
  const int w1ok = (M % G::BM == 0) && (N % G::BN == 0);
  gemm_4w<FM, FN, TC><<<dim3(grid), 256, lds, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, (int)lda,
                                                       (int)ldb, ldc, bias, alpha, w1ok);
  UVA_LAUNCH_CHECK();
  return 0;
}

// 1 = launched, 0 = not eligible (caller falls back), < 0 = -hipError
extern "C" int uva_gemm4_try(int out_dtype, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                             long long ldb, long long ldc, const float* bias, float alpha, hipStream_t s) {
  if (!g_gemm4_on) return 0;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8 || N % 8 || lda < K || ldb < K) return 0;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return 0;
  if (2.0 * (double)M * (double)lda >= 4.0e9 || 2.0 * (double)N * (double)ldb >= 4.0e9) return 0;
  if (bias && ((uintptr_t)bias % 16)) return 0;
  const G4Choice c = g4_plan(M, N, K);
  if (c.cfg < 0) return 0;
  int r;
  if (out_dtype == UVA_DT_BF16) r = g4_launch<8, 6, bf16>(A, B, C, M, N, K, lda, ldb, ldc, bias, alpha, c.grid, s);
  else r = g4_launch<8, 6, float>(A, B, C, M, N, K, lda, ldb, ldc, bias, alpha, c.grid, s);
  return r ? -r : 1;
}

// measurement switches (tests / tools only): on = 0 routes every product back to gemm_8ph; force = config
// index (-1 automatic).  Return the previous value; -2 queries.
extern "C" int uva_gemm4_set(int on, int force) {
  const int prev = g_gemm4_on | ((g_gemm4_force + 1) << 1);
  if (on != -2) g_gemm4_on = on;
  if (force != -2) g_gemm4_force = force;
  return prev;
}

extern "C" long long uva_gemm4_plan(int M, int N, int K) {
  const G4Choice c = g4_plan(M, N, K);
  return c.cfg < 0 ? -1 : (long long)c.cfg | ((long long)c.grid << 8);
}
