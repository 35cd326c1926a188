// gemm_8w -- persistent 8-wave (two waves per SIMD) bf16 GEMM for the K-contiguous products of the timm
// Block (mar_con_unified.py:201-249): the same block tile, LDS ring, DMA and substep schedule as gemm_4w
// (gemm4.hip), but with 8 waves of 64 x 96 (96 accumulator AGPRs each, so two waves fit a SIMD's 512
// registers) instead of 4 waves of 128 x 96.  The point is the epilogue: at one wave per SIMD nothing
// runs beside gemm_4w's epilogue, so the elementwise work a timm Mlp puts after fc1 / fc2 (GELU, dropout,
// residual) costs its full issue time there (runtime.py mlp_split_epilogue).  Here each wave can DEFER
// its tile's epilogue: the outputs are rounded to bf16 and packed (48 VGPRs), and the epilogue's VALU and
// stores are spread over the next tile's first substeps, one fragment row per substep, between that
// wave's own MFMAs -- while the partner wave on the SIMD keeps the matrix pipe busy.
//
//   C[m][n] = epi(alpha * sum_k A[m][k] B[n][k] + bias[n]),  A [M][K] (lda), B [N][K] (ldb), both
//   K-contiguous, fp32 accumulation.
//   EPI 0: plain (bf16 / fp32 out).
//   EPI 1 (timm Mlp fc1, training): P = bf16(acc + bias) stored to C2 (the GELU input the backward needs),
//          C = bf16(drop(gelu(P))) with the counter-hash dropout of common.h on the flat element index --
//          bit-identical to the split route (bias-only GEMM -> act_drop_fwd).
//   EPI 2 (timm Mlp fc2 / attention proj, training): C (fp32) = R + drop(bf16(acc + bias)), R an fp32
//          residual [M][ldc] -- bit-identical to bias-only GEMM -> act_drop_fwd(residual).
//   EPI 3 (timm Mlp backward through GELU + dropout, the fc2 dX product): dA = bf16(acc) (fc2's input
//          gradient, as the split route stores it), C = bf16(gelu'(P) * drop(dA)) with P the saved fc1
//          pre-activation (C2, bf16) -- bit-identical to dX GEMM -> act_bwd_bias -- and the column sums of C
//          (fc1's bias gradient) as per-64-row partials, part[(m0 + 64 wr) / 64][n], reduced by
//          colsum_final in a second launch (the same values summed in another order than act_bwd_bias).
#include "common.h"

#include <algorithm>
#include <type_traits>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// diagnostics (tools/build_variant.py gemm8w.hip -DUVA_G8_DBG=n): 1 no EPI 3 column partials, 2 s_nop after each
// EPI 3 store, 4 vmcnt(0) after a tile's epilogue
#ifndef UVA_G8_DBG
#define UVA_G8_DBG 0
#endif
// 1: EPI 3 row inputs (the saved pre-activation) loaded one fragment row ahead; 0: each segment loads its own just
// before use.  (EPI 2's residual rows ahead measured no faster: fc2 157 vs 154 us, profiles/r06/g8w_prefetch.txt)
#ifndef UVA_G8_PREFETCH
#define UVA_G8_PREFETCH 1
#endif

namespace {

template <int FM_, int FN_, int NW_>
struct G8Cfg {
  static constexpr int FM = FM_, FN = FN_, NW = NW_;
  static constexpr int WM = NW / 2, WN = 2;                       // wave grid
  static constexpr int BM = 16 * FM * WM, BN = 16 * FN * WN;      // block tile
  static constexpr int GA = BM / (8 * NW), GB = BN / (8 * NW), G = GA + GB;  // DMA instructions per wave per K-tile
  static constexpr int A_BYTES = BM * 128, REGION = (BM + BN) * 128, RING = 2 * REGION;
  static_assert(GA * 8 * NW == BM && GB * 8 * NW == BN, "DMA split");
};

__device__ __forceinline__ int g8_xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// 16-B chunk swizzle of a k-major image row [64 k][W] (TA / TB = 1 operands), as gemm4.hip's: the 8 rows a
// 32-lane group of ds_read_b64_tr_b16 touches fall on distinct 32-B bank slots
template <int W>
__device__ __forceinline__ int g8_kswz(int k) {
  static_assert(W == 256 || W == 192, "row width");
  if constexpr (W == 256) return ((k & 3) << 1) | (((k >> 3) & 1) << 3);
  else return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2);
}

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2_t));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

}  // namespace

struct G8Epi {
  const float* bias;
  float alpha;
  void* C2;              // EPI 1: the pre-activation (bf16, ldc)
  const float* R;        // EPI 2: fp32 residual (ldc)
  float* part;           // EPI 3: column-sum partials [tm * 4][N]
  const uint32_t* plane; // dropout keep bits of the [M][N] output (elementwise.hip drop_plane_kernel), or null:
                         // then the counter hash (key, thresh) is evaluated per element
  uint32_t key;          // dropout: drop_key(seed)
  uint32_t thresh;       // 0 = no dropout
  float dscale;
};

// DM: dropout in the fused epilogues -- 0 none, 1 the counter hash per element, 2 a keep-bit plane (compile-time:
// runtime branches per segment split the epilogue into small basic blocks the scheduler cannot interleave)
// NW = 8: one workgroup per CU (two waves per SIMD in lockstep: both reach the epilogue together), the bias
// row in LDS.  NW = 4: a 128 x 192 block tile, two independent workgroups per CU (80 KB of ring each: the
// bias comes from L2 instead), so one workgroup's epilogue can run beside the other's MFMA loop.
// TA / TB = 1 (the dW products: A [K][M], B [K][N], M- / N-contiguous; EPI 0, fp32 C): k-major LDS images read
// by ds_read_b64_tr_b16, and work items (tile, K-slice) writing fp32 partial slabs C + slice * slab_bytes
// (reduced by splitk_reduce) when splits > 1.
template <int FM, int FN, int NW, int EPI, int NDEF, typename TC, int DM, int TA = 0, int TB = 0>
__global__ __launch_bounds__(64 * NW, 8 / NW) void gemm_8w(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       TC* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                       int ldc, G8Epi ep, int w1ok, int splits, int kps,
                                                       int slab_bytes) {
  using G = G8Cfg<FM, FN, NW>;
  static_assert((TA == 0 && TB == 0) || (EPI == 0 && NDEF == 0 && sizeof(TC) == 4), "k-major operands: plain fp32");
  static_assert(EPI == 0 || sizeof(TC) == (EPI == 2 ? 4 : 2), "EPI output type");
  // stores per wave per item: one 16-B store per (fragment row, column pair) (fp32: two); EPI 1 also P;
  // EPI 3 the tile's column-sum partials (two per column pair)
  constexpr int E = FM * (FN / 2) * (sizeof(TC) == 2 ? 1 : 2) * (EPI == 1 ? 2 : 1) + (EPI == 3 ? FN : 0);
  constexpr int NM = FM * FN, NR = FM + FN;
  constexpr int RAW_AT = G::G + 2;
  static_assert(RAW_AT + 2 * FM - 2 < NM && RAW_AT + 2 * FN - 1 < NM + 2 * FN && FM * FN - 1 < NM, "schedule");
  constexpr int DS = NM;  // the refill DMAs spread over the whole odd substep
  constexpr int NB = (RAW_AT * G::G + DS - 1) / DS < G::G ? (RAW_AT * G::G + DS - 1) / DS : G::G;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wr = w >> 1, wc = w & 1;
  const int tm = (M + G::BM - 1) / G::BM, tn = (N + G::BN - 1) / G::BN, ntiles = tm * tn;
  const int nitems = ntiles * splits;
  const int grid = gridDim.x;
  const int slot = g8_xcd_remap(blockIdx.x, grid);
  if (slot >= nitems) return;
  const int my_items = (nitems - slot + grid - 1) / grid;

  float* sbias = (float*)(smem + G::RING);
  const bool has_bias = ep.bias != nullptr;
  constexpr bool LDS_BIAS = NW == 8;
  const auto rsBias = __builtin_amdgcn_make_buffer_rsrc((void*)(has_bias ? ep.bias : (const float*)A), 0,
                                                        has_bias ? 4 * N : 0, 0x00020000);
  if (LDS_BIAS && has_bias) {
    for (int i = threadIdx.x; i < tn * G::BN; i += 64 * NW) sbias[i] = i < N ? ep.bias[i] : 0.f;
    __syncthreads();
  }

  constexpr int GROUP = 8;
  // item -> (tile: GROUP-8 raster, K-slice sl: the slow index, so concurrent items share one K range)
  auto item_of = [&](int pid, int& m0, int& n0) __attribute__((always_inline)) {
    const int t = pid % ntiles;
    const int group = t / (GROUP * tn), first_m = group * GROUP;
    const int gsz = min(tm - first_m, GROUP);
    m0 = (first_m + (t % (GROUP * tn)) % gsz) * G::BM;
    n0 = ((t % (GROUP * tn)) / gsz) * G::BN;
  };

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A, 0, (int)(unsigned)(2ull * (unsigned)(TA ? K : M) * (unsigned)lda), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)B, 0, (int)(unsigned)(2ull * (unsigned)(TB ? K : N) * (unsigned)ldb), 0x00020000);
  // T = 1: the k-major image [64][W] taken 1 KB per DMA instruction in byte order; lane l of piece j: byte
  // j KB + 16 l -> (k, chunk), global chunk = chunk ^ kswz(k)
  auto lane_src_k = [&](auto WC, int piece, int ld) __attribute__((always_inline)) -> unsigned {
    constexpr int W = decltype(WC)::value;
    const int b = piece * 1024 + lane * 16;
    const int k = b / (W * 2), c = (b % (W * 2)) >> 4;
    return (unsigned)k * (unsigned)ld * 2u + (unsigned)((c ^ g8_kswz<W>(k)) * 16);
  };
  using WAc = std::integral_constant<int, G::BM>;
  using WBc = std::integral_constant<int, G::BN>;
  constexpr int stepA = TA ? 0 : 128, stepB = TB ? 0 : 128;  // bytes per K-tile (T = 1: 64 rows of ld, runtime)
  const int stA = TA ? 64 * lda * 2 : stepA, stB = TB ? 64 * ldb * 2 : stepB;
  // per-lane DMA sources: instruction i of wave w covers image rows 8 (w G + i) .. +7 of 128 B; lane l: row
  // (l >> 3), LDS chunk (l & 7) <- global chunk (l & 7) ^ (row & 7); the K-tile step is the soffset
  unsigned offA[G::GA], offB[G::GB];
  auto dma_offsets = [&](int pid) __attribute__((always_inline)) {
    int m0, n0;
    item_of(pid, m0, n0);
    const int kb = (pid / ntiles) * kps;
    const unsigned a0 = (unsigned)__builtin_amdgcn_readfirstlane(TA ? (kb * lda + m0) * 2 : (m0 * lda + kb) * 2);
    const unsigned b0 = (unsigned)__builtin_amdgcn_readfirstlane(TB ? (kb * ldb + n0) * 2 : (n0 * ldb + kb) * 2);
#pragma unroll
    for (int i = 0; i < G::GA; ++i) {
      const int row = 8 * (w * G::GA + i) + (lane >> 3);
      if constexpr (TA != 0) offA[i] = a0 + lane_src_k(WAc{}, w * G::GA + i, lda);
      else offA[i] = a0 + (unsigned)row * (unsigned)lda * 2u + (unsigned)(((lane & 7) ^ (row & 7)) * 16);
    }
#pragma unroll
    for (int i = 0; i < G::GB; ++i) {
      const int row = 8 * (w * G::GB + i) + (lane >> 3);
      if constexpr (TB != 0) offB[i] = b0 + lane_src_k(WBc{}, w * G::GB + i, ldb);
      else offB[i] = b0 + (unsigned)row * (unsigned)ldb * 2u + (unsigned)(((lane & 7) ^ (row & 7)) * 16);
    }
  };
  auto dma_one = [&](int r, int i, int kt) __attribute__((always_inline)) {
    if (i < G::GA)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + (w * G::GA + i) * 1024), 16,
          (int)offA[i < G::GA ? i : 0], __builtin_amdgcn_readfirstlane(kt * stA), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + G::A_BYTES + (w * G::GB + i - G::GA) * 1024),
          16, (int)offB[i < G::GA ? 0 : i - G::GA], __builtin_amdgcn_readfirstlane(kt * stB), 0, 0);
  };
  dma_offsets(slot);

  const int lrow = lane & 15;
  const int lofs0 = lrow * 128 + (((lane >> 4) ^ (lrow & 7)) << 4);
  const int lofs1 = lrow * 128 + (((4 + (lane >> 4)) ^ (lrow & 7)) << 4);
  const int a0o = wr * (FM * 16), b0o = wc * (FN * 16);
  // T = 1: two ds_read_b64_tr_b16 of the k-major image (rows k and k + 4 of the lane's quad, 4 columns each),
  // the hardware transpose gathering the lane's 8 consecutive k (the same k order as the T = 0 read).  The
  // swizzle of rows k, k + 4, k + 32, k + 36 is one lane constant sw (kswz reads bits 0-3 of k, q + 4 < 8) and
  // the fragment's 8-column chunk c0 / 8 is even and wave-uniform, so an address is lane constant + ((c0 / 8 ^
  // sw) << 4) + immediate: two VALU per fragment instead of a hoisted address register per (fragment, half)
  // (those spilled 14 VGPRs).  The empty asm keeps hipcc from hoisting the per-fragment values again.
  const int kq = (lane >> 4) * 8 + ((lane >> 2) & 3);
  auto frag_k = [&](auto WC, int base, int c0, int h) __attribute__((always_inline)) -> bf16x8 {
    constexpr int W = decltype(WC)::value;
    int sw = g8_kswz<W>(kq);
    asm volatile("" : "+v"(sw));
    const int lb = kq * W * 2 + ((lane >> 1) & 1) * 16 + (lane & 1) * 8;
    const char* a0 = smem + base + h * 32 * W * 2 + lb + (((c0 >> 3) ^ sw) << 4);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0 + 4 * W * 2));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };
  auto fragA = [&](int r, int f, int h) __attribute__((always_inline)) {
    if constexpr (TA) return frag_k(WAc{}, r * G::REGION, a0o + f * 16, h);
    else return *(const bf16x8*)(smem + r * G::REGION + (a0o + f * 16) * 128 + (h ? lofs1 : lofs0));
  };
  auto fragB = [&](int r, int g, int h) __attribute__((always_inline)) {
    if constexpr (TB) return frag_k(WBc{}, r * G::REGION + G::A_BYTES, b0o + g * 16, h);
    else return *(const bf16x8*)(smem + r * G::REGION + G::A_BYTES + (b0o + g * 16) * 128 + (h ? lofs1 : lofs0));
  };

  f32x4 acc[FM][FN];
  bf16x8 fa[2][FM], fb[FN];

#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(0, i, 0);
#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(1, i, 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::G) : "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int f = 0; f < FM; ++f) fa[0][f] = fragA(0, f, 0);
#pragma unroll
  for (int g = 0; g < FN; ++g) fb[g] = fragB(0, g, 0);

  // ---- epilogue pieces ------------------------------------------------------------------------------
  const int csub = ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;  // the lane's 8 columns in a 32-col pair
  const unsigned long long cbytes = (unsigned long long)M * (unsigned long long)ldc * sizeof(TC) +
                                    (unsigned long long)(splits - 1) * (unsigned)slab_bytes;
  const auto rsC = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)(unsigned)cbytes, 0x00020000);
  int cslab = 0;  // byte offset of the current item's partial slab
  const auto rsP = __builtin_amdgcn_make_buffer_rsrc((EPI == 1 || EPI == 3) ? ep.C2 : (void*)C, 0,
                                                     (int)(unsigned)((EPI == 1 || EPI == 3) ? 2ull * M * ldc : cbytes),
                                                     0x00020000);
  float cs[EPI == 3 ? FN / 2 : 1][8];  // EPI 3: the lane's column sums over its fragment rows
  constexpr bool use_plane = EPI != 0 && DM == 2;
  const auto rsK = __builtin_amdgcn_make_buffer_rsrc((void*)(use_plane ? ep.plane : (const uint32_t*)C), 0,
                                                     (int)(unsigned)(use_plane ? (unsigned long long)M * N / 8 : 4ull),
                                                     0x00020000);
  // the 8 keep bits of a lane's segment (row, 8 columns from col, col % 8 == 0; N % 32 == 0 with a plane)
  auto keep8 = [&](bool ok, int row, int col) __attribute__((always_inline)) -> uint32_t {
    const int koff = ok ? ((row * N + (col & ~31)) >> 5) * 4 : 0x7fff8000;
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsK, koff, 0, 0) >> (col & 31);
  };
  const auto rsR = __builtin_amdgcn_make_buffer_rsrc(EPI == 2 ? (void*)ep.R : (void*)C, 0, (int)(unsigned)cbytes,
                                                     0x00020000);
  // (acc row f, pair p) -> 8 consecutive fp32 values of one output row: v[e] = alpha * acc + bias
  auto gather = [&](int f, int p, int n0, float (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][2 * p][q]),
                                                      __float_as_uint(acc[f][2 * p + 1][q]), false, false);
      v[q] = __uint_as_float(x[0]);
      v[4 + q] = __uint_as_float(x[1]);
    }
    if (has_bias) {
      f32x4 x0, x1;
      if constexpr (LDS_BIAS) {
        x0 = *(const f32x4*)(sbias + n0 + wc * (FN * 16) + p * 32 + csub);
        x1 = *(const f32x4*)(sbias + n0 + wc * (FN * 16) + p * 32 + csub + 4);
      } else {  // columns past N read zeros (buffer range)
        const int bo = (n0 + wc * (FN * 16) + p * 32 + csub) * 4;
        x0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsBias, bo, 0, 0));
        x1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsBias, bo + 16, 0, 0));
      }
      const float bv[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaf(ep.alpha, v[e], bv[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= ep.alpha;
    }
  };
  // final values of one (row, 8 columns) segment -> stores.  pk: the 8 outputs as bf16 (EPI 0 bf16 / 1 / 2)
  // or the fp32 v (EPI 0 fp32)
  // a segment's row inputs -- EPI 3: the saved pre-activation (a); EPI 2: the fp32 residual (a, b) -- loaded one
  // fragment row ahead of their use (prefetch_in)
  struct RowIn {
    u32x4 a, b;
  };
  auto load_in = [&](int row, int col) __attribute__((always_inline)) -> RowIn {
    RowIn r{};
    const bool ok = row < M && col < N;
    if constexpr (EPI == 3) {
      r.a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsP, ok ? (row * ldc + col) * 2 : 0x7fff8000, 0, 0));
    } else if constexpr (EPI == 2) {
      const int voff = ok ? (row * ldc + col) * (int)sizeof(TC) : 0x7fff8000;
      r.a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsR, voff, 0, 0));
      r.b = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsR, voff + 16, 0, 0));
    }
    return r;
  };
  // the counter hash's first word for the segment's first pair: its flat index row * N + col is a multiple of 8
  // (col % 8 == 0, N % 8 == 0), so pairs p0 + j (j < 4) differ from p0 in the low two bits only and their first
  // words are x0 ^ j (common.h drop_first)
  auto seg_hash0 = [&](int row, int col) __attribute__((always_inline)) -> uint32_t {
    return drop_first(ep.key, ((unsigned long long)row * (unsigned)N + (unsigned)col) >> 1);
  };
  // keep ? v * dscale : +0 without a branch: left to itself hipcc sank the GELU into an exec-masked block per
  // element (48 s_cbranch_execz per tile row set in the fc1 epilogue); the empty asm pins v as computed
  auto drop_sel = [&](float v, bool keep) __attribute__((always_inline)) -> float {
    float x = v * ep.dscale;
    asm volatile("" : "+v"(x));
    return keep ? x : 0.f;
  };
  // (have_in false: the deferred rows, which load their inputs here)
  auto finish = [&](int row, int col, int pi, const uint32_t (&pk)[4], const float (&v)[8], const RowIn& in_,
                    bool have_in) __attribute__((always_inline)) {
    const RowIn in = have_in ? in_ : load_in(row, col);
    const bool ok = row < M && col < N;
    const int voff = ok ? (row * ldc + col) * (int)sizeof(TC) + cslab : 0x7fff8000;
    if constexpr (EPI == 0) {
      if constexpr (sizeof(TC) == 2) {
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){pk[0], pk[1], pk[2], pk[3]}, rsC, voff, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, (f32x4){v[0], v[1], v[2], v[3]}), rsC, voff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, (f32x4){v[4], v[5], v[6], v[7]}), rsC, voff + 16, 0, 0);
      }
    } else if constexpr (EPI == 1) {
      // P stored; GELU + dropout on the bf16 P (autocast: fc1's output is bf16 before the activation)
      const int poff = ok ? (row * ldc + col) * 2 : 0x7fff8000;
      uint32_t kb = 0u;
      if constexpr (use_plane) kb = keep8(ok, row, col);
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){pk[0], pk[1], pk[2], pk[3]}, rsP, poff, 0, 0);
      const uint32_t x0 = seg_hash0(row, col);
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a0 = gelu_erf(bf_lo(pk[j])), a1 = gelu_erf(bf_hi(pk[j]));
        if constexpr (DM == 2) {
          a0 = (kb >> (2 * j)) & 1u ? a0 * ep.dscale : 0.f;
          a1 = (kb >> (2 * j + 1)) & 1u ? a1 * ep.dscale : 0.f;
        } else if constexpr (DM == 1) {
          const uint32_t h = drop_mix(x0 ^ (uint32_t)j);
          a0 = drop_sel(a0, (h & 0xFFFFu) >= ep.thresh);
          a1 = drop_sel(a1, (h >> 16) >= ep.thresh);
        }
        o[j] = pk_bf16(a0, a1);
      }
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){o[0], o[1], o[2], o[3]}, rsC, poff, 0, 0);
    } else if constexpr (EPI == 3) {
      // dA (bf16) -> dropout -> x GELU'(P) -> bf16; column sums of the stored values
      const int poff = ok ? (row * ldc + col) * 2 : 0x7fff8000;
      const u32x4 pp = in.a;
      uint32_t kb = 0u;
      if constexpr (use_plane) kb = keep8(ok, row, col);
      const uint32_t x0 = seg_hash0(row, col);
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d0 = bf_lo(pk[j]), d1 = bf_hi(pk[j]);
        if constexpr (DM == 2) {
          d0 = (kb >> (2 * j)) & 1u ? d0 * ep.dscale : 0.f;
          d1 = (kb >> (2 * j + 1)) & 1u ? d1 * ep.dscale : 0.f;
        } else if constexpr (DM == 1) {
          const uint32_t h = drop_mix(x0 ^ (uint32_t)j);
          d0 = (h & 0xFFFFu) >= ep.thresh ? d0 * ep.dscale : 0.f;
          d1 = (h >> 16) >= ep.thresh ? d1 * ep.dscale : 0.f;
        }
        o[j] = pk_bf16(d0 * gelu_erf_grad(bf_lo(pp[j])), d1 * gelu_erf_grad(bf_hi(pp[j])));
        cs[pi][2 * j] += bf_lo(o[j]);
        cs[pi][2 * j + 1] += bf_hi(o[j]);
      }
      __builtin_amdgcn_raw_buffer_store_b128((u32x4){o[0], o[1], o[2], o[3]}, rsC, poff, 0, 0);
      if (UVA_G8_DBG & 2) asm volatile("s_nop 7\n s_nop 7" ::: "memory");
    } else {
      const f32x4 r0 = __builtin_bit_cast(f32x4, in.a), r1 = __builtin_bit_cast(f32x4, in.b);
      uint32_t kb = 0u;
      if constexpr (use_plane) kb = keep8(ok, row, col);
      const uint32_t x0 = seg_hash0(row, col);
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a0 = bf_lo(pk[j]), a1 = bf_hi(pk[j]);
        if constexpr (DM == 2) {
          a0 = (kb >> (2 * j)) & 1u ? a0 * ep.dscale : 0.f;
          a1 = (kb >> (2 * j + 1)) & 1u ? a1 * ep.dscale : 0.f;
        } else if constexpr (DM == 1) {
          const uint32_t h = drop_mix(x0 ^ (uint32_t)j);
          a0 = drop_sel(a0, (h & 0xFFFFu) >= ep.thresh);
          a1 = drop_sel(a1, (h >> 16) >= ep.thresh);
        }
        o[2 * j] = a0;
        o[2 * j + 1] = a1;
      }
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, (f32x4){r0[0] + o[0], r0[1] + o[1], r0[2] + o[2], r0[3] + o[3]}), rsC, voff, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, (f32x4){r1[0] + o[4], r1[1] + o[5], r1[2] + o[6], r1[3] + o[7]}), rsC, voff + 16, 0, 0);
    }
  };
  auto seg_row = [&](int m0, int f) __attribute__((always_inline)) { return m0 + wr * (FM * 16) + f * 16 + lrow; };
  auto seg_col = [&](int n0, int p) __attribute__((always_inline)) { return n0 + wc * (FN * 16) + p * 32 + csub; };
  // immediate epilogue of one fragment row
  constexpr bool PF = EPI == 3 && UVA_G8_PREFETCH;
  auto epi_row = [&](int f, int m0, int n0, const RowIn (&in_row)[FN / 2]) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < FN / 2; ++p) {
      float v[8];
      gather(f, p, n0, v);
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pk[j] = pk_bf16(v[2 * j], v[2 * j + 1]);
      finish(seg_row(m0, f), seg_col(n0, p), p, pk, v, in_row[p], PF);
    }
  };
  // EPI 3 loads row f + 1's inputs before finishing row f (the wave otherwise sits in s_waitcnt for each
  // segment's load: SQ_WAIT_ANY 0.47 of the kernel's cycles, profiles/r06/g8w_pmc.txt; 234 vs 255 us)
  RowIn in_buf[2][FN / 2];
  auto prefetch_in = [&](int f, int m0, int n0) __attribute__((always_inline)) {
    if constexpr (PF) {
#pragma unroll
      for (int p = 0; p < FN / 2; ++p) in_buf[f & 1][p] = load_in(seg_row(m0, f), seg_col(n0, p));
    }
  };
  // deferred epilogue: the last NDEF fragment rows of a tile are packed to bf16 (every EPI form rounds there
  // first) and finished in the next tile's first even substeps; rows 0 .. FM - NDEF - 1 finish at once
  constexpr int ND = NDEF > 0 ? NDEF : 1, F0 = FM - NDEF;
  uint32_t pend[ND][FN / 2][4];
  int pm0 = 0, pn0 = 0;
  bool have_pend = false;
  auto pack_def = [&](int n0) __attribute__((always_inline)) {
    if constexpr (NDEF > 0) {
#pragma unroll
      for (int d = 0; d < NDEF; ++d)
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) {
          float v[8];
          gather(F0 + d, p, n0, v);
#pragma unroll
          for (int j = 0; j < 4; ++j) pend[d][p][j] = pk_bf16(v[2 * j], v[2 * j + 1]);
        }
    }
  };
  auto pend_row = [&](int d) __attribute__((always_inline)) {
    if constexpr (NDEF > 0) {
#pragma unroll
      for (int p = 0; p < FN / 2; ++p) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] = bf_lo(pend[d][p][j]);
          v[2 * j + 1] = bf_hi(pend[d][p][j]);
        }
        finish(seg_row(pm0, F0 + d), seg_col(pn0, p), p, pend[d][p], v, in_buf[0][0], false);
      }
    }
  };
  // stores per fragment row, and of the rows finished at a tile's end
  constexpr int SPR = (FN / 2) * (sizeof(TC) == 2 ? 1 : 2) * (EPI == 1 ? 2 : 1);
  constexpr int EIMM = F0 * SPR + (EPI == 3 ? FN : 0);
  static_assert(E == FM * SPR + (EPI == 3 ? FN : 0), "store count");
  static_assert(EPI != 3 || NDEF == 0, "EPI 3 finishes every row at the tile end (its column sums)");

  // one substep (as gemm_4w).  U: 0 / 2 even (regions 0 / 1), 1 / 3 odd; ZERO: first substep of an item;
  // post (odd substeps): which stores younger than the awaited DMA may stay in flight at the RAW wait --
  // bit 0 a tile end's immediate rows (EIMM), bit 1 one deferred row (SPR); kt: the K-tile an odd substep
  // refills its region with; ed: deferred row finished after this (even) substep's MFMAs (-1: none)
  auto substep = [&](auto UC, auto ZC, int post, int kt, int ed) __attribute__((always_inline)) {
    constexpr int u = decltype(UC)::value;
    constexpr bool ZERO = decltype(ZC)::value;
    constexpr bool ODD = (u & 1) != 0;
    constexpr int r = u >> 1, b = u & 1;
    constexpr int rn = ODD ? (r ^ 1) : r, hn = ODD ? 0 : 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (ODD) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mi = 0; mi < NM; ++mi) {
      // column-major MFMA order: B fragment g is dead after its column (FM MFMAs), so the B fragments are
      // single-buffered (re-read for the next substep right after their column); A fragments double-buffered
      const int g = mi / FM, f = mi % FM;
      if (ODD && mi == RAW_AT) {
        // the refill DMAs issued so far, and the epilogue stores younger than the awaited DMA, may stay in
        // flight (vmcnt counts both, in issue order)
        constexpr int W0 = NB, W1 = NB + EIMM > 63 ? 63 : NB + EIMM, W2 = NB + SPR > 63 ? 63 : NB + SPR,
                      W3 = NB + EIMM + SPR > 63 ? 63 : NB + EIMM + SPR;
        if (post == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W0) : "memory");
        else if (post == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W1) : "memory");
        else if (post == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W2) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(W3) : "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (ZERO)
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[g], fa[b][f], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      else
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[g], fa[b][f], acc[f][g], 0, 0, 0);
      if constexpr (ODD) {
        const int di = (mi * G::G + DS - 1) / DS;
        if (di < G::G && (di * DS) / G::G == mi) dma_one(r, di < G::G ? di : 0, kt);
      }
      // next substep's fragments: A row f' at ODD ? RAW_AT + 2 f' : 2 f' + 1; B column g' after its last
      // use (mi = FM g' + FM - 1), in odd substeps not before the RAW barrier
#pragma unroll
      for (int q = 0; q < FM; ++q)
        if (mi == (ODD ? RAW_AT + 2 * q : 2 * q + 1)) fa[b ^ 1][q] = fragA(rn, q, hn);
#pragma unroll
      for (int q = 0; q < FN; ++q) {
        const int at0 = FM * q + FM - 1, at1 = RAW_AT + 1 + 2 * q;
        if (mi == (ODD ? (at0 > at1 ? at0 : at1) : at0)) fb[q] = fragB(rn, q, hn);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NDEF > 0 && !ODD) {
      if (ed >= 0) {
#pragma unroll
        for (int d = 0; d < NDEF; ++d)
          if (d == ed) pend_row(d);
      }
    }
  };
  using U0 = std::integral_constant<int, 0>;
  using U1 = std::integral_constant<int, 1>;
  using U2 = std::integral_constant<int, 2>;
  using U3 = std::integral_constant<int, 3>;
  using ZT = std::integral_constant<bool, true>;
  using ZF = std::integral_constant<bool, false>;
  // two K-tiles; imm: its first odd substep follows a tile end's immediate rows; e0 / e1: deferred rows
  // finished after its two even substeps (-1: none)
  auto group = [&](auto ZC, bool imm, int kt0, int e0, int e1) __attribute__((always_inline)) {
    substep(U0{}, ZC, 0, kt0, e0);
    substep(U1{}, ZF{}, (imm ? 1 : 0) | (e0 >= 0 ? 2 : 0), kt0, -1);
    substep(U2{}, ZF{}, 0, kt0 + 1, e1);
    substep(U3{}, ZF{}, e1 >= 0 ? 2 : 0, kt0 + 1, -1);
  };

  for (int ii = 0; ii < my_items; ++ii) {
    int m0, n0;
    const int t = slot + ii * grid;
    item_of(t, m0, n0);
    const int sl = t / ntiles, kb = sl * kps;
    const int nkt = (min(K, kb + kps) - kb) / 64;
    cslab = sl * slab_bytes;
    const int nxt = ii + 1 < my_items ? t + grid : t;
    const int ngroups = nkt / 2;
    const bool imm = ii > 0 && w1ok && EIMM > 0;
    int it0 = 1;
    if constexpr (NDEF > 0) {
      // the previous tile's deferred rows in the peeled groups 0 (and 1): straight-line code, the packed
      // outputs are dead in the runtime loop that follows (needs ngroups >= 3: checked by the launcher)
      if (have_pend) {
        group(ZT{}, imm, 2, 0, NDEF > 1 ? 1 : -1);
        if constexpr (NDEF > 2) group(ZF{}, false, 4, 2, NDEF > 3 ? 3 : -1);
      } else {
        group(ZT{}, imm, 2, -1, -1);
        if constexpr (NDEF > 2) group(ZF{}, false, 4, -1, -1);
      }
      it0 = NDEF > 2 ? 2 : 1;
    } else {
      group(ZT{}, imm, 2, -1, -1);
    }
    for (int it = it0; it < ngroups - 1; ++it) group(ZF{}, false, 2 * it + 2, -1, -1);
    dma_offsets(nxt);
    // (UVA_G8_PREFETCH & 2: row 0's inputs issued before the tile's last K-group, ahead of its refill DMAs:
    // older than every DMA the group's RAW waits count, so those waits only get stricter)
    if constexpr ((UVA_G8_PREFETCH & 2) != 0) prefetch_in(0, m0, n0);
    group(ZF{}, false, 0, -1, -1);
    pack_def(n0);
    if constexpr (EPI == 3) {
#pragma unroll
      for (int p = 0; p < FN / 2; ++p)
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[p][e] = 0.f;
    }
    if constexpr ((UVA_G8_PREFETCH & 2) == 0) prefetch_in(0, m0, n0);
#pragma unroll
    for (int f = 0; f < F0; ++f) {
      __builtin_amdgcn_sched_barrier(0);
      if (f + 1 < F0) prefetch_in(f + 1, m0, n0);
      epi_row(f, m0, n0, in_buf[f & 1]);
    }
    if (UVA_G8_DBG & 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (EPI == 3 && !(UVA_G8_DBG & 1)) {
      // the wave's 64-row column sums: over the 16 row lanes of each DPP row (lane & 15), stored by lane 0
      // of each row group to part[(m0 + 64 wr) / 64][col] (every wave stores: rows past M contributed zeros)
      const auto rsS = __builtin_amdgcn_make_buffer_rsrc((void*)ep.part, 0,
                                                         (int)(unsigned)(4ull * (unsigned)(tm * (G::BM / 64)) * (unsigned)N), 0x00020000);
#pragma unroll
      for (int p = 0; p < FN / 2; ++p) {
        f32x4 s0, s1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] = row16_sum(cs[p][e]);
          s1[e] = row16_sum(cs[p][4 + e]);
        }
        const int col = seg_col(n0, p);
        const int soff = (lrow == 0 && col < N) ? (((m0 >> 6) + wr) * N + col) * 4 : 0x7fff8000;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s0), rsS, soff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s1), rsS, soff + 16, 0, 0);
      }
    }
    pm0 = m0;
    pn0 = n0;
    have_pend = NDEF > 0;
    if (NDEF > 0 && !w1ok) {
      // ragged edges: the deferred rows finish here too (the next tile's RAW waits then over-wait: safe)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        __builtin_amdgcn_sched_barrier(0);
        pend_row(d);
      }
      have_pend = false;
    }
  }
  if (NDEF > 0 && have_pend) {
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      __builtin_amdgcn_sched_barrier(0);
      pend_row(d);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int g8_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

static int g_gemm8w_on = 0;        // plain products (measurement switch; the fused forms are called directly)
static int g_gemm8w_mode = 0;     // bit 1: 64 x 64 wave tiles; bits 2..4: deferred rows (64 x 64 only: 4);
                                  // bit 5 / 6: every product on two 4-wave workgroups per CU (NW = 4) / on
                                  // one 8-wave workgroup (NW = 8); neither: EPI 3 on NW = 4, the rest NW = 8
                                  // (fc2 dX + GELU' 222-232 vs 230-237 us, fc1 + GELU 247-250 vs 235-242,
                                  // profiles/r06/g8w_nw4_final.txt); bit 7: the dW products
                                  // (uva_gemm8w_tt_try)

template <int FN, int EPI, int NDEF, typename TC, int DM, int NW>
static int g8_launch1(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                     const G8Epi& ep, hipStream_t s) {
  using G = G8Cfg<4, FN, NW>;
  const int tn = (N + G::BN - 1) / G::BN;
  const long long tiles = (long long)((M + G::BM - 1) / G::BM) * tn;
  const int grid = (int)std::min<long long>(tiles, (long long)g8_cus() * (8 / NW));
  const int lds = G::RING + (NW == 8 && ep.bias ? tn * G::BN * 4 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_8w<4, FN, NW, EPI, NDEF, TC, DM>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, NW == 8 ? 163840 : G::RING);
    attr = true;
  }
  const int w1ok = (M % G::BM == 0) && (N % G::BN == 0);
  gemm_8w<4, FN, NW, EPI, NDEF, TC, DM><<<dim3(grid), 64 * NW, lds, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N,
                                                                       K, lda, ldb, ldc, ep, w1ok, 1, K, 0);
  UVA_LAUNCH_CHECK();
  return 0;
}

// dW products (A [K][M], B [K][N], K = tokens): split-K plan -- enough (tile, K-slice) items for one round of
// the chip, slices of whole 128-deep pairs, >= 256 deep each
struct G8Split {
  int splits, kps, grid;
};
static G8Split g8_plan_tt(int M, int N, int K, long long ws_floats, bool need_ws) {
  G8Split p{0, 0, 0};
  if (K % 128 != 0 || K < 256 || M < 256 || N < 192) return p;
  const int cus = g8_cus();
  const long long tiles = (long long)((M + 255) / 256) * ((N + 191) / 192);
  int splits = (int)std::max<long long>(1, (cus + tiles / 2) / tiles);
  if (splits > K / 256) splits = K / 256;
  while (splits > 1 && (long long)splits * M * N > ws_floats) --splits;
  if (splits == 1 && need_ws && (long long)M * N > ws_floats) return p;
  int kps = K;
  for (; splits > 1; --splits) {
    kps = ((K + splits - 1) / splits + 127) / 128 * 128;
    const int sp = (K + kps - 1) / kps;
    if (K - (sp - 1) * kps >= 256) {
      splits = sp;
      break;
    }
  }
  if (splits <= 1) {
    splits = 1;
    kps = K;
  }
  p.splits = splits;
  p.kps = kps;
  p.grid = (int)std::min<long long>(tiles * splits, cus);
  return p;
}
// rows of EPI 3 column-sum partials the launch writes (every wave of every row tile stores its 64 rows)
static bool g8_nw4(int epi) { return (g_gemm8w_mode & 32) || (!(g_gemm8w_mode & 64) && epi == 3); }
static int g8_part_rows(int M) { return g8_nw4(3) ? (M + 127) / 128 * 2 : (M + 255) / 256 * 4; }

// the dropout form is a template parameter (DM): none for plain products / p = 0, else hash or plane
template <int FN, int EPI, int NDEF, typename TC, int NW = 8>
static int g8_launch(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                     const G8Epi& ep, hipStream_t s) {
  if constexpr (EPI == 0) {
    return g8_launch1<FN, EPI, NDEF, TC, 0, NW>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  } else {
    if (!ep.thresh) return g8_launch1<FN, EPI, NDEF, TC, 0, NW>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    if (ep.plane) return g8_launch1<FN, EPI, NDEF, TC, 2, NW>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    return g8_launch1<FN, EPI, NDEF, TC, 1, NW>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  }
}

// deferred rows ride in the peeled groups 0 (1 .. 2 rows) and 1 (3 .. 4 rows) of the next tile, neither of
// them its last group: 2 rows need K >= 256 (two groups), 3 .. 4 rows K >= 384
template <int EPI, typename TC>
static int g8_dispatch(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                       const G8Epi& ep, hipStream_t s) {
  // built: 64 x 96 wave tiles with the immediate epilogue (the default), and 64 x 64 tiles with all four rows
  // deferred.  64 x 96 with 1-3 deferred rows spills (8-100 VGPRs: the main loop already holds ~240) and
  // 64 x 64 tiles lose 5-8 % on the plain products (profiles/r06/g8w_bench_first.txt)
  // (deferred rows are held as bf16: a plain fp32-output product finishes every row at once)
  const int nd = (EPI == 0 && sizeof(TC) == 4) ? 0 : (g_gemm8w_mode >> 2) & 7;
#define G8L(FN_, ND_) g8_launch<FN_, EPI, ND_, TC>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
  if (g_gemm8w_mode & 32) return g8_launch<6, EPI, 0, TC, 4>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  if (g_gemm8w_mode & 2) return (nd && K / 128 >= 3) ? G8L(4, 4) : G8L(4, 0);
  // 64 x 96 tiles with 1 or 2 deferred rows spill 7-50 VGPRs and measured no faster on the fused Mlp
  // epilogues (profiles/r06/g8w_dm.txt): the wide tile always finishes its rows immediately
  return G8L(6, 0);
#undef G8L
}

// shape / size conditions shared by every form: K-contiguous operands, every byte offset a 32-bit int
static bool g8_ok(const void* A, const void* B, const void* C, int M, int N, int K, long long lda, long long ldb,
                  long long ldc, int csize, const float* bias) {
  if (M < 256 || N < 192 || K < 256 || K % 128) return false;
  if (lda % 8 || ldb % 8 || ldc % 8 || N % 8 || lda < K || ldb < K) return false;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return false;
  if (bias && ((uintptr_t)bias % 16)) return false;
  if (2.0 * (double)M * (double)lda >= 2147483648.0 || 2.0 * (double)N * (double)ldb >= 2147483648.0) return false;
  if ((double)M * (double)ldc * csize > (double)0x7fff0000) return false;
  const int tn = (N + 191) / 192;
  if (tn * 192 * 4 + 114688 > 163840) return false;  // bias in LDS
  return true;
}

static uint32_t g8_key(unsigned long long seed) { return drop_key(seed); }

// the dW products on gemm_8w (mode bit 7: 128): 1 = launched: *reduce = 0 -> C holds alpha * A^T B; *reduce = s > 0
// -> ws holds s fp32 partial slabs of M x N (ld N) the caller reduces into C (alpha, beta).  0 = not eligible / off
extern "C" int uva_gemm8w_tt_try(const void* A, const void* B, float* C, int M, int N, int K, long long lda,
                                 long long ldb, long long ldc, float alpha, float beta, float* ws, long long ws_floats,
                                 int* reduce, hipStream_t s) {
  *reduce = 0;
  if (!(g_gemm8w_mode & 128)) return 0;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8 || M % 8 || N % 8 || lda < M || ldb < N) return 0;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)ws) % 16) return 0;
  if (2.0 * (double)K * (double)lda >= 2147483648.0 || 2.0 * (double)K * (double)ldb >= 2147483648.0) return 0;
  const G8Split p = g8_plan_tt(M, N, K, ws ? ws_floats : 0, beta != 0.f);
  if (p.splits == 0) return 0;
  const bool direct = p.splits == 1 && beta == 0.f;
  if (direct ? (double)M * (double)ldc * 4.0 > (double)0x7fff0000
             : (double)p.splits * (double)M * (double)N * 4.0 > (double)0x7fff0000)
    return 0;
  if (!direct && !ws) return 0;
  using G = G8Cfg<4, 6, 8>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_8w<4, 6, 8, 0, 0, float, 0, 1, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  const int w1ok = (M % G::BM == 0) && (N % G::BN == 0);
  G8Epi ep{nullptr, direct ? alpha : 1.f, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 1.f};
  gemm_8w<4, 6, 8, 0, 0, float, 0, 1, 1><<<dim3(p.grid), 512, G::RING, s>>>(
      (const bf16*)A, (const bf16*)B, direct ? C : ws, M, N, K, (int)lda, (int)ldb, direct ? (int)ldc : N, ep, w1ok,
      p.splits, p.kps, (int)((long long)M * N * 4));
  UVA_LAUNCH_CHECK();
  if (!direct) *reduce = p.splits;
  return 1;
}

// plain product (measurement route): 1 = launched, 0 = not eligible / off, < 0 = -hipError
extern "C" int uva_gemm8w_try(int out_dtype, const void* A, const void* B, void* C, int M, int N, int K, long long lda,
                              long long ldb, long long ldc, const float* bias, float alpha, hipStream_t s) {
  if (!g_gemm8w_on) return 0;
  if (!g8_ok(A, B, C, M, N, K, lda, ldb, ldc, out_dtype == UVA_DT_BF16 ? 2 : 4, bias)) return 0;
  G8Epi ep{bias, alpha, nullptr, nullptr, nullptr, nullptr, 0u, 0u, 1.f};
  const int r = out_dtype == UVA_DT_BF16
                    ? g8_dispatch<0, bf16>(A, B, C, M, N, K, (int)lda, (int)ldb, (int)ldc, ep, s)
                    : g8_dispatch<0, float>(A, B, C, M, N, K, (int)lda, (int)ldb, (int)ldc, ep, s);
  return r ? -r : 1;
}

// measurement switches (tests / tools): on = route plain K-contiguous products here; mode as
// g_gemm8w_mode.  Return the previous on | mode << 1; -2 leaves a value.
extern "C" int uva_gemm8w_set(int on, int mode) {
  const int prev = g_gemm8w_on | (g_gemm8w_mode << 1);
  if (on != -2) g_gemm8w_on = on;
  if (mode != -2) g_gemm8w_mode = mode;
  return prev;
}

// timm Mlp fc1 forward, fused: pre = bf16(x W^T + b) -> pre_out; out = bf16(drop(gelu(pre))).
// 1 = launched, 0 = not eligible, < 0 = -hipError
extern "C" int uva_linear_gelu_drop(const void* X, const void* W, const float* bias, void* pre_out, void* out, int M,
                                    int N, int K, float drop_p, unsigned long long seed, const void* plane,
                                    hipStream_t s) {
  if (!g8_ok(X, W, out, M, N, K, K, K, N, 2, bias) || ((uintptr_t)pre_out % 16)) return 0;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  if (plane && (N % 32 || !th || ((uintptr_t)plane % 4))) return (int)-hipErrorInvalidValue;
  G8Epi ep{bias, 1.f, pre_out, nullptr, nullptr, (const uint32_t*)plane, th ? g8_key(seed) : 0u, th, ds};
  const int r = g8_dispatch<1, bf16>(X, W, out, M, N, K, K, K, N, ep, s);
  return r ? -r : 1;
}

int uva_colsum_final_launch(const float* part, int nrows, int cols, float* out, int accum, hipStream_t s);

// timm Mlp backward through fc2 -> dropout -> GELU, fused into the fc2 dX product (EPI 3):
// dpre = bf16(gelu'(pre) * drop(bf16(dY Wt^T))), dbias (+)= column sums of dpre (the fc1 bias gradient).
// dY [M][K] bf16, Wt [N][K] (fc2's transposed weight copy), pre / dpre [M][N] bf16; part: (M / 256 + 1) * 4 * N
// floats of workspace.  1 = launched, 0 = not eligible, < 0 = -hipError
extern "C" int uva_linear_dgelu_drop(const void* dY, const void* Wt, const void* pre, void* dpre, float* dbias,
                                     int accum_bias, float* part, int M, int N, int K, float drop_p,
                                     unsigned long long seed, const void* plane, hipStream_t s) {
  if (!g8_ok(dY, Wt, dpre, M, N, K, K, K, N, 2, nullptr) || (((uintptr_t)pre | (uintptr_t)part) % 16) || !dbias)
    return 0;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  if (plane && (N % 32 || !th || ((uintptr_t)plane % 4))) return (int)-hipErrorInvalidValue;
  G8Epi ep{nullptr, 1.f, (void*)pre, nullptr, part, (const uint32_t*)plane, th ? g8_key(seed) : 0u, th, ds};
  int r = g8_nw4(3) ? g8_launch<6, 3, 0, bf16, 4>(dY, Wt, dpre, M, N, K, K, K, N, ep, s)
                                : g8_launch<6, 3, 0, bf16>(dY, Wt, dpre, M, N, K, K, K, N, ep, s);
  if (r) return -r;
  r = uva_colsum_final_launch(part, g8_part_rows(M), N, dbias, accum_bias, s);
  return r ? -r : 1;
}

// timm Mlp fc2 / attention proj forward, fused: out (fp32) = R + drop(bf16(x W^T + b)).
extern "C" int uva_linear_drop_res(const void* X, const void* W, const float* bias, const float* R, float* out, int M,
                                   int N, int K, float drop_p, unsigned long long seed, const void* plane,
                                   hipStream_t s) {
  if (!g8_ok(X, W, out, M, N, K, K, K, N, 4, bias) || ((uintptr_t)R % 16)) return 0;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  if (plane && (N % 32 || !th || ((uintptr_t)plane % 4))) return (int)-hipErrorInvalidValue;
  G8Epi ep{bias, 1.f, nullptr, R, nullptr, (const uint32_t*)plane, th ? g8_key(seed) : 0u, th, ds};
  const int r = g8_dispatch<2, float>(X, W, out, M, N, K, K, K, N, ep, s);
  return r ? -r : 1;
}
