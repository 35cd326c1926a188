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

#include <algorithm>
#include <type_traits>

// diagnostic builds only (tools/build_variant.py gemm4.hip -DUVA_G4_DIAG=n; results are WRONG): bit 1 no
// DMA inside the K loop, 2 no wait / barrier, 4 no epilogue stores, 8 no fragment reads inside the K loop,
// 16 every tile stores to the first tile's location, 32 every K-tile reads the item's first K-tile
#ifndef UVA_G4_DIAG
#define UVA_G4_DIAG 0
#endif
// the odd substep's refill DMAs spread over its first UVA_G4_SPREAD MFMAs of the K-contiguous products
// (0: one after each of the first G MFMAs).  Measured (tools/gemm4_bench.py, profiles/r05/gemm4_diag.txt):
// spreading over the whole substep is 5-8 % faster on the forward / dX products (the DMA queue drains
// under MFMAs instead of stalling the issuing wave); the dW products (k-major operands) keep the early
// burst -- their loads' latency is long enough that issuing later costs 2.5x
#ifndef UVA_G4_SPREAD
#define UVA_G4_SPREAD 48
#endif
#ifndef UVA_G4_ROT
#define UVA_G4_ROT 0
#endif
#ifndef UVA_G4_TBLK
#define UVA_G4_TBLK 0
#endif


typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

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

// 16-B chunk swizzle of a k-major image row [64 k][W] (T = 1 operands), chosen so that the 8 rows
// {8g + q} a 32-lane group of ds_read_b64_tr_b16 touches (32 B each) fall on 8 distinct 32-B bank
// slots: 512-B rows (W = 256) all start on one bank -> XOR by 8 distinct even chunk offsets; 384-B rows
// (W = 192) alternate between two bank halves -> 4 offsets within 128 B suffice (and keep the XOR
// inside each 8-chunk group of the 24-chunk row)
template <int W>
__device__ __forceinline__ int g4_kswz(int k) {
  static_assert(W == 256 || W == 192, "row width");
  if constexpr (W == 256) return ((k & 3) << 1) | (((k >> 3) & 1) << 3);
  else return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2);
}

}  // namespace

// TA / TB: 0 = K-contiguous operand (A [M][K], B [N][K]); 1 = M- / N-contiguous (A [K][M], B [K][N]: the
// dW products, mar_con_unified.py Block backward).  SPLIT: work items are (tile, K-slice) pairs writing
// fp32 partial slabs C + slice * slab (reduced afterwards by splitk_reduce, which applies alpha / beta).
template <int FM, int FN, int TA, int TB, typename TC>
__global__ __launch_bounds__(256, 1) void gemm_4w(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  TC* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                  long long ldc, const float* __restrict__ bias, float alpha,
                                                  int w1ok, int splits, int kps, long long slab) {
  using G = G4Cfg<FM, FN>;
  constexpr int E = FM * (FN / 2) * (sizeof(TC) == 2 ? 1 : 2);  // epilogue stores per thread per item
  // the odd substep's RAW point (MFMA index)
  constexpr int RAW_AT = G::G + 2;
  // refill DMA i follows MFMA (i * DS) / G of the odd substep; NB of them precede the RAW wait
  constexpr int DS = (UVA_G4_SPREAD && !TA && !TB) ? (UVA_G4_SPREAD < FM * FN ? UVA_G4_SPREAD : FM * FN) : G::G;
  constexpr int NB = (RAW_AT * G::G + DS - 1) / DS < G::G ? (RAW_AT * G::G + DS - 1) / DS : G::G;
  constexpr int WGE = (NB + E) > 63 ? 63 : (NB + E);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wr = w >> 1, wc = w & 1;
  const int tm = (M + G::BM - 1) / G::BM, tn = (N + G::BN - 1) / G::BN, ntiles = tm * tn;
  const int nitems = ntiles * splits;
  const int grid = gridDim.x;
  const int slot = g4_xcd_remap(blockIdx.x, grid);
  if (slot >= nitems) return;
  const int my_items = (nitems - slot + grid - 1) / grid;

  // bias -> LDS (fp32, tn * BN entries, zero past N), before any DMA is in flight
  float* sbias = (float*)(smem + G::RING);
  const bool has_bias = bias != nullptr;
  if (has_bias) {
    for (int i = threadIdx.x; i < tn * G::BN; i += 256) sbias[i] = i < N ? bias[i] : 0.f;
    __syncthreads();
  }

  // item pid -> (tile: GROUP-8 raster, K-slice); slices are the slow index (concurrent items share one
  // K range, so neighbouring tiles share operand rows in L2)
  constexpr int GROUP = 8;
  auto item_of = [&](int pid, int& m0, int& n0, int& kb, int& nkt, int& t) __attribute__((always_inline)) {
    const int sl = pid / ntiles;
    t = pid - sl * ntiles;
    const int group = t / (GROUP * tn), first_m = group * GROUP;
    const int gsz = min(tm - first_m, GROUP);
    m0 = (first_m + (t % (GROUP * tn)) % gsz) * G::BM;
    n0 = ((t % (GROUP * tn)) / gsz) * G::BN;
    kb = sl * kps;
    nkt = (min(K, kb + kps) - kb) / 64;
  };

  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)A, 0, (int)(unsigned)min(2ull * (unsigned long long)(TA ? K : M) * (unsigned)lda, 0xffffffffull), 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)B, 0, (int)(unsigned)min(2ull * (unsigned long long)(TB ? K : N) * (unsigned)ldb, 0xffffffffull), 0x00020000);
  // per-lane source offsets of the DMA target item.  T = 0: instruction i of wave w covers image rows
  // 8 (w G + i) .. +7 of 128 B; lane l: row (l >> 3), LDS chunk (l & 7) <- global chunk (l & 7) ^ (row & 7).
  // T = 1: the k-major image [64][W] taken 1 KB per instruction in byte order; lane l of instruction j:
  // byte j KB + 16 l -> (k, chunk), global chunk = chunk ^ kswz(k).  The K-tile step is the soffset
  // (128 B for T = 0, 64 rows of ld for T = 1).
  auto lane_src = [&](auto TC_, auto WC, int i, int gi, int ld) __attribute__((always_inline)) -> unsigned {
    constexpr int T = decltype(TC_)::value, W = decltype(WC)::value;
    if constexpr (T == 0) {
      const int row = 8 * (w * gi + i) + (lane >> 3);
      return (unsigned)row * (unsigned)ld * 2u + (unsigned)(((lane & 7) ^ (row & 7)) * 16);
    } else {
#if UVA_G4_TBLK
      // blocked image [W / 64][64 k][64 cols]: instruction j = 8 k-rows x 128 B of one 64-col block
      const int j = w * gi + i, k = 8 * (j & 7) + (lane >> 3);
      return (unsigned)k * (unsigned)ld * 2u + (unsigned)((j >> 3) * 128 + (((lane & 7) ^ g4_kswz<192>(k)) * 16));
#else
      const int b = (w * gi + i) * 1024 + lane * 16;
      const int k = b / (W * 2), c = (b % (W * 2)) >> 4;
      return (unsigned)k * (unsigned)ld * 2u + (unsigned)((c ^ g4_kswz<W>(k)) * 16);
#endif
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using WAc = std::integral_constant<int, G::BM>;
  using WBc = std::integral_constant<int, G::BN>;
  unsigned offA[G::GA], offB[G::GB];
  int rot_o = 0, nkt_o = 0;  // the offsets' item: K-tile rotation, K-tile count
  auto dma_offsets = [&](int pid) __attribute__((always_inline)) {
    int m0, n0, kb, nkt, t;
    item_of(pid, m0, n0, kb, nkt, t);
    nkt_o = nkt;
    rot_o = UVA_G4_ROT ? ((t % (UVA_G4_ROT > 0 ? UVA_G4_ROT : 1)) * 2) % nkt : 0;
    // the item's origin (uniform): T = 0 rows m0, column kb; T = 1 row kb, column m0
    const unsigned a0 = (unsigned)__builtin_amdgcn_readfirstlane(TA ? (kb * lda + m0) * 2 : (m0 * lda + kb) * 2);
    const unsigned b0 = (unsigned)__builtin_amdgcn_readfirstlane(TB ? (kb * ldb + n0) * 2 : (n0 * ldb + kb) * 2);
#pragma unroll
    for (int i = 0; i < G::GA; ++i)
      offA[i] = a0 + (TA ? lane_src(I1{}, WAc{}, i, G::GA, lda) : lane_src(I0{}, WAc{}, i, G::GA, lda));
#pragma unroll
    for (int i = 0; i < G::GB; ++i)
      offB[i] = b0 + (TB ? lane_src(I1{}, WBc{}, i, G::GB, ldb) : lane_src(I0{}, WBc{}, i, G::GB, ldb));
  };
#if UVA_G4_DIAG & 32
  // timing only: every K-tile re-reads the item's first K-tile (operands resident in L2)
  const int stepA = 0, stepB = 0;
#else
  const int stepA = TA ? 64 * lda * 2 : 128, stepB = TB ? 64 * ldb * 2 : 128;  // bytes per K-tile
#endif
  // DMA instruction i (A first) of K-tile kt of the offsets' item into region r
  auto dma_one = [&](int r, int i, int kt) __attribute__((always_inline)) {
    if (i < G::GA)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsA, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + (w * G::GA + i) * 1024), 16,
          (int)offA[i < G::GA ? i : 0], __builtin_amdgcn_readfirstlane(kt * stepA), 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(smem + r * G::REGION + G::A_BYTES + (w * G::GB + i - G::GA) * 1024),
          16, (int)offB[i < G::GA ? 0 : i - G::GA], __builtin_amdgcn_readfirstlane(kt * stepB), 0, 0);
  };
  dma_offsets(slot);
  auto kphys = [&](int kt) __attribute__((always_inline)) {
    const int k = kt + rot_o;
    return k >= nkt_o ? k - nkt_o : k;
  };

  // fragment reads of 16 rows (m or n) x 32 k, half h of a K-tile.  T = 0: row (lane & 15), 16-B chunk
  // h*4 + (lane >> 4) of a 128-B row (XOR row & 7).  T = 1: two ds_read_b64_tr_b16 of the k-major image
  // (rows k and k + 4 of the lane's quad, 4 columns each), the hardware transpose gathering the lane's
  // 8 consecutive k (as gemm_8ph's frag8)
  const int lrow = lane & 15;
  const int lofs0 = lrow * 128 + ((((lane >> 4)) ^ (lrow & 7)) << 4);
  const int lofs1 = lrow * 128 + (((4 + (lane >> 4)) ^ (lrow & 7)) << 4);
  const int a0o = wr * (FM * 16), b0o = wc * (FN * 16);  // first row (T = 0) / column (T = 1) of the wave
  auto frag = [&](auto TC_, auto WC, int base, int r0, int h) __attribute__((always_inline)) -> bf16x8 {
    constexpr int T = decltype(TC_)::value, W = decltype(WC)::value;
    if constexpr (T == 0) {
      return *(const bf16x8*)(smem + base + r0 * 128 + (h ? lofs1 : lofs0));
    } else {
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      const int k = h * 32 + g * 8 + q;
      const int col = r0 + 4 * p;
      const int c = col >> 3, o = (col & 7) * 2;
#if UVA_G4_TBLK
      const char* a0 = smem + base + (c >> 3) * 8192 + k * 128 + (((c & 7) ^ g4_kswz<192>(k)) << 4) + o;
      const char* a1 = smem + base + (c >> 3) * 8192 + (k + 4) * 128 + (((c & 7) ^ g4_kswz<192>(k + 4)) << 4) + o;
#else
      const char* a0 = smem + base + k * W * 2 + ((c ^ g4_kswz<W>(k)) << 4) + o;
      const char* a1 = smem + base + (k + 4) * W * 2 + ((c ^ g4_kswz<W>(k + 4)) << 4) + o;
#endif
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, v);
    }
  };
  auto fragA = [&](int r, int f, int h) __attribute__((always_inline)) {
    return TA ? frag(I1{}, WAc{}, r * G::REGION, a0o + f * 16, h) : frag(I0{}, WAc{}, r * G::REGION, a0o + f * 16, h);
  };
  auto fragB = [&](int r, int g, int h) __attribute__((always_inline)) {
    return TB ? frag(I1{}, WBc{}, r * G::REGION + G::A_BYTES, b0o + g * 16, h)
              : frag(I0{}, WBc{}, r * G::REGION + G::A_BYTES, b0o + g * 16, h);
  };

  f32x4 acc[FM][FN];
  bf16x8 fa[2][FM], fb[2][FN];

  // prologue: K-tiles 0 and 1 into regions 0 and 1, wait for region 0, read substep 0's fragments
#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(0, i, kphys(0));
#pragma unroll
  for (int i = 0; i < G::G; ++i) dma_one(1, i, kphys(1));
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::G) : "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int f = 0; f < FM; ++f) fa[0][f] = fragA(0, f, 0);
#pragma unroll
  for (int g = 0; g < FN; ++g) fb[0][g] = fragB(0, g, 0);

  // ---- register epilogue, one 16-row fragment row at a time: 8 consecutive columns per lane per
  // fragment pair (v_permlane16_swap), + bias (LDS copy), cvt, one 16-B store per pair
  const int csub = ((lane >> 4) & 1) * 16 + (lane >> 5) * 8;  // the lane's 8 columns in a 32-col pair
  auto epi_bias = [&](int n0, float (&bv)[FN / 2][8]) __attribute__((always_inline)) {
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
  };
  // stores go through a buffer descriptor: a masked-off segment (row / column past the edge) gets an
  // offset beyond the range and is dropped by the hardware -- no exec-mask branch, and every wave issues
  // the same number of stores (the vmcnt counts rely on it)
  const unsigned long long cbytes = (unsigned long long)M * (unsigned long long)ldc * sizeof(TC) +
                                    (unsigned long long)(splits - 1) * (unsigned long long)slab * sizeof(TC);
  const auto rsC = __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (int)(unsigned)min(cbytes, 0x7fff0000ull), 0x00020000);
  auto epi_row = [&](int f, int m0, int n0, long long cofs, const float (&bv)[FN / 2][8]) __attribute__((always_inline)) {
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
      const bool ok = (UVA_G4_DIAG & 4) ? alpha == 12345.f : (row < M && col < N);
#if UVA_G4_DIAG & 16
      // timing only: every tile writes the first tile's location (no HBM write traffic, the same stores)
      const int voff = (int)(((unsigned)(row % G::BM) * (unsigned)ldc + (unsigned)(col % G::BN)) * (unsigned)sizeof(TC));
#else
      const int voff = ok ? (int)((cofs + (long long)row * ldc + col) * (long long)sizeof(TC)) : 0x7fff8000;
#endif
      if constexpr (sizeof(TC) == 2) {
        bf16x8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) ov[e] = (bf16)fmaf(alpha, v[e], bv[p][e]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ov), rsC, voff, 0, 0);
      } else {
        f32x4 o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o0[e] = fmaf(alpha, v[e], bv[p][e]);
          o1[e] = fmaf(alpha, v[4 + e], bv[p][4 + e]);
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o0), rsC, voff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o1), rsC, voff + 16, 0, 0);
      }
    }
  };

  // one substep.  U: 0 / 2 even (regions 0 / 1), 1 / 3 odd; ZERO: first substep of an item (MFMAs start
  // from the inline constant 0); post: first odd substep after an epilogue (its stores are younger than
  // the awaited DMA); kt: the K-tile an odd substep refills its region with (of the offsets' item)
  auto substep = [&](auto UC, auto ZC, bool post, int kt) __attribute__((always_inline)) {
    constexpr int u = decltype(UC)::value;
    constexpr bool ZERO = decltype(ZC)::value;
    constexpr bool ODD = (u & 1) != 0;
    constexpr int r = u >> 1, b = u & 1;
    // the fragments read during this substep: odd half of this region (even substep) / even half of
    // the other region (odd substep)
    constexpr int rn = ODD ? (r ^ 1) : r, hn = ODD ? 0 : 1;
    // odd substep: a WAR barrier first (every wave is past its reads of region r: the refill may
    // start), the refill's G DMAs among the first MFMAs, then -- RAW_AT MFMAs in, to give the other
    // region's DMA (issued one K-tile earlier) that much more time to land -- the RAW wait and barrier
    // before the first read of the other region
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (ODD && !(UVA_G4_DIAG & 2)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    constexpr int NM = FM * FN, NR = FM + FN;
    // odd: one DMA after each of the first G MFMAs, from RAW_AT one read after every second MFMA;
    // even: one read after every third MFMA
    constexpr int RS = ODD ? RAW_AT : 0, RP = ODD ? 2 : 3;
    static_assert(!ODD || (RAW_AT + 2 * (NR - 1) < NM && DS <= NM && DS >= G::G), "schedule");
#pragma unroll
    for (int mi = 0; mi < NM; ++mi) {
      const int f = mi / FN, g = mi % FN;
      if (ODD && mi == RAW_AT) {
        if constexpr (!(UVA_G4_DIAG & 2)) {
          // the G refill DMAs (and an epilogue's E stores before them) may stay in flight
          if (post) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WGE) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB) : "memory");
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (ZERO)
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b][g], fa[b][f], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      else
        acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b][g], fa[b][f], acc[f][g], 0, 0, 0);
      if constexpr (ODD && !(UVA_G4_DIAG & 1)) {
        const int di = (mi * G::G + DS - 1) / DS;  // the DMA (if any) issued after this MFMA
        if (di < G::G && (di * DS) / G::G == mi) dma_one(r, di < G::G ? di : 0, kt);
      }
      if (mi >= RS && (mi - RS) % RP == 0 && (mi - RS) / RP < NR) {
        const int ri = (mi - RS) / RP;
        if constexpr (!(UVA_G4_DIAG & 8)) {
          if (ri < FM) fa[b ^ 1][ri < FM ? ri : 0] = fragA(rn, ri < FM ? ri : 0, hn);
          else fb[b ^ 1][ri < FM ? 0 : ri - FM] = fragB(rn, ri < FM ? 0 : ri - FM, hn);
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
  // two K-tiles (regions 0, 1); their odd substeps refill with K-tiles kt0 and kt0 + 1 of the offsets' item
  auto group = [&](auto ZC, bool post, int kt0) __attribute__((always_inline)) {
    const int ka = UVA_G4_ROT ? kphys(kt0) : kt0, kb = UVA_G4_ROT ? kphys(kt0 + 1) : kt0 + 1;
    substep(U0{}, ZC, false, ka);
    substep(U1{}, ZF{}, post, ka);
    substep(U2{}, ZF{}, false, kb);
    substep(U3{}, ZF{}, false, kb);
  };

  for (int ii = 0; ii < my_items; ++ii) {
    int m0, n0, kb, nkt, t;
    item_of(slot + ii * grid, m0, n0, kb, nkt, t);
    const int sl = (slot + ii * grid) / ntiles;
    const bool post = ii > 0 && w1ok;
    // the K-tile stream is two ahead: the last group's refills load the NEXT item's K-tiles 0 and 1
    // (past the last item: this item's again -- valid addresses, never read)
    const int nxt = ii + 1 < my_items ? slot + (ii + 1) * grid : slot + ii * grid;
    const int ngroups = nkt / 2;
    group(ZT{}, post, 2);  // (every item has >= 4 K-tiles: checked by the launcher)
    for (int it = 1; it < ngroups - 1; ++it) group(ZF{}, false, 2 * it + 2);
    dma_offsets(nxt);
    group(ZF{}, false, 0);
    float bv[FN / 2][8];
    epi_bias(n0, bv);
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      __builtin_amdgcn_sched_barrier(0);  // one fragment row at a time (bounds the AGPR -> VGPR reads in flight)
      epi_row(f, m0, n0, (long long)sl * slab, bv);
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

// -1 = automatic; otherwise the configuration index (1: 256 x 192)
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

template <int FM, int FN, int TA, int TB, typename TC>
static int g4_launch(const void* A, const void* B, void* C, int M, int N, int K, long long lda, long long ldb,
                     long long ldc, const float* bias, float alpha, int grid, int splits, int kps, long long slab,
                     hipStream_t s) {
  using G = G4Cfg<FM, FN>;
  const int tn = (N + G::BN - 1) / G::BN;
  const int lds = G::RING + (bias ? tn * G::BN * 4 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_4w<FM, FN, TA, TB, TC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              163840);
    attr = true;
  }
  const int w1ok = (M % G::BM == 0) && (N % G::BN == 0);
  gemm_4w<FM, FN, TA, TB, TC><<<dim3(grid), 256, lds, s>>>((const bf16*)A, (const bf16*)B, (TC*)C, M, N, K, (int)lda,
                                                           (int)ldb, ldc, bias, alpha, w1ok, splits, kps, slab);
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
  // every byte offset the kernel forms (operand origins, lane offsets, the K-step soffset, the C store
  // offset) is a 32-bit int and the C descriptor's range is clamped to 0x7fff0000: larger operands or
  // outputs go to gemm_8ph
  if (2.0 * (double)M * (double)lda >= 2147483648.0 || 2.0 * (double)N * (double)ldb >= 2147483648.0) return 0;
  if ((double)M * (double)ldc * (out_dtype == UVA_DT_BF16 ? 2.0 : 4.0) > (double)0x7fff0000) return 0;
  if (bias && ((uintptr_t)bias % 16)) return 0;
  const G4Choice c = g4_plan(M, N, K);
  if (c.cfg < 0) return 0;
  int r;
  if (out_dtype == UVA_DT_BF16) {
    r = g4_launch<8, 6, 0, 0, bf16>(A, B, C, M, N, K, lda, ldb, ldc, bias, alpha, c.grid, 1, K, 0, s);
  } else {
    r = g4_launch<8, 6, 0, 0, float>(A, B, C, M, N, K, lda, ldb, ldc, bias, alpha, c.grid, 1, K, 0, s);
  }
  return r ? -r : 1;
}

// dW products (A [K][M], B [K][N], both M- / N-contiguous; K = tokens): split-K plan -- enough (tile,
// K-slice) items for one round of the chip, slices of whole 128-deep pairs, >= 4 K-tiles each
struct G4Split {
  int splits, kps, grid;
};
static G4Split g4_plan_tt(int M, int N, int K, long long ws_floats, bool need_ws) {
  G4Split p{0, 0, 0};
  if (K % 128 != 0 || K < 256 || M < 256 || N < 192) return p;
  const int cus = g4_cus();
  const long long tiles = (long long)((M + 255) / 256) * ((N + 191) / 192);
  // measured against gemm_8ph (tools/gemm4_bench.py dw): ahead on 768 x 768 (12 tiles, 20 slices:
  // 62 vs 68 us at 32768 tokens), level on 2304 x 768, 20-25 % behind on 3072 x 768 / 768 x 3072 (the
  // k-major loads' latency: a 4-wave CU cannot keep enough of them in flight) -- few-tile products only
  if (tiles > 16) return p;
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

// 1 = launched: *reduce = 0 -> C holds alpha * A^T B; *reduce = s > 0 -> ws holds s fp32 partial slabs of
// M x N (ld N), the caller reduces them into C (alpha, beta).  0 = not eligible, < 0 = -hipError
extern "C" int uva_gemm4_tt_try(const void* A, const void* B, float* C, int M, int N, int K, long long lda,
                                long long ldb, long long ldc, float alpha, float beta, float* ws, long long ws_floats,
                                int* reduce, hipStream_t s) {
  *reduce = 0;
  if (!g_gemm4_on) return 0;
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if (lda % 8 || ldb % 8 || ldc % 8 || M % 8 || N % 8 || lda < M || ldb < N) return 0;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)ws) % 16) return 0;
  if (2.0 * (double)K * (double)lda >= 2147483648.0 || 2.0 * (double)K * (double)ldb >= 2147483648.0) return 0;
  const G4Split p = g4_plan_tt(M, N, K, ws ? ws_floats : 0, beta != 0.f);
  if (p.splits == 0) return 0;
  // the C (or slab workspace) byte range must fit the store descriptor (see uva_gemm4_try)
  if (p.splits == 1 && beta == 0.f ? (double)M * (double)ldc * 4.0 > (double)0x7fff0000
                                   : (double)p.splits * (double)M * (double)N * 4.0 > (double)0x7fff0000)
    return 0;
  int r;
  if (p.splits == 1 && beta == 0.f) {
    r = g4_launch<8, 6, 1, 1, float>(A, B, C, M, N, K, lda, ldb, ldc, nullptr, alpha, p.grid, 1, K, 0, s);
  } else {
    if (!ws) return 0;
    r = g4_launch<8, 6, 1, 1, float>(A, B, ws, M, N, K, lda, ldb, N, nullptr, 1.f, p.grid, p.splits, p.kps,
                                     (long long)M * N, s);
    *reduce = p.splits;
  }
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

extern "C" long long uva_gemm4_plan_tt(int M, int N, int K, long long ws_floats) {
  const G4Split p = g4_plan_tt(M, N, K, ws_floats, true);
  return p.splits == 0 ? -1 : (long long)p.splits | ((long long)p.grid << 8);
}
