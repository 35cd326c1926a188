// conv3x3_4w -- persistent 4-wave 3x3 / stride-1 / pad-1 convolution for the KL-VAE encoder's
// Ci = Co = 128 ResnetBlock convs (vae/vaekl.py:56-113 conv1 / conv2 with the Normalize + swish that
// precede them, :9-17, 94-104): out = bias (+ residual) + conv(silu(gn(x))), NHWC bf16, and the
// per-128-pixel GroupNorm(32) partial sums of the stored output for the next GroupNorm
// (uva_groupnorm_finalize_tiles, tile_rows 128).
//
// The machinery of gemm4.hip applied to the halo conv (one wave per SIMD, accumulators in AGPRs, an
// explicitly ordered issue stream), built on v_mfma_f32_32x32x16_bf16: that instruction holds the
// SIMD's vector issue for 8 of its 32 cycles, so each MFMA gap has ~24 cycles for the LDS reads, the
// DMA issue and the GroupNorm + SiLU staging VALU (a 16x16x32 gap has 8: the first form of this kernel,
// 16x16x32 on 16 x 16 tiles, ran its staging VALU almost entirely un-hidden, 18 % of its time)
//   * workgroup = 4 waves, one per CU, persistent over 8 x 32-pixel output tiles (image-major,
//     XCD-contiguous slots); wave w owns tile rows 2w, 2w+1 x all 128 output channels: 2 x 4 32x32
//     accumulator blocks (128 AGPRs), the weight fragment as the MFMA A operand, so a lane holds runs
//     of 4 consecutive channels (= one GroupNorm group) of one pixel;
//   * K = 2 channel chunks (64) x 9 taps = 18 K-tiles of 64, each two 32-deep substeps (2 MFMA k-steps
//     of 16).  A (pixels) comes from the chunk's 10 x 34-pixel halo image in LDS (144-B pixel pitch =
//     9 x 16-B slots: a 32-pixel fragment row at any tap offset is bank-conflict-free, and every read
//     is the lane's base + a compile-time offset); B (weights, 128 x 64 per K-tile) streams from L2 by
//     LDS-DMA through a 3-region ring, two K-tiles ahead (16-B chunk XOR ((co >> 1) & 7): conflict-free
//     for 32-row fragments);
//   * the halo of the NEXT chunk is DMA'd raw (pre-activation) into the idle halo buffer as soon as
//     the previous occupant's last fragment read has passed a barrier (the odd substep of K-tile 8 /
//     17), then GroupNorm + SiLU'd IN PLACE by 11 staging rounds (one per substep, ds_read -> VALU ->
//     ds_write) whose VALU is spread over the substep's MFMA gaps;
//   * the residual tile is loaded into registers 7 K-tiles before the epilogue; the register epilogue
//     (v_permlane32_swap pairs -> 16-B channel runs, + bias from LDS, + residual, bf16 stores through
//     a buffer descriptor) also forms the GroupNorm partial sums (two waves per 128-pixel slot, added
//     through LDS).
// Every global access of the K loop is counted: the vmcnt immediates come from the static issue
// schedule (g4c_allowed below), so no wait ever drains more than the operand it protects.
#include "common.h"

#include <algorithm>
#include <type_traits>

#ifndef UVA_CONV4_DIAG
#define UVA_CONV4_DIAG 0  // timing builds only (results WRONG): 1 no staging VALU, 2 no weight DMA in the
                          // loop, 4 no epilogue stores, 8 no waits / barriers in the loop, 16 no halo DMA, 32 halo DMAs
                          // from one image (L2-hot)
#endif

namespace {

constexpr int C4_TH = 8, C4_TW = 32;            // output tile
constexpr int C4_HW = C4_TW + 2, C4_HH = C4_TH + 2;  // halo 34 x 10
constexpr int C4_HPIX = C4_HW * C4_HH;          // 340 halo pixels
constexpr int C4_PITCH = 144;                   // bytes per halo pixel (64 channels = 128 B + 16 B pad)
constexpr int C4_HSLOT = C4_PITCH / 16;         // 9
constexpr int C4_HDMA_W = 12;                   // 1-KB raw-halo DMA instructions per wave (48 x 64 >= 340 x 9)
constexpr int C4_HBUF = 4 * C4_HDMA_W * 1024;   // halo buffer bytes (DMA footprint, 49152)
constexpr int C4_WREG = 128 * 128;              // weight region: 128 co x 64 k bf16
// LDS: the weight ring first (every B fragment read = lane base + a 16-bit immediate), then the two
// halo buffers, the bias and the partial-sum slots
constexpr int C4_H0 = 3 * C4_WREG;
constexpr int C4_BIAS = C4_H0 + 2 * C4_HBUF;
constexpr int C4_PART = C4_BIAS + 512;
constexpr int C4_LDS = C4_PART + 2 * 64 * 4;
constexpr int C4_ROUNDS = 11;                   // staging rounds per chunk (2720 16-B slots / 256)
constexpr int C4_LAST = C4_HPIX * 8 - (C4_ROUNDS - 1) * 256;  // threads with a slot in the last round (160)
constexpr int C4_RL = 10;                       // K-tile whose odd substep loads the residual tile
constexpr int C4_RAW_AT = 3;                    // odd substep: MFMA index of the RAW wait
constexpr int C4_EOPS = 16 + 16;                // epilogue vm ops per wave: 16 output + 16 partial stores

// vm operations issued per substep position (per wave), in issue order:
//   even substep t >= 1: GroupNorm scale / shift loads GL (t = 9; t = 0 too), then the weights W of
//     K-tile t + 2 (into the region K-tile t - 1 left; t = 16, 17: the next tile's K-tiles 0, 1);
//   odd substep 17: the next tile's K-tile-2 weights (region 2, free since its WAR barrier), then the
//     raw next-chunk halo H (odd substep 8 too); odd substep C4_RL: the residual R;
//   between odd 17 and even 0: the epilogue's EOPS stores.
constexpr int c4_H(int t) { return (t == 8 || t == 17) ? C4_HDMA_W : 0; }
constexpr int c4_R(int t, bool res) { return (res && t == C4_RL) ? 16 : 0; }
constexpr int c4_GL(int t, bool gn) { return (gn && (t == 0 || t == 9)) ? 4 : 0; }
constexpr int c4_W(int t) { return t == 0 ? 0 : 4; }
// RAW wait of odd substep t (before reading K-tile t + 1): the weights of K-tile t + 1 (even substep
// t - 1; t = 1: odd 17; t = 0: even 17) complete, everything issued after them may stay in flight
constexpr int g4c_allowed(int t, bool gn, bool res) {
  if (t == 0) return 4 + C4_HDMA_W + C4_EOPS + c4_GL(0, gn);
  if (t == 1) return C4_HDMA_W + C4_EOPS + c4_GL(0, gn) + c4_GL(1, gn) + c4_W(1);
  // (odd 17: its own K-tile-2 weights issued before the RAW point, 3 of them, are younger too)
  return c4_H(t - 1) + c4_R(t - 1, res) + c4_GL(t, gn) + c4_W(t) + (t == 17 ? C4_RAW_AT : 0);
}
// epilogue: the residual loads of odd substep C4_RL complete; younger: even C4_RL+1 .. 17, odd 17
constexpr int g4c_res_allowed(bool gn) {
  int n = 4 + C4_HDMA_W;
  for (int t = C4_RL + 1; t < 18; ++t) n += c4_W(t) + c4_GL(t, gn);
  return n;
}
static_assert(g4c_allowed(0, true, true) <= 63 && g4c_allowed(1, true, true) <= 63 && g4c_res_allowed(true) <= 63,
              "vmcnt immediates");

__device__ __forceinline__ int c4_xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <int N>
__device__ __forceinline__ void c4_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace

typedef __attribute__((ext_vector_type(4))) unsigned c4u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned c4u32x2;
typedef __attribute__((ext_vector_type(16))) float c4f32x16;

// GN: 0 none (plain conv, zero padding), 1 GroupNorm apply, 2 GroupNorm + SiLU.  RES: residual.
template <int GN, bool RES>
__global__ __launch_bounds__(256, 1) void conv3x3_4w(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                     bf16* __restrict__ out, const float* __restrict__ bias,
                                                     const bf16* __restrict__ residual,
                                                     const float* __restrict__ gn_scale,
                                                     const float* __restrict__ gn_shift, float* __restrict__ gn_part,
                                                     int Nimg, int H, int W) {
  constexpr bool HASGN = GN != 0;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = W / C4_TW, tiles_y = H / C4_TH, tpi = tiles_x * tiles_y, ntiles = Nimg * tpi;
  const int grid = gridDim.x;
  const int slot = c4_xcd_remap(blockIdx.x, grid);
  if (slot >= ntiles) return;
  const int my_tiles = (ntiles - slot + grid - 1) / grid;
  const long long img_elems = (long long)H * W * 128;

  float* sbias = (float*)(smem + C4_BIAS);
  float* spart = (float*)(smem + C4_PART);
  if (tid < 128) sbias[tid] = bias ? bias[tid] : 0.f;

  struct Tile {
    int n, oh0, ow0, t;  // t: tile index inside its image
  };
  auto tile_of = [&](int pid) __attribute__((always_inline)) {
    Tile c;
    c.n = pid / tpi;
    c.t = pid - c.n * tpi;
    c.oh0 = (c.t / tiles_x) * C4_TH;
    c.ow0 = (c.t % tiles_x) * C4_TW;
    return c;
  };

  // ---- weights: LDS-DMA, instruction i (wave w: 4w .. 4w+3) = output channels 8i .. 8i+7 x 128 B;
  // LDS chunk (lane & 7) of row co holds global chunk (lane & 7) ^ ((co >> 1) & 7)
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)wt, 0, 128 * 1152 * 2, 0x00020000);
  unsigned woff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = 8 * (4 * w + i) + (lane >> 3);
    woff[i] = (unsigned)(co * 2304 + (((lane & 7) ^ ((co >> 1) & 7)) << 4));
  }
  auto wdma = [&](int region, int i, int kt) __attribute__((always_inline)) {
    const int soff = __builtin_amdgcn_readfirstlane((((kt % 9) * 128) + (kt / 9) * 64) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rsW, (__attribute__((address_space(3))) void*)(smem + region * C4_WREG + (4 * w + i) * 1024), 16,
        (int)woff[i], soff, 0, 0);
  };

  // ---- raw halo DMA of a tile's chunk: instruction j of wave w covers 16-B slots (w + 4j) * 64 + lane
  // of the padded image (slot s = pixel s / 9, chunk s % 9; chunk 8 and pixels past the halo or the
  // image read zero through the descriptor's range check)
  auto hoff_of = [&](const Tile& c, int j) __attribute__((always_inline)) -> unsigned {
    const int s = (w + 4 * j) * 64 + lane;
    const int p = s / C4_HSLOT, k = s - p * C4_HSLOT;
    const int hy = p / C4_HW, hx = p - hy * C4_HW;
    const int ih = c.oh0 - 1 + hy, iw = c.ow0 - 1 + hx;
    const bool ok = p < C4_HPIX && k < 8 && ih >= 0 && ih < H && iw >= 0 && iw < W;
    return ok ? (unsigned)(((ih * W + iw) * 128 + k * 8) * 2) : 0x7ffffff0u;
  };
  unsigned hoff[C4_HDMA_W];
  auto in_rsrc = [&](const Tile& c) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(in + (long long)c.n * img_elems), 0, (int)(img_elems * 2),
                                             0x00020000);
  };
  auto hdma = [&](const __amdgpu_buffer_rsrc_t& rs, int hbuf, int j, int cc) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rs, (__attribute__((address_space(3))) void*)(smem + C4_H0 + hbuf * C4_HBUF + (w + 4 * j) * 1024), 16,
        (int)hoff[j], __builtin_amdgcn_readfirstlane(cc * 128), 0, 0);
  };

  // ---- staging rounds: slot q = tid + 256 r (pixel q >> 3, channel chunk tid & 7), in place
  const int act_base = (tid >> 3) * C4_PITCH + (tid & 7) * 16;
  float gsc[8], gsh[8];
  auto gn_load = [&](const Tile& c, int cc) __attribute__((always_inline)) {
    if constexpr (HASGN) {
      const float* sc = gn_scale + (long long)c.n * 128 + cc * 64 + (tid & 7) * 8;
      const float* sh = gn_shift + (long long)c.n * 128 + cc * 64 + (tid & 7) * 8;
      const float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
      const float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
      gsc[0] = s0.x; gsc[1] = s0.y; gsc[2] = s0.z; gsc[3] = s0.w; gsc[4] = s1.x; gsc[5] = s1.y; gsc[6] = s1.z; gsc[7] = s1.w;
      gsh[0] = h0.x; gsh[1] = h0.y; gsh[2] = h0.z; gsh[3] = h0.w; gsh[4] = h1.x; gsh[5] = h1.y; gsh[6] = h1.z; gsh[7] = h1.w;
    }
  };
  // bit r: round r's pixel lies outside the image (activated value replaced by the zero padding)
  auto oob_mask = [&](const Tile& c) __attribute__((always_inline)) {
    unsigned m = 0;
#pragma unroll
    for (int r = 0; r < C4_ROUNDS; ++r) {
      const int p = (tid >> 3) + 32 * r;
      const int hy = p / C4_HW, hx = p - hy * C4_HW;
      const int ih = c.oh0 - 1 + hy, iw = c.ow0 - 1 + hx;
      if (!(ih >= 0 && ih < H && iw >= 0 && iw < W)) m |= 1u << r;
    }
    return m;
  };
  c4u32x4 araw;             // the round's raw slot (read one substep ahead)
  float au[8], ar[8];       // GroupNorm'd values, sigmoid terms
  auto act_read = [&](int hbuf, int r) __attribute__((always_inline)) {
    if (r < C4_ROUNDS - 1 || tid < C4_LAST)
      araw = *(const c4u32x4*)(smem + C4_H0 + hbuf * C4_HBUF + act_base + r * 32 * C4_PITCH);
  };
  // unit u (0..31) of a round: stage u / 4 of pair q = u % 4 (elements 2q, 2q+1); gap i of a substep
  // runs units 2i, 2i+1 (two pairs, one stage), so consecutive stages of a pair are two gaps apart and
  // a gap carries 16-32 cycles of VALU: 0 unpack + GN e0, 1 GN e1 + exp args, 2 / 3 exp, 4 +1,
  // 5 / 6 rcp, 7 SiLU products + cvt + padding select
  typedef __attribute__((ext_vector_type(2))) __bf16 c4bf16x2;
  // (every produced value goes through an empty asm: pure VALU is not ordered by sched_barrier and
  // would otherwise sink to its first use -- one burst at the substep's end)
  auto pin = [](float& v) __attribute__((always_inline)) { asm volatile("" : "+v"(v)); };
  auto act_unit = [&](int u, unsigned oob, int r) __attribute__((always_inline)) {
    if constexpr (UVA_CONV4_DIAG & 1) return;
    const int st = u / 4, q = u % 4, e0 = 2 * q, e1 = 2 * q + 1;
    if (st == 0) {
      const unsigned wv = araw[q];
      au[e0] = __uint_as_float(wv << 16);
      au[e1] = __uint_as_float(wv & 0xffff0000u);
      if constexpr (HASGN) au[e0] = fmaf(au[e0], gsc[e0], gsh[e0]);
      pin(au[e0]);
      pin(au[e1]);
    } else if (st == 1) {
      if constexpr (HASGN) au[e1] = fmaf(au[e1], gsc[e1], gsh[e1]);
      pin(au[e1]);
      if constexpr (GN == 2) {
        ar[e0] = au[e0] * -1.4426950408889634f;
        ar[e1] = au[e1] * -1.4426950408889634f;
        pin(ar[e0]);
        pin(ar[e1]);
      }
    } else if (GN == 2 && st == 2) {
      ar[e0] = __builtin_amdgcn_exp2f(ar[e0]);
      pin(ar[e0]);
    } else if (GN == 2 && st == 3) {
      ar[e1] = __builtin_amdgcn_exp2f(ar[e1]);
      pin(ar[e1]);
    } else if (GN == 2 && st == 4) {
      ar[e0] += 1.f;
      ar[e1] += 1.f;
      pin(ar[e0]);
      pin(ar[e1]);
    } else if (GN == 2 && st == 5) {
      ar[e0] = __builtin_amdgcn_rcpf(ar[e0]);
      pin(ar[e0]);
    } else if (GN == 2 && st == 6) {
      ar[e1] = __builtin_amdgcn_rcpf(ar[e1]);
      pin(ar[e1]);
    } else if (st == 7) {
      float y0 = au[e0], y1 = au[e1];
      if constexpr (GN == 2) {
        y0 *= ar[e0];
        y1 *= ar[e1];
      }
      const unsigned pk = __builtin_bit_cast(unsigned, (c4bf16x2){(bf16)y0, (bf16)y1});
      unsigned o = ((oob >> r) & 1u) ? 0u : pk;
      asm volatile("" : "+v"(o));
      araw[q] = o;
    }
  };
  auto act_write = [&](int hbuf, int r) __attribute__((always_inline)) {
    if constexpr (UVA_CONV4_DIAG & 1) return;
    if (r < C4_ROUNDS - 1 || tid < C4_LAST)
      *(c4u32x4*)(smem + C4_H0 + hbuf * C4_HBUF + act_base + r * 32 * C4_PITCH) = araw;
  };

  // ---- fragment reads (k-step ks of a K-tile: k 16 ks .. 16 ks + 15).  A (MFMA B operand): pixel
  // lane & 31 of tile row 2w + f at tap (kh, kw), channels 8 (lane >> 5) .. +7 of the k-step.  B (MFMA A
  // operand): weight row g * 32 + (lane & 31), the same 8 k
  const int abase = ((2 * w) * C4_HW + (lane & 31)) * C4_PITCH + (lane >> 5) * 16;
  const int wrow = lane & 31;
  int bofs[4];  // per k-step: row wrow's chunk 2 ks + (lane >> 5), XOR-swizzled
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) bofs[ks] = wrow * 128 + (((2 * ks + (lane >> 5)) ^ ((wrow >> 1) & 7)) << 4);
  auto fragA = [&](int kt, int f, int ks) __attribute__((always_inline)) -> bf16x8 {
    const int hb = (kt / 9) & 1, tap = kt % 9, kh = tap / 3, kw = tap % 3;
    return *(const bf16x8*)(smem + C4_H0 + hb * C4_HBUF + abase + ((f + kh) * C4_HW + kw) * C4_PITCH + ks * 32);
  };
  auto fragB = [&](int kt, int g, int ks) __attribute__((always_inline)) -> bf16x8 {
    return *(const bf16x8*)(smem + (kt % 3) * C4_WREG + g * 4096 + bofs[ks]);
  };

  c4f32x16 acc[2][4];
  bf16x8 fa[2][2][2], fb[2][2][4];  // [set][k-step of the half][row | co-block]
  bf16x8 rres[16];                  // residual tile (RES): 2 rows x 4 co-blocks x 2 runs of 8

  // ---- prologue: weights of K-tiles 0..2, the first tile's raw chunks, then chunk 0 activated
  int pid = slot;
  Tile cur = tile_of(pid);
  {
    const auto rs = in_rsrc(cur);
#pragma unroll
    for (int j = 0; j < C4_HDMA_W; ++j) hoff[j] = hoff_of(cur, j);
#pragma unroll
    for (int kt = 0; kt < 3; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) wdma(kt, i, kt);
#pragma unroll
    for (int j = 0; j < C4_HDMA_W; ++j) hdma(rs, 0, j, 0);
#pragma unroll
    for (int j = 0; j < C4_HDMA_W; ++j) hdma(rs, 1, j, 1);
    gn_load(cur, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned oob = oob_mask(cur);
#pragma unroll
    for (int r = 0; r < C4_ROUNDS; ++r) {
      act_read(0, r);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < 32; ++u) act_unit(u, oob, r);
      act_write(0, r);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int f = 0; f < 2; ++f) fa[0][ks][f] = fragA(0, f, ks);
#pragma unroll
      for (int g = 0; g < 4; ++g) fb[0][ks][g] = fragB(0, g, ks);
    }
  }

  const int run8 = 8 * (lane >> 5);  // the lane's 8-channel run inside each 16-channel half-block

  for (int ii = 0; ii < my_tiles; ++ii) {
    const bool more = ii + 1 < my_tiles;
    const Tile nxt = tile_of(more ? pid + grid : pid);
#if UVA_CONV4_DIAG & 32
    const auto rs_next = in_rsrc(tile_of(slot));  // timing only: every halo DMA re-reads the first tile's image
#else
    const auto rs_next = in_rsrc(nxt);
#endif
    const unsigned oob_cur = oob_mask(cur), oob_nxt = oob_mask(nxt);
    const long long obase = (long long)cur.n * img_elems;
    const auto rsO = __builtin_amdgcn_make_buffer_rsrc((void*)(out + obase), 0, (int)(img_elems * 2), 0x00020000);
    // the lane's pixel of tile row 2w + f, channel run of (co-block g, half jp): byte offset in the image
    auto out_off = [&](int f, int g, int jp) __attribute__((always_inline)) {
      return (((cur.oh0 + 2 * w + f) * W + cur.ow0 + (lane & 31)) * 128 + g * 32 + jp * 16 + run8) * 2;
    };

    // one substep.  KT: K-tile 0..17 (compile-time), ODD: k-half 1
    auto substep = [&](auto KTC, auto ODC) __attribute__((always_inline)) {
      constexpr int kt = decltype(KTC)::value;
      constexpr bool ODD = decltype(ODC)::value;
      constexpr int b = ODD ? 1 : 0;
      constexpr bool ZERO = kt == 0 && !ODD;
      // staging rounds: buffer 1 (this tile's chunk 1) in E3 .. E8, buffer 0 (next tile's chunk 0) in
      // E12 .. E17; a substep's index in its window = its round
      constexpr int sidx = 2 * kt + (ODD ? 1 : 0);
      constexpr int r1 = sidx - 6, r0 = sidx - 24;
      constexpr bool ACT1 = r1 >= 0 && r1 < C4_ROUNDS, ACT0 = r0 >= 0 && r0 < C4_ROUNDS;
      constexpr int ar_ = ACT1 ? r1 : r0, ahb = ACT1 ? 1 : 0;
      constexpr int nr1 = sidx + 1 - 6, nr0 = sidx + 1 - 24;  // the next substep's round (raw read)
      constexpr bool NACT1 = nr1 >= 0 && nr1 < C4_ROUNDS, NACT0 = nr0 >= 0 && nr0 < C4_ROUNDS;
      const unsigned oob = ACT1 ? oob_cur : oob_nxt;

      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (ODD && !(UVA_CONV4_DIAG & 8)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!ODD && HASGN && kt == 0) gn_load(cur, 1);
      if constexpr (!ODD && HASGN && kt == 9) gn_load(nxt, 0);
      if constexpr (ODD && (kt == 7 || kt == 16)) {
        // the raw-halo DMA offsets of the next tile, one substep before their use
#pragma unroll
        for (int j = 0; j < C4_HDMA_W; ++j) hoff[j] = hoff_of(nxt, j);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < 16; ++mi) {
        const int ks = mi / 8, f = (mi / 4) % 2, g = mi % 4;
        if (ODD && mi == C4_RAW_AT && !(UVA_CONV4_DIAG & 8)) {
          c4_vmcnt<g4c_allowed(kt, HASGN, RES)>();
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (ZERO) {
          if (ks == 0)
            acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[b][ks][g], fa[b][ks][f], (c4f32x16){}, 0, 0, 0);
          else
            acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[b][ks][g], fa[b][ks][f], acc[f][g], 0, 0, 0);
        } else {
          acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[b][ks][g], fa[b][ks][f], acc[f][g], 0, 0, 0);
        }
        if constexpr (!ODD) {
          // weights of K-tile kt + 2 into the region K-tile kt - 1 left (free since odd kt - 1's barrier)
          if (!(UVA_CONV4_DIAG & 2) && kt >= 1 && mi >= 4 && mi < 16 && (mi - 4) % 3 == 0)
            wdma((kt + 2) % 3, (mi - 4) / 3, (kt + 2) % 18);
          // reads of this K-tile's k-steps 2, 3
          if (mi >= 2 && mi < 14) {
            const int rks = (mi - 2) / 6, ri = (mi - 2) % 6;
            if (ri < 2) fa[1][rks][ri < 2 ? ri : 0] = fragA(kt, ri < 2 ? ri : 0, 2 + rks);
            else fb[1][rks][ri < 2 ? 0 : ri - 2] = fragB(kt, ri < 2 ? 0 : ri - 2, 2 + rks);
          }
        } else {
          // odd 17: the next tile's K-tile-2 weights, before its halo DMAs
          if (!(UVA_CONV4_DIAG & 2) && kt == 17 && mi < 4) wdma(2, mi, 2);
          // the next tile's raw chunk 0 (K-tile 8: buffer 0 is past its last read) / chunk 1 (17)
          if (!(UVA_CONV4_DIAG & 16) && kt == 8 && mi >= 4 && mi < 4 + C4_HDMA_W) hdma(rs_next, 0, mi - 4, 0);
          if (!(UVA_CONV4_DIAG & 16) && kt == 17 && mi >= 4 && mi < 4 + C4_HDMA_W) hdma(rs_next, 1, mi - 4, 1);
          if constexpr (RES && kt == C4_RL) {
            // residual runs: one per MFMA gap from the RAW point, the remaining ones after the loop
            if (mi >= C4_RAW_AT) {
              const int j = mi - C4_RAW_AT;
              const auto rsR = __builtin_amdgcn_make_buffer_rsrc((void*)(residual + obase), 0, (int)(img_elems * 2),
                                                                 0x00020000);
              rres[j] = __builtin_bit_cast(
                  bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsR, out_off(j / 8, (j / 2) % 4, j % 2), 0, 0));
            }
          }
          // reads of the next K-tile's k-steps 0, 1 (after the RAW point; 17 -> the next tile's K-tile 0)
          constexpr int nk = (kt + 1) % 18;
          if (mi >= C4_RAW_AT && mi < C4_RAW_AT + 12) {
            const int j = mi - C4_RAW_AT, rks = j / 6, ri = j % 6;
            if (ri < 2) fa[0][rks][ri < 2 ? ri : 0] = fragA(nk, ri < 2 ? ri : 0, rks);
            else fb[0][rks][ri < 2 ? 0 : ri - 2] = fragB(nk, ri < 2 ? 0 : ri - 2, rks);
          }
        }
        if constexpr (ACT1 || ACT0) {
          act_unit(2 * mi, oob, ar_);
          act_unit(2 * mi + 1, oob, ar_);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (RES && ODD && kt == C4_RL) {
        const auto rsR = __builtin_amdgcn_make_buffer_rsrc((void*)(residual + obase), 0, (int)(img_elems * 2),
                                                           0x00020000);
#pragma unroll
        for (int j = 16 - C4_RAW_AT; j < 16; ++j)
          rres[j] = __builtin_bit_cast(
              bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsR, out_off(j / 8, (j / 2) % 4, j % 2), 0, 0));
      }
      if constexpr (ACT1 || ACT0) act_write(ahb, ar_);
      if constexpr (NACT1) act_read(1, nr1);
      if constexpr (NACT0) act_read(0, nr0);
      __builtin_amdgcn_sched_barrier(0);
    };
    using F = std::false_type;
    using T = std::true_type;
#define C4_KT(n)                                         \
  substep(std::integral_constant<int, n>{}, F{});        \
  substep(std::integral_constant<int, n>{}, T{});
    C4_KT(0) C4_KT(1) C4_KT(2) C4_KT(3) C4_KT(4) C4_KT(5) C4_KT(6) C4_KT(7) C4_KT(8)
    C4_KT(9) C4_KT(10) C4_KT(11) C4_KT(12) C4_KT(13) C4_KT(14) C4_KT(15) C4_KT(16) C4_KT(17)
#undef C4_KT

    // ---- register epilogue: per block (f, g) and half jp, v_permlane32_swap turns the two lanes'
    // 4-channel runs into one 8-channel run per lane (lanes 0-31: channels 16 jp .. +7, lanes 32-63:
    // 16 jp + 8 .. +15 of the block)
    if constexpr (RES) c4_vmcnt<g4c_res_allowed(HASGN)>();
    float ps[4][2][4];  // per (co-block, half): sum / sumsq of the lane's two groups
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
#pragma unroll
        for (int e = 0; e < 4; ++e) ps[g][jp][e] = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[f][g][8 * jp + r]),
                                                            __float_as_uint(acc[f][g][8 * jp + 4 + r]), false, false);
            v[r] = __uint_as_float(x[0]);
            v[4 + r] = __uint_as_float(x[1]);
          }
          const int cb = g * 32 + jp * 16 + run8;
          const float4 b0 = *(const float4*)(sbias + cb), b1 = *(const float4*)(sbias + cb + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
          if constexpr (RES) {
            const bf16x8 rq = rres[f * 8 + g * 2 + jp];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += (float)rq[e];
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(c4u32x4, o), rsO,
                                                 (UVA_CONV4_DIAG & 4) ? 0x7ffffff0 : out_off(f, g, jp), 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = (float)o[e], c = (float)o[4 + e];
            ps[g][jp][0] += a;
            ps[g][jp][1] += a * a;
            ps[g][jp][2] += c;
            ps[g][jp][3] += c * c;
          }
        }
      }
    }
    // GroupNorm partial sums: over the 32 pixel lanes of each half, then waves 2k + 1 hand theirs to
    // 2k through LDS (the two waves of one 128-pixel slot = tile rows 4k .. 4k+3); every wave issues
    // the 16 stores (odd waves' and non-leading lanes' out of range), so the vm count stays uniform
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = row16_sum(ps[g][jp][e]);
          t += __shfl_xor(t, 16, 64);
          ps[g][jp][e] = t;
        }
    const bool lead32 = (lane & 31) == 0;
    if ((w & 1) && lead32) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp)
          *(float4*)(spart + (w >> 1) * 64 + (((lane >> 5) * 8 + g * 2 + jp) * 4)) =
              make_float4(ps[g][jp][0], ps[g][jp][1], ps[g][jp][2], ps[g][jp][3]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // LDS only: the stores in flight stay in flight
    {
      const bool lead = !(w & 1) && lead32 && gn_part != nullptr;
      const long long slot128 = (long long)cur.n * (tpi * 2) + cur.t * 2 + (w >> 1);
      const auto rsP = __builtin_amdgcn_make_buffer_rsrc((void*)gn_part, 0, gn_part ? 0x7ffff000 : 0, 0x00020000);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const float4 o4 = *(const float4*)(spart + (w >> 1) * 64 + (((lane >> 5) * 8 + g * 2 + jp) * 4));
          const int grp = (g * 32 + jp * 16 + run8) / 4;
          const int off = lead ? (int)((slot128 * 32 + grp) * 8) : 0x7ffffff0;
          const float2 ga = make_float2(ps[g][jp][0] + o4.x, ps[g][jp][1] + o4.y);
          const float2 gb = make_float2(ps[g][jp][2] + o4.z, ps[g][jp][3] + o4.w);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(c4u32x2, ga), rsP, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(c4u32x2, gb), rsP, off + 8, 0, 0);
        }
    }
    pid += grid;
    cur = nxt;
  }
  // the refills past the end land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
static int c4_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

static int g_conv4_on = 1;

// 1 = eligible shape: 3x3 / s1 / p1, Ci = Co = 128, H a multiple of 8, W of 32, one image < 2 GB
extern "C" int uva_conv4_ok(int Nimg, int H, int W, int Ci, int Co) {
  return g_conv4_on && Nimg > 0 && Ci == 128 && Co == 128 && H % C4_TH == 0 && W % C4_TW == 0 && H >= C4_TH &&
         W >= C4_TW && (long long)H * W * 256 < 0x7fff0000LL;
}

extern "C" int uva_conv4_set(int on) {
  const int prev = g_conv4_on;
  if (on >= 0) g_conv4_on = on;
  return prev;
}

template <int GN, bool RES>
static int c4_launch(const void* in, const void* w, void* out, const float* bias, const void* residual,
                     const float* sc, const float* sh, float* part, int Nimg, int H, int W, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3x3_4w<GN, RES>, hipFuncAttributeMaxDynamicSharedMemorySize, C4_LDS);
    attr = true;
  }
  const long long tiles = (long long)Nimg * (H / C4_TH) * (W / C4_TW);
  const int grid = (int)std::min<long long>(tiles, c4_cus());
  conv3x3_4w<GN, RES><<<dim3(grid), 256, C4_LDS, s>>>((const bf16*)in, (const bf16*)w, (bf16*)out, bias,
                                                      (const bf16*)residual, sc, sh, part, Nimg, H, W);
  UVA_LAUNCH_CHECK();
  return 0;
}

// 1 = launched, 0 = not eligible, < 0 = -hipError.  gn_scale / gn_shift: both or neither
extern "C" int uva_conv4_try(const void* in, const void* w, void* out, const float* bias, const void* residual,
                             int Nimg, int H, int W, int Ci, int Co, const float* gn_scale, const float* gn_shift,
                             int gn_silu, float* gn_part, hipStream_t s) {
  if (!uva_conv4_ok(Nimg, H, W, Ci, Co)) return 0;
  if (((uintptr_t)in | (uintptr_t)w | (uintptr_t)out | (uintptr_t)residual | (uintptr_t)gn_part) % 16) return 0;
  if ((gn_scale == nullptr) != (gn_shift == nullptr)) return 0;
  if (gn_scale && (((uintptr_t)gn_scale | (uintptr_t)gn_shift) % 16)) return 0;
  // GroupNorm + SiLU prologue only (every Ci = Co = 128 3x3 conv of the encoder); the kernel also
  // has the plain / GN-only staging forms (GN = 0 / 1), not instantiated
  if (!gn_scale || !gn_silu) return 0;
  int r;
#define C4L(G, R) r = c4_launch<G, R>(in, w, out, bias, residual, gn_scale, gn_shift, gn_part, Nimg, H, W, s)
  if (residual) C4L(2, true);
  else C4L(2, false);
#undef C4L
  return r ? -r : 1;
}
