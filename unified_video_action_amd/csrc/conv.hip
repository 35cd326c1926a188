// Direct 3x3 / stride-1 / pad-1 convolution over NHWC bf16 with the input patch staged ONCE
// per 64-channel chunk into LDS (halo tile) and GroupNorm-apply + SiLU fused into that staging.
//
// Replaces nn.Conv2d(k=3, s=1, p=1) of the KL-VAE encoder ResnetBlock conv1/conv2 and conv_out
// (reference vae/vaekl.py:56-113, 246-273) together with the Normalize + nonlinearity that
// precede them (vaekl.py:9-17, 94-104, 270-271): out = bias + residual + conv(silu(gn(x))).
//
// Work decomposition (one workgroup per output tile; TR = 8: 256 threads, 2 workgroups / CU):
//   * output tile = 16 x 16 pixels x BN output channels (BN = 128 or 256);
//   * K loop = (64-channel chunk cc) x (9 taps); per chunk the 18 x 18 x 64 input halo is
//     loaded to registers at tap 0, normalised + SiLU'd (zero padding applied AFTER the
//     activation, as F.conv2d pads the activated tensor) and written to the other halo buffer
//     at tap 8 -- every input element is read from HBM/L2 once per chunk instead of 9x
//     (implicit-GEMM im2col).  The GN prologue is supported, but its VALU work is not hidden
//     under the MFMAs (level-0 conv 8.8 ms fused vs 5.5 ms + 1.6 ms separate apply pass; a
//     variant streaming one activated round per tap between the MFMA k-steps measured 10.9 ms),
//     so the VAE runs this kernel on pre-activated inputs (vae/vaekl.py _resblock);
//   * the weight tile of each (chunk, tap) step -- BN rows x 64 k -- is staged by LDS-DMA
//     (global_load_lds, 16 B/lane) one step ahead into a 2-deep ring;
//   * A fragments (16 pixels of one tile row x 32 channels) are read from the halo image at
//     the tap's (kh, kw) offset: pixel p's 16-B channel chunk c sits at slot c ^ (p & 7), which
//     is bank-conflict-free for every tap offset (ds_read_b128, 16-lane groups);
//   * v_mfma_f32_16x16x32_bf16, fp32 accumulation; waves 2(M) x 4(N) of 128 px x 64 co (BN 256)
//     or 4(M) x 2(N) of 64 x 64 (BN 128);
//   * epilogue: bias + bf16 residual, 16-B stores, and the deterministic per-(128-pixel half, group)
//     GroupNorm(32) partial sums of the stored output for the NEXT GroupNorm
//     (uva_groupnorm_finalize_tiles, tile_rows 128).  The GN (register-B) form finishes from
//     registers: its product is formed transposed (lane = 4 channels of one pixel), one
//     v_permlane16_swap per accumulator word turns that into 16-B channel runs, the bias seeds the
//     accumulators; no LDS image, no barrier (level-0 6.48 -> 6.22 ms; 8-B runs straight from the
//     transposed accumulators measured 6.80: the stores split into 16 x 32-B pieces per
//     instruction).  The plain form stages the fp32 tile through LDS (128-pixel halves).
#include "common.h"

#define CH_T 16   // tile width (pixels)
#define CH_W 18   // halo width
#define CH_H 18   // conv_in halo (16 x 16 tile)
#define CH_HPIX (CH_H * CH_H)

// TR = tile rows: 16 (512 threads, 1 workgroup / CU) or 8 (256 threads, 2 workgroups / CU: the two
// co-resident tiles drift apart, so one tile's prologue / epilogue HBM traffic runs under the
// other's MFMA loop instead of every CU loading and storing in lockstep)
template <int BN, int TR, bool R3 = false, bool HD = false, bool RB = false>
struct ConvHCfg {
  static constexpr int NTH = TR * 32, NW = NTH / 64;
  // BN = 128: waves of 64 px x 64 co; RB: waves of 128 px x 32 co (each wave streams only its
  // own 32 weight columns from L2, so the workgroup's B traffic equals the LDS ring's)
  static constexpr int WN = RB ? NW : 2, WM = NW / WN;
  static constexpr int FM = TR / WM;            // tile rows (16-pixel fragments) per wave
  static constexpr int FN = BN / WN / 16;       // 16-channel fragments per wave
  static constexpr int HR = TR + 2;             // halo rows
  static constexpr int HPIX = HR * CH_W;
  // HD: the halo is staged by LDS-DMA, HD_I wave-instructions (8 pixels x 128 B each) per wave,
  // the image padded to HPIX_P pixels
  static constexpr int HD_I = ((HPIX + 7) / 8 + NW - 1) / NW;
  static constexpr int HPIX_P = HD_I * NW * 8;
  // RB: padded pixel pitch of 80 elements (160 B = 10 x 16 B): for a fragment read, lane l reads
  // 16 B at pixel (l & 15), channel chunk (l >> 4), i.e. 16-B slot ((l & 15) * 10 + (l >> 4)) mod 16
  // of the 64-bank row -- distinct inside each of ds_read_b128's four 16-lane groups
  // ({0-3,12-15,20-27}, ...), so the A reads are conflict-free with no swizzle and every fragment
  // offset is the lane's base + a compile-time constant.  (A 144-B pitch, conflict-free only for 16
  // CONSECUTIVE lanes, was up to 8-way conflicted in the real lane groups.)
  static constexpr int PP = RB ? 80 : 64;
  static constexpr int HALO_ELEMS = (HD ? HPIX_P : HPIX) * PP;
  static constexpr int ROUNDS = (HPIX * 8 + NTH - 1) / NTH;
  static constexpr int BT = BN * 64;            // weight tile elements
  static constexpr int NI = BT / (NW * 512);    // DMA instructions per thread per weight tile
  // R3: one halo buffer (restaged between chunks) and a 3-slot weight ring (DMA two steps ahead);
  // otherwise two halo buffers and a 2-slot ring
  static constexpr int NHB = R3 ? 1 : 2, NWB = R3 ? 3 : 2;
  static constexpr int MAIN_BYTES = (NHB * HALO_ELEMS + (RB ? 0 : NWB * BT)) * 2;  // RB: weights in VGPRs
  static constexpr int TP = BN + 4;             // epilogue fp32 pitch
  static constexpr int EPI_BYTES = 128 * TP * 4 + NW * (BN / 8) * 8 * 2 * 4;
  // RB finishes from registers: no epilogue image
  static constexpr int LDS_BYTES = (RB || MAIN_BYTES > EPI_BYTES) ? MAIN_BYTES : EPI_BYTES;
};

// workgroup barrier ordering LDS only: the epilogue's global stores stay in flight across it
// (__syncthreads drains vmcnt, i.e. waits for every store of the half before the next step)
__device__ __forceinline__ void ch_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// v + v[lane ^ o]: o = 16 / 32 by v_permlane16/32_swap (VALU; ds_bpermute for the rest)
__device__ __forceinline__ float xor_lane_sum(float v, int o) {
  if (o == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  if (o == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return v + __shfl_xor(v, o, 64);
}

__device__ __forceinline__ int ch_xcd_remap(int bid, int nblk) {
  int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// 16-B LDS read hidden from hipcc's wait insertion; the caller orders completion with explicit
// s_waitcnt lgkmcnt + sched_barrier before the consumer
__device__ __forceinline__ bf16x8 lds_read16(const bf16* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)LDS_PTR(char, p)) : "memory");
  return v;
}

typedef __attribute__((ext_vector_type(4))) unsigned ch_u32x4;

// Halo geometry in 32-bit lane arithmetic: thread chunk p of a halo with CH_W = 18 columns sits at
// (p / 18, p % 18); p < 2^15, so p / 18 = (p * 3641) >> 16 on the full-rate 24-bit multiplier (hipcc
// lowers the plain division to a quarter-rate v_mul_hi_u32)
__device__ __forceinline__ int ch_div18(int p) { return (int)(__umul24((unsigned)p, 3641u) >> 16); }
// buffer descriptor over one image [H][W][C] bf16 (byte offsets < 2^31): per-lane offsets stay 32-bit
// and the per-image base is scalar (no 64-bit address VALU per load)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ch_img_rsrc(const bf16* base, long long img, int img_elems) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)(base + img * img_elems), 0,
                                           __builtin_amdgcn_readfirstlane(img_elems * 2), 0x00020000);
}
// byte offset of halo round i's pixel (clamped into the image) for the lane's 16-B channel chunk hc
// of a 64-channel chunk (the chunk's offset goes into soffset)
__device__ __forceinline__ unsigned ch_halo_off(int p, int oh0, int ow0, int H, int W, int Ci, int hc) {
  const int hy = ch_div18(p), hx = p - hy * CH_W;
  const int ih = min(max(oh0 - 1 + hy, 0), H - 1), iw = min(max(ow0 - 1 + hx, 0), W - 1);
  return (__umul24(__umul24((unsigned)ih, (unsigned)W) + (unsigned)iw, (unsigned)Ci) + (unsigned)hc * 8u) * 2u;
}
// GroupNorm-apply (+ SiLU) of one staged 16-B chunk, zeroed for a pixel outside the image (F.conv2d
// pads the ACTIVATED tensor): packed-f32 math, the select on the four packed words
#ifndef UVA_CONV_SCALAR_GN
#define UVA_CONV_SCALAR_GN 0
#endif
template <bool SILU>
__device__ __forceinline__ bf16x8 ch_gn_act(bf16x8 v, const float (&gsc)[8], const float (&gsh)[8], bool inb) {
  bf16x8 o;
  if constexpr (UVA_CONV_SCALAR_GN != 0) {
    // scalar f32 (the same IEEE operations per element as the packed form below, so the same bits): packed
    // f32 VALU beside MFMAs costs more issue time than two scalar instructions (MI355X_MICROARCH.md)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float u = fmaf((float)v[j], gsc[j], gsh[j]);
      if constexpr (SILU) {
        const float d = __builtin_amdgcn_exp2f(u * -1.4426950408889634f) + 1.f;
        u = u * __builtin_amdgcn_rcpf(d);
      }
      o[j] = (bf16)u;
    }
    ch_u32x4 w = __builtin_bit_cast(ch_u32x4, o);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = inb ? w[k] : 0u;
    return __builtin_bit_cast(bf16x8, w);
  }
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const f32x2 x = {(float)v[j], (float)v[j + 1]};
    f32x2 u = x * (f32x2){gsc[j], gsc[j + 1]} + (f32x2){gsh[j], gsh[j + 1]};
    if constexpr (SILU) {
      const f32x2 t = u * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
      const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + (f32x2){1.f, 1.f};
      u = u * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    }
    o[j] = (bf16)u.x;
    o[j + 1] = (bf16)u.y;
  }
  ch_u32x4 w = __builtin_bit_cast(ch_u32x4, o);
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = inb ? w[k] : 0u;
  return __builtin_bit_cast(bf16x8, w);
}

// s_waitcnt vmcnt(n) for the few counts the 3-slot ring can need (the immediate is compile-time);
// an unlisted count falls back to vmcnt(0) (over-waiting is always safe)
template <int NI, int NR, int NP>
__device__ __forceinline__ void conv_vm_wait(int n) {
#define CVW(V) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(V) : "memory")
  if (n == NI + NR) CVW(NI + NR);
  else if (n == NI + NP) CVW(NI + NP);
  else if (n == NI) CVW(NI);
  else if (n == NR) CVW(NR);
  else if (n == NP) CVW(NP);
  else CVW(0);
#undef CVW
}

// VAR bits (the library builds non-GN = 12 and GN = 64 only): 64 weights in VGPRs (RB below; A
// reads pipelined by k-half across taps measured slower: 5.75 -> 6.16 ms); 4 both k-halves' fragment
// reads issued before the MFMAs (inline-asm reads, counted lgkmcnt); 8 halo staged by LDS-DMA
// (non-GN; no register staging, zeros from the buffer descriptor's range check).  Compile-time
// alternatives measured slower and not built: 16 the next chunk's halo staging spread over taps
// 1..ROUNDS; 2 one halo buffer + a 3-slot weight ring.
#ifndef UVA_CONV_ILV_T0
#define UVA_CONV_ILV_T0 2      // ILV: first tap that stages a round (the halo loads issue at tap 0)
#endif
#ifndef UVA_CONV_ILV_RATIO
#define UVA_CONV_ILV_RATIO 2   // ILV: staging VALU instructions placed after each MFMA
#endif
template <int BN, bool GN, int VAR, int TR, bool SILU = true>
__global__ __launch_bounds__(TR * 32, 16 / TR) void conv3x3_halo(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                       bf16* __restrict__ out, const float* __restrict__ bias,
                                                       const bf16* __restrict__ residual,
                                                       const float* __restrict__ gn_scale,
                                                       const float* __restrict__ gn_shift, int gn_silu,
                                                       float* __restrict__ gn_part, int Nimg, int H, int W, int Ci,
                                                       int Co) {
  constexpr bool R3 = (VAR & 2) != 0;
  constexpr bool HD = (VAR & 8) != 0 && !GN && !R3;
  constexpr bool SPREAD = (VAR & 16) != 0 && !HD && !R3;  // halo staging spread over taps 1..ROUNDS
  // RB (GN only): weight fragments straight from L2 into VGPRs one tap ahead (buffer loads, the
  // K offset in the SGPR soffset) instead of an LDS ring, so the taps need no barrier (one per
  // 64-channel chunk, for the halo swap); padded halo pitch, taps unrolled: every A-fragment read is
  // base + immediate offset (no per-step address VALU)
  constexpr bool RB = (VAR & 64) != 0 && GN && !R3 && !SPREAD;
  // PIPE (RB only): the next tap's A fragment (ks, f) is read into the slot right after the two
  // MFMAs of this tap that consume it, so a tap's LDS reads run under the previous tap's MFMAs
  // (otherwise every tap opens with the latency of its first reads: the 16 fragment registers are
  // reused tap after tap and hipcc issues the next tap's reads only after the last MFMA)
  constexpr bool PIPE = RB && (VAR & 128) != 0;
  // ILV (RB only): the next chunk's GN + SiLU staging is cut into its ROUNDS rounds, one per tap
  // 2..ROUNDS+1, each interleaved instruction by instruction with that tap's 32 MFMAs
  // (sched_group_barrier), so the staging VALU issues in the MFMAs' shadow instead of as a burst
  // after tap 8 (PMC: VALU and MFMA co-execute in 2-3 % of the cycles with the burst)
  constexpr bool ILV = RB && !PIPE && (VAR & 1024) != 0;
  static_assert(!SPREAD || ConvHCfg<BN, TR>::ROUNDS <= 8, "one staging round per tap 1..8");
  static_assert(!RB || TR == 8, "the register epilogue writes one 128-pixel GroupNorm unit per tile");
  using G = ConvHCfg<BN, TR, R3, HD, RB>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = (bf16*)smem;
  bf16* bimg = halo + G::NHB * G::HALO_ELEMS;
  const int tiles_x = W / CH_T, tiles_y = H / TR, ncb = Co / BN;
  const int nblk = Nimg * tiles_y * tiles_x * ncb;
  const int pid = ch_xcd_remap(blockIdx.x, nblk);
  const int cb = pid % ncb;
  const int sp = pid / ncb;  // spatial tile id, image-major
  const int tx = sp % tiles_x, ty = (sp / tiles_x) % tiles_y, n = sp / (tiles_x * tiles_y);
  const int oh0 = ty * TR, ow0 = tx * CH_T, n0 = cb * BN;
  const int K = 9 * Ci, nch = Ci / 64, S = nch * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / G::WN, wn = wid % G::WN;

  // ---- weight tile of step s (chunk s/9, tap s%9) -> ring slot b; K-major [BN][64] image,
  //      16-B chunk c of row r at slot c ^ (r & 7), swizzle applied on the per-lane source
  auto dma_w = [&](int s, int b) {
    const int cc = s / 9, tap = s - cc * 9;
    const bf16* base = wt + (long long)n0 * K + tap * Ci + cc * 64;
    bf16* img = bimg + b * G::BT;
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
      const int e = (wid * G::NI + i) * 512 + lane * 8;
      const int row = e >> 6, slot = (e & 63) >> 3;
      const bf16* src = base + (long long)row * K + ((slot ^ (row & 7)) << 3);
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(img + (wid * G::NI + i) * 512), 16,
                                       0, 0);
    }
  };

  // ---- halo: thread t owns 16-B chunk c = t & 7 of pixels p = (t + NTH i) >> 3
  const int hc = tid & 7;
  bf16x8 hreg[G::ROUNDS];
  float gsc[8], gsh[8];
  const __amdgpu_buffer_rsrc_t rs_in = ch_img_rsrc(in, n, H * W * Ci);
  auto halo_load = [&](int cc) {
#pragma unroll
    for (int i = 0; i < G::ROUNDS; ++i) {
      const int p = min((tid + i * G::NTH) >> 3, G::HPIX - 1);  // clamped pixel: always in bounds
      hreg[i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_in, ch_halo_off(p, oh0, ow0, H, W, Ci, hc), cc * 128, 0));
    }
    if constexpr (GN) {
      const float* sc = gn_scale + (long long)n * Ci + cc * 64 + hc * 8;
      const float* sh = gn_shift + (long long)n * Ci + cc * 64 + hc * 8;
      const float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
      const float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
      gsc[0] = s0.x; gsc[1] = s0.y; gsc[2] = s0.z; gsc[3] = s0.w; gsc[4] = s1.x; gsc[5] = s1.y; gsc[6] = s1.z; gsc[7] = s1.w;
      gsh[0] = h0.x; gsh[1] = h0.y; gsh[2] = h0.z; gsh[3] = h0.w; gsh[4] = h1.x; gsh[5] = h1.y; gsh[6] = h1.z; gsh[7] = h1.w;
    }
  };
  auto halo_store_round = [&](int hb, int i) __attribute__((always_inline)) {
    bf16* img = halo + hb * G::HALO_ELEMS;
    {
      const int p = (tid + i * G::NTH) >> 3;
      if (p < G::HPIX) {
        const int hy = p / CH_W, hx = p - hy * CH_W;
        const int ih = oh0 - 1 + hy, iw = ow0 - 1 + hx;
        bf16x8 v = hreg[i];
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) {
          v = (bf16x8){};
        } else if constexpr (GN) {
          // packed pairs: v_pk_fma / v_pk_mul / v_pk_add for everything but the two transcendentals
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f32x2 x = {(float)v[j], (float)v[j + 1]};
            f32x2 u = x * (f32x2){gsc[j], gsc[j + 1]} + (f32x2){gsh[j], gsh[j + 1]};
            if constexpr (SILU) {
              const f32x2 t = u * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
              const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + (f32x2){1.f, 1.f};
              u = u * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
            }
            v[j] = (bf16)u.x;
            v[j + 1] = (bf16)u.y;
          }
        }
        if constexpr (RB) *(bf16x8*)(img + p * G::PP + hc * 8) = v;
        else *(bf16x8*)(img + p * 64 + ((hc ^ (p & 7)) << 3)) = v;
      }
    }
  };
  auto halo_store = [&](int hb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < G::ROUNDS; ++i) halo_store_round(hb, i);
  };
  // ILV: the same round without branches (one basic block with the MFMAs it is interleaved with):
  // out-of-image pixels by select on the packed words, the pixel index clamped (a clamped thread
  // rewrites pixel HPIX-1 with the value its owner stores)
  auto halo_store_round_bf = [&](int hb, int i) __attribute__((always_inline)) {
    bf16* img = halo + hb * G::HALO_ELEMS;
    const int p = min((tid + i * G::NTH) >> 3, G::HPIX - 1);
    const int hy = ch_div18(p), hx = p - hy * CH_W;
    const int ih = oh0 - 1 + hy, iw = ow0 - 1 + hx;
    const bool inb = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    *(bf16x8*)(img + p * G::PP + hc * 8) = ch_gn_act<SILU>(hreg[i], gsc, gsh, inb);
  };

  // ---- HD: halo by LDS-DMA through a per-image buffer descriptor. LDS pixel block b (8 pixels)
  //      is wave-instruction b; lane l writes pixel 8b + l/8, slot l%8 = channel chunk
  //      (l%8) ^ (p & 7) (the swizzle goes on the source). Pixels outside the image (and the
  //      padding past HPIX) get an offset beyond the descriptor's range: the DMA writes zeros.
  unsigned hoff[HD ? G::HD_I : 1];
  if constexpr (HD) {
#pragma unroll
    for (int i = 0; i < G::HD_I; ++i) {
      const int p = (wid * G::HD_I + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (p & 7);
      const int hy = p / CH_W, hx = p - hy * CH_W;
      const int ih = oh0 - 1 + hy, iw = ow0 - 1 + hx;
      const bool ok = p < G::HPIX && ih >= 0 && ih < H && iw >= 0 && iw < W;
      hoff[i] = ok ? (unsigned)(((ih * W + iw) * Ci + c * 8) * 2) : 0x80000000u;
    }
  }
  auto halo_dma = [&](int cc, int hb) {
    bf16* img = halo + hb * G::HALO_ELEMS;
#pragma unroll
    for (int i = 0; i < G::HD_I; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (__attribute__((address_space(3))) void*)(img + (wid * G::HD_I + i) * 512),
                                               16, (int)hoff[i], cc * 128, 0, 0);
  };

  const int frow = lane & 15, fk = lane >> 4;
  // RB: the product is formed transposed (weights as the MFMA A operand, pixels as B), so lane
  // (frow, fk) accumulates channels c0 + g*16 .. +3 (c0 = n0 + wn*32 + fk*4) of pixel (row f, column
  // frow): one GroupNorm group (Co = 128) or a quarter / half of one in a lane, 8-B output runs, and
  // the epilogue finishes from registers (no LDS image, no barrier); the bias seeds the accumulators
  f32x4 acc[G::FM][G::FN];
#pragma unroll
  for (int j = 0; j < G::FN; ++j) {
    f32x4 b0 = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (RB && bias) {
      const float4 b = *(const float4*)(bias + n0 + wn * (G::FN * 16) + j * 16 + fk * 4);
      b0 = (f32x4){b.x, b.y, b.z, b.w};
    }
#pragma unroll
    for (int i = 0; i < G::FM; ++i) acc[i][j] = b0;
  }
  // RB: B fragment (ks, g) of step s for this lane: 16 B at wt[(n0 + wn*32 + g*16 + frow) * K +
  // tap*Ci + cc*64 + ks*32 + fk*8]; per-lane part in vb[g] (+ ks*64 B immediate), step part in
  // soffset.  Step 0's fragments are issued ahead of the halo so their latency overlaps it.
  __amdgpu_buffer_rsrc_t rs_w;
  int vb[G::FN];
  bf16x8 bq[2][2][G::FN];  // [register set][ks][g]
  auto bload = [&](int s, bf16x8 (&dst)[2][G::FN]) __attribute__((always_inline)) {
    const int cc = s / 9, tap = s - cc * 9;
    const int soff = __builtin_amdgcn_readfirstlane((tap * Ci + cc * 64) * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < G::FN; ++g)
        dst[ks][g] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_w, vb[g] + ks * 64, soff, 0));
  };
  if constexpr (RB) {
    rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)wt, 0, __builtin_amdgcn_readfirstlane(Co * K * 2), 0x00020000);
#pragma unroll
    for (int g = 0; g < G::FN; ++g) vb[g] = ((n0 + wn * (G::FN * 16) + g * 16 + frow) * K + fk * 8) * 2;
    bload(0, bq[0]);
  }

  // ---- prologue: weight tile 0 (and 1 with the 3-slot ring) + halo of chunk 0
  if (!RB) dma_w(0, 0);
  if (R3 && S > 1) dma_w(1, 1);
  if constexpr (HD) {
    halo_dma(0, 0);
  } else {
    halo_load(0);
    halo_store(0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // epilogue geometry.  The first ROUNDS of the tile's residual row chunks are loaded at tap 0 of
  // the LAST chunk into hreg (free there: no next halo), so the step barriers cover their HBM
  // latency (loaded at the epilogue's start, ~1.5-3k cycles stayed exposed per tile, +0.7 ms at
  // the level-0 shape); a separate register array for them spilled the GN variant
  constexpr int C8 = BN / 8, RPP = G::NTH / C8, NHALF = TR / 8;
  const int c8 = tid % C8, rsub = tid / C8;
  const int col0 = n0 + c8 * 8;
  constexpr int NIT = 128 / RPP;
  constexpr int NPRE = G::ROUNDS < NHALF * NIT ? G::ROUNDS : NHALF * NIT;
  auto res_ptr = [&](int idx) {
    const int half = idx / NIT, it = idx % NIT;
    const int rl = it * RPP + rsub;
    const int oh = oh0 + half * 8 + (rl >> 4), ow = ow0 + (rl & 15);
    return (const bf16x8*)(residual + (((long long)n * H + oh) * W + ow) * Co + col0);
  };
  auto res_load = [&]() {
#pragma unroll
    for (int i = 0; i < NPRE; ++i) hreg[i] = *res_ptr(i);
  };
  int prev_loads = 0;  // R3: global loads the previous step issued after its weight DMA
  if constexpr (RB) {
    // A fragment (ks, f) of tap (kh, kw): halo pixel (wm*FM + f + kh, frow + kw), channels
    // (ks*4 + fk)*8.. -> lane base + ((f + kh) * 18 + kw) * PP + ks * 32
    const int abase = (wm * G::FM * CH_W + frow) * G::PP + fk * 8;
    // residual of the lane's outputs (8 B each), loaded at tap 0 of the last chunk (no next halo there)
    // (rows >= RQ_PRE at the epilogue's start: all 8 rows up front spilled)
    constexpr int RQ_PRE = G::ROUNDS < G::FM ? G::ROUNDS : G::FM;
    static_assert(G::FN == 2, "the permlane16 pairing joins the wave's two 16-channel fragments");
    const int c0 = n0 + wn * (G::FN * 16) + fk * 4;
    // residual loads / output stores through per-image descriptors: 32-bit lane offset of (row 0, column
    // frow, the lane's 8-channel run), the row in soffset
    const int cs_ = n0 + wn * (G::FN * 16) + (fk & 1) * 16 + (fk >> 1) * 8;
    const unsigned pbase = (unsigned)(((oh0 * W + ow0 + frow) * Co + cs_) * 2);
    const __amdgpu_buffer_rsrc_t rs_res = ch_img_rsrc(residual, n, H * W * Co);
    const __amdgpu_buffer_rsrc_t rs_out = ch_img_rsrc(out, n, H * W * Co);
    auto res_row = [&](int f) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs_res, pbase, __builtin_amdgcn_readfirstlane(f * W * Co * 2), 0));
    };
    auto chunk_ilv = [&](int cc, auto stc) __attribute__((always_inline)) {
      constexpr bool STG = decltype(stc)::value;  // a next chunk exists: stage it under these taps
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int s = cc * 9 + tap;
        const int cur = tap & 1, nxt = cur ^ 1;
        // unconditional (the last step reloads its own fragments): no branch join before the
        // staging's first use of hreg, where hipcc's merged wait count would drain this load too
        bload(s + 1 < S ? s + 1 : s, bq[nxt]);
        if constexpr (STG) {
          if (tap == 0) halo_load(cc + 1);
        } else {
          if (tap == 0 && residual) {
#pragma unroll
            for (int f = 0; f < RQ_PRE; ++f) hreg[f] = res_row(f);
            if constexpr ((VAR & 256) != 0) {
              // rows RQ_PRE.. into the GroupNorm scale registers (no staging in the last chunk)
#pragma unroll
              for (int f = RQ_PRE; f < G::FM; ++f) {
                const f32x4 v = __builtin_bit_cast(f32x4, res_row(f));
#pragma unroll
                for (int j = 0; j < 4; ++j) gsc[(f - RQ_PRE) * 4 + j] = v[j];
              }
            }
          }
        }
        const int kh = tap / 3, kw = tap % 3;
        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] = *(const bf16x8*)(hcur + ((f + kh) * CH_W + kw) * G::PP + ks * 32);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);
        if constexpr (STG) {
          if (tap >= UVA_CONV_ILV_T0 && tap - UVA_CONV_ILV_T0 < G::ROUNDS) {
            halo_store_round_bf((cc + 1) & 1, tap - UVA_CONV_ILV_T0);
#pragma unroll
            for (int k = 0; k < 28; ++k) {
              __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  // one MFMA
              __builtin_amdgcn_sched_group_barrier(0x002, UVA_CONV_ILV_RATIO, 0);  // VALU of the staging round
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
          }
        }
        __builtin_amdgcn_s_setprio(0);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int g = 0; g < G::FN; ++g) bq[0][ks][g] = bq[1][ks][g];
      if constexpr (STG) ch_lds_barrier();
    };
    if constexpr (ILV) {
      int cc = 0;
      for (; cc + 1 < nch; ++cc) chunk_ilv(cc, std::true_type{});
      chunk_ilv(cc, std::false_type{});
    } else
    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + (cc & 1) * G::HALO_ELEMS + abase;
      const bool more = cc + 1 < nch;
      bf16x8 fp[2][G::FM];  // PIPE: the fragments of the current tap, refilled for the next one
      if constexpr (PIPE) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f) fp[ks][f] = *(const bf16x8*)(hcur + f * CH_W * G::PP + ks * 32);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int s = cc * 9 + tap;
        const int cur = tap & 1, nxt = cur ^ 1;  // tap 8's next set is copied to set 0 below
        if constexpr (PIPE) {
          bload(s + 1 < S ? s + 1 : s, bq[nxt]);  // unconditional: no block boundary inside a chunk
        } else {
          if (s + 1 < S) bload(s + 1, bq[nxt]);
        }
        if (tap == 0 && more) halo_load(cc + 1);
        if (tap == 0 && !more && residual) {
          // rows 0..RQ_PRE-1 into the (now free) halo staging registers (the epilogue's 16-B runs)
#pragma unroll
          for (int f = 0; f < RQ_PRE; ++f) hreg[f] = res_row(f);
          if constexpr ((VAR & 256) != 0) {
            // the remaining rows too, into the GroupNorm scale registers (dead in the last chunk; the
            // same variables, so the allocator needs no new ones): no residual load is left for the
            // epilogue to wait on
            static_assert(G::FM - RQ_PRE <= 2, "two late rows fit gsc");
#pragma unroll
            for (int f = RQ_PRE; f < G::FM; ++f) {
              const f32x4 v = __builtin_bit_cast(f32x4, res_row(f));
#pragma unroll
              for (int j = 0; j < 4; ++j) gsc[(f - RQ_PRE) * 4 + j] = v[j];
            }
          }
        }
        const int kh = tap / 3, kw = tap % 3;
        if constexpr (PIPE) {
          const int kh1 = (tap + 1) / 3, kw1 = (tap + 1) % 3;
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int f = 0; f < G::FM; ++f) {
#pragma unroll
              for (int g = 0; g < G::FN; ++g)
                acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fp[ks][f], acc[f][g], 0, 0, 0);
              __builtin_amdgcn_sched_group_barrier(0x008, G::FN, 0);
              if (tap < 8) {
                fp[ks][f] = *(const bf16x8*)(hcur + ((f + kh1) * CH_W + kw1) * G::PP + ks * 32);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
              }
            }
          __builtin_amdgcn_s_setprio(0);
          continue;
        }
        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] = *(const bf16x8*)(hcur + ((f + kh) * CH_W + kw) * G::PP + ks * 32);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      // tap 8 loaded step s+1 into set 1; the next chunk's tap 0 reads set 0
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int g = 0; g < G::FN; ++g) bq[0][ks][g] = bq[1][ks][g];
      if (more) {
        // every wave is done with chunk cc-1's buffer since the previous chunk barrier: stage the
        // next chunk into it, then one barrier orders the staging before chunk cc+1's reads
        halo_store((cc + 1) & 1);
        ch_lds_barrier();
      }
    }
    // ---- register epilogue.  One v_permlane16_swap per accumulator word pairs lane rows fk, fk^1 so that
    //      each lane holds 8 consecutive channels cs.. of its pixel (16-B runs; the 4 rows of a wave
    //      cover the 64-B channel range of each pixel): 8-channel runs at rows 0/1/2/3 = +0/+16/+8/+24.
    //      Then + residual (16 B), bf16 16-B stores, and the GroupNorm partial sums of the stored
    //      values (lane: its 8 rows; then the 16 columns (lanes frow); then rows fk, fk^2 for gsz 16)
    const int cs = n0 + wn * (G::FN * 16) + (fk & 1) * 16 + (fk >> 1) * 8;
    bf16x8 rq[G::FM];
    if (residual) {
#pragma unroll
      for (int f = 0; f < G::FM; ++f)
        if (f < RQ_PRE) {
          rq[f] = hreg[f];
        } else if constexpr ((VAR & 256) != 0) {
          const int o = ((f - RQ_PRE) & 1) * 4;
          rq[f] = __builtin_bit_cast(bf16x8, (f32x4){gsc[o], gsc[o + 1], gsc[o + 2], gsc[o + 3]});
        } else {
          rq[f] = res_row(f);
        }
    }
    float sa = 0.f, sb = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
    for (int f = 0; f < G::FM; ++f) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][0][i]), __float_as_uint(acc[f][1][i]),
                                                        false, false);
        v[i] = __uint_as_float(r[0]);
        v[4 + i] = __uint_as_float(r[1]);
      }
      if (residual) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rq[f][e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ch_u32x4, o), rs_out, pbase,
                                             __builtin_amdgcn_readfirstlane(f * W * Co * 2), 0);
      if (gn_part) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float q = (float)o[e], w2 = (float)o[4 + e];
          sa += q;
          qa += q * q;
          sb += w2;
          qb += w2 * w2;
        }
      }
    }
    if (gn_part) {
      const int gsz = Co / 32;  // 4 (two groups per lane), 8 (one) or 16 (one, with row fk^2)
      if (gsz >= 8) {
        sa += sb;
        qa += qb;
      }
      sa = row16_sum(sa);
      qa = row16_sum(qa);
      sb = row16_sum(sb);
      qb = row16_sum(qb);
      if (gsz >= 16) {
        sa = xor_lane_sum(sa, 32);
        qa = xor_lane_sum(qa, 32);
      }
      if (frow == 0 && (gsz < 16 || fk < 2)) {
        const long long t128 = (long long)n * (tiles_x * tiles_y) + (sp % (tiles_x * tiles_y));
        float* gp = gn_part + (t128 * 32 + cs / gsz) * 2;
        *(float2*)gp = make_float2(sa, qa);
        if (gsz == 4) *(float2*)(gp + 2) = make_float2(sb, qb);
      }
    }
    return;
  } else
  for (int cc = 0; cc < nch; ++cc) {
    const bf16* hcur = halo + (R3 ? 0 : (cc & 1)) * G::HALO_ELEMS;
    const bool more = cc + 1 < nch;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int s = cc * 9 + tap;
      int cur_loads = 0;
      if constexpr (R3) {
        // ring slot (s+2)%3 was last read in step s-1; every wave passed the barrier that ended it
        if (s + 2 < S) dma_w(s + 2, (s + 2) % 3);
      } else {
        // ring slot (s+1)&1 was last read in step s-1; every wave passed the barrier that ended it
        if (s + 1 < S) dma_w(s + 1, (s + 1) & 1);
      }
      __builtin_amdgcn_sched_barrier(0);  // counted waits below: the weight DMA is issued first
      if (tap == 0 && more) {
        if constexpr (HD) {
          halo_dma(cc + 1, (cc + 1) & 1);  // buffer last read in chunk cc-1
          cur_loads = G::HD_I;
        } else {
          halo_load(cc + 1);
          cur_loads = G::ROUNDS;
        }
      }
      if (tap == 0 && !more && residual) {
        res_load();
        cur_loads = NPRE;
      }
      const bf16* bcur = bimg + (R3 ? s % 3 : (s & 1)) * G::BT;
      const int kh = tap / 3, kw = tap % 3;
      if constexpr ((VAR & 4) != 0) {
        // both k-halves' fragments issued up front: the second half's LDS reads run under the
        // first half's MFMAs
        // inline-asm reads (hipcc drains lgkmcnt(0) before the first MFMA otherwise): the k-half
        // 0 MFMAs wait for the first 8 reads only, completion ordered by asm waits + sched_barrier
        bf16x8 fa[2][G::FM], fb[2][G::FN];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + fk;
#pragma unroll
          for (int f = 0; f < G::FM; ++f) {
            const int p = (wm * G::FM + f + kh) * CH_W + frow + kw;
            fa[ks][f] = lds_read16(hcur + p * 64 + ((c ^ (p & 7)) << 3));
          }
#pragma unroll
          for (int g = 0; g < G::FN; ++g) {
            const int r = wn * (G::FN * 16) + g * 16 + frow;
            fb[ks][g] = lds_read16(bcur + r * 64 + ((c ^ (r & 7)) << 3));
          }
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          if (ks == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(G::FM + G::FN) : "memory");
          else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[ks][f], fb[ks][g], acc[f][g], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
      } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + fk;
        bf16x8 fa[G::FM], fb[G::FN];
#pragma unroll
        for (int f = 0; f < G::FM; ++f) {
          const int p = (wm * G::FM + f + kh) * CH_W + frow + kw;
          fa[f] = *(const bf16x8*)(hcur + p * 64 + ((c ^ (p & 7)) << 3));
        }
#pragma unroll
        for (int g = 0; g < G::FN; ++g) {
          const int r = wn * (G::FN * 16) + g * 16 + frow;
          fb[g] = *(const bf16x8*)(bcur + r * 64 + ((c ^ (r & 7)) << 3));
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int f = 0; f < G::FM; ++f)
#pragma unroll
          for (int g = 0; g < G::FN; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[f], fb[g], acc[f][g], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      }
      if constexpr (R3) {
        // wait for weight tile s+1 only: younger are [this step's W(s+2) DMA] and the global loads
        // issued after W(s+1) -- by the previous step (after its DMA) and by this one. The halo
        // loads of tap 0 so stay in flight until the end of tap 2 (the vector-memory counter
        // retires in issue order); the last step drains everything for the epilogue
        const int younger = s + 1 < S ? prev_loads + (s + 2 < S ? G::NI : 0) + cur_loads : 0;
        conv_vm_wait<G::NI, G::ROUNDS, NPRE>(younger);
        prev_loads = cur_loads;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (tap == 8 && more) {
          // single halo buffer: every wave is done with chunk cc (barrier above); restage it
          halo_store(0);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
      } else if constexpr (HD) {
        // weight tile s+1 only: tap 0's halo DMA / residual loads (issued after it) may stay in
        // flight one more step; every other step drains (its weight DMA is the youngest)
        if (cur_loads == G::HD_I) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::HD_I) : "memory");
        else if (cur_loads == NPRE) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPRE) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      } else if constexpr (SPREAD) {
        // the next chunk's GN + SiLU staging spread over taps 1..ROUNDS, one round per step after
        // this step's MFMAs.  Measured SLOWER than the one burst at tap 8 (level-0 conv 7.12 vs
        // 6.85 ms, same box): the co-resident workgroup already runs its MFMAs under the burst.
        // The halo loads of tap 0 were issued after W(s+1): only they may stay in flight
        if (more) {
#pragma unroll
          for (int i = 0; i < G::ROUNDS; ++i)
            if (tap == 1 + i) halo_store_round((cc + 1) & 1, i);  // buffer last read in chunk cc-1
        }
        if (cur_loads == G::ROUNDS) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::ROUNDS) : "memory");
        else if (cur_loads == NPRE) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPRE) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      } else {
        if (tap == 8 && more) halo_store((cc + 1) & 1);  // buffer last read in chunk cc-1
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    }
  }

  // ---- epilogue: 128-pixel halves (tile rows 0-7 [, 8-15]) staged through LDS as fp32
  float* T = (float*)smem;
  float bv[8];
  if (bias) {
    const float4 b0 = *(const float4*)(bias + col0), b1 = *(const float4*)(bias + col0 + 4);
    bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  }
  const int tiles_img = tiles_x * tiles_y;
  bf16x8 rres[NHALF][NIT];
  if (residual) {
#pragma unroll
    for (int i = 0; i < NHALF * NIT; ++i) rres[i / NIT][i % NIT] = i < NPRE ? hreg[i] : *res_ptr(i);
  }
#pragma unroll
  for (int half = 0; half < NHALF; ++half) {
    if ((wm * G::FM) / 8 == half) {
#pragma unroll
      for (int f = 0; f < G::FM; ++f)
#pragma unroll
        for (int g = 0; g < G::FN; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            T[((wm * G::FM + f - half * 8) * 16 + fk * 4 + r) * G::TP + wn * (G::FN * 16) + g * 16 + frow] = acc[f][g][r];
    }
    ch_lds_barrier();
    float gs[8], gq[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) gs[e] = gq[e] = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int rl = it * RPP + rsub;  // pixel inside the half: row half*8 + rl/16, column rl%16
      const int oh = oh0 + half * 8 + (rl >> 4), ow = ow0 + (rl & 15);
      const long long ob = (((long long)n * H + oh) * W + ow) * Co + col0;
      const float4 a = *(const float4*)(T + rl * G::TP + c8 * 8);
      const float4 b = *(const float4*)(T + rl * G::TP + c8 * 8 + 4);
      float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      if (residual) {
        const bf16x8 rv = rres[half][it];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bv[e], v[e] += (float)rv[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bv[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
      *(bf16x8*)(out + ob) = o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float q = (float)o[e];
        gs[e] += q;
        gq[e] += q * q;
      }
    }
    if (gn_part) {
      // per-column sums over the half's 128 pixels (lanes sharing c8, then the NW waves via LDS)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = C8; o < 64; o <<= 1) {
          gs[e] = xor_lane_sum(gs[e], o);
          gq[e] = xor_lane_sum(gq[e], o);
        }
      }
      float* red = T + 128 * G::TP;  // [NW waves][C8][8][2]
      if (lane < C8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[((wid * C8 + lane) * 8 + e) * 2 + 0] = gs[e];
          red[((wid * C8 + lane) * 8 + e) * 2 + 1] = gq[e];
        }
      }
      ch_lds_barrier();
      // the tile's ngroups groups x (NW waves x gsz channels) partial pairs: 2 per thread, then a
      // shuffle tree over the group's NTH/ngroups consecutive lanes (a serial 32-thread loop over
      // the 64 LDS values of a group cost ~6k cycles per half)
      const int gsz = Co / 32;
      const int ngroups = BN / gsz;               // 32, 16 or 8 (Co = 128, 256, 512)
      const int tpg = G::NTH / ngroups;           // lanes per group (inside one wave)
      const int gl = tid / tpg, j = tid % tpg;
      float sum = 0.f, sq = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int idx = j * 2 + u, w = idx / gsz, c = gl * gsz + idx % gsz;
        sum += red[((w * C8 + (c >> 3)) * 8 + (c & 7)) * 2 + 0];
        sq += red[((w * C8 + (c >> 3)) * 8 + (c & 7)) * 2 + 1];
      }
      for (int o = 1; o < tpg; o <<= 1) {
        sum += __shfl_xor(sum, o, 64);
        sq += __shfl_xor(sq, o, 64);
      }
      if (j == 0) {
        const int g = n0 / gsz + gl;
        const long long t128 = ((long long)n * tiles_img + (sp % tiles_img)) * NHALF + half;
        gn_part[(t128 * 32 + g) * 2 + 0] = sum;
        gn_part[(t128 * 32 + g) * 2 + 1] = sq;
      }
    }
    ch_lds_barrier();
  }
}

// =====================================================================================
// GN conv, strip form (Ci = 128, i.e. two 64-channel chunks): one workgroup walks a vertical strip of
// 8 x 16 tiles (one tile column of one image, top to bottom) instead of one tile.  Consecutive tiles
// of a strip share two halo rows: the bottom two rows of tile ty's 10-row halo ARE the top two of tile
// ty+1's, already GroupNorm'd + SiLU'd in LDS, so each later tile stages 8 new rows (144 of 180 halo
// pixels) and copies two inside LDS -- 20 % less of the GN+SiLU staging (the kernel's VALU: two
// transcendentals per element) and of the halo loads.  With two chunks the buffers never alternate
// away from their chunk (chunk c always lives in buffer c), so both chunks' previous halos are still
// in LDS when the next tile starts.  Everything per tile is the register-B kernel above (weights
// streamed from L2 into VGPRs one tap ahead -- across the tile boundary too -- bias-seeded
// accumulators, register epilogue with bias / residual / GroupNorm partial sums).
// =====================================================================================
template <int VAR>
__global__ __launch_bounds__(256, 2) void conv3x3_gn_strip(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                           bf16* __restrict__ out, const float* __restrict__ bias,
                                                           const bf16* __restrict__ residual,
                                                           const float* __restrict__ gn_scale,
                                                           const float* __restrict__ gn_shift, int gn_silu,
                                                           float* __restrict__ gn_part, int Nimg, int H, int W) {
  using G = ConvHCfg<128, 8, false, false, true>;
  constexpr int Ci = 128, Co = 128, nch = 2, S = 18, K = 9 * Ci;
  constexpr int NEWP = 8 * CH_W;                               // 144 new halo pixels (rows 2..9)
  constexpr int ROUNDS_NEW = (NEWP * 8 + G::NTH - 1) / G::NTH;  // 5
  static_assert(ROUNDS_NEW <= G::ROUNDS, "new-row staging fits the full-staging registers");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = (bf16*)smem;
  const int tiles_x = W / CH_T, tiles_y = H / 8;
  const int nstrip = Nimg * tiles_x;
  const int st = ch_xcd_remap(blockIdx.x, nstrip);
  const int tx = st % tiles_x, n = st / tiles_x;
  const int ow0 = tx * CH_T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wn = __builtin_amdgcn_readfirstlane(tid >> 6);  // WM = 1: wave = 32 output channels
  const int frow = lane & 15, fk = lane >> 4;
  auto opaque = [](int v) __attribute__((always_inline)) {
    asm volatile("" : "+v"(v));
    return v;
  };

  // ---- halo staging.  full: rows 0..9 (tile 0 of the strip); new: rows 2..9 (later tiles)
  bf16x8 hreg[G::ROUNDS];
  float gsc[8], gsh[8];
  auto gn_load = [&](int cc) __attribute__((always_inline)) {
    const int hc = opaque(tid) & 7;
    const float* sc = gn_scale + (long long)n * Ci + cc * 64 + hc * 8;
    const float* sh = gn_shift + (long long)n * Ci + cc * 64 + hc * 8;
    const float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
    const float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
    gsc[0] = s0.x; gsc[1] = s0.y; gsc[2] = s0.z; gsc[3] = s0.w; gsc[4] = s1.x; gsc[5] = s1.y; gsc[6] = s1.z; gsc[7] = s1.w;
    gsh[0] = h0.x; gsh[1] = h0.y; gsh[2] = h0.z; gsh[3] = h0.w; gsh[4] = h1.x; gsh[5] = h1.y; gsh[6] = h1.z; gsh[7] = h1.w;
  };
  // pixel of staging round i: full p in [0, 180), new p in [36, 180)
  // (the thread index goes through an empty asm so the per-round pixel geometry is recomputed at each
  // use instead of being hoisted out of the strip loop into ~40 long-lived registers, which spilled)
  auto pix_of = [&](bool full, int i) __attribute__((always_inline)) {
    const int t = opaque(tid);
    return full ? (t + i * G::NTH) >> 3 : 2 * CH_W + ((t + i * G::NTH) >> 3);
  };
  auto halo_load = [&](bool full, int oh0, int cc) __attribute__((always_inline)) {
    const int hc = opaque(tid) & 7;
    const int nr = full ? G::ROUNDS : ROUNDS_NEW;
#pragma unroll
    for (int i = 0; i < G::ROUNDS; ++i) {
      if (i < nr) {
        const int p = min(pix_of(full, i), G::HPIX - 1);
        const int hy = p / CH_W, hx = p - hy * CH_W;
        const int ih = min(max(oh0 - 1 + hy, 0), H - 1), iw = min(max(ow0 - 1 + hx, 0), W - 1);
        hreg[i] = *(const bf16x8*)(in + (((long long)n * H + ih) * W + iw) * Ci + cc * 64 + hc * 8);
      }
    }
    gn_load(cc);
  };
  auto halo_store = [&](bool full, int oh0, int hb) __attribute__((always_inline)) {
    bf16* img = halo + hb * G::HALO_ELEMS;
    const int hc = opaque(tid) & 7;
    const int nr = full ? G::ROUNDS : ROUNDS_NEW;
#pragma unroll
    for (int i = 0; i < G::ROUNDS; ++i) {
      const int p = pix_of(full, i);
      if (i < nr && p < G::HPIX) {
        const int hy = p / CH_W, hx = p - hy * CH_W;
        const int ih = oh0 - 1 + hy, iw = ow0 - 1 + hx;
        if (!full && p >= 8 * CH_W) {
          // rows 8,9 of the previous tile are rows 0,1 of this one: this thread is the only one that
          // overwrites this 16-B slot, so moving it first needs no barrier
          *(bf16x8*)(img + (p - 8 * CH_W) * G::PP + hc * 8) = *(const bf16x8*)(img + p * G::PP + hc * 8);
        }
        bf16x8 v = hreg[i];
        if (ih < 0 || ih >= H || iw < 0 || iw >= W) {
          v = (bf16x8){};
        } else {
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const f32x2 x = {(float)v[j], (float)v[j + 1]};
            f32x2 u = x * (f32x2){gsc[j], gsc[j + 1]} + (f32x2){gsh[j], gsh[j + 1]};
            if (gn_silu) {
              const f32x2 t = u * (f32x2){-1.4426950408889634f, -1.4426950408889634f};
              const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + (f32x2){1.f, 1.f};
              u = u * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
            }
            v[j] = (bf16)u.x;
            v[j + 1] = (bf16)u.y;
          }
        }
        *(bf16x8*)(img + p * G::PP + hc * 8) = v;
      }
    }
  };
  // ---- weights: B fragment (ks, g) of step s = 16 B at wt[(wn*32 + g*16 + frow) * K + tap*Ci + cc*64 + ks*32 + fk*8]
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc((void*)wt, 0, __builtin_amdgcn_readfirstlane(Co * K * 2), 0x00020000);
  int vb[G::FN];
#pragma unroll
  for (int g = 0; g < G::FN; ++g) vb[g] = ((wn * (G::FN * 16) + g * 16 + frow) * K + fk * 8) * 2;
  bf16x8 bq[2][2][G::FN];
  auto bload = [&](int s, bf16x8 (&dst)[2][G::FN]) __attribute__((always_inline)) {
    const int cc = s / 9, tap = s - cc * 9;
    const int soff = __builtin_amdgcn_readfirstlane((tap * Ci + cc * 64) * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < G::FN; ++g)
        dst[ks][g] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_w, vb[g] + ks * 64, soff, 0));
  };
  bload(0, bq[0]);

  // ---- tile 0 of the strip: chunk 0's full halo; chunk 1's full halo is staged at tap 8 of chunk 0
  halo_load(true, 0, 0);
  halo_store(true, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int abase = frow * G::PP + fk * 8;
  constexpr int RQ_PRE = G::ROUNDS < G::FM ? G::ROUNDS : G::FM;
  const int cs = wn * (G::FN * 16) + (fk & 1) * 16 + (fk >> 1) * 8;  // the lane's 8-channel output run
#pragma unroll 1
  for (int ty = 0; ty < tiles_y; ++ty) {
    const int oh0 = ty * 8;
    const bool first = ty == 0, last = ty + 1 == tiles_y;
    const long long pix0 = ((long long)n * H + oh0) * W + ow0 + frow;
    f32x4 acc[G::FM][G::FN];  // bias-seeded (re-read per tile from L1: no registers held across tiles)
#pragma unroll
    for (int j = 0; j < G::FN; ++j) {
      f32x4 b0 = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (bias) {
        const float4 b = *(const float4*)(bias + wn * (G::FN * 16) + j * 16 + fk * 4);
        b0 = (f32x4){b.x, b.y, b.z, b.w};
      }
#pragma unroll
      for (int f = 0; f < G::FM; ++f) acc[f][j] = b0;
    }
#pragma unroll 1
    for (int cc = 0; cc < nch; ++cc) {
      const bf16* hcur = halo + cc * G::HALO_ELEMS + opaque(abase);
      const bool more = cc + 1 < nch;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int s = cc * 9 + tap;
        const int cur = tap & 1, nxt = cur ^ 1;
        if (s + 1 < S) bload(s + 1, bq[nxt]);
        else if (!last) bload(0, bq[nxt]);  // the next tile's first step: same weights
        if (tap == 0 && more) halo_load(first, oh0, cc + 1);
        if (tap == 0 && !more && residual) {
#pragma unroll
          for (int f = 0; f < RQ_PRE; ++f) hreg[f] = *(const bf16x8*)(residual + (pix0 + (long long)f * W) * Co + cs);
        }
        const int kh = tap / 3, kw = tap % 3;
        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] = *(const bf16x8*)(hcur + ((f + kh) * CH_W + kw) * G::PP + ks * 32);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int g = 0; g < G::FN; ++g) bq[0][ks][g] = bq[1][ks][g];
      if (more) {
        // chunk 1's buffer: every wave finished the previous tile's chunk 1 before the tile-start
        // barrier (for ty > 0 its rows 0,1 were refilled there)
        halo_store(first, oh0, 1);
        ch_lds_barrier();
      }
    }
    // ---- register epilogue (as the register-B kernel)
    bf16x8 rq[G::FM];
    if (residual) {
#pragma unroll
      for (int f = 0; f < G::FM; ++f)
        rq[f] = f < RQ_PRE ? hreg[f] : *(const bf16x8*)(residual + (pix0 + (long long)f * W) * Co + cs);
    }
    float sa = 0.f, sb = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
    for (int f = 0; f < G::FM; ++f) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][0][i]), __float_as_uint(acc[f][1][i]),
                                                        false, false);
        v[i] = __uint_as_float(r[0]);
        v[4 + i] = __uint_as_float(r[1]);
      }
      if (residual) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rq[f][e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
      *(bf16x8*)(out + (pix0 + (long long)f * W) * Co + cs) = o;
      if (gn_part) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float q = (float)o[e], w2 = (float)o[4 + e];
          sa += q;
          qa += q * q;
          sb += w2;
          qb += w2 * w2;
        }
      }
    }
    if (gn_part) {
      // Co = 128: GroupNorm(32) groups of 4 channels, two per lane
      sa = row16_sum(sa);
      qa = row16_sum(qa);
      sb = row16_sum(sb);
      qb = row16_sum(qb);
      if (frow == 0) {
        const long long t128 = (long long)n * (tiles_x * tiles_y) + ty * tiles_x + tx;
        float* gp = gn_part + (t128 * 32 + cs / 4) * 2;
        *(float2*)gp = make_float2(sa, qa);
        *(float2*)(gp + 2) = make_float2(sb, qb);
      }
    }
    if (!last) {
      // next tile's chunk-0 halo (new rows 2..9; rows 0,1 moved inside LDS); chunk 1's new rows are
      // loaded at tap 0 of the next tile's chunk 0 and stored after it, as in the single-tile kernel
      halo_load(false, oh0 + 8, 0);
      ch_lds_barrier();  // every wave is past its reads of this tile's halos
      halo_store(false, oh0 + 8, 0);
      ch_lds_barrier();
    }
  }
}

// =====================================================================================
// GN conv, persistent form (PT; Ci = Co = 128): 2 workgroups per CU walk tiles
// pid = i * grid + xcd_remap(block).  The register-B / interleaved-staging tile body of
// conv3x3_halo, plus: during a tile's LAST chunk the NEXT tile's chunk 0 is loaded (tap 0) and its
// GN + SiLU staging interleaved with the MFMAs (taps 2..7) into halo buffer 0 -- free since chunk 0's
// barrier -- so a tile starts with its halo already in LDS instead of the load-latency + staging
// burst + barrier every single-tile workgroup opens with.  The residual rows reuse the staging
// registers as they free up (row r at tap 3 + r; rows 6, 7 in the GroupNorm scale registers at tap
// 8).  After the grid's last tile the current tile is restaged (harmless: nothing reads it).
// =====================================================================================
template <bool SILU>
__global__ __launch_bounds__(256, 2) void conv3x3_gn_pt(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                        bf16* __restrict__ out, const float* __restrict__ bias,
                                                        const bf16* __restrict__ residual,
                                                        const float* __restrict__ gn_scale,
                                                        const float* __restrict__ gn_shift, int gn_silu,
                                                        float* __restrict__ gn_part, int Nimg, int H, int W) {
  using G = ConvHCfg<128, 8, false, false, true>;
  constexpr int Ci = 128, Co = 128, S = 18, K = 9 * Ci;
  static_assert(G::ROUNDS == 6 && G::FM == 8 && G::FN == 2, "tile geometry of the register-B body");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = (bf16*)smem;
  const int tiles_x = W / CH_T, tiles_y = H / 8, ntiles = Nimg * tiles_x * tiles_y;
  const int G_ = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fk = lane >> 4;
  // the thread index goes through an empty asm at each use: otherwise hipcc hoists every round's
  // pixel geometry (and the residual row addresses) out of the tile loop into long-lived registers
  auto opaque = [](int v) __attribute__((always_inline)) {
    asm volatile("" : "+v"(v));
    return v;
  };
  struct Tile {
    int n, oh0, ow0;
  };
  auto tile_of = [&](int pid) __attribute__((always_inline)) {
    Tile t;
    const int tx = pid % tiles_x, ty = (pid / tiles_x) % tiles_y;
    t.n = pid / (tiles_x * tiles_y);
    t.oh0 = ty * 8;
    t.ow0 = tx * CH_T;
    return t;
  };
  bf16x8 hreg[G::ROUNDS];
  float gsc[8], gsh[8];
  auto halo_load = [&](const Tile& t, int cc) __attribute__((always_inline)) {
    const int tid = opaque(threadIdx.x), hc = tid & 7;
    const __amdgpu_buffer_rsrc_t rs_in = ch_img_rsrc(in, t.n, H * W * Ci);
#pragma unroll
    for (int i = 0; i < G::ROUNDS; ++i) {
      const int p = min((tid + i * G::NTH) >> 3, G::HPIX - 1);
      hreg[i] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_in, ch_halo_off(p, t.oh0, t.ow0, H, W, Ci, hc), cc * 128, 0));
    }
    const float* sc = gn_scale + (long long)t.n * Ci + cc * 64 + hc * 8;
    const float* sh = gn_shift + (long long)t.n * Ci + cc * 64 + hc * 8;
    const float4 s0 = *(const float4*)sc, s1 = *(const float4*)(sc + 4);
    const float4 h0 = *(const float4*)sh, h1 = *(const float4*)(sh + 4);
    gsc[0] = s0.x; gsc[1] = s0.y; gsc[2] = s0.z; gsc[3] = s0.w; gsc[4] = s1.x; gsc[5] = s1.y; gsc[6] = s1.z; gsc[7] = s1.w;
    gsh[0] = h0.x; gsh[1] = h0.y; gsh[2] = h0.z; gsh[3] = h0.w; gsh[4] = h1.x; gsh[5] = h1.y; gsh[6] = h1.z; gsh[7] = h1.w;
  };
  // branch-free staging round (as conv3x3_halo's ILV round)
  auto stage_round = [&](const Tile& t, int hb, int i) __attribute__((always_inline)) {
    const int tid = opaque(threadIdx.x), hc = tid & 7;
    bf16* img = halo + hb * G::HALO_ELEMS;
    const int p = min((tid + i * G::NTH) >> 3, G::HPIX - 1);
    const int hy = ch_div18(p), hx = p - hy * CH_W;
    const int ih = t.oh0 - 1 + hy, iw = t.ow0 - 1 + hx;
    const bool inb = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    *(bf16x8*)(img + p * G::PP + hc * 8) = ch_gn_act<SILU>(hreg[i], gsc, gsh, inb);
  };
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc((void*)wt, 0, __builtin_amdgcn_readfirstlane(Co * K * 2), 0x00020000);
  int vb[G::FN];
#pragma unroll
  for (int g = 0; g < G::FN; ++g) vb[g] = ((wn * (G::FN * 16) + g * 16 + frow) * K + fk * 8) * 2;
  bf16x8 bq[2][2][G::FN];
  auto bload = [&](int s, bf16x8 (&dst)[2][G::FN]) __attribute__((always_inline)) {
    const int cc = s / 9, tap = s - cc * 9;
    const int soff = __builtin_amdgcn_readfirstlane((tap * Ci + cc * 64) * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < G::FN; ++g)
        dst[ks][g] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_w, vb[g] + ks * 64, soff, 0));
  };
  const int abase = frow * G::PP + fk * 8;
  const int cs = wn * (G::FN * 16) + (fk & 1) * 16 + (fk >> 1) * 8;  // the lane's 8-channel output run

  int pid = ch_xcd_remap(blockIdx.x, G_);
  if (pid >= ntiles) return;
  Tile cur = tile_of(pid);
  bload(0, bq[0]);
  halo_load(cur, 0);
#pragma unroll
  for (int i = 0; i < G::ROUNDS; ++i) stage_round(cur, 0, i);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (;;) {
    const int npid = pid + G_;
    const bool more = npid < ntiles;
    const Tile nxt = tile_of(more ? npid : pid);
    // residual loads / output stores through per-image descriptors: 32-bit lane offset of (row 0,
    // column frow, the lane's 8-channel run), the row in soffset
    const unsigned obase = (unsigned)(((cur.oh0 * W + cur.ow0 + frow) * Co + cs) * 2);
    const __amdgpu_buffer_rsrc_t rs_res = ch_img_rsrc(residual, cur.n, H * W * Co);
    auto res_row = [&](int f) __attribute__((always_inline)) {
      return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                            rs_res, obase, __builtin_amdgcn_readfirstlane(f * W * Co * 2), 0));
    };
    f32x4 acc[G::FM][G::FN];
#pragma unroll
    for (int j = 0; j < G::FN; ++j) {
      f32x4 b0 = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (bias) {
        const float4 b = *(const float4*)(bias + wn * (G::FN * 16) + j * 16 + fk * 4);
        b0 = (f32x4){b.x, b.y, b.z, b.w};
      }
#pragma unroll
      for (int f = 0; f < G::FM; ++f) acc[f][j] = b0;
    }
    // LAST = 0: chunk 0, staging this tile's chunk 1 into buffer 1
    // LAST = 1: chunk 1, staging the next tile's chunk 0 into buffer 0 + the residual rows
    auto chunk = [&](auto lc) __attribute__((always_inline)) {
      constexpr int LAST = decltype(lc)::value;
      const bf16* hcur = halo + LAST * G::HALO_ELEMS + opaque(abase);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int s = LAST * 9 + tap;
        const int cb = tap & 1, nb = cb ^ 1;
        bload(s + 1 < S ? s + 1 : 0, bq[nb]);  // after the last step: the next tile's step 0
        // chunk 0: this tile's chunk 1 loads at tap 0 (staged at taps 2..7), the NEXT tile's chunk 0
        // at tap 8 (staged during chunk 1's taps 1..6), so the residual rows can follow the staging
        // rounds as they free their registers: row r at tap r + 2, rows 6, 7 at tap 7
        if constexpr (!LAST) {
          if (tap == 0) halo_load(cur, 1);
          if (tap == 8) halo_load(nxt, 0);
        } else {
          if (tap >= 2 && tap < 8 && residual) hreg[tap - 2] = res_row(tap - 2);
          if (tap == 7 && residual) {
#pragma unroll
            for (int f = 6; f < 8; ++f) {
              const f32x4 v = __builtin_bit_cast(f32x4, res_row(f));
#pragma unroll
              for (int j = 0; j < 4; ++j) gsc[(f - 6) * 4 + j] = v[j];
            }
          }
        }
        const int kh = tap / 3, kw = tap % 3;
        bf16x8 fa[2][G::FM];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
            fa[ks][f] = *(const bf16x8*)(hcur + ((f + kh) * CH_W + kw) * G::PP + ks * 32);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int f = 0; f < G::FM; ++f)
#pragma unroll
            for (int g = 0; g < G::FN; ++g)
              acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cb][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);
        constexpr int T0 = LAST ? 1 : 2;
        if (tap >= T0 && tap - T0 < G::ROUNDS) {
          if constexpr (LAST) stage_round(nxt, 0, tap - T0);
          else stage_round(cur, 1, tap - T0);
#pragma unroll
          for (int k = 0; k < 28; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int g = 0; g < G::FN; ++g) bq[0][ks][g] = bq[1][ks][g];
      // chunk 0: buffer 1 staged, every wave done with buffer 0 (restaged during chunk 1);
      // chunk 1: the next tile's buffer 0 staged, every wave done with buffer 1
      ch_lds_barrier();
    };
    chunk(std::integral_constant<int, 0>{});
    chunk(std::integral_constant<int, 1>{});

    // ---- register epilogue (as conv3x3_halo's register-B form, Co = 128: two groups per lane)
    const __amdgpu_buffer_rsrc_t rs_out = ch_img_rsrc(out, cur.n, H * W * Co);
    float sa = 0.f, sb = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
    for (int f = 0; f < G::FM; ++f) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][0][i]), __float_as_uint(acc[f][1][i]),
                                                        false, false);
        v[i] = __uint_as_float(r[0]);
        v[4 + i] = __uint_as_float(r[1]);
      }
      if (residual) {
        const bf16x8 rq = f < 6 ? hreg[f]
                                : __builtin_bit_cast(bf16x8, (f32x4){gsc[(f - 6) * 4], gsc[(f - 6) * 4 + 1],
                                                                     gsc[(f - 6) * 4 + 2], gsc[(f - 6) * 4 + 3]});
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)rq[e];
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
      // per-image descriptor, 32-bit lane offset, the row in soffset (no 64-bit address registers
      // live across the tile loop: they spilled)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ch_u32x4, o), rs_out, obase,
                                             __builtin_amdgcn_readfirstlane(f * W * Co * 2), 0);
      if (gn_part) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float q = (float)o[e], w2 = (float)o[4 + e];
          sa += q;
          qa += q * q;
          sb += w2;
          qb += w2 * w2;
        }
      }
    }
    if (gn_part) {
      sa = row16_sum(sa);
      qa = row16_sum(qa);
      sb = row16_sum(sb);
      qb = row16_sum(qb);
      if (frow == 0) {
        float* gp = gn_part + ((long long)pid * 32 + cs / 4) * 2;  // Co = 128: tile = pid
        *(float2*)gp = make_float2(sa, qa);
        *(float2*)(gp + 2) = make_float2(sb, qb);
      }
    }
    if (!more) break;
    pid = npid;
    cur = nxt;
  }
}

// =====================================================================================
// Downsample conv (vaekl.py:59-72: F.pad(x, (0, 1, 0, 1)) then 3x3 / stride 2 / no padding) as a
// halo-tile kernel.  Output tile 8 x 16 pixels x 128 channels, 256 threads, two workgroups per CU;
// per 64-channel chunk the 17 x 33-pixel input halo (zero past the bottom / right edge = the pad)
// is staged ONCE in LDS -- the implicit-GEMM route re-gathered every input element 2.25x from L2
// (455 TFLOP/s at the level-0 shape) -- with the columns de-interleaved into an even plane (17
// pixels per row) and an odd plane (16): tap column kw = 0 / 1 / 2 of output column ow reads
// pixel ow / ow / ow + 1 of the even / odd / even plane, so every A fragment is 16 CONSECUTIVE
// pixels of one plane row, as in the stride-1 kernel.  Channel-chunk-major image: 16-B chunk c of
// plane pixel p at (c * 576 + p) * 16 B, so a fragment read is 16 consecutive 16-B slots (no bank
// conflict) at the lane's base + a compile-time offset (an XOR swizzle made every address a VALU
// computation and spilled), 73.7 KB per workgroup.  The halo is written by LDS-DMA (buffer loads
// into LDS, 16 B per lane, 18 wave-instructions per wave all in flight at once, per-lane source
// offsets computed once).  Level-0 shape (n256 256x256 C128), same box: implicit-GEMM route 2.72 ms
// (455 TFLOP/s); VGPR-staged fill (~3 loads per thread in flight) 2.56; this 2.07-2.15 ms (~590).
// Rejected: 32-channel chunks double-buffered so chunk cc + 1's DMA runs under chunk cc's taps
// (2.26 ms; a weight ring one chunk deep so no waited load follows the DMA: 2.50) -- two workgroups
// per CU already overlap one's fill with the other's taps.
// Weights as in the register-B stride-1 kernel: the transposed product (weights = A operand,
// pixels = B), each wave 32 output channels x the tile's 128 pixels, weight fragments streamed
// from L2 into VGPRs one tap ahead (buffer loads, K offset in soffset); bias-seeded accumulators;
// register epilogue (permlane16 pairing into 16-B channel runs) with the GroupNorm(32) partial
// sums of the stored output per 128-pixel tile for the next level's first GroupNorm.
// =====================================================================================
#define S2_HW 33                      // halo columns: 2 x 16 + 1
#define S2_HH 17                      // halo rows: 2 x 8 + 1
#define S2_PE (S2_HH * 17)            // even-plane pixels (17 per row); the odd plane follows (16 per row)
#define S2_HPIX (S2_HH * S2_HW)       // 561
#define S2_CS 576                     // slots per channel chunk (561 rounded up to whole wave-instructions)
#define S2_DI 18                      // LDS-DMA wave-instructions per wave: 8 * 576 / 64 / 4
#define S2_LDS (S2_CS * 8 * 16)       // 73728 B
__global__ __launch_bounds__(256, 2) void conv3x3s2_kernel(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                          bf16* __restrict__ out, const float* __restrict__ bias,
                                                          float* __restrict__ gn_part, int Nimg, int Hin, int Win,
                                                          int Ci, int Co) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* halo = (bf16*)smem;
  constexpr int FM = 8, FN = 2;
  const int Hout = Hin / 2, Wout = Win / 2;
  const int tiles_x = Wout / 16, tiles_y = Hout / 8, ncb = Co / 128;
  const int nblk = Nimg * tiles_y * tiles_x * ncb;
  const int pid = ch_xcd_remap(blockIdx.x, nblk);
  const int cb = pid % ncb, sp = pid / ncb;
  const int tx = sp % tiles_x, ty = (sp / tiles_x) % tiles_y, n = sp / (tiles_x * tiles_y);
  const int oh0 = ty * 8, ow0 = tx * 16, n0 = cb * 128;
  const int ih0 = 2 * oh0, iw0 = 2 * ow0;
  const int K = 9 * Ci, nch = Ci / 64, S = nch * 9;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wn = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, fk = lane >> 4;

  // chunk cc of the input halo -> LDS by LDS-DMA through a per-image descriptor: slot j = 64 b + lane
  // of wave-instruction b = wid * 18 + i holds chunk c = j / 576 of plane pixel p = j % 576; the
  // channel chunk cc goes in soffset.  Pixels past the bottom / right edge (the F.pad border) and
  // the slots past 561 get an offset beyond the descriptor's range: the DMA writes zeros.
  const __amdgpu_buffer_rsrc_t rs_in = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(in + (long long)n * Hin * Win * Ci), 0, __builtin_amdgcn_readfirstlane(Hin * Win * Ci * 2), 0x00020000);
  unsigned hoff[S2_DI];
#pragma unroll
  for (int i = 0; i < S2_DI; ++i) {
    const int j = (wn * S2_DI + i) * 64 + lane;
    const int c = j / S2_CS, p = j - c * S2_CS;
    const bool odd = p >= S2_PE;
    const int q = odd ? p - S2_PE : p, wdt = odd ? 16 : 17;
    const int hy = q / wdt, hx = 2 * (q - hy * wdt) + (odd ? 1 : 0);
    const int ih = ih0 + hy, iw = iw0 + hx;
    hoff[i] = (p < S2_HPIX && ih < Hin && iw < Win) ? (unsigned)(((ih * Win + iw) * Ci + c * 8) * 2) : 0x80000000u;
  }
  auto halo_fill = [&](int cc) __attribute__((always_inline)) {
    const int soff = __builtin_amdgcn_readfirstlane(cc * 128);
#pragma unroll
    for (int i = 0; i < S2_DI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_in, (__attribute__((address_space(3))) void*)(halo + (wn * S2_DI + i) * 512),
                                               16, (int)hoff[i], soff, 0, 0);
  };

  // bias-seeded accumulators: acc[f][g] = out[pixel (row f, column frow)][channel n0 + wn*32 + g*16 + fk*4 + r]
  f32x4 acc[FM][FN];
#pragma unroll
  for (int g = 0; g < FN; ++g) {
    f32x4 b0 = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (bias) {
      const float4 b = *(const float4*)(bias + n0 + wn * 32 + g * 16 + fk * 4);
      b0 = (f32x4){b.x, b.y, b.z, b.w};
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[f][g] = b0;
  }
  // weight fragment (ks, g) of step s: 16 B at wt[(n0 + wn*32 + g*16 + frow) * K + tap*Ci + cc*64 + ks*32 + fk*8]
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc((void*)wt, 0, __builtin_amdgcn_readfirstlane(Co * K * 2), 0x00020000);
  int vb[FN];
#pragma unroll
  for (int g = 0; g < FN; ++g) vb[g] = ((n0 + wn * 32 + g * 16 + frow) * K + fk * 8) * 2;
  bf16x8 bq[2][2][FN];  // [register set][ks][g]
  auto bload = [&](int s, bf16x8 (&dst)[2][FN]) __attribute__((always_inline)) {
    const int cc = s / 9, tap = s - cc * 9;
    const int soff = __builtin_amdgcn_readfirstlane((tap * Ci + cc * 64) * 2);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < FN; ++g)
        dst[ks][g] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs_w, vb[g] + ks * 64, soff, 0));
  };
  bload(0, bq[0]);
  const bf16* abase = halo + (fk * S2_CS + frow) * 8;  // lane part of every A fragment address

  for (int cc = 0; cc < nch; ++cc) {
    if (cc > 0) ch_lds_barrier();  // every wave is done with chunk cc-1's halo
    halo_fill(cc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int s = cc * 9 + tap;
      const int cur = tap & 1, nxt = cur ^ 1;  // tap 8's next set is copied to set 0 below
      if (s + 1 < S) bload(s + 1, bq[nxt]);
      const int kh = tap / 3, kw = tap % 3;
      bf16x8 fa[2][FM];
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int hy = 2 * f + kh;
        const int p0 = kw == 1 ? S2_PE + hy * 16 : hy * 17 + (kw == 2 ? 1 : 0);  // compile-time
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) fa[ks][f] = *(const bf16x8*)(abase + (ks * 4 * S2_CS + p0) * 8);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[cur][ks][g], fa[ks][f], acc[f][g], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int g = 0; g < FN; ++g) bq[0][ks][g] = bq[1][ks][g];
  }

  // ---- register epilogue (as the stride-1 register-B kernel): channel runs cs .. cs + 7 of pixel
  //      (row f, column frow), bf16 16-B stores, GroupNorm partial sums of the stored values
  const long long pix0 = ((long long)n * Hout + oh0) * Wout + ow0 + frow;
  const int cs = n0 + wn * 32 + (fk & 1) * 16 + (fk >> 1) * 8;
  float sa = 0.f, sb = 0.f, qa = 0.f, qb = 0.f;
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][0][i]), __float_as_uint(acc[f][1][i]),
                                                      false, false);
      v[i] = __uint_as_float(r[0]);
      v[4 + i] = __uint_as_float(r[1]);
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
    *(bf16x8*)(out + (pix0 + (long long)f * Wout) * Co + cs) = o;
    if (gn_part) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float q = (float)o[e], w2 = (float)o[4 + e];
        sa += q;
        qa += q * q;
        sb += w2;
        qb += w2 * w2;
      }
    }
  }
  if (gn_part) {
    const int gsz = Co / 32;  // 4 (two groups per lane), 8 (one) or 16 (one, with row fk^2)
    if (gsz >= 8) {
      sa += sb;
      qa += qb;
    }
    sa = row16_sum(sa);
    qa = row16_sum(qa);
    sb = row16_sum(sb);
    qb = row16_sum(qb);
    if (gsz >= 16) {
      sa = xor_lane_sum(sa, 32);
      qa = xor_lane_sum(qa, 32);
    }
    if (frow == 0 && (gsz < 16 || fk < 2)) {
      const long long t128 = (long long)n * (tiles_x * tiles_y) + (sp % (tiles_x * tiles_y));
      float* gp = gn_part + (t128 * 32 + cs / gsz) * 2;
      *(float2*)gp = make_float2(sa, qa);
      if (gsz == 4) *(float2*)(gp + 2) = make_float2(sb, qb);
    }
  }
}

extern "C" int uva_conv3x3s2_ok(int Nimg, int Hin, int Win, int Ci, int Co) {
  return Nimg > 0 && Hin % 16 == 0 && Win % 32 == 0 && Ci % 64 == 0 && Ci >= 64 && Co % 128 == 0 &&
         (long long)Co * 9 * Ci * 2 < (1LL << 31);
}

extern "C" int uva_conv3x3s2_halo(const void* in, const void* w, void* out, const float* bias, int Nimg, int Hin,
                                  int Win, int Ci, int Co, float* gn_part, hipStream_t stream) {
  if (Nimg <= 0) return 0;
  if (!uva_conv3x3s2_ok(Nimg, Hin, Win, Ci, Co) || (((uintptr_t)in | (uintptr_t)w | (uintptr_t)out) % 16))
    return (int)hipErrorInvalidValue;
  const long long nblk = (long long)Nimg * (Hin / 16) * (Win / 32) * (Co / 128);
  if (nblk >= (1ll << 31)) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3x3s2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, S2_LDS);
    attr = true;
  }
  conv3x3s2_kernel<<<dim3((unsigned)nblk), 256, S2_LDS, stream>>>((const bf16*)in, (const bf16*)w, (bf16*)out, bias,
                                                                   gn_part, Nimg, Hin, Win, Ci, Co);
  UVA_LAUNCH_CHECK();
  return 0;
}

// eligibility of the halo kernel (host side mirror: native/ops.py conv_halo_ok)
static int halo_bn(int Nimg, int H, int W, int Ci, int Co) {
  if (H % CH_T || W % CH_T || Ci % 64 || Ci < 64) return 0;
  const long long tiles = (long long)Nimg * (H / CH_T) * (W / CH_T);
  (void)tiles;  // BN = 256 (2 x 4 waves of 128 x 64) spills at 256 VGPRs in this form: 128 only
  if (Co % 128 == 0) return 128;
  return 0;
}

extern "C" int uva_conv3x3_halo_bn(int Nimg, int H, int W, int Ci, int Co) { return halo_bn(Nimg, H, W, Ci, Co); }

extern "C" int uva_conv3x3_halo(const void* in, const void* w, void* out, const float* bias, const void* residual,
                                int Nimg, int H, int W, int Ci, int Co, const float* gn_scale, const float* gn_shift,
                                int gn_silu, float* gn_part, hipStream_t stream) {
  if (Nimg <= 0) return 0;
  const int bn = halo_bn(Nimg, H, W, Ci, Co);
  if (!bn || (((uintptr_t)in | (uintptr_t)w | (uintptr_t)out | (uintptr_t)residual) % 16)) return (int)hipErrorInvalidValue;
  if ((gn_scale == nullptr) != (gn_shift == nullptr)) return (int)hipErrorInvalidValue;
  // 8-row tiles: two co-resident 256-thread workgroups per CU (16-row tiles at one 512-thread
  // workgroup per CU measured slower: level-0 7.54 vs 6.77 ms)
  constexpr int tr = 8;
  const long long nblk = (long long)Nimg * (H / tr) * (W / CH_T) * (Co / bn);
  if (nblk >= (1ll << 31)) return (int)hipErrorInvalidValue;
#define CH_LAUNCH(BNV, GNV, VARV, TRV, SILUV)                                                                  \
  do {                                                                                                         \
    static bool attr = false;                                                                                  \
    const int lb = ConvHCfg<BNV, TRV, ((VARV) & 2) != 0, ((VARV) & 8) != 0 && !(GNV) && !((VARV) & 2),          \
                            ((VARV) & 64) != 0 && (GNV) && !((VARV) & 2) && !((VARV) & 16)>::LDS_BYTES;          \
    if (!attr) {                                                                                               \
      (void)hipFuncSetAttribute((const void*)conv3x3_halo<BNV, GNV, VARV, TRV, SILUV>,                        \
                                hipFuncAttributeMaxDynamicSharedMemorySize, lb);                               \
      attr = true;                                                                                             \
    }                                                                                                          \
    conv3x3_halo<BNV, GNV, VARV, TRV, SILUV><<<dim3((unsigned)nblk), TRV * 32, lb, stream>>>(                  \
        (const bf16*)in, (const bf16*)w, (bf16*)out, bias, (const bf16*)residual, gn_scale, gn_shift, gn_silu, \
        gn_part, Nimg, H, W, Ci, Co);                                                                          \
  } while (0)
  // non-GN: 12 = halo by LDS-DMA (8) + both k-halves' fragment reads issued up front (4);
  // GN: 64 = weights in VGPRs, one barrier per chunk (same-box level-0 conv 6.61 -> 6.49 ms with the
  // bias + residual + GN-stats epilogue, 7.02 -> 6.79 ms in the bench).  The other VAR bits are the
  // measured-slower alternatives, compile-time only and not built.
#ifndef UVA_CONV_GN_VAR
#define UVA_CONV_GN_VAR 1088
#endif
#ifndef UVA_CONV_GN_STRIP
#define UVA_CONV_GN_STRIP 0
#endif
#ifndef UVA_CONV_GN_PT
#define UVA_CONV_GN_PT 1
#endif
#ifndef UVA_CONV_GN_PT_RES
#define UVA_CONV_GN_PT_RES 0
#endif
  if (gn_scale && Ci == 128 && Co == 128 && (residual == nullptr || (UVA_CONV_GN_PT_RES)) && (UVA_CONV_GN_PT)) {
    // persistent form (above): two workgroups per CU.  Without a residual only: with one, its late
    // rows cost what the next tile's early halo saves (level 0 6.61 vs 6.64 ms; without: 6.25 ->
    // 6.15-6.19 ms, level 1 1.575 -> 1.55 ms; profiles/r04/ab_gnconv_persistent.txt)
    using GS = ConvHCfg<128, 8, false, false, true>;
    static bool attr_p = false;
    static int cus = 0;
    if (!attr_p) {
      (void)hipFuncSetAttribute((const void*)conv3x3_gn_pt<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                GS::LDS_BYTES);
      (void)hipFuncSetAttribute((const void*)conv3x3_gn_pt<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                GS::LDS_BYTES);
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
      attr_p = true;
    }
    const long long grid = std::min<long long>(nblk, 2LL * cus);
    if (gn_silu)
      conv3x3_gn_pt<true><<<dim3((unsigned)grid), 256, GS::LDS_BYTES, stream>>>(
          (const bf16*)in, (const bf16*)w, (bf16*)out, bias, (const bf16*)residual, gn_scale, gn_shift, gn_silu,
          gn_part, Nimg, H, W);
    else
      conv3x3_gn_pt<false><<<dim3((unsigned)grid), 256, GS::LDS_BYTES, stream>>>(
          (const bf16*)in, (const bf16*)w, (bf16*)out, bias, (const bf16*)residual, gn_scale, gn_shift, gn_silu,
          gn_part, Nimg, H, W);
    UVA_LAUNCH_CHECK();
    return 0;
  }
  if (gn_scale && Ci == 128 && Co == 128 && (UVA_CONV_GN_STRIP)) {
    // strip form (above): one workgroup per (image, tile column)
    using GS = ConvHCfg<128, 8, false, false, true>;
    static bool attr_s = false;
    if (!attr_s) {
      (void)hipFuncSetAttribute((const void*)conv3x3_gn_strip<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                GS::LDS_BYTES);
      attr_s = true;
    }
    conv3x3_gn_strip<0><<<dim3((unsigned)(Nimg * (W / CH_T))), 256, GS::LDS_BYTES, stream>>>(
        (const bf16*)in, (const bf16*)w, (bf16*)out, bias, (const bf16*)residual, gn_scale, gn_shift, gn_silu, gn_part,
        Nimg, H, W);
    UVA_LAUNCH_CHECK();
    return 0;
  }
  if (gn_scale && gn_silu) CH_LAUNCH(128, true, UVA_CONV_GN_VAR, 8, true);
  else if (gn_scale) CH_LAUNCH(128, true, UVA_CONV_GN_VAR, 8, false);
  else CH_LAUNCH(128, false, 12, 8, true);
#undef CH_LAUNCH
  UVA_LAUNCH_CHECK();
  return 0;
}

// =====================================================================================
// conv_in: 3x3 / s1 / p1 from the 8-channel padded RGB frame (vaekl.py:246-249 Encoder.conv_in,
// Ci = 3 zero-padded to 8 by uva_resize_select) to Co = 128.  K = 9 taps x 8 = 72 -> three
// 16x16x32 MFMA k-steps (k-group = one tap; taps 9..11 are zero).  The op is bound by its
// 16.8 MB/image bf16 output stream, so the kernel is built around the store:
//   * transposed product D^T = W . X^T: rows = output channels, so each lane's accumulator
//     holds 4 CONSECUTIVE channels = exactly one GroupNorm(32) group of one pixel;
//   * the 16 x 16 x 8 input tile + halo (5 KB) is staged once in LDS; weights live in registers;
//   * per 16-pixel row: 24 MFMAs, bias, bf16, GN partial sums, then the 16 px x 128 ch tile goes
//     through a per-wave LDS slab so the global stores are 4 fully contiguous 1-KiB wave stores.
// =====================================================================================
// weights and bias staged in LDS once per workgroup, which then walks CI_TPW consecutive 16x16
// tiles; padded LDS pitches (weights 224 B, output slab 272 B) keep every fragment read and slab
// write conflict-free or 2-way.  The first form (weights in 96 VGPRs, unpadded slab: 16-way
// conflicts on every slab write, 600M conflict cycles per launch) took 1.78 ms at the level-0 shape,
// this one 1.38 ms.  Taps 9..13 of the padded weight row are zero, so every read is unconditional.
#define CI_WK 112  // weight row pitch (elements): 12 taps x 8 + 16 pad -> conflict-free ds_read_b128 (224 B)
#define CI_SP 136  // slab pixel pitch (elements): 128 + 8 pad (unpadded, the 16 lanes of a b64 write
                   // hit one bank: 16-way conflicts, 600M conflict cycles per launch)
#define CI_TPW 4   // tiles per workgroup
__global__ __launch_bounds__(256) void conv_in_kernel(const bf16* __restrict__ in, const bf16* __restrict__ wt,
                                                      const float* __restrict__ bias, bf16* __restrict__ out,
                                                      float* __restrict__ gn_part, int Nimg, int H, int W) {
  __shared__ __attribute__((aligned(16))) bf16 sx[CH_HPIX * 8];
  __shared__ __attribute__((aligned(16))) bf16 sw[128 * CI_WK];
  __shared__ __attribute__((aligned(16))) bf16 slab[4][16 * CI_SP];
  __shared__ float sb[128];
  __shared__ float red[4][32][2];
  const int tiles_x = W / CH_T, tiles_y = H / CH_T;
  const int ntiles = Nimg * tiles_x * tiles_y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int frow = lane & 15, fk = lane >> 4;
  // weights [128][72] -> LDS [128][CI_WK] (16-B chunks; chunks 9..13 of each row zero)
  for (int i = tid; i < 128 * 14; i += 256) {
    const int r = i / 14, c = i - r * 14;
    bf16x8 v = (bf16x8){};
    if (c < 9) v = *(const bf16x8*)(wt + r * 72 + c * 8);
    *(bf16x8*)(sw + r * CI_WK + c * 8) = v;
  }
  if (tid < 128) sb[tid] = bias ? bias[tid] : 0.f;
  bf16* myslab = slab[wid];
  // halo of a tile: 324 pixels x 16 B, 2 per thread, loaded into registers one tile AHEAD (the
  // load of tile t+1 is in flight while tile t computes; loaded at the tile's start, its HBM
  // latency was exposed once per tile)
  constexpr int HR = (CH_HPIX + 255) / 256;
  bf16x8 hv[HR];
  auto halo_ld = [&](int sp) {
    const int tx = sp % tiles_x, ty = (sp / tiles_x) % tiles_y, n = sp / (tiles_x * tiles_y);
#pragma unroll
    for (int i = 0; i < HR; ++i) {
      const int p = tid + i * 256;
      const int hy = p / CH_H, hx = p - hy * CH_H;
      const int ih = ty * CH_T - 1 + hy, iw = tx * CH_T - 1 + hx;
      hv[i] = (bf16x8){};
      if (p < CH_HPIX && ih >= 0 && ih < H && iw >= 0 && iw < W)
        hv[i] = *(const bf16x8*)(in + (((long long)n * H + ih) * W + iw) * 8);
    }
  };
  const int sp_end = min(ntiles, (int)(blockIdx.x + 1) * CI_TPW);
  if ((int)blockIdx.x * CI_TPW < sp_end) halo_ld(blockIdx.x * CI_TPW);
#pragma unroll 1
  for (int sp = blockIdx.x * CI_TPW; sp < sp_end; ++sp) {
    const int tx = sp % tiles_x, ty = (sp / tiles_x) % tiles_y, n = sp / (tiles_x * tiles_y);
    const int oh0 = ty * CH_T, ow0 = tx * CH_T;
    // (the previous tile's readers passed the barrier ending its iteration)
#pragma unroll
    for (int i = 0; i < HR; ++i)
      if (tid + i * 256 < CH_HPIX) *(bf16x8*)(sx + (tid + i * 256) * 8) = hv[i];
    __syncthreads();
    if (sp + 1 < sp_end) halo_ld(sp + 1);
    float gs[8], gq[8];
#pragma unroll
    for (int f = 0; f < 8; ++f) gs[f] = gq[f] = 0.f;
#pragma unroll 1
    for (int rr = 0; rr < 4; ++rr) {
      const int row = wid * 4 + rr;  // tile row
      bf16x8 xf[3];
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int tap = ks * 4 + fk;
        const int kh = tap / 3, kw = tap % 3;
        xf[ks] = tap < 9 ? *(const bf16x8*)(sx + ((row + kh) * CH_H + frow + kw) * 8) : (bf16x8){};
      }
      // acc[f][r] = out[pixel frow][channel f*16 + fk*4 + r]   (A = weights: row = channel f*16 + frow).
      // k-step-major issue: 8 independent accumulators between dependent MFMAs (f-major, the three
      // chained MFMAs of each f stalled on one another and on the accumulator read-back)
      f32x4 acc[8];
#pragma unroll
      for (int f = 0; f < 8; ++f) acc[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        bf16x8 wf[8];
#pragma unroll
        for (int f = 0; f < 8; ++f) wf[f] = *(const bf16x8*)(sw + (f * 16 + frow) * CI_WK + (ks * 4 + fk) * 8);
#pragma unroll
        for (int f = 0; f < 8; ++f) acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[f], xf[ks], acc[f], 0, 0, 0);
      }
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        const float4 b4 = *(const float4*)(sb + f * 16 + fk * 4);
        const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
        bf16x4 o;
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (bf16)(acc[f][r] + bb[r]);
          const float v = (float)o[r];
          s += v;
          q += v * v;
        }
        gs[f] += s;
        gq[f] += q;
        *(bf16x4*)(myslab + frow * CI_SP + f * 16 + fk * 4) = o;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): slab writes done (wave-private slab)
      __builtin_amdgcn_wave_barrier();
      const long long ob = (((long long)n * H + oh0 + row) * W + ow0) * 128;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = (i * 64 + lane) * 8;  // 16 px x 128 ch contiguous in NHWC
        *(bf16x8*)(out + ob + e) = *(const bf16x8*)(myslab + (e >> 7) * CI_SP + (e & 127));
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (gn_part) {
      // group g = f*4 + fk: reduce over the 16 pixel lanes sharing fk
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        gs[f] = row16_sum(gs[f]);
        gq[f] = row16_sum(gq[f]);
      }
      if (frow == 0) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          red[wid][f * 4 + fk][0] = gs[f];
          red[wid][f * 4 + fk][1] = gq[f];
        }
      }
      __syncthreads();
      if (tid < 64) {
        const int half = tid >> 5, g = tid & 31;  // half 0 = waves 0,1 (tile rows 0-7)
        const float s = red[half * 2][g][0] + red[half * 2 + 1][g][0];
        const float q = red[half * 2][g][1] + red[half * 2 + 1][g][1];
        const long long t128 = ((long long)n * tiles_x * tiles_y + (sp % (tiles_x * tiles_y))) * 2 + half;
        gn_part[(t128 * 32 + g) * 2 + 0] = s;
        gn_part[(t128 * 32 + g) * 2 + 1] = q;
      }
    }
    __syncthreads();  // sx / red reused by the next tile
  }
}

extern "C" int uva_conv_in8(const void* in, const void* w, void* out, const float* bias, int Nimg, int H, int W,
                            float* gn_part, hipStream_t stream) {
  if (Nimg <= 0) return 0;
  if (H % CH_T || W % CH_T || (((uintptr_t)in | (uintptr_t)w | (uintptr_t)out) % 16)) return (int)hipErrorInvalidValue;
  const long long nblk = ((long long)Nimg * (H / CH_T) * (W / CH_T) + CI_TPW - 1) / CI_TPW;
  conv_in_kernel<<<dim3((unsigned)nblk), 256, 0, stream>>>((const bf16*)in, (const bf16*)w, bias, (bf16*)out, gn_part,
                                                           Nimg, H, W);
  UVA_LAUNCH_CHECK();
  return 0;
}

