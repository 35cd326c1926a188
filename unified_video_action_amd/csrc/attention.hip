// Fused multi-head attention (non-causal, head_dim 64, bf16 in/out, fp32 softmax) for the
// 24 timm Blocks of the MAR (mar_con_unified.py:201-249; timm Attention = SDPA with
// dropout_p = attn_drop while training).  Reads Q/K/V straight from the qkv GEMM output
// [B, N, 3, H, 64] and writes O as [B, N, H, 64] (the proj GEMM input) -- no permutes.
//
// Layout trick (CDNA4 v_mfma_f32_16x16x32_bf16, 64-lane waves): forward scores are computed
// transposed, S^T = K Q^T, so each lane owns one query column (lane & 15) and 16 keys in
// registers.  P^T then feeds O^T = V^T P^T directly as the B operand (no LDS round trip):
// the k order inside each 32-deep step is the permutation pi(8g+j) = tileA*16+4g+j (j<4),
// tileB*16+4g+j-4 (j>=4), matched on the V side by choosing the row bases of the two
// ds_read_b64_tr_b16 transposed reads.  Softmax statistics are per lane (query); the O^T
// rescale is lazy (only when a row max grows by > 2^8, wave-uniform branch) and the row sum
// stays lane-partial until the epilogue.
//
// Dropout (attn_drop p): the keep decision of element (b,h,q,key) is the counter hash of
// ((b*H+h)*N+q)*N+key (common.h, shared with the materialised softmax path).  One mask
// kernel evaluates it once per step and writes two bit planes in the lane orders of the
// MFMA kernels, so forward and backward only test bits (v_bfe_i32 + v_and per element):
//   MQ [bh][key tile kv][q]   u64, bit g*16+kt*4+r  <-> key kv*64 + kt*16 + 4g + r
//   MK [bh][query tile qb][key] u64, bit g*16+qt*4+r <-> query qb*64 + qt*16 + 4g + r
// (the 16 bits a lane of quad g needs are the u16 at offset g).  MK comes from MQ's rows by a
// 6-stage 64x64 bit transpose across the wave (lane L computes the query whose MK bit is L).
//
// Backward (two kernels, FA2 recompute, no atomics -> bitwise reproducible):
//   attn_bwd_dkdv : block = 128 keys (4 waves x 32), sweeps all 64-query tiles; S and dP with
//                   the key on the lane, so Pd and dS are already the B operands of
//                   dV^T += dO'^T Pd and dK^T += Q^T dS (pi order).
//   attn_bwd_dq   : block = 128 queries, sweeps all 64-key tiles (forward's lane view).
// A fused single pass with dQ summed by fp32 atomics was measured slower at this shape: d = 64
// gives only 640 FLOP per atomic byte, so the 0.8 GB of dQ adds per layer ran at the chip's
// atomic rate (+0.28 ms per layer), more than the recomputed S/dP of the dQ kernel costs.
// The dropout scale dsc = 1 / (1 - p) never enters the loops: they run on the unscaled dO with
// D' = rowsum(dO * O) / dsc formed by the dQ kernel, which runs first (dS = dsc P (keep dP - D')), and dsc multiplies dK,
// dQ and dV once when they are stored.
#include "common.h"

#ifndef UVA_ATT_PIPE
#define UVA_ATT_PIPE 0
#endif
#ifndef UVA_ATT_PIPE_DQ
#define UVA_ATT_PIPE_DQ 0
#endif
// UVA_ATT_PRIO: s_setprio(1) around the MFMA blocks, so that on a SIMD the wave in its matrix phase
// wins the issue slots over the co-resident wave's softmax / staging phase (the GN conv measured
// 37 % slower without its equivalent)
// forward: on (0.162-0.168 vs 0.166-0.171 ms at B32/N1024/H12); backward: off (p = 0.1: 0.70 vs
// 0.49 ms -- the barrier the builtin puts in hipcc's schedule splits the dropout-bit / softmax
// interleave), profiles/r04/ab_attn_setprio.txt
#ifndef UVA_ATT_PRIO
#define UVA_ATT_PRIO 1
#endif
#ifndef UVA_ATT_PRIO_BWD
#define UVA_ATT_PRIO_BWD 0
#endif
#define ATT_PRIO_HI() do { if (UVA_ATT_PRIO) __builtin_amdgcn_s_setprio(1); } while (0)
#define ATT_PRIO_LO() do { if (UVA_ATT_PRIO) __builtin_amdgcn_s_setprio(0); } while (0)
#define ATT_PRIO_HI_BWD() do { if (UVA_ATT_PRIO_BWD) __builtin_amdgcn_s_setprio(1); } while (0)
#define ATT_PRIO_LO_BWD() do { if (UVA_ATT_PRIO_BWD) __builtin_amdgcn_s_setprio(0); } while (0)
// 64 x 64 bf16 tile images with 160-B rows (80 elements).  Under gfx950's LDS lane groups
// (MI355X_MICROARCH.md 'LDS banking': ds_read_b128 in 4 x 16 lanes {0-3,12-15,20-27} ...,
// ds_read_b64_tr_b16 in 2 x 32) both fragment reads below are conflict-free
// (tools/lds_swizzle_check.py); 144-B rows (72) cost 2 LDS cycles per lane group on both
// (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.40-0.43 in every attention kernel,
// profiles/r05/pmc_attn_lds.txt).  A linear stride keeps every fragment address base + immediate (an
// XOR-swizzled 128-B row, also conflict-free, put the compile-time ks / dt bits under the XOR: the
// forward with dropout ran 16 % slower).
#define AT_LD 80
#define AT_TILE (64 * AT_LD)

__device__ __forceinline__ bf16x8 lds_row_frag(const bf16* lds, int row0, int ks) {
  const int l = threadIdx.x & 63;
  return *(const bf16x8*)(lds + (row0 + (l & 15)) * AT_LD + ks * 32 + 8 * (l >> 4));
}

__device__ __forceinline__ bf16x8 lds_tr_frag(const bf16* lds, int rowA, int rowB, int col0) {
  const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const bf16* a0 = lds + (rowA + 4 * g + q) * AT_LD + col0 + 4 * p;
  const bf16* a1 = lds + (rowB + 4 * g + q) * AT_LD + col0 + 4 * p;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// two f32 -> one dword of two bf16 (RNE, as the (bf16) cast): one v_cvt_pk_bf16_f32 per pair.  Plain
// casts of individually masked values compiled to one cvt per element + a v_perm per pair.
// (a vector conversion, not inline asm: the result feeds MFMAs, whose operand hazards hipcc only
// tracks for instructions it emitted itself)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
__device__ __forceinline__ bf16x8 pack_pi(const f32x4& a, const f32x4& b) {
  const u32x4 u = {cvt_pk_bf16(a[0], a[1]), cvt_pk_bf16(a[2], a[3]), cvt_pk_bf16(b[0], b[1]), cvt_pk_bf16(b[2], b[3])};
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 64 rows x 64 cols of a strided bf16 matrix -> 2 chunks (16 B) per thread.  Tiles are always
// full (N % 64 == 0 is an ABI precondition), so no per-row guard (its exec-mask branches
// serialised the loads); the uniform tile base is formed once, per-thread offsets are hoisted.
__device__ __forceinline__ void stage_load(const bf16* __restrict__ g, long long ld, int row0, int nrows,
                                           bf16x8 (&r)[2]) {
  (void)nrows;
  const int t = threadIdx.x;
  const bf16* base = g + (long long)row0 * ld;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = t + i * 256, row = id >> 3, c = (id & 7) * 8;
    r[i] = *(const bf16x8*)(base + (long long)row * ld + c);
  }
}
__device__ __forceinline__ void stage_store(bf16* lds, const bf16x8 (&r)[2]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int id = t + i * 256, row = id >> 3, c = (id & 7) * 8;
    *(bf16x8*)(lds + row * AT_LD + c) = r[i];
  }
}

// workgroup barrier that orders LDS only: outstanding global loads / atomics stay in flight
// (__syncthreads would drain vmcnt, i.e. wait for every dQ atomic of the tile)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }
// keep-bit b of a mask word as an all-ones / all-zeros 32-bit mask.  (A v_bfe_i32 in inline asm
// saves hipcc's v_and + v_cmp + v_cndmask lowering but measured slower in the dK/dV loop: the
// asm statements constrain its scheduling.)
__device__ __forceinline__ float keep_and(float v, uint32_t w, int b) {
  return __int_as_float(__float_as_int(v) & __builtin_amdgcn_sbfe(w, b, 1));
}
// the same as two instructions (v_bfe_i32 + v_and_b32): from the builtin form hipcc derives a bit test
// + v_cmp + v_cndmask (three) in the forward and dQ loops
__device__ __forceinline__ float keep_bfe(float v, uint32_t w, int b) {
  int m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(w), "s"(b));
  return __int_as_float(__float_as_int(v) & m);
}
// max of two MFMA outputs without the canonicalising v_max hipcc inserts in front of fmaxf
// (med3(a, b, +inf) == max(a, b); the compiler fuses chains of it into v_max3_f32)
__device__ __forceinline__ float fmax_nc(float a, float b) { return __builtin_amdgcn_fmed3f(a, b, INFINITY); }
// max over lanes l, l^16, l^32, l^48 by v_permlane16/32_swap (VALU) instead of two ds_bpermute.
// Builtins only: an inline-asm producer is invisible to hipcc's permlane / trans / MFMA hazard
// wait-state insertion (an asm v_max feeding the second swap read a stale register).
__device__ __forceinline__ float quad_max(float v) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// position of element k (0..63) of a 64-wide tile inside an MQ / MK word (an involution)
__host__ __device__ constexpr int mask_pos(int k) { return ((k >> 2) & 3) * 16 + (k >> 4) * 4 + (k & 3); }

// =====================================================================================
// dropout bit planes: one wave per (bh, query tile qb, MASK_TPW consecutive key tiles)
// =====================================================================================
// Lane L hashes the 32 pairs of (query q, 64 keys of tile kv) and shifts each element's DROP bit
// (the sign of u16 - th) into its plane word by v_alignbit, visiting positions 63..0 in descending
// order (pair j holds positions mask_pos(2j), even, and +1): two ops per element instead of the
// and / sub / shift / or sequence (hash-only floor 65 us, kernel 81 vs 108 us at B32 N1024 H12,
// bit-identical planes; tools/probe/mask_probe.hip).  Several key tiles per wave amortise the
// (wave-uniform) index arithmetic.
constexpr int MASK_TPW = 4;
__device__ __forceinline__ uint32_t shift_in_sign(uint32_t acc, uint32_t t) {
  return __builtin_amdgcn_alignbit(acc, t, 31);  // (acc << 1) | (t >> 31)
}
__global__ __launch_bounds__(256) void attn_mask_kernel(uint64_t* __restrict__ MQ, uint64_t* __restrict__ MK, int N,
                                                        int nt, long long waves, uint32_t th, uint64_t seed) {
  // wave index in an SGPR (the host bounds waves < 2^31), so the index divisions are scalar
  const long long wv = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4u + (threadIdx.x >> 6)));
  if (wv >= waves) return;  // wave-uniform
  const int L = threadIdx.x & 63;
  const int per_row = (nt + MASK_TPW - 1) / MASK_TPW;
  const int kv0 = (int)(wv % per_row) * MASK_TPW;
  const long long t2 = wv / per_row;
  const int qb = (int)(t2 % nt);
  const long long bh = t2 / nt;
  const int q = qb * 64 + mask_pos(L);  // lane L holds the query whose MK bit is L
  const uint32_t key = drop_key(seed);
  const uint64_t rowpair = (((uint64_t)bh * N + q) * (uint64_t)N) >> 1;
#pragma unroll 1
  for (int kv = kv0; kv < kv0 + MASK_TPW && kv < nt; ++kv) {
    // pair0 = rowpair + 32 kv is a multiple of 32 (N % 64 == 0), so pair0 + j (j < 32) changes only
    // its low 5 bits: drop_hash's first word for pair j is x0 ^ j
    const uint32_t x0 = drop_first(key, rowpair + (uint64_t)kv * 32);
    uint32_t lo = 0, hi = 0;  // DROP bits of this lane's query (bit mask_pos(k) <-> key kv*64 + k)
#pragma unroll
    for (int P = 31; P >= 0; --P) {
      const uint32_t x = drop_mix(x0 ^ (uint32_t)(mask_pos(2 * P) >> 1));
      const uint32_t t0 = (x & 0xFFFFu) - th, t1 = (x >> 16) - th;  // dropped iff negative
      if (P >= 16) {
        hi = shift_in_sign(shift_in_sign(hi, t1), t0);
      } else {
        lo = shift_in_sign(shift_in_sign(lo, t1), t0);
      }
    }
    lo = ~lo;
    hi = ~hi;
    MQ[((long long)bh * nt + kv) * N + q] = ((uint64_t)hi << 32) | lo;
    // 64x64 bit transpose across the wave (rows = lanes): afterwards lane L' holds, at bit L, the
    // bit mask_pos(L') of lane L, i.e. keep(query with MK position L, key kv*64 + mask_pos(L')).
    // Branch-free: per stage the lane's shift amounts and keep mask are selects, the exchange a
    // ds_swizzle (xor within 32 lanes) or v_permlane32_swap (the 32-lane stage).
    {
      const bool up = L & 32;
      const auto r = __builtin_amdgcn_permlane32_swap(up ? lo : hi, up ? lo : hi, false, false);
      const uint32_t o = up ? r[0] : r[1];  // the other half's word
      if (up) lo = o; else hi = o;
    }
#define UVA_TSTAGE(J, M)                                                                    \
  {                                                                                         \
    const bool up = L & (J);                                                                \
    const uint32_t sr = up ? 0u : (uint32_t)(J); /* down lanes send and receive the high halves */ \
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

// =====================================================================================
// forward
// =====================================================================================
// KT = keys per LDS tile: 64 at three waves per SIMD (168 VGPRs, 36.9 KB of
// LDS per workgroup): the loop is latency-bound (PMC: 0.39 of wave-cycles issue-stalled, MFMA busy
// 0.20, VALU active 0.33 at two waves per SIMD), so the third wave buys more than the 128-key tile's
// longer compute rounds (0.167 vs 0.174 ms at B32 N1024 H12 p0.1, same box).  A 32x32x16 variant
// (a quarter of the MFMA issue slots, conflict-free XOR-swizzled LDS images, per-subtile software
// pipelining) used fewer cycles but ran 15-20 % slower in wall time: the 32x32 shape holds a lower
// clock under load (MI355X_MICROARCH 'DVFS give-back' item 7).
template <bool DROP, int KT, int OCC>
__global__ __launch_bounds__(256, OCC) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                       float* __restrict__ lse2, const uint64_t* __restrict__ MQ,
                                                       int N, int H, float c, float dsc) {
  constexpr int NKT = KT / 16;   // 16-key MFMA tiles per LDS tile
  constexpr int NH = KT / 64;    // 64-key mask words per LDS tile
  __shared__ __attribute__((aligned(16))) bf16 sK[2][NH * AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][NH * AT_TILE];
  int bx, bh;
  xcd_grid2(bx, bh);
  const int b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int q0 = bx * 128 + w * 32;
  const int nkv = N / KT, n64 = N / 64;
  const uint16_t* mq = DROP ? (const uint16_t*)(MQ + (long long)bh * n64 * N) : nullptr;  // [kv64][q][4 x u16]

  bf16x8 qf[2][2];
  uint32_t mw[2][NH], mwn[2][NH];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int row = q0 + qt * 16 + li;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = row < N ? *(const bf16x8*)(Qg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
#pragma unroll
    for (int hh = 0; hh < NH; ++hh) {
      mw[qt][hh] = (DROP && row < N) ? mq[((long long)hh * N + row) * 4 + g] : 0u;
      mwn[qt][hh] = 0u;
    }
  }
  float m[2] = {-INFINITY, -INFINITY}, rs[2] = {0.f, 0.f};
  f32x4 o[2][4];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rk[NH][2], rv[NH][2];
#pragma unroll
  for (int hh = 0; hh < NH; ++hh) {
    stage_load(Kg, ld, hh * 64, N, rk[hh]);
    stage_load(Vg, ld, hh * 64, N, rv[hh]);
  }
#pragma unroll
  for (int hh = 0; hh < NH; ++hh) {
    stage_store(sK[0] + hh * AT_TILE, rk[hh]);
    stage_store(sV[0] + hh * AT_TILE, rv[hh]);
  }
  __syncthreads();
  int cur = 0;
  for (int kv = 0; kv < nkv; ++kv) {
    const bool more = kv + 1 < nkv;
    if (more) {
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        stage_load(Kg, ld, (kv + 1) * KT + hh * 64, N, rk[hh]);
        stage_load(Vg, ld, (kv + 1) * KT + hh * 64, N, rv[hh]);
      }
      if (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const int row = q0 + qt * 16 + li;
#pragma unroll
          for (int hh = 0; hh < NH; ++hh)
            mwn[qt][hh] = row < N ? mq[((long long)((kv + 1) * NH + hh) * N + row) * 4 + g] : 0u;
        }
      }
    }
    const bf16* cK = sK[cur];
    const bf16* cV = sV[cur];
    f32x4 s[NKT][2];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    ATT_PRIO_HI();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        const bf16x8 kf = lds_row_frag(cK, kt * 16, ks);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) s[kt][qt] = mfma16(kf, qf[qt][ks], s[kt][qt]);
      }
    }
    ATT_PRIO_LO();
    // row max (lane: NKT*4 keys of its query; the 4 quads of a query meet through two shuffles)
    float mx[2];
    bool need = false;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      // (the lane's scores come straight from the MFMAs: inline-asm VALU on them would bypass the
      // compiler's MFMA-result hazard wait states, so this chain stays on builtins -- hipcc fuses it
      // into v_max3_f32)
      float a = fmax_nc(s[0][qt][0], s[0][qt][1]);
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = (kt == 0 ? 2 : 0); r < 4; ++r) a = fmax_nc(a, s[kt][qt][r]);
      a = quad_max(a);
      mx[qt] = a * c;
      need |= mx[qt] > m[qt] + 8.0f;
    }
    // lazy rescale: the reference max only moves when some row grew by more than 2^8
    if (__builtin_amdgcn_ballot_w64(need)) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const float mnew = fmaxf(m[qt], mx[qt]);
        const float alpha = exp2_fast(m[qt] - mnew);
        rs[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
        m[qt] = mnew;
      }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const float nm = -m[qt];
      float ps[4] = {0.f, 0.f, 0.f, 0.f};  // four independent partial row sums
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2_fast(fmaf(s[kt][qt][r], c, nm));
          ps[r] += p;
          s[kt][qt][r] = DROP ? keep_bfe(p, mw[qt][kt >> 2], (kt & 3) * 4 + r) : p;
        }
      rs[qt] += (ps[0] + ps[1]) + (ps[2] + ps[3]);
    }
    ATT_PRIO_HI();
#pragma unroll
    for (int ks = 0; ks < KT / 32; ++ks) {
      bf16x8 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) pf[qt] = pack_pi(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 vf = lds_tr_frag(cV, 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) o[qt][dt] = mfma16(vf, pf[qt], o[qt][dt]);
      }
    }
    ATT_PRIO_LO();
    if (more) {
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        stage_store(sK[cur ^ 1] + hh * AT_TILE, rk[hh]);
        stage_store(sV[cur ^ 1] + hh * AT_TILE, rv[hh]);
      }
      if (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int hh = 0; hh < NH; ++hh) mw[qt][hh] = mwn[qt][hh];
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  const long long ldo = (long long)H * 64;
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float lsum = rs[qt];
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    const int q = q0 + qt * 16 + li;
    if (q >= N) continue;
    const float inv = dsc / lsum;
    bf16* orow = out + ((long long)b * N + q) * ldo + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v = {(bf16)(o[qt][dt][0] * inv), (bf16)(o[qt][dt][1] * inv), (bf16)(o[qt][dt][2] * inv),
                  (bf16)(o[qt][dt][3] * inv)};
      *(bf16x4*)(orow + dt * 16 + 4 * g) = v;
    }
    if (g == 0) lse2[(long long)bh * N + q] = m[qt] + __log2f(lsum);
  }
}

// =====================================================================================
// backward dK, dV (block = 4 waves x 32 keys, sweeps all 64-query tiles)
//   lane view of S / dP / Pd / dS: q = qt*16 + 4g + r, key = k0 + kt*16 + li
// =====================================================================================
template <bool DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv,
                                                               const bf16* __restrict__ dOs,
                                                               const float* __restrict__ lse2,
                                                               const float* __restrict__ Dvec,
                                                               const uint64_t* __restrict__ MK, bf16* __restrict__ dqkv,
                                                               int N, int H, float scale, float c, float vsc,
                                                               float* __restrict__ cpart) {
  __shared__ __attribute__((aligned(16))) bf16 sQ[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sO[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) float sL[2][64];
  __shared__ __attribute__((aligned(16))) float sD[2][64];
  int bx, bh;
  xcd_grid2(bx, bh);
  const int b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64, ldo = (long long)H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const bf16* dOg = dOs + (long long)b * N * ldo + h * 64;
  const float* Lg = lse2 + (long long)bh * N;
  const float* Dg = Dvec + (long long)bh * N;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int k0 = bx * 128 + w * 32;
  const int nq = N / 64;
  const uint16_t* mk = DROP ? (const uint16_t*)(MK + (long long)bh * nq * N) : nullptr;  // [qb][key][4 x u16]

  bf16x8 kf[2][2], vf[2][2];
  uint32_t mw[2] = {0u, 0u}, mwn[2] = {0u, 0u};
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int row = k0 + kt * 16 + li;
    const bool ok = row < N;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[kt][ks] = ok ? *(const bf16x8*)(Kg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
      vf[kt][ks] = ok ? *(const bf16x8*)(Vg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
    }
    if (DROP) mw[kt] = ok ? mk[(long long)row * 4 + g] : 0u;
  }
  f32x4 dv[4][2], dk[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) dv[dt][kt] = dk[dt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rq[2], ro[2];
  stage_load(Qg, ld, 0, N, rq);
  stage_load(dOg, ldo, 0, N, ro);
  stage_store(sQ[0], rq);
  stage_store(sO[0], ro);
  if (threadIdx.x < 64) { sL[0][threadIdx.x] = Lg[threadIdx.x]; sD[0][threadIdx.x] = Dg[threadIdx.x]; }
  __syncthreads();
  int cur = 0;
  for (int qi = 0; qi < nq; ++qi) {
    const bool more = qi + 1 < nq;
    float nl = 0.f, nd = 0.f;
    if (more) {
      stage_load(Qg, ld, (qi + 1) * 64, N, rq);
      stage_load(dOg, ldo, (qi + 1) * 64, N, ro);
      if (threadIdx.x < 64) { nl = Lg[(qi + 1) * 64 + threadIdx.x]; nd = Dg[(qi + 1) * 64 + threadIdx.x]; }
      if (DROP) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const int row = k0 + kt * 16 + li;
          mwn[kt] = row < N ? mk[((long long)(qi + 1) * N + row) * 4 + g] : 0u;
        }
      }
    }
    // S[q][key] = Q K^T ; dP'[q][key] = dO' V^T
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) s[qt][kt] = dp[qt][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#if UVA_ATT_PIPE
    // software-pipelined form: the tile is walked in query halves so that every MFMA run has
    // independent VALU beside it -- S / dP of queries 32..63 beside the softmax of 0..31, dV / dK of
    // 0..31 beside the softmax of 32..63 (hipcc otherwise issues the 32 S / dP MFMAs, then all the
    // softmax VALU, then the 32 dV / dK MFMAs: each wave alternates matrix-only and vector-only runs)
    auto sdp = [&](int qt) __attribute__((always_inline)) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 a = lds_row_frag(sQ[cur], qt * 16, ks);
        const bf16x8 e = lds_row_frag(sO[cur], qt * 16, ks);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qt][kt] = mfma16(a, kf[kt][ks], s[qt][kt]);
          dp[qt][kt] = mfma16(e, vf[kt][ks], dp[qt][kt]);
        }
      }
    };
    auto soft = [&](int qt) __attribute__((always_inline)) {
      const f32x4 Lq = *(const f32x4*)&sL[cur][qt * 16 + 4 * g];
      const f32x4 Dq = *(const f32x4*)&sD[cur][qt * 16 + 4 * g];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const float p = exp2_fast(fmaf(s[qt][kt][r], c, -Lq[r]));
          if (DROP) {
            const float pd = keep_bfe(p, mw[kt], qt * 4 + r);
            s[qt][kt][r] = pd;
            dp[qt][kt][r] = fmaf(pd, dp[qt][kt][r], -(p * Dq[r]));
          } else {
            s[qt][kt][r] = p;
            dp[qt][kt][r] = p * (dp[qt][kt][r] - Dq[r]);
          }
        }
    };
    auto dkdv = [&](int ks) __attribute__((always_inline)) {
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        pb[kt] = pack_pi(s[2 * ks][kt], s[2 * ks + 1][kt]);
        sb[kt] = pack_pi(dp[2 * ks][kt], dp[2 * ks + 1][kt]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 oa = lds_tr_frag(sO[cur], 32 * ks, 32 * ks + 16, dt * 16);
        const bf16x8 qa = lds_tr_frag(sQ[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[dt][kt] = mfma16(oa, pb[kt], dv[dt][kt]);
          dk[dt][kt] = mfma16(qa, sb[kt], dk[dt][kt]);
        }
      }
    };
    sdp(0);
    sdp(1);
    __builtin_amdgcn_sched_barrier(0);
    sdp(2);
    sdp(3);
    soft(0);
    soft(1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 1);  // VALU
    }
    __builtin_amdgcn_sched_barrier(0);
    dkdv(0);
    soft(2);
    soft(3);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, 6, 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    dkdv(1);
#else
    ATT_PRIO_HI_BWD();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        bf16x8 a = lds_row_frag(sQ[cur], qt * 16, ks);
        bf16x8 e = lds_row_frag(sO[cur], qt * 16, ks);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[qt][kt] = mfma16(a, kf[kt][ks], s[qt][kt]);
          dp[qt][kt] = mfma16(e, vf[kt][ks], dp[qt][kt]);
        }
      }
    ATT_PRIO_LO_BWD();
    // P = exp2(S c - L);  Pd = keep P;  dS = P (keep dP' - D)      (s <- Pd, dp <- dS)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const f32x4 Lq = *(const f32x4*)&sL[cur][qt * 16 + 4 * g];
      const f32x4 Dq = *(const f32x4*)&sD[cur][qt * 16 + 4 * g];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const float p = exp2_fast(fmaf(s[qt][kt][r], c, -Lq[r]));
          if (DROP) {
            // dS = P (keep dP' - D) = Pd dP' - P D: one mask op (Pd) instead of two
            const float pd = keep_bfe(p, mw[kt], qt * 4 + r);
            s[qt][kt][r] = pd;
            dp[qt][kt][r] = fmaf(pd, dp[qt][kt][r], -(p * Dq[r]));
          } else {
            s[qt][kt][r] = p;
            dp[qt][kt][r] = p * (dp[qt][kt][r] - Dq[r]);
          }
        }
    }
    // dV^T[d][key] += dO'^T Pd ; dK^T[d][key] += Q^T dS      (k = q, permuted by pi)
    ATT_PRIO_HI_BWD();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 pb[2], sb[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        pb[kt] = pack_pi(s[2 * ks][kt], s[2 * ks + 1][kt]);
        sb[kt] = pack_pi(dp[2 * ks][kt], dp[2 * ks + 1][kt]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x8 oa = lds_tr_frag(sO[cur], 32 * ks, 32 * ks + 16, dt * 16);
        bf16x8 qa = lds_tr_frag(sQ[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[dt][kt] = mfma16(oa, pb[kt], dv[dt][kt]);
          dk[dt][kt] = mfma16(qa, sb[kt], dk[dt][kt]);
        }
      }
    }
    ATT_PRIO_LO_BWD();
#endif
    if (more) {
      stage_store(sQ[cur ^ 1], rq);
      stage_store(sO[cur ^ 1], ro);
      if (threadIdx.x < 64) { sL[cur ^ 1][threadIdx.x] = nl; sD[cur ^ 1][threadIdx.x] = nd; }
      if (DROP) { mw[0] = mwn[0]; mw[1] = mwn[1]; }
    }
    lds_barrier();
    cur ^= 1;
  }
  // lane holds [d = dt*16+4g+r][key = kt*16+li]
  if (cpart) {
    // the qkv bias gradient's K / V columns: sums over this block's 128 keys of the values as stored
    // (bf16), per wave by DPP row sums over the 16 key lanes, then over the 4 waves through LDS
    float* red = (float*)&sQ[0][0];  // [4 waves][128] (the loop is over: the last barrier passed)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sk = 0.f, sv = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const bool ok = k0 + kt * 16 + li < N;
          sk += ok ? (float)(bf16)(dk[dt][kt][r] * scale) : 0.f;
          sv += ok ? (float)(bf16)(dv[dt][kt][r] * vsc) : 0.f;
        }
        sk = row16_sum(sk);
        sv = row16_sum(sv);
        if (li == 0) {
          red[w * 128 + dt * 16 + 4 * g + r] = sk;
          red[w * 128 + 64 + dt * 16 + 4 * g + r] = sv;
        }
      }
    __syncthreads();
    if (threadIdx.x < 128) {
      const int t = threadIdx.x;
      const float v = (red[t] + red[128 + t]) + (red[256 + t] + red[384 + t]);
      const long long rowp = (long long)b * gridDim.x + bx;
      cpart[rowp * (3LL * H * 64) + (t < 64 ? H * 64 : 2 * H * 64) + h * 64 + (t & 63)] = v;
    }
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + kt * 16 + li;
    if (key >= N) continue;
    bf16* krow = dqkv + ((long long)b * N + key) * ld + H * 64 + h * 64;
    bf16* vrow = krow + H * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 a = {(bf16)(dk[dt][kt][0] * scale), (bf16)(dk[dt][kt][1] * scale), (bf16)(dk[dt][kt][2] * scale),
                  (bf16)(dk[dt][kt][3] * scale)};
      bf16x4 e = {(bf16)(dv[dt][kt][0] * vsc), (bf16)(dv[dt][kt][1] * vsc), (bf16)(dv[dt][kt][2] * vsc),
                  (bf16)(dv[dt][kt][3] * vsc)};
      *(bf16x4*)(krow + dt * 16 + 4 * g) = a;
      *(bf16x4*)(vrow + dt * 16 + 4 * g) = e;
    }
  }
}

// =====================================================================================
// backward dQ (block = 4 waves x 32 queries, sweeps all 64-key tiles; transposed lane view as
// in the forward: q = qt*16 + li, key = kt*16 + 4g + r)
//   S^T = K Q^T, dP'^T = V dO'^T, dQ^T[d][q] += K^T dS^T  (dS^T packed in pi order as the B operand)
// =====================================================================================
template <bool DROP>
#ifndef UVA_ATT_DQ_OCC
#define UVA_ATT_DQ_OCC 2
#endif
// D' = dmul * rowsum(dO * O) is formed here for the block's own queries (the lanes of a query hold
// its 64 dO / O values in four 16-element runs: two permlane-free shuffles) and written to Dvec for the
// dK / dV kernel that runs after this one: no separate prologue pass (its 2 x 25 MB per layer of dO / O
// reads and launch), O read once more here instead.
__global__ __launch_bounds__(256, UVA_ATT_DQ_OCC) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dOs,
                                                             const bf16* __restrict__ Os,
                                                             const float* __restrict__ lse2,
                                                             float* __restrict__ Dvec,
                                                             const uint64_t* __restrict__ MQ, bf16* __restrict__ dqkv,
                                                             int N, int H, float scale, float c, float dmul,
                                                             float* __restrict__ cpart) {
  __shared__ __attribute__((aligned(16))) bf16 sK[2][AT_TILE];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][AT_TILE];
  int bx, bh;
  xcd_grid2(bx, bh);
  const int b = bh / H, h = bh % H;
  const long long ld = 3LL * H * 64, ldo = (long long)H * 64;
  const bf16* Qg = qkv + (long long)b * N * ld + h * 64;
  const bf16* Kg = Qg + H * 64;
  const bf16* Vg = Qg + 2 * H * 64;
  const bf16* dOg = dOs + (long long)b * N * ldo + h * 64;
  const bf16* Og = Os + (long long)b * N * ldo + h * 64;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, li = l & 15;
  const int q0 = bx * 128 + w * 32;
  const int nkv = N / 64;
  const uint16_t* mq = DROP ? (const uint16_t*)(MQ + (long long)bh * nkv * N) : nullptr;  // [kv][q][4 x u16]

  bf16x8 qf[2][2], of[2][2];
  float L[2], Dq[2];
  uint32_t mw[2] = {0u, 0u}, mwn[2] = {0u, 0u};
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int row = q0 + qt * 16 + li;
    const bool ok = row < N;
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = ok ? *(const bf16x8*)(Qg + (long long)row * ld + ks * 32 + 8 * g) : (bf16x8){};
      of[qt][ks] = ok ? *(const bf16x8*)(dOg + (long long)row * ldo + ks * 32 + 8 * g) : (bf16x8){};
      const bf16x8 ov = ok ? *(const bf16x8*)(Og + (long long)row * ldo + ks * 32 + 8 * g) : (bf16x8){};
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += (float)ov[j] * (float)of[qt][ks][j];
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    Dq[qt] = ok ? dsum * dmul : 0.f;
    if (ok && g == 0) Dvec[(long long)bh * N + row] = Dq[qt];
    L[qt] = ok ? lse2[(long long)bh * N + row] : 0.f;
    if (DROP) mw[qt] = ok ? mq[(long long)row * 4 + g] : 0u;
  }
  f32x4 dq[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  bf16x8 rk[2], rv[2];
  stage_load(Kg, ld, 0, N, rk);
  stage_load(Vg, ld, 0, N, rv);
  stage_store(sK[0], rk);
  stage_store(sV[0], rv);
  __syncthreads();
  int cur = 0;
  for (int kv = 0; kv < nkv; ++kv) {
    const bool more = kv + 1 < nkv;
    if (more) {
      stage_load(Kg, ld, (kv + 1) * 64, N, rk);
      stage_load(Vg, ld, (kv + 1) * 64, N, rv);
      if (DROP) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const int row = q0 + qt * 16 + li;
          mwn[qt] = row < N ? mq[((long long)(kv + 1) * N + row) * 4 + g] : 0u;
        }
      }
    }
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) s[kt][qt] = dp[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#if UVA_ATT_PIPE_DQ
    // software-pipelined in key halves (as dK / dV): S / dP of keys 32..63 beside the softmax of keys
    // 0..31, dQ of keys 0..31 beside the softmax of 32..63
    auto sdp = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 ka = lds_row_frag(sK[cur], kt * 16, ks);
        const bf16x8 va = lds_row_frag(sV[cur], kt * 16, ks);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          s[kt][qt] = mfma16(ka, qf[qt][ks], s[kt][qt]);
          dp[kt][qt] = mfma16(va, of[qt][ks], dp[kt][qt]);
        }
      }
    };
    auto soft = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2_fast(fmaf(s[kt][qt][r], c, -L[qt]));
          float dpt = dp[kt][qt][r];
          if (DROP) dpt = keep_bfe(dpt, mw[qt], kt * 4 + r);
          s[kt][qt][r] = p * (dpt - Dq[qt]);
        }
    };
    auto dqk = [&](int ks) __attribute__((always_inline)) {
      bf16x8 sb[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) sb[qt] = pack_pi(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 ka = lds_tr_frag(sK[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = mfma16(ka, sb[qt], dq[dt][qt]);
      }
    };
    sdp(0);
    sdp(1);
    __builtin_amdgcn_sched_barrier(0);
    sdp(2);
    sdp(3);
    soft(0);
    soft(1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    dqk(0);
    soft(2);
    soft(3);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
      __builtin_amdgcn_sched_group_barrier(0x002, 10, 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    dqk(1);
#else
    ATT_PRIO_HI_BWD();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8 ka = lds_row_frag(sK[cur], kt * 16, ks);
        const bf16x8 va = lds_row_frag(sV[cur], kt * 16, ks);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          s[kt][qt] = mfma16(ka, qf[qt][ks], s[kt][qt]);
          dp[kt][qt] = mfma16(va, of[qt][ks], dp[kt][qt]);
        }
      }
    ATT_PRIO_LO_BWD();
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = exp2_fast(fmaf(s[kt][qt][r], c, -L[qt]));
          float dpt = dp[kt][qt][r];
          if (DROP) dpt = keep_bfe(dpt, mw[qt], kt * 4 + r);
          s[kt][qt][r] = p * (dpt - Dq[qt]);
        }
    ATT_PRIO_HI_BWD();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 sb[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) sb[qt] = pack_pi(s[2 * ks][qt], s[2 * ks + 1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 ka = lds_tr_frag(sK[cur], 32 * ks, 32 * ks + 16, dt * 16);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) dq[dt][qt] = mfma16(ka, sb[qt], dq[dt][qt]);
      }
    }
    ATT_PRIO_LO_BWD();
#endif
    if (more) {
      stage_store(sK[cur ^ 1], rk);
      stage_store(sV[cur ^ 1], rv);
      if (DROP) { mw[0] = mwn[0]; mw[1] = mwn[1]; }
    }
    lds_barrier();
    cur ^= 1;
  }
  // lane holds dQ^T[d = dt*16+4g+r][q = qt*16+li]
  if (cpart) {
    // the qkv bias gradient's Q columns: sums over this block's 128 queries of the values as stored
    float* red = (float*)&sK[0][0];  // [4 waves][64]
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float sq = 0.f;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          sq += q0 + qt * 16 + li < N ? (float)(bf16)(dq[dt][qt][r] * scale) : 0.f;
        sq = row16_sum(sq);
        if (li == 0) red[w * 64 + dt * 16 + 4 * g + r] = sq;
      }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int t = threadIdx.x;
      const float v = (red[t] + red[64 + t]) + (red[128 + t] + red[192 + t]);
      const long long rowp = (long long)b * gridDim.x + bx;
      cpart[rowp * (3LL * H * 64) + h * 64 + t] = v;
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = q0 + qt * 16 + li;
    if (q >= N) continue;
    bf16* qrow = dqkv + ((long long)b * N + q) * ld + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 a = {(bf16)(dq[dt][qt][0] * scale), (bf16)(dq[dt][qt][1] * scale), (bf16)(dq[dt][qt][2] * scale),
                  (bf16)(dq[dt][qt][3] * scale)};
      *(bf16x4*)(qrow + dt * 16 + 4 * g) = a;
    }
  }
}

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" long long uva_attn_mask_bytes(int B, int N, int H) {
  return 2LL * B * H * (long long)N * (N / 64) * 8;
}

extern "C" long long uva_attn_bwd_workspace(int B, int N, int H, float drop_p) {
  (void)B; (void)N; (void)H; (void)drop_p;
  return 0;  // the loops run on the unscaled dO (no scaled copy)
}

extern "C" int uva_attn_dropmask(void* mask, int B, int N, int H, float drop_p, unsigned long long seed,
                                 hipStream_t s) {
  if (N % 64 != 0 || !(drop_p > 0.f) || mask == nullptr) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const int nt = N / 64;
  uint64_t* MQ = (uint64_t*)mask;
  uint64_t* MK = MQ + (long long)B * H * N * nt;
  const long long waves = (long long)B * H * nt * ((nt + MASK_TPW - 1) / MASK_TPW);
  if (waves > 0x7FFFFFFFLL) return (int)hipErrorInvalidValue;
  attn_mask_kernel<<<dim3((unsigned)((waves + 3) / 4)), 256, 0, s>>>(MQ, MK, N, nt, waves, th, seed);
  UVA_LAUNCH_CHECK();
  return 0;
}

extern "C" int uva_attn_fwd(const void* qkv, void* out, float* lse2, const void* mask, int B, int N, int H,
                            float scale, float drop_p, hipStream_t s) {
  if (N % 64 != 0) return (int)hipErrorInvalidValue;
  const bool drop = drop_p > 0.f;
  if (drop && mask == nullptr) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  dim3 grid((N + 127) / 128, B * H);
  const float c = scale * 1.4426950408889634f;
  const uint64_t* MQ = drop ? (const uint64_t*)mask : nullptr;
  if (drop)
    attn_fwd_kernel<true, 64, 3><<<grid, 256, 0, s>>>((const bf16*)qkv, (bf16*)out, lse2, MQ, N, H, c, ds);
  else
    attn_fwd_kernel<false, 64, 3><<<grid, 256, 0, s>>>((const bf16*)qkv, (bf16*)out, lse2, nullptr, N, H, c, 1.0f);
  UVA_LAUNCH_CHECK();
  return 0;
}

static int attn_bwd_launch(const void* qkv, const void* out, const void* dout, const float* lse2, const void* mask,
                           float* Dvec, void* dqkv, int B, int N, int H, float scale, float drop_p, float* cpart,
                           hipStream_t s);

extern "C" int uva_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, const void* mask,
                            float* Dvec, void* dqkv, void* workspace, int B, int N, int H, float scale, float drop_p,
                            hipStream_t s) {
  (void)workspace;
  return attn_bwd_launch(qkv, out, dout, lse2, mask, Dvec, dqkv, B, N, H, scale, drop_p, nullptr, s);
}

int uva_colsum_final_launch(const float* part, int nrows, int cols, float* out, int accum, hipStream_t s);

// + the qkv Linear's bias gradient (the column sums of dqkv as stored): per-(batch, 128-row block) partials
// written by the two kernels' epilogues into `part` ((B * ceil(N / 128)) * 3 H 64 floats), reduced into dbias
extern "C" int uva_attn_bwd_bias(const void* qkv, const void* out, const void* dout, const float* lse2,
                                 const void* mask, float* Dvec, void* dqkv, float* dbias, int accum, float* part, int B,
                                 int N, int H, float scale, float drop_p, hipStream_t s) {
  if (!dbias || !part) return (int)hipErrorInvalidValue;
  int r = attn_bwd_launch(qkv, out, dout, lse2, mask, Dvec, dqkv, B, N, H, scale, drop_p, part, s);
  if (r) return r;
  return uva_colsum_final_launch(part, B * ((N + 127) / 128), 3 * H * 64, dbias, accum, s);
}

static int attn_bwd_launch(const void* qkv, const void* out, const void* dout, const float* lse2, const void* mask,
                           float* Dvec, void* dqkv, int B, int N, int H, float scale, float drop_p, float* cpart,
                           hipStream_t s) {
  if (N % 64 != 0) return (int)hipErrorInvalidValue;
  const bool drop = drop_p > 0.f;
  if (drop && mask == nullptr) return (int)hipErrorInvalidValue;
  uint32_t th;
  float ds;
  uva_drop_params(drop_p, &th, &ds);
  const long long rows = (long long)B * N * H;
  // the dropout scale 1/(1-p) is not applied to dO: dP' = dsc dO V^T, so dS = dsc P (keep dP - D / dsc),
  // i.e. the loops run on the unscaled dO with D' = D / dsc, and dsc goes on dK, dQ, dV once at the
  // end (no scaled dO copy: one [B N H 64] bf16 write + its re-reads per layer saved)
  (void)rows;
  const int nt = N / 64;
  const uint64_t* MQ = (const uint64_t*)mask;
  const uint64_t* MK = drop ? MQ + (long long)B * H * N * nt : nullptr;
  const bf16* dO = (const bf16*)dout;
  dim3 grid((N + 127) / 128, B * H);
  const float c = scale * 1.4426950408889634f;
  const float sk = scale * ds;
  // dQ first: it forms D' (= rowsum(dO O) / dsc) for its queries and writes Dvec, which dK / dV reads
  const bf16* O = (const bf16*)out;
  if (drop) {
    attn_bwd_dq_kernel<true><<<grid, 256, 0, s>>>((const bf16*)qkv, dO, O, lse2, Dvec, MQ, (bf16*)dqkv, N, H, sk, c,
                                                  1.0f / ds, cpart);
    attn_bwd_dkdv_kernel<true><<<grid, 256, 0, s>>>((const bf16*)qkv, dO, lse2, Dvec, MK, (bf16*)dqkv, N, H, sk, c, ds,
                                                    cpart);
  } else {
    attn_bwd_dq_kernel<false><<<grid, 256, 0, s>>>((const bf16*)qkv, dO, O, lse2, Dvec, nullptr, (bf16*)dqkv, N, H,
                                                   sk, c, 1.0f, cpart);
    attn_bwd_dkdv_kernel<false><<<grid, 256, 0, s>>>((const bf16*)qkv, dO, lse2, Dvec, nullptr, (bf16*)dqkv, N, H,
                                                     sk, c, ds, cpart);
  }
  UVA_LAUNCH_CHECK();
  return 0;
}
