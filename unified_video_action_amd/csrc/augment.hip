// Video training augmentation on the device: the UMI image chain of
// config/task/umi_lazy.yaml:50-72 (kornia 0.8 VideoSequential, dataset/base_lazy_dataset.py:365-411)
// and the Libero ColorJitter of dataset/libero_replay_image_dataset.py:229-247 (torchvision 0.16).
// Both libraries run in the reference's CPU dataloader workers.  Here the chain is three launches,
// each over (frame, 8-row band) workgroups (448 frames x 28 bands = 12.5k workgroups for UMI B=56),
// with the frame-wide statistics passed between them as per-band partials (summed in band order:
// deterministic) and every neighbourhood op served from LDS row buffers:
//   K1 vaug_stage1     geometry (crop + bilinear resize) + the jitter ops before contrast (all of
//                      them when contrast is off) -> mid, per-band grayscale sums (contrast mean)
//   K2 vaug_stage2     contrast (mean from K1) + the jitter ops after it over the band's rows of mid
//                      and one halo row each side, staged in LDS; sharpness 3x3 blend -> mid2;
//                      per-band per-channel min / max for autocontrast
//   K3 vaug_post_blur  autocontrast + grayscale of the band and two reflected halo rows each side
//                      into LDS (all of a thread's loads issued first), separable 5-tap reflect
//                      blur (x, then y) -> out
// Every pixel's geometry and jitter run once; 4 consecutive pixels per thread item (float4 loads
// and stores where the data is contiguous); reciprocals instead of IEEE divisions and exact
// range-limited fmod forms (the library fmodf is an iterative software routine).  UMI B=56 x 8
// frames of 224^2, every op on: 0.81 ms (K1 / K2 / K3 about a third each, VALU-bound by the HSV
// hue path).  The first form -- one 1024-thread workgroup per frame running every pass through a
// frame-sized scratch slot -- took 1.18 ms.
// Parameters: one row of UVA_AUG_NP floats per video (utils/augment.py documents the layout);
// every frame of a video shares its row (VideoSequential same_on_frame / one seed per video).
#include "common.h"

namespace {

constexpr int AUG_NP = 24;

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

// fmodf(a, m) for m > 0: on (-m, m) the value itself, on [m, 2m) a - m (exact: Sterbenz), which
// covers every call below; the library routine (an iterative software fmod, the kernel's largest
// VALU cost) only outside that range
__device__ __forceinline__ float fmod_pos(float a, float m) {
  if (a > -m && a < m) return a;
  if (a >= m && a < 2.f * m) return a - m;
  return fmodf(a, m);
}

// torch.remainder for floats: fmod, then shifted into the divisor's sign (m > 0 here).
__device__ __forceinline__ float floor_mod(float a, float m) {
  float r = fmod_pos(a, m);
  if (r != 0.f && ((m < 0.f) != (r < 0.f))) r += m;
  return r;
}

__device__ __forceinline__ int reflect_i(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

// bilinear (align_corners=False) sample of the cs x cs window at (top, left), resized to S x S
__device__ __forceinline__ float resized(const float* __restrict__ plane, int S, bool crop, int top, int left, int cs,
                                         int y, int x) {
  if (!crop) return plane[y * S + x];
  const float sc = (float)cs / (float)S;
  float sy = ((float)y + 0.5f) * sc - 0.5f, sx = ((float)x + 0.5f) * sc - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int y1 = y0 + 1 < cs ? y0 + 1 : cs - 1, x1 = x0 + 1 < cs ? x0 + 1 : cs - 1;
  const float ly = sy - (float)y0, lx = sx - (float)x0;
  const float* r0 = plane + (top + y0) * S + left;
  const float* r1 = plane + (top + y1) * S + left;
  const float a = r0[x0] * (1.f - lx) + r0[x1] * lx;
  const float b = r1[x0] * (1.f - lx) + r1[x1] * lx;
  return a * (1.f - ly) + b * ly;
}

// (i / S, i % S) for i < 2^16 via a float reciprocal (exact: i + 0.5 is never within 2^-10 of a
// multiple of S)
__device__ __forceinline__ void split_idx(int i, int S, float invS, int& y, int& x) {
  y = (int)(((float)i + 0.5f) * invS);
  x = i - y * S;
}

__device__ __forceinline__ float gray_of(float r, float g, float b, bool tv) {
  return tv ? 0.2989f * r + 0.587f * g + 0.114f * b : 0.299f * r + 0.587f * g + 0.114f * b;
}

// kornia.color.rgb_to_hsv -> hue shift (radians, fmod 2pi) -> hsv_to_rgb
__device__ __forceinline__ void hue_kornia(float& r, float& g, float& b, float fac) {
  const float mx = fmaxf(fmaxf(r, g), b), mn = fminf(fminf(r, g), b);
  const float d0 = mx - mn;
  // reciprocals instead of IEEE divisions (the division sequence dominated the kernel; the oracle
  // comparison is a tolerance, not bit-exact)
  const float s = d0 * __builtin_amdgcn_rcpf(mx + 1e-8f);
  const float d = d0 == 0.f ? 1.f : d0;
  const float rd = __builtin_amdgcn_rcpf(d);
  const float rc = mx - r, gc = mx - g, bc = mx - b;
  float h;
  if (r == mx) h = (bc - gc) * rd;  // first channel wins a tie (torch.max index)
  else if (g == mx) h = ((rc - bc) + 2.f * d) * rd;
  else h = ((gc - rc) + 4.f * d) * rd;
  h = floor_mod(h * (1.f / 6.f), 1.f);
  h = 6.2831855f * h;
  h = fmod_pos(h + fac, 6.2831855f);
  const float v = mx;
  const float hn = h * 0.15915494f;
  const float hi = floor_mod(floorf(hn * 6.f), 6.f);
  const float f = floor_mod(hn * 6.f, 6.f) - hi;
  const float p = v * (1.f - s), q = v * (1.f - f * s), t = v * (1.f - (1.f - f) * s);
  switch ((int)hi) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// torchvision F_t._rgb2hsv -> (h + fac) % 1 -> _hsv2rgb (clamped p / q / t)
__device__ __forceinline__ void hue_tv(float& r, float& g, float& b, float fac) {
  const float mx = fmaxf(fmaxf(r, g), b), mn = fminf(fminf(r, g), b);
  const bool eq = mx == mn;
  const float cr = mx - mn;
  const float s = cr * __builtin_amdgcn_rcpf(eq ? 1.f : mx);
  const float rcrd = __builtin_amdgcn_rcpf(eq ? 1.f : cr);
  const float rc = (mx - r) * rcrd, gc = (mx - g) * rcrd, bc = (mx - b) * rcrd;
  float h;
  if (mx == r) h = bc - gc;
  else if (mx == g) h = 2.f + rc - bc;
  else h = 4.f + gc - rc;
  h = fmod_pos(h * (1.f / 6.f) + 1.f, 1.f);
  h = floor_mod(h + fac, 1.f);
  const float v = mx;
  const float fi = floorf(h * 6.f);
  const float f = h * 6.f - fi;
  int i = ((int)fi) % 6;
  i = i < 0 ? i + 6 : i;
  const float p = clamp01(v * (1.f - s)), q = clamp01(v * (1.f - s * f)), t = clamp01(v * (1.f - s * (1.f - f)));
  switch (i) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// one ColorJitter op (0 brightness, 1 contrast, 2 saturation, 3 hue) in the style's formulation
__device__ __forceinline__ void jitter_op(int op, float& r, float& g, float& b, const float* __restrict__ p,
                                          float mean, bool tv) {
  const float fac = p[8 + op];
  if (op == 0) {
    r = clamp01(fac * r); g = clamp01(fac * g); b = clamp01(fac * b);
  } else if (op == 1) {
    const float m = (1.f - fac) * mean;
    r = clamp01(fac * r + m); g = clamp01(fac * g + m); b = clamp01(fac * b + m);
  } else if (op == 2) {
    const float m = (1.f - fac) * gray_of(r, g, b, tv);
    r = clamp01(fac * r + m); g = clamp01(fac * g + m); b = clamp01(fac * b + m);
  } else if (fac != 0.f) {
    if (tv) hue_tv(r, g, b, fac);
    else hue_kornia(r, g, b, fac);
  }
}

constexpr int BAND = 8;      // output rows per workgroup
constexpr int BT = 256;      // threads per workgroup
constexpr int MAXS = 256;    // largest frame side the LDS row buffers hold
// per-thread items (4 pixels each) of the K1 / K2 / K3 row loops at S = MAXS (fixed trip counts)
constexpr int IT1 = (BAND * (MAXS / 4) + BT - 1) / BT;
constexpr int IT2 = ((BAND + 2) * (MAXS / 4) + BT - 1) / BT;
constexpr int IT3 = ((BAND + 4) * (MAXS / 4) + BT - 1) / BT;

struct VParams {
  bool crop, jit, sharp, ac, gray, blur, tv;
  int top, left, cs, cpos, nj;
  int ord[4];
};

__device__ __forceinline__ VParams vparams(const float* __restrict__ p) {
  VParams v;
  v.crop = p[0] != 0.f; v.jit = p[3] != 0.f; v.sharp = p[12] != 0.f; v.ac = p[14] != 0.f;
  v.gray = p[15] != 0.f; v.blur = p[16] != 0.f; v.tv = p[22] != 0.f;
  v.top = (int)p[1]; v.left = (int)p[2]; v.cs = (int)p[23];
  v.nj = v.jit ? 4 : 0;
  v.cpos = 4;  // position of the contrast op in the jitter order (4: not applied)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v.ord[k] = (int)p[4 + k];
    if (v.jit && v.ord[k] == 1) v.cpos = k;
  }
  return v;
}

// geometry + jitter ops [k0, k1) of pixel (y, x): the image entering the sharpness stage when
// k0 = 0, k1 = nj and `mean` is the frame's pre-contrast grayscale mean
__device__ __forceinline__ void jittered(const float* __restrict__ src, int S, const VParams& v,
                                         const float* __restrict__ p, int k1, float mean, int y, int x, float& r,
                                         float& g, float& b) {
  const int npx = S * S;
  r = resized(src, S, v.crop, v.top, v.left, v.cs, y, x);
  g = resized(src + npx, S, v.crop, v.top, v.left, v.cs, y, x);
  b = resized(src + 2 * npx, S, v.crop, v.top, v.left, v.cs, y, x);
  for (int k = 0; k < k1; ++k) jitter_op(v.ord[k], r, g, b, p, mean, v.tv);
}

template <int NV, bool MAX>
__device__ __forceinline__ void wg_reduce(float (&a)[NV], float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float w = __shfl_xor(a[k], o, 64);
      a[k] = MAX ? fmaxf(a[k], w) : a[k] + w;
    }
    if (lane == 0) red[wid * NV + k] = a[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float s = red[k];
    for (int w = 1; w < BT / 64; ++w) s = MAX ? fmaxf(s, red[w * NV + k]) : s + red[w * NV + k];
    a[k] = s;
  }
}

// K1: geometry + the jitter ops before contrast (all of them when contrast is not applied) of the
// band's rows -> mid, and the band's grayscale sum of that image for the contrast mean
__global__ __launch_bounds__(BT) void vaug_stage1(const float* __restrict__ img, const float* __restrict__ prm,
                                                  float* __restrict__ mid, float* __restrict__ part1, int T, int S,
                                                  int nb) {
  __shared__ float red[BT / 64];
  const int fr = blockIdx.x / nb, band = blockIdx.x % nb;
  const float* p = prm + (size_t)(fr / T) * AUG_NP;
  const VParams v = vparams(p);
  const int npx = S * S;
  const float* src = img + (size_t)fr * 3 * npx;
  float* dst = mid + (size_t)fr * 3 * npx;
  const int k1 = v.cpos < v.nj ? v.cpos : v.nj;
  const int y0 = band * BAND, rows = min(BAND, S - y0);
  const int S4 = S / 4;
  const float invS4 = 1.f / (float)S4;
  const int n = rows * S4;
  float acc[1] = {0.f};
#pragma unroll
  for (int it = 0; it < IT1; ++it) {  // 4 consecutive pixels per item
    const int i = (int)threadIdx.x + it * BT;
    if (i >= n) break;
    int y, xq;
    split_idx(i, S4, invS4, y, xq);
    y += y0;
    float r[4], g[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) jittered(src, S, v, p, k1, 0.f, y, 4 * xq + u, r[u], g[u], b[u]);
    const int o = y * S + 4 * xq;
    *(float4*)(dst + o) = make_float4(r[0], r[1], r[2], r[3]);
    *(float4*)(dst + npx + o) = make_float4(g[0], g[1], g[2], g[3]);
    *(float4*)(dst + 2 * npx + o) = make_float4(b[0], b[1], b[2], b[3]);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[0] += gray_of(r[u], g[u], b[u], v.tv);
  }
  if (v.cpos < v.nj) {  // workgroup-uniform
    wg_reduce<1, false>(acc, red);
    if (threadIdx.x == 0) part1[(size_t)fr * nb + band] = acc[0];
  }
}

// K2: the jitter ops from contrast on (contrast mean = K1's band sums, summed in band order) over
// the band's rows of mid and, with sharpness, one halo row on each side, staged in LDS; sharpness
// 3x3 blend -> mid2; per-band per-channel min / max for autocontrast -> part2
__global__ __launch_bounds__(BT) void vaug_stage2(const float* __restrict__ mid, const float* __restrict__ prm,
                                                  const float* __restrict__ part1, float* __restrict__ mid2,
                                                  float* __restrict__ part2, int T, int S, int nb) {
  __shared__ float J[(BAND + 2) * 3 * MAXS];
  __shared__ float red[(BT / 64) * 6];
  const int fr = blockIdx.x / nb, band = blockIdx.x % nb;
  const float invS = 1.f / (float)S;
  const float* p = prm + (size_t)(fr / T) * AUG_NP;
  const VParams v = vparams(p);
  const int npx = S * S;
  const float* src = mid + (size_t)fr * 3 * npx;
  const bool contrast = v.cpos < v.nj;
  float mean = 0.f;
  if (contrast) {
    const float* ps = part1 + (size_t)fr * nb;
    for (int i = 0; i < nb; ++i) mean += ps[i];
    mean /= (float)npx;
  }
  const int y0 = band * BAND, rows = min(BAND, S - y0);
  // staged rows: y0 - 1 .. y0 + rows (inside the image) at LDS row (y - y0 + 1)
  const int ya = v.sharp ? max(y0 - 1, 0) : y0, yb = v.sharp ? min(y0 + rows, S - 1) : y0 + rows - 1;
  const int S4 = S / 4;
  const float invS4 = 1.f / (float)S4;
  const int n2 = (yb - ya + 1) * S4;
#pragma unroll
  for (int it = 0; it < IT2; ++it) {
    const int i = (int)threadIdx.x + it * BT;
    if (i >= n2) break;
    int y, xq;
    split_idx(i, S4, invS4, y, xq);
    y += ya;
    const int o = y * S + 4 * xq;
    float4 R = *(const float4*)(src + o), G = *(const float4*)(src + npx + o), Bv = *(const float4*)(src + 2 * npx + o);
    if (contrast) {
      float r[4] = {R.x, R.y, R.z, R.w}, g[4] = {G.x, G.y, G.z, G.w}, b[4] = {Bv.x, Bv.y, Bv.z, Bv.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        for (int k = v.cpos; k < v.nj; ++k) jitter_op(v.ord[k], r[u], g[u], b[u], p, mean, v.tv);
      R = make_float4(r[0], r[1], r[2], r[3]);
      G = make_float4(g[0], g[1], g[2], g[3]);
      Bv = make_float4(b[0], b[1], b[2], b[3]);
    }
    float* row = J + (y - y0 + 1) * 3 * MAXS + 4 * xq;
    *(float4*)row = R;
    *(float4*)(row + MAXS) = G;
    *(float4*)(row + 2 * MAXS) = Bv;
  }
  __syncthreads();
  const float sf = p[13];
  // autocontrast statistics as one max-reduction: {-min r, -min g, -min b, max r, max g, max b}
  float mm[6] = {-3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
  float* dst = mid2 + (size_t)fr * 3 * npx;
  for (int i = threadIdx.x; i < rows * S; i += BT) {
    int y, x;
    split_idx(i, S, invS, y, x);
    y += y0;
    const bool interior = y > 0 && y < S - 1 && x > 0 && x < S - 1;
    const float* rw = J + (y - y0 + 1) * 3 * MAXS;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* q1 = rw + c * MAXS + x;
      float val = *q1;
      if (v.sharp) {
        float deg = val;
        if (interior) {
          const float* q0 = q1 - 3 * MAXS;
          const float* q2 = q1 + 3 * MAXS;
          float acc = 0.f;
          acc += q0[-1] * (1.f / 13.f); acc += q0[0] * (1.f / 13.f); acc += q0[1] * (1.f / 13.f);
          acc += q1[-1] * (1.f / 13.f); acc += q1[0] * (5.f / 13.f); acc += q1[1] * (1.f / 13.f);
          acc += q2[-1] * (1.f / 13.f); acc += q2[0] * (1.f / 13.f); acc += q2[1] * (1.f / 13.f);
          deg = clamp01(acc);
        }
        val = clamp01(deg + (val - deg) * sf);
      }
      dst[c * npx + y * S + x] = val;
      mm[c] = fmaxf(mm[c], -val);
      mm[3 + c] = fmaxf(mm[3 + c], val);
    }
  }
  if (v.ac) {
    wg_reduce<6, true>(mm, red);
    if (threadIdx.x < 6) part2[((size_t)fr * nb + band) * 6 + threadIdx.x] = mm[threadIdx.x];
  }
}

// K3: autocontrast (frame min / max from K2's band values) + grayscale per pixel of the staged
// rows y0-2 .. y0+rows+1 (reflected at the image edges), then the separable 5-tap blur (x, then y)
// from LDS; without blur the pointwise result is written directly
__global__ __launch_bounds__(BT) void vaug_post_blur(const float* __restrict__ mid, const float* __restrict__ prm,
                                                     const float* __restrict__ part2, float* __restrict__ out, int T,
                                                     int S, int nb) {
  __shared__ float P[(BAND + 4) * 3 * MAXS];
  __shared__ float Hb[(BAND + 4) * 3 * MAXS];
  const int fr = blockIdx.x / nb, band = blockIdx.x % nb;
  const float invS = 1.f / (float)S;
  const float* p = prm + (size_t)(fr / T) * AUG_NP;
  const VParams v = vparams(p);
  const int npx = S * S;
  float lo[3] = {0.f, 0.f, 0.f}, sc[3] = {1.f, 1.f, 1.f};
  if (v.ac) {
    float mm[6] = {-3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
    const float* q = part2 + (size_t)fr * nb * 6;
    for (int i = 0; i < nb; ++i)
#pragma unroll
      for (int k = 0; k < 6; ++k) mm[k] = fmaxf(mm[k], q[i * 6 + k]);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      lo[c] = -mm[c];
      sc[c] = mm[3 + c] - lo[c] + 1e-6f;
    }
  }
  const float rs[3] = {1.f / sc[0], 1.f / sc[1], 1.f / sc[2]};
  const float* src = mid + (size_t)fr * 3 * npx;
  float* dst = out + (size_t)fr * 3 * npx;
  auto post4_load = [&](int idx, float (&r)[4], float (&g)[4], float (&b)[4]) {
    const float4 R = *(const float4*)(src + idx), G = *(const float4*)(src + npx + idx),
                 Bv = *(const float4*)(src + 2 * npx + idx);
    r[0] = R.x; r[1] = R.y; r[2] = R.z; r[3] = R.w;
    g[0] = G.x; g[1] = G.y; g[2] = G.z; g[3] = G.w;
    b[0] = Bv.x; b[1] = Bv.y; b[2] = Bv.z; b[3] = Bv.w;
  };
  auto post4_math = [&](float (&r)[4], float (&g)[4], float (&b)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v.ac) {
        r[u] = clamp01((r[u] - lo[0]) * rs[0]); g[u] = clamp01((g[u] - lo[1]) * rs[1]);
        b[u] = clamp01((b[u] - lo[2]) * rs[2]);
      }
      if (v.gray) {
        const float l = gray_of(r[u], g[u], b[u], false);
        r[u] = l; g[u] = l; b[u] = l;
      }
    }
  };
  const int y0 = band * BAND, rows = min(BAND, S - y0);
  if (!v.blur) {
    for (int i = threadIdx.x; i < rows * S / 4; i += BT) {
      const int idx = y0 * S + 4 * i;
      float r[4], g[4], b[4];
      post4_load(idx, r, g, b);
      post4_math(r, g, b);
      *(float4*)(dst + idx) = make_float4(r[0], r[1], r[2], r[3]);
      *(float4*)(dst + npx + idx) = make_float4(g[0], g[1], g[2], g[3]);
      *(float4*)(dst + 2 * npx + idx) = make_float4(b[0], b[1], b[2], b[3]);
    }
    return;
  }
  const int nst = rows + 4;  // staged rows y0-2 .. y0+rows+1
  const int S4 = S / 4;
  const float invS4 = 1.f / (float)S4;
  const int n3 = nst * S4;
  float rr[IT3][4], gg[IT3][4], bb[IT3][4];
#pragma unroll
  for (int it = 0; it < IT3; ++it) {  // every item's loads first, then the math and LDS stores
    const int i = min((int)threadIdx.x + it * BT, n3 - 1);
    int j, xq;
    split_idx(i, S4, invS4, j, xq);
    post4_load(reflect_i(y0 - 2 + j, S) * S + 4 * xq, rr[it], gg[it], bb[it]);
  }
#pragma unroll
  for (int it = 0; it < IT3; ++it) {
    const int i = min((int)threadIdx.x + it * BT, n3 - 1);
    int j, xq;
    split_idx(i, S4, invS4, j, xq);
    post4_math(rr[it], gg[it], bb[it]);
    float* row = P + j * 3 * MAXS + 4 * xq;
    *(float4*)row = make_float4(rr[it][0], rr[it][1], rr[it][2], rr[it][3]);
    *(float4*)(row + MAXS) = make_float4(gg[it][0], gg[it][1], gg[it][2], gg[it][3]);
    *(float4*)(row + 2 * MAXS) = make_float4(bb[it][0], bb[it][1], bb[it][2], bb[it][3]);
  }
  __syncthreads();
  const float k0 = p[17], k1 = p[18], k2 = p[19], k3 = p[20], k4 = p[21];
  for (int i = threadIdx.x; i < nst * S; i += BT) {
    int j, x;
    split_idx(i, S, invS, j, x);
    const int a0 = reflect_i(x - 2, S), a1 = reflect_i(x - 1, S), a3 = reflect_i(x + 1, S), a4 = reflect_i(x + 2, S);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* row = P + (j * 3 + c) * MAXS;
      float acc = 0.f;
      acc += k0 * row[a0]; acc += k1 * row[a1]; acc += k2 * row[x]; acc += k3 * row[a3]; acc += k4 * row[a4];
      Hb[(j * 3 + c) * MAXS + x] = acc;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < rows * S4; i += BT) {
    int jr, xq;  // output row y0 + jr = staged row jr + 2
    split_idx(i, S4, invS4, jr, xq);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* col = Hb + c * MAXS + 4 * xq;
      float4 t[5];
#pragma unroll
      for (int d = 0; d < 5; ++d) t[d] = *(const float4*)(col + (jr + d) * 3 * MAXS);
      float o[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* e0 = (const float*)&t[0]; const float* e1 = (const float*)&t[1];
        const float* e2 = (const float*)&t[2]; const float* e3 = (const float*)&t[3];
        const float* e4 = (const float*)&t[4];
        float acc = 0.f;
        acc += k0 * e0[u]; acc += k1 * e1[u]; acc += k2 * e2[u]; acc += k3 * e3[u]; acc += k4 * e4[u];
        o[u] = acc;
      }
      *(float4*)(dst + c * npx + (y0 + jr) * S + 4 * xq) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
}

}  // namespace

extern "C" int uva_video_augment(const float* img, float* out, float* scratch, const float* params, int B, int T,
                                 int S, hipStream_t s) {
  if (B <= 0 || T <= 0 || S < 4 || S % 4 || S > MAXS || img == nullptr || out == nullptr || scratch == nullptr ||
      params == nullptr || img == out) {
    return (int)hipErrorInvalidValue;
  }
  const int F = B * T, nb = (S + BAND - 1) / BAND;
  // scratch: mid [F, 3, S, S] | mid2 [F, 3, S, S] | part1 [F, nb] | part2 [F, nb, 6]
  float* mid = scratch;
  float* mid2 = mid + (size_t)F * 3 * S * S;
  float* part1 = mid2 + (size_t)F * 3 * S * S;
  float* part2 = part1 + (size_t)F * nb;
  const dim3 grid((unsigned)(F * nb));
  vaug_stage1<<<grid, BT, 0, s>>>(img, params, mid, part1, T, S, nb);
  vaug_stage2<<<grid, BT, 0, s>>>(mid, params, part1, mid2, part2, T, S, nb);
  vaug_post_blur<<<grid, BT, 0, s>>>(mid2, params, part2, out, T, S, nb);
  UVA_LAUNCH_CHECK();
  return 0;
}
