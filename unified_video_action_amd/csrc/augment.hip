// Video training augmentation on the device: the UMI image chain of
// config/task/umi_lazy.yaml:50-72 (kornia 0.8 VideoSequential, dataset/base_lazy_dataset.py:365-411)
// and the Libero ColorJitter of dataset/libero_replay_image_dataset.py:229-247 (torchvision 0.16).
// Both libraries run in the reference's CPU dataloader workers; here one workgroup owns one frame
// and runs the whole chain over it, passing the intermediate images through a per-frame scratch
// slot (L2 / MALL resident for a 224^2 frame) with workgroup barriers between the passes that need
// neighbours or frame statistics:
//   A  crop + bilinear resize, jitter ops before contrast, grayscale sum for the contrast mean
//   B  contrast + the jitter ops after it                         (only when contrast is applied)
//   C  sharpness 3x3 blend, per-channel min / max for autocontrast (only when either is applied)
//   D  autocontrast + grayscale applied per tap inside the separable 5-tap reflect blur, or
//      pointwise when there is no blur.
// Parameters: one row of UVA_AUG_NP floats per video (utils/augment.py documents the layout);
// every frame of a video shares its row (VideoSequential same_on_frame / one seed per video).
#include "common.h"

namespace {

constexpr int AUG_NP = 24;
constexpr int AUG_THREADS = 1024;

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

// torch.remainder for floats: fmod, then shifted into the divisor's sign.
__device__ __forceinline__ float floor_mod(float a, float m) {
  float r = fmodf(a, m);
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

__device__ __forceinline__ float gray_of(float r, float g, float b, bool tv) {
  return tv ? 0.2989f * r + 0.587f * g + 0.114f * b : 0.299f * r + 0.587f * g + 0.114f * b;
}

// kornia.color.rgb_to_hsv -> hue shift (radians, fmod 2pi) -> hsv_to_rgb
__device__ __forceinline__ void hue_kornia(float& r, float& g, float& b, float fac) {
  const float mx = fmaxf(fmaxf(r, g), b), mn = fminf(fminf(r, g), b);
  const float d0 = mx - mn;
  const float s = d0 / (mx + 1e-8f);
  const float d = d0 == 0.f ? 1.f : d0;
  const float rc = mx - r, gc = mx - g, bc = mx - b;
  float h;
  if (r == mx) h = (bc - gc) / d;  // first channel wins a tie (torch.max index)
  else if (g == mx) h = ((rc - bc) + 2.f * d) / d;
  else h = ((gc - rc) + 4.f * d) / d;
  h = floor_mod(h / 6.f, 1.f);
  h = 6.2831855f * h;
  h = fmodf(h + fac, 6.2831855f);
  const float v = mx;
  const float hn = h / 6.2831855f;
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
  const float s = cr / (eq ? 1.f : mx);
  const float crd = eq ? 1.f : cr;
  const float rc = (mx - r) / crd, gc = (mx - g) / crd, bc = (mx - b) / crd;
  float h;
  if (mx == r) h = bc - gc;
  else if (mx == g) h = 2.f + rc - bc;
  else h = 4.f + gc - rc;
  h = fmodf(h / 6.f + 1.f, 1.f);
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

// workgroup reduction of NV values (sum or min/max per slot); every thread gets the result
template <int NV>
__device__ __forceinline__ void block_reduce(float (&v)[NV], const bool (&is_max)[NV], const bool (&is_min)[NV],
                                             float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float w = __shfl_xor(v[k], o, 64);
      v[k] = is_max[k] ? fmaxf(v[k], w) : is_min[k] ? fminf(v[k], w) : v[k] + w;
    }
    if (lane == 0) red[wid * NV + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float a = red[k];
    for (int w = 1; w < AUG_THREADS / 64; ++w) {
      const float x = red[w * NV + k];
      a = is_max[k] ? fmaxf(a, x) : is_min[k] ? fminf(a, x) : a + x;
    }
    v[k] = a;
  }
  __syncthreads();
}

__global__ __launch_bounds__(AUG_THREADS) void video_augment_kernel(const float* __restrict__ img,
                                                                    float* __restrict__ out,
                                                                    float* __restrict__ scratch,
                                                                    const float* __restrict__ prm, int T, int S) {
  __shared__ float red[(AUG_THREADS / 64) * 6];
  const int fr = blockIdx.x;
  const float* p = prm + (size_t)(fr / T) * AUG_NP;
  const int npx = S * S;
  const float* src = img + (size_t)fr * 3 * npx;
  float* s0 = scratch + (size_t)fr * 6 * npx;
  float* s1 = s0 + 3 * npx;
  float* dst = out + (size_t)fr * 3 * npx;
  const bool crop = p[0] != 0.f, jit = p[3] != 0.f, sharp = p[12] != 0.f, ac = p[14] != 0.f, gray = p[15] != 0.f,
             blur = p[16] != 0.f, tv = p[22] != 0.f;
  const int top = (int)p[1], left = (int)p[2], cs = (int)p[23];
  int ord[4] = {(int)p[4], (int)p[5], (int)p[6], (int)p[7]};
  int cpos = 4;  // position of the contrast op in the jitter order (4: not applied)
  if (jit) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (ord[k] == 1) cpos = k;
  }
  const int nj = jit ? 4 : 0;

  // ---- A: geometry + jitter prefix (+ grayscale sum for the contrast mean) ----
  float gsum = 0.f;
  for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
    const int y = i / S, x = i - (i / S) * S;
    float r = resized(src, S, crop, top, left, cs, y, x);
    float g = resized(src + npx, S, crop, top, left, cs, y, x);
    float b = resized(src + 2 * npx, S, crop, top, left, cs, y, x);
    for (int k = 0; k < (cpos < nj ? cpos : nj); ++k) jitter_op(ord[k], r, g, b, p, 0.f, tv);
    if (cpos < nj) gsum += gray_of(r, g, b, tv);
    s0[i] = r; s0[npx + i] = g; s0[2 * npx + i] = b;
  }
  __syncthreads();

  // ---- B: contrast (frame mean of the grayscale image before it) + jitter suffix ----
  if (cpos < nj) {
    float v[1] = {gsum};
    const bool mxk[1] = {false}, mnk[1] = {false};
    block_reduce<1>(v, mxk, mnk, red);
    const float mean = v[0] / (float)npx;
    for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
      float r = s0[i], g = s0[npx + i], b = s0[2 * npx + i];
      for (int k = cpos; k < nj; ++k) jitter_op(ord[k], r, g, b, p, mean, tv);
      s0[i] = r; s0[npx + i] = g; s0[2 * npx + i] = b;
    }
    __syncthreads();
  }

  // ---- C: sharpness (3x3 smoothing on the interior, blended back) + autocontrast statistics ----
  const float* cur = s0;
  float mm[6] = {3.4e38f, 3.4e38f, 3.4e38f, -3.4e38f, -3.4e38f, -3.4e38f};
  if (sharp || ac) {
    const float sf = p[13];
    for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
      const int y = i / S, x = i - (i / S) * S;
      const bool interior = y > 0 && y < S - 1 && x > 0 && x < S - 1;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* pl = s0 + c * npx;
        float val = pl[i];
        if (sharp) {
          float deg = val;
          if (interior) {
            const float* q0 = pl + (y - 1) * S + x;
            const float* q1 = q0 + S;
            const float* q2 = q1 + S;
            float acc = 0.f;
            acc += q0[-1] * (1.f / 13.f); acc += q0[0] * (1.f / 13.f); acc += q0[1] * (1.f / 13.f);
            acc += q1[-1] * (1.f / 13.f); acc += q1[0] * (5.f / 13.f); acc += q1[1] * (1.f / 13.f);
            acc += q2[-1] * (1.f / 13.f); acc += q2[0] * (1.f / 13.f); acc += q2[1] * (1.f / 13.f);
            deg = clamp01(acc);
          }
          val = clamp01(deg + (val - deg) * sf);
          s1[c * npx + i] = val;
        }
        mm[c] = fminf(mm[c], val);
        mm[3 + c] = fmaxf(mm[3 + c], val);
      }
    }
    if (sharp) cur = s1;
    if (ac) {
      const bool mxk[6] = {false, false, false, true, true, true}, mnk[6] = {true, true, true, false, false, false};
      block_reduce<6>(mm, mxk, mnk, red);
    }
    __syncthreads();
  }

  // ---- D: autocontrast + grayscale per sample, inside the separable reflect blur ----
  float lo[3], sc[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    lo[c] = mm[c];
    sc[c] = mm[3 + c] - mm[c] + 1e-6f;
  }
  auto post = [&](int idx, float& r, float& g, float& b) {
    r = cur[idx]; g = cur[npx + idx]; b = cur[2 * npx + idx];
    if (ac) {
      r = clamp01((r - lo[0]) / sc[0]); g = clamp01((g - lo[1]) / sc[1]); b = clamp01((b - lo[2]) / sc[2]);
    }
    if (gray) {
      const float l = gray_of(r, g, b, false);
      r = l; g = l; b = l;
    }
  };
  if (!blur) {
    for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
      float r, g, b;
      post(i, r, g, b);
      dst[i] = r; dst[npx + i] = g; dst[2 * npx + i] = b;
    }
    return;
  }
  const float k0 = p[17], k1 = p[18], k2 = p[19], k3 = p[20], k4 = p[21];
  float* tmp = (cur == s0) ? s1 : s0;
  for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
    const int y = i / S, x = i - (i / S) * S;
    const int row = y * S;
    float ar = 0.f, ag = 0.f, ab = 0.f, r, g, b;
    post(row + reflect_i(x - 2, S), r, g, b); ar += k0 * r; ag += k0 * g; ab += k0 * b;
    post(row + reflect_i(x - 1, S), r, g, b); ar += k1 * r; ag += k1 * g; ab += k1 * b;
    post(row + x, r, g, b); ar += k2 * r; ag += k2 * g; ab += k2 * b;
    post(row + reflect_i(x + 1, S), r, g, b); ar += k3 * r; ag += k3 * g; ab += k3 * b;
    post(row + reflect_i(x + 2, S), r, g, b); ar += k4 * r; ag += k4 * g; ab += k4 * b;
    tmp[i] = ar; tmp[npx + i] = ag; tmp[2 * npx + i] = ab;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < npx; i += AUG_THREADS) {
    const int y = i / S, x = i - (i / S) * S;
    const int r0 = reflect_i(y - 2, S) * S + x, r1 = reflect_i(y - 1, S) * S + x, r3 = reflect_i(y + 1, S) * S + x,
              r4 = reflect_i(y + 2, S) * S + x;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* t = tmp + c * npx;
      float a = 0.f;
      a += k0 * t[r0]; a += k1 * t[r1]; a += k2 * t[i]; a += k3 * t[r3]; a += k4 * t[r4];
      dst[c * npx + i] = a;
    }
  }
}

}  // namespace

extern "C" int uva_video_augment(const float* img, float* out, float* scratch, const float* params, int B, int T,
                                 int S, hipStream_t s) {
  if (B <= 0 || T <= 0 || S < 3 || img == nullptr || out == nullptr || scratch == nullptr || params == nullptr ||
      img == out) {
    return (int)hipErrorInvalidValue;
  }
  video_augment_kernel<<<dim3((unsigned)(B * T)), AUG_THREADS, 0, s>>>(img, out, scratch, params, T, S);
  UVA_LAUNCH_CHECK();
  return 0;
}
