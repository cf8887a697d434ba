// GPU SimCLR augmentation: the whole torchvision pipeline of the reference
// (main_supcon.py:170-179: RandomResizedCrop(size, scale=(0.2,1)), RandomHorizontalFlip,
// RandomApply(ColorJitter(0.4,0.4,0.4,0.1), p=0.8), RandomGrayscale(p=0.2), ToTensor,
// Normalize) for a batch of uint8 HWC images resident in HBM, writing the network input
// directly: NHWC bf16 with channels padded to 8 (16-byte pixels for the stem conv's
// implicit-GEMM gather), views stacked view-major ([v0 batch; v1 batch]) as the
// reference's torch.cat([images[0], images[1]]) (main_supcon.py:256).
//
// One 256-thread workgroup per (sample, view). Randomness is a counter-based hash of
// (seed, sample index, view, draw), so a step is reproducible and needs no RNG state.
// Contrast needs the image mean at its position in the (random) jitter order, so the
// pixel pipeline runs twice when contrast is active: pass 1 up to the contrast op
// (block-reduced grey mean), pass 2 the full chain.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t key;
  uint32_t ctr;
  __device__ float uni() {  // [0, 1)
    const uint64_t v = mix64(key ^ mix64(0x1234567ull + ctr++));
    return (float)(v >> 40) * (1.0f / 16777216.0f);
  }
};

struct AugParams {
  const uint8_t* data;     // [n_data][H][W][3], or ragged (offs != nullptr): image i at data + offs[i]
  const int64_t* offs;     // optional [n_data] byte offsets of native-resolution images
  const int32_t* hw;       // optional [n_data][2] their (height, width)
  long n_data;             // images in `data` (bounds checks)
  const int64_t* idx;      // [B]
  uint16_t* out;           // [n_views*B][S][S][8]
  int B, H, W, S, n_views;
  uint64_t seed;
  const int64_t* seed_dev;   // optional: seed read from device memory (hipGraph replays)
  float mean[3], inv_std[3];
  float scale_lo, scale_hi, ratio_lo, ratio_hi;
  float jitter_p, bright, contrast, sat, hue, gray_p;
  int do_crop, do_flip;
};

struct ViewParams {
  float ci, cj, ch, cw;    // crop box (top, left, height, width) in source pixels
  bool flip, jitter, gray;
  float fb, fc, fs, fh;    // jitter factors
  int order[4];            // 0 brightness, 1 contrast, 2 saturation, 3 hue
};

__device__ void make_view_params(const AugParams& p, Rng& rng, ViewParams& v, int Hi, int Wi) {
  const float H = Hi, W = Wi;
  v.ci = 0.f; v.cj = 0.f; v.ch = H; v.cw = W;
  if (p.do_crop) {
    const float area = H * W;
    const float lr0 = logf(p.ratio_lo), lr1 = logf(p.ratio_hi);
    bool found = false;
    for (int t = 0; t < 10 && !found; ++t) {
      const float target = area * (p.scale_lo + (p.scale_hi - p.scale_lo) * rng.uni());
      const float ar = expf(lr0 + (lr1 - lr0) * rng.uni());
      const float w = rintf(sqrtf(target * ar)), h = rintf(sqrtf(target / ar));
      if (w > 0.f && w <= W && h > 0.f && h <= H) {
        v.ci = floorf(rng.uni() * (H - h + 1.f));
        v.cj = floorf(rng.uni() * (W - w + 1.f));
        v.ch = h; v.cw = w;
        found = true;
      }
    }
    if (!found) {  // central crop, ratio clamped (torchvision fallback)
      const float in_ratio = W / H;
      float w, h;
      if (in_ratio < p.ratio_lo) { w = W; h = rintf(w / p.ratio_lo); }
      else if (in_ratio > p.ratio_hi) { h = H; w = rintf(h * p.ratio_hi); }
      else { w = W; h = H; }
      v.ci = floorf((H - h) * 0.5f); v.cj = floorf((W - w) * 0.5f); v.ch = h; v.cw = w;
    }
  }
  v.flip = p.do_flip && rng.uni() < 0.5f;
  v.jitter = rng.uni() < p.jitter_p;
  v.fb = 1.f + p.bright * (2.f * rng.uni() - 1.f);
  v.fc = 1.f + p.contrast * (2.f * rng.uni() - 1.f);
  v.fs = 1.f + p.sat * (2.f * rng.uni() - 1.f);
  v.fh = p.hue * (2.f * rng.uni() - 1.f);
  // random permutation of the 4 jitter ops (Fisher-Yates)
  for (int i = 0; i < 4; ++i) v.order[i] = i;
  for (int i = 3; i > 0; --i) {
    const int j = (int)(rng.uni() * (i + 1)) % (i + 1);
    const int t = v.order[i]; v.order[i] = v.order[j]; v.order[j] = t;
  }
  v.gray = rng.uni() < p.gray_p;
  if (p.bright <= 0.f && p.contrast <= 0.f && p.sat <= 0.f && p.hue <= 0.f) v.jitter = false;
}

__device__ __forceinline__ float grey(float r, float g, float b) { return 0.2989f * r + 0.587f * g + 0.114f * b; }
__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

__device__ void adjust_hue(float& r, float& g, float& b, float hf) {
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b));
  const float cr = mx - mn;
  const float v = mx;
  const float s = cr / (mx == 0.f ? 1.f : mx);
  const float crd = cr == 0.f ? 1.f : cr;
  const float rc = (mx - r) / crd, gc = (mx - g) / crd, bc = (mx - b) / crd;
  float h;
  if (mx == r) h = bc - gc;
  else if (mx == g) h = 2.f + rc - bc;
  else h = 4.f + gc - rc;
  h = h / 6.f + 1.f;
  h = h - floorf(h);
  h = h + hf;
  h = h - floorf(h);
  const float h6 = h * 6.f;
  const float i = floorf(h6);
  const float f = h6 - i;
  const float pp = clamp01(v * (1.f - s)), q = clamp01(v * (1.f - s * f)), t = clamp01(v * (1.f - s * (1.f - f)));
  switch (((int)i) % 6) {
    case 0: r = v; g = t; b = pp; break;
    case 1: r = q; g = v; b = pp; break;
    case 2: r = pp; g = v; b = t; break;
    case 3: r = pp; g = q; b = v; break;
    case 4: r = t; g = pp; b = v; break;
    default: r = v; g = pp; b = q; break;
  }
}

// bilinear sample (align_corners=False) of the crop box, then flip
__device__ void sample_pixel(const AugParams& p, const uint8_t* img, int H, int W, const ViewParams& v, int oy,
                             int ox, float& r, float& g, float& b) {
  const int xs = v.flip ? (p.S - 1 - ox) : ox;
  float sy = (oy + 0.5f) * (v.ch / p.S) - 0.5f + v.ci;
  float sx = (xs + 0.5f) * (v.cw / p.S) - 0.5f + v.cj;
  sy = fminf(fmaxf(sy, v.ci), v.ci + v.ch - 1.f);
  sx = fminf(fmaxf(sx, v.cj), v.cj + v.cw - 1.f);
  const int y0 = (int)floorf(sy), x0 = (int)floorf(sx);
  const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
  const float wy = sy - y0, wx = sx - x0;
  SDX_DCHECK(y0 >= 0 && x0 >= 0 && y0 < H && x0 < W && y1 < H && x1 < W);
  const uint8_t* p00 = img + ((size_t)y0 * W + x0) * 3;
  const uint8_t* p01 = img + ((size_t)y0 * W + x1) * 3;
  const uint8_t* p10 = img + ((size_t)y1 * W + x0) * 3;
  const uint8_t* p11 = img + ((size_t)y1 * W + x1) * 3;
  float c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float top = p00[k] + (p01[k] - (float)p00[k]) * wx;
    const float bot = p10[k] + (p11[k] - (float)p10[k]) * wx;
    c[k] = (top + (bot - top) * wy) * (1.f / 255.f);
  }
  r = c[0]; g = c[1]; b = c[2];
}

// apply jitter ops order[0..n_ops) (contrast uses `cmean`)
__device__ void jitter_ops(const ViewParams& v, int n_ops, float cmean, float& r, float& g, float& b) {
  for (int k = 0; k < n_ops; ++k) {
    switch (v.order[k]) {
      case 0: r = clamp01(r * v.fb); g = clamp01(g * v.fb); b = clamp01(b * v.fb); break;
      case 1:
        r = clamp01(v.fc * r + (1.f - v.fc) * cmean);
        g = clamp01(v.fc * g + (1.f - v.fc) * cmean);
        b = clamp01(v.fc * b + (1.f - v.fc) * cmean);
        break;
      case 2: {
        const float gy = grey(r, g, b);
        r = clamp01(v.fs * r + (1.f - v.fs) * gy);
        g = clamp01(v.fs * g + (1.f - v.fs) * gy);
        b = clamp01(v.fs * b + (1.f - v.fs) * gy);
        break;
      }
      default: adjust_hue(r, g, b, v.fh); break;
    }
  }
}

__global__ __launch_bounds__(256) void aug_kernel(AugParams p) {
  __shared__ float red[4];
  __shared__ ViewParams vp;
  const int b = blockIdx.x, view = blockIdx.y;
  const int64_t src = p.idx[b];
  SDX_DCHECK(p.n_data <= 0 || (src >= 0 && src < p.n_data));
  // dense [N][H][W][3] store, or native-resolution images (ImageFolder: RandomResizedCrop
  // samples its box from the original pixels, as torchvision does on the decoded image)
  const int H = p.offs ? p.hw[2 * src] : p.H, W = p.offs ? p.hw[2 * src + 1] : p.W;
  const uint8_t* img = p.offs ? p.data + p.offs[src] : p.data + (size_t)src * p.H * p.W * 3;
  if (threadIdx.x == 0) {
    const uint64_t seed = p.seed_dev ? (uint64_t)p.seed_dev[0] : p.seed;
    Rng rng{mix64(seed * 0x100000001b3ull + (uint64_t)src * 31ull + (uint64_t)view * 0x9E37ull + (uint64_t)b), 0};
    make_view_params(p, rng, vp, H, W);
  }
  __syncthreads();
  const ViewParams v = vp;
  const int npix = p.S * p.S;
  // pass 1: grey mean at the contrast position (only if contrast is applied)
  float cmean = 0.f;
  int cpos = -1;
  if (v.jitter)
    for (int k = 0; k < 4; ++k)
      if (v.order[k] == 1) cpos = k;
  if (cpos >= 0) {
    float acc = 0.f;
    for (int pix = threadIdx.x; pix < npix; pix += 256) {
      float r, g, bb;
      sample_pixel(p, img, H, W, v, pix / p.S, pix % p.S, r, g, bb);
      jitter_ops(v, cpos, 0.f, r, g, bb);
      acc += grey(r, g, bb);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    cmean = (red[0] + red[1] + red[2] + red[3]) / (float)npix;
  }
  uint16_t* out = p.out + ((size_t)view * p.B + b) * npix * 8;
  for (int pix = threadIdx.x; pix < npix; pix += 256) {
    float r, g, bb;
    sample_pixel(p, img, H, W, v, pix / p.S, pix % p.S, r, g, bb);
    if (v.jitter) jitter_ops(v, 4, cmean, r, g, bb);
    if (v.gray) { const float gy = grey(r, g, bb); r = g = bb = gy; }
    r = (r - p.mean[0]) * p.inv_std[0];
    g = (g - p.mean[1]) * p.inv_std[1];
    bb = (bb - p.mean[2]) * p.inv_std[2];
    reinterpret_cast<uint4*>(out)[pix] = make_uint4(pack_bf2(r, g), pack_bf2(bb, 0.f), 0u, 0u);
  }
}

}  // namespace

hipError_t launch_gpu_augment(const uint8_t* data, const int64_t* idx, int B, int H, int W, int S, int n_views,
                              uint64_t seed, const float* mean, const float* std, float scale_lo, float scale_hi,
                              float ratio_lo, float ratio_hi, float jitter_p, float bright, float contrast,
                              float sat, float hue, float gray_p, int do_crop, int do_flip, const int64_t* seed_dev,
                              void* out, hipStream_t s, long n_data, const int64_t* offs, const int32_t* hw) {
  AugParams p{};
  p.offs = offs;
  p.hw = hw;
  p.n_data = n_data;
  p.data = data; p.idx = idx; p.out = (uint16_t*)out;
  p.B = B; p.H = H; p.W = W; p.S = S; p.n_views = n_views; p.seed = seed;
  for (int k = 0; k < 3; ++k) { p.mean[k] = mean[k]; p.inv_std[k] = 1.f / std[k]; }
  p.scale_lo = scale_lo; p.scale_hi = scale_hi; p.ratio_lo = ratio_lo; p.ratio_hi = ratio_hi;
  p.jitter_p = jitter_p; p.bright = bright; p.contrast = contrast; p.sat = sat; p.hue = hue; p.gray_p = gray_p;
  p.do_crop = do_crop; p.do_flip = do_flip;
  p.seed_dev = seed_dev;
  hipLaunchKernelGGL(aug_kernel, dim3(B, n_views), dim3(256), 0, s, p);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
