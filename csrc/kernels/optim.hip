// Fused optimizer kernels over the flat fp32 parameter / gradient / momentum buffers.
//
// The reference steps torch.optim.SGD over 163 separate tensors (util.py:79-84,
// main_supcon.py:323-325). Here all parameters live in ONE flat buffer (views handed to
// the modules), so an SGD step is a single streaming kernel (16-B accesses) that also
// folds in the data-parallel gradient averaging (grad_scale = 1/W) and reads the
// learning rate from device memory (no host sync, graph-replayable when the lr
// changes). LARS (config 5) adds one segmented-norm pass per step.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

// torch SGD semantics (dampening 0): d = s·g + wd·p; buf = m·buf + d; p -= lr·(nesterov ? d + m·buf : buf)
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, long n4, const float* __restrict__ lr_ptr,
                                                  float momentum, float wd, float gscale, int nesterov) {
  const float lr = lr_ptr[0];
  float4* P = reinterpret_cast<float4*>(p);
  const float4* G = reinterpret_cast<const float4*>(g);
  float4* Bf = reinterpret_cast<float4*>(buf);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pv = P[i];
    const float4 gv = G[i];
    float4 bv = Bf[i];
    float* pp = reinterpret_cast<float*>(&pv);
    const float* gg = reinterpret_cast<const float*>(&gv);
    float* bb = reinterpret_cast<float*>(&bv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = gscale * gg[k] + wd * pp[k];
      bb[k] = momentum * bb[k] + d;
      const float step = nesterov ? d + momentum * bb[k] : bb[k];
      pp[k] -= lr * step;
    }
    P[i] = pv;
    Bf[i] = bv;
  }
}

__device__ __forceinline__ int find_seg(const long* __restrict__ off, int nseg, long e) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// per-segment Σp² and Σ(s·g + wd·p)² (wd only on adapted segments) -> out[2*nseg] (zeroed)
__global__ __launch_bounds__(256) void seg_norms_kernel(const float* __restrict__ p, const float* __restrict__ g,
                                                        const long* __restrict__ off, const int* __restrict__ adapt,
                                                        int nseg, long n, float wd, float gscale,
                                                        float* __restrict__ out) {
  // each block handles a contiguous chunk of 4096 elements; chunks never straddle segments
  // because every segment is padded to a multiple of 4096 by the flat-buffer allocator.
  const long base = (long)blockIdx.x * 4096;
  if (base >= n) return;
  const int seg = find_seg(off, nseg, base);
  const float w = adapt[seg] ? wd : 0.f;
  float sp = 0.f, sd = 0.f;
  for (long e = base + threadIdx.x; e < base + 4096 && e < n; e += 256) {
    const float pv = p[e];
    const float d = gscale * g[e] + w * pv;
    sp += pv * pv;
    sd += d * d;
  }
  sp = wave_sum(sp);
  sd = wave_sum(sd);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out + 2 * seg, sp);
    atomicAdd(out + 2 * seg + 1, sd);
  }
}

// LARS: d = s·g + wd·p (adapted) | s·g; trust = eta·||p||/||d|| (adapted, both > 0) | 1;
// buf = m·buf + lr·trust·d; p -= buf
__global__ __launch_bounds__(256) void lars_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ buf, const long* __restrict__ off,
                                                   const int* __restrict__ adapt, const float* __restrict__ norms,
                                                   int nseg, long n, const float* __restrict__ lr_ptr, float momentum,
                                                   float wd, float gscale, float eta) {
  const float lr = lr_ptr[0];
  const long base = (long)blockIdx.x * 4096;
  if (base >= n) return;
  const int seg = find_seg(off, nseg, base);
  const bool ad = adapt[seg] != 0;
  float trust = 1.f;
  if (ad) {
    const float pn = sqrtf(norms[2 * seg]), dn = sqrtf(norms[2 * seg + 1]);
    if (pn > 0.f && dn > 0.f) trust = eta * pn / dn;
  }
  const float w = ad ? wd : 0.f;
  const float scale = lr * trust;
  for (long e = base + threadIdx.x; e < base + 4096 && e < n; e += 256) {
    const float pv = p[e];
    const float d = gscale * g[e] + w * pv;
    const float b = momentum * buf[e] + scale * d;
    buf[e] = b;
    p[e] = pv - b;
  }
}

}  // namespace

hipError_t launch_sgd(float* p, const float* g, float* buf, long n, const float* lr, float momentum, float wd,
                      float gscale, int nesterov, hipStream_t s, int max_blocks) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  const long n4 = n / 4;
  long grid = (n4 + 255) / 256;
  if (grid > 4096) grid = 4096;
  // a capped grid (grid-stride loop) trickles an early per-bucket update along beside the
  // backward instead of taking every CU for a short burst
  if (max_blocks > 0 && grid > max_blocks) grid = max_blocks;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid), dim3(256), 0, s, p, g, buf, n4, lr, momentum, wd, gscale, nesterov);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_lars(float* p, const float* g, float* buf, const long* seg_off, const int* adapt, int nseg, long n,
                       const float* lr, float momentum, float wd, float gscale, float eta, float* norms,
                       hipStream_t s) {
  hipError_t e = hipMemsetAsync(norms, 0, sizeof(float) * 2 * nseg, s);
  if (e != hipSuccess) return e;
  const long blocks = (n + 4095) / 4096;
  hipLaunchKernelGGL(seg_norms_kernel, dim3(blocks), dim3(256), 0, s, p, g, seg_off, adapt, nseg, n, wd, gscale,
                     norms);
  SDX_LAUNCH_CHECK();
  hipLaunchKernelGGL(lars_kernel, dim3(blocks), dim3(256), 0, s, p, g, buf, seg_off, adapt, norms, nseg, n, lr,
                     momentum, wd, gscale, eta);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
