// Projection-feature row norms (reference main_supcon.py:283 and :295-317).
//
//  * rownorm_fwd / rownorm_bwd: y = x / max(||x||, eps) per row (F.normalize, dim=1) and its
//    exact gradient dx = (dy − y·(y·dy)) / ||x|| (||x|| > eps) or dy / eps (clamped rows).
//    One wave per row, D <= 256 (4 elements per lane): the contrastive loss's input.
//  * norm_stats: the SEC / L2-reg logging statistics of the UN-normalised features in one
//    single-block, single-pass launch: Σ||x||, Σ||x||² (fp64), then (mode 1) the finalize — norm mean /
//    variance over the global rows, the record_norm_mean EMA update (state kept on device),
//    loss_sec = Σ_local (||x|| − rec)² / n_global and loss_l2 = Σ_local ||x||² / n_global.
//    With >1 rank the host all-reduces the sums between mode 0 and mode 2.
//    Replaces ~15 small torch launches per step (and their host cost, which leaves the GPU
//    idle between the forward and the backward).
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

template <int PER>
__global__ __launch_bounds__(256) void rownorm_fwd_kernel(const float* __restrict__ x, int N, int D, float eps,
                                                          float* __restrict__ y, float* __restrict__ norms) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* xr = x + (size_t)row * D;
  float v[PER], s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = lane + 64 * k;
    v[k] = c < D ? xr[c] : 0.f;
    s = fmaf(v[k], v[k], s);
  }
  const float nrm = sqrtf(wave_sum(s));
  const float inv = 1.f / fmaxf(nrm, eps);
  float* yr = y + (size_t)row * D;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = lane + 64 * k;
    if (c < D) yr[c] = v[k] * inv;
  }
  if (lane == 0) norms[row] = nrm;
}

template <int PER>
__global__ __launch_bounds__(256) void rownorm_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                          const float* __restrict__ norms, int N, int D, float eps,
                                                          float* __restrict__ dx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* dyr = dy + (size_t)row * D;
  const float* yr = y + (size_t)row * D;
  float g[PER], yy[PER], s = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = lane + 64 * k;
    g[k] = c < D ? dyr[c] : 0.f;
    yy[k] = c < D ? yr[c] : 0.f;
    s = fmaf(g[k], yy[k], s);
  }
  const float nrm = norms[row];
  const bool clamped = !(nrm > eps);
  const float dot = clamped ? 0.f : wave_sum(s);
  const float inv = 1.f / fmaxf(nrm, eps);
  float* dxr = dx + (size_t)row * D;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = lane + 64 * k;
    if (c < D) dxr[c] = (g[k] - yy[k] * dot) * inv;
  }
}

// mode 0: local sums -> sums; mode 1: local sums + finalize; mode 2: finalize with the
// (all-reduced) sums given. out = [norm_mean, norm_var, record_norm_mean, loss_sec, loss_l2]
// One pass: 16 lanes per row (float4 loads when D % 4 == 0), 64 rows in flight per block
// pass; loss_sec = Σ(||x|| − rec)² is expanded as Σ||x||² − 2·rec·Σ||x|| + N·rec² (fp64), so
// the features are read once (a second pass over the rows made this single-block kernel
// latency-bound: 45 us per step at 512 x 128)
__global__ __launch_bounds__(1024) void norm_stats_kernel(const float* __restrict__ x, int N, int D, int mode,
                                                          double* __restrict__ sums, double n_global,
                                                          float momentum, float* __restrict__ rec,
                                                          float* __restrict__ valid, float* __restrict__ out) {
  __shared__ double red[2][16];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  const int sub = lane & 15, grp = tid >> 4, ngrp = blockDim.x >> 4;
  const bool vec = (D & 3) == 0;
  double a1 = 0.0, a2 = 0.0;
#pragma unroll 4
  for (int row = grp; row < N; row += ngrp) {
    const float* xr = x + (size_t)row * D;
    float s = 0.f;
    if (vec) {
      for (int c = 4 * sub; c < D; c += 64) {
        const float4 v = *reinterpret_cast<const float4*>(xr + c);
        s = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, fmaf(v.w, v.w, s))));
      }
    } else {
      for (int c = sub; c < D; c += 16) s = fmaf(xr[c], xr[c], s);
    }
    s += __shfl_xor(s, 8);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 1);
    if (sub == 0) {
      a1 += sqrt((double)s);
      a2 += (double)s;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    a1 += __shfl_xor(a1, o);
    a2 += __shfl_xor(a2, o);
  }
  if (lane == 0) {
    red[0][wv] = a1;
    red[1][wv] = a2;
  }
  __syncthreads();
  if (tid != 0) return;
  double s1 = 0.0, s2 = 0.0;   // local sums
  for (int w = 0; w < nw; ++w) {
    s1 += red[0][w];
    s2 += red[1][w];
  }
  if (mode == 0) {
    sums[0] = s1;
    sums[1] = s2;
    return;
  }
  const double g1 = mode == 1 ? s1 : sums[0], g2 = mode == 1 ? s2 : sums[1];
  const double mean = g1 / n_global, var = g2 / n_global - mean * mean;
  const float r = valid[0] > 0.f ? (float)((1.0 - momentum) * rec[0] + momentum * mean) : (float)mean;
  rec[0] = r;
  valid[0] = 1.f;
  const double rd = (double)r;
  out[0] = (float)mean;
  out[1] = (float)var;
  out[2] = r;
  out[3] = (float)(fmax(s2 - 2.0 * rd * s1 + (double)N * rd * rd, 0.0) / n_global);
  out[4] = (float)(s2 / n_global);
}

}  // namespace

hipError_t launch_rownorm_fwd(const float* x, int N, int D, float eps, float* y, float* norms, hipStream_t s) {
  if (N < 1 || D < 1 || D > 256) return hipErrorInvalidValue;
  const dim3 g((N + 3) / 4), b(256);
  if (D <= 64) hipLaunchKernelGGL((rownorm_fwd_kernel<1>), g, b, 0, s, x, N, D, eps, y, norms);
  else if (D <= 128) hipLaunchKernelGGL((rownorm_fwd_kernel<2>), g, b, 0, s, x, N, D, eps, y, norms);
  else hipLaunchKernelGGL((rownorm_fwd_kernel<4>), g, b, 0, s, x, N, D, eps, y, norms);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_rownorm_bwd(const float* dy, const float* y, const float* norms, int N, int D, float eps, float* dx,
                              hipStream_t s) {
  if (N < 1 || D < 1 || D > 256) return hipErrorInvalidValue;
  const dim3 g((N + 3) / 4), b(256);
  if (D <= 64) hipLaunchKernelGGL((rownorm_bwd_kernel<1>), g, b, 0, s, dy, y, norms, N, D, eps, dx);
  else if (D <= 128) hipLaunchKernelGGL((rownorm_bwd_kernel<2>), g, b, 0, s, dy, y, norms, N, D, eps, dx);
  else hipLaunchKernelGGL((rownorm_bwd_kernel<4>), g, b, 0, s, dy, y, norms, N, D, eps, dx);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_norm_stats(const float* x, int N, int D, int mode, double* sums, double n_global, float momentum,
                             float* rec, float* valid, float* out, hipStream_t s) {
  if (N < 1 || D < 1 || mode < 0 || mode > 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(norm_stats_kernel, dim3(1), dim3(1024), 0, s, x, N, D, mode, sums, n_global, momentum, rec,
                     valid, out);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
