// Pooling kernels for NHWC bf16 activations (gfx950).
//
// * max-pool 3x3 / stride 2 / pad 1 of the ImageNet stem (the CIFAR
//   stem at 224² does not fit BS=4096 in 288 GB; the 7x7/2 + maxpool stem cuts
//   activations 16x). Backward recomputes the window argmax from the saved input and
//   gathers: every input element sums the gradients of the windows whose max it is
//   (first max in scan order, as torch) — no index tensor stored, no atomics.
// * global average pool forward (fp32 [N, C] out) and backward (broadcast dy/HW).
// Vectorised over 8 channels (16-B loads) per lane.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

struct PoolGeom {
  int N, H, W, C, P, Q, k, stride, pad;
};

// IDX: also store, per window and channel, the position (ddy·k + ddx) of its FIRST maximum
// in scan order (uint8 [N][P][Q][C]); the backward then needs neither x nor y
template <bool IDX>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeom g, long total8) {
  const int C8 = g.C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % C8);
    long r = e / C8;
    const int q = (int)(r % g.Q); r /= g.Q;
    const int p = (int)(r % g.P);
    const int n = (int)(r / g.P);
    float m[8];
    int at[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      m[i] = -INFINITY;
      at[i] = 0;
    }
    for (int dy = 0; dy < g.k; ++dy) {
      const int yy = p * g.stride - g.pad + dy;
      if (yy < 0 || yy >= g.H) continue;
      for (int dx = 0; dx < g.k; ++dx) {
        const int xx = q * g.stride - g.pad + dx;
        if (xx < 0 || xx >= g.W) continue;
        float v[8];
        unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + yy) * g.W + xx) * C8 + c8], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (IDX && v[i] > m[i]) at[i] = dy * g.k + dx;   // strict: the first maximum wins
          m[i] = fmaxf(m[i], v[i]);
        }
      }
    }
    reinterpret_cast<uint4*>(y)[e] = pack8(m);
    if constexpr (IDX) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo |= (uint32_t)at[i] << (8 * i);
        hi |= (uint32_t)at[4 + i] << (8 * i);
      }
      reinterpret_cast<uint2*>(idx)[e] = make_uint2(lo, hi);
    }
  }
}

// dx[n,h,w,c] = Σ over windows (p,q) containing (h,w) whose stored first-max position is
// (h,w): dy[n,p,q,c] — windows in (p, q) order, the same sums as the recomputing kernel
// below, from 8 B of index + 16 B of dy per window instead of re-reading its 9 inputs
__global__ __launch_bounds__(256) void maxpool_bwd_idx_kernel(const uint8_t* __restrict__ idx,
                                                              const uint16_t* __restrict__ dy,
                                                              uint16_t* __restrict__ dx, PoolGeom g, long total8) {
  const int C8 = g.C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % C8);
    long r = e / C8;
    const int w = (int)(r % g.W); r /= g.W;
    const int h = (int)(r % g.H);
    const int n = (int)(r / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int p_lo = max(0, (h + g.pad - g.k + g.stride) / g.stride), p_hi = min(g.P - 1, (h + g.pad) / g.stride);
    const int q_lo = max(0, (w + g.pad - g.k + g.stride) / g.stride), q_hi = min(g.Q - 1, (w + g.pad) / g.stride);
    for (int p = p_lo; p <= p_hi; ++p) {
      for (int q = q_lo; q <= q_hi; ++q) {
        const long oi = (((long)n * g.P + p) * g.Q + q) * C8 + c8;
        const uint2 iv = reinterpret_cast<const uint2*>(idx)[oi];
        float gv[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[oi], gv);
        const uint32_t pos = (uint32_t)((h - (p * g.stride - g.pad)) * g.k + (w - (q * g.stride - g.pad)));
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t at = ((i < 4 ? iv.x : iv.y) >> (8 * (i & 3))) & 0xffu;
          if (at == pos) acc[i] += gv[i];
        }
      }
    }
    reinterpret_cast<uint4*>(dx)[e] = pack8(acc);
  }
}

// dx[n,h,w,c] = Σ over windows (p,q) containing (h,w) whose FIRST maximum is (h,w): dy[n,p,q,c]
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
                                                          const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx,
                                                          PoolGeom g, long total8) {
  const int C8 = g.C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % C8);
    long r = e / C8;
    const int w = (int)(r % g.W); r /= g.W;
    const int h = (int)(r % g.H);
    const int n = (int)(r / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // output windows that contain (h, w)
    const int p_lo = max(0, (h + g.pad - g.k + g.stride) / g.stride), p_hi = min(g.P - 1, (h + g.pad) / g.stride);
    const int q_lo = max(0, (w + g.pad - g.k + g.stride) / g.stride), q_hi = min(g.Q - 1, (w + g.pad) / g.stride);
    for (int p = p_lo; p <= p_hi; ++p) {
      for (int q = q_lo; q <= q_hi; ++q) {
        float yv[8], gv[8];
        const long oi = (((long)n * g.P + p) * g.Q + q) * C8 + c8;
        unpack8(reinterpret_cast<const uint4*>(y)[oi], yv);
        unpack8(reinterpret_cast<const uint4*>(dy)[oi], gv);
        // first position (scan order) in the window holding the max, per channel
        int first[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) first[i] = -1;
        for (int ddy = 0; ddy < g.k; ++ddy) {
          const int yy = p * g.stride - g.pad + ddy;
          if (yy < 0 || yy >= g.H) continue;
          for (int ddx = 0; ddx < g.k; ++ddx) {
            const int xx = q * g.stride - g.pad + ddx;
            if (xx < 0 || xx >= g.W) continue;
            float v[8];
            unpack8(reinterpret_cast<const uint4*>(x)[(((long)n * g.H + yy) * g.W + xx) * C8 + c8], v);
#pragma unroll
            for (int i = 0; i < 8; ++i)
              if (first[i] < 0 && v[i] == yv[i]) first[i] = yy * g.W + xx;
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (first[i] == h * g.W + w) acc[i] += gv[i];
      }
    }
    reinterpret_cast<uint4*>(dx)[e] = pack8(acc);
  }
}

// global average pool: y[n][c] = mean_{h,w} x[n,h,w,c] (fp32 out)
__global__ __launch_bounds__(256) void gap_fwd_kernel(const uint16_t* __restrict__ x, float* __restrict__ y, int HW,
                                                      int C, long total8) {
  const int C8 = C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % C8);
    const long n = e / C8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < HW; ++i) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(x)[(n * HW + i) * C8 + c8], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    const float s = 1.f / HW;
    float4* out = reinterpret_cast<float4*>(y + n * C + c8 * 8);
    out[0] = make_float4(acc[0] * s, acc[1] * s, acc[2] * s, acc[3] * s);
    out[1] = make_float4(acc[4] * s, acc[5] * s, acc[6] * s, acc[7] * s);
  }
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const float* __restrict__ dy, uint16_t* __restrict__ dx, int HW,
                                                      int C, long total8) {
  const int C8 = C / 8;
  const float s = 1.f / HW;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % C8);
    const long n = e / C8 / HW;
    const float4* src = reinterpret_cast<const float4*>(dy + n * C + c8 * 8);
    const float4 a = src[0], b = src[1];
    const float v[8] = {a.x * s, a.y * s, a.z * s, a.w * s, b.x * s, b.y * s, b.z * s, b.w * s};
    reinterpret_cast<uint4*>(dx)[e] = pack8(v);
  }
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

hipError_t launch_maxpool_fwd(const void* x, void* y, int N, int H, int W, int C, int P, int Q, int k, int stride,
                              int pad, hipStream_t s) {
  PoolGeom g{N, H, W, C, P, Q, k, stride, pad};
  const long total8 = (long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel<false>, dim3(grid_for(total8)), dim3(256), 0, s, (const uint16_t*)x,
                     (uint16_t*)y, nullptr, g, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_maxpool_fwd_idx(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q,
                                  int k, int stride, int pad, hipStream_t s) {
  if (k * k > 255) return hipErrorInvalidValue;
  PoolGeom g{N, H, W, C, P, Q, k, stride, pad};
  const long total8 = (long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel<true>, dim3(grid_for(total8)), dim3(256), 0, s, (const uint16_t*)x,
                     (uint16_t*)y, idx, g, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_maxpool_bwd_idx(const uint8_t* idx, const void* dy, void* dx, int N, int H, int W, int C, int P,
                                  int Q, int k, int stride, int pad, hipStream_t s) {
  PoolGeom g{N, H, W, C, P, Q, k, stride, pad};
  const long total8 = (long)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_idx_kernel, dim3(grid_for(total8)), dim3(256), 0, s, idx, (const uint16_t*)dy,
                     (uint16_t*)dx, g, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_maxpool_bwd(const void* x, const void* y, const void* dy, void* dx, int N, int H, int W, int C,
                              int P, int Q, int k, int stride, int pad, hipStream_t s) {
  PoolGeom g{N, H, W, C, P, Q, k, stride, pad};
  const long total8 = (long)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total8)), dim3(256), 0, s, (const uint16_t*)x,
                     (const uint16_t*)y, (const uint16_t*)dy, (uint16_t*)dx, g, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_gap_fwd(const void* x, float* y, int N, int HW, int C, hipStream_t s) {
  const long total8 = (long)N * (C / 8);
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(grid_for(total8)), dim3(256), 0, s, (const uint16_t*)x, y, HW, C, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_gap_bwd(const float* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  const long total8 = (long)N * HW * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for(total8)), dim3(256), 0, s, dy, (uint16_t*)dx, HW, C, total8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
