// BN3 fold of the identity bottleneck backward (csrc/bindings/conv_bn_ops.cpp block_bwd,
// SDX_BN3_FOLD): the output BatchNorm's input gradient dy3 = A·dz + D·y3 + E (per-channel
// A, D, E of bn_coef_one) is never materialised. With y3 = a2·W3ᵀ (1x1 conv3, bf16 weights
// W3 [C][K]) the two GEMMs that consumed dy3 are rewritten over dz and a2:
//
//   dgrad  da2 = dy3·W3        = dz·(diag(A)·W3) + a2·(W3ᵀ·diag(D)·W3) + Eᵀ·W3
//                                 └ dgrad, weights Wd ┘ └ T = FWD GEMM, weights Mx, bias b ┘
//   wgrad  dW3 = dy3ᵀ·a2       = diag(A)·G + diag(D)·W3·S + E ⊗ Σa2
//          with G = dzᵀ·a2 (the wgrad GEMM on dz), S = a2ᵀ·a2, Σa2 the column sums of a2
//
// so the elementwise BN-backward pass over the block's widest tensor (read dz, y3; write
// dy3) disappears. The fold's own matrices are C·K² small (K = conv3's input channels, 64
// or 128 in the layers where it is applied); these two kernels build them.
// Reference: networks/resnet_big.py:57-67 (conv3 -> bn3 -> + shortcut -> relu).
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

// blocks [0, K): row l of Mx (Mx[l][k] = Σ_c W[c][l]·D[c]·W[c][k], symmetric) and b[l];
// blocks [K, gridDim.x): Wd[k][c] = A[c]·Wt[k][c] (dgrad layout of diag(A)·W3), grid-stride.
__global__ __launch_bounds__(256) void bnfold_prep_kernel(const float* __restrict__ coef, const uint16_t* __restrict__ w,
                                                          const uint16_t* __restrict__ wt, int C, int K,
                                                          uint16_t* __restrict__ wd, uint16_t* __restrict__ mx,
                                                          float* __restrict__ bias) {
  extern __shared__ float sm[];   // [C] W[c][l]·D[c], then [256] reduction
  const float* A = coef;
  const float* D = coef + C;
  const float* E = coef + 2 * C;
  if ((int)blockIdx.x < K) {
    const int l = blockIdx.x;
    float eb = 0.f;
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float wl = bf2f(w[(size_t)c * K + l]);
      sm[c] = wl * D[c];
      eb = fmaf(E[c], wl, eb);
    }
    float* red = sm + C;
    red[threadIdx.x] = eb;
    __syncthreads();
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
      float acc = 0.f;
      for (int c = 0; c < C; ++c) acc = fmaf(sm[c], bf2f(w[(size_t)c * K + k]), acc);
      mx[(size_t)l * K + k] = f2bf(acc);
    }
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) bias[l] = red[0];
    return;
  }
  const long n = (long)K * C;
  const long stride = (long)(gridDim.x - K) * blockDim.x;
  for (long e = (long)(blockIdx.x - K) * blockDim.x + threadIdx.x; e < n; e += stride) {
    const int c = (int)(e % C);
    wd[e] = f2bf(A[c] * bf2f(wt[e]));
  }
}

// sink[c][k] (+)= A[c]·G[c][k] + D[c]·Σ_l W[c][l]·S[l][k] + E[c]·cs[k]; one block per c
__global__ __launch_bounds__(256) void bnfold_wgrad_kernel(const float* __restrict__ coef, const float* __restrict__ G,
                                                           const float* __restrict__ S, const float* __restrict__ cs,
                                                           const uint16_t* __restrict__ w, int C, int K,
                                                           float* __restrict__ sink, int accumulate) {
  extern __shared__ float wrow[];   // [K] W[c][:]
  const int c = blockIdx.x;
  for (int l = threadIdx.x; l < K; l += blockDim.x) wrow[l] = bf2f(w[(size_t)c * K + l]);
  __syncthreads();
  const float a = coef[c], d = coef[C + c], e = coef[2 * C + c];
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float ws = 0.f;
    for (int l = 0; l < K; ++l) ws = fmaf(wrow[l], S[(size_t)l * K + k], ws);
    const size_t o = (size_t)c * K + k;
    const float v = a * G[o] + d * ws + e * cs[k];
    sink[o] = accumulate ? sink[o] + v : v;
  }
}

}  // namespace

hipError_t launch_bnfold_prep(const float* coef, const void* w, const void* wt, int C, int K, void* wd, void* mx,
                              float* bias, hipStream_t s) {
  if (C <= 0 || K <= 0 || C > 8192) return hipErrorInvalidValue;
  const long n = (long)K * C;
  int gw = (int)((n + 255) / 256);
  if (gw > 512) gw = 512;
  const size_t lds = (size_t)(C + 256) * sizeof(float);
  hipLaunchKernelGGL(bnfold_prep_kernel, dim3(K + gw), dim3(256), lds, s, coef, (const uint16_t*)w,
                     (const uint16_t*)wt, C, K, (uint16_t*)wd, (uint16_t*)mx, bias);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bnfold_wgrad(const float* coef, const float* G, const float* S, const float* cs, const void* w, int C,
                               int K, float* sink, int accumulate, hipStream_t s) {
  if (C <= 0 || K <= 0 || K > 8192) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_wgrad_kernel, dim3(C), dim3(K < 256 ? ((K + 63) / 64) * 64 : 256),
                     (size_t)K * sizeof(float), s, coef, G, S, cs, (const uint16_t*)w, C, K, sink, accumulate);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
