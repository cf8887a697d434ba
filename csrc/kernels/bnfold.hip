// BN3 fold of the identity bottleneck backward (csrc/bindings/conv_bn_ops.cpp block_bwd,
// SDX_BN3_FOLD): the output BatchNorm's input gradient dy3 = A·dz + D·y3 + E (per-channel
// A, D, E of bn_coef_one) is never materialised. With y3 = a2·W3ᵀ (1x1 conv3, bf16 weights
// W3 [C][K]) the two GEMMs that consumed dy3 are rewritten over dz and a2:
//
//   dgrad  da2 = dy3·W3        = dz·(diag(A)·W3) + a2·(W3ᵀ·diag(D)·W3) + Eᵀ·W3
//                                 └ weights Wd ┘      └ weights Mx ┘        └ bias b ┘
//          one K-concatenated GEMM [dz | a2]·[Wd ; Mx] + b (igemm.hip a2 operand, fp32 bias
//          before the rounding); fallback: a separate T = a2·Mx + b added by the dgrad epilogue
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
// A row block splits the C-long reductions over P = NT/K lane groups (K <= NT), each
// summing every P-th channel with 8 independent loads in flight, then adds the groups.
constexpr int PREP_NT = 1024;
// Coherent-rounding correction (mu, cs given): Wd and Mx are rounded to bf16 once and then
// applied to every row, so their rounding errors do not average out over the batch the way
// the per-element rounding of a materialised dy3 does — the BN-parameter gradients of the
// layers below (sums over all rows) pick up a bias ∝ rows. The row-mean part of that error,
// mean(dz)·(A·W3 − Wd) + mean(a2)·(Mx − bf16(Mx)), is added back exactly through the fp32
// bias b; what remains is zero-mean over the rows. mean(dz)[c] = −(E + D·μ)/A (A ≠ 0).
__global__ __launch_bounds__(PREP_NT) void bnfold_prep_kernel(const float* __restrict__ coef, const uint16_t* __restrict__ w,
                                                          const uint16_t* __restrict__ wt, int C, int K,
                                                          uint16_t* __restrict__ wd, uint16_t* __restrict__ mx,
                                                          int ldw, int ldm, float* __restrict__ bias,
                                                          const float* __restrict__ mu, const float* __restrict__ cs,
                                                          float inv_rows) {
  extern __shared__ float sm[];   // [C] W[c][l]·D[c], then [PREP_NT] partial sums
  const float* A = coef;
  const float* D = coef + C;
  const float* E = coef + 2 * C;
  const int t = threadIdx.x;
  if ((int)blockIdx.x < K) {
    const int l = blockIdx.x;
    float* red = sm + C;
    float eb = 0.f;
    for (int c = t; c < C; c += PREP_NT) {
      const float wl = bf2f(w[(size_t)c * K + l]);
      sm[c] = wl * D[c];
      eb = fmaf(E[c], wl, eb);
      if (mu != nullptr && A[c] != 0.f) {
        const float m1 = -(E[c] + D[c] * mu[c]) / A[c];
        const float ex = A[c] * wl;
        eb = fmaf(m1, ex - bf2f(f2bf(ex)), eb);
      }
    }
    red[t] = eb;
    __syncthreads();
    for (int off = PREP_NT / 2; off > 0; off >>= 1) {
      if (t < off) red[t] += red[t + off];
      __syncthreads();
    }
    float bsum = red[0];
    __syncthreads();
    const int KW = K >= PREP_NT ? PREP_NT : K;   // k lanes per group
    const int P = PREP_NT / KW;                  // lane groups splitting the channel sum
    const int grp = t / KW;
    float ca = 0.f;                              // Σ_k mean(a2)[k]·(Mx − bf16(Mx))[l][k]
    for (int k0 = 0; k0 < K; k0 += KW) {
      const int k = k0 + t % KW;
      float acc = 0.f;
#pragma unroll 8
      for (int c = grp; c < C; c += P) acc = fmaf(sm[c], bf2f(w[(size_t)c * K + k]), acc);
      red[t] = acc;
      __syncthreads();
      if (grp == 0) {
        float v = acc;
        for (int q = 1; q < P; ++q) v += red[t + q * KW];
        const uint16_t r = f2bf(v);
        mx[(size_t)l * ldm + k] = r;
        if (cs != nullptr) ca = fmaf(cs[k] * inv_rows, v - bf2f(r), ca);
      }
      __syncthreads();
    }
    red[t] = ca;
    __syncthreads();
    for (int off = PREP_NT / 2; off > 0; off >>= 1) {
      if (t < off) red[t] += red[t + off];
      __syncthreads();
    }
    if (t == 0) bias[l] = bsum + red[0];
    return;
  }
  const long n = (long)K * C;
  const long stride = (long)(gridDim.x - K) * PREP_NT;
  for (long e = (long)(blockIdx.x - K) * PREP_NT + t; e < n; e += stride) {
    const int c = (int)(e % C);
    wd[(e / C) * ldw + c] = f2bf(A[c] * bf2f(wt[e]));
  }
}

// per-block column sums of a [rows][K] bf16 tensor: partial[blockIdx][K] (fp32). Lanes keep
// a fixed 8-channel group (the grid stride is a multiple of K/8).
__global__ __launch_bounds__(256) void bnfold_colsum_kernel(const uint16_t* __restrict__ x, long n8, int K,
                                                            float* __restrict__ partial) {
  __shared__ float red[256][9];
  const int K8 = K / 8;
  const long stride = (long)gridDim.x * 256;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // 4 chunks per trip in flight: at 512 blocks (2 per CU) one load per trip left the loop
  // latency-bound (21 µs for a 67 MB layer-1 a2, ~2.5x its HBM time); same summation order
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  long e = blockIdx.x * 256L + threadIdx.x;
  for (; e + 3 * stride < n8; e += 4 * stride) {
    uint4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = ld16s<true>(xv + e + u * stride);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v[8];
      unpack8(q[u], v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[i];
    }
  }
  for (; e < n8; e += stride) {
    float v[8];
    unpack8(ld16s<true>(xv + e), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += v[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x][i] = acc[i];
  __syncthreads();
  if ((int)threadIdx.x < K8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int q = threadIdx.x; q < 256; q += K8)
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += red[q][i];
#pragma unroll
    for (int i = 0; i < 8; ++i) partial[(size_t)blockIdx.x * K + threadIdx.x * 8 + i] = s[i];
  }
}

// cs[k] = Σ_b partial[b][k]: a block per 64 columns, 16 lane groups over b, then LDS
__global__ __launch_bounds__(1024) void bnfold_colsum_finish_kernel(const float* __restrict__ partial, int nb, int K,
                                                                    float* __restrict__ cs) {
  __shared__ float red[16][64];
  const int kl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + kl;
  float s = 0.f;
  if (k < K) {
    // 8 loads in flight per trip, added in the same (b ascending) order
    int b = grp;
    for (; b + 7 * 16 < nb; b += 8 * 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = partial[(size_t)(b + 16 * u) * K + k];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < nb; b += 16) s += partial[(size_t)b * K + k];
  }
  red[grp][kl] = s;
  __syncthreads();
  if (grp == 0 && k < K) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += red[q][kl];
    cs[k] = v;
  }
}

// sink[c][k] (+)= A[c]·G[c][k] + D[c]·Σ_l W[c][l]·S[l][k] + E[c]·Σ_b cs[b][k]; one block per c
__global__ __launch_bounds__(256) void bnfold_wgrad_kernel(const float* __restrict__ coef, const float* __restrict__ G,
                                                           const float* __restrict__ S, const float* __restrict__ cs,
                                                           int ncs, const uint16_t* __restrict__ w, int C, int K,
                                                           float* __restrict__ sink, int accumulate) {
  extern __shared__ float wrow[];   // [K] W[c][:]
  const int c = blockIdx.x;
  for (int l = threadIdx.x; l < K; l += blockDim.x) wrow[l] = bf2f(w[(size_t)c * K + l]);
  __syncthreads();
  const float a = coef[c], d = coef[C + c], e = coef[2 * C + c];
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float ws = 0.f, sk = 0.f;
#pragma unroll 8
    for (int l = 0; l < K; ++l) ws = fmaf(wrow[l], S[(size_t)l * K + k], ws);
#pragma unroll 8
    for (int b = 0; b < ncs; ++b) sk += cs[(size_t)b * K + k];
    const size_t o = (size_t)c * K + k;
    const float v = a * G[o] + d * ws + e * sk;
    sink[o] = accumulate ? sink[o] + v : v;
  }
}

// forward-folded BN3 (its y = a2·Wᵀ never stored): Σ_rows dz·y per channel from the fold's
// G = dzᵀ·a2 as Σ_k W[c][k]·G[c][k] (fp64), written as two extra rows of a BN-backward
// statistics slab [2][2][C]: set 0 = 0, set 1 = the value split into fp32 hi + lo (the fp64
// column reduction restores it); one wave per channel
__global__ __launch_bounds__(64) void bnfold_rowdot_kernel(const float* __restrict__ G, const uint16_t* __restrict__ w,
                                                           int C, int K, int ns, float* __restrict__ out) {
  const int c = blockIdx.x, lane = threadIdx.x;
  double acc = 0.0;
  for (int k = lane; k < K; k += 64) acc += (double)bf2f(w[(size_t)c * K + k]) * (double)G[(size_t)c * K + k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) {
    const float hi = (float)acc, lo = (float)(acc - (double)hi);
    // two slab rows of ns sets: [0, hi(, 0)] and [0, lo(, 0)] (set 2 = a projection block's
    // shortcut sums, which its own dgrad epilogue computed)
    for (int r = 0; r < 2; ++r)
      for (int j = 0; j < ns; ++j) out[(r * ns + j) * C + c] = j == 1 ? (r == 0 ? hi : lo) : 0.f;
  }
}

}  // namespace

hipError_t launch_bnfold_rowdot(const float* G, const void* w, int C, int K, int ns, float* out_rows, hipStream_t s) {
  if (C <= 0 || K <= 0 || ns < 2 || ns > 3) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_rowdot_kernel, dim3(C), dim3(64), 0, s, G, (const uint16_t*)w, C, K, ns, out_rows);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bnfold_prep(const float* coef, const void* w, const void* wt, int C, int K, void* wd, void* mx,
                              float* bias, const float* mu, const float* cs, long rows, hipStream_t s, int ldw,
                              int ldm) {
  if (ldw == 0) ldw = C;
  if (ldm == 0) ldm = K;
  if (ldw < C || ldm < K) return hipErrorInvalidValue;
  if (C <= 0 || K <= 0 || C > 8192 || (K < PREP_NT ? PREP_NT % K : K % PREP_NT) != 0) return hipErrorInvalidValue;
  const long n = (long)K * C;
  int gw = (int)((n + PREP_NT - 1) / PREP_NT);
  if (gw > 256) gw = 256;
  const size_t lds = (size_t)(C + PREP_NT) * sizeof(float);
  hipLaunchKernelGGL(bnfold_prep_kernel, dim3(K + gw), dim3(PREP_NT), lds, s, coef, (const uint16_t*)w,
                     (const uint16_t*)wt, C, K, (uint16_t*)wd, (uint16_t*)mx, ldw, ldm, bias, mu, cs,
                     rows > 0 ? 1.f / (float)rows : 0.f);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

// cs: [ncs][K] partial column sums of a2 (launch_bnfold_colsum)
hipError_t launch_bnfold_wgrad(const float* coef, const float* G, const float* S, const float* cs, int ncs,
                               const void* w, int C, int K, float* sink, int accumulate, hipStream_t s) {
  if (C <= 0 || K <= 0 || K > 8192 || ncs <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bnfold_wgrad_kernel, dim3(C), dim3(K < 256 ? ((K + 63) / 64) * 64 : 256),
                     (size_t)K * sizeof(float), s, coef, G, S, cs, ncs, (const uint16_t*)w, C, K, sink, accumulate);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

int bnfold_colsum_blocks() { return 512; }

// cs[K] fp32 = column sums of x [rows][K] bf16; partial: [bnfold_colsum_blocks()][K] scratch
hipError_t launch_bnfold_colsum(const void* x, long rows, int K, float* partial, float* cs, hipStream_t s) {
  if (K % 8 != 0 || K > 2048 || 256 % (K / 8) != 0) return hipErrorInvalidValue;
  const int nb = bnfold_colsum_blocks();
  hipLaunchKernelGGL(bnfold_colsum_kernel, dim3(nb), dim3(256), 0, s, (const uint16_t*)x, rows * K / 8, K, partial);
  SDX_LAUNCH_CHECK();
  hipLaunchKernelGGL(bnfold_colsum_finish_kernel, dim3((K + 63) / 64), dim3(1024), 0, s, partial, nb, K, cs);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
