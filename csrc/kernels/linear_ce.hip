// Linear-probe classifier on the native path (reference main_linear.py:166-180:
// nn.Linear(feat_dim, n_cls) on frozen encoder features, nn.CrossEntropyLoss (mean),
// util.accuracy top-1 / top-5, torch.optim.SGD(momentum, weight_decay)) in TWO launches
// per training step instead of ~15 torch kernels (library GEMM, log-softmax, NLL, top-k,
// the two backward GEMMs, the bias reduction, the foreach SGD):
//
//   linear_ce_fwd  block = 4 rows x all classes. Every lane keeps its K/64 feature columns
//                  of the 4 rows in registers; wave w evaluates classes w, w+4, ... as 4
//                  fused dot products over the lanes (W rows read once per block, 16-B
//                  loads) + a DPP wave reduction, logits land in LDS; then wave r runs row
//                  r's softmax: loss_r = lse − z[label], dz = (softmax − onehot)·gscale
//                  (gscale = 1/B: the mean), hits@1/@5 = #{z_c > z_label} < k.
//   linear_ce_sgd  thread = 4 consecutive weights of one class: g = Σ_b dz[b][c]·x[b][k..k+3]
//                  (fixed row order: deterministic), then the SGD update in place
//                  (d = g + wd·w; buf = m·buf + d, buf = d on the first step; w −= lr·buf);
//                  the last block does the bias the same way and sums the per-row loss /
//                  hit counters into stats[3] in row order.
//
// fp32 throughout, as the reference's classifier (its GEMMs are ~0.1 GFLOP per step: the
// cost is launch count and latency, not FLOPs).
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

constexpr int kRows = 4;          // rows per forward block (one wave per row for the softmax)
constexpr int kMaxClasses = 1024;

__device__ __forceinline__ float lane_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float lane_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// KJ = K / 64 feature columns per lane
template <int KJ>
__global__ __launch_bounds__(256) void linear_ce_fwd_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                            const float* __restrict__ bias,
                                                            const int64_t* __restrict__ labels, int B, int C,
                                                            float gscale, float* __restrict__ logits,
                                                            float* __restrict__ dz, float* __restrict__ rowstat) {
  constexpr int K = 64 * KJ;
  __shared__ float z[kRows][kMaxClasses];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * kRows;
  float xv[kRows][KJ];
#pragma unroll
  for (int r = 0; r < kRows; ++r) {
    const int row = r0 + r;
#pragma unroll
    for (int j = 0; j < KJ; ++j) xv[r][j] = row < B ? x[(size_t)row * K + 64 * j + lane] : 0.f;
  }
  for (int c = wv; c < C; c += 4) {
    const float* wr = W + (size_t)c * K;
    float acc[kRows] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KJ; ++j) {
      const float w = wr[64 * j + lane];
#pragma unroll
      for (int r = 0; r < kRows; ++r) acc[r] = fmaf(xv[r][j], w, acc[r]);
    }
    const float b = bias[c];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const float s = lane_sum(acc[r]);
      if (lane == 0) z[r][c] = s + b;
    }
  }
  __syncthreads();
  // row softmax / cross-entropy / top-k hits: wave wv owns row r0 + wv
  const int row = r0 + wv;
  if (row >= B) return;
  const int lab = (int)labels[row];
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, z[wv][c]);
  m = lane_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(z[wv][c] - m);
  s = lane_sum(s);
  const float lse = m + __logf(s);
  const bool ok = lab >= 0 && lab < C;
  const float zl = ok ? z[wv][lab] : 0.f;
  float above = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = z[wv][c];
    logits[(size_t)row * C + c] = v;
    above += v > zl ? 1.f : 0.f;
    if (dz != nullptr) dz[(size_t)row * C + c] = (__expf(v - lse) - (c == lab ? 1.f : 0.f)) * gscale;
  }
  above = lane_sum(above);
  if (lane == 0) {
    rowstat[(size_t)row * 3 + 0] = ok ? lse - zl : NAN;
    rowstat[(size_t)row * 3 + 1] = (ok && above < 1.f) ? 1.f : 0.f;
    rowstat[(size_t)row * 3 + 2] = (ok && above < 5.f) ? 1.f : 0.f;
  }
}

// grid: ceil(C*K/4 / 256) weight blocks + 1 (bias + statistics); W == nullptr: statistics only
__global__ __launch_bounds__(256) void linear_ce_sgd_kernel(const float* __restrict__ x, const float* __restrict__ dz,
                                                            int B, int K, int C, float* __restrict__ W,
                                                            float* __restrict__ bias, float* __restrict__ bufW,
                                                            float* __restrict__ bufb, float lr, float mom, float wd,
                                                            int first, const float* __restrict__ rowstat,
                                                            float* __restrict__ stats) {
  const int nw4 = C * K / 4;
  if (blockIdx.x + 1 < gridDim.x) {
    if (W == nullptr) return;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= nw4) return;
    const int c = e / (K / 4), k = (e - c * (K / 4)) * 4;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int b = 0; b < B; ++b) {
      const float d = dz[(size_t)b * C + c];
      const float4 v = *reinterpret_cast<const float4*>(x + (size_t)b * K + k);
      g.x = fmaf(d, v.x, g.x);
      g.y = fmaf(d, v.y, g.y);
      g.z = fmaf(d, v.z, g.z);
      g.w = fmaf(d, v.w, g.w);
    }
    float4* wp = reinterpret_cast<float4*>(W + (size_t)c * K + k);
    float4* bp = reinterpret_cast<float4*>(bufW + (size_t)c * K + k);
    float4 w = *wp, bu = *bp;
    const float gg[4] = {g.x, g.y, g.z, g.w};
    float* ww = reinterpret_cast<float*>(&w);
    float* bb = reinterpret_cast<float*>(&bu);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float d = gg[q] + wd * ww[q];
      bb[q] = first ? d : fmaf(mom, bb[q], d);
      ww[q] -= lr * bb[q];
    }
    *wp = w;
    *bp = bu;
    return;
  }
  // last block: bias gradient + update, statistics in row order
  if (W != nullptr) {
    for (int c = threadIdx.x; c < C; c += 256) {
      float g = 0.f;
      for (int b = 0; b < B; ++b) g += dz[(size_t)b * C + c];
      const float d = g + wd * bias[c];
      bufb[c] = first ? d : fmaf(mom, bufb[c], d);
      bias[c] -= lr * bufb[c];
    }
  }
  if (threadIdx.x < 3) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += rowstat[(size_t)b * 3 + threadIdx.x];
    stats[threadIdx.x] = s;
  }
}

}  // namespace

bool linear_ce_supported(int K, int C) { return K % 64 == 0 && K >= 64 && K <= 64 * 32 && C >= 1 && C <= kMaxClasses; }

hipError_t launch_linear_ce_fwd(const float* x, const float* W, const float* bias, const int64_t* labels, int B,
                                int K, int C, float gscale, float* logits, float* dz, float* rowstat, hipStream_t s) {
  if (!linear_ce_supported(K, C) || B < 1) return hipErrorInvalidValue;
  const dim3 grid((B + kRows - 1) / kRows), blk(256);
  switch (K / 64) {
#define SDX_LCE(KJ)                                                                                          \
  case KJ:                                                                                                  \
    hipLaunchKernelGGL((linear_ce_fwd_kernel<KJ>), grid, blk, 0, s, x, W, bias, labels, B, C, gscale, logits, dz, \
                       rowstat);                                                                            \
    break;
    SDX_LCE(1) SDX_LCE(2) SDX_LCE(4) SDX_LCE(8) SDX_LCE(16) SDX_LCE(32)
#undef SDX_LCE
    default:
      return hipErrorInvalidValue;   // K / 64 must be a power of two <= 32
  }
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_linear_ce_sgd(const float* x, const float* dz, int B, int K, int C, float* W, float* bias,
                                float* bufW, float* bufb, float lr, float mom, float wd, int first,
                                const float* rowstat, float* stats, hipStream_t s) {
  if (B < 1 || K % 4 != 0 || C < 1) return hipErrorInvalidValue;
  const int nw4 = C * K / 4;
  const dim3 grid(W != nullptr ? (nw4 + 255) / 256 + 1 : 1), blk(256);
  hipLaunchKernelGGL(linear_ce_sgd_kernel, grid, blk, 0, s, x, dz, B, K, C, W, bias, bufW, bufb, lr, mom, wd, first,
                     rowstat, stats);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
