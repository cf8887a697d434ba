// Per-step weight preparation: one launch converts EVERY conv weight of the model from
// the fp32 master copy (flat buffer, channels_last i.e. KRSC physical) into the two bf16
// layouts the implicit-GEMM kernels consume:
//   fwd   Wk [K][R][S][Cp]   (input channels zero-padded to Cp, e.g. 3 -> 8 for the stem)
//   dgrad Wt [C][R][S][K]    (transposed)
// replacing ~2 x 53 small cast/permute launches per step. A segment table (one row per
// conv) maps each thread's element to its layer by binary search.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

struct WSeg {
  long src;      // element offset of W[K][R][S][C] (fp32) in the master buffer
  long dst_k;    // element offset of Wk in the bf16 output (fwd layout)
  long dst_t;    // element offset of Wt in the bf16 output (dgrad layout), -1: none
  int K, RS, C, Cp;
  long n;        // K*RS*Cp (fwd elements of this segment)
  long start;    // first tile of this segment: prefix sum of ceil(K/64)·ceil(Cp/64)·RS
};

// One block per 64(k) x 64(c) tile at one filter tap rs, over ALL segments: block b belongs to
// the last segment whose first tile is <= b (binary search over the uniform segment table).
// A [largest conv's tiles] x [segments] grid launched ~57k blocks for ~7k tiles of work
// (the head's 2048x2048 Linear sets the largest); the empty ones cost dispatch time.
// Reads of the fp32 master and writes of Wk are coalesced along c; the transposed Wt tile
// goes through LDS so its writes are coalesced along k. Segments with C % 4 == 0 and no
// channel padding (every conv but the stem, and the head's Linear layers) move 16-B float4
// loads and 8-B bf16x4 stores per thread (a scalar fp32 load / 2-B store per element made
// this a latency-bound 72 us pass per step).
__global__ __launch_bounds__(256) void wprep_kernel(const float* __restrict__ master, uint16_t* __restrict__ out,
                                                    const WSeg* __restrict__ segs, int nseg) {
  __shared__ uint16_t tile[64][66];
  const long b = blockIdx.x;
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].start <= b) lo = mid;
    else hi = mid - 1;
  }
  const WSeg s = segs[lo];
  const int kt = (s.K + 63) / 64, ct = (s.Cp + 63) / 64;
  int t = (int)(b - s.start);
  if (t < 0 || t >= kt * ct * s.RS) return;
  const int cti = t % ct; t /= ct;
  const int rs = t % s.RS;
  const int kti = t / s.RS;
  const int k0 = kti * 64, c0 = cti * 64;
  const bool vec = (s.C & 3) == 0 && s.Cp == s.C && (s.K & 3) == 0;
  if (vec) {
    // 16 threads per 64-channel row, 16 rows per pass, all 4 passes' loads in flight
    const int cq = (threadIdx.x & 15) * 4, r0 = threadIdx.x >> 4;
    const int c = c0 + cq;
    float4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + r0 + 16 * i;
      v[i] = (k < s.K && c < s.C) ? *reinterpret_cast<const float4*>(master + s.src + ((long)k * s.RS + rs) * s.C + c)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = r0 + 16 * i, k = k0 + kk;
      const uint16_t b0 = f2bf(v[i].x), b1 = f2bf(v[i].y), b2 = f2bf(v[i].z), b3 = f2bf(v[i].w);
      if (k < s.K && c < s.C)
        *reinterpret_cast<uint2*>(out + s.dst_k + ((long)k * s.RS + rs) * s.Cp + c) =
            make_uint2((uint32_t)b0 | ((uint32_t)b1 << 16), (uint32_t)b2 | ((uint32_t)b3 << 16));
      tile[kk][cq] = b0;
      tile[kk][cq + 1] = b1;
      tile[kk][cq + 2] = b2;
      tile[kk][cq + 3] = b3;
    }
    if (s.dst_t < 0) return;
    __syncthreads();
    // transposed: 4 consecutive k of one input channel per thread (8-B stores along k)
    const int kq = (threadIdx.x & 15) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cc = r0 + 16 * i, cw = c0 + cc, k = k0 + kq;
      if (cw < s.C && k < s.K)
        *reinterpret_cast<uint2*>(out + s.dst_t + ((long)cw * s.RS + rs) * s.K + k) =
            make_uint2((uint32_t)tile[kq][cc] | ((uint32_t)tile[kq + 1][cc] << 16),
                       (uint32_t)tile[kq + 2][cc] | ((uint32_t)tile[kq + 3][cc] << 16));
    }
    return;
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int kk = ty; kk < 64; kk += 4) {
    const int k = k0 + kk, c = c0 + tx;
    if (k < s.K && c < s.Cp) {
      const float v = c < s.C ? master[s.src + ((long)k * s.RS + rs) * s.C + c] : 0.f;
      const uint16_t b = f2bf(v);
      out[s.dst_k + ((long)k * s.RS + rs) * s.Cp + c] = b;
      tile[kk][tx] = b;
    }
  }
  if (s.dst_t < 0) return;
  __syncthreads();
  for (int cc = ty; cc < 64; cc += 4) {
    const int c = c0 + cc, k = k0 + tx;
    if (c < s.C && k < s.K) out[s.dst_t + ((long)c * s.RS + rs) * s.K + k] = tile[tx][cc];
  }
}

// dst[r][c] += src[r][c] for c < C of a channel-padded [rows][Cp] fp32 weight gradient (the
// stem's 3 input channels are padded to 8 for its conv kernels): the fp32 gradient sink keeps
// the unpadded [K][R][S][C] layout
__global__ __launch_bounds__(256) void unpad_add_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                        int rows, int Cp, int C) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * C) return;
  const int r = e / C, c = e - r * C;
  dst[e] += src[(long)r * Cp + c];
}

}  // namespace

hipError_t launch_unpad_add(const float* src, float* dst, int rows, int Cp, int C, hipStream_t s) {
  if (rows < 1 || C < 1 || C > Cp) return hipErrorInvalidValue;
  hipLaunchKernelGGL(unpad_add_kernel, dim3((rows * C + 255) / 256), dim3(256), 0, s, src, dst, rows, Cp, C);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_wprep(const float* master, void* out, const void* segs, int nseg, long total, hipStream_t s) {
  // `total` = the tile count of all segments (Σ ceil(K/64)·ceil(Cp/64)·R·S); segs[i].start =
  // the prefix of it (host-computed, ops/weights.py)
  if (total < 1 || nseg < 1 || total > (1L << 31) - 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wprep_kernel, dim3((unsigned)total), dim3(256), 0, s, master, (uint16_t*)out,
                     (const WSeg*)segs, nseg);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
