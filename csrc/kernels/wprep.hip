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
  long n;        // K*RS*Cp (fwd elements; the work index space of this segment)
  long start;    // prefix sum of n
};

__global__ __launch_bounds__(256) void wprep_kernel(const float* __restrict__ master, uint16_t* __restrict__ out,
                                                    const WSeg* __restrict__ segs, int nseg, long total) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (segs[mid].start <= e) lo = mid; else hi = mid - 1;
    }
    const WSeg s = segs[lo];
    const long i = e - s.start;               // index into Wk [K][RS][Cp]
    const int cp = (int)(i % s.Cp);
    const long t = i / s.Cp;
    const int rs = (int)(t % s.RS);
    const int k = (int)(t / s.RS);
    float v = 0.f;
    if (cp < s.C) v = master[s.src + ((long)k * s.RS + rs) * s.C + cp];
    const uint16_t b = f2bf(v);
    out[s.dst_k + i] = b;
    if (s.dst_t >= 0 && cp < s.C) out[s.dst_t + ((long)cp * s.RS + rs) * s.K + k] = b;
  }
}

}  // namespace

hipError_t launch_wprep(const float* master, void* out, const void* segs, int nseg, long total, hipStream_t s) {
  long grid = (total + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(wprep_kernel, dim3(grid), dim3(256), 0, s, master, (uint16_t*)out, (const WSeg*)segs, nseg,
                     total);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
