// Small elementwise kernels of the projection-head executor (csrc/bindings/head_ops.cpp).
// The head's GEMMs themselves are igemm.hip launches (1x1 implicit GEMMs with bias / ReLU /
// fp32 epilogues); what is left is the precision hand-off around them.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

// fp32 -> bf16 (round to nearest even), 8 elements per lane
__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                            long n8) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n8; e += (long)gridDim.x * blockDim.x) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * e];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * e + 1];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    reinterpret_cast<uint4*>(y)[e] = pack8(v);
  }
}

}  // namespace

hipError_t launch_cast_f32_bf16(const float* x, void* y, long n, hipStream_t s) {
  if (n % 8 != 0) return hipErrorInvalidValue;
  const long n8 = n / 8;
  long g = (n8 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)g), dim3(256), 0, s, x, (uint16_t*)y, n8);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
