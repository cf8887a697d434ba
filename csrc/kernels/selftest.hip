// Toolchain / MFMA-layout self test: one wave computes a 16x16 = (16x32)·(32x16) bf16
// product with v_mfma_f32_16x16x32_bf16. Used by tests/test_gpu_selftest.py to pin the
// lane maps (asymmetric operands) before any larger kernel relies on them.
#include "common.h"
#include "launchers.h"

using namespace sdx;

__global__ __launch_bounds__(64) void mfma16_selftest_kernel(const uint16_t* __restrict__ A,  // [16][32]
                                                             const uint16_t* __restrict__ B,  // [32][16]
                                                             float* __restrict__ C) {          // [16][16]
  const int l = threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (l >> 4) + j;
    a[j] = (short)A[(l & 15) * 32 + k];
    b[j] = (short)B[k * 16 + (l & 15)];
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}

hipError_t launch_mfma16_selftest(const void* A, const void* B, float* C, hipStream_t s) {
  hipLaunchKernelGGL(mfma16_selftest_kernel, dim3(1), dim3(64), 0, s, (const uint16_t*)A,
                     (const uint16_t*)B, C);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
