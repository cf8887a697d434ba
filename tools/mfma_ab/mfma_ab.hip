// MFMA shape A/B on the conv kernels' wave tile (verdict r4 item 1b): a 64x64 fp32 output
// tile per wave, 8 waves per block (two per SIMD, as the 256x128 / 128x256 conv tiles), bf16
// operands re-read from LDS every k-step in the conv kernels' swizzled K-inner image
// ([rows][64] bf16, 16-B chunk ^ (row & 7)), random data, one block per CU x 4 rounds.
//   V16: v_mfma_f32_16x16x32_bf16, per 32-deep k-step 4 A + 4 B fragment reads, 16 MFMAs
//   V32: v_mfma_f32_32x32x16_bf16, per 32-deep k-step 4 A + 4 B fragment reads, 8 MFMAs
// Same LDS bytes per FLOP (the wave tile, not the instruction, sets them); the difference is
// the MFMA count and the clock the chip holds for each shape.
//
// hipcc --offload-arch=gfx950 -O3 -o mfma_ab tools/mfma_ab/mfma_ab.hip && ./mfma_ab
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr int NT = 512;                 // 8 waves
constexpr int ROWS = 256;               // A image rows (4 waves x 64) + B image rows (2 x 64)
constexpr int LDS_BYTES = 2 * ROWS * 128;   // two images of [256][64] bf16 (A, B)

__device__ __forceinline__ int kin_off(int row, int ch) { return row * 128 + ((ch ^ (row & 7)) << 4); }

template <int V>
__global__ __launch_bounds__(NT, 2) void mfma_loop(const uint4* __restrict__ src, float* __restrict__ out, int steps) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  for (int i = threadIdx.x; i < LDS_BYTES / 16; i += NT)
    reinterpret_cast<uint4*>(smem)[i] = src[(blockIdx.x * (LDS_BYTES / 16) + i) % (1 << 20)];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wm = wv >> 1, wn = wv & 1;     // 4 x 2 waves: wave tile rows wm*64, cols wn*64
  const unsigned char* A = smem;
  const unsigned char* B = smem + ROWS * 128;
  if constexpr (V == 16) {
    const int h = lane >> 4, c = lane & 15;
    f32x4 acc[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < steps; ++s) {
      const int u = s & 1;   // the two 32-deep halves of a 64-wide image row
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + kin_off(wm * 64 + 16 * i + c, 4 * u + h));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(B + kin_off(wn * 64 + 16 * j + c, 4 * u + h));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    }
    float t = 0.f;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    out[blockIdx.x * NT + threadIdx.x] = t;
  } else {
    // 32x32x16: lane (h = lane/32, c = lane%32) holds rows c, k = 8h..8h+7 of a 16-deep slice
    const int h = lane >> 5, c = lane & 31;
    f32x16 acc[2][2];
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int s = 0; s < steps; ++s) {
      const int u = s & 1;
#pragma unroll
      for (int q = 0; q < 2; ++q) {          // two 16-deep slices of the 32-deep step
        bf16x8 a[2], b[2];
        const int ch = 4 * u + 2 * q + h;
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(A + kin_off(wm * 64 + 32 * i + c, ch));
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const bf16x8*>(B + kin_off(wn * 64 + 32 * j + c, ch));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      }
    }
    float t = 0.f;
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    out[blockIdx.x * NT + threadIdx.x] = t;
  }
}

int main() {
  const int blocks = 256 * 4, steps = 4096;
  std::vector<uint16_t> h(1 << 23);
  unsigned x = 12345;
  for (auto& v : h) {   // random bf16 in [-1, 1): the clock the chip holds depends on the data
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) & 0xffff) / 32768.f - 1.f;
    unsigned u;
    std::memcpy(&u, &f, 4);
    v = (uint16_t)(u >> 16);
  }
  uint4* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, (size_t)blocks * NT * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double flop = 2.0 * blocks * 8 * 64 * 64 * 32.0 * steps;
  for (int round = 0; round < 3; ++round) {
    for (int v : {16, 32}) {
      for (int w = 0; w < 3; ++w) {   // warm (and let the clock settle)
        if (v == 16) hipLaunchKernelGGL(mfma_loop<16>, dim3(blocks), dim3(NT), 0, 0, src, out, steps);
        else hipLaunchKernelGGL(mfma_loop<32>, dim3(blocks), dim3(NT), 0, 0, src, out, steps);
      }
      CHECK(hipEventRecord(e0));
      const int reps = 10;
      for (int r = 0; r < reps; ++r) {
        if (v == 16) hipLaunchKernelGGL(mfma_loop<16>, dim3(blocks), dim3(NT), 0, 0, src, out, steps);
        else hipLaunchKernelGGL(mfma_loop<32>, dim3(blocks), dim3(NT), 0, 0, src, out, steps);
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("round %d  v_mfma_f32_%s_bf16: %.3f ms/launch  %.0f TFLOP/s\n", round,
                  v == 16 ? "16x16x32" : "32x32x16", ms / reps, flop / (ms / reps * 1e-3) / 1e12);
    }
  }
  return 0;
}
