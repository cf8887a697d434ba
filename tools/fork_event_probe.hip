// Cost of a stream fork point on the producing stream: a chain of N small dependent kernels on
// stream A, with after each kernel either nothing (mode 0), hipEventRecord + a wait on stream B
// (mode 1), or the same event bound to the kernel itself as hipExtLaunchKernelGGL's stop event
// (mode 2). Event flags: DisableTiming (+ DisableSystemFence with argv[1] = 1).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/fork_event_probe tools/fork_event_probe.hip
//   /tmp/fork_event_probe [nofence]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void axpy(float* __restrict__ y, const float* __restrict__ x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = y[i] * 0.999f + x[i];
}

int main(int argc, char** argv) {
  const bool nofence = argc > 1 && atoi(argv[1]) != 0;
  const int n = 1 << 20, N = 2000;
  float *x, *y, *z;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&z, n * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, n * 4));
  CK(hipMemset(z, 0, n * 4));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(N);
  const unsigned fl = hipEventDisableTiming | (nofence ? hipEventDisableSystemFence : 0u);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, fl));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const dim3 grid(n / 256), blk(256);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, a));
      for (int i = 0; i < N; ++i) {
        if (mode == 2) {
          hipExtLaunchKernelGGL(axpy, grid, blk, 0, a, nullptr, ev[i], 0, y, x, n);
          CK(hipGetLastError());
        } else {
          hipLaunchKernelGGL(axpy, grid, blk, 0, a, y, x, n);
          CK(hipGetLastError());
          if (mode == 1) CK(hipEventRecord(ev[i], a));
        }
        if (mode != 0 && i % 8 == 0) {
          // the consumer: a wait + a small kernel on stream B every 8th fork
          CK(hipStreamWaitEvent(b, ev[i], 0));
          hipLaunchKernelGGL(axpy, dim3(64), blk, 0, b, z, x, 64 * 256);
          CK(hipGetLastError());
        }
      }
      CK(hipEventRecord(t1, a));
      CK(hipDeviceSynchronize());
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      printf("mode %d (%s) rep %d: %.2f us per kernel on stream A\n", mode,
             mode == 0 ? "chain" : mode == 1 ? "record after each" : "stop event bound", rep, ms * 1e3f / N);
    }
  }
  printf("event flags: DisableTiming%s\n", nofence ? " | DisableSystemFence" : "");
  return 0;
}
