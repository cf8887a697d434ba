// One-shot all-reduce for small, latency-bound messages over xGMI peer memory
// (the 53 + 49 SyncBN statistic all-reduces per step, ≤16 KiB each, sit on
// the critical path; a ring collective pays 2(W−1) link latencies for each of them).
//
// Every rank owns an IPC-shared receive arena in uncached device memory:
//   data [2 parity][W senders][cap] fp64,   flags [2 parity][W senders][64 groups] u32
//   (this kernel uses group 0; the SyncBN column reduction of bn.hip one flag per
//   64-channel group — every call uses group 0, so the parity argument below holds for
//   any mix of the two).
// A call with epoch e (host counter, starting at 1) and parity e&1:
//   1. each rank stores its n values straight into slot [parity][me] of EVERY rank's arena
//      (remote stores travel over the point-to-point xGMI link to that peer);
//   2. each storing wave drains its stores, then one lane publishes `e` into flags
//      [parity][me] of every arena with a system-scope release store;
//   3. each rank polls its own W flags, acquires, and sums the W slots in rank order —
//      every rank computes bit-identical results. The poll is bounded by a wall-clock
//      deadline (the 100 MHz constant clock, --comm_timeout): a dead or lagging peer makes
//      the kernel give up, skip the sum and store 1 + that peer's rank into the error word,
//      which lives in host-pinned memory — the native communicator's host watchdog
//      (comm_ops.cpp) reads it without a device copy and ends the process with status 3
//      instead of training on stale statistics.
// Two parities make the arena reusable without a second barrier: a rank can only start
// call e+2 (same parity) after it saw every peer's flag for e+1, which each peer wrote
// after it had finished reading call e.
//
// The emulation kernel runs the SAME protocol with W virtual ranks = W blocks of one launch
// on one GPU (arenas in ordinary device memory, agent scope suffices there): it exercises
// the slot/flag/parity logic on the single-GPU test box.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {


template <int SCOPE>
__device__ void oneshot_body(const double* __restrict__ in, double* __restrict__ out, int n, const XgmiPeers& peers,
                             int me, int world, unsigned epoch_host, int* err, long long timeout_ticks,
                             unsigned* ctr = nullptr) {
  // the arena's device epoch (XgmiCol::epoch_ctr: [epoch, ticket]) when given, else the host's
  __shared__ unsigned ep_s;
  if (threadIdx.x == 0)
    ep_s = ctr != nullptr ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : epoch_host;
  __syncthreads();
  const unsigned epoch = ep_s;
  const int par = epoch & 1;
  const size_t cap = peers.cap;
  // 1. scatter my contribution into every arena
  for (int q = 0; q < world; ++q) {
    double* dst = peers.data[q] + ((size_t)par * world + me) * cap;
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = in[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 2. publish
  if (threadIdx.x < world) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (SCOPE == 1)
      __hip_atomic_store(peers.flags[threadIdx.x] + (par * world + me) * kXgmiFlagGroups, epoch, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(peers.flags[threadIdx.x] + (par * world + me) * kXgmiFlagGroups, epoch, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // 3. wait for every sender's flag in my arena
  __shared__ int ok_all;
  if (threadIdx.x == 0) ok_all = 1;
  __syncthreads();
  if (threadIdx.x < world) {
    unsigned* f = peers.flags[me] + (par * world + threadIdx.x) * kXgmiFlagGroups;
    const long long t0 = wall_clock64();
    unsigned spins = 0;
    while (true) {
      const unsigned v = SCOPE == 1 ? __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)
                                    : __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (v == epoch) break;
      if ((++spins & 63) == 0 && wall_clock64() - t0 > timeout_ticks) {
        atomicExch(&ok_all, 0);
        // host-pinned word for the real arena (system scope), device word for the emulation
        if (err) __hip_atomic_store(err, 1 + (int)threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (ctr != nullptr && threadIdx.x == 0) __hip_atomic_store(ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!ok_all) return;
  if (SCOPE == 1)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const double* base = peers.data[me] + (size_t)par * world * cap;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    double s = 0.0;
    for (int q = 0; q < world; ++q) s += __hip_atomic_load(base + (size_t)q * cap + i, __ATOMIC_RELAXED,
                                                            SCOPE == 1 ? __HIP_MEMORY_SCOPE_SYSTEM
                                                                       : __HIP_MEMORY_SCOPE_AGENT);
    out[i] = s;
  }
}

__global__ __launch_bounds__(256) void oneshot_kernel(const double* in, double* out, int n, XgmiPeers peers, int me,
                                                      int world, unsigned epoch, int* err, long long timeout_ticks,
                                                      unsigned* ctr) {
  oneshot_body<1>(in, out, n, peers, me, world, epoch, err, timeout_ticks, ctr);
}

// block b = virtual rank b; in/out are [W][n]; peers.data/flags are the W local arenas
__global__ __launch_bounds__(256) void oneshot_emulate_kernel(const double* in, double* out, int n, XgmiPeers peers,
                                                              int world, unsigned epoch, int* err) {
  const int me = blockIdx.x;
  // all virtual ranks are co-resident blocks of this launch: a missing flag is a protocol
  // bug, reported after ~1 s of the 100 MHz clock
  oneshot_body<0>(in + (size_t)me * n, out + (size_t)me * n, n, peers, me, world, epoch, err, 100000000LL);
}

// Bounded GPU stall for the watchdog tests: one wave sleeps until `ticks` of the 100 MHz
// constant clock have passed (never longer), standing in for a collective whose peer hangs.
__global__ __launch_bounds__(64) void stall_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace

hipError_t launch_xgmi_allreduce(const double* in, double* out, int n, const XgmiPeers& peers, int me, int world,
                                 unsigned epoch, int* err, long long timeout_ticks, hipStream_t s, unsigned* epoch_ctr) {
  if (n < 0 || (size_t)n > peers.cap || world < 1 || world > kXgmiMaxPeers || timeout_ticks <= 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(oneshot_kernel, dim3(1), dim3(256), 0, s, in, out, n, peers, me, world, epoch, err,
                     timeout_ticks, epoch_ctr);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_xgmi_emulate(const double* in, double* out, int n, const XgmiPeers& peers, int world,
                               unsigned epoch, int* err, hipStream_t s) {
  if (n < 0 || (size_t)n > peers.cap || world < 1 || world > kXgmiMaxPeers) return hipErrorInvalidValue;
  hipLaunchKernelGGL(oneshot_emulate_kernel, dim3(world), dim3(256), 0, s, in, out, n, peers, world, epoch, err);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_gpu_stall(long long ticks, hipStream_t s) {
  if (ticks < 0 || ticks > 2000000000LL) return hipErrorInvalidValue;   // at most 20 s
  hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, s, ticks);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
