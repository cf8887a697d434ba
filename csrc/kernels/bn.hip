// BatchNorm (training + eval) kernels for NHWC bf16 activations on gfx950.
//
// Forward statistics come from the convolution epilogue (igemm.hip: per-M-tile Σy, Σy²);
// here they are reduced in fp64 (bn_stats_reduce), optionally all-reduced across ranks
// by the caller (SyncBN: one fp64 all-reduce of [2][C] per layer), and turned into the
// per-channel affine (bn_finalize, which also updates running_mean / running_var with
// the unbiased variance, momentum 0.1 as torch BatchNorm2d). The affine is applied by
// one fused elementwise pass together with the residual branch and the ReLU
// (bn_apply: relu(bn(y) [+ bn'(y') | + x])) — reference: networks/resnet_big.py:57-67.
//
// Backward: bn_bwd_reduce recomputes dz = dout·[out>0] and accumulates Σdz and
// Σdz·(y−μ) for up to two BNs sharing dz (residual branch + projection shortcut);
// bn_bwd_coef folds those into per-channel (A, D, E) so that dy = A·dz + D·y + E, plus
// dγ/dβ; bn_bwd_apply is one elementwise pass producing dy (and dz for an identity
// shortcut). All elementwise kernels move 8 bf16 (16 B) per lane.
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "bn_epilogue.h"

using namespace sdx;

namespace {

#ifndef SDX_EW_UNROLL
#define SDX_EW_UNROLL 1
#endif
// rows per trip of the column reduction's row loop (col_reduce_kernel); 4 = round-2 code
#ifndef SDX_CR_UNROLL
#define SDX_CR_UNROLL 8
#endif

// slab [rows][NS][C] fp32 -> sums [NS][C] fp64 in one launch. grid (ceil(C/64), gy): block
// (x, y) sums its contiguous row range for 64 channels (4 thread rows, fp64) into
// scratch[y][NS][C]; it then takes an agent-scope ticket on counters[x], and the block that
// draws gy-1 adds the gy partials in fixed order — deterministic for any dispatch order /
// XCD placement — writes the sums, runs the per-channel epilogue and resets the counter for
// the next launch (counters are zeroed once at allocation). The partials are handed off
// with write-through (sc1) stores and read back with sc1 loads, so no agent-scope release
// fence is needed: such a fence would write back the whole L2 (still dirty with the
// producing conv's output) in every block.
//
// XG != 0: SyncBN exchange before the epilogue (launchers.h XgmiCol). The last block of
// group x stores its [NS][64] sums into slot [parity][me] of every rank's arena with
// write-through (system scope: the arenas are uncached, IPC-mapped peer memory; agent
// scope for the single-GPU emulation) stores, drains them (s_waitcnt vmcnt(0): the
// stores are acknowledged), publishes the epoch in flag [parity][me][x] of every arena,
// and polls its own W flags of group x against the wall-clock deadline. The slots are
// then summed in rank order, so every rank holds bit-identical global sums, and the
// epilogue (finalize / coefficients, with the global count) runs on them. Every 64-channel
// group is an independent instance of the two-parity protocol of xgmi.hip. With real peers
// (mode 1) no block waits on another block of its own launch. In the single-GPU emulation
// (mode 2) virtual rank z's last block of group x DOES spin on the other ranks' last blocks
// of the same launch, so progress needs them co-resident: launch_col_reduce bounds the
// spinners (groups x W <= 512, far below the 256-CU residency) — solo mode (one rank's
// share) polls only its own flag.
template <int NS, int XG>
__device__ bool xg_exchange(double (&t)[NS], int c, int C, const XgmiCol& xg, int me) {
  constexpr int kScope = XG == 1 ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT;
  const int W = xg.world;
  // this exchange's epoch: the rank's device epoch + 1 (graph-replay safe), else the host's.
  // Pair [epoch, ticket] per rank (per virtual rank when emulated); the group finishing last
  // stores the new epoch, after every group of this launch has read the old one
  unsigned* ctr = xg.epoch_ctr != nullptr ? xg.epoch_ctr + 2 * (XG == 2 ? me : 0) : nullptr;
  __shared__ unsigned ep_s;
  if (threadIdx.x == 0)
    ep_s = ctr != nullptr ? __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : xg.epoch;
  __syncthreads();
  const unsigned epoch = ep_s;
  const int par = epoch & 1;
  const size_t cap = xg.peers.cap;
  __shared__ int ok;
  if (threadIdx.x < 64 && c < C) {
    for (int p = 0; p < W; ++p) {
      unsigned long long* dst =
          reinterpret_cast<unsigned long long*>(xg.peers.data[p] + ((size_t)par * W + me) * cap);
#pragma unroll
      for (int q = 0; q < NS; ++q)
        __hip_atomic_store(dst + (size_t)q * C + c, (unsigned long long)__double_as_longlong(t[q]), __ATOMIC_RELAXED,
                           kScope);
    }
  }
  // Ordering argument (why no system-scope release / acquire fences).
  //  Producer: every data store above is a system-scope atomic store (sc0 sc1: write-
  //   through, never held in this GPU's L1/L2) into the destination rank's arena, which is
  //   allocated uncached (hipDeviceMallocUncached) and, for peers, reached over xGMI. The
  //   vmcnt(0) below returns only when each store is ACKNOWLEDGED by the memory that owns the
  //   arena (its memory controller, behind which that GPU's own uncached loads are served),
  //   i.e. the bytes are globally visible. Only then does the same wave (lanes p < W, after
  //   the barrier) issue the flag stores, themselves system-scope write-through: a flag can
  //   never be visible before the data it publishes. A release fence would add nothing for
  //   these bytes -- its buffer_wbl2 writes back DIRTY L2 lines, and the payload never sits
  //   in L2 -- but it would write back the whole XCD L2 (the producing conv's output) in
  //   every exchange: ~2-7 us x 106 exchanges per step.
  //  Consumer: wave 0 polls its flags with system-scope loads (sc0 sc1: fetched from the
  //   arena's memory on every poll, never from a cache), waits for the value (the compare
  //   consumes it), passes the barrier and only THEN issues the data loads, also system-scope
  //   loads of the uncached arena that bypass L1/L2. No load of the payload can be served from
  //   a cache line older than the flag, so the acquire's buffer_inv (which would drop the
  //   XCD's L2) is not needed either.
  //  Both arguments rest on every payload and flag access being a system-scope atomic on the
  //   uncached arena (checked: no plain load or store of xg.peers.* exists) and on vmcnt
  //   acknowledgement meaning completion at the destination for write-through stores, which
  //   is how CDNA reports them. Same-device IPC (tests/test_gpu_dist.py, 4 processes,
  //   >300 exchanges) and the emulation exercise the same instruction sequence; a cross-
  //   device run is the remaining check (the default transport is RCCL until then).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's data stores are acknowledged
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  if (threadIdx.x < W) {
    // wave 0: the same wave that stored the data, after its drain. Every lane p < W publishes
    // this rank's flag to peer p; solo mode (one rank's share, diagnostic) then polls only
    // its own slot (the other W-1 ranks count as already published)
    const int p = threadIdx.x;
    __hip_atomic_store(xg.peers.flags[p] + ((size_t)par * W + me) * kXgmiFlagGroups + blockIdx.x, epoch,
                       __ATOMIC_RELAXED, kScope);
  }
  if (threadIdx.x < W && !(XG == 2 && xg.solo && threadIdx.x != me)) {
    const int p = threadIdx.x;
    unsigned* f = xg.peers.flags[me] + ((size_t)par * W + p) * kXgmiFlagGroups + blockIdx.x;
    const long long t0 = wall_clock64();
    unsigned spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, kScope) != epoch) {
      if ((++spins & 63) == 0 && wall_clock64() - t0 > xg.timeout_ticks) {
        atomicExch(&ok, 0);
        if (xg.err) __hip_atomic_store(xg.err, 1 + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (ctr != nullptr && threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {   // every column group of this launch has taken its epoch
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (!ok) return false;
  if (threadIdx.x < 64 && c < C) {
    const unsigned long long* base =
        reinterpret_cast<const unsigned long long*>(xg.peers.data[me] + (size_t)par * W * cap);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      double v = 0.0;
      for (int p = 0; p < W; ++p)
        v += __longlong_as_double(
            (long long)__hip_atomic_load(base + (size_t)p * cap + (size_t)q * C + c, __ATOMIC_RELAXED, kScope));
      t[q] = v;
    }
  }
  return true;
}

template <int NS, int EPI, int XG>
__global__ __launch_bounds__(256) void col_reduce_kernel(const float* __restrict__ slab, int rows, int C,
                                                         double* scratch, unsigned* counters,
                                                         double* __restrict__ sums, BnFinalizeArgs fa, BnCoefArgs ca,
                                                         XgmiCol xg) {
  __shared__ double red[NS][4][64];
  __shared__ int is_last;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // emulated ranks (XG == 2): virtual rank z = blockIdx.z has its own slab, scratch and counters
  const int vz = XG == 2 ? (int)blockIdx.z : 0;
  if constexpr (XG == 2) {
    slab += (size_t)vz * xg.slab_zstride;
    scratch += (size_t)vz * gridDim.y * NS * C;
    counters += vz * 64;
  }
  const int c = blockIdx.x * 64 + tx;
  const int gy = gridDim.y;
  const int per = (rows + gy - 1) / gy;
  const int r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  double acc[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) acc[q] = 0.0;
  if (c < C) {
    // SDX_CR_UNROLL rows per trip: that many x NS independent loads in flight per thread. The
    // loop is latency-bound (the slab was just written by a conv epilogue on other CUs /
    // XCDs), so the trip count, not the bytes, sets its time: 8 rows per trip halves the
    // trips of the former 4.
    constexpr int U = SDX_CR_UNROLL;
    int r = r0 + ty;
    for (; r + 4 * (U - 1) < r1; r += 4 * U) {
      float v[U][NS];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < NS; ++q) v[u][q] = slab[((size_t)(r + 4 * u) * NS + q) * C + c];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < NS; ++q) acc[q] += (double)v[u][q];
    }
    for (; r < r1; r += 4)
#pragma unroll
      for (int q = 0; q < NS; ++q) acc[q] += (double)slab[((size_t)r * NS + q) * C + c];
  }
#pragma unroll
  for (int q = 0; q < NS; ++q) red[q][ty][tx] = acc[q];
  __syncthreads();
  unsigned long long* sc = reinterpret_cast<unsigned long long*>(scratch);
  if (ty == 0 && c < C) {
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const double v = red[q][0][tx] + red[q][1][tx] + red[q][2][tx] + red[q][3][tx];
      __hip_atomic_store(sc + ((size_t)blockIdx.y * NS + q) * C + c, (unsigned long long)__double_as_longlong(v),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1 write-through
    }
  }
  if (gy > 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(counters + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      is_last = (t == (unsigned)gy - 1u);
    }
    __syncthreads();
    if (!is_last) return;
  }
  // combine: thread row ty sums partials y = ty, ty+4, ... (all loads issued up front), then
  // the 4 row sums are added in fixed order
  {
    double t[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) t[q] = 0.0;
    if (c < C) {
      constexpr int MAXY = 16;   // gy <= 64
      unsigned long long v[MAXY][NS];
#pragma unroll
      for (int k = 0; k < MAXY; ++k) {
        const int y = ty + 4 * k;
        if (y < gy) {
#pragma unroll
          for (int q = 0; q < NS; ++q)
            v[k][q] = __hip_atomic_load(sc + ((size_t)y * NS + q) * C + c, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);   // sc1 loads
        }
      }
#pragma unroll
      for (int k = 0; k < MAXY; ++k)
        if (ty + 4 * k < gy)
#pragma unroll
          for (int q = 0; q < NS; ++q) t[q] += __longlong_as_double((long long)v[k][q]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NS; ++q) red[q][ty][tx] = t[q];
    __syncthreads();
  }
  double t[NS];
#pragma unroll
  for (int q = 0; q < NS; ++q) t[q] = red[q][0][tx] + red[q][1][tx] + red[q][2][tx] + red[q][3][tx];
  bool go = true;
  if constexpr (XG != 0) go = xg_exchange<NS, XG>(t, c, C, xg, XG == 2 ? vz : xg.me);
  if (go && ty == 0 && c < C && vz == 0) {
#pragma unroll
    for (int q = 0; q < NS; ++q) sums[(size_t)q * C + c] = t[q];
    if constexpr (EPI == 1) bn_finalize_one(c, t[0], t[1], fa);
    if constexpr (EPI == 2) bn_coef_one(c, C, t, NS - 1, ca);
    if constexpr (EPI == 3) ca.dbeta_a[c] += (float)(t[0] * ca.grad_scale);
  }
  if (gy > 1 && threadIdx.x == 0) __hip_atomic_store(counters + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void bn_finalize_kernel(const double* __restrict__ sums, int C, BnFinalizeArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) bn_finalize_one(c, sums[c], sums[C + c], a);
}

// eval-mode affine from running statistics
__global__ void bn_eval_affine_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                      float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f;
  scale[c] = g * invstd;
  shift[c] = (beta ? beta[c] : 0.f) - rm[c] * g * invstd;
}

__device__ __forceinline__ void load8c(const float* __restrict__ p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// out = act(y*sc + sh [+ r*sc2 + sh2 | + r])     res_mode: 0 none, 1 bn'd residual, 2 raw residual
// 32-bit indexing (tensors < 2^31 elements). When the grid stride is a multiple of C/8
// (always for power-of-two C <= 2048) the channel group is fixed per thread: the per-channel
// coefficients are loaded once into registers.
// 1 bit per element of 8 packed bf16: set iff the value is > 0 (the ReLU mask of a block
// output, kept for backward at 1/16 of the activation's bytes)
__device__ __forceinline__ uint8_t relu_bits(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = w[q] & 0xffffu, hi = w[q] >> 16;
    b |= (uint32_t)((lo & 0x7fffu) != 0 && !(lo & 0x8000u)) << (2 * q);
    b |= (uint32_t)((hi & 0x7fffu) != 0 && !(hi & 0x8000u)) << (2 * q + 1);
  }
  return (uint8_t)b;
}

template <int RES, bool RELU>
struct ApplyOp {
  float ss[8], tt[8], aa[8], bb[8];
  __device__ __forceinline__ void load(const float* sc, const float* sh, const float* sc2, const float* sh2, int c0) {
    load8c(sc + c0, ss);
    load8c(sh + c0, tt);
    if (RES == 1) {
      load8c(sc2 + c0, aa);
      load8c(sh2 + c0, bb);
    }
  }
  __device__ __forceinline__ uint4 run(uint4 yv, uint4 rv4) const {
    float v[8];
    unpack8(yv, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = v[i] * ss[i] + tt[i];
    if (RES != 0) {
      float rv[8];
      unpack8(rv4, rv);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += RES == 1 ? rv[i] * aa[i] + bb[i] : rv[i];
    }
    if (RELU) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], 0.f);
    }
    return pack8(v);
  }
};

template <int RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ y, const float* __restrict__ sc,
                                                       const float* __restrict__ sh, const uint16_t* __restrict__ r,
                                                       const float* __restrict__ sc2, const float* __restrict__ sh2,
                                                       uint16_t* __restrict__ out, long n8l, int C8,
                                                       uint8_t* __restrict__ mask_out) {
  const int n8 = (int)n8l, stride = gridDim.x * blockDim.x;
  const int e0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* Y = reinterpret_cast<const uint4*>(y);
  const uint4* R = reinterpret_cast<const uint4*>(r);
  uint4* O = reinterpret_cast<uint4*>(out);
  ApplyOp<RES, RELU> op;
  if ((stride % C8) == 0) {
    op.load(sc, sh, sc2, sh2, (e0 % C8) * 8);
    int e = e0;
    // SDX_EW_UNROLL grid-stride iterations per trip: all their loads are issued before
    // the first store, so each lane keeps U (x2 with a residual) 16-B loads in flight
    for (; e + (SDX_EW_UNROLL - 1) * stride < n8; e += SDX_EW_UNROLL * stride) {
      uint4 yv[SDX_EW_UNROLL], rv[SDX_EW_UNROLL];
#pragma unroll
      for (int u = 0; u < SDX_EW_UNROLL; ++u) {
        yv[u] = ld16s<SDX_NT_EW_LOAD != 0>(Y + e + u * stride);
        rv[u] = RES != 0 ? ld16s<SDX_NT_EW_LOAD != 0>(R + e + u * stride) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < SDX_EW_UNROLL; ++u) {
        const uint4 o = op.run(yv[u], rv[u]);
        st16<SDX_NT_EW != 0>(O + e + u * stride, o);
        if (mask_out) mask_out[e + u * stride] = relu_bits(o);
      }
    }
    for (; e < n8; e += stride) {
      const uint4 o = op.run(ld16s<SDX_NT_EW_LOAD != 0>(Y + e),
                             RES != 0 ? ld16s<SDX_NT_EW_LOAD != 0>(R + e) : make_uint4(0, 0, 0, 0));
      st16<SDX_NT_EW != 0>(O + e, o);
      if (mask_out) mask_out[e] = relu_bits(o);
    }
  } else {
    for (int e = e0; e < n8; e += stride) {
      op.load(sc, sh, sc2, sh2, (e % C8) * 8);
      const uint4 o = op.run(Y[e], RES != 0 ? R[e] : make_uint4(0, 0, 0, 0));
      O[e] = o;
      if (mask_out) mask_out[e] = relu_bits(o);
    }
  }
}

// Σdz, Σdz·(ya−μa) [, Σdz·(yb−μb)] with dz = dout·[out>0] (or dout when out == nullptr).
// Threads keep a fixed 8-channel group (grid stride is a multiple of C/8).
template <bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dout,
                                                            const uint16_t* __restrict__ outv,
                                                            const uint16_t* __restrict__ ya, const float* __restrict__ ma,
                                                            const uint16_t* __restrict__ yb, const float* __restrict__ mb,
                                                            long n8, int C8, int C, float* __restrict__ partial,
                                                            const float* __restrict__ msc,
                                                            const float* __restrict__ msh,
                                                            const uint8_t* __restrict__ omask) {
  constexpr int NS = TWO ? 3 : 2;
  __shared__ float red[NS][256][8];
  const long tid = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int grp = (int)(tid % C8);
  const int c0 = grp * 8;
  float mua[8], mub[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mua[i] = ma[c0 + i];
    mub[i] = TWO ? mb[c0 + i] : 0.f;
  }
  // ReLU mask recomputed from the BN input when the activation itself was never stored
  // (its consumer applied BN+ReLU in its load prologue): out > 0  <=>  ya·msc + msh > 0
  const bool mask_y = outv == nullptr && omask == nullptr && msc != nullptr;
  float mks[8], mkt[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mks[i] = mask_y ? msc[c0 + i] : 0.f;
    mkt[i] = mask_y ? msh[c0 + i] : 0.f;
  }
  float s0[8] = {0}, s1[8] = {0}, s2[8] = {0};
  const uint4* D = reinterpret_cast<const uint4*>(dout);
  const uint4* OV = reinterpret_cast<const uint4*>(outv);
  const uint4* YA = reinterpret_cast<const uint4*>(ya);
  const uint4* YB = reinterpret_cast<const uint4*>(yb);
  auto accum = [&](uint4 dv, uint4 ov, uint4 av, uint4 bv, uint32_t mbits) {
    float d[8], a[8];
    unpack8(dv, d);
    unpack8(av, a);
    if (omask) {
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = (mbits >> i) & 1u ? d[i] : 0.f;
    } else if (outv) {
      float o[8];
      unpack8(ov, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = o[i] > 0.f ? d[i] : 0.f;
    } else if (mask_y) {
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = a[i] * mks[i] + mkt[i] > 0.f ? d[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s0[i] += d[i];
      s1[i] += d[i] * (a[i] - mua[i]);
    }
    if (TWO) {
      float b[8];
      unpack8(bv, b);
#pragma unroll
      for (int i = 0; i < 8; ++i) s2[i] += d[i] * (b[i] - mub[i]);
    }
  };
  const uint4 z = make_uint4(0, 0, 0, 0);
  // (a 2-chunk unrolled trip measured slower on the 256-channel layer-1 tensors)
  for (long e = tid; e < n8; e += stride)
    accum(D[e], outv ? OV[e] : z, YA[e], TWO ? YB[e] : z, omask ? (uint32_t)omask[e] : 0u);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[0][threadIdx.x][i] = s0[i];
    red[1][threadIdx.x][i] = s1[i];
    if (TWO) red[NS - 1][threadIdx.x][i] = s2[i];
  }
  __syncthreads();
  // threads t and t + k*C8 (k>=1) within the block share the channel group
  if ((int)threadIdx.x < C8 && C8 <= 256) {
    double acc[NS][8];
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[q][i] = 0.0;
    for (int t = threadIdx.x; t < 256; t += C8)
#pragma unroll
      for (int q = 0; q < NS; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[q][i] += red[q][t][i];
    const int g0 = (int)threadIdx.x * 8;
#pragma unroll
    for (int q = 0; q < NS; ++q)
#pragma unroll
      for (int i = 0; i < 8; ++i) partial[((size_t)blockIdx.x * NS + q) * C + g0 + i] = (float)acc[q][i];
  }
}

__global__ void bn_bwd_coef_kernel(const double* __restrict__ sums, int nsets, int C, BnCoefArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double t[3];
  for (int q = 0; q <= nsets; ++q) t[q] = sums[(size_t)q * C + c];
  bn_coef_one(c, C, t, nsets, a);
}

template <bool TWO>
struct BwdApplyOp {
  float A[8], Dc[8], E[8], B2[8], D2[8], E2[8], ms[8], mt[8];
  bool use_mask;
  __device__ __forceinline__ void load(const float* ca, const float* cb, const float* msc, const float* msh, int C,
                                       int c0) {
    load8c(ca + c0, A);
    load8c(ca + C + c0, Dc);
    load8c(ca + 2 * C + c0, E);
    if (TWO) {
      load8c(cb + c0, B2);
      load8c(cb + C + c0, D2);
      load8c(cb + 2 * C + c0, E2);
    }
    use_mask = msc != nullptr;   // (an explicit bitmask takes precedence, see run())
    if (use_mask) {
      load8c(msc + c0, ms);
      load8c(msh + c0, mt);
    }
  }
  // returns dz (masked dout) in d, writes dya / dyb values
  __device__ __forceinline__ void run(uint4 dv, uint4 ov, bool has_out, uint4 av, uint4 bv, float (&d)[8],
                                      uint4& ra, uint4& rb, const uint8_t* omask, int e) const {
    float a[8], r[8];
    unpack8(dv, d);
    unpack8(av, a);
    if (omask) {
      const uint32_t mb = omask[e];
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = (mb >> i) & 1u ? d[i] : 0.f;
    } else if (has_out) {
      float o[8];
      unpack8(ov, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = o[i] > 0.f ? d[i] : 0.f;
    } else if (use_mask) {
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = a[i] * ms[i] + mt[i] > 0.f ? d[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = A[i] * d[i] + Dc[i] * a[i] + E[i];
    ra = pack8(r);
    if (TWO) {
      unpack8(bv, a);
#pragma unroll
      for (int i = 0; i < 8; ++i) r[i] = B2[i] * d[i] + D2[i] * a[i] + E2[i];
      rb = pack8(r);
    }
  }
};

template <bool TWO>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const uint16_t* __restrict__ dout,
                                                           const uint16_t* __restrict__ outv,
                                                           const uint16_t* __restrict__ ya, const float* __restrict__ ca,
                                                           const uint16_t* __restrict__ yb, const float* __restrict__ cb,
                                                           uint16_t* __restrict__ dya, uint16_t* __restrict__ dyb,
                                                           uint16_t* __restrict__ dz_out, long n8l, int C8, int C,
                                                           const float* __restrict__ msc,
                                                           const float* __restrict__ msh,
                                                           const uint8_t* __restrict__ omask) {
  const int n8 = (int)n8l, stride = gridDim.x * blockDim.x;
  const int e0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4* D = reinterpret_cast<const uint4*>(dout);
  const uint4* OV = reinterpret_cast<const uint4*>(outv);
  const uint4* YA = reinterpret_cast<const uint4*>(ya);
  const uint4* YB = reinterpret_cast<const uint4*>(yb);
  uint4* DA = reinterpret_cast<uint4*>(dya);
  uint4* DB = reinterpret_cast<uint4*>(dyb);
  uint4* DZ = reinterpret_cast<uint4*>(dz_out);
  const bool has_out = outv != nullptr;
  const uint4 z = make_uint4(0, 0, 0, 0);
  BwdApplyOp<TWO> op;
  auto one = [&](int e, uint4 dv, uint4 ov, uint4 av, uint4 bv) {
    float d[8];
    uint4 ra, rb;
    op.run(dv, ov, has_out, av, bv, d, ra, rb, omask, e);
    if (DZ) st16<SDX_NT_EW != 0>(DZ + e, pack8(d));
    st16<SDX_NT_EW != 0>(DA + e, ra);
    if (TWO) st16<SDX_NT_EW != 0>(DB + e, rb);
  };
  if ((stride % C8) == 0) {
    op.load(ca, cb, msc, msh, C, (e0 % C8) * 8);
    int e = e0;
    for (; e + (SDX_EW_UNROLL - 1) * stride < n8; e += SDX_EW_UNROLL * stride) {
      uint4 dv[SDX_EW_UNROLL], ov[SDX_EW_UNROLL], av[SDX_EW_UNROLL], bv[SDX_EW_UNROLL];
#pragma unroll
      for (int u = 0; u < SDX_EW_UNROLL; ++u) {
        const int eu = e + u * stride;
        dv[u] = ld16s<SDX_NT_EW_LOAD != 0>(D + eu);
        ov[u] = has_out ? ld16s<SDX_NT_EW_LOAD != 0>(OV + eu) : z;
        av[u] = ld16s<SDX_NT_EW_LOAD != 0>(YA + eu);
        bv[u] = TWO ? ld16s<SDX_NT_EW_LOAD != 0>(YB + eu) : z;
      }
#pragma unroll
      for (int u = 0; u < SDX_EW_UNROLL; ++u) one(e + u * stride, dv[u], ov[u], av[u], bv[u]);
    }
    for (; e < n8; e += stride)
      one(e, ld16s<SDX_NT_EW_LOAD != 0>(D + e), has_out ? ld16s<SDX_NT_EW_LOAD != 0>(OV + e) : z,
          ld16s<SDX_NT_EW_LOAD != 0>(YA + e), TWO ? ld16s<SDX_NT_EW_LOAD != 0>(YB + e) : z);
  } else {
    for (int e = e0; e < n8; e += stride) {
      op.load(ca, cb, msc, msh, C, (e % C8) * 8);
      one(e, D[e], has_out ? OV[e] : z, YA[e], TWO ? YB[e] : z);
    }
  }
}

int ew_grid(long n8, bool bwd = false) {
  // enough lanes for SDX_EW_UNROLL elements each, at most 2048 blocks (one per-CU residency
  // of 8 blocks; in-step 11.97 vs 12.04 ms/step at 4096, profiles/knob_revalidate_r5.txt).
  // SDX_EW_BLOCKS overrides the cap, SDX_EW_BLOCKS_BWD that of bn_bwd_apply alone; rounded
  // to a multiple of 8 blocks (A/B knobs)
  auto env_cap = [](const char* name, long dflt) {
    const char* e = getenv(name);
    const long v = e ? atol(e) : 0;
    return v >= 8 ? v / 8 * 8 : dflt;
  };
  static const long cap_fwd = env_cap("SDX_EW_BLOCKS", 2048L);
  static const long cap_bwd = env_cap("SDX_EW_BLOCKS_BWD", cap_fwd);
  const long cap = bwd ? cap_bwd : cap_fwd;
  long g = (n8 + 256L * SDX_EW_UNROLL - 1) / (256L * SDX_EW_UNROLL);
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

int col_reduce_gy(int rows) {
  // balance the per-block row loop (rows/gy/4 trips) against the final combine (gy/4 loads);
  // SDX_CR_GY scales the sqrt(rows) rule (A/B knob)
  static const double scale = [] {
    const char* e = getenv("SDX_CR_GY");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 0.5;
  }();
  int gy = (int)(sqrt((double)rows) * scale + 0.5);
  if (gy > 64) gy = 64;
  if (gy < 1) gy = 1;
  return gy;
}

hipError_t launch_col_reduce(const float* slab, int rows, int nsets, int C, double* scratch, unsigned* counters,
                             double* sums, int epi, const BnFinalizeArgs* fa, const BnCoefArgs* ca, hipStream_t s,
                             const XgmiCol* xg) {
  if (rows < 1 || C < 1 || (epi == 1 && (nsets != 2 || !fa)) || (epi == 2 && (nsets < 2 || !ca)) ||
      (epi == 3 && (nsets > 2 || !ca || !ca->dbeta_a)) || (nsets == 1 && epi != 0 && epi != 3))
    return hipErrorInvalidValue;
  const int xm = xg ? xg->mode : 0;
  if (xg && (xm < 1 || xm > 2 || xg->world < 1 || xg->world > kXgmiMaxPeers || xg->me < 0 || xg->me >= xg->world ||
             (size_t)nsets * C > xg->peers.cap || (C + 63) / 64 > kXgmiFlagGroups || xg->timeout_ticks <= 0))
    return hipErrorInvalidValue;
  if (xg && xm == 2 && xg->slab_zstride < 0) return hipErrorInvalidValue;
  // emulation: the spinning last blocks (one per group and virtual rank) must stay co-resident
  if (xg && xm == 2 && !xg->solo && ((C + 63) / 64) * xg->world > 512) return hipErrorInvalidValue;
  if (xg && xg->solo && (xm != 2 || xg->me != 0)) return hipErrorInvalidValue;
  const dim3 grid((C + 63) / 64, col_reduce_gy(rows), xm == 2 && !xg->solo ? xg->world : 1), blk(256);
  const BnFinalizeArgs f = fa ? *fa : BnFinalizeArgs{};
  const BnCoefArgs k = ca ? *ca : BnCoefArgs{};
  const XgmiCol x = xg ? *xg : XgmiCol{};
#define SDX_CR(NS, EPI)                                                                                              \
  do {                                                                                                               \
    if (xm == 0)                                                                                                     \
      hipLaunchKernelGGL((col_reduce_kernel<NS, EPI, 0>), grid, blk, 0, s, slab, rows, C, scratch, counters, sums, f, \
                         k, x);                                                                                      \
    else if (xm == 1)                                                                                                \
      hipLaunchKernelGGL((col_reduce_kernel<NS, EPI, 1>), grid, blk, 0, s, slab, rows, C, scratch, counters, sums, f, \
                         k, x);                                                                                      \
    else                                                                                                             \
      hipLaunchKernelGGL((col_reduce_kernel<NS, EPI, 2>), grid, blk, 0, s, slab, rows, C, scratch, counters, sums, f, \
                         k, x);                                                                                      \
  } while (0)
  if (nsets == 1) {
    if (epi == 0) SDX_CR(1, 0); else SDX_CR(1, 3);
  } else if (nsets == 2) {
    if (epi == 0) SDX_CR(2, 0); else if (epi == 1) SDX_CR(2, 1); else if (epi == 2) SDX_CR(2, 2); else SDX_CR(2, 3);
  } else if (nsets == 3) {
    if (epi == 0) SDX_CR(3, 0); else SDX_CR(3, 2);
  } else {
    return hipErrorInvalidValue;
  }
#undef SDX_CR
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bn_finalize(const double* sums, int C, const BnFinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, sums, C, a);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bn_eval_affine(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                 float eps, float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, rm, rv, eps,
                     scale, shift);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bn_apply(const void* y, const float* sc, const float* sh, const void* r, const float* sc2,
                           const float* sh2, int res_mode, int relu, void* out, long numel, int C, hipStream_t s,
                           void* mask_out) {
  const long n8 = numel / 8;
  const int C8 = C / 8;
  const dim3 grid(ew_grid(n8)), blk(256);
  const uint16_t* yy = (const uint16_t*)y;
  const uint16_t* rr = (const uint16_t*)r;
  uint16_t* oo = (uint16_t*)out;
#define SDX_APPLY(RM, RL) \
  hipLaunchKernelGGL((bn_apply_kernel<RM, RL>), grid, blk, 0, s, yy, sc, sh, rr, sc2, sh2, oo, n8, C8, (uint8_t*)mask_out)
  if (res_mode == 0) { if (relu) SDX_APPLY(0, true); else SDX_APPLY(0, false); }
  else if (res_mode == 1) { if (relu) SDX_APPLY(1, true); else SDX_APPLY(1, false); }
  else { if (relu) SDX_APPLY(2, true); else SDX_APPLY(2, false); }
#undef SDX_APPLY
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

int bn_bwd_reduce_blocks(long numel, int C) {
  const long n8 = numel / 8;
  long g = (n8 + 256 * 16 - 1) / (256 * 16);   // ~16 chunks per thread
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  (void)C;
  return (int)g;
}

hipError_t launch_bn_bwd_reduce(const void* dout, const void* outv, const void* ya, const float* ma, const void* yb,
                                const float* mb, long numel, int C, float* partial, double* scratch,
                                unsigned* counters, double* sums, int epi, const BnCoefArgs* ca, hipStream_t s,
                                const float* msc, const float* msh, const void* omask, const XgmiCol* xg) {
  const int nsets = yb ? 3 : 2;
  const long n8 = numel / 8;
  const int C8 = C / 8;
  // grid stride must be a multiple of C8 (fixed channel group per thread): 256 % C8 == 0
  const int g = bn_bwd_reduce_blocks(numel, C);
  if (yb)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<true>), dim3(g), dim3(256), 0, s, (const uint16_t*)dout,
                       (const uint16_t*)outv, (const uint16_t*)ya, ma, (const uint16_t*)yb, mb, n8, C8, C, partial,
                       msc, msh, (const uint8_t*)omask);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<false>), dim3(g), dim3(256), 0, s, (const uint16_t*)dout,
                       (const uint16_t*)outv, (const uint16_t*)ya, ma, (const uint16_t*)nullptr, (const float*)nullptr,
                       n8, C8, C, partial, msc, msh, (const uint8_t*)omask);
  SDX_LAUNCH_CHECK();
  // emulated ranks (xg mode 2) all reduce the same partial slab (identical ranks)
  if (xg && xg->mode == 2 && xg->slab_zstride != 0) return hipErrorInvalidValue;
  return launch_col_reduce(partial, g, nsets, C, scratch, counters, sums, epi, nullptr, ca, s, xg);
}

hipError_t launch_bn_bwd_coef(const double* sums, int nsets, int C, const BnCoefArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, s, sums, nsets, C, a);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_bn_bwd_apply(const void* dout, const void* outv, const void* ya, const float* ca, const void* yb,
                               const float* cb, void* dya, void* dyb, void* dz_out, long numel, int C, hipStream_t s,
                               const float* msc, const float* msh, const void* omask) {
  const long n8 = numel / 8;
  const int C8 = C / 8;
  if (yb)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<true>), dim3(ew_grid(n8, true)), dim3(256), 0, s, (const uint16_t*)dout,
                       (const uint16_t*)outv, (const uint16_t*)ya, ca, (const uint16_t*)yb, cb, (uint16_t*)dya,
                       (uint16_t*)dyb, (uint16_t*)dz_out, n8, C8, C, msc, msh, (const uint8_t*)omask);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<false>), dim3(ew_grid(n8, true)), dim3(256), 0, s, (const uint16_t*)dout,
                       (const uint16_t*)outv, (const uint16_t*)ya, ca, (const uint16_t*)nullptr, (const float*)nullptr,
                       (uint16_t*)dya, (uint16_t*)nullptr, (uint16_t*)dz_out, n8, C8, C, msc, msh,
                       (const uint8_t*)omask);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}
