// Common device helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
// Everything here is written for wave64 and the CDNA4 MFMA register maps; there is
// no portability layer and no CUDA-compatible path.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <type_traits>

// Device-side checks, compiled in only for the checked build (csrc/build.py --checked):
// a violated condition prints its location and traps the wave.
#ifdef SDX_CHECKED
#define SDX_DCHECK(cond)                                                                    \
  do {                                                                                      \
    if (!(cond)) {                                                                          \
      printf("SDX_DCHECK failed %s:%d: %s (block %d thread %d)\n", __FILE__, __LINE__, #cond, \
             (int)blockIdx.x, (int)threadIdx.x);                                            \
      __builtin_trap();                                                                     \
    }                                                                                       \
  } while (0)
#else
#define SDX_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

namespace sdx {

constexpr int kWave = 64;   // CDNA wavefront width (never 32)
constexpr int kNumXcd = 8;  // MI355X: 8 XCDs x 32 CUs

typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (4 VGPR)
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;    // 16x16 accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16;  // 32x32 accumulator
typedef __attribute__((ext_vector_type(2))) float f32x2;

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even float -> bf16 via the hardware conversion (keeps NaN a NaN).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// two fp32 -> packed bf16x2 (RNE) in ONE v_cvt_pk_bf16_f32 (two scalar conversions cost
// 2 cvt + and + shift + or)
typedef __bf16 sdx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float sdx_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  const sdx_f32x2 v = {lo, hi};
  const sdx_bf16x2 r = __builtin_convertvector(v, sdx_bf16x2);
  return __builtin_bit_cast(uint32_t, r);
}

// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E) — for bodies that
// index register arrays, which a runtime (not fully unrolled) loop would place in scratch
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// 8 packed bf16 (16 B) <-> 8 floats
__device__ __forceinline__ void unpack8(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

// Sum over the 16 lanes of each DPP row (lanes 16r..16r+15), result in every lane of the
// row: 4 DPP-modified adds (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror),
// no LDS traffic (a __shfl_xor lowers to ds_bpermute).
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, true));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md T1): consecutive logical
// tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < kNumXcd) return bid;
  const int q = nwg / kNumXcd, r = nwg % kNumXcd;
  const int xcd = bid % kNumXcd, idx = bid / kNumXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Division by a runtime-invariant divisor via multiply-high (Granlund-Montgomery);
// exact for 0 <= x < 2^31.
struct FastDiv {
  uint32_t d, mul, shr;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{d, 0u, 0u};
  if (d > 1) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    f.shr = l;
  }
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t x, const FastDiv& f) {
  return (__umulhi(x, f.mul) + x) >> f.shr;
}

}  // namespace sdx

#ifndef SDX_NT_EW
#define SDX_NT_EW 0   // 1: non-temporal 16-B stores in the elementwise BN kernels (A/B experiment)
#endif
#ifndef SDX_NT_EW_LOAD
// non-temporal loads of the elementwise BN kernels' read-once inputs: step 12.90 -> 12.77 ms
// on the same box (profiles/nt_store_r2.txt); 0 = cached loads
#define SDX_NT_EW_LOAD 1
#endif
#ifndef SDX_NT_PART
#define SDX_NT_PART 0      // 1: non-temporal split-K partial slab stores + reduction loads (A/B)
#endif
// 16-B load of a read-once input (non-temporal when enabled)
template <bool NT>
__device__ __forceinline__ uint4 ld16s(const void* p) {
  if constexpr (NT) {
    typedef unsigned int nt_u32x4 __attribute__((ext_vector_type(4)));
    const nt_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x4*>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}
// 16-B store of a streamed output that no kernel re-reads soon (non-temporal when enabled)
template <bool NT>
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr (NT) {
    typedef unsigned int nt_u32x4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(nt_u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<nt_u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

#define SDX_LAUNCH_CHECK() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return e__; } while (0)
