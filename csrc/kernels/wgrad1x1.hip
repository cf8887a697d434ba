// Stride-1 1x1 weight gradient on gfx950 MFMA, NHWC bf16 -> fp32:
//
//   dW[k][c] = Σ_pixels dy[p][k] · x[p][c]
//
// A plain GEMM whose reduction runs over pixels, so both operands are K-outer (the pixel is
// the slow dimension of dy and x). The generic implicit-GEMM wgrad (igemm.hip MODE_WGRAD,
// 4 waves, one K-tile of register prefetch) runs these at ~450 TFLOP/s with ~4 VALU per
// MFMA; this kernel is the tap-reuse 3x3 kernel's (wgrad3x3.hip) schedule applied to the
// 1x1 case: 8 waves (2 x 4) over a 128 x BN output tile, 32-pixel steps, operand loads
// FOUR steps ahead through a branch-free register ring (base + step·stride addressing, tail
// steps read the zero page), step-invariant fragment offsets, and one wave of ~256 blocks.
//
// LDS images are [32 pixels][COLS] bf16 with igemm.hip's K-outer chunk swizzle for
// COLS >= 128 (row & 3, bit 3 of the row), read with ds_read_b64_tr_b16. The MFMA is issued
// as D = Bᵀ·Aᵀ (each lane holds 4 consecutive output columns of one output row). Output: an
// fp32 partial slab per K-split, reduced deterministically by igemm.hip's split-K reduction.
//
// Shapes: K % 128 == 0, C % BN == 0 (BN = 256, or 128 when C is not a multiple of 256),
// N·P·Q % 32 == 0 — layers 2-4 of the CIFAR/ImageNet ResNet bottlenecks (reference
// networks/resnet_big.py:44-49, conv1/conv3 of each Bottleneck), and the strided projection
// shortcuts (:50-55) on the pipelined kernel (an x chunk reads its pixel at base + step·const
// when a step is whole output rows, else from g / Q per step). The layer-1 1x1 wgrads (64
// channels on one side, HBM-bound) run on the same kernel over a pixel-pair view (w1_pairs).
#include <atomic>
#include <type_traits>

#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

// SDX_W1_ORDER=1 (build define): issue a step's LDS traffic and refill loads before its
// MFMAs in wgrad1x1_pipe_kernel. Measured 2-3 % slower per kernel than the compiler's order
// (47.3 -> 48.5 us, profiles/wgrad_order_r4.txt), so off; the 3x3 kernels gain (SDX_W3_ORDER)
#ifndef SDX_W1_ORDER
#define SDX_W1_ORDER 0
#endif

constexpr int W1_NT = 512;      // 8 waves: 2 (output rows) x 4 (output columns)
constexpr int W1_BM = 128;      // output channels (dW rows) per block
constexpr int W1_PF = 4;        // steps of loads in flight (register ring of 4 named slots)

typedef __attribute__((address_space(3))) bf16x4 w1_lds_bf16x4;

__device__ __attribute__((aligned(16))) uint16_t w1_zero16[8];
typedef const __attribute__((address_space(1))) uint16_t* w1_gptr;

// K-outer image [rows][COLS] bf16: 16-B chunk ch of row r (igemm.hip kout_off, COLS >= 128);
// the chunk XOR depends on row bits 0, 1 and 3 only
template <int COLS>
__device__ __forceinline__ int kout_swz_w1(int r) {
  static_assert(COLS >= 128, "swizzle spans 16 chunks");
  return ((r & 3) | (((r >> 3) & 1) << 2)) << 1;
}
template <int COLS>
__device__ __forceinline__ int w1_off(int r, int ch) {
  return r * (COLS * 2) + ((ch ^ kout_swz_w1<COLS>(r)) << 4);
}

struct W1Params {
  const uint16_t* dy;   // [P][K]
  const uint16_t* x;    // [P][C]
  float* part;          // [splits][K][C]
  int K, C;
  int steps_total;      // dy pixels / 32
  // x pixel of dy pixel j of a step (pipelined kernel): stride 1: j; stride st (H = st·P,
  // W = st·Q, Q | 32): st·(W·(j / Q) + j % Q). x step stride in elements (32·C at stride 1;
  // 0 for the GEN kernels)
  int xst, xq, xw;
  int x_step;
  // GEN kernels (a step is not whole output rows, 32 % Q != 0): the x pixel of step pixel
  // g = 32·step + j is xst·(xw·(g / Q) + g % Q), with g / Q = umulhi(g, xmagic) (exact for
  // g·Q < 2^32, host check)
  unsigned xmagic;
  int steps_per_split;
  int k_tiles, c_tiles, splits;
  // pixel pairs (a 64-channel side, stride 1): K, C above are the doubled widths of the
  // [pixels / 2][2·K0] / [pixels / 2][2·C0] views; only the diagonal blocks (even pixel x even
  // pixel, odd x odd) are stored, into slices 2·split and 2·split + 1 of a [2·splits][K0][C0] slab
  int pairs, K0, C0;
};

template <int BN>
__global__ __launch_bounds__(W1_NT, 1) void wgrad1x1_kernel(W1Params p) {
  constexpr int A_BYTES = 32 * W1_BM * 2;
  constexpr int STAGE = A_BYTES + 32 * BN * 2;
  constexpr int A_CPR = W1_BM / 8, B_CPR = BN / 8;        // 16-B chunks per image row
  constexpr int NCH = 32 * (A_CPR + B_CPR) / W1_NT;       // chunks per thread per step
  static_assert(NCH == 2 || NCH == 3, "loader layout");
  constexpr int WN_COLS = BN / 4, TN = WN_COLS / 16;      // wave tile: 64 rows x BN/4 columns
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;

  // ---- tile / split (split-major: an XCD's co-resident blocks share one pixel range) ----
  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * W1_BM, c0 = (tile % p.c_tiles) * BN;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  // ---- loader: chunk f = tid + u·512 (u < NCH); f < 512: dy chunk (pixel f/16, channel
  // chunk f%16 of the 128 rows), else x chunk e = f − 512 (pixel e/B_CPR, chunk e%B_CPR) ----
  struct Chunk {
    const uint16_t* base;   // element of step 0
    long stride;            // elements per step
    int dst;                // LDS byte offset within a stage
  };
  auto chunk = [&](int u) -> Chunk {
    const int f = tid + u * W1_NT;
    if (f < 32 * A_CPR) {
      const int px = f / A_CPR, ch = f % A_CPR;
      return {p.dy + (long)px * p.K + k0 + ch * 8, 32L * p.K, w1_off<W1_BM>(px, ch)};
    }
    const int e = f - 32 * A_CPR, px = e / B_CPR, ch = e % B_CPR;
    return {p.x + (long)px * p.C + c0 + ch * 8, 32L * p.C, A_BYTES + w1_off<BN>(px, ch)};
  };
  const Chunk ck0 = chunk(0), ck1 = chunk(1), ck2 = chunk(NCH == 3 ? 2 : 1);
  // register ring: slot s holds the step ≡ s_begin + s (mod 4); every value is a named
  // register selected at compile time (arrays indexed inside the lambdas go to scratch)
  struct Regs {
    uint4 a, b, c;
  };
  Regs r0, r1, r2, r3;
  auto slot = [&](auto S) -> Regs& {
    if constexpr (decltype(S)::value == 0) return r0;
    else if constexpr (decltype(S)::value == 1) return r1;
    else if constexpr (decltype(S)::value == 2) return r2;
    else return r3;
  };
  auto ld = [&](const Chunk& ck, int step, bool ok) -> uint4 {
    return *reinterpret_cast<const uint4*>(ok ? ck.base + (long)step * ck.stride : w1_zero16);
  };
  auto load = [&](int step, Regs& r) {
    const bool ok = step < s_end;
    r.a = ld(ck0, step, ok);
    r.b = ld(ck1, step, ok);
    if constexpr (NCH == 3) r.c = ld(ck2, step, ok);
  };
  auto store = [&](int buf, const Regs& r) {
    unsigned char* sb = smem + buf * STAGE;
    *reinterpret_cast<uint4*>(sb + ck0.dst) = r.a;
    *reinterpret_cast<uint4*>(sb + ck1.dst) = r.b;
    if constexpr (NCH == 3) *reinterpret_cast<uint4*>(sb + ck2.dst) = r.c;
  };

  // ---- fragment offsets (step-invariant): lane (h4, c16 = 4q + pp) reads pixel rows
  // 8h4+q and +4, columns col0 + 4pp .. +3 ----
  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q, p_hi = p_lo + 4;
  auto kout = [&](auto cols_tag, int row, int col0) {
    constexpr int COLS = decltype(cols_tag)::value;
    const int col = col0 + 4 * pp;
    return w1_off<COLS>(row, col >> 3) + (col & 7) * 2;
  };
  int ao_lo[4], ao_hi[4], bo_lo[TN], bo_hi[TN];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ao_lo[i] = kout(std::integral_constant<int, W1_BM>{}, p_lo, wm * 64 + 16 * i);
    ao_hi[i] = kout(std::integral_constant<int, W1_BM>{}, p_hi, wm * 64 + 16 * i);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    bo_lo[j] = A_BYTES + kout(std::integral_constant<int, BN>{}, p_lo, wn * WN_COLS + 16 * j);
    bo_hi[j] = A_BYTES + kout(std::integral_constant<int, BN>{}, p_hi, wn * WN_COLS + 16 * j);
  }
  auto frag = [&](const unsigned char* b, int o_lo, int o_hi) -> bf16x8 {
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o_lo));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o_hi));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const unsigned char* b = smem + buf * STAGE;
    bf16x8 af[4], bfr[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag(b, bo_lo[j], bo_hi[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(b, ao_lo[i], ao_hi[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

  // ---- K loop (as wgrad3x3.hip): compute step k from LDS buffer k&1, move step k+1 from
  // its ring slot into the other buffer, refill the slot with step k+1+4, one barrier ----
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  auto iter = [&](int b0, auto U) {
    constexpr int u = decltype(U)::value;
    using N = std::integral_constant<int, (u + 1) % W1_PF>;
    compute(u & 1);
    store((u + 1) & 1, slot(N{}));
    load(b0 + u + 1 + W1_PF, slot(N{}));
    __syncthreads();
  };
  load(s_begin, r0);
  load(s_begin + 1, r1);
  load(s_begin + 2, r2);
  load(s_begin + 3, r3);
  store(0, r0);
  load(s_begin + W1_PF, r0);
  __syncthreads();
  for (int b0 = s_begin; b0 < s_end; b0 += W1_PF) {
    iter(b0, I0{});
    iter(b0, I1{});
    iter(b0, I2{});
    iter(b0, I3{});
  }

  // ---- epilogue: fp32 partial rows, 4 consecutive columns per lane ----
  if (p.pairs) {
    // the diagonal blocks only: row m of dy half e = m / K0, column n of x half n / C0 (4
    // consecutive columns never straddle C0, a multiple of 64)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = k0 + wm * 64 + 16 * i + c16;
      const int e = m >= p.K0;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = c0 + wn * WN_COLS + 16 * j + 4 * h4;
        if ((n >= p.C0) != e) continue;
        const f32x4 a = acc[i][j];
        float* o = p.part + ((size_t)(2 * split + e) * p.K0 + (m - e * p.K0)) * p.C0 + (n - e * p.C0);
        st16<SDX_NT_PART != 0>(o, make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                             __float_as_uint(a[3])));
      }
    }
    return;
  }
  float* out = p.part + (size_t)split * p.K * p.C;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = k0 + wm * 64 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = c0 + wn * WN_COLS + 16 * j + 4 * h4;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * p.C + n,
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}

// ---------------------------------------------------------------------------------------
// Fragment-pipelined variant (default; SDX_W1_PIPE=0 restores the loop above). Above, every
// step waits after its barrier for its own fragment reads (LDS latency under load) before
// the first MFMA, and both waves of a SIMD leave the barrier together, so that latency and
// the step's ds_write transfers are exposed once per 32 pixels (~32 % MFMA-busy on the
// layer-3 shapes). Here the LDS ring has THREE buffers and the fragments are
// double-buffered in registers: iteration k reads step k+1's fragments (stored one
// iteration earlier, visible since the last barrier), runs step k's MFMAs on the fragments
// read during iteration k-1, and stores step k+2 from the register ring into the buffer
// step k-1 vacated — one barrier per step, no LDS latency in front of the MFMAs. (An
// LDS-DMA version of this kernel, 3-stage ring of 64-pixel steps, measured 12-48 % slower
// per kernel: profiles/ablate_wgrad_r3.txt.)
template <int BN, bool GEN>
__global__ __launch_bounds__(W1_NT, 1) void wgrad1x1_pipe_kernel(W1Params p) {
  constexpr int A_BYTES = 32 * W1_BM * 2;
  constexpr int STAGE = A_BYTES + 32 * BN * 2;
  constexpr int A_CPR = W1_BM / 8, B_CPR = BN / 8;
  constexpr int NCH = 32 * (A_CPR + B_CPR) / W1_NT;
  static_assert(NCH == 2 || NCH == 3, "loader layout");
  constexpr int WN_COLS = BN / 4, TN = WN_COLS / 16;
  __shared__ __attribute__((aligned(16))) unsigned char smem[3 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;

  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * W1_BM, c0 = (tile % p.c_tiles) * BN;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  // loader: chunk u of this thread (u < NCH) is a dy chunk (pixel f/16 of the 32-pixel
  // step, channel chunk f%16 of the 128 rows) for f = tid + 512u < 512, else an x chunk;
  // chunk 0 is always dy, chunks 1 and 2 always x. Sources are 32-bit element offsets plus a
  // uniform (scalar) step offset (host check: P·K, P·C < 2^31); past s_end the zero page,
  // whose address lives in an SGPR pair the compiler cannot rematerialise (else it re-runs
  // s_getpc + a GOT load + lgkmcnt(0) — draining the in-flight fragment reads — per select)
  static_assert(32 * A_CPR == W1_NT, "chunk 0 = dy, chunks 1.. = x");
  const int a_off = (tid / A_CPR) * p.K + k0 + (tid % A_CPR) * 8;
  const int a_dst = w1_off<W1_BM>(tid / A_CPR, tid % A_CPR);
  const int e1 = tid, e2 = tid + W1_NT;   // x chunk indices of chunks 1, 2
  // x pixel of step pixel j (a strided 1x1 reads every st-th pixel of every st-th row)
  auto xpix = [&](int j) { return p.xst * (p.xw * (j / p.xq) + j % p.xq); };
  const int x_off1 = xpix(e1 / B_CPR) * p.C + c0 + (e1 % B_CPR) * 8;
  const int x_off2 = xpix(e2 / B_CPR) * p.C + c0 + (e2 % B_CPR) * 8;
  // GEN: element offset of x chunk e at step `step` (pixel g = 32·step + e / B_CPR)
  auto xgen = [&](int step, int e) __attribute__((always_inline)) {
    const unsigned g = 32u * (unsigned)step + (unsigned)(e / B_CPR);
    const unsigned q = __umulhi(g, p.xmagic);
    return (int)(p.xst * (p.xw * q + (g - q * p.xq))) * p.C + c0 + (e % B_CPR) * 8;
  };
  const int x_dst1 = A_BYTES + w1_off<BN>(e1 / B_CPR, e1 % B_CPR);
  const int x_dst2 = A_BYTES + w1_off<BN>(e2 / B_CPR, e2 % B_CPR);
  const int sA = 32 * p.K, sB = p.x_step;
  w1_gptr zp = (w1_gptr)w1_zero16;
  asm volatile("" : "+s"(zp));
  const w1_gptr gdy = (w1_gptr)p.dy, gx = (w1_gptr)p.x;
  // native vectors (a HIP uint4 read through an address-space-1 pointer becomes a memcpy
  // that keeps the ring in scratch)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  struct Regs {
    u32x4 a, b, c;
  };
  Regs r0, r1, r2, r3;
  auto slot = [&](auto S) __attribute__((always_inline)) -> Regs& {
    if constexpr (decltype(S)::value == 0) return r0;
    else if constexpr (decltype(S)::value == 1) return r1;
    else if constexpr (decltype(S)::value == 2) return r2;
    else return r3;
  };
  typedef const __attribute__((address_space(1))) u32x4* g16;
  auto load = [&](int step, Regs& r) __attribute__((always_inline)) {
    const bool ok = step < s_end;
    r.a = *(g16)(ok ? gdy + (a_off + step * sA) : zp);
    if constexpr (GEN) {
      r.b = *(g16)(ok ? gx + xgen(step, e1) : zp);
      if constexpr (NCH == 3) r.c = *(g16)(ok ? gx + xgen(step, e2) : zp);
    } else {
      r.b = *(g16)(ok ? gx + (x_off1 + step * sB) : zp);
      if constexpr (NCH == 3) r.c = *(g16)(ok ? gx + (x_off2 + step * sB) : zp);
    }
  };
  auto store = [&](unsigned char* sb, const Regs& r) __attribute__((always_inline)) {
    *reinterpret_cast<u32x4*>(sb + a_dst) = r.a;
    *reinterpret_cast<u32x4*>(sb + x_dst1) = r.b;
    if constexpr (NCH == 3) *reinterpret_cast<u32x4*>(sb + x_dst2) = r.c;
  };

  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q;   // fragment pixel rows p_lo and p_lo + 4
  auto kout = [&](auto cols_tag, int row, int col0) __attribute__((always_inline)) {
    constexpr int COLS = decltype(cols_tag)::value;
    const int col = col0 + 4 * pp;
    return w1_off<COLS>(row, col >> 3) + (col & 7) * 2;
  };
  // pixel row p_hi = p_lo + 4 differs from p_lo in row bit 2 only, which the swizzle
  // ignores: its fragment half sits a constant 4 rows further (an immediate ds_read offset)
  int ao[4], bo[TN];
#pragma unroll
  for (int i = 0; i < 4; ++i) ao[i] = kout(std::integral_constant<int, W1_BM>{}, p_lo, wm * 64 + 16 * i);
#pragma unroll
  for (int j = 0; j < TN; ++j) bo[j] = A_BYTES + kout(std::integral_constant<int, BN>{}, p_lo, wn * WN_COLS + 16 * j);
  auto frag = [&](const unsigned char* b, int o, auto cols_tag) __attribute__((always_inline)) -> bf16x8 {
    constexpr int COLS = decltype(cols_tag)::value;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o + 4 * COLS * 2));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment register sets (named, selected at compile time by step parity)
  bf16x8 fa0[4], fb0[TN], fa1[4], fb1[TN];
  auto read_frags = [&](const unsigned char* b, bf16x8 (&fa)[4], bf16x8 (&fb)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = frag(b, bo[j], std::integral_constant<int, BN>{});
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag(b, ao[i], std::integral_constant<int, W1_BM>{});
  };
  auto mfmas = [&](const bf16x8 (&fa)[4], const bf16x8 (&fb)[TN]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };

  // LDS buffers of steps k, k+1, k+2 (rotating)
  unsigned char* b_cur = smem;
  unsigned char* b_nxt = smem + STAGE;
  unsigned char* b_st = smem + 2 * STAGE;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // iteration for step k = base + U: read step k+1's fragments, MFMAs of step k, store step
  // k+2 (ring slot (U+2)%4) into the buffer step k-1 vacated, refill that slot with k+6
  auto iter = [&](int b0, auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    using S = std::integral_constant<int, (u + 2) % 4>;
#if SDX_W1_ORDER
    // every LDS access of the step (next fragments, the store of step k+2) and the refill
    // loads are ISSUED before this step's MFMAs, so they complete under them: left to
    // itself the scheduler put the fragment reads after the MFMAs, and the barrier's
    // lgkmcnt(0) then exposed their whole latency plus the store transfer every step
    if constexpr ((u & 1) == 0) read_frags(b_nxt, fa1, fb1);
    else read_frags(b_nxt, fa0, fb0);
    store(b_st, slot(S{}));
    load(b0 + u + 6, slot(S{}));
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((u & 1) == 0) mfmas(fa0, fb0);
    else mfmas(fa1, fb1);
    __builtin_amdgcn_sched_barrier(0);   // (the MFMAs would otherwise sink past the barrier)
#else
    if constexpr ((u & 1) == 0) {
      read_frags(b_nxt, fa1, fb1);
      mfmas(fa0, fb0);
    } else {
      read_frags(b_nxt, fa0, fb0);
      mfmas(fa1, fb1);
    }
    store(b_st, slot(S{}));
    load(b0 + u + 6, slot(S{}));
#endif
    __syncthreads();
    unsigned char* t = b_cur;
    b_cur = b_nxt;
    b_nxt = b_st;
    b_st = t;
  };
  load(s_begin, r0);
  load(s_begin + 1, r1);
  load(s_begin + 2, r2);
  load(s_begin + 3, r3);
  store(b_cur, r0);
  store(b_nxt, r1);
  load(s_begin + 4, r0);
  load(s_begin + 5, r1);
  __syncthreads();
  read_frags(b_cur, fa0, fb0);
  for (int b0 = s_begin; b0 < s_end; b0 += 4) {
    iter(b0, I0{});
    iter(b0, I1{});
    iter(b0, I2{});
    iter(b0, I3{});
  }

  if (p.pairs) {
    // the diagonal blocks only: row m of dy half e = m / K0, column n of x half n / C0 (4
    // consecutive columns never straddle C0, a multiple of 64)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = k0 + wm * 64 + 16 * i + c16;
      const int e = m >= p.K0;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = c0 + wn * WN_COLS + 16 * j + 4 * h4;
        if ((n >= p.C0) != e) continue;
        const f32x4 a = acc[i][j];
        float* o = p.part + ((size_t)(2 * split + e) * p.K0 + (m - e * p.K0)) * p.C0 + (n - e * p.C0);
        st16<SDX_NT_PART != 0>(o, make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                             __float_as_uint(a[3])));
      }
    }
    return;
  }
  float* out = p.part + (size_t)split * p.K * p.C;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = k0 + wm * 64 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = c0 + wn * WN_COLS + 16 * j + 4 * h4;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * p.C + n,
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256-row LDS-DMA variant (default for K % 256 == 0; SDX_W1_BIG=0 restores the kernels
// above). The kernels above move 24 KB of operands per 32-pixel step for a 128 x 256 output
// tile through a 4-deep register ring, and per CU they stream at ~48 GB/s even with the
// chip to themselves (32 blocks: 1000 cycles per step against 512 of MFMA work,
// profiles/w1_split_r6.txt): one block per CU, ~96 KB in flight, the L2 misses of a step
// (the first tile to touch a pixel range fetches it from HBM) are latency-bound. Here a
// block owns a 256 x BN tile (BN = 256, or 128), so a step's 32 KB feed twice the MFMA
// work (1.5x fewer operand bytes per FLOP), and the operands are staged by LDS-DMA
// (global_load_lds_dwordx4) into a 4-slot ring with THREE steps in flight across every
// barrier (no staging registers: 128 accumulator + 48 fragment VGPRs fit two waves per
// SIMD).
//
// LDS image: the same K-outer chunk swizzle as above (w1_off), so the fragment reads are
// the transposed ds_read_b64_tr_b16 pair of the kernels above. LDS-DMA writes a wave's
// 64 x 16 B linearly, so the swizzle moves to the SOURCE: the lane that lands in chunk
// slot s of row r fetches logical chunk s ^ swz(r) (cdna_hip_programming.md §5, rule 21).
// Per 32-pixel step: A = dy [32][256] (16 KiB, 16 wave-DMAs), B = x [32][BN] (16 or 8).
//
// Loop (step k in slot k % 4): see the pipeline note at the loop; three steps' DMAs are in
// flight under every step's MFMAs.
// No other vector-memory instruction runs in the loop, so the counted vmcnt is exact (a
// compiler spill to scratch would only make it stricter: vmcnt(N) then retires one more of
// the older DMAs, never fewer), and
// the barrier is the raw s_barrier (a __syncthreads() would drain the ring, vmcnt(0)).
// Steps past the split's end DMA the zero page into their (never read) slot, keeping the
// per-iteration DMA count uniform.
constexpr int W1B_BM = 256;
constexpr int W1B_NS = 4;   // LDS slots

// One 16-B LDS-DMA per lane into LDS byte address lds_addr (wave-uniform) + 16·lane, as
// inline asm: hipcc never learns that it writes LDS, so it does not order the builtin
// fragment reads behind it (through __builtin_amdgcn_global_load_lds every ds_read of the
// loop was preceded by an s_waitcnt vmcnt(0) that drained the ring -- it cannot tell that
// the DMA targets another slot). The reads stay builtins, so hipcc's own lgkmcnt waits
// guard their uses; the DMAs are ordered for the reads only by the counted vmcnt + barrier
// of the loop. (Reads in asm instead are unsafe: hipcc may touch an asm output register --
// a v_bfi re-packing the two halves of a fragment -- while its LDS load is still in flight.)
__device__ __forceinline__ void w1_glds16(w1_gptr src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void w1_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void w1_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BN>
__global__ __launch_bounds__(W1_NT, 1) void wgrad1x1_big_kernel(W1Params p) {
  constexpr int A_BYTES = 32 * W1B_BM * 2;             // 16 KiB
  constexpr int B_BYTES = 32 * BN * 2;                 // 16 / 8 KiB
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ND_A = A_BYTES / 1024 / 8;             // DMAs per wave per step: 2
  constexpr int ND_B = B_BYTES / 1024 / 8;             // 2 / 1
  constexpr int ND = ND_A + ND_B;
  constexpr int A_CPR = W1B_BM / 8, B_CPR = BN / 8;     // 16-B chunks per image row
  constexpr int A_RPD = 64 / A_CPR, B_RPD = 64 / B_CPR; // image rows per wave-DMA
  constexpr int WN_COLS = BN / 4, TN = WN_COLS / 16;   // wave tile 128 x BN/4
  constexpr int TM = 8;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[W1B_NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;

  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * W1B_BM, c0 = (tile % p.c_tiles) * BN;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  // ---- DMA sources (32-bit element offsets of step 0; host check P*K, H*W*C < 2^31) ----
  int a_src[ND_A], b_src[ND_B];
#pragma unroll
  for (int i = 0; i < ND_A; ++i) {
    const int d = wv * ND_A + i;                     // wave-DMA index within the A image
    const int r = d * A_RPD + lane / A_CPR, s = lane % A_CPR;
    a_src[i] = r * p.K + k0 + ((s ^ kout_swz_w1<W1B_BM>(r)) << 3);
  }
#pragma unroll
  for (int i = 0; i < ND_B; ++i) {
    const int d = wv * ND_B + i;
    const int r = d * B_RPD + lane / B_CPR, s = lane % B_CPR;
    const int xp = p.xst * (p.xw * (r / p.xq) + r % p.xq);
    b_src[i] = xp * p.C + c0 + ((s ^ kout_swz_w1<BN>(r)) << 3);
  }
  const int sA = 32 * p.K, sB = p.x_step;
  w1_gptr zp = (w1_gptr)w1_zero16;
  asm volatile("" : "+s"(zp));
  const w1_gptr gdy = (w1_gptr)p.dy, gx = (w1_gptr)p.x;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)smem;
  auto issue = [&](int step) __attribute__((always_inline)) {
    const bool ok = step < s_end;
    const uint32_t st = lds0 + (uint32_t)((step % W1B_NS) * STAGE);
#pragma unroll
    for (int i = 0; i < ND_A; ++i)
      w1_glds16(ok ? gdy + (a_src[i] + step * sA) : zp, st + (wv * ND_A + i) * 1024);
#pragma unroll
    for (int i = 0; i < ND_B; ++i)
      w1_glds16(ok ? gx + (b_src[i] + step * sB) : zp, st + A_BYTES + (wv * ND_B + i) * 1024);
  };

  // ---- fragment offsets (as wgrad1x1_pipe_kernel) ----
  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q;
  auto kout = [&](auto cols_tag, int row, int col0) __attribute__((always_inline)) {
    constexpr int COLS = decltype(cols_tag)::value;
    const int col = col0 + 4 * pp;
    return w1_off<COLS>(row, col >> 3) + (col & 7) * 2;
  };
  // stage-0 byte offsets of the fragments (a stage adds k % 4 · STAGE); pixel row p_hi =
  // p_lo + 4 is a constant 4·COLS·2 bytes further (the swizzle ignores row bit 2)
  int ao[TM], bo[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) ao[i] = kout(std::integral_constant<int, W1B_BM>{}, p_lo, wm * 128 + 16 * i);
#pragma unroll
  for (int j = 0; j < TN; ++j) bo[j] = A_BYTES + kout(std::integral_constant<int, BN>{}, p_lo, wn * WN_COLS + 16 * j);
  auto frag = [&](const unsigned char* b, int o, auto cols_tag) __attribute__((always_inline)) -> bf16x8 {
    constexpr int HI = 4 * decltype(cols_tag)::value * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1_lds_bf16x4*)(b + o + HI));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software-pipelined over two named fragment sets: iteration k waits for step k+1's DMA,
  // passes the barrier (its lgkmcnt(0) also completes step k's fragment reads, issued one
  // iteration earlier), issues step k+1's fragment reads and step k+4's DMA into step k's
  // slot (every wave has finished reading it: the barrier), then runs step k's MFMAs on the
  // fragments in registers -- the reads and the DMA fly under the MFMAs.
  auto read_set = [&](int k, bf16x8 (&fa)[TM], bf16x8 (&fb)[TN]) __attribute__((always_inline)) {
    const unsigned char* b = smem + (k % W1B_NS) * STAGE;
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = frag(b, bo[j], std::integral_constant<int, BN>{});
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = frag(b, ao[i], std::integral_constant<int, W1B_BM>{});
  };
  auto iter = [&](int k, bf16x8 (&ca)[TM], bf16x8 (&cb)[TN], bf16x8 (&na)[TM], bf16x8 (&nb)[TN])
      __attribute__((always_inline)) {
    w1_vm_wait<2 * ND>();
    w1_lds_barrier();
    read_set(k + 1, na, nb);
    issue(k + 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cb[j], ca[i], acc[i][j], 0, 0, 0);
  };
  bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  issue(s_begin);
  issue(s_begin + 1);
  issue(s_begin + 2);
  issue(s_begin + 3);
  w1_vm_wait<3 * ND>();
  w1_lds_barrier();
  read_set(s_begin, fa0, fb0);
  for (int k = s_begin; k < s_end; k += 2) {
    iter(k, fa0, fb0, fa1, fb1);
    if (k + 1 < s_end) iter(k + 1, fa1, fb1, fa0, fb0);
  }
  w1_vm_wait<0>();   // the tail DMAs (zero page) land before the block's LDS is released

  float* out = p.part + (size_t)split * p.K * p.C;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = k0 + wm * 128 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = c0 + wn * WN_COLS + 16 * j + 4 * h4;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * p.C + n,
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}

// SDX_W1_BN=128 forces the 128-column tile on every shape (co-residency experiments: the
// non-pipelined 128x128 kernel holds 112 VGPRs, so an 8-wave main-stream block fits beside it)
// pixel-pair view (stride 1, a 64-channel side: the layer-1 bottleneck 1x1 convs, reference
// networks/resnet_big.py:44,48 at planes = 64): two consecutive pixels' 64 channels form one
// 128-wide row, so the kernel's 128-row / 128-column tiles stay whole. The GEMM over the
// pair view also forms the even x odd cross blocks (MFMA work thrown away: these GEMMs are
// HBM-bound), while dy and x are read at full 16-B chunks in one pass
//
// Opt-in (SDX_W1_PAIRS=1, or wgrad1x1_pairs_set): measured no faster than the generic
// kernel at CIFAR (65-68 vs 70 us stand-alone at 256 blocks, in-step within noise) and slower
// at config 5 (71.3 vs 70.5 ms/step): the 32-pixel-pair step loop is latency-bound once its
// MFMA work doubles (profiles/wgrad1x1_pairs_r5.txt)
std::atomic<int>& w1_pairs_flag() {
  static std::atomic<int> on{[] {
    const char* e = getenv("SDX_W1_PAIRS");
    return e != nullptr && atoi(e) != 0 ? 1 : 0;
  }()};
  return on;
}
bool w1_pairs(const ConvGeom& g) {
  return w1_pairs_flag().load(std::memory_order_relaxed) != 0 && g.stride == 1 && g.R == 1 && g.S == 1 && g.pad == 0 && (g.K == 64 || g.C == 64) && g.K % 64 == 0 &&
         g.C % 64 == 0 && ((long)g.N * g.P * g.Q) % 64 == 0;
}
int w1_kv(const ConvGeom& g) { return w1_pairs(g) ? 2 * g.K : g.K; }
int w1_cv(const ConvGeom& g) { return w1_pairs(g) ? 2 * g.C : g.C; }

// the 256-row LDS-DMA kernel: dy channels % 256, the non-GEN x addressing (stride 1, or a
// strided shortcut whose 32-pixel step is whole output rows), not the pixel-pair view.
// SDX_W1_BIG=0: the 128-row kernels for every shape
bool w1_pipe_enabled(const ConvGeom& g);
std::atomic<int>& w1_big_flag() {
  static std::atomic<int> on{[] {
    const char* e = getenv("SDX_W1_BIG");
    return e == nullptr ? 1 : atoi(e) < 0 ? 0 : atoi(e) > 2 ? 2 : atoi(e);
  }()};
  return on;
}
// SDX_W1_BIG / wgrad1x1_big_set: 0 off, 1 (default) by the rule below, 2 every eligible shape.
// Only for GEMMs with steps_total x tiles >= SDX_W1_BIG_MIN (default 8192: >= 64 steps per
// split at the 128-block in-step target). Stand-alone the kernel is 2-12 % faster on every
// layer 2-4 shape; in the step, on every shape, it made the step 0.04 ms SLOWER (11.786 vs
// 11.749 ms, 3 interleaved rounds, profiles/w1_big_ab_r6.txt): its 128 KiB of LDS per block
// leaves no room for a main-stream block on its CU, and at 32 steps per split its fp32 slab
// round trip (twice the old kernel's at the same block count) eats the gain. The long-split
// shapes (projection blocks, l2 expand convs) keep 9-12 %.
bool w1_big(const ConvGeom& g) {
  static const long min_work = [] {
    const char* e = getenv("SDX_W1_BIG_MIN");
    return e ? atol(e) : 8192L;
  }();
  const int mode = w1_big_flag().load(std::memory_order_relaxed);   // 0 off, 1 by the rule, 2 always
  if (!(mode != 0 && !w1_pairs(g) && g.K % W1B_BM == 0 && g.C % 128 == 0 &&
        w1_pipe_enabled(g) && (g.stride == 1 || 32 % g.Q == 0)))
    return false;
  const long steps = (long)g.N * g.P * g.Q / 32;
  const long tiles = (long)(g.K / W1B_BM) * (g.C / (g.C % 256 == 0 ? 256 : 128));
  return mode == 2 || steps * tiles >= min_work;
}

int wgrad1x1_bn(const ConvGeom& g) {
  static const int force = [] {
    const char* e = getenv("SDX_W1_BN");
    return e ? atoi(e) : 0;
  }();
  if (force == 128) return 128;
  return w1_cv(g) % 256 == 0 ? 256 : 128;
}

bool w1_pipe_enabled(const ConvGeom& g) {
  static const bool on = [] {
    const char* e = getenv("SDX_W1_PIPE");
    return e == nullptr || atoi(e) != 0;
  }();
  // 32-bit element offsets: dy (output pixels) and x (input pixels)
  return on && (long)g.N * g.P * g.Q * g.K < (1L << 31) && (long)g.N * g.H * g.W * g.C < (1L << 31);
}

}  // namespace

// stride 1 (any image size), or a strided 1x1 (projection shortcut, reference
// networks/resnet_big.py:50-55) on the pipelined kernel when the input is exactly st x the
// output (Q | 32: the x source of a step pixel is base + step·const; otherwise the GEN
// instantiation divides the step pixel index by Q)
bool wgrad1x1_supported(const ConvGeom& g) {
  static const bool strided_on = [] {   // SDX_W1_STRIDED=0: strided shortcuts on the generic kernel
    const char* e = getenv("SDX_W1_STRIDED");
    return e == nullptr || atoi(e) != 0;
  }();
  const bool strided_ok = strided_on && g.stride > 1 && g.H == g.stride * g.P && g.W == g.stride * g.Q &&
                          (long)g.N * g.P * g.Q * g.Q < (1L << 32) &&
                          w1_pipe_enabled(g);
  if (g.R == 1 && g.S == 1 && g.pad == 0 && g.stride == 1 && g.P == g.H && g.Q == g.W && w1_pairs(g))
    return w1_pipe_enabled(g);
  return g.R == 1 && g.S == 1 && g.pad == 0 && (g.stride == 1 ? (g.P == g.H && g.Q == g.W) : strided_ok) &&
         g.K % W1_BM == 0 && g.C % 128 == 0 && ((long)g.N * g.P * g.Q) % 32 == 0;
}

int wgrad1x1_tiles(const ConvGeom& g) {
  if (w1_big(g)) return (g.K / W1B_BM) * (g.C / wgrad1x1_bn(g));
  return (w1_kv(g) / W1_BM) * (w1_cv(g) / wgrad1x1_bn(g));
}

int wgrad1x1_steps(const ConvGeom& g) { return (int)((long)g.N * g.P * g.Q / (w1_pairs(g) ? 64 : 32)); }

int wgrad1x1_slices(const ConvGeom& g, int splits) { return w1_pairs(g) ? 2 * splits : splits; }

bool wgrad1x1_pair_view(const ConvGeom& g) { return w1_pairs(g); }

int wgrad1x1_pairs_set(int on) { return w1_pairs_flag().exchange(on ? 1 : 0); }

int wgrad1x1_big_set(int mode) { return w1_big_flag().exchange(mode < 0 ? 0 : mode > 2 ? 2 : mode); }

hipError_t launch_wgrad1x1(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int splits,
                           int accumulate, hipStream_t s) {
  if (!wgrad1x1_supported(g) || splits < 1) return hipErrorInvalidValue;
  W1Params p{};
  p.dy = (const uint16_t*)dy;
  p.x = (const uint16_t*)x;
  p.pairs = w1_pairs(g) ? 1 : 0;
  p.K0 = g.K;
  p.C0 = g.C;
  p.K = w1_kv(g);
  p.C = w1_cv(g);
  p.steps_total = wgrad1x1_steps(g);
  if (g.stride == 1) {
    p.xst = 1, p.xq = 32, p.xw = 32;   // xpix(j) = j
    p.x_step = 32 * p.C;
  } else {
    p.xst = g.stride, p.xq = g.Q, p.xw = g.W;
    p.x_step = 32 % g.Q == 0 ? g.stride * g.W * (32 / g.Q) * g.C : 0;
    p.xmagic = (unsigned)((1ULL << 32) / (unsigned)g.Q + 1);
  }
  p.steps_per_split = (p.steps_total + splits - 1) / splits;
  p.splits = (p.steps_total + p.steps_per_split - 1) / p.steps_per_split;
  const int bn = wgrad1x1_bn(g);
  const bool big = w1_big(g);
  p.k_tiles = p.K / (big ? W1B_BM : W1_BM);
  p.c_tiles = p.C / bn;
  const bool direct = p.splits == 1 && !accumulate && !p.pairs;
  if (!direct && partial == nullptr) return hipErrorInvalidValue;
  p.part = direct ? dw : partial;
  const dim3 grid(p.k_tiles * p.c_tiles * p.splits), block(W1_NT);
  if (big) {
    if (bn == 256) hipLaunchKernelGGL(wgrad1x1_big_kernel<256>, grid, block, 0, s, p);
    else hipLaunchKernelGGL(wgrad1x1_big_kernel<128>, grid, block, 0, s, p);
  } else if (w1_pipe_enabled(g)) {   // (a strided shape is supported only when it is)
    const bool gen = g.stride > 1 && 32 % g.Q != 0;
    if (gen) {
      if (bn == 256) hipLaunchKernelGGL((wgrad1x1_pipe_kernel<256, true>), grid, block, 0, s, p);
      else hipLaunchKernelGGL((wgrad1x1_pipe_kernel<128, true>), grid, block, 0, s, p);
    } else if (bn == 256) {
      hipLaunchKernelGGL((wgrad1x1_pipe_kernel<256, false>), grid, block, 0, s, p);
    } else {
      hipLaunchKernelGGL((wgrad1x1_pipe_kernel<128, false>), grid, block, 0, s, p);
    }
  } else if (bn == 256) {
    hipLaunchKernelGGL(wgrad1x1_kernel<256>, grid, block, 0, s, p);
  } else {
    hipLaunchKernelGGL(wgrad1x1_kernel<128>, grid, block, 0, s, p);
  }
  SDX_LAUNCH_CHECK();
  if (direct) return hipSuccess;
  return launch_splitk_reduce(partial, p.pairs ? 2 * p.splits : p.splits, (long)g.K * g.C / 4, dw, accumulate, s);
}
