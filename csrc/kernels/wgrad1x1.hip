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
// N·H·W % 32 == 0 — layers 2-4 of the CIFAR/ImageNet ResNet bottlenecks (reference
// networks/resnet_big.py:44-49, conv1/conv3 of each Bottleneck). The layer-1 1x1 wgrads
// (64 channels on one side) are HBM-bound and stay on the generic kernel.
#include <type_traits>

#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

constexpr int W1_NT = 512;      // 8 waves: 2 (output rows) x 4 (output columns)
constexpr int W1_BM = 128;      // output channels (dW rows) per block
constexpr int W1_PF = 4;        // steps of loads in flight (register ring of 4 named slots)

typedef __attribute__((address_space(3))) bf16x4 w1_lds_bf16x4;

__device__ __attribute__((aligned(16))) uint16_t w1_zero16[8];

// K-outer image [32][COLS] bf16: 16-B chunk ch of row r (igemm.hip kout_off, COLS >= 128)
template <int COLS>
__device__ __forceinline__ int w1_off(int r, int ch) {
  const int swz = ((r & 3) | (((r >> 3) & 1) << 2)) << 1;
  return r * (COLS * 2) + ((ch ^ swz) << 4);
}

struct W1Params {
  const uint16_t* dy;   // [P][K]
  const uint16_t* x;    // [P][C]
  float* part;          // [splits][K][C]
  int K, C;
  int steps_total;      // P / 32
  int steps_per_split;
  int k_tiles, c_tiles, splits;
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

int wgrad1x1_bn(const ConvGeom& g) { return g.C % 256 == 0 ? 256 : 128; }

}  // namespace

bool wgrad1x1_supported(const ConvGeom& g) {
  return g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0 && g.P == g.H && g.Q == g.W && g.K % W1_BM == 0 &&
         g.C % 128 == 0 && ((long)g.N * g.H * g.W) % 32 == 0;
}

int wgrad1x1_tiles(const ConvGeom& g) { return (g.K / W1_BM) * (g.C / wgrad1x1_bn(g)); }

int wgrad1x1_steps(const ConvGeom& g) { return (int)((long)g.N * g.H * g.W / 32); }

hipError_t launch_wgrad1x1(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int splits,
                           int accumulate, hipStream_t s) {
  if (!wgrad1x1_supported(g) || splits < 1) return hipErrorInvalidValue;
  W1Params p{};
  p.dy = (const uint16_t*)dy;
  p.x = (const uint16_t*)x;
  p.K = g.K;
  p.C = g.C;
  p.steps_total = wgrad1x1_steps(g);
  p.steps_per_split = (p.steps_total + splits - 1) / splits;
  p.splits = (p.steps_total + p.steps_per_split - 1) / p.steps_per_split;
  const int bn = wgrad1x1_bn(g);
  p.k_tiles = g.K / W1_BM;
  p.c_tiles = g.C / bn;
  const bool direct = p.splits == 1 && !accumulate;
  if (!direct && partial == nullptr) return hipErrorInvalidValue;
  p.part = direct ? dw : partial;
  const dim3 grid(p.k_tiles * p.c_tiles * p.splits), block(W1_NT);
  if (bn == 256) hipLaunchKernelGGL(wgrad1x1_kernel<256>, grid, block, 0, s, p);
  else hipLaunchKernelGGL(wgrad1x1_kernel<128>, grid, block, 0, s, p);
  SDX_LAUNCH_CHECK();
  if (direct) return hipSuccess;
  return launch_splitk_reduce(partial, p.splits, (long)g.K * g.C / 4, dw, accumulate, s);
}
