// Tap-reuse 3x3 weight gradient (stride 1, pad 1) on gfx950 MFMA, NHWC bf16 -> fp32.
//
//   dW[k][r][s][c] = Σ_{n,h,w} dy[n][h][w][k] · x[n][h+r−1][w+s−1][c]
//
// The generic implicit-GEMM wgrad (igemm.hip, MODE_WGRAD) treats the 9 taps as 9 separate
// column tiles, so every tap tile re-reads the dy tile and its own shifted copy of x. Here
// one 512-thread block owns 64 output channels × 64 input channels × ALL 9 taps (576 GEMM
// columns) and walks its K-split 32 pixels at a time: per step it stages the 32×64 dy tile
// and a zero-padded window of x — the 3 source rows (h−1, h, h+1) of every image row of
// the step, one zero column on each side — ONCE in LDS, and the 9 taps read that window at
// row/column offsets (r, s). Operand traffic per MFMA is ~2.3x lower than the tap-tiled GEMM.
//
// Shapes: square images of width W ∈ {4, 8, 16, 32} (a 32-pixel step is 32/W whole image rows, which
// may span several images; each row's source rows are validated against its own image),
// C % 64 == 0, K % 64 == 0 — every 3x3 conv of the CIFAR ResNets (reference
// networks/resnet_big.py:41-47, conv2 of each Bottleneck / both convs of a BasicBlock).
// Other shapes use the generic kernel.
//
// LDS rows are 64 bf16 (128 B); the 16-B chunk index is XOR-swizzled by g(R) = (R/2 + 2·(R/8))
// mod 4 (in 32-B blocks). A ds_read_b64_tr_b16 half-wave reads 8 rows x 32 B: rows R0+{0..3}
// and R0+{8..11} (+16k) for consecutive pixels, and this swizzle puts them on distinct banks
// for ANY R0 — i.e. for every tap shift. Multi-row steps keep that pattern by padding the
// window row pitch to P ≡ 8 (mod 16) rows between pixel rows 8 apart (W=8: P=24, W=4: P=12;
// W=16/32 read within one row). Fragments follow igemm.hip's convention: the MFMA is issued
// as D = Bᵀ·Aᵀ, so each lane holds 4 consecutive output columns of one output row. Output:
// an fp32 partial slab per K-split, reduced deterministically by the split-K reduction of
// igemm.hip (no atomics).
#include <type_traits>

#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

// SDX_W3_ORDER (default 1): a step's LDS stores and refill loads are issued before its
// fragment reads and MFMAs (sched_barrier-pinned; otherwise the stores trail the MFMAs and
// the barrier's lgkmcnt(0) waits for them): 6-8 % faster per kernel (81.7 vs 88.5 us at l3,
// profiles/wgrad_order_r4.txt); 0 = the compiler's order
#ifndef SDX_W3_ORDER
#define SDX_W3_ORDER 1
#endif

constexpr int W3_NT = 512;      // 8 waves: 2 (output channels) x 4 (columns)
constexpr int W3_ROWB = 128;    // LDS row: 64 bf16
constexpr int W3_DY_BYTES = 32 * W3_ROWB;
constexpr int W3_PF = 4;        // steps of loads in flight (register ring of 4 named slots)

typedef __attribute__((address_space(3))) bf16x4 w3_lds_bf16x4;

__device__ __attribute__((aligned(16))) uint16_t w3_zero16[8];
typedef const __attribute__((address_space(1))) uint16_t* w3_gptr;
typedef unsigned int w3_u32x4 __attribute__((ext_vector_type(4)));   // (a HIP uint4 cannot be read
typedef const __attribute__((address_space(1))) w3_u32x4* w3_g16;     //  through an AS-1 pointer)

// byte offset of 16-B chunk ch of LDS row R
__device__ __forceinline__ int w3_off(int R, int ch) {
  const int g = ((R >> 1) + 2 * (R >> 3)) & 3;
  return R * W3_ROWB + ((ch ^ (g << 1)) << 4);
}

struct W3Params {
  const uint16_t* dy;   // [N*H*W][K]
  const uint16_t* x;    // [N*H*W][C]
  float* part;          // [splits][K][9*C]
  int K, C;
  int steps_total;      // N*H*W / 32
  int steps_per_split;
  int k_tiles, c_tiles, splits;
  int h, w;             // image size (wgrad3x3_pad_kernel)
};

template <int W>
struct W3Geom {
  static constexpr int RPS = 32 / W;                                   // image rows per step
  static constexpr int P = W == 32 ? 34 : W == 16 ? 18 : W == 8 ? 24 : 12;   // window row pitch
  static_assert(P >= W + 2, "pad columns");
  static constexpr int XROWS = 3 * RPS * P;                            // LDS rows of the x window
  static constexpr int STAGE = W3_DY_BYTES + XROWS * W3_ROWB;
};

template <int W>
__global__ __launch_bounds__(W3_NT, 1) void wgrad3x3_kernel(W3Params p) {
  using G = W3Geom<W>;
  constexpr int RPS = G::RPS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;

  // ---- tile / split (split-major: an XCD's co-resident blocks share one pixel range) ----
  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * 64, c0 = (tile % p.c_tiles) * 64;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  // ---- zero the pad columns of both x windows (never written by the loads) ----
  for (int e = tid; e < 2 * 3 * RPS * 2 * 8; e += W3_NT) {
    const int ch = e & 7, side = (e >> 3) & 1, ri = (e >> 4) % (3 * RPS), buf = (e >> 4) / (3 * RPS);
    const int row = ri * G::P + (side ? W + 1 : 0);
    *reinterpret_cast<uint4*>(smem + buf * G::STAGE + W3_DY_BYTES + w3_off(row, ch)) = make_uint4(0u, 0u, 0u, 0u);
  }

  // ---- loader: 1024 16-B chunks per step, 2 per thread: chunk tid is a dy chunk for the
  // first 256 threads and an x-window chunk otherwise; chunk tid + 512 is always x ----
  // x-window chunk e (0..767): channel chunk e%8 of pixel w of window row ri = (r, i)
  // Per-thread loader state, fixed for the whole K loop: a step moves every chunk by 32
  // pixels (dy: 32 rows of K; x: RPS image rows of W pixels = 32 pixels of C), so a load is
  // base + step·stride plus, for x, the validity of its source row. Steps at or past s_end
  // (the unrolled loop's tail) load the zero page: they add nothing.
  // x-window chunk e (0..767): channel chunk e%8 of pixel w of window row ri = (r, i)
  // zero page pinned in an SGPR pair: otherwise every select re-materialises its address
  // (s_getpc + a GOT load + lgkmcnt(0), which also drains this wave's LDS traffic) and the
  // divergent selects become exec-masked branches
  w3_gptr zp = (w3_gptr)w3_zero16;
  asm volatile("" : "+s"(zp));
  struct XChunk {
    w3_gptr base;   // x element of step 0 (may lie outside x: used only when valid)
    int i, r;       // window image row within the step, tap row
  };
  auto x_chunk = [&](int e) -> XChunk {
    const int ch = e & 7, rest = e >> 3;
    const int w = rest % W, ri = rest / W;
    const int r = ri / RPS, i = ri % RPS;
    return {(w3_gptr)p.x + ((long)(i + r - 1) * W + w) * p.C + c0 + ch * 8, i, r};
  };
  auto x_src = [&](const XChunk& xc, int step) -> w3_gptr {
    const int hs = ((step * RPS + xc.i) & (W - 1)) + xc.r - 1;   // H == W
    const bool ok = step < s_end && (unsigned)hs < (unsigned)W;
    return ok ? xc.base + (long)step * 32 * p.C : zp;
  };
  auto x_dst = [&](int e) -> int {
    const int ch = e & 7, rest = e >> 3;
    return W3_DY_BYTES + w3_off((rest / W) * G::P + rest % W + 1, ch);
  };
  const bool first_dy = tid < 256;
  const int e0 = tid - 256, e1 = tid + 256;          // x chunk indices of chunks tid, tid + 512
  const int dst0 = first_dy ? w3_off(tid >> 3, tid & 7) : x_dst(e0);
  const int dst1 = x_dst(e1);
  const XChunk xc0 = x_chunk(first_dy ? 0 : e0), xc1 = x_chunk(e1);
  const w3_gptr dy_base = (w3_gptr)p.dy + (long)(tid >> 3) * p.K + k0 + (tid & 7) * 8;
  // register ring of 4 prefetched steps: slot u holds the step ≡ s_begin + u (mod 4). Named
  // registers selected at compile time (an array indexed inside the lambdas goes to scratch)
  w3_u32x4 ra0, rb0, ra1, rb1, ra2, rb2, ra3, rb3;
  auto slot_a = [&](auto U) -> w3_u32x4& {
    if constexpr (decltype(U)::value == 0) return ra0;
    else if constexpr (decltype(U)::value == 1) return ra1;
    else if constexpr (decltype(U)::value == 2) return ra2;
    else return ra3;
  };
  auto slot_b = [&](auto U) -> w3_u32x4& {
    if constexpr (decltype(U)::value == 0) return rb0;
    else if constexpr (decltype(U)::value == 1) return rb1;
    else if constexpr (decltype(U)::value == 2) return rb2;
    else return rb3;
  };
  auto load = [&](int step, w3_u32x4& a, w3_u32x4& b) {
    const w3_gptr s0 = first_dy ? (step < s_end ? dy_base + (long)step * 32 * p.K : zp) : x_src(xc0, step);
    a = *(w3_g16)s0;
    b = *(w3_g16)x_src(xc1, step);
  };
  auto store = [&](int buf, const w3_u32x4& a, const w3_u32x4& b) {
    *reinterpret_cast<w3_u32x4*>(smem + buf * G::STAGE + dst0) = a;
    *reinterpret_cast<w3_u32x4*>(smem + buf * G::STAGE + dst1) = b;
  };

  // ---- fragment addressing: lane (h4, c16 = 4q + pp) reads K rows (pixels) 8h4+q and +4,
  // columns col0 + 4pp .. +3 (ds_read_b64_tr_b16 transposes across the 4 q-lanes). The byte
  // offsets are step-invariant: computed once (2 A + 9 B fragments, lo/hi rows). ----
  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q, p_hi = p_lo + 4;
  const int xb_lo = (p_lo / W) * G::P + (p_lo % W);   // x-window row of pixel p, tap (0, 0)
  const int xb_hi = (p_hi / W) * G::P + (p_hi % W);
  auto lane_off = [&](int row, int col0) {
    const int col = col0 + 4 * pp;
    return w3_off(row, col >> 3) + (col & 7) * 2;
  };
  int ao_lo[2], ao_hi[2], bo_lo[9], bo_hi[9];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ao_lo[i] = lane_off(p_lo, wm * 32 + 16 * i);
    ao_hi[i] = lane_off(p_hi, wm * 32 + 16 * i);
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int n = wn * 144 + 16 * j;             // wave column tile: one tap, 16 channels
    const int t = n >> 6, r = t / 3, s = t - 3 * r;
    const int off = r * RPS * G::P + s;
    bo_lo[j] = W3_DY_BYTES + lane_off(xb_lo + off, n & 63);
    bo_hi[j] = W3_DY_BYTES + lane_off(xb_hi + off, n & 63);
  }
  auto frag = [&](const unsigned char* base, int o_lo, int o_hi) -> bf16x8 {
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_lo));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_hi));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const unsigned char* base = smem + buf * G::STAGE;
    bf16x8 af[2], bfr[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) bfr[j] = frag(base, bo_lo[j], bo_hi[j]);
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag(base, ao_lo[i], ao_hi[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

  // ---- K loop: two LDS buffers, one barrier per step. The loads of step k+1+W3_PF are
  // issued as step k+1 leaves the ring for LDS, so W3_PF steps of loads are always in
  // flight: one step's MFMAs (~300 cycles a wave) are far shorter than an HBM miss. The loop
  // is unrolled by W3_PF (even) and runs whole groups, so ring slots and LDS parity are
  // compile-time. ----
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  // step k = base + U of the unrolled loop: compute from LDS buffer U&1, move step k+1 from
  // its ring slot into the other buffer, refill that slot with step k+1+4. Branch-free (the
  // tail steps read zeros), so the compiler's vmcnt waits retire only the oldest step's loads
  auto iter = [&](int base, auto U) {
    constexpr int u = decltype(U)::value;
    using N = std::integral_constant<int, (u + 1) % W3_PF>;
#if SDX_W3_ORDER
    // the store of step k+1 (other buffer) and the refill loads issue before step k's
    // fragment reads + MFMAs and complete under them instead of in front of the barrier
    store((u + 1) & 1, slot_a(N{}), slot_b(N{}));
    load(base + u + 1 + W3_PF, slot_a(N{}), slot_b(N{}));
    __builtin_amdgcn_sched_barrier(0);
    compute(u & 1);
    __builtin_amdgcn_sched_barrier(0);
#else
    compute(u & 1);
    store((u + 1) & 1, slot_a(N{}), slot_b(N{}));
    load(base + u + 1 + W3_PF, slot_a(N{}), slot_b(N{}));
#endif
    __syncthreads();
  };
  load(s_begin, ra0, rb0);
  load(s_begin + 1, ra1, rb1);
  load(s_begin + 2, ra2, rb2);
  load(s_begin + 3, ra3, rb3);
  store(0, ra0, rb0);
  load(s_begin + W3_PF, ra0, rb0);
  __syncthreads();
  for (int base = s_begin; base < s_end; base += W3_PF) {
    iter(base, I0{});
    iter(base, I1{});
    iter(base, I2{});
    iter(base, I3{});
  }

  // ---- epilogue: fp32 partial rows, 4 consecutive columns (same tap) per lane ----
  const int Ncol = 9 * p.C;
  float* out = p.part + (size_t)split * p.K * Ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = k0 + wm * 32 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int n = wn * 144 + 16 * j + 4 * h4;
      const int t = n >> 6;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * Ncol + t * p.C + c0 + (n & 63),
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}


// ---------------------------------------------------------------------------------------
// Stride-2 variant (the first 3x3 conv of layers 2-4, reference networks/resnet_big.py:45):
//
//   dW[k][r][s][c] = Σ dy[n][ho][wo][k] · x[n][2ho+r−1][2wo+s−1][c]
//
// Same block tile (64 output x 64 input channels x all 9 taps), same 32-pixel steps (RPS =
// 32/Q whole output rows) and the same fragment images as wgrad3x3_kernel; only the x window
// differs. Consecutive output pixels read every other input column, so each window row (tap
// row r, output row i — input row 2ho+r−1) is stored DE-INTERLEAVED: an odd block
// O[0..Q] = input columns −1, 1, ..., 2Q−1 (O[0] is the zero pad) and an even block
// E[0..Q−1] = columns 0, 2, ..., 2Q−2. Tap s = 0 / 1 / 2 of output column wo then reads
// O[wo] / E[wo] / O[wo+1]: consecutive pixels are consecutive LDS rows again, so the
// swizzle stays conflict-free; the window row pitch PT keeps pixels 8 apart at a distance
// ≡ 8 (mod 16) rows (Q = 8: PT = 24; Q = 4: two output rows, PT = 12). Per step: 256 dy
// chunks + 3·RPS·2Q·8 = 1536 x chunks (every input column of 3·RPS input rows), 3.5 per
// thread; a 2-deep register ring keeps VGPRs at the stride-1 kernel's level.
template <int Q>
struct W3S2Geom {
  static constexpr int RPS = 32 / Q;
  static constexpr int PT = Q >= 16 ? 2 * Q + 1 : Q == 8 ? 24 : 12;
  static_assert(PT >= 2 * Q + 1, "window row");
  static constexpr int XROWS = 3 * RPS * PT;
  static constexpr int STAGE = W3_DY_BYTES + XROWS * W3_ROWB;
  static constexpr int XCH = 3 * RPS * 2 * Q * 8;    // x chunks per step (1536)
  static_assert(XCH == 1536, "loader layout");
};

// PAD: output width pq = p.w / 2 < Q slots (not a power of two: the 224x224 config's 28 / 14 /
// 7 on 32 / 16 / 8 slots); slots c >= pq and input columns >= 2·pq read the zero page
template <int Q, bool PAD>
__global__ __launch_bounds__(W3_NT, 1) void wgrad3x3_s2_kernel(W3Params p) {
  using G = W3S2Geom<Q>;
  constexpr int RPS = G::RPS, W = 2 * Q;
  const int Wr = PAD ? p.w : W, pq = PAD ? p.w / 2 : Q;   // real input / output widths
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;

  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * 64, c0 = (tile % p.c_tiles) * 64;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  // zero pads O[0] of every window row in both buffers (never written by the loads)
  for (int e = tid; e < 2 * 3 * RPS * 8; e += W3_NT) {
    const int ch = e & 7, ri = (e >> 3) % (3 * RPS), buf = (e >> 3) / (3 * RPS);
    *reinterpret_cast<uint4*>(smem + buf * G::STAGE + W3_DY_BYTES + w3_off(ri * G::PT, ch)) =
        make_uint4(0u, 0u, 0u, 0u);
  }

  // loader: chunk f = tid + 512u (u < 4, f < 1792): f < 256 a dy chunk (pixel f/8, channel
  // chunk f%8), else x chunk e = f − 256: channel chunk e%8 of input column e/8 % 2Q of
  // window row ri = e/(16Q) = (r, i). Output row Rg = step·RPS + i (global over images, H =
  // 2P) reads input row 2Rg + r − 1: x element base + step·(2·RPS·W·C)
  w3_gptr zp = (w3_gptr)w3_zero16;   // pinned in SGPRs (see wgrad3x3_kernel)
  asm volatile("" : "+s"(zp));
  struct XChunk {
    w3_gptr base;   // element of step 0 (used only when valid)
    int i, r, dst;
    bool cok;       // input column inside the image (PAD)
  };
  auto x_chunk = [&](int e) -> XChunk {
    const int ch = e & 7, rest = e >> 3;
    const int col = rest % W, ri = rest / W;
    const int r = ri / RPS, i = ri % RPS;
    const int lrow = ri * G::PT + ((col & 1) ? (col + 1) >> 1 : Q + 1 + (col >> 1));
    return {(w3_gptr)p.x + ((long)(2 * i + r - 1) * Wr + col) * p.C + c0 + ch * 8, i, r, W3_DY_BYTES + w3_off(lrow, ch),
            col < Wr};
  };
  const long x_step = 2L * RPS * Wr * p.C;
  auto x_src = [&](const XChunk& xc, int step) -> w3_gptr {
    const int ho = PAD ? (step * RPS + xc.i) % pq : (step * RPS + xc.i) & (Q - 1);
    const int hi = 2 * ho + xc.r - 1;   // input row within the image
    const bool ok = step < s_end && (unsigned)hi < (unsigned)Wr && (!PAD || xc.cok);
    return ok ? xc.base + (long)step * x_step : zp;
  };
  const bool first_dy = tid < 256, last_x = tid < 256;
  const XChunk xa = x_chunk(first_dy ? 0 : tid - 256), xb = x_chunk(tid + 256), xc_ = x_chunk(tid + 768),
               xd = x_chunk(last_x ? tid + 1280 : 0);
  const int dst_a = first_dy ? w3_off(tid >> 3, tid & 7) : xa.dst;
  // dy slot j = tid/8 = (i, c) = (j / Q, j % Q): output pixel i·pq + c of the step (c < pq)
  const int dslot = tid >> 3;
  const bool dy_ok = !PAD || dslot % Q < pq;
  const long dy_step = PAD ? (long)RPS * pq * p.K : 32L * p.K;
  const w3_gptr dy_base =
      (w3_gptr)p.dy + (long)(PAD ? (dslot / Q) * pq + dslot % Q : dslot) * p.K + k0 + (tid & 7) * 8;
  // 2-step register ring of named vectors (a struct of uint4 read through the lambdas ends up
  // in scratch)
  w3_u32x4 ra0, rb0, rc0, rd0, ra1, rb1, rc1, rd1;
  auto load = [&](int step, w3_u32x4& a, w3_u32x4& b, w3_u32x4& c, w3_u32x4& d) {
    a = *(w3_g16)(first_dy ? (step < s_end && dy_ok ? dy_base + (long)step * dy_step : zp) : x_src(xa, step));
    b = *(w3_g16)x_src(xb, step);
    c = *(w3_g16)x_src(xc_, step);
    d = *(w3_g16)(last_x ? x_src(xd, step) : zp);
  };
  auto store = [&](int buf, const w3_u32x4& a, const w3_u32x4& b, const w3_u32x4& c, const w3_u32x4& d) {
    unsigned char* sb = smem + buf * G::STAGE;
    *reinterpret_cast<w3_u32x4*>(sb + dst_a) = a;
    *reinterpret_cast<w3_u32x4*>(sb + xb.dst) = b;
    *reinterpret_cast<w3_u32x4*>(sb + xc_.dst) = c;
    if (last_x) *reinterpret_cast<w3_u32x4*>(sb + xd.dst) = d;
  };

  // fragments (as wgrad3x3_kernel): pixel p = (i, wo) = (p / Q, p % Q); tap (r, s) reads
  // window row r·RPS + i at O[wo] (s = 0), E[wo] (s = 1), O[wo + 1] (s = 2)
  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q, p_hi = p_lo + 4;
  auto lane_off = [&](int row, int col0) {
    const int col = col0 + 4 * pp;
    return w3_off(row, col >> 3) + (col & 7) * 2;
  };
  auto xrow = [&](int px, int r, int s_) {
    const int i = px / Q, wo = px % Q;
    return (r * RPS + i) * G::PT + (s_ == 1 ? Q + 1 + wo : wo + (s_ >> 1));
  };
  int ao_lo[2], ao_hi[2], bo_lo[9], bo_hi[9];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ao_lo[i] = lane_off(p_lo, wm * 32 + 16 * i);
    ao_hi[i] = lane_off(p_hi, wm * 32 + 16 * i);
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int n = wn * 144 + 16 * j;
    const int t = n >> 6, r = t / 3, s_ = t - 3 * r;
    bo_lo[j] = W3_DY_BYTES + lane_off(xrow(p_lo, r, s_), n & 63);
    bo_hi[j] = W3_DY_BYTES + lane_off(xrow(p_hi, r, s_), n & 63);
  }
  auto frag = [&](const unsigned char* base, int o_lo, int o_hi) -> bf16x8 {
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_lo));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_hi));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    const unsigned char* base = smem + buf * G::STAGE;
    bf16x8 af[2], bfr[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) bfr[j] = frag(base, bo_lo[j], bo_hi[j]);
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag(base, ao_lo[i], ao_hi[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };

  // K loop (wgrad3x3_kernel's, with a 2-step register ring): compute step k from buffer k&1,
  // move step k+1 from its slot into the other buffer, refill the slot with step k+3
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto iter = [&](int base, auto U) {
    constexpr int u = decltype(U)::value;
#if !SDX_W3_ORDER
    compute(u);
#endif
    if constexpr (u == 0) {   // slot 1 holds step base+1
      store(1, ra1, rb1, rc1, rd1);
      load(base + 3, ra1, rb1, rc1, rd1);
    } else {                  // slot 0 holds step base+2
      store(0, ra0, rb0, rc0, rd0);
      load(base + 4, ra0, rb0, rc0, rd0);
    }
#if SDX_W3_ORDER
    __builtin_amdgcn_sched_barrier(0);
    compute(u);
    __builtin_amdgcn_sched_barrier(0);
#endif
    __syncthreads();
  };
  load(s_begin, ra0, rb0, rc0, rd0);
  load(s_begin + 1, ra1, rb1, rc1, rd1);
  store(0, ra0, rb0, rc0, rd0);
  load(s_begin + 2, ra0, rb0, rc0, rd0);
  __syncthreads();
  for (int base = s_begin; base < s_end; base += 2) {
    iter(base, I0{});
    iter(base, I1{});
  }

  const int Ncol = 9 * p.C;
  float* out = p.part + (size_t)split * p.K * Ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = k0 + wm * 32 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int n = wn * 144 + 16 * j + 4 * h4;
      const int t = n >> 6;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * Ncol + t * p.C + c0 + (n & 63),
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}

// ---------------------------------------------------------------------------------------
// Stride-1 3x3 wgrad for image widths that are not a power of two (the 224x224 ImageNet-stem
// ResNets: 56 / 28 / 14 / 7). The 32 pixel SLOTS of a step are RPS segments of SW = min(WS,
// 32) slots, WS = the next power of two >= W: a segment is one image row (W <= 32, slots
// w >= W hold zeros) or one half of a row (32 < W <= 64). Slot (i, c) of step k is column
// w = half·SW + c of row Rg = G / SPR, G = k·RPS + i, half = G % SPR (SPR = WS / SW segments
// per row); its dy row is read when w < W (else the zero page: it adds nothing). The x window
// of segment i holds, for each tap row r, the SW + 2 columns half·SW − 1 … half·SW + SW of
// image row Rg + r − 1, every one loaded with its own validity (image edge, w >= W), so a
// half-row segment sees its real neighbours across the split. Fragment images, swizzle and
// the schedule are wgrad3x3_s2_kernel's (2-step register ring, stores before the MFMAs).
template <int WS>
struct W3PadGeom {
  static constexpr int SW = WS < 32 ? WS : 32;
  static constexpr int SPR = WS / SW;                 // segments per image row
  static constexpr int RPS = 32 / SW;                 // segments per step
  static constexpr int P = SW == 32 ? 34 : SW == 16 ? 18 : 24;   // as W3Geom<SW>
  static constexpr int XROWS = 3 * RPS * P;
  static constexpr int STAGE = W3_DY_BYTES + XROWS * W3_ROWB;
  static constexpr int XCH = 3 * RPS * (SW + 2) * 8;  // x chunks per step (816 / 864 / 960)
  static_assert(XCH > 768 && XCH <= 1280, "loader layout: 3 chunks per thread");
};

template <int WS>
__global__ __launch_bounds__(W3_NT, 1) void wgrad3x3_pad_kernel(W3Params p) {
  using G = W3PadGeom<WS>;
  constexpr int SW = G::SW, SPR = G::SPR, RPS = G::RPS;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h4 = lane >> 4, c16 = lane & 15;
  const int wm = wv >> 2, wn = wv & 3;
  const int W = p.w, H = p.h;

  const int tiles = p.k_tiles * p.c_tiles;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lin % tiles, split = lin / tiles;
  const int k0 = (tile / p.c_tiles) * 64, c0 = (tile % p.c_tiles) * 64;
  const int s_begin = split * p.steps_per_split;
  const int s_end = min(p.steps_total, s_begin + p.steps_per_split);

  w3_gptr zp = (w3_gptr)w3_zero16;   // pinned in SGPRs (see wgrad3x3_kernel)
  asm volatile("" : "+s"(zp));
  const w3_gptr gdy = (w3_gptr)p.dy, gx = (w3_gptr)p.x;
  // loader: chunk f = tid + 512u (u < 3): f < 256 a dy chunk (slot f/8, channel chunk f%8),
  // else x chunk e = f − 256 < XCH: channel chunk e%8 of window column e/8 % (SW+2) of window
  // row e/(8(SW+2)) = (r, i)
  struct Src {
    int i, col, r, ch;   // segment in step, column within the segment (x: −1 … SW), tap row, chunk
    bool x, has;
    int dst;
  };
  auto chunk = [&](int f) -> Src {
    if (f < 256) return {(f >> 3) / SW, (f >> 3) % SW, 1, f & 7, false, true, w3_off(f >> 3, f & 7)};
    const int e = f - 256, ch = e & 7, rest = e >> 3;
    const int cw = rest % (SW + 2), ri = rest / (SW + 2);
    return {ri % RPS, cw - 1, ri / RPS, ch, true, e < G::XCH, W3_DY_BYTES + w3_off(ri * G::P + cw, ch)};
  };
  const Src sa = chunk(tid), sb = chunk(tid + 512), sc = chunk(tid + 1024);
  auto src = [&](const Src& c, int step) -> w3_gptr {
    const int seg = step * RPS + c.i;
    const int rg = seg / SPR, w = (seg % SPR) * SW + c.col;   // image row (global), column
    const int hs = rg % H + c.r - 1;                           // source row within the image
    const bool ok = c.has && step < s_end && (unsigned)w < (unsigned)W && (unsigned)hs < (unsigned)H;
    const long pix = (long)(rg + c.r - 1) * W + w;
    return ok ? (c.x ? gx + pix * p.C + c0 + c.ch * 8 : gdy + pix * p.K + k0 + c.ch * 8) : zp;
  };
  w3_u32x4 ra0, rb0, rc0, ra1, rb1, rc1;
  auto load = [&](int step, w3_u32x4& a, w3_u32x4& b, w3_u32x4& c) {
    a = *(w3_g16)src(sa, step);
    b = *(w3_g16)src(sb, step);
    c = *(w3_g16)src(sc, step);
  };
  auto store = [&](int buf, const w3_u32x4& a, const w3_u32x4& b, const w3_u32x4& c) {
    unsigned char* s_ = smem + buf * G::STAGE;
    *reinterpret_cast<w3_u32x4*>(s_ + sa.dst) = a;
    *reinterpret_cast<w3_u32x4*>(s_ + sb.dst) = b;
    if (sc.has) *reinterpret_cast<w3_u32x4*>(s_ + sc.dst) = c;
  };

  // fragments: slot p = (i, c) = (p / SW, p % SW); tap (r, s) reads window row r·RPS + i,
  // column c + s (window column 0 is the segment's column −1)
  const int q = c16 >> 2, pp = c16 & 3;
  const int p_lo = 8 * h4 + q, p_hi = p_lo + 4;
  const int xb_lo = (p_lo / SW) * G::P + (p_lo % SW), xb_hi = (p_hi / SW) * G::P + (p_hi % SW);
  auto lane_off = [&](int row, int col0) {
    const int col = col0 + 4 * pp;
    return w3_off(row, col >> 3) + (col & 7) * 2;
  };
  int ao_lo[2], ao_hi[2], bo_lo[9], bo_hi[9];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ao_lo[i] = lane_off(p_lo, wm * 32 + 16 * i);
    ao_hi[i] = lane_off(p_hi, wm * 32 + 16 * i);
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int n = wn * 144 + 16 * j;
    const int t = n >> 6, r = t / 3, s_ = t - 3 * r;
    const int off = r * RPS * G::P + s_;
    bo_lo[j] = W3_DY_BYTES + lane_off(xb_lo + off, n & 63);
    bo_hi[j] = W3_DY_BYTES + lane_off(xb_hi + off, n & 63);
  }
  auto frag = [&](const unsigned char* base, int o_lo, int o_hi) -> bf16x8 {
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_lo));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_bf16x4*)(base + o_hi));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    const unsigned char* base = smem + buf * G::STAGE;
    bf16x8 af[2], bfr[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) bfr[j] = frag(base, bo_lo[j], bo_hi[j]);
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = frag(base, ao_lo[i], ao_hi[i]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  auto iter = [&](int base, auto U) {
    constexpr int u = decltype(U)::value;
    if constexpr (u == 0) {   // slot 1 holds step base+1
      store(1, ra1, rb1, rc1);
      load(base + 3, ra1, rb1, rc1);
    } else {                  // slot 0 holds step base+2
      store(0, ra0, rb0, rc0);
      load(base + 4, ra0, rb0, rc0);
    }
    __builtin_amdgcn_sched_barrier(0);
    compute(u);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  load(s_begin, ra0, rb0, rc0);
  load(s_begin + 1, ra1, rb1, rc1);
  store(0, ra0, rb0, rc0);
  load(s_begin + 2, ra0, rb0, rc0);
  __syncthreads();
  for (int base = s_begin; base < s_end; base += 2) {
    iter(base, I0{});
    iter(base, I1{});
  }

  const int Ncol = 9 * p.C;
  float* out = p.part + (size_t)split * p.K * Ncol;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = k0 + wm * 32 + 16 * i + c16;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int n = wn * 144 + 16 * j + 4 * h4;
      const int t = n >> 6;
      const f32x4 a = acc[i][j];
      st16<SDX_NT_PART != 0>(out + (size_t)m * Ncol + t * p.C + c0 + (n & 63),
                             make_uint4(__float_as_uint(a[0]), __float_as_uint(a[1]), __float_as_uint(a[2]),
                                        __float_as_uint(a[3])));
    }
  }
}

// padded-slot kernel: slot width WS (next power of two >= W) for stride-1 widths that are not
// one of {4, 8, 16, 32}
int w3_pad_ws(const ConvGeom& g) {
  static const bool on = [] {   // SDX_W3_PAD=0: those widths on the generic kernel
    const char* e = getenv("SDX_W3_PAD");
    return e == nullptr || atoi(e) != 0;
  }();
  if (!on || g.stride != 1 || g.W == 4 || g.W == 8 || g.W == 16 || g.W == 32 || g.W < 5 || g.W > 64) return 0;
  const int ws = g.W <= 8 ? 8 : g.W <= 16 ? 16 : g.W <= 32 ? 32 : 64;
  const int sw = ws < 32 ? ws : 32, spr = ws / sw, rps = 32 / sw;
  return ((long)g.N * g.H * spr) % rps == 0 ? ws : 0;
}

// stride-2 slots per output row: Q itself (4/8/16/32), else the next of 8/16/32 above it
// (0: unsupported); a step is 32/slots whole output rows
int w3_s2_slots(const ConvGeom& g) {
  if (g.Q == 4 || g.Q == 8 || g.Q == 16 || g.Q == 32) return g.Q;
  // (w3_pad_ws of the output-sized stride-1 geometry: honours SDX_W3_PAD)
  if (g.Q < 5 || g.Q > 32 || !w3_pad_ws(ConvGeom{g.N, g.P, g.Q, g.C, g.K, 3, 3, g.P, g.Q, 1, 1})) return 0;
  const int sq = g.Q <= 8 ? 8 : g.Q <= 16 ? 16 : 32;
  return ((long)g.N * g.P) % (32 / sq) == 0 ? sq : 0;
}

}  // namespace

bool wgrad3x3_supported(const ConvGeom& g) {
  static const bool s2_on = [] {   // SDX_W3_S2=0: stride-2 3x3 wgrads on the generic kernel
    const char* e = getenv("SDX_W3_S2");
    return e == nullptr || atoi(e) != 0;
  }();
  const bool q_ok = g.Q == 4 || g.Q == 8 || g.Q == 16 || g.Q == 32;
  if (g.stride == 2 && s2_on && g.R == 3 && g.S == 3 && g.pad == 1 && g.P == g.Q && g.H == 2 * g.P &&
      g.W == 2 * g.Q && g.C % 64 == 0 && g.K % 64 == 0 && !q_ok && w3_s2_slots(g) > 0)
    return true;   // padded output rows
  const bool geo = g.stride == 1 ? (g.P == g.H && g.Q == g.W)
                                 : (s2_on && g.stride == 2 && g.H == 2 * g.P && g.W == 2 * g.Q);
  const bool base = g.R == 3 && g.S == 3 && g.pad == 1 && g.P == g.Q && geo && g.C % 64 == 0 && g.K % 64 == 0;
  if (base && g.stride == 1 && g.H == g.W && w3_pad_ws(g) > 0) return true;   // padded slots
  return base && q_ok && ((long)g.N * g.P * g.Q) % 32 == 0;
}

int wgrad3x3_tiles(const ConvGeom& g) { return (g.K / 64) * (g.C / 64); }

int wgrad3x3_steps(const ConvGeom& g) {
  const int ws = (g.stride == 1 && g.H == g.W) ? w3_pad_ws(g) : 0;
  if (ws > 0) {   // segments of the padded-slot kernel / segments per step
    const int sw = ws < 32 ? ws : 32;
    return (int)((long)g.N * g.H * (ws / sw) / (32 / sw));
  }
  if (g.stride == 2 && !(g.Q == 4 || g.Q == 8 || g.Q == 16 || g.Q == 32)) {   // padded rows
    const int sq = w3_s2_slots(g);
    return (int)((long)g.N * g.P / (32 / sq));
  }
  return (int)((long)g.N * g.P * g.Q / 32);
}

hipError_t launch_wgrad3x3(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int splits,
                           int accumulate, hipStream_t s) {
  if (!wgrad3x3_supported(g) || splits < 1) return hipErrorInvalidValue;
  W3Params p{};
  p.dy = (const uint16_t*)dy;
  p.x = (const uint16_t*)x;
  p.K = g.K;
  p.C = g.C;
  p.steps_total = wgrad3x3_steps(g);
  p.steps_per_split = (p.steps_total + splits - 1) / splits;
  p.splits = (p.steps_total + p.steps_per_split - 1) / p.steps_per_split;
  p.k_tiles = g.K / 64;
  p.c_tiles = g.C / 64;
  // one split straight into dW (unless accumulating into it)
  const bool direct = p.splits == 1 && !accumulate;
  if (!direct && partial == nullptr) return hipErrorInvalidValue;
  p.part = direct ? dw : partial;
  const dim3 grid(p.k_tiles * p.c_tiles * p.splits), block(W3_NT);
  p.h = g.H;
  p.w = g.W;
  const int ws = (g.stride == 1 && g.H == g.W) ? w3_pad_ws(g) : 0;
  if (ws > 0) {
    switch (ws) {
      case 8: hipLaunchKernelGGL(wgrad3x3_pad_kernel<8>, grid, block, 0, s, p); break;
      case 16: hipLaunchKernelGGL(wgrad3x3_pad_kernel<16>, grid, block, 0, s, p); break;
      case 32: hipLaunchKernelGGL(wgrad3x3_pad_kernel<32>, grid, block, 0, s, p); break;
      default: hipLaunchKernelGGL(wgrad3x3_pad_kernel<64>, grid, block, 0, s, p); break;
    }
  } else if (g.stride == 2) {
    const bool pad = !(g.Q == 4 || g.Q == 8 || g.Q == 16 || g.Q == 32);
    const int sq = w3_s2_slots(g);
    if (pad) {
      switch (sq) {
        case 8: hipLaunchKernelGGL((wgrad3x3_s2_kernel<8, true>), grid, block, 0, s, p); break;
        case 16: hipLaunchKernelGGL((wgrad3x3_s2_kernel<16, true>), grid, block, 0, s, p); break;
        default: hipLaunchKernelGGL((wgrad3x3_s2_kernel<32, true>), grid, block, 0, s, p); break;
      }
    } else {
      switch (g.Q) {
        case 4: hipLaunchKernelGGL((wgrad3x3_s2_kernel<4, false>), grid, block, 0, s, p); break;
        case 8: hipLaunchKernelGGL((wgrad3x3_s2_kernel<8, false>), grid, block, 0, s, p); break;
        case 16: hipLaunchKernelGGL((wgrad3x3_s2_kernel<16, false>), grid, block, 0, s, p); break;
        default: hipLaunchKernelGGL((wgrad3x3_s2_kernel<32, false>), grid, block, 0, s, p); break;
      }
    }
  } else {
    switch (g.W) {
      case 4: hipLaunchKernelGGL(wgrad3x3_kernel<4>, grid, block, 0, s, p); break;
      case 8: hipLaunchKernelGGL(wgrad3x3_kernel<8>, grid, block, 0, s, p); break;
      case 16: hipLaunchKernelGGL(wgrad3x3_kernel<16>, grid, block, 0, s, p); break;
      default: hipLaunchKernelGGL(wgrad3x3_kernel<32>, grid, block, 0, s, p); break;
    }
  }
  SDX_LAUNCH_CHECK();
  if (direct) return hipSuccess;
  return launch_splitk_reduce(partial, p.splits, (long)g.K * 9 * g.C / 4, dw, accumulate, s);
}
