// Implicit-GEMM convolution on gfx950 MFMA (bf16 in, fp32 accumulate), NHWC.
//
// One kernel template implements the three convolution GEMMs of training
// (reference model: networks/resnet_big.py:38-118, every nn.Conv2d of the encoder):
//
//   FWD   y[m=(n,p,q)][co]        = Σ_{k=(r,s,ci)} x[n][p·st−pad+r][q·st−pad+s][ci] · W[co][r][s][ci]
//   DGRAD dx[m=(n,h,w)][ci]       = Σ_{k=(r,s,co)} dy[n][(h+pad−r)/st][(w+pad−s)/st][co] · Wt[ci][r][s][co]
//   WGRAD dW[co][j=(r,s,ci)]     += Σ_{kk=(n,p,q)} dy[kk][co] · x[n][p·st−pad+r][q·st−pad+s][ci]   (split-K)
//
// Tiles: BM x BN output per 256-thread workgroup (4 waves, each a 64x64 sub-tile of
// 4x4 v_mfma_f32_16x16x32_bf16 accumulators), BK = 64. Operands are register-staged
// (16-byte global loads, im2col gather with zero padding done in the address
// computation) into a double-buffered LDS image: the next K-tile's global loads are
// issued before the current tile's MFMAs and written to the other LDS buffer after them
// (one barrier per K-tile). "K-inner" images ([rows][64] bf16, 128-B rows, XOR-swizzled
// by row) are read with ds_read_b128; "K-outer" images ([64][cols], used by WGRAD whose
// operands are both strided along K) are read with ds_read_b64_tr_b16 transposed reads.
//
// Epilogues: FWD stores bf16 y through an LDS transpose (coalesced 16-B row stores) and
// emits per-channel BatchNorm statistics of the stored values (per-tile Σy and Σy², one
// slab row per M-tile, reduced in fp64 by bn_stats_reduce — no atomics here);
// DGRAD stores bf16 dx; WGRAD adds fp32 partial sums into dW with atomics.
// Block→tile order is XCD-aware (all N-tiles of one M-tile on one XCD's L2).
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int BK = 64;

struct IgemmParams {
  ConvGeom g;
  const uint16_t* a;   // FWD: x, DGRAD: dy, WGRAD: dy
  const uint16_t* b;   // FWD: W [K][R][S][C], DGRAD: Wt [C][R][S][K], WGRAD: x
  void* out;           // FWD/DGRAD: bf16 [M][Ncol]; WGRAD: fp32 [K][R*S*C]
  float* stats;        // FWD: [m_tiles][2][Ncol] (Σy, Σy²) or nullptr
  int M, Ncol, Kdim;
  int m_tiles, n_tiles, splits, k_per_split;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// K-inner image: [rows][BK] bf16, 128-B rows; 16-B chunk swizzle conflict-free for 16 rows.
__device__ __forceinline__ int kin_off(int row, int ch) {
  return row * (BK * 2) + ((ch ^ ((row >> 1) & 7)) << 4);
}

// K-outer image: [BK][COLS] bf16; chunk swizzle keeps the transposed reads of a 32-lane
// half (8 rows x 2 chunks) on distinct banks.
template <int COLS>
__device__ __forceinline__ int kout_off(int row, int ch) {
  int sw;
  if (COLS >= 128) sw = ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  else sw = (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
  return row * (COLS * 2) + ((ch ^ sw) << 4);
}

__device__ __forceinline__ uint4 ld16(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }

template <int MODE, int BM, int BN>
struct Tile {
  static constexpr bool A_KIN = MODE != MODE_WGRAD;
  static constexpr bool B_KIN = MODE != MODE_WGRAD;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  // chunks (16 B) per thread
  static constexpr int A_CH = BM * BK / 8 / 256;
  static constexpr int B_CH = BN * BK / 8 / 256;
};

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256, 2) void igemm_kernel(IgemmParams p) {
  using T = Tile<MODE, BM, BN>;
  constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == 4, "4 waves of 64x64");
  constexpr int LDS = 2 * T::STAGE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const ConvGeom& g = p.g;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int wm = wv / WN, wn = wv % WN;

  // ---- tile coordinates (XCD-aware) ----
  const int nwg = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nwg);
  int split = 0, tile = lin;
  if (MODE == MODE_WGRAD) { split = lin % p.splits; tile = lin / p.splits; }
  const int mt = tile / p.n_tiles, nt = tile % p.n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  int k_begin = 0, k_end = p.Kdim;
  if (MODE == MODE_WGRAD) {
    k_begin = split * p.k_per_split;
    k_end = min(p.Kdim, k_begin + p.k_per_split);
  }
  const int nk = (k_end - k_begin + BK - 1) / BK;

  // ---- per-thread loader state ----
  // K-inner operands: thread owns chunk column ch = tid % 8 and rows tid/8 + 32*i.
  const int kin_ch = tid & 7;
  const int kin_row0 = tid >> 3;
  // FWD/DGRAD A gather rows
  int a_n[T::A_CH], a_y[T::A_CH], a_x[T::A_CH];
  if (MODE != MODE_WGRAD) {
    const int hw_out = (MODE == MODE_FWD) ? g.P * g.Q : g.H * g.W;
    const int wdim = (MODE == MODE_FWD) ? g.Q : g.W;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) {
      const int m = m0 + kin_row0 + 32 * i;
      if (m < p.M) {
        const int n = m / hw_out, rem = m - n * hw_out;
        const int yy = rem / wdim, xx = rem - yy * wdim;
        a_n[i] = n;
        if (MODE == MODE_FWD) { a_y[i] = yy * g.stride - g.pad; a_x[i] = xx * g.stride - g.pad; }
        else { a_y[i] = yy + g.pad; a_x[i] = xx + g.pad; }
      } else {
        a_n[i] = -1; a_y[i] = 0; a_x[i] = 0;
      }
    }
  }
  // WGRAD: K-outer images. A: [BK pixels][BM couts], B: [BK pixels][BN (r,s,ci)].
  constexpr int A_CPR = BM / 8, B_CPR = BN / 8;  // chunks per row
  int wb_r = 0, wb_s = 0, wb_c = 0;
  bool wb_ok = false;
  if (MODE == MODE_WGRAD) {
    const int j0 = n0 + (tid % B_CPR) * 8;
    wb_ok = j0 < p.Ncol;
    const int jj = wb_ok ? j0 : 0;
    wb_c = jj % g.C;
    const int rs = jj / g.C;
    wb_r = rs / g.S;
    wb_s = rs - wb_r * g.S;
  }

  uint4 ra[T::A_CH], rb[T::B_CH];

  auto load_tile = [&](int k0) {
    if (MODE == MODE_FWD || MODE == MODE_DGRAD) {
      // A: gather 8 consecutive k (same (r,s), 8 channels) for each owned row
      const int k = k0 + kin_ch * 8;
      const int cdim = (MODE == MODE_FWD) ? g.C : g.K;
      const bool kok = k < k_end;
      const int cc = k % cdim;
      const int rs = k / cdim;
      const int r = rs / g.S, s = rs - (rs / g.S) * g.S;
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kok && a_n[i] >= 0) {
          if (MODE == MODE_FWD) {
            const int yy = a_y[i] + r, xx = a_x[i] + s;
            if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W)
              v = ld16(p.a + (((size_t)a_n[i] * g.H + yy) * g.W + xx) * g.C + cc);
          } else {
            int ty = a_y[i] - r, tx = a_x[i] - s;
            if (ty >= 0 && tx >= 0) {
              bool ok = true;
              if (g.stride != 1) {
                ok = (ty % g.stride == 0) && (tx % g.stride == 0);
                ty /= g.stride;
                tx /= g.stride;
              }
              if (ok && ty < g.P && tx < g.Q)
                v = ld16(p.a + (((size_t)a_n[i] * g.P + ty) * g.Q + tx) * g.K + cc);
            }
          }
        }
        ra[i] = v;
      }
      // B: weights [Ncol][Kdim] K-contiguous
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int col = n0 + kin_row0 + 32 * i;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kok && col < p.Ncol) v = ld16(p.b + (size_t)col * p.Kdim + k);
        rb[i] = v;
      }
    } else {
      // WGRAD A: dy rows (pixels) x BM couts
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int e = tid + 256 * i;
        const int row = e / A_CPR, ch = e % A_CPR;
        const int kk = k0 + row, co = m0 + ch * 8;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (kk < k_end && co < p.M) v = ld16(p.a + (size_t)kk * g.K + co);
        ra[i] = v;
      }
      // WGRAD B: im2col(x) rows (pixels) x BN (r,s,ci); the column chunk is fixed per thread
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int e = tid + 256 * i;
        const int row = e / B_CPR;
        const int kk = k0 + row;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (wb_ok && kk < k_end) {
          const int pq = g.P * g.Q;
          const int n = kk / pq, rem = kk - n * pq;
          const int pp = rem / g.Q, qq = rem - pp * g.Q;
          const int yy = pp * g.stride - g.pad + wb_r, xx = qq * g.stride - g.pad + wb_s;
          if (yy >= 0 && yy < g.H && xx >= 0 && xx < g.W)
            v = ld16(p.b + (((size_t)n * g.H + yy) * g.W + xx) * g.C + wb_c);
        }
        rb[i] = v;
      }
    }
  };

  auto store_tile = [&](int buf) {
    unsigned char* sa = smem + buf * T::STAGE;
    unsigned char* sb = sa + T::A_BYTES;
    if (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i)
        *reinterpret_cast<uint4*>(sa + kin_off(kin_row0 + 32 * i, kin_ch)) = ra[i];
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i)
        *reinterpret_cast<uint4*>(sb + kin_off(kin_row0 + 32 * i, kin_ch)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int e = tid + 256 * i;
        *reinterpret_cast<uint4*>(sa + kout_off<BM>(e / A_CPR, e % A_CPR)) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int e = tid + 256 * i;
        *reinterpret_cast<uint4*>(sb + kout_off<BN>(e / B_CPR, e % B_CPR)) = rb[i];
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment readers
  auto frag_kin = [&](const unsigned char* img, int row, int u) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(img + kin_off(row, 4 * u + h));
  };
  auto frag_kout = [&](const unsigned char* img, int col0, int u, auto cols_tag) -> bf16x8 {
    constexpr int COLS = decltype(cols_tag)::value;
    const int q = c >> 2, pp = c & 3;
    const int col = col0 + 4 * pp;            // this lane supplies columns col..col+3
    const int ch = col >> 3, half = (col & 7) * 2;
    const int r0 = 32 * u + 8 * h + q;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4*)(img + kout_off<COLS>(r0, ch) + half));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4*)(img + kout_off<COLS>(r0 + 4, ch) + half));
    bf16x8 f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  };

  if (nk > 0) {
    load_tile(k_begin);
    store_tile(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_tile(k_begin + (kt + 1) * BK);
    const unsigned char* sa = smem + buf * T::STAGE;
    const unsigned char* sb = sa + T::A_BYTES;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (T::A_KIN) af[i] = frag_kin(sa, wm * 64 + 16 * i + c, u);
        else af[i] = frag_kout(sa, wm * 64 + 16 * i, u, std::integral_constant<int, BM>{});
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (T::B_KIN) bfr[j] = frag_kin(sb, wn * 64 + 16 * j + c, u);
        else bfr[j] = frag_kout(sb, wn * 64 + 16 * j, u, std::integral_constant<int, BN>{});
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_tile(buf ^ 1);
    __syncthreads();
  }

  // ---------------------------------- epilogues ----------------------------------
  // acc[i][j][r] = C[m0 + wm*64 + 16i + 4h + r][n0 + wn*64 + 16j + c]
  if (MODE == MODE_WGRAD) {
    float* out = reinterpret_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + 16 * j + c;
        if (col >= p.Ncol) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + 16 * i + 4 * h + r;
          if (row < p.M) atomicAdd(out + (size_t)row * p.Ncol + col, acc[i][j][r]);
        }
      }
    return;
  }

  // bf16 rounding (stats describe the stored tensor)
  uint16_t ov[4][4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ov[i][j][r] = f2bf(acc[i][j][r]);

  // stage the C tile through LDS ([BM][BN] bf16, padded rows) for coalesced stores
  constexpr int CRS = BN * 2 + 16;
  static_assert(BM * CRS <= LDS, "C tile must fit the staging LDS");
  uint16_t* ctile = reinterpret_cast<uint16_t*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ctile[((wm * 64 + 16 * i + 4 * h + r) * CRS) / 2 + wn * 64 + 16 * j + c] = ov[i][j][r];
  __syncthreads();
  {
    uint16_t* out = reinterpret_cast<uint16_t*>(p.out);
    constexpr int CPR = BN / 8;
    for (int e = tid; e < BM * CPR; e += 256) {
      const int row = e / CPR, ch = e % CPR;
      const int m = m0 + row, col = n0 + ch * 8;
      if (m < p.M && col < p.Ncol) {
        const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const unsigned char*>(ctile) + row * CRS + ch * 16);
        *reinterpret_cast<uint4*>(out + (size_t)m * p.Ncol + col) = v;
      }
    }
  }

  if (MODE == MODE_FWD && p.stats != nullptr) {
    // per-column (Σy, Σy²) over this tile's valid rows, from the rounded (stored) values;
    // one slab row per M-tile, reduced in fp64 by bn_stats_reduce (no atomics here).
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [WM][2][BN]
    const int valid_rows = min(BM, p.M - m0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * 64 + 16 * i + 4 * h + r;
          const float v = (row < valid_rows) ? bf2f(ov[i][j][r]) : 0.f;
          s1 += v;
          s2 += v * v;
        }
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (h == 0) {
        red[(wm * 2 + 0) * BN + wn * 64 + 16 * j + c] = s1;
        red[(wm * 2 + 1) * BN + wn * 64 + 16 * j + c] = s2;
      }
    }
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += 256) {
      const int which = e / BN, col = e % BN;
      float s = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WM; ++w2) s += red[(w2 * 2 + which) * BN + col];
      if (n0 + col < p.Ncol) p.stats[((size_t)mt * 2 + which) * p.Ncol + n0 + col] = s;
    }
  }
}

template <int MODE, int BM, int BN>
hipError_t launch_cfg(IgemmParams p, hipStream_t s) {
  p.m_tiles = (p.M + BM - 1) / BM;
  p.n_tiles = (p.Ncol + BN - 1) / BN;
  const int grid = p.m_tiles * p.n_tiles * (MODE == MODE_WGRAD ? p.splits : 1);
  hipLaunchKernelGGL((igemm_kernel<MODE, BM, BN>), dim3(grid), dim3(256), 0, s, p);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

template <int MODE>
hipError_t launch_any(IgemmParams p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<MODE, 128, 128>(p, s);
    case 1: return launch_cfg<MODE, 256, 64>(p, s);
    case 2: return launch_cfg<MODE, 64, 256>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int igemm_tile_m(int cfg) { return cfg == 0 ? 128 : cfg == 1 ? 256 : 64; }
int igemm_tile_n(int cfg) { return cfg == 0 ? 128 : cfg == 1 ? 64 : 256; }

hipError_t launch_conv_fwd(const ConvGeom& g, const void* x, const void* w, void* y, float* stats, int cfg,
                           hipStream_t s) {
  IgemmParams p{};
  p.g = g;
  p.a = (const uint16_t*)x;
  p.b = (const uint16_t*)w;
  p.out = y;
  p.stats = stats;
  p.M = g.N * g.P * g.Q;
  p.Ncol = g.K;
  p.Kdim = g.R * g.S * g.C;
  return launch_any<MODE_FWD>(p, cfg, s);
}

hipError_t launch_conv_dgrad(const ConvGeom& g, const void* dy, const void* wt, void* dx, int cfg,
                             hipStream_t s) {
  IgemmParams p{};
  p.g = g;
  p.a = (const uint16_t*)dy;
  p.b = (const uint16_t*)wt;
  p.out = dx;
  p.M = g.N * g.H * g.W;
  p.Ncol = g.C;
  p.Kdim = g.R * g.S * g.K;
  return launch_any<MODE_DGRAD>(p, cfg, s);
}

hipError_t launch_conv_wgrad(const ConvGeom& g, const void* dy, const void* x, float* dw, int cfg, int splits,
                             hipStream_t s) {
  IgemmParams p{};
  p.g = g;
  p.a = (const uint16_t*)dy;
  p.b = (const uint16_t*)x;
  p.out = dw;
  p.M = g.K;
  p.Ncol = g.R * g.S * g.C;
  p.Kdim = g.N * g.P * g.Q;
  if (splits < 1) splits = 1;
  int per = (p.Kdim + splits - 1) / splits;
  per = ((per + BK - 1) / BK) * BK;
  p.k_per_split = per;
  p.splits = (p.Kdim + per - 1) / per;
  return launch_any<MODE_WGRAD>(p, cfg, s);
}
