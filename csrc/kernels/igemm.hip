// Implicit-GEMM convolution on gfx950 MFMA (bf16 in, fp32 accumulate), NHWC.
//
// One kernel template implements the three convolution GEMMs of training
// (reference model: networks/resnet_big.py:38-118, every nn.Conv2d of the encoder):
//
//   FWD   y[m=(n,p,q)][co]    = Σ_{k=(r,s,ci)} x[n][p·st−pad+r][q·st−pad+s][ci] · W[co][r][s][ci]
//   DGRAD dx[m=(n,h,w)][ci]   = Σ_{k=(r,s,co)} dy[n][(h+pad−r)/st][(w+pad−s)/st][co] · Wt[ci][r][s][co]
//   WGRAD dW[co][j=(r,s,ci)]  = Σ_{kk=(n,p,q)} dy[kk][co] · x[n][p·st−pad+r][q·st−pad+s][ci]   (split-K)
//
// Strided DGRAD is decomposed into st² sub-pixel classes (h ≡ ph, w ≡ pw mod st): within
// a class only the taps r ≡ ph+pad (mod st) contribute and (h+pad−r)/st is exact, so every
// MFMA does useful work (a plain masked gather wastes 3/4 of it at stride 2).
//
// Tiles: BM x BN output per 256-thread workgroup (4 waves, each a 64x64 sub-tile of 4x4
// v_mfma_f32_16x16x32_bf16 accumulators), BK = 64. Operands are register-staged (16-byte
// global loads, im2col gather + zero padding in 32-bit address math, k decoded
// incrementally) into a double-buffered LDS image: the next K-tile's loads are issued
// before the current tile's MFMAs and written to the other buffer after them (one barrier
// per K-tile). "K-inner" images ([rows][64] bf16, XOR-swizzled 128-B rows) are read with
// ds_read_b128; "K-outer" images ([64][cols], WGRAD, both operands strided along K) with
// ds_read_b64_tr_b16 transposed reads.
//
// The MFMA is issued as D = Bᵀ·Aᵀ, so each lane's accumulator holds FOUR CONSECUTIVE OUTPUT
// COLUMNS of one output row: the epilogues write 8-byte (bf16) / 16-byte (fp32) pieces.
// FWD/DGRAD store bf16 through an LDS-staged tile as whole 16-B row chunks (optionally to
// remapped rows: DGRAD sub-pixel classes); FWD also emits per-channel BatchNorm statistics
// (per-M-tile Σy, Σy² of the stored values → one slab row, reduced in fp64 by
// bn_stats_reduce). WGRAD writes an fp32 partial slab per K-split (deterministic; reduced
// by igemm_splitk_reduce), never atomics. Block→tile order is XCD-aware.
#include <atomic>

#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int BK = 64;
#ifndef SDX_PRIO_HALF
#define SDX_PRIO_HALF 1
#endif
#ifndef SDX_W1_ABL
#define SDX_W1_ABL 0   // DEPTH 6: honour the SDX_IGEMM_ABLATE bits (diagnostic builds only)
#endif
#ifndef SDX_W1_SGB
#define SDX_W1_SGB 1   // DEPTH 6: sched_group_barrier interleave of the second half
#endif
#ifndef SDX_ADD_PRE
// DGRAD addend added to the fp32 accumulators before rounding when the launch asks for it
// (GemmEpi::add_pre, BN3 fold): without it the fold's small mean-removal addend is swamped
// by the bf16 rounding of the main term (profiles/bn3_fold_r2.txt)
#define SDX_ADD_PRE 1
#endif
#ifndef SDX_NT_LOAD
// non-temporal loads of the dgrad epilogue's read-once operands (addend, BN inputs): step
// 13.15 -> 13.05 ms on the same box (profiles/nt_store_r2.txt); 0 = cached loads
#define SDX_NT_LOAD 1
#endif
#ifndef SDX_NT_STORE
// non-temporal stores of the bf16 conv outputs (they are re-read only by later kernels):
// plain dgrad 2.69 -> 2.44 ms, fwd 2.53 -> 2.27 ms per step, step -2.5 % (same box,
// profiles/nt_store_r2.txt); 0 restores write-back stores
#define SDX_NT_STORE 1
#endif
#ifndef SDX_NT_STORE_DGRAD
// the DGRAD outputs' store hint on its own (they are re-read at once by the BN-backward
// passes, unlike most forward outputs); default: as SDX_NT_STORE
#define SDX_NT_STORE_DGRAD SDX_NT_STORE
#endif

// Diagnostic main-loop timeline (SDX_IGEMM_TRACE=1, tools/igemm_trace.py): lane 0 of waves 0
// and 4 of block 0 store s_memtime stamps (vector stores) at fixed events; row w of
// [2][kTraceSlots]: 0 kernel start, 1 loop start, 2 + 3·kt + {0: fragment reads + DMA issued,
// 1: after the load barrier, 2: MFMAs issued}, kTraceSlots-4 loop end, -3 epilogue staged,
// -2 end, -1 s_memrealtime at the end (100 MHz) with slot -5 the one at the start.
constexpr int kTraceSlots = 512;
__device__ unsigned long long g_igemm_trace[2 * kTraceSlots];

struct IgemmParams {
  ConvGeom g;
  const uint16_t* a;   // FWD: x, DGRAD: dy, WGRAD: dy
  const uint16_t* b;   // FWD: W [K][R][S][C], DGRAD: class taps of Wt [C][nr][ns][K], WGRAD: x
  void* out;           // FWD/DGRAD: bf16 rows of Ncol; WGRAD: fp32 partial slab [splits][M][Ncol]
  float* stats;        // FWD: [m_tiles][2][Ncol] (Σy, Σy²) or nullptr
  const uint16_t* addend;   // DGRAD: optional bf16 tensor (same layout as out) added in the epilogue
  // DGRAD: addend_sub = s > 1: the addend is COMPACT, [N][ceil(H/s)][ceil(W/s)][C], and is
  // added only at output pixels (h, w) with h % s == w % s == 0 (a strided 1x1 shortcut's
  // data gradient, which is zero everywhere else)
  int addend_sub;
  // optional fused BatchNorm+ReLU on the activation operand as it is loaded (FWD: A = x,
  // WGRAD: B = x): x' = max(x·in_scale[c] + in_shift[c], 0); padding taps stay exactly 0
  const float* in_scale;
  const float* in_shift;
  // diagnostic ablation (SDX_IGEMM_ABLATE bits, timing only — results are wrong):
  // 1 skip LDS stores, 2 skip global loads / LDS-DMA, 4 skip MFMAs, 8 skip the fragment
  // reads (DEPTH 6, builds with SDX_W1_ABL=1)
  int ablate;
  // log2(Q), log2(P*Q) when both are powers of two, else -1 (WGRAD pixel decode)
  int lq, lpq;
  // DGRAD addend ReLU bitmask (uint8, bit per element): addend element used iff its bit is set
  const uint8_t* addend_mask;
  // operand sizes in elements (bounds checks of the checked build)
  long a_elems, b_elems;
  // DGRAD, stride-1 1x1 (BN3 fold, K-concatenated): the reduction runs over g.K channels of
  // dy (rows of g.K) and then a2_ch channels of a2 (rows of a2_ch = g.K >> a2_sh, the same
  // pixels): [dy | a2]·[Wd ; Mx] in one GEMM. bias_pre: fp32 per-output-column bias added to
  // the accumulators before the bf16 rounding (the fold's Eᵀ·W3)
  const uint16_t* a2;
  int a2_ch, a2_sh;
  long a2_elems;
  const float* bias_pre;
  // DGRAD: fused BN-backward statistics of the stored output (BnBwdStat; bs.slab null = off)
  BnBwdStat bs;
  // FWD / DGRAD plain-GEMM epilogue (projection head, csrc/bindings/head_ops.cpp): optional
  // per-output-column fp32 bias and ReLU on the fp32 accumulators; out_f32 = fp32 output
  // rows stored straight from the accumulators (no bf16 rounding, no BN statistics)
  const float* bias;
  int relu, out_f32;
  int add_pre;   // GemmEpi::add_pre
  int trace;     // g_igemm_trace stamps (diagnostic)
  // FWD VAR 2 (GemmEpi::bn_scale): the block-output BatchNorm applied in the epilogue —
  // out = relu(bf16(y)·bn_sc + bn_sh + addend), its ReLU bits to mask_out (1 bit per element);
  // bn_rsc / bn_rsh (projection blocks): the addend is the shortcut's pre-BN output and gets
  // its own BatchNorm, addend·bn_rsc + bn_rsh (bn_apply residual mode 1)
  const float* bn_sc;
  const float* bn_sh;
  const float* bn_rsc;
  const float* bn_rsh;
  uint8_t* mask_out;
  // WGRAD block order: 1 split-major (SDX_WGRAD_ORDER, default), 0 tile-major
  int worder;
  int M, Ncol, Kdim;
  // FWD / DGRAD weight operand addressing: output column col, logical k = (kr, ks, kc) reads
  // b[col·b_row + b_t0 + kr·b_tr + ks·b_ts + kc]. FWD W [K][R][S][Cp] and stride-1 DGRAD Wt
  // [C][R][S][K] give b_row = Kdim and k itself; a strided DGRAD class reads its taps
  // r = r0 + st·kr, s = s0 + st·ks straight from the full Wt (no per-class weight copies)
  int b_row, b_t0, b_tr, b_ts;
  int m_tiles, n_tiles, splits, k_per_split;
  // DGRAD sub-pixel class: output rows h = st·h' + ph, taps r = r0 + st·ir (ir < nr)
  int ph, pw, Hc, Wc, r0, s0, nr, ns;
  // DGRAD, ncls > 1: all stride² sub-pixel classes in ONE launch. Block tiles interleave the
  // classes (tile t -> class t % ncls, its tile t / ncls < cls.tile_end = that class's tile
  // count); each block loads its class's fields over the per-class ones above (M, Kdim, b_t0,
  // m_tiles, bs.row0 included)
  struct Cls {
    int ph, pw, Hc, Wc, r0, s0, nr, ns, M, Kdim, b_t0, m_tiles, row0, tile_end;
  };
  int ncls;
  Cls cls[4];
  FastDiv div_pq, div_q;   // WGRAD pixel decode
  // DEPTH 7 / 8 (tap-reuse 3x3 fwd / stride-1 dgrad, launch_tap): the tile's input window —
  // its image rows plus a pad row / column on each side, the "halo" — is staged ONCE per
  // 64-channel chunk and all 9 taps read it at a uniform pixel offset. Halo pixel
  // (img, hy, hx) is LDS row img·t_is + hy·t_rs + hx (t_rs = W + 2); its 16-B chunk q sits at
  // q ^ ((hx + t_ky·hy) & 7), conflict-free fragment reads for every tap (see tap_halo_kb).
  // t_hp halo pixels = t_nhp 1-KiB LDS-DMA pieces; t_nch channel chunks; the tile's first
  // image row y0 within image n0. t_rw > 0: padded rows — an image row of W pixels is t_rw
  // (a power of two) virtual output rows, so a tile of whole rows exists when W does not divide
  // BM (56x56, 28x28: config 5); the t_rw − W padded rows compute garbage from neighbouring halo
  // pixels, are zeroed before the epilogue and never stored
  int t_rs, t_is, t_ky, t_hp, t_nhp, t_nch, t_imgs, t_rw;
};

// DEPTH 7 / 8 halo buffer size in KiB: the largest window a BM-row tile needs over the
// supported image widths (BM = 256: 4 images of 8x8 = 4·10·10 pixels = 50 KiB at 64
// channels; BM = 128: 8 images of 4x4 = 8·6·6 pixels = 36 KiB)
constexpr int tap_halo_kb(int bm) { return bm == 256 ? 50 : 36; }

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// K-inner image: [rows][BK] bf16, 128-B rows; 16-B chunk swizzle conflict-free for 16 rows.
__device__ __forceinline__ int kin_off(int row, int ch) {
  // XOR swizzle by row&7: conflict-free for the fragment ds_read_b128 lane groups, and an
  // 8-row x 128-B block stays one contiguous 1 KiB piece in which lane L of a
  // global_load_lds instruction always carries logical chunk (L&7)^(L>>3)
  return row * (BK * 2) + ((ch ^ (row & 7)) << 4);
}

// K-outer image: [BK][COLS] bf16; chunk swizzle keeps the transposed reads of a 32-lane
// half (8 rows x 2 chunks) on distinct banks.
template <int COLS>
__device__ __forceinline__ int kout_swz(int row) {
  if (COLS >= 128) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
}
template <int COLS>
__device__ __forceinline__ int kout_off(int row, int ch) {
  return row * (COLS * 2) + ((ch ^ kout_swz<COLS>(row)) << 4);
}

__device__ __forceinline__ uint4 ld16(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// 16 zero bytes in global memory: out-of-bounds operand chunks (padding taps, tail rows,
// K tail) load from here instead of being skipped, so every staging load is unconditional.
// A predicated load makes hipcc branch around it and drain the whole load queue
// (vmcnt(0)) before the LDS write, which defeats any prefetch depth.
__device__ __attribute__((aligned(16))) uint16_t g_zero16[8];
// g_zero16's address in an SGPR pair the compiler cannot rematerialise: otherwise it re-runs
// s_getpc + a GOT s_load + s_waitcnt lgkmcnt(0) before every zero-page select of the K loop
typedef const __attribute__((address_space(1))) uint16_t* gptr16;
__device__ __forceinline__ gptr16 opaque_zero() {
  gptr16 z = (gptr16)g_zero16;
  asm volatile("" : "+s"(z));
  return z;
}

// One 16-B LDS-DMA (global_load_lds_dwordx4). The source address goes through an empty asm
// that pins it in a VGPR pair: hipcc otherwise splits "ok ? row address : zero page" into
// two exec-masked branches, each with its own glds (the zero page through the scalar-base
// form), which doubles the DMA instructions and serialises them behind SALU exec juggling
// (seen in the .s of every LDS-DMA variant; issue cost ~1000 cycles per K-tile per wave).
__device__ __forceinline__ void glds16(gptr16 src, void* lds) {
  asm volatile("" : "+v"(src));
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// relu(x·s + t) on 8 packed bf16 channels (fp32 math, one rounding: same as bn_apply)
__device__ __forceinline__ uint4 bnrelu8(uint4 v, const float (&s)[8], const float (&t)[8]) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = fmaxf(__uint_as_float(w[q] << 16) * s[2 * q] + t[2 * q], 0.f);
    const float b = fmaxf(__uint_as_float(w[q] & 0xffff0000u) * s[2 * q + 1] + t[2 * q + 1], 0.f);
    w[q] = pack_bf2(a, b);
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt at their maxima); gfx9 encoding: vmcnt in
// bits [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}

// raw workgroup barrier: this wave's LDS reads complete first; LDS-DMA stays in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ReLU bitmask byte of 8 packed bf16 (bit q: element q > 0), as bn.hip's apply kernel
__device__ __forceinline__ uint32_t relu_bits8(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = w[q] & 0xffffu, hi = w[q] >> 16;
    b |= (uint32_t)((lo & 0x7fffu) != 0 && !(lo & 0x8000u)) << (2 * q);
    b |= (uint32_t)((hi & 0x7fffu) != 0 && !(hi & 0x8000u)) << (2 * q + 1);
  }
  return b;
}

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <int MODE, int BM, int BN, int NT>
struct Tile {
  static constexpr bool A_KIN = MODE != MODE_WGRAD;
  static constexpr bool B_KIN = MODE != MODE_WGRAD;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  // chunks (16 B) per thread
  static constexpr int A_CH = BM * BK / 8 / NT;
  static constexpr int B_CH = BN * BK / 8 / NT;
};

// DEPTH: 1 / 2 = register-staged operands, 1 or 2 K-tiles of prefetch; 3 = LDS-DMA
// (global_load_lds) staging of both K-inner operands (FWD / DGRAD without the BN prologue):
// no staging registers and no ds_write — the ds_write_b128 transfer path was the busiest
// LDS resource of the register-staged loop.
// VAR, DGRAD: 1 = fused BN-backward statistics epilogue (p.bs) — a separate variant so
// the plain dgrad keeps its register budget; 2 = the same, storing the gradient ReLU-masked.
// VAR, FWD: 2 = block-output BN-apply epilogue. ONE (LDS-DMA, reduction <= BK): a single
// K-tile needs no second LDS buffer; the smaller static LDS (one stage or the C tile) lets
// twice as many blocks share a CU, hiding the load -> MFMA -> store latency of these
// memory-bound 1x1 layer-1 GEMMs across blocks.
// Every configuration is held to 2 waves per SIMD (<= 256 VGPRs): 8-wave blocks one per CU,
// 4-wave blocks two per CU.
template <int MODE, int BM, int BN, int WM, int WN, int DEPTH, int VAR, bool ONE>
__global__ __launch_bounds__(64 * WM * WN, 2) void igemm_kernel(
    IgemmParams p_in) {
  // a block-local copy: a merged strided-dgrad launch overwrites its class's fields (uniform
  // values: SROA keeps the untouched fields in the kernel arguments)
  IgemmParams p = p_in;
  constexpr int NT = 64 * WM * WN;   // threads per block (4 or 8 waves)
  using T = Tile<MODE, BM, BN, NT>;
  constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert((WM * WN == 4 || WM * WN == 8) && TM >= 1 && TN >= 1, "4 or 8 waves");
  static_assert(T::A_CH >= 1 && T::B_CH >= 1, "tile too small for the thread count");
  constexpr int LDS_C = BM * (BN * 2 + 8);   // C-tile staging (epilogue)
  // DEPTH 7 / 8: 2 / 1 halo buffers, one junk KiB (LDS-DMA target of the unused halo issue
  // slots), a 3-buffer ring of weight tiles
  constexpr int LDS_TAP = (DEPTH == 7 ? 2 : 1) * tap_halo_kb(BM) * 1024 + 1024 + 3 * T::B_BYTES;
  constexpr int LDS = ONE ? (T::STAGE > LDS_C ? T::STAGE : LDS_C)
                          : DEPTH >= 7 ? LDS_TAP : (DEPTH == 6 ? 3 : 2) * T::STAGE;
  static_assert(!ONE || DEPTH == 3, "single-stage variant is LDS-DMA only");
  static_assert(DEPTH < 4 || MODE != MODE_WGRAD, "LDS-DMA ring is FWD/DGRAD only");
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS];

  const ConvGeom& g = p.g;
  const gptr16 zp = opaque_zero();
  // the address-space cast keeps these global_load (the opaque zero pointer is generic: a
  // select with it would otherwise become a flat load, counted by lgkmcnt as well)
  auto ld16_or_zero = [&](const uint16_t* q, bool ok) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)(ok ? (gptr16)q : zp);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  // read-once epilogue operands (addend, BN input): optionally non-temporal
  auto ld16_stream = [&](const uint16_t* q, bool ok) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const auto* ptr = (const __attribute__((address_space(1))) u32x4*)(ok ? (gptr16)q : zp);
    u32x4 v;
    if constexpr (SDX_NT_LOAD != 0) v = __builtin_nontemporal_load(ptr);
    else v = *ptr;
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int wm = wv / WN, wn = wv % WN;
  const bool trace_on = p.trace && blockIdx.x == 0 && lane == 0 && (wv == 0 || wv == 4);
  auto stamp = [&](int slot) {
    if (trace_on) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      __hip_atomic_store(&g_igemm_trace[(wv == 4) * kTraceSlots + slot], t, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  if (trace_on)
    __hip_atomic_store(&g_igemm_trace[(wv == 4) * kTraceSlots + kTraceSlots - 5], __builtin_amdgcn_s_memrealtime(),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(0);

  // ---- tile coordinates (XCD-aware) ----
  const int nwg = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nwg);
  int split = 0, tile = lin;
  if (MODE == MODE_WGRAD) {
    // split-major (default): the blocks an XCD runs together are ALL output tiles of a few
    // K-splits, so every tile re-reads the same dy / x pixel rows from that XCD's L2
    // (tile-major put one tile's splits together: disjoint K ranges, no L2 reuse)
    const int nt_all = p.m_tiles * p.n_tiles;
    if (p.worder) { tile = lin % nt_all; split = lin / nt_all; }
    else { split = lin % p.splits; tile = lin / p.splits; }
  }
  if constexpr (MODE == MODE_DGRAD) {
    if (p_in.ncls > 1) {
      // classes interleaved tile by tile: the XCD-aware order gives every XCD an equal share
      // of each class (class-major order put a stride-2 1x1 dgrad's only non-empty class on
      // two XCDs: 2x slower)
      const int cid = tile % p_in.ncls;
      tile /= p_in.ncls;
      const IgemmParams::Cls& cd = p_in.cls[cid];
      if (tile >= cd.tile_end) return;   // this class has fewer tiles than the largest
      p.ph = cd.ph; p.pw = cd.pw; p.Hc = cd.Hc; p.Wc = cd.Wc; p.r0 = cd.r0; p.s0 = cd.s0;
      p.nr = cd.nr; p.ns = cd.ns; p.M = cd.M; p.Kdim = cd.Kdim; p.b_t0 = cd.b_t0;
      p.m_tiles = cd.m_tiles; p.bs.row0 = cd.row0;
    }
  }
  const int mt = tile / p.n_tiles, nt = tile % p.n_tiles;
  const int m0 = mt * BM, n0 = nt * BN;
  int k_begin = 0, k_end = p.Kdim;
  if (MODE == MODE_WGRAD) {
    k_begin = split * p.k_per_split;
    k_end = min(p.Kdim, k_begin + p.k_per_split);
  }
  const int nk = k_end > k_begin ? (k_end - k_begin + BK - 1) / BK : 0;

  // ---- per-thread loader state (32-bit address math: tensors < 2^31 elements) ----
  // K-inner operands. Register staging: thread owns chunk column ch = tid % 8 and rows
  // tid/8 + (NT/8)*i. LDS-DMA: instruction i of wave w fills rows 8*(w*CH + i) .. +7 (1 KiB),
  // lane L row +L/8 at physical chunk L%8, i.e. logical chunk (L&7)^(L>>3).
  constexpr bool GL = DEPTH >= 3;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int kin_ch = GL ? ((lane & 7) ^ ((lane >> 3) & 7)) : (tid & 7);
  const int kin_row0 = tid >> 3;
  auto a_row = [&](int i) { return GL ? 8 * (wvu * T::A_CH + i) + (lane >> 3) : kin_row0 + (NT / 8) * i; };
  auto b_row = [&](int i) { return GL ? 8 * (wvu * T::B_CH + i) + (lane >> 3) : kin_row0 + (NT / 8) * i; };
  // VAR, WGRAD: bit 0 = 1x1 stride-1 unpadded filter (plain GEMM operand addressing, no
  // pixel decode or bounds tests), bit 1 = fused BN+ReLU prologue on x (p.in_scale). Each
  // is its own instantiation: the generic loader's address math and the prologue's
  // registers otherwise sit in every wgrad main loop (VALU-bound: ~6-10 VALU per MFMA).
  constexpr bool W1X1 = MODE == MODE_WGRAD && (VAR & 1);
  constexpr bool WPRO = MODE == MODE_WGRAD && (VAR & 2);
  const bool is1x1 = (MODE == MODE_WGRAD) ? W1X1 : (g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0);
  // A rows: element offset of the row base, and its spatial origin (FWD: top-left input
  // tap; DGRAD: dy coordinate of tap (r0, s0))
  int a_base[T::A_CH], a_y[T::A_CH], a_x[T::A_CH];
  int a_rb[T::A_CH];   // LDS-DMA path: row base incl. its spatial origin (0 for rows past M)
  int b_off[T::B_CH];
  // k decode of this thread's chunk: k = kc + cdim*(ks + ns*kr)
  int kc = 0, ks = 0, kr = 0;
  const int cdim = (MODE == MODE_FWD) ? g.C : g.K + p.a2_ch;
  const int tap_s = (MODE == MODE_DGRAD) ? p.ns : g.S;
  if (MODE != MODE_WGRAD) {
    const int hw_out = (MODE == MODE_FWD) ? g.P * g.Q : p.Hc * p.Wc;
    const int wdim = (MODE == MODE_FWD) ? g.Q : p.Wc;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) {
      const int m = m0 + a_row(i);
      if (m < p.M) {
        const int n = m / hw_out, rem = m - n * hw_out;
        const int yy = rem / wdim, xx = rem - yy * wdim;
        if (MODE == MODE_FWD) {
          a_y[i] = yy * g.stride - g.pad;
          a_x[i] = xx * g.stride - g.pad;
          a_base[i] = ((n * g.H + a_y[i]) * g.W + a_x[i]) * g.C;
        } else {
          // (h + pad − r0) is a multiple of st by construction of the class
          a_y[i] = (yy * g.stride + p.ph + g.pad - p.r0) / g.stride;
          a_x[i] = (xx * g.stride + p.pw + g.pad - p.s0) / g.stride;
          a_base[i] = n * g.P * g.Q * g.K;
        }
      } else {
        a_y[i] = -(1 << 28);   // fails every bounds test
        a_x[i] = -(1 << 28);
        a_base[i] = 0;
      }
    }
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) {
      const bool row_ok = a_y[i] > -(1 << 27);
      a_rb[i] = !row_ok ? 0 : (MODE == MODE_FWD ? a_base[i] : a_base[i] + (a_y[i] * g.Q + a_x[i]) * g.K);
    }
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i) {
      const int col = n0 + b_row(i);
      b_off[i] = col < p.Ncol ? col * p.b_row : -1;
    }
    const int k = k_begin + kin_ch * 8;
    kc = k % cdim;
    const int rs = k / cdim;
    kr = rs / tap_s;
    ks = rs - kr * tap_s;
  }
  // Uniform-tap fast path of the LDS-DMA loader: when the channel dim is a multiple of BK
  // every K-tile lies inside one filter tap, so the tap (and the channel base) is
  // wave-uniform: per-row validity over all taps is precomputed as a bitmask and a chunk
  // address is row base + uniform tap offset + lane constant (no per-chunk multiplies).
  const int taps = (MODE == MODE_FWD) ? g.R * g.S : p.nr * p.ns;
  // (always on in DEPTH 6, whose host routing guarantees cdim % BK == 0 and taps <= 32: it
  // halves the address VALU of the DMA issue, which is interleaved with the MFMAs there)
  const bool fast_taps = DEPTH == 6 && MODE != MODE_WGRAD;
  constexpr int FCH = (GL && MODE != MODE_WGRAD) ? T::A_CH : 1;
  unsigned vmask[FCH];
  int rbase[FCH];
  int u_c0 = 0, u_ks = 0, u_kr = 0;
  if (fast_taps) {
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      unsigned mbits = 0;
      const bool row_ok = a_y[i] > -(1 << 27);
      const int nrr = (MODE == MODE_FWD) ? g.R : p.nr;
      for (int r = 0; r < nrr; ++r)
        for (int q = 0; q < tap_s; ++q) {
          bool v;
          if (MODE == MODE_FWD)
            v = (unsigned)(a_y[i] + r) < (unsigned)g.H && (unsigned)(a_x[i] + q) < (unsigned)g.W;
          else
            v = (unsigned)(a_y[i] - r) < (unsigned)g.P && (unsigned)(a_x[i] - q) < (unsigned)g.Q;
          if (row_ok && v) mbits |= 1u << (r * tap_s + q);
        }
      vmask[i] = mbits;
      rbase[i] = !row_ok ? 0
                 : (MODE == MODE_FWD ? a_base[i] : a_base[i] + (a_y[i] * g.Q + a_x[i]) * g.K);
    }
  }
  // output pixel index -> (image, row, col): shifts when P and Q are powers of two
  // (every ResNet stage at 32x32 / 224x224-derived sizes), magic-number division otherwise
  auto pix_decode = [&](int kk, int& n, int& pp, int& qq) {
    if (p.lq >= 0) {
      n = kk >> p.lpq;
      const int rem = kk & ((1 << p.lpq) - 1);
      pp = rem >> p.lq;
      qq = rem & ((1 << p.lq) - 1);
    } else {
      n = (int)fdiv((unsigned)kk, p.div_pq);
      const int rem = kk - n * g.P * g.Q;
      pp = (int)fdiv((unsigned)rem, p.div_q);
      qq = rem - pp * g.Q;
    }
  };
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
  // WGRAD with LDS-DMA: instruction i of wave w fills bytes [1 KiB x (w*CH + i), +1 KiB) of
  // the K-outer image; lane L lands at byte 16L of it = (row, physical chunk), which holds
  // logical chunk phys ^ swizzle(row). B columns (r, s, c) are decoded once per instruction.
  constexpr int GB_CH = (MODE == MODE_WGRAD && GL) ? T::B_CH : 1;
  int gb_row[GB_CH], gb_r[GB_CH], gb_s[GB_CH], gb_c[GB_CH];
  bool gb_ok[GB_CH];
  if (MODE == MODE_WGRAD && GL) {
#pragma unroll
    for (int i = 0; i < GB_CH; ++i) {
      const int byte = (wvu * T::B_CH + i) * 1024 + lane * 16;
      const int row = byte / (BN * 2), phys = (byte % (BN * 2)) >> 4;
      const int ch = phys ^ kout_swz<BN>(row);
      const int j0 = n0 + ch * 8;
      gb_row[i] = row;
      gb_ok[i] = j0 < p.Ncol;
      const int jj = gb_ok[i] ? j0 : 0;
      gb_c[i] = jj % g.C;
      const int rs = jj / g.C;
      gb_r[i] = rs / g.S;
      gb_s[i] = rs - gb_r[i] * g.S;
    }
  }
  // WGRAD generic (not 1x1) register-staged B loader: per chunk, the image index and the
  // pixel-within-image of its row, decoded once and advanced by BK per load_tile call (the
  // calls go in K order), instead of a division-based decode of every chunk of every tile
  constexpr int WB = (MODE == MODE_WGRAD && !W1X1) ? T::B_CH : 1;
  int wb_n[WB], wb_pix[WB];
  const int wb_pq = g.P * g.Q;
  int wb_dn = 0, wb_dpix = 0;
  if (MODE == MODE_WGRAD && !W1X1 && !GL) {
    wb_dn = BK / wb_pq;
    wb_dpix = BK - wb_dn * wb_pq;
#pragma unroll
    for (int i = 0; i < WB; ++i) {
      const int kk = k_begin + (tid + NT * i) / B_CPR;
      int n, pp, qq;
      pix_decode(kk, n, pp, qq);
      wb_n[i] = n;
      wb_pix[i] = kk - n * wb_pq;
    }
  }
  // WGRAD: fused BN+ReLU of the activation operand (channel chunk fixed per thread)
  const bool wb_bn = WPRO && p.in_scale != nullptr;
  float wsc[8], wsh[8];
  if (wb_bn) {
    load8f(p.in_scale + wb_c, wsc);
    load8f(p.in_shift + wb_c, wsh);
  }

  // One register stage: the tile's operand chunks in flight from global memory. The fused
  // BN+ReLU prologue is applied when a stage is written to LDS (after the MFMAs of the
  // current tile), never right after the global load — that would put the load latency
  // back on the critical path. Bit i of ld_mask = chunk i was loaded in-bounds (padding
  // taps / tail rows stay exactly 0).
  struct Stage {
    uint4 ra[T::A_CH], rb[T::B_CH];
    unsigned ld_mask;
    float isc[8], ish[8];
  };
  const bool bn_in = (MODE == MODE_FWD) && p.in_scale != nullptr;

  auto load_tile = [&](int k0, Stage& st) {
    if (p.ablate & 2) return;
    uint4 (&ra)[T::A_CH] = st.ra;
    uint4 (&rb)[T::B_CH] = st.rb;
    unsigned& ld_mask = st.ld_mask;
    float (&isc)[8] = st.isc;
    float (&ish)[8] = st.ish;
    if (MODE == MODE_FWD || MODE == MODE_DGRAD) {
      // A: gather 8 consecutive k (same tap, 8 channels) for each owned row
      const int k = k0 + kin_ch * 8;
      const bool kok = k < k_end;
      if (bn_in) ld_mask = 0;
      if (bn_in && kok) {
        load8f(p.in_scale + kc, isc);
        load8f(p.in_shift + kc, ish);
      }
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        bool ok;
        int off;
        if (MODE == MODE_FWD) {
          if (is1x1) {
            ok = kok && a_y[i] >= 0;
            off = a_base[i] + kc;
          } else {
            const int yy = a_y[i] + kr, xx = a_x[i] + ks;
            ok = kok && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W;
            off = a_base[i] + (kr * g.W + ks) * g.C + kc;
          }
          if (ok) ld_mask |= 1u << i;
        } else {
          const int ty = a_y[i] - kr, tx = a_x[i] - ks;
          ok = kok && (unsigned)ty < (unsigned)g.P && (unsigned)tx < (unsigned)g.Q;
          off = a_base[i] + (ty * g.Q + tx) * g.K + kc;
        }
        SDX_DCHECK(!ok || (off >= 0 && off + 8 <= p.a_elems));
        ra[i] = ld16_or_zero(p.a + off, ok);
      }
      // B: weights, 8 channels of one tap per chunk (b_row / b_t0 / b_tr / b_ts addressing)
      const int kb = p.b_t0 + kr * p.b_tr + ks * p.b_ts + kc;
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        SDX_DCHECK(!(kok && b_off[i] >= 0) || (long)b_off[i] + kb + 8 <= p.b_elems);
        rb[i] = ld16_or_zero(p.b + b_off[i] + kb, kok && b_off[i] >= 0);
      }
      // advance the k decode by one tile
      kc += BK;
      while (kc >= cdim) {
        kc -= cdim;
        if (++ks == tap_s) { ks = 0; ++kr; }
      }
    } else {
      // WGRAD A: dy rows (pixels) x BM couts
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int e = tid + NT * i;
        const int row = e / A_CPR, ch = e % A_CPR;
        const int kk = k0 + row, co = m0 + ch * 8;
        SDX_DCHECK(!(kk < k_end && co < p.M) || (long)kk * g.K + co + 8 <= p.a_elems);
        ra[i] = ld16_or_zero(p.a + kk * g.K + co, kk < k_end && co < p.M);
      }
      // WGRAD B: im2col(x) rows (pixels) x BN (r,s,ci); the column chunk is fixed per thread
      if (wb_bn) ld_mask = 0;
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int e = tid + NT * i;
        const int row = e / B_CPR;
        const int kk = k0 + row;
        bool ok = wb_ok && kk < k_end;
        int off;
        if (is1x1) {
          off = kk * g.C + wb_c;
        } else {
          const int n = wb_n[i], pix = wb_pix[i];
          const int pp = p.lq >= 0 ? pix >> p.lq : (int)fdiv((unsigned)pix, p.div_q);
          const int qq = pix - pp * g.Q;
          const int yy = pp * g.stride - g.pad + wb_r, xx = qq * g.stride - g.pad + wb_s;
          ok = ok && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W;
          off = ((n * g.H + yy) * g.W + xx) * g.C + wb_c;
          // next K-tile: BK pixels on
          int np = pix + wb_dpix, nn = n + wb_dn;
          if (np >= wb_pq) { np -= wb_pq; ++nn; }
          wb_pix[i] = np;
          wb_n[i] = nn;
        }
        if (ok) ld_mask |= 1u << i;
        SDX_DCHECK(!ok || (off >= 0 && off + 8 <= p.b_elems));
        rb[i] = ld16_or_zero(p.b + off, ok);
      }
    }
  };

  // LDS-DMA staging of one K-tile into LDS buffer `buf` (out-of-range chunks copy the zero page)
  auto issue_glds = [&](int k0, int buf) {
    if constexpr (DEPTH != 6) {
      if (p.ablate & 2) return;
    }
    unsigned char* sa = smem + buf * T::STAGE;
    unsigned char* sb = sa + T::A_BYTES;
    if (MODE == MODE_WGRAD) {
      // A: dy [pixels][K] rows of the tile, BM couts each
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int byte = (wvu * T::A_CH + i) * 1024 + lane * 16;
        const int row = byte / (BM * 2), phys = (byte % (BM * 2)) >> 4;
        const int ch = phys ^ kout_swz<BM>(row);
        const int kk = k0 + row, co = m0 + ch * 8;
        const bool ok = kk < k_end && co < p.M;
        SDX_DCHECK(!ok || (long)kk * g.K + co + 8 <= p.a_elems);
        const gptr16 src = ok ? (gptr16)(p.a + kk * g.K + co) : zp;
        glds16(src, sa + (wvu * T::A_CH + i) * 1024);
      }
      // B: im2col(x) rows (pixels) x BN (r, s, c) columns
#pragma unroll
      for (int i = 0; i < GB_CH; ++i) {
        const int kk = k0 + gb_row[i];
        bool ok = gb_ok[i] && kk < k_end;
        int off;
        if (is1x1) {
          off = kk * g.C + gb_c[i];
        } else {
          int n, pp, qq;
          pix_decode(kk, n, pp, qq);
          const int yy = pp * g.stride - g.pad + gb_r[i], xx = qq * g.stride - g.pad + gb_s[i];
          ok = ok && (unsigned)yy < (unsigned)g.H && (unsigned)xx < (unsigned)g.W;
          off = ((n * g.H + yy) * g.W + xx) * g.C + gb_c[i];
        }
        SDX_DCHECK(!ok || (off >= 0 && off + 8 <= p.b_elems));
        const gptr16 src = ok ? (gptr16)(p.b + off) : zp;
        glds16(src, sb + (wvu * T::B_CH + i) * 1024);
      }
      return;
    }
    const int k = k0 + kin_ch * 8;
    // DEPTH 6: K-tiles never straddle k_end (Kdim % BK == 0), so the test is wave-uniform
    const bool kok = DEPTH == 6 ? k0 < k_end : k < k_end;
    if (fast_taps) {
      const int tap = u_kr * tap_s + u_ks;
      const int toff = (MODE == MODE_FWD) ? (u_kr * g.W + u_ks) * g.C + u_c0 : -(u_kr * g.Q + u_ks) * g.K + u_c0;
      const int lane_c = kin_ch * 8;
      // K-concatenated second operand (wave-uniform: g.K % BK == 0)
      const bool cat2 = MODE == MODE_DGRAD && u_c0 >= g.K;
#pragma unroll
      for (int i = 0; i < FCH; ++i) {
        const bool ok = kok && ((vmask[i] >> tap) & 1u);
        const int off = cat2 ? (rbase[i] >> p.a2_sh) + (u_c0 - g.K) + lane_c : rbase[i] + toff + lane_c;
        SDX_DCHECK(!ok || (off >= 0 && off + 8 <= (cat2 ? p.a2_elems : p.a_elems)));
        const gptr16 src = ok ? (gptr16)((cat2 ? p.a2 : p.a) + off) : zp;
        glds16(src, sa + 8 * (wvu * T::A_CH + i) * BK * 2);
      }
      const int kb = p.b_t0 + u_kr * p.b_tr + u_ks * p.b_ts + u_c0 + lane_c;
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const bool ok = kok && b_off[i] >= 0;
        SDX_DCHECK(!ok || (long)b_off[i] + kb + 8 <= p.b_elems);
        const gptr16 src = ok ? (gptr16)(p.b + b_off[i] + kb) : zp;
        glds16(src, sb + 8 * (wvu * T::B_CH + i) * BK * 2);
      }
      u_c0 += BK;
      if constexpr (DEPTH == 6) {
        // branch-free (keeps the DMA issue in the MFMA basic block)
        const bool w1 = u_c0 == cdim;
        u_c0 = w1 ? 0 : u_c0;
        u_ks += w1 ? 1 : 0;
        const bool w2 = u_ks == tap_s;
        u_ks = w2 ? 0 : u_ks;
        u_kr += w2 ? 1 : 0;
      } else if (u_c0 == cdim) {
        u_c0 = 0;
        if (++u_ks == tap_s) { u_ks = 0; ++u_kr; }
      }
      return;
    }
    // the tap offset of this thread's chunk column is the same for every row it stages:
    // one multiply per K-tile, then per row a bounds test and an add (no 1x1 special case:
    // its taps stay (0, 0))
    const int toff = (MODE == MODE_FWD) ? (kr * g.W + ks) * g.C + kc : kc - (kr * g.Q + ks) * g.K;
    // K-concatenated second operand (1x1: kr = ks = 0; the side is uniform per K-tile)
    const bool cat2 = MODE == MODE_DGRAD && kc >= g.K;
#pragma unroll
    for (int i = 0; i < T::A_CH; ++i) {
      bool ok;
      if (MODE == MODE_FWD)
        ok = kok && (unsigned)(a_y[i] + kr) < (unsigned)g.H && (unsigned)(a_x[i] + ks) < (unsigned)g.W;
      else
        ok = kok && (unsigned)(a_y[i] - kr) < (unsigned)g.P && (unsigned)(a_x[i] - ks) < (unsigned)g.Q;
      const int off = cat2 ? (a_rb[i] >> p.a2_sh) + (kc - g.K) : a_rb[i] + toff;
      SDX_DCHECK(!ok || (off >= 0 && off + 8 <= (cat2 ? p.a2_elems : p.a_elems)));
      const gptr16 src = ok ? (gptr16)((cat2 ? p.a2 : p.a) + off) : zp;
      glds16(src, sa + 8 * (wvu * T::A_CH + i) * BK * 2);
    }
    const int kb = p.b_t0 + kr * p.b_tr + ks * p.b_ts + kc;
#pragma unroll
    for (int i = 0; i < T::B_CH; ++i) {
      const bool ok = kok && b_off[i] >= 0;
      SDX_DCHECK(!ok || (long)b_off[i] + kb + 8 <= p.b_elems);
      const gptr16 src = ok ? (gptr16)(p.b + b_off[i] + kb) : zp;
      glds16(src, sb + 8 * (wvu * T::B_CH + i) * BK * 2);
    }
    kc += BK;
    if constexpr (DEPTH == 6) {
      // cdim % BK == 0 (host routing): at most one wrap per K-tile, branch-free
      const bool w1 = kc >= cdim;
      kc = w1 ? kc - cdim : kc;
      ks += w1 ? 1 : 0;
      const bool w2 = ks == tap_s;
      ks = w2 ? 0 : ks;
      kr += w2 ? 1 : 0;
    } else {
      while (kc >= cdim) {
        kc -= cdim;
        if (++ks == tap_s) { ks = 0; ++kr; }
      }
    }
  };

  auto store_tile = [&](int buf, Stage& st) {
    if (p.ablate & 1) return;
    uint4 (&ra)[T::A_CH] = st.ra;
    uint4 (&rb)[T::B_CH] = st.rb;
    const unsigned ld_mask = st.ld_mask;
    const float (&isc)[8] = st.isc;
    const float (&ish)[8] = st.ish;
    unsigned char* sa = smem + buf * T::STAGE;
    unsigned char* sb = sa + T::A_BYTES;
    if (bn_in) {
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i)
        if (ld_mask & (1u << i)) ra[i] = bnrelu8(ra[i], isc, ish);
    }
    if (wb_bn) {
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i)
        if (ld_mask & (1u << i)) rb[i] = bnrelu8(rb[i], wsc, wsh);
    }
    if (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i)
        *reinterpret_cast<uint4*>(sa + kin_off(kin_row0 + (NT / 8) * i, kin_ch)) = ra[i];
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i)
        *reinterpret_cast<uint4*>(sb + kin_off(kin_row0 + (NT / 8) * i, kin_ch)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < T::A_CH; ++i) {
        const int e = tid + NT * i;
        *reinterpret_cast<uint4*>(sa + kout_off<BM>(e / A_CPR, e % A_CPR)) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const int e = tid + NT * i;
        *reinterpret_cast<uint4*>(sb + kout_off<BN>(e / B_CPR, e % B_CPR)) = rb[i];
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment readers: lane (h, c) gets row/col c of the 16-wide tile, k = 8h..8h+7 of step u
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

  // all fragments of both 32-deep k-steps of a K-tile (distinct registers, so the MFMAs of
  // step 0 overlap the LDS latency of step 1 and no lgkmcnt(0) drain sits between MFMA
  // groups: the compiler otherwise recycles two A-fragment registers and stalls on each refill)
  auto read_frags = [&](int buf, bf16x8 (&af)[2][TM], bf16x8 (&bfr)[2][TN]) {
    const unsigned char* sa = smem + buf * T::STAGE;
    const unsigned char* sb = sa + T::A_BYTES;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (T::B_KIN) bfr[u][j] = frag_kin(sb, wn * WTN + 16 * j + c, u);
        else bfr[u][j] = frag_kout(sb, wn * WTN + 16 * j, u, std::integral_constant<int, BN>{});
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (T::A_KIN) af[u][i] = frag_kin(sa, wm * WTM + 16 * i + c, u);
        else af[u][i] = frag_kout(sa, wm * WTM + 16 * i, u, std::integral_constant<int, BM>{});
      }
    }
  };
  auto mfma_tile = [&](const bf16x8 (&af)[2][TM], const bf16x8 (&bfr)[2][TN]) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          // D = Bᵀ·Aᵀ: accumulator column = output row (lane c), rows = output columns (4h + r)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[u][j], af[u][i], acc[i][j], 0, 0, 0);
  };
  // one 32-deep k-step u of a K-tile (DEPTH 6 keeps two such sets in flight)
  auto read_frags_u = [&](int buf, int u, bf16x8 (&af)[TM], bf16x8 (&bfr)[TN]) {
    const unsigned char* sa = smem + buf * T::STAGE;
    const unsigned char* sb = sa + T::A_BYTES;
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag_kin(sb, wn * WTN + 16 * j + c, u);
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = frag_kin(sa, wm * WTM + 16 * i + c, u);
  };
  auto mfma_u = [&](const bf16x8 (&af)[TM], const bf16x8 (&bfr)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };
  auto compute = [&](int buf) {
    if (p.ablate & 4) return;
    bf16x8 af[2][TM], bfr[2][TN];
    read_frags(buf, af, bfr);
    mfma_tile(af, bfr);
  };

  // 8-wave blocks: the second-dispatched half loses VALU/issue arbitration to the older half
  // on every segment; one static priority raise for it (no per-cluster flips). SDX_PRIO_HALF
  if (SDX_PRIO_HALF && NT == 512 && __builtin_amdgcn_readfirstlane(tid) >= 256)
    __builtin_amdgcn_s_setprio(1);
  // K loop: two LDS buffers, one barrier per K-tile. DEPTH 1: the loads of tile k+1 are in
  // flight during the MFMAs of tile k. DEPTH 2: two register stages, so tile k+2's loads
  // are issued while tile k computes and the LDS write of tile k+1 waits only for loads
  // issued a whole K-tile earlier (load latency covered by two tiles of MFMA work).
  if constexpr (DEPTH == 7 || DEPTH == 8) {
    // Tap-reuse 3x3 (stride 1, pad 1) loop. The implicit GEMM above re-gathers a shifted copy
    // of the A tile for every tap (9 LDS-DMA fills of BM rows per 64 channels, the per-CU fill
    // bandwidth sets the pace: profiles/conv_core_r4.txt). Here the tile's input window (the
    // halo: its image rows plus the pad ring) is staged ONCE per 64-channel chunk and each of
    // the 9 taps is a step that reads it at a uniform pixel offset; only the weight tile
    // (BN x 64, L2-resident) is staged per step, through a 3-buffer ring. The step structure
    // is DEPTH 6's: step-1 fragments read under step-0 MFMAs, ONE raw barrier per step, then
    // the freed weight buffer is refilled with step s+3 and step-0 fragments of s+1 are read,
    // interleaved with step-1 MFMAs. The 9 taps of a chunk are unrolled: every tap-dependent
    // quantity (fragment address variant, weight ring buffer — 9 steps per chunk keep the
    // ring's phase —, halo piece of the step) is a compile-time constant, and an A fragment
    // address is ONE VALU op (precomputed lane base + the tap's uniform row offset).
    // DEPTH 7 double-buffers the halo: chunk c+1's window is issued one 1-KiB piece per step
    // during chunk c (a wave has at most 8 pieces; the 9th slot and unused ones DMA the zero
    // page into a junk KiB, so every step issues exactly NL DMAs and one counted vmcnt covers
    // them). DEPTH 8: a single chunk (C = 64), one halo buffer.
    // RAW: a weight tile / halo piece issued in step i (after its barrier) is retired by the
    // vmcnt(NL) of step i+2 (the NL youngest are step i+1's), before that step's barrier;
    // chunk c+1's pieces go out in steps 9c-1 .. 9c+6 and are first read after the barrier of
    // step 9c+8. WAR: the weight buffer of step s is refilled after the barrier that follows
    // its last reads; halo buffer (c+1)&1 held chunk c-1, last read before the barrier of step
    // 9c-1, refilled from after that barrier on.
    constexpr int NW = NT / 64;
    constexpr int NHB = DEPTH == 7 ? 2 : 1;
    constexpr int HKB = tap_halo_kb(BM);
    constexpr int NHW = (HKB + NW - 1) / NW;    // halo pieces per wave per chunk (max)
    static_assert(DEPTH == 8 || NHW <= 8, "a chunk's halo pieces must be issued within 8 steps");
    constexpr int NL = T::B_CH + (DEPTH == 7 ? 1 : 0);   // LDS-DMAs per wave per step
    // fragment-address variants per row: the swizzle phase of tap (rr, ss) is
    // (F0 + ss + t_ky·rr) & 7 with t_ky in {0, 4} (4 only for 4x4 images, BM = 128 tiles):
    // it depends on ss and, for t_ky = 4, on rr & 1
    constexpr int NV = BM == 128 ? 6 : 3;
    unsigned char* const junk = smem + NHB * HKB * 1024;
    unsigned char* const bring = junk + 1024;
    const int HW = g.H * g.W;
    const int RW = p.t_rw > 0 ? p.t_rw : g.W;   // virtual pixels per image row
    const int HWv = g.H * RW;
    const int nimg0 = m0 / HWv;
    const int y0 = p.t_imgs > 0 ? 0 : (m0 - nimg0 * HWv) / RW;   // t_imgs 0: a band of one image
    const int nch = p.t_nch;
    // halo pieces of this wave: piece wvu + NW·i; lane L carries pixel 8·piece + L/8, physical
    // chunk L%8 = logical chunk (L%8) ^ swizzle. Source element (chunk 0) or -1 (zero: pad ring,
    // images past N, pixels past the window)
    int hsrc[NHW];
#pragma unroll
    for (int i = 0; i < NHW; ++i) {
      const int P = (wvu + NW * i) * 8 + (lane >> 3);
      const int img = P / p.t_is, rem = P - img * p.t_is;
      const int hy = rem / p.t_rs, hx = rem - hy * p.t_rs;
      const int n = nimg0 + img, yin = y0 - 1 + hy, xin = hx - 1;
      const int q = (lane & 7) ^ ((hx + p.t_ky * hy) & 7);
      const bool ok = P < p.t_hp && n < g.N && (unsigned)yin < (unsigned)g.H && (unsigned)xin < (unsigned)g.W;
      SDX_DCHECK(!ok || (long)((n * g.H + yin) * g.W + xin) * cdim + nch * 64 <= p.a_elems);
      hsrc[i] = ok ? ((n * g.H + yin) * g.W + xin) * cdim + q * 8 : -1;
    }
    auto halo_piece = [&](int i, int src, int ch, int hbuf, bool real) {
      const int pc = wvu + NW * i;
      real = real && pc < p.t_nhp;
      unsigned char* dst = real ? smem + hbuf * (HKB * 1024) + pc * 1024 : junk;
      const gptr16 s = (real && src >= 0) ? (gptr16)(p.a + src + ch * 64) : zp;
      glds16(s, dst);
    };
    // A fragment lane bases: za[i][v] = byte address (step 0 of the k-step pair, u = 0) of the
    // lane's output pixel's halo row at tap column ss = v % 3 (and rr parity v / 3), swizzle
    // applied; a tap adds rr·t_rs·128 (+ the halo buffer), k-step u = 1 flips bit 6
    int za[TM][NV];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * WTM + 16 * i + c;
      int img, y, x;
      if (p.t_imgs > 0) {
        img = ml / HW;
        const int rem = ml - img * HW;
        y = rem / g.W;
        x = rem - y * g.W;
      } else {
        img = 0;
        y = ml / RW;
        x = ml - y * RW;
      }
      const int P0 = img * p.t_is + y * p.t_rs + x, F0 = x + p.t_ky * y;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int ss = v % 3, rpar = v / 3;
        za[i][v] = (P0 + ss) * 128 + ((h ^ ((F0 + ss + p.t_ky * rpar) & 7)) << 4);
      }
    }
    const int rs128 = p.t_rs * 128;
    // A fragments of tap TAP (static) of chunk ch, k-step U (static)
    auto read_a7 = [&](auto TAPc, int ch, auto Uc, bf16x8 (&af)[TM]) {
      constexpr int tap = decltype(TAPc)::value, u = decltype(Uc)::value;
      constexpr int rr = MODE == MODE_FWD ? tap / 3 : 2 - tap / 3;
      constexpr int ss = MODE == MODE_FWD ? tap % 3 : 2 - tap % 3;
      constexpr int v = NV == 6 ? ss + 3 * (rr & 1) : ss;
      const int off = (NHB == 2 ? (ch & 1) * (HKB * 1024) : 0) + rr * rs128;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int a = (u ? (za[i][v] ^ 64) : za[i][v]) + off;
        af[i] = *reinterpret_cast<const bf16x8*>(smem + a);
      }
    };
    auto read_b7 = [&](auto BBc, auto Uc, bf16x8 (&bfr)[TN]) {
      constexpr int bb = decltype(BBc)::value, u = decltype(Uc)::value;
      const unsigned char* sb = bring + bb * T::B_BYTES;
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag_kin(sb, wn * WTN + 16 * j + c, u);
    };
    // weight tile of tap TAP of chunk ch into ring buffer TAP % 3 (past the last chunk: zero page)
    auto issue_b7 = [&](auto TAPc, int ch) {
      constexpr int tap = decltype(TAPc)::value, r = tap / 3, s = tap % 3, bb = tap % 3;
      const bool kok = ch < nch;
      const int kb = p.b_t0 + r * p.b_tr + s * p.b_ts + ch * 64 + kin_ch * 8;
#pragma unroll
      for (int i = 0; i < T::B_CH; ++i) {
        const bool ok = kok && b_off[i] >= 0;
        SDX_DCHECK(!ok || (long)b_off[i] + kb + 8 <= p.b_elems);
        const gptr16 src = ok ? (gptr16)(p.b + b_off[i] + kb) : zp;
        glds16(src, bring + bb * T::B_BYTES + 8 * (wvu * T::B_CH + i) * BK * 2);
      }
    };
    // the halo slot of the step that reads tap J of chunk cc (after its barrier): piece J of
    // chunk cc + 1 (into halo buffer (cc + 1) & 1), or a junk DMA
    auto halo_slot = [&](auto Jc, int cc) {
      if constexpr (DEPTH == 7) {
        constexpr int j = decltype(Jc)::value;
        if constexpr (j < NHW) halo_piece(j, hsrc[j], cc + 1, (cc + 1) & 1, cc + 1 < nch);
        else glds16(zp, junk);
      }
    };
    // prologue: chunk 0's window, the weight tiles of taps 0-2 (+ the halo slots of steps
    // -3, -2 (none) and -1 (piece 0 of chunk 1))
#pragma unroll
    for (int i = 0; i < NHW; ++i) halo_piece(i, hsrc[i], 0, 0, true);
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    issue_b7(I0{}, 0);
    if constexpr (DEPTH == 7) glds16(zp, junk);
    issue_b7(I1{}, 0);
    if constexpr (DEPTH == 7) glds16(zp, junk);
    issue_b7(std::integral_constant<int, 2>{}, 0);
    halo_slot(I0{}, 0);
    vm_wait<2 * NL>();   // chunk 0's window and tap 0's weights landed
    lds_barrier();
    stamp(1);
    bf16x8 a0[TM], b0[TN], a1[TM], b1[TN];
    read_a7(I0{}, 0, I0{}, a0);
    read_b7(I0{}, I0{}, b0);
    for (int ch = 0; ch < nch; ++ch) {
      static_for<0, 9>([&](auto TAPc) {
        constexpr int tap = decltype(TAPc)::value;
        constexpr int tap1 = (tap + 1) % 9, tap3 = (tap + 3) % 9;
        const int ch1 = tap == 8 ? ch + 1 : ch;          // chunk of the next step
        const int ch3 = tap + 3 >= 9 ? ch + 1 : ch;      // chunk of step + 3
        read_a7(TAPc, ch, I1{}, a1);
        read_b7(std::integral_constant<int, tap % 3>{}, I1{}, b1);
        mfma_u(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        const int kt = 9 * ch + tap;
        if (kt < 160) stamp(2 + 3 * kt);
        vm_wait<NL>();
        lds_barrier();
        if (kt < 160) stamp(3 + 3 * kt);
        // the next step (after the last one: a harmless read inside the LDS image, never used)
        read_a7(std::integral_constant<int, tap1>{}, NHB == 2 ? ch1 : 0, I0{}, a0);
        read_b7(std::integral_constant<int, tap1 % 3>{}, I0{}, b0);
        issue_b7(std::integral_constant<int, tap3>{}, ch3);
        halo_slot(std::integral_constant<int, tap1>{}, ch1);
        mfma_u(a1, b1);
        if constexpr (SDX_W1_SGB) static_for<0, TM * TN>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // up to 5 VALU
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // up to 1 VMEM read (LDS-DMA)
          __builtin_amdgcn_sched_group_barrier(0x004, 2, 0);   // up to 2 SALU
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    // the zero-page DMAs past the end must land before any wave's epilogue reuses the LDS
    vm_wait<0>();
    __syncthreads();
  } else if constexpr (DEPTH == 6) {
    // 8-wave 256x128 / 128x256 tiles (64x64 wave tiles, two waves per SIMD) over a 3-buffer
    // LDS-DMA ring, pipelined inside each wave. A K-tile is two 32-deep k-steps: the fragments of step 1 are read
    // while step 0's MFMAs run, then ONE raw barrier (every wave's reads of this tile are
    // done and its own DMAs of tile k+1 retired by the counted vmcnt), then the buffer just
    // freed is refilled with tile k+3 and step 0 of tile k+1 is read, both interleaved with
    // step 1's MFMAs — the matrix pipe idles only for the barrier.
    // RAW: tile k+1 is read after the barrier of iteration k, which every wave reaches after
    // retiring its own DMAs of tile k+1. WAR: tile k+3 overwrites tile k's buffer only after
    // that barrier, which every wave reaches after its last read of tile k completed
    // (lds_barrier: lgkmcnt(0)). The DMA issue is unconditional (tiles past the end load the
    // zero page into the free buffer and are never read; host routing guarantees
    // cdim % BK == 0, so the k decode advances branch-free), keeping the second half one
    // basic block for the MFMA/DMA interleave; the queue is drained after the loop.
    constexpr int NL = T::A_CH + T::B_CH;   // LDS-DMA instructions per wave per tile
    bf16x8 a0[TM], b0[TN], a1[TM], b1[TN];
    issue_glds(k_begin, 0);
    issue_glds(k_begin + BK, 1);
    issue_glds(k_begin + 2 * BK, 2);
    vm_wait<2 * NL>();
    lds_barrier();
    stamp(1);
    read_frags_u(0, 0, a0, b0);
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (!(SDX_W1_ABL && (p.ablate & 8))) read_frags_u(buf, 1, a1, b1);
      if (!(SDX_W1_ABL && (p.ablate & 4))) mfma_u(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (kt < 160) stamp(2 + 3 * kt);
      vm_wait<NL>();   // own DMAs of tile kt+1 retired; tile kt+2 stays in flight
      lds_barrier();
      if (kt < 160) stamp(3 + 3 * kt);
      const int nbuf = buf == 2 ? 0 : buf + 1;
      if (!(SDX_W1_ABL && (p.ablate & 8))) read_frags_u(nbuf, 0, a0, b0);
      if (!(SDX_W1_ABL && (p.ablate & 2))) issue_glds(k_begin + (kt + 3) * BK, buf);
      if (!(SDX_W1_ABL && (p.ablate & 4))) mfma_u(a1, b1);
      // the DMA issue (address VALU + LDS-DMA) interleaved with the second half's MFMAs
      // instead of ahead of them (the matrix pipe would idle through it)
      if constexpr (SDX_W1_SGB) static_for<0, TM * TN>([&](auto) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // up to 5 VALU
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // up to 1 VMEM read (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x004, 2, 0);   // up to 2 SALU
      });
      __builtin_amdgcn_sched_barrier(0);
      buf = nbuf;
    }
    // the zero-page DMAs issued past the end must land before ANY wave's epilogue reuses the
    // LDS (C staging): this wave's drain, then a barrier behind every wave's drain
    vm_wait<0>();
    __syncthreads();
  } else if constexpr (DEPTH == 3 && ONE) {
    // single stage: each K-tile is loaded, then computed, in turn (no overlap inside the
    // block). With a short reduction (SDX_IGEMM_ONE_K) the half-size LDS lets more blocks
    // share a CU, and their loads overlap each other's MFMAs and epilogues instead
    for (int kt = 0; kt < nk; ++kt) {
      issue_glds(k_begin + kt * BK, 0);
      __syncthreads();
      if (kt == 0) stamp(1);
      compute(0);
      __syncthreads();
    }
  } else if constexpr (DEPTH == 3) {
    // the DMA of tile k+1 overlaps the MFMAs of tile k; the barrier's vmcnt(0) lands it
    if (nk > 0) issue_glds(k_begin, 0);
    __syncthreads();
    stamp(1);
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) issue_glds(k_begin + (kt + 1) * BK, buf ^ 1);
      compute(buf);
      __syncthreads();
    }
  } else if (DEPTH == 1) {
    Stage s0;
    if (nk > 0) {
      load_tile(k_begin, s0);
      store_tile(0, s0);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      const bool more = kt + 1 < nk;
      load_tile(k_begin + (kt + 1) * BK, s0);   // past the end: zero-page loads (uniform vmcnt)
      compute(buf);
      if (more) store_tile(buf ^ 1, s0);
      __syncthreads();
    }
  } else {
    Stage s0, s1;
    if (nk > 0) {
      load_tile(k_begin, s0);
      store_tile(0, s0);
    }
    load_tile(k_begin + BK, s1);
    __syncthreads();
    // prefetch loads are issued unconditionally (past the end they read the zero page):
    // a conditional load block makes hipcc assume the shortest load queue and wait for
    // the loads just issued before the LDS write
    for (int kt = 0; kt < nk; kt += 2) {
      // buffer 0 holds tile kt; s1 carries tile kt+1
      load_tile(k_begin + (kt + 2) * BK, s0);
      compute(0);
      if (kt + 1 < nk) store_tile(1, s1);
      __syncthreads();
      if (kt + 1 >= nk) break;
      // buffer 1 holds tile kt+1; s0 carries tile kt+2
      load_tile(k_begin + (kt + 3) * BK, s1);
      compute(1);
      if (kt + 2 < nk) store_tile(0, s0);
      __syncthreads();
    }
  }

  stamp(kTraceSlots - 4);
  if constexpr (DEPTH == 7 || DEPTH == 8) {
    if (p.t_rw > 0) {
      // padded rows (x >= W; m0 is a multiple of t_rw): exact zeros, as the statistics read
      // the accumulators
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bool pad = ((wm * WTM + 16 * i + c) & (p.t_rw - 1)) >= g.W;
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = pad ? 0.f : acc[i][j][r];
      }
    }
  }
  // ---------------------------------- epilogues ----------------------------------
  // acc[i][j][r] = C[m0 + wm*64 + 16i + c][n0 + wn*64 + 16j + 4h + r]
  // (not compiled into the BN-statistics DGRAD variant: its register budget sits at the
  // 128-VGPR occupancy step)
  if (MODE != MODE_WGRAD && !VAR && (p.bias != nullptr || p.relu)) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = n0 + wn * WTN + 16 * j + 4 * h + r;
        const float b = (p.bias != nullptr && col < p.Ncol) ? p.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float v = acc[i][j][r] + b;
          acc[i][j][r] = p.relu ? fmaxf(v, 0.f) : v;
        }
      }
  }
  if (MODE == MODE_WGRAD || (!VAR && p.out_f32)) {
    // fp32 rows straight from the accumulators: 4 consecutive columns per lane (WGRAD: this
    // split's partial slab; FWD / DGRAD out_f32: stride-1 GEMM rows, host-checked)
    float* out = reinterpret_cast<float*>(p.out) + (MODE == MODE_WGRAD ? (size_t)split * p.M * p.Ncol : 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * WTM + 16 * i + c;
      if (row >= p.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WTN + 16 * j + 4 * h;
        if (col < p.Ncol)
          st16<SDX_NT_PART != 0 && MODE == MODE_WGRAD>(
              out + (size_t)row * p.Ncol + col,
              make_uint4(__float_as_uint(acc[i][j][0]), __float_as_uint(acc[i][j][1]), __float_as_uint(acc[i][j][2]),
                         __float_as_uint(acc[i][j][3])));
      }
    }
    return;
  }

  if (MODE == MODE_DGRAD && p.bias_pre != nullptr) {
    // per-column fp32 bias joins the accumulators before the single bf16 rounding
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WTN + 16 * j + 4 * h;
      if (col < p.Ncol) {
        const float4 b = *reinterpret_cast<const float4*>(p.bias_pre + col);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          acc[i][j][0] += b.x;
          acc[i][j][1] += b.y;
          acc[i][j][2] += b.z;
          acc[i][j][3] += b.w;
        }
      }
    }
  }
#if SDX_ADD_PRE
  if (MODE == MODE_DGRAD && p.add_pre && p.addend != nullptr) {
    // the addend joins the fp32 accumulators, so the sum is rounded to bf16 once (a small
    // addend added after rounding is swamped: profiles/bn3_fold_r2.txt). Stride-1 rows.
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = m0 + wm * WTM + 16 * i + c;
      if (row >= p.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * WTN + 16 * j + 4 * h;
        if (col < p.Ncol) {
          const uint2 a = *reinterpret_cast<const uint2*>(p.addend + (size_t)row * p.Ncol + col);
          acc[i][j][0] += __uint_as_float(a.x << 16);
          acc[i][j][1] += __uint_as_float(a.x & 0xffff0000u);
          acc[i][j][2] += __uint_as_float(a.y << 16);
          acc[i][j][3] += __uint_as_float(a.y & 0xffff0000u);
        }
      }
    }
  }
#endif
  // bf16 rounding (stats describe the stored tensor); pack 4 consecutive columns
  uint2 ov[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      ov[i][j] = make_uint2(pack_bf2(acc[i][j][0], acc[i][j][1]), pack_bf2(acc[i][j][2], acc[i][j][3]));

  // Store loop: thread tid writes the 16-B chunks e = tid + it·NT (it < ITER) of the
  // [BM][BN] tile — always the same column chunk my_ch. The epilogue's own global operands
  // (DGRAD: residual addend + its ReLU bits; fused BN-backward statistics: y_a, y_b + ReLU
  // bits) are prefetched PF iterations ahead through a register ring, the first PF issued
  // before the LDS staging, so their latency overlaps it instead of stalling every chunk.
  constexpr int CPR = BN / 8;
  constexpr int ITER = BM * CPR / NT;
  constexpr int PF = ITER < 4 ? ITER : 4;
  static_assert(NT % CPR == 0 && CPR <= 64 && (BM * CPR) % NT == 0, "fixed column chunk per thread");
  const bool has_add = MODE == MODE_DGRAD && p.addend != nullptr && !(SDX_ADD_PRE && p.add_pre);
  constexpr bool bst = MODE == MODE_DGRAD && VAR != 0;
  constexpr bool bnap = MODE == MODE_FWD && VAR == 2;   // block-output BN apply (+ residual, ReLU, bits)
  const int my_ch = tid % CPR, my_col = n0 + my_ch * 8;
  int eo[ITER];   // output element offset of each chunk (-1: outside the tensor)
  int ea[ITER];   // addend element offset (-1: no addend there)
  const int asub = (MODE == MODE_DGRAD) ? p.addend_sub : 0;
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int row = (tid + it * NT) / CPR;
    const int m = m0 + row;
    int o = -1, oa = -1;
    bool mok = m < p.M;
    int mr = m;
    if ((DEPTH == 7 || DEPTH == 8) && p.t_rw > 0) {
      // padded-row tile: virtual row -> pixel, or none
      const int HWv = g.H * p.t_rw;
      const int n = m / HWv, rem = m - n * HWv;
      const int yy = rem / p.t_rw, xx = rem - yy * p.t_rw;
      mok = n < g.N && xx < g.W;
      mr = (n * g.H + yy) * g.W + xx;
    }
    if (mok && my_col < p.Ncol) {
      int orow = mr;
      if (MODE == MODE_DGRAD && g.stride != 1) {
        const int hw = p.Hc * p.Wc;
        const int n = m / hw, rem = m - n * hw;
        const int yy = rem / p.Wc, xx = rem - yy * p.Wc;
        orow = (n * g.H + yy * g.stride + p.ph) * g.W + xx * g.stride + p.pw;
      }
      o = orow * p.Ncol + my_col;
      oa = o;
      if (asub > 1) {
        const int hw = g.H * g.W;
        const int n = orow / hw, rem = orow - n * hw;
        const int hh = rem / g.W, ww = rem - hh * g.W;
        const int Hs = (g.H + asub - 1) / asub, Ws = (g.W + asub - 1) / asub;
        oa = (hh % asub == 0 && ww % asub == 0) ? ((n * Hs + hh / asub) * Ws + ww / asub) * p.Ncol + my_col : -1;
      }
    }
    eo[it] = o;
    ea[it] = oa;
  }
  uint4 pf_add[PF], pf_ya[PF], pf_yb[PF];
  uint32_t pf_am[PF], pf_bm[PF];
  auto prefetch = [&](auto IT, auto SL) __attribute__((always_inline)) {
    constexpr int it = decltype(IT)::value, sl = decltype(SL)::value;
    const int o = eo[it];
    const bool ok = o >= 0;
    if (MODE == MODE_DGRAD && has_add) {
      // (the zero page, not a private zero: a select between a global and a private
      // address would turn the load into a flat load and spill the zero to scratch)
      const int oa = ea[it];
      pf_add[sl] = ld16_stream(p.addend + (oa >= 0 ? oa : 0), oa >= 0);
      pf_am[sl] = (ok && p.addend_mask != nullptr) ? (uint32_t)p.addend_mask[o >> 3] : 0xffu;
    }
    if constexpr (bnap) pf_add[sl] = ld16_stream(p.addend + (ok ? o : 0), ok);   // the residual
    if (MODE == MODE_DGRAD && bst) {
      // ya == nullptr (a forward-folded BN3 whose y was never stored): y = 0, so the second
      // sum is −μ·Σdz and the caller appends the Σdz·y rows (bnfold.hip rowdot)
      const bool oky = ok && p.bs.ya != nullptr;
      pf_ya[sl] = ld16_stream(reinterpret_cast<const uint16_t*>(p.bs.ya) + (oky ? o : 0), oky);
      const bool okb = ok && p.bs.yb != nullptr;
      pf_yb[sl] = ld16_stream(reinterpret_cast<const uint16_t*>(p.bs.yb) + (okb ? o : 0), okb);
      pf_bm[sl] = (ok && p.bs.mask != nullptr) ? (uint32_t)p.bs.mask[o >> 3] : 0xffu;
    }
  };
  // FWD without an output tensor: a statistics-only pass (forward-folded BN3, first pass)
  const bool store_out = !(MODE == MODE_FWD && p.out == nullptr);
  if ((MODE == MODE_DGRAD && (has_add || bst)) || bnap) {
    static_for<0, PF>([&](auto I) { prefetch(I, I); });
  }

  // stage the C tile through LDS ([BM][BN] bf16, rows padded by 8 B: 16 lanes writing 8 B
  // at the same column of 16 consecutive rows hit distinct banks)
  constexpr int CRS = BN * 2 + 8;
  static_assert(BM * CRS <= LDS, "C tile must fit the staging LDS");
  if (store_out) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        *reinterpret_cast<uint2*>(smem + (wm * WTM + 16 * i + c) * CRS + (wn * WTN + 16 * j + 4 * h) * 2) = ov[i][j];
  }
  __syncthreads();
  stamp(kTraceSlots - 3);
  // fused BN-backward statistics (DGRAD): per-thread sums for column chunk my_ch
  const int bs_ns = p.bs.yb != nullptr ? 3 : 2;
  float bmu_a[8], bmu_b[8], bmk_s[8], bmk_t[8], bsum[3][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bmu_a[q] = bmu_b[q] = bmk_s[q] = bmk_t[q] = 0.f;
    bsum[0][q] = bsum[1][q] = bsum[2][q] = 0.f;
  }
  float bsc[8], bsh[8], rsc[8], rsh[8];
  const bool raff = bnap && p.bn_rsc != nullptr;
  if constexpr (bnap) {
    if (my_col < p.Ncol) {
      load8f(p.bn_sc + my_col, bsc);
      load8f(p.bn_sh + my_col, bsh);
      if (raff) {
        load8f(p.bn_rsc + my_col, rsc);
        load8f(p.bn_rsh + my_col, rsh);
      }
    }
  }
  if (MODE == MODE_DGRAD && bst && my_col < p.Ncol) {
    load8f(p.bs.ma + my_col, bmu_a);
    if (p.bs.yb) load8f(p.bs.mb + my_col, bmu_b);
    if (p.bs.mask == nullptr && p.bs.msc != nullptr) {
      load8f(p.bs.msc + my_col, bmk_s);
      load8f(p.bs.msh + my_col, bmk_t);
    }
  }
  if (store_out) {
    uint16_t* out = reinterpret_cast<uint16_t*>(p.out);
    static_for<0, ITER>([&](auto I) {
      constexpr int it = decltype(I)::value, sl = it % PF;
      const uint4 a_in = pf_add[sl], ya_in = pf_ya[sl], yb_in = pf_yb[sl];
      const uint32_t am = pf_am[sl], bm = pf_bm[sl];
      if constexpr (it + PF < ITER) {
        if ((MODE == MODE_DGRAD && (has_add || bst)) || bnap)
          prefetch(std::integral_constant<int, it + PF>{}, std::integral_constant<int, sl>{});
      }
      const int o = eo[it];
      if (o >= 0) {
        const int row = (tid + it * NT) / CPR;
        const unsigned char* src = smem + row * CRS + my_ch * 16;
        const uint2 lo = *reinterpret_cast<const uint2*>(src);
        const uint2 hi = *reinterpret_cast<const uint2*>(src + 8);
        uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
        if (MODE == MODE_DGRAD && has_add) {
          // fused residual-gradient accumulation: out = dgrad + addend (may alias out: every
          // chunk is read and written by the same thread); with addend_mask the addend is
          // dout·[out > 0] from the block output's 1-bit ReLU mask (no dz tensor)
          uint4 a = a_in;
          uint32_t* aw2 = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t keep = ((am >> (2 * q)) & 1u ? 0x0000ffffu : 0u) | ((am >> (2 * q + 1)) & 1u ? 0xffff0000u : 0u);
            aw2[q] &= keep;
          }
          const uint32_t* vw = reinterpret_cast<const uint32_t*>(&v);
          const uint32_t* aw = reinterpret_cast<const uint32_t*>(&a);
          uint32_t r[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float x0 = __uint_as_float(vw[q] << 16) + __uint_as_float(aw[q] << 16);
            const float x1 = __uint_as_float(vw[q] & 0xffff0000u) + __uint_as_float(aw[q] & 0xffff0000u);
            r[q] = pack_bf2(x0, x1);
          }
          v = make_uint4(r[0], r[1], r[2], r[3]);
        }
        if constexpr (bnap) {
          // bn_apply mode 2 on the bf16-rounded conv output (the value y3 would have been
          // stored as): the same operations in the same order, so the block output is the
          // one the separate pass writes
          float yv[8], rv[8];
          unpack8(v, yv);
          unpack8(a_in, rv);
#pragma unroll
          for (int q = 0; q < 8; ++q) yv[q] = yv[q] * bsc[q] + bsh[q];
          if (raff) {
#pragma unroll
            for (int q = 0; q < 8; ++q) yv[q] += rv[q] * rsc[q] + rsh[q];
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) yv[q] += rv[q];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) yv[q] = fmaxf(yv[q], 0.f);
          v = pack8(yv);
          if (p.mask_out != nullptr) p.mask_out[o >> 3] = (uint8_t)relu_bits8(v);
        }
        // VAR 2 stores once, after the ReLU-backward mask below
        constexpr bool NTS = MODE == MODE_DGRAD ? SDX_NT_STORE_DGRAD != 0 : SDX_NT_STORE != 0;
        if (VAR != 2 || !(MODE == MODE_DGRAD && bst)) st16<NTS>(out + o, v);
        if (MODE == MODE_DGRAD && bst) {
          // statistics of the stored (bf16-rounded) values, as bn_bwd_reduce would read them
          float d[8], ya[8];
          unpack8(v, d);
          unpack8(ya_in, ya);
          if (p.bs.mask != nullptr) {
#pragma unroll
            for (int q = 0; q < 8; ++q) d[q] = (bm >> q) & 1u ? d[q] : 0.f;
          } else if (p.bs.msc != nullptr) {
#pragma unroll
            for (int q = 0; q < 8; ++q) d[q] = ya[q] * bmk_s[q] + bmk_t[q] > 0.f ? d[q] : 0.f;
          }
          // VAR 2: ReLU backward applied to the stored gradient too (head: dh = (dz·W2)·[h > 0];
          // BN3 fold: dz = dout·[out > 0] of the previous block): the chunk is stored masked
          // (bf16 values already, so the repack is exact). Its own variant: the
          // BN-statistics kernels sit at the 128-VGPR occupancy step
          if constexpr (VAR == 2) st16<SDX_NT_STORE_DGRAD != 0>(out + o, pack8(d));
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            bsum[0][q] += d[q];
            bsum[1][q] = fmaf(d[q], ya[q] - bmu_a[q], bsum[1][q]);
          }
          if (p.bs.yb != nullptr) {
            float yb[8];
            unpack8(yb_in, yb);
#pragma unroll
            for (int q = 0; q < 8; ++q) bsum[2][q] = fmaf(d[q], yb[q] - bmu_b[q], bsum[2][q]);
          }
        }
      }
    });
  }

  if (MODE == MODE_DGRAD && bst) {
    // lanes my_ch, my_ch + CPR, ... of a wave hold the same columns: butterfly over them,
    // then one [NS][BN] row per wave through LDS, summed in wave order (deterministic)
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        for (int off = CPR; off < 64; off <<= 1) bsum[k][q] += __shfl_xor(bsum[k][q], off);
    __syncthreads();   // C-tile reads of the store loop are done
    float* red = reinterpret_cast<float*>(smem);   // [NT/64][3][BN]
    static_assert((NT / 64) * 3 * BN * 4 <= LDS, "BN-bwd stat reduction must fit the staging LDS");
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int q = 0; q < 8; ++q) red[(wv * 3 + k) * BN + my_ch * 8 + q] = bsum[k][q];
    }
    __syncthreads();
    for (int e = tid; e < bs_ns * BN; e += NT) {
      const int k = e / BN, col = e % BN;
      float s = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NT / 64; ++w2) s += red[(w2 * 3 + k) * BN + col];
      if (n0 + col < p.Ncol) {
        p.bs.slab[((size_t)(p.bs.row0 + mt) * bs_ns + k) * p.Ncol + n0 + col] = s;
      }
    }
  }

  if (MODE == MODE_FWD && p.stats != nullptr) {
    // per-column (Σy, Σy²) over this tile's rows, from the fp32 accumulators (rows past M
    // are exact zeros: their A rows were zero-filled); one slab row per M-tile. Rows are
    // reduced in registers over i, then over the 16 lanes c with DPP row adds.
    float s1[TN][4], s2[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float v = acc[i][j][r];
          a1 += v;
          a2 = fmaf(v, v, a2);
        }
        s1[j][r] = row16_sum(a1);
        s2[j][r] = row16_sum(a2);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [WM][2][BN]
    if (c == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          red[(wm * 2 + 0) * BN + wn * WTN + 16 * j + 4 * h + r] = s1[j][r];
          red[(wm * 2 + 1) * BN + wn * WTN + 16 * j + 4 * h + r] = s2[j][r];
        }
    }
    __syncthreads();
    for (int e = tid; e < 2 * BN; e += NT) {
      const int which = e / BN, col = e % BN;
      float s = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WM; ++w2) s += red[(w2 * 2 + which) * BN + col];
      if (n0 + col < p.Ncol) {
        p.stats[((size_t)mt * 2 + which) * p.Ncol + n0 + col] = s;
      }
    }
  }
  stamp(kTraceSlots - 2);
  if (trace_on)
    __hip_atomic_store(&g_igemm_trace[(wv == 4) * kTraceSlots + kTraceSlots - 1], __builtin_amdgcn_s_memrealtime(),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// dW = Σ_split partial[split] (fp32); optional accumulate into dW. A block owns 64 float4
// columns; its 4 thread rows sum interleaved splits with 4 independent accumulators each
// (many loads in flight), then combine through LDS — deterministic order.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, long n4,
                                                            float* __restrict__ out, int accumulate) {
  __shared__ float4 red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + tx;
  const float4* P = reinterpret_cast<const float4*>(part);
  float4 a[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n4) {
    int k = ty;
    for (; k + 12 < splits; k += 16) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 u = ld16s<SDX_NT_PART != 0>(P + (size_t)(k + 4 * q) * n4 + e);
        const float4 v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
        a[q].x += v.x; a[q].y += v.y; a[q].z += v.z; a[q].w += v.w;
      }
    }
    for (; k < splits; k += 4) {
      const uint4 u = ld16s<SDX_NT_PART != 0>(P + (size_t)k * n4 + e);
      const float4 v = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  float4 s = a[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) { s.x += a[q].x; s.y += a[q].y; s.z += a[q].z; s.w += a[q].w; }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && e < n4) {
    float4 t = accumulate ? reinterpret_cast<const float4*>(out)[e] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 4; ++q) { t.x += red[q][tx].x; t.y += red[q][tx].y; t.z += red[q][tx].z; t.w += red[q][tx].w; }
    reinterpret_cast<float4*>(out)[e] = t;
  }
}

// register-prefetch depth of the K loop (SDX_IGEMM_DEPTH=1|2, default 2)
int igemm_depth() {
  static const int d = [] {
    const char* e = getenv("SDX_IGEMM_DEPTH");
    return (e && e[0] == '1') ? 1 : 2;
  }();
  return d;
}

// LDS-DMA operand staging: 0 off, 1 FWD/DGRAD (default), 2 FWD/DGRAD/WGRAD
int igemm_glds() {
  static const int a = [] {
    const char* e = getenv("SDX_IGEMM_GLDS");
    return e ? atoi(e) : 1;
  }();
  return a;
}

int igemm_trace_on() {
  static const int v = [] {
    const char* e = getenv("SDX_IGEMM_TRACE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int igemm_ablate() {
  static const int a = [] {
    const char* e = getenv("SDX_IGEMM_ABLATE");
    return e ? atoi(e) : 0;
  }();
  return a;
}

int igemm_worder() {
  static const int v = [] {
    const char* e = getenv("SDX_WGRAD_ORDER");
    return e ? atoi(e) : 1;
  }();
  return v;
}

int igemm_one() {
  static const int v = [] {
    const char* e = getenv("SDX_IGEMM_ONE");
    return e ? atoi(e) : 1;
  }();
  return v;
}
// longest reduction (GEMM K) run on the single-stage DEPTH 3 form: forward
// SDX_IGEMM_ONE_K (default 256), data gradient SDX_IGEMM_ONE_K_DGRAD (default BK = one
// K-tile, the only case before round 6). Up to 256 the forward 1x1 GEMMs gain 5-12 % (3
// blocks per CU instead of 2: l3.x.c3 32.1 -> 29.6 us, l2.x.c3 47.2 -> 42.3, stem 34.2 ->
// 28.7); the dgrads are mixed (l1.0.c3 61.9 -> 56.4, l3.0.c1 65.0 -> 71.3), and K = 512
// loses on both (profiles/one_stage_r6.txt)
std::atomic<int>& igemm_one_k_ref(int mode) {
  static std::atomic<int> f{[] {
    const char* e = getenv("SDX_IGEMM_ONE_K");
    return e ? atoi(e) : 256;
  }()};
  static std::atomic<int> d{[] {
    const char* e = getenv("SDX_IGEMM_ONE_K_DGRAD");
    return e ? atoi(e) : BK;
  }()};
  return mode == MODE_FWD ? f : d;
}
int igemm_one_k(int mode) { return igemm_one_k_ref(mode).load(std::memory_order_relaxed); }

template <int MODE, int BM, int BN, int WM, int WN, int DEPTH, int VAR>
hipError_t launch_v(bool one, int grid, const IgemmParams& p, hipStream_t s) {
  const dim3 g(grid), b(64 * WM * WN);
  if constexpr (DEPTH == 3) {
    if (one) {
      hipLaunchKernelGGL((igemm_kernel<MODE, BM, BN, WM, WN, DEPTH, VAR, true>), g, b, 0, s, p);
      SDX_LAUNCH_CHECK();
      return hipSuccess;
    }
  }
  hipLaunchKernelGGL((igemm_kernel<MODE, BM, BN, WM, WN, DEPTH, VAR, false>), g, b, 0, s, p);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

template <int MODE, int BM, int BN, int WM, int WN, int DEPTH>
hipError_t launch_k(bool bs, int grid, const IgemmParams& p, hipStream_t s) {
  // LDS-DMA main loops (DEPTH 3: two buffers; 6: in-wave pipelined ring; 7 / 8: tap reuse)
  // carry every epilogue variant; the single-stage (ONE) form is DEPTH 3 at one K-tile
  constexpr bool GLK = (DEPTH == 3 || DEPTH >= 6) && MODE != MODE_WGRAD;
  const bool one = DEPTH == 3 && p.Kdim <= igemm_one_k(MODE) && igemm_one();
  if (MODE == MODE_FWD && p.bn_sc != nullptr) {
    // block-output BN-apply epilogue (forward-folded BN3): LDS-DMA tiles only
    if constexpr (MODE == MODE_FWD && GLK) return launch_v<MODE, BM, BN, WM, WN, DEPTH, 2>(one, grid, p, s);
    return hipErrorInvalidValue;
  }
  if (bs && p.bs.store_masked) {
    // masked-store statistics variant (projection head, BN3 fold): LDS-DMA tiles only
    if constexpr (MODE == MODE_DGRAD && GLK) return launch_v<MODE, BM, BN, WM, WN, DEPTH, 2>(one, grid, p, s);
    return hipErrorInvalidValue;
  }
  if constexpr (MODE == MODE_DGRAD) {
    if (bs) return launch_v<MODE, BM, BN, WM, WN, DEPTH, 1>(one, grid, p, s);
  }
  return launch_v<MODE, BM, BN, WM, WN, DEPTH, 0>(one, grid, p, s);
}

// WGRAD launch of variant VAR (bit 0: 1x1 fast path, bit 1: BN prologue) at the depth
// launch_cfg picks for WGRAD
template <int BM, int BN, int WM, int WN, int VAR>
hipError_t launch_w(int grid, const IgemmParams& p, hipStream_t s) {
  const dim3 g(grid), b(64 * WM * WN);
  constexpr bool kDepth2 = BM == 64 && BN == 64;
  if (VAR < 2 && igemm_glds() == 2)
    hipLaunchKernelGGL((igemm_kernel<MODE_WGRAD, BM, BN, WM, WN, 3, VAR, false>), g, b, 0, s, p);
  else if (kDepth2 && igemm_depth() == 2)
    hipLaunchKernelGGL((igemm_kernel<MODE_WGRAD, BM, BN, WM, WN, kDepth2 ? 2 : 1, VAR, false>), g, b, 0, s, p);
  else
    hipLaunchKernelGGL((igemm_kernel<MODE_WGRAD, BM, BN, WM, WN, 1, VAR, false>), g, b, 0, s, p);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

template <int MODE, int BM, int BN, int WM, int WN>
hipError_t launch_cfg(IgemmParams p, hipStream_t s) {
  p.ablate = igemm_ablate();
  p.trace = igemm_trace_on();
  p.m_tiles = (p.M + BM - 1) / BM;
  p.n_tiles = (p.Ncol + BN - 1) / BN;
  int grid = p.m_tiles * p.n_tiles * (MODE == MODE_WGRAD ? p.splits : 1);
  if (MODE == MODE_DGRAD && p.ncls > 1) {
    // merged sub-pixel classes: class-major tiles, each class's BN-statistics slab rows after
    // the previous classes' (as the per-class launches advanced bs.row0)
    int most = 0, row = p.bs.row0;
    for (int c = 0; c < p.ncls; ++c) {
      IgemmParams::Cls& cd = p.cls[c];
      cd.m_tiles = (cd.M + BM - 1) / BM;
      cd.row0 = row;
      row += cd.m_tiles;
      cd.tile_end = cd.m_tiles * p.n_tiles;
      most = cd.tile_end > most ? cd.tile_end : most;
    }
    grid = most * p.ncls;
    if (grid == 0) return hipSuccess;
  }
  if constexpr (MODE == MODE_WGRAD) {
    const ConvGeom& g = p.g;
    const bool k1 = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;
    if (p.in_scale != nullptr) return launch_w<BM, BN, WM, WN, 2>(grid, p, s);
    if (k1) return launch_w<BM, BN, WM, WN, 1>(grid, p, s);
    return launch_w<BM, BN, WM, WN, 0>(grid, p, s);
  } else {
  // depth 2 only where the second register stage fits without spilling (checked with
  // -Rpass-analysis=kernel-resource-usage)
  constexpr bool kDepth2 = (BM == 64 && BN == 64) || (MODE == MODE_FWD && BM != 256);
  const bool bs = MODE == MODE_DGRAD && p.bs.slab != nullptr;
  {
    // 8-wave 256x128 / 128x256 tiles at more than two K-tiles whose channel dim (FWD C,
    // DGRAD K) is a multiple of BK (branch-free K decode): the in-wave pipelined loop (DEPTH 6)
    constexpr bool kW1 = WM * WN == 8 && BM * BN == 256 * 128;
    const int cdim_h = MODE == MODE_FWD ? p.g.C : p.g.K + p.a2_ch;
    const int taps_h = MODE == MODE_FWD ? p.g.R * p.g.S : p.nr * p.ns;
    const bool w1 = kW1 && p.Kdim > 2 * BK && p.in_scale == nullptr && cdim_h % BK == 0 && taps_h <= 32;
    if (p.in_scale == nullptr && igemm_glds() != 0) {
      if constexpr (kW1) {
        if (w1) return launch_k<MODE, BM, BN, WM, WN, 6>(bs, grid, p, s);
      }
      return launch_k<MODE, BM, BN, WM, WN, 3>(bs, grid, p, s);
    }
  }
  if (p.a2 != nullptr) return hipErrorInvalidValue;   // K-concatenation: LDS-DMA loops only
  if constexpr (kDepth2) {
    if (igemm_depth() == 2 && !bs) {
      hipLaunchKernelGGL((igemm_kernel<MODE, BM, BN, WM, WN, 2, 0, false>), dim3(grid), dim3(64 * WM * WN), 0, s, p);
      SDX_LAUNCH_CHECK();
      return hipSuccess;
    }
  }
  return launch_k<MODE, BM, BN, WM, WN, 1>(bs, grid, p, s);
  }
}

// Geometry of the tap-reuse loop (DEPTH 7 / 8) for a BM-row tile; false = not supported:
// a pad-1 3x3 stride-1 conv (DGRAD: the stride-1 class) whose tile rows are whole image
// rows of whole images or of one image band, a channel dim of 64-channel chunks and a window
// that fits the halo buffer. Swizzle phase t_ky: fragments of 16 output pixels span 1 row
// (W >= 16), 2 rows (W = 8: ky = 0) or 4 rows (W = 4: ky = 4) — conflict-free ds_read_b128
// lane groups for every tap (checked by brute force over the lane groups of the LDS table in
// MI355X_MICROARCH.md); other widths are correct, not conflict-free.
// SDX_TAP_PAD=0: no padded-row tiles (widths that do not divide BM stay on the implicit GEMM)
bool tap_pad_enabled() {
  static const bool on = [] {
    const char* e = getenv("SDX_TAP_PAD");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

bool tap_geom(IgemmParams& p, int bm, int depth, int mode) {
  const ConvGeom& g = p.g;
  if (g.R != 3 || g.S != 3 || g.stride != 1 || g.pad != 1 || g.P != g.H || g.Q != g.W) return false;
  if (mode == MODE_DGRAD && (p.ncls > 1 || p.ph != 0 || p.pw != 0 || p.nr != 3 || p.ns != 3)) return false;
  const int cdim = mode == MODE_FWD ? g.C : g.K;
  const int HW = g.H * g.W;
  if (cdim % 64 != 0) return false;
  p.t_rw = 0;
  int rw = g.W;
  if (bm % g.W != 0 || !(HW % bm == 0 || bm % HW == 0)) {
    // padded rows: a band of bm / rw whole image rows of rw = pow2 >= W virtual pixels each
    // (fragments of 16 virtual pixels stay inside one row: rw >= 16). Single-chunk DEPTH-8
    // tiles only: 56x56x64 fwd / dgrad 376 / 378 us vs 389 / 427 on the best implicit-GEMM
    // tile, but the 128-row DEPTH-7 tile at 28x28x128 runs 446 / 419 vs 258 / 266
    // (profiles/tap_pad_r6.txt, 1024 views)
    rw = 16;
    while (rw < g.W) rw <<= 1;
    if (!tap_pad_enabled() || depth != 8 || bm % rw != 0 || g.H % (bm / rw) != 0) return false;
    p.t_rw = rw;
  }
  p.t_rs = g.W + 2;
  p.t_imgs = (p.t_rw == 0 && bm >= HW) ? bm / HW : 0;
  const int rows = p.t_imgs > 0 ? g.H : bm / rw;
  p.t_is = (rows + 2) * p.t_rs;
  p.t_hp = (p.t_imgs > 0 ? p.t_imgs : 1) * p.t_is;
  p.t_nhp = (p.t_hp + 7) / 8;
  p.t_ky = g.W == 4 ? 4 : 0;
  p.t_nch = cdim / 64;
  if (p.t_nhp > tap_halo_kb(bm)) return false;
  // padded rows: the last row's padded fragments read up to pixel (rows + 1)·t_rs + rw + 1,
  // still inside the halo buffer
  if (p.t_rw > 0 && (rows + 1) * p.t_rs + rw + 2 > tap_halo_kb(bm) * 8) return false;
  if (bm == 256 && p.t_ky != 0) return false;   // the BM = 256 loop keeps 3 address variants
  if (depth == 8 && p.t_nch != 1) return false;
  return true;
}

template <int MODE, int BM, int BN, int WM, int WN, int DEPTH>
hipError_t launch_tap(IgemmParams p, hipStream_t s) {
  if (!tap_geom(p, BM, DEPTH, MODE)) return hipErrorInvalidValue;
  // the in-kernel statistics reduction and the BN+ReLU operand prologue are not built here
  if (p.in_scale != nullptr) return hipErrorInvalidValue;
  p.ablate = igemm_ablate();
  p.trace = igemm_trace_on();
  // (padded rows: the virtual rows tile exactly — H is a multiple of the band height)
  p.m_tiles = p.t_rw > 0 ? p.g.N * p.g.H * p.t_rw / BM : (p.M + BM - 1) / BM;
  p.n_tiles = (p.Ncol + BN - 1) / BN;
  const bool bs = MODE == MODE_DGRAD && p.bs.slab != nullptr;
  return launch_k<MODE, BM, BN, WM, WN, DEPTH>(bs, p.m_tiles * p.n_tiles, p, s);
}

// tile configs: 0 128x128 (2x2 waves of 64x64), 1 256x64 (4x1), 2 64x256 (1x4), 3 64x64 (2x2 waves of 32x32),
// 4 128x128 with 8 waves (2x4 of 64x32: twice the waves per SIMD for latency hiding),
// 5 256x128 with 8 waves (4x2 of 64x64, one block per CU), 6 128x256 with 8 waves (2x4 of
// 64x64); both run the in-wave pipelined loop (DEPTH 6, 144 KiB LDS ring) at K > 128.
// (7 / 8, 4-wave 64x128 wave tiles, measured slower than 5 / 6 in round 4 and removed.)
template <int MODE>
hipError_t launch_any(IgemmParams p, int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch_cfg<MODE, 128, 128, 2, 2>(p, s);
    case 1: return launch_cfg<MODE, 256, 64, 4, 1>(p, s);
    case 2: return launch_cfg<MODE, 64, 256, 1, 4>(p, s);
    case 3: return launch_cfg<MODE, 64, 64, 2, 2>(p, s);
    case 4: return launch_cfg<MODE, 128, 128, 2, 4>(p, s);
    case 5: return launch_cfg<MODE, 256, 128, 4, 2>(p, s);
    case 6: return launch_cfg<MODE, 128, 256, 2, 4>(p, s);
    // tap-reuse 3x3 (FWD / stride-1 DGRAD only): 11 256x64 with 4 waves of 64x64 and one halo
    // buffer (C = 64: two blocks per CU), 12 256x128 with 8 waves (4x2 of 64x64), 13 128x128
    // with 8 waves (2x4 of 64x32)
    case 11:
      if constexpr (MODE != MODE_WGRAD) return launch_tap<MODE, 256, 64, 4, 1, 8>(p, s);
      return hipErrorInvalidValue;
    case 12:
      if constexpr (MODE != MODE_WGRAD) return launch_tap<MODE, 256, 128, 4, 2, 7>(p, s);
      return hipErrorInvalidValue;
    case 13:
      if constexpr (MODE != MODE_WGRAD) return launch_tap<MODE, 128, 128, 2, 4, 7>(p, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

int igemm_tile_m(int cfg) {
  static const int m[14] = {128, 256, 64, 64, 128, 256, 128, 0, 0, 0, 0, 256, 256, 128};
  return (cfg >= 0 && cfg < 14) ? m[cfg] : 0;
}
int igemm_tile_n(int cfg) {
  static const int n[14] = {128, 64, 256, 64, 128, 128, 256, 0, 0, 0, 0, 64, 128, 128};
  return (cfg >= 0 && cfg < 14) ? n[cfg] : 0;
}

// tap-reuse tile config for a conv (FWD, or the stride-1 DGRAD with cdim = K, ncol = C), or -1
int igemm_tap_cfg(const ConvGeom& g, int cdim, int ncol) {
  if (g.R != 3 || g.S != 3 || g.stride != 1 || g.pad != 1 || cdim % 64 != 0) return -1;
  const int cands[3] = {cdim == 64 && ncol <= 64 ? 11 : -1, g.W >= 8 ? 12 : -1, 13};
  for (int cfg : cands) {
    if (cfg < 0) continue;
    IgemmParams p{};
    p.g = g;
    p.g.C = cdim;   // checked as a FWD geometry whose reduction channels are cdim
    if (tap_geom(p, igemm_tile_m(cfg), cfg == 11 ? 8 : 7, MODE_FWD)) return cfg;
  }
  return -1;
}

// M-tiles (statistics-slab rows) of a stride-1 fwd / dgrad conv of M output rows under cfg: a
// padded-row tap tile counts its virtual rows
int64_t igemm_conv_mtiles(const ConvGeom& g, int cdim, int cfg, int64_t M) {
  const int bm = igemm_tile_m(cfg);
  if (bm <= 0) return 0;
  if (cfg >= 11 && cfg <= 13) {
    IgemmParams p{};
    p.g = g;
    p.g.C = cdim;
    if (tap_geom(p, bm, cfg == 11 ? 8 : 7, MODE_FWD) && p.t_rw > 0) return (int64_t)g.N * g.H * p.t_rw / bm;
  }
  return (M + bm - 1) / bm;
}

namespace {
void set_epi(IgemmParams& p, const GemmEpi* epi) {
  if (epi == nullptr) return;
  p.bias = epi->bias;
  p.relu = epi->relu;
  p.out_f32 = epi->out_f32;
  p.add_pre = epi->add_pre;
  p.bn_sc = epi->bn_scale;
  p.bn_sh = epi->bn_shift;
  p.bn_rsc = epi->resid_scale;
  p.a2 = reinterpret_cast<const uint16_t*>(epi->cat_a);
  p.a2_ch = epi->cat_ch;
  p.bias_pre = epi->bias_pre;
  p.bn_rsh = epi->resid_shift;
  p.mask_out = epi->mask_out;
  if (epi->resid != nullptr) p.addend = reinterpret_cast<const uint16_t*>(epi->resid);
}
}  // namespace

hipError_t launch_conv_fwd(const ConvGeom& g, const void* x, const void* w, void* y, float* stats, int cfg,
                           hipStream_t s, const float* in_scale, const float* in_shift, const GemmEpi* epi) {
  IgemmParams p{};
  set_epi(p, epi);
  if (p.out_f32 && stats != nullptr) return hipErrorInvalidValue;
  // BN-apply epilogue: stride-1 1x1 geometry (the residual shares the output rows), no
  // statistics / fp32 output / bias; statistics-only pass: y == nullptr needs stats
  if (p.bn_sc != nullptr &&
      (p.bn_sh == nullptr || p.addend == nullptr || (p.bn_rsc == nullptr) != (p.bn_rsh == nullptr) ||
       stats != nullptr || p.out_f32 || p.bias != nullptr || p.relu || in_scale != nullptr || y == nullptr || g.R != 1 || g.S != 1 || g.stride != 1 || g.pad != 0))
    return hipErrorInvalidValue;
  if (y == nullptr && (stats == nullptr || p.bn_sc != nullptr)) return hipErrorInvalidValue;
  p.in_scale = in_scale;
  p.in_shift = in_shift;
  p.g = g;
  p.a = (const uint16_t*)x;
  p.b = (const uint16_t*)w;
  p.out = y;
  p.stats = stats;
  p.M = g.N * g.P * g.Q;
  p.Ncol = g.K;
  p.Kdim = g.R * g.S * g.C;
  p.b_row = p.Kdim;
  p.b_t0 = 0;
  p.b_tr = g.S * g.C;
  p.b_ts = g.C;
  p.a_elems = (long)g.N * g.H * g.W * g.C;
  p.b_elems = (long)p.Ncol * p.Kdim;
  return launch_any<MODE_FWD>(p, cfg, s);
}

void conv_dgrad_class(const ConvGeom& g, int ph, int pw, int* r0, int* nr, int* s0, int* ns, int* Hc, int* Wc) {
  const int st = g.stride;
  *r0 = (ph + g.pad) % st;
  *s0 = (pw + g.pad) % st;
  *nr = *r0 < g.R ? (g.R - *r0 + st - 1) / st : 0;
  *ns = *s0 < g.S ? (g.S - *s0 + st - 1) / st : 0;
  *Hc = ph < g.H ? (g.H - ph + st - 1) / st : 0;
  *Wc = pw < g.W ? (g.W - pw + st - 1) / st : 0;
}

int conv_dgrad_class_mtiles(const ConvGeom& g, int ph, int pw, int cfg) {
  int r0, nr, s0, ns, Hc, Wc;
  conv_dgrad_class(g, ph, pw, &r0, &nr, &s0, &ns, &Hc, &Wc);
  const int M = g.N * Hc * Wc, bm = igemm_tile_m(cfg);
  if (g.stride == 1) return (int)igemm_conv_mtiles(g, g.K, cfg, M);   // (a tap tile may pad rows)
  return (M + bm - 1) / bm;
}

// K-concatenated dgrad [dy | a2]·[Wd ; Mx] (BN3 fold): a stride-1 unpadded 1x1 whose dy
// width is a power-of-two multiple of a2's (both multiples of BK), on the LDS-DMA loops
bool conv_dgrad_cat_supported(const ConvGeom& g, int cat_ch) {
  if (cat_ch <= 0 || g.R != 1 || g.S != 1 || g.stride != 1 || g.pad != 0 || g.P != g.H || g.Q != g.W) return false;
  if (g.K % BK != 0 || cat_ch % BK != 0 || g.K % cat_ch != 0) return false;
  const unsigned r = (unsigned)(g.K / cat_ch);
  return (r & (r - 1)) == 0 && igemm_glds() != 0;
}

hipError_t launch_conv_dgrad_class(const ConvGeom& g, int ph, int pw, const void* dy, const void* wt, void* dx,
                                   const void* addend, int cfg, hipStream_t s, const void* addend_mask,
                                   const BnBwdStat* bstat, int addend_sub, const GemmEpi* epi) {
  IgemmParams p{};
  set_epi(p, epi);
  if (p.out_f32 && (g.stride != 1 || addend != nullptr || (bstat != nullptr && bstat->slab != nullptr)))
    return hipErrorInvalidValue;
  p.addend_sub = addend_sub;
  if (bstat != nullptr) p.bs = *bstat;
  p.addend_mask = (const uint8_t*)addend_mask;
  p.g = g;
  p.a = (const uint16_t*)dy;
  p.b = (const uint16_t*)wt;   // the full Wt [C][R][S][K]; the class's taps are strided into it
  p.out = dx;
  p.addend = (const uint16_t*)addend;
  p.ph = ph;
  p.pw = pw;
  conv_dgrad_class(g, ph, pw, &p.r0, &p.nr, &p.s0, &p.ns, &p.Hc, &p.Wc);
  p.M = g.N * p.Hc * p.Wc;
  if (p.M == 0) return hipSuccess;
  p.Ncol = g.C;
  p.Kdim = p.nr * p.ns * g.K;
  p.b_row = g.R * g.S * g.K;
  if (p.a2 != nullptr || p.a2_ch != 0) {
    if (p.a2 == nullptr || !conv_dgrad_cat_supported(g, p.a2_ch)) return hipErrorInvalidValue;
    p.a2_sh = __builtin_ctz((unsigned)(g.K / p.a2_ch));
    p.a2_elems = (long)g.N * g.P * g.Q * p.a2_ch;
    p.Kdim += p.a2_ch;
    p.b_row += p.a2_ch;
  }
  if (p.bias_pre != nullptr && (g.stride != 1 || (reinterpret_cast<uintptr_t>(p.bias_pre) & 15) != 0))
    return hipErrorInvalidValue;
  p.b_t0 = (p.r0 * g.S + p.s0) * g.K;
  p.b_tr = g.stride * g.S * g.K;
  p.b_ts = g.stride * g.K;
  p.a_elems = (long)g.N * g.P * g.Q * g.K;
  p.b_elems = (long)p.Ncol * p.b_row;
  return launch_any<MODE_DGRAD>(p, cfg, s);
}

hipError_t launch_conv_dgrad_merged(const ConvGeom& g, const void* dy, const void* wt, void* dx, const void* addend,
                                    int cfg, hipStream_t s, const void* addend_mask, const BnBwdStat* bstat,
                                    int addend_sub) {
  const int st = g.stride;
  if (st < 2 || st * st > 4) return hipErrorInvalidValue;
  IgemmParams p{};
  p.addend_sub = addend_sub;
  if (bstat != nullptr) p.bs = *bstat;
  p.addend_mask = (const uint8_t*)addend_mask;
  p.g = g;
  p.a = (const uint16_t*)dy;
  p.b = (const uint16_t*)wt;
  p.out = dx;
  p.addend = (const uint16_t*)addend;
  p.Ncol = g.C;
  p.b_row = g.R * g.S * g.K;
  p.b_tr = st * g.S * g.K;
  p.b_ts = st * g.K;
  p.a_elems = (long)g.N * g.P * g.Q * g.K;
  p.b_elems = (long)p.Ncol * p.b_row;
  // classes with more taps first (longest blocks dispatched first)
  int order[4], n = 0;
  for (int ph = 0; ph < st; ++ph)
    for (int pw = 0; pw < st; ++pw) order[n++] = ph * st + pw;
  auto taps = [&](int id) {
    int r0, nr, s0, ns, Hc, Wc;
    conv_dgrad_class(g, id / st, id % st, &r0, &nr, &s0, &ns, &Hc, &Wc);
    return nr * ns;
  };
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && taps(order[j]) > taps(order[j - 1]); --j) std::swap(order[j], order[j - 1]);
  int maxk = 0, maxm = 0, maxt = 0, nc = 0;
  for (int i = 0; i < n; ++i) {
    IgemmParams::Cls& cd = p.cls[nc];
    cd.ph = order[i] / st;
    cd.pw = order[i] % st;
    conv_dgrad_class(g, cd.ph, cd.pw, &cd.r0, &cd.nr, &cd.s0, &cd.ns, &cd.Hc, &cd.Wc);
    cd.M = g.N * cd.Hc * cd.Wc;
    if (cd.M == 0) continue;
    cd.Kdim = cd.nr * cd.ns * g.K;
    cd.b_t0 = (cd.r0 * g.S + cd.s0) * g.K;
    maxk = cd.Kdim > maxk ? cd.Kdim : maxk;
    maxm = cd.M > maxm ? cd.M : maxm;
    maxt = cd.nr * cd.ns > maxt ? cd.nr * cd.ns : maxt;
    ++nc;
  }
  if (nc == 0) return hipSuccess;
  p.ncls = nc;
  // launch-level choices (main loop, single-stage form) see the largest class; the per-class
  // fields below are the first class's (every block overwrites them with its own)
  const IgemmParams::Cls& c0 = p.cls[0];
  p.ph = c0.ph; p.pw = c0.pw; p.Hc = c0.Hc; p.Wc = c0.Wc; p.r0 = c0.r0; p.s0 = c0.s0;
  p.nr = c0.nr; p.ns = c0.ns; p.b_t0 = c0.b_t0;
  p.M = maxm;
  p.Kdim = maxk;
  (void)maxt;
  return launch_any<MODE_DGRAD>(p, cfg, s);
}

int conv_wgrad_splits(const ConvGeom& g, int cfg, int splits) {
  const int Kd = g.N * g.P * g.Q;
  if (splits < 1) splits = 1;
  int per = (Kd + splits - 1) / splits;
  per = ((per + BK - 1) / BK) * BK;
  return (Kd + per - 1) / per;
}

hipError_t launch_conv_wgrad(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int cfg,
                             int splits, int accumulate, hipStream_t s, const float* in_scale,
                             const float* in_shift) {
  IgemmParams p{};
  p.in_scale = in_scale;
  p.in_shift = in_shift;
  p.g = g;
  p.a = (const uint16_t*)dy;
  p.b = (const uint16_t*)x;
  p.M = g.K;
  p.Ncol = g.R * g.S * g.C;
  p.Kdim = g.N * g.P * g.Q;
  p.a_elems = (long)g.N * g.P * g.Q * g.K;
  p.b_elems = (long)g.N * g.H * g.W * g.C;
  if (splits < 1) splits = 1;
  int per = (p.Kdim + splits - 1) / splits;
  per = ((per + BK - 1) / BK) * BK;
  p.k_per_split = per;
  p.splits = (p.Kdim + per - 1) / per;
  p.div_pq = make_fastdiv((unsigned)(g.P * g.Q));
  p.div_q = make_fastdiv((unsigned)g.Q);
  auto log2_exact = [](int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return (1 << l) == v ? l : -1;
  };
  p.worder = igemm_worder();
  p.lq = log2_exact(g.Q);
  p.lpq = log2_exact(g.P * g.Q);
  if (p.lq < 0 || p.lpq < 0) p.lq = p.lpq = -1;
  // a single split writes straight into dW (unless accumulating)
  const bool direct = p.splits == 1 && !accumulate;
  p.out = direct ? (void*)dw : (void*)partial;
  hipError_t e = launch_any<MODE_WGRAD>(p, cfg, s);
  if (e != hipSuccess || direct) return e;
  return launch_splitk_reduce(partial, p.splits, (long)p.M * p.Ncol / 4, dw, accumulate, s);
}

// Deferred split-K reductions (SplitkDefer, launchers.h): while a stream is registered, the
// reductions launched on it are queued and later issued as ONE multi-tensor launch
// (splitk_flush), block b of which serves job j = the first with b < tiles_end[j] — a
// residual block's 3-4 weight gradients become one reduction launch instead of 3-4.
namespace {
constexpr int kMaxSplitkJobs = 16;
struct SplitkJobs {
  const float* part[kMaxSplitkJobs];
  float* dw[kMaxSplitkJobs];
  long n4[kMaxSplitkJobs];
  int splits[kMaxSplitkJobs];
  int acc[kMaxSplitkJobs];
  int tiles_end[kMaxSplitkJobs];
  int n;
};
thread_local hipStream_t g_defer_stream = nullptr;
thread_local SplitkJobs g_jobs{};

__global__ __launch_bounds__(256) void splitk_reduce_multi_kernel(SplitkJobs jobs) {
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.tiles_end[j]) ++j;
  const int b = blockIdx.x - (j ? jobs.tiles_end[j - 1] : 0);
  __shared__ float4 red[4][64];
  const float* __restrict__ part = jobs.part[j];
  const long n4 = jobs.n4[j];
  const int splits = jobs.splits[j];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long e = (long)b * 64 + tx;
  const float4* P = reinterpret_cast<const float4*>(part);
  float4 a[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n4) {
    int k = ty;
    for (; k + 12 < splits; k += 16) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = P[(size_t)(k + 4 * q) * n4 + e];
        a[q].x += v.x; a[q].y += v.y; a[q].z += v.z; a[q].w += v.w;
      }
    }
    for (; k < splits; k += 4) {
      const float4 v = P[(size_t)k * n4 + e];
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  float4 sm = a[0];
#pragma unroll
  for (int q = 1; q < 4; ++q) { sm.x += a[q].x; sm.y += a[q].y; sm.z += a[q].z; sm.w += a[q].w; }
  red[ty][tx] = sm;
  __syncthreads();
  if (ty == 0 && e < n4) {
    float4* out = reinterpret_cast<float4*>(jobs.dw[j]);
    float4 t = jobs.acc[j] ? out[e] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 4; ++q) { t.x += red[q][tx].x; t.y += red[q][tx].y; t.z += red[q][tx].z; t.w += red[q][tx].w; }
    out[e] = t;
  }
}
}  // namespace

void splitk_defer_begin(hipStream_t s) {
  g_defer_stream = s;
  g_jobs.n = 0;
}

bool splitk_deferring(hipStream_t s) { return g_defer_stream != nullptr && s == g_defer_stream; }

void splitk_defer_cancel() {
  g_defer_stream = nullptr;
  g_jobs.n = 0;
}

hipError_t splitk_flush() {
  hipStream_t s = g_defer_stream;
  g_defer_stream = nullptr;
  if (g_jobs.n == 0) return hipSuccess;
  const int grid = g_jobs.tiles_end[g_jobs.n - 1];
  hipLaunchKernelGGL(splitk_reduce_multi_kernel, dim3(grid), dim3(256), 0, s, g_jobs);
  g_jobs.n = 0;
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

hipError_t launch_splitk_reduce(const float* partial, int splits, long n4, float* dw, int accumulate, hipStream_t s) {
  if (splitk_deferring(s)) {
    // the queued jobs run unordered in one launch: a second job into the same sink would race
    // its read-modify-write with the first (a shared or tied weight) — issue the queue first
    bool dup = false;
    for (int i = 0; i < g_jobs.n; ++i) dup = dup || g_jobs.dw[i] == dw;
    if (g_jobs.n == kMaxSplitkJobs || dup) {
      // queue full: issue what is queued and keep deferring
      hipStream_t keep = g_defer_stream;
      const hipError_t e = splitk_flush();
      if (e != hipSuccess) return e;
      splitk_defer_begin(keep);
    }
    const int i = g_jobs.n++;
    g_jobs.part[i] = partial;
    g_jobs.dw[i] = dw;
    g_jobs.n4[i] = n4;
    g_jobs.splits[i] = splits;
    g_jobs.acc[i] = accumulate;
    g_jobs.tiles_end[i] = (i ? g_jobs.tiles_end[i - 1] : 0) + (int)((n4 + 63) / 64);
    return hipSuccess;
  }
  const long grid = (n4 + 63) / 64;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, s, partial, splits, n4, dw, accumulate);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

// the BN-apply epilogue runs on the LDS-DMA tiles, not the register-staged ones
bool conv_fwd_bnapply_supported() { return igemm_glds() != 0; }

// the diagnostic timeline of the last traced launch (SDX_IGEMM_TRACE=1): 2 x kTraceSlots u64
int igemm_trace_slots() { return kTraceSlots; }
hipError_t igemm_trace_copy(unsigned long long* host, hipStream_t s) {
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_igemm_trace), sizeof(unsigned long long) * 2 * kTraceSlots, 0,
                             hipMemcpyDeviceToHost);
}

// single-stage reduction limits at run time (tests, A/B): mode 0 forward, 1 data gradient;
// returns the previous limit
int igemm_one_k_set(int mode, int k) { return igemm_one_k_ref(mode == 0 ? MODE_FWD : MODE_DGRAD).exchange(k); }
