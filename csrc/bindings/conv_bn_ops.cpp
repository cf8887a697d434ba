// Bindings for the implicit-GEMM convolution (igemm.hip) and BatchNorm (bn.hip) kernels.
// Host-side shape/dtype/layout checks run before every launch.
#include "ops_decl.h"
#include "conv_internal.h"
#include "launchers.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <atomic>
#include <cmath>
#include <map>
#include <mutex>

namespace sdx_bind {

using OptT = c10::optional<torch::Tensor>;

void check_bf16_nhwc(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(), name, " must be a contiguous 4-D (NHWC) tensor");
  TORCH_CHECK(t.size(3) % 8 == 0, name, ": channel count must be a multiple of 8");
  TORCH_CHECK(t.numel() < (1LL << 31), name, " too large for 32-bit GEMM indexing");
}

void check_vec(const torch::Tensor& t, int64_t C, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == C, name,
              " must be a contiguous float32 GPU vector of length C");
}

const float* opt_ptr(const OptT& t, int64_t C, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_vec(*t, C, name);
  return t->data_ptr<float>();
}

// fused BN+ReLU input prologue: both vectors or neither
void in_bn_ptrs(const OptT& sc, const OptT& sh, int64_t C, const float** ps, const float** pt) {
  *ps = opt_ptr(sc, C, "in_scale");
  *pt = opt_ptr(sh, C, "in_shift");
  TORCH_CHECK((*ps == nullptr) == (*pt == nullptr), "in_scale and in_shift must be given together");
}

// Pick the tile config (0 128x128, 1 256x64, 2 64x256, 3 64x64) minimising
//   padded work x per-config efficiency penalty x grid fill,
// where fill = (launch rounds x resident slots) / tiles charges a grid that leaves CUs idle
// in its last round (e.g. M=8192 x N=512: 256 tiles of 128x128 fill only half of the 512
// two-per-CU slots). The small 64x64 tile is only penalised when the GEMM is
// compute-bound (long K); short-K (memory-bound) GEMMs favour its higher occupancy.
// Calibrated with tools/conv_bench.py --cfg 0..3 on the ResNet-50 shapes.
// SDX_CONV_CFG=c pins the fwd/dgrad tile config (tests): the BN-statistics epilogue's per-tile
// fp32 partial sums then cover the same rows whatever the per-rank batch, so a W-rank step
// reproduces the single-rank statistics bit for bit (tests/test_gpu_dist.py)
int pinned_cfg() {
  static const int pinned = [] {
    const char* e = getenv("SDX_CONV_CFG");
    const int v = e != nullptr ? atoi(e) : -1;
    return v >= 0 && v <= 8 ? v : -1;
  }();
  return pinned;
}

// fwd / dgrad tile config of a conv: the tap-reuse 3x3 loop where it applies (pad-1 stride-1
// 3x3; not with a pinned config, the in-kernel statistics reduction or the BN+ReLU operand
// prologue), else auto_cfg. SDX_TAP3=0 disables it. Per shape (tools/tap3_sweep.py,
// profiles/tap3_r5.txt) it beats the best implicit-GEMM tile at every CIFAR ResNet-50 3x3:
// fwd / dgrad l1 52 / 51 vs 67 / 68 us, l2 45 / 42 vs 47 / 45, l3 34 / 34 vs 38 / 37,
// l4 38 / 38 vs 58 / 56
std::atomic<int>& tap3_flag() {
  static std::atomic<int> on{[] {
    const char* e = getenv("SDX_TAP3");
    return e == nullptr ? 1 : atoi(e);
  }()};
  return on;
}

// runtime switch of the tap-reuse loop (tests / in-process A/B); returns the previous value
int64_t tap3_set(int64_t on) { return tap3_flag().exchange((int)on); }

//
// Then per-pass corrections to auto_cfg from the round-5 re-calibration (every fwd / dgrad
// of the CIFAR ResNet-50 at 512 views under every tile config, the dgrads with their
// BN-statistics epilogue: tools/cfg_sweep.py, profiles/cfg_sweep_r5.txt; 5.32 -> 5.24 ms
// summed stand-alone). Three corrections won stand-alone; in the step (bench A/B, same box,
// SDX_CFG_RULES bit mask) only bit 4 does, so it alone is on by default:
//  1 the 128x256 DEPTH-6 tile only when it fills the chip (>= 256 tiles): l4 1x1 / strided
//    3x3 fwd at M = 8192 on the 8-wave 128x128 (52.8 vs 58.1 us) — neutral in the step;
//  2 expanding stride-1 dgrads (dx has >= 256 and >= twice the reduction's channels) on the
//    64x256 tile (l1 137.8 vs 146.3 us) — +0.05 ms in the step (12.21 vs 12.155 ms): more
//    blocks per CU under the heavy epilogue is exactly what the side-stream wgrads lose;
//  4 strided dgrads with 256-multiple outputs on DEPTH 6 (l3.0 3x3 84.4 vs 90.4 us, l3.0
//    shortcut 127.3 vs 135.9) — -0.03 ms in the step (12.12 vs 12.155)
int conv_cfg(const ConvGeom& g, int cdim, int ncol, int64_t M, int64_t Kdim, bool plain, bool dgrad) {
  if (tap3_flag().load(std::memory_order_relaxed) > 0 && plain && pinned_cfg() < 0) {
    const int t = igemm_tap_cfg(g, cdim, ncol);
    if (t >= 0) return t;
  }
  int cfg = auto_cfg(M, ncol, Kdim, true);
  static const int rules = [] {   // SDX_CFG_RULES: bit mask of the corrections below (A/B)
    const char* e = getenv("SDX_CFG_RULES");
    return e == nullptr ? 4 : atoi(e);
  }();
  if (pinned_cfg() >= 0) return cfg;
  auto tiles = [&](int c) { return ((M + igemm_tile_m(c) - 1) / igemm_tile_m(c)) * ((ncol + igemm_tile_n(c) - 1) / igemm_tile_n(c)); };
  if ((rules & 1) && cfg == 6 && tiles(6) < 256) cfg = 4;
  if ((rules & 2) && dgrad && g.stride == 1 && ncol >= 256 && 2 * Kdim <= ncol) cfg = 2;
  if ((rules & 4) && dgrad && g.stride > 1 && ncol % 256 == 0 && Kdim * g.stride * g.stride >= 1024) cfg = 6;
  return cfg;
}

int auto_cfg(int64_t M, int64_t Ncol, int64_t Kdim, bool fill) {
  const int pinned = pinned_cfg();
  if (fill && pinned >= 0) return pinned;
  const int64_t bm[4] = {128, 256, 64, 64}, bn[4] = {128, 64, 256, 64};
  const bool long_k = Kdim == 0 || Kdim > 256;
  const double pen_long[4] = {1.0, 1.04, 1.04, 1.35}, pen_short[4] = {1.0, 1.0, 1.0, 1.05};
  const double slots[4] = {512, 512, 512, 1280};   // resident blocks chip-wide (LDS/VGPR-limited)
  int best = 0;
  double best_s = 1e300;
  for (int c = 0; c < 4; ++c) {
    const int64_t mt = (M + bm[c] - 1) / bm[c], nt = (Ncol + bn[c] - 1) / bn[c];
    const double padded = (double)(mt * bm[c]) * (double)(nt * bn[c]);
    double f = 1.0;
    if (fill) {
      const double tiles = (double)(mt * nt);
      f = std::ceil(tiles / slots[c]) * slots[c] / tiles;
    }
    const double sc = padded * (long_k ? pen_long[c] : pen_short[c]) * f;
    if (sc < best_s) { best_s = sc; best = c; }
  }
  // fwd/dgrad: the 8-wave 128x128 tile (cfg 4, 2x4 waves of 64x32) beats the 4-wave one by
  // 3-12% on every ResNet-50 shape with a reduction of >= 128 (more waves hide the LDS-DMA
  // and epilogue latency); on the K=64 layer-1 GEMMs its longer prologue costs more than it
  // hides. wgrad keeps the 4-wave tiles (its split-K slabs are short). profiles/conv_cfg4_r1.txt
  if (fill && best == 0 && Kdim >= 128) best = 4;
  // long-K GEMMs whose output width is a multiple of 256 (layers 3-4): the 8-wave 128x256 tile
  // on the in-wave pipelined LDS-DMA ring (cfg 6, DEPTH 6) — l3 3x3 fwd/dgrad 41.3 -> 38.1 us,
  // l4.0.sc dgrad 67.5 -> 64.8 us; it loses on narrower or short-K GEMMs, where one tile per CU
  // leaves its prologue/epilogue exposed (profiles/conv_core_r4.txt)
  static const bool d6 = [] {
    const char* e = getenv("SDX_CONV_D6");
    return e == nullptr || atoi(e) != 0;
  }();
  if (fill && d6 && Ncol % 256 == 0 && Kdim >= 1024) best = 6;
  return best;
}

namespace {

// no_out: statistics only, the output is not stored (first pass of a forward-folded BN3)
std::vector<torch::Tensor> conv_fwd_impl(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad,
                                         bool want_stats, int64_t cfg, OptT in_scale, OptT in_shift,
                                         const GemmEpi* epi = nullptr, bool no_out = false) {
  check_bf16_nhwc(x, "x");
  check_bf16_nhwc(w, "w");
  TORCH_CHECK(w.size(3) == x.size(3), "weight Cin != input C");
  TORCH_CHECK(stride >= 1 && pad >= 0, "bad stride/pad");
  ConvGeom g{};
  g.N = x.size(0); g.H = x.size(1); g.W = x.size(2); g.C = x.size(3);
  g.K = w.size(0); g.R = w.size(1); g.S = w.size(2);
  g.stride = stride; g.pad = pad;
  g.P = (g.H + 2 * pad - g.R) / stride + 1;
  g.Q = (g.W + 2 * pad - g.S) / stride + 1;
  TORCH_CHECK(g.P > 0 && g.Q > 0, "empty output");
  TORCH_CHECK(g.K % 8 == 0, "Cout must be a multiple of 8");
  c10::DeviceGuard dg(x.device());
  const int64_t M = (int64_t)g.N * g.P * g.Q;
  if (cfg < 0)
    cfg = conv_cfg(g, g.C, g.K, M, (int64_t)g.R * g.S * g.C, !in_scale.has_value(), false);
  TORCH_CHECK(!no_out || (want_stats && epi == nullptr), "statistics-only conv: stats, no epilogue");
  auto y = no_out ? torch::Tensor() : torch::empty({g.N, g.P, g.Q, g.K}, x.options());
  torch::Tensor slab;
  float* sp = nullptr;
  if (want_stats) {
    const int64_t mt = g.stride == 1 ? igemm_conv_mtiles(g, g.C, (int)cfg, M)
                                     : (M + igemm_tile_m(cfg) - 1) / igemm_tile_m(cfg);
    slab = torch::empty({mt, 2, g.K}, x.options().dtype(at::kFloat));
    sp = slab.data_ptr<float>();
  } else {
    slab = torch::empty({0}, x.options().dtype(at::kFloat));
  }
  const float *isc, *ish;
  in_bn_ptrs(in_scale, in_shift, g.C, &isc, &ish);
  check_hip(launch_conv_fwd(g, x.data_ptr(), w.data_ptr(), no_out ? nullptr : y.data_ptr(), sp, (int)cfg, cur_stream(),
                            isc, ish, epi),
            "conv_fwd");
  return {y, slab};
}

// conv with a per-output-channel fp32 bias (+ ReLU) applied to the fp32 accumulators before
// the bf16 rounding, no statistics: an eval-mode conv + BatchNorm (+ ReLU) with the BN
// folded into the weights and the bias (linear-probe encoder, ops/linear_probe.py)
torch::Tensor conv_fwd_bias(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, torch::Tensor bias,
                            bool relu) {
  check_vec(bias, w.size(0), "bias");
  GemmEpi epi{};
  epi.bias = bias.data_ptr<float>();
  epi.relu = relu ? 1 : 0;
  return conv_fwd_impl(x, w, stride, pad, false, -1, c10::nullopt, c10::nullopt, &epi)[0];
}

std::vector<torch::Tensor> conv_fwd(torch::Tensor x, torch::Tensor w, int64_t stride, int64_t pad, bool want_stats,
                                    int64_t cfg, OptT in_scale, OptT in_shift) {
  return conv_fwd_impl(x, w, stride, pad, want_stats, cfg, in_scale, in_shift);
}

// bs (optional): fused BN-backward statistics; its slab must hold conv_dgrad_slab_rows rows
// set around the BN3 fold's conv3 dgrad (block_bwd): its T addend is added before rounding
int& fold_add_pre() {
  thread_local int on = 0;
  return on;
}

// scoped fold_add_pre(): restored on every exit path, so an exception inside a folded
// dgrad can never leave later dgrads on this thread in pre-rounding add mode
struct AddPreScope {
  int saved;
  AddPreScope() : saved(fold_add_pre()) { fold_add_pre() = 1; }
  ~AddPreScope() { fold_add_pre() = saved; }
  AddPreScope(const AddPreScope&) = delete;
  AddPreScope& operator=(const AddPreScope&) = delete;
};

// K-concatenated BN3-fold dgrad (igemm.hip a2): the next stride-1 1x1 dgrad on this thread
// reduces over [dy | a2] with wt = [Wd | Mx] ([C][1][1][K + K2]) and adds the fp32 bias
// before rounding — da2 = dz·Wd + a2·Mx + b in one GEMM instead of a separate T = a2·Mx + b
// GEMM whose bf16 output the dgrad epilogue re-reads. Scoped like AddPreScope.
struct FoldCat {
  const torch::Tensor* a2 = nullptr;
  const torch::Tensor* bias = nullptr;
};
FoldCat& fold_cat() {
  thread_local FoldCat c;
  return c;
}
struct CatScope {
  FoldCat saved;
  CatScope(const torch::Tensor& a2, const torch::Tensor& bias) : saved(fold_cat()) { fold_cat() = {&a2, &bias}; }
  ~CatScope() { fold_cat() = saved; }
  CatScope(const CatScope&) = delete;
  CatScope& operator=(const CatScope&) = delete;
};

torch::Tensor conv_dgrad_impl(torch::Tensor dy, torch::Tensor wt, int64_t H, int64_t W, int64_t stride, int64_t pad,
                              int64_t cfg, c10::optional<torch::Tensor> out, c10::optional<torch::Tensor> addend,
                              c10::optional<torch::Tensor> addend_mask, BnBwdStat* bs, int64_t addend_sub = 0) {
  check_bf16_nhwc(dy, "dy");
  check_bf16_nhwc(wt, "wt");
  const FoldCat cat = fold_cat();
  fold_cat() = FoldCat{};   // consumed by this dgrad only
  const int64_t cat_ch = cat.a2 != nullptr ? cat.a2->size(3) : 0;
  TORCH_CHECK(wt.size(3) == dy.size(3) + cat_ch, "wt last dim must be Cout (+ the concatenated operand's channels)");
  if (cat.a2 != nullptr) {
    check_bf16_nhwc(*cat.a2, "cat a2");
    TORCH_CHECK(stride == 1 && pad == 0 && wt.size(1) == 1 && wt.size(2) == 1 && !addend.has_value() &&
                    cat.a2->size(0) == dy.size(0) && cat.a2->size(1) == dy.size(1) && cat.a2->size(2) == dy.size(2),
                "K-concatenated dgrad: stride-1 1x1, no addend, a2 on dy's pixels");
    TORCH_CHECK(cat.bias->is_cuda() && cat.bias->scalar_type() == at::kFloat && cat.bias->is_contiguous() &&
                    cat.bias->numel() == wt.size(0),
                "K-concatenated dgrad: fp32 bias [C]");
  }
  ConvGeom g{};
  g.N = dy.size(0); g.P = dy.size(1); g.Q = dy.size(2); g.K = dy.size(3);
  g.C = wt.size(0); g.R = wt.size(1); g.S = wt.size(2);
  g.H = H; g.W = W; g.stride = stride; g.pad = pad;
  TORCH_CHECK((g.H + 2 * pad - g.R) / stride + 1 == g.P && (g.W + 2 * pad - g.S) / stride + 1 == g.Q,
              "dgrad geometry mismatch");
  TORCH_CHECK(g.C % 8 == 0, "Cin must be a multiple of 8");
  c10::DeviceGuard dg(dy.device());
  const int64_t M = (int64_t)g.N * g.H * g.W / (stride * stride);
  if (cfg < 0) cfg = conv_cfg(g, g.K, g.C, M, (int64_t)g.R * g.S * (g.K + cat_ch) / (stride * stride), true, true);
  torch::Tensor dx;
  if (out.has_value()) {
    dx = *out;
    check_bf16_nhwc(dx, "out");
    TORCH_CHECK(dx.size(0) == g.N && dx.size(1) == g.H && dx.size(2) == g.W && dx.size(3) == g.C, "out shape");
  } else {
    dx = torch::empty({g.N, g.H, g.W, g.C}, dy.options());
  }
  const void* add = nullptr;
  TORCH_CHECK(addend_sub >= 0, "addend_sub");
  if (addend.has_value()) {
    check_bf16_nhwc(*addend, "addend");
    if (addend_sub > 1) {
      // compact addend on the stride-s subgrid (h, w ≡ 0 mod s)
      const int64_t s_ = addend_sub;
      TORCH_CHECK(addend->size(0) == g.N && addend->size(1) == (g.H + s_ - 1) / s_ &&
                      addend->size(2) == (g.W + s_ - 1) / s_ && addend->size(3) == g.C,
                  "compact addend shape [N, ceil(H/s), ceil(W/s), C]");
      TORCH_CHECK(!addend_mask.has_value(), "addend_mask is not supported with a compact addend");
    } else {
      TORCH_CHECK(addend->sizes() == dx.sizes(), "addend shape");
    }
    add = addend->data_ptr();
  }
  const void* amask = nullptr;
  if (addend_mask.has_value()) {
    TORCH_CHECK(add != nullptr, "addend_mask needs an addend");
    TORCH_CHECK(addend_mask->is_cuda() && addend_mask->scalar_type() == at::kByte && addend_mask->is_contiguous() &&
                    addend_mask->numel() * 8 == dx.numel(),
                "addend_mask: uint8 [numel/8]");
    amask = addend_mask->data_ptr();
  }
  if (bs) bs->row0 = 0;
  if (stride == 1) {
    // BN3 fold: the addend joins the accumulators before rounding (kernels built with SDX_ADD_PRE)
    static const GemmEpi pre{nullptr, 0, 0, 1};
    const GemmEpi* epi = (fold_add_pre() && add != nullptr && addend_sub == 0 && amask == nullptr) ? &pre : nullptr;
    GemmEpi ce{};
    if (cat.a2 != nullptr) {
      ce.cat_a = cat.a2->data_ptr();
      ce.cat_ch = (int)cat_ch;
      ce.bias_pre = cat.bias->data_ptr<float>();
      epi = &ce;
    }
    check_hip(launch_conv_dgrad_class(g, 0, 0, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), add, (int)cfg,
                                      cur_stream(), amask, bs, add ? (int)addend_sub : 0, epi),
              "conv_dgrad");
    return dx;
  }
  // sub-pixel classes: each gets the taps r ≡ ph+pad, s ≡ pw+pad (mod stride); by default all
  // of them in one launch (SDX_DGRAD_MERGE=0: one launch per class)
  // SDX_DGRAD_MERGE: 0 one launch per class, 1 merged for every strided dgrad, 2 merged for
  // strided 3x3 only (default: a strided 1x1 has one non-empty class, whose launch is faster
  // on its own — profiles/dgrad_merge_r4.txt)
  static const int merge = [] {
    const char* e = getenv("SDX_DGRAD_MERGE");
    return e == nullptr ? 2 : atoi(e);
  }();
  if (stride == 2 && (merge == 1 || (merge == 2 && g.R > 1))) {
    check_hip(launch_conv_dgrad_merged(g, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), add, (int)cfg, cur_stream(),
                                       amask, bs, add ? (int)addend_sub : 0),
              "conv_dgrad(merged classes)");
    return dx;
  }
  for (int ph = 0; ph < stride; ++ph)
    for (int pw = 0; pw < stride; ++pw) {
      // each class reads its taps straight from the full Wt (no per-class weight copy; a
      // class without taps writes zeros and never reads B)
      check_hip(launch_conv_dgrad_class(g, ph, pw, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), add, (int)cfg,
                                        cur_stream(), amask, bs, add ? (int)addend_sub : 0),
                "conv_dgrad(class)");
      if (bs) bs->row0 += conv_dgrad_class_mtiles(g, ph, pw, (int)cfg);
    }
  return dx;
}

torch::Tensor conv_dgrad(torch::Tensor dy, torch::Tensor wt, int64_t H, int64_t W, int64_t stride, int64_t pad,
                         int64_t cfg, c10::optional<torch::Tensor> out, c10::optional<torch::Tensor> addend,
                         c10::optional<torch::Tensor> addend_mask, int64_t addend_sub = 0) {
  return conv_dgrad_impl(dy, wt, H, W, stride, pad, cfg, out, addend, addend_mask, nullptr, addend_sub);
}

// dgrad + fused BN-backward statistics of dx for the BN whose pre-BN tensor is ya (and yb,
// a second BN fed by the same gradient: projection shortcut). ReLU mask from `mask_bits`
// (1 bit per element) or recomputed as ya·msc + msh > 0. Returns [dx, slab [rows][2|3][C]].
std::vector<torch::Tensor> conv_dgrad_bnstat_impl(torch::Tensor dy, torch::Tensor wt, int64_t H, int64_t W,
                                                  int64_t stride, int64_t pad, int64_t cfg, OptT out, OptT addend,
                                                  OptT addend_mask, torch::Tensor ya, torch::Tensor ma, OptT yb,
                                                  OptT mb, OptT mask_bits, OptT msc, OptT msh, int64_t addend_sub,
                                                  int store_masked = 0, int64_t extra_rows = 0) {
  const int64_t C = wt.size(0);
  // an empty ya: the BN input was never stored (forward-folded BN3) — the epilogue sums
  // Σdz and Σdz·(0 − μ); the caller fills extra_rows rows of the slab with the Σdz·y terms
  const bool no_y = !ya.defined() || ya.numel() == 0;
  const int64_t elems = dy.size(0) * H * W * C;
  if (!no_y) {
    check_bf16_nhwc(ya, "ya");
    TORCH_CHECK(ya.size(0) == dy.size(0) && ya.size(1) == H && ya.size(2) == W && ya.size(3) == C, "ya shape");
  }
  TORCH_CHECK(extra_rows >= 0 && (!no_y || !msc.has_value()), "no-ya statistics: ReLU mask from bits");
  check_vec(ma, C, "ma");
  BnBwdStat bs{};
  bs.ya = no_y ? nullptr : ya.data_ptr();
  bs.ma = ma.data_ptr<float>();
  if (yb.has_value()) {
    check_bf16_nhwc(*yb, "yb");
    TORCH_CHECK(yb->size(0) == dy.size(0) && yb->size(1) == H && yb->size(2) == W && yb->size(3) == C, "yb shape");
    TORCH_CHECK(mb.has_value(), "mb required with yb");
    check_vec(*mb, C, "mb");
    bs.yb = yb->data_ptr();
    bs.mb = mb->data_ptr<float>();
  }
  if (mask_bits.has_value()) {
    TORCH_CHECK(mask_bits->is_cuda() && mask_bits->scalar_type() == at::kByte && mask_bits->is_contiguous() &&
                    mask_bits->numel() * 8 == elems,
                "mask_bits: uint8 [numel/8]");
    bs.mask = mask_bits->data_ptr<uint8_t>();
  } else if (msc.has_value()) {
    TORCH_CHECK(msh.has_value(), "msh required with msc");
    check_vec(*msc, C, "msc");
    check_vec(*msh, C, "msh");
    bs.msc = msc->data_ptr<float>();
    bs.msh = msh->data_ptr<float>();
  }
  ConvGeom g{};
  g.N = dy.size(0); g.P = dy.size(1); g.Q = dy.size(2); g.K = dy.size(3);
  g.C = C; g.R = wt.size(1); g.S = wt.size(2);
  g.H = H; g.W = W; g.stride = stride; g.pad = pad;
  const int64_t M = (int64_t)g.N * g.H * g.W / (stride * stride);
  const int64_t cat_ch = fold_cat().a2 != nullptr ? fold_cat().a2->size(3) : 0;   // (CatScope)
  if (cfg < 0) cfg = conv_cfg(g, g.K, g.C, M, (int64_t)g.R * g.S * (g.K + cat_ch) / (stride * stride), true, true);
  int rows = 0;
  for (int ph = 0; ph < stride; ++ph)
    for (int pw = 0; pw < stride; ++pw) rows += conv_dgrad_class_mtiles(g, ph, pw, (int)cfg);
  const int ns = yb.has_value() ? 3 : 2;
  auto slab = torch::empty({rows + extra_rows, ns, C}, dy.options().dtype(at::kFloat));
  bs.slab = slab.data_ptr<float>();
  TORCH_CHECK(!store_masked || (mask_bits.has_value() && stride == 1), "store_masked: stride-1 with a ReLU bitmask");
  bs.store_masked = store_masked;
  auto dx = conv_dgrad_impl(dy, wt, H, W, stride, pad, cfg, out, addend, addend_mask, &bs, addend_sub);
  return {dx, slab};
}

std::vector<torch::Tensor> conv_dgrad_bnstat(torch::Tensor dy, torch::Tensor wt, int64_t H, int64_t W,
                                             int64_t stride, int64_t pad, int64_t cfg, OptT out, OptT addend,
                                             OptT addend_mask, torch::Tensor ya, torch::Tensor ma, OptT yb, OptT mb,
                                             OptT mask_bits, OptT msc, OptT msh, int64_t addend_sub = 0,
                                             int store_masked = 0, int64_t extra_rows = 0) {
  return conv_dgrad_bnstat_impl(dy, wt, H, W, stride, pad, cfg, out, addend, addend_mask, ya, ma, yb, mb, mask_bits,
                                msc, msh, addend_sub, store_masked, extra_rows);
}

}  // namespace

// tensors read by side-stream wgrads, released after the join (no recordStream: blocks
// return to the allocator in program order instead of behind side-stream events)
std::vector<torch::Tensor>& side_stash() {
  static std::vector<torch::Tensor> v;
  return v;
}

// a split-K slab whose reduction was queued (splitk_defer_begin) stays alive until the side
// stream is joined (side_stash), i.e. past its deferred reduction launch
void keep_deferred_partial(const torch::Tensor& part) {
  if (part.defined() && splitk_deferring(cur_stream())) side_stash().push_back(part);
}

// block target of the dedicated 1x1 / 3x3 wgrad kernels' split heuristic: SDX_W3_BLOCKS
// (default 128, half the chip: the eager step runs them on the side stream beside the
// critical path). A step captured as one hipGraph chain runs them alone, in line, so
// PretrainEngine.enable_cuda_graph raises it to the whole chip for the capture
// (wgrad_block_target_set).
std::atomic<int64_t>& wgrad_block_target_ref() {
  static std::atomic<int64_t> t{[] {
    const char* e = getenv("SDX_W3_BLOCKS");
    return e ? atoll(e) : 128LL;
  }()};
  return t;
}
int64_t wgrad_block_target() { return wgrad_block_target_ref().load(std::memory_order_relaxed); }
int64_t wgrad_block_target_set(int64_t n) {
  TORCH_CHECK(n >= 1 && n <= 4096, "block target in [1, 4096]");
  return wgrad_block_target_ref().exchange(n);
}

torch::Tensor conv_wgrad(torch::Tensor dy, torch::Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                         int64_t splits, int64_t cfg, c10::optional<torch::Tensor> out, bool accumulate,
                         OptT in_scale, OptT in_shift) {
  check_bf16_nhwc(dy, "dy");
  check_bf16_nhwc(x, "x");
  TORCH_CHECK(dy.size(0) == x.size(0), "batch mismatch");
  ConvGeom g{};
  g.N = x.size(0); g.H = x.size(1); g.W = x.size(2); g.C = x.size(3);
  g.P = dy.size(1); g.Q = dy.size(2); g.K = dy.size(3);
  g.R = R; g.S = S; g.stride = stride; g.pad = pad;
  TORCH_CHECK((g.H + 2 * pad - R) / stride + 1 == g.P && (g.W + 2 * pad - S) / stride + 1 == g.Q,
              "wgrad geometry mismatch");
  c10::DeviceGuard dg(x.device());
  const int64_t M = g.K, Ncol = (int64_t)R * S * g.C, Kd = (int64_t)g.N * g.P * g.Q;
  // cfg 9 = the tap-reuse 3x3 kernel (wgrad3x3.hip), which auto (cfg -1) picks for every
  // shape it supports (SDX_WGRAD3=0: generic implicit GEMM only); cfg -2 = generic auto
  static const bool w3_on = [] {
    const char* e = getenv("SDX_WGRAD3");
    return e == nullptr || atoi(e) != 0;
  }();
  const bool w3 = (cfg == 9 || (cfg == -1 && w3_on && splits <= 0)) && !in_scale.has_value() && wgrad3x3_supported(g);
  TORCH_CHECK(cfg != 9 || w3, "conv_wgrad: cfg 9 needs a pad-1 3x3 conv of stride 1 or 2 on square images with output width in {4,8,16,32}, C,K % 64 == 0");
  // cfg 10 = the stride-1 1x1 kernel (wgrad1x1.hip), auto-picked for every shape it supports
  // (SDX_WGRAD1=0: generic only)
  static const bool w1_on = [] {
    const char* e = getenv("SDX_WGRAD1");
    return e == nullptr || atoi(e) != 0;
  }();
  const bool w1 = (cfg == 10 || (cfg == -1 && w1_on && splits <= 0)) && !in_scale.has_value() && wgrad1x1_supported(g);
  TORCH_CHECK(cfg != 10 || w1, "conv_wgrad: cfg 10 needs a 1x1 conv with K,C % 128 == 0 (stride 1, or stride s with H = s*P, W = s*Q), or stride 1 with K or C = 64");
  // 64-output-channel GEMMs with a wide reduction side (layer-1 3x3: 64 x 576): the 64x256
  // tile (four 64x64 wave tiles) beats the exact-fit 64x64 one despite its padding, at
  // ~512 blocks (tools/wgrad_split_probe.py: 145 -> 124 us)
  static const bool wide64 = [] {
    const char* e = getenv("SDX_WGRAD_WIDE64");
    return e == nullptr || atoi(e) != 0;
  }();
  // The stage-1 weight gradients (the most pixels) are the last work of the backward: when
  // they run, the main stream has (almost) nothing left, so the half-chip block target that
  // keeps the side stream off the critical-path kernels only leaves CUs idle in the step's
  // tail (profiles: a 390 us gap before the SGD at 256 images/GPU). GEMMs with at least
  // SDX_W3_TAIL_PIX pixels (2^18 = stage 1 at 128 and 256 images/GPU) get
  // SDX_W3_TAIL_BLOCKS (default 256) blocks. Default 0 (off): the gap shrinks to 180 us but
  // the wider stage-1 wgrads slow the concurrent stage-1 dgrads more, 12.43 vs 12.37 ms
  // (512 blocks: 12.52; same-box A/B, profiles/tail_ab_r4.txt)
  static const int64_t tail_pix = [] {
    const char* e = getenv("SDX_W3_TAIL_PIX");
    return e ? atoll(e) : 0LL;
  }();
  static const int64_t tail_blocks = [] {
    const char* e = getenv("SDX_W3_TAIL_BLOCKS");
    return e ? atoll(e) : 256LL;
  }();
  const bool tail = tail_pix > 0 && Kd >= tail_pix;
  if (w1) {
    // as for the 3x3 kernel: SDX_W3_BLOCKS (128) 8-wave blocks, >= 8 steps each
    const int64_t steps = wgrad1x1_steps(g);
    if (splits <= 0) {
      const int64_t target0 = wgrad_block_target();
      // pixel-pair shapes (HBM-bound, twice the MFMA work per byte): SDX_W1_PAIR_BLOCKS
      static const int64_t pair_target = [] {
        const char* e = getenv("SDX_W1_PAIR_BLOCKS");
        return e ? atoll(e) : 256LL;
      }();
      const int64_t target = tail ? tail_blocks : (wgrad1x1_pair_view(g) ? pair_target : target0);
      splits = std::max<int64_t>(1, target / wgrad1x1_tiles(g));
      splits = std::min(splits, std::max<int64_t>(1, steps / 8));
    }
    const int64_t per = (steps + splits - 1) / splits;
    splits = (steps + per - 1) / per;
  } else if (w3) {
    if (splits <= 0) {
      // SDX_W3_BLOCKS (default 128) 8-wave blocks, >= 8 steps per split. Standalone, 256
      // blocks (one per CU) is fastest (tools/w3_sweep.py), but in the training step these
      // kernels run on the wgrad side stream: a block holds ~416 of a SIMD lane's 512 VGPRs,
      // so the critical-path kernels (128-VGPR dgrads, the BN reductions) cannot co-reside on
      // its CU. 128 blocks leave half the CUs to the main stream: step 13.71 -> 13.34 ms at
      // 256 images/GPU, 8.48 -> 8.20 ms at 128 (profiles/wgrad3x3_r2.txt)
      const int64_t target0 = wgrad_block_target();
      const int64_t target = tail ? tail_blocks : target0;
      const int64_t tiles = wgrad3x3_tiles(g), steps = wgrad3x3_steps(g);
      splits = std::max<int64_t>(1, target / tiles);
      splits = std::min(splits, std::max<int64_t>(1, steps / 8));
    }
    const int64_t steps = wgrad3x3_steps(g);
    const int64_t per = (steps + splits - 1) / splits;
    splits = (steps + per - 1) / per;
  } else {
    if (wide64 && cfg < 0 && splits <= 0 && M <= 64 && Ncol >= 512) cfg = 2;
    if (cfg < 0) cfg = auto_cfg(M, Ncol);
    if (splits <= 0) {
      const int64_t tiles = ((M + igemm_tile_m(cfg) - 1) / igemm_tile_m(cfg)) *
                            ((Ncol + igemm_tile_n(cfg) - 1) / igemm_tile_n(cfg));
      // SDX_WGRAD_TARGET: block target of the generic wgrad split heuristic (default 512)
      static const int64_t gen_target = [] {
        const char* e = getenv("SDX_WGRAD_TARGET");
        return e ? atoll(e) : 512LL;
      }();
      splits = std::max<int64_t>(1, gen_target / tiles);
      const int64_t max_splits = std::max<int64_t>(1, Kd / 512);   // >= 8 K-tiles per split
      splits = std::min(splits, max_splits);
      // bound the fp32 partial slab to ~64 MiB, and to ~16 MiB / 256 splits for 1x1 GEMMs with
      // a small output (M*Ncol <= 64K: the layer-1/2 pointwise convs), where the slab round
      // trip outweighs the extra splits' parallelism (profiles/wgrad_sweep_r1.txt: 83 -> 67 us
      // on the 256x64 layer-1 GEMMs; the 3x3 and larger GEMMs keep more splits)
      const bool small_1x1 = R == 1 && S == 1 && M * Ncol <= 65536;
      splits = std::min<int64_t>(splits, std::max<int64_t>(1, (small_1x1 ? (4LL << 20) : (16LL << 20)) / (M * Ncol)));
      if (small_1x1) splits = std::min<int64_t>(splits, 256);
    }
    splits = conv_wgrad_splits(g, (int)cfg, (int)splits);
  }
  torch::Tensor dw;
  if (out.has_value()) {
    dw = *out;
    TORCH_CHECK(dw.is_cuda() && dw.scalar_type() == at::kFloat && dw.numel() == M * Ncol, "out: fp32 [K,R,S,C]");
    const bool krsc = dw.dim() == 4 && ((dw.size(0) == g.K && dw.size(1) == g.C && dw.size(2) == R &&
                                         dw.is_contiguous(at::MemoryFormat::ChannelsLast)) ||
                                        (dw.size(1) == R && dw.size(3) == g.C && dw.is_contiguous()));
    TORCH_CHECK(krsc, "out must be KRSC-contiguous (channels_last [K,C,R,S] or contiguous [K,R,S,C])");
  } else {
    dw = torch::empty({g.K, R, S, g.C}, x.options().dtype(at::kFloat));
    accumulate = false;
  }
  const float *isc, *ish;
  in_bn_ptrs(in_scale, in_shift, g.C, &isc, &ish);
  torch::Tensor part;
  const int64_t slices = w1 ? wgrad1x1_slices(g, (int)splits) : splits;
  if (slices > 1 || accumulate)
    part = torch::empty({slices * M * Ncol}, x.options().dtype(at::kFloat));
  if (w1) {
    check_hip(launch_wgrad1x1(g, dy.data_ptr(), x.data_ptr(), part.defined() ? part.data_ptr<float>() : nullptr,
                              dw.data_ptr<float>(), (int)splits, accumulate ? 1 : 0, cur_stream()),
              "conv_wgrad(1x1)");
    keep_deferred_partial(part);
    return dw;
  }
  if (w3) {
    check_hip(launch_wgrad3x3(g, dy.data_ptr(), x.data_ptr(), part.defined() ? part.data_ptr<float>() : nullptr,
                              dw.data_ptr<float>(), (int)splits, accumulate ? 1 : 0, cur_stream()),
              "conv_wgrad(3x3)");
    keep_deferred_partial(part);
    return dw;
  }
  check_hip(launch_conv_wgrad(g, dy.data_ptr(), x.data_ptr(), part.defined() ? part.data_ptr<float>() : nullptr,
                              dw.data_ptr<float>(), (int)cfg, (int)splits, accumulate ? 1 : 0, cur_stream(), isc, ish),
            "conv_wgrad");
  keep_deferred_partial(part);
  return dw;
}

// Ticket counters of the single-launch column reduction: zeroed once per device, reset by
// each launch's last block; consecutive launches rotate through slots so launches on
// different streams never share a counter.
// nslots consecutive slots: one per emulated rank of a fused SyncBN exchange (XgmiCol mode 2)
unsigned* reduce_counters(const torch::Device& dev, int nslots) {
  constexpr int kSlots = 256, kPerSlot = 64;   // 64 column groups = 4096 channels
  TORCH_CHECK(nslots >= 1 && nslots <= kXgmiMaxPeers, "counter slots");
  static std::mutex mu;
  static std::map<int, std::pair<torch::Tensor, int>> pool;
  std::lock_guard<std::mutex> lk(mu);
  auto& e = pool[dev.index()];
  if (!e.first.defined())
    e.first = torch::zeros({kSlots * kPerSlot}, torch::TensorOptions().dtype(at::kInt).device(dev));
  int slot = e.second;
  if (slot + nslots > kSlots) slot = 0;
  e.second = (slot + nslots) % kSlots;
  return reinterpret_cast<unsigned*>(e.first.data_ptr<int>()) + slot * kPerSlot;
}

void check_slab(const torch::Tensor& slab, int64_t nsets) {
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.dim() == 3 && slab.size(1) == nsets &&
                  slab.is_contiguous(),
              "slab must be [rows, ", nsets, ", C] float32");
  TORCH_CHECK(slab.size(2) <= 4096, "C <= 4096");
}

torch::Tensor reduce_scratch(const torch::Tensor& like, int64_t rows, int64_t nsets, int64_t C, int z) {
  return torch::empty({z * col_reduce_gy((int)rows) * nsets * C}, like.options().dtype(at::kDouble));
}

// the fused SyncBN exchange of one BN (xGMI communicators; csrc/kernels/bn.hip XgmiCol)
FusedX fused_exchange(int64_t comm) {
  FusedX f;
  if (comm != 0) f.on = small_comm_fused(comm, &f.x);
  return f;
}

namespace {

torch::Tensor bn_stats_reduce(torch::Tensor slab) {
  check_slab(slab, 2);
  c10::DeviceGuard dg(slab.device());
  const int64_t rows = slab.size(0), C = slab.size(2);
  auto out = torch::empty({2, C}, slab.options().dtype(at::kDouble));
  auto scratch = reduce_scratch(slab, rows, 2, C);
  check_hip(launch_col_reduce(slab.data_ptr<float>(), rows, 2, C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device()), out.data_ptr<double>(), 0, nullptr, nullptr,
                              cur_stream()),
            "bn_stats_reduce");
  return out;
}

struct FinalizeOut {
  torch::Tensor scale, shift, mean, invstd;
};

BnFinalizeArgs finalize_args(const torch::Tensor& like, int64_t C, double count, const OptT& gamma, const OptT& beta,
                             double eps, double momentum, bool update, const OptT& running_mean,
                             const OptT& running_var, FinalizeOut& o) {
  BnFinalizeArgs a{};
  a.count = count;
  a.gamma = opt_ptr(gamma, C, "gamma");
  a.beta = opt_ptr(beta, C, "beta");
  a.eps = (float)eps;
  a.momentum = (float)momentum;
  a.update_running = update ? 1 : 0;
  if (update) {
    TORCH_CHECK(running_mean.has_value() && running_var.has_value(), "running stats required for update");
    check_vec(*running_mean, C, "running_mean");
    check_vec(*running_var, C, "running_var");
    a.running_mean = running_mean->data_ptr<float>();
    a.running_var = running_var->data_ptr<float>();
  }
  auto fo = like.options().dtype(at::kFloat);
  o.scale = torch::empty({C}, fo);
  o.shift = torch::empty({C}, fo);
  o.mean = torch::empty({C}, fo);
  o.invstd = torch::empty({C}, fo);
  a.scale = o.scale.data_ptr<float>();
  a.shift = o.shift.data_ptr<float>();
  a.mean = o.mean.data_ptr<float>();
  a.invstd = o.invstd.data_ptr<float>();
  return a;
}

std::vector<torch::Tensor> bn_finalize(torch::Tensor sums, double count, OptT gamma, OptT beta, double eps,
                                       double momentum, bool update, OptT running_mean, OptT running_var) {
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.dim() == 2 && sums.size(0) == 2 &&
                  sums.is_contiguous(),
              "sums must be [2, C] float64");
  const int64_t C = sums.size(1);
  c10::DeviceGuard dg(sums.device());
  FinalizeOut o;
  const BnFinalizeArgs a =
      finalize_args(sums, C, count, gamma, beta, eps, momentum, update, running_mean, running_var, o);
  check_hip(launch_bn_finalize(sums.data_ptr<double>(), C, a, cur_stream()), "bn_finalize");
  return {o.scale, o.shift, o.mean, o.invstd};
}

// conv stat slab -> (scale, shift, mean, invstd) in ONE launch (no cross-rank reduction)
// fx (fused SyncBN exchange): the sums are exchanged across ranks inside the same launch
// and `count` must be the global row count
std::vector<torch::Tensor> bn_stats_finalize_x(torch::Tensor slab, double count, OptT gamma, OptT beta, double eps,
                                               double momentum, bool update, OptT running_mean, OptT running_var,
                                               const FusedX* fx) {
  check_slab(slab, 2);
  c10::DeviceGuard dg(slab.device());
  const int64_t rows = slab.size(0), C = slab.size(2);
  FinalizeOut o;
  const BnFinalizeArgs a =
      finalize_args(slab, C, count, gamma, beta, eps, momentum, update, running_mean, running_var, o);
  auto sums = torch::empty({2, C}, slab.options().dtype(at::kDouble));
  const int z = fx ? fx->z() : 1;
  auto scratch = reduce_scratch(slab, rows, 2, C, z);
  check_hip(launch_col_reduce(slab.data_ptr<float>(), rows, 2, C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device(), z), sums.data_ptr<double>(), 1, &a, nullptr, cur_stream(),
                              fx ? fx->p() : nullptr),
            "bn_stats_finalize");
  return {o.scale, o.shift, o.mean, o.invstd};
}

std::vector<torch::Tensor> bn_stats_finalize(torch::Tensor slab, double count, OptT gamma, OptT beta, double eps,
                                             double momentum, bool update, OptT running_mean, OptT running_var) {
  return bn_stats_finalize_x(slab, count, gamma, beta, eps, momentum, update, running_mean, running_var, nullptr);
}

std::vector<torch::Tensor> bn_eval_affine(OptT gamma, OptT beta, torch::Tensor rm, torch::Tensor rv, double eps) {
  const int64_t C = rm.numel();
  check_vec(rm, C, "running_mean");
  check_vec(rv, C, "running_var");
  c10::DeviceGuard dg(rm.device());
  auto scale = torch::empty({C}, rm.options()), shift = torch::empty({C}, rm.options());
  check_hip(launch_bn_eval_affine(C, opt_ptr(gamma, C, "gamma"), opt_ptr(beta, C, "beta"), rm.data_ptr<float>(),
                                  rv.data_ptr<float>(), (float)eps, scale.data_ptr<float>(), shift.data_ptr<float>(),
                                  cur_stream()),
            "bn_eval_affine");
  return {scale, shift};
}

// ReLU bitmask of an activation: uint8 [numel/8], bit i of byte e = value 8e+i > 0
void check_mask(const torch::Tensor& m, int64_t numel, const char* name) {
  TORCH_CHECK(m.is_cuda() && m.scalar_type() == at::kByte && m.is_contiguous() && m.numel() * 8 == numel, name,
              " must be a contiguous uint8 GPU tensor of numel/8 bytes");
}

torch::Tensor bn_apply(torch::Tensor y, torch::Tensor scale, torch::Tensor shift, OptT r, OptT scale2, OptT shift2,
                       int64_t res_mode, bool relu, OptT mask_out) {
  check_bf16_nhwc(y, "y");
  const int64_t C = y.size(3);
  check_vec(scale, C, "scale");
  check_vec(shift, C, "shift");
  const void* rp = nullptr;
  const float *s2 = nullptr, *t2 = nullptr;
  TORCH_CHECK(res_mode >= 0 && res_mode <= 2, "res_mode");
  if (res_mode != 0) {
    TORCH_CHECK(r.has_value(), "residual tensor required");
    check_bf16_nhwc(*r, "residual");
    TORCH_CHECK(r->sizes() == y.sizes(), "residual shape mismatch");
    rp = r->data_ptr();
    if (res_mode == 1) {
      s2 = opt_ptr(scale2, C, "scale2");
      t2 = opt_ptr(shift2, C, "shift2");
      TORCH_CHECK(s2 && t2, "scale2/shift2 required for res_mode 1");
    }
  }
  c10::DeviceGuard dg(y.device());
  auto out = torch::empty_like(y);
  void* mp = nullptr;
  if (mask_out.has_value()) {
    check_mask(*mask_out, y.numel(), "mask_out");
    mp = mask_out->data_ptr();
  }
  check_hip(launch_bn_apply(y.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(), rp, s2, t2, (int)res_mode,
                            relu ? 1 : 0, out.data_ptr(), y.numel(), C, cur_stream(), mp),
            "bn_apply");
  return out;
}

void check_bwd_C(int64_t C) {
  TORCH_CHECK(C <= 2048 && (C & (C - 1)) == 0 && C >= 8, "bn backward supports power-of-two C in [8, 2048]");
}

struct BwdIn {
  const void* op = nullptr;
  const void* om = nullptr;   // ReLU bitmask instead of the activation
  const void* ybp = nullptr;
  const float* mbp = nullptr;
  const float* mk_s = nullptr;
  const float* mk_t = nullptr;
  int64_t C = 0;
};

BwdIn bwd_inputs(const torch::Tensor& dout, const OptT& outv, const torch::Tensor& ya, const torch::Tensor& ma,
                 const OptT& yb, const OptT& mb, const OptT& msc, const OptT& msh) {
  BwdIn in;
  check_bf16_nhwc(dout, "dout");
  check_bf16_nhwc(ya, "ya");
  in.C = dout.size(3);
  check_bwd_C(in.C);
  TORCH_CHECK(ya.sizes() == dout.sizes(), "ya shape");
  check_vec(ma, in.C, "mean_a");
  if (outv.has_value()) {
    if (outv->scalar_type() == at::kByte) {
      check_mask(*outv, dout.numel(), "out (bitmask)");
      in.om = outv->data_ptr();
    } else {
      check_bf16_nhwc(*outv, "out");
      TORCH_CHECK(outv->sizes() == dout.sizes(), "out shape");
      in.op = outv->data_ptr();
    }
  }
  if (yb.has_value()) {
    check_bf16_nhwc(*yb, "yb");
    TORCH_CHECK(yb->sizes() == dout.sizes(), "yb shape");
    TORCH_CHECK(mb.has_value(), "mean_b required");
    check_vec(*mb, in.C, "mean_b");
    in.ybp = yb->data_ptr();
    in.mbp = mb->data_ptr<float>();
  }
  in_bn_ptrs(msc, msh, in.C, &in.mk_s, &in.mk_t);
  return in;
}

// ReLU mask: from the stored activation `outv`, or (outv None, msc/msh given) recomputed as
// ya·msc + msh > 0 for an activation that was never materialised
torch::Tensor bn_bwd_reduce(torch::Tensor dout, OptT outv, torch::Tensor ya, torch::Tensor ma, OptT yb, OptT mb,
                            OptT msc, OptT msh) {
  const BwdIn in = bwd_inputs(dout, outv, ya, ma, yb, mb, msc, msh);
  c10::DeviceGuard dg(dout.device());
  const int64_t C = in.C;
  const int nsets = in.ybp ? 3 : 2;
  const int g = bn_bwd_reduce_blocks(dout.numel(), C);
  auto sums = torch::empty({nsets, C}, dout.options().dtype(at::kDouble));
  auto partial = torch::empty({g, nsets, C}, dout.options().dtype(at::kFloat));
  auto scratch = reduce_scratch(dout, g, nsets, C);
  check_hip(launch_bn_bwd_reduce(dout.data_ptr(), in.op, ya.data_ptr(), ma.data_ptr<float>(), in.ybp, in.mbp,
                                 dout.numel(), C, partial.data_ptr<float>(), scratch.data_ptr<double>(),
                                 reduce_counters(dout.device()), sums.data_ptr<double>(), 0, nullptr, cur_stream(),
                                 in.mk_s, in.mk_t, in.om),
            "bn_bwd_reduce");
  return sums;
}

struct CoefOut {
  torch::Tensor coef_a, coef_b, dga, dba, dgb, dbb;
};

// dγ/dβ go to freshly allocated tensors, or are ADDED into caller-provided gradient
// sinks (sink_ga, sink_ba, sink_gb, sink_bb: the parameters' .grad views).
BnCoefArgs coef_args(const torch::Tensor& like, int64_t C, int nsets, double count, const OptT& g_a,
                     const torch::Tensor& mean_a, const torch::Tensor& inv_a, const OptT& g_b, const OptT& mean_b,
                     const OptT& inv_b, const OptT& sink_ga, const OptT& sink_ba, const OptT& sink_gb,
                     const OptT& sink_bb, CoefOut& o, double grad_scale = 1.0) {
  TORCH_CHECK(nsets == 1 || nsets == 2, "1 or 2 BN sets");
  check_vec(mean_a, C, "mean_a");
  check_vec(inv_a, C, "inv_a");
  auto fo = like.options().dtype(at::kFloat);
  const bool sinks = sink_ga.has_value();
  TORCH_CHECK(!sinks || (sink_ba.has_value() && (nsets == 1 || (sink_gb.has_value() && sink_bb.has_value()))),
              "all gradient sinks must be given together");
  BnCoefArgs a{};
  a.count = count;
  a.accumulate = sinks ? 1 : 0;
  a.grad_scale = grad_scale;
  o.coef_a = torch::empty({3, C}, fo);
  o.dga = sinks ? *sink_ga : torch::empty({C}, fo);
  o.dba = sinks ? *sink_ba : torch::empty({C}, fo);
  if (sinks) {
    check_vec(o.dga, C, "sink_ga");
    check_vec(o.dba, C, "sink_ba");
  }
  a.g_a = opt_ptr(g_a, C, "g_a");
  a.mean_a = mean_a.data_ptr<float>();
  a.inv_a = inv_a.data_ptr<float>();
  a.coef_a = o.coef_a.data_ptr<float>();
  a.dgamma_a = o.dga.data_ptr<float>();
  a.dbeta_a = o.dba.data_ptr<float>();
  if (nsets == 2) {
    o.coef_b = torch::empty({3, C}, fo);
    o.dgb = sinks ? *sink_gb : torch::empty({C}, fo);
    o.dbb = sinks ? *sink_bb : torch::empty({C}, fo);
    if (sinks) {
      check_vec(o.dgb, C, "sink_gb");
      check_vec(o.dbb, C, "sink_bb");
    }
    a.g_b = opt_ptr(g_b, C, "g_b");
    a.mean_b = opt_ptr(mean_b, C, "mean_b");
    a.inv_b = opt_ptr(inv_b, C, "inv_b");
    TORCH_CHECK(a.mean_b && a.inv_b, "mean_b/inv_b required");
    a.coef_b = o.coef_b.data_ptr<float>();
    a.dgamma_b = o.dgb.data_ptr<float>();
    a.dbeta_b = o.dbb.data_ptr<float>();
  } else {
    o.coef_b = o.dgb = o.dbb = torch::empty({0}, fo);
  }
  return a;
}

std::vector<torch::Tensor> bn_bwd_coef(torch::Tensor sums, double count, OptT g_a, torch::Tensor mean_a,
                                       torch::Tensor inv_a, OptT g_b, OptT mean_b, OptT inv_b, OptT sink_ga,
                                       OptT sink_ba, OptT sink_gb, OptT sink_bb, double grad_scale = 1.0) {
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.dim() == 2 && sums.is_contiguous(),
              "sums must be [nsets+1, C] float64");
  const int64_t C = sums.size(1);
  const int nsets = (int)sums.size(0) - 1;
  c10::DeviceGuard dg(sums.device());
  CoefOut o;
  const BnCoefArgs a = coef_args(sums, C, nsets, count, g_a, mean_a, inv_a, g_b, mean_b, inv_b, sink_ga, sink_ba,
                                 sink_gb, sink_bb, o, grad_scale);
  check_hip(launch_bn_bwd_coef(sums.data_ptr<double>(), nsets, C, a, cur_stream()), "bn_bwd_coef");
  return {o.coef_a, o.coef_b, o.dga, o.dba, o.dgb, o.dbb};
}

// bn_bwd_reduce + bn_bwd_coef in one elementwise launch + one reduction launch (no
// cross-rank all-reduce of the sums in between)
std::vector<torch::Tensor> bn_bwd_reduce_coef_x(torch::Tensor dout, OptT outv, torch::Tensor ya, torch::Tensor ma,
                                                OptT yb, OptT mb, OptT msc, OptT msh, double count, OptT g_a,
                                                torch::Tensor inv_a, OptT g_b, OptT inv_b, OptT sink_ga, OptT sink_ba,
                                                OptT sink_gb, OptT sink_bb, const FusedX* fx, double grad_scale) {
  const BwdIn in = bwd_inputs(dout, outv, ya, ma, yb, mb, msc, msh);
  c10::DeviceGuard dg(dout.device());
  const int64_t C = in.C;
  const int nsum = in.ybp ? 3 : 2;
  CoefOut o;
  const BnCoefArgs a = coef_args(dout, C, nsum - 1, count, g_a, ma, inv_a, g_b, mb, inv_b, sink_ga, sink_ba, sink_gb,
                                 sink_bb, o, grad_scale);
  const int g = bn_bwd_reduce_blocks(dout.numel(), C);
  const int z = fx ? fx->z() : 1;
  auto sums = torch::empty({nsum, C}, dout.options().dtype(at::kDouble));
  auto partial = torch::empty({g, nsum, C}, dout.options().dtype(at::kFloat));
  auto scratch = reduce_scratch(dout, g, nsum, C, z);
  check_hip(launch_bn_bwd_reduce(dout.data_ptr(), in.op, ya.data_ptr(), ma.data_ptr<float>(), in.ybp, in.mbp,
                                 dout.numel(), C, partial.data_ptr<float>(), scratch.data_ptr<double>(),
                                 reduce_counters(dout.device(), z), sums.data_ptr<double>(), 2, &a, cur_stream(),
                                 in.mk_s, in.mk_t, in.om, fx ? fx->p() : nullptr),
            "bn_bwd_reduce_coef");
  return {o.coef_a, o.coef_b, o.dga, o.dba, o.dgb, o.dbb};
}

std::vector<torch::Tensor> bn_bwd_reduce_coef(torch::Tensor dout, OptT outv, torch::Tensor ya, torch::Tensor ma,
                                              OptT yb, OptT mb, OptT msc, OptT msh, double count, OptT g_a,
                                              torch::Tensor inv_a, OptT g_b, OptT inv_b, OptT sink_ga, OptT sink_ba,
                                              OptT sink_gb, OptT sink_bb) {
  return bn_bwd_reduce_coef_x(dout, outv, ya, ma, yb, mb, msc, msh, count, g_a, inv_a, g_b, inv_b, sink_ga, sink_ba,
                              sink_gb, sink_bb, nullptr, 1.0);
}

std::vector<torch::Tensor> bn_bwd_apply(torch::Tensor dout, OptT outv, torch::Tensor ya, torch::Tensor ca, OptT yb,
                                        OptT cb, bool want_dz, OptT msc, OptT msh) {
  check_bf16_nhwc(dout, "dout");
  check_bf16_nhwc(ya, "ya");
  const int64_t C = dout.size(3);
  TORCH_CHECK(ya.sizes() == dout.sizes(), "ya shape");
  TORCH_CHECK(ca.is_cuda() && ca.scalar_type() == at::kFloat && ca.numel() == 3 * C && ca.is_contiguous(), "coef_a");
  const void* op = nullptr;
  const void* om = nullptr;
  if (outv.has_value()) {
    if (outv->scalar_type() == at::kByte) {
      check_mask(*outv, dout.numel(), "out (bitmask)");
      om = outv->data_ptr();
    } else {
      check_bf16_nhwc(*outv, "out");
      TORCH_CHECK(outv->sizes() == dout.sizes(), "out shape");
      op = outv->data_ptr();
    }
  }
  c10::DeviceGuard dg(dout.device());
  auto dya = torch::empty_like(dout);
  torch::Tensor dyb, dz;
  const void* ybp = nullptr;
  const float* cbp = nullptr;
  if (yb.has_value()) {
    check_bf16_nhwc(*yb, "yb");
    TORCH_CHECK(yb->sizes() == dout.sizes(), "yb shape");
    TORCH_CHECK(cb.has_value() && cb->numel() == 3 * C && cb->scalar_type() == at::kFloat, "coef_b");
    ybp = yb->data_ptr();
    cbp = cb->data_ptr<float>();
    dyb = torch::empty_like(dout);
  } else {
    dyb = torch::empty({0}, dout.options());
  }
  const float *mk_s, *mk_t;
  in_bn_ptrs(msc, msh, C, &mk_s, &mk_t);
  dz = want_dz ? torch::empty_like(dout) : torch::empty({0}, dout.options());
  check_hip(launch_bn_bwd_apply(dout.data_ptr(), op, ya.data_ptr(), ca.data_ptr<float>(), ybp, cbp, dya.data_ptr(),
                                ybp ? dyb.data_ptr() : nullptr, want_dz ? dz.data_ptr() : nullptr, dout.numel(), C,
                                cur_stream(), mk_s, mk_t, om),
            "bn_bwd_apply");
  return {dya, dyb, dz};
}


// =====================================================================================
// Native residual-block executor: the whole forward / backward kernel sequence of a
// Bottleneck or BasicBlock (reference math: networks/resnet_big.py:7-67) in ONE host
// call, so the per-kernel Python + binding overhead (≈15-25 µs per launch, measured)
// leaves the training step. SyncBN statistics go through a native small communicator
// (comm_ops.cpp: a dedicated RCCL communicator or a one-shot xGMI arena) called in place
// on the compute stream — no Python or c10d work queue between a BN's reduction and its
// finalize. Weight gradients run on the caller's side stream (fork/join by events,
// tensors recorded on that stream for the allocator).
// =====================================================================================

struct BnState {          // per-BN forward results kept for backward
  torch::Tensor sc, sh, mu, iv;
};

// comm: small-communicator handle (comm_ops.cpp); 0 = this process's statistics only.
// With a communicator, the per-channel (Σy, Σy²) are summed over its ranks (fp64, in place,
// on the compute stream) between the reduction and the finalize — SyncBN semantics.
BnState bn_forward(const torch::Tensor& slab, double count, const torch::Tensor& g, const torch::Tensor& b,
                   const torch::Tensor& rm, const torch::Tensor& rv, double eps, double mom, bool training,
                   int64_t comm) {
  if (training) {
    if (comm != 0 && small_comm_world(comm) > 1) {
      const FusedX fx = fused_exchange(comm);
      if (fx.on) {   // reduce + exchange + finalize: one launch
        auto r = bn_stats_finalize_x(slab, count * small_comm_world(comm), g, b, eps, mom, true, rm, rv, &fx);
        small_comm_fused_issued(comm);
        return {r[0], r[1], r[2], r[3]};
      }
      auto sums = bn_stats_reduce(slab);
      small_all_reduce_(comm, sums);
      auto r = bn_finalize(sums, count * small_comm_world(comm), g, b, eps, mom, true, rm, rv);
      return {r[0], r[1], r[2], r[3]};
    }
    auto r = bn_stats_finalize(slab, count, g, b, eps, mom, true, rm, rv);
    return {r[0], r[1], r[2], r[3]};
  }
  auto r = bn_eval_affine(g, b, rm, rv, eps);
  return {r[0], r[1], torch::Tensor(), torch::Tensor()};
}

double rows_of(const torch::Tensor& y) { return (double)(y.numel() / y.size(3)); }

// conv + BN forward: the conv's epilogue emits per-tile statistics, one launch reduces and
// finalizes them (or reduce -> SyncBN exchange -> finalize)
std::pair<torch::Tensor, BnState> conv_bn_fwd(const torch::Tensor& x, const torch::Tensor& w, int64_t stride,
                                              int64_t pad, const torch::Tensor& g, const torch::Tensor& b,
                                              const torch::Tensor& rm, const torch::Tensor& rv, double eps,
                                              double mom, bool training, int64_t comm) {
  auto c = conv_fwd(x, w, stride, pad, training, -1, c10::nullopt, c10::nullopt);
  return {c[0], bn_forward(c[1], rows_of(c[0]), g, b, rm, rv, eps, mom, training, comm)};
}

// bn_bwd_reduce_coef, or (communicator of >1 ranks) reduce -> in-place all-reduce of the
// [Σdz, Σdz·y(, Σdz·y_b)] sums -> coefficients, with count scaled to the global row count
std::vector<torch::Tensor> bn_bwd_sync(int64_t comm, torch::Tensor dout, OptT outv, torch::Tensor ya,
                                       torch::Tensor ma, OptT yb, OptT mb, OptT msc, OptT msh, double count,
                                       OptT g_a, torch::Tensor inv_a, OptT g_b, OptT inv_b, OptT sink_ga,
                                       OptT sink_ba, OptT sink_gb, OptT sink_bb) {
  if (comm == 0 || small_comm_world(comm) == 1)
    return bn_bwd_reduce_coef(dout, outv, ya, ma, yb, mb, msc, msh, count, g_a, inv_a, g_b, inv_b, sink_ga, sink_ba,
                              sink_gb, sink_bb);
  const int w = small_comm_world(comm);
  const FusedX fx = fused_exchange(comm);
  if (fx.on) {
    auto r = bn_bwd_reduce_coef_x(dout, outv, ya, ma, yb, mb, msc, msh, count * w, g_a, inv_a, g_b, inv_b, sink_ga,
                                  sink_ba, sink_gb, sink_bb, &fx, 1.0 / w);
    small_comm_fused_issued(comm);
    return r;
  }
  auto sums = bn_bwd_reduce(dout, outv, ya, ma, yb, mb, msc, msh);
  small_all_reduce_(comm, sums);
  return bn_bwd_coef(sums, count * w, g_a, ma, inv_a, g_b, mb, inv_b, sink_ga, sink_ba, sink_gb, sink_bb, 1.0 / w);
}

// event pool for side-stream fork points
hipEvent_t next_event() {
  static std::mutex mu;
  static std::vector<hipEvent_t> pool;
  static size_t next = 0;
  std::lock_guard<std::mutex> lk(mu);
  if (pool.empty()) {
    // The pool only orders the two streams of one device (record on one, hipStreamWaitEvent
    // on the other); the kernels' own dispatch fences publish their writes device-wide. A
    // record's default system-scope release (L2 writeback + invalidate) is for host / peer
    // visibility, which nothing here needs: without it the main stream's bubble at each fork
    // point drops from ~7.0 to ~5.0 us (48 forks per step) and the step by 0.11 ms (3/3
    // same-box rounds, profiles/event_fence_r6.txt). SDX_EV_FENCE: 0 = the default fence,
    // 1 = hipEventDisableSystemFence (default), 2 = hipEventReleaseToDevice (-0.03 ms)
    const char* ef = getenv("SDX_EV_FENCE");
    const int fm = ef ? atoi(ef) : 1;
    const unsigned fl = hipEventDisableTiming | (fm == 1 ? hipEventDisableSystemFence : 0u) |
                        (fm == 2 ? hipEventReleaseToDevice : 0u);
    pool.resize(512);
    for (auto& e : pool) check_hip(hipEventCreateWithFlags(&e, fl), "hipEventCreate");
  }
  hipEvent_t e = pool[next];
  next = (next + 1) % pool.size();
  return e;
}

// BN-backward coefficients from a fused-dgrad statistics slab [rows][2|3][C]: one column
// reduction whose last block evaluates the coefficients, or (communicator of >1 ranks)
// reduce -> in-place all-reduce -> coefficients
std::vector<torch::Tensor> bn_bwd_coef_slab(int64_t comm, torch::Tensor slab, double count, OptT g_a,
                                            torch::Tensor mean_a, torch::Tensor inv_a, OptT g_b, OptT mean_b,
                                            OptT inv_b, OptT sink_ga, OptT sink_ba, OptT sink_gb, OptT sink_bb) {
  TORCH_CHECK(slab.dim() == 3 && (slab.size(1) == 2 || slab.size(1) == 3), "slab: [rows][2|3][C]");
  check_slab(slab, slab.size(1));
  c10::DeviceGuard dg(slab.device());
  const int64_t rows = slab.size(0), nsum = slab.size(1), C = slab.size(2);
  auto sums = torch::empty({nsum, C}, slab.options().dtype(at::kDouble));
  const FusedX fx = fused_exchange(comm);
  if (fx.on) {   // reduce + exchange + coefficients: one launch (global count, this rank's 1/W of dγ/dβ)
    const int w = small_comm_world(comm);
    CoefOut o;
    const BnCoefArgs a = coef_args(slab, C, (int)nsum - 1, count * w, g_a, mean_a, inv_a, g_b, mean_b, inv_b,
                                   sink_ga, sink_ba, sink_gb, sink_bb, o, 1.0 / w);
    auto scratch = reduce_scratch(slab, rows, nsum, C, fx.z());
    check_hip(launch_col_reduce(slab.data_ptr<float>(), rows, (int)nsum, C, scratch.data_ptr<double>(),
                                reduce_counters(slab.device(), fx.z()), sums.data_ptr<double>(), 2, nullptr, &a,
                                cur_stream(), fx.p()),
              "bn_bwd_coef_slab(fused exchange)");
    small_comm_fused_issued(comm);
    return {o.coef_a, o.coef_b, o.dga, o.dba, o.dgb, o.dbb};
  }
  auto scratch = reduce_scratch(slab, rows, nsum, C);
  if (comm != 0 && small_comm_world(comm) > 1) {
    check_hip(launch_col_reduce(slab.data_ptr<float>(), rows, (int)nsum, C, scratch.data_ptr<double>(),
                                reduce_counters(slab.device()), sums.data_ptr<double>(), 0, nullptr, nullptr,
                                cur_stream()),
              "bn_bwd_coef_slab(reduce)");
    small_all_reduce_(comm, sums);
    const int w = small_comm_world(comm);
    return bn_bwd_coef(sums, count * w, g_a, mean_a, inv_a, g_b, mean_b, inv_b, sink_ga, sink_ba, sink_gb, sink_bb,
                       1.0 / w);
  }
  CoefOut o;
  const BnCoefArgs a = coef_args(slab, C, (int)nsum - 1, count, g_a, mean_a, inv_a, g_b, mean_b, inv_b, sink_ga,
                                 sink_ba, sink_gb, sink_bb, o);
  check_hip(launch_col_reduce(slab.data_ptr<float>(), rows, (int)nsum, C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device()), sums.data_ptr<double>(), 2, nullptr, &a, cur_stream()),
            "bn_bwd_coef_slab");
  return {o.coef_a, o.coef_b, o.dga, o.dba, o.dgb, o.dbb};
}

bool sub_addend_enabled() {
  static const bool on = [] {
    const char* e = getenv("SDX_SUB_ADDEND");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

bool dgrad_bnstat_enabled() {
  static const bool on = [] {
    const char* e = getenv("SDX_DGRAD_BNSTAT");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

// SDX_SPLITK_MERGE=0 (or splitk_merge_set(False)): one split-K reduction launch per weight
// gradient (round-3 behaviour)
std::atomic<int>& splitk_merge_flag() {
  static std::atomic<int> on{[] {
    const char* e = getenv("SDX_SPLITK_MERGE");
    return e == nullptr || atoi(e) != 0 ? 1 : 0;
  }()};
  return on;
}
bool splitk_merge_enabled() { return splitk_merge_flag().load(std::memory_order_relaxed) != 0; }
int64_t splitk_merge_set(bool on) { return splitk_merge_flag().exchange(on ? 1 : 0); }

// tensors read by side-stream wgrads, released after the join (no recordStream: blocks
// return to the allocator in program order instead of behind side-stream events)

void side_stash_release() { side_stash().clear(); }

// dW (+)= wgrad(dy, x) into the parameter's gradient sink, on the side stream if given
void side_wgrad(const torch::Tensor& dy, const torch::Tensor& x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                const torch::Tensor& sink, int64_t side) {
  if (side == 0) {
    conv_wgrad(dy, x, R, S, stride, pad, 0, -1, sink, true, c10::nullopt, c10::nullopt);
    return;
  }
  hipStream_t main = cur_stream();
  hipStream_t ss = reinterpret_cast<hipStream_t>(side);
  hipEvent_t ev = next_event();
  check_hip(hipEventRecord(ev, main), "hipEventRecord");
  check_hip(hipStreamWaitEvent(ss, ev, 0), "hipStreamWaitEvent");
  auto hs = c10::hip::getStreamFromExternal(ss, dy.device().index());
  // dy / x stay alive until the side stream is joined (ops/streams.py join -> side_stash_release)
  side_stash().push_back(dy);
  side_stash().push_back(x);
  c10::hip::HIPStreamGuard guard(hs);
  // the reduction into the parameter sink joins the block's one multi-tensor launch
  // (block_bwd flushes it before returning, i.e. before the sinks are announced final)
  if (splitk_merge_enabled() && !splitk_deferring(ss)) splitk_defer_begin(ss);
  conv_wgrad(dy, x, R, S, stride, pad, 0, -1, sink, true, c10::nullopt, c10::nullopt);
}

// BN3 fold (bnfold.hip): dW3 (+)= diag(A)·G + diag(D)·W3·S + E ⊗ Σa2 with G = dzᵀ·a2 and
// S = a2ᵀ·a2 (two 1x1 wgrad GEMMs) — on the side stream after the coefficients are known
// S = a2ᵀ·a2 [K][1][1][K] and cs = Σ_rows a2 [K] (fp32) on the current stream
std::vector<torch::Tensor> fold_gram_now(const torch::Tensor& a2) {
  const int64_t K3 = a2.size(3);
  auto opt = a2.options().dtype(at::kFloat);
  auto Sm = torch::empty({K3, 1, 1, K3}, opt);
  conv_wgrad(a2, a2, 1, 1, 1, 0, 0, -1, Sm, false, c10::nullopt, c10::nullopt);
  auto part = torch::empty({bnfold_colsum_blocks(), K3}, opt);
  auto cs = torch::empty({K3}, opt);
  check_hip(launch_bnfold_colsum(a2.data_ptr(), a2.numel() / K3, (int)K3, part.data_ptr<float>(), cs.data_ptr<float>(),
                                 cur_stream()),
            "bnfold_colsum");
  return {Sm, cs, part};
}

// the Gram of a folded conv's input, issued at forward time on the (then idle) side stream;
// backward consumes it on the same stream (FIFO), so no further synchronisation is needed
std::vector<torch::Tensor> fold_gram(torch::Tensor a2, int64_t side) {
  check_bf16_nhwc(a2, "a2");
  if (side == 0) return fold_gram_now(a2);
  hipEvent_t ev = next_event();
  check_hip(hipEventRecord(ev, cur_stream()), "hipEventRecord");
  hipStream_t ss = reinterpret_cast<hipStream_t>(side);
  check_hip(hipStreamWaitEvent(ss, ev, 0), "hipStreamWaitEvent");
  side_stash().push_back(a2);
  c10::hip::HIPStreamGuard guard(c10::hip::getStreamFromExternal(ss, a2.device().index()));
  return fold_gram_now(a2);
}

// Gpre: G = dzᵀ·a2 already computed on the main stream (forward-folded BN3, whose backward
// statistics need it first)
void side_fold_wgrad(const torch::Tensor& dz, const torch::Tensor& a2, const torch::Tensor& w3,
                     const torch::Tensor& coef, const torch::Tensor& sink, int64_t side,
                     const torch::Tensor* gram = nullptr, const torch::Tensor* Gpre = nullptr) {
  // its own split-K reductions (G, S) are read right after by bnfold_wgrad: issue any queued
  // sink reductions first and keep this call's undeferred
  if (side != 0 && splitk_deferring(reinterpret_cast<hipStream_t>(side))) check_hip(splitk_flush(), "splitk_flush");
  const int64_t C3 = dz.size(3), K3 = a2.size(3);
  auto body = [&]() {
    auto opt = coef.options();
    torch::Tensor G;
    if (Gpre != nullptr) {
      G = *Gpre;
    } else {
      G = torch::empty({C3, 1, 1, K3}, opt);
      conv_wgrad(dz, a2, 1, 1, 1, 0, 0, -1, G, false, c10::nullopt, c10::nullopt);
    }
    torch::Tensor Sm, cs, part;
    if (gram != nullptr) {
      Sm = gram[0];
      cs = gram[1];
    } else {
      auto g3 = fold_gram_now(a2);
      Sm = g3[0];
      cs = g3[1];
      part = g3[2];
    }
    check_hip(launch_bnfold_wgrad(coef.data_ptr<float>(), G.data_ptr<float>(), Sm.data_ptr<float>(),
                                  cs.data_ptr<float>(), 1, w3.data_ptr(), (int)C3, (int)K3, sink.data_ptr<float>(),
                                  1, cur_stream()),
              "bnfold_wgrad");
    if (side != 0) {
      side_stash().push_back(G);
      side_stash().push_back(Sm);
      side_stash().push_back(cs);
      if (part.defined()) side_stash().push_back(part);
    }
  };
  if (side == 0) {
    body();
    return;
  }
  hipStream_t main = cur_stream();
  hipStream_t ss = reinterpret_cast<hipStream_t>(side);
  hipEvent_t ev = next_event();
  check_hip(hipEventRecord(ev, main), "hipEventRecord");
  check_hip(hipStreamWaitEvent(ss, ev, 0), "hipStreamWaitEvent");
  auto hs = c10::hip::getStreamFromExternal(ss, dz.device().index());
  for (const auto* t : {&dz, &a2, &w3, &coef}) side_stash().push_back(*t);
  c10::hip::HIPStreamGuard guard(hs);
  body();
}

// BN3 fold, main-stream part. K-concatenated (SDX_FOLD_CAT, default): one [K][1][1][C + K]
// bf16 tensor [Wd | Mx] with Wd = diag(A)·W3 (dgrad layout) and Mx = W3ᵀ·diag(D)·W3, plus the
// fp32 bias b = Eᵀ·W3 — conv3's dgrad then reduces over [dz | a2] (CatScope). Otherwise Wd and
// T = a2·Mx + b (bf16), the D·y3 + E part of dy3 pushed through conv3's data gradient and
// added by its epilogue.
struct FoldOps {
  torch::Tensor w;      // Wd, or [Wd | Mx] when cat
  torch::Tensor t;      // T (not cat)
  torch::Tensor bias;   // b (cat)
  bool cat = false;
};
bool fold_cat_enabled() {
  static const bool on = [] {
    const char* e = getenv("SDX_FOLD_CAT");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}
FoldOps fold_dgrad_operands(const torch::Tensor& coef, const torch::Tensor& w3, const torch::Tensor& wt3,
                            const torch::Tensor& a2, const torch::Tensor& mu, const torch::Tensor* gram) {
  const int64_t C3 = w3.size(0), K3 = w3.size(3);
  TORCH_CHECK(w3.size(1) == 1 && w3.size(2) == 1 && wt3.size(0) == K3 && wt3.size(3) == C3 && a2.size(3) == K3 &&
                  coef.numel() == 3 * C3,
              "bn3 fold: conv3 must be 1x1 [C][1][1][K] with a2 of K channels");
  const int64_t rows = a2.numel() / K3;
  TORCH_CHECK(rows < (1LL << 31), "bn3 fold: too many rows");
  check_vec(mu, C3, "fold mu");
  ConvGeom gd{};   // conv3's dgrad: dy = dz (C3 channels) on a2's pixels
  gd.N = a2.size(0); gd.H = gd.P = a2.size(1); gd.W = gd.Q = a2.size(2);
  gd.K = (int)C3; gd.C = (int)K3; gd.R = gd.S = 1; gd.stride = 1; gd.pad = 0;
  FoldOps r;
  r.bias = torch::empty({K3}, coef.options());
  const float* cs = gram != nullptr ? gram[1].data_ptr<float>() : nullptr;
  if (fold_cat_enabled() && conv_dgrad_cat_supported(gd, (int)K3)) {
    r.cat = true;
    r.w = torch::empty({K3, 1, 1, C3 + K3}, w3.options());
    uint16_t* wc = reinterpret_cast<uint16_t*>(r.w.data_ptr());
    check_hip(launch_bnfold_prep(coef.data_ptr<float>(), w3.data_ptr(), wt3.data_ptr(), (int)C3, (int)K3, wc, wc + C3,
                                 r.bias.data_ptr<float>(), mu.data_ptr<float>(), cs, (long)rows, cur_stream(),
                                 (int)(C3 + K3), (int)(C3 + K3)),
              "bnfold_prep");
    return r;
  }
  r.w = torch::empty_like(wt3);
  auto mx = torch::empty({K3, 1, 1, K3}, w3.options());
  check_hip(launch_bnfold_prep(coef.data_ptr<float>(), w3.data_ptr(), wt3.data_ptr(), (int)C3, (int)K3, r.w.data_ptr(),
                               mx.data_ptr(), r.bias.data_ptr<float>(), mu.data_ptr<float>(), cs, (long)rows,
                               cur_stream()),
            "bnfold_prep");
  ConvGeom g{};
  g.N = (int)rows; g.H = g.W = 1; g.C = (int)K3; g.K = (int)K3;
  g.R = g.S = 1; g.P = g.Q = 1; g.stride = 1; g.pad = 0;
  r.t = torch::empty_like(a2);
  const GemmEpi epi{r.bias.data_ptr<float>(), 0, 0};
  check_hip(launch_conv_fwd(g, a2.data_ptr(), mx.data_ptr(), r.t.data_ptr(), nullptr, auto_cfg(rows, K3, K3, true),
                            cur_stream(), nullptr, nullptr, &epi),
            "bnfold T gemm");
  return r;
}

// bn: [gamma, beta, running_mean, running_var] per BN, in the order bn1, bn2, (bn3), (shortcut bn)
// returns [out, y1, a1, y2, a2|-, y3|-, ys|-, omask (uint8 ReLU bits of out; training only),
//          then sc, sh, mu, iv per BN]
//
// fold_fwd (bottleneck, training; ops/block.py decides): the forward half of the BN3 fold —
// conv3 runs twice, first for its BN statistics only (nothing stored), then with the BN3
// apply + residual + ReLU + output bits in its epilogue, so y3 is never written nor re-read
// (≈2 passes over the block's widest tensor); its backward takes Σdz·y3 from W3 and dzᵀ·a2
// (block_bwd, bnfold_rowdot) instead of re-reading y3. Projection blocks: the residual is the
// shortcut's pre-BN output with the shortcut BN applied in the same epilogue (that BN's
// statistics are final before pass 2), which replaces the separate two-input apply pass
//
// side (optional HIP stream): a projection block's shortcut conv (+ its statistics slab) runs
// there, concurrently with the main branch conv1 -> bn1 -> conv2 -> ...; its BN finalize (and
// any SyncBN exchange) stays on the compute stream after the join, so exchanges keep one order
std::vector<torch::Tensor> block_fwd(torch::Tensor x, std::vector<torch::Tensor> w, std::vector<torch::Tensor> bn,
                                     int64_t stride, bool bottleneck, bool proj, bool training, double eps,
                                     double momentum, int64_t comm, bool fold_fwd = false, int64_t side = 0) {
  const int nconv = bottleneck ? 3 : 2;
  TORCH_CHECK((int)w.size() == nconv + (proj ? 1 : 0), "block_fwd: weight count");
  TORCH_CHECK(bn.size() == w.size() * 4, "block_fwd: 4 BN tensors per conv");
  auto B = [&](int i, int k) { return bn[i * 4 + k]; };
  std::vector<BnState> st;
  std::vector<torch::Tensor> out(7);
  // shortcut conv on the side stream: outputs allocated on the compute stream (they are
  // read there after the join), the side stream only writes them
  torch::Tensor ys_side, slab_side;
  hipEvent_t sc_done = nullptr;
  if (proj && training && side != 0) {
    const torch::Tensor& ws = w[nconv];
    check_bf16_nhwc(x, "x");
    check_bf16_nhwc(ws, "w_shortcut");
    TORCH_CHECK(ws.size(3) == x.size(3) && ws.size(1) == 1 && ws.size(2) == 1, "block_fwd: 1x1 shortcut");
    ConvGeom gs{};
    gs.N = x.size(0); gs.H = x.size(1); gs.W = x.size(2); gs.C = x.size(3);
    gs.K = ws.size(0); gs.R = gs.S = 1; gs.stride = stride; gs.pad = 0;
    gs.P = (gs.H - 1) / stride + 1;
    gs.Q = (gs.W - 1) / stride + 1;
    const int64_t M = (int64_t)gs.N * gs.P * gs.Q;
    const int cfg = auto_cfg(M, gs.K, gs.C, true);
    ys_side = torch::empty({gs.N, gs.P, gs.Q, gs.K}, x.options());
    slab_side = torch::empty({(M + igemm_tile_m(cfg) - 1) / igemm_tile_m(cfg), 2, gs.K}, x.options().dtype(at::kFloat));
    hipEvent_t fork = next_event();
    hipStream_t ss = reinterpret_cast<hipStream_t>(side);
    check_hip(hipEventRecord(fork, cur_stream()), "hipEventRecord");
    check_hip(hipStreamWaitEvent(ss, fork, 0), "hipStreamWaitEvent");
    check_hip(launch_conv_fwd(gs, x.data_ptr(), ws.data_ptr(), ys_side.data_ptr(), slab_side.data_ptr<float>(), cfg,
                              ss),
              "block_fwd shortcut conv (side stream)");
    sc_done = next_event();
    check_hip(hipEventRecord(sc_done, ss), "hipEventRecord");
  }
  const int64_t s1 = bottleneck ? 1 : stride, p1 = bottleneck ? 0 : 1;
  auto c1 = conv_bn_fwd(x, w[0], s1, p1, B(0, 0), B(0, 1), B(0, 2), B(0, 3), eps, momentum, training, comm);
  st.push_back(c1.second);
  auto a1 = bn_apply(c1.first, st[0].sc, st[0].sh, c10::nullopt, c10::nullopt, c10::nullopt, 0, true, c10::nullopt);
  const int64_t s2 = bottleneck ? stride : 1;
  auto c2 = conv_bn_fwd(a1, w[1], s2, 1, B(1, 0), B(1, 1), B(1, 2), B(1, 3), eps, momentum, training, comm);
  st.push_back(c2.second);
  torch::Tensor last = c2.first, a2;
  int lastbn = 1;
  // identity blocks: the residual is x (stride 1, same width); projection blocks: the
  // shortcut's pre-BN output ys, normalised in the same epilogue
  fold_fwd = fold_fwd && bottleneck && training && w[2].size(1) == 1 && w[2].size(2) == 1 &&
             (proj || (stride == 1 && w[2].size(0) == x.size(3))) && conv_fwd_bnapply_supported();
  torch::Tensor o, ys;
  // the projection shortcut's output and BN statistics (joins the side stream if it ran there)
  auto shortcut = [&] {
    if (sc_done != nullptr) {
      check_hip(hipStreamWaitEvent(cur_stream(), sc_done, 0), "hipStreamWaitEvent");
      st.push_back(bn_forward(slab_side, rows_of(ys_side), B(nconv, 0), B(nconv, 1), B(nconv, 2), B(nconv, 3), eps,
                              momentum, training, comm));
      ys = ys_side;
    } else {
      auto cs = conv_bn_fwd(x, w[nconv], stride, 0, B(nconv, 0), B(nconv, 1), B(nconv, 2), B(nconv, 3), eps, momentum,
                            training, comm);
      st.push_back(cs.second);
      ys = cs.first;
    }
  };
  // the block output's ReLU mask for backward: 1 bit per element instead of re-reading out
  // (identity blocks: out has x's shape; projection / strided blocks: the last conv's)
  torch::Tensor omask;
  if (bottleneck) {
    a2 = bn_apply(c2.first, st[1].sc, st[1].sh, c10::nullopt, c10::nullopt, c10::nullopt, 0, true, c10::nullopt);
    if (fold_fwd) {
      // pass 1: BN3 statistics (nothing stored) -> finalize (SyncBN: fused exchange) ;
      // pass 2: out = relu(bn3(y3) + x) (projection: + bn_s(ys)) and its bits straight from
      // conv3's epilogue
      auto c3s = conv_fwd_impl(a2, w[2], 1, 0, true, -1, c10::nullopt, c10::nullopt, nullptr, true);
      st.push_back(bn_forward(c3s[1], rows_of(a2), B(2, 0), B(2, 1), B(2, 2), B(2, 3), eps, momentum, training, comm));
      GemmEpi epi{};
      epi.bn_scale = st[2].sc.data_ptr<float>();
      epi.bn_shift = st[2].sh.data_ptr<float>();
      if (proj) {
        shortcut();
        TORCH_CHECK(ys.size(0) == a2.size(0) && ys.size(1) == a2.size(1) && ys.size(2) == a2.size(2) &&
                        ys.size(3) == w[2].size(0),
                    "block_fwd: shortcut output shape");
        epi.resid = ys.data_ptr();
        epi.resid_scale = st[3].sc.data_ptr<float>();
        epi.resid_shift = st[3].sh.data_ptr<float>();
      } else {
        epi.resid = x.data_ptr();
      }
      omask = torch::empty({rows_of(a2) * w[2].size(0) / 8}, x.options().dtype(at::kByte));
      epi.mask_out = omask.data_ptr<uint8_t>();
      o = conv_fwd_impl(a2, w[2], 1, 0, false, -1, c10::nullopt, c10::nullopt, &epi)[0];
      last = torch::Tensor();
    } else {
      auto c3 = conv_bn_fwd(a2, w[2], 1, 0, B(2, 0), B(2, 1), B(2, 2), B(2, 3), eps, momentum, training, comm);
      st.push_back(c3.second);
      last = c3.first;
    }
    lastbn = 2;
  }
  if (training && !omask.defined())
    omask = torch::empty({last.numel() / 8}, last.options().dtype(at::kByte));
  const OptT om = training ? OptT(omask) : OptT();
  if (fold_fwd) {
    // out computed by conv3's epilogue
  } else if (proj) {
    shortcut();
    o = bn_apply(last, st[lastbn].sc, st[lastbn].sh, ys, st[nconv].sc, st[nconv].sh, 1, true, om);
  } else {
    o = bn_apply(last, st[lastbn].sc, st[lastbn].sh, x, c10::nullopt, c10::nullopt, 2, true, om);
  }
  out.push_back(omask);    // index 7 (before the per-BN state)
  out[0] = o;
  out[1] = c1.first;
  out[2] = a1;
  out[3] = c2.first;
  out[4] = bottleneck ? a2 : torch::Tensor();
  out[5] = bottleneck ? last : torch::Tensor();   // undefined with fold_fwd (y3 never stored)
  out[6] = ys;
  // layout: [out, y1, a1, y2, a2, y3, ys, omask, then sc, sh, mu, iv per BN]
  for (auto& b : st) {
    out.push_back(b.sc);
    out.push_back(b.sh);
    out.push_back(b.mu);
    out.push_back(b.iv);
  }
  return out;
}

// saved: [x, y1, a1, y2, a2|-, y3|-, ys|-, out or its uint8 ReLU bitmask] ;
// bnst: [sc, sh, mu, iv] per BN (fwd order)
// wt: dgrad-layout weights (conv order); dw: fp32 gradient sinks (conv order);
// bng: [gamma, dgamma_sink, dbeta_sink] per BN. Returns dx.
//
// Cross-block BN-statistics hand-off (SDX_DGRAD_BNSTAT): in_slab (optional) holds this
// block's OUTPUT-BN backward sums [rows][2|3][C], computed by the NEXT block's final dgrad
// (the one that produced dout); prev = [y_last, mean_last, y_short|-, mean_short|-, omask]
// of the PREVIOUS native block (whose output is x): the final dgrad here computes that
// block's sums from the dx it stores. Returns [dx, slab for the previous block | undefined].
std::vector<torch::Tensor> block_bwd(torch::Tensor dout, std::vector<torch::Tensor> saved,
                                     std::vector<torch::Tensor> bnst, std::vector<torch::Tensor> wt,
                                     std::vector<torch::Tensor> dw, std::vector<torch::Tensor> bng, int64_t stride,
                                     bool bottleneck, bool proj, int64_t side, int64_t comm, OptT in_slab,
                                     std::vector<torch::Tensor> prev, std::vector<torch::Tensor> fold_w) {
  const int nconv = bottleneck ? 3 : 2;
  const int nbn = nconv + (proj ? 1 : 0);
  // the side-stream sink reductions queued by side_wgrad go out as one launch when the block
  // is done (before the caller announces the sinks final); dropped if the block throws
  struct DeferGuard {
    bool ok = false;
    ~DeferGuard() {
      if (!ok) splitk_defer_cancel();
    }
  } defer_guard;
  TORCH_CHECK((int)wt.size() == nbn && (int)dw.size() == nbn && (int)bng.size() == 3 * nbn &&
                  (int)bnst.size() == 4 * nbn && saved.size() == 8,
              "block_bwd: argument counts");
  const torch::Tensor &x = saved[0], &y1 = saved[1], &a1 = saved[2], &y2 = saved[3], &a2 = saved[4],
                      &y3 = saved[5], &ys = saved[6], &out = saved[7];
  auto S = [&](int i, int k) { return bnst[i * 4 + k]; };
  auto G = [&](int i, int k) { return bng[i * 3 + k]; };
  const int64_t H = x.size(1), W = x.size(2);
  const int lastbn = nconv - 1;
  const torch::Tensor& ylast = bottleneck ? y3 : y2;
  // forward-folded BN3 (block_fwd fold_fwd): y3 was never stored
  const bool no_y3 = bottleneck && (!y3.defined() || y3.numel() == 0);
  const double cnt_last = rows_of(y2), cnt1 = rows_of(y1);   // conv3 is 1x1 stride 1: y3 rows = y2 rows
  torch::Tensor dylast, dys, dz;
  const bool have_slab = in_slab.has_value() && in_slab->defined() && in_slab->numel() > 0;
  if (have_slab) TORCH_CHECK(in_slab->size(1) == (proj ? 3 : 2), "block_bwd: in_slab set count");
  // BN3 fold (bnfold.hip): fold_w = [conv3 forward weights] was passed because this block
  // published the fold marker (prev[5]) to the next block, whose final dgrad then stored
  // dout already masked (dz = dout·[out > 0]) together with in_slab
  // projection blocks: fold_w = [conv3, shortcut] folds both BNs (stride-1 shortcut only: its
  // input is then x itself); fold_w = [conv3] folds BN3 and materialises only the shortcut's dys
  // fold_w may be followed by the forward-time Grams of the folded convs' inputs (fold_gram):
  // [W3, (Ws)] or [W3, (Ws), S3, cs3, (Ss, css)]
  const size_t nfw = fold_w.size() == 3 || fold_w.size() == 6 ? fold_w.size() / 3 : fold_w.size();
  const bool grams = nfw != fold_w.size();
  const bool fold = bottleneck && have_slab && nfw >= 1 && nfw <= (proj ? 2u : 1u) && fold_w[0].defined() &&
                    (nfw == 1 || (stride == 1 && fold_w[1].defined()));
  const bool fold_sc = fold && proj && nfw == 2;
  TORCH_CHECK(!no_y3 || fold, "block_bwd: a forward-folded block needs its BN3 fold (next block's slab)");
  const torch::Tensor* gram3 = grams ? &fold_w[nfw] : nullptr;
  const torch::Tensor* grams_sc = grams && nfw == 2 ? &fold_w[nfw + 2] : nullptr;
  torch::Tensor coef3, coefs, Gfold;
  if (no_y3) {
    // Σdz·y3 = Σ_k W3[c][k]·(dzᵀ·a2)[c][k]: G on the main stream (the fold's wgrad reuses it),
    // written into the two extra rows the next block's final dgrad left in in_slab (a
    // projection block's third set, Σdz·(ys − μs), came from that dgrad's epilogue)
    const int64_t C3 = dout.size(3), K3 = a2.size(3), ns = in_slab->size(1);
    TORCH_CHECK(in_slab->size(0) > 2 && in_slab->size(2) == C3 && fold_w[0].size(0) == C3 &&
                    fold_w[0].size(3) == K3,
                "block_bwd: forward-folded BN3 slab / weights");
    Gfold = torch::empty({C3, 1, 1, K3}, dout.options().dtype(at::kFloat));
    conv_wgrad(dout, a2, 1, 1, 1, 0, 0, -1, Gfold, false, c10::nullopt, c10::nullopt);
    float* rows = in_slab->data_ptr<float>() + (in_slab->size(0) - 2) * ns * C3;
    check_hip(launch_bnfold_rowdot(Gfold.data_ptr<float>(), fold_w[0].data_ptr(), (int)C3, (int)K3, (int)ns, rows,
                                   cur_stream()),
              "bnfold_rowdot");
  }
  if (proj) {
    auto c = have_slab
                 ? bn_bwd_coef_slab(comm, *in_slab, cnt_last, G(lastbn, 0), S(lastbn, 2), S(lastbn, 3), G(nconv, 0),
                                    S(nconv, 2), S(nconv, 3), G(lastbn, 1), G(lastbn, 2), G(nconv, 1), G(nconv, 2))
                 : bn_bwd_sync(comm, dout, out, ylast, S(lastbn, 2), ys, S(nconv, 2), c10::nullopt, c10::nullopt,
                               cnt_last, G(lastbn, 0), S(lastbn, 3), G(nconv, 0), S(nconv, 3), G(lastbn, 1),
                               G(lastbn, 2), G(nconv, 1), G(nconv, 2));
    if (fold) {
      coef3 = c[0];
      dz = dout;
      if (fold_sc)
        coefs = c[1];
      else   // dout is already masked: dys = A'·dz + D'·ys + E' without a ReLU mask
        dys = bn_bwd_apply(dz, c10::nullopt, ys, c[1], c10::nullopt, c10::nullopt, false, c10::nullopt,
                           c10::nullopt)[0];
    } else {
      auto r = bn_bwd_apply(dout, out, ylast, c[0], ys, c[1], false, c10::nullopt, c10::nullopt);
      dylast = r[0];
      dys = r[1];
    }
  } else {
    auto c = have_slab
                 ? bn_bwd_coef_slab(comm, *in_slab, cnt_last, G(lastbn, 0), S(lastbn, 2), S(lastbn, 3), c10::nullopt,
                                    c10::nullopt, c10::nullopt, G(lastbn, 1), G(lastbn, 2), c10::nullopt, c10::nullopt)
                 : bn_bwd_sync(comm, dout, out, ylast, S(lastbn, 2), c10::nullopt, c10::nullopt, c10::nullopt,
                               c10::nullopt, cnt_last, G(lastbn, 0), S(lastbn, 3), c10::nullopt, c10::nullopt,
                               G(lastbn, 1), G(lastbn, 2), c10::nullopt, c10::nullopt);
    if (fold) {
      coef3 = c[0];
      dz = dout;
    } else {
      // identity shortcut: its gradient dz = dout·[out > 0] is never materialised when the ReLU
      // bitmask is available — the last dgrad epilogue adds dout under the mask
      const bool bitmask = out.scalar_type() == at::kByte;
      auto r = bn_bwd_apply(dout, out, ylast, c[0], c10::nullopt, c10::nullopt, !bitmask, c10::nullopt,
                            c10::nullopt);
      dylast = r[0];
      dz = bitmask ? torch::Tensor() : r[2];
    }
  }
  // dgrad whose output da is the gradient of the block-internal BN i's ReLU output; the BN's
  // Σda·m, Σda·m·(y−μ) come from the dgrad epilogue (SDX_DGRAD_BNSTAT=0: separate pass)
  auto dgrad_bn = [&](const torch::Tensor& dyo, const torch::Tensor& w, const torch::Tensor& y, int64_t st,
                      int64_t pad, int i, double cnt, OptT add = c10::nullopt) -> std::pair<torch::Tensor, torch::Tensor> {
    if (dgrad_bnstat_enabled()) {
      auto r = conv_dgrad_bnstat(dyo, w, y.size(1), y.size(2), st, pad, -1, c10::nullopt, add,
                                 c10::nullopt, y, S(i, 2), c10::nullopt, c10::nullopt, c10::nullopt, S(i, 0), S(i, 1));
      auto c = bn_bwd_coef_slab(comm, r[1], cnt, G(i, 0), S(i, 2), S(i, 3), c10::nullopt, c10::nullopt,
                                c10::nullopt, G(i, 1), G(i, 2), c10::nullopt, c10::nullopt);
      return {r[0], c[0]};
    }
    auto da = conv_dgrad(dyo, w, y.size(1), y.size(2), st, pad, -1, c10::nullopt, add, c10::nullopt);
    auto c = bn_bwd_sync(comm, da, c10::nullopt, y, S(i, 2), c10::nullopt, c10::nullopt, S(i, 0), S(i, 1), cnt,
                         G(i, 0), S(i, 3), c10::nullopt, c10::nullopt, G(i, 1), G(i, 2), c10::nullopt, c10::nullopt);
    return {da, c[0]};
  };
  torch::Tensor dy1;
  if (bottleneck) {
    std::pair<torch::Tensor, torch::Tensor> r2;
    if (fold) {
      // da2 = dz·(diag(A)·W3) + T: no dy3 tensor; dW3 from dzᵀ·a2 and a2ᵀ·a2 on the side stream
      auto op = fold_dgrad_operands(coef3, fold_w[0], wt[2], a2, S(lastbn, 2), gram3);
      side_fold_wgrad(dz, a2, fold_w[0], coef3, dw[2], side, gram3, Gfold.defined() ? &Gfold : nullptr);
      if (op.cat) {
        CatScope cs(a2, op.bias);
        r2 = dgrad_bn(dz, op.w, y2, 1, 0, 1, cnt_last);
      } else {
        AddPreScope pre;
        r2 = dgrad_bn(dz, op.w, y2, 1, 0, 1, cnt_last, op.t);
      }
    } else {
      side_wgrad(dylast, a2, 1, 1, 1, 0, dw[2], side);
      r2 = dgrad_bn(dylast, wt[2], y2, 1, 0, 1, cnt_last);
    }
    auto dy2 = bn_bwd_apply(r2.first, c10::nullopt, y2, r2.second, c10::nullopt, c10::nullopt, false, S(1, 0),
                            S(1, 1))[0];
    side_wgrad(dy2, a1, 3, 3, stride, 1, dw[1], side);
    auto r1 = dgrad_bn(dy2, wt[1], y1, stride, 1, 0, cnt1);
    dy1 = bn_bwd_apply(r1.first, c10::nullopt, y1, r1.second, c10::nullopt, c10::nullopt, false, S(0, 0),
                       S(0, 1))[0];
    side_wgrad(dy1, x, 1, 1, 1, 0, dw[0], side);
  } else {
    side_wgrad(dylast, a1, 3, 3, 1, 1, dw[1], side);
    auto r1 = dgrad_bn(dylast, wt[1], y1, 1, 1, 0, cnt1);
    dy1 = bn_bwd_apply(r1.first, c10::nullopt, y1, r1.second, c10::nullopt, c10::nullopt, false, S(0, 0),
                       S(0, 1))[0];
    side_wgrad(dy1, x, 3, 3, stride, 1, dw[0], side);
  }
  const int64_t s1 = bottleneck ? 1 : stride, p1 = bottleneck ? 0 : 1;
  // the final dgrad (the one that stores dx) optionally emits the previous block's output-BN sums
  const bool want_prev = dgrad_bnstat_enabled() && prev.size() >= 5 && prev[4].defined() && prev[4].numel() > 0;
  // the previous block folds its BN3 backward: store its dz = dx·[out_prev > 0], not dx
  const bool prev_fold = want_prev && prev.size() >= 6 && prev[5].defined() && prev[5].numel() > 0;
  torch::Tensor prev_slab;
  auto last_dgrad = [&](OptT o, OptT add, OptT amask, int64_t asub = 0) -> torch::Tensor {
    if (!want_prev) return conv_dgrad(dy1, wt[0], H, W, s1, p1, -1, o, add, amask, asub);
    const bool two = prev[2].defined() && prev[2].numel() > 0;
    // the previous block folded its BN3 forward too (no y3): Σdz and −μ·Σdz here, two slab
    // rows left for its Σdz·y3 (block_bwd no_y3)
    const bool prev_noy = !prev[0].defined() || prev[0].numel() == 0;
    TORCH_CHECK(!prev_noy || prev_fold, "block_bwd: previous block without y3 must fold");
    auto r = conv_dgrad_bnstat(dy1, wt[0], H, W, s1, p1, -1, o, add, amask, prev[0], prev[1],
                               two ? OptT(prev[2]) : OptT(), two ? OptT(prev[3]) : OptT(), prev[4], c10::nullopt,
                               c10::nullopt, asub, prev_fold ? 1 : 0, prev_noy ? 2 : 0);
    prev_slab = r[1];
    return r[0];
  };
  torch::Tensor dx;
  if (fold_sc) {
    // shortcut BN folded like BN3: dx_sc = dz·(diag(A')·Ws) + x·(Wsᵀ·diag(D')·Ws) + E'ᵀ·Ws
    auto op = fold_dgrad_operands(coefs, fold_w[1], wt[nconv], x, S(nconv, 2), grams_sc);
    side_fold_wgrad(dz, x, fold_w[1], coefs, dw[nconv], side, grams_sc);
    if (op.cat) {
      CatScope cs(x, op.bias);
      dx = conv_dgrad(dz, op.w, H, W, 1, 0, -1, c10::nullopt, c10::nullopt, c10::nullopt, 0);
    } else {
      AddPreScope pre;
      dx = conv_dgrad(dz, op.w, H, W, 1, 0, -1, c10::nullopt, op.t, c10::nullopt, 0);
    }
    dx = last_dgrad(dx, dx, c10::nullopt);
  } else if (proj) {
    side_wgrad(dys, x, 1, 1, stride, 0, dw[nconv], side);
    if (stride > 1 && sub_addend_enabled()) {
      // the strided 1x1 shortcut's data gradient lives on the stride-s subgrid only: compute
      // it compactly (a stride-1 1x1 dgrad on the P x Q grid) and let the final dgrad add it
      // there — no zero sub-pixel classes written, no zeros re-read as the addend
      auto dxs = conv_dgrad(dys, wt[nconv], dys.size(1), dys.size(2), 1, 0, -1, c10::nullopt, c10::nullopt,
                            c10::nullopt, 0);
      dx = last_dgrad(c10::nullopt, dxs, c10::nullopt, stride);
    } else {
      dx = conv_dgrad(dys, wt[nconv], H, W, stride, 0, -1, c10::nullopt, c10::nullopt, c10::nullopt, 0);
      dx = last_dgrad(dx, dx, c10::nullopt);
    }
  } else if (dz.defined()) {
    dx = last_dgrad(c10::nullopt, dz, c10::nullopt);
  } else {
    dx = last_dgrad(c10::nullopt, dout, out);
  }
  check_hip(splitk_flush(), "splitk_flush");
  defer_guard.ok = true;
  return {dx, prev_slab};
}

// Column reduction + cross-rank exchange of a statistics slab in ONE launch (the fused
// SyncBN path without an epilogue): tests, the start-up self-check of an xGMI communicator
// and the per-BN latency probe (tools/syncbn_latency.py). Real communicator: slab
// [rows][nsets][C] -> global sums [nsets][C]. Emulated (XEMU): slab [W][rows][nsets][C],
// virtual rank z reduces slab[z], or [rows][nsets][C] shared by identical ranks; rank 0's
// global sums are returned.
torch::Tensor syncbn_exchange_sums(int64_t comm, torch::Tensor slab) {
  FusedX fx = fused_exchange(comm);
  TORCH_CHECK(fx.on, "syncbn_exchange_sums: not a fused (xGMI) communicator of > 1 ranks");
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.is_contiguous(), "slab: contiguous fp32");
  const bool emu = fx.x.mode == 2;
  // emulated ranks: [W][rows][nsets][C] (rank z reduces slab[z]) or [rows][nsets][C] (identical ranks)
  TORCH_CHECK(slab.dim() == 3 || (emu && slab.dim() == 4), "slab: [rows][nsets][C]",
              emu ? " or [W][rows][nsets][C]" : "");
  if (slab.dim() == 4) TORCH_CHECK(slab.size(0) == fx.x.world, "slab: one block per emulated rank");
  const int64_t rows = slab.size(-3), nsets = slab.size(-2), C = slab.size(-1);
  TORCH_CHECK(nsets >= 1 && nsets <= 3 && C >= 1 && C <= 4096 && rows >= 1, "slab shape");
  if (slab.dim() == 4) fx.x.slab_zstride = (long)(rows * nsets * C);
  c10::DeviceGuard dg(slab.device());
  auto sums = torch::empty({nsets, C}, slab.options().dtype(at::kDouble));
  auto scratch = reduce_scratch(slab, rows, nsets, C, fx.z());
  check_hip(launch_col_reduce(slab.data_ptr<float>(), (int)rows, (int)nsets, (int)C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device(), fx.z()), sums.data_ptr<double>(), 0, nullptr, nullptr,
                              cur_stream(), fx.p()),
            "syncbn_exchange_sums");
  small_comm_fused_issued(comm);
  return sums;
}

}  // namespace

void register_conv_bn(pybind11::module& m) {
  m.def("conv_fwd_bias", &conv_fwd_bias,
        "implicit-GEMM conv forward with a per-channel fp32 bias (+ReLU) epilogue (eval-mode folded BN)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("bias"),
        pybind11::arg("relu"));
  m.def("wgrad1x1_pairs_set", [](int64_t on) { return (int64_t)wgrad1x1_pairs_set((int)on); },
        "pixel-pair 1x1 wgrad for 64-channel sides on (1) / off (0); returns the previous value", pybind11::arg("on"));
  m.def("igemm_one_k_set", [](int64_t mode, int64_t k) { return (int64_t)igemm_one_k_set((int)mode, (int)k); },
        "longest GEMM reduction on the single-stage LDS-DMA loop (mode 0 fwd, 1 dgrad); returns the previous limit",
        pybind11::arg("mode"), pybind11::arg("k"));
  m.def("wgrad_block_target_set", &wgrad_block_target_set,
        "block target of the dedicated 1x1/3x3 wgrad kernels' split heuristic (SDX_W3_BLOCKS); returns the previous value",
        pybind11::arg("n"));
  m.def("wgrad1x1_big_set", [](int64_t on) { return (int64_t)wgrad1x1_big_set((int)on); },
        "256-row LDS-DMA 1x1 wgrad kernel: 0 off, 1 long-split shapes (default), 2 every eligible shape; returns the previous value",
        pybind11::arg("mode"));
  m.def("conv_plan", [](int64_t N, int64_t H, int64_t W, int64_t C, int64_t K, int64_t R, int64_t S, int64_t stride,
                        int64_t pad, bool dgrad) {
    // host-only: the tile config auto dispatch picks for a plain fwd / dgrad and the M-tile
    // count of its statistics slab (padded-row tap tiles count virtual rows)
    ConvGeom g{};
    g.N = (int)N; g.H = (int)H; g.W = (int)W; g.C = (int)C; g.K = (int)K; g.R = (int)R; g.S = (int)S;
    g.stride = (int)stride; g.pad = (int)pad;
    g.P = (g.H + 2 * g.pad - g.R) / g.stride + 1;
    g.Q = (g.W + 2 * g.pad - g.S) / g.stride + 1;
    const int64_t M = dgrad ? N * H * W : (int64_t)g.N * g.P * g.Q;
    const int cdim = dgrad ? g.K : g.C, ncol = dgrad ? g.C : g.K;
    const int cfg = dgrad ? conv_cfg(g, cdim, ncol, M, (int64_t)R * S * K / (stride * stride), true, true)
                          : conv_cfg(g, cdim, ncol, M, (int64_t)R * S * C, true, false);
    const int64_t mt = dgrad ? (g.stride == 1 ? conv_dgrad_class_mtiles(g, 0, 0, cfg) : -1)
                             : (g.stride == 1 ? igemm_conv_mtiles(g, g.C, cfg, M)
                                              : (M + igemm_tile_m(cfg) - 1) / igemm_tile_m(cfg));
    return pybind11::make_tuple(cfg, mt);
  }, "host-only dispatch plan of a plain conv: (tile config, statistics-slab M-tiles; -1 for strided dgrads)",
        pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("K"),
        pybind11::arg("R"), pybind11::arg("S"), pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("dgrad"));
  m.def("tap3_set", &tap3_set,
        "tap-reuse 3x3 conv loop on (1) / off (0) for auto tile selection; returns the previous value",
        pybind11::arg("on"));
  m.def("syncbn_exchange_sums", &syncbn_exchange_sums,
        "column reduction + cross-rank exchange of a BN statistics slab in one launch (fused xGMI communicators)");
  m.def("igemm_trace", [] {
    const int n = 2 * igemm_trace_slots();
    auto t = torch::empty({n}, torch::TensorOptions().dtype(at::kLong));
    check_hip(igemm_trace_copy(reinterpret_cast<unsigned long long*>(t.data_ptr<int64_t>()), cur_stream()),
              "igemm_trace");
    return t.view({2, n / 2});
  }, "diagnostic conv main-loop timeline of the last traced launch (SDX_IGEMM_TRACE=1)");
  m.def("conv_fwd", &conv_fwd, "implicit-GEMM conv forward (NHWC bf16) + BN stat slab [+ BN+ReLU prologue]",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("stride"), pybind11::arg("pad"),
        pybind11::arg("want_stats"), pybind11::arg("cfg") = -1, pybind11::arg("in_scale") = pybind11::none(),
        pybind11::arg("in_shift") = pybind11::none());
  m.def("conv_dgrad", &conv_dgrad, "implicit-GEMM conv data gradient (strided: sub-pixel classes)",
        pybind11::arg("dy"), pybind11::arg("wt"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("stride"),
        pybind11::arg("pad"), pybind11::arg("cfg") = -1, pybind11::arg("out") = pybind11::none(),
        pybind11::arg("addend") = pybind11::none(), pybind11::arg("addend_mask") = pybind11::none(),
        pybind11::arg("addend_sub") = 0);
  m.def("conv_dgrad_cat",
        [](torch::Tensor dy, torch::Tensor wt, torch::Tensor a2, torch::Tensor bias, int64_t cfg,
           c10::optional<torch::Tensor> ya, c10::optional<torch::Tensor> ma) -> std::vector<torch::Tensor> {
          CatScope cs(a2, bias);
          if (ya.has_value())
            return conv_dgrad_bnstat(dy, wt, dy.size(1), dy.size(2), 1, 0, cfg, c10::nullopt, c10::nullopt,
                                     c10::nullopt, *ya, *ma, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt,
                                     c10::nullopt);
          return {conv_dgrad(dy, wt, dy.size(1), dy.size(2), 1, 0, cfg, c10::nullopt, c10::nullopt, c10::nullopt)};
        },
        "K-concatenated stride-1 1x1 data gradient dx = dy·Wt[:, :K] + a2·Wt[:, K:] + bias (BN3 fold); with ya / ma "
        "also the BN-backward statistics slab (ReLU mask recomputed as ya > 0 is not applied: raw sums)",
        pybind11::arg("dy"), pybind11::arg("wt"), pybind11::arg("a2"), pybind11::arg("bias"), pybind11::arg("cfg") = -1,
        pybind11::arg("ya") = pybind11::none(), pybind11::arg("ma") = pybind11::none());
  m.def("conv_wgrad", &conv_wgrad, "implicit-GEMM conv weight gradient (fp32, split-K slab)", pybind11::arg("dy"),
        pybind11::arg("x"), pybind11::arg("R"), pybind11::arg("S"), pybind11::arg("stride"), pybind11::arg("pad"),
        pybind11::arg("splits") = 0, pybind11::arg("cfg") = -1, pybind11::arg("out") = pybind11::none(),
        pybind11::arg("accumulate") = false, pybind11::arg("in_scale") = pybind11::none(),
        pybind11::arg("in_shift") = pybind11::none());
  m.def("bn_stats_reduce", &bn_stats_reduce);
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_stats_finalize", &bn_stats_finalize, "conv stat slab -> BN affine in one launch");
  m.def("bn_eval_affine", &bn_eval_affine);
  m.def("bn_apply", &bn_apply, pybind11::arg("y"), pybind11::arg("scale"), pybind11::arg("shift"),
        pybind11::arg("r") = pybind11::none(), pybind11::arg("scale2") = pybind11::none(),
        pybind11::arg("shift2") = pybind11::none(), pybind11::arg("res_mode") = 0, pybind11::arg("relu") = true,
        pybind11::arg("mask_out") = pybind11::none());
  m.def("bn_bwd_reduce", &bn_bwd_reduce, pybind11::arg("dout"), pybind11::arg("outv"), pybind11::arg("ya"),
        pybind11::arg("ma"), pybind11::arg("yb") = pybind11::none(), pybind11::arg("mb") = pybind11::none(),
        pybind11::arg("msc") = pybind11::none(), pybind11::arg("msh") = pybind11::none());
  m.def("bn_bwd_coef", &bn_bwd_coef, pybind11::arg("sums"), pybind11::arg("count"), pybind11::arg("g_a"),
        pybind11::arg("mean_a"), pybind11::arg("inv_a"), pybind11::arg("g_b") = pybind11::none(),
        pybind11::arg("mean_b") = pybind11::none(), pybind11::arg("inv_b") = pybind11::none(),
        pybind11::arg("sink_ga") = pybind11::none(), pybind11::arg("sink_ba") = pybind11::none(),
        pybind11::arg("sink_gb") = pybind11::none(), pybind11::arg("sink_bb") = pybind11::none(),
        pybind11::arg("grad_scale") = 1.0);
  m.def("bn_bwd_reduce_coef", &bn_bwd_reduce_coef, pybind11::arg("dout"), pybind11::arg("outv"),
        pybind11::arg("ya"), pybind11::arg("ma"), pybind11::arg("yb") = pybind11::none(),
        pybind11::arg("mb") = pybind11::none(), pybind11::arg("msc") = pybind11::none(),
        pybind11::arg("msh") = pybind11::none(), pybind11::arg("count") = 1.0, pybind11::arg("g_a") = pybind11::none(),
        pybind11::arg("inv_a") = pybind11::none(), pybind11::arg("g_b") = pybind11::none(),
        pybind11::arg("inv_b") = pybind11::none(), pybind11::arg("sink_ga") = pybind11::none(),
        pybind11::arg("sink_ba") = pybind11::none(), pybind11::arg("sink_gb") = pybind11::none(),
        pybind11::arg("sink_bb") = pybind11::none());
  m.def("splitk_merge_set", &splitk_merge_set,
        "merge a residual block's side-stream split-K reductions into one launch (returns the previous setting)");
  m.def("side_stash_release", &side_stash_release, "drop the tensors kept alive for side-stream wgrads (after join)");
  m.def("conv_dgrad_bnstat", &conv_dgrad_bnstat,
        "dgrad + fused BN-backward statistics of dx (slab [rows][2|3][C] for bn_bwd_coef_slab)",
        pybind11::arg("dy"), pybind11::arg("wt"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("stride"),
        pybind11::arg("pad"), pybind11::arg("cfg") = -1, pybind11::arg("out") = pybind11::none(),
        pybind11::arg("addend") = pybind11::none(), pybind11::arg("addend_mask") = pybind11::none(),
        pybind11::arg("ya"), pybind11::arg("ma"), pybind11::arg("yb") = pybind11::none(),
        pybind11::arg("mb") = pybind11::none(), pybind11::arg("mask_bits") = pybind11::none(),
        pybind11::arg("msc") = pybind11::none(), pybind11::arg("msh") = pybind11::none(),
        pybind11::arg("addend_sub") = 0, pybind11::arg("store_masked") = 0, pybind11::arg("extra_rows") = 0);
  m.def("bn_bwd_coef_slab", &bn_bwd_coef_slab, "BN-backward coefficients (+dγ/dβ into sinks) from a dgrad stat slab",
        pybind11::arg("comm"), pybind11::arg("slab"), pybind11::arg("count"), pybind11::arg("g_a"),
        pybind11::arg("mean_a"), pybind11::arg("inv_a"), pybind11::arg("g_b") = pybind11::none(),
        pybind11::arg("mean_b") = pybind11::none(), pybind11::arg("inv_b") = pybind11::none(),
        pybind11::arg("sink_ga") = pybind11::none(), pybind11::arg("sink_ba") = pybind11::none(),
        pybind11::arg("sink_gb") = pybind11::none(), pybind11::arg("sink_bb") = pybind11::none());
  m.def("block_fwd", &block_fwd, "native residual-block forward (whole kernel sequence; comm: SyncBN handle or 0)",
        pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bn"), pybind11::arg("stride"),
        pybind11::arg("bottleneck"), pybind11::arg("proj"), pybind11::arg("training"), pybind11::arg("eps"),
        pybind11::arg("momentum"), pybind11::arg("comm") = 0, pybind11::arg("fold_fwd") = false,
        pybind11::arg("side") = 0);
  m.def("fold_gram", &fold_gram,
        "BN3 fold: [a2ᵀ·a2, Σ_rows a2, scratch] of a folded conv's input, issued on the side stream",
        pybind11::arg("a2"), pybind11::arg("side"));
  m.def("block_bwd", &block_bwd, "native residual-block backward (dgrad chain + side-stream wgrads)",
        pybind11::arg("dout"), pybind11::arg("saved"), pybind11::arg("bnst"), pybind11::arg("wt"),
        pybind11::arg("dw"), pybind11::arg("bng"), pybind11::arg("stride"), pybind11::arg("bottleneck"),
        pybind11::arg("proj"), pybind11::arg("side"), pybind11::arg("comm") = 0,
        pybind11::arg("in_slab") = pybind11::none(), pybind11::arg("prev") = std::vector<torch::Tensor>(),
        pybind11::arg("fold_w") = std::vector<torch::Tensor>());
  m.def("bn_bwd_apply", &bn_bwd_apply, pybind11::arg("dout"), pybind11::arg("outv"), pybind11::arg("ya"),
        pybind11::arg("ca"), pybind11::arg("yb") = pybind11::none(), pybind11::arg("cb") = pybind11::none(),
        pybind11::arg("want_dz") = false, pybind11::arg("msc") = pybind11::none(),
        pybind11::arg("msh") = pybind11::none());
}

}  // namespace sdx_bind
