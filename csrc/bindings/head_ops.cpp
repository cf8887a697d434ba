// Projection head on the native path (reference networks/resnet_big.py:159-181: MLP
// Linear(dim_in, dim_in) -> ReLU -> Linear(dim_in, feat_dim), or one Linear), executed as
// 1x1 implicit GEMMs of igemm.hip (hand-written MFMA kernels) with fused epilogues — no
// library GEMM, one host call per direction:
//
//   forward   fb = bf16(feat)                         cast kernel (head.hip)
//             h  = relu(fb·W1ᵀ + b1)   (bf16)         FWD GEMM, bias + ReLU epilogue
//             z  = h·W2ᵀ + b2          (fp32)         FWD GEMM, bias + fp32-store epilogue
//   backward  dzb = bf16(dz); db2 += Σ_rows dz        cast + column reduction (sink add)
//             dW2 += dzbᵀ·h                           WGRAD GEMM (split-K, into the sink)
//             dh = (dzb·W2)·[h > 0]; db1 += Σ_rows dh  DGRAD GEMM, ReLU-backward store +
//                                                     column-sum slab epilogue, reduction
//             dW1 += dhᵀ·fb                           WGRAD GEMM
//             dfeat = dh·W1            (fp32)         DGRAD GEMM, fp32-store epilogue
//
// Numerics: bf16 operands, fp32 accumulation, fp32 biases added to the fp32 accumulators,
// bf16 hidden activation (as torch autocast), fp32 output features.
#include "conv_internal.h"
#include "launchers.h"
#include "ops_decl.h"

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>

#include <map>
#include <mutex>
#include <tuple>

hipError_t launch_cast_f32_bf16(const float* x, void* y, long n, hipStream_t s);

namespace sdx_bind {
std::vector<torch::Tensor>& side_stash();   // conv_bn_ops.cpp: released at the side-stream join

namespace {

void check_w(const torch::Tensor& w, int64_t rows, int64_t cols, const char* name) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.numel() == rows * cols, name,
              " must be a contiguous bf16 GPU tensor of ", rows, "x", cols, " elements");
}

void check_2d(const torch::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == 2 && t.is_contiguous(), name,
              " must be a contiguous 2-D GPU tensor of ", c10::toString(dt));
  TORCH_CHECK(t.size(1) % 8 == 0, name, ": columns must be a multiple of 8");
  TORCH_CHECK(t.numel() < (1LL << 31), name, " too large for 32-bit GEMM indexing");
}

// constant per-column vectors (0 / 1) of the ReLU-backward statistics epilogue, cached
const torch::Tensor& const_vec(const torch::Device& dev, int64_t n, float v) {
  static std::mutex mu;
  static std::map<std::tuple<int, int64_t, float>, torch::Tensor> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto& t = cache[std::make_tuple((int)dev.index(), n, v)];
  if (!t.defined()) t = torch::full({n}, v, torch::TensorOptions().dtype(at::kFloat).device(dev));
  return t;
}

// the head's GEMMs have few rows (one per view on this rank): the 64x64 tile is the only
// one that puts enough blocks on the chip for their long reductions (512 rows, 2048 -> 2048:
// 22.0 vs 28.6 us auto; 2048 -> 128: 15.5 us, profiles/head_gemm_r5.txt)
int head_cfg(int64_t rows, int64_t ncol, int64_t kdim) {
  return rows <= 2048 ? 3 : auto_cfg(rows, ncol, kdim, true);
}

ConvGeom gemm_geom(int64_t rows, int64_t in, int64_t out) {
  // a [rows] x [in] -> [out] GEMM as a 1x1 conv over `rows` single-pixel images
  ConvGeom g{};
  g.N = (int)rows; g.H = g.W = 1; g.C = (int)in; g.K = (int)out;
  g.R = g.S = 1; g.P = g.Q = 1; g.stride = 1; g.pad = 0;
  return g;
}

// y[rows][out] = x[rows][in] · W[out][in]ᵀ (+ bias) (ReLU); bf16 or fp32 output
torch::Tensor gemm_fwd(const torch::Tensor& x, const torch::Tensor& w, const torch::Tensor& bias, bool relu,
                       bool out_f32) {
  const int64_t rows = x.size(0), in = x.size(1), out = bias.numel();
  check_w(w, out, in, "W");
  check_vec(bias, out, "bias");
  TORCH_CHECK(out % 8 == 0, "output features must be a multiple of 8");
  auto y = torch::empty({rows, out}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  const GemmEpi epi{bias.data_ptr<float>(), relu ? 1 : 0, out_f32 ? 1 : 0};
  const ConvGeom g = gemm_geom(rows, in, out);
  check_hip(launch_conv_fwd(g, x.data_ptr(), w.data_ptr(), y.data_ptr(), nullptr, head_cfg(rows, out, in),
                            cur_stream(), nullptr, nullptr, &epi),
            "head gemm_fwd");
  return y;
}

torch::Tensor to_bf16(const torch::Tensor& x) {
  if (x.scalar_type() == at::kBFloat16) return x;
  check_2d(x, at::kFloat, "x");
  auto y = torch::empty(x.sizes(), x.options().dtype(at::kBFloat16));
  check_hip(launch_cast_f32_bf16(x.data_ptr<float>(), y.data_ptr(), x.numel(), cur_stream()), "cast_f32_bf16");
  return y;
}

// sink[c] += Σ_rows slab[rows][nsets][C] set 0 (fp64 reduction, one launch)
void colsum_into(const torch::Tensor& slab, int64_t rows, int nsets, int64_t C, torch::Tensor& sink) {
  check_vec(sink, C, "bias sink");
  BnCoefArgs a{};
  a.dbeta_a = sink.data_ptr<float>();
  a.grad_scale = 1.0;
  auto sums = torch::empty({nsets, C}, slab.options().dtype(at::kDouble));
  auto scratch = reduce_scratch(slab, rows, nsets, C);
  check_hip(launch_col_reduce(slab.data_ptr<float>(), (int)rows, nsets, (int)C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device()), sums.data_ptr<double>(), 3, nullptr, &a, cur_stream()),
            "head bias-gradient reduction");
}

// dW (+)= dyᵀ·x into an fp32 [out][in] sink
void gemm_wgrad(const torch::Tensor& dy, const torch::Tensor& x, torch::Tensor& sink) {
  const int64_t rows = dy.size(0), out = dy.size(1), in = x.size(1);
  TORCH_CHECK(sink.is_cuda() && sink.scalar_type() == at::kFloat && sink.is_contiguous() && sink.numel() == out * in,
              "weight sink must be a contiguous fp32 [out, in] tensor");
  conv_wgrad(dy.view({rows, 1, 1, out}), x.view({rows, 1, 1, in}), 1, 1, 1, 0, 0, -1, sink.view({out, 1, 1, in}),
             true, c10::nullopt, c10::nullopt);
}

// dx[rows][in] = dy[rows][out] · Wt[in][out]ᵀ, optionally ReLU-masked by (ref > 0) with the
// masked column sums added into `bias_sink` (the hidden layer's bias gradient)
// (slab_out: the caller reduces the bias-gradient slab itself, e.g. on another stream)
torch::Tensor gemm_dgrad(const torch::Tensor& dy, const torch::Tensor& wt, int64_t in, bool out_f32,
                         const torch::Tensor* relu_ref, torch::Tensor* bias_sink, torch::Tensor* slab_out = nullptr) {
  const int64_t rows = dy.size(0), out = dy.size(1);
  check_w(wt, in, out, "Wt");
  TORCH_CHECK(in % 8 == 0, "input features must be a multiple of 8");
  const ConvGeom g = gemm_geom(rows, in, out);
  // the masked-store statistics variant exists for the 64x64 LDS-DMA tile only (igemm.hip)
  const int cfg = relu_ref != nullptr ? 3 : head_cfg(rows, in, out);
  auto dx = torch::empty({rows, in}, dy.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  const GemmEpi epi{nullptr, 0, out_f32 ? 1 : 0};
  if (relu_ref == nullptr) {
    check_hip(launch_conv_dgrad_class(g, 0, 0, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), nullptr, cfg,
                                      cur_stream(), nullptr, nullptr, 0, &epi),
              "head gemm_dgrad");
    return dx;
  }
  TORCH_CHECK(!out_f32 && bias_sink != nullptr, "masked dgrad: bf16 output with a bias sink");
  check_2d(*relu_ref, at::kBFloat16, "relu_ref");
  TORCH_CHECK(relu_ref->size(0) == rows && relu_ref->size(1) == in, "relu_ref shape");
  const int64_t mt = conv_dgrad_class_mtiles(g, 0, 0, cfg);
  auto slab = torch::empty({mt, 2, in}, dy.options().dtype(at::kFloat));
  BnBwdStat bs{};
  bs.slab = slab.data_ptr<float>();
  bs.ya = relu_ref->data_ptr();
  bs.ma = const_vec(dy.device(), in, 0.f).data_ptr<float>();
  bs.msc = const_vec(dy.device(), in, 1.f).data_ptr<float>();   // mask: ref·1 + 0 > 0
  bs.msh = bs.ma;
  bs.store_masked = 1;
  check_hip(launch_conv_dgrad_class(g, 0, 0, dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), nullptr, cfg, cur_stream(),
                                    nullptr, &bs, 0, &epi),
            "head gemm_dgrad(relu)");
  if (slab_out != nullptr) *slab_out = slab;
  else colsum_into(slab, mt, 2, in, *bias_sink);
  return dx;
}

// the head's side-stream fork: everything queued on the compute stream so far, then `keep`
// stays alive until the side stream is joined (side_stash). Own small event pool: two forks
// per step; no system-scope fence (same-device stream ordering, conv_bn_ops.cpp next_event)
void head_fork(hipStream_t main, hipStream_t ss, std::initializer_list<torch::Tensor> keep) {
  static std::mutex mu;
  static std::vector<hipEvent_t> pool;
  static size_t next = 0;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (pool.empty()) {
      pool.resize(64);
      for (auto& e : pool)
        check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreate");
    }
    ev = pool[next];
    next = (next + 1) % pool.size();
  }
  check_hip(hipEventRecord(ev, main), "hipEventRecord");
  check_hip(hipStreamWaitEvent(ss, ev, 0), "hipStreamWaitEvent");
  for (const auto& t : keep) side_stash().push_back(t);
}

// feat [N][D] fp32|bf16; w1 [O1][D] bf16 (+ b1 fp32); MLP: w2 [O2][O1] bf16 (+ b2).
// Returns [z fp32 [N][O_last], fb bf16 [N][D], h bf16 [N][O1] (MLP; empty otherwise)].
std::vector<torch::Tensor> head_fwd(torch::Tensor feat, torch::Tensor w1, torch::Tensor b1, OptT w2, OptT b2) {
  TORCH_CHECK(feat.dim() == 2, "feat must be [N, D]");
  feat = feat.contiguous();
  check_2d(feat, feat.scalar_type() == at::kBFloat16 ? at::kBFloat16 : at::kFloat, "feat");
  c10::DeviceGuard dg(feat.device());
  auto fb = to_bf16(feat);
  if (!w2.has_value()) {
    auto z = gemm_fwd(fb, w1, b1, false, true);
    return {z, fb, torch::empty({0}, fb.options())};
  }
  TORCH_CHECK(b2.has_value(), "b2 required with w2");
  auto h = gemm_fwd(fb, w1, b1, true, false);
  auto z = gemm_fwd(h, *w2, *b2, false, true);
  return {z, fb, h};
}

// dz [N][O_last] fp32; w1t [D][O1] / w2t [O1][O2] bf16 (dgrad layouts, Wᵀ); sinks fp32.
// Accumulates every parameter gradient into its sink; returns dfeat fp32 [N][D].
// side (a stream handle, 0 = none): the weight gradients and the output bias gradient run
// on the wgrad side stream, off the data-gradient chain into the encoder's backward
torch::Tensor head_bwd(torch::Tensor dz, torch::Tensor fb, OptT h, torch::Tensor w1t, OptT w2t, torch::Tensor sw1,
                       torch::Tensor sb1, OptT sw2, OptT sb2, int64_t side) {
  dz = dz.contiguous();
  check_2d(dz, at::kFloat, "dz");
  check_2d(fb, at::kBFloat16, "fb");
  TORCH_CHECK(dz.size(0) == fb.size(0), "dz / fb rows");
  c10::DeviceGuard dg(dz.device());
  const int64_t rows = dz.size(0), D = fb.size(1), O = dz.size(1);
  auto dzb = to_bf16(dz);
  const bool mlp = w2t.has_value();
  torch::Tensor& sb_last = mlp ? *sb2 : sb1;
  if (side != 0 && mlp) {
    TORCH_CHECK(h.has_value() && sw2.has_value() && sb2.has_value(), "MLP head: h, sw2, sb2 required");
    check_2d(*h, at::kBFloat16, "h");
    const int64_t O1 = h->size(1);
    hipStream_t main = cur_stream(), ss = reinterpret_cast<hipStream_t>(side);
    auto hs = c10::hip::getStreamFromExternal(ss, dz.device().index());
    head_fork(main, ss, {dz, dzb, *h});
    {
      c10::hip::HIPStreamGuard guard(hs);
      colsum_into(dz, rows, 1, O, sb_last);
      gemm_wgrad(dzb, *h, *sw2);
    }
    torch::Tensor slab1;   // the hidden bias gradient's column sums, reduced on the side stream
    auto dh = gemm_dgrad(dzb, *w2t, O1, false, &*h, &sb1, &slab1);
    head_fork(main, ss, {dh, fb, slab1});
    {
      c10::hip::HIPStreamGuard guard(hs);
      colsum_into(slab1, slab1.size(0), 2, O1, sb1);
      gemm_wgrad(dh, fb, sw1);
    }
    return gemm_dgrad(dh, w1t, D, true, nullptr, nullptr);
  }
  colsum_into(dz, rows, 1, O, sb_last);   // db_last += Σ_rows dz (dz viewed as a [rows][1][O] slab)
  if (!mlp) {
    gemm_wgrad(dzb, fb, sw1);
    return gemm_dgrad(dzb, w1t, D, true, nullptr, nullptr);
  }
  TORCH_CHECK(h.has_value() && sw2.has_value() && sb2.has_value(), "MLP head: h, sw2, sb2 required");
  check_2d(*h, at::kBFloat16, "h");
  const int64_t O1 = h->size(1);
  gemm_wgrad(dzb, *h, *sw2);
  auto dh = gemm_dgrad(dzb, *w2t, O1, false, &*h, &sb1);
  gemm_wgrad(dh, fb, sw1);
  return gemm_dgrad(dh, w1t, D, true, nullptr, nullptr);
}

}  // namespace

void register_head(pybind11::module& m) {
  m.def("head_fwd", &head_fwd, "projection head forward on igemm MFMA GEMMs -> [z fp32, fb bf16, h bf16]",
        pybind11::arg("feat"), pybind11::arg("w1"), pybind11::arg("b1"), pybind11::arg("w2") = pybind11::none(),
        pybind11::arg("b2") = pybind11::none());
  m.def("head_bwd", &head_bwd, "projection head backward: gradients into the sinks, returns dfeat fp32",
        pybind11::arg("dz"), pybind11::arg("fb"), pybind11::arg("h"), pybind11::arg("w1t"), pybind11::arg("w2t"),
        pybind11::arg("sw1"), pybind11::arg("sb1"), pybind11::arg("sw2") = pybind11::none(),
        pybind11::arg("sb2") = pybind11::none(), pybind11::arg("side") = 0);
}

}  // namespace sdx_bind
