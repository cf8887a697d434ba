// Linear-probe classifier (linear_ce.hip): fused logits + cross-entropy + top-k hits, and
// the gradient + SGD update, for the native linear evaluation (ops/linear_probe.py;
// reference main_linear.py:166-244).
#include "conv_internal.h"
#include "launchers.h"
#include "ops_decl.h"

bool linear_ce_supported(int K, int C);
hipError_t launch_linear_ce_fwd(const float* x, const float* W, const float* bias, const int64_t* labels, int B,
                                int K, int C, float gscale, float* logits, float* dz, float* rowstat, hipStream_t s);
hipError_t launch_linear_ce_sgd(const float* x, const float* dz, int B, int K, int C, float* W, float* bias,
                                float* bufW, float* bufb, float lr, float mom, float wd, int first,
                                const float* rowstat, float* stats, hipStream_t s);

namespace sdx_bind {
namespace {

void check_f32(const torch::Tensor& t, std::vector<int64_t> shape, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.sizes() == shape, name,
              " must be a contiguous fp32 GPU tensor of shape ", shape);
}

// One classifier batch. train: logits, the mean-CE gradient and the SGD update of (W, b)
// with momentum buffers (bufW, bufb; `first` = no momentum history yet); eval: logits only.
// Returns [logits [B][C], stats [3] = (Σ_rows CE, top-1 hits, top-5 hits)].
std::vector<torch::Tensor> linear_ce_step(torch::Tensor x, torch::Tensor W, torch::Tensor b, torch::Tensor labels,
                                          OptT bufW, OptT bufb, double lr, double momentum, double wd, bool first,
                                          bool train) {
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2, "x [B][K], W [C][K]");
  const int64_t B = x.size(0), K = x.size(1), C = W.size(0);
  check_f32(x, {B, K}, "x");
  check_f32(W, {C, K}, "W");
  check_f32(b, {C}, "b");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.numel() == B && labels.is_contiguous(),
              "labels: int64 [B]");
  TORCH_CHECK(linear_ce_supported((int)K, (int)C) && ((K / 64) & (K / 64 - 1)) == 0,
              "linear_ce: K = 64·2^j <= 2048, C <= 1024");
  TORCH_CHECK(B * C < (1LL << 31) && B * K < (1LL << 31), "linear_ce: sizes");
  if (train) {
    TORCH_CHECK(bufW.has_value() && bufb.has_value(), "momentum buffers required for a training step");
    check_f32(*bufW, {C, K}, "bufW");
    check_f32(*bufb, {C}, "bufb");
  }
  c10::DeviceGuard dg(x.device());
  auto fo = x.options();
  auto logits = torch::empty({B, C}, fo);
  auto rowstat = torch::empty({B, 3}, fo);
  auto stats = torch::empty({3}, fo);
  torch::Tensor dz;
  if (train) dz = torch::empty({B, C}, fo);
  check_hip(launch_linear_ce_fwd(x.data_ptr<float>(), W.data_ptr<float>(), b.data_ptr<float>(),
                                 labels.data_ptr<int64_t>(), (int)B, (int)K, (int)C, (float)(1.0 / B),
                                 logits.data_ptr<float>(), train ? dz.data_ptr<float>() : nullptr,
                                 rowstat.data_ptr<float>(), cur_stream()),
            "linear_ce_fwd");
  check_hip(launch_linear_ce_sgd(x.data_ptr<float>(), train ? dz.data_ptr<float>() : nullptr, (int)B, (int)K, (int)C,
                                 train ? W.data_ptr<float>() : nullptr, train ? b.data_ptr<float>() : nullptr,
                                 train ? bufW->data_ptr<float>() : nullptr, train ? bufb->data_ptr<float>() : nullptr,
                                 (float)lr, (float)momentum, (float)wd, first ? 1 : 0, rowstat.data_ptr<float>(),
                                 stats.data_ptr<float>(), cur_stream()),
            "linear_ce_sgd");
  return {logits, stats};
}

}  // namespace

void register_probe(pybind11::module& m) {
  m.def("linear_ce_step", &linear_ce_step,
        "linear classifier + mean cross-entropy + top-1/5 hits (+ gradient and SGD update when train)",
        pybind11::arg("x"), pybind11::arg("W"), pybind11::arg("b"), pybind11::arg("labels"), pybind11::arg("bufW"),
        pybind11::arg("bufb"), pybind11::arg("lr"), pybind11::arg("momentum"), pybind11::arg("wd"),
        pybind11::arg("first"), pybind11::arg("train"));
}

}  // namespace sdx_bind
