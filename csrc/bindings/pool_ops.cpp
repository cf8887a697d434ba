// Bindings for the NHWC pooling kernels (pool.hip).
#include "ops_decl.h"
#include "launchers.h"

namespace sdx_bind {
namespace {

void check_nhwc(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 && t.is_contiguous() &&
                  t.size(3) % 8 == 0,
              name, " must be a contiguous NHWC bf16 GPU tensor with C % 8 == 0");
}

torch::Tensor maxpool_fwd(torch::Tensor x, int64_t k, int64_t stride, int64_t pad) {
  check_nhwc(x, "x");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0 && pad < k, "bad pool geometry");
  c10::DeviceGuard dg(x.device());
  auto y = torch::empty({N, P, Q, C}, x.options());
  check_hip(launch_maxpool_fwd(x.data_ptr(), y.data_ptr(), N, H, W, C, P, Q, k, stride, pad, cur_stream()),
            "maxpool_fwd");
  return y;
}

torch::Tensor maxpool_bwd(torch::Tensor x, torch::Tensor y, torch::Tensor dy, int64_t k, int64_t stride, int64_t pad) {
  check_nhwc(x, "x");
  check_nhwc(y, "y");
  check_nhwc(dy, "dy");
  TORCH_CHECK(y.sizes() == dy.sizes(), "y/dy shape");
  c10::DeviceGuard dg(x.device());
  auto dx = torch::empty_like(x);
  check_hip(launch_maxpool_bwd(x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.size(0), x.size(1),
                               x.size(2), x.size(3), y.size(1), y.size(2), k, stride, pad, cur_stream()),
            "maxpool_bwd");
  return dx;
}

// max-pool forward + per-window first-max positions (uint8, same shape as y)
std::vector<torch::Tensor> maxpool_fwd_idx(torch::Tensor x, int64_t k, int64_t stride, int64_t pad) {
  check_nhwc(x, "x");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0 && pad < k && k * k <= 255, "bad pool geometry");
  c10::DeviceGuard dg(x.device());
  auto y = torch::empty({N, P, Q, C}, x.options());
  auto idx = torch::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  check_hip(launch_maxpool_fwd_idx(x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), N, H, W, C, P, Q, k, stride,
                                   pad, cur_stream()),
            "maxpool_fwd_idx");
  return {y, idx};
}

// max-pool backward from the recorded positions: dx [N, H, W, C]
torch::Tensor maxpool_bwd_idx(torch::Tensor idx, torch::Tensor dy, int64_t H, int64_t W, int64_t k, int64_t stride,
                              int64_t pad) {
  check_nhwc(dy, "dy");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.sizes() == dy.sizes(),
              "idx: contiguous uint8 of dy's shape");
  TORCH_CHECK((H + 2 * pad - k) / stride + 1 == dy.size(1) && (W + 2 * pad - k) / stride + 1 == dy.size(2),
              "pool geometry mismatch");
  c10::DeviceGuard dg(dy.device());
  auto dx = torch::empty({dy.size(0), H, W, dy.size(3)}, dy.options());
  check_hip(launch_maxpool_bwd_idx(idx.data_ptr<uint8_t>(), dy.data_ptr(), dx.data_ptr(), dy.size(0), H, W,
                                   dy.size(3), dy.size(1), dy.size(2), k, stride, pad, cur_stream()),
            "maxpool_bwd_idx");
  return dx;
}

torch::Tensor gap_fwd(torch::Tensor x) {
  check_nhwc(x, "x");
  c10::DeviceGuard dg(x.device());
  auto y = torch::empty({x.size(0), x.size(3)}, x.options().dtype(at::kFloat));
  check_hip(launch_gap_fwd(x.data_ptr(), y.data_ptr<float>(), x.size(0), x.size(1) * x.size(2), x.size(3),
                           cur_stream()),
            "gap_fwd");
  return y;
}

torch::Tensor gap_bwd(torch::Tensor dy, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kFloat && dy.dim() == 2 && dy.is_contiguous() &&
                  dy.size(1) % 8 == 0,
              "dy must be contiguous float32 [N, C]");
  c10::DeviceGuard dg(dy.device());
  auto dx = torch::empty({dy.size(0), H, W, dy.size(1)}, dy.options().dtype(at::kBFloat16));
  check_hip(launch_gap_bwd(dy.data_ptr<float>(), dx.data_ptr(), dy.size(0), H * W, dy.size(1), cur_stream()),
            "gap_bwd");
  return dx;
}

}  // namespace

void register_pool(pybind11::module& m) {
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("maxpool_fwd_idx", &maxpool_fwd_idx, "max-pool forward + per-window first-max positions (uint8)");
  m.def("maxpool_bwd_idx", &maxpool_bwd_idx, "max-pool backward from the recorded positions",
        pybind11::arg("idx"), pybind11::arg("dy"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("k"),
        pybind11::arg("stride"), pybind11::arg("pad"));
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
}

}  // namespace sdx_bind
