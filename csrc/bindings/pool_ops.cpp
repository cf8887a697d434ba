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
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
}

}  // namespace sdx_bind
