// Bindings for the fused contrastive-loss kernels (supcon.hip).
#include "ops_decl.h"
#include "launchers.h"

namespace sdx_bind {
namespace {

void check_rows(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.dim() == 2 && t.is_contiguous(), name, " must be a contiguous 2-D tensor");
}

void check_idx(const torch::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous(), name,
              " must be a contiguous int32 GPU tensor");
  TORCH_CHECK(t.dim() == 1 && t.size(0) == n, name, " has the wrong length");
}

// Returns (loss[1], lse[Na], invcnt[Na], row_loss[Na]).
std::vector<torch::Tensor> supcon_fwd(torch::Tensor A, torch::Tensor C, torch::Tensor a_self,
                                      torch::Tensor a_key, torch::Tensor c_key, double inv_temp,
                                      double temp_ratio, double scale) {
  check_rows(A, "A");
  check_rows(C, "C");
  const int64_t Na = A.size(0), N = C.size(0), D = A.size(1);
  TORCH_CHECK(C.size(1) == D, "A and C feature dims differ");
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "feature dim must be 64, 128 or 256");
  TORCH_CHECK(Na >= 1 && N >= 1 && N < (1 << 30), "bad row counts");
  check_idx(a_self, Na, "a_self");
  check_idx(a_key, Na, "a_key");
  check_idx(c_key, N, "c_key");
  c10::DeviceGuard g(A.device());
  const int S = supcon_num_splits((int)Na, (int)N);
  auto fo = A.options();
  auto part = torch::empty({4 * S * Na}, fo);
  auto lse = torch::empty({Na}, fo);
  auto invcnt = torch::empty({Na}, fo);
  auto row_loss = torch::empty({Na}, fo);
  auto loss = torch::empty({1}, fo);
  check_hip(launch_supcon_fwd(A.data_ptr<float>(), C.data_ptr<float>(), a_self.data_ptr<int>(),
                              a_key.data_ptr<int>(), c_key.data_ptr<int>(), (int)Na, (int)N, (int)D,
                              (float)inv_temp, (float)temp_ratio, (float)scale, S, part.data_ptr<float>(),
                              lse.data_ptr<float>(), invcnt.data_ptr<float>(), row_loss.data_ptr<float>(),
                              loss.data_ptr<float>(), cur_stream()),
            "supcon_fwd");
  return {loss, lse, invcnt, row_loss};
}

// Returns (dA, dC) for loss = scale * Σ ℓ_i, upstream grad `g` (device scalar).
std::vector<torch::Tensor> supcon_bwd(torch::Tensor A, torch::Tensor C, torch::Tensor a_self,
                                      torch::Tensor a_key, torch::Tensor c_key, torch::Tensor lse,
                                      torch::Tensor invcnt, torch::Tensor g, double inv_temp, double w) {
  check_rows(A, "A");
  check_rows(C, "C");
  const int64_t Na = A.size(0), N = C.size(0), D = A.size(1);
  TORCH_CHECK(C.size(1) == D && (D == 64 || D == 128 || D == 256), "bad feature dim");
  check_idx(a_self, Na, "a_self");
  check_idx(a_key, Na, "a_key");
  check_idx(c_key, N, "c_key");
  TORCH_CHECK(lse.is_cuda() && lse.numel() == Na && invcnt.numel() == Na, "lse/invcnt shape");
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.numel() == 1, "g must be a GPU float scalar");
  c10::DeviceGuard dg(A.device());
  auto gc = g.contiguous();
  auto dA = torch::zeros_like(A);
  auto dC = torch::zeros_like(C);
  check_hip(launch_supcon_bwd(A.data_ptr<float>(), C.data_ptr<float>(), a_self.data_ptr<int>(),
                              a_key.data_ptr<int>(), c_key.data_ptr<int>(), lse.data_ptr<float>(),
                              invcnt.data_ptr<float>(), (int)Na, (int)N, (int)D, (float)inv_temp, (float)w,
                              gc.data_ptr<float>(), dA.data_ptr<float>(), dC.data_ptr<float>(), cur_stream()),
            "supcon_bwd");
  return {dA, dC};
}

}  // namespace

void register_supcon(pybind11::module& m) {
  m.def("supcon_fwd", &supcon_fwd, "fused SupCon/NT-Xent forward (row form)");
  m.def("supcon_bwd", &supcon_bwd, "fused SupCon/NT-Xent backward (row form)");
}

}  // namespace sdx_bind
