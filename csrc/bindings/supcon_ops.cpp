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
  auto dA = torch::empty_like(A);
  auto dC = torch::empty_like(C);
  auto ws = torch::empty({std::max<long>(1, supcon_bwd_workspace((int)Na, (int)N, (int)D))}, A.options());
  check_hip(launch_supcon_bwd(A.data_ptr<float>(), C.data_ptr<float>(), a_self.data_ptr<int>(),
                              a_key.data_ptr<int>(), c_key.data_ptr<int>(), lse.data_ptr<float>(),
                              invcnt.data_ptr<float>(), (int)Na, (int)N, (int)D, (float)inv_temp, (float)w,
                              gc.data_ptr<float>(), dA.data_ptr<float>(), dC.data_ptr<float>(),
                              ws.data_ptr<float>(), cur_stream()),
            "supcon_bwd");
  return {dA, dC};
}

// anchors == contrasts (single rank, contrast_mode all): the gradient w.r.t. the one
// feature tensor, dA + dC summed in the split reduction (one launch less, no add kernel)
torch::Tensor supcon_bwd_sum(torch::Tensor X, torch::Tensor a_self, torch::Tensor a_key, torch::Tensor c_key,
                             torch::Tensor lse, torch::Tensor invcnt, torch::Tensor g, double inv_temp, double w) {
  check_rows(X, "X");
  const int64_t N = X.size(0), D = X.size(1);
  TORCH_CHECK(D == 64 || D == 128 || D == 256, "bad feature dim");
  check_idx(a_self, N, "a_self");
  check_idx(a_key, N, "a_key");
  check_idx(c_key, N, "c_key");
  TORCH_CHECK(lse.is_cuda() && lse.numel() == N && invcnt.numel() == N, "lse/invcnt shape");
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.numel() == 1, "g must be a GPU float scalar");
  c10::DeviceGuard dg(X.device());
  auto gc = g.contiguous();
  auto dX = torch::empty_like(X);
  auto ws = torch::empty({std::max<long>(1, supcon_bwd_sum_workspace((int)N, (int)D))}, X.options());
  check_hip(launch_supcon_bwd_sum(X.data_ptr<float>(), a_self.data_ptr<int>(), a_key.data_ptr<int>(),
                                  c_key.data_ptr<int>(), lse.data_ptr<float>(), invcnt.data_ptr<float>(), (int)N,
                                  (int)D, (float)inv_temp, (float)w, gc.data_ptr<float>(), dX.data_ptr<float>(),
                                  ws.data_ptr<float>(), cur_stream()),
            "supcon_bwd_sum");
  return dX;
}

// F.normalize(x, dim=1) as one launch: returns (y, row norms)
std::vector<torch::Tensor> rownorm_fwd(torch::Tensor x, double eps) {
  check_rows(x, "x");
  TORCH_CHECK(x.size(1) <= 256, "feature dim must be <= 256");
  c10::DeviceGuard dg(x.device());
  auto y = torch::empty_like(x);
  auto norms = torch::empty({x.size(0)}, x.options());
  check_hip(launch_rownorm_fwd(x.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (float)eps, y.data_ptr<float>(),
                               norms.data_ptr<float>(), cur_stream()),
            "rownorm_fwd");
  return {y, norms};
}

torch::Tensor rownorm_bwd(torch::Tensor dy, torch::Tensor y, torch::Tensor norms, double eps) {
  check_rows(dy, "dy");
  check_rows(y, "y");
  TORCH_CHECK(dy.sizes() == y.sizes() && norms.is_cuda() && norms.scalar_type() == at::kFloat &&
                  norms.numel() == y.size(0),
              "rownorm_bwd shapes");
  c10::DeviceGuard dg(dy.device());
  auto dx = torch::empty_like(dy);
  check_hip(launch_rownorm_bwd(dy.data_ptr<float>(), y.data_ptr<float>(), norms.contiguous().data_ptr<float>(),
                               (int)dy.size(0), (int)dy.size(1), (float)eps, dx.data_ptr<float>(), cur_stream()),
            "rownorm_bwd");
  return dx;
}

// SEC / L2-reg statistics of un-normalised features (featnorm.hip). mode 0: local sums into
// `sums` ([2] fp64) only; 1: local sums + finalize; 2: finalize from the given (all-reduced)
// sums. rec / valid: the record_norm_mean EMA state ([] fp32, updated in place).
// Returns out [5] = (norm_mean, norm_var, record_norm_mean, loss_sec, loss_l2).
torch::Tensor norm_stats(torch::Tensor x, int64_t mode, torch::Tensor sums, double n_global, double momentum,
                         torch::Tensor rec, torch::Tensor valid) {
  check_rows(x, "x");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kDouble && sums.numel() == 2 && sums.is_contiguous(),
              "sums: [2] float64");
  TORCH_CHECK(rec.is_cuda() && rec.scalar_type() == at::kFloat && rec.numel() == 1, "rec: float scalar");
  TORCH_CHECK(valid.is_cuda() && valid.scalar_type() == at::kFloat && valid.numel() == 1, "valid: float scalar");
  c10::DeviceGuard dg(x.device());
  auto out = torch::empty({5}, x.options());
  check_hip(launch_norm_stats(x.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)mode, sums.data_ptr<double>(),
                              n_global, (float)momentum, rec.data_ptr<float>(), valid.data_ptr<float>(),
                              out.data_ptr<float>(), cur_stream()),
            "norm_stats");
  return out;
}

}  // namespace

void register_supcon(pybind11::module& m) {
  m.def("rownorm_fwd", &rownorm_fwd, "row L2 normalisation (F.normalize dim=1) -> (y, norms)");
  m.def("rownorm_bwd", &rownorm_bwd, "gradient of row L2 normalisation");
  m.def("norm_stats", &norm_stats, "SEC/L2-reg feature-norm statistics + record_norm_mean EMA (one launch)");
  m.def("supcon_fwd", &supcon_fwd, "fused SupCon/NT-Xent forward (row form)");
  m.def("supcon_bwd", &supcon_bwd, "fused SupCon/NT-Xent backward (row form)");
  m.def("supcon_bwd_sum", &supcon_bwd_sum, "SupCon backward when anchors are the contrasts: dA + dC in one reduce");
}

}  // namespace sdx_bind
