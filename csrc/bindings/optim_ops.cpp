// Bindings for the fused flat-buffer optimizers (optim.hip).
#include "ops_decl.h"
#include "launchers.h"

namespace sdx_bind {
namespace {

void check_flat(const torch::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 1 && t.numel() == n,
              name, " must be a contiguous flat float32 GPU tensor of the parameter size");
}

void sgd_step(torch::Tensor p, torch::Tensor g, torch::Tensor buf, torch::Tensor lr, double momentum, double wd,
              double gscale, bool nesterov, int64_t max_blocks) {
  const int64_t n = p.numel();
  check_flat(p, n, "p");
  check_flat(g, n, "g");
  check_flat(buf, n, "buf");
  TORCH_CHECK(n % 4 == 0, "flat size must be a multiple of 4");
  TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat && lr.numel() == 1, "lr must be a GPU float scalar");
  c10::DeviceGuard dg(p.device());
  check_hip(launch_sgd(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(), n, lr.data_ptr<float>(),
                       (float)momentum, (float)wd, (float)gscale, nesterov ? 1 : 0, cur_stream(), (int)max_blocks),
            "sgd_step");
}

void lars_step(torch::Tensor p, torch::Tensor g, torch::Tensor buf, torch::Tensor seg_off, torch::Tensor adapt,
               torch::Tensor lr, double momentum, double wd, double gscale, double eta, torch::Tensor norms) {
  const int64_t n = p.numel();
  check_flat(p, n, "p");
  check_flat(g, n, "g");
  check_flat(buf, n, "buf");
  const int64_t nseg = seg_off.numel();
  TORCH_CHECK(seg_off.is_cuda() && seg_off.scalar_type() == at::kLong && seg_off.is_contiguous(), "seg_off int64");
  TORCH_CHECK(adapt.is_cuda() && adapt.scalar_type() == at::kInt && adapt.numel() == nseg, "adapt int32[nseg]");
  TORCH_CHECK(norms.is_cuda() && norms.scalar_type() == at::kFloat && norms.numel() == 2 * nseg, "norms [2*nseg]");
  TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat && lr.numel() == 1, "lr must be a GPU float scalar");
  c10::DeviceGuard dg(p.device());
  check_hip(launch_lars(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(), seg_off.data_ptr<int64_t>(),
                        adapt.data_ptr<int>(), (int)nseg, n, lr.data_ptr<float>(), (float)momentum, (float)wd,
                        (float)gscale, (float)eta, norms.data_ptr<float>(), cur_stream()),
            "lars_step");
}

// zero a contiguous GPU buffer with the runtime's fill (hipMemsetAsync on the current stream):
// the flat gradient buffer's per-step reset without a torch elementwise kernel in the step
void zero_async(torch::Tensor t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_async: contiguous GPU tensor");
  c10::DeviceGuard dg(t.device());
  check_hip(hipMemsetAsync(t.data_ptr(), 0, t.nbytes(), cur_stream()), "zero_async");
}

}  // namespace

void register_optim(pybind11::module& m) {
  m.def("zero_async", &zero_async, "hipMemsetAsync(0) of a contiguous GPU tensor on the current stream");
  m.def("sgd_step", &sgd_step, "fused flat-buffer SGD (momentum, wd, grad scale, device lr)", pybind11::arg("p"),
        pybind11::arg("g"), pybind11::arg("buf"), pybind11::arg("lr"), pybind11::arg("momentum"), pybind11::arg("wd"),
        pybind11::arg("gscale"), pybind11::arg("nesterov"), pybind11::arg("max_blocks") = 0);
  m.def("lars_step", &lars_step, "fused flat-buffer LARS");
}

}  // namespace sdx_bind

namespace sdx_bind {
namespace {

void wprep(torch::Tensor master, torch::Tensor out, torch::Tensor segs, int64_t total) {
  TORCH_CHECK(master.is_cuda() && master.scalar_type() == at::kFloat && master.is_contiguous(), "master fp32");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous(), "out bf16");
  TORCH_CHECK(segs.is_cuda() && segs.scalar_type() == at::kLong && segs.dim() == 2 && segs.size(1) == 7 &&
                  segs.is_contiguous(),
              "segs int64 [nseg, 7]");
  c10::DeviceGuard dg(master.device());
  check_hip(launch_wprep(master.data_ptr<float>(), out.data_ptr(), segs.data_ptr(), (int)segs.size(0), total,
                         cur_stream()),
            "wprep");
}

// dst (fp32 [..., C], contiguous) += src[..., :C] (fp32 [..., Cp], contiguous), same leading dims
void unpad_add(torch::Tensor src, torch::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat && src.is_contiguous(), "src fp32 contiguous");
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.is_contiguous(), "dst fp32 contiguous");
  TORCH_CHECK(src.dim() == dst.dim() && src.dim() >= 1, "same rank");
  for (int64_t d = 0; d + 1 < src.dim(); ++d) TORCH_CHECK(src.size(d) == dst.size(d), "leading dims");
  const int64_t Cp = src.size(-1), C = dst.size(-1);
  TORCH_CHECK(C <= Cp && src.numel() / Cp * C < (1LL << 31), "C <= Cp");
  c10::DeviceGuard dg(src.device());
  check_hip(launch_unpad_add(src.data_ptr<float>(), dst.data_ptr<float>(), (int)(src.numel() / Cp), (int)Cp, (int)C,
                             cur_stream()),
            "unpad_add");
}

}  // namespace

void register_wprep(pybind11::module& m) {
  m.def("wprep", &wprep, "fp32 master -> bf16 fwd/dgrad conv weights");
  m.def("unpad_add", &unpad_add, "dst += src[..., :C] of a channel-padded fp32 tensor");
}

}  // namespace sdx_bind
