// Python bindings for the gfx950 kernels (torch extension module
// `simclr_pytorch_distributed_amd._C`). Every op validates shapes/dtypes on the host
// BEFORE launching (a mis-shaped launch of a hand-written kernel can fault the GPU),
// then launches on the caller's current HIP stream so torch stream semantics and
// hipGraph capture work unchanged.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "launchers.h"
#include "ops_decl.h"

namespace sdx_bind {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

torch::Tensor mfma16_selftest(torch::Tensor A, torch::Tensor B) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda(), "selftest: tensors must be on the GPU");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "bf16 only");
  TORCH_CHECK(A.sizes() == at::IntArrayRef({16, 32}) && B.sizes() == at::IntArrayRef({32, 16}),
              "selftest shapes are fixed: A[16,32], B[32,16]");
  A = A.contiguous();
  B = B.contiguous();
  c10::DeviceGuard g(A.device());
  auto C = torch::empty({16, 16}, A.options().dtype(at::kFloat));
  check_hip(launch_mfma16_selftest(A.data_ptr(), B.data_ptr(), C.data_ptr<float>(), cur_stream()),
            "mfma16_selftest");
  return C;
}

}  // namespace sdx_bind

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "MI355X (gfx950) native kernels for simclr_pytorch_distributed_amd";
  m.def("mfma16_selftest", &sdx_bind::mfma16_selftest, "16x16x32 bf16 MFMA layout self-test");
  sdx_bind::register_ops(m);
}
