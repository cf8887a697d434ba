// Bindings for the GPU data-pipeline kernels (aug.hip).
#include "ops_decl.h"
#include "launchers.h"

namespace sdx_bind {
namespace {

// seed_t (optional int64 GPU scalar) overrides `seed` at kernel run time, so a captured
// hipGraph draws fresh augmentations on every replay.
torch::Tensor gpu_augment(torch::Tensor data, torch::Tensor idx, int64_t S, int64_t n_views, int64_t seed,
                          std::vector<double> mean, std::vector<double> std, double scale_lo, double scale_hi,
                          double ratio_lo, double ratio_hi, double jitter_p, double bright, double contrast,
                          double sat, double hue, double gray_p, bool do_crop, bool do_flip,
                          c10::optional<torch::Tensor> seed_t, c10::optional<torch::Tensor> offs,
                          c10::optional<torch::Tensor> hw) {
  const bool ragged = offs.has_value();
  TORCH_CHECK(ragged == hw.has_value(), "offs and hw must be given together");
  if (ragged) {
    TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 1 && data.is_contiguous(),
                "ragged data must be a contiguous uint8 GPU byte vector");
    TORCH_CHECK(offs->is_cuda() && offs->scalar_type() == at::kLong && offs->dim() == 1 && offs->is_contiguous(),
                "offs must be a contiguous int64 GPU vector");
    TORCH_CHECK(hw->is_cuda() && hw->scalar_type() == at::kInt && hw->dim() == 2 && hw->size(1) == 2 &&
                    hw->size(0) == offs->size(0) && hw->is_contiguous(),
                "hw must be a contiguous int32 [N, 2] GPU tensor");
  } else {
    TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 4 && data.size(3) == 3 &&
                    data.is_contiguous(),
                "data must be a contiguous uint8 [N,H,W,3] GPU tensor");
  }
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(),
              "idx must be a contiguous int64 GPU vector");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "mean/std need 3 values");
  TORCH_CHECK(S >= 1 && n_views >= 1 && idx.size(0) >= 1, "bad sizes");
  const int64_t* sd_dev = nullptr;
  if (seed_t.has_value()) {
    TORCH_CHECK(seed_t->is_cuda() && seed_t->scalar_type() == at::kLong && seed_t->numel() == 1,
                "seed_t must be an int64 GPU scalar");
    sd_dev = seed_t->data_ptr<int64_t>();
  }
  c10::DeviceGuard dg(data.device());
  const int64_t B = idx.size(0);
  auto out = torch::empty({n_views * B, S, S, 8}, data.options().dtype(at::kBFloat16));
  float m[3], sd[3];
  for (int k = 0; k < 3; ++k) { m[k] = (float)mean[k]; sd[k] = (float)std[k]; }
  const int H = ragged ? 0 : (int)data.size(1), W = ragged ? 0 : (int)data.size(2);
  const long n_data = ragged ? (long)offs->size(0) : (long)data.size(0);
  check_hip(launch_gpu_augment(data.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(), (int)B, H, W, (int)S, (int)n_views,
                               (uint64_t)seed, m, sd, (float)scale_lo,
                               (float)scale_hi, (float)ratio_lo, (float)ratio_hi, (float)jitter_p, (float)bright,
                               (float)contrast, (float)sat, (float)hue, (float)gray_p, do_crop ? 1 : 0,
                               do_flip ? 1 : 0, sd_dev, out.data_ptr(), cur_stream(), n_data,
                               ragged ? offs->data_ptr<int64_t>() : nullptr, ragged ? hw->data_ptr<int32_t>() : nullptr),
            "gpu_augment");
  return out;
}

}  // namespace

void register_data(pybind11::module& m) {
  m.def("gpu_augment", &gpu_augment, "fused SimCLR augmentation -> NHWC bf16 (C padded to 8)",
        pybind11::arg("data"), pybind11::arg("idx"), pybind11::arg("S"), pybind11::arg("n_views"),
        pybind11::arg("seed"), pybind11::arg("mean"), pybind11::arg("std"), pybind11::arg("scale_lo"),
        pybind11::arg("scale_hi"), pybind11::arg("ratio_lo"), pybind11::arg("ratio_hi"), pybind11::arg("jitter_p"),
        pybind11::arg("bright"), pybind11::arg("contrast"), pybind11::arg("sat"), pybind11::arg("hue"),
        pybind11::arg("gray_p"), pybind11::arg("do_crop"), pybind11::arg("do_flip"),
        pybind11::arg("seed_t") = pybind11::none(), pybind11::arg("offs") = pybind11::none(),
        pybind11::arg("hw") = pybind11::none());
}

}  // namespace sdx_bind
