// Host helpers of the conv/BN binding layer (conv_bn_ops.cpp) shared with the other
// executors built on the same kernels (head_ops.cpp: the projection head as 1x1 GEMMs).
#pragma once
#include <torch/extension.h>

#include "launchers.h"

namespace sdx_bind {
using OptT = c10::optional<torch::Tensor>;

void check_bf16_nhwc(const torch::Tensor& t, const char* name);
void check_vec(const torch::Tensor& t, int64_t C, const char* name);
const float* opt_ptr(const OptT& t, int64_t C, const char* name);
// tile config for an M x Ncol GEMM with reduction Kdim (fill: charge idle CUs of the last round)
int auto_cfg(int64_t M, int64_t Ncol, int64_t Kdim = 0, bool fill = false);
// dW (+)= wgrad(dy, x) (fp32, KRSC), split-K slab reduced deterministically
torch::Tensor conv_wgrad(torch::Tensor dy, torch::Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                         int64_t splits, int64_t cfg, OptT out, bool accumulate, OptT in_scale, OptT in_shift);
// ticket counters + fp64 scratch of the single-launch column reduction (bn.hip col_reduce)
// (nslots / z: one block per emulated rank of a fused SyncBN exchange, XgmiCol mode 2)
unsigned* reduce_counters(const torch::Device& dev, int nslots = 1);
torch::Tensor reduce_scratch(const torch::Tensor& like, int64_t rows, int64_t nsets, int64_t C, int z = 1);
// the fused SyncBN exchange of one BN on communicator `comm` (off: reduce -> all-reduce -> epilogue)
struct FusedX {
  XgmiCol x{};
  bool on = false;
  int z() const { return on && x.mode == 2 && !x.solo ? x.world : 1; }
  const XgmiCol* p() const { return on ? &x : nullptr; }
};
FusedX fused_exchange(int64_t comm);
}  // namespace sdx_bind
