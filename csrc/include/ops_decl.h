// Registration hooks of the per-family binding translation units. Splitting the
// bindings keeps each torch-header-heavy TU small so incremental rebuilds stay fast.
#pragma once
#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include "launchers.h"

namespace sdx_bind {
hipStream_t cur_stream();
void check_hip(hipError_t e, const char* what);

void register_ops(pybind11::module& m);

// native small communicators (comm_ops.cpp): handle 0 = single process
int small_comm_world(int64_t h);
void small_all_reduce_(int64_t h, torch::Tensor& x);
// fused SyncBN exchange inside the BN-statistics column reduction (xGMI kinds): fills the
// arguments of one exchange, or returns false (use reduce -> small_all_reduce_ -> epilogue)
bool small_comm_fused(int64_t h, XgmiCol* out);
void small_comm_fused_issued(int64_t h);   // arm the watchdog behind the fused launch
}  // namespace sdx_bind
