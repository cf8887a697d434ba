// Native small-message collectives for SyncBN inside the C++ block executor.
//
// The reference's SyncBN (main_supcon.py:222-224 -> torch.nn.SyncBatchNorm) issues one
// all-gather per BN in forward and one all-reduce in backward, each a Python-level c10d
// call (≈106 per ResNet-50 step, all on the critical path). Here a "small communicator"
// is a handle the executor (conv_bn_ops.cpp block_fwd / block_bwd) calls directly on the
// compute stream, with no Python or c10d work queue in between:
//
//   kind RCCL  — a dedicated RCCL communicator (ncclCommInitRank from a unique id the
//                Python side broadcasts once through torch.distributed); ncclAllReduce
//                in place on the current stream. Separate from torch's communicators, so
//                the gradient buckets (their own process group / stream) never queue in
//                front of a SyncBN statistic.
//   kind XGMI  — a one-shot IPC arena of xgmi_ops.cpp (direct peer stores + epoch flags).
//   kind EMU   — W virtual ranks holding identical data in ONE process (tests): the sum is
//                x·W, so every SyncBN code path of the executor runs on a single GPU and
//                must reproduce the single-process result (statistics exactly, dγ/dβ ×W).
//
// The process links torch's own librccl.so (csrc/build.py puts torch/lib first), so there
// is exactly one RCCL runtime in the process.
#include "ops_decl.h"

#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace sdx_bind {

// xgmi_ops.cpp
torch::Tensor xgmi_allreduce_ext(int64_t id, torch::Tensor x);
int64_t xgmi_world(int64_t id);

namespace {

enum Kind { KIND_RCCL = 1, KIND_XGMI = 2, KIND_EMU = 3 };

struct SmallComm {
  Kind kind;
  ncclComm_t nccl = nullptr;
  int64_t xgmi_id = -1;
  int world = 1, rank = 0, device = 0;
};

std::mutex g_mu;
std::vector<std::unique_ptr<SmallComm>> g_comms;   // handle = index + 1 (0 = none)

void check_nccl(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, what, " failed: ", ncclGetErrorString(r));
}

SmallComm& get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 1 && h <= (int64_t)g_comms.size() && g_comms[h - 1], "bad small-communicator handle ", h);
  return *g_comms[h - 1];
}

int64_t add(std::unique_ptr<SmallComm> c) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(std::move(c));
  return (int64_t)g_comms.size();
}

torch::Tensor rccl_unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  auto t = torch::empty({(int64_t)sizeof(id)}, torch::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr<uint8_t>(), &id, sizeof(id));
  return t;
}

int64_t rccl_comm_init(torch::Tensor id_bytes, int64_t world, int64_t rank) {
  TORCH_CHECK(!id_bytes.is_cuda() && id_bytes.scalar_type() == at::kByte &&
                  id_bytes.numel() == (int64_t)sizeof(ncclUniqueId),
              "id: CPU uint8 [", sizeof(ncclUniqueId), "]");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rank/world");
  ncclUniqueId id;
  auto ic = id_bytes.contiguous();
  std::memcpy(&id, ic.data_ptr<uint8_t>(), sizeof(id));
  auto c = std::make_unique<SmallComm>();
  c->kind = KIND_RCCL;
  c->world = (int)world;
  c->rank = (int)rank;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  check_nccl(ncclCommInitRank(&c->nccl, (int)world, id, (int)rank), "ncclCommInitRank");
  return add(std::move(c));
}

int64_t xgmi_small_comm(int64_t xgmi_id, int64_t rank) {
  auto c = std::make_unique<SmallComm>();
  c->kind = KIND_XGMI;
  c->xgmi_id = xgmi_id;
  c->world = (int)xgmi_world(xgmi_id);
  c->rank = (int)rank;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  return add(std::move(c));
}

int64_t emu_small_comm(int64_t world) {
  TORCH_CHECK(world >= 1, "world >= 1");
  auto c = std::make_unique<SmallComm>();
  c->kind = KIND_EMU;
  c->world = (int)world;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  return add(std::move(c));
}

void small_comm_destroy(int64_t h) {
  std::unique_ptr<SmallComm> c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(h >= 1 && h <= (int64_t)g_comms.size() && g_comms[h - 1], "bad small-communicator handle ", h);
    c = std::move(g_comms[h - 1]);
  }
  if (c->kind == KIND_RCCL && c->nccl) {
    (void)hipDeviceSynchronize();
    (void)ncclCommDestroy(c->nccl);
  }
}

void small_all_reduce_py(int64_t h, torch::Tensor x) { small_all_reduce_(h, x); }

}  // namespace

int small_comm_world(int64_t h) { return h == 0 ? 1 : get(h).world; }

// in-place SUM over the communicator's ranks, ordered on the current stream
void small_all_reduce_(int64_t h, torch::Tensor& x) {
  if (h == 0) return;
  SmallComm& c = get(h);
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "small all-reduce: contiguous GPU tensor");
  TORCH_CHECK(x.device().index() == c.device, "small all-reduce: tensor on device ", x.device().index(),
              ", communicator on ", c.device);
  if (c.world == 1) return;
  if (c.kind == KIND_RCCL) {
    ncclDataType_t dt;
    switch (x.scalar_type()) {
      case at::kDouble: dt = ncclFloat64; break;
      case at::kFloat: dt = ncclFloat32; break;
      case at::kInt: dt = ncclInt32; break;
      default: TORCH_CHECK(false, "small all-reduce: fp64 / fp32 / int32 only");
    }
    check_nccl(ncclAllReduce(x.data_ptr(), x.data_ptr(), (size_t)x.numel(), dt, ncclSum, c.nccl, cur_stream()),
               "ncclAllReduce");
  } else if (c.kind == KIND_EMU) {
    x.mul_((double)c.world);
  } else {
    TORCH_CHECK(x.scalar_type() == at::kDouble, "xGMI small all-reduce: fp64 only");
    auto r = xgmi_allreduce_ext(c.xgmi_id, x);
    x.copy_(r);
  }
}

void register_comm(pybind11::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId as CPU uint8 bytes (rank 0; broadcast it)");
  m.def("rccl_comm_init", &rccl_comm_init, "dedicated RCCL communicator for SyncBN statistics -> handle",
        pybind11::arg("id"), pybind11::arg("world"), pybind11::arg("rank"));
  m.def("xgmi_small_comm", &xgmi_small_comm, "wrap a one-shot xGMI arena as a small-communicator handle");
  m.def("emu_small_comm", &emu_small_comm, "W identical virtual ranks in one process (tests): sum = x*W");
  m.def("small_comm_destroy", &small_comm_destroy);
  m.def("small_comm_world", &small_comm_world);
  m.def("small_all_reduce_", &small_all_reduce_py, "in-place SUM on the current stream");
}

}  // namespace sdx_bind
