// Bindings for the one-shot xGMI all-reduce (xgmi.hip): IPC arena lifetime, handle
// exchange (the Python side moves the 64-byte handles over the process group), calls, and
// the single-GPU W-rank emulation used by the tests.
#include "ops_decl.h"
#include "launchers.h"
#include "conv_internal.h"

#include <algorithm>
#include <memory>
#include <mutex>
#include <vector>

namespace sdx_bind {
namespace {

struct Arena {
  bool emulated = false;           // W virtual ranks' arenas in this device's memory (tests)
  bool solo = false;               // emulated: one rank's share only (XgmiCol::solo)
  int device = 0;
  int rank = 0;
  int world = 1;
  size_t cap = 0;
  void* base = nullptr;            // own arena: data then flags
  std::vector<void*> opened;       // peer arenas mapped through IPC
  XgmiPeers peers{};
  unsigned epoch = 0;
  unsigned* epoch_dev = nullptr;   // device [epoch, ticket] per (virtual) rank (XgmiCol::epoch_ctr)
  int* err = nullptr;              // host-pinned, GPU-written error word (sender index + 1)
  long long timeout_ticks = 0;     // flag-poll deadline in 100 MHz wall-clock ticks
  double ticks_per_s = 1e8;        // wall-clock rate
  // Stream-order invariant of the device epoch (bn.hip XgmiCol::epoch_ctr): a launch reads
  // ctr + 1 at its start and stores it back at its end, so two launches on one arena must
  // never overlap -- they would read the same epoch / flag parity and could pass on each
  // other's flags. Every call is issued on the stream of the previous one, or (order_on) the
  // new stream first waits for the previous stream's work.
  hipStream_t last_stream = nullptr;
  hipEvent_t order_ev = nullptr;
};

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// serialise arena use across streams (see Arena::last_stream). Inside a stream capture the
// capturing code orders its streams itself (torch.cuda.graph warm-up / capture streams
// wait on the previous stream), and an event node must not leak into the graph, so no event
// is recorded or waited then. Streams come from torch's pool, which never destroys them.
void order_on(Arena& a, hipStream_t s) {
  if (a.last_stream == s) return;
  if (a.last_stream != nullptr && !capturing(s) && !capturing(a.last_stream)) {
    if (a.order_ev == nullptr)
      check_hip(hipEventCreateWithFlags(&a.order_ev, hipEventDisableTiming), "hipEventCreate(arena order)");
    check_hip(hipEventRecord(a.order_ev, a.last_stream), "hipEventRecord(arena order)");
    check_hip(hipStreamWaitEvent(s, a.order_ev, 0), "hipStreamWaitEvent(arena order)");
  }
  a.last_stream = s;
}

// a per-call deadline (start-up self-checks: seconds, not --comm_timeout) capped by the arena's
long long call_ticks(const Arena& a, double timeout_s) {
  if (!(timeout_s > 0)) return a.timeout_ticks;
  return std::min(a.timeout_ticks, std::max(1LL, (long long)(timeout_s * a.ticks_per_s)));
}

std::mutex g_mu;
std::vector<std::unique_ptr<Arena>> g_arenas;

size_t arena_bytes(int world, size_t cap) {
  const size_t data = 2ull * world * cap * sizeof(double);
  // flags [2][W][kXgmiFlagGroups] u32 after the data (≤ 4 KiB), 256-B aligned block
  const size_t flags = 2ull * world * kXgmiFlagGroups * sizeof(unsigned);
  return data + (flags + 255) / 256 * 256;
}

Arena& get(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(id >= 0 && id < (int64_t)g_arenas.size() && g_arenas[id], "bad xgmi arena id");
  return *g_arenas[id];
}

void set_ptrs(XgmiPeers& p, int q, void* base, int world, size_t cap) {
  p.data[q] = static_cast<double*>(base);
  p.flags[q] = reinterpret_cast<unsigned*>(static_cast<char*>(base) + 2ull * world * cap * sizeof(double));
}

int64_t xgmi_create(int64_t rank, int64_t world, int64_t cap, double timeout_s) {
  TORCH_CHECK(world >= 1 && world <= kXgmiMaxPeers && rank >= 0 && rank < world, "1 <= world <= 8");
  TORCH_CHECK(cap > 0 && cap <= (1 << 20), "cap in (0, 2^20]");
  TORCH_CHECK(timeout_s > 0 && timeout_s < 86400, "timeout_s in (0, 1 day)");
  auto a = std::make_unique<Arena>();
  check_hip(hipGetDevice(&a->device), "hipGetDevice");
  a->rank = (int)rank;
  a->world = (int)world;
  a->cap = (size_t)cap;
  const size_t bytes = arena_bytes(a->world, a->cap);
  // uncached: peers' remote stores must be seen by this GPU's loads without cache maintenance
  check_hip(hipExtMallocWithFlags(&a->base, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  check_hip(hipMemset(a->base, 0, bytes), "hipMemset");
  check_hip(hipMalloc(reinterpret_cast<void**>(&a->epoch_dev), 2 * sizeof(unsigned)), "hipMalloc(epochs)");
  check_hip(hipMemset(a->epoch_dev, 0, 2 * sizeof(unsigned)), "hipMemset(epochs)");
  a->peers.cap = a->cap;
  set_ptrs(a->peers, a->rank, a->base, a->world, a->cap);
  // error word in coherent host memory: the kernel stores it (system scope) and the host
  // watchdog (comm_ops.cpp) polls it with plain loads — no device copy on any stream
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&a->err), sizeof(int), hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(err)");
  *reinterpret_cast<volatile int*>(a->err) = 0;
  int rate_khz = 0;
  check_hip(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, a->device), "wall clock rate");
  a->ticks_per_s = 1000.0 * (rate_khz > 0 ? rate_khz : 100000);
  a->timeout_ticks = (long long)(timeout_s * a->ticks_per_s);
  std::lock_guard<std::mutex> lk(g_mu);
  g_arenas.push_back(std::move(a));
  return (int64_t)g_arenas.size() - 1;
}

torch::Tensor xgmi_handle(int64_t id) {
  Arena& a = get(id);
  hipIpcMemHandle_t h;
  check_hip(hipIpcGetMemHandle(&h, a.base), "hipIpcGetMemHandle");
  auto t = torch::empty({HIP_IPC_HANDLE_SIZE}, torch::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr<uint8_t>(), &h, HIP_IPC_HANDLE_SIZE);
  return t;
}

void xgmi_open(int64_t id, torch::Tensor handles) {
  Arena& a = get(id);
  TORCH_CHECK(handles.dtype() == at::kByte && handles.dim() == 2 && handles.size(0) == a.world &&
                  handles.size(1) == HIP_IPC_HANDLE_SIZE && !handles.is_cuda(),
              "handles: CPU uint8 [world, 64]");
  auto hc = handles.contiguous();
  for (int q = 0; q < a.world; ++q) {
    if (q == a.rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, hc.data_ptr<uint8_t>() + (size_t)q * HIP_IPC_HANDLE_SIZE, HIP_IPC_HANDLE_SIZE);
    void* p = nullptr;
    check_hip(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    a.opened.push_back(p);
    set_ptrs(a.peers, q, p, a.world, a.cap);
  }
}

torch::Tensor xgmi_allreduce(int64_t id, torch::Tensor x, double timeout_s) {
  Arena& a = get(id);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kDouble && x.is_contiguous(), "x: contiguous fp64 GPU tensor");
  TORCH_CHECK((size_t)x.numel() <= a.cap, "message larger than the arena slot");
  c10::DeviceGuard dg(x.device());
  auto out = torch::empty_like(x);
  order_on(a, cur_stream());
  a.epoch += 1;
  check_hip(launch_xgmi_allreduce(x.data_ptr<double>(), out.data_ptr<double>(), (int)x.numel(), a.peers, a.rank,
                                  a.world, a.epoch, a.err, call_ticks(a, timeout_s), cur_stream(), a.epoch_dev),
            "xgmi_allreduce");
  return out;
}

int64_t xgmi_error(int64_t id) {
  Arena& a = get(id);
  return *reinterpret_cast<volatile int*>(a.err);
}

void xgmi_destroy(int64_t id) {
  std::unique_ptr<Arena> a;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    TORCH_CHECK(id >= 0 && id < (int64_t)g_arenas.size() && g_arenas[id], "bad xgmi arena id");
    a = std::move(g_arenas[id]);
  }
  (void)hipDeviceSynchronize();
  for (void* p : a->opened) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(a->base);
  (void)hipFree(a->epoch_dev);
  (void)hipHostFree(a->err);
  if (a->order_ev != nullptr) (void)hipEventDestroy(a->order_ev);
}

// W virtual ranks on this device (single-GPU emulation of the fused SyncBN exchange, the
// XEMU small-communicator kind): W arenas in one ordinary device allocation (agent scope),
// error word host-pinned like a real arena's so the watchdog reads it the same way
int64_t xgmi_emu_create(int64_t world, int64_t cap, double timeout_s) {
  TORCH_CHECK(world >= 1 && world <= kXgmiMaxPeers, "1 <= world <= 8");
  TORCH_CHECK(cap > 0 && cap <= (1 << 20), "cap in (0, 2^20]");
  auto a = std::make_unique<Arena>();
  a->emulated = true;
  {
    const char* e = getenv("SDX_SYNCBN_EMU_SOLO");
    a->solo = e != nullptr && atoi(e) != 0;
    // a timing diagnostic only (tools/syncbn_latency.py): the W-1 other slots are summed
    // although no rank wrote them, so BN statistics of a training run are wrong under it
    if (a->solo)
      fprintf(stderr, "warning: SDX_SYNCBN_EMU_SOLO=1: emulated SyncBN runs one rank's share only "
                      "(timing diagnostic; the BN statistics are NOT valid)\n");
  }
  check_hip(hipGetDevice(&a->device), "hipGetDevice");
  a->world = (int)world;
  a->cap = (size_t)cap;
  const size_t one = arena_bytes(a->world, a->cap);
  check_hip(hipMalloc(&a->base, one * world), "hipMalloc(emulated arenas)");
  check_hip(hipMemset(a->base, 0, one * world), "hipMemset");
  check_hip(hipMalloc(reinterpret_cast<void**>(&a->epoch_dev), (size_t)world * 2 * sizeof(unsigned)),
            "hipMalloc(epochs)");
  check_hip(hipMemset(a->epoch_dev, 0, (size_t)world * 2 * sizeof(unsigned)), "hipMemset(epochs)");
  a->peers.cap = a->cap;
  for (int q = 0; q < a->world; ++q) set_ptrs(a->peers, q, static_cast<char*>(a->base) + one * q, a->world, a->cap);
  check_hip(hipHostMalloc(reinterpret_cast<void**>(&a->err), sizeof(int), hipHostMallocCoherent | hipHostMallocMapped),
            "hipHostMalloc(err)");
  *reinterpret_cast<volatile int*>(a->err) = 0;
  int rate_khz = 0;
  check_hip(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, a->device), "wall clock rate");
  a->ticks_per_s = 1000.0 * (rate_khz > 0 ? rate_khz : 100000);
  a->timeout_ticks = (long long)(timeout_s * a->ticks_per_s);
  std::lock_guard<std::mutex> lk(g_mu);
  g_arenas.push_back(std::move(a));
  return (int64_t)g_arenas.size() - 1;
}

// W virtual ranks on this GPU: `in` [W, n] fp64; runs `iters` calls (epochs 1..iters, so both
// parities and arena reuse are exercised) and returns the last result [W, n].
torch::Tensor xgmi_emulate(torch::Tensor in, int64_t iters) {
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kDouble && in.dim() == 2 && in.is_contiguous(),
              "in: [W, n] fp64 GPU");
  const int world = (int)in.size(0);
  const int n = (int)in.size(1);
  TORCH_CHECK(world >= 1 && world <= kXgmiMaxPeers && iters >= 1, "1 <= W <= 8");
  c10::DeviceGuard dg(in.device());
  const size_t cap = (size_t)std::max(n, 1);
  auto opts = in.options().dtype(at::kByte);
  std::vector<torch::Tensor> arenas;
  XgmiPeers peers{};
  peers.cap = cap;
  for (int q = 0; q < world; ++q) {
    arenas.push_back(torch::zeros({(int64_t)arena_bytes(world, cap)}, opts));
    set_ptrs(peers, q, arenas.back().data_ptr(), world, cap);
  }
  auto out = torch::empty_like(in);
  auto err = torch::zeros({1}, in.options().dtype(at::kInt));
  for (int64_t e = 1; e <= iters; ++e)
    check_hip(launch_xgmi_emulate(in.data_ptr<double>(), out.data_ptr<double>(), n, peers, world, (unsigned)e,
                                  err.data_ptr<int>(), cur_stream()),
              "xgmi_emulate");
  const int ev = err.cpu().item<int>();
  TORCH_CHECK(ev == 0, "xgmi emulation: flag wait timed out (sender ", ev - 1, ")");
  return out;
}

}  // namespace

// for comm_ops.cpp / conv_bn_ops.cpp: arguments of one fused SyncBN exchange on arena id
// (epoch advanced; mode 1 real peers, 2 emulated ranks)
XgmiCol xgmi_col_args(int64_t id) {
  Arena& a = get(id);
  order_on(a, cur_stream());
  XgmiCol x{};
  x.peers = a.peers;
  x.mode = a.emulated ? 2 : 1;
  x.me = a.rank;
  x.world = a.world;
  x.epoch = ++a.epoch;
  // real peers: this rank's counter row; emulated: one row per virtual rank (z)
  x.epoch_ctr = a.epoch_dev;
  x.err = a.err;
  x.timeout_ticks = a.timeout_ticks;
  x.slab_zstride = 0;
  x.solo = a.solo ? 1 : 0;
  return x;
}
bool xgmi_emulated(int64_t id) { return get(id).emulated; }

// The fused SyncBN exchange (bn.hip col_reduce + XgmiCol) of a statistics slab directly on
// an arena, with a per-call deadline: the start-up self-check runs it BEFORE the arena is
// wrapped as a small communicator, so a peer that never answers makes the check fail (and
// every rank fall back to RCCL) instead of tripping the communicator watchdog.
// slab [rows][nsets][C] fp32 -> global sums [nsets][C] (fp64).
torch::Tensor xgmi_exchange_sums(int64_t id, torch::Tensor slab, double timeout_s) {
  TORCH_CHECK(slab.is_cuda() && slab.scalar_type() == at::kFloat && slab.is_contiguous() && slab.dim() == 3,
              "slab: contiguous fp32 [rows][nsets][C]");
  const int64_t rows = slab.size(0), nsets = slab.size(1), C = slab.size(2);
  TORCH_CHECK(rows >= 1 && nsets >= 1 && nsets <= 3 && C >= 1 && C <= 4096, "slab shape");
  XgmiCol x = xgmi_col_args(id);
  x.timeout_ticks = call_ticks(get(id), timeout_s);
  c10::DeviceGuard dg(slab.device());
  const int z = x.mode == 2 && !x.solo ? x.world : 1;
  auto sums = torch::empty({nsets, C}, slab.options().dtype(at::kDouble));
  auto scratch = reduce_scratch(slab, rows, nsets, C, z);
  check_hip(launch_col_reduce(slab.data_ptr<float>(), (int)rows, (int)nsets, (int)C, scratch.data_ptr<double>(),
                              reduce_counters(slab.device(), z), sums.data_ptr<double>(), 0, nullptr, nullptr,
                              cur_stream(), &x),
            "xgmi_exchange_sums");
  return sums;
}
int64_t xgmi_emu_create_ext(int64_t world, int64_t cap, double timeout_s) { return xgmi_emu_create(world, cap, timeout_s); }

// for comm_ops.cpp (small-communicator wrapper of an arena)
torch::Tensor xgmi_allreduce_ext(int64_t id, torch::Tensor x) { return xgmi_allreduce(id, x, -1.0); }
int64_t xgmi_world(int64_t id) { return get(id).world; }
int64_t xgmi_error_ext(int64_t id) { return xgmi_error(id); }
// watchdog sweep: never throws; 0 once the arena is gone (the read happens under the
// registry lock, and xgmi_destroy unlinks an arena under that lock before freeing it)
int64_t xgmi_error_nothrow(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (id < 0 || id >= (int64_t)g_arenas.size() || !g_arenas[id]) return 0;
  return *reinterpret_cast<volatile int*>(g_arenas[id]->err);
}
std::vector<int64_t> xgmi_debug(int64_t id) {
  Arena& a = get(id);
  return {(int64_t)(uintptr_t)a.err, (int64_t)*reinterpret_cast<volatile int*>(a.err), (int64_t)a.world};
}

void register_xgmi(pybind11::module& m) {
  m.def("xgmi_create", &xgmi_create, "allocate this rank's IPC receive arena (uncached device memory)",
        pybind11::arg("rank"), pybind11::arg("world"), pybind11::arg("cap"), pybind11::arg("timeout_s") = 600.0);
  m.def("xgmi_handle", &xgmi_handle, "64-byte IPC handle of this rank's arena");
  m.def("xgmi_open", &xgmi_open, "map every peer's arena from their IPC handles [W, 64]");
  m.def("xgmi_allreduce", &xgmi_allreduce, "one-shot fp64 all-reduce (sum) of a small tensor",
        pybind11::arg("id"), pybind11::arg("x"), pybind11::arg("timeout_s") = -1.0);
  m.def("xgmi_exchange_sums", &xgmi_exchange_sums,
        "fused SyncBN exchange of a [rows][nsets][C] statistics slab on an arena (per-call deadline)",
        pybind11::arg("id"), pybind11::arg("slab"), pybind11::arg("timeout_s") = -1.0);
  m.def("xgmi_error", &xgmi_error, "nonzero: a peer's flag never arrived (1 + sender)");
  m.def("xgmi_destroy", &xgmi_destroy);
  m.def("xgmi_debug", &xgmi_debug);
  m.def("xgmi_emulate", &xgmi_emulate, "single-GPU W-rank emulation of the one-shot protocol");
  m.def("xgmi_emu_create", &xgmi_emu_create, "W emulated ranks' arenas on this device (fused SyncBN exchange tests)",
        pybind11::arg("world"), pybind11::arg("cap") = 12288, pybind11::arg("timeout_s") = 10.0);
}

}  // namespace sdx_bind
