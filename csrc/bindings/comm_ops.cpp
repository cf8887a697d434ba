// Native small-message collectives for SyncBN inside the C++ block executor.
//
// The reference's SyncBN (main_supcon.py:222-224 -> torch.nn.SyncBatchNorm) issues one
// all-gather per BN in forward and one all-reduce in backward, each a Python-level c10d
// call (≈106 per ResNet-50 step, all on the critical path). Here a "small communicator"
// is a handle the executor (conv_bn_ops.cpp block_fwd / block_bwd) calls directly on the
// compute stream, with no Python or c10d work queue in between:
//
//   kind RCCL  — a dedicated RCCL communicator (ncclCommInitRankConfig from a unique id
//                the Python side broadcasts once through torch.distributed); ncclAllReduce
//                in place on the current stream.
//   kind XGMI  — a one-shot IPC arena of xgmi_ops.cpp (direct peer stores + epoch flags).
//   kind EMU   — W virtual ranks holding identical data in ONE process (tests): the sum is
//                x·W, so every SyncBN code path of the executor runs on a single GPU and
//                must reproduce the single-process result.
//   kind XEMU  — EMU semantics, but the executor's BN statistics take the FUSED xGMI path
//                (bn.hip col_reduce + exchange): W virtual ranks are W z-slices of each
//                launch exchanging through W arenas in device memory (xgmi_emu_create).
//
// Fused SyncBN exchange (kinds XGMI / XEMU): small_comm_fused() hands the executor the
// arena arguments of one exchange; the column reduction of the BN statistics then stores,
// exchanges and sums them and runs the finalize / coefficient epilogue in the same launch
// (one launch per BN instead of reduce + collective + finalize).
//
// Failure handling. The RCCL communicator is created NON-blocking
// (config.blocking = 0): initialisation is polled against a deadline and aborted on
// expiry, so a peer that never joins raises here instead of hanging. Every communicator
// of >1 rank is watched by ONE host watchdog thread: after a collective is enqueued the
// issuing thread moves a HIP event behind it (throttled: see arm()); if that event has
// not completed one --comm_timeout after it was recorded, or an xGMI arena's host-pinned
// error word is set (a peer's flag missed
// the kernel's deadline), the watchdog aborts the RCCL communicator (so its kernels
// return) and ends the process with status 3 — the same status as a c10d collective
// failure (utils/faults.py). A stalled peer therefore never hangs a rank forever and never
// lets it continue on stale BN statistics.
//
// Ordering against the gradient buckets. The bucket all-reduces run on torch's own
// communicator (c10d, its internal stream); the SyncBN statistics on this one, on the
// compute stream. Each communicator's operations are issued by the main thread in the
// same program order on every rank (the backward, and so the bucket hooks, are
// deterministic), and each lives on a single stream, so each sees one consistent sequence
// on all ranks. HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues in creation order,
// identically on every rank, so wherever two streams share a queue their packets
// interleave in the same host issue order everywhere; an RCCL kernel occupies a few CUs,
// so two communicators' kernels are always co-resident. No rank can therefore wait on a
// collective that its peer has queued behind a collective the first rank has not reached.
//
// The process links torch's own librccl.so (csrc/build.py puts torch/lib first), so there
// is exactly one RCCL runtime in the process.
#include "ops_decl.h"
#include "launchers.h"

#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace sdx_bind {

// xgmi_ops.cpp
torch::Tensor xgmi_allreduce_ext(int64_t id, torch::Tensor x);
int64_t xgmi_world(int64_t id);
int64_t xgmi_error_ext(int64_t id);
int64_t xgmi_error_nothrow(int64_t id);
int64_t xgmi_emu_create_ext(int64_t world, int64_t cap, double timeout_s);
XgmiCol xgmi_col_args(int64_t id);

namespace {

using Clock = std::chrono::steady_clock;
constexpr int kCommFailureExit = 3;   // utils/faults.py COLLECTIVE_FAILURE_EXIT_CODE

enum Kind { KIND_RCCL = 1, KIND_XGMI = 2, KIND_EMU = 3, KIND_XEMU = 4 };

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

struct SmallComm {
  Kind kind;
  ncclComm_t nccl = nullptr;
  int64_t xgmi_id = -1;
  int world = 1, rank = 0, device = 0;
  double timeout_s = 600.0;
  // watchdog state: one armed event at a time (armed by the issuing thread, cleared by
  // the watchdog once complete)
  hipEvent_t ev = nullptr;
  std::atomic<bool> armed{false};
  std::atomic<int64_t> armed_at{0};   // steady-clock ns of the armed record
  std::atomic<long> ops{0};
};

// handle = index + 1 (0 = none). Heap-allocated and never destroyed: the detached
// watchdog thread may still sweep it while static destructors run at process exit.
struct Registry {
  std::mutex mu;
  std::vector<std::shared_ptr<SmallComm>> comms;
};
Registry& reg() {
  static Registry* r = new Registry;
  return *r;
}

void check_nccl(ncclResult_t r, const char* what) {
  TORCH_CHECK(r == ncclSuccess, what, " failed: ", ncclGetErrorString(r));
}

std::shared_ptr<SmallComm> get(int64_t h) {
  Registry& R = reg();
  std::lock_guard<std::mutex> lk(R.mu);
  TORCH_CHECK(h >= 1 && h <= (int64_t)R.comms.size() && R.comms[h - 1], "bad small-communicator handle ", h);
  return R.comms[h - 1];
}

// ---- watchdog ----------------------------------------------------------------------
[[noreturn]] void fail_exit(SmallComm& c, const char* why) {
  std::fprintf(stderr,
               "rank %d: collective failure on the native SyncBN communicator (%s): %s; "
               "aborting the process with status %d\n",
               c.rank, c.kind == KIND_RCCL ? "RCCL" : c.kind == KIND_XGMI ? "xGMI" : "emulated", why,
               kCommFailureExit);
  std::fflush(stderr);
  if (c.kind == KIND_RCCL && c.nccl) (void)ncclCommAbort(c.nccl);   // lets its kernels return
  std::_Exit(kCommFailureExit);
}

std::atomic<bool> g_stop{false};
std::thread* g_thread = nullptr;   // leaked on purpose (joined by the atexit hook)

void sweep() {
  Registry& R = reg();
  std::lock_guard<std::mutex> lk(R.mu);
  for (auto& c : R.comms) {
    if (!c || c->world <= 1) continue;
    if (c->kind == KIND_XGMI || c->kind == KIND_XEMU) {
      const int64_t e = xgmi_error_nothrow(c->xgmi_id);
      if (e != 0) {
        char buf[200];
        std::snprintf(buf, sizeof(buf), "flag of peer rank %d missed the %.0f s deadline (arena %lld)", (int)e - 1,
                      c->timeout_s, (long long)c->xgmi_id);
        fail_exit(*c, buf);
      }
    }
    if (c->kind == KIND_RCCL && c->nccl) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        fail_exit(*c, ncclGetErrorString(ae));
    }
    if (!c->armed.load(std::memory_order_acquire)) continue;
    const hipError_t q = hipEventQuery(c->ev);
    if (q == hipSuccess) {
      continue;
    } else if (q == hipErrorCapturedEvent) {
      // the event was last recorded inside a stream capture (arm() skips capturing streams,
      // so only a record from before that rule could do this): it keeps refusing queries,
      // so its deadline could never fire -- disarm; the next eager collective re-arms it
      c->armed.store(false, std::memory_order_release);
      continue;
    } else if (q >= hipErrorStreamCaptureUnsupported && q <= hipErrorStreamCaptureWrongThread) {
      // a global-mode capture in progress refuses the query: no verdict this sweep (the
      // deadline keeps running from the armed record)
      continue;
    } else if (q == hipErrorNotReady) {
      const double waited = 1e-9 * (double)(now_ns() - c->armed_at.load());
      if (waited > c->timeout_s) {
        char buf[160];
        std::snprintf(buf, sizeof(buf), "a collective did not complete within %.1f s (a peer died or stalled)",
                      c->timeout_s);
        fail_exit(*c, buf);
      }
    } else {
      fail_exit(*c, hipGetErrorString(q));
    }
  }
}

// the whole sweep holds the registry lock, so small_comm_destroy / abort never tear down
// a communicator under it
void watchdog_loop() {
  while (!g_stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (g_stop.load()) break;
    // (an exception must never leave this detached thread: std::terminate would take
    // the process down without the diagnostic)
    try {
      sweep();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "native communicator watchdog: sweep error ignored: %s\n", e.what());
    } catch (...) {
      std::fprintf(stderr, "native communicator watchdog: sweep error ignored\n");
    }
  }
}

// Stop the sweep before process teardown: the HIP runtime frees host-pinned memory (the
// xGMI error words) and its events in its own exit hooks, which were registered before
// this one and so run after it.
void stop_watchdog() {
  g_stop.store(true);
  if (g_thread && g_thread->joinable()) g_thread->join();
}

void ensure_watchdog() {
  static std::once_flag once;
  std::call_once(once, [] {
    g_thread = new std::thread(watchdog_loop);
    std::atexit(stop_watchdog);
  });
}

// after a collective was enqueued on `s`: move the communicator's watch event behind it
// (re-recording a pending event is legal) and stamp the issue time, at most once per
// 200 µs (≈30 records per ResNet-50 step instead of 106). A collective that never
// completes keeps every later record pending, so the last record before the host blocks
// times out. A hang inside the last < 200 µs of collectives before the host blocks is
// caught by the next collective issued, or else by the c10d watchdog: torch's own
// collectives (gradient buckets, loss gather, metrics) queue behind it and time out.
// The stamp is stored BEFORE the record, so the watchdog never pairs a fresh pending
// record with an old stamp.
void arm(SmallComm& c, hipStream_t s) {
  c.ops.fetch_add(1, std::memory_order_relaxed);
  if (c.world <= 1) return;
  // a collective captured into a hipGraph: an event recorded here would become a graph node
  // and, queried later, refuse with hipErrorCapturedEvent; replays are watched by the next
  // eager collective's record (or the c10d watchdog)
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;
  const int64_t t = now_ns();
  if (c.armed.load(std::memory_order_acquire) && t - c.armed_at.load() < 200000) return;
  c.armed_at.store(t);
  check_hip(hipEventRecord(c.ev, s), "hipEventRecord(watchdog)");
  c.armed.store(true, std::memory_order_release);
}

int64_t add(std::shared_ptr<SmallComm> c) {
  check_hip(hipEventCreateWithFlags(&c->ev, hipEventDisableTiming), "hipEventCreate(watchdog)");
  if (c->world > 1) ensure_watchdog();
  Registry& R = reg();
  std::lock_guard<std::mutex> lk(R.mu);
  R.comms.push_back(std::move(c));
  return (int64_t)R.comms.size();
}

// SDX_SYNCBN_FUSED=0: the xGMI kinds fall back to reduce -> one-shot all-reduce -> finalize
bool fused_disabled() {
  static const bool off = [] {
    const char* e = getenv("SDX_SYNCBN_FUSED");
    return e != nullptr && atoi(e) == 0;
  }();
  return off;
}

// abort + clear the RCCL communicator under the registry lock: the watchdog sweep reads
// c.nccl under that lock, so it never queries a communicator mid-abort
void abort_locked(SmallComm& c) {
  std::lock_guard<std::mutex> lk(reg().mu);
  if (c.nccl) (void)ncclCommAbort(c.nccl);
  c.nccl = nullptr;
}

// poll a non-blocking communicator until its pending operation settles (deadline)
void settle(SmallComm& c, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return;
  TORCH_CHECK(r == ncclInProgress, what, " failed: ", ncclGetErrorString(r));
  const auto t0 = Clock::now();
  while (true) {
    ncclResult_t ae = ncclInProgress;
    check_nccl(ncclCommGetAsyncError(c.nccl, &ae), "ncclCommGetAsyncError");
    if (ae == ncclSuccess) return;
    if (ae != ncclInProgress) {
      abort_locked(c);
      TORCH_CHECK(false, what, " failed: ", ncclGetErrorString(ae));
    }
    if (std::chrono::duration<double>(Clock::now() - t0).count() > c.timeout_s) {
      abort_locked(c);
      TORCH_CHECK(false, what, " timed out after ", c.timeout_s, " s (a peer rank did not join or stalled)");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

torch::Tensor rccl_unique_id() {
  ncclUniqueId id;
  check_nccl(ncclGetUniqueId(&id), "ncclGetUniqueId");
  auto t = torch::empty({(int64_t)sizeof(id)}, torch::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr<uint8_t>(), &id, sizeof(id));
  return t;
}

int64_t rccl_comm_init(torch::Tensor id_bytes, int64_t world, int64_t rank, double timeout_s) {
  TORCH_CHECK(!id_bytes.is_cuda() && id_bytes.scalar_type() == at::kByte &&
                  id_bytes.numel() == (int64_t)sizeof(ncclUniqueId),
              "id: CPU uint8 [", sizeof(ncclUniqueId), "]");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rank/world");
  TORCH_CHECK(timeout_s > 0, "timeout_s > 0");
  ncclUniqueId id;
  auto ic = id_bytes.contiguous();
  std::memcpy(&id, ic.data_ptr<uint8_t>(), sizeof(id));
  auto c = std::make_shared<SmallComm>();
  c->kind = KIND_RCCL;
  c->world = (int)world;
  c->rank = (int)rank;
  c->timeout_s = timeout_s;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  const ncclResult_t r = ncclCommInitRankConfig(&c->nccl, (int)world, id, (int)rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (c->nccl) (void)ncclCommAbort(c->nccl);
    TORCH_CHECK(false, "ncclCommInitRankConfig failed: ", ncclGetErrorString(r));
  }
  settle(*c, r, "ncclCommInitRankConfig");
  return add(std::move(c));
}

int64_t xgmi_small_comm(int64_t xgmi_id, int64_t rank, double timeout_s) {
  auto c = std::make_shared<SmallComm>();
  c->kind = KIND_XGMI;
  c->xgmi_id = xgmi_id;
  c->world = (int)xgmi_world(xgmi_id);
  c->rank = (int)rank;
  c->timeout_s = timeout_s;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  return add(std::move(c));
}

int64_t xgmi_emu_small_comm(int64_t world, double timeout_s) {
  TORCH_CHECK(world >= 1 && world <= kXgmiMaxPeers, "1 <= world <= 8");
  auto c = std::make_shared<SmallComm>();
  c->kind = KIND_XEMU;
  c->world = (int)world;
  c->timeout_s = timeout_s;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  c->xgmi_id = xgmi_emu_create_ext(world, 12288, timeout_s);
  return add(std::move(c));
}

int64_t emu_small_comm(int64_t world, double timeout_s) {
  TORCH_CHECK(world >= 1, "world >= 1");
  auto c = std::make_shared<SmallComm>();
  c->kind = KIND_EMU;
  c->world = (int)world;
  c->timeout_s = timeout_s;
  check_hip(hipGetDevice(&c->device), "hipGetDevice");
  return add(std::move(c));
}

void small_comm_destroy(int64_t h) {
  std::shared_ptr<SmallComm> c;
  {
    Registry& R = reg();
    std::lock_guard<std::mutex> lk(R.mu);
    TORCH_CHECK(h >= 1 && h <= (int64_t)R.comms.size() && R.comms[h - 1], "bad small-communicator handle ", h);
    c = std::move(R.comms[h - 1]);   // out of the watchdog's sight from here on
  }
  if (c->kind == KIND_RCCL && c->nccl) {
    (void)hipDeviceSynchronize();
    (void)ncclCommDestroy(c->nccl);
    c->nccl = nullptr;
  }
  if (c->ev) (void)hipEventDestroy(c->ev);
}

// local teardown for a failed set-up (ranks agreed to fall back): ncclCommAbort never
// waits for peers, unlike a destroy that may flush operations they will never match
void small_comm_abort(int64_t h) {
  std::shared_ptr<SmallComm> c;
  {
    Registry& R = reg();
    std::lock_guard<std::mutex> lk(R.mu);
    TORCH_CHECK(h >= 1 && h <= (int64_t)R.comms.size() && R.comms[h - 1], "bad small-communicator handle ", h);
    c = std::move(R.comms[h - 1]);
  }
  if (c->kind == KIND_RCCL && c->nccl) {
    (void)ncclCommAbort(c->nccl);
    c->nccl = nullptr;
  }
  if (c->ev) (void)hipEventDestroy(c->ev);
}

void small_all_reduce_py(int64_t h, torch::Tensor x) { small_all_reduce_(h, x); }

// watchdog drill: a bounded GPU stall (seconds) on the current stream followed by a
// collective on handle h, so the armed event waits behind the stall
void small_comm_stall_(int64_t h, double seconds, torch::Tensor x) {
  check_hip(launch_gpu_stall((long long)(seconds * 1e8), cur_stream()), "gpu_stall");
  small_all_reduce_(h, x);
}

int64_t small_comm_ops(int64_t h) { return get(h)->ops.load(); }

// 0 none, 1 RCCL, 2 xGMI, 3 emulated
int64_t small_comm_kind(int64_t h) { return h == 0 ? 0 : (int64_t)get(h)->kind; }
int64_t small_comm_rank(int64_t h) { return h == 0 ? 0 : (int64_t)get(h)->rank; }

ncclDataType_t nccl_type(const torch::Tensor& x, const char* what) {
  switch (x.scalar_type()) {
    case at::kDouble: return ncclFloat64;
    case at::kFloat: return ncclFloat32;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    default: TORCH_CHECK(false, what, ": fp64 / fp32 / int32 / int64 only");
  }
}

SmallComm& gather_comm(int64_t h, const torch::Tensor& x, const char* what) {
  SmallComm& c = *get(h);
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.device().index() == c.device, what,
              ": contiguous tensor on the communicator's device");
  TORCH_CHECK(c.kind != KIND_XGMI, what, ": RCCL or emulated communicator only");
  if (c.kind == KIND_RCCL) TORCH_CHECK(c.nccl, what, ": RCCL communicator was aborted");
  return c;
}

// in place: rows [rank·n, (rank+1)·n) of `out` ([W·n, ...]) hold this rank's block on entry;
// on exit every block holds its rank's rows. Emulated ranks are identical: block copies.
void all_gather_inplace(SmallComm& c, torch::Tensor& out, int64_t block_elems) {
  if (c.world == 1 && c.kind != KIND_RCCL) return;   // (a 1-rank RCCL call is a tested no-op)
  hipStream_t s = cur_stream();
  const int64_t bytes = block_elems * out.element_size();
  char* base = static_cast<char*>(out.data_ptr());
  if (c.kind == KIND_RCCL) {
    settle(c, ncclAllGather(base + c.rank * bytes, base, (size_t)block_elems, nccl_type(out, "all-gather"), c.nccl, s),
           "ncclAllGather");
  } else {
    for (int r = 0; r < c.world; ++r)
      if (r != c.rank)
        check_hip(hipMemcpyAsync(base + r * bytes, base + c.rank * bytes, bytes, hipMemcpyDeviceToDevice, s),
                  "emulated all-gather");
  }
  arm(c, s);
}

// x [n, ...] -> [W·n, ...] (rank-major), ordered on the current stream
torch::Tensor small_all_gather(int64_t h, torch::Tensor x) {
  SmallComm& c = gather_comm(h, x, "small all-gather");
  auto sizes = x.sizes().vec();
  sizes[0] *= c.world;
  auto out = torch::empty(sizes, x.options());
  out.narrow(0, c.rank * x.size(0), x.size(0)).copy_(x);
  all_gather_inplace(c, out, x.numel());
  return out;
}

// g [W·n, ...] -> Σ_ranks g[rank block] ([n, ...]) (emulated: W identical ranks -> W·g[block])
torch::Tensor small_reduce_scatter(int64_t h, torch::Tensor g) {
  SmallComm& c = gather_comm(h, g, "small reduce-scatter");
  TORCH_CHECK(g.size(0) % c.world == 0, "small reduce-scatter: rows not divisible by the world size");
  const int64_t n = g.size(0) / c.world;
  auto sizes = g.sizes().vec();
  sizes[0] = n;
  if (c.world == 1 && c.kind != KIND_RCCL) return g.clone();
  hipStream_t s = cur_stream();
  torch::Tensor out;
  if (c.kind == KIND_RCCL) {
    out = torch::empty(sizes, g.options());
    settle(c, ncclReduceScatter(g.data_ptr(), out.data_ptr(), (size_t)out.numel(), nccl_type(g, "reduce-scatter"),
                                ncclSum, c.nccl, s),
           "ncclReduceScatter");
  } else {
    out = g.narrow(0, c.rank * n, n).mul((double)c.world);
  }
  arm(c, s);
  return out;
}

// Contrastive-loss input: L2-normalise this rank's projections straight
// into its block of the gathered contrast matrix, then all-gather in place — the loss
// kernel reads the result directly. Returns (C [W·n, d] fp32, row norms [n]).
std::vector<torch::Tensor> rownorm_gather(int64_t h, torch::Tensor x, double eps) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 2 && x.is_contiguous() && x.size(1) <= 256,
              "rownorm_gather: contiguous fp32 [n, d <= 256]");
  SmallComm& c = gather_comm(h, x, "rownorm_gather");
  c10::DeviceGuard dg(x.device());
  const int64_t n = x.size(0), d = x.size(1);
  auto C = torch::empty({c.world * n, d}, x.options());
  auto norms = torch::empty({n}, x.options());
  float* mine = C.data_ptr<float>() + c.rank * n * d;
  check_hip(launch_rownorm_fwd(x.data_ptr<float>(), (int)n, (int)d, (float)eps, mine, norms.data_ptr<float>(),
                               cur_stream()),
            "rownorm_fwd");
  all_gather_inplace(c, C, n * d);
  return {C, norms};
}

// backward of rownorm_gather: reduce-scatter the contrast-matrix gradient to the owners,
// then the row-normalisation gradient. y: this rank's normalised rows (C's block).
torch::Tensor rownorm_gather_bwd(int64_t h, torch::Tensor gC, torch::Tensor y, torch::Tensor norms, double eps) {
  TORCH_CHECK(gC.is_cuda() && gC.scalar_type() == at::kFloat && gC.dim() == 2, "gC: fp32 [W·n, d]");
  gC = gC.contiguous();
  y = y.contiguous();
  c10::DeviceGuard dg(gC.device());
  auto g = small_reduce_scatter(h, gC);
  TORCH_CHECK(g.sizes() == y.sizes() && norms.numel() == y.size(0), "rownorm_gather_bwd shapes");
  auto dx = torch::empty_like(g);
  check_hip(launch_rownorm_bwd(g.data_ptr<float>(), y.data_ptr<float>(), norms.contiguous().data_ptr<float>(),
                               (int)g.size(0), (int)g.size(1), (float)eps, dx.data_ptr<float>(), cur_stream()),
            "rownorm_bwd");
  return dx;
}

}  // namespace

int small_comm_world(int64_t h) { return h == 0 ? 1 : get(h)->world; }

// fused SyncBN exchange (XGMI / XEMU kinds of >1 ranks): the arena arguments of ONE exchange
// (epoch advanced); false for any other communicator (reduce -> small_all_reduce_ -> finalize)
bool small_comm_fused(int64_t h, XgmiCol* out) {
  if (h == 0) return false;
  auto cp = get(h);
  if (cp->world <= 1 || (cp->kind != KIND_XGMI && cp->kind != KIND_XEMU) || fused_disabled()) return false;
  *out = xgmi_col_args(cp->xgmi_id);
  return true;
}

// after the fused launch was enqueued on the current stream: watchdog event behind it
void small_comm_fused_issued(int64_t h) {
  auto cp = get(h);
  arm(*cp, cur_stream());
}

// in-place SUM over the communicator's ranks, ordered on the current stream
void small_all_reduce_(int64_t h, torch::Tensor& x) {
  if (h == 0) return;
  auto cp = get(h);
  SmallComm& c = *cp;
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "small all-reduce: contiguous GPU tensor");
  TORCH_CHECK(x.device().index() == c.device, "small all-reduce: tensor on device ", x.device().index(),
              ", communicator on ", c.device);
  if (c.world == 1) return;
  hipStream_t s = cur_stream();
  if (c.kind == KIND_RCCL) {
    TORCH_CHECK(c.nccl, "small all-reduce: RCCL communicator was aborted");
    ncclDataType_t dt;
    switch (x.scalar_type()) {
      case at::kDouble: dt = ncclFloat64; break;
      case at::kFloat: dt = ncclFloat32; break;
      case at::kInt: dt = ncclInt32; break;
      default: TORCH_CHECK(false, "small all-reduce: fp64 / fp32 / int32 only");
    }
    settle(c, ncclAllReduce(x.data_ptr(), x.data_ptr(), (size_t)x.numel(), dt, ncclSum, c.nccl, s), "ncclAllReduce");
  } else if (c.kind == KIND_EMU || c.kind == KIND_XEMU) {
    x.mul_((double)c.world);
  } else {
    TORCH_CHECK(x.scalar_type() == at::kDouble, "xGMI small all-reduce: fp64 only");
    auto r = xgmi_allreduce_ext(c.xgmi_id, x);
    x.copy_(r);
  }
  arm(c, s);
}

void register_comm(pybind11::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId as CPU uint8 bytes (rank 0; broadcast it)");
  m.def("rccl_comm_init", &rccl_comm_init,
        "dedicated non-blocking RCCL communicator for SyncBN statistics (init polled against timeout_s) -> handle",
        pybind11::arg("id"), pybind11::arg("world"), pybind11::arg("rank"), pybind11::arg("timeout_s") = 600.0);
  m.def("xgmi_small_comm", &xgmi_small_comm, "wrap a one-shot xGMI arena as a small-communicator handle",
        pybind11::arg("xgmi_id"), pybind11::arg("rank"), pybind11::arg("timeout_s") = 600.0);
  m.def("xgmi_emu_small_comm", &xgmi_emu_small_comm,
        "W identical virtual ranks whose BN statistics take the fused xGMI exchange (W arenas on this device)",
        pybind11::arg("world"), pybind11::arg("timeout_s") = 10.0);
  m.def("emu_small_comm", &emu_small_comm, "W identical virtual ranks in one process (tests): sum = x*W",
        pybind11::arg("world"), pybind11::arg("timeout_s") = 600.0);
  m.def("small_comm_destroy", &small_comm_destroy);
  m.def("small_comm_abort", &small_comm_abort, "local abort of a communicator whose set-up the ranks gave up");
  m.def("small_comm_world", &small_comm_world);
  m.def("small_comm_ops", &small_comm_ops, "collectives issued on a handle so far");
  m.def("small_all_reduce_", &small_all_reduce_py, "in-place SUM on the current stream");
  m.def("small_comm_kind", &small_comm_kind, "0 none, 1 RCCL, 2 xGMI, 3 emulated, 4 emulated fused xGMI");
  m.def("small_comm_rank", &small_comm_rank, "this process's rank on the communicator");
  m.def("small_all_gather", &small_all_gather, "rank-major all-gather along dim 0 (RCCL / emulated)");
  m.def("small_reduce_scatter", &small_reduce_scatter, "SUM reduce-scatter along dim 0 (RCCL / emulated)");
  m.def("rownorm_gather", &rownorm_gather,
        "row L2-normalise into this rank's block of the contrast matrix + in-place all-gather -> (C, norms)");
  m.def("rownorm_gather_bwd", &rownorm_gather_bwd, "reduce-scatter of dC + row-normalisation gradient");
  m.def("small_comm_stall_", &small_comm_stall_,
        "watchdog drill: bounded GPU stall, then a collective whose completion event waits behind it");
}

}  // namespace sdx_bind
