// C++ launcher declarations shared by the HIP kernel translation units and the
// torch binding layer. Launchers take raw device pointers plus the caller's HIP
// stream and never allocate or synchronise, so every one of them is safe to capture
// into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- selftest -------------------------------------------------------------------
hipError_t launch_mfma16_selftest(const void* A, const void* B, float* C, hipStream_t s);

// ---- projection-feature row norms (featnorm.hip) --------------------------------
hipError_t launch_rownorm_fwd(const float* x, int N, int D, float eps, float* y, float* norms, hipStream_t s);
hipError_t launch_rownorm_bwd(const float* dy, const float* y, const float* norms, int N, int D, float eps, float* dx,
                              hipStream_t s);
hipError_t launch_norm_stats(const float* x, int N, int D, int mode, double* sums, double n_global, float momentum,
                             float* rec, float* valid, float* out, hipStream_t s);

// ---- fused SupCon / NT-Xent loss (supcon.hip) ---------------------------------
int supcon_num_splits(int n_own, int n_other);
hipError_t launch_supcon_fwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, int Na, int N, int D, float inv_temp, float temp_ratio,
                             float scale, int n_split, float* part, float* lse, float* invcnt,
                             float* row_loss, float* loss, hipStream_t s);
// ws: fp32 workspace of supcon_bwd_workspace(Na, N, D) elements (per-split partial slabs)
long supcon_bwd_workspace(int Na, int N, int D);
// anchors == contrasts (one [N][D] tensor): dX = dA + dC through one split reduction;
// ws: supcon_bwd_sum_workspace(N, D) elements
long supcon_bwd_sum_workspace(int N, int D);
hipError_t launch_supcon_bwd_sum(const float* X, const int* a_self, const int* a_key, const int* c_key,
                                 const float* lse, const float* invcnt, int N, int D, float inv_temp, float w,
                                 const float* gscale, float* dX, float* ws, hipStream_t s);
hipError_t launch_supcon_bwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, const float* lse, const float* invcnt, int Na, int N, int D,
                             float inv_temp, float w, const float* gscale, float* dA, float* dC, float* ws,
                             hipStream_t s);

// ---- BN3 fold of the identity bottleneck backward (bnfold.hip) -----------------
// coef: [3][C] (A, D, E); w: conv3 forward weights bf16 [C][K]; wt: its dgrad layout [K][C].
// prep: wd = dgrad layout of diag(A)·W3 [K][C] bf16, mx = W3ᵀ·diag(D)·W3 [K][K] bf16,
// bias = Eᵀ·W3 [K] fp32. wgrad: sink (+)= diag(A)·G + diag(D)·W3·S + E ⊗ cs ([C][K] fp32).
// mu ([C] mean of y3) / cs ([K] column sums of a2 over `rows`): optional coherent-rounding
// correction folded into bias (see bnfold.hip)
// ldw / ldm: row strides of wd / mx in elements (0 = C / K; the K-concatenated fold writes
// both into one [K][C + K] tensor: wd at column 0, mx at column C)
hipError_t launch_bnfold_prep(const float* coef, const void* w, const void* wt, int C, int K, void* wd, void* mx,
                              float* bias, const float* mu, const float* cs, long rows, hipStream_t s, int ldw = 0,
                              int ldm = 0);
hipError_t launch_bnfold_wgrad(const float* coef, const float* G, const float* S, const float* cs, int ncs,
                               const void* w, int C, int K, float* sink, int accumulate, hipStream_t s);
// cs[K] = column sums of a [rows][K] bf16 tensor (partial: [bnfold_colsum_blocks()][K] scratch)
int bnfold_colsum_blocks();
// two BN-backward slab rows [2][ns][C] carrying Σ_k W[c][k]·G[c][k] (fp64 as fp32 hi + lo) in set 1
hipError_t launch_bnfold_rowdot(const float* G, const void* w, int C, int K, int ns, float* out_rows, hipStream_t s);
hipError_t launch_bnfold_colsum(const void* x, long rows, int K, float* partial, float* cs, hipStream_t s);

// ---- implicit-GEMM convolution (igemm.hip) ------------------------------------
struct ConvGeom {
  int N, H, W, C;   // input NHWC
  int K;            // output channels
  int R, S;         // filter
  int P, Q;         // output spatial
  int stride, pad;
};
// DGRAD epilogue BatchNorm-backward statistics of the stored dx (= the output gradient of
// the BN whose input the conv read): per M-tile Σd·m, Σd·m·(ya−μa) [, Σd·m·(yb−μb)] with
// m the ReLU mask — bitmask bit (mask), or ya·msc + msh > 0 (msc/msh), or 1 — written to
// slab row row0 + m_tile of a [rows][2|3][C] fp32 slab (reduced like the forward stats).
struct BnBwdStat {
  float* slab;
  const void* ya;
  const float* ma;
  const void* yb;        // optional second BN (projection shortcut) reading the same dx
  const float* mb;
  const uint8_t* mask;   // 1 bit per dx element
  const float* msc;
  const float* msh;
  int row0;
  int store_masked;      // store dx·m instead of dx (ReLU backward fused into the store)
};
// plain-GEMM epilogue of FWD / DGRAD launches (projection head): per-column fp32 bias,
// ReLU, fp32 output (stride-1 geometry, no BN statistics / addend with out_f32)
struct GemmEpi {
  const float* bias;
  int relu;
  int out_f32;
  // DGRAD (stride 1): add the bf16 addend to the fp32 accumulators before the single bf16
  // rounding instead of after it (builds with SDX_ADD_PRE=1; BN3 fold experiment)
  int add_pre;
  // FWD, stride-1 1x1 only: the block-output BatchNorm in the epilogue (forward-folded BN3) —
  // out = relu(bf16(y)·bn_scale + bn_shift + resid) and its ReLU bits (1 bit per element)
  const float* bn_scale;
  const float* bn_shift;
  const void* resid;
  uint8_t* mask_out;
  // projection blocks: resid is the shortcut conv's pre-BN output, normalised in the epilogue
  // as resid·resid_scale + resid_shift (both or neither)
  const float* resid_scale;
  const float* resid_shift;
  // DGRAD, stride-1 1x1 only (BN3 fold): K-concatenated second A operand cat_a [pixels][cat_ch]
  // (reduction over dy's K then cat_a's cat_ch channels; Wt rows of K + cat_ch) and an fp32
  // per-column bias added before the bf16 rounding
  const void* cat_a;
  int cat_ch;
  const float* bias_pre;
};
bool conv_dgrad_cat_supported(const ConvGeom& g, int cat_ch);
bool conv_fwd_bnapply_supported();
int igemm_tile_m(int cfg);
// diagnostic main-loop timeline (SDX_IGEMM_TRACE=1): block 0, waves 0 and 4, s_memtime stamps
int igemm_trace_slots();
hipError_t igemm_trace_copy(unsigned long long* host, hipStream_t s);
int igemm_tile_n(int cfg);
// tap-reuse 3x3 tile config (11-13) for a pad-1 stride-1 3x3 conv whose reduction runs over
// cdim channels and whose output has ncol channels (DGRAD: cdim = K, ncol = C), or -1
int igemm_tap_cfg(const ConvGeom& g, int cdim, int ncol);
// in_scale/in_shift (optional, [C] fp32): fused BN+ReLU prologue on the input activation
hipError_t launch_conv_fwd(const ConvGeom& g, const void* x, const void* w, void* y, float* stats, int cfg,
                           hipStream_t s, const float* in_scale = nullptr, const float* in_shift = nullptr,
                           const GemmEpi* epi = nullptr);
// strided dgrad = stride² sub-pixel classes; wt = the full Wt [C][R][S][K] (each class reads
// its taps r0::st, s0::st in place)
void conv_dgrad_class(const ConvGeom& g, int ph, int pw, int* r0, int* nr, int* s0, int* ns, int* Hc, int* Wc);
// addend (optional, may alias dx): bf16 tensor of dx's shape added in the epilogue
hipError_t launch_conv_dgrad_class(const ConvGeom& g, int ph, int pw, const void* dy, const void* wt, void* dx,
                                   const void* addend, int cfg, hipStream_t s, const void* addend_mask = nullptr,
                                   const BnBwdStat* bstat = nullptr, int addend_sub = 0,
                                   const GemmEpi* epi = nullptr);
// every sub-pixel class of a strided dgrad (stride 2) in ONE launch; bstat->row0 = the first
// class's slab row (the classes' rows follow in the kernel's class order)
hipError_t launch_conv_dgrad_merged(const ConvGeom& g, const void* dy, const void* wt, void* dx, const void* addend,
                                    int cfg, hipStream_t s, const void* addend_mask = nullptr,
                                    const BnBwdStat* bstat = nullptr, int addend_sub = 0);
// M-tiles of one sub-pixel class launch (= its slab rows with a BnBwdStat)
// statistics-slab rows (M-tiles) of a stride-1 fwd / dgrad conv with reduction channels cdim
// under tile config cfg (padded-row tap tiles count virtual rows)
int64_t igemm_conv_mtiles(const ConvGeom& g, int cdim, int cfg, int64_t M);
int conv_dgrad_class_mtiles(const ConvGeom& g, int ph, int pw, int cfg);
int conv_wgrad_splits(const ConvGeom& g, int cfg, int splits);
// partial: fp32 [splits][K][R*S*C] workspace (unused when splits == 1 and !accumulate)
hipError_t launch_conv_wgrad(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int cfg,
                             int splits, int accumulate, hipStream_t s, const float* in_scale = nullptr,
                             const float* in_shift = nullptr);
// dW (+)= Σ_split partial[split] (fp32 [splits][n4*4]), deterministic order
hipError_t launch_splitk_reduce(const float* partial, int splits, long n4, float* dw, int accumulate, hipStream_t s);
// Deferral of the split-K reductions launched on stream s (this host thread): they are queued
// until splitk_flush(), which issues them as one multi-tensor launch on s. The caller keeps
// the partial slabs alive until then and must not read the queued dW before the flush.
void splitk_defer_begin(hipStream_t s);
bool splitk_deferring(hipStream_t s);
hipError_t splitk_flush();
void splitk_defer_cancel();   // drop the queue (error paths)
// Tap-reuse 3x3 wgrad (wgrad3x3.hip): stride 1 or 2, pad 1, output width in {4,8,16,32}, C,K % 64 == 0.
// partial: fp32 [splits][K][9C] (unused when splits == 1 and !accumulate)
bool wgrad3x3_supported(const ConvGeom& g);
int wgrad3x3_tiles(const ConvGeom& g);
int wgrad3x3_steps(const ConvGeom& g);
hipError_t launch_wgrad3x3(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int splits,
                           int accumulate, hipStream_t s);
// 1x1 wgrad (wgrad1x1.hip): K % 128 == 0, C % 128 == 0, N*H*W % 32 == 0 (stride 1 or a
// whole-subgrid strided shortcut), or stride 1 with a 64-channel side (pixel pairs, N*H*W % 64).
// partial: fp32 [wgrad1x1_slices(g, splits)][K][C] (unused when splits == 1, !accumulate and
// no pixel pairs)
bool wgrad1x1_supported(const ConvGeom& g);
int wgrad1x1_tiles(const ConvGeom& g);
int wgrad1x1_steps(const ConvGeom& g);
int wgrad1x1_slices(const ConvGeom& g, int splits);
bool wgrad1x1_pair_view(const ConvGeom& g);
// runtime switch of the pixel-pair view (tests / A/B); returns the previous value
int wgrad1x1_pairs_set(int on);
// the 256-row LDS-DMA kernel: 0 off, 1 long-split shapes only (default), 2 every eligible
// shape (SDX_W1_BIG); returns the previous setting
int wgrad1x1_big_set(int mode);
// longest GEMM reduction on the single-stage LDS-DMA loop (mode 0 forward, 1 data gradient;
// SDX_IGEMM_ONE_K / _DGRAD); returns the previous limit
int igemm_one_k_set(int mode, int k);
hipError_t launch_wgrad1x1(const ConvGeom& g, const void* dy, const void* x, float* partial, float* dw, int splits,
                           int accumulate, hipStream_t s);

// ---- BatchNorm (bn.hip) ---------------------------------------------------------
// Per-channel finalize (forward) and coefficient (backward) arguments, evaluated either by
// their own kernels (SyncBN: after the cross-rank all-reduce of the sums) or inside the
// last block of the single-launch column reduction (no cross-rank reduction needed).
struct BnFinalizeArgs {
  double count;
  const float* gamma;
  const float* beta;
  float eps, momentum;
  int update_running;
  float* running_mean;
  float* running_var;
  float *scale, *shift, *mean, *invstd;
};
struct BnCoefArgs {
  double count;
  const float *g_a, *mean_a, *inv_a, *g_b, *mean_b, *inv_b;
  float *coef_a, *coef_b, *dgamma_a, *dbeta_a, *dgamma_b, *dbeta_b;
  int accumulate;
  // factor on the dγ/dβ written to the sinks. SyncBN over W ranks sums Σdz, Σdz·ŷ over the
  // ranks before the coefficients; the parameter gradient must stay this rank's share
  // (global / W, like torch SyncBatchNorm's local grad_weight after the DDP mean), so the
  // bucket reducer's sum × 1/W yields global / W and not the global value.
  double grad_scale = 1.0;
};
// ---- xGMI peer arenas (xgmi.hip, bn.hip) ----------------------------------------------
constexpr int kXgmiMaxPeers = 8;
constexpr int kXgmiFlagGroups = 64;   // per-sender flags per parity: one per 64-channel column group
struct XgmiPeers {
  double* data[kXgmiMaxPeers];     // each rank's receive arena: [2][W][cap] fp64 (IPC-mapped)
  unsigned* flags[kXgmiMaxPeers];  // each rank's flags: [2][W][kXgmiFlagGroups] u32
  size_t cap;                      // elements per slot
};
// SyncBN statistics exchanged INSIDE the column reduction (bn.hip): the last block of
// every 64-channel group stores its [nsets][64] fp64 sums into every rank's arena slot
// [parity][me], publishes the group's flag, waits for every sender's flag of that group
// and sums the W slots in rank order (bit-identical on every rank) before its epilogue —
// reduce + all-reduce + finalize/coefficients in ONE launch.
//   mode 1: real peers (IPC-mapped uncached arenas, system scope).
//   mode 2: single-GPU emulation — `world` virtual ranks are gridDim.z of the SAME launch
//           (arenas in device memory, agent scope); rank z reduces slab + z·slab_zstride
//           (0: identical ranks, the EMU semantics Σ = W·x) and only rank 0 writes the sums
//           and runs the epilogue. counters/scratch are W consecutive per-rank blocks.
struct XgmiCol {
  XgmiPeers peers;
  int mode = 0, me = 0, world = 1;
  unsigned epoch = 0;
  // device-side epoch (null: the host `epoch`): per rank (emulated: per virtual rank) a pair
  // [epoch, groups-done ticket]. Every column group's last block takes epoch + 1 for this
  // exchange; the last group to finish stores it back. One epoch sequence per rank for every
  // exchange and one-shot call on the arena, so parities alternate launch by launch, and a
  // launch replayed from a hipGraph advances its own epoch (a host argument would be frozen
  // at capture and the flag waits would pass on stale flags)
  unsigned* epoch_ctr = nullptr;
  int* err = nullptr;               // host-pinned: 1 + sender whose flag missed the deadline
  long long timeout_ticks = 0;      // 100 MHz wall-clock ticks
  long slab_zstride = 0;            // mode 2: elements between virtual ranks' slabs
  // mode 2, one rank's share (SDX_SYNCBN_EMU_SOLO / tools/syncbn_latency.py): only virtual
  // rank 0 runs (grid z = 1); it reduces, stores to all W arenas, publishes all W flags and
  // polls only its own flag — the other W-1 ranks count as already published — so the
  // kernel time is one real rank's reduce + W stores + poll + W-slot sum + epilogue
  int solo = 0;
};

// Deterministic reduction of a [rows][nsets][C] fp32 slab to fp64 sums [nsets][C] in ONE
// launch (per-block partials + last-arriver combine; no memset). epi: 0 sums only,
// 1 + BN finalize (nsets 2), 2 + BN backward coefficients (nsets 2|3), 3 gradient-sink add
// of set 0 (ca->dbeta_a[c] += Σ·ca->grad_scale: a bias gradient; nsets 1|2).
int col_reduce_gy(int rows);
// xg (optional): cross-rank exchange of the sums before the epilogue (see XgmiCol); the
// epilogue's count must then be the global row count
hipError_t launch_col_reduce(const float* slab, int rows, int nsets, int C, double* scratch, unsigned* counters,
                             double* sums, int epi, const BnFinalizeArgs* fa, const BnCoefArgs* ca, hipStream_t s,
                             const XgmiCol* xg = nullptr);
hipError_t launch_bn_finalize(const double* sums, int C, const BnFinalizeArgs& a, hipStream_t s);
hipError_t launch_bn_eval_affine(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                                 float eps, float* scale, float* shift, hipStream_t s);
hipError_t launch_bn_apply(const void* y, const float* sc, const float* sh, const void* r, const float* sc2,
                           const float* sh2, int res_mode, int relu, void* out, long numel, int C, hipStream_t s,
                           void* mask_out = nullptr);   // optional uint8 [numel/8]: bit i = out[8e+i] > 0
int bn_bwd_reduce_blocks(long numel, int C);
// partial [bn_bwd_reduce_blocks][nsets][C] written by the elementwise pass, then reduced
// by launch_col_reduce (epi 0: sums only; epi 2: fused coefficients from `ca`)
hipError_t launch_bn_bwd_reduce(const void* dout, const void* outv, const void* ya, const float* ma, const void* yb,
                                const float* mb, long numel, int C, float* partial, double* scratch,
                                unsigned* counters, double* sums, int epi, const BnCoefArgs* ca, hipStream_t s,
                                const float* msc = nullptr, const float* msh = nullptr, const void* omask = nullptr,
                                const XgmiCol* xg = nullptr);
hipError_t launch_bn_bwd_coef(const double* sums, int nsets, int C, const BnCoefArgs& a, hipStream_t s);
hipError_t launch_bn_bwd_apply(const void* dout, const void* outv, const void* ya, const float* ca, const void* yb,
                               const float* cb, void* dya, void* dyb, void* dz_out, long numel, int C, hipStream_t s,
                               const float* msc = nullptr, const float* msh = nullptr, const void* omask = nullptr);

// ---- GPU augmentation (aug.hip) -------------------------------------------------
hipError_t launch_gpu_augment(const uint8_t* data, const int64_t* idx, int B, int H, int W, int S, int n_views,
                              uint64_t seed, const float* mean, const float* std, float scale_lo, float scale_hi,
                              float ratio_lo, float ratio_hi, float jitter_p, float bright, float contrast,
                              float sat, float hue, float gray_p, int do_crop, int do_flip, const int64_t* seed_dev,
                              void* out, hipStream_t s, long n_data = 0, const int64_t* offs = nullptr,
                              const int32_t* hw = nullptr);

// ---- optimizers (optim.hip) -----------------------------------------------------
hipError_t launch_sgd(float* p, const float* g, float* buf, long n, const float* lr, float momentum, float wd,
                      float gscale, int nesterov, hipStream_t s, int max_blocks = 0);
hipError_t launch_lars(float* p, const float* g, float* buf, const long* seg_off, const int* adapt, int nseg, long n,
                       const float* lr, float momentum, float wd, float gscale, float eta, float* norms,
                       hipStream_t s);

// ---- pooling (pool.hip) ---------------------------------------------------------
hipError_t launch_maxpool_fwd(const void* x, void* y, int N, int H, int W, int C, int P, int Q, int k, int stride,
                              int pad, hipStream_t s);
hipError_t launch_maxpool_bwd(const void* x, const void* y, const void* dy, void* dx, int N, int H, int W, int C,
                              int P, int Q, int k, int stride, int pad, hipStream_t s);
// forward that also records each window's first-max position (uint8 [N][P][Q][C], k*k <= 255)
// and the backward that scatters from it (no re-read of the pooled input)
hipError_t launch_maxpool_fwd_idx(const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int P, int Q,
                                  int k, int stride, int pad, hipStream_t s);
hipError_t launch_maxpool_bwd_idx(const uint8_t* idx, const void* dy, void* dx, int N, int H, int W, int C, int P,
                                  int Q, int k, int stride, int pad, hipStream_t s);
hipError_t launch_gap_fwd(const void* x, float* y, int N, int HW, int C, hipStream_t s);
hipError_t launch_gap_bwd(const float* dy, void* dx, int N, int HW, int C, hipStream_t s);

// ---- weight preparation (wprep.hip) ---------------------------------------------
// segs: device table of nseg rows {src, dst_k, dst_t, K|RS<<32, C|Cp<<32, n, start} (int64)
hipError_t launch_wprep(const float* master, void* out, const void* segs, int nseg, long total, hipStream_t s);
// dst[r][c] += src[r][c], c < C, of a channel-padded [rows][Cp] fp32 tensor (stem weight gradient)
hipError_t launch_unpad_add(const float* src, float* dst, int rows, int Cp, int C, hipStream_t s);

// ---- one-shot small all-reduce over xGMI peer memory (xgmi.hip) --------------------
// err: host-pinned int (1 + rank of a peer whose flag missed the deadline of timeout_ticks
// of the 100 MHz wall clock; the sum is then skipped)
// epoch_ctr (optional): the arena's device epoch pair (XgmiCol::epoch_ctr); `epoch` then unused
hipError_t launch_xgmi_allreduce(const double* in, double* out, int n, const XgmiPeers& peers, int me, int world,
                                 unsigned epoch, int* err, long long timeout_ticks, hipStream_t s,
                                 unsigned* epoch_ctr = nullptr);
// bounded single-wave sleep on stream s (watchdog tests)
hipError_t launch_gpu_stall(long long ticks, hipStream_t s);
hipError_t launch_xgmi_emulate(const double* in, double* out, int n, const XgmiPeers& peers, int world,
                               unsigned epoch, int* err, hipStream_t s);
