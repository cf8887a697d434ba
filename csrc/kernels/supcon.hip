// Fused SupCon / SimCLR (NT-Xent) loss for gfx950: cosine-similarity tiles on MFMA,
// online log-sum-exp, positive-set statistics and the analytic backward, without ever
// materialising the N x N logits (reference: losses.py:17-93, main_supcon.py:283-293).
//
// Row form (see losses/supcon.py): anchors are rows of the gathered, L2-normalised
// contrast matrix C[N][D]; anchor i has contrast index self[i] and key akey[i];
// contrast j has key ckey[j]; positive(i,j) <=> akey[i]==ckey[j] && j!=self[i].
//
// The backward is deterministic: every split writes its own slice of a partial slab and
// the slices are summed in split order (no atomics).
//
// One kernel template serves three modes. A workgroup (4 waves) owns 64 "own" rows
// (16 per wave, one own row per lane column of the MFMA tile) and streams the "other"
// rows through LDS in 32-row tiles (shared by the 4 waves):
//   FWD   own = anchors,   other = contrasts: per-(split,anchor) partial (max, sumexp,
//         positive-logit sum, positive count)
//   BWD_A own = anchors,   other = contrasts: dA_i += Σ_j G_ij c_j
//   BWD_C own = contrasts, other = anchors:   dC_j += Σ_i G_ij a_i
// with G_ij = w·(softmax_ij − pos_ij/|P_i|). The tile product is computed as
// S^T = other·ownᵀ so the other-row index sits in the accumulator registers; the
// backward product Σ_other other^T·G^T then takes G^T straight from the accumulators
// as the MFMA B operand (cdna_hip_programming.md §3 "accumulator as operand"), and the
// matching A operand is fetched with ds_read_b64_tr_b16 transposed LDS reads.
//
// Precision: fp32 inputs are split into bf16 hi + lo and every product uses three
// v_mfma_f32_16x16x32_bf16 (hi·hi + hi·lo + lo·hi): ~2^-16 relative error (fp32-class
// logits) at 3/16 of the cost of the fp32-input MFMA.
#include "common.h"
#include "launchers.h"

using namespace sdx;

namespace {

enum { MODE_FWD = 0, MODE_BWD_A = 1, MODE_BWD_C = 2 };

constexpr int OTHER_TILE = 32;   // other rows per LDS tile
constexpr int OWN_PER_WG = 64;   // 4 waves x 16

struct SupconParams {
  const float* own;      // [n_own][D]
  const float* other;    // [n_other][D]
  const int* a_self;     // [Na]
  const int* a_key;      // [Na]
  const int* c_key;      // [N]
  const float* lse;      // [Na]   (bwd)
  const float* invcnt;   // [Na]   (bwd; <0 marks an anchor without positives)
  float* part;           // fwd: [4][S][n_own]
  float* out;            // bwd: [n_split][n_own][D] partial slab (one slice per split; the
                         // direct output when n_split == 1), summed in fixed split order
  const float* gscale;   // bwd: device scalar (upstream gradient), multiplies w
  int n_own, n_other, other_per_split, n_split;
  float inv_temp, w;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ void split_hi_lo(float x, uint16_t& hi, uint16_t& lo) {
  hi = f2bf(x);
  lo = f2bf(x - bf2f(hi));
}

// LDS image of the 32 staged other rows (bf16 hi and lo images). D >= 128: unpadded
// 2D-byte rows with the 16-B chunk index XOR-swizzled by sw(r) = (r & 7) << 1, chosen for
// the three access patterns and their lane groups (MI355X_MICROARCH.md §LDS):
//   * tile-product ds_read_b128 (groups {0–3,12–15,20–27}, ...: rows c of one 16-row tile,
//     chunk k for h = 0 and k|1 for h = 1): each group hits all 16 slots of the 256-B row;
//   * backward ds_read_b64_tr_b16 (32-lane halves: 8 rows x 2 adjacent chunks): sw/2 is a
//     permutation of the 8 rows, so 16 distinct slots;
//   * staging ds_write_b128 (8 contiguous lanes = 8 consecutive chunks of one row, banks mod
//     128 B): distinct slots for any sw.
// (Round 2's +16-B row padding: 2-way conflicts on the staging writes, ~50 % of LDS cycles
// at N = 8192, profiles/pmc_conv_supcon_r1_v2.txt; a first swizzle with a row-bit-3 term in
// bit 0 fixed the writes but left the b128 reads 2-way: 28-40 %, profiles/pmc_supcon_r3.txt.)
// D = 64 keeps the padded rows.
template <int D>
__device__ __forceinline__ int sc_off(int row, int byte) {
  if constexpr (D >= 128) {
    const int sw = (row & 7) << 1;
    return row * (D * 2) + ((((byte >> 4) ^ sw)) << 4) + (byte & 15);
  } else {
    return row * (D * 2 + 16) + byte;
  }
}

template <int D, int MODE>
__global__ __launch_bounds__(256) void supcon_tile_kernel(SupconParams p) {
  constexpr int KS = D / 32;                 // MFMA k-steps over the feature dim
  constexpr int RS = D >= 128 ? D * 2 : D * 2 + 16;   // LDS row stride (bytes) of a bf16 row
  constexpr int TILE_BYTES = OTHER_TILE * RS;
  constexpr int STAGE_BYTES = 2 * TILE_BYTES;             // hi + lo
  constexpr int OSTR = D + 4;                // fp32 transpose rows padded by 16 B (bank spread)
  constexpr int OUT_BYTES = (MODE == MODE_FWD) ? 0 : OWN_PER_WG * OSTR * 4;
  constexpr int LDS_BYTES = STAGE_BYTES > OUT_BYTES ? STAGE_BYTES : OUT_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  unsigned char* lds_hi = smem;
  unsigned char* lds_lo = smem + TILE_BYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int h = lane >> 4;       // 16-lane group
  const int c = lane & 15;       // column within the MFMA tile (= own row of this lane)
  const int own0 = blockIdx.x * OWN_PER_WG + wv * 16;
  const int own = own0 + c;
  const int own_ld = own < p.n_own ? own : (p.n_own - 1);

  // ---- own-row fragments (MFMA B operand of the tile product), kept in registers ----
  bf16x8 ob_hi[KS], ob_lo[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const float4* src = reinterpret_cast<const float4*>(p.own + (size_t)own_ld * D + 32 * s + 8 * h);
    const float4 v0 = src[0], v1 = src[1];
    const float xs[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint16_t hi, lo;
      split_hi_lo(xs[j], hi, lo);
      ob_hi[s][j] = (short)hi;
      ob_lo[s][j] = (short)lo;
    }
  }

  // ---- per-own constants ----
  int own_self = 0, own_key = 0;
  float own_lse = 0.f, own_ic = 0.f;
  if (MODE == MODE_BWD_C) {
    own_key = p.c_key[own_ld];
  } else {
    own_self = p.a_self[own_ld];
    own_key = p.a_key[own_ld];
    if (MODE == MODE_BWD_A) {
      own_lse = p.lse[own_ld];
      own_ic = p.invcnt[own_ld];
    }
  }

  const float wscale = (MODE == MODE_FWD) ? 0.f : p.w * p.gscale[0];
  // fwd running statistics for this lane's own row (over the other rows it sees)
  float run_m = -INFINITY, run_l = 0.f, run_ps = 0.f, run_pc = 0.f;
  // bwd accumulators: out^T tiles [d = 16q + 4h + r][own = c]
  f32x4 acc2[D / 16];
#pragma unroll
  for (int q = 0; q < D / 16; ++q) acc2[q] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int o_begin = blockIdx.y * p.other_per_split;
  int o_end = o_begin + p.other_per_split;
  if (o_end > p.n_other) o_end = p.n_other;

  for (int ob = o_begin; ob < o_end; ob += OTHER_TILE) {
    // ---- stage 32 other rows into LDS as bf16 hi/lo: thread = one 8-float chunk, the 16..32
    // lanes of a row adjacent (coalesced 32-B global reads, conflict-free LDS writes) ----
    {
      constexpr int CPR = D / 8;                     // 16-B bf16 chunks per row
      constexpr int RPP = 256 / CPR;                 // rows per pass
#pragma unroll
      for (int pass = 0; pass < OTHER_TILE / RPP; ++pass) {
        const int r = pass * RPP + tid / CPR;
        const int k = tid % CPR;
        const int orow = ob + r;
        float xs[8];
        if (orow < o_end) {
          const float4* src = reinterpret_cast<const float4*>(p.other + (size_t)orow * D + 8 * k);
          const float4 v0 = src[0], v1 = src[1];
          xs[0] = v0.x; xs[1] = v0.y; xs[2] = v0.z; xs[3] = v0.w;
          xs[4] = v1.x; xs[5] = v1.y; xs[6] = v1.z; xs[7] = v1.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) xs[j] = 0.f;
        }
        uint4 vh, vl;
        uint16_t hh[8], ll[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) split_hi_lo(xs[j], hh[j], ll[j]);
        vh.x = hh[0] | (hh[1] << 16); vh.y = hh[2] | (hh[3] << 16);
        vh.z = hh[4] | (hh[5] << 16); vh.w = hh[6] | (hh[7] << 16);
        vl.x = ll[0] | (ll[1] << 16); vl.y = ll[2] | (ll[3] << 16);
        vl.z = ll[4] | (ll[5] << 16); vl.w = ll[6] | (ll[7] << 16);
        const int o = sc_off<D>(r, 16 * k);
        *reinterpret_cast<uint4*>(lds_hi + o) = vh;
        *reinterpret_cast<uint4*>(lds_lo + o) = vl;
      }
    }
    __syncthreads();

    // ---- S^T tiles: acc[t][r] = <other[ob+16t+4h+r], own[c]> ----
    f32x4 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int off = sc_off<D>(16 * t + c, (32 * s + 8 * h) * 2);
        const bf16x8 a_hi = *reinterpret_cast<const bf16x8*>(lds_hi + off);
        const bf16x8 a_lo = *reinterpret_cast<const bf16x8*>(lds_lo + off);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_hi, ob_hi[s], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_hi, ob_lo[s], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a_lo, ob_hi[s], acc[t], 0, 0, 0);
      }
    }

    if (MODE == MODE_FWD) {
      float sv[8];
      bool valid[8];
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = ob + 16 * t + 4 * h + r;
          const int k = 4 * t + r;
          sv[k] = acc[t][r] * p.inv_temp;
          valid[k] = (o < o_end) && (o != own_self);
          if (valid[k]) {
            tmax = fmaxf(tmax, sv[k]);
            if (p.c_key[o] == own_key) { run_ps += sv[k]; run_pc += 1.f; }
          }
        }
      if (tmax > -INFINITY) {
        const float mn = fmaxf(run_m, tmax);
        float l = run_l * __expf(run_m - mn);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (valid[k]) l += __expf(sv[k] - mn);
        run_m = mn;
        run_l = l;
      }
    } else {
      // ---- G^T in the accumulator layout, split into bf16 hi/lo B fragments ----
      bf16x8 g_hi, g_lo;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int o = ob + 16 * t + 4 * h + r;
          const float s = acc[t][r] * p.inv_temp;
          float g = 0.f;
          if (o < o_end) {
            if (MODE == MODE_BWD_A) {
              if (o != own_self && own_ic >= 0.f) {
                const float pos = (p.c_key[o] == own_key) ? own_ic : 0.f;
                g = wscale * (__expf(s - own_lse) - pos);
              }
            } else {
              const float ic = p.invcnt[o];
              if (p.a_self[o] != own && ic >= 0.f) {
                const float pos = (p.a_key[o] == own_key) ? ic : 0.f;
                g = wscale * (__expf(s - p.lse[o]) - pos);
              }
            }
          }
          uint16_t hi, lo;
          split_hi_lo(g, hi, lo);
          g_hi[4 * t + r] = (short)hi;
          g_lo[4 * t + r] = (short)lo;
        }
      // ---- out^T[d][own] += Σ_o other[o][d] G^T[o][own]; A operand by transposed LDS reads ----
      const int qq = c >> 2, pp = c & 3;
#pragma unroll
      for (int q = 0; q < D / 16; ++q) {
        bf16x8 a2_hi, a2_lo;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int off = sc_off<D>(16 * tt + 4 * h + qq, (16 * q + 4 * pp) * 2);
          const bf16x4 th = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds_hi + off));
          const bf16x4 tl = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds_lo + off));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a2_hi[4 * tt + e] = th[e];
            a2_lo[4 * tt + e] = tl[e];
          }
        }
        acc2[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2_hi, g_hi, acc2[q], 0, 0, 0);
        acc2[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2_hi, g_lo, acc2[q], 0, 0, 0);
        acc2[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2_lo, g_hi, acc2[q], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  if (MODE == MODE_FWD) {
    // combine the 4 lane groups that hold the same own row
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float m2 = __shfl_xor(run_m, off, 64);
      const float l2 = __shfl_xor(run_l, off, 64);
      const float mn = fmaxf(run_m, m2);
      float l = 0.f;
      if (mn > -INFINITY) l = run_l * __expf(run_m - mn) + l2 * __expf(m2 - mn);
      run_m = mn;
      run_l = l;
      run_ps += __shfl_xor(run_ps, off, 64);
      run_pc += __shfl_xor(run_pc, off, 64);
    }
    if (h == 0 && own < p.n_own) {
      const size_t stride = (size_t)p.n_split * p.n_own;
      const size_t idx = (size_t)blockIdx.y * p.n_own + own;
      p.part[idx] = run_m;
      p.part[stride + idx] = run_l;
      p.part[2 * stride + idx] = run_ps;
      p.part[3 * stride + idx] = run_pc;
    }
  } else {
    // transpose through LDS so each wave stores whole contiguous rows of this split's
    // slice (no atomics: the splits are summed in fixed order by supcon_split_reduce)
    float* out_lds = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int q = 0; q < D / 16; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) out_lds[(wv * 16 + c) * OSTR + 16 * q + 4 * h + r] = acc2[q][r];
    __syncthreads();
    float* slice = p.out + (size_t)blockIdx.y * p.n_own * D;
    for (int rr = 0; rr < 16; ++rr) {
      const int orow = own0 + rr;
      if (orow >= p.n_own) break;
#pragma unroll
      for (int d = 4 * lane; d < D; d += 256)
        *reinterpret_cast<float4*>(slice + (size_t)orow * D + d) =
            *reinterpret_cast<const float4*>(out_lds + (wv * 16 + rr) * OSTR + d);
    }
  }
}

// out[e] = Σ_{s < n_split} part[s][e] in split order (deterministic), float4 per thread
__global__ __launch_bounds__(256) void supcon_split_reduce_kernel(const float* __restrict__ part, int n_split,
                                                                  long n4, float* __restrict__ out) {
  const long e = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (e >= n4) return;
  const float4* P = reinterpret_cast<const float4*>(part);
  float4 a = P[e];
  for (int s = 1; s < n_split; ++s) {
    const float4 v = P[(size_t)s * n4 + e];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  reinterpret_cast<float4*>(out)[e] = a;
}

hipError_t split_reduce(const float* part, int n_split, long n, float* out, hipStream_t s) {
  const long n4 = n / 4;
  hipLaunchKernelGGL(supcon_split_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, part, n_split,
                     n4, out);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

// Combine the per-split partials: lse_i, 1/|P_i| (or -1), and the scaled loss sum.
__global__ __launch_bounds__(1024) void supcon_finalize_kernel(const float* __restrict__ part, int n_split, int n_own,
                                                              float temp_ratio, float scale, float* __restrict__ lse,
                                                              float* __restrict__ invcnt, float* __restrict__ row_loss,
                                                              float* __restrict__ loss) {
  __shared__ float red[16];
  const size_t stride = (size_t)n_split * n_own;
  float acc = 0.f;
  for (int i = threadIdx.x; i < n_own; i += blockDim.x) {
    float m = -INFINITY, l = 0.f, ps = 0.f, pc = 0.f;
    for (int s = 0; s < n_split; ++s) {
      const size_t idx = (size_t)s * n_own + i;
      const float m2 = part[idx], l2 = part[stride + idx];
      const float mn = fmaxf(m, m2);
      if (mn > -INFINITY) l = l * __expf(m - mn) + l2 * __expf(m2 - mn);
      m = mn;
      ps += part[2 * stride + idx];
      pc += part[3 * stride + idx];
    }
    const float L = m + __logf(l);
    lse[i] = L;
    float li = 0.f;
    if (pc > 0.f) {
      invcnt[i] = 1.f / pc;
      li = -temp_ratio * (ps / pc - L);
    } else {
      invcnt[i] = -1.f;
    }
    row_loss[i] = li;
    acc += li;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    loss[0] = t * scale;
  }
}

template <int MODE>
hipError_t launch_mode(int D, const SupconParams& p, hipStream_t s) {
  const dim3 grid((p.n_own + OWN_PER_WG - 1) / OWN_PER_WG, p.n_split);
  switch (D) {
    case 64: hipLaunchKernelGGL((supcon_tile_kernel<64, MODE>), grid, dim3(256), 0, s, p); break;
    case 128: hipLaunchKernelGGL((supcon_tile_kernel<128, MODE>), grid, dim3(256), 0, s, p); break;
    case 256: hipLaunchKernelGGL((supcon_tile_kernel<256, MODE>), grid, dim3(256), 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

int pick_splits(int n_own, int n_other) {
  // aim for >= ~512 workgroups while keeping >= 2 other tiles per split
  const int own_blocks = (n_own + OWN_PER_WG - 1) / OWN_PER_WG;
  int s = (512 + own_blocks - 1) / own_blocks;
  const int max_s = (n_other + 2 * OTHER_TILE - 1) / (2 * OTHER_TILE);
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return s;
}

}  // namespace

int supcon_num_splits(int n_own, int n_other) { return pick_splits(n_own, n_other); }

namespace {
// the split counts the two backward passes actually use (other_per_split rounded to tiles)
int bwd_splits(int n_own, int n_other, int* per_out) {
  int ns = pick_splits(n_own, n_other);
  int per = (n_other + ns - 1) / ns;
  per = ((per + OTHER_TILE - 1) / OTHER_TILE) * OTHER_TILE;
  *per_out = per;
  return (n_other + per - 1) / per;
}
}  // namespace

long supcon_bwd_workspace(int Na, int N, int D) {
  int per;
  const int sa = bwd_splits(Na, N, &per), sc = bwd_splits(N, Na, &per);
  return (sa > 1 ? (long)sa * Na * D : 0) + (sc > 1 ? (long)sc * N * D : 0);
}

hipError_t launch_supcon_fwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, int Na, int N, int D, float inv_temp, float temp_ratio,
                             float scale, int n_split, float* part, float* lse, float* invcnt,
                             float* row_loss, float* loss, hipStream_t s) {
  SupconParams p{};
  p.own = A; p.other = C; p.a_self = a_self; p.a_key = a_key; p.c_key = c_key;
  p.part = part; p.n_own = Na; p.n_other = N; p.n_split = n_split;
  const int per = (N + n_split - 1) / n_split;
  p.other_per_split = ((per + OTHER_TILE - 1) / OTHER_TILE) * OTHER_TILE;
  p.inv_temp = inv_temp;
  hipError_t e = launch_mode<MODE_FWD>(D, p, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(supcon_finalize_kernel, dim3(1), dim3(1024), 0, s, part, n_split, Na, temp_ratio, scale, lse,
                     invcnt, row_loss, loss);
  SDX_LAUNCH_CHECK();
  return hipSuccess;
}

// anchors == contrasts (single rank, contrast_mode all: A and C are one tensor): d(A) + d(C)
// in ONE reduction — both passes write split slabs of the same [N][D] layout back to back,
// and one split reduce sums all of them (no separate reduce per pass, no elementwise add)
long supcon_bwd_sum_workspace(int N, int D) {
  int per;
  return (long)2 * bwd_splits(N, N, &per) * N * D;
}

hipError_t launch_supcon_bwd_sum(const float* X, const int* a_self, const int* a_key, const int* c_key,
                                 const float* lse, const float* invcnt, int N, int D, float inv_temp, float w,
                                 const float* gscale, float* dX, float* ws, hipStream_t s) {
  SupconParams p{};
  p.gscale = gscale;
  p.a_self = a_self; p.a_key = a_key; p.c_key = c_key; p.lse = lse; p.invcnt = invcnt;
  p.inv_temp = inv_temp; p.w = w;
  p.own = X; p.other = X; p.n_own = N; p.n_other = N;
  const int sa = bwd_splits(N, N, &p.other_per_split);
  p.n_split = sa;
  p.out = ws;
  hipError_t e = launch_mode<MODE_BWD_A>(D, p, s);
  if (e != hipSuccess) return e;
  const int sc = bwd_splits(N, N, &p.other_per_split);
  p.n_split = sc;
  p.out = ws + (long)sa * N * D;
  if ((e = launch_mode<MODE_BWD_C>(D, p, s)) != hipSuccess) return e;
  return split_reduce(ws, sa + sc, (long)N * D, dX, s);
}

hipError_t launch_supcon_bwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, const float* lse, const float* invcnt, int Na, int N, int D,
                             float inv_temp, float w, const float* gscale, float* dA, float* dC, float* ws,
                             hipStream_t s) {
  SupconParams p{};
  p.gscale = gscale;
  p.a_self = a_self; p.a_key = a_key; p.c_key = c_key; p.lse = lse; p.invcnt = invcnt;
  p.inv_temp = inv_temp; p.w = w;
  // dA: own = anchors, other = contrasts
  p.own = A; p.other = C; p.n_own = Na; p.n_other = N;
  p.n_split = bwd_splits(Na, N, &p.other_per_split);
  float* ws_a = ws;
  p.out = p.n_split > 1 ? ws_a : dA;
  hipError_t e = launch_mode<MODE_BWD_A>(D, p, s);
  if (e != hipSuccess) return e;
  if (p.n_split > 1 && (e = split_reduce(ws_a, p.n_split, (long)Na * D, dA, s)) != hipSuccess) return e;
  float* ws_c = ws + (p.n_split > 1 ? (long)p.n_split * Na * D : 0);
  // dC: own = contrasts, other = anchors
  p.own = C; p.other = A; p.n_own = N; p.n_other = Na;
  p.n_split = bwd_splits(N, Na, &p.other_per_split);
  p.out = p.n_split > 1 ? ws_c : dC;
  e = launch_mode<MODE_BWD_C>(D, p, s);
  if (e != hipSuccess) return e;
  if (p.n_split > 1) return split_reduce(ws_c, p.n_split, (long)N * D, dC, s);
  return hipSuccess;
}
