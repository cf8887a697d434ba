// Per-channel BatchNorm epilogues shared by the stand-alone BN kernels and the single-launch
// column reduction (bn.hip): forward finalize (affine + running statistics) and backward
// coefficients (+ dγ/dβ into the gradient sinks).
#pragma once
#include "launchers.h"

namespace sdx {
// ---- per-channel epilogues (shared by the stand-alone kernels and the fused reduction) ----
// (Σy, Σy²) over `count` rows -> scale/shift, mean/invstd (for backward), running stats
// (unbiased variance, as torch BatchNorm2d)
__device__ __forceinline__ void bn_finalize_one(int c, double s1, double s2, const BnFinalizeArgs& a) {
  const double mean = s1 / a.count;
  double var = s2 / a.count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
  const float g = a.gamma ? a.gamma[c] : 1.f;
  const float b = a.beta ? a.beta[c] : 0.f;
  a.scale[c] = g * invstd;
  a.shift[c] = b - (float)mean * g * invstd;
  a.mean[c] = (float)mean;
  a.invstd[c] = invstd;
  if (a.update_running) {
    const double unbiased = a.count > 1.0 ? var * a.count / (a.count - 1.0) : var;
    a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * (float)mean;
    a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * (float)unbiased;
  }
}

// sums: Σdz, Σdz·(ya−μa) [, Σdz·(yb−μb)] -> per-channel dy = A·dz + D·y + E and dγ/dβ
// (accumulated into the parameter-gradient sinks when a.accumulate)
__device__ __forceinline__ void bn_coef_one(int c, int C, const double* s, int nsets, const BnCoefArgs& a) {
  const double sdz = s[0];
  for (int set = 0; set < nsets; ++set) {
    const float* gg = set == 0 ? a.g_a : a.g_b;
    const float* mm = set == 0 ? a.mean_a : a.mean_b;
    const float* iv = set == 0 ? a.inv_a : a.inv_b;
    float* coef = set == 0 ? a.coef_a : a.coef_b;
    const double sdzy = s[1 + set];
    const double inv = iv[c], mu = mm[c], gam = gg ? gg[c] : 1.0;
    const double A = gam * inv;
    const double m1 = sdz / a.count, m2 = sdzy / a.count;
    const double D = -A * inv * inv * m2;
    const double E = -A * m1 - D * mu;
    coef[c] = (float)A;
    coef[C + c] = (float)D;
    coef[2 * C + c] = (float)E;
    float* dg = set == 0 ? a.dgamma_a : a.dgamma_b;
    float* db = set == 0 ? a.dbeta_a : a.dbeta_b;
    if (dg) dg[c] = (float)(sdzy * inv * a.grad_scale) + (a.accumulate ? dg[c] : 0.f);
    if (db) db[c] = (float)(sdz * a.grad_scale) + (a.accumulate ? db[c] : 0.f);
  }
}

}  // namespace sdx
