// C++ launcher declarations shared by the HIP kernel translation units and the
// torch binding layer. Launchers take raw device pointers plus the caller's HIP
// stream and never allocate or synchronise, so every one of them is safe to capture
// into a hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// ---- selftest -------------------------------------------------------------------
hipError_t launch_mfma16_selftest(const void* A, const void* B, float* C, hipStream_t s);

// ---- fused SupCon / NT-Xent loss (supcon.hip) ---------------------------------
int supcon_num_splits(int n_own, int n_other);
hipError_t launch_supcon_fwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, int Na, int N, int D, float inv_temp, float temp_ratio,
                             float scale, int n_split, float* part, float* lse, float* invcnt,
                             float* row_loss, float* loss, hipStream_t s);
hipError_t launch_supcon_bwd(const float* A, const float* C, const int* a_self, const int* a_key,
                             const int* c_key, const float* lse, const float* invcnt, int Na, int N, int D,
                             float inv_temp, float w, const float* gscale, float* dA, float* dC,
                             hipStream_t s);
