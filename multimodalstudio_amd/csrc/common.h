// Shared helpers for the MMS MI355X (gfx950) HIP kernels.
//
// Every kernel in this library is reached through an `extern "C"` entry point declared in
// include/mms_hip.h.  Entry points take plain device pointers + sizes + a hipStream_t (passed
// as void*), never synchronise, never allocate, and return 0 on success or a negative status
// whose text is available from mms_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

// The public declarations: every entry point's definition is checked against its header prototype by the
// compiler (a parameter-list drift between header and definition is a "conflicting declaration" error, so the
// ctypes argtypes _lib.py derives from the header always match the code).
#include "mms_hip.h"

#define MMS_EXPORT extern "C" __attribute__((visibility("default")))

namespace mms {

// Thread-local error text (re-entrant: one buffer per host thread).
inline char* err_buf() {
  static thread_local char buf[512];
  return buf;
}

inline int set_error(const char* fn, const char* msg) {
  snprintf(err_buf(), 512, "%s: %s", fn, msg);
  return -1;
}

inline int check_launch(const char* fn) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(err_buf(), 512, "%s: launch failed: %s", fn, hipGetErrorString(e));
    return -2;
  }
  return 0;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned grid_for(int64_t n, int block, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// torch.exp / torch.sigmoid as the reference's CPU build evaluates them, bit for bit: ATen's vectorised float
// sigmoid is reciprocal(1 + exp(0 - x)) with Vectorized<float>::exp = SLEEF's expf_u10 (Cody-Waite reduction
// by ln2 in two FMA steps, degree-6 polynomial in FMA Horner form, ldexp in two halves).  Checked against
// torch.sigmoid on 2e7 floats in [-90, 90] and N(0, 30): 0 mismatches (tests/test_oracle_golden.py pins the
// host restatement).  The NeuS sampler needs it: its searchsorted indices and bins are compared bit-exactly
// with the reference (ray_samplers.py:545-546).
__device__ __forceinline__ float pow2i_(int q) { return __int_as_float((q + 0x7f) << 23); }

__device__ __forceinline__ float sleef_expf_u10(float d) {
#pragma clang fp contract(off)
  const int q = (int)__builtin_rintf(d * 1.442695040888963407359924681001892137426645954152985934135449406931f);
  const float qf = (float)q;
  float s = __builtin_fmaf(qf, -0.693145751953125f, d);
  s = __builtin_fmaf(qf, -1.428606765330187045e-06f, s);
  float u = 0.000198527617612853646278381f;
  u = __builtin_fmaf(u, s, 0.00139304355252534151077271f);
  u = __builtin_fmaf(u, s, 0.00833336077630519866943359f);
  u = __builtin_fmaf(u, s, 0.0416664853692054748535156f);
  u = __builtin_fmaf(u, s, 0.166666671633720397949219f);
  u = __builtin_fmaf(u, s, 0.5f);
  u = 1.0f + __builtin_fmaf(s * s, u, s);
  const int q1 = q >> 1;
  u = u * pow2i_(q1);
  u = u * pow2i_(q - q1);
  if (d < -104.f) u = 0.f;
  if (d > 100.f) u = __builtin_inff();
  return u;
}

__device__ __forceinline__ float torch_cpu_sigmoid(float x) { return 1.0f / (1.0f + sleef_expf_u10(0.0f - x)); }

// torch.sum(x[0:n]) of a contiguous float row as ATen's CPU reduction orders it (SumKernel.cpp cascade_sum ->
// vectorized_inner_sum with 8-wide vectors, row_sum's 4 ILP partials, scalar tail first, then the 8 partial lanes):
// matches torch.sum over dim=-1 bit for bit for rows of 33..65 elements (checked in this container).  n < 8 rows
// take ATen's scalar path, a plain sequential sum.
__device__ __forceinline__ float torch_cpu_row_sum(const float* x, int n) {
#pragma clang fp contract(off)
  if (n < 8) {
    float s = 0.f;
    for (int k = 0; k < n; ++k) s = s + x[k];
    return s;
  }
  float P[4][8];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int l = 0; l < 8; ++l) P[k][l] = 0.f;
  const int V = n >> 3, nI = V >> 2;
  for (int i = 0; i < nI; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < 8; ++l) P[k][l] = P[k][l] + x[8 * (4 * i + k) + l];
  for (int i = 4 * nI; i < V; ++i)
#pragma unroll
    for (int l = 0; l < 8; ++l) P[0][l] = P[0][l] + x[8 * i + l];
#pragma unroll
  for (int k = 1; k < 4; ++k)
#pragma unroll
    for (int l = 0; l < 8; ++l) P[0][l] = P[0][l] + P[k][l];
  float fin = 0.f;
  for (int k = 8 * V; k < n; ++k) fin = fin + x[k];
#pragma unroll
  for (int l = 0; l < 8; ++l) fin = fin + P[0][l];
  return fin;
}

// MLP activations for GEMM epilogues (ids: 0 none, 1 ReLU, 2 Softplus(beta, threshold), 3 Sigmoid; derivative-only
// id 4: Sigmoid' evaluated from the forward OUTPUT, so the forward stores no pre-activation -- ReLU' is the same from
// either side, id 1).
// Built on the hardware transcendentals (v_exp_f32 = 2^x, v_log_f32 = log2, v_rcp_f32; ~1 ulp): the
// accurate libm log1pf/expf forms cost ~150 VALU ops per element, which made the epilogue of a 270k x 256
// layer compute-bound (~250 us).  Softplus(x) = ln2 * log2(1 + 2^(beta x log2 e)) / beta, exact to ~1e-7
// relative where it matters; for beta x < -17 it returns 0 instead of e^(beta x)/beta (< 4e-10 absolute).
__device__ __forceinline__ float act_fwd_fast(int act, float v, float beta, float thr) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: {
      const float bx = v * beta;
      if (bx > thr) return v;
      const float e = __builtin_amdgcn_exp2f(bx * 1.4426950408889634f);
      return __builtin_amdgcn_logf(1.0f + e) * (0.6931471805599453f * __builtin_amdgcn_rcpf(beta));
    }
    case 3: return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
    default: return v;
  }
}

// accurate libm forms (the fp32 parity mode): torch CPU's softplus / sigmoid expressions
__device__ __forceinline__ float act_fwd_exact(int act, float v, float beta, float thr) {
  switch (act) {
    case 1: return v > 0.f ? v : 0.f;
    case 2: { const float bx = v * beta; return bx > thr ? v : log1pf(expf(bx)) / beta; }
    case 3: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ float act_grad_exact(int act, float z, float beta, float thr) {
  switch (act) {
    case 1: return z > 0.f ? 1.f : 0.f;
    case 2: { const float bx = z * beta; if (bx > thr) return 1.f; const float e = expf(bx); return e / (e + 1.0f); }
    case 3: { const float s = 1.0f / (1.0f + expf(-z)); return s * (1.0f - s); }
    case 4: return z * (1.0f - z);  // Sigmoid' from the layer OUTPUT y (torch's sigmoid_backward form)
    default: return 1.f;
  }
}

// d act / d x evaluated at the pre-activation z
__device__ __forceinline__ float act_grad_fast(int act, float z, float beta, float thr) {
  switch (act) {
    case 1: return z > 0.f ? 1.f : 0.f;
    case 2: {
      const float bx = z * beta;
      if (bx > thr) return 1.f;
      return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-bx * 1.4426950408889634f));
    }
    case 3: {
      const float s = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * 1.4426950408889634f));
      return s * (1.0f - s);
    }
    case 4: return z * (1.0f - z);  // Sigmoid' from the layer OUTPUT y
    default: return 1.f;
  }
}

}  // namespace mms

#define MMS_REQUIRE(cond, fn, msg) \
  do {                             \
    if (!(cond)) return mms::set_error(fn, msg); \
  } while (0)
