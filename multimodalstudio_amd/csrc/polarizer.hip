// PolarizationHead Stokes post-processing (one wave per ray, lane = sample):
//   s0 <- leaky_relu(s0)                                   field_heads.py:103
//   n = normalize(d x z), theta = acos(clamp(n . up, +-(1 - 1e-4))) - pi/2   polarizer.py:54-79
//   a = R(theta) s, R = [[1,0,0],[0,c,s],[0,-s,c]], c = cos 2theta, s = sin 2theta   polarizer.py:38-52, :81
//   I = 0.5 [[1,1,0],[1,0,1],[1,-1,0],[1,0,-1]] a            polarizer.py:84-101
// (paths under /root/reference/src/.)  Backward returns d stokes and accumulates d dirs, d ups.
#include "common.h"

namespace {

struct PolGeom {
  float n0, n1, n2, cost, c, s;
  bool clamped;
  float nraw;
};

__device__ __forceinline__ PolGeom pol_geom(const float* d, const float* up) {
  PolGeom g;
  const float x0 = d[1], x1 = -d[0], x2 = 0.0f;  // d x (0, 0, 1)
  const float nn = sqrtf(x0 * x0 + x1 * x1 + x2 * x2);
  g.nraw = nn;
  const float dn = fmaxf(nn, 1e-12f);
  g.n0 = x0 / dn; g.n1 = x1 / dn; g.n2 = x2 / dn;
  const float ct = g.n0 * up[0] + g.n1 * up[1] + g.n2 * up[2];
  g.clamped = !(ct >= -1.0f + 1e-4f && ct <= 1.0f - 1e-4f);
  g.cost = fminf(fmaxf(ct, -1.0f + 1e-4f), 1.0f - 1e-4f);
  const float theta = acosf(g.cost) - 1.57079632679489661923f;
  g.c = cosf(2.0f * theta);
  g.s = sinf(2.0f * theta);
  return g;
}

__global__ void polarizer_fwd_kernel(const float* __restrict__ stokes, const float* __restrict__ dirs,
                                     const float* __restrict__ ups, int64_t M, int S, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ray = i / S;
    const PolGeom g = pol_geom(dirs + ray * 3, ups + ray * 3);
    const float s0r = stokes[i * 3], s1 = stokes[i * 3 + 1], s2 = stokes[i * 3 + 2];
    const float a0 = s0r > 0.f ? s0r : 0.01f * s0r;
    const float a1 = g.c * s1 + g.s * s2;
    const float a2 = -g.s * s1 + g.c * s2;
    out[i * 4] = 0.5f * a0 + 0.5f * a1;
    out[i * 4 + 1] = 0.5f * a0 + 0.5f * a2;
    out[i * 4 + 2] = 0.5f * a0 - 0.5f * a1;
    out[i * 4 + 3] = 0.5f * a0 - 0.5f * a2;
  }
}

__global__ __launch_bounds__(256) void polarizer_bwd_kernel(const float* __restrict__ stokes,
                                                            const float* __restrict__ dirs,
                                                            const float* __restrict__ ups, int64_t R, int S,
                                                            const float* __restrict__ dout,
                                                            float* __restrict__ dstokes, float* __restrict__ ddirs,
                                                            float* __restrict__ dups) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const float* d = dirs + ray * 3;
  const float* up = ups + ray * 3;
  const PolGeom g = pol_geom(d, up);
  float gd0 = 0.f, gd1 = 0.f, gu0 = 0.f, gu1 = 0.f, gu2 = 0.f;
  for (int k = lane; k < S; k += 64) {
    const int64_t i = ray * S + k;
    const float s0r = stokes[i * 3], s1 = stokes[i * 3 + 1], s2 = stokes[i * 3 + 2];
    const float* dI = dout + i * 4;
    const float da0 = 0.5f * (dI[0] + dI[1] + dI[2] + dI[3]);
    const float da1 = 0.5f * (dI[0] - dI[2]);
    const float da2 = 0.5f * (dI[1] - dI[3]);
    dstokes[i * 3] = da0 * (s0r > 0.f ? 1.0f : 0.01f);
    dstokes[i * 3 + 1] = g.c * da1 - g.s * da2;
    dstokes[i * 3 + 2] = g.s * da1 + g.c * da2;
    const float dtheta = da1 * (-2.0f * g.s * s1 + 2.0f * g.c * s2) + da2 * (-2.0f * g.c * s1 - 2.0f * g.s * s2);
    float dcos = g.clamped ? 0.f : -dtheta / sqrtf(1.0f - g.cost * g.cost);
    // cos = n . up
    gu0 += dcos * g.n0; gu1 += dcos * g.n1; gu2 += dcos * g.n2;
    const float dn0 = dcos * up[0], dn1 = dcos * up[1], dn2 = dcos * up[2];
    // normalize backward (x = (d1, -d0, 0))
    float dx0, dx1;
    if (g.nraw > 1e-12f) {
      const float dot = dn0 * g.n0 + dn1 * g.n1 + dn2 * g.n2;
      dx0 = (dn0 - dot * g.n0) / g.nraw;
      dx1 = (dn1 - dot * g.n1) / g.nraw;
    } else {
      dx0 = dn0 / 1e-12f;
      dx1 = dn1 / 1e-12f;
    }
    gd1 += dx0;   // x0 = d1
    gd0 -= dx1;   // x1 = -d0
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    gd0 += __shfl_xor(gd0, o); gd1 += __shfl_xor(gd1, o);
    gu0 += __shfl_xor(gu0, o); gu1 += __shfl_xor(gu1, o); gu2 += __shfl_xor(gu2, o);
  }
  if (lane == 0) {
    if (ddirs) { ddirs[ray * 3] += gd0; ddirs[ray * 3 + 1] += gd1; }
    if (dups) { dups[ray * 3] += gu0; dups[ray * 3 + 1] += gu1; dups[ray * 3 + 2] += gu2; }
  }
}

}  // namespace

MMS_EXPORT int mms_polarizer_fwd(const float* stokes, const float* dirs, const float* ups, int64_t M, int S,
                                 float* out, void* stream) {
  const char* fn = "mms_polarizer_fwd";
  if (M == 0) return 0;
  hipLaunchKernelGGL(polarizer_fwd_kernel, dim3(mms::grid_for(M, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                     stokes, dirs, ups, M, S, out);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_polarizer_bwd(const float* stokes, const float* dirs, const float* ups, int64_t R, int S,
                                 const float* dout, float* dstokes, float* ddirs, float* dups, void* stream) {
  const char* fn = "mms_polarizer_bwd";
  if (R == 0) return 0;
  hipLaunchKernelGGL(polarizer_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), stokes, dirs, ups, R, S, dout, dstokes, ddirs, dups);
  return mms::check_launch(fn);
}
