// Ray generation (pinhole + OpenCV undistortion + pose refinement) and the sphere collider.
//
// Reference (paths under /root/reference/src):
//   RayGenerator.forward                model_components/ray_generators.py:54-81
//   Cameras._generate_rays_from_coords  cameras/cameras.py:460-703 (perspective cameras)
//   radial_and_tangential_undistort     cameras/camera_utils.py:280-383 (params read [k1,k2,k3,k4,p1,p2])
//   pose_utils.multiply                 utils/poses.py:53-67   (c2w o camera_opt_to_camera)
//   SphereCollider.forward              model_components/scene_colliders.py:60-80
//   update_ray_bundles_for_background   model_components/scene_colliders.py:107-113
// The SO(3)xR^3 exponential map of the (1 x 6) pose delta is O(1) work and stays in PyTorch autograd on
// the host side; these kernels take the resulting 3x4 matrices and return dL/dmatrix (atomics).
#include "common.h"

#pragma clang fp contract(off)

namespace {

__device__ void undistort(float& x, float& y, const float* dp) {
  const float xd = x, yd = y;
  const float k1 = dp[0], k2 = dp[1], k3 = dp[2], k4 = dp[3], p1 = dp[4], p2 = dp[5];
  for (int it = 0; it < 10; ++it) {
    const float r = x * x + y * y;
    const float d = 1.0f + r * (k1 + r * (k2 + r * (k3 + r * k4)));
    const float fx = d * x + 2 * p1 * x * y + p2 * (r + 2 * x * x) - xd;
    const float fy = d * y + 2 * p2 * x * y + p1 * (r + 2 * y * y) - yd;
    const float d_r = k1 + r * (2.0f * k2 + r * (3.0f * k3 + r * 4.0f * k4));
    const float d_x = 2.0f * x * d_r;
    const float d_y = 2.0f * y * d_r;
    const float fx_x = d + d_x * x + 2.0f * p1 * y + 6.0f * p2 * x;
    const float fx_y = d_y * x + 2.0f * p1 * x + 2.0f * p2 * y;
    const float fy_x = d_x * y + 2.0f * p2 * y + 2.0f * p1 * x;
    const float fy_y = d + d_y * y + 2.0f * p2 * x + 6.0f * p1 * y;
    const float den = fy_x * fx_y - fx_x * fy_y;
    const float xn = fx * fy_y - fy * fx_y;
    const float yn = fy * fx_x - fx * fy_x;
    const bool ok = fabsf(den) > 1e-3f;
    x = x + (ok ? xn / den : 0.0f);
    y = y + (ok ? yn / den : 0.0f);
  }
}

struct Pose {
  float R[3][3];
  float t[3];
};

// c2w o mat (poses.py:53-67): R = R1 R2, t = t1 + R1 t2
__device__ __forceinline__ Pose compose(const float* c2w, const float* mat) {
  Pose P;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) {
      float s = c2w[i * 4 + 0] * mat[0 * 4 + j];
      s = s + c2w[i * 4 + 1] * mat[1 * 4 + j];
      s = s + c2w[i * 4 + 2] * mat[2 * 4 + j];
      P.R[i][j] = s;
    }
    float s = c2w[i * 4 + 0] * mat[0 * 4 + 3];
    s = s + c2w[i * 4 + 1] * mat[1 * 4 + 3];
    s = s + c2w[i * 4 + 2] * mat[2 * 4 + 3];
    P.t[i] = c2w[i * 4 + 3] + s;
  }
  return P;
}

__device__ __forceinline__ void cam_coords(int xi, int yi, float off, float fx, float fy, float cx, float cy,
                                           const float* dp, float u[3], float v[3]) {
  const float x = (float)xi + off, y = (float)yi + off;
  u[0] = (x - cx) / fx;       v[0] = -(y - cy) / fy;
  u[1] = (x - cx + 1) / fx;   v[1] = -(y - cy) / fy;
  u[2] = (x - cx) / fx;       v[2] = -(y - cy + 1) / fy;
  if (dp) {
    for (int s = 0; s < 3; ++s) undistort(u[s], v[s], dp);
  }
}

__device__ __forceinline__ void rotate(const Pose& P, float u, float v, float o[3]) {
  for (int i = 0; i < 3; ++i) {
    float s = u * P.R[i][0];
    s = s + v * P.R[i][1];
    s = s + (-1.0f) * P.R[i][2];
    o[i] = s;
  }
}

// the normalised ray direction of camera-plane point (u, v) under pose P (returns the norm before normalising)
__device__ __forceinline__ float unit_dir(const Pose& P, float u, float v, float* w) {
  float o[3];
  rotate(P, u, v, o);
  const float n = sqrtf(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
  const float dn = fmaxf(n, 1e-12f);
  for (int i = 0; i < 3; ++i) w[i] = o[i] / dn;
  return n;
}

__global__ void raygen_fwd_kernel(const int* __restrict__ coords, int64_t N, const float* __restrict__ fxs,
                                  const float* __restrict__ fys, const float* __restrict__ cxs,
                                  const float* __restrict__ cys, const float* __restrict__ c2w,
                                  const float* __restrict__ dist, const float* __restrict__ mats, int mat_per_cam,
                                  float off, float* __restrict__ origins, float* __restrict__ dirs,
                                  float* __restrict__ ups, float* __restrict__ area, float* __restrict__ dnorm) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
    const int c = coords[r * 3], yi = coords[r * 3 + 1], xi = coords[r * 3 + 2];
    float u[3], v[3];
    cam_coords(xi, yi, off, fxs[c], fys[c], cxs[c], cys[c], dist ? dist + c * 6 : nullptr, u, v);
    const Pose P = compose(c2w + c * 12, mats + (mat_per_cam ? c * 12 : 0));
    float w[3][3];
    for (int s = 0; s < 3; ++s) {
      const float n = unit_dir(P, u[s], v[s], w[s]);
      if (s == 0 && dnorm) dnorm[r] = n;
    }
    for (int i = 0; i < 3; ++i) {
      dirs[r * 3 + i] = w[0][i];
      origins[r * 3 + i] = P.t[i];
      if (ups) ups[r * 3 + i] = P.R[i][1];
    }
    if (area) {
      float ax = 0.f, ay = 0.f;
      for (int i = 0; i < 3; ++i) {
        const float a = w[0][i] - w[1][i], b = w[0][i] - w[2][i];
        ax = ax + a * a;
        ay = ay + b * b;
      }
      area[r] = sqrtf(ax) * sqrtf(ay);
    }
  }
}

// dL/dmat (accumulated with atomics; per camera when mat_per_cam, else one shared matrix)
__global__ __launch_bounds__(256) void raygen_bwd_kernel(const int* __restrict__ coords, int64_t N,
                                                         const float* __restrict__ fxs, const float* __restrict__ fys,
                                                         const float* __restrict__ cxs, const float* __restrict__ cys,
                                                         const float* __restrict__ c2w,
                                                         const float* __restrict__ dist,
                                                         const float* __restrict__ mats, int mat_per_cam, float off,
                                                         const float* __restrict__ dorig,
                                                         const float* __restrict__ ddirs,
                                                         const float* __restrict__ dups, float* __restrict__ dmats) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float g[12];
  for (int k = 0; k < 12; ++k) g[k] = 0.f;
  int cam = 0;
  if (r < N) {
    const int c = coords[r * 3], yi = coords[r * 3 + 1], xi = coords[r * 3 + 2];
    cam = c;
    float u[3], v[3];
    cam_coords(xi, yi, off, fxs[c], fys[c], cxs[c], cys[c], dist ? dist + c * 6 : nullptr, u, v);
    const float* A = c2w + c * 12;
    const Pose P = compose(A, mats + (mat_per_cam ? c * 12 : 0));
    float dR[3][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
    float dt[3] = {0.f, 0.f, 0.f};
    if (ddirs) {
      float o[3];
      rotate(P, u[0], v[0], o);
      const float n = sqrtf(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
      const float gd[3] = {ddirs[r * 3], ddirs[r * 3 + 1], ddirs[r * 3 + 2]};
      float dv[3];
      if (n > 1e-12f) {
        const float dot = (gd[0] * o[0] + gd[1] * o[1] + gd[2] * o[2]) / (n * n);
        for (int i = 0; i < 3; ++i) dv[i] = (gd[i] - dot * o[i]) / n;
      } else {
        for (int i = 0; i < 3; ++i) dv[i] = gd[i] / 1e-12f;
      }
      const float dc[3] = {u[0], v[0], -1.0f};
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) dR[i][j] += dv[i] * dc[j];
    }
    if (dups) {
      for (int i = 0; i < 3; ++i) dR[i][1] += dups[r * 3 + i];
    }
    if (dorig) {
      for (int i = 0; i < 3; ++i) dt[i] = dorig[r * 3 + i];
    }
    // R = A_R M_R -> dM_R = A_R^T dR ; t = A_t + A_R M_t -> dM_t = A_R^T dt
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) {
        g[i * 4 + j] = A[0 * 4 + i] * dR[0][j] + A[1 * 4 + i] * dR[1][j] + A[2 * 4 + i] * dR[2][j];
      }
      g[i * 4 + 3] = A[0 * 4 + i] * dt[0] + A[1 * 4 + i] * dt[1] + A[2 * 4 + i] * dt[2];
    }
  }
  if (mat_per_cam) {
    if (r < N)
      for (int k = 0; k < 12; ++k) atomicAdd(dmats + cam * 12 + k, g[k]);
    return;
  }
  // shared: reduce the block, 12 atomics per block
  __shared__ float red[4][12];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < 12; ++k) {
    float s = g[k];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < 12) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(dmats + threadIdx.x, s);
  }
}

// ------------------------------------------------------------------ collider
// the sphere collider's (d . o, ||o||^2-term discriminant) of one ray -- shared by the collider and the fused hit
// count (mms_count_hits), so both decide hits bit-identically
__device__ __forceinline__ float sphere_under(const float* o, const float* d, float radius, float& dot) {
  dot = d[0] * o[0];
  dot = dot + d[1] * o[1];
  dot = dot + d[2] * o[2];
  // origins.norm(p=2): ATen's CPU norm accumulates the squares with FMAs (bit-exact to torch.norm)
  const float on = sqrtf(__builtin_fmaf(o[2], o[2], __builtin_fmaf(o[1], o[1], o[0] * o[0])));
  return dot * dot - (on * on - radius * radius);
}

__global__ void collider_fwd_kernel(const float* __restrict__ origins, const float* __restrict__ dirs, int64_t N,
                                    float radius, float* __restrict__ nears, float* __restrict__ fars,
                                    unsigned char* __restrict__ mask, float* __restrict__ bg_nears,
                                    float* __restrict__ bg_fars) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
    const float* o = origins + r * 3;
    const float* d = dirs + r * 3;
    float dot;
    const float under = sphere_under(o, d, radius, dot);
    const bool hit = under > 0.01f;
    const float sq = sqrtf(fmaxf(under, 0.01f));
    const float nr = fmaxf(sq * -1.0f - dot, 0.01f);
    const float fr = fmaxf(sq * 1.0f - dot, 0.01f);
    nears[r] = nr;
    fars[r] = fr;
    mask[r] = hit ? 1 : 0;
    if (bg_nears) bg_nears[r] = hit ? fr : nr;
    if (bg_fars) bg_fars[r] = fr + 3.0f;
  }
}

// d near / d far (full-length [N] arrays, may be null) -> d origins, d dirs (accumulate)
__global__ void collider_bwd_kernel(const float* __restrict__ origins, const float* __restrict__ dirs, int64_t N,
                                    float radius, const float* __restrict__ dnears, const float* __restrict__ dfars,
                                    const float* __restrict__ dbg_nears, const float* __restrict__ dbg_fars,
                                    float* __restrict__ dorig, float* __restrict__ ddirs) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
    const float* o = origins + r * 3;
    const float* d = dirs + r * 3;
    float dot = d[0] * o[0];
    dot = dot + d[1] * o[1];
    dot = dot + d[2] * o[2];
    // origins.norm(p=2): ATen's CPU norm accumulates the squares with FMAs (bit-exact to torch.norm)
    const float on = sqrtf(__builtin_fmaf(o[2], o[2], __builtin_fmaf(o[1], o[1], o[0] * o[0])));
    const float under = dot * dot - (on * on - radius * radius);
    const bool hit = under > 0.01f;
    const float sq = sqrtf(fmaxf(under, 0.01f));
    const float nraw = sq * -1.0f - dot, fraw = sq * 1.0f - dot;
    float dn = dnears ? dnears[r] : 0.f;
    float df = dfars ? dfars[r] : 0.f;
    if (dbg_nears) { if (hit) df += dbg_nears[r]; else dn += dbg_nears[r]; }
    if (dbg_fars) df += dbg_fars[r];
    if (!(nraw >= 0.01f)) dn = 0.f;
    if (!(fraw >= 0.01f)) df = 0.f;
    const float dsq = -dn + df;
    float ddot = -dn - df;
    float dunder = (under >= 0.01f) ? dsq * 0.5f / sq : 0.f;
    ddot += 2.0f * dot * dunder;
    const float don = -2.0f * on * dunder;
    for (int c = 0; c < 3; ++c) {
      float go = ddot * d[c];
      if (on > 0.f) go += don * o[c] / on;
      dorig[r * 3 + c] += go;
      ddirs[r * 3 + c] += ddot * o[c];
    }
  }
}

// order-preserving compaction of mask -> idx (int64), count; single block, chunked scan
__global__ __launch_bounds__(1024) void compact_kernel(const unsigned char* __restrict__ mask, int64_t N,
                                                       int64_t* __restrict__ idx, int64_t* __restrict__ count) {
  __shared__ int64_t base;
  __shared__ int wsum[16];
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t start = 0; start < N; start += blockDim.x) {
    const int64_t i = start + threadIdx.x;
    const int f = (i < N && mask[i]) ? 1 : 0;
    const unsigned long long bal = __ballot(f);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (f) idx[base + off + pre] = i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += wsum[k];
      base += tot;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) count[0] = base;
}

// fixed-capacity variant for static-shape (graph-captured) steps: after the compaction above, rows
// [count, cap) are padding -- gather index = first hit (or 0: always a valid row), scatter index = N
// (a dummy row one past the real ones).  Work on padding rows is discarded (their loss weight is zero).
__global__ __launch_bounds__(1024) void compact_pad_kernel(int64_t N, int64_t cap, int64_t* __restrict__ idx,
                                                           int64_t* __restrict__ sidx,
                                                           int64_t* __restrict__ count) {
  const int64_t c = count[0] < cap ? count[0] : cap;
  const int64_t pad = c > 0 ? idx[0] : 0;
  __syncthreads();
  if (threadIdx.x == 0) count[0] = c;  // consumers read the clamped count
  for (int64_t i = threadIdx.x; i < cap; i += blockDim.x) {
    if (sidx) sidx[i] = i < c ? idx[i] : N;
    if (i >= c) idx[i] = pad;
  }
}

// Every modality's hit rays in one launch (BaseModel batches all modalities through the shared fields): block m
// compacts segment m = rays [m N, (m + 1) N) of the concatenated batch (order-preserving, as base_model.py:88-93 per
// modality) into scratch row m, then lays out `cap` rows per segment: gidx = global ray index of the hit (rows past
// the segment's hit count repeat its first hit, or its first ray when nothing hit: always a valid row), sidx =
// the hit's index within its modality (N for padding rows: the dummy row one past the modality's rays), count =
// min(hits, cap).
__global__ __launch_bounds__(1024) void compact_segments_kernel(const unsigned char* __restrict__ mask, int64_t N,
                                                                int64_t cap, int64_t* __restrict__ scratch,
                                                                int64_t* __restrict__ gidx,
                                                                int64_t* __restrict__ sidx,
                                                                int64_t* __restrict__ count) {
  __shared__ int64_t base;
  __shared__ int wsum[16];
  const int64_t seg = blockIdx.x;
  const int64_t g0 = seg * N;
  if (threadIdx.x == 0) base = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t start = 0; start < N; start += blockDim.x) {
    const int64_t i = start + threadIdx.x;
    const int f = (i < N && mask[g0 + i]) ? 1 : 0;
    const unsigned long long bal = __ballot(f);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += wsum[k];
    if (f) scratch[g0 + base + off + pre] = g0 + i;
    __syncthreads();
    if (threadIdx.x == 0) {
      int tot = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += wsum[k];
      base += tot;
    }
    __syncthreads();
  }
  __threadfence_block();
  __syncthreads();
  const int64_t c = base < cap ? base : cap;
  const int64_t pad = c > 0 ? scratch[g0] : g0;
  for (int64_t i = threadIdx.x; i < cap; i += blockDim.x) {
    const int64_t gi = i < c ? scratch[g0 + i] : pad;
    gidx[seg * cap + i] = gi;
    if (sidx) sidx[seg * cap + i] = i < c ? gi - g0 : N;
  }
  if (threadIdx.x == 0) count[seg] = c;
}

// ---- SO(3) x R^3 exponential map of the pose deltas (lie_groups.py:28-63): thread per camera delta.
// R = I + f1 K + f2 K^2 with K = skew(w), theta = sqrt(max(|w|^2, 1e-4)), f1 = sin(theta) / theta,
// f2 = (1 - cos(theta)) / theta^2; the translation column is t.  Same float operation order as the reference's
// torch expression (fac1 * K + fac2 * K K) + I.
struct Skew {
  float k[3][3];
};

__device__ __forceinline__ Skew skew_of(const float* w) {
  Skew s;
  s.k[0][0] = 0.f;   s.k[0][1] = -w[2]; s.k[0][2] = w[1];
  s.k[1][0] = w[2];  s.k[1][1] = 0.f;   s.k[1][2] = -w[0];
  s.k[2][0] = -w[1]; s.k[2][1] = w[0];  s.k[2][2] = 0.f;
  return s;
}

__device__ __forceinline__ void pose_exp_one(const float* __restrict__ tv, float* __restrict__ o) {
  const float w[3] = {tv[3], tv[4], tv[5]};
  const float nrm = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const float ang = sqrtf(fmaxf(nrm, 1e-4f));
  const float inv = 1.0f / ang;
  const float f1 = inv * sinf(ang);
  const float f2 = inv * inv * (1.0f - cosf(ang));
  const Skew K = skew_of(w);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float k2 = K.k[i][0] * K.k[0][j] + K.k[i][1] * K.k[1][j] + K.k[i][2] * K.k[2][j];
      o[4 * i + j] = (f1 * K.k[i][j] + f2 * k2) + (i == j ? 1.f : 0.f);
    }
    o[4 * i + 3] = tv[i];
  }
}

__global__ void pose_exp_fwd_kernel(const float* __restrict__ tangent, int64_t B, float* __restrict__ mats) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  pose_exp_one(tangent + 6 * b, mats + 12 * b);
}

// The next step's hit count in ONE launch (graphs.GraphTrainer's tail): pose exp map (or the given matrices; every block
// forms them in LDS), ray origin / direction and the sphere hit test of every ray, and the count added into count[0]
// (zeroed beforehand) -- the same device functions as pose_exp_fwd / raygen_fwd / collider_fwd + compact, so the
// count is the one the step's own compaction will find.  One ray per thread over the grid (a single block walking
// 2048 rays measured slower than the four launches it replaces).
constexpr int kCountMaxMats = 256;
__global__ __launch_bounds__(256) void count_hits_kernel(const int* __restrict__ coords, int64_t N,
                                                          const float* __restrict__ fxs, const float* __restrict__ fys,
                                                          const float* __restrict__ cxs, const float* __restrict__ cys,
                                                          const float* __restrict__ c2w, const float* __restrict__ dist,
                                                          const float* __restrict__ tangent,
                                                          const float* __restrict__ mats_in, int B, int mat_per_cam,
                                                          float off, float radius, int64_t* __restrict__ count) {
  __shared__ float smats[kCountMaxMats * 12];
  __shared__ int wsum[16];
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if (tangent != nullptr) {
      pose_exp_one(tangent + 6 * b, smats + 12 * b);
    } else {
      for (int k = 0; k < 12; ++k) smats[12 * b + k] = mats_in[12 * b + k];
    }
  }
  __syncthreads();
  int cnt = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (int64_t)gridDim.x * blockDim.x) {
    const int c = coords[r * 3], yi = coords[r * 3 + 1], xi = coords[r * 3 + 2];
    float u[3], v[3];
    cam_coords(xi, yi, off, fxs[c], fys[c], cxs[c], cys[c], dist ? dist + c * 6 : nullptr, u, v);
    const Pose P = compose(c2w + c * 12, smats + (mat_per_cam ? c * 12 : 0));
    float d[3];
    unit_dir(P, u[0], v[0], d);
    float dot;
    cnt += sphere_under(P.t, d, radius, dot) > 0.01f ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) tot += (unsigned long long)wsum[k];
    if (tot) atomicAdd(reinterpret_cast<unsigned long long*>(count), tot);
  }
}

// d tangent from d mats [B, 3, 4]: dt = dM[:, 3]; dK = f1 G + f2 (G K^T + K^T G), df1 = <G, K>, df2 = <G, K^2>,
// and through theta (only where |w|^2 > 1e-4: the clamp passes no gradient below it) dtheta / dw = w / theta.
__global__ void pose_exp_bwd_kernel(const float* __restrict__ tangent, const float* __restrict__ dmats, int64_t B,
                                    float* __restrict__ dtangent) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* tv = tangent + 6 * b;
  const float* g = dmats + 12 * b;
  const float w[3] = {tv[3], tv[4], tv[5]};
  const float nrm = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  const float ang = sqrtf(fmaxf(nrm, 1e-4f));
  const float inv = 1.0f / ang;
  const float sn = sinf(ang), cs = cosf(ang);
  const float f1 = inv * sn;
  const float f2 = inv * inv * (1.0f - cs);
  const Skew K = skew_of(w);
  float G[3][3], dK[3][3];
  float df1 = 0.f, df2 = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) G[i][j] = g[4 * i + j];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float k2 = K.k[i][0] * K.k[0][j] + K.k[i][1] * K.k[1][j] + K.k[i][2] * K.k[2][j];
      df1 += G[i][j] * K.k[i][j];
      df2 += G[i][j] * k2;
      // (G K^T + K^T G)_ij = sum_l G_il K_jl + K_li G_lj
      float s = 0.f;
#pragma unroll
      for (int l = 0; l < 3; ++l) s += G[i][l] * K.k[j][l] + K.k[l][i] * G[l][j];
      dK[i][j] = f1 * G[i][j] + f2 * s;
    }
  }
  float dw[3] = {dK[2][1] - dK[1][2], dK[0][2] - dK[2][0], dK[1][0] - dK[0][1]};
  if (nrm > 1e-4f) {
    const float df1da = cs * inv - sn * inv * inv;
    const float df2da = sn * inv * inv - 2.0f * (1.0f - cs) * inv * inv * inv;
    const float da = df1 * df1da + df2 * df2da;
#pragma unroll
    for (int k = 0; k < 3; ++k) dw[k] += da * w[k] * inv;
  }
  float* d = dtangent + 6 * b;   // accumulated: the pose parameter's own gradient buffer (functions.grad_target)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    d[i] += g[4 * i + 3];
    d[3 + i] += dw[i];
  }
}

// ---- hit-ray gather (TensorDataclass.__getitem__ with the collider mask, base_model.py:88-93): one thread per
// compacted ray copies (origins 3, directions 3, up 3, near 1, far 1) from row idx[r]; the backward scatter-adds the
// five gradients back (atomics: padding rows of a fixed-capacity batch repeat the first hit's index, with zero
// gradients).
__global__ void hit_gather_fwd_kernel(const int64_t* __restrict__ idx, int64_t R, const float* __restrict__ o,
                                      const float* __restrict__ d, const float* __restrict__ u,
                                      const float* __restrict__ n, const float* __restrict__ f, float* __restrict__ oh,
                                      float* __restrict__ dh, float* __restrict__ uh, float* __restrict__ nh,
                                      float* __restrict__ fh) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int64_t i = idx[r];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    oh[r * 3 + c] = o[i * 3 + c];
    dh[r * 3 + c] = d[i * 3 + c];
    uh[r * 3 + c] = u[i * 3 + c];
  }
  nh[r] = n[i];
  fh[r] = f[i];
}

__global__ void hit_gather_bwd_kernel(const int64_t* __restrict__ idx, int64_t R, const float* __restrict__ doh,
                                      const float* __restrict__ ddh, const float* __restrict__ duh,
                                      const float* __restrict__ dnh, const float* __restrict__ dfh,
                                      float* __restrict__ dO, float* __restrict__ dD, float* __restrict__ dU,
                                      float* __restrict__ dN, float* __restrict__ dF) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const int64_t i = idx[r];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (doh) atomicAdd(dO + i * 3 + c, doh[r * 3 + c]);
    if (ddh) atomicAdd(dD + i * 3 + c, ddh[r * 3 + c]);
    if (duh) atomicAdd(dU + i * 3 + c, duh[r * 3 + c]);
  }
  if (dnh) atomicAdd(dN + i, dnh[r]);
  if (dfh) atomicAdd(dF + i, dfh[r]);
}

}  // namespace

MMS_EXPORT int mms_hit_gather_fwd(const int64_t* idx, int64_t R, const float* o, const float* d, const float* u,
                                  const float* n, const float* f, float* oh, float* dh, float* uh, float* nh, float* fh,
                                  void* stream) {
  const char* fn = "mms_hit_gather_fwd";
  if (R == 0) return 0;
  MMS_REQUIRE(idx && o && d && u && n && f && oh && dh && uh && nh && fh, fn, "null pointer");
  hipLaunchKernelGGL(hit_gather_fwd_kernel, dim3(mms::grid_for(R, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), idx, R, o, d, u, n, f, oh, dh, uh, nh, fh);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hit_gather_bwd(const int64_t* idx, int64_t R, const float* doh, const float* ddh, const float* duh,
                                  const float* dnh, const float* dfh, float* dorig, float* ddirs, float* dups,
                                  float* dnears, float* dfars, void* stream) {
  const char* fn = "mms_hit_gather_bwd";
  if (R == 0) return 0;
  MMS_REQUIRE(idx && dorig && ddirs && dups && dnears && dfars, fn, "null pointer");
  hipLaunchKernelGGL(hit_gather_bwd_kernel, dim3(mms::grid_for(R, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), idx, R, doh, ddh, duh, dnh, dfh, dorig, ddirs, dups, dnears, dfars);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_pose_exp_fwd(const float* tangent, int64_t B, float* mats, void* stream) {
  const char* fn = "mms_pose_exp_fwd";
  if (B == 0) return 0;
  MMS_REQUIRE(tangent && mats, fn, "null pointer");
  hipLaunchKernelGGL(pose_exp_fwd_kernel, dim3(mms::grid_for(B, 64)), dim3(64), 0, mms::as_stream(stream), tangent, B,
                     mats);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_pose_exp_bwd(const float* tangent, const float* dmats, int64_t B, float* dtangent, void* stream) {
  const char* fn = "mms_pose_exp_bwd";
  if (B == 0) return 0;
  MMS_REQUIRE(tangent && dmats && dtangent, fn, "null pointer");
  hipLaunchKernelGGL(pose_exp_bwd_kernel, dim3(mms::grid_for(B, 64)), dim3(64), 0, mms::as_stream(stream), tangent,
                     dmats, B, dtangent);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_raygen_fwd(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx,
                              const float* cy, const float* c2w, const float* dist, const float* mats, int mat_per_cam,
                              float pixel_offset, float* origins, float* dirs, float* ups, float* area, float* dnorm,
                              void* stream) {
  const char* fn = "mms_raygen_fwd";
  if (N == 0) return 0;
  MMS_REQUIRE(coords && c2w && mats && origins && dirs, fn, "null pointer");
  hipLaunchKernelGGL(raygen_fwd_kernel, dim3(mms::grid_for(N, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                     coords, N, fx, fy, cx, cy, c2w, dist, mats, mat_per_cam, pixel_offset, origins, dirs, ups, area,
                     dnorm);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_raygen_bwd(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx,
                              const float* cy, const float* c2w, const float* dist, const float* mats, int mat_per_cam,
                              float pixel_offset, const float* dorig, const float* ddirs, const float* dups,
                              float* dmats, void* stream) {
  const char* fn = "mms_raygen_bwd";
  if (N == 0) return 0;
  hipLaunchKernelGGL(raygen_bwd_kernel, dim3(mms::grid_for(N, 256, INT32_MAX)), dim3(256), 0, mms::as_stream(stream),
                     coords, N, fx, fy, cx, cy, c2w, dist, mats, mat_per_cam, pixel_offset, dorig, ddirs, dups, dmats);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_collider_fwd(const float* origins, const float* dirs, int64_t N, float radius, float* nears,
                                float* fars, unsigned char* mask, float* bg_nears, float* bg_fars, void* stream) {
  const char* fn = "mms_collider_fwd";
  if (N == 0) return 0;
  hipLaunchKernelGGL(collider_fwd_kernel, dim3(mms::grid_for(N, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                     origins, dirs, N, radius, nears, fars, mask, bg_nears, bg_fars);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_collider_bwd(const float* origins, const float* dirs, int64_t N, float radius, const float* dnears,
                                const float* dfars, const float* dbg_nears, const float* dbg_fars, float* dorig,
                                float* ddirs, void* stream) {
  const char* fn = "mms_collider_bwd";
  if (N == 0) return 0;
  hipLaunchKernelGGL(collider_bwd_kernel, dim3(mms::grid_for(N, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                     origins, dirs, N, radius, dnears, dfars, dbg_nears, dbg_fars, dorig, ddirs);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_count_hits(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx,
                              const float* cy, const float* c2w, const float* dist, const float* tangent,
                              const float* mats, int B, int mat_per_cam, float pixel_offset, float radius,
                              int64_t* count, void* stream) {
  const char* fn = "mms_count_hits";
  MMS_REQUIRE(B >= 1 && B <= kCountMaxMats, fn, "1 to 256 pose matrices");
  MMS_REQUIRE(coords && fx && fy && cx && cy && c2w && count && (tangent || mats), fn, "null pointer");
  MMS_REQUIRE(N >= 0, fn, "negative ray count");
  if (N == 0) return 0;
  hipLaunchKernelGGL(count_hits_kernel, dim3(mms::grid_for(N, 256, 1024)), dim3(256), 0, mms::as_stream(stream), coords,
                     N, fx, fy, cx, cy, c2w, dist, tangent, mats, B, mat_per_cam, pixel_offset, radius, count);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_compact(const unsigned char* mask, int64_t N, int64_t* idx, int64_t* count, void* stream) {
  const char* fn = "mms_compact";
  hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(1024), 0, mms::as_stream(stream), mask, N, idx, count);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_compact_padded(const unsigned char* mask, int64_t N, int64_t cap, int64_t* idx, int64_t* sidx,
                                  int64_t* count, void* stream) {
  const char* fn = "mms_compact_padded";
  MMS_REQUIRE(cap >= 1 && cap <= N, fn, "capacity must be in [1, N]");
  MMS_REQUIRE(idx && count, fn, "null pointer");
  hipStream_t s = mms::as_stream(stream);
  // the scan writes hit indices below the true count: idx needs N entries when more than cap rays hit,
  // so the caller passes an [N] buffer and uses its first cap entries
  hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(1024), 0, s, mask, N, idx, count);
  hipLaunchKernelGGL(compact_pad_kernel, dim3(1), dim3(1024), 0, s, N, cap, idx, sidx, count);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_compact_segments(const unsigned char* mask, int n_seg, int64_t N, int64_t cap, int64_t* scratch,
                                    int64_t* gidx, int64_t* sidx, int64_t* count, void* stream) {
  const char* fn = "mms_compact_segments";
  MMS_REQUIRE(n_seg >= 1 && n_seg <= 65535, fn, "segment count must be in [1, 65535]");
  MMS_REQUIRE(cap >= 1 && cap <= N, fn, "capacity must be in [1, N]");
  MMS_REQUIRE(mask && scratch && gidx && count, fn, "null pointer");
  hipLaunchKernelGGL(compact_segments_kernel, dim3(n_seg), dim3(1024), 0, mms::as_stream(stream), mask, N, cap,
                     scratch, gidx, sidx, count);
  return mms::check_launch(fn);
}
