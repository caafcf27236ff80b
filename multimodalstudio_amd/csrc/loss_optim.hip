// Loss terms and the fused optimizer step.
//
// Losses (/root/reference/src/model_components/losses.py):
//   L1 radiance loss (nn.L1Loss, mean)                       :68-90
//   SkipSaturationLoss: saturated targets -> output := first saturated target value   :152-164
//   EikonalLoss: MSE(||grad||, 1)                             :107-119
//   CurvatureLoss: L1(sum(hessian), 0)                        :121-150
// Optimizer (pipelines/base_pipeline.py:232-248 + torch.optim.AdamW, method_configs.py:260-269):
//   clip_grad_norm_(max_norm) over an optimizer's parameters, then AdamW (decoupled weight decay).
// Every scalar stays on the device (no host synchronisation inside a step).
#include "common.h"

#include <math.h>

namespace {

__device__ __forceinline__ float block_reduce_sum(float v) {
  __shared__ float red[16];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  }
  return t;  // valid on thread 0
}

// first flattened index with target > thr (atomicMin), init must be INT64 max
__global__ void first_saturated_kernel(const float* __restrict__ tgt, int64_t n, float thr,
                                       unsigned long long* __restrict__ first) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (tgt[i] > thr) atomicMin(first, (unsigned long long)i);
  }
}

// out/tgt are [N, C] with row strides; loss += sum |o - t| / (N C)
__device__ __forceinline__ void l1_fwd_body(const float* __restrict__ out, int64_t ldo, const float* __restrict__ tgt,
                                            int64_t N, int C, float thr, const unsigned long long* __restrict__ first,
                                            float* __restrict__ loss, int64_t blk, int64_t nblk) {
  const int64_t n = N * C;
  float fill = 0.f;
  bool sat = false;
  if (first != nullptr && first[0] < (unsigned long long)n) { sat = true; fill = tgt[first[0]]; }
  float s = 0.f;
  for (int64_t i = blk * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
    const int64_t r = i / C, c = i - r * C;
    const float t = tgt[i];
    float o = out[r * ldo + c];
    if (sat && t > thr) o = fill;
    s += fabsf(o - t);
  }
  s = block_reduce_sum(s);
  if (threadIdx.x == 0) atomicAdd(loss, s / (float)n);
}

__global__ __launch_bounds__(256) void l1_fwd_kernel(const float* __restrict__ out, int64_t ldo,
                                                     const float* __restrict__ tgt, int64_t N, int C, float thr,
                                                     const unsigned long long* __restrict__ first,
                                                     float* __restrict__ loss) {
  l1_fwd_body(out, ldo, tgt, N, C, thr, first, loss, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ void l1_bwd_body(const float* __restrict__ out, int64_t ldo, const float* __restrict__ tgt,
                                            int64_t N, int C, float thr, const unsigned long long* __restrict__ first,
                                            const float* __restrict__ dloss, float scale, float* __restrict__ dout,
                                            int64_t lddo, int64_t blk, int64_t nblk) {
  const int64_t n = N * C;
  const bool sat = first != nullptr && first[0] < (unsigned long long)n;
  const float g = dloss[0] * scale / (float)n;
  for (int64_t i = blk * blockDim.x + threadIdx.x; i < n; i += nblk * blockDim.x) {
    const int64_t r = i / C, c = i - r * C;
    const float t = tgt[i];
    const float o = out[r * ldo + c];
    float d = (o > t) ? g : ((o < t) ? -g : 0.f);
    if (sat && t > thr) d = 0.f;  // masked_fill: output replaced by a constant
    dout[r * lddo + c] += d;
  }
}

__global__ void l1_bwd_kernel(const float* __restrict__ out, int64_t ldo, const float* __restrict__ tgt, int64_t N,
                              int C, float thr, const unsigned long long* __restrict__ first,
                              const float* __restrict__ dloss, float scale, float* __restrict__ dout, int64_t lddo) {
  l1_bwd_body(out, ldo, tgt, N, C, thr, first, dloss, scale, dout, lddo, blockIdx.x, gridDim.x);
}

// eikonal: sum over rows of (||g|| - 1)^2 / M_total ; curvature: sum |h0 + h1 + h2| / M_total.
// Fixed-capacity batches (graph-captured steps, graphs.py): with `count`, only rows [0, count[0] * S) are real, and
// 1 / M_total = 1 / max(1, S * sum(counts_all)) is formed on the device -- the hit counts never reach the host.
__device__ __forceinline__ float inv_rows(const int64_t* counts_all, int n_counts, int S, float inv_total) {
  if (counts_all == nullptr) return inv_total;
  int64_t t = 0;
  for (int k = 0; k < n_counts; ++k) t += counts_all[k];
  t *= S;
  return 1.0f / (float)(t > 1 ? t : 1);
}

__device__ __forceinline__ void geo_fwd_body(const float* __restrict__ grads, const float* __restrict__ hess, int64_t M,
                                             const int64_t* __restrict__ count, int S, float inv_total,
                                             const int64_t* __restrict__ counts_all, int n_counts,
                                             float* __restrict__ eik, float* __restrict__ curv, int64_t blk,
                                             int64_t nblk) {
  const int64_t lim = count ? (count[0] * S < M ? count[0] * S : M) : M;
  const float inv = inv_rows(counts_all, n_counts, S, inv_total);
  float se = 0.f, sc = 0.f;
  for (int64_t i = blk * blockDim.x + threadIdx.x; i < lim; i += nblk * blockDim.x) {
    if (grads) {
      const float g0 = grads[i * 3], g1 = grads[i * 3 + 1], g2 = grads[i * 3 + 2];
      const float n = sqrtf(g0 * g0 + g1 * g1 + g2 * g2);
      se += (n - 1.0f) * (n - 1.0f);
    }
    if (hess) sc += fabsf(hess[i * 3] + hess[i * 3 + 1] + hess[i * 3 + 2]);
  }
  se = block_reduce_sum(se);
  __syncthreads();
  sc = block_reduce_sum(sc);
  if (threadIdx.x == 0) {
    if (eik) atomicAdd(eik, se * inv);
    if (curv) atomicAdd(curv, sc * inv);
  }
}

__global__ __launch_bounds__(256) void geo_loss_fwd_kernel(const float* __restrict__ grads,
                                                           const float* __restrict__ hess, int64_t M,
                                                           const int64_t* __restrict__ count, int S, float inv_total,
                                                           const int64_t* __restrict__ counts_all, int n_counts,
                                                           float* __restrict__ eik, float* __restrict__ curv) {
  geo_fwd_body(grads, hess, M, count, S, inv_total, counts_all, n_counts, eik, curv, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ void geo_bwd_body(const float* __restrict__ grads, const float* __restrict__ hess, int64_t M,
                                             const int64_t* __restrict__ count, int S, float inv_total,
                                             const int64_t* __restrict__ counts_all, int n_counts,
                                             const float* __restrict__ deik, float eik_scale,
                                             const float* __restrict__ dcurv, float curv_scale,
                                             float* __restrict__ dgrads, float* __restrict__ dhess, int64_t blk,
                                             int64_t nblk) {
  const int64_t lim = count ? (count[0] * S < M ? count[0] * S : M) : M;
  const float inv = inv_rows(counts_all, n_counts, S, inv_total);
  const float ge = deik ? deik[0] * eik_scale * inv : 0.f;
  const float gc = dcurv ? dcurv[0] * curv_scale * inv : 0.f;
  for (int64_t i = blk * blockDim.x + threadIdx.x; i < lim; i += nblk * blockDim.x) {
    if (grads && dgrads && deik) {
      const float g0 = grads[i * 3], g1 = grads[i * 3 + 1], g2 = grads[i * 3 + 2];
      const float n = sqrtf(g0 * g0 + g1 * g1 + g2 * g2);
      const float f = n > 0.f ? 2.0f * (n - 1.0f) * ge / n : 0.f;
      dgrads[i * 3] += f * g0;
      dgrads[i * 3 + 1] += f * g1;
      dgrads[i * 3 + 2] += f * g2;
    }
    if (hess && dhess && dcurv) {
      const float l = hess[i * 3] + hess[i * 3 + 1] + hess[i * 3 + 2];
      const float d = l > 0.f ? gc : (l < 0.f ? -gc : 0.f);
      dhess[i * 3] += d;
      dhess[i * 3 + 1] += d;
      dhess[i * 3 + 2] += d;
    }
  }
}

__global__ void geo_loss_bwd_kernel(const float* __restrict__ grads, const float* __restrict__ hess, int64_t M,
                                    const int64_t* __restrict__ count, int S, float inv_total,
                                    const int64_t* __restrict__ counts_all, int n_counts,
                                    const float* __restrict__ deik, float eik_scale,
                                    const float* __restrict__ dcurv, float curv_scale, float* __restrict__ dgrads,
                                    float* __restrict__ dhess) {
  geo_bwd_body(grads, hess, M, count, S, inv_total, counts_all, n_counts, deik, eik_scale, dcurv, curv_scale, dgrads,
               dhess, blockIdx.x, gridDim.x);
}

// The step loss's L1 terms and geometric terms in ONE launch each way (graph-replayed steps: every launch boundary
// costs ~4-5 us): segment k owns blocks [b0[k], b0[k + 1]) -- the blocks its own launch would have had -- and runs
// that launch's body (mms_l1_loss_* / mms_geo_loss_*_masked, same arithmetic).
constexpr int kMaxLossSeg = 8;
struct LossSegs {
  int n_l1, n_geo;
  int b0[2 * kMaxLossSeg + 1];
  const float* out[kMaxLossSeg];
  int64_t ldo[kMaxLossSeg];
  const float* tgt[kMaxLossSeg];
  int64_t N[kMaxLossSeg];
  int C[kMaxLossSeg];
  float thr[kMaxLossSeg];
  const unsigned long long* first[kMaxLossSeg];
  float* l1[kMaxLossSeg];          // fwd: the term; bwd: dout
  int64_t lddo[kMaxLossSeg];
  const float* grads[kMaxLossSeg];
  const float* hess[kMaxLossSeg];
  float* dgrads[kMaxLossSeg];
  float* dhess[kMaxLossSeg];
  int64_t rows[kMaxLossSeg];
  const int64_t* count[kMaxLossSeg];
  const int64_t* counts_all;
  int n_counts, S;
  float inv_total;
  float* eik;
  float* curv;
  const float* dloss;
  float eik_scale, curv_scale;
};

__device__ __forceinline__ int loss_seg_of(const LossSegs& a, int b) {
  int k = 0;
  while (k + 1 < a.n_l1 + a.n_geo && b >= a.b0[k + 1]) ++k;
  return k;
}

__global__ __launch_bounds__(256) void step_loss_fwd_kernel(LossSegs a) {
  const int k = loss_seg_of(a, blockIdx.x);
  const int64_t blk = blockIdx.x - a.b0[k], nblk = a.b0[k + 1] - a.b0[k];
  if (k < a.n_l1)
    l1_fwd_body(a.out[k], a.ldo[k], a.tgt[k], a.N[k], a.C[k], a.thr[k], a.first[k], a.l1[k], blk, nblk);
  else {
    const int j = k - a.n_l1;
    geo_fwd_body(a.grads[j], a.hess[j], a.rows[j], a.count[j], a.S, a.inv_total, a.counts_all, a.n_counts, a.eik,
                 a.curv, blk, nblk);
  }
}

__global__ __launch_bounds__(256) void step_loss_bwd_kernel(LossSegs a) {
  const int k = loss_seg_of(a, blockIdx.x);
  const int64_t blk = blockIdx.x - a.b0[k], nblk = a.b0[k + 1] - a.b0[k];
  if (k < a.n_l1)
    l1_bwd_body(a.out[k], a.ldo[k], a.tgt[k], a.N[k], a.C[k], a.thr[k], a.first[k], a.dloss, 1.0f, a.l1[k],
                a.lddo[k], blk, nblk);
  else {
    const int j = k - a.n_l1;
    geo_bwd_body(a.grads[j], a.hess[j], a.rows[j], a.count[j], a.S, a.inv_total, a.counts_all, a.n_counts, a.dloss,
                 a.eik_scale, a.dloss, a.curv_scale, a.dgrads[j], a.dhess[j], blk, nblk);
  }
}

// ------------------------------------------------------------------ optimizer
// Launch shape measured on the bench step (scripts/gpu_iter20.sh / gpu_iter21.sh, rocprofv3 per-step tables,
// profiles/round3d_ab.txt): the blocks' partial sums meet in ONE float atomic, which serializes at the memory side,
// so fewer, fuller blocks win -- 2048 blocks x 4 loads 22.3 us per launch (avg of the two groups), 8192: 57.6,
// 1024: 18.5, 512: 15.6, 256 x 8 loads: 14.3.
#ifndef MMS_SUMSQ_UNROLL
#define MMS_SUMSQ_UNROLL 8   // independent 16-B loads in flight per lane per iteration
#endif
#ifndef MMS_SUMSQ_GRID
#define MMS_SUMSQ_GRID 256   // blocks (grid-stride): one per CU
#endif
// one block's share of sum(x^2) over x[0, n), blocks [0, nblk) of the segment; added into acc
__device__ __forceinline__ void sumsq_seg(const float* __restrict__ x, int64_t n, float* __restrict__ acc, int64_t blk,
                                          int64_t nblk) {
  constexpr int U = MMS_SUMSQ_UNROLL;
  const int64_t n4 = n / 4;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  // U independent 16-B loads in flight per lane per iteration (one dependent load per iteration left the 138 MB
  // gradient read at 3.1 TB/s), then the remainder one at a time
  const int64_t stride = nblk * blockDim.x;
  int64_t i = blk * blockDim.x + threadIdx.x;
  float ps[U];
#pragma unroll
  for (int u = 0; u < U; ++u) ps[u] = 0.f;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x4[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) ps[u] += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
  }
  for (; i < n4; i += stride) {
    const float4 v = x4[i];
    ps[0] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) s += ps[u];
  for (int64_t i = n4 * 4 + blk * blockDim.x + threadIdx.x; i < n; i += stride) s += x[i] * x[i];
  s = block_reduce_sum(s);
  if (threadIdx.x == 0) atomicAdd(acc, s);
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ acc) {
  sumsq_seg(x, n, acc, blockIdx.x, gridDim.x);
}

// Several optimizer groups in one launch (graph-replayed steps: each launch boundary costs ~4-5 us): segment k owns
// blocks [b0[k], b0[k + 1]) of the grid -- the blocks its own launch would have had -- and its own operands.
constexpr int kMaxSeg = 8;
struct OptSegs {
  int n;
  int b0[kMaxSeg + 1];
  float* p[kMaxSeg];
  const float* g[kMaxSeg];
  float* m[kMaxSeg];
  float* v[kMaxSeg];
  int64_t len[kMaxSeg];
  float* acc[kMaxSeg];          // sumsq: accumulators; adamw: the groups' sums of squares (read)
  float max_norm[kMaxSeg];
  const float* hyper[kMaxSeg];
};

__device__ __forceinline__ int seg_of(const OptSegs& a, int b) {
  int k = 0;
  while (k + 1 < a.n && b >= a.b0[k + 1]) ++k;
  return k;
}

__global__ __launch_bounds__(256) void sumsq_multi_kernel(OptSegs a) {
  const int k = seg_of(a, blockIdx.x);
  sumsq_seg(a.g[k], a.len[k], a.acc[k], blockIdx.x - a.b0[k], a.b0[k + 1] - a.b0[k]);
}

// zero fill of several buffers (the groups' gradients and sum-of-squares accumulators), 16 B per lane where aligned
__global__ __launch_bounds__(256) void zero_multi_kernel(OptSegs a) {
  const int k = seg_of(a, blockIdx.x);
  float* x = a.p[k];
  const int64_t n = a.len[k];
  const int64_t stride = (int64_t)(a.b0[k + 1] - a.b0[k]) * blockDim.x;
  const int64_t t0 = (int64_t)(blockIdx.x - a.b0[k]) * blockDim.x + threadIdx.x;
  const bool al = ((uintptr_t)x & 15) == 0;
  const int64_t n4 = al ? n / 4 : 0;
  for (int64_t i = t0; i < n4; i += stride) reinterpret_cast<float4*>(x)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = n4 * 4 + t0; i < n; i += stride) x[i] = 0.f;
}

// AdamW with the clip coefficient coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) applied to g, in the operation
// order of torch.optim.AdamW's single-tensor CPU step (the reference's optimizer):
//   p *= decay;  m = lerp(m, g, 1 - b1) = fma(1 - b1, g - m, m)  (ATen's vectorised lerp, small weight);
//   v = v * b2 + ((1 - b2) * g) * g  (addcmul);  p = p + ((-step_size) * m) / (sqrt(v) / bc2_sqrt + eps)  (addcdiv)
// with the scalars rounded from the double values Python computes (mms_adamw_scalars): hyper = [decay, 1 - b1, b2,
// 1 - b2, eps, -step_size, bc2_sqrt].  Contraction off: only the lerp is fused, as in ATen.
__device__ __forceinline__ void adamw_apply(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                            float* __restrict__ v, int64_t n, const float* __restrict__ sumsq,
                                            float max_norm, float decay, float w1, float b2, float w2, float eps,
                                            float neg_step, float bc2_sqrt) {
#pragma clang fp contract(off)
  float coef = 1.0f;
  if (sumsq != nullptr && max_norm > 0.f) {
    const float total = sqrtf(sumsq[0]);
    coef = fminf(max_norm / (total + 1e-6f), 1.0f);
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * coef;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = __builtin_fmaf(w1, gi - mi, mi);
    const float vi = v[i] * b2 + (w2 * gi) * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + (neg_step * mi) / denom;
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    const float* __restrict__ sumsq, float max_norm, float decay,
                                                    float w1, float b2, float w2, float eps, float neg_step,
                                                    float bc2_sqrt) {
  adamw_apply(p, g, m, v, n, sumsq, max_norm, decay, w1, b2, w2, eps, neg_step, bc2_sqrt);
}

// adamw_dev_kernel of several groups in one launch (segment k: blocks [b0[k], b0[k + 1]), its own scalars)
__global__ __launch_bounds__(256) void adamw_dev_multi_kernel(OptSegs a) {
#pragma clang fp contract(off)
  const int k = seg_of(a, blockIdx.x);
  const float* h = a.hyper[k];
  const float* __restrict__ g = a.g[k];
  float* __restrict__ p = a.p[k];
  float* __restrict__ m = a.m[k];
  float* __restrict__ v = a.v[k];
  const int64_t n = a.len[k];
  const float decay = h[0], w1 = h[1], b2 = h[2], w2 = h[3], eps = h[4], neg_step = h[5], bc2_sqrt = h[6];
  float coef = 1.0f;
  if (a.acc[k] != nullptr && a.max_norm[k] > 0.f) {
    const float total = sqrtf(a.acc[k][0]);
    coef = fminf(a.max_norm[k] / (total + 1e-6f), 1.0f);
  }
  const int64_t stride = (int64_t)(a.b0[k + 1] - a.b0[k]) * blockDim.x;
  for (int64_t i = (int64_t)(blockIdx.x - a.b0[k]) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gi = g[i] * coef;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = __builtin_fmaf(w1, gi - mi, mi);
    const float vi = v[i] * b2 + (w2 * gi) * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi + (neg_step * mi) / denom;
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// the per-step scalars read on the device (graph replays): hyper = mms_adamw_scalars' 7 floats
__global__ __launch_bounds__(256) void adamw_dev_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                        const float* __restrict__ sumsq, float max_norm,
                                                        const float* __restrict__ hyper) {
  adamw_apply(p, g, m, v, n, sumsq, max_norm, hyper[0], hyper[1], hyper[2], hyper[3], hyper[4], hyper[5], hyper[6]);
}

}  // namespace

MMS_EXPORT int mms_l1_loss_fwd(const float* out, int64_t ldo, const float* tgt, int64_t N, int C, float sat_thr,
                               unsigned long long* first_scratch, float* loss, void* stream) {
  const char* fn = "mms_l1_loss_fwd";
  if (N == 0) return 0;
  hipStream_t s = mms::as_stream(stream);
  if (first_scratch) {
    if (hipMemsetAsync(first_scratch, 0xFF, sizeof(unsigned long long), s) != hipSuccess)
      return mms::set_error(fn, "memset failed");
    hipLaunchKernelGGL(first_saturated_kernel, dim3(mms::grid_for(N * C, 256, 1024)), dim3(256), 0, s, tgt, N * C,
                       sat_thr, first_scratch);
  }
  hipLaunchKernelGGL(l1_fwd_kernel, dim3(mms::grid_for(N * C, 256, 1024)), dim3(256), 0, s, out, ldo, tgt, N, C,
                     sat_thr, first_scratch, loss);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_l1_loss_bwd(const float* out, int64_t ldo, const float* tgt, int64_t N, int C, float sat_thr,
                               const unsigned long long* first_scratch, const float* dloss, float scale, float* dout,
                               int64_t lddo, void* stream) {
  const char* fn = "mms_l1_loss_bwd";
  if (N == 0) return 0;
  hipLaunchKernelGGL(l1_bwd_kernel, dim3(mms::grid_for(N * C, 256, 4096)), dim3(256), 0, mms::as_stream(stream), out,
                     ldo, tgt, N, C, sat_thr, first_scratch, dloss, scale, dout, lddo);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_geo_loss_fwd(const float* grads, const float* hess, int64_t M, float inv_total, float* eik,
                                float* curv, void* stream) {
  const char* fn = "mms_geo_loss_fwd";
  if (M == 0) return 0;
  hipLaunchKernelGGL(geo_loss_fwd_kernel, dim3(mms::grid_for(M, 256, 1024)), dim3(256), 0, mms::as_stream(stream),
                     grads, hess, M, nullptr, 1, inv_total, nullptr, 0, eik, curv);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_geo_loss_fwd_masked(const float* grads, const float* hess, int64_t M, int S, const int64_t* count,
                                       const int64_t* counts_all, int n_counts, float* eik, float* curv,
                                       void* stream) {
  const char* fn = "mms_geo_loss_fwd_masked";
  MMS_REQUIRE(S >= 1 && count != nullptr && counts_all != nullptr && n_counts >= 1, fn,
              "needs S >= 1, this batch's device hit count and every batch's");
  if (M == 0) return 0;
  hipLaunchKernelGGL(geo_loss_fwd_kernel, dim3(mms::grid_for(M, 256, 1024)), dim3(256), 0, mms::as_stream(stream),
                     grads, hess, M, count, S, 0.f, counts_all, n_counts, eik, curv);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_geo_loss_bwd(const float* grads, const float* hess, int64_t M, float inv_total, const float* deik,
                                float eik_scale, const float* dcurv, float curv_scale, float* dgrads, float* dhess,
                                void* stream) {
  const char* fn = "mms_geo_loss_bwd";
  if (M == 0) return 0;
  hipLaunchKernelGGL(geo_loss_bwd_kernel, dim3(mms::grid_for(M, 256, 8192)), dim3(256), 0, mms::as_stream(stream),
                     grads, hess, M, nullptr, 1, inv_total, nullptr, 0, deik, eik_scale, dcurv, curv_scale, dgrads, dhess);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_geo_loss_bwd_masked(const float* grads, const float* hess, int64_t M, int S, const int64_t* count,
                                       const int64_t* counts_all, int n_counts, const float* deik, float eik_scale,
                                       const float* dcurv, float curv_scale, float* dgrads, float* dhess,
                                       void* stream) {
  const char* fn = "mms_geo_loss_bwd_masked";
  MMS_REQUIRE(S >= 1 && count != nullptr && counts_all != nullptr && n_counts >= 1, fn,
              "needs S >= 1, this batch's device hit count and every batch's");
  if (M == 0) return 0;
  hipLaunchKernelGGL(geo_loss_bwd_kernel, dim3(mms::grid_for(M, 256, 8192)), dim3(256), 0, mms::as_stream(stream),
                     grads, hess, M, count, S, 0.f, counts_all, n_counts, deik, eik_scale, dcurv, curv_scale, dgrads,
                     dhess);
  return mms::check_launch(fn);
}

// the shared argument table of mms_step_loss_fwd / _bwd (block counts as the per-launch entry points size them)
static int fill_loss_segs(const char* fn, LossSegs& a, int n_l1, const float* const* out, const int64_t* ldo,
                          const float* const* tgt, const int64_t* N, const int* C, const float* thr,
                          const unsigned long long* const* first, int n_geo, const float* const* grads,
                          const float* const* hess, const int64_t* rows, int S, const int64_t* const* count,
                          const int64_t* counts_all, int n_counts, float inv_total, int l1_grid, int geo_grid) {
  MMS_REQUIRE(n_l1 >= 0 && n_l1 <= kMaxLossSeg && n_geo >= 0 && n_geo <= kMaxLossSeg && n_l1 + n_geo >= 1, fn,
              "0 to 8 L1 and 0 to 8 geometric segments");
  MMS_REQUIRE(n_l1 == 0 || (out && ldo && tgt && N && C && thr && first), fn, "null L1 segment table");
  MMS_REQUIRE(n_geo == 0 || (grads && hess && rows && count), fn, "null geometric segment table");
  a.n_l1 = n_l1;
  a.n_geo = n_geo;
  a.b0[0] = 0;
  int k = 0;
  for (int i = 0; i < n_l1; ++i, ++k) {
    a.out[i] = out[i]; a.ldo[i] = ldo[i]; a.tgt[i] = tgt[i]; a.N[i] = N[i]; a.C[i] = C[i]; a.thr[i] = thr[i];
    a.first[i] = first[i];
    const int64_t n = N[i] * C[i];
    a.b0[k + 1] = a.b0[k] + (n > 0 ? (int)mms::grid_for(n, 256, l1_grid) : 0);
  }
  for (int j = 0; j < n_geo; ++j, ++k) {
    a.grads[j] = grads[j]; a.hess[j] = hess[j]; a.rows[j] = rows[j]; a.count[j] = count[j];
    a.b0[k + 1] = a.b0[k] + (rows[j] > 0 ? (int)mms::grid_for(rows[j], 256, geo_grid) : 0);
  }
  a.counts_all = counts_all;
  a.n_counts = n_counts;
  a.S = S;
  a.inv_total = inv_total;
  return 0;
}

MMS_EXPORT int mms_step_loss_fwd(int n_l1, const float* const* out, const int64_t* ldo, const float* const* tgt,
                                 const int64_t* N, const int* C, const float* thr,
                                 const unsigned long long* const* first, float* const* loss, int n_geo,
                                 const float* const* grads, const float* const* hess, const int64_t* rows, int S,
                                 const int64_t* const* count, const int64_t* counts_all, int n_counts, float inv_total,
                                 float* eik, float* curv, void* stream) {
  const char* fn = "mms_step_loss_fwd";
  LossSegs a{};
  int rc = fill_loss_segs(fn, a, n_l1, out, ldo, tgt, N, C, thr, first, n_geo, grads, hess, rows, S, count,
                          counts_all, n_counts, inv_total, 1024, 1024);
  if (rc) return rc;
  MMS_REQUIRE(n_l1 == 0 || loss, fn, "null loss terms");
  for (int i = 0; i < n_l1; ++i) a.l1[i] = loss[i];
  a.eik = eik;
  a.curv = curv;
  if (a.b0[n_l1 + n_geo] == 0) return 0;
  hipLaunchKernelGGL(step_loss_fwd_kernel, dim3(a.b0[n_l1 + n_geo]), dim3(256), 0, mms::as_stream(stream), a);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_step_loss_bwd(int n_l1, const float* const* out, const int64_t* ldo, const float* const* tgt,
                                 const int64_t* N, const int* C, const float* thr,
                                 const unsigned long long* const* first, float* const* dout, const int64_t* lddo,
                                 int n_geo, const float* const* grads, const float* const* hess, const int64_t* rows,
                                 int S, const int64_t* const* count, const int64_t* counts_all, int n_counts,
                                 float inv_total, const float* dloss, float eik_scale, float curv_scale,
                                 float* const* dgrads, float* const* dhess, void* stream) {
  const char* fn = "mms_step_loss_bwd";
  LossSegs a{};
  int rc = fill_loss_segs(fn, a, n_l1, out, ldo, tgt, N, C, thr, first, n_geo, grads, hess, rows, S, count,
                          counts_all, n_counts, inv_total, 4096, 8192);
  if (rc) return rc;
  MMS_REQUIRE(dloss != nullptr && (n_l1 == 0 || (dout && lddo)) && (n_geo == 0 || (dgrads && dhess)), fn,
              "null gradient table");
  for (int i = 0; i < n_l1; ++i) { a.l1[i] = dout[i]; a.lddo[i] = lddo[i]; }
  for (int j = 0; j < n_geo; ++j) { a.dgrads[j] = dgrads[j]; a.dhess[j] = dhess[j]; }
  a.dloss = dloss;
  a.eik_scale = eik_scale;
  a.curv_scale = curv_scale;
  if (a.b0[n_l1 + n_geo] == 0) return 0;
  hipLaunchKernelGGL(step_loss_bwd_kernel, dim3(a.b0[n_l1 + n_geo]), dim3(256), 0, mms::as_stream(stream), a);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_sumsq(const float* x, int64_t n, float* acc, void* stream) {
  const char* fn = "mms_sumsq";
  if (n == 0) return 0;
  MMS_REQUIRE(((uintptr_t)x & 15) == 0, fn, "buffer must be 16-byte aligned");
  hipLaunchKernelGGL(sumsq_kernel, dim3(mms::grid_for(n / 4 + 1, 256, MMS_SUMSQ_GRID)), dim3(256), 0, mms::as_stream(stream), x,
                     n, acc);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_adamw_scalars(double lr, double wd, double beta1, double beta2, double eps, int64_t step,
                                 float* hyper) {
  const char* fn = "mms_adamw_scalars";
  MMS_REQUIRE(hyper != nullptr, fn, "null output");
  MMS_REQUIRE(step >= 1, fn, "step counts from 1 (torch.optim.AdamW increments before use)");
  // torch/optim/adamw.py (single-tensor): Python doubles, rounded to float where they meet a float tensor
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  hyper[0] = (float)(1.0 - lr * wd);
  hyper[1] = (float)(1.0 - beta1);
  hyper[2] = (float)beta2;
  hyper[3] = (float)(1.0 - beta2);
  hyper[4] = (float)eps;
  hyper[5] = (float)(-(lr / bc1));
  hyper[6] = (float)pow(bc2, 0.5);
  return 0;
}

MMS_EXPORT int mms_adamw(float* p, const float* g, float* m, float* v, int64_t n, const float* sumsq, float max_norm,
                         double lr, double wd, double beta1, double beta2, double eps, int64_t step, void* stream) {
  const char* fn = "mms_adamw";
  float h[7];
  const int rc = mms_adamw_scalars(lr, wd, beta1, beta2, eps, step, h);
  if (rc) return rc;
  if (n == 0) return 0;
  hipLaunchKernelGGL(adamw_kernel, dim3(mms::grid_for(n, 256, 8192)), dim3(256), 0, mms::as_stream(stream), p, g, m, v,
                     n, sumsq, max_norm, h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* sumsq, float max_norm,
                             const float* hyper, void* stream) {
  const char* fn = "mms_adamw_dev";
  MMS_REQUIRE(hyper != nullptr, fn, "null hyper-parameter buffer");
  if (n == 0) return 0;
  hipLaunchKernelGGL(adamw_dev_kernel, dim3(mms::grid_for(n, 256, 8192)), dim3(256), 0, mms::as_stream(stream), p, g, m,
                     v, n, sumsq, max_norm, hyper);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_zero_multi(int nbuf, float* const* x, const int64_t* n, void* stream) {
  const char* fn = "mms_zero_multi";
  MMS_REQUIRE(nbuf >= 1 && nbuf <= kMaxSeg && x && n, fn, "1 to 8 buffers");
  OptSegs a{};
  a.n = nbuf;
  a.b0[0] = 0;
  for (int k = 0; k < nbuf; ++k) {
    MMS_REQUIRE(n[k] >= 0 && (n[k] == 0 || x[k] != nullptr), fn, "null buffer");
    a.p[k] = x[k];
    a.len[k] = n[k];
    a.b0[k + 1] = a.b0[k] + (int)mms::grid_for(n[k] / 4 + 1, 256, 2048);
  }
  hipLaunchKernelGGL(zero_multi_kernel, dim3(a.b0[nbuf]), dim3(256), 0, mms::as_stream(stream), a);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_sumsq_multi(int nseg, const float* const* x, const int64_t* n, float* const* acc, void* stream) {
  const char* fn = "mms_sumsq_multi";
  MMS_REQUIRE(nseg >= 1 && nseg <= kMaxSeg && x && n && acc, fn, "1 to 8 segments");
  OptSegs a{};
  a.n = nseg;
  a.b0[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    MMS_REQUIRE(n[k] >= 0 && acc[k] != nullptr && (n[k] == 0 || x[k] != nullptr), fn, "null buffer");
    MMS_REQUIRE(((uintptr_t)x[k] & 15) == 0, fn, "buffers must be 16-byte aligned");
    a.g[k] = x[k];
    a.len[k] = n[k];
    a.acc[k] = acc[k];
    a.b0[k + 1] = a.b0[k] + (int)mms::grid_for(n[k] / 4 + 1, 256, MMS_SUMSQ_GRID);
  }
  hipLaunchKernelGGL(sumsq_multi_kernel, dim3(a.b0[nseg]), dim3(256), 0, mms::as_stream(stream), a);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_adamw_dev_multi(int nseg, float* const* p, const float* const* g, float* const* m, float* const* v,
                                   const int64_t* n, const float* const* sumsq, const float* max_norm,
                                   const float* const* hyper, void* stream) {
  const char* fn = "mms_adamw_dev_multi";
  MMS_REQUIRE(nseg >= 1 && nseg <= kMaxSeg && p && g && m && v && n && sumsq && max_norm && hyper, fn,
              "1 to 8 segments");
  OptSegs a{};
  a.n = nseg;
  a.b0[0] = 0;
  for (int k = 0; k < nseg; ++k) {
    MMS_REQUIRE(n[k] >= 0 && hyper[k] != nullptr, fn, "null hyper-parameter buffer");
    MMS_REQUIRE(n[k] == 0 || (p[k] && g[k] && m[k] && v[k]), fn, "null buffer");
    a.p[k] = p[k];
    a.g[k] = g[k];
    a.m[k] = m[k];
    a.v[k] = v[k];
    a.len[k] = n[k];
    a.acc[k] = const_cast<float*>(sumsq[k]);
    a.max_norm[k] = max_norm[k];
    a.hyper[k] = hyper[k];
    a.b0[k + 1] = a.b0[k] + (int)mms::grid_for(n[k], 256, 8192);
  }
  hipLaunchKernelGGL(adamw_dev_multi_kernel, dim3(a.b0[nseg]), dim3(256), 0, mms::as_stream(stream), a);
  return mms::check_launch(fn);
}

namespace {
struct WSumArgs {
  float w[16];
};
// total = ((x0 w0 + x1 w1) + x2 w2) + ...: the reference's left-to-right sum of the weighted loss terms
// (LossManager.compute_loss, losses.py:224-265), one lane
__global__ void weighted_sum_kernel(const float* __restrict__ x, int n, WSumArgs a, float* __restrict__ out) {
  float t = x[0] * a.w[0];
  for (int i = 1; i < n; ++i) t += x[i] * a.w[i];
  out[0] = t;
}
}  // namespace

namespace {
// SingleVarianceNetwork's reported 1 / inv_variance = 1 / clip(exp(10 s), 1e-6, 1e6) (single_variance.py:34-36), the
// float operations of its torch form (mul, exp, clamp, reciprocal) in one thread
__global__ void inv_variance_kernel(const float* __restrict__ s, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float e = expf(s[0] * 10.0f);
    out[0] = 1.0f / fminf(fmaxf(e, 1e-6f), 1e6f);
  }
}
}  // namespace

MMS_EXPORT int mms_inv_variance(const float* s, float* out, void* stream) {
  const char* fn = "mms_inv_variance";
  MMS_REQUIRE(s && out, fn, "null pointer");
  hipLaunchKernelGGL(inv_variance_kernel, dim3(1), dim3(64), 0, mms::as_stream(stream), s, out);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_weighted_sum(const float* x, int n, const float* w, float* out, void* stream) {
  const char* fn = "mms_weighted_sum";
  MMS_REQUIRE(n >= 1 && n <= 16, fn, "1 to 16 terms");
  MMS_REQUIRE(x && w && out, fn, "null pointer");
  WSumArgs a{};
  for (int i = 0; i < n; ++i) a.w[i] = w[i];
  hipLaunchKernelGGL(weighted_sum_kernel, dim3(1), dim3(1), 0, mms::as_stream(stream), x, n, a, out);
  return mms::check_launch(fn);
}
