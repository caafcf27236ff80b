// Weight-norm and reduction helpers around the MLP GEMMs.
//
//   weight_norm (torch.nn.utils.parametrizations.weight_norm, dim=0; /root/reference/src/field_components/mlp.py:206-209)
//     W[n, :] = v[n, :] * (g[n] / ||v[n, :]||)
//   backward:
//     dg[n]    = sum_k dW[n,k] v[n,k] / ||v_n||
//     dv[n, k] = (g/||v||) dW[n,k] - (g dg / ||v||^2) v[n,k]
//   colsum: db[n] += sum_m dZ[m, n]          (bias gradient)
//   act_bwd: dZ = dY * act'(Z)               (output-activation derivative)
#include "common.h"

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// one weight row n (a 256-thread block): the same reduction order for the single-layer and the batched launch
__device__ __forceinline__ void wn_row(const float* __restrict__ g, const float* __restrict__ v, int64_t n, int64_t K,
                                       float* __restrict__ W, int64_t ldw, float* __restrict__ norms, float* red) {
  const float* vr = v + n * K;
  float s = 0.f;
  for (int64_t k = threadIdx.x; k < K; k += blockDim.x) s += vr[k] * vr[k];
  s = block_sum(s, red);
  const float nrm = sqrtf(s);
  const float scale = g[n] / nrm;
  for (int64_t k = threadIdx.x; k < K; k += blockDim.x) W[n * ldw + k] = vr[k] * scale;
  if (threadIdx.x == 0 && norms) norms[n] = nrm;
}

__global__ __launch_bounds__(256) void wn_fwd_kernel(const float* __restrict__ g, const float* __restrict__ v,
                                                     int64_t N, int64_t K, float* __restrict__ W, int64_t ldw,
                                                     float* __restrict__ norms) {
  __shared__ float red[4];
  wn_row(g, v, blockIdx.x, K, W, ldw, norms, red);
}

// every layer of a model in one launch: block b handles row b - items[i].row0 of the item i it falls in
__global__ __launch_bounds__(256) void wn_fwd_batched_kernel(const MmsNormItem* __restrict__ items, int n_items) {
  __shared__ float red[4];
  int i = 0;
  while (i + 1 < n_items && (int64_t)blockIdx.x >= items[i + 1].row0) ++i;
  const MmsNormItem it = items[i];
  wn_row(it.g, it.v, (int64_t)blockIdx.x - it.row0, it.K, it.W, it.ldw, it.norms, red);
}

__device__ __forceinline__ void wn_bwd_row(const float* __restrict__ g, const float* __restrict__ v,
                                           const float* __restrict__ norms, int64_t n, int64_t K,
                                           const float* __restrict__ dW, int64_t lddw, float* __restrict__ dg,
                                           float* __restrict__ dv, float* red) {
  const float* vr = v + n * K;
  const float* dr = dW + n * lddw;
  float s = 0.f;
  for (int64_t k = threadIdx.x; k < K; k += blockDim.x) s += dr[k] * vr[k];
  s = block_sum(s, red);
  const float nrm = norms[n];
  const float dgn = s / nrm;
  const float a = g[n] / nrm;
  const float b = g[n] * dgn / (nrm * nrm);
  for (int64_t k = threadIdx.x; k < K; k += blockDim.x) dv[n * K + k] += a * dr[k] - b * vr[k];
  if (threadIdx.x == 0) dg[n] += dgn;
}

__global__ __launch_bounds__(256) void wn_bwd_kernel(const float* __restrict__ g, const float* __restrict__ v,
                                                     const float* __restrict__ norms, int64_t N, int64_t K,
                                                     const float* __restrict__ dW, int64_t lddw,
                                                     float* __restrict__ dg, float* __restrict__ dv) {
  __shared__ float red[4];
  wn_bwd_row(g, v, norms, blockIdx.x, K, dW, lddw, dg, dv, red);
}

// all of a backward's weight-norm gradients in one launch; the item list travels by value in the kernel arguments
// (graph-capturable with no device table: every step's dW buffers are new allocations)
constexpr int kMaxWnBwd = 32;
struct WnBwdBatch {
  MmsWnBwdItem it[kMaxWnBwd];
  int n;
};

__global__ __launch_bounds__(256) void wn_bwd_batched_kernel(WnBwdBatch b) {
  __shared__ float red[4];
  int i = 0;
  while (i + 1 < b.n && (int64_t)blockIdx.x >= b.it[i + 1].row0) ++i;
  const MmsWnBwdItem& it = b.it[i];
  wn_bwd_row(it.g, it.v, it.norms, (int64_t)blockIdx.x - it.row0, it.K, it.dW, it.lddw, it.dg, it.dv, red);
}

// db[n] += sum over rows; blockDim = 256 columns-chunk, grid.x = column chunks, grid.y = row splits
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ A, int64_t M, int64_t N, int64_t lda,
                                                     float* __restrict__ out, int64_t rows_per) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += A[r * lda + n];
  atomicAdd(out + n, s);
}

// act ids as common.h act_grad_fast: 0 none, 1 relu, 2 softplus(beta, thr), 3 sigmoid
__global__ void act_bwd_kernel(const float* __restrict__ dY, int64_t ldy, const float* __restrict__ Z, int64_t ldz,
                               int64_t M, int64_t N, int act, float beta, float thr, float* __restrict__ dZ,
                               int64_t lddz) {
  const int64_t total = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, n = i - m * N;
    const float z = Z[m * ldz + n];
    dZ[m * lddz + n] = dY[m * ldy + n] * mms::act_grad_exact(act, z, beta, thr);
  }
}

}  // namespace

MMS_EXPORT int mms_weight_norm_bwd_batched(const void* items, int n_items, int64_t total_rows, void* stream) {
  const char* fn = "mms_weight_norm_bwd_batched";
  MMS_REQUIRE(items && n_items > 0 && n_items <= kMaxWnBwd && total_rows > 0, fn, "1 .. 32 items per batch");
  WnBwdBatch b;
  memcpy(b.it, items, sizeof(MmsWnBwdItem) * n_items);
  b.n = n_items;
  hipLaunchKernelGGL(wn_bwd_batched_kernel, dim3((unsigned)total_rows), dim3(256), 0, mms::as_stream(stream), b);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_weight_norm_fwd_batched(const void* items, int n_items, int64_t total_rows, void* stream) {
  const char* fn = "mms_weight_norm_fwd_batched";
  MMS_REQUIRE(items && n_items > 0 && total_rows > 0, fn, "empty batch");
  hipLaunchKernelGGL(wn_fwd_batched_kernel, dim3((unsigned)total_rows), dim3(256), 0, mms::as_stream(stream),
                     reinterpret_cast<const MmsNormItem*>(items), n_items);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_weight_norm_fwd(const float* g, const float* v, int64_t N, int64_t K, float* W, int64_t ldw,
                                   float* norms, void* stream) {
  const char* fn = "mms_weight_norm_fwd";
  MMS_REQUIRE(N >= 0 && K > 0 && ldw >= K, fn, "bad shape");
  if (N == 0) return 0;
  hipLaunchKernelGGL(wn_fwd_kernel, dim3((unsigned)N), dim3(256), 0, mms::as_stream(stream), g, v, N, K, W, ldw, norms);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_weight_norm_bwd(const float* g, const float* v, const float* norms, int64_t N, int64_t K,
                                   const float* dW, int64_t lddw, float* dg, float* dv, void* stream) {
  const char* fn = "mms_weight_norm_bwd";
  MMS_REQUIRE(N >= 0 && K > 0 && lddw >= K, fn, "bad shape");
  if (N == 0) return 0;
  hipLaunchKernelGGL(wn_bwd_kernel, dim3((unsigned)N), dim3(256), 0, mms::as_stream(stream), g, v, norms, N, K, dW,
                     lddw, dg, dv);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_colsum(const float* A, int64_t M, int64_t N, int64_t lda, float* out, void* stream) {
  const char* fn = "mms_colsum";
  MMS_REQUIRE(M >= 0 && N >= 0 && lda >= N, fn, "bad shape");
  if (M == 0 || N == 0) return 0;
  const int64_t chunks_n = (N + 255) / 256;
  int64_t splits = (M + 511) / 512;
  if (splits > 4096) splits = 4096;
  const int64_t rows_per = (M + splits - 1) / splits;
  splits = (M + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)chunks_n, (unsigned)splits), dim3(256), 0, mms::as_stream(stream),
                     A, M, N, lda, out, rows_per);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_act_bwd(const float* dY, int64_t ldy, const float* Z, int64_t ldz, int64_t M, int64_t N, int act,
                           float beta, float thr, float* dZ, int64_t lddz, void* stream) {
  const char* fn = "mms_act_bwd";
  MMS_REQUIRE(act >= 0 && act <= 4, fn, "bad activation");
  if (M == 0 || N == 0) return 0;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(mms::grid_for(M * N, 256, 8192)), dim3(256), 0, mms::as_stream(stream), dY,
                     ldy, Z, ldz, M, N, act, beta, thr, dZ, lddz);
  return mms::check_launch(fn);
}
