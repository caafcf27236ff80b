// Ray-sampling kernels: stratified bins, spacing -> euclidean samples (+ backward to near/far and
// the ray), and the NeuS importance up-sampling step.
//
// Reference (paths under /root/reference/src/model_components/ray_samplers.py):
//   SpacedSampler.generate_ray_samples :183-233   (uniform: g = id, disparity: g = 1/x)
//   spacing_to_euclidean_fn             :178-181   e = g^-1(g(far) b + g(near) (1 - b))
//   NeuSSampler.generate_ray_samples    :464-514   4 iterations, inv_s = 64 * 2^i
//   rendering_sdf_with_fixed_inv_s      :516-551
//   PDFSampler.generate_ray_samples     :357-403   (include_original=False, padding 1e-5, single jitter)
//   merge_ray_samples                   :38-68     (sort of the two start lists + max end)
// and cameras/rays.py:201-217 (weights from alphas), :69-81 (start positions o + d * start).
//
// Bin values depend only on float32 arithmetic performed in the reference's order (no contraction): the
// transmittance product and the CDF are sequential in double like torch.cumprod / cumsum on CPU, the weight sum
// follows ATen's vectorised CPU reduction order and the sigmoid is torch's CPU SLEEF form (common.h), so bins,
// searchsorted indices and the merge order (sorted_index) equal the reference's bit for bit
// (tests/test_gpu_sampler.py against tests/golden/neus_sampler.npz).
#include "common.h"

#pragma clang fp contract(off)

namespace {

// torch.sigmoid exactly as the reference's CPU path computes it (common.h: SLEEF expf_u10 + IEEE division)
__device__ __forceinline__ float sigm(float x) { return mms::torch_cpu_sigmoid(x); }

// stratified bins: lin [S+1]; t either per ray ([R,1], tstride=1, tcols=1) or per bin ([R, S+1])
__global__ void stratified_bins_kernel(const float* __restrict__ lin, int nb, const float* __restrict__ t, int tcols,
                                       int64_t R, float* __restrict__ bins) {
  const int64_t total = R * nb;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / nb;
    const int k = (int)(e - r * nb);
    if (t == nullptr) { bins[e] = lin[k]; continue; }
    const float tk = t[r * tcols + (tcols == 1 ? 0 : k)];
    // centers c_k = (b_{k+1} + b_k) / 2 ; upper = [c_0..c_{n-2}, b_{n-1}] ; lower = [b_0, c_0..c_{n-2}]
    const float upper = (k < nb - 1) ? (lin[k + 1] + lin[k]) / 2.0f : lin[nb - 1];
    const float lower = (k > 0) ? (lin[k] + lin[k - 1]) / 2.0f : lin[0];
    bins[e] = lower + (upper - lower) * tk;
  }
}

__device__ __forceinline__ float to_euclid(float b, float nr, float fr, int kind) {
  if (kind == 0) return fr * b + nr * (1 - b);
  const float sn = 1.0f / nr, sf = 1.0f / fr;
  return 1.0f / (sf * b + sn * (1 - b));
}

// de/dnear, de/dfar for a bin value b
__device__ __forceinline__ void euclid_grad(float b, float nr, float fr, int kind, float& dn, float& df) {
  if (kind == 0) { dn = 1 - b; df = b; return; }
  const float sn = 1.0f / nr, sf = 1.0f / fr;
  const float A = sf * b + sn * (1 - b);
  const float iA2 = 1.0f / (A * A);
  dn = iA2 * (1 - b) / (nr * nr);
  df = iA2 * b / (fr * fr);
}

// bins [R, nb] (ldb) -> starts/ends/deltas [R, S = nb-1] and positions [R*S, 3]
__global__ void samples_fwd_kernel(const float* __restrict__ bins, int64_t ldb, int nb, const float* __restrict__ nears,
                                   const float* __restrict__ fars, const float* __restrict__ origins,
                                   const float* __restrict__ dirs, int kind, int64_t R, float* __restrict__ starts,
                                   float* __restrict__ ends, float* __restrict__ deltas, float* __restrict__ pos) {
  const int S = nb - 1;
  const int64_t total = R * S;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / S;
    const int k = (int)(e - r * S);
    const float nr = nears[r], fr = fars[r];
    const float s0 = to_euclid(bins[r * ldb + k], nr, fr, kind);
    const float s1 = to_euclid(bins[r * ldb + k + 1], nr, fr, kind);
    if (starts) starts[e] = s0;
    if (ends) ends[e] = s1;
    if (deltas) deltas[e] = s1 - s0;
    if (pos) {
      const float* o = origins + r * 3;
      const float* d = dirs + r * 3;
      pos[e * 3] = o[0] + d[0] * s0;
      pos[e * 3 + 1] = o[1] + d[1] * s0;
      pos[e * 3 + 2] = o[2] + d[2] * s0;
    }
  }
}

// backward: one wave per ray, lane = bin edge (nb <= 65: the last edge handled by lane 0)
__global__ __launch_bounds__(256) void samples_bwd_kernel(const float* __restrict__ bins, int64_t ldb, int nb,
                                                          const float* __restrict__ nears,
                                                          const float* __restrict__ fars,
                                                          const float* __restrict__ dirs, int kind, int64_t R,
                                                          const float* __restrict__ dpos,
                                                          const float* __restrict__ ddeltas,
                                                          const float* __restrict__ dstarts,
                                                          float* __restrict__ dnears, float* __restrict__ dfars,
                                                          float* __restrict__ dorigins, float* __restrict__ ddirs) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const int S = nb - 1;
  const float nr = nears[r], fr = fars[r];
  const float* d = dirs + r * 3;
  float gn = 0.f, gf = 0.f, go0 = 0.f, go1 = 0.f, go2 = 0.f, gd0 = 0.f, gd1 = 0.f, gd2 = 0.f;
  for (int k = lane; k < nb; k += 64) {
    const float b = bins[r * ldb + k];
    const float e = to_euclid(b, nr, fr, kind);
    float de = 0.f;
    if (k < S) {
      const int64_t i = r * S + k;
      if (dpos) {
        const float p0 = dpos[i * 3], p1 = dpos[i * 3 + 1], p2 = dpos[i * 3 + 2];
        go0 += p0; go1 += p1; go2 += p2;
        gd0 += p0 * e; gd1 += p1 * e; gd2 += p2 * e;
        de += p0 * d[0] + p1 * d[1] + p2 * d[2];
      }
      if (ddeltas) de -= ddeltas[i];
      if (dstarts) de += dstarts[i];
    }
    if (k > 0 && ddeltas) de += ddeltas[r * S + k - 1];
    float dn, df;
    euclid_grad(b, nr, fr, kind, dn, df);
    gn += de * dn;
    gf += de * df;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    gn += __shfl_xor(gn, o); gf += __shfl_xor(gf, o);
    go0 += __shfl_xor(go0, o); go1 += __shfl_xor(go1, o); go2 += __shfl_xor(go2, o);
    gd0 += __shfl_xor(gd0, o); gd1 += __shfl_xor(gd1, o); gd2 += __shfl_xor(gd2, o);
  }
  if (lane == 0) {
    if (dnears) dnears[r] += gn;
    if (dfars) dfars[r] += gf;
    if (dorigins) { dorigins[r * 3] += go0; dorigins[r * 3 + 1] += go1; dorigins[r * 3 + 2] += go2; }
    if (ddirs) { ddirs[r * 3] += gd0; ddirs[r * 3 + 1] += gd1; ddirs[r * 3 + 2] += gd2; }
  }
}

// ------------------------------------------------------------------ NeuS up-sampling step (one wave per ray)
// Lane k owns sample k: its sdf gather, section cosine, the two sigmoids and alpha run in parallel across the wave.
// The transmittance cumprod, the weight sum and the CDF cumsum keep the reference's sequential double order: every
// lane runs the same uniform loop over the broadcast values, so the results are those of a single sequential thread
// bit for bit.  The inverse-CDF lookups (lane j = new bin j) and the stable merge (each element's output slot = its
// own index + the number of elements of the other list before it) are parallel again.  One wave per ray spreads a
// step over every CU (a thread per ray kept a ~1700-ray step on 27 waves).
constexpr int kMaxBins = 64;   // samples + 1 edges per ray held on the lanes
constexpr int kWavesPerBlock = 4;

// the wave's LDS writes are visible to its later LDS reads (program order within one wave; no compiler reordering)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(256) void neus_step_kernel(
    int64_t R, int S, const float* __restrict__ bins, const float* __restrict__ sdf_prev, int s_prev,
    const float* __restrict__ sdf_new, int n_prev_new, const int* __restrict__ prev_idx,
    const float* __restrict__ nears, const float* __restrict__ fars, float inv_s, const float* __restrict__ rand,
    const float* __restrict__ u_lin, int n_new, float* __restrict__ sdf_out, float* __restrict__ new_bins,
    float* __restrict__ merged_bins, int* __restrict__ sorted_idx) {
  __shared__ float s_b[kWavesPerBlock][kMaxBins];     // bin edges b[0..S]
  __shared__ float s_w[kWavesPerBlock][kMaxBins];     // padded weights, then the CDF (cdf[0..S])
  __shared__ float s_n[kWavesPerBlock][kMaxBins];     // new bins
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + wv;
  if (r >= R) return;                                  // wave-uniform
  float* sb = s_b[wv];
  float* sw = s_w[wv];
  float* sn = s_n[wv];
  const float* b = bins + r * (S + 1);
  const float bk = lane <= S ? b[lane] : 0.f;
  if (lane <= S) sb[lane] = bk;
  // (a) merged sdf for the current samples
  float sdf_k = 0.f;
  if (lane < S) {
    if (prev_idx) {
      const int id = prev_idx[r * S + lane];
      sdf_k = id < s_prev ? sdf_prev[r * s_prev + id] : sdf_new[r * n_prev_new + (id - s_prev)];
    } else {
      sdf_k = sdf_new[r * S + lane];
    }
    sdf_out[r * S + lane] = sdf_k;
  }
  const float nr = nears[r], fr = fars[r];
  // (b-d) section k = [k, k+1] (k < S - 1): cosine with the previous section's, alpha
  const float e_k = fr * bk + nr * (1 - bk);
  const float e_n = __shfl_down(e_k, 1);
  const float sdf_n = __shfl_down(sdf_k, 1);
  const float dl = e_n - e_k;
  const float mid = (sdf_k + sdf_n) * 0.5f;
  const float cs = (sdf_n - sdf_k) / (dl + 1e-5f);
  float prev_cos = __shfl_up(cs, 1);
  if (lane == 0) prev_cos = 0.0f;
  float cmin = fminf(prev_cos, cs);
  cmin = fminf(fmaxf(cmin, -1e3f), 0.0f);
  const float pe = mid - cmin * dl * 0.5f;
  const float ne = mid + cmin * dl * 0.5f;
  float alpha = 0.f;
  if (lane < S - 1) {
    const float pc = sigm(pe * inv_s), nc = sigm(ne * inv_s);
    alpha = (pc - nc + 1e-5f) / (pc + 1e-5f);
  }
  // sequential transmittance (torch.cumprod on CPU: double accumulation, float outputs), uniform across the wave
  double T = 1.0;
  float w_k = 0.0f;   // w_{S-1} = 0
  for (int k = 0; k < S - 1; ++k) {
    const float a = __shfl(alpha, k);
    const float w = a * (float)T;
    if (lane == k) w_k = w;
    T = T * (double)(1.0f - a + 1e-7f);
  }
  // (e) pdf / cdf with padding 1e-5 (histogram_padding) and eps 1e-5
  const float wp = w_k + 1e-5f;
  if (lane < S) sw[lane] = wp;
  wave_sync();
  // torch.sum(weights, -1) in ATen's CPU summation order (not sequential), so weights_sum has the same bits
  float wsum = mms::torch_cpu_row_sum(sw, S);
  const float pad = fmaxf(1e-5f - wsum, 0.f);
  const float padk = pad / (float)S;
  wsum = wsum + pad;
  double run = 0.0;
  float cdf_k1 = 0.f;   // lane k: cdf[k + 1]
  for (int k = 0; k < S; ++k) {
    const float w = __shfl(wp, k) + padk;
    run = run + (double)(w / wsum);
    if (lane == k) cdf_k1 = fminf(1.0f, (float)run);
  }
  // cdf[0] = 0, cdf[k + 1] from lane k (the weights above are consumed: the array is reused)
  wave_sync();
  if (lane < S) sw[lane + 1] = cdf_k1;
  if (lane == 0) sw[0] = 0.f;
  wave_sync();
  // (f-g) inverse CDF at u_j = lin_j + rand / nb (searchsorted right), lane j = new bin j
  const int nb = n_new + 1;
  // training: u_j = lin_j + rand / nb (single jitter); eval: u_j = lin_j + 1 / (2 nb) (ray_samplers.py:365-377)
  const float rj = rand ? rand[r] / (float)nb : (float)(1.0 / (2.0 * nb));
  float nbo = 0.f;
  if (lane < nb) {
    const float u = u_lin[lane] + rj;
    int lo = 0, hi = S + 1;  // first index with cdf > u
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (sw[m] > u) hi = m; else lo = m + 1;
    }
    const int inds = lo;
    const int below = min(max(inds - 1, 0), S);
    const int above = min(max(inds, 0), S);
    const float c0 = sw[below], c1 = sw[above];
    const float b0 = sb[below], b1 = sb[above];
    float t = (u - c0) / (c1 - c0);
    if (isnan(t)) t = 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);
    nbo = b0 + t * (b1 - b0);
    new_bins[r * nb + lane] = nbo;
    sn[lane] = nbo;
  }
  wave_sync();
  // (h) stable merge of the start lists (ties: the first list first); end = max of the ends
  float* mb = merged_bins + r * (S + n_new + 1);
  int* si = sorted_idx + r * (S + n_new);
  if (lane < S) {
    int before = 0;
    for (int j = 0; j < n_new; ++j) before += sn[j] < bk;
    mb[lane + before] = bk;
    si[lane + before] = lane;
  }
  if (lane < n_new) {
    int before = 0;
    for (int i = 0; i < S; ++i) before += sb[i] <= nbo;
    mb[lane + before] = nbo;
    si[lane + before] = S + lane;
  }
  if (lane == 0) mb[S + n_new] = fmaxf(sb[S], sn[n_new]);
}

}  // namespace

MMS_EXPORT int mms_stratified_bins(const float* lin, int nb, const float* t, int tcols, int64_t R, float* bins,
                                   void* stream) {
  const char* fn = "mms_stratified_bins";
  if (R == 0) return 0;
  hipLaunchKernelGGL(stratified_bins_kernel, dim3(mms::grid_for(R * nb, 256, 16384)), dim3(256), 0,
                     mms::as_stream(stream), lin, nb, t, tcols, R, bins);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_samples_fwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars,
                               const float* origins, const float* dirs, int kind, int64_t R, float* starts, float* ends,
                               float* deltas, float* pos, void* stream) {
  const char* fn = "mms_samples_fwd";
  MMS_REQUIRE(nb >= 2, fn, "need at least two bin edges");
  if (R == 0) return 0;
  hipLaunchKernelGGL(samples_fwd_kernel, dim3(mms::grid_for(R * (nb - 1), 256, 16384)), dim3(256), 0,
                     mms::as_stream(stream), bins, ldb, nb, nears, fars, origins, dirs, kind, R, starts, ends, deltas,
                     pos);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_samples_bwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars,
                               const float* dirs, int kind, int64_t R, const float* dpos, const float* ddeltas,
                               const float* dstarts, float* dnears, float* dfars, float* dorigins, float* ddirs,
                               void* stream) {
  const char* fn = "mms_samples_bwd";
  if (R == 0) return 0;
  hipLaunchKernelGGL(samples_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), bins, ldb, nb, nears, fars, dirs, kind, R, dpos, ddeltas, dstarts, dnears,
                     dfars, dorigins, ddirs);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_neus_step(int64_t R, int S, const float* bins, const float* sdf_prev, int s_prev,
                             const float* sdf_new, int n_prev_new, const int* prev_idx, const float* nears,
                             const float* fars, float inv_s, const float* rand, const float* u_lin, int n_new,
                             float* sdf_out, float* new_bins, float* merged_bins, int* sorted_idx, void* stream) {
  const char* fn = "mms_neus_step";
  MMS_REQUIRE(S >= 2 && S + 1 <= kMaxBins && n_new + 1 <= kMaxBins, fn, "sample count out of range (one wave per ray)");
  if (R == 0) return 0;
  hipLaunchKernelGGL(neus_step_kernel, dim3((unsigned)((R + kWavesPerBlock - 1) / kWavesPerBlock)),
                     dim3(64 * kWavesPerBlock), 0, mms::as_stream(stream), R, S, bins, sdf_prev, s_prev, sdf_new,
                     n_prev_new, prev_idx, nears, fars, inv_s, rand, u_lin, n_new, sdf_out, new_bins, merged_bins,
                     sorted_idx);
  return mms::check_launch(fn);
}
