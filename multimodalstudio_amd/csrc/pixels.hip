// GPU-resident uniform pixel sampler: the training frames stay in HBM and every step's pixel draws, coordinates and
// target values are produced on the device -- no host sampling, no host-to-device copy, and the launch can sit in a
// captured graph (the draw counter lives in device memory and advances on the device).
//
// Reference: UniformPixelSampler.sample (/root/reference/src/cameras/pixel_samplers.py:71-89) over the cached frames
// of CacheDataloader (data/dataloaders.py:107-167): per modality, frame ~ U{0..n_frames-1}, x ~ U{0..W-1},
// y ~ U{0..H-1}; coordinates [frame_index, y, x] (int32) and values images[frame, y, x, :].  The draws here come
// from a counter-based generator (Philox4x32-10, key = seed, counter = (draw counter + i, stream)), so the sample
// STREAM differs from torch.Generator's -- the host sampler (pipeline.UniformPixelSampler) remains the bit-exact one;
// this one is statistically the same distribution (multiply-high mapping, bias < n / 2^32).
#include "common.h"

namespace {

__device__ __forceinline__ void philox_round(uint32_t (&c)[4], uint32_t (&k)[2]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
  const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
  const uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
  k[0] += 0x9E3779B9u;
  k[1] += 0xBB67AE85u;
}

__device__ __forceinline__ void philox4x32(uint64_t seed, uint64_t ctr, uint32_t stream, uint32_t (&out)[4]) {
  uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), stream, 0u};
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
#pragma unroll
  for (int r = 0; r < 10; ++r) philox_round(c, k);
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
}

__device__ __forceinline__ uint32_t below(uint32_t u, uint32_t n) { return __umulhi(u, n); }

// one thread per sampled pixel; draw order per pixel: frame, x, y (the reference's draw order per modality)
__global__ __launch_bounds__(256) void pixel_sample_kernel(uint64_t seed, uint32_t stream, const uint64_t* counter,
                                                           int64_t n, int n_frames, int H, int W,
                                                           const int32_t* frame_ids, const float* images, int C,
                                                           int32_t* coords, int64_t* sel, float* values) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t u[4];
  philox4x32(seed, *counter + (uint64_t)i, stream, u);
  const uint32_t f = below(u[0], (uint32_t)n_frames);
  const uint32_t x = below(u[1], (uint32_t)W);
  const uint32_t y = below(u[2], (uint32_t)H);
  coords[3 * i] = frame_ids ? frame_ids[f] : (int32_t)f;
  coords[3 * i + 1] = (int32_t)y;
  coords[3 * i + 2] = (int32_t)x;
  if (sel) sel[i] = f;
  if (values) {
    const float* px = images + (((int64_t)f * H + y) * W + x) * C;
    for (int c = 0; c < C; ++c) values[i * C + c] = px[c];
  }
}

__global__ void advance_kernel(uint64_t* counter, int64_t n) { *counter += (uint64_t)n; }

// U[0, 1) floats (24-bit mantissa draws), four per Philox call: out[i] from counter *counter + offset + i / 4
__global__ __launch_bounds__(256) void uniform_kernel(uint64_t seed, uint32_t stream, const uint64_t* counter,
                                                      int64_t offset, int64_t n, float* out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * q >= n) return;
  uint32_t u[4];
  philox4x32(seed, *counter + (uint64_t)offset + (uint64_t)q, stream, u);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (4 * q + j < n) out[4 * q + j] = (float)(u[j] >> 8) * (1.0f / 16777216.0f);
}

}  // namespace

MMS_EXPORT int mms_uniform(uint64_t seed, uint32_t stream_id, const uint64_t* counter, int64_t offset, int64_t n,
                           float* out, void* stream) {
  const char* fn = "mms_uniform";
  MMS_REQUIRE(n >= 0 && offset >= 0, fn, "bad sizes");
  MMS_REQUIRE(counter && (n == 0 || out), fn, "null pointer");
  if (n == 0) return 0;
  const int64_t calls = (n + 3) / 4;
  hipLaunchKernelGGL(uniform_kernel, dim3((unsigned)((calls + 255) / 256)), dim3(256), 0, mms::as_stream(stream), seed,
                     stream_id, counter, offset, n, out);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_counter_advance(uint64_t* counter, int64_t n, void* stream) {
  const char* fn = "mms_counter_advance";
  MMS_REQUIRE(counter, fn, "null pointer");
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, mms::as_stream(stream), counter, n);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_pixel_sample(uint64_t seed, uint32_t stream_id, uint64_t* counter, int64_t n, int n_frames, int H,
                                int W, const int32_t* frame_ids, const float* images, int C, int32_t* coords,
                                int64_t* sel, float* values, void* stream) {
  const char* fn = "mms_pixel_sample";
  MMS_REQUIRE(n >= 0 && n_frames > 0 && H > 0 && W > 0 && C > 0, fn, "bad shapes");
  MMS_REQUIRE(counter && coords, fn, "null pointer");
  MMS_REQUIRE(values == nullptr || images != nullptr, fn, "values need the frames");
  if (n == 0) return 0;
  hipStream_t s = mms::as_stream(stream);
  hipLaunchKernelGGL(pixel_sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, seed, stream_id, counter,
                     n, n_frames, H, W, frame_ids, images, C, coords, sel, values);
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, s, counter, n);
  return mms::check_launch(fn);
}
