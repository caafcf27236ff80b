// Narrow weight-normed linear layers (C <= 16 outputs) for gfx950: the background NeRF's density head
// (256 -> 1, Softplus; nerf_field.py:92-105 / field_heads.py:71-88) and the background modality heads
// (128 -> C, Sigmoid or none; background_model.py:101-109), forward and backward in one launch each.
//
// A 128 x 128-tile GEMM spends 127/128 of its MFMA work and a whole launch per pass on these (the round-3a trace:
// six mms_gemm launches, 0.22 ms per step serialized, 0.0002 of the MFMA peak); they are row-wise dot products and
// outer products, i.e. HBM-bound VALU work.  16 lanes own one row (lane q: columns [q KC, (q + 1) KC), KC = K / 16,
// float4 loads), the weights sit in LDS, sums over the 16 lanes by xor shuffles.  fp32 throughout (accurate
// transcendentals): at least the precision of every preset's GEMM mode.
//   forward:  Y[m, c] = act(sum_k X[m, k] W[c, k] + b[c])
//   backward: dz = dY * act'(Y) (act' from the OUTPUT: ReLU y > 0, Softplus 1 - exp(-beta y), Sigmoid y (1 - y));
//             dX[m, :] (+)= dz W;  dW += dz^T X, db += sum_m dz  (per-lane partials over the block's rows, reduced
//             over the lanes of each column chunk by shuffles and LDS, one atomic per element per block).
#include "common.h"

namespace {

constexpr int kMaxC = 16;
constexpr int kMaxK = 512;

__device__ __forceinline__ float act_out_grad(int act, float y, float beta, float thr) {
  switch (act) {
    case 1: return y > 0.f ? 1.f : 0.f;
    case 2: { const float by = y * beta; return by > thr ? 1.f : 1.0f - expf(-by); }
    case 3: return y * (1.0f - y);
    default: return 1.f;
  }
}

__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

template <int KC>
__device__ __forceinline__ void load_chunk(const float* __restrict__ row, int q, float (&x)[KC]) {
#pragma unroll
  for (int j = 0; j < KC; j += 4) {
    const float4 v = *reinterpret_cast<const float4*>(row + q * KC + j);
    x[j] = v.x; x[j + 1] = v.y; x[j + 2] = v.z; x[j + 3] = v.w;
  }
}

template <int KC>
__global__ __launch_bounds__(256) void small_linear_fwd_kernel(const float* __restrict__ X, int64_t ldx, int64_t M,
                                                               const float* __restrict__ W, const float* __restrict__ b,
                                                               int C, int act, float beta, float thr,
                                                               float* __restrict__ Y, int64_t ldy) {
  constexpr int K = 16 * KC;
  __shared__ __attribute__((aligned(16))) float sw[kMaxC][K];
  __shared__ float sb[kMaxC];
  for (int i = threadIdx.x; i < C * K; i += 256) sw[i / K][i % K] = W[i];
  if (threadIdx.x < C) sb[threadIdx.x] = b != nullptr ? b[threadIdx.x] : 0.f;
  __syncthreads();
  const int q = threadIdx.x & 15;
  for (int64_t m = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; m < M; m += (int64_t)gridDim.x * 16) {
    float x[KC];
    load_chunk<KC>(X + m * ldx, q, x);
    float mine = 0.f;
    for (int c = 0; c < C; ++c) {
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < KC; j += 4) {
        const float4 w = *reinterpret_cast<const float4*>(&sw[c][q * KC + j]);
        p = __builtin_fmaf(x[j], w.x, p);
        p = __builtin_fmaf(x[j + 1], w.y, p);
        p = __builtin_fmaf(x[j + 2], w.z, p);
        p = __builtin_fmaf(x[j + 3], w.w, p);
      }
      p = sum16(p);
      if (q == c) mine = p;
    }
    if (q < C) Y[m * ldy + q] = mms::act_fwd_exact(act, mine + sb[q], beta, thr);
  }
}

template <int KC, int CM>
__global__ __launch_bounds__(256) void small_linear_bwd_kernel(const float* __restrict__ X, int64_t ldx, int64_t M,
                                                               const float* __restrict__ W, int C, int act,
                                                               float beta, float thr, const float* __restrict__ Yo,
                                                               int64_t ldy, const float* __restrict__ dY,
                                                               int64_t lddy, float* __restrict__ dX, int64_t lddx,
                                                               int accumulate, float* __restrict__ dW,
                                                               float* __restrict__ db) {
  constexpr int K = 16 * KC;
  __shared__ __attribute__((aligned(16))) float sw[CM][K];
  __shared__ __attribute__((aligned(16))) float sred[4][CM][K];
  __shared__ float sdb[4][CM];
  for (int i = threadIdx.x; i < C * K; i += 256) sw[i / K][i % K] = W[i];
  __syncthreads();
  const int q = threadIdx.x & 15, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[CM][KC];
  float dbacc[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    dbacc[c] = 0.f;
#pragma unroll
    for (int j = 0; j < KC; ++j) acc[c][j] = 0.f;
  }
  // the block's rows are interleaved with the other blocks' (stride gridDim.x * 16); blocks_for_bwd sizes the grid so
  // each lane walks only a few rows and many rows' loads are in flight at once
  for (int64_t m = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; m < M; m += (int64_t)gridDim.x * 16) {
    float dz[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c)
      dz[c] = c < C ? dY[m * lddy + c] * act_out_grad(act, Yo[m * ldy + c], beta, thr) : 0.f;
    float x[KC];
    if (dW != nullptr) load_chunk<KC>(X + m * ldx, q, x);
    if (dX != nullptr) {
      float* xr = dX + m * lddx + q * KC;
#pragma unroll
      for (int j = 0; j < KC; j += 4) {
        float4 v = accumulate ? *reinterpret_cast<const float4*>(xr + j) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int c = 0; c < CM; ++c) {
          if (c < C) {
            const float4 w = *reinterpret_cast<const float4*>(&sw[c][q * KC + j]);
            v.x = __builtin_fmaf(dz[c], w.x, v.x);
            v.y = __builtin_fmaf(dz[c], w.y, v.y);
            v.z = __builtin_fmaf(dz[c], w.z, v.z);
            v.w = __builtin_fmaf(dz[c], w.w, v.w);
          }
        }
        *reinterpret_cast<float4*>(xr + j) = v;
      }
    }
    if (dW != nullptr) {
#pragma unroll
      for (int c = 0; c < CM; ++c)
#pragma unroll
        for (int j = 0; j < KC; ++j) acc[c][j] = __builtin_fmaf(dz[c], x[j], acc[c][j]);
    }
#pragma unroll
    for (int c = 0; c < CM; ++c) dbacc[c] += q == 0 ? dz[c] : 0.f;
  }
  // block reduction: the 4 row slots of a wave (lanes q, q + 16, q + 32, q + 48) by shuffles, then the 4 waves in LDS
#pragma unroll
  for (int c = 0; c < CM; ++c) {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      float v = acc[c][j];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      acc[c][j] = v;
    }
    float d = dbacc[c];
    d += __shfl_xor(d, 16);
    d += __shfl_xor(d, 32);
    dbacc[c] = d;
  }
  if (lane < 16) {
#pragma unroll
    for (int c = 0; c < CM; ++c) {
#pragma unroll
      for (int j = 0; j < KC; ++j) sred[wave][c][q * KC + j] = acc[c][j];
      if (q == 0) sdb[wave][c] = dbacc[c];
    }
  }
  __syncthreads();
  if (dW != nullptr)
    for (int i = threadIdx.x; i < C * K; i += 256) {
      const int c = i / K, k = i % K;
      atomicAdd(dW + i, ((sred[0][c][k] + sred[1][c][k]) + sred[2][c][k]) + sred[3][c][k]);
    }
  if (db != nullptr && threadIdx.x < C) {
    const int c = threadIdx.x;
    atomicAdd(db + c, ((sdb[0][c] + sdb[1][c]) + sdb[2][c]) + sdb[3][c]);
  }
}

// column sums of a [rows][ld] partials matrix: block (x = column chunk of 256, y = row slice), one atomic per column
__global__ __launch_bounds__(256) void rowsum_add_kernel(const float* __restrict__ src, int64_t rows, int64_t cols,
                                                         int64_t ld, float* __restrict__ dst_a, int64_t na,
                                                         float* __restrict__ dst_b) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = (int64_t)blockIdx.y * per, r1 = r0 + per < rows ? r0 + per : rows;
  float v = 0.f;
  for (int64_t r = r0; r < r1; ++r) v += src[r * ld + c];
  if (r1 > r0) atomicAdd(c < na ? dst_a + c : dst_b + (c - na), v);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

unsigned blocks_for(int64_t M) {
  int64_t b = (M + 63) / 64;
  if (b > 512) b = 512;
  return (unsigned)(b < 1 ? 1 : b);
}

// backward: about two rows per lane group (each block reduces its dW partials once, C K atomics per block)
unsigned blocks_for_bwd(int64_t M) {
  int64_t b = (M + 31) / 32;
  if (b > 2048) b = 2048;
  return (unsigned)(b < 1 ? 1 : b);
}

template <int KC, int CM>
void launch_bwd(unsigned g, hipStream_t s, const float* X, int64_t ldx, int64_t M, const float* W, int C, int act,
                float beta, float thr, const float* Y, int64_t ldy, const float* dY, int64_t lddy, float* dX,
                int64_t lddx, int accumulate, float* dW, float* db) {
  hipLaunchKernelGGL((small_linear_bwd_kernel<KC, CM>), dim3(g), dim3(256), 0, s, X, ldx, M, W, C, act, beta, thr, Y,
                     ldy, dY, lddy, dX, lddx, accumulate, dW, db);
}

}  // namespace

MMS_EXPORT int mms_small_linear_fwd(const float* X, int64_t ldx, int64_t M, int K, const float* W, const float* b,
                                    int C, int act, float beta, float thr, float* Y, int64_t ldy, void* stream) {
  const char* fn = "mms_small_linear_fwd";
  MMS_REQUIRE(C >= 1 && C <= kMaxC, fn, "1 to 16 outputs");
  MMS_REQUIRE(K == 128 || K == 256 || K == 512, fn, "K must be 128, 256 or 512");
  MMS_REQUIRE(act >= 0 && act <= 3, fn, "bad activation id");
  MMS_REQUIRE(M >= 0 && ldy >= C, fn, "bad shapes");
  if (M == 0) return 0;
  MMS_REQUIRE(X && W && Y, fn, "null pointer");
  MMS_REQUIRE(aligned16(X) && ldx % 4 == 0 && ldx >= K, fn, "input rows must be 16-B aligned");
  hipStream_t s = mms::as_stream(stream);
  const unsigned g = blocks_for(M);
  if (K == 128) hipLaunchKernelGGL(small_linear_fwd_kernel<8>, dim3(g), dim3(256), 0, s, X, ldx, M, W, b, C, act, beta, thr, Y, ldy);
  else if (K == 256) hipLaunchKernelGGL(small_linear_fwd_kernel<16>, dim3(g), dim3(256), 0, s, X, ldx, M, W, b, C, act, beta, thr, Y, ldy);
  else hipLaunchKernelGGL(small_linear_fwd_kernel<32>, dim3(g), dim3(256), 0, s, X, ldx, M, W, b, C, act, beta, thr, Y, ldy);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_small_linear_bwd(const float* X, int64_t ldx, int64_t M, int K, const float* W, int C, int act,
                                    float beta, float thr, const float* Y, int64_t ldy, const float* dY, int64_t lddy,
                                    float* dX, int64_t lddx, int accumulate, float* dW, float* db, void* stream) {
  const char* fn = "mms_small_linear_bwd";
  MMS_REQUIRE(C >= 1 && C <= kMaxC, fn, "1 to 16 outputs");
  MMS_REQUIRE(K == 128 || K == 256 || K == 512, fn, "K must be 128, 256 or 512");
  MMS_REQUIRE((K == 128 && C <= 16) || (K == 256 && C <= 8) || (K == 512 && C <= 4), fn,
              "C x K too large for the per-lane weight-gradient partials (K 128: C <= 16, 256: <= 8, 512: <= 4)");
  MMS_REQUIRE(act >= 0 && act <= 3, fn, "bad activation id");
  MMS_REQUIRE(M >= 0 && ldy >= C && lddy >= C, fn, "bad shapes");
  if (M == 0) return 0;
  MMS_REQUIRE(W && Y && dY, fn, "null pointer");
  MMS_REQUIRE(dW == nullptr || (X && aligned16(X) && ldx % 4 == 0 && ldx >= K), fn, "input rows must be 16-B aligned");
  MMS_REQUIRE(dX == nullptr || (aligned16(dX) && lddx % 4 == 0 && lddx >= K), fn, "dX rows must be 16-B aligned");
  hipStream_t s = mms::as_stream(stream);
  const unsigned g = blocks_for_bwd(M);
  // the per-lane partials are CM x KC registers: CM = the smallest of 1 / 4 / (8, 16) that holds C
#define MMS_SL_BWD(KC, CM) launch_bwd<KC, CM>(g, s, X, ldx, M, W, C, act, beta, thr, Y, ldy, dY, lddy, dX, lddx, \
                                              accumulate, dW, db)
  if (K == 128) {
    if (C == 1) MMS_SL_BWD(8, 1); else if (C <= 4) MMS_SL_BWD(8, 4); else MMS_SL_BWD(8, 16);
  } else if (K == 256) {
    if (C == 1) MMS_SL_BWD(16, 1); else if (C <= 4) MMS_SL_BWD(16, 4); else MMS_SL_BWD(16, 8);
  } else {
    if (C == 1) MMS_SL_BWD(32, 1); else MMS_SL_BWD(32, 4);
  }
#undef MMS_SL_BWD
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_rowsum_add(const float* src, int64_t rows, int64_t cols, int64_t ld, float* dst_a, int64_t na,
                              float* dst_b, void* stream) {
  const char* fn = "mms_rowsum_add";
  MMS_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols && na >= 0 && na <= cols, fn, "bad shapes");
  if (rows == 0 || cols == 0) return 0;
  MMS_REQUIRE(src && (na == 0 || dst_a) && (na == cols || dst_b), fn, "null pointer");
  const unsigned gx = (unsigned)((cols + 255) / 256);
  const unsigned gy = (unsigned)(rows < 64 ? rows : 64);
  hipLaunchKernelGGL(rowsum_add_kernel, dim3(gx, gy), dim3(256), 0, mms::as_stream(stream), src, rows, cols, ld, dst_a,
                     na, dst_b);
  return mms::check_launch(fn);
}
