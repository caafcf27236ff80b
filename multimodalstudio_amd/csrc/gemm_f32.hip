// fp32-exact GEMM on gfx950 matrix cores (v_mfma_f32_32x32x2_f32) with fused MLP epilogues.
//
// This is the parity-mode engine for every nn.Linear of the reference MLPs
// (/root/reference/src/field_components/mlp.py:152-171): Y = act(X W^T + b).  The f32-input MFMA is
// bitwise an fmaf chain (no reduced-precision path), so it reproduces fp32 PyTorch numerics up to
// summation order.
//
//   mode NT: C[M,N] = A[M,K] * B[N,K]^T        forward           (A = X, B = W)
//   mode NN: C[M,N] = A[M,K] * B[K,N]          backward data     (A = dZ, B = W  [N_out, K_in])
//   mode TN: C[M,N] = A[K,M]^T * B[K,N]        backward weights  (A = dZ, B = X; K = rows)
//
// Block tile 128x128x16, 256 threads = 2x2 waves of 64x64 (2x2 MFMA 32x32 tiles per wave).
// Operands are staged through LDS k-major so every fragment read is one conflict-free ds_read_b32;
// global tiles are register-prefetched one k-step ahead.  Split-K (grid.z) accumulates with
// hardware f32 atomics (used for the tall-skinny TN reductions over millions of samples).
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16, PAD = 4;
constexpr int LDA_S = BM + PAD, LDB_S = BN + PAD;

enum Mode { NT = 0, NN = 1, TN = 2 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SOFTPLUS = 2, ACT_SIGMOID = 3 };

struct Epi {
  const float* bias;   // [N] or null
  float* Z;            // store pre-activation (acc + bias) or null
  int64_t ldz;
  const float* aux;    // backward: multiply by act'(aux[m, n]) (aux = pre-activation) or null
  int64_t ldaux;
  int act;             // forward activation applied to output
  int dact;            // derivative applied with aux
  float beta, thr;     // softplus parameters
  int accumulate;      // 0: C = v; 1: C += v (atomic when split-K)
};

__device__ __forceinline__ float act_fwd(int act, float v, float beta, float thr) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_SOFTPLUS: {
      const float bx = v * beta;
      return bx > thr ? v : log1pf(expf(bx)) / beta;
    }
    case ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ float act_grad(int act, float z, float beta, float thr) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_SOFTPLUS: {
      const float bx = z * beta;
      if (bx > thr) return 1.f;
      const float e = expf(bx);
      return e / (e + 1.0f);
    }
    case ACT_SIGMOID: {
      const float s = 1.0f / (1.0f + expf(-z));
      return s * (1.0f - s);
    }
    default: return 1.f;
  }
}

// Load one operand tile (16 k x 128 {m|n}) into registers.
//  transposed_src: source row-major [rows(m|n), K] with leading dim ld -> element (k, r) at r*ld + k
//  otherwise:      source row-major [K, cols] -> element (k, r) at k*ld + r
template <bool TRANS_SRC>
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                          int64_t k0, int64_t kmax, float (&reg)[8]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = t + 256 * i;
    int kk, rr;
    if (TRANS_SRC) { rr = e >> 4; kk = e & 15; }   // 16 consecutive k of one row per 16 lanes
    else           { kk = e >> 7; rr = e & 127; }  // 128 consecutive columns of one k-row
    const int64_t r = r0 + rr, k = k0 + kk;
    reg[i] = (r < rmax && k < kmax) ? src[TRANS_SRC ? (r * ld + k) : (k * ld + r)] : 0.f;
  }
}

template <bool TRANS_SRC>
__device__ __forceinline__ void store_tile(float* lds, int lds_ld, const float (&reg)[8]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int e = t + 256 * i;
    int kk, rr;
    if (TRANS_SRC) { rr = e >> 4; kk = e & 15; }
    else           { kk = e >> 7; rr = e & 127; }
    lds[kk * lds_ld + rr] = reg[i];
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void gemm_f32_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                       int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                       float* __restrict__ C, int64_t ldc, Epi ep,
                                                       int64_t k_per_split) {
  __shared__ float As[BK * LDA_S];
  __shared__ float Bs[BK * LDB_S];
  // A source: NT/NN -> A row-major [M, K] (transposed staging); TN -> A row-major [K, M] (direct)
  constexpr bool A_TRANS = (MODE != TN);
  // B source: NT -> B row-major [N, K] (transposed staging); NN/TN -> B row-major [K, N] (direct)
  constexpr bool B_TRANS = (MODE == NT);

  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int64_t n0 = (int64_t)blockIdx.y * BN;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = (kbeg + k_per_split < K) ? kbeg + k_per_split : K;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float ra[8], rb[8];
  if (kbeg < kend) {
    load_tile<A_TRANS>(A, lda, m0, M, kbeg, kend, ra);
    load_tile<B_TRANS>(B, ldb, n0, N, kbeg, kend, rb);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    store_tile<A_TRANS>(As, LDA_S, ra);
    store_tile<B_TRANS>(Bs, LDB_S, rb);
    __syncthreads();
    if (k0 + BK < kend) {
      load_tile<A_TRANS>(A, lda, m0, M, k0 + BK, kend, ra);
      load_tile<B_TRANS>(B, ldb, n0, N, k0 + BK, kend, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int krow = kk + (lane >> 5);
      float a0 = As[krow * LDA_S + wm * 64 + (lane & 31)];
      float a1 = As[krow * LDA_S + wm * 64 + 32 + (lane & 31)];
      float b0 = Bs[krow * LDB_S + wn * 64 + (lane & 31)];
      float b1 = Bs[krow * LDB_S + wn * 64 + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }

  // epilogue: C/D map of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= N) continue;
      const float bval = (ep.bias != nullptr && !split) ? ep.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        float v = acc[i][j][r] + bval;
        if (ep.Z != nullptr) ep.Z[row * ep.ldz + col] = v;
        if (ep.act != ACT_NONE) v = act_fwd(ep.act, v, ep.beta, ep.thr);
        if (ep.aux != nullptr) v *= act_grad(ep.dact, ep.aux[row * ep.ldaux + col], ep.beta, ep.thr);
        float* dst = C + row * ldc + col;
        if (split) atomicAdd(dst, v);
        else if (ep.accumulate) *dst += v;
        else *dst = v;
      }
    }
  }
}

}  // namespace

// C = epilogue(op(A) op(B)); see header for argument meaning.
MMS_EXPORT int mms_gemm_f32(int mode, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                            const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, float* Z,
                            int64_t ldz, const float* aux, int64_t ldaux, int act, int dact, float beta,
                            float thr, int accumulate, int splits, void* stream) {
  const char* fn = "mms_gemm_f32";
  MMS_REQUIRE(mode >= 0 && mode <= 2, fn, "mode must be 0 (NT), 1 (NN) or 2 (TN)");
  MMS_REQUIRE(M >= 0 && N >= 0 && K >= 0, fn, "negative size");
  MMS_REQUIRE(act >= 0 && act <= 3 && dact >= 0 && dact <= 3, fn, "bad activation id");
  if (M == 0 || N == 0) return 0;
  MMS_REQUIRE(A && B && C, fn, "null operand");
  if (splits < 1) splits = 1;
  MMS_REQUIRE(splits == 1 || (accumulate && Z == nullptr && aux == nullptr && act == ACT_NONE && bias == nullptr),
              fn, "split-K requires a plain accumulating epilogue");
  int64_t kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  if (kps < BK) kps = BK;
  const int64_t zs = K == 0 ? 1 : (K + kps - 1) / kps;
  Epi ep{bias, Z, ldz, aux, ldaux, act, dact, beta, thr, accumulate};
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + BN - 1) / BN), (unsigned)zs);
  MMS_REQUIRE((N + BN - 1) / BN <= 65535 && zs <= 65535, fn, "N or split count too large");
  hipStream_t s = mms::as_stream(stream);
  if (K == 0) {
    // degenerate: epilogue over zero accumulators (bias only)
    kps = 0;
  }
  switch (mode) {
    case NT: hipLaunchKernelGGL(gemm_f32_kernel<NT>, grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps); break;
    case NN: hipLaunchKernelGGL(gemm_f32_kernel<NN>, grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps); break;
    default: hipLaunchKernelGGL(gemm_f32_kernel<TN>, grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps); break;
  }
  return mms::check_launch(fn);
}
