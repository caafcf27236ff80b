// MLP GEMM engine for gfx950: C[M,N] = epilogue(A . B^T) with A, B given either k-contiguous
// ([rows][K], "N" source) or row-contiguous ([K][rows], "T" source), so one kernel serves
//   forward          Y  = act(X W^T + b)    A = X  [M,K] (N),  B = W  [N,K] (N)
//   backward data    dX = dZ W              A = dZ [M,Nout] (N), B = W seen as [K=Nout][N=Kin] (T)
//   backward weight  dW = dZ^T X            A = dZ seen as [K=rows][M=Nout] (T), B = X [K=rows][N=Kin] (T)
// (the nn.Linear layers of /root/reference/src/field_components/mlp.py:152-171).
//
// Precision modes (template PREC):
//   F32    v_mfma_f32_32x32x2_f32  — exact fp32 (bitwise an fmaf chain); the parity mode
//   BF16   v_mfma_f32_32x32x16_bf16 on RNE-rounded operands, fp32 accumulate
//   BF16X3 split operands x = hi + lo (both bf16); acc += hi.hi + hi.lo + lo.hi  (~2^-16 relative
//          operand precision, fp32 accumulate) — 16x/3 the f32-MFMA rate at near-fp32 accuracy, used
//          for the SDF MLP whose 4-tap finite differences need the extra mantissa.
//
// Tiling: 128x128 block tile, BK = 32, 256 threads = 2x2 waves of 64x64 (2x2 MFMA 32x32 tiles/wave).
// Operands are register-prefetched one k-step ahead with 16-byte loads and staged in LDS k-contiguous
// per row ([row][BK+pad]); fragments are one ds_read_b32 (F32, pad 1: conflict-free) or two
// ds_read_b128 (BF16*, pad 4: 16-B aligned, conflict-free per 16-lane group).  The block -> tile map
// keeps the N-tiles of one M panel on one XCD (ids b and b+8), so the A panel is fetched into one L2.
// Split-K over grid.z accumulates with hardware f32 atomics (tall-skinny weight gradients).
#include "common.h"

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

enum Prec { P_F32 = 0, P_BF16 = 1, P_BF16X3 = 2 };
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SOFTPLUS = 2, ACT_SIGMOID = 3 };

constexpr int BM = 128, BN = 128, BK = 32;

template <int PREC>
struct LdsK {
  static constexpr int v = (PREC == P_F32) ? (BK + 1) : (BK + 4);
};

struct Epi {
  const float* bias;
  float* Z;
  int64_t ldz;
  const float* aux;
  int64_t ldaux;
  int act, dact;
  float beta, thr;
  int accumulate;
  int ones_col;  // >= 0: also write 1.0 at C[row, ones_col] (bias-gradient column for the next TN GEMM)
};

__device__ __forceinline__ float act_fwd(int act, float v, float beta, float thr) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_SOFTPLUS: { const float bx = v * beta; return bx > thr ? v : log1pf(expf(bx)) / beta; }
    case ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}

__device__ __forceinline__ float act_grad(int act, float z, float beta, float thr) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_SOFTPLUS: { const float bx = z * beta; if (bx > thr) return 1.f; const float e = expf(bx); return e / (e + 1.0f); }
    case ACT_SIGMOID: { const float s = 1.0f / (1.0f + expf(-z)); return s * (1.0f - s); }
    default: return 1.f;
  }
}

// ---------------------------------------------------------------------------- staging
// N source ([rows][K], k contiguous): 1024 float4 per 128x32 tile, thread t covers idx = t + 256 i:
//   row = idx >> 3, kc = idx & 7  -> 8 lanes read one row's 128 contiguous bytes.
// T source ([K][rows], rows contiguous): kr = (idx & 7) | ((idx >> 8) << 3), cc = (idx >> 3) & 31.
template <bool T, bool VEC>
__device__ __forceinline__ void stage_load(const float* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                           int64_t k0, int64_t kmax, float4 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + 256 * i;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!T) {
      const int64_t r = r0 + (idx >> 3), k = k0 + 4 * (idx & 7);
      if (VEC) {
        if (r < rmax && k < kmax) v = *reinterpret_cast<const float4*>(src + r * ld + k);
      } else if (r < rmax) {
        const float* p = src + r * ld + k;
        if (k < kmax) v.x = p[0];
        if (k + 1 < kmax) v.y = p[1];
        if (k + 2 < kmax) v.z = p[2];
        if (k + 3 < kmax) v.w = p[3];
      }
    } else {
      const int64_t k = k0 + ((idx & 7) | ((idx >> 8) << 3)), r = r0 + 4 * ((idx >> 3) & 31);
      if (VEC) {
        if (k < kmax && r < rmax) v = *reinterpret_cast<const float4*>(src + k * ld + r);
      } else if (k < kmax) {
        const float* p = src + k * ld + r;
        if (r < rmax) v.x = p[0];
        if (r + 1 < rmax) v.y = p[1];
        if (r + 2 < rmax) v.z = p[2];
        if (r + 3 < rmax) v.w = p[3];
      }
    }
    reg[i] = v;
  }
}

template <bool T, int LDK>
__device__ __forceinline__ void stage_store(float* lds, const float4 (&reg)[4]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + 256 * i;
    if (!T) {
      float* p = lds + (idx >> 3) * LDK + 4 * (idx & 7);
      if (LDK % 4 == 0) {
        *reinterpret_cast<float4*>(p) = reg[i];
      } else {
        p[0] = reg[i].x; p[1] = reg[i].y; p[2] = reg[i].z; p[3] = reg[i].w;
      }
    } else {
      const int kr = (idx & 7) | ((idx >> 8) << 3), c = 4 * ((idx >> 3) & 31);
      float* p = lds + c * LDK + kr;
      p[0] = reg[i].x; p[LDK] = reg[i].y; p[2 * LDK] = reg[i].z; p[3 * LDK] = reg[i].w;
    }
  }
}

__device__ __forceinline__ bf16x8 to_bf16(const float4 lo, const float4 hi) {
  bf16x8 r;
  r[0] = (__bf16)lo.x; r[1] = (__bf16)lo.y; r[2] = (__bf16)lo.z; r[3] = (__bf16)lo.w;
  r[4] = (__bf16)hi.x; r[5] = (__bf16)hi.y; r[6] = (__bf16)hi.z; r[7] = (__bf16)hi.w;
  return r;
}

__device__ __forceinline__ void split_bf16(const float4 lo, const float4 hi, bf16x8& h, bf16x8& l) {
  h = to_bf16(lo, hi);
  float4 rlo, rhi;
  rlo.x = lo.x - (float)h[0]; rlo.y = lo.y - (float)h[1]; rlo.z = lo.z - (float)h[2]; rlo.w = lo.w - (float)h[3];
  rhi.x = hi.x - (float)h[4]; rhi.y = hi.y - (float)h[5]; rhi.z = hi.z - (float)h[6]; rhi.w = hi.w - (float)h[7];
  l = to_bf16(rlo, rhi);
}

template <int PREC, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                   int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                   float* __restrict__ C, int64_t ldc, Epi ep, int64_t k_per_split,
                                                   int m_tiles_pad, int n_tiles) {
  constexpr int LDK = LdsK<PREC>::v;
  __shared__ __attribute__((aligned(16))) float lds[(BM + BN) * LDK];
  float* As = lds;
  float* Bs = lds + BM * LDK;

  // XCD-aware tile map: ids b and b + 8 (same XCD under round-robin dispatch) take the N-tiles of one M panel
  const int id = blockIdx.x;
  const int nt = (id >> 3) % n_tiles;
  const int mt = (id & 7) + 8 * (id / (8 * n_tiles));
  if (mt >= m_tiles_pad) return;
  const int64_t m0 = (int64_t)mt * BM;
  const int64_t n0 = (int64_t)nt * BN;
  if (m0 >= M) return;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = (kbeg + k_per_split < K) ? kbeg + k_per_split : K;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  float4 ra[4], rb[4];
  if (kbeg < kend) {
    stage_load<TA, VEC>(A, lda, m0, M, kbeg, kend, ra);
    stage_load<TB, VEC>(B, ldb, n0, N, kbeg, kend, rb);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    stage_store<TA, LDK>(As, ra);
    stage_store<TB, LDK>(Bs, rb);
    __syncthreads();
    if (k0 + BK < kend) {
      stage_load<TA, VEC>(A, lda, m0, M, k0 + BK, kend, ra);
      stage_load<TB, VEC>(B, ldb, n0, N, k0 + BK, kend, rb);
    }
    const float* a0p = As + (wm * 64 + r) * LDK;
    const float* a1p = As + (wm * 64 + 32 + r) * LDK;
    const float* b0p = Bs + (wn * 64 + r) * LDK;
    const float* b1p = Bs + (wn * 64 + 32 + r) * LDK;
    if (PREC == P_F32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const float a0 = a0p[kk + h], a1 = a1p[kk + h], b0 = b0p[kk + h], b1 = b1p[kk + h];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK; ks += 16) {
        const int kb = ks + 8 * h;
        const float4 a0l = *reinterpret_cast<const float4*>(a0p + kb), a0h = *reinterpret_cast<const float4*>(a0p + kb + 4);
        const float4 a1l = *reinterpret_cast<const float4*>(a1p + kb), a1h = *reinterpret_cast<const float4*>(a1p + kb + 4);
        const float4 b0l = *reinterpret_cast<const float4*>(b0p + kb), b0h = *reinterpret_cast<const float4*>(b0p + kb + 4);
        const float4 b1l = *reinterpret_cast<const float4*>(b1p + kb), b1h = *reinterpret_cast<const float4*>(b1p + kb + 4);
        if (PREC == P_BF16) {
          const bf16x8 A0 = to_bf16(a0l, a0h), A1 = to_bf16(a1l, a1h);
          const bf16x8 B0 = to_bf16(b0l, b0h), B1 = to_bf16(b1l, b1h);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1, acc[1][1], 0, 0, 0);
        } else {
          bf16x8 A0h, A0l, A1h, A1l, B0h, B0l, B1h, B1l;
          split_bf16(a0l, a0h, A0h, A0l);
          split_bf16(a1l, a1h, A1h, A1l);
          split_bf16(b0l, b0h, B0h, B0l);
          split_bf16(b1l, b1h, B1h, B1l);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0l, B0h, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0l, B1h, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1l, B0h, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1l, B1h, acc[1][1], 0, 0, 0);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0h, B0l, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0h, B1l, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1h, B0l, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1h, B1l, acc[1][1], 0, 0, 0);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0h, B0h, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0h, B1h, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1h, B0h, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1h, B1h, acc[1][1], 0, 0, 0);
        }
      }
    }
  }

  // epilogue: 32x32 C/D map (all dtypes): col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn * 64 + j * 32 + r;
      if (col >= N) continue;
      const float bval = (ep.bias != nullptr && !split) ? ep.bias[col] : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t row = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row >= M) continue;
        float v = acc[i][j][e] + bval;
        if (ep.Z != nullptr) ep.Z[row * ep.ldz + col] = v;
        if (ep.act != ACT_NONE) v = act_fwd(ep.act, v, ep.beta, ep.thr);
        if (ep.aux != nullptr) v *= act_grad(ep.dact, ep.aux[row * ep.ldaux + col], ep.beta, ep.thr);
        float* dst = C + row * ldc + col;
        if (split) atomicAdd(dst, v);
        else if (ep.accumulate) *dst += v;
        else *dst = v;
        if (ep.ones_col >= 0 && col == 0) C[row * ldc + ep.ones_col] = 1.0f;
      }
    }
  }
}

template <int PREC, bool TA, bool TB>
int launch(bool vec, dim3 grid, hipStream_t s, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
           const float* B, int64_t ldb, float* C, int64_t ldc, Epi ep, int64_t kps, int mtp, int nt) {
  if (vec)
    hipLaunchKernelGGL((gemm_kernel<PREC, TA, TB, true>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, ep,
                       kps, mtp, nt);
  else
    hipLaunchKernelGGL((gemm_kernel<PREC, TA, TB, false>), grid, dim3(256), 0, s, M, N, K, A, lda, B, ldb, C, ldc, ep,
                       kps, mtp, nt);
  return 0;
}

template <int PREC>
int dispatch_ta_tb(bool ta, bool tb, bool vec, dim3 grid, hipStream_t s, int64_t M, int64_t N, int64_t K,
                   const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, Epi ep,
                   int64_t kps, int mtp, int nt) {
  if (!ta && !tb) return launch<PREC, false, false>(vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, mtp, nt);
  if (!ta && tb) return launch<PREC, false, true>(vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, mtp, nt);
  if (ta && tb) return launch<PREC, true, true>(vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, mtp, nt);
  return launch<PREC, true, false>(vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kps, mtp, nt);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

MMS_EXPORT int mms_gemm(int prec, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                        int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, float* Z,
                        int64_t ldz, const float* aux, int64_t ldaux, int act, int dact, float beta, float thr,
                        int accumulate, int splits, int ones_col, void* stream) {
  const char* fn = "mms_gemm";
  MMS_REQUIRE(prec >= 0 && prec <= 2, fn, "prec must be 0 (f32), 1 (bf16) or 2 (bf16x3)");
  MMS_REQUIRE(M >= 0 && N >= 0 && K >= 0, fn, "negative size");
  MMS_REQUIRE(act >= 0 && act <= 3 && dact >= 0 && dact <= 3, fn, "bad activation id");
  if (M == 0 || N == 0) return 0;
  MMS_REQUIRE(A && B && C, fn, "null operand");
  if (splits < 1) splits = 1;
  MMS_REQUIRE(splits == 1 || (accumulate && Z == nullptr && aux == nullptr && act == ACT_NONE && bias == nullptr &&
                              ones_col < 0),
              fn, "split-K requires a plain accumulating epilogue");
  // vector path: 16-B aligned bases, contiguous dims and leading dims multiples of 4
  const int64_t acont = trans_a ? M : K, bcont = trans_b ? N : K;
  const bool vec = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0 && acont % 4 == 0 && bcont % 4 == 0;
  int64_t kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  if (kps < BK) kps = BK;
  const int64_t zs = K == 0 ? 1 : (K + kps - 1) / kps;
  MMS_REQUIRE(zs <= 65535, fn, "too many K splits");
  const int64_t mt = (M + BM - 1) / BM;
  const int64_t mtp = ((mt + 7) / 8) * 8;
  const int64_t nt = (N + BN - 1) / BN;
  MMS_REQUIRE(mtp * nt <= INT32_MAX, fn, "grid too large");
  Epi ep{bias, Z, ldz, aux, ldaux, act, dact, beta, thr, accumulate, ones_col};
  dim3 grid((unsigned)(mtp * nt), 1, (unsigned)zs);
  hipStream_t s = mms::as_stream(stream);
  switch (prec) {
    case P_F32: dispatch_ta_tb<P_F32>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, K == 0 ? 0 : kps, (int)mtp, (int)nt); break;
    case P_BF16: dispatch_ta_tb<P_BF16>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, K == 0 ? 0 : kps, (int)mtp, (int)nt); break;
    default: dispatch_ta_tb<P_BF16X3>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, K == 0 ? 0 : kps, (int)mtp, (int)nt); break;
  }
  return mms::check_launch(fn);
}
