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
//   BF16X3 split operands x = hi + lo (both bf16); acc += lo.hi + hi.lo + hi.hi  (~2^-16 relative
//          operand precision, fp32 accumulate) — 16x/3 the f32-MFMA rate at near-fp32 accuracy, used
//          for the SDF MLP whose 4-tap finite differences need the extra mantissa.
//
// Tiling: 128x128 block tile, 256 threads = 2x2 waves of 64x64 (2x2 MFMA 32x32 tiles per wave).
// Operands are register-prefetched one k-step ahead with 16-byte loads and staged in LDS already in
// the MFMA input format (f32, or bf16 / bf16 hi+lo converted once per element at staging):
//   N source -> [row][BK + pad] image, fragments by ds_read_b32 (F32) / ds_read_b128 (bf16)
//   T source -> [k][128 + pad] image (no transpose on the way in), fragments by ds_read_b32 (F32:
//               consecutive lanes read consecutive rows) / ds_read_b64_tr_b16 (bf16: the hardware
//               transposing read delivers 4 k-values of one row per lane; two reads per 32x32x16 fragment).
// BK = 32 (F32, BF16X3) or 64 (BF16).  The block -> tile map keeps the N-tiles of one M panel on one XCD
// (ids b and b+8); split-K (small outputs, long K: weight gradients) folds the K slice into blockIdx.x
// and accumulates with hardware f32 atomics.
#include "common.h"

#include <type_traits>
#include <utility>

// Diagnostic ablation builds only (scripts/gemm_ablate.py compiles them separately; the product library is
// built with 0): bit 0 drops the epilogue stores, bit 1 the MFMAs, bit 2 the global loads.
#ifndef MMS_GEMM_ABLATE
#define MMS_GEMM_ABLATE 0
#endif
// Diagnostic ablation builds of the wide weight-gradient kernel (scripts/wide_ablate.py; the product library is built
// with 0): bit 0 drops the output atomics, bit 1 the MFMAs, bit 2 the global loads, bit 3 the LDS image stores.
#ifndef MMS_WIDE_ABLATE
#define MMS_WIDE_ABLATE 0
#endif
#ifndef MMS_WIDE_PIPE
#define MMS_WIDE_PIPE 1   // the wide kernel's two-register-set pipeline (scripts/wide_ablate.py variants pipe*)
#endif
#ifndef MMS_GEMM_XCDSPLIT
#define MMS_GEMM_XCDSPLIT 1
#endif

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4_ __attribute__((ext_vector_type(4)));
typedef short short8_ __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short4_ lds_short4;

enum Prec { P_F32 = 0, P_BF16 = 1, P_BF16X3 = 2, P_F16 = 5 };   // P_F16: the wide weight-gradient kernel only
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SOFTPLUS = 2, ACT_SIGMOID = 3 };

constexpr int BM = 128, BN = 128;

// ---------------------------------------------------------------------------- per-precision geometry
template <int PREC>
struct Geo {
  static constexpr int BK = (PREC == P_BF16) ? 64 : 32;
  using elem = typename std::conditional<PREC == P_F32, float, __bf16>::type;
  static constexpr int NIMG = (PREC == P_BF16X3) ? 2 : 1;          // hi (+ lo) images per operand
  // N image: [128][LDN]; T image: [BK][LDT]  (elements)
  static constexpr int LDN = (PREC == P_F32) ? BK + 1 : BK + 8;     // f32: odd stride; bf16: 16-B rows
  static constexpr int LDT = (PREC == P_F32) ? 128 + 4 : 128 + 32;  // bf16: 320-B rows, tr reads conflict-free
  template <bool T>
  static constexpr int img_elems() { return T ? BK * LDT : 128 * LDN; }
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
  int splits;    // K slices folded into blockIdx.x
  float* colsum; // TA only: colsum[m] += sum_k A[k][m] (bias gradient of the weight-gradient GEMM), or null
};

// ---------------------------------------------------------------------------- global -> registers
// NV = float4 per thread per operand tile = 128 * BK / 4 / 256 = BK / 8.
// N source ([rows][K]): idx = t + 256 i -> row = idx / (BK/4), kc = idx % (BK/4)  (a row's BK floats by BK/4 lanes)
// T source ([K][rows]): idx -> k = idx / 32, c = idx % 32                         (a k-row's 128 floats by 32 lanes)
template <int BK, bool T, bool VEC>
__device__ __forceinline__ uint32_t stage_load(const float* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                               int64_t k0, int64_t kmax, float4 (&reg)[BK / 8]) {
  // Branch-free: every load is issued unconditionally from a clamped (always valid) address; the validity of
  // each element is returned as a bit mask and applied by stage_store, i.e. at the consumer, so the loads stay
  // in flight across the compute phase.  (A load under a per-element condition makes hipcc wait vmcnt(0)
  // inside each branch, and a select right after the load waits for it: both serialise the tile's loads.)
  // VEC: 16-B aligned rows (ld % 4 == 0, so a float4 starting below the row length stays inside the row).
  const int t = threadIdx.x;
  uint32_t mask = 0;
#pragma unroll
  for (int i = 0; i < BK / 8; ++i) {
    const int idx = t + 256 * i;
    // (outer, inner): N source (row, k) with inner bound kmax; T source (k, row) with inner bound rmax
    const int64_t o = T ? k0 + idx / 32 : r0 + idx / (BK / 4);
    const int64_t in = T ? r0 + 4 * (idx % 32) : k0 + 4 * (idx % (BK / 4));
    const int64_t omax = T ? kmax : rmax, inmax = T ? rmax : kmax;
    const bool ok = o < omax;
    const float* row = src + (ok ? o : omax - 1) * ld;
    float4 v;
    if (VEC) {
      const int64_t last = (inmax - 1) & ~(int64_t)3;
      v = *reinterpret_cast<const float4*>(row + (in < inmax ? in : last));
    } else {
      v.x = row[in < inmax ? in : inmax - 1];
      v.y = row[in + 1 < inmax ? in + 1 : inmax - 1];
      v.z = row[in + 2 < inmax ? in + 2 : inmax - 1];
      v.w = row[in + 3 < inmax ? in + 3 : inmax - 1];
    }
    const int64_t nin = ok ? inmax - in : 0;   // valid elements in this float4
    const uint32_t m4 = nin >= 4 ? 15u : (nin <= 0 ? 0u : ((1u << nin) - 1u));
    mask |= m4 << (4 * i);
    reg[i] = v;
  }
  return mask;
}

__device__ __forceinline__ bf16x4 cvt4(const float4 v) {
  bf16x4 r;
  r[0] = (__bf16)v.x; r[1] = (__bf16)v.y; r[2] = (__bf16)v.z; r[3] = (__bf16)v.w;
  return r;
}

__device__ __forceinline__ float4 resid4(const float4 v, const bf16x4 h) {
  return make_float4(v.x - (float)h[0], v.y - (float)h[1], v.z - (float)h[2], v.w - (float)h[3]);
}

// ---------------------------------------------------------------------------- registers -> LDS image(s)
template <int PREC, bool T>
__device__ __forceinline__ void stage_store(typename Geo<PREC>::elem* img, float4 (&reg)[Geo<PREC>::BK / 8],
                                            uint32_t mask) {
  using G = Geo<PREC>;
  constexpr int BK = G::BK;
  const int t = threadIdx.x;
  if (mask != (BK / 8 == 8 ? 0xffffffffu : ((1u << (4 * (BK / 8))) - 1u))) {   // edge tile: zero invalid elements
#pragma unroll
    for (int i = 0; i < BK / 8; ++i) {
      const uint32_t m = mask >> (4 * i);
      reg[i].x = (m & 1u) ? reg[i].x : 0.f;
      reg[i].y = (m & 2u) ? reg[i].y : 0.f;
      reg[i].z = (m & 4u) ? reg[i].z : 0.f;
      reg[i].w = (m & 8u) ? reg[i].w : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < BK / 8; ++i) {
    const int idx = t + 256 * i;
    const int off = T ? (idx / 32) * G::LDT + 4 * (idx % 32) : (idx / (BK / 4)) * G::LDN + 4 * (idx % (BK / 4));
    if constexpr (PREC == P_F32) {
      float* p = img + off;
      if (T) {
        *reinterpret_cast<float4*>(p) = reg[i];
      } else {
        p[0] = reg[i].x; p[1] = reg[i].y; p[2] = reg[i].z; p[3] = reg[i].w;
      }
    } else {
      const bf16x4 hi = cvt4(reg[i]);
      *reinterpret_cast<bf16x4*>(img + off) = hi;
      if constexpr (PREC == P_BF16X3) {
        *reinterpret_cast<bf16x4*>(img + G::template img_elems<T>() + off) = cvt4(resid4(reg[i], hi));
      }
    }
  }
}

// ---------------------------------------------------------------------------- LDS -> MFMA fragments
// bf16 32x32x16 operand fragment for rows [row0, row0+32), k-step ks: lane l holds X[row0 + (l&31)][ks + 8(l>>5) + j].
template <bool T, int LDN, int LDT>
__device__ __forceinline__ bf16x8 frag_bf16(const __bf16* img, int row0, int ks) {
  const int lane = threadIdx.x & 63;
  if (!T) {
    return *reinterpret_cast<const bf16x8*>(img + (row0 + (lane & 31)) * LDN + ks + 8 * (lane >> 5));
  } else {
    // ds_read_b64_tr_b16: per 16-lane group g, lane 4q+p addresses k-row (kb + q), columns 4p..4p+3 of the
    // group's 16-row block; lane i of the group receives row (block + i) at k = kb + 0..3.
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int kb = ks + 8 * (g >> 1);
    const __bf16* a = img + (kb + q) * LDT + row0 + 16 * (g & 1) + 4 * p;
    const short4_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a));
    const short4_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a + 4 * LDT));
    const short8_ v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// f32 32x32x2 operand: lane l holds X[row0 + (l&31)][kk + (l>>5)]
template <bool T, int LDN, int LDT>
__device__ __forceinline__ float frag_f32(const float* img, int row0, int kk) {
  const int lane = threadIdx.x & 63;
  if (!T) return img[(row0 + (lane & 31)) * LDN + kk + (lane >> 5)];
  return img[(kk + (lane >> 5)) * LDT + row0 + (lane & 31)];
}

// ---------------------------------------------------------------------------- epilogue
// one 32x32 accumulator tile -> C (bias, Z = pre-activation, activation, aux act-grad, store/accumulate/atomic).
// C/D map (all dtypes): col = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5).
// Activations: the fp32 parity mode keeps the accurate libm forms; the bf16 modes use the hardware
// transcendentals (common.h act_fwd_fast: the accurate forms made a 270k x 256 epilogue compute-bound).
template <int PREC>
__device__ __forceinline__ void epi_tile(const floatx16& a, int64_t rbase, int64_t col, int64_t M, int64_t N,
                                         float* __restrict__ C, int64_t ldc, const Epi& ep) {
  if (col >= N) return;
  const bool split = ep.splits > 1;
  const float bval = (ep.bias != nullptr && !split) ? ep.bias[col] : 0.f;
  // operands the epilogue reads (activation-gradient aux, or C for a read-modify-write) are loaded for all
  // 16 rows first, unconditionally from clamped rows, so they issue back to back (see stage_load)
  float rd[16];
  const bool rmw = ep.accumulate && !split;
  if (ep.aux != nullptr || rmw) {
    const float* base = ep.aux != nullptr ? ep.aux : C;
    const int64_t ld = ep.aux != nullptr ? ep.ldaux : ldc;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t row = rbase + (e & 3) + 8 * (e >> 2);
      rd[e] = base[(row < M ? row : M - 1) * ld + col];
    }
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t row = rbase + (e & 3) + 8 * (e >> 2);
    if (row < M) {
      float v = a[e] + bval;
      if (ep.Z != nullptr && ((MMS_GEMM_ABLATE & 1) == 0 || v == 1234.5f)) ep.Z[row * ep.ldz + col] = v;
      if (ep.act != ACT_NONE)
        v = PREC == P_F32 ? mms::act_fwd_exact(ep.act, v, ep.beta, ep.thr) : mms::act_fwd_fast(ep.act, v, ep.beta, ep.thr);
      if (ep.aux != nullptr)
        v *= PREC == P_F32 ? mms::act_grad_exact(ep.dact, rd[e], ep.beta, ep.thr)
                           : mms::act_grad_fast(ep.dact, rd[e], ep.beta, ep.thr);
      float* dst = C + row * ldc + col;
      if ((MMS_GEMM_ABLATE & 1) && v != 1234.5f) continue;
      if (split) atomicAdd(dst, v);
      else if (rmw) *dst = rd[e] + v;
      else *dst = v;
      if (ep.ones_col >= 0 && col == 0) C[row * ldc + ep.ones_col] = 1.0f;
    }
  }
}

// ---------------------------------------------------------------------------- kernel
// split-K tile map: id -> (tile, slice).  XCD-grouped: the tiles of one K slice share an XCD (ids x, x + 8, x + 16, ...
// under round-robin dispatch), so the slice's rows -- read by every tile of its row / column -- come from HBM into that
// XCD's L2 once; the slices spread over the 8 XCDs (the slice count is padded to a multiple of 8 at launch).
// Returns false for a padding id.
__device__ __forceinline__ bool split_map(int id, int m_tiles_pad, int n_tiles, int splits, int& mt, int& nt,
                                          int& slice) {
  const int tiles = m_tiles_pad * n_tiles;
#if MMS_GEMM_XCDSPLIT
  const int j = id >> 3;
  const int t = j % tiles;
  slice = (j / tiles) * 8 + (id & 7);
  if (slice >= splits) return false;
#else
  const int t = id % tiles;
  slice = id / tiles;
#endif
  mt = t % m_tiles_pad;
  nt = t / m_tiles_pad;
  return true;
}

// one 128 x 128 output tile (mt, nt) over K slice `slice`
template <int PREC, bool TA, bool TB, bool VEC>
__device__ __forceinline__ void gemm_block(int mt, int nt, int slice, int64_t M, int64_t N, int64_t K,
                                           const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                           int64_t ldb, float* __restrict__ C, int64_t ldc, const Epi& ep,
                                           int64_t k_per_split) {
  using G = Geo<PREC>;
  using E = typename G::elem;
  constexpr int BK = G::BK;
  constexpr int A_ELEMS = G::NIMG * G::template img_elems<TA>();
  constexpr int B_ELEMS = G::NIMG * G::template img_elems<TB>();
  __shared__ __attribute__((aligned(16))) E lds[A_ELEMS + B_ELEMS];
  E* As = lds;
  E* Bs = lds + A_ELEMS;

  const int64_t m0 = (int64_t)mt * BM;
  const int64_t n0 = (int64_t)nt * BN;
  if (m0 >= M) return;
  const int64_t kbeg = (int64_t)slice * k_per_split;
  const int64_t kend = (kbeg + k_per_split < K) ? kbeg + k_per_split : K;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  floatx16 acc00 = {}, acc01 = {}, acc10 = {}, acc11 = {};

  // fused bias gradient (TA): a T-source thread always holds columns 4 (t % 32) .. +3 of its k-rows
  const bool do_cs = TA && ep.colsum != nullptr && nt == 0;
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  auto colsum_acc = [&](const float4 (&reg)[BK / 8]) {
#pragma unroll
    for (int i = 0; i < BK / 8; ++i) {
      cs.x += reg[i].x; cs.y += reg[i].y; cs.z += reg[i].z; cs.w += reg[i].w;
    }
  };

  const int ar0 = wm * 64, br0 = wn * 64;
  auto compute = [&]() {
    if constexpr ((MMS_GEMM_ABLATE & 2) != 0) {
      acc00[0] += (float)As[lane] + (float)Bs[lane];  // keep the staging alive
    } else if constexpr (PREC == P_F32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const float a0 = frag_f32<TA, G::LDN, G::LDT>(As, ar0, kk), a1 = frag_f32<TA, G::LDN, G::LDT>(As, ar0 + 32, kk);
        const float b0 = frag_f32<TB, G::LDN, G::LDT>(Bs, br0, kk), b1 = frag_f32<TB, G::LDN, G::LDT>(Bs, br0 + 32, kk);
        acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc11, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK; ks += 16) {
        const bf16x8 a0 = frag_bf16<TA, G::LDN, G::LDT>(As, ar0, ks), a1 = frag_bf16<TA, G::LDN, G::LDT>(As, ar0 + 32, ks);
        const bf16x8 b0 = frag_bf16<TB, G::LDN, G::LDT>(Bs, br0, ks), b1 = frag_bf16<TB, G::LDN, G::LDT>(Bs, br0 + 32, ks);
        if constexpr (PREC == P_BF16X3) {
          constexpr int AO = G::template img_elems<TA>(), BO = G::template img_elems<TB>();
          const bf16x8 a0l = frag_bf16<TA, G::LDN, G::LDT>(As + AO, ar0, ks);
          const bf16x8 a1l = frag_bf16<TA, G::LDN, G::LDT>(As + AO, ar0 + 32, ks);
          const bf16x8 b0l = frag_bf16<TB, G::LDN, G::LDT>(Bs + BO, br0, ks);
          const bf16x8 b1l = frag_bf16<TB, G::LDN, G::LDT>(Bs + BO, br0 + 32, ks);
          acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0l, b0, acc00, 0, 0, 0);
          acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0l, b1, acc01, 0, 0, 0);
          acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1l, b0, acc10, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1l, b1, acc11, 0, 0, 0);
          acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0l, acc00, 0, 0, 0);
          acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1l, acc01, 0, 0, 0);
          acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0l, acc10, 0, 0, 0);
          acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1l, acc11, 0, 0, 0);
        }
        acc00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc00, 0, 0, 0);
        acc01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc01, 0, 0, 0);
        acc10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc10, 0, 0, 0);
        acc11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc11, 0, 0, 0);
      }
    }
  };

  float4 ra[BK / 8], rb[BK / 8];
  uint32_t ma = 0, mb = 0;
  if (kbeg < kend) {
    ma = stage_load<BK, TA, VEC>(A, lda, m0, M, kbeg, kend, ra);
    mb = stage_load<BK, TB, VEC>(B, ldb, n0, N, kbeg, kend, rb);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    stage_store<PREC, TA>(As, ra, ma);
    stage_store<PREC, TB>(Bs, rb, mb);
    if (do_cs) colsum_acc(ra);
    __syncthreads();
    if (k0 + BK < kend) {
      ma = stage_load<BK, TA, VEC>(A, lda, m0, M, k0 + BK, kend, ra);
      mb = stage_load<BK, TB, VEC>(B, ldb, n0, N, k0 + BK, kend, rb);
    }
    compute();
  }

  if (do_cs) {  // reduce the 8 threads sharing t % 32 through LDS, then one atomic per column
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
    const int t = threadIdx.x;
    *reinterpret_cast<float4*>(red + (t >> 5) * 128 + 4 * (t & 31)) = cs;
    __syncthreads();
    if (t < 128 && m0 + t < M) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) v += red[j * 128 + t];
      atomicAdd(ep.colsum + m0 + t, v);
    }
  }

  const int64_t rbase = m0 + wm * 64 + 4 * (lane >> 5);
  const int64_t cbase = n0 + wn * 64 + (lane & 31);
  epi_tile<PREC>(acc00, rbase, cbase, M, N, C, ldc, ep);
  epi_tile<PREC>(acc01, rbase, cbase + 32, M, N, C, ldc, ep);
  epi_tile<PREC>(acc10, rbase + 32, cbase, M, N, C, ldc, ep);
  epi_tile<PREC>(acc11, rbase + 32, cbase + 32, M, N, C, ldc, ep);
}

template <int PREC, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(256) void gemm_kernel(int64_t M, int64_t N, int64_t K, const float* __restrict__ A,
                                                   int64_t lda, const float* __restrict__ B, int64_t ldb,
                                                   float* __restrict__ C, int64_t ldc, Epi ep, int64_t k_per_split,
                                                   int m_tiles_pad, int n_tiles) {
  // Unsplit: XCD-aware -- ids b and b + 8 (same XCD under round-robin dispatch) take the N-tiles of one M panel, so
  // the panel is fetched into one L2.  Split-K: split_map.
  const int id = blockIdx.x;
  int mt, nt, slice = 0;
  if (ep.splits > 1) {
    if (!split_map(id, m_tiles_pad, n_tiles, ep.splits, mt, nt, slice)) return;
  } else {
    nt = (id >> 3) % n_tiles;
    mt = (id & 7) + 8 * (id / (8 * n_tiles));
    if (mt >= m_tiles_pad) return;
  }
  gemm_block<PREC, TA, TB, VEC>(mt, nt, slice, M, N, K, A, lda, B, ldb, C, ldc, ep, k_per_split);
}

// ---------------------------------------------------------------------------- grouped weight gradients
// The weight gradients of every layer of one MLP in ONE launch: dW_i += dZ_i^T X_i (+ the bias-gradient column sums),
// item i owning a contiguous, 8-aligned run of block ids.  Sharing the launch lets each layer fill the chip with 8x
// fewer K slices than a launch of its own (the items' tiles together make the blocks), and the split-K atomics --
// one 64 KB tile of float adds per block, at the memory side's ~1.3 TB/s -- shrink with the slice count.
struct TnItem {
  int64_t M, N, K;   // C[M, N] += A^T B, A [K, M] (lda), B [K, N] (ldb): M = out units, N = in units, K = rows
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  float* colsum;
  int64_t kps;       // rows per slice
  int mt, nt, zs;    // tiles and K slices
  int blocks;        // 8 * ceil(mt nt zs / 8)... (mt nt * zs rounded so every item starts on an XCD-group boundary)
};
constexpr int kMaxTnItems = 5;
struct TnGroup {
  TnItem it[kMaxTnItems];
  int n;
};

template <int PREC, bool VEC>
__global__ __launch_bounds__(256) void gemm_tn_grouped_kernel(TnGroup g) {
  int id = blockIdx.x, i = 0;
  while (i + 1 < g.n && id >= g.it[i].blocks) {
    id -= g.it[i].blocks;
    ++i;
  }
  const TnItem& t = g.it[i];
  int mt, nt, slice;
  if (!split_map(id, t.mt, t.nt, t.zs, mt, nt, slice)) return;
  Epi ep{nullptr, nullptr, 0, nullptr, 0, ACT_NONE, ACT_NONE, 1.f, 20.f, 1, -1, t.zs > 1 ? t.zs : 2, t.colsum};
  gemm_block<PREC, true, true, VEC>(mt, nt, slice, t.M, t.N, t.K, t.A, t.lda, t.B, t.ldb, t.C, t.ldc, ep, t.kps);
}

// ---------------------------------------------------------------------------- wide weight gradients
// dW[Mo, Ni] += dZ^T X over the rows of a K slice with a 256 x 256 output tile per block (8 waves of 64 x 128, 2 x 4
// MFMA tiles each): every operand row is read ONCE per slice -- the 128 x 128 tiles of gemm_tn_grouped_kernel read
// each 256-wide operand twice (the tiles of one slice share rows; profiles/pmc_traffic_fast.json: 1.4x the
// algorithmic bytes for the SDF MLP's 1.27 GB).  Both operands are T sources ([rows][units], 16-B rows); a stage of
// 32 rows is loaded into registers one stage ahead, split into bf16 hi (+ lo) and stored into one of two LDS image
// sets ([k][256 + 32] per image, ds_read_b64_tr_b16 fragments), so one barrier per stage.  LDS: 144 KB (split-bf16x3)
// -> one block of 8 waves per CU.  Output tiles past Mo / Ni are skipped per wave-tile (the SDF input layer's 71
// columns run 3 of 8 column tiles).  The slices' partial tiles are added with float atomics (one per element per
// block), the bias gradients (column sums of dZ) reduced in LDS first.
constexpr int kWT = 256;            // output tile edge
constexpr int kWLD = kWT + 32;      // image row pitch (elements): 576-B rows, conflict-free transposing reads

struct WideItem {
  int64_t M, N, K;   // C[M, N] += A^T B: A [K rows, M] (lda), B [K rows, N] (ldb)
  const float* A;    // P_F16: fp16 rows (lda in halves), row k scaled by 1 / ainv[k]
  int64_t lda;
  const float* ainv;       // P_F16: per-row inverse scales of A (powers of two)
  const unsigned* emax;    // P_F16: max over rows of log2(ainv) + 14 + 1000 (0: A is all zero)
  const float* B;    // fp32 rows, or (b16) fp16 rows (ldb in halves, 8-B aligned)
  int64_t ldb;
  int b16;
  float* C;
  int64_t ldc;
  float* colsum;
  int64_t kps;       // rows per slice
  int mt, nt, zs;    // 256-tiles along M and N, K slices
  int blocks;        // mt * nt * zs
};
struct WideGroup {
  WideItem it[kMaxTnItems];
  int n;
  float* ws;         // non-null: each block stores its partial tile here ([block][256][256]) for the reduce kernel,
                     // instead of adding it to C with float atomics
};

// the fp16 items' stages: 32 rows (2 images of 32 rows in the LDS split bf16x3's 4 images of 16 take; one barrier per
// 32 rows; 0.141 -> 0.138 ms per launch, 3 x 2 A/B) with two register sets (16-row stages with 2, 3 or 4 sets measured
// equal: the loads are not latency-bound)
#ifndef MMS_WIDE_WK16
#define MMS_WIDE_WK16 32
#endif
#ifndef MMS_WIDE_DEPTH16
#define MMS_WIDE_DEPTH16 2   // register sets of the fp16 items' pipeline (split-bf16x3 items: 2)
#endif
template <typename F, int... I>
__device__ __forceinline__ void wide_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void wide_for(F&& f) {   // f(integral_constant<i>) for i < N, unrolled
  wide_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ float4 ld_f4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ uint2 ld_u2(const unsigned short* p) { return *reinterpret_cast<const uint2*>(p); }

// One block's tile and K slice of item t.  PREC: the item's operand mode (P_BF16 / P_BF16X3: fp32 A rows; P_F16: fp16
// A rows, see WideItem); B16: fp16 B rows (their values widened exactly, then split or scaled like fp32 rows).  lds:
// the kernel's image buffers, scs: [8][256] floats.
template <int PREC, int WK, bool B16>
__device__ __forceinline__ void wide_block(const WideItem& t, int id, float* part, __bf16* lds, float (*scs)[kWT]) {
  constexpr int kWK = WK;             // rows per stage (16 or 32)
  constexpr int NLD = WK / 8;         // float4 loads per thread per operand and stage
  constexpr int NIMG = PREC == P_BF16X3 ? 2 : 1;
  constexpr int IMG = kWK * kWLD;                        // elements per image
  constexpr int BUF = 2 * NIMG * IMG;                     // elements per image set (A hi, (A lo), B hi, (B lo))
  // P_F16 (mms_gemm_tn_wide16): A = fp16 dZ rows in their row scale (1 / ainv[k]), rescaled per row by
  // ainv[k] 2^(14 - emax) <= 1 to the launch's common scale 2^(14 - emax) and rounded to fp16 again, B = X rounded to
  // fp16; the common factor is undone on the accumulators before they are added to C; one fp16 MFMA per product, one
  // image per operand
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  const int tiles = t.mt * t.nt;
  const int tile = id % tiles, slice = id / tiles;
  const int64_t m0 = (int64_t)(tile % t.mt) * kWT, n0 = (int64_t)(tile / t.mt) * kWT;
  const int64_t kbeg = (int64_t)slice * t.kps;
  const int64_t kend = kbeg + t.kps < t.K ? kbeg + t.kps : t.K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;
  // staging: thread -> float4 column (lane) of rows (w + 8 i), i < WK / 8, for A and B
  const int64_t ca = m0 + 4 * lane, cb = n0 + 4 * lane;
  const int64_t ca_c = ca + 3 < t.M ? ca : ((t.M - 1) & ~(int64_t)3);   // clamped (always valid) 16-B column
  const int64_t cb_c = cb + 3 < t.N ? cb : ((t.N - 1) & ~(int64_t)3);
  const int va = (int)(t.M - ca < 0 ? 0 : (t.M - ca > 4 ? 4 : t.M - ca));   // valid elements of the float4
  const int vb = (int)(t.N - cb < 0 ? 0 : (t.N - cb > 4 ? 4 : t.N - cb));
  const bool do_cs = t.colsum != nullptr && n0 == 0;
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
  float bsc = 1.f, osc = 1.f;
  if constexpr (PREC == P_F16) {
    const unsigned eb = *t.emax;
    const int emx = eb > 0u ? (int)eb - 1000 : 14;
    bsc = __builtin_amdgcn_ldexpf(1.f, 14 - emx);
    osc = __builtin_amdgcn_ldexpf(1.f, emx - 14);
  }
  // one B load: float4, or (B16) the 4 fp16 values' bits in .x / .y
  auto ldB = [&](int64_t rc) {
    if constexpr (B16) {
      const uint2 hv = ld_u2(reinterpret_cast<const unsigned short*>(t.B) + rc * t.ldb + cb_c);
      return make_float4(__uint_as_float(hv.x), __uint_as_float(hv.y), 0.f, 0.f);
    } else {
      return ld_f4(t.B + rc * t.ldb + cb_c);
    }
  };
  // B16 rows widened to float4 (exact)
  auto widenB = [](float4 v) {
    if constexpr (B16) {
      const f16x2 p0 = __builtin_bit_cast(f16x2, __float_as_uint(v.x));
      const f16x2 p1 = __builtin_bit_cast(f16x2, __float_as_uint(v.y));
      return make_float4((float)p0[0], (float)p0[1], (float)p1[0], (float)p1[1]);
    } else {
      return v;
    }
  };
  // one A load: float4, or (P_F16) the 4 fp16 values' bits in .x / .y and the row's inverse scale in .z
  auto ldA = [&](int64_t rc) {
    if constexpr (PREC == P_F16) {
      const uint2 hv = ld_u2(reinterpret_cast<const unsigned short*>(t.A) + rc * t.lda + ca_c);
      return make_float4(__uint_as_float(hv.x), __uint_as_float(hv.y), t.ainv[rc], 0.f);
    } else {
      return ld_f4(t.A + rc * t.lda + ca_c);
    }
  };
#if MMS_WIDE_PIPE
  // two register sets: stage s + 2's loads are issued before stage s's MFMAs, and stage s + 1's image stores sit in
  // the same basic block as those MFMAs (no branch between them), so the scheduler can interleave the conversions and
  // LDS writes with the MFMAs and one whole stage of MFMA time covers each load's latency
  // DEPTH register sets: stage s + DEPTH's loads are issued at stage s (the fp16 items' short stages need more loads
  // in flight than split-bf16x3's: their global loads were half the launch time, MMS_WIDE_ABLATE=4 A/B)
  constexpr int DEPTH = PREC == P_F16 ? MMS_WIDE_DEPTH16 : 2;
  float4 rset[DEPTH][2][NLD];
  int nset[DEPTH] = {};
  auto load2 = [&](int s, auto setc) {
    constexpr int Q = decltype(setc)::value;
    const int64_t r0 = kbeg + (int64_t)s * kWK;
    nset[Q] = (int)(kend - r0 < kWK ? kend - r0 : kWK);   // <= 0 past the slice: the store writes zeros
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int64_t r = r0 + w + 8 * i;
      const int64_t rc = r < kend ? r : kend - 1;
      if constexpr ((MMS_WIDE_ABLATE & 4) != 0) {
        rset[Q][0][i] = make_float4((float)rc, 1.f, 2.f, 3.f);
        rset[Q][1][i] = make_float4(1.f, (float)rc, 3.f, 4.f);
      } else {
        rset[Q][0][i] = ldA(rc);
        rset[Q][1][i] = ldB(rc);
      }
    }
  };
#endif
  float4 ra[NLD], rb[NLD];
  int nrows = 0;
  auto load = [&](int s) {
    const int64_t r0 = kbeg + (int64_t)s * kWK;
    nrows = (int)(kend - r0 < kWK ? kend - r0 : kWK);
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int64_t r = r0 + w + 8 * i;
      const int64_t rc = r < kend ? r : kend - 1;
      if constexpr ((MMS_WIDE_ABLATE & 4) != 0) {
        ra[i] = make_float4((float)rc, 1.f, 2.f, 3.f);
        rb[i] = make_float4(1.f, (float)rc, 3.f, 4.f);
      } else {
        ra[i] = ldA(rc);
        rb[i] = ldB(rc);
      }
    }
  };
  auto mask4 = [](float4 v, int valid, bool row_ok) {
    if (!row_ok) return make_float4(0.f, 0.f, 0.f, 0.f);
    v.x = valid > 0 ? v.x : 0.f;
    v.y = valid > 1 ? v.y : 0.f;
    v.z = valid > 2 ? v.z : 0.f;
    v.w = valid > 3 ? v.w : 0.f;
    return v;
  };
  auto store_from = [&](int buf, const float4* xa, const float4* xb, int nr) {
    if constexpr ((MMS_WIDE_ABLATE & 8) != 0) return;
    __bf16* base = lds + buf * BUF;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const bool ok = w + 8 * i < nr;
      if constexpr (PREC == P_F16) {
        // A: the fp16 bits as loaded (invalid columns / rows zeroed); B: scaled by the row's factor, rounded to fp16
        const uint32_t k0 = !ok ? 0u : (va > 1 ? 0xffffffffu : (va > 0 ? 0xffffu : 0u));
        const uint32_t k1 = !ok ? 0u : (va > 3 ? 0xffffffffu : (va > 2 ? 0xffffu : 0u));
        const uint32_t u0 = __float_as_uint(xa[i].x) & k0, u1 = __float_as_uint(xa[i].y) & k1;
        const float rin = xa[i].z;
        const f16x2 p0 = __builtin_bit_cast(f16x2, u0), p1 = __builtin_bit_cast(f16x2, u1);
        if (do_cs) {
          cs.x += (float)p0[0] * rin; cs.y += (float)p0[1] * rin;
          cs.z += (float)p1[0] * rin; cs.w += (float)p1[1] * rin;
        }
        // A: the row-scaled values brought to the launch's common scale (each row by 2^(e_r - e_max) <= 1: the
        // largest |dZ| at 2^14, rows down to 2^-28 of it keep fp16's full precision -- the reference's loss-scaled
        // fp16 dZ); B: X rounded to fp16 as it is (the autocast's fp16 activations)
        const float f = rin * bsc;
        const f16x4 ah = {(_Float16)((float)p0[0] * f), (_Float16)((float)p0[1] * f), (_Float16)((float)p1[0] * f),
                          (_Float16)((float)p1[1] * f)};
        // (an all-zero dZ row -- rinv 0, e.g. a fixed-capacity padding row -- contributes nothing, whatever its X row
        // holds; X beyond fp16's range saturates instead of turning 0 x inf into NaN)
        const float4 b = mask4(widenB(xb[i]), vb, ok && rin != 0.f);
        auto sat = [](float v) { return fminf(fmaxf(v, -65504.f), 65504.f); };
        const f16x4 bh = {(_Float16)sat(b.x), (_Float16)sat(b.y), (_Float16)sat(b.z), (_Float16)sat(b.w)};
        const int off = (w + 8 * i) * kWLD + 4 * lane;
        *reinterpret_cast<f16x4*>(base + off) = ah;
        *reinterpret_cast<f16x4*>(base + NIMG * IMG + off) = bh;
        continue;
      }
      const float4 a = mask4(xa[i], va, ok), b = mask4(widenB(xb[i]), vb, ok);
      if (do_cs) { cs.x += a.x; cs.y += a.y; cs.z += a.z; cs.w += a.w; }
      const int off = (w + 8 * i) * kWLD + 4 * lane;
      const bf16x4 ah = cvt4(a), bh = cvt4(b);
      *reinterpret_cast<bf16x4*>(base + off) = ah;
      *reinterpret_cast<bf16x4*>(base + NIMG * IMG + off) = bh;
      if constexpr (PREC == P_BF16X3) {
        *reinterpret_cast<bf16x4*>(base + IMG + off) = cvt4(resid4(a, ah));
        *reinterpret_cast<bf16x4*>(base + 3 * IMG + off) = cvt4(resid4(b, bh));
      }
    }
  };
  auto store = [&](int buf) { store_from(buf, ra, rb, nrows); };
  // wave-tile activity (wave-uniform): rows 64 wm + 32 i, columns 128 wn + 32 j of the block tile
  bool act_i[2], act_j[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) act_i[i] = m0 + 64 * wm + 32 * i < t.M;
#pragma unroll
  for (int j = 0; j < 4; ++j) act_j[j] = n0 + 128 * wn + 32 * j < t.N;
  floatx16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx16{};
  auto compute = [&](int buf, auto allc) {
    constexpr bool ALL = decltype(allc)::value;   // every wave-tile active: no per-tile branches around the MFMAs
    const __bf16* Ai = lds + buf * BUF;
    const __bf16* Bi = lds + buf * BUF + NIMG * IMG;
#pragma unroll
    for (int ks = 0; ks < kWK; ks += 16) {
      bf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = frag_bf16<true, 8, kWLD>(Ai, 64 * wm + 32 * i, ks);
        if constexpr (PREC == P_BF16X3) al[i] = frag_bf16<true, 8, kWLD>(Ai + IMG, 64 * wm + 32 * i, ks);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bh[j] = frag_bf16<true, 8, kWLD>(Bi, 128 * wn + 32 * j, ks);
        if constexpr (PREC == P_BF16X3) bl[j] = frag_bf16<true, 8, kWLD>(Bi + IMG, 128 * wn + 32 * j, ks);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (!ALL && !act_i[i]) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!ALL && !act_j[j]) continue;
          if constexpr ((MMS_WIDE_ABLATE & 2) != 0) {
            acc[i][j][0] += (float)ah[i][0] + (float)bh[j][0];   // keeps the fragment reads live
            continue;
          }
          if constexpr (PREC == P_F16) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah[i]),
                                                               __builtin_bit_cast(f16x8, bh[j]), acc[i][j], 0, 0, 0);
            continue;
          }
          if constexpr (PREC == P_BF16X3) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };
  const int S = (int)((kend - kbeg + kWK - 1) / kWK);
#if MMS_WIDE_PIPE
  if (S > 0) {
    load2(0, std::integral_constant<int, 0>{});
    store_from(0, rset[0][0], rset[0][1], nset[0]);
    wide_for<DEPTH - 1>([&](auto dc) { load2(decltype(dc)::value + 1, std::integral_constant<int, decltype(dc)::value + 1>{}); });
  }
  __syncthreads();
  // one branch per wave for the whole loop: a wave whose tiles are all active runs the branch-free body (its MFMAs,
  // conversions and LDS stores one basic block the scheduler interleaves)
  auto loop = [&](auto allc) {
    for (int s = 0; s < S; s += DEPTH) {
      // stage s + j: set j held it (already in LDS buffer (s + j) & 1) and takes stage s + j + DEPTH; set (j + 1) % DEPTH
      // holds stage s + j + 1, stored into buffer (s + j + 1) & 1 (s, S block-uniform: every thread skips alike)
      wide_for<DEPTH>([&](auto jc) {
        constexpr int j = decltype(jc)::value, jn = (j + 1) % DEPTH;
        if (s + j >= S) return;
        load2(s + j + DEPTH, std::integral_constant<int, j>{});
        compute((s + j) & 1, allc);
        store_from((s + j + 1) & 1, rset[jn][0], rset[jn][1], nset[jn]);
        __syncthreads();
      });
    }
  };
  const bool all_act = act_i[0] && act_i[1] && act_j[0] && act_j[1] && act_j[2] && act_j[3];
  if (all_act) loop(std::true_type{});
  else loop(std::false_type{});
#else
  if (S > 0) {
    load(0);
    store(0);
    if (S > 1) load(1);
  }
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    compute(s & 1, std::false_type{});
    if (s + 1 < S) {
      store((s + 1) & 1);
      if (s + 2 < S) load(s + 2);
    }
    __syncthreads();
  }
#endif
  if (do_cs) {
    *reinterpret_cast<float4*>(&scs[w][4 * lane]) = cs;
    __syncthreads();
    if (tid < kWT && m0 + tid < t.M) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) v += scs[j][tid];
      atomicAdd(t.colsum + m0 + tid, v);
    }
  }
  // C/D map: column = lane & 31, row = (e & 3) + 8 (e >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!act_i[i]) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!act_j[j]) continue;
      const int tc = 128 * wn + 32 * j + (lane & 31);
      const int tr0 = 64 * wm + 32 * i + 4 * (lane >> 5);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int tr = tr0 + (e & 3) + 8 * (e >> 2);
        if ((MMS_WIDE_ABLATE & 1) != 0 && acc[i][j][e] != 1234.5f) continue;
        const float v = PREC == P_F16 ? acc[i][j][e] * osc : acc[i][j][e];
        if (part != nullptr) {
          part[tr * kWT + tc] = v;    // 128-B row segments per instruction: plain, coalesced stores
        } else if (m0 + tr < t.M && n0 + tc < t.N) {
          atomicAdd(t.C + (m0 + tr) * t.ldc + n0 + tc, v);
        }
      }
    }
  }
}

// P_F16 launches (mms_gemm_tn_wide16) mix modes per item: fp16 A rows (ainv set) run P_F16, fp32 A rows split bf16x3;
// B rows fp16 or fp32 per item.  The image buffers are sized for split bf16x3 (4 images of WK rows = 2 of 2 WK).
template <int PREC, int WK>
__global__ __launch_bounds__(512) void gemm_tn_wide_kernel(WideGroup g) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][4 * WK * kWLD];   // [buffer][A hi, (A lo), B hi, (B lo)]
  __shared__ float scs[8][kWT];                                             // bias-gradient partials per wave
  int id = blockIdx.x, ii = 0;
  while (ii + 1 < g.n && id >= g.it[ii].blocks) {
    id -= g.it[ii].blocks;
    ++ii;
  }
  // (a copy: the item's fields in registers once, not re-read from the kernel arguments inside the stage loop)
  const WideItem t = g.it[ii];
  float* part = g.ws != nullptr ? g.ws + (int64_t)blockIdx.x * (kWT * kWT) : nullptr;
  if constexpr (PREC == P_F16) {
    if (t.ainv != nullptr) {
      // (MMS_WIDE_WK16 rows per stage for the fp16 items: the same LDS holds 2 images of 2 WK rows)
      if (t.b16) wide_block<P_F16, MMS_WIDE_WK16, true>(t, id, part, &lds[0][0], scs);
      else wide_block<P_F16, MMS_WIDE_WK16, false>(t, id, part, &lds[0][0], scs);
    } else {
      if (t.b16) wide_block<P_BF16X3, WK, true>(t, id, part, &lds[0][0], scs);
      else wide_block<P_BF16X3, WK, false>(t, id, part, &lds[0][0], scs);
    }
  } else {
    wide_block<PREC, WK, false>(t, id, part, &lds[0][0], scs);
  }
}

// The slices' partial tiles summed per output element in slice order and added to C: one thread per element of a tile,
// blockIdx.y = the tile (over every item of the group), reads coalesced across the block; one float atomic per output
// element and item (instead of one per element and slice).
// Only the wave-tiles the wide kernel computed are read (the others it did not write).
__global__ __launch_bounds__(256) void gemm_tn_wide_reduce_kernel(WideGroup g) {
  int tile = blockIdx.y, ii = 0, base = 0;
  while (ii + 1 < g.n && tile >= g.it[ii].mt * g.it[ii].nt) {
    tile -= g.it[ii].mt * g.it[ii].nt;
    base += g.it[ii].blocks;
    ++ii;
  }
  const WideItem& t = g.it[ii];
  const int tiles = t.mt * t.nt;
  const int64_t m0 = (int64_t)(tile % t.mt) * kWT, n0 = (int64_t)(tile / t.mt) * kWT;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int tr = e / kWT, tc = e % kWT;
  // the kernel above skips whole 32 x 32 wave-tiles past M / N: only elements inside the written tiles are read
  const bool in_tile = m0 + (tr & ~31) < t.M && n0 + (tc & ~31) < t.N;
  if (!in_tile || m0 + tr >= t.M || n0 + tc >= t.N) return;
  const float* p = g.ws + (int64_t)(base + tile) * (kWT * kWT) + e;
  float v = 0.f;
  for (int sl = 0; sl < t.zs; ++sl) v += p[(int64_t)sl * tiles * (kWT * kWT)];
  // an atomic add: items of one launch may share an output (the SDF taps item adds into the last layer's dW row 0)
  atomicAdd(t.C + (m0 + tr) * t.ldc + n0 + tc, v);
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
                        int accumulate, int splits, int ones_col, float* colsum, void* stream) {
  const char* fn = "mms_gemm";
  MMS_REQUIRE(colsum == nullptr || trans_a, fn, "the fused column sum needs a transposed (T-source) A");
  MMS_REQUIRE(prec >= 0 && prec <= 2, fn, "prec must be 0 (f32), 1 (bf16) or 2 (bf16x3)");
  MMS_REQUIRE(M >= 0 && N >= 0 && K >= 0, fn, "negative size");
  MMS_REQUIRE(act >= 0 && act <= 3 && dact >= 0 && dact <= 4, fn, "bad activation id");
  if (M == 0 || N == 0) return 0;
  MMS_REQUIRE(A && B && C, fn, "null operand");
  if (splits < 1) splits = 1;
  MMS_REQUIRE(splits == 1 || (accumulate && Z == nullptr && aux == nullptr && act == ACT_NONE && bias == nullptr &&
                              ones_col < 0),
              fn, "split-K requires a plain accumulating epilogue");
  // vector path: 16-B aligned bases and leading dims multiples of 4 (ragged contiguous dims are masked per float4)
  const bool vec = aligned16(A) && aligned16(B) && lda % 4 == 0 && ldb % 4 == 0;
  const int BK = prec == P_BF16 ? Geo<P_BF16>::BK : Geo<P_F32>::BK;
  int64_t kps = (K + splits - 1) / splits;
  kps = ((kps + BK - 1) / BK) * BK;
  if (kps < BK) kps = BK;
  const int64_t zs = K == 0 ? 1 : (K + kps - 1) / kps;
  const int64_t mt = (M + BM - 1) / BM;
  const int64_t mtp = zs > 1 ? mt : ((mt + 7) / 8) * 8;
  const int64_t nt = (N + BN - 1) / BN;
  MMS_REQUIRE(mtp * nt * (zs + 7) <= INT32_MAX, fn, "grid too large");
  Epi ep{bias, Z, ldz, aux, ldaux, act, dact, beta, thr, accumulate, ones_col, (int)zs, colsum};
  const int64_t zs_grid = (zs > 1 && MMS_GEMM_XCDSPLIT) ? (zs + 7) / 8 * 8 : zs;
  dim3 grid((unsigned)(mtp * nt * zs_grid), 1, 1);
  hipStream_t s = mms::as_stream(stream);
  const int64_t kp = K == 0 ? 0 : kps;
  switch (prec) {
    case P_F32: dispatch_ta_tb<P_F32>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kp, (int)mtp, (int)nt); break;
    case P_BF16: dispatch_ta_tb<P_BF16>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kp, (int)mtp, (int)nt); break;
    default: dispatch_ta_tb<P_BF16X3>(trans_a, trans_b, vec, grid, s, M, N, K, A, lda, B, ldb, C, ldc, ep, kp, (int)mtp, (int)nt); break;
  }
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_gemm_tn_grouped(int prec, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                                   const float* const* A, const int64_t* lda, const float* const* B,
                                   const int64_t* ldb, float* const* C, const int64_t* ldc, float* const* colsum,
                                   int target_blocks, void* stream) {
  const char* fn = "mms_gemm_tn_grouped";
  MMS_REQUIRE(prec >= 0 && prec <= 2, fn, "prec must be 0 (f32), 1 (bf16) or 2 (bf16x3)");
  MMS_REQUIRE(n >= 1 && n <= kMaxTnItems, fn, "1 to 5 weight-gradient items per launch");
  MMS_REQUIRE(M && N && K && A && lda && B && ldb && C && ldc, fn, "null argument array");
  if (target_blocks < 1) target_blocks = 256;
  const int BK = prec == P_BF16 ? Geo<P_BF16>::BK : Geo<P_F32>::BK;
  TnGroup g{};
  double work = 0.0;
  for (int i = 0; i < n; ++i) {
    MMS_REQUIRE(M[i] >= 0 && N[i] >= 0 && K[i] >= 0, fn, "negative size");
    MMS_REQUIRE(M[i] == 0 || N[i] == 0 || K[i] == 0 || (A[i] && B[i] && C[i]), fn, "null operand");
    work += (double)((M[i] + BM - 1) / BM) * ((N[i] + BN - 1) / BN) * (double)K[i];
  }
  bool vec = true;
  int64_t total = 0;
  int m = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] == 0 || N[i] == 0 || K[i] == 0) continue;   // nothing to add
    TnItem& t = g.it[m++];
    t.M = M[i]; t.N = N[i]; t.K = K[i];
    t.A = A[i]; t.lda = lda[i]; t.B = B[i]; t.ldb = ldb[i]; t.C = C[i]; t.ldc = ldc[i];
    t.colsum = colsum ? colsum[i] : nullptr;
    t.mt = (int)((t.M + BM - 1) / BM);
    t.nt = (int)((t.N + BN - 1) / BN);
    // K slices in proportion to the item's share of the work (every block then streams the same number of rows),
    // rounded to a multiple of 8 so the slices of each tile spread evenly over the 8 XCDs (split_map), at least
    // 512 rows each
    const double share = (double)t.mt * t.nt * (double)t.K / work;
    int64_t zs = (int64_t)(share * target_blocks / (t.mt * t.nt) + 0.5);
    zs = zs >= 8 ? (zs + 4) / 8 * 8 : zs;
    if (zs > t.K / 512) zs = t.K / 512;
    if (zs < 1) zs = 1;
    int64_t kps = (t.K + zs - 1) / zs;
    kps = (kps + BK - 1) / BK * BK;
    t.kps = kps;
    t.zs = (int)((t.K + kps - 1) / kps);
    t.blocks = t.mt * t.nt * ((t.zs + 7) / 8 * 8);
    total += t.blocks;
    vec = vec && ((uintptr_t)t.A & 15) == 0 && ((uintptr_t)t.B & 15) == 0 && t.lda % 4 == 0 && t.ldb % 4 == 0;
  }
  g.n = m;
  if (m == 0) return 0;
  MMS_REQUIRE(total <= INT32_MAX, fn, "grid too large");
  hipStream_t s = mms::as_stream(stream);
  dim3 grid((unsigned)total), blk(256);
  switch (prec) {
    case P_F32:
      if (vec) hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_F32, true>), grid, blk, 0, s, g);
      else hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_F32, false>), grid, blk, 0, s, g);
      break;
    case P_BF16:
      if (vec) hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_BF16, true>), grid, blk, 0, s, g);
      else hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_BF16, false>), grid, blk, 0, s, g);
      break;
    default:
      if (vec) hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_BF16X3, true>), grid, blk, 0, s, g);
      else hipLaunchKernelGGL((gemm_tn_grouped_kernel<P_BF16X3, false>), grid, blk, 0, s, g);
      break;
  }
  return mms::check_launch(fn);
}

namespace {

// a split-bf16x3 item's per-row cost beside fp16 items, relative to its bytes' share (with 32-row fp16 stages, same-box
// step A/B 1.0 / 1.2 / 1.5 / 2.0: 3.155 / 3.146-3.150 / 3.167 / 3.176 ms; with 16-row stages 1.5 was best for the launch
// alone; 320 blocks instead of 256: 3.213 ms)
#ifndef MMS_WIDE_X3COST
#define MMS_WIDE_X3COST 1.2
#endif
// K slices of each item (g.it[0 .. g.n) with M, N, K set) in proportion to its share of the work -- tiles x rows x the
// operand bytes per row element (the kernel streams its operands from HBM) -- so every block takes about the same time
// (>= 1024 rows per slice); returns the total block count
int64_t plan_wide(WideGroup& g, int target_blocks) {
  if (target_blocks < 1) target_blocks = 256;
  // (a split-bf16x3 item's rows cost more than their bytes' share beside fp16 items: its three MFMAs and four images
  // per product; 16-row fp16 stages, A/B 1.0 / 1.5 / 2.2: the launch 154 / 141 / 143 us)
  auto cost = [](const WideItem& t) {
    return (double)((t.M + kWT - 1) / kWT) * ((t.N + kWT - 1) / kWT) * (double)t.K *
           ((t.ainv ? 2.0 : 4.0) + (t.b16 ? 2.0 : 4.0)) * (t.ainv ? 1.0 : MMS_WIDE_X3COST);
  };
  double work = 0.0;
  for (int i = 0; i < g.n; ++i) work += cost(g.it[i]);
  int64_t total = 0;
  for (int i = 0; i < g.n; ++i) {
    WideItem& t = g.it[i];
    t.mt = (int)((t.M + kWT - 1) / kWT);
    t.nt = (int)((t.N + kWT - 1) / kWT);
    const double share = cost(t) / work;
    int64_t zs = (int64_t)(share * target_blocks / (t.mt * t.nt) + 0.5);
    if (zs > t.K / 1024) zs = t.K / 1024;
    if (zs < 1) zs = 1;
    int64_t kps = (t.K + zs - 1) / zs;
    kps = (kps + 31) / 32 * 32;
    t.kps = kps;
    t.zs = (int)((t.K + kps - 1) / kps);
    t.blocks = t.mt * t.nt * t.zs;
    total += t.blocks;
  }
  return total;
}

template <int PREC>
void launch_wide(WideGroup& g, int64_t total, int stage_rows, float* workspace, int64_t workspace_floats,
                 hipStream_t s) {
  // partial tiles through the workspace when it holds them all (else float atomics into C)
  g.ws = (workspace != nullptr && workspace_floats >= total * (int64_t)(kWT * kWT)) ? workspace : nullptr;
  int all_tiles = 0;
  for (int i = 0; i < g.n; ++i) all_tiles += g.it[i].mt * g.it[i].nt;
  const dim3 grid((unsigned)total), blk(512);
  if (stage_rows == 32) hipLaunchKernelGGL((gemm_tn_wide_kernel<PREC, 32>), grid, blk, 0, s, g);
  else hipLaunchKernelGGL((gemm_tn_wide_kernel<PREC, 16>), grid, blk, 0, s, g);
  if (g.ws != nullptr)
    hipLaunchKernelGGL(gemm_tn_wide_reduce_kernel, dim3(kWT * kWT / 256, all_tiles), dim3(256), 0, s, g);
}

}  // namespace

MMS_EXPORT int mms_gemm_tn_wide(int prec, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                                const float* const* A, const int64_t* lda, const float* const* B, const int64_t* ldb,
                                float* const* C, const int64_t* ldc, float* const* colsum, int target_blocks,
                                int stage_rows, float* workspace, int64_t workspace_floats, void* stream) {
  const char* fn = "mms_gemm_tn_wide";
  MMS_REQUIRE(stage_rows == 16 || stage_rows == 32, fn, "stage_rows must be 16 or 32");
  MMS_REQUIRE(prec == 1 || prec == 2, fn, "prec must be 1 (bf16) or 2 (bf16x3)");
  MMS_REQUIRE(n >= 1 && n <= kMaxTnItems, fn, "1 to 5 weight-gradient items per launch");
  MMS_REQUIRE(M && N && K && A && lda && B && ldb && C && ldc, fn, "null argument array");
  WideGroup g{};
  int m = 0;
  for (int i = 0; i < n; ++i) {
    MMS_REQUIRE(M[i] >= 0 && N[i] >= 0 && K[i] >= 0, fn, "negative size");
    if (M[i] == 0 || N[i] == 0 || K[i] == 0) continue;   // nothing to add
    MMS_REQUIRE(A[i] && B[i] && C[i], fn, "null operand");
    MMS_REQUIRE(aligned16(A[i]) && aligned16(B[i]) && lda[i] % 4 == 0 && ldb[i] % 4 == 0, fn,
                "operand rows must be 16-B aligned");
    MMS_REQUIRE(lda[i] >= M[i] && ldb[i] >= N[i], fn, "leading dimension smaller than the row");
    WideItem& t = g.it[m++];
    t.M = M[i]; t.N = N[i]; t.K = K[i];
    t.A = A[i]; t.lda = lda[i]; t.B = B[i]; t.ldb = ldb[i]; t.C = C[i]; t.ldc = ldc[i];
    t.colsum = colsum ? colsum[i] : nullptr;
  }
  g.n = m;
  if (m == 0) return 0;
  const int64_t total = plan_wide(g, target_blocks);
  MMS_REQUIRE(total <= INT32_MAX, fn, "grid too large");
  hipStream_t s = mms::as_stream(stream);
  if (prec == P_BF16) launch_wide<P_BF16>(g, total, stage_rows, workspace, workspace_floats, s);
  else launch_wide<P_BF16X3>(g, total, stage_rows, workspace, workspace_floats, s);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_gemm_tn_wide16(int n, const int64_t* M, const int64_t* N, const int64_t* K, const void* const* A,
                                  const int64_t* lda, const float* const* ainv, const unsigned* const* emax,
                                  const void* const* B, const int64_t* ldb, const int* b16, float* const* C,
                                  const int64_t* ldc, float* const* colsum, int target_blocks, void* stream) {
  const char* fn = "mms_gemm_tn_wide16";
  MMS_REQUIRE(n >= 1 && n <= kMaxTnItems, fn, "1 to 5 weight-gradient items per launch");
  MMS_REQUIRE(M && N && K && A && lda && B && ldb && C && ldc, fn, "null argument array");
  WideGroup g{};
  int m = 0;
  for (int i = 0; i < n; ++i) {
    MMS_REQUIRE(M[i] >= 0 && N[i] >= 0 && K[i] >= 0, fn, "negative size");
    if (M[i] == 0 || N[i] == 0 || K[i] == 0) continue;
    const bool a16 = ainv && ainv[i], bh = b16 && b16[i];
    MMS_REQUIRE(A[i] && B[i] && C[i] && (!a16 || (emax && emax[i])), fn, "null operand");
    MMS_REQUIRE(((uintptr_t)A[i] & (a16 ? 7 : 15)) == 0 && lda[i] % 4 == 0 && ((uintptr_t)B[i] & (bh ? 7 : 15)) == 0 &&
                    ldb[i] % 4 == 0, fn, "fp16 rows must be 8-B aligned, fp32 rows 16-B aligned");
    MMS_REQUIRE(lda[i] >= M[i] && ldb[i] >= N[i], fn, "leading dimension smaller than the row");
    WideItem& t = g.it[m++];
    t.M = M[i]; t.N = N[i]; t.K = K[i];
    t.A = reinterpret_cast<const float*>(A[i]); t.lda = lda[i];
    t.ainv = a16 ? ainv[i] : nullptr; t.emax = a16 ? emax[i] : nullptr;
    t.B = reinterpret_cast<const float*>(B[i]); t.ldb = ldb[i]; t.b16 = bh ? 1 : 0;
    t.C = C[i]; t.ldc = ldc[i];
    t.colsum = colsum ? colsum[i] : nullptr;
  }
  g.n = m;
  if (m == 0) return 0;
  const int64_t total = plan_wide(g, target_blocks);
  MMS_REQUIRE(total <= INT32_MAX, fn, "grid too large");
  launch_wide<P_F16>(g, total, 16, nullptr, 0, mms::as_stream(stream));
  return mms::check_launch(fn);
}
