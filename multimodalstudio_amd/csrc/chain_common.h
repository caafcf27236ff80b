// Used by the fused MLP chain kernels (mlp_chain.hip: 32x32x16 MFMA, one wave per SIMD): argument structs, activations and their derivatives, split-bf16 conversion, the LDS-DMA
// weight / input staging and the exact-count wait + barrier.  Reference layers: weight-normed nn.Linear + activation
// (/root/reference/src/field_components/mlp.py:152-209).
#pragma once

#include <utility>

#include <hip/hip_runtime.h>

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// streamed activations bypass the caches' retention (non-temporal), so the packed weights the waves re-read
// from L2 at every k-step stay resident
__device__ __forceinline__ f32x4 ld_nt4(const float* p) { return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p)); }
__device__ __forceinline__ void st_nt4(float* p, f32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p)); }

struct ChainLayer {
  const __bf16* a_hi;  // packed A operand [32 nt][16 ks] (mms_mlp_pack)
  const __bf16* a_lo;  // split-bf16x3 residual image, or null
  const float* bias;   // forward: [N], or null
  const float* aux;    // backward: forward output Y [rows][ldaux] whose act' scales the product, or null
  int64_t ldaux;
  float* out;          // fp32 store [rows][ldo] of the layer result, or null; with rinv: fp16 store (see rinv)
  int64_t ldo;
  int N;               // valid output columns
  int act;             // forward: activation; backward: derivative taken at aux
  // backward prec 6, hidden layers: non-null -> `out` holds the layer's dZ as fp16 [rows][ldo] in the row scale of the
  // next layer's fp16 operands (each row's largest |dZ| in [2^13, 2^14)), rinv[row] = the inverse scale 2^(e - 14)
  // (0 for an all-zero row), and *emax = max over rows of e + 1000 (0: every row zero) -- the weight gradients' fp16
  // operands (mms_gemm_tn_wide16)
  float* rinv;
  unsigned* emax;
  // hidden layers: forward -> `out` holds fp16 rows [rows][ldo] of the activations (the backward's act' source and the
  // weight gradients' X); backward -> `aux` is such an fp16 row buffer
  int f16;
};

typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
// 4 floats -> 4 fp16 values, stored as one 8-B (non-temporal) write
__device__ __forceinline__ void st_nt4h(float* base_as_half, int64_t off, f32x4 v) {
  const f16x4_t h = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
  __builtin_nontemporal_store(h, reinterpret_cast<f16x4_t*>(reinterpret_cast<_Float16*>(base_as_half) + off));
}
// 4 fp16 values loaded as 8 B, carried in .x / .y of an f32x4 until widened (the load stays in flight)
__device__ __forceinline__ f32x4 ld_nt4h(const float* base_as_half, int64_t off) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = __builtin_nontemporal_load(
      reinterpret_cast<const u32x2*>(reinterpret_cast<const _Float16*>(base_as_half) + off));
  return f32x4{__uint_as_float(v[0]), __uint_as_float(v[1]), 0.f, 0.f};
}
__device__ __forceinline__ f32x4 widen4h(f32x4 v) {
  const f16x2_t p0 = __builtin_bit_cast(f16x2_t, __float_as_uint(v[0]));
  const f16x2_t p1 = __builtin_bit_cast(f16x2_t, __float_as_uint(v[1]));
  return f32x4{(float)p0[0], (float)p0[1], (float)p1[0], (float)p1[1]};
}

struct ChainArgs {
  const float* X;      // layer-0 input [rows][ldx], K0 valid columns (16-B aligned rows)
  int64_t ldx;
  int K0;
  int64_t M;
  int64_t rows_full;   // SDF tap rows (>= rows_full): forward keeps only column 0 of the last layer,
                       // backward reads only column 0 of the input
  const float* xaux;   // backward: input first scaled by act'(xaux) (the last forward activation), or null
  int64_t ldxaux;
  int xact;
  float* xout;         // backward: store of the scaled input (dZ of the last forward layer), or null
  int64_t ldxout;
  float beta, thr;     // Softplus(beta, threshold)
  const float* w2row0; // forward: fp32 row 0 of the last layer's weight for the single-output row blocks
  float* tap_part;     // backward, SDF taps: per-block partials [blocks from rows_full / 128][ld_tap] of
  int64_t ld_tap;      //   sum over rows >= rows_full of X[m, 0] * aux0[m, :] (cols < N0) and of X[m, 0] (col N0)
  ChainLayer L[4];     // 3 or 4 layers (kernel template NL)
};

// activation derivative from the forward OUTPUT y (compile-time activation: branch-free epilogues)
template <int ACT>
__device__ __forceinline__ float act_grad_out(float y, float beta, float thr) {
  if constexpr (ACT == 1) return y > 0.f ? 1.f : 0.f;
  if constexpr (ACT == 2) {
    const float by = y * beta;
    return by > thr ? 1.f : 1.0f - __builtin_amdgcn_exp2f(-by * 1.4426950408889634f);
  }
  if constexpr (ACT == 3) return y * (1.0f - y);
  return 1.f;
}

// forward activation (the bf16 modes' hardware-transcendental forms of mms::act_fwd_fast, without branches)
template <int ACT>
__device__ __forceinline__ float act_fwd(float v, float beta, float thr) {
  if constexpr (ACT == 1) return v > 0.f ? v : 0.f;
  if constexpr (ACT == 2) {
    const float bx = v * beta;
    const float e = __builtin_amdgcn_exp2f(bx * 1.4426950408889634f);
    const float sp = __builtin_amdgcn_logf(1.0f + e) * (0.6931471805599453f * __builtin_amdgcn_rcpf(beta));
    return bx > thr ? v : sp;
  }
  if constexpr (ACT == 3) return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-v * 1.4426950408889634f));
  return v;
}

// PREC 5: fp16 operands (the reference GPU's autocast precision, trainer.py:51), one image, the fp16 bits carried in the
// bf16x8 vector type (mma reinterprets them)
template <int PREC>
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
  if constexpr (PREC == 5) {
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
    f16x8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)v[j];
    hi = __builtin_bit_cast(bf16x8, h);
    lo = hi;
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b = (__bf16)v[j];
    hi[j] = b;
    if constexpr (PREC >= 2) lo[j] = (__bf16)(v[j] - (float)b);
  }
}

template <int PREC>
constexpr int nimg() { return PREC == 2 ? 2 : 1; }

typedef __attribute__((address_space(3))) void lds_void;

// wait until at most N vector-memory operations of this wave are outstanding and its LDS reads have returned,
// then the block barrier (one asm statement with a memory clobber: no LDS read of the ring moves above either).
// lgkmcnt(0): gfx950's back-off barrier gets no compiler-inserted wait before an asm s_barrier, so without it a
// lagging wave's ds_read of slot (s - 1) % 3 could still be in flight when another wave's LDS-DMA overwrites that
// slot as (s + 2) % 3.  The MFMAs already wait on those reads, so the extra wait costs nothing.
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// 16 B per lane, global -> LDS (lane-linear at lds_addr), issued as inline asm: the compiler does not see an LDS
// DMA, so it does not guard every later LDS read of the ring with a full vmcnt(0) drain (which waited out the
// prefetch of the next two k-steps); the ring's ordering is the explicit wait_vm_barrier above.
__device__ __forceinline__ void lds_dma16(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}
// the same for streamed data read once (activations): non-temporal, so it does not evict the weights every block
// re-reads from L2
__device__ __forceinline__ void lds_dma16_nt(const void* src, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(src), "s"(lds_addr) : "memory", "m0");
}

// compile-time loop: f(std::integral_constant<int, i>) for i in [0, N)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

}  // namespace
