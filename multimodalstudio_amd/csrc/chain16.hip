// Fused weight-normed MLP chains at TWO waves per SIMD: the SDF field's 71 -> 256 -> 256 -> 257 Softplus(100) MLP,
// forward (training: hidden layers stored; sampler: no stores, single-output rows) and backward-data, one launch each.
//
// Reference layers: nn.Linear + activation under weight norm (/root/reference/src/field_components/mlp.py:152-209)
// inside FeatureGridAndMLP (field_components/feature_structures.py:153-169) for SDFField (fields/surface_field.py:99-116);
// the 4-tap gradient rows (model_components/surface_model.py:137-153) need only the sdf column of the last layer.
//
// Why a second kernel family (mlp_chain.hip holds the first).  The 32x32x16 chain keeps a layer's 256 accumulators per
// lane plus the previous layer's operand in registers -- ~470 VGPR+AGPR, one wave per SIMD -- and its MFMA pipe sat
// 74-79 % idle (profiles/round4_pmc_mfma_summary.txt): with nothing else on the SIMD, every LDS read latency, every
// barrier and the lazy epilogue's VALU (bias, Softplus, bf16 split: ~12 instructions per element, as much issue time
// as the MFMAs leave free) stalled the pipe.  Here a wave carries 16 data rows through v_mfma_f32_16x16x32_bf16: the
// accumulator of a 256-unit layer is 64 registers instead of 128 and the register-fed operand of the next layer 64 (hi +
// lo) instead of 128, so a wave fits in 256 registers and two share each SIMD: one wave's epilogue, waits and LDS
// latency run under the other's MFMAs.  Same FLOPs per MFMA cycle; a 128-row block of 8 waves reads each weight
// fragment from L2 once, as before.
//
// Orientation (as mlp_chain.hip): H^T[n][m] = sum_k W[n][k] X[m][k], data rows m on the MFMA column (lane) axis.  The
// 16x16 accumulator gives lane l data row l & 15 and units 4 (l >> 4) + i of the tile; the next layer's B operand of
// k-step s (32 units) takes tiles 2 s and 2 s + 1 straight from registers, K position 8 g + j <- unit 32 s + 4 g + j
// (j < 4) or 32 s + 16 + 4 g + j - 4 (mms_mlp_pack's 16x16x32 permuted layout).  Layer-0 and backward inputs, and the
// backward's activation-derivative sources, arrive by LDS-DMA one k-step ahead (2-slot rings, one barrier per k-step,
// exact vmcnt accounting -- run_layer16).  Precision: PREC 1 bf16 operands, PREC 2 split bf16x3 (3 MFMAs per
// product), fp32 accumulation.
#include "common.h"
#include "chain_common.h"

namespace {

// Diagnostic builds only (scripts/lib_variants.py "c16a<N>"; the product library has 0): ablation bits -- 1: no MFMA
// (the fragment reads kept), 2: no weight DMA, 4: no block barrier (waits kept), 8: no epilogue VALU / stores,
// 16: no input DMA (pre), 32: no vmcnt wait (the DMAs still issued), 64: weight DMA into the spare chunk only
#ifndef MMS_C16_ABL
#define MMS_C16_ABL 0
#endif

// k-steps a load is issued ahead of its use in the SDF chains (the radiance chains' LDS holds one: depth 1)
#ifndef MMS_C16_SDF_DEPTH
#define MMS_C16_SDF_DEPTH 1
#endif

constexpr int kW16 = 8;                 // waves per block (two per SIMD), 16 rows each
constexpr int kRows16 = 16 * kW16;      // 128 rows per block
constexpr int kMaxT16 = 20;             // widest layer: 20 tiles (the radiance backward's 317 input columns)

template <int PREC>
__device__ __forceinline__ void mma16(f32x4& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                      const bf16x8& bl) {
  if constexpr (PREC == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// streamed inputs (layer-0 rows, xaux, the backward's Y sources) by non-temporal LDS-DMA (MMS_C16_NT, default on)
#ifndef MMS_C16_NT
#define MMS_C16_NT 1
#endif
__device__ __forceinline__ void dma_stream(const void* src, uint32_t lds_addr) {
  if constexpr ((MMS_C16_ABL & 16) != 0) return;
  if constexpr (MMS_C16_NT != 0) lds_dma16_nt(src, lds_addr);
  else lds_dma16(src, lds_addr);
}

// per-wave streamed inputs (layer-0 rows, xaux, the backward's Y sources) loaded straight into VGPRs one k-step ahead
// (MMS_C16_VIN) instead of by LDS-DMA; the k-step then consumes them (get_b) BEFORE issuing the next step's loads, so the
// compiler's own vmcnt waits never count the invisible weight DMAs issued after a load
#ifndef MMS_C16_VIN
#define MMS_C16_VIN 0
#endif

template <int N>
__device__ __forceinline__ void wait16() {
  if constexpr ((MMS_C16_ABL & 32) != 0)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else if constexpr ((MMS_C16_ABL & 4) != 0)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  else
    wait_vm_barrier<N>();
}

// LDS-DMA instructions per wave per k-step staging NT tiles (uniform over the 8 waves: padded with dummy loads)
template <int PREC, int NT>
constexpr int stage_per16() { return (nimg<PREC>() * NT + kW16 - 1) / kW16; }

// k-step s's weight fragments of tiles [0, NT) (hi, then lo) into ring slot s % RING.  Packed images are fragment-major:
// fragment (k-step s, tile t) is one contiguous 1 KiB block at element ((s * NT + t) * 64 + lane) * 8.
template <int PREC, int NT, int SLOT, int RING>
__device__ __forceinline__ void stage16(const ChainLayer& Ly, int s, int wave, int lane, bf16x8 (*ring)[SLOT][64]) {
  if constexpr ((MMS_C16_ABL & 2) != 0) return;
  constexpr int TOTAL = nimg<PREC>() * NT;
#pragma unroll
  for (int i = 0; i < stage_per16<PREC, NT>(); ++i) {
    const int c = wave + kW16 * i;
    const bool real = c < TOTAL;
    const int cc = real ? c : 0;
    const int img = cc / NT, t = cc - img * NT;
    const __bf16* base = Ly.a_hi;
    if constexpr (PREC == 2) base = img ? Ly.a_lo : Ly.a_hi;
    const __bf16* src = base + ((int64_t)(s * NT + t) * 64 + lane) * 8;
    const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>(
        (lds_void*)&ring[s % RING][(real && (MMS_C16_ABL & 64) == 0) ? c : SLOT - 1][0]);
    lds_dma16(src, __builtin_amdgcn_readfirstlane(dst));
  }
}

// One layer: acc[t] (t < nt) += sum_{s < ks} A(s, t) . B(s), B(s) = get_b(s) (compile-time s after unrolling).  ks is
// block-uniform (every wave takes every barrier), nt <= NT may be smaller per wave.  Pipeline one k-step deep: step s
// issues pre(s + 1) (PRE LDS-DMA instructions: inputs / derivative sources) and the weight DMA of step s + 1, then
// get_b(s) (GOPS vector-memory instructions: the stores of the lazy epilogue).  The wait before step s is exact: only
// get_b(s - 1)'s stores may stay in flight, so no store or prefetch holds a k-step up (vmcnt retires in issue order).
// The same staging through VGPRs (MMS_C16_VSTAGE): global_load_dwordx4 at step s - 1, ds_write_b128 into the slot after
// that step's MFMAs (the loads have the whole step to land)
#ifndef MMS_C16_VSTAGE
#define MMS_C16_VSTAGE 0
#endif
template <int PREC, int NT>
__device__ __forceinline__ void stage16_load(const ChainLayer& Ly, int s, int wave, int lane,
                                             bf16x8 (&w)[stage_per16<PREC, NT>()]) {
  constexpr int TOTAL = nimg<PREC>() * NT;
#pragma unroll
  for (int i = 0; i < stage_per16<PREC, NT>(); ++i) {
    const int c = wave + kW16 * i;
    const int cc = c < TOTAL ? c : 0;
    const int img = cc / NT, t = cc - img * NT;
    const __bf16* base = Ly.a_hi;
    if constexpr (PREC == 2) base = img ? Ly.a_lo : Ly.a_hi;
    w[i] = *reinterpret_cast<const bf16x8*>(base + ((int64_t)(s * NT + t) * 64 + lane) * 8);
  }
}
template <int PREC, int NT, int SLOT>
__device__ __forceinline__ void stage16_store(bf16x8 (*slot)[64], int wave, int lane,
                                              const bf16x8 (&w)[stage_per16<PREC, NT>()]) {
  constexpr int TOTAL = nimg<PREC>() * NT;
#pragma unroll
  for (int i = 0; i < stage_per16<PREC, NT>(); ++i) {
    const int c = wave + kW16 * i;
    if (c < TOTAL) slot[c][lane] = w[i];
  }
}

template <int GOPS>
constexpr int gops16(int s) { return s < 0 ? 0 : GOPS; }

template <int PREC, int NT, int KS, int PRE, int GOPS, int SLOT, int DEP, typename Pre, typename GetB>
__device__ __forceinline__ void run_layer16(const ChainLayer& Ly, int ks, int nt, f32x4 (&acc)[NT], int wave, int lane,
                                            bf16x8 (*ring)[SLOT][64], Pre&& pre, GetB&& get_b) {
  constexpr int kDep16 = DEP, kRing16 = DEP + 1;
  constexpr int PER = stage_per16<PREC, NT>();
  wait16<63>();  // every wave is done with the ring slots (previous layer / launch prologue)
  if constexpr (MMS_C16_VSTAGE != 0) {
    static_assert(DEP == 1, "register staging: one k-step ahead");
    bf16x8 w[PER];
    if (ks > 0) {
      pre(0);
      stage16_load<PREC, NT>(Ly, 0, wave, lane, w);
      stage16_store<PREC, NT, SLOT>(ring[0], wave, lane, w);
    }
    static_for<KS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if (s < ks) {
        wait16<gops16<GOPS>(s - 1)>();
        if (s + 1 < ks) {
          pre(s + 1);
          stage16_load<PREC, NT>(Ly, s + 1, wave, lane, w);
        }
        bf16x8 bh, bl;
        get_b(s, bh, bl);
        const bf16x8* slot = &ring[s & 1][0][0];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (t < nt) {
            const bf16x8 ah = slot[t * 64 + lane];
            const bf16x8 al = PREC == 2 ? slot[(NT + t) * 64 + lane] : ah;
            mma16<PREC>(acc[t], ah, al, bh, bl);
          }
        }
        if (s + 1 < ks) stage16_store<PREC, NT, SLOT>(ring[(s + 1) & 1], wave, lane, w);
      }
    });
    return;
  }
  if constexpr (MMS_C16_VIN != 0) {
    static_assert(DEP == 1, "VGPR-staged inputs: one k-step ahead");
    if (ks > 0) {
      pre(0);
      stage16<PREC, NT, SLOT, kRing16>(Ly, 0, wave, lane, ring);
    }
    static_for<KS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      if (s < ks) {
        wait16<0>();   // step s's loads and DMAs landed, and get_b(s - 1)'s stores (issued before them) retired
        bf16x8 bh, bl;
        get_b(s, bh, bl);
        if (s + 1 < ks) {
          pre(s + 1);
          stage16<PREC, NT, SLOT, kRing16>(Ly, s + 1, wave, lane, ring);
        }
        const bf16x8* slot = &ring[s & 1][0][0];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if (t < nt) {
            const bf16x8 ah = slot[t * 64 + lane];
            const bf16x8 al = PREC == 2 ? slot[(NT + t) * 64 + lane] : ah;
            mma16<PREC>(acc[t], ah, al, bh, bl);
          }
        }
      }
    });
    return;
  }
#pragma unroll
  for (int j = 0; j < kDep16; ++j) {
    if (j < ks) {
      pre(j);
      stage16<PREC, NT, SLOT, kRing16>(Ly, j, wave, lane, ring);
    }
  }
  static_for<KS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (s < ks) {
      // younger than this wave's step-s loads: get_b(s - kDep16 .. s - 1) and the loads of the steps already issued
      // after s (min(kDep16 - 1, ks - 1 - s) of them)
      static_assert(kDep16 == 1 || kDep16 == 2, "one or two k-steps ahead");
      constexpr int kG = gops16<GOPS>(s - 1) + (kDep16 == 2 ? gops16<GOPS>(s - 2) : 0);
      if (kDep16 == 2 && s + 1 < ks) wait16<kG + PRE + PER>();
      else wait16<kG>();
      if (s + kDep16 < ks) {
        pre(s + kDep16);
        stage16<PREC, NT, SLOT, kRing16>(Ly, s + kDep16, wave, lane, ring);
      }
      bf16x8 bh, bl;
      get_b(s, bh, bl);
      const bf16x8* slot = &ring[s % kRing16][0][0];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (t < nt) {
          const bf16x8 ah = slot[t * 64 + lane];
          const bf16x8 al = PREC == 2 ? slot[(NT + t) * 64 + lane] : ah;
          if constexpr ((MMS_C16_ABL & 1) != 0)
            asm volatile("" ::"v"(ah), "v"(al), "v"(bh), "v"(bl));
          else
            mma16<PREC>(acc[t], ah, al, bh, bl);
        }
      }
    }
  });
}

// sum over the 16 lanes of a DPP row (lanes with the same l >> 4: the 16 data rows of one unit group); lane 15 of the
// row holds the total
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// Activations are template arguments (forward ids or, backward, derivative ids: A0 of the backward's first register-fed
// product -- the last hidden forward layer --, A1 of the next).  Forward: KS0 k-steps of the input X (K0 columns),
// NT0 / NT1 / NT2 16-unit tiles; the epilogue of layer l (bias, activation, KEEP: fp32 store of 16 B per lane per tile,
// bf16 split) runs lazily in layer l + 1's k-step s for tiles 2 s, 2 s + 1.  Backward: the same on the transposed
// weights, last layer first; dZ = acc * act'(Y) with Y arriving by LDS-DMA, stored (for the weight gradients) and split.
template <int PREC, int KS0, int NT0, int NT1, int NT2, bool BWD, int A0, int A1, int A2, int XA, bool KEEP, int DEP>
__global__ __launch_bounds__(512) void chain16_kernel(ChainArgs a) {
  constexpr int kRing16 = DEP + 1;   // ring slots: the one being read + DEP in flight
  constexpr int NTMAX = NT0 > NT1 ? (NT0 > NT2 ? NT0 : NT2) : (NT1 > NT2 ? NT1 : NT2);
  static_assert(NTMAX <= kMaxT16, "layer wider than the ring");
  constexpr int SLOT = nimg<PREC>() * NTMAX + 1;   // 1 KiB chunks per ring slot: hi + lo images, + 1 spare (dummy loads)
  __shared__ __attribute__((aligned(1024))) bf16x8 ring[kRing16][SLOT][64];
  // per-wave input slices (layer 0) and derivative sources (backward layers 1, 2): [slot][wave][2 x 64 lane chunks]
  __shared__ __attribute__((aligned(1024))) f32x4 xring[kRing16][kW16][2][64];
  // backward of the radiance chain (XIO): the input is scaled by the last forward ReLU's derivative (xaux, its
  // slices beside the input's) and the scaled rows stored (xout: dZ of the last forward layer, for the weight gradients)
  constexpr bool XIO = BWD && XA != 0;
  __shared__ __attribute__((aligned(1024))) f32x4 aring[XIO ? kRing16 : 1][XIO ? kW16 : 1][2][64];
  __shared__ __attribute__((aligned(16))) float sbias[BWD ? 1 : 3][BWD ? 1 : 16 * kMaxT16];
  __shared__ __attribute__((aligned(16))) float sw0[BWD ? 1 : 16 * NT1];   // forward: last layer's weight row 0
  // the SDF backward: the taps' share of the last forward layer's weight-gradient row 0 (per-wave partial rows)
  constexpr bool kTapW = BWD && A0 == 2;
  __shared__ __attribute__((aligned(16))) float stap[kTapW ? kW16 : 1][kTapW ? 16 * NT0 + 4 : 1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int64_t mb = (int64_t)blockIdx.x * kRows16;
  const int64_t m0 = mb + 16 * wave;
  const int64_t m = m0 + r;
  const bool mval = m < a.M;
  // rows past M run on row M - 1 (every load / store issued; stores write row M - 1's own bits again)
  const int64_t mc = mval ? m : a.M - 1;
  const bool rowfull = mc < a.rows_full;
  const bool anyfull = m0 < a.rows_full;    // wave-uniform
  const bool blockfull = mb < a.rows_full;  // block-uniform
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  if constexpr (!BWD) {
    for (int l = 0; l < 3; ++l)
      for (int i = threadIdx.x; i < 16 * kMaxT16; i += 512)
        sbias[l][i] = (a.L[l].bias != nullptr && i < a.L[l].N) ? a.L[l].bias[i] : 0.f;
    for (int i = threadIdx.x; i < 16 * NT1; i += 512) sw0[i] = (a.w2row0 != nullptr && i < a.L[1].N) ? a.w2row0[i] : 0.f;
  }  // (visible after the first layer's opening barrier)
  float x0 = 0.f;   // backward, tap rows: dY[m, 0] (the taps' dW row 0 weight)
  const bool tapw = kTapW && a.tap_part != nullptr && mb + kRows16 > a.rows_full;   // block-uniform
  if constexpr (kTapW) {
    if (tapw) {
      const float v = a.X[mc * a.ldx];
      x0 = (mval && m >= a.rows_full) ? v : 0.f;
#pragma unroll
      for (int i = threadIdx.x; i < kW16 * (16 * NT0 + 4); i += 512) (&stap[0][0])[i] = 0.f;
    }
  }

  f32x4 vin[2][2], vina[2][2];   // MMS_C16_VIN: the streamed inputs' register ring [slot][piece]
  // ---- layer 0: B operand from memory (lane (r, g) takes columns 32 s + 8 g .. + 7 of its row), natural K order
  f32x4 acc0[NT0];
#pragma unroll
  for (int t = 0; t < NT0; ++t) acc0[t] = zero;
  {
    const float* xr = a.X + mc * a.ldx;
    const float* xa = XIO ? a.xaux + mc * a.ldxaux : nullptr;
    float* xo = XIO ? a.xout + mc * a.ldxout : nullptr;
    // backward on tap rows: only input column 0 is live (a block of tap rows needs k-step 0 alone)
    const int ks0 = (BWD && !blockfull) ? 1 : KS0;
    auto pre = [&](int s) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = 32 * s + 8 * g + 4 * j;
        const int c = col < a.K0 ? col : 0;
        if constexpr (MMS_C16_VIN != 0) {
          vin[s & 1][j] = ld_nt4(xr + c);
          if constexpr (XIO) vina[s & 1][j] = ld_nt4(xa + c);
          continue;
        }
        dma_stream(xr + c, __builtin_amdgcn_readfirstlane(
                              (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&xring[s % kRing16][wave][j][0])));
        if constexpr (XIO)
          dma_stream(xa + c, __builtin_amdgcn_readfirstlane(
                                (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&aring[s % kRing16][wave][j][0])));
      }
    };
    auto get_b = [&](int s, bf16x8& bh, bf16x8& bl) {
      const int k0 = 32 * s + 8 * g;
      const f32x4 x0v = MMS_C16_VIN ? vin[s & 1][0] : xring[s % kRing16][wave][0][lane];
      const f32x4 x1v = MMS_C16_VIN ? vin[s & 1][1] : xring[s % kRing16][wave][1][lane];
      float v[8] = {x0v[0], x0v[1], x0v[2], x0v[3], x1v[0], x1v[1], x1v[2], x1v[3]};
      if constexpr (XIO) {
        // scaled first, masked after: columns past K0 hold whatever the padded rows hold (possibly non-finite)
        const f32x4 w0 = MMS_C16_VIN ? vina[s & 1][0] : aring[s % kRing16][wave][0][lane];
        const f32x4 w1 = MMS_C16_VIN ? vina[s & 1][1] : aring[s % kRing16][wave][1][lane];
        const float wv[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= act_grad_out<XA>(wv[j], a.beta, a.thr);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j >= a.K0) v[j] = 0.f;
      if constexpr (BWD) {
        if (!rowfull) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (k0 + j > 0) v[j] = 0.f;
        }
        if constexpr (XIO) {
          // xout rows hold at least 32 ks0 columns (dispatch): two unguarded 16-B stores, zeros past K0
          st_nt4(xo + k0, f32x4{v[0], v[1], v[2], v[3]});
          st_nt4(xo + k0 + 4, f32x4{v[4], v[5], v[6], v[7]});
        }
      }
      split8<PREC>(v, bh, bl);
    };
    run_layer16<PREC, NT0, KS0, XIO ? 4 : 2, XIO ? 2 : 0, SLOT, DEP>(a.L[0], ks0, NT0, acc0, wave, lane, ring, pre, get_b);
  }
  if constexpr (kTapW) asm volatile("" ::"v"(x0));   // x0's load waited for here, not inside a k-loop

  // register-fed operand of k-step s from tiles 2 s, 2 s + 1 of the previous layer's accumulators.  Forward (act =
  // forward id): + bias, activation, (KEEP) store, split.  Backward (act = derivative id): * act'(Y) with Y from the
  // ring (pre_y), store dZ, split; TAPW: the taps' dW row 0 partial sums.
  auto pre_y = [&](const ChainLayer& Lp) {
    return [&, lp = &Lp](int s) {
      const float* yr = lp->aux + mc * lp->ldaux;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if constexpr (MMS_C16_VIN != 0)
          vin[s & 1][j] = ld_nt4(yr + 32 * s + 16 * j + 4 * g);
        else
          dma_stream(yr + 32 * s + 16 * j + 4 * g, __builtin_amdgcn_readfirstlane(
                      (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&xring[s % kRing16][wave][j][0])));
    };
  };
  auto nopre = [](int) {};
  constexpr int kGOPS = (MMS_C16_ABL & 8) ? 0 : ((BWD || KEEP) ? 2 : 0);

  // ---- layer 1
  f32x4 acc1[NT1];
#pragma unroll
  for (int t = 0; t < NT1; ++t) acc1[t] = zero;
  auto feed = [&](auto& accp, const ChainLayer& Lp, const float* sb, auto actc, bool tap, int s, bf16x8& bh,
                  bf16x8& bl) {
    constexpr int ACT = decltype(actc)::value;
    float v[8];
    if constexpr ((MMS_C16_ABL & 8) != 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = accp[2 * s][i];
        v[4 + i] = accp[2 * s + 1][i];
      }
    } else if constexpr (!BWD) {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(sb + 32 * s + 4 * g);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(sb + 32 * s + 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = act_fwd<ACT>(accp[2 * s][i] + b0[i], a.beta, a.thr);
        v[4 + i] = act_fwd<ACT>(accp[2 * s + 1][i] + b1[i], a.beta, a.thr);
      }
      if constexpr (KEEP) {
        float* o = Lp.out + mc * Lp.ldo + 32 * s + 4 * g;
        st_nt4(o, f32x4{v[0], v[1], v[2], v[3]});
        st_nt4(o + 16, f32x4{v[4], v[5], v[6], v[7]});
      }
    } else {
      const f32x4 y0 = MMS_C16_VIN ? vin[s & 1][0] : xring[s % kRing16][wave][0][lane];
      const f32x4 y1 = MMS_C16_VIN ? vin[s & 1][1] : xring[s % kRing16][wave][1][lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = accp[2 * s][i] * act_grad_out<ACT>(y0[i], a.beta, a.thr);
        v[4 + i] = accp[2 * s + 1][i] * act_grad_out<ACT>(y1[i], a.beta, a.thr);
      }
      float* o = Lp.out + mc * Lp.ldo + 32 * s + 4 * g;
      st_nt4(o, f32x4{v[0], v[1], v[2], v[3]});
      st_nt4(o + 16, f32x4{v[4], v[5], v[6], v[7]});
      if constexpr (kTapW) {
        if (tap) {
          // dW_last[0, n] += sum over the wave's tap rows of dY[m, 0] Y[m, n] (n = the 8 units of this lane's group)
          float p[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            p[i] = row16_sum(x0 * y0[i]);
            p[4 + i] = row16_sum(x0 * y1[i]);
          }
          if (r == 15) {
            float* sp = &stap[wave][32 * s + 4 * g];
            *reinterpret_cast<f32x4*>(sp) = f32x4{p[0], p[1], p[2], p[3]};
            *reinterpret_cast<f32x4*>(sp + 16) = f32x4{p[4], p[5], p[6], p[7]};
          }
        }
      }
    }
    split8<PREC>(v, bh, bl);
  };
  {
    auto get_b = [&](int s, bf16x8& bh, bf16x8& bl) {
      feed(acc0, a.L[0], sbias[0], std::integral_constant<int, A0>{}, tapw, s, bh, bl);
    };
    if constexpr (BWD)
      run_layer16<PREC, NT1, NT0 / 2, 2, kGOPS, SLOT, DEP>(a.L[1], NT0 / 2, NT1, acc1, wave, lane, ring, pre_y(a.L[0]),
                                                     get_b);
    else
      run_layer16<PREC, NT1, NT0 / 2, 0, kGOPS, SLOT, DEP>(a.L[1], NT0 / 2, NT1, acc1, wave, lane, ring, nopre, get_b);
  }

  // ---- layer 2 (the last)
  if (BWD || blockfull) {
    f32x4 acc2[NT2];
#pragma unroll
    for (int t = 0; t < NT2; ++t) acc2[t] = zero;
    // forward, a wave of tap rows: only the sdf column's tile
    const int nt2 = (!BWD && !anyfull) ? 1 : NT2;
    auto get_b = [&](int s, bf16x8& bh, bf16x8& bl) {
      feed(acc1, a.L[1], sbias[BWD ? 0 : 1], std::integral_constant<int, A1>{}, false, s, bh, bl);
    };
    if constexpr (BWD)
      run_layer16<PREC, NT2, NT1 / 2, 2, kGOPS, SLOT, DEP>(a.L[2], NT1 / 2, nt2, acc2, wave, lane, ring, pre_y(a.L[1]),
                                                     get_b);
    else
      run_layer16<PREC, NT2, NT1 / 2, 0, kGOPS, SLOT, DEP>(a.L[2], NT1 / 2, nt2, acc2, wave, lane, ring, nopre, get_b);
    // epilogue: forward + bias (+ activation A2), backward dx; columns < N (forward tap rows: column 0 alone)
    if (a.L[2].out != nullptr) {
      float* orow = a.L[2].out + mc * a.L[2].ldo;
      const int N = a.L[2].N;
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        if (t < nt2) {
          const int n0 = 16 * t + 4 * g;
          f32x4 v = acc2[t];
          if constexpr (!BWD) {
            const f32x4 bq = *reinterpret_cast<const f32x4*>(&sbias[2][n0]);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = act_fwd<A2>(v[i] + bq[i], a.beta, a.thr);
          }
          const bool col0_only = !BWD && !rowfull;
          if (col0_only) {
            if (n0 == 0) __builtin_nontemporal_store(v[0], orow);
          } else if (n0 + 4 <= N) {
            st_nt4(orow + n0, v);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (n0 + i < N) __builtin_nontemporal_store(v[i], orow + n0 + i);
          }
        }
      }
    }
  } else if constexpr (!BWD) {
    // a block of single-output rows (SDF taps, the sampler's queries): layer 1's epilogue, then output 0 of the last
    // layer as a 256-long fp32 dot product on the VALU (W row 0 from LDS) -- no ring k-steps for one column tile
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < NT1; ++t) {
      const int n0 = 16 * t + 4 * g;
      const f32x4 bq = *reinterpret_cast<const f32x4*>(&sbias[1][n0]);
      const f32x4 w = *reinterpret_cast<const f32x4*>(&sw0[n0]);
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = act_fwd<A1>(acc1[t][i] + bq[i], a.beta, a.thr);
        p = __builtin_fmaf(v[i], w[i], p);
      }
      if constexpr (KEEP) st_nt4(a.L[1].out + mc * a.L[1].ldo + n0, v);
    }
    p += __shfl_xor(p, 16);
    p += __shfl_xor(p, 32);
    if (mval && g == 0 && a.L[2].out != nullptr) __builtin_nontemporal_store(p + sbias[2][0], a.L[2].out + m * a.L[2].ldo);
  }

  if constexpr (kTapW) {
    if (tapw) {
      // column N0: sum of dY[m, 0] over the wave's tap rows (the bias gradient's share)
      const float xs = row16_sum(g == 0 ? x0 : 0.f);
      if (lane == 15) stap[wave][16 * NT0] = xs;
      __syncthreads();
      float* row = a.tap_part + (int64_t)(blockIdx.x - a.rows_full / kRows16) * a.ld_tap;
      for (int i = threadIdx.x; i <= 16 * NT0; i += 512) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kW16; ++w) v += stap[w][i];
        row[i] = v;
      }
    }
  }
}

template <int PREC, int KS0, int NT0, int NT1, int NT2, bool BWD, int A0, int A1, int A2, int XA, bool KEEP,
          int DEP = 1>
void launch_chain16(const ChainArgs& a, hipStream_t s) {
  const unsigned blocks = (unsigned)((a.M + kRows16 - 1) / kRows16);
  hipLaunchKernelGGL((chain16_kernel<PREC, KS0, NT0, NT1, NT2, BWD, A0, A1, A2, XA, KEEP, DEP>), dim3(blocks), dim3(512),
                     0, s, a);
}

// The served chains (ks0 = ceil(K0 / 32), nt_l = ceil(N_l / 16)):
//   SDF 71-256-256-257, Softplus(100) hidden layers, identity output (surface_field.py:99-116).  Forward with the
//     hidden layers stored (training) or not (the sampler's queries); backward with the derivative ids of layers 1, 0.
//   radiance 317-256-256-256, ReLU x 3 (radiance_field.py:72-77).  Forward with the hidden layers stored; backward
//     with the input scaled by the last ReLU's derivative (xaux, stored to xout).
template <int PREC>
bool dispatch_chain16(int ks0, const int* nt, bool bwd, const ChainArgs& a, hipStream_t s) {
  const int a0 = a.L[0].act, a1 = a.L[1].act, a2 = a.L[2].act;
  const bool hidden_full = a.L[0].N == 256 && a.L[1].N == 256;
  const bool keep = a.L[0].out != nullptr && a.L[1].out != nullptr;
  const bool nokeep = a.L[0].out == nullptr && a.L[1].out == nullptr;
  const bool bwd_hidden = a.L[0].aux && a.L[0].out && a.L[1].aux && a.L[1].out;
  const bool noxa = a.xaux == nullptr && a.xout == nullptr;
  if (!hidden_full) return false;
  if (!bwd && ks0 == 3 && nt[0] == 16 && nt[1] == 16 && nt[2] == 17 && a0 == 2 && a1 == 2 && a2 == 0) {
    if (keep) { launch_chain16<PREC, 3, 16, 16, 17, false, 2, 2, 0, 0, true, MMS_C16_SDF_DEPTH>(a, s); return true; }
    if (nokeep) { launch_chain16<PREC, 3, 16, 16, 17, false, 2, 2, 0, 0, false, MMS_C16_SDF_DEPTH>(a, s); return true; }
    return false;
  }
  if (bwd && ks0 == 9 && nt[0] == 16 && nt[1] == 16 && nt[2] == 5 && a0 == 2 && a1 == 2 && a2 == 0 && noxa &&
      bwd_hidden) {
    launch_chain16<PREC, 9, 16, 16, 5, true, 2, 2, 0, 0, false, MMS_C16_SDF_DEPTH>(a, s);
    return true;
  }
  if (!bwd && ks0 == 10 && nt[0] == 16 && nt[1] == 16 && nt[2] == 16 && a0 == 1 && a1 == 1 && a2 == 1 && keep &&
      a.rows_full >= a.M) {
    launch_chain16<PREC, 10, 16, 16, 16, false, 1, 1, 1, 0, true>(a, s);
    return true;
  }
  if (bwd && ks0 == 8 && nt[0] == 16 && nt[1] == 16 && nt[2] == 20 && a0 == 1 && a1 == 1 && a2 == 0 && bwd_hidden &&
      a.xaux != nullptr && a.xact == 1 && a.xout != nullptr && a.ldxout >= 32 * ks0 && a.rows_full >= a.M) {
    launch_chain16<PREC, 8, 16, 16, 20, true, 1, 1, 0, 1, false>(a, s);
    return true;
  }
  return false;
}

inline bool aligned16_(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

MMS_EXPORT int mms_mlp_chain16(int prec, int backward, int n_layers, const float* X, int64_t ldx, int K0, int64_t M,
                               int64_t rows_full, const float* xaux, int64_t ldxaux, int xact, float* xout,
                               int64_t ldxout, const void* const* a_hi, const void* const* a_lo,
                               const float* const* bias, const float* const* aux, const int64_t* ldaux,
                               float* const* out, const int64_t* ldo, const int* N, const int* act, float beta,
                               float thr, const float* w2row0, float* tap_part, int64_t ld_tap, void* stream) {
  const char* fn = "mms_mlp_chain16";
  MMS_REQUIRE(prec == 1 || prec == 2, fn, "prec must be 1 (bf16) or 2 (split bf16x3)");
  MMS_REQUIRE(n_layers == 3, fn, "3-layer chains only");
  MMS_REQUIRE(M >= 0 && K0 > 0, fn, "bad shape");
  if (M == 0) return 0;
  MMS_REQUIRE(X && a_hi && N && act && out && ldo, fn, "null pointer");
  MMS_REQUIRE(aligned16_(X) && ldx % 4 == 0 && ldx >= K0, fn, "input rows must be 16-B aligned");
  MMS_REQUIRE(!backward || xaux == nullptr || (aligned16_(xaux) && ldxaux % 4 == 0 && ldxaux >= K0), fn,
              "xaux rows must be 16-B aligned");
  MMS_REQUIRE(!backward || xout == nullptr || (aligned16_(xout) && ldxout % 4 == 0), fn, "xout rows must be 16-B aligned");
  ChainArgs a;
  a.X = X; a.ldx = ldx; a.K0 = K0; a.M = M; a.rows_full = rows_full < 0 ? M : rows_full;
  a.xaux = backward ? xaux : nullptr; a.ldxaux = ldxaux; a.xact = xact;
  a.xout = backward ? xout : nullptr; a.ldxout = ldxout;
  a.beta = beta; a.thr = thr;
  a.w2row0 = backward ? nullptr : w2row0;
  a.tap_part = backward ? tap_part : nullptr;
  a.ld_tap = ld_tap;
  MMS_REQUIRE(tap_part == nullptr || !backward || (act[0] == 2 && N[0] == 256 && ld_tap > N[0] && rows_full >= 0 &&
                                                   rows_full < M), fn,
              "the taps' weight-gradient partials (tap_part) are a feature of the SDF backward chain");
  MMS_REQUIRE(backward || rows_full >= M || w2row0 != nullptr, fn,
              "forward with single-output rows (rows_full < M) needs the last layer's fp32 weight row 0");
  int nt[4] = {0, 0, 0, 0};
  for (int l = 0; l < 4; ++l) a.L[l] = ChainLayer{};
  for (int l = 0; l < n_layers; ++l) {
    MMS_REQUIRE(a_hi[l] != nullptr && N[l] > 0, fn, "missing layer weights");
    MMS_REQUIRE(prec != 2 || (a_lo && a_lo[l] != nullptr), fn, "split bf16x3 needs the residual images");
    MMS_REQUIRE(act[l] >= 0 && act[l] <= 3, fn, "bad activation id");
    ChainLayer& L = a.L[l];
    L.a_hi = reinterpret_cast<const __bf16*>(a_hi[l]);
    L.a_lo = prec == 2 ? reinterpret_cast<const __bf16*>(a_lo[l]) : nullptr;
    L.bias = (!backward && bias) ? bias[l] : nullptr;
    L.aux = (backward && aux) ? aux[l] : nullptr;
    L.ldaux = (backward && ldaux) ? ldaux[l] : 0;
    MMS_REQUIRE(L.aux == nullptr || (aligned16_(L.aux) && L.ldaux % 4 == 0), fn, "aux rows must be 16-B aligned");
    L.out = out[l];
    L.ldo = ldo[l];
    const bool col0_only = !backward && l == n_layers - 1 && a.rows_full == 0;
    MMS_REQUIRE(L.out == nullptr || (col0_only && L.ldo >= 1) ||
                    (aligned16_(L.out) && L.ldo % 4 == 0 && L.ldo >= N[l]), fn, "output rows must be 16-B aligned");
    L.N = N[l];
    L.act = act[l];
    nt[l] = (N[l] + 15) / 16;
  }
  const int ks0 = (K0 + 31) / 32;
  hipStream_t s = mms::as_stream(stream);
  const bool ok = prec == 1 ? dispatch_chain16<1>(ks0, nt, backward != 0, a, s)
                            : dispatch_chain16<2>(ks0, nt, backward != 0, a, s);
  MMS_REQUIRE(ok, fn, "unsupported chain shape or activations (SDF 71-256-256-257 Softplus and radiance "
                      "317-256-256-256 ReLU chains only)");
  return mms::check_launch(fn);
}
