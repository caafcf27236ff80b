// Fused weight-normed MLP chains on gfx950: the SDF field's 71 -> 256 -> 256 -> 257 Softplus(100) MLP and the
// radiance field's 317 -> 256 -> 256 -> 256 ReLU MLP, forward and backward-data, one kernel launch each.
//
// Reference layers: nn.Linear + activation under weight norm (/root/reference/src/field_components/mlp.py:152-209)
// inside FeatureGridAndMLP (field_components/feature_structures.py:153-169) for SDFField
// (fields/surface_field.py:99-116) and RadianceField (fields/radiance_field.py:72-77).
//
// Orientation: every layer is computed transposed, H^T[n][m] = sum_k W[n][k] X[m][k], with the data rows m on
// the MFMA column (lane) axis and the output units n on its row (register) axis.  The 32x32 accumulator of
// v_mfma_f32_32x32x16_bf16 keeps its column on the lane and its rows in 16 registers, so the next layer --
// which sums over n, the tile's ROW index -- takes it as its B operand straight from registers (registers
// 8s..8s+7 = k-step s; cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand"): no LDS
// image, no barrier and no HBM round trip between layers.  Inside a register-fed k-step the operand holds
// units 0-3, 8-11, 4-7, 12-15 of the step, so mms_mlp_pack stores those layers' weight columns in that order
// and every A fragment stays one 16-byte load.  One wave carries 32 data rows through the whole chain; the
// weights stream from L2 as A fragments.
//
// Forward epilogue: + bias, activation, fp32 store of each layer's output (the backward reads it).
// Backward-data: dZ_l = (W_{l+1}^T dZ_{l+1}) * act'(Y_l), with act' taken from the stored forward OUTPUT
// (ReLU: Y > 0; Softplus(b): 1 - exp(-b Y) = sigmoid(b Z); Sigmoid: Y (1 - Y)) -- no pre-activation is ever
// stored -- and an fp32 store of every dZ for the weight-gradient GEMMs.
// PREC 1: bf16 operands; PREC 2: split bf16x3 (x = hi + lo, acc += lo.hi + hi.lo + hi.hi); PREC 3: split
// activations only (bf16 weights W~ = bf16(W), acc += W~ (h_hi + h_lo): the chain computes the MLP of the rounded
// weights with ~16-bit activations, so the SDF's tap differences stay exact differences of ONE function -- its
// weights' rounding is the mixed-precision "bf16 weights, fp32 master" one -- at 2 MFMAs and half the weight
// traffic of PREC 2); PREC 5: fp16 operands (forward chains); PREC 6 (backward chains): layer 0 as PREC 2, the
// register-fed layers fp16 with a per-row power-of-two scale (row_scale); fp32 accumulation.
#include "common.h"
#include "chain_common.h"

namespace {

template <int PREC>
__device__ __forceinline__ void mma(floatx16& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                    const bf16x8& bl) {
  if constexpr (PREC == 2) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  }
  if constexpr (PREC == 3) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  if constexpr (PREC == 5) {
    typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, bh), acc, 0,
                                                 0, 0);
    return;
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

// ---- weight fragments: block-shared, staged in LDS by LDS-DMA.  All four waves of a block multiply the SAME weight
// fragments (the A operand) with their own rows, so each k-step's fragments are fetched once per block
// (global_load_lds_dwordx4: no VGPRs, lane-linear 1 KiB per wave-instruction) into a 3-slot ring, two k-steps
// ahead of the MFMAs, with one barrier per k-step.  Per-wave streaming of the fragments from L2 right before their
// MFMAs (one wave per SIMD) left every k-step waiting on L2 latency: 6 % of the MFMA rate.
// Packed images are fragment-major (mms_mlp_pack): fragment (k-step s, tile t) is one contiguous 1 KiB block at
// element ((s * NT + t) * 64 + lane) * 8.
// The ring is D + 1 slots deep (D = k-steps a load is issued ahead of its use): D = MMS_CHAIN_DEPTH where the block's
// LDS allows it (chain_kernel's kD), else 2.  A slot holds the largest k-step of the kernel's layers (hi + lo images of
// its tiles) + 1 spare chunk (the dummy loads that even out the waves' DMA counts).
#ifndef MMS_CHAIN_DEPTH
#define MMS_CHAIN_DEPTH 2
#endif
// waves per block (32 rows each): 4 (one block of 128 rows per CU), or 2 (64-row blocks, two of them per CU when the
// LDS allows: their k-step barriers and epilogues then run independently of each other)
#ifndef MMS_CHAIN_NW
#define MMS_CHAIN_NW 4
#endif
constexpr int kNW = MMS_CHAIN_NW;
constexpr int kRowsB = 32 * kNW;
constexpr int kMaxTiles = 10;  // widest chain layer: 10 column tiles (320 units)

// Diagnostic build only (MMS_CHAIN_STAMPS=1, scripts/lib_variants.py "stamps"; the product library has none): each
// wave accumulates s_memtime deltas per layer l -- [4 l] the k-steps' wait + barrier, [4 l + 1] ring / input issue and
// get_b (the lazy epilogue, the backward's dZ stores), [4 l + 2] fragment reads + MFMA issue, [4 l + 3] the layer's
// entry (the previous layer's last MFMAs and the work between layers) -- and [16] the tail, written per (block, wave)
// to g_chain_stamps at the end.  Read their shares, not their sums: every stamp drains the wave's LDS reads.
#ifndef MMS_CHAIN_STAMPS
#define MMS_CHAIN_STAMPS 0
#endif
constexpr int kStamps = 17;
#if MMS_CHAIN_STAMPS
__device__ unsigned long long g_chain_stamps[1 << 20];
__device__ __forceinline__ unsigned long long chain_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif
__device__ __forceinline__ void stamp_seg(unsigned long long* st, unsigned long long* last, int k) {
#if MMS_CHAIN_STAMPS
  if (st != nullptr) {
    const unsigned long long n = chain_stamp();
    st[k] += n - *last;
    *last = n;
  }
#else
  (void)st; (void)last; (void)k;
#endif
}

// loads per wave per k-step when NTL tiles are staged (uniform over the block's waves: padded with dummy loads)
template <int PREC, int NTL>
constexpr int stage_per() { return (nimg<PREC>() * NTL + kNW - 1) / kNW; }

// issue k-step s's fragments of tiles [0, NTL) (hi, then lo) into ring slot s % (D + 1)
constexpr int cmax(int x, int y) { return x > y ? x : y; }

template <int PREC, int NT, int NTL, int D, int SLOT>
__device__ __forceinline__ void stage(const ChainLayer& Ly, int s, int wave, int lane, bf16x8 (*ring)[SLOT][64]) {
  static_assert(nimg<PREC>() * NTL < SLOT, "ring slot too small");
  constexpr int TOTAL = nimg<PREC>() * NTL;
#pragma unroll
  for (int i = 0; i < stage_per<PREC, NTL>(); ++i) {
    const int c = wave + kNW * i;
    const bool real = c < TOTAL;
    const int cc = real ? c : 0;
    const int img = cc / NTL, t = cc - img * NTL;
    const __bf16* base = Ly.a_hi;
    if constexpr (PREC == 2) base = img ? Ly.a_lo : Ly.a_hi;  // a select of two values (no divergent address)
    const __bf16* src = base + ((int64_t)(s * NT + t) * 64 + lane) * 8;
    const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&ring[s % (D + 1)][real ? c : SLOT - 1][0]);
    lds_dma16(src, __builtin_amdgcn_readfirstlane(dst));
  }
}

// vector-memory instructions get_b(s) issues: GE at even s, GO at odd s (none before the layer starts)
template <int GE, int GO>
constexpr int gops(int s) { return s < 0 ? 0 : ((s & 1) ? GO : GE); }

// the exact wait before a k-step: KG younger get_b instructions plus n = min(N, f) younger steps' PP loads each
template <int KG, int PP, int N>
__device__ __forceinline__ void wait_younger(int f) {
  if constexpr (N == 0) {
    wait_vm_barrier<KG>();
  } else {
    if (f >= N) wait_vm_barrier<KG + N * PP>();
    else wait_younger<KG, PP, N - 1>(f);
  }
}

// sum of gops over the D get_b steps before s
template <int GE, int GO, int D>
constexpr int gops_before(int s) { return D == 0 ? 0 : gops<GE, GO>(s - D) + gops_before<GE, GO, (D > 0 ? D - 1 : 0)>(s); }

// one layer: acc[t] (t < nt) += sum_{s < ks} A(s, t) . B(s); B(s) = get_b(s) (compile-time s: register arrays).
// ks and NTL are block-uniform (every wave takes part in every barrier); nt may be smaller per wave (nt <= NTL).
// Pipeline, D k-steps deep for everything a k-step reads from memory: step t issues pre(t + D) (the layer-0 input
// slices, PRE instructions) and the ring DMA of step t + D (PER instructions), then get_b(t) (GE / GO instructions:
// the lazy epilogue's stores, the backward's dZ stores).  The wait before step s is EXACT: it lets every instruction
// issued after step s's own loads stay in flight -- get_b(s - D .. s - 1) and the pre / DMA of the steps already
// issued after s -- so neither a store nor a later prefetch holds up a k-step (vmcnt retires in issue order, stores
// included).  Every counted instruction is issued unconditionally (clamped rows, no exec-skipped branches), so the
// counts are exact for every wave.
template <int PREC, int NT, int NTL, int KS, int PRE, int GE, int GO, int D, int SLOT, typename Pre, typename GetB>
__device__ __forceinline__ void run_layer(const ChainLayer& Ly, int ks, int nt, floatx16 (&acc)[NT], int wave,
                                          int lane, bf16x8 (*ring)[SLOT][64], Pre&& pre, GetB&& get_b,
                                          unsigned long long* st = nullptr, unsigned long long* st_last = nullptr) {
  constexpr int PER = stage_per<PREC, NTL>();
  static_assert(D >= 1 && D <= 4, "ring depth");
  stamp_seg(st, st_last, 3);
  wait_vm_barrier<63>();  // every wave is done with the ring (previous layer / launch prologue)
#pragma unroll
  for (int j = 0; j < D; ++j) {
    if (j < ks) {
      pre(j);
      stage<PREC, NT, NTL, D>(Ly, j, wave, lane, ring);
    }
  }
  static_for<KS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (s < ks) {
      // this wave's loads of step s have landed, and (barrier) every wave's; slot (s + D) % (D + 1) is free.
      // Younger instructions: get_b(s - D .. s - 1) and the min(D - 1, ks - 1 - s) steps issued after s.
      constexpr int kG = gops_before<GE, GO, D>(s);
      static_assert(kG + (D - 1) * (PRE + PER) <= 63, "vmcnt range");
      stamp_seg(st, st_last, 2);
      wait_younger<kG, PRE + PER, D - 1>(ks - 1 - s);
      stamp_seg(st, st_last, 0);
      if (s + D < ks) {
        pre(s + D);
        stage<PREC, NT, NTL, D>(Ly, s + D, wave, lane, ring);
      }
      bf16x8 bh, bl;
      get_b(s, bh, bl);
      stamp_seg(st, st_last, 1);
      const bf16x8* slot = &ring[s % (D + 1)][0][0];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (t < nt) {
          const bf16x8 ah = slot[t * 64 + lane];
          const bf16x8 al = PREC == 2 ? slot[(NTL + t) * 64 + lane] : ah;
          mma<PREC>(acc[t], ah, al, bh, bl);
        }
      }
    }
  });
}

// Epilogue of one accumulator tile t, in place.  Lane (m, h): register 4 g + i holds unit n = 32 t + 8 g + 4 h + i
// of data row m.  Forward: + bias (zero-padded LDS copy), activation.  Backward: * act'(aux), the aux row's four
// 16-B loads of the tile issued together (unconditional: a quad past N reads quad 0 and is zeroed; quads below N
// lie inside the row since the pitch is a multiple of 4 >= N).
template <bool BWD, int ACT>
__device__ __forceinline__ void epi_tile(floatx16& acc, int t, const ChainLayer& Ly, const float* sb, const float* ar,
                                         float* orow, bool only_col0, int h, float beta, float thr) {
  f32x4 q[4];
  if (BWD && ar != nullptr) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int n0 = 32 * t + 8 * g + 4 * h;
      q[g] = ld_nt4(ar + (n0 < Ly.N ? n0 : 0));
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n0 = 32 * t + 8 * g + 4 * h;
    f32x4 bq = {};
    if (!BWD) bq = *reinterpret_cast<const f32x4*>(sb + n0);
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x = acc[4 * g + i];
      if constexpr (!BWD) {
        x = act_fwd<ACT>(x + bq[i], beta, thr);
      } else {
        if (ar != nullptr) x *= act_grad_out<ACT>(n0 + i < Ly.N ? q[g][i] : 0.f, beta, thr);
      }
      acc[4 * g + i] = x;
      v[i] = x;
    }
    if (orow != nullptr) {
      if (only_col0) {
        if (n0 == 0) __builtin_nontemporal_store(v[0], orow);
      } else if (n0 + 4 <= Ly.N) {
        st_nt4(orow + n0, v);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (n0 + i < Ly.N) __builtin_nontemporal_store(v[i], orow + n0 + i);
      }
    }
  }
}

// The forward's lazy epilogue of a full 32-unit tile (hidden layers: N = 32 NT, checked at dispatch): bias,
// activation, and (KEEP) the fp32 store of the tile's 32 rows x 128 B, with no guards at all, so it schedules in one
// basic block with the MFMAs around it.  The store goes through the wave's LDS scratch (row pitch 36 floats: both
// the accumulator-layout writes and the row-contiguous reads are bank-conflict free): the accumulator gives each lane
// four 16-B pieces spread over its row, so storing from registers put 64 rows x 16 B into every store instruction and
// every 128-B row segment was written by 8 partial stores (2-3x write traffic, PMC WRITE_SIZE); from the scratch each
// of the 4 store instructions writes 8 whole 128-B row segments.  Rows past M store row M - 1's values there again
// (identical bits).  Still exactly 4 vector-memory instructions per lane (run_layer's counted waits).
constexpr int kScr = 36;  // scratch row pitch (floats)
#ifndef MMS_CHAIN_YAHEAD
// backward epilogue: Y tiles loaded ahead (1 = one tile ahead, the round-3c kernel; scripts/lib_variants.py, step
// A/B: SDF backward 370 -> 345 us at 2 or 4, radiance 165 at 1-4 but 177 at 8, where the 4-layer chains spill)
#define MMS_CHAIN_YAHEAD 4
#endif
#ifndef MMS_CHAIN_YAHEAD4
#define MMS_CHAIN_YAHEAD4 4  // the same for the 4-layer chains
#endif

template <int ACT, bool KEEP>
__device__ __forceinline__ void epi_tile_full(floatx16& acc, int t, const float* sb, float* obase, int64_t ldo,
                                              int64_t m0, int64_t M, float* scr, int lane, float beta, float thr,
                                              bool o16) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int n0 = 32 * t + 8 * g + 4 * h;
    const f32x4 bq = *reinterpret_cast<const f32x4*>(sb + n0);
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = act_fwd<ACT>(acc[4 * g + i] + bq[i], beta, thr);
      acc[4 * g + i] = v[i];
    }
    if constexpr (KEEP) *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) = v;
  }
  if constexpr (KEEP) {
    const int q = lane & 7;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * j + (lane >> 3);
      const f32x4 v = *reinterpret_cast<const f32x4*>(scr + row * kScr + 4 * q);
      const int64_t mr = m0 + row < M ? m0 + row : M - 1;
      if (o16) st_nt4h(obase, mr * ldo + 32 * t + 4 * q, v);
      else st_nt4(obase + mr * ldo + 32 * t + 4 * q, v);
    }
  }
}

// epi_tile_full in two parts, for the one-tile-ahead forward (MMS_CHAIN_AHEAD): bias + activation in place ...
template <int ACT>
__device__ __forceinline__ void epi_tile_act(floatx16& acc, int t, const float* sb, int lane, float beta, float thr) {
  const int h = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 bq = *reinterpret_cast<const f32x4*>(sb + 32 * t + 8 * g + 4 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[4 * g + i] = act_fwd<ACT>(acc[4 * g + i] + bq[i], beta, thr);
  }
}
// ... and (KEEP) the staged row-contiguous store of the activated tile (4 vector-memory instructions per lane)
template <bool KEEP>
__device__ __forceinline__ void epi_tile_store(const floatx16& acc, int t, float* obase, int64_t ldo, int64_t m0,
                                               int64_t M, float* scr, int lane, bool o16) {
  if constexpr (KEEP) {
    const int r = lane & 31, h = lane >> 5, q = lane & 7;
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) =
          f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * j + (lane >> 3);
      const f32x4 v = *reinterpret_cast<const f32x4*>(scr + row * kScr + 4 * q);
      const int64_t mr = m0 + row < M ? m0 + row : M - 1;
      if (o16) st_nt4h(obase, mr * ldo + 32 * t + 4 * q, v);   // (one store instruction either way)
      else st_nt4(obase + mr * ldo + 32 * t + 4 * q, v);
    }
  }
}

// Backward epilogue of a full 256-unit hidden layer, through the wave's LDS scratch like the forward's stores:
// dZ = acc * act'(Y) with the forward output Y read row-contiguously (each load instruction 8 rows x 128 B, the next
// tile's rows in flight while this tile is processed) and dZ stored the same way; both sides pass the accumulator
// layout through the scratch.  Rows past M read / write row M - 1 (identical values).
// TAPW (the SDF backward's first layer, W_last^T): the single-output rows' (rows >= rows_full, the taps) share of the
// last forward layer's weight-gradient row 0, dW[0, n] += sum_m X[m, 0] Y[m, n], accumulated from the Y rows this
// epilogue loads anyway (the grouped weight-gradient launch would re-read 4 M rows x 1 KB of Y for that one row):
// per lane 4 rows x 4 columns per tile, reduced over the wave's rows by xor shuffles into the wave's LDS row `sp`
// (plain LDS stores: nothing here adds a vector-memory instruction the k-loops' exact vmcnt waits would count); the
// block writes its partial row once, at the end of the kernel.  (Storing the per-lane partials unreduced, 8 rows per
// wave, and summing them at the end measured equal: tap blocks -2 %, the step within noise, round 5.)
// Diagnostic builds only (MMS_CHAIN_EPI_ABL bits, scripts/lib_variants.py with the stamp build): 1 = no Y loads
// (constant activations), 2 = no dZ stores, 4 = no scratch round trips (accumulator-layout values used as they are).
#ifndef MMS_CHAIN_EPI_ABL
#define MMS_CHAIN_EPI_ABL 0
#endif
template <int NT, int ACT, bool TAPW = false, int YMAX = MMS_CHAIN_YAHEAD>
__device__ __forceinline__ void epilogue_bwd_staged(floatx16 (&acc)[NT], const ChainLayer& Ly, int64_t m0, int64_t M,
                                                    float* scr, int lane, float beta, float thr,
                                                    const ChainArgs* ta = nullptr, float* sp = nullptr) {
  const int r = lane & 31, h = lane >> 5, q = lane & 7;
  int64_t rows[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t mr = m0 + 8 * j + (lane >> 3);
    rows[j] = mr < M ? mr : M - 1;
  }
  float x0[4] = {0.f, 0.f, 0.f, 0.f};   // TAPW: X[m, 0] of the lane's 4 rows (0 for centre rows and rows past M)
  if constexpr (TAPW) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t mr = m0 + 8 * j + (lane >> 3);
      const float v = ta->X[rows[j] * ta->ldx];
      x0[j] = (mr < M && mr >= ta->rows_full) ? v : 0.f;
    }
  }
  // Y tiles in flight: YA tiles are loaded before the first is used and tile t + YA is issued once tile t's registers
  // are free, so the layer's epilogue waits out the HBM latency about once instead of once per tile (one wave per
  // SIMD: no other wave hides it)
  constexpr int YA = NT < YMAX ? NT : YMAX;
  const bool st32 = Ly.rinv == nullptr;   // fp32 dZ stored here; fp16 dZ after the row scale (store_dz16)
  f32x4 y[YA][4];
  const bool y16 = Ly.f16 != 0;           // fp16 Y rows: 8-B loads, widened when used
  auto load = [&](int t, f32x4* dst) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr ((MMS_CHAIN_EPI_ABL & 1) != 0) dst[j] = f32x4{0.3f, 0.2f, 0.1f, 0.4f};
      else if (y16) dst[j] = ld_nt4h(Ly.aux, rows[j] * Ly.ldaux + 32 * t + 4 * q);
      else dst[j] = ld_nt4(Ly.aux + rows[j] * Ly.ldaux + 32 * t + 4 * q);
    }
  };
#pragma unroll
  for (int t = 0; t < YA; ++t) load(t, y[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    f32x4 (&yt)[4] = y[t % YA];
    if (y16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) yt[j] = widen4h(yt[j]);
    }
    if constexpr (TAPW) {
      f32x4 sw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) sw[c] = __builtin_fmaf(x0[j], yt[j][c], sw[c]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v = sw[c];
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        sw[c] = v;
      }
      if (lane < 8) *reinterpret_cast<f32x4*>(sp + 32 * t + 4 * q) = sw;
    }
    constexpr bool kScrRT = (MMS_CHAIN_EPI_ABL & 4) == 0;
    f32x4 ycopy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (kScrRT) *reinterpret_cast<f32x4*>(scr + (8 * j + (lane >> 3)) * kScr + 4 * q) = yt[j];
      else ycopy[j] = yt[j];
    }
    if (t + YA < NT) load(t + YA, yt);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 yv = kScrRT ? *reinterpret_cast<const f32x4*>(scr + r * kScr + 8 * g + 4 * h) : ycopy[g];
      f32x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = acc[t][4 * g + i] * act_grad_out<ACT>(yv[i], beta, thr);
        acc[t][4 * g + i] = v[i];
      }
      if constexpr (kScrRT) {
        if (st32) *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) = v;
      } else {
        ycopy[g] = v;
      }
    }
    if (st32) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = kScrRT ? *reinterpret_cast<const f32x4*>(scr + (8 * j + (lane >> 3)) * kScr + 4 * q) : ycopy[j];
        if constexpr ((MMS_CHAIN_EPI_ABL & 2) == 0) st_nt4(Ly.out + rows[j] * Ly.ldo + 32 * t + 4 * q, v);
      }
    }
  }
  if constexpr (TAPW) {
    float v = (q == 0) ? ((x0[0] + x0[1]) + (x0[2] + x0[3])) : 0.f;
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane == 0) sp[32 * NT] = v;
  }
}

// The backward's last layer (dx, no activation derivative): its tiles through the wave's LDS scratch like the hidden
// layers' dZ, so each store instruction writes 8 whole 128-B row segments instead of 64 rows x 16 B (the unstaged
// stores wrote the 71- / 317- / 256-column dx rows in 32-B pieces: 1.3-1.5x the algorithmic write bytes, PMC
// WRITE_SIZE).  Columns past N are not written (a partial quad stores its valid elements), nor rows past M.
template <int NT>
__device__ __forceinline__ void epilogue_out_staged(floatx16 (&acc)[NT], const ChainLayer& Ly, int nt, int64_t m0,
                                                    int64_t M, float* scr, int lane) {
  const int r = lane & 31, h = lane >> 5, q = lane & 7;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t < nt) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) =
            f32x4{acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 8 * j + (lane >> 3);
        const f32x4 v = *reinterpret_cast<const f32x4*>(scr + row * kScr + 4 * q);
        const int64_t mr = m0 + row;
        const int col = 32 * t + 4 * q;
        if (mr < M) {
          float* o = Ly.out + mr * Ly.ldo + col;
          if (col + 4 <= Ly.N) {
            st_nt4(o, v);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (col + e < Ly.N) __builtin_nontemporal_store(v[e], o + e);
          }
        }
      }
    }
  }
}

// The forward's last layer the same way: + bias, activation, then staged row-contiguous stores.  SDF tap rows (rows
// >= rows_full, only in the one block that straddles the boundary: whole tap blocks take the VALU path) store
// column 0 alone.
template <int NT, int ACT>
__device__ __forceinline__ void epilogue_fwd_out_staged(floatx16 (&acc)[NT], const ChainLayer& Ly, const float* sb,
                                                        int nt, int64_t m0, int64_t M, int64_t rows_full, float* scr,
                                                        int lane, float beta, float thr) {
  const int r = lane & 31, h = lane >> 5, q = lane & 7;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t < nt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n0 = 32 * t + 8 * g + 4 * h;
        const f32x4 bq = *reinterpret_cast<const f32x4*>(sb + n0);
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = act_fwd<ACT>(acc[t][4 * g + i] + bq[i], beta, thr);
        *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) = v;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 8 * j + (lane >> 3);
        const f32x4 v = *reinterpret_cast<const f32x4*>(scr + row * kScr + 4 * q);
        const int64_t mr = m0 + row;
        const int col = 32 * t + 4 * q;
        if (mr < M) {
          float* o = Ly.out + mr * Ly.ldo + col;
          if (mr >= rows_full) {
            if (col == 0) __builtin_nontemporal_store(v[0], o);
          } else if (col + 4 <= Ly.N) {
            st_nt4(o, v);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (col + e < Ly.N) __builtin_nontemporal_store(v[e], o + e);
          }
        }
      }
    }
  }
}

template <int NT, bool BWD, int ACT>
__device__ __forceinline__ void epilogue(floatx16 (&acc)[NT], const ChainLayer& Ly, const float* sb, int nt, int64_t m,
                                         int64_t mc, bool mval, bool only_col0, int h, float beta, float thr) {
  const float* ar = (BWD && Ly.aux != nullptr) ? Ly.aux + mc * Ly.ldaux : nullptr;
  float* orow = (Ly.out != nullptr && mval) ? Ly.out + m * Ly.ldo : nullptr;
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if (t < nt) epi_tile<BWD, ACT>(acc[t], t, Ly, sb, ar, orow, only_col0, h, beta, thr);
}

// accumulator tile -> the next layer's B fragments of k-steps 2 t, 2 t + 1 (registers 8 s .. 8 s + 7)
template <int PREC>
__device__ __forceinline__ void tile_to_b(const floatx16& acc, bf16x8* bh, bf16x8* bl) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[8 * s + j];
    split8<PREC>(v, bh[s], bl[s]);
  }
}

template <int PREC, int NT>
__device__ __forceinline__ void to_b(const floatx16 (&acc)[NT], bf16x8 (&bh)[2 * NT], bf16x8 (&bl)[2 * NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) tile_to_b<PREC>(acc[t], &bh[2 * t], &bl[2 * t]);
}

// The forward's lazy epilogue of register-fed layer l + 1's B operand, at k-step s (compile-time after unrolling):
// tile t = s / 2 of layer l is consumed by steps 2 t and 2 t + 1.  MMS_CHAIN_AHEAD (default): tile t + 1's bias,
// activation and bf16 split run at step 2 t -- independent of that step's MFMAs, so the scheduler can issue them
// between the MFMAs (one wave per SIMD: the stamp build measured the in-step epilogue as long as the MFMA issue, not
// overlapped) -- and tile t's store stays at step 2 t (4 stores per even step: run_layer's exact vmcnt counts).
#ifndef MMS_CHAIN_AHEAD
#define MMS_CHAIN_AHEAD 1
#endif
template <int PREC, int ACT, bool KEEP, int NT>
__device__ __forceinline__ void lazy_fwd_b(int s, floatx16 (&accp)[NT], bf16x8* bh, bf16x8* bl, const float* sb,
                                           float* obase, int64_t ldo, int64_t m0, int64_t M, float* scr, int lane,
                                           float beta, float thr, bool o16) {
  if ((s & 1) != 0) return;
  const int t = s >> 1;
#if MMS_CHAIN_AHEAD
  if (t == 0) {
    epi_tile_act<ACT>(accp[0], 0, sb, lane, beta, thr);
    tile_to_b<PREC>(accp[0], &bh[0], &bl[0]);
  }
  epi_tile_store<KEEP>(accp[t], t, obase, ldo, m0, M, scr, lane, o16);
  if (t + 1 < NT) {
    epi_tile_act<ACT>(accp[t + 1], t + 1, sb, lane, beta, thr);
    tile_to_b<PREC>(accp[t + 1], &bh[2 * t + 2], &bl[2 * t + 2]);
  }
#else
  epi_tile_full<ACT, KEEP>(accp[t], t, sb, obase, ldo, m0, M, scr, lane, beta, thr, o16);
  tile_to_b<PREC>(accp[t], &bh[s], &bl[s]);
#endif
}

// PREC 6 (backward chains only): layer 0 (B from memory) in split-bf16x3, the register-fed layers on fp16 operands
// with a per-row power-of-two scale.  row_scale: the row's largest |dZ| (both unit halves: lanes r, r + 32) brought
// to [2^13, 2^14) -- fp16's 11 significant bits for every value within 2^-27 of the row maximum, no overflow -- in
// place, before the B split; returns the inverse scale the next layer's accumulators (same data row on the lane) are
// multiplied by (exact: powers of two).
// eb: the row's e + 1000 (> 0), or 0 for an all-zero row -- the biased exponent store_dz16 reduces into *emax.
template <int NT>
__device__ __forceinline__ float row_scale(floatx16 (&acc)[NT], int& eb) {
  float mx = 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fabsf(acc[t][i]));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  int e = __builtin_amdgcn_frexp_expf(mx);  // mx < 2^e (0 for mx = 0)
  e = e < -100 ? -100 : (e > 100 ? 100 : e);
  eb = mx > 0.f ? e + 1000 : 0;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = __builtin_amdgcn_ldexpf(acc[t][i], 14 - e);
  return __builtin_amdgcn_ldexpf(1.f, e - 14);
}

// The row-scaled dZ of a hidden layer (after row_scale: the values the next layer's fp16 B operands are made of) as
// fp16 rows for the weight gradients (ChainLayer::rinv non-null): each tile through the wave's LDS scratch like the
// fp32 stores (8-B pieces of 64-B row segments), the row's inverse scale, and the wave's largest biased exponent
// into *emax (one vector atomic per wave).  Rows past M are not written.
template <int NT>
__device__ __forceinline__ void store_dz16(const floatx16 (&acc)[NT], const ChainLayer& Ly, int64_t m0, int64_t M,
                                           float* scr, int lane, float inv, int eb) {
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  const int r = lane & 31, h = lane >> 5, q = lane & 7;
  _Float16* o16 = reinterpret_cast<_Float16*>(Ly.out);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<f32x4*>(scr + r * kScr + 8 * g + 4 * h) =
          f32x4{acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * j + (lane >> 3);
      const f32x4 v = *reinterpret_cast<const f32x4*>(scr + row * kScr + 4 * q);
      const f16x4 hv = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
      if (m0 + row < M)
        __builtin_nontemporal_store(hv, reinterpret_cast<f16x4*>(o16 + (m0 + row) * Ly.ldo + 32 * t + 4 * q));
    }
  }
  const bool valid = m0 + r < M;
  // an all-zero row stores rinv 0: the weight gradients scale its X row by rinv (a zero row's row scale, 2^-14, would
  // lift X above fp16's range in a launch whose largest exponent is negative -- e.g. fixed-capacity padding rows)
  if (h == 0 && valid) Ly.rinv[m0 + r] = eb > 0 ? inv : 0.f;
  int e = valid ? eb : 0;
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) e = max(e, __shfl_xor(e, d));
  if (lane == 0 && e > 0) atomicMax(Ly.emax, (unsigned)e);
}

template <int NT>
__device__ __forceinline__ void unscale(floatx16 (&acc)[NT], float inv) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] *= inv;
}

// Activations are template arguments (A0..A2: layer activations, forward ids or backward derivative ids; XA: the
// backward's input scaling).  The forward's epilogue of layer l is LAZY: tile t is finished (bias, activation,
// store, bf16 split) inside layer l + 1's k-step 2 t, right before the MFMAs that consume it, so its VALU and
// transcendental work issues between the previous k-step's MFMAs (one wave per SIMD: nothing else hides it).
// NL = 4: a middle register-fed layer of NT1 tiles with activation A1 sits between layer 1 and the last layer (the
// background NeRF MLPs, 4 layers).  Backward: the same structure on the transposed weights, last layer first.
template <int PREC, int KS0, int NT0, int NT1, int NT2, bool BWD, int A0, int A1, int A2, int XA, bool KEEP, int NL>
__global__ __launch_bounds__(64 * kNW) void chain_kernel(ChainArgs a) {
  // operand modes: layer 0 and the register-fed layers (differ only for the backward's PREC 6)
  constexpr int P0 = PREC == 6 ? 2 : PREC, PR = PREC == 6 ? 5 : PREC;
  static_assert(PREC != 6 || BWD, "PREC 6 is a backward mode");
  // ring slot: the largest k-step (images x tiles) of the kernel's layers + the spare chunk; depth: MMS_CHAIN_DEPTH
  // where the block's LDS holds it
  constexpr int kSlotK = cmax(nimg<P0>() * NT0, nimg<PR>() * cmax(NT1, NT2)) + 1;
  constexpr bool kXio = BWD && XA != 0;
  constexpr int kStageB = (BWD || KEEP) ? kNW * 32 * kScr * 4 : 16;
  auto lds_for = [](int d) constexpr {
    return (d + 1) * (kSlotK * 1024 + (kXio ? 2 : 1) * 2048 * kNW) + kStageB + NL * 32 * kMaxTiles * 4 +
           32 * NT1 * 4 + kNW * (32 * NT0 + 4) * 4;
  };
  constexpr int kLdsCap = (kNW >= 4 ? 160 : 160 * kNW / 4) * 1024;   // the block's share of the CU's 160 KiB
  constexpr int kD = (MMS_CHAIN_DEPTH >= 4 && lds_for(4) <= kLdsCap) ? 4
                     : (MMS_CHAIN_DEPTH >= 3 && lds_for(3) <= kLdsCap) ? 3 : 2;
  __shared__ __attribute__((aligned(1024))) bf16x8 ring[kD + 1][kSlotK][64];
  // layer-0 input slices (and, backward radiance chain, the xaux slices): [slot][wave][2 x 64 lane chunks]
  __shared__ __attribute__((aligned(1024))) f32x4 xring[kD + 1][kNW][128];
  __shared__ __attribute__((aligned(1024))) f32x4 aring[kXio ? kD + 1 : 1][kNW][128];
  __shared__ __attribute__((aligned(16))) float sbias[NL][32 * kMaxTiles];  // forward biases, zero padded
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar staging addresses
  const int r = lane & 31, h = lane >> 5;
  // kRowsB rows per block, 32 per wave.  Waves past M keep running on clamped rows (no stores): every wave takes part
  // in the block's barriers.
  const int64_t mb = (int64_t)blockIdx.x * kRowsB;
  const int64_t m0 = mb + 32 * wave;
  const int64_t m = m0 + r;
  const bool mval = m < a.M;
  const int64_t mc = mval ? m : a.M - 1;
  // clamped rows past M replicate row M - 1 exactly (their stores land on it): the tap-row test uses the clamped row
  const bool rowfull = mc < a.rows_full;
  const bool anyfull = m0 < a.rows_full;   // wave-uniform
  const bool blockfull = mb < a.rows_full;  // block-uniform
  const floatx16 zero = {};
#if MMS_CHAIN_STAMPS
  unsigned long long st[kStamps] = {};
  unsigned long long st_last = chain_stamp();
#define MMS_ST(l) , st + 4 * (l), &st_last
#else
#define MMS_ST(l)
#endif
  __shared__ __attribute__((aligned(16))) float sw0[BWD ? 1 : 32 * NT1];  // forward: last layer's weight row 0 (fp32)
  // per-wave staging of the row-contiguous stores (forward KEEP) and of the backward's Y loads / dZ stores
  constexpr bool kStage = BWD || KEEP;
  __shared__ __attribute__((aligned(16))) float sscr[kStage ? kNW : 1][32 * kScr];
  float* scr = &sscr[kStage ? wave : 0][0];
  // the SDF backward (3 layers, Softplus, input = the last forward layer's dY): the taps' dW_last row-0 partials
  constexpr bool kTapW = BWD && NL == 3 && A0 == 2 && XA == 0;
  __shared__ __attribute__((aligned(16))) float stap[kTapW ? kNW : 1][32 * NT0 + 4];
  if constexpr (!BWD) {
#pragma unroll
    for (int l = 0; l < NL; ++l)
      for (int i = threadIdx.x; i < 32 * kMaxTiles; i += 64 * kNW)
        sbias[l][i] = (a.L[l].bias != nullptr && i < a.L[l].N) ? a.L[l].bias[i] : 0.f;
    for (int i = threadIdx.x; i < 32 * NT1; i += 64 * kNW) sw0[i] = (a.w2row0 != nullptr && i < a.L[1].N) ? a.w2row0[i] : 0.f;
  }  // (visible after the first layer's opening barrier)

  // ---- layer 0: B operand from memory, natural k order
  floatx16 acc0[NT0];
#pragma unroll
  for (int t = 0; t < NT0; ++t) acc0[t] = zero;
  {
    // backward of the radiance chain (XIO): the input is scaled by the last forward ReLU's derivative (xaux) and the
    // scaled rows are stored (xout: dZ of the last forward layer, for the weight gradients).  Rows past M use the
    // clamped row (identical values), so every load / store below is issued by every wave (exact vmcnt counts).
    constexpr bool XIO = BWD && XA != 0;
    const float* xr = a.X + mc * a.ldx;
    const float* xa = XIO ? a.xaux + mc * a.ldxaux : nullptr;
    float* xo = XIO ? a.xout + mc * a.ldxout : nullptr;
    // backward on SDF tap rows: only input column 0 is live (a block of tap rows needs k-step 0 alone)
    const int ks0 = (BWD && !blockfull) ? 1 : KS0;
    // k-step s's input slices (16 columns of the wave's 32 rows) land in LDS by LDS-DMA, two steps ahead, like the
    // weights: instruction j, lane i loads row (i & 31)'s quad q = 2 j + (i >> 5) to lane-linear LDS, i.e. quad-major
    // [q][row] images, so each lane's two 16-B reads of its row are bank-conflict free.  The compiler never sees these
    // loads, so it inserts no vmcnt waits of its own into the k-loop (compiler-visible loads drew vmcnt(0..3) waits
    // there that also drained the weight prefetch).  Quads past K0 read column 0 and are zeroed in get_b.
    auto pre = [&](int s) {
      const int slot = s % (kD + 1);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = 16 * s + 4 * (2 * j + (lane >> 5));
        const int c = col < a.K0 ? col : 0;
        lds_dma16(xr + c, __builtin_amdgcn_readfirstlane(
                              (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&xring[slot][wave][64 * j])));
        if constexpr (XIO)
          lds_dma16(xa + c, __builtin_amdgcn_readfirstlane(
                                (uint32_t)reinterpret_cast<uintptr_t>((lds_void*)&aring[slot][wave][64 * j])));
      }
    };
    auto get_b = [&](int s, bf16x8& bh, bf16x8& bl) {
      const int k0 = 16 * s + 8 * h;
      const f32x4* xs = &xring[s % (kD + 1)][wave][0];
      const f32x4 x0 = xs[64 * h + r], x1 = xs[64 * h + 32 + r];
      float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
      if constexpr (XIO) {
        // scaled first, masked after: columns past K0 hold whatever the padded rows hold (possibly non-finite)
        const f32x4* as = &aring[s % (kD + 1)][wave][0];
        const f32x4 w0 = as[64 * h + r], w1 = as[64 * h + 32 + r];
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
          // xout rows hold at least 16 ks0 columns (dispatch): two unguarded 16-B stores, zeros past K0
          st_nt4(xo + k0, f32x4{v[0], v[1], v[2], v[3]});
          st_nt4(xo + k0 + 4, f32x4{v[4], v[5], v[6], v[7]});
        }
      }
      split8<P0>(v, bh, bl);
    };
    run_layer<P0, NT0, NT0, KS0, XIO ? 4 : 2, XIO ? 2 : 0, XIO ? 2 : 0, kD>(a.L[0], ks0, NT0, acc0, wave, lane, ring,
                                                                         pre, get_b MMS_ST(0));
  }
  auto nopre = [](int) {};
  // forward layers 1 and 2: get_b(s) of an even step finishes (and with KEEP stores, 4 x 16 B per lane) one tile of the
  // previous layer; backward layers 1 and 2 take B from registers (no memory instructions)
  constexpr int kGE = (!BWD && KEEP) ? 4 : 0;
  bf16x8 b1h[2 * NT0], b1l[2 * NT0];
  float inv1 = 1.f;   // PREC 6: inverse scale of layer 1's accumulators
  if constexpr (BWD) {
    // the SDF backward (3 layers, Softplus, input = the last forward layer's dY): the taps' dW_last row 0 on the way
    if (kTapW && a.tap_part != nullptr && mb + kRowsB > a.rows_full)
      epilogue_bwd_staged<NT0, A0, kTapW>(acc0, a.L[0], m0, a.M, scr, lane, a.beta, a.thr, &a, &stap[wave][0]);
    else
      epilogue_bwd_staged<NT0, A0, false, NL == 4 ? MMS_CHAIN_YAHEAD4 : MMS_CHAIN_YAHEAD>(acc0, a.L[0], m0, a.M, scr,
                                                                                        lane, a.beta, a.thr);
    if constexpr (PREC == 6) {
      int eb;
      inv1 = row_scale<NT0>(acc0, eb);
      if (a.L[0].rinv != nullptr) store_dz16<NT0>(acc0, a.L[0], m0, a.M, scr, lane, inv1, eb);
    }
    to_b<PR, NT0>(acc0, b1h, b1l);
  }

  // ---- layer 1: B operand from layer 0's registers
  floatx16 acc1[NT1];
#pragma unroll
  for (int t = 0; t < NT1; ++t) acc1[t] = zero;
  {
    run_layer<PR, NT1, NT1, 2 * NT0, 0, kGE, 0, kD>(a.L[1], 2 * NT0, NT1, acc1, wave, lane, ring, nopre,
                                       [&](int s, bf16x8& bh, bf16x8& bl) {
      if constexpr (!BWD)
        lazy_fwd_b<PREC, A0, KEEP, NT0>(s, acc0, b1h, b1l, sbias[0], a.L[0].out, a.L[0].ldo, m0, a.M, scr, lane, a.beta,
                                        a.thr, a.L[0].f16 != 0);
      bh = b1h[s]; bl = b1l[s];
    } MMS_ST(1));
  }
  // ---- the last layer (index LL = NL - 1), fed by the registers of layer LP = LL - 1 (NT1 tiles, activation A1).
  // Forward: SDF tap rows need only the sdf column tile; a block of tap rows stages only that tile.
  auto last_layer = [&](floatx16 (&accp)[NT1], auto lpc, float invp) {
    constexpr int LP = decltype(lpc)::value, LL = LP + 1;
    bf16x8 b2h[2 * NT1], b2l[2 * NT1];
    float inv2 = 1.f;
    if constexpr (BWD) {
      if constexpr (PREC == 6) unscale<NT1>(accp, invp);
      epilogue_bwd_staged<NT1, A1, false, NL == 4 ? MMS_CHAIN_YAHEAD4 : MMS_CHAIN_YAHEAD>(accp, a.L[LP], m0, a.M, scr,
                                                                                        lane, a.beta, a.thr);
      if constexpr (PREC == 6) {
        int eb;
        inv2 = row_scale<NT1>(accp, eb);
        if (a.L[LP].rinv != nullptr) store_dz16<NT1>(accp, a.L[LP], m0, a.M, scr, lane, inv2, eb);
      }
      to_b<PR, NT1>(accp, b2h, b2l);
    }
    floatx16 acc2[NT2];
#pragma unroll
    for (int t = 0; t < NT2; ++t) acc2[t] = zero;
    const int nt2 = (!BWD && !anyfull) ? 1 : NT2;
    auto get_b2 = [&](int s, bf16x8& bh, bf16x8& bl) {
      if constexpr (!BWD)
        lazy_fwd_b<PREC, A1, KEEP, NT1>(s, accp, b2h, b2l, sbias[LP], a.L[LP].out, a.L[LP].ldo, m0, a.M, scr, lane,
                                        a.beta, a.thr, a.L[LP].f16 != 0);
      bh = b2h[s]; bl = b2l[s];
    };
    if (BWD || blockfull) {
      run_layer<PR, NT2, NT2, 2 * NT1, 0, kGE, 0, kD>(a.L[LL], 2 * NT1, nt2, acc2, wave, lane, ring, nopre, get_b2
                                                    MMS_ST(LL));
    } else {
      // a block of SDF tap rows (or the sampler's inference rows) needs only output 0 of the last layer: a 256-long
      // dot product per row, done in fp32 on the VALU (W row 0 from LDS) instead of 2 NT1 ring k-steps of one
      // bf16x3 column tile -- no barriers, no weight streaming, and fp32 instead of split-bf16 operand precision
      float p = 0.f;
#pragma unroll
      for (int t = 0; t < NT1; ++t) {
        epi_tile_full<A1, KEEP>(accp[t], t, sbias[LP], a.L[LP].out, a.L[LP].ldo, m0, a.M, scr, lane, a.beta, a.thr,
                                a.L[LP].f16 != 0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(sw0 + 32 * t + 8 * g + 4 * h);
#pragma unroll
          for (int i = 0; i < 4; ++i) p = __builtin_fmaf(accp[t][4 * g + i], w[i], p);
        }
      }
      p += __shfl_xor(p, 32);   // the two halves of the row's units (lanes r and r + 32)
      if (mval && h == 0 && a.L[LL].out != nullptr)
        __builtin_nontemporal_store(p + sbias[LL][0], a.L[LL].out + m * a.L[LL].ldo);
      return;
    }
    if constexpr (PREC == 6) unscale<NT2>(acc2, inv2);
    if constexpr (BWD && A2 == 0) {
      if (a.L[LL].out != nullptr) epilogue_out_staged<NT2>(acc2, a.L[LL], nt2, m0, a.M, scr, lane);
    } else if constexpr (!BWD && KEEP) {   // (the per-wave scratch exists for KEEP forwards)
      if (a.L[LL].out != nullptr)
        epilogue_fwd_out_staged<NT2, A2>(acc2, a.L[LL], sbias[LL], nt2, m0, a.M, a.rows_full, scr, lane, a.beta,
                                         a.thr);
    } else {
      epilogue<NT2, BWD, A2>(acc2, a.L[LL], sbias[LL], nt2, m, mc, mval, !BWD && !rowfull, h, a.beta, a.thr);
    }
  };

  // (the block's taps partial row is written after the last layer, below)
  if constexpr (NL == 4) {
    // ---- middle layer 2: B operand from layer 1's registers (same width and activation as layer 1)
    bf16x8 bmh[2 * NT1], bml[2 * NT1];
    float invm = 1.f;
    if constexpr (BWD) {
      if constexpr (PREC == 6) unscale<NT1>(acc1, inv1);
      epilogue_bwd_staged<NT1, A1, false, MMS_CHAIN_YAHEAD4>(acc1, a.L[1], m0, a.M, scr, lane, a.beta, a.thr);
      if constexpr (PREC == 6) {
        int eb;
        invm = row_scale<NT1>(acc1, eb);
        if (a.L[1].rinv != nullptr) store_dz16<NT1>(acc1, a.L[1], m0, a.M, scr, lane, invm, eb);
      }
      to_b<PR, NT1>(acc1, bmh, bml);
    }
    floatx16 accm[NT1];
#pragma unroll
    for (int t = 0; t < NT1; ++t) accm[t] = zero;
    run_layer<PR, NT1, NT1, 2 * NT1, 0, kGE, 0, kD>(a.L[2], 2 * NT1, NT1, accm, wave, lane, ring, nopre,
                                                  [&](int s, bf16x8& bh, bf16x8& bl) {
      if constexpr (!BWD)
        lazy_fwd_b<PREC, A1, KEEP, NT1>(s, acc1, bmh, bml, sbias[1], a.L[1].out, a.L[1].ldo, m0, a.M, scr, lane, a.beta,
                                        a.thr, a.L[1].f16 != 0);
      bh = bmh[s]; bl = bml[s];
    } MMS_ST(2));
    last_layer(accm, std::integral_constant<int, 2>{}, invm);
  } else {
    last_layer(acc1, std::integral_constant<int, 1>{}, inv1);
  }
#if MMS_CHAIN_STAMPS
  stamp_seg(st, &st_last, 16);
  if (lane == 0) {
    unsigned long long* o = g_chain_stamps + ((int64_t)blockIdx.x * 4 + wave) * kStamps;
    if (((int64_t)blockIdx.x * 4 + wave + 1) * kStamps <= (1 << 20))
      for (int i = 0; i < kStamps; ++i) o[i] = st[i];
  }
#endif
#undef MMS_ST
  if constexpr (kTapW) {
    if (a.tap_part != nullptr && mb + kRowsB > a.rows_full) {
      __syncthreads();
      float* row = a.tap_part + (int64_t)(blockIdx.x - a.rows_full / kRowsB) * a.ld_tap;
      for (int i = threadIdx.x; i <= 32 * NT0; i += 64 * kNW) {
        float v = stap[0][i];
#pragma unroll
        for (int w = 1; w < kNW; ++w) v += stap[w][i];
        row[i] = v;
      }
    }
  }
}

template <int PREC, int KS0, int NT0, int NT1, int NT2, bool BWD, int A0, int A1, int A2, int XA, bool KEEP = false,
          int NL = 3>
void launch_chain(const ChainArgs& a, hipStream_t s) {
  const unsigned blocks = (unsigned)((a.M + kRowsB - 1) / kRowsB);
  hipLaunchKernelGGL((chain_kernel<PREC, KS0, NT0, NT1, NT2, BWD, A0, A1, A2, XA, KEEP, NL>), dim3(blocks), dim3(64 * kNW), 0,
                     s, a);
}

// The served chains (ks0 = ceil(K0 / 16), nt_l = ceil(N_l / 32)) with their activations:
//   3 layers: SDF Softplus(100), Softplus(100), identity; radiance ReLU x 3 (backward: derivative ids of layers 1, 0
//             and none, the input scaled by the last ReLU's derivative).  Forward: both hidden layers full (256
//             units) and stored together (keep) or neither.
//   4 layers: the background NeRF base 39-256-256-256-256 and head 283-256-256-256-128 MLPs, ReLU throughout
//             (nerf_field.py:92-105), hidden layers stored.
template <int PREC>
bool dispatch_chain(int nl, int ks0, const int* nt, bool bwd, const ChainArgs& a, hipStream_t s) {
  const int a0 = a.L[0].act, a1 = a.L[1].act, a2 = a.L[2].act, a3 = nl == 4 ? a.L[3].act : -1;
  const bool noxa = a.xaux == nullptr;
  const int nh = nl - 1;  // hidden (stored) layers
  bool hidden_full = true, keep = true, nokeep = true, bwd_hidden = true, hidden64 = true;
  for (int l = 0; l < nh; ++l) {
    hidden_full = hidden_full && a.L[l].N == 256;
    hidden64 = hidden64 && a.L[l].N == 64;
    keep = keep && a.L[l].out != nullptr;
    nokeep = nokeep && a.L[l].out == nullptr;
    // backward: every hidden layer's dZ is stored and scaled by act'(Y) (the staged epilogue assumes all)
    bwd_hidden = bwd_hidden && a.L[l].aux != nullptr && a.L[l].out != nullptr;
  }
  const bool bwd_stored = bwd_hidden;
  bwd_hidden = bwd_stored && hidden_full;
  // the input scaling stores 16 ks0 columns per row (zeros past K0)
  const bool xio = !noxa && a.xact == 1 && a.xout != nullptr && a.ldxout >= 16 * ks0;
  const bool xio3 = !noxa && a.xact == 3 && a.xout != nullptr && a.ldxout >= 16 * ks0;
  if (nl == 3) {
    if (PREC != 6 && !bwd && ks0 == 5 && nt[0] == 8 && nt[1] == 8 && nt[2] == 9 && a0 == 2 && a1 == 2 && a2 == 0 && hidden_full &&
        (keep || nokeep)) {
      if constexpr (PREC != 6) {
        if (keep) launch_chain<PREC, 5, 8, 8, 9, false, 2, 2, 0, 0, true>(a, s);
        else launch_chain<PREC, 5, 8, 8, 9, false, 2, 2, 0, 0, false>(a, s);
      }
      return true;
    }
    if constexpr (PREC != 3 && PREC != 5 && PREC != 6) {   // (split activations: the SDF chains only)
      if (!bwd && ks0 == 20 && nt[0] == 8 && nt[1] == 8 && nt[2] == 8 && a0 == 1 && a1 == 1 && a2 == 1 &&
          hidden_full && keep) {
        launch_chain<PREC, 20, 8, 8, 8, false, 1, 1, 1, 0, true>(a, s);
        return true;
      }
    }
    if constexpr (PREC != 3 && PREC != 5) {   // (fp16 chains: forward only; PREC 6 is their backward)
      if (bwd && ks0 == 16 && nt[0] == 8 && nt[1] == 8 && nt[2] == 10 && a0 == 1 && a1 == 1 && a2 == 0 && xio &&
          bwd_hidden) {
        launch_chain<PREC, 16, 8, 8, 10, true, 1, 1, 0, 1>(a, s);
        return true;
      }
    }
    if (bwd && ks0 == 17 && nt[0] == 8 && nt[1] == 8 && nt[2] == 3 && a0 == 2 && a1 == 2 && a2 == 0 && noxa &&
        a.xout == nullptr && bwd_hidden) {
      launch_chain<PREC, 17, 8, 8, 3, true, 2, 2, 0, 0>(a, s);
      return true;
    }
    if constexpr (PREC == 5) {
      // fp16 forward chains: radiance 317-256-256-256 ReLU, the plain / polarization heads 256-64-64-C
      if (!bwd && ks0 == 20 && nt[0] == 8 && nt[1] == 8 && nt[2] == 8 && a0 == 1 && a1 == 1 && a2 == 1 &&
          hidden_full && keep) {
        launch_chain<PREC, 20, 8, 8, 8, false, 1, 1, 1, 0, true>(a, s);
        return true;
      }
      if (!bwd && ks0 == 16 && nt[0] == 2 && nt[1] == 2 && nt[2] == 1 && a0 == 1 && a1 == 1 && hidden64 && keep &&
          (a2 == 3 || a2 == 0)) {
        if (a2 == 3) launch_chain<PREC, 16, 2, 2, 1, false, 1, 1, 3, 0, true>(a, s);
        else launch_chain<PREC, 16, 2, 2, 1, false, 1, 1, 0, 0, true>(a, s);
        return true;
      }
    }
    if constexpr (PREC == 6) {
      // the modality heads' backward (plain: input scaled by the Sigmoid's derivative; polarization: plain)
      if (bwd && ks0 == 1 && nt[0] == 2 && nt[1] == 2 && nt[2] == 8 && a0 == 1 && a1 == 1 && a2 == 0 && bwd_stored &&
          hidden64) {
        if (xio3) { launch_chain<PREC, 1, 2, 2, 8, true, 1, 1, 0, 3>(a, s); return true; }
        if (noxa && a.xout == nullptr) { launch_chain<PREC, 1, 2, 2, 8, true, 1, 1, 0, 0>(a, s); return true; }
      }
    }
    if constexpr (PREC == 1 || PREC == 2) {
      // the plain modality heads 256-64-64-C (ReLU, ReLU, Sigmoid; field_heads.py:71-88), C <= 32, bf16 or split-bf16x3
      if (!bwd && ks0 == 16 && nt[0] == 2 && nt[1] == 2 && nt[2] == 1 && a0 == 1 && a1 == 1 && a2 == 3 && hidden64 &&
          keep) {
        launch_chain<PREC, 16, 2, 2, 1, false, 1, 1, 3, 0, true>(a, s);
        return true;
      }
      if (bwd && ks0 == 1 && nt[0] == 2 && nt[1] == 2 && nt[2] == 8 && a0 == 1 && a1 == 1 && a2 == 0 && xio3 &&
          bwd_stored && hidden64) {
        launch_chain<PREC, 1, 2, 2, 8, true, 1, 1, 0, 3>(a, s);
        return true;
      }
      // the polarization heads 256-64-64-3 (Stokes, no output activation; field_heads.py:90-106)
      if (!bwd && ks0 == 16 && nt[0] == 2 && nt[1] == 2 && nt[2] == 1 && a0 == 1 && a1 == 1 && a2 == 0 && hidden64 &&
          keep) {
        launch_chain<PREC, 16, 2, 2, 1, false, 1, 1, 0, 0, true>(a, s);
        return true;
      }
      if (bwd && ks0 == 1 && nt[0] == 2 && nt[1] == 2 && nt[2] == 8 && a0 == 1 && a1 == 1 && a2 == 0 && noxa &&
          a.xout == nullptr && bwd_stored && hidden64) {
        launch_chain<PREC, 1, 2, 2, 8, true, 1, 1, 0, 0>(a, s);
        return true;
      }
    }
    return false;
  }
  // 4-layer chains: the background MLPs, bf16 or split-bf16x3 (fp16: forward only; PREC 6: backward only)
  if constexpr (PREC == 1 || PREC == 2 || PREC == 5 || PREC == 6) {
    if (nl != 4 || nt[0] != 8 || nt[1] != 8 || nt[2] != 8 || a0 != 1 || a1 != 1 || a2 != 1) return false;
    if (PREC != 6 && !bwd && hidden_full && keep && a3 == 1) {
      // base 39-256x4 (NeRF background), head 283-256-256-256-128 (NeRF) / -256 (config-5 grid background)
      if constexpr (PREC != 6) {
        if (ks0 == 3 && nt[3] == 8) { launch_chain<PREC, 3, 8, 8, 8, false, 1, 1, 1, 0, true, 4>(a, s); return true; }
        if (ks0 == 18 && nt[3] == 4) { launch_chain<PREC, 18, 8, 8, 4, false, 1, 1, 1, 0, true, 4>(a, s); return true; }
        if (ks0 == 18 && nt[3] == 8) { launch_chain<PREC, 18, 8, 8, 8, false, 1, 1, 1, 0, true, 4>(a, s); return true; }
      }
    }
    if (PREC != 5 && bwd && a3 == 0 && xio && bwd_hidden) {
      if (ks0 == 16 && nt[3] == 2) { launch_chain<PREC, 16, 8, 8, 2, true, 1, 1, 0, 1, false, 4>(a, s); return true; }
      if (ks0 == 8 && nt[3] == 9) { launch_chain<PREC, 8, 8, 8, 9, true, 1, 1, 0, 1, false, 4>(a, s); return true; }
      if (ks0 == 16 && nt[3] == 9) { launch_chain<PREC, 16, 8, 8, 9, true, 1, 1, 0, 1, false, 4>(a, s); return true; }
    }
  }
  return false;
}

// perm(q): swap bits 2 and 3 of the in-step column (units 0-3, 8-11, 4-7, 12-15 of a register-fed k-step)
__device__ __forceinline__ int64_t perm_col(int64_t c) {
  const int64_t q = c & 15;
  return (c & ~(int64_t)15) | (q & 3) | ((q & 4) << 1) | ((q & 8) >> 1);
}

// one element i of a packed image, fragment-major ((k-step of 16, tile of 32) block, lane r + 32 (q >> 3)).
// permute bit 0: the register-fed column order
__device__ __forceinline__ void pack_elem(const float* __restrict__ W, int64_t N, int64_t K, int64_t ldw, int transpose,
                                          int permute, int64_t rows, int64_t cols, __bf16* __restrict__ hi,
                                          __bf16* __restrict__ lo, int64_t i) {
  const int64_t R = transpose ? K : N, C = transpose ? N : K;
  const int64_t nt = rows / 32;
  const int64_t row = i / cols, c = i - row * cols;
  const int64_t src = (permute & 1) ? perm_col(c) : c;
  float v = 0.f;
  if (row < R && src < C) v = transpose ? W[src * ldw + row] : W[row * ldw + src];
  const int64_t s = c >> 4, q = c & 15, t = row >> 5, r = row & 31;
  const int64_t o = ((s * nt + t) * 64 + r + 32 * (q >> 3)) * 8 + (q & 7);
  if (permute & 4) {   // fp16 image (bits stored in the bf16 buffer; mms_mlp_chain prec 5)
    hi[o] = __builtin_bit_cast(__bf16, (_Float16)v);
    return;
  }
  const __bf16 b = (__bf16)v;
  hi[o] = b;
  if (lo != nullptr) lo[o] = (__bf16)(v - (float)b);
}

__global__ void pack_kernel(const float* __restrict__ W, int64_t N, int64_t K, int64_t ldw, int transpose,
                            int permute, int64_t rows, int64_t cols, __bf16* __restrict__ hi, __bf16* __restrict__ lo) {
  const int64_t total = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    pack_elem(W, N, K, ldw, transpose, permute, rows, cols, hi, lo, i);
}

// every packed image of a model in one launch: element e of the concatenation belongs to the item whose elem0 range
// holds it (items sorted by elem0)
// (the items' start offsets staged in LDS and binary-searched: a linear scan of the ~35 items' global elem0 per
// element made this launch 20 us per forward)
constexpr int kPackLdsItems = 128;
__global__ void pack_batched_kernel(const MmsPackItem* __restrict__ items, int n_items, int64_t total) {
  __shared__ int64_t e0[kPackLdsItems];
  const bool lds = n_items <= kPackLdsItems;
  if (lds) {
    for (int j = threadIdx.x; j < n_items; j += blockDim.x) e0[j] = items[j].elem0;
    __syncthreads();
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int i = 0;
    if (lds) {
      // the last item whose elem0 <= e
      int lo = 0, hi = n_items - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (e0[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      i = lo;
    } else {
      while (i + 1 < n_items && e >= items[i + 1].elem0) ++i;
    }
    const MmsPackItem& it = items[i];
    pack_elem(it.W, it.N, it.K, it.ldw, it.transpose, it.permute, it.rows, it.cols,
              reinterpret_cast<__bf16*>(it.hi), reinterpret_cast<__bf16*>(it.lo), e - it.elem0);
  }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

#if MMS_CHAIN_STAMPS
// diagnostic build only: copy / clear the per-(block, wave) stamp sums (kStamps each)
MMS_EXPORT int mms_chain_stamps(unsigned long long* host, int64_t n, int clear) {
  if (n > (1 << 20)) n = 1 << 20;
  if (clear) {
    void* addr = nullptr;
    if (hipGetSymbolAddress(&addr, HIP_SYMBOL(g_chain_stamps)) != hipSuccess) return 1;
    return hipMemset(addr, 0, sizeof(unsigned long long) << 20) == hipSuccess ? 0 : 1;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chain_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

MMS_EXPORT int mms_mlp_pack_batched(const void* items, int n_items, int64_t total, void* stream) {
  const char* fn = "mms_mlp_pack_batched";
  MMS_REQUIRE(items && n_items > 0 && total > 0, fn, "empty batch");
  hipLaunchKernelGGL(pack_batched_kernel, dim3(mms::grid_for(total, 256, 8192)), dim3(256), 0, mms::as_stream(stream),
                     reinterpret_cast<const MmsPackItem*>(items), n_items, total);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_mlp_pack(const float* W, int64_t N, int64_t K, int64_t ldw, int transpose, int permute,
                            int64_t rows, int64_t cols, void* hi, void* lo, void* stream) {
  const char* fn = "mms_mlp_pack";
  MMS_REQUIRE(N > 0 && K > 0 && ldw >= K, fn, "bad weight shape");
  MMS_REQUIRE(rows >= (transpose ? K : N) && cols >= (transpose ? N : K), fn, "packed image smaller than the weight");
  MMS_REQUIRE((permute & ~5) == 0, fn, "permute: bit 0 (register-fed order) and bit 2 (fp16 image) only");
  MMS_REQUIRE(rows % 32 == 0 && cols % 16 == 0, fn, "packed image must be [32 x tiles][16 x k-steps]");
  MMS_REQUIRE(W && hi, fn, "null pointer");
  hipLaunchKernelGGL(pack_kernel, dim3(mms::grid_for(rows * cols, 256, 4096)), dim3(256), 0, mms::as_stream(stream), W,
                     N, K, ldw, transpose, permute, rows, cols, reinterpret_cast<__bf16*>(hi),
                     reinterpret_cast<__bf16*>(lo));
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_mlp_chain_block_rows(void) { return kRowsB; }

MMS_EXPORT int mms_mlp_chain(int prec, int backward, int n_layers, const float* X, int64_t ldx, int K0, int64_t M,
                             int64_t rows_full, const float* xaux, int64_t ldxaux, int xact, float* xout,
                             int64_t ldxout, const void* const* a_hi, const void* const* a_lo,
                             const float* const* bias, const float* const* aux, const int64_t* ldaux,
                             float* const* out, const int64_t* ldo, const int* N, const int* act, float beta,
                             float thr, const float* w2row0, float* tap_part, int64_t ld_tap, float* const* rinv,
                             unsigned* emax, const int* f16, void* stream) {
  const char* fn = "mms_mlp_chain";
  MMS_REQUIRE((prec >= 1 && prec <= 3) || prec == 5 || (prec == 6 && backward), fn,
              "prec must be 1 (bf16), 2 (split bf16x3), 3 (split activations), 5 (fp16, forward chains) or 6 (backward: "
              "split bf16x3 first layer, row-scaled fp16 after)");
  MMS_REQUIRE(n_layers == 3 || n_layers == 4, fn, "chains of 3 or 4 layers");
  MMS_REQUIRE(M >= 0 && K0 > 0, fn, "bad shape");
  if (M == 0) return 0;
  MMS_REQUIRE(X && a_hi && N && act && out && ldo, fn, "null pointer");
  MMS_REQUIRE(aligned16(X) && ldx % 4 == 0 && ldx >= K0, fn, "input rows must be 16-B aligned");
  MMS_REQUIRE(!backward || xaux == nullptr || (aligned16(xaux) && ldxaux % 4 == 0), fn, "xaux rows must be 16-B aligned");
  ChainArgs a;
  a.X = X; a.ldx = ldx; a.K0 = K0; a.M = M; a.rows_full = rows_full < 0 ? M : rows_full;
  a.xaux = backward ? xaux : nullptr; a.ldxaux = ldxaux; a.xact = xact;
  a.xout = backward ? xout : nullptr; a.ldxout = ldxout;
  a.beta = beta; a.thr = thr;
  a.w2row0 = backward ? nullptr : w2row0;
  a.tap_part = backward ? tap_part : nullptr;
  a.ld_tap = ld_tap;
  MMS_REQUIRE(tap_part == nullptr || !backward || (n_layers == 3 && act[0] == 2 && xaux == nullptr && N[0] <= 256 &&
                                                   ld_tap > N[0] && rows_full >= 0 && rows_full < M), fn,
              "the taps' weight-gradient partials (tap_part) are a feature of the SDF backward chain");
  MMS_REQUIRE(backward || rows_full >= M || w2row0 != nullptr, fn,
              "forward with single-output rows (rows_full < M) needs the last layer's fp32 weight row 0");
  MMS_REQUIRE(n_layers == 3 || rows_full < 0 || rows_full >= M, fn, "single-output rows are a 3-layer (SDF) feature");
  int nt[4] = {0, 0, 0, 0};
  for (int l = 0; l < 4; ++l) a.L[l] = ChainLayer{};
  for (int l = 0; l < n_layers; ++l) {
    MMS_REQUIRE(a_hi[l] != nullptr && N[l] > 0, fn, "missing layer weights");
    const bool split = prec == 2 || (prec == 6 && l == 0);
    MMS_REQUIRE(!split || (a_lo && a_lo[l] != nullptr), fn, "split bf16x3 needs the residual images");
    MMS_REQUIRE(act[l] >= 0 && act[l] <= 3, fn, "bad activation id");
    ChainLayer& L = a.L[l];
    L.a_hi = reinterpret_cast<const __bf16*>(a_hi[l]);
    L.a_lo = split ? reinterpret_cast<const __bf16*>(a_lo[l]) : nullptr;
    L.bias = (!backward && bias) ? bias[l] : nullptr;
    L.aux = (backward && aux) ? aux[l] : nullptr;
    L.ldaux = (backward && ldaux) ? ldaux[l] : 0;
    L.f16 = (f16 && f16[l]) ? 1 : 0;
    if (L.f16) {
      // fp16 hidden activations: the forward's stored rows, the backward's act' source
      MMS_REQUIRE(l < n_layers - 1 && (backward ? L.aux != nullptr : out[l] != nullptr), fn,
                  "fp16 rows (f16) are a hidden-layer feature: forward out / backward aux");
      const void* p = backward ? (const void*)L.aux : (const void*)out[l];
      const int64_t ld = backward ? L.ldaux : ldo[l];
      MMS_REQUIRE(((uintptr_t)p & 7) == 0 && ld % 4 == 0 && ld >= 32 * ((N[l] + 31) / 32),
                  fn, "fp16 rows must be 8-B aligned and hold whole 32-column tiles");
    }
    MMS_REQUIRE(L.aux == nullptr || L.f16 || (aligned16(L.aux) && L.ldaux % 4 == 0), fn, "aux rows must be 16-B aligned");
    L.out = out[l];
    L.ldo = ldo[l];
    L.rinv = rinv ? rinv[l] : nullptr;
    L.emax = L.rinv ? emax + l : nullptr;
    if (L.rinv != nullptr) {
      // fp16 dZ rows of a hidden layer (prec 6 backward): 8-B stores of whole 32-column tiles
      MMS_REQUIRE(prec == 6 && backward && l < n_layers - 1 && emax != nullptr, fn,
                  "fp16 dZ stores (rinv) are a prec-6 backward hidden-layer feature and need emax");
      MMS_REQUIRE(L.out != nullptr && ((uintptr_t)L.out & 7) == 0 && L.ldo % 4 == 0 && L.ldo >= 32 * ((N[l] + 31) / 32),
                  fn, "fp16 dZ rows must be 8-B aligned and hold whole 32-column tiles");
    }
    // a forward whose rows all take the single-output path (rows_full = 0, the sampler's SDF queries) stores only
    // column 0 of the last layer, one scalar per row: any pitch >= 1 (a dense [M] sdf vector with ldo = 1)
    const bool col0_only = !backward && l == n_layers - 1 && a.rows_full == 0;
    MMS_REQUIRE(L.out == nullptr || L.rinv != nullptr || (L.f16 && !backward) || (col0_only && L.ldo >= 1) ||
                    (aligned16(L.out) && L.ldo % 4 == 0 && L.ldo >= N[l]), fn, "output rows must be 16-B aligned");
    L.N = N[l];
    L.act = act[l];
    nt[l] = (N[l] + 31) / 32;
  }
  const int ks0 = (K0 + 15) / 16;
  hipStream_t s = mms::as_stream(stream);
  const bool ok = prec == 1   ? dispatch_chain<1>(n_layers, ks0, nt, backward != 0, a, s)
                  : prec == 2 ? dispatch_chain<2>(n_layers, ks0, nt, backward != 0, a, s)
                  : prec == 5 ? dispatch_chain<5>(n_layers, ks0, nt, backward != 0, a, s)
                  : prec == 6 ? dispatch_chain<6>(n_layers, ks0, nt, backward != 0, a, s)
                              : dispatch_chain<3>(n_layers, ks0, nt, backward != 0, a, s);
  MMS_REQUIRE(ok, fn, "unsupported chain shape or activations (SDF 71-256-256-257 Softplus, radiance 317-256-256-256 "
                      "ReLU, background 39-256x4 and 283-256-256-256-128 ReLU chains only)");
  return mms::check_launch(fn);
}
