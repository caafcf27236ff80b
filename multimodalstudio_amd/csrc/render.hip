// Per-ray volume-rendering kernels: one 64-lane wavefront per ray, lane = sample (S <= 64).
//
//   NeuS alpha      /root/reference/src/model_components/volume_rendering.py:185-213
//   NeuS weights    volume_rendering.py:177-183 (T = cumprod([1, 1 - a + 1e-7]), w = a T[:-1])
//   density alphas  /root/reference/src/cameras/rays.py:138-151 (a = 1 - exp(-delta sigma)) + rays.py:201-217
//   composite       /root/reference/src/model_components/renderers.py:75-174 (+ accumulation / depth / normals)
//
// Transmittance products are formed sequentially (same association as torch.cumprod on CPU) by
// broadcasting the running product across lanes with one shuffle per sample.
#include "common.h"

namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// exclusive sequential product: T_i = ((c_0 c_1) c_2 ...) c_{i-1}; returns T_i for this lane.
// Accumulated in double and rounded per output, as torch.cumprod does on CPU (acc_type<float> = double).
__device__ __forceinline__ float excl_cumprod_seq(float c, int lane, int S, float& total) {
  double run = 1.0;
  float mine = 1.0f;
  for (int j = 0; j < S; ++j) {
    if (lane == j) mine = (float)run;
    const float cj = __shfl(c, j);
    run = run * (double)cj;
  }
  total = (float)run;
  return mine;
}

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

struct AlphaIn {
  float sdf, g0, g1, g2, delta;
};

// ------------------------------------------------------------------ NeuS alpha + weights
__global__ __launch_bounds__(256) void neus_weights_fwd_kernel(const float* __restrict__ sdf, int64_t lds,
                                                               const float* __restrict__ grads,
                                                               const float* __restrict__ dirs,
                                                               const float* __restrict__ deltas,
                                                               const float* __restrict__ s_param, float cos_anneal,
                                                               int64_t R, int S, float* __restrict__ alpha_out,
                                                               float* __restrict__ weights) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  float s = expf(s_param[0] * 10.0f);
  s = fminf(fmaxf(s, 1e-6f), 1e6f);
  const float* d = dirs + ray * 3;
  float alpha = 0.f;
  const int64_t i = ray * S + lane;
  if (lane < S) {
    const float* g = grads + i * 3;
    float tc = d[0] * g[0];
    tc = tc + d[1] * g[1];
    tc = tc + d[2] * g[2];
    const float ic = -(fmaxf(-tc * 0.5f + 0.5f, 0.f) * (1.0f - cos_anneal) + fmaxf(-tc, 0.f) * cos_anneal);
    const float sd = sdf[i * lds];
    const float dl = deltas[i];
    const float nxt = sd + ic * dl * 0.5f;
    const float prv = sd - ic * dl * 0.5f;
    const float pc = sigm(prv * s), nc = sigm(nxt * s);
    alpha = (pc - nc + 1e-5f) / (pc + 1e-5f);
    alpha = fminf(fmaxf(alpha, 0.f), 1.f);
  }
  const float c = lane < S ? (1.0f - alpha + 1e-7f) : 1.0f;
  float tot;
  const float T = excl_cumprod_seq(c, lane, S, tot);
  if (lane < S) {
    alpha_out[i] = alpha;
    weights[i] = alpha * T;
  }
}

// backward: d sdf (written to dsdf[i * ldds]), d grads (+=), d dirs (+=), d deltas (+=), d s_param (atomic)
__global__ __launch_bounds__(256) void neus_weights_bwd_kernel(
    const float* __restrict__ sdf, int64_t lds, const float* __restrict__ grads, const float* __restrict__ dirs,
    const float* __restrict__ deltas, const float* __restrict__ s_param, float cos_anneal, int64_t R, int S,
    const float* __restrict__ alpha_in, const float* __restrict__ dweights, float* __restrict__ dsdf, int64_t ldds,
    float* __restrict__ dgrads, float* __restrict__ ddirs, float* __restrict__ ddeltas, float* __restrict__ ds_param) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const float e10 = expf(s_param[0] * 10.0f);
  const bool s_clipped = !(e10 >= 1e-6f && e10 <= 1e6f);
  const float s = fminf(fmaxf(e10, 1e-6f), 1e6f);
  const float* d = dirs + ray * 3;
  const int64_t i = ray * S + lane;
  const float alpha = lane < S ? alpha_in[i] : 0.f;
  const float c = lane < S ? (1.0f - alpha + 1e-7f) : 1.0f;
  float tot;
  const float T = excl_cumprod_seq(c, lane, S, tot);
  const float dw = lane < S ? dweights[i] : 0.f;
  // dT_i = dw_i * alpha_i ; dc_i = sum_{j>i} dT_j T_j / c_i
  const float q = dw * alpha * T;
  // suffix sum (exclusive) of q
  float incl = q;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_down(incl, o);
    if (lane + o < 64) incl += t;
  }
  const float excl_suffix = incl - q;
  const float dc = excl_suffix / c;
  float dalpha = dw * T - dc;
  float gd0 = 0.f, gd1 = 0.f, gd2 = 0.f, gs = 0.f;
  if (lane < S) {
    const float* g = grads + i * 3;
    float tc = d[0] * g[0];
    tc = tc + d[1] * g[1];
    tc = tc + d[2] * g[2];
    const float r1 = -tc * 0.5f + 0.5f, r2 = -tc;
    const float ic = -(fmaxf(r1, 0.f) * (1.0f - cos_anneal) + fmaxf(r2, 0.f) * cos_anneal);
    const float sd = sdf[i * lds];
    const float dl = deltas[i];
    const float nxt = sd + ic * dl * 0.5f;
    const float prv = sd - ic * dl * 0.5f;
    const float pc = sigm(prv * s), nc = sigm(nxt * s);
    const float u = pc - nc + 1e-5f, v = pc + 1e-5f;
    const float raw = u / v;
    if (!(raw >= 0.f && raw <= 1.f)) dalpha = 0.f;
    const float dpc = dalpha * (1.0f / v - u / (v * v));
    const float dnc = -dalpha / v;
    const float dprv_arg = dpc * pc * (1.0f - pc);
    const float dnxt_arg = dnc * nc * (1.0f - nc);
    const float dprv = dprv_arg * s, dnxt = dnxt_arg * s;
    gs = dprv_arg * prv + dnxt_arg * nxt;
    dsdf[i * ldds] = dprv + dnxt;
    const float dic = (dnxt - dprv) * dl * 0.5f;
    ddeltas[i] += (dnxt - dprv) * ic * 0.5f;
    const float dtc = (0.5f * (1.0f - cos_anneal) * (r1 > 0.f ? 1.f : 0.f) + cos_anneal * (r2 > 0.f ? 1.f : 0.f)) * dic;
    float* dg = dgrads + i * 3;
    dg[0] += dtc * d[0];
    dg[1] += dtc * d[1];
    dg[2] += dtc * d[2];
    gd0 = dtc * g[0];
    gd1 = dtc * g[1];
    gd2 = dtc * g[2];
  }
  gd0 = wave_sum(gd0);
  gd1 = wave_sum(gd1);
  gd2 = wave_sum(gd2);
  gs = wave_sum(gs);
  if (lane == 0) {
    if (ddirs) {
      ddirs[ray * 3] += gd0;
      ddirs[ray * 3 + 1] += gd1;
      ddirs[ray * 3 + 2] += gd2;
    }
    if (ds_param && !s_clipped) atomicAdd(ds_param, gs * 10.0f * e10);
  }
}

// ------------------------------------------------------------------ density -> alpha -> weights (background)
__global__ __launch_bounds__(256) void density_weights_fwd_kernel(const float* __restrict__ density, int64_t ldd,
                                                                  const float* __restrict__ deltas, int64_t R, int S,
                                                                  float* __restrict__ alpha_out,
                                                                  float* __restrict__ weights) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const int64_t i = ray * S + lane;
  float a = 0.f;
  if (lane < S) a = 1.0f - expf(-(deltas[i] * density[i * ldd]));
  const float c = lane < S ? (1.0f - a + 1e-7f) : 1.0f;
  float tot;
  const float T = excl_cumprod_seq(c, lane, S, tot);
  if (lane < S) {
    alpha_out[i] = a;
    weights[i] = a * T;
  }
}

__global__ __launch_bounds__(256) void density_weights_bwd_kernel(const float* __restrict__ density, int64_t ldd,
                                                                  const float* __restrict__ deltas, int64_t R, int S,
                                                                  const float* __restrict__ alpha_in,
                                                                  const float* __restrict__ dweights,
                                                                  float* __restrict__ ddensity, int64_t lddd,
                                                                  float* __restrict__ ddeltas) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const int64_t i = ray * S + lane;
  const float a = lane < S ? alpha_in[i] : 0.f;
  const float c = lane < S ? (1.0f - a + 1e-7f) : 1.0f;
  float tot;
  const float T = excl_cumprod_seq(c, lane, S, tot);
  const float dw = lane < S ? dweights[i] : 0.f;
  const float q = dw * a * T;
  float incl = q;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_down(incl, o);
    if (lane + o < 64) incl += t;
  }
  const float dc = (incl - q) / c;
  const float da = dw * T - dc;
  if (lane < S) {
    // a = 1 - exp(-x), x = delta * sigma -> da/dx = exp(-x)
    const float x = deltas[i] * density[i * ldd];
    const float dx = da * expf(-x);
    ddensity[i * lddd] = dx * deltas[i];
    if (ddeltas) ddeltas[i] += dx * density[i * ldd];
  }
}

// ------------------------------------------------------------------ composite
// out[n, :] = sum_s w c  (+ bg (1 - sum w) if bg != null); rows of a compacted ray set scatter to rows idx[r]
// of the full [N, C] output when idx != null.
__global__ __launch_bounds__(256) void composite_fwd_kernel(const float* __restrict__ w, const float* __restrict__ vals,
                                                            int64_t ldv, int C, const float* __restrict__ bg,
                                                            int64_t R, int S, const int64_t* __restrict__ idx,
                                                            int64_t nout, const unsigned char* __restrict__ hit,
                                                            unsigned cblocks, float* __restrict__ out) {
  if (blockIdx.x >= cblocks) {
    // the rows no ray of the batch lands on keep the background (instead of a copy of it made before the launch)
    const int64_t n = nout * C;
    for (int64_t e = (int64_t)(blockIdx.x - cblocks) * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)(gridDim.x - cblocks) * blockDim.x)
      if (!hit[e / C]) out[e] = bg[e];
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const int64_t orow = idx ? idx[ray] : ray;
  if (orow >= nout) return;   // a padding ray: discarded (wave-uniform)
  const int64_t i = ray * S + lane;
  const float wi = lane < S ? w[i] : 0.f;
  const float acc = wave_sum(wi);
  for (int c = 0; c < C; ++c) {
    const float v = lane < S ? wi * vals[i * ldv + c] : 0.f;
    const float sum = wave_sum(v);
    if (lane == 0) {
      float r = sum;
      if (bg) r = r + bg[orow * C + c] * (1.0f - acc);
      out[orow * C + c] = r;
    }
  }
}

// backward: dvals[i, c] = dout * w ; dw[i] += sum_c dout_c (vals_c - bg_c) ; dbg[orow] = dout (1 - acc)
__global__ __launch_bounds__(256) void composite_bwd_kernel(const float* __restrict__ w, const float* __restrict__ vals,
                                                            int64_t ldv, int C, const float* __restrict__ bg,
                                                            int64_t R, int S, const int64_t* __restrict__ idx,
                                                            int64_t nout, const unsigned char* __restrict__ hit,
                                                            unsigned cblocks, const float* __restrict__ dout,
                                                            float* __restrict__ dvals, int64_t lddv,
                                                            float* __restrict__ dw, float* __restrict__ dbg) {
  if (blockIdx.x >= cblocks) {
    // the background's pass-through gradient on the rows no ray of the batch lands on
    const int64_t n = nout * C;
    for (int64_t e = (int64_t)(blockIdx.x - cblocks) * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)(gridDim.x - cblocks) * blockDim.x)
      if (!hit[e / C]) dbg[e] = dout[e];
    return;
  }
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  const int64_t i = ray * S + lane;
  const float wi = lane < S ? w[i] : 0.f;
  const float acc = wave_sum(wi);
  const int64_t orow = idx ? idx[ray] : ray;
  const bool live = orow < nout;   // a padding ray (discarded in the forward): zero gradients
  float gw = 0.f;
  for (int c = 0; c < C; ++c) {
    const float g = live ? dout[orow * C + c] : 0.f;
    if (lane < S) {
      if (dvals) dvals[i * lddv + c] = g * wi;
      gw += g * vals[i * ldv + c];
      // (a padding ray's orow is nout, one row past bg: no read -- its gradients are zero)
      if (bg && live) gw -= g * bg[orow * C + c];
    }
    if (lane == 0 && bg && dbg && live) dbg[orow * C + c] = g * (1.0f - acc);  // hit rows: overwrite the pass-through dout
  }
  if (lane < S && dw) dw[i] = gw;  // every weight of the ray is written (no accumulation: dw needs no zero fill)
}

// ------------------------------------------------------------------ render statistics (no grad)
// Accumulation / normals / depth renderers (renderers.py:176-242) for compacted rays scattered to rows idx[r]:
// acc = sum_s w, nrm = sum_s w n, dep = sum_s w (start + end) / 2, and the depth's clip range: the min / max of all
// sample midpoints (torch.clip(depth, steps.min(), steps.max()), renderers.py:205-214) reduced into range[2] by
// atomics (order-independent: min / max are exact) as range = (max(-mid), max(mid)), each kept as the order-preserving
// unsigned image of the float (ord_f32), so a zeroed range (the step's zero arena, no fill launch) is below every
// value; range must hold zeros before the launch.
__device__ __forceinline__ unsigned ord_f32(float x) {
  const unsigned u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(unsigned u) {
  if (u == 0u) return -INFINITY;   // nothing reduced: as the -inf the float form started from
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__global__ __launch_bounds__(256) void render_stats_kernel(const float* __restrict__ w, const float* __restrict__ nrm,
                                                           const float* __restrict__ starts,
                                                           const float* __restrict__ ends, int64_t R, int S,
                                                           const int64_t* __restrict__ idx, float* __restrict__ out,
                                                           int64_t ldo, float* __restrict__ range) {
  // a wave per ray, grid-stride over rays; the midpoint range is reduced per wave, then per block in LDS, then one
  // atomic pair per block (a pair per ray serialised ~1700 same-address atomics: 50 us)
  __shared__ float sl[4], sh[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float lo = INFINITY, hi = -INFINITY;
  for (int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; ray < R;
       ray += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t i = ray * S + lane;
    const bool on = lane < S;
    const float wi = on ? w[i] : 0.f;
    const float mid = on ? (starts[i] + ends[i]) / 2.0f : 0.f;
    const float acc = wave_sum(wi);
    const float n0 = wave_sum(on ? wi * nrm[i * 3] : 0.f);
    const float n1 = wave_sum(on ? wi * nrm[i * 3 + 1] : 0.f);
    const float n2 = wave_sum(on ? wi * nrm[i * 3 + 2] : 0.f);
    const float dep = wave_sum(on ? wi * mid : 0.f);
    if (on) { lo = fminf(lo, mid); hi = fmaxf(hi, mid); }
    if (lane == 0) {
      float* o = out + (idx ? idx[ray] : ray) * ldo;
      o[0] = acc; o[1] = n0; o[2] = n1; o[3] = n2; o[4] = dep;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o));
    hi = fmaxf(hi, __shfl_xor(hi, o));
  }
  if (lane == 0) { sl[wave] = lo; sh[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    lo = fminf(fminf(sl[0], sl[1]), fminf(sl[2], sl[3]));
    hi = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
    if (lo <= hi) {
      atomicMax(reinterpret_cast<unsigned*>(range), ord_f32(-lo));
      atomicMax(reinterpret_cast<unsigned*>(range) + 1, ord_f32(hi));
    }
  }
}

// depth of the hit rows clipped to the midpoint range (rows not written by render_stats_kernel stay 0)
__global__ void render_clip_kernel(int64_t R, const int64_t* __restrict__ idx, float* __restrict__ out, int64_t ldo,
                                   const float* __restrict__ range) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float* d = out + (idx ? idx[r] : r) * ldo + 4;
  const unsigned* ur = reinterpret_cast<const unsigned*>(range);
  d[0] = fminf(fmaxf(d[0], -unord_f32(ur[0])), unord_f32(ur[1]));
}

// Every modality's statistics in one launch pair: segment m (blockIdx.y) holds the rays [off[m], off[m + 1]) of the
// batched hit set; its rows scatter to out rows m * seg_rows + sidx[r] and its depth clips to its own midpoint range
// (range + 2 m), as one DepthRenderer call per modality does (renderers.py:205-214).
constexpr int kMaxSeg = 8;
struct SegOff {
  int64_t off[kMaxSeg + 1];
};

__global__ __launch_bounds__(256) void render_stats_seg_kernel(const float* __restrict__ w,
                                                               const float* __restrict__ nrm,
                                                               const float* __restrict__ starts,
                                                               const float* __restrict__ ends, SegOff so, int S,
                                                               const int64_t* __restrict__ sidx,
                                                               float* __restrict__ out, int64_t ldo, int64_t seg_rows,
                                                               float* __restrict__ range) {
  __shared__ float sl[4], sh[4];
  const int seg = blockIdx.y;
  const int64_t r0 = so.off[seg], r1 = so.off[seg + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* o_seg = out + seg * seg_rows * ldo;
  float lo = INFINITY, hi = -INFINITY;
  for (int64_t ray = r0 + (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); ray < r1;
       ray += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t i = ray * S + lane;
    const bool on = lane < S;
    const float wi = on ? w[i] : 0.f;
    const float mid = on ? (starts[i] + ends[i]) / 2.0f : 0.f;
    const float acc = wave_sum(wi);
    const float n0 = wave_sum(on ? wi * nrm[i * 3] : 0.f);
    const float n1 = wave_sum(on ? wi * nrm[i * 3 + 1] : 0.f);
    const float n2 = wave_sum(on ? wi * nrm[i * 3 + 2] : 0.f);
    const float dep = wave_sum(on ? wi * mid : 0.f);
    if (on) { lo = fminf(lo, mid); hi = fmaxf(hi, mid); }
    if (lane == 0) {
      float* o = o_seg + sidx[ray] * ldo;
      o[0] = acc; o[1] = n0; o[2] = n1; o[3] = n2; o[4] = dep;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o));
    hi = fmaxf(hi, __shfl_xor(hi, o));
  }
  if (lane == 0) { sl[wave] = lo; sh[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    lo = fminf(fminf(sl[0], sl[1]), fminf(sl[2], sl[3]));
    hi = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
    if (lo <= hi) {
      atomicMax(reinterpret_cast<unsigned*>(range) + 2 * seg, ord_f32(-lo));
      atomicMax(reinterpret_cast<unsigned*>(range) + 2 * seg + 1, ord_f32(hi));
    }
  }
}

__global__ void render_clip_seg_kernel(SegOff so, const int64_t* __restrict__ sidx, float* __restrict__ out,
                                       int64_t ldo, int64_t seg_rows, const float* __restrict__ range) {
  const int seg = blockIdx.y;
  const int64_t r = so.off[seg] + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= so.off[seg + 1]) return;
  float* d = out + (seg * seg_rows + sidx[r]) * ldo + 4;
  const unsigned* ur = reinterpret_cast<const unsigned*>(range);
  d[0] = fminf(fmaxf(d[0], -unord_f32(ur[2 * seg])), unord_f32(ur[2 * seg + 1]));
}

}  // namespace

MMS_EXPORT int mms_render_stats_segments(const float* w, const float* normals, const float* starts, const float* ends,
                                         int n_seg, const int64_t* seg_off, int S, const int64_t* sidx, float* out,
                                         int64_t ldo, int64_t seg_rows, float* range, void* stream) {
  const char* fn = "mms_render_stats_segments";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  MMS_REQUIRE(ldo >= 5, fn, "output rows hold (acc, n0, n1, n2, depth)");
  MMS_REQUIRE(n_seg >= 1 && n_seg <= kMaxSeg, fn, "segment count must be in [1, 8]");
  MMS_REQUIRE(seg_off, fn, "null pointer");
  SegOff so{};
  int64_t most = 0;
  for (int m = 0; m <= n_seg; ++m) so.off[m] = seg_off[m];
  for (int m = 0; m < n_seg; ++m) {
    MMS_REQUIRE(so.off[m + 1] >= so.off[m], fn, "segment offsets must be non-decreasing");
    most = so.off[m + 1] - so.off[m] > most ? so.off[m + 1] - so.off[m] : most;
  }
  if (most == 0) return 0;   // no hit ray in any segment
  MMS_REQUIRE(sidx && out && range, fn, "null pointer");
  hipStream_t s = mms::as_stream(stream);
  hipLaunchKernelGGL(render_stats_seg_kernel, dim3(mms::grid_for(most * 64, 256, 256), n_seg), dim3(256), 0, s, w,
                     normals, starts, ends, so, S, sidx, out, ldo, seg_rows, range);
  hipLaunchKernelGGL(render_clip_seg_kernel, dim3(mms::grid_for(most, 256, INT32_MAX), n_seg), dim3(256), 0, s, so,
                     sidx, out, ldo, seg_rows, range);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_neus_weights_fwd(const float* sdf, int64_t lds, const float* grads, const float* dirs,
                                    const float* deltas, const float* s_param, float cos_anneal, int64_t R, int S,
                                    float* alpha, float* weights, void* stream) {
  const char* fn = "mms_neus_weights_fwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  hipLaunchKernelGGL(neus_weights_fwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), sdf, lds, grads, dirs, deltas, s_param, cos_anneal, R, S, alpha, weights);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_neus_weights_bwd(const float* sdf, int64_t lds, const float* grads, const float* dirs,
                                    const float* deltas, const float* s_param, float cos_anneal, int64_t R, int S,
                                    const float* alpha, const float* dweights, float* dsdf, int64_t ldds,
                                    float* dgrads, float* ddirs, float* ddeltas, float* ds_param, void* stream) {
  const char* fn = "mms_neus_weights_bwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  hipLaunchKernelGGL(neus_weights_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), sdf, lds, grads, dirs, deltas, s_param, cos_anneal, R, S, alpha, dweights,
                     dsdf, ldds, dgrads, ddirs, ddeltas, ds_param);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_density_weights_fwd(const float* density, int64_t ldd, const float* deltas, int64_t R, int S,
                                       float* alpha, float* weights, void* stream) {
  const char* fn = "mms_density_weights_fwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  hipLaunchKernelGGL(density_weights_fwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), density, ldd, deltas, R, S, alpha, weights);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_density_weights_bwd(const float* density, int64_t ldd, const float* deltas, int64_t R, int S,
                                       const float* alpha, const float* dweights, float* ddensity, int64_t lddd,
                                       float* ddeltas, void* stream) {
  const char* fn = "mms_density_weights_bwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  hipLaunchKernelGGL(density_weights_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), density, ldd, deltas, R, S, alpha, dweights, ddensity, lddd, ddeltas);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_composite_fwd(const float* w, const float* vals, int64_t ldv, int C, const float* bg, int64_t R,
                                 int S, const int64_t* idx, int64_t nout, const unsigned char* hit, float* out,
                                 void* stream) {
  const char* fn = "mms_composite_fwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  MMS_REQUIRE(hit == nullptr || (bg != nullptr && idx != nullptr), fn, "hit rows need a background and a scatter index");
  const unsigned cb = R > 0 ? mms::grid_for(R * 64, 256, INT32_MAX) : 0;
  const unsigned pb = hit != nullptr && nout > 0 ? mms::grid_for(nout * C, 256, 4096) : 0;
  if (cb + pb == 0) return 0;
  hipLaunchKernelGGL(composite_fwd_kernel, dim3(cb + pb), dim3(256), 0, mms::as_stream(stream), w, vals, ldv, C, bg, R,
                     S, idx, nout, hit, cb, out);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_render_stats(const float* w, const float* normals, const float* starts, const float* ends,
                                int64_t R, int S, const int64_t* idx, float* out, int64_t ldo, float* range,
                                void* stream) {
  const char* fn = "mms_render_stats";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  MMS_REQUIRE(ldo >= 5, fn, "output rows hold (acc, n0, n1, n2, depth)");
  if (R == 0) return 0;
  hipStream_t s = mms::as_stream(stream);
  hipLaunchKernelGGL(render_stats_kernel, dim3(mms::grid_for(R * 64, 256, 256)), dim3(256), 0, s, w, normals,
                     starts, ends, R, S, idx, out, ldo, range);
  hipLaunchKernelGGL(render_clip_kernel, dim3(mms::grid_for(R, 256, INT32_MAX)), dim3(256), 0, s, R, idx, out, ldo,
                     range);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_composite_bwd(const float* w, const float* vals, int64_t ldv, int C, const float* bg, int64_t R,
                                 int S, const int64_t* idx, int64_t nout, const unsigned char* hit, const float* dout,
                                 float* dvals, int64_t lddv, float* dw, float* dbg, void* stream) {
  const char* fn = "mms_composite_bwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  MMS_REQUIRE(hit == nullptr || (bg != nullptr && idx != nullptr), fn, "hit rows need a background and a scatter index");
  const unsigned cb = R > 0 ? mms::grid_for(R * 64, 256, INT32_MAX) : 0;
  const unsigned pb = hit != nullptr && dbg != nullptr && nout > 0 ? mms::grid_for(nout * C, 256, 4096) : 0;
  if (cb + pb == 0) return 0;
  hipLaunchKernelGGL(composite_bwd_kernel, dim3(cb + pb), dim3(256), 0, mms::as_stream(stream), w, vals, ldv, C, bg, R,
                     S, idx, nout, hit, cb, dout, dvals, lddv, dw, dbg);
  return mms::check_launch(fn);
}
