// Multi-resolution hash-grid encoding (Instant-NGP style) for gfx950.
//
// Semantics follow the reference's torch path (the tcnn path is not pinnable here):
//   FeatureGrid.forward                 /root/reference/src/field_components/feature_structures.py:78-83
//     x_hat = (x + r) / (2 r), features *= coarse-to-fine mask (levels >= active zeroed, :85-88)
//   HashEncoding.hash_fn / pytorch_fwd   /root/reference/src/field_components/encodings.py:244-304
//     scaled = x_hat * floor(min_res * g^l); corners from ceil/floor; ceil corner weight = frac;
//     index = (c0 * 1 ^ c1 * 2654435761 ^ c2 * 805459861) mod 2^log2T + l * 2^log2T;
//     lerp x, then y, then z; output level-major [l0f0, l0f1, l1f0, ...].
//
// Layout: table [L * T, 2] f32 (one float2 per entry), positions [M, ldx] f32 (first 3 columns),
// output [M, ldo] f32 written at columns 0 .. 2L-1 (ldo lets the caller write straight into the
// MLP input panel).  One thread per (point, level); 16 consecutive lanes cover one point's levels
// so each wave writes 4 contiguous 128-byte output rows.
#include "common.h"
#include "sh.h"

// Bit-exact corner selection needs the rounded product x_hat * s before floor/frac (a fused
// multiply-subtract would change the fractional weights), so contraction is off in this file; the
// kernels are gather-bound, the extra VALU is free.
#pragma clang fp contract(off)

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kMaxLevels = 16;
constexpr uint32_t kP1 = 2654435761u;
constexpr uint32_t kP2 = 805459861u;

struct GridParams {
  float scale[kMaxLevels];
  int levels;         // L
  int active_levels;  // coarse-to-fine: levels >= active contribute 0
  int log2T;
  float inv_2r;       // 1 / (2 r)
  float radius;       // r
  int smooth;         // interpolation "Smoothstep" (tcnn): weights S(t) = t^2 (3 - 2 t) of the fraction t
};

__device__ __forceinline__ float smoothstep(float t) { return t * t * (3.0f - 2.0f * t); }
__device__ __forceinline__ float smoothstep_grad(float t) { return 6.0f * t * (1.0f - t); }

__device__ __forceinline__ uint32_t hash3(int cx, int cy, int cz, uint32_t mask) {
  return (((uint32_t)cx) ^ ((uint32_t)cy * kP1) ^ ((uint32_t)cz * kP2)) & mask;
}

struct Corners {
  uint32_t idx[8];  // reference order f_0..f_7
  float ox, oy, oz;
};

// Corner order (encodings.py:274-281): 0:(c,c,c) 1:(c,f,c) 2:(f,f,c) 3:(f,c,c)
//                                      4:(c,c,f) 5:(c,f,f) 6:(f,f,f) 7:(f,c,f)
__device__ __forceinline__ Corners make_corners(float x, float y, float z, float radius, float inv_2r,
                                                float s, int level, int log2T, bool smooth) {
  Corners c;
  // (x + r) / (2r): reference computes a true division by (2r); for r in {1, 2} the reciprocal
  // multiply is exact, but keep the division for bit-exact corner indices in general.
  // radius 0: the input is already x_hat (HashEncoding called directly, encodings.py:263-304)
  const float two_r = 2.0f * radius;
  const bool norm = radius > 0.f;
  const float hx = norm ? (x + radius) / two_r : x;
  const float hy = norm ? (y + radius) / two_r : y;
  const float hz = norm ? (z + radius) / two_r : z;
  (void)inv_2r;
  const float sx = hx * s, sy = hy * s, sz = hz * s;
  const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
  const int cxc = (int)ceilf(sx), cyc = (int)ceilf(sy), czc = (int)ceilf(sz);
  const int cxf = (int)fx, cyf = (int)fy, czf = (int)fz;
  c.ox = sx - fx;
  c.oy = sy - fy;
  c.oz = sz - fz;
  if (smooth) {  // the ceil corner's weight S(frac), the floor corner's 1 - S(frac)
    c.ox = smoothstep(c.ox);
    c.oy = smoothstep(c.oy);
    c.oz = smoothstep(c.oz);
  }
  const uint32_t mask = (1u << log2T) - 1u;
  const uint32_t base = (uint32_t)level << log2T;
  c.idx[0] = base + hash3(cxc, cyc, czc, mask);
  c.idx[1] = base + hash3(cxc, cyf, czc, mask);
  c.idx[2] = base + hash3(cxf, cyf, czc, mask);
  c.idx[3] = base + hash3(cxf, cyc, czc, mask);
  c.idx[4] = base + hash3(cxc, cyc, czf, mask);
  c.idx[5] = base + hash3(cxc, cyf, czf, mask);
  c.idx[6] = base + hash3(cxf, cyf, czf, mask);
  c.idx[7] = base + hash3(cxf, cyc, czf, mask);
  return c;
}

// Block order in XCD-contiguous chunks: the dispatcher sends block b to XCD b % 8, so consecutive blocks -- whose
// points are consecutive samples of the same rays, sharing their coarse cells -- would fetch the same table lines
// into eight different L2s; block b instead takes position k = b / 8 of XCD (b % 8)'s contiguous chunk of the grid.
// MMS_HASH_XCD=0 restores the plain order (diagnostic builds).
#ifndef MMS_HASH_XCD
#define MMS_HASH_XCD 1
#endif
__device__ __forceinline__ int64_t xcd_block() {
#if MMS_HASH_XCD
  const int64_t nb = gridDim.x, b = blockIdx.x;
  const int64_t q = nb >> 3, r = nb & 7, x = b & 7, k = b >> 3;
  return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
#else
  return blockIdx.x;
#endif
}

// G > 1 (the SDF panel: centre rows g, tap rows g + j * gstride, j < G): the lanes walk the points in (g, j) order, so
// the centre and the 4 taps of one sample -- which share their cells at every level coarser than the tap offset --
// and the next samples of the same ray are gathered by the same wave: their corner lines are fetched from MALL / HBM
// into one L2 once instead of by five waves on (under round-robin dispatch) five different XCDs.
template <bool ALIGNED, int G>
__global__ __launch_bounds__(256) void hashgrid_fwd_kernel(const float* __restrict__ pos, int64_t Mg,
                                                           int64_t gstride, int64_t ldx,
                                                           const float2* __restrict__ table, GridParams p,
                                                           float* __restrict__ out, int64_t ldo) {
  const int64_t tid = xcd_block() * blockDim.x + threadIdx.x;
  const int64_t q = tid >> 4;
  const int level = (int)(tid & 15);
  const int64_t g = G == 1 ? q : q / G;
  const int64_t pt = G == 1 ? q : g + (q - g * G) * gstride;
  if (g >= Mg || level >= p.levels) return;
  float2 r = make_float2(0.f, 0.f);
  if (level < p.active_levels) {
    const float* xp = pos + pt * ldx;
    Corners c = make_corners(xp[0], xp[1], xp[2], p.radius, p.inv_2r, p.scale[level], level, p.log2T, p.smooth != 0);
    float2 f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = table[c.idx[i]];
    const float ox = c.ox, oy = c.oy, oz = c.oz;
    const float nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
    float2 f03, f12, f56, f47, f0312, f4756;
    f03.x = f[0].x * ox + f[3].x * nx;  f03.y = f[0].y * ox + f[3].y * nx;
    f12.x = f[1].x * ox + f[2].x * nx;  f12.y = f[1].y * ox + f[2].y * nx;
    f56.x = f[5].x * ox + f[6].x * nx;  f56.y = f[5].y * ox + f[6].y * nx;
    f47.x = f[4].x * ox + f[7].x * nx;  f47.y = f[4].y * ox + f[7].y * nx;
    f0312.x = f03.x * oy + f12.x * ny;  f0312.y = f03.y * oy + f12.y * ny;
    f4756.x = f47.x * oy + f56.x * ny;  f4756.y = f47.y * oy + f56.y * ny;
    r.x = f0312.x * oz + f4756.x * nz;
    r.y = f0312.y * oz + f4756.y * nz;
  }
  float* o = out + pt * ldo + 2 * level;
  if (ALIGNED) {
    *reinterpret_cast<float2*>(o) = r;  // 8-B aligned: one dwordx2 store
  } else {
    o[0] = r.x;  // panels with the grid at an odd column (SDF panel col 39): two dword stores
    o[1] = r.y;
  }
}

// The SDF field's whole MLP input panel in one launch (SDFField.forward, surface_field.py:99-116; FeatureGridAndMLP,
// feature_structures.py:153-169): per point the position x (centre, or centre + k_t delta for tap t,
// surface_model.py:137-153), its positional encoding (encodings.py:161-182: sin(x_i 2^k), then sin(x_i 2^k + pi/2))
// and its hash-grid features, in one row [x(3) | PE(6F) | grid(2L)].  Same values as mms_geo_input_fwd followed by
// mms_hashgrid_fwd_grouped (the tap offsets are +-delta exactly, the PE the same sinf expressions), but each point's
// row is written whole by one 16-lane group (x / PE columns lane, lane + 16, lane + 32; the level's 2 features) instead
// of in two launches writing 156-B and 128-B parts of every 288-B row.  G = 5: points in (sample, tap) order as the
// grouped gather; G = 1: the sampler's inference batches.
__constant__ float kTapH[4][3] = {{1.f, -1.f, -1.f}, {-1.f, -1.f, 1.f}, {-1.f, 1.f, -1.f}, {1.f, 1.f, 1.f}};
constexpr float kHalfPiH = 1.57079632679489661923f;  // fl32(pi / 2)

// RAYS (the NeuS sampler's inference batches, G = 1): point q is the start of sample k = q % S of ray r = q / S of
// the spacing bins [R, S + 1] (ldb), o_r + d_r * (f_r b + n_r (1 - b)) -- SamplesFunction's positions
// (mms_samples_fwd, uniform spacing: sampler.hip to_euclid kind 0; contraction off in both files, same bits) -- so
// the sampler's position launch before every panel is gone.
struct RaySrc {
  const float* bins;
  int64_t ldb;
  int nb;
  const float* nears;
  const float* fars;
  const float* origins;
  const float* dirs;
};

template <int G, bool RAYS = false>
__global__ __launch_bounds__(256) void sdf_panel_fwd_kernel(const float* __restrict__ cpos, int64_t ldp, int64_t Mg,
                                                            float delta, int F, const float2* __restrict__ table,
                                                            GridParams p, float* __restrict__ X, int64_t ldx,
                                                            RaySrc rs) {
  const int64_t tid = xcd_block() * blockDim.x + threadIdx.x;
  const int64_t q = tid >> 4;
  const int l16 = (int)(tid & 15);
  const int64_t g = G == 1 ? q : q / G;
  const int t = G == 1 ? 0 : (int)(q - g * G);
  const int64_t pt = G == 1 ? q : g + t * Mg;
  if (g >= Mg) return;
  float x[3];
  if constexpr (RAYS) {
    const int S = rs.nb - 1;
    const int64_t r = q / S;
    const int k = (int)(q - r * S);
    const float nr = rs.nears[r], fr = rs.fars[r];
    const float b = rs.bins[r * rs.ldb + k];
    const float s0 = fr * b + nr * (1 - b);
#pragma unroll
    for (int c = 0; c < 3; ++c) x[c] = rs.origins[r * 3 + c] + rs.dirs[r * 3 + c] * s0;
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      x[c] = cpos[g * ldp + c];
      if (t > 0) x[c] = x[c] + kTapH[t - 1][c] * delta;
    }
  }
  float* row = X + pt * ldx;
  const int W = 3 + 6 * F;
  for (int c = l16; c < W; c += 16) {
    int coord = c, k = 0;
    bool cosine = false;
    if (c >= 3 && c < 3 + 3 * F) {
      coord = (c - 3) / F;
      k = (c - 3) - coord * F;
    } else if (c >= 3 + 3 * F) {
      coord = (c - 3 - 3 * F) / F;
      k = (c - 3 - 3 * F) - coord * F;
      cosine = true;
    }
    const float xc = coord == 0 ? x[0] : (coord == 1 ? x[1] : x[2]);
    float v = xc;
    if (c >= 3) {
      const float sc = xc * (float)(1 << k);
      v = cosine ? sinf(sc + kHalfPiH) : sinf(sc);
    }
    row[c] = v;
  }
  const int level = l16;
  if (level >= p.levels) return;
  float2 r = make_float2(0.f, 0.f);
  if (level < p.active_levels) {
    Corners c = make_corners(x[0], x[1], x[2], p.radius, p.inv_2r, p.scale[level], level, p.log2T, p.smooth != 0);
    float2 f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = table[c.idx[i]];
    const float ox = c.ox, oy = c.oy, oz = c.oz;
    const float nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
    float2 f03, f12, f56, f47, f0312, f4756;
    f03.x = f[0].x * ox + f[3].x * nx;  f03.y = f[0].y * ox + f[3].y * nx;
    f12.x = f[1].x * ox + f[2].x * nx;  f12.y = f[1].y * ox + f[2].y * nx;
    f56.x = f[5].x * ox + f[6].x * nx;  f56.y = f[5].y * ox + f[6].y * nx;
    f47.x = f[4].x * ox + f[7].x * nx;  f47.y = f[4].y * ox + f[7].y * nx;
    f0312.x = f03.x * oy + f12.x * ny;  f0312.y = f03.y * oy + f12.y * ny;
    f4756.x = f47.x * oy + f56.x * ny;  f4756.y = f47.y * oy + f56.y * ny;
    r.x = f0312.x * oz + f4756.x * nz;
    r.y = f0312.y * oz + f4756.y * nz;
  }
  row[W + 2 * level] = r.x;
  row[W + 2 * level + 1] = r.y;
}

// The radiance field's MLP input panel in one launch (RadianceField.forward, radiance_field.py:72-77, with
// FeatureGridAndMLP, feature_structures.py:153-169): rows [x(3) | SH(25) of the ray direction | geo feature(G) | n.v |
// hash grid(2L)] -- the values mms_rad_input_fwd followed by mms_hashgrid_fwd_grouped write (bit for bit), each point's
// row written by one 16-lane group: x and SH columns by lane, geo columns lane + 16 j, n.v by lane 0, level lane's two
// grid features.
__global__ __launch_bounds__(256) void rad_panel_fwd_kernel(const float* __restrict__ pos, int64_t ldp,
                                                            const float* __restrict__ dirs,
                                                            const float* __restrict__ normals,
                                                            const float* __restrict__ geo, int64_t ldg, int64_t M,
                                                            int S, int G, const float2* __restrict__ table,
                                                            GridParams p, float* __restrict__ X, int64_t ldx) {
  const int64_t tid = xcd_block() * blockDim.x + threadIdx.x;
  const int64_t i = tid >> 4;
  const int l16 = (int)(tid & 15);
  if (i >= M) return;
  float* row = X + i * ldx;
  const float* d = dirs + (i / S) * 3;
  const float x0 = pos[i * ldp], x1 = pos[i * ldp + 1], x2 = pos[i * ldp + 2];
  if (l16 < 3) row[l16] = l16 == 0 ? x0 : (l16 == 1 ? x1 : x2);
  {
    float sh[25];
    sh25(d[0], d[1], d[2], sh);
#pragma unroll
    for (int k = 0; k < 25; ++k)
      if ((k & 15) == l16) row[3 + k] = sh[k];
  }
  const float* gr = geo + i * ldg;
  for (int k = l16; k < G; k += 16) row[28 + k] = gr[k];
  if (l16 == 0) row[28 + G] = ndv3(normals + i * 3, d);
  const int level = l16;
  if (level >= p.levels) return;
  float2 r = make_float2(0.f, 0.f);
  if (level < p.active_levels) {
    Corners c = make_corners(x0, x1, x2, p.radius, p.inv_2r, p.scale[level], level, p.log2T, p.smooth != 0);
    float2 f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = table[c.idx[k]];
    const float ox = c.ox, oy = c.oy, oz = c.oz;
    const float nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
    float2 f03, f12, f56, f47, f0312, f4756;
    f03.x = f[0].x * ox + f[3].x * nx;  f03.y = f[0].y * ox + f[3].y * nx;
    f12.x = f[1].x * ox + f[2].x * nx;  f12.y = f[1].y * ox + f[2].y * nx;
    f56.x = f[5].x * ox + f[6].x * nx;  f56.y = f[5].y * ox + f[6].y * nx;
    f47.x = f[4].x * ox + f[7].x * nx;  f47.y = f[4].y * ox + f[7].y * nx;
    f0312.x = f03.x * oy + f12.x * ny;  f0312.y = f03.y * oy + f12.y * ny;
    f4756.x = f47.x * oy + f56.x * ny;  f4756.y = f47.y * oy + f56.y * ny;
    r.x = f0312.x * oz + f4756.x * nz;
    r.y = f0312.y * oz + f4756.y * nz;
  }
  row[29 + G + 2 * level] = r.x;
  row[29 + G + 2 * level + 1] = r.y;
}

// The same panel rows staged through LDS: a block's 16 points' rows [x | SH | geo | n.v | grid] are assembled in LDS
// (the geo columns read block-wide, consecutive threads on consecutive floats of the 16 rows) and written out
// block-wide in row-major order, so every wave-store covers 256 contiguous bytes of a row instead of four 64-B pieces
// of four rows.  Same values, bit for bit.
constexpr int kRadPts = 16;
constexpr int kRadCols = 29 + 256 + 2 * kMaxLevels;   // the widest row: G = 256
__global__ __launch_bounds__(256) void rad_panel_fwd_staged_kernel(const float* __restrict__ pos, int64_t ldp,
                                                                   const float* __restrict__ dirs,
                                                                   const float* __restrict__ normals,
                                                                   const float* __restrict__ geo, int64_t ldg,
                                                                   int64_t M, int S, int G,
                                                                   const float2* __restrict__ table, GridParams p,
                                                                   float* __restrict__ X, int64_t ldx) {
  __shared__ float srow[kRadPts * kRadCols];
  const int t = threadIdx.x;
  const int64_t i0 = xcd_block() * (int64_t)kRadPts;
  const int np = (int)((M - i0) < kRadPts ? (M - i0) : kRadPts);
  const int C = 29 + G + 2 * p.levels;
  // geo columns: block-wide coalesced reads of the np rows
  for (int e = t; e < np * G; e += 256) {
    const int r = e / G, c = e - r * G;
    srow[r * C + 28 + c] = geo[(i0 + r) * ldg + c];
  }
  const int pi = t >> 4;
  const int l16 = t & 15;
  if (pi < np) {
    const int64_t i = i0 + pi;
    float* row = srow + pi * C;
    const float* d = dirs + (i / S) * 3;
    const float x0 = pos[i * ldp], x1 = pos[i * ldp + 1], x2 = pos[i * ldp + 2];
    if (l16 < 3) row[l16] = l16 == 0 ? x0 : (l16 == 1 ? x1 : x2);
    {
      float sh[25];
      sh25(d[0], d[1], d[2], sh);
#pragma unroll
      for (int k = 0; k < 25; ++k)
        if ((k & 15) == l16) row[3 + k] = sh[k];
    }
    if (l16 == 0) row[28 + G] = ndv3(normals + i * 3, d);
    const int level = l16;
    if (level < p.levels) {
      float2 r = make_float2(0.f, 0.f);
      if (level < p.active_levels) {
        Corners c = make_corners(x0, x1, x2, p.radius, p.inv_2r, p.scale[level], level, p.log2T, p.smooth != 0);
        float2 f[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = table[c.idx[k]];
        const float ox = c.ox, oy = c.oy, oz = c.oz;
        const float nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
        float2 f03, f12, f56, f47, f0312, f4756;
        f03.x = f[0].x * ox + f[3].x * nx;  f03.y = f[0].y * ox + f[3].y * nx;
        f12.x = f[1].x * ox + f[2].x * nx;  f12.y = f[1].y * ox + f[2].y * nx;
        f56.x = f[5].x * ox + f[6].x * nx;  f56.y = f[5].y * ox + f[6].y * nx;
        f47.x = f[4].x * ox + f[7].x * nx;  f47.y = f[4].y * ox + f[7].y * nx;
        f0312.x = f03.x * oy + f12.x * ny;  f0312.y = f03.y * oy + f12.y * ny;
        f4756.x = f47.x * oy + f56.x * ny;  f4756.y = f47.y * oy + f56.y * ny;
        r.x = f0312.x * oz + f4756.x * nz;
        r.y = f0312.y * oz + f4756.y * nz;
      }
      row[29 + G + 2 * level] = r.x;
      row[29 + G + 2 * level + 1] = r.y;
    }
  }
  __syncthreads();
  // row-major write-out: thread t walks element t, t + 256, ... of the np rows (C > 256: at most one row step each)
  int r = t / C, c = t - (t / C) * C;
  for (int e = t; e < np * C; e += 256) {
    X[(i0 + r) * ldx + c] = srow[e];
    c += 256;
    while (c >= C) { c -= C; ++r; }
  }
}

// DPP lane moves (gfx9 encodings): quad_perm [1,0,3,2] / [2,3,0,1], row_ror:4 / :8 (rotation inside a 16-lane row),
// row_bcast:15 / :31 (lane 15 / 31 of a row into the next row(s), masked by ROWS).  Rows not in ROWS read 0.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, false));
}

// sum over the wave's 64 lanes, complete in lane 63: each 16-lane row by rotations and quad swaps (VALU, no LDS
// permutes), then row 0 + row 1 and row 2 + row 3 by row_bcast:15, the halves by row_bcast:31
__device__ __forceinline__ float wave_sum_to_63(float v) {
  v += dpp<0x128>(v);  // row_ror:8
  v += dpp<0x124>(v);  // row_ror:4
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v += dpp<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

// Table-gradient merge buffer of one workgroup: kLines 64-B table lines (8 entries x 2 features) in LDS, open
// addressing on the line index.  Scattered float atomics cost one memory-side request per 64-B line an
// instruction touches (~20 G requests/s chip-wide, MI355X_MICROARCH.md §Global float atomics), so the walk adds
// every corner gradient into LDS and the block flushes each touched line once, its nonzero floats in one
// 16-lane segment: the centre and taps of a sample share most corners at the fine levels (their cells are
// neighbours -- shared corners sit in different corner slots of the two points) and consecutive samples of a ray
// share cells at the coarse ones.  On the hash_bench geometry this is ~3.9 M line requests per SDF batch instead of
// the per-lane pending merge's 9.3 M.  A line that finds no slot within kMaxProbe probes goes straight to memory.
// Diagnostic variant builds (scripts/hash_variants.py compiles them separately; the product library uses the
// defaults): MMS_HASH_LOG_LINES = log2 of the merge-table lines, MMS_HASH_CH5 = samples per block of the SDF batch,
// MMS_HASH_FINE = first level whose pending gradients go straight to memory instead of through the LDS merge
// (MMS_HASH_FINE1 / MMS_HASH_CH1: the same for the plain, one-row-per-point walk).
#ifndef MMS_HASH_LOG_LINES
#define MMS_HASH_LOG_LINES 9
#endif
#ifndef MMS_HASH_CH5
#define MMS_HASH_CH5 4
#endif
#ifndef MMS_HASH_FINE
#define MMS_HASH_FINE 12
#endif
#ifndef MMS_HASH_FINE1
#define MMS_HASH_FINE1 MMS_HASH_FINE
#endif
#ifndef MMS_HASH_CH1
#define MMS_HASH_CH1 8
#endif
constexpr int kLogLines = MMS_HASH_LOG_LINES;
constexpr int kLines = 1 << kLogLines;
constexpr int kMaxProbe = 32;
constexpr uint32_t kEmpty = 0xffffffffu;

__device__ __forceinline__ void merge_add(uint32_t* keys, float* vals, float* __restrict__ dtable, uint32_t entry,
                                          int feat, float v) {
  const uint32_t line = entry >> 3;
  uint32_t h = (line * 0x9E3779B1u) >> (32 - kLogLines);
#pragma unroll 1
  for (int probe = 0; probe < kMaxProbe; ++probe) {
    // one LDS round trip per probe: the compare-and-swap claims an empty slot or returns its owner
    const uint32_t k = atomicCAS(&keys[h], kEmpty, line);
    if (k == kEmpty || k == line) {
      atomicAdd(&vals[h * 16 + (entry & 7) * 2 + feat], v);
      return;
    }
    h = (h + 1) & (kLines - 1);
  }
  atomicAdd(dtable + 2 * (int64_t)entry + feat, v);
}

// Backward ("walk"): one workgroup = 16 level groups x 16 lanes and owns CH consecutive point groups (rows
// g0 .. g0+CH-1 and, for G = 5, their tap rows g + j * gstride).  A level group walks the CH * G points in order
// (centre, then its 4 taps, then the next sample); lane q holds one (corner, feature) slot -- (y, z) corner pair
// q >> 2, x side (q >> 1) & 1, feature q & 1 -- and keeps ONE pending (table entry, gradient) accumulator that goes
// to the LDS merge buffer (merge_add) only when its entry changes; the buffer's lines are added to the table gradient
// at the end, one 16-lane segment per line.  Measured on the SDF batch (scripts/hash_bench.py): 0.48 ms against
// 0.53 ms for per-lane global atomics; the merge's LDS round trips (compare-and-swap, then add) now bound the walk --
// issuing all of a lane's lookups together (unrolled two-pass form) measured slower (0.72 ms).
// The block first stages its points' normalised positions x_hat = (x + r) / (2 r) (one exact division per
// coordinate per point instead of one per lane and level) and their output-gradient rows (coalesced 128-B rows
// instead of 4-B loads replicated over 8 lanes) in LDS.  Position gradients are summed over the wave's 4 levels x
// 16 lanes by DPP moves (wave_sum_to_63) into a per-wave LDS slot -- plain stores, no LDS atomics -- and the 4 waves'
// partials are added in wave order at the end: dpos is deterministic.
template <int G, int CH, int FINE>
__global__ __launch_bounds__(256) void hashgrid_bwd_walk_kernel(const float* __restrict__ pos, int64_t Mg,
                                                                int64_t gstride, int64_t ldx,
                                                                const float* __restrict__ table, GridParams p,
                                                                const float* __restrict__ dout, int64_t ldd,
                                                                float* __restrict__ dtable, float* __restrict__ dpos,
                                                                int64_t lddx) {
  constexpr int NP = CH * G;
  __shared__ float shat[NP][3];
  __shared__ float sde[NP][2 * kMaxLevels];
  __shared__ float sdp[4][NP][3];
  __shared__ uint32_t skeys[kLines];
  __shared__ f4 svals[kLines * 4];
  float* vals = reinterpret_cast<float*>(svals);
  const int t = threadIdx.x;
  const int level = t >> 4;
  const int wave = t >> 6;
  const int q = t & 15;
  const int pr = q >> 2;                // 0: (y c, z c)  1: (y f, z c)  2: (y c, z f)  3: (y f, z f)
  const bool xc = ((q >> 1) & 1) == 0;  // x = ceil corner
  const bool yc = (pr & 1) == 0, zc = pr < 2;
  const int feat = q & 1;
  const int64_t g0 = xcd_block() * CH;
  const int nck = (int)((Mg - g0) < CH ? (Mg - g0) : CH);
  const int np = nck * G;
  const int nlv = p.levels < p.active_levels ? p.levels : p.active_levels;  // levels with a gradient
  const int nc = 2 * p.levels;
  // point i of the block: sample k = i / G, tap j = i % G (walk order)
  auto row_of = [&](int i) {
    const int k = i / G, j = i - k * G;
    return g0 + k + (int64_t)j * gstride;
  };
  {
    const float two_r = 2.0f * p.radius;
    const bool norm = p.radius > 0.f;
    if ((t & 3) < 3)
      for (int pi = t >> 2; pi < np; pi += 64) {
        const float x = pos[row_of(pi) * ldx + (t & 3)];
        shat[pi][t & 3] = norm ? (x + p.radius) / two_r : x;  // make_corners' rounding (bit-exact corners)
      }
    if ((t & 31) < nc)
      for (int pi = t >> 5; pi < np; pi += 8) sde[pi][t & 31] = dout[row_of(pi) * ldd + (t & 31)];
    if (dpos != nullptr)
      for (int i = t; i < 4 * NP * 3; i += 256) (&sdp[0][0][0])[i] = 0.f;
    if (dtable != nullptr) {
      for (int i = t; i < kLines; i += 256) skeys[i] = kEmpty;
      for (int i = t; i < 4 * kLines; i += 256) svals[i] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  // a wave runs if any of its 4 levels has a gradient (its inactive rows contribute zeros and read no table entry)
  if (4 * wave < nlv) {
    const bool live = level < nlv;
    const float s = p.scale[level];
    const uint32_t hmask = (1u << p.log2T) - 1u;
    const uint32_t base = live ? (uint32_t)level << p.log2T : 0u;
    const bool sm = p.smooth != 0;
    uint32_t pidx = 0u;
    float pacc = 0.f;
    for (int i = 0; i < np; ++i) {
      const float sx = shat[i][0] * s, sy = shat[i][1] * s, sz = shat[i][2] * s;
      const float dE = live ? sde[i][2 * level + feat] : 0.f;
      const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
      const float tx = sx - fx, ty = sy - fy, tz = sz - fz;
      const float ox = sm ? smoothstep(tx) : tx, oy = sm ? smoothstep(ty) : ty, oz = sm ? smoothstep(tz) : tz;
      const int cx = xc ? (int)ceilf(sx) : (int)fx;
      const int cy = yc ? (int)ceilf(sy) : (int)fy;
      const int cz = zc ? (int)ceilf(sz) : (int)fz;
      const uint32_t idx = base + (live ? hash3(cx, cy, cz, hmask) : 0u);
      const float wx = xc ? ox : 1.0f - ox, wy = yc ? oy : 1.0f - oy, wz = zc ? oz : 1.0f - oz;
      // the position gradient's table value: issued before the merge work below, used after it
      const float tv = (dpos != nullptr && live) ? table[2 * (int64_t)idx + feat] : 0.f;
      if (dtable != nullptr) {
        // autograd order of encodings.py:292-302 reversed: ((dE * w_z) * w_y) * w_x
        const float df = ((dE * wz) * wy) * wx;
        if (idx == pidx) {
          pacc += df;
        } else {
          if (pacc != 0.f) {
            if (level >= FINE) atomicAdd(dtable + 2 * (int64_t)pidx + feat, pacc);
            else merge_add(skeys, vals, dtable, pidx, feat, pacc);
          }
          pidx = idx;
          pacc = df;
        }
      }
      if (dpos != nullptr) {
        const float e = dE * tv;
        float gx = (xc ? e : -e) * (wz * wy);
        float gy = (yc ? e : -e) * (wz * wx);
        float gz = (zc ? e : -e) * (wy * wx);
        if (sm) {  // d weight / d frac = +-S'(frac)
          gx *= smoothstep_grad(tx);
          gy *= smoothstep_grad(ty);
          gz *= smoothstep_grad(tz);
        }
        // d x_hat * s per level; the wave's 4 levels summed in lane 63
        gx = wave_sum_to_63(gx * s);
        gy = wave_sum_to_63(gy * s);
        gz = wave_sum_to_63(gz * s);
        if ((t & 63) == 63) {
          sdp[wave][i][0] = gx;
          sdp[wave][i][1] = gy;
          sdp[wave][i][2] = gz;
        }
      }
    }
    if (dtable != nullptr && pacc != 0.f) {
      if (level >= FINE) atomicAdd(dtable + 2 * (int64_t)pidx + feat, pacc);
      else merge_add(skeys, vals, dtable, pidx, feat, pacc);
    }
  }
  __syncthreads();
  if (dtable != nullptr) {
    // flush: 4 lines per wave-instruction, lane (t & 15) = float (entry (t & 15) / 2, feature t & 1) of the line
    for (int sl = t >> 4; sl < kLines; sl += 16) {
      const uint32_t k = skeys[sl];
      const float v = vals[sl * 16 + (t & 15)];
      if (k != kEmpty && v != 0.f) atomicAdd(dtable + (int64_t)k * 16 + (t & 15), v);
    }
  }
  if (dpos != nullptr) {
    const float two_r = p.radius > 0.f ? 2.0f * p.radius : 1.0f;
    if ((t & 3) < 3)
      for (int pi = t >> 2; pi < np; pi += 64) {
        const int c = t & 3;
        const float v = ((sdp[0][pi][c] + sdp[1][pi][c]) + sdp[2][pi][c]) + sdp[3][pi][c];
        dpos[row_of(pi) * lddx + c] += v / two_r;
      }
  }
}

// Position gradient alone, as a gather like the forward (thread per (point, level), 16 lanes per point, the SDF
// batch in (sample, tap) order): every lane's 8 corner loads are independent, so they are all in flight at once --
// the walk kernel's per-point table re-gather sat on one global-load latency per point, serially.  Per level:
// d out_f / d x_axis = s / (2 r) sum_c T[c][f] dw_c / d o_axis (w_c the trilinear -- or smoothstep -- corner weight,
// +-1 times the other two axes' weights, times S'(t) in Smoothstep mode); the 16 levels are summed by xor shuffles.
template <int G>
__global__ __launch_bounds__(256) void hashgrid_dpos_kernel(const float* __restrict__ pos, int64_t Mg, int64_t gstride,
                                                            int64_t ldx, const float2* __restrict__ table, GridParams p,
                                                            const float* __restrict__ dout, int64_t ldd,
                                                            float* __restrict__ dpos, int64_t lddx) {
  const int64_t tid = xcd_block() * blockDim.x + threadIdx.x;
  const int64_t q = tid >> 4;
  const int level = (int)(tid & 15);
  const int64_t g = G == 1 ? q : q / G;
  const int64_t pt = G == 1 ? q : g + (q - g * G) * gstride;
  if (g >= Mg) return;   // whole 16-lane groups (one point) leave together
  const int nlv = p.levels < p.active_levels ? p.levels : p.active_levels;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  if (level < nlv) {
    const float* xp = pos + pt * ldx;
    const float s = p.scale[level];
    const float two_r = 2.0f * p.radius;
    const bool norm = p.radius > 0.f;
    const float hx = norm ? (xp[0] + p.radius) / two_r : xp[0];   // make_corners' rounding (same corners)
    const float hy = norm ? (xp[1] + p.radius) / two_r : xp[1];
    const float hz = norm ? (xp[2] + p.radius) / two_r : xp[2];
    Corners c = make_corners(xp[0], xp[1], xp[2], p.radius, p.inv_2r, s, level, p.log2T, p.smooth != 0);
    float2 f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = table[c.idx[i]];
    const float dE0 = dout[pt * ldd + 2 * level], dE1 = dout[pt * ldd + 2 * level + 1];
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = dE0 * f[i].x + dE1 * f[i].y;
    const float ox = c.ox, oy = c.oy, oz = c.oz, nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
    // corners (x, y, z sides; c = ceil, weight o; f = floor, weight 1 - o):
    // 0 ccc, 1 cfc, 2 ffc, 3 fcc, 4 ccf, 5 cff, 6 fff, 7 fcf
    gx = ((e[0] * oy + e[1] * ny) * oz + (e[4] * oy + e[5] * ny) * nz) -
         ((e[3] * oy + e[2] * ny) * oz + (e[7] * oy + e[6] * ny) * nz);
    gy = ((e[0] * ox + e[3] * nx) * oz + (e[4] * ox + e[7] * nx) * nz) -
         ((e[1] * ox + e[2] * nx) * oz + (e[5] * ox + e[6] * nx) * nz);
    gz = ((e[0] * ox + e[3] * nx) * oy + (e[1] * ox + e[2] * nx) * ny) -
         ((e[4] * ox + e[7] * nx) * oy + (e[5] * ox + e[6] * nx) * ny);
    if (p.smooth) {
      const float sx = hx * s, sy = hy * s, sz = hz * s;
      gx *= smoothstep_grad(sx - floorf(sx));
      gy *= smoothstep_grad(sy - floorf(sy));
      gz *= smoothstep_grad(sz - floorf(sz));
    }
    gx *= s;
    gy *= s;
    gz *= s;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    gx += __shfl_xor(gx, o);
    gy += __shfl_xor(gy, o);
    gz += __shfl_xor(gz, o);
  }
  if (level == 0) {
    const float two_r = p.radius > 0.f ? 2.0f * p.radius : 1.0f;
    float* d = dpos + pt * lddx;
    d[0] += gx / two_r;
    d[1] += gy / two_r;
    d[2] += gz / two_r;
  }
}

int fill_params(const char* fn, GridParams& p, int L, int log2T, int interp, const float* scales, float radius,
                int active_levels) {
  if (L < 1 || L > kMaxLevels) return mms::set_error(fn, "num_levels must be in [1, 16]");
  if (interp != 0 && interp != 1) return mms::set_error(fn, "interp must be 0 (Linear) or 1 (Smoothstep)");
  p.smooth = interp;
  if (log2T < 1 || log2T > 24) return mms::set_error(fn, "log2_hashmap_size must be in [1, 24]");
  if (!(radius >= 0.f)) return mms::set_error(fn, "radius must be >= 0 (0: inputs already in [0, 1])");
  p.levels = L;
  p.active_levels = active_levels < 0 ? L : (active_levels > L ? L : active_levels);
  p.log2T = log2T;
  p.radius = radius;
  p.inv_2r = radius > 0.f ? 1.0f / (2.0f * radius) : 1.0f;
  for (int i = 0; i < kMaxLevels; ++i) p.scale[i] = i < L ? scales[i] : 0.f;
  return 0;
}

}  // namespace

MMS_EXPORT int mms_hashgrid_fwd_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                                        const float* table, int L, int log2T, int F, int interp, const float* scales,
                                        float radius, int active_levels, float* out, int64_t ldo, void* stream) {
  const char* fn = "mms_hashgrid_fwd_grouped";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(Mg >= 0 && ldx >= 3 && ldo >= 2 * L, fn, "bad shapes");
  MMS_REQUIRE(group == 1 || group == 5, fn, "group must be 1 (plain) or 5 (centre + 4 taps)");
  MMS_REQUIRE(group == 1 || gstride >= Mg, fn, "group rows overlap (gstride < groups)");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (Mg == 0) return 0;
  MMS_REQUIRE(pos && table && out, fn, "null pointer");
  MMS_REQUIRE(((uintptr_t)out & 3) == 0, fn, "output must be 4-B aligned");
  const int64_t threads = Mg * group * 16;
  const unsigned blocks = mms::grid_for(threads, 256, INT32_MAX);
  const bool aligned = ((uintptr_t)out & 7) == 0 && (ldo & 1) == 0;
  const float2* t2 = reinterpret_cast<const float2*>(table);
  hipStream_t s = mms::as_stream(stream);
  if (group == 5) {
    if (aligned)
      hipLaunchKernelGGL((hashgrid_fwd_kernel<true, 5>), dim3(blocks), dim3(256), 0, s, pos, Mg, gstride, ldx, t2, p,
                         out, ldo);
    else
      hipLaunchKernelGGL((hashgrid_fwd_kernel<false, 5>), dim3(blocks), dim3(256), 0, s, pos, Mg, gstride, ldx, t2, p,
                         out, ldo);
  } else {
    if (aligned)
      hipLaunchKernelGGL((hashgrid_fwd_kernel<true, 1>), dim3(blocks), dim3(256), 0, s, pos, Mg, Mg, ldx, t2, p, out,
                         ldo);
    else
      hipLaunchKernelGGL((hashgrid_fwd_kernel<false, 1>), dim3(blocks), dim3(256), 0, s, pos, Mg, Mg, ldx, t2, p, out,
                         ldo);
  }
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hashgrid_fwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L,
                                int log2T, int F, int interp, const float* scales, float radius, int active_levels,
                                float* out, int64_t ldo, void* stream) {
  return mms_hashgrid_fwd_grouped(pos, M, 1, M, ldx, table, L, log2T, F, interp, scales, radius, active_levels, out,
                                  ldo, stream);
}

MMS_EXPORT int mms_sdf_panel_fwd(const float* cpos, int64_t ldp, int64_t M, int ntaps, float delta, int pe_freqs,
                                 const float* table, int L, int log2T, int F, int interp, const float* scales,
                                 float radius, int active_levels, float* X, int64_t ldx, void* stream) {
  const char* fn = "mms_sdf_panel_fwd";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(ntaps == 0 || ntaps == 4, fn, "ntaps must be 0 or 4");
  MMS_REQUIRE(pe_freqs >= 1 && pe_freqs <= 16, fn, "1 to 16 encoding frequencies");
  MMS_REQUIRE(M >= 0 && ldp >= 3 && ldx >= 3 + 6 * pe_freqs + 2 * L, fn, "bad shapes");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (M == 0) return 0;
  MMS_REQUIRE(cpos && table && X, fn, "null pointer");
  const int group = ntaps + 1;
  const unsigned blocks = mms::grid_for(M * group * 16, 256, INT32_MAX);
  const float2* t2 = reinterpret_cast<const float2*>(table);
  hipStream_t s = mms::as_stream(stream);
  if (group == 5)
    hipLaunchKernelGGL((sdf_panel_fwd_kernel<5>), dim3(blocks), dim3(256), 0, s, cpos, ldp, M, delta, pe_freqs, t2, p,
                       X, ldx, RaySrc{});
  else
    hipLaunchKernelGGL((sdf_panel_fwd_kernel<1>), dim3(blocks), dim3(256), 0, s, cpos, ldp, M, delta, pe_freqs, t2, p,
                       X, ldx, RaySrc{});
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_sdf_panel_rays_fwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars,
                                      const float* origins, const float* dirs, int64_t R, int pe_freqs,
                                      const float* table, int L, int log2T, int F, int interp, const float* scales,
                                      float radius, int active_levels, float* X, int64_t ldx, void* stream) {
  const char* fn = "mms_sdf_panel_rays_fwd";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(pe_freqs >= 1 && pe_freqs <= 16, fn, "1 to 16 encoding frequencies");
  MMS_REQUIRE(R >= 0 && nb >= 2 && ldb >= nb && ldx >= 3 + 6 * pe_freqs + 2 * L, fn, "bad shapes");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (R == 0) return 0;
  MMS_REQUIRE(bins && nears && fars && origins && dirs && table && X, fn, "null pointer");
  const int64_t M = R * (nb - 1);
  const RaySrc rs{bins, ldb, nb, nears, fars, origins, dirs};
  hipLaunchKernelGGL((sdf_panel_fwd_kernel<1, true>), dim3(mms::grid_for(M * 16, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), nullptr, 3, M, 0.0f, pe_freqs, reinterpret_cast<const float2*>(table), p,
                     X, ldx, rs);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_rad_panel_fwd(const float* pos, int64_t ldp, const float* dirs, const float* normals,
                                 const float* geo, int64_t ldg, int64_t M, int S, int G, const float* table, int L,
                                 int log2T, int F, int interp, const float* scales, float radius, int active_levels,
                                 float* X, int64_t ldx, void* stream) {
  const char* fn = "mms_rad_panel_fwd";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(S >= 1 && G >= 0 && M >= 0 && ldp >= 3 && ldx >= 29 + G + 2 * L, fn, "bad shapes");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (M == 0) return 0;
  MMS_REQUIRE(pos && dirs && normals && table && X && (G == 0 || geo), fn, "null pointer");
  static const bool staged = [] {
    const char* e = getenv("MMS_RAD_STAGED");
    return e == nullptr || e[0] != '0';
  }();
  if (staged && G <= 256)
    hipLaunchKernelGGL(rad_panel_fwd_staged_kernel, dim3(mms::grid_for(M, kRadPts, INT32_MAX)), dim3(256), 0,
                       mms::as_stream(stream), pos, ldp, dirs, normals, geo, ldg, M, S, G,
                       reinterpret_cast<const float2*>(table), p, X, ldx);
  else
    hipLaunchKernelGGL(rad_panel_fwd_kernel, dim3(mms::grid_for(M * 16, 256, INT32_MAX)), dim3(256), 0,
                       mms::as_stream(stream), pos, ldp, dirs, normals, geo, ldg, M, S, G,
                       reinterpret_cast<const float2*>(table), p, X, ldx);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hashgrid_bwd_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                                        const float* table, int L, int log2T, int F, int interp,
                                        const float* scales, float radius, int active_levels, const float* dout,
                                        int64_t ldd, float* dtable, float* dpos, int64_t lddx, void* stream) {
  const char* fn = "mms_hashgrid_bwd_grouped";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(Mg >= 0 && ldx >= 3 && ldd >= 2 * L, fn, "bad shapes");
  MMS_REQUIRE(group == 1 || group == 5, fn, "group must be 1 (plain) or 5 (centre + 4 taps)");
  MMS_REQUIRE(group == 1 || gstride >= Mg, fn, "group rows overlap (gstride < groups)");
  MMS_REQUIRE(dpos == nullptr || lddx >= 3, fn, "bad dpos stride");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (Mg == 0 || (dtable == nullptr && dpos == nullptr)) return 0;
  MMS_REQUIRE(pos && table && dout, fn, "null pointer");
  // CH: about 260 touched lines per block on the SDF batch (kLines = 512 merge slots: 4 blocks per CU)
  if (group == 5) {
    constexpr int CH = MMS_HASH_CH5;
    hipLaunchKernelGGL((hashgrid_bwd_walk_kernel<5, CH, MMS_HASH_FINE>), dim3(mms::grid_for(Mg, CH, INT32_MAX)), dim3(256), 0,
                       mms::as_stream(stream), pos, Mg, gstride, ldx, table, p, dout, ldd, dtable, dpos, lddx);
  } else {
    constexpr int CH = MMS_HASH_CH1;
    hipLaunchKernelGGL((hashgrid_bwd_walk_kernel<1, CH, MMS_HASH_FINE1>), dim3(mms::grid_for(Mg, CH, INT32_MAX)), dim3(256), 0,
                       mms::as_stream(stream), pos, Mg, Mg, ldx, table, p, dout, ldd, dtable, dpos, lddx);
  }
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hashgrid_bwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L,
                                int log2T, int F, int interp, const float* scales, float radius, int active_levels,
                                const float* dout, int64_t ldd, float* dtable, float* dpos, int64_t lddx,
                                void* stream) {
  return mms_hashgrid_bwd_grouped(pos, M, 1, M, ldx, table, L, log2T, F, interp, scales, radius, active_levels, dout,
                                  ldd, dtable, dpos, lddx, stream);
}

MMS_EXPORT int mms_hashgrid_dpos_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                                         const float* table, int L, int log2T, int F, int interp, const float* scales,
                                         float radius, int active_levels, const float* dout, int64_t ldd, float* dpos,
                                         int64_t lddx, void* stream) {
  const char* fn = "mms_hashgrid_dpos_grouped";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(Mg >= 0 && ldx >= 3 && ldd >= 2 * L && lddx >= 3, fn, "bad shapes");
  MMS_REQUIRE(group == 1 || group == 5, fn, "group must be 1 (plain) or 5 (centre + 4 taps)");
  MMS_REQUIRE(group == 1 || gstride >= Mg, fn, "group rows overlap (gstride < groups)");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, interp, scales, radius, active_levels);
  if (rc) return rc;
  if (Mg == 0) return 0;
  MMS_REQUIRE(pos && table && dout && dpos, fn, "null pointer");
  const unsigned blocks = mms::grid_for(Mg * group * 16, 256, INT32_MAX);
  const float2* t2 = reinterpret_cast<const float2*>(table);
  hipStream_t s = mms::as_stream(stream);
  if (group == 5)
    hipLaunchKernelGGL((hashgrid_dpos_kernel<5>), dim3(blocks), dim3(256), 0, s, pos, Mg, gstride, ldx, t2, p, dout, ldd,
                       dpos, lddx);
  else
    hipLaunchKernelGGL((hashgrid_dpos_kernel<1>), dim3(blocks), dim3(256), 0, s, pos, Mg, Mg, ldx, t2, p, dout, ldd,
                       dpos, lddx);
  return mms::check_launch(fn);
}
