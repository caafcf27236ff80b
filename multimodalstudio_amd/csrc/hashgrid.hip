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

// Bit-exact corner selection needs the rounded product x_hat * s before floor/frac (a fused
// multiply-subtract would change the fractional weights), so contraction is off in this file; the
// kernels are gather-bound, the extra VALU is free.
#pragma clang fp contract(off)

namespace {

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
};

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
                                                float s, int level, int log2T) {
  Corners c;
  // (x + r) / (2r): reference computes a true division by (2r); for r in {1, 2} the reciprocal
  // multiply is exact, but keep the division for bit-exact corner indices in general.
  const float two_r = 2.0f * radius;
  const float hx = (x + radius) / two_r;
  const float hy = (y + radius) / two_r;
  const float hz = (z + radius) / two_r;
  (void)inv_2r;
  const float sx = hx * s, sy = hy * s, sz = hz * s;
  const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
  const int cxc = (int)ceilf(sx), cyc = (int)ceilf(sy), czc = (int)ceilf(sz);
  const int cxf = (int)fx, cyf = (int)fy, czf = (int)fz;
  c.ox = sx - fx;
  c.oy = sy - fy;
  c.oz = sz - fz;
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

__global__ __launch_bounds__(256) void hashgrid_fwd_kernel(const float* __restrict__ pos, int64_t M,
                                                           int64_t ldx, const float2* __restrict__ table,
                                                           GridParams p, float* __restrict__ out,
                                                           int64_t ldo) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pt = tid >> 4;
  const int level = (int)(tid & 15);
  if (pt >= M || level >= p.levels) return;
  float2 r = make_float2(0.f, 0.f);
  if (level < p.active_levels) {
    const float* xp = pos + pt * ldx;
    Corners c = make_corners(xp[0], xp[1], xp[2], p.radius, p.inv_2r, p.scale[level], level, p.log2T);
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
  *reinterpret_cast<float2*>(out + pt * ldo + 2 * level) = r;
}

// Backward: dtable (atomic accumulate) and optional dx (accumulate into dpos[:, 0:3]).
//
// Points come in groups of G rows (row = g + j * gstride, j < G): the SDF batch is [centre | 4 taps]
// with the taps a few 1e-3 apart (surface_model.py:138-160), so at all but the finest levels the G points
// of a group fall into one grid cell.  Each lane walks the G points of its group and merges the corner
// gradients of consecutive points that share the cell before issuing the atomics: the table gradient is
// bound by scattered f32 atomics, and this removes up to (G-1)/G of them.
// One lane per (group, level, feature): the two features of a table entry are added by lanes 2j, 2j+1 of the
// same atomic instruction, i.e. in one 64-B memory-side atomic request instead of two (scattered f32 atomics
// cost per request, MI355X_MICROARCH.md §Global float atomics).
__device__ __forceinline__ void flush_corners(float* __restrict__ dtable, int feat, const uint32_t (&idx)[8],
                                              const float (&acc)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    // merge duplicate corners inside the cell (integer coordinates => ceil == floor)
    bool dup = false;
    float a = acc[i];
#pragma unroll
    for (int j = 0; j < i; ++j) dup |= (idx[j] == idx[i]);
    if (dup) continue;
#pragma unroll
    for (int j = i + 1; j < 8; ++j)
      if (idx[j] == idx[i]) a += acc[j];
    atomicAdd(dtable + 2 * (int64_t)idx[i] + feat, a);
  }
}

template <int G>
__global__ __launch_bounds__(256) void hashgrid_bwd_kernel(const float* __restrict__ pos, int64_t Mg,
                                                           int64_t gstride, int64_t ldx,
                                                           const float* __restrict__ table, GridParams p,
                                                           const float* __restrict__ dout, int64_t ldd,
                                                           float* __restrict__ dtable, float* __restrict__ dpos,
                                                           int64_t lddx) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t grp = tid >> 5;
  const int level = (int)((tid >> 1) & 15);
  const int feat = (int)(tid & 1);
  const bool live = grp < Mg && level < p.levels && level < p.active_levels;
  const float s = p.scale[level];
  uint32_t pidx[8];
  float pacc[8];
  bool pending = false;
#pragma unroll
  for (int i = 0; i < 8; ++i) { pidx[i] = 0; pacc[i] = 0.f; }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int64_t pt = grp + (int64_t)j * gstride;
    float gx = 0.f, gy = 0.f, gz = 0.f;
    if (live) {
      const float* xp = pos + pt * ldx;
      const Corners c = make_corners(xp[0], xp[1], xp[2], p.radius, p.inv_2r, s, level, p.log2T);
      const float dE = dout[pt * ldd + 2 * level + feat];
      const float ox = c.ox, oy = c.oy, oz = c.oz;
      const float nx = 1.0f - ox, ny = 1.0f - oy, nz = 1.0f - oz;
      // autograd order of encodings.py:292-302 reversed (per feature)
      const float d0312 = dE * oz, d4756 = dE * nz;
      const float d03 = d0312 * oy, d12 = d0312 * ny, d47 = d4756 * oy, d56 = d4756 * ny;
      float df[8];
      df[0] = d03 * ox; df[3] = d03 * nx;
      df[1] = d12 * ox; df[2] = d12 * nx;
      df[5] = d56 * ox; df[6] = d56 * nx;
      df[4] = d47 * ox; df[7] = d47 * nx;
      if (dtable != nullptr) {
        // same 8 table entries as the pending point (same cell) -> merge, else flush the pending set
        bool same = pending;
#pragma unroll
        for (int i = 0; i < 8; ++i) same &= (pidx[i] == c.idx[i]);
        if (same) {
#pragma unroll
          for (int i = 0; i < 8; ++i) pacc[i] += df[i];
        } else {
          if (pending) flush_corners(dtable, feat, pidx, pacc);
#pragma unroll
          for (int i = 0; i < 8; ++i) { pidx[i] = c.idx[i]; pacc[i] = df[i]; }
          pending = true;
        }
      }
      if (dpos != nullptr) {
        float f[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = table[2 * (int64_t)c.idx[i] + feat];
        const float f03 = f[0] * ox + f[3] * nx, f12 = f[1] * ox + f[2] * nx;
        const float f56 = f[5] * ox + f[6] * nx, f47 = f[4] * ox + f[7] * nx;
        const float f0312 = f03 * oy + f12 * ny, f4756 = f47 * oy + f56 * ny;
        gz = dE * (f0312 - f4756) * s;
        gy = (d0312 * (f03 - f12) + d4756 * (f47 - f56)) * s;
        gx = (d03 * (f[0] - f[3]) + d12 * (f[1] - f[2]) + d56 * (f[5] - f[6]) + d47 * (f[4] - f[7])) * s;
      }
    }
    if (dpos != nullptr) {
      // reduce over the 16 levels x 2 features of a point (32 consecutive lanes)
#pragma unroll
      for (int off = 16; off >= 1; off >>= 1) {
        gx += __shfl_xor(gx, off, 32);
        gy += __shfl_xor(gy, off, 32);
        gz += __shfl_xor(gz, off, 32);
      }
      if ((tid & 31) == 0 && grp < Mg) {
        float* dp = dpos + pt * lddx;
        const float two_r = 2.0f * p.radius;
        dp[0] += gx / two_r;
        dp[1] += gy / two_r;
        dp[2] += gz / two_r;
      }
    }
  }
  if (pending) flush_corners(dtable, feat, pidx, pacc);
}

int fill_params(const char* fn, GridParams& p, int L, int log2T, const float* scales, float radius,
                int active_levels) {
  if (L < 1 || L > kMaxLevels) return mms::set_error(fn, "num_levels must be in [1, 16]");
  if (log2T < 1 || log2T > 24) return mms::set_error(fn, "log2_hashmap_size must be in [1, 24]");
  if (!(radius > 0.f)) return mms::set_error(fn, "radius must be > 0");
  p.levels = L;
  p.active_levels = active_levels < 0 ? L : (active_levels > L ? L : active_levels);
  p.log2T = log2T;
  p.radius = radius;
  p.inv_2r = 1.0f / (2.0f * radius);
  for (int i = 0; i < kMaxLevels; ++i) p.scale[i] = i < L ? scales[i] : 0.f;
  return 0;
}

}  // namespace

MMS_EXPORT int mms_hashgrid_fwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L,
                                int log2T, int F, const float* scales, float radius, int active_levels,
                                float* out, int64_t ldo, void* stream) {
  const char* fn = "mms_hashgrid_fwd";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(M >= 0 && ldx >= 3 && ldo >= 2 * L, fn, "bad shapes");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, scales, radius, active_levels);
  if (rc) return rc;
  if (M == 0) return 0;
  MMS_REQUIRE(pos && table && out, fn, "null pointer");
  const int64_t threads = M * 16;
  hipLaunchKernelGGL(hashgrid_fwd_kernel, dim3(mms::grid_for(threads, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), pos, M, ldx, reinterpret_cast<const float2*>(table), p, out,
                     ldo);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hashgrid_bwd_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                                        const float* table, int L, int log2T, int F, const float* scales,
                                        float radius, int active_levels, const float* dout, int64_t ldd,
                                        float* dtable, float* dpos, int64_t lddx, void* stream) {
  const char* fn = "mms_hashgrid_bwd_grouped";
  MMS_REQUIRE(F == 2, fn, "features_per_level must be 2");
  MMS_REQUIRE(Mg >= 0 && ldx >= 3 && ldd >= 2 * L, fn, "bad shapes");
  MMS_REQUIRE(group == 1 || group == 5, fn, "group must be 1 (plain) or 5 (centre + 4 taps)");
  MMS_REQUIRE(group == 1 || gstride >= Mg, fn, "group rows overlap (gstride < groups)");
  MMS_REQUIRE(dpos == nullptr || lddx >= 3, fn, "bad dpos stride");
  GridParams p;
  int rc = fill_params(fn, p, L, log2T, scales, radius, active_levels);
  if (rc) return rc;
  if (Mg == 0 || (dtable == nullptr && dpos == nullptr)) return 0;
  MMS_REQUIRE(pos && table && dout, fn, "null pointer");
  const int64_t threads = Mg * 32;
  const dim3 grid(mms::grid_for(threads, 256, INT32_MAX));
  if (group == 5)
    hipLaunchKernelGGL(hashgrid_bwd_kernel<5>, grid, dim3(256), 0, mms::as_stream(stream), pos, Mg, gstride, ldx,
                       table, p, dout, ldd, dtable, dpos, lddx);
  else
    hipLaunchKernelGGL(hashgrid_bwd_kernel<1>, grid, dim3(256), 0, mms::as_stream(stream), pos, Mg, Mg, ldx,
                       table, p, dout, ldd, dtable, dpos, lddx);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_hashgrid_bwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L,
                                int log2T, int F, const float* scales, float radius, int active_levels,
                                const float* dout, int64_t ldd, float* dtable, float* dpos, int64_t lddx,
                                void* stream) {
  return mms_hashgrid_bwd_grouped(pos, M, 1, M, ldx, table, L, log2T, F, scales, radius, active_levels, dout, ldd,
                                  dtable, dpos, lddx, stream);
}
