// Input-panel assembly kernels for the geometry / radiance / background MLPs, and the
// numerical-gradient combine.  All panels are row-major [rows, ld] fp32; the hash-grid kernel writes
// its 32 feature columns straight into the same panels (see hashgrid.hip), so no concat copies exist.
//
// Reference semantics (paths under /root/reference/src):
//   NeRFEncoding.forward   field_components/encodings.py:161-182   [x, sin(x_i 2^k), sin(x_i 2^k + pi/2)]
//   SurfaceModel.gradient  model_components/surface_model.py:137-153 (4 taps, delta/sqrt(3))
//   SDF input columns      field_components/feature_structures.py:155-164  [x(3), PE-tail(36), grid(32)]
//   Radiance input columns radiance_model.py:114-132 + radiance_field.py:74 + feature_structures.py:155-164
//                          [x(3), SH(25), geo(256), n.v(1), grid(32)]
//   SH degree 4            utils/math.py:21-83 (SURVEY §8(c) patch 2)
//   SceneContraction(inf)  field_components/spatial_distortions.py:90-97
#include "common.h"
#include "sh.h"

// PE arguments must be the rounded products/sums the reference computes; keep the compiler from
// fusing them.
#pragma clang fp contract(off)

namespace {

__constant__ float kTap[4][3] = {{1.f, -1.f, -1.f}, {-1.f, -1.f, 1.f}, {-1.f, 1.f, -1.f}, {1.f, 1.f, 1.f}};
constexpr float kHalfPi = 1.57079632679489661923f;  // fl32(pi / 2)

// PE of one coordinate value into panel row: cols [3 + i*F + k] and [3 + 3F + i*F + k]
__device__ __forceinline__ void pe_write(float* row, int i, float xi, int F) {
  float f = 1.0f;
  for (int k = 0; k < F; ++k) {
    const float s = xi * f;
    row[3 + i * F + k] = sinf(s);
    row[3 + 3 * F + i * F + k] = sinf(s + kHalfPi);
    f *= 2.0f;
  }
}

__device__ __forceinline__ float pe_bwd(const float* drow, int i, float xi, int F) {
  float f = 1.0f, g = 0.f;
  for (int k = 0; k < F; ++k) {
    const float s = xi * f;
    g += drow[3 + i * F + k] * cosf(s) * f;
    g += drow[3 + 3 * F + i * F + k] * cosf(s + kHalfPi) * f;
    f *= 2.0f;
  }
  return g;
}

// rows [0, M) = centre points, [M (t+1), M (t+2)) = tap t (t = 0..ntaps-1)
// One thread per (row, column) of the [x(3), PE(6F)] head of the panel rows: consecutive lanes write consecutive
// columns, so a wave stores ~1.6 contiguous 156-B row heads (a thread per row wrote its 39 columns with a 288-B lane
// stride: 64 lines per store instruction, 58 us for the 278k-row SDF batch).  Column c < 3: x_c; 3 <= c < 3 + 3F:
// sin(x_i 2^k); then sin(x_i 2^k + pi/2), i = coordinate, k = frequency (pe_write's layout, same rounded arguments).
// IDX: the index type of the (row, column) decomposition -- uint32_t whenever the panel head has < 2^32 elements
// (the 64-bit divisions by the run-time width and row count cost more than the element's own work)
template <typename IDX>
__global__ __launch_bounds__(256) void geo_input_fwd_kernel(const float* __restrict__ pos, int64_t ldp, int64_t M,
                                                            int ntaps, float delta, int F, float* __restrict__ X,
                                                            int64_t ldx) {
  const int W = 3 + 6 * F;
  const IDX total = (IDX)(M * (1 + ntaps) * W);
  for (IDX q = (IDX)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (IDX)gridDim.x * blockDim.x) {
    const IDX r = q / (IDX)W;
    const int c = (int)(q - r * (IDX)W);
    const IDX t = r / (IDX)M, i = r - t * (IDX)M;
    int coord, k = 0;
    bool cosine = false;
    if (c < 3) {
      coord = c;
    } else if (c < 3 + 3 * F) {
      coord = (c - 3) / F;
      k = (c - 3) - coord * F;
    } else {
      coord = (c - 3 - 3 * F) / F;
      k = (c - 3 - 3 * F) - coord * F;
      cosine = true;
    }
    float x = pos[(int64_t)i * ldp + coord];
    if (t > 0) x = x + kTap[t - 1][coord] * delta;
    float v = x;
    if (c >= 3) {
      const float s = x * (float)(1 << k);   // 2^k exactly, as pe_write's running f *= 2
      v = cosine ? sinf(s + kHalfPi) : sinf(s);
    }
    X[(int64_t)r * ldx + c] = v;
  }
}

// dpos[i] += sum over the 1+ntaps rows of (dX[:, 0:3] + PE'(dX[:, 3:3+6F]) + dP[r])  (dP may be null)
__global__ void geo_input_bwd_kernel(const float* __restrict__ X, int64_t ldx, const float* __restrict__ dX,
                                     int64_t lddx, const float* __restrict__ dP, int64_t lddp, int64_t M, int ntaps,
                                     int F, float* __restrict__ dpos, int64_t lddpos) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    float g[3] = {0.f, 0.f, 0.f};
    for (int t = 0; t <= ntaps; ++t) {
      const int64_t r = t * M + i;
      const float* xr = X + r * ldx;
      const float* dr = dX + r * lddx;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        g[c] += dr[c] + pe_bwd(dr, c, xr[c], F);
        if (dP) g[c] += dP[r * lddp + c];
      }
    }
    float* o = dpos + i * lddpos;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] += g[c];
  }
}

// Same sums with 16 lanes per point: lane j < 3 (1 + ntaps) takes row t = j / 3 (the centre or a tap) and coordinate
// c = j % 3 -- its x column, its 2F PE columns and its dP entry -- so one point's 5 rows x 3 coordinates are read
// and their sin / cos evaluated by 15 lanes at once (a thread per point walked them one by one: 58 us for the 278k-row
// SDF batch); lanes c then add the rows of their coordinate, in row order, from the group by shuffles.
__global__ __launch_bounds__(256) void geo_input_bwd_lanes_kernel(const float* __restrict__ X, int64_t ldx,
                                                                  const float* __restrict__ dX, int64_t lddx,
                                                                  const float* __restrict__ dP, int64_t lddp,
                                                                  int64_t M, int ntaps, int F,
                                                                  float* __restrict__ dpos, int64_t lddpos) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = tid >> 4;
  const int j = (int)(tid & 15);
  const int t = j / 3, c = j - 3 * (j / 3);
  float g = 0.f;
  if (i < M && t <= ntaps) {
    const int64_t r = t * M + i;
    const float* dr = dX + r * lddx;
    g = dr[c] + pe_bwd(dr, c, X[r * ldx + c], F);
    if (dP) g += dP[r * lddp + c];
  }
  // lane c of the group sums the rows of coordinate c (lanes c, c + 3, ..., in row order, as the thread-per-point
  // kernel did)
  const int base = threadIdx.x & ~15;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 5; ++k) s += __shfl(g, base + c + 3 * k);
  if (i < M && j < 3) dpos[i * lddpos + c] += s;
}

// sdf5 rows: [centre M | tap0 M | .. | tap3 M] at column 0 of `out` (ld ldo).
// grads = sum_t k_t s_t / (4 delta); hxx = ((s0+s1+s2+s3)/2 - 2 y) / delta^2; hess = [hxx]*3 / 3;
// normals = grads / max(|grads|, 1e-12)
__global__ void taps_combine_fwd_kernel(const float* __restrict__ out, int64_t ldo, int64_t M, float inv4d,
                                        float inv_d2, float* __restrict__ grads, float* __restrict__ hess,
                                        float* __restrict__ normals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const float y = out[i * ldo];
    float s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) s[t] = out[((t + 1) * M + i) * ldo];
    float gr[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float a = kTap[0][c] * s[0];
      a = a + kTap[1][c] * s[1];
      a = a + kTap[2][c] * s[2];
      a = a + kTap[3][c] * s[3];
      gr[c] = a / inv4d;  // inv4d carries (4 delta) as computed by the reference
    }
    const float hxx = ((s[0] + s[1] + s[2] + s[3]) / 2.0f - 2.0f * y) / inv_d2;
    const float h3 = hxx / 3.0f;
    const float n = sqrtf(gr[0] * gr[0] + gr[1] * gr[1] + gr[2] * gr[2]);
    const float dn = fmaxf(n, 1e-12f);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      grads[i * 3 + c] = gr[c];
      hess[i * 3 + c] = h3;
      if (normals) normals[i * 3 + c] = gr[c] / dn;
    }
  }
}

// dst[r, c] = src[r, c] (zeros when src is null), r < M, c < G: one element per thread of the blocks
// [b0, gridDim.x), consecutive threads on consecutive columns (coalesced on both sides; a wave per row measured
// slower: 36 -> 52 us in the radiance panel).  The (row, column) split of the element index in 32 bits when the
// copy has < 2^32 elements (measured the same as the 64-bit split: profiles/round3d_ab.txt).
template <typename IDX>
__device__ __forceinline__ void copy_cols(const float* __restrict__ src, int64_t lds, float* __restrict__ dst,
                                          int64_t ldd, int64_t M, int G, unsigned b0) {
  const IDX n = (IDX)(M * G);
  for (IDX e = (IDX)(blockIdx.x - b0) * blockDim.x + threadIdx.x; e < n; e += (IDX)(gridDim.x - b0) * blockDim.x) {
    const IDX r = e / (IDX)G, c = e - r * (IDX)G;
    dst[(int64_t)r * ldd + c] = src ? src[(int64_t)r * lds + c] : 0.f;
  }
}
__device__ __forceinline__ void copy_cols_any(const float* __restrict__ src, int64_t lds, float* __restrict__ dst,
                                              int64_t ldd, int64_t M, int G, unsigned b0) {
  const int64_t span = (int64_t)(gridDim.x - b0) * blockDim.x;
  if (M * G < ((int64_t)1 << 32) - span)
    copy_cols<uint32_t>(src, lds, dst, ldd, M, G, b0);
  else
    copy_cols<int64_t>(src, lds, dst, ldd, M, G, b0);
}

// dst[r, 1 + c] = src[r, c] for c < G with 16-B aligned rows on both sides (dst's row pitch and base, src's): thread
// per (row, 16-B destination chunk) -- chunk 0 writes columns 1..3 alone (column 0 is the other blocks' sdf gradient),
// the others one float4 each, built from the source chunk and its predecessor's last element; the destination's
// columns past G + 1 inside the last chunk get zeros (the chains mask columns past K0).  A quarter of copy_cols'
// instructions for the SDF's 256 geo columns.
__device__ __forceinline__ void copy_cols_shift1_vec(const float* __restrict__ src, int64_t lds, float* __restrict__ dst,
                                                     int64_t ldd, int64_t M, int G, unsigned b0) {
  const int nch = (G + 1 + 3) / 4;   // destination chunks covering columns 0 .. G
  const int64_t n = M * nch;
  for (int64_t e = (int64_t)(blockIdx.x - b0) * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)(gridDim.x - b0) * blockDim.x) {
    const int64_t r = e / nch;
    const int k = (int)(e - r * nch);
    const float* sr = src + r * lds;
    float* dr = dst + r * ldd;
    if (k == 0) {
      for (int c = 1; c < 4 && c <= G; ++c) dr[c] = sr[c - 1];
      continue;
    }
    const int c0 = 4 * k - 1;          // source column of the chunk's first element
    // the source chunks k - 1 and k (16-B aligned; chunk k's columns past G lie inside the source row and are dropped)
    const float4 prev = *reinterpret_cast<const float4*>(sr + 4 * k - 4);
    const float4 cur = 4 * k < G ? *reinterpret_cast<const float4*>(sr + 4 * k) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v;
    v.x = prev.w;
    v.y = c0 + 1 < G ? cur.x : 0.f;
    v.z = c0 + 2 < G ? cur.y : 0.f;
    v.w = c0 + 3 < G ? cur.z : 0.f;
    *reinterpret_cast<float4*>(dr + 4 * k) = v;
  }
}

// backward: writes d sdf into column 0 of dOut rows (centre + taps) (overwrite), plus the centre rows' own sdf
// gradient (dsdf) and, in the blocks past tap_blocks, the geo-feature gradient into columns 1..G of the centre rows
// (copy_cols)
__global__ void taps_combine_bwd_kernel(const float* __restrict__ grads, const float* __restrict__ dgrads,
                                        const float* __restrict__ dhess, const float* __restrict__ dnormals,
                                        int64_t M, float four_delta, float delta_sq, float* __restrict__ dout,
                                        int64_t lddo, const float* __restrict__ dsdf, int64_t ldds,
                                        const float* __restrict__ dgeo, int64_t ldg, int G, unsigned tap_blocks) {
  if (blockIdx.x >= tap_blocks) {
    const bool vec = dgeo != nullptr && ((uintptr_t)dout & 15) == 0 && lddo % 4 == 0 && lddo >= 4 * ((G + 4) / 4) &&
                     ((uintptr_t)dgeo & 15) == 0 && ldg % 4 == 0 && ldg >= 4 * ((G + 3) / 4);
    if (vec) copy_cols_shift1_vec(dgeo, ldg, dout, lddo, M, G, tap_blocks);
    else copy_cols_any(dgeo, ldg, dout + 1, lddo, M, G, tap_blocks);
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)tap_blocks * blockDim.x) {
    float dg[3] = {0.f, 0.f, 0.f};
    if (dgrads) {
#pragma unroll
      for (int c = 0; c < 3; ++c) dg[c] = dgrads[i * 3 + c];
    }
    if (dnormals) {
      const float g0 = grads[i * 3], g1 = grads[i * 3 + 1], g2 = grads[i * 3 + 2];
      const float n = sqrtf(g0 * g0 + g1 * g1 + g2 * g2);
      if (n > 1e-12f) {
        const float d0 = dnormals[i * 3], d1 = dnormals[i * 3 + 1], d2 = dnormals[i * 3 + 2];
        const float dot = (d0 * g0 + d1 * g1 + d2 * g2) / (n * n);
        dg[0] += (d0 - dot * g0) / n;
        dg[1] += (d1 - dot * g1) / n;
        dg[2] += (d2 - dot * g2) / n;
      } else {
        dg[0] += dnormals[i * 3] / 1e-12f;
        dg[1] += dnormals[i * 3 + 1] / 1e-12f;
        dg[2] += dnormals[i * 3 + 2] / 1e-12f;
      }
    }
    float dh = 0.f;
    if (dhess) dh = (dhess[i * 3] + dhess[i * 3 + 1] + dhess[i * 3 + 2]) / 3.0f / delta_sq;
    dout[i * lddo] = dsdf ? -2.0f * dh + dsdf[i * ldds] : -2.0f * dh;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float ds = (kTap[t][0] * dg[0] + kTap[t][1] * dg[1] + kTap[t][2] * dg[2]) / four_delta + 0.5f * dh;
      dout[((t + 1) * M + i) * lddo] = ds;
    }
  }
}

// ---------------------------------------------------------------- spherical harmonics (degree 4, 25): sh25 in sh.h
// d/d(x,y,z) of sum_k dsh[k] * sh_k
__device__ __forceinline__ void sh25_bwd(float x, float y, float z, const float* d, float* g) {
  const float xx = x * x, yy = y * y, zz = z * z;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  const float c1 = 0.4886025119029199f;
  gy += d[1] * c1; gz += d[2] * c1; gx += d[3] * c1;
  const float c2 = 1.0925484305920792f;
  gx += d[4] * c2 * y; gy += d[4] * c2 * x;
  gy += d[5] * c2 * z; gz += d[5] * c2 * y;
  gz += d[6] * 0.9461746957575601f * 2 * z;
  gx += d[7] * c2 * z; gz += d[7] * c2 * x;
  gx += d[8] * 0.5462742152960396f * 2 * x; gy -= d[8] * 0.5462742152960396f * 2 * y;
  { const float c = 0.5900435899266435f; gx += d[9] * c * y * 6 * x; gy += d[9] * c * (3 * xx - 3 * yy); }
  { const float c = 2.890611442640554f; gx += d[10] * c * y * z; gy += d[10] * c * x * z; gz += d[10] * c * x * y; }
  { const float c = 0.4570457994644658f; gy += d[11] * c * (5 * zz - 1); gz += d[11] * c * y * 10 * z; }
  { const float c = 0.3731763325901154f; gz += d[12] * c * (15 * zz - 3); }
  { const float c = 0.4570457994644658f; gx += d[13] * c * (5 * zz - 1); gz += d[13] * c * x * 10 * z; }
  { const float c = 1.445305721320277f; gz += d[14] * c * (xx - yy); gx += d[14] * c * z * 2 * x; gy -= d[14] * c * z * 2 * y; }
  { const float c = 0.5900435899266435f; gx += d[15] * c * (3 * xx - 3 * yy); gy += d[15] * c * x * (-6 * y); }
  { const float c = 2.5033429417967046f; gx += d[16] * c * y * (3 * xx - yy); gy += d[16] * c * x * (xx - 3 * yy); }
  { const float c = 1.7701307697799304f; gx += d[17] * c * y * z * 6 * x; gy += d[17] * c * z * (3 * xx - 3 * yy);
    gz += d[17] * c * y * (3 * xx - yy); }
  { const float c = 0.9461746957575601f; gx += d[18] * c * y * (7 * zz - 1); gy += d[18] * c * x * (7 * zz - 1);
    gz += d[18] * c * x * y * 14 * z; }
  { const float c = 0.6690465435572892f; gy += d[19] * c * (7 * zz - 3); gz += d[19] * c * y * 14 * z; }
  { const float c = 0.10578554691520431f; gz += d[20] * c * (140 * zz * z - 60 * z); }
  { const float c = 0.6690465435572892f; gx += d[21] * c * z * (7 * zz - 3); gz += d[21] * c * x * (21 * zz - 3); }
  { const float c = 0.47308734787878004f; gx += d[22] * c * 2 * x * (7 * zz - 1); gy -= d[22] * c * 2 * y * (7 * zz - 1);
    gz += d[22] * c * (xx - yy) * 14 * z; }
  { const float c = 1.7701307697799304f; gx += d[23] * c * z * (3 * xx - 3 * yy); gy += d[23] * c * x * z * (-6 * y);
    gz += d[23] * c * x * (xx - 3 * yy); }
  { const float c = 0.4425326924449826f; gx += d[24] * c * (4 * xx * x - 12 * x * yy); gy += d[24] * c * (4 * yy * y - 12 * xx * y); }
  g[0] = gx; g[1] = gy; g[2] = gz;
}

// Radiance panel [M, ld]: [pos 3 | SH 25 | geo 256 | ndv 1 | grid 32 (hashgrid kernel)]
// pos rows i; direction per ray = dirs[i / S]; normals [M, 3]; geo from geometry-MLP output rows i, cols 1..256.
// Blocks [0, row_blocks): one thread per row writes x, SH(d) and n.v; the blocks after them copy the geo feature
// columns one element per thread (copy_cols: consecutive threads on consecutive columns, coalesced on both sides --
// a thread per row copying its own 256 columns touched 64 rows per instruction).
__global__ void rad_input_fwd_kernel(const float* __restrict__ pos, int64_t ldp, const float* __restrict__ dirs,
                                     const float* __restrict__ normals, const float* __restrict__ geo, int64_t ldg,
                                     int64_t M, int S, int G, float* __restrict__ X, int64_t ldx,
                                     unsigned row_blocks) {
  if (blockIdx.x >= row_blocks) {
    copy_cols_any(geo, ldg, X + 28, ldx, M, G, row_blocks);
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)row_blocks * blockDim.x) {
    const float* d = dirs + (i / S) * 3;
    float* row = X + i * ldx;
    row[0] = pos[i * ldp];
    row[1] = pos[i * ldp + 1];
    row[2] = pos[i * ldp + 2];
    float sh[25];
    sh25(d[0], d[1], d[2], sh);
#pragma unroll
    for (int k = 0; k < 25; ++k) row[3 + k] = sh[k];
    row[28 + G] = ndv3(normals + i * 3, d);
  }
}

// dpos[i] += dX[i, 0:3] (+ dP from the grid); dgeo rows <- dX[:, 28:28+G]; ddirs[ray] += SH' + dndv * (-n)
// One wave per ray: lane = sample (S <= 64).
__global__ __launch_bounds__(256) void rad_input_bwd_kernel(const float* __restrict__ dX, int64_t lddx,
                                                            const float* __restrict__ dP, int64_t lddp,
                                                            const float* __restrict__ dirs,
                                                            const float* __restrict__ normals, int64_t R, int S, int G,
                                                            float* __restrict__ dpos, int64_t lddpos,
                                                            float* __restrict__ dgeo, int64_t lddg,
                                                            float* __restrict__ ddirs) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  float gd0 = 0.f, gd1 = 0.f, gd2 = 0.f;
  const float* d = dirs + ray * 3;
  if (lane < S) {
    const int64_t i = ray * S + lane;
    const float* dr = dX + i * lddx;
    if (dpos) {
      float* o = dpos + i * lddpos;
      o[0] += dr[0] + (dP ? dP[i * lddp] : 0.f);
      o[1] += dr[1] + (dP ? dP[i * lddp + 1] : 0.f);
      o[2] += dr[2] + (dP ? dP[i * lddp + 2] : 0.f);
    }
    if (dgeo) {
      float* gg = dgeo + i * lddg;
      for (int k = 0; k < G; ++k) gg[k] = dr[28 + k];
    }
    if (ddirs) {
      float g[3];
      sh25_bwd(d[0], d[1], d[2], dr + 3, g);
      const float dndv = dr[28 + G];
      const float* n = normals + i * 3;
      gd0 = g[0] - dndv * n[0];
      gd1 = g[1] - dndv * n[1];
      gd2 = g[2] - dndv * n[2];
    }
  }
  if (ddirs) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      gd0 += __shfl_xor(gd0, o);
      gd1 += __shfl_xor(gd1, o);
      gd2 += __shfl_xor(gd2, o);
    }
    if (lane == 0) {
      ddirs[ray * 3] += gd0;
      ddirs[ray * 3 + 1] += gd1;
      ddirs[ray * 3 + 2] += gd2;
    }
  }
}

// ---------------------------------------------------------------- background panels
// positions p = o + d * start (rows ray*S + s); contraction (L-inf, |p|>=1); X [M, 39] = [c, PE6(c)];
// D [M, ldd] at column offset dcol: [d, PE4(d)] (27)
__global__ void bg_input_fwd_kernel(const float* __restrict__ pos, int64_t M, const float* __restrict__ dirs, int S,
                                    float* __restrict__ X, int64_t ldx, float* __restrict__ D, int64_t ldd,
                                    int64_t dcol) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    float p[3] = {pos[i * 3], pos[i * 3 + 1], pos[i * 3 + 2]};
    const float mag = fmaxf(fmaxf(fabsf(p[0]), fabsf(p[1])), fabsf(p[2]));
    if (mag >= 1.0f) {
      const float s = 2.0f - (1.0f / mag);
#pragma unroll
      for (int c = 0; c < 3; ++c) p[c] = s * (p[c] / mag);
    }
    float* row = X + i * ldx;
#pragma unroll
    for (int c = 0; c < 3; ++c) row[c] = p[c];
#pragma unroll
    for (int c = 0; c < 3; ++c) pe_write(row, c, p[c], 6);
    const float* d = dirs + (i / S) * 3;
    float* dro = D + i * ldd + dcol;
#pragma unroll
    for (int c = 0; c < 3; ++c) dro[c] = d[c];
#pragma unroll
    for (int c = 0; c < 3; ++c) pe_write(dro, c, d[c], 4);
  }
}

// backward to raw positions (through contraction) and to ray directions (wave per ray, lane = sample)
__global__ __launch_bounds__(256) void bg_input_bwd_kernel(const float* __restrict__ pos, const float* __restrict__ X,
                                                           int64_t ldx, const float* __restrict__ dX, int64_t lddx,
                                                           const float* __restrict__ dirs,
                                                           const float* __restrict__ dD, int64_t lddd, int64_t dcol,
                                                           int64_t R, int S, float* __restrict__ dpos,
                                                           float* __restrict__ ddirs) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (ray >= R) return;
  float gd[3] = {0.f, 0.f, 0.f};
  if (lane < S) {
    const int64_t i = ray * S + lane;
    const float* xr = X + i * ldx;
    const float* dr = dX + i * lddx;
    float gc[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) gc[c] = dr[c] + pe_bwd(dr, c, xr[c], 6);
    if (dpos) {
      const float p[3] = {pos[i * 3], pos[i * 3 + 1], pos[i * 3 + 2]};
      const float ax = fabsf(p[0]), ay = fabsf(p[1]), az = fabsf(p[2]);
      const float mag = fmaxf(fmaxf(ax, ay), az);
      float gp[3];
      if (mag >= 1.0f) {
        // c = (2 - 1/m) p / m ; m = max|p_k| (argmax k*)
        const int ks = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
        const float s = 2.0f - 1.0f / mag;
        float dot = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) { gp[c] = gc[c] * s / mag; dot += gc[c] * p[c]; }
        // d/dm of (2 - 1/m) p / m = p (1/m^3 - (2 - 1/m)/m^2) = p (2/m^3 - 2/m^2)
        const float dm = dot * (2.0f / (mag * mag * mag) - 2.0f / (mag * mag));
        gp[ks] += dm * (p[ks] >= 0.f ? 1.f : -1.f);
      } else {
#pragma unroll
        for (int c = 0; c < 3; ++c) gp[c] = gc[c];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) dpos[i * 3 + c] = gp[c];
    }
    if (ddirs && dD) {
      const float* dd = dD + i * lddd + dcol;
      const float* d = dirs + ray * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) gd[c] = dd[c] + pe_bwd(dd, c, d[c], 4);
    }
  }
  if (ddirs && dD) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
      for (int c = 0; c < 3; ++c) gd[c] += __shfl_xor(gd[c], o);
    }
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) ddirs[ray * 3 + c] += gd[c];
    }
  }
}

}  // namespace

MMS_EXPORT int mms_geo_input_fwd(const float* pos, int64_t ldp, int64_t M, int ntaps, float delta, int F, float* X,
                                 int64_t ldx, void* stream) {
  const char* fn = "mms_geo_input_fwd";
  MMS_REQUIRE(ntaps == 0 || ntaps == 4, fn, "ntaps must be 0 or 4");
  MMS_REQUIRE(ldx >= 3 + 6 * F, fn, "panel too narrow");
  MMS_REQUIRE(F >= 0 && F <= 24, fn, "PE frequencies must be in [0, 24]");
  if (M == 0) return 0;
  const int64_t total = M * (1 + ntaps) * (3 + 6 * F);
  const dim3 grid(mms::grid_for(total, 256, 65536));
  if (total < ((int64_t)1 << 32) - (int64_t)grid.x * 256)   // (the grid-stride index stays below 2^32 too)
    hipLaunchKernelGGL(geo_input_fwd_kernel<uint32_t>, grid, dim3(256), 0, mms::as_stream(stream), pos, ldp, M, ntaps,
                       delta, F, X, ldx);
  else
    hipLaunchKernelGGL(geo_input_fwd_kernel<int64_t>, grid, dim3(256), 0, mms::as_stream(stream), pos, ldp, M, ntaps,
                       delta, F, X, ldx);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_geo_input_bwd(const float* X, int64_t ldx, const float* dX, int64_t lddx, const float* dP,
                                 int64_t lddp, int64_t M, int ntaps, int F, float* dpos, int64_t lddpos, void* stream) {
  const char* fn = "mms_geo_input_bwd";
  if (M == 0) return 0;
  if (ntaps <= 4) {
    hipLaunchKernelGGL(geo_input_bwd_lanes_kernel, dim3(mms::grid_for(M * 16, 256, INT32_MAX)), dim3(256), 0,
                       mms::as_stream(stream), X, ldx, dX, lddx, dP, lddp, M, ntaps, F, dpos, lddpos);
  } else {
    hipLaunchKernelGGL(geo_input_bwd_kernel, dim3(mms::grid_for(M, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                       X, ldx, dX, lddx, dP, lddp, M, ntaps, F, dpos, lddpos);
  }
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_taps_combine_fwd(const float* out, int64_t ldo, int64_t M, float four_delta, float delta_sq,
                                    float* grads, float* hess, float* normals, void* stream) {
  const char* fn = "mms_taps_combine_fwd";
  if (M == 0) return 0;
  hipLaunchKernelGGL(taps_combine_fwd_kernel, dim3(mms::grid_for(M, 256, 16384)), dim3(256), 0, mms::as_stream(stream),
                     out, ldo, M, four_delta, delta_sq, grads, hess, normals);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_taps_combine_bwd(const float* grads, const float* dgrads, const float* dhess, const float* dnormals,
                                    int64_t M, float four_delta, float delta_sq, float* dout, int64_t lddo,
                                    const float* dsdf, int64_t ldds, const float* dgeo, int64_t ldg, int G,
                                    void* stream) {
  const char* fn = "mms_taps_combine_bwd";
  if (M == 0) return 0;
  MMS_REQUIRE(G >= 0 && lddo >= G + 1, fn, "dout rows hold the sdf column and G geo columns");
  const unsigned tb = mms::grid_for(M, 256, 16384);
  const unsigned gb = G > 0 ? mms::grid_for(M * G, 256, 16384) : 0;
  hipLaunchKernelGGL(taps_combine_bwd_kernel, dim3(tb + gb), dim3(256), 0, mms::as_stream(stream), grads, dgrads, dhess,
                     dnormals, M, four_delta, delta_sq, dout, lddo, dsdf, ldds, dgeo, ldg, G, tb);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_rad_input_fwd(const float* pos, int64_t ldp, const float* dirs, const float* normals,
                                 const float* geo, int64_t ldg, int64_t M, int S, int G, float* X, int64_t ldx,
                                 void* stream) {
  const char* fn = "mms_rad_input_fwd";
  MMS_REQUIRE(ldx >= 29 + G, fn, "panel too narrow");
  if (M == 0) return 0;
  const unsigned rb = mms::grid_for(M, 256, 16384);
  const unsigned gb = G > 0 ? mms::grid_for(M * G, 256, 16384) : 0;
  hipLaunchKernelGGL(rad_input_fwd_kernel, dim3(rb + gb), dim3(256), 0, mms::as_stream(stream), pos, ldp, dirs, normals,
                     geo, ldg, M, S, G, X, ldx, rb);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_rad_input_bwd(const float* dX, int64_t lddx, const float* dP, int64_t lddp, const float* dirs,
                                 const float* normals, int64_t R, int S, int G, float* dpos, int64_t lddpos,
                                 float* dgeo, int64_t lddg, float* ddirs, void* stream) {
  const char* fn = "mms_rad_input_bwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  hipLaunchKernelGGL(rad_input_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), dX, lddx, dP, lddp, dirs, normals, R, S, G, dpos, lddpos, dgeo, lddg,
                     ddirs);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_bg_input_fwd(const float* pos, int64_t M, const float* dirs, int S, float* X, int64_t ldx, float* D,
                                int64_t ldd, int64_t dcol, void* stream) {
  const char* fn = "mms_bg_input_fwd";
  if (M == 0) return 0;
  hipLaunchKernelGGL(bg_input_fwd_kernel, dim3(mms::grid_for(M, 256, 16384)), dim3(256), 0, mms::as_stream(stream), pos,
                     M, dirs, S, X, ldx, D, ldd, dcol);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_bg_input_bwd(const float* pos, const float* X, int64_t ldx, const float* dX, int64_t lddx,
                                const float* dirs, const float* dD, int64_t lddd, int64_t dcol, int64_t R, int S,
                                float* dpos, float* ddirs, void* stream) {
  const char* fn = "mms_bg_input_bwd";
  MMS_REQUIRE(S >= 1 && S <= 64, fn, "samples per ray must be in [1, 64]");
  if (R == 0) return 0;
  // (an LDS-staged variant of this kernel -- each ray's rows copied column-contiguously first -- measured no faster on
  // the config-5 step, 545.2k vs 546.7k rays/s, gpurun_out r4a, and was removed)
  hipLaunchKernelGGL(bg_input_bwd_kernel, dim3(mms::grid_for(R * 64, 256, INT32_MAX)), dim3(256), 0,
                     mms::as_stream(stream), pos, X, ldx, dX, lddx, dirs, dD, lddd, dcol, R, S, dpos, ddirs);
  return mms::check_launch(fn);
}
