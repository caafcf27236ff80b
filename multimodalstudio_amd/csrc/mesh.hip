// Iso-surface extraction from a dense SDF grid (mesh export, /root/reference/src/evaluator_components/
// mesh_extractors.py:63 -> utils/marching_cubes.py:35 get_surface_sliding).  The reference triangulates with
// skimage's marching cubes, which is not available offline; here every grid cell is split into the 6 tetrahedra
// around its main diagonal (corner 0 -> corner 6) and each tetrahedron is triangulated (marching tetrahedra): the
// same zero level set, watertight across cells (neighbouring cells share face diagonals), with more triangles than
// marching cubes.  Triangles are oriented with their normal towards increasing SDF (outward).
//
// Grid: values [nx * ny * nz] f32, x-major (index (i * ny + j) * nz + k, point origin + spacing * (i, j, k)).
// Two passes: count triangles per cell, exclusive scan (caller), emit.  Every vertex lies on a grid edge between a
// point and a neighbour at a non-negative offset (1..7 = the offset's xyz bits), recorded as an edge key
// base_index * 8 + offset for vertex welding by the caller.
#include "common.h"

namespace {

// corner c of a cell: (c & 1 ^ (c >> 1 & 1), c >> 1 & 1, c >> 2 & 1) in the order 0:(0,0,0) 1:(1,0,0) 2:(1,1,0)
// 3:(0,1,0) 4:(0,0,1) 5:(1,0,1) 6:(1,1,1) 7:(0,1,1)
__constant__ int kCx[8] = {0, 1, 1, 0, 0, 1, 1, 0};
__constant__ int kCy[8] = {0, 0, 1, 1, 0, 0, 1, 1};
__constant__ int kCz[8] = {0, 0, 0, 0, 1, 1, 1, 1};
__constant__ int kTet[6][4] = {{0, 5, 1, 6}, {0, 1, 2, 6}, {0, 2, 3, 6}, {0, 3, 7, 6}, {0, 7, 4, 6}, {0, 4, 5, 6}};

struct Cell {
  float v[8];
  int64_t g[8];  // grid index of each corner
};

__device__ __forceinline__ Cell load_cell(const float* vals, int ny, int nz, int i, int j, int k) {
  Cell c;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int64_t gi = ((int64_t)(i + kCx[q]) * ny + (j + kCy[q])) * nz + (k + kCz[q]);
    c.g[q] = gi;
    c.v[q] = vals[gi];
  }
  return c;
}

__device__ __forceinline__ int tet_tris(const Cell& c, int t, float level) {
  int n = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) n += c.v[kTet[t][q]] < level;
  return (n == 0 || n == 4) ? 0 : (n == 2 ? 2 : 1);
}

__global__ void count_kernel(const float* __restrict__ vals, int nx, int ny, int nz, float level,
                             int32_t* __restrict__ counts) {
  const int64_t cells = (int64_t)(nx - 1) * (ny - 1) * (nz - 1);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cells; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % (nz - 1));
    const int j = (int)((e / (nz - 1)) % (ny - 1));
    const int i = (int)(e / ((int64_t)(nz - 1) * (ny - 1)));
    const Cell c = load_cell(vals, ny, nz, i, j, k);
    int n = 0;
#pragma unroll
    for (int t = 0; t < 6; ++t) n += tet_tris(c, t, level);
    counts[e] = n;
  }
}

struct Vtx {
  float p[3];
  int64_t key;
};

__device__ __forceinline__ Vtx edge_vertex(const Cell& c, int a, int b, float level, const float* origin,
                                           const float* spacing, int i, int j, int k) {
  // order the edge from the lower to the upper grid point (non-negative offset)
  if (c.g[a] > c.g[b]) { const int t = a; a = b; b = t; }
  const float va = c.v[a], vb = c.v[b];
  const float den = vb - va;
  const float w = den != 0.f ? (level - va) / den : 0.5f;
  Vtx v;
  const float pa[3] = {(float)(i + kCx[a]), (float)(j + kCy[a]), (float)(k + kCz[a])};
  const float pb[3] = {(float)(i + kCx[b]), (float)(j + kCy[b]), (float)(k + kCz[b])};
#pragma unroll
  for (int d = 0; d < 3; ++d) v.p[d] = origin[d] + spacing[d] * (pa[d] + w * (pb[d] - pa[d]));
  const int off = (kCx[b] - kCx[a]) | ((kCy[b] - kCy[a]) << 1) | ((kCz[b] - kCz[a]) << 2);
  v.key = c.g[a] * 8 + off;
  return v;
}

__device__ __forceinline__ void put_tri(Vtx v0, Vtx v1, Vtx v2, const float* out_dir, float* verts, int64_t* keys,
                                        int64_t slot) {
  // orient the normal towards increasing SDF (out_dir: inside centroid -> outside centroid)
  const float e1[3] = {v1.p[0] - v0.p[0], v1.p[1] - v0.p[1], v1.p[2] - v0.p[2]};
  const float e2[3] = {v2.p[0] - v0.p[0], v2.p[1] - v0.p[1], v2.p[2] - v0.p[2]};
  const float nrm[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
  if (nrm[0] * out_dir[0] + nrm[1] * out_dir[1] + nrm[2] * out_dir[2] < 0.f) { const Vtx t = v1; v1 = v2; v2 = t; }
  const Vtx vv[3] = {v0, v1, v2};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
#pragma unroll
    for (int d = 0; d < 3; ++d) verts[(slot * 3 + q) * 3 + d] = vv[q].p[d];
    keys[slot * 3 + q] = vv[q].key;
  }
}

__global__ void emit_kernel(const float* __restrict__ vals, int nx, int ny, int nz, float level, float ox, float oy,
                            float oz, float sx, float sy, float sz, const int64_t* __restrict__ offsets,
                            float* __restrict__ verts, int64_t* __restrict__ keys) {
  const int64_t cells = (int64_t)(nx - 1) * (ny - 1) * (nz - 1);
  const float origin[3] = {ox, oy, oz}, spacing[3] = {sx, sy, sz};
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cells; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % (nz - 1));
    const int j = (int)((e / (nz - 1)) % (ny - 1));
    const int i = (int)(e / ((int64_t)(nz - 1) * (ny - 1)));
    const Cell c = load_cell(vals, ny, nz, i, j, k);
    int64_t slot = offsets[e];
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      int in[4], out[4], ni = 0, no = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cq = kTet[t][q];
        if (c.v[cq] < level) in[ni++] = cq; else out[no++] = cq;
      }
      if (ni == 0 || no == 0) continue;
      float dir[3] = {0.f, 0.f, 0.f};
      for (int q = 0; q < no; ++q) { dir[0] += kCx[out[q]] / (float)no; dir[1] += kCy[out[q]] / (float)no; dir[2] += kCz[out[q]] / (float)no; }
      for (int q = 0; q < ni; ++q) { dir[0] -= kCx[in[q]] / (float)ni; dir[1] -= kCy[in[q]] / (float)ni; dir[2] -= kCz[in[q]] / (float)ni; }
#pragma unroll
      for (int d = 0; d < 3; ++d) dir[d] *= spacing[d];
      if (ni == 1 || no == 1) {
        const int apex = ni == 1 ? in[0] : out[0];
        const int* rest = ni == 1 ? out : in;
        const Vtx a = edge_vertex(c, apex, rest[0], level, origin, spacing, i, j, k);
        const Vtx b = edge_vertex(c, apex, rest[1], level, origin, spacing, i, j, k);
        const Vtx d = edge_vertex(c, apex, rest[2], level, origin, spacing, i, j, k);
        put_tri(a, b, d, dir, verts, keys, slot++);
      } else {
        // quad across the 4 edges in0-out0, in0-out1, in1-out1, in1-out0 (a cycle)
        const Vtx a = edge_vertex(c, in[0], out[0], level, origin, spacing, i, j, k);
        const Vtx b = edge_vertex(c, in[0], out[1], level, origin, spacing, i, j, k);
        const Vtx d = edge_vertex(c, in[1], out[1], level, origin, spacing, i, j, k);
        const Vtx f = edge_vertex(c, in[1], out[0], level, origin, spacing, i, j, k);
        put_tri(a, b, d, dir, verts, keys, slot++);
        put_tri(a, d, f, dir, verts, keys, slot++);
      }
    }
  }
}

}  // namespace

MMS_EXPORT int mms_iso_count(const float* vals, int nx, int ny, int nz, float level, int32_t* counts, void* stream) {
  const char* fn = "mms_iso_count";
  MMS_REQUIRE(nx >= 2 && ny >= 2 && nz >= 2, fn, "grid needs >= 2 points per axis");
  MMS_REQUIRE(vals && counts, fn, "null pointer");
  const int64_t cells = (int64_t)(nx - 1) * (ny - 1) * (nz - 1);
  hipLaunchKernelGGL(count_kernel, dim3(mms::grid_for(cells, 256, 65536)), dim3(256), 0, mms::as_stream(stream), vals,
                     nx, ny, nz, level, counts);
  return mms::check_launch(fn);
}

MMS_EXPORT int mms_iso_emit(const float* vals, int nx, int ny, int nz, float level, const float* origin,
                            const float* spacing, const int64_t* offsets, float* verts, int64_t* keys, void* stream) {
  const char* fn = "mms_iso_emit";
  MMS_REQUIRE(nx >= 2 && ny >= 2 && nz >= 2, fn, "grid needs >= 2 points per axis");
  MMS_REQUIRE(vals && origin && spacing && offsets && verts && keys, fn, "null pointer");
  const int64_t cells = (int64_t)(nx - 1) * (ny - 1) * (nz - 1);
  hipLaunchKernelGGL(emit_kernel, dim3(mms::grid_for(cells, 256, 65536)), dim3(256), 0, mms::as_stream(stream), vals,
                     nx, ny, nz, level, origin[0], origin[1], origin[2], spacing[0], spacing[1], spacing[2], offsets,
                     verts, keys);
  return mms::check_launch(fn);
}
