// Degree-4 real spherical harmonics (25 components) of a unit direction, shared by the radiance-panel kernels of
// encode.hip and hashgrid.hip (both include it before any fp-contract pragma, so both compile the same expressions the
// same way).  Reference: components_from_spherical_harmonics, /root/reference/src/utils/math.py:21-83 (the torch
// stand-in for tcnn's SphericalHarmonics).
#pragma once

__device__ __forceinline__ void sh25(float x, float y, float z, float* o) {
  // no contraction: the same products and sums in every kernel that includes this, whatever its own fp-contract
#pragma clang fp contract(off)
  const float xx = x * x, yy = y * y, zz = z * z;
  o[0] = 0.28209479177387814f;
  o[1] = 0.4886025119029199f * y;
  o[2] = 0.4886025119029199f * z;
  o[3] = 0.4886025119029199f * x;
  o[4] = 1.0925484305920792f * x * y;
  o[5] = 1.0925484305920792f * y * z;
  o[6] = 0.9461746957575601f * zz - 0.31539156525251999f;
  o[7] = 1.0925484305920792f * x * z;
  o[8] = 0.5462742152960396f * (xx - yy);
  o[9] = 0.5900435899266435f * y * (3 * xx - yy);
  o[10] = 2.890611442640554f * x * y * z;
  o[11] = 0.4570457994644658f * y * (5 * zz - 1);
  o[12] = 0.3731763325901154f * z * (5 * zz - 3);
  o[13] = 0.4570457994644658f * x * (5 * zz - 1);
  o[14] = 1.445305721320277f * z * (xx - yy);
  o[15] = 0.5900435899266435f * x * (xx - 3 * yy);
  o[16] = 2.5033429417967046f * x * y * (xx - yy);
  o[17] = 1.7701307697799304f * y * z * (3 * xx - yy);
  o[18] = 0.9461746957575601f * x * y * (7 * zz - 1);
  o[19] = 0.6690465435572892f * y * (7 * zz - 3);
  o[20] = 0.10578554691520431f * (35 * zz * zz - 30 * zz + 3);
  o[21] = 0.6690465435572892f * x * z * (7 * zz - 3);
  o[22] = 0.47308734787878004f * (xx - yy) * (7 * zz - 1);
  o[23] = 1.7701307697799304f * x * z * (xx - 3 * yy);
  o[24] = 0.4425326924449826f * (xx * (xx - 3 * yy) - yy * (3 * xx - yy));
}


// torch.sum(normals * -directions, dim=-1): the three products rounded, summed left to right (no fused multiply-add,
// as the reference's CPU reduction), identical in every kernel that writes or differentiates it
__device__ __forceinline__ float ndv3(const float* n, const float* d) {
#pragma clang fp contract(off)
  float v = n[0] * -d[0];
  v = v + n[1] * -d[1];
  v = v + n[2] * -d[2];
  return v;
}
