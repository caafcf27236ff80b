/*
 * mms_hip.h — C ABI of libmms_hip.so, the MI355X (gfx950) kernels of MultimodalStudio's per-ray
 * training hot path.  This is the drop-in boundary: the reference's Python plugin classes
 * (Encoding / FieldComponent / fields / samplers / renderer, /root/reference/src) bind it through
 * ctypes (multimodalstudio_amd/_lib.py; INTEGRATION.md shows the stubs a maintainer would add).
 *
 * Conventions:
 *   - every pointer is a device pointer to fp32 (or int) memory owned by the caller (PyTorch);
 *     row-major matrices take an explicit leading dimension (elements);
 *   - `stream` is a hipStream_t passed as void*; calls are stream-ordered, never synchronise and
 *     never allocate (graph-capturable);
 *   - return 0 on success, negative on error; mms_last_error() gives the thread-local message;
 *   - "accumulate" outputs (+=) are marked; the library never owns parameters.
 *
 * Each entry point names the reference interface it replaces (file:line under /root/reference/src).
 */
#ifndef MMS_HIP_H
#define MMS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* mms_version(void);
const char* mms_last_error(void);

/* ---- multires hash grid: HashEncoding (field_components/encodings.py:184-310) inside FeatureGrid
 * (field_components/feature_structures.py:78-88).  pos [M, ldx] (cols 0..2), table [L*2^log2T, F=2],
 * scales [L] host array (floor(min_res*g^l)), out [M, ldo] cols 0..2L-1.  Levels >= active_levels are
 * zero (coarse-to-fine mask).  bwd: dtable += (atomic), dpos[:, 0:3] += (either may be NULL).
 * radius r > 0: pos is the FeatureGrid input, x_hat = (x + r) / (2 r); r = 0: pos is already x_hat (a bare
 * HashEncoding.forward, encodings.py:263-304).
 * interp: 0 = "Linear" (trilinear weights frac / 1 - frac: the reference torch path, parity-pinned); 1 = "Smoothstep"
 * (HashEncodingConfig.interpolation, encodings.py:64-67, the tcnn default: weights S(frac) = frac^2 (3 - 2 frac),
 * position gradient through S'(frac) = 6 frac (1 - frac); tcnn is absent here, so this mode is parity-unpinned). */
int mms_hashgrid_fwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L, int log2T, int F,
                     int interp, const float* scales, float radius, int active_levels, float* out, int64_t ldo, void* stream);
/* Forward over Mg groups of `group` rows (row = g + j * gstride, j < group; group 1 or 5): the SDF batch
 * [centre | 4 taps] (surface_model.py:138-160) gathered in (sample, tap) order, so a sample's centre and taps --
 * which share cells at the coarse levels -- hit one L2.  Same values as mms_hashgrid_fwd on every row. */
int mms_hashgrid_fwd_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                             const float* table, int L, int log2T, int F, int interp, const float* scales,
                             float radius, int active_levels, float* out, int64_t ldo, void* stream);
int mms_hashgrid_bwd(const float* pos, int64_t M, int64_t ldx, const float* table, int L, int log2T, int F,
                     int interp, const float* scales, float radius, int active_levels, const float* dout, int64_t ldd,
                     float* dtable, float* dpos, int64_t lddx, void* stream);
/* Same, for Mg groups of `group` rows (row = g + j * gstride, j < group; group 1 or 5): the SDF batch
 * [centre | 4 taps] (surface_model.py:138-160) -- the taps' shared-cell corner gradients are merged
 * in-thread before the table atomics. */
int mms_hashgrid_bwd_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                             const float* table, int L, int log2T, int F, int interp, const float* scales,
                             float radius, int active_levels, const float* dout, int64_t ldd, float* dtable,
                             float* dpos, int64_t lddx, void* stream);
/* The position gradient alone (dpos[:, 0:3] +=), as a forward-style gather (thread per (point, level)): with
 * mms_hashgrid_bwd_grouped(dtable, dpos = NULL) the same two gradients in two launches, the table walk then free of
 * table loads.  Same arguments and grouping as mms_hashgrid_bwd_grouped. */
int mms_hashgrid_dpos_grouped(const float* pos, int64_t Mg, int group, int64_t gstride, int64_t ldx,
                              const float* table, int L, int log2T, int F, int interp, const float* scales,
                              float radius, int active_levels, const float* dout, int64_t ldd, float* dpos,
                              int64_t lddx, void* stream);
/* The SDF field's MLP input panel in one launch: rows [x(3) | PE(6 pe_freqs) | hash grid(2L)] of ldx floats, for the M
 * centre positions cpos [M, ldp] and (ntaps = 4) their tap points centre + k_t delta, rows t * M + i (t = 0 centre).
 * Replaces SDFField.forward's input stage (surface_field.py:99-116: NeRFEncoding encodings.py:161-182 + FeatureGrid
 * feature_structures.py:78-83 + the 4-tap points of surface_model.py:137-153); the same values as mms_geo_input_fwd
 * followed by mms_hashgrid_fwd_grouped. */
int mms_sdf_panel_fwd(const float* cpos, int64_t ldp, int64_t M, int ntaps, float delta, int pe_freqs,
                      const float* table, int L, int log2T, int F, int interp, const float* scales, float radius,
                      int active_levels, float* X, int64_t ldx, void* stream);

/* mms_sdf_panel_fwd (ntaps 0) of the start positions of the samples of uniform spacing bins [R, nb] (ldb) on rays
 * (nears, fars, origins [R, 3], dirs [R, 3]): row r (nb - 1) + k is the point o_r + d_r (f_r b_k + n_r (1 - b_k)),
 * the positions mms_samples_fwd writes (SpacingToEuclidean + RaySamples.get_positions, ray_samplers.py:89-116,
 * rays.py:69-81), bit for bit.  The NeuS sampler's inference batches (ray_samplers.py:448-514: sdf_fn(ray_samples))
 * in one launch instead of two. */
int mms_sdf_panel_rays_fwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars,
                           const float* origins, const float* dirs, int64_t R, int pe_freqs, const float* table, int L,
                           int log2T, int F, int interp, const float* scales, float radius, int active_levels, float* X,
                           int64_t ldx, void* stream);

/* The radiance field's MLP input panel in one launch: rows [x(3) | SH(25) of dirs[i / S] | geo [M, G] (ldg) | n.v of
 * normals [M, 3] and -dirs | hash grid(2L)] of ldx floats.  Replaces RadianceModel.forward's input stage
 * (radiance_model.py:94-151: SHEncoding encodings.py:368-392, n.v, RadianceField radiance_field.py:72-77 +
 * FeatureGrid feature_structures.py:78-83); the same values as mms_rad_input_fwd followed by mms_hashgrid_fwd. */
int mms_rad_panel_fwd(const float* pos, int64_t ldp, const float* dirs, const float* normals, const float* geo,
                      int64_t ldg, int64_t M, int S, int G, const float* table, int L, int log2T, int F, int interp,
                      const float* scales, float radius, int active_levels, float* X, int64_t ldx, void* stream);

/* ---- MLP GEMM engine (field_components/mlp.py:152-171): C = epilogue(op(A) op(B)^T).
 * trans_a = 0: A is [M, K] (lda); 1: A is stored [K, M].  trans_b = 0: B is [N, K]; 1: B is stored [K, N].
 * prec 0 = exact fp32 MFMA, 1 = bf16 MFMA (fp32 accumulate), 2 = split bf16x3 (near-fp32 operands).
 * Epilogue: v = acc + bias[n]; Z[m,n] = v (optional); v = act(v); v *= dact'(aux[m,n]) (optional);
 * C = v or C += v (accumulate; atomic when splits > 1).  act/dact: 0 none, 1 ReLU, 2 Softplus(beta,thr),
 * 3 Sigmoid; dact 4 = Sigmoid' from the forward OUTPUT (aux = y; ReLU' is the same from y, id 1).  ones_col >= 0 also writes 1.0 at column ones_col of every output row. */
int mms_gemm(int prec, int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
             const float* B, int64_t ldb, float* C, int64_t ldc, const float* bias, float* Z, int64_t ldz,
             const float* aux, int64_t ldaux, int act, int dact, float beta, float thr, int accumulate, int splits,
             int ones_col, float* colsum, void* stream);
/* The weight gradients of up to 5 layers in ONE launch (the layers of one MLP after its fused backward): for each
 * item i, C_i[M_i, N_i] += A_i^T B_i with A_i stored [K_i, M_i] (dZ, lda_i) and B_i stored [K_i, N_i] (X, ldb_i),
 * K_i = rows, plus colsum_i[m] += sum_k A_i[k][m] (the bias gradient) when colsum (or colsum[i]) is non-null.
 * Replaces the per-layer mms_gemm(trans_a = trans_b = 1, ...) calls of the nn.Linear weight gradients
 * (field_components/mlp.py:152-171 under autograd); the K slices (split-K, float atomics) are sized per item for
 * about target_blocks blocks in all. */
int mms_gemm_tn_grouped(int prec, int n, const int64_t* M, const int64_t* N, const int64_t* K,
                        const float* const* A, const int64_t* lda, const float* const* B, const int64_t* ldb,
                        float* const* C, const int64_t* ldc, float* const* colsum, int target_blocks, void* stream);

/* The same weight gradients with 256 x 256 output tiles (blocks of 8 waves, every operand row read once per K slice),
 * bf16 (prec 1) or split bf16x3 (prec 2) operands, 16-B aligned operand rows; stage_rows = 16 or 32 rows per LDS
 * stage (72 / 144 KB of LDS for split bf16x3).  workspace (scratch, >= blocks x 65536 floats, blocks <= target_blocks
 * + 16): the K slices' partial tiles are stored there and summed by a second launch in slice order instead of being
 * added with float atomics; NULL (or too small): atomics.  Same reference interface as mms_gemm_tn_grouped. */
int mms_gemm_tn_wide(int prec, int n, const int64_t* M, const int64_t* N, const int64_t* K, const float* const* A,
                     const int64_t* lda, const float* const* B, const int64_t* ldb, float* const* C,
                     const int64_t* ldc, float* const* colsum, int target_blocks, int stage_rows, float* workspace,
                     int64_t workspace_floats, void* stream);
/* The same weight gradients with fp16 operands where the producers stored them (preset fast_h16c; fp32 accumulate: the
 * reference GPU's fp16-autocast nn.Linear backward, trainer.py:51,57-62), items of mixed modes in ONE launch:
 *  - ainv[i] non-NULL: A_i = the dZ rows as mms_mlp_chain prec 6 stores them (fp16 [K_i rows][lda_i], 8-B aligned, row
 *    k scaled by 1 / ainv_i[k]; ainv 0 for an all-zero row), emax[i] = that launch's largest biased row exponent;
 *    each A row rescaled by ainv_i[k] 2^(14 - e_max) <= 1 to one common scale (the largest |dZ| at 2^14: the
 *    reference's loss-scaled fp16 dZ) and rounded to fp16, B_i rounded to fp16 (the autocast's fp16 activations), the
 *    common scale undone on the fp32 accumulators: one fp16 MFMA per product;
 *  - ainv NULL (or ainv[i] NULL): A_i fp32 rows (16-B aligned), split bf16x3 as mms_gemm_tn_wide;
 *  - b16[i] non-zero: B_i holds fp16 rows (8-B aligned, ldb in halves), else fp32 rows (16-B aligned).
 * colsum_i[m] += sum_k dZ_i[k][m] (the bias gradient). */
int mms_gemm_tn_wide16(int n, const int64_t* M, const int64_t* N, const int64_t* K, const void* const* A,
                       const int64_t* lda, const float* const* ainv, const unsigned* const* emax, const void* const* B,
                       const int64_t* ldb, const int* b16, float* const* C, const int64_t* ldc, float* const* colsum,
                       int target_blocks, void* stream);

/* ---- fused MLP chains (MLP.forward mlp.py:152-171 under weight norm :206-209, all layers in one launch) for the
 * SDF field (71-256-256-257, Softplus(100), surface_field.py:99-116), the radiance field (317-256-256-256, ReLU,
 * radiance_field.py:72-77) and the background NeRF (n_layers = 4: base 39-256-256-256-256 and head
 * 283-256-256-256-128, ReLU, nerf_field.py:92-105).  Layers are computed transposed so each layer's MFMA
 * accumulator feeds the next layer from registers.  prec 1 = bf16, 2 = split bf16x3 operands (fp32 accumulate),
 * 3 = split activations x bf16 weights (SDF), 5 = fp16 operands (forward radiance / head / background chains: the
 * reference GPU's fp16 autocast precision, trainer.py:51; fp16-packed weights, permute bit 2), 6 = backward only:
 * the first layer (B = dY from memory) split bf16x3 (a_lo[0] required), the register-fed layers on fp16 operands with
 * a per-row power-of-two scale (each row's largest |dZ| to [2^13, 2^14), undone on the fp32 accumulators) -- the
 * reference's fp16 autocast backward without a global loss scale; layers >= 1 packed as for prec 5.
 * Per-layer arrays (a_hi, a_lo, bias, aux, ldaux, out, ldo, N, act) have n_layers entries.
 * Forward (backward = 0): out[l] = act_l(X_l W_l^T + b_l) (the hidden outs are stored together or, 3 layers, not at
 *   all); rows >= rows_full compute / store only output column 0 of the last layer (the SDF taps), in fp32 from
 *   w2row0 = the last layer's fp32 weight row 0 (required when rows_full < M).  With rows_full = 0 the last
 *   layer's out may have any pitch >= 1 (e.g. a dense [M] sdf vector).
 * Backward-data (backward = 1): X = dY of the last forward layer (rows >= rows_full: column 0 only), optionally
 *   scaled by act'(xaux) (stored to xout); out[l] = (prev . W^T) * act_l'(aux[l]) with act' evaluated from the
 *   forward output aux[l] (NULL: no scaling); the last out = dX.
 * SDF backward only (3 layers, Softplus, rows_full < M): tap_part [ceil(M / B) - rows_full / B][ld_tap > N[0]]
 *   (B = mms_mlp_chain_block_rows()) receives one row per B-row block holding rows >= rows_full: that block's share of
 *   the last forward layer's
 *   weight-gradient row 0, sum over its rows >= rows_full of X[m, 0] * aux[0][m, :] (columns < N[0]), and of the bias
 *   gradient, sum of X[m, 0] (column N[0]) -- the taps' sdf column, surface_model.py:137-153 (reduce with
 *   mms_rowsum_add); NULL: not computed.
 * prec 6 backward, hidden layers l < n_layers - 1: rinv[l] non-NULL stores out[l] as fp16 [rows][ldo] (8-B aligned,
 *   ldo >= 32 ceil(N/32)) holding the ROW-SCALED dZ the next layer's fp16 operands are made of (each row's largest
 *   |dZ| in [2^13, 2^14)), rinv[l][row] = the row's inverse scale 2^(e - 14) (0 for an all-zero row), and
 *   atomically raises emax[l] to the
 *   largest e + 1000 of its rows (emax zeroed by the caller; 0 = every row zero): the fp16 weight-gradient operands of
 *   mms_gemm_tn_wide16.  rinv NULL (or rinv[l] NULL): fp32 dZ as before.
 * f16 (NULL: none): per layer, hidden layers l < n_layers - 1 only -- forward: out[l] holds fp16 activation rows
 *   (8-B aligned, ldo >= 32 ceil(N/32)), the reference autocast's fp16 activations; backward: aux[l] is such an fp16
 *   row buffer (act' evaluated from the fp16 values). 
 * a_hi / a_lo: per-layer packed weights from mms_mlp_pack (bf16, 32 ceil(N/32) x 16 ceil(K/16)); layers >= 1 are
 * register-fed and must be packed with permute = 1.  All row pitches multiples of 4 floats, 16-B aligned. */
/* Rows per mms_mlp_chain block (128; 64 in a build with two blocks per CU): the tap_part row granularity. */
int mms_mlp_chain_block_rows(void);
int mms_mlp_chain(int prec, int backward, int n_layers, const float* X, int64_t ldx, int K0, int64_t M,
                  int64_t rows_full, const float* xaux, int64_t ldxaux, int xact, float* xout, int64_t ldxout,
                  const void* const* a_hi, const void* const* a_lo, const float* const* bias, const float* const* aux,
                  const int64_t* ldaux, float* const* out, const int64_t* ldo, const int* N, const int* act,
                  float beta, float thr, const float* w2row0, float* tap_part, int64_t ld_tap, float* const* rinv,
                  unsigned* emax, const int* f16, void* stream);
/* bf16 (hi, and lo = residual if non-NULL) image of W [N, K] (ldw) as an MFMA A operand of rows x cols:
 * transpose = 0 -> A = W, 1 -> A = W^T; permute bit 0 stores each k-step in register-fed order (columns 0-3, 8-11,
 * 4-7, 12-15 of a 16-column step); bit 2 writes an fp16 image (hi only, fp16 bits in the 16-bit buffer:
 * mms_mlp_chain prec 5).  Zero padded; rows % 32 == 0, cols % 16 == 0.  Fragment-major: the fragment of (k-step s, row tile t) is
 * one 1 KiB block at element ((s * tiles + t) * 64 + lane) * 8. */
int mms_mlp_pack(const float* W, int64_t N, int64_t K, int64_t ldw, int transpose, int permute, int64_t rows,
                 int64_t cols, void* hi, void* lo, void* stream);

/* ---- batched weight preparation: every weight-normed layer of a model (and every packed MMA image of them) in one
 * launch each, once per step (the item tables live in device memory; row0 / elem0 = the item's first block row /
 * element in the concatenation, items in increasing order).  Same arithmetic as mms_weight_norm_fwd /
 * mms_mlp_pack per item. */
typedef struct {
  const float* g;
  const float* v;
  int64_t N, K;
  float* W;
  int64_t ldw;
  float* norms;
  int64_t row0;
} MmsNormItem;
typedef struct {
  const float* W;
  int64_t N, K, ldw;
  int64_t transpose, permute;
  int64_t rows, cols;
  void* hi;
  void* lo;
  int64_t elem0;
} MmsPackItem;
int mms_weight_norm_fwd_batched(const void* items, int n_items, int64_t total_rows, void* stream);
/* a backward's weight-norm gradients (dg += , dv += as mms_weight_norm_bwd), up to 32 layers per launch; items is a
 * HOST array (copied into the kernel arguments). */
typedef struct {
  const float* g;
  const float* v;
  const float* norms;
  int64_t N, K;
  const float* dW;
  int64_t lddw;
  float* dg;
  float* dv;
  int64_t row0;
} MmsWnBwdItem;
int mms_weight_norm_bwd_batched(const void* items, int n_items, int64_t total_rows, void* stream);
int mms_mlp_pack_batched(const void* items, int n_items, int64_t total, void* stream);

/* ---- weight norm (mlp.py:206-209; torch weight_norm dim=0): W = v * (g / ||v||_row); bwd dg += , dv += */
int mms_weight_norm_fwd(const float* g, const float* v, int64_t N, int64_t K, float* W, int64_t ldw, float* norms,
                        void* stream);
int mms_weight_norm_bwd(const float* g, const float* v, const float* norms, int64_t N, int64_t K, const float* dW,
                        int64_t lddw, float* dg, float* dv, void* stream);
/* bias gradient: out[n] += sum_m A[m, n] */
int mms_colsum(const float* A, int64_t M, int64_t N, int64_t lda, float* out, void* stream);
/* dZ = dY * act'(Z)  (act 4: Sigmoid' from the output, Z = y) */
int mms_act_bwd(const float* dY, int64_t ldy, const float* Z, int64_t ldz, int64_t M, int64_t N, int act,
                float beta, float thr, float* dZ, int64_t lddz, void* stream);

/* ---- SDF-field input panel [x, PE(x)] (NeRFEncoding encodings.py:161-182; SDFField surface_field.py:99-116)
 * for the centre rows [0, M) and, with ntaps = 4, the 4 numerical-gradient taps x + k_t * delta
 * (SurfaceModel.gradient, surface_model.py:137-153) at rows [M (t+1), M (t+2)).  bwd: dpos += */
int mms_geo_input_fwd(const float* pos, int64_t ldp, int64_t M, int ntaps, float delta, int F, float* X, int64_t ldx,
                      void* stream);
int mms_geo_input_bwd(const float* X, int64_t ldx, const float* dX, int64_t lddx, const float* dP, int64_t lddp,
                      int64_t M, int ntaps, int F, float* dpos, int64_t lddpos, void* stream);
/* gradients / hessians / normals from the 5 SDF evaluations (surface_model.py:143-151, :91);
 * four_delta = 4 delta, delta_sq = delta^2.  bwd writes d sdf into column 0 of dout rows (all 5M). */
int mms_taps_combine_fwd(const float* out, int64_t ldo, int64_t M, float four_delta, float delta_sq, float* grads,
                         float* hess, float* normals, void* stream);
/* bwd also adds the centre rows' own d sdf (dsdf [M] with row stride ldds, may be NULL) into column 0 and writes the
 * geo-feature gradient dgeo [M, G] (ldg; NULL: zeros) into columns 1..G of the centre rows: dout is complete. */
int mms_taps_combine_bwd(const float* grads, const float* dgrads, const float* dhess, const float* dnormals,
                         int64_t M, float four_delta, float delta_sq, float* dout, int64_t lddo, const float* dsdf,
                         int64_t ldds, const float* dgeo, int64_t ldg, int G, void* stream);

/* ---- radiance input panel [x, SH4(d), geo, n.v, (grid)] (RadianceModel.forward radiance_model.py:94-151,
 * RadianceField radiance_field.py:72-77, SH utils/math.py:21-83).  One ray = S consecutive rows. */
int mms_rad_input_fwd(const float* pos, int64_t ldp, const float* dirs, const float* normals, const float* geo,
                      int64_t ldg, int64_t M, int S, int G, float* X, int64_t ldx, void* stream);
int mms_rad_input_bwd(const float* dX, int64_t lddx, const float* dP, int64_t lddp, const float* dirs,
                      const float* normals, int64_t R, int S, int G, float* dpos, int64_t lddpos, float* dgeo,
                      int64_t lddg, float* ddirs, void* stream);

/* ---- background NeRF inputs: L-inf SceneContraction (spatial_distortions.py:90-97), PE6(pos) -> X[:, 0:39],
 * PE4(dir) -> D[:, dcol:dcol+27] (NeRFField nerf_field.py:92-105).  bwd: dpos = , ddirs += */
int mms_bg_input_fwd(const float* pos, int64_t M, const float* dirs, int S, float* X, int64_t ldx, float* D,
                     int64_t ldd, int64_t dcol, void* stream);
int mms_bg_input_bwd(const float* pos, const float* X, int64_t ldx, const float* dX, int64_t lddx, const float* dirs,
                     const float* dD, int64_t lddd, int64_t dcol, int64_t R, int S, float* dpos, float* ddirs,
                     void* stream);

/* ---- NeuS alpha + transmittance weights (NeuSVolumeRendering volume_rendering.py:177-213), one wave per ray,
 * S <= 64.  bwd: dsdf = (strided), dgrads +=, ddirs +=, ddeltas +=, ds_param += (atomic). */
int mms_neus_weights_fwd(const float* sdf, int64_t lds, const float* grads, const float* dirs, const float* deltas,
                         const float* s_param, float cos_anneal, int64_t R, int S, float* alpha, float* weights,
                         void* stream);
int mms_neus_weights_bwd(const float* sdf, int64_t lds, const float* grads, const float* dirs, const float* deltas,
                         const float* s_param, float cos_anneal, int64_t R, int S, const float* alpha,
                         const float* dweights, float* dsdf, int64_t ldds, float* dgrads, float* ddirs,
                         float* ddeltas, float* ds_param, void* stream);
/* density -> alpha -> weights (RaySamples.get_alphas + get_weights_from_alphas, cameras/rays.py:138-217) */
int mms_density_weights_fwd(const float* density, int64_t ldd, const float* deltas, int64_t R, int S, float* alpha,
                            float* weights, void* stream);
int mms_density_weights_bwd(const float* density, int64_t ldd, const float* deltas, int64_t R, int S,
                            const float* alpha, const float* dweights, float* ddensity, int64_t lddd, float* ddeltas,
                            void* stream);
/* composite sum_s w c (+ bg (1 - sum w)), scattering compacted rays to rows idx[r] of out [nout, C]
 * (Renderer.render / RadianceRenderer renderers.py:75-174; BackgroundModel sum background_model.py:101-109); a ray
 * with idx[r] >= nout (the padding rays of a fixed-capacity batch) is discarded: no output row, zero gradients.
 * bwd: dvals and dw [R, S] are written (not accumulated); dbg[idx[r]] is written for hit rows.  The other rows:
 * with hit = null the caller pre-fills out = bg and dbg = dout; with hit [nout] (uint8, the collider's mask: 1 exactly
 * on the rows some ray of the batch lands on) the same launch writes out = bg / dbg = dout on the rows with hit 0. */
int mms_composite_fwd(const float* w, const float* vals, int64_t ldv, int C, const float* bg, int64_t R, int S,
                      const int64_t* idx, int64_t nout, const unsigned char* hit, float* out, void* stream);
int mms_composite_bwd(const float* w, const float* vals, int64_t ldv, int C, const float* bg, int64_t R, int S,
                      const int64_t* idx, int64_t nout, const unsigned char* hit, const float* dout, float* dvals,
                      int64_t lddv, float* dw, float* dbg, void* stream);
/* Accumulation / normals / depth renderers (renderers.py:176-242, no grad) of compacted rays scattered to rows idx[r]:
 * out [rows, ldo >= 5] = (sum w, sum w n, sum w mid) per hit row (other rows untouched), depth clipped to the range of
 * all sample midpoints; range [2] is scratch (order-preserving unsigned images of the extremes), zeros on entry. */
int mms_render_stats(const float* w, const float* normals, const float* starts, const float* ends, int64_t R, int S,
                     const int64_t* idx, float* out, int64_t ldo, float* range, void* stream);
/* the same for every modality of a batched hit set in one launch pair: segment m = rays [seg_off[m], seg_off[m+1])
 * (seg_off: HOST array of n_seg + 1 <= 9 offsets), its rays scatter to out rows m * seg_rows + sidx[r] (sidx: the
 * ray's row within its modality) and its depth clips to its own midpoint range (range [2 n_seg] scratch, zeros on
 * entry) -- one DepthRenderer call per modality's RayBundle (renderers.py:205-214, base_model.py:146-159). */
int mms_render_stats_segments(const float* w, const float* normals, const float* starts, const float* ends, int n_seg,
                              const int64_t* seg_off, int S, const int64_t* sidx, float* out, int64_t ldo,
                              int64_t seg_rows, float* range, void* stream);

/* dst_a[c] += sum_r src[r][c] for c < na and dst_b[c - na] += sum_r src[r][c] for na <= c < cols (src [rows][ld]):
 * the reduction of per-block partial rows (mms_mlp_chain's tap_part) into a weight-gradient row and its bias. */
int mms_rowsum_add(const float* src, int64_t rows, int64_t cols, int64_t ld, float* dst_a, int64_t na, float* dst_b,
                   void* stream);

/* ---- narrow weight-normed linear layers (C <= 16 outputs, K = 128 / 256 / 512 inputs): the background density head
 * (nerf_field.py:92-105, 256 -> 1 Softplus) and the 1-layer background modality heads (background_model.py:101-109,
 * field_heads.py:71-88, 128 -> C).  fwd: Y[m, c] = act(X[m] . W[c] + b[c]) (W [C, K] row-major, the weight-normed
 * weight; act 0 none, 1 ReLU, 2 Softplus(beta, thr), 3 Sigmoid).  bwd: dz = dY * act'(Y) (from the output);
 * dX = (or += with accumulate) dz W; dW += dz^T X; db += sum dz (dW, db, dX may be NULL).  fp32 VALU. */
int mms_small_linear_fwd(const float* X, int64_t ldx, int64_t M, int K, const float* W, const float* b, int C, int act,
                         float beta, float thr, float* Y, int64_t ldy, void* stream);
int mms_small_linear_bwd(const float* X, int64_t ldx, int64_t M, int K, const float* W, int C, int act, float beta,
                         float thr, const float* Y, int64_t ldy, const float* dY, int64_t lddy, float* dX,
                         int64_t lddx, int accumulate, float* dW, float* db, void* stream);

/* ---- PolarizationHead Stokes alignment + intensities (field_heads.py:90-106; polarizer.py:54-101).
 * stokes [M,3] (MLP output), dirs/ups per ray [M/S, 3]; out [M,4]; bwd dstokes =, ddirs +=, dups += */
int mms_polarizer_fwd(const float* stokes, const float* dirs, const float* ups, int64_t M, int S, float* out,
                      void* stream);
int mms_polarizer_bwd(const float* stokes, const float* dirs, const float* ups, int64_t R, int S, const float* dout,
                      float* dstokes, float* ddirs, float* dups, void* stream);

/* ---- samplers (model_components/ray_samplers.py) */
/* stratified jittered bins (SpacedSampler :209-221): lin [nb] host-computed torch.linspace values (device copy),
 * t [R, tcols] (tcols = 1 single jitter, nb per-bin jitter) or NULL (eval) */
int mms_stratified_bins(const float* lin, int nb, const float* t, int tcols, int64_t R, float* bins, void* stream);
/* spacing bins -> euclidean starts/ends/deltas/positions (spacing_to_euclidean_fn :178-181, rays.py:69-81,
 * 304-349); kind 0 uniform, 1 linear disparity.  bwd: d near/far/origins/dirs += */
int mms_samples_fwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars,
                    const float* origins, const float* dirs, int kind, int64_t R, float* starts, float* ends,
                    float* deltas, float* pos, void* stream);
int mms_samples_bwd(const float* bins, int64_t ldb, int nb, const float* nears, const float* fars, const float* dirs,
                    int kind, int64_t R, const float* dpos, const float* ddeltas, const float* dstarts,
                    float* dnears, float* dfars, float* dorigins, float* ddirs, void* stream);
/* one NeuS up-sampling iteration (NeuSSampler :480-511): sdf gather-merge, fixed-inv_s alpha (:516-551),
 * weights, PDF inverse CDF (PDFSampler :357-403), stable merge (merge_ray_samples :38-68). */
int mms_neus_step(int64_t R, int S, const float* bins, const float* sdf_prev, int s_prev, const float* sdf_new,
                  int n_prev_new, const int* prev_idx, const float* nears, const float* fars, float inv_s,
                  const float* rand, const float* u_lin, int n_new, float* sdf_out, float* new_bins,
                  float* merged_bins, int* sorted_idx, void* stream);

/* ---- rays (cameras/cameras.py:460-703, camera_utils.py:280-383, poses.py:53-67, ray_generators.py:54-81).
 * coords int [N, 3] = (camera, y, x); mats = camera_opt_to_camera [C or 1, 3, 4]; bwd dmats += (atomic). */
/* SO(3) x R^3 exponential map of the camera-pose deltas (lie_groups.py:28-63, camera_optimizers.py:86-119):
 * tangent [B, 6] = (t, w) -> mats [B, 3, 4] = [R(w) | t]; bwd adds d tangent [B, 6] from dmats [B, 3, 4] into dtangent. */
int mms_pose_exp_fwd(const float* tangent, int64_t B, float* mats, void* stream);
/* count[0] += the number of rays of coords [N, 3] whose ray (mms_raygen_fwd with the pose matrices exp(tangent [B, 6])
 * -- or the given mats [B, 3, 4] when tangent is null --, B <= 256) hits the sphere of mms_collider_fwd (count zeroed
 * by the caller), in one launch: the pose exp map, ray generation, collider and compaction count of the next step's
 * rays (the same device functions, so the count is the one the step's own compaction finds). */
int mms_count_hits(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx, const float* cy,
                   const float* c2w, const float* dist, const float* tangent, const float* mats, int B,
                   int mat_per_cam, float pixel_offset, float radius, int64_t* count, void* stream);
int mms_pose_exp_bwd(const float* tangent, const float* dmats, int64_t B, float* dtangent, void* stream);
int mms_raygen_fwd(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx, const float* cy,
                   const float* c2w, const float* dist, const float* mats, int mat_per_cam, float pixel_offset,
                   float* origins, float* dirs, float* ups, float* area, float* dnorm, void* stream);
int mms_raygen_bwd(const int* coords, int64_t N, const float* fx, const float* fy, const float* cx, const float* cy,
                   const float* c2w, const float* dist, const float* mats, int mat_per_cam, float pixel_offset,
                   const float* dorig, const float* ddirs, const float* dups, float* dmats, void* stream);
/* SphereCollider (scene_colliders.py:60-80) + background near/far (:107-113); mask uint8 */
int mms_collider_fwd(const float* origins, const float* dirs, int64_t N, float radius, float* nears, float* fars,
                     unsigned char* mask, float* bg_nears, float* bg_fars, void* stream);
int mms_collider_bwd(const float* origins, const float* dirs, int64_t N, float radius, const float* dnears,
                     const float* dfars, const float* dbg_nears, const float* dbg_fars, float* dorig, float* ddirs,
                     void* stream);
/* order-preserving mask compaction (TensorDataclass.__getitem__ with a bool mask, base_model.py:88-93) */
int mms_compact(const unsigned char* mask, int64_t N, int64_t* idx, int64_t* count, void* stream);
/* hit-ray gather of the compacted rays (base_model.py:88-93): (o, d, up [N,3], near, far [N]) rows idx[r] ->
 * [R,3] x 3, [R] x 2; bwd: dorig, ddirs, dups [N,3], dnears, dfars [N] += scatter of the five gradients (any input
 * gradient may be NULL; atomic: repeated indices allowed). */
int mms_hit_gather_fwd(const int64_t* idx, int64_t R, const float* o, const float* d, const float* u, const float* n,
                       const float* f, float* oh, float* dh, float* uh, float* nh, float* fh, void* stream);
int mms_hit_gather_bwd(const int64_t* idx, int64_t R, const float* doh, const float* ddh, const float* duh,
                       const float* dnh, const float* dfh, float* dorig, float* ddirs, float* dups, float* dnears,
                       float* dfars, void* stream);
/* fixed-capacity form for static-shape (graph-captured) steps: idx [N] buffer, its first cap entries are used;
 * rows [count, cap) are padding (gather index = first hit, scatter index sidx = N, a dummy row); count is
 * clamped to cap on the device.  sidx may be NULL. */
int mms_compact_padded(const unsigned char* mask, int64_t N, int64_t cap, int64_t* idx, int64_t* sidx,
                       int64_t* count, void* stream);
/* every modality's compaction in one launch (BaseModel runs all modalities' rays through the shared fields as one
 * batch, base_model.py:86-99 per modality): mask [n_seg N] = n_seg segments of N rays; segment m's hits are laid out
 * in rows [m cap, (m+1) cap) of gidx (global ray index; padding rows past min(hits, cap) repeat the segment's first
 * hit) and sidx (index within the segment; N for padding rows), count [n_seg] = min(hits, cap); scratch [n_seg N].
 * cap = N keeps every hit (dynamic-shape steps read count and use the first count rows of each segment). */
int mms_compact_segments(const unsigned char* mask, int n_seg, int64_t N, int64_t cap, int64_t* scratch, int64_t* gidx,
                         int64_t* sidx, int64_t* count, void* stream);

/* ---- losses (model_components/losses.py): L1 (+ SkipSaturation fill), eikonal, curvature; scalars on device */
int mms_l1_loss_fwd(const float* out, int64_t ldo, const float* tgt, int64_t N, int C, float sat_thr,
                    unsigned long long* first_scratch, float* loss, void* stream);
int mms_l1_loss_bwd(const float* out, int64_t ldo, const float* tgt, int64_t N, int C, float sat_thr,
                    const unsigned long long* first_scratch, const float* dloss, float scale, float* dout,
                    int64_t lddo, void* stream);
int mms_geo_loss_fwd(const float* grads, const float* hess, int64_t M, float inv_total, float* eik, float* curv,
                     void* stream);
int mms_geo_loss_bwd(const float* grads, const float* hess, int64_t M, float inv_total, const float* deik,
                     float eik_scale, const float* dcurv, float curv_scale, float* dgrads, float* dhess,
                     void* stream);
/* fixed-capacity batches (graph-captured steps): rows >= count[0] * S are padding and skipped, and the mean runs over
 * 1 / max(1, S * sum(counts_all[0 .. n_counts))) formed on the device, so no hit count reaches the host */
int mms_geo_loss_fwd_masked(const float* grads, const float* hess, int64_t M, int S, const int64_t* count,
                            const int64_t* counts_all, int n_counts, float* eik, float* curv, void* stream);
int mms_geo_loss_bwd_masked(const float* grads, const float* hess, int64_t M, int S, const int64_t* count,
                            const int64_t* counts_all, int n_counts, const float* deik, float eik_scale,
                            const float* dcurv, float curv_scale, float* dgrads, float* dhess, void* stream);

/* The step loss's terms in one launch each way (StepLossFunction, losses.py:224-265; graph-replayed steps): n_l1 L1
 * segments (mms_l1_loss_fwd / _bwd of out[i] [N[i], C[i]] (ldo[i]) against tgt[i], SkipSaturation threshold thr[i]
 * with the first_saturated index first[i] already formed, or null) and n_geo eikonal / curvature segments
 * (mms_geo_loss_*_masked of grads[j] / hess[j] (rows[j] rows, count[j] or null; 1 / M_total from counts_all, or
 * inv_total when counts_all is null)); fwd adds into loss[i], eik, curv; bwd adds d / d out into dout[i] (lddo[i]) and
 * d / d grads, d / d hess (scales: dloss eik_scale, dloss curv_scale) into dgrads[j], dhess[j].  Host arrays of
 * device pointers, at most 8 segments of each kind; the same arithmetic as the per-segment entry points. */
int mms_step_loss_fwd(int n_l1, const float* const* out, const int64_t* ldo, const float* const* tgt,
                      const int64_t* N, const int* C, const float* thr, const unsigned long long* const* first,
                      float* const* loss, int n_geo, const float* const* grads, const float* const* hess,
                      const int64_t* rows, int S, const int64_t* const* count, const int64_t* counts_all, int n_counts,
                      float inv_total, float* eik, float* curv, void* stream);
int mms_step_loss_bwd(int n_l1, const float* const* out, const int64_t* ldo, const float* const* tgt,
                      const int64_t* N, const int* C, const float* thr, const unsigned long long* const* first,
                      float* const* dout, const int64_t* lddo, int n_geo, const float* const* grads,
                      const float* const* hess, const int64_t* rows, int S, const int64_t* const* count,
                      const int64_t* counts_all, int n_counts, float inv_total, const float* dloss, float eik_scale,
                      float curv_scale, float* const* dgrads, float* const* dhess, void* stream);

/* out[0] = 1 / clip(exp(10 s[0]), 1e-6, 1e6): SingleVarianceNetwork's reported 1 / inv_variance
 * (single_variance.py:34-36, the model output inv_s) in one launch instead of four elementwise ones. */
int mms_inv_variance(const float* s, float* out, void* stream);

/* out[0] = sum_i x[i] * w[i] in index order (device x[n], host weights w[n], n <= 16): the total training loss from
 * its terms, LossManager.compute_loss's weighted sum (losses.py:224-265; weights 1 per L1 term, 0.1 eikonal,
 * 5e-4 x schedule curvature, method_configs.py:252-253). */
int mms_weighted_sum(const float* x, int n, const float* w, float* out, void* stream);

/* ---- optimizer (pipelines/base_pipeline.py:232-248 clip_gradients, torch.optim.AdamW single-tensor step,
 * method_configs.py:260-269): acc += sum x^2 ; AdamW with clip coefficient min(1, max_norm / (sqrt(*sumsq) + 1e-6))
 * read on device.  lr / wd / betas / eps are torch.optim.AdamW's hyper-parameters, step the optimizer's step count
 * (1 on the first update); the scalars are formed in double like torch's Python code and rounded to float. */
int mms_sumsq(const float* x, int64_t n, float* acc, void* stream);
int mms_adamw(float* p, const float* g, float* m, float* v, int64_t n, const float* sumsq, float max_norm, double lr,
              double wd, double beta1, double beta2, double eps, int64_t step, void* stream);
/* HOST function: the 7 per-step floats the kernel uses, into host memory hyper[7] = [1 - lr wd, 1 - beta1, beta2,
 * 1 - beta2, eps, -lr / (1 - beta1^step), (1 - beta2^step)^0.5] */
int mms_adamw_scalars(double lr, double wd, double beta1, double beta2, double eps, int64_t step, float* hyper);
/* the same step with its per-step scalars read on the device from hyper[7] (mms_adamw_scalars' layout; graph replays:
 * the host rewrites the 7 floats before each launch) */
int mms_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* sumsq, float max_norm,
                  const float* hyper, void* stream);
/* Several optimizer groups per launch (graph-replayed steps; each launch boundary costs ~4-5 us): the groups
 * given by host arrays of device pointers (nseg / nbuf <= 8).  mms_zero_multi: x[k][0, n[k]) = 0 (the groups' gradients and their
 * sum-of-squares accumulators, one launch); mms_sumsq_multi: acc[k] += sum(x[k]^2), as mms_sumsq per group;
 * mms_adamw_dev_multi: mms_adamw_dev of every group (its sum of squares, max_norm and device scalars), bit for bit. */
int mms_zero_multi(int nbuf, float* const* x, const int64_t* n, void* stream);
int mms_sumsq_multi(int nseg, const float* const* x, const int64_t* n, float* const* acc, void* stream);
int mms_adamw_dev_multi(int nseg, float* const* p, const float* const* g, float* const* m, float* const* v,
                        const int64_t* n, const float* const* sumsq, const float* max_norm, const float* const* hyper,
                        void* stream);

/* ---- GPU-resident uniform pixel sampler (UniformPixelSampler.sample, cameras/pixel_samplers.py:71-89, over the
 * frames CacheDataloader caches, data/dataloaders.py:107-167): n draws of (frame, x, y) from Philox4x32-10
 * (key seed, counter *counter + i, stream_id; *counter += n on the device afterwards, so graph replays advance it).
 * coords [n, 3] int32 = [frame_ids[frame] (or frame), y, x]; sel [n] int64 = frame (optional); values [n, C]
 * = images[frame, y, x, :] of images [n_frames, H, W, C] f32 (optional). */
int mms_pixel_sample(uint64_t seed, uint32_t stream_id, uint64_t* counter, int64_t n, int n_frames, int H, int W,
                     const int32_t* frame_ids, const float* images, int C, int32_t* coords, int64_t* sel,
                     float* values, void* stream);
/* Training-mode uniform draws of the model's forward (the NeuS jitter, PDF and background draws that the reference
 * takes from torch.rand, ray_samplers.py:183-296 / :357-403): out[i] ~ U[0, 1) (24-bit), Philox4x32-10 keyed by
 * seed at counter *counter + offset + i / 4 in stream stream_id (the device counter is read, not advanced:
 * mms_counter_advance moves it once per step, in a captured graph too). */
int mms_uniform(uint64_t seed, uint32_t stream_id, const uint64_t* counter, int64_t offset, int64_t n, float* out,
                void* stream);
int mms_counter_advance(uint64_t* counter, int64_t n, void* stream);

/* ---- marching cubes over a dense SDF crop (mesh export: MeshExtractor.extract, evaluator_components/
 * mesh_extractors.py:63 -> utils/marching_cubes.py:97-188, skimage.measure.marching_cubes per 256^3 crop).
 * values [nx * ny * nz] x-major (numpy meshgrid(indexing="ij").ravel()).  Per cube the sign changes on its 12 edges
 * are joined face by face (ambiguous faces by the asymptotic decider) into loops, fanned into triangles facing
 * increasing SDF.  count: counts[cube] = triangles ((nx-1)(ny-1)(nz-1) cubes); emit: with offsets = exclusive scan of
 * counts (int64), verts [T * 3, 3] f32 and keys [T * 3] int64 (3 * grid index of the vertex edge's lower end + axis,
 * for welding).  origin / spacing: HOST arrays of 3 floats (point (i,j,k) = origin + spacing * (i,j,k)). */
int mms_mc_count(const float* vals, int nx, int ny, int nz, float level, int32_t* counts, void* stream);
int mms_mc_emit(const float* vals, int nx, int ny, int nz, float level, const float* origin, const float* spacing,
                const int64_t* offsets, float* verts, int64_t* keys, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* MMS_HIP_H */
