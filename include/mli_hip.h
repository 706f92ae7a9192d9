/*
 * mli_hip.h -- C ABI of libmli_hip.so, the MI355X (gfx950) kernels of the MLI-NeRF
 * stage-b volume-rendering hot path.
 *
 * Every entry point has the shape   int mli_<op>(const mli_<op>_args* a, hipStream_t s)
 * and returns a hipError_t value (0 = success).  No exceptions cross the ABI.
 *
 * Ownership: the caller (PyTorch on the Python side) allocates every buffer; the library
 * never allocates or frees device memory and never synchronises.  Entry points are
 * re-entrant (no global mutable state) and enqueue on the given stream only, so they
 * can be captured into a hipGraph.
 *
 * Scratch sizing: every op whose arguments include caller-provided scratch has a host-only
 * query   int mli_<op>_workspace(const mli_<op>_args* a, int64_t* bytes)   that reads only the
 * shape / mode fields of `a` (no pointer is dereferenced, no GPU call is made) and writes the
 * byte size of each scratch buffer into bytes[], in the order listed with the query.
 *
 * Determinism: results are bit-reproducible run to run except where an op documents fp32
 * atomics; those ops (mli_wgrad, mli_hash_bwd) take a `deterministic` flag that switches to a
 * fixed-order reduction through their workspace.
 *
 * Layout conventions (R rays, N samples per ray, S = R*N, B = 1 image per rank as in
 * every reference config, syn_hotdog_b.yaml:38):
 *   [R,3]      ray-major xyz
 *   [N][R]     sample-major per-sample scalars: element (ray r, sample k) at k*R + r
 *   [N][R][c]  sample-major per-sample vectors
 *   "tile order" for the MLP kernels: m = r*N + k, tiles of 32 consecutive m (a wave),
 *   workgroups of 256 (8 waves).  S must be a multiple of 32.
 *   frag image: fp16 activations of a 32-sample tile in MFMA B-operand register order,
 *   [S/32][ksteps][64 lanes][8 halves] (16 B per lane per k-step, 1 KiB per wave load).
 *   Element j of lane l = c + 32 h of k-step q is sample c of the tile and feature
 *     NAT order: 16 q + 8 h + j                        (the hash-grid encodings)
 *     ACC order: 16 q + 8 (j >> 2) + 4 h + (j & 3)    (an MFMA accumulator tile's registers:
 *                h0, feat, and every training activation / gradient image the weight
 *                gradients read -- x0 (= feat_frag), xT, dzT, dz4T, dz1T; ABI 15;
 *                stage a's dZ0 of the SDF layer 0, ABI 16)
 *   feature-major: [features][S] fp16 rows (S contiguous), in tile order m.
 *   tile-blocked (ABI 14): [S/256][features][256] fp16 -- the 256 samples of one workgroup
 *   of every feature row contiguous (still accepted by mli_wgrad).
 *
 * Reference interface each entry point replaces is cited per function
 * (paths relative to the liulisixin/MLI-NeRF checkout).
 */
#ifndef MLI_HIP_H
#define MLI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mli_stream_t; /* == hipStream_t */

#define MLI_ABI_VERSION 17
#define MLI_HIDDEN 256
#define MLI_LEVELS 16
#define MLI_LEVEL_FEAT 8
#define MLI_HEAD_K0 304 /* packed head layer-0 input rows: feat 256 | p,n 6 | pad 10 | light 16 | view 16 */

/* Per-level hash-grid geometry, passed BY VALUE (host fills it from layout/level_table). */
typedef struct {
  float scale[MLI_LEVELS];
  uint32_t res[MLI_LEVELS];
  uint32_t size[MLI_LEVELS];
  uint32_t offset[MLI_LEVELS];
  uint64_t modmagic[MLI_LEVELS]; /* Lemire fastmod M = 2^64 / size + 1 (dense levels)  */
} mli_grid_levels;

int mli_abi_version(void);
const char* mli_error_string(int code);

/* ---------------------------------------------------------------- rays + bounds
 * Replaces camera.get_center_and_ray + slice_by_ray_idx (projects/nerf/utils/camera.py:283-311,
 * projects/nerf/utils/nerf_util.py:127-131), get_center (NeuralLumen/utils/utils.py:61-79),
 * F.normalize (NeuralLumen/model.py:125) and get_dist_bounds (neuralangelo/model.py:420-430,
 * nerf_util.py:199-205, NeuralLumen/utils/utils.py:86-123).  Only the R sampled rays are built. */
typedef struct {
  const float* intr;      /* [3,3] intrinsics (inverted in-kernel, camera.py:259)          */
  const float* pose;      /* [3,4] world-to-camera [R|t] (Pose.invert in-kernel, camera.py:46-52) */
  const float* pose_light; /* [3,4] world-to-light; pts_light = its camera center          */
  const int64_t* ray_idx; /* [R] flat pixel index y*W + x (NULL: ray r = pixel first+r)   */
  int64_t first_pixel;    /* used when ray_idx == NULL (full-image chunks)                */
  int R, W;
  int bounding;           /* 0: unit sphere, 1: AABB                                      */
  float aabb[6];
  float* center;          /* [R,3] */
  float* ray_unit;        /* [R,3] */
  float* ray_norm;        /* [R]   ||ray|| (depth = dist / ||ray||, NeuralLumen/model.py:103) */
  float* pts_light;       /* [R,3] */
  float* near_;           /* [R]   */
  float* far_;            /* [R]   */
  uint8_t* outside;       /* [R]   */
} mli_rays_args;
int mli_rays(const mli_rays_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- hash-grid encode
 * Replaces tcnn.Encoding(HashGrid) forward (neuralangelo/utils/modules.py:42-50,83-86);
 * semantics restated in oracle/hashgrid.py.  Standalone op (the fused SDF kernels below
 * call the same device code). */
typedef struct {
  const float* x01;       /* [n,3] in [0,1] = (p + 2) / 4                                  */
  const uint16_t* table;  /* fp16 shadow of neural_sdf.tcnn_encoding.params [entries*8]    */
  mli_grid_levels levels;
  int n;
  float* out;             /* [n,128] fp32, level-major                                     */
} mli_hashgrid_args;
int mli_hashgrid_fwd(const mli_hashgrid_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- neural SDF
 * Replaces NeuralSDF.forward/sdf (neuralangelo/utils/modules.py:68-95), MLPforNeuralSDF
 * layer 0 + sdf head (neuralangelo/utils/mlp.py:55-69) and, in FIELD mode, the 4-tap
 * numerical gradient/hessian (modules.py:157-175) + outside overwrite (NeuralLumen/model.py:343).
 * Points are p = center_r + ray_unit_r * dists[k][r] with sample m = r*n_per_ray + k.
 * Weights: `wsdf` from mli_pack (layout MLI_SDF_PACK_*). */
#define MLI_SDF_MODE_SDF 0   /* sdf only                                                   */
#define MLI_SDF_MODE_FIELD 1 /* sdf (+outside), grad, hess, h0 frag image                  */
typedef struct {
  int mode;
  int R, n_per_ray;
  const float* center;
  const float* ray_unit;
  const float* dists;     /* [n_per_ray][R] */
  const uint8_t* outside; /* [R] (FIELD) */
  const uint16_t* table;  /* fp16 hash table */
  mli_grid_levels levels;
  const void* wsdf;       /* packed SDF layer-0 block (mli_pack) */
  float eps;              /* tap epsilon = normal_eps / sqrt(3) (fp32)                    */
  float grad_den;         /* fp32(4 * eps)      (modules.py:167)                           */
  float hess_den;         /* fp32(eps ** 2)     (modules.py:172)                           */
  float outside_val;      /* 1000                                                          */
  int with_hessian;
  float* sdf;             /* [n_per_ray][R] */
  float* grad;            /* [n_per_ray][R][3] (FIELD) */
  float* hess;            /* [n_per_ray][R][3] (FIELD, with_hessian) */
  uint16_t* h0;           /* frag image [S/32][16][64][8] (FIELD) */
  uint16_t* enc;          /* FIELD scratch: hash encodings of the 5 points (center + 4 taps)
                             as MFMA B-fragment images [S/32][5][8][64][8] fp16 (S*640 halves) */
  int active_levels;      /* coarse-to-fine mask (modules.py:91-93,110-113): levels >= this
                             encode to 0 (stage b / c2f off: MLI_LEVELS)                     */
} mli_sdf_args;
int mli_sdf(const mli_sdf_args* a, mli_stream_t s);
/* bytes[0]: enc (FIELD mode; 0 in SDF mode). */
int mli_sdf_workspace(const mli_sdf_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- sampling
 * Replaces nerf_util.sample_dists (nerf_util.py:20-38), sample_dists_hierarchical
 * (neuralangelo/model.py:467-484), sample_dists_from_pdf (nerf_util.py:41-68) and the
 * cat + sort + gather of sample_dists_all (neuralangelo/model.py:449-465). */
typedef struct {
  const float* near_; const float* far_;
  const float* u;         /* [R][Nc] stratified uniforms, NULL -> 0.5 (eval) */
  int R, Nc;
  float* dists;           /* [Nc][R] */
} mli_sample_coarse_args;
int mli_sample_coarse(const mli_sample_coarse_args* a, mli_stream_t s);

typedef struct {
  int R;
  const float* dists_a; const float* sdf_a; int Na;  /* sorted list so far [Na][R]        */
  const float* dists_b; const float* sdf_b; int Nb;  /* previous fine samples (Nb may be 0) */
  float* dists_out; float* sdf_out;                  /* merged [Na+Nb][R] (sdf_out may be NULL) */
  int Nf;                 /* fine samples to draw (0: merge only)                          */
  float inv_s;            /* 64 * 2^h                                                      */
  const float* u_fine;    /* [Nf] midpoint quantiles (torch.linspace semantics, host)       */
  float* fine_out;        /* [Nf][R] */
} mli_sample_fine_args;
int mli_sample_fine(const mli_sample_fine_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- light-conditioned heads
 * Replaces MLPforNeuralSDF layer 1 (feat, mlp.py:61-64) and LumenRGB.forward mode
 * 'rgb_r_s' (NeuralLumen/utils/modules.py:106-109,148-163): SH16 of the view direction and
 * of the raw light position (spherical_harmonics.py:47-84), three weight-normed
 * 5-layer ReLU MLPs (nerf_util.py:158-196) and sigmoid outputs, on fp16 MFMA with fp32
 * accumulation.  Training mode also writes what mli_rgb_bwd / mli_wgrad need. */
typedef struct {
  int R, N;
  const float* center; const float* ray_unit; const float* pts_light;
  const float* dists;     /* [N][R] */
  const float* grad;      /* [N][R][3] normals = normalize(grad)                           */
  const uint16_t* h0;     /* frag image from mli_sdf FIELD                                 */
  const void* wfwd;       /* packed forward weight chunks (mli_pack)                       */
  float* y;               /* [N][R][8] rgb(3) o_r(3) o_s(1) pad                            */
  uint16_t* feat_frag;    /* the heads' layer-0 input image x0, [S/32][MLI_HEAD_K0/16][64][8] ACC
                             order: k-steps 0..15 the SDF feature (SDF layer 1's output, the
                             heads re-read it), in training also k-steps 16..18 (p, normal,
                             pad, SH(light), SH(view)) -- the WIDE dW operand (ABI 15)         */
  /* training outputs (NULL in inference) */
  uint16_t* xT;           /* [3 heads][4 layers] x [S/32][16][64][8] ACC frag images X1..X4 */
  uint32_t* masks;        /* [3][4][S/32][64][4] ReLU bit masks of X1..X4                   */
  int n_heads;            /* 3: LumenRGB 'rgb_r_s' (stage b); 1: mode 'rgb' (stage a, head mlp) */
  /* Output-layer partials (training, N % 32 == 0; both NULL: off).  The composite weights do not
   * depend on the heads, so d loss / d z4[c,s] = D[r,c] * w_s * y_sc (1 - y_sc) with the per-ray
   * D of mli_composite_loss / mli_composite_bwd (`dray`); the forward reduces, per 256-sample
   * workgroup wg and ray segment seg (ray floor(256 wg / N) + seg),
   * q4[wg][seg][head][f][c] = sum_{s of the ray in wg} MLI_Q4_SCALE * w_s y_sc (1 - y_sc) * X3[f,s]
   * (f < 256; row 256: the sums without X3) while X3 is in registers, and mli_dw4 contracts it
   * with D.  X3 (the output layer's input) is then not written: xT holds X1..X3 = 3 layers per
   * head.  Segments past the workgroup's last ray are not written. */
  const float* weights;   /* [N][R] composite weights of this render (mli_composite_fwd, y = NULL) */
  float* q4;              /* [S/256][MLI_Q4_SEGS(N)][n_heads][257][4] fp32 */
} mli_rgb_fwd_args;
#define MLI_Q4_SCALE 65536.0f
/* ray segments per 256-sample workgroup (an upper bound; N % 32 == 0) */
#define MLI_Q4_SEGS(N) ((256 % (N)) == 0 ? 256 / (N) : ((N) % 256 == 0 ? 1 : 256 / (N) + 2))
int mli_rgb_fwd(const mli_rgb_fwd_args* a, mli_stream_t s);
/* bytes[0..5]: y, feat_frag, 0, xT, masks, q4 (xT, masks 0 unless `train` = xT != NULL is
 * requested by setting a->xT to any non-NULL value before the query; q4 0 unless a->weights is
 * non-NULL, which also drops X3 from xT). */
int mli_rgb_fwd_workspace(const mli_rgb_fwd_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- compositing
 * Replaces compute_neus_alphas/_get_iter_cos (neuralangelo/model.py:492-515),
 * alpha_compositing_weights + composite (nerf/utils/render.py:87-112) and the intrinsic
 * assembly of render_rays_lumen (NeuralLumen/model.py:266-305) incl. white background
 * and o_re; eval adds opacity, gradient and depth (NeuralLumen/model.py:101-104). */
typedef struct {
  int R, N;
  const float* dists; const float* far_; const float* ray_unit; const float* ray_norm;
  const float* sdf; const float* grad; const float* y;
  const float* s_var;     /* device scalar: inv_s = exp(s_var)                             */
  float anneal;           /* min(progress / anneal_end, 1)                                 */
  int white_bg;
  float* weights;         /* [N][R] */
  float* rgb; float* o_r; float* o_s; float* o_re;   /* [R,3],[R,3],[R],[R,3]             */
  float* opacity; float* gradient; float* depth;     /* [R],[R,3],[R] (NULL to skip)      */
  float* blend_dist;      /* [R] sum_k w_k d_k (light visibility camera ray start) or NULL   */
} mli_composite_args;
/* y == NULL: only the weights (the heads' PQ mode needs them before the heads run); the
 * composited outputs are then not written. */
int mli_composite_fwd(const mli_composite_args* a, mli_stream_t s);

/* Backward of the composite w.r.t. the head outputs: per-sample dZ4 = dy*y*(1-y)*scale. */
typedef struct {
  int R, N;
  const float* weights; const float* y;
  const float* o_r; const float* o_s;                 /* composited [R,3], [R] */
  const float* d_rgb; const float* d_o_r; const float* d_o_s; const float* d_o_re;
  float grad_scale;       /* power of two, undone in mli_grad_assemble                     */
  float* dz4;             /* [N][R][8] scaled pre-sigmoid grads: rgb(3) r(3) s(1) pad       */
  float* dray;            /* [R][8] or NULL: d loss / d composited rgb(3) o_r(3) o_s (after the
                             o_re chain, unscaled), the per-ray factor of dz4 (mli_dw4)       */
} mli_composite_bwd_args;
int mli_composite_bwd(const mli_composite_bwd_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- heads backward
 * dX chain of the three heads (ReLU masks from the forward), writing feature-major
 * dZ_l for the weight gradients.  Replaces autograd through MLPwithSkipConnection. */
typedef struct {
  int R, N;
  const float* dz4;       /* [N][R][8] */
  const void* wbwd;       /* packed transposed weight chunks (mli_pack)                     */
  const uint32_t* masks;  /* from mli_rgb_fwd */
  uint16_t* dzT;          /* [3 heads][4 layers] x [S/32][16][64][8] ACC frag images dZ0..dZ3
                             (scaled)                                                        */
  uint16_t* dz4T;         /* [3 heads] x [S/32][1][64][8] frag images of dZ4 (rows 0..2, scaled),
                             or NULL (PQ mode: the output-layer dW comes from mli_dw4)         */
} mli_rgb_bwd_args;
int mli_rgb_bwd(const mli_rgb_bwd_args* a, mli_stream_t s);
/* bytes[0..1]: dzT, dz4T. */
int mli_rgb_bwd_workspace(const mli_rgb_bwd_args* a, int64_t* bytes);

/* Weight/bias gradients dW_l = dZ_l^T X_l, db_l = sum dZ_l (split-K MFMA GEMM).  Default: the
 * k-slices add into dw/db (caller-zeroed) by fp32 atomics, in arbitrary order.  deterministic:
 * every k-slice writes its partial tile into the workspace and a second launch sums the slices
 * in slice order into dw/db (overwritten; no zeroing needed): bit-reproducible.  Jobs are
 * described in mli_nerf_amd/engine.py.
 * Jobs fall into three launch classes by shape: BIG (M > 32, K <= 256: 256 x 256 tiles),
 * WIDE (M > 32, K > 256: 256 x 320 tiles, the 304-wide layer-0 input) and THIN (M <= 32:
 * 32 x 256); whole-width tiles stream every dZ row once.  `classes` selects which classes
 * this call launches (bit mask), so a caller can time them separately.  Split-K is sized
 * per class to fill the 256 CUs. */
typedef struct {
  const uint16_t* a_rows; /* dZ^T [M rows][S samples] in layout a_tiled */
  const uint16_t* b_rows; /* X^T  [K rows][S samples] in layout b_tiled */
  int M, K;               /* logical rows of A and B */
  float* dw;              /* [M][ldw] fp32; this job writes columns [0, K) */
  float* db;              /* [M] fp32 or NULL */
  int ldw;                /* row stride of dw (>= K) */
  int a_tiled, b_tiled;   /* operand layout (MLI_WGRAD_LAYOUT_*): 0 feature-major rows [rows][S];
                             1 tile-blocked (S % 256 == 0): sample m of row r at
                             (m / 256) * rows * 256 + r * 256 + m % 256; 2 / 3 frag image in ACC /
                             NAT order (S % 64 == 0): the tile of sample m at (m / 32) * kst
                             k-steps -- the layout mli_rgb_fwd / mli_rgb_bwd / mli_geo_bwd write
                             (ABI 15).  A job's two operands are both frag images or neither.    */
  int a_kst, b_kst;       /* frag images: k-steps per 32-sample tile (>= ceil(rows / 16)); else 0 */
  const uint16_t* b2_rows; /* frag images only, or NULL: B's k-steps b2_q .. come from this second
                              frag image (b2_kst k-steps per tile, B's order and tile count) -- the
                              SDF layer-0 input [enc 128 | p 3] of mli_sdf_bwd (ABI 16)            */
  int b2_q, b2_kst;
} mli_wgrad_job;
#define MLI_WGRAD_LAYOUT_ROWS 0
#define MLI_WGRAD_LAYOUT_TILED 1
#define MLI_WGRAD_LAYOUT_FRAG_ACC 2
#define MLI_WGRAD_LAYOUT_FRAG_NAT 3
#define MLI_WGRAD_BIG 1
#define MLI_WGRAD_WIDE 2
#define MLI_WGRAD_THIN 4
typedef struct {
  int S;                  /* samples (multiple of 64) */
  int n_jobs;
  const mli_wgrad_job* jobs; /* HOST array (copied into the kernel arguments) */
  int classes;            /* MLI_WGRAD_* mask */
  int deterministic;      /* 0: fp32 atomics; 1: slice partials + ordered reduction */
  float* workspace;       /* deterministic: mli_wgrad_workspace bytes (reused across classes) */
} mli_wgrad_args;
int mli_wgrad(const mli_wgrad_args* a, mli_stream_t s);
/* bytes[0]: workspace (0 unless deterministic): the largest class in `classes`. */
int mli_wgrad_workspace(const mli_wgrad_args* a, int64_t* bytes);

/* Output-layer weight / bias gradients of the heads from the forward's partials (PQ mode of
 * mli_rgb_fwd): dW4[c][f] = scale * sum_(wg,seg) dray[ray(wg,seg)][off_h + c] * q4[wg][seg][h][f][c],
 * db4[c] the same over row 256, off_h = 3h.  Replaces the THIN mli_wgrad class (the autograd dW /
 * db of the last nn.Linear of each MLPwithSkipConnection, nerf_util.py:186-196).  Two launches:
 * per-slice partial sums into the workspace, then a sum over the slices in slice order
 * (bit-reproducible; dw / db overwritten). */
typedef struct {
  int R, N, n_heads;      /* S = R*N, N % 32 == 0 */
  const float* q4;        /* [S/256][MLI_Q4_SEGS(N)][n_heads][257][4] from mli_rgb_fwd */
  const float* dray;      /* [R][8] */
  float scale;            /* grad_scale / MLI_Q4_SCALE (the dw / db land at the split-K dW scale) */
  float* dw[3];           /* per head: [k_out][256] */
  float* db[3];           /* per head: [k_out] */
  int k_out[3];           /* 3, 3, 1 (LumenRGB 'rgb_r_s') */
  float* workspace;       /* bytes[0] */
} mli_dw4_args;
int mli_dw4(const mli_dw4_args* a, mli_stream_t s);
/* bytes[0]: workspace (slice partials). */
int mli_dw4_workspace(const mli_dw4_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- stage a (geometry training)
 * Backward of the whole render w.r.t. the geometry: replaces autograd through
 * compute_neus_alphas (neuralangelo/model.py:492-515), alpha_compositing_weights/composite
 * (render.py:87-112), the single 'rgb' head (NeuralLumen/utils/modules.py:164-174) down to
 * its inputs (feat, normals), F.normalize, compute_gradients taps=4 (modules.py:157-175),
 * MLPforNeuralSDF (mlp.py:55-69), the coarse-to-fine mask and the tcnn HashGrid backward
 * (scatter-add into the table; restated in oracle/hashgrid.py).  grad_scale: the power-of-two
 * loss scale of every fp16 gradient image (undone in fp32 at the outputs). */

/* Composite backward with geometry terms, one wave per ray: dz4 (rgb head output grads,
 * scaled), d total / d sdf (after the outside overwrite), d total / d grad through the NeuS
 * iter_cos, and d total / d s_var (written by a second launch). */
typedef struct {
  int R, N;
  const float* dists; const float* far_; const float* ray_unit;
  const float* sdf; const float* grad; const float* y;   /* y: [N][R][8], rgb in 0..2 */
  const float* s_var;
  float anneal;
  int white_bg;
  const float* d_rgb;     /* [R,3] d total / d rgb */
  float grad_scale;
  float* dz4;             /* [N][R][8] scaled */
  float* d_sdf;           /* [N][R] */
  float* d_grad;          /* [N][R][3] */
  float* d_inv_s_part;    /* scratch [R] per-ray d inv_s partials, summed in ray order */
  float* d_s_var;         /* device scalar out: exp(s_var) * d_inv_s */
} mli_composite_bwd_geo_args;
int mli_composite_bwd_geo(const mli_composite_bwd_geo_args* a, mli_stream_t s);
/* bytes[0..3]: dz4, d_sdf, d_grad, d_inv_s_part. */
int mli_composite_bwd_geo_workspace(const mli_composite_bwd_geo_args* a, int64_t* bytes);

/* dX chain of the single head down to its inputs, then through SDF layer 1:
 * dZ3..dZ0 (ACC frag images, for the head dW), dX0 -> d feat (frag order) and d normal,
 * dZ1sdf = d feat * softplus'(z1) (ACC frag image, for dW of neural_sdf.mlp.linears.1) and
 * d h0 of the center point = W1^T dZ1sdf (frag image, ACC order as the h0 image). */
typedef struct {
  int R, N;
  const float* dz4;       /* [N][R][8] */
  const void* wgeo;       /* packed chunks (mli_pack): W4^T, W3^T, W2^T, W1^T, W0^T (9 n-tiles),
                             W1sdf^T of the stage-a layout (mli_nerf_amd/layout.py geo_plan) */
  const uint32_t* masks;  /* head 0 masks from mli_rgb_fwd */
  const uint16_t* feat_frag; /* x0 image from mli_rgb_fwd (feat = its k-steps 0..15) */
  uint16_t* dzT;          /* [4 layers] x [S/32][16][64][8] ACC frag images dZ0..dZ3 (scaled) */
  uint16_t* dz4T;         /* [S/32][1][64][8] frag image of dZ4 (rows 0..2, scaled) */
  float* d_nrm;           /* [N][R][4] scaled d total / d normal (xyz, pad) */
  uint16_t* dz1T;         /* [S/32][16][64][8] ACC frag image dZ1sdf (scaled) */
  uint16_t* dh0_frag;     /* [S/32][16][64][8] d h0 (scaled, layer-1 path only) */
} mli_geo_bwd_args;
int mli_geo_bwd(const mli_geo_bwd_args* a, mli_stream_t s);
/* bytes[0..5]: dzT, dz4T, d_nrm, dz1T, dh0_frag (and 0). */
int mli_geo_bwd_workspace(const mli_geo_bwd_args* a, int64_t* bytes);

/* SDF layer 0 + sdf head backward for the 5 points of every sample (center + 4 taps):
 * combines d sdf / d grad (composite), eikonal / curvature gradients, the normalize
 * backward of d normal and the tap stencils into d sdf_i; recomputes layer 0 of every point
 * from the FIELD encodings; writes d enc (fp32, for mli_hash_bwd), the dZ0 and p fragment
 * images of the layer-0 weight gradient (ABI 16: mli_wgrad reads them beside the FIELD
 * encodings, no row conversion) and dW/db of linear_sdf (per-wave sums in
 * LDS, per-workgroup partials in `partials`, summed in workgroup order by a second launch). */
typedef struct {
  int R, N;
  const float* center; const float* ray_unit; const float* dists;
  const uint8_t* outside;
  const float* grad; const float* hess;   /* forward [N][R][3] */
  const float* d_sdf; const float* d_grad; /* from mli_composite_bwd_geo */
  const float* d_nrm;     /* [N][R][4] scaled, from mli_geo_bwd */
  const uint16_t* dh0_frag; /* from mli_geo_bwd */
  const uint16_t* enc;    /* FIELD encodings [S/32][5][8][64][8] */
  const void* wsdf;       /* mli_pack_sdf block */
  const void* wsdf_t;     /* W0_enc^T block (mli_pack_sdf_t) */
  float eps, grad_den, hess_den;
  float w_eikonal, w_curvature;  /* loss weights / (R*N) are applied in-kernel */
  float grad_scale;
  float* d_enc;           /* [S/32][5][8][64][8] fp32 (unscaled) */
  uint16_t* dz0_frag;     /* [S/32][5][16][64][8] fp16 ACC frag image of the scaled dZ0 of the 5 points:
                             5S samples in the enc image's order (32-sample tile t of point pi is
                             image tile 5 t + pi)                                               */
  uint16_t* p_frag;       /* [S/32][5][1][64][8] fp16 NAT frag image of the points p (features
                             0..2, rest 0), the same tile order: the layer-0 input's last k-step  */
  float* dw_sdf;          /* [256] scaled (written) */
  float* db_sdf;          /* [1] scaled (written) */
  const float* d_grad_ext; /* optional [N][R][3] d loss / d gradients from outside (autograd) */
  const float* d_hess_ext; /* optional [N][R][3] d loss / d hessians from outside (autograd) */
  float* partials;        /* scratch [workgroups][257] */
} mli_sdf_bwd_args;
int mli_sdf_bwd(const mli_sdf_bwd_args* a, mli_stream_t s);
/* bytes[0..3]: d_enc, dz0_frag, p_frag, partials. */
int mli_sdf_bwd_workspace(const mli_sdf_bwd_args* a, int64_t* bytes);

/* W0_enc^T fragments (A operand of d enc = W0_enc^T dZ0; rows ordered so each lane half
 * holds 8 features of one level) -- MLI_SDF_T_PACK_BYTES. */
typedef struct {
  const float* v0; const float* g0;   /* linears.0 [256,131] */
  uint8_t* dst;
} mli_pack_sdf_t_args;
#define MLI_SDF_T_PACK_BYTES 65536
int mli_pack_sdf_t(const mli_pack_sdf_t_args* a, mli_stream_t s);

/* Hash-grid backward: d table[(offset_l + idx) * 8 + f] += w_corner * d enc, for the 5
 * points of every sample (taps in the center's cell share its corners: one atomic per
 * corner feature), levels < active_levels.  Default: fp32 atomics into the caller-zeroed
 * d_table.  deterministic: the run totals are added as fixed-point int64 (2^-40 units) into
 * the caller-zeroed workspace -- integer sums do not depend on their order -- and a second
 * launch writes d_table = float(sum * 2^-40) (overwritten): bit-reproducible.  The fixed point
 * quantizes as well as reorders: every added run total is rounded to the nearest 2^-40
 * (9.1e-13), so an element of n contributions is within n * 2^-41 of the exact sum before its
 * final float rounding, run totals below 4.5e-13 vanish, and |sum| must stay below 2^23.
 * The workspace is 8 B per table element (2.9 GB at 2^22 entries per level). */
typedef struct {
  int R, N;
  const float* center; const float* ray_unit; const float* dists;
  const float* d_enc;     /* from mli_sdf_bwd */
  mli_grid_levels levels;
  float eps;
  int active_levels;
  float* d_table;         /* [entries*8] fp32 */
  int deterministic;
  int64_t* workspace;     /* deterministic: [entries*8] int64, zeroed by the caller */
  int64_t n_params;       /* entries*8 (deterministic: the workspace / d_table length) */
} mli_hash_bwd_args;
int mli_hash_bwd(const mli_hash_bwd_args* a, mli_stream_t s);
/* bytes[0]: workspace (0 unless deterministic). */
int mli_hash_bwd_workspace(const mli_hash_bwd_args* a, int64_t* bytes);

/* Frag image -> feature-major rows: src [tiles][tile_stride halves], k-step q of tile t at
 * src + t*tile_stride + q*512; element (q, lane half h, j) of sample t*32 + (lane & 31) goes
 * to row row0 + k(q,h,j) (order 0: NAT 16q+8h+j, 1: ACC) at column col0 + sample. */
typedef struct {
  const uint16_t* src;
  int64_t tile_stride;
  int tiles, k_steps, order;
  uint16_t* dst;
  int64_t ld;             /* row stride (elements) */
  int64_t col0;
  int row0;
} mli_frag_rows_args;
int mli_frag_rows(const mli_frag_rows_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- light visibility
 * Replaces get_light_visibility (NeuralLumen/model.py:133-184, method 'sphere_tracing') with
 * sphere_tracing_intersection (neuralangelo/model.py:298-325) on the camera ray (camera_ray_type
 * 0: blend_z_sphere_tracing from the composited depth, 1: blend_z, 2: sphere_tracing from near)
 * and on the light ray (visibility bounds get_dist_bounds_visibility :186-199), then
 * visibility = !hit | !inside, normal_x_light = relu(normalize(-gradient) . light_dir),
 * pseudo_shading = normal_x_light * visibility (^ 1/gamma).  Four launches. */
typedef struct {
  int R;
  const float* center; const float* ray_unit; const float* pts_light;   /* [R,3] */
  const float* near_; const float* far_;                               /* camera ray bounds [R] */
  const float* blend_dist;   /* [R] from mli_composite_fwd */
  const float* gradient;     /* [R,3] composited gradients (eval) */
  int camera_ray_type, iters;
  int vis_box;               /* 0: sphere of radius^2 vis_r2, 1: the AABB */
  float vis_r2; float aabb[6];
  float gamma;               /* 0: none */
  const uint16_t* table; mli_grid_levels levels; int active_levels; const void* wsdf;
  float* light_unit; float* near_l; float* far_t; uint8_t* inside;    /* scratch [R,3],[R],[R],[R] */
  float* inter_dist; uint8_t* inter_mask; float* inter_pts;           /* [R],[R],[R,3] */
  uint8_t* visibility; float* normal_x_light; float* pseudo_shading; /* [R] */
} mli_light_visibility_args;
int mli_light_visibility(const mli_light_visibility_args* a, mli_stream_t s);
/* bytes[0..4]: light_unit, near_l, far_t, inside, inter_pts. */
int mli_light_visibility_workspace(const mli_light_visibility_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- on-device ray batch
 * Replaces the per-sample CPU draw of NeuralLumen/data.py:120-132 / data_blender.py:179-195
 * (ray_idx = randperm(H*W)[:R], then gathers of the image and the pseudo labels): ray r takes
 * pixel pi(r) of a seeded bijection pi of [0, n_pixels) (4-round Feistel network with cycle
 * walking), so the R indices are distinct by construction and drawn in parallel; the
 * device-resident image / pseudo-label planes are gathered in the same launch. */
typedef struct {
  uint64_t seed;
  int64_t n_pixels;
  int R;
  const float* image;     /* [3][n_pixels] (torchvision to_tensor layout) or NULL */
  const float* ref;       /* [3][n_pixels] pseudo_reflectance or NULL */
  const float* sha;       /* [n_pixels] pseudo_shading_gamma or NULL */
  const float* cert;      /* [n_pixels] visibility_certainty or NULL */
  int64_t* ray_idx;       /* [R] */
  float* image_sampled;   /* [R,3] */
  float* ref_sampled;     /* [R,3] */
  float* sha_sampled;     /* [R] */
  float* cert_sampled;    /* [R] */
} mli_ray_batch_args;
int mli_ray_batch(const mli_ray_batch_args* a, mli_stream_t s);

/* ---------------------------------------------------------------- losses
 * Stage-b loss terms and d(total)/d(rgb, o_r, o_s, o_re) in one call (three launches):
 * replaces NeuralLumen/trainer.py:133-149 (_compute_loss) with eikonal/curvature
 * (neuralangelo/utils/misc.py:74-90), intrinsic_loss / regularize_re_loss
 * (NeuralLumen/utils/utils.py:142-174) and _get_total_loss (imaginaire/trainers/base.py:534-544).
 * Deterministic: workgroup partial sums go to `scratch` and one launch sums them in order. */
typedef struct {
  int R, N;
  const float* rgb; const float* o_r; const float* o_s; const float* o_re; /* [R,3],[R,3],[R],[R,3] */
  const float* gt;        /* image_sampled [R,3] */
  const float* ref; const float* sha; const float* cert; /* pseudo labels [R,3],[R],[R] (NULL: intrinsic off) */
  const uint8_t* outside; /* [R] */
  const float* grad; const float* hess; /* [N][R][3] (NULL skips eikonal / curvature) */
  float w_render, w_eikonal, w_curvature, w_intrinsic, w_re;
  float range_sha_lo, range_sha_hi, range_vis_lo, range_vis_hi, f_ref, f_sha;
  float f_neg, f_pos, e_pos;
  float* d_rgb; float* d_o_r; float* d_o_s; float* d_o_re; /* d total / d output */
  float* losses;          /* [8]: render, eikonal, curvature, intrinsic, regularize_re, total, psnr, mse */
  float* scratch;         /* mli_stage_b_loss_workspace bytes: min/max of the pseudo maps + the
                             workgroup partial sums (no zeroing needed) */
} mli_loss_args;
int mli_stage_b_loss(const mli_loss_args* a, mli_stream_t s);
/* bytes[0]: scratch; bytes[1..4]: d_rgb, d_o_r, d_o_s, d_o_re. */
int mli_stage_b_loss_workspace(const mli_loss_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- fused training tail
 * mli_composite_fwd (training outputs) + mli_stage_b_loss + mli_composite_bwd in one launch,
 * one wave per ray (the fused stage-b train step), plus a one-workgroup launch that sums the
 * loss partials: the composited outputs and the loss gradients stay in registers.  Outputs
 * (weights, rgb, o_r, o_s, o_re) and dz4 equal the three-call path bit for bit (one definition
 * of each formula); the loss values are the same sums in another fixed order, so repeated
 * calls are bit-identical.
 * Replaces the same reference functions as those three calls. */
typedef struct {
  mli_composite_args comp; /* opacity, gradient, depth, blend_dist: ignored (training)          */
  mli_loss_args loss;      /* rgb, o_r, o_s, o_re, d_rgb, d_o_r, d_o_s, d_o_re: ignored;
                              scratch = workspace bytes[0] (no zeroing needed)                  */
  float grad_scale;        /* as mli_composite_bwd_args */
  float* dz4;              /* [N][R][8], as mli_composite_bwd_args */
  int defer_finalize;      /* 1: leave the loss values to mli_composite_loss_finalize (the
                              gradients do not need them; the host issues it where the GPU is
                              idle, e.g. after the weight gradients)                           */
  float* dray;             /* [R][8] or NULL, as mli_composite_bwd_args                         */
} mli_composite_loss_args;
int mli_composite_loss(const mli_composite_loss_args* a, mli_stream_t s);
/* The loss values of a deferred mli_composite_loss (same args, same scratch). */
int mli_composite_loss_finalize(const mli_composite_loss_args* a, mli_stream_t s);
/* bytes[0]: scratch (workgroup partials); bytes[1]: dz4. */
int mli_composite_loss_workspace(const mli_composite_loss_args* a, int64_t* bytes);

/* ---------------------------------------------------------------- parameters
 * Weight-norm W = g * v / ||v||_row (torch.nn.utils.weight_norm dim=0) folded once per
 * step and packed into the fp16 MFMA chunk images the kernels stream; layer descriptors
 * built on the host (mli_nerf_amd/layout.py). */
typedef struct {
  const float* v; const float* g; const float* bias; /* reference tensors (fp32)         */
  int n_out, k_ref;       /* v is [n_out][k_ref]                                          */
  int transpose;          /* 0: pack W (rows n_out), 1: pack W^T (rows k_ref)              */
  int n_tiles, k_steps;   /* packed geometry: rows n_tiles*32, k_steps*16                  */
  const int16_t* kmap;    /* [k_steps*16] packed k -> source index (-1: zero)              */
  const uint8_t* kmode;   /* [k_steps] 0: NAT, 1: ACC ordering                             */
  int64_t dst_offset;     /* byte offset of the first chunk in dst                         */
  int chunk_stride;       /* bytes per chunk (k_steps*1024 + 128)                          */
  const int16_t* nmap;    /* transpose only: [n_tiles*32] packed row -> W column (-1: zero);
                             NULL: identity                                                 */
} mli_pack_layer;
typedef struct {
  int n_layers;
  const mli_pack_layer* layers; /* DEVICE array of descriptors */
  uint8_t* dst;
  float* row_scale;       /* scratch [n_layers][256]: g / ||v_row|| (n_out <= 256)           */
} mli_pack_args;
int mli_pack(const mli_pack_args* a, mli_stream_t s);
/* bytes[0]: row_scale. */
int mli_pack_workspace(const mli_pack_args* a, int64_t* bytes);

/* SDF layer-0 block: fp16 fragments of W0[:, 3:] + fp32 row constants (see layout.py). */
typedef struct {
  const float* v0; const float* g0; const float* b0;  /* linears.0 [256,131]              */
  const float* w_sdf; const float* b_sdf;             /* linear_sdf [1,256], [1]          */
  uint8_t* dst;           /* MLI_SDF_PACK_BYTES */
} mli_pack_sdf_args;
#define MLI_SDF_PACK_BYTES (65536 + 5 * 1024 + 16)
int mli_pack_sdf(const mli_pack_sdf_args* a, mli_stream_t s);

/* dW (packed-k order) -> reference-layout grads of weight_v / weight_g / bias through the
 * weight-norm backward, scaled by 1/grad_scale, written into the flat grad buffer. */
typedef struct {
  const float* dw; const float* db;    /* [n_out][k_pack], [n_out] */
  const float* v; const float* g;
  int n_out, k_ref, k_pack;
  const int16_t* kinv;    /* [k_ref] reference column -> packed k                         */
  float* grad_v; float* grad_g; float* grad_b;
  const float* extra_db;  /* NULL */
  int plain;              /* 1: plain Linear (no weight norm): grad_v = dW * inv_scale */
} mli_assemble_layer;
typedef struct {
  int n_layers;
  const mli_assemble_layer* layers; /* DEVICE array */
  float inv_scale;
  int zero_dw;            /* ABI 17: 1 = every dw / db element read is left 0 (the next split-K
                             accumulation adds into a zeroed buffer without a fill launch) */
} mli_assemble_args;
int mli_grad_assemble(const mli_assemble_args* a, mli_stream_t s);

/* AdamW over one flat fp32 parameter buffer (torch.optim.AdamW semantics,
 * imaginaire/trainers/utils/get_trainer.py:106-150, base.yaml:117-127). */
typedef struct {
  float* p; float* g; float* m; float* v;
  int64_t n;
  double lr, beta1, beta2, eps, weight_decay; /* double, as torch's Python scalars: the step
                           coefficients (1 - beta, lr / bias correction ...) are formed in double
                           and rounded to fp32 once, as torch.optim.AdamW does */
  int step;               /* 1-based step after increment */
  uint16_t* p16;          /* optional fp16 copy of the updated p (hash-table shadow), or NULL */
  int zero_grad;          /* ABI 17: 1 = leave g all zero for the next scatter (g[i] = 0 stored
                           only where g[i] != 0: the sparse hash-table gradient's touched lines,
                           instead of a dense fill of the whole buffer before mli_hash_bwd) */
} mli_adamw_args;
int mli_adamw(const mli_adamw_args* a, mli_stream_t s);

/* fp32 -> fp16 copy (hash-table shadow). */
typedef struct { const float* src; uint16_t* dst; int64_t n; } mli_cast_args;
int mli_cast_f16(const mli_cast_args* a, mli_stream_t s);

/* sha256 prefix (16 hex digits) of the sources and compile flags this library was built from
 * (mli_nerf_amd/build.py source_hash): the Python host refuses a library whose hash differs
 * from its in-tree sources. */
const char* mli_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* MLI_HIP_H */
