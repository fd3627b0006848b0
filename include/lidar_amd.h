/*
 * lidar_amd.h — C-ABI of the MI355X (gfx950) LiDAR hot-path library, liblidar_amd.so.
 *
 * This is the drop-in boundary.  The reference (FortuneMU2025/LIDAR_AI_Recommendation_Software)
 * is pure Python; its hot path is the operator set in utils/data_processing.py and
 * models/crowd_density_model.py.  Each entry point below names the reference
 * interface it replaces (file:line in /root/reference).  The Python host layer
 * (lidar_ai_recommendation_software_amd/) binds these with ctypes, mirroring the
 * reference's Python signatures; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every array pointer is a DEVICE pointer
 *    (hipMalloc / torch CUDA tensor storage) unless the name ends in `_host`.
 *  - The caller owns every input/output buffer.  The library owns only the scratch
 *    workspace inside a handle (grown on demand; lidar_reserve() pre-sizes it so a
 *    later call can be captured into a hipGraph).
 *  - Calls are asynchronous on `stream` (a hipStream_t; NULL = legacy default stream).
 *  - Return 0 on success, a negative LIDAR_E* code on failure; nothing throws across
 *    the ABI.  lidar_last_error() returns a thread-local message for the last failure.
 *  - A handle is bound to one device.  Use one handle per (thread, stream): calls on
 *    one handle must not run concurrently (the scratch workspace is shared).
 *  - Frames are batched: `batch` frames of `n` points, (batch, n, 3) row-major, unless a
 *    CSR `offsets` array is given (Tier R, ragged frames).
 */
#ifndef LIDAR_AMD_H
#define LIDAR_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIDAR_OK 0
#define LIDAR_EINVAL -1   /* bad argument (shape, size, null pointer) */
#define LIDAR_EHIP -2     /* a HIP runtime call failed */
#define LIDAR_ENOMEM -3   /* workspace allocation failed */
#define LIDAR_EDEVICE -4  /* device is not gfx950 */
#define LIDAR_EPARSE -5   /* a text token the C parser does not reproduce exactly (caller falls back) */

typedef struct lidar_handle lidar_handle;

/* ------------------------------------------------------------------ handle */
int lidar_create(int device, lidar_handle **out);
int lidar_destroy(lidar_handle *h);
/* grow the scratch workspace to at least `bytes` now (not inside graph capture).  Growth never
 * synchronises the device: the replaced block is retired (queued kernels may still read it) and
 * freed by lidar_destroy or lidar_trim. */
int lidar_reserve(lidar_handle *h, uint64_t bytes);
/* free the workspaces retired by growth (*freed = their bytes, may be NULL); the caller guarantees
 * that the work it queued with this handle before the growth has completed */
int lidar_trim(lidar_handle *h, uint64_t *freed);
const char *lidar_last_error(void);
int lidar_version(void); /* 5 (what changed per version) */

/* Per-phase timing of a handle's launches (bench.py's in-window kernel durations): with
 * lidar_profile(h, 1) every kernel phase issued on h is bracketed by two HIP events on its
 * stream; lidar_profile_read waits for them and returns, in launch order, the phase names
 * ('\n'-separated into names, NUL terminated) and durations in ms; lidar_profile(h, 0) stops.
 * The Tier R entry points (preprocess, DBSCAN, people, density grid) record phases. */
int lidar_profile(lidar_handle *h, int32_t enable);
int lidar_profile_read(lidar_handle *h, char *names, int64_t names_cap, float *ms, int64_t cap, int64_t *count);

/* ============================================================ Tier N (SA stack)
 * North_star operators.  The reference has no PointNet++ code; these
 * are exposed beside utils/data_processing.py:231 (downsample_point_cloud) and drive
 * CrowdDensityModel's optional PointNet++ backbone (models/crowd_density_model.py:14).
 */

/* workspace bytes the FPS entry points take from a handle for (batch, n) (for lidar_reserve) */
uint64_t lidar_fps_workspace_bytes(int64_t batch, int64_t n);

/* farthest-point sampling: idx (batch, npoint) int32; optionally new_xyz (batch, npoint, 3)
 * = xyz[idx] (pass NULL to skip).  Start index 0, fp32 no-FMA distances, lowest index on
 * ties.  Optional first_zero (batch) receives the first step whose winning distance was 0
 * (npoint if none).  Optional prefix_ok (batch): when xyz are the first points of a parent
 * FPS ordering, pass the parent's first_zero — frames with npoint <= prefix_ok[b] get the
 * exact identity result without running (nested SA levels).  Replaces:
 * downsample_point_cloud's random subset (utils/data_processing.py:231-249) where a
 * spatially uniform subset is wanted. */
int lidar_fps_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                  int32_t *idx, float *new_xyz, int32_t *first_zero, const int32_t *prefix_ok,
                  void *stream);
/* the same with an explicit workgroup size per frame: threads 0 (default, 1024), 1024 or 512.
 * 512 takes ~25 % longer per step and half the CU footprint (throughput pipelines that run
 * other kernels beside FPS).  Identical results. */
int lidar_fps_ex_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, int64_t npoint,
                     int32_t *idx, float *new_xyz, int32_t *first_zero, const int32_t *prefix_ok,
                     int32_t threads, void *stream);

/* ball query: idx (batch, m, nsample) int32 — the first `nsample` point indices (ascending)
 * with d < radius^2, padded with the first hit, 0 when there is none.  Replaces the eps-ball
 * query the reference runs through sklearn (utils/data_processing.py:197,
 * models/crowd_flow_model.py:216,228 query_radius) with a bounded-nsample form. */
int lidar_ball_query_f32(lidar_handle *h, const float *xyz, const float *centres, int64_t batch,
                         int64_t n, int64_t m, float radius, int32_t nsample, int32_t *idx,
                         void *stream);

/* the same query with an explicit kernel: mode 0 = auto (grid for n >= 1024), 1 = the
 * index-order scan, 2 = the (index window, cell) grid.  Results are identical. */
int lidar_ball_query_mode_f32(lidar_handle *h, const float *xyz, const float *centres,
                              int64_t batch, int64_t n, int64_t m, float radius, int32_t nsample,
                              int32_t mode, int32_t *idx, void *stream);

/* the grid path in two steps, so the binning of a frame (it depends only on xyz) can run
 * ahead on another stream: lidar_ball_query_bin_f32 writes the grid of every frame into a
 * caller-owned device buffer of lidar_ball_query_grid_bytes(batch, n) bytes;
 * lidar_ball_query_binned_f32 answers queries from it.  A grid binned for radius r answers
 * any radius exactly (radii above r fall back to scanning whole windows); nsample only tunes
 * the window size. */
uint64_t lidar_ball_query_grid_bytes(int64_t batch, int64_t n);
int lidar_ball_query_bin_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, float radius,
                             int32_t nsample, void *grid, void *stream);
int lidar_ball_query_binned_f32(lidar_handle *h, const float *xyz, const void *grid, const float *centres,
                                int64_t batch, int64_t n, int64_t m, float radius, int32_t nsample,
                                int32_t *idx, void *stream);

/* dense layer on MFMA: y (rows, cout) = relu(x (rows, k) W (k, cout) + b), fp32.
 * If pool_rows > 0: y is (rows / pool_rows, cout) = max over each run of pool_rows rows
 * (group_all's max-pool, fused); y must then be zeroed by the caller first.
 * k a multiple of 16, cout a multiple of 128, rows a multiple of 128
 * (pool_rows a multiple of 128 when used). */
int lidar_dense_relu_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k,
                         const float *w, const float *bias, int32_t cout, int32_t pool_rows,
                         float *y, void *stream);

/* as lidar_dense_relu_f32 with the ReLU optional (relu_on = 0: y = x W + b); the fused
 * max-pool requires relu_on. */
int lidar_dense_f32(lidar_handle *h, const float *x, int64_t rows, int32_t k, const float *w,
                    const float *bias, int32_t cout, int32_t relu_on, int32_t pool_rows, float *y,
                    void *stream);

/* The dense GEMM of the fp32 contract ("h3" arithmetic, csrc/h3.hpp: operands scaled by powers of
 * two and split exactly into fp16 hi + lo, products ah*bh + ah*bl + al*bh accumulated in fp32 on
 * the fp16 matrix cores, unscaled once: <= ~3 2^-22 |a b| per product) runs on a weight image packed
 * once: lidar_dense_x3_packed_size(k, cout) bytes, filled on the device by lidar_dense_x3_pack_f32
 * from W (k, cout) fp32 (fp16 hi / lo MFMA B fragments of W 2^s, K padded to 32, s in the image's
 * tail).  lidar_dense_x1_pack_f32 fills the same size with the bf16 image of the bf16 spec (X1). */
int64_t lidar_dense_x3_packed_size(int32_t k, int32_t cout);
int lidar_dense_x3_pack_f32(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed, void *stream);
int lidar_dense_x1_pack_f32(lidar_handle *h, const float *w, int32_t k, int32_t cout, void *packed, void *stream);

/* y = x W + b on that image (csrc/dense_x3s.hip): A = fp32 rows (rows, k) of row stride lda
 * (k % 4 == 0; elements k..lda-1 are read and must be finite), each wave scales and splits the
 * fragments it reads.  mode 0: y [ReLU] as fp32 rows (rows, ldo); mode 2: ReLU and max over runs
 * of pool_rows rows into fp32 (rows/pool_rows, ldo), out zeroed by the caller.  rows % 128 == 0,
 * cout % 128 == 0; o_plane is unused (0).  Mode flag 4 (mode 0 only, lidar_dense_x1_pack_f32's
 * image): one bf16 product per MFMA, bf16(x) bf16(w) in fp32 — the bf16 spec. */
int lidar_dense_x3f_f32(lidar_handle *h, const float *a, int32_t lda, int64_t rows, int32_t k, const void *packed,
                        const float *bias, int32_t cout, int32_t mode, int32_t relu_on, int32_t pool_rows, void *out,
                        int64_t o_plane, int64_t ldo, void *stream);

/* group_all's h3 chain (csrc/dense_x3s.hip): the same GEMM with the activations split ONCE, by the
 * producing layer.  A: fp32 rows (a_exp NULL; k % 4 == 0, lda % 4 == 0, elements k..lda-1 read and
 * finite) or h3 planes (a_exp (rows,) int32: |x| < 2^e per row; the fp16 hi plane (rows, lda) at a, the
 * lo plane at a + rows*lda halves, hi + lo = x 2^(14 - e) up to 2^-22; lda = k rounded up to 32, zeros
 * past k) — what mode 1 writes.  mode 0: fp32 rows (rows, ldo) [+ ReLU]; 1: h3 planes of y [+ ReLU]
 * (hi at out, lo at out + rows*ldo halves, ldo == cout) and out_exp (rows,): an exponent bound shared
 * by every column tile, 2^e_in w_colsum + b_max (w_colsum >= max_c sum_k |W_kc|, b_max >= max |b|,
 * the caller's, rounded up); 2: ReLU and max over runs of pool_rows rows (fp32, out zeroed by the
 * caller).  rows % 128 == 0, cout % 128 == 0; packed: lidar_dense_x3_pack_f32's image. */
int lidar_dense_h3p_f32(lidar_handle *h, const void *a, int32_t lda, int64_t rows, int32_t k, const int32_t *a_exp,
                        const void *packed, const float *bias, int32_t cout, int32_t mode, int32_t relu_on,
                        int32_t pool_rows, void *out, int32_t *out_exp, int64_t ldo, float w_colsum, float b_max,
                        void *stream);

/* SA branch in the bf16 spec (BASELINE configs[4]) on the fused 16-row kernel of
 * lidar_sa_group_mlp_x3_f32 with one bf16 product per MFMA: layer inputs and weights rounded to
 * bf16 (RNE), fp32 accumulation, bias / ReLU / max-pool in fp32.  layer1_mode 0 (xyz level):
 * p = the level's points (batch, n, 3), q = centres (batch, m, 3).  layer1_mode 2 (feature
 * level): p (batch*n, p_stride) = bf16(f) bf16(W1_f) + b1 per point (lidar_dense_x3f_f32 with
 * mode flag 4), xyz = the level's points, centres = (batch, m, 3); a grouped row's layer 1 is
 * relu(p[k] + bf16(W1_xyz) . bf16(x_k - c)).  packed: lidar_mlp_packed_size_x1(c1, c2, c3)
 * bytes from lidar_mlp_pack_x1_f32 (host).  Shapes: those of lidar_sa_group_mlp_x3_f32. */
int64_t lidar_mlp_packed_size_x1(int32_t c1, int32_t c2, int32_t c3);
int lidar_mlp_pack_x1_f32(int32_t c1, int32_t c2, int32_t c3, const float *w1, const float *b1, const float *w2,
                          const float *b2, const float *w3, const float *b3, void *packed);
int lidar_sa_group_mlp_x1_f32(lidar_handle *h, int32_t layer1_mode, const float *p, int64_t p_stride, const float *q,
                              const float *xyz, const float *centres, const int32_t *idx, int64_t batch, int64_t n,
                              int64_t m, int32_t nsample, int32_t c1, int32_t c2, int32_t c3, const void *packed,
                              float *out, int64_t out_stride, int64_t out_offset, void *stream);

/* Grouped shared MLP (3 layers, BN folded, ReLU) + max-pool over nsample for one SA branch,
 * fused with the grouping gather, on the native fp32 matrix cores (v_mfma_f32_16x16x4_f32,
 * 16 grouped rows per wave; the strict-fp32 path):
 *   row (b, c, s) = [xyz[b, idx[b,c,s]] - centres[b,c], feats[b, idx[b,c,s]]]
 *   out[b, c, out_offset + j] = max_s relu(...relu(row W1 + b1)... W3 + b3)[j]
 * xyz_level != 0 (a level without features): p = xyz (batch*n, 3), q = centres (batch*m, 3),
 * layer 1 runs in-kernel.  xyz_level = 0: layer 1 was applied per point beforehand — p
 * (batch*n, p_stride) = [f, x] W1 + b1 for every point of the level, q (batch*m, p_stride) =
 * centre W1_xyz (lidar_dense_f32 / lidar_dense_x3f_f32, relu off); a grouped row's layer 1 is
 * relu(p[k] - q[c]).
 * packed: the lidar_mlp_pack16_f32 image of lidar_mlp_packed_size16 floats (w1 is read only
 * for an xyz level: its 3 xyz rows).  Same outputs up to fp32 re-association. */
int64_t lidar_mlp_packed_size16(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3);
int lidar_mlp_pack16_f32(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3, const float *w1_host,
                         const float *b1_host, const float *w2_host, const float *b2_host,
                         const float *w3_host, const float *b3_host, float *packed_host);
int lidar_sa_group_mlp16_f32(lidar_handle *h, int32_t xyz_level, const float *p, int64_t p_stride,
                             const float *q, const int32_t *idx, int64_t batch, int64_t n,
                             int64_t m, int32_t nsample, int32_t c1, int32_t c2, int32_t c3,
                             const float *packed, float *out, int64_t out_stride,
                             int64_t out_offset, void *stream);

/* "x3" variants of the 16-row kernels: layers 2-3 in fp32 arithmetic carried by the bf16
 * matrix cores — every operand split exactly into bf16 hi + lo, products accumulated as
 * ah*bh + ah*bl + al*bh (v_mfma_f32_16x16x32_bf16, fp32 accumulation; error <= ~2^-15 per
 * product, within the fp32 path's 1e-4 contract).  Arguments as lidar_sa_group_mlp16_f32;
 * packed: lidar_mlp_pack_x3_f32's image of lidar_mlp_packed_size_x3 BYTES. */
int64_t lidar_mlp_packed_size_x3(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3);
int lidar_mlp_pack_x3_f32(int32_t xyz_level, int32_t c1, int32_t c2, int32_t c3, const float *w1_host,
                          const float *b1_host, const float *w2_host, const float *b2_host,
                          const float *w3_host, const float *b3_host, void *packed_host);
int lidar_sa_group_mlp_x3_f32(lidar_handle *h, int32_t xyz_level, const float *p, int64_t p_stride,
                              const float *q, const int32_t *idx, int64_t batch, int64_t n,
                              int64_t m, int32_t nsample, int32_t c1, int32_t c2, int32_t c3,
                              const void *packed, float *out, int64_t out_stride,
                              int64_t out_offset, void *stream);

/* An xyz level's SA branch with its ball queries answered inside the MLP kernel: grid =
 * lidar_ball_query_bin_f32(xyz, radius, nsample) for these frames; each wavefront queries its
 * centre from the grid into LDS, then groups, runs the MLP and max-pools.  Equal bit for bit to
 * lidar_ball_query_binned_f32 followed by lidar_sa_group_mlp_x3_f32 (x1 = 0; packed from
 * lidar_mlp_pack_x3_f32 with xyz_level = 1) or lidar_sa_group_mlp_x1_f32 mode 0 (x1 = 1; packed
 * from lidar_mlp_pack_x1_f32).  xyz (batch, n, 3), centres (batch, m, 3); out_idx (batch, m,
 * nsample) int32 or NULL receives the ball-query indices.  Shapes: (c1, c2, c3, nsample) in
 * {(64, 64, 128, 32), (32, 32, 64, 16), (64, 96, 128, 128)}.  Replaces, for these levels, the
 * pointnet2 `ball_query` + `group_points` + shared-MLP sequence behind the north_star's SA layer
 * (no reference counterpart: SURVEY §0). */
int lidar_sa_group_mlp_bq_f32(lidar_handle *h, int32_t x1, const float *xyz, const void *grid, const float *centres,
                              int64_t batch, int64_t n, int64_t m, float radius, int32_t nsample, int32_t c1,
                              int32_t c2, int32_t c3, const void *packed, float *out, int64_t out_stride,
                              int64_t out_offset, int32_t *out_idx, void *stream);

/* A set-abstraction branch of any shape (csrc/sa_generic.hip; the fused kernels above cover six):
 * grouped rows -> the dense GEMMs (lidar_dense_x3f_f32 / lidar_dense_f32, one per layer, ReLU)
 * -> the max over each group's nsample rows.  Replaces, for every other (c1, c2, c3, nsample),
 * pointnet2's QueryAndGroup(use_xyz) + shared MLP + max_pool2d of PointnetSAModuleMSG.forward.
 *
 * lidar_sa_group_rows_f32: rows_out[(b*m + j)*nsample + s] = [feat[b*n + idx] (cfeat columns,
 * row stride ldf; feat may be NULL when cfeat = 0), xyz[b*n + idx] - centres[b*m + j] (fp32),
 * zeros to ldr]; rows_out rows [batch*m*nsample, rows) are zeroed.  ldr % 4 == 0, ldr >= cfeat + 3.
 * lidar_group_max_f32: out[g*ldo + out_offset + c] = max_s in[(g*nsample + s)*ldi + c], c < C,
 * g < groups (a NaN propagates). */
int lidar_sa_group_rows_f32(lidar_handle *h, const float *feat, int64_t ldf, int32_t cfeat, const float *xyz,
                            const float *centres, const int32_t *idx, int64_t batch, int64_t n, int64_t m,
                            int32_t nsample, float *rows_out, int64_t rows, int64_t ldr, void *stream);
int lidar_group_max_f32(lidar_handle *h, const float *in, int64_t ldi, int64_t groups, int32_t nsample, int32_t c,
                        float *out, int64_t ldo, int64_t out_offset, void *stream);

/* y (batch*m, ldy) columns [col0, col0+3) = xyz rows; columns [col0+3, ldy) zeroed —
 * builds group_all's input [feats, xyz, 0-pad] next to features already in y. */
int lidar_concat_xyz_pad_f32(lidar_handle *h, const float *xyz, int64_t rows, float *y,
                             int64_t ldy, int64_t col0, void *stream);

/* voxel downsample.  The voxel of a point is calculate_grid_density's grid hash
 * (utils/data_processing.py:305-319) per axis: edges np.arange(lo - 2v, (hi + 2v) + v, v) over the
 * frame's extent, histogram2d's searchsorted-right binning with the last edge closed; key =
 * (bx*ny + by)*nz + bz.  Per-point voxel id (rank of its key, ascending; -1 outside every bin),
 * centroids (sequential fp32 sums in point order / count), counts; *nvox_host receives V
 * (synchronises `stream`).  centroids/counts must hold n entries.  LIDAR_EINVAL when the extent
 * is not finite or the grid has 2^32 keys or more. */
int lidar_voxel_downsample_f32(lidar_handle *h, const float *xyz, int64_t n, double voxel,
                               int32_t *voxel_id, float *centroids, int32_t *counts,
                               int64_t *nvox_host, void *stream);

/* Voxel downsampling of `batch` frames of n points over the whole chip (csrc/voxel_batch.hip):
 * xyz (batch, n, 3) fp32; voxel_id (batch, n) int32; centroids (batch, n, 3) and counts (batch, n),
 * the first nvox[f] rows of frame f valid; nvox (batch,) int32 on the device (-1: the frame's extent
 * is not finite or its grid has 2^32 keys or more; library bugs, never expected, and sticky — they win over
 * the count: -2 a bounded in-launch wait timed out, -3 an inconsistent bucket table).  No host
 * synchronisation; per frame equal to lidar_voxel_downsample_f32.  Workspace:
 * lidar_voxel_batch_workspace_bytes(batch, n), plus the handle's own voxel tag block (the in-launch
 * hand-offs' epoch-tagged granules, 8 KiB per 8 192-point tile; grown and zeroed on demand, written by
 * voxel calls only).  Calls on one handle must not run concurrently (as for the workspace). */
uint64_t lidar_voxel_batch_workspace_bytes(int64_t batch, int64_t n);
int lidar_voxel_downsample_batch_f32(lidar_handle *h, const float *xyz, int64_t batch, int64_t n, double voxel,
                                     int32_t *voxel_id, float *centroids, int32_t *counts, int32_t *nvox,
                                     void *stream);

/* ======================================================= Tier R (density path)
 * Bit-exact replacements for the reference's CPU path. */

/* eps-ball neighbour count over scaled points (self included, fp64,
 * ((dx*dx+dy*dy)+dz*dz) <= eps*eps) and DBSCAN labels (min_samples).  Replaces
 * sklearn DBSCAN(eps, min_samples).fit(x).labels_ at utils/data_processing.py:197. */
int lidar_dbscan_f64(lidar_handle *h, const double *x, int64_t n, double eps, int32_t min_samples,
                     int64_t *labels, int32_t *counts, void *stream);

/* KDTree(x).query_radius(x, r, count_only=True): counts[i] = #{j : ((dx*dx+dy*dy)+dz*dz)
 * <= r*r} in fp64, i itself included (utils/visualization.py:41-48, :165-168;
 * app_simplified.py:156-159).  x (n, 3) device; 2-D data with z = 0.  Synchronises. */
int lidar_radius_count_f64(lidar_handle *h, const double *x, int64_t n, double r, int64_t *counts,
                           void *stream);

/* np.histogram2d(a, b, bins=(bx, by), range=...) counts (float64, bx*by row-major) with
 * numpy's edges passed in (xedges bx+1, yedges by+1, device): searchsorted-right bins, the
 * last edge closed, outside / NaN dropped (utils/visualization.py:125-137). */
int lidar_histogram2d_f64(lidar_handle *h, const double *a, const double *b, int64_t n, const double *xedges,
                          int64_t bx, const double *yedges, int64_t by, double *counts, void *stream);

/* Host-only: the PCD / PLY ASCII data section of load_lidar_data (utils/data_processing.py
 * :43-104).  From 0-based line `first` (max_lines < 0: to the end; else that many lines),
 * every line with >= 3 whitespace-separated tokens yields float(tok0..2) into out (3 per
 * point, cap points); *n_out = points written.  LIDAR_EPARSE: some token needs Python's own
 * float() (the caller falls back to the reference's loop for the exact result / error). */
int lidar_parse_ascii_xyz(const char *buf, int64_t len, int64_t first, int64_t max_lines, double *out,
                          int64_t cap, int64_t *n_out);

/* Whole preprocess_lidar_data (utils/data_processing.py:127-229) on one frame already in
 * device memory (n >= 1 points, (n,3) f64).  Outputs (device, caller-allocated with n rows):
 *   mask (n) u8 inlier flag; colors, normals, compact_xyz (n,3) f64 of the inliers in input
 *   order (first n_in rows valid); labels (n) int64 over the inliers (ground -1);
 *   scalars (64 f64):
 *   [0] n_in  [1] n_ground  [2] n_nonground  [3] z_threshold  [4] eps  [5..10] x/y/z min,max
 *   [11..14] ground plane  [15] status (0 ok, 1 = no inliers -> reference IndexError)
 *   [16..18] 3-sigma mean  [19..21] std  [22..24] scaler mean  [25..27] scaler scale
 *   [28..33] scaled bbox  [39] n_clusters  [40] plane kind (0 lstsq, 1 min-z fallback,
 *   2 rank-deficient ground).  Asynchronous on `stream`. */
int lidar_preprocess_f64(lidar_handle *h, const double *xyz, int64_t n, uint8_t *mask,
                         double *colors, double *normals, double *compact_xyz, int64_t *labels,
                         double *scalars, void *stream);

/* lidar_preprocess_f64 over `frames` frames in one launch per phase (frames in
 * CSR layout).  xyz: the frames' rows concatenated; offsets: DEVICE int64[frames + 1] row
 * offsets (frame f = rows [offsets[f], offsets[f+1])); max_n >= every frame's size.  The
 * per-point outputs use the same row offsets (a frame's compact_xyz / labels rows start at
 * offsets[f] and run for its own n_in = scalars[f*64 + 0]); scalars holds 64 doubles per
 * frame, with [15] status: 0 ok, 1 no inlier (IndexError), 2 empty frame (ValueError). */
int lidar_preprocess_batch_f64(lidar_handle *h, const double *xyz, const int64_t *offsets, int32_t frames,
                               int64_t max_n, uint8_t *mask, double *colors, double *normals,
                               double *compact_xyz, int64_t *labels, double *scalars, void *stream);

/* The Streamlit apps' variant preprocess_point_cloud (app_simplified.py:76-137,
 * app_with_db.py:80-141): lidar_preprocess_batch_f64's phases, then DBSCAN(eps,
 * min_samples=5) on the UNSCALED non-ground points (no StandardScaler / eps heuristic;
 * the reference passes eps = 0.3).  offsets == NULL: one frame of max_n points.  Same
 * outputs and status codes; scalars [22..27] = 0 / 1 and [28..33] = the unscaled bbox. */
int lidar_preprocess_eps_batch_f64(lidar_handle *h, const double *xyz, const int64_t *offsets,
                                   int32_t frames, int64_t max_n, double eps, uint8_t *mask,
                                   double *colors, double *normals, double *compact_xyz,
                                   int64_t *labels, double *scalars, void *stream);

/* The variant's analyze_crowd_density grid (app_simplified.py:262-282): for the edges xg
 * (nxg), yg (nyg) (np.arange, device), out (nyg-1, nxg-1) row-major [j][i] = #{people p :
 * (cx-px)^2 + (cy-py)^2 <= r*r} / divisor with centre ((xg[i]+xg[i+1])/2, (yg[j]+yg[j+1])/2)
 * — len(KDTree(people).query_radius([centre], r)[0]) / divisor.  people (k, 2) device. */
int lidar_cell_radius_density_f64(lidar_handle *h, const double *people, int64_t k, const double *xg,
                                  int64_t nxg, const double *yg, int64_t nyg, double r, double divisor,
                                  double *out, void *stream);

/* Optional global density over a FIXED venue grid (the reference derives its grid
 * per frame, models/crowd_density_model.py:49-54): counts (nx, ny) int32 += the histogram2d of
 * people (k, 2) over calculate_grid_density's edges (utils/data_processing.py:305-319:
 * np.arange(x0, ., grid) with x0 = x_min - 2 grid, searchsorted right, the last edge closed,
 * outside dropped).  Counts add, so the frames of a rank and then (one RCCL all-reduce, int32
 * sum) the ranks accumulate; counts / grid^2 is calculate_grid_density of all their people. */
int lidar_venue_counts_f64(lidar_handle *h, const double *people, int64_t k, double x0, double y0, double grid,
                           int64_t nx, int64_t ny, int32_t *counts, void *stream);

/* downsample_point_cloud's gather (utils/data_processing.py:247-249): dst[r] = src[idx[r]] for k
 * rows of row_bytes bytes each (any dtype: rows are moved as raw bytes); idx (k) int64 device,
 * the indices the host drew from the global legacy NumPy RNG (out-of-range indices skipped). */
int lidar_gather_rows(lidar_handle *h, const void *src, int64_t n_rows, int64_t row_bytes, const int64_t *idx,
                      int64_t k, void *dst, void *stream);

/* ---- models/crowd_flow_model.py, HOST code (host pointers): the
 * model's deciding arithmetic is glibc sin / cos / pow and sklearn's KD-tree traversal,
 * reproduced bit for bit on the host.
 * _generate_simulated_flow (crowd_flow_model.py:88-184) after its RNG draws: positions
 * (nx*ny, 2) = meshgrid(x_grid, y_grid) raveled, vectors (m, 2), magnitudes (m);
 * bottlenecks (nb, 2) = the (x, y) uniform draws. */
int lidar_flow_field_f64(const double *x_grid, int64_t nx, const double *y_grid, int64_t ny, double exit_x,
                         double exit_y, int32_t complexity, const double *bottlenecks, int32_t nb,
                         double speed_min, double speed_max, double *positions, double *vectors,
                         double *magnitudes);
/* _identify_bottlenecks (crowd_flow_model.py:186-279): nodes with magnitude <= slow, >=
 * min_close neighbours within r_close and >= min_far more within r_far (sklearn KDTree
 * query_radius order), severity > 1 -> (out_x, out_y, out_severity = min(10, round())) in
 * node order (out_raw: the unrounded severity, optional); *n_out = candidates. */
int lidar_flow_bottlenecks_f64(const double *positions, const double *vectors, const double *magnitudes,
                               int64_t m, double slow, double r_close, double r_far, int32_t min_close,
                               int32_t min_far, double *out_x, double *out_y, int64_t *out_severity,
                               double *out_raw, int64_t cap, int64_t *n_out);
/* sklearn KDTree(x, leaf_size).get_arrays()[1]: the build's index permutation (x (n, d)). */
int lidar_kdtree_order_f64(const double *x, int64_t n, int32_t d, int32_t leaf_size, int64_t *perm);

/* extract_people_positions for every frame of a preprocess batch: people rows of frame f
 * start at row offsets[f] (K_f rows); kdev (device int64[frames]) receives K_f.  Async. */
int lidar_people_batch_f64(lidar_handle *h, const double *compact_xyz, const int64_t *labels,
                           const int64_t *offsets, int32_t frames, int64_t max_n, const double *scalars,
                           double *people, int64_t *kdev, void *stream);

/* the density grid + statistics + hotspots of every frame with K_f > 0.  jobs: device
 * double[8 * frames] rows (xa = x_min - 2g, ya = y_min - 2g, g, nx, ny (lidar_grid_dims),
 * output offset, scratch offset, 0); out at a frame's offset: grid_x (nx) | grid_y (ny) |
 * density (nx*ny) | flat_x | flat_y | stats (8) | hot (5 int64); scratch_doubles = sum over
 * frames of nx*ny + ceil(nx*ny/2) + nx + ny + 2.  Asynchronous. */
int lidar_density_batch_f64(lidar_handle *h, const double *people, const int64_t *offsets,
                            const int64_t *kdev, int32_t frames, const double *jobs, double *out,
                            int64_t scratch_doubles, void *stream);

/* people positions (extract_people_positions, utils/data_processing.py:251-280):
 * centroid (x, y) of every label >= 0, sequential index-order sums;
 * people (n,2) f64, *k_host receives K (synchronises). */
int lidar_people_f64(lidar_handle *h, const double *xyz, const int64_t *labels, int64_t n,
                     double *people, int64_t *k_host, void *stream);

/* grid density (calculate_grid_density, utils/data_processing.py:282-328, and the statistics
 * of CrowdDensityModel.analyze, models/crowd_density_model.py:56-82): np.arange edges
 * a + i*((a+g)-a), histogram2d binning (searchsorted right, last edge closed), /g^2.
 * lidar_grid_dims gives nx, ny (host arithmetic of np.arange's length).  Outputs: grid_x (nx),
 * grid_y (ny); `density` must hold 3*nx*ny + 13 doubles laid out as
 *   density (nx*ny) | flat_x (nx*ny) | flat_y (nx*ny) | stats (8) | hotspot index (5, int64)
 * stats = [max, avg of occupied cells (numpy pairwise mean), threshold, n_hotspots,
 * n_occupied, k].  Synchronises `stream`. */
int lidar_grid_dims(double xmin, double xmax, double ymin, double ymax, double grid,
                    int64_t *nx, int64_t *ny);
int lidar_density_grid_f64(lidar_handle *h, const double *people, int64_t k, double xmin,
                           double xmax, double ymin, double ymax, double grid, int64_t nx,
                           int64_t ny, double *grid_x, double *grid_y, double *density,
                           void *stream);

#ifdef __cplusplus
}
#endif
#endif
