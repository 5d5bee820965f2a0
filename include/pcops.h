/*
 * pcops.h -- C-ABI of libpcops.so, the MI355X (gfx950) implementation of the
 * SVDFormer / PointSea per-batch completion hot path.
 *
 * Conventions (all entry points):
 *   - plain device pointers (fp32 / int32, C-contiguous) and sizes, no torch
 *     types; every function launches asynchronously on `stream` (a
 *     hipStream_t; NULL = the legacy default stream) and never allocates,
 *     frees or synchronises, so callers may capture it into a hipGraph;
 *   - outputs are fully written (the reference zero-initialises them in
 *     C++/Python -- sampling.cpp:25-27, dist_chamfer_3D.py:33-42,56-60 -- so
 *     "zero + accumulate" outputs are zeroed here with hipMemsetAsync);
 *   - scratch is caller-provided through `workspace` (size from the matching
 *     *_workspace_bytes query);
 *   - the return value is a status code (PCOPS_OK == 0).  The reference
 *     exits the process (cuda_utils.h:30-39) or prints and returns 0/-1
 *     (chamfer3D.cu:145-151, emd_cuda.cu:236-249); here nothing exits and
 *     pcops_status_string() gives the message the Python shim raises.
 *
 * Each declaration cites the reference interface it replaces (path:line in
 * shiyuan0806/SVDFormer_PointSea).
 */
#ifndef PCOPS_H_
#define PCOPS_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *pcops_stream_t; /* == hipStream_t */

enum pcops_status {
  PCOPS_OK = 0,
  PCOPS_ERR_INVALID = 1,   /* bad sizes / null pointers */
  PCOPS_ERR_LAUNCH = 2,    /* hipGetLastError after a launch */
  PCOPS_ERR_WORKSPACE = 3, /* workspace missing or too small */
  PCOPS_ERR_UNSUPPORTED = 4
};

const char *pcops_status_string(int status);
/* version of the ABI below; bumped on any signature change */
int pcops_abi_version(void);

/* ---------------- pointnet2_ops (bindings.cpp:6-19) ---------------- */

/* furthest_point_sampling(points, nsamples): sampling.cpp:66-87,
 * sampling_gpu.cu:69-229.  xyz (B,N,3) -> idx (B,M) int32.
 * workspace: pcops_fps_workspace_bytes(B,N) bytes (0 when the cloud fits
 * the register-resident kernel, N <= 16384). */
unsigned long long pcops_fps_workspace_bytes(int B, int N);
int pcops_furthest_point_sampling(const float *xyz, int B, int N, int M, int *idx, void *workspace,
                                  unsigned long long workspace_bytes, pcops_stream_t stream);
/* The same over zero-padded clouds whose valid rows are known: counts (B,) int32 on the device;
 * row k >= counts[b] of cloud b is absent -- the result equals pcops_furthest_point_sampling on the
 * buffer whose rows >= counts[b] are zero (sampling_gpu.cu:100-101 skips |p|^2 <= 1e-3 rows), and
 * the sweep stops at the count.  Caller: seprate_point_cloud's batched crop (utils/helpers.py:
 * 79-119 runs FPS per sample on the ragged clouds). Same workspace as above. */
int pcops_furthest_point_sampling_counts(const float *xyz, const int *counts, int B, int N, int M, int *idx,
                                         void *workspace, unsigned long long workspace_bytes,
                                         pcops_stream_t stream);
/* seprate_point_cloud's crop (utils/helpers.py:96-111: torch.argsort of the distances to the crop centre,
 * then idx[num_crop:] / idx[:num_crop] of each sample), batched: dist (B,N) fp32, xyz (B,N,3) fp32; the
 * points of cloud b ordered by distance ascending (ties by point index, NaN last), ranks
 * start[b] .. start[b] + count[b] - 1 written to rows 0.. of out (B,n_max,3), rows j >= count[b] hold
 * the rank-(start[b]+j, clamped to N-1) point times 0; counts (B) int32 <- count[b] (may be NULL).
 * start / count int64 (B) on the device; count NULL means N - start[b].  N <= 16384. */
int pcops_crop_pack(const float *dist, const float *xyz, const long long *start, const long long *count, int B, int N,
                    int n_max, float *out, int *counts, pcops_stream_t stream);

/* gather_points(points, idx): sampling.cpp:15-38, sampling_gpu.cu:8-30.
 * points (B,C,N), idx (B,M) -> out (B,C,M). */
int pcops_gather_points(const float *points, const int *idx, int B, int C, int N, int M, float *out,
                        pcops_stream_t stream);
/* gather_points_grad(grad_out, idx, n): sampling.cpp:40-64, sampling_gpu.cu:34-57.
 * grad_out (B,C,M) -> grad_points (B,C,N) (overwritten). */
int pcops_gather_points_grad(const float *grad_out, const int *idx, int B, int C, int N, int M, float *grad_points,
                             pcops_stream_t stream);

/* group_points(points, idx): group_points.cpp:12-36, group_points_gpu.cu:8-39.
 * points (B,C,N), idx (B,S,K) -> out (B,C,S,K). */
int pcops_group_points(const float *points, const int *idx, int B, int C, int N, int S, int K, float *out,
                       pcops_stream_t stream);
/* group_points_grad(grad_out, idx, n): group_points.cpp:38-62, group_points_gpu.cu:43-75. */
int pcops_group_points_grad(const float *grad_out, const int *idx, int B, int C, int N, int S, int K,
                            float *grad_points, pcops_stream_t stream);

/* Fused SA-module grouping: sample_and_group_knn (models/model_utils.py:323-356)
 * from the kNN indices onward, written in the channels_last layout the first
 * 1x1 conv reads.  xyz (B,N,3), new_xyz (B,S,3), points_t (B,N,C) token-major
 * (NULL when C == 0), idx (B,S,K) -> out (B,S,K,3+C) row-major:
 *   out[b,s,k,c<3]  = xyz[b,idx,c] - new_xyz[b,s,c]      (grouped_xyz - centre)
 *   out[b,s,k,3+c]  = points_t[b,idx,c]                  (grouped points)
 * out_dtype 0 = fp32, 1 = bf16 (rounded once).  Replaces group_points x 2,
 * the repeat/subtract, torch.cat and the channels_last copy. */
int pcops_sa_group(const float *xyz, const float *new_xyz, const float *points_t, const int *idx, int B, int N, int S,
                   int K, int C, void *out, int out_dtype, pcops_stream_t stream);
/* grad_points_t (B,N,C) fp32, overwritten: scatter-add of grad_out[..., 3:] by idx
 * (group_points_gpu.cu:43-64, token-major).  grad_dtype 0 = fp32, 1 = bf16. */
int pcops_sa_group_grad(const void *grad_out, int grad_dtype, const int *idx, int B, int N, int S, int K, int C,
                        float *grad_points_t, pcops_stream_t stream);

/* EdgeConv edge features (models/model_utils.py:847-881, models_PointSea/model_utils.py:551-585):
 * group_local's neighbour gather (:812-845), `central - neigh`, torch.cat((edge, central), 1) and
 * the channels_last copy of the first 1x1 conv's input in one pass.  x (B,N,C) token-major fp32,
 * idx (B,N,K) int32 (the feature-space kNN) -> out (B,N,K,2C) row-major:
 *   out[b,n,k,c] = x[b,n,c] - x[b,idx,c],  out[b,n,k,C+c] = x[b,n,c]
 * out_dtype 0 = fp32, 1 = bf16 (the difference rounded once). */
int pcops_edge_group(const float *x, const int *idx, int B, int N, int K, int C, void *out, int out_dtype,
                     pcops_stream_t stream);
/* grad_x (B,N,C) fp32, overwritten: sum_k (g[b,n,k,c] + g[b,n,k,C+c]) minus the scatter of
 * g[..., :C] by idx (index_points' backward).  grad_dtype 0 = fp32, 1 = bf16. */
int pcops_edge_group_grad(const void *grad_out, int grad_dtype, const int *idx, int B, int N, int K, int C,
                          float *grad_x, pcops_stream_t stream);

/* pcops_max_k: torch.max(x, dim=3) of a (B, C, S, K) conv output held channels_last, i.e. over
 *   the middle dim of a contiguous (rows = B*S, K, C) tensor (models/model_utils.py:354, 862-864):
 *   out[r][c] = max_k x[r][k][c], arg[r][c] = the first maximising k (NaN is the maximum, as
 *   torch).  dtype 0 fp32 / 1 bf16 for x and out; C % 8 == 0, K <= 255.
 * pcops_max_k_grad: grad_x[r][k][c] = k == arg[r][c] ? grad_out[r][c] : 0 (fully written). */
int pcops_max_k(const void *x, int dtype, long long rows, int K, int C, void *out, unsigned char *arg,
                pcops_stream_t stream);
int pcops_max_k_grad(const void *grad_out, int dtype, const unsigned char *arg, long long rows, int K, int C,
                     void *grad_x, pcops_stream_t stream);

/* ball_query(new_xyz, xyz, radius, nsample): ball_query.cpp:8-32, ball_query_gpu.cu:9-54.
 * new_xyz (B,M,3), xyz (B,N,3) -> idx (B,M,nsample). */
int pcops_ball_query(const float *new_xyz, const float *xyz, int B, int N, int M, float radius, int nsample, int *idx,
                     pcops_stream_t stream);

/* three_nn(unknowns, knows): interpolate.cpp:14-39, interpolate_gpu.cu:9-68.
 * unknown (B,N,3), known (B,M,3) -> dist2 (B,N,3) squared, idx (B,N,3). */
int pcops_three_nn(const float *unknown, const float *known, int B, int N, int M, float *dist2, int *idx,
                   pcops_stream_t stream);
/* three_interpolate(points, idx, weight): interpolate.cpp:40-68, interpolate_gpu.cu:72-111.
 * points (B,C,M), idx/weight (B,N,3) -> out (B,C,N). */
int pcops_three_interpolate(const float *points, const int *idx, const float *weight, int B, int C, int M, int N,
                            float *out, pcops_stream_t stream);
/* three_interpolate_grad(grad_out, idx, weight, m): interpolate.cpp:69-99, interpolate_gpu.cu:116-154. */
int pcops_three_interpolate_grad(const float *grad_out, const int *idx, const float *weight, int B, int C, int N,
                                 int M, float *grad_points, pcops_stream_t stream);

/* ---------------- kNN (models/model_utils.py:258-286, :807-845) ----------------
 * query_knn / query_knn_point: K nearest points of p for every query q, in
 * ascending (squared distance, index) order; distance evaluated exactly as
 * square_distance's fp32 torch expression.  q (B,S,C), p (B,N,C) channel-last;
 * pad leading neighbours are skipped (query_knn include_self=False -> 1).
 * idx (B,S,K) int32; dist (B,S,K) optional (may be NULL).  C <= 512, K+pad <= 64. */
int pcops_knn(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx, float *dist,
              pcops_stream_t stream);
/* The same with scratch (pcops_knn_workspace_bytes(B, S, N, C, K + pad); 0 = none needed): a
 * feature-space search (C >= 32, C % 4 == 0, K + pad <= 32) streams the candidates split over
 * blocks (knnC3_kernel) and merges the partial sorted lists as (distance, index) pairs -- the same
 * output bit for bit; every other case, or a short workspace, is pcops_knn. */
unsigned long long pcops_knn_workspace_bytes(int B, int S, int N, int C, int K);
int pcops_knn_ws(const float *q, const float *p, int B, int S, int N, int C, int K, int pad, int *idx, float *dist,
                 void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);

/* ---------------- Chamfer (metrics/CD/chamfer3D) ----------------
 * chamfer_3D.forward(xyz1, xyz2, dist1, dist2, idx1, idx2): chamfer_cuda.cpp:17-33,
 * chamfer3D.cu:12-154. */
int pcops_chamfer_forward(const float *xyz1, const float *xyz2, int B, int N, int M, float *dist1, float *dist2,
                          int *idx1, int *idx2, pcops_stream_t stream);
/* pcops_chamfer_forward_ws: pcops_chamfer_forward through a spatially culled search for large clouds
 *   (N, M >= 256, N * M >= 2^24, both <= 32768): both clouds counting-sorted by a 16^3 Morton cell code, targets in
 *   64-point tiles with exact boxes, each wave (64 sorted queries) taking tiles nearest-first and
 *   skipping every tile beyond its queries' bounds under a rigorous fp32 margin; the reference's
 *   distance bits and lowest-index tie rule, including its non-finite behaviour (culling off for a
 *   batch holding a non-finite coordinate).  workspace:
 *   pcops_chamfer_workspace_bytes (0: the sizes take pcops_chamfer_forward, as does a short
 *   workspace).  Replaces the same call as pcops_chamfer_forward (chamfer_cuda.cpp:17-24). */
unsigned long long pcops_chamfer_workspace_bytes(int B, int N, int M);
int pcops_chamfer_forward_ws(const float *xyz1, const float *xyz2, int B, int N, int M, float *dist1, float *dist2,
                             int *idx1, int *idx2, void *workspace, unsigned long long workspace_bytes,
                             pcops_stream_t stream);
/* chamfer_3D.backward(xyz1, xyz2, gradxyz1, gradxyz2, graddist1, graddist2, idx1, idx2):
 * chamfer3D.cu:155-195.  gradxyz1/2 are overwritten. */
int pcops_chamfer_backward(const float *xyz1, const float *xyz2, int B, int N, int M, const float *graddist1,
                           const float *graddist2, const int *idx1, const int *idx2, float *gradxyz1, float *gradxyz2,
                           pcops_stream_t stream);
/* pcops_chamfer_sqrt_mean_grad: the distance gradients of the sqrt-mean Chamfer losses
 * (utils/loss_utils.py:10-31 chamfer_sqrt / chamfer_single_side_sqrt: torch.sqrt, torch.mean and
 * "/ 2" on dist1 / dist2) in autograd's order, from the loss gradient grad_out (one float on the
 * device), scale (0.5 for chamfer_sqrt, 1 single-sided) and the forward's s = sqrt(dist) (n1 / n2
 * elements; s2 NULL: gd2 = 0):  gd = ((g * scale) * (1 / n)) / (2 s).  Feeds pcops_chamfer_backward;
 * replaces the autograd chain between the loss and chamfer_3D.backward (dist_chamfer_3D.py:56-60). */
int pcops_chamfer_sqrt_mean_grad(const float *grad_out, float scale, const float *s1, long long n1, const float *s2,
                                 long long n2, float *gd1, float *gd2, pcops_stream_t stream);

/* ---------------- 3x3 / stride 2 / pad 1 max pool (torchvision resnet stem, PointSea ResEncoder)
 * pcops_maxpool3s2_fwd: nn.MaxPool2d(3, 2, 1) on a channels_last (N, H, W, C) activation (dtype 0
 * fp32, 1 bf16) -> y (N, ceil(H/2), ceil(W/2), C) and each output's winning window offset (uint8,
 * 3 i + j), torch's NHWC rule (first maximum, a NaN takes the slot).  pcops_maxpool3s2_bwd: the
 * input gradient, per element the gradients of the windows it won summed in fp32 in (ph, pw) order
 * (max_pool_backward_nhwc).  Replaces torch's max_pool2d_with_indices(_backward) for that pool
 * (models_PointSea/PointSea.py:37-61, torchvision resnet18 maxpool). */
int pcops_maxpool3s2_fwd(const void *x, int dtype, int N, int H, int W, int C, void *y, unsigned char *argmax,
                         pcops_stream_t stream);
int pcops_maxpool3s2_bwd(const void *gy, const unsigned char *argmax, int dtype, int N, int H, int W, int C, void *gx,
                         pcops_stream_t stream);

/* ---------------- EMD (metrics/EMD) ----------------
 * emd.forward(xyz1, xyz2, dist, assignment, price, assignment_inv, bid, bid_increments,
 *             max_increments, unass_idx, unass_cnt, unass_cnt_sum, cnt_tmp, max_idx, eps, iters):
 * emd.cpp:14-31, emd_cuda.cu:23-282.  The reference's 12 scratch tensors are
 * one workspace here.  n must equal m; deterministic auction. */
unsigned long long pcops_emd_workspace_bytes(int B, int n);
int pcops_emd_forward(const float *xyz1, const float *xyz2, int B, int n, float eps, int iters, float *dist,
                      int *assignment, void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* emd.backward(xyz1, xyz2, gradxyz, graddist, idx): emd_cuda.cu:284-316 (grad for xyz1 only; overwritten). */
int pcops_emd_backward(const float *xyz1, const float *xyz2, const float *graddist, const int *assignment, int B, int n,
                       float *gradxyz1, pcops_stream_t stream);

/* ---------------- attention core (nn.MultiheadAttention inside
 * self_attention / cross_attention, models/model_utils.py:542-617) ----------------
 * O = softmax(scale * Q K^T) V per (batch, head), flash-style (no L x L
 * matrix in HBM).  Element (b, h, row, d) of each tensor is read at
 * base + b*sb + h*sh + row*srow + d (elements), so nn.MultiheadAttention's
 * seq-first (L, B, H*hd) projections [sb = H*hd, sh = hd, srow = B*H*hd] and
 * batch-first (B, L, H*hd) tensors [sb = L*H*hd, sh = hd, srow = H*hd] are used
 * in place.  dtype 0 = fp32 (exact f32 MFMA, parity build), 1 = bf16 in/out
 * with fp32 accumulation.  lse (B*H, Lq) fp32 log-sum-exp (natural log) for
 * the backward.  head_dim D in {32, 64, 96, 128}; pointers and strides must be
 * 16-byte aligned (else PCOPS_ERR_UNSUPPORTED). */
int pcops_attention_forward(const void *q, const void *k, const void *v, void *o, float *lse, int B, int H, int Lq,
                            int Lk, int D, float scale, int dtype, long long q_sb, long long q_sh, long long q_srow,
                            long long k_sb, long long k_sh, long long k_srow, long long v_sb, long long v_sh,
                            long long v_srow, long long o_sb, long long o_sh, long long o_srow, pcops_stream_t stream);
/* Backward of the above (dq/dk/dv use the q/k/v strides, dout the o strides).
 * workspace: pcops_attention_bwd_workspace_bytes(B, H, Lq, Lk, D). */
unsigned long long pcops_attention_bwd_workspace_bytes(int B, int H, int Lq, int Lk, int D);
int pcops_attention_backward(const void *q, const void *k, const void *v, const void *o, const void *dout,
                             const float *lse, void *dq, void *dk, void *dv, int B, int H, int Lq, int Lk, int D,
                             float scale, int dtype, long long q_sb, long long q_sh, long long q_srow, long long k_sb,
                             long long k_sh, long long k_srow, long long v_sb, long long v_sh, long long v_srow,
                             long long o_sb, long long o_sh, long long o_srow, void *workspace,
                             unsigned long long workspace_bytes, pcops_stream_t stream);
/* The three launches of pcops_attention_backward, exposed separately so a
 * caller can time or overlap them: delta = rowsum(dO o O) into workspace,
 * then dQ (query-on-lane pass), then dK/dV (key-on-lane pass). */
int pcops_attention_bwd_preprocess(const void *o, const void *dout, int B, int H, int Lq, int D, int dtype,
                                   long long o_sb, long long o_sh, long long o_srow, void *workspace,
                                   unsigned long long workspace_bytes, pcops_stream_t stream);
int pcops_attention_bwd_dq(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                           void *dq, int B, int H, int Lq, int Lk, int D, float scale, int dtype, long long q_sb,
                           long long q_sh, long long q_srow, long long k_sb, long long k_sh, long long k_srow,
                           long long v_sb, long long v_sh, long long v_srow, long long o_sb, long long o_sh,
                           long long o_srow, const void *workspace, unsigned long long workspace_bytes,
                           pcops_stream_t stream);
/* preprocess + dQ in one launch (bf16): each query lane forms its delta from the dO
 * fragment it holds and the matching chunks of o, writes it to workspace for the dK/dV
 * pass, and computes dQ.  fp32 falls back to the two launches above. */
int pcops_attention_bwd_dq_delta(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                 const float *lse, void *dq, int B, int H, int Lq, int Lk, int D, float scale,
                                 int dtype, long long q_sb, long long q_sh, long long q_srow, long long k_sb,
                                 long long k_sh, long long k_srow, long long v_sb, long long v_sh, long long v_srow,
                                 long long o_sb, long long o_sh, long long o_srow, void *workspace,
                                 unsigned long long workspace_bytes, pcops_stream_t stream);
int pcops_attention_bwd_dkv(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                            void *dk, void *dv, int B, int H, int Lq, int Lk, int D, float scale, int dtype,
                            long long q_sb, long long q_sh, long long q_srow, long long k_sb, long long k_sh,
                            long long k_srow, long long v_sb, long long v_sh, long long v_srow, long long o_sb,
                            long long o_sh, long long o_srow, const void *workspace,
                            unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_attention_bwd_dq_delta / _dkv that also return the column sums of the
 * gradients they store, per head over batch and rows: dq_colsum[h * D + d] =
 * sum over (b, row) of dq(b, h, row, d) as stored (bf16), fp32 accumulation --
 * the bias gradient of the in_proj segment that produced q (nn.MultiheadAttention's
 * in_proj_bias, models/model_utils.py:552 / :594 self_attn / multihead_attn), so
 * the Linear backward needs no column-sum pass over the packed gradient.  Same
 * dk_colsum / dv_colsum for dK / dV.  bf16 only (else PCOPS_ERR_UNSUPPORTED);
 * workspace: pcops_attention_bwd_colsum_workspace_bytes (delta first, as above,
 * then the per-block partials), shared by the two calls in this order. */
unsigned long long pcops_attention_bwd_colsum_workspace_bytes(int B, int H, int Lq, int Lk, int D);
int pcops_attention_bwd_dq_delta_colsum(const void *q, const void *k, const void *v, const void *o, const void *dout,
                                        const float *lse, void *dq, float *dq_colsum, int B, int H, int Lq, int Lk,
                                        int D, float scale, int dtype, long long q_sb, long long q_sh,
                                        long long q_srow, long long k_sb, long long k_sh, long long k_srow,
                                        long long v_sb, long long v_sh, long long v_srow, long long o_sb,
                                        long long o_sh, long long o_srow, void *workspace,
                                        unsigned long long workspace_bytes, pcops_stream_t stream);
int pcops_attention_bwd_dkv_colsum(const void *q, const void *k, const void *v, const void *dout, const float *lse,
                                   void *dk, void *dv, float *dk_colsum, float *dv_colsum, int B, int H, int Lq,
                                   int Lk, int D, float scale, int dtype, long long q_sb, long long q_sh,
                                   long long q_srow, long long k_sb, long long k_sh, long long k_srow, long long v_sb,
                                   long long v_sh, long long v_srow, long long o_sb, long long o_sh, long long o_srow,
                                   void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* The whole backward in one call (models/model_utils.py:542-617, the autograd of
 * nn.MultiheadAttention's attention core): dq, dk, dv, and -- when dq_colsum, dk_colsum
 * and dv_colsum are all non-NULL (bf16 only) -- their per-head column sums as above.
 * bf16 with D >= 96: the dK/dV pass also stores dS^T (bf16) into workspace and dQ = dS K
 * is read back from it (no S / dP recompute; dQ bitwise equal to the two-pass form);
 * otherwise the two-pass sequence.  workspace:
 * pcops_attention_bwd_fused_workspace_bytes (includes the B*H x Lk x Lq bf16 dS^T
 * buffer, rounded up, for bf16 D >= 96). */
unsigned long long pcops_attention_bwd_fused_workspace_bytes(int B, int H, int Lq, int Lk, int D, int dtype);
int pcops_attention_bwd_fused(const void *q, const void *k, const void *v, const void *o, const void *dout,
                              const float *lse, void *dq, void *dk, void *dv, float *dq_colsum, float *dk_colsum,
                              float *dv_colsum, int B, int H, int Lq, int Lk, int D, float scale, int dtype,
                              long long q_sb, long long q_sh, long long q_srow, long long k_sb, long long k_sh,
                              long long k_srow, long long v_sb, long long v_sh, long long v_srow, long long o_sb,
                              long long o_sh, long long o_srow, void *workspace, unsigned long long workspace_bytes,
                              pcops_stream_t stream);

/* ---------------- attention-block glue (self_attention / cross_attention,
 * models/model_utils.py:584-617 and :542-582: the permute(2,0,1) / permute(1,2,0)
 * layout changes, `src1 + src12`, norm13 / norm12 LayerNorms) ----------------
 * dtype codes: 0 = fp32, 1 = bf16.  Rows are C contiguous elements.
 * pcops_transpose_add: out[b][c][r] = a[b][r][c] (+ b[b][r][c] when b != NULL);
 *   out2 (optional) receives the same values in out2_dtype. */
int pcops_transpose_add(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype, void *out2,
                        int out2_dtype, int B, int R, int C, pcops_stream_t stream);
/* pcops_add: out[i] = a[i] + b[i] for i < n in the promoted dtype (fp32 unless both are bf16),
 * stored as out_dtype (torch.add(a, b, out=out) with type promotion; the attention blocks' residual + FFN sum
 * that feeds only GEMMs, models/model_utils.py:616).  16-byte aligned operands. */
int pcops_add(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype, long long n,
              pcops_stream_t stream);
/* pcops_linear_skinny: y[t][n] = bf16(sum_k x[t][k] A[n][k] (+ bias[n])) for a row-major (rows, K) x,
 * (N, K) A and (rows, N) y, all bf16 (bias bf16 or NULL), fp32 accumulation on the matrix cores.  The 1x1
 * convolutions of EdgeConv's first layer (models/model_utils.py:847-881: Conv2d 6 -> 32, 32 -> 32,
 * 32 -> 64 over B x N x k edge rows, channels_last) -- forward with A = the conv weight, input gradient with
 * A = its transpose and no bias -- in place of the GEMM library's call.  K in {6, 32, 64}, N in {32, 64};
 * 16-byte aligned x / y when K % 8 == 0 (8-byte otherwise); A and bias at any bf16 address. */
int pcops_linear_skinny(const void *x, long long rows, int K, const void *A, const void *bias, void *y, int N,
                        pcops_stream_t stream);
/* pcops_add_rows: pcops_add over a contiguous (rows, C) a / b with out's rows ld_out elements apart: the
 * refinement stage's two decoder outputs (SVDFormer.py:79-86, each `s + f` of a block feeding only conv_ps)
 * written straight into the channel halves of `torch.cat([F_Q_, F_H_], 1)` (SVDFormer.py:86), which
 * replaces the two sums plus the concatenation's copy.  C % 8 == 0, ld_out % 8 == 0, 16-byte aligned. */
int pcops_add_rows(const void *a, int a_dtype, const void *b, int b_dtype, void *out, int out_dtype, long long rows,
                   int C, long long ld_out, pcops_stream_t stream);
/* pcops_add_posemb: out[b][m][h] = a[b][m][h] + E[b][h*N + m] for (B, N, H) token-major a / out,
 * where E (B, N*H) is SinusoidalPositionalEmbedding(cd) (models/model_utils.py:883-917:
 * E[b][n*H + 2i] = sin(cd[b][n] * div_term[i]), E[b][n*H + 2i + 1] = cos(...)) read through SDG's
 * raw .reshape(B, hidden, N).permute (SVDFormer.py:77-80, PointSea SDG the same): the query /
 * key input `with_pos_embed(src1, pos)` of the SDG's first self_attention, summed in fp32 and
 * stored once as out_dtype.  H % 8 == 0, 16-byte aligned a / out. */
int pcops_add_posemb(const void *a, int a_dtype, const float *cd, const float *div_term, int B, int N, int H,
                     void *out, int out_dtype, pcops_stream_t stream);
/* pcops_layernorm_fwd: x = a (+ b); y = (x - mean) * rstd * gamma + beta per row
 * (torch.nn.LayerNorm over the last dim), written as fp32 (y32) and/or bf16
 * (y16); mean / rstd (rows) saved for the backward.  C <= 1024, C % 8 == 0,
 * rows 16-byte aligned. */
int pcops_layernorm_fwd(const void *a, int a_dtype, const void *b, int b_dtype, const float *gamma, const float *beta,
                        float eps, int rows, int C, float *y32, void *y16, float *mean, float *rstd,
                        pcops_stream_t stream);
/* pcops_layernorm_bwd: dy = dy32 + dy16 (either may be NULL); dx written as
 * fp32 (dx32) and/or bf16 (dx16) -- the gradient of both a and b; dgamma /
 * dbeta (C) are overwritten.  workspace: pcops_layernorm_bwd_workspace_bytes. */
unsigned long long pcops_layernorm_bwd_workspace_bytes(int rows, int C);
int pcops_layernorm_bwd(const float *dy32, const void *dy16, const void *a, int a_dtype, const void *b, int b_dtype,
                        const float *gamma, const float *mean, const float *rstd, int rows, int C, float *dx32,
                        void *dx16, float *dgamma, float *dbeta, void *workspace, unsigned long long workspace_bytes,
                        pcops_stream_t stream);
/* pcops_layernorm_bwd_colsum: pcops_layernorm_bwd plus dsum[c] = sum_r dx[r][c] (C values):
 *   the bias gradient of the Linear / 1x1 conv whose output is a LayerNorm input (a or b),
 *   summed over dx as stored -- dx16's bf16 values (dsum_src bit 0 = 1) or dx32's (bit 0 = 0) --
 *   in the same launch (replaces that layer's separate pcops_colsum over dx).  dsum_src bit 1:
 *   dsum stored bf16 (rounded once from the fp32 sum: the consuming bias's dtype), else fp32.
 *   workspace: pcops_layernorm_bwd_colsum_workspace_bytes. */
unsigned long long pcops_layernorm_bwd_colsum_workspace_bytes(int rows, int C);
int pcops_layernorm_bwd_colsum(const float *dy32, const void *dy16, const void *a, int a_dtype, const void *b,
                               int b_dtype, const float *gamma, const float *mean, const float *rstd, int rows, int C,
                               float *dx32, void *dx16, float *dgamma, float *dbeta, void *dsum, int dsum_src,
                               void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_adam_flat: torch's Adam (adamw = 0; weight decay added to the gradient) or AdamW (adamw = 1;
 *   decoupled decay) over n fp32 master weights `param` with its exp_avg / exp_avg_sq state
 *   (core/train_pcn.py:57-60, core/train_55.py:86-88): gradients [0, n16) from grad16 (bf16) when
 *   given, everything else from grad32; the new weights of [0, n16) also written to shadow16 (bf16)
 *   when given.  step_dev: the step count AFTER this update (device fp32 scalar, incremented by the
 *   caller); lr_dev: a device fp32 learning rate (NULL: `lr`).  Hyper-parameters are doubles and
 *   enter the arithmetic as torch's fused Adam has them (products with them formed in double).
 *   Replaces optimizer.step() with the gradient widening and the bf16 weight refresh around it. */
int pcops_adam_flat(float *param, const void *grad16, const float *grad32, long long n16, long long n,
                    float *exp_avg, float *exp_avg_sq, void *shadow16, const float *lr_dev, double lr,
                    const float *step_dev, double beta1, double beta2, double eps, double weight_decay, int adamw,
                    pcops_stream_t stream);
/* pcops_blend_fwd / pcops_blend_bwd: PointSea's path selection out = s * a + (1 - s) * b over n
 *   elements (n % 8 == 0; models_PointSea/PointSea.py:128-131), s `score_dtype` (0 fp32, 1 bf16), a, b,
 *   da, db fp32, out `out_dtype` (bf16: the value autocast hands the next GEMM), g `g_dtype`, dscore in
 *   s's dtype.  torch's per-op roundings: for a bf16 s, 1 - s is rounded to bf16 and
 *   dscore = bf16(bf16(g * a) - bf16(g * b)).  da / db / dscore may be NULL (not needed). */
int pcops_blend_fwd(const void *score, int score_dtype, const float *a, const float *b, long long n, void *out,
                    int out_dtype, pcops_stream_t stream);
int pcops_blend_bwd(const void *g, int g_dtype, const void *score, int score_dtype, const float *a, const float *b,
                    long long n, float *da, float *db, void *dscore, pcops_stream_t stream);
/* pcops_layernorm_bwd_bf16g: pcops_layernorm_bwd(_colsum) with BOTH upstream gradients bf16:
 *   dy = dy_a + dy16, dy_a the gradient of the fp32 output y32 as a bf16 consumer produced it
 *   (the block sum bf16(y32 + f): replaces widening it to fp32 in a separate pass; the sum is
 *   the same fp32 value bit for bit).  dsum = NULL: no column sum (workspace
 *   pcops_layernorm_bwd_workspace_bytes), else as pcops_layernorm_bwd_colsum (its workspace).
 *   Replaces the autograd cast in front of nn.LayerNorm's backward (models/model_utils.py:600-617). */
int pcops_layernorm_bwd_bf16g(const void *dy_a, const void *dy16, const void *a, int a_dtype, const void *b,
                              int b_dtype, const float *gamma, const float *mean, const float *rstd, int rows, int C,
                              float *dx32, void *dx16, float *dgamma, float *dbeta, void *dsum, int dsum_src,
                              void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_layernorm_bwd_ex: pcops_layernorm_bwd(_colsum / _bf16g) with dy = (dy + dy_x) + dy16:
 *   dy (dy_dtype 0 fp32 / 1 bf16) the fp32 output's gradient with its rows ld_dy elements apart (a channel
 *   slice of a wider gradient: the concatenation of SVDFormer.py:86 handed back without a contiguity copy);
 *   dy_x (bf16, contiguous, optional, dy fp32 only) a second gradient of the same output, added to dy first --
 *   the order autograd accumulates them in (the SDG query's positional add, `with_pos_embed(src1, pos)` of
 *   models/model_utils.py:607, whose widening cast and accumulation this replaces); dy16 (bf16, optional) the
 *   bf16 output's gradient.  dsum / dsum_src / workspace as pcops_layernorm_bwd_bf16g. */
int pcops_layernorm_bwd_ex(const void *dy, int dy_dtype, long long ld_dy, const void *dy_x, const void *dy16,
                           const void *a, int a_dtype, const void *b, int b_dtype, const float *gamma,
                           const float *mean, const float *rstd, int rows, int C, float *dx32, void *dx16,
                           float *dgamma, float *dbeta, void *dsum, int dsum_src, void *workspace,
                           unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_gelu_bwd_colsum: du = dy * GELU'(u) (exact erf GELU, torch's GeluBackward expression in
 *   fp32) over a row-major (rows, C) matrix, dy / u / du all `dtype` (0 fp32, 1 bf16), C % 8 == 0;
 *   when dsum != NULL also dsum[c] = sum_r du[r][c] over du as stored (C values, fp32 accumulation,
 *   stored as dsum_dtype: the consuming bias's dtype): the bias gradient of the Linear whose output u
 *   the GELU consumed (the blocks' linear11, models/model_utils.py:612), in place of a separate
 *   pcops_colsum.  workspace: pcops_colsum_workspace_bytes(rows, C) when dsum. */
int pcops_gelu_bwd_colsum(const void *dy, const void *u, int dtype, long long rows, int C, void *du, void *dsum,
                          int dsum_dtype, void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_colsum: out[c] = sum_r g[r][c] over a row-major (rows, C) matrix, C % 8 == 0,
 *   fp32 accumulation in a fixed order (deterministic); g / out dtype codes 0 fp32, 1 bf16.
 *   Replaces the bias-gradient reduction autograd runs for nn.Linear / 1x1 nn.Conv*d biases
 *   (torch's g.sum(0) behind F.linear's backward; models/model_utils.py Linear / Conv1d layers).
 *   workspace: pcops_colsum_workspace_bytes(rows, C). */
/* pcops_sum_rows: out[i] = sum_{s < S} part[s][i] for a row-major (S, N) fp32 matrix, fixed order, rounded
 *   once to out_dtype (0 fp32, 1 bf16); N % 4 == 0, 16-byte aligned.  The split-K weight gradient's
 *   partial sum + cast (torch's part.sum(0).to(dtype) behind the blocks' Linear layers). */
int pcops_sum_rows(const float *part, int S, long long N, void *out, int out_dtype, pcops_stream_t stream);
/* pcops_wgrad_skinny: dw[co][ci] = sum_t g[t][co] * x[t][ci] for g (T, Co), x (T, Ci) bf16 row-major,
 *   Ci == 6, Co % 8 == 0, Co <= 64 (EdgeConv's first 1x1 conv, models/model_utils.py:855-866: 2*3 edge
 *   channels); fp32 accumulation in a fixed order, dw (Co, Ci) as fp32 (0) or bf16 (1).
 *   workspace: pcops_wgrad_skinny_workspace_bytes(Co, Ci). */
unsigned long long pcops_wgrad_skinny_workspace_bytes(int Co, int Ci);
int pcops_wgrad_skinny(const void *g, const void *x, long long T, int Co, int Ci, void *dw, int dw_dtype,
                       void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
unsigned long long pcops_colsum_workspace_bytes(long long rows, int C);
int pcops_colsum(const void *g, int g_dtype, long long rows, int C, void *out, int out_dtype, void *workspace,
                 unsigned long long workspace_bytes, pcops_stream_t stream);
/* pcops_colsum_ld: the same over rows ld elements apart (ld >= C, ld % 8 == 0): a channel slice of a
 *   wider gradient (the Linear's output was concatenated / split after it) summed in place instead of
 *   after a contiguous copy. */
int pcops_colsum_ld(const void *g, int g_dtype, long long rows, int C, long long ld, void *out, int out_dtype,
                    void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);

/* ---------------- BatchNorm (+ residual) (+ ReLU / LeakyReLU) on channels_last activations ----------------
 * Replaces torch.nn.BatchNorm2d's forward / backward (MIOpen) together with the activation and
 * residual add that follow it in the reference's encoders: ResNet BasicBlock (models/resnet.py:56-70,
 * relu(bn1(conv1 x)), relu(bn2(conv2 .) + identity)), the SVFNet stem (models/SVDFormer.py:139-146),
 * EdgeConv's bn + LeakyReLU(0.2) (models/model_utils.py:855-866) and PointSea's resnet18
 * (models_PointSea/PointSea.py:37-61).  x is the (rows, C) memory of an NCHW tensor in channels_last
 * order (rows = N*H*W), C % 8 == 0, C <= 512, rows*C/8 < 2^31, 16-byte aligned.
 * dtype codes 0 fp32, 1 bf16 (x, y, dy, dx, dres share `dtype`; res has res_dtype); gamma, beta,
 * running stats, save_mean / save_invstd fp32 (C).  act: 0 none, 1 ReLU, 2 LeakyReLU(slope).
 * pcops_batchnorm_fwd: batch_stats = 1 (training): mean / biased var over the rows, saved as
 *   save_mean / save_invstd = 1/sqrt(var + eps); running stats (either both NULL or both given)
 *   updated with `momentum` and the unbiased var, as torch; batch_stats = 0 (eval): running stats.
 *   y = act((x - mean) * invstd * gamma + beta (+ res)).
 * pcops_batchnorm_bwd: dy is the gradient of y; y (the forward output) gives the activation's mask.
 *   dx = the gradient of x; dres (optional) = the gradient of res (dy through the activation);
 *   dgamma / dbeta (optional, C) overwritten.
 * workspace (both): pcops_batchnorm_workspace_bytes(rows, C).
 * num_batches_tracked (optional, int64): incremented by the training forward when running stats are given. */
unsigned long long pcops_batchnorm_workspace_bytes(long long rows, int C);
int pcops_batchnorm_fwd(const void *x, int dtype, const void *res, int res_dtype, long long rows, int C,
                        const float *gamma, const float *beta, float *running_mean, float *running_var, float momentum,
                        float eps, int batch_stats, int act, float slope, void *y, float *save_mean, float *save_invstd,
                        void *workspace, unsigned long long workspace_bytes, long long *num_batches_tracked,
                        pcops_stream_t stream);
int pcops_batchnorm_bwd(const void *dy, const void *y, const void *x, int dtype, long long rows, int C,
                        const float *gamma, const float *save_mean, const float *save_invstd, int batch_stats, int act,
                        float slope, void *dx, void *dres, float *dgamma, float *dbeta, void *workspace,
                        unsigned long long workspace_bytes, pcops_stream_t stream);

/* ---------------- 3x3 convolution, stride 1, pad 1, no bias, on channels_last bf16 ----------------
 * The ResNet BasicBlock convs of SVDFormer's image encoder (models/resnet.py:36-70 via
 * models/SVDFormer.py:139-146), replacing torch.nn.Conv2d's MIOpen forward / backward.
 * x, y: (N, H, W, C) bf16 (an NCHW tensor in channels_last memory), C in {16, 32}, 16-byte aligned.
 * pcops_conv3x3_fwd: y[n][h][w][co] = sum_{kh,kw,ci} x[n][h+kh-1][w+kw-1][ci] * w[co][kh][kw][ci]
 *   (w: OHWI bf16, zero padding).  The input gradient of the same conv is
 *   pcops_conv3x3_fwd(dy, w', dx) with w'[ci][kh][kw][co] = w[co][ci][2-kh][2-kw].
 * pcops_conv3x3_wgrad: dw[co][ci][kh][kw] = sum_{n,h,w} dy[n][h][w][co] * x[n][h+kh-1][w+kw-1][ci],
 *   written as fp32 (dw_dtype 0) or bf16 (1), in OIHW (dw_ohwi 0) or OHWI (1) memory order;
 *   fp32 accumulation, block partials summed in a fixed order.
 *   workspace: pcops_conv3x3_wgrad_workspace_bytes(C). */
int pcops_conv3x3_fwd(const void *x, const void *w, int N, int H, int W, int C, void *y, pcops_stream_t stream);
/* pcops_conv3x3_fwd_res: pcops_conv3x3_fwd plus a residual: y = bf16(float(bf16(conv(x, w))) + float(res)),
 *   res bf16 in y's layout.  The input gradient of a ResNet BasicBlock's first conv (the dgrad form of this
 *   conv) fused with the gradient the block input also gets through the identity branch -- autograd's
 *   bf16 accumulation of the two (models/resnet.py:56-70: `out += identity`), without its separate add pass. */
int pcops_conv3x3_fwd_res(const void *x, const void *w, int N, int H, int W, int C, const void *res, void *y,
                          pcops_stream_t stream);
unsigned long long pcops_conv3x3_wgrad_workspace_bytes(int C);
int pcops_conv3x3_wgrad(const void *x, const void *dy, int N, int H, int W, int C, void *dw, int dw_dtype,
                        int dw_ohwi, void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);

/* The single-channel stem of the same encoder, nn.Conv2d(1, 16, 3, padding=1, bias=False)
 * (models/SVDFormer.py:139-140): x (N, H, W) fp32 (rounded to bf16 as autocast's conv does),
 * w (16, 1, 3, 3) fp32, y (N, H, W, 16) bf16 channels_last; fp32 accumulation.
 * pcops_conv3x3_c1_wgrad: dw (16, 1, 3, 3) as fp32 (dw_dtype 0) or bf16 (1).
 *   workspace: pcops_conv3x3_c1_wgrad_workspace_bytes(). */
int pcops_conv3x3_c1_fwd(const float *x, const float *w, int N, int H, int W, void *y, pcops_stream_t stream);
unsigned long long pcops_conv3x3_c1_wgrad_workspace_bytes(void);
int pcops_conv3x3_c1_wgrad(const float *x, const void *dy, int N, int H, int W, void *dw, int dw_dtype, void *workspace,
                           unsigned long long workspace_bytes, pcops_stream_t stream);

/* ---------------- PCSA spectral gating (models/model_utils.py:358-430) ----------------
 * Per patch p (= b*S + s) of K neighbours x C channels stored [p][k][c] (the
 * channels_last memory order of the (B, C, S, K) conv output):
 *   out[p] = D^T diag(gates[p]) D x[p]      (D = basis, K x K row-major fp32)
 * pcops_pcsa_backward: dx[p] = (D^T diag(g) D)^T dout[p];
 *   dgates[p][k] = sum_c (D dout[p])[k][c] * (D x[p])[k][c].
 * dtype codes 0 = fp32, 1 = bf16 (x, out, dx share x_dtype; dgates has
 * gates_dtype).  K in {4, 8, 16, 32}. */
int pcops_pcsa_forward(const void *x, int x_dtype, const void *gates, int gates_dtype, const float *basis, int patches,
                       int K, int C, void *out, pcops_stream_t stream);
int pcops_pcsa_backward(const void *x, int x_dtype, const void *dout, int dout_dtype, const void *gates,
                        int gates_dtype, const float *basis, int patches, int K, int C, void *dx, void *dgates,
                        pcops_stream_t stream);

/* ---------------- depth renderers ----------------
 * PCViews.get_img (models/model_utils.py:1196-1234 -> points2depth :1080-1115 ->
 * distribute :1004-1077, size 1): points (B,N,3); rot (V,3,3) row-major =
 * euler2mat(angle).transpose(1,2); trans (V,3) -> img (B*V, H, W), image
 * r = b*V + v.  workspace: pcops_points2depth_workspace_bytes. */
unsigned long long pcops_points2depth_workspace_bytes(int B, int V, int H, int W);
int pcops_points2depth(const float *points, const float *rot, const float *trans, int B, int N, int V, int H, int W,
                       float *img, void *workspace, unsigned long long workspace_bytes, pcops_stream_t stream);
/* PCViews_Real.get_img (models_PointSea/mv_utils_zs.py:136-195): points (B,N,3),
 * rot/rot2 (V,3,3), trans (V,3), kern (3,3) Gaussian (get3DGaussianKernel :197-212)
 * -> img (B*V, 3, R, R).  grid (B*V, D, R, R) is an output too (the
 * intermediate voxel grid, [img][z][x][y]). */
int pcops_points2grid(const float *points, const float *rot, const float *rot2, const float *trans, int B, int N,
                      int V, int R, int D, float *grid, pcops_stream_t stream);
int pcops_grid2image(const float *grid, const float *kern, int BV, int D, int R, float *img, void *workspace,
                     unsigned long long workspace_bytes, pcops_stream_t stream);
unsigned long long pcops_grid2image_workspace_bytes(int BV, int D, int R);

#ifdef __cplusplus
}
#endif
#endif /* PCOPS_H_ */
