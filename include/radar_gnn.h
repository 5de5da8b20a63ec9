/*
 * radar_gnn.h -- C ABI of the MI355X-native radar GNN hot path (libradargnn.so).
 *
 * The library replaces the implicit numpy / ATen / PyG kernels of the
 * reference's per-frame path (UditBhaskar19/GRAPH_NEURAL_NETWORK_FOR_RADAR_PERCEPTION v2):
 *   graph build      modules/compute_features/graph_features.py:11-164
 *   model forward    modules/neural_net/gnn/gnn_detector.py:141-201,
 *                    modules/neural_net/gnn/gnn_blocks.py:19-389,
 *                    modules/neural_net/common.py:185-267
 * Each entry point names the reference interface it replaces.
 *
 * Conventions
 *  - every pointer is a DEVICE pointer unless its name ends in _host;
 *  - buffers are owned by the caller (the library allocates nothing that
 *    outlives a call; scratch comes from a caller workspace sized by the
 *    matching *_workspace_size function);
 *  - work is enqueued asynchronously on `stream` (a hipStream_t); no entry point
 *    synchronises the host, so a caller may capture them in a hipGraph;
 *  - a batch of radar frames is a disjoint union: nodes of frame f are the rows
 *    [frame_ptr[f], frame_ptr[f+1]) of every node array (frame_ptr: int32[B+1]);
 *  - the adjacency is CSR (row_ptr int32[N+1], col int32[E]) with rows and
 *    columns ascending: position p of row i is edge_index[:, p] = (i, col[p]) of
 *    the reference's np.where order (graph_features.py:79);
 *  - return value 0 = success; otherwise an RG_ERR_* code and rg_last_error()
 *    describes it (the Python layer raises RuntimeError with that text).
 */
#ifndef RADAR_GNN_H
#define RADAR_GNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RG_OK 0
#define RG_ERR_ARG 1
#define RG_ERR_HIP 2
#define RG_ERR_UNSUPPORTED 3

/* element types */
#define RG_F32 0
#define RG_BF16 1
#define RG_F16 6 /* IEEE binary16: the fp16 path (BASELINE config 5) of the 16-bit kernels */
#define RG_F32X3 7 /* rg_mlp_chain: float32 arithmetic on the bf16 matrix cores (every product
                      from exact three-term bf16 splits, f32 accumulation); layers packed
                      RG_BF16 | RG_PACK_X3; training tapes allowed */
/* packed-weight formats of rg_pack_linear: RG_F32 / RG_BF16 for rg_mlp_chain, and
 * the two 32x32x16 bf16 formats of rg_mlp_chain_fast (first layer / chained layers) */
#define RG_PACK_FAST_IN 2
#define RG_PACK_FAST_CHAIN 3
#define RG_PACK_FAST_UPD 4 /* update layer of rg_conv_layer_fused: cat(x, aggregate) */
/* float32 32x32x2 fragments of the register-resident f32 kernels (rg_mlp_chain_f32,
 * rg_conv_layer_f32): fragment (m, s4) = 1 KiB at byte (m * K/8 + s4) * 1024, lane l's
 * 16 B = W[32m + (l & 31)][8 s4 + 4 (l >> 5) + u], u = 0..3 (K padded to 8, N to 32),
 * then the bias in accumulator order [m][h][16] (entry 4g + t = b[32m + 8g + 4h + t]) */
#define RG_PACK_F32_FAST 5
/* OR-ed into a RG_PACK_FAST_* format for a layer followed by channel_normalization:
 * the rows of W and b are shifted to zero mean over the outputs (W - 1 mean_o(W),
 * b - mean(b)).  The normalisation then sees (x - mean) directly -- it is invariant
 * to that shift -- and skips its mean pass.  Mark such layers RG_LAYER_CENTERED. */
#define RG_PACK_CENTERED 0x100
/* OR-ed into RG_F32: `weight` holds the TRANSPOSE of the packed layer, i.e. a row-major
 * [in_dim][out_dim] matrix (the backward data GEMM dX = dZ W packs W^T this way) */
#define RG_PACK_TRANSPOSE 0x200
/* OR-ed into a RG_PACK_FAST_* format: the exact three-term bf16 split of every weight,
 * w = w0 + w1 + w2 (w0 = bf16(w), w1 = bf16(w - w0), w2 = bf16(w - w0 - w1), each residue
 * exact in float32), as three planes of that format back to back, then the float32 bias in
 * accumulator order -- the operand format of the float32 kernels on bf16 matrix cores
 * (rg_conv_layer_x3) */
#define RG_PACK_X3 0x400
/* OR-ed into a RG_PACK_FAST_* format: IEEE fp16 fragments instead of bf16 (round to nearest
 * even); mark such layers RG_LAYER_F16 -- the 16-bit kernels then take fp16 operands */
#define RG_PACK_F16 0x800

/* activations (modules/neural_net/common.py:256-267) */
#define RG_ACT_NONE 0
#define RG_ACT_RELU 1
#define RG_ACT_LEAKY 2
#define RG_ACT_SWISH 3

/* graph modes */
#define RG_GRAPH_KNN 0        /* compute_adjacency_information     graph_features.py:58-84  */
#define RG_GRAPH_RADIUS 1     /* np.where(compute_ball_query(D,eps)) graph_features.py:11-22 */
#define RG_GRAPH_KNN_RADIUS 2 /* compute_adjacency_information_v2  graph_features.py:87-114 */

/* segment reductions (PyG aggr, gnn_blocks.py:57; cluster max gnn_blocks.py:384-387) */
#define RG_REDUCE_SUM 0
#define RG_REDUCE_MEAN 1
#define RG_REDUCE_MAX 2

/* chain input prologues */
#define RG_IN_DENSE 0   /* row r <- in0[r]                                           */
#define RG_IN_CONCAT2 1 /* row r <- cat(in0[r], in1[r])          gnn_blocks.py:108   */
#define RG_IN_GATHER3 2 /* row r <- cat(in0[idx0[r]], in0[idx1[r]], in2[r])
                           = cat(x_i, x_j, e) of MessagePassing.message, gnn_blocks.py:113 */
#define RG_IN_PAIRADD 3 /* row r <- in0[idx0[r]] + in0[idx1[r]]  gnn_blocks.py:297   */
#define RG_IN_PAIRPRE 4 /* rg_mlp_chain_x3 only: layer 0's pre-activation <- in0[idx0[r]] +
                           in0[idx1[r]] + b0, in0 = per-node rows W0 x (layer 0 is linear
                           before its norm, gnn_blocks.py:292-297); layer 0's weights unread */

const char* rg_last_error(void);
int rg_version(void);

/* ---------------------------------------------------------------- graph build */

/* Bytes of scratch rg_build_graph needs. */
size_t rg_build_graph_workspace_size(int n_nodes, int n_frames, int max_frame_nodes, int k,
                                     int mode);

/* Batched compute_adjacency_information (graph_features.py:58-84):
 *   D[i,j] = dx*dx + dy*dy in float32 without FMA (graph_features.py:69-76);
 *   ball_degree[i] = #{j != i : D[i,j] <= eps2}          (:11-22, :78);
 *   kNN: the k+1 smallest (D, j) pairs of each row (all j if k >= N_f),
 *        ties -> lower j (a stable argsort; the reference's default argsort is
 *        unstable, so at exact ties it is implementation-defined) (:25-44);
 *   adjacency = knn | knn^T minus the diagonal (mode KNN), the ball query
 *   (mode RADIUS) or their union (mode KNN_RADIUS);
 *   row_ptr/col = np.where(adjacency) as CSR (:79), global node ids.
 * px, py:        float32[n_nodes]
 * frame_ptr:     int32[n_frames+1] (device)
 * col:           int32[col_capacity]; rg_build_graph fails with RG_ERR_ARG
 *                through *n_edges_out > col_capacity (checked on device: the
 *                overflowing rows are not written and n_edges_out reports the need)
 * n_edges_out:   int32[1] device scalar = E
 */
int rg_build_graph(const float* px, const float* py, const int* frame_ptr, int n_nodes,
                   int n_frames, int max_frame_nodes, int k, float eps2, int mode,
                   int* row_ptr, int* col, long col_capacity, int* ball_degree,
                   int* n_edges_out, void* workspace, size_t workspace_bytes, void* stream);

/* compute_node_features(include_region_confidence=True) (graph_features.py:117-144),
 * cast to float32 as datagen_gnn.py:122 does.  out: float32[n_nodes][6] =
 * (vr, rcs, t_norm, degree/10, range_conf, azimuth_conf). */
int rg_node_features(const float* px, const float* py, const float* vr, const float* rcs,
                     const int64_t* timestamp, const int* ball_degree, const int* frame_ptr,
                     int n_nodes, int n_frames, double min_range, double max_range,
                     double min_azimuth, double max_azimuth, float* out, void* stream);

/* compute_edge_features (graph_features.py:147-164) -> float32[E][7]
 * (dx, dy, dl, dvx, dvy, dv, dt) of every edge src[p] -> dst[p].  With
 * (src, dst) = (edge_index[0], edge_index[1]) this is the reference layout; the
 * message passing passes its destination-major (source, destination) arrays.
 * n_edges_dev (optional device int32) overrides n_edges (then the capacity). */
int rg_edge_features(const float* px, const float* py, const float* vx, const float* vy,
                     const int64_t* timestamp, const int* src, const int* dst,
                     const int* n_edges_dev, long n_edges, float* out, void* stream);

/* The float64 arrays compute_node_features / compute_edge_features themselves return
 * (graph_features.py:144,164: np.stack promotes the float32 columns exactly, while
 * t_norm, degree/10, range_conf and dt are float64 computations), same layouts. */
int rg_node_features_f64(const float* px, const float* py, const float* vr, const float* rcs,
                         const int64_t* timestamp, const int* ball_degree, const int* frame_ptr,
                         int n_nodes, int n_frames, double min_range, double max_range,
                         double min_azimuth, double max_azimuth, double* out, void* stream);
int rg_edge_features_f64(const float* px, const float* py, const float* vx, const float* vy,
                         const int64_t* timestamp, const int* src, const int* dst, long n_edges,
                         double* out, void* stream);

/* rg_edge_features from node kinematics packed once per batch: kin = float4[n_nodes]
 * (px, py, vx, vy) from rg_pack_kinematics (16-B aligned).  Same results, two gathers
 * per edge endpoint instead of five. */
int rg_pack_kinematics(const float* px, const float* py, const float* vx, const float* vy,
                       int n_nodes, void* kin, void* stream);
int rg_edge_features_packed(const void* kin, const int64_t* timestamp, const int* src,
                            const int* dst, const int* n_edges_dev, long n_edges, float* out,
                            void* stream);

/* edge_formation's pairs from a DENSE adjacency (gnn_blocks.py:295-296: torch.nonzero(
 * torch.triu(adj, 1), as_tuple=True), row-major), in two calls so the caller sizes the
 * pair arrays from the count (the one host synchronisation, where torch.nonzero syncs too):
 *   rg_dense_pair_rows: adj = uint8 / bool [n][n] (n <= 46340) -> row_ptr int32[n + 1]
 *     (exclusive scan of each row's entries right of the diagonal), n_pairs int32[1];
 *     workspace O(n);
 *   rg_dense_pair_emit: pair_src / pair_dst int32[n_pairs], rows in order, columns
 *     ascending. */
size_t rg_dense_pair_rows_workspace_size(int n_nodes);
int rg_dense_pair_rows(const void* adj, int n_nodes, int* row_ptr, int* n_pairs, void* workspace,
                       size_t workspace_bytes, void* stream);
int rg_dense_pair_emit(const void* adj, int n_nodes, const int* row_ptr, int* pair_src,
                       int* pair_dst, void* stream);
/* out[r][0..w) = x[idx0[r]] + x[idx1[r]] in float32 (edge_formation's x[i] + x[j],
 * gnn_blocks.py:297) */
int rg_pair_add_rows_f32(const float* x, int ldx, int w, const int* idx0, const int* idx1,
                         long rows, float* out, int ld_out, void* stream);

/* Undirected link pairs of edge_formation (gnn_blocks.py:295-296):
 * nonzero(triu(adj,1)) row-major == CSR positions with col > row.
 * pair_ptr int32[n_nodes+1]; pair_src/pair_dst int32[capacity]; n_pairs int32[1]. */
size_t rg_link_pairs_workspace_size(int n_nodes);
int rg_link_pairs(const int* row_ptr, const int* col, int n_nodes, int* pair_ptr, int* pair_src,
                  int* pair_dst, long pair_capacity, int* n_pairs, void* workspace,
                  size_t workspace_bytes, void* stream);

/* Link pairs of an arbitrary edge_index (int64[2][E], reference order): the
 * positions with edge_index[0] < edge_index[1], in edge order; equals
 * nonzero(triu(adj,1)) when edge_index = np.where(adj) (graph_features.py:79). */
size_t rg_pairs_from_edge_index_workspace_size(long n_edges);
int rg_pairs_from_edge_index(const int64_t* edge_index, long n_edges, int* pair_src, int* pair_dst,
                             int* n_pairs, void* workspace, size_t workspace_bytes, void* stream);

/* out[p] = row of CSR position p (edge_index[0]; destination of a dst-major edge). */
int rg_csr_rows(const int* row_ptr, int n_rows, int* out, void* stream);

/* Capacity guard for a graph built by rg_build_graph into a capacity the host has not
 * checked (radius graphs without a host sync, graph_features.py:build_graph_batch):
 * need_out[0] = the true edge count (int32 in device memory, or in pinned host memory -- the
 * kernel stores it directly, no copy launch); if it exceeds capacity, row_ptr is cut at a
 * row boundary (the rows rg_build_graph left unwritten become empty) and *n_edges_dev =
 * that boundary, so every consumer stays in bounds.  The host
 * reads need_out later (no sync on the launch path) and treats the step as invalid when
 * need_out[0] > capacity.  (The cut is at the last boundary <= capacity / 2: a cut graph is
 * not symmetric, and the link-pair arrays hold capacity / 2 + 1 pairs.) */
int rg_csr_clamp(int* row_ptr, int n_rows, int* n_edges_dev, long capacity, int* need_out,
                 void* stream);

/* Destination-major CSR of an arbitrary edge_index (int64[2][E], reference order):
 * dst_ptr int32[n_nodes+1]; perm int32[E] (dst-major position -> reference
 * position), ordered by (dst, src, reference position); src_sorted int32[E]. */
size_t rg_csr_by_dst_workspace_size(int n_nodes, long n_edges);
int rg_csr_by_dst(const int64_t* edge_index, long n_edges, int n_nodes, int* dst_ptr, int* perm,
                  int* src_sorted, void* workspace, size_t workspace_bytes, void* stream);

/* Dense views for the numpy-level drop-in compute_adjacency_information of ONE
 * frame: adj uint8[N][N] from the CSR and dist float32[N][N] (either may be NULL). */
int rg_dense_adjacency(const float* px, const float* py, const int* row_ptr, const int* col,
                       int n_nodes, uint8_t* adj, float* dist, void* stream);

/* out[r] = (int64) in[r] (edge_index boundary: datagen_gnn.py:123 int64) */
int rg_i32_to_i64(const int* in, long n, int64_t* out, void* stream);

/* out[r][:] = in[idx[r]][:] for float32 rows of width w */
int rg_gather_rows_f32(const float* in, const int* idx, long rows, int w, float* out,
                       void* stream);

/* --------------------------------------------------------- dense MLP chains */

/* Bytes of one packed Linear(in_dim -> out_dim) in `dtype`. */
size_t rg_packed_linear_bytes(int in_dim, int out_dim, int dtype);

/* Pack a torch nn.Linear (weight float32 [out_dim][in_dim] row-major, bias
 * float32[out_dim] or NULL; device) into the MFMA fragment order the chain
 * kernels read, zero padded, followed by the bias padded to a multiple of 16. */
int rg_pack_linear(const float* weight, const float* bias, int in_dim, int out_dim, int dtype,
                   void* packed, void* stream);

/* Many float32 packs in ONE launch (the training step re-packs every layer's images after
 * each optimizer step: `optimizer.step()` at training.py:80 changes every nn.Linear).  Each
 * job is what rg_pack_linear(weight, bias, in_dim, out_dim, fmt | (transpose ?
 * RG_PACK_TRANSPOSE : 0), packed) writes, for fmt RG_F32 or RG_PACK_F32_FAST.  jobs: a
 * DEVICE array of n_jobs entries (built once; the weights are read at launch time). */
typedef struct rg_pack_job {
  const float* weight;  /* [out][in] ([in][out] with transpose) */
  const float* bias;    /* [out] or NULL */
  void* packed;         /* rg_packed_linear_bytes(in_dim, out_dim, fmt) bytes */
  int in_dim, out_dim, fmt, transpose;
  int ld;               /* weight's row stride in floats (0: dense rows) */
} rg_pack_job;
int rg_pack_linear_jobs(const rg_pack_job* jobs, int n_jobs, void* stream);
/* rg_pack_linear for RG_F32 / RG_PACK_F32_FAST (| RG_PACK_TRANSPOSE) from a column block of a
 * wider row-major matrix: rows ld floats apart (0: dense).  The training step packs the
 * x_i / x_j / e column blocks of msg0 (gnn_blocks.py:100-101) this way for its factorised
 * message backward. */
int rg_pack_linear_ld(const float* weight, const float* bias, int in_dim, int out_dim, int dtype,
                      int ld, void* packed, void* stream);

/* One ffn_block (common.py:185-205): Linear -> [channel_normalization] -> activation. */
typedef struct rg_layer {
  const void* w_packed;  /* rg_pack_linear output (weights + bias)             */
  const float* norm_mu;  /* channel_normalization.mu  (1,) or NULL (no norm)     */
  const float* norm_std; /* channel_normalization.std (1,)                       */
  int in_dim;
  int out_dim;
  int act;   /* RG_ACT_* */
  int flags; /* RG_LAYER_* */
  /* training forward (rg_mlp_chain, RG_F32 only; NULL for inference): the layer's
   * pre-normalisation output z = x W^T + b and its post-activation output a, both
   * float32 [rows][out_dim] -- the tape rg_ffn_backward / rg_linear_grad read */
  float* save_pre;
  float* save_out;
} rg_layer;

#define RG_LAYER_CENTERED 1 /* w_packed was packed with RG_PACK_CENTERED */
#define RG_LAYER_F16 2      /* w_packed holds fp16 fragments (RG_PACK_F16): the fast chain /
                               fused conv then read and write RG_F16 activations */

#define RG_MAX_LAYERS 8

/* A chain of up to RG_MAX_LAYERS ffn_blocks over `rows` rows (widths <= 256),
 * fused in one kernel; activations never leave the chip between layers.
 * Covers graph_feature_encoding (gnn_blocks.py:19-42), the message and update
 * MLPs of residual_graph_conv_block (:104-113), the stems and
 * FFN_TaskSpecificHead of every task head (:167-389).
 *   dtype    RG_F32 (f32 MFMA), RG_BF16 / RG_F16 (16-bit operands, f32 accumulation;
 *            RG_F16's layers packed RG_BF16 | RG_PACK_F16), RG_F32X3
 *   in_mode  RG_IN_*: how row r's input vector is formed from in0/in1/in2
 *   in_dtype element type of in0/in1/in2 (RG_F32, RG_BF16 or RG_F16)
 *   rows_dev optional device int32 row count (overrides `rows` when non-NULL;
 *            `rows` is then the capacity used for the grid)
 *   residual optional [rows][out_dim] added after the last layer (:109)
 *   out      [rows][ld_out] in out_dtype
 */
int rg_mlp_chain(int dtype, const rg_layer* layers_host, int n_layers, long rows,
                 const int* rows_dev, int in_mode, int in_dtype, const void* in0, int ld0,
                 int w0, const void* in1, int ld1, int w1, const void* in2, int ld2, int w2,
                 const int* idx0, const int* idx1, const void* residual, int ld_res,
                 int res_dtype, void* out, int ld_out, int out_dtype, void* stream);

/* Register-resident bf16 chain (same semantics as rg_mlp_chain with dtype RG_BF16)
 * for the widths of the shipped architecture: layer 0 packed as RG_PACK_FAST_IN,
 * later layers as RG_PACK_FAST_CHAIN.  Returns RG_ERR_UNSUPPORTED (and launches
 * nothing) when the shape has no compiled instantiation; the caller then uses
 * rg_mlp_chain. */
int rg_mlp_chain_fast(const rg_layer* layers_host, int n_layers, long rows, const int* rows_dev,
                      int in_mode, int in_dtype, const void* in0, int ld0, int w0,
                      const void* in1, int ld1, int w1, const void* in2, int ld2, int w2,
                      const int* idx0, const int* idx1, const void* residual, int ld_res,
                      int res_dtype, void* out, int ld_out, int out_dtype, void* stream);

/* Register-resident float32 chain (same semantics as rg_mlp_chain with dtype RG_F32,
 * exact f32 products on v_mfma_f32_32x32x2_f32) for the widths of the shipped
 * architecture: every layer packed RG_PACK_F32_FAST, no RG_LAYER_CENTERED.  in_mode
 * RG_IN_DENSE (float32 rows; <= 8 features with an un-normalised first layer = the
 * encoders, gnn_blocks.py:19-42) or RG_IN_PAIRADD (edge_formation, gnn_blocks.py:297).
 * Returns RG_ERR_UNSUPPORTED (launching nothing) for shapes without an instantiation;
 * the caller then uses rg_mlp_chain.  Replaces the ffn_block chains of common.py:185-220
 * called from gnn_blocks.py:19-42 and :167-389. */
int rg_mlp_chain_f32(const rg_layer* layers_host, int n_layers, long rows, const int* rows_dev,
                     int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                     const int* idx1, float* out, int ld_out, void* stream);
/* rg_mlp_chain_f32 with every input mode and the training tape: in_mode also
 * RG_IN_GATHER3 (cat(in0[idx0], in0[idx1], in2) with 64-wide parts: the message MLP,
 * gnn_blocks.py:104-113) and RG_IN_CONCAT2 (cat(in0, in1), 64 + 64: the update MLP,
 * :108); optional residual (out = residual + chain, :109); when every layer's save_pre /
 * save_out is set, each layer's z and a rows are written as rg_mlp_chain writes them (the
 * training forward of training.py:66-85); the LAST layer's save_out may be NULL (its
 * activation is the chain output, never read back by the backward).  RG_ERR_UNSUPPORTED (launching nothing) for
 * shapes without an instantiation. */
int rg_mlp_chain_f32_ex(const rg_layer* layers_host, int n_layers, long rows, const int* rows_dev,
                        int in_mode, const float* in0, int ld0, int w0, const float* in1, int ld1,
                        int w1, const float* in2, int ld2, int w2, const int* idx0,
                        const int* idx1, const float* residual, int ld_res, float* out,
                        int ld_out, void* stream);

/* The same float32 chains on the bf16 matrix cores: every product formed from the exact
 * three-term bf16 splits of both operands (RG_PACK_X3, see rg_conv_layer_x3), f32
 * accumulation -- float32 accuracy at 2.7x the f32 MFMA rate.  Layer 0 packed
 * RG_PACK_FAST_IN | RG_PACK_X3, later layers RG_PACK_FAST_CHAIN | RG_PACK_X3, no
 * RG_LAYER_CENTERED; in_mode and the rest as rg_mlp_chain_f32 (dense inputs of <= 8 features
 * with an un-normalised first layer, or widths that are multiples of 16).  Returns
 * RG_ERR_UNSUPPORTED (launching nothing) for shapes without an instantiation, and for the
 * <= 8-input (encoder) shapes also unless the output rows are full width (last out_dim a
 * multiple of 32), ld_out % 4 == 0 and rows * ld_out * 4 <= 0x7ff00000 (their rows are
 * written by buffer stores with 32-bit byte offsets). */
int rg_mlp_chain_x3(const rg_layer* layers_host, int n_layers, long rows, const int* rows_dev,
                    int in_mode, const float* in0, int ld0, int w0, const int* idx0,
                    const int* idx1, float* out, int ld_out, void* stream);

/* One fused FLOAT32 residual_graph_conv_block (gnn_blocks.py:96-113, the reference
 * precision) for the shipped widths (C = 64, message MLP 192 -> 128 -> 64, update
 * 128 -> 64, channel_normalization + LeakyReLU on every block), aggregation add or mean
 * (the PyG propagate of gnn_blocks.py:57,106).  layers[4], all RG_PACK_F32_FAST:
 *   [0] the per-node projection 64 -> 256: rows 0..127 = W_msg0[:, 0:64] (x_i columns),
 *       rows 128..255 = W_msg0[:, 64:128] (x_j columns); bias = [b_msg0; 0]; no norm / act
 *   [1] W_msg0[:, 128:192] (the edge columns) 64 -> 128, no bias, msg0's norm + act
 *   [2] msg1 128 -> 64 (bias, norm, act)     [3] upd 128 -> 64 on cat(x, agg)
 * seg_ptr / src / dst: destination-major CSR (sources ascending per segment); e rows in
 * that order.  x_out[i] = x[i] + upd(cat(x[i], AGG_p msg(cat(x[i], x[src p], e[p])))),
 * the sum in edge order.  workspace: rg_conv_layer_f32_workspace_size(n_nodes) bytes,
 * no initialisation needed (two launches: projections, which also reset the block
 * counters, then the fused layer); one workspace per stream. */
size_t rg_conv_layer_f32_workspace_size(int n_nodes);
int rg_conv_layer_f32(const rg_layer* layers, int aggr, const float* x, int ldx, const float* e,
                      int lde, const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                      float* x_out, int ld_out, void* workspace, size_t workspace_bytes,
                      void* stream);

/* The same FLOAT32 layer on the bf16 matrix cores: every product of the MLPs is formed
 * from the exact three-term bf16 splits of both operands (six bf16 products of total
 * weight <= 2 per product, f32 accumulation; dropped terms < 2^-23 |a b|), so the layer
 * keeps float32 accuracy at 2.7x the matrix rate of the f32 MFMA path.  Two launches per
 * layer (edge: layers [0], [1] and the in-order segmented sum; node: [2] and next_pq):
 *   layers[3], all RG_PACK_X3: [0] W_msg0[:, 128:192] (edge columns, FAST_IN) with msg0's
 *     norm + act, bias unused; [1] msg1 (FAST_CHAIN); [2] upd on cat(x, agg) (FAST_IN over
 *     the 128 concatenated inputs)
 *   pq        [n_nodes][256] float32: P | Q = W_msg0[:, 0:64] x + b_msg0 | W_msg0[:, 64:128] x,
 *             from rg_conv_proj_x3 (first layer) or the previous layer's pq_out
 *   next_pq   NULL, or the NEXT layer's projection (64 -> 256, FAST_CHAIN | X3, bias
 *             [b_msg0'; 0]): then pq_out [n_nodes][256] receives it from x_out's registers
 *   workspace rg_conv_layer_x3_workspace_size(n_nodes) bytes, block counters ZEROED before
 *             the first call (every completed launch leaves them zero); one per stream.
 * Same results contract as rg_conv_layer_f32 (sum in edge order, mean = sum / max(deg, 1)). */
size_t rg_conv_layer_x3_workspace_size(int n_nodes);
int rg_conv_layer_x3(const rg_layer* layers, const rg_layer* next_pq, int aggr, const float* x,
                     int ldx, const float* e, int lde, const float* pq, const int* seg_ptr,
                     const int* src, const int* dst, int n_nodes, float* x_out, int ld_out,
                     float* pq_out, void* workspace, size_t workspace_bytes, void* stream);
/* The same layer with the edge launch's wave table from rg_conv_x3_blocks (built once per
 * graph instead of once per layer): per wave of the one-wave-per-SIMD edge launch S pieces
 * of whole destinations (one per slab of its XCD's node range), equal edge counts.  Same
 * results. */
int rg_conv_layer_x3_blocks(const rg_layer* layers, const rg_layer* next_pq, int aggr,
                            const float* x, int ldx, const float* e, int lde, const float* pq,
                            const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                            float* x_out, int ld_out, float* pq_out, const int* table,
                            void* workspace, size_t workspace_bytes, void* stream);
/* table: rg_conv_x3_blocks_bytes(n_nodes) bytes of device memory -- int32 boundaries of
 * W x S node pieces with equal edge counts in node order (piece q = destinations
 * [table[q], table[q + 1])); wave j of XCD x (W / 8 waves per XCD) takes the pieces
 * (x S + k) W / 8 + j, k = 0 .. S - 1, so the XCD's waves walk its slabs together -- from
 * seg_ptr[n_nodes + 1]. */
size_t rg_conv_x3_blocks_bytes(int n_nodes);
int rg_conv_x3_blocks(const int* seg_ptr, int n_nodes, int* table, void* stream);
/* P | Q of the first layer for dense float32 rows x [n_nodes][ldx >= 64]: pq layer packed
 * RG_PACK_FAST_IN | RG_PACK_X3 (64 -> 256, bias [b_msg0; 0]). */
int rg_conv_proj_x3(const rg_layer* pq, const float* x, int ldx, int n_nodes, float* pq_out,
                    void* stream);

/* One fused residual_graph_conv_block (gnn_blocks.py:96-113) for the shipped
 * widths (node / edge channels 64, msg MLP 192->128->64, update 128->64, all with
 * channel_normalization), bf16 operands, aggregation add or mean:
 *   x_out[i] = x[i] + upd(cat(x[i], AGG_{p in seg i} msg(cat(x[i], x[src[p]], e[p]))))
 * seg_ptr / src / dst: destination-major CSR (dst[p] = segment of p); e rows in
 * the same order.  msg_layers[0] packed RG_PACK_FAST_IN, msg_layers[1]
 * RG_PACK_FAST_CHAIN, upd_layer RG_PACK_FAST_UPD.  Returns RG_ERR_UNSUPPORTED for
 * other shapes / aggregations (use rg_mlp_chain + rg_segment_reduce).
 * workspace: rg_conv_layer_workspace_size() bytes, ZEROED before the first call (block
 * counters; every completed launch leaves them zero again, so no per-call memset; a
 * failed launch re-zeroes them).  One workspace per stream: two launches in flight on
 * different streams must not share it. */
size_t rg_conv_layer_workspace_size(void);
int rg_conv_layer_fused(const rg_layer* msg_layers, const rg_layer* upd_layer, int aggr,
                        const void* x, int ldx, const void* e, int lde, const int* seg_ptr,
                        const int* src, const int* dst, int n_nodes, void* x_out, int ld_out,
                        void* workspace, void* stream);
/* The same layer over edge-balanced work blocks: block b = destination nodes
 * [blk_nodes[2b], blk_nodes[2b+1]), *n_blocks_dev blocks (both from rg_conv_blocks; both
 * NULL = runs of 8 nodes, i.e. rg_conv_layer_fused).  Same results, better balance for
 * graphs with few, skewed-degree runs (dense radius frames). */
int rg_conv_layer_fused_blocks(const rg_layer* msg_layers, const rg_layer* upd_layer, int aggr,
                               const void* x, int ldx, const void* e, int lde,
                               const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                               void* x_out, int ld_out, const int* blk_nodes,
                               const int* n_blocks_dev, void* workspace, void* stream);
/* Work blocks for rg_conv_layer_fused_blocks from the destination-major seg_ptr[N+1]:
 * every run of 8 nodes, split at node boundaries where its edge count would pass
 * max(128, E / 4096); written as (first node, end node) pairs in dequeue order, each of
 * the 8 XCD shares sorted by edge tiles, largest first.  blk_nodes: int32[2N] capacity;
 * n_blocks: int32[1] (device). */
size_t rg_conv_blocks_workspace_size(int n_nodes);
int rg_conv_blocks(const int* seg_ptr, int n_nodes, int* blk_nodes, int* n_blocks,
                   void* workspace, size_t workspace_bytes, void* stream);
/* A static schedule for the same layer: wave rank w of an n_waves-wave grid (n_waves a
 * multiple of 64: 8 waves per workgroup, 8 XCDs) owns the destination nodes
 * [wave_nodes[w], wave_nodes[w+1]), equal shares of degree + 4 per node (the block head and
 * update in edge units), and walks them in 8-node blocks with no work counters -- no
 * dequeue latency and no tail of whole blocks (one dense frame: BASELINE config 5).
 * wave_nodes: int32[n_waves + 1] (device), from rg_conv_wave_nodes once per graph.  Same
 * results as rg_conv_layer_fused (each destination's edges summed in CSR order by one wave). */
int rg_conv_wave_nodes(const int* seg_ptr, int n_nodes, int n_waves, int* wave_nodes,
                       void* stream);
int rg_conv_layer_fused_waves(const rg_layer* msg_layers, const rg_layer* upd_layer, int aggr,
                              const void* x, int ldx, const void* e, int lde,
                              const int* seg_ptr, const int* src, const int* dst, int n_nodes,
                              void* x_out, int ld_out, const int* wave_nodes, int n_waves,
                              void* workspace, void* stream);

/* ------------------------------------------- object-classifier finetuning */

/* gnn_detector.py:511-513: out[c] = argmax(bincount(node_labels[members of c])) (first
 * maximum) for the proposal clusters (cluster_ptr int32 [n+1], cluster_idx int32);
 * *bad_label (device int32, caller-zeroed) is set when a label is outside [0, n_classes). */
int rg_cluster_majority_label(const int64_t* node_labels, const int* cluster_ptr,
                              const int* cluster_idx, int n_clusters, int n_classes,
                              int64_t* out, int* bad_label, void* stream);
/* Loss_Object_Class (loss.py:79-89): sum_r CE(logits_r, one_hot(label_r)) / n, and
 * compute_accuracy (gnn_detector.py:24-28); loss, accuracy: device float32 [1] */
int rg_cross_entropy(const float* logits, int ld, const int64_t* labels, int n, int nc,
                     float* loss, float* accuracy, void* stream);
/* its gradient: d_logits = g (softmax - one_hot) / n, g a device float32 scalar */
int rg_cross_entropy_backward(const float* logits, int ld, const int64_t* labels, int n, int nc,
                              const float* g, float* d_logits, int ld_d, void* stream);

/* ------------------------------------------- frame-wide normalisations */

/* layer_normalization (groups = 1) / group_normalization (groups = G) of
 * modules/neural_net/common.py:223-253 over row segments (one segment = one frame's rows,
 * the tensor the reference normalises) + the block's activation:
 *   out[r][c] = [residual[r][c] +] act(std_param * (z[r][c] - mean_{s,g}) / (std_{s,g} + 1e-5)
 *               + mu_param),
 * mean / unbiased std over the segment's rows x group g's C/G features.  seg_ptr: device
 * int32 [n_seg+1]; z and out float32 [rows][C] (may alias); residual optional (the conv
 * block's identity, gnn_blocks.py:109).  Deterministic. */
size_t rg_frame_norm_workspace_size(int n_seg, int groups);
int rg_frame_norm(const float* z, int ldz, int C, int groups, const int* seg_ptr, int n_seg,
                  const float* norm_mu, const float* norm_std, int act, const float* residual,
                  int ld_res, float* out, int ld_out, void* workspace, size_t workspace_bytes,
                  void* stream);
/* Backward of rg_frame_norm (training through common.py:223-253, loss.backward()): from
 * the saved pre-norm rows z and the gradient da of the activation output, writes
 * dz = d out / d z (float32 [rows][C]) and ADDS the gradients of the scalar std / mu
 * parameters to *d_std / *d_mu (device float32[1] each, nullable together).  The segment
 * statistics are recomputed as rg_frame_norm computes them; every sum runs in float64 in
 * a fixed order (deterministic). */
size_t rg_frame_norm_backward_workspace_size(int n_seg, int groups);
int rg_frame_norm_backward(const float* z, int ldz, const float* da, int ldda, int C, int groups,
                           const int* seg_ptr, int n_seg, const float* norm_mu,
                           const float* norm_std, int act, float* dz, int lddz, float* d_mu,
                           float* d_std, void* workspace, size_t workspace_bytes, void* stream);
/* out[t] = table[idx[t]] (device int32; per-frame edge offsets = seg_ptr[frame_ptr]) */
int rg_gather_i32(const int* table, const int* idx, int n, int* out, void* stream);
/* out[t] = first position p in sorted[0..n) with sorted[p] >= queries[t] (n from
 * n_sorted_dev when non-NULL, capped at n_sorted): per-frame offsets of rows sorted by
 * node (link pairs by source, clusters by first member) */
int rg_lower_bound_i32(const int* sorted, const int* n_sorted_dev, long n_sorted,
                       const int* queries, int n_queries, int* out, void* stream);

/* ----------------------------------------------------- segment reductions */

/* out[s][c] = reduce_{p in [seg_ptr[s], seg_ptr[s+1])} src[row(p)][c], row(p) =
 * idx ? idx[p] : p.  Sum in segment order (== the reference CPU scatter_add_ order
 * for a destination-major CSR), mean = sum / max(count,1), max with empty -> 0
 * (PyG scatter_reduce include_self=False).  src dtype RG_F32/RG_BF16, out float32
 * or bf16; C <= 256. */
int rg_segment_reduce(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                      const int* idx, int n_seg, int C, int op, void* out, int out_dtype,
                      int ld_out, void* stream);

/* Longest-first schedule for rg_segment_reduce_ordered: order int32[n_seg] = a
 * permutation of the segments by length (seg_ptr[s+1] - seg_ptr[s], capped at 255),
 * descending (a counting sort in one workgroup; ties in timing order).  Computed once
 * per graph, reused by every layer's aggregation.  workspace:
 * rg_segment_order_workspace_size() bytes (currently 0; may be NULL). */
size_t rg_segment_order_workspace_size(void);
int rg_segment_order(const int* seg_ptr, int n_seg, int* order, void* workspace,
                     size_t workspace_bytes, void* stream);
/* rg_segment_reduce (no row index, C a multiple of 64) with lane group i reducing
 * segment order[i]: the segments one wave holds then have similar lengths (a wave waits
 * for its longest).  Graphs of more than 65 536 segments keep the plain order (their
 * rows' locality is worth more: M's kNN CSR).  Same results as rg_segment_reduce, bit for bit: every segment is
 * still summed from its first row in order.  Replaces the PyG aggregation scatter at
 * edge_index[1] (gnn_blocks.py:57, 106) like rg_segment_reduce. */
int rg_segment_reduce_ordered(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                              const int* order, int n_seg, int C, int op, void* out,
                              int out_dtype, int ld_out, void* stream);
/* rg_segment_reduce / _ordered (order nullable) with an explicit schedule instead of the
 * measured defaults: groups = segments per lane group of the streaming kernel (0: the
 * one-segment-per-group kernel), rows_in_flight per lane, narrow_lanes = 1: 16-bit rows
 * as 8-B lane loads.  Compiled schedules: groups 0; (1, 4 / 8 / 12 / 16); (2, 4 / 8);
 * (4, 8); with an order, groups 1 only -- anything else returns RG_ERR_UNSUPPORTED.  Same
 * results, bit for bit, under every schedule (the parity tests sweep them; the library's
 * own entries never read the environment). */
int rg_segment_reduce_sched(const void* src, int src_dtype, int ld_src, const int* seg_ptr,
                            const int* order, int n_seg, int C, int op, void* out, int out_dtype,
                            int ld_out, int groups, int rows_in_flight, int narrow_lanes,
                            void* stream);

/* The same reductions over explicit row ranges [seg_begin[s], seg_end[s]) of src
 * [n_rows] (ranges may overlap): the per-object max-pool of the classifier GNN, whose
 * reference ranges are not a CSR (classifier/classifier.py:60-68, see
 * rg_object_row_ranges) and overlap heavily.  For op = max with a workspace of
 * rg_segment_reduce_ranges_workspace_size() bytes, a first pass writes 32-row block
 * maxima and a long range reads its head rows, its whole blocks and its tail rows
 * (exact); without one every row of every range is read. */
size_t rg_segment_reduce_ranges_workspace_size(long n_rows, int C, int src_dtype);
int rg_segment_reduce_ranges(const void* src, int src_dtype, int ld_src, long n_rows,
                             const int* seg_begin, const int* seg_end, int n_seg, int C, int op,
                             void* out, int out_dtype, int ld_out, void* workspace,
                             size_t workspace_bytes, void* stream);

/* ------------------------------------------- cluster-level classifier GNN */

/* compute_edge_index (data_generator/datagen_classifier.py:124-133): block-diagonal
 * union of complete graphs, one per object of object_size[c] (int64) measurements,
 * no self loops, np.nonzero order.  n_nodes = sum(object_size), n_edges =
 * sum(n (n - 1)).  row_ptr int32[n_nodes+1], col int32[n_edges] (nullable),
 * edge_index int64[2][n_edges] (nullable).  The graph is symmetric: the CSR is also
 * the destination-major view rg_segment_reduce reads. */
size_t rg_object_graph_workspace_size(int n_obj);
int rg_object_complete_graph(const int64_t* object_size, int n_obj, int n_nodes, long n_edges,
                             int* row_ptr, int* col, int64_t* edge_index, void* workspace,
                             size_t workspace_bytes, void* stream);

/* Pooling ranges of the classifier's Model_Inference.forward (classifier.py:60-68),
 * for a batch of samples: sample s owns objects [sample_obj_ptr[s], sample_obj_ptr[s+1])
 * and its rows start at sample_node_base[s] (both int32; NULL = one sample at row 0).
 * Per sample: begin[0] = 0, begin[c] = object_size[c-1], end = cumsum(object_size),
 * each + the sample's row base -- the reference's startidx, reproduced as written.
 * int32 [n_obj] each; workspace rg_object_graph_workspace_size(n_obj). */
int rg_object_row_ranges(const int64_t* object_size, int n_obj, const int* sample_obj_ptr,
                         const int* sample_node_base, int n_samples, int* begin, int* end,
                         void* workspace, size_t workspace_bytes, void* stream);

/* Classifier Loss (classifier/loss.py:5-14): torchvision sigmoid_focal_loss with
 * alpha = -1, gamma = 2 on one-hot targets, summed over classes, averaged over the
 * n objects.  logits f32 [n][ld], labels int64 [n]; out f32 [1].  One workgroup,
 * fixed-order f64 reduction (deterministic). */
int rg_object_focal_loss(const float* logits, int ld, const int64_t* labels, int n, int nc,
                         float* out, void* stream);
/* Its gradient: d_logits[n][ldd] = (g_loss[0] / n) * d(loss_row)/d(logits) (g_loss: f32 [1]
 * on the device, the upstream gradient of the scalar loss). */
int rg_object_focal_loss_backward(const float* logits, int ld, const int64_t* labels, int n,
                                  int nc, const float* g_loss, float* d_logits, int ldd,
                                  void* stream);
/* Backward of the classifier's per-object channel max over rows [begin[o], end[o])
 * (classifier/blocks.py:171-176, torch.max(dim=0)): dx[first argmax row][c] +=
 * d_pooled[o][c] (atomic: the reference's ranges overlap).  x, dx f32. */
int rg_range_max_backward(const float* x, int ldx, int C, const int* begin, const int* end,
                          int n_obj, const float* d_pooled, int ldp, float* dx, int lddx,
                          void* stream);
/* Backward of PyG aggr='max' (scatter_reduce amax, include_self=False) over a
 * destination-major CSR whose position p is message row p: d_msg[p][c] = d_agg[s][c] /
 * (number of maxima) for the messages equal to the segment maximum, else 0 (torch's
 * amax backward).  f32. */
int rg_segment_amax_backward(const float* msg, int ldm, int C, const int* seg_ptr, int n_seg,
                             const float* d_agg, int ldd, float* d_msg, int ldo, void* stream);


/* ------------------------------------------------------------ real-data front-end */

/* read_data.extract_and_sync_radar_data + extract_frame (read_data.py:227-303, 442-486)
 * for a window of n_scans scans already in device memory (measurements of scan s at
 * [scan_ptr[s], scan_ptr[s+1])): the stationary gate of identify_stationary_measurements
 * (meas_selection.py:22-70, 169-200, |predicted - measured range rate| <= gamma; RANSAC
 * below), vr_cartesian_vf (meas_sync.py:15-20) and the ego compensation into the
 * window's current scan (meas_sync.py:23-103), float32 outputs.  A batch of windows is
 * one call: scan_ref[s] = the current scan of scan s's window (NULL: one window whose
 * current scan is the last).  mount: f64 [n_scans][3] (x, y, yaw); odometry: f64
 * [n_scans][5] (x_seq, y_seq, yaw_seq, vx, yaw_rate).  stationary: u8 [n_meas]. */
int rg_frontend_sync(const float* x_cc, const float* y_cc, const float* azimuth_sc,
                     const float* vr, const float* vr_compensated, const int* scan_ptr,
                     int n_scans, const int* scan_ref, const double* mount,
                     const double* odometry,
                     float gamma_stationary, int n_meas, float* px, float* py, float* vx,
                     float* vy, uint8_t* stationary, void* stream);
/* RANSAC stationary-measurement rejection (meas_selection.py:96-166, applied by
 * identify_stationary_measurements to each scan's gated measurements, :188-199), in two
 * calls around the host's random draws (the reference draws np.random.shuffle consensus
 * sets; the host draws the same from numpy's generator, so a seeded generator reproduces
 * the reference):
 *   rg_frontend_gate_lists: gated_idx [n_meas] receives, at each scan's offset scan_ptr[s],
 *     the indices of the scan's measurements whose stationary flag is set, in order;
 *     gated_cnt [n_scans] their count.
 *   rg_frontend_ransac: for each scan with more than min_num_meas gated measurements,
 *     consensus_sets [n_scans][n_iter][n_samples] (positions 0 .. gated_cnt[s) - 1 in the
 *     scan's gated list) -> per set the least-squares sensor velocity (:72-93) and its
 *     inliers (|vr - predicted| <= error_margin) among the other gated measurements; the
 *     first set with the most inliers then sets the gated measurements' stationary flags
 *     (float64 arithmetic over float32 cos / sin, as numpy).  Scans with <= min_num_meas
 *     gated measurements: every flag 0 (the reference's empty inlier set).  in_ratio
 *     [n_scans] f64 = (inliers + n_samples) / gated (0 when skipped), is_valid [n_scans] u8
 *     = in_ratio >= ratio_threshold.  n_iter <= 256. */
int rg_frontend_gate_lists(const uint8_t* stationary, const int* scan_ptr, int n_scans,
                           int* gated_idx, int* gated_cnt, void* stream);
/* Host only (no device work): the consensus sets numpy's legacy generator would draw, for
 * gated_cnt [n_scans] (host) -- per scan with more than min_num_meas, n_iter in-place
 * np.random.shuffle passes over arange(count) (MT19937 + masked-rejection random_interval,
 * numpy/random/mtrand.pyx, distributions.c), the first n_samples of each -- into
 * consensus_sets [n_scans][n_iter][n_samples] (host).  mt_key [624] / *mt_pos: numpy's
 * np.random.get_state()[1] / [2], advanced in place exactly as the shuffles would (write
 * them back with np.random.set_state). */
int rg_ransac_consensus_sets(uint32_t* mt_key, int* mt_pos, const int* gated_cnt, int n_scans,
                             int n_iter, int n_samples, int min_num_meas, int* consensus_sets);
int rg_frontend_ransac(const float* azimuth_sc, const float* vr, const int* scan_ptr, int n_scans,
                       const int* gated_idx, const int* gated_cnt, const int* consensus_sets,
                       int n_iter, int n_samples, double error_margin, int min_num_meas,
                       double ratio_threshold, uint8_t* stationary, double* in_ratio,
                       uint8_t* is_valid, void* stream);
/* compute_ground_truth (compute_node_labels.py:50-105): class labels (tracked: the
 * old -> new label id map, labels.py:90-100; untracked: FALSE = 6 / STATIC = 7 by the
 * stationary flag) and offsets to each track's mean position (track_key int32, 0 = no
 * track, keys <= n_tracks).  f32 outputs. */
size_t rg_frontend_labels_workspace_size(int n_tracks);
int rg_frontend_labels(const int* track_key, int n_tracks, const int64_t* label_id,
                       const uint8_t* stationary, const int* old_to_new, int n_old,
                       const float* px, const float* py, int n_meas, float* cls,
                       float* offset_x, float* offset_y, void* workspace,
                       size_t workspace_bytes, void* stream);
/* select_meas_within_the_grid (grid_features.py:162-174) + select_moving_data
 * (graph_features.py:167-182): index[0..*n_selected) = the measurements inside
 * [min_x, max_x) x [min_y, max_y) whose class is not static_id, in order.  With a batch
 * of windows (measurements of window w at [win_ptr[w], win_ptr[w+1])), frame_ptr
 * [n_windows + 1] receives each window's range of selected rows (the graph build's
 * frame_ptr); both may be NULL. */
size_t rg_frontend_select_workspace_size(int n_meas);
int rg_frontend_select(const float* px, const float* py, const float* cls, int n_meas,
                       float min_x, float max_x, float min_y, float max_y, float static_id,
                       const int* win_ptr, int n_windows, int* frame_ptr, int* index,
                       int* n_selected, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------ proposal branch */

/* Predicted cluster centres (gnn_detector.py:164-167): unnormalize_gt_offsets
 * (compute_offsets.py:13-17, offset * sigma + mu) added to other_features[:, :2];
 * float32, no FMA.  offsets: f32 [N][ld_off] (node_offsets_predictions), xy: f32
 * [N][ld_xy]; cx, cy: f32 [N]. */
int rg_proposal_centres(const float* offsets, int ld_off, const float* xy, int ld_xy, int n_nodes,
                        float mu_x, float mu_y, float sigma_x, float sigma_y, float* cx,
                        float* cy, void* stream);

/* Connected components of the eps-graph on the centres, per frame
 * (Simple_DBSCAN with compute_adjacency_mat_from_predicted_offsets, clustering.py:26-93:
 * an edge where the SQUARED distance <= eps2).  labels: int32 [N], label = the
 * component's lowest global node index. */
size_t rg_cluster_radius_workspace_size(int n_nodes, int n_frames, int max_frame_nodes);
int rg_cluster_radius(const float* px, const float* py, const int* frame_ptr, int n_nodes,
                      int n_frames, int max_frame_nodes, float eps2, int* labels,
                      void* workspace, size_t workspace_bytes, void* stream);

/* Connected components over predicted links (compute_adjacency_mat_from_predicted_edges,
 * clustering.py:8-23): pair p = (pair_src[p], pair_dst[p]) is an edge when
 * link_logits[p][1] > link_logits[p][0] (the argmax of gnn_detector.py:158-159) and
 * sqrt(dx^2 + dy^2) < eps on the centres.  labels as rg_cluster_radius. */
int rg_cluster_pairs(const float* px, const float* py, const int* pair_src, const int* pair_dst,
                     const int* n_pairs_dev, long n_pairs, const float* link_logits,
                     int ld_logits, float eps, int n_nodes, int* labels, void* stream);

/* Cluster ids in the reference's order (ascending lowest node index; frames are
 * concatenated, each numbered from its own first cluster) and the member lists,
 * ascending (gnn_detector.py:180-184): cluster_of int32 [N], cluster_ptr int32 [N+1]
 * (entries past *n_clusters repeat N), cluster_idx int32 [N], *n_clusters device int. */
size_t rg_cluster_lists_workspace_size(int n_nodes);
int rg_cluster_lists(const int* labels, int n_nodes, int* cluster_of, int* cluster_ptr,
                     int* cluster_idx, int* n_clusters, void* workspace, size_t workspace_bytes,
                     void* stream);


/* ------------------------------------------------------------------ training */
/* The backward of the hot path (Model_Training + Loss_Graph + loss.backward(),
 * gnn_detector.py:428-478, loss.py:37-76, training.py:66-85), float32.  Forward
 * tapes come from rg_mlp_chain with rg_layer.save_pre / save_out set. */

/* Backward of channel_normalization + activation (common.py:208-220, 256-267) for
 * `rows` rows of width C: from the saved pre-normalisation z and the gradient of the
 * activation output da, dz (may alias da) and the gradients of the scalar parameters,
 * ACCUMULATED into *d_mu / *d_std (device; deterministic order).  has_norm = 0: only
 * the activation.  workspace: rg_ffn_backward_workspace_size() bytes. */
size_t rg_ffn_backward_workspace_size(void);
int rg_ffn_backward(const float* z, int ldz, const float* da, int ldda, long rows, int C,
                    int has_norm, const float* mu, const float* std_, int act, float* dz,
                    int lddz, float* d_mu, float* d_std, void* workspace, void* stream);
/* The same with the activation gradient gathered: row r reads da[gidx[r]] (times
 * gscale[gidx[r]] when gscale is non-NULL) -- d msg = d agg[dst] of the message MLP's last
 * layer (sum / mean aggregation, gnn_blocks.py:104-113) without materialising d msg;
 * the same values as rg_gather_segment_sum followed by rg_ffn_backward.  dz may not alias da. */
int rg_ffn_backward_gather(const float* z, int ldz, const float* da, int ldda, const int* gidx,
                           const float* gscale, long rows, int C, int has_norm, const float* mu,
                           const float* std_, int act, float* dz, int lddz, float* d_mu,
                           float* d_std, void* workspace, void* stream);

/* dA = dz_next W (layer: ONE transposed RG_F32 | RG_PACK_F32_FAST image, in_dim = the width of
 * dz_next, out_dim = C, as the backward's dX launches use) with the previous ffn_block's
 * channel_normalization + activation backward (common.py:208-220, 256-267) applied in the
 * same registers: dz = rg_ffn_backward(z, dA), d_mu / d_std ACCUMULATED -- dA never reaches
 * memory.  has_norm is implied (mu / std required); act RG_ACT_NONE or RG_ACT_LEAKY; (in_dim,
 * C) in {(64, 128), (128, 128), (64, 64)}, else RG_ERR_UNSUPPORTED (the caller runs the two
 * steps).  Row sums in float32, their sums over rows in float64 in a fixed order:
 * bit-reproducible.  workspace: rg_dx_norm_backward_workspace_size(rows) bytes. */
size_t rg_dx_norm_backward_workspace_size(long rows);
int rg_dx_norm_backward(const rg_layer* layer, long rows, const float* dz_next, int ld_dzn,
                        const float* z, int ldz, const float* mu, const float* std_, int act,
                        float* dz, int lddz, float* d_mu, float* d_std, void* workspace,
                        size_t workspace_bytes, void* stream);

/* Weight / bias gradient of nn.Linear (common.py:195): dW[out][in] += sum_r dz[r]^T x[r],
 * db[out] += sum_r dz[r] (db may be NULL), x[r] formed from in0/in1/in2 by in_mode as in
 * rg_mlp_chain (float32 inputs).  Rows are reduced in fixed chunks, the chunk partials
 * in a fixed order: bit-reproducible.  workspace: rg_linear_grad_workspace_size(). */
size_t rg_linear_grad_workspace_size(long rows, int out_dim, int in_dim);
int rg_linear_grad(const float* dz, int lddz, long rows, int out_dim, int in_dim, int in_mode,
                   const float* in0, int ld0, int w0, const float* in1, int ld1, int w1,
                   const float* in2, int ld2, int w2, const int* idx0, const int* idx1,
                   float* dW, float* db, void* workspace, size_t workspace_bytes, void* stream);
/* The same into a column block of a wider dW: rows ld_dw floats apart (>= in_dim). */
int rg_linear_grad_ld(const float* dz, int lddz, long rows, int out_dim, int in_dim, int in_mode,
                      const float* in0, int ld0, int w0, const float* in1, int ld1, int w1,
                      const float* in2, int ld2, int w2, const int* idx0, const int* idx1,
                      float* dW, int ld_dw, float* db, void* workspace, size_t workspace_bytes,
                      void* stream);

/* Incidence lists: for node n, every u < n_items with a[u] == n or b[u] == n (b may be
 * NULL), ascending: ptr int32 [n_nodes+1], list int32 [n_items * (b ? 2 : 1)].  The
 * transpose of an index_select (PyG x_j = x[edge_index[0]], the link pairs' x[i] + x[j]),
 * used to sum its gradient per node in a fixed order. */
size_t rg_incidence_workspace_size(int n_nodes, long n_items);
int rg_incidence(const int* a, const int* b, long n_items, int n_nodes, int* ptr, int* list,
                 void* workspace, size_t workspace_bytes, void* stream);

/* out[n][0:width] (+)= sum_{k in [ptr[n], ptr[n+1])} src[row(k)][col0 : col0 + width],
 * row(k) = list ? list[k] : k; scale (per row of src, may be NULL) multiplies each term
 * (PyG mean: 1 / count).  accumulate = 0 overwrites.  float32, width <= 256. */
int rg_gather_segment_sum(const float* src, int ld_src, int col0, int width, const int* ptr,
                          const int* list, const float* scale, int n_nodes, float* out,
                          int ld_out, int accumulate, void* stream);

/* Backward of the per-cluster channel max (object_classification gnn_blocks.py:384-387,
 * torch.max(dim=0)): dh[argmax_c(f)][f] += dpooled[c][f], argmax = first maximum in
 * list order.  h float32 [N][ld_h]; cluster lists as rg_segment_reduce's idx CSR. */
int rg_segment_max_backward(const float* h, int ld_h, int C, const int* cluster_ptr,
                            const int* cluster_idx, int n_clusters, const float* dpooled,
                            int ld_p, float* dh, int ld_dh, void* stream);

/* Loss_Graph.forward (loss.py:37-76) + compute_accuracy (gnn_detector.py:24-28).
 * node_cls f32 [N][nc], node_reg f32 [N][2], link f32 [U][2], obj f32 [Ncl][nc];
 * labels int64 (node_class [N], edge_class [U], obj_class [Ncl]); node_offsets f32
 * [N][2] raw (normalised inside: (o - mu) / sigma, compute_offsets.py:6-11);
 * class_w f32 [nc].  losses f32 [4] = weighted (node_cls, node_reg, edge_cls, obj_cls)
 * as loss.py:71-75, acc f32 [3] = (segment, edge, object) accuracy (device). */
typedef struct rg_loss_args {
  const float* node_cls; const float* node_reg; const float* link; const float* obj;
  const long long* node_class; const float* node_offsets; const long long* edge_class;
  const long long* obj_class; const float* class_w;
  long n_nodes; long n_pairs; long n_clusters; int n_classes;
  float mu_x, mu_y, sigma_x, sigma_y;
  float w_node_cls, w_node_reg, w_edge_cls, w_obj_cls;
} rg_loss_args;
size_t rg_loss_workspace_size(long n_nodes, long n_pairs, long n_clusters);
int rg_loss_graph(const rg_loss_args* args, float* losses, float* acc, void* workspace,
                  size_t workspace_bytes, void* stream);
/* d(sum_i g[i] * losses[i]) / d(logits) (g: device f32 [4], the upstream gradients of
 * the four losses): d_node_cls [N][nc], d_node_reg [N][2], d_link [U][2], d_obj [Ncl][nc]. */
int rg_loss_graph_backward(const rg_loss_args* args, const float* g, float* d_node_cls,
                           float* d_node_reg, float* d_link, float* d_obj, void* stream);

/* torch.optim.SGD step (dampening 0, no nesterov; set_param_for_training_gnn.py:46) on
 * flat float32 arrays: d = grad_scale g + wd p; buf = first ? d : momentum buf + d;
 * p -= lr buf.  grad_scale = 1 / world_size averages an all-reduced (summed) gradient
 * as DistributedDataParallel does; 1 on one GPU (exact). */
int rg_sgd_step(float* param, const float* grad, float* momentum_buf, long n, float lr,
                float momentum, float weight_decay, int first_step, float grad_scale,
                void* stream);

/* The optimizer step of the reference's train_model loop (training.py:66-85) with its two
 * host-side rules evaluated on the device, so a data-parallel step needs no host sync:
 *  - skip_batch (training.py:40-45, 79-85): when losses[0] + ... + losses[n_losses-1]
 *    (float32, left to right) is NaN, param and the optimizer state are left untouched and
 *    the step is not counted.  The DDP trainer all-reduces the losses in the same bucket as
 *    the gradients, so a NaN on any rank reaches every rank and all ranks skip together.
 *    losses = NULL: never skip.
 *  - MultiStepLR (set_param_for_training_gnn.py:51-56, stepped only after an applied step,
 *    training.py:83-84): applied step k (0-based) uses lr[j], j = the number of distinct
 *    milestones ms[i] <= k.  The host fills lr[] exactly as the scheduler chains it (in
 *    double: lr[j] = lr[j-1] * gamma ** multiplicity(ms[j-1])); milestones < 0 never fire
 *    and are dropped by the host, milestone 0 fires before the first step.
 * step_state: device int[2], the applied-step counter ping-ponged between launches: the
 * launch reads step_state[parity] and writes step_state[parity ^ 1]; the caller flips
 * parity every launch (both zero before the first).  The first applied step (k = 0)
 * initialises the momentum buffer (torch's momentum_buffer = None). */
#define RG_LR_MILESTONES_MAX 16
typedef struct rg_lr_schedule {
  int n_milestones;                        /* distinct, ascending, >= 0 */
  int milestones[RG_LR_MILESTONES_MAX];
  double lr[RG_LR_MILESTONES_MAX + 1];
} rg_lr_schedule;
int rg_sgd_step_sched(float* param, const float* grad, float* momentum_buf, long n,
                      const rg_lr_schedule* sched, float momentum, float weight_decay,
                      float grad_scale, const float* losses, int n_losses, int* step_state,
                      int parity, void* stream);
/* torch.optim.AdamW (set_param_for_training_gnn.py:47; amsgrad off, the foreach update
 * order) with the same skip / schedule / step_state rules (the hyper-parameters are
 * doubles, as Python holds them; each scalar is formed in double, then rounded): t = k + 1;
 * p *= 1 - lr wd; m = lerp(m, g, 1 - beta1); v = beta2 v + (1 - beta2) g g;
 * p += -(lr / (1 - beta1^t)) m / (sqrt(v) / sqrt(1 - beta2^t) + eps). */
int rg_adamw_step_sched(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        long n, const rg_lr_schedule* sched, double beta1, double beta2,
                        double eps, double weight_decay, float grad_scale, const float* losses,
                        int n_losses,
                        int* step_state, int parity, void* stream);

/* ---------------------------------------------------------------- diagnostics */

/* Shader-clock calibration (bench.py; no product path calls it): n_blocks workgroups of
 * 256 threads, each wave one dependent chain of n_mfma (a multiple of 64)
 * v_mfma_f32_32x32x16_bf16 on register operands, stamped with s_memtime / s_memrealtime
 * around the chain.  out: device u64
 * [n_blocks][2] = (shader cycles, wall-clock ticks) of each workgroup's wave 0; sink: device
 * f32 [n_blocks * 4] (the chains' results); *wall_clock_khz_host = the wall-clock tick rate
 * (hipDeviceAttributeWallClockRate).  clock = cycles / ticks x rate. */
int rg_clock_probe(int n_blocks, int n_mfma, unsigned long long* out, float* sink,
                   int* wall_clock_khz_host, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RADAR_GNN_H */
