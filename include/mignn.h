/*
 * mignn.h -- C ABI of libmignn.so, the MI355X (gfx950) GNN message-passing
 * engine behind FlowGNN.forward (reference: gnn_model.py:104-197).
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer owned by the caller (PyTorch's
 *     caching allocator in the shipped host code).  The library never
 *     allocates persistent device memory, never frees, never synchronises the
 *     stream: scratch is passed in, `stream` is a hipStream_t passed as void*.
 *   - Row-major fp32 activations; `ld*` arguments are row strides in elements
 *     and must be multiples of 4 (16-byte rows) where a kernel loads float4.
 *   - Return value: 0 = MIGNN_OK; nonzero codes below.  mignn_last_error()
 *     returns a thread-local description of the last failure.  The host shim
 *     maps failures inside a layer to the reference's
 *     RuntimeError("Message passing failed in layer i (type): ...")
 *     (gnn_model.py:173-181).
 *   - Re-entrant per stream; no internal host threads.
 */
#ifndef MIGNN_H
#define MIGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIGNN_ABI_VERSION 1

enum mignn_status {
    MIGNN_OK = 0,
    MIGNN_ERR_ARG = 1,          /* bad shape / null pointer / alignment        */
    MIGNN_ERR_UNSUPPORTED = 2,  /* configuration without a kernel              */
    MIGNN_ERR_HIP = 3,          /* HIP launch / runtime error                  */
    MIGNN_ERR_SCRATCH = 4       /* scratch buffer too small                    */
};

int mignn_abi_version(void);
const char* mignn_last_error(void);

/* In-kernel protocol failures, sticky per device (a __device__ word of the
 * library, not caller memory): MIGNN_DEVERR_SPIN = a bounded wait inside a
 * fused layer kernel (gcn_f16x3.hip's LDS hand-offs) ran out -- that
 * launch's output is wrong.  Reads (synchronously, after the device is idle)
 * and optionally clears the word of the current device into *out. */
/* MIGNN_DEVERR_PLAN = a window-kernel launch whose plan header does not match
 * it (another grid size, width or row range: mignn_gcn_win_plan was built for
 * a different launch); the launch writes nothing. */
enum { MIGNN_DEVERR_SPIN = 1, MIGNN_DEVERR_PLAN = 2 };
int mignn_device_errors(unsigned int* out, int clear);

/* ------------------------------------------------------------------------
 * Graph structure.
 * Replaces, on the device and without host syncs:
 *   - the edge validation / silent filtering / all-invalid self-loop fallback
 *     of gnn_model.py:125-149 (the reference does two .item() syncs here);
 *   - PyG add_remaining_self_loops + gcn_norm's degree (GCNConv, gnn_model.py:63)
 *     and remove_self_loops + add_self_loops (GATConv, gnn_model.py:65-68):
 *     mode MIGNN_CSR_ONE_SELF_LOOP;
 *   - the verbatim edge list GINConv / TransformerConv aggregate over
 *     (gnn_model.py:70-80): mode MIGNN_CSR_VERBATIM.
 * Output: destination-major CSR (row_ptr[N+1], col[<= E+N]) with the
 * in-row order equal to the edge order of `edge_index` (stable), the
 * appended self-loop last; dinv[i] = deg_i^-1/2 (ONE_SELF_LOOP mode, may be
 * NULL).  info (device int64[4], may be NULL) = {kept edges, invalid edges,
 * nnz, all-invalid fallback taken}.
 * ------------------------------------------------------------------------ */
/* | MIGNN_CSR_TRANSPOSE: the CSR of the reversed edges (rows keyed by the
 * source; same filtering and self-loop rules), i.e. the transpose of the
 * aggregation -- the backward of a sum aggregation (training).
 * dinv is then the source-side degree and unused by the backward. */
enum { MIGNN_CSR_VERBATIM = 0, MIGNN_CSR_ONE_SELF_LOOP = 1, MIGNN_CSR_TRANSPOSE = 4 };

size_t mignn_csr_scratch_bytes(int64_t num_edges, int64_t num_nodes);
/* As mignn_csr_build, with every valid node id x of edge_index mapped to
 * relabel[x] (a permutation of [0, N), e.g. the inverse locality order
 * below): the CSR of the relabelled graph.  In-row order is still the edge
 * order of edge_index.  mignn_csr_build == this with relabel = NULL. */
int mignn_csr_build_relabeled(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                              int mode, const int32_t* relabel, int32_t* row_ptr, int32_t* col,
                              float* dinv, int64_t* info, void* scratch, size_t scratch_bytes,
                              void* stream);
/* As mignn_csr_build_relabeled; in ONE_SELF_LOOP mode `ew` (nullable, one
 * float per CSR entry) also receives the PyG gcn_norm weights of
 * mignn_gcn_norm over all rows (bit-identical: dinv[src] * dinv[i]) -- the
 * GCN forward's CSR in one pass. */
int mignn_csr_build_gcn(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes, int mode,
                        const int32_t* relabel, int32_t* row_ptr, int32_t* col, float* dinv,
                        float* ew, int64_t* info, void* scratch, size_t scratch_bytes,
                        void* stream);
/* As mignn_csr_build_gcn for one node-range shard (mignn.dist.RangeLayout):
 * edge_index holds GLOBAL ids (destinations in [lo, hi) of num_nodes), mapped
 * in the build's first pass to the shard's local ids exactly as
 * mignn_range_relabel maps them (inv, ghost_rank as there) -- the CSR of the
 * relabelled list without writing that list.  n_local = n_own + ghosts (the
 * CSR's node count); scratch as mignn_csr_scratch_bytes(num_edges, n_local).
 * No transposed mode.  (Replaces mignn_range_relabel + mignn_csr_build_gcn on
 * the shard route; the reference has no sharded path) */
int mignn_csr_build_range(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                          int64_t lo, int64_t hi, const int64_t* inv, const int64_t* ghost_rank,
                          int64_t n_local, int mode, int32_t* row_ptr, int32_t* col, float* dinv,
                          float* ew, int64_t* info, void* scratch, size_t scratch_bytes,
                          void* stream);

/* Locality order of the nodes for the internal activation layout (no
 * reference counterpart: the forward's results are the same up to fp32
 * summation order).  pos: [n, >=3] cell centres (FlowGNN's node features,
 * reference graph_constructor.py:259), row stride ldp.  Cells of the mesh
 * spacing (per axis, from the edges) are grouped into 4x4x4 blocks (a 64-row
 * tile of the fused layer each), the blocks into panels of 4x4 block columns
 * swept along the third axis.
 * Outputs perm[new] = old node id and inv[old] = new (int32, n each); stable
 * (ties keep input order).  Scratch: mignn_locality_order_scratch_bytes(n). */
size_t mignn_locality_order_scratch_bytes(int64_t n);
int mignn_locality_order(const float* pos, int64_t ldp, int64_t n, const int64_t* edge_index,
                         int64_t num_edges, int32_t* perm, int32_t* inv, void* scratch,
                         size_t scratch_bytes, void* stream);
/* Column order (the window GCN kernel's): cells grouped into 8 x 8 columns
 * along the third axis, a column's cells in (z, y, x) order -- every 64-row
 * tile of a full column is one z-plane -- full columns first in row-major
 * (y, x) column order, then the ragged edges' columns.  info (nullable,
 * device int32[4]) = {1, planes per column, full columns, full columns per
 * row}: pass it to mignn_gcn_win_plan.  Same scratch as mignn_locality_order. */
int mignn_locality_order_cols(const float* pos, int64_t ldp, int64_t n, const int64_t* edge_index,
                              int64_t num_edges, int32_t* perm, int32_t* inv, int32_t* info,
                              void* scratch, size_t scratch_bytes, void* stream);
int mignn_csr_build(const int64_t* edge_index, /* [2, E] int64, contiguous */
                    int64_t num_edges, int64_t num_nodes, int mode,
                    int32_t* row_ptr, int32_t* col, float* dinv, int64_t* info,
                    void* scratch, size_t scratch_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Dense node transforms (MFMA f32 16x16x4, exact fp32).
 * C[m, :] = epi( [A | A2][m, :] . W^T ),  W is [n, k + k2] (torch Linear layout).
 * epi (flags): +bias[n] -> relu_pre? -> +residual -> *scale+shift -> relu.
 * Used for nn.Linear (input_proj gnn_model.py:55, output_proj :90-100, GIN nn
 * :70-74) and the conv transforms.  k, k2 multiples of 4.
 * ------------------------------------------------------------------------ */
enum {
    MIGNN_EPI_BIAS = 1,
    MIGNN_EPI_RESIDUAL = 2,
    MIGNN_EPI_AFFINE = 4, /* BatchNorm eval affine: v*scale + shift */
    MIGNN_EPI_RELU = 8,
    /* the product entry points reject any other flag bit (timing ablations
     * live in include/mignn_diag.h, behind mignn_diag_* entry points) */
    MIGNN_EPI_MASK = 15
};
int mignn_linear(const float* a, int64_t lda, int64_t m, int k,
                 const float* a2, int64_t lda2, int k2,
                 const float* w, int n,
                 const float* bias, const float* residual, int64_t ldr,
                 const float* scale, const float* shift, int flags,
                 float* c, int64_t ldc, void* stream);

/* The same transform in split-fp16 MFMA arithmetic ("f16x3", ~2^-22 relative
 * per product, 16x the f32 MFMA rate), for the shapes the fused layer kernels
 * do not cover (k or n > 128: the H = 256 layers, GAT's head-mean GEMM,
 * TransformerConv's Q~K / output GEMMs).  W [n, k + k2] is split once into a
 * device image (mignn_linear_f16x3_prep_bytes(n, k + k2) bytes, 16-B aligned;
 * fp16 hi/lo MFMA fragments + one scale exponent per output column); rebuild
 * it whenever W changes.  A rows are scaled by an online per-row power of two
 * (no pre-pass).  Same epilogue flags and layout rules as mignn_linear;
 * k1, k2, lda, lda2 multiples of 4. */
size_t mignn_linear_f16x3_prep_bytes(int n, int k);
int mignn_linear_f16x3_prep(const float* w, int n, int k, void* img, size_t img_bytes,
                            void* stream);
int mignn_linear_f16x3(const float* a, int64_t lda, int64_t m, int k1,
                       const float* a2, int64_t lda2, int k2,
                       const void* img, int n,
                       const float* bias, const float* residual, int64_t ldr,
                       const float* scale, const float* shift, int flags,
                       float* c, int64_t ldc, void* stream);

/* Linear(in_dim -> h) with in_dim <= 8 on the VALU (K too thin for MFMA):
 * input_proj, gnn_model.py:55, :159. */
int mignn_input_proj(const float* x, int64_t n, int in_dim, const float* w, const float* b,
                     int h, float* out, int64_t ldo, void* stream);
/* out row r = Linear(x row rows[r]) (rows = NULL: r): the projection gathered
 * into the locality order. */
int mignn_input_proj_rows(const float* x, int64_t n, int in_dim, const int32_t* rows,
                          const float* w, const float* b, int h, float* out, int64_t ldo,
                          void* stream);

/* BatchNorm1d eval fold: scale = w / sqrt(var + eps), shift = b - mean*scale
 * (the same fold ATen's CPU batch_norm applies).  BatchNorm, gnn_model.py:87. */
int mignn_bn_fold(const float* weight, const float* bias, const float* mean, const float* var,
                  float eps, int h, float* scale, float* shift, void* stream);

/* ------------------------------------------------------------------------
 * Aggregations (rows [row_begin, row_end) of the CSR; out row r at out+r*ldo).
 * ------------------------------------------------------------------------ */
/* GCN: out_i = sum_{j in row i} dinv_j dinv_i x_j  (PyG gcn_norm weights) */
int mignn_gcn_aggregate(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                        const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                        float* out, int64_t ldo, void* stream);
/* GIN: out_i = sum_{j in row i} x_j + self_scale * x_i  (self_scale = 1 + eps) */
int mignn_sum_aggregate(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                        float self_scale, int64_t row_begin, int64_t row_end, int h,
                        float* out, int64_t ldo, void* stream);
/* GAT (heads <= 8): logits [N, 2*heads] = (a_src | a_dst).
 * out_i[hd] = sum_j softmax_j(LeakyReLU(a_src[j,hd] + a_dst[i,hd])) x_j, out [*, heads*h] */
int mignn_gat_aggregate(const int32_t* row_ptr, const int32_t* col, const float* logits,
                        const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                        int heads, float negative_slope, float* out, int64_t ldo, void* stream);
/* TransformerConv (heads <= 8): qt row = [q~_0 .. q~_{heads-1} | c_0 .. c_{heads-1}]
 * (q~_hd = Wk_hd^T q_hd, c_hd = q_hd . bk_hd, ldq >= heads*h + heads).
 * s_ji = (q~_i . x_j + c_i) * score_scale; alpha = softmax over row i;
 * out row = [sum_j alpha x_j per head | sum_j alpha per head]. */
int mignn_transformer_aggregate(const int32_t* row_ptr, const int32_t* col, const float* qt,
                                int64_t ldq, const float* x, int64_t ldx, int64_t row_begin,
                                int64_t row_end, int h, int heads, float score_scale,
                                float* out, int64_t ldo, void* stream);

/* Whole GATConv / TransformerConv eval layers (+ residual, BN eval affine,
 * ReLU: flags as mignn_linear) in one call each (csrc/attn_layers.hip), over
 * rows [row_begin, row_end) of x (x holds every row the CSR references:
 * n_x rows, own + halo).  Transforms in split-fp16 arithmetic when the
 * weight's mignn_linear_f16x3_prep image is given, else exact fp32.
 * GAT: wlog [2*heads, h] = per-head W^T att_src | W^T att_dst (re-associated
 * logit weights), wcat [h, heads*h] = head-mean blocks of W; `logits`
 * ([n_x, 2*heads], ldl = 2*heads) may be given instead of wlog (a sharded
 * caller's exchanged logits).  Transformer: wqk [heads*h, h] = Wk^T Wq per
 * head and bqk [heads*h] = Wk^T bq per head (q~ of mignn_transformer_aggregate;
 * its per-head constant c = q . bk is left out: the softmax cancels it),
 * wout [h, heads*h + heads + h] = [Wv / heads | bv / heads | W_skip], bout =
 * b_skip.  scratch: the *_scratch_bytes sizes, 16-B aligned, device memory.
 * GAT flags may also carry MIGNN_GAT_LAUNCHES: the aggregate + transform
 * launch sequence even where the fused kernel applies (same results up to
 * fp32 summation order; an explicit per-call choice, no library state). */
enum { MIGNN_GAT_LAUNCHES = 64 };
size_t mignn_gat_layer_scratch_bytes(int64_t n_x, int64_t rows, int h, int heads);
int mignn_gat_layer(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                    int64_t n_x, int64_t row_begin, int64_t row_end, int h, int heads,
                    float negative_slope, const float* wlog, const float* logits, int64_t ldl,
                    const float* wcat, const void* wcat_img, const float* bias,
                    const float* scale, const float* shift, int flags, void* scratch,
                    size_t scratch_bytes, float* out, int64_t ldo, void* stream);
/* mignn_gat_layer that also writes the NEXT GAT layer's logits of its rows,
 * logits_next[r][2*heads] = out[r] . wlog_next^T (wlog_next: the next layer's
 * wlog), from the fused kernel's epilogue (the [rows, 2*heads] logit GEMV of
 * the next call is then skipped by passing logits_next as its `logits`). */
int mignn_gat_layer_next(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                         int64_t n_x, int64_t row_begin, int64_t row_end, int h, int heads,
                         float negative_slope, const float* wlog, const float* logits,
                         int64_t ldl, const float* wcat, const void* wcat_img, const float* bias,
                         const float* scale, const float* shift, int flags, void* scratch,
                         size_t scratch_bytes, float* out, int64_t ldo, const float* wlog_next,
                         float* logits_next, void* stream);
size_t mignn_transformer_layer_scratch_bytes(int64_t rows, int h, int heads);
int mignn_transformer_layer(const int32_t* row_ptr, const int32_t* col, const float* x,
                            int64_t ldx, int64_t row_begin, int64_t row_end, int h, int heads,
                            float score_scale, const float* wqk, const void* wqk_img,
                            const float* bqk, const float* wout, const void* wout_img,
                            const float* bout, const float* scale, const float* shift, int flags,
                            void* scratch, size_t scratch_bytes, float* out, int64_t ldo,
                            void* stream);
/* TransformerConv at h = 256, 4 heads (configs[3]) with the aggregation and
 * the output transform in one kernel (the [rows, heads*h + heads] aggregate
 * never reaches memory): qt = x wqk^T + bqk (split-fp16 GEMM into scratch),
 * then per row the scores, softmax and weighted sums feed the output
 * transform directly.  wout_fimg: mignn_transformer_fused_prep's image of
 * wout (same wout as mignn_transformer_layer, k reordered for the kernel);
 * the other arguments and the scratch size as mignn_transformer_layer.
 * Rows with more than 24 CSR entries are correct, not fast. */
size_t mignn_transformer_fused_prep_bytes(int h, int heads);
int mignn_transformer_fused_prep(const float* wout, int h, int heads, void* img, size_t img_bytes,
                                 void* stream);
int mignn_transformer_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* x,
                                  int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                                  int heads, float score_scale, const void* wqk_img,
                                  const float* bqk, const void* wout_fimg, const float* bout,
                                  const float* scale, const float* shift, int flags, void* scratch,
                                  size_t scratch_bytes, float* out, int64_t ldo, void* stream);

/* PyG gcn_norm edge weights per CSR entry (rows [row_begin, row_end)):
 *   ew[e] = dinv[col[e]] * dinv[i]   (= dinv[src] * 1 * dinv[dst], GCNConv gnn_model.py:63) */
int mignn_gcn_norm(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                   int64_t row_begin, int64_t row_end, float* ew, void* stream);

/* ------------------------------------------------------------------------
 * Fused GCN layer (the north-star hot kernel):
 *   out_i = relu( ((x_i + (sum_{e in row i} ew_e x_{col e}) W^T + bias) * scale + shift) )
 * i.e. GCNConv + residual + BatchNorm(eval) + ReLU of gnn_model.py:166,184-191
 * in one pass: CSR gather into an LDS tile, MFMA transform, fused epilogue.
 * ew: per-CSR-entry weights from mignn_gcn_norm.
 * flags: MIGNN_EPI_* (BIAS|RESIDUAL|AFFINE|RELU as the model configures).
 * h in {64, 128} (other h: mignn_gcn_aggregate + mignn_linear).
 * ------------------------------------------------------------------------ */
int mignn_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* ew,
                    const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                    const float* w, const float* bias, const float* scale, const float* shift,
                    int flags, float* out, int64_t ldo, void* stream);

/* Same layer, split-precision transform ("f16x3"): every fp32 operand of the
 * node transform is split into two power-of-two-scaled fp16 halves and the
 * product is formed by three fp16 MFMAs with fp32 accumulation (relative
 * error per product ~2^-22, i.e. within a few fp32 ulps; 16x the f32 MFMA
 * rate).  In-tile CSR entries (a locality order, mignn_locality_order, puts
 * most of a mesh's entries there) are read from an LDS image of the tile's
 * own rows; the rest are gathered.  Sum order: a row's in-tile entries in CSR
 * order, then its out-of-tile entries in CSR order.  h in {64, 128}; same
 * arguments and flags as mignn_gcn_layer. */
int mignn_gcn_layer_f16x3(const int32_t* row_ptr, const int32_t* col, const float* ew,
                          const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                          const float* w, const float* bias, const float* scale,
                          const float* shift, int flags, float* out, int64_t ldo, void* stream);

/* Ring form of mignn_gcn_layer_f16x3 (csrc/gcn_ring.hip), the route of a
 * block-ordered H = 64 row range (a shard's): own rows, plan records and
 * out-of-tile rows all arrive by LDS-DMA issued up to 1.5 tiles ahead, one
 * 8-wave workgroup per CU.  Its plan (mignn_gcn_ring_plan, size
 * mignn_gcn_ring_plan_bytes) also fixes the kernel's schedule (the LDS ring
 * slot of every tile): build it on the device that runs the layer; its
 * header (grid, h, row range) is checked at launch (MIGNN_DEVERR_PLAN on a
 * mismatch, no rows written).  Sum
 * order: a row's CSR entries in CSR order.  stats (nullable, device uint64[4]):
 * tiles over the out-of-tile capacity, entries gathered synchronously, rows
 * with more than 7 entries, max out-of-tile entries of a tile. */
size_t mignn_gcn_ring_plan_bytes(int64_t row_begin, int64_t row_end, int h);
int mignn_gcn_ring_plan(const int32_t* row_ptr, const int32_t* col, const float* ew,
                        int64_t row_begin, int64_t row_end, int h, void* plan, size_t plan_bytes,
                        unsigned long long* stats, void* stream);
int mignn_gcn_layer_ring(const void* plan, const int32_t* row_ptr, const int32_t* col,
                         const float* ew, const float* x, int64_t ldx, int64_t row_begin,
                         int64_t row_end, int h, const float* w, const float* bias,
                         const float* scale, const float* shift, int flags, float* out,
                         int64_t ldo, void* stream);
/* The GCN aggregation alone by the ring kernel (mignn_gcn_ring_plan's plan
 * for the same h): out_i = sum_e ew_e x_{col e} in CSR order, fp32. */
int mignn_gcn_aggregate_ring(const void* plan, const int32_t* row_ptr, const int32_t* col,
                             const float* ew, const float* x, int64_t ldx, int64_t row_begin,
                             int64_t row_end, int h, float* out, int64_t ldo, void* stream);
/* Window form of the same layer (csrc/gcn_win.hip), the product route at
 * H = 64 and 128: a tile is a 64-row slice of the node order; a workgroup
 * walks consecutive tiles (in the column order of mignn_locality_order_cols:
 * one z-plane of an 8 x 8-cell column after another), keeping the previous
 * and the current tile in LDS, so only a plane's lateral faces are
 * out-of-tile rows.  The plan (mignn_gcn_win_plan, size
 * mignn_gcn_win_plan_bytes; device memory, 16-B aligned) carries a header
 * with the launch grid and schedule, checked by the layer kernel
 * (MIGNN_DEVERR_PLAN on a mismatch), and a 16-B record per row: the
 * neighbours' LDS codes with their degree classes -- the weights are rebuilt
 * as dinv_j dinv_i (dinv = (deg + 1)^-1/2), so a row whose ew is not that
 * gcn_norm product bitwise (a weighted graph, a neighbour of degree > 8) is
 * planned onto the CSR path, which reads ew itself: any CSR stays correct.
 * order_info (nullable: the int32[4] info of mignn_locality_order_cols,
 * rows from row_begin = 0 in that order -- the whole graph, or a shard's
 * interior range with its boundary planes moved out) selects the column
 * schedule, with the planes per column taken as the smaller of the info's
 * and the CSR's own run of tiles chaining as z-planes.  Build the plan
 * on the device that runs the layer.  Sum order: a row's entries in CSR order
 * except its one next-tile entry, added last.  stats (nullable, device
 * uint64[4]): tiles over the out-of-tile capacity, rows on the CSR path, rows
 * with a next-tile entry, max out-of-tile entries of a tile. */
size_t mignn_gcn_win_plan_bytes(int64_t row_begin, int64_t row_end, int h);
int mignn_gcn_win_plan(const int32_t* row_ptr, const int32_t* col, const float* ew,
                       int64_t row_begin, int64_t row_end, int h, const int32_t* order_info,
                       void* plan, size_t plan_bytes, unsigned long long* stats, void* stream);
int mignn_gcn_layer_win(const void* plan, const int32_t* row_ptr, const int32_t* col,
                        const float* ew, const float* x, int64_t ldx, int64_t row_begin,
                        int64_t row_end, int h, const float* w, const float* bias,
                        const float* scale, const float* shift, int flags, float* out,
                        int64_t ldo, void* stream);
/* Layer 1 of the GCN stack straight from layer 0's row codes (the codes
 * form, h = 128): codes [rows, ldc >= 8] from mignn_gcn_layer0_codes (D = 3),
 * xcoef = the [h][8] table mignn_gcn_layer0_coords takes for D = 3; the
 * kernel expands every row it reads, x_j = relu(xcoef . (code_j, 1)) with
 * layer 0's fma chain, so out equals mignn_gcn_layer_win over the rows
 * mignn_gcn_layer0_coords would have written, bitwise.  Same plan. */
int mignn_gcn_layer_win_codes(const void* plan, const int32_t* row_ptr, const int32_t* col,
                              const float* ew, const float* codes, int64_t ldc,
                              int64_t row_begin, int64_t row_end, int h, const float* xcoef,
                              const float* w, const float* bias, const float* scale,
                              const float* shift, int flags, float* out, int64_t ldo,
                              void* stream);
/* The GCN aggregation alone by the window kernel (same plan): out_i =
 * sum_e ew_e x_{col e}, fp32 (the SURVEY 8(d) "aggregate kernel alone"). */
int mignn_gcn_aggregate_win(const void* plan, const int32_t* row_ptr, const int32_t* col,
                            const float* ew, const float* x, int64_t ldx, int64_t row_begin,
                            int64_t row_end, int h, float* out, int64_t ldo, void* stream);
/* Fused output head (output_proj, gnn_model.py:90-100, :195) in split-fp16
 * MFMA arithmetic, h in {64, 128, 256}, out_dim 1..8:
 *   out = W4 relu(W3 relu(W2 relu(W1 x + b1) + b2) + b3) + b4
 * with W1, W2: [h, h], W3: [h/2, h], W4: [out_dim, h/2] (torch Linear layout).
 * mignn_mlp_head_prep writes the head image (fp16 hi/lo weight fragments,
 * one scale exponent per matrix, biases in accumulator order) into `img`
 * (mignn_mlp_head_prep_bytes(h) bytes, 16-B aligned, device memory); call
 * it again whenever a weight or bias changes.  Replaces the four nn.Linear
 * launches of FlowGNN.output_proj (eval mode: Dropout is the identity).
 * Error vs fp64 ~1e-6 relative.  x: n rows of h floats, 16-B aligned rows;
 * result row r goes to out row out_rows[r] (NULL: r), i.e. back from the
 * locality order to the caller's node order.  h = 256 (configs[3]/[4]):
 * per-column weight exponents and per-row activation exponents, the three
 * wide transforms chained in registers (agg_gemm.hip head256_kernel). */
size_t mignn_mlp_head_prep_bytes(int h);
int mignn_mlp_head_prep(const float* w1, const float* b1, const float* w2, const float* b2,
                        const float* w3, const float* b3, const float* w4, const float* b4,
                        int h, int out_dim, void* img, size_t img_bytes, void* stream);
int mignn_mlp_head(const float* x, int64_t ldx, int64_t n, int h, const void* img, int out_dim,
                   float* out, int64_t ldo, const int32_t* out_rows, void* stream);

/* input_proj + GCN layer 0 in one pass (gnn_model.py:159, :162-192): both are
 * linear up to the ReLU, so with C_i = sum_{j in row i} ew_j pos_j and
 * s_i = sum ew_j (CSR row incl. the self-loop):
 *   out_i = relu( A pos_i + B C_i + d s_i + e )
 * coef: [h][2*in_dim + 2] floats per output column n = {A[n][:], B[n][:], d[n],
 * e[n]} with A = diag(sc) W_in, B = diag(sc) W W_in, d = sc*(W b_in),
 * e = sc*(b_in + b) + sh (composed by the caller, fp64).  pos: rows of
 * in_dim (1..4) features, stride ldp, in the CSR's node order.  h = 4*2^k. */
int mignn_gcn_layer0_coords(const int32_t* row_ptr, const int32_t* col, const float* ew,
                            const float* pos, int64_t ldp, int in_dim, int64_t row_begin,
                            int64_t row_end, const float* coef, int h, float* out, int64_t ldo,
                            void* stream);
/* Layer 0's row codes instead of its rows: codes_i = (c_i, C_i, s_i, 0...)
 * (8 floats, in_dim 1..3; the values mignn_gcn_layer0_coords expands with
 * its coefficients), rows row_begin..row_end at codes + i * ldc. */
int mignn_gcn_layer0_codes(const int32_t* row_ptr, const int32_t* col, const float* ew,
                           const float* pos, int64_t ldp, int in_dim, int64_t row_begin,
                           int64_t row_end, float* codes, int64_t ldc, void* stream);

/* Fused GIN layer (gnn_model.py:70-75, :166, :184-191), h in {64, 128}:
 *   tmp_i = relu(nn.0( sum_{j in row i} x_j + (1 + eps) x_i ))      (rows rb..re -> tmp[0..])
 *   out_i = epi( nn.2(tmp_i) ) with residual x_i, BN affine, ReLU   (flags as above)
 * tmp: caller scratch of (re - rb) rows, stride ldt. */
int mignn_gin_layer(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                    int64_t row_begin, int64_t row_end, int h, float eps,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    const float* scale, const float* shift, int flags,
                    float* tmp, int64_t ldt, float* out, int64_t ldo, void* stream);

/* Fused H = 256 layers in split-fp16 arithmetic (csrc/agg_gemm.hip): the
 * aggregate (and GIN's hidden layer) never reaches memory -- one kernel per
 * layer instead of aggregate + GEMM (+ GEMM).  Rows [rb, re) of the CSR, out
 * row r at out + r*ldo (as mignn_gcn_layer).  Sum order per row: CSR order,
 * then GIN's (1 + eps) x_i term.
 *   GIN (configs[4], gnn_model.py:70-75):
 *     out_i = epi( relu((sum_j x_j + (1+eps) x_i) W1^T + b1) W2^T + b2 )
 *     img1 = mignn_linear_f16x3_prep(W1 = nn.0.weight, 256, 256);
 *     img2 = mignn_gin_fused_prep(W2 = nn.2.weight): the same image with k
 *     permuted to the first transform's accumulator layout;
 *     b1 = nn.0.bias (always applied, + ReLU); b2 with MIGNN_EPI_BIAS.
 *   GCN at H = 256 (gnn_model.py:63):
 *     out_i = epi( (sum_e ew_e x_{col e}) W^T + bias ),  img = linear_f16x3 image of W.
 * Replaces mignn_sum_aggregate / mignn_gcn_aggregate + mignn_linear_f16x3 (x2). */
size_t mignn_gin_fused_prep_bytes(int h);
int mignn_gin_fused_prep(const float* w2, int h, void* img, size_t img_bytes, void* stream);
int mignn_gin_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* x,
                          int64_t ldx, int64_t row_begin, int64_t row_end, int h, float eps,
                          const void* img1, const float* b1, const void* img2, const float* b2,
                          const float* scale, const float* shift, int flags, float* out,
                          int64_t ldo, void* stream);
/* TransformerConv layer 0 (4 heads, h in {64, 128, 256}) from the node
 * coordinates: with x = pos W_in^T + b_in the layer reduces to 3-vectors --
 * scores (G_h pos_i + g_h) . pos_j * score_scale (the row term q_i . b_in
 * cancels in the softmax), per head P_h = sum_j a_ij pos_j and S_h = sum_j
 * a_ij, out_i = relu?( sum_h (A_h P_h + S_h e_h) + B pos_i + d ).  gt [4][12]
 * = G_h (3x3, row-major) | g_h; table [h][20] per output column = A_0..A_3
 * (3 each) | e_0..e_3 | B (3) | d, with the bias, residual and BN affine
 * folded in by the caller (fp64 composition: FlowGNN._tf_layer0_tables).
 * No [N, h] input, no Q~K transform, no gathered feature row. */
int mignn_transformer_layer0_coords(const int32_t* row_ptr, const int32_t* col, const float* pos,
                                    int64_t ldp, int d, int64_t row_begin, int64_t row_end, int h,
                                    int heads, float score_scale, const float* table,
                                    const float* gt, int relu, float* out, int64_t ldo,
                                    void* stream);
/* GATConv layer 0 collapsed the same way (what FlowGNN runs): scores
 * LeakyReLU(lw[h] . (pos_j, 1) + lw[4 + h] . (pos_i, 1)) (lw as
 * mignn_gat_layer0_fused's), table [h][20] = A_0..A_3 | e_0..e_3 | B | d with
 * A_h = Wcat_h W_in, e_h = Wcat_h b_in and the bias, residual and BN affine
 * folded in.  No MFMA transform, no gathered feature row.  wlog_next /
 * logits_next (both or neither): also the next GAT layer's logits of the
 * written rows, as mignn_gat_layer_next. */
int mignn_gat_layer0_coords(const int32_t* row_ptr, const int32_t* col, const float* pos,
                            int64_t ldp, int d, int64_t row_begin, int64_t row_end, int h,
                            int heads, float negative_slope, const float* table, const float* lw,
                            int relu, float* out, int64_t ldo, const float* wlog_next,
                            float* logits_next, void* stream);
/* GAT layer 0 (4 heads, h in {64, 128}) from the node coordinates
 * (input_proj composed in: with x = pos W_in^T + b_in, the logits are
 * pos . lw[:, :3] + lw[:, 3] for lw = [wlog W_in | wlog b_in] ([8][4], rows
 * as mignn_gat_layer's wlog), head k's weighted sum is W_in P_k + S_k b_in
 * with P_k = sum_j alpha_jk pos_j and S_k = sum_j alpha_jk, and the residual
 * x_i is recomputed): neither input_proj's [N, h] output nor the logits are
 * written, and no feature row is gathered.  pos [N, d] (d <= 3, stride ldp)
 * in the CSR's node order; wcat_img as mignn_gat_layer. */
int mignn_gat_layer0_fused(const int32_t* row_ptr, const int32_t* col, const float* pos,
                           int64_t ldp, int d, int64_t row_begin, int64_t row_end, int h,
                           float negative_slope, const float* w_in, const float* b_in,
                           const float* lw, const void* wcat_img, const float* bias,
                           const float* scale, const float* shift, int flags, float* out,
                           int64_t ldo, void* stream);
/* GIN layer 0 at h = 256 from the node coordinates (input_proj composed
 * into the aggregate: a_i = W_in (sum_j pos_j + (1+eps) pos_i) + (deg_i + 1 +
 * eps) b_in; the residual x_i = W_in pos_i + b_in recomputed in the
 * epilogue): input_proj's [N, 256] output is never written and the layer
 * gathers 12 B per CSR entry instead of a 1-KB row.  pos [N, d] (d <= 3,
 * stride ldp) in the CSR's node order; w_in [256, d], b_in [256] =
 * input_proj; the rest as mignn_gin_layer_fused. */
int mignn_gin_layer0_fused(const int32_t* row_ptr, const int32_t* col, const float* pos,
                           int64_t ldp, int d, int64_t row_begin, int64_t row_end, int h, float eps,
                           const float* w_in, const float* b_in, const void* img1, const float* b1,
                           const void* img2, const float* b2, const float* scale,
                           const float* shift, int flags, float* out, int64_t ldo, void* stream);
int mignn_gcn_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* ew,
                          const float* x, int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                          const void* img, const float* bias, const float* scale,
                          const float* shift, int flags, float* out, int64_t ldo, void* stream);

/* ------------------------------------------------------------------------
 * Mesh -> graph (reference graph_constructor.py).
 * owner [n_faces] / neighbour [n_internal_faces] int64 cell ids as read from
 * the OpenFOAM polyMesh, cell_centers float64 [n_cells, 3].
 *   mode ALL:     build_edge_index (:28-56) + build_graph's validation (:166-172)
 *   mode FIRST_N: build_graph(filter_internal=True, n_internal_cells=n_first)
 *   mode MASK:    build_graph(filter_internal=True) with the mesh internal_mask
 * isolated = 1: nodes in no edge get an appended self-loop (:174-187, :221-226);
 * 0: not (build_edge_index alone).  Same edge order, rules and float64 edge
 * attributes (rounded to float32) as the reference.
 * mignn_mesh_graph_count writes device counts[4] = {n_nodes, face edges,
 * isolated self-loops, total edges E}; the caller reads E, allocates
 * edge_index [2, E] int64, edge_attr [E, 4] and x [n_nodes, ldx] and calls
 * mignn_mesh_graph_emit with the SAME scratch.  x row i = features row of the
 * i-th kept cell (feat_dim float64 values, rounded to float32); x may be NULL.
 * ------------------------------------------------------------------------ */
enum { MIGNN_MESH_ALL = 0, MIGNN_MESH_FIRST_N = 1, MIGNN_MESH_MASK = 2 };
size_t mignn_mesh_graph_scratch_bytes(int64_t n_faces, int64_t n_cells);
int mignn_mesh_graph_count(const int64_t* owner, int64_t n_faces, const int64_t* neighbour,
                           int64_t n_internal_faces, int64_t n_cells, int mode,
                           const uint8_t* mask, int64_t n_first, int isolated, int64_t* counts,
                           void* scratch, size_t scratch_bytes, void* stream);
int mignn_mesh_graph_emit(const int64_t* owner, int64_t n_faces, const int64_t* neighbour,
                          int64_t n_internal_faces, int64_t n_cells, int mode,
                          const double* cell_centers, const double* features, int feat_dim,
                          int64_t num_edges, int64_t* edge_index, float* edge_attr, float* x,
                          int64_t ldx, void* scratch, size_t scratch_bytes, void* stream);
/* compute_edge_attributes (:58-90) of any [2, E] edge list over n cells;
 * an out-of-range index gives zeros (build_graph's check, :196-200) */
int mignn_edge_attributes(const int64_t* edge_index, int64_t num_edges, int64_t n,
                          const double* cell_centers, float* edge_attr, void* stream);
/* get_boundary_mask (:276-296): mask[c] = 1 for owners of the patch's faces */
int mignn_boundary_mask(const int64_t* owner, int64_t n_faces, int64_t start_face,
                        int64_t n_boundary_faces, int64_t n_cells, uint8_t* mask, void* stream);

/* ------------------------------------------------------------------------
 * Output side (reference normalization.py, inference.py).
 * mignn_field_affine: per column c < ncol (<= 30) of x (float32, or float64
 * when x_is_f64), inverse = 1: y = x * std[c] + mean[c]
 * (FieldNormalizer.inverse_transform, normalization.py:110-133); inverse = 0:
 * y = (x - mean[c]) / std[c] (transform, :86-108).  float64 arithmetic
 * without FMA into y (float64, stride ldy) -- NumPy >= 2 promotion; columns in
 * legacy_mask use float32 arithmetic into y32 instead (numpy < 2 value-based
 * casting of float64 scalar scalers on float32 fields).
 * mignn_field_moments: per column mean and population std (fit, :18-84),
 * float64, two passes.
 * mignn_write_openfoam_field: HOST function; writes one field file exactly as
 * save_fields_openfoam_format (inference.py:90-178) does: "%.6e" values, NaN
 * as "nan"; values are host float64 [n, ncomp] (ncomp 1 or 3), row stride ld.
 * ------------------------------------------------------------------------ */
int mignn_field_affine(const void* x, int x_is_f64, int64_t ldx, int64_t n, int ncol,
                       const double* mean, const double* std_, int inverse, int legacy_mask,
                       double* y, float* y32, int64_t ldy, void* stream);
int mignn_field_moments(const void* x, int x_is_f64, int64_t ldx, int64_t n, int ncol,
                        double* mean, double* std_, void* stream);
int mignn_write_openfoam_field(const char* path, const char* field_class, const char* object,
                               const char* location, const char* dimensions,
                               const double* values, int64_t n, int ncomp, int64_t ld);

/* ------------------------------------------------------------------------
 * OpenFOAM ASCII reader (reference openfoam_loader.py), HOST
 * functions with the reference's exact parsing rules and quirks (see
 * csrc/foam_reader.hip).  Each parser takes the file's bytes (buf, len) and
 * host output arrays of capacity cap (rows for points / vector fields);
 * counts come back through the n_* pointers.
 * ------------------------------------------------------------------------ */
/* labelList (owner / neighbour): compat 0 = the reference's read_array
 * (openfoam_loader.py:53-65) including the header-digit quirk; compat 1 = the
 * list as OpenFOAM defines it (count after the FoamFile header). */
int mignn_foam_parse_labels(const char* buf, int64_t len, int compat, int64_t* out, int64_t cap,
                            int64_t* n_out);
int mignn_foam_parse_points(const char* buf, int64_t len, double* out, int64_t cap_rows,
                            int64_t* n_rows);
int mignn_foam_parse_faces(const char* buf, int64_t len, int64_t* offsets, int64_t cap_faces,
                           int64_t* verts, int64_t cap_verts, int64_t* n_faces, int64_t* n_verts);
int mignn_foam_parse_scalar_field(const char* buf, int64_t len, double* out, int64_t cap,
                                  int64_t* n_out);
int mignn_foam_parse_vector_field(const char* buf, int64_t len, double* out, int64_t cap_rows,
                                  int64_t* n_rows);
/* get_cell_centers (openfoam_loader.py:191-227): per cell the mean of the
 * unique vertices of its owner faces then neighbour faces, summed in CPython's
 * set iteration order (emulated) so the float64 results match bit for bit. */
int mignn_foam_cell_centers(const double* points, int64_t n_points, const int64_t* owner,
                            int64_t n_owner, const int64_t* neighbour, int64_t n_neighbour,
                            const int64_t* face_off, const int64_t* face_verts, int64_t n_faces,
                            int64_t n_cells, double* centers);

/* ------------------------------------------------------------------------
 * Training (csrc/train.hip): model.train() forward pieces
 * and the backward of FlowGNN(GCN) + WeightedMSELoss (train.py:158-196).
 * Scratch: mignn_train_scratch_bytes(n, h) bytes for the column reductions;
 * mignn_gemm takes optional scratch for its split reduction partials.
 * ------------------------------------------------------------------------ */
size_t mignn_train_scratch_bytes(int64_t n, int h);
/* C[i, j] = sum_k A(i, k) B(k, j) (+ R[i, j]), A(i, k) = a[i*sai + k*sak],
 * B(k, j) = b[k*sbk + j*sbj] -- f32 MFMA, exact products.  dX = dY.W of a
 * Linear (nn.Linear backward, gnn_model.py:55, 90-100; GCNConv lin :63) and
 * dW = dY^T.X (the reduction over the nodes split over scratch partials and
 * summed in a fixed order when scratch is given and R is NULL). */
int mignn_gemm(const float* a, int64_t sai, int64_t sak, const float* b, int64_t sbk, int64_t sbj,
               int64_t m, int64_t n, int64_t k, const float* r, int64_t ldr, float* c,
               int64_t ldc, void* scratch, size_t scratch_bytes, void* stream);
/* sums[c] = sum_m x[m, c] (bias gradients), double accumulation, deterministic */
int mignn_col_sums(const float* x, int64_t ldx, int64_t n, int h, float* sums, void* scratch,
                   size_t scratch_bytes, void* stream);
/* BatchNorm1d training statistics (gnn_model.py:87, 188 in model.train()):
 * batch mean / 1/sqrt(biased var + eps); running_mean/var (may be NULL)
 * updated with momentum and the unbiased variance; num_batches_tracked += 1.
 * momentum < 0 means BatchNorm1d(momentum=None): cumulative average, factor
 * 1 / num_batches_tracked (after the increment). */
int mignn_bn_train_stats(const float* z, int64_t ldz, int64_t n, int h, float eps, float momentum,
                         float* mean, float* invstd, float* running_mean, float* running_var,
                         int64_t* num_batches_tracked, void* scratch, size_t scratch_bytes,
                         void* stream);
/* y = dropout_p(relu(BN(z))) (gnn_model.py:188-191); gamma NULL: no BN.
 * Dropout mask = counter hash of (seed, m*h + c), regenerated by the backward. */
int mignn_bn_act_forward(const float* z, int64_t ldz, int64_t n, int h, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int relu,
                         float p, uint64_t seed, float* y, int64_t ldy, void* stream);
/* dz (and dgamma, dbeta) from dy of mignn_bn_act_forward's output */
int mignn_bn_act_backward(const float* dout, int64_t ldd, const float* z, int64_t ldz, int64_t n,
                          int h, const float* mean, const float* invstd, const float* gamma,
                          const float* beta, int relu, float p, uint64_t seed, float* dz,
                          int64_t lddz, float* dgamma, float* dbeta, void* scratch,
                          size_t scratch_bytes, void* stream);
/* WeightedMSELoss.forward (normalization.py:176-250): weights[7] = per-column
 * field weights (U, U, U, p, k, epsilon, nut); fieldwise = use_fieldwise;
 * prw = pressure_ref_weight; weights is a HOST array.  loss: device float scalar; stats: device
 * double[1] kept for the backward. */
int mignn_wmse_loss(const float* pred, int64_t ldp, const float* tgt, int64_t ldt, int64_t n,
                    int ncol, const float* weights, float prw, int fieldwise, float* loss,
                    double* stats, void* scratch, size_t scratch_bytes, void* stream);
/* dpred = grad_loss (device scalar) * d loss / d pred */
int mignn_wmse_loss_backward(const float* pred, int64_t ldp, const float* tgt, int64_t ldt,
                             int64_t n, int ncol, const float* weights, float prw, int fieldwise,
                             const double* stats, const float* grad_loss, float* dpred,
                             int64_t ldd, void* stream);
/* the dropout keep-scale mask of (p, seed) as an [n, h] array (tests) */
int mignn_dropout_mask(int64_t n, int h, float p, uint64_t seed, float* mask, void* stream);

/* GATConv(H, H, heads, concat=False, dropout=p) training (gnn_model.py:65-68, :168;
 * csrc/gat_train.hip).  logits [n, 2*heads] = x . [v_src | v_dst]^T (ld 2*heads).
 * Forward: y[i, k*h + c] = sum_{j in row i} drop(alpha_jik) x[j, c], alpha = PyG
 * softmax of LeakyReLU(a_src[j,k] + a_dst[i,k]); attention dropout keyed on
 * (seed, i, j, k).  Backward, given dy [n, heads*h]: dlogits [n, 2*heads] and
 * dx = dz + sum_{i,k} drop alpha_jik dy[i, k] (dz may be NULL).  stats = caller
 * buffer of n*3*heads floats: the forward writes the softmax state into it
 * (nullable there), the backward reads it (y = the forward's output).   Row/col CSRs: mode
 * MIGNN_CSR_ONE_SELF_LOOP and its MIGNN_CSR_TRANSPOSE. */
int mignn_gat_train_forward(const int32_t* row_ptr, const int32_t* col, const float* logits,
                            const float* x, int64_t ldx, int64_t n, int h, int heads,
                            float negative_slope, float p, uint64_t seed, float* y, int64_t ldy,
                            float* stats, void* stream);
int mignn_gat_train_backward(const int32_t* row_ptr, const int32_t* col, const int32_t* rowt_ptr,
                             const int32_t* colt, const float* logits, const float* x,
                             int64_t ldx, const float* dy, int64_t lddy, const float* y,
                             int64_t ldy, const float* dz, int64_t lddz, int64_t n, int h,
                             int heads, float negative_slope,
                             float p, uint64_t seed, float* stats, float* dlogits, float* dx,
                             int64_t lddx, void* stream);

/* ------------------------------------------------------------------------
 * Multi-GPU halo helpers and synthetic inputs.
 * ------------------------------------------------------------------------ */
/* dst[r, :] = src[idx[r], :] for r < n (halo pack / unpack by index list) */
int mignn_rows_gather(const float* src, int64_t lds, const int32_t* idx, int64_t n, int h,
                      float* dst, int64_t ldd, void* stream);
/* A node-range shard's marks in one pass over its in-edges edge_index [2, E]
 * (global ids; mignn.dist.RangeLayout): ghost_mark[src] = 1 (int32 [N],
 * zeroed by the caller) for every source outside [lo, hi), boundary_mark[dst
 * - lo] = 1 (int8 [hi - lo]) for its destination, bad[0] = 1 if a
 * destination lies outside [lo, hi), bad[1] = 1 if a source lies outside
 * [0, N) (int32 [2], zeroed; such edges mark nothing). */
int mignn_range_mark(const int64_t* edge_index, int64_t E, int64_t lo, int64_t hi, int64_t N,
                     int32_t* ghost_mark, int8_t* boundary_mark, int32_t* bad, void* stream);
/* A node-range shard's local edge list (mignn.dist.RangeLayout; the caller
 * has validated the ids): edge_index [2, E] global ids, destinations in
 * [lo, hi).  out [2, E]: a source in [lo, hi) -> inv[src - lo], any other
 * (a ghost) -> n_own + ghost_rank[src] - 1 (ghost_rank: inclusive prefix sum
 * of the ghost marks over the global ids); a destination -> inv[dst - lo]. */
int mignn_range_relabel(const int64_t* edge_index, int64_t E, int64_t lo, int64_t hi,
                        const int64_t* inv, const int64_t* ghost_rank, int64_t n_own,
                        int64_t* out, void* stream);
/* The shard's local order: a stable partition of base [n_own] (a permutation
 * of the owned offsets) by boundary[offset] (0/1 bytes) -- interior rows
 * first, then boundary rows, each in base order.  ci [n_own] = the inclusive
 * prefix count of interior rows along base, n_int = their total.
 * perm[local position] = owned offset, inv = its inverse. */
int mignn_range_partition(const int64_t* base, const uint8_t* boundary, const int32_t* ci,
                          int64_t n_own, int64_t n_int, int64_t* perm, int64_t* inv,
                          void* stream);
/* Periodic nx*ny*nz hex grid, k-slab [z_begin, z_begin+z_count): writes
 * edge_index [2, 6*n] (src = neighbour, dst = node; global ids) and
 * x [n, 3] = cell centres in [0,1]^3.  n = nx*ny*z_count. */
int mignn_grid_graph(int nx, int ny, int nz, int z_begin, int z_count, int64_t* edge_index,
                     float* x, void* stream);

/* TransformerConv(H, H, heads, concat=False, dropout=p) training, edge_attr=None
 * (gnn_model.py:77-80, :170; csrc/transformer_train.hip).  qkv [n, 3*heads*h] =
 * [Q | K | V] (head k at column k*h of each block), verbatim CSR.
 * Forward: out_i = x_i + (1/heads) sum_k sum_j drop(alpha_jik) V_j[k],
 * alpha = softmax_j(score_scale <Q_i[k], K_j[k]>) (+1e-16), attention dropout
 * keyed on (seed, i, j, k).  Backward, given dz [n, h] (dout = dz): writes the
 * dQ | dK | dV blocks of dqkv.  The forward optionally writes the per-head
 * aggregates yh [n, heads*h] and the softmax state into stats (n*3*heads
 * floats); the backward needs both. */
int mignn_transformer_train_forward(const int32_t* row_ptr, const int32_t* col, const float* qkv,
                                    int64_t ldq, const float* x, int64_t ldx, int64_t n, int h,
                                    int heads, float score_scale, float p, uint64_t seed,
                                    float* out, int64_t ldo, float* yh, int64_t ldyh,
                                    float* stats, void* stream);
int mignn_transformer_train_backward(const int32_t* row_ptr, const int32_t* col,
                                     const int32_t* rowt_ptr, const int32_t* colt,
                                     const float* qkv, int64_t ldq, const float* dz, int64_t lddz,
                                     const float* yh, int64_t ldyh, int64_t n, int h, int heads, float score_scale, float p,
                                     uint64_t seed, float* stats, float* dqkv, int64_t ldd,
                                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MIGNN_H */
