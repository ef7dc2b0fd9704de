// GATConv and TransformerConv eval layers as single C-ABI calls (SURVEY.md
// §8b: mignn_gat_layer / mignn_transformer_layer), each the composition of
// its kernels on one stream with caller-owned scratch -- what FlowGNN._layer
// runs for these layer types (gnn_model.py:65-68, :77-80, :166-192):
//
//   GAT:          logits = x . wlog^T                  (mignn_linear, [n_x, 2 heads];
//                                                       skipped if the caller gives them)
//                 agg    = softmax-weighted sums        (mignn_gat_aggregate, [rows, heads h])
//                 out    = relu(BN(x + agg . wcat^T + b))
//   Transformer:  qt     = x . wqk^T + bqk               ([rows, heads h])
//                 agg    = softmax-weighted sums | alpha sums (mignn_transformer_aggregate)
//                 out    = relu(BN(x + [agg | x] . wout^T + bout))
//
// The transforms run in split-fp16 MFMA arithmetic when the caller passes the
// weight's image (mignn_linear_f16x3_prep), else in exact fp32
// (mignn_linear).  The re-associated weights (wlog = W_k^T att per head, wcat
// = head-mean blocks of W; wqk = W_k^T W_q per head, bqk = W_k^T b_q, wout =
// [W_v / heads | b_v / heads | W_skip]) are built by the host layer once per
// weight version (mignn/gnn_model.py _gat_weights / _tf_weights).  The score's
// per-head constant q_i . b_k (mignn_transformer_aggregate's c) is not formed:
// it shifts every score of a row's head alike and the softmax cancels it, so
// the Q~K transform is heads*h columns wide (four whole 256-column GEMM tiles
// at h = 256 instead of four and a 4-column fifth).
#include "common.hpp"

namespace {

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

#ifdef MIGNN_DIAG
bool g_gat_fused = true;     // mignn_diag_set_gat_fused (A/B timing against the launch sequence)
#else
constexpr bool g_gat_fused = true;
#endif

// the transform of either arithmetic: img != NULL -> split fp16, else fp32 w
int transform(const float* a, int64_t lda, int64_t m, int k1, const float* a2, int64_t lda2,
              int k2, const float* w, const void* img, int n, const float* bias,
              const float* residual, int64_t ldr, const float* scale, const float* shift,
              int flags, float* c, int64_t ldc, void* stream) {
    if (img != nullptr)
        return mignn_linear_f16x3(a, lda, m, k1, a2, lda2, k2, img, n, bias, residual, ldr, scale,
                                  shift, flags, c, ldc, stream);
    return mignn_linear(a, lda, m, k1, a2, lda2, k2, w, n, bias, residual, ldr, scale, shift,
                        flags, c, ldc, stream);
}

}  // namespace

using namespace mignn;

extern "C" size_t mignn_gat_layer_scratch_bytes(int64_t n_x, int64_t rows, int h, int heads) {
    if (n_x < 0 || rows < 0 || h <= 0 || heads <= 0) return 0;
    return align256(static_cast<size_t>(n_x) * 2 * heads * 4) +
           align256(static_cast<size_t>(rows) * heads * h * 4);
}

static int gat_layer_impl(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                          int64_t n_x, int64_t row_begin, int64_t row_end, int h, int heads,
                          float negative_slope, const float* wlog, const float* logits,
                          int64_t ldl, const float* wcat, const void* wcat_img, const float* bias,
                          const float* scale, const float* shift, int flags, void* scratch,
                          size_t scratch_bytes, float* out, int64_t ldo, void* stream,
                          const float* wlog_next, float* logits_next) {
    MIGNN_REQUIRE((flags & ~(MIGNN_EPI_MASK | MIGNN_GAT_LAUNCHES)) == 0,
                  "gat_layer: unknown flags 0x%x", flags);
    const bool launches = (flags & MIGNN_GAT_LAUNCHES) != 0 || !g_gat_fused;
    flags &= MIGNN_EPI_MASK;
    MIGNN_REQUIRE(row_ptr && col && x && out && (logits || wlog) && (wcat || wcat_img),
                  "gat_layer: null pointer");
    MIGNN_REQUIRE(row_begin >= 0 && row_end >= row_begin && n_x >= row_end,
                  "gat_layer: bad row range");
    MIGNN_REQUIRE(logits == nullptr || ldl >= 2 * heads, "gat_layer: ldl < 2*heads");
    const int64_t rows = row_end - row_begin;
    if (rows == 0) return MIGNN_OK;
    const size_t need = mignn_gat_layer_scratch_bytes(logits ? 0 : n_x, rows, h, heads);
    MIGNN_REQUIRE(scratch && aligned16(scratch) && scratch_bytes >= need,
                  "gat_layer: scratch %zu < required %zu", scratch_bytes, need);
    char* base = static_cast<char*>(scratch);
    const float* lg = logits;
    int64_t ld_lg = ldl;
    if (lg == nullptr) {   // logits of every row the CSR references
        float* l = reinterpret_cast<float*>(base);
        base += align256(static_cast<size_t>(n_x) * 2 * heads * 4);
        if (int rc = mignn_linear(x, ldx, n_x, h, nullptr, 0, 0, wlog, 2 * heads, nullptr, nullptr,
                                  0, nullptr, nullptr, 0, l, 2 * heads, stream))
            return rc;
        lg = l;
        ld_lg = 2 * heads;
    }
    MIGNN_REQUIRE(ld_lg == 2 * heads, "gat_layer: logits must be [n, 2*heads] contiguous");
    // split-fp16 transform, 4 heads, h in {64, 128}: aggregation and head-mean
    // transform in one kernel (agg_gemm.hip) -- the [rows, heads h] aggregate
    // never reaches memory
    if (wcat_img != nullptr && heads == 4 && (h == 64 || h == 128) && !launches)
        return gat_layer_fused(row_ptr, col, lg, x, ldx, row_begin, row_end, h, negative_slope,
                               wcat_img, bias, scale, shift, flags, out, ldo, stream, wlog_next,
                               logits_next);
    float* agg = reinterpret_cast<float*>(base);
    const int64_t lda = static_cast<int64_t>(heads) * h;
    // the aggregation writes row r at agg + r * lda for r in [row_begin, row_end)
    if (int rc = mignn_gat_aggregate(row_ptr, col, lg, x, ldx, row_begin, row_end, h, heads,
                                     negative_slope, agg - row_begin * lda, lda, stream))
        return rc;
    if (int rc = transform(agg, lda, rows, heads * h, nullptr, 0, 0, wcat, wcat_img, h, bias,
                           x + row_begin * ldx, ldx, scale, shift, flags, out + row_begin * ldo,
                           ldo, stream))
        return rc;
    if (logits_next == nullptr) return MIGNN_OK;
    // the next layer's logits of the rows just written
    return mignn_linear(out + row_begin * ldo, ldo, rows, h, nullptr, 0, 0, wlog_next, 2 * heads,
                        nullptr, nullptr, 0, nullptr, nullptr, 0, logits_next + row_begin * 2 * heads,
                        2 * heads, stream);
}

extern "C" int mignn_gat_layer(const int32_t* row_ptr, const int32_t* col, const float* x,
                               int64_t ldx, int64_t n_x, int64_t row_begin, int64_t row_end, int h,
                               int heads, float negative_slope, const float* wlog,
                               const float* logits, int64_t ldl, const float* wcat,
                               const void* wcat_img, const float* bias, const float* scale,
                               const float* shift, int flags, void* scratch, size_t scratch_bytes,
                               float* out, int64_t ldo, void* stream) {
    return gat_layer_impl(row_ptr, col, x, ldx, n_x, row_begin, row_end, h, heads, negative_slope,
                          wlog, logits, ldl, wcat, wcat_img, bias, scale, shift, flags, scratch,
                          scratch_bytes, out, ldo, stream, nullptr, nullptr);
}

extern "C" int mignn_gat_layer_next(const int32_t* row_ptr, const int32_t* col, const float* x,
                                    int64_t ldx, int64_t n_x, int64_t row_begin, int64_t row_end,
                                    int h, int heads, float negative_slope, const float* wlog,
                                    const float* logits, int64_t ldl, const float* wcat,
                                    const void* wcat_img, const float* bias, const float* scale,
                                    const float* shift, int flags, void* scratch,
                                    size_t scratch_bytes, float* out, int64_t ldo,
                                    const float* wlog_next, float* logits_next, void* stream) {
    MIGNN_REQUIRE(wlog_next && logits_next && aligned16(logits_next),
                  "gat_layer_next: wlog_next / 16-B aligned logits_next");
    return gat_layer_impl(row_ptr, col, x, ldx, n_x, row_begin, row_end, h, heads, negative_slope,
                          wlog, logits, ldl, wcat, wcat_img, bias, scale, shift, flags, scratch,
                          scratch_bytes, out, ldo, stream, wlog_next, logits_next);
}

extern "C" size_t mignn_transformer_layer_scratch_bytes(int64_t rows, int h, int heads) {
    if (rows < 0 || h <= 0 || heads <= 0) return 0;
    // rows of qt / agg: heads h sums | heads alpha sums, padded to 16 B
    const size_t k1 = static_cast<size_t>(heads) * h + heads;
    const size_t ldq = (k1 + 3) / 4 * 4;
    return 2 * align256(static_cast<size_t>(rows) * ldq * 4);
}

extern "C" int mignn_transformer_layer(const int32_t* row_ptr, const int32_t* col, const float* x,
                                       int64_t ldx, int64_t row_begin, int64_t row_end, int h,
                                       int heads, float score_scale, const float* wqk,
                                       const void* wqk_img, const float* bqk, const float* wout,
                                       const void* wout_img, const float* bout,
                                       const float* scale, const float* shift, int flags,
                                       void* scratch, size_t scratch_bytes, float* out,
                                       int64_t ldo, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "transformer_layer: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(row_ptr && col && x && out && bqk && (wqk || wqk_img) && (wout || wout_img),
                  "transformer_layer: null pointer");
    MIGNN_REQUIRE(row_begin >= 0 && row_end >= row_begin, "transformer_layer: bad row range");
    const int64_t rows = row_end - row_begin;
    if (rows == 0) return MIGNN_OK;
    const size_t need = mignn_transformer_layer_scratch_bytes(rows, h, heads);
    MIGNN_REQUIRE(scratch && aligned16(scratch) && scratch_bytes >= need,
                  "transformer_layer: scratch %zu < required %zu", scratch_bytes, need);
    const int k1 = heads * h + heads;   // agg: [heads h sums | heads alpha sums]
    // rows of qt / agg padded to 16 B (the aggregation loads qt rows as float4)
    const int64_t ldq = (k1 + 3) / 4 * 4;
    MIGNN_REQUIRE(static_cast<size_t>(rows) * ldq * 4 <= need / 2, "transformer_layer: layout");
    float* qt = static_cast<float*>(scratch);
    float* agg = reinterpret_cast<float*>(static_cast<char*>(scratch) + need / 2);
    if (int rc = transform(x + row_begin * ldx, ldx, rows, h, nullptr, 0, 0, wqk, wqk_img,
                           heads * h, bqk, nullptr, 0, nullptr, nullptr, MIGNN_EPI_BIAS, qt, ldq,
                           stream))
        return rc;
    if (int rc = transformer_aggregate_rows(row_ptr, col, qt - row_begin * ldq, ldq, x, ldx,
                                            row_begin, row_end, h, heads, score_scale,
                                            agg - row_begin * ldq, ldq, false, stream))
        return rc;
    // [agg | x] . wout^T + bout, residual x, BN, ReLU (flags)
    return transform(agg, ldq, rows, k1, x + row_begin * ldx, ldx, h, wout, wout_img, h, bout,
                     x + row_begin * ldx, ldx, scale, shift, flags, out + row_begin * ldo, ldo,
                     stream);
}

extern "C" size_t mignn_transformer_fused_prep_bytes(int h, int heads) {
    return h == 256 && heads == 4 ? tf_fused_prep_bytes() : 0;
}

extern "C" int mignn_transformer_fused_prep(const float* wout, int h, int heads, void* img,
                                            size_t img_bytes, void* stream) {
    MIGNN_REQUIRE(wout && img, "transformer_fused_prep: null pointer");
    MIGNN_REQUIRE(h == 256 && heads == 4, "transformer_fused_prep: h = 256, heads = 4 only");
    MIGNN_REQUIRE(img_bytes >= tf_fused_prep_bytes(), "transformer_fused_prep: image too small");
    MIGNN_REQUIRE(aligned16(img), "transformer_fused_prep: image not 16-B aligned");
    return tf_fused_prep(wout, img, stream);
}

extern "C" int mignn_transformer_layer_fused(
    const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx, int64_t row_begin,
    int64_t row_end, int h, int heads, float score_scale, const void* wqk_img, const float* bqk,
    const void* wout_fimg, const float* bout, const float* scale, const float* shift, int flags,
    void* scratch, size_t scratch_bytes, float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "transformer_layer_fused: unknown flags 0x%x",
                  flags);
    MIGNN_REQUIRE(row_ptr && col && x && out && bqk && wqk_img && wout_fimg,
                  "transformer_layer_fused: null pointer");
    MIGNN_REQUIRE(h == 256 && heads == 4, "transformer_layer_fused: h = 256, heads = 4 only");
    MIGNN_REQUIRE(row_begin >= 0 && row_end >= row_begin, "transformer_layer_fused: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "transformer_layer_fused: affine");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bout, "transformer_layer_fused: bias");
    const int64_t rows = row_end - row_begin;
    if (rows == 0) return MIGNN_OK;
    const size_t need = mignn_transformer_layer_scratch_bytes(rows, h, heads);
    MIGNN_REQUIRE(scratch && aligned16(scratch) && scratch_bytes >= need,
                  "transformer_layer_fused: scratch %zu < required %zu", scratch_bytes, need);
    const int64_t ldq = static_cast<int64_t>(heads) * h;   // qt rows: 4 x 256 floats
    float* qt = static_cast<float*>(scratch);
    if (int rc = mignn_linear_f16x3(x + row_begin * ldx, ldx, rows, h, nullptr, 0, 0, wqk_img,
                                    heads * h, bqk, nullptr, 0, nullptr, nullptr, MIGNN_EPI_BIAS,
                                    qt, ldq, stream))
        return rc;
    return tf_fused(row_ptr, col, qt - row_begin * ldq, ldq, x, ldx, row_begin, row_end,
                    score_scale, wout_fimg, bout, scale, shift, flags, out, ldo, stream);
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_set_gat_fused(int on) {
    g_gat_fused = on != 0;
    return MIGNN_OK;
}
#endif
