// Neighbour aggregation over the destination-major CSR (graph_build.hip).
//
// Layout: a "row group" of LPR lanes owns one destination row; lane c of the
// group owns float4 chunks c, c+LPR, ... (CPL chunks) of the H-wide feature
// row, so every gathered neighbour row is read as LPR*16 contiguous bytes
// (one 512-B burst per half-wave at H = 128).  64/LPR rows per wavefront.
// Edges are visited in CSR order == edge_index order (stable CSR), which is
// also the order PyG's scatter-add visits them on the CPU.
//
//  gcn_aggregate_kernel   GCNConv message/aggregate with gcn_norm weights
//  sum_aggregate_kernel   GINConv: sum_j x_j + (1+eps) x_i
//  gat_aggregate_kernel   GATConv: LeakyReLU logits, per-row max / sum-exp
//                         (+1e-16), alpha-weighted sums of x_j for every head
//  transformer_aggregate  TransformerConv: online softmax of (q~_i . x_j + c_i)
//                         * 1/sqrt(C) with alpha-weighted sums of x_j per head
// The per-head transforms are applied afterwards by one MFMA GEMM
// (`mignn_linear`) with the weights re-associated on the host side
// (see mignn/gnn_model.py), so the [N, heads*C] projected tensors of the
// reference are never materialised.
#include "common.hpp"

namespace mignn {
namespace {

constexpr float kSoftmaxEps = 1e-16f;  // PyG utils.softmax

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int LPR>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

struct RowCursor {
    int64_t row;
    int c;  // lane index inside the row group
};

template <int LPR>
__device__ __forceinline__ RowCursor row_of(int64_t row_begin) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    return {row_begin + wave * (64 / LPR) + lane / LPR, lane % LPR};
}

template <int LPR>
__device__ __forceinline__ int64_t row_stride() {
    return ((int64_t)gridDim.x * blockDim.x >> 6) * (64 / LPR);
}

// ---------------------------------------------------------------- GCN / GIN
template <int LPR, int CPL, bool GCN>
__global__ __launch_bounds__(256) void weighted_sum_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ dinv, const float* __restrict__ x, int64_t ldx, float self_scale,
    int64_t row_begin, int64_t row_end, int h4, float* __restrict__ out, int64_t ldo) {
    RowCursor rc = row_of<LPR>(row_begin);
    const int64_t stride = row_stride<LPR>();
    for (int64_t row = rc.row; row < row_end; row += stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        const float di = GCN ? dinv[row] : 1.f;
        float4 acc[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        int e = beg;
        for (; e + 4 <= end; e += 4) {
            int j[4];
            float w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) j[u] = col[e + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) w[u] = GCN ? dinv[j[u]] * di : 1.f;
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int q = 0; q < CPL; ++q) {
                    const int ch = rc.c + q * LPR;
                    if (ch < h4) acc[q] = fma4(w[u], ld4(x + (int64_t)j[u] * ldx + 4 * ch), acc[q]);
                }
        }
        for (; e < end; ++e) {
            const int j = col[e];
            const float w = GCN ? dinv[j] * di : 1.f;
#pragma unroll
            for (int q = 0; q < CPL; ++q) {
                const int ch = rc.c + q * LPR;
                if (ch < h4) acc[q] = fma4(w, ld4(x + (int64_t)j * ldx + 4 * ch), acc[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            const int ch = rc.c + q * LPR;
            if (ch >= h4) continue;
            float4 v = acc[q];
            if (!GCN) {  // GINConv: out + (1 + eps) * x_i
                const float4 xi = ld4(x + row * ldx + 4 * ch);
                v.x = v.x + self_scale * xi.x;
                v.y = v.y + self_scale * xi.y;
                v.z = v.z + self_scale * xi.z;
                v.w = v.w + self_scale * xi.w;
            }
            st4(out + row * ldo + 4 * ch, v);
        }
    }
}

// ---------------------------------------------------------------- GAT
template <int LPR, int CPL, int HEADS>
__global__ __launch_bounds__(256) void gat_aggregate_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx, int64_t row_begin,
    int64_t row_end, int h, float slope, float* __restrict__ out, int64_t ldo) {
    const int h4 = h >> 2;
    RowCursor rc = row_of<LPR>(row_begin);
    const int64_t stride = row_stride<LPR>();
    for (int64_t row = rc.row; row < row_end; row += stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        float ad[HEADS], mx[HEADS], sm[HEADS];
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) {
            ad[hd] = logits[row * (2 * HEADS) + HEADS + hd];
            mx[hd] = -INFINITY;
            sm[hd] = 0.f;
        }
        // pass 1: per-head max of LeakyReLU(a_src[j] + a_dst[i])
        for (int e = beg + rc.c; e < end; e += LPR) {
            const int j = col[e];
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                float v = logits[(int64_t)j * (2 * HEADS) + hd] + ad[hd];
                v = v > 0.f ? v : v * slope;
                mx[hd] = fmaxf(mx[hd], v);
            }
        }
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) mx[hd] = group_max<LPR>(mx[hd]);
        // pass 2: per-head sum of exp(v - max)
        for (int e = beg + rc.c; e < end; e += LPR) {
            const int j = col[e];
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                float v = logits[(int64_t)j * (2 * HEADS) + hd] + ad[hd];
                v = v > 0.f ? v : v * slope;
                sm[hd] += expf(v - mx[hd]);
            }
        }
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) sm[hd] = group_sum<LPR>(sm[hd]) + kSoftmaxEps;
        // pass 3: alpha-weighted neighbour sums, all heads from one gather
        float4 acc[HEADS][CPL];
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd)
#pragma unroll
            for (int q = 0; q < CPL; ++q) acc[hd][q] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int e = beg; e < end; ++e) {
            const int j = col[e];
            float4 xj[CPL];
#pragma unroll
            for (int q = 0; q < CPL; ++q) {
                const int ch = rc.c + q * LPR;
                xj[q] = ch < h4 ? ld4(x + (int64_t)j * ldx + 4 * ch) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                float v = logits[(int64_t)j * (2 * HEADS) + hd] + ad[hd];
                v = v > 0.f ? v : v * slope;
                const float alpha = expf(v - mx[hd]) / sm[hd];
#pragma unroll
                for (int q = 0; q < CPL; ++q) acc[hd][q] = fma4(alpha, xj[q], acc[hd][q]);
            }
        }
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd)
#pragma unroll
            for (int q = 0; q < CPL; ++q) {
                const int ch = rc.c + q * LPR;
                if (ch < h4) st4(out + row * ldo + hd * h + 4 * ch, acc[hd][q]);
            }
    }
}

// ---------------------------------------------------------------- Transformer
template <int LPR, int CPL, int HEADS>
__global__ __launch_bounds__(256) void transformer_aggregate_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ qt, int64_t ldq, const float* __restrict__ x, int64_t ldx,
    int64_t row_begin, int64_t row_end, int h, float scale, float* __restrict__ out, int64_t ldo) {
    const int h4 = h >> 2;
    RowCursor rc = row_of<LPR>(row_begin);
    const int64_t stride = row_stride<LPR>();
    for (int64_t row = rc.row; row < row_end; row += stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        float4 q[HEADS][CPL];
        float cq[HEADS], m[HEADS], l[HEADS];
        float4 acc[HEADS][CPL];
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) {
            cq[hd] = qt[row * ldq + HEADS * h + hd];
            m[hd] = -INFINITY;
            l[hd] = 0.f;
#pragma unroll
            for (int qq = 0; qq < CPL; ++qq) {
                const int ch = rc.c + qq * LPR;
                q[hd][qq] = ch < h4 ? ld4(qt + row * ldq + hd * h + 4 * ch)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
                acc[hd][qq] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        for (int e = beg; e < end; ++e) {
            const int j = col[e];
            float4 xj[CPL];
#pragma unroll
            for (int qq = 0; qq < CPL; ++qq) {
                const int ch = rc.c + qq * LPR;
                xj[qq] = ch < h4 ? ld4(x + (int64_t)j * ldx + 4 * ch) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                float d = 0.f;
#pragma unroll
                for (int qq = 0; qq < CPL; ++qq) {
                    d = fmaf(q[hd][qq].x, xj[qq].x, d);
                    d = fmaf(q[hd][qq].y, xj[qq].y, d);
                    d = fmaf(q[hd][qq].z, xj[qq].z, d);
                    d = fmaf(q[hd][qq].w, xj[qq].w, d);
                }
                d = group_sum<LPR>(d);
                const float s = (d + cq[hd]) * scale;
                const float mn = fmaxf(m[hd], s);
                const float corr = expf(m[hd] - mn);  // 0 on the first edge (m = -inf)
                const float p = expf(s - mn);
                l[hd] = l[hd] * corr + p;
#pragma unroll
                for (int qq = 0; qq < CPL; ++qq) {
                    float4 a = acc[hd][qq];
                    a.x = fmaf(p, xj[qq].x, a.x * corr);
                    a.y = fmaf(p, xj[qq].y, a.y * corr);
                    a.z = fmaf(p, xj[qq].z, a.z * corr);
                    a.w = fmaf(p, xj[qq].w, a.w * corr);
                    acc[hd][qq] = a;
                }
                m[hd] = mn;
            }
        }
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) {
            const float inv = 1.f / (l[hd] + kSoftmaxEps);
#pragma unroll
            for (int qq = 0; qq < CPL; ++qq) {
                const int ch = rc.c + qq * LPR;
                if (ch < h4) {
                    float4 a = acc[hd][qq];
                    a.x *= inv; a.y *= inv; a.z *= inv; a.w *= inv;
                    st4(out + row * ldo + hd * h + 4 * ch, a);
                }
            }
            if (rc.c == 0) out[row * ldo + HEADS * h + hd] = l[hd] * inv;  // sum_j alpha
        }
    }
}

inline int lanes_per_row(int h4) {
    int lpr = 1;
    while (lpr < h4 && lpr < 64) lpr <<= 1;
    return lpr;
}

inline unsigned agg_grid(int64_t rows, int lpr) {
    const int64_t waves = (rows + (64 / lpr) - 1) / (64 / lpr);
    return grid_for(waves * 64, 256, 8192);
}

}  // namespace
}  // namespace mignn

using namespace mignn;

// Dispatch on (LPR, CPL): LPR = pow2 >= h/4 capped at 64; CPL = ceil(h/4 / 64).
#define MIGNN_DISPATCH_LPR(h4, BODY)                                      \
    do {                                                                  \
        const int lpr_ = lanes_per_row(h4);                               \
        const int cpl_ = (h4 + 63) / 64;                                  \
        if (cpl_ == 1) {                                                  \
            switch (lpr_) {                                               \
                case 1: { constexpr int LPR = 1, CPL = 1; BODY; } break;  \
                case 2: { constexpr int LPR = 2, CPL = 1; BODY; } break;  \
                case 4: { constexpr int LPR = 4, CPL = 1; BODY; } break;  \
                case 8: { constexpr int LPR = 8, CPL = 1; BODY; } break;  \
                case 16: { constexpr int LPR = 16, CPL = 1; BODY; } break;\
                case 32: { constexpr int LPR = 32, CPL = 1; BODY; } break;\
                default: { constexpr int LPR = 64, CPL = 1; BODY; } break;\
            }                                                             \
        } else if (cpl_ == 2) {                                           \
            constexpr int LPR = 64, CPL = 2; BODY;                        \
        } else if (cpl_ <= 4) {                                           \
            constexpr int LPR = 64, CPL = 4; BODY;                        \
        } else {                                                          \
            set_error("aggregate: h=%d > 1024 unsupported", 4 * h4);      \
            return MIGNN_ERR_UNSUPPORTED;                                 \
        }                                                                 \
    } while (0)

#define MIGNN_DISPATCH_HEADS(heads, BODY)                                 \
    do {                                                                  \
        switch (heads) {                                                  \
            case 1: { constexpr int HEADS = 1; BODY; } break;             \
            case 2: { constexpr int HEADS = 2; BODY; } break;             \
            case 4: { constexpr int HEADS = 4; BODY; } break;             \
            case 8: { constexpr int HEADS = 8; BODY; } break;             \
            default:                                                      \
                set_error("heads=%d unsupported (1,2,4,8)", heads);       \
                return MIGNN_ERR_UNSUPPORTED;                             \
        }                                                                 \
    } while (0)

static int check_common(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                        int64_t rb, int64_t re, int h, const float* out, int64_t ldo) {
    MIGNN_REQUIRE(row_ptr && col && x && out, "aggregate: null pointer");
    MIGNN_REQUIRE(h > 0 && h % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0,
                  "aggregate: h=%d / strides must be multiples of 4", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out), "aggregate: unaligned x/out");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "aggregate: bad row range");
    return MIGNN_OK;
}

extern "C" int mignn_gcn_aggregate(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                                   const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                   float* out, int64_t ldo, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    MIGNN_REQUIRE(dinv, "gcn_aggregate: null dinv");
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_LPR(h4, (weighted_sum_kernel<LPR, CPL, true><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, as_stream(stream)>>>( row_ptr, col, dinv, x, ldx, 1.f,
                                               rb, re, h4, out, ldo)));
    return launch_status("gcn_aggregate");
}

extern "C" int mignn_sum_aggregate(const int32_t* row_ptr, const int32_t* col, const float* x,
                                   int64_t ldx, float self_scale, int64_t rb, int64_t re, int h,
                                   float* out, int64_t ldo, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_LPR(h4, (weighted_sum_kernel<LPR, CPL, false><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, as_stream(stream)>>>( row_ptr, col, nullptr, x, ldx,
                                               self_scale, rb, re, h4, out, ldo)));
    return launch_status("sum_aggregate");
}

extern "C" int mignn_gat_aggregate(const int32_t* row_ptr, const int32_t* col,
                                   const float* logits, const float* x, int64_t ldx, int64_t rb,
                                   int64_t re, int h, int heads, float slope, float* out,
                                   int64_t ldo, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    MIGNN_REQUIRE(logits, "gat_aggregate: null logits");
    MIGNN_REQUIRE(ldo >= (int64_t)heads * h, "gat_aggregate: ldo < heads*h");
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_HEADS(heads, MIGNN_DISPATCH_LPR(h4, (gat_aggregate_kernel<LPR, CPL, HEADS><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, as_stream(stream)>>>( row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo))));
    return launch_status("gat_aggregate");
}

extern "C" int mignn_transformer_aggregate(const int32_t* row_ptr, const int32_t* col,
                                           const float* qt, int64_t ldq, const float* x,
                                           int64_t ldx, int64_t rb, int64_t re, int h, int heads,
                                           float score_scale, float* out, int64_t ldo,
                                           void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    MIGNN_REQUIRE(qt && aligned16(qt) && ldq % 4 == 0 && ldq >= (int64_t)heads * h + heads,
                  "transformer_aggregate: bad qt");
    MIGNN_REQUIRE(ldo >= (int64_t)heads * h + heads, "transformer_aggregate: ldo too small");
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_HEADS(heads, MIGNN_DISPATCH_LPR(h4, (transformer_aggregate_kernel<LPR, CPL, HEADS><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, as_stream(stream)>>>( row_ptr, col, qt, ldq, x, ldx, rb, re, h, score_scale,
        out, ldo))));
    return launch_status("transformer_aggregate");
}
