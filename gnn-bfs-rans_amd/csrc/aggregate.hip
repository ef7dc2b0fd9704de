// Neighbour aggregation over the destination-major CSR (graph_build.hip).
//
// Layout: a "row group" of LPR lanes owns one destination row; lane c of the
// group owns float4 chunks c, c+LPR, ... (CPL chunks) of the H-wide feature
// row, so every gathered neighbour row is read as LPR*16 contiguous bytes
// (one 512-B burst per half-wave at H = 128).  64/LPR rows per wavefront.
// Edges are visited in CSR order == edge_index order (stable CSR), which is
// also the order PyG's scatter-add visits them on the CPU.
//
//  sum_rows_kernel        GCNConv (gcn_norm weights) / GINConv (sum_j x_j +
//                         (1+eps) x_i), CSR entries 8 at a time
//  gat_rows_kernel        GATConv, 4 heads (h 32..256): LeakyReLU logits,
//                         per-row max / sum-exp (+1e-16), alpha-weighted sums
//  tf_rows_kernel         TransformerConv, 4 heads (h 64..256): online softmax
//                         of (q~_i . x_j + c_i) / sqrt(C), alpha-weighted sums
//  gat_aggregate_kernel / transformer_aggregate_kernel: the same for any other
//                         head count / width, one CSR entry at a time
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
    int64_t row_begin, int64_t row_end, int h, float scale, float* __restrict__ out, int64_t ldo,
    bool use_cq) {
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
            cq[hd] = use_cq ? qt[row * ldq + HEADS * h + hd] : 0.f;
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

// ================================================================ batched
// Batched row gather (the eval aggregations at the common widths): a row
// group of LPR lanes owns one destination row and takes its CSR entries
// kB = 8 at a time -- the 8 columns loaded together, then the 8 neighbour
// rows issued together (8 x CPL 16-B loads in flight per lane before the
// first is used), so a row costs one memory round trip per 8 entries instead
// of one per entry (the kernels above).  Entries past the row's end (the
// last batch) read the row's last column and are masked (branch-free loads,
// no per-load waits).  Rows: each XCD (blockIdx & 7) sweeps a contiguous
// eighth of [rb, re), so the neighbour rows a wave gathers were mostly
// fetched into that XCD's L2 by the waves next to it.
constexpr int kB = 8;

template <int LPR>
struct XcdRows {
    int64_t row, stride, end;   // this lane's first row, step, the XCD range's end
};
template <int LPR>
__device__ __forceinline__ XcdRows<LPR> xcd_rows(int64_t rb, int64_t re) {
    constexpr int RPW = 64 / LPR;
    const int64_t n = re - rb;
    const int xcd = blockIdx.x & 7;
    const int64_t wpb = blockDim.x >> 6;
    // the wave index, made visibly wave-uniform: at LPR = 64 (one row per
    // wave) the row, its row_ptr pair, column indices and gather bases are
    // then scalar -- s_load through the constant cache instead of one vector
    // load per index (half the vector-memory instructions of a 1-KB-row sum)
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int64_t wi = static_cast<int64_t>(blockIdx.x >> 3) * wpb + wv;
    const int64_t r0 = rb + n * xcd / 8, r1 = rb + n * (xcd + 1) / 8;
    return {r0 + wi * RPW + (threadIdx.x & 63) / LPR, static_cast<int64_t>(gridDim.x >> 3) * wpb * RPW,
            r1};
}

// blocks of 256 threads for `rows` rows at RPW rows per wave: a multiple of 8
// (one share per XCD), at most `cap`.  The cap sets how many rows an XCD has
// in flight, i.e. how far its waves spread over the row order -- the L2
// working set of the neighbour gathers.  Measured in the locality order
// (scripts/agg_bench.py AGG_LOCAL=1, profiles/r02_agg_grid.json): the 1-KB-row
// sum is fastest at 1024 blocks (4 per CU: 9.9 vs 11.4 ms at 8 per CU), the
// TransformerConv aggregation at h = 256 at 512 (2 per CU: 20.0 vs 24.6 ms;
// at h = 128, 1M rows, the default 2048 stays 7 % faster).
inline unsigned batched_grid(int64_t rows, int lpr, int cap = 2048) {
    const int64_t waves = (rows + 64 / lpr - 1) / (64 / lpr);
    int64_t g = (waves + 3) / 4;
    g = (g + 7) / 8 * 8;
    return static_cast<unsigned>(g < cap ? (g < 8 ? 8 : g) : cap);
}
constexpr int kSumGrid = 1024, kTfGrid = 512;

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf,
                                                              0xf, false));
}
// DPP partners: 0xB1 = lane ^ 1, 0x4E = lane ^ 2 (quad_perm), 0x141 = lane ^ 7
// (row_half_mirror), 0x140 = lane ^ 15 (row_mirror)
constexpr int kX1 = 0xB1, kX2 = 0x4E, kX7 = 0x141, kX15 = 0x140;

// one butterfly step of a reduce-scatter: lanes with bit BIT clear keep the
// sum of value a over the lane and its DPP partner, lanes with it set of b
template <int CTRL, int BIT>
__device__ __forceinline__ float bfly(float a, float b, int lane) {
    const bool hi = ((lane >> BIT) & 1) != 0;
    return (hi ? b : a) + dppf<CTRL>(hi ? a : b);
}

__device__ __forceinline__ void swap_sum32(float& a, float b) {   // lane l: l <-> l ^ 32
    const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a),
                                                    __builtin_bit_cast(unsigned, b), false, false);
    a = __builtin_bit_cast(float, static_cast<unsigned>(r[0])) +
        __builtin_bit_cast(float, static_cast<unsigned>(r[1]));
}
__device__ __forceinline__ void swap_sum16(float& a, float b) {   // lane l: l <-> l ^ 16
    const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a),
                                                    __builtin_bit_cast(unsigned, b), false, false);
    a = __builtin_bit_cast(float, static_cast<unsigned>(r[0])) +
        __builtin_bit_cast(float, static_cast<unsigned>(r[1]));
}

// Reduce-scatter of 32 per-lane partial sums v[i] (i = 8 head + entry) over
// the LPR lanes of a row group.  Afterwards v[0] (and v[1] at LPR = 16) hold
// complete sums, of value index
//   LPR = 64: lane >> 1 (lanes l, l ^ 1 hold the same value)
//   LPR = 32: lane & 31
//   LPR = 16: 2 (lane & 15) + k   (k = 0, 1)
template <int LPR>
__device__ __forceinline__ void reduce_scatter32(float (&v)[32], int lane) {
    static_assert(LPR == 16 || LPR == 32 || LPR == 64, "reduce_scatter32: LPR");
    if constexpr (LPR == 64) {
#pragma unroll
        for (int k = 0; k < 16; ++k) swap_sum32(v[k], v[k + 16]);
#pragma unroll
        for (int k = 0; k < 8; ++k) swap_sum16(v[k], v[k + 8]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = bfly<kX15, 3>(v[k], v[k + 4], lane);
#pragma unroll
        for (int k = 0; k < 2; ++k) v[k] = bfly<kX7, 2>(v[k], v[k + 2], lane);
        v[0] = bfly<kX2, 1>(v[0], v[1], lane);
        v[0] = v[0] + dppf<kX1>(v[0]);
    } else if constexpr (LPR == 32) {
#pragma unroll
        for (int k = 0; k < 16; ++k) swap_sum16(v[k], v[k + 16]);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = bfly<kX15, 3>(v[k], v[k + 8], lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = bfly<kX7, 2>(v[k], v[k + 4], lane);
#pragma unroll
        for (int k = 0; k < 2; ++k) v[k] = bfly<kX2, 1>(v[k], v[k + 2], lane);
        v[0] = bfly<kX1, 0>(v[0], v[1], lane);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = bfly<kX15, 3>(v[k], v[k + 16], lane);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = bfly<kX7, 2>(v[k], v[k + 8], lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = bfly<kX2, 1>(v[k], v[k + 4], lane);
#pragma unroll
        for (int k = 0; k < 2; ++k) v[k] = bfly<kX1, 0>(v[k], v[k + 2], lane);
    }
}

// max / sum over the lanes holding one head's 8 entries in that layout
template <int LPR, bool MAX>
__device__ __forceinline__ float head_reduce(float v) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    v = op(v, dppf<kX1>(v));
    v = op(v, dppf<kX2>(v));
    if constexpr (LPR >= 32) v = op(v, dppf<kX7>(v));
    if constexpr (LPR == 64) v = op(v, dppf<kX15>(v));
    return v;
}

// ---------------------------------------------------------------- sum
template <int LPR, int CPL, bool GCN>
__global__ __launch_bounds__(256) void sum_rows_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ dinv, const float* __restrict__ x, int64_t ldx, float self_scale,
    int64_t rb, int64_t re, int h4, float* __restrict__ out, int64_t ldo) {
    const XcdRows<LPR> xr = xcd_rows<LPR>(rb, re);
    const int c = static_cast<int>(threadIdx.x & 63) % LPR;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t row = xr.row; row < xr.end; row += xr.stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        const float di = GCN ? dinv[row] : 1.f;
        float4 acc[CPL];
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc[q] = zero;
        for (int e0 = beg; e0 < end; e0 += kB) {
            int j[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) j[t] = col[min(e0 + t, end - 1)];
            float w[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) w[t] = GCN ? dinv[j[t]] * di : 1.f;
            float4 xv[kB][CPL];
#pragma unroll
            for (int t = 0; t < kB; ++t)
#pragma unroll
                for (int q = 0; q < CPL; ++q) {
                    const int ch = c + q * LPR;
                    xv[t][q] = ch < h4 ? ld4(x + (int64_t)j[t] * ldx + 4 * ch) : zero;
                }
#pragma unroll
            for (int t = 0; t < kB; ++t) {
                const bool ok = e0 + t < end;
#pragma unroll
                for (int q = 0; q < CPL; ++q) acc[q] = fma4(w[t], ok ? xv[t][q] : zero, acc[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
            const int ch = c + q * LPR;
            if (ch >= h4) continue;
            float4 v = acc[q];
            if (!GCN) {  // GINConv: out + (1 + eps) * x_i
                const float4 xi = ld4(x + row * ldx + 4 * ch);
                v.x = v.x + self_scale * xi.x;
                v.y = v.y + self_scale * xi.y;
                v.z = v.z + self_scale * xi.z;
                v.w = v.w + self_scale * xi.w;
            }
            st4_nt(out + row * ldo + 4 * ch, v);
        }
    }
}

// ---------------------------------------------------------------- GAT (4 heads)
// Softmax work is spread over the row group: lane c owns the (head, entry)
// pairs p = c' + M k (c' = c mod M, M = min(LPR, 32), k < 32 / M; head = p /
// 8, entry t = p mod 8 = c mod 8) -- its score is one logit load, not a
// dot product.  Pass 1: per-head max, pass 2: sum of exp (both over the 8
// lanes of a head, DPP), pass 3: alpha of each pair -> LDS -> every lane
// reads the row's 32 alphas and accumulates its chunk of the 8 gathered rows.
template <int LPR>
__global__ __launch_bounds__(256) void gat_rows_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx, int64_t rb,
    int64_t re, int h, float slope, float* __restrict__ out, int64_t ldo) {
    static_assert(LPR >= 8 && LPR <= 64, "gat_rows: LPR");
    constexpr int HEADS = 4, M = LPR < 32 ? LPR : 32, NPL = 32 / M, RPW = 64 / LPR;
    __shared__ __attribute__((aligned(16))) float s_alpha[4][RPW][32];
    const XcdRows<LPR> xr = xcd_rows<LPR>(rb, re);
    const int lane = static_cast<int>(threadIdx.x & 63);
    const int c = lane % LPR, g = lane / LPR;
    float* const AL = s_alpha[threadIdx.x >> 6][g];
    const int t_own = c & 7;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t row = xr.row; row < xr.end; row += xr.stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        float ad[NPL], mx[NPL], sm[NPL];
#pragma unroll
        for (int k = 0; k < NPL; ++k) {
            const int hd = ((c % M) + M * k) >> 3;
            ad[k] = logits[row * (2 * HEADS) + HEADS + hd];
            mx[k] = -INFINITY;
            sm[k] = 0.f;
        }
        auto score = [&](int jt, int k) {
            const int hd = ((c % M) + M * k) >> 3;
            float v = logits[(int64_t)jt * (2 * HEADS) + hd] + ad[k];
            return v > 0.f ? v : v * slope;
        };
        for (int e0 = beg; e0 < end; e0 += kB) {          // pass 1: max
            const bool ok = e0 + t_own < end;
            const int jt = col[min(e0 + t_own, end - 1)];
#pragma unroll
            for (int k = 0; k < NPL; ++k)
                if (ok) mx[k] = fmaxf(mx[k], score(jt, k));
        }
#pragma unroll
        for (int k = 0; k < NPL; ++k) mx[k] = head_reduce<32, true>(mx[k]);
        for (int e0 = beg; e0 < end; e0 += kB) {          // pass 2: sum of exp
            const bool ok = e0 + t_own < end;
            const int jt = col[min(e0 + t_own, end - 1)];
#pragma unroll
            for (int k = 0; k < NPL; ++k) sm[k] += ok ? expf(score(jt, k) - mx[k]) : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NPL; ++k)
            sm[k] = head_reduce<32, false>(sm[k]) + kSoftmaxEps;
        float4 acc[HEADS];
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) acc[hd] = zero;
        for (int e0 = beg; e0 < end; e0 += kB) {          // pass 3: alpha-weighted rows
            int j[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) j[t] = col[min(e0 + t, end - 1)];
            float4 xv[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) xv[t] = ld4(x + (int64_t)j[t] * ldx + 4 * c);
            {
                const bool ok = e0 + t_own < end;
                const int jt = j[t_own];
#pragma unroll
                for (int k = 0; k < NPL; ++k) {
                    const float a = ok ? expf(score(jt, k) - mx[k]) / sm[k] : 0.f;
                    if (c < 32) AL[(c % M) + M * k] = a;
                }
            }
#pragma unroll
            for (int t = 0; t < kB; ++t)
                if (e0 + t >= end) xv[t] = zero;
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                const float4 a0 = *reinterpret_cast<const float4*>(AL + 8 * hd);
                const float4 a1 = *reinterpret_cast<const float4*>(AL + 8 * hd + 4);
                const float al[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                for (int t = 0; t < kB; ++t) acc[hd] = fma4(al[t], xv[t], acc[hd]);
            }
        }
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) st4_nt(out + row * ldo + hd * h + 4 * c, acc[hd]);
    }
}

// ---------------------------------------------------------------- Transformer (4 heads)
// Per batch of 8 entries: 4 heads x 8 entries partial dots per lane,
// reduce_scatter32 over the row group (each lane then holds one or two
// complete scores), online softmax per head in that layout (DPP), the
// exp-weights and the per-head rescale factors -> LDS -> every lane updates
// its chunk of the 4 head accumulators from the 8 rows already in registers.
template <int LPR>
__global__ __launch_bounds__(256) void tf_rows_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ qt, int64_t ldq, const float* __restrict__ x, int64_t ldx,
    int64_t rb, int64_t re, int h, float scale, float* __restrict__ out, int64_t ldo, bool use_cq) {
    constexpr int HEADS = 4, RPW = 64 / LPR, NV = LPR == 16 ? 2 : 1;
    // per row group: P[32] | C[4] (rescale) | I[4] (1 / (l + eps))
    __shared__ __attribute__((aligned(16))) float s_w[4][RPW][40];
    const XcdRows<LPR> xr = xcd_rows<LPR>(rb, re);
    const int lane = static_cast<int>(threadIdx.x & 63);
    const int c = lane % LPR, g = lane / LPR;
    float* const SW = s_w[threadIdx.x >> 6][g];
    // value index of the reduced layout (v[k] -> pair ix(k) = 8 head + entry)
    auto ix = [&](int k) -> int {
        if constexpr (LPR == 64) return lane >> 1;
        else if constexpr (LPR == 32) return lane & 31;
        else return 2 * (lane & 15) + k;
    };
    const int my_hd = ix(0) >> 3;     // the head of this lane's value(s)
    const bool writer = LPR == 64 ? (lane & 1) == 0 : true;
    const bool head_lead = (ix(0) & 7) == 0 && writer;   // one lane per head
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t row = xr.row; row < xr.end; row += xr.stride) {
        const int beg = row_ptr[row], end = row_ptr[row + 1];
        float4 q[HEADS], acc[HEADS];
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) {
            q[hd] = ld4(qt + row * ldq + hd * h + 4 * c);
            acc[hd] = zero;
        }
        const float cq = use_cq ? qt[row * ldq + HEADS * h + my_hd] : 0.f;
        float m = -INFINITY, l = 0.f;      // this lane's head, reduced layout
        for (int e0 = beg; e0 < end; e0 += kB) {
            int j[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) j[t] = col[min(e0 + t, end - 1)];
            float4 xv[kB];
#pragma unroll
            for (int t = 0; t < kB; ++t) xv[t] = ld4(x + (int64_t)j[t] * ldx + 4 * c);
            float v[32];
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd)
#pragma unroll
                for (int t = 0; t < kB; ++t) {
                    float d = 0.f;
                    d = fmaf(q[hd].x, xv[t].x, d);
                    d = fmaf(q[hd].y, xv[t].y, d);
                    d = fmaf(q[hd].z, xv[t].z, d);
                    d = fmaf(q[hd].w, xv[t].w, d);
                    v[8 * hd + t] = d;
                }
            reduce_scatter32<LPR>(v, lane);
            float s[NV], bm = -INFINITY;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                s[k] = e0 + (ix(k) & 7) < end ? (v[k] + cq) * scale : -INFINITY;
                bm = fmaxf(bm, s[k]);
            }
            bm = head_reduce<LPR, true>(bm);
            const float mn = fmaxf(m, bm);
            const float corr = m == -INFINITY ? 0.f : expf(m - mn);
            float ps = 0.f;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const float p = expf(s[k] - mn);
                if (writer) SW[ix(k)] = p;
                ps += (LPR == 64 && !writer) ? 0.f : p;
            }
            l = l * corr + head_reduce<LPR, false>(ps);
            m = mn;
            if (head_lead) SW[32 + my_hd] = corr;
#pragma unroll
            for (int t = 0; t < kB; ++t)
                if (e0 + t >= end) xv[t] = zero;
            const float4 cr = *reinterpret_cast<const float4*>(SW + 32);
            const float crs[4] = {cr.x, cr.y, cr.z, cr.w};
#pragma unroll
            for (int hd = 0; hd < HEADS; ++hd) {
                const float4 p0 = *reinterpret_cast<const float4*>(SW + 8 * hd);
                const float4 p1 = *reinterpret_cast<const float4*>(SW + 8 * hd + 4);
                const float pv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
                float4 a = acc[hd];
                a.x *= crs[hd]; a.y *= crs[hd]; a.z *= crs[hd]; a.w *= crs[hd];
#pragma unroll
                for (int t = 0; t < kB; ++t) a = fma4(pv[t], xv[t], a);
                acc[hd] = a;
            }
        }
        const float inv = 1.f / (l + kSoftmaxEps);
        if (head_lead) {
            SW[36 + my_hd] = inv;
            __builtin_nontemporal_store(l * inv, &out[row * ldo + HEADS * h + my_hd]);   // sum_j alpha
        }
        const float4 iv = *reinterpret_cast<const float4*>(SW + 36);
        const float ivs[4] = {iv.x, iv.y, iv.z, iv.w};
#pragma unroll
        for (int hd = 0; hd < HEADS; ++hd) {
            float4 a = acc[hd];
            a.x *= ivs[hd]; a.y *= ivs[hd]; a.z *= ivs[hd]; a.w *= ivs[hd];
            st4_nt(out + row * ldo + hd * h + 4 * c, a);
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

// batched kernels: h a multiple of 4 with LPR = pow2 >= h/4 (<= 64), any CPL
#define MIGNN_DISPATCH_SUM(h4, BODY)                                      \
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

extern "C" int mignn_gcn_aggregate(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                                   const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                   float* out, int64_t ldo, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    MIGNN_REQUIRE(dinv, "gcn_aggregate: null dinv");
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_SUM(h4, (sum_rows_kernel<LPR, CPL, true><<<dim3(batched_grid(re - rb, LPR, kSumGrid)), dim3(256), 0, as_stream(stream)>>>(
                               row_ptr, col, dinv, x, ldx, 1.f, rb, re, h4, out, ldo)));
    return launch_status("gcn_aggregate");
}

extern "C" int mignn_sum_aggregate(const int32_t* row_ptr, const int32_t* col, const float* x,
                                   int64_t ldx, float self_scale, int64_t rb, int64_t re, int h,
                                   float* out, int64_t ldo, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    MIGNN_DISPATCH_SUM(h4, (sum_rows_kernel<LPR, CPL, false><<<dim3(batched_grid(re - rb, LPR, kSumGrid)), dim3(256), 0, as_stream(stream)>>>(
                               row_ptr, col, nullptr, x, ldx, self_scale, rb, re, h4, out, ldo)));
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
    hipStream_t st = as_stream(stream);
    // batched: 4 heads, h = 4 LPR (LPR in 8..64)
    if (heads == 4 && (h == 32 || h == 64 || h == 128 || h == 256)) {
        switch (h) {
            case 32: gat_rows_kernel<8><<<dim3(batched_grid(re - rb, 8)), dim3(256), 0, st>>>(row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo); break;
            case 64: gat_rows_kernel<16><<<dim3(batched_grid(re - rb, 16)), dim3(256), 0, st>>>(row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo); break;
            case 128: gat_rows_kernel<32><<<dim3(batched_grid(re - rb, 32)), dim3(256), 0, st>>>(row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo); break;
            default: gat_rows_kernel<64><<<dim3(batched_grid(re - rb, 64)), dim3(256), 0, st>>>(row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo); break;
        }
        return launch_status("gat_aggregate");
    }
    MIGNN_DISPATCH_HEADS(heads, MIGNN_DISPATCH_LPR(h4, (gat_aggregate_kernel<LPR, CPL, HEADS><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, st>>>( row_ptr, col, logits, x, ldx, rb, re, h, slope, out, ldo))));
    return launch_status("gat_aggregate");
}

namespace mignn {
// use_cq = false: the per-head score constant c_i = q_i . b_k is left out
// (qt's last `heads` columns are not read): it shifts every score of a row's
// head by the same amount, which the softmax cancels -- the layer entry
// (attn_layers.hip) does not compute it
int transformer_aggregate_rows(const int32_t* row_ptr, const int32_t* col, const float* qt,
                               int64_t ldq, const float* x, int64_t ldx, int64_t rb, int64_t re,
                               int h, int heads, float score_scale, float* out, int64_t ldo,
                               bool use_cq, void* stream) {
    if (int rc = check_common(row_ptr, col, x, ldx, rb, re, h, out, ldo)) return rc;
    MIGNN_REQUIRE(qt && aligned16(qt) && ldq % 4 == 0 &&
                      ldq >= (int64_t)heads * h + (use_cq ? heads : 0),
                  "transformer_aggregate: bad qt");
    MIGNN_REQUIRE(ldo >= (int64_t)heads * h + heads, "transformer_aggregate: ldo too small");
    if (re == rb) return MIGNN_OK;
    const int h4 = h / 4;
    hipStream_t st = as_stream(stream);
    // batched: 4 heads, h = 4 LPR (LPR in 16..64)
    if (heads == 4 && (h == 64 || h == 128 || h == 256)) {
        switch (h) {
            case 64: tf_rows_kernel<16><<<dim3(batched_grid(re - rb, 16)), dim3(256), 0, st>>>(row_ptr, col, qt, ldq, x, ldx, rb, re, h, score_scale, out, ldo, use_cq); break;
            case 128: tf_rows_kernel<32><<<dim3(batched_grid(re - rb, 32)), dim3(256), 0, st>>>(row_ptr, col, qt, ldq, x, ldx, rb, re, h, score_scale, out, ldo, use_cq); break;
            default: tf_rows_kernel<64><<<dim3(batched_grid(re - rb, 64, kTfGrid)), dim3(256), 0, st>>>(row_ptr, col, qt, ldq, x, ldx, rb, re, h, score_scale, out, ldo, use_cq); break;
        }
        return launch_status("transformer_aggregate");
    }
    MIGNN_DISPATCH_HEADS(heads, MIGNN_DISPATCH_LPR(h4, (transformer_aggregate_kernel<LPR, CPL, HEADS><<<dim3(agg_grid(re - rb, LPR)), dim3(256), 0, st>>>( row_ptr, col, qt, ldq, x, ldx, rb, re, h, score_scale,
        out, ldo, use_cq))));
    return launch_status("transformer_aggregate");
}
}  // namespace mignn

extern "C" int mignn_transformer_aggregate(const int32_t* row_ptr, const int32_t* col,
                                           const float* qt, int64_t ldq, const float* x,
                                           int64_t ldx, int64_t rb, int64_t re, int h, int heads,
                                           float score_scale, float* out, int64_t ldo,
                                           void* stream) {
    return transformer_aggregate_rows(row_ptr, col, qt, ldq, x, ldx, rb, re, h, heads, score_scale,
                                      out, ldo, true, stream);
}
