// GATConv training path (PyG GATConv(H, H, heads, concat=False,
// dropout=p) as constructed at gnn_model.py:65-68 and called at :168).
//
// The layer is computed re-associated, as in eval (gnn_model.py host layer):
//   logits [N, 2*heads] = x . [v_src | v_dst]^T      (v_k = W_k^T att_k)
//   Y_i[k]  = sum_{j in row i} drop(alpha_jik) x_j   (this file, forward)
//   z       = Y . Wcat^T + b + x                      (MFMA epilogue, residual)
// with alpha = per-destination softmax of LeakyReLU(a_src[j] + a_dst[i])
// (PyG softmax: exp(e - max) / (sum + 1e-16)) and the attention dropout of
// GATConv.message applied after the softmax.  Dropout mask: counter hash of
// (seed, dst, src, head), regenerated in the backward -- nothing stored.
//
// Backward (dY = dz . Wcat given):
//   dalpha_jik = drop_jik * <dY_i[k], x_j>
//   de_jik     = alpha_jik (dalpha_jik - c_ik),  c_ik = sum_j alpha_jik dalpha_jik
//   ds_jik     = de_jik * (pre > 0 ? 1 : slope)
//   dlogits[i, heads + k] = sum_j ds_jik          (rows kernel, forward CSR)
//   dlogits[j, k]         = sum_i ds_jik          (cols kernel, reversed CSR)
//   dx_j = dz_j + sum_{i,k} drop alpha_jik dY_i[k] (+ dlogits . [v_src|v_dst] by GEMM)
// The forward leaves (max, 1/(sum+1e-16)) per (row, head); the rows kernel
// adds c = <dY_i[k], Y_i[k]> (Y = the forward's aggregate, so no extra pass)
// and needs one pass over the row; the cols kernel recomputes alpha for any
// edge from the two logits and those values: no edge-id map between the two
// CSR orders, no atomics, deterministic.
//
// One 64-lane wave per row, channels c = lane + 64 v (coalesced row reads),
// scalar softmax state replicated across the wave.
#include "common.hpp"

namespace mignn {
namespace {

constexpr int kWaves = 4;   // rows per 256-thread block


__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float leaky(float s, float slope) { return s > 0.f ? s : s * slope; }

constexpr int kMaxHeads = 8;

// All heads in one pass over the row: the scalar softmax state of every head
// first (logit rows only, [2*heads] floats per node), then each neighbour row
// x_j is read once and feeds all heads' accumulators.
template <int VPL>
__global__ __launch_bounds__(256) void gat_fwd_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx, int64_t n, int h,
    int heads, float slope, EdgeDrop drop, float* __restrict__ y, int64_t ldy,
    float* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (i >= n) return;
    const int beg = row_ptr[i], end = row_ptr[i + 1];
    const int ldl = 2 * heads;
    float ad[kMaxHeads], m[kMaxHeads], inv[kMaxHeads], acc[kMaxHeads][VPL];
#pragma unroll
    for (int k = 0; k < kMaxHeads; ++k) {
        ad[k] = k < heads ? logits[i * ldl + heads + k] : 0.f;
        m[k] = -INFINITY;
        inv[k] = 0.f;
#pragma unroll
        for (int v = 0; v < VPL; ++v) acc[k][v] = 0.f;
    }
    for (int e = beg; e < end; ++e) {
        const int64_t j = col[e];
#pragma unroll
        for (int k = 0; k < kMaxHeads; ++k)
            if (k < heads) m[k] = fmaxf(m[k], leaky(logits[j * ldl + k] + ad[k], slope));
    }
    for (int e = beg; e < end; ++e) {
        const int64_t j = col[e];
#pragma unroll
        for (int k = 0; k < kMaxHeads; ++k)
            if (k < heads) inv[k] += expf(leaky(logits[j * ldl + k] + ad[k], slope) - m[k]);
    }
#pragma unroll
    for (int k = 0; k < kMaxHeads; ++k) {
        inv[k] = 1.f / (inv[k] + 1e-16f);
        if (k < heads && stats && lane == 0) {   // softmax state for the backward
            stats[i * 3 * heads + k] = m[k];
            stats[i * 3 * heads + heads + k] = inv[k];
        }
    }
    for (int e = beg; e < end; ++e) {
        const int64_t j = col[e];
        float xv[VPL];
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
            const int c = lane + 64 * v;
            xv[v] = c < h ? x[j * ldx + c] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < kMaxHeads; ++k) {
            if (k >= heads) break;
            const float a = expf(leaky(logits[j * ldl + k] + ad[k], slope) - m[k]) * inv[k] *
                            drop.keep(i, j, k);
#pragma unroll
            for (int v = 0; v < VPL; ++v) acc[k][v] += a * xv[v];
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxHeads; ++k) {
        if (k >= heads) break;
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
            const int c = lane + 64 * v;
            if (c < h) y[i * ldy + int64_t(k) * h + c] = acc[k][v];
        }
    }
}

// rows (destinations) of the forward CSR: dlogits[:, heads + k], head by head
// (a head-fused variant held 4 x VPL gradients in VGPRs and ran slower)
template <int VPL>
__global__ __launch_bounds__(256) void gat_bwd_rows_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ yf, int64_t ldyf,
    int64_t n, int h, int heads, float slope, EdgeDrop drop, float* __restrict__ stats,
    float* __restrict__ dlog) {
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (i >= n) return;
    const int beg = row_ptr[i], end = row_ptr[i + 1];
    const int ldl = 2 * heads;
    for (int k = 0; k < heads; ++k) {
        const float ad = logits[i * ldl + heads + k];
        const float m = stats[i * 3 * heads + k];          // from the forward
        const float inv = stats[i * 3 * heads + heads + k];
        float g[VPL];
        float d0 = 0.f;
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
            const int c = lane + 64 * v;
            g[v] = c < h ? dy[i * lddy + int64_t(k) * h + c] : 0.f;
            if (c < h) d0 += g[v] * yf[i * ldyf + int64_t(k) * h + c];
        }
        // c = sum_j alpha dalpha = <dY_i[k], Y_i[k]> (Y = the forward's aggregate)
        const float cs = wave_sum(d0);
        float a1 = 0.f, a2 = 0.f;
        for (int e = beg; e < end; ++e) {
            const int64_t j = col[e];
            const float pre = logits[j * ldl + k] + ad;
            const float lp = pre > 0.f ? 1.f : slope;
            const float alpha = expf(leaky(pre, slope) - m) * inv;
            float d = 0.f;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                const int c = lane + 64 * v;
                if (c < h) d += g[v] * x[j * ldx + c];
            }
            const float da = wave_sum(d) * drop.keep(i, j, k);
            a1 += alpha * da * lp;
            a2 += alpha * lp;
        }
        if (lane == 0) {
            stats[i * 3 * heads + 2 * heads + k] = cs;
            dlog[i * ldl + heads + k] = a1 - cs * a2;
        }
    }
}

// rows (sources) of the reversed CSR: dx_j (+ dz_j) and dlogits[:, k]
template <int VPL>
__global__ __launch_bounds__(256) void gat_bwd_cols_kernel(
    const int32_t* __restrict__ rowt_ptr, const int32_t* __restrict__ colt,
    const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ dz, int64_t lddz,
    int64_t n, int h, int heads, float slope, EdgeDrop drop, const float* __restrict__ stats,
    float* __restrict__ dlog, float* __restrict__ dx, int64_t lddx) {
    const int lane = threadIdx.x & 63;
    const int64_t j = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (j >= n) return;
    const int beg = rowt_ptr[j], end = rowt_ptr[j + 1];
    const int ldl = 2 * heads;
    float xj[VPL], acc[VPL];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
        const int c = lane + 64 * v;
        xj[v] = c < h ? x[j * ldx + c] : 0.f;
        acc[v] = (c < h && dz) ? dz[j * lddz + c] : 0.f;
    }
    for (int k = 0; k < heads; ++k) {
        const float as = logits[j * ldl + k];
        float das = 0.f;
        for (int e = beg; e < end; ++e) {
            const int64_t i = colt[e];
            const float m = stats[i * 3 * heads + k];
            const float inv = stats[i * 3 * heads + heads + k];
            const float cs = stats[i * 3 * heads + 2 * heads + k];
            const float pre = as + logits[i * ldl + heads + k];
            const float lp = pre > 0.f ? 1.f : slope;
            const float alpha = expf(leaky(pre, slope) - m) * inv;
            const float kp = drop.keep(i, j, k);
            const float w = alpha * kp;
            float d = 0.f;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                const int c = lane + 64 * v;
                if (c < h) {
                    const float gv = dy[i * lddy + int64_t(k) * h + c];
                    acc[v] += w * gv;
                    d += gv * xj[v];
                }
            }
            const float da = wave_sum(d) * kp;
            das += alpha * (da - cs) * lp;
        }
        if (lane == 0) dlog[j * ldl + k] = das;
    }
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
        const int c = lane + 64 * v;
        if (c < h) dx[j * lddx + c] = acc[v];
    }
}

int vpl_for(int h) { return h <= 64 ? 1 : h <= 128 ? 2 : h <= 256 ? 4 : 0; }

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_gat_train_forward(const int32_t* row_ptr, const int32_t* col,
                                       const float* logits, const float* x, int64_t ldx,
                                       int64_t n, int h, int heads, float negative_slope, float p,
                                       uint64_t seed, float* y, int64_t ldy, float* stats,
                                       void* stream) {
    MIGNN_REQUIRE(n >= 0 && h > 0 && heads > 0 && heads <= 8, "gat_train_forward: bad shape");
    MIGNN_REQUIRE(vpl_for(h) > 0, "gat_train_forward: hidden %d > 256", h);
    MIGNN_REQUIRE(ldx >= h && ldy >= int64_t(heads) * h, "gat_train_forward: bad leading dims");
    if (n == 0) return 0;
    MIGNN_REQUIRE(row_ptr && col && logits && x && y, "gat_train_forward: null pointer");
    const EdgeDrop d = make_edge_drop(p, seed, n, heads);
    const dim3 grid(static_cast<unsigned>((n + kWaves - 1) / kWaves)), block(64 * kWaves);
    hipStream_t st = as_stream(stream);
    switch (vpl_for(h)) {
        case 1: gat_fwd_kernel<1><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, n, h, heads, negative_slope, d, y, ldy, stats); break;
        case 2: gat_fwd_kernel<2><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, n, h, heads, negative_slope, d, y, ldy, stats); break;
        default: gat_fwd_kernel<4><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, n, h, heads, negative_slope, d, y, ldy, stats); break;
    }
    return launch_status("gat_fwd_kernel");
}

extern "C" int mignn_gat_train_backward(const int32_t* row_ptr, const int32_t* col,
                                        const int32_t* rowt_ptr, const int32_t* colt,
                                        const float* logits, const float* x, int64_t ldx,
                                        const float* dy, int64_t lddy, const float* y,
                                        int64_t ldy, const float* dz,
                                        int64_t lddz, int64_t n, int h, int heads,
                                        float negative_slope, float p, uint64_t seed,
                                        float* stats, float* dlogits, float* dx, int64_t lddx,
                                        void* stream) {
    MIGNN_REQUIRE(n >= 0 && h > 0 && heads > 0 && heads <= 8, "gat_train_backward: bad shape");
    MIGNN_REQUIRE(vpl_for(h) > 0, "gat_train_backward: hidden %d > 256", h);
    MIGNN_REQUIRE(ldx >= h && lddx >= h && lddy >= int64_t(heads) * h && (!dz || lddz >= h),
                  "gat_train_backward: bad leading dims");
    if (n == 0) return 0;
    MIGNN_REQUIRE(ldy >= int64_t(heads) * h, "gat_train_backward: bad ldy");
    MIGNN_REQUIRE(row_ptr && col && rowt_ptr && colt && logits && x && dy && y && stats && dlogits && dx,
                  "gat_train_backward: null pointer");
    const EdgeDrop d = make_edge_drop(p, seed, n, heads);
    const dim3 grid(static_cast<unsigned>((n + kWaves - 1) / kWaves)), block(64 * kWaves);
    hipStream_t st = as_stream(stream);
    int rc;
    switch (vpl_for(h)) {
        case 1: gat_bwd_rows_kernel<1><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, dy, lddy, y, ldy, n, h, heads, negative_slope, d, stats, dlogits); break;
        case 2: gat_bwd_rows_kernel<2><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, dy, lddy, y, ldy, n, h, heads, negative_slope, d, stats, dlogits); break;
        default: gat_bwd_rows_kernel<4><<<grid, block, 0, st>>>(row_ptr, col, logits, x, ldx, dy, lddy, y, ldy, n, h, heads, negative_slope, d, stats, dlogits); break;
    }
    if ((rc = launch_status("gat_bwd_rows_kernel"))) return rc;
    switch (vpl_for(h)) {
        case 1: gat_bwd_cols_kernel<1><<<grid, block, 0, st>>>(rowt_ptr, colt, logits, x, ldx, dy, lddy, dz, lddz, n, h, heads, negative_slope, d, stats, dlogits, dx, lddx); break;
        case 2: gat_bwd_cols_kernel<2><<<grid, block, 0, st>>>(rowt_ptr, colt, logits, x, ldx, dy, lddy, dz, lddz, n, h, heads, negative_slope, d, stats, dlogits, dx, lddx); break;
        default: gat_bwd_cols_kernel<4><<<grid, block, 0, st>>>(rowt_ptr, colt, logits, x, ldx, dy, lddy, dz, lddz, n, h, heads, negative_slope, d, stats, dlogits, dx, lddx); break;
    }
    return launch_status("gat_bwd_cols_kernel");
}
