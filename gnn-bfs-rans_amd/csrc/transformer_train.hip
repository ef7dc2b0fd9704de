// TransformerConv training path (PyG TransformerConv(H, H,
// heads, concat=False, dropout=p, edge_dim=None, beta=False) as constructed at
// gnn_model.py:77-80, called at :170 with edge_attr=None).
//
// Training keeps Q, K, V explicit (one MFMA launch for [Wq;Wk;Wv]):
//   s_ji   = <Q_i[k], K_j[k]> / sqrt(H)           over edge_index as given
//   alpha  = per-destination softmax (exp(s - max) / (sum + 1e-16)), then
//            attention dropout (counter hash of (seed, dst, src, head))
//   O_i    = (1/heads) sum_k sum_j drop(alpha_jik) V_j[k]   (+ x_i, residual)
//   z      = O + x + lin_skip(x)                              (MFMA epilogue)
// A row with no incoming edge aggregates to 0 (PyG's empty scatter).
//
// Backward, dY_i[k] = dz_i / heads:
//   dalpha_jik = drop * <dY_i[k], V_j[k]>,  c_ik = sum_j alpha dalpha
//   ds_jik     = alpha (dalpha - c_ik) / sqrt(H)
//   dQ_i[k] = sum_j ds K_j[k]                       (rows kernel, forward CSR)
//   dK_j[k] = sum_i ds Q_i[k],  dV_j[k] = sum_i drop alpha dY_i[k]
//                                                   (cols kernel, reversed CSR)
// The forward leaves (max, 1/(sum+1e-16)) per (row, head) and the per-head
// aggregates Y_i[k]; the rows kernel takes c = <dY_i[k], Y_i[k]> from them and
// makes one pass over the row; the cols kernel recomputes alpha from
// Q_i . K_j and those values: no edge map, no atomics.
// One 64-lane wave per row, channels c = lane + 64 v.
#include "common.hpp"

namespace mignn {
namespace {

constexpr int kWaves = 4;


__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int VPL>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int lane, int h, float (&v)[VPL]) {
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int c = lane + 64 * u;
        v[u] = c < h ? p[c] : 0.f;
    }
}

// two independent wave reductions with their shuffle chains interleaved
__device__ __forceinline__ void wave_sum2(float& a, float& b) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
}

template <int VPL>
__device__ __forceinline__ float dot_row(const float (&a)[VPL], const float* __restrict__ p, int lane,
                                         int h) {
    float d = 0.f;
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int c = lane + 64 * u;
        if (c < h) d += a[u] * p[c];
    }
    return wave_sum(d);
}

struct QKV {
    const float* base;
    int64_t ld;
    int h, heads;
    __device__ __forceinline__ const float* q(int64_t r, int k) const { return base + r * ld + int64_t(k) * h; }
    __device__ __forceinline__ const float* kk(int64_t r, int k) const { return base + r * ld + int64_t(heads + k) * h; }
    __device__ __forceinline__ const float* v(int64_t r, int k) const { return base + r * ld + int64_t(2 * heads + k) * h; }
};

template <int VPL>
__global__ __launch_bounds__(256) void tf_fwd_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, QKV t, float scale,
    EdgeDrop drop, const float* __restrict__ x, int64_t ldx, int64_t n, float* __restrict__ o,
    int64_t ldo, float* __restrict__ yh, int64_t ldyh, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (i >= n) return;
    const int h = t.h, beg = row_ptr[i], end = row_ptr[i + 1];
    const float hinv = 1.f / t.heads;
    float out[VPL];
    load_row<VPL>(x + i * ldx, lane, h, out);   // residual x_i
    for (int k = 0; k < t.heads; ++k) {
        float q[VPL], acc[VPL];
        load_row<VPL>(t.q(i, k), lane, h, q);
        float m = -INFINITY, s = 0.f;
#pragma unroll
        for (int u = 0; u < VPL; ++u) acc[u] = 0.f;
        auto step = [&](int64_t j, float sc) {   // online softmax, edge order
            if (sc > m) {
                const float r = expf(m - sc);
                s *= r;
#pragma unroll
                for (int u = 0; u < VPL; ++u) acc[u] *= r;
                m = sc;
            }
            const float w = expf(sc - m);
            s += w;
            const float wk = w * drop.keep(i, j, k);
            const float* vj = t.v(j, k);
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                const int c = lane + 64 * u;
                if (c < h) acc[u] += wk * vj[c];
            }
        };
        int e = beg;
        for (; e + 1 < end; e += 2) {   // two scores per pass: interleaved reductions
            const int64_t j0 = col[e], j1 = col[e + 1];
            float k0[VPL], k1[VPL];
            load_row<VPL>(t.kk(j0, k), lane, h, k0);
            load_row<VPL>(t.kk(j1, k), lane, h, k1);
            float d0 = 0.f, d1 = 0.f;
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                d0 += q[u] * k0[u];
                d1 += q[u] * k1[u];
            }
            wave_sum2(d0, d1);
            step(j0, d0 * scale);
            step(j1, d1 * scale);
        }
        if (e < end) step(col[e], dot_row<VPL>(q, t.kk(col[e], k), lane, h) * scale);
        const float inv = 1.f / (s + 1e-16f);
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            const int c = lane + 64 * u;
            const float yv = acc[u] * inv;   // per-head aggregate Y_i[k]
            out[u] += yv * hinv;
            if (yh && c < h) yh[i * ldyh + int64_t(k) * h + c] = yv;
        }
        if (stats && lane == 0) {   // softmax state for the backward
            stats[i * 3 * t.heads + k] = m;
            stats[i * 3 * t.heads + t.heads + k] = inv;
        }
    }
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int c = lane + 64 * u;
        if (c < h) o[i * ldo + c] = out[u];
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void tf_bwd_rows_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, QKV t, float scale,
    EdgeDrop drop, const float* __restrict__ dz, int64_t lddz, const float* __restrict__ yh,
    int64_t ldyh, int64_t n, float* __restrict__ stats, float* __restrict__ dqkv, int64_t ldd) {
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (i >= n) return;
    const int h = t.h, heads = t.heads, beg = row_ptr[i], end = row_ptr[i + 1];
    float dy[VPL];
    load_row<VPL>(dz + i * lddz, lane, h, dy);
#pragma unroll
    for (int u = 0; u < VPL; ++u) dy[u] *= 1.f / heads;
    for (int k = 0; k < heads; ++k) {
        float q[VPL], dq[VPL];
        load_row<VPL>(t.q(i, k), lane, h, q);
        const float m = stats[i * 3 * heads + k];          // from the forward
        const float inv = stats[i * 3 * heads + heads + k];
        // c = sum_j alpha dalpha = <dY_i[k], Y_i[k]> (Y = the forward's per-head aggregate)
        const float cs = dot_row<VPL>(dy, yh + i * ldyh + int64_t(k) * h, lane, h);
#pragma unroll
        for (int u = 0; u < VPL; ++u) dq[u] = 0.f;
        for (int e = beg; e < end; ++e) {
            const int64_t j = col[e];
            float kv[VPL], vv[VPL];
            load_row<VPL>(t.kk(j, k), lane, h, kv);
            load_row<VPL>(t.v(j, k), lane, h, vv);
            float d1 = 0.f, d2 = 0.f;
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                d1 += q[u] * kv[u];
                d2 += dy[u] * vv[u];
            }
            wave_sum2(d1, d2);
            const float alpha = expf(d1 * scale - m) * inv;
            const float da = d2 * drop.keep(i, j, k);
            const float ds = alpha * (da - cs) * scale;
#pragma unroll
            for (int u = 0; u < VPL; ++u) dq[u] += ds * kv[u];
        }
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            const int c = lane + 64 * u;
            if (c < h) dqkv[i * ldd + int64_t(k) * h + c] = dq[u];
        }
        if (lane == 0) stats[i * 3 * heads + 2 * heads + k] = cs;
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void tf_bwd_cols_kernel(
    const int32_t* __restrict__ rowt_ptr, const int32_t* __restrict__ colt, QKV t, float scale,
    EdgeDrop drop, const float* __restrict__ dz, int64_t lddz, int64_t n,
    const float* __restrict__ stats, float* __restrict__ dqkv, int64_t ldd) {
    const int lane = threadIdx.x & 63;
    const int64_t j = static_cast<int64_t>(blockIdx.x) * kWaves + (threadIdx.x >> 6);
    if (j >= n) return;
    const int h = t.h, heads = t.heads, beg = rowt_ptr[j], end = rowt_ptr[j + 1];
    const float hinv = 1.f / heads;
    for (int k = 0; k < heads; ++k) {
        float kj[VPL], vj[VPL], dk[VPL], dv[VPL];
        load_row<VPL>(t.kk(j, k), lane, h, kj);
        load_row<VPL>(t.v(j, k), lane, h, vj);
#pragma unroll
        for (int u = 0; u < VPL; ++u) dk[u] = dv[u] = 0.f;
        for (int e = beg; e < end; ++e) {
            const int64_t i = colt[e];
            float qv[VPL], gv[VPL];
            load_row<VPL>(t.q(i, k), lane, h, qv);
            load_row<VPL>(dz + i * lddz, lane, h, gv);
            const float m = stats[i * 3 * heads + k];
            const float inv = stats[i * 3 * heads + heads + k];
            const float cs = stats[i * 3 * heads + 2 * heads + k];
            float d1 = 0.f, d2 = 0.f;
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                d1 += kj[u] * qv[u];
                d2 += vj[u] * gv[u];
            }
            wave_sum2(d1, d2);
            const float alpha = expf(d1 * scale - m) * inv;
            const float kp = drop.keep(i, j, k);
            const float da = d2 * hinv * kp;
            const float ds = alpha * (da - cs) * scale;
            const float wv = alpha * kp * hinv;
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                dv[u] += wv * gv[u];
                dk[u] += ds * qv[u];
            }
        }
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            const int c = lane + 64 * u;
            if (c < h) {
                dqkv[j * ldd + int64_t(heads + k) * h + c] = dk[u];
                dqkv[j * ldd + int64_t(2 * heads + k) * h + c] = dv[u];
            }
        }
    }
}

int vpl_for(int h) { return h <= 64 ? 1 : h <= 128 ? 2 : h <= 256 ? 4 : 0; }

}  // namespace
}  // namespace mignn

using namespace mignn;

#define MIGNN_TF_DISPATCH(KERNEL, ...)                                                        \
    switch (vpl_for(h)) {                                                                    \
        case 1: KERNEL<1><<<grid, block, 0, st>>>(__VA_ARGS__); break;                       \
        case 2: KERNEL<2><<<grid, block, 0, st>>>(__VA_ARGS__); break;                       \
        default: KERNEL<4><<<grid, block, 0, st>>>(__VA_ARGS__); break;                      \
    }

extern "C" int mignn_transformer_train_forward(const int32_t* row_ptr, const int32_t* col,
                                               const float* qkv, int64_t ldq, const float* x,
                                               int64_t ldx, int64_t n, int h, int heads,
                                               float score_scale, float p, uint64_t seed,
                                               float* out, int64_t ldo, float* yh, int64_t ldyh,
                                               float* stats, void* stream) {
    MIGNN_REQUIRE(n >= 0 && h > 0 && heads > 0 && heads <= 8, "transformer_train_forward: bad shape");
    MIGNN_REQUIRE(vpl_for(h) > 0, "transformer_train_forward: hidden %d > 256", h);
    MIGNN_REQUIRE(ldq >= int64_t(3) * heads * h && ldx >= h && ldo >= h,
                  "transformer_train_forward: bad leading dims");
    if (n == 0) return 0;
    MIGNN_REQUIRE(row_ptr && col && qkv && x && out, "transformer_train_forward: null pointer");
    const QKV t{qkv, ldq, h, heads};
    const EdgeDrop d = make_edge_drop(p, seed, n, heads);
    const dim3 grid(static_cast<unsigned>((n + kWaves - 1) / kWaves)), block(64 * kWaves);
    hipStream_t st = as_stream(stream);
    MIGNN_REQUIRE(!yh || ldyh >= int64_t(heads) * h, "transformer_train_forward: bad ldyh");
    MIGNN_TF_DISPATCH(tf_fwd_kernel, row_ptr, col, t, score_scale, d, x, ldx, n, out, ldo, yh, ldyh,
                      stats)
    return launch_status("tf_fwd_kernel");
}

extern "C" int mignn_transformer_train_backward(const int32_t* row_ptr, const int32_t* col,
                                                const int32_t* rowt_ptr, const int32_t* colt,
                                                const float* qkv, int64_t ldq, const float* dz,
                                                int64_t lddz, const float* yh, int64_t ldyh,
                                                int64_t n, int h, int heads,
                                                float score_scale, float p, uint64_t seed,
                                                float* stats, float* dqkv, int64_t ldd,
                                                void* stream) {
    MIGNN_REQUIRE(n >= 0 && h > 0 && heads > 0 && heads <= 8, "transformer_train_backward: bad shape");
    MIGNN_REQUIRE(vpl_for(h) > 0, "transformer_train_backward: hidden %d > 256", h);
    MIGNN_REQUIRE(ldq >= int64_t(3) * heads * h && ldd >= int64_t(3) * heads * h && lddz >= h,
                  "transformer_train_backward: bad leading dims");
    if (n == 0) return 0;
    MIGNN_REQUIRE(ldyh >= int64_t(heads) * h, "transformer_train_backward: bad ldyh");
    MIGNN_REQUIRE(row_ptr && col && rowt_ptr && colt && qkv && dz && yh && stats && dqkv,
                  "transformer_train_backward: null pointer");
    const QKV t{qkv, ldq, h, heads};
    const EdgeDrop d = make_edge_drop(p, seed, n, heads);
    const dim3 grid(static_cast<unsigned>((n + kWaves - 1) / kWaves)), block(64 * kWaves);
    hipStream_t st = as_stream(stream);
    int rc;
    MIGNN_TF_DISPATCH(tf_bwd_rows_kernel, row_ptr, col, t, score_scale, d, dz, lddz, yh, ldyh, n,
                      stats, dqkv, ldd)
    if ((rc = launch_status("tf_bwd_rows_kernel"))) return rc;
    MIGNN_TF_DISPATCH(tf_bwd_cols_kernel, rowt_ptr, colt, t, score_scale, d, dz, lddz, n, stats, dqkv, ldd)
    return launch_status("tf_bwd_cols_kernel");
}
