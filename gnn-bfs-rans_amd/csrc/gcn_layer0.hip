// input_proj + first GCN layer in one pass over the coordinates.
//
// FlowGNN's first two steps (gnn_model.py:159, :162-192 with GCNConv) are
//   x0_i = W_in c_i + b_in                                   (c_i: D <= 8 features)
//   y_i  = relu( sc * (x0_i + b + W sum_j w_ij x0_j) + sh )  (eval BN folded in sc, sh)
// and both maps are linear up to the ReLU, so with C_i = sum_j w_ij c_j and
// s_i = sum_j w_ij (the CSR row incl. the self-loop, PyG gcn_norm weights):
//   y_i = relu( A c_i + B C_i + d s_i + e ),
//   A = diag(sc) W_in, B = diag(sc) W W_in, d = sc * (W b_in), e = sc * (b_in + b) + sh
// (coefficients composed in fp64 by the host, mignn.h).  The [N, H] x0 is
// never materialised: the kernel reads 12-32 B per neighbour instead of a
// 512-B row and writes y once -- an HBM-write-bound pass (N*H*4 bytes).
//
// Layout: a workgroup of 4 gather waves + 4 store waves (below); gather
// lane = row: aggregate (c_i, C_i, s_i) in CSR order into LDS; store role: 32
// lanes x 16 B per row, each lane owning 4 output columns (their 4 x (2D+2)
// coefficients in registers), two rows per store instruction (non-temporal).
#include "common.hpp"

namespace mignn {
namespace {

constexpr int kWaves = 4;

// Split roles: a workgroup of 4 gather waves + 4 store waves walks 256-row
// blocks.  At iteration i the
// gather waves (lane = row, as pass 1 above) aggregate block i into LDS
// buffer i % 2 while the store waves expand and write block i - 1 from the
// other buffer; one barrier per block.  The write stream (N*H*4 bytes, the
// bound) no longer waits behind each wave's three dependent gather round
// trips (row_ptr -> col / ew -> pos) -- 1.52 -> 1.09 ms at 10M nodes against
// the one-role form of round 1.
constexpr int kSplitRows = kWaves * 64;   // rows per block

// a row's D coordinates: V4 (D <= 4, rows padded to 16 B, ldp 4): one 16-B
// load instead of D 4-B loads (the gathers are TA-bound: a quarter of the
// instructions for the same bytes)
template <int D, bool V4>
__device__ __forceinline__ void layer0_pos(const float* __restrict__ pos, int64_t ldp, int64_t r,
                                           float (&p)[D]) {
    if constexpr (V4) {
        const float4 v = ld4(pos + r * 4);
        const float q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int a = 0; a < D; ++a) p[a] = q[a];
    } else {
#pragma unroll
        for (int a = 0; a < D; ++a) p[a] = pos[r * ldp + a];
    }
}

// (c_i, C_i = sum_j w_ij c_j, s_i = sum_j w_ij) of row ri, CSR order (the
// split kernel's gather role and the codes kernel: the same arithmetic)
template <int D, bool V4>
__device__ __forceinline__ void layer0_gather(const int32_t* __restrict__ row_ptr,
                                              const int32_t* __restrict__ col,
                                              const float* __restrict__ ew,
                                              const float* __restrict__ pos, int64_t ldp,
                                              int64_t ri, float (&c)[D], float (&C)[D],
                                              float& sum) {
    sum = 0.f;
    layer0_pos<D, V4>(pos, ldp, ri, c);
#pragma unroll
    for (int a = 0; a < D; ++a) C[a] = 0.f;
    const int32_t e0 = row_ptr[ri], e1 = row_ptr[ri + 1];
    constexpr int kU = 8;
    int32_t jj[kU];
    float ww[kU];
    float pv[kU][D];
    if (e1 > e0) {
        // the first kU entries' loads unconditional, past the row's end
        // clamped to its last entry (valid ids, values unused): no
        // per-entry branches between them -- one round trip per stage
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int32_t ek = e0 + k < e1 ? e0 + k : e1 - 1;
            jj[k] = col[ek];
            ww[k] = ew[ek];
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) layer0_pos<D, V4>(pos, ldp, jj[k], pv[k]);
    } else {
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            jj[k] = 0;
            ww[k] = 0.f;
#pragma unroll
            for (int a = 0; a < D; ++a) pv[k][a] = 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
        if (e0 + k < e1) {
            sum += ww[k];
#pragma unroll
            for (int a = 0; a < D; ++a) C[a] = fmaf(ww[k], pv[k][a], C[a]);
        }
    }
    for (int32_t e = e0 + kU; e < e1; ++e) {
        const int64_t j = col[e];
        const float w = ew[e];
        sum += w;
        float pj[D];
        layer0_pos<D, V4>(pos, ldp, j, pj);
#pragma unroll
        for (int a = 0; a < D; ++a) C[a] = fmaf(w, pj[a], C[a]);
    }
}

template <int D, bool V4 = false>
__global__ __launch_bounds__(2 * kWaves * 64) void gcn_layer0_split_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ pos, int64_t ldp, int64_t row_begin,
    int64_t row_end, const float* __restrict__ coef, int h, float* __restrict__ out,
    int64_t ldo) {
    constexpr int K = 2 * D + 2;
    __shared__ float agg[2][kSplitRows][K];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const bool gather = wave < kWaves;
    const int64_t nrows = row_end - row_begin;
    const int64_t nblk = (nrows + kSplitRows - 1) / kSplitRows;
    // store role: lane owns columns cq .. cq + 3 of rps rows per instruction
    const int cpl = h / 4, rps = 64 / cpl;
    const int sub = lane / cpl, cq = (lane % cpl) * 4;
    const bool active = sub < rps;
    float cf[4][K];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int k = 0; k < K; ++k)
            cf[q][k] = (!gather && active) ? coef[(int64_t)(cq + q) * K + k] : 0.f;
    // blocks b = blockIdx.x + i * gridDim.x; iteration i gathers b_i, stores b_{i-1}
    for (int64_t i = 0;; ++i) {
        const int64_t bg = blockIdx.x + i * (int64_t)gridDim.x;        // gathered now
        const int64_t bs = bg - gridDim.x;                              // stored now
        if (bs >= nblk) break;
        const int buf = static_cast<int>(i & 1);
        if (gather) {
            const int64_t r = bg * kSplitRows + wave * 64 + lane;
            if (bg < nblk && r < nrows) {
                float c[D], C[D], sum;
                layer0_gather<D, V4>(row_ptr, col, ew, pos, ldp, row_begin + r, c, C, sum);
                float* const ag = agg[buf][wave * 64 + lane];
#pragma unroll
                for (int a = 0; a < D; ++a) { ag[a] = c[a]; ag[D + a] = C[a]; }
                ag[2 * D] = sum;
            }
        } else if (bs >= 0) {
            // store wave w - kWaves: rows [64 (w - kWaves), +64) of block bs
            const int64_t base = bs * kSplitRows + (wave - kWaves) * 64;
            const int64_t nb = nrows - base < 64 ? nrows - base : 64;
            const float(*ag)[K] = agg[buf ^ 1] + (wave - kWaves) * 64;
            for (int rr = 0; rr < nb; rr += rps) {
                const int rl = rr + sub;
                if (active && rl < nb) {
                    float v[K - 1];
#pragma unroll
                    for (int k = 0; k < K - 1; ++k) v[k] = ag[rl][k];
                    float o[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float t = cf[q][K - 1];
#pragma unroll
                        for (int k = 0; k < K - 1; ++k) t = fmaf(cf[q][k], v[k], t);
                        o[q] = relu_nan(t);
                    }
                    __builtin_nontemporal_store(
                        f32x4{o[0], o[1], o[2], o[3]},
                        reinterpret_cast<f32x4*>(out + (row_begin + base + rl) * ldo + cq));
                }
            }
        }
        __syncthreads();   // buffer i % 2 filled; buffer (i - 1) % 2 drained
    }
}

// Layer-0 codes (the codes form of the window GCN kernel, gcn_win.hip): per
// row the 8 floats (c_i, C_i, s_i, 0...) -- the values the split kernel's
// store role expands -- instead of the [H] row: 32 B written per row.
template <int D, bool V4 = false>
__global__ __launch_bounds__(256) void gcn_layer0_codes_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ pos, int64_t ldp, int64_t row_begin,
    int64_t row_end, float* __restrict__ codes, int64_t ldc) {
    for (int64_t ri = row_begin + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; ri < row_end;
         ri += (int64_t)gridDim.x * blockDim.x) {
        float c[D], C[D], sum;
        layer0_gather<D, V4>(row_ptr, col, ew, pos, ldp, ri, c, C, sum);
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < D; ++a) { v[a] = c[a]; v[D + a] = C[a]; }
        v[2 * D] = sum;
        float* const o = codes + ri * ldc;
        *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_gcn_layer0_codes(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                      const float* pos, int64_t ldp, int in_dim,
                                      int64_t row_begin, int64_t row_end, float* codes,
                                      int64_t ldc, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && pos && codes, "gcn_layer0_codes: null pointer");
    MIGNN_REQUIRE(in_dim >= 1 && in_dim <= 3, "gcn_layer0_codes: in_dim must be 1..3 (got %d)", in_dim);
    MIGNN_REQUIRE(ldp >= in_dim, "gcn_layer0_codes: ldp < in_dim");
    MIGNN_REQUIRE(ldc % 4 == 0 && ldc >= 8 && aligned16(codes), "gcn_layer0_codes: codes rows must be 16-B aligned, >= 8 wide");
    MIGNN_REQUIRE(row_begin >= 0 && row_end >= row_begin, "gcn_layer0_codes: bad row range");
    if (row_end == row_begin) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    const int64_t blocks = (row_end - row_begin + 255) / 256;
    const unsigned grid = static_cast<unsigned>(blocks < 8192 ? blocks : 8192);
    switch (in_dim) {
    case 1: hipLaunchKernelGGL(gcn_layer0_codes_kernel<1>, dim3(grid), dim3(256), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, codes, ldc); break;
    case 2: hipLaunchKernelGGL(gcn_layer0_codes_kernel<2>, dim3(grid), dim3(256), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, codes, ldc); break;
    default:
        if (ldp == 4 && aligned16(pos))
            hipLaunchKernelGGL((gcn_layer0_codes_kernel<3, true>), dim3(grid), dim3(256), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, codes, ldc);
        else
            hipLaunchKernelGGL(gcn_layer0_codes_kernel<3>, dim3(grid), dim3(256), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, codes, ldc);
        break;
    }
    return launch_status("gcn_layer0_codes_kernel");
}

extern "C" int mignn_gcn_layer0_coords(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                       const float* pos, int64_t ldp, int in_dim,
                                       int64_t row_begin, int64_t row_end, const float* coef,
                                       int h, float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && pos && coef && out, "gcn_layer0: null pointer");
    MIGNN_REQUIRE(in_dim >= 1 && in_dim <= 4, "gcn_layer0: in_dim must be 1..4 (got %d)", in_dim);
    MIGNN_REQUIRE(ldp >= in_dim, "gcn_layer0: ldp < in_dim");
    MIGNN_REQUIRE(h % 4 == 0 && h >= 4 && h <= 256 && (64 % (h / 4)) == 0,
                  "gcn_layer0: h must be 4*2^k <= 256 (got %d)", h);
    MIGNN_REQUIRE(ldo % 4 == 0 && aligned16(out), "gcn_layer0: out rows must be 16-B aligned");
    MIGNN_REQUIRE(row_begin >= 0 && row_end >= row_begin, "gcn_layer0: bad row range");
    if (row_end == row_begin) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    // split roles: 8-wave workgroups, a few 256-row blocks each (2 per CU)
    const int64_t blocks = (row_end - row_begin + kSplitRows - 1) / kSplitRows;
    const unsigned grid = static_cast<unsigned>(blocks < 512 ? blocks : 512);
    switch (in_dim) {
    case 1: hipLaunchKernelGGL(gcn_layer0_split_kernel<1>, dim3(grid), dim3(2 * kWaves * 64), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, coef, h, out, ldo); break;
    case 2: hipLaunchKernelGGL(gcn_layer0_split_kernel<2>, dim3(grid), dim3(2 * kWaves * 64), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, coef, h, out, ldo); break;
    case 3:
        if (ldp == 4 && aligned16(pos))
            hipLaunchKernelGGL((gcn_layer0_split_kernel<3, true>), dim3(grid), dim3(2 * kWaves * 64), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, coef, h, out, ldo);
        else
            hipLaunchKernelGGL(gcn_layer0_split_kernel<3>, dim3(grid), dim3(2 * kWaves * 64), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, coef, h, out, ldo);
        break;
    default: hipLaunchKernelGGL(gcn_layer0_split_kernel<4>, dim3(grid), dim3(2 * kWaves * 64), 0, st, row_ptr, col, ew, pos, ldp, row_begin, row_end, coef, h, out, ldo); break;
    }
    return launch_status("gcn_layer0_split_kernel");
}

