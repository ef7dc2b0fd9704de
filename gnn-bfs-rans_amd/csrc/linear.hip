// Dense node transforms on MFMA (v_mfma_f32_16x16x4_f32: exact fp32, the
// f32 matrix rate of 157 TF on MI355X) with a fused epilogue.
//
//   C[m, n] = epi( sum_k [A | A2][m, k] * W[n, k] )       (torch Linear layout)
//
// Covers nn.Linear in FlowGNN (input_proj gnn_model.py:55 via the VALU kernel
// below, output_proj :90-100, GIN's nn :70-74) and the conv transforms of the
// GAT / TransformerConv paths.
//
// Tiling: 256 threads = 4 waves in a 2x2 arrangement, block tile 64x64, wave
// tile 32x32 = 2x2 MFMA blocks.  K advances in chunks of 16: lane (r, g) =
// (l & 15, l >> 4) loads one float4 of an A row and one float4 of a W row at
// k + 4g; MFMA step u in 0..3 consumes component u, i.e. lane group g feeds
// k = k0 + 4g + u.  A and W use the same k permutation, so the sum is exact
// fp32 over all k (only the association order differs from a CPU GEMM).
// Fragments are loaded straight from global memory (L1/L2-resident weights);
// FlowGNN's layer / head shapes (K, N <= 128) go to the register-resident-W
// persistent kernel in tile_gemm.hip; this kernel covers everything else.
#include "common.hpp"

#include <algorithm>

namespace mignn {
namespace {

constexpr int BM = 64, BN = 64;

__device__ __forceinline__ float4 load_frag(const float* base, int64_t ld, int64_t row,
                                            int64_t rows, int k, int K) {
    if (k >= K) return make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t rr = row < rows ? row : rows - 1;
    return ld4(base + rr * ld + k);
}

__global__ __launch_bounds__(256) void linear_kernel(
    const float* __restrict__ A, int64_t lda, int64_t M, int K1, const float* __restrict__ A2,
    int64_t lda2, int K2, const float* __restrict__ W, int N, const float* __restrict__ bias,
    const float* __restrict__ R, int64_t ldr, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ C, int64_t ldc) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    const int64_t m0 = (int64_t)blockIdx.x * BM + wm * 32;
    const int n0 = blockIdx.y * BN + wn * 32;
    const int ldw = K1 + K2;

    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto run_segment = [&](const float* __restrict__ Aseg, int64_t ldaseg, int Kseg, int wcol0) {
        for (int k0 = 0; k0 < Kseg; k0 += 16) {
            const int k = k0 + 4 * g;
            float4 a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = load_frag(Aseg, ldaseg, m0 + i * 16 + r, M, k, Kseg);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                b[j] = load_frag(W + wcol0, ldw, n0 + j * 16 + r, N, k, Kseg);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = mfma16x16x4(a[i].x, b[j].x, acc[i][j]);
                    acc[i][j] = mfma16x16x4(a[i].y, b[j].y, acc[i][j]);
                    acc[i][j] = mfma16x16x4(a[i].z, b[j].z, acc[i][j]);
                    acc[i][j] = mfma16x16x4(a[i].w, b[j].w, acc[i][j]);
                }
        }
    };
    run_segment(A, lda, K1, 0);
    if (K2 > 0) run_segment(A2, lda2, K2, K1);

#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int col = n0 + j * 16 + r;
        if (col >= N) continue;
        const float bv = (flags & MIGNN_EPI_BIAS) ? bias[col] : 0.f;
        const float sc = (flags & MIGNN_EPI_AFFINE) ? scale[col] : 1.f;
        const float sh = (flags & MIGNN_EPI_AFFINE) ? shift[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = m0 + i * 16 + g * 4 + q;
                if (row >= M) continue;
                const float res = (flags & MIGNN_EPI_RESIDUAL) ? R[row * ldr + col] : 0.f;
                C[row * ldc + col] = epilogue(acc[i][j][q], flags, bv, res, sc, sh);
            }
        }
    }
}

// Linear(in_dim -> h) for in_dim <= 8: thread (row slot, column quad) with
// its 4 W rows and biases in registers; 32-bit index math only (a 64-bit
// div/mod per element made this store-bound kernel 6x slower).
__global__ __launch_bounds__(256) void input_proj_kernel(
    const float* __restrict__ x, int64_t n, int in_dim, const int32_t* __restrict__ rows,
    const float* __restrict__ w, const float* __restrict__ b, int h, float* __restrict__ out,
    int64_t ldo) {
    const int h4 = h >> 2;
    const int rpi = blockDim.x / h4;                 // rows per block iteration
    const int slot = threadIdx.x / h4;
    const int c = (threadIdx.x % h4) * 4;
    if (slot >= rpi) return;
    float wr[4][8], bq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        bq[q] = b[c + q];
#pragma unroll
        for (int k = 0; k < 8; ++k) wr[q][k] = k < in_dim ? w[(c + q) * in_dim + k] : 0.f;
    }
    for (int64_t row = (int64_t)blockIdx.x * rpi + slot; row < n; row += (int64_t)gridDim.x * rpi) {
        float xv[8];
        const int64_t src = rows != nullptr ? static_cast<int64_t>(rows[row]) : row;
#pragma unroll
        for (int k = 0; k < 8; ++k) xv[k] = k < in_dim ? x[src * in_dim + k] : 0.f;
        float o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (k < in_dim) s = fmaf(xv[k], wr[q][k], s);
            o[q] = s + bq[q];
        }
        st4(out + row * ldo + c, make_float4(o[0], o[1], o[2], o[3]));
    }
}

// Narrow transform (n <= 8 output columns, k in {64, 128, 256}, bias / ReLU
// epilogue): GAT's logits [N, 8], the head's last layer.  A row group of
// LPR = k / 4 lanes holds one row (a float4 per lane) and its lanes' float4
// slices of the n weight rows (registers); n partial dots are reduced over
// the group by xor-shuffles.  A pure stream over A -- the tiled MFMA kernel
// spends a whole 16-column tile on n <= 8 (0.23 ms vs ~0.1 ms at 1M x 128).
template <int LPR>
__global__ __launch_bounds__(256) void narrow_linear_kernel(const float* __restrict__ a, int64_t lda,
                                                            int64_t m, int k,
                                                            const float* __restrict__ w, int n,
                                                            const float* __restrict__ bias, int flags,
                                                            float* __restrict__ c, int64_t ldc) {
    constexpr int RPW = 64 / LPR;
    const int lane = static_cast<int>(threadIdx.x & 63);
    const int cl = lane % LPR, grp = lane / LPR;
    f32x4 wv[8];
#pragma unroll
    for (int o = 0; o < 8; ++o)
        wv[o] = o < n ? *reinterpret_cast<const f32x4*>(w + o * k + 4 * cl) : f32x4{0.f, 0.f, 0.f, 0.f};
    const int64_t wave = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 4 * RPW;
    for (int64_t row = wave * RPW + grp; row < m; row += stride) {
        const f32x4 xv = *reinterpret_cast<const f32x4*>(a + row * lda + 4 * cl);
        float v[8];
#pragma unroll
        for (int o = 0; o < 8; ++o) {
            float d = xv[0] * wv[o][0];
            d = fmaf(xv[1], wv[o][1], d);
            d = fmaf(xv[2], wv[o][2], d);
            d = fmaf(xv[3], wv[o][3], d);
            v[o] = d;
        }
#pragma unroll
        for (int off = LPR / 2; off > 0; off >>= 1)
#pragma unroll
            for (int o = 0; o < 8; ++o) v[o] += __shfl_xor(v[o], off);
        if (cl == 0) {
#pragma unroll
            for (int o = 0; o < 8; ++o)
                if (o < n) {
                    float y = v[o];
                    if (flags & MIGNN_EPI_BIAS) y += bias[o];
                    if (flags & MIGNN_EPI_RELU) y = relu_nan(y);
                    c[row * ldc + o] = y;
                }
        }
    }
}

}  // namespace
}  // namespace mignn

using namespace mignn;

static int linear_impl(const float* a, int64_t lda, int64_t m, int k, const float* a2,
                                 int64_t lda2, int k2, const float* w, int n, const float* bias,
                                 const float* residual, int64_t ldr, const float* scale,
                                 const float* shift, int flags, float* c, int64_t ldc,
                                 void* stream);

extern "C" int mignn_linear(const float* a, int64_t lda, int64_t m, int k, const float* a2,
                            int64_t lda2, int k2, const float* w, int n, const float* bias,
                            const float* residual, int64_t ldr, const float* scale,
                            const float* shift, int flags, float* c, int64_t ldc, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "linear: unknown flags 0x%x", flags);
    return linear_impl(a, lda, m, k, a2, lda2, k2, w, n, bias, residual, ldr, scale, shift,
                             flags, c, ldc, stream);
}

static int linear_impl(const float* a, int64_t lda, int64_t m, int k, const float* a2,
                                 int64_t lda2, int k2, const float* w, int n, const float* bias,
                                 const float* residual, int64_t ldr, const float* scale,
                                 const float* shift, int flags, float* c, int64_t ldc,
                                 void* stream) {
    MIGNN_REQUIRE(m >= 0 && k > 0 && k2 >= 0 && n > 0, "linear: bad sizes m=%lld k=%d k2=%d n=%d",
                  (long long)m, k, k2, n);
    MIGNN_REQUIRE(k % 4 == 0 && k2 % 4 == 0, "linear: k=%d k2=%d must be multiples of 4", k, k2);
    MIGNN_REQUIRE(lda % 4 == 0 && (k2 == 0 || lda2 % 4 == 0), "linear: lda not a multiple of 4");
    MIGNN_REQUIRE(a && w && c && aligned16(a) && aligned16(w) && (k2 == 0 || (a2 && aligned16(a2))),
                  "linear: null or unaligned operand");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "linear: bias flag without bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_RESIDUAL) || residual, "linear: residual flag without R");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "linear: affine w/o params");
    if (m == 0) return MIGNN_OK;
    if (k2 == 0 && n <= 8 && (k == 64 || k == 128 || k == 256) &&
        !(flags & (MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE))) {
        const int64_t waves = (m * (k / 4) + 63) / 64;
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>((waves + 3) / 4, 4096));
        hipStream_t st = as_stream(stream);
        switch (k) {
            case 64: narrow_linear_kernel<16><<<grid, 256, 0, st>>>(a, lda, m, k, w, n, bias, flags, c, ldc); break;
            case 128: narrow_linear_kernel<32><<<grid, 256, 0, st>>>(a, lda, m, k, w, n, bias, flags, c, ldc); break;
            default: narrow_linear_kernel<64><<<grid, 256, 0, st>>>(a, lda, m, k, w, n, bias, flags, c, ldc); break;
        }
        return launch_status("narrow_linear_kernel");
    }
    if (k2 == 0) {
        bool handled = false;
        const int rc = tile_linear(a, lda, m, k, w, n, bias, residual, ldr, scale, shift, flags,
                                   c, ldc, as_stream(stream), &handled);
        if (handled) return rc;
    }
    const int64_t gm = (m + BM - 1) / BM;
    MIGNN_REQUIRE(gm < (int64_t(1) << 31), "linear: m too large");
    dim3 grid(static_cast<unsigned>(gm), static_cast<unsigned>((n + BN - 1) / BN));
    hipLaunchKernelGGL(linear_kernel, grid, dim3(256), 0, as_stream(stream), a, lda, m, k, a2,
                       lda2, k2, w, n, bias, residual, ldr, scale, shift, flags, c, ldc);
    return launch_status("linear_kernel");
}

extern "C" int mignn_input_proj(const float* x, int64_t n, int in_dim, const float* w,
                                const float* b, int h, float* out, int64_t ldo, void* stream) {
    return mignn_input_proj_rows(x, n, in_dim, nullptr, w, b, h, out, ldo, stream);
}

extern "C" int mignn_input_proj_rows(const float* x, int64_t n, int in_dim, const int32_t* rows,
                                     const float* w, const float* b, int h, float* out,
                                     int64_t ldo, void* stream) {
    MIGNN_REQUIRE(in_dim > 0 && in_dim <= 8 && h % 4 == 0 && ldo % 4 == 0,
                  "input_proj: in_dim=%d h=%d", in_dim, h);
    MIGNN_REQUIRE(x && w && b && out && aligned16(out), "input_proj: null/unaligned");
    if (n == 0) return MIGNN_OK;
    MIGNN_REQUIRE(h / 4 <= 1024, "input_proj: h too large");
    const int h4 = h / 4;
    const int block = h4 >= 256 ? h4 : (256 / h4) * h4;
    const int64_t rpi = block / h4;
    hipLaunchKernelGGL(input_proj_kernel, dim3(grid_for((n + rpi - 1) / rpi, 1, 16384)),
                       dim3(block), 0, as_stream(stream), x, n, in_dim, rows, w, b, h, out, ldo);
    return launch_status("input_proj_kernel");
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_linear(const float* a, int64_t lda, int64_t m, int k, const float* a2,
                                 int64_t lda2, int k2, const float* w, int n, const float* bias,
                                 const float* residual, int64_t ldr, const float* scale,
                                 const float* shift, int flags, float* c, int64_t ldc,
                                 void* stream) {
    return linear_impl(a, lda, m, k, a2, lda2, k2, w, n, bias, residual, ldr, scale, shift, flags, c, ldc, stream);
}
#endif
