// Fused GCN layer -- the north-star hot kernel.
//
//   out_i = relu( (x_i + (sum_{j in row i} dinv_j dinv_i x_j) W^T + b) * scale + shift )
//
// = GCNConv (gnn_model.py:63, :166; PyG gcn_norm with one self-loop per node)
// + residual (:184) + BatchNorm eval (:188) + ReLU (:191), in ONE pass over
// HBM: every x row is read (gathered) and every out row written once; the
// aggregate-then-transform order (A x) W^T == A (x W^T) needs no [N, H]
// intermediate.
//
// Structure (persistent; 256 threads = 4 waves; row tile BM = 64):
//   * Each wave owns H/4 output columns; its slice of W (H/4 x H fp32) lives
//     in VGPRs for the whole launch (64 VGPRs at H = 128), loaded once.
//   * Gather: a row group of H/4 lanes (float4 per lane) owns one destination
//     row; the row's neighbour ids and gcn weights are fetched by the group's
//     lanes in one coalesced load and broadcast with ds_bpermute, then up to
//     8 neighbour rows are in flight per group.  The aggregated row is
//     written to an LDS tile [64][H+8] (row stride = 8 mod 64 floats: the
//     quad-interleaved ds_read_b128 pattern below is bank-conflict free).
//   * Transform: MFMA f32 16x16x4.  Lane (r, g) = (l & 15, l >> 4) reads
//     A[16 ib + r][16 kc + 4g .. +3] (ds_read_b128) and feeds k = 16 kc + 4g + u
//     at MFMA step u -- the same permutation its W registers were loaded in.
//   * Epilogue: accumulators are staged through LDS (stride H+4: conflict-free
//     ds_write_b32) and written back as whole 16-B-per-lane rows with the
//     bias / residual / BN affine / ReLU applied on the way out.
//   * Tile order is XCD-aware: the grid is a multiple of 8 and at step t the
//     chip covers tiles [t G, (t+1) G); XCD group x (= blockIdx % 8) takes a
//     contiguous run of G/8 tiles, so the +-1 and +-plane-row neighbours a
//     run gathers stay in that XCD's L2 and the whole chip sweeps one front
//     (the +-k-plane neighbours stay in the 256 MB Infinity Cache).
#include "common.hpp"

namespace mignn {
namespace {

constexpr int BM = 64;
constexpr int NTHREADS = 256;

template <int H>
struct GcnCfg {
    static constexpr int LPR = H / 4;               // lanes per gathered row
    static constexpr int RPW = 64 / LPR;            // rows per wave per gather step
    static constexpr int COLS = H / 4;              // output columns per wave
    static constexpr int JB = COLS / 16;            // 16-wide MFMA column blocks per wave
    static constexpr int KC = H / 16;               // 16-deep k chunks
    static constexpr int A_LD = H + 8;              // LDS A-tile row stride (floats)
    static constexpr int O_LD = H + 4;              // LDS out-tile row stride (floats)
    static constexpr int LDS_FLOATS = BM * A_LD;
    static_assert(H == 64 || H == 128, "register-resident W variant: H in {64, 128}");
};

template <int H>
__global__ __launch_bounds__(NTHREADS, 3) void gcn_layer_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ dinv, const float* __restrict__ x, int64_t ldx, int64_t row_begin,
    int64_t row_end, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo) {
    using C = GcnCfg<H>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;

    // ---- W slice -> registers (k permutation: chunk kc, lane group g -> k = 16kc + 4g + u)
    float4 breg[C::JB][C::KC];
#pragma unroll
    for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc)
            breg[jb][kc] = ld4(W + (int64_t)(wave * C::COLS + jb * 16 + r) * H + kc * 16 + 4 * g);

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + BM - 1) / BM;
    const int G = gridDim.x;          // multiple of 8 (host guarantees)
    const int xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3;
    const int per_xcd = G >> 3;

    // gather geometry
    const int grp = lane / C::LPR;        // row group inside the wave
    const int c = lane % C::LPR;          // float4 chunk owned by this lane
    const int grp_base = grp * C::LPR;    // first lane of the group

    for (int64_t step = 0;; ++step) {
        const int64_t tile = step * G + (int64_t)xcd * per_xcd + slot;
        if (step * G >= ntiles) break;
        const bool active = tile < ntiles;   // uniform per workgroup
        const int64_t t0 = row_begin + tile * BM;

        // ------------------------------------------------ gather -> LDS A tile
        if (active) {
            for (int rr = wave * (BM / 4); rr < (wave + 1) * (BM / 4); rr += C::RPW) {
                const int lr = rr + grp;
                const int64_t row = t0 + lr;
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                if (row < row_end) {
                    const int beg = row_ptr[row];
                    const int deg = row_ptr[row + 1] - beg;
                    const float di = dinv[row];
                    for (int base = 0; base < deg; base += C::LPR) {
                        int jj = static_cast<int>(row);
                        float ww = 0.f;
                        if (base + c < deg) {
                            jj = col[beg + base + c];
                            ww = dinv[jj] * di;   // PyG: dinv[src] * 1 * dinv[dst]
                        }
                        const int n = min(C::LPR, deg - base);
                        for (int u0 = 0; u0 < n; u0 += 8) {
                            int j[8];
                            float w[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int srcl = grp_base + min(u0 + u, C::LPR - 1);
                                j[u] = __shfl(jj, srcl, 64);
                                w[u] = __shfl(ww, srcl, 64);
                            }
                            float4 v[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) v[u] = ld4(x + (int64_t)j[u] * ldx + 4 * c);
#pragma unroll
                            for (int u = 0; u < 8; ++u)
                                if (u0 + u < n) acc = fma4(w[u], v[u], acc);
                        }
                    }
                }
                st4(&lds[lr * C::A_LD + 4 * c], acc);
            }
        }
        __syncthreads();

        // ------------------------------------------------ MFMA transform
        f32x4 accm[4][C::JB];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
            for (int jb = 0; jb < C::JB; ++jb) accm[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (active) {
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                float4 a[4];
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
                    a[ib] = *reinterpret_cast<const float4*>(&lds[(ib * 16 + r) * C::A_LD + kc * 16 + 4 * g]);
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                    for (int jb = 0; jb < C::JB; ++jb) {
                        accm[ib][jb] = mfma16x16x4(a[ib].x, breg[jb][kc].x, accm[ib][jb]);
                        accm[ib][jb] = mfma16x16x4(a[ib].y, breg[jb][kc].y, accm[ib][jb]);
                        accm[ib][jb] = mfma16x16x4(a[ib].z, breg[jb][kc].z, accm[ib][jb]);
                        accm[ib][jb] = mfma16x16x4(a[ib].w, breg[jb][kc].w, accm[ib][jb]);
                    }
            }
        }
        __syncthreads();

        // ------------------------------------------------ stage accumulators in LDS
        if (active) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        lds[(ib * 16 + 4 * g + q) * C::O_LD + wave * C::COLS + jb * 16 + r] =
                            accm[ib][jb][q];
        }
        __syncthreads();

        // ------------------------------------------------ fused epilogue, whole-row stores
        if (active) {
            constexpr int H4 = H / 4;
            for (int idx = tid; idx < BM * H4; idx += NTHREADS) {
                const int lr = idx / H4;
                const int c4 = idx % H4;
                const int64_t row = t0 + lr;
                if (row >= row_end) continue;
                float4 v = *reinterpret_cast<const float4*>(&lds[lr * C::O_LD + 4 * c4]);
                float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f), r4 = b4, s4 = make_float4(1.f, 1.f, 1.f, 1.f), h4 = b4;
                if (flags & MIGNN_EPI_BIAS) b4 = ld4(bias + 4 * c4);
                if (flags & MIGNN_EPI_RESIDUAL) r4 = ld4(x + row * ldx + 4 * c4);
                if (flags & MIGNN_EPI_AFFINE) { s4 = ld4(scale + 4 * c4); h4 = ld4(shift + 4 * c4); }
                v.x = epilogue(v.x, flags, b4.x, r4.x, s4.x, h4.x);
                v.y = epilogue(v.y, flags, b4.y, r4.y, s4.y, h4.y);
                v.z = epilogue(v.z, flags, b4.z, r4.z, s4.z, h4.z);
                v.w = epilogue(v.w, flags, b4.w, r4.w, s4.w, h4.w);
                st4(out + row * ldo + 4 * c4, v);
            }
        }
        __syncthreads();
    }
}

template <int H>
int launch_gcn(const int32_t* row_ptr, const int32_t* col, const float* dinv, const float* x,
               int64_t ldx, int64_t rb, int64_t re, const float* W, const float* bias,
               const float* scale, const float* shift, int flags, float* out, int64_t ldo,
               hipStream_t st) {
    static int grid_cache[64] = {0};
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& G = grid_cache[dev & 63];
    if (G == 0) {
        int cus = 0, per_cu = 0;
        MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        MIGNN_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gcn_layer_kernel<H>,
                                                                NTHREADS, 0));
        if (per_cu < 1) per_cu = 1;
        G = ((cus * per_cu) / 8) * 8;
        if (G < 8) G = 8;
    }
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    int grid = G;
    if (ntiles < grid) grid = static_cast<int>(((ntiles + 7) / 8) * 8);
    hipLaunchKernelGGL(gcn_layer_kernel<H>, dim3(grid), dim3(NTHREADS), 0, st, row_ptr, col, dinv,
                       x, ldx, rb, re, W, bias, scale, shift, flags, out, ldo);
    return launch_status("gcn_layer_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                               const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                               const float* w, const float* bias, const float* scale,
                               const float* shift, int flags, float* out, int64_t ldo,
                               void* stream) {
    MIGNN_REQUIRE(row_ptr && col && dinv && x && w && out, "gcn_layer: null pointer");
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(w), "gcn_layer: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "gcn_layer: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || (bias && aligned16(bias)), "gcn_layer: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift && aligned16(scale) &&
                                                  aligned16(shift)),
                  "gcn_layer: affine params");
    MIGNN_REQUIRE(x != out, "gcn_layer: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    switch (h) {
        case 64: return launch_gcn<64>(row_ptr, col, dinv, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 128: return launch_gcn<128>(row_ptr, col, dinv, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        default:
            set_error("gcn_layer: fused kernel supports h in {64,128} (got %d); use "
                      "mignn_gcn_aggregate + mignn_linear", h);
            return MIGNN_ERR_UNSUPPORTED;
    }
}
