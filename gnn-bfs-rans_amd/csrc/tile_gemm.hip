// Persistent row-tile GEMM with a fused A-tile producer and epilogue:
//
//   out[i, :] = epi( A_i . W^T ),   A_i = one of
//     AGG_GCN : sum_{j in row i} dinv_j dinv_i x_j          (GCNConv, gnn_model.py:63)
//     AGG_SUM : sum_{j in row i} x_j + (1 + eps) x_i         (GINConv, gnn_model.py:70-75)
//     ROWS    : a[i, :]                                      (nn.Linear)
//   epi = +bias -> +residual -> *scale+shift (BatchNorm eval) -> ReLU (flags).
//
// The AGG_GCN instance is the north-star hot kernel: GCNConv + residual +
// BatchNorm + ReLU of one layer (gnn_model.py:166, :184-191) in ONE pass over
// HBM -- every x row is gathered and every output row written once; the
// aggregate-then-transform order (A x) W^T == A (x W^T) needs no [N, H]
// intermediate.
//
// Workgroup = 8 waves (512 threads), row tile BM = 64, two workgroups per CU
// (4 waves per SIMD, <= 128 VGPRs), persistent grid = CUs x 2 (multiple of 8):
//   * Every wave owns 8 rows of the tile for the gather and a 16-column (or
//     WROWS x 16) slice of the output for the MFMA; its slice of W lives in
//     VGPRs for the whole launch (32 VGPRs at K = 128).
//   * CSR indices never touch LDS: lanes 0..8 hold the wave's row_ptr, lane t
//     holds the t-th (neighbour id, dinv_j) of the wave's rows; row groups
//     fetch them with ds_bpermute.  The next tile's indices are loaded while
//     this tile's MFMAs run, so a tile costs only its x-row round trips
//     (2 at K = 128: 16 neighbour rows in flight per row group).
//   * Gathered rows are summed in CSR order (== edge_index order): bitwise
//     deterministic.  The aggregated tile goes to LDS [64][K+8] (row stride
//     8 mod 64 floats: conflict-free quad-interleaved ds_read_b128).
//   * MFMA v_mfma_f32_16x16x4_f32 (exact fp32): lane (r, g) = (l & 15, l >> 4)
//     reads A[16 ib + r][16 kc + 4g .. +3] and feeds k = 16 kc + 4g + u at step
//     u -- the permutation its W registers were loaded in; the IB accumulator
//     chains are interleaved so back-to-back MFMAs are independent.
//   * Epilogue from the accumulators (residual prefetched before the MFMAs):
//     each store instruction writes 4 rows x 64 B.
//   * XCD-aware tile order: at step t the chip covers tiles [tG, (t+1)G); the
//     workgroups of XCD group x = blockIdx % 8 take one contiguous run of G/8
//     tiles, so the +-1 / +-row neighbours a run gathers share that XCD's L2
//     and the chip sweeps a single front (+-plane neighbours stay in the
//     256 MB Infinity Cache).
#include "common.hpp"

namespace mignn {
namespace {

constexpr int BM = 64;
constexpr int NW = 8;               // waves per workgroup
constexpr int NTHREADS = NW * 64;
constexpr int GROWS = BM / NW;      // rows gathered per wave (8)

enum { AGG_GCN = 0, AGG_SUM = 1, ROWS = 2 };

template <int K, int N, int MODE>
struct Cfg {
    static_assert(K % 16 == 0 && K <= 256, "K in 16..256, multiple of 16");
    static constexpr int WN = N / 16 < NW ? N / 16 : NW;   // column slices
    static constexpr int WM_ = NW / WN;
    static constexpr int WM = WM_ > 4 ? 4 : WM_;           // row slices (>= 16 rows each)
    static constexpr int MW = WM * WN;                     // waves doing MFMA
    static constexpr int WROWS = BM / WM;
    static constexpr int WCOLS = N / WN;
    static_assert(WCOLS % 16 == 0 && WROWS % 16 == 0, "wave tile must be 16-aligned");
    static constexpr int IB = WROWS / 16;
    static constexpr int JB = WCOLS / 16;
    static constexpr int KC = K / 16;
    static constexpr int LPR = K / 4;                      // lanes per A row (16 B each)
    static constexpr int RPW = 64 / LPR;                   // rows per wave instruction
    static constexpr int RSTEPS = GROWS / RPW;             // row steps per wave
    static constexpr int RIF = (RSTEPS < 2 || K > 64 || MODE == AGG_GCN) ? 1 : 2;   // VGPR cap 128
    static constexpr int A_LD = K + 8;
    static constexpr int A_FLOATS = BM * A_LD;
};

struct WaveIdx {        // CSR indices of a wave's 8 rows, in lane registers
    int rp;             // lanes 0..8: row_ptr[r0 + lane] (clamped)
    float dr;           // lanes 0..7: dinv[r0 + lane]
    int j;              // lane t < ne: col[e0 + t]
    float dj;           // lane t < ne: dinv[col[e0 + t]]
};

template <int MODE>
__device__ __forceinline__ void load_rp(WaveIdx& w, const int32_t* __restrict__ row_ptr,
                                        const float* __restrict__ dinv, int64_t r0,
                                        int64_t row_end, int lane) {
    const int64_t rr = r0 + lane < row_end ? r0 + lane : row_end;
    w.rp = lane <= GROWS ? row_ptr[rr] : 0;
    w.dr = (MODE == AGG_GCN && lane < GROWS && r0 + lane < row_end) ? dinv[r0 + lane] : 0.f;
}

template <int MODE>
__device__ __forceinline__ void load_cols(WaveIdx& w, const int32_t* __restrict__ col,
                                          const float* __restrict__ dinv, int lane) {
    const int e0 = __shfl(w.rp, 0, 64);
    const int ne = __shfl(w.rp, GROWS, 64) - e0;
    w.j = lane < ne ? col[e0 + lane] : 0;
    w.dj = 1.f;
    if constexpr (MODE == AGG_GCN) w.dj = lane < ne ? dinv[w.j] : 0.f;
}

template <int K, int N, int MODE>
__global__ __launch_bounds__(NTHREADS, 4) void fused_tile_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ dinv, float self_scale, const float* __restrict__ x, int64_t ldx,
    int64_t row_begin, int64_t row_end, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ R, int64_t ldr,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags, int n_valid,
    float* __restrict__ out, int64_t ldo) {
    using C = Cfg<K, N, MODE>;
    __shared__ __attribute__((aligned(16))) float A[C::A_FLOATS];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // SGPR: uniform bases below

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + BM - 1) / BM;
    const int G = gridDim.x;            // multiple of 8 (host guarantees)
    const int xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3;
    const int per_xcd = G >> 3;
    auto tile_of = [&](int64_t s) -> int64_t { return s * G + (int64_t)xcd * per_xcd + slot; };

    // MFMA role
    const bool mw = wave < C::MW;
    const int r = lane & 15, g = lane >> 4;
    const int wm = wave / C::WN, wn = wave % C::WN;
    float4 breg[C::JB][C::KC];
#pragma unroll
    for (int jb = 0; jb < C::JB; ++jb) {
        const int n = wn * C::WCOLS + jb * 16 + r;
        const bool ok = mw && n < n_valid;
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc)
            breg[jb][kc] = ok ? ld4(W + (int64_t)n * K + kc * 16 + 4 * g)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
    }

    WaveIdx idx{0, 0.f, 0, 0.f};
    int64_t tile = tile_of(0);
    if (MODE != ROWS && tile < ntiles) {
        const int64_t r0 = row_begin + tile * BM + wave * GROWS;
        load_rp<MODE>(idx, row_ptr, dinv, r0, row_end, lane);
        load_cols<MODE>(idx, col, dinv, lane);
    }

    for (int64_t s = 0; tile < ntiles; ++s) {
        // Opaque per-iteration copies of the lane coordinates: stops LICM from
        // hoisting dozens of lane-dependent address offsets out of the tile
        // loop (they would pin VGPRs for the whole launch and spill at the
        // 128-VGPR cap of two workgroups per CU).
        int lane_ = lane;
        asm volatile("" : "+v"(lane_));
        const int r = lane_ & 15, g = lane_ >> 4;
        const int c = lane_ % C::LPR;
        const int grp = lane_ / C::LPR;
        const int64_t t0 = row_begin + tile * BM;
        const int64_t r0 = t0 + wave * GROWS;          // first gathered row of this wave

        // ------------------------------------------------ A tile -> LDS
        if constexpr (MODE == ROWS) {
            constexpr int CH = GROWS * C::LPR;                 // 16-B chunks per wave
            constexpr int NQ = (CH + 63) / 64;
            float4 v[NQ];
            const float* xb = x + r0 * ldx;                    // uniform base, 32-bit offsets
            const int nr = static_cast<int>(row_end - r0 < GROWS ? row_end - r0 : GROWS);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int id = q * 64 + lane_;
                const int lr = id / C::LPR, cc = id % C::LPR;
                v[q] = (id < CH && lr < nr) ? ld4(xb + (lr * static_cast<int>(ldx) + 4 * cc))
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int id = q * 64 + lane_;
                const int lr = id / C::LPR, cc = id % C::LPR;
                if (id < CH) st4(&A[(wave * GROWS + lr) * C::A_LD + 4 * cc], v[q]);
            }
        } else {
            const int e0 = __shfl(idx.rp, 0, 64);
            const int ne = __shfl(idx.rp, GROWS, 64) - e0;
            const bool in_regs = ne <= 64;                     // wave-uniform
            // Wave-uniform edge-loop bound: the ids live in lanes across the
            // whole wave, so every lane must stay in the loop while any row
            // group still reads them through ds_bpermute.
            int dmax = lane_ < GROWS ? __shfl(idx.rp, lane_ + 1, 64) - idx.rp : 0;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) dmax = max(dmax, __shfl_xor(dmax, o, 64));
#pragma unroll 1
            for (int st = 0; st < C::RSTEPS; st += C::RIF) {
                int lrow[C::RIF], beg[C::RIF], deg[C::RIF];
                float di[C::RIF];
                float4 acc[C::RIF];
#pragma unroll
                for (int q = 0; q < C::RIF; ++q) {
                    lrow[q] = (st + q) * C::RPW + grp;         // row inside the wave slice
                    const int b = __shfl(idx.rp, lrow[q], 64);
                    beg[q] = b - e0;
                    deg[q] = __shfl(idx.rp, lrow[q] + 1, 64) - b;
                    di[q] = __shfl(idx.dr, lrow[q], 64);
                    acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                for (int u0 = 0; u0 < dmax; u0 += 8) {
                    float4 v[C::RIF][8];
                    float w[C::RIF][8];
#pragma unroll
                    for (int q = 0; q < C::RIF; ++q)
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            const bool ok = u0 + u < deg[q];
                            const int e = beg[q] + (ok ? u0 + u : 0);
                            int jj;
                            float dj;
                            if (in_regs) {
                                jj = __shfl(idx.j, e, 64);
                                dj = __shfl(idx.dj, e, 64);
                            } else {
                                jj = col[e0 + e];
                                dj = MODE == AGG_GCN ? dinv[jj] : 1.f;
                            }
                            // PyG gcn_norm: dinv[src] * 1 * dinv[dst]
                            w[q][u] = ok ? (MODE == AGG_GCN ? dj * di[q] : 1.f) : 0.f;
                            v[q][u] = ok ? ld4(x + (int64_t)jj * ldx + 4 * c)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
                        }
#pragma unroll
                    for (int q = 0; q < C::RIF; ++q)
#pragma unroll
                        for (int u = 0; u < 8; ++u) {
                            if (u0 + u < deg[q]) {
                                if constexpr (MODE == AGG_GCN) {
                                    acc[q] = fma4(w[q][u], v[q][u], acc[q]);
                                } else {
                                    acc[q].x += v[q][u].x; acc[q].y += v[q][u].y;
                                    acc[q].z += v[q][u].z; acc[q].w += v[q][u].w;
                                }
                            }
                        }
                }
#pragma unroll
                for (int q = 0; q < C::RIF; ++q) {
                    const int64_t row = r0 + lrow[q];
                    if constexpr (MODE == AGG_SUM) {
                        // GINConv: out = sum_j x_j; out = out + (1 + eps) * x_i
                        if (row < row_end) {
                            const float4 xi = ld4(x + row * ldx + 4 * c);
                            acc[q].x = acc[q].x + self_scale * xi.x;
                            acc[q].y = acc[q].y + self_scale * xi.y;
                            acc[q].z = acc[q].z + self_scale * xi.z;
                            acc[q].w = acc[q].w + self_scale * xi.w;
                        }
                    }
                    st4(&A[(wave * GROWS + lrow[q]) * C::A_LD + 4 * c], acc[q]);
                }
            }
        }
        __syncthreads();

        // next tile's CSR indices: row_ptr now, neighbour ids after the MFMAs
        const int64_t tile_next = tile_of(s + 1);
        if (MODE != ROWS && tile_next < ntiles)
            load_rp<MODE>(idx, row_ptr, dinv, row_begin + tile_next * BM + wave * GROWS, row_end,
                          lane);

        if (mw) {
            // residual prefetch: D[row = 4g + q][col = r] of every (ib, jb)
            const int64_t m0 = t0 + wm * C::WROWS;            // uniform
            const int mr = static_cast<int>(row_end - m0 < C::WROWS ? row_end - m0 : C::WROWS);
            float res[C::IB][C::JB][4];
            const float* Rb = (flags & MIGNN_EPI_RESIDUAL) ? R + m0 * ldr : nullptr;
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = ib * 16 + 4 * g + q;
                        const int n = wn * C::WCOLS + jb * 16 + r;
                        res[ib][jb][q] = (Rb && lr < mr && n < n_valid)
                                             ? Rb[lr * static_cast<int>(ldr) + n] : 0.f;
                    }
            f32x4 accm[C::IB][C::JB];
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) accm[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                float4 a[C::IB];
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib)
                    a[ib] = *reinterpret_cast<const float4*>(
                        &A[(wm * C::WROWS + ib * 16 + r) * C::A_LD + kc * 16 + 4 * g]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) accm[ib][jb] = mfma16x16x4(a[ib].x, breg[jb][kc].x, accm[ib][jb]);
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) accm[ib][jb] = mfma16x16x4(a[ib].y, breg[jb][kc].y, accm[ib][jb]);
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) accm[ib][jb] = mfma16x16x4(a[ib].z, breg[jb][kc].z, accm[ib][jb]);
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) accm[ib][jb] = mfma16x16x4(a[ib].w, breg[jb][kc].w, accm[ib][jb]);
                }
                // keep the A fragments of one k-chunk live at a time (VGPR cap 128)
                __builtin_amdgcn_sched_barrier(0);
            }
            // epilogue straight from the accumulators
#pragma unroll
            for (int jb = 0; jb < C::JB; ++jb) {
                const int n = wn * C::WCOLS + jb * 16 + r;
                if (n >= n_valid) continue;
                const float bv = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
                const float sc = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
                const float sh = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
                float* ob = out + m0 * ldo;
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = ib * 16 + 4 * g + q;
                        if (lr < mr)
                            ob[lr * static_cast<int>(ldo) + n] =
                                epilogue(accm[ib][jb][q], flags, bv, res[ib][jb][q], sc, sh);
                    }
            }
        }
        if (MODE != ROWS && tile_next < ntiles) load_cols<MODE>(idx, col, dinv, lane);
        __syncthreads();
        tile = tile_next;
    }
}

struct TileArgs {
    const int32_t* row_ptr; const int32_t* col; const float* dinv; float self_scale;
    const float* x; int64_t ldx; int64_t rb, re;
    const float* W; const float* bias; const float* R; int64_t ldr;
    const float* scale; const float* shift; int flags; int n_valid; float* out; int64_t ldo;
};

template <int K, int N, int MODE>
int launch_tile(const TileArgs& a, hipStream_t st) {
    auto kern = fused_tile_kernel<K, N, MODE>;
    static int grid_cache[64] = {0};
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& G = grid_cache[dev & 63];
    if (G == 0) {
        int cus = 0, per_cu = 0;
        MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        MIGNN_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NTHREADS, 0));
        if (per_cu < 1) per_cu = 1;
        G = ((cus * per_cu) / 8) * 8;
        if (G < 8) G = 8;
    }
    const int64_t ntiles = (a.re - a.rb + BM - 1) / BM;
    int grid = G;
    if (ntiles < grid) grid = static_cast<int>(((ntiles + 7) / 8) * 8);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHREADS), 0, st, a.row_ptr, a.col, a.dinv,
                       a.self_scale, a.x, a.ldx, a.rb, a.re, a.W, a.bias, a.R, a.ldr, a.scale,
                       a.shift, a.flags, a.n_valid, a.out, a.ldo);
    return launch_status("fused_tile_kernel");
}

// Instances: (K, N) shapes of FlowGNN at hidden 64 / 128 (layers and output MLP).
template <int MODE>
int dispatch_tile(int K, int N, const TileArgs& a, hipStream_t st) {
#define MIGNN_TILE(KK, NN) \
    if (K == KK && N == NN) return launch_tile<KK, NN, MODE>(a, st);
    MIGNN_TILE(128, 128)
    MIGNN_TILE(64, 64)
    if constexpr (MODE == ROWS) {
        MIGNN_TILE(128, 64)
        MIGNN_TILE(64, 32)
        MIGNN_TILE(64, 16)
        MIGNN_TILE(32, 16)
    }
#undef MIGNN_TILE
    set_error("tile GEMM: no instance for K=%d N=%d", K, N);
    return MIGNN_ERR_UNSUPPORTED;
}

bool tile_supported(int mode, int K, int N) {
    if (K == N && (K == 64 || K == 128)) return true;
    if (mode != ROWS) return false;
    return (K == 128 && N == 64) || (K == 64 && N == 32) || (K == 64 && N == 16) ||
           (K == 32 && N == 16);
}

}  // namespace

// Used by linear.hip: register-resident-W path for the FlowGNN head shapes.
int tile_linear(const float* a, int64_t lda, int64_t m, int k, const float* w, int n,
                const float* bias, const float* residual, int64_t ldr, const float* scale,
                const float* shift, int flags, float* c, int64_t ldc, hipStream_t st,
                bool* handled) {
    *handled = false;
    const int npad = n < 16 ? 16 : n;
    if (!tile_supported(ROWS, k, npad) || !aligned16(a) || !aligned16(w) || (lda & 3)) return 0;
    *handled = true;
    TileArgs t{nullptr, nullptr, nullptr, 0.f, a, lda, 0, m, w, bias, residual, ldr,
               scale, shift, flags, n, c, ldc};
    return dispatch_tile<ROWS>(k, npad, t, st);
}

}  // namespace mignn

using namespace mignn;

extern "C" int mignn_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                               const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                               const float* w, const float* bias, const float* scale,
                               const float* shift, int flags, float* out, int64_t ldo,
                               void* stream) {
    MIGNN_REQUIRE(row_ptr && col && dinv && x && w && out, "gcn_layer: null pointer");
    MIGNN_REQUIRE(aligned16(x) && aligned16(w), "gcn_layer: unaligned x / w");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldx >= h && ldo >= h, "gcn_layer: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer: affine params");
    MIGNN_REQUIRE(x != out, "gcn_layer: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    if (!tile_supported(AGG_GCN, h, h)) {
        set_error("gcn_layer: fused kernel supports h in {64,128} (got %d); use "
                  "mignn_gcn_aggregate + mignn_linear", h);
        return MIGNN_ERR_UNSUPPORTED;
    }
    TileArgs t{row_ptr, col, dinv, 1.f, x, ldx, rb, re, w, bias, x, ldx, scale, shift, flags, h,
               out, ldo};
    return dispatch_tile<AGG_GCN>(h, h, t, as_stream(stream));
}

extern "C" int mignn_gin_layer(const int32_t* row_ptr, const int32_t* col, const float* x,
                               int64_t ldx, int64_t rb, int64_t re, int h, float eps,
                               const float* w1, const float* b1, const float* w2,
                               const float* b2, const float* scale, const float* shift, int flags,
                               float* tmp, int64_t ldt, float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && x && w1 && b1 && w2 && b2 && tmp && out,
                  "gin_layer: null pointer");
    MIGNN_REQUIRE(aligned16(x) && aligned16(tmp) && aligned16(w1) && aligned16(w2),
                  "gin_layer: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldt % 4 == 0, "gin_layer: bad strides");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gin_layer: affine params");
    MIGNN_REQUIRE(x != out && tmp != x, "gin_layer: aliasing");
    if (re == rb) return MIGNN_OK;
    if (!tile_supported(AGG_SUM, h, h)) {
        set_error("gin_layer: fused kernel supports h in {64,128} (got %d)", h);
        return MIGNN_ERR_UNSUPPORTED;
    }
    hipStream_t st = as_stream(stream);
    // h1 = relu(nn.0(sum_j x_j + (1+eps) x_i)) for rows [rb, re) -> tmp rows [0, re-rb)
    TileArgs t1{row_ptr, col, nullptr, 1.f + eps, x, ldx, rb, re, w1, b1, nullptr, 0, nullptr,
                nullptr, MIGNN_EPI_BIAS | MIGNN_EPI_RELU, h, tmp - rb * ldt, ldt};
    int rc = dispatch_tile<AGG_SUM>(h, h, t1, st);
    if (rc) return rc;
    // out = epi(nn.2(h1)) with residual x (gnn_model.py:184-191)
    TileArgs t2{nullptr, nullptr, nullptr, 0.f, tmp - rb * ldt, ldt, rb, re, w2, b2, x, ldx,
                scale, shift, flags, h, out, ldo};
    return dispatch_tile<ROWS>(h, h, t2, st);
}
