// Persistent, wave-specialized row-tile GEMM with a fused A-tile producer and
// epilogue:
//
//   out[i, :] = epi( A_i . W^T ),   A_i = one of
//     AGG_GCN : sum_{e in row i} w_e x_{col e}     w_e = dinv_src dinv_dst  (GCNConv, gnn_model.py:63)
//     AGG_SUM : sum_{e in row i} x_{col e} + (1 + eps) x_i              (GINConv, gnn_model.py:70-75)
//     ROWS    : a[i, :]                                                 (nn.Linear)
//   epi = +bias -> +residual -> *scale+shift (BatchNorm eval) -> ReLU (flags).
//
// The AGG_GCN instance is the north-star hot kernel: GCNConv + residual +
// BatchNorm + ReLU of one layer (gnn_model.py:166, :184-191) in ONE pass over
// HBM -- every x row is gathered and every output row written once; the
// aggregate-then-transform order (A x) W^T == A (x W^T) needs no [N, H]
// intermediate.
//
// One 12-wave workgroup per CU (persistent, grid = #CUs rounded to 8), row
// tile BM = 64, one barrier per tile:
//   * waves 4..11 PRODUCE tile s+1 into LDS buffer (s+1)&1 while waves 0..3
//     CONSUME tile s from buffer s&1 -- gather latency and MFMA overlap inside
//     the workgroup (measured: two co-resident workgroups that each alternate
//     gather and MFMA phases run in lockstep and overlap nothing).  A
//     producer keeps all 32 neighbour rows of its slice in flight: the gather
//     is bound by bytes in flight (Infinity-Cache latency x rate), not issue.
//   * producer wave p owns rows 8p..8p+7.  Its CSR indices never touch LDS:
//     lanes 0..8 hold row_ptr, lane t holds entry t (and t+64) of the rows'
//     (column id, edge weight) -- fetched by ds_bpermute.  The index chain is
//     pipelined: row_ptr of tile s+3 and the entries of tile s+2 load during
//     the gather of tile s+1, so a tile costs its x-row round trips only.
//     Rows are summed in CSR order (== edge_index order): bitwise
//     deterministic.  A row group of K/4 lanes (16 B per lane) owns one row.
//   * consumer waves (WM x WN) hold nothing big in registers: W [N, K] is
//     staged in LDS once per launch; A and B fragments are read with
//     ds_read_b128 from row stride K+8 (= 8 mod 64 floats: the
//     quad-interleaved pattern is bank-conflict free).  MFMA is
//     v_mfma_f32_16x16x4_f32 (exact fp32); lane (r, g) = (l & 15, l >> 4)
//     feeds k = 16 kc + 4g + u at step u for both operands.  The residual is
//     prefetched before the MFMAs; the epilogue runs from the accumulators
//     with non-temporal stores (the 5 GB of output must not evict x rows).
//   * XCD-aware tile order: at step t the chip covers tiles [tG, (t+1)G); the
//     workgroups of XCD group x = blockIdx % 8 take one contiguous run of G/8
//     tiles, so the +-1 / +-row neighbours a run gathers share that XCD's L2
//     and the chip sweeps a single front (+-plane neighbours stay in the
//     256 MB Infinity Cache).
#include "common.hpp"

namespace mignn {
namespace {

constexpr int BM = 48;                 // rows per tile
constexpr int NCW = 4;                 // consumer waves (one per SIMD: MFMA issue saturates)
constexpr int NPW = 12;                // producer waves
constexpr int NTHREADS = (NCW + NPW) * 64;
constexpr int PROWS = BM / NPW;        // rows per producer wave (4)
constexpr int IREG = 1;                // index registers per lane: 64 CSR entries per wave

enum { AGG_GCN = 0, AGG_SUM = 1, ROWS = 2 };

template <int K, int N, int MODE>
struct Cfg {
    static_assert(K % 16 == 0 && K <= 256 && N % 16 == 0, "K, N multiples of 16, K <= 256");
    static constexpr int WN = N / 16 < NCW ? N / 16 : NCW;    // consumer column slices
    static constexpr int WM = 1;                               // consumers own all 48 rows
    static constexpr int MW = WM * WN;                         // consumer waves with work
    static constexpr int WROWS = BM / WM;
    static constexpr int WCOLS = N / WN;
    static constexpr int IB = WROWS / 16;
    static constexpr int JB = WCOLS / 16;
    static constexpr int KC = K / 16;
    static constexpr int LPR = K / 4;                          // lanes per A row (16 B each)
    static constexpr int RPW = 64 / LPR;                       // rows per wave instruction
    static constexpr int RSTEPS = PROWS >= RPW ? PROWS / RPW : 1;   // row steps per producer wave
    static constexpr int RIF = RSTEPS;                         // every row step in flight
    static constexpr int LD = K + 8;                           // LDS row stride (floats)
    static constexpr int A_FLOATS = BM * LD;
    static constexpr int W_FLOATS = N * LD;
    static constexpr int LDS_FLOATS = 2 * A_FLOATS + W_FLOATS;
    static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};

struct TileIdx {            // CSR indices of one producer wave's 8 rows, in lane registers
    int rp;                 // lanes 0..8: row_ptr[r0 + lane] (clamped to row_end)
    int j[IREG];            // lane t: col[e0 + t + 64 q]
    float w[IREG];          // lane t: ew[e0 + t + 64 q]  (GCN weights)
};

__device__ __forceinline__ int load_rp(const int32_t* __restrict__ row_ptr, int64_t r0,
                                       int64_t row_end, int lane) {
    const int64_t rr = r0 + lane < row_end ? r0 + lane : row_end;
    return (r0 < row_end && lane <= PROWS) ? row_ptr[rr] : 0;
}

template <int MODE>
__device__ __forceinline__ void load_entries(TileIdx& t, const int32_t* __restrict__ col,
                                             const float* __restrict__ ew, int lane) {
    const int e0 = __shfl(t.rp, 0, 64);
    const int ne = __shfl(t.rp, PROWS, 64) - e0;
#pragma unroll
    for (int q = 0; q < IREG; ++q) {
        const int e = lane + 64 * q;
        t.j[q] = e < ne ? col[e0 + e] : 0;
        t.w[q] = (MODE == AGG_GCN && e < ne) ? ew[e0 + e] : 1.f;
    }
}

template <int K, int N, int MODE>
// 16 waves per CU = 4 per SIMD -> <= 128 VGPRs: 16 gathered rows in flight per
// producer wave (12 producers: 192 KB per CU)
__global__ __launch_bounds__(NTHREADS, 4) void fused_tile_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, float self_scale, const float* __restrict__ x, int64_t ldx,
    int64_t row_begin, int64_t row_end, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ R, int64_t ldr,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags, int n_valid,
    float* __restrict__ out, int64_t ldo) {
    using C = Cfg<K, N, MODE>;
    __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];
    float* const A0 = lds;
    float* const Wl = lds + 2 * C::A_FLOATS;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + BM - 1) / BM;
    const int G = gridDim.x;            // multiple of 8 (host guarantees)
    const int xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3;
    const int per_xcd = G >> 3;
    const int64_t nsteps = (ntiles + G - 1) / G;
    auto tile_of = [&](int64_t s) -> int64_t { return s * G + (int64_t)xcd * per_xcd + slot; };

    // W -> LDS (rows n >= n_valid padded with zeros)
    for (int i = tid; i < N * (K / 4); i += NTHREADS) {
        const int n = i / (K / 4), k4 = i % (K / 4);
        st4(&Wl[n * C::LD + 4 * k4], n < n_valid ? ld4(W + (int64_t)n * K + 4 * k4)
                                               : make_float4(0.f, 0.f, 0.f, 0.f));
    }

    if (wave >= NCW) {
        // ============================================================ producer
        const int pw = wave - NCW;
        auto first_row = [&](int64_t tile) { return row_begin + tile * BM + pw * PROWS; };

        auto gather = [&](int64_t tile, const TileIdx& ix, float* A) {
            int lane_ = lane;
            asm volatile("" : "+v"(lane_));   // keep lane-derived offsets out of LICM
            const int c = lane_ % C::LPR, grp = lane_ / C::LPR;
            const int64_t r0 = first_row(tile);
            if constexpr (MODE == ROWS) {
                constexpr int CH = PROWS * C::LPR;
                constexpr int NQ = (CH + 63) / 64;
                const float* xb = x + r0 * ldx;
                const int nr = static_cast<int>(row_end - r0 < PROWS ? row_end - r0 : PROWS);
                float4 v[NQ];
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
                    if (id < CH) st4(&A[(pw * PROWS + lr) * C::LD + 4 * cc], v[q]);
                }
            } else {
                const int e0 = __shfl(ix.rp, 0, 64);
                const int ne = __shfl(ix.rp, PROWS, 64) - e0;
                const int safe_row = static_cast<int>(row_end - 1);   // valid x row
                const bool in_regs = ne <= 64 * IREG;              // wave-uniform
                // wave-uniform edge-loop bound: ids live in lanes across the whole
                // wave, so every lane stays in the loop while any row reads them
                int dmax = lane_ < PROWS ? __shfl(ix.rp, lane_ + 1, 64) - ix.rp : 0;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) dmax = max(dmax, __shfl_xor(dmax, o, 64));
                if (in_regs) {
#pragma unroll
                for (int st = 0; st < C::RSTEPS; st += C::RIF) {
                    int lrow[C::RIF], beg[C::RIF], deg[C::RIF];
                    float4 acc[C::RIF];
#pragma unroll
                    for (int q = 0; q < C::RIF; ++q) {
                        lrow[q] = (st + q) * C::RPW + grp;
                        const int lq = lrow[q] < PROWS ? lrow[q] : PROWS - 1;
                        const int bq = __shfl(ix.rp, lq, 64);
                        beg[q] = bq - e0;
                        deg[q] = lrow[q] < PROWS ? __shfl(ix.rp, lq + 1, 64) - bq : 0;
                        acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                    for (int u0 = 0; u0 < dmax; u0 += 8) {
                        // (1) issue every neighbour-row load of the RIF row steps; invalid
                        //     slots re-read a valid entry and get weight 0 below, so the
                        //     loads need no select and only the data stays live
                        float4 v[C::RIF][8];
#pragma unroll
                        for (int q = 0; q < C::RIF; ++q)
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int e = beg[q] + min(u0 + u, max(deg[q] - 1, 0));
                                const int s0 = __shfl(ix.j[0], e & 63, 64);
                                const int s1 = IREG > 1 ? __shfl(ix.j[IREG - 1], e & 63, 64) : s0;
                                // empty / masked row: re-read a valid row (row_end-1), weight 0
                                const int jj = deg[q] > 0 ? (e < 64 ? s0 : s1) : safe_row;
                                v[q][u] = ld4(x + (int64_t)jj * ldx + 4 * c);
                            }
                        // (2) weights after the loads are in flight; accumulate in CSR order
#pragma unroll
                        for (int q = 0; q < C::RIF; ++q)
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const bool ok = u0 + u < deg[q];
                                float ww = 1.f;
                                if constexpr (MODE == AGG_GCN) {
                                    const int e = beg[q] + min(u0 + u, max(deg[q] - 1, 0));
                                    const float w0 = __shfl(ix.w[0], e & 63, 64);
                                    const float w1 = IREG > 1 ? __shfl(ix.w[IREG - 1], e & 63, 64) : w0;
                                    ww = e < 64 ? w0 : w1;
                                }
                                // invalid slot: weight 0 (GIN: fma(1, x, acc) == acc + x exactly)
                                acc[q] = fma4(ok ? ww : 0.f, v[q][u], acc[q]);
                            }
                    }
#pragma unroll
                    for (int q = 0; q < C::RIF; ++q) {
                        if constexpr (MODE == AGG_SUM) {
                            // GINConv: out = sum_j x_j; out = out + (1 + eps) * x_i
                            const int64_t row = r0 + lrow[q];
                            if (row < row_end) {
                                const float4 xi = ld4(x + row * ldx + 4 * c);
                                acc[q].x = acc[q].x + self_scale * xi.x;
                                acc[q].y = acc[q].y + self_scale * xi.y;
                                acc[q].z = acc[q].z + self_scale * xi.z;
                                acc[q].w = acc[q].w + self_scale * xi.w;
                            }
                        }
                        if (lrow[q] < PROWS) st4(&A[(pw * PROWS + lrow[q]) * C::LD + 4 * c], acc[q]);
                    }
                }
                } else {   // > 64 CSR entries in this wave's rows: indices from memory
#pragma unroll
                for (int st = 0; st < C::RSTEPS; st += 1) {
                    int lrow[1], beg[1], deg[1];
                    float4 acc[1];
#pragma unroll
                    for (int q = 0; q < 1; ++q) {
                        lrow[q] = (st + q) * C::RPW + grp;
                        const int lq = lrow[q] < PROWS ? lrow[q] : PROWS - 1;
                        const int bq = __shfl(ix.rp, lq, 64);
                        beg[q] = bq - e0;
                        deg[q] = lrow[q] < PROWS ? __shfl(ix.rp, lq + 1, 64) - bq : 0;
                        acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                    }
                    for (int u0 = 0; u0 < dmax; u0 += 8) {
                        // (1) issue every neighbour-row load of the RIF row steps; invalid
                        //     slots re-read a valid entry and get weight 0 below, so the
                        //     loads need no select and only the data stays live
                        float4 v[1][8];
#pragma unroll
                        for (int q = 0; q < 1; ++q)
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const int e = beg[q] + min(u0 + u, max(deg[q] - 1, 0));
                                const int jj = deg[q] > 0 ? col[e0 + e] : safe_row;
                                v[q][u] = ld4(x + (int64_t)jj * ldx + 4 * c);
                            }
                        // (2) weights after the loads are in flight; accumulate in CSR order
#pragma unroll
                        for (int q = 0; q < 1; ++q)
#pragma unroll
                            for (int u = 0; u < 8; ++u) {
                                const bool ok = u0 + u < deg[q];
                                float ww = 1.f;
                                if constexpr (MODE == AGG_GCN) {
                                    const int e = beg[q] + min(u0 + u, max(deg[q] - 1, 0));
                                    ww = ok ? ew[e0 + e] : 0.f;
                                }
                                // invalid slot: weight 0 (GIN: fma(1, x, acc) == acc + x exactly)
                                acc[q] = fma4(ok ? ww : 0.f, v[q][u], acc[q]);
                            }
                    }
#pragma unroll
                    for (int q = 0; q < 1; ++q) {
                        if constexpr (MODE == AGG_SUM) {
                            // GINConv: out = sum_j x_j; out = out + (1 + eps) * x_i
                            const int64_t row = r0 + lrow[q];
                            if (row < row_end) {
                                const float4 xi = ld4(x + row * ldx + 4 * c);
                                acc[q].x = acc[q].x + self_scale * xi.x;
                                acc[q].y = acc[q].y + self_scale * xi.y;
                                acc[q].z = acc[q].z + self_scale * xi.z;
                                acc[q].w = acc[q].w + self_scale * xi.w;
                            }
                        }
                        if (lrow[q] < PROWS) st4(&A[(pw * PROWS + lrow[q]) * C::LD + 4 * c], acc[q]);
                    }
                }
                }
            }
        };

        // index pipeline: cur = tile s+1 entries, nrp = row_ptr of tile s+2
        TileIdx cur{}, nxt{};
        int rp2 = 0;
        const bool prod = !(flags & MIGNN_DIAG_NO_PRODUCE);
        if (MODE != ROWS) {
            cur.rp = load_rp(row_ptr, first_row(tile_of(0)), row_end, lane);
            nxt.rp = load_rp(row_ptr, first_row(tile_of(1)), row_end, lane);
            load_entries<MODE>(cur, col, ew, lane);
            load_entries<MODE>(nxt, col, ew, lane);
            rp2 = load_rp(row_ptr, first_row(tile_of(2)), row_end, lane);
        }
        if (prod && tile_of(0) < ntiles) gather(tile_of(0), cur, A0);
        __syncthreads();
        for (int64_t s = 0; s < nsteps; ++s) {
            const int64_t tn = tile_of(s + 1);
            TileIdx nn{};
            if (MODE != ROWS) {
                nn.rp = rp2;                                          // tile s+2
                load_entries<MODE>(nn, col, ew, lane);
                rp2 = load_rp(row_ptr, first_row(tile_of(s + 3)), row_end, lane);
            }
            if (prod && s + 1 < nsteps && tn < ntiles)
                gather(tn, nxt, A0 + ((s + 1) & 1) * C::A_FLOATS);
            nxt = nn;
            __syncthreads();
        }
        return;
    }

    // ================================================================ consumer
    const int wm = wave / C::WN, wn = wave % C::WN;
    const bool mw = wave < C::MW && !(flags & MIGNN_DIAG_NO_MFMA);
    __syncthreads();   // W staged, tile 0 produced
    for (int64_t s = 0; s < nsteps; ++s) {
        const int64_t tile = tile_of(s);
        if (mw && tile < ntiles) {
            const float* A = A0 + (s & 1) * C::A_FLOATS;
            int lane_ = lane;
            asm volatile("" : "+v"(lane_));
            const int rr = lane_ & 15, gg = lane_ >> 4;
            const int64_t m0 = row_begin + tile * BM + wm * C::WROWS;      // uniform
            const int mr = static_cast<int>(row_end - m0 < C::WROWS ? row_end - m0 : C::WROWS);
            // residual prefetch for D[row = 4g + q][col = r]
            float res[C::IB][C::JB][4];
            const float* Rb = (flags & MIGNN_EPI_RESIDUAL) ? R + m0 * ldr : nullptr;
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = ib * 16 + 4 * gg + q;
                        const int n = wn * C::WCOLS + jb * 16 + rr;
                        res[ib][jb][q] = (Rb && lr < mr && n < n_valid)
                                             ? Rb[lr * static_cast<int>(ldr) + n] : 0.f;
                    }
            f32x4 acc[C::IB][C::JB];
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) acc[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                float4 a[C::IB], b[C::JB];
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib)
                    a[ib] = *reinterpret_cast<const float4*>(
                        &A[(wm * C::WROWS + ib * 16 + rr) * C::LD + kc * 16 + 4 * gg]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
                    b[jb] = *reinterpret_cast<const float4*>(
                        &Wl[(wn * C::WCOLS + jb * 16 + rr) * C::LD + kc * 16 + 4 * gg]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(a[ib].x, b[jb].x, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(a[ib].y, b[jb].y, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(a[ib].z, b[jb].z, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(a[ib].w, b[jb].w, acc[ib][jb]);
            }
            float* ob = out + m0 * ldo;
#pragma unroll
            for (int jb = 0; jb < C::JB; ++jb) {
                const int n = wn * C::WCOLS + jb * 16 + rr;
                if (n >= n_valid) continue;
                const float bv = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
                const float sc = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
                const float sh = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lr = ib * 16 + 4 * gg + q;
                        if (lr < mr)   // non-temporal: keep L2 / MALL for the gathered rows
                            __builtin_nontemporal_store(
                                epilogue(acc[ib][jb][q], flags, bv, res[ib][jb][q], sc, sh),
                                ob + lr * static_cast<int>(ldo) + n);
                    }
            }
        }
        __syncthreads();
    }
}

struct TileArgs {
    const int32_t* row_ptr; const int32_t* col; const float* ew; float self_scale;
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
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NTHREADS), 0, st, a.row_ptr, a.col, a.ew,
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

extern "C" int mignn_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* ew,
                               const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                               const float* w, const float* bias, const float* scale,
                               const float* shift, int flags, float* out, int64_t ldo,
                               void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && x && w && out, "gcn_layer: null pointer");
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
    TileArgs t{row_ptr, col, ew, 1.f, x, ldx, rb, re, w, bias, x, ldx, scale, shift, flags, h,
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
