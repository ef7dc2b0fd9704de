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
#include <type_traits>

#include "common.hpp"

namespace mignn {
namespace {

constexpr int BM = 48;                 // rows per tile
constexpr int NCW = 8;                 // consumer (MFMA) waves: two per SIMD
constexpr int NPW = 8;                 // producer (gather) waves
constexpr int NTHREADS = (NCW + NPW) * 64;
constexpr int PROWS = BM / NPW;        // rows per producer wave (6)
static_assert(NCW * PROWS == BM, "consumer waves store PROWS rows each");
constexpr int SLOTS = 7;               // neighbour rows per row and chunk: 42 loads in flight

enum { AGG_GCN = 0, AGG_SUM = 1, ROWS = 2 };

// Diagnostic timeline (MIGNN_DIAG_TRACE): s_memtime stamps of one producer and
// one consumer wave of workgroups 0..7, steps 0..63 -> g_trace[(b*64+s)*8+slot]
__device__ unsigned long long* g_trace = nullptr;
__device__ __forceinline__ void stamp(int flags, int lane, int64_t s, int slot) {
    if ((flags & MIGNN_DIAG_TRACE) && blockIdx.x < 8 && s < 64 && lane == 0 && g_trace)
        g_trace[(blockIdx.x * 64 + s) * 8 + slot] = __builtin_amdgcn_s_memtime();
}

template <int K, int N, int MODE>
struct Cfg {
    static_assert(K % 16 == 0 && K <= 256 && N % 16 == 0, "K, N multiples of 16, K <= 256");
    static constexpr int WN = N / 16 < NCW ? N / 16 : NCW;    // consumer column slices
    static constexpr int WM = 1;                               // consumers own all BM rows
    static constexpr int MW = WM * WN;                         // consumer waves with work
    static constexpr int WROWS = BM / WM;
    static constexpr int WCOLS = N / WN;
    static constexpr int IB = WROWS / 16;
    static constexpr int JB = WCOLS / 16;
    static constexpr int KC = K / 16;
    static constexpr int LPR = K / 4;                          // ROWS: lanes per A row (16 B each)
    static constexpr int VPL = K / 64;                         // AGG: floats per lane of a row
    static constexpr int RPW = 64 / LPR;                       // rows per wave instruction
    static constexpr int RSTEPS = PROWS >= RPW ? PROWS / RPW : 1;   // row steps per producer wave
    static constexpr int RIF = RSTEPS;                         // every row step in flight
    static constexpr int LD = K + 8;                           // LDS row stride (floats)
    static constexpr int A_FLOATS = BM * LD;
    static constexpr int LDN = N + 8;                          // R / C tile row stride
    static constexpr int R_FLOATS = BM * LDN;
    static constexpr int NC4 = N / 4;                          // 16-B chunks per R / C row
    // double-buffered A tile; 3-deep ring of R/C tiles (residual in, result
    // out): at step s the producers fill R[(s+1)%3], the consumers compute in
    // R[s%3] and store the finished R[(s-1)%3]
    static constexpr int LDS_FLOATS = 2 * A_FLOATS + 3 * R_FLOATS;
    static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
};

// Per-producer-wave CSR indices of one tile, one CSR entry per lane:
// lanes 0..PROWS of rpv hold row_ptr[r0 + lane] (clamped to row_end); lane t of
// ej / ew holds entry e0 + t of the wave's rows (t < 64).  Loaded one tile
// ahead (rpv two ahead), read with v_readlane at wave-uniform lane ids.
struct WaveIdx {
    int rpv;
    int ej;
    float ew;
};

__device__ __forceinline__ int load_rpv(const int32_t* __restrict__ row_ptr, int64_t r0,
                                        int64_t row_end, int lane) {
    const int64_t r = r0 + lane < row_end ? r0 + lane : row_end;
    return lane <= PROWS ? row_ptr[r] : 0;
}

template <int MODE>
__device__ __forceinline__ void load_wave_entries(WaveIdx& t, const int32_t* __restrict__ col,
                                                  const float* __restrict__ ew, int lane) {
    const int e0 = __builtin_amdgcn_readlane(t.rpv, 0);
    const int ne = __builtin_amdgcn_readlane(t.rpv, PROWS) - e0;
    t.ej = lane < ne ? col[e0 + lane] : 0;
    t.ew = (MODE == AGG_GCN && lane < ne) ? ew[e0 + lane] : 1.f;
}

template <int K, int N, int MODE, bool VEC>
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
    float* const R0 = lds + 2 * C::A_FLOATS;
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + BM - 1) / BM;
    const int G = gridDim.x;            // multiple of 8 (host guarantees)
    const int xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3;
    const int per_xcd = G >> 3;
    // interleaved (default): at step s the chip covers tiles [sG, (s+1)G), XCD x a
    // contiguous run of G/8 of them.  XCD-major: XCD x sweeps its own contiguous
    // 1/8 of the tiles, G/8 per step (a locality-ordered graph keeps each XCD's
    // working set in its own L2).  Tiles past the range map to ntiles (skipped).
    const bool xmajor = (flags & MIGNN_SCHED_XCD_MAJOR) != 0;
    const int64_t tx = (ntiles + 7) / 8;
    const int64_t nsteps = xmajor ? (tx + per_xcd - 1) / per_xcd : (ntiles + G - 1) / G;
    auto tile_of = [&](int64_t s) -> int64_t {
        if (!xmajor) return s * G + (int64_t)xcd * per_xcd + slot;
        const int64_t l = s * per_xcd + slot;
        const int64_t t = (int64_t)xcd * tx + l;
        return l < tx && t < ntiles ? t : ntiles;
    };

    if (wave >= NCW) {
        // ============================================================ producer
        const int pw = wave - NCW;
        auto first_row = [&](int64_t tile) { return row_begin + tile * BM + pw * PROWS; };

        auto gather = [&](int64_t tile, const WaveIdx& ix, float* A, float* Rt) {
            int lane_ = lane;
            asm volatile("" : "+v"(lane_));   // keep lane-derived offsets out of LICM
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
                // one row per wave instruction: row bounds, column ids and edge
                // weights are wave-uniform (scalar loads into SGPRs, SALU address
                // arithmetic); per neighbour row the vector work is one 8-B load
                // and VPL fmas per lane.  All PROWS x 8 loads are issued before
                // the first fma.
                constexpr int VPL = C::VPL;
                int rp[PROWS + 1];
#pragma unroll
                for (int q = 0; q <= PROWS; ++q) rp[q] = __builtin_amdgcn_readlane(ix.rpv, q);
                const int e0 = rp[0];
                // wave-uniform: every entry of the wave's rows in lanes 0..62; lanes
                // past them hold column 0 / weight 0 (a valid row, never summed)
                const bool in_regs = rp[PROWS] - e0 < 64;
                int deg[PROWS], dmax = 0;
#pragma unroll
                for (int q = 0; q < PROWS; ++q) {
                    deg[q] = rp[q + 1] - rp[q];
                    dmax = max(dmax, deg[q]);
                }
                float acc[PROWS][VPL];
#pragma unroll
                for (int q = 0; q < PROWS; ++q)
#pragma unroll
                    for (int t = 0; t < VPL; ++t) acc[q][t] = 0.f;
                const int loff = lane_ * (4 * VPL);   // byte offset of this lane's floats
                const uint32_t ldxb = static_cast<uint32_t>(ldx) * 4u;
                // one buffer descriptor per gathered row, built with SALU only: the
                // row base (32x32->64-bit product) is wave-uniform, the lane offset
                // is the 32-bit voffset
                const uint64_t xbase = reinterpret_cast<uint64_t>(x);
                auto xload = [&](uint32_t r, float (&v)[VPL]) {
                    const i32x4 rs = buffer_rsrc(xbase + (uint64_t)r * ldxb, K * 4);
                    if constexpr (VPL == 2) {
                        const f32x2 t = raw_buffer_load_f32x2(rs, loff, 0, 0);
                        v[0] = t[0];
                        v[1] = t[1];
                    } else {
                        v[0] = raw_buffer_load_f32(rs, loff, 0, 0);
                    }
                };
                // slot u of row q reads entry rp[q] + min(u, deg-1): slots past the row
                // re-read its last entry (loads stay unconditional), weight 0
                int tq[PROWS], dm1[PROWS];
#pragma unroll
                for (int q = 0; q < PROWS; ++q) {
                    tq[q] = rp[q] - e0;
                    dm1[q] = max(deg[q] - 1, 0);
                }
                if (in_regs) {
                    for (int u0 = 0; u0 < dmax; u0 += SLOTS) {   // dmax > 0: the range has entries
                        float v[PROWS][SLOTS][VPL];
#pragma unroll
                        for (int q = 0; q < PROWS; ++q)
#pragma unroll
                            for (int u = 0; u < SLOTS; ++u) {
                                const int t = tq[q] + min(u0 + u, dm1[q]);
                                xload(static_cast<uint32_t>(__builtin_amdgcn_readlane(ix.ej, t)),
                                      v[q][u]);
                            }
                        // CSR order; weight-0 slots leave acc unchanged (finite x);
                        // GIN: fma(1, x, acc) == acc + x exactly
#pragma unroll
                        for (int q = 0; q < PROWS; ++q) {
                            // one row's weights at a time (keeps SGPR pressure low)
                            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                            for (int u = 0; u < SLOTS; ++u) {
                                float we = 1.f;
                                if constexpr (MODE == AGG_GCN) {
                                    const int t = tq[q] + min(u0 + u, dm1[q]);
                                    we = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                                       __builtin_bit_cast(int, ix.ew), t));
                                }
                                const float w = u0 + u < deg[q] ? we : 0.f;
#pragma unroll
                                for (int t = 0; t < VPL; ++t)
                                    acc[q][t] = fmaf(w, v[q][u][t], acc[q][t]);
                            }
                        }
                        // GCN residual x_i: the last slot re-reads the row's last entry,
                        // which in the CSR the layer takes (MIGNN_CSR_ONE_SELF_LOOP,
                        // mignn.h) is its self loop, appended after the edges as
                        // add_remaining_self_loops does
                        if (MODE == AGG_GCN && has_res) {
#pragma unroll
                            for (int q = 0; q < PROWS; ++q)
                                stv<VPL>(&Rt[(pw * PROWS + q) * C::LDN + VPL * lane_],
                                         v[q][SLOTS - 1]);
                        }
                    }
                } else {
                    // > 63 entries in the wave's rows (hubs): one neighbour row at a
                    // time, indices by scalar loads -- correct, not fast
#pragma unroll 1
                    for (int q = 0; q < PROWS; ++q) {
#pragma unroll 1
                        for (int u = 0; u < deg[q]; ++u) {
                            const int e = rp[q] + u;
                            float vv[VPL];
                            xload(static_cast<uint32_t>(col[e]), vv);
                            const float w = MODE == AGG_GCN ? ew[e] : 1.f;
#pragma unroll
                            for (int t = 0; t < VPL; ++t) acc[q][t] = fmaf(w, vv[t], acc[q][t]);
                            if (MODE == AGG_GCN && has_res && u == deg[q] - 1)
                                stv<VPL>(&Rt[(pw * PROWS + q) * C::LDN + VPL * lane_], vv);
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < PROWS; ++q) {
                    const int64_t row = r0 + q;
                    if constexpr (MODE == AGG_SUM) {
                        // GINConv: out = sum_j x_j; out = out + (1 + eps) * x_i
                        if (row < row_end) {
                            float xi[VPL];
                            xload(static_cast<uint32_t>(row), xi);
#pragma unroll
                            for (int t = 0; t < VPL; ++t) acc[q][t] = acc[q][t] + self_scale * xi[t];
                        }
                    }
                    stv<VPL>(&A[(pw * PROWS + q) * C::LD + VPL * lane_], acc[q]);
                }
            }
            // residual rows -> R tile (contiguous 16-B chunks); GCN: copied from
            // the self-loop slot of the gather above (R == x, one self loop per row)
            if (MODE != AGG_GCN && has_res) {
                constexpr int CH = PROWS * C::NC4;
                constexpr int NQ = (CH + 63) / 64;
                float4 v[NQ];
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int id = q * 64 + lane_;
                    const int lr = id / C::NC4, cc = id % C::NC4;
                    const int64_t row = r0 + lr;
                    v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (id < CH && row < row_end) {
                        if constexpr (VEC) v[q] = ld4(R + row * ldr + 4 * cc);
                        else v[q] = ld4_masked(R + row * ldr, 4 * cc, n_valid);
                    }
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int id = q * 64 + lane_;
                    const int lr = id / C::NC4, cc = id % C::NC4;
                    if (id < CH) st4(&Rt[(pw * PROWS + lr) * C::LDN + 4 * cc], v[q]);
                }
            }
        };

        // index pipeline: x rows of tile s+1 gather while the entries of tile s+2
        // and row_ptr of tile s+3 load
        const bool prod = !(flags & MIGNN_DIAG_NO_PRODUCE);
        WaveIdx cur{}, nxt{};
        int rp3 = 0;
        if constexpr (MODE != ROWS) {   // cur = tile 0, nxt = tile 1, rp3 = tile 2
            cur.rpv = load_rpv(row_ptr, first_row(tile_of(0)), row_end, lane);
            rp3 = load_rpv(row_ptr, first_row(tile_of(1)), row_end, lane);
            load_wave_entries<MODE>(cur, col, ew, lane);
            nxt.rpv = rp3;
            load_wave_entries<MODE>(nxt, col, ew, lane);
            rp3 = load_rpv(row_ptr, first_row(tile_of(2)), row_end, lane);
        }
        // step s gathers tile s+1 (s = -1: the prologue), stores tile s-1
        for (int64_t s = -1; s < nsteps; ++s) {
            const int64_t tn = tile_of(s + 1);
            if (pw == 0 && s >= 0) stamp(flags, lane, s, 0);
            WaveIdx nn{};
            if constexpr (MODE != ROWS) {
                nn.rpv = rp3;                                         // tile s+2
                load_wave_entries<MODE>(nn, col, ew, lane);
                rp3 = load_rpv(row_ptr, first_row(tile_of(s + 4)), row_end, lane);
            }
            float* const Rn = R0 + ((s + 1) % 3) * C::R_FLOATS;
            if (prod && s + 1 < nsteps && tn < ntiles)
                gather(tn, cur, A0 + ((s + 1) & 1) * C::A_FLOATS, Rn);
            if (pw == 0 && s >= 0) stamp(flags, lane, s, 1);
            cur = nxt;
            nxt = nn;
            __syncthreads();
        }
        return;
    }

    // ================================================================ consumer
    // No global memory traffic here: A and the residual come from LDS, the
    // result goes back to LDS (the producers store whole rows next step).
    const int wm = wave / C::WN, wn = wave % C::WN;
    const bool mw = wave < C::MW && !(flags & MIGNN_DIAG_NO_MFMA);
    int lane_ = lane;
    asm volatile("" : "+v"(lane_));
    const int rr = lane_ & 15, gg = lane_ >> 4;
    // this wave's W slice as MFMA A-operand fragments, held for the whole launch:
    // lane (r, g) holds W[n = slice + 16 jb + r][k = 16 kc + 4 g .. +3]; operands
    // swapped (acc = W_slice . A^T): lane (r, g) owns output row 16 ib + r,
    // columns 16 jb + 4 g .. +3
    float4 wf[C::JB][C::KC];
    float4 bv[C::JB], sc[C::JB], sh[C::JB];
#pragma unroll
    for (int jb = 0; jb < C::JB; ++jb) {
        const int nw = wn * C::WCOLS + jb * 16 + rr;
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc)
            wf[jb][kc] = (mw && nw < n_valid) ? ld4(W + (int64_t)nw * K + kc * 16 + 4 * gg)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
        const int n = wn * C::WCOLS + jb * 16 + 4 * gg;
        bv[jb] = make_float4(0.f, 0.f, 0.f, 0.f);
        sc[jb] = make_float4(1.f, 1.f, 1.f, 1.f);
        sh[jb] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (mw) {
            if constexpr (VEC) {
                if (flags & MIGNN_EPI_BIAS) bv[jb] = ld4(bias + n);
                if (flags & MIGNN_EPI_AFFINE) { sc[jb] = ld4(scale + n); sh[jb] = ld4(shift + n); }
            } else {
                if (flags & MIGNN_EPI_BIAS) bv[jb] = ld4_masked(bias, n, n_valid);
                if (flags & MIGNN_EPI_AFFINE) {
                    sc[jb] = ld4_masked(scale, n, n_valid);
                    sh[jb] = ld4_masked(shift, n, n_valid);
                }
            }
        }
    }
// consumer wave w stores rows 6w..6w+5 of a finished tile: C tile (LDS) ->
// out, whole rows.  Consumers issue no loads, so these stores never sit
// in front of a vmcnt wait (loads and stores share the in-order counter)
    auto store_out = [&](int64_t tile, const float* Ct) {
        int lane_ = lane;
        asm volatile("" : "+v"(lane_));
        const int64_t r0 = row_begin + tile * BM + wave * PROWS;
        constexpr int CH = PROWS * C::NC4;
        constexpr int NQ = (CH + 63) / 64;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int id = q * 64 + lane_;
            const int lr = id / C::NC4, cc = id % C::NC4;
            const int64_t row = r0 + lr;
            if (id < CH && row < row_end) {
                const float4 t = ld4(&Ct[(wave * PROWS + lr) * C::LDN + 4 * cc]);
                float* o = out + row * ldo + 4 * cc;
                if constexpr (VEC) {
                    // non-temporal: keep L2 / MALL for the gathered rows
                    __builtin_nontemporal_store(f32x4{t.x, t.y, t.z, t.w},
                                                reinterpret_cast<f32x4*>(o));
                } else {
                    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (4 * cc + u < n_valid) __builtin_nontemporal_store(tv[u], o + u);
                }
            }
        }
    };

    __syncthreads();   // tile 0 produced
    for (int64_t s = 0; s < nsteps; ++s) {
        if (wave == 0) stamp(flags, lane, s, 2);
        if (s >= 1 && tile_of(s - 1) < ntiles)
            store_out(tile_of(s - 1), R0 + ((s + 2) % 3) * C::R_FLOATS);   // (s-1)%3
        const int64_t tile = tile_of(s);
        if (mw && tile < ntiles) {
            const float* A = A0 + (s & 1) * C::A_FLOATS;
            float* const Rt = R0 + (s % 3) * C::R_FLOATS;
            f32x4 acc[C::IB][C::JB];
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib)
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) acc[ib][jb] = f32x4{0.f, 0.f, 0.f, 0.f};
            // A fragments of step kc + 1 are read while step kc's MFMAs run
            float4 fa[2][C::IB];
            auto load_frag = [&](int buf, int kc) {
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib)
                    fa[buf][ib] = *reinterpret_cast<const float4*>(
                        &A[(wm * C::WROWS + ib * 16 + rr) * C::LD + kc * 16 + 4 * gg]);
            };
            load_frag(0, 0);
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                const int cb = kc & 1;
                if (kc + 1 < C::KC) load_frag(cb ^ 1, kc + 1);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(wf[jb][kc].x, fa[cb][ib].x, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(wf[jb][kc].y, fa[cb][ib].y, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(wf[jb][kc].z, fa[cb][ib].z, acc[ib][jb]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int ib = 0; ib < C::IB; ++ib) acc[ib][jb] = mfma16x16x4(wf[jb][kc].w, fa[cb][ib].w, acc[ib][jb]);
            }
            if (wave == 0) stamp(flags, lane, s, 3);
            // epilogue in place in the R/C tile: each lane reads its residual
            // chunk and writes the result to the same 16 B (no other wave
            // touches them this step)
#pragma unroll
            for (int jb = 0; jb < C::JB; ++jb) {
                const int n = wn * C::WCOLS + jb * 16 + 4 * gg;
#pragma unroll
                for (int ib = 0; ib < C::IB; ++ib) {
                    float* const rc = &Rt[(wm * C::WROWS + ib * 16 + rr) * C::LDN + n];
                    const float4 rv = has_res ? ld4(rc) : make_float4(0.f, 0.f, 0.f, 0.f);
                    st4(rc, make_float4(
                                epilogue(acc[ib][jb][0], flags, bv[jb].x, rv.x, sc[jb].x, sh[jb].x),
                                epilogue(acc[ib][jb][1], flags, bv[jb].y, rv.y, sc[jb].y, sh[jb].y),
                                epilogue(acc[ib][jb][2], flags, bv[jb].z, rv.z, sc[jb].z, sh[jb].z),
                                epilogue(acc[ib][jb][3], flags, bv[jb].w, rv.w, sc[jb].w, sh[jb].w)));
                }
            }
            if (wave == 0) stamp(flags, lane, s, 4);
        }
        __syncthreads();
    }
    if (nsteps >= 1 && tile_of(nsteps - 1) < ntiles)
        store_out(tile_of(nsteps - 1), R0 + ((nsteps - 1) % 3) * C::R_FLOATS);
}

struct TileArgs {
    const int32_t* row_ptr; const int32_t* col; const float* ew; float self_scale;
    const float* x; int64_t ldx; int64_t rb, re;
    const float* W; const float* bias; const float* R; int64_t ldr;
    const float* scale; const float* shift; int flags; int n_valid; float* out; int64_t ldo;
};

template <int K, int N, int MODE, bool VEC>
int launch_tile_v(const TileArgs& a, hipStream_t st) {
    auto kern = fused_tile_kernel<K, N, MODE, VEC>;
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

template <int K, int N, int MODE>
int launch_tile(const TileArgs& a, hipStream_t st) {
    // VEC: 16-B epilogue (every column valid, 16-B aligned rows and vectors)
    auto al = [](const void* p) { return p == nullptr || aligned16(p); };
    const bool vec = a.n_valid == N && al(a.out) && (a.ldo & 3) == 0 && al(a.R) &&
                     (a.ldr & 3) == 0 && al(a.bias) && al(a.scale) && al(a.shift);
    if constexpr (MODE == ROWS) {
        return vec ? launch_tile_v<K, N, MODE, true>(a, st) : launch_tile_v<K, N, MODE, false>(a, st);
    } else {
        if (!vec) {
            set_error("fused layer: out / bias / scale / shift must be 16-B aligned, ld %% 4 == 0");
            return MIGNN_ERR_ARG;
        }
        return launch_tile_v<K, N, MODE, true>(a, st);
    }
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

static int gcn_layer_impl(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                    const float* w, const float* bias, const float* scale,
                                    const float* shift, int flags, float* out, int64_t ldo,
                                    void* stream);

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_set_trace(void* buf) {
    MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)));
    return MIGNN_OK;
}
#endif

extern "C" int mignn_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* ew,
                               const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                               const float* w, const float* bias, const float* scale,
                               const float* shift, int flags, float* out, int64_t ldo,
                               void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer: unknown flags 0x%x", flags);
    return gcn_layer_impl(row_ptr, col, ew, x, ldx, rb, re, h, w, bias, scale, shift, flags,
                                out, ldo, stream);
}

static int gcn_layer_impl(const int32_t* row_ptr, const int32_t* col, const float* ew,
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
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gin_layer: unknown flags 0x%x", flags);
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

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_gcn_layer(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                    const float* w, const float* bias, const float* scale,
                                    const float* shift, int flags, float* out, int64_t ldo,
                                    void* stream) {
    return gcn_layer_impl(row_ptr, col, ew, x, ldx, rb, re, h, w, bias, scale, shift, flags, out, ldo, stream);
}
#endif
