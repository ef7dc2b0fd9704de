// Fused GCN layer over a per-graph tile plan -- the north-star hot kernel
// (GCNConv + residual + BatchNorm(eval) + ReLU, reference gnn_model.py:63,
// :166, :184-191; the conv is PyG GCNConv: out_i = sum_{j->i} w_ij h_j + b,
// w_ij = dinv_i dinv_j over add_remaining_self_loops):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Arithmetic as gcn_f16x3.hip (fp32 aggregation, the aggregate split into
// fp16 hi + lo with a power-of-two row scale, three fp16 MFMA products with
// fp32 accumulation, ~2^-22 relative per product); the sum order of a row is
// the same (its out-of-tile entries in CSR order, then its in-tile entries
// in CSR order), so the two kernels agree bit for bit on rows of the plan's
// fast path.  What changes is the structure:
//
//   * The tile plan (mignn_gcn_plan, built once per graph and row range, the
//     CSR's companion): per row a 64-B record -- up to 7 CSR entries, the
//     in-tile ones from the front as {LDS image offset, w}, the out-of-tile
//     ones from the back as {column, w}, the counts, and a per-wave summary
//     (max in-tile / out-of-tile counts).  The kernel no longer builds lookup
//     tables per tile and layer (ballots, prefix counts, scattered LDS
//     writes: ~40 % of the old kernel's VALU instructions).
//   * Independent 4-wave workgroups, two per CU at H = 128 (three at H = 64),
//     each running whole tiles: the tile's own rows and plan records arrive
//     by LDS-DMA; every wave aggregates 16 rows (quad layout: a row = 16
//     lanes x 32 B, the LDS image read conflict-free whatever the
//     neighbours), splits them into the shared A image, then transforms 32
//     output columns of all 64 rows (split W held in registers), stages its
//     results and stores whole rows.  The next tile's DMA is issued as soon
//     as the A image is complete, under the MFMAs, epilogue and stores; the
//     co-resident workgroup covers each one's waits.  No producer / consumer
//     hand-offs, no LDS spin waits: four s_barriers per tile.
//
// Rows whose CSR row does not fit the record (more than 7 entries besides
// none: hubs) put their wave on a one-row-at-a-time path over the CSR.
#include "common.hpp"

namespace mignn {
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x4 = __attribute__((ext_vector_type(4))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_g;

constexpr int kRecBytes = 64;   // plan record per row
constexpr int kSlots = 7;       // CSR entries per record

template <int H, bool AGG>
struct TCfg {
    static_assert(H == 64 || H == 128, "tile plan GCN layer: H in {64, 128}");
    static constexpr int BM = 64;                  // rows per tile
    static constexpr int NW = 4;                   // waves per workgroup
    static constexpr int NT = NW * 64;
    static constexpr int F = H / 16;               // floats per lane of a row (16 lanes / row)
    static constexpr int CH = F / 4;               // 16-B chunks per lane of a row
    static constexpr int ROWB = H * 4;             // bytes per image row
    static constexpr int AS = H + 16;              // A row stride, halfs
    static constexpr int X_BYTES = BM * ROWB;
    static constexpr int A_BYTES = AGG ? 0 : BM * AS * 2;
    static constexpr int TAB_BYTES = BM * kRecBytes;
    static constexpr int OFF_ZERO = X_BYTES;                       // a zero row
    static constexpr int OFF_TAB = OFF_ZERO + ROWB;                // plan records of the tile
    static constexpr int OFF_AH = OFF_TAB + TAB_BYTES;
    static constexpr int OFF_AL = OFF_AH + A_BYTES;
    static constexpr int OFF_REXP = OFF_AL + A_BYTES;
    static constexpr int OFF_EPI = OFF_REXP + (AGG ? 0 : BM * 4);  // bias | scale | shift [H]
    static constexpr int LDS_BYTES = OFF_EPI + (AGG ? 0 : 3 * H * 4);
    static constexpr int OFF_STG = OFF_AH;                         // staging tile (A image space)
    static constexpr int EXR = 3;                  // out-of-tile rows per row held in registers
    static constexpr int UB = H == 128 ? 2 : 4;    // in-tile slots per LDS batch
    static constexpr int VPL = H / 64;             // floats per lane, row-per-wave path
    static constexpr int JB = H / 16 / NW;         // 16-column output blocks per wave
    static constexpr int KC = H / 32;              // 32-deep k chunks
    static constexpr int IB = BM / 16;             // 16-row blocks
    static constexpr int RPP = 1024 / ROWB;        // rows per 1-KB DMA piece
    static constexpr int LPR = 64 / RPP;           // lanes per row in a piece
    static constexpr int NPX = X_BYTES / 1024 / NW;   // own-row pieces per wave
    static constexpr int LPRW = ROWB / 16;         // lanes per row in a store instruction
    static constexpr int RPI = 64 / LPRW;          // rows per store instruction
    static constexpr int NSTG = 16 / RPI;          // row-store instructions per wave (16 rows)
    static constexpr int NST_AGG = CH * 4;         // aggregate-only stores per wave (4 quads)
    // row stores issued AFTER a tile's DMA (the fused layer stores its staged
    // rows after issuing the next tile's DMA; the aggregate stores before it)
    static constexpr int YST = AGG ? 0 : NSTG;
    static constexpr int WG_PER_CU = AGG ? 3 : (H == 128 ? 2 : 3);
    static_assert(AGG || BM * ROWB <= 2 * A_BYTES, "staging tile fits the A image");
    static_assert(LDS_BYTES * WG_PER_CU <= 160 * 1024, "LDS budget");
    static_assert(X_BYTES % (1024 * NW) == 0, "own-row pieces");
};

// waitcnt immediates (gfx9 layout): vmcnt(n) with lgkmcnt / expcnt untouched,
// and vmcnt(n) + lgkmcnt(0)
constexpr int vm_only(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xF00; }
constexpr int vm_lgkm0(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70; }
constexpr int kLgkm0 = 0xC07F;

template <int WAITCNT>
__device__ __forceinline__ void wait_cnt() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(WAITCNT);
    asm volatile("" ::: "memory");
}
template <int WAITCNT>
__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(WAITCNT);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint32_t lds_off(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_g)(p)));
}

// LDS-DMA of 16 B per lane to the wave-uniform LDS address dst (+16 x lane);
// invisible to the compiler's waitcnt bookkeeping (waited for by hand)
__device__ __forceinline__ void dma16(const void* src, uint32_t dst) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(__builtin_amdgcn_readfirstlane(static_cast<int>(dst)))
        : "memory");
}

__device__ __forceinline__ int split_exp(uint32_t mbits) {   // gcn_f16x3.hip scale_exp
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}

__device__ __forceinline__ uint32_t dpp_row_max(uint32_t v) {
    int t = static_cast<int>(v);
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x124, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x128, 0xf, 0xf, false)));
    return static_cast<uint32_t>(t);
}

__device__ __forceinline__ uint32_t dpp_wave_max(uint32_t v) {
    const uint32_t t = dpp_row_max(v);
    const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 0));
    const uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 16));
    const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 32));
    const uint32_t d = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 48));
    return max(max(a, b), max(c, d));
}

__device__ __forceinline__ f32x4 mfma_h(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __attribute__((aligned(16))) float g_tile_zero_row[256];

// ---------------------------------------------------------------- the plan
// One 64-thread block per tile, a thread per row.  Record of row r (tile t,
// local row lr): dwords 2s, 2s+1 (s < 7) = slot s {code, w}; in-tile entries
// fill slots 0, 1, .. (code = LDS image offset of the neighbour's row:
// off * ROWB | (off & 7) << 4), out-of-tile entries slots 6, 5, ..
// (code = column); dword 14 = nin | next << 8 | slow << 16 (slow: more than 7
// entries); dword 15 = the summary of the row's wave (rows 16w .. 16w+15 of
// the tile): max nin | max next << 8 | any slow << 16.
__global__ __launch_bounds__(64) void gcn_plan_kernel(const int32_t* __restrict__ row_ptr,
                                                      const int32_t* __restrict__ col,
                                                      const float* __restrict__ ew, int64_t rb,
                                                      int64_t re, int64_t ntiles, int rowb,
                                                      uint4* __restrict__ plan) {
    const int lr = threadIdx.x;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t t0 = rb + t * 64;
        const int64_t r = t0 + lr;
        const uint32_t nloc = static_cast<uint32_t>(re - t0 < 64 ? re - t0 : 64);
        uint32_t rec[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) rec[i] = 0u;
        int nin = 0, next = 0;
        if (r < re) {
            const int e0 = row_ptr[r], e1 = row_ptr[r + 1];
            for (int e = e0; e < e1; ++e) {
                const int c = col[e];
                const uint32_t wb = __float_as_uint(ew[e]);
                const uint32_t off = static_cast<uint32_t>(static_cast<int64_t>(c) - t0);
                const bool in = static_cast<int64_t>(c) >= t0 && off < nloc;
                if (nin + next < kSlots) {
                    const int s = in ? nin : kSlots - 1 - next;
                    const uint32_t code = in ? (off * static_cast<uint32_t>(rowb)) | ((off & 7u) << 4)
                                             : static_cast<uint32_t>(c);
#pragma unroll
                    for (int q = 0; q < kSlots; ++q)
                        if (q == s) {
                            rec[2 * q] = code;
                            rec[2 * q + 1] = wb;
                        }
                }
                if (in) ++nin;
                else ++next;
            }
        }
        const uint32_t slow = nin + next > kSlots ? 1u : 0u;
        const uint32_t cin = slow ? 0u : static_cast<uint32_t>(nin);
        const uint32_t cex = slow ? 0u : static_cast<uint32_t>(next);
        rec[14] = cin | (cex << 8) | (slow << 16);
        // wave summary over the 16 rows of the quarter (threads 16w .. 16w+15)
        uint32_t mi = cin, mx = cex, sl = slow;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            mi = max(mi, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mi), d, 16)));
            mx = max(mx, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mx), d, 16)));
            sl |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(sl), d, 16));
        }
        rec[15] = mi | (mx << 8) | (sl << 16);
        uint4* dst = plan + (t * 64 + lr) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[i] = make_uint4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
    }
}

// ------------------------------------------------------------- the layer
// AGG = true: the aggregate alone (out_i = sum_e ew_e x_{col e}, fp32), the
// GCN aggregation of mignn_gcn_aggregate over the plan
// MODE (timing ablations, mignn_diag_gcn_tile only; 0 in the product): 1 no
// out-of-tile gathers, 2 no in-tile sums, 4 no MFMAs, 8 no row stores
template <int H, bool AGG, int MODE = 0>
__global__ __launch_bounds__((TCfg<H, AGG>::NT), (TCfg<H, AGG>::WG_PER_CU)) void gcn_tile_kernel(
    const uint4* __restrict__ plan, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ col, const float* __restrict__ ew, const float* __restrict__ x,
    int64_t ldx, int64_t row_begin, int64_t row_end, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    using C = TCfg<H, AGG>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    _Float16* const AH = reinterpret_cast<_Float16*>(lds + C::OFF_AH);
    _Float16* const AL = reinterpret_cast<_Float16*>(lds + C::OFF_AL);
    int* const REXP = reinterpret_cast<int*>(lds + C::OFF_REXP);
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + C::BM - 1) / C::BM;
    const int G = gridDim.x;                  // multiple of 8 (host)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = G >> 3;
    const int64_t nsteps = (ntiles + G - 1) / G;
    // each XCD walks its own contiguous run of tiles, per_xcd at a time (the
    // locality order's panels stay in that XCD's L2)
    auto tile_of = [&](int64_t s) -> int64_t {
        return (int64_t)xcd * nsteps * per_xcd + s * per_xcd + slot;
    };

    // quad layout: lane group gq = lane >> 4 owns row 4 qd + gq of the wave's
    // 16, lane iq = lane & 15 the 16-B chunks c0(iq) + 16 j (gcn_f16x3.hip:
    // two rows of a ds_read_b128 lane group hit disjoint bank halves)
    const int gq = lane >> 4, iq = lane & 15;
    const int hb = (iq >= 4 && iq < 12) ? 1 : 0;
    const int c0 = (hb ? iq - 4 : (iq < 4 ? iq : iq - 8)) | (hb << 3);
    uint32_t coff[C::CH];
#pragma unroll
    for (int j = 0; j < C::CH; ++j) coff[j] = static_cast<uint32_t>((c0 + 16 * j) << 4);
    const uint64_t xbase = reinterpret_cast<uint64_t>(x);
    const uint64_t ldxb = static_cast<uint64_t>(ldx) * 4u;

    // DMA of a tile: this wave's 16 plan records (1 KB), then its share of the
    // own rows (chunk c of row lr at position c ^ (lr & 7))
    auto issue_dma = [&](int64_t tile) {
        const int64_t t0 = row_begin + tile * C::BM;
        int l = lane;
        asm volatile("" : "+v"(l));
        dma16(reinterpret_cast<const unsigned char*>(plan + (tile * C::BM + 16 * wave) * 4) + 16 * l,
              lds_off(lds + C::OFF_TAB + wave * 1024));
#pragma unroll
        for (int pp = 0; pp < C::NPX; ++pp) {
            const int p = pp * C::NW + wave;
            const int lr = p * C::RPP + l / C::LPR;
            const int pos = l % C::LPR;
            int64_t row = t0 + lr;
            if (row >= row_end) row = row_end - 1;         // any valid row: never stored
            const float* g = x + row * ldx + 4 * (pos ^ (lr & 7));
            dma16(g, lds_off(lds + p * 1024));
        }
    };

    // ---------------------------------------------------------- prologue
    for (int i = tid; i < C::ROWB / 4; i += C::NT) reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
    const int rr = lane & 15, gg = lane >> 4;
    const int n0 = wave * 16 * C::JB;
    f16x8 wh[C::JB][C::KC], wl[C::JB][C::KC];
    int qw = 0;
    if constexpr (!AGG) {
        float wv[C::JB][C::KC][8];
        uint32_t m = 0;
#pragma unroll
        for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                const float* p = W + (int64_t)(n0 + 16 * jb + rr) * H + 32 * kc + 8 * gg;
                const float4 a = ld4(p), b = ld4(p + 4);
                float* w8 = wv[jb][kc];
                w8[0] = a.x; w8[1] = a.y; w8[2] = a.z; w8[3] = a.w;
                w8[4] = b.x; w8[5] = b.y; w8[6] = b.z; w8[7] = b.w;
#pragma unroll
                for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(fabsf(w8[j])));
            }
        qw = split_exp(dpp_wave_max(m));
#pragma unroll
        for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float s = ldexpf(wv[jb][kc][j], qw);
                    const _Float16 h = static_cast<_Float16>(s);
                    wh[jb][kc][j] = h;
                    wl[jb][kc][j] = static_cast<_Float16>(s - static_cast<float>(h));
                }
        if (lane < 16 * C::JB) {
            const int n = n0 + lane;
            EPI[n] = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
            EPI[H + n] = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
            EPI[2 * H + n] = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
        }
    }
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    if (tile_of(0) < ntiles) issue_dma(tile_of(0));
    bar<kLgkm0>();   // zero row, epilogue terms

    unsigned char* const TABW = lds + C::OFF_TAB + wave * 1024;
    for (int64_t s = 0; s < nsteps; ++s) {
        const int64_t tile = tile_of(s);
        if (tile >= ntiles) break;                     // uniform over the workgroup
        const int64_t t0 = row_begin + tile * C::BM;
        const int64_t rem = row_end - t0;
        const uint32_t nloc = static_cast<uint32_t>(rem < C::BM ? rem : C::BM);
        // (1) this wave's plan records landed (own-row pieces and the last
        //     tile's row stores may still fly)
        if (s == 0 || C::YST == 0) wait_cnt<vm_only(C::NPX)>();
        else wait_cnt<vm_only(C::NPX + C::YST)>();
        const uint32_t summ = static_cast<uint32_t>(
            __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(TABW + 60)));
        const int max_in = static_cast<int>(summ & 0xffu);
        const int max_ex = static_cast<int>((summ >> 8) & 0xffu);
        const bool slow = (summ >> 16) != 0u;
        const int nex = (slow || (MODE & 1)) ? 0 : (max_ex < C::EXR ? max_ex : C::EXR);

        // (2) out-of-tile rows -> registers (slots 6, 5, 4 of each record)
        f32x4 xv[4][C::EXR][C::CH];
        float we[4][C::EXR];
        uint32_t cnt[4];
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const unsigned char* rec = TABW + (4 * qd + gq) * kRecBytes;
            const uint4 s45 = *reinterpret_cast<const uint4*>(rec + 32);
            const uint4 s6c = *reinterpret_cast<const uint4*>(rec + 48);
            cnt[qd] = s6c.z;
            const uint32_t nx = (s6c.z >> 8) & 0xffu;
            const uint32_t code[3] = {s6c.x, s45.z, s45.x};
            const uint32_t wbit[3] = {s6c.y, s45.w, s45.y};
#pragma unroll
            for (int e = 0; e < C::EXR; ++e) {
                if (e < nex) {
                    const bool v = static_cast<uint32_t>(e) < nx;
                    we[qd][e] = v ? __uint_as_float(wbit[e]) : 0.f;
                    const unsigned char* rowp =
                        v ? reinterpret_cast<const unsigned char*>(xbase + static_cast<uint64_t>(code[e]) * ldxb)
                          : reinterpret_cast<const unsigned char*>(g_tile_zero_row);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) xv[qd][e][j] = *reinterpret_cast<const f32x4*>(rowp + coff[j]);
                } else {
                    we[qd][e] = 0.f;
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) xv[qd][e][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
            }
        }
        // (3) own rows landed in every wave: wait for this wave's pieces (all
        //     but the stores and the gathers just issued), then the barrier
        {
            const int ng = nex * 4 * C::CH;
            // vmcnt immediates: younger stores + ng, ng in {0, 4CH, 8CH, 12CH}
            if (s == 0 || C::YST == 0) {
                if (ng == 0) bar<vm_lgkm0(0)>();
                else if (ng == 4 * C::CH) bar<vm_lgkm0(4 * C::CH)>();
                else if (ng == 8 * C::CH) bar<vm_lgkm0(8 * C::CH)>();
                else bar<vm_lgkm0(12 * C::CH)>();
            } else {
                if (ng == 0) bar<vm_lgkm0(C::YST)>();
                else if (ng == 4 * C::CH) bar<vm_lgkm0(C::YST + 4 * C::CH)>();
                else if (ng == 8 * C::CH) bar<vm_lgkm0(C::YST + 8 * C::CH)>();
                else bar<vm_lgkm0(C::YST + 12 * C::CH)>();
            }
        }

        // (4) aggregate the wave's 16 rows: out-of-tile entries, then in-tile
        f32x4 acc[4][C::CH];
        if (!slow) {
            // out-of-tile entries from the registers (CSR order), then the
            // rare ones beyond the register slots
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) {
#pragma unroll
                for (int j = 0; j < C::CH; ++j) acc[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int e = 0; e < C::EXR; ++e)
                    if (e < nex)
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                acc[qd][j][r] = fmaf(we[qd][e], xv[qd][e][j][r], acc[qd][j][r]);
            }
            if (!(MODE & 1) && max_ex > C::EXR) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    const unsigned char* rec = TABW + (4 * qd + gq) * kRecBytes;
                    const uint32_t nx = (cnt[qd] >> 8) & 0xffu;
#pragma unroll 1
                    for (int e = C::EXR; e < max_ex; ++e) {
                        const uint2 cw = *reinterpret_cast<const uint2*>(rec + (kSlots - 1 - e) * 8);
                        const bool v = static_cast<uint32_t>(e) < nx;
                        const float w = v ? __uint_as_float(cw.y) : 0.f;
                        const unsigned char* rowp =
                            v ? reinterpret_cast<const unsigned char*>(xbase + static_cast<uint64_t>(cw.x) * ldxb)
                              : reinterpret_cast<const unsigned char*>(g_tile_zero_row);
#pragma unroll
                        for (int j = 0; j < C::CH; ++j) {
                            const f32x4 vv = *reinterpret_cast<const f32x4*>(rowp + coff[j]);
#pragma unroll
                            for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, vv[r], acc[qd][j][r]);
                        }
                    }
                }
            }
            // in-tile entries (CSR order) from the own-row image, UB slots of
            // all four quads per LDS batch
#pragma unroll 1
            for (int u0 = 0; u0 < ((MODE & 2) ? 0 : max_in); u0 += C::UB) {
                uint4 rcd[4][C::UB / 2];
#pragma unroll
                for (int qd = 0; qd < 4; ++qd)
#pragma unroll
                    for (int b = 0; b < C::UB / 2; ++b)
                        rcd[qd][b] = *reinterpret_cast<const uint4*>(TABW + (4 * qd + gq) * kRecBytes + 8 * u0 + 16 * b);
                f32x4 vv[4][C::UB][C::CH];
                float wu[4][C::UB];
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    const uint32_t ni = cnt[qd] & 0xffu;
#pragma unroll
                    for (int uu = 0; uu < C::UB; ++uu) {
                        const uint4 rc = rcd[qd][uu / 2];
                        const bool v = static_cast<uint32_t>(u0 + uu) < ni;
                        const uint32_t P = v ? ((uu & 1) ? rc.z : rc.x) : static_cast<uint32_t>(C::OFF_ZERO);
                        wu[qd][uu] = v ? __uint_as_float((uu & 1) ? rc.w : rc.y) : 0.f;
#pragma unroll
                        for (int j = 0; j < C::CH; ++j) vv[qd][uu][j] = *reinterpret_cast<const f32x4*>(lds + (P ^ coff[j]));
                    }
                }
#pragma unroll
                for (int qd = 0; qd < 4; ++qd)
#pragma unroll
                    for (int uu = 0; uu < C::UB; ++uu)
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
#pragma unroll
                            for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(wu[qd][uu], vv[qd][uu][j][r], acc[qd][j][r]);
            }
        }

        if constexpr (AGG) {
            // ---------------------------------------------- aggregate only
            if (!slow) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    const int64_t row = t0 + 16 * wave + 4 * qd + gq;
                    if (row < row_end && !(MODE & 8))
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
                            __builtin_nontemporal_store(
                                acc[qd][j], reinterpret_cast<f32x4*>(reinterpret_cast<unsigned char*>(out + row * ldo) + coff[j]));
                }
            } else {
                // row-per-wave path (rows with more than 7 entries in the wave)
                const int loff = lane * (4 * C::VPL);
#pragma unroll 1
                for (int q = 0; q < 16; ++q) {
                    const int64_t row = t0 + 16 * wave + q;
                    if (row >= row_end) break;
                    const int e_begin = __builtin_amdgcn_readfirstlane(row_ptr[row]);
                    const int e_end = __builtin_amdgcn_readfirstlane(row_ptr[row + 1]);
                    float a[C::VPL];
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k) a[k] = 0.f;
#pragma unroll 1
                    for (int e = e_begin; e < e_end; ++e) {
                        const int c = __builtin_amdgcn_readfirstlane(col[e]);
                        const float w = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ew[e])));
                        const uint32_t off = static_cast<uint32_t>(static_cast<int64_t>(c) - t0);
                        float vv[C::VPL];
                        if (static_cast<int64_t>(c) >= t0 && off < nloc)
                            ldv<C::VPL>(reinterpret_cast<const float*>(lds + (off * C::ROWB + (static_cast<uint32_t>(loff) ^ ((off & 7u) << 4)))), vv);
                        else
                            ldv<C::VPL>(reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(x + (int64_t)c * ldx) + loff), vv);
#pragma unroll
                        for (int k = 0; k < C::VPL; ++k) a[k] = fmaf(w, vv[k], a[k]);
                    }
                    stv<C::VPL>(reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(out + row * ldo) + loff), a);
                }
            }
            // every wave done reading the own-row image: the next tile's DMA
            bar<kLgkm0>();
            if (s + 1 < nsteps && tile_of(s + 1) < ntiles) issue_dma(tile_of(s + 1));
            continue;
        } else {
            // ---------------------------------------------- fused layer
            if (!slow) {
#pragma unroll
                for (int qd = 0; qd < 4; ++qd) {
                    uint32_t m = 0;
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) m = max(m, __float_as_uint(fabsf(acc[qd][j][r])));
                    m = dpp_row_max(m);
                    const int p = split_exp(m);
                    const float sc = __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
                    const int lrow = 16 * wave + 4 * qd + gq;
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        f16x4 h, l;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float sv = acc[qd][j][r] * sc;
                            const _Float16 hh = static_cast<_Float16>(sv);
                            h[r] = hh;
                            l[r] = static_cast<_Float16>(sv - static_cast<float>(hh));
                        }
                        const int hc = 4 * (c0 + 16 * j);
                        *reinterpret_cast<f16x4*>(&AH[lrow * C::AS + hc]) = h;
                        *reinterpret_cast<f16x4*>(&AL[lrow * C::AS + hc]) = l;
                    }
                    if (iq == 0) REXP[lrow] = p;
                }
            } else {
                const int loff = lane * (4 * C::VPL);
#pragma unroll 1
                for (int q = 0; q < 16; ++q) {
                    const int64_t row = t0 + 16 * wave + q;
                    float a[C::VPL];
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k) a[k] = 0.f;
                    if (row < row_end) {
                        const int e_begin = __builtin_amdgcn_readfirstlane(row_ptr[row]);
                        const int e_end = __builtin_amdgcn_readfirstlane(row_ptr[row + 1]);
#pragma unroll 1
                        for (int e = e_begin; e < e_end; ++e) {
                            const int c = __builtin_amdgcn_readfirstlane(col[e]);
                            const float w = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ew[e])));
                            const uint32_t off = static_cast<uint32_t>(static_cast<int64_t>(c) - t0);
                            float vv[C::VPL];
                            if (static_cast<int64_t>(c) >= t0 && off < nloc)
                                ldv<C::VPL>(reinterpret_cast<const float*>(lds + (off * C::ROWB + (static_cast<uint32_t>(loff) ^ ((off & 7u) << 4)))), vv);
                            else
                                ldv<C::VPL>(reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(x + (int64_t)c * ldx) + loff), vv);
#pragma unroll
                            for (int k = 0; k < C::VPL; ++k) a[k] = fmaf(w, vv[k], a[k]);
                        }
                    }
                    uint32_t m = __float_as_uint(fabsf(a[0]));
                    if constexpr (C::VPL == 2) m = max(m, __float_as_uint(fabsf(a[1])));
                    const int p = split_exp(dpp_wave_max(m));
                    const int lrow = 16 * wave + q;
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k) {
                        const float sv = ldexpf(a[k], p);
                        const _Float16 hh = static_cast<_Float16>(sv);
                        AH[lrow * C::AS + C::VPL * lane + k] = hh;
                        AL[lrow * C::AS + C::VPL * lane + k] = static_cast<_Float16>(sv - static_cast<float>(hh));
                    }
                    if (lane == 0) REXP[lrow] = p;
                }
            }
            // residual + bias of the wave's output block (rows of all 64, its
            // 16 JB columns) from the own-row image, before it is overwritten
            f32x4 seed[C::IB][C::JB];
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib) {
                const int lr = ib * 16 + rr;
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
                    const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[n0 + 16 * jb + 4 * gg]);
                    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (has_res) {
                        const int ch = ((n0 + 16 * jb) >> 2) + gg;
                        rv = *reinterpret_cast<const float4*>(lds + lr * C::ROWB + ((ch ^ (lr & 7)) << 4));
                    }
                    seed[ib][jb] = f32x4{rv.x + bo[0], rv.y + bo[1], rv.z + bo[2], rv.w + bo[3]};
                }
            }
            // (5) A image complete, own-row image and plan records free
            bar<kLgkm0>();
            if (s + 1 < nsteps && tile_of(s + 1) < ntiles) issue_dma(tile_of(s + 1));
            // (6) transform: 32 (JB x 16) output columns of all 64 rows
            int pr[C::IB];
            f32x4 accm[C::IB][C::JB];
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib) {
                pr[ib] = REXP[ib * 16 + rr];
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) accm[ib][jb][r] = ldexpf(seed[ib][jb][r], pr[ib] + qw);
            }
            {
                int fb = rr * C::AS + 8 * gg;
                asm volatile("" : "+v"(fb));
                const _Float16* const AHb = AH + fb;
                const _Float16* const ALb = AL + fb;
                auto frag = [&](int t, f16x8& bh, f16x8& bl) {
                    const int kc = t / C::IB, ib = t % C::IB;
                    bh = *reinterpret_cast<const f16x8*>(&AHb[ib * 16 * C::AS + 32 * kc]);
                    bl = *reinterpret_cast<const f16x8*>(&ALb[ib * 16 * C::AS + 32 * kc]);
                };
                f16x8 fh[2], fl[2];
                frag(0, fh[0], fl[0]);
#pragma unroll
                for (int t = 0; t < ((MODE & 4) ? 0 : C::KC * C::IB); ++t) {
                    const int kc = t / C::IB, ib = t % C::IB;
                    if (t + 1 < C::KC * C::IB) frag(t + 1, fh[(t + 1) & 1], fl[(t + 1) & 1]);
#pragma unroll
                    for (int jb = 0; jb < C::JB; ++jb) {
                        accm[ib][jb] = mfma_h(wh[jb][kc], fh[t & 1], accm[ib][jb]);
                        accm[ib][jb] = mfma_h(wh[jb][kc], fl[t & 1], accm[ib][jb]);
                        accm[ib][jb] = mfma_h(wl[jb][kc], fh[t & 1], accm[ib][jb]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // (7) every wave done with the A image: stage the results there
            bar<kLgkm0>();
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib) {
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
                    const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + n0 + 16 * jb + 4 * gg]);
                    const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + n0 + 16 * jb + 4 * gg]);
                    float o[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = ldexpf(accm[ib][jb][r], -(pr[ib] + qw));
                        if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                        if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                        o[r] = v;
                    }
                    const int lr = ib * 16 + rr;
                    const int ch = ((n0 + 16 * jb) >> 2) + gg;
                    *reinterpret_cast<f32x4*>(lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4)) =
                        f32x4{o[0], o[1], o[2], o[3]};
                }
            }
            // (8) staged: whole rows out, wave w stores rows 16w .. 16w+15
            bar<kLgkm0>();
            {
                const int ch = lane % C::LPRW;
#pragma unroll
                for (int i = 0; i < C::NSTG; ++i) {
                    const int lr = 16 * wave + i * C::RPI + lane / C::LPRW;
                    const f32x4 v = *reinterpret_cast<const f32x4*>(
                        lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4));
                    // (rows past the end: the store is skipped, the count of
                    // vector-memory instructions stays NSTG per wave -- the
                    // waits above count on it)
                    float* dst = out + (t0 + lr < row_end ? (t0 + lr) * ldo + 4 * ch : 0);
                    if (t0 + lr < row_end && !(MODE & 8)) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
                }
            }
        }
    }
}

template <int H, bool AGG, int MODE = 0>
int launch_tile(const void* plan, const int32_t* row_ptr, const int32_t* col, const float* ew,
                const float* x, int64_t ldx, int64_t rb, int64_t re, const float* w,
                const float* bias, const float* scale, const float* shift, int flags, float* out,
                int64_t ldo, hipStream_t st) {
    using C = TCfg<H, AGG>;
    static int cus_cache[64] = {0};
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& cus = cus_cache[dev & 63];
    if (cus == 0) {
        MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        if (cus < 1) cus = 1;
    }
    int G = ((cus * C::WG_PER_CU) / 8) * 8;
    if (G < 8) G = 8;
    const int64_t ntiles = (re - rb + C::BM - 1) / C::BM;
    if (ntiles < G) G = static_cast<int>(((ntiles + 7) / 8) * 8);
    hipLaunchKernelGGL((gcn_tile_kernel<H, AGG, MODE>), dim3(G), dim3(C::NT), 0, st,
                       static_cast<const uint4*>(plan), row_ptr, col, ew, x, ldx, rb, re, w, bias,
                       scale, shift, flags, out, ldo);
    return launch_status(AGG ? "gcn_tile_kernel<agg>" : "gcn_tile_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_gcn_plan_bytes(int64_t row_begin, int64_t row_end) {
    if (row_end <= row_begin) return 0;
    const int64_t ntiles = (row_end - row_begin + 63) / 64;
    return static_cast<size_t>(ntiles) * 64 * kRecBytes;
}

extern "C" int mignn_gcn_plan(const int32_t* row_ptr, const int32_t* col, const float* ew,
                              int64_t rb, int64_t re, int h, void* plan, size_t plan_bytes,
                              void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && plan, "gcn_plan: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_plan: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_plan: bad row range");
    MIGNN_REQUIRE(aligned16(plan), "gcn_plan: unaligned plan");
    if (re == rb) return MIGNN_OK;
    MIGNN_REQUIRE(plan_bytes >= mignn_gcn_plan_bytes(rb, re), "gcn_plan: plan buffer too small");
    const int64_t ntiles = (re - rb + 63) / 64;
    const unsigned grid = static_cast<unsigned>(ntiles < (1 << 20) ? ntiles : (1 << 20));
    hipLaunchKernelGGL(gcn_plan_kernel, dim3(grid), dim3(64), 0, as_stream(stream), row_ptr, col, ew,
                       rb, re, ntiles, 4 * h, static_cast<uint4*>(plan));
    return launch_status("gcn_plan_kernel");
}

static int check_tile_args(const void* plan, const int32_t* row_ptr, const int32_t* col,
                           const float* ew, const float* x, int64_t ldx, int64_t rb, int64_t re,
                           int h, const float* out, int64_t ldo, const char* what) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && x && out, "%s: null pointer", what);
    MIGNN_REQUIRE(h == 64 || h == 128, "%s: h must be 64 or 128 (got %d)", what, h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(plan), "%s: unaligned", what);
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "%s: bad strides", what);
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "%s: bad row range", what);
    MIGNN_REQUIRE(x != out, "%s: in-place not supported (neighbours read x)", what);
    return MIGNN_OK;
}

extern "C" int mignn_gcn_layer_planned(const void* plan, const int32_t* row_ptr,
                                       const int32_t* col, const float* ew, const float* x,
                                       int64_t ldx, int64_t rb, int64_t re, int h, const float* w,
                                       const float* bias, const float* scale, const float* shift,
                                       int flags, float* out, int64_t ldo, void* stream) {
    if (int rc = check_tile_args(plan, row_ptr, col, ew, x, ldx, rb, re, h, out, ldo,
                                 "gcn_layer_planned"))
        return rc;
    MIGNN_REQUIRE(w && aligned16(w), "gcn_layer_planned: weight");
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_planned: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_planned: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_planned: affine");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    return h == 128 ? launch_tile<128, false>(plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale,
                                              shift, flags, out, ldo, st)
                    : launch_tile<64, false>(plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale,
                                             shift, flags, out, ldo, st);
}

extern "C" int mignn_gcn_aggregate_planned(const void* plan, const int32_t* row_ptr,
                                           const int32_t* col, const float* ew, const float* x,
                                           int64_t ldx, int64_t rb, int64_t re, int h, float* out,
                                           int64_t ldo, void* stream) {
    if (int rc = check_tile_args(plan, row_ptr, col, ew, x, ldx, rb, re, h, out, ldo,
                                 "gcn_aggregate_planned"))
        return rc;
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    return h == 128 ? launch_tile<128, true>(plan, row_ptr, col, ew, x, ldx, rb, re, nullptr, nullptr,
                                             nullptr, nullptr, 0, out, ldo, st)
                    : launch_tile<64, true>(plan, row_ptr, col, ew, x, ldx, rb, re, nullptr, nullptr,
                                            nullptr, nullptr, 0, out, ldo, st);
}

// timing ablations of the tile kernels (MODE above; results wrong by design
// for mode != 0): agg = 1 the aggregate alone
#ifdef MIGNN_DIAG
extern "C" int mignn_diag_gcn_tile(int mode, int agg, const void* plan, const int32_t* row_ptr,
                                   const int32_t* col, const float* ew, const float* x,
                                   int64_t ldx, int64_t rb, int64_t re, int h, const float* w,
                                   const float* bias, const float* scale, const float* shift,
                                   int flags, float* out, int64_t ldo, void* stream) {
    if (int rc = check_tile_args(plan, row_ptr, col, ew, x, ldx, rb, re, h, out, ldo, "diag_gcn_tile"))
        return rc;
    MIGNN_REQUIRE(h == 128, "diag_gcn_tile: h = 128 only");
    // (the fused layer's waits count its row stores: mode 8 only for the aggregate)
    MIGNN_REQUIRE(agg || !(mode & 8), "diag_gcn_tile: mode 8 needs agg");
    hipStream_t st = as_stream(stream);
#define MIGNN_TILE_MODE(M)                                                                      \
    case M:                                                                                     \
        return agg ? launch_tile<128, true, M>(plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, \
                                               scale, shift, flags, out, ldo, st)               \
                   : launch_tile<128, false, M>(plan, row_ptr, col, ew, x, ldx, rb, re, w,      \
                                                bias, scale, shift, flags, out, ldo, st);
    switch (mode) {
        MIGNN_TILE_MODE(0) MIGNN_TILE_MODE(1) MIGNN_TILE_MODE(2) MIGNN_TILE_MODE(3)
        MIGNN_TILE_MODE(4) MIGNN_TILE_MODE(8) MIGNN_TILE_MODE(11) MIGNN_TILE_MODE(15)
        MIGNN_TILE_MODE(12) MIGNN_TILE_MODE(7)
        default: break;
    }
#undef MIGNN_TILE_MODE
    set_error("diag_gcn_tile: unknown mode %d", mode);
    return MIGNN_ERR_ARG;
}
#endif
