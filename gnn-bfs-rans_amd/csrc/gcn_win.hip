// Fused GCN layer, window form -- the north-star hot kernel (GCNConv + residual
// + BatchNorm(eval) + ReLU, reference gnn_model.py:63, :166, :184-191; PyG
// GCNConv: out_i = sum_{j->i} w_ij h_j + b, w_ij = dinv_i dinv_j over
// add_remaining_self_loops):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Arithmetic: fp32 aggregation, the aggregate split into fp16 hi + lo with a
// power-of-two row scale, three fp16 MFMA products with fp32 accumulation
// (~2^-22 relative per product) -- gcn_f16x3.hip's scheme.
//
// Why this structure.  Per 64-row tile a fused layer streams 64 rows in and
// 64 rows out of its CU; what else crosses the CU is the tile's out-of-tile
// ("ext") neighbour rows.  With 4 x 4 x 4-cell tiles (the block order) that is
// 96 rows per tile -- 1.5 per own row, L2 -> LDS traffic larger than the own
// rows themselves, and the measured lever of the ring kernel (gcn_ring.hip:
// from the zero row its aggregation ran 2.26 -> 1.84 ms).  Here a tile is one
// z-plane of an 8 x 8-cell column (the column order,
// mignn_locality_order_cols) and a workgroup walks its column along z, so the
// previous and the current tile stay in LDS: a row's -z neighbour is in the
// previous tile, its in-plane neighbours in the current one, its +z neighbour
// in the next tile -- DMA'd a step ahead anyway, its one term is added at the
// next step ("phase B": the row's partial sum is carried in registers).  Only
// the 4 x 8 lateral face rows of a plane are ext rows: 0.5 per own row.
//
// Pipeline of step s (tile s = this workgroup's s-th tile; LDS slot s % 3):
//   B0  ext rows of step s landed (older: own rows of tile s + 1, records)
//   P1  phase A of tile s (in-window and ext entries, CSR order, the +z entry
//       held back), phase B of tile s - 1 (its +z term, from tile s), split
//       of tile s - 1 into the A image, its residual seeds
//   B2  A image complete, slot (s-1) % 3 and the ext area free
//       -> DMA ext rows of step s + 1, records of step s + 2, own rows of
//       tile s + 2 into slot (s+2) % 3 (issued between the MFMAs)
//   MFMA (tile s - 1, W split in registers)  B3  staging  B4  whole-row stores
// Every global read of the tile loop is an LDS-DMA counted by hand
// (global_load_lds_dwordx4); one workgroup per CU at H = 128 (8 waves), two
// at H = 64.
//
// Schedule (the plan header; mignn_gcn_win_plan): rounds of L steps -- in
// round r workgroup p (XCD-major position) walks tiles [(rG + p) L, +L), a
// column or a z-segment of one, while its XCD's workgroups walk the next
// columns of the same y-row -- for the full columns of the order, then the
// remaining tiles as contiguous chunks.  Any CSR is correct under any order:
// the plan classifies every entry by where its row is resident at that step.
// Plan records: 16 B per row -- slots 0..6 u16 codes in CSR order (code = the
// LDS offset of the neighbour row, >> 1 at H = 128, | its degree class), slot
// 7 the +z (next-tile) entry; the weights dinv_j dinv_i are rebuilt in LDS
// from the classes (win_rexp).  Waves with a row outside that form (degree >
// 8, ext capacity exceeded, a weight that is not dv[c_j] dv[c_i]) take the
// CSR path (row_ptr / col / ew, global x).
#include <type_traits>

#include "common.hpp"

namespace mignn {
MIGNN_DMA_OOB_WORD
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_w;
using f16x8w = __attribute__((ext_vector_type(8))) _Float16;
using f16x4w = __attribute__((ext_vector_type(4))) _Float16;

// A-fragment prefetch depth of the H = 128 transform, in t-steps of 3 MFMAs
// (10M-row layer: PD 1 2.87 ms, 2 2.72, 3 2.68, 5 2.67).  Measured and
// removed (round 6 prune): the staged whole-row epilogue at H = 128 (two
// more block barriers per step, 2.92 vs 2.87 ms), 4 column pairs x 32 rows
// per wave (2.79-3.05 vs 2.78 ms), the codes expansion as VALU fma chains
// (3.14-3.27 vs the MFMA expansion's 2.71 ms).
#ifndef MIGNN_WIN_PD
#define MIGNN_WIN_PD 3
#endif
constexpr int kWinPD = MIGNN_WIN_PD;
// Plan record of a row: 8 u16 codes (16 B), each with the neighbour's degree
// class in its low 3 bits (the code's LDS offset is 16-B aligned: those bits
// are free), plus the row's own class in a nibble of its wave's list.  The
// weight w_ij = dinv_j dinv_i is rebuilt in LDS from the plan's class table
// (round 6: 48 -> 16 B per row; the 8 f32 weights were 0.32 GB per launch)
constexpr int kWRec = 16;                 // plan bytes per row (global)
constexpr int kWA = 7;                    // slots 0..6: phase A; slot 7: the next-tile entry
constexpr int kWHdr = 256;                // plan header bytes
constexpr uint32_t kWMagic = 0x4E495747u;

// H = 128: the A-image kernel (gcn_win_kernel).  8 waves per workgroup, one
// workgroup per CU.  (16 waves -- four per SIMD, RPW = 4 -- measured slower:
// 3.27 vs 2.94 ms per 10M-row layer, the aggregate alone faster: 2.16 vs
// 2.26 ms)
template <int H>
struct WCfg {
    static_assert(H == 128, "window GCN layer, A-image form: H = 128");
    static constexpr int SWZ = 7;                      // own / ext row swizzle: chunk ^ (row & SWZ)
    static constexpr int BM = 64, NW = 8, NT = NW * 64;
    static constexpr int RPW = BM / NW;                // rows per wave (quad layout: RPW / 4 quads)
    static constexpr int F = H / 16, CH = F / 4;       // floats / 16-B chunks per lane of a row
    static constexpr int ROWB = H * 4;
    static constexpr int X_BYTES = BM * ROWB;
    static constexpr int NSLOT = 3;                    // own-row slots: tiles s-1, s, s+1
    static constexpr int KX = 32;                      // ext rows per tile (an 8x8 plane's faces)
    static constexpr int EXT_BYTES = KX * ROWB;
    static constexpr int EPW = KX / NW;                // ext rows DMA'd per wave
    static constexpr int XLW = (EPW + 4) / 4 * 4;      // ext-list group per wave: EPW columns, summary, row classes
    static constexpr int RECG = RPW * kWRec + XLW * 4; // a wave's codes + list in the plan (DMA'd as is)
    static constexpr int OFF_RL = RPW * kWRec;         // in a wave's LDS records: the list
    static constexpr int OFF_RW = RECG;                // the weights [RPW][8] (rebuilt in LDS)
    static constexpr int RECW = RECG + RPW * 32;       // a wave's records in LDS
    static constexpr int TLANES = RECG / 16;
    static constexpr int TAB_G = NW * RECG;            // plan bytes per tile
    static constexpr int TAB_BYTES = NW * RECW;        // LDS bytes per tile
    static constexpr int A_BYTES = BM * H * 2;         // hi or lo image (16-B chunks swizzled)
    // LDS: X[3] | EXT | ZERO (the code-addressed region) | TAB[2] | AH | AL | REXP | EPI | DV
    static constexpr int OFF_X = 0;
    static constexpr int OFF_EXT = NSLOT * X_BYTES;
    static constexpr int OFF_ZERO = OFF_EXT + EXT_BYTES;
    static constexpr int CODE_END = OFF_ZERO + ROWB;
    static constexpr int CSH = H == 64 ? 0 : 1;        // code = LDS byte offset >> CSH
    static constexpr int OFF_TAB = CODE_END;
    static constexpr int OFF_AH = OFF_TAB + 2 * TAB_BYTES;
    static constexpr int OFF_AL = OFF_AH + A_BYTES;
    static constexpr int OFF_REXP = OFF_AL + A_BYTES;
    static constexpr int OFF_EPI = OFF_REXP + BM * 4;
    static constexpr int OFF_DV = OFF_EPI + 3 * H * 4; // the plan's dinv table [8]
    static constexpr int LDS_BYTES = OFF_DV + 32;
    // layer 1 from layer-0 codes (MODE 64): per wave 8 own-row + 4 ext-row
    // codes (32 B each) DMA'd per step, the [H][8] expansion table
    static constexpr int CODEB = 32, CODE_W = (RPW + KX / NW) * CODEB;
    static constexpr int OFF_CODE = LDS_BYTES;
    static constexpr int OFF_COEF = OFF_CODE + NW * CODE_W;
    static constexpr int LDS_BYTES_X0 = OFF_COEF + H * 8 * 4;
    static constexpr int WGPC = H == 64 ? 2 : 1;       // workgroups per CU
    static constexpr int NQ = RPW / 4;                 // row quads per wave
    static constexpr int KC = H / 32;
    static constexpr int RPP = 1024 / ROWB, LPR = 64 / RPP;   // rows / lanes per row of a DMA piece
    static constexpr int NPX = X_BYTES / 1024 / NW;    // own-row pieces per wave
    static constexpr int NPE = EXT_BYTES / 1024 / NW;  // ext pieces per wave
    static constexpr int LPRW = ROWB / 16, RPI = 64 / LPRW;
    static constexpr int NST = RPW / RPI;              // row stores per wave
    static_assert(LDS_BYTES * WGPC <= 160 * 1024, "LDS budget");
    static_assert(LDS_BYTES_X0 * WGPC <= 160 * 1024, "LDS budget (codes form)");
    static_assert(RPW == 8 && KX / NW == 4 && CODE_W / 16 <= 64, "codes DMA: 16 own + 8 ext lanes");
    static_assert(EPW == NPE * RPP && EPW + 1 + RPW / 8 <= XLW, "ext rows per wave, row classes");
    static_assert((CODE_END >> CSH) <= 65536, "u16 codes");
    static_assert(RECG % 16 == 0 && TLANES <= 64 && RECW % 16 == 0, "records DMA");
};

// H = 64: the wave-independent kernel (gcn_win64_kernel).  4 waves of 16 rows
// per workgroup, two workgroups per CU (2 waves per SIMD, 256 VGPRs): each
// wave aggregates its rows straight into the MFMA B-operand layout (lane
// (r, g): row r, columns 32 kc + 8 g .. +7), splits and transforms them with
// W in registers and stages its own output rows -- no A image, no cross-wave
// hand-off, two barriers per step.  Rows are swizzled by (row & 15) so that
// the 16 rows of a wave's b128 reads land on distinct banks.
template <>
struct WCfg<64> {
    static constexpr int H = 64, SWZ = 15;
    static constexpr int BM = 64, NW = 4, NT = NW * 64;
    static constexpr int RPW = BM / NW;                // 16
    static constexpr int ROWB = H * 4;
    static constexpr int X_BYTES = BM * ROWB;
    static constexpr int NSLOT = 3;
    static constexpr int KX = 32;
    static constexpr int EXT_BYTES = KX * ROWB;
    static constexpr int EPW = KX / NW;                // 8
    static constexpr int XLW = (EPW + 4) / 4 * 4;      // 12
    static constexpr int RECG = RPW * kWRec + XLW * 4;
    static constexpr int OFF_RL = RPW * kWRec, OFF_RW = RECG;
    static constexpr int RECW = RECG + RPW * 32;
    static constexpr int TLANES = RECG / 16;
    static constexpr int TAB_G = NW * RECG;
    static constexpr int TAB_BYTES = NW * RECW;
    static constexpr int STG_BYTES = RPW * ROWB;       // a wave's output staging
    // LDS: X[3] | EXT | ZERO (code-addressed) | TAB[2] | STG[NW] | EPI | DV
    static constexpr int OFF_X = 0;
    static constexpr int OFF_EXT = NSLOT * X_BYTES;
    static constexpr int OFF_ZERO = OFF_EXT + EXT_BYTES;
    static constexpr int CODE_END = OFF_ZERO + ROWB;
    static constexpr int CSH = 0;
    static constexpr int OFF_TAB = CODE_END;
    static constexpr int OFF_STG = OFF_TAB + 2 * TAB_BYTES;
    static constexpr int OFF_EPI = OFF_STG + NW * STG_BYTES;
    static constexpr int OFF_DV = OFF_EPI + 3 * H * 4;
    static constexpr int LDS_BYTES = OFF_DV + 32;
    static constexpr int WGPC = 2;
    static constexpr int RPP = 1024 / ROWB, LPR = 64 / RPP;   // 4 rows of 16 lanes per DMA piece
    static constexpr int NPX = X_BYTES / 1024 / NW;    // 4
    static constexpr int NPE = EXT_BYTES / 1024 / NW;  // 2
    static constexpr int NST = RPW / RPP;              // 4 whole-row stores per wave
    static_assert(LDS_BYTES * WGPC <= 160 * 1024, "LDS budget");
    static_assert(EPW == NPE * RPP && EPW + 1 + RPW / 8 <= XLW, "ext rows per wave, row classes");
    static_assert(CODE_END <= 65536, "u16 codes");
    static_assert(RECG % 16 == 0 && TLANES <= 64 && RECW % 16 == 0 && OFF_STG % 16 == 0, "records DMA");
};

// ------------------------------------------------------------------ schedule
// Plan header (first kWHdr bytes of the plan).  Round / chunk schedule: for
// s < R1 L, workgroup position p at step s has tile ((s / L) G + p) L + s % L;
// then tiles [t2, ntiles) as chunks of `chunk` per position.
struct WinHdr {
    uint32_t magic;
    int32_t G, h, L;
    int32_t R1, chunk, nsteps, Z;
    int64_t ntiles, t2, rb, re;
    int32_t zrun;   // (plan build) tiles from tile 0 that chain as z-planes of one column
    float dv[8];    // degree class c -> dinv = (c + 1)^-1/2 (csr_finalize_kernel's expression)
};
static_assert(sizeof(WinHdr) <= kWHdr, "plan header");

struct WinSched {
    int64_t ntiles, t2;
    int G, L, R1, chunk;
};

__host__ __device__ inline int64_t win_tile(const WinSched& S, int p, int64_t s) {
    if (s < 0) return -1;
    const int64_t s1 = static_cast<int64_t>(S.R1) * S.L;
    if (s < s1) return ((s / S.L) * S.G + p) * S.L + s % S.L;
    const int64_t j = s - s1;
    if (j >= S.chunk) return -1;
    const int64_t t = S.t2 + static_cast<int64_t>(p) * S.chunk + j;
    return t < S.ntiles ? t : -1;
}

// 32-bit forms for the plan kernel (tiles < 2^25: rows are int32)
__device__ inline int win_tile32(const WinSched& S, int p, int s) {
    if (s < 0) return -1;
    const int s1 = S.R1 * S.L;
    if (s < s1) return ((s / S.L) * S.G + p) * S.L + s % S.L;
    const int j = s - s1;
    if (j >= S.chunk) return -1;
    const int t = static_cast<int>(S.t2) + p * S.chunk + j;
    return t < S.ntiles ? t : -1;
}
__device__ inline void win_where32(const WinSched& S, int t, int& p, int& s) {
    const int t2 = static_cast<int>(S.t2);
    if (t < t2) {
        const int i = t / S.L;
        p = i % S.G;
        s = (i / S.G) * S.L + t % S.L;
    } else {
        const int u = t - t2;
        p = u / S.chunk;
        s = S.R1 * S.L + u % S.chunk;
    }
}

// the column run of the plan's rows: tile t + 1 continues tile t as the next
// z-plane of its column when tile t's first row has tile t + 1's first row
// among its entries; zrun = the first t + 1 where that breaks (a column's
// plane count from the CSR itself -- a shard's interior range has the column
// order with its boundary planes moved out, fewer planes than the order's Z)
__global__ void win_zrun_init_kernel(WinHdr* hdr, int64_t ntiles) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        hdr->zrun = static_cast<int32_t>(ntiles < (1ll << 30) ? ntiles : (1ll << 30));
}
__global__ void win_zrun_kernel(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                                int64_t rb, int64_t re, int64_t ntiles, WinHdr* hdr) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t + 1 < ntiles;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r0 = rb + t * 64, r1 = r0 + 64;
        bool cont = false;
        if (r1 < re)
            for (int32_t e = row_ptr[r0]; e < row_ptr[r0 + 1]; ++e) cont |= col[e] == r1;
        if (!cont) atomicMin(&hdr->zrun, static_cast<int32_t>(t + 1));
    }
}

// the header: schedule parameters from the order's column info (nullable:
// {1, Z tiles per full column, full columns, ...}, mignn_locality_order_cols),
// Z capped by the CSR's own column run (win_zrun_kernel)
__global__ void win_hdr_kernel(WinHdr* hdr, const int32_t* __restrict__ info, int64_t ntiles, int G,
                               int h, int64_t rb, int64_t re) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t Z = 0, C = 0;
    if (info != nullptr && info[0] == 1) {
        Z = info[1] < hdr->zrun ? info[1] : hdr->zrun;
        C = info[2];
    }
    // contiguous chunks (no column structure)
    int bestL = 1, bestR1 = 0;
    int64_t bestChunk = (ntiles + G - 1) / G;
    double best = 1.25 * static_cast<double>(bestChunk);
    if (Z > 0 && C > 0) {
        for (int nseg = 1; nseg <= 16; ++nseg) {
            if (Z % nseg != 0 || Z / nseg < 4) continue;
            const int64_t L = Z / nseg;
            int64_t R1 = (C * nseg) / G;
            const int64_t rmax = ntiles / (static_cast<int64_t>(G) * L);
            if (R1 > rmax) R1 = rmax;
            if (R1 <= 0) continue;
            const int64_t t2 = R1 * G * L;
            const int64_t chunk = (ntiles - t2 + G - 1) / G;
            const double S = static_cast<double>(R1 * L + chunk);
            // steps, window breaks (one per segment), the chunks' poorer locality
            const double cost = S * (1.0 + 0.02 * nseg) + 0.25 * static_cast<double>(chunk);
            if (cost < best) {
                best = cost;
                bestL = static_cast<int>(L);
                bestR1 = static_cast<int>(R1);
                bestChunk = chunk;
            }
        }
    }
    hdr->magic = kWMagic;
    hdr->G = G;
    hdr->h = h;
    hdr->L = bestL;
    hdr->R1 = bestR1;
    hdr->chunk = static_cast<int32_t>(bestChunk);
    hdr->nsteps = static_cast<int32_t>(static_cast<int64_t>(bestR1) * bestL + bestChunk);
    hdr->Z = static_cast<int32_t>(Z);
    hdr->ntiles = ntiles;
    hdr->t2 = static_cast<int64_t>(bestR1) * G * bestL;
    hdr->rb = rb;
    hdr->re = re;
    for (int c = 0; c < 8; ++c) hdr->dv[c] = 1.0f / sqrtf(static_cast<float>(c + 1));
}

__device__ inline WinSched win_sched(const WinHdr* h) {
    WinSched S;
    S.ntiles = h->ntiles;
    S.t2 = h->t2;
    S.G = h->G;
    S.L = h->L;
    S.R1 = h->R1;
    S.chunk = h->chunk;
    return S;
}

// the tile of step s = q L + m (0 <= m < L): the kernels walk (q, m) one
// step at a time -- win_tile's 64-bit s / L, s % L are long scalar sequences
struct WinCursor {
    int s, q, m;
    __device__ __forceinline__ void next(int L) {
        ++s;
        if (++m == L) {
            m = 0;
            ++q;
        }
    }
};
__device__ __forceinline__ int64_t win_tile_c(const WinSched& S, int p, const WinCursor& c) {
    if (c.q < S.R1) return static_cast<int64_t>(c.q * S.G + p) * S.L + c.m;
    const int j = c.s - S.R1 * S.L;
    if (j >= S.chunk) return -1;
    const int64_t t = S.t2 + static_cast<int64_t>(p) * S.chunk + j;
    return t < S.ntiles ? t : -1;
}

int win_grid(int64_t ntiles, int wgpc) {
    static int cus_cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    int& cus = cus_cache[dev & 63];
    if (cus == 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -1;
        cus = c < 1 ? 1 : c;
    }
    int G = (cus * wgpc / 8) * 8;
    if (G < 8) G = 8;
    if (ntiles < G) G = static_cast<int>(((ntiles + 7) / 8) * 8);
    return G;
}

// the device word for plan / launch mismatches (mignn_device_errors)
__device__ unsigned int g_win_errors = 0u;

constexpr int wvm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xF00; }   // vmcnt(n)
constexpr int kWLgkm0 = 0xC07F;

template <int W>
__device__ __forceinline__ void wwait() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(W);
    asm volatile("" ::: "memory");
}
template <int W>
__device__ __forceinline__ void wbar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(W);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// The H = 128 epilogue stores 64-B row pieces (each of 8 waves its 16
// columns of 16 rows, at different times of a step): plain stores, so L2
// merges a row's pieces into whole lines -- as nontemporal stores 1/3 of the
// lines went to HBM in pieces (WRITE_SIZE 6.83 vs 5.12 GB per 10M-row launch,
// 2.2 % of the layer's time; `profiles/r06_kpmc_st_*.json`)
__device__ __forceinline__ void wstore(const f32x4& v, f32x4* p) { *p = v; }

__device__ __forceinline__ uint32_t wlds(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_w)(p)));
}

__device__ __forceinline__ void wdma(const void* src, uint32_t dst) {
    MIGNN_DMA_BOUND(dst);
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

__device__ __forceinline__ uint64_t wuni(const void* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<int>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void wdma_s(const void* base, uint32_t voff, uint32_t dst) {
    MIGNN_DMA_BOUND(dst);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(wuni(base)), "s"(__builtin_amdgcn_readfirstlane(static_cast<int>(dst)))
        : "memory");
}

__device__ __forceinline__ int wsplit_exp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}
__device__ __forceinline__ uint32_t wrow_max(uint32_t v) {
    int t = static_cast<int>(v);
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x124, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x128, 0xf, 0xf, false)));
    return static_cast<uint32_t>(t);
}
__device__ __forceinline__ uint32_t wwave_max(uint32_t v) {
    const uint32_t t = wrow_max(v);
    const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 0));
    const uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 16));
    const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 32));
    const uint32_t d = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 48));
    return max(max(a, b), max(c, d));
}

// A-image 16-B chunk swizzle of row R (conflict-free fragment reads: the
// lanes of one ds_read_b128 group cover the 64 banks once)
template <int H>
__device__ __forceinline__ int asw(int R) {
    return H == 64 ? ((R >> 1) & 7) : (R & 15);
}

__device__ __attribute__((aligned(16))) float g_win_zero_row[256];

// diagnostic timeline (mignn_diag_win_trace): s_memtime stamps of waves 0
// and 4 of workgroups 0..7, steps 0..63 -> trace[((b * 64 + s) * 2 + w/4) * 16 + point]
#ifdef MIGNN_DIAG
__device__ unsigned long long* g_win_trace = nullptr;
#endif
struct WTrace {
    unsigned long long* tr;   // null: tracing off (the product build)
    uint32_t lo, hi;
    int lane;
    __device__ __forceinline__ void stamp(int pt) {
        if (tr == nullptr) return;
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        lo = lane == pt ? static_cast<uint32_t>(t) : lo;
        hi = lane == pt ? static_cast<uint32_t>(t >> 32) : hi;
    }
    __device__ __forceinline__ void flush(int wave, int64_t s) {
        if (tr == nullptr || blockIdx.x >= 8 || s < 0 || s >= 64 || (wave != 0 && wave != 4)) return;
        if (lane < 8)
            tr[((blockIdx.x * 64 + s) * 2 + (wave >> 2)) * 16 + lane] =
                (static_cast<unsigned long long>(hi) << 32) | lo;
    }
};

// The weights of a wave's records in LDS (RW: its TAB slot region), from
// the codes' degree classes: lane (row, slot) writes w = dv[c_j] dv[c_i]
// (csr_finalize_kernel's dinv_j * dinv_i, bitwise -- the plan checked every
// entry) and clears the code's class bits.  Run on records this wave DMA'd
// itself once its vmcnt covers them; wave-local (LDS is in order within a
// wave), so no barrier.
template <class C>
__device__ __forceinline__ void win_rexp(unsigned char* RW, const float* DV, int lane) {
    // (lane opaque: its offsets hoisted out of the step loop would be live
    // through the kernels' register peak)
    asm volatile("" : "+v"(lane));
#pragma unroll
    for (int it = 0; it < C::RPW / 8; ++it) {
        const int row = 8 * it + (lane >> 3), u = lane & 7;
        uint16_t* const cp = reinterpret_cast<uint16_t*>(RW + row * kWRec) + u;
        const uint32_t cd = *cp;
        const uint32_t cw = *reinterpret_cast<const uint32_t*>(RW + C::OFF_RL + 4 * (C::EPW + 1 + it));
        const uint32_t ci = (cw >> (4 * (row & 7))) & 7u;
        *reinterpret_cast<float*>(RW + C::OFF_RW + row * 32 + 4 * u) = DV[cd & 7u] * DV[ci];
        *cp = static_cast<uint16_t>(cd & ~7u);
    }
}

// ------------------------------------------------------------------ plan
// One 64-thread block per tile, a thread per row.  Entry classes at the
// tile's step: the current tile (slot s % 3), the workgroup's previous tile
// ((s-1) % 3), the first entry in its next tile ((s+1) % 3, slot 7: phase B),
// else an ext slot (numbered in row-major order of the tile's ext entries, a
// wave-wide prefix sum; slot k at LDS ext row k, its column in list entry
// (k / EPW) * XLW + k % EPW); a row with more than 7 phase-A entries, more
// than 8 entries or an ext slot past KX makes its wave take the CSR path.
template <int H>
__global__ __launch_bounds__(64) void win_plan_kernel(const int32_t* __restrict__ row_ptr,
                                                      const int32_t* __restrict__ col,
                                                      const float* __restrict__ ew,
                                                      const WinHdr* __restrict__ hdr,
                                                      unsigned char* __restrict__ tabs,
                                                      unsigned long long* __restrict__ stats) {
    using C = WCfg<H>;
    const int lr = threadIdx.x;
    const WinSched S = win_sched(hdr);
    const int64_t rb = hdr->rb, re = hdr->re, ntiles = hdr->ntiles;
    __shared__ uint32_t xl[C::NW * C::XLW];
    const uint32_t zcode = static_cast<uint32_t>(C::OFF_ZERO >> C::CSH);
    float dv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) dv[c] = hdr->dv[c];
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        int p, s;
        win_where32(S, static_cast<int>(t), p, s);
        const int64_t tprev = win_tile32(S, p, s - 1), tnext = win_tile32(S, p, s + 1);
        const int sc = static_cast<int>(s % 3), sp = static_cast<int>((s + 2) % 3),
                  sn = static_cast<int>((s + 1) % 3);
        const int64_t t0 = rb + t * C::BM;
        const int64_t nloc = re - t0 < C::BM ? re - t0 : C::BM;
        auto in_tile = [&](int64_t c, int64_t tt, int64_t& off) -> bool {
            if (tt < 0) return false;
            const int64_t b0 = rb + tt * C::BM;
            const int64_t nl = re - b0 < C::BM ? re - b0 : C::BM;
            off = c - b0;
            return off >= 0 && off < nl;
        };
        auto xcode = [&](int slot, int64_t off) -> uint32_t {
            const uint32_t o = static_cast<uint32_t>(off);
            return ((C::OFF_X + slot * C::X_BYTES + o * C::ROWB) | ((o & C::SWZ) << 4)) >> C::CSH;
        };
        for (int i = lr; i < C::NW * C::XLW; i += 64) xl[i] = 0u;   // unused: row 0, never read
        const int64_t r = t0 + lr;
        int e0 = 0, deg = 0;
        if (lr < nloc) {
            e0 = row_ptr[r];
            deg = row_ptr[r + 1] - e0;
        }
        // the row's entries, loaded at once into registers (a loop over deg
        // serialised one load latency per entry); rows of degree > 8 take
        // the CSR path -- their entries are not read, their ext slots not
        // counted
        const bool small = deg <= 8;
        int cj[8];
        uint32_t wj[8];
        if (small && deg > 0) {
            // (loads unconditional, past the row's end clamped to its last
            // entry: no per-entry branches between them)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int ek = e0 + (e < deg ? e : deg - 1);
                const int cv = col[ek];
                const uint32_t wv = __float_as_uint(ew[ek]);
                cj[e] = e < deg ? cv : -1;
                wj[e] = e < deg ? wv : 0u;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                cj[e] = -1;
                wj[e] = 0u;
            }
        }
        // degree classes: the row's own from its self entry (weight dv[c]^2),
        // each entry's c_j with weight == dv[c_j] dv[c_i] bitwise (the
        // kernel rebuilds exactly that product); a row with an entry outside
        // that form (no self entry, a weighted graph, a degree > 8) takes
        // the CSR path, which reads ew itself
        int ci = -1;
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (cj[e] >= 0 && static_cast<int64_t>(cj[e]) == r)
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    if (__float_as_uint(dv[c] * dv[c]) == wj[e]) ci = c;
        const float di = dv[ci >= 0 ? ci : 0];
        bool wok = ci >= 0 || deg == 0;
        uint32_t cls[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            int k = -1;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if (__float_as_uint(dv[c] * di) == wj[e]) k = c;
            if (cj[e] >= 0 && k < 0) wok = false;
            cls[e] = k >= 0 ? static_cast<uint32_t>(k) : 0u;
        }
        // pass 1: ext entries of the row
        int next = 0, nA = 0;
        bool haveN = false;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            if (cj[e] < 0) continue;
            const int64_t c = cj[e];
            int64_t off;
            if (in_tile(c, t, off) || in_tile(c, tprev, off)) {
                ++nA;
            } else if (!haveN && in_tile(c, tnext, off)) {
                haveN = true;
            } else {
                ++nA;
                ++next;
            }
        }
        int pre = next;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(pre, d, 64);
            if (lr >= d) pre += v;
        }
        pre -= next;
        __syncthreads();
        bool far = !small || nA > kWA || pre + next > C::KX || !wok;
        uint32_t code[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) code[q] = zcode;
        if (lr < nloc && deg > 0 && small) {
            int k = pre, a = 0;
            bool usedN = false;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (cj[e] < 0) continue;
                const int64_t c = cj[e];
                int64_t off;
                uint32_t cd;
                int slot;
                if (in_tile(c, t, off)) {
                    cd = xcode(sc, off);
                    slot = a++;
                } else if (in_tile(c, tprev, off)) {
                    cd = xcode(sp, off);
                    slot = a++;
                } else if (!usedN && in_tile(c, tnext, off)) {
                    usedN = true;
                    cd = xcode(sn, off);
                    slot = 7;
                } else {
                    if (k < C::KX) {
                        cd = ((C::OFF_EXT + k * C::ROWB) | ((static_cast<uint32_t>(k) & C::SWZ) << 4)) >> C::CSH;
                        xl[(k / C::EPW) * C::XLW + k % C::EPW] = static_cast<uint32_t>(c);
                    } else {
                        cd = zcode;
                    }
                    ++k;
                    slot = a++;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (q == slot) code[q] = cd | cls[e];
            }
        }
        // summary of the row's wave (RPW rows): max phase-A count | any CSR-path row
        uint32_t md = far ? 0u : static_cast<uint32_t>(nA), af = far ? 1u : 0u;
#pragma unroll
        for (int d = 1; d < C::RPW; d <<= 1) {
            md = max(md, static_cast<uint32_t>(__shfl_xor(static_cast<int>(md), d, C::RPW)));
            af |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(af), d, C::RPW));
        }
        if ((lr % C::RPW) == 0) xl[(lr / C::RPW) * C::XLW + C::EPW] = md | (af << 8);
        // the row's class: nibble lr % 8 of list word EPW + 1 + (lr % RPW) / 8
        if (lr < nloc && ci > 0)
            atomicOr(&xl[(lr / C::RPW) * C::XLW + C::EPW + 1 + (lr % C::RPW) / 8],
                     static_cast<uint32_t>(ci) << (4 * (lr & 7)));
        __syncthreads();
        // per wave: its rows' codes, then its list (one contiguous DMA)
        unsigned char* const base = tabs + t * C::TAB_G;
        *reinterpret_cast<uint4*>(base + (lr / C::RPW) * C::RECG + (lr % C::RPW) * kWRec) =
            make_uint4(code[0] | (code[1] << 16), code[2] | (code[3] << 16),
                       code[4] | (code[5] << 16), code[6] | (code[7] << 16));
        for (int i = lr; i < C::NW * C::XLW; i += 64)
            *reinterpret_cast<uint32_t*>(base + (i / C::XLW) * C::RECG + C::OFF_RL + 4 * (i % C::XLW)) = xl[i];
        if (stats != nullptr) {
            if (far && lr < nloc) atomicAdd(&stats[1], 1ull);
            const int kt = __shfl(pre + next, 63, 64);
            if (lr == 63 && kt > C::KX) atomicAdd(&stats[0], 1ull);
            if (lr == 63) atomicMax(&stats[3], static_cast<unsigned long long>(kt));
            if (haveN && lr < nloc) atomicAdd(&stats[2], 1ull);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- layer
// MODE: 32 aggregate only (mignn_gcn_aggregate_win: the fp32 sums are the
// output); 64 layer 1 from layer-0 codes (mignn_gcn_layer_win_codes: x =
// codes [rows, 8], xcoef = the [H][8] expansion, see "codes form" below);
// timing ablations (mignn_diag_win only): 1 ext rows from the zero
// row, 2 own rows from the zero row, 4 no MFMAs.  EPIF: the epilogue flags at compile time (15, 11; -1: from
// `flags`).
template <int H, int MODE = 0, int EPIF = -1>
__global__ __launch_bounds__(WCfg<H>::NT, WCfg<H>::NW / 4 * WCfg<H>::WGPC) void gcn_win_kernel(
    const unsigned char* __restrict__ plan, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ col, const float* __restrict__ ew, const float* __restrict__ x,
    int64_t ldx, int64_t rb, int64_t re, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo,
    const float* __restrict__ xcoef) {
    using C = WCfg<H>;
    constexpr bool AGG = (MODE & 32) != 0;
    constexpr bool X0 = (MODE & 64) != 0;
    static_assert(!X0 || !AGG, "codes form: the full layer only");
    if constexpr (EPIF >= 0) flags = EPIF;
    __shared__ __attribute__((aligned(16))) unsigned char lds[X0 ? C::LDS_BYTES_X0 : C::LDS_BYTES];
    _Float16* const AH = reinterpret_cast<_Float16*>(lds + C::OFF_AH);
    _Float16* const AL = reinterpret_cast<_Float16*>(lds + C::OFF_AL);
    int* const REXP = reinterpret_cast<int*>(lds + C::OFF_REXP);
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the two waves of a SIMD (w, w + NW / 2) at different priorities: both
    // meet at the same barriers and would reach their MFMA groups and their
    // LDS / VALU phases together; the first now runs ahead and the second
    // fills its gaps (same-box A/B, DESIGN 3.17: H = 128 -0.75 %, H = 64
    // -2.3 %, codes form -0.75 %)
    if (wave < C::NW / 2) __builtin_amdgcn_s_setprio(1);

    const WinHdr* const hdr = reinterpret_cast<const WinHdr*>(plan);
    {
        const bool ok = hdr->magic == kWMagic && hdr->G == static_cast<int>(gridDim.x) &&
                        hdr->h == H && hdr->rb == rb && hdr->re == re;
        if (!ok) {
            if (tid == 0)
                __hip_atomic_fetch_or(&g_win_errors, static_cast<unsigned>(MIGNN_DEVERR_PLAN),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            plan_mismatch_fill(out, ldo, rb, re, H);
            return;
        }
    }
    const WinSched S = win_sched(hdr);
    const unsigned char* const tabs = plan + kWHdr;
    const int per_xcd = static_cast<int>(gridDim.x) >> 3;
    const int p = (static_cast<int>(blockIdx.x) & 7) * per_xcd + (static_cast<int>(blockIdx.x) >> 3);
    auto tile_of = [&](int64_t s) -> int64_t { return win_tile(S, p, s); };
    if (tile_of(0) < 0) return;                   // no work (uniform): no DMA issued
#ifdef MIGNN_DIAG
    WTrace wtr{(blockIdx.x < 8 && (wave == 0 || wave == 4)) ? g_win_trace : nullptr, 0u, 0u, lane};
#else
    WTrace wtr{nullptr, 0u, 0u, lane};
#endif

    const int gq = lane >> 4, iq = lane & 15;
    const int hb = (iq >= 4 && iq < 12) ? 1 : 0;
    const int c0 = (hb ? iq - 4 : (iq < 4 ? iq : iq - 8)) | (hb << 3);
    const uint32_t coff0 = static_cast<uint32_t>(c0 << 4);
    auto decode = [&](uint32_t cd) -> uint32_t { return (cd << C::CSH) ^ coff0; };

    // own-row DMA of a tile: SGPR base, per-lane offsets fixed for the launch
    const uint32_t ldxb = static_cast<uint32_t>(ldx) * 4u;
    uint32_t xoff[C::NPX];
#pragma unroll
    for (int pp = 0; pp < C::NPX; ++pp) {
        const int pc = pp * C::NW + wave;
        const int lr = pc * C::RPP + lane / C::LPR;
        const int pos = lane % C::LPR;
        xoff[pp] = static_cast<uint32_t>(lr) * ldxb + 16u * static_cast<uint32_t>(pos ^ (lr & 7));
    }
    const uint32_t toff = static_cast<uint32_t>(wave * C::RECG + 16 * lane);
    // records of tile t (or tile 0: a dummy of the same op count) -> TAB slot q
    auto dma_tab = [&](int64_t t, int q) {
        if (lane < C::TLANES)
            wdma_s(tabs + (t >= 0 ? t : 0) * C::TAB_G, toff,
                   wlds(lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW));
    };
    // the weights of the wave's records in TAB slot q (landed: this wave's
    // own DMA, waited by vmcnt; wave-local, LDS in order -- no barrier):
    // lane (row, slot) writes dv[c_j] dv[c_i] and clears the code's class bits
    float* const DV = reinterpret_cast<float*>(lds + C::OFF_DV);
    auto rexp = [&](int q) { win_rexp<C>(lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW, DV, lane); };
    // own rows of tile t (dummy: tile 0) -> X slot q, piece pp
    auto dma_own = [&](int64_t t, int q, int pp) {
        const int64_t tt = t >= 0 ? t : 0;
        const int64_t t0 = rb + tt * C::BM;
        const int pc = pp * C::NW + wave;
        unsigned char* const X = lds + C::OFF_X + q * C::X_BYTES;
        if constexpr ((MODE & 2) != 0) {
            wdma(g_win_zero_row + 4 * (lane & 31), wlds(X + pc * 1024));
        } else if (t0 + C::BM <= re) {
            wdma_s(x + t0 * ldx, xoff[pp], wlds(X + pc * 1024));
        } else {
            int l = lane;
            asm volatile("" : "+v"(l));
            const int lr = pc * C::RPP + l / C::LPR;
            const int pos = l % C::LPR;
            int64_t row = t0 + lr;
            if (row >= re) row = re - 1;
            wdma(x + row * ldx + 4 * (pos ^ (lr & 7)), wlds(X + pc * 1024));
        }
    };
    // ext rows of the step whose records sit in TAB slot q (dummy: the zero row)
    auto ext_src = [&](int q, int i, bool real) -> const unsigned char* {
        const unsigned char* const tab = lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW + C::OFF_RL;
        int l = lane;
        asm volatile("" : "+v"(l));
        const int kk = i * C::RPP + l / C::LPR;
        const int k = wave * C::EPW + kk;
        const int pos = l % C::LPR;
        const uint32_t c = *reinterpret_cast<const uint32_t*>(tab + 4 * kk);
        return ((MODE & 1) || !real) ? reinterpret_cast<const unsigned char*>(g_win_zero_row + 4 * (pos & 31))
                                     : reinterpret_cast<const unsigned char*>(x) + static_cast<uint64_t>(c) * ldxb +
                                           16u * static_cast<uint32_t>(pos ^ (k & 7));
    };
    auto ext_dma = [&](int i, const unsigned char* src) {
        wdma(src, wlds(lds + C::OFF_EXT + (wave * C::EPW + i * C::RPP) * C::ROWB));
    };

    // ---- codes form (X0): layer 1 straight from layer 0's row codes.  Layer
    // 0 of the GCN stack is relu(coef . (c_i, C_i, s_i, 1)) per feature
    // (gcn_layer0.hip); mignn_gcn_layer0_codes writes the 32-B code (c, C, s,
    // 0) of a row instead of its 512-B row, and this kernel expands the rows
    // it needs into its LDS slots with the same fma chain (bitwise the rows
    // layer 0 would have written).  Per step a wave DMAs the codes of its 8
    // own rows of tile s + 2 (lanes 0..15) and of its 4 ext rows of step s + 1
    // (lanes 16..23, from the records in TAB slot q) into its CODE area and,
    // after the MFMAs, expands them into slot (s + 2) % 3 and the ext area.
    auto code_dma = [&](int64_t t, int q, bool ext) {
        if (lane < (ext ? 24 : 16)) {
            int l = lane;
            asm volatile("" : "+v"(l));
            int64_t row;
            if (l < 16) {
                const int64_t tt = t >= 0 ? t : 0;
                row = rb + tt * C::BM + C::RPW * wave + (l >> 1);
                if (row >= re) row = re - 1;
            } else {
                const unsigned char* const tab = lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW + C::OFF_RL;
                row = *reinterpret_cast<const uint32_t*>(tab + 4 * ((l - 16) >> 1));
            }
            wdma(x + row * ldx + 4 * (l & 1), wlds(lds + C::OFF_CODE + wave * C::CODE_W));
        }
    };
    // (COEF: the table k-major per 16-B feature chunk -- chunk c, input k
    // (7: the constant) -> features 4c .. 4c + 3 in one f32x4: per feature
    // the fma sequence of gcn_layer0.hip, which the compiler packs in pairs)
    // ---- the row expansion as f32 MFMAs: wave w computes
    // features 16 w .. 16 w + 15 of every expanded row, a 16-row block per
    // v_mfma_f32_16x16x4_f32 pair (inputs 0..3, then 4..6 and a zero; the
    // accumulator starts at the constant e) -- on gfx950 an exact fma chain
    // in k order, i.e. layer 0's chain -- off the VALU.  Lane l: A = the
    // coefficient of feature 16 w + (l & 15), input 4 kg + (l >> 4); B =
    // input 4 kg + (l >> 4) of row l & 15's code; D = features 16 w + 4 (l
    // >> 4) .. + 3 of row l & 15 (one 16-B chunk).  Row blocks 0..3: the
    // tile's own rows (CODE of wave j >> 3, row j & 7), 4, 5: its ext rows
    // (wave k >> 2, row RPW + (k & 3)) -- every wave reads every wave's codes.
    [[maybe_unused]] constexpr int NXB = (C::BM + C::KX) / 16;
    float xa0 = 0.f, xa1 = 0.f;
    f32x4 xe = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X0) {
        const int f = 16 * wave + (lane & 15), kq = lane >> 4;
        xa0 = xcoef[f * 8 + kq];
        xa1 = kq < 3 ? xcoef[f * 8 + 4 + kq] : 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) xe[v] = xcoef[(16 * wave + 4 * kq + v) * 8 + 7];
    }
    [[maybe_unused]] auto xblock_mfma = [&](int rbk) -> f32x4 {
        const int l16 = lane & 15, kq = lane >> 4;
        uint32_t off;
        if (rbk < C::BM / 16) {
            const int j = 16 * rbk + l16;
            off = (j >> 3) * C::CODE_W + (j & 7) * C::CODEB;
        } else {
            const int k = 16 * (rbk - C::BM / 16) + l16;
            off = (k >> 2) * C::CODE_W + (C::RPW + (k & 3)) * C::CODEB;
        }
        const float* const cp = reinterpret_cast<const float*>(lds + C::OFF_CODE + off);
        const float b0 = cp[kq], b1 = cp[4 + kq];
        const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(xa0, b0, xe, 0, 0, 0);
        return __builtin_amdgcn_mfma_f32_16x16x4f32(xa1, b1, d, 0, 0, 0);
    };
    [[maybe_unused]] auto xblock_store = [&](int slot, int rbk, const f32x4& d) {
        const int l16 = lane & 15, ch = 4 * wave + (lane >> 4);
        const f32x4 o = f32x4{relu_nan(d[0]), relu_nan(d[1]), relu_nan(d[2]), relu_nan(d[3])};
        unsigned char* dst;
        if (rbk < C::BM / 16) {
            const int r = 16 * rbk + l16;
            dst = lds + C::OFF_X + slot * C::X_BYTES + r * C::ROWB + ((ch ^ (r & 7)) << 4);
        } else {
            const int k = 16 * (rbk - C::BM / 16) + l16;
            dst = lds + C::OFF_EXT + k * C::ROWB + ((ch ^ (k & 7)) << 4);
        }
        *reinterpret_cast<f32x4*>(dst) = o;
    };

    // ------------------------------------------------------------ prologue
    for (int i = tid; i < C::ROWB / 4; i += C::NT) reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
    if (tid < 8) DV[tid] = hdr->dv[tid];
    if constexpr (X0)
        for (int i = tid; i < H * 2; i += C::NT) {   // i = chunk * 8 + k
            const int c4 = i >> 3, k = i & 7;
            const float* const src = xcoef + 4 * c4 * 8 + k;
            *reinterpret_cast<f32x4*>(lds + C::OFF_COEF + 16 * i) = f32x4{src[0], src[8], src[16], src[24]};
        }
    const int rr0 = lane & 15, gg0 = lane >> 4;
    constexpr int CPW = 1;                        // 16-column blocks per wave
    constexpr int WN = H / 16 / CPW, WM = C::NW / WN, IBW = (C::BM / 16) / WM;
    static_assert(WN * WM == C::NW && IBW * WM * 16 == C::BM, "window transform grid");
    const int wn = wave % WN, wm = wave / WN;
    const int n0 = 16 * CPW * wn;
    f16x8w wh[CPW][C::KC], wl[CPW][C::KC];
    int qw[CPW];
    if constexpr (!AGG) {
#pragma unroll
        for (int cp = 0; cp < CPW; ++cp) {
            float wv[C::KC][8];
            uint32_t m = 0;
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                const float* pw = W + static_cast<int64_t>(n0 + 16 * cp + rr0) * H + 32 * kc + 8 * gg0;
                const float4 a = ld4(pw), b = ld4(pw + 4);
                float* w8 = wv[kc];
                w8[0] = a.x; w8[1] = a.y; w8[2] = a.z; w8[3] = a.w;
                w8[4] = b.x; w8[5] = b.y; w8[6] = b.z; w8[7] = b.w;
#pragma unroll
                for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(fabsf(w8[j])));
            }
            qw[cp] = wsplit_exp(wwave_max(m));    // one exponent per 16-column block
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float sv = ldexpf(wv[kc][j], qw[cp]);
                    const _Float16 hh = static_cast<_Float16>(sv);
                    wh[cp][kc][j] = hh;
                    wl[cp][kc][j] = static_cast<_Float16>(sv - static_cast<float>(hh));
                }
        }
        if (wm == 0 && lane < 16 * CPW) {
            const int n = n0 + lane;
            EPI[n] = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
            EPI[H + n] = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
            EPI[2 * H + n] = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
        }
    }
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;

    // records and rows of steps 0 and 1, then step 0's ext rows
    if constexpr (X0) {
        dma_tab(tile_of(0), 0);
        dma_tab(tile_of(1), 1);
        code_dma(tile_of(0), 0, false);
        wbar<wvm(0) & kWLgkm0>();                 // (all waves), zero row, EPI, COEF
        rexp(0);
#pragma unroll
        for (int rbk = 0; rbk < C::BM / 16; ++rbk) xblock_store(0, rbk, xblock_mfma(rbk));
        wbar<kWLgkm0>();                          // every wave's CODE reads before the refill
        code_dma(tile_of(1), 0, true);
        wbar<wvm(0) & kWLgkm0>();
#pragma unroll
        for (int rbk = 0; rbk < NXB; ++rbk) xblock_store(1, rbk, xblock_mfma(rbk));
    } else {
        dma_tab(tile_of(0), 0);
#pragma unroll
        for (int pp = 0; pp < C::NPX; ++pp) dma_own(tile_of(0), 0, pp);
        dma_tab(tile_of(1), 1);
#pragma unroll
        for (int pp = 0; pp < C::NPX; ++pp) dma_own(tile_of(1), 1, pp);
        wbar<wvm(0) & kWLgkm0>();                 // (all waves), zero row, EPI
        rexp(0);
        const unsigned char* es[C::NPE];
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(0, i, true);
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) ext_dma(i, es[i]);
    }

    // layer 0's per-feature chain for 4 features from a row code (the codes
    // form's CSR path, round-5 loop: the coefficient chunks in registers)
    [[maybe_unused]] auto expand4r = [&](const f32x4 (&cf)[8], const float (&v)[7]) -> f32x4 {
        f32x4 t = cf[7];
#pragma unroll
        for (int k = 0; k < 7; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) t[q] = fmaf(cf[k][q], v[k], t[q]);
        return f32x4{relu_nan(t[0]), relu_nan(t[1]), relu_nan(t[2]), relu_nan(t[3])};
    };
    // ---- phase A of a tile (its records in TAB slot tq, its rows in X): the
    // in-window / ext entries from LDS in CSR order, the +z entry held back
    // for phase B (ncn, nwn), or the CSR path for a wave with a row outside
    // the plan's form.  mid(G), G = 0..3, runs between the slot batches (after
    // batch G's loads, before its FMAs) -- the pipelined transform puts a
    // quarter of the previous tile's MFMAs there; every G runs exactly once
    // whatever the path.
    auto phase_a = [&](int tq, int64_t t0, int64_t nloc, const unsigned char* X, bool live,
                       f32x4 (&accn)[C::NQ][C::CH], uint32_t (&ncn)[C::NQ], float (&nwn)[C::NQ],
                       auto&& mid) {
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            ncn[qd] = C::OFF_ZERO >> C::CSH;
            nwn[qd] = 0.f;
#pragma unroll
            for (int j = 0; j < C::CH; ++j) accn[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // (the four mid() calls sit in straight-line code, once each: copies
        // of the MFMA groups in the branches cost ~100 spilled VGPRs)
        const unsigned char* const RW = lds + C::OFF_TAB + tq * C::TAB_BYTES + wave * C::RECW;
        const uint32_t summ = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
            *reinterpret_cast<const int*>(RW + C::OFF_RL + 4 * C::EPW)));
        const bool far = live && ((summ >> 8) & 1u) != 0u;
        const int maxa = (live && !far) ? static_cast<int>(summ & 0xffu) : 0;
        {
            {
                // the codes held for the whole phase; each batch's weights read
                // with its rows (registers: the pipelined transform's
                // fragments and accumulators are live through phase A)
                uint4 cds[C::NQ];
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
                    cds[qd] = *reinterpret_cast<const uint4*>(RW + (4 * qd + gq) * kWRec);
                auto codeof = [&](int qd, int u) -> uint32_t {
                    const uint32_t d = u < 2 ? cds[qd].x : u < 4 ? cds[qd].y : u < 6 ? cds[qd].z : cds[qd].w;
                    return (u & 1) ? (d >> 16) : (d & 0xffffu);
                };
                auto wld = [&](int qd, int u) -> float {
                    return *reinterpret_cast<const float*>(RW + C::OFF_RW + (4 * qd + gq) * 32 + 4 * u);
                };
                float wv[C::NQ][2];
                // slots in batches of 2: loads of a batch, mid(G), then its FMAs
                // (batches of 2: the VGPR budget of 2 waves per SIMD beside
                // the pipelined transform's fragments)
                f32x4 vv[C::NQ][2][C::CH];
                auto bload = [&](auto U0, auto NB) {
                    constexpr int u0 = decltype(U0)::value, nb = decltype(NB)::value;
#pragma unroll
                    for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                        for (int uu = 0; uu < nb; ++uu) {
                            const uint32_t ad = decode(codeof(qd, u0 + uu));
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
                                vv[qd][uu][j] = *reinterpret_cast<const f32x4*>(lds + ad + 256 * j);
                            wv[qd][uu] = wld(qd, u0 + uu);
                        }
                };
                auto bfma = [&](auto, auto NB) {
                    constexpr int nb = decltype(NB)::value;
#pragma unroll
                    for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                        for (int uu = 0; uu < nb; ++uu) {
                            const float w = wv[qd][uu];
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
#pragma unroll
                                for (int r = 0; r < 4; ++r) accn[qd][j][r] = fmaf(w, vv[qd][uu][j][r], accn[qd][j][r]);
                        }
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                using I2 = std::integral_constant<int, 2>;
                using I3 = std::integral_constant<int, 3>;
                using I4 = std::integral_constant<int, 4>;
                using I6 = std::integral_constant<int, 6>;
                if (maxa > 0) bload(I0{}, I2{});
                mid(I0{});
                if (maxa > 0) bfma(I0{}, I2{});
                if (maxa > 2) bload(I2{}, I2{});
                mid(I1{});
                if (maxa > 2) bfma(I2{}, I2{});
                if (maxa > 4) bload(I4{}, I2{});
                mid(I2{});
                if (maxa > 4) bfma(I4{}, I2{});
                if (maxa > 6) bload(I6{}, I1{});
                mid(I3{});
                if (maxa > 6) bfma(I6{}, I1{});
                if (live && !far) {
#pragma unroll
                    for (int qd = 0; qd < C::NQ; ++qd) {
                        ncn[qd] = codeof(qd, 7);
                        nwn[qd] = wld(qd, 7);
                    }
                }
            }
        }
        return far;
    };
    // the CSR path of phase A (a wave with a row outside the plan's form;
    // phase_a returned true): every entry of the wave's rows in CSR order,
    // the current tile from LDS, everything else from x (L2); the full sum
    // (no phase B).  Run by the caller where the fewest registers are live
    // (the pipelined step: after tile s - 2's stores).  The codes form keeps
    // its own CSR path in its loop.
    auto phase_a_far = [&](int64_t t0, int64_t nloc, const unsigned char* X, f32x4 (&accn)[C::NQ][C::CH]) {
        // CSR path: every entry of the wave's rows in CSR order, the
        // current tile from LDS, everything else from x (L2); the full
        // sum (no phase B)
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            const int lrow = C::RPW * wave + 4 * qd + gq;
            if (lrow < nloc) {
                const int64_t row = t0 + lrow;
                const int eb = row_ptr[row], ee = row_ptr[row + 1];
                for (int e = eb; e < ee; e += 4) {
                    int cj[4];
                    float wj[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const bool v = e + k < ee;
                        cj[k] = v ? col[e + k] : -1;
                        wj[k] = v ? ew[e + k] : 0.f;
                    }
                    f32x4 vv[4][C::CH];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int64_t off = static_cast<int64_t>(cj[k]) - t0;
                        if (cj[k] < 0) {
#pragma unroll
                            for (int j = 0; j < C::CH; ++j) vv[k][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                        } else if (off >= 0 && off < nloc) {
                            const uint32_t o = static_cast<uint32_t>(off);
                            const uint32_t a = (static_cast<uint32_t>(X - lds) + o * C::ROWB + ((o & 7u) << 4)) ^ coff0;
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
                                vv[k][j] = *reinterpret_cast<const f32x4*>(lds + a + 256 * j);
                        } else {
                            const float* rp = x + static_cast<int64_t>(cj[k]) * ldx + 4 * c0;
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
                                vv[k][j] = *reinterpret_cast<const f32x4*>(rp + 64 * j);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k)
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
#pragma unroll
                            for (int r = 0; r < 4; ++r) accn[qd][j][r] = fmaf(wj[k], vv[k][j][r], accn[qd][j][r]);
                }
            }
        }
    };
        auto no_mid = [](auto) {};

    if constexpr (X0) {
    // ---- the codes form keeps the round-5 step: the row expansion (12 f32
    // MFMAs and 6 row-block stores per wave) interleaved with the transform's
    // MFMAs after B2 -- in the pipelined step it lands on the post-B1 tail
    // (2.98 vs 2.78 ms per launch in the bench)
    // phase-B carry: tile s-1's partial sums and +z entries
    f32x4 accp[C::NQ][C::CH];
    uint32_t ncode[C::NQ];
    float nwt[C::NQ];
#pragma unroll
    for (int qd = 0; qd < C::NQ; ++qd) {
        ncode[qd] = C::OFF_ZERO >> C::CSH;
        nwt[qd] = 0.f;
#pragma unroll
        for (int j = 0; j < C::CH; ++j) accp[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // schedule: cur / nx1 = tiles of steps s / s + 1, the cursor at s + 2
    int64_t prv = -1, cur = tile_of(0), nx1 = tile_of(1);
    WinCursor c2{0, 0, 0};
    c2.next(S.L);
    c2.next(S.L);
    int xs = 0;                                   // X slot of step s (s % 3)
    for (int s = 0;; ++s) {
        if (cur < 0 && prv < 0) break;            // (uniform)
        const int64_t nx2 = win_tile_c(S, p, c2);
        const int rr = rr0, gg = gg0;
        const int iql = iq;
        // (the REXP row recomputed from an opaque lane: hoisted out of the
        // step loop it is a register too many at H = 64)
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int xp = xs == 0 ? 2 : xs - 1;      // slot of tile s - 1
        const int xn2 = xp;                       // slot of tile s + 2 (= (s-1) % 3)
        const int tq = static_cast<int>(s & 1);   // TAB slot of step s
        const int64_t t0 = rb + (cur >= 0 ? cur : 0) * C::BM;
        const int64_t nloc = cur >= 0 ? (re - t0 < C::BM ? re - t0 : C::BM) : 0;
        const int64_t tp0 = rb + (prv >= 0 ? prv : 0) * C::BM;
        const int64_t nlocp = prv >= 0 ? (re - tp0 < C::BM ? re - tp0 : C::BM) : 0;
        const unsigned char* const X = lds + C::OFF_X + xs * C::X_BYTES;
        const unsigned char* const XP = lds + C::OFF_X + xp * C::X_BYTES;
        // (B0) every row of the step was expanded by a ds_write of the last
        //      step; the records of step s + 1 landed (the ext list of the
        //      codes DMA'd below); younger only the last step's stores
        wtr.flush(wave, s - 1);
        wtr.stamp(0);
        if (s < 2) wbar<wvm(0) & kWLgkm0>();
        else wbar<wvm(C::NST) & kWLgkm0>();
        // this step's codes: own rows of tile s + 2, ext rows of step s + 1
        // (landing under phase A; expanded between the transform's MFMAs)
        code_dma(nx2, tq ^ 1, true);

        wtr.stamp(1);
        // ---- (P1) phase A of tile s
        f32x4 accn[C::NQ][C::CH];
        uint32_t ncn[C::NQ];
        float nwn[C::NQ];
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            ncn[qd] = C::OFF_ZERO >> C::CSH;
            nwn[qd] = 0.f;
#pragma unroll
            for (int j = 0; j < C::CH; ++j) accn[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (cur >= 0) {
            const unsigned char* const RW = lds + C::OFF_TAB + tq * C::TAB_BYTES + wave * C::RECW;
            const uint32_t summ = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
                *reinterpret_cast<const int*>(RW + C::OFF_RL + 4 * C::EPW)));
            const int maxa = static_cast<int>(summ & 0xffu);
            const bool far = ((summ >> 8) & 1u) != 0u;
            if (!far) {
                uint4 cds[C::NQ], w03[C::NQ], w47[C::NQ];
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    const unsigned char* wr = RW + C::OFF_RW + (4 * qd + gq) * 32;
                    cds[qd] = *reinterpret_cast<const uint4*>(RW + (4 * qd + gq) * kWRec);
                    w03[qd] = *reinterpret_cast<const uint4*>(wr);
                    w47[qd] = *reinterpret_cast<const uint4*>(wr + 16);
                }
                auto codeof = [&](int qd, int u) -> uint32_t {
                    const uint32_t d = u < 2 ? cds[qd].x : u < 4 ? cds[qd].y : u < 6 ? cds[qd].z : cds[qd].w;
                    return (u & 1) ? (d >> 16) : (d & 0xffffu);
                };
                auto wof = [&](int qd, int u) -> float {
                    const uint32_t d = u == 0 ? w03[qd].x : u == 1 ? w03[qd].y : u == 2 ? w03[qd].z
                                     : u == 3 ? w03[qd].w : u == 4 ? w47[qd].x : u == 5 ? w47[qd].y
                                     : u == 6 ? w47[qd].z : w47[qd].w;
                    return __uint_as_float(d);
                };
                // slots in batches of 2: loads of a batch first
                auto batch = [&](auto U0, auto NB) {
                    constexpr int u0 = decltype(U0)::value, nb = decltype(NB)::value;
                    f32x4 vv[C::NQ][nb][C::CH];
#pragma unroll
                    for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                        for (int uu = 0; uu < nb; ++uu) {
                            const uint32_t a = decode(codeof(qd, u0 + uu));
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
                                vv[qd][uu][j] = *reinterpret_cast<const f32x4*>(lds + a + 256 * j);
                        }
#pragma unroll
                    for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                        for (int uu = 0; uu < nb; ++uu) {
                            const float w = wof(qd, u0 + uu);
#pragma unroll
                            for (int j = 0; j < C::CH; ++j)
#pragma unroll
                                for (int r = 0; r < 4; ++r) accn[qd][j][r] = fmaf(w, vv[qd][uu][j][r], accn[qd][j][r]);
                        }
                };
                // (batches of 2: the 128-VGPR budget of 4 waves per SIMD)
                if (maxa > 0) batch(std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{});
                if (maxa > 2) batch(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{});
                if (maxa > 4) batch(std::integral_constant<int, 4>{}, std::integral_constant<int, 2>{});
                if (maxa > 6) batch(std::integral_constant<int, 6>{}, std::integral_constant<int, 1>{});
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    ncn[qd] = codeof(qd, 7);
                    nwn[qd] = wof(qd, 7);
                }
            } else {
                // CSR path: every entry of the wave's rows in CSR order, the
                // current tile from LDS, everything else from x (L2); the full
                // sum (no phase B)
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    const int lrow = C::RPW * wave + 4 * qd + gq;
                    if (lrow < nloc) {
                        const int64_t row = t0 + lrow;
                        const int eb = row_ptr[row], ee = row_ptr[row + 1];
                        for (int e = eb; e < ee; e += 4) {
                            int cj[4];
                            float wj[4];
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                const bool v = e + k < ee;
                                cj[k] = v ? col[e + k] : -1;
                                wj[k] = v ? ew[e + k] : 0.f;
                            }
                            {
                                // codes form: one entry at a time (registers), rows
                                // outside the tile expanded from their codes
#pragma unroll 1
                                for (int k = 0; k < 4; ++k) {
                                    if (cj[k] < 0) continue;
                                    f32x4 vk[C::CH];
                                    const int64_t off = static_cast<int64_t>(cj[k]) - t0;
                                    if (off >= 0 && off < nloc) {
                                        const uint32_t o = static_cast<uint32_t>(off);
                                        const uint32_t a = (static_cast<uint32_t>(X - lds) + o * C::ROWB + ((o & 7u) << 4)) ^ coff0;
#pragma unroll
                                        for (int j = 0; j < C::CH; ++j)
                                            vk[j] = *reinterpret_cast<const f32x4*>(lds + a + 256 * j);
                                    } else {
                                        const float* cp = x + static_cast<int64_t>(cj[k]) * ldx;
                                        const float4 v0 = ld4(cp), v1 = ld4(cp + 4);
                                        const float v[7] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z};
#pragma unroll 1
                                        for (int j = 0; j < C::CH; ++j) {
                                            f32x4 cf[8];
#pragma unroll
                                            for (int q = 0; q < 8; ++q)
                                                cf[q] = *reinterpret_cast<const f32x4*>(
                                                    lds + C::OFF_COEF + ((c0 + 16 * j) * 8 + q) * 16);
                                            vk[j] = expand4r(cf, v);
                                        }
                                    }
#pragma unroll
                                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                                        for (int r = 0; r < 4; ++r) accn[qd][j][r] = fmaf(wj[k], vk[j][r], accn[qd][j][r]);
                                }
                            }
                        }
                    }
                }
            }
        }

        wtr.stamp(2);
        // ---- (P1) phase B of tile s - 1, its split and residual seeds
        f32x4 seed[IBW][CPW];
        if (prv >= 0) {
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd) {
                const uint32_t a = decode(ncode[qd]);
#pragma unroll
                for (int j = 0; j < C::CH; ++j) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(lds + a + 256 * j);
#pragma unroll
                    for (int r = 0; r < 4; ++r) accp[qd][j][r] = fmaf(nwt[qd], v[r], accp[qd][j][r]);
                }
            }
            {
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    uint32_t m = 0;
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) m = max(m, __float_as_uint(fabsf(accp[qd][j][r])));
                    m = wrow_max(m);
                    const int pe = wsplit_exp(m);
                    const float sc = __uint_as_float(static_cast<uint32_t>(pe + 127) << 23);
                    const int lrow = C::RPW * wave + 4 * qd + gq;
                    const int sw = asw<H>(lrow);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        f16x4w hv, lv;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float sv = accp[qd][j][r] * sc;
                            const _Float16 hh = static_cast<_Float16>(sv);
                            hv[r] = hh;
                            lv[r] = static_cast<_Float16>(sv - static_cast<float>(hh));
                        }
                        const int cc = c0 + 16 * j;             // the lane's 16-B fp32 chunk
                        const int ao = lrow * H + 8 * ((cc >> 1) ^ sw) + 4 * (cc & 1);
                        *reinterpret_cast<f16x4w*>(&AH[ao]) = hv;
                        *reinterpret_cast<f16x4w*>(&AL[ao]) = lv;
                    }
                    if (iql == 0) {
                        // (the row index recomputed from an opaque lane: hoisted
                        // out of the step loop it is a register too many at H = 64)
                        REXP[C::RPW * wave + 4 * qd + (ln >> 4)] = pe;
                    }
                }
                // residual + bias of my output blocks (tile s-1's rows of my
                // row group, my columns), before slot (s-1) % 3 is refilled
#pragma unroll
                for (int cp = 0; cp < CPW; ++cp) {
                    const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[n0 + 16 * cp + 4 * gg]);
#pragma unroll
                    for (int ib = 0; ib < IBW; ++ib) {
                        const int lr = (wm * IBW + ib) * 16 + rr;
                        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (has_res) {
                            const int ch = ((n0 + 16 * cp) >> 2) + gg;
                            rv = *reinterpret_cast<const float4*>(XP + lr * C::ROWB + ((ch ^ (lr & 7)) << 4));
                        }
                        seed[ib][cp] = f32x4{rv.x + bo[0], rv.y + bo[1], rv.z + bo[2], rv.w + bo[3]};
                    }
                }
            }
        }
        // (B2) A image complete; every read of slot (s-1) % 3, the ext area
        // and this step's records done
        wtr.stamp(3);
        wbar<wvm(0) & kWLgkm0>();                 // (+ every wave's codes)
        wtr.stamp(4);
        // the DMA of this step: the records of step s + 2 (into this step's
        // TAB slot; the rows' codes went at B0)
        const int64_t tn2 = nx2;
        auto dma_piece = [&](int) { dma_tab(tn2, tq); };
        constexpr int NPC = 1;

        if (prv >= 0) {
            {
                // (3) transform: my output column blocks x my row blocks
                int pr[IBW];
                f32x4 accm[IBW][CPW];
#pragma unroll
                for (int ib = 0; ib < IBW; ++ib) {
                    pr[ib] = REXP[(wm * IBW + ib) * 16 + rr];
#pragma unroll
                    for (int cp = 0; cp < CPW; ++cp)
#pragma unroll
                        for (int r = 0; r < 4; ++r) accm[ib][cp][r] = ldexpf(seed[ib][cp][r], pr[ib] + qw[cp]);
                }
                {
                    const int sw = asw<H>(rr);
                    auto frag = [&](int t, f16x8w& bh, f16x8w& bl) {
                        const int kc = t / IBW, ib = t % IBW;
                        const int R = (wm * IBW + ib) * 16 + rr;
                        const int ao = R * H + 8 * ((4 * kc + gg) ^ sw);
                        bh = *reinterpret_cast<const f16x8w*>(&AH[ao]);
                        bl = *reinterpret_cast<const f16x8w*>(&AL[ao]);
                    };
                    __builtin_amdgcn_sched_barrier(0);
                    constexpr int PD = 5, NF = PD + 1, NTT = C::KC * IBW;
                    f16x8w fh[NF], fl[NF];
#pragma unroll
                    for (int t = 0; t < PD && t < NTT; ++t) frag(t, fh[t], fl[t]);
                    // codes form: the expansion rows between the MFMAs, one
                    // every XS t-steps from t = XT (the codes DMA'd at B0)
                    constexpr int XT = 2, XS = 2;
                    f32x4 xd[2];
#pragma unroll
                    for (int t = 0; t < NTT; ++t) {
                        const int kc = t / IBW, ib = t % IBW;
                        if (t < NPC) dma_piece(t);
                        {
                            // block i's MFMAs, block i - 1's store (its result landed)
                            static_assert(XT + XS * (NXB - 1) < NTT, "expansion inside the transform");
                            const int i = (t - XT) / XS;
                            if (t >= XT && (t - XT) % XS == 0 && i < NXB) {
                                xd[i & 1] = xblock_mfma(i);
                                if (i > 0) xblock_store(xn2, i - 1, xd[(i - 1) & 1]);
                            }
                        }
                        if (MODE & 4) continue;
                        if (t + PD < NTT) frag(t + PD, fh[(t + PD) % NF], fl[(t + PD) % NF]);
#pragma unroll
                        for (int cp = 0; cp < CPW; ++cp) {
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cp][kc], fh[t % NF], accm[ib][cp], 0, 0, 0);
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cp][kc], fl[t % NF], accm[ib][cp], 0, 0, 0);
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[cp][kc], fh[t % NF], accm[ib][cp], 0, 0, 0);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int t = NTT; t < NPC; ++t) dma_piece(t);
                    xblock_store(xn2, NXB - 1, xd[(NXB - 1) & 1]);
                }
                wtr.stamp(5);
                {
                    // epilogue stored straight from the accumulators: lane (rr, gg) of
                    // block (ib, cp) holds row 16 ib + rr, columns n0 + 16 cp + 4 gg .. +3
                    static_assert(IBW * CPW == C::NST, "one store per block keeps the per-step store count");
#pragma unroll
                    for (int cp = 0; cp < CPW; ++cp) {
                        const int nc = n0 + 16 * cp + 4 * gg;
                        const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + nc]);
                        const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + nc]);
#pragma unroll
                        for (int ib = 0; ib < IBW; ++ib) {
                            f32x4 o;
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                float v = ldexpf(accm[ib][cp][r], -(pr[ib] + qw[cp]));
                                if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                                if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                                o[r] = v;
                            }
                            const int lr = (wm * IBW + ib) * 16 + rr;
                            if (lr < nlocp)
                                wstore(o, reinterpret_cast<f32x4*>(out + (tp0 + lr) * ldo + nc));
                        }
                    }
                }
                wtr.stamp(7);
            }
        } else {
#pragma unroll
            for (int q = 0; q < NPC; ++q) dma_piece(q);
            if constexpr (X0) {
#pragma unroll
                for (int rbk = 0; rbk < NXB; ++rbk) xblock_store(xn2, rbk, xblock_mfma(rbk));
            }
        }
        rexp(tq ^ 1);                             // tile s + 1's weights (records landed at B0)
        // carry tile s into phase B
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            ncode[qd] = ncn[qd];
            nwt[qd] = nwn[qd];
#pragma unroll
            for (int j = 0; j < C::CH; ++j) accp[qd][j] = accn[qd][j];
        }
        xs = xs == 2 ? 0 : xs + 1;
        prv = cur;
        cur = nx1;
        nx1 = nx2;
        c2.next(S.L);
    }
        wwait<wvm(0)>();   // no LDS-DMA may outlive the workgroup
    } else if constexpr (!AGG) {
        // ---- the pipelined step (every full-layer mode but the codes form).  Step s runs phase
        // A of tile s with the transform of tile s - 2 (its 48 MFMAs in four
        // groups between phase A's slot batches: the matrix pipe works under
        // the aggregation's LDS reads and FMAs instead of in a phase of its
        // own), then phase B and the split of tile s - 1 into the A image:
        //   B0  ext rows of step s landed (older: this step's records, the own
        //       rows of tile s, the stores of tile s - 3); younger: the records
        //       of step s + 1, the own rows of tile s + 1
        //   phase A(s) || MFMAs(s - 2) (A image and REXP of tile s - 2);
        //   epilogue and stores of tile s - 2; residual seeds of tile s - 1
        //   B1  every read of slot (s-1) % 3, the ext area, this step's
        //       records and the A image done
        //       -> DMA ext rows of step s + 1, records of step s + 2, own rows
        //       of tile s + 2 into slot (s-1) % 3
        //   phase B(s - 1) (its +z term from tile s), split -> A image, REXP
        f32x4 accp[C::NQ][C::CH];
        uint32_t ncode[C::NQ];
        float nwt[C::NQ];
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            ncode[qd] = C::OFF_ZERO >> C::CSH;
            nwt[qd] = 0.f;
#pragma unroll
            for (int j = 0; j < C::CH; ++j) accp[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        // residual + bias of tile s - 1's rows in the transform's layout (lane
        // (rr, gg) of block (ib, cp): row 16 (wm IBW + ib) + rr, columns n0 +
        // 16 cp + 4 gg ..), read at step s, used by step s + 1's MFMAs
        f32x4 seedc[IBW][CPW];
#pragma unroll
        for (int ib = 0; ib < IBW; ++ib)
#pragma unroll
            for (int cp = 0; cp < CPW; ++cp) seedc[ib][cp] = f32x4{0.f, 0.f, 0.f, 0.f};
        int64_t prv2 = -1, prv = -1, cur = tile_of(0), nx1 = tile_of(1);
        WinCursor c2{0, 0, 0};
        c2.next(S.L);
        c2.next(S.L);
        int xs = 0;                               // X slot of step s (s % 3)
        const int rr = rr0, gg = gg0;
        constexpr int PD = kWinPD, NF = PD + 1, NTT = C::KC * IBW, TG = NTT / 4;
        static_assert(NTT % 4 == 0 && PD < NTT, "four MFMA groups");
        for (int s = 0;; ++s) {
            if (cur < 0 && prv < 0 && prv2 < 0) break;   // (uniform)
            const int64_t nx2 = win_tile_c(S, p, c2);
            // (the REXP row recomputed from an opaque lane)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int xp = xs == 0 ? 2 : xs - 1;  // slot of tile s - 1 (and of tile s + 2)
            const int tq = static_cast<int>(s & 1);
            const int64_t t0 = rb + (cur >= 0 ? cur : 0) * C::BM;
            const int64_t nloc = cur >= 0 ? (re - t0 < C::BM ? re - t0 : C::BM) : 0;
            const int64_t t20 = rb + (prv2 >= 0 ? prv2 : 0) * C::BM;
            const int64_t nloc2 = prv2 >= 0 ? (re - t20 < C::BM ? re - t20 : C::BM) : 0;
            const unsigned char* const X = lds + C::OFF_X + xs * C::X_BYTES;
            const unsigned char* const XP = lds + C::OFF_X + xp * C::X_BYTES;
            wtr.flush(wave, s - 1);
            wtr.stamp(0);
            // (B0)
            if (s == 0) wbar<wvm(0) & kWLgkm0>();
            else wbar<wvm(1 + C::NPX) & kWLgkm0>();
            wtr.stamp(1);

            // ---- the transform of tile s - 2, as four MFMA groups
            const bool mf = prv2 >= 0;             // (uniform)
            int pr2[IBW];
            f32x4 accm[IBW][CPW];
            f16x8w fh[NF], fl[NF];
            const int sw = asw<H>(rr);
            auto frag = [&](int t, f16x8w& bh, f16x8w& bl) {
                const int kc = t / IBW, ib = t % IBW;
                const int R = (wm * IBW + ib) * 16 + rr;
                const int ao = R * H + 8 * ((4 * kc + gg) ^ sw);
                bh = *reinterpret_cast<const f16x8w*>(&AH[ao]);
                bl = *reinterpret_cast<const f16x8w*>(&AL[ao]);
            };
            if (mf) {
#pragma unroll
                for (int ib = 0; ib < IBW; ++ib) {
                    pr2[ib] = REXP[(wm * IBW + ib) * 16 + rr];
#pragma unroll
                    for (int cp = 0; cp < CPW; ++cp)
#pragma unroll
                        for (int r = 0; r < 4; ++r) accm[ib][cp][r] = ldexpf(seedc[ib][cp][r], pr2[ib] + qw[cp]);
                }
#pragma unroll
                for (int t = 0; t < PD; ++t) frag(t, fh[t], fl[t]);
            }
            auto mid = [&](auto G) {
                constexpr int g = decltype(G)::value;
                if (!mf) return;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = g * TG; t < (g + 1) * TG; ++t) {
                    const int kc = t / IBW, ib = t % IBW;
                    if constexpr ((MODE & 4) == 0) {
                        if (t + PD < NTT) frag(t + PD, fh[(t + PD) % NF], fl[(t + PD) % NF]);
#pragma unroll
                        for (int cp = 0; cp < CPW; ++cp) {
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cp][kc], fh[t % NF], accm[ib][cp], 0, 0, 0);
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cp][kc], fl[t % NF], accm[ib][cp], 0, 0, 0);
                            accm[ib][cp] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[cp][kc], fh[t % NF], accm[ib][cp], 0, 0, 0);
                        }
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            };

            // ---- phase A of tile s (the MFMA groups between its batches)
            f32x4 accn[C::NQ][C::CH];
            uint32_t ncn[C::NQ];
            float nwn[C::NQ];
            const bool far = phase_a(tq, t0, nloc, X, cur >= 0, accn, ncn, nwn, mid);
            wtr.stamp(2);
            // epilogue of tile s - 2 in registers (gnn_model.py:184-191: conv
            // + bias, + x, BN, ReLU); lane (rr, gg) of block (ib, cp) holds row
            // 16 (wm IBW + ib) + rr, columns n0 + 16 cp + 4 gg .. + 3
            if (mf) {
#pragma unroll
                for (int cp = 0; cp < CPW; ++cp) {
                    const int nc = n0 + 16 * cp + 4 * gg;
                    const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + nc]);
                    const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + nc]);
#pragma unroll
                    for (int ib = 0; ib < IBW; ++ib)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float v = ldexpf(accm[ib][cp][r], -(pr2[ib] + qw[cp]));
                            if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                            if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                            accm[ib][cp][r] = v;
                        }
                }
                // the stores of tile s - 2 (before B1 and this step's DMAs; a
                // partial tile is the last of its workgroup -- fewer stores
                // there change no wait that matters: the later steps' records
                // and rows are dummies)
                static_assert(IBW * CPW == C::NST, "one store per block keeps the per-step store count");
                // (the lane's store offsets from an opaque lane: hoisted, its
                // 64-bit row pointer is spilled and reloaded under a vmcnt(0))
                int ls = lane;
                asm volatile("" : "+v"(ls));
#pragma unroll
                for (int cp = 0; cp < CPW; ++cp) {
                    const int nc = n0 + 16 * cp + 4 * (ls >> 4);
#pragma unroll
                    for (int ib = 0; ib < IBW; ++ib) {
                        const int lr = (wm * IBW + ib) * 16 + (ls & 15);
                        if (lr < nloc2)
                            wstore(accm[ib][cp], reinterpret_cast<f32x4*>(out + (t20 + lr) * ldo + nc));
                    }
                }
            }
            if (far) phase_a_far(t0, nloc, X, accn);
            // residual + bias of tile s - 1, before slot (s-1) % 3 is refilled
            f32x4 seedn[IBW][CPW];
            if (prv >= 0) {
#pragma unroll
                for (int cp = 0; cp < CPW; ++cp) {
                    const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[n0 + 16 * cp + 4 * gg]);
#pragma unroll
                    for (int ib = 0; ib < IBW; ++ib) {
                        const int lr = (wm * IBW + ib) * 16 + rr;
                        float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (has_res) {
                            const int ch = ((n0 + 16 * cp) >> 2) + gg;
                            rv = *reinterpret_cast<const float4*>(XP + lr * C::ROWB + ((ch ^ (lr & 7)) << 4));
                        }
                        seedn[ib][cp] = f32x4{rv.x + bo[0], rv.y + bo[1], rv.z + bo[2], rv.w + bo[3]};
                    }
                }
            }
            // (B1)
            wtr.stamp(3);
            wbar<kWLgkm0>();
            const int64_t tn1 = nx1, tn2 = nx2;
            // DMA pieces of this step: ext rows of step s + 1, the records of
            // step s + 2, the own rows of tile s + 2, issued between phase B's
            // and the split's VALU work
            // (as a burst after B1 they stall the vector memory pipe: 3.26
            // vs 2.86 ms)
            // this wave's records of step s + 1 landed (its ext list);
            // younger: the own rows of tile s + 1, the stores of tile s - 2
            if (s == 0) wwait<wvm(0)>();
            else if (s == 1) wwait<wvm(C::NPX)>();
            else wwait<wvm(C::NPX + C::NST)>();
            rexp(tq ^ 1);                         // tile s + 1's weights (same-box A/B:
                                                  // here, at B0 on tile s, or at the step's
                                                  // end within 0.3 %)
            const unsigned char* es[C::NPE];
#pragma unroll
            for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(tq ^ 1, i, tn1 >= 0);
            constexpr int NPC = C::NPE + 1 + C::NPX;
            auto dpiece = [&](int q) {
                if (q < C::NPE) ext_dma(q, es[q]);
                else if (q == C::NPE) dma_tab(tn2, tq);
                else dma_own(tn2, xp, q - C::NPE - 1);
            };
            // pieces [q0, q1)
            auto dpieces = [&](int q0, int q1) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = q0; q < q1 && q < NPC; ++q) dpiece(q);
                __builtin_amdgcn_sched_barrier(0);
            };
            if (prv < 0) dpieces(0, NPC);
            wtr.stamp(4);
            // ---- phase B of tile s - 1 (its +z term, from tile s), split
            if (prv >= 0) {
                f32x4 pv[C::NQ][C::CH];
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    const uint32_t ad = decode(ncode[qd]);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) pv[qd][j] = *reinterpret_cast<const f32x4*>(lds + ad + 256 * j);
                }
                dpieces(0, 3);
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) accp[qd][j][r] = fmaf(nwt[qd], pv[qd][j][r], accp[qd][j][r]);
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    if (qd == 1) dpieces(3, 5);
                    uint32_t m = 0;
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) m = max(m, __float_as_uint(fabsf(accp[qd][j][r])));
                    m = wrow_max(m);
                    const int pe = wsplit_exp(m);
                    const float sc = __uint_as_float(static_cast<uint32_t>(pe + 127) << 23);
                    const int lrow = C::RPW * wave + 4 * qd + gq;
                    const int swr = asw<H>(lrow);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        f16x4w hv, lv;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float sv = accp[qd][j][r] * sc;
                            const _Float16 hh = static_cast<_Float16>(sv);
                            hv[r] = hh;
                            lv[r] = static_cast<_Float16>(sv - static_cast<float>(hh));
                        }
                        const int cc = c0 + 16 * j;             // the lane's 16-B fp32 chunk
                        const int ao = lrow * H + 8 * ((cc >> 1) ^ swr) + 4 * (cc & 1);
                        *reinterpret_cast<f16x4w*>(&AH[ao]) = hv;
                        *reinterpret_cast<f16x4w*>(&AL[ao]) = lv;
                    }
                    if (iq == 0) REXP[C::RPW * wave + 4 * qd + (ln >> 4)] = pe;
                }
                dpieces(5, NPC);
            }
            wtr.stamp(5);
            // carry
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd) {
                ncode[qd] = ncn[qd];
                nwt[qd] = nwn[qd];
#pragma unroll
                for (int j = 0; j < C::CH; ++j) accp[qd][j] = accn[qd][j];
            }
#pragma unroll
            for (int ib = 0; ib < IBW; ++ib)
#pragma unroll
                for (int cp = 0; cp < CPW; ++cp) seedc[ib][cp] = seedn[ib][cp];
            xs = xs == 2 ? 0 : xs + 1;
            prv2 = prv;
            prv = cur;
            cur = nx1;
            nx1 = nx2;
            c2.next(S.L);
        }
        wwait<wvm(0)>();   // no LDS-DMA may outlive the workgroup
    } else {
        // ---- the aggregate alone (mignn_gcn_aggregate_win: the fp32 sums are
        // the output).  Step s: B0 (ext rows of step s landed; younger: the
        // records of step s + 1, the own rows of tile s + 2, the last step's
        // stores), phase A of tile s, phase B of tile s - 1, B2 (every read of
        // slot (s-1) % 3, the ext area and this step's records done), the DMA
        // of step s + 1's ext rows, step s + 2's records and tile s + 2's own
        // rows, tile s - 1's stores
        f32x4 accp[C::NQ][C::CH];
        uint32_t ncode[C::NQ];
        float nwt[C::NQ];
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd) {
            ncode[qd] = C::OFF_ZERO >> C::CSH;
            nwt[qd] = 0.f;
#pragma unroll
            for (int j = 0; j < C::CH; ++j) accp[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        int64_t prv = -1, cur = tile_of(0), nx1 = tile_of(1);
        WinCursor c2{0, 0, 0};
        c2.next(S.L);
        c2.next(S.L);
        int xs = 0;                               // X slot of step s (s % 3)
        for (int s = 0;; ++s) {
            if (cur < 0 && prv < 0) break;        // (uniform)
            const int64_t nx2 = win_tile_c(S, p, c2);
            const int xp = xs == 0 ? 2 : xs - 1;  // slot of tile s - 1 (and of tile s + 2)
            const int tq = static_cast<int>(s & 1);
            const int64_t t0 = rb + (cur >= 0 ? cur : 0) * C::BM;
            const int64_t nloc = cur >= 0 ? (re - t0 < C::BM ? re - t0 : C::BM) : 0;
            const int64_t tp0 = rb + (prv >= 0 ? prv : 0) * C::BM;
            const int64_t nlocp = prv >= 0 ? (re - tp0 < C::BM ? re - tp0 : C::BM) : 0;
            const unsigned char* const X = lds + C::OFF_X + xs * C::X_BYTES;
            wtr.flush(wave, s - 1);
            wtr.stamp(0);
            if (s == 0) wbar<wvm(0) & kWLgkm0>();
            else if (s == 1) wbar<wvm(1 + C::NPX) & kWLgkm0>();
            else wbar<wvm(1 + C::NPX + C::NST) & kWLgkm0>();
            wtr.stamp(1);
            f32x4 accn[C::NQ][C::CH];
            uint32_t ncn[C::NQ];
            float nwn[C::NQ];
            if (phase_a(tq, t0, nloc, X, cur >= 0, accn, ncn, nwn, no_mid)) phase_a_far(t0, nloc, X, accn);
            wtr.stamp(2);
            if (prv >= 0) {
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd) {
                    const uint32_t ad = decode(ncode[qd]);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        const f32x4 v = *reinterpret_cast<const f32x4*>(lds + ad + 256 * j);
#pragma unroll
                        for (int r = 0; r < 4; ++r) accp[qd][j][r] = fmaf(nwt[qd], v[r], accp[qd][j][r]);
                    }
                }
            }
            wtr.stamp(3);
            wbar<kWLgkm0>();                      // (B2)
            wtr.stamp(4);
            // the records of step s + 1 landed (younger: the own rows of tile
            // s + 1 and the last step's stores)
            if (s == 0) wwait<wvm(0)>();
            else if (s == 1) wwait<wvm(C::NPX)>();
            else wwait<wvm(C::NPX + C::NST)>();
            const int64_t tn1 = nx1, tn2 = nx2;
            const unsigned char* es[C::NPE];
#pragma unroll
            for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(tq ^ 1, i, tn1 >= 0);
#pragma unroll
            for (int i = 0; i < C::NPE; ++i) ext_dma(i, es[i]);
            dma_tab(tn2, tq);
#pragma unroll
            for (int pp = 0; pp < C::NPX; ++pp) dma_own(tn2, xp, pp);
            if (prv >= 0) {
                static_assert(C::NQ * C::CH == C::NST, "aggregate stores keep the per-step store count");
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        // (a partial tile is the last of its workgroup: fewer stores
                        // there change no later wait)
                        const int lrow = C::RPW * wave + 4 * qd + gq;
                        if (lrow < nlocp)
                            __builtin_nontemporal_store(accp[qd][j], reinterpret_cast<f32x4*>(out + (tp0 + lrow) * ldo + 4 * (c0 + 16 * j)));
                    }
            }
            rexp(tq ^ 1);                         // tile s + 1's weights (records waited after B2)
            // carry tile s into phase B
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd) {
                ncode[qd] = ncn[qd];
                nwt[qd] = nwn[qd];
#pragma unroll
                for (int j = 0; j < C::CH; ++j) accp[qd][j] = accn[qd][j];
            }
            xs = xs == 2 ? 0 : xs + 1;
            prv = cur;
            cur = nx1;
            nx1 = nx2;
            c2.next(S.L);
        }
        wwait<wvm(0)>();   // no LDS-DMA may outlive the workgroup
    }
}

// max over the 4 lanes of a row of the B layout (l, l ^ 16, l ^ 32, l ^ 48)
__device__ __forceinline__ uint32_t wrow4_max(uint32_t m) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m = max(static_cast<uint32_t>(r16[0]), static_cast<uint32_t>(r16[1]));
    const auto r32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return max(static_cast<uint32_t>(r32[0]), static_cast<uint32_t>(r32[1]));
}

// ------------------------------------------------------------ layer, H = 64
// Step s of a wave (rows 16 w .. 16 w + 15 of the tiles; lane (r, g) holds
// fp32 chunks 8 kc + 2 g + {0, 1} of row r, kc = 0, 1):
//   B0  ext rows of step s landed (older: own rows of tile s, the records)
//   phase A of tile s (in-window / ext entries from LDS, the +z entry held
//   back); the residual of tile s - 1 (slot (s-1) % 3) into registers
//   B1  slot (s-1) % 3, the ext area and this step's records free
//       -> DMA ext rows of step s + 1, records of step s + 2, own rows of
//       tile s + 2
//   phase B of tile s - 1 (its +z term, from tile s), split (row exponent
//   over the row's 4 lanes), 24 MFMAs 16x16x32 f16 (W split in registers),
//   epilogue, the wave's 16 rows staged in its own LDS region, whole-row
//   stores.
// MODE: 32 aggregate only; diag 1 ext / 2 own rows from the zero row, 4 no MFMAs.
template <int MODE = 0, int EPIF = -1>
__global__ __launch_bounds__(WCfg<64>::NT, 2) void gcn_win64_kernel(
    const unsigned char* __restrict__ plan, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ col, const float* __restrict__ ew, const float* __restrict__ x,
    int64_t ldx, int64_t rb, int64_t re, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    using C = WCfg<64>;
    constexpr int H = 64;
    constexpr bool AGG = (MODE & 32) != 0;
    if constexpr (EPIF >= 0) flags = EPIF;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the two waves of a SIMD (w, w + NW / 2) at different priorities: both
    // meet at the same barriers and would reach their MFMA groups and their
    // LDS / VALU phases together; the first now runs ahead and the second
    // fills its gaps (same-box A/B, DESIGN 3.17: H = 128 -0.75 %, H = 64
    // -2.3 %, codes form -0.75 %)
    if (wave < C::NW / 2) __builtin_amdgcn_s_setprio(1);

    const WinHdr* const hdr = reinterpret_cast<const WinHdr*>(plan);
    {
        const bool ok = hdr->magic == kWMagic && hdr->G == static_cast<int>(gridDim.x) &&
                        hdr->h == H && hdr->rb == rb && hdr->re == re;
        if (!ok) {
            if (tid == 0)
                __hip_atomic_fetch_or(&g_win_errors, static_cast<unsigned>(MIGNN_DEVERR_PLAN),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            plan_mismatch_fill(out, ldo, rb, re, H);
            return;
        }
    }
    const WinSched S = win_sched(hdr);
    const unsigned char* const tabs = plan + kWHdr;
    const int per_xcd = static_cast<int>(gridDim.x) >> 3;
    const int p = (static_cast<int>(blockIdx.x) & 7) * per_xcd + (static_cast<int>(blockIdx.x) >> 3);
    auto tile_of = [&](int64_t s) -> int64_t { return win_tile(S, p, s); };
    if (tile_of(0) < 0) return;                   // no work (uniform): no DMA issued
#ifdef MIGNN_DIAG
    WTrace wtr{(blockIdx.x < 8 && wave == 0) ? g_win_trace : nullptr, 0u, 0u, lane};
#else
    WTrace wtr{nullptr, 0u, 0u, lane};
#endif

    const int r = lane & 15, g = lane >> 4;
    // the wave row of lane (r, g): lanes r in {0-3, 12-15} take the even rows,
    // r in {4-11} the odd ones.  A ds_read_b128 lane group holds the first
    // set at chunk 2 g and the second at 2 g + 2 (or the reverse), so with
    // the (row & 15) swizzle the in-plane neighbours (row offsets 0, +-1,
    // +-8) land on 16 distinct 16-B bank slots -- with rows in lane order
    // the +-1 neighbours are 2-way conflicts (SQ_LDS_BANK_CONFLICT 26 % of
    // the LDS cycles).  The MFMA is indifferent: B-operand column r is row rw.
    const int rw = (2 * r + ((r >= 4 && r < 12) ? 9 : 0)) & 15;
    const int lrow = C::RPW * wave + rw;          // the lane's row in a tile (lrow & 15 == rw)
    // the lane's 16-B chunks of a row: k = 2 kc + hf -> chunk 8 kc + 2 g + hf
    uint32_t coff[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) coff[k] = static_cast<uint32_t>((8 * (k >> 1) + 2 * g + (k & 1)) << 4);

    // own-row DMA: SGPR base, per-lane offsets fixed for the launch
    const uint32_t ldxb = static_cast<uint32_t>(ldx) * 4u;
    uint32_t xoff[C::NPX];
#pragma unroll
    for (int pp = 0; pp < C::NPX; ++pp) {
        const int pc = pp * C::NW + wave;
        const int lr = pc * C::RPP + lane / C::LPR;
        const int pos = lane % C::LPR;
        xoff[pp] = static_cast<uint32_t>(lr) * ldxb + 16u * static_cast<uint32_t>(pos ^ (lr & C::SWZ));
    }
    const uint32_t toff = static_cast<uint32_t>(wave * C::RECG + 16 * lane);
    auto dma_tab = [&](int64_t t, int q) {
        if (lane < C::TLANES)
            wdma_s(tabs + (t >= 0 ? t : 0) * C::TAB_G, toff,
                   wlds(lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW));
    };
    float* const DV = reinterpret_cast<float*>(lds + C::OFF_DV);
    auto rexp = [&](int q) { win_rexp<C>(lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW, DV, lane); };
    auto dma_own = [&](int64_t t, int q, int pp) {
        const int64_t tt = t >= 0 ? t : 0;
        const int64_t t0 = rb + tt * C::BM;
        const int pc = pp * C::NW + wave;
        unsigned char* const X = lds + C::OFF_X + q * C::X_BYTES;
        if constexpr ((MODE & 2) != 0) {
            wdma(g_win_zero_row + 4 * (lane & 15), wlds(X + pc * 1024));
        } else if (t0 + C::BM <= re) {
            wdma_s(x + t0 * ldx, xoff[pp], wlds(X + pc * 1024));
        } else {
            int l = lane;
            asm volatile("" : "+v"(l));
            const int lr = pc * C::RPP + l / C::LPR;
            const int pos = l % C::LPR;
            int64_t row = t0 + lr;
            if (row >= re) row = re - 1;
            wdma(x + row * ldx + 4 * (pos ^ (lr & C::SWZ)), wlds(X + pc * 1024));
        }
    };
    auto ext_src = [&](int q, int i, bool real) -> const unsigned char* {
        const unsigned char* const tab = lds + C::OFF_TAB + q * C::TAB_BYTES + wave * C::RECW + C::OFF_RL;
        int l = lane;
        asm volatile("" : "+v"(l));
        const int kk = i * C::RPP + l / C::LPR;
        const int k = wave * C::EPW + kk;
        const int pos = l % C::LPR;
        const uint32_t c = *reinterpret_cast<const uint32_t*>(tab + 4 * kk);
        return ((MODE & 1) || !real) ? reinterpret_cast<const unsigned char*>(g_win_zero_row + 4 * pos)
                                     : reinterpret_cast<const unsigned char*>(x) + static_cast<uint64_t>(c) * ldxb +
                                           16u * static_cast<uint32_t>(pos ^ (k & C::SWZ));
    };
    auto ext_dma = [&](int i, const unsigned char* src) {
        wdma(src, wlds(lds + C::OFF_EXT + (wave * C::EPW + i * C::RPP) * C::ROWB));
    };

    // ------------------------------------------------------------ prologue
    for (int i = tid; i < C::ROWB / 4; i += C::NT) reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
    if (tid < 8) DV[tid] = hdr->dv[tid];
    // W split in registers: A fragment (cb, kc) of lane l = W[16 cb + (l & 15)]
    // [32 kc + 8 (l >> 4) .. +7], one exponent per 16-column block
    f16x8w wh[4][2], wl[4][2];
    int qw[4] = {0, 0, 0, 0};
    if constexpr (!AGG) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            float wv[2][8];
            uint32_t m = 0;
#pragma unroll
            for (int kc = 0; kc < 2; ++kc) {
                const float* pw = W + static_cast<int64_t>(16 * cb + r) * H + 32 * kc + 8 * g;
                const float4 a = ld4(pw), b = ld4(pw + 4);
                float* w8 = wv[kc];
                w8[0] = a.x; w8[1] = a.y; w8[2] = a.z; w8[3] = a.w;
                w8[4] = b.x; w8[5] = b.y; w8[6] = b.z; w8[7] = b.w;
#pragma unroll
                for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(fabsf(w8[j])));
            }
            qw[cb] = wsplit_exp(wwave_max(m));
#pragma unroll
            for (int kc = 0; kc < 2; ++kc)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float sv = ldexpf(wv[kc][j], qw[cb]);
                    const _Float16 hh = static_cast<_Float16>(sv);
                    wh[cb][kc][j] = hh;
                    wl[cb][kc][j] = static_cast<_Float16>(sv - static_cast<float>(hh));
                }
        }
        if (tid < H) {
            EPI[tid] = (flags & MIGNN_EPI_BIAS) ? bias[tid] : 0.f;
            EPI[H + tid] = (flags & MIGNN_EPI_AFFINE) ? scale[tid] : 1.f;
            EPI[2 * H + tid] = (flags & MIGNN_EPI_AFFINE) ? shift[tid] : 0.f;
        }
    }
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    unsigned char* const STG = lds + C::OFF_STG + wave * C::STG_BYTES;

    dma_tab(tile_of(0), 0);
#pragma unroll
    for (int pp = 0; pp < C::NPX; ++pp) dma_own(tile_of(0), 0, pp);
    dma_tab(tile_of(1), 1);
#pragma unroll
    for (int pp = 0; pp < C::NPX; ++pp) dma_own(tile_of(1), 1, pp);
    wbar<wvm(0) & kWLgkm0>();
    rexp(0);
    {
        const unsigned char* es[C::NPE];
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(0, i, true);
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) ext_dma(i, es[i]);
    }

    f32x4 accp[4];
    uint32_t ncode = C::OFF_ZERO;
    float nwt = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) accp[k] = f32x4{0.f, 0.f, 0.f, 0.f};

    // schedule: cur / nx1 = tiles of steps s / s + 1, the cursor at s + 2
    int64_t prv = -1, cur = tile_of(0), nx1 = tile_of(1);
    WinCursor c2{0, 0, 0};
    c2.next(S.L);
    c2.next(S.L);
    int xs = 0;
    // ---- the pipelined step: phase B and the split of tile
    // s - 1 first (its +z rows are in tile s, landed at B0), its 24 MFMAs in
    // four groups between phase A's slot batches of tile s, its epilogue,
    // staging and stores before B1, then this step's DMA pieces
    for (int s = 0;; ++s) {
        if (cur < 0 && prv < 0) break;            // (uniform)
        const int64_t nx2 = win_tile_c(S, p, c2);
        const int xp = xs == 0 ? 2 : xs - 1;      // slot of tile s - 1 (and of tile s + 2)
        const int tq = static_cast<int>(s & 1);
        const int64_t t0 = rb + (cur >= 0 ? cur : 0) * C::BM;
        const int64_t nloc = cur >= 0 ? (re - t0 < C::BM ? re - t0 : C::BM) : 0;
        const int64_t tp0 = rb + (prv >= 0 ? prv : 0) * C::BM;
        const int64_t nlocp = prv >= 0 ? (re - tp0 < C::BM ? re - tp0 : C::BM) : 0;
        const unsigned char* const X = lds + C::OFF_X + xs * C::X_BYTES;
        const unsigned char* const XP = lds + C::OFF_X + xp * C::X_BYTES;
        wtr.flush(wave, s - 1);
        wtr.stamp(0);
        // (B0) this step's ext rows and the records of step s + 1 landed;
        // younger: the own rows of tile s + 1 (the last step's stores are
        // older: issued before its B1)
        if (s == 0) wbar<wvm(0) & kWLgkm0>();
        else wbar<wvm(C::NPX) & kWLgkm0>();
        wtr.stamp(1);
        // phase B of tile s - 1 and its split (registers only)
        const bool mf = !AGG && prv >= 0;         // (uniform)
        f16x8w bh[2], bl[2];
        f32x4 acc[4];
        int pe = 0;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (prv >= 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f32x4 v = *reinterpret_cast<const f32x4*>(lds + (ncode ^ coff[k]));
#pragma unroll
                for (int t = 0; t < 4; ++t) accp[k][t] = fmaf(nwt, v[t], accp[k][t]);
            }
        }
        if constexpr (AGG) {
            // the aggregate alone: tile s - 1's sums are its output -- staged
            // and stored before phase A of tile s (the stores drain under it)
            if (prv >= 0) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    *reinterpret_cast<f32x4*>(STG + rw * C::ROWB + (((coff[k] >> 4) ^ rw) << 4)) = accp[k];
                const int ch = lane & 15;
                f32x4 v[C::NST];
#pragma unroll
                for (int i = 0; i < C::NST; ++i) {
                    const int sr = i * C::RPP + (lane >> 4);
                    v[i] = *reinterpret_cast<const f32x4*>(STG + sr * C::ROWB + ((ch ^ sr) << 4));
                }
#pragma unroll
                for (int i = 0; i < C::NST; ++i) {
                    const int lr = C::RPW * wave + i * C::RPP + (lane >> 4);
                    if (lr < nlocp)
                        __builtin_nontemporal_store(v[i], reinterpret_cast<f32x4*>(out + (tp0 + lr) * ldo + 4 * ch));
                }
            }
        }
        if (mf) {
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int t = 0; t < 4; ++t) m = max(m, __float_as_uint(fabsf(accp[k][t])));
            pe = wsplit_exp(wrow4_max(m));
            const float sc = __uint_as_float(static_cast<uint32_t>(pe + 127) << 23);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float sv = accp[k][t] * sc;
                    const _Float16 hh = static_cast<_Float16>(sv);
                    bh[k >> 1][4 * (k & 1) + t] = hh;
                    bl[k >> 1][4 * (k & 1) + t] = static_cast<_Float16>(sv - static_cast<float>(hh));
                }
        }
        // MFMA group g: column block g, both k-chunks
        auto mid = [&](auto G) {
            constexpr int cb = decltype(G)::value;
            if (!mf) return;
            __builtin_amdgcn_sched_barrier(0);
            if constexpr ((MODE & 4) == 0) {
#pragma unroll
                for (int kc = 0; kc < 2; ++kc) {
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cb][kc], bh[kc], acc[cb], 0, 0, 0);
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cb][kc], bl[kc], acc[cb], 0, 0, 0);
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[cb][kc], bh[kc], acc[cb], 0, 0, 0);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        // ---- phase A of tile s (the four MFMA groups between its batches)
        f32x4 accn[4];
        uint32_t ncn = C::OFF_ZERO;
        float nwn = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) accn[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        const unsigned char* const RW = lds + C::OFF_TAB + tq * C::TAB_BYTES + wave * C::RECW;
        const uint32_t summ = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
            *reinterpret_cast<const int*>(RW + C::OFF_RL + 4 * C::EPW)));
        const bool live = cur >= 0;
        const bool far = live && ((summ >> 8) & 1u) != 0u;
        const int maxa = (live && !far) ? static_cast<int>(summ & 0xffu) : 0;
        {
            const uint4 cds = *reinterpret_cast<const uint4*>(RW + rw * kWRec);
            auto codeof = [&](int u) -> uint32_t {
                const uint32_t d = u < 2 ? cds.x : u < 4 ? cds.y : u < 6 ? cds.z : cds.w;
                return (u & 1) ? (d >> 16) : (d & 0xffffu);
            };
            const unsigned char* const wr = RW + C::OFF_RW + rw * 32;
            auto wld = [&](int u) -> float { return *reinterpret_cast<const float*>(wr + 4 * u); };
            f32x4 vv[2][4];
            float wv[2];
            auto bload = [&](auto U0, auto NB) {
                constexpr int u0 = decltype(U0)::value, nb = decltype(NB)::value;
#pragma unroll
                for (int uu = 0; uu < nb; ++uu) {
                    const uint32_t cd = codeof(u0 + uu);
#pragma unroll
                    for (int k = 0; k < 4; ++k) vv[uu][k] = *reinterpret_cast<const f32x4*>(lds + (cd ^ coff[k]));
                    wv[uu] = wld(u0 + uu);
                }
            };
            auto bfma = [&](auto NB) {
                constexpr int nb = decltype(NB)::value;
#pragma unroll
                for (int uu = 0; uu < nb; ++uu)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
#pragma unroll
                        for (int t = 0; t < 4; ++t) accn[k][t] = fmaf(wv[uu], vv[uu][k][t], accn[k][t]);
            };
            using U0 = std::integral_constant<int, 0>;
            using U2 = std::integral_constant<int, 2>;
            using U4 = std::integral_constant<int, 4>;
            using U6 = std::integral_constant<int, 6>;
            using N1 = std::integral_constant<int, 1>;
            using N2 = std::integral_constant<int, 2>;
            if (maxa > 0) bload(U0{}, N2{});
            mid(I0{});
            if (maxa > 0) bfma(N2{});
            if (maxa > 2) bload(U2{}, N2{});
            mid(I1{});
            if (maxa > 2) bfma(N2{});
            if (maxa > 4) bload(U4{}, N2{});
            mid(I2{});
            if (maxa > 4) bfma(N2{});
            if (maxa > 6) bload(U6{}, N1{});
            mid(I3{});
            if (maxa > 6) bfma(N1{});
            if (live && !far) {
                ncn = codeof(7);
                nwn = wld(7);
            }
        }
        if (far && lrow < nloc) {
            // CSR path: the full sum in CSR order, the current tile from
            // LDS, every other row from x (L2); 2 entries at a time
            const int64_t row = t0 + lrow;
            const int eb = row_ptr[row], ee = row_ptr[row + 1];
            for (int e = eb; e < ee; e += 2) {
                int cj[2];
                float wj[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const bool v = e + u < ee;
                    cj[u] = v ? col[e + u] : -1;
                    wj[u] = v ? ew[e + u] : 0.f;
                }
                f32x4 vv[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int64_t off = static_cast<int64_t>(cj[u]) - t0;
                    if (cj[u] < 0) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) vv[u][k] = f32x4{0.f, 0.f, 0.f, 0.f};
                    } else if (off >= 0 && off < nloc) {
                        const uint32_t o = static_cast<uint32_t>(off);
                        const uint32_t a = (static_cast<uint32_t>(X - lds) + o * C::ROWB) | ((o & C::SWZ) << 4);
#pragma unroll
                        for (int k = 0; k < 4; ++k) vv[u][k] = *reinterpret_cast<const f32x4*>(lds + (a ^ coff[k]));
                    } else {
                        const float* rp = x + static_cast<int64_t>(cj[u]) * ldx;
#pragma unroll
                        for (int k = 0; k < 4; ++k) vv[u][k] = *reinterpret_cast<const f32x4*>(rp + (coff[k] >> 2));
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
#pragma unroll
                        for (int t = 0; t < 4; ++t) accn[k][t] = fmaf(wj[u], vv[u][k][t], accn[k][t]);
            }
        }
        wtr.stamp(2);
        // epilogue of tile s - 1 (residual from slot (s-1) % 3, before B1),
        // the wave's 16 rows staged in its own LDS region and read back whole
        f32x4 vst[C::NST];
        if (mf) {
#pragma unroll
            for (int cb = 0; cb < 4; ++cb) {
                const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[16 * cb + 4 * g]);
                f32x4 rv = f32x4{0.f, 0.f, 0.f, 0.f};
                if (has_res)
                    rv = *reinterpret_cast<const f32x4*>(XP + lrow * C::ROWB + (((4 * cb + g) ^ rw) << 4));
                const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + 16 * cb + 4 * g]);
                const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + 16 * cb + 4 * g]);
                f32x4 o;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    float v = ldexpf(acc[cb][t], -(pe + qw[cb])) + (rv[t] + bo[t]);
                    if (flags & MIGNN_EPI_AFFINE) v = v * so[t] + ho[t];
                    if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                    o[t] = v;
                }
                *reinterpret_cast<f32x4*>(STG + rw * C::ROWB + (((4 * cb + g) ^ rw) << 4)) = o;
            }
            const int ch = lane & 15;
#pragma unroll
            for (int i = 0; i < C::NST; ++i) {
                const int sr = i * C::RPP + (lane >> 4);
                vst[i] = *reinterpret_cast<const f32x4*>(STG + sr * C::ROWB + ((ch ^ sr) << 4));
            }
#pragma unroll
            for (int i = 0; i < C::NST; ++i) {
                const int lr = C::RPW * wave + i * C::RPP + (lane >> 4);
                if (lr < nlocp)
                    __builtin_nontemporal_store(vst[i], reinterpret_cast<f32x4*>(out + (tp0 + lr) * ldo + 4 * ch));
            }
        }
        wtr.stamp(3);
        // (B1) slot (s-1) % 3, the ext area and this step's records free
        wbar<kWLgkm0>();
        {
            const int64_t tn2 = nx2;
            // (the ext list of step s + 1 landed at B0; its TAB slot is not
            // refilled this step)
            const unsigned char* es[C::NPE];
#pragma unroll
            for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(tq ^ 1, i, nx1 >= 0);
#pragma unroll
            for (int i = 0; i < C::NPE; ++i) ext_dma(i, es[i]);
            dma_tab(tn2, tq);
#pragma unroll
            for (int pp = 0; pp < C::NPX; ++pp) dma_own(tn2, xp, pp);
        }
        wtr.stamp(5);
        rexp(tq ^ 1);                             // tile s + 1's weights (its records landed at B0)
#pragma unroll
        for (int k = 0; k < 4; ++k) accp[k] = accn[k];
        ncode = ncn;
        nwt = nwn;
        xs = xs == 2 ? 0 : xs + 1;
        prv = cur;
        cur = nx1;
        nx1 = nx2;
        c2.next(S.L);
    }
    wwait<wvm(0)>();   // no LDS-DMA may outlive the workgroup
}

#ifdef MIGNN_DIAG
int win_trace_set(void* buf) {
    MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_win_trace), &buf, sizeof(buf)));
    return MIGNN_OK;
}
#endif

template <int H, int MODE, int EPIF>
void launch_win_k(int G, hipStream_t st, const void* plan, const int32_t* row_ptr,
                  const int32_t* col, const float* ew, const float* x, int64_t ldx, int64_t rb,
                  int64_t re, const float* w, const float* bias, const float* scale,
                  const float* shift, int flags, float* out, int64_t ldo, const float* xcoef) {
    if constexpr (H == 64)
        hipLaunchKernelGGL((gcn_win64_kernel<MODE, EPIF>), dim3(G), dim3(WCfg<64>::NT), 0, st,
                           static_cast<const unsigned char*>(plan), row_ptr, col, ew, x, ldx, rb, re, w,
                           bias, scale, shift, flags, out, ldo);
    else
        hipLaunchKernelGGL((gcn_win_kernel<H, MODE, EPIF>), dim3(G), dim3(WCfg<H>::NT), 0, st,
                           static_cast<const unsigned char*>(plan), row_ptr, col, ew, x, ldx, rb, re, w,
                           bias, scale, shift, flags, out, ldo, xcoef);
}

template <int H, int MODE>
void launch_win_h(int G, hipStream_t st, const void* plan, const int32_t* row_ptr,
                  const int32_t* col, const float* ew, const float* x, int64_t ldx, int64_t rb,
                  int64_t re, const float* w, const float* bias, const float* scale,
                  const float* shift, int flags, float* out, int64_t ldo, const float* xcoef) {
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    constexpr bool EPIC = MODE == 0 || MODE == 64;   // the product modes: flags at compile time
    if (EPIC && flags == kBN)
        launch_win_k<H, MODE, kBN>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, xcoef);
    else if (EPIC && flags == kNoBN)
        launch_win_k<H, MODE, kNoBN>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, xcoef);
    else
        launch_win_k<H, MODE, -1>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, xcoef);
}

template <int MODE = 0>
int launch_win(int h, const void* plan, const int32_t* row_ptr, const int32_t* col,
               const float* ew, const float* x, int64_t ldx, int64_t rb, int64_t re,
               const float* w, const float* bias, const float* scale, const float* shift,
               int flags, float* out, int64_t ldo, hipStream_t st, const float* xcoef = nullptr) {
    const int64_t ntiles = (re - rb + 63) / 64;
    const int G = win_grid(ntiles, h == 128 ? WCfg<128>::WGPC : WCfg<64>::WGPC);
    MIGNN_REQUIRE(G > 0, "gcn_win: device query failed");
    if (h == 128)
        launch_win_h<128, MODE>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, xcoef);
    else if constexpr ((MODE & 64) == 0)
        launch_win_h<64, MODE>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, xcoef);
    return launch_status("gcn_win_kernel");
}

}  // namespace

int win_device_errors(unsigned int* out, int clear) {
    unsigned int v = 0u;
    MIGNN_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_win_errors), sizeof(unsigned int), 0,
                                  hipMemcpyDeviceToHost));
    *out |= v;
    if (clear) {
        const unsigned int zero = 0u;
        MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_win_errors), &zero, sizeof(unsigned int), 0,
                                    hipMemcpyHostToDevice));
    }
    return MIGNN_OK;
}

}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_gcn_win_plan_bytes(int64_t row_begin, int64_t row_end, int h) {
    if (row_end <= row_begin || (h != 64 && h != 128)) return 0;
    const int64_t ntiles = (row_end - row_begin + 63) / 64;
    return kWHdr + static_cast<size_t>(ntiles) * (h == 128 ? WCfg<128>::TAB_G : WCfg<64>::TAB_G);
}

extern "C" int mignn_gcn_win_plan(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                  int64_t rb, int64_t re, int h, const int32_t* order_info,
                                  void* plan, size_t plan_bytes, unsigned long long* stats,
                                  void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && plan, "gcn_win_plan: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_win_plan: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_win_plan: bad row range");
    MIGNN_REQUIRE(aligned16(plan), "gcn_win_plan: unaligned plan");
    if (re == rb) return MIGNN_OK;
    MIGNN_REQUIRE(plan_bytes >= mignn_gcn_win_plan_bytes(rb, re, h), "gcn_win_plan: plan buffer too small");
    const int64_t ntiles = (re - rb + 63) / 64;
    const int G = win_grid(ntiles, h == 128 ? WCfg<128>::WGPC : WCfg<64>::WGPC);
    MIGNN_REQUIRE(G > 0, "gcn_win_plan: device query failed");
    hipStream_t st = as_stream(stream);
    WinHdr* hdr = static_cast<WinHdr*>(plan);
    if (order_info != nullptr) {
        hipLaunchKernelGGL(win_zrun_init_kernel, dim3(1), dim3(64), 0, st, hdr, ntiles);
        int rc0 = launch_status("win_zrun_init_kernel");
        if (rc0) return rc0;
        hipLaunchKernelGGL(win_zrun_kernel, dim3(grid_for(ntiles, 256, 4096)), dim3(256), 0, st,
                           row_ptr, col, rb, re, ntiles, hdr);
        if ((rc0 = launch_status("win_zrun_kernel"))) return rc0;
    }
    hipLaunchKernelGGL(win_hdr_kernel, dim3(1), dim3(64), 0, st, hdr, order_info, ntiles, G, h, rb, re);
    int rc = launch_status("win_hdr_kernel");
    if (rc) return rc;
    unsigned char* tabs = static_cast<unsigned char*>(plan) + kWHdr;
    const unsigned grid = static_cast<unsigned>(ntiles < (1 << 20) ? ntiles : (1 << 20));
    if (h == 128)
        hipLaunchKernelGGL(win_plan_kernel<128>, dim3(grid), dim3(64), 0, st, row_ptr, col, ew, hdr, tabs, stats);
    else
        hipLaunchKernelGGL(win_plan_kernel<64>, dim3(grid), dim3(64), 0, st, row_ptr, col, ew, hdr, tabs, stats);
    return launch_status("win_plan_kernel");
}

extern "C" int mignn_gcn_layer_win(const void* plan, const int32_t* row_ptr, const int32_t* col,
                                   const float* ew, const float* x, int64_t ldx, int64_t rb,
                                   int64_t re, int h, const float* w, const float* bias,
                                   const float* scale, const float* shift, int flags, float* out,
                                   int64_t ldo, void* stream) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && x && w && out, "gcn_layer_win: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_layer_win: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(plan) && aligned16(w),
                  "gcn_layer_win: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "gcn_layer_win: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_win: bad row range");
    MIGNN_REQUIRE(x != out, "gcn_layer_win: in-place not supported (neighbours read x)");
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_win: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_win: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_win: affine");
    if (re == rb) return MIGNN_OK;
    return launch_win(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out,
                      ldo, as_stream(stream));
}

extern "C" int mignn_gcn_layer_win_codes(const void* plan, const int32_t* row_ptr,
                                         const int32_t* col, const float* ew, const float* codes,
                                         int64_t ldc, int64_t rb, int64_t re, int h,
                                         const float* xcoef, const float* w, const float* bias,
                                         const float* scale, const float* shift, int flags,
                                         float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && codes && xcoef && w && out,
                  "gcn_layer_win_codes: null pointer");
    MIGNN_REQUIRE(h == 128, "gcn_layer_win_codes: h must be 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(codes) && aligned16(out) && aligned16(plan) && aligned16(w) &&
                      aligned16(xcoef),
                  "gcn_layer_win_codes: unaligned");
    MIGNN_REQUIRE(ldc % 4 == 0 && ldc >= 8 && ldo % 4 == 0 && ldo >= h,
                  "gcn_layer_win_codes: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_win_codes: bad row range");
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_win_codes: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_win_codes: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_win_codes: affine");
    if (re == rb) return MIGNN_OK;
    return launch_win<64>(h, plan, row_ptr, col, ew, codes, ldc, rb, re, w, bias, scale, shift,
                          flags, out, ldo, as_stream(stream), xcoef);
}

extern "C" int mignn_gcn_aggregate_win(const void* plan, const int32_t* row_ptr, const int32_t* col,
                                       const float* ew, const float* x, int64_t ldx, int64_t rb,
                                       int64_t re, int h, float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && x && out, "gcn_aggregate_win: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_aggregate_win: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(plan), "gcn_aggregate_win: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h,
                  "gcn_aggregate_win: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_aggregate_win: bad row range");
    MIGNN_REQUIRE(x != out, "gcn_aggregate_win: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    return launch_win<32>(h, plan, row_ptr, col, ew, x, ldx, rb, re, nullptr, nullptr, nullptr,
                          nullptr, 0, out, ldo, as_stream(stream));
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_win_trace(void* buf) { return win_trace_set(buf); }

extern "C" int mignn_diag_win(int mode, const void* plan, const int32_t* row_ptr,
                              const int32_t* col, const float* ew, const float* x, int64_t ldx,
                              int64_t rb, int64_t re, int h, const float* w, const float* bias,
                              const float* scale, const float* shift, int flags, float* out,
                              int64_t ldo, void* stream) {
    hipStream_t st = as_stream(stream);
    switch (mode) {
        case 0: return launch_win<0>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 1: return launch_win<1>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 2: return launch_win<2>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 3: return launch_win<3>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 4: return launch_win<4>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 32: return launch_win<32>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        case 33: return launch_win<33>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        default: break;
    }
    set_error("diag_win: unknown mode %d", mode);
    return MIGNN_ERR_ARG;
}
#endif

MIGNN_DMA_OOB_EXPORT(mignn_diag_dma_oob_win)
