// Fused GCN layer, ring form -- the north-star hot kernel (GCNConv + residual
// + BatchNorm(eval) + ReLU, reference gnn_model.py:63, :166, :184-191; PyG
// GCNConv: out_i = sum_{j->i} w_ij h_j + b, w_ij = dinv_i dinv_j over
// add_remaining_self_loops):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Arithmetic: fp32 aggregation in CSR order (the order of PyG's scatter-add),
// the aggregate split into fp16 hi + lo with a power-of-two row scale, three
// fp16 MFMA products with fp32 accumulation (~2^-22 relative per product) --
// gcn_f16x3.hip's scheme.
//
// Why this structure.  A layer streams 64 KB per 64-row tile through its CU
// (32 KB of own rows in, 32 KB out) plus ~48 KB of neighbour rows from L2.
// vmcnt completes in issue order, so any load the kernel consumes every tile
// forces every OLDER load to have landed: a next-tile DMA issued before it
// gets at most one tile of lead.  Here nothing in the tile loop is a
// compiler-visible load -- every global read is an LDS-DMA (inline asm,
// counted by hand):
//   * own rows and the tile's plan records: a 2-deep ring, issued 1.5 tiles
//     ahead;
//   * out-of-tile ("ext") rows: DMA'd with per-lane source addresses into an
//     LDS ext area half a tile ahead (they are mostly L2 hits: the
//     XCD-contiguous tile order keeps a tile's neighbour tiles in flight on
//     the same XCD).
// With both in LDS, every CSR entry of a row is one {LDS offset, w} slot of
// its plan record, and the aggregation is one branch-free loop (8 FMAs + 1
// XOR per slot and lane).  One 8-wave workgroup per CU (2 waves per SIMD):
// each wave sums 8 rows (quad layout: a row = 16 lanes x 32 B), splits them
// into the shared A image, transforms 16 output columns of all 64 rows (W
// split in registers), stages its part; whole rows are stored.  Four
// s_barriers per tile, no spin waits.
//
// The plan (mignn_gcn_ring_plan; built per graph, row range and h): a 64-B
// record per row -- 8 slots {code, w} in CSR order (code = the LDS offset of
// the neighbour row: the tile's ring slot, chosen by the tile's step parity
// under the kernel's fixed schedule, or an ext slot; empty slots point at a
// zero row with w = 0; entries past the ext capacity are "far": bit 31 +
// column, gathered synchronously) -- and per tile the ext columns in the
// order of the DMA pieces with each wave's summary (max degree, far, slow).
#include "common.hpp"

namespace mignn {
MIGNN_DMA_OOB_WORD
namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_r;
using f16x8r = __attribute__((ext_vector_type(8))) _Float16;
using f16x4r = __attribute__((ext_vector_type(4))) _Float16;

constexpr int kRec = 64;        // bytes per plan record
constexpr int kSl = 8;          // slots per record
constexpr uint32_t kFar = 0x80000000u;

template <int H>
struct RCfg {
    static_assert(H == 64 || H == 128, "ring GCN layer: H in {64, 128}");
    // 64-row tiles (the locality order's 4 x 4 x 4 blocks).  (32-row tiles at
    // H = 128 -- 4 x 4 x 2 slabs, two workgroups per CU -- measured slower:
    // 3.15 vs 3.09 ms, their 2:1 out-of-tile rows per own row cost more
    // than the second workgroup gains; BM = 32 builds, KX = 64 then)
    static constexpr int BM = 64, NW = BM / 8, NT = NW * 64;
    static constexpr int F = H / 16, CH = F / 4;       // floats / 16-B chunks per lane of a row
    static constexpr int ROWB = H * 4;
    static constexpr int AS = H + 16;                  // A row stride, halfs
    static constexpr int X_BYTES = BM * ROWB;
    static constexpr int KX = BM == 32 ? 64 : 96;      // ext rows per tile in LDS
    static constexpr int EXT_BYTES = KX * ROWB;
    static constexpr int EPW = KX / NW;                // ext rows DMA'd per wave (12 or 16)
    static constexpr int XLW = (EPW + 4) / 4 * 4;      // ext-list group per wave: EPW columns, the summary
    static constexpr int RECW = 8 * kRec + XLW * 4;    // a wave's records + list in LDS
    static constexpr int TLANES = RECW / 16;           // lanes of its DMA
    static constexpr int TAB_BYTES = BM * kRec + NW * XLW * 4;   // records + ext list (4608)
    static constexpr int A_BYTES = BM * AS * 2;
    // E2 (where LDS allows): the ext rows double-buffered and DMA'd a whole
    // step ahead (at the top of the previous step), the records 3 steps ahead
    static constexpr bool E2 = false;   // (measured no faster at H = 64)
    // X1: one own-row slot (the next tile's rows DMA'd once this tile's are
    // consumed), which leaves LDS for WGPC = 2 workgroups per CU
    static constexpr bool X1 = H == 64;
    static constexpr int WGPC = X1 ? 2 : 1;
    static_assert(!(X1 && E2), "X1 with E2: not built");
    static constexpr int NE = E2 ? 2 : 1;              // ext areas
    static constexpr int NTB = E2 ? 3 : 2;             // record (TAB) slots
    // LDS: X[2] | EXT[NE] | TAB[NTB] | zero row | AH | AL | REXP | EPI
    static constexpr int OFF_X0 = 0;
    static constexpr int OFF_X1 = X1 ? 0 : X_BYTES;
    static constexpr int OFF_EXT = (X1 ? 1 : 2) * X_BYTES;
    static constexpr int OFF_TAB = OFF_EXT + NE * EXT_BYTES;
    static constexpr int OFF_ZERO = OFF_TAB + NTB * TAB_BYTES;
    static constexpr int OFF_AH = OFF_ZERO + ROWB;
    static constexpr int OFF_AL = OFF_AH + A_BYTES;
    static constexpr int OFF_REXP = OFF_AL + A_BYTES;
    static constexpr int OFF_EPI = OFF_REXP + BM * 4;
    static constexpr int LDS_BYTES = OFF_EPI + 3 * H * 4;
    static constexpr int OFF_STG = OFF_AH;
    static constexpr int NQ = 2;                       // row quads per wave (8 rows)
    static constexpr int UB = 4;                       // slots per LDS batch
    static constexpr int VPL = H / 64;
    static constexpr int WN = H / 16;                  // 16-column blocks
    static constexpr int WM = NW / WN;                 // row groups (1 or 2)
    static constexpr int IBW = (BM / 16) / WM;         // 16-row blocks per wave
    static constexpr int KC = H / 32;
    static constexpr int RPP = 1024 / ROWB, LPR = 64 / RPP;   // rows / lanes per row of a piece
    static constexpr int NPX = X_BYTES / 1024 / NW;    // own-row pieces per wave
    static constexpr int NPE = EXT_BYTES / 1024 / NW;  // ext pieces per wave
    static constexpr int LPRW = ROWB / 16, RPI = 64 / LPRW;
    static constexpr int NST = 8 / RPI;                // row stores per wave (8 rows)
    static constexpr int NDMA = 1 + NPX;               // ring DMA ops per wave per tile
    static_assert(LDS_BYTES * WGPC <= 160 * 1024, "LDS budget");
    static_assert(BM * ROWB <= 2 * A_BYTES, "staging tile fits the A image");
    static_assert(EPW == NPE * RPP && EPW < XLW && RECW % 16 == 0 && TLANES <= 64, "ext rows per wave");
    static_assert(OFF_EXT + NE * EXT_BYTES <= (1 << 17), "codes below bit 17");
};

// the launch grid of the ring kernel and the step parity of each tile under
// its schedule (tile_of below): both the plan and the launch use these
__host__ __device__ inline int64_t ring_steps(int64_t ntiles, int G) { return (ntiles + G - 1) / G; }
__host__ __device__ inline int ring_parity(int64_t tile, int64_t ntiles, int G) {
    const int64_t per_xcd = G / 8;
    const int64_t chunk = ring_steps(ntiles, G) * per_xcd;
    return static_cast<int>(((tile % chunk) / per_xcd) & 1);
}

// plan header (the first kRHdr bytes): the grid the schedule was built for,
// checked by the kernel (a mismatch: MIGNN_DEVERR_PLAN, the rows set to NaN)
constexpr int kRHdr = 256;
constexpr uint32_t kRMagic = 0x474E4952u;
struct RingHdr {
    uint32_t magic;
    int32_t G, h, pad;
    int64_t rb, re;
};
__device__ unsigned int g_ring_errors = 0u;

int ring_grid(int64_t ntiles, int wgpc) {
    static int cus_cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    int& cus = cus_cache[dev & 63];
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -1;
        if (cus < 1) cus = 1;
    }
    int G = (cus * wgpc / 8) * 8;
    if (G < 8) G = 8;
    if (ntiles < G) G = static_cast<int>(((ntiles + 7) / 8) * 8);
    return G;
}

constexpr int rvm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xF00; }   // vmcnt(n)
constexpr int rvm_l(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70; }         // + lgkmcnt(0)
constexpr int kRLgkm0 = 0xC07F;

template <int W>
__device__ __forceinline__ void rwait() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(W);
    asm volatile("" ::: "memory");
}
template <int W>
__device__ __forceinline__ void rbar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(W);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint32_t rlds(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_r)(p)));
}

__device__ __forceinline__ void rdma(const void* src, uint32_t dst) {
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

// a wave-uniform 64-bit address, in SGPRs
__device__ __forceinline__ uint64_t runi(const void* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<int>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// the same with an SGPR base address and a per-lane 32-bit offset (no
// per-piece address arithmetic: the offsets are fixed per lane)
__device__ __forceinline__ void rdma_s(const void* base, uint32_t voff, uint32_t dst) {
    MIGNN_DMA_BOUND(dst);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(runi(base)), "s"(__builtin_amdgcn_readfirstlane(static_cast<int>(dst)))
        : "memory");
}

__device__ __forceinline__ int rsplit_exp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}
__device__ __forceinline__ uint32_t rrow_max(uint32_t v) {
    int t = static_cast<int>(v);
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x124, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x128, 0xf, 0xf, false)));
    return static_cast<uint32_t>(t);
}
__device__ __forceinline__ uint32_t rwave_max(uint32_t v) {
    const uint32_t t = rrow_max(v);
    const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 0));
    const uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 16));
    const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 32));
    const uint32_t d = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(t), 48));
    return max(max(a, b), max(c, d));
}

__device__ __attribute__((aligned(16))) float g_ring_zero_row[256];

// diagnostic timeline (mignn_diag_ring_trace): s_memtime stamps of waves 0
// and 4 of workgroups 0..7, steps 0..63 -> trace[((b * 64 + s) * 2 + w/4) * 16 + point]
#ifdef MIGNN_DIAG
__device__ unsigned long long* g_ring_trace = nullptr;
#endif
// stamps of one step collect in lanes 0..7 of a VGPR pair (v_writelane: no
// memory traffic); the previous step's are written by ONE store at the next
// step's top, after its barrier
struct RTrace {
    unsigned long long* tr;   // null: tracing off (the product build)
    uint32_t lo, hi;
    int lane;
    __device__ __forceinline__ void stamp(int pt) {
        if (tr == nullptr) return;
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        lo = lane == pt ? static_cast<uint32_t>(t) : lo;
        hi = lane == pt ? static_cast<uint32_t>(t >> 32) : hi;
    }
    __device__ __forceinline__ void flush(int wave, int lane, int64_t s) {
        if (tr == nullptr || blockIdx.x >= 8 || s < 0 || s >= 64 || (wave != 0 && wave != 4)) return;
        if (lane < 8)
            tr[((blockIdx.x * 64 + s) * 2 + (wave >> 2)) * 16 + lane] =
                (static_cast<unsigned long long>(hi) << 32) | lo;
    }
};

// ------------------------------------------------------------------ plan
// One 64-thread block per tile, a thread per row.  Ext slots are numbered in
// row-major order of the tile's out-of-tile entries (a wave-wide prefix sum),
// not deduplicated; slot k < KX lives at LDS row k of the ext area, its column
// in list entry (k / EPW) * XLW + k % EPW (the DMA pieces of wave k / EPW).
template <int H>
__global__ __launch_bounds__(RCfg<H>::BM) void ring_plan_kernel(const int32_t* __restrict__ row_ptr,
                                                       const int32_t* __restrict__ col,
                                                       const float* __restrict__ ew, int64_t rb,
                                                       int64_t re, int64_t ntiles, int G,
                                                       unsigned char* __restrict__ plan,
                                                       unsigned long long* __restrict__ stats) {
    using C = RCfg<H>;
    const int lr = threadIdx.x;
    __shared__ uint32_t xl[C::NW * C::XLW];
    if (blockIdx.x == 0 && lr == 0) {
        RingHdr* const hd = reinterpret_cast<RingHdr*>(plan);
        hd->magic = kRMagic;
        hd->G = G;
        hd->h = H;
        hd->pad = 0;
        hd->rb = rb;
        hd->re = re;
    }
    plan += kRHdr;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t t0 = rb + t * C::BM;
        const int64_t r = t0 + lr;
        const uint32_t nloc = static_cast<uint32_t>(re - t0 < C::BM ? re - t0 : C::BM);
        const int tpar = ring_parity(t, ntiles, G);
        const uint32_t xoff = tpar ? C::OFF_X1 : C::OFF_X0;
        const uint32_t eoff = C::OFF_EXT + (C::E2 && tpar ? C::EXT_BYTES : 0);
        for (int i = lr; i < C::NW * C::XLW; i += C::BM) xl[i] = 0u;   // unused: row 0, never read
        int e0 = 0, deg = 0, next = 0;
        if (r < re) {
            e0 = row_ptr[r];
            deg = row_ptr[r + 1] - e0;
            if (deg <= kSl)
                for (int e = 0; e < deg; ++e) {
                    const int64_t c = col[e0 + e];
                    if (!(c >= t0 && c < t0 + nloc)) ++next;
                }
        }
        // exclusive prefix of the ext counts over the tile's rows
        int pre = next;
#pragma unroll
        for (int d = 1; d < C::BM; d <<= 1) {
            const int v = __shfl_up(pre, d, C::BM);
            if (lr >= d) pre += v;
        }
        pre -= next;
        __syncthreads();
        uint32_t rec[16];
#pragma unroll
        for (int s = 0; s < kSl; ++s) {
            rec[2 * s] = C::OFF_ZERO;
            rec[2 * s + 1] = 0u;
        }
        const bool slow = deg > kSl;
        unsigned long long nfar = 0;
        if (r < re && !slow) {
            int k = pre;
            for (int e = 0; e < deg; ++e) {
                const int64_t c = col[e0 + e];
                const uint32_t wb = __float_as_uint(ew[e0 + e]);
                uint32_t code;
                if (c >= t0 && c < t0 + nloc) {
                    const uint32_t off = static_cast<uint32_t>(c - t0);
                    code = (xoff + off * C::ROWB) | ((off & 7u) << 4);
                } else if (k < C::KX) {
                    code = (eoff + k * C::ROWB) | ((static_cast<uint32_t>(k) & 7u) << 4);
                    xl[(k / C::EPW) * C::XLW + k % C::EPW] = static_cast<uint32_t>(c);
                    ++k;
                } else {
                    code = kFar | static_cast<uint32_t>(c);
                    ++nfar;
                    ++k;
                }
#pragma unroll
                for (int s = 0; s < kSl; ++s)
                    if (s == e) {
                        rec[2 * s] = code;
                        rec[2 * s + 1] = wb;
                    }
            }
        }
        const uint32_t far = nfar ? 1u : 0u;
        const uint32_t d8 = slow ? 0u : static_cast<uint32_t>(deg);
        // summary of the row's wave (8 rows): max degree | any far | any slow,
        // kept in entry 12 of the wave's ext-list group
        uint32_t md = d8, af = far, as = slow ? 1u : 0u;
#pragma unroll
        for (int d = 1; d < 8; d <<= 1) {
            md = max(md, static_cast<uint32_t>(__shfl_xor(static_cast<int>(md), d, 8)));
            af |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(af), d, 8));
            as |= static_cast<uint32_t>(__shfl_xor(static_cast<int>(as), d, 8));
        }
        if ((lr & 7) == 0) xl[(lr >> 3) * C::XLW + C::EPW] = md | (af << 8) | (as << 16);
        __syncthreads();
        unsigned char* const base = plan + t * C::TAB_BYTES;
        uint4* dst = reinterpret_cast<uint4*>(base + lr * kRec);
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[i] = make_uint4(rec[4 * i], rec[4 * i + 1], rec[4 * i + 2], rec[4 * i + 3]);
        for (int i = lr; i < C::NW * C::XLW; i += C::BM)
            reinterpret_cast<uint32_t*>(base + C::BM * kRec)[i] = xl[i];
        if (stats != nullptr) {
            const int kt = __shfl(pre + next, C::BM - 1, C::BM);
            if (nfar) atomicAdd(&stats[1], nfar);
            if (slow) atomicAdd(&stats[2], 1ull);
            if (lr == C::BM - 1 && kt > C::KX) atomicAdd(&stats[0], 1ull);
            if (lr == C::BM - 1) atomicMax(&stats[3], static_cast<unsigned long long>(kt));
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- layer
// MODE (timing ablations, mignn_diag_ring only; 0 in the product; every
// variant keeps the DMA op counts): 1 ext rows from the zero row, 2 no
// aggregation sums, 4 no MFMAs, 8 own rows DMA'd from the zero row; 16 the
// epilogue stored straight from the accumulators (no staging, 2 barriers per
// step instead of 4); 64 two 16-column blocks per wave (each A fragment feeds
// both: half the A-image LDS reads); 32 aggregate only (product:
// mignn_gcn_aggregate_ring)
// EPIF: the epilogue flags at compile time (15 = BIAS|RESIDUAL|AFFINE|RELU,
// 11 = BIAS|RESIDUAL|RELU: FlowGNN with / without BatchNorm), -1: from `flags`
template <int H, int MODE = 0, int EPIF = -1>
__global__ __launch_bounds__(RCfg<H>::NT, RCfg<H>::WGPC) void gcn_ring_kernel(
    const unsigned char* __restrict__ plan, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ col, const float* __restrict__ ew, const float* __restrict__ x,
    int64_t ldx, int64_t row_begin, int64_t row_end, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    using C = RCfg<H>;
    constexpr bool AGG = (MODE & 32) != 0;   // aggregate only (mignn_gcn_aggregate_ring)
    if constexpr (EPIF >= 0) flags = EPIF;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    _Float16* const AH = reinterpret_cast<_Float16*>(lds + C::OFF_AH);
    _Float16* const AL = reinterpret_cast<_Float16*>(lds + C::OFF_AL);
    int* const REXP = reinterpret_cast<int*>(lds + C::OFF_REXP);
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    {
        const RingHdr* const hd = reinterpret_cast<const RingHdr*>(plan);
        const bool ok = hd->magic == kRMagic && hd->G == static_cast<int>(gridDim.x) && hd->h == H &&
                        hd->rb == row_begin && hd->re == row_end;
        if (!ok) {
            if (tid == 0)
                __hip_atomic_fetch_or(&g_ring_errors, static_cast<unsigned>(MIGNN_DEVERR_PLAN),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            plan_mismatch_fill(out, ldo, row_begin, row_end, H);
            return;
        }
    }
    plan += kRHdr;
    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + C::BM - 1) / C::BM;
    const int G = gridDim.x;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = G >> 3;
    const int64_t nsteps = ring_steps(ntiles, G);
#ifdef MIGNN_DIAG
    RTrace rtr{(blockIdx.x < 8 && (wave == 0 || wave == 4)) ? g_ring_trace : nullptr, 0u, 0u, lane};
#else
    RTrace rtr{nullptr, 0u, 0u, lane};
#endif
    auto tile_of = [&](int64_t s) -> int64_t { return (int64_t)xcd * nsteps * per_xcd + s * per_xcd + slot; };
    // a tile of this workgroup's schedule, or (past its end) tile 0: the DMA
    // op counts stay uniform, the loads are never read
    auto tile_or0 = [&](int64_t s) -> int64_t {
        const int64_t t = tile_of(s);
        return (s < nsteps && t < ntiles) ? t : 0;
    };

    const int gq = lane >> 4, iq = lane & 15;
    const int hb = (iq >= 4 && iq < 12) ? 1 : 0;
    const int c0 = (hb ? iq - 4 : (iq < 4 ? iq : iq - 8)) | (hb << 3);
    const uint32_t coff0 = static_cast<uint32_t>(c0 << 4);

    // ring DMA of step s: this wave's 8 records + its ext-list group (36
    // lanes), then its share of the tile's own rows; SGPR bases, per-lane
    // offsets fixed for the launch (a partial last tile clamps per lane)
    const uint32_t ldxb = static_cast<uint32_t>(ldx) * 4u;
    uint32_t xoff[C::NPX];
#pragma unroll
    for (int pp = 0; pp < C::NPX; ++pp) {
        const int p = pp * C::NW + wave;
        const int lr = p * C::RPP + lane / C::LPR;
        const int pos = lane % C::LPR;
        xoff[pp] = static_cast<uint32_t>(lr) * ldxb + 16u * static_cast<uint32_t>(pos ^ (lr & 7));
    }
    const uint32_t toff = lane < 32 ? static_cast<uint32_t>(wave * 512 + 16 * lane)
                                    : static_cast<uint32_t>(C::BM * kRec + wave * (C::XLW * 4) + 16 * (lane - 32));
    // the record slot of step s
    auto tslot = [&](int64_t s) -> int { return C::E2 ? static_cast<int>(s % 3) : static_cast<int>(s & 1); };
    auto dma_tab = [&](int64_t s) {
        const int64_t tile = tile_or0(s);
        if (lane < C::TLANES)
            rdma_s(plan + tile * C::TAB_BYTES, toff,
                   rlds(lds + C::OFF_TAB + tslot(s) * C::TAB_BYTES + wave * C::RECW));
    };
    // piece q of step s's ring DMA: q = 0 the records (E2: those of step
    // s + 1), 1 .. NPX own rows
    auto dma_tile_piece = [&](int64_t s, int q) {
        if (q == 0) {
            dma_tab(C::E2 ? s + 1 : s);
            return;
        }
        const int64_t tile = tile_or0(s);
        const int64_t t0 = row_begin + tile * C::BM;
        const int par = static_cast<int>(s & 1);
        const int pp = q - 1;
        const int p = pp * C::NW + wave;
        unsigned char* const X = lds + (par ? C::OFF_X1 : C::OFF_X0);
        if ((MODE & 8) == 0 && t0 + C::BM <= row_end) {
            rdma_s(x + t0 * ldx, xoff[pp], rlds(X + p * 1024));
        } else {
            int l = lane;
            asm volatile("" : "+v"(l));
            const int lr = p * C::RPP + l / C::LPR;
            const int pos = l % C::LPR;
            int64_t row = t0 + lr;
            if (row >= row_end) row = row_end - 1;
            rdma((MODE & 8) ? g_ring_zero_row + 4 * (pos & 31) : x + row * ldx + 4 * (pos ^ (lr & 7)),
                 rlds(X + p * 1024));
        }
    };
    auto dma_tile = [&](int64_t s) {
#pragma unroll
        for (int q = 0; q <= C::NPX; ++q) dma_tile_piece(s, q);
    };
    // piece q of the ring DMA issued after B1 of step s: the records of step
    // s + 2 (E2: s + 3), then the own rows of step s + 2 (X1: s + 1, into the
    // slot step s just released)
    auto ring_piece = [&](int64_t s, int q) {
        if (q == 0) dma_tab(C::E2 ? s + 3 : s + 2);
        else dma_tile_piece(C::X1 ? s + 1 : s + 2, q);
    };
    // ext rows of step s (its records' ext list): piece i of this wave's
    // ext rows k = EPW wave .. +EPW (chunk c of row k at position c ^ (k & 7));
    // unused list entries hold column 0 (loaded, never read)
    auto ext_src = [&](int64_t s, int i) -> const unsigned char* {
        const unsigned char* const tab = lds + C::OFF_TAB + tslot(s) * C::TAB_BYTES + wave * C::RECW + 512;
        int l = lane;
        asm volatile("" : "+v"(l));
        const int kk = i * C::RPP + l / C::LPR;          // within the wave's rows
        const int k = wave * C::EPW + kk;
        const int pos = l % C::LPR;
        const uint32_t c = *reinterpret_cast<const uint32_t*>(tab + 4 * kk);
        return (MODE & 1) ? reinterpret_cast<const unsigned char*>(g_ring_zero_row + 4 * pos)
                          : reinterpret_cast<const unsigned char*>(x) + static_cast<uint64_t>(c) * ldxb +
                                16u * static_cast<uint32_t>(pos ^ (k & 7));
    };
    auto ext_dma = [&](int64_t s, int i, const unsigned char* src) {
        rdma(src, rlds(lds + C::OFF_EXT + (C::E2 && (s & 1) ? C::EXT_BYTES : 0) +
                       (wave * C::EPW + i * C::RPP) * C::ROWB));
    };
    auto dma_ext = [&](int64_t s) {
        const unsigned char* es[C::NPE];
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) es[i] = ext_src(s, i);   // (the list reads first)
#pragma unroll
        for (int i = 0; i < C::NPE; ++i) ext_dma(s, i, es[i]);
    };

    // ------------------------------------------------------------ prologue
    for (int i = tid; i < C::ROWB / 4; i += C::NT) reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
    const int rr = lane & 15, gg = lane >> 4;
    // the transform's wave grid: CPW 16-column blocks x IBW 16-row blocks per
    // wave (CPW = 2: every A fragment read from LDS feeds both column blocks)
    constexpr int CPW = ((MODE & 64) || H / 16 > C::NW) ? 2 : 1;
    constexpr int WN = H / (16 * CPW), WM = C::NW / WN, IBW = (C::BM / 16) / WM;
    static_assert(WN * WM == C::NW && IBW * WM * 16 == C::BM, "ring transform grid");
    const int wn = wave % WN, wm = wave / WN;
    const int n0 = 16 * CPW * wn;                 // column block cb: n0 + 16 cb
    f16x8r wh[CPW][C::KC], wl[CPW][C::KC];
    int qw[CPW];
#pragma unroll
    for (int cb = 0; cb < CPW; ++cb) {
        qw[cb] = 0;
        if constexpr (AGG) continue;
        float wv[C::KC][8];
        uint32_t m = 0;
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc) {
            const float* p = W + (int64_t)(n0 + 16 * cb + rr) * H + 32 * kc + 8 * gg;
            const float4 a = ld4(p), b = ld4(p + 4);
            float* w8 = wv[kc];
            w8[0] = a.x; w8[1] = a.y; w8[2] = a.z; w8[3] = a.w;
            w8[4] = b.x; w8[5] = b.y; w8[6] = b.z; w8[7] = b.w;
#pragma unroll
            for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(fabsf(w8[j])));
        }
        qw[cb] = rsplit_exp(rwave_max(m));    // one exponent per 16-column block
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float s = ldexpf(wv[kc][j], qw[cb]);
                const _Float16 h = static_cast<_Float16>(s);
                wh[cb][kc][j] = h;
                wl[cb][kc][j] = static_cast<_Float16>(s - static_cast<float>(h));
            }
    }
    if (!AGG && wm == 0 && lane < 16 * CPW) {
        const int n = n0 + lane;
        EPI[n] = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
        EPI[H + n] = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
        EPI[2 * H + n] = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
    }
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;

    if constexpr (C::X1) {
        dma_tile(0);                  // records and rows of step 0
        dma_tab(1);
        rbar<rvm_l(0)>();             // (all waves), zero row, EPI
        dma_ext(0);
    } else if constexpr (C::E2) {
        dma_tab(0);
        dma_tile(0);                  // records of step 1, rows of step 0
        dma_tile(1);                  // records of step 2, rows of step 1
        rbar<rvm_l(0)>();             // (all waves), zero row, EPI
        dma_ext(0);
    } else {
        dma_tile(0);
        rbar<rvm_l(0)>();             // step 0's records and rows (all waves), zero row, EPI
        dma_ext(0);
        dma_tile(1);
    }

    unsigned char* const REC = lds + C::OFF_TAB;      // + slot * TAB_BYTES + wave * RECW
    for (int64_t s = 0; s < nsteps; ++s) {
        const int64_t tile = tile_of(s);
        if (tile >= ntiles) break;                    // uniform over the workgroup
        const int64_t t0 = row_begin + tile * C::BM;
        const int64_t rem = row_end - t0;
        const uint32_t nloc = static_cast<uint32_t>(rem < C::BM ? rem : C::BM);
        const int par = static_cast<int>(s & 1);
        const unsigned char* const X = lds + (par ? C::OFF_X1 : C::OFF_X0);
        const unsigned char* const RW = REC + tslot(s) * C::TAB_BYTES + wave * C::RECW;   // my 8 records
        rtr.stamp(0);
        // (B0) this step's ext rows landed in every wave (and, older, its own
        //      rows and records): younger ops = the next tile's ring DMA and
        //      the last tile's row stores
        // (E2: older than these ext rows are the records of step s + 1 too;
        //  X1: this step's own rows were issued after them: only the last
        //  tile's stores may fly)
        if (s == 0) rbar<rvm_l((C::E2 || C::X1) ? 0 : C::NDMA)>();
        else rbar<rvm_l(C::X1 ? C::NST : C::NDMA + C::NST)>();
        if constexpr (C::E2) dma_ext(s + 1);     // into the ext area step s - 1 used
        rtr.flush(wave, lane, s - 1);
        rtr.stamp(1);
        const uint32_t summ = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(
            *reinterpret_cast<const int*>(RW + 512 + 4 * C::EPW)));
        const int maxdeg = static_cast<int>(summ & 0xffu);
        const bool far = ((summ >> 8) & 1u) != 0u;
        const bool slow = (summ >> 16) != 0u;
        // row-per-wave sum of local row 8 wave + q (lane: VPL consecutive
        // columns), CSR order: the path of waves holding a hub row
        auto slow_row = [&](int q, float (&a)[C::VPL]) {
            const int loff = lane * (4 * C::VPL);
            const int64_t row = t0 + 8 * wave + q;
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
                        ldv<C::VPL>(reinterpret_cast<const float*>(X + (off * C::ROWB + (static_cast<uint32_t>(loff) ^ ((off & 7u) << 4)))), vv);
                    else
                        ldv<C::VPL>(reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(x + (int64_t)c * ldx) + loff), vv);
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k) a[k] = fmaf(w, vv[k], a[k]);
                }
            }
        };

        // (1) aggregate my 8 rows in CSR order
        f32x4 acc[C::NQ][C::CH];
#pragma unroll
        for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
            for (int j = 0; j < C::CH; ++j) acc[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!slow && !far) {
#pragma unroll 1
            for (int u0 = 0; u0 < ((MODE & 2) ? 0 : maxdeg); u0 += C::UB) {
                uint4 rcd[C::NQ][C::UB / 2];
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int b = 0; b < C::UB / 2; ++b)
                        rcd[qd][b] = *reinterpret_cast<const uint4*>(RW + (4 * qd + gq) * kRec + 8 * u0 + 16 * b);
                f32x4 vv[C::NQ][C::UB][C::CH];
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int uu = 0; uu < C::UB; ++uu) {
                        const uint4 rc = rcd[qd][uu / 2];
                        const uint32_t a = ((uu & 1) ? rc.z : rc.x) ^ coff0;
#pragma unroll
                        for (int j = 0; j < C::CH; ++j) vv[qd][uu][j] = *reinterpret_cast<const f32x4*>(lds + a + 256 * j);
                    }
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int uu = 0; uu < C::UB; ++uu) {
                        const uint4 rc = rcd[qd][uu / 2];
                        const float w = __uint_as_float((uu & 1) ? rc.w : rc.y);
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
#pragma unroll
                            for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, vv[qd][uu][j][r], acc[qd][j][r]);
                    }
            }
        } else if (!slow) {
            // far entries (past the ext capacity): gathered from memory, synchronous
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd) {
                const unsigned char* rec = RW + (4 * qd + gq) * kRec;
#pragma unroll 1
                for (int u = 0; u < maxdeg; ++u) {
                    const uint2 pw = *reinterpret_cast<const uint2*>(rec + 8 * u);
                    const float w = __uint_as_float(pw.y);
                    f32x4 vv[C::CH];
                    if (pw.x & kFar) {
                        const unsigned char* rowp = reinterpret_cast<const unsigned char*>(
                            x + static_cast<int64_t>(pw.x & ~kFar) * ldx) + coff0;
#pragma unroll
                        for (int j = 0; j < C::CH; ++j) vv[j] = *reinterpret_cast<const f32x4*>(rowp + 256 * j);
                    } else {
#pragma unroll
                        for (int j = 0; j < C::CH; ++j) vv[j] = *reinterpret_cast<const f32x4*>(lds + (pw.x ^ coff0) + 256 * j);
                    }
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, vv[j][r], acc[qd][j][r]);
                }
            }
        }
        rtr.stamp(2);
        if constexpr (AGG) {
            // aggregate only: the fp32 sums are the output.  Slow waves sum
            // row by row and come back to the lane layout through their own
            // rows of the (unused) A image
            if (slow) {
                unsigned char* const stg = lds + C::OFF_AH + 8 * wave * C::ROWB;
#pragma unroll 1
                for (int q = 0; q < 8; ++q) {
                    float a[C::VPL];
                    slow_row(q, a);
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k)
                        reinterpret_cast<float*>(stg + q * C::ROWB)[C::VPL * lane + k] = a[k];
                }
#pragma unroll
                for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
                        acc[qd][j] = *reinterpret_cast<const f32x4*>(stg + (4 * qd + gq) * C::ROWB + 16 * (c0 + 16 * j));
            }
            // (B1) every wave done with this step's rows
            rbar<kRLgkm0>();
            if constexpr (!C::E2) {
                if (s == 0) rwait<rvm(C::NPX)>();
                else rwait<rvm(C::NPX + C::NST)>();
                dma_ext(s + 1);
            }
#pragma unroll
            for (int q = 0; q <= C::NPX; ++q) ring_piece(s, q);
            static_assert(C::NQ * C::CH == C::NST, "aggregate stores keep the per-step store count");
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd)
#pragma unroll
                for (int j = 0; j < C::CH; ++j) {
                    const int lrow = 8 * wave + 4 * qd + gq;
                    if (t0 + lrow < row_end)
                        __builtin_nontemporal_store(acc[qd][j], reinterpret_cast<f32x4*>(out + (t0 + lrow) * ldo + 4 * (c0 + 16 * j)));
                }
            continue;
        }
        // (2) split into the A image (or the row-per-wave path for slow waves)
        if (!slow) {
#pragma unroll
            for (int qd = 0; qd < C::NQ; ++qd) {
                uint32_t m = 0;
#pragma unroll
                for (int j = 0; j < C::CH; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) m = max(m, __float_as_uint(fabsf(acc[qd][j][r])));
                m = rrow_max(m);
                const int p = rsplit_exp(m);
                const float sc = __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
                const int lrow = 8 * wave + 4 * qd + gq;
#pragma unroll
                for (int j = 0; j < C::CH; ++j) {
                    f16x4r h, l;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float sv = acc[qd][j][r] * sc;
                        const _Float16 hh = static_cast<_Float16>(sv);
                        h[r] = hh;
                        l[r] = static_cast<_Float16>(sv - static_cast<float>(hh));
                    }
                    const int hc = 4 * (c0 + 16 * j);
                    *reinterpret_cast<f16x4r*>(&AH[lrow * C::AS + hc]) = h;
                    *reinterpret_cast<f16x4r*>(&AL[lrow * C::AS + hc]) = l;
                }
                if (iq == 0) REXP[lrow] = p;
            }
        } else {
#pragma unroll 1
            for (int q = 0; q < 8; ++q) {
                float a[C::VPL];
                slow_row(q, a);
                uint32_t m = __float_as_uint(fabsf(a[0]));
                if constexpr (C::VPL == 2) m = max(m, __float_as_uint(fabsf(a[1])));
                const int p = rsplit_exp(rwave_max(m));
                const int lrow = 8 * wave + q;
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
        // residual + bias of my output block (rows of my row group, my 16
        // columns), before the ring slot is refilled
        f32x4 seed[CPW][IBW];
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb) {
            const int nb = n0 + 16 * cb;
            const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[nb + 4 * gg]);
#pragma unroll
            for (int ib = 0; ib < IBW; ++ib) {
                const int lr = (wm * IBW + ib) * 16 + rr;
                float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
                if (has_res) {
                    const int ch = (nb >> 2) + gg;
                    rv = *reinterpret_cast<const float4*>(X + lr * C::ROWB + ((ch ^ (lr & 7)) << 4));
                }
                seed[cb][ib] = f32x4{rv.x + bo[0], rv.y + bo[1], rv.z + bo[2], rv.w + bo[3]};
            }
        }
        // (B1) A image complete; this step's own rows, records and ext rows read
        rbar<kRLgkm0>();
        rtr.stamp(3);
        // next step's ext rows (its records landed: younger than them = its
        // own rows and the last tile's stores), then step s+2's ring DMA into
        // the slot just freed
        if constexpr (!C::E2) {
            if (s == 0) rwait<rvm(C::NPX)>();
            else rwait<rvm(C::NPX + C::NST)>();
        }
        // (their NPE + NDMA pieces -- E2: the NDMA -- are issued between the
        // MFMAs below)
        rtr.stamp(4);
        // (3) transform: 16 output columns x my row blocks
        int pr[IBW];
        f32x4 accm[CPW][IBW];
#pragma unroll
        for (int ib = 0; ib < IBW; ++ib) {
            pr[ib] = REXP[(wm * IBW + ib) * 16 + rr];
#pragma unroll
            for (int cb = 0; cb < CPW; ++cb)
#pragma unroll
                for (int r = 0; r < 4; ++r) accm[cb][ib][r] = ldexpf(seed[cb][ib][r], pr[ib] + qw[cb]);
        }
        {
            int fb = (wm * IBW * 16 + rr) * C::AS + 8 * gg;
            asm volatile("" : "+v"(fb));
            const _Float16* const AHb = AH + fb;
            const _Float16* const ALb = AL + fb;
            auto frag = [&](int t, f16x8r& bh, f16x8r& bl) {
                const int kc = t / IBW, ib = t % IBW;
                bh = *reinterpret_cast<const f16x8r*>(&AHb[ib * 16 * C::AS + 32 * kc]);
                bl = *reinterpret_cast<const f16x8r*>(&ALb[ib * 16 * C::AS + 32 * kc]);
            };
            // the next step's ext sources, all list reads before the loop (a
            // list read per piece inside it would wait on the fragment reads)
            constexpr int NPE1 = C::E2 ? 0 : C::NPE;
            const unsigned char* es[NPE1 > 0 ? NPE1 : 1];
#pragma unroll
            for (int i = 0; i < NPE1; ++i) es[i] = ext_src(s + 1, i);
            __builtin_amdgcn_sched_barrier(0);
            // A fragments PD steps ahead (a ring of PD + 1): a read issued one
            // step ahead waited its LDS latency behind a single MFMA
            constexpr int PD = 1, NF = PD + 1, NTT = C::KC * IBW;
            f16x8r fh[NF], fl[NF];
#pragma unroll
            for (int t = 0; t < PD && t < NTT; ++t) frag(t, fh[t], fl[t]);
            // one DMA piece per MFMA step: step s+1's ext rows, then step
            // s+2's ring DMA (the rest after the loop)
            auto dma_piece = [&](int t) {
                if (t < NPE1) ext_dma(s + 1, t, es[t]);
                else ring_piece(s, t - NPE1);
            };
            constexpr int NPC = NPE1 + C::NDMA;
#pragma unroll
            for (int t = 0; t < C::KC * IBW; ++t) {
                const int kc = t / IBW, ib = t % IBW;
                if (t < NPC) dma_piece(t);
                if (MODE & 4) continue;
                if (t + PD < NTT) frag(t + PD, fh[(t + PD) % NF], fl[(t + PD) % NF]);
#pragma unroll
                for (int cb = 0; cb < CPW; ++cb) {
                    accm[cb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cb][kc], fh[t % NF], accm[cb][ib], 0, 0, 0);
                    accm[cb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[cb][kc], fl[t % NF], accm[cb][ib], 0, 0, 0);
                    accm[cb][ib] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[cb][kc], fh[t % NF], accm[cb][ib], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int t = C::KC * IBW; t < NPC; ++t) dma_piece(t);
        }
        rtr.stamp(5);
        if constexpr ((MODE & 16) != 0) {
            // epilogue straight from the accumulators: lane (rr, gg) holds
            // row lr's columns n0 + 4 gg .. + 3 -- one 16-B store per row block
            // (16 rows x 64 B per instruction; no staging, no barrier)
            static_assert(C::NST == CPW * IBW, "direct stores keep the per-step store count");
#pragma unroll
            for (int cb = 0; cb < CPW; ++cb) {
                const int nb = n0 + 16 * cb;
                const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + nb + 4 * gg]);
                const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + nb + 4 * gg]);
#pragma unroll
                for (int ib = 0; ib < IBW; ++ib) {
                    f32x4 o;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = ldexpf(accm[cb][ib][r], -(pr[ib] + qw[cb]));
                        if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                        if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                        o[r] = v;
                    }
                    const int lr = (wm * IBW + ib) * 16 + rr;
                    if (t0 + lr < row_end)
                        __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + (t0 + lr) * ldo + nb + 4 * gg));
                }
            }
            rtr.stamp(6);
            rtr.stamp(7);
            continue;
        }
        // (B2) every wave done with the A image: stage there
        rbar<kRLgkm0>();
#pragma unroll
        for (int cb = 0; cb < CPW; ++cb) {
            const int nb = n0 + 16 * cb;
            const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + nb + 4 * gg]);
            const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + nb + 4 * gg]);
#pragma unroll
            for (int ib = 0; ib < IBW; ++ib) {
                float o[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = ldexpf(accm[cb][ib][r], -(pr[ib] + qw[cb]));
                    if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                    if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                    o[r] = v;
                }
                const int lr = (wm * IBW + ib) * 16 + rr;
                const int ch = (nb >> 2) + gg;
                *reinterpret_cast<f32x4*>(lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4)) =
                    f32x4{o[0], o[1], o[2], o[3]};
            }
        }
        rtr.stamp(6);
        // (B3) staged: my 8 rows out, whole rows
        rbar<kRLgkm0>();
        {
            const int ch = lane % C::LPRW;
            f32x4 v[C::NST];
#pragma unroll
            for (int i = 0; i < C::NST; ++i) {
                const int lr = 8 * wave + i * C::RPI + lane / C::LPRW;
                v[i] = *reinterpret_cast<const f32x4*>(lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4));
            }
#pragma unroll
            for (int i = 0; i < C::NST; ++i) {
                const int lr = 8 * wave + i * C::RPI + lane / C::LPRW;
                if (t0 + lr < row_end)
                    __builtin_nontemporal_store(v[i], reinterpret_cast<f32x4*>(out + (t0 + lr) * ldo + 4 * ch));
            }
        }
        rtr.stamp(7);
    }
    rwait<rvm(0)>();   // no LDS-DMA may outlive the workgroup
    rtr.flush(wave, lane, nsteps - 1);
}

template <int H, int MODE, int EPIF>
void launch_ring_k(int G, hipStream_t st, const void* plan, const int32_t* row_ptr,
                   const int32_t* col, const float* ew, const float* x, int64_t ldx, int64_t rb,
                   int64_t re, const float* w, const float* bias, const float* scale,
                   const float* shift, int flags, float* out, int64_t ldo) {
    hipLaunchKernelGGL((gcn_ring_kernel<H, MODE, EPIF>), dim3(G), dim3(RCfg<H>::NT), 0, st,
                       static_cast<const unsigned char*>(plan), row_ptr, col, ew, x, ldx, rb, re, w,
                       bias, scale, shift, flags, out, ldo);
}

template <int H, int MODE>
void launch_ring_h(int G, hipStream_t st, const void* plan, const int32_t* row_ptr,
                   const int32_t* col, const float* ew, const float* x, int64_t ldx, int64_t rb,
                   int64_t re, const float* w, const float* bias, const float* scale,
                   const float* shift, int flags, float* out, int64_t ldo) {
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    if (MODE == 0 && flags == kBN)
        launch_ring_k<H, MODE, kBN>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    else if (MODE == 0 && flags == kNoBN)
        launch_ring_k<H, MODE, kNoBN>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    else
        launch_ring_k<H, MODE, -1>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
}

template <int MODE = 0>
int launch_ring(int h, const void* plan, const int32_t* row_ptr, const int32_t* col,
                const float* ew, const float* x, int64_t ldx, int64_t rb, int64_t re,
                const float* w, const float* bias, const float* scale, const float* shift,
                int flags, float* out, int64_t ldo, hipStream_t st) {
    const int bm = h == 128 ? RCfg<128>::BM : RCfg<64>::BM;
    const int64_t ntiles = (re - rb + bm - 1) / bm;
    const int G = ring_grid(ntiles, h == 128 ? RCfg<128>::WGPC : RCfg<64>::WGPC);
    MIGNN_REQUIRE(G > 0, "gcn_ring: device query failed");
    if (h == 128)
        launch_ring_h<128, MODE>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    else
        launch_ring_h<64, MODE>(G, st, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    return launch_status("gcn_ring_kernel");
}

}  // namespace

int ring_device_errors(unsigned int* out, int clear) {
    unsigned int v = 0u;
    MIGNN_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ring_errors), sizeof(unsigned int), 0,
                                  hipMemcpyDeviceToHost));
    *out |= v;
    if (clear) {
        const unsigned int zero = 0u;
        MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ring_errors), &zero, sizeof(unsigned int), 0,
                                    hipMemcpyHostToDevice));
    }
    return MIGNN_OK;
}

}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_gcn_ring_plan_bytes(int64_t row_begin, int64_t row_end, int h) {
    if (row_end <= row_begin || (h != 64 && h != 128)) return 0;
    const int bm = h == 128 ? RCfg<128>::BM : RCfg<64>::BM;
    const int64_t ntiles = (row_end - row_begin + bm - 1) / bm;
    return kRHdr + static_cast<size_t>(ntiles) * (h == 128 ? RCfg<128>::TAB_BYTES : RCfg<64>::TAB_BYTES);
}

extern "C" int mignn_gcn_ring_plan(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                   int64_t rb, int64_t re, int h, void* plan, size_t plan_bytes,
                                   unsigned long long* stats, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && plan, "gcn_ring_plan: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_ring_plan: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_ring_plan: bad row range");
    MIGNN_REQUIRE(aligned16(plan), "gcn_ring_plan: unaligned plan");
    if (re == rb) return MIGNN_OK;
    MIGNN_REQUIRE(plan_bytes >= mignn_gcn_ring_plan_bytes(rb, re, h),
                  "gcn_ring_plan: plan buffer too small");
    const int bm = h == 128 ? RCfg<128>::BM : RCfg<64>::BM;
    const int64_t ntiles = (re - rb + bm - 1) / bm;
    const int G = ring_grid(ntiles, h == 128 ? RCfg<128>::WGPC : RCfg<64>::WGPC);
    MIGNN_REQUIRE(G > 0, "gcn_ring_plan: device query failed");
    const unsigned grid = static_cast<unsigned>(ntiles < (1 << 20) ? ntiles : (1 << 20));
    if (h == 128)
        hipLaunchKernelGGL(ring_plan_kernel<128>, dim3(grid), dim3(RCfg<128>::BM), 0, as_stream(stream), row_ptr,
                           col, ew, rb, re, ntiles, G, static_cast<unsigned char*>(plan), stats);
    else
        hipLaunchKernelGGL(ring_plan_kernel<64>, dim3(grid), dim3(RCfg<64>::BM), 0, as_stream(stream), row_ptr,
                           col, ew, rb, re, ntiles, G, static_cast<unsigned char*>(plan), stats);
    return launch_status("ring_plan_kernel");
}

extern "C" int mignn_gcn_layer_ring(const void* plan, const int32_t* row_ptr, const int32_t* col,
                                    const float* ew, const float* x, int64_t ldx, int64_t rb,
                                    int64_t re, int h, const float* w, const float* bias,
                                    const float* scale, const float* shift, int flags, float* out,
                                    int64_t ldo, void* stream) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && x && w && out, "gcn_layer_ring: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_layer_ring: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(plan) && aligned16(w),
                  "gcn_layer_ring: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "gcn_layer_ring: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_ring: bad row range");
    MIGNN_REQUIRE(x != out, "gcn_layer_ring: in-place not supported (neighbours read x)");
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_ring: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_ring: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_ring: affine");
    if (re == rb) return MIGNN_OK;
    return launch_ring(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out,
                       ldo, as_stream(stream));
}

extern "C" int mignn_gcn_aggregate_ring(const void* plan, const int32_t* row_ptr,
                                        const int32_t* col, const float* ew, const float* x,
                                        int64_t ldx, int64_t rb, int64_t re, int h, float* out,
                                        int64_t ldo, void* stream) {
    MIGNN_REQUIRE(plan && row_ptr && col && ew && x && out, "gcn_aggregate_ring: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_aggregate_ring: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(plan), "gcn_aggregate_ring: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h,
                  "gcn_aggregate_ring: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_aggregate_ring: bad row range");
    MIGNN_REQUIRE(x != out, "gcn_aggregate_ring: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    return launch_ring<32>(h, plan, row_ptr, col, ew, x, ldx, rb, re, nullptr, nullptr, nullptr,
                           nullptr, 0, out, ldo, as_stream(stream));
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_ring_trace(void* buf) {
    MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ring_trace), &buf, sizeof(buf)));
    return MIGNN_OK;
}
#endif

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_ring(int mode, const void* plan, const int32_t* row_ptr,
                               const int32_t* col, const float* ew, const float* x, int64_t ldx,
                               int64_t rb, int64_t re, int h, const float* w, const float* bias,
                               const float* scale, const float* shift, int flags, float* out,
                               int64_t ldo, void* stream) {
    hipStream_t st = as_stream(stream);
    switch (mode) {
#define MIGNN_RING_MODE(M) \
    case M: return launch_ring<M>(h, plan, row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, flags, out, ldo, st);
        MIGNN_RING_MODE(0) MIGNN_RING_MODE(1) MIGNN_RING_MODE(2) MIGNN_RING_MODE(3)
        MIGNN_RING_MODE(4) MIGNN_RING_MODE(6) MIGNN_RING_MODE(7) MIGNN_RING_MODE(8)
        MIGNN_RING_MODE(15) MIGNN_RING_MODE(16) MIGNN_RING_MODE(17) MIGNN_RING_MODE(18)
        MIGNN_RING_MODE(20) MIGNN_RING_MODE(64) MIGNN_RING_MODE(80)
        MIGNN_RING_MODE(32) MIGNN_RING_MODE(33) MIGNN_RING_MODE(34) MIGNN_RING_MODE(40)
#undef MIGNN_RING_MODE
        default: break;
    }
    set_error("diag_ring: unknown mode %d", mode);
    return MIGNN_ERR_ARG;
}
#endif

MIGNN_DMA_OOB_EXPORT(mignn_diag_dma_oob_ring)
