// Fused GCN layer, split-fp16 ("f16x3") MFMA variant -- the north-star hot
// kernel (GCNConv + residual + BatchNorm(eval) + ReLU, gnn_model.py:166,
// :184-191, one pass over HBM):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Why a second variant next to tile_gemm.hip's exact-fp32 kernel: on gfx950
// the f32-input MFMA runs at the f32 VECTOR rate (157 TF), so at H = 128 the
// node transform alone needs >= 2.2 ms per 10M-node layer -- more than the
// layer's HBM time.  Here every fp32 operand is split into two fp16 halves,
//     a = 2^-p (a_hi + a_lo),   a_hi = fp16(2^p a),   a_lo = fp16(2^p a - a_hi),
// with a power-of-two scale 2^p per A row and per consumer wave's W columns
// (max |.| lands in [2^13, 2^14): no fp16 overflow; elements below ~2^-24 of
// their block's max lose relative, not absolute, precision), and
//     a.w = 2^-(p+q) [ a_hi w_hi + a_hi w_lo + a_lo w_hi ] + O(2^-22 |a w|)
// is formed by three v_mfma_f32_16x16x32_f16 into ONE fp32 accumulator (the
// fp16 products are exact in fp32): 16x the f32 MFMA rate, so the transform
// drops well below the HBM time.  Relative error per product ~2^-22 (fp32:
// 2^-24); the measured field error stays far inside the north star's 1e-5
// (tests/test_gpu_parity.py).
//
// Structure: one 12-wave workgroup per CU, persistent over 64-row tiles,
// XCD-aware tile order (as tile_gemm.hip), one barrier per tile step.
//   * Own-row image (2 buffers): a tile's rows x[t0, t0+64) are copied
//     HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) issued by the consumer
//     waves one step ahead, unpadded, 16-B chunks XOR-swizzled by (row & 7)
//     on the SOURCE address.  In the locality order (mignn_locality_order:
//     4x4x4-cell blocks, one per 64-row tile, in panels of 4x4 block columns)
//     ~75 % of a mesh's CSR entries point inside their tile.
//   * 8 producer waves, 8 rows each (two quads of 4 rows; a row = 16 lanes x
//     32 B).  Per tile, vectorised over the wave's CSR entries (lane = entry),
//     two lookup tables are built in LDS: in-tile entries -> {image address,
//     w}, out-of-tile entries -> {column, w}.  Out-of-tile rows are gathered
//     into registers (EX slots per row) one whole step before they are summed
//     (branch-free: empty slots read a zero row); in-tile entries are read
//     from the own-row image.  Sum order of a row: its out-of-tile entries
//     (CSR order), then its in-tile entries (CSR order) -- deterministic.  The
//     finished row is scaled, split and written to the A image (fp16 hi / lo)
//     with its exponent.
//   * 4 consumer waves (one per SIMD), 32 output columns each, split W held in
//     registers for the whole launch.  (residual + bias) * 2^(p_row + q_w)
//     seeds the accumulator, 3 MFMAs per 16x16x32 block, epilogue (unscale,
//     BN affine, ReLU) from the accumulators into an LDS staging tile, then
//     whole rows out: a half-wave stores
//     one 512-B row (H = 128) -- the accumulator layout would store 16 rows x
//     64 B per instruction, measured 1.5x slower as a plain copy
//     (profiles/r02_kbench_store_patterns.json) and 2 % (H = 128) / 9 %
//     (H = 64) slower in this kernel.
//   * Hand-offs (LDS counters, relaxed: a wave's LDS operations execute in
//     order): consumers bump cntX once they hold their residual -- then the
//     own-row buffer takes the tile two steps on; they bump cntA once their
//     MFMAs have read the (single) A image -- then producers may write the
//     next tile's rows into it; cntS once their blocks are staged.  Every
//     spin is bounded: one that runs out sets the device error word
//     (mignn_device_errors) instead of falling through silently.
#include <type_traits>

#include "common.hpp"

namespace mignn {
MIGNN_DMA_OOB_WORD
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f16x4 = __attribute__((ext_vector_type(4))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// two own-row image buffers (the own rows DMA'd one step ahead) and an output
// staging tile: the consumers write their accumulator blocks there and store
// whole rows (512 B per half-wave at H = 128) instead of 16 rows x 64 B per
// instruction
// NC: consumer waves -- 4 (one per SIMD, 32 output columns each) or 8 (two
// per SIMD, 16 columns each: half the per-wave MFMA / epilogue chain, the two
// waves of a SIMD overlap; 16 waves per CU, <= 128 VGPRs)
template <int H, int NC = 4>
struct SCfg {
    static_assert(H == 64 || H == 128, "f16x3 GCN layer: H in {64, 128}");
    static_assert(NC == 4 || NC == 8, "consumer waves");
    static constexpr int BM = 64;                  // rows per tile
    static constexpr int NPW = 8;                  // producer waves
    static constexpr int NCW = NC;                 // consumer waves
    static constexpr int NT = (NPW + NCW) * 64;
    static constexpr int PROWS = BM / NPW;         // rows per producer wave (8)
    static constexpr int NQD = PROWS / 4;          // row quads per producer wave
    static constexpr int F = H / 16;               // floats per lane of a row (16 lanes / row)
    static constexpr int CH = F / 4;               // 16-B chunks per lane of a row
    static constexpr int EX = H == 128 ? (NC == 8 ? 3 : 4) : 6;   // out-of-tile register slots per row
    static constexpr int UB = H == 128 ? 2 : 4;    // in-tile slots per LDS batch (H = 128: 4
                                                   // spills at 3 waves / SIMD, 8 % slower;
                                                   // H = 64: 4 is 7 % faster than 2)
    static constexpr int LTS = 12;                 // in-tile table slots per row
    static constexpr int ETS = 6;                  // out-of-tile table slots per row (even)
    static constexpr int TAB_BYTES = PROWS * (LTS + ETS) * 8;
    static constexpr int VPL = H / 64;             // floats per lane, row-per-wave slow path
    static constexpr int ROWB = H * 4;             // bytes per own-image row (unpadded)
    static constexpr int AS = 144;                 // A row stride, halfs (72 words = 8 mod 64)
    static constexpr int JB = NC == 8 ? 1 : 2;     // 16-column blocks per consumer
    static constexpr int WN = H / 16 / JB;         // consumer column groups
    static constexpr int WM = NCW / WN;            // consumer row groups
    static constexpr int IB = BM / 16 / WM;        // 16-row blocks per consumer
    static constexpr int NST = IB * JB;            // row stores per consumer per tile
    static constexpr int KC = H / 32;              // 32-deep k chunks
    static constexpr int RPP = 1024 / ROWB;        // rows per 1-KB DMA piece
    static constexpr int LPR = 64 / RPP;           // lanes per row in a piece
    static constexpr int NPIECE = BM / RPP;        // pieces per tile
    static constexpr int NPC = NPIECE / NCW;       // DMA pieces per consumer per tile
    static constexpr int XBUF = 2;                 // own-row image buffers
    static constexpr int X_BYTES = BM * ROWB;
    static constexpr int A_BYTES = BM * AS * 2;
    // Xs[2] | zero row | Ah | Al | rexp[BM] | tables[2][NPW] | epi | counters |
    // staging tile (own-image rows and the zero row sit at ROWB multiples: an
    // image address is P ^ chunk offset, see the producer)
    static constexpr int OFF_ZERO = XBUF * X_BYTES;
    static constexpr int OFF_AH = OFF_ZERO + ROWB;
    static constexpr int OFF_AL = OFF_AH + A_BYTES;
    static constexpr int OFF_REXP = OFF_AL + A_BYTES;
    static constexpr int OFF_TAB = OFF_REXP + BM * 4;
    static constexpr int OFF_EPI = OFF_TAB + 2 * NPW * TAB_BYTES;   // bias | scale | shift [H]
    static constexpr int OFF_CNT = OFF_EPI + 3 * H * 4;             // cntX, cntA, cntS
    static constexpr int OFF_STG = OFF_CNT + 16;                     // [BM][ROWB]
    static constexpr int LDS_BYTES = OFF_STG + BM * ROWB;
    static constexpr int NSTG = BM * ROWB / 1024 / NCW;             // row stores per consumer
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
    static_assert(NPIECE % NCW == 0, "DMA pieces per consumer");
    static_assert(NQD == 2, "two row quads per producer wave");
    static_assert(PROWS * LTS % 2 == 0 && PROWS * LTS / 2 <= 64 && PROWS * ETS <= 64, "tables");
};

// power-of-two scale exponent for a block whose max |value| has f32 bits m:
// max * 2^p lands in [2^13, 2^14) (p = 140 - biased exponent), capped at 2^50
// so that a seed (residual + bias) * 2^(p_row + q_w) cannot overflow for
// |residual + bias| < 2^27 (blocks below 2^-36 keep fp16-normal hi parts down
// to 2^-64 of their max: absolute error stays negligible)
__device__ __forceinline__ int scale_exp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}

__device__ __forceinline__ void split16(float a, int p, _Float16& hi, _Float16& lo) {
    const float s = ldexpf(a, p);
    hi = static_cast<_Float16>(s);
    lo = static_cast<_Float16>(s - static_cast<float>(hi));
}

// max over the 64 lanes of a wave (uint bits of non-negative floats; NaN / inf
// order above every finite value); result wave-uniform
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    int t = static_cast<int>(v);
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x124, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x128, 0xf, 0xf, false)));
    const uint32_t a = static_cast<uint32_t>(__builtin_amdgcn_readlane(t, 0));
    const uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_readlane(t, 16));
    const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(t, 32));
    const uint32_t d = static_cast<uint32_t>(__builtin_amdgcn_readlane(t, 48));
    return max(max(a, b), max(c, d));
}

// max over each DPP row of 16 lanes (the lanes of one row in the producer's
// quad layout); every lane of the row gets it
__device__ __forceinline__ uint32_t row_max_u32(uint32_t v) {
    int t = static_cast<int>(v);
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x124, 0xf, 0xf, false)));
    t = max(static_cast<uint32_t>(t),
            static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x128, 0xf, 0xf, false)));
    return static_cast<uint32_t>(t);
}

__device__ __forceinline__ f32x4 mfma16x16x32h(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// 32-bit LDS address of a pointer into the kernel's LDS array
__device__ __forceinline__ uint32_t lds_addr(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(p)));
}

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4) to the wave-uniform LDS
// address `dst` (+16 x lane).  Inline asm on purpose: the compiler neither
// counts it nor inserts conservative vmcnt(0) waits before later LDS reads;
// the issuing wave waits for it itself (block_barrier with a counted vmcnt).
__device__ __forceinline__ void glds16(const void* src, uint32_t dst) {
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

// s_waitcnt <imm> + s_barrier through builtins (the compiler's waitcnt pass
// sees the wait); empty asm statements keep memory operations from moving
// across.  Encodings: vmcnt(n) lgkmcnt(0) = 0x70 | n (n < 16); lgkmcnt(0)
// alone = 0xC07F.
template <int WAITCNT>
__device__ __forceinline__ void block_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(WAITCNT);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

}  // namespace

// the device error word (mignn_device_errors)
__device__ unsigned int g_device_errors = 0u;

namespace {

__device__ __forceinline__ void device_error(unsigned int code) {
    __hip_atomic_fetch_or(&g_device_errors, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// relaxed LDS counter: bump / bounded spin until >= target.  A spin that runs
// out (2^22 polls, ~0.1 s: a hand-off that never came) records
// MIGNN_DEVERR_SPIN in the device error word -- the launch still drains (every
// wave reaches every barrier), its output is flagged wrong by
// mignn_device_errors() instead of passing silently
__device__ __forceinline__ void lds_bump(int* c) {
    asm volatile("" ::: "memory");
    __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_wait(int* c, int target) {
    asm volatile("" ::: "memory");
    bool ok = false;
    for (int it = 0; it < (1 << 22); ++it) {
        if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
            ok = true;
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) device_error(MIGNN_DEVERR_SPIN);
    asm volatile("" ::: "memory");
}

// Diagnostic timeline (MIGNN_DIAG_TRACE, mignn_diag_set_trace_f16x3): s_memtime
// stamps of producer wave 0 (slots 0..3) and consumer wave 0 (slots 4..7) of
// workgroups 0..7, steps 0..63 -> trace[(b*64+s)*8+slot]
__device__ __forceinline__ void stamp(unsigned long long* trace, int lane, int64_t s, int slot) {
    if (trace != nullptr && blockIdx.x < 8 && s >= 0 && s < 64 && lane == 0)
        trace[(blockIdx.x * 64 + s) * 8 + slot] = __builtin_amdgcn_s_memtime();
}
#ifdef MIGNN_DIAG
unsigned long long* g_trace16_host = nullptr;   // set by mignn_diag_set_trace_f16x3
#else
constexpr unsigned long long* g_trace16_host = nullptr;
#endif

// zeros read by the empty out-of-tile slots (a valid, always-cached address)
__device__ __attribute__((aligned(16))) float g_zero_row[256];

struct PIdx {      // one producer wave's CSR indices of one tile
    int rpv;       // lanes 0..PROWS: row_ptr of the wave's rows (clamped)
    int ej;        // lane t: column of entry e0 + t
    float ew;      // lane t: GCN weight of entry e0 + t
};

template <int PROWS>
__device__ __forceinline__ int p_load_rpv(const int32_t* __restrict__ row_ptr, int64_t r0,
                                          int64_t row_end, int lane) {
    const int64_t r = r0 + lane < row_end ? r0 + lane : row_end;
    return lane <= PROWS ? row_ptr[r] : 0;
}

template <int PROWS>
__device__ __forceinline__ void p_load_entries(PIdx& t, const int32_t* __restrict__ col,
                                               const float* __restrict__ ew, int lane) {
    const int e0 = __builtin_amdgcn_readlane(t.rpv, 0);
    const int ne = __builtin_amdgcn_readlane(t.rpv, PROWS) - e0;
    t.ej = lane < ne ? col[e0 + lane] : 0;
    t.ew = lane < ne ? ew[e0 + lane] : 0.f;
}

// EPIF: the flags at compile time (the model's 15 / 11: no schedule or
// ablation bits), -1: `flags`
template <int H, int NC, int EPIF = -1>
__global__ __launch_bounds__((SCfg<H, NC>::NT)) void gcn_f16x3_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t row_begin,
    int64_t row_end, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo, unsigned long long* trace) {
    using C = SCfg<H, NC>;
    if constexpr (EPIF >= 0) flags = EPIF;
    constexpr int UBE = C::UB;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    int* const cntX = reinterpret_cast<int*>(lds + C::OFF_CNT);
    int* const cntA = cntX + 1;
    int* const cntS = cntX + 2;
    _Float16* const AH = reinterpret_cast<_Float16*>(lds + C::OFF_AH);
    _Float16* const AL = reinterpret_cast<_Float16*>(lds + C::OFF_AL);
    int* const REXP = reinterpret_cast<int*>(lds + C::OFF_REXP);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + C::BM - 1) / C::BM;
    const int G = gridDim.x;            // multiple of 8 (host guarantees)
    const int xcd = blockIdx.x & 7;
    const int slot = blockIdx.x >> 3;
    const int per_xcd = G >> 3;
    const int64_t nsteps = (ntiles + G - 1) / G;
    // XCD x walks its own contiguous range of nsteps * per_xcd tiles
    // (per_xcd per step), so in the locality order (two z-levels of a 4x4
    // block-column panel per step) a tile's lateral neighbours are read by the
    // same XCD in the same step and its z neighbours a step apart, in its L2.
    // MIGNN_SCHED_INTERLEAVED (the round-1 schedule): at step s the chip
    // covers tiles [sG, (s+1)G), XCD x a run of per_xcd of them.
    const bool chunks = (flags & MIGNN_SCHED_INTERLEAVED) == 0;
    const int64_t chunk = chunks ? nsteps * per_xcd : per_xcd;
    const int64_t sstride = chunks ? per_xcd : G;
    auto tile_of = [&](int64_t s) -> int64_t { return (int64_t)xcd * chunk + s * sstride + slot; };
    // own-row image buffer of a tile of this workgroup: (its step index) mod 2
    auto xbuf_of = [&](int64_t tile) -> int {
        return static_cast<int>(((tile - (int64_t)xcd * chunk) / sstride) % C::XBUF);
    };

    if (tid == 0) {
        cntX[0] = 0;
        cntA[0] = 0;
        cntS[0] = 0;
    }

    // static wave priority (diagnostic schedules): consumers or producers
    // win instruction arbitration on their SIMD
    if ((flags & MIGNN_SCHED_PRIO_CONSUMERS) && wave < C::NCW) __builtin_amdgcn_s_setprio(1);
    if ((flags & MIGNN_SCHED_PRIO_PRODUCERS) && wave >= C::NCW) __builtin_amdgcn_s_setprio(1);

    if (wave >= C::NCW) {
        // ================================================================ producer
        const int pw = wave - C::NCW;
        auto first_row = [&](int64_t tile) { return row_begin + tile * C::BM + pw * C::PROWS; };
        int lane_ = lane;
        asm volatile("" : "+v"(lane_));
        // zero row (read by the empty slots of the in-tile pass)
        for (int i = lane_ + pw * 64; i < C::ROWB / 4; i += C::NPW * 64)
            reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
        // lookup tables of tile parity tb: LT [PROWS][LTS] {P, w}, ET [PROWS][ETS] {col, w}
        auto LTb = [&](int tb) { return lds + C::OFF_TAB + (tb * C::NPW + pw) * C::TAB_BYTES; };
        auto ETb = [&](int tb) { return LTb(tb) + C::PROWS * C::LTS * 8; };

        // quad lanes: group g = lane >> 4 owns row 4 qd + g of the wave; lane
        // i = lane & 15 owns the 16-B chunks c0(i) + 16 j of the row.  c0 puts
        // bit 3 = [i in 4..11]: in every ds_read_b128 lane group the two rows'
        // lanes then hit disjoint bank halves whatever their XOR swizzles.
        const int gq = lane_ >> 4, iq = lane_ & 15;
        const int hb = (iq >= 4 && iq < 12) ? 1 : 0;
        const int c0 = (hb ? iq - 4 : (iq < 4 ? iq : iq - 8)) | (hb << 3);
        uint32_t coff[C::CH];                         // byte offset of my chunks in a row
#pragma unroll
        for (int j = 0; j < C::CH; ++j) coff[j] = static_cast<uint32_t>((c0 + 16 * j) << 4);
        // out-of-tile row c (empty slot: c = ~0u -> the zero row)
        auto xrow = [&](uint32_t c) -> const unsigned char* {
            return c != 0xffffffffu ? reinterpret_cast<const unsigned char*>(x + (int64_t)c * ldx)
                                    : reinterpret_cast<const unsigned char*>(g_zero_row);
        };
        bool a_free = false;     // this step may write the A image (consumers done reading)
        auto wait_a = [&](int64_t s) {
            if (!a_free) {
                lds_wait(cntA, C::NCW * static_cast<int>(s + 1));
                a_free = true;
            }
        };

        // ---- slow path (a wave's rows with > 64 entries, > LTS in-tile or > ETS
        // out-of-tile entries in a row): a row per wave instruction, one entry
        // at a time, indices by scalar loads -- correct, not fast
        const uint64_t xbase = reinterpret_cast<uint64_t>(x);
        const uint32_t ldxb = static_cast<uint32_t>(ldx) * 4u;
        auto slow_rows = [&](int64_t tile, int rpv, int64_t s) {
            const int64_t t0 = row_begin + tile * C::BM;
            const int64_t rem = row_end - t0;
            const uint32_t nloc = static_cast<uint32_t>(rem < C::BM ? rem : C::BM);
            const uint32_t xb = static_cast<uint32_t>(xbuf_of(tile) * C::X_BYTES);
            const int loff = lane_ * (4 * C::VPL);
#pragma unroll 1
            for (int q = 0; q < C::PROWS; ++q) {
                const int e_begin = __builtin_amdgcn_readlane(rpv, q);
                const int e_end = __builtin_amdgcn_readlane(rpv, q + 1);
                float acc[C::VPL];
#pragma unroll
                for (int k = 0; k < C::VPL; ++k) acc[k] = 0.f;
#pragma unroll 1
                for (int e = e_begin; e < e_end; ++e) {
                    const int c = __builtin_amdgcn_readfirstlane(col[e]);
                    const float we = __builtin_bit_cast(
                        float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, ew[e])));
                    const uint32_t off = static_cast<uint32_t>(c - static_cast<int>(t0));
                    float vv[C::VPL];
                    if (off < nloc) {
                        const uint32_t a = (xb + off * C::ROWB) +
                                           (static_cast<uint32_t>(loff) ^ ((off & 7u) << 4));
                        ldv<C::VPL>(reinterpret_cast<const float*>(lds + a), vv);
                    } else {
                        const i32x4 rs = buffer_rsrc(xbase + (uint64_t)static_cast<uint32_t>(c) * ldxb, H * 4);
                        if constexpr (C::VPL == 2) {
                            const f32x2 t = raw_buffer_load_f32x2(rs, loff, 0, 0);
                            vv[0] = t[0];
                            vv[1] = t[1];
                        } else {
                            vv[0] = raw_buffer_load_f32(rs, loff, 0, 0);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < C::VPL; ++k) acc[k] = fmaf(we, vv[k], acc[k]);
                }
                // scale, split, store (a row per wave: lane owns VPL floats)
                uint32_t m = __float_as_uint(fabsf(acc[0]));
                if constexpr (C::VPL == 2) m = max(m, __float_as_uint(fabsf(acc[1])));
                const int p = scale_exp(wave_max_u32(m));
                const int lrow = pw * C::PROWS + q;
                wait_a(s);
#pragma unroll
                for (int k = 0; k < C::VPL; ++k) {
                    _Float16 h, l;
                    split16(acc[k], p, h, l);
                    AH[lrow * C::AS + C::VPL * lane_ + k] = h;
                    AL[lrow * C::AS + C::VPL * lane_ + k] = l;
                }
                if (lane_ == 0) REXP[lrow] = p;
            }
        };

        // ---- lookup tables of one tile (lane t <-> CSR entry e0 + t):
        //      in-tile entry -> LT[row][u] = {image address P, w}
        //      out-of-tile   -> ET[row][k] = {column, w}
        // returns (slow, max row degree, max out-of-tile entries per row)
        struct TInfo { int slow, maxdeg, maxext; };
        auto build_tables = [&](int64_t tile, const PIdx& ix, int tb) -> TInfo {
            unsigned char* const LT = LTb(tb);
            unsigned char* const ET = ETb(tb);
            {
                uint32_t zo = C::OFF_ZERO, zz = 0u;
                asm volatile("" : "+v"(zo), "+v"(zz));   // rematerialised per call, never spilled
                const uint4 z4 = make_uint4(zo, zz, zo, zz);
                if (lane_ < C::PROWS * C::LTS / 2) *reinterpret_cast<uint4*>(LT + 16 * lane_) = z4;
                if (lane_ < C::PROWS * C::ETS)
                    *reinterpret_cast<uint2*>(ET + 8 * lane_) = make_uint2(~zz, zz);
            }
            if (tile >= ntiles) return TInfo{0, 0, 0};
            const int64_t t0 = row_begin + tile * C::BM;
            const int64_t rem = row_end - t0;
            const uint32_t nloc = static_cast<uint32_t>(rem < C::BM ? rem : C::BM);
            const uint32_t xb = static_cast<uint32_t>(xbuf_of(tile) * C::X_BYTES);
            int rp[C::PROWS + 1];
#pragma unroll
            for (int q = 0; q <= C::PROWS; ++q) rp[q] = __builtin_amdgcn_readlane(ix.rpv, q);
            const int e0 = rp[0];
            const int ne = rp[C::PROWS] - e0;
            if (ne > 64) return TInfo{1, 0, 0};
            const int t = lane_;
            int q = 0, rs = 0;
#pragma unroll
            for (int qq = 1; qq < C::PROWS; ++qq) {
                const int b = rp[qq] - e0;
                const bool ge = t >= b;
                q += ge ? 1 : 0;
                rs = ge ? b : rs;
            }
            const int u = t - rs;
            const bool valid = t < ne;
            const uint32_t off = static_cast<uint32_t>(ix.ej - static_cast<int>(t0));
            const bool local = valid && off < nloc;
            const bool ext = valid && !local;
            const uint64_t M = __ballot(ext);
            const int mb = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(M >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(M), 0u));
            const int k = mb - __builtin_amdgcn_ds_bpermute(rs << 2, mb);
            const bool ovf = (local && u >= C::LTS) || (ext && k >= C::ETS);
            if (__ballot(ovf) != 0ull) return TInfo{1, 0, 0};
            const uint32_t wb = __builtin_bit_cast(uint32_t, ix.ew);
            if (local) {
                const uint32_t P = (xb + off * C::ROWB) | ((off & 7u) << 4);
                *reinterpret_cast<uint2*>(LT + (q * C::LTS + u) * 8) = make_uint2(P, wb);
            }
            if (ext) *reinterpret_cast<uint2*>(ET + (q * C::ETS + k) * 8) = make_uint2(static_cast<uint32_t>(ix.ej), wb);
            int maxdeg = 0;
#pragma unroll
            for (int qq = 0; qq < C::PROWS; ++qq) maxdeg = max(maxdeg, rp[qq + 1] - rp[qq]);
            const uint32_t kk = ext ? static_cast<uint32_t>(k + 1) : 0u;
            const int maxext = static_cast<int>(wave_max_u32(kk));
            return TInfo{0, maxdeg, maxext};
        };

        // ---- out-of-tile rows of a tile (tables tb) -> registers, EX per row
        using XV = f32x4[C::NQD][C::EX][C::CH];
        auto issue_ext = [&](int tb, XV& xv) {
            asm volatile("" ::: "memory");   // after the table writes
            const unsigned char* const ET = ETb(tb);
            // all columns first (one LDS round trip), then the row loads
            uint32_t cc[C::NQD][C::EX];
#pragma unroll
            for (int qd = 0; qd < C::NQD; ++qd) {
                const int row = 4 * qd + gq;
#pragma unroll
                for (int e = 0; e < C::EX; e += 2) {
                    const uint4 t = *reinterpret_cast<const uint4*>(ET + (row * C::ETS + e) * 8);
                    cc[qd][e] = t.x;
                    if (e + 1 < C::EX) cc[qd][e + 1] = t.z;
                }
            }
#pragma unroll
            for (int qd = 0; qd < C::NQD; ++qd)
#pragma unroll
                for (int e = 0; e < C::EX; ++e) {
                    // empty slot: exec-masked off (no request; a slot empty in
                    // every row of the wave is skipped whole)
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) xv[qd][e][j] = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (cc[qd][e] != 0xffffffffu) {
                        // (derived from x: a global, not flat, load -- flat loads
                        // would also count on lgkmcnt and stall every LDS wait)
                        const unsigned char* rowp = reinterpret_cast<const unsigned char*>(x) +
                                                    static_cast<uint64_t>(cc[qd][e]) * ldxb;
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
                            xv[qd][e][j] = *reinterpret_cast<const f32x4*>(rowp + coff[j]);
                    }
                }
        };
        // their weighted sum, CSR order (empty slots: zeros, w 0), + the rest
        // beyond the register slots (rare; synchronous loads)
        using ACC = f32x4[C::NQD][C::CH];
        auto sum_ext = [&](int tb, const XV& xv, const TInfo& info, ACC& acc) {
            const unsigned char* const ET = ETb(tb);
#pragma unroll
            for (int qd = 0; qd < C::NQD; ++qd) {
                const int row = 4 * qd + gq;
#pragma unroll
                for (int j = 0; j < C::CH; ++j) acc[qd][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int e = 0; e < C::EX; ++e) {
                    const float w = __builtin_bit_cast(
                        float, *reinterpret_cast<const uint32_t*>(ET + (row * C::ETS + e) * 8 + 4));
#pragma unroll
                    for (int j = 0; j < C::CH; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, xv[qd][e][j][r], acc[qd][j][r]);
                }
#pragma unroll 1
                for (int e = C::EX; e < info.maxext; ++e) {
                    const uint2 cw = *reinterpret_cast<const uint2*>(ET + (row * C::ETS + e) * 8);
                    const float w = __builtin_bit_cast(float, cw.y);
                    const unsigned char* rowp = xrow(cw.x);
#pragma unroll
                    for (int j = 0; j < C::CH; ++j) {
                        const f32x4 vv = *reinterpret_cast<const f32x4*>(rowp + coff[j]);
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, vv[r], acc[qd][j][r]);
                    }
                }
            }
        };

        // ---- in-tile entries of a tile (tables tb) on top of acc, then scale,
        //      split and write the wave's rows to the A image
        auto finish_tile = [&](int tb, const TInfo& info, ACC& acc, int64_t s) {
            const unsigned char* const LT = LTb(tb);
#pragma unroll
            for (int qd = 0; qd < C::NQD; ++qd) {
                const int row = 4 * qd + gq;
                const int ndeg = (flags & MIGNN_DIAG_NO_LOCAL) ? 0 : info.maxdeg;
                for (int u0 = 0; u0 < ndeg; u0 += UBE) {
                    uint2 pw_[UBE];
#pragma unroll
                    for (int uu = 0; uu < UBE; ++uu)
                        pw_[uu] = *reinterpret_cast<const uint2*>(LT + (row * C::LTS + u0 + uu) * 8);
                    f32x4 v[UBE][C::CH];
#pragma unroll
                    for (int uu = 0; uu < UBE; ++uu)
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
                            v[uu][j] = *reinterpret_cast<const f32x4*>(lds + (pw_[uu].x ^ coff[j]));
#pragma unroll
                    for (int uu = 0; uu < UBE; ++uu) {
                        const float w = __builtin_bit_cast(float, pw_[uu].y);
#pragma unroll
                        for (int j = 0; j < C::CH; ++j)
#pragma unroll
                            for (int r = 0; r < 4; ++r) acc[qd][j][r] = fmaf(w, v[uu][j][r], acc[qd][j][r]);
                    }
                }
                if (qd == 0 && pw == 0) stamp(trace, lane_, s, 2);
                // scale exponent (max over the row's 16 lanes: one DPP row), split, store
                uint32_t m = 0;
#pragma unroll
                for (int j = 0; j < C::CH; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) m = max(m, __float_as_uint(fabsf(acc[qd][j][r])));
                m = row_max_u32(m);
                const int p = scale_exp(m);
                const float sc = __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
                const int lrow = pw * C::PROWS + row;
                f16x4 h[C::CH], l[C::CH];
#pragma unroll
                for (int j = 0; j < C::CH; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float sv = acc[qd][j][r] * sc;
                        const _Float16 hh = static_cast<_Float16>(sv);
                        h[j][r] = hh;
                        l[j][r] = static_cast<_Float16>(sv - static_cast<float>(hh));
                    }
                wait_a(s);
#pragma unroll
                for (int j = 0; j < C::CH; ++j) {
                    const int hc = 4 * (c0 + 16 * j);  // first half of my chunk in the row
                    *reinterpret_cast<f16x4*>(&AH[lrow * C::AS + hc]) = h[j];
                    *reinterpret_cast<f16x4*>(&AL[lrow * C::AS + hc]) = l[j];
                }
                if (iq == 0) REXP[lrow] = p;
            }
        };

        // ---- pipeline: at step s the wave
        //   1. loads the CSR indices of tile s+3 (row_ptr of tile s+4),
        //   2. builds tile s+2's tables and issues its out-of-tile gathers,
        //   3. finishes tile s+1 (its out-of-tile sums were formed a step ago),
        //   4. sums tile s+2's gathered rows into the accumulators.
        XV xv;
        ACC acc;
        PIdx pa{}, pb{};
        pa.rpv = p_load_rpv<C::PROWS>(row_ptr, first_row(tile_of(0)), row_end, lane_);
        p_load_entries<C::PROWS>(pa, col, ew, lane_);
        pb.rpv = p_load_rpv<C::PROWS>(row_ptr, first_row(tile_of(1)), row_end, lane_);
        p_load_entries<C::PROWS>(pb, col, ew, lane_);
        int rpc = p_load_rpv<C::PROWS>(row_ptr, first_row(tile_of(2)), row_end, lane_);
        TInfo ia = build_tables(tile_of(0), pa, 0);
        issue_ext(0, xv);
        sum_ext(0, xv, ia, acc);
        int rpa = pa.rpv;
        block_barrier<0xC07F>();   // zero row, counters, own rows of tile 0 (lgkmcnt(0))
        for (int64_t s = -1; s < nsteps; ++s) {
            const int ta = static_cast<int>((s + 1) & 1), tbb = ta ^ 1;
            PIdx pc{};
            pc.rpv = rpc;
            p_load_entries<C::PROWS>(pc, col, ew, lane_);                      // tile s+3
            const int rpd = p_load_rpv<C::PROWS>(row_ptr, first_row(tile_of(s + 4)), row_end, lane_);
            if (pw == 0) stamp(trace, lane_, s, 0);
            // (re)built every step: past the last tile this only resets the
            // tables to empty slots, so the gathers never see stale columns
            const bool prod = !(flags & MIGNN_DIAG_NO_PRODUCE);
            const bool dext = prod && !(flags & MIGNN_DIAG_NO_EXT);
            const TInfo ib = (prod && !(flags & MIGNN_DIAG_NO_TABLES))
                                 ? build_tables(tile_of(s + 2), pb, tbb) : TInfo{0, 7, 0};
            if (dext) issue_ext(tbb, xv);
            if (pw == 0) stamp(trace, lane_, s, 1);
            a_free = s < 0;
            const int64_t t1 = tile_of(s + 1);
            if (s + 1 < nsteps && t1 < ntiles && prod) {
                if (ia.slow) slow_rows(t1, rpa, s);
                else finish_tile(ta, ia, acc, s);
            }
            if (pw == 0) stamp(trace, lane_, s, 3);
            if (dext) sum_ext(tbb, xv, ib, acc);
            rpa = pb.rpv;
            pb = pc;
            rpc = rpd;
            ia = ib;
            block_barrier<0xC07F>();   // this step's LDS writes done (lgkmcnt(0))
        }
        return;
    }

    // ==================================================================== consumer
    // wave (wm, wn): rows [wm * IB * 16, +IB * 16) x columns [32 wn, 32 wn + 32)
    const int wn = wave % C::WN, wm = wave / C::WN;
    int lane_ = lane;
    asm volatile("" : "+v"(lane_));
    const int rr = lane_ & 15, gg = lane_ >> 4;
    const int n0 = wn * 16 * C::JB;

    // own rows of a tile -> own-row image (LDS-DMA, 1 KB pieces, chunk c of
    // row lr stored at chunk position c ^ (lr & 7)); returns pieces issued
    auto x_dma = [&](int64_t tile) -> bool {
        if (tile >= ntiles) return false;
        const int64_t t0 = row_begin + tile * C::BM;
        const int buf = xbuf_of(tile);
        int l = lane_;
        asm volatile("" : "+v"(l));   // recompute the addresses per call (no hoisted 64-bit regs)
#pragma unroll
        for (int pp = 0; pp < C::NPC; ++pp) {
            const int p = pp * C::NCW + wave;
            const int lr = p * C::RPP + l / C::LPR;
            const int pos = l % C::LPR;
            int64_t row = t0 + lr;
            if (row >= row_end) row = row_end - 1;       // any valid row: never read
            const float* g = x + row * ldx + 4 * (pos ^ (lr & 7));
            glds16(g, lds_addr(lds + buf * C::X_BYTES + p * 1024));
        }
        return true;
    };

    // W rows n0 + 16 jb + rr as split fp16 MFMA A-operands: lane (r, g) holds
    // W[n][32 kc + 8 g + j], j < 8, scaled by 2^qw (one exponent per wave)
    f16x8 wh[C::JB][C::KC], wl[C::JB][C::KC];
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);
    int qw;
    {
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
        qw = scale_exp(wave_max_u32(m));
#pragma unroll
        for (int jb = 0; jb < C::JB; ++jb)
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    _Float16 h, l;
                    split16(wv[jb][kc][j], qw, h, l);
                    wh[jb][kc][j] = h;
                    wl[jb][kc][j] = l;
                }
    }
    // bias / BN scale / shift of the wave's 32 columns -> LDS (read per tile)
    if (lane_ < 16 * C::JB) {
        const int n = n0 + lane_;
        EPI[n] = (flags & MIGNN_EPI_BIAS) ? bias[n] : 0.f;
        EPI[H + n] = (flags & MIGNN_EPI_AFFINE) ? scale[n] : 1.f;
        EPI[2 * H + n] = (flags & MIGNN_EPI_AFFINE) ? shift[n] : 0.f;
    }
    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;

    x_dma(tile_of(0));             // (tile 1 at step -1)
    block_barrier<0x70>();   // own rows of tile 0 landed: vmcnt(0) lgkmcnt(0)
    for (int64_t s = -1; s < nsteps; ++s) {
        const int64_t tile = tile_of(s);
        const bool work = s >= 0 && tile < ntiles;
        const bool mm = work && !(flags & MIGNN_DIAG_NO_MFMA);
        f32x4 acc[C::IB][C::JB];
        int pr[C::IB];
        if (work) {
            // seed: (residual + bias) * 2^(p_row + q_w)
            const unsigned char* const X = lds + xbuf_of(tile) * C::X_BYTES;
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib) {
                const int lr = (wm * C::IB + ib) * 16 + rr;
                pr[ib] = REXP[lr];
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
                    const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[n0 + 16 * jb + 4 * gg]);
                    float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (has_res) {
                        const int ch = ((n0 + 16 * jb) >> 2) + gg;
                        rv = *reinterpret_cast<const float4*>(X + lr * C::ROWB + ((ch ^ (lr & 7)) << 4));
                    }
                    const float rvv[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[ib][jb][r] = ldexpf(rvv[r] + bo[r], pr[ib] + qw);
                }
            }
        }
        // residual taken (or nothing to take): once every consumer has, the
        // buffer takes the own rows of tile s+2
        if (s >= 0 && lane_ == 0) lds_bump(cntX);
        lds_wait(cntX, C::NCW * static_cast<int>(s + 1));
        if (wave == 0) stamp(trace, lane_, s, 4);
        // own rows of tile s+2 into the buffer just freed: before the MFMAs, or
        // (MIGNN_SCHED_DMA_LATE) after the epilogue stores, away from the
        // producers' gather burst at the start of the step
        const bool dma_late = (flags & MIGNN_SCHED_DMA_LATE) != 0;
        if (!dma_late && s + C::XBUF < nsteps) x_dma(tile_of(s + C::XBUF));
        if (wave == 0) stamp(trace, lane_, s, 5);
        if (mm) {
            // fragments of block (kc, ib) = step t = kc * IB + ib; the next
            // block's pair is read while this block's 3 x JB MFMAs run
            // per-tile base (laundered: keeps the 2 x KC x IB fragment addresses
            // from being hoisted into registers; they become immediate offsets)
            int fb = (wm * C::IB * 16 + rr) * C::AS + 8 * gg;
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
            for (int t = 0; t < C::KC * C::IB; ++t) {
                const int kc = t / C::IB, ib = t % C::IB;
                if (t + 1 < C::KC * C::IB) frag(t + 1, fh[(t + 1) & 1], fl[(t + 1) & 1]);
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
                    acc[ib][jb] = mfma16x16x32h(wh[jb][kc], fh[t & 1], acc[ib][jb]);
                    acc[ib][jb] = mfma16x16x32h(wh[jb][kc], fl[t & 1], acc[ib][jb]);
                    acc[ib][jb] = mfma16x16x32h(wl[jb][kc], fh[t & 1], acc[ib][jb]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // A image read (the last fragment pair is consumed by the MFMAs
        // above): producers may overwrite it with the next tile
        if (s >= 0 && lane_ == 0) lds_bump(cntA);
        if (wave == 0) stamp(trace, lane_, s, 6);
        bool stored = false;
        if (mm) {
            // epilogue: unscale, BN affine, ReLU -> the staging tile (row lr,
            // 16-B chunk ch at position ch ^ (lr & 15))
            const int64_t t0 = row_begin + tile * C::BM;
            stored = t0 + C::BM <= row_end;    // every row of the tile stored below
#pragma unroll
            for (int ib = 0; ib < C::IB; ++ib) {
#pragma unroll
                for (int jb = 0; jb < C::JB; ++jb) {
                    const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + n0 + 16 * jb + 4 * gg]);
                    const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + n0 + 16 * jb + 4 * gg]);
                    float o[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v = ldexpf(acc[ib][jb][r], -(pr[ib] + qw));
                        if (flags & MIGNN_EPI_AFFINE) v = v * so[r] + ho[r];
                        if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
                        o[r] = v;
                    }
                    const int lr = (wm * C::IB + ib) * 16 + rr;
                    const int ch = ((n0 + 16 * jb) >> 2) + gg;
                    *reinterpret_cast<f32x4*>(lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4)) =
                        f32x4{o[0], o[1], o[2], o[3]};
                }
            }
        }
        // every consumer's blocks staged -> whole rows: consumer w stores
        // rows 16 w .. 16 w + 15, two per instruction (a half-wave per row)
        if (s >= 0 && lane_ == 0) lds_bump(cntS);
        if (mm) {
            lds_wait(cntS, C::NCW * static_cast<int>(s + 1));
            const int64_t t0 = row_begin + tile * C::BM;
            constexpr int LPRW = C::ROWB / 16;          // lanes per row (32 at H = 128)
            constexpr int RPI = 64 / LPRW;              // rows per store instruction
            const int ch = lane_ % LPRW;
#pragma unroll
            for (int i = 0; i < C::NSTG; ++i) {
                const int lr = wave * (C::BM / C::NCW) + i * RPI + lane_ / LPRW;
                const f32x4 v = *reinterpret_cast<const f32x4*>(
                    lds + C::OFF_STG + lr * C::ROWB + ((ch ^ (lr & 15)) << 4));
                if (t0 + lr < row_end)
                    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + (t0 + lr) * ldo + 4 * ch));
            }
        }
        if (dma_late && s + C::XBUF < nsteps) x_dma(tile_of(s + C::XBUF));
        if (wave == 0) stamp(trace, lane_, s, 7);
        // this step's DMA (tile s+2) is read by the producers next step -- it
        // must land now; the row stores (the youngest vector-memory
        // operations) may fly
        if (stored) block_barrier<0x70 | C::NSTG>();
        else block_barrier<0x70>();
    }
}

template <int H, int NC>
int launch_f16x3(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                 int64_t ldx, int64_t rb, int64_t re, const float* w, const float* bias,
                 const float* scale, const float* shift, int flags, float* out, int64_t ldo,
                 hipStream_t st) {
    using C = SCfg<H, NC>;
    static int grid_cache[64] = {0};
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& G = grid_cache[dev & 63];
    if (G == 0) {
        int cus = 0;
        MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        G = (cus / 8) * 8;
        if (G < 8) G = 8;
    }
    const int64_t ntiles = (re - rb + C::BM - 1) / C::BM;
    int grid = G;
    if (ntiles < grid) grid = static_cast<int>(((ntiles + 7) / 8) * 8);
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(C::NT), 0, st, row_ptr, col, ew, x, ldx, rb, re, w,
                           bias, scale, shift, flags, out, ldo,
                           (flags & MIGNN_DIAG_TRACE) ? g_trace16_host : nullptr);
    };
    if (flags == kBN) go(gcn_f16x3_kernel<H, NC, kBN>);
    else if (flags == kNoBN) go(gcn_f16x3_kernel<H, NC, kNoBN>);
    else go(gcn_f16x3_kernel<H, NC>);
    return launch_status("gcn_f16x3_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

static int gcn_f16x3_impl(const int32_t* row_ptr, const int32_t* col,
                                          const float* ew, const float* x, int64_t ldx,
                                          int64_t rb, int64_t re, int h, const float* w,
                                          const float* bias, const float* scale,
                                          const float* shift, int flags, float* out, int64_t ldo,
                                          void* stream);

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_set_trace_f16x3(void* buf) {
    g_trace16_host = static_cast<unsigned long long*>(buf);
    return MIGNN_OK;
}
#endif

extern "C" int mignn_device_errors(unsigned int* out, int clear) {
    MIGNN_REQUIRE(out, "device_errors: null pointer");
    MIGNN_HIP(hipDeviceSynchronize());
    MIGNN_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_device_errors), sizeof(unsigned int), 0,
                                  hipMemcpyDeviceToHost));
    if (clear) {
        const unsigned int zero = 0u;
        MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_device_errors), &zero, sizeof(unsigned int), 0,
                                    hipMemcpyHostToDevice));
    }
    const int rc = win_device_errors(out, clear);
    return rc ? rc : ring_device_errors(out, clear);
}

extern "C" int mignn_gcn_layer_f16x3(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                     const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                     const float* w, const float* bias, const float* scale,
                                     const float* shift, int flags, float* out, int64_t ldo,
                                     void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_f16x3: unknown flags 0x%x", flags);
    return gcn_f16x3_impl(row_ptr, col, ew, x, ldx, rb, re, h, w, bias, scale, shift,
                                      flags, out, ldo, stream);
}

static int gcn_f16x3_impl(const int32_t* row_ptr, const int32_t* col,
                                          const float* ew, const float* x, int64_t ldx,
                                          int64_t rb, int64_t re, int h, const float* w,
                                          const float* bias, const float* scale,
                                          const float* shift, int flags, float* out, int64_t ldo,
                                          void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && x && w && out, "gcn_layer_f16x3: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_layer_f16x3: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(w) && aligned16(out), "gcn_layer_f16x3: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h,
                  "gcn_layer_f16x3: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_f16x3: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_f16x3: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_f16x3: affine");
    MIGNN_REQUIRE(x != out, "gcn_layer_f16x3: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    if (flags & MIGNN_SCHED_NC8)
        return h == 128 ? launch_f16x3<128, 8>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale,
                                               shift, flags, out, ldo, st)
                        : launch_f16x3<64, 8>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale,
                                              shift, flags, out, ldo, st);
    return h == 128 ? launch_f16x3<128, 4>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift,
                                           flags, out, ldo, st)
                    : launch_f16x3<64, 4>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift,
                                          flags, out, ldo, st);
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_gcn_layer_f16x3(const int32_t* row_ptr, const int32_t* col,
                                          const float* ew, const float* x, int64_t ldx,
                                          int64_t rb, int64_t re, int h, const float* w,
                                          const float* bias, const float* scale,
                                          const float* shift, int flags, float* out, int64_t ldo,
                                          void* stream) {
    return gcn_f16x3_impl(row_ptr, col, ew, x, ldx, rb, re, h, w, bias, scale, shift, flags, out, ldo, stream);
}
#endif

MIGNN_DMA_OOB_EXPORT(mignn_diag_dma_oob_pc)
