// Fused GCN layer in split-fp16 MFMA arithmetic -- the north-star hot kernel
// (GCNConv + residual + BatchNorm(eval) + ReLU, gnn_model.py:166, :184-191):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// One pass over HBM: every x row is read once from HBM into an LDS image of
// its 64-row tile and reused from there by its in-tile neighbours; out-of-
// tile neighbours come through L2 (the internal locality order,
// mignn_locality_order, keeps most of a mesh's CSR entries in-tile); every
// output row is written once.
//
// Structure: one 4-wave workgroup per CU (one wave per SIMD), persistent over
// 64-row tiles in an XCD-contiguous order (each XCD walks its own run of
// tiles, 32 at a time: its L2 holds the tiles' z-neighbours).  The four waves
// are symmetric -- wave w owns rows [16 w, 16 w + 16) of the tile and runs
// the whole layer for them in registers, in the v_mfma_f32_16x16x32_f16
// B-operand layout (lane (r, g) = row r, 16-B chunks 4 h + g, h < H/16):
//   1. own rows of tile s+1 -> LDS image (LDS-DMA, issued a step ahead);
//   2. out-of-tile rows of tile s+1 -> registers (EX per row, issued a step
//      ahead), their CSR entries compacted per lane;
//   3. tile s: sum of the prefetched out-of-tile rows, then the in-tile
//      entries from the image (CSR order within each group), fp32;
//   4. split: the row's 4 lanes agree on 2^p (row max in [2^13, 2^14)),
//      a 2^p = hi + lo in fp16 -- already the MFMA B fragments;
//   5. transform: D[n][row] = W'.agg^T, three 16x16x32 MFMAs per block
//      (hi.hi + hi.lo + lo.hi); W' = diag(BN scale) W split once per launch
//      into fragments held in LDS;
//   6. epilogue from the accumulators (row r, columns 16 nb + 4 g + i):
//      out = relu(acc 2^-(p+q) + x sc + (b sc + shift)), residual x from the
//      image, 16-B stores (16 rows x 64 B per instruction).
// One block barrier per step (the image buffers change hands); everything
// else is per wave.
//
// Arithmetic: a.w = 2^-(p+q) (ah wh + ah wl + al wh) + O(2^-22 |a||w|) per
// product, fp32 accumulation (q per 16 output columns).  Scales clamped to
// [2^-60, 2^60]: |values| < 2^70 (fp16 hi overflow beyond).  Sum order per
// row: out-of-tile entries (CSR order), then in-tile entries (CSR order) --
// deterministic, no atomics.
#include "common.hpp"

namespace mignn {
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_f;

template <int H>
struct FCfg {
    static_assert(H == 64 || H == 128, "gcn_fused: H in {64, 128}");
    static constexpr int NW = 4;                      // waves (one per SIMD)
    static constexpr int NT = NW * 64;
    static constexpr int BM = 64;                     // rows per tile
    static constexpr int RW = 16;                     // rows per wave
    static constexpr int NH = H / 16;                 // 16-B chunks per lane of a row
    static constexpr int KC = H / 32;                 // 32-deep k chunks
    static constexpr int NB = H / 16;                 // 16-column output blocks
    static constexpr int ROWB = H * 4;                // bytes per row
    static constexpr int NCH = ROWB / 16;             // 16-B chunks per row
    static constexpr int X_BYTES = BM * ROWB;         // one own-row image
    static constexpr int FRAG = 1024;
    static constexpr int S = 8;                       // CSR entries per row in registers
    static constexpr int EX = 3;                      // out-of-tile rows per row in registers
    static constexpr int OFF_X = 0;                   // two images
    static constexpr int OFF_ZERO = 2 * X_BYTES;      // a zero row
    static constexpr int OFF_W = OFF_ZERO + ROWB;     // W' fragments [kc][nb][hi, lo]
    static constexpr int OFF_TA = OFF_W + KC * NB * 2 * FRAG;  // residual multiplier per column
    static constexpr int OFF_TB = OFF_TA + H * 4;              // additive term per column
    static constexpr int OFF_Q = OFF_TB + H * 4;               // exponent per column block
    // CSR tables of a wave's 16 rows (two steps: the one summed, the next):
    // LT [16][S] {in-tile row or -1, weight}; ET [16][4] {column or -1, weight}
    static constexpr int LT_BYTES = RW * S * 8;
    static constexpr int TAB_BYTES = LT_BYTES + RW * 4 * 8;
    static constexpr int OFF_TAB = OFF_Q + 16 * 4;
    static constexpr int LDS_BYTES = OFF_TAB + 2 * NW * TAB_BYTES;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
    static constexpr int NPIECE = X_BYTES / 1024 / NW;   // LDS-DMA pieces per wave per tile
    static constexpr int RPP = 1024 / ROWB;              // rows per 1-KB piece
    static constexpr int NST = NB;                       // row stores per wave per tile
};

__device__ __attribute__((aligned(16))) float g_zero_row_f[256];

__device__ __forceinline__ float p2f(int p) {
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}

// max * 2^p in [2^13, 2^14), clamped to [-60, 60] (zero / tiny blocks: 60)
__device__ __forceinline__ int fexp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return max(-60, min(140 - eb, 60));
}

__device__ __forceinline__ uint32_t lds_off(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_f)(p)));
}

// LDS-DMA of 16 B per lane (global_load_lds_dwordx4) to the wave-uniform LDS
// byte address `dst` (+16 x lane).  Inline asm: the compiler neither counts
// it in its vmcnt bookkeeping nor inserts vmcnt(0) before later LDS reads;
// the kernel waits for it itself (the counted wait before each step's
// barrier).
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

// s_waitcnt <imm> + s_barrier (vmcnt(n) lgkmcnt(0) = 0x70 | n, n < 16)
template <int WAITCNT>
__device__ __forceinline__ void step_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(WAITCNT);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// XM (experiments): 1 no table build, 2 no out-of-tile gather, 4 no in-tile sum
template <int H, int XM = 0>
__global__ __launch_bounds__(FCfg<H>::NT, 1) void gcn_fused_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t rb,
    int64_t re, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo) {
    using C = FCfg<H>;
    constexpr int S = C::S, EX = C::EX, NH = C::NH;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    float* const TA = reinterpret_cast<float*>(lds + C::OFF_TA);
    float* const TB = reinterpret_cast<float*>(lds + C::OFF_TB);
    uint32_t* const QM = reinterpret_cast<uint32_t*>(lds + C::OFF_Q);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const bool aff = (flags & MIGNN_EPI_AFFINE) != 0;

    // ---------------------------------------------------------------- prologue
    // epilogue terms per column; W' = diag(sc) W split per 16-column block
    // into fragments: lane (m, g) of (kc, nb) holds W'[16 nb + m][k] at
    // k = 32 kc + 4 g + (j & 3) + 16 (j >> 2) -- the k of B-fragment element
    // j of the lane's gathered chunks 4 (2 kc + (j >> 2)) + g
    if (tid < H) {
        const float s = aff ? scale[tid] : 1.f;
        const float b = (flags & MIGNN_EPI_BIAS) ? bias[tid] : 0.f;
        TA[tid] = (flags & MIGNN_EPI_RESIDUAL) ? s : 0.f;
        TB[tid] = aff ? fmaf(b, s, shift[tid]) : b;
    }
    if (tid < C::NB) QM[tid] = 0u;
    for (int i = tid; i < C::ROWB / 4; i += C::NT)
        reinterpret_cast<float*>(lds + C::OFF_ZERO)[i] = 0.f;
    __syncthreads();
    constexpr int NTASK = C::KC * C::NB * 64;
    auto wvals = [&](int task, float (&v)[8]) -> int {
        const int ln = task & 63, fb = task >> 6;
        const int nb = fb % C::NB, kc = fb / C::NB;
        const int m = 16 * nb + (ln & 15), gg = ln >> 4;
        const float s = aff ? scale[m] : 1.f;
        const float* wp = W + static_cast<int64_t>(m) * H + 32 * kc + 4 * gg;
        const float4 a = ld4(wp), b = ld4(wp + 16);
        v[0] = a.x * s; v[1] = a.y * s; v[2] = a.z * s; v[3] = a.w * s;
        v[4] = b.x * s; v[5] = b.y * s; v[6] = b.z * s; v[7] = b.w * s;
        return nb;
    };
    for (int task = tid; task < NTASK; task += C::NT) {
        float v[8];
        const int nb = wvals(task, v);
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(fabsf(v[j])));
        atomicMax(&QM[nb], m);
    }
    __syncthreads();
    for (int task = tid; task < NTASK; task += C::NT) {
        float v[8];
        const int nb = wvals(task, v);
        const float sq = p2f(fexp(QM[nb]));
        f16x8 hv, lv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float s = v[j] * sq;
            const _Float16 hh = static_cast<_Float16>(s);
            hv[j] = hh;
            lv[j] = static_cast<_Float16>(s - static_cast<float>(hh));
        }
        const int fb = task >> 6, ln = task & 63;
        *reinterpret_cast<f16x8*>(lds + C::OFF_W + (2 * fb) * C::FRAG + ln * 16) = hv;
        *reinterpret_cast<f16x8*>(lds + C::OFF_W + (2 * fb + 1) * C::FRAG + ln * 16) = lv;
    }
    __syncthreads();
    if (tid < C::NB) QM[tid] = static_cast<uint32_t>(fexp(QM[tid]));

    // ---------------------------------------------------------------- schedule
    const int64_t nrows = re - rb;
    const int64_t ntiles = (nrows + C::BM - 1) / C::BM;
    const int G = gridDim.x;                     // multiple of 8 (host)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = G >> 3;
    const int64_t nsteps = (ntiles + G - 1) / G;
    const int64_t chunk = nsteps * per_xcd;
    auto tile_of = [&](int64_t s) -> int64_t { return (int64_t)xcd * chunk + s * per_xcd + slot; };
    auto valid = [&](int64_t s) -> bool { return s < nsteps && tile_of(s) < ntiles; };

    // own rows of step s -> image buffer (s & 1): 1-KB pieces of RPP rows,
    // chunk c of tile row lr stored at chunk position c ^ (lr & 15)
    auto issue_dma = [&](int64_t s) {
        if (!valid(s)) return;
        const int64_t t0 = rb + tile_of(s) * C::BM;
        unsigned char* const X = lds + C::OFF_X + (s & 1) * C::X_BYTES;
        int l = lane;
        asm volatile("" : "+v"(l));
#pragma unroll
        for (int pc = 0; pc < C::NPIECE; ++pc) {
            const int piece = wave * C::NPIECE + pc;
            const int lr = piece * C::RPP + l / C::NCH;
            const int pos = l % C::NCH;
            int64_t row = t0 + lr;
            if (row >= re) row = re - 1;         // any valid row: never read
            const float* src = x + row * ldx + 4 * (pos ^ (lr & 15));
            dma16(src, lds_off(X + piece * 1024));
        }
    };
    // CSR of a wave's 16 rows at step s: row_ptr (lane i <= 16: row 16 w + i;
    // rows past the end read as empty), then the entries lane-per-entry
    auto load_rpv = [&](int64_t s) -> int {
        int64_t row = rb + tile_of(s) * C::BM + 16 * wave + (lane < 17 ? lane : 16);
        if (!valid(s)) return 0;
        if (row > re) row = re;
        return row_ptr[row];
    };
    struct Ent { int c[2]; float w[2]; };
    auto load_ent = [&](int rpv, Ent& en) {
        const int e0 = __builtin_amdgcn_readlane(rpv, 0);
        const int ne = __builtin_amdgcn_readlane(rpv, 16) - e0;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int idx = lane + 64 * hf;
            en.c[hf] = -1;
            en.w[hf] = 0.f;
            if (idx < ne) {
                en.c[hf] = col[e0 + idx];
                en.w[hf] = ew[e0 + idx];
            }
        }
    };
    // the tables of step s: LT[row][slot] = in-tile entries (the image row),
    // ET[row][k] = the k-th out-of-tile entry of the row; returns the max
    // degree and whether a row overflows them (> S entries or > EX
    // out-of-tile ones: the step then takes the general path)
    auto build = [&](int64_t s, int rpv, const Ent& en, int& maxd, bool& slow) {
        unsigned char* const T = lds + C::OFF_TAB + ((s & 1) * C::NW + wave) * C::TAB_BYTES;
        for (int i = lane; i < C::LT_BYTES / 16; i += 64)
            *reinterpret_cast<uint4*>(T + 16 * i) = make_uint4(~0u, 0u, ~0u, 0u);
        *reinterpret_cast<uint2*>(T + C::LT_BYTES + 8 * lane) = make_uint2(~0u, 0u);
        maxd = 0;
        slow = false;
        if (!valid(s)) return;
        const int64_t t0 = rb + tile_of(s) * C::BM;
        const int64_t rem = re - t0;
        const uint32_t nloc = static_cast<uint32_t>(rem < C::BM ? rem : C::BM);
        int rp[17];
#pragma unroll
        for (int i = 0; i <= 16; ++i) rp[i] = __builtin_amdgcn_readlane(rpv, i);
        const int e0 = rp[0];
        const int ne = rp[16] - e0;
#pragma unroll
        for (int i = 0; i < 16; ++i) maxd = max(maxd, rp[i + 1] - rp[i]);
        if (ne > 128) {
            slow = true;
            return;
        }
        uint64_t B0 = 0;
        bool over = false;
        auto below = [&](uint64_t m, int n) -> int {   // set bits of m below bit n (n in [0, 64])
            const uint64_t mk = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
            return __builtin_popcountll(m & mk);
        };
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int idx = lane + 64 * hf;
            const bool has = idx < ne;
            int q = 0, rs = 0;
#pragma unroll
            for (int i = 1; i < 16; ++i) {
                const int b = rp[i] - e0;
                const bool ge = idx >= b;
                q += ge ? 1 : 0;
                rs = ge ? b : rs;
            }
            const int u = idx - rs;
            const uint32_t off = static_cast<uint32_t>(en.c[hf] - static_cast<int>(t0));
            const bool in = has && off < nloc;
            const bool ext = has && !in;
            const uint64_t Bm = __builtin_amdgcn_ballot_w64(ext);
            if (hf == 0) B0 = Bm;
            // rank among the row's out-of-tile entries: set bits in [rs, idx)
            const int k = hf == 0 ? below(Bm, idx) - below(Bm, rs)
                                  : below(B0, 64) + below(Bm, idx - 64) -
                                        (rs >= 64 ? below(B0, 64) + below(Bm, rs - 64) : below(B0, rs));
            if (has && u < S)
                *reinterpret_cast<uint2*>(T + (q * S + u) * 8) =
                    make_uint2(in ? off : ~0u, in ? __float_as_uint(en.w[hf]) : 0u);
            if (ext && k < EX)
                *reinterpret_cast<uint2*>(T + C::LT_BYTES + (q * 4 + k) * 8) =
                    make_uint2(static_cast<uint32_t>(en.c[hf]), __float_as_uint(en.w[hf]));
            over = over || (has && u >= S) || (ext && k >= EX);
        }
        slow = __builtin_amdgcn_ballot_w64(over) != 0ull;
    };
    // out-of-tile rows of step s (ET) -> registers: lane (r, g) loads
    // chunks 4 h + g of the row; empty slots read a zero row
    const float* const zrow = g_zero_row_f + 4 * g;
    using XE = f32x4[EX][NH];
    auto gather_ext = [&](int64_t s, XE& xe) {
        const unsigned char* const T = lds + C::OFF_TAB + ((s & 1) * C::NW + wave) * C::TAB_BYTES;
        const uint4 e01 = *reinterpret_cast<const uint4*>(T + C::LT_BYTES + (r * 4) * 8);
        const uint2 e2 = *reinterpret_cast<const uint2*>(T + C::LT_BYTES + (r * 4 + 2) * 8);
        const int xc[3] = {static_cast<int>(e01.x), static_cast<int>(e01.z), static_cast<int>(e2.x)};
#pragma unroll
        for (int k = 0; k < EX; ++k) {
            const float* src = xc[k] >= 0 ? x + static_cast<int64_t>(xc[k]) * ldx + 4 * g : zrow;
#pragma unroll
            for (int h = 0; h < NH; ++h) xe[k][h] = *reinterpret_cast<const f32x4*>(src + 16 * h);
        }
    };

    // ---------------------------------------------------------------- pipeline
    // at step s: image s (DMA'd at step s-1), tables of s (built at step
    // s-1) and their out-of-tile rows (gathered at step s-1); entries of s+1
    // and row_ptr of s+2 (loaded at step s-1)
    XE xe;
    int rpv1, rpv2, maxd_c, maxd_n;
    bool slow_c, slow_n;
    Ent en1;
    {
        const int rpv0 = load_rpv(0);
        Ent en0;
        load_ent(rpv0, en0);
        rpv1 = load_rpv(1);
        issue_dma(0);
        load_ent(rpv1, en1);
        rpv2 = load_rpv(2);
        build(0, rpv0, en0, maxd_c, slow_c);
        gather_ext(0, xe);
    }
    step_barrier<0x70>();    // image 0 landed (every wave's pieces), lgkmcnt(0)

    const bool relu = (flags & MIGNN_EPI_RELU) != 0;
    const bool res_on = (flags & MIGNN_EPI_RESIDUAL) != 0;
    for (int64_t s = 0; s < nsteps; ++s) {
        const bool vs = valid(s);
        const int64_t t0 = rb + tile_of(s) * C::BM;
        unsigned char* const T = lds + C::OFF_TAB + ((s & 1) * C::NW + wave) * C::TAB_BYTES;
        // own rows of step s+1 into the other image (its last readers, step
        // s-1, are behind the barrier that ended that step)
        issue_dma(s + 1);
        // ---- 1. out-of-tile rows of step s (prefetched) -> agg
        f32x4 agg[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) agg[h] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!slow_c) {
            const uint4 e01 = *reinterpret_cast<const uint4*>(T + C::LT_BYTES + (r * 4) * 8);
            const uint2 e2 = *reinterpret_cast<const uint2*>(T + C::LT_BYTES + (r * 4 + 2) * 8);
            const float xw[3] = {__uint_as_float(e01.y), __uint_as_float(e01.w), __uint_as_float(e2.y)};
#pragma unroll
            for (int k = 0; k < EX; ++k)
#pragma unroll
                for (int h = 0; h < NH; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i) agg[h][i] = fmaf(xw[k], xe[k][h][i], agg[h][i]);
        }
        // ---- 2. step s+1: tables and out-of-tile rows; CSR of s+2, s+3
        if constexpr (!(XM & 1)) build(s + 1, rpv1, en1, maxd_n, slow_n);
        else { maxd_n = 7; slow_n = false; }
        if constexpr (!(XM & 2)) gather_ext(s + 1, xe);
        load_ent(rpv2, en1);
        rpv1 = rpv2;
        rpv2 = load_rpv(s + 3);
        // ---- 3. in-tile entries of step s from the image (CSR order)
        unsigned char* const X = lds + C::OFF_X + (s & 1) * C::X_BYTES;
        if (!slow_c && !(XM & 4)) {
            const int xoff = C::OFF_X + static_cast<int>(s & 1) * C::X_BYTES;
#pragma unroll
            for (int e = 0; e < S; ++e) {
                if (e >= maxd_c) break;
                const uint2 lw = *reinterpret_cast<const uint2*>(T + (r * S + e) * 8);
                const int lr = static_cast<int>(lw.x);
                // row lr, chunk 4 h + g at position (4 h + g) ^ (lr & 15):
                // byte offset base + 64 (h ^ (key >> 2)); empty -> the zero row
                const int key = lr & 15;
                const int base = lr >= 0 ? xoff + lr * C::ROWB + 16 * (g ^ (key & 3))
                                         : C::OFF_ZERO + 16 * g;
                const int kh = lr >= 0 ? (key & 12) << 4 : 0;
                f32x4 v[NH];
#pragma unroll
                for (int h = 0; h < NH; ++h)
                    v[h] = *reinterpret_cast<const f32x4*>(lds + (((64 * h) ^ kh) + base));
                const float w = __uint_as_float(lw.y);
#pragma unroll
                for (int h = 0; h < NH; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i) agg[h][i] = fmaf(w, v[h][i], agg[h][i]);
            }
        }
        else if (vs && !(XM & 4)) {
            // general path (rows with > S entries or > EX out-of-tile ones):
            // every entry of the lane's row, one at a time, CSR order
            const int64_t row = t0 + 16 * wave + r;
            int e0 = 0, deg = 0;
            if (row < re) {
                e0 = row_ptr[row];
                deg = row_ptr[row + 1] - e0;
            }
            for (int e = 0; e < maxd_c; ++e) {
                const bool has = e < deg;
                int c = 0;
                float w = 0.f;
                if (has) {
                    c = col[e0 + e];
                    w = ew[e0 + e];
                }
                const uint32_t off = static_cast<uint32_t>(c - static_cast<int>(t0));
                const bool in = has && off < static_cast<uint32_t>(C::BM) && t0 + off < re;
                f32x4 v[NH];
                if (in) {
                    const int lr = static_cast<int>(off);
                    const unsigned char* rp = X + lr * C::ROWB;
#pragma unroll
                    for (int h = 0; h < NH; ++h)
                        v[h] = *reinterpret_cast<const f32x4*>(rp + 16 * ((4 * h + g) ^ (lr & 15)));
                } else {
                    const float* src = has ? x + static_cast<int64_t>(c) * ldx + 4 * g : zrow;
#pragma unroll
                    for (int h = 0; h < NH; ++h) v[h] = *reinterpret_cast<const f32x4*>(src + 16 * h);
                }
#pragma unroll
                for (int h = 0; h < NH; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i) agg[h][i] = fmaf(w, v[h][i], agg[h][i]);
            }
        }
        // ---- 4. split with the row's scale (max over the row's 4 lanes)
        uint32_t mb = 0;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) mb = max(mb, __float_as_uint(fabsf(agg[h][i])));
        {
            const auto r16 = __builtin_amdgcn_permlane16_swap(mb, mb, false, false);
            mb = max(static_cast<uint32_t>(r16[0]), static_cast<uint32_t>(r16[1]));
            const auto r32 = __builtin_amdgcn_permlane32_swap(mb, mb, false, false);
            mb = max(static_cast<uint32_t>(r32[0]), static_cast<uint32_t>(r32[1]));
        }
        const int p = fexp(mb);
        const float sp = p2f(p);
        // ---- 5. transform
        f32x4 acc[C::NB];
#pragma unroll
        for (int nb = 0; nb < C::NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
        int wofs = lane * 16;
        asm volatile("" : "+v"(wofs));            // fragments re-read per step
        const unsigned char* const wf = lds + C::OFF_W + wofs;
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc) {
            f16x8 bh, bl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sv = agg[2 * kc + (j >> 2)][j & 3] * sp;
                const _Float16 hh = static_cast<_Float16>(sv);
                bh[j] = hh;
                bl[j] = static_cast<_Float16>(sv - static_cast<float>(hh));
            }
#pragma unroll
            for (int nb = 0; nb < C::NB; ++nb) {
                const int fb = kc * C::NB + nb;
                const f16x8 wh = *reinterpret_cast<const f16x8*>(wf + (2 * fb) * C::FRAG);
                const f16x8 wl = *reinterpret_cast<const f16x8*>(wf + (2 * fb + 1) * C::FRAG);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[nb], 0, 0, 0);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[nb], 0, 0, 0);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[nb], 0, 0, 0);
            }
        }
        // ---- 6. epilogue: residual from the image (own row 16 w + r), BN,
        // ReLU, 16-B stores
        {
            const int lr = 16 * wave + r;
            const int64_t grow = t0 + lr;
            int eofs = 16 * g;
            asm volatile("" : "+v"(eofs));
#pragma unroll
            for (int nb = 0; nb < C::NB; ++nb) {
                const float u = p2f(-(p + static_cast<int>(QM[nb])));
                const f32x4 ta = *reinterpret_cast<const f32x4*>(lds + C::OFF_TA + 64 * nb + eofs);
                const f32x4 tb = *reinterpret_cast<const f32x4*>(lds + C::OFF_TB + 64 * nb + eofs);
                const int ch = 4 * nb + g;
                f32x4 xr = f32x4{0.f, 0.f, 0.f, 0.f};
                if (res_on) xr = *reinterpret_cast<const f32x4*>(X + lr * C::ROWB + 16 * (ch ^ (lr & 15)));
                f32x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = fmaf(acc[nb][i], u, fmaf(xr[i], ta[i], tb[i]));
                    if (relu) v = v < 0.0f ? 0.0f : v;
                    o[i] = v;
                }
                if (vs && grow < re)
                    __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + grow * ldo + 4 * ch));
            }
        }
        // the next image (DMA'd this step), the out-of-tile rows and CSR
        // entries of step s+1 must have landed, and every wave be done with
        // this step's image before the next step overwrites it; this step's
        // row stores (the youngest vector-memory operations) may fly
        maxd_c = maxd_n;
        slow_c = slow_n;
        if (vs && t0 + 16 * wave + C::RW <= re) step_barrier<0x70 | C::NST>();
        else step_barrier<0x70>();
    }
}

template <int H, int XM>
int launch_fused(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                 int64_t ldx, int64_t rb, int64_t re, const float* w, const float* bias,
                 const float* scale, const float* shift, int flags, float* out, int64_t ldo,
                 hipStream_t st) {
    using C = FCfg<H>;
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
    hipLaunchKernelGGL((gcn_fused_kernel<H, XM>), dim3(grid), dim3(C::NT), 0, st, row_ptr, col, ew, x,
                       ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    return launch_status("gcn_fused_kernel");
}

}  // namespace

int gcn_fused_layer(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                    int64_t ldx, int64_t rb, int64_t re, int h, const float* w, const float* bias,
                    const float* scale, const float* shift, int flags, float* out, int64_t ldo,
                    void* stream, int xm) {
    hipStream_t st = as_stream(stream);
#define MIGNN_FUSED(XM) \
    return h == 128 ? launch_fused<128, XM>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, \
                                            flags, out, ldo, st) \
                    : launch_fused<64, XM>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, \
                                           flags, out, ldo, st)
    if (xm == 7) MIGNN_FUSED(7);
    if (xm == 3) MIGNN_FUSED(3);
    MIGNN_FUSED(0);
#undef MIGNN_FUSED
}

}  // namespace mignn
