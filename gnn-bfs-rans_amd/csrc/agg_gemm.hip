// Fused aggregate -> split-fp16 transform(s) for the H = 256 convolutions
// (configs[4]'s GIN H256 L8 and GCN at H = 256):
//
//   GIN (gnn_model.py:70-75, PyG GINConv, eps buffer):
//       a_i   = sum_{j in row i} x_j + (1 + eps) x_i        (CSR order, verbatim)
//       h_i   = relu(a_i W1^T + b1)                          (nn.0, nn.1)
//       out_i = epi(h_i W2^T + b2; residual x_i, BN, ReLU)  (nn.2, gnn_model.py:184-191)
//   GCN (gnn_model.py:63, PyG GCNConv):
//       a_i   = sum_{e in row i} ew_e x_{col e}              (gcn_norm weights, self loop in CSR)
//       out_i = epi(a_i W^T + b; residual x_i, BN, ReLU)
//
// Neither a nor h reaches HBM: per layer the kernel reads x (own rows and the
// gathered neighbour rows, mostly L2 hits in the locality order) and writes
// out -- the aggregate + GEMM + GEMM chain it replaces wrote and re-read a and
// h ([N, 256] fp32 each: 26 GB per 12.6M-node GIN layer).
//
// Layout (one wave = 16 rows; lane (r, g) = row r, lane group g):
//   * the aggregate is formed one 32-wide k chunk at a time directly in the
//     MFMA B-operand layout: lane (r, g) gathers row r's neighbours' values
//     k = 32 kc + 8 g .. + 7 (two 16-B loads per CSR entry), sums them in
//     fp32 (CSR order), and splits them with the row's ONLINE exponent (the
//     split-fp16 GEMM's scheme, gemm_f16x3.hip: lowered with an exact rescale
//     of the row's accumulators when a chunk's max needs it);
//   * D[n][row] = W . a^T, three v_mfma_f32_16x16x32_f16 per 16x16x32 block
//     (hi.hi + hi.lo + lo.hi), W = the mignn_linear_f16x3_prep image streamed
//     through LDS one 32-KB k chunk at a time (LDS-DMA, double-buffered,
//     shared by the block's waves: one barrier per chunk);
//   * GIN's second transform takes h from the accumulators as they stand:
//     lane (r, g) holds h[r][16 cb + 4 g + i], which is B-operand element j of
//     chunk kc for cb = 2 kc + j / 4, i = j % 4 -- a fixed permutation of k,
//     applied to W2's image instead (mignn_gin_fused_prep: k-permuted image),
//     so h never leaves registers;
//   * epilogue from the accumulators (unscale, bias, residual x_i, BN affine,
//     ReLU), 16-B non-temporal stores.
// The next chunk's neighbour rows are loaded while the current chunk's MFMAs
// run.  Rows with more than AS CSR entries take the extra entries one by one
// (correct, not fast).  Sum order per row: CSR order, then (GIN) the
// (1 + eps) x_i term -- as PyG GINConv (out + (1 + eps) * x_r).
#include "common.hpp"

namespace mignn {
MIGNN_DMA_OOB_WORD
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_ag;

constexpr int AH = 256;               // width (K = N = 256)
constexpr int AKP = AH / 32;          // 32-deep k chunks
constexpr int ACB = AH / 16;          // 16-column blocks
constexpr int AFRAG = 1024;           // one MFMA operand fragment (64 lanes x 16 B)
constexpr int ACHUNK = ACB * 2 * AFRAG;   // one k chunk of a W image: 32 KB
constexpr int AS = 8;                 // CSR entry slots per row gathered per chunk
enum { AGG_GIN = 0, AGG_GCN = 1 };

__device__ __attribute__((aligned(16))) float g_zero_row_ag[AH];

// max * 2^p in [2^13, 2^14); 100 for zero / tiny maxima (gemm_f16x3.hip)
__device__ __forceinline__ int sexp_ag(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 100);
}
__device__ __forceinline__ float p2_ag(int p) {
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}
// 2^-q for q in [-126, 126] in one v_mad_i32_i24 (the per-column unscale of
// a split image: acc 2^-q is exact, so acc 2^-q 2^-p rounds like ldexp)
__device__ __forceinline__ float p2neg_ag(int q) {
    return __uint_as_float(static_cast<uint32_t>(__mul24(q, -8388608) + 0x3f800000));
}
// Output-column order of the GIN nn.2 image (mignn_gin_fused_prep): image
// column m = 16 cb + 4 g + i (the accumulator position of lane (r, g), block
// cb) holds output feature 32 (cb >> 1) + 8 g + 4 (cb & 1) + i -- the
// features lane (r, g) reads of its own row in the B-operand layout of chunk
// cb >> 1 during the aggregation, so the residual x_i stays in its registers
// (one HBM read of the own rows per layer).  A bijection on [0, 256).
__host__ __device__ __forceinline__ int gin_operm(int m) {
    const int cb = m >> 4, g = (m >> 2) & 3, i = m & 3;
    return 32 * (cb >> 1) + 8 * g + 4 * (cb & 1) + i;
}
__device__ __forceinline__ uint32_t lds_addr_ag(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_ag)(p)));
}
// LDS-DMA of 16 B per lane (inline asm: the compiler does not count it; the
// kernel's explicit vmcnt(0) before each chunk barrier covers it)
__device__ __forceinline__ void glds16_ag(const void* src, uint32_t dst) {
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
// max over the 4 lanes of a row (l, l^16, l^32, l^48)
__device__ __forceinline__ uint32_t rowmax4(uint32_t m) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
    m = max(static_cast<uint32_t>(r16[0]), static_cast<uint32_t>(r16[1]));
    const auto r32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return max(static_cast<uint32_t>(r32[0]), static_cast<uint32_t>(r32[1]));
}
__device__ __forceinline__ void chunk_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x70);          // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(N) lgkmcnt(0) + s_barrier (N < 16)
template <int N>
__device__ __forceinline__ void vm_barrier() {
    static_assert(N >= 0 && N < 16, "vmcnt");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x70 | N);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(N) lgkmcnt(0) + s_barrier, N < 64 (vmcnt bits 3:0 and 15:14;
// N = 63: LDS reads only)
template <int N>
__device__ __forceinline__ void vm_barrier64() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// sum over the 4 lanes of a row (every lane gets the same value)
__device__ __forceinline__ float rowsum4(float v) {
    const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(static_cast<uint32_t>(r16[0])) + __uint_as_float(static_cast<uint32_t>(r16[1]));
    const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(static_cast<uint32_t>(r32[0])) + __uint_as_float(static_cast<uint32_t>(r32[1]));
}

// Staged epilogue of the fused kernels (call with the LDS free, every wave):
// each wave DMAs its 16 own rows (the residual) into staging rows of NCB*64 B
// (16-B chunk c of row li at position c ^ (li & 15)), every lane replaces its
// NCB*4 values -- row lself, columns 16 cb + 4 g + i: bias, residual, BN, ReLU
// (gnn_model.py:184-191 order: conv + bias, + x, BN, ReLU) -- in place, and
// the wave stores whole rows (the accumulator layout would store 16 rows x
// 64 B per instruction).  EV = [2^-q | bias (0: off) | scale | shift][NCB*16] in LDS,
// written by the caller before the call.
// CRES: the residual is not read but computed, x_i[n] = TB[n] . (c0, c1, c2, 1)
// (GIN layer 0 from the coordinates: x = input_proj(pos), TB = [W_in | b_in])
// LG: also the next GAT layer's logits of each finished row, x_out . WLN^T
// (WLN [8][N] in LDS) -> lgn[row][8] (the row's 4 lanes summed)
// OPERM (GIN, NCB = 16): the accumulators are in gin_operm's output order --
// EV is indexed by image column, each value lands at its feature's staging
// slot, and the residual comes from RES (the lane's own-row values of the
// aggregation, RES[kc][h] = x_i[32 kc + 8 g + 4 h ..]) or, with CRES, is
// computed for the feature.
template <int NCB, bool CRES = false, bool LG = false, bool OPERM = false>
__device__ __forceinline__ void staged_epilogue(unsigned char* STG, const float* EV,
                                                const f32x4 (&acc)[NCB], int p, int flags,
                                                const float* __restrict__ x, int64_t ldx,
                                                float* __restrict__ out, int64_t ldo, int64_t t0,
                                                int64_t re, int wave, int lane, int lself, int g,
                                                const float* TB = nullptr, float c0 = 0.f,
                                                float c1 = 0.f, float c2 = 0.f,
                                                const float* WLN = nullptr,
                                                float* __restrict__ lgn = nullptr,
                                                const f32x4 (*RES)[2] = nullptr) {
    constexpr int N = NCB * 16, CPR = NCB * 4, ROWB = NCB * 64, RPI = 64 / CPR, NI = 16 / RPI;
    static_assert(!OPERM || (NCB == 16 && !LG), "gin_operm: H = 256");
    const bool res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    int l = lane;
    asm volatile("" : "+v"(l));
    const int ci = l % CPR, ri = l / CPR;
    if (res && !CRES && !OPERM) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if constexpr (RPI == 1) {          // one row per instruction: scalar row address
                int64_t rr = t0 + 16 * wave + i;
                if (rr >= re) rr = re - 1;
                glds16_ag(x + rr * ldx + 4 * (l ^ i), lds_addr_ag(STG + (16 * wave + i) * ROWB));
            } else {
                const int li = 16 * wave + RPI * i + ri;
                int64_t rr = t0 + li;
                if (rr >= re) rr = re - 1;
                glds16_ag(x + rr * ldx + 4 * (ci ^ (li & 15)), lds_addr_ag(STG + (16 * wave + RPI * i) * ROWB));
            }
        }
    }
    vm_barrier<0>();                           // (EV of every wave; this wave's rows landed)
    unsigned char* const srow = STG + lself * ROWB;
    const float spr = p2_ag(-p);               // the row's 2^-p (p in [-116, 100])
    float lp[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
        const int n = 16 * cb + 4 * g;
        const int nf = OPERM ? gin_operm(n) : n;          // the feature of accumulator n
        f32x4* const slot = reinterpret_cast<f32x4*>(srow + 16 * ((nf >> 2) ^ (lself & 15)));
        f32x4 xv = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (CRES) {
            if (res) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const f32x4 t = *reinterpret_cast<const f32x4*>(TB + 4 * (nf + i));
                    xv[i] = fmaf(t[2], c2, fmaf(t[1], c1, fmaf(t[0], c0, t[3])));
                }
            }
        } else if constexpr (OPERM) {
            if (res) xv = RES[cb >> 1][cb & 1];
        } else if (res) {
            xv = *slot;
        }
        const f32x4 sq = *reinterpret_cast<const f32x4*>(EV + n);
        const f32x4 bo = *reinterpret_cast<const f32x4*>(EV + N + n);
        const f32x4 so = *reinterpret_cast<const f32x4*>(EV + 2 * N + n);
        const f32x4 ho = *reinterpret_cast<const f32x4*>(EV + 3 * N + n);
        f32x4 o;
        // acc 2^-q exact (= the output 2^p), times 2^-p exact, + bias (0 when
        // the flag is off) rounded once: ldexp(acc, -(p + q)) + bias
#pragma unroll
        for (int i = 0; i < 4; ++i)
            o[i] = epilogue(fmaf(acc[cb][i] * sq[i], spr, bo[i]), flags & ~MIGNN_EPI_BIAS, 0.f,
                            xv[i], so[i], ho[i]);
        *slot = o;
    }
    if constexpr (LG) {
        // (a second pass over this lane's own staged values: the accumulators
        // are dead by now, which keeps the registers below the spill line)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const int n = 16 * cb + 4 * g;
            const f32x4 o = *reinterpret_cast<const f32x4*>(srow + 16 * ((4 * cb + g) ^ (lself & 15)));
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(WLN + q * N + n);
#pragma unroll
                for (int i = 0; i < 4; ++i) lp[q] = fmaf(o[i], w[i], lp[q]);
            }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) lp[q] = rowsum4(lp[q]);
        if (g == 0 && t0 + lself < re) {
            f32x4* const dst = reinterpret_cast<f32x4*>(lgn + (t0 + lself) * 8);
            dst[0] = f32x4{lp[0], lp[1], lp[2], lp[3]};
            dst[1] = f32x4{lp[4], lp[5], lp[6], lp[7]};
        }
    }
    // this wave's rows out (its own staging rows: in-order LDS)
    if constexpr (RPI == 1) {                  // ((16 wave + i) & 15 == i; the row is uniform)
        f32x4 v[NI];                           // (every read issued before the first store)
#pragma unroll
        for (int i = 0; i < NI; ++i)
            v[i] = *reinterpret_cast<const f32x4*>(STG + (16 * wave + i) * ROWB + l * 16);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int64_t rr = t0 + 16 * wave + i;
            if (rr < re)
                __builtin_nontemporal_store(v[i], reinterpret_cast<f32x4*>(out + rr * ldo + 4 * (l ^ i)));
        }
    } else {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int li = 16 * wave + RPI * i + ri;
            const f32x4 v = *reinterpret_cast<const f32x4*>(STG + li * ROWB + ci * 16);
            if (t0 + li < re)
                __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + (t0 + li) * ldo + 4 * (ci ^ (li & 15))));
        }
    }
}

// Block: 8 waves x 16 rows = a 128-row tile (two 4x4x4 blocks of the
// locality order), one block per CU (LDS 160 KB):
//   W ring   [2][32 KB]   the streamed W chunks (LDS-DMA, one chunk ahead)
//   own ring [3][16 KB]   chunk kc of the tile's own rows (LDS-DMA, two
//                         chunks ahead); 16-B segment s of local row li at
//                         position (s + li) & 7 (bank spread)
//   ext      [8][3][2][1 KB]  per wave: chunk kc of each row's out-of-tile
//                         neighbours, up to ES = 3 per row (LDS-DMA with
//                         per-lane addresses, one chunk ahead)
// Every load of the chunk loop is an LDS-DMA the compiler does not track, so
// the counted waits are exact: at the top of step kc everything but the own
// rows of chunk kc+1 (the youngest 2 pieces) must have landed.  A row whose
// first AS entries hold more than ES out-of-tile ones, or with more than AS
// entries, takes all its entries one at a time (correct, not fast).
// EPIF: the epilogue flags at compile time (the model's 15 / 11), -1: `flags`
template <int MODE, bool CHAIN, int EPIF = -1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void agg_gemm_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t rb,
    int64_t re, float self_scale, const unsigned char* __restrict__ img1,
    const float* __restrict__ b1, const unsigned char* __restrict__ img2,
    const float* __restrict__ b2, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    if constexpr (EPIF >= 0) flags = EPIF;
    constexpr int AW = 8, BM = 16 * AW;
    constexpr int NC = AKP * (CHAIN ? 2 : 1);          // W chunks streamed per tile
    constexpr int OWNB = BM * 128;                      // one own-row chunk slice
    constexpr int ES = 3;                               // out-of-tile slots per row
    constexpr int EXTB = ES * 2 * 1024;                 // per wave
    constexpr int OFF_OWN = 2 * ACHUNK;
    constexpr int OFF_EXT = OFF_OWN + 3 * OWNB;
    constexpr int LDS_BYTES = OFF_EXT + AW * EXTB;
    static_assert(LDS_BYTES <= 160 * 1024, "agg_gemm LDS");
    constexpr int WPC = ACHUNK / 1024 / AW;             // W pieces per wave per chunk (4)
    constexpr int OPC = OWNB / 1024 / AW;               // own-row pieces per wave per chunk (2)
    constexpr size_t FB = static_cast<size_t>(AKP) * ACB * 2 * AFRAG;   // image exponent table
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;

    // tile: each XCD takes a contiguous run of tiles (locality order: the
    // neighbour rows of a tile are the XCD's recent rows, in its L2)
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t per_xcd = gridDim.x >> 3;
    const int64_t tile = static_cast<int64_t>(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= ntiles) return;
    const int64_t t0 = rb + tile * BM;
    const int nloc = static_cast<int>(re - t0 < BM ? re - t0 : BM);
    const int64_t row = t0 + 16 * wave + r;
    const bool rv = row < re;
    const int64_t rowc = rv ? row : re - 1;
    const int lself = 16 * wave + r;

    // ---- LDS-DMA streams
    auto w_dma = [&](int c) {                  // W chunk c (W1's, then W2's) -> buffer c & 1
        if (c >= NC || (flags & MIGNN_SCHED_INTERLEAVED)) return;
        const unsigned char* src = c < AKP ? img1 + static_cast<size_t>(c) * ACHUNK
                                           : img2 + static_cast<size_t>(c - AKP) * ACHUNK;
        unsigned char* dst = lds + (c & 1) * ACHUNK;
#pragma unroll
        for (int pc = 0; pc < WPC; ++pc) {
            const int piece = wave + pc * AW;
            glds16_ag(src + piece * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
        }
    };
    auto own_dma = [&](int kc, int buf) {      // own rows' chunk kc -> ring buffer buf
        const int kk = kc < AKP ? kc : AKP - 1;    // (past the last chunk: a dummy refill
        unsigned char* dst = lds + OFF_OWN + buf * OWNB;   // of a free buffer: the count stays fixed)
        int l = lane;
        asm volatile("" : "+v"(l));
#pragma unroll
        for (int pc = 0; pc < OPC; ++pc) {
            const int piece = wave + pc * AW;
            const int li = 8 * piece + (l >> 3), sg = ((l & 7) - li) & 7;
            int64_t rr = t0 + li;
            if (rr >= re) rr = re - 1;                 // any valid row: never read
            glds16_ag(x + rr * ldx + 32 * kk + 4 * sg, lds_addr_ag(dst + piece * 1024));
        }
    };

    // ---- the row's CSR entries: per slot e < AS a code -- local row li (in
    // this tile), 256 + k (the row's k-th out-of-tile entry, column xc[k]),
    // -1 (empty); rows the slots cannot hold take the slow path
    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    int code[AS];
    float wgt[AS];
    int xc[ES];
#pragma unroll
    for (int k = 0; k < ES; ++k) xc[k] = -1;
    int next = 0;
    // (the slots' loads unconditional, past the row's end clamped to its last
    // entry -- values unused -- so no per-entry branch separates them)
    int cl[AS];
    float wl[AS];
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        const int ek = e0 + (e < deg ? e : (deg > 0 ? deg - 1 : 0));
        cl[e] = deg > 0 ? col[ek] : -1;
        wl[e] = (MODE == AGG_GCN && deg > 0) ? ew[ek] : 1.f;
    }
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        const int c = e < deg ? cl[e] : -1;
        // (GIN: weight 1 -- the sum as FMAs, so an empty slot is a weight-0
        // read of the row's own x_i, finite whenever the output is: no select)
        wgt[e] = e < deg ? wl[e] : 0.f;
        const uint32_t off = static_cast<uint32_t>(c - static_cast<int>(t0));
        if (c < 0) {
            code[e] = -1;
        } else if (off < static_cast<uint32_t>(nloc)) {
            code[e] = static_cast<int>(off);
        } else {
            code[e] = 256 + next;
#pragma unroll
            for (int k = 0; k < ES; ++k)
                if (k == next) xc[k] = c;
            ++next;
        }
    }
    const bool slow = deg > AS || next > ES;
    if (slow) {
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            code[e] = -1;
            wgt[e] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < ES; ++k) xc[k] = -1;
    }
    const bool any_slow = __builtin_amdgcn_ballot_w64(slow) != 0ull;
    // slots past every row's degree are skipped (a uniform branch)
    int maxdeg = 0;
#pragma unroll
    for (int e = 1; e <= AS; ++e)
        if (__builtin_amdgcn_ballot_w64(!slow && deg >= e) != 0ull) maxdeg = e;
    unsigned char* const EXT = lds + OFF_EXT + wave * EXTB;
    // (slots no row of the wave uses are skipped: only the own rows' refill,
    // issued last, is counted by the waits)
    bool xs_used[ES];
#pragma unroll
    for (int k = 0; k < ES; ++k) xs_used[k] = __builtin_amdgcn_ballot_w64(xc[k] >= 0) != 0ull;
    auto ext_dma = [&](int kc) {               // chunk kc of the row's out-of-tile entries
#pragma unroll
        for (int k = 0; k < ES; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!xs_used[k]) continue;
                const float* sp = xc[k] >= 0 ? x + static_cast<int64_t>(xc[k]) * ldx + 32 * kc + 8 * g + 4 * h
                                             : g_zero_row_ag + 32 * kc + 8 * g + 4 * h;
                glds16_ag(sp, lds_addr_ag(EXT + (2 * k + h) * 1024));
            }
    };

    own_dma(0, 0);
    own_dma(1, 1);
    w_dma(0);
    ext_dma(0);

    f32x4 acc[ACB];
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // GIN (chained, the nn.2 image in gin_operm order): the own row's values
    // of every chunk, the epilogue's residual
    constexpr bool OPERM = MODE == AGG_GIN && CHAIN;
    f32x4 resx[OPERM ? AKP : 1][2];
    int p = 100;                                   // the row's running exponent
    bool fresh = true;                             // (the row's first chunk not seen yet)
    const unsigned char* const wl0 = lds + lane * 16;

    // ---------------------------------------------------------------- transform 1
    // (not unrolled: the residual's register index is a select chain -- the
    // unrolled loop measured slower, 15.8 vs 15.0 ms per 12.6M-row layer)
#pragma unroll 1
    for (int kc = 0; kc < AKP; ++kc) {
        // chunk kc's W, own rows and out-of-tile rows landed (only the own rows
        // of chunk kc+1 may fly), every wave done with the buffers refilled below
        if (kc == 0) vm_barrier<0>();
        else vm_barrier<OPC>();
        w_dma(kc + 1);                             // into the buffer chunk kc-1 used
        const unsigned char* const ob = lds + OFF_OWN + (kc % 3) * OWNB;
        // the aggregate's 8 values of this chunk (CSR order)
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
        const bool dsum = !(flags & MIGNN_DIAG_NO_PRODUCE);
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            if (!dsum || e >= maxdeg) continue;   // (uniform)
            const int c = code[e];
            uint32_t ad0, ad1;                     // LDS byte offsets of the 2 x 16 B
            if (c >= 256) {
                ad0 = static_cast<uint32_t>(OFF_EXT + wave * EXTB + (2 * (c - 256)) * 1024 + lane * 16);
                ad1 = ad0 + 1024;
            } else {
                const int li = c < 0 ? lself : c;  // (empty: the own row, weight 0)
                const uint32_t rp = static_cast<uint32_t>(OFF_OWN + (kc % 3) * OWNB + li * 128);
                ad0 = rp + 16 * ((2 * g + li) & 7);
                ad1 = rp + 16 * ((2 * g + 1 + li) & 7);
            }
            const f32x4 v0 = *reinterpret_cast<const f32x4*>(lds + ad0);
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(lds + ad1);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0[i] = fmaf(wgt[e], v0[i], a0[i]);
                a1[i] = fmaf(wgt[e], v1[i], a1[i]);
            }
            if ((e & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        if (any_slow && slow) {
            // every entry of the row, one at a time (CSR order)
            for (int e = 0; e < deg; ++e) {
                const int c = col[e0 + e];
                const float w = MODE == AGG_GCN ? ew[e0 + e] : 1.f;
                const float* sp = x + static_cast<int64_t>(c) * ldx + 8 * g + 32 * kc;
                const f32x4 u0 = *reinterpret_cast<const f32x4*>(sp);
                const f32x4 u1 = *reinterpret_cast<const f32x4*>(sp + 4);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a0[i] = fmaf(w, u0[i], a0[i]);
                    a1[i] = fmaf(w, u1[i], a1[i]);
                }
            }
        }
        if constexpr (MODE == AGG_GIN) {
            const unsigned char* rp = ob + lself * 128;
            const f32x4 s0 = *reinterpret_cast<const f32x4*>(rp + 16 * ((2 * g + lself) & 7));
            const f32x4 s1 = *reinterpret_cast<const f32x4*>(rp + 16 * ((2 * g + 1 + lself) & 7));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0[i] = fmaf(self_scale, s0[i], a0[i]);
                a1[i] = fmaf(self_scale, s1[i], a1[i]);
            }
            if constexpr (OPERM) {
                // the residual of the epilogue (gin_operm order): kept, not re-read
#pragma unroll
                for (int k = 0; k < AKP; ++k)
                    if (k == kc) {
                        resx[k][0] = s0;
                        resx[k][1] = s1;
                    }
            }
        }
        // refills: this wave's out-of-tile rows of chunk kc+1 (its reads of
        // the ext buffer above are issued: an LDS-DMA does not overtake them),
        // the own rows of chunk kc+2 into the buffer chunk kc-1 used
        if (kc + 1 < AKP && !(flags & MIGNN_DIAG_NO_EXT)) ext_dma(kc + 1);
        if (!(flags & MIGNN_DIAG_NO_TABLES)) own_dma(kc + 2, (kc + 2) % 3);
        // split with the row's online exponent
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            m = max(m, max(__float_as_uint(fabsf(a0[i])), __float_as_uint(fabsf(a1[i]))));
        const int pc = sexp_ag(rowmax4(m));
        // the row's first nonzero chunk sets the scale with 2 bits of headroom
        // (accumulators still zero: nothing to rescale), so later chunks
        // rarely lower it; a lowering is a uniform branch, exact rescale
        if (fresh) p = pc - 2;
        if (!fresh && __builtin_amdgcn_ballot_w64(pc < p) != 0ull) {
            const int dp = pc < p ? pc - p : 0;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], dp);
            p = pc < p ? pc : p;
        }
        fresh = false;
        const float spv = p2_ag(p);
        f16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = (j < 4 ? a0[j] : a1[j - 4]) * spv;
            const _Float16 hh = static_cast<_Float16>(v);
            bh[j] = hh;
            bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
        }
        const unsigned char* wb = wl0 + (kc & 1) * ACHUNK;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            if (flags & MIGNN_DIAG_NO_MFMA) break;
            const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
            const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[cb], 0, 0, 0);
        }
    }

    if constexpr (CHAIN) {
        // ------------------------------------------------------------ transform 2
        // h = relu(acc 2^-(p + q1) + b1) in the accumulator layout: lane (r, g)
        // holds h[r][16 cb + 4 g + i]; one exponent per row over all 256
        const int32_t* const q1 = reinterpret_cast<const int32_t*>(img1 + FB);
        const float spr1 = p2_ag(-p);
        uint32_t m = 0;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            const int4 q = *reinterpret_cast<const int4*>(q1 + 16 * cb + 4 * g);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + 16 * cb + 4 * g);
            const int qn[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // (the staged epilogue's unscale; h >= +0 or NaN: its bits are the max key)
                const float h = __builtin_elementwise_maximum(
                    fmaf(acc[cb][i] * p2neg_ag(qn[i]), spr1, bb[i]), 0.f);
                acc[cb][i] = h;
                m = max(m, __float_as_uint(h));
            }
        }
        p = sexp_ag(rowmax4(m));
        const float spv = p2_ag(p);
        f16x8 hh[AKP], hl[AKP];
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = acc[2 * kc + (j >> 2)][j & 3] * spv;
                const _Float16 t = static_cast<_Float16>(v);
                hh[kc][j] = t;
                hl[kc][j] = static_cast<_Float16>(v - static_cast<float>(t));
            }
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc) {
            vm_barrier<0>();                       // W2 chunk kc landed
            w_dma(AKP + kc + 1);
            const unsigned char* wb = wl0 + ((AKP + kc) & 1) * ACHUNK;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb) {
                if (flags & MIGNN_DIAG_NO_MFMA) break;
                const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
                const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hh[kc], acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hl[kc], acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, hh[kc], acc[cb], 0, 0, 0);
            }
        }
    }

    // -------------------------------------------------------------------- epilogue
    // drain (no LDS-DMA may land after the loop: the dummy own-row refills),
    // then the whole LDS is free: staging rows [BM][1 KB] | epilogue vectors.
    // Each wave DMAs its 16 own rows in whole (the residual), every lane
    // replaces its 64 values -- rows r, columns 16 cb + 4 g + i: bias,
    // residual, BN, ReLU (gnn_model.py:184-191 order: conv + bias, + x, BN,
    // ReLU) -- in place, and the wave stores whole 1-KB rows (the accumulator
    // layout would store 16 rows x 64 B per instruction).  16-B chunk c of
    // staging row li at position c ^ (li & 15).
    vm_barrier<0>();
    const bool hb = (flags & MIGNN_EPI_BIAS) != 0, ha = (flags & MIGNN_EPI_AFFINE) != 0;
    if (flags & MIGNN_DIAG_NO_LOCAL) {         // (ablation: no epilogue)
        if (rv && acc[0][0] == 12345.f) out[rowc * ldo] = acc[1][1];
        return;
    }
    float* const EV = reinterpret_cast<float*>(lds + BM * 1024);   // q | bias | scale | shift
    if (tid < AH) {
        const int32_t* const qf = reinterpret_cast<const int32_t*>((CHAIN ? img2 : img1) + FB);
        const float* const bf = CHAIN ? b2 : b1;
        const int nf = OPERM ? gin_operm(tid) : tid;       // (EV by image column)
        EV[tid] = p2neg_ag(qf[tid]);
        EV[AH + tid] = hb ? bf[nf] : 0.f;
        EV[2 * AH + tid] = ha ? scale[nf] : 1.f;
        EV[3 * AH + tid] = ha ? shift[nf] : 0.f;
    }
    if constexpr (OPERM)
        staged_epilogue<ACB, false, false, true>(lds, EV, acc, p, flags, x, ldx, out, ldo, t0, re, wave,
                                                 lane, lself, g, nullptr, 0.f, 0.f, 0.f, nullptr,
                                                 nullptr, resx);
    else
        staged_epilogue<ACB>(lds, EV, acc, p, flags, x, ldx, out, ldo, t0, re, wave, lane, lself, g);
}

// GIN layer 0 at H = 256 from the coordinates (input_proj composed into the
// aggregate, as gcn_layer0.hip does for GCN): with x = pos W_in^T + b_in,
//   a_i = sum_j x_j + (1 + eps) x_i = W_in P_i + c_i b_in,
//   P_i = sum_j pos_j + (1 + eps) pos_i,  c_i = deg_i + 1 + eps,
// so the layer reads 12 B of coordinates per CSR entry instead of a 1-KB row,
// and input_proj's [N, 256] output is never written.  The chain (nn.0, ReLU,
// nn.2) and the epilogue are agg_gemm_kernel<AGG_GIN, true>'s; the residual
// x_i is recomputed from pos_i.  LDS: W ring [2][32 KB] | (epilogue: staging
// rows [128][1 KB] | q bias scale shift) | [W_in | b_in] table [256][4].
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void gin0_fused_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ pos, int64_t ldp, int D, int64_t rb, int64_t re, float self_scale,
    const float* __restrict__ w_in, const float* __restrict__ b_in,
    const unsigned char* __restrict__ img1, const float* __restrict__ b1,
    const unsigned char* __restrict__ img2, const float* __restrict__ b2,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo) {
    constexpr int AW = 8, BM = 16 * AW;
    constexpr int WPC = ACHUNK / 1024 / AW;
    constexpr size_t FB = static_cast<size_t>(AKP) * ACB * 2 * AFRAG;
    constexpr int OFF_EV = BM * 1024;
    constexpr int OFF_TB = OFF_EV + 4 * AH * 4;
    constexpr int LDS_BYTES = OFF_TB + AH * 16;
    static_assert(LDS_BYTES <= 160 * 1024, "gin0 LDS");
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t per_xcd = gridDim.x >> 3;
    const int64_t tile = static_cast<int64_t>(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= ntiles) return;
    const int64_t t0 = rb + tile * BM;
    const int64_t row = t0 + 16 * wave + r;
    const bool rv = row < re;
    const int64_t rowc = rv ? row : re - 1;
    const int lself = 16 * wave + r;

    // [W_in | b_in] -> LDS (ordinary loads, before the DMAs)
    float* const TB = reinterpret_cast<float*>(lds + OFF_TB);
    if (tid < AH) {
        f32x4 t;
#pragma unroll
        for (int d = 0; d < 3; ++d) t[d] = d < D ? w_in[tid * D + d] : 0.f;
        t[3] = b_in[tid];
        *reinterpret_cast<f32x4*>(TB + 4 * tid) = t;
    }
    auto w_dma = [&](int c) {                  // W1's chunks, then W2's -> buffer c & 1
        if (c >= 2 * AKP) return;
        const unsigned char* src = c < AKP ? img1 + static_cast<size_t>(c) * ACHUNK
                                           : img2 + static_cast<size_t>(c - AKP) * ACHUNK;
        unsigned char* dst = lds + (c & 1) * ACHUNK;
#pragma unroll
        for (int pc = 0; pc < WPC; ++pc) {
            const int piece = wave + pc * AW;
            glds16_ag(src + piece * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
        }
    };
    w_dma(0);

    // P_i (CSR order, then the self term) and c_i
    float pi[3], P[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) pi[d] = d < D ? pos[rowc * ldp + d] : 0.f;
    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    P[0] = P[1] = P[2] = 0.f;
    for (int e = 0; e < deg; ++e) {
        const int64_t j = col[e0 + e];
#pragma unroll
        for (int d = 0; d < 3; ++d) P[d] += d < D ? pos[j * ldp + d] : 0.f;
    }
#pragma unroll
    for (int d = 0; d < 3; ++d) P[d] = fmaf(self_scale, pi[d], P[d]);
    const float cnt = static_cast<float>(deg) + self_scale;

    f32x4 acc[ACB];
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p = 100;
    bool fresh = true;                             // (the row's first chunk not seen yet)
    const unsigned char* const wl0 = lds + lane * 16;
    auto mfma3 = [&](const unsigned char* wb, const f16x8& bh, const f16x8& bl) {
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
            const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[cb], 0, 0, 0);
        }
    };
    // ---- nn.0 over a = W_in P + c b_in, formed chunk by chunk in the B layout
#pragma unroll 1
    for (int kc = 0; kc < AKP; ++kc) {
        vm_barrier<0>();                       // W1 chunk kc landed (and the table, kc = 0)
        w_dma(kc + 1);
        float a[8];
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const f32x4 t = *reinterpret_cast<const f32x4*>(TB + 4 * (32 * kc + 8 * g + j));
            a[j] = fmaf(t[3], cnt, fmaf(t[2], P[2], fmaf(t[1], P[1], t[0] * P[0])));
            m = max(m, __float_as_uint(fabsf(a[j])));
        }
        const int pc = sexp_ag(rowmax4(m));
        // the row's first nonzero chunk sets the scale with 2 bits of headroom
        // (accumulators still zero: nothing to rescale), so later chunks
        // rarely lower it; a lowering is a uniform branch, exact rescale
        if (fresh) p = pc - 2;
        if (!fresh && __builtin_amdgcn_ballot_w64(pc < p) != 0ull) {
            const int dp = pc < p ? pc - p : 0;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], dp);
            p = pc < p ? pc : p;
        }
        fresh = false;
        const float spv = p2_ag(p);
        f16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = a[j] * spv;
            const _Float16 hh = static_cast<_Float16>(v);
            bh[j] = hh;
            bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
        }
        mfma3(wl0 + (kc & 1) * ACHUNK, bh, bl);
    }
    // ---- nn.2 over h = relu(acc 2^-(p + q1) + b1) from the accumulators (k-permuted W2)
    {
        const int32_t* const q1 = reinterpret_cast<const int32_t*>(img1 + FB);
        const float spr1 = p2_ag(-p);
        uint32_t m = 0;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            const int4 q = *reinterpret_cast<const int4*>(q1 + 16 * cb + 4 * g);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(b1 + 16 * cb + 4 * g);
            const int qn[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // (the staged epilogue's unscale; h >= +0 or NaN: its bits are the max key)
                const float h = __builtin_elementwise_maximum(
                    fmaf(acc[cb][i] * p2neg_ag(qn[i]), spr1, bb[i]), 0.f);
                acc[cb][i] = h;
                m = max(m, __float_as_uint(h));
            }
        }
        p = sexp_ag(rowmax4(m));
        const float spv = p2_ag(p);
        f16x8 hh[AKP], hl[AKP];
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = acc[2 * kc + (j >> 2)][j & 3] * spv;
                const _Float16 t = static_cast<_Float16>(v);
                hh[kc][j] = t;
                hl[kc][j] = static_cast<_Float16>(v - static_cast<float>(t));
            }
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc) {
            vm_barrier<0>();                   // W2 chunk kc landed
            w_dma(AKP + kc + 1);
            mfma3(wl0 + ((AKP + kc) & 1) * ACHUNK, hh[kc], hl[kc]);
        }
    }
    // ---- epilogue (staged; the residual x_i = W_in pos_i + b_in recomputed)
    vm_barrier<0>();
    const bool hb = (flags & MIGNN_EPI_BIAS) != 0, ha = (flags & MIGNN_EPI_AFFINE) != 0;
    float* const EV = reinterpret_cast<float*>(lds + OFF_EV);
    if (tid < AH) {
        const int nf = gin_operm(tid);         // (the nn.2 image's output order)
        EV[tid] = p2neg_ag(reinterpret_cast<const int32_t*>(img2 + FB)[tid]);
        EV[AH + tid] = hb ? b2[nf] : 0.f;
        EV[2 * AH + tid] = ha ? scale[nf] : 1.f;
        EV[3 * AH + tid] = ha ? shift[nf] : 0.f;
    }
    staged_epilogue<ACB, true, false, true>(lds, EV, acc, p, flags, nullptr, 0, out, ldo, t0, re, wave,
                                            lane, lself, g, TB, pi[0], pi[1], pi[2]);
}

// TransformerConv layer 0 from the coordinates (heads = 4, any H = 64 CPL):
// with x = pos W_in^T + b_in the whole layer collapses to 3-vectors.  The
// score's row term cancels in the softmax, so
//   s_ij^h = (G_h pos_i + g_h) . pos_j / sqrt(C)      (G_h = W_in^T M_h W_in, 3x3)
//   P_h = sum_j a_ij^h pos_j,  S_h = sum_j a_ij^h      (softmax + 1e-16)
//   out_i = relu( sum_h (A_h P_h + S_h e_h) + B pos_i + d )
// where A_h = Wv_h/heads W_in, e_h = Wv_h/heads b_in + bv_h/heads, B = W_skip
// W_in and d = W_skip b_in + b_skip, with the residual (+ W_in pos_i + b_in)
// and the BN affine folded in (host, fp64): 20 numbers per output column
// (T [H][20]), 12 per head (GT [4][12] = G_h | g_h).  No [N, H] input, no
// Q~K transform, no gathered feature row: ~26 FMAs per output value.
// Block: 4 waves; a wave takes 64 rows at a time -- lane l forms row l's
// P, S (online softmax over its CSR entries) into LDS, then the wave writes
// the 64 rows one by one, lane l owning columns CPL l .. CPL l + CPL - 1
// (table in registers).
// GAT = true: GATConv layer 0 in the same form -- scores LeakyReLU(ls_h .
// (pos_j, 1) + ld_h . (pos_i, 1)) from the composed logit weights (GT = lw
// [8][4] = [wlog W_in | wlog b_in]), A_h = Wcat_h W_in, e_h = Wcat_h b_in.
template <int CPL, bool GAT = false>
__global__ __launch_bounds__(256) void tf0_kernel(const int32_t* __restrict__ row_ptr,
                                                  const int32_t* __restrict__ col,
                                                  const float* __restrict__ pos, int64_t ldp,
                                                  int D, int64_t rb, int64_t re, float score_scale,
                                                  const float* __restrict__ T,
                                                  const float* __restrict__ GT, int relu,
                                                  float* __restrict__ out, int64_t ldo,
                                                  const float* __restrict__ wlog_next = nullptr,
                                                  float* __restrict__ lg_next = nullptr) {
    constexpr int HEADS = 4, NW = 4, SL = 20;
    // (GAT, lg_next given: each written row's next-layer logits, out . wlog_next^T,
    // summed over the wave's 64 lanes)
    const bool lgn = GAT && lg_next != nullptr;
    __shared__ __attribute__((aligned(16))) float slot[NW][64][SL];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    float tb[CPL][SL];
#pragma unroll
    for (int k = 0; k < CPL; ++k)
#pragma unroll
        for (int i = 0; i < SL; ++i) tb[k][i] = T[(lane * CPL + k) * SL + i];
    float wn[8][CPL];
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int k = 0; k < CPL; ++k) wn[q][k] = lgn ? wlog_next[q * (64 * CPL) + lane * CPL + k] : 0.f;
    const int64_t nb = (re - rb + 63) / 64;
    const int64_t groups = (nb + NW - 1) / NW;
    for (int64_t b = static_cast<int64_t>(blockIdx.x); b < groups; b += gridDim.x) {
        // (b indexes groups of NW batches: every wave of the block runs the
        // same number of iterations -- the __syncthreads below are uniform)
        const int64_t batch = b * NW + wave;
        const int64_t row = rb + batch * 64 + lane;
        // ---- lane = row: P_h, S_h
        if (row < re) {
            float pi[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) pi[d] = d < D ? pos[row * ldp + d] : 0.f;
            float u[HEADS][3], ub[HEADS];           // score = u . dpos (+ ub: GAT)
#pragma unroll
            for (int h = 0; h < HEADS; ++h) {
                if constexpr (GAT) {
                    // a_s[j] + a_d[i] = ls . dpos + (ls + ld) . (pos_i, 1)
                    const float* ls = GT + 4 * h;
                    const float* ld = GT + 4 * (HEADS + h);
#pragma unroll
                    for (int a = 0; a < 3; ++a) u[h][a] = ls[a];
                    ub[h] = fmaf(ls[2] + ld[2], pi[2], fmaf(ls[1] + ld[1], pi[1],
                                 fmaf(ls[0] + ld[0], pi[0], ls[3] + ld[3])));
                } else {
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        const float* gr = GT + h * 12 + 3 * a;
                        u[h][a] = (fmaf(gr[2], pi[2], fmaf(gr[1], pi[1], fmaf(gr[0], pi[0], GT[h * 12 + 9 + a])))) * score_scale;
                    }
                    ub[h] = 0.f;
                }
            }
            float m[HEADS], l[HEADS], P[HEADS][3];
#pragma unroll
            for (int h = 0; h < HEADS; ++h) {
                m[h] = -INFINITY;
                l[h] = 0.f;
                P[h][0] = P[h][1] = P[h][2] = 0.f;
            }
            const int e0 = row_ptr[row], e1 = row_ptr[row + 1];
            // (scores and sums on pos_j - pos_i: the softmax is shift-invariant and
            // the neighbour offsets are small, so neither loses precision to the
            // coordinates' magnitude; P_h = sum a (pos_j - pos_i) + S_h pos_i)
            for (int e = e0; e < e1; ++e) {
                const int64_t j = col[e];
                float pj[3];
#pragma unroll
                for (int d = 0; d < 3; ++d) pj[d] = d < D ? pos[j * ldp + d] - pi[d] : 0.f;
#pragma unroll
                for (int h = 0; h < HEADS; ++h) {
                    float sc = fmaf(u[h][2], pj[2], fmaf(u[h][1], pj[1], fmaf(u[h][0], pj[0], ub[h])));
                    if constexpr (GAT) sc = sc > 0.f ? sc : sc * score_scale;   // LeakyReLU(slope)
                    const float mn = fmaxf(m[h], sc);
                    const float corr = m[h] == -INFINITY ? 0.f : expf(m[h] - mn);
                    const float w = expf(sc - mn);
                    l[h] = fmaf(l[h], corr, w);
#pragma unroll
                    for (int d = 0; d < 3; ++d) P[h][d] = fmaf(P[h][d], corr, w * pj[d]);
                    m[h] = mn;
                }
            }
            float* const sl = slot[wave][lane];
#pragma unroll
            for (int h = 0; h < HEADS; ++h) {
                const float inv = 1.f / (l[h] + 1e-16f);
                const float S = l[h] * inv;
#pragma unroll
                for (int d = 0; d < 3; ++d) sl[3 * h + d] = fmaf(S, pi[d], P[h][d] * inv);
                sl[12 + h] = S;
            }
#pragma unroll
            for (int d = 0; d < 3; ++d) sl[16 + d] = pi[d];
        }
        __syncthreads();
        // ---- the wave's 64 rows, lane = CPL columns
        const int64_t rows = re - (rb + batch * 64) < 64 ? re - (rb + batch * 64) : 64;
        for (int rr = 0; rr < rows; ++rr) {
            const float* const sl = slot[wave][rr];
            float v[SL - 1];
#pragma unroll
            for (int i = 0; i < SL - 1; ++i) v[i] = sl[i];
            float o[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                float acc = tb[k][19];
#pragma unroll
                for (int i = 0; i < 19; ++i) acc = fmaf(tb[k][i], v[i], acc);
                o[k] = relu ? fmaxf(acc, 0.f) : acc;
            }
            float* const dst = out + (rb + batch * 64 + rr) * ldo + lane * CPL;
            if constexpr (CPL == 4) {
                __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(dst));
            } else {
#pragma unroll
                for (int k = 0; k < CPL; ++k) dst[k] = o[k];
            }
            if (lgn) {
                float lq[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < CPL; ++k) a = fmaf(o[k], wn[q][k], a);
#pragma unroll
                    for (int sh = 32; sh > 0; sh >>= 1) a += __shfl_xor(a, sh);
                    lq[q] = a;
                }
                if (lane == 0) {
                    f32x4* const ld = reinterpret_cast<f32x4*>(lg_next + (rb + batch * 64 + rr) * 8);
                    ld[0] = f32x4{lq[0], lq[1], lq[2], lq[3]};
                    ld[1] = f32x4{lq[4], lq[5], lq[6], lq[7]};
                }
            }
        }
        __syncthreads();
    }
}

#ifdef MIGNN_DIAG
int g_fused_diag_flags = 0;   // mignn_diag_set_fused_flags (timing ablations; wrong results)
#else
constexpr int g_fused_diag_flags = 0;   // the product library has no ablation state
#endif

// k-permuted split image of W2 [256, 256] for the chained transform: element
// j of lane (m, g) in fragment (kc, cb) = W2[16 cb + m][16 (2 kc + j / 4) +
// 4 g + j % 4] * 2^q (q per output column, as gprep_exp_kernel); layout and
// exponent table as mignn_linear_f16x3_prep's image
// (n <= 256 output columns; columns past n are zero, exponent 100)
__global__ __launch_bounds__(256) void perm_exp_kernel(const float* __restrict__ w, int n,
                                                       int32_t* __restrict__ q, bool operm) {
    const int colm = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int src = operm ? gin_operm(colm) : colm;   // the W row image column colm holds
    uint32_t m = 0;
    if (colm < n)
        for (int i = lane; i < AH; i += 64) m = max(m, __float_as_uint(fabsf(w[src * AH + i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o)));
    if (lane == 0) q[colm] = sexp_ag(m);
}
__global__ __launch_bounds__(256) void perm_frag_kernel(const float* __restrict__ w, int n,
                                                        const int32_t* __restrict__ q,
                                                        unsigned char* __restrict__ img, bool operm) {
    const int t = blockIdx.x * 256 + threadIdx.x;   // (kc, cb, lane)
    if (t >= AKP * ACB * 64) return;
    const int lane = t & 63;
    const int cb = (t >> 6) % ACB;
    const int kc = (t >> 6) / ACB;
    const int colm = 16 * cb + (lane & 15);
    const int src = operm ? gin_operm(colm) : colm;
    const int gq = lane >> 4;
    const float sc = p2_ag(q[colm]);
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = 16 * (2 * kc + (j >> 2)) + 4 * gq + (j & 3);
        const float v = colm < n ? w[src * AH + kk] * sc : 0.f;
        const _Float16 hh = static_cast<_Float16>(v);
        h[j] = hh;
        l[j] = static_cast<_Float16>(v - static_cast<float>(hh));
    }
    unsigned char* base = img + ((static_cast<size_t>(kc) * ACB + cb) * 2) * AFRAG + lane * 16;
    *reinterpret_cast<f16x8*>(base) = h;
    *reinterpret_cast<f16x8*>(base + AFRAG) = l;
}

// k-permuted image of W [n <= 256, 256] (layout of mignn_linear_f16x3_prep's
// image, 16 column blocks, exponent table after the fragments)
// operm: output columns in gin_operm order (n = 256; the GIN nn.2 image)
int perm_prep(const float* w, int n, unsigned char* img, hipStream_t st, bool operm = false) {
    int32_t* q = reinterpret_cast<int32_t*>(img + static_cast<size_t>(AKP) * ACB * 2 * AFRAG);
    hipLaunchKernelGGL(perm_exp_kernel, dim3(AH / 4), dim3(256), 0, st, w, n, q, operm);
    int rc = launch_status("perm_exp_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(perm_frag_kernel, dim3((AKP * ACB * 64 + 255) / 256), dim3(256), 0, st, w, n,
                       q, img, operm);
    return launch_status("perm_frag_kernel");
}

// ------------------------------------------------------------------ H = 256 output head
// output_proj at H = 256 (gnn_model.py:90-100, :195; configs[3] / configs[4]):
//   out = W4 relu(W3 relu(W2 relu(W1 x + b1) + b2) + b3) + b4,
//   W1, W2 [256, 256], W3 [128, 256], W4 [out_dim <= 8, 128]
// in one launch: per wave 16 rows; the three wide transforms in split-fp16
// MFMA arithmetic chained through the accumulators (transforms 2 and 3 take
// the previous one's relu'd accumulator as their B operand, with k-permuted
// images -- §3.13 of DESIGN.md), W chunks streamed through LDS; the last
// layer (128 -> out_dim) in fp32 VALU from the accumulators, its dot products
// summed over the row's 4 lanes.  The three [N, 256 | 128] intermediates of
// the launch sequence never reach memory.
// Image: W1 (linear_f16x3 image) | W2 (k-permuted) | W3 (k-permuted, 128
// columns in 16 padded blocks) | b1 b2 b3 b4 (fp32, 4 KB) | W4 [8][128] fp32.
constexpr size_t HIMG = static_cast<size_t>(AKP) * ACB * 2 * AFRAG + AH * 4;   // one W image
constexpr size_t HOFF_B = 3 * HIMG;
constexpr size_t HOFF_W4 = HOFF_B + 4096;
constexpr size_t HEAD256_BYTES = HOFF_W4 + 8 * 128 * 4;

__global__ __launch_bounds__(256) void head256_vec_kernel(const float* __restrict__ b1,
                                                          const float* __restrict__ b2,
                                                          const float* __restrict__ b3,
                                                          const float* __restrict__ w4,
                                                          const float* __restrict__ b4, int out_dim,
                                                          unsigned char* __restrict__ img) {
    float* bv = reinterpret_cast<float*>(img + HOFF_B);
    float* w = reinterpret_cast<float*>(img + HOFF_W4);
    for (int i = threadIdx.x; i < 256; i += 256) {
        bv[i] = b1[i];
        bv[256 + i] = b2[i];
        if (i < 128) bv[512 + i] = b3[i];
        if (i < 8) bv[640 + i] = i < out_dim ? b4[i] : 0.f;
    }
    for (int i = threadIdx.x; i < 8 * 128; i += 256) w[i] = (i / 128) < out_dim ? w4[i] : 0.f;
}

// Block: 8 waves x 16 rows; W chunks through a 2-buffer LDS ring (LDS-DMA one
// chunk ahead, one barrier per chunk), x rows one chunk ahead in registers.
// (A 3-deep W ring with x by LDS-DMA and counted waits measured slower: 13.7
// vs 13.0 ms at 12.6M rows.)
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void head256_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t n, const unsigned char* __restrict__ img,
    int out_dim, float* __restrict__ out, int64_t ldo, const int32_t* __restrict__ out_rows) {
    constexpr int AW = 8, BM = 16 * AW;
    constexpr int NC = 3 * AKP;                          // W1, W2, W3 chunks
    constexpr int OFF_V = 2 * ACHUNK;                    // b1 b2 b3 b4 | W4 copies
    __shared__ __attribute__((aligned(16))) unsigned char lds[OFF_V + 4096 + 8 * 128 * 4];
    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    // the two waves of a SIMD at different priorities (the barrier per W
    // chunk puts them in the same phase): 13.06 -> 12.55 ms at 12.6M rows
    // (no gain in agg_gemm_kernel / the H = 128 head)
    if (wave < AW / 2) __builtin_amdgcn_s_setprio(1);
    const int64_t ntiles = (n + BM - 1) / BM;
    const int64_t per_xcd = gridDim.x >> 3;
    const int64_t tile = static_cast<int64_t>(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= ntiles) return;
    const int64_t row = tile * BM + 16 * wave + r;
    const bool rv = row < n;
    const int64_t rowc = rv ? row : n - 1;

    // W chunk c: transform c / 8, k chunk c % 8 (W3: its 8 real column blocks only)
    auto w_dma = [&](int c) {
        if (c >= NC) return;
        const int t = c / AKP, kc = c % AKP;
        const unsigned char* src = img + t * HIMG + static_cast<size_t>(kc) * ACHUNK;
        unsigned char* dst = lds + (c & 1) * ACHUNK;
        const int npieces = t == 2 ? ACHUNK / 2 / 1024 : ACHUNK / 1024;
        for (int piece = wave; piece < npieces; piece += AW)
            glds16_ag(src + piece * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
    };
    w_dma(0);
    // biases and W4 -> LDS (read after the first barrier)
    for (int i = tid; i < (4096 + 8 * 128 * 4) / 16; i += AW * 64)
        reinterpret_cast<f32x4*>(lds + OFF_V)[i] = reinterpret_cast<const f32x4*>(img + HOFF_B)[i];
    const float* const BV = reinterpret_cast<const float*>(lds + OFF_V);
    const float* const W4 = reinterpret_cast<const float*>(lds + OFF_V + 4096);

    // x chunk kc of the row (B-operand layout), one chunk ahead in registers
    const float* const xrow = x + rowc * ldx + 8 * g;
    f32x4 xa[2], xb[2];
    xa[0] = *reinterpret_cast<const f32x4*>(xrow);
    xa[1] = *reinterpret_cast<const f32x4*>(xrow + 4);

    f32x4 acc[ACB];
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p = 100;
    bool fresh = true;                             // (the row's first chunk not seen yet)
    const unsigned char* const wl0 = lds + lane * 16;
    auto mfma3 = [&](const unsigned char* wb, int ncb, const f16x8& bh, const f16x8& bl) {
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            if (cb >= ncb) break;
            const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
            const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[cb], 0, 0, 0);
        }
    };
    // ---- transform 1: x W1^T, A split chunk by chunk with the online exponent
    auto step1 = [&](int kc, f32x4 (&cur)[2], f32x4 (&nxt)[2]) {
        chunk_barrier();                       // W1 chunk kc and x chunk kc landed
        w_dma(kc + 1);
        if (kc + 1 < AKP) {
            nxt[0] = *reinterpret_cast<const f32x4*>(xrow + 32 * (kc + 1));
            nxt[1] = *reinterpret_cast<const f32x4*>(xrow + 32 * (kc + 1) + 4);
        }
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            m = max(m, max(__float_as_uint(fabsf(cur[0][i])), __float_as_uint(fabsf(cur[1][i]))));
        const int pc = sexp_ag(rowmax4(m));
        // the row's first nonzero chunk sets the scale with 2 bits of headroom
        // (accumulators still zero: nothing to rescale), so later chunks
        // rarely lower it; a lowering is a uniform branch, exact rescale
        if (fresh) p = pc - 2;
        if (!fresh && __builtin_amdgcn_ballot_w64(pc < p) != 0ull) {
            const int dp = pc < p ? pc - p : 0;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], dp);
            p = pc < p ? pc : p;
        }
        fresh = false;
        const float spv = p2_ag(p);
        f16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = cur[j >> 2][j & 3] * spv;
            const _Float16 hh = static_cast<_Float16>(v);
            bh[j] = hh;
            bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
        }
        mfma3(wl0 + (kc & 1) * ACHUNK, ACB, bh, bl);
    };
#pragma unroll 1
    for (int kc = 0; kc < AKP; kc += 2) {
        step1(kc, xa, xb);
        step1(kc + 1, xb, xa);
    }
    // ---- transforms 2 and 3 from the relu'd accumulators (k-permuted images)
    f16x8 hh[AKP], hl[AKP];
    auto relu_split = [&](int t, int ncb, const float* bias) {
        const int32_t* const q = reinterpret_cast<const int32_t*>(img + t * HIMG + HIMG - AH * 4);
        const float spr1 = p2_ag(-p);
        uint32_t m = 0;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            if (cb >= ncb) break;
            const int4 qv = *reinterpret_cast<const int4*>(q + 16 * cb + 4 * g);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + 16 * cb + 4 * g);
            const int qn[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                // (the staged epilogue's unscale; h >= +0 or NaN: its bits are the max key)
                const float h = __builtin_elementwise_maximum(
                    fmaf(acc[cb][i] * p2neg_ag(qn[i]), spr1, bb[i]), 0.f);
                acc[cb][i] = h;
                m = max(m, __float_as_uint(h));
            }
        }
        p = sexp_ag(rowmax4(m));
        const float spv = p2_ag(p);
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = acc[2 * kc + (j >> 2)][j & 3] * spv;
                const _Float16 t16 = static_cast<_Float16>(v);
                hh[kc][j] = t16;
                hl[kc][j] = static_cast<_Float16>(v - static_cast<float>(t16));
            }
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    relu_split(0, ACB, BV);                          // h1 = relu(x W1^T + b1)
#pragma unroll
    for (int kc = 0; kc < AKP; ++kc) {
        chunk_barrier();
        w_dma(AKP + kc + 1);
        mfma3(wl0 + ((AKP + kc) & 1) * ACHUNK, ACB, hh[kc], hl[kc]);
    }
    relu_split(1, ACB, BV + 256);                    // h2 = relu(h1 W2^T + b2)
#pragma unroll
    for (int kc = 0; kc < AKP; ++kc) {
        chunk_barrier();
        w_dma(2 * AKP + kc + 1);
        mfma3(wl0 + ((2 * AKP + kc) & 1) * ACHUNK, ACB / 2, hh[kc], hl[kc]);
    }
    // ---- h3 = relu(h2 W3^T + b3): lane (r, g) holds h3[r][16 cb + 4 g + i], cb < 8;
    // out[r][o] = sum_k h3[k] W4[o][k] + b4[o] (fp32; summed over the row's 4 lanes)
    const int32_t* const q3 = reinterpret_cast<const int32_t*>(img + 2 * HIMG + HIMG - AH * 4);
    float h3[ACB / 2][4];
#pragma unroll
    for (int cb = 0; cb < ACB / 2; ++cb) {
        const int4 qv = *reinterpret_cast<const int4*>(q3 + 16 * cb + 4 * g);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(BV + 512 + 16 * cb + 4 * g);
        const int qn[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float h = ldexpf(acc[cb][i], -(p + qn[i])) + bb[i];
            h3[cb][i] = relu_nan(h);
        }
    }
    float o[8];
#pragma unroll
    for (int oc = 0; oc < 8; ++oc) {
        float sacc = 0.f;
        if (oc < out_dim) {
#pragma unroll
            for (int cb = 0; cb < ACB / 2; ++cb) {
                const f32x4 wv = *reinterpret_cast<const f32x4*>(W4 + oc * 128 + 16 * cb + 4 * g);
#pragma unroll
                for (int i = 0; i < 4; ++i) sacc = fmaf(h3[cb][i], wv[i], sacc);
            }
            sacc = rowsum4(sacc) + BV[640 + oc];
        }
        o[oc] = sacc;
    }
    if (rv && g == 0) {
        const int64_t orow = out_rows != nullptr ? static_cast<int64_t>(out_rows[row]) : row;
#pragma unroll
        for (int oc = 0; oc < 8; ++oc)
            if (oc < out_dim) out[orow * ldo + oc] = o[oc];
    }
}

// ------------------------------------------------------------------ GATConv
// Fused GAT layer (gnn_model.py:65-68; heads = 4, concat=False; H in {64, 128}):
//   alpha_ijk = softmax_j( LeakyReLU(a_s[j][k] + a_d[i][k]) )   (+1e-16, PyG utils.softmax)
//   out_i     = epi( sum_k (sum_j alpha_ijk x_j) Wcat_k^T + b; residual x_i, BN, ReLU )
// with the logits a_s | a_d = x wlog^T precomputed ([n, 8], mignn_gat_layer)
// and Wcat_k = W_k / heads (the head-mean folded into the weights): the
// per-head aggregates [rows, 4H] never reach memory.  Per wave 16 rows; lane
// (r, g) first owns head g of row r (scores, max, sum of exp, alphas -> LDS,
// then every lane reads its row's 32 alphas), then per 32-column x chunk it
// gathers its 8 columns of the row's neighbours once and forms the 4 heads'
// weighted sums -- the B operands of W chunks (head k, chunk c) -- split with
// the row's online exponent, 3 MFMAs per 16x16x32 block.  The 4 W chunks of
// an x chunk (4 x H/16 column blocks of the linear_f16x3 image of Wcat
// [H, 4H]) are LDS-DMA'd together (double-buffered where the LDS budget of
// two blocks per CU allows it: H = 64; H = 128 refills its one buffer after
// the step's MFMAs), one barrier per x chunk.
#ifndef GAT_AW
#define GAT_AW 4
#endif
template <int H>
struct GatCfg {
    static_assert(H == 64 || H == 128, "gat_fused: H in {64, 128}");
    // 4 waves x 16 rows per block, two blocks per CU: one block's dependent
    // CSR -> logit -> row loads run under the other's MFMAs (8 waves x 16
    // rows, one block per CU: 1.10 ms per 1M-node H = 128 layer)
    static constexpr int AW = GAT_AW, NT = AW * 64, BM = 16 * AW;
    static constexpr int NCB = H / 16;                 // output column blocks (N = H)
    static constexpr int XC = H / 32;                  // x chunks
    static constexpr int NPB = 16;                     // column blocks per image chunk (padded)
    static constexpr int WCH = NCB * 2 * AFRAG;        // real bytes of one W chunk
    static constexpr int REST = AW * 16 * 4 * 8 * 4 + AW * 16 * 4 * 8 + 4 * H * 4 + H * 16;
    // W steps: the 4 heads' chunks of one x chunk, double-buffered (the next
    // step's chunks DMA'd under this step's MFMAs) -- or, where two such
    // buffers leave no room for a second block on the CU (H = 128, 4 waves),
    // 2 heads per step, two steps per x chunk (round 5 kept ONE 4-head buffer
    // there, refilled after the chunk's MFMAs: every refill's latency exposed)
    static constexpr int HPS = (AW == 4 && 2 * 4 * WCH + REST > 80 * 1024) ? 2 : 4;
    static constexpr int NG = 4 / HPS;                  // W steps per x chunk
    static constexpr int NSTEP = XC * NG;
    static constexpr int STEPW = HPS * WCH;             // bytes of one W step
    static constexpr int WB = 2;
    static constexpr int OFF_AL = WB * STEPW;          // alphas [AW][16][4][8]
    static constexpr int OFF_ST = OFF_AL + AW * 16 * 4 * 8 * 4;   // (max, sum) [AW][16][4]
    static constexpr int OFF_EPI = OFF_ST + AW * 16 * 4 * 8;       // QF | BF | SC | SH [H]
    static constexpr int OFF_TB = OFF_EPI + 4 * H * 4;  // (layer 0) [W_in | b_in] [H][4]
    static constexpr int LDS_BYTES = OFF_TB + H * 16;
    static_assert(LDS_BYTES <= 160 * 1024, "gat_fused LDS");
};

// L0 (layer 0 from the coordinates, x = pos W_in^T + b_in never formed): the
// logits come from pos through the composed [wlog W_in | wlog b_in] (lw [8][4]),
// every lane forms its row's 4 heads' P = sum_j alpha_j pos_j and S = sum_j
// alpha_j in registers, and every chunk's weighted sums are W_in[c] . P +
// S b_in[c] -- no row gathers; the residual is recomputed from pos_i in the
// epilogue.  (A first form had lane g compute head g only and pass P, S to
// the row's other lanes through LDS: it gave wrong rows in waves 4-7 of some
// tiles, run to run, with or without extra barriers; the register form is
// exact and deterministic.)
template <int H, bool L0 = false, bool LG = false, int EPIF = -1>
__global__ __launch_bounds__(GatCfg<H>::NT) __attribute__((amdgpu_waves_per_eu(2))) void
gat_fused_kernel(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                 const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx,
                 int64_t rb, int64_t re, float slope, const unsigned char* __restrict__ img,
                 const float* __restrict__ bias, const float* __restrict__ scale,
                 const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo,
                 const float* __restrict__ w_in = nullptr, const float* __restrict__ b_in = nullptr,
                 const float* __restrict__ lw = nullptr, int D = 0,
                 const float* __restrict__ wlog_next = nullptr, float* __restrict__ lg_next = nullptr) {
    using C = GatCfg<H>;
    constexpr int HEADS = 4;
    if constexpr (EPIF >= 0) flags = EPIF;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    int32_t* const QF = reinterpret_cast<int32_t*>(lds + C::OFF_EPI);
    float* const BF = reinterpret_cast<float*>(QF + H);
    float* const SC = BF + H;
    float* const SH = SC + H;

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int64_t ntiles = (re - rb + C::BM - 1) / C::BM;
    const int64_t per_xcd = gridDim.x >> 3;
    const int64_t tile = static_cast<int64_t>(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= ntiles) return;
    const int64_t row = rb + tile * C::BM + 16 * wave + r;
    const bool rv = row < re;
    const int64_t rowc = rv ? row : re - 1;

    // W step j (x chunk j / NG, heads (j % NG) HPS .. + HPS - 1: image chunks
    // k XC + t) -> buffer j & 1
    auto w_dma = [&](int j) {
        if (j >= C::NSTEP || (flags & MIGNN_SCHED_INTERLEAVED)) return;
        const int t = j / C::NG, k0 = (j % C::NG) * C::HPS;
        unsigned char* dst = lds + (j & 1) * C::STEPW;
#pragma unroll
        for (int pc = 0; pc < C::STEPW / 1024 / C::AW; ++pc) {
            const int piece = wave + pc * C::AW;              // 1-KB piece of the step
            const int hd = k0 + piece / (C::WCH / 1024), q = piece % (C::WCH / 1024);
            const unsigned char* src = img + static_cast<size_t>(hd * C::XC + t) * C::NPB * 2 * AFRAG;
            glds16_ag(src + q * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
        }
    };
    w_dma(0);
    if (tid < H) {
        const int32_t* q = reinterpret_cast<const int32_t*>(
            img + static_cast<size_t>(4 * C::XC) * C::NPB * 2 * AFRAG);
        QF[tid] = q[tid];
        BF[tid] = (flags & MIGNN_EPI_BIAS) ? bias[tid] : 0.f;
        SC[tid] = (flags & MIGNN_EPI_AFFINE) ? scale[tid] : 1.f;
        SH[tid] = (flags & MIGNN_EPI_AFFINE) ? shift[tid] : 0.f;
    }
    float* const TB = reinterpret_cast<float*>(lds + C::OFF_TB);
    if constexpr (L0) {
        if (tid < H) {
            f32x4 t;
#pragma unroll
            for (int d = 0; d < 3; ++d) t[d] = d < D ? w_in[tid * D + d] : 0.f;
            t[3] = b_in[tid];
            *reinterpret_cast<f32x4*>(TB + 4 * tid) = t;
        }
    }

    // ---- CSR slots, scores of head g, softmax statistics, alphas
    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    int cj[AS];
    // (the slots' loads unconditional -- past the row's end clamped to its
    // last entry, values unused -- so the chain CSR -> logit -> row has no
    // per-entry branches between its loads)
    if (deg > 0) {
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            const int cv = col[e0 + (e < deg ? e : deg - 1)];
            cj[e] = e < deg ? cv : -1;
        }
    } else {
#pragma unroll
        for (int e = 0; e < AS; ++e) cj[e] = -1;
    }
    const bool extra = __builtin_amdgcn_ballot_w64(deg > AS) != 0ull;
    auto leaky = [&](float v) { return v > 0.f ? v : v * slope; };
    float* const AL = reinterpret_cast<float*>(lds + C::OFF_AL) + ((wave * 16 + r) * 4) * 8;
    float pi[3] = {0.f, 0.f, 0.f};
    f32x4 PSK[HEADS];                          // (L0) per head: P = sum alpha pos_j | S = sum alpha
    if constexpr (L0) {
        // logits from the coordinates; every lane forms all 4 heads' P and S
#pragma unroll
        for (int d = 0; d < 3; ++d) pi[d] = d < D ? x[rowc * ldx + d] : 0.f;
        auto posj = [&](int j, float (&pj)[3]) {
#pragma unroll
            for (int d = 0; d < 3; ++d) pj[d] = d < D ? x[static_cast<int64_t>(j) * ldx + d] : 0.f;
        };
        float pj[AS][3];
#pragma unroll
        for (int e = 0; e < AS; ++e) posj(cj[e] >= 0 ? cj[e] : 0, pj[e]);
#pragma unroll
        for (int k = 0; k < HEADS; ++k) {
            const f32x4 ls = *reinterpret_cast<const f32x4*>(lw + 4 * k);
            const f32x4 ld = *reinterpret_cast<const f32x4*>(lw + 4 * (HEADS + k));
            const float ad0 = fmaf(ld[2], pi[2], fmaf(ld[1], pi[1], fmaf(ld[0], pi[0], ld[3])));
            auto score = [&](const float (&q)[3]) {
                return leaky(fmaf(ls[2], q[2], fmaf(ls[1], q[1], fmaf(ls[0], q[0], ls[3]))) + ad0);
            };
            float sc0[AS];
            float mx0 = -INFINITY;
#pragma unroll
            for (int e = 0; e < AS; ++e) {
                sc0[e] = cj[e] >= 0 ? score(pj[e]) : -INFINITY;
                mx0 = fmaxf(mx0, sc0[e]);
            }
            if (extra)
                for (int e = AS; e < deg; ++e) {
                    float q[3];
                    posj(col[e0 + e], q);
                    mx0 = fmaxf(mx0, score(q));
                }
            float sm0 = 0.f;
#pragma unroll
            for (int e = 0; e < AS; ++e)
                if (cj[e] >= 0) sm0 += expf(sc0[e] - mx0);
            if (extra)
                for (int e = AS; e < deg; ++e) {
                    float q[3];
                    posj(col[e0 + e], q);
                    sm0 += expf(score(q) - mx0);
                }
            sm0 += 1e-16f;
            f32x4 PS = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < AS; ++e) {
                if (cj[e] < 0) continue;
                const float a = expf(sc0[e] - mx0) / sm0;
#pragma unroll
                for (int d = 0; d < 3; ++d) PS[d] = fmaf(a, pj[e][d], PS[d]);
                PS[3] += a;
            }
            if (extra)
                for (int e = AS; e < deg; ++e) {
                    float q[3];
                    posj(col[e0 + e], q);
                    const float a = expf(score(q) - mx0) / sm0;
#pragma unroll
                    for (int d = 0; d < 3; ++d) PS[d] = fmaf(a, q[d], PS[d]);
                    PS[3] += a;
                }
            PSK[k] = PS;
        }
    }
    const float ad = L0 ? 0.f : logits[rowc * (2 * HEADS) + HEADS + g];
    float sc[AS];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        if constexpr (L0) break;
        const float lv = logits[static_cast<int64_t>(cj[e] >= 0 ? cj[e] : rowc) * (2 * HEADS) + g];
        sc[e] = cj[e] >= 0 ? leaky(lv + ad) : -INFINITY;
        mx = fmaxf(mx, sc[e]);
    }
    if (extra && !L0)
        for (int e = AS; e < deg; ++e)
            mx = fmaxf(mx, leaky(logits[static_cast<int64_t>(col[e0 + e]) * (2 * HEADS) + g] + ad));
    float sm = 0.f;
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        if constexpr (L0) break;
        if (cj[e] >= 0) sm += expf(sc[e] - mx);
    }
    if (extra && !L0)
        for (int e = AS; e < deg; ++e)
            sm += expf(leaky(logits[static_cast<int64_t>(col[e0 + e]) * (2 * HEADS) + g] + ad) - mx);
    sm += 1e-16f;
    float* const ST = reinterpret_cast<float*>(lds + C::OFF_ST) + ((wave * 16 + r) * 4) * 2;
    if constexpr (!L0) {
        f32x4 a0, a1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            a0[e] = cj[e] >= 0 ? expf(sc[e] - mx) / sm : 0.f;
            a1[e] = cj[e + 4] >= 0 ? expf(sc[e + 4] - mx) / sm : 0.f;
        }
        *reinterpret_cast<f32x4*>(AL + g * 8) = a0;
        *reinterpret_cast<f32x4*>(AL + g * 8 + 4) = a1;
        ST[g * 2] = mx;
        ST[g * 2 + 1] = sm;
    }
    f32x4 gv[AS][2];
    // (row addresses recomputed per chunk from the 32-bit columns: 64-bit
    // pointers held across the loop cost 16 registers)
    auto gather = [&](int t) {
        if constexpr (L0) return;
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            const float* sp = cj[e] >= 0 ? x + static_cast<int64_t>(cj[e]) * ldx + 8 * g + 32 * t
                                         : g_zero_row_ag + 8 * g + 32 * t;
            gv[e][0] = *reinterpret_cast<const f32x4*>(sp);
            gv[e][1] = *reinterpret_cast<const f32x4*>(sp + 4);
        }
    };
    gather(0);
    f32x4 acc[C::NCB];
#pragma unroll
    for (int cb = 0; cb < C::NCB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p = 100;
    bool fresh = true;                             // (the row's first chunk not seen yet)
    const unsigned char* const wl0 = lds + lane * 16;

#pragma unroll 1
    for (int t = 0; t < C::XC; ++t) {
        chunk_barrier();                           // W step t NG and this chunk's rows landed
        w_dma(t * C::NG + 1);
        // the 4 heads' weighted sums of this x chunk (CSR order)
        f32x4 a[HEADS][2];
#pragma unroll
        for (int k = 0; k < HEADS; ++k) {
            a[k][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            a[k][1] = a[k][0];
            if constexpr (L0) {                // W_in[c] . P_k + S_k b_in[c]
                const f32x4 PS = PSK[k];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const f32x4 tb = *reinterpret_cast<const f32x4*>(TB + 4 * (32 * t + 8 * g + j));
                    a[k][j >> 2][j & 3] =
                        fmaf(tb[3], PS[3], fmaf(tb[2], PS[2], fmaf(tb[1], PS[1], tb[0] * PS[0])));
                }
                continue;
            }
            // the row's alphas of head k (LDS, written by this wave: in order)
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(AL + k * 8);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(AL + k * 8 + 4);
#pragma unroll
            for (int e = 0; e < AS; ++e) {
                const float w = e < 4 ? w0[e] : w1[e - 4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a[k][0][i] = fmaf(w, gv[e][0][i], a[k][0][i]);
                    a[k][1][i] = fmaf(w, gv[e][1][i], a[k][1][i]);
                }
            }
        }
        if (extra && !L0) {
            // entries past the register slots: alphas from the saved statistics
            for (int e = AS; e < deg; ++e) {
                const int j = col[e0 + e];
                const float* sp = x + static_cast<int64_t>(j) * ldx + 8 * g + 32 * t;
                const f32x4 u0 = *reinterpret_cast<const f32x4*>(sp);
                const f32x4 u1 = *reinterpret_cast<const f32x4*>(sp + 4);
#pragma unroll
                for (int k = 0; k < HEADS; ++k) {
                    const float adk = logits[rowc * (2 * HEADS) + HEADS + k];
                    const float w = expf(leaky(logits[static_cast<int64_t>(j) * (2 * HEADS) + k] + adk) -
                                         ST[k * 2]) / ST[k * 2 + 1];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        a[k][0][i] = fmaf(w, u0[i], a[k][0][i]);
                        a[k][1][i] = fmaf(w, u1[i], a[k][1][i]);
                    }
                }
            }
        }
        // (the next chunk's loads not hoisted above the sums: two gather
        // buffers live at once spilled registers)
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < C::XC && !(flags & MIGNN_DIAG_NO_PRODUCE)) gather(t + 1);
#pragma unroll
        for (int k = 0; k < HEADS; ++k) {
            const int j = t * C::NG + k / C::HPS;          // this head's W step
            if (C::NG > 1 && k > 0 && k % C::HPS == 0) {
                // W step j landed (younger: the next chunk's 2 AS row loads),
                // every wave's reads of buffer (j + 1) & 1 done -> its refill
                if (L0 || t + 1 >= C::XC || (flags & MIGNN_DIAG_NO_PRODUCE)) vm_barrier64<0>();
                else vm_barrier64<2 * AS>();
                w_dma(j + 1);
            }
            const unsigned char* wb = wl0 + (j & 1) * C::STEPW + (k % C::HPS) * C::WCH;
            uint32_t m = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                m = max(m, max(__float_as_uint(fabsf(a[k][0][i])), __float_as_uint(fabsf(a[k][1][i]))));
            const int pc = sexp_ag(rowmax4(m));
            // the row's first nonzero chunk sets the scale with 2 bits of headroom
            // (accumulators still zero: nothing to rescale), so later chunks
            // rarely lower it; a lowering is a uniform branch, exact rescale
            if (fresh) p = pc - 2;
            if (!fresh && __builtin_amdgcn_ballot_w64(pc < p) != 0ull) {
                const int dp = pc < p ? pc - p : 0;
#pragma unroll
                for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], dp);
                p = pc < p ? pc : p;
            }
            fresh = false;
            const float spv = p2_ag(p);
            f16x8 bh, bl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = (j < 4 ? a[k][0][j] : a[k][1][j - 4]) * spv;
                const _Float16 hh = static_cast<_Float16>(v);
                bh[j] = hh;
                bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
            }
#pragma unroll
            for (int cb = 0; cb < C::NCB; ++cb) {
                if (flags & MIGNN_DIAG_NO_MFMA) break;
                const unsigned char* wf = wb + (2 * cb) * AFRAG;
                const f16x8 wh = *reinterpret_cast<const f16x8*>(wf);
                const f16x8 wl = *reinterpret_cast<const f16x8*>(wf + AFRAG);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[cb], 0, 0, 0);
            }
            // (one head's fragments at a time: hoisting the next heads' LDS
            // reads above these MFMAs spilled registers)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // epilogue (staged, whole-row stores): the W / alpha buffers are free once
    // every wave is past its last MFMA; the vectors move after the staging rows
    vm_barrier<0>();
    if (flags & MIGNN_DIAG_NO_LOCAL) {         // (ablation: no epilogue)
        if (rv && acc[0][0] == 12345.f) out[rowc * ldo] = acc[1][1];
        return;
    }
    float* const EV2 = reinterpret_cast<float*>(lds + C::BM * H * 4);
    if (tid < H) {
        EV2[tid] = p2neg_ag(QF[tid]);
        EV2[H + tid] = BF[tid];
        EV2[2 * H + tid] = SC[tid];
        EV2[3 * H + tid] = SH[tid];
    }
    float* const WLN = EV2 + 4 * H;                // (LG) the next layer's logit weights [8][H]
    if constexpr (LG)
        for (int i = tid; i < 8 * H; i += C::NT) WLN[i] = wlog_next[i];
    staged_epilogue<C::NCB, L0, LG>(lds, EV2, acc, p, flags, x, ldx, out, ldo, rb + tile * C::BM,
                                    re, wave, lane, 16 * wave + r, g, TB, pi[0], pi[1], pi[2], WLN,
                                    lg_next);
}

// ------------------------------------------------------------------ TransformerConv
// H = 256, 4 heads (configs[3]; gnn_model.py:65-68, PyG TransformerConv,
// concat=False, root_weight): with qt_i = [W_k^T q_i per head] (the Q~K
// transform, one split-fp16 GEMM before this kernel; attn_layers.hip):
//   s_ij^h  = qt_i^h . x_j / sqrt(C)                      (score, per head)
//   a_ij^h  = softmax_j(s_ij^h)                           (PyG utils.softmax, +1e-16)
//   out_i   = epi([sum_j a_ij^h x_j (4 heads) | sum_j a_ij^h | x_i] . wout^T + b)
// in one kernel: pass 1 forms the 4 x 8 scores of a row's first 8 CSR entries
// in registers (lane (r, g) dots its 64 columns, the row's 4 lanes sum), the
// softmax statistics per head (online over further groups of 8 for longer
// rows); pass 2 builds the weighted sums one 32-wide k chunk at a time for the
// 4 heads in the MFMA B-operand layout and feeds them, split with the row's
// online exponent, straight into the output transform (image k order: chunk
// 4 kc + head, then x_i's 8 chunks, then the alpha-sum chunk --
// mignn_transformer_fused_prep).  Neither the [rows, 4 x 256 + 4] aggregate
// nor its re-read reach HBM.  Entries past the 8th: raw scores of the next 16
// kept in LDS, later ones recomputed (correct, not fast).
constexpr int TF_HEADS = 4;
constexpr int TF_KIN = TF_HEADS * AH + TF_HEADS + AH;   // wout: [W_v / heads | b_v / heads | W_skip]
constexpr int TF_NC = TF_HEADS * AKP + AKP + 1;          // 41 k chunks of the fused image
constexpr size_t TF_IMG_FRAG = static_cast<size_t>(TF_NC) * ACB * 2 * AFRAG;
constexpr size_t TF_IMG_BYTES = TF_IMG_FRAG + AH * 4;
constexpr int TF_XS = 16;                                // extra raw scores per row kept in LDS
constexpr float TF_EPS = 1e-16f;                         // PyG utils.softmax

__device__ __forceinline__ int tf_src_k(int kk) {       // fused-image k -> wout column (-1: 0)
    const int t = kk >> 5, i = kk & 31;
    if (t < TF_HEADS * AKP) return (t & 3) * AH + 32 * (t >> 2) + i;
    if (t < TF_HEADS * AKP + AKP) return TF_HEADS * AH + TF_HEADS + 32 * (t - TF_HEADS * AKP) + i;
    return i < TF_HEADS ? TF_HEADS * AH + i : -1;
}

__global__ __launch_bounds__(256) void tf_prep_exp_kernel(const float* __restrict__ w,
                                                          int32_t* __restrict__ q) {
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint32_t m = 0;
    for (int i = lane; i < TF_KIN; i += 64) m = max(m, __float_as_uint(fabsf(w[c * TF_KIN + i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o)));
    if (lane == 0) q[c] = sexp_ag(m);
}

__global__ __launch_bounds__(256) void tf_prep_frag_kernel(const float* __restrict__ w,
                                                           const int32_t* __restrict__ q,
                                                           unsigned char* __restrict__ img) {
    const int t = blockIdx.x * 256 + threadIdx.x;        // (chunk, cb, lane)
    if (t >= TF_NC * ACB * 64) return;
    const int lane = t & 63, cb = (t >> 6) % ACB, kc = (t >> 6) / ACB;
    const int c = 16 * cb + (lane & 15);
    const float sc = p2_ag(q[c]);
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = tf_src_k(32 * kc + 8 * (lane >> 4) + j);
        const float v = k >= 0 ? w[c * TF_KIN + k] * sc : 0.f;
        const _Float16 hh = static_cast<_Float16>(v);
        h[j] = hh;
        l[j] = static_cast<_Float16>(v - static_cast<float>(hh));
    }
    unsigned char* base = img + ((static_cast<size_t>(kc) * ACB + cb) * 2) * AFRAG + lane * 16;
    *reinterpret_cast<f16x8*>(base) = h;
    *reinterpret_cast<f16x8*>(base + AFRAG) = l;
}


// Block: 8 waves x 16 rows (128-row tile), one block per CU.  LDS: W ring
// [3][32 KB] (LDS-DMA two chunks ahead, one counted wait + barrier per chunk)
// | per row TF_XS extra raw scores; after the loop the whole LDS is the
// staged epilogue's (rows [128][1 KB] | q bias scale shift).
template <int EPIF = -1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void tf_fused_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ qt, int64_t ldq, const float* __restrict__ x, int64_t ldx,
    int64_t rb, int64_t re, float score_scale, const unsigned char* __restrict__ img,
    const float* __restrict__ bias, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    if constexpr (EPIF >= 0) flags = EPIF;
    constexpr int AW = 8, BM = 16 * AW;
    constexpr int WPC = ACHUNK / 1024 / AW;              // W pieces per wave per chunk (4)
    constexpr int OFF_XS = 3 * ACHUNK;
    constexpr int OFF_AL = OFF_XS + BM * TF_XS * 16;     // per row the 8 x 4 softmax weights
    constexpr int LDS_BYTES = OFF_AL + BM * 128;
    static_assert(OFF_AL >= BM * 1024 && LDS_BYTES >= BM * 1024 + 4 * AH * 4, "tf_fused LDS");
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t per_xcd = gridDim.x >> 3;
    const int64_t tile = static_cast<int64_t>(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (tile >= ntiles) return;
    const int64_t t0 = rb + tile * BM;
    const int64_t row = t0 + 16 * wave + r;
    const bool rv = row < re;
    const int64_t rowc = rv ? row : re - 1;
    const int lself = 16 * wave + r;

    auto w_dma = [&](int c) {                  // chunk c -> buffer c % 3 (dummy past the last)
        const int cc = c < TF_NC ? c : TF_NC - 1;
        const unsigned char* src = img + static_cast<size_t>(cc) * ACHUNK;
        unsigned char* dst = lds + (c % 3) * ACHUNK;
#pragma unroll
        for (int pc = 0; pc < WPC; ++pc) {
            const int piece = wave + pc * AW;
            glds16_ag(src + piece * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
        }
    };
    w_dma(0);
    w_dma(1);

    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    const float* const qrow = qt + rowc * ldq + 8 * g;
    auto xrow = [&](int c) -> const float* {   // lane's columns of row c (the zero row for c < 0)
        return c >= 0 ? x + static_cast<int64_t>(c) * ldx + 8 * g : g_zero_row_ag + 8 * g;
    };
    // 8-term dot as a pairwise tree (the score's rounding: short chains, as
    // transformer_aggregate's per-lane dots + tree reduction)
    auto dot8 = [](const f32x4& a0, const f32x4& a1, const f32x4& b0, const f32x4& b1, float d) {
        const float p0 = fmaf(a0[1], b0[1], a0[0] * b0[0]);
        const float p1 = fmaf(a0[3], b0[3], a0[2] * b0[2]);
        const float p2 = fmaf(a1[1], b1[1], a1[0] * b1[0]);
        const float p3 = fmaf(a1[3], b1[3], a1[2] * b1[2]);
        return d + ((p0 + p1) + (p2 + p3));
    };
    // scores of 8 entries (columns cj, -1 = none), 4 heads
    auto scores8 = [&](const int (&cj)[8], float (&sc)[TF_HEADS][8]) {
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h)
#pragma unroll
            for (int t = 0; t < 8; ++t) sc[h][t] = 0.f;
#pragma unroll 1
        for (int kc = 0; kc < AKP; ++kc) {
            f32x4 q0[TF_HEADS], q1[TF_HEADS];
#pragma unroll
            for (int h = 0; h < TF_HEADS; ++h) {
                q0[h] = *reinterpret_cast<const f32x4*>(qrow + h * AH + 32 * kc);
                q1[h] = *reinterpret_cast<const f32x4*>(qrow + h * AH + 32 * kc + 4);
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const float* xp = xrow(cj[t]) + 32 * kc;
                const f32x4 v0 = *reinterpret_cast<const f32x4*>(xp);
                const f32x4 v1 = *reinterpret_cast<const f32x4*>(xp + 4);
#pragma unroll
                for (int h = 0; h < TF_HEADS; ++h) sc[h][t] += dot8(q0[h], q1[h], v0, v1, 0.f);
                if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h)
#pragma unroll
            for (int t = 0; t < 8; ++t) sc[h][t] = rowsum4(sc[h][t]) * score_scale;
    };
    // the 4 scores of one entry (column c), recomputed
    auto score1 = [&](int c, float (&r4)[TF_HEADS]) {
        float d[TF_HEADS] = {0.f, 0.f, 0.f, 0.f};
        const float* const xp0 = xrow(c);
#pragma unroll 1
        for (int kc = 0; kc < AKP; ++kc) {
            const f32x4 v0 = *reinterpret_cast<const f32x4*>(xp0 + 32 * kc);
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(xp0 + 32 * kc + 4);
#pragma unroll
            for (int h = 0; h < TF_HEADS; ++h)
                d[h] += dot8(*reinterpret_cast<const f32x4*>(qrow + h * AH + 32 * kc),
                             *reinterpret_cast<const f32x4*>(qrow + h * AH + 32 * kc + 4), v0, v1, 0.f);
        }
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h) r4[h] = rowsum4(d[h]) * score_scale;
    };

    // ---- pass 1: scores and softmax statistics
    int cj[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) cj[t] = t < deg ? col[e0 + t] : -1;
    float s[TF_HEADS][8];
    if (flags & MIGNN_DIAG_NO_EXT) {           // (ablation: no pass 1)
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h)
#pragma unroll
            for (int t = 0; t < 8; ++t) s[h][t] = 0.f;
    } else {
        scores8(cj, s);
    }
    float m[TF_HEADS], l[TF_HEADS];
#pragma unroll
    for (int h = 0; h < TF_HEADS; ++h) {
        float mm = -INFINITY;
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (t < deg) mm = fmaxf(mm, s[h][t]);
        float ll = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (t < deg) ll += expf(s[h][t] - mm);
        m[h] = mm;
        l[h] = ll;
    }
    const bool slow = deg > 8;
    const bool any_slow = __builtin_amdgcn_ballot_w64(slow) != 0ull;
    float* const XS = reinterpret_cast<float*>(lds + OFF_XS) + lself * TF_XS * 4;
    if (any_slow && slow) {                    // further groups of 8: online statistics
        for (int eb = 8; eb < deg; eb += 8) {
            int cj2[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) cj2[t] = eb + t < deg ? col[e0 + eb + t] : -1;
            float s2[TF_HEADS][8];
            scores8(cj2, s2);
#pragma unroll
            for (int h = 0; h < TF_HEADS; ++h) {
                float bm = -INFINITY;
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (eb + t < deg) bm = fmaxf(bm, s2[h][t]);
                const float mn = fmaxf(m[h], bm);
                float ll = l[h] * expf(m[h] - mn);
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (eb + t < deg) ll += expf(s2[h][t] - mn);
                m[h] = mn;
                l[h] = ll;
            }
            if (g == 0) {
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (eb + t < deg && eb + t - 8 < TF_XS)
                        *reinterpret_cast<f32x4*>(XS + 4 * (eb + t - 8)) =
                            f32x4{s2[0][t], s2[1][t], s2[2][t], s2[3][t]};
            }
        }
    }
    // softmax weights of the first 8 entries -> LDS (entry t: 4 heads; lane
    // group g writes entries 2g, 2g + 1; read back by the row's 4 lanes)
    float inv[TF_HEADS];
#pragma unroll
    for (int h = 0; h < TF_HEADS; ++h) inv[h] = 1.f / (l[h] + TF_EPS);
    float* const AL = reinterpret_cast<float*>(lds + OFF_AL) + lself * 32;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        f32x4 av;
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h) av[h] = t < deg ? expf(s[h][t] - m[h]) * inv[h] : 0.f;
        if ((t >> 1) == g) *reinterpret_cast<f32x4*>(AL + 4 * t) = av;
    }

    // ---- pass 2: weighted sums -> output transform (41 k chunks)
    f32x4 acc[ACB];
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p = 100;
    bool fresh = true;                             // (the row's first chunk not seen yet)
    int c = 0;
    const unsigned char* const wl0 = lds + lane * 16;
    auto step = [&](const f32x4& a0, const f32x4& a1) {
        // split with the row's online exponent
        uint32_t mb = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            mb = max(mb, max(__float_as_uint(fabsf(a0[i])), __float_as_uint(fabsf(a1[i]))));
        const int pc = sexp_ag(rowmax4(mb));
        // the row's first nonzero chunk sets the scale with 2 bits of headroom
        // (accumulators still zero: nothing to rescale), so later chunks
        // rarely lower it; a lowering is a uniform branch, exact rescale
        if (fresh) p = pc - 2;
        if (!fresh && __builtin_amdgcn_ballot_w64(pc < p) != 0ull) {
            const int dp = pc < p ? pc - p : 0;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], dp);
            p = pc < p ? pc : p;
        }
        fresh = false;
        const float spv = p2_ag(p);
        f16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = (j < 4 ? a0[j] : a1[j - 4]) * spv;
            const _Float16 hh = static_cast<_Float16>(v);
            bh[j] = hh;
            bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
        }
        // chunk c landed (only chunk c + 1's pieces may fly), every wave done
        // with the buffer refilled next
        vm_barrier<WPC>();
        w_dma(c + 2);
        const unsigned char* wb = wl0 + (c % 3) * ACHUNK;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            if (flags & MIGNN_DIAG_NO_MFMA) break;
            const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
            const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[cb], 0, 0, 0);
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh, acc[cb], 0, 0, 0);
        }
        ++c;
    };
#pragma unroll 1
    for (int kc = 0; kc < AKP; ++kc) {
        f32x4 a0[TF_HEADS], a1[TF_HEADS];
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h) a0[h] = a1[h] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (flags & MIGNN_DIAG_NO_PRODUCE) break;   // (ablation: no weighted sums)
            const float* xp = xrow(cj[t]) + 32 * kc;
            const f32x4 v0 = *reinterpret_cast<const f32x4*>(xp);
            const f32x4 v1 = *reinterpret_cast<const f32x4*>(xp + 4);
            const f32x4 av = *reinterpret_cast<const f32x4*>(AL + 4 * t);
#pragma unroll
            for (int h = 0; h < TF_HEADS; ++h)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a0[h][i] = fmaf(av[h], v0[i], a0[h][i]);
                    a1[h][i] = fmaf(av[h], v1[i], a1[h][i]);
                }
            if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        if (any_slow && slow) {
            for (int e = 8; e < deg; ++e) {
                const int ce = col[e0 + e];
                float r4[TF_HEADS];
                if (e - 8 < TF_XS) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(XS + 4 * (e - 8));
#pragma unroll
                    for (int h = 0; h < TF_HEADS; ++h) r4[h] = v[h];
                } else {
                    score1(ce, r4);
                }
                const float* xp = xrow(ce) + 32 * kc;
                const f32x4 v0 = *reinterpret_cast<const f32x4*>(xp);
                const f32x4 v1 = *reinterpret_cast<const f32x4*>(xp + 4);
#pragma unroll
                for (int h = 0; h < TF_HEADS; ++h) {
                    const float a = expf(r4[h] - m[h]) * inv[h];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        a0[h][i] = fmaf(a, v0[i], a0[h][i]);
                        a1[h][i] = fmaf(a, v1[i], a1[h][i]);
                    }
                }
            }
        }
#pragma unroll
        for (int h = 0; h < TF_HEADS; ++h) step(a0[h], a1[h]);
    }
    // x_i (lin_skip), 8 chunks
    const float* const xi = x + rowc * ldx + 8 * g;
#pragma unroll 1
    for (int kc = 0; kc < AKP; ++kc)
        step(*reinterpret_cast<const f32x4*>(xi + 32 * kc), *reinterpret_cast<const f32x4*>(xi + 32 * kc + 4));
    // alpha sums (x b_v / heads): k = 0..3 of the last chunk, lane group 0
    {
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g == 0) a0 = f32x4{l[0] * inv[0], l[1] * inv[1], l[2] * inv[2], l[3] * inv[3]};
        step(a0, f32x4{0.f, 0.f, 0.f, 0.f});
    }

    // ---- epilogue: drain (the dummy refills), LDS free -> staged epilogue
    vm_barrier<0>();
    const bool hb = (flags & MIGNN_EPI_BIAS) != 0, ha = (flags & MIGNN_EPI_AFFINE) != 0;
    float* const EV = reinterpret_cast<float*>(lds + BM * 1024);   // q | bias | scale | shift
    if (tid < AH) {
        EV[tid] = p2neg_ag(reinterpret_cast<const int32_t*>(img + TF_IMG_FRAG)[tid]);
        EV[AH + tid] = hb ? bias[tid] : 0.f;
        EV[2 * AH + tid] = ha ? scale[tid] : 1.f;
        EV[3 * AH + tid] = ha ? shift[tid] : 0.f;
    }
    staged_epilogue<ACB>(lds, EV, acc, p, flags, x, ldx, out, ldo, t0, re, wave, lane, lself, g);
}

template <int MODE, bool CHAIN>
int launch_agg_gemm(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                    int64_t ldx, int64_t rb, int64_t re, float self_scale, const void* img1,
                    const float* b1, const void* img2, const float* b2, const float* scale,
                    const float* shift, int flags, float* out, int64_t ldo, hipStream_t st) {
    constexpr int BM = 128;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "agg_gemm: too many rows");
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nb)), dim3(512), 0, st, row_ptr, col,
                           ew, x, ldx, rb, re, self_scale, static_cast<const unsigned char*>(img1),
                           b1, static_cast<const unsigned char*>(img2), b2, scale, shift, flags,
                           out, ldo);
    };
    if (flags == kBN) go(agg_gemm_kernel<MODE, CHAIN, kBN>);
    else if (flags == kNoBN) go(agg_gemm_kernel<MODE, CHAIN, kNoBN>);
    else go(agg_gemm_kernel<MODE, CHAIN>);
    return launch_status("agg_gemm_kernel");
}


template <int H, bool L0 = false>
int launch_gat_fused(const int32_t* row_ptr, const int32_t* col, const float* logits,
                     const float* x, int64_t ldx, int64_t rb, int64_t re, float slope,
                     const void* img, const float* bias, const float* scale, const float* shift,
                     int flags, float* out, int64_t ldo, hipStream_t st,
                     const float* w_in = nullptr, const float* b_in = nullptr,
                     const float* lw = nullptr, int d = 0, const float* wlog_next = nullptr,
                     float* lg_next = nullptr) {
    using C = GatCfg<H>;
    const int64_t ntiles = (re - rb + C::BM - 1) / C::BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "gat_fused: too many rows");
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    auto go = [&](auto kern, const float* wn, float* ln) {
        hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nb)), dim3(C::NT), 0, st, row_ptr, col,
                           logits, x, ldx, rb, re, slope, static_cast<const unsigned char*>(img),
                           bias, scale, shift, flags, out, ldo, w_in, b_in, lw, d, wn, ln);
    };
    if (!L0 && lg_next != nullptr) {
        if (flags == kBN) go(gat_fused_kernel<H, false, true, kBN>, wlog_next, lg_next);
        else if (flags == kNoBN) go(gat_fused_kernel<H, false, true, kNoBN>, wlog_next, lg_next);
        else go(gat_fused_kernel<H, false, true>, wlog_next, lg_next);
    } else {
        if (flags == kBN) go(gat_fused_kernel<H, L0, false, kBN>, nullptr, nullptr);
        else if (flags == kNoBN) go(gat_fused_kernel<H, L0, false, kNoBN>, nullptr, nullptr);
        else go(gat_fused_kernel<H, L0>, nullptr, nullptr);
    }
    return launch_status("gat_fused_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_gin_fused_prep_bytes(int h) {
    return h == AH ? static_cast<size_t>(AKP) * ACB * 2 * AFRAG + AH * 4 : 0;
}

extern "C" int mignn_gin_fused_prep(const float* w2, int h, void* img, size_t img_bytes,
                                    void* stream) {
    MIGNN_REQUIRE(w2 && img && h == AH, "gin_fused_prep: h must be 256");
    MIGNN_REQUIRE(img_bytes >= mignn_gin_fused_prep_bytes(h), "gin_fused_prep: image too small");
    MIGNN_REQUIRE(aligned16(img), "gin_fused_prep: image not 16-B aligned");
    return perm_prep(w2, AH, static_cast<unsigned char*>(img), as_stream(stream), true);
}

static int check_common(const int32_t* row_ptr, const int32_t* col, const float* x, int64_t ldx,
                        int64_t rb, int64_t re, int h, const void* img1, const float* scale,
                        const float* shift, int flags, const float* out, int64_t ldo,
                        const char* what) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "%s: unknown flags 0x%x", what, flags);
    MIGNN_REQUIRE(row_ptr && col && x && img1 && out, "%s: null pointer", what);
    MIGNN_REQUIRE(h == AH, "%s: h must be 256 (got %d)", what, h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(img1), "%s: unaligned", what);
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "%s: bad strides", what);
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "%s: bad row range", what);
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "%s: affine", what);
    MIGNN_REQUIRE(x != out, "%s: in-place not supported (neighbours read x)", what);
    return MIGNN_OK;
}

extern "C" int mignn_gin_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* x,
                                     int64_t ldx, int64_t rb, int64_t re, int h, float eps,
                                     const void* img1, const float* b1, const void* img2,
                                     const float* b2, const float* scale, const float* shift,
                                     int flags, float* out, int64_t ldo, void* stream) {
    int rc = check_common(row_ptr, col, x, ldx, rb, re, h, img1, scale, shift, flags, out, ldo,
                          "gin_layer_fused");
    if (rc) return rc;
    MIGNN_REQUIRE(img2 && b1 && aligned16(img2), "gin_layer_fused: img2 / b1");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || b2, "gin_layer_fused: bias");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    const float s = 1.0f + eps;
    flags |= g_fused_diag_flags;
    return launch_agg_gemm<AGG_GIN, true>(row_ptr, col, nullptr, x, ldx, rb, re, s, img1, b1,
                                             img2, b2, scale, shift, flags, out, ldo, st);
}

extern "C" int mignn_gcn_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                     const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                     const void* img, const float* bias, const float* scale,
                                     const float* shift, int flags, float* out, int64_t ldo,
                                     void* stream) {
    int rc = check_common(row_ptr, col, x, ldx, rb, re, h, img, scale, shift, flags, out, ldo,
                          "gcn_layer_fused");
    if (rc) return rc;
    MIGNN_REQUIRE(ew, "gcn_layer_fused: ew");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_fused: bias");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    flags |= g_fused_diag_flags;
    return launch_agg_gemm<AGG_GCN, false>(row_ptr, col, ew, x, ldx, rb, re, 1.f, img, bias,
                                              nullptr, nullptr, scale, shift, flags, out, ldo, st);
}


// the fused GAT layer (see gat_fused_kernel); called by mignn_gat_layer when
// it has the split image of wcat, heads = 4 and h in {64, 128}
namespace mignn {
int gat_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* logits,
                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h, float slope,
                    const void* img, const float* bias, const float* scale, const float* shift,
                    int flags, float* out, int64_t ldo, void* stream, const float* wlog_next,
                    float* lg_next) {
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(img) && ldx % 4 == 0 && ldo % 4 == 0,
                  "gat_layer: fused path needs 16-B aligned rows");
    MIGNN_REQUIRE(x != out, "gat_layer: in-place not supported (neighbours read x)");
    hipStream_t st = as_stream(stream);
    flags |= g_fused_diag_flags;
    return h == 128 ? launch_gat_fused<128>(row_ptr, col, logits, x, ldx, rb, re, slope, img, bias,
                                            scale, shift, flags, out, ldo, st, nullptr, nullptr,
                                            nullptr, 0, wlog_next, lg_next)
                    : launch_gat_fused<64>(row_ptr, col, logits, x, ldx, rb, re, slope, img, bias,
                                           scale, shift, flags, out, ldo, st, nullptr, nullptr,
                                           nullptr, 0, wlog_next, lg_next);
}
}  // namespace mignn

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_set_fused_flags(int flags) {
    g_fused_diag_flags = flags & (MIGNN_DIAG_NO_PRODUCE | MIGNN_DIAG_NO_MFMA | MIGNN_DIAG_NO_EXT |
                                  MIGNN_DIAG_NO_TABLES | MIGNN_DIAG_NO_LOCAL |
                                  MIGNN_SCHED_INTERLEAVED);
    return MIGNN_OK;
}
#endif

namespace mignn {
size_t head256_prep_bytes() { return HEAD256_BYTES; }

int head256_prep(const float* w1, const float* b1, const float* w2, const float* b2,
                 const float* w3, const float* b3, const float* w4, const float* b4, int out_dim,
                 void* img, void* stream) {
    hipStream_t st = as_stream(stream);
    auto* im = static_cast<unsigned char*>(img);
    if (int rc = mignn_linear_f16x3_prep(w1, AH, AH, im, HIMG, stream)) return rc;
    if (int rc = perm_prep(w2, AH, im + HIMG, st)) return rc;
    if (int rc = perm_prep(w3, AH / 2, im + 2 * HIMG, st)) return rc;
    hipLaunchKernelGGL(head256_vec_kernel, dim3(1), dim3(256), 0, st, b1, b2, b3, w4, b4, out_dim, im);
    return launch_status("head256_vec_kernel");
}

int head256(const float* x, int64_t ldx, int64_t n, const void* img, int out_dim, float* out,
            int64_t ldo, const int32_t* out_rows, void* stream) {
    const int64_t ntiles = (n + 127) / 128;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "mlp_head: too many rows");
    hipLaunchKernelGGL(head256_kernel, dim3(static_cast<unsigned>(nb)), dim3(512), 0,
                       as_stream(stream), x, ldx, n, static_cast<const unsigned char*>(img),
                       out_dim, out, ldo, out_rows);
    return launch_status("head256_kernel");
}
}  // namespace mignn

// ------------------------------------------------------------------ TransformerConv, fused
namespace mignn {
size_t tf_fused_prep_bytes() { return TF_IMG_BYTES; }

int tf_fused_prep(const float* wout, void* img, void* stream) {
    hipStream_t st = as_stream(stream);
    auto* base = static_cast<unsigned char*>(img);
    int32_t* q = reinterpret_cast<int32_t*>(base + TF_IMG_FRAG);
    hipLaunchKernelGGL(tf_prep_exp_kernel, dim3(AH / 4), dim3(256), 0, st, wout, q);
    if (int rc = launch_status("tf_prep_exp_kernel")) return rc;
    hipLaunchKernelGGL(tf_prep_frag_kernel, dim3((TF_NC * ACB * 64 + 255) / 256), dim3(256), 0, st,
                       wout, q, base);
    return launch_status("tf_prep_frag_kernel");
}

int tf_fused(const int32_t* row_ptr, const int32_t* col, const float* qt, int64_t ldq,
             const float* x, int64_t ldx, int64_t rb, int64_t re, float score_scale,
             const void* img, const float* bias, const float* scale, const float* shift, int flags,
             float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(img) && aligned16(qt) &&
                      ldx % 4 == 0 && ldo % 4 == 0 && ldq % 4 == 0 && ldq >= TF_HEADS * AH,
                  "transformer_layer: fused path needs 16-B aligned rows");
    MIGNN_REQUIRE(x != out, "transformer_layer: in-place not supported (neighbours read x)");
    constexpr int BM = 128;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "transformer_layer: too many rows");
    const auto* im = static_cast<const unsigned char*>(img);
    flags |= g_fused_diag_flags;
    constexpr int kBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_AFFINE | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nb)), dim3(512), 0, as_stream(stream),
                           row_ptr, col, qt, ldq, x, ldx, rb, re, score_scale, im, bias, scale,
                           shift, flags, out, ldo);
    };
    if (flags == kBN) go(tf_fused_kernel<kBN>);
    else if (flags == kNoBN) go(tf_fused_kernel<kNoBN>);
    else go(tf_fused_kernel<>);
    return launch_status("tf_fused_kernel");
}
}  // namespace mignn

extern "C" int mignn_gin_layer0_fused(const int32_t* row_ptr, const int32_t* col, const float* pos,
                                      int64_t ldp, int d, int64_t rb, int64_t re, int h, float eps,
                                      const float* w_in, const float* b_in, const void* img1,
                                      const float* b1, const void* img2, const float* b2,
                                      const float* scale, const float* shift, int flags,
                                      float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gin_layer0_fused: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(row_ptr && col && pos && w_in && b_in && img1 && b1 && img2 && out,
                  "gin_layer0_fused: null pointer");
    MIGNN_REQUIRE(h == AH, "gin_layer0_fused: h must be 256 (got %d)", h);
    MIGNN_REQUIRE(d >= 1 && d <= 3 && ldp >= d, "gin_layer0_fused: 1..3 coordinates per node");
    MIGNN_REQUIRE(aligned16(out) && aligned16(img1) && aligned16(img2) && ldo % 4 == 0 && ldo >= h,
                  "gin_layer0_fused: unaligned");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gin_layer0_fused: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gin_layer0_fused: affine");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || b2, "gin_layer0_fused: bias");
    if (re == rb) return MIGNN_OK;
    constexpr int BM = 128;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "gin_layer0_fused: too many rows");
    hipLaunchKernelGGL(gin0_fused_kernel, dim3(static_cast<unsigned>(nb)), dim3(512), 0,
                       as_stream(stream), row_ptr, col, pos, ldp, d, rb, re, 1.0f + eps, w_in, b_in,
                       static_cast<const unsigned char*>(img1), b1,
                       static_cast<const unsigned char*>(img2), b2, scale, shift, flags, out, ldo);
    return launch_status("gin0_fused_kernel");
}

extern "C" int mignn_gat_layer0_fused(const int32_t* row_ptr, const int32_t* col, const float* pos,
                                      int64_t ldp, int d, int64_t rb, int64_t re, int h,
                                      float negative_slope, const float* w_in, const float* b_in,
                                      const float* lw, const void* wcat_img, const float* bias,
                                      const float* scale, const float* shift, int flags,
                                      float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gat_layer0_fused: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(row_ptr && col && pos && w_in && b_in && lw && wcat_img && out,
                  "gat_layer0_fused: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gat_layer0_fused: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(d >= 1 && d <= 3 && ldp >= d, "gat_layer0_fused: 1..3 coordinates per node");
    MIGNN_REQUIRE(aligned16(out) && aligned16(wcat_img) && aligned16(lw) && ldo % 4 == 0 && ldo >= h,
                  "gat_layer0_fused: unaligned");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gat_layer0_fused: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gat_layer0_fused: affine");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gat_layer0_fused: bias");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    flags |= g_fused_diag_flags;
    return h == 128 ? launch_gat_fused<128, true>(row_ptr, col, nullptr, pos, ldp, rb, re,
                                                  negative_slope, wcat_img, bias, scale, shift,
                                                  flags, out, ldo, st, w_in, b_in, lw, d)
                    : launch_gat_fused<64, true>(row_ptr, col, nullptr, pos, ldp, rb, re,
                                                 negative_slope, wcat_img, bias, scale, shift,
                                                 flags, out, ldo, st, w_in, b_in, lw, d);
}

extern "C" int mignn_transformer_layer0_coords(const int32_t* row_ptr, const int32_t* col,
                                               const float* pos, int64_t ldp, int d,
                                               int64_t rb, int64_t re, int h, int heads,
                                               float score_scale, const float* table,
                                               const float* gt, int relu, float* out,
                                               int64_t ldo, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && pos && table && gt && out, "transformer_layer0_coords: null pointer");
    MIGNN_REQUIRE(heads == 4 && (h == 64 || h == 128 || h == 256),
                  "transformer_layer0_coords: heads = 4, h in {64, 128, 256}");
    MIGNN_REQUIRE(d >= 1 && d <= 3 && ldp >= d, "transformer_layer0_coords: 1..3 coordinates per node");
    MIGNN_REQUIRE(ldo >= h && (h != 256 || (aligned16(out) && ldo % 4 == 0)),
                  "transformer_layer0_coords: bad output");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "transformer_layer0_coords: bad row range");
    if (re == rb) return MIGNN_OK;
    const int64_t nb = (re - rb + 63) / 64;
    const int64_t groups = (nb + 3) / 4;
    const unsigned grid = static_cast<unsigned>(groups < 256 * 16 ? groups : 256 * 16);
    hipStream_t st = as_stream(stream);
    switch (h) {
        case 256: hipLaunchKernelGGL(tf0_kernel<4>, dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, score_scale, table, gt, relu, out, ldo); break;
        case 128: hipLaunchKernelGGL(tf0_kernel<2>, dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, score_scale, table, gt, relu, out, ldo); break;
        default: hipLaunchKernelGGL(tf0_kernel<1>, dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, score_scale, table, gt, relu, out, ldo); break;
    }
    return launch_status("tf0_kernel");
}

extern "C" int mignn_gat_layer0_coords(const int32_t* row_ptr, const int32_t* col, const float* pos,
                                       int64_t ldp, int d, int64_t rb, int64_t re, int h,
                                       int heads, float negative_slope, const float* table,
                                       const float* lw, int relu, float* out, int64_t ldo,
                                       const float* wlog_next, float* logits_next, void* stream) {
    MIGNN_REQUIRE((wlog_next == nullptr) == (logits_next == nullptr) &&
                      (logits_next == nullptr || aligned16(logits_next)),
                  "gat_layer0_coords: wlog_next and 16-B aligned logits_next go together");
    MIGNN_REQUIRE(row_ptr && col && pos && table && lw && out, "gat_layer0_coords: null pointer");
    MIGNN_REQUIRE(heads == 4 && (h == 64 || h == 128 || h == 256),
                  "gat_layer0_coords: heads = 4, h in {64, 128, 256}");
    MIGNN_REQUIRE(d >= 1 && d <= 3 && ldp >= d, "gat_layer0_coords: 1..3 coordinates per node");
    MIGNN_REQUIRE(ldo >= h && (h != 256 || (aligned16(out) && ldo % 4 == 0)),
                  "gat_layer0_coords: bad output");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gat_layer0_coords: bad row range");
    if (re == rb) return MIGNN_OK;
    const int64_t nb = (re - rb + 63) / 64;
    const int64_t groups = (nb + 3) / 4;
    const unsigned grid = static_cast<unsigned>(groups < 256 * 16 ? groups : 256 * 16);
    hipStream_t st = as_stream(stream);
    switch (h) {
        case 256: hipLaunchKernelGGL((tf0_kernel<4, true>), dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, negative_slope, table, lw, relu, out, ldo, wlog_next, logits_next); break;
        case 128: hipLaunchKernelGGL((tf0_kernel<2, true>), dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, negative_slope, table, lw, relu, out, ldo, wlog_next, logits_next); break;
        default: hipLaunchKernelGGL((tf0_kernel<1, true>), dim3(grid), dim3(256), 0, st, row_ptr, col, pos, ldp, d, rb, re, negative_slope, table, lw, relu, out, ldo, wlog_next, logits_next); break;
    }
    return launch_status("tf0_kernel<gat>");
}

MIGNN_DMA_OOB_EXPORT(mignn_diag_dma_oob_agg)
