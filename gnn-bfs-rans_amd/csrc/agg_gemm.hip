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
__device__ __forceinline__ uint32_t lds_addr_ag(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_ag)(p)));
}
// LDS-DMA of 16 B per lane (inline asm: the compiler does not count it; the
// kernel's explicit vmcnt(0) before each chunk barrier covers it)
__device__ __forceinline__ void glds16_ag(const void* src, uint32_t dst) {
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

// (two waves per SIMD: <= 256 VGPRs; AW = 4 -> two blocks per CU)
template <int MODE, bool CHAIN, int AW>
__global__ __launch_bounds__(AW * 64) __attribute__((amdgpu_waves_per_eu(2))) void agg_gemm_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t rb,
    int64_t re, float self_scale, const unsigned char* __restrict__ img1,
    const float* __restrict__ b1, const unsigned char* __restrict__ img2,
    const float* __restrict__ b2, const float* __restrict__ scale,
    const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    constexpr int NT = AW * 64;
    constexpr int BM = 16 * AW;
    constexpr int NC = AKP * (CHAIN ? 2 : 1);          // W chunks streamed per tile
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * ACHUNK + 6 * AH * 4];
    int32_t* const Q1 = reinterpret_cast<int32_t*>(lds + 2 * ACHUNK);   // W1 column exponents
    float* const B1 = reinterpret_cast<float*>(Q1 + AH);               // GIN: nn.0 bias
    int32_t* const QF = reinterpret_cast<int32_t*>(B1 + AH);            // final transform's exponents
    float* const BF = reinterpret_cast<float*>(QF + AH);               // final bias (0 without BIAS)
    float* const SC = BF + AH;                                          // BN scale (1) / shift (0)
    float* const SH = SC + AH;

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
    const int64_t row = rb + tile * BM + 16 * wave + r;
    const bool rv = row < re;
    const int64_t rowc = rv ? row : re - 1;

    // W chunk c (W1 chunks, then W2's) -> LDS buffer c & 1: 32 pieces of 1 KB
    auto w_dma = [&](int c) {
        if (c >= NC) return;
        const unsigned char* src = c < AKP ? img1 + static_cast<size_t>(c) * ACHUNK
                                           : img2 + static_cast<size_t>(c - AKP) * ACHUNK;
        unsigned char* dst = lds + (c & 1) * ACHUNK;
#pragma unroll
        for (int pc = 0; pc < ACHUNK / 1024 / AW; ++pc) {
            const int piece = wave + pc * AW;
            glds16_ag(src + piece * 1024 + lane * 16, lds_addr_ag(dst + piece * 1024));
        }
    };
    w_dma(0);

    // per-column vectors of the epilogues
    if (tid < AH) {
        constexpr size_t FB = static_cast<size_t>(AKP) * ACB * 2 * AFRAG;
        Q1[tid] = reinterpret_cast<const int32_t*>(img1 + FB)[tid];
        B1[tid] = CHAIN ? b1[tid] : 0.f;
        QF[tid] = reinterpret_cast<const int32_t*>((CHAIN ? img2 : img1) + FB)[tid];
        BF[tid] = (flags & MIGNN_EPI_BIAS) ? (CHAIN ? b2 : b1)[tid] : 0.f;
        SC[tid] = (flags & MIGNN_EPI_AFFINE) ? scale[tid] : 1.f;
        SH[tid] = (flags & MIGNN_EPI_AFFINE) ? shift[tid] : 0.f;
    }

    // the row's CSR entries (first AS in registers; empty slots -> the zero row)
    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    const float* src[AS];
    float wgt[AS];
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        const int c = e < deg ? col[e0 + e] : -1;
        src[e] = c >= 0 ? x + static_cast<int64_t>(c) * ldx + 8 * g : g_zero_row_ag + 8 * g;
        wgt[e] = (MODE == AGG_GCN && e < deg) ? ew[e0 + e] : 0.f;
    }
    const float* const xself = x + rowc * ldx + 8 * g;
    // wave-uniform: does any row have entries past the register slots?
    const bool extra = __builtin_amdgcn_ballot_w64(deg > AS) != 0ull;

    // one chunk's gathered values: AS entries (+ GIN's own row), 8 floats each
    constexpr int NV = AS + (MODE == AGG_GIN ? 1 : 0);
    f32x4 gv[NV][2];
    auto gather = [&](int kc) {
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            gv[e][0] = *reinterpret_cast<const f32x4*>(src[e] + 32 * kc);
            gv[e][1] = *reinterpret_cast<const f32x4*>(src[e] + 32 * kc + 4);
        }
        if constexpr (MODE == AGG_GIN) {
            gv[AS][0] = *reinterpret_cast<const f32x4*>(xself + 32 * kc);
            gv[AS][1] = *reinterpret_cast<const f32x4*>(xself + 32 * kc + 4);
        }
    };
    gather(0);

    f32x4 acc[ACB];
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p = 100;                                   // the row's running exponent
    const unsigned char* const wl0 = lds + lane * 16;

    // ---------------------------------------------------------------- transform 1
#pragma unroll 1
    for (int kc = 0; kc < AKP; ++kc) {
        chunk_barrier();                           // W chunk kc and this chunk's rows landed
        w_dma(kc + 1);                             // into the buffer chunk kc-1 used
        // the aggregate's 8 values of this chunk (CSR order)
        f32x4 a0 = f32x4{0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
        for (int e = 0; e < AS; ++e) {
            if constexpr (MODE == AGG_GCN) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a0[i] = fmaf(wgt[e], gv[e][0][i], a0[i]);
                    a1[i] = fmaf(wgt[e], gv[e][1][i], a1[i]);
                }
            } else {
                a0 += gv[e][0];
                a1 += gv[e][1];
            }
        }
        if (extra) {
            // entries past the register slots, one at a time (CSR order)
            for (int e = AS; e < deg; ++e) {
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
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0[i] = fmaf(self_scale, gv[AS][0][i], a0[i]);
                a1[i] = fmaf(self_scale, gv[AS][1][i], a1[i]);
            }
        }
        // the next chunk's rows fly while this chunk's MFMAs run
        if (kc + 1 < AKP) gather(kc + 1);
        // split with the row's online exponent
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            m = max(m, max(__float_as_uint(fabsf(a0[i])), __float_as_uint(fabsf(a1[i]))));
        const int pc = sexp_ag(rowmax4(m));
        if (pc < p) {                              // lower the row's scale: exact rescale
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], pc - p);
            p = pc;
        }
        const float sp = p2_ag(p);
        f16x8 bh, bl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = (j < 4 ? a0[j] : a1[j - 4]) * sp;
            const _Float16 hh = static_cast<_Float16>(v);
            bh[j] = hh;
            bl[j] = static_cast<_Float16>(v - static_cast<float>(hh));
        }
        const unsigned char* wb = wl0 + (kc & 1) * ACHUNK;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
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
        uint32_t m = 0;
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) {
            const int4 q = *reinterpret_cast<const int4*>(&Q1[16 * cb + 4 * g]);
            const f32x4 bb = *reinterpret_cast<const f32x4*>(&B1[16 * cb + 4 * g]);
            const int qn[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float h = ldexpf(acc[cb][i], -(p + qn[i])) + bb[i];
                h = h < 0.f ? 0.f : h;
                acc[cb][i] = h;
                m = max(m, __float_as_uint(fabsf(h)));
            }
        }
        p = sexp_ag(rowmax4(m));
        const float sp = p2_ag(p);
        f16x8 hh[AKP], hl[AKP];
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = acc[2 * kc + (j >> 2)][j & 3] * sp;
                const _Float16 t = static_cast<_Float16>(v);
                hh[kc][j] = t;
                hl[kc][j] = static_cast<_Float16>(v - static_cast<float>(t));
            }
#pragma unroll
        for (int cb = 0; cb < ACB; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < AKP; ++kc) {
            chunk_barrier();                       // W2 chunk kc landed
            w_dma(AKP + kc + 1);
            const unsigned char* wb = wl0 + ((AKP + kc) & 1) * ACHUNK;
#pragma unroll
            for (int cb = 0; cb < ACB; ++cb) {
                const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * AFRAG);
                const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * AFRAG);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hh[kc], acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, hl[kc], acc[cb], 0, 0, 0);
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, hh[kc], acc[cb], 0, 0, 0);
            }
        }
    }

    // -------------------------------------------------------------------- epilogue
    // lane (r, g): row r, columns 16 cb + 4 g + i; bias, residual x_i, BN, ReLU
    // (gnn_model.py:184-191 order: conv + bias, + x, BN, ReLU)
    const bool res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    const float* const xr = x + rowc * ldx + 4 * g;
    float* const orow = out + rowc * ldo + 4 * g;
#pragma unroll
    for (int cb = 0; cb < ACB; ++cb) {
        const int n = 16 * cb + 4 * g;
        const int4 q = *reinterpret_cast<const int4*>(&QF[n]);
        const f32x4 bo = *reinterpret_cast<const f32x4*>(&BF[n]);
        const f32x4 so = *reinterpret_cast<const f32x4*>(&SC[n]);
        const f32x4 ho = *reinterpret_cast<const f32x4*>(&SH[n]);
        const f32x4 xv = res ? *reinterpret_cast<const f32x4*>(xr + 16 * cb) : f32x4{0.f, 0.f, 0.f, 0.f};
        const int qn[4] = {q.x, q.y, q.z, q.w};
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            o[i] = epilogue(ldexpf(acc[cb][i], -(p + qn[i])), flags, bo[i], xv[i], so[i], ho[i]);
        if (rv) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(orow + 16 * cb));
    }
}

// k-permuted split image of W2 [256, 256] for the chained transform: element
// j of lane (m, g) in fragment (kc, cb) = W2[16 cb + m][16 (2 kc + j / 4) +
// 4 g + j % 4] * 2^q (q per output column, as gprep_exp_kernel); layout and
// exponent table as mignn_linear_f16x3_prep's image
__global__ __launch_bounds__(256) void perm_exp_kernel(const float* __restrict__ w,
                                                       int32_t* __restrict__ q) {
    const int colm = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint32_t m = 0;
    for (int i = lane; i < AH; i += 64) m = max(m, __float_as_uint(fabsf(w[colm * AH + i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o)));
    if (lane == 0) q[colm] = sexp_ag(m);
}
__global__ __launch_bounds__(256) void perm_frag_kernel(const float* __restrict__ w,
                                                        const int32_t* __restrict__ q,
                                                        unsigned char* __restrict__ img) {
    const int t = blockIdx.x * 256 + threadIdx.x;   // (kc, cb, lane)
    if (t >= AKP * ACB * 64) return;
    const int lane = t & 63;
    const int cb = (t >> 6) % ACB;
    const int kc = (t >> 6) / ACB;
    const int colm = 16 * cb + (lane & 15);
    const int gq = lane >> 4;
    const float sc = p2_ag(q[colm]);
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = 16 * (2 * kc + (j >> 2)) + 4 * gq + (j & 3);
        const float v = w[colm * AH + kk] * sc;
        const _Float16 hh = static_cast<_Float16>(v);
        h[j] = hh;
        l[j] = static_cast<_Float16>(v - static_cast<float>(hh));
    }
    unsigned char* base = img + ((static_cast<size_t>(kc) * ACB + cb) * 2) * AFRAG + lane * 16;
    *reinterpret_cast<f16x8*>(base) = h;
    *reinterpret_cast<f16x8*>(base + AFRAG) = l;
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
// [H, 4H]) are LDS-DMA'd together, double-buffered, one barrier per x chunk.
template <int H>
struct GatCfg {
    static_assert(H == 64 || H == 128, "gat_fused: H in {64, 128}");
    static constexpr int AW = 8, NT = AW * 64, BM = 16 * AW;
    static constexpr int NCB = H / 16;                 // output column blocks (N = H)
    static constexpr int XC = H / 32;                  // x chunks
    static constexpr int NPB = 16;                     // column blocks per image chunk (padded)
    static constexpr int WCH = NCB * 2 * AFRAG;        // real bytes of one W chunk
    static constexpr int STEPW = 4 * WCH;              // the 4 heads' chunks of one x chunk
    static constexpr int OFF_AL = 2 * STEPW;           // alphas [AW][16][4][8]
    static constexpr int OFF_ST = OFF_AL + AW * 16 * 4 * 8 * 4;   // (max, sum) [AW][16][4]
    static constexpr int OFF_EPI = OFF_ST + AW * 16 * 4 * 8;       // QF | BF | SC | SH [H]
    static constexpr int LDS_BYTES = OFF_EPI + 4 * H * 4;
    static_assert(LDS_BYTES <= 160 * 1024, "gat_fused LDS");
};

template <int H>
__global__ __launch_bounds__(GatCfg<H>::NT) __attribute__((amdgpu_waves_per_eu(2))) void
gat_fused_kernel(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                 const float* __restrict__ logits, const float* __restrict__ x, int64_t ldx,
                 int64_t rb, int64_t re, float slope, const unsigned char* __restrict__ img,
                 const float* __restrict__ bias, const float* __restrict__ scale,
                 const float* __restrict__ shift, int flags, float* __restrict__ out, int64_t ldo) {
    using C = GatCfg<H>;
    constexpr int HEADS = 4;
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

    // W chunks of x chunk t (heads 0..3: image chunks k XC + t) -> buffer t & 1
    auto w_dma = [&](int t) {
        if (t >= C::XC) return;
        unsigned char* dst = lds + (t & 1) * C::STEPW;
#pragma unroll
        for (int pc = 0; pc < C::STEPW / 1024 / C::AW; ++pc) {
            const int piece = wave + pc * C::AW;              // 1-KB piece of the step
            const int hd = piece / (C::WCH / 1024), q = piece % (C::WCH / 1024);
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

    // ---- CSR slots, scores of head g, softmax statistics, alphas
    const int e0 = row_ptr[rowc];
    const int deg = rv ? row_ptr[rowc + 1] - e0 : 0;
    int cj[AS];
#pragma unroll
    for (int e = 0; e < AS; ++e) cj[e] = e < deg ? col[e0 + e] : -1;
    const bool extra = __builtin_amdgcn_ballot_w64(deg > AS) != 0ull;
    auto leaky = [&](float v) { return v > 0.f ? v : v * slope; };
    const float ad = logits[rowc * (2 * HEADS) + HEADS + g];
    float sc[AS];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < AS; ++e) {
        sc[e] = cj[e] >= 0 ? leaky(logits[static_cast<int64_t>(cj[e]) * (2 * HEADS) + g] + ad) : -INFINITY;
        mx = fmaxf(mx, sc[e]);
    }
    if (extra)
        for (int e = AS; e < deg; ++e)
            mx = fmaxf(mx, leaky(logits[static_cast<int64_t>(col[e0 + e]) * (2 * HEADS) + g] + ad));
    float sm = 0.f;
#pragma unroll
    for (int e = 0; e < AS; ++e)
        if (cj[e] >= 0) sm += expf(sc[e] - mx);
    if (extra)
        for (int e = AS; e < deg; ++e)
            sm += expf(leaky(logits[static_cast<int64_t>(col[e0 + e]) * (2 * HEADS) + g] + ad) - mx);
    sm += 1e-16f;
    float* const AL = reinterpret_cast<float*>(lds + C::OFF_AL) + ((wave * 16 + r) * 4) * 8;
    float* const ST = reinterpret_cast<float*>(lds + C::OFF_ST) + ((wave * 16 + r) * 4) * 2;
    {
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
    const unsigned char* const wl0 = lds + lane * 16;

#pragma unroll 1
    for (int t = 0; t < C::XC; ++t) {
        chunk_barrier();                           // W chunks of t and this chunk's rows landed
        w_dma(t + 1);
        // the 4 heads' weighted sums of this x chunk (CSR order)
        f32x4 a[HEADS][2];
#pragma unroll
        for (int k = 0; k < HEADS; ++k) {
            a[k][0] = f32x4{0.f, 0.f, 0.f, 0.f};
            a[k][1] = a[k][0];
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
        if (extra) {
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
        if (t + 1 < C::XC) gather(t + 1);
        const unsigned char* wb = wl0 + (t & 1) * C::STEPW;
#pragma unroll
        for (int k = 0; k < HEADS; ++k) {
            uint32_t m = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                m = max(m, max(__float_as_uint(fabsf(a[k][0][i])), __float_as_uint(fabsf(a[k][1][i]))));
            const int pc = sexp_ag(rowmax4(m));
            if (pc < p) {
#pragma unroll
                for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc[cb][i] = ldexpf(acc[cb][i], pc - p);
                p = pc;
            }
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
                const unsigned char* wf = wb + k * C::WCH + (2 * cb) * AFRAG;
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
    // epilogue: lane (r, g) = row r, columns 16 cb + 4 g + i
    const bool res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    const float* const xr = x + rowc * ldx + 4 * g;
    float* const orow = out + rowc * ldo + 4 * g;
#pragma unroll
    for (int cb = 0; cb < C::NCB; ++cb) {
        const int n = 16 * cb + 4 * g;
        const int4 q = *reinterpret_cast<const int4*>(&QF[n]);
        const f32x4 bo = *reinterpret_cast<const f32x4*>(&BF[n]);
        const f32x4 so = *reinterpret_cast<const f32x4*>(&SC[n]);
        const f32x4 ho = *reinterpret_cast<const f32x4*>(&SH[n]);
        const f32x4 xv = res ? *reinterpret_cast<const f32x4*>(xr + 16 * cb) : f32x4{0.f, 0.f, 0.f, 0.f};
        const int qn[4] = {q.x, q.y, q.z, q.w};
        f32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            o[i] = epilogue(ldexpf(acc[cb][i], -(p + qn[i])), flags, bo[i], xv[i], so[i], ho[i]);
        if (rv) __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(orow + 16 * cb));
    }
}

template <int MODE, bool CHAIN, int AW>
int launch_agg_gemm(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                    int64_t ldx, int64_t rb, int64_t re, float self_scale, const void* img1,
                    const float* b1, const void* img2, const float* b2, const float* scale,
                    const float* shift, int flags, float* out, int64_t ldo, hipStream_t st) {
    constexpr int BM = 16 * AW;
    const int64_t ntiles = (re - rb + BM - 1) / BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "agg_gemm: too many rows");
    hipLaunchKernelGGL((agg_gemm_kernel<MODE, CHAIN, AW>), dim3(static_cast<unsigned>(nb)),
                       dim3(AW * 64), 0, st, row_ptr, col, ew, x, ldx, rb, re, self_scale,
                       static_cast<const unsigned char*>(img1), b1,
                       static_cast<const unsigned char*>(img2), b2, scale, shift, flags, out, ldo);
    return launch_status("agg_gemm_kernel");
}

int g_agg_waves = 8;     // mignn_diag_set_agg_gemm_waves (timing study: 4 or 8)

template <int H>
int launch_gat_fused(const int32_t* row_ptr, const int32_t* col, const float* logits,
                     const float* x, int64_t ldx, int64_t rb, int64_t re, float slope,
                     const void* img, const float* bias, const float* scale, const float* shift,
                     int flags, float* out, int64_t ldo, hipStream_t st) {
    using C = GatCfg<H>;
    const int64_t ntiles = (re - rb + C::BM - 1) / C::BM;
    const int64_t nb = (ntiles + 7) / 8 * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "gat_fused: too many rows");
    hipLaunchKernelGGL((gat_fused_kernel<H>), dim3(static_cast<unsigned>(nb)), dim3(C::NT), 0, st,
                       row_ptr, col, logits, x, ldx, rb, re, slope,
                       static_cast<const unsigned char*>(img), bias, scale, shift, flags, out, ldo);
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
    hipStream_t st = as_stream(stream);
    auto* base = static_cast<unsigned char*>(img);
    int32_t* q = reinterpret_cast<int32_t*>(base + static_cast<size_t>(AKP) * ACB * 2 * AFRAG);
    hipLaunchKernelGGL(perm_exp_kernel, dim3(AH / 4), dim3(256), 0, st, w2, q);
    int rc = launch_status("perm_exp_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(perm_frag_kernel, dim3((AKP * ACB * 64 + 255) / 256), dim3(256), 0, st, w2,
                       q, base);
    return launch_status("perm_frag_kernel");
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
    if (g_agg_waves == 4)
        return launch_agg_gemm<AGG_GIN, true, 4>(row_ptr, col, nullptr, x, ldx, rb, re, s, img1, b1,
                                                 img2, b2, scale, shift, flags, out, ldo, st);
    return launch_agg_gemm<AGG_GIN, true, 8>(row_ptr, col, nullptr, x, ldx, rb, re, s, img1, b1,
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
    if (g_agg_waves == 4)
        return launch_agg_gemm<AGG_GCN, false, 4>(row_ptr, col, ew, x, ldx, rb, re, 1.f, img, bias,
                                                  nullptr, nullptr, scale, shift, flags, out, ldo, st);
    return launch_agg_gemm<AGG_GCN, false, 8>(row_ptr, col, ew, x, ldx, rb, re, 1.f, img, bias,
                                              nullptr, nullptr, scale, shift, flags, out, ldo, st);
}

extern "C" int mignn_diag_set_agg_gemm_waves(int waves) {
    MIGNN_REQUIRE(waves == 4 || waves == 8, "set_agg_gemm_waves: 4 or 8");
    g_agg_waves = waves;
    return MIGNN_OK;
}

// the fused GAT layer (see gat_fused_kernel); called by mignn_gat_layer when
// it has the split image of wcat, heads = 4 and h in {64, 128}
namespace mignn {
int gat_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* logits,
                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h, float slope,
                    const void* img, const float* bias, const float* scale, const float* shift,
                    int flags, float* out, int64_t ldo, void* stream) {
    MIGNN_REQUIRE(aligned16(x) && aligned16(out) && aligned16(img) && ldx % 4 == 0 && ldo % 4 == 0,
                  "gat_layer: fused path needs 16-B aligned rows");
    MIGNN_REQUIRE(x != out, "gat_layer: in-place not supported (neighbours read x)");
    hipStream_t st = as_stream(stream);
    return h == 128 ? launch_gat_fused<128>(row_ptr, col, logits, x, ldx, rb, re, slope, img, bias,
                                            scale, shift, flags, out, ldo, st)
                    : launch_gat_fused<64>(row_ptr, col, logits, x, ldx, rb, re, slope, img, bias,
                                           scale, shift, flags, out, ldo, st);
}
}  // namespace mignn
