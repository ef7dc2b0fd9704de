// Dense node transform in split-fp16 ("f16x3") MFMA arithmetic for the shapes
// the fused layer kernels do not cover (K or N > 128: the H = 256 layers of
// configs[3] / configs[4], GAT's head-mean GEMM, TransformerConv's Q~K and
// output GEMMs, the H = 256 output head):
//
//   C[m, n] = epi( sum_k [A | A2][m, k] * W[n, k] )        (torch Linear layout)
//
// Arithmetic (as gcn_f16x3.hip): every fp32 operand is split into fp16 hi + lo
// of a power-of-two-scaled value, a.w = 2^-(p+q) (ah wh + ah wl + al wh), three
// v_mfma_f32_16x16x32_f16 into one fp32 accumulator, ~2^-22 relative per
// product (16x the f32 MFMA rate: the GEMM drops to the HBM roofline).
//   * W: one exponent q_n per output column, split once per weight version
//     into an image of MFMA A-operand fragments (mignn_linear_f16x3_prep);
//   * A: an ONLINE exponent per row, as online softmax keeps its running max:
//     each 32-wide k chunk is split with the row's exponent so far, lowered
//     when the chunk's max needs it, and the row's accumulators are rescaled
//     by the (exact) power of two -- one pass over A, no pre-scan.
// Orientation D[n][row] = W . A^T: the A rows are the MFMA B operand (lane
// (r, g) loads row r's 8 values k = 32kc + 8g.., splits them in registers),
// the D fragment of lane (r, g) holds row r's columns 16cb + 4g + {0..3}: the
// epilogue stores 16 B per lane.
//
// Tiling: 512 threads = 8 waves x 16 RPW rows per block (RPW = 1: 128 rows,
// two blocks per CU), 256 output columns (16 column blocks) per block; W
// fragments of a k chunk (32 KB) LDS-DMA'd once per block, double-buffered,
// one barrier per chunk; A loads go straight to registers two chunks ahead.
// Blocks of consecutive tiles (the column tiles of a row tile first) share
// an XCD, so the A rows of the column tiles are L2 hits.
// Measured alternatives (scripts/gemm_bench.py, M = 2M rows, round 2):
// RPW = 2 (half the W traffic), BN = 128, a 2x4 wave grid over a block-split
// A image, and a persistent variant with 3-4-deep A prefetch across row
// tiles were all 0-25 % slower than this form.  What mattered was the
// compiler's wait placement: K-masking at load time, a conditional second
// step of the unrolled pair, or an LDS-DMA issued before a wait the compiler
// places made it wait for loads in flight (checked in the ISA).
#include "common.hpp"

namespace mignn {
MIGNN_DMA_OOB_WORD
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int GW = 8;                 // waves per block
constexpr int GNT = GW * 64;          // threads
#ifndef GEMM_NT
#define GEMM_NT 1   // non-temporal row stores (Q~K GEMM 4.88 -> 4.71 ms at M = 2M)
#endif
#ifndef GEMM_RPW
#define GEMM_RPW 1
#endif
constexpr int RPW = GEMM_RPW;         // 16-row blocks per wave
constexpr int GBM = 16 * RPW * GW;    // rows per block
#ifndef GEMM_CBT
#define GEMM_CBT 16
#endif
constexpr int CBT = GEMM_CBT;         // 16-column blocks per block
constexpr int GBN = 16 * CBT;         // columns per block
constexpr int FRAG = 64 * 16;         // bytes of one fragment (64 lanes x 8 halfs)
constexpr int CHUNK_BYTES = CBT * 2 * FRAG;   // one k chunk of a column tile: 32 KB

// max * 2^p in [2^13, 2^14); capped at 100 for zero / tiny maxima (2^p stays
// a normal float for every p this returns: p in [-115, 100])
__device__ __forceinline__ int sexp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 100);
}

__device__ __forceinline__ float p2(int p) {
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}

__device__ __forceinline__ uint32_t lds_addr_g(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(p)));
}

__device__ __forceinline__ void glds16_g(const void* src, uint32_t dst) {
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

// ---- image: [kc][cb (padded to CBT)][hi, lo][64 lanes][8 halfs], then q [NPB*16] int32
struct GImg {
    int kp, npb;        // k chunks, column blocks (multiple of CBT)
    __host__ __device__ static size_t frag_bytes(int kp, int npb) {
        return static_cast<size_t>(kp) * npb * 2 * FRAG;
    }
};

__global__ __launch_bounds__(256) void gprep_exp_kernel(const float* __restrict__ w, int n, int k,
                                                        int npb, int32_t* __restrict__ q) {
    // one wave per output column
    const int col = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (col >= npb * 16) return;
    uint32_t m = 0;
    if (col < n)
        for (int i = lane; i < k; i += 64) m = max(m, __float_as_uint(fabsf(w[(int64_t)col * k + i])));
    for (int o = 32; o > 0; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o)));
    if (lane == 0) q[col] = sexp(m);
}

__global__ __launch_bounds__(256) void gprep_frag_kernel(const float* __restrict__ w, int n, int k,
                                                         int kp, int npb,
                                                         const int32_t* __restrict__ q,
                                                         unsigned char* __restrict__ img) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (kc, cb, lane)
    if (t >= (int64_t)kp * npb * 64) return;
    const int lane = static_cast<int>(t & 63);
    const int cb = static_cast<int>((t >> 6) % npb);
    const int kc = static_cast<int>((t >> 6) / npb);
    const int col = 16 * cb + (lane & 15);
    const float sc = p2(q[col]);
    f16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = 32 * kc + 8 * (lane >> 4) + j;
        const float v = (col < n && kk < k) ? w[(int64_t)col * k + kk] * sc : 0.f;
        const _Float16 hh = static_cast<_Float16>(v);
        h[j] = hh;
        l[j] = static_cast<_Float16>(v - static_cast<float>(hh));
    }
    unsigned char* base = img + ((static_cast<size_t>(kc) * npb + cb) * 2) * FRAG + lane * 16;
    *reinterpret_cast<f16x8*>(base) = h;
    *reinterpret_cast<f16x8*>(base + FRAG) = l;
}

// 8 A values of row `row` at k = kk..kk+7 from [A | A2] (k1 % 4 == 0: each
// 4-float group lies in one segment).  Exactly one load per group, also past
// K (a dummy read of k = 0, which the caller zeroes when it consumes the
// values -- masking here would make the compiler wait for the load at once):
// the chunk loop's vmcnt bookkeeping counts on two loads per call.
__device__ __forceinline__ void load_a8(const float* __restrict__ A, int64_t lda,
                                        const float* __restrict__ A2, int64_t lda2, int k1, int K,
                                        int64_t row, int kk, f32x4& lo4, f32x4& hi4) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = kk + 4 * h;
        const int kr = k < K ? k : 0;
        const float* p = kr < k1 ? A + row * lda + kr : A2 + row * lda2 + (kr - k1);
        const f32x4 v = *reinterpret_cast<const f32x4*>(p);   // past K: zeroed by the user
        if (h == 0) lo4 = v; else hi4 = v;
    }
}

// EPIF: the flags at compile time (the callers' common sets, no diagnostic
// bits), -1: `flags`
template <int EPIF = -1>
__global__ __launch_bounds__(GNT, RPW == 1 ? 2 : 1) void gemm_f16x3_kernel(
    const float* __restrict__ A, int64_t lda, int64_t M, int k1, const float* __restrict__ A2,
    int64_t lda2, int K, const unsigned char* __restrict__ img, int kp, int npb, int N,
    const float* __restrict__ bias, const float* __restrict__ R, int64_t ldr,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ C, int64_t ldc, int64_t ntiles_m, int ntiles_n) {
    if constexpr (EPIF >= 0) flags = EPIF;
    __shared__ __attribute__((aligned(16))) unsigned char lds[2 * CHUNK_BYTES + GBN * 16];
    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;

    // tile of this block: the XCDs take contiguous runs of the (row tile,
    // column tile) sequence, column tiles of a row tile adjacent
    const int64_t nb = (int64_t)gridDim.x;
    const int64_t lin = (int64_t)(blockIdx.x & 7) * (nb >> 3) + (blockIdx.x >> 3);
    if (lin >= ntiles_m * ntiles_n) return;
    const int64_t tm = lin / ntiles_n;
    const int tn = static_cast<int>(lin - tm * ntiles_n);
    // my two rows: RPW = 2 row blocks of 16 per wave
    const int64_t row0 = tm * GBM + RPW * 16 * wave;
    int64_t row[RPW], rowl[RPW];
#pragma unroll
    for (int h = 0; h < RPW; ++h) {
        row[h] = row0 + 16 * h + r;
        const int64_t rc = row[h] < M ? row[h] : M - 1;
        // MIGNN_DIAG_NO_PRODUCE: the loads all read row 0 (L2 hits; not skipped
        // -- a conditional load would make the compiler wait for it)
        rowl[h] = (flags & MIGNN_DIAG_NO_PRODUCE) ? 0 : rc;
    }
    const int cb0 = tn * CBT;                       // first column block of the tile
    const int ncb = min(CBT, (N + 15) / 16 - cb0);  // column blocks with columns (uniform)

    // per-column W exponents and epilogue vectors of the tile -> LDS
    int32_t* const QL = reinterpret_cast<int32_t*>(lds + 2 * CHUNK_BYTES);
    float* const BL = reinterpret_cast<float*>(lds + 2 * CHUNK_BYTES + GBN * 4);
    float* const SL = BL + GBN;
    float* const HL = SL + GBN;
    if (tid < GBN) {
        const int col = cb0 * 16 + tid;
        const int32_t* qimg = reinterpret_cast<const int32_t*>(img + GImg::frag_bytes(kp, npb));
        QL[tid] = qimg[col];
        BL[tid] = (col < N && (flags & MIGNN_EPI_BIAS)) ? bias[col] : 0.f;
        SL[tid] = (col < N && (flags & MIGNN_EPI_AFFINE)) ? scale[col] : 1.f;
        HL[tid] = (col < N && (flags & MIGNN_EPI_AFFINE)) ? shift[col] : 0.f;
    }

    // W chunk kc of this column tile -> LDS buffer (kc & 1): 32 pieces of 1 KB
    auto w_dma = [&](int kc) {
        if (kc >= kp) return;
        const unsigned char* src = img + ((static_cast<size_t>(kc) * npb + cb0) * 2) * FRAG;
        unsigned char* dst = lds + (kc & 1) * CHUNK_BYTES;
#pragma unroll
        for (int pc = 0; pc < CHUNK_BYTES / 1024 / GW; ++pc) {
            const int piece = wave + pc * GW;   // fragment (column block piece / 2, hi | lo)
            // column blocks past N (zero padding of a narrow tile, e.g. GAT's
            // N = 128 head-mean GEMM): not copied, their MFMAs are skipped.
            // (Uniform per wave; fewer DMA pieces only make the counted
            // vmcnt waits below more conservative.)
            if ((piece >> 1) >= ncb) continue;
            glds16_g(src + piece * 1024 + lane * 16, lds_addr_g(dst + piece * 1024));
        }
    };

    f32x4 acc[RPW][CBT];
#pragma unroll
    for (int h = 0; h < RPW; ++h)
#pragma unroll
        for (int i = 0; i < CBT; ++i) acc[h][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int p[RPW];                                     // the rows' running exponents
#pragma unroll
    for (int h = 0; h < RPW; ++h) p[h] = 100;

    // A chunks in two register buffers (even / odd chunks), the k loop
    // unrolled by two so no buffer is ever copied: a copy would wait for the
    // load in flight and serialise the HBM latency into every chunk
    using AB = f32x4[RPW][2];
    AB xa, ya;
#pragma unroll
    for (int h = 0; h < RPW; ++h) {
        load_a8(A, lda, A2, lda2, k1, K, rowl[h], 8 * g, xa[h][0], xa[h][1]);
        load_a8(A, lda, A2, lda2, k1, K, rowl[h], 32 + 8 * g, ya[h][0], ya[h][1]);
    }
    w_dma(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0x70);              // vmcnt(0): chunk 0's W landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    auto step = [&](int kc, AB& va) {
        f16x8 bh[RPW], bl[RPW];
#pragma unroll
        for (int h = 0; h < RPW; ++h) {
            // this chunk's 8 values of row h (zero past K); the row max over its 4 lanes
            f32x4 vl = va[h][0], vh = va[h][1];
            if (32 * kc + 8 * g >= K) vl = f32x4{0.f, 0.f, 0.f, 0.f};
            if (32 * kc + 8 * g + 4 >= K) vh = f32x4{0.f, 0.f, 0.f, 0.f};
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                m = max(m, max(__float_as_uint(fabsf(vl[j])), __float_as_uint(fabsf(vh[j]))));
            {   // max over the row's 4 lanes (l, l^16, l^32, l^48): VALU lane
                // swaps instead of two LDS-crossbar shuffles (0.5-2 % per GEMM)
                const auto r16 = __builtin_amdgcn_permlane16_swap(m, m, false, false);
                m = max(static_cast<uint32_t>(r16[0]), static_cast<uint32_t>(r16[1]));
                const auto r32 = __builtin_amdgcn_permlane32_swap(m, m, false, false);
                m = max(static_cast<uint32_t>(r32[0]), static_cast<uint32_t>(r32[1]));
            }
            const int pc = sexp(m);
            if (pc < p[h]) {                        // lower the row's scale: exact rescale
#pragma unroll
                for (int i = 0; i < CBT; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[h][i][j] = ldexpf(acc[h][i][j], pc - p[h]);
                p[h] = pc;
            }
            const float sp = p2(p[h]);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = (j < 4 ? vl[j] : vh[j - 4]) * sp;
                const _Float16 hh = static_cast<_Float16>(v);
                bh[h][j] = hh;
                bl[h][j] = static_cast<_Float16>(v - static_cast<float>(hh));
            }
        }
        // next chunk's W into the other buffer -- after the split: the compiler
        // does not count the DMA, so a wait it places for the split's registers
        // must not have DMAs behind it
        w_dma(kc + 1);
        // the buffers are free: chunk kc+2 into them (2 loads per row, always issued)
#pragma unroll
        for (int h = 0; h < RPW; ++h)
            load_a8(A, lda, A2, lda2, k1, K, rowl[h], 32 * (kc + 2) + 8 * g, va[h][0], va[h][1]);
        const unsigned char* wb = lds + (kc & 1) * CHUNK_BYTES + lane * 16;
        // all CBT column blocks: the image pads a partial tile with zero columns
#pragma unroll
        for (int cb = 0; cb < CBT; ++cb) {
            // column blocks past N (a ragged last column tile, e.g. the 4
            // per-head columns of TransformerConv's Q~K GEMM, N = 4H + 4):
            // no MFMAs (uniform branch, nothing in flight behind it)
            if ((flags & MIGNN_DIAG_NO_MFMA) || cb >= ncb) break;
            const f16x8 wh = *reinterpret_cast<const f16x8*>(wb + (2 * cb) * FRAG);
            const f16x8 wl = *reinterpret_cast<const f16x8*>(wb + (2 * cb + 1) * FRAG);
#pragma unroll
            for (int h = 0; h < RPW; ++h) {
                acc[h][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh[h], acc[h][cb], 0, 0, 0);
                acc[h][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl[h], acc[h][cb], 0, 0, 0);
                acc[h][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, bh[h], acc[h][cb], 0, 0, 0);
            }
        }
        // the next chunk's W must have landed before anyone reads it, and
        // every wave be done with this buffer before chunk kc+2 refills it;
        // vmcnt(2 RPW): only the A loads just issued may still fly
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0x70 | (2 * RPW));
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    // (unconditional pairs: on the back edge the compiler then knows the
    // explicit vmcnt has retired the buffer the next step reads)
    int kc = 0;
    for (; kc + 1 < kp; kc += 2) {
        step(kc, xa);
        step(kc + 1, ya);
    }
    if (kc < kp) step(kc, xa);

    // epilogue: D[n][row] in lane (r, g): columns 16cb + 4g + i of my rows
    if (flags & MIGNN_DIAG_NO_EXT) return;
    // Staged stores (RPW = 1, 16-B aligned C rows): the accumulator layout
    // would store 16 rows x 64 B per instruction; instead each wave writes
    // half its 16 x 256 tile (8 column blocks) into its own 8 KB of the W
    // chunk buffers (free after the k loop's last barrier) and stores rows:
    // a half-wave per 512-B row segment (hot-kernel measurement: whole rows
    // stream ~1.2-1.5x faster).
    const bool staged = RPW == 1 && !(flags & MIGNN_DIAG_PLAIN_STORE) &&
                        (((uintptr_t)C) & 15) == 0 && (ldc & 3) == 0;
    if (staged) {
        unsigned char* const stg = lds + wave * 8192;
        const int64_t rbase = tm * GBM + 16 * wave;         // first row of this wave
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            if (8 * hf >= ncb) break;          // a half tile past N: nothing to store
#pragma unroll
            for (int c8 = 0; c8 < 8; ++c8) {
                const int cb = 8 * hf + c8;
                const int lc = 16 * cb + 4 * g;                 // column in the tile
                const int col = cb0 * 16 + lc;
                const int4 qv = *reinterpret_cast<const int4*>(&QL[lc]);
                const f32x4 bo = *reinterpret_cast<const f32x4*>(&BL[lc]);
                const f32x4 so = *reinterpret_cast<const f32x4*>(&SL[lc]);
                const f32x4 ho = *reinterpret_cast<const f32x4*>(&HL[lc]);
                const float4 rv = (flags & MIGNN_EPI_RESIDUAL) && row[0] < M
                                      ? ld4_masked(R + row[0] * ldr, col, N)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
                const int qn[4] = {qv.x, qv.y, qv.z, qv.w};
                const float res[4] = {rv.x, rv.y, rv.z, rv.w};
                f32x4 o;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    o[i] = epilogue(ldexpf(acc[0][cb][i], -(p[0] + qn[i])), flags, bo[i], res[i],
                                    so[i], ho[i]);
                // row r, 16-B chunk 4 c8 + g of the half, at chunk ^ r
                const int ch = 4 * c8 + g;
                *reinterpret_cast<f32x4*>(stg + r * 512 + ((ch ^ r) << 4)) = o;
            }
            // rows out: instruction i = rows 2i, 2i+1 (lanes 0-31 / 32-63), 16 B per lane
            const int ch = lane & 31;
            const int col = cb0 * 16 + 128 * hf + 4 * ch;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int rr = 2 * i + (lane >> 5);
                const f32x4 v = *reinterpret_cast<const f32x4*>(stg + rr * 512 + ((ch ^ rr) << 4));
                const int64_t grow = rbase + rr;
                if (grow < M && col < N) {
                    float* dst = C + grow * ldc + col;
                    if (col + 4 <= N) {
#if GEMM_NT
                        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
#else
                        *reinterpret_cast<f32x4*>(dst) = v;
#endif
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (col + j < N) dst[j] = v[j];
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int h = 0; h < RPW; ++h) {
        if (row[h] >= M) continue;
#pragma unroll
        for (int cb = 0; cb < CBT; ++cb) {
            if (cb < ncb) {
                const int lc = 16 * cb + 4 * g;                 // column in the tile
                const int col = cb0 * 16 + lc;
                const int4 qv = *reinterpret_cast<const int4*>(&QL[lc]);
                const f32x4 bo = *reinterpret_cast<const f32x4*>(&BL[lc]);
                const f32x4 so = *reinterpret_cast<const f32x4*>(&SL[lc]);
                const f32x4 ho = *reinterpret_cast<const f32x4*>(&HL[lc]);
                const float4 rv = (flags & MIGNN_EPI_RESIDUAL)
                                      ? ld4_masked(R + row[h] * ldr, col, N)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
                const int qn[4] = {qv.x, qv.y, qv.z, qv.w};
                const float res[4] = {rv.x, rv.y, rv.z, rv.w};
                float o[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    o[i] = epilogue(ldexpf(acc[h][cb][i], -(p[h] + qn[i])), flags, bo[i], res[i],
                                    so[i], ho[i]);
                float* dst = C + row[h] * ldc + col;
                if (col + 4 <= N && (((uintptr_t)dst) & 15) == 0) {
                    *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (col + i < N) dst[i] = o[i];
                }
            }
        }
    }
}

}  // namespace
}  // namespace mignn

using namespace mignn;

static int linear_f16x3_impl(const float* a, int64_t lda, int64_t m, int k1,
                                       const float* a2, int64_t lda2, int k2, const void* img,
                                       int n, const float* bias, const float* residual,
                                       int64_t ldr, const float* scale, const float* shift,
                                       int flags, float* c, int64_t ldc, void* stream);

extern "C" size_t mignn_linear_f16x3_prep_bytes(int n, int k) {
    if (n <= 0 || k <= 0) return 0;
    const int kp = (k + 31) / 32;
    const int npb = ((n + 15) / 16 + CBT - 1) / CBT * CBT;
    return GImg::frag_bytes(kp, npb) + static_cast<size_t>(npb) * 16 * 4;
}

extern "C" int mignn_linear_f16x3_prep(const float* w, int n, int k, void* img, size_t img_bytes,
                                       void* stream) {
    MIGNN_REQUIRE(w && img && n > 0 && k > 0, "linear_f16x3_prep: bad arguments");
    MIGNN_REQUIRE(img_bytes >= mignn_linear_f16x3_prep_bytes(n, k), "linear_f16x3_prep: image too small");
    MIGNN_REQUIRE(aligned16(img), "linear_f16x3_prep: image not 16-B aligned");
    const int kp = (k + 31) / 32;
    const int npb = ((n + 15) / 16 + CBT - 1) / CBT * CBT;
    hipStream_t st = as_stream(stream);
    auto* base = static_cast<unsigned char*>(img);
    int32_t* q = reinterpret_cast<int32_t*>(base + GImg::frag_bytes(kp, npb));
    hipLaunchKernelGGL(gprep_exp_kernel, dim3((npb * 16 + 3) / 4), dim3(256), 0, st, w, n, k, npb, q);
    int rc = launch_status("gprep_exp_kernel");
    if (rc) return rc;
    const int64_t nt = (int64_t)kp * npb * 64;
    hipLaunchKernelGGL(gprep_frag_kernel, dim3(static_cast<unsigned>((nt + 255) / 256)), dim3(256), 0,
                       st, w, n, k, kp, npb, q, base);
    return launch_status("gprep_frag_kernel");
}

extern "C" int mignn_linear_f16x3(const float* a, int64_t lda, int64_t m, int k1, const float* a2,
                                  int64_t lda2, int k2, const void* img, int n, const float* bias,
                                  const float* residual, int64_t ldr, const float* scale,
                                  const float* shift, int flags, float* c, int64_t ldc,
                                  void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "linear_f16x3: unknown flags 0x%x", flags);
    return linear_f16x3_impl(a, lda, m, k1, a2, lda2, k2, img, n, bias, residual, ldr, scale,
                                   shift, flags, c, ldc, stream);
}

static int linear_f16x3_impl(const float* a, int64_t lda, int64_t m, int k1,
                                       const float* a2, int64_t lda2, int k2, const void* img,
                                       int n, const float* bias, const float* residual,
                                       int64_t ldr, const float* scale, const float* shift,
                                       int flags, float* c, int64_t ldc, void* stream) {
    MIGNN_REQUIRE(m >= 0 && k1 > 0 && k2 >= 0 && n > 0, "linear_f16x3: bad sizes");
    MIGNN_REQUIRE(k1 % 4 == 0 && k2 % 4 == 0 && lda % 4 == 0 && (k2 == 0 || lda2 % 4 == 0),
                  "linear_f16x3: k and lda must be multiples of 4");
    MIGNN_REQUIRE(a && img && c && aligned16(a) && aligned16(img) && (k2 == 0 || (a2 && aligned16(a2))),
                  "linear_f16x3: null or unaligned operand");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "linear_f16x3: bias flag without bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_RESIDUAL) || residual, "linear_f16x3: residual flag without R");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "linear_f16x3: affine w/o params");
    if (m == 0) return MIGNN_OK;
    const int K = k1 + k2;
    const int kp = (K + 31) / 32;
    const int npb = ((n + 15) / 16 + CBT - 1) / CBT * CBT;
    const int64_t tmr = (m + GBM - 1) / GBM;
    const int tnr = npb / CBT;
    int64_t nb = ((tmr * tnr + 7) / 8) * 8;
    MIGNN_REQUIRE(nb < (int64_t(1) << 31), "linear_f16x3: m too large");
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(nb)), dim3(GNT), 0, as_stream(stream), a,
                           lda, m, k1, k2 ? a2 : a, lda2, K, static_cast<const unsigned char*>(img),
                           kp, npb, n, bias, residual, ldr, scale, shift, flags, c, ldc, tmr, tnr);
    };
    constexpr int kB = MIGNN_EPI_BIAS, kBR = MIGNN_EPI_BIAS | MIGNN_EPI_RELU;
    constexpr int kNoBN = MIGNN_EPI_BIAS | MIGNN_EPI_RESIDUAL | MIGNN_EPI_RELU;
    constexpr int kBN = kNoBN | MIGNN_EPI_AFFINE;
    switch (flags) {
        case 0: go(gemm_f16x3_kernel<0>); break;
        case kB: go(gemm_f16x3_kernel<kB>); break;
        case kBR: go(gemm_f16x3_kernel<kBR>); break;
        case kNoBN: go(gemm_f16x3_kernel<kNoBN>); break;
        case kBN: go(gemm_f16x3_kernel<kBN>); break;
        default: go(gemm_f16x3_kernel<>); break;
    }
    return launch_status("gemm_f16x3_kernel");
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_linear_f16x3(const float* a, int64_t lda, int64_t m, int k1,
                                       const float* a2, int64_t lda2, int k2, const void* img,
                                       int n, const float* bias, const float* residual,
                                       int64_t ldr, const float* scale, const float* shift,
                                       int flags, float* c, int64_t ldc, void* stream) {
    return linear_f16x3_impl(a, lda, m, k1, a2, lda2, k2, img, n, bias, residual, ldr, scale, shift, flags, c, ldc, stream);
}
#endif

MIGNN_DMA_OOB_EXPORT(mignn_diag_dma_oob_gemm)
