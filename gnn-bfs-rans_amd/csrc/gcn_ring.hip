// Fused GCN layer, split-fp16 MFMA, "tile ring" variant -- the north-star hot
// kernel (GCNConv + residual + BatchNorm(eval) + ReLU, reference
// gnn_model.py:166, :184-191; PyG GCNConv with gcn_norm weights):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Arithmetic: as gcn_f16x3.hip (every fp32 operand of the transform split
// into power-of-two-scaled fp16 hi + lo; three v_mfma_f32_16x16x32_f16 per
// product block into one fp32 accumulator; ~2^-22 relative per product).
//
// Structure (why): a plain CSR gather of 7 neighbour rows through L1/L2 runs
// at ~3.5 ms per 10M-node layer on MI355X -- the per-CU L2 gather rate, not
// HBM, binds.  So every row should enter a CU once and its repeated
// neighbour reads be served from LDS:
//   * one 256-thread workgroup per CU (4 waves, one per SIMD), persistent;
//     it walks a contiguous run of 64-row tiles (segments of `seg_tiles`
//     tiles, XCD-aware: the 8 XCDs get disjoint blocks of segments);
//   * an LDS ring of NSLOT tile images holds the tiles of the previous, the
//     current and the next step (plus tiles in flight, LDS-DMA, D steps
//     ahead).  In a locality order (mignn_locality_order: k-pencils of the
//     mesh) the +-k neighbours of a tile are the previous / next tile, so
//     nearly every CSR entry is an LDS read;
//   * the few entries outside the ring ("ext") are gathered into registers
//     one step ahead (EX slots per row; more: synchronous loads);
//   * each wave owns 16 rows of the tile end to end: lane (r, g) aggregates
//     the 16-B chunks {4i + g} of row r in registers, so its fp32 sums ARE
//     the MFMA B fragment (k permuted: fragment kc of lane g holds columns
//     32kc + 4g + {0..3} and 32kc + 16 + 4g + {0..3}); the whole split W
//     (H x H, hi and lo, same k permutation) stays in registers for the
//     launch; the MFMA output D[n][r] lands in the lane that owns row r, at
//     exactly the columns whose residual it reads -- no LDS hand-off, no
//     producer / consumer split, one barrier per tile step (ring reuse).
// Sum order of a row: its ring entries (CSR order), then its first EX ext
// entries (CSR order); rows with more ext entries or > MAXE entries: the rest
// in CSR order, then the EX ext slots -- deterministic run to run.
#include "common.hpp"

namespace mignn {
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int H>
struct RCfg {
    static_assert(H == 64 || H == 128, "ring GCN layer: H in {64, 128}");
    static constexpr int BM = 64;                  // rows per tile
    static constexpr int NW = 4;                   // waves, 16 rows each
    static constexpr int NT = NW * 64;
    static constexpr int NCH = H / 16;             // 16-B chunks per lane of a row
    static constexpr int NCB = H / 16;             // 16-column output blocks
    static constexpr int KC = H / 32;              // 32-deep k chunks
    static constexpr int CPR = H / 4 + 1;          // 16-B chunks per padded image row
    static constexpr int PITCH = CPR * 16;         // image row pitch (one pad chunk)
    static constexpr int SLOT = BM * PITCH;        // one tile image
    static constexpr int PIECES = BM * CPR / 64;   // 1-KB LDS-DMA pieces per tile
    static_assert((BM * CPR) % 64 == 0, "pieces");
    static constexpr int NSLOT = H == 128 ? 4 : 8;
    static constexpr int D = NSLOT - 2;            // DMA lead (steps)
    static constexpr int EX = 2;                   // ext register slots per row
    static constexpr int MAXE = 8;                 // entries per row on the fast path
    static constexpr int OFF_EPI = NSLOT * SLOT;   // bias | scale | shift [H]
    static constexpr int LDS_BYTES = OFF_EPI + 3 * H * 4;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ int scale_exp_r(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}

__device__ __forceinline__ float pow2f(int p) {   // 2^p, p in [-126, 127]
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}

__device__ __forceinline__ uint32_t wave_max_u32_r(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), o)));
    return v;
}

// One 16-column output block: c += sum_kc (wh wl)[kc] x (bh bl)[kc] as 3 fp16
// MFMAs per k chunk (hi.hi, hi.lo, lo.hi).  Inline asm so that the split W
// stays in AGPRs as the MFMA A operand for the whole launch (with the
// builtin the compiler keeps A operands in VGPRs and shuttles W through
// v_accvgpr_read every step).  The leading s_nop covers VALU writes of the B
// fragments / seed just before; the caller pads before reading c with the
// VALU (16x16x32 f16: 8 passes).
template <int KC>
__device__ __forceinline__ f32x4 mfma_block(const f16x8 (&wh)[KC], const f16x8 (&wl)[KC],
                                            const f16x8 (&bh)[KC], const f16x8 (&bl)[KC],
                                            f32x4 c) {
    static_assert(KC == 2 || KC == 4, "KC");
    if constexpr (KC == 4) {
        asm("s_nop 4\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %1, %9, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %1, %13, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %5, %9, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %2, %10, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %2, %14, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %6, %10, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %11, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %15, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %7, %11, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %12, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %16, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %8, %12, %0"
            : "+v"(c)
            : "a"(wh[0]), "a"(wh[1]), "a"(wh[2]), "a"(wh[3]), "a"(wl[0]), "a"(wl[1]),
              "a"(wl[2]), "a"(wl[3]), "v"(bh[0]), "v"(bh[1]), "v"(bh[2]), "v"(bh[3]),
              "v"(bl[0]), "v"(bl[1]), "v"(bl[2]), "v"(bl[3]));
    } else {
        asm("s_nop 4\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %1, %5, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %1, %7, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %3, %5, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %2, %6, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %2, %8, %0\n\t"
            "v_mfma_f32_16x16x32_f16 %0, %4, %6, %0"
            : "+v"(c)
            : "a"(wh[0]), "a"(wh[1]), "a"(wl[0]), "a"(wl[1]), "v"(bh[0]), "v"(bh[1]),
              "v"(bl[0]), "v"(bl[1]));
    }
    return c;
}

__device__ __forceinline__ uint32_t lds_addr_r(const unsigned char* p) {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_ptr_t)(p)));
}

// LDS-DMA of 16 B per lane to LDS address dst + 16 * lane (global_load_lds_dwordx4);
// inline asm: the compiler does not count it, the wave waits for it itself
__device__ __forceinline__ void glds16_r(const void* src, uint32_t dst) {
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

template <int VMCNT>
__device__ __forceinline__ void wait_barrier() {
    static_assert(VMCNT < 64, "vmcnt");
    asm volatile("" ::: "memory");
    // vmcnt(n): bits [3:0] = n & 15, [15:14] = n >> 4; lgkmcnt(0); expcnt(7)
    __builtin_amdgcn_s_waitcnt((VMCNT & 15) | ((VMCNT >> 4) << 14) | (7 << 4));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Diagnostic timeline (mignn_diag_set_trace_ring): s_memtime of wave 0 of
// workgroups 0..7 at the phase boundaries of steps 0..63 -> trace[(b*64+s)*16+k]
__device__ __forceinline__ void rstamp(unsigned long long* trace, int lane, int wave, int64_t s,
                                       int k) {
    if (trace != nullptr && blockIdx.x < 8 && wave == 0 && s >= 0 && s < 64) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (lane == 0) trace[(blockIdx.x * 64 + s) * 16 + k] = t;
        __builtin_amdgcn_sched_barrier(0);
    }
}
unsigned long long* g_ring_trace = nullptr;   // set by mignn_diag_set_trace_ring

template <int H>
__global__ __launch_bounds__(256, 1) void gcn_ring_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t row_begin,
    int64_t row_end, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo, int64_t seg_tiles, unsigned long long* trace) {
    using C = RCfg<H>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    float* const EPI = reinterpret_cast<float*>(lds + C::OFF_EPI);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;

    // ---- schedule: segment sid = tiles [sid*T, sid*T + T); round q of this
    // workgroup takes segment q*G + mapb, mapb XCD-blocked (blocks b, b+8, ...
    // share an XCD and take consecutive segments)
    const int64_t nrows = row_end - row_begin;
    const int64_t ntiles = (nrows + C::BM - 1) / C::BM;
    const int G = gridDim.x;
    const int64_t mapb = (int64_t)(blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
    const int64_t T = seg_tiles;
    int64_t nsteps = 0;
    for (int64_t q = 0;; ++q) {
        const int64_t t0 = (q * G + mapb) * T;
        if (t0 >= ntiles) break;
        nsteps += min(T, ntiles - t0);
    }
    // tiles of steps s-1 .. s+WIN-2 (tw[k] = tile of step s-1+k, -1 past the
    // end), advanced one step at a time (no 64-bit divisions in the loop)
    constexpr int WIN = (C::D > 3 ? C::D : 3) + 2;
    int64_t tw[WIN];
    int64_t gq = 0, gj = 0, gs = 0;   // generator: next step to produce = gs
    auto gen_next = [&]() -> int64_t {
        if (gs >= nsteps) return -1;
        const int64_t t = (gq * G + mapb) * T + gj;
        ++gs;
        if (++gj == T) { gj = 0; ++gq; }
        return t;
    };
    tw[0] = -1;
#pragma unroll
    for (int k = 1; k < WIN; ++k) tw[k] = gen_next();

    // ---- W as split fp16 MFMA A-operands, one exponent for the matrix:
    // lane (n, g) of block (cb, kc) holds W[16cb + n][32kc + 4g + j] (j < 4)
    // and W[16cb + n][32kc + 16 + 4g + j - 4] (j >= 4)
    f16x8 wh[C::NCB][C::KC], wl[C::NCB][C::KC];
    int qw;
    {
        uint32_t m = 0;
        for (int i = lane; i < H * H / 4; i += 64) {
            const float4 v = ld4(W + 4 * i);
            m = max(m, max(max(__float_as_uint(fabsf(v.x)), __float_as_uint(fabsf(v.y))),
                           max(__float_as_uint(fabsf(v.z)), __float_as_uint(fabsf(v.w)))));
        }
        qw = scale_exp_r(wave_max_u32_r(m));
        const float sq = pow2f(qw);
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb)
#pragma unroll
            for (int kc = 0; kc < C::KC; ++kc) {
                const float* p = W + (int64_t)(16 * cb + r) * H + 32 * kc + 4 * g;
                const float4 a = ld4(p), b = ld4(p + 16);
                const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float s = v[j] * sq;
                    const _Float16 hh = static_cast<_Float16>(s);
                    wh[cb][kc][j] = hh;
                    wl[cb][kc][j] = static_cast<_Float16>(s - static_cast<float>(hh));
                }
            }
    }
    if (tid < H) {
        EPI[tid] = (flags & MIGNN_EPI_BIAS) ? bias[tid] : 0.f;
        EPI[H + tid] = (flags & MIGNN_EPI_AFFINE) ? scale[tid] : 1.f;
        EPI[2 * H + tid] = (flags & MIGNN_EPI_AFFINE) ? shift[tid] : 0.f;
    }

    // ---- LDS-DMA of a tile into its ring slot: image position P (16-B
    // chunks, CPR per padded row) = row P / CPR, chunk P % CPR (the pad chunk
    // reads chunk 0 again); this wave's pieces: wave, wave + 4, ... -- the
    // per-lane (row, chunk) of each piece is the same for every tile
    constexpr int PPW = (C::PIECES + C::NW - 1) / C::NW;
    const uint32_t ldx32 = static_cast<uint32_t>(ldx);
    const int re32 = static_cast<int>(row_end);
    auto dma_tile = [&](int64_t tile, int64_t s) {
        if (tile < 0) return;
        const int64_t t0 = row_begin + tile * C::BM;
        const float* const xt = x + t0 * ldx;
        unsigned char* const slot = lds + (s & (C::NSLOT - 1)) * C::SLOT;
        const int nlast = static_cast<int>(row_end - 1 - t0);   // last valid tile row
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int p = wave + q * C::NW;
            if (p < C::PIECES) {
                const int P = p * 64 + lane;
                int lr = P / C::CPR;
                int ch = P - lr * C::CPR;
                ch = ch < H / 4 ? ch : 0;
                lr = lr < nlast ? lr : nlast;                   // past the last row: any valid row
                glds16_r(xt + (static_cast<uint32_t>(lr) * ldx32 + 4u * static_cast<uint32_t>(ch)),
                         lds_addr_r(slot + p * 1024));
            }
        }
    };

    // ---- CSR indices of a step's rows (lane (r, g): row 16 wave + r)
    struct Idx {
        int rlo, rhi;          // row_ptr of my row (empty row past row_end)
        int c0, c1;            // lane t: col of entry e0 + t, e0 + 64 + t
        float w0, w1;
    };
    auto load_rp = [&](int64_t tile, Idx& ix) {
        if (tile < 0) { ix.rlo = ix.rhi = 0; return; }
        int64_t row = row_begin + tile * C::BM + 16 * wave + r;
        const int64_t a = row < row_end ? row : row_end;
        const int64_t b = row < row_end ? row + 1 : row_end;
        ix.rlo = row_ptr[a];
        ix.rhi = row_ptr[b];
    };
    auto load_cols = [&](Idx& ix) {
        const int e0 = __builtin_amdgcn_readlane(ix.rlo, 0);
        const int ne = __builtin_amdgcn_readlane(ix.rhi, 15) - e0;
        ix.c0 = lane < ne ? col[e0 + lane] : 0;
        ix.w0 = lane < ne ? ew[e0 + lane] : 0.f;
        ix.c1 = lane + 64 < ne ? col[e0 + 64 + lane] : 0;
        ix.w1 = lane + 64 < ne ? ew[e0 + 64 + lane] : 0.f;
    };
    // max over rows 0..15 (lanes 0..15 hold every row once): DPP row shifts
    auto max_rows = [&](int v) -> int {
        v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false));   // row_shr:1
        v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false));   // row_shr:2
        v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false));   // row_shr:4
        v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false));   // row_shr:8
        return __builtin_amdgcn_readlane(v, 15);
    };
    // the ring of a step: its tile's first row, whether the tiles of the
    // previous / next step are the adjacent tiles, and the step (slot base)
    struct Ring {
        int row0;        // first row of the step's tile (row ids fit in int32)
        bool lo, hi;
        int s;           // the step (mod NSLOT)
    };
    // LDS byte offset of source row c's image (+ 16 g) in the ring, or -1 (ext)
    auto classify = [&](int c, const Ring& R) -> int {
        const int d = c - R.row0 + C::BM;                 // 0..3*BM-1 inside the ring
        const bool in = static_cast<unsigned>(d) < 3u * C::BM && c < re32 &&
                        (d >= C::BM || R.lo) && (d < 2 * C::BM || R.hi);
        const int slot = (R.s - 1 + (d >> 6)) & (C::NSLOT - 1);
        return in ? slot * C::SLOT + (d & 63) * C::PITCH + 16 * g : -1;
    };
    auto entry_cw = [&](const Idx& ix, int u, int& c, float& w) {
        const int a = (u & 63) << 2;
        const int c0 = __builtin_amdgcn_ds_bpermute(a, ix.c0);
        const int c1 = __builtin_amdgcn_ds_bpermute(a, ix.c1);
        const int w0 = __builtin_amdgcn_ds_bpermute(a, __float_as_int(ix.w0));
        const int w1 = __builtin_amdgcn_ds_bpermute(a, __float_as_int(ix.w1));
        c = u < 64 ? c0 : c1;
        w = __int_as_float(u < 64 ? w0 : w1);
    };

    // ---- decoded entries of a step (lane (r, g): row r, CSR order)
    //   ring entries -> la[e] (LDS byte offset of the row's chunk g), lw[e];
    //   the first EX ext entries -> register slots, gathered here (empty
    //   slots read my own row with weight 0: a fixed instruction count);
    //   slow = a row with > MAXE entries, > EX ext entries, or > 128 entries
    //   in the wave's rows: that step runs the generic loop instead
    struct Dec {
        int la[C::MAXE];
        float lw[C::MAXE];
        int maxdeg;
        bool slow;
    };
    using XV = f32x4[C::EX][C::NCH];
    auto decode = [&](const Idx& ix, const Ring& R, Dec& dc, XV& xv, float (&wx)[C::EX]) {
        const int e0 = __builtin_amdgcn_readlane(ix.rlo, 0);
        const int ne = __builtin_amdgcn_readlane(ix.rhi, 15) - e0;
        const int rs = ix.rlo - e0, deg = ix.rhi - ix.rlo;
        const int maxdeg = max_rows(deg);
        dc.maxdeg = maxdeg;
        const int dummy = R.s * C::SLOT + (16 * wave + r) * C::PITCH + 16 * g;
        int cx[C::EX];
#pragma unroll
        for (int kk = 0; kk < C::EX; ++kk) { cx[kk] = -1; wx[kk] = 0.f; }
        int k = 0;
        const bool fast = maxdeg <= C::MAXE && ne <= 128;
        if (fast) {
            int cc[C::MAXE];
            float ww[C::MAXE];
#pragma unroll
            for (int e = 0; e < C::MAXE; ++e) entry_cw(ix, rs + (e < deg ? e : 0), cc[e], ww[e]);
#pragma unroll
            for (int e = 0; e < C::MAXE; ++e) {
                const bool valid = e < deg;
                const int la = classify(cc[e], R);
                dc.la[e] = (valid && la >= 0) ? la : dummy;
                dc.lw[e] = (valid && la >= 0) ? ww[e] : 0.f;
                const bool isext = valid && la < 0;
#pragma unroll
                for (int kk = 0; kk < C::EX; ++kk)
                    if (isext && k == kk) { cx[kk] = cc[e]; wx[kk] = ww[e]; }
                k += isext ? 1 : 0;
            }
        } else {
            for (int e = 0; e < maxdeg; ++e) {
                int c = 0;
                float w = 0.f;
                const int u = rs + (e < deg ? e : 0);
                if (ne <= 128) entry_cw(ix, u, c, w);
                else if (e < deg) { c = col[e0 + u]; w = ew[e0 + u]; }
                const bool isext = e < deg && classify(c, R) < 0;
#pragma unroll
                for (int kk = 0; kk < C::EX; ++kk)
                    if (isext && k == kk) { cx[kk] = c; wx[kk] = w; }
                k += isext ? 1 : 0;
            }
        }
        dc.slow = !fast || __ballot(k > C::EX) != 0ull;
        // empty slots read row 0 (one cache line per instruction for all of
        // them) with weight 0: every wave issues the same instruction count
#pragma unroll
        for (int kk = 0; kk < C::EX; ++kk) {
            const uint32_t src = cx[kk] >= 0 ? static_cast<uint32_t>(cx[kk]) : 0u;
            const float* p = x + static_cast<uint64_t>(src) * ldx32 + 4 * g;
#pragma unroll
            for (int i = 0; i < C::NCH; ++i) xv[kk][i] = *reinterpret_cast<const f32x4*>(p + 16 * i);
        }
    };
    auto ring_at = [&](int k, int64_t s) -> Ring {   // ring of the step whose tile is tw[k]
        Ring R;
        R.row0 = static_cast<int>(row_begin + (tw[k] >= 0 ? tw[k] : 0) * C::BM);
        R.lo = tw[k - 1] >= 0 && tw[k - 1] == tw[k] - 1;
        R.hi = tw[k + 1] >= 0 && tw[k + 1] == tw[k] + 1;
        R.s = static_cast<int>(s & (C::NSLOT - 1));
        return R;
    };

    Idx i0{}, i1{}, i2{};
    XV xv;
    float wx[C::EX];
    Dec dc;
    load_rp(tw[1], i0);
    load_rp(tw[2], i1);
    load_rp(tw[3], i2);
    load_cols(i0);
    load_cols(i1);
    decode(i0, ring_at(1, 0), dc, xv, wx);
#pragma unroll
    for (int k = 0; k < C::D; ++k) dma_tile(tw[1 + k], k);
    wait_barrier<(C::D - 2) * (C::PIECES / C::NW)>();   // tiles of steps 0, 1; EPI

    const bool has_res = (flags & MIGNN_EPI_RESIDUAL) != 0;
    for (int64_t s = 0; s < nsteps; ++s) {
        rstamp(trace, lane, wave, s, 0);
        // 1. indices: row_ptr of step s+3, cols of step s+2
        Idx i3{};
        load_rp(tw[4], i3);
        load_cols(i2);
        rstamp(trace, lane, wave, s, 1);
        // 2. the DMA of step s+D (its slot was freed by the barrier that ended
        // step s-1)
        dma_tile(tw[C::D + 1], s + C::D);
        rstamp(trace, lane, wave, s, 2);
        // 3. ring entries of this step (decoded at the end of step s-1)
        f32x4 acc[C::NCH];
#pragma unroll
        for (int i = 0; i < C::NCH; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!dc.slow) {
#pragma unroll
            for (int e = 0; e < C::MAXE; ++e) {
                if (e < dc.maxdeg) {
                    f32x4 v0[C::NCH];
                    const unsigned char* b0 = lds + dc.la[e];
#pragma unroll
                    for (int i = 0; i < C::NCH; ++i) v0[i] = *reinterpret_cast<const f32x4*>(b0 + 64 * i);
#pragma unroll
                    for (int i = 0; i < C::NCH; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(dc.lw[e], v0[i][j], acc[i][j]);
                }
            }
        } else {
            // generic: CSR order, ring rows from LDS, ext entries beyond the
            // register slots by synchronous loads
            const Ring R = ring_at(1, s);
            const int e0 = __builtin_amdgcn_readlane(i0.rlo, 0);
            const int ne = __builtin_amdgcn_readlane(i0.rhi, 15) - e0;
            const int rs = i0.rlo - e0, deg = i0.rhi - i0.rlo;
            int k = 0;
            for (int e = 0; e < dc.maxdeg; ++e) {
                int c = 0;
                float w = 0.f;
                const int u = rs + (e < deg ? e : 0);
                if (ne <= 128) entry_cw(i0, u, c, w);
                else if (e < deg) { c = col[e0 + u]; w = ew[e0 + u]; }
                const bool valid = e < deg;
                const int la = valid ? classify(c, R) : 0;
                if (valid && la < 0) {
                    if (k >= C::EX) {
                        const float* p = x + static_cast<uint64_t>(static_cast<uint32_t>(c)) * ldx32 + 4 * g;
#pragma unroll
                        for (int i = 0; i < C::NCH; ++i) {
                            const f32x4 v = *reinterpret_cast<const f32x4*>(p + 16 * i);
#pragma unroll
                            for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(w, v[j], acc[i][j]);
                        }
                    }
                    ++k;
                } else {
                    const unsigned char* base = lds + (la < 0 ? 0 : la);
                    const float wv = valid ? w : 0.f;
#pragma unroll
                    for (int i = 0; i < C::NCH; ++i) {
                        const f32x4 v = *reinterpret_cast<const f32x4*>(base + 64 * i);
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(wv, v[j], acc[i][j]);
                    }
                }
            }
        }
        rstamp(trace, lane, wave, s, 3);
        // 4. ext sums (gathered at the end of the previous step)
#pragma unroll
        for (int kk = 0; kk < C::EX; ++kk)
#pragma unroll
            for (int i = 0; i < C::NCH; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(wx[kk], xv[kk][i][j], acc[i][j]);
        rstamp(trace, lane, wave, s, 4);
        // 5. scale exponent of my row (max over its 4 lanes), split, seed
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < C::NCH; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) m = max(m, __float_as_uint(fabsf(acc[i][j])));
        m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), 16)));
        m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), 32)));
        const int p = scale_exp_r(m);
        const float sp = pow2f(p);
        f16x8 bh[C::KC], bl[C::KC];
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = acc[2 * kc + (j >> 2)][j & 3] * sp;
                const _Float16 hh = static_cast<_Float16>(v);
                bh[kc][j] = hh;
                bl[kc][j] = static_cast<_Float16>(v - static_cast<float>(hh));
            }
        const int pq = p + qw;
        const unsigned char* own = lds + (s & (C::NSLOT - 1)) * C::SLOT + (16 * wave + r) * C::PITCH + 16 * g;
        f32x4 o[C::NCB];
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb) {
            const f32x4 bo = *reinterpret_cast<const f32x4*>(&EPI[16 * cb + 4 * g]);
            const f32x4 rv = has_res ? *reinterpret_cast<const f32x4*>(own + 64 * cb)
                                     : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j) o[cb][j] = ldexpf(rv[j] + bo[j], pq);
        }
        rstamp(trace, lane, wave, s, 5);
        // 6. transform: D[n][row] += W[n][k] B[k][row], 3 fp16 MFMAs per block
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb) o[cb] = mfma_block<C::KC>(wh[cb], wl[cb], bh, bl, o[cb]);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");   // MFMA -> VALU read
        rstamp(trace, lane, wave, s, 6);
        // 7. epilogue: unscale, BN affine, ReLU; 16-B stores of my row's columns
        const int64_t grow = row_begin + tw[1] * C::BM + 16 * wave + r;
        float* const orow = out + (grow < row_end ? grow : row_end - 1) * ldo + 4 * g;
#pragma unroll
        for (int cb = 0; cb < C::NCB; ++cb) {
            const f32x4 so = *reinterpret_cast<const f32x4*>(&EPI[H + 16 * cb + 4 * g]);
            const f32x4 ho = *reinterpret_cast<const f32x4*>(&EPI[2 * H + 16 * cb + 4 * g]);
            f32x4 v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float y = ldexpf(o[cb][j], -pq);
                if (flags & MIGNN_EPI_AFFINE) y = y * so[j] + ho[j];
                if (flags & MIGNN_EPI_RELU) y = y < 0.0f ? 0.0f : y;
                v[j] = y;
            }
            if (grow < row_end) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(orow + 16 * cb));
        }
        rstamp(trace, lane, wave, s, 7);
        // 8. decode step s+1 (its ring: tiles tw[1..3]) and gather its ext rows
        decode(i1, ring_at(2, s + 1), dc, xv, wx);
        rstamp(trace, lane, wave, s, 8);
        // 9. rotate; the tile of step s+2 must have landed (DMA issued D steps
        // ago; younger: the DMAs of D-2 steps, this step's stores and ext
        // loads) and every wave be done with this step's ring
        i0 = i1;
        i1 = i2;
        i2 = i3;
#pragma unroll
        for (int k = 0; k + 1 < WIN; ++k) tw[k] = tw[k + 1];
        tw[WIN - 1] = gen_next();
        rstamp(trace, lane, wave, s, 9);
        wait_barrier<(C::D - 2) * (C::PIECES / C::NW) + C::NCB + C::EX * C::NCH>();
    }
}

template <int H>
int launch_ring(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                int64_t ldx, int64_t rb, int64_t re, const float* w, const float* bias,
                const float* scale, const float* shift, int flags, float* out, int64_t ldo,
                int64_t seg_tiles, hipStream_t st) {
    using C = RCfg<H>;
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
    int64_t T = seg_tiles > 0 ? seg_tiles : (ntiles + grid - 1) / grid;
    if (T < 1) T = 1;
    hipLaunchKernelGGL(gcn_ring_kernel<H>, dim3(grid), dim3(C::NT), 0, st, row_ptr, col, ew, x,
                       ldx, rb, re, w, bias, scale, shift, flags, out, ldo, T, g_ring_trace);
    return launch_status("gcn_ring_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_diag_set_trace_ring(void* buf) {
    g_ring_trace = static_cast<unsigned long long*>(buf);
    return MIGNN_OK;
}

extern "C" int mignn_gcn_layer_ring(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                    const float* w, const float* bias, const float* scale,
                                    const float* shift, int flags, float* out, int64_t ldo,
                                    int64_t seg_tiles, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && ew && x && w && out, "gcn_layer_ring: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_layer_ring: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(w) && aligned16(out), "gcn_layer_ring: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h,
                  "gcn_layer_ring: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_ring: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_ring: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_ring: affine");
    MIGNN_REQUIRE(x != out, "gcn_layer_ring: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    return h == 128 ? launch_ring<128>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift,
                                       flags, out, ldo, seg_tiles, st)
                    : launch_ring<64>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift,
                                      flags, out, ldo, seg_tiles, st);
}
