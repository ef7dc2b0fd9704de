// Fused GCN layer, split-fp16 MFMA, wave-independent form (the north-star hot
// kernel: GCNConv + residual + BatchNorm(eval) + ReLU, gnn_model.py:166,
// :184-191, one pass over HBM):
//
//   out_i = relu( (x_i + bias + (sum_{e in row i} ew_e x_{col e}) W^T) * scale + shift )
//
// Structure.  Every wave owns whole 16-row tiles and runs a tile start to end
// by itself -- no producer / consumer roles, no per-step block barrier:
//   1. gather: the row's CSR entries two at a time; lane (r, g) of the wave
//      loads 16 B at bytes 64 h + 16 g (h < H/16) of row r's neighbour (so a
//      wave instruction moves 16 rows x 64 contiguous bytes) and accumulates
//      in fp32, CSR order;
//   2. split: the 4 lanes of a row agree on a power-of-two scale 2^p (row max
//      in [2^13, 2^14)), each value a*2^p = hi + lo in fp16 -- in registers,
//      already in the MFMA B-operand layout (no LDS image);
//   3. transform: D[n][row] = W'.agg^T by v_mfma_f32_16x16x32_f16, three per
//      16x16x32 block (hi.hi + hi.lo + lo.hi), W' = diag(BN scale) W split
//      once per launch into fragments held in LDS (one exponent per 16
//      output columns);
//   4. epilogue in the accumulator layout (lane (r, g): row r, columns
//      16 nb + 4 g + i -- the same bytes as its gather chunks):
//      out = relu(acc 2^-(p+q) + x * sc + (bias * sc + shift)), 16-B
//      non-temporal stores.
// The next tile's CSR indices are loaded while this tile transforms; the
// waves of a CU (2 workgroups x 8) hide each other's gather latency.
//
// Arithmetic (as gcn_f16x3.hip): a.w = 2^-(p+q) (ah wh + ah wl + al wh) +
// O(2^-22 |a||w|) per product, fp32 accumulation.  Scales are clamped to
// [2^-60, 2^60]: |values| < 2^70 (fp16 hi overflow beyond), and rows below
// 2^-47 keep an absolute error far below any fp32 rounding of the output.
// Sum order per row: CSR order (deterministic, no atomics).
#include "common.hpp"

namespace mignn {
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

template <int H>
struct WCfg {
    static_assert(H == 64 || H == 128, "gcn_wave: H in {64, 128}");
    static constexpr int NB = H / 16;                 // 16-column output blocks
    static constexpr int KC = H / 32;                 // 32-deep k chunks
    static constexpr int NH = H / 16;                 // 16-B chunks per lane of a row
    static constexpr int FRAG = 1024;                 // one MFMA operand fragment (64 x 16 B)
    static constexpr int W_BYTES = KC * NB * 2 * FRAG;
    static constexpr int OFF_TA = W_BYTES;            // residual multiplier per column
    static constexpr int OFF_TB = OFF_TA + H * 4;     // additive term per column
    static constexpr int OFF_Q = OFF_TB + H * 4;      // exponent (first: max bits) per block
    static constexpr int LDS_BYTES = OFF_Q + NB * 4;
    static constexpr int NT = 512;                    // 8 waves per workgroup
    static constexpr int SLOTS = 8;                   // CSR entries per row held in registers
};

__device__ __attribute__((aligned(16))) float g_zero_row_w[256];

__device__ __forceinline__ float pow2f(int p) {
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}

// scale exponent of a block whose max |value| has f32 bits m: max * 2^p in
// [2^13, 2^14), clamped to [-60, 60] (zero / tiny blocks: 60)
__device__ __forceinline__ int wexp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return max(-60, min(140 - eb, 60));
}

// max over the wave (non-negative ints), wave-uniform result
__device__ __forceinline__ int wave_max_i(int v) {
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false));    // quad_perm 1,0,3,2
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false));    // quad_perm 2,3,0,1
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, false));   // row_ror 4
    v = max(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false));   // row_ror 8
    const int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}

// one tile's CSR view for this lane's row: first entry, degree, and the
// first SLOTS columns / weights (column -1: empty)
template <int S>
struct TileIdx {
    int rp0, deg;
    int c[S];
    float w[S];
};

template <int H, int S>
__device__ __forceinline__ void load_rp(TileIdx<S>& t, const int32_t* __restrict__ row_ptr,
                                        int64_t row, int64_t re) {
    if (row < re) {
        t.rp0 = row_ptr[row];
        t.deg = row_ptr[row + 1] - t.rp0;
    } else {
        t.rp0 = 0;
        t.deg = 0;
    }
}

template <int S>
__device__ __forceinline__ void load_slots(TileIdx<S>& t, const int32_t* __restrict__ col,
                                           const float* __restrict__ ew) {
#pragma unroll
    for (int e = 0; e < S; ++e) {
        int c = -1;
        float w = 0.f;
        if (e < t.deg) {
            c = col[t.rp0 + e];
            w = ew[t.rp0 + e];
        }
        t.c[e] = c;
        t.w[e] = w;
    }
}

template <int H>
__device__ __forceinline__ const float* row_src(const float* __restrict__ x, int64_t ldx, int c,
                                                int g) {
    return c >= 0 ? x + static_cast<int64_t>(c) * ldx + 4 * g : g_zero_row_w + 4 * g;
}

// an MFMA operand fragment (8 halfs = 4 dwords) moved across lanes:
// lane l gets the fragment of lane addr / 4
__device__ __forceinline__ f16x8 permute_frag(f16x8 v, int addr) {
    using i32x4v = __attribute__((ext_vector_type(4))) int;
    i32x4v d = __builtin_bit_cast(i32x4v, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_ds_bpermute(addr, d[q]);
    return __builtin_bit_cast(f16x8, d);
}

template <int NH>
__device__ __forceinline__ void load_row(const float* p, f32x4 (&v)[NH]) {
#pragma unroll
    for (int h = 0; h < NH; ++h) v[h] = *reinterpret_cast<const f32x4*>(p + 16 * h);
}

// WPS: waves per SIMD (workgroups of 8 waves: WPS / 2 per CU); GRP: CSR
// entries gathered per round trip; LATE_RES: residual rows loaded after the
// transform instead of before it; COAL: gathers, residual loads and stores in
// the coalesced lane layout (lane l: row l >> 2, 16-B chunk 4 h + (l & 3):
// every 4 consecutive lanes move 64 contiguous bytes) with the split B
// fragments and the accumulators moved between it and the MFMA layout (lane
// n + 16 g) by ds_bpermute -- else every load / store in the MFMA layout
template <int H, int WPS, int GRP, bool LATE_RES, bool COAL = false>
__global__ __launch_bounds__(WCfg<H>::NT, WPS) void gcn_wave_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t ldx, int64_t rb,
    int64_t re, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ scale, const float* __restrict__ shift, int flags,
    float* __restrict__ out, int64_t ldo) {
    using C = WCfg<H>;
    constexpr int S = C::SLOTS;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    float* const TA = reinterpret_cast<float*>(lds + C::OFF_TA);
    float* const TB = reinterpret_cast<float*>(lds + C::OFF_TB);
    uint32_t* const QM = reinterpret_cast<uint32_t*>(lds + C::OFF_Q);

    const int tid = threadIdx.x;
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // this lane's row of a tile and 16-B chunk column (see COAL)
    const int r = COAL ? (lane >> 2) : (lane & 15);
    const int g = COAL ? (lane & 3) : (lane >> 4);
    // ds_bpermute byte addresses: MFMA lane n + 16 g <- coalesced lane 4 n + g,
    // and back
    const int to_mfma = 4 * (4 * (lane & 15) + (lane >> 4));
    const int to_coal = 4 * ((lane >> 2) + 16 * (lane & 3));
    const bool aff = (flags & MIGNN_EPI_AFFINE) != 0;

    // ---- prologue: per-column epilogue terms; W' = diag(sc) W as split
    // fragments, lane (m, g) of fragment (kc, nb) holding W'[16 nb + m][k] at
    // k = 32 kc + 4 g + (j & 3) + 16 (j >> 2) -- the k order of the gathered
    // chunks (h = 2 kc + (j >> 2))
    if (tid < H) {
        const float s = aff ? scale[tid] : 1.f;
        const float b = (flags & MIGNN_EPI_BIAS) ? bias[tid] : 0.f;
        TA[tid] = (flags & MIGNN_EPI_RESIDUAL) ? s : 0.f;
        TB[tid] = aff ? fmaf(b, s, shift[tid]) : b;
    }
    if (tid < C::NB) QM[tid] = 0u;
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
        const float sq = pow2f(wexp(QM[nb]));
        f16x8 hv, lv;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float s = v[j] * sq;
            const _Float16 hh = static_cast<_Float16>(s);
            hv[j] = hh;
            lv[j] = static_cast<_Float16>(s - static_cast<float>(hh));
        }
        const int fb = task >> 6, ln = task & 63;
        *reinterpret_cast<f16x8*>(lds + (2 * fb) * C::FRAG + ln * 16) = hv;
        *reinterpret_cast<f16x8*>(lds + (2 * fb + 1) * C::FRAG + ln * 16) = lv;
    }
    __syncthreads();
    if (tid < C::NB) QM[tid] = static_cast<uint32_t>(wexp(QM[tid]));
    __syncthreads();

    // ---- tile schedule: XCD x (blocks b, b + 8, ... share one) walks a
    // contiguous eighth of the tiles; its waves take consecutive tiles
    const int64_t nrows = re - rb;
    const int64_t ntiles = (nrows + 15) / 16;
    const int G = gridDim.x;                 // multiple of 8 (host)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int64_t wpx = static_cast<int64_t>(G >> 3) * (C::NT / 64);   // waves per XCD
    const int64_t chunk = (ntiles + 7) / 8;
    const int64_t tend = min(ntiles, (xcd + 1) * chunk);
    int64_t t = xcd * chunk + static_cast<int64_t>(slot) * (C::NT / 64) + wave;
    if (t >= tend) return;

    const uint64_t ldxb = static_cast<uint64_t>(ldx);
    TileIdx<S> cur, nxt;
    load_rp<H, S>(cur, row_ptr, rb + 16 * t + r, re);
    load_slots<S>(cur, col, ew);
    load_rp<H, S>(nxt, row_ptr, rb + 16 * (t + wpx) + r, re);

    for (; t < tend; t += wpx) {
        const int64_t row = rb + 16 * t + r;
        const int64_t rowc = row < re ? row : re - 1;
        // ---- 1. gather, two CSR entries per round trip
        f32x4 agg[C::NH];
#pragma unroll
        for (int h = 0; h < C::NH; ++h) agg[h] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int maxd = wave_max_i(cur.deg);
#pragma unroll
        for (int e0 = 0; e0 < S; e0 += GRP) {
            if (e0 >= maxd) break;
            f32x4 v[GRP][C::NH];
#pragma unroll
            for (int u = 0; u < GRP; ++u) load_row<C::NH>(row_src<H>(x, ldx, cur.c[e0 + u], g), v[u]);
#pragma unroll
            for (int u = 0; u < GRP; ++u) {
                const float w = cur.w[e0 + u];
#pragma unroll
                for (int h = 0; h < C::NH; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i) agg[h][i] = fmaf(w, v[u][h][i], agg[h][i]);
            }
        }
        // rows with more than S entries (rare on meshes): one at a time
        for (int e = S; e < maxd; ++e) {
            int c = -1;
            float w = 0.f;
            if (e < cur.deg) {
                c = col[cur.rp0 + e];
                w = ew[cur.rp0 + e];
            }
            f32x4 va[C::NH];
            load_row<C::NH>(row_src<H>(x, ldx, c, g), va);
#pragma unroll
            for (int h = 0; h < C::NH; ++h)
#pragma unroll
                for (int i = 0; i < 4; ++i) agg[h][i] = fmaf(w, va[h][i], agg[h][i]);
        }
        // ---- residual rows (this tile's own rows, in the epilogue layout):
        // before the transform (LATE_RES = false) or after it (fewer live
        // registers; the rows were just read as the self-loop entries)
        f32x4 xres[C::NH];
        auto load_res = [&]() {
            if (flags & MIGNN_EPI_RESIDUAL) {
                load_row<C::NH>(x + rowc * static_cast<int64_t>(ldxb) + 4 * g, xres);
            } else {
#pragma unroll
                for (int h = 0; h < C::NH; ++h) xres[h] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        };
        if constexpr (!LATE_RES) load_res();
        // ---- next tile's CSR view (its row_ptr arrived a tile ago)
        const int64_t tn = t + wpx;
        if (tn < tend) {
            cur = nxt;
            load_slots<S>(cur, col, ew);
            load_rp<H, S>(nxt, row_ptr, rb + 16 * (tn + wpx) + r, re);
        }
        // ---- 2. split with the row's scale (max over the row's 4 lanes)
        uint32_t mb = 0;
#pragma unroll
        for (int h = 0; h < C::NH; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) mb = max(mb, __float_as_uint(fabsf(agg[h][i])));
        if constexpr (COAL) {   // the row's 4 lanes are a DPP quad
            int t = static_cast<int>(mb);
            t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0xB1, 0xf, 0xf, false)));
            t = max(static_cast<uint32_t>(t), static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(t, 0x4E, 0xf, 0xf, false)));
            mb = static_cast<uint32_t>(t);
        } else {
            const auto r16 = __builtin_amdgcn_permlane16_swap(mb, mb, false, false);
            mb = max(static_cast<uint32_t>(r16[0]), static_cast<uint32_t>(r16[1]));
            const auto r32 = __builtin_amdgcn_permlane32_swap(mb, mb, false, false);
            mb = max(static_cast<uint32_t>(r32[0]), static_cast<uint32_t>(r32[1]));
        }
        const int p = wexp(mb);
        const float sp = pow2f(p);
        // ---- 3. transform: acc[nb] = W'[16 nb .., :] . agg^T (3 MFMAs per block)
        f32x4 acc[C::NB];
#pragma unroll
        for (int nb = 0; nb < C::NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
        // (laundered per tile: the fragments are loop-invariant, and hoisting
        // all of them out of the tile loop would need 256 registers)
        int wofs = lane * 16;
        asm volatile("" : "+v"(wofs));
        const unsigned char* const wl = lds + wofs;
#pragma unroll
        for (int kc = 0; kc < C::KC; ++kc) {
            f16x8 bh, bl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float s = agg[2 * kc + (j >> 2)][j & 3] * sp;
                const _Float16 hh = static_cast<_Float16>(s);
                bh[j] = hh;
                bl[j] = static_cast<_Float16>(s - static_cast<float>(hh));
            }
            if constexpr (COAL) {
                bh = permute_frag(bh, to_mfma);
                bl = permute_frag(bl, to_mfma);
            }
#pragma unroll
            for (int nb = 0; nb < C::NB; ++nb) {
                const int fb = kc * C::NB + nb;
                const f16x8 wh = *reinterpret_cast<const f16x8*>(wl + (2 * fb) * C::FRAG);
                const f16x8 wlo = *reinterpret_cast<const f16x8*>(wl + (2 * fb + 1) * C::FRAG);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bh, acc[nb], 0, 0, 0);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, bl, acc[nb], 0, 0, 0);
                acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wlo, bh, acc[nb], 0, 0, 0);
            }
        }
        if constexpr (COAL) {
#pragma unroll
            for (int nb = 0; nb < C::NB; ++nb)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[nb][i] = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(
                        to_coal, __float_as_int(acc[nb][i])));
        }
        if constexpr (LATE_RES) load_res();
        // ---- 4. epilogue: lane (r, g) = row r, columns 16 nb + 4 g + i
        const bool relu = (flags & MIGNN_EPI_RELU) != 0;
        int eofs = 16 * g;
        asm volatile("" : "+v"(eofs));
#pragma unroll
        for (int nb = 0; nb < C::NB; ++nb) {
            const float u = pow2f(-(p + static_cast<int>(QM[nb])));
            const f32x4 ta = *reinterpret_cast<const f32x4*>(lds + C::OFF_TA + 64 * nb + eofs);
            const f32x4 tb = *reinterpret_cast<const f32x4*>(lds + C::OFF_TB + 64 * nb + eofs);
            f32x4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = fmaf(acc[nb][i], u, fmaf(xres[nb][i], ta[i], tb[i]));
                if (relu) v = v < 0.0f ? 0.0f : v;
                o[i] = v;
            }
            if (row < re)
                __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(out + row * ldo + 16 * nb + 4 * g));
        }
    }
}

template <int H, int WPS, int GRP, bool LATE_RES, bool COAL = false>
int launch_wave(const int32_t* row_ptr, const int32_t* col, const float* ew, const float* x,
                int64_t ldx, int64_t rb, int64_t re, const float* w, const float* bias,
                const float* scale, const float* shift, int flags, float* out, int64_t ldo,
                hipStream_t st) {
    using C = WCfg<H>;
    static int grid_cache[64] = {0};
    static_assert(WPS == 2 || WPS == 4, "WPS");
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& G = grid_cache[dev & 63];
    if (G == 0) {
        int cus = 0;
        MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        G = (cus / 8) * 8 * (WPS / 2);      // WPS / 2 8-wave workgroups per CU
        if (G < 8) G = 8;
    }
    const int64_t ntiles = (re - rb + 15) / 16;
    const int64_t wavesneed = (ntiles + 7) / 8 * 8;
    int grid = G;
    const int64_t need_blocks = (wavesneed + C::NT / 64 - 1) / (C::NT / 64);
    if (need_blocks < grid) grid = static_cast<int>(((need_blocks + 7) / 8) * 8);
    hipLaunchKernelGGL((gcn_wave_kernel<H, WPS, GRP, LATE_RES, COAL>), dim3(grid), dim3(C::NT), 0, st, row_ptr, col, ew, x,
                       ldx, rb, re, w, bias, scale, shift, flags, out, ldo);
    return launch_status("gcn_wave_kernel");
}

}  // namespace
}  // namespace mignn

using namespace mignn;

// EXPERIMENTAL (round 3): the wave-independent split-fp16 GCN layer; same
// contract as mignn_gcn_layer_f16x3 (sum order: CSR order)
extern "C" int mignn_gcn_layer_wave(const int32_t* row_ptr, const int32_t* col, const float* ew,
                                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h,
                                    const float* w, const float* bias, const float* scale,
                                    const float* shift, int flags, float* out, int64_t ldo,
                                    int variant, void* stream) {
    MIGNN_REQUIRE((flags & ~MIGNN_EPI_MASK) == 0, "gcn_layer_wave: unknown flags 0x%x", flags);
    MIGNN_REQUIRE(row_ptr && col && ew && x && w && out, "gcn_layer_wave: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128, "gcn_layer_wave: h must be 64 or 128 (got %d)", h);
    MIGNN_REQUIRE(aligned16(x) && aligned16(w) && aligned16(out), "gcn_layer_wave: unaligned");
    MIGNN_REQUIRE(ldx % 4 == 0 && ldo % 4 == 0 && ldx >= h && ldo >= h, "gcn_layer_wave: bad strides");
    MIGNN_REQUIRE(rb >= 0 && re >= rb, "gcn_layer_wave: bad row range");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_BIAS) || bias, "gcn_layer_wave: bias");
    MIGNN_REQUIRE(!(flags & MIGNN_EPI_AFFINE) || (scale && shift), "gcn_layer_wave: affine");
    MIGNN_REQUIRE(x != out, "gcn_layer_wave: in-place not supported (neighbours read x)");
    if (re == rb) return MIGNN_OK;
    if (variant >= 10 && variant < 20)    // the fused tile kernel (gcn_fused.hip)
        return gcn_fused_layer(row_ptr, col, ew, x, ldx, rb, re, h, w, bias, scale, shift, flags,
                               out, ldo, stream, variant - 10);
    hipStream_t st = as_stream(stream);
#define MIGNN_WAVE(HH, WPS, GRP, LR, ...) \
    return launch_wave<HH, WPS, GRP, LR, ##__VA_ARGS__>(row_ptr, col, ew, x, ldx, rb, re, w, bias, scale, shift, \
                                         flags, out, ldo, st)
    if (h == 128) {
        switch (variant) {
            case 1: MIGNN_WAVE(128, 2, 4, false);
            case 2: MIGNN_WAVE(128, 4, 2, false);
            case 3: MIGNN_WAVE(128, 2, 2, false);
            case 4: MIGNN_WAVE(128, 2, 2, false, true);
            case 5: MIGNN_WAVE(128, 4, 2, true, true);
            case 6: MIGNN_WAVE(128, 2, 4, false, true);
            default: MIGNN_WAVE(128, 4, 2, true);
        }
    }
    switch (variant) {
        case 1: MIGNN_WAVE(64, 2, 4, false);
        case 2: MIGNN_WAVE(64, 4, 2, false);
        case 3: MIGNN_WAVE(64, 2, 2, false);
        case 4: MIGNN_WAVE(64, 2, 2, false, true);
        case 5: MIGNN_WAVE(64, 4, 2, true, true);
        case 6: MIGNN_WAVE(64, 4, 4, false, true);
        default: MIGNN_WAVE(64, 4, 4, false);
    }
#undef MIGNN_WAVE
}
