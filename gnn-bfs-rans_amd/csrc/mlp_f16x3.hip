// Fused output head of FlowGNN (output_proj, gnn_model.py:90-100, :195):
//   out = L4( relu( L3( relu( L2( relu( L1(x) ) ) ) ) ) ),  H -> H -> H -> H/2 -> out
// in ONE pass over x, split-fp16 ("f16x3") MFMA arithmetic (see gcn_f16x3.hip:
// every operand = 2^-p (hi + lo) with fp16 hi / lo, three MFMAs per product
// block, fp32 accumulation; relative error per product ~2^-22).
//
// Why fused: the 4-launch fp32 path writes and re-reads three [N, H]
// activations (3 x 2 x 5.12 GB at N = 10M, H = 128) and runs on the f32
// MFMA rate; here x is read once, 28 B per row are written, and the
// transforms run at 16x the f32 MFMA rate.
//
// Layout: one wave owns 32 rows at a time (persistent over 32-row blocks,
// 8 waves per workgroup, each on its own blocks).  Every layer is
// v_mfma_f32_32x32x16_f16 in the orientation D[n][row] = W . act^T, so a
// lane (row = l & 31, half h = l >> 5) holds 16 output features of its row
// per 32-feature block -- registers 8 s .. 8 s + 7 of a block are, after the
// split, directly the next layer's B-operand fragment of k-step s (the
// accumulator-as-operand chaining of cdna_hip_programming.md §3); the
// weights are stored pre-permuted to match, so activations never leave the
// registers.  Per-row scale exponents: max over the row's features = the
// lane and its partner lane l ^ 32 (v_permlane32_swap).
//
// Weights: a prep kernel (mignn_mlp_head_prep, once per weight version)
// splits each matrix with one power-of-two exponent per matrix into fp16
// hi / lo fragment images and lays the biases out in accumulator-register
// order; the head kernel copies W1..W3's images into LDS (exactly 160 KiB
// at H = 128: 2 x 64 KiB + 32 KiB) and reads W4 / the biases through L1/L2.
#include "common.hpp"

// W-fragment prefetch depth of the head's MFMA loops, in (block, k-step)
// steps of 3 MFMAs
#ifndef MIGNN_HEAD_WPD
#define MIGNN_HEAD_WPD 1
#endif

namespace mignn {
namespace {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int H>
struct MCfg {
    static_assert(H == 64 || H == 128, "fused head: H in {64, 128}");
    static constexpr int NW = 8;                   // waves per workgroup
    static constexpr int NT = NW * 64;
    static constexpr int NB1 = H / 32, KT1 = H / 16;   // L1: H -> H
    static constexpr int NB2 = H / 32, KT2 = H / 16;   // L2: H -> H
    static constexpr int NB3 = H / 64, KT3 = H / 16;   // L3: H -> H/2
    static constexpr int KT4 = H / 32;                  // L4: H/2 -> out (<= 8 used of 32)
    static constexpr int FRAG = 2 * 64 * 8 * 2;         // bytes: hi + lo fragment, one (nb, t)
    static constexpr int W1_BYTES = NB1 * KT1 * FRAG;
    static constexpr int W2_BYTES = NB2 * KT2 * FRAG;
    static constexpr int W3_BYTES = NB3 * KT3 * FRAG;
    static constexpr int W4_BYTES = KT4 * FRAG;
    static constexpr int LDS_BYTES = W1_BYTES + W2_BYTES + W3_BYTES;   // W4 via L1/L2
    // biases: [layer][nb][h][16 floats in accumulator-register order]
    static constexpr int BOFF1 = 0, BOFF2 = BOFF1 + NB1 * 128, BOFF3 = BOFF2 + NB2 * 128,
                         BOFF4 = BOFF3 + NB3 * 128, BIAS_BYTES = BOFF4 + 128;
    static constexpr int BIAS_AT = LDS_BYTES + W4_BYTES;
    static constexpr int EXP_AT = BIAS_AT + BIAS_BYTES;                // 4 ints
    static constexpr int IMG_BYTES = EXP_AT + 16;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// max * 2^p in [2^13, 2^14): p = 140 - biased exponent of the max, capped
__device__ __forceinline__ int head_scale_exp(uint32_t mbits) {
    const int eb = static_cast<int>((mbits >> 23) & 0xffu);
    return min(140 - eb, 50);
}

__device__ __forceinline__ float exp2_int(int p) {   // 2^p, p in [-126, 127]
    return __uint_as_float(static_cast<uint32_t>(p + 127) << 23);
}

__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// feature index of k-step t, lane half h, element j when the operand comes
// from a previous layer's 32x32 accumulator (chained) or from x (natural)
__device__ __forceinline__ int chained_k(int t, int h, int j) {
    return 32 * (t >> 1) + 16 * (t & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}
__device__ __forceinline__ int natural_k(int t, int h, int j) { return 16 * t + 8 * h + j; }

// max over the lane and its partner l ^ 32 (the two halves of one row)
__device__ __forceinline__ uint32_t pair_max(uint32_t m) {
    const auto sw = __builtin_amdgcn_permlane32_swap(m, m, false, false);
    return max(static_cast<uint32_t>(sw[0]), static_cast<uint32_t>(sw[1]));
}

// 8 floats times the power of two f -> hi / lo fp16 fragments (split_pair:
// mixed-precision FMAs, no packed fp32)
__device__ __forceinline__ void split8(const float* a, float f, f16x8& hi, f16x8& lo) {
    using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
    u32x4 h, l;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t hq, lq;
        split_pair(a[2 * q], a[2 * q + 1], f, hq, lq);
        h[q] = hq;
        l[q] = lq;
    }
    hi = __builtin_bit_cast(f16x8, h);
    lo = __builtin_bit_cast(f16x8, l);
}

// raw bias of one accumulator block, in register order (16 floats at bl)
__device__ __forceinline__ f32x16 ldbias(const float* bl) {
    f32x16 a;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = ld4(bl + 4 * q);
        a[4 * q + 0] = v.x;
        a[4 * q + 1] = v.y;
        a[4 * q + 2] = v.z;
        a[4 * q + 3] = v.w;
    }
    return a;
}

// relu of NBN accumulator blocks (scaled by 2^pq) -> the next layer's split
// operand fragments (k-step 2 nb + s = registers 8 s .. 8 s + 7 of block
// nb); returns the new per-row exponent p' (values of the unscaled
// activation times 2^p').  The max is taken on the scaled accumulator, so
// p' = 140 - (e_acc - pq) and one multiply by 2^(p' - pq) rescales.
template <int NBN, int NBNEXT>
__device__ __forceinline__ int chain(f32x16* a, int pq, f16x8* oh, f16x8* ol,
                                     const float* bnext) {
    uint32_t mm = 0;
#pragma unroll
    for (int nb = 0; nb < NBN; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            // relu on the bit pattern: negative floats are negative int32
            const int bits = max(__float_as_int(a[nb][r]), 0);
            a[nb][r] = __int_as_float(bits);
            mm = max(mm, static_cast<uint32_t>(bits));
        }
    mm = pair_max(mm);
    const int eb = static_cast<int>((mm >> 23) & 0xffu);
    const int pn = min(140 - eb + pq, 50);
    const float f = exp2_int(max(min(pn - pq, 127), -126));
#pragma unroll
    for (int nb = 0; nb < NBN; ++nb)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = a[nb][8 * s + j];
            split8(v, f, oh[2 * nb + s], ol[2 * nb + s]);
            // a[nb] consumed: start the next layer's raw bias load into it
            if (s == 1 && nb < NBNEXT) a[nb] = ldbias(bnext + nb * 32);
        }
    return pn;
}

// a layer's LDS base + lane offset, opaque: its fragment reads then carry
// their distance from it in the 16-bit ds_read offset field (past 64 KiB the
// compiler otherwise adds the constant to the lane offset once per read)
__device__ __forceinline__ uint32_t lds_base(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

// One layer: acc[nb] = acc[nb] sc + W[nb] . act (acc[nb] holds the raw
// bias on entry) for NB 32-feature output blocks, KT
// 16-deep k-steps, three MFMAs per (nb, t); W fragments from LDS (fragment
// (nb, t) at wl + (nb KT + t) FRAG, lane slice at byte offset loff), loaded
// one step ahead.
template <int NB, int KT, bool PRIO = false>
__device__ __forceinline__ void layer_mfma(f32x16* acc, float sc, const unsigned char* wl,
                                           uint32_t loff, const f16x8* ah, const f16x8* al) {
    constexpr int FRAG = 2 * 64 * 16;
    // PRIO: this wave's MFMA segment wins instruction arbitration over the
    // SIMD partner's VALU segment (s_setprio), so the matrix pipe is fed
    // first and the partner's split / ReLU work fills the gaps
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
    auto ld = [&](int i, f16x8& hi, f16x8& lo) {
        hi = *reinterpret_cast<const f16x8*>(wl + i * FRAG + loff);
        lo = *reinterpret_cast<const f16x8*>(wl + i * FRAG + 64 * 16 + loff);
    };
    constexpr int WPD = MIGNN_HEAD_WPD, WNF = WPD + 1;
    f16x8 wh[WNF], wo[WNF];
#pragma unroll
    for (int i = 0; i < WPD; ++i) ld(i, wh[i], wo[i]);
#pragma unroll
    for (int i = 0; i < NB * KT; ++i) {
        const int nb = i / KT, t = i % KT;
        if (t == 0) acc[nb] *= sc;   // raw bias (loaded early) -> seed: waits here only
        if (i + WPD < NB * KT) ld(i + WPD, wh[(i + WPD) % WNF], wo[(i + WPD) % WNF]);
        acc[nb] = mfma32(wh[i % WNF], ah[t], acc[nb]);
        acc[nb] = mfma32(wh[i % WNF], al[t], acc[nb]);
        acc[nb] = mfma32(wo[i % WNF], ah[t], acc[nb]);
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
}

// ---- prep: one workgroup per layer -- exponent, split, permuted fragments,
// bias in register order.  Image of matrix m: [nb][t] x {hi: 64 lanes x 8
// halfs, lo: same}; element j of lane (n = l & 31, h = l >> 5) =
// W[32 nb + n][k(t, h, j)] * 2^q (0 for rows >= n_out).
template <int H>
__global__ __launch_bounds__(256) void mlp_prep_kernel(
    const float* __restrict__ w1, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ w3, const float* __restrict__ b3,
    const float* __restrict__ w4, const float* __restrict__ b4, int out_dim,
    unsigned char* __restrict__ img) {
    using C = MCfg<H>;
    const int m = blockIdx.x;
    const float* W = m == 0 ? w1 : m == 1 ? w2 : m == 2 ? w3 : w4;
    const float* B = m == 0 ? b1 : m == 1 ? b2 : m == 2 ? b3 : b4;
    const int n_out = m < 2 ? H : m == 2 ? H / 2 : out_dim;
    const int k_in = m < 3 ? H : H / 2;
    const int nb_n = m < 2 ? H / 32 : m == 2 ? H / 64 : 1;
    const int kt_n = k_in / 16;
    const int off = m == 0 ? 0 : m == 1 ? C::W1_BYTES : m == 2 ? C::W1_BYTES + C::W2_BYTES
                                                              : C::LDS_BYTES;
    const int boff = m == 0 ? C::BOFF1 : m == 1 ? C::BOFF2 : m == 2 ? C::BOFF3 : C::BOFF4;
    __shared__ uint32_t smax;
    if (threadIdx.x == 0) smax = 0;
    __syncthreads();
    uint32_t mx = 0;
    for (int i = threadIdx.x; i < n_out * k_in; i += blockDim.x)
        mx = max(mx, __float_as_uint(fabsf(W[i])));
    atomicMax(&smax, mx);
    __syncthreads();
    const int q = head_scale_exp(smax);
    if (threadIdx.x == 0) reinterpret_cast<int*>(img + C::EXP_AT)[m] = q;
    _Float16* const base = reinterpret_cast<_Float16*>(img + off);
    const int total = nb_n * kt_n * 64 * 8;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int j = i & 7, lane = (i >> 3) & 63, t = (i >> 9) % kt_n, nb = (i >> 9) / kt_n;
        const int n = 32 * nb + (lane & 31), h = lane >> 5;
        const int k = m == 0 ? natural_k(t, h, j) : chained_k(t, h, j);
        const float w = n < n_out ? W[n * k_in + k] : 0.f;
        const float s = ldexpf(w, q);
        const _Float16 hi = static_cast<_Float16>(s);
        const _Float16 lo = static_cast<_Float16>(s - static_cast<float>(hi));
        _Float16* const f = base + (nb * kt_n + t) * (2 * 64 * 8);
        f[lane * 8 + j] = hi;
        f[64 * 8 + lane * 8 + j] = lo;
    }
    float* const bias = reinterpret_cast<float*>(img + C::BIAS_AT + boff);
    for (int i = threadIdx.x; i < nb_n * 32; i += blockDim.x) {
        const int r = i & 15, h = (i >> 4) & 1, nb = i >> 5;
        const int n = 32 * nb + (r & 3) + 8 * (r >> 2) + 4 * h;
        bias[i] = n < n_out ? B[n] : 0.f;
    }
}

// ---- head kernel (DIAG: timing ablations, results wrong by design:
// 1 = no x loads, 2 = no MFMAs; 4 = MFMA segments at raised priority, results
// exact).  NWV waves per workgroup: 8 (two per SIMD, the next block's x rows
// prefetched into registers during layer 3) or 12 (three per SIMD at <= 168
// VGPRs: no register prefetch, the third wave covers the loads)
template <int H, int DIAG = 0, int NWV = 8>
__global__ __launch_bounds__(NWV * 64) void mlp_head_kernel(
    const float* __restrict__ x, int64_t ldx, int64_t nrows, const unsigned char* __restrict__ img,
    int out_dim, float* __restrict__ out, int64_t ldo, const int32_t* __restrict__ out_rows) {
    using C = MCfg<H>;
    __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS_BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int h = lane >> 5, r32 = lane & 31;

    // W1..W3 images -> LDS (16 B per thread per step)
    for (int i = threadIdx.x; i < C::LDS_BYTES / 16; i += NWV * 64)
        reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(img)[i];
    const int* qv = reinterpret_cast<const int*>(img + C::EXP_AT);
    const int q1 = qv[0], q2 = qv[1], q3 = qv[2], q4 = qv[3];
    __syncthreads();

    const int64_t nblk = (nrows + 31) / 32;
    constexpr bool PF = NWV == 8;        // register prefetch of the next block's x
    const int64_t stride = static_cast<int64_t>(gridDim.x) * NWV;
    // x row fragments of a block: k-step t -> x[row][16 t + 8 h .. +7];
    // rows past the end (and blocks past the last) read a valid row
    float xv[C::KT1][8];
    auto load_x = [&](int64_t b) {
        int64_t r = b * 32 + r32;
        r = r < nrows ? r : nrows - 1;
        const float* xr = x + r * ldx + 8 * h;
#pragma unroll
        for (int t = 0; t < C::KT1; ++t) {
            if constexpr ((DIAG & 1) != 0) {
#pragma unroll
                for (int j = 0; j < 8; ++j) xv[t][j] = static_cast<float>(lane - 8 * t + j);
                continue;
            }
            const float4 u = ld4(xr + 16 * t), v = ld4(xr + 16 * t + 4);
            xv[t][0] = u.x; xv[t][1] = u.y; xv[t][2] = u.z; xv[t][3] = u.w;
            xv[t][4] = v.x; xv[t][5] = v.y; xv[t][6] = v.z; xv[t][7] = v.w;
        }
    };
    int64_t blk = static_cast<int64_t>(blockIdx.x) * NWV + wave;
    if constexpr (PF) load_x(blk);
    for (; blk < nblk; blk += stride) {
        if constexpr (!PF) load_x(blk);
        // opaque per-block offsets: keep the loop-invariant LDS fragment, W4
        // and bias loads inside the loop instead of hoisted into registers
        uint32_t loff = static_cast<uint32_t>(lane) * 16;
        asm volatile("" : "+v"(loff));
        uint32_t boff = static_cast<uint32_t>(h) * 64;
        asm volatile("" : "+v"(boff));
        const float* const bimg = reinterpret_cast<const float*>(img + C::BIAS_AT + boff);
        f32x16 acc[C::NB1];
#pragma unroll
        for (int nb = 0; nb < C::NB1; ++nb) acc[nb] = ldbias(bimg + (C::BOFF1 >> 2) + nb * 32);
        float fm = 0.f;
#pragma unroll
        for (int t = 0; t < C::KT1; ++t)
#pragma unroll
            for (int j = 0; j < 8; ++j) fm = __builtin_fmaxf(fm, fabsf(xv[t][j]));
        int p = head_scale_exp(pair_max(__float_as_uint(fm)));
        f16x8 ah[C::KT1], al[C::KT1];
        {
            const float sc = exp2_int(p);
#pragma unroll
            for (int t = 0; t < C::KT1; ++t) split8(xv[t], sc, ah[t], al[t]);
        }
        // ---- L1 (H -> H) + ReLU
        if constexpr ((DIAG & 2) == 0)
            layer_mfma<C::NB1, C::KT1, (DIAG & 4) != 0>(acc, exp2_int(p + q1), lds, loff, ah, al);
        p = chain<C::NB1, C::NB2>(acc, p + q1, ah, al, bimg + (C::BOFF2 >> 2));
        // ---- L2 (H -> H) + ReLU
        if constexpr ((DIAG & 2) == 0)
            layer_mfma<C::NB2, C::KT2, (DIAG & 4) != 0>(acc, exp2_int(p + q2), lds,
                                                         lds_base(C::W1_BYTES + loff), ah, al);
        p = chain<C::NB2, C::NB3>(acc, p + q2, ah, al, bimg + (C::BOFF3 >> 2));
        // ---- L3 (H -> H/2) + ReLU.  Issued ahead of its MFMAs: W4 fragments,
        // L4's bias and the NEXT block's x rows (registers free from here on)
        f16x8 w4h[C::KT4], w4l[C::KT4];
#pragma unroll
        for (int t = 0; t < C::KT4; ++t) {
            const unsigned char* f4 = img + C::LDS_BYTES + t * C::FRAG + loff;
            w4h[t] = *reinterpret_cast<const f16x8*>(f4);
            w4l[t] = *reinterpret_cast<const f16x8*>(f4 + 64 * 16);
        }
        f32x16 o = ldbias(bimg + (C::BOFF4 >> 2));
        const int64_t row = blk * 32 + r32;
        if constexpr (PF) load_x(blk + stride);
        if constexpr ((DIAG & 2) == 0)
            layer_mfma<C::NB3, C::KT3, (DIAG & 4) != 0>(acc, exp2_int(p + q3), lds,
                                                         lds_base(C::W1_BYTES + C::W2_BYTES + loff), ah, al);
        p = chain<C::NB3, 0>(acc, p + q3, ah, al, nullptr);
        // ---- L4 (H/2 -> out), no activation
        o *= exp2_int(p + q4);
#pragma unroll
        for (int t = 0; t < C::KT4 * ((DIAG & 2) == 0 ? 1 : 0); ++t) {
            o = mfma32(w4h[t], ah[t], o);
            o = mfma32(w4h[t], al[t], o);
            o = mfma32(w4l[t], ah[t], o);
        }
        // lane (row, h) holds outputs 4 h .. 4 h + 3 in registers 0..3
        if (row < nrows) {
            const float un = exp2_int(max(-(p + q4), -126));
            const int64_t orow = out_rows != nullptr ? static_cast<int64_t>(out_rows[row]) : row;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int oc = 4 * h + r;
                if (oc < out_dim) out[orow * ldo + oc] = o[r] * un;
            }
        }
    }
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_mlp_head_prep_bytes(int h) {
    return h == 256 ? head256_prep_bytes()
                    : h == 128 ? MCfg<128>::IMG_BYTES : h == 64 ? MCfg<64>::IMG_BYTES : 0;
}

extern "C" int mignn_mlp_head_prep(const float* w1, const float* b1, const float* w2,
                                   const float* b2, const float* w3, const float* b3,
                                   const float* w4, const float* b4, int h, int out_dim,
                                   void* img, size_t img_bytes, void* stream) {
    MIGNN_REQUIRE(w1 && b1 && w2 && b2 && w3 && b3 && w4 && b4 && img,
                  "mlp_head_prep: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128 || h == 256, "mlp_head_prep: h must be 64, 128 or 256 (got %d)", h);
    MIGNN_REQUIRE(out_dim >= 1 && out_dim <= 8, "mlp_head_prep: out_dim must be 1..8 (got %d)",
                  out_dim);
    MIGNN_REQUIRE(img_bytes >= mignn_mlp_head_prep_bytes(h), "mlp_head_prep: image too small");
    MIGNN_REQUIRE(aligned16(img), "mlp_head_prep: unaligned image");
    if (h == 256) return head256_prep(w1, b1, w2, b2, w3, b3, w4, b4, out_dim, img, stream);
    hipStream_t st = as_stream(stream);
    auto* im = static_cast<unsigned char*>(img);
    if (h == 128)
        hipLaunchKernelGGL(mlp_prep_kernel<128>, dim3(4), dim3(256), 0, st, w1, b1, w2, b2, w3,
                           b3, w4, b4, out_dim, im);
    else
        hipLaunchKernelGGL(mlp_prep_kernel<64>, dim3(4), dim3(256), 0, st, w1, b1, w2, b2, w3, b3,
                           w4, b4, out_dim, im);
    return launch_status("mlp_prep_kernel");
}

extern "C" int mignn_mlp_head(const float* x, int64_t ldx, int64_t n, int h, const void* img,
                              int out_dim, float* out, int64_t ldo, const int32_t* out_rows,
                              void* stream) {
    MIGNN_REQUIRE(x && img && out, "mlp_head: null pointer");
    MIGNN_REQUIRE(h == 64 || h == 128 || h == 256, "mlp_head: h must be 64, 128 or 256 (got %d)", h);
    MIGNN_REQUIRE(out_dim >= 1 && out_dim <= 8, "mlp_head: out_dim must be 1..8 (got %d)",
                  out_dim);
    MIGNN_REQUIRE(aligned16(x) && ldx % 4 == 0 && ldx >= h, "mlp_head: x must be 16-B rows");
    MIGNN_REQUIRE(ldo >= out_dim, "mlp_head: bad ldo");
    MIGNN_REQUIRE(aligned16(img), "mlp_head: unaligned image");
    if (n <= 0) return MIGNN_OK;
    if (h == 256) return head256(x, ldx, n, img, out_dim, out, ldo, out_rows, stream);
    hipStream_t st = as_stream(stream);
    static int cus_cache[64] = {0};
    int dev = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    int& cus = cus_cache[dev & 63];
    if (cus == 0) MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t nblk = (n + 31) / 32;
    const int64_t want = (nblk + MCfg<128>::NW - 1) / MCfg<128>::NW;
    // H = 128 fills LDS (one workgroup per CU); H = 64 fits three
    const int64_t cap = h == 128 ? cus : 3 * static_cast<int64_t>(cus);
    const int grid = static_cast<int>(want < cap ? want : cap);
    if (h == 128)
        hipLaunchKernelGGL(mlp_head_kernel<128>, dim3(grid), dim3(MCfg<128>::NT), 0, st, x, ldx, n,
                           static_cast<const unsigned char*>(img), out_dim, out, ldo, out_rows);
    else
        hipLaunchKernelGGL(mlp_head_kernel<64>, dim3(grid), dim3(MCfg<64>::NT), 0, st, x, ldx, n,
                           static_cast<const unsigned char*>(img), out_dim, out, ldo, out_rows);
    return launch_status("mlp_head_kernel");
}

#ifdef MIGNN_DIAG
extern "C" int mignn_diag_mlp_head(int mode, const float* x, int64_t n, const void* img,
                                   float* out, void* stream) {
    MIGNN_REQUIRE(x && img && out && n > 0 && mode >= 0 && mode <= 5, "diag_mlp_head: bad args");
    hipStream_t st = as_stream(stream);
    int dev = 0, cus = 0;
    MIGNN_HIP(hipGetDevice(&dev));
    MIGNN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int64_t want = ((n + 31) / 32 + 7) / 8;
    const int grid = static_cast<int>(want < cus ? want : cus);
    const auto* im = static_cast<const unsigned char*>(img);
    switch (mode) {
    case 0: hipLaunchKernelGGL((mlp_head_kernel<128, 0>), dim3(grid), dim3(512), 0, st, x, 128, n, im, 7, out, 7, nullptr); break;
    case 1: hipLaunchKernelGGL((mlp_head_kernel<128, 1>), dim3(grid), dim3(512), 0, st, x, 128, n, im, 7, out, 7, nullptr); break;
    case 2: hipLaunchKernelGGL((mlp_head_kernel<128, 2>), dim3(grid), dim3(512), 0, st, x, 128, n, im, 7, out, 7, nullptr); break;
    case 3: hipLaunchKernelGGL((mlp_head_kernel<128, 3>), dim3(grid), dim3(512), 0, st, x, 128, n, im, 7, out, 7, nullptr); break;
    case 4: hipLaunchKernelGGL((mlp_head_kernel<128, 4>), dim3(grid), dim3(512), 0, st, x, 128, n, im, 7, out, 7, nullptr); break;
    default: {   // 12 waves per workgroup (exact results)
        const int64_t w12 = ((n + 31) / 32 + 11) / 12;
        const int g12 = static_cast<int>(w12 < cus ? w12 : cus);
        hipLaunchKernelGGL((mlp_head_kernel<128, 0, 12>), dim3(g12), dim3(768), 0, st, x, 128, n, im, 7, out, 7, nullptr);
        break;
    }
    }
    return launch_status("mlp_head_kernel(diag)");
}
#endif
