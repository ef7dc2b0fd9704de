// Diagnostic kernels (timing studies only; declared in include/mignn_diag.h,
// not part of the product ABI): what the memory system delivers for the GCN
// gather pattern with and without CSR index traffic.
//
//   mode 0  CSR gather, half-wave per row, all edges of a row in flight
//           (deg <= 8), weights from ew -> out[i] = sum w_e x[col_e]
//   mode 1  stencil gather on the periodic (nx, ny, nz) grid: neighbour ids
//           computed from the row id (no index loads) -> the memory system's
//           best case for this access pattern
//   mode 2  streaming copy out[i] = x[i] (16 B per lane)
//   mode 3  the same copy in the store pattern of a 16x16 MFMA accumulator
//           tile: a wave owns 16 rows, lane (r, g) moves 16 B at column
//           16 cb + 4 g of row r -- every instruction 16 rows x 64 B
//   | 4     XCD-aware block -> row remap (contiguous row chunks per XCD per step)
//   | 8     non-temporal output stores
#include "common.hpp"

#ifdef MIGNN_DIAG   // diagnostic library only (libmignn_diag.so)

namespace mignn {
namespace {

template <int MODE, bool REMAP, bool NT>
__global__ __launch_bounds__(256) void diag_gather_kernel(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ x, int64_t n, int nx, int ny, int nz,
    float* __restrict__ out) {
    constexpr int H = 128, LPR = 32;
    const int lane = threadIdx.x & 63;
    const int c = lane % LPR;
    const int64_t nrow_groups = ((int64_t)gridDim.x * blockDim.x) / LPR;
    int64_t blk = blockIdx.x;
    if (REMAP) {   // steps of S = 8 * 256 blocks; XCD group x gets a contiguous run of 256
        constexpr int64_t S = 8 * 256;
        const int64_t step = blk / S, i = blk % S;
        blk = step * S + (i % 8) * 256 + i / 8;
    }
    for (int64_t row = (blk * blockDim.x + threadIdx.x) / LPR; row < n; row += nrow_groups) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (MODE == 0) {
            const int beg = row_ptr[row], deg = row_ptr[row + 1] - beg;
            int j[8];
            float w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                j[u] = u < deg ? col[beg + u] : static_cast<int>(row);
                w[u] = u < deg ? ew[beg + u] : 0.f;
            }
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ld4(x + (int64_t)j[u] * H + 4 * c);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = fma4(w[u], v[u], acc);
        } else if constexpr (MODE == 1) {
            const int64_t plane = (int64_t)nx * ny;
            const int i = static_cast<int>(row % nx);
            const int jj = static_cast<int>((row / nx) % ny);
            const int k = static_cast<int>(row / plane);
            const int64_t nb[7] = {
                row,
                (int64_t)k * plane + (int64_t)jj * nx + (i + nx - 1) % nx,
                (int64_t)k * plane + (int64_t)jj * nx + (i + 1) % nx,
                (int64_t)k * plane + (int64_t)((jj + ny - 1) % ny) * nx + i,
                (int64_t)k * plane + (int64_t)((jj + 1) % ny) * nx + i,
                (int64_t)((k + nz - 1) % nz) * plane + (int64_t)jj * nx + i,
                (int64_t)((k + 1) % nz) * plane + (int64_t)jj * nx + i};
            float4 v[7];
#pragma unroll
            for (int u = 0; u < 7; ++u) v[u] = ld4(x + nb[u] * H + 4 * c);
#pragma unroll
            for (int u = 0; u < 7; ++u) acc = fma4(0.14285715f, v[u], acc);
        } else if constexpr (MODE == 3) {
            // row = this lane group's 16-row block id (LPR = 32 lanes -> 2
            // groups per wave; use the wave instead: 16 rows per wave)
            const int64_t wave = (blk * blockDim.x + threadIdx.x) >> 6;
            const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
            const int r = lane & 15, g = lane >> 4;
            for (int64_t b = wave; b * 16 < n; b += nwaves) {
                const int64_t rr = b * 16 + r;
                if (rr < n) {
                    float4 v[8];
#pragma unroll
                    for (int cb = 0; cb < 8; ++cb) v[cb] = ld4(x + rr * H + 16 * cb + 4 * g);
#pragma unroll
                    for (int cb = 0; cb < 8; ++cb) {
                        const f32x4 w = {v[cb].x, v[cb].y, v[cb].z, v[cb].w};
                        if (NT) __builtin_nontemporal_store(w, reinterpret_cast<f32x4*>(out + rr * H + 16 * cb + 4 * g));
                        else *reinterpret_cast<f32x4*>(out + rr * H + 16 * cb + 4 * g) = w;
                    }
                }
            }
            return;
        } else {
            acc = ld4(x + row * H + 4 * c);
        }
        if (NT) {
            const f32x4 v = {acc.x, acc.y, acc.z, acc.w};
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(out + row * H + 4 * c));
        } else {
            st4(out + row * H + 4 * c, acc);
        }
    }
}

// mode 16 | D: the fused layer's streaming skeleton -- one 4-wave block per
// CU, persistent over 64-row tiles (XCD-contiguous order), own rows LDS-DMA'd
// D-1 steps ahead into a ring of D images, each wave copies its 16 rows out
// of the image in the accumulator store pattern (16 rows x 64 B, non-temporal)
__device__ __forceinline__ void dma16_diag(const void* src, uint32_t dst) {
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

// VAR 0: stores in the accumulator pattern, a block barrier per step;
// VAR 1: whole-row stores (a half-wave per 512-B row), barrier per step;
// VAR 2: whole-row stores, no barrier (each wave DMAs exactly its own 16 rows
//        and waits for them itself)
template <int D, int VAR>
__global__ __launch_bounds__(256, 1) void diag_stream_kernel(const float* __restrict__ x, int64_t n,
                                                             float* __restrict__ out) {
    constexpr int H = 128, BM = 64, ROWB = 512, XB = BM * ROWB, NPIECE = XB / 1024 / 4;
    constexpr int NST = 8;
    // vmcnt(N) lgkmcnt(0) at the end of step s: ops younger than step s+1's
    // DMA = the stores of steps s-D+2 .. s and the DMAs of steps s+2 .. s+D-1
    constexpr int N = (D - 1) * NST + (D - 2) * NPIECE;
    constexpr int WAIT = (N & 15) | ((N >> 4) << 14) | (7 << 4);
    // VAR 2, at the start of step s for step s's own DMA: younger = the stores
    // of steps s-D+1 .. s-1 and the DMAs of steps s+1 .. s+D-1
    constexpr int N2 = (D - 1) * NST + (D - 1) * NPIECE;
    constexpr int WAIT2 = (N2 & 15) | ((N2 >> 4) << 14) | (7 << 4);
    __shared__ __attribute__((aligned(16))) unsigned char lds[D * XB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int64_t ntiles = n / BM;                   // host: n % 64 == 0
    const int G = gridDim.x;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = G >> 3;
    const int64_t nsteps = (ntiles + G - 1) / G;
    const int64_t chunk = nsteps * per_xcd;
    auto tile_of = [&](int64_t s) -> int64_t { return (int64_t)xcd * chunk + s * per_xcd + slot; };
    auto issue = [&](int64_t s) {
        int64_t t = tile_of(s);
        if (s >= nsteps || t >= ntiles) t = 0;        // keep the op count uniform
        unsigned char* const X = lds + (s % D) * XB;
#pragma unroll
        for (int pc = 0; pc < NPIECE; ++pc) {
            const int piece = wave * NPIECE + pc;
            const int lr = piece * 2 + lane / 32;
            const int pos = lane % 32;
            dma16_diag(x + (t * BM + lr) * H + 4 * (pos ^ (lr & 15)), static_cast<uint32_t>(
                reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)(X + piece * 1024))));
        }
    };
    for (int d = 0; d < D - 1; ++d) issue(d);
    __builtin_amdgcn_s_waitcnt(0x70);
    __builtin_amdgcn_s_barrier();
    for (int64_t s = 0; s < nsteps; ++s) {
        issue(s + D - 1);
        const int64_t t = tile_of(s);
        const unsigned char* const X = lds + (s % D) * XB;
        if constexpr (VAR >= 1) {
            if constexpr (VAR == 2) {
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_waitcnt(WAIT2);     // my own pieces of step s landed
                asm volatile("" ::: "memory");
            }
            const int ch = lane & 31;
            f32x4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int lr = 16 * wave + 2 * i + (lane >> 5);
                v[i] = *reinterpret_cast<const f32x4*>(X + lr * ROWB + 16 * (ch ^ (lr & 15)));
            }
            const int64_t tt = t < ntiles ? t : 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int lr = 16 * wave + 2 * i + (lane >> 5);
                __builtin_nontemporal_store(v[i], reinterpret_cast<f32x4*>(out + (tt * BM + lr) * H + 4 * ch));
            }
            if constexpr (VAR == 1) {
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_waitcnt(WAIT);
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
            continue;
        }
        const int lr = 16 * wave + r;
        f32x4 v[8];
#pragma unroll
        for (int nb = 0; nb < 8; ++nb)
            v[nb] = *reinterpret_cast<const f32x4*>(X + lr * ROWB + 16 * ((4 * nb + g) ^ (lr & 15)));
        if (t < ntiles) {
#pragma unroll
            for (int nb = 0; nb < 8; ++nb)
                __builtin_nontemporal_store(v[nb], reinterpret_cast<f32x4*>(out + (t * BM + lr) * H + 16 * nb + 4 * g));
        } else {
#pragma unroll
            for (int nb = 0; nb < 8; ++nb)
                __builtin_nontemporal_store(v[nb], reinterpret_cast<f32x4*>(out + lr * H + 16 * nb + 4 * g));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(WAIT);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_s_waitcnt(0x70);
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_diag_gather(int mode, const int32_t* row_ptr, const int32_t* col,
                                 const float* ew, const float* x, int64_t n, int nx, int ny,
                                 int nz, int blocks, float* out, void* stream) {
    hipStream_t st = as_stream(stream);
    const int g = blocks > 0 ? blocks : static_cast<int>(grid_for(n * 32, 256, 1 << 20));
#define MIGNN_DIAG(M, R, T) \
    hipLaunchKernelGGL((diag_gather_kernel<M, R, T>), dim3(g), dim3(256), 0, st, row_ptr, col, ew, x, n, nx, ny, nz, out)
    if (mode >= 16) {
        MIGNN_REQUIRE(n % 64 == 0 && blocks > 0 && blocks % 8 == 0, "diag stream: n % 64, blocks % 8");
        const int d = mode & 15, var = (mode >> 5) & 3;
#define MIGNN_STREAM(DD, VV) \
        if (d == DD && var == VV) hipLaunchKernelGGL((diag_stream_kernel<DD, VV>), dim3(blocks), dim3(256), 0, st, x, n, out)
        MIGNN_STREAM(2, 0); else MIGNN_STREAM(3, 0); else MIGNN_STREAM(4, 0);
        else MIGNN_STREAM(2, 1); else MIGNN_STREAM(3, 1); else MIGNN_STREAM(4, 1);
        else MIGNN_STREAM(2, 2); else MIGNN_STREAM(3, 2); else MIGNN_STREAM(4, 2);
        else { set_error("diag stream: depth 2..4, variant 0..2"); return MIGNN_ERR_ARG; }
#undef MIGNN_STREAM
        return launch_status("diag_stream_kernel");
    }
    const int base = mode & 3;
    const bool remap = mode & 4, nt = mode & 8;
    if (remap && blocks > 0) { set_error("diag: remap needs a full grid"); return MIGNN_ERR_ARG; }
    if (base == 0) {
        if (remap) { if (nt) MIGNN_DIAG(0, true, true); else MIGNN_DIAG(0, true, false); }
        else { if (nt) MIGNN_DIAG(0, false, true); else MIGNN_DIAG(0, false, false); }
    } else if (base == 1) {
        if (remap) { if (nt) MIGNN_DIAG(1, true, true); else MIGNN_DIAG(1, true, false); }
        else { if (nt) MIGNN_DIAG(1, false, true); else MIGNN_DIAG(1, false, false); }
    } else if (base == 2) {
        if (nt) MIGNN_DIAG(2, false, true); else MIGNN_DIAG(2, false, false);
    } else {
        if (nt) MIGNN_DIAG(3, false, true); else MIGNN_DIAG(3, false, false);
    }
#undef MIGNN_DIAG
    return launch_status("diag_gather_kernel");
}

// ---- shader clock probe: every workgroup runs `iters` dependent FMAs per
// lane and records (s_memtime delta, s_memrealtime delta); clock MHz =
// dt_shader / dt_real * 100 (MI355X_MICROARCH.md: s_memrealtime ticks at 100 MHz)
namespace {
__global__ __launch_bounds__(256) void clock_probe_kernel(int iters, int64_t* out) {
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    float a = static_cast<float>(threadIdx.x) * 1e-3f, b = 1.0000001f, c = 1e-7f;
    for (int i = 0; i < iters; ++i) {
        a = fmaf(a, b, c);
        a = fmaf(a, b, c);
        a = fmaf(a, b, c);
        a = fmaf(a, b, c);
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = static_cast<int64_t>(t1 - t0);
        out[2 * blockIdx.x + 1] = static_cast<int64_t>(r1 - r0);
    }
    if (a == 12345.f) out[0] = 0;   // keep the chain
}
}  // namespace

extern "C" int mignn_diag_clock(int blocks, int iters, int64_t* out, void* stream) {
    MIGNN_REQUIRE(out && blocks > 0 && iters > 0, "diag_clock: bad args");
    hipLaunchKernelGGL(clock_probe_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), iters,
                       out);
    return launch_status("clock_probe_kernel");
}

// ---- v_pk_fma_f32 forms of the row-code expansion.
// out[i][f] = relu(coef[f][7] + sum_{k<7} coef[f][k] v[i][k]) as layer 0's
// fma chain (gcn_layer0.hip, gcn_win.hip expand4), one lane per (row, feature
// pair f, f + 1):
//   form 0  scalar v_fma_f32 chain (the reference the other forms must equal bitwise)
//   form 1  inline v_pk_fma_f32, the input broadcast to both halves by
//           op_sel_hi:[1,0,1] (the high result takes src1's LOW half)
//   form 2  the same instruction without the op_sel_hi modifier (its
//           default, op_sel_hi:[1,1,1]): the high result takes src1's HIGH
//           half -- with the inputs loaded as pairs {v[k], v[k+1]} that is
//           the neighbouring input, so feature f + 1 is wrong in every row
//   form 3  the packed form the compiler emits itself (__builtin_elementwise_fma
//           on 2-vectors)
namespace {
template <int FORM>
__global__ __launch_bounds__(256) void pk_fma_kernel(const float* __restrict__ codes, int64_t n,
                                                     const float* __restrict__ coef, int h,
                                                     float* __restrict__ out) {
    const int pairs = h / 2;
    for (int64_t id = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; id < n * pairs;
         id += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t i = id / pairs;
        const int f = 2 * static_cast<int>(id % pairs);
        const float* v = codes + i * 8;
        const float* c0 = coef + f * 8;
        const float* c1 = coef + (f + 1) * 8;
        float r0, r1;
        if constexpr (FORM == 0) {
            float t0 = c0[7], t1 = c1[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                // (explicit v_fma_f32: plain fmaf here is SLP-packed into
                // v_pk_fma_f32 by the compiler, which is form 3's subject)
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(t0) : "v"(c0[k]), "v"(v[k]));
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(t1) : "v"(c1[k]), "v"(v[k]));
            }
            r0 = t0;
            r1 = t1;
        } else if constexpr (FORM == 3) {
            f32x2 t = f32x2{c0[7], c1[7]};
#pragma unroll
            for (int k = 0; k < 7; ++k)
                t = __builtin_elementwise_fma(f32x2{c0[k], c1[k]}, f32x2{v[k], v[k]}, t);
            r0 = t[0];
            r1 = t[1];
        } else {
            f32x2 t = f32x2{c0[7], c1[7]};
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                const f32x2 cp = f32x2{c0[k], c1[k]};
                const f32x2 vp = f32x2{v[k], v[k + 1]};   // inputs as loaded: a pair
                if constexpr (FORM == 1)
                    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(t) : "v"(cp), "v"(vp));
                else
                    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(t) : "v"(cp), "v"(vp));
            }
            r0 = t[0];
            r1 = t[1];
        }
        out[i * h + f] = relu_nan(r0);
        out[i * h + f + 1] = relu_nan(r1);
    }
}
}  // namespace

extern "C" int mignn_diag_pk_fma(int form, const float* codes, int64_t n, const float* coef, int h,
                                 float* out, void* stream) {
    MIGNN_REQUIRE(codes && coef && out && n >= 0 && h > 0 && h % 2 == 0, "diag_pk_fma: bad args");
    if (n == 0) return MIGNN_OK;
    const unsigned g = static_cast<unsigned>(grid_for(n * (h / 2), 256, 4096));
    hipStream_t st = as_stream(stream);
    switch (form) {
        case 0: hipLaunchKernelGGL(pk_fma_kernel<0>, dim3(g), dim3(256), 0, st, codes, n, coef, h, out); break;
        case 1: hipLaunchKernelGGL(pk_fma_kernel<1>, dim3(g), dim3(256), 0, st, codes, n, coef, h, out); break;
        case 2: hipLaunchKernelGGL(pk_fma_kernel<2>, dim3(g), dim3(256), 0, st, codes, n, coef, h, out); break;
        case 3: hipLaunchKernelGGL(pk_fma_kernel<3>, dim3(g), dim3(256), 0, st, codes, n, coef, h, out); break;
        default: set_error("diag_pk_fma: form 0..3"); return MIGNN_ERR_ARG;
    }
    return launch_status("pk_fma_kernel");
}

#endif  // MIGNN_DIAG
