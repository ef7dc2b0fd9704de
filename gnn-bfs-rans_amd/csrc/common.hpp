// Shared helpers for the libmignn HIP sources (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/mignn.h"
#include "../../include/mignn_diag.h"

namespace mignn {

// Thread-local description of the last failure (mignn_last_error()).
void set_error(const char* fmt, ...);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Check the launch that was just enqueued.
inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return MIGNN_ERR_HIP;
    }
    return MIGNN_OK;
}

#define MIGNN_REQUIRE(cond, ...)                  \
    do {                                          \
        if (!(cond)) {                            \
            ::mignn::set_error(__VA_ARGS__);      \
            return MIGNN_ERR_ARG;                 \
        }                                         \
    } while (0)


#define MIGNN_HIP(call)                                                        \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) {                                                \
            ::mignn::set_error("%s: %s", #call, hipGetErrorString(e_));        \
            return MIGNN_ERR_HIP;                                              \
        }                                                                      \
    } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

inline unsigned grid_for(int64_t work, int block, int64_t cap = 1 << 20) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return static_cast<unsigned>(g);
}

// f32 MFMA 16x16x4: lane l supplies A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
// acc[r] = D[row=(l>>4)*4+r][col=l&15].  Exact fp32 (k-ordered fmaf chain).
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// streaming store (non-temporal): the written rows do not displace gathered
// rows from L2
__device__ __forceinline__ void st4_nt(float* p, float4 v) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
}

// Raw buffer loads through a hand-built 128-bit descriptor (the clang
// __builtin_amdgcn_raw_buffer_load_b64 of this toolchain lowers to a 4-byte
// load, so the LLVM intrinsics are bound directly).  Descriptor: base (48
// bit, stride 0), num_records = bytes, dword3 = 0x00020000 (gfx9 raw buffer).
using i32x4 = __attribute__((ext_vector_type(4))) int;
using f32x2 = __attribute__((ext_vector_type(2))) float;
__device__ f32x2 raw_buffer_load_f32x2(i32x4 rsrc, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.raw.buffer.load.v2f32");
__device__ float raw_buffer_load_f32(i32x4 rsrc, int voffset, int soffset, int aux) __asm(
    "llvm.amdgcn.raw.buffer.load.f32");

// Structured buffer (idxen): address = base + vindex * stride + voffset; a
// lane whose vindex >= num_records reads zeros and generates no memory
// request (per-lane range check: a branch-free "no load" for empty slots).
__device__ f32x4 struct_buffer_load_f32x4(i32x4 rsrc, int vindex, int voffset, int soffset,
                                          int aux) __asm("llvm.amdgcn.struct.buffer.load.v4f32");

__device__ __forceinline__ i32x4 struct_rsrc(uint64_t base, uint32_t stride_bytes,
                                             uint32_t num_records) {
    return i32x4{static_cast<int>(static_cast<uint32_t>(base)),
                 static_cast<int>((static_cast<uint32_t>(base >> 32) & 0xffffu) |
                                  ((stride_bytes & 0x3fffu) << 16)),
                 static_cast<int>(num_records), 0x00020000};
}

__device__ __forceinline__ i32x4 buffer_rsrc(uint64_t base, uint32_t bytes) {
    return i32x4{static_cast<int>(static_cast<uint32_t>(base)),
                 static_cast<int>(static_cast<uint32_t>(base >> 32) & 0xffffu),
                 static_cast<int>(bytes), 0x00020000};
}

// VPL (1 or 2) consecutive floats, one 4-/8-B access
template <int VPL>
__device__ __forceinline__ void ldv(const float* p, float (&v)[VPL]) {
    static_assert(VPL == 1 || VPL == 2, "VPL");
    if constexpr (VPL == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x;
        v[1] = t.y;
    } else {
        v[0] = *p;
    }
}
template <int VPL>
__device__ __forceinline__ void stv(float* p, const float (&v)[VPL]) {
    if constexpr (VPL == 2) *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
    else *p = v[0];
}

// p[n .. n+3] with components >= n_valid read as 0; a 16-B load when all four
// are valid and p + n is 16-B aligned, scalar loads otherwise.
__device__ __forceinline__ float4 ld4_masked(const float* p, int n, int n_valid) {
    const float* q = p + n;
    if (n + 4 <= n_valid && (reinterpret_cast<uintptr_t>(q) & 15u) == 0) return ld4(q);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n + 0 < n_valid) v.x = q[0];
    if (n + 1 < n_valid) v.y = q[1];
    if (n + 2 < n_valid) v.z = q[2];
    if (n + 3 < n_valid) v.w = q[3];
    return v;
}

__device__ __forceinline__ float4 fma4(float s, float4 x, float4 acc) {
    acc.x = fmaf(s, x.x, acc.x);
    acc.y = fmaf(s, x.y, acc.y);
    acc.z = fmaf(s, x.z, acc.z);
    acc.w = fmaf(s, x.w, acc.w);
    return acc;
}

// Split-fp16 pair: (a0, a1) times the power of two f -> hi = f16(a f),
// lo = f16(a f - hi) packed two halves a dword (element 0 in the low half).
// a f and a f - hi are exact in fp32, so each half is one rounding of the
// same value as converting the scaled product and its remainder.  The
// mixed-precision FMA writes each half straight from the fp32 operands
// (v_fma_mixlo / mixhi_f16, hi's half as an f16 source for lo): 4 VALU per
// pair, where the compiler's own form of the same arithmetic is SLP-packed
// v_pk_mul_f32 + v_cvt_pk_f16_f32 + 2 v_cvt_f32_f16 + v_pk_fma_f32 + a
// second v_cvt_pk_f16_f32.
__device__ __forceinline__ void split_pair(float a0, float a1, float f, uint32_t& hi,
                                           uint32_t& lo) {
    asm("v_fma_mixlo_f16 %0, %1, %3, 0\n\t"
        "v_fma_mixhi_f16 %0, %2, %3, 0"
        : "=&v"(hi) : "v"(a0), "v"(a1), "v"(f));
    asm("v_fma_mixlo_f16 %0, %1, %3, -%4 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %0, %2, %3, -%4 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(lo) : "v"(a0), "v"(a1), "v"(f), "v"(hi));
}

// Reference epilogue order (gnn_model.py:184-191 with the conv bias first):
//   v = acc + bias; v = residual + v; v = v*scale + shift; relu.
// ReLU in one v_maximum3_f32: NaN-propagating, like torch.relu (-0 -> +0)
__device__ __forceinline__ float relu_nan(float v) { return __builtin_elementwise_maximum(v, 0.0f); }

// A planned layer launch whose plan header does not match it: besides the
// device error bit, every output row of the launch's range becomes NaN (the
// whole grid, grid-stride, vector stores) -- a caller that does not read the
// error word still cannot take the buffer's old contents for layer output.
__device__ inline void plan_mismatch_fill(float* out, int64_t ldo, int64_t rb, int64_t re, int h) {
    const float qnan = __builtin_nanf("");
    const int64_t n = (re - rb) * static_cast<int64_t>(h);
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x)
        out[(rb + i / h) * ldo + i % h] = qnan;
}

__device__ __forceinline__ float epilogue(float acc, int flags, float bias, float res, float sc,
                                          float sh) {
    float v = acc;
    if (flags & MIGNN_EPI_BIAS) v = v + bias;
    if (flags & MIGNN_EPI_RESIDUAL) v = res + v;
    if (flags & MIGNN_EPI_AFFINE) v = v * sc + sh;
    if (flags & MIGNN_EPI_RELU) v = relu_nan(v);
    return v;
}

// Register-resident-W persistent row-tile GEMM (tile_gemm.hip) for the
// FlowGNN layer / head shapes; *handled=false when (k, n) has no instance.
// mignn_transformer_aggregate with the per-head score constant optional
// (aggregate.hip; use_cq = false: qt's last `heads` columns are not read)
int transformer_aggregate_rows(const int32_t* row_ptr, const int32_t* col, const float* qt,
                               int64_t ldq, const float* x, int64_t ldx, int64_t rb, int64_t re,
                               int h, int heads, float score_scale, float* out, int64_t ldo,
                               bool use_cq, void* stream);
// the fused GAT layer (agg_gemm.hip): heads = 4, h in {64, 128}, wcat image
int gat_layer_fused(const int32_t* row_ptr, const int32_t* col, const float* logits,
                    const float* x, int64_t ldx, int64_t rb, int64_t re, int h, float slope,
                    const void* img, const float* bias, const float* scale, const float* shift,
                    int flags, float* out, int64_t ldo, void* stream,
                    const float* wlog_next = nullptr, float* lg_next = nullptr);
// the fused TransformerConv (H = 256, 4 heads; agg_gemm.hip): image of wout
// in the fused k order, and the aggregate + output transform kernel over qt
size_t tf_fused_prep_bytes();
int tf_fused_prep(const float* wout, void* img, void* stream);
int tf_fused(const int32_t* row_ptr, const int32_t* col, const float* qt, int64_t ldq,
             const float* x, int64_t ldx, int64_t rb, int64_t re, float score_scale,
             const void* img, const float* bias, const float* scale, const float* shift, int flags,
             float* out, int64_t ldo, void* stream);
// the fused H = 256 output head (agg_gemm.hip), arguments checked by mlp_f16x3.hip
size_t head256_prep_bytes();
int head256_prep(const float* w1, const float* b1, const float* w2, const float* b2,
                 const float* w3, const float* b3, const float* w4, const float* b4, int out_dim,
                 void* img, void* stream);
int head256(const float* x, int64_t ldx, int64_t n, const void* img, int out_dim, float* out,
            int64_t ldo, const int32_t* out_rows, void* stream);
// LDS-DMA destination bound (diag builds only): a global_load_lds_dwordx4
// writes 1 KiB from the wave-uniform LDS address `dst`; it must end inside
// the issuing kernel's static LDS allocation (__builtin_amdgcn_groupstaticsize:
// the block's own bytes -- past them lie a co-resident block's).  A violation
// sets the translation unit's word g_dma_oob (mignn_diag_dma_oob_<unit>).
#ifdef MIGNN_DIAG
#define MIGNN_DMA_OOB_WORD namespace { __device__ unsigned int g_dma_oob = 0u; }
#define MIGNN_DMA_BOUND(dst)                                                               \
    do {                                                                                   \
        if (static_cast<uint32_t>(dst) + 1024u >                                           \
                static_cast<uint32_t>(__builtin_amdgcn_groupstaticsize()) &&               \
            (threadIdx.x & 63u) == 0u)                                                     \
            __hip_atomic_fetch_or(&g_dma_oob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    } while (0)
#define MIGNN_DMA_OOB_EXPORT(name)                                                          \
    extern "C" int name(unsigned int* out, int clear) {                                     \
        unsigned int v = 0u;                                                                \
        MIGNN_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(mignn::g_dma_oob), sizeof(v), 0,       \
                                      hipMemcpyDeviceToHost));                              \
        *out = v;                                                                           \
        if (clear) {                                                                        \
            const unsigned int zero = 0u;                                                   \
            MIGNN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(mignn::g_dma_oob), &zero, sizeof(zero), 0, \
                                        hipMemcpyHostToDevice));                            \
        }                                                                                   \
        return MIGNN_OK;                                                                    \
    }
#else
#define MIGNN_DMA_OOB_WORD
#define MIGNN_DMA_BOUND(dst) \
    do {                     \
    } while (0)
#define MIGNN_DMA_OOB_EXPORT(name)
#endif
// the window GCN kernel's device error word, OR-ed into *out (gcn_win.hip)
int win_device_errors(unsigned int* out, int clear);
// the ring GCN kernel's device error word, OR-ed into *out (gcn_ring.hip)
int ring_device_errors(unsigned int* out, int clear);
int tile_linear(const float* a, int64_t lda, int64_t m, int k, const float* w, int n,
                const float* bias, const float* residual, int64_t ldr, const float* scale,
                const float* shift, int flags, float* c, int64_t ldc, hipStream_t st,
                bool* handled);

// Attention-dropout mask of the GAT / Transformer training kernels
// (gat_train.hip, transformer_train.hip): splitmix64 counter hash of
// (seed, dst, src, head), regenerated in the backward -- nothing stored.
__device__ __forceinline__ uint32_t edge_hash(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;   // splitmix64
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return static_cast<uint32_t>(z >> 32);
}

struct EdgeDrop {
    uint64_t seed;
    uint32_t thresh;   // drop if hash < thresh (0: no dropout)
    float scale;       // 1 / (1 - p); 0 when p >= 1
    int64_t n;
    int heads;
    __device__ __forceinline__ float keep(int64_t i, int64_t j, int k) const {
        if (thresh == 0u) return scale;
        const uint64_t idx = (static_cast<uint64_t>(i) * n + j) * heads + k;
        return edge_hash(seed, idx) >= thresh ? scale : 0.f;
    }
};

inline EdgeDrop make_edge_drop(float p, uint64_t seed, int64_t n, int heads) {
    EdgeDrop d{seed, 0u, 1.f, n, heads};
    if (p >= 1.f) {
        d.thresh = 0xFFFFFFFFu;
        d.scale = 0.f;
    } else if (p > 0.f) {
        d.thresh = static_cast<uint32_t>(static_cast<double>(p) * 4294967296.0);
        d.scale = 1.f / (1.f - p);
    }
    return d;
}

}  // namespace mignn
