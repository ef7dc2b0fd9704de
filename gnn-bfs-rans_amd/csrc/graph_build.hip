// Graph structure on the device: edge validation + destination-major CSR
// (replaces gnn_model.py:125-149 and PyG's self-loop handling / gcn_norm
// degree), the synthetic periodic hex grid, the BatchNorm eval fold and the
// halo row gather.
//
// CSR build (all on `stream`, no host sync):
//   K0 csr_keys     : per edge, key = dst (valid, kept), N (dropped: invalid
//                     index, or a self-loop in ONE_SELF_LOOP mode); value = src.
//                     Counts kept / invalid edges with one atomic per block.
//   K1 radix sort   : rocprim::radix_sort_pairs over the low ceil(log2(N+1))
//                     bits -- stable, so in-row order == edge order.
//   K2 row_bounds   : row_ptr0[i] = first sorted position with key >= i.
//   K3 csr_expand   : final row_ptr/col; ONE_SELF_LOOP mode appends (i, i) to
//                     every row and writes dinv = deg^-1/2; VERBATIM mode with
//                     E > 0 and zero kept edges takes the reference's
//                     all-invalid fallback (one self-loop per node,
//                     gnn_model.py:144-149).
#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <cstring>

#include "common.hpp"

namespace mignn {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

namespace {

constexpr int kBlock = 256;

__global__ void csr_keys_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t N, int mode,
                                int transpose, const int32_t* __restrict__ relabel,
                                uint32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                unsigned long long* __restrict__ counters) {
    __shared__ unsigned int s_kept, s_bad;
    if (threadIdx.x == 0) { s_kept = 0; s_bad = 0; }
    __syncthreads();
    unsigned kept = 0, bad = 0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        // transposed: rows keyed by the source (backward of the aggregation)
        const int64_t s = ei[transpose ? E + e : e];
        const int64_t d = ei[transpose ? e : E + e];
        const bool valid = (s >= 0) & (s < N) & (d >= 0) & (d < N);
        bool keep = valid;
        if (mode == MIGNN_CSR_ONE_SELF_LOOP && s == d) keep = false;
        int64_t sn = s, dn = d;
        if (relabel != nullptr && valid) {   // node ids in the internal (relabelled) order
            sn = relabel[s];
            dn = relabel[d];
        }
        keys[e] = keep ? static_cast<uint32_t>(dn) : static_cast<uint32_t>(N);
        vals[e] = valid ? static_cast<int32_t>(sn) : 0;
        kept += keep ? 1u : 0u;
        bad += valid ? 0u : 1u;
    }
    if (kept) atomicAdd(&s_kept, kept);
    if (bad) atomicAdd(&s_bad, bad);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_kept) atomicAdd(&counters[0], (unsigned long long)s_kept);
        if (s_bad) atomicAdd(&counters[1], (unsigned long long)s_bad);
    }
}

// row_ptr0[i] = lower_bound(keys, i) for i in [0, N]; keys sorted, capped at N.
__global__ void row_bounds_kernel(const uint32_t* __restrict__ keys, int64_t E, int64_t N,
                                  int32_t* __restrict__ row_ptr0) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= E;
         p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t prev = (p == 0) ? -1 : (int64_t)min<uint32_t>(keys[p - 1], (uint32_t)N);
        const int64_t cur = (p == E) ? N : (int64_t)min<uint32_t>(keys[p], (uint32_t)N);
        for (int64_t i = prev + 1; i <= cur; ++i) row_ptr0[i] = static_cast<int32_t>(p);
    }
}

__global__ void csr_expand_nodes_kernel(const int32_t* __restrict__ row_ptr0,
                                        const int32_t* __restrict__ sorted_src, int64_t E,
                                        int64_t N, int mode,
                                        const unsigned long long* __restrict__ counters,
                                        int32_t* __restrict__ row_ptr, int32_t* __restrict__ col,
                                        float* __restrict__ dinv) {
    const bool fallback = (mode == MIGNN_CSR_VERBATIM) && (E > 0) && (counters[0] == 0);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= N;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (mode == MIGNN_CSR_ONE_SELF_LOOP) {
            const int32_t b = row_ptr0[i];
            row_ptr[i] = b + static_cast<int32_t>(i);
            if (i < N) {
                const int32_t e = row_ptr0[i + 1];
                const int32_t base = b + static_cast<int32_t>(i);
                for (int32_t t = b; t < e; ++t) col[base + (t - b)] = sorted_src[t];
                col[base + (e - b)] = static_cast<int32_t>(i);
                // PyG gcn_norm: deg.pow(-0.5); deg >= 1 here (self-loop added).
                if (dinv) dinv[i] = 1.0f / sqrtf(static_cast<float>(e - b + 1));
            }
        } else if (fallback) {
            row_ptr[i] = static_cast<int32_t>(i);
            if (i < N) col[i] = static_cast<int32_t>(i);
        } else {
            row_ptr[i] = row_ptr0[i];
        }
    }
}

__global__ void copy_i32_kernel(const int32_t* __restrict__ src, int32_t* __restrict__ dst,
                                const int32_t* __restrict__ count_at, int64_t E,
                                const unsigned long long* __restrict__ counters, int mode) {
    if (mode != MIGNN_CSR_VERBATIM || (E > 0 && counters[0] == 0)) return;
    const int64_t n = *count_at;
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
         p += (int64_t)gridDim.x * blockDim.x)
        dst[p] = src[p];
}

__global__ void csr_info_kernel(const unsigned long long* __restrict__ counters,
                                const int32_t* __restrict__ row_ptr, int64_t E, int64_t N,
                                int mode, int64_t* __restrict__ info) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        info[0] = (int64_t)counters[0];
        info[1] = (int64_t)counters[1];
        info[2] = row_ptr[N];
        info[3] = (mode == MIGNN_CSR_VERBATIM && E > 0 && counters[0] == 0) ? 1 : 0;
    }
}

inline size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

inline unsigned key_bits(int64_t N) {
    unsigned bits = 1;
    while ((uint64_t(1) << bits) <= static_cast<uint64_t>(N)) ++bits;
    return bits;
}

struct CsrScratch {
    size_t off_keys_in, off_keys_out, off_vals_in, off_vals_out, off_rowptr0, off_counters,
        off_temp, temp_bytes, total;
};

int csr_layout(int64_t E, int64_t N, CsrScratch* L) {
    size_t o = 0;
    const size_t e = static_cast<size_t>(E > 0 ? E : 1);
    L->off_keys_in = o; o = align_up(o + e * 4);
    L->off_keys_out = o; o = align_up(o + e * 4);
    L->off_vals_in = o; o = align_up(o + e * 4);
    L->off_vals_out = o; o = align_up(o + e * 4);
    L->off_rowptr0 = o; o = align_up(o + static_cast<size_t>(N + 1) * 4);
    L->off_counters = o; o = align_up(o + 4 * sizeof(unsigned long long));
    L->off_temp = o;
    size_t temp = 0;
    hipError_t err = rocprim::radix_sort_pairs(nullptr, temp, (uint32_t*)nullptr,
                                               (uint32_t*)nullptr, (int32_t*)nullptr,
                                               (int32_t*)nullptr, static_cast<size_t>(e), 0u, key_bits(N));
    if (err != hipSuccess) {
        set_error("rocprim::radix_sort_pairs size query: %s", hipGetErrorString(err));
        return MIGNN_ERR_HIP;
    }
    L->temp_bytes = temp;
    L->total = align_up(o + temp);
    return MIGNN_OK;
}

__global__ void grid_graph_kernel(int nx, int ny, int nz, int z_begin, int z_count,
                                  int64_t* __restrict__ ei, float* __restrict__ x) {
    const int64_t plane = (int64_t)nx * ny;
    const int64_t n = plane * z_count;
    const int64_t E = 6 * n;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        const int i = static_cast<int>(v % nx);
        const int j = static_cast<int>((v / nx) % ny);
        const int k = z_begin + static_cast<int>(v / plane);
        const int64_t gid = (int64_t)k * plane + (int64_t)j * nx + i;
        auto id = [&](int ii, int jj, int kk) -> int64_t {
            return (int64_t)kk * plane + (int64_t)jj * nx + ii;
        };
        const int64_t nb[6] = {
            id((i + nx - 1) % nx, j, k), id((i + 1) % nx, j, k),
            id(i, (j + ny - 1) % ny, k), id(i, (j + 1) % ny, k),
            id(i, j, (k + nz - 1) % nz), id(i, j, (k + 1) % nz),
        };
#pragma unroll
        for (int d = 0; d < 6; ++d) {
            ei[6 * v + d] = nb[d];      // src (neighbour)
            ei[E + 6 * v + d] = gid;    // dst (this node)
        }
        x[3 * v + 0] = (i + 0.5f) / nx;
        x[3 * v + 1] = (j + 0.5f) / ny;
        x[3 * v + 2] = (k + 0.5f) / nz;
    }
}

__global__ void bn_fold_kernel(const float* __restrict__ w, const float* __restrict__ b,
                               const float* __restrict__ mean, const float* __restrict__ var,
                               float eps, int h, float* __restrict__ scale,
                               float* __restrict__ shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < h) {
        // ATen batch_norm_cpu_transform_input: alpha = invstd * w; beta = b - mean * alpha
        const float invstd = 1.0f / sqrtf(var[c] + eps);
        const float a = w ? invstd * w[c] : invstd;
        scale[c] = a;
        shift[c] = (b ? b[c] : 0.0f) - mean[c] * a;
    }
}

// PyG gcn_norm edge weights per CSR entry: w_e = dinv[src] * 1 * dinv[dst].
__global__ void gcn_norm_kernel(const int32_t* __restrict__ row_ptr,
                                const int32_t* __restrict__ col, const float* __restrict__ dinv,
                                int64_t rb, int64_t re, float* __restrict__ ew) {
    for (int64_t i = rb + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < re;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float di = dinv[i];
        for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) ew[e] = dinv[col[e]] * di;
    }
}

__global__ void rows_gather_kernel(const float* __restrict__ src, int64_t lds,
                                   const int32_t* __restrict__ idx, int64_t n, int h4,
                                   float* __restrict__ dst, int64_t ldd) {
    const int64_t total = n * h4;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / h4;
        const int c = static_cast<int>(t % h4);
        st4(dst + r * ldd + 4 * c, ld4(src + (int64_t)idx[r] * lds + 4 * c));
    }
}

// any width / alignment (the head output, 7 columns)
__global__ void rows_gather1_kernel(const float* __restrict__ src, int64_t lds,
                                    const int32_t* __restrict__ idx, int64_t n, int h,
                                    float* __restrict__ dst, int64_t ldd) {
    const int64_t total = n * h;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = t / h;
        const int c = static_cast<int>(t % h);
        dst[r * ldd + c] = src[(int64_t)idx[r] * lds + c];
    }
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_abi_version(void) { return MIGNN_ABI_VERSION; }
extern "C" const char* mignn_last_error(void) { return g_err; }

extern "C" size_t mignn_csr_scratch_bytes(int64_t num_edges, int64_t num_nodes) {
    CsrScratch L;
    if (csr_layout(num_edges, num_nodes, &L) != MIGNN_OK) return 0;
    return L.total;
}

extern "C" int mignn_csr_build(const int64_t* edge_index, int64_t E, int64_t N, int mode,
                               int32_t* row_ptr, int32_t* col, float* dinv, int64_t* info,
                               void* scratch, size_t scratch_bytes, void* stream_) {
    return mignn_csr_build_relabeled(edge_index, E, N, mode, nullptr, row_ptr, col, dinv, info,
                                     scratch, scratch_bytes, stream_);
}

extern "C" int mignn_csr_build_relabeled(const int64_t* edge_index, int64_t E, int64_t N,
                                         int mode, const int32_t* relabel, int32_t* row_ptr,
                                         int32_t* col, float* dinv, int64_t* info, void* scratch,
                                         size_t scratch_bytes, void* stream_) {
    MIGNN_REQUIRE(N >= 0 && E >= 0, "csr_build: negative sizes (E=%lld N=%lld)", (long long)E,
                  (long long)N);
    MIGNN_REQUIRE(E + N < (int64_t(1) << 31) - 1, "csr_build: E+N exceeds int32 CSR range");
    const int transpose = (mode & MIGNN_CSR_TRANSPOSE) ? 1 : 0;
    mode &= ~MIGNN_CSR_TRANSPOSE;
    MIGNN_REQUIRE(mode == MIGNN_CSR_VERBATIM || mode == MIGNN_CSR_ONE_SELF_LOOP,
                  "csr_build: bad mode %d", mode);
    MIGNN_REQUIRE(row_ptr && col && scratch && (E == 0 || edge_index),
                  "csr_build: null pointer");
    hipStream_t st = as_stream(stream_);
    CsrScratch L;
    int rc = csr_layout(E, N, &L);
    if (rc) return rc;
    if (scratch_bytes < L.total) {
        set_error("csr_build: scratch %zu < required %zu", scratch_bytes, L.total);
        return MIGNN_ERR_SCRATCH;
    }
    char* base = static_cast<char*>(scratch);
    uint32_t* keys_in = reinterpret_cast<uint32_t*>(base + L.off_keys_in);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(base + L.off_keys_out);
    int32_t* vals_in = reinterpret_cast<int32_t*>(base + L.off_vals_in);
    int32_t* vals_out = reinterpret_cast<int32_t*>(base + L.off_vals_out);
    int32_t* row_ptr0 = reinterpret_cast<int32_t*>(base + L.off_rowptr0);
    auto* counters = reinterpret_cast<unsigned long long*>(base + L.off_counters);
    MIGNN_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(unsigned long long), st));
    if (E > 0) {
        hipLaunchKernelGGL(csr_keys_kernel, dim3(grid_for(E, kBlock, 4096)), dim3(kBlock), 0, st,
                           edge_index, E, N, mode, transpose, relabel, keys_in, vals_in,
                           counters);
        if ((rc = launch_status("csr_keys_kernel"))) return rc;
        const unsigned bits = key_bits(N);
        size_t temp = L.temp_bytes;
        hipError_t err = rocprim::radix_sort_pairs(base + L.off_temp, temp, keys_in, keys_out,
                                                   vals_in, vals_out, static_cast<size_t>(E), 0u,
                                                   bits, st);
        if (err != hipSuccess) {
            set_error("rocprim::radix_sort_pairs: %s", hipGetErrorString(err));
            return MIGNN_ERR_HIP;
        }
    }
    hipLaunchKernelGGL(row_bounds_kernel, dim3(grid_for(E + 1, kBlock, 65536)), dim3(kBlock), 0,
                       st, keys_out, E, N, row_ptr0);
    if ((rc = launch_status("row_bounds_kernel"))) return rc;
    hipLaunchKernelGGL(csr_expand_nodes_kernel, dim3(grid_for(N + 1, kBlock, 65536)),
                       dim3(kBlock), 0, st, row_ptr0, vals_out, E, N, mode, counters, row_ptr,
                       col, dinv);
    if ((rc = launch_status("csr_expand_nodes_kernel"))) return rc;
    if (mode == MIGNN_CSR_VERBATIM && E > 0) {
        hipLaunchKernelGGL(copy_i32_kernel, dim3(grid_for(E, kBlock, 65536)), dim3(kBlock), 0,
                           st, vals_out, col, row_ptr0 + N, E, counters, mode);
        if ((rc = launch_status("copy_i32_kernel"))) return rc;
    }
    if (info) {
        hipLaunchKernelGGL(csr_info_kernel, dim3(1), dim3(64), 0, st, counters, row_ptr, E, N,
                           mode, info);
        if ((rc = launch_status("csr_info_kernel"))) return rc;
    }
    return MIGNN_OK;
}

extern "C" int mignn_grid_graph(int nx, int ny, int nz, int z_begin, int z_count,
                                int64_t* edge_index, float* x, void* stream) {
    MIGNN_REQUIRE(nx > 0 && ny > 0 && nz > 0 && z_begin >= 0 && z_count > 0 &&
                      z_begin + z_count <= nz,
                  "grid_graph: bad dims %d %d %d slab [%d,+%d)", nx, ny, nz, z_begin, z_count);
    MIGNN_REQUIRE(edge_index && x, "grid_graph: null pointer");
    const int64_t n = (int64_t)nx * ny * z_count;
    hipLaunchKernelGGL(grid_graph_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0,
                       as_stream(stream), nx, ny, nz, z_begin, z_count, edge_index, x);
    return launch_status("grid_graph_kernel");
}

extern "C" int mignn_bn_fold(const float* weight, const float* bias, const float* mean,
                             const float* var, float eps, int h, float* scale, float* shift,
                             void* stream) {
    MIGNN_REQUIRE(mean && var && scale && shift && h > 0, "bn_fold: bad args");
    hipLaunchKernelGGL(bn_fold_kernel, dim3((h + 255) / 256), dim3(256), 0, as_stream(stream),
                       weight, bias, mean, var, eps, h, scale, shift);
    return launch_status("bn_fold_kernel");
}

extern "C" int mignn_gcn_norm(const int32_t* row_ptr, const int32_t* col, const float* dinv,
                              int64_t rb, int64_t re, float* ew, void* stream) {
    MIGNN_REQUIRE(row_ptr && col && dinv && ew && rb >= 0 && re >= rb, "gcn_norm: bad args");
    if (re == rb) return MIGNN_OK;
    hipLaunchKernelGGL(gcn_norm_kernel, dim3(grid_for(re - rb, kBlock, 65536)), dim3(kBlock), 0,
                       as_stream(stream), row_ptr, col, dinv, rb, re, ew);
    return launch_status("gcn_norm_kernel");
}

extern "C" int mignn_rows_gather(const float* src, int64_t lds, const int32_t* idx, int64_t n,
                                 int h, float* dst, int64_t ldd, void* stream) {
    MIGNN_REQUIRE(h >= 0 && lds >= h && ldd >= h, "rows_gather: bad widths");
    MIGNN_REQUIRE((src && dst && idx) || n == 0, "rows_gather: null pointer");
    if (n == 0 || h == 0) return MIGNN_OK;
    if (h % 4 != 0 || lds % 4 != 0 || ldd % 4 != 0 || !aligned16(src) || !aligned16(dst)) {
        hipLaunchKernelGGL(rows_gather1_kernel, dim3(grid_for(n * h, kBlock, 65536)),
                           dim3(kBlock), 0, as_stream(stream), src, lds, idx, n, h, dst, ldd);
        return launch_status("rows_gather1_kernel");
    }
    hipLaunchKernelGGL(rows_gather_kernel, dim3(grid_for(n * (h / 4), kBlock, 65536)),
                       dim3(kBlock), 0, as_stream(stream), src, lds, idx, n, h / 4, dst, ldd);
    return launch_status("rows_gather_kernel");
}
