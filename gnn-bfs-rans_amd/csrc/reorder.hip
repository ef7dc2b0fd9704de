// Locality order of the mesh nodes (internal layout of the activations; the
// forward's results are unchanged up to fp32 summation order, see
// mignn.h:mignn_locality_order).
//
// Why: the fused GCN layer reads every CSR neighbour row once per layer.  In
// the lexicographic cell order of a blockMesh / structured mesh (and of the
// synthetic hex grid) the +-k neighbours of a 64-row tile sit
// one plane (nx*ny rows, 25.6 MB at 250x200) away -- out of the 4 MB L2 of
// the XCD, so they come from the MALL or from HBM: 2 of the 4 out-of-tile
// rows per node.  Relabelled into 4x4x4-cell blocks (a 64-row tile each),
// grouped into panels of 4x4 block columns swept along z (16 blocks per
// z-level of a panel, consecutive): out-of-tile rows per node drop from 4 to
// 1.5, and with the fused layer's XCD-contiguous tile schedule an XCD walks
// a panel two z-levels per step, so the lateral neighbour blocks are read by
// that XCD in the same step and the z neighbours a step apart -- only the
// panel perimeter reaches beyond its L2 (round 2: fabric reads 11.0 -> 7.1
// GB per 10M-node layer, L2 hit rate 0.32 -> 0.49; the round-1 order of 4x4
// pencils left the y faces a whole pencil row away).
//
// Node features of FlowGNN are the cell centres (reference
// graph_constructor.py:259), so the order is computed from them:
//   K1 bbox      : per-axis min / max (ordered-uint atomics)
//   K2 cell size : per axis, the mean |delta| of the edges that run mainly
//                  along that axis (periodic wrap edges, |delta| > extent/2,
//                  excluded) -- the mesh spacing, also for anisotropic cells
//   K3 keys      : c = round((pos - min) / h) per axis, t = c / 4 (block),
//                  key = ((((ty/4 * NPX + tx/4) * NTZ + tz) * 16 + (ty%4)*4 + tx%4) * 64
//                         + (cz%4)*16 + (cy%4)*4 + cx%4
//                  (NPX panels along x, NTZ blocks along z), coarsened until
//                  the key range fits 32 bits
//   K4 sort      : rocprim::radix_sort_pairs (stable: ties keep input order)
//   K5 inverse   : inv[perm[p]] = p
#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"

namespace mignn {
namespace {

constexpr int kB = 256;

struct OrderStats {
    unsigned int lo[3], hi[3];        // ordered-uint encoded bbox
    double sum[3];                    // sum of |delta| of axis-dominant edges
    unsigned long long cnt[3];
};

__device__ __forceinline__ unsigned int f2ord(float f) {
    const unsigned int u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ void order_init_kernel(OrderStats* st) {
    if (threadIdx.x < 3) {
        st->lo[threadIdx.x] = 0xffffffffu;
        st->hi[threadIdx.x] = 0u;
        st->sum[threadIdx.x] = 0.0;
        st->cnt[threadIdx.x] = 0ull;
    }
}

__global__ __launch_bounds__(kB) void bbox_kernel(const float* __restrict__ pos, int64_t ldp,
                                                  int64_t n, OrderStats* st) {
    unsigned int lo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, hi[3] = {0u, 0u, 0u};
    auto upd = [&](int a, float v) {
        if (v == v) {   // NaN-free
            lo[a] = min(lo[a], f2ord(v));
            hi[a] = max(hi[a], f2ord(v));
        }
    };
    const int64_t stride = (int64_t)gridDim.x * kB;
    if (ldp == 3 && (reinterpret_cast<uintptr_t>(pos) & 15u) == 0) {
        // dense [n, 3]: the 3n floats as 16-B loads (the row-wise form read
        // each row with three 4-B loads at a 12-B stride), axis = index % 3
        const int64_t nf = 3 * n, nq = nf / 4;
        for (int64_t q = blockIdx.x * (int64_t)kB + threadIdx.x; q < nq; q += stride) {
            const float4 v = ld4(pos + 4 * q);
            int a = static_cast<int>((4 * q) % 3);
            const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                // (a is 0, 1 or 2: unrolled selects keep lo / hi in registers)
                const float x = e[k];
                if (a == 0) upd(0, x); else if (a == 1) upd(1, x); else upd(2, x);
                a = a == 2 ? 0 : a + 1;
            }
        }
        for (int64_t f = 4 * nq + blockIdx.x * (int64_t)kB + threadIdx.x; f < nf; f += stride) {
            const int a = static_cast<int>(f % 3);
            if (a == 0) upd(0, pos[f]); else if (a == 1) upd(1, pos[f]); else upd(2, pos[f]);
        }
    } else {
        for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += stride) {
#pragma unroll
            for (int a = 0; a < 3; ++a) upd(a, pos[i * ldp + a]);
        }
    }
    __shared__ unsigned int s_lo[3], s_hi[3];
    if (threadIdx.x < 3) { s_lo[threadIdx.x] = 0xffffffffu; s_hi[threadIdx.x] = 0u; }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int o = 32; o > 0; o >>= 1) {
            lo[a] = min(lo[a], static_cast<unsigned>(__shfl_xor(static_cast<int>(lo[a]), o)));
            hi[a] = max(hi[a], static_cast<unsigned>(__shfl_xor(static_cast<int>(hi[a]), o)));
        }
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            atomicMin(&s_lo[a], lo[a]);
            atomicMax(&s_hi[a], hi[a]);
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) {   // one global atomic per block and value
        atomicMin(&st->lo[threadIdx.x], s_lo[threadIdx.x]);
        atomicMax(&st->hi[threadIdx.x], s_hi[threadIdx.x]);
    }
}

__global__ __launch_bounds__(kB) void spacing_kernel(const float* __restrict__ pos, int64_t ldp,
                                                     int64_t n, const int64_t* __restrict__ ei,
                                                     int64_t E, OrderStats* st) {
    float ext[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) ext[a] = ord2f(st->hi[a]) - ord2f(st->lo[a]);
    double sum[3] = {0.0, 0.0, 0.0};
    unsigned long long cnt[3] = {0ull, 0ull, 0ull};
    const int64_t ns = E < (int64_t(1) << 18) ? E : (int64_t(1) << 18);
    for (int64_t t = blockIdx.x * (int64_t)kB + threadIdx.x; t < ns; t += (int64_t)gridDim.x * kB) {
        const int64_t e = ns == E ? t : (t * E) / ns;   // evenly strided sample
        const int64_t s = ei[e], d = ei[E + e];
        if (s < 0 || s >= n || d < 0 || d >= n || s == d) continue;
        float dl[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) dl[a] = fabsf(pos[s * ldp + a] - pos[d * ldp + a]);
        const int a = (dl[0] >= dl[1] && dl[0] >= dl[2]) ? 0 : (dl[1] >= dl[2] ? 1 : 2);
        if (dl[a] > 0.f && dl[a] <= 0.5f * ext[a]) {
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (b == a) { sum[b] += dl[a]; cnt[b] += 1; }
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int o = 32; o > 0; o >>= 1) {
            sum[a] += __shfl_xor(sum[a], o);
            cnt[a] += __shfl_xor(cnt[a], o);
        }
    }
    __shared__ double s_sum[3];
    __shared__ unsigned long long s_cnt[3];
    if (threadIdx.x < 3) { s_sum[threadIdx.x] = 0.0; s_cnt[threadIdx.x] = 0ull; }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (cnt[a]) {
                atomicAdd(&s_sum[a], sum[a]);
                atomicAdd(&s_cnt[a], cnt[a]);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 3 && s_cnt[threadIdx.x]) {
        atomicAdd(&st->sum[threadIdx.x], s_sum[threadIdx.x]);
        atomicAdd(&st->cnt[threadIdx.x], s_cnt[threadIdx.x]);
    }
}

// key range of the block order (order_keys_kernel) / of the column order
// (order_col_keys_kernel, remainder columns included) for a cell grid
__device__ double block_key_range(const int64_t cells[3]) {
    return static_cast<double>(((cells[1] + 3) / 4 + 3) / 4) *
           static_cast<double>(((cells[0] + 3) / 4 + 3) / 4) *
           static_cast<double>((cells[2] + 3) / 4) * 1024.0;
}
__device__ double col_key_range(const int64_t cells[3]) {
    const double full = static_cast<double>(cells[0] >> 3) * static_cast<double>(cells[1] >> 3);
    const double all = static_cast<double>((cells[0] + 7) >> 3) * static_cast<double>((cells[1] + 7) >> 3);
    return (full + all) * static_cast<double>(cells[2]) * 64.0;
}

// per-axis spacing h (edge mean, else extent / cbrt(n)), cells per axis;
// coarsened until the order's key range fits 32 bits
template <bool COLS = false>
__device__ void order_grid(const OrderStats* st, int64_t n, float lo[3], float inv_h[3],
                           int64_t cells[3]) {
    const double fallback = cbrt(static_cast<double>(n > 0 ? n : 1));
    double ih[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = ord2f(st->lo[a]);
        double ext = static_cast<double>(ord2f(st->hi[a])) - lo[a];
        if (!(ext >= 0.0) || !(ext < 3.0e38)) ext = 0.0;    // all-NaN / infinite coordinates
        double h = st->cnt[a] ? st->sum[a] / static_cast<double>(st->cnt[a]) : ext / fallback;
        if (!(h > 0.0) || !(ext >= 0.0)) h = 1.0;       // degenerate axis / NaN extents
        ih[a] = 1.0 / h;
        cells[a] = static_cast<int64_t>(fmin(ext * ih[a] + 0.5, 1.0e15)) + 1;
    }
    // coarsen until the key range fits 32 bits
    for (int it = 0; it < 8; ++it) {
        const double range = COLS ? col_key_range(cells) : block_key_range(cells);
        if (range < 4294967295.0) break;
        const double f = cbrt(range / 2147483648.0) * 1.01;
        for (int a = 0; a < 3; ++a) {
            ih[a] /= f;
            double ext = static_cast<double>(ord2f(st->hi[a])) - lo[a];
            if (!(ext >= 0.0) || !(ext < 3.0e38)) ext = 0.0;
            cells[a] = static_cast<int64_t>(fmin(ext * ih[a] + 0.5, 1.0e15)) + 1;
        }
    }
    for (int a = 0; a < 3; ++a) inv_h[a] = static_cast<float>(ih[a]);
}

__global__ __launch_bounds__(kB) void order_keys_kernel(const float* __restrict__ pos,
                                                        int64_t ldp, int64_t n,
                                                        const OrderStats* st,
                                                        uint32_t* __restrict__ keys,
                                                        int32_t* __restrict__ ids) {
    __shared__ float s_lo[3], s_ih[3];
    __shared__ int64_t s_cells[3];
    if (threadIdx.x == 0) {
        float lo[3], ih[3];
        int64_t cells[3];
        order_grid(st, n, lo, ih, cells);
        for (int a = 0; a < 3; ++a) { s_lo[a] = lo[a]; s_ih[a] = ih[a]; s_cells[a] = cells[a]; }
    }
    __syncthreads();
    const int64_t npx = ((s_cells[0] + 3) / 4 + 3) / 4;   // panels along x
    const int64_t ntz = (s_cells[2] + 3) / 4;             // blocks along z
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        int64_t c[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = (pos[i * ldp + a] - s_lo[a]) * s_ih[a] + 0.5f;
            int64_t q = v >= 0.f ? static_cast<int64_t>(v) : 0;   // NaN -> 0
            c[a] = q < s_cells[a] ? q : s_cells[a] - 1;
        }
        const int64_t tx = c[0] >> 2, ty = c[1] >> 2, tz = c[2] >> 2;
        const uint64_t blk = ((static_cast<uint64_t>(ty >> 2) * npx + (tx >> 2)) * ntz + tz) * 16 +
                             (ty & 3) * 4 + (tx & 3);
        const uint64_t key = blk * 64 + (c[2] & 3) * 16 + (c[1] & 3) * 4 + (c[0] & 3);
        keys[i] = static_cast<uint32_t>(key);
        ids[i] = static_cast<int32_t>(i);
    }
}

// Column order (mignn_locality_order_cols; the window GCN kernel gcn_win.hip):
// cells grouped into 8 x 8 columns along the third axis, a column's cells in
// (z, y, x) order so that each 64-row tile of a full column is one z-plane and
// its -z / +z neighbours are the previous / next tile.  Full columns
// (bx < cells_x / 8, by < cells_y / 8) first, in row-major (by, bx) order --
// a workgroup walks one column along z while its XCD's workgroups walk the
// next columns of the same y-row (gcn_win.hip's schedule) -- then the
// remainder columns of the ragged x / y edges in the same (column, z, y, x)
// order.  key = (col * nz + cz) * 64 + (cy & 7) * 8 + (cx & 7) (+ the full
// columns' key range for the remainder).  info[0..3] = {1, nz, full
// columns, full columns per y-row}: the plan's schedule parameters.
__global__ __launch_bounds__(kB) void order_col_keys_kernel(const float* __restrict__ pos,
                                                            int64_t ldp, int64_t n,
                                                            const OrderStats* st,
                                                            uint32_t* __restrict__ keys,
                                                            int32_t* __restrict__ ids,
                                                            int32_t* __restrict__ info) {
    __shared__ float s_lo[3], s_ih[3];
    __shared__ int64_t s_cells[3];
    if (threadIdx.x == 0) {
        float lo[3], ih[3];
        int64_t cells[3];
        order_grid<true>(st, n, lo, ih, cells);
        for (int a = 0; a < 3; ++a) { s_lo[a] = lo[a]; s_ih[a] = ih[a]; s_cells[a] = cells[a]; }
        if (blockIdx.x == 0 && info != nullptr) {
            const int64_t fx = cells[0] >> 3, fy = cells[1] >> 3;
            info[0] = 1;
            info[1] = static_cast<int32_t>(cells[2]);
            info[2] = static_cast<int32_t>(fx * fy);
            info[3] = static_cast<int32_t>(fx);
        }
    }
    __syncthreads();
    const int64_t nz = s_cells[2];
    const int64_t fx = s_cells[0] >> 3, fy = s_cells[1] >> 3;
    const int64_t ax = (s_cells[0] + 7) >> 3;            // columns per y-row, remainder included
    const uint64_t full_range = static_cast<uint64_t>(fx * fy) * nz * 64;
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        int64_t c[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = (pos[i * ldp + a] - s_lo[a]) * s_ih[a] + 0.5f;
            int64_t q = v >= 0.f ? static_cast<int64_t>(v) : 0;   // NaN -> 0
            c[a] = q < s_cells[a] ? q : s_cells[a] - 1;
        }
        const int64_t bx = c[0] >> 3, by = c[1] >> 3;
        const uint64_t inner = static_cast<uint64_t>((c[1] & 7) * 8 + (c[0] & 7));
        uint64_t key;
        if (bx < fx && by < fy)
            key = (static_cast<uint64_t>(by * fx + bx) * nz + c[2]) * 64 + inner;
        else
            key = full_range + (static_cast<uint64_t>(by * ax + bx) * nz + c[2]) * 64 + inner;
        keys[i] = static_cast<uint32_t>(key);
        ids[i] = static_cast<int32_t>(i);
    }
}

__global__ void inverse_kernel(const int32_t* __restrict__ perm, int64_t n,
                               int32_t* __restrict__ inv) {
    for (int64_t p = blockIdx.x * (int64_t)kB + threadIdx.x; p < n; p += (int64_t)gridDim.x * kB)
        inv[perm[p]] = static_cast<int32_t>(p);
}

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct OrderScratch {
    size_t keys_in, keys_out, ids, stats, temp, temp_bytes, total;
};

int order_layout(int64_t n, OrderScratch* L) {
    const size_t m = static_cast<size_t>(n > 0 ? n : 1);
    size_t o = 0;
    L->keys_in = o; o = align256(o + m * 4);
    L->keys_out = o; o = align256(o + m * 4);
    L->ids = o; o = align256(o + m * 4);
    L->stats = o; o = align256(o + sizeof(OrderStats));
    L->temp = o;
    size_t temp = 0;
    hipError_t err = rocprim::radix_sort_pairs(nullptr, temp, (uint32_t*)nullptr,
                                               (uint32_t*)nullptr, (int32_t*)nullptr,
                                               (int32_t*)nullptr, m, 0u, 32u);
    if (err != hipSuccess) {
        set_error("rocprim::radix_sort_pairs size query: %s", hipGetErrorString(err));
        return MIGNN_ERR_HIP;
    }
    L->temp_bytes = temp;
    L->total = align256(o + temp);
    return MIGNN_OK;
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_locality_order_scratch_bytes(int64_t n) {
    OrderScratch L;
    return order_layout(n, &L) == MIGNN_OK ? L.total : 0;
}

static int locality_order_impl(const float* pos, int64_t ldp, int64_t n, const int64_t* edge_index,
                               int64_t E, int32_t* perm, int32_t* inv, int32_t* info, bool cols,
                               void* scratch, size_t scratch_bytes, void* stream);

extern "C" int mignn_locality_order(const float* pos, int64_t ldp, int64_t n,
                                    const int64_t* edge_index, int64_t E, int32_t* perm,
                                    int32_t* inv, void* scratch, size_t scratch_bytes,
                                    void* stream) {
    return locality_order_impl(pos, ldp, n, edge_index, E, perm, inv, nullptr, false, scratch,
                               scratch_bytes, stream);
}

extern "C" int mignn_locality_order_cols(const float* pos, int64_t ldp, int64_t n,
                                         const int64_t* edge_index, int64_t E, int32_t* perm,
                                         int32_t* inv, int32_t* info, void* scratch,
                                         size_t scratch_bytes, void* stream) {
    return locality_order_impl(pos, ldp, n, edge_index, E, perm, inv, info, true, scratch,
                               scratch_bytes, stream);
}

static int locality_order_impl(const float* pos, int64_t ldp, int64_t n, const int64_t* edge_index,
                               int64_t E, int32_t* perm, int32_t* inv, int32_t* info, bool cols,
                               void* scratch, size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(n >= 0 && E >= 0 && n < (int64_t(1) << 31), "locality_order: bad sizes");
    MIGNN_REQUIRE(ldp >= 3, "locality_order: pos needs 3 columns (ldp %lld)", (long long)ldp);
    MIGNN_REQUIRE((pos && perm && inv && scratch) || n == 0, "locality_order: null pointer");
    MIGNN_REQUIRE(E == 0 || edge_index, "locality_order: null edge_index");
    if (n == 0) return MIGNN_OK;
    OrderScratch L;
    int rc = order_layout(n, &L);
    if (rc) return rc;
    if (scratch_bytes < L.total) {
        set_error("locality_order: scratch %zu < required %zu", scratch_bytes, L.total);
        return MIGNN_ERR_SCRATCH;
    }
    hipStream_t st = as_stream(stream);
    char* base = static_cast<char*>(scratch);
    auto* keys_in = reinterpret_cast<uint32_t*>(base + L.keys_in);
    auto* keys_out = reinterpret_cast<uint32_t*>(base + L.keys_out);
    auto* ids = reinterpret_cast<int32_t*>(base + L.ids);
    auto* stats = reinterpret_cast<OrderStats*>(base + L.stats);
    hipLaunchKernelGGL(order_init_kernel, dim3(1), dim3(64), 0, st, stats);
    if ((rc = launch_status("order_init_kernel"))) return rc;
    hipLaunchKernelGGL(bbox_kernel, dim3(grid_for(n, kB, 1024)), dim3(kB), 0, st, pos, ldp, n,
                       stats);
    if ((rc = launch_status("bbox_kernel"))) return rc;
    if (E > 0) {
        // the spacing is a mean over edges: a strided sample of <= 2^18 edges
        // (every edge when fewer) is plenty and keeps the gathers off the step
        hipLaunchKernelGGL(spacing_kernel, dim3(grid_for(E < (1 << 18) ? E : (1 << 18), kB, 1024)),
                           dim3(kB), 0, st, pos, ldp, n, edge_index, E, stats);
        if ((rc = launch_status("spacing_kernel"))) return rc;
    }
    if (cols) {
        hipLaunchKernelGGL(order_col_keys_kernel, dim3(grid_for(n, kB, 8192)), dim3(kB), 0, st, pos,
                           ldp, n, stats, keys_in, ids, info);
        if ((rc = launch_status("order_col_keys_kernel"))) return rc;
    } else {
        hipLaunchKernelGGL(order_keys_kernel, dim3(grid_for(n, kB, 8192)), dim3(kB), 0, st, pos,
                           ldp, n, stats, keys_in, ids);
        if ((rc = launch_status("order_keys_kernel"))) return rc;
    }
    size_t temp = L.temp_bytes;
    hipError_t err = rocprim::radix_sort_pairs(base + L.temp, temp, keys_in, keys_out, ids, perm,
                                               static_cast<size_t>(n), 0u, 32u, st);
    if (err != hipSuccess) {
        set_error("rocprim::radix_sort_pairs: %s", hipGetErrorString(err));
        return MIGNN_ERR_HIP;
    }
    hipLaunchKernelGGL(inverse_kernel, dim3(grid_for(n, kB, 8192)), dim3(kB), 0, st, perm, n, inv);
    return launch_status("inverse_kernel");
}
