// Graph structure on the device: edge validation + destination-major CSR
// (replaces gnn_model.py:125-149 and PyG's self-loop handling / gcn_norm
// degree), the synthetic periodic hex grid, the BatchNorm eval fold and the
// halo row gather.
//
// CSR build (all on `stream`, no host sync): a counting sort by destination,
// made deterministic and stable by a per-row sort on the edge index:
//   K0 csr_count    : per edge, key = dst (valid, kept) or N (dropped: invalid
//                     index, or a self-loop in ONE_SELF_LOOP mode), value = src
//                     (both relabelled when a locality order is given);
//                     deg[key]++ (atomic); kept / invalid counts, one atomic
//                     per block.
//   K1 scan         : row_ptr0 = exclusive prefix sum of deg (rocprim).
//   K2 csr_scatter  : kept edge e -> slot row_ptr0[key] + (atomic fill index),
//                     (edge index, value) stored there; a run of equal keys in
//                     a wave takes consecutive slots with one atomic -- slot
//                     order within a row is otherwise arbitrary here; the
//                     gcn_norm weight of each entry (ew) is written with it...
//   K3 csr_finalize : ...and restored per row by sorting on the edge index
//                     (already sorted: skipped; <= 16 entries: a register
//                     network; longer: in memory): in-row order == edge order,
//                     exactly as a stable sort by key.
// K0 / K2 aggregate runs of equal keys in a wave into one atomic (a mesh edge
// list keeps a node's edges together; same-address atomics serialise).
//                     Final row_ptr / col; ONE_SELF_LOOP mode appends (i, i) to
//                     every row and writes dinv = deg^-1/2; VERBATIM mode with
//                     E > 0 and zero kept edges takes the reference's
//                     all-invalid fallback (one self-loop per node,
//                     gnn_model.py:144-149).
// (Round 1 used a rocprim radix sort of (key, src) pairs for K1-K2: ~1.2 ms of
// the 10M-node / 60M-edge build against ~0.4 ms for K1-K3 here.)
#include <rocprim/device/device_scan.hpp>

#include <cmath>
#include <cstring>

#include "common.hpp"

// gcn_norm weights written by csr_scatter (1) or per row by csr_finalize (0)
#ifndef MIGNN_CSR_EW_SCATTER
#define MIGNN_CSR_EW_SCATTER 0
#endif

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

// Runs of equal keys in consecutive lanes of a wave (mesh edge lists keep a
// node's edges together): one atomic per run instead of per edge -- same-
// address atomics of one wave serialise.  Returns whether this lane heads
// its run; head_lane / run_len of the lane's run.  Every lane of the wave
// must call it (inactive lanes with active = false).
__device__ __forceinline__ bool wave_run(uint32_t key, bool active, int lane, int& head_lane,
                                         int& run_len) {
    const uint32_t prev = static_cast<uint32_t>(__shfl_up(static_cast<int>(key), 1));
    const uint64_t act = __ballot(active);
    const bool prev_active = lane > 0 && ((act >> (lane - 1)) & 1ull);
    const bool head = active && (!prev_active || prev != key);
    const uint64_t heads = __ballot(head);
    const uint64_t below = heads & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
    head_lane = below ? 63 - __clzll(static_cast<long long>(below)) : 0;
    const uint64_t breaks = heads | ~act;               // a run ends before a head or an inactive lane
    const uint64_t above = head_lane == 63 ? 0ull : (breaks & ~((2ull << head_lane) - 1ull));
    run_len = (above ? __ffsll(static_cast<long long>(above)) - 1 : 64) - head_lane;
    return head;
}

// Range mode (RangeIds.inv != nullptr, mignn_csr_build_range): edge ids are
// GLOBAL ids of a node-range shard [lo, hi) of `ng` nodes, mapped on the fly
// to the shard's local ids as mignn_range_relabel does (owned -> inv[id - lo],
// a ghost -> n_own - 1 + ghost_rank[id]); valid = destination owned, source
// in [0, ng).  N is then the local node count (n_own + ghosts).
struct RangeIds {
    const int64_t* inv;
    const int64_t* ghost_rank;
    int64_t lo, hi, ng;
};

__global__ void csr_count_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t N, int mode,
                                 int transpose, const int32_t* __restrict__ relabel, RangeIds rg,
                                 uint32_t* __restrict__ keys, int32_t* __restrict__ vals,
                                 int32_t* __restrict__ deg,
                                 unsigned long long* __restrict__ counters) {
    __shared__ unsigned int s_kept, s_bad;
    if (threadIdx.x == 0) { s_kept = 0; s_bad = 0; }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    unsigned kept = 0, bad = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // kU edges per lane per trip, their loads (edge ends, then relabels)
    // issued together: the per-edge chain load -> relabel -> atomic is
    // latency-bound at one edge in flight per lane
    constexpr int kU = 4;
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < E; base += kU * stride) {
        int64_t s[kU], d[kU];
        bool in[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t e = base + u * stride + threadIdx.x;   // uniform trip count: whole waves
            in[u] = e < E;
            s[u] = -1;
            d[u] = -1;
            if (in[u]) {
                // transposed: rows keyed by the source (backward of the aggregation)
                s[u] = ei[transpose ? E + e : e];
                d[u] = ei[transpose ? e : E + e];
            }
        }
        bool valid[kU];
        int64_t sn[kU], dn[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            sn[u] = s[u];
            dn[u] = d[u];
            if (rg.inv != nullptr) {                // a shard: global ids -> local ids
                valid[u] = in[u] & (s[u] >= 0) & (s[u] < rg.ng) & (d[u] >= rg.lo) & (d[u] < rg.hi);
                if (valid[u]) {
                    const int64_t n_own = rg.hi - rg.lo;
                    sn[u] = (s[u] >= rg.lo && s[u] < rg.hi) ? rg.inv[s[u] - rg.lo]
                                                            : n_own - 1 + rg.ghost_rank[s[u]];
                    dn[u] = rg.inv[d[u] - rg.lo];
                }
                continue;
            }
            valid[u] = in[u] & (s[u] >= 0) & (s[u] < N) & (d[u] >= 0) & (d[u] < N);
            if (relabel != nullptr && valid[u]) {   // node ids in the internal (relabelled) order
                sn[u] = relabel[s[u]];
                dn[u] = relabel[d[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t e = base + u * stride + threadIdx.x;
            bool keep = valid[u];
            if (mode == MIGNN_CSR_ONE_SELF_LOOP && s[u] == d[u]) keep = false;
            const uint32_t key = keep ? static_cast<uint32_t>(dn[u]) : static_cast<uint32_t>(N);
            if (in[u]) {
                keys[e] = key;
                vals[e] = valid[u] ? static_cast<int32_t>(sn[u]) : 0;
            }
            int hl, rl;
            if (wave_run(key, keep, lane, hl, rl)) atomicAdd(&deg[key], rl);
            kept += keep ? 1u : 0u;
            bad += (in[u] && !valid[u]) ? 1u : 0u;
        }
    }
    if (kept) atomicAdd(&s_kept, kept);
    if (bad) atomicAdd(&s_bad, bad);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_kept) atomicAdd(&counters[0], (unsigned long long)s_kept);
        if (s_bad) atomicAdd(&counters[1], (unsigned long long)s_bad);
    }
}

// kept edge e -> its slot in the final col array (row_ptr0[key] + fill index,
// + key in ONE_SELF_LOOP mode: every earlier row gains its self-loop); a run
// of equal keys takes consecutive slots in edge order with one atomic, so a
// row filled by ONE run is in edge order already -- rows filled by several
// runs are flagged for csr_finalize's sort, and only their entries record
// the edge index (slot_eid) the sort keys on.  ew (optional): the entry's
// gcn_norm weight (deg_j + 1)^-1/2 (deg_i + 1)^-1/2 from the kept-edge
// counts, in csr_finalize's former per-row form (bitwise the same); a
// flagged row's weights are rewritten after its sort.
__global__ void csr_scatter_kernel(const uint32_t* __restrict__ keys,
                                   const int32_t* __restrict__ vals, int64_t E, int64_t N,
                                   int one_loop, const int32_t* __restrict__ row_ptr0,
                                   const int32_t* __restrict__ deg,
                                   int32_t* __restrict__ fill, int32_t* __restrict__ slot_eid,
                                   int32_t* __restrict__ col, float* __restrict__ ew,
                                   uint8_t* __restrict__ unsorted) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    constexpr int kU = 4;   // edges per lane per trip, loads issued together (as csr_count)
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < E; base += kU * stride) {
        uint32_t kk[kU];
        int32_t vv[kU], b0[kU], b1[kU], dj[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t e = base + u * stride + threadIdx.x;
            const bool in = e < E;
            kk[u] = in ? keys[e] : static_cast<uint32_t>(N);
            vv[u] = in ? vals[e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {   // the rows' bounds (every kept lane: L1 hits)
            const bool keep = kk[u] < static_cast<uint32_t>(N);
            b0[u] = keep ? row_ptr0[kk[u]] : 0;
            b1[u] = keep ? row_ptr0[kk[u] + 1] : 0;
            dj[u] = (MIGNN_CSR_EW_SCATTER && keep && ew != nullptr) ? deg[vv[u]] : 0;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t e = base + u * stride + threadIdx.x;
            const uint32_t k = kk[u];
            const bool keep = k < static_cast<uint32_t>(N);
            int hl, rl;
            int32_t pos0 = 0;
            if (wave_run(k, keep, lane, hl, rl)) {
                pos0 = b0[u] + atomicAdd(&fill[k], rl);
                if (rl != b1[u] - b0[u]) unsorted[k] = 1;
            }
            pos0 = __shfl(pos0, hl);
            if (keep) {
                const int32_t pos = pos0 + (lane - hl);
                const int32_t off = one_loop ? static_cast<int32_t>(k) : 0;
                if (rl != b1[u] - b0[u]) slot_eid[pos] = static_cast<int32_t>(e);
                col[pos + off] = vv[u];
                if (MIGNN_CSR_EW_SCATTER && ew != nullptr)
                    ew[pos + off] = 1.0f / sqrtf(static_cast<float>(dj[u] + 1)) *
                                    (1.0f / sqrtf(static_cast<float>(b1[u] - b0[u] + 1)));
            }
        }
    }
}

// in-place sort of (eid, val)[b, e) by eid (distinct) -- or, when the ids are
// one contiguous range, val placed by id (eid left as is).  Short rows (the mesh
// case) in registers by an odd-even transposition network over 16 slots;
// longer rows by insertion sort (<= 64) or heap sort in memory.
__device__ void sort_row(int32_t* __restrict__ ke, int32_t* __restrict__ kv, int b, int e) {
    // kv = values at the same positions as ke (a shifted view of col)
    const int n = e - b;
    if (n <= 1) return;
    if (n <= 16) {
        int32_t K[16], V[16];
        int32_t mn = 0x7fffffff, mx = -1;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            K[t] = t < n ? ke[b + t] : 0x7fffffff;
            V[t] = t < n ? kv[b + t] : 0;
            if (t < n) { mn = min(mn, K[t]); mx = max(mx, K[t]); }
        }
        // the row's edges one contiguous range of the edge list (a mesh row
        // split over two waves' runs): entry t belongs at K[t] - mn -- placed
        // directly (its slot_eid is not read again)
        if (mx - mn + 1 == n) {
#pragma unroll
            for (int t = 0; t < 16; ++t)
                if (t < n) kv[b + K[t] - mn] = V[t];
            return;
        }
#pragma unroll
        for (int round = 0; round < 16; ++round) {
#pragma unroll
            for (int t = round & 1; t + 1 < 16; t += 2) {
                const bool sw = K[t] > K[t + 1];
                const int32_t k0 = sw ? K[t + 1] : K[t], k1 = sw ? K[t] : K[t + 1];
                const int32_t v0 = sw ? V[t + 1] : V[t], v1 = sw ? V[t] : V[t + 1];
                K[t] = k0; K[t + 1] = k1; V[t] = v0; V[t + 1] = v1;
            }
        }
#pragma unroll
        for (int t = 0; t < 16; ++t)
            if (t < n) {
                ke[b + t] = K[t];
                kv[b + t] = V[t];
            }
        return;
    }
    if (n <= 64) {
        for (int a = b + 1; a < e; ++a) {
            const int32_t k = ke[a], v = kv[a];
            int c = a - 1;
            while (c >= b && ke[c] > k) {
                ke[c + 1] = ke[c];
                kv[c + 1] = kv[c];
                --c;
            }
            ke[c + 1] = k;
            kv[c + 1] = v;
        }
        return;
    }
    int32_t* const K = ke + b;
    int32_t* const V = kv + b;
    auto sift = [&](int root, int end) {
        while (true) {
            int child = 2 * root + 1;
            if (child >= end) break;
            if (child + 1 < end && K[child + 1] > K[child]) ++child;
            if (K[root] >= K[child]) break;
            const int32_t tk = K[root], tv = V[root];
            K[root] = K[child];
            V[root] = V[child];
            K[child] = tk;
            V[child] = tv;
            root = child;
        }
    };
    for (int r = n / 2 - 1; r >= 0; --r) sift(r, n);
    for (int end = n - 1; end > 0; --end) {
        const int32_t tk = K[0], tv = V[0];
        K[0] = K[end];
        V[0] = V[end];
        K[end] = tk;
        V[end] = tv;
        sift(0, end);
    }
}

// per row: the flagged rows' sort (slot_eid, col), row_ptr, the self-loop
// entry and dinv (ONE_SELF_LOOP); ew (optional) = the PyG gcn_norm weights
// dinv[src] * dinv[i], dinv[j] = (deg_j + 1)^-1/2 from row_ptr0
__global__ void csr_finalize_kernel(const int32_t* __restrict__ row_ptr0,
                                    int32_t* __restrict__ slot_eid,
                                    const uint8_t* __restrict__ unsorted, int64_t E, int64_t N,
                                    int mode, const unsigned long long* __restrict__ counters,
                                    int32_t* __restrict__ row_ptr, int32_t* __restrict__ col,
                                    float* __restrict__ dinv, float* __restrict__ ew) {
    const bool fallback = (mode == MIGNN_CSR_VERBATIM) && (E > 0) && (counters[0] == 0);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= N;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (fallback) {
            row_ptr[i] = static_cast<int32_t>(i);
            if (i < N) col[i] = static_cast<int32_t>(i);
            continue;
        }
        const int32_t b = row_ptr0[i];
        const int32_t off = mode == MIGNN_CSR_ONE_SELF_LOOP ? static_cast<int32_t>(i) : 0;
        row_ptr[i] = b + off;
        if (i == N) continue;
        const int32_t e = row_ptr0[i + 1];
        if (unsorted[i]) sort_row(slot_eid, col + off, b, e);
        if (mode == MIGNN_CSR_ONE_SELF_LOOP) {
            col[e + off] = static_cast<int32_t>(i);
            // PyG gcn_norm: deg.pow(-0.5); deg >= 1 here (self-loop added).
            const float di = 1.0f / sqrtf(static_cast<float>(e - b + 1));
            if (dinv) dinv[i] = di;
            if (ew) {
                if (unsorted[i] || !MIGNN_CSR_EW_SCATTER)   // (csr_scatter's: in the sorted order)
                    for (int32_t t = b + off; t < e + off; ++t) {
                        const int32_t j = col[t];
                        ew[t] = 1.0f / sqrtf(static_cast<float>(row_ptr0[j + 1] - row_ptr0[j] + 1)) * di;
                    }
                ew[e + off] = di * di;
            }
        }
    }
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

struct CsrScratch {
    size_t off_keys, off_vals, off_slot_eid, off_deg, off_fill, off_unsorted, off_rowptr0,
        off_counters, off_temp, temp_bytes, total;
};

int csr_layout(int64_t E, int64_t N, CsrScratch* L) {
    size_t o = 0;
    const size_t e = static_cast<size_t>(E > 0 ? E : 1);
    const size_t n1 = static_cast<size_t>(N + 1);
    L->off_keys = o; o = align_up(o + e * 4);
    L->off_vals = o; o = align_up(o + e * 4);
    L->off_slot_eid = o; o = align_up(o + e * 4);
    L->off_deg = o; o = align_up(o + n1 * 4);       // deg | fill | unsorted: one memset
    L->off_fill = o; o = align_up(o + n1 * 4);
    L->off_unsorted = o; o = align_up(o + n1);
    L->off_rowptr0 = o; o = align_up(o + n1 * 4);
    L->off_counters = o; o = align_up(o + 4 * sizeof(unsigned long long));
    L->off_temp = o;
    size_t temp = 0;
    hipError_t err = rocprim::exclusive_scan(nullptr, temp, (int32_t*)nullptr, (int32_t*)nullptr,
                                             0, n1, rocprim::plus<int32_t>());
    if (err != hipSuccess) {
        set_error("rocprim::exclusive_scan size query: %s", hipGetErrorString(err));
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

// a node-range shard's marks in one pass over its in-edges (mignn.dist.
// RangeLayout): ghost_mark[src] = 1 for a source outside [lo, hi) (the ghost
// ids), boundary_mark[dst - lo] = 1 for an owned destination with such a
// source, bad[0] / bad[1] = 1 for a destination outside [lo, hi) / a source
// outside [0, N) (those edges mark nothing).  Same-value plain stores.
__global__ void range_mark_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t lo,
                                  int64_t hi, int64_t N, int32_t* __restrict__ ghost_mark,
                                  int8_t* __restrict__ boundary_mark, int32_t* __restrict__ bad) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = ei[e], d = ei[E + e];
        const bool dok = d >= lo && d < hi, sok = s >= 0 && s < N;
        if (!dok) bad[0] = 1;
        if (!sok) bad[1] = 1;
        if (dok && sok && (s < lo || s >= hi)) {
            ghost_mark[s] = 1;
            boundary_mark[d - lo] = 1;
        }
    }
}

// a node-range shard's local order (mignn.dist.RangeLayout): interior rows
// first, boundary rows last, each in the base order -- a stable partition of
// base by the boundary flag, from ci = the inclusive prefix count of interior
// rows along base: position p (row b = base[p]) goes to ci[p] - 1 when
// interior, n_int + (p + 1 - ci[p]) - 1 when boundary; perm[dest] = b,
// inv[b] = dest.
__global__ void range_partition_kernel(const int64_t* __restrict__ base,
                                       const uint8_t* __restrict__ boundary,
                                       const int32_t* __restrict__ ci, int64_t n_own, int64_t n_int,
                                       int64_t* __restrict__ perm, int64_t* __restrict__ inv) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n_own;
         p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = base[p];
        const int64_t c = ci[p];
        const int64_t dest = boundary[b] ? n_int + (p + 1 - c) - 1 : c - 1;
        perm[dest] = b;
        inv[b] = dest;
    }
}

// a node-range shard's local edge list (mignn.dist.RangeLayout): source ids
// in [lo, hi) -> the owned row's local position inv[id - lo], others (ghosts)
// -> n_own + the ghost's rank among the ghost ids (ghost_rank[id] - 1: the
// inclusive prefix sum of the ghost marks); destination ids (owned) ->
// inv[id - lo].  out = [2, E] (row 0 sources, row 1 destinations).
__global__ void range_relabel_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t lo,
                                     int64_t hi, const int64_t* __restrict__ inv,
                                     const int64_t* __restrict__ ghost_rank, int64_t n_own,
                                     int64_t* __restrict__ out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = ei[e], d = ei[E + e];
        out[e] = (s >= lo && s < hi) ? inv[s - lo] : n_own - 1 + ghost_rank[s];
        out[E + e] = inv[d - lo];
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

// any width / alignment (coordinates, the head output): a thread per row
// (a 64-bit division per element made this 4x slower)
__global__ void rows_gather1_kernel(const float* __restrict__ src, int64_t lds,
                                    const int32_t* __restrict__ idx, int64_t n, int h,
                                    float* __restrict__ dst, int64_t ldd) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const float* s = src + (int64_t)idx[r] * lds;
        float* d = dst + r * ldd;
        for (int c = 0; c < h; ++c) d[c] = s[c];
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
    return mignn_csr_build_gcn(edge_index, E, N, mode, relabel, row_ptr, col, dinv, nullptr, info,
                               scratch, scratch_bytes, stream_);
}

static int csr_build_impl(const int64_t* edge_index, int64_t E, int64_t N, int mode,
                          const int32_t* relabel, RangeIds rg, int32_t* row_ptr, int32_t* col,
                          float* dinv, float* ew, int64_t* info, void* scratch,
                          size_t scratch_bytes, void* stream_);

extern "C" int mignn_csr_build_gcn(const int64_t* edge_index, int64_t E, int64_t N, int mode,
                                   const int32_t* relabel, int32_t* row_ptr, int32_t* col,
                                   float* dinv, float* ew, int64_t* info, void* scratch,
                                   size_t scratch_bytes, void* stream_) {
    return csr_build_impl(edge_index, E, N, mode, relabel, RangeIds{nullptr, nullptr, 0, 0, 0},
                          row_ptr, col, dinv, ew, info, scratch, scratch_bytes, stream_);
}

extern "C" int mignn_csr_build_range(const int64_t* edge_index, int64_t E, int64_t num_nodes,
                                     int64_t lo, int64_t hi, const int64_t* inv,
                                     const int64_t* ghost_rank, int64_t n_local, int mode,
                                     int32_t* row_ptr, int32_t* col, float* dinv, float* ew,
                                     int64_t* info, void* scratch, size_t scratch_bytes,
                                     void* stream_) {
    MIGNN_REQUIRE(lo >= 0 && hi >= lo && num_nodes >= hi && n_local >= hi - lo,
                  "csr_build_range: bad range [%lld, %lld) of %lld, n_local %lld", (long long)lo,
                  (long long)hi, (long long)num_nodes, (long long)n_local);
    MIGNN_REQUIRE(E == 0 || (inv && ghost_rank), "csr_build_range: null pointer");
    MIGNN_REQUIRE(!(mode & MIGNN_CSR_TRANSPOSE), "csr_build_range: no transposed mode");
    return csr_build_impl(edge_index, E, n_local, mode, nullptr,
                          RangeIds{E ? inv : nullptr, ghost_rank, lo, hi, num_nodes}, row_ptr, col,
                          dinv, ew, info, scratch, scratch_bytes, stream_);
}

static int csr_build_impl(const int64_t* edge_index, int64_t E, int64_t N, int mode,
                          const int32_t* relabel, RangeIds rg, int32_t* row_ptr, int32_t* col,
                          float* dinv, float* ew, int64_t* info, void* scratch,
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
    MIGNN_REQUIRE(!ew || mode == MIGNN_CSR_ONE_SELF_LOOP, "csr_build: ew needs ONE_SELF_LOOP mode");
    hipStream_t st = as_stream(stream_);
    CsrScratch L;
    int rc = csr_layout(E, N, &L);
    if (rc) return rc;
    if (scratch_bytes < L.total) {
        set_error("csr_build: scratch %zu < required %zu", scratch_bytes, L.total);
        return MIGNN_ERR_SCRATCH;
    }
    char* base = static_cast<char*>(scratch);
    auto* keys = reinterpret_cast<uint32_t*>(base + L.off_keys);
    auto* vals = reinterpret_cast<int32_t*>(base + L.off_vals);
    auto* slot_eid = reinterpret_cast<int32_t*>(base + L.off_slot_eid);
    auto* unsorted = reinterpret_cast<uint8_t*>(base + L.off_unsorted);
    auto* deg = reinterpret_cast<int32_t*>(base + L.off_deg);
    auto* fill = reinterpret_cast<int32_t*>(base + L.off_fill);
    auto* row_ptr0 = reinterpret_cast<int32_t*>(base + L.off_rowptr0);
    auto* counters = reinterpret_cast<unsigned long long*>(base + L.off_counters);
    MIGNN_HIP(hipMemsetAsync(deg, 0, L.off_rowptr0 - L.off_deg, st));   // deg, fill, unsorted
    MIGNN_HIP(hipMemsetAsync(counters, 0, 4 * sizeof(unsigned long long), st));
    if (E > 0) {
        hipLaunchKernelGGL(csr_count_kernel, dim3(grid_for(E, kBlock, 8192)), dim3(kBlock), 0, st,
                           edge_index, E, N, mode, transpose, relabel, rg, keys, vals, deg,
                           counters);
        if ((rc = launch_status("csr_count_kernel"))) return rc;
    }
    size_t temp = L.temp_bytes;
    hipError_t err = rocprim::exclusive_scan(base + L.off_temp, temp, deg, row_ptr0, 0,
                                             static_cast<size_t>(N + 1),
                                             rocprim::plus<int32_t>(), st);
    if (err != hipSuccess) {
        set_error("rocprim::exclusive_scan: %s", hipGetErrorString(err));
        return MIGNN_ERR_HIP;
    }
    if (E > 0) {
        hipLaunchKernelGGL(csr_scatter_kernel, dim3(grid_for(E, kBlock, 8192)), dim3(kBlock), 0,
                           st, keys, vals, E, N, mode == MIGNN_CSR_ONE_SELF_LOOP ? 1 : 0, row_ptr0,
                           deg, fill, slot_eid, col, ew, unsorted);
        if ((rc = launch_status("csr_scatter_kernel"))) return rc;
    }
    hipLaunchKernelGGL(csr_finalize_kernel, dim3(grid_for(N + 1, kBlock, 65536)), dim3(kBlock), 0,
                       st, row_ptr0, slot_eid, unsorted, E, N, mode, counters, row_ptr, col, dinv,
                       ew);
    if ((rc = launch_status("csr_finalize_kernel"))) return rc;
    if (info) {
        hipLaunchKernelGGL(csr_info_kernel, dim3(1), dim3(64), 0, st, counters, row_ptr, E, N,
                           mode, info);
        if ((rc = launch_status("csr_info_kernel"))) return rc;
    }
    return MIGNN_OK;
}

extern "C" int mignn_range_mark(const int64_t* edge_index, int64_t E, int64_t lo, int64_t hi,
                                int64_t N, int32_t* ghost_mark, int8_t* boundary_mark,
                                int32_t* bad, void* stream) {
    MIGNN_REQUIRE(E >= 0 && lo >= 0 && hi >= lo && N >= hi, "range_mark: bad sizes");
    if (E == 0) return MIGNN_OK;
    MIGNN_REQUIRE(edge_index && ghost_mark && boundary_mark && bad, "range_mark: null pointer");
    hipLaunchKernelGGL(range_mark_kernel, dim3(grid_for(E, kBlock, 8192)), dim3(kBlock), 0,
                       as_stream(stream), edge_index, E, lo, hi, N, ghost_mark, boundary_mark, bad);
    return launch_status("range_mark_kernel");
}

extern "C" int mignn_range_partition(const int64_t* base, const uint8_t* boundary,
                                     const int32_t* ci, int64_t n_own, int64_t n_int,
                                     int64_t* perm, int64_t* inv, void* stream) {
    MIGNN_REQUIRE(n_own >= 0 && n_int >= 0 && n_int <= n_own, "range_partition: bad sizes");
    if (n_own == 0) return MIGNN_OK;
    MIGNN_REQUIRE(base && boundary && ci && perm && inv, "range_partition: null pointer");
    hipLaunchKernelGGL(range_partition_kernel, dim3(grid_for(n_own, kBlock, 65536)), dim3(kBlock), 0,
                       as_stream(stream), base, boundary, ci, n_own, n_int, perm, inv);
    return launch_status("range_partition_kernel");
}

extern "C" int mignn_range_relabel(const int64_t* edge_index, int64_t E, int64_t lo, int64_t hi,
                                   const int64_t* inv, const int64_t* ghost_rank, int64_t n_own,
                                   int64_t* out, void* stream) {
    MIGNN_REQUIRE(E >= 0 && lo >= 0 && hi >= lo && n_own == hi - lo, "range_relabel: bad sizes");
    if (E == 0) return MIGNN_OK;
    MIGNN_REQUIRE(edge_index && inv && ghost_rank && out, "range_relabel: null pointer");
    hipLaunchKernelGGL(range_relabel_kernel, dim3(grid_for(E, kBlock, 8192)), dim3(kBlock), 0,
                       as_stream(stream), edge_index, E, lo, hi, inv, ghost_rank, n_own, out);
    return launch_status("range_relabel_kernel");
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
        hipLaunchKernelGGL(rows_gather1_kernel, dim3(grid_for(n, kBlock, 65536)),
                           dim3(kBlock), 0, as_stream(stream), src, lds, idx, n, h, dst, ldd);
        return launch_status("rows_gather1_kernel");
    }
    hipLaunchKernelGGL(rows_gather_kernel, dim3(grid_for(n * (h / 4), kBlock, 65536)),
                       dim3(kBlock), 0, as_stream(stream), src, lds, idx, n, h / 4, dst, ldd);
    return launch_status("rows_gather_kernel");
}
