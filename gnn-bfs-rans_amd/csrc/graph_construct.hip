// Mesh -> graph: the reference's GraphConstructor
// (graph_constructor.py:28-56 build_edge_index, :58-90 compute_edge_attributes,
// :92-269 build_graph) on the device, with its exact edge order and rules:
//
//   unfiltered (mode ALL, build_edge_index + :166-172 validation):
//     face f < n_internal: (o, n), (n, o);  face f >= n_internal: (o, o);
//     edges with an index >= n_nodes dropped (order kept)
//   filtered (FIRST_N: cells [0, n); MASK: the mesh's internal_mask) (:136-153):
//     internal faces whose two cells are kept: (o', n'), (n', o') in new ids
//   then (:174-187) nodes that appear in no edge get a self-loop, ascending,
//   appended (no edges at all: every node, :221-226 -- the same rule);
//   edge_attr (:189-219) = (dst - src) / |dst - src|, |dst - src| in float64
//   (sum of squares in x, y, z order; no FMA), rounded to float32; 0 for
//   self-loops; x = cell centres of the kept cells, float64 -> float32.
//
// The reference does this with per-edge Python loops (0.6-1.3 s at 12k cells,
// hours at 10M); here: a per-face count, two rocprim scans and one emit pass.
// Two calls: count (device counts, one host read of E by the caller), emit.
#include <rocprim/device/device_scan.hpp>

#include "common.hpp"

// numpy rounds every multiply and add separately: no FMA contraction here
#pragma clang fp contract(off)

namespace mignn {
namespace {

constexpr int kB = 256;

struct MeshScratch {
    size_t map, inv, cnt, pos, flag, isopos, counts, temp, temp_bytes, total;
};

inline size_t al256(size_t v) { return (v + 255) & ~size_t(255); }

int mesh_layout(int64_t n_faces, int64_t n_cells, MeshScratch* L) {
    const size_t f = static_cast<size_t>(n_faces > 0 ? n_faces : 1);
    const size_t c = static_cast<size_t>(n_cells > 0 ? n_cells : 1);
    size_t o = 0;
    L->map = o; o = al256(o + c * 4);
    L->inv = o; o = al256(o + c * 4);
    L->cnt = o; o = al256(o + (f > c ? f : c) * 4);
    L->pos = o; o = al256(o + f * 4);
    L->flag = o; o = al256(o + c * 4);
    L->isopos = o; o = al256(o + c * 4);
    L->counts = o; o = al256(o + 8 * sizeof(int64_t));
    L->temp = o;
    size_t t1 = 0, t2 = 0;
    const size_t m = f > c ? f : c;
    if (rocprim::exclusive_scan(nullptr, t1, (int32_t*)nullptr, (int32_t*)nullptr, 0, m,
                                rocprim::plus<int32_t>()) != hipSuccess ||
        rocprim::exclusive_scan(nullptr, t2, (int32_t*)nullptr, (int32_t*)nullptr, 0, c,
                                rocprim::plus<int32_t>()) != hipSuccess) {
        set_error("rocprim::exclusive_scan size query failed");
        return MIGNN_ERR_HIP;
    }
    L->temp_bytes = t1 > t2 ? t1 : t2;
    L->total = al256(o + L->temp_bytes);
    return MIGNN_OK;
}

// keep flag per cell (modes FIRST_N / MASK); ALL: identity map
__global__ void mesh_keep_kernel(int64_t n_cells, int mode, const uint8_t* __restrict__ mask,
                                 int64_t n_first, int32_t* __restrict__ keep) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n_cells;
         i += (int64_t)gridDim.x * kB)
        keep[i] = mode == MIGNN_MESH_ALL ? 1 : mode == MIGNN_MESH_FIRST_N ? (i < n_first ? 1 : 0)
                                                                          : (mask[i] ? 1 : 0);
}

// map[old] = new id or -1; inv[new] = old; counts[0] = n_nodes
__global__ void mesh_map_kernel(int64_t n_cells, const int32_t* __restrict__ keep,
                                const int32_t* __restrict__ scan, int32_t* __restrict__ map,
                                int32_t* __restrict__ inv, int64_t* __restrict__ counts) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n_cells;
         i += (int64_t)gridDim.x * kB) {
        const int32_t k = keep[i];
        map[i] = k ? scan[i] : -1;
        if (k) inv[scan[i]] = static_cast<int32_t>(i);
        if (i == n_cells - 1) counts[0] = scan[i] + k;
    }
}

__device__ __forceinline__ int32_t mapped(const int32_t* map, int64_t n_cells, int64_t c) {
    return (c >= 0 && c < n_cells) ? map[c] : -1;
}

// edges contributed by face f (0, 1 or 2)
__device__ __forceinline__ int face_edges(int64_t f, const int64_t* owner, const int64_t* neighbour,
                                          int64_t n_int, int64_t n_cells, int mode,
                                          const int32_t* map, int32_t* a, int32_t* b) {
    const int32_t o = mapped(map, n_cells, owner[f]);
    if (f < n_int) {
        const int32_t n = mapped(map, n_cells, neighbour[f]);
        *a = o;
        *b = n;
        return (o >= 0 && n >= 0) ? 2 : 0;
    }
    *a = o;
    *b = o;
    return (mode == MIGNN_MESH_ALL && o >= 0) ? 1 : 0;
}

__global__ void mesh_face_count_kernel(const int64_t* __restrict__ owner, int64_t n_faces,
                                       const int64_t* __restrict__ neighbour, int64_t n_int,
                                       int64_t n_cells, int mode, const int32_t* __restrict__ map,
                                       int32_t* __restrict__ cnt, int32_t* __restrict__ flag) {
    for (int64_t f = blockIdx.x * (int64_t)kB + threadIdx.x; f < n_faces;
         f += (int64_t)gridDim.x * kB) {
        int32_t a, b;
        const int c = face_edges(f, owner, neighbour, n_int, n_cells, mode, map, &a, &b);
        cnt[f] = c;
        if (c) {          // connected nodes (benign same-value races)
            flag[a] = 1;
            flag[b] = 1;
        }
    }
}

// counts[1] = face edges (after the face scan); flag[i] -> iso[i] = node i
// (< n_nodes = counts[0]) appears in no edge, in place
__global__ void mesh_iso_kernel(int64_t n_cells, int32_t* __restrict__ flag,
                                const int32_t* __restrict__ cnt, const int32_t* __restrict__ pos,
                                int64_t n_faces, int isolated, int64_t* __restrict__ counts) {
    const int64_t n_nodes = counts[0];
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n_cells;
         i += (int64_t)gridDim.x * kB)
        flag[i] = (isolated && i < n_nodes && !flag[i]) ? 1 : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0)
        counts[1] = n_faces > 0 ? (int64_t)pos[n_faces - 1] + cnt[n_faces - 1] : 0;
}

// counts[2] = isolated nodes, counts[3] = total edges
__global__ void mesh_total_kernel(int64_t n_cells, const int32_t* __restrict__ iso,
                                  const int32_t* __restrict__ isopos,
                                  int64_t* __restrict__ counts) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        counts[2] = (int64_t)isopos[n_cells - 1] + iso[n_cells - 1];
        counts[3] = counts[1] + counts[2];
    }
}

__device__ __forceinline__ void edge_attr(const double* cc, int32_t s, int32_t d,
                                          const int32_t* inv, float* out) {
    if (s == d) {
        out[0] = out[1] = out[2] = out[3] = 0.f;
        return;
    }
    const double* ps = cc + 3 * (int64_t)inv[s];
    const double* pd = cc + 3 * (int64_t)inv[d];
    const double dx = (pd[0] - ps[0]), dy = (pd[1] - ps[1]),
                 dz = (pd[2] - ps[2]);
    const double sq = (((dx * dx) + (dy * dy)) + (dz * dz));
    const double dist = sqrt(sq);
    double ux = dx, uy = dy, uz = dz;
    if (dist > 0.0) {
        ux = (dx / dist);
        uy = (dy / dist);
        uz = (dz / dist);
    }
    out[0] = static_cast<float>(ux);
    out[1] = static_cast<float>(uy);
    out[2] = static_cast<float>(uz);
    out[3] = static_cast<float>(dist);
}

__global__ void mesh_emit_faces_kernel(const int64_t* __restrict__ owner, int64_t n_faces,
                                       const int64_t* __restrict__ neighbour, int64_t n_int,
                                       int64_t n_cells, int mode, const int32_t* __restrict__ map,
                                       const int32_t* __restrict__ inv,
                                       const int32_t* __restrict__ pos,
                                       const double* __restrict__ cc, int64_t E,
                                       int64_t* __restrict__ ei, float* __restrict__ ea) {
    for (int64_t f = blockIdx.x * (int64_t)kB + threadIdx.x; f < n_faces;
         f += (int64_t)gridDim.x * kB) {
        int32_t a, b;
        const int c = face_edges(f, owner, neighbour, n_int, n_cells, mode, map, &a, &b);
        if (!c) continue;
        const int64_t p = pos[f];
        ei[p] = a;
        ei[E + p] = b;
        if (ea) edge_attr(cc, a, b, inv, ea + 4 * p);
        if (c == 2) {
            ei[p + 1] = b;
            ei[E + p + 1] = a;
            if (ea) edge_attr(cc, b, a, inv, ea + 4 * (p + 1));
        }
    }
}

__global__ void mesh_emit_iso_kernel(int64_t n_cells, const int32_t* __restrict__ iso,
                                     const int32_t* __restrict__ isopos, const int64_t* counts,
                                     int64_t E, int64_t* __restrict__ ei, float* __restrict__ ea,
                                     const double* __restrict__ feat, int feat_dim,
                                     const int32_t* __restrict__ inv, float* __restrict__ x,
                                     int64_t ldx) {
    const int64_t e_face = counts[1], n_nodes = counts[0];
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n_nodes && i < n_cells;
         i += (int64_t)gridDim.x * kB) {
        if (iso[i]) {
            const int64_t p = e_face + isopos[i];
            ei[p] = i;
            ei[E + p] = i;
            if (ea) {
                float* o = ea + 4 * p;
                o[0] = o[1] = o[2] = o[3] = 0.f;
            }
        }
        if (x) {
            const double* c = feat + feat_dim * (int64_t)inv[i];
            for (int a = 0; a < feat_dim; ++a) x[i * ldx + a] = static_cast<float>(c[a]);
        }
    }
}

// compute_edge_attributes (graph_constructor.py:58-90) of any edge list;
// an index outside [0, n) gives zeros, as build_graph's loop (:196-200)
__global__ void edge_attr_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t n,
                                 const double* __restrict__ cc, float* __restrict__ ea) {
    for (int64_t e = blockIdx.x * (int64_t)kB + threadIdx.x; e < E; e += (int64_t)gridDim.x * kB) {
        const int64_t s = ei[e], d = ei[E + e];
        float* o = ea + 4 * e;
        if (s < 0 || s >= n || d < 0 || d >= n || s == d) {
            o[0] = o[1] = o[2] = o[3] = 0.f;
            continue;
        }
        const double* ps = cc + 3 * s;
        const double* pd = cc + 3 * d;
        const double dx = (pd[0] - ps[0]), dy = (pd[1] - ps[1]),
                     dz = (pd[2] - ps[2]);
        const double dist = sqrt(
            (((dx * dx) + (dy * dy)) + (dz * dz)));
        const double r = dist > 0.0 ? dist : 1.0;
        o[0] = static_cast<float>(dist > 0.0 ? (dx / r) : dx);
        o[1] = static_cast<float>(dist > 0.0 ? (dy / r) : dy);
        o[2] = static_cast<float>(dist > 0.0 ? (dz / r) : dz);
        o[3] = static_cast<float>(dist);
    }
}

// get_boundary_mask (graph_constructor.py:276-296): owners of faces
// [start, start + nfaces) that exist
__global__ void boundary_mask_kernel(const int64_t* __restrict__ owner, int64_t n_faces,
                                     int64_t start, int64_t nfaces, int64_t n_cells,
                                     uint8_t* __restrict__ mask) {
    for (int64_t t = blockIdx.x * (int64_t)kB + threadIdx.x; t < nfaces;
         t += (int64_t)gridDim.x * kB) {
        const int64_t f = start + t;
        if (f >= 0 && f < n_faces) {
            const int64_t c = owner[f];
            if (c >= 0 && c < n_cells) mask[c] = 1;
        }
    }
}

struct MeshPtrs {
    int32_t *map, *inv, *cnt, *pos, *flag, *isopos;
    int64_t* counts;
    void* temp;
};

MeshPtrs mesh_ptrs(void* scratch, const MeshScratch& L) {
    char* b = static_cast<char*>(scratch);
    return MeshPtrs{reinterpret_cast<int32_t*>(b + L.map), reinterpret_cast<int32_t*>(b + L.inv),
                    reinterpret_cast<int32_t*>(b + L.cnt), reinterpret_cast<int32_t*>(b + L.pos),
                    reinterpret_cast<int32_t*>(b + L.flag), reinterpret_cast<int32_t*>(b + L.isopos),
                    reinterpret_cast<int64_t*>(b + L.counts), b + L.temp};
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_mesh_graph_scratch_bytes(int64_t n_faces, int64_t n_cells) {
    MeshScratch L;
    return mesh_layout(n_faces, n_cells, &L) == MIGNN_OK ? L.total : 0;
}

extern "C" int mignn_mesh_graph_count(const int64_t* owner, int64_t n_faces,
                                      const int64_t* neighbour, int64_t n_internal_faces,
                                      int64_t n_cells, int mode, const uint8_t* mask,
                                      int64_t n_first, int isolated, int64_t* counts,
                                      void* scratch, size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(n_faces >= 0 && n_internal_faces >= 0 && n_internal_faces <= n_faces &&
                      n_cells >= 0 && n_cells < (int64_t(1) << 31) &&
                      n_faces < (int64_t(1) << 30),
                  "mesh_graph: bad sizes");
    MIGNN_REQUIRE(mode == MIGNN_MESH_ALL || mode == MIGNN_MESH_FIRST_N || mode == MIGNN_MESH_MASK,
                  "mesh_graph: bad mode %d", mode);
    MIGNN_REQUIRE(mode != MIGNN_MESH_MASK || mask, "mesh_graph: MASK mode needs a mask");
    MIGNN_REQUIRE(mode != MIGNN_MESH_FIRST_N || (n_first >= 0 && n_first <= n_cells),
                  "mesh_graph: n_first %lld outside [0, %lld]", (long long)n_first,
                  (long long)n_cells);
    MIGNN_REQUIRE(scratch && counts && (n_faces == 0 || owner) &&
                      (n_internal_faces == 0 || neighbour),
                  "mesh_graph: null pointer");
    MeshScratch L;
    int rc = mesh_layout(n_faces, n_cells, &L);
    if (rc) return rc;
    if (scratch_bytes < L.total) {
        set_error("mesh_graph: scratch %zu < required %zu", scratch_bytes, L.total);
        return MIGNN_ERR_SCRATCH;
    }
    hipStream_t st = as_stream(stream);
    MeshPtrs P = mesh_ptrs(scratch, L);
    MIGNN_HIP(hipMemsetAsync(P.counts, 0, 8 * sizeof(int64_t), st));
    if (n_cells == 0) return MIGNN_OK;
    const unsigned gc = grid_for(n_cells, kB, 4096), gf = grid_for(n_faces, kB, 4096);
    // node map: keep flags -> exclusive scan -> map / inv / n_nodes
    hipLaunchKernelGGL(mesh_keep_kernel, dim3(gc), dim3(kB), 0, st, n_cells, mode, mask, n_first,
                       P.cnt);
    if ((rc = launch_status("mesh_keep_kernel"))) return rc;
    size_t tb = L.temp_bytes;
    if (rocprim::exclusive_scan(P.temp, tb, P.cnt, P.pos, 0, static_cast<size_t>(n_cells),
                                rocprim::plus<int32_t>(), st) != hipSuccess) {
        set_error("rocprim::exclusive_scan (nodes) failed");
        return MIGNN_ERR_HIP;
    }
    hipLaunchKernelGGL(mesh_map_kernel, dim3(gc), dim3(kB), 0, st, n_cells, P.cnt, P.pos, P.map,
                       P.inv, P.counts);
    if ((rc = launch_status("mesh_map_kernel"))) return rc;
    // face edge counts + connected flags; node count known only on the device:
    // flags cover n_cells >= n_nodes entries
    MIGNN_HIP(hipMemsetAsync(P.flag, 0, static_cast<size_t>(n_cells) * 4, st));
    if (n_faces > 0) {
        hipLaunchKernelGGL(mesh_face_count_kernel, dim3(gf), dim3(kB), 0, st, owner, n_faces,
                           neighbour, n_internal_faces, n_cells, mode, P.map, P.cnt, P.flag);
        if ((rc = launch_status("mesh_face_count_kernel"))) return rc;
        tb = L.temp_bytes;
        if (rocprim::exclusive_scan(P.temp, tb, P.cnt, P.pos, 0, static_cast<size_t>(n_faces),
                                    rocprim::plus<int32_t>(), st) != hipSuccess) {
            set_error("rocprim::exclusive_scan (faces) failed");
            return MIGNN_ERR_HIP;
        }
    }
    hipLaunchKernelGGL(mesh_iso_kernel, dim3(gc), dim3(kB), 0, st, n_cells, P.flag, P.cnt, P.pos,
                       n_faces, isolated, P.counts);
    if ((rc = launch_status("mesh_iso_kernel"))) return rc;
    tb = L.temp_bytes;
    if (rocprim::exclusive_scan(P.temp, tb, P.flag, P.isopos, 0, static_cast<size_t>(n_cells),
                                rocprim::plus<int32_t>(), st) != hipSuccess) {
        set_error("rocprim::exclusive_scan (isolated) failed");
        return MIGNN_ERR_HIP;
    }
    hipLaunchKernelGGL(mesh_total_kernel, dim3(1), dim3(64), 0, st, n_cells, P.flag, P.isopos,
                       P.counts);
    if ((rc = launch_status("mesh_total_kernel"))) return rc;
    return hipMemcpyAsync(counts, P.counts, 4 * sizeof(int64_t), hipMemcpyDeviceToDevice, st) ==
                   hipSuccess
               ? MIGNN_OK
               : MIGNN_ERR_HIP;
}

extern "C" int mignn_mesh_graph_emit(const int64_t* owner, int64_t n_faces,
                                     const int64_t* neighbour, int64_t n_internal_faces,
                                     int64_t n_cells, int mode, const double* cell_centers,
                                     const double* features, int feat_dim, int64_t num_edges,
                                     int64_t* edge_index, float* edge_attr, float* x, int64_t ldx,
                                     void* scratch, size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(num_edges >= 0 && (num_edges == 0 || edge_index), "mesh_graph_emit: outputs");
    MIGNN_REQUIRE(cell_centers || n_cells == 0, "mesh_graph_emit: null cell_centers");
    MIGNN_REQUIRE(!x || (features && feat_dim >= 1 && ldx >= feat_dim),
                  "mesh_graph_emit: x needs features with feat_dim <= ldx");
    MeshScratch L;
    int rc = mesh_layout(n_faces, n_cells, &L);
    if (rc) return rc;
    if (scratch_bytes < L.total) {
        set_error("mesh_graph_emit: scratch %zu < required %zu", scratch_bytes, L.total);
        return MIGNN_ERR_SCRATCH;
    }
    if (n_cells == 0) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    MeshPtrs P = mesh_ptrs(scratch, L);
    if (n_faces > 0 && num_edges > 0) {
        hipLaunchKernelGGL(mesh_emit_faces_kernel, dim3(grid_for(n_faces, kB, 4096)), dim3(kB), 0,
                           st, owner, n_faces, neighbour, n_internal_faces, n_cells, mode, P.map,
                           P.inv, P.pos, cell_centers, num_edges, edge_index, edge_attr);
        if ((rc = launch_status("mesh_emit_faces_kernel"))) return rc;
    }
    hipLaunchKernelGGL(mesh_emit_iso_kernel, dim3(grid_for(n_cells, kB, 4096)), dim3(kB), 0, st,
                       n_cells, P.flag, P.isopos, P.counts, num_edges, edge_index, edge_attr,
                       features, feat_dim, P.inv, x, ldx);
    return launch_status("mesh_emit_iso_kernel");
}

extern "C" int mignn_edge_attributes(const int64_t* edge_index, int64_t num_edges, int64_t n,
                                     const double* cell_centers, float* edge_attr, void* stream) {
    MIGNN_REQUIRE(num_edges >= 0 && n >= 0, "edge_attributes: bad sizes");
    if (num_edges == 0) return MIGNN_OK;
    MIGNN_REQUIRE(edge_index && edge_attr && (cell_centers || n == 0),
                  "edge_attributes: null pointer");
    hipLaunchKernelGGL(edge_attr_kernel, dim3(grid_for(num_edges, kB, 4096)), dim3(kB), 0,
                       as_stream(stream), edge_index, num_edges, n, cell_centers, edge_attr);
    return launch_status("edge_attr_kernel");
}

extern "C" int mignn_boundary_mask(const int64_t* owner, int64_t n_faces, int64_t start_face,
                                   int64_t n_boundary_faces, int64_t n_cells, uint8_t* mask,
                                   void* stream) {
    MIGNN_REQUIRE(n_faces >= 0 && n_boundary_faces >= 0 && n_cells >= 0 && mask &&
                      (owner || n_faces == 0),
                  "boundary_mask: bad arguments");
    hipStream_t st = as_stream(stream);
    MIGNN_HIP(hipMemsetAsync(mask, 0, static_cast<size_t>(n_cells), st));
    if (n_boundary_faces == 0) return MIGNN_OK;
    hipLaunchKernelGGL(boundary_mask_kernel, dim3(grid_for(n_boundary_faces, kB, 4096)), dim3(kB),
                       0, st, owner, n_faces, start_face, n_boundary_faces, n_cells, mask);
    return launch_status("boundary_mask_kernel");
}
