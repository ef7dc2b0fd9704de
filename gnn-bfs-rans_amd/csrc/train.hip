// Training-mode forward pieces and the backward: what
// train.py:158-196 needs from FlowGNN in model.train() -- batch-statistics
// BatchNorm (gnn_model.py:87, 188), ReLU + dropout (:190-191, output_proj
// :90-100), the gradients of every Linear / GCNConv / BatchNorm, and the
// reference's WeightedMSELoss (normalization.py:136-250).
//
//   gemm_kernel      C = A.B (+R) for arbitrarily strided A, B on the f32
//                    MFMA (v_mfma_f32_16x16x4f32, exact fp32 products): the
//                    data gradient dX = dY.W (W in torch Linear layout, no
//                    transpose copy) and the weight gradient dW = dY^T.X
//                    (reduction over the nodes, split over blockIdx.z into
//                    partial tiles that reduce_splits_kernel sums in a fixed
//                    order -- deterministic, no float atomics).
//   col_reduce       per-column double-precision sums over the node rows
//                    (block partials + an ordered finalize), fused with the
//                    element function of each use: BN batch moments, BN
//                    backward sums (sum g, sum g*xhat, g recomputed from the
//                    saved pre-BN z and the regenerated dropout mask), loss.
//   bn_act_fwd/bwd   BN-apply + ReLU + dropout, and its backward, elementwise.
//   dropout          counter-based: keep(m, c) = hash(seed, m*h + c) >= p*2^32,
//                    so the backward regenerates the mask instead of storing it.
//
// The backward of the GCN aggregation is the aggregation over the reversed
// edges (mignn_csr_build with MIGNN_CSR_TRANSPOSE) with the forward's dinv:
// PyG's gcn_norm weight dinv_j*dinv_i is symmetric in the edge's endpoints.
#include "common.hpp"

namespace mignn {
namespace {

constexpr int GB = 64;   // GEMM block tile (rows and columns of C)
constexpr int GK = 16;   // reduction chunk staged through LDS
constexpr int GPAD = 16; // LDS row padding: lanes (g, r) hit banks 16g + r

// A_KROW: A's k index is unit-stride (data gradients dY.W) -- staged in its
// native [i][k] order (row pad 1: conflict-free-ish stores and MFMA reads);
// otherwise staged [k][i] (row pad 16).
template <bool A_KROW>
__global__ __launch_bounds__(256) void gemm_kernel(
    const float* __restrict__ A, int64_t sai, int64_t sak, const float* __restrict__ B,
    int64_t sbk, int64_t sbj, int64_t M, int64_t N, int64_t K, int64_t kchunk,
    const float* __restrict__ R, int64_t ldr, float* __restrict__ C, int64_t ldc,
    int64_t split_stride) {
    constexpr int AS = A_KROW ? GB * (GK + 1) : GK * (GB + GPAD);
    constexpr int BS = GK * (GB + GPAD);
    // two LDS stages: chunk c+1 is fetched into registers while chunk c
    // feeds the MFMAs, then stored to the other stage -- one barrier per chunk
    __shared__ float As[2][AS];
    __shared__ float Bs[2][BS];   // Bs[k][j]
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    // column tiles fastest: the blocks sharing one A row panel (data
    // gradients, N = 2-4 tiles) run back to back, so the panel is read from
    // HBM once and hit in L2 by its neighbours
    const int64_t ntn = (N + GB - 1) / GB;
    const int64_t i0 = static_cast<int64_t>(blockIdx.x / ntn) * GB;
    const int64_t j0 = static_cast<int64_t>(blockIdx.x % ntn) * GB;
    const int64_t kb = static_cast<int64_t>(blockIdx.z) * kchunk;
    const int64_t ke = min(K, kb + kchunk);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // staging map (consecutive threads along each operand's unit-stride dim)
    int a_off[4], b_off[4];
    float ra[4], rb[4];
    auto fetch = [&](int64_t k0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int e = tid + t * 256;
            int ii, kk;
            if (A_KROW) { kk = e & 15; ii = e >> 4; }
            else { ii = e & 63; kk = e >> 6; }
            a_off[t] = A_KROW ? ii * (GK + 1) + kk : kk * (GB + GPAD) + ii;
            const int64_t gi = i0 + ii, gk = k0 + kk;
            ra[t] = (gi < M && gk < ke) ? A[gi * sai + gk * sak] : 0.f;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int e = tid + t * 256;
            int jj, kk;
            if (sbj == 1) { jj = e & 63; kk = e >> 6; }
            else { kk = e & 15; jj = e >> 4; }
            b_off[t] = kk * (GB + GPAD) + jj;
            const int64_t gj = j0 + jj, gk = k0 + kk;
            rb[t] = (gj < N && gk < ke) ? B[gk * sbk + gj * sbj] : 0.f;
        }
    };
    auto stash = [&](int stage) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            As[stage][a_off[t]] = ra[t];
            Bs[stage][b_off[t]] = rb[t];
        }
    };

    if (kb < ke) {
        fetch(kb);
        stash(0);
    }
    __syncthreads();
    int stage = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += GK) {
        const bool more = k0 + GK < ke;
        if (more) fetch(k0 + GK);   // in flight during the MFMAs below
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ai = wm * 32 + i * 16 + r, ak = u * 4 + g;
                a[i] = A_KROW ? As[stage][ai * (GK + 1) + ak] : As[stage][ak * (GB + GPAD) + ai];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[stage][(u * 4 + g) * (GB + GPAD) + wn * 32 + j * 16 + r];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
        }
        if (more) stash(stage ^ 1);
        __syncthreads();
        stage ^= 1;
    }
    float* Cz = C + static_cast<int64_t>(blockIdx.z) * split_stride;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int64_t col = j0 + wn * 32 + j * 16 + r;
            if (col >= N) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t row = i0 + wm * 32 + i * 16 + g * 4 + q;
                if (row >= M) continue;
                float v = acc[i][j][q];
                if (R != nullptr) v += R[row * ldr + col];
                Cz[row * ldc + col] = v;
            }
        }
}

// C[i, j] = sum_z P[z][i * N + j], z ascending
__global__ void reduce_splits_kernel(const float* __restrict__ P, int nsplit, int64_t M,
                                     int64_t N, float* __restrict__ C, int64_t ldc) {
    const int64_t mn = M * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < mn;
         e += (int64_t)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int z = 0; z < nsplit; ++z) s += P[z * mn + e];
        C[(e / N) * ldc + (e % N)] = s;
    }
}

// ---------------------------------------------------------------- dropout
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;   // splitmix64
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return static_cast<uint32_t>(z >> 32);
}

struct Drop {
    uint64_t seed;
    uint32_t thresh;   // drop if hash < thresh
    float scale;       // 1 / (1 - p) (0 when p == 1)
    __device__ __forceinline__ float keep(int64_t m, int h, int c) const {
        if (thresh == 0u) return scale;
        return drop_hash(seed, static_cast<uint64_t>(m) * h + c) >= thresh ? scale : 0.f;
    }
};

Drop make_drop(float p, uint64_t seed) {
    Drop d;
    d.seed = seed;
    if (p <= 0.f) {
        d.thresh = 0u;
        d.scale = 1.f;
    } else if (p >= 1.f) {
        d.thresh = 0xffffffffu;
        d.scale = 0.f;
    } else {
        const double t = static_cast<double>(p) * 4294967296.0;
        d.thresh = t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
        d.scale = 1.f / (1.f - p);
    }
    return d;
}

// ------------------------------------------------------- column reductions
enum { RED_MOMENTS = 0, RED_BN_BWD = 1, RED_SQDIFF = 2 };
constexpr int RED_CC = 8;          // h <= 64 * RED_CC
constexpr int RED_MAX_BLOCKS = 2048;   // 8 blocks (32 waves) per CU to hide the row loads

struct RedArgs {
    const float* a; int64_t lda;   // MOMENTS: x; BN_BWD: dout; SQDIFF: pred
    const float* b; int64_t ldb;   // BN_BWD: z (pre-BN); SQDIFF: target
    const float* mean; const float* invstd; const float* gamma; const float* beta;
    int relu;
    Drop drop;
};

template <int MODE>
__global__ __launch_bounds__(256) void col_reduce_kernel(RedArgs p, int64_t n, int h,
                                                         double* __restrict__ partial) {
    __shared__ double red[2][4][64 * RED_CC];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double s1[RED_CC], s2[RED_CC];
#pragma unroll
    for (int cc = 0; cc < RED_CC; ++cc) s1[cc] = s2[cc] = 0.0;
    for (int64_t m = blockIdx.x * 4 + wave; m < n; m += (int64_t)gridDim.x * 4) {
#pragma unroll
        for (int cc = 0; cc < RED_CC; ++cc) {
            const int c = lane + 64 * cc;
            if (c >= h) break;
            const float av = p.a[m * p.lda + c];
            if constexpr (MODE == RED_MOMENTS) {
                s1[cc] += av;
                s2[cc] += static_cast<double>(av) * av;
            } else if constexpr (MODE == RED_BN_BWD) {
                const float xh = (p.b[m * p.ldb + c] - p.mean[c]) * p.invstd[c];
                const float yb = p.gamma ? fmaf(p.gamma[c], xh, p.beta[c]) : xh;
                const float gv = (!p.relu || yb > 0.f) ? av * p.drop.keep(m, h, c) : 0.f;
                s1[cc] += gv;
                s2[cc] += static_cast<double>(gv) * xh;
            } else {
                const float d = av - p.b[m * p.ldb + c];
                s1[cc] += static_cast<double>(d) * d;
                s2[cc] += d;
            }
        }
    }
#pragma unroll
    for (int cc = 0; cc < RED_CC; ++cc) {
        red[0][wave][lane + 64 * cc] = s1[cc];
        red[1][wave][lane + 64 * cc] = s2[cc];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < h; c += blockDim.x) {
        double t1 = 0.0, t2 = 0.0;
        for (int w = 0; w < 4; ++w) {
            t1 += red[0][w][c];
            t2 += red[1][w][c];
        }
        partial[(static_cast<int64_t>(blockIdx.x) * 2) * h + c] = t1;
        partial[(static_cast<int64_t>(blockIdx.x) * 2 + 1) * h + c] = t2;
    }
}


// BN batch statistics (torch BatchNorm1d training: biased variance for the
// normalisation, unbiased for running_var, running = (1-m)*running + m*batch)
// one 256-thread block per column: the block's threads take the partials
// k = tid, tid + 256, ... and a fixed-shape LDS tree sums them (deterministic;
// the one-thread-per-column loop over the partials was latency-bound)
__device__ __forceinline__ void block_sum_partials(const double* partial, int nblk, int h, int c,
                                                   double* s1, double* s2) {
    __shared__ double r1[256], r2[256];
    const int tid = threadIdx.x;
    double a = 0.0, b = 0.0;
    for (int k = tid; k < nblk; k += 256) {
        a += partial[(static_cast<int64_t>(k) * 2) * h + c];
        b += partial[(static_cast<int64_t>(k) * 2 + 1) * h + c];
    }
    r1[tid] = a;
    r2[tid] = b;
    __syncthreads();
#pragma unroll
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) {
            r1[tid] += r1[tid + w];
            r2[tid] += r2[tid + w];
        }
        __syncthreads();
    }
    *s1 = r1[0];
    *s2 = r2[0];
}

__global__ __launch_bounds__(256) void bn_stats_finalize_kernel(const double* __restrict__ partial, int nblk, int64_t n,
                                         int h, float eps, float momentum,
                                         float* __restrict__ mean, float* __restrict__ invstd,
                                         float* __restrict__ running_mean,
                                         float* __restrict__ running_var,
                                         int64_t* __restrict__ num_batches) {
    const int c = blockIdx.x;   // one block per column
    double s1, s2;
    block_sum_partials(partial, nblk, h, c, &s1, &s2);
    if (threadIdx.x != 0) return;
    // momentum < 0: BatchNorm1d(momentum=None), the cumulative average with
    // factor 1 / num_batches_tracked after this batch's increment (the
    // counter itself is bumped by bn_count_kernel after this launch, so every
    // block reads the same pre-increment value)
    if (momentum < 0.f)
        momentum = 1.f / static_cast<float>((num_batches != nullptr ? *num_batches : 0) + 1);
    const double mu = s1 / n;
    double var = s2 / n - mu * mu;
    if (var < 0.0) var = 0.0;
    mean[c] = static_cast<float>(mu);
    invstd[c] = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
    if (running_mean != nullptr) {
        running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * static_cast<float>(mu);
        const double unb = n > 1 ? var * n / (n - 1) : var;
        running_var[c] = (1.f - momentum) * running_var[c] + momentum * static_cast<float>(unb);
    }
}

__global__ void bn_count_kernel(int64_t* __restrict__ num_batches) {
    if (threadIdx.x == 0) *num_batches += 1;
}

// out1[c] = float(sum1), out2[c] = float(sum2) (either may be NULL)
__global__ __launch_bounds__(256) void sums_finalize_kernel(
    const double* __restrict__ partial, int nblk, int h, float* __restrict__ out1,
    float* __restrict__ out2) {
    const int c = blockIdx.x;   // one block per column
    double s1, s2;
    block_sum_partials(partial, nblk, h, c, &s1, &s2);
    if (threadIdx.x != 0) return;
    if (out1) out1[c] = static_cast<float>(s1);
    if (out2) out2[c] = static_cast<float>(s2);
}

// ---------------------------------------------------------- elementwise
// y = drop(relu(gamma*(z - mean)*invstd + beta)); gamma == NULL: no BN
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(
    const float* __restrict__ z, int64_t ldz, int64_t n, int h, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int relu, Drop drop, float* __restrict__ y, int64_t ldy) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    if (c >= h) return;
    const float mu = gamma ? mean[c] : 0.f, is = gamma ? invstd[c] : 1.f;
    const float ga = gamma ? gamma[c] : 1.f, be = gamma ? beta[c] : 0.f;
    for (int64_t m = blockIdx.y * 4 + (threadIdx.x >> 6); m < n; m += (int64_t)gridDim.y * 4) {
        float v = relu < 0 ? 1.f : z[m * ldz + c];   // relu < 0: the mask itself
        if (gamma) v = fmaf(ga, (v - mu) * is, be);
        if (relu) v = fmaxf(v, 0.f);
        y[m * ldy + c] = v * drop.keep(m, h, c);
    }
}

// dz = gamma*invstd*(g - sum_g/n - xhat*sum_gxh/n), g = dout*keep*(yb > 0)
// (no BN: dz = g)
__global__ __launch_bounds__(256) void bn_act_bwd_kernel(
    const float* __restrict__ dout, int64_t ldd, const float* __restrict__ z, int64_t ldz,
    int64_t n, int h, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ sum_g, const float* __restrict__ sum_gx, int relu, Drop drop,
    float* __restrict__ dz, int64_t lddz) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    if (c >= h) return;
    const float mu = gamma ? mean[c] : 0.f, is = gamma ? invstd[c] : 1.f;
    const float ga = gamma ? gamma[c] : 1.f, be = gamma ? beta[c] : 0.f;
    const float mg = gamma ? sum_g[c] / static_cast<float>(n) : 0.f;
    const float mgx = gamma ? sum_gx[c] / static_cast<float>(n) : 0.f;
    for (int64_t m = blockIdx.y * 4 + (threadIdx.x >> 6); m < n; m += (int64_t)gridDim.y * 4) {
        const float zv = z[m * ldz + c];
        const float xh = gamma ? (zv - mu) * is : zv;
        const float yb = gamma ? fmaf(ga, xh, be) : zv;
        float gv = dout[m * ldd + c] * drop.keep(m, h, c);
        if (relu && !(yb > 0.f)) gv = 0.f;
        dz[m * lddz + c] = gamma ? ga * is * (gv - mg - xh * mgx) : gv;
    }
}

// loss: s1[c] = sum (pred - tgt)^2, s2[c] = sum (pred - tgt)
struct LossW {
    float w[8];
};

__global__ __launch_bounds__(256) void wmse_finalize_kernel(const double* __restrict__ partial, int nblk, int64_t n,
                                     int ncol, LossW wt, float prw, int fieldwise,
                                     float* __restrict__ loss, double* __restrict__ stats) {
    __shared__ double s_sq[8], s_df[8];
    for (int c = 0; c < 7; ++c) {   // block-parallel, fixed-order column sums
        double a, b;
        block_sum_partials(partial, nblk, ncol, c, &a, &b);
        if (threadIdx.x == 0) {
            s_sq[c] = a;
            s_df[c] = b;
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const double* sq = s_sq;
    const double* df = s_df;
    const double dn = static_cast<double>(n);
    double L;
    if (fieldwise) {
        const double pm = df[3] / dn;   // mean(p_pred) - mean(p_target)
        L = wt.w[0] * ((sq[0] + sq[1] + sq[2]) / (3.0 * dn));
        L += wt.w[3] * (sq[3] / dn + (prw > 0.f ? prw * pm * pm : 0.0));
        L += wt.w[4] * (sq[4] / dn) + wt.w[5] * (sq[5] / dn) + wt.w[6] * (sq[6] / dn);
        stats[0] = pm;
    } else {
        L = 0.0;
        for (int c = 0; c < 7; ++c) L += wt.w[c] * sq[c];
        L /= 7.0 * dn;
        stats[0] = 0.0;
    }
    *loss = static_cast<float>(L);
}

__global__ __launch_bounds__(256) void wmse_bwd_kernel(
    const float* __restrict__ pred, int64_t ldp, const float* __restrict__ tgt, int64_t ldt,
    int64_t n, int ncol, LossW coef, float pref, const double* __restrict__ stats,
    const float* __restrict__ gout, float* __restrict__ dpred, int64_t ldd) {
    const float go = *gout;
    const float pterm = pref * static_cast<float>(stats[0]);
    const int64_t total = n * ncol;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t m = e / ncol;
        const int c = static_cast<int>(e - m * ncol);
        float v = 0.f;
        if (c < 7) {
            const float d = pred[m * ldp + c] - tgt[m * ldt + c];
            v = coef.w[c] * 2.f * d + (c == 3 ? pterm : 0.f);
        }
        dpred[m * ldd + c] = go * v;
    }
}

int red_blocks(int64_t n) {
    int64_t b = (n + 63) / 64;
    if (b < 1) b = 1;
    if (b > RED_MAX_BLOCKS) b = RED_MAX_BLOCKS;
    return static_cast<int>(b);
}

dim3 ew_grid(int64_t n, int h) {
    int64_t gy = (n + 3) / 4;
    if (gy > 4096) gy = 4096;
    if (gy < 1) gy = 1;
    return dim3(static_cast<unsigned>((h + 63) / 64), static_cast<unsigned>(gy));
}

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" size_t mignn_train_scratch_bytes(int64_t n, int h) {
    (void)n;
    return static_cast<size_t>(RED_MAX_BLOCKS) * 2 * (h > 8 ? h : 8) * sizeof(double) + 64;
}

extern "C" int mignn_gemm(const float* a, int64_t sai, int64_t sak, const float* b, int64_t sbk,
                          int64_t sbj, int64_t m, int64_t n, int64_t k, const float* r,
                          int64_t ldr, float* c, int64_t ldc, void* scratch,
                          size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(m >= 0 && n >= 0 && k >= 0, "gemm: negative sizes");
    MIGNN_REQUIRE(c && (k == 0 || (a && b)), "gemm: null operand");
    MIGNN_REQUIRE(ldc >= n, "gemm: ldc %lld < n %lld", (long long)ldc, (long long)n);
    if (m == 0 || n == 0) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    const int64_t tiles = ((m + GB - 1) / GB) * ((n + GB - 1) / GB);
    // split the reduction when the output is small and k long (weight
    // gradients: k = nodes) and the caller gave room for the partial tiles
    int64_t nsplit = 1;
    if (r == nullptr && scratch != nullptr && tiles < 512 && k >= 2048) {
        nsplit = (1024 + tiles - 1) / tiles;
        const int64_t by_k = k / 1024;
        if (nsplit > by_k) nsplit = by_k;
        const int64_t by_mem = static_cast<int64_t>(scratch_bytes / (sizeof(float) * m * n));
        if (nsplit > by_mem) nsplit = by_mem;
        if (nsplit > 1024) nsplit = 1024;
        if (nsplit < 1) nsplit = 1;
    }
    int64_t kchunk = (k + nsplit - 1) / nsplit;
    kchunk = ((kchunk + GK - 1) / GK) * GK;
    if (kchunk < GK) kchunk = GK;
    nsplit = (k + kchunk - 1) / kchunk;
    if (nsplit < 1) nsplit = 1;
    MIGNN_REQUIRE(tiles < (int64_t(1) << 31), "gemm: grid too large");
    dim3 grid(static_cast<unsigned>(tiles), 1, static_cast<unsigned>(nsplit));
    auto kern = (sak == 1) ? gemm_kernel<true> : gemm_kernel<false>;
    if (nsplit == 1) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, a, sai, sak, b, sbk, sbj, m, n,
                           k, k > 0 ? kchunk : GK, r, ldr, c, ldc, (int64_t)0);
        return launch_status("gemm_kernel");
    }
    float* P = static_cast<float*>(scratch);
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, a, sai, sak, b, sbk, sbj, m, n, k,
                       kchunk, (const float*)nullptr, (int64_t)0, P, n, m * n);
    int rc = launch_status("gemm_kernel(split)");
    if (rc) return rc;
    hipLaunchKernelGGL(reduce_splits_kernel, dim3(grid_for(m * n, 256, 4096)), dim3(256), 0, st,
                       P, static_cast<int>(nsplit), m, n, c, ldc);
    return launch_status("reduce_splits_kernel");
}

extern "C" int mignn_col_sums(const float* x, int64_t ldx, int64_t n, int h, float* sums,
                              void* scratch, size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(x && sums && scratch && n >= 0 && h > 0 && h <= 64 * RED_CC,
                  "col_sums: bad arguments (h=%d)", h);
    MIGNN_REQUIRE(scratch_bytes >= mignn_train_scratch_bytes(n, h), "col_sums: scratch too small");
    hipStream_t st = as_stream(stream);
    RedArgs p{};
    p.a = x;
    p.lda = ldx;
    const int nb = red_blocks(n);
    double* part = static_cast<double*>(scratch);
    hipLaunchKernelGGL(col_reduce_kernel<RED_MOMENTS>, dim3(nb), dim3(256), 0, st, p, n, h, part);
    int rc = launch_status("col_reduce_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(sums_finalize_kernel, dim3(h), dim3(256), 0, st, part, nb, h,
                       sums, (float*)nullptr);
    return launch_status("sums_finalize_kernel");
}

extern "C" int mignn_bn_train_stats(const float* z, int64_t ldz, int64_t n, int h, float eps,
                                    float momentum, float* mean, float* invstd,
                                    float* running_mean, float* running_var,
                                    int64_t* num_batches_tracked, void* scratch,
                                    size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(z && mean && invstd && scratch && n > 0 && h > 0 && h <= 64 * RED_CC,
                  "bn_train_stats: bad arguments (n=%lld h=%d)", (long long)n, h);
    MIGNN_REQUIRE(!running_mean == !running_var, "bn_train_stats: running_mean/var pair");
    MIGNN_REQUIRE(scratch_bytes >= mignn_train_scratch_bytes(n, h),
                  "bn_train_stats: scratch too small");
    hipStream_t st = as_stream(stream);
    RedArgs p{};
    p.a = z;
    p.lda = ldz;
    const int nb = red_blocks(n);
    double* part = static_cast<double*>(scratch);
    hipLaunchKernelGGL(col_reduce_kernel<RED_MOMENTS>, dim3(nb), dim3(256), 0, st, p, n, h, part);
    int rc = launch_status("col_reduce_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3(h), dim3(256), 0, st, part,
                       nb, n, h, eps, momentum, mean, invstd, running_mean, running_var,
                       num_batches_tracked);
    rc = launch_status("bn_stats_finalize_kernel");
    if (rc || num_batches_tracked == nullptr) return rc;
    hipLaunchKernelGGL(bn_count_kernel, dim3(1), dim3(64), 0, st, num_batches_tracked);
    return launch_status("bn_count_kernel");
}

extern "C" int mignn_bn_act_forward(const float* z, int64_t ldz, int64_t n, int h,
                                    const float* mean, const float* invstd, const float* gamma,
                                    const float* beta, int relu, float p, uint64_t seed, float* y,
                                    int64_t ldy, void* stream) {
    MIGNN_REQUIRE(z && y && n >= 0 && h > 0, "bn_act_forward: bad arguments");
    MIGNN_REQUIRE(!gamma || (mean && invstd && beta), "bn_act_forward: BN parameters");
    if (n == 0) return MIGNN_OK;
    hipLaunchKernelGGL(bn_act_fwd_kernel, ew_grid(n, h), dim3(256), 0, as_stream(stream), z, ldz,
                       n, h, mean, invstd, gamma, beta, relu, make_drop(p, seed), y, ldy);
    return launch_status("bn_act_fwd_kernel");
}

extern "C" int mignn_bn_act_backward(const float* dout, int64_t ldd, const float* z, int64_t ldz,
                                     int64_t n, int h, const float* mean, const float* invstd,
                                     const float* gamma, const float* beta, int relu, float p,
                                     uint64_t seed, float* dz, int64_t lddz, float* dgamma,
                                     float* dbeta, void* scratch, size_t scratch_bytes,
                                     void* stream) {
    MIGNN_REQUIRE(dout && z && dz && n >= 0 && h > 0 && h <= 64 * RED_CC,
                  "bn_act_backward: bad arguments");
    MIGNN_REQUIRE(!gamma || (mean && invstd && beta && dgamma && dbeta && scratch),
                  "bn_act_backward: BN parameters / gradients / scratch");
    if (n == 0) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    const Drop drop = make_drop(p, seed);
    if (gamma) {
        MIGNN_REQUIRE(scratch_bytes >= mignn_train_scratch_bytes(n, h),
                      "bn_act_backward: scratch too small");
        RedArgs ra{};
        ra.a = dout;
        ra.lda = ldd;
        ra.b = z;
        ra.ldb = ldz;
        ra.mean = mean;
        ra.invstd = invstd;
        ra.gamma = gamma;
        ra.beta = beta;
        ra.relu = relu;
        ra.drop = drop;
        const int nb = red_blocks(n);
        double* part = static_cast<double*>(scratch);
        hipLaunchKernelGGL(col_reduce_kernel<RED_BN_BWD>, dim3(nb), dim3(256), 0, st, ra, n, h,
                           part);
        int rc = launch_status("col_reduce_kernel<BN_BWD>");
        if (rc) return rc;
        hipLaunchKernelGGL(sums_finalize_kernel, dim3(h), dim3(256), 0, st, part,
                           nb, h, dbeta, dgamma);
        if ((rc = launch_status("sums_finalize_kernel"))) return rc;
    }
    hipLaunchKernelGGL(bn_act_bwd_kernel, ew_grid(n, h), dim3(256), 0, st, dout, ldd, z, ldz, n,
                       h, mean, invstd, gamma, beta, dbeta, dgamma, relu, drop, dz, lddz);
    return launch_status("bn_act_bwd_kernel");
}

extern "C" int mignn_wmse_loss(const float* pred, int64_t ldp, const float* tgt, int64_t ldt,
                               int64_t n, int ncol, const float* weights, float prw,
                               int fieldwise, float* loss, double* stats, void* scratch,
                               size_t scratch_bytes, void* stream) {
    MIGNN_REQUIRE(pred && tgt && weights && loss && stats && scratch && n > 0,
                  "wmse_loss: bad arguments");
    MIGNN_REQUIRE(fieldwise ? ncol >= 7 : ncol == 7, "wmse_loss: %d columns", ncol);
    MIGNN_REQUIRE(scratch_bytes >= mignn_train_scratch_bytes(n, ncol), "wmse_loss: scratch");
    hipStream_t st = as_stream(stream);
    RedArgs ra{};
    ra.a = pred;
    ra.lda = ldp;
    ra.b = tgt;
    ra.ldb = ldt;
    const int nb = red_blocks(n);
    double* part = static_cast<double*>(scratch);
    hipLaunchKernelGGL(col_reduce_kernel<RED_SQDIFF>, dim3(nb), dim3(256), 0, st, ra, n, ncol,
                       part);
    int rc = launch_status("col_reduce_kernel<SQDIFF>");
    if (rc) return rc;
    LossW w{};
    for (int c = 0; c < 7; ++c) w.w[c] = weights[c];
    hipLaunchKernelGGL(wmse_finalize_kernel, dim3(1), dim3(256), 0, st, part, nb, n, ncol, w, prw,
                       fieldwise, loss, stats);
    return launch_status("wmse_finalize_kernel");
}

extern "C" int mignn_wmse_loss_backward(const float* pred, int64_t ldp, const float* tgt,
                                        int64_t ldt, int64_t n, int ncol, const float* weights,
                                        float prw, int fieldwise, const double* stats,
                                        const float* grad_loss, float* dpred, int64_t ldd,
                                        void* stream) {
    MIGNN_REQUIRE(pred && tgt && weights && stats && grad_loss && dpred && n > 0,
                  "wmse_loss_backward: bad arguments");
    MIGNN_REQUIRE(fieldwise ? ncol >= 7 : ncol == 7, "wmse_loss_backward: %d columns", ncol);
    LossW coef{};
    const float dn = static_cast<float>(n);
    float pref = 0.f;
    if (fieldwise) {
        for (int c = 0; c < 3; ++c) coef.w[c] = weights[0] / (3.f * dn);
        for (int c = 3; c < 7; ++c) coef.w[c] = weights[c] / dn;
        // d/dp_m of w_p * prw * (mean(p) - mean(t))^2 = w_p * prw * 2 * pm / n
        if (prw > 0.f) pref = weights[3] * prw * 2.f / dn;
    } else {
        for (int c = 0; c < 7; ++c) coef.w[c] = weights[c] / (7.f * dn);
    }
    hipLaunchKernelGGL(wmse_bwd_kernel, dim3(grid_for(n * ncol, 256, 8192)), dim3(256), 0,
                       as_stream(stream), pred, ldp, tgt, ldt, n, ncol, coef, pref, stats,
                       grad_loss, dpred, ldd);
    return launch_status("wmse_bwd_kernel");
}

// standalone mask (tests / debugging): mask[m*h + c] = keep scale of (m, c)
extern "C" int mignn_dropout_mask(int64_t n, int h, float p, uint64_t seed, float* mask,
                                  void* stream) {
    MIGNN_REQUIRE(mask && n >= 0 && h > 0, "dropout_mask: bad arguments");
    if (n == 0) return MIGNN_OK;
    hipLaunchKernelGGL(bn_act_fwd_kernel, ew_grid(n, h), dim3(256), 0, as_stream(stream),
                       (const float*)nullptr, (int64_t)0, n, h, (const float*)nullptr,
                       (const float*)nullptr, (const float*)nullptr, (const float*)nullptr, -1,
                       make_drop(p, seed), mask, (int64_t)h);
    return launch_status("bn_act_fwd_kernel(mask)");
}
