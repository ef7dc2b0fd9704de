// Output side: the reference's FieldNormalizer
// (normalization.py:18-133) and its OpenFOAM ASCII writer
// (inference.py:90-178), native.
//
//   mignn_field_affine   transform  y = (x - mean) / std          (:86-108)
//                        inverse    y = x * std + mean            (:110-133)
//     per column, float64 arithmetic (separately rounded multiply and add,
//     no FMA -- numpy's order), input float32 or float64, output float64 (the
//     NumPy >= 2 promotion of float32 * float64); legacy mode: numpy < 2
//     value-based casting, where a float64 *scalar* std/mean leaves a
//     float32 field float32 (the arithmetic in float32).
//   mignn_field_moments  fit's mean / population std per column (:18-84):
//     float64, two passes (mean, then the mean squared deviation) like
//     numpy.mean / numpy.std; within a few ulp of numpy (numpy sums pairwise).
//   mignn_write_openfoam_field  host-side writer: byte-identical to
//     save_fields_openfoam_format ("%.6e" values, the same header / footer).
#include <cerrno>
#include <cstring>

#include "common.hpp"

// numpy rounds every multiply and add separately: no FMA contraction here
#pragma clang fp contract(off)

namespace mignn {
namespace {

constexpr int kB = 256;

template <typename T>
__global__ void field_affine_kernel(const T* __restrict__ x, int64_t ldx, int64_t n, int ncol,
                                    const double* __restrict__ mean, const double* __restrict__ std_,
                                    int inverse, int legacy_mask, double* __restrict__ y,
                                    float* __restrict__ y32, int64_t ldy) {
    const int64_t total = n * ncol;
    for (int64_t t = blockIdx.x * (int64_t)kB + threadIdx.x; t < total;
         t += (int64_t)gridDim.x * kB) {
        const int64_t r = t / ncol;
        const int c = static_cast<int>(t % ncol);
        const T v = x[r * ldx + c];
        if ((legacy_mask >> c) & 1) {   // float32 arithmetic (numpy < 2, scalar scaler)
            const float m = static_cast<float>(mean[c]), s = static_cast<float>(std_[c]);
            const float f = static_cast<float>(v);
            y32[r * ldy + c] = inverse ? ((f * s) + m) : ((f - m) / s);
        } else {
            const double d = static_cast<double>(v);
            y[r * ldy + c] = inverse ? ((d * std_[c]) + mean[c])
                                     : ((d - mean[c]) / std_[c]);
        }
    }
}

// one block per column: mean, then population variance (two passes)
template <typename T>
__global__ __launch_bounds__(kB) void field_moments_kernel(const T* __restrict__ x, int64_t ldx,
                                                           int64_t n, double* __restrict__ mean,
                                                           double* __restrict__ std_) {
    __shared__ double red[kB];
    const int c = blockIdx.x;
    double s = 0.0;
    for (int64_t r = threadIdx.x; r < n; r += kB) s += static_cast<double>(x[r * ldx + c]);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = kB / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double mu = n > 0 ? red[0] / static_cast<double>(n) : 0.0;
    __syncthreads();
    double q = 0.0;
    for (int64_t r = threadIdx.x; r < n; r += kB) {
        const double d = static_cast<double>(x[r * ldx + c]) - mu;
        q += d * d;
    }
    red[threadIdx.x] = q;
    __syncthreads();
    for (int o = kB / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        mean[c] = mu;
        std_[c] = n > 0 ? sqrt(red[0] / static_cast<double>(n)) : 0.0;
    }
}

const char* kBanner =
    "/*--------------------------------*- C++ -*----------------------------------*\\\n"
    "| =========                 |                                                 |\n"
    "| \\\\      /  F ield         | OpenFOAM: The Open Source CFD Toolbox           |\n"
    "|  \\\\    /   O peration     | Version:  v2406                                 |\n"
    "|   \\\\  /    A nd           | Website:  www.openfoam.com                      |\n"
    "|    \\\\/     M anipulation  |                                                 |\n"
    "\\*---------------------------------------------------------------------------*/\n";

}  // namespace
}  // namespace mignn

using namespace mignn;

extern "C" int mignn_field_affine(const void* x, int x_is_f64, int64_t ldx, int64_t n, int ncol,
                                  const double* mean, const double* std_, int inverse,
                                  int legacy_mask, double* y, float* y32, int64_t ldy,
                                  void* stream) {
    MIGNN_REQUIRE(n >= 0 && ncol >= 1 && ncol <= 30 && ldx >= ncol && ldy >= ncol,
                  "field_affine: bad shape");
    MIGNN_REQUIRE(x && mean && std_, "field_affine: null pointer");
    const int full = (1 << ncol) - 1;
    MIGNN_REQUIRE((legacy_mask & ~full) == 0, "field_affine: legacy mask beyond ncol");
    MIGNN_REQUIRE((legacy_mask == full || y) && (legacy_mask == 0 || y32),
                  "field_affine: missing output buffer");
    MIGNN_REQUIRE(!(legacy_mask && x_is_f64), "field_affine: legacy (float32) mode needs float32 x");
    if (n == 0) return MIGNN_OK;
    hipStream_t st = as_stream(stream);
    const unsigned g = grid_for(n * ncol, kB, 16384);
    if (x_is_f64)
        hipLaunchKernelGGL(field_affine_kernel<double>, dim3(g), dim3(kB), 0, st,
                           static_cast<const double*>(x), ldx, n, ncol, mean, std_, inverse,
                           legacy_mask, y, y32, ldy);
    else
        hipLaunchKernelGGL(field_affine_kernel<float>, dim3(g), dim3(kB), 0, st,
                           static_cast<const float*>(x), ldx, n, ncol, mean, std_, inverse,
                           legacy_mask, y, y32, ldy);
    return launch_status("field_affine_kernel");
}

extern "C" int mignn_field_moments(const void* x, int x_is_f64, int64_t ldx, int64_t n, int ncol,
                                   double* mean, double* std_, void* stream) {
    MIGNN_REQUIRE(n >= 0 && ncol >= 1 && ldx >= ncol && x && mean && std_,
                  "field_moments: bad arguments");
    hipStream_t st = as_stream(stream);
    if (x_is_f64)
        hipLaunchKernelGGL(field_moments_kernel<double>, dim3(ncol), dim3(kB), 0, st,
                           static_cast<const double*>(x), ldx, n, mean, std_);
    else
        hipLaunchKernelGGL(field_moments_kernel<float>, dim3(ncol), dim3(kB), 0, st,
                           static_cast<const float*>(x), ldx, n, mean, std_);
    return launch_status("field_moments_kernel");
}

// Host-side: values are HOST float64 [n, ncomp] (row stride ld); ncomp 1 or 3.
extern "C" int mignn_write_openfoam_field(const char* path, const char* field_class,
                                          const char* object, const char* location,
                                          const char* dimensions, const double* values,
                                          int64_t n, int ncomp, int64_t ld) {
    MIGNN_REQUIRE(path && field_class && object && location && dimensions,
                  "write_openfoam_field: null string");
    MIGNN_REQUIRE(n >= 0 && (ncomp == 1 || ncomp == 3) && ld >= ncomp && (values || n == 0),
                  "write_openfoam_field: bad shape");
    FILE* f = fopen(path, "wb");
    if (!f) {
        set_error("write_openfoam_field: %s: %s", path, strerror(errno));
        return MIGNN_ERR_ARG;
    }
    static thread_local char buf[1 << 20];
    setvbuf(f, buf, _IOFBF, sizeof(buf));
    fputs(kBanner, f);
    fprintf(f, "FoamFile\n{\n    version     2.0;\n    format      ascii;\n");
    fprintf(f, "    class       %s;\n    location    \"%s\";\n    object      %s;\n}\n",
            field_class, location, object);
    fputs("// * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * * //\n\n", f);
    fprintf(f, "dimensions      %s;\n\n", dimensions);
    fprintf(f, "internalField   nonuniform List<%s>\n%lld\n(\n", ncomp == 3 ? "vector" : "scalar",
            static_cast<long long>(n));
    // Python's format(v, ".6e") == C's "%.6e" (both correctly rounded) except
    // for NaN, which Python prints as "nan" whatever its sign
    char t[3][64];
    auto fmt = [](char* o, double v) {
        if (v != v) strcpy(o, "nan");
        else snprintf(o, 64, "%.6e", v);
    };
    for (int64_t i = 0; i < n; ++i) {
        const double* v = values + i * ld;
        if (ncomp == 3) {
            fmt(t[0], v[0]);
            fmt(t[1], v[1]);
            fmt(t[2], v[2]);
            fprintf(f, "(%s %s %s)\n", t[0], t[1], t[2]);
        } else {
            fmt(t[0], v[0]);
            fprintf(f, "%s\n", t[0]);
        }
    }
    fputs(")\n;\n\nboundaryField\n{\n    // Placeholder - boundary conditions not predicted\n}\n\n"
          "// ************************************************************************* //\n", f);
    if (fclose(f) != 0) {
        set_error("write_openfoam_field: closing %s failed", path);
        return MIGNN_ERR_ARG;
    }
    return MIGNN_OK;
}
