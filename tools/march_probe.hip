// march_probe.hip -- what bounds the short-recurrence line marches (gk_sr.hpp)?
// One pass of PCG's first march at 4096^2 (fp64): u = z + beta p, write u,
// dot <A u, u> -- 24 B per unknown compulsory -- in several geometries, beside
// the flat streaming kernel of the same stream mix (read 2, write 1) and the
// production k_sr_march<2, SRK_CG_P> itself.  The Infinity Cache is flushed
// (a 1 GiB memset) before every timed launch, so every byte comes from HBM.
// Prints one line per variant: median us, GB/s, fraction of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I gmres_amd/csrc \
//         tools/march_probe.hip -o tools/march_probe_bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gk_sr.hpp"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

using i64 = long long;

// The march: TPBm threads x VEC points per line window, JT lines per workgroup,
// raw inputs of PD + 1 lines in flight ahead of the line being formed.
// Interior-only simplification: lines past the grid read the zero line.
template <int VEC, int TPBm, int PD>
__global__ __launch_bounds__(TPBm) void k_march(const double *__restrict__ z, const double *__restrict__ p,
                                                double *__restrict__ u_out, const double *__restrict__ zl, int N,
                                                int nlines, int JT, double beta, double *part) {
    __shared__ double sm[TPBm / 64];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPBm * VEC) + (i64)VEC * threadIdx.x;
    const int j0 = blockIdx.y * JT;
    const int j1 = min(j0 + JT, nlines);
    auto src = [&](const double *b, int jj) -> const double * {
        return (jj >= 0 && jj < nlines) ? b + (i64)jj * N : zl;
    };
    auto ld = [&](const double *q, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = *reinterpret_cast<const double2 *>(q);
            v[0] = t.x;
            v[1] = t.y;
        } else if constexpr (VEC == 4) {
            const double2 t0 = *reinterpret_cast<const double2 *>(q);
            const double2 t1 = *reinterpret_cast<const double2 *>(q + 2);
            v[0] = t0.x;
            v[1] = t0.y;
            v[2] = t1.x;
            v[3] = t1.y;
        } else {
            v[0] = q[0];
        }
    };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + VEC : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double um[VEC], uc[VEC], up[VEC];
    double rz[PD + 1][VEC], rp[PD + 1][VEC];
    double ez[2], ep[2];
    {
        double a[VEC], b[VEC];
        ld(src(z, j0 - 1) + i0, a);
        ld(src(p, j0 - 1) + i0, b);
        for (int k = 0; k < VEC; ++k) um[k] = a[k] + beta * b[k];
        ld(src(z, j0) + i0, a);
        ld(src(p, j0) + i0, b);
        for (int k = 0; k < VEC; ++k) uc[k] = a[k] + beta * b[k];
        ld(src(z, j0 + 1) + i0, a);
        ld(src(p, j0 + 1) + i0, b);
        for (int k = 0; k < VEC; ++k) up[k] = a[k] + beta * b[k];
    }
#pragma unroll
    for (int d = 0; d < PD; ++d) {
        ld(src(z, j0 + 2 + d) + i0, rz[d]);
        ld(src(p, j0 + 2 + d) + i0, rp[d]);
    }
    ez[0] = src(z, j0)[ei];
    ep[0] = src(p, j0)[ei];
    double acc = 0.0;
    for (int j = j0; j < j1; ++j) {
        ld(src(z, j + 2 + PD) + i0, rz[PD]);
        ld(src(p, j + 2 + PD) + i0, rp[PD]);
        ez[1] = src(z, j + 1)[ei];
        ep[1] = src(p, j + 1)[ei];
        double left = __shfl_up(uc[VEC - 1], 1, 64);
        double right = __shfl_down(uc[0], 1, 64);
        const double et = ez[0] + beta * ep[0];
        left = lane == 0 ? et : left;
        right = lane == 63 ? et : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + VEC >= N ? 0.0 : right;
        double yv[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double W = k == 0 ? left : uc[k - 1];
            const double E = k == VEC - 1 ? right : uc[k + 1];
            yv[k] = 4.0 * uc[k] - (((W + E) + up[k]) + um[k]);
            acc += yv[k] * uc[k];
        }
        if constexpr (VEC == 1) {
            u_out[(i64)j * N + i0] = uc[0];
        } else {
#pragma unroll
            for (int k = 0; k < VEC; k += 2)
                *reinterpret_cast<double2 *>(u_out + (i64)j * N + i0 + k) = double2{uc[k], uc[k + 1]};
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            um[k] = uc[k];
            uc[k] = up[k];
            up[k] = rz[0][k] + beta * rp[0][k];
        }
#pragma unroll
        for (int d = 0; d < PD; ++d)
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                rz[d][k] = rz[d + 1][k];
                rp[d][k] = rp[d + 1][k];
            }
        ez[0] = ez[1];
        ep[0] = ep[1];
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int w = 0; w < TPBm / 64; ++w) s += sm[w];
        part[blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

// Flat stream of the same mix: out = z + beta p, dot <out, out>; grid-stride double2, U in flight.
template <int U>
__global__ __launch_bounds__(256) void k_flat(const double2 *__restrict__ z, const double2 *__restrict__ p,
                                              double2 *__restrict__ o, i64 n2, double beta, double *part) {
    __shared__ double sm[4];
    double acc = 0.0;
    const i64 stride = (i64)gridDim.x * 256;
    for (i64 e0 = (i64)blockIdx.x * 256 + threadIdx.x; e0 < n2; e0 += U * stride) {
        double2 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = e0 + u * stride;
            a[u] = e < n2 ? z[e] : double2{0, 0};
            b[u] = e < n2 ? p[e] : double2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = e0 + u * stride;
            const double2 r{a[u].x + beta * b[u].x, a[u].y + beta * b[u].y};
            if (e < n2) o[e] = r;
            acc += r.x * r.x + r.y * r.y;
        }
    }
    for (int k = 32; k > 0; k >>= 1) acc += __shfl_xor(acc, k, 64);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}

struct Bufs {
    double *z, *p, *o, *zl, *part, *flush;
    size_t flush_bytes;
    int N;
};

template <class F>
static void timeit(const char *name, const Bufs &b, F launch, double bytes, int reps = 12) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipMemsetAsync(b.flush, r & 0xff, b.flush_bytes, 0));
        CK(hipEventRecord(e0, 0));
        launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipGetLastError());
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3;
    std::printf("%-44s %8.2f us %8.1f GB/s  frac %.3f  (min %.2f)\n", name, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0,
                t[0] * 1e3);
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int VEC, int TPBm, int PD>
static void march(const Bufs &b, int JT) {
    const int N = b.N;
    const int gx = (N + TPBm * VEC - 1) / (TPBm * VEC);
    const int gy = (N + JT - 1) / JT;
    char name[96];
    std::snprintf(name, sizeof name, "march VEC%d TPB%d PD%d JT%d (%d wg)", VEC, TPBm, PD, JT, gx * gy);
    const double bytes = 24.0 * N * (double)N;
    timeit(name, b, [&] {
        k_march<VEC, TPBm, PD><<<dim3(gx, gy), TPBm>>>(b.z, b.p, b.o, b.zl, N, N, JT, 0.5, b.part);
    }, bytes);
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 4096;
    const i64 n = (i64)N * N;
    Bufs b{};
    b.N = N;
    b.flush_bytes = size_t(1) << 30;
    CK(hipMalloc(&b.z, n * 8));
    CK(hipMalloc(&b.p, n * 8));
    CK(hipMalloc(&b.o, n * 8));
    CK(hipMalloc(&b.zl, (size_t)N * 8 + 64));
    CK(hipMalloc(&b.part, 1 << 22));
    CK(hipMalloc(&b.flush, b.flush_bytes));
    CK(hipMemset(b.z, 0, n * 8));
    CK(hipMemset(b.p, 0, n * 8));
    CK(hipMemset(b.o, 0, n * 8));
    CK(hipMemset(b.zl, 0, (size_t)N * 8 + 64));
    const double bytes = 24.0 * (double)n;
    for (int g : {1024, 2048, 4096, 8192}) {
        char name[64];
        std::snprintf(name, sizeof name, "flat read2 write1 U4 (%d wg)", g);
        timeit(name, b, [&] {
            k_flat<4><<<g, 256>>>((const double2 *)b.z, (const double2 *)b.p, (double2 *)b.o, n / 2, 0.5, b.part);
        }, bytes);
    }
    // the production pass (no finaliser), at the production geometry and beside it
    {
        gk::SrDev *sd;
        CK(hipMalloc(&sd, sizeof(gk::SrDev)));
        CK(hipMemset(sd, 0, sizeof(gk::SrDev)));
        for (int JT : {32, 64, 128}) {
            gk::SrArgs a{};
            a.in0 = b.z;
            a.in1 = b.p;
            a.zl = b.zl;
            a.ou = b.o;
            a.part0 = b.part;
            a.sd = sd;
            a.N = N;
            a.nlines = N;
            a.JT = JT;
            a.fin = gk::FIN_NONE;
            const int gx = (N + gk::TPB * 2 - 1) / (gk::TPB * 2), gy = (N + JT - 1) / JT;
            char name[96];
            std::snprintf(name, sizeof name, "k_sr_march<2,CG_P> JT%d (%d wg)", JT, gx * gy);
            timeit(name, b, [&] { gk::k_sr_march<2, gk::SRK_CG_P><<<dim3(gx, gy), gk::TPB>>>(a); }, bytes);
        }
    }
    for (int JT : {16, 32, 64, 128}) {
        march<2, 256, 0>(b, JT);
        march<2, 256, 1>(b, JT);
        march<2, 256, 3>(b, JT);
    }
    for (int JT : {16, 32, 64}) {
        march<1, 256, 0>(b, JT);
        march<1, 256, 2>(b, JT);
        march<2, 128, 0>(b, JT);
        march<2, 128, 2>(b, JT);
        march<2, 64, 0>(b, JT);
        march<2, 64, 2>(b, JT);
        march<4, 128, 0>(b, JT);
        march<4, 128, 1>(b, JT);
        march<2, 512, 0>(b, JT);
        march<2, 512, 2>(b, JT);
    }
    return 0;
}
