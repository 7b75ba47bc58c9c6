// march_probe.hip -- what bounds the short-recurrence line marches (gk_sr.hpp)?
// One pass of PCG's first march at 4096^2 (fp64): u = z + beta p, write u,
// dot <A u, u> -- 24 B per unknown compulsory -- in several geometries, beside
// the flat streaming kernel of the same stream mix (read 2, write 1) and the
// production k_sr_march<2, SRK_CG_P> itself.  The caches are flushed
// (a 1 GiB read) before every timed launch, so every byte comes from HBM; the
// pass chains run back to back (the Krylov pattern: each pass reads what the
// previous one wrote) in the same or alternating march direction.
// Prints one line per variant: median us, GB/s, fraction of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I gmres_amd/csrc \
//         tools/march_probe.hip -o tools/march_probe_bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <utility>
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
template <int VEC, int TPBm, int PD, bool DN = false>
__global__ __launch_bounds__(TPBm) void k_march(const double *__restrict__ z, const double *__restrict__ p,
                                                double *__restrict__ u_out, const double *__restrict__ zl, int N,
                                                int nlines, int JT, double beta, double *part) {
    __shared__ double sm[TPBm / 64];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPBm * VEC) + (i64)VEC * threadIdx.x;
    const int jb0 = blockIdx.y * JT;
    const int jb1 = min(jb0 + JT, nlines);
    // DN: march from the block's last line down (dd = -1); "p" = the line ahead
    const int dd = DN ? -1 : 1;
    const int j0 = DN ? jb1 - 1 : jb0;
    auto src = [&](const double *b, int jj) -> const double * {
        return (jj >= 0 && jj < nlines) ? b + (i64)jj * N : zl;  // (interior probe: no halo slabs)
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
        ld(src(z, j0 - dd) + i0, a);
        ld(src(p, j0 - dd) + i0, b);
        for (int k = 0; k < VEC; ++k) um[k] = a[k] + beta * b[k];
        ld(src(z, j0) + i0, a);
        ld(src(p, j0) + i0, b);
        for (int k = 0; k < VEC; ++k) uc[k] = a[k] + beta * b[k];
        ld(src(z, j0 + dd) + i0, a);
        ld(src(p, j0 + dd) + i0, b);
        for (int k = 0; k < VEC; ++k) up[k] = a[k] + beta * b[k];
    }
#pragma unroll
    for (int d = 0; d < PD; ++d) {
        ld(src(z, j0 + (2 + d) * dd) + i0, rz[d]);
        ld(src(p, j0 + (2 + d) * dd) + i0, rp[d]);
    }
    ez[0] = src(z, j0)[ei];
    ep[0] = src(p, j0)[ei];
    double acc = 0.0;
    for (int s = 0; s < jb1 - jb0; ++s) {
        const int j = j0 + s * dd;
        ld(src(z, j + (2 + PD) * dd) + i0, rz[PD]);
        ld(src(p, j + (2 + PD) * dd) + i0, rp[PD]);
        ez[1] = src(z, j + dd)[ei];
        ep[1] = src(p, j + dd)[ei];
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

// Ring pipeline without register moves: the loop is unrolled by R (the ring
// depth), so ring slot S = step % R is a compile-time index and a register that
// a load is still filling is never copied (a copy makes the wave wait for the
// load).  Slot S holds, at step s (line j): the raw operand inputs of line
// j + 2, and the edge inputs of line j; after use each is refilled R lines ahead.
template <int S>
using ic = std::integral_constant<int, S>;

template <int VEC, int TPBm, int R, bool DN = false>
__global__ __launch_bounds__(TPBm) void k_march2(const double *__restrict__ z, const double *__restrict__ p,
                                                 double *__restrict__ u_out, const double *__restrict__ zl, int N,
                                                 int nlines, int JT, double beta, double *part) {
    __shared__ double sm[TPBm / 64];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPBm * VEC) + (i64)VEC * threadIdx.x;
    const int jb0 = blockIdx.y * JT;
    const int jb1 = min(jb0 + JT, nlines);
    const int dd = DN ? -1 : 1;
    const int j0 = DN ? jb1 - 1 : jb0;
    const int cnt = jb1 - jb0;
    auto src = [&](const double *b, int jj) -> const double * {
        return (jj >= 0 && jj < nlines) ? b + (i64)jj * N : zl;
    };
    auto ld = [&](const double *q, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = *reinterpret_cast<const double2 *>(q);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = q[0];
        }
    };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + VEC : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double um[VEC], uc[VEC], up[VEC];
    double rz[R][VEC], rp[R][VEC], ez[R], ep[R];
    {
        double a[VEC], b[VEC];
        ld(src(z, j0 - dd) + i0, a);
        ld(src(p, j0 - dd) + i0, b);
        for (int k = 0; k < VEC; ++k) um[k] = a[k] + beta * b[k];
        ld(src(z, j0) + i0, a);
        ld(src(p, j0) + i0, b);
        for (int k = 0; k < VEC; ++k) uc[k] = a[k] + beta * b[k];
        ld(src(z, j0 + dd) + i0, a);
        ld(src(p, j0 + dd) + i0, b);
        for (int k = 0; k < VEC; ++k) up[k] = a[k] + beta * b[k];
    }
#pragma unroll
    for (int d = 0; d < R; ++d) {
        ld(src(z, j0 + (2 + d) * dd) + i0, rz[d]);
        ld(src(p, j0 + (2 + d) * dd) + i0, rp[d]);
        ez[d] = src(z, j0 + d * dd)[ei];
        ep[d] = src(p, j0 + d * dd)[ei];
    }
    double acc = 0.0;
    auto step = [&](int s, auto sc) {
        constexpr int S = decltype(sc)::value;
        const int j = j0 + s * dd;
        double left = __shfl_up(uc[VEC - 1], 1, 64);
        double right = __shfl_down(uc[0], 1, 64);
        const double et = ez[S] + beta * ep[S];
        left = lane == 0 ? et : left;
        right = lane == 63 ? et : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + VEC >= N ? 0.0 : right;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double W = k == 0 ? left : uc[k - 1];
            const double E = k == VEC - 1 ? right : uc[k + 1];
            const double yv = 4.0 * uc[k] - (((W + E) + up[k]) + um[k]);
            acc += yv * uc[k];
        }
        if constexpr (VEC == 1) {
            u_out[(i64)j * N + i0] = uc[0];
        } else {
            *reinterpret_cast<double2 *>(u_out + (i64)j * N + i0) = double2{uc[0], uc[1]};
        }
        const int jr = j + R * dd;  // refill: edges of line j + R, raw of line j + 2 + R
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            um[k] = uc[k];
            uc[k] = up[k];
            up[k] = rz[S][k] + beta * rp[S][k];
        }
        // the slot's old values are dead from here: keep the refill loads below
        // this point so they can land in the same registers (no copy, no wait)
        __builtin_amdgcn_sched_barrier(0);
        ez[S] = src(z, jr)[ei];
        ep[S] = src(p, jr)[ei];
        ld(src(z, jr + 2 * dd) + i0, rz[S]);
        ld(src(p, jr + 2 * dd) + i0, rp[S]);
    };
    int s = 0;
    for (; s + R <= cnt; s += R) {
        step(s, ic<0>{});
        if constexpr (R > 1) step(s + 1, ic<1>{});
        if constexpr (R > 2) step(s + 2, ic<2>{});
        if constexpr (R > 3) step(s + 3, ic<3>{});
    }
    if (s < cnt) step(s, ic<0>{});
    if constexpr (R > 1) if (s + 1 < cnt) step(s + 1, ic<1 % R>{});
    if constexpr (R > 2) if (s + 2 < cnt) step(s + 2, ic<2 % R>{});
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < TPBm / 64; ++w) t += sm[w];
        part[blockIdx.y * gridDim.x + blockIdx.x] = t;
    }
}

// Fully unrolled march (compile-time JTC lines per workgroup): no loop back-edge,
// so no loop-carried register copies; ring slot S = s % R (R lines of loads in flight).
template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F &&f, std::integer_sequence<int, I...>) {
    (f(ic<I>{}), ...);
}

template <int VEC, int TPBm, int R, int JTC>
__global__ __launch_bounds__(TPBm) void k_march3(const double *__restrict__ z, const double *__restrict__ p,
                                                 double *__restrict__ u_out, const double *__restrict__ zl, int N,
                                                 int nlines, double beta, double *part) {
    __shared__ double sm[TPBm / 64];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPBm * VEC) + (i64)VEC * threadIdx.x;
    const int j0 = blockIdx.y * JTC;
    // line j0 + rel of input b: rel is a compile-time step offset; only the
    // lines just outside the block (rel = -1, rel = JTC) can be a boundary
    const double *zlo = j0 > 0 ? z + (i64)(j0 - 1) * N : zl, *plo = j0 > 0 ? p + (i64)(j0 - 1) * N : zl;
    const double *zhi = j0 + JTC < nlines ? z + (i64)(j0 + JTC) * N : zl;
    const double *phi = j0 + JTC < nlines ? p + (i64)(j0 + JTC) * N : zl;
    const double *zb = z + (i64)j0 * N, *pb = p + (i64)j0 * N;
    auto line = [&](auto rc, bool second) -> const double * {
        constexpr int rel = decltype(rc)::value;
        if constexpr (rel < 0) return second ? plo : zlo;
        else if constexpr (rel >= JTC) return second ? phi : zhi;
        else return (second ? pb : zb) + (i64)rel * N;
    };
    auto ld = [&](const double *q, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = *reinterpret_cast<const double2 *>(q);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = q[0];
        }
    };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + VEC : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double um[VEC], uc[VEC], up[VEC];
    double rz[R][VEC], rp[R][VEC], ez[R], ep[R];
    {
        double a[VEC], b[VEC];
        ld(line(ic<-1>{}, false) + i0, a);
        ld(line(ic<-1>{}, true) + i0, b);
        for (int k = 0; k < VEC; ++k) um[k] = a[k] + beta * b[k];
        ld(line(ic<0>{}, false) + i0, a);
        ld(line(ic<0>{}, true) + i0, b);
        for (int k = 0; k < VEC; ++k) uc[k] = a[k] + beta * b[k];
        ld(line(ic<1>{}, false) + i0, a);
        ld(line(ic<1>{}, true) + i0, b);
        for (int k = 0; k < VEC; ++k) up[k] = a[k] + beta * b[k];
    }
    unroll_seq([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        ld(line(ic<2 + d>{}, false) + i0, rz[d]);
        ld(line(ic<2 + d>{}, true) + i0, rp[d]);
        ez[d] = line(ic<d>{}, false)[ei];
        ep[d] = line(ic<d>{}, true)[ei];
    }, std::make_integer_sequence<int, R>{});
    double acc = 0.0;
    double *ob = u_out + (i64)j0 * N + i0;
    auto step = [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        constexpr int S = s % R;
        double left = __shfl_up(uc[VEC - 1], 1, 64);
        double right = __shfl_down(uc[0], 1, 64);
        const double et = ez[S] + beta * ep[S];
        left = lane == 0 ? et : left;
        right = lane == 63 ? et : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + VEC >= N ? 0.0 : right;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double W = k == 0 ? left : uc[k - 1];
            const double E = k == VEC - 1 ? right : uc[k + 1];
            const double yv = 4.0 * uc[k] - (((W + E) + up[k]) + um[k]);
            acc += yv * uc[k];
        }
        if constexpr (VEC == 1) {
            ob[(i64)s * N] = uc[0];
        } else {
            *reinterpret_cast<double2 *>(ob + (i64)s * N) = double2{uc[0], uc[1]};
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            um[k] = uc[k];
            uc[k] = up[k];
            up[k] = rz[S][k] + beta * rp[S][k];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s + R < JTC) {  // refill: edges of line s + R, raw of line s + R + 2
            ez[S] = line(ic<s + R>{}, false)[ei];
            ep[S] = line(ic<s + R>{}, true)[ei];
        }
        if constexpr (s + R + 2 <= JTC) {
            ld(line(ic<s + R + 2>{}, false) + i0, rz[S]);
            ld(line(ic<s + R + 2>{}, true) + i0, rp[S]);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    if (j0 + JTC <= nlines) unroll_seq(step, std::make_integer_sequence<int, JTC>{});
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < TPBm / 64; ++w) t += sm[w];
        part[blockIdx.y * gridDim.x + blockIdx.x] = t;
    }
}

// Staggered start: block by marches [j0 + r, j1) then [j0, j0 + r), r = (by * rot) % cnt,
// so concurrently running blocks touch different line offsets (two primings per block).
// XM: XCD-aware placement on a 1-D grid of gx * gy workgroups -- workgroup id w
// runs on XCD w % 8 (round-robin dispatch); all gx windows of a line block are
// given to one XCD, so the edge lanes' reads of the neighbouring windows' cache
// lines hit that XCD's L2 instead of fetching them again.
template <int VEC, int TPBm, bool XM = false>
__global__ __launch_bounds__(TPBm) void k_march_st(const double *__restrict__ z, const double *__restrict__ p,
                                                   double *__restrict__ u_out, const double *__restrict__ zl, int N,
                                                   int nlines, int JT, int rot, double beta, double *part) {
    __shared__ double sm[TPBm / 64];
    const int lane = threadIdx.x & 63;
    int bx = blockIdx.x, by = blockIdx.y;
    const int gx = XM ? (N + TPBm * VEC - 1) / (TPBm * VEC) : gridDim.x;
    if constexpr (XM) {
        const int gy = (nlines + JT - 1) / JT;
        const int w = blockIdx.x, x = w & 7, q = w >> 3;
        const int per = (gy + 7) / 8;  // line blocks per XCD
        bx = q % gx;
        by = x * per + q / gx;
        if (by >= gy) return;
    }
    const i64 i0 = (i64)bx * (TPBm * VEC) + (i64)VEC * threadIdx.x;
    const int jb0 = by * JT;
    const int jb1 = min(jb0 + JT, nlines);
    const int cnt = jb1 - jb0;
    const int r = (int)(((long long)by * rot) % cnt);
    auto src = [&](const double *b, int jj) -> const double * {
        return (jj >= 0 && jj < nlines) ? b + (i64)jj * N : zl;
    };
    auto ld = [&](const double *q, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = *reinterpret_cast<const double2 *>(q);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = q[0];
        }
    };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + VEC : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double acc = 0.0;
    auto seg = [&](int ja, int jb) {
        double um[VEC], uc[VEC], up[VEC], rz[VEC], rp[VEC], ez0, ep0;
        {
            double a[VEC], b[VEC];
            ld(src(z, ja - 1) + i0, a);
            ld(src(p, ja - 1) + i0, b);
            for (int k = 0; k < VEC; ++k) um[k] = a[k] + beta * b[k];
            ld(src(z, ja) + i0, a);
            ld(src(p, ja) + i0, b);
            for (int k = 0; k < VEC; ++k) uc[k] = a[k] + beta * b[k];
            ld(src(z, ja + 1) + i0, a);
            ld(src(p, ja + 1) + i0, b);
            for (int k = 0; k < VEC; ++k) up[k] = a[k] + beta * b[k];
        }
        ez0 = src(z, ja)[ei];
        ep0 = src(p, ja)[ei];
        for (int j = ja; j < jb; ++j) {
            ld(src(z, j + 2) + i0, rz);
            ld(src(p, j + 2) + i0, rp);
            const double ez1 = src(z, j + 1)[ei], ep1 = src(p, j + 1)[ei];
            double left = __shfl_up(uc[VEC - 1], 1, 64);
            double right = __shfl_down(uc[0], 1, 64);
            const double et = ez0 + beta * ep0;
            left = lane == 0 ? et : left;
            right = lane == 63 ? et : right;
            left = i0 == 0 ? 0.0 : left;
            right = i0 + VEC >= N ? 0.0 : right;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const double W = k == 0 ? left : uc[k - 1];
                const double E = k == VEC - 1 ? right : uc[k + 1];
                const double yv = 4.0 * uc[k] - (((W + E) + up[k]) + um[k]);
                acc += yv * uc[k];
            }
            if constexpr (VEC == 1) {
                u_out[(i64)j * N + i0] = uc[0];
            } else {
                *reinterpret_cast<double2 *>(u_out + (i64)j * N + i0) = double2{uc[0], uc[1]};
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                um[k] = uc[k];
                uc[k] = up[k];
                up[k] = rz[k] + beta * rp[k];
            }
            ez0 = ez1;
            ep0 = ep1;
        }
    };
    seg(jb0 + r, jb1);
    if (r > 0) seg(jb0, jb0 + r);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < TPBm / 64; ++w) t += sm[w];
        part[by * gx + bx] = t;
    }
}

// cbpr2 march (the one-level cg_z pass: read r, write z = cbpr2(r), dot <r, z>), 16 B per
// unknown; DM selects how t = r / d is formed: 0 IEEE division, 1 multiplication by 1/d
// (timing only: not the reference's rounding), 2 one FMA correction of r * (1/d) (Markstein).
template <int DM>
__device__ __forceinline__ double divd(double u, double d, double dinv) {
    if constexpr (DM == 0) return u / d;
    else if constexpr (DM == 1) return u * dinv;
    else {
        const double q = u * dinv;
        const double rr = __builtin_fma(-q, d, u);
        return __builtin_fma(rr, dinv, q);
    }
}

template <int DM>
__global__ __launch_bounds__(256) void k_cbz(const double *__restrict__ r, double *__restrict__ z,
                                             const double *__restrict__ zl, int N, int nlines, int JT, double d,
                                             double dinv, double ca, double *part) {
    __shared__ double sm[4];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * 512 + 2 * threadIdx.x;
    const int j0 = blockIdx.y * JT;
    const int j1 = min(j0 + JT, nlines);
    auto src = [&](int jj) -> const double * { return (jj >= 0 && jj < nlines) ? r + (i64)jj * N : zl; };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + 2 : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double um[2], uc[2], up[2], tm[2], tc[2], tp[2];
    auto ld = [&](int jj, double (&u)[2], double (&t)[2]) {
        const double2 v = *reinterpret_cast<const double2 *>(src(jj) + i0);
        u[0] = v.x;
        u[1] = v.y;
        t[0] = divd<DM>(u[0], d, dinv);
        t[1] = divd<DM>(u[1], d, dinv);
    };
    ld(j0 - 1, um, tm);
    ld(j0, uc, tc);
    ld(j0 + 1, up, tp);
    double ec = src(j0)[ei];
    double acc = 0.0;
    for (int j = j0; j < j1; ++j) {
        const double2 rn = *reinterpret_cast<const double2 *>(src(j + 2) + i0);
        const double en = src(j + 1)[ei];
        double left = __shfl_up(tc[1], 1, 64);
        double right = __shfl_down(tc[0], 1, 64);
        const double et = divd<DM>(ec, d, dinv);
        left = lane == 0 ? et : left;
        right = lane == 63 ? et : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + 2 >= N ? 0.0 : right;
        double y[2];
        for (int k = 0; k < 2; ++k) {
            const double W = k == 0 ? left : tc[0];
            const double E = k == 1 ? right : tc[1];
            const double ax = 4.0 * tc[k] - 1.0 * (((W + E) + tp[k]) + tm[k]);
            y[k] = tc[k] + ca * (uc[k] - ax);
            acc += uc[k] * y[k];
        }
        *reinterpret_cast<double2 *>(z + (i64)j * N + i0) = double2{y[0], y[1]};
        for (int k = 0; k < 2; ++k) {
            um[k] = uc[k];
            tm[k] = tc[k];
            uc[k] = up[k];
            tc[k] = tp[k];
        }
        up[0] = rn.x;
        up[1] = rn.y;
        tp[0] = divd<DM>(up[0], d, dinv);
        tp[1] = divd<DM>(up[1], d, dinv);
        ec = en;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}

// Flat stream of the same mix: out = z + beta p, dot <out, out>; grid-stride double2, U in flight.
template <int U, int NT = 0>  // NT: 1 non-temporal stores, 2 also non-temporal loads
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
            if constexpr (NT >= 2) {
                typedef double d2v __attribute__((ext_vector_type(2)));
                const d2v ta = e < n2 ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(z + e)) : d2v{0, 0};
                const d2v tb = e < n2 ? __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p + e)) : d2v{0, 0};
                a[u] = double2{ta.x, ta.y};
                b[u] = double2{tb.x, tb.y};
            } else {
                a[u] = e < n2 ? z[e] : double2{0, 0};
                b[u] = e < n2 ? p[e] : double2{0, 0};
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = e0 + u * stride;
            const double2 r{a[u].x + beta * b[u].x, a[u].y + beta * b[u].y};
            if (e < n2) {
                if constexpr (NT >= 1) {
                    typedef double d2v __attribute__((ext_vector_type(2)));
                    __builtin_nontemporal_store(d2v{r.x, r.y}, reinterpret_cast<d2v *>(o + e));
                } else {
                    o[e] = r;
                }
            }
            acc += r.x * r.x + r.y * r.y;
        }
    }
    for (int k = 32; k > 0; k >>= 1) acc += __shfl_xor(acc, k, 64);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}

// Cache flush by READING 1 GiB: dirty lines of the previous launch are written
// back here, outside the timed launch, and the caches are left holding clean lines.
__global__ __launch_bounds__(256) void k_flush(const double2 *__restrict__ f, i64 n2, double *out) {
    double acc = 0.0;
    for (i64 e = (i64)blockIdx.x * 256 + threadIdx.x; e < n2; e += (i64)gridDim.x * 256) acc += f[e].x;
    if (acc == 12345.0) out[0] = acc;
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
        k_flush<<<4096, 256>>>((const double2 *)b.flush, (i64)(b.flush_bytes / 16), b.part);
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

template <int VEC, int TPBm, int R>
static void march2(const Bufs &b, int JT) {
    const int N = b.N;
    const int gx = (N + TPBm * VEC - 1) / (TPBm * VEC);
    const int gy = (N + JT - 1) / JT;
    char name[96];
    std::snprintf(name, sizeof name, "march2 VEC%d TPB%d R%d JT%d (%d wg)", VEC, TPBm, R, JT, gx * gy);
    const double bytes = 24.0 * N * (double)N;
    timeit(name, b, [&] {
        k_march2<VEC, TPBm, R><<<dim3(gx, gy), TPBm>>>(b.z, b.p, b.o, b.zl, N, N, JT, 0.5, b.part);
    }, bytes);
}

template <int VEC, int TPBm, int R, int JTC>
static void march3(const Bufs &b) {
    const int N = b.N;
    const int gx = (N + TPBm * VEC - 1) / (TPBm * VEC);
    const int gy = (N + JTC - 1) / JTC;
    char name[96];
    std::snprintf(name, sizeof name, "march3 VEC%d TPB%d R%d JT%d (%d wg)", VEC, TPBm, R, JTC, gx * gy);
    const double bytes = 24.0 * N * (double)N;
    timeit(name, b, [&] {
        k_march3<VEC, TPBm, R, JTC><<<dim3(gx, gy), TPBm>>>(b.z, b.p, b.o, b.zl, N, N, 0.5, b.part);
    }, bytes);
}

static void march_xm(const Bufs &b, int JT) {
    const int N = b.N;
    const int gx = N / 512, gy = (N + JT - 1) / JT;
    const int nw = 8 * gx * ((gy + 7) / 8);
    char name[96];
    std::snprintf(name, sizeof name, "xcd-aware VEC2 TPB256 JT%d (%d wg)", JT, nw);
    timeit(name, b, [&] {
        k_march_st<2, 256, true><<<nw, 256>>>(b.z, b.p, b.o, b.zl, N, N, JT, 0, 0.5, b.part);
    }, 24.0 * N * (double)N);
}

static void march_st(const Bufs &b, int JT, int rot) {
    const int N = b.N;
    const int gx = N / 512, gy = (N + JT - 1) / JT;
    char name[96];
    std::snprintf(name, sizeof name, "staggered VEC2 TPB256 JT%d rot%d (%d wg)", JT, rot, gx * gy);
    timeit(name, b, [&] {
        k_march_st<2, 256><<<dim3(gx, gy), 256>>>(b.z, b.p, b.o, b.zl, N, N, JT, rot, 0.5, b.part);
    }, 24.0 * N * (double)N);
}

// The same cbpr2 march with V points per lane (V / 2 double2 loads per lane per line in flight).
template <int V>
__global__ __launch_bounds__(256) void k_cbzv(const double *__restrict__ r, double *__restrict__ z,
                                              const double *__restrict__ zl, int N, int nlines, int JT, double d,
                                              double ca, double *part) {
    __shared__ double sm[4];
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (256 * V) + (i64)V * threadIdx.x;
    const int j0 = blockIdx.y * JT;
    const int j1 = min(j0 + JT, nlines);
    auto src = [&](int jj) -> const double * { return (jj >= 0 && jj < nlines) ? r + (i64)jj * N : zl; };
    i64 ei = lane == 0 ? i0 - 1 : (lane == 63 ? i0 + V : i0);
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    double uc[V], up[V], tm[V], tc[V], tp[V];
    auto ld = [&](int jj, double (&u)[V]) {
#pragma unroll
        for (int k = 0; k < V; k += 2) {
            const double2 v = *reinterpret_cast<const double2 *>(src(jj) + i0 + k);
            u[k] = v.x;
            u[k + 1] = v.y;
        }
    };
    {
        double um[V];
        ld(j0 - 1, um);
        ld(j0, uc);
        ld(j0 + 1, up);
#pragma unroll
        for (int k = 0; k < V; ++k) {
            tm[k] = um[k] / d;
            tc[k] = uc[k] / d;
            tp[k] = up[k] / d;
        }
    }
    double ec = src(j0)[ei];
    double acc = 0.0;
    for (int j = j0; j < j1; ++j) {
        double rn[V];
        ld(j + 2, rn);
        const double en = src(j + 1)[ei];
        double left = __shfl_up(tc[V - 1], 1, 64);
        double right = __shfl_down(tc[0], 1, 64);
        const double et = ec / d;
        left = lane == 0 ? et : left;
        right = lane == 63 ? et : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + V >= N ? 0.0 : right;
        double y[V];
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const double W = k == 0 ? left : tc[k - 1];
            const double E = k == V - 1 ? right : tc[k + 1];
            const double ax = 4.0 * tc[k] - 1.0 * (((W + E) + tp[k]) + tm[k]);
            y[k] = tc[k] + ca * (uc[k] - ax);
            acc += uc[k] * y[k];
        }
#pragma unroll
        for (int k = 0; k < V; k += 2)
            *reinterpret_cast<double2 *>(z + (i64)j * N + i0 + k) = double2{y[k], y[k + 1]};
#pragma unroll
        for (int k = 0; k < V; ++k) {
            tm[k] = tc[k];
            uc[k] = up[k];
            tc[k] = tp[k];
            up[k] = rn[k];
            tp[k] = rn[k] / d;
        }
        ec = en;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) sm[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.y * gridDim.x + blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}

template <int V>
static void cbzv(const Bufs &b, int JT) {
    const int N = b.N;
    const int gx = N / (256 * V), gy = (N + JT - 1) / JT;
    char name[96];
    std::snprintf(name, sizeof name, "cbz march V%d JT%d (%d wg)", V, JT, gx * gy);
    timeit(name, b, [&] {
        k_cbzv<V><<<dim3(gx, gy), 256>>>(b.z, b.o, b.zl, N, N, JT, 4.2, 0.2516835977628125, b.part);
    }, 16.0 * N * (double)N);
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
    CK(hipMemset(b.flush, 0, b.flush_bytes));
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
        for (int JT : {32, 64, 128, 48, 56, 60, 62, 63, 65, 66, 72, 80, 96, 40, 36, 33}) {
            if (argc > 2 && (argv[2][0] == 'x' || argv[2][0] == 'c') && JT != 64) continue;
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
    if (argc > 2 && argv[2][0] == 'd') {  // the cbpr2 march: division cost
        const int JT = 64, gx = N / 512, gy = N / JT;
        const double d = 4.2, dinv = 1.0 / 4.2, ca = 0.2516835977628125;
        for (int rep = 0; rep < 2; ++rep) {
            timeit("cbz march IEEE division", b, [&] {
                k_cbz<0><<<dim3(gx, gy), 256>>>(b.z, b.o, b.zl, N, N, JT, d, dinv, ca, b.part);
            }, 16.0 * (double)n);
            timeit("cbz march x (1/d) (timing only)", b, [&] {
                k_cbz<1><<<dim3(gx, gy), 256>>>(b.z, b.o, b.zl, N, N, JT, d, dinv, ca, b.part);
            }, 16.0 * (double)n);
            timeit("cbz march Markstein (1 fma correction)", b, [&] {
                k_cbz<2><<<dim3(gx, gy), 256>>>(b.z, b.o, b.zl, N, N, JT, d, dinv, ca, b.part);
            }, 16.0 * (double)n);
            for (int JT : {16, 32, 64, 128}) cbzv<2>(b, JT);
            for (int JT : {16, 32, 64}) cbzv<4>(b, JT);
            for (int JT : {8, 16, 32}) cbzv<8>(b, JT);
            timeit("copy-like flat read1 write1 (k_flat with p = z)", b, [&] {
                k_flat<4><<<2048, 256>>>((const double2 *)b.z, (const double2 *)b.z, (double2 *)b.o, n / 2, 0.5,
                                         b.part);
            }, 16.0 * (double)n);
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'x') {
        for (int rep = 0; rep < 2; ++rep)
            for (int JT : {32, 48, 64, 65, 66, 72, 128}) {
                march_st(b, JT, 0);
                march_xm(b, JT);
            }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 's') {
        for (int JT : {64, 65, 128})
            for (int rot : {0, 1, 5, 17, 23, 37}) march_st(b, JT, rot);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'j') return 0;
    const bool chain_only = argc > 2 && argv[2][0] == 'c';
    if (!chain_only) {
    march3<2, 256, 2, 64>(b);
    march3<2, 256, 4, 64>(b);
    march3<2, 256, 6, 64>(b);
    march3<2, 256, 2, 32>(b);
    march3<2, 256, 4, 32>(b);
    march3<2, 256, 4, 16>(b);
    march3<2, 128, 4, 64>(b);
    march3<2, 128, 4, 32>(b);
    march3<1, 256, 4, 64>(b);
    march3<1, 256, 4, 32>(b);
    for (int JT : {32, 64}) {
        march<2, 256, 0>(b, JT);
        march2<2, 256, 1>(b, JT);
        march2<2, 256, 2>(b, JT);
        march2<2, 256, 3>(b, JT);
        march2<2, 256, 4>(b, JT);
    }
    for (int JT : {16, 32}) {
        march2<2, 256, 2>(b, JT);
        march2<2, 256, 4>(b, JT);
    }
    march2<2, 128, 2>(b, 64);
    march2<2, 128, 4>(b, 64);
    march2<2, 512, 2>(b, 32);
    march2<2, 512, 4>(b, 32);
    march2<1, 256, 4>(b, 64);
    }
    if (argc > 2 && !chain_only) return 0;
    // Pass chains: every pass reads the previous pass's output and an older
    // vector and writes a third (buffers rotate over 4), 24 passes timed
    // together without flushing -- the Krylov pattern.  Same direction every
    // pass vs alternating (the last lines written are the first read).
    {
        double *v[4] = {b.z, b.p, b.o, nullptr};
        CK(hipMalloc(&v[3], n * 8));
        CK(hipMemset(v[3], 0, n * 8));
        const int JT = 64, gx = N / 512, gy = N / JT;
        for (int rep = 0; rep < 3; ++rep)
            for (int alt = 0; alt < 2; ++alt) {
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                CK(hipMemsetAsync(b.flush, 0, b.flush_bytes, 0));
                CK(hipEventRecord(e0, 0));
                const int P = 24;
                for (int i = 0; i < P; ++i) {
                    const double *in0 = v[(i + 2) & 3], *in1 = v[i & 3];
                    double *out = v[(i + 3) & 3];
                    if (alt && (i & 1))
                        k_march<2, 256, 0, true><<<dim3(gx, gy), 256>>>(in0, in1, out, b.zl, N, N, JT, 0.5, b.part);
                    else
                        k_march<2, 256, 0, false><<<dim3(gx, gy), 256>>>(in0, in1, out, b.zl, N, N, JT, 0.5, b.part);
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / P;
                std::printf("chain of %d passes, %s: %8.2f us per pass %8.1f GB/s frac %.3f\n", P,
                            alt ? "alternating direction" : "same direction", us, bytes / us / 1e3,
                            bytes / us / 1e3 / 8000.0);
                std::fflush(stdout);
            }
        // the same chains on the flat kernel (contiguous sweep order)
        for (int rep = 0; rep < 6; ++rep) {
            const int nt = rep % 3;
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipMemsetAsync(b.flush, 0, b.flush_bytes, 0));
            CK(hipEventRecord(e0, 0));
            const int P = 24;
            for (int i = 0; i < P; ++i) {
                const double2 *x0 = (const double2 *)v[(i + 2) & 3], *x1 = (const double2 *)v[i & 3];
                double2 *y = (double2 *)v[(i + 3) & 3];
                if (nt == 0) k_flat<4, 0><<<2048, 256>>>(x0, x1, y, n / 2, 0.5, b.part);
                if (nt == 1) k_flat<4, 1><<<2048, 256>>>(x0, x1, y, n / 2, 0.5, b.part);
                if (nt == 2) k_flat<4, 2><<<2048, 256>>>(x0, x1, y, n / 2, 0.5, b.part);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / P;
            std::printf("chain of %d passes, flat (nt %d): %8.2f us per pass %8.1f GB/s frac %.3f\n", P, nt, us, bytes / us / 1e3,
                        bytes / us / 1e3 / 8000.0);
        }
    }
    if (argc > 2) return 0;
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
