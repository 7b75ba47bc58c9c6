// gk_kernels.hpp -- CDNA4 (gfx950) HIP kernels for the GMRES(m) inner cycle.
//
// Every kernel is HBM-bandwidth bound (fp64, ~0.1-0.3 flop/B), so the design
// rules are: 16-byte (double2) coalesced accesses along the fast grid index i,
// enough independent loads in flight per wave, one pass over each vector per
// launch, and reductions that never leave the device.  No MFMA: nothing here
// is GEMM-shaped except the off-metric Gram diagnostic.
//
// Reductions are deterministic: every producer writes one partial per
// workgroup into a fixed-length slab; the consumer kernel (the next launch in
// the MGS chain) re-reduces the slab in a fixed order in its prologue
// ("launch-boundary reduce", cdna_hip_programming.md 5, item 2), so a dot
// product never needs an atomic, a grid barrier or a host round trip, and on
// N GPUs the slab itself is what RCCL all-reduces.
//
// Compiled with -ffp-contract=off: elementwise results are bit-identical to
// the CPU oracle (same association order as the Fortran reference); only the
// dot-product summation order differs.
#pragma once
#include "gk_common.hpp"
#include "gk_cheb.hpp"
#include "gk_res.hpp"

namespace gk {

// --------------------------------------------------------------------------
// Projection kernel: the MGS-R / Householder inner cascade
// (gmres_mgsr.f90:343-358, gmres_hh.f90:269-304).
//
//   h    = sum(pin[0..npin))            (the previous launch's dot, reduced)
//   w   -= (coef*h) * va                (AXPY with the just-finished dot)
//   acc += w * vb   or   w * w          (the NEXT dot, fused into the same pass)
//
// One launch = one AXPY of projection i fused with the dot of projection i+1:
// reads w, va, vb and writes w (32 B/unknown) where the reference's separate
// dot + AXPY move 40 B/unknown.
// --------------------------------------------------------------------------
enum { PJ_DOT = 0, PJ_AXPY = 1, PJ_AXPY_DOT = 2, PJ_AXPY_NORM = 3 };


template <int MODE, bool NT = false, int U = UNR>
__global__ __launch_bounds__(TPB) void k_proj(double *__restrict__ w, const double *__restrict__ va,
                                              const double *__restrict__ vb,
                                              const double *__restrict__ pin, int npin,
                                              double *__restrict__ pout, double *__restrict__ hslot,
                                              double coef, i64 n, i64 tail0, int blocked,
                                              int hstore) {
    __shared__ double sm[WAVES];
    const i64 n2 = n >> 1;
    double2 *__restrict__ W2 = reinterpret_cast<double2 *>(w);
    const double2 *__restrict__ A2 = reinterpret_cast<const double2 *>(va);
    const double2 *__restrict__ B2 = reinterpret_cast<const double2 *>(vb);
    // Work mapping: grid-stride over U*TPB double2 chunks (default), or one
    // contiguous range per workgroup (blocked).
    i64 lo, hi, step;
    if (blocked) {
        const i64 chunk = (i64)TPB * U;
        const i64 per = ((n2 + gridDim.x - 1) / gridDim.x + chunk - 1) / chunk * chunk;
        lo = (i64)blockIdx.x * per;
        hi = min(lo + per, n2);
        step = chunk;
    } else {
        lo = (i64)blockIdx.x * TPB * U;
        hi = n2;
        step = (i64)gridDim.x * TPB * U;
    }
    double2 wv[U], av[U], bv[U];
    i64 idx[U];
    auto issue = [&](i64 base) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = base + (i64)u * TPB;
            idx[u] = (e < hi) ? e : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = idx[u];
            if (e >= 0) {
                wv[u] = W2[e];
                if (MODE != PJ_DOT) av[u] = ldv<NT>(A2 + e);
                if (MODE == PJ_DOT || MODE == PJ_AXPY_DOT) bv[u] = ldv<NT>(B2 + e);
            }
        }
    };
    // The first chunk's loads do not depend on h: issue them before the
    // slab-reduce prologue so their latency hides behind it (matters when a
    // launch is only a few microseconds: small grids, many GPUs).
    i64 base = lo + threadIdx.x;
    if (base < hi) issue(base);
    double ch = 0.0;
    if (MODE != PJ_DOT) {
        const double h = reduce_slab(pin, npin, sm);
        // H(i,j) = H(i,j) + h: the first MGS pass starts from H(i,j) = 0
        if (hslot != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *hslot = (hstore ? 0.0 : *hslot) + h;
        ch = coef * h;
    }
    double acc = 0.0;
    while (base < hi) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = idx[u];
            if (e >= 0) {
                if (MODE != PJ_DOT) {
                    wv[u].x = wv[u].x - ch * av[u].x;
                    wv[u].y = wv[u].y - ch * av[u].y;
                    W2[e] = wv[u];
                }
                if (MODE == PJ_DOT || MODE == PJ_AXPY_DOT) {
                    acc = acc + wv[u].x * bv[u].x;
                    acc = acc + wv[u].y * bv[u].y;
                }
                if (MODE == PJ_AXPY_NORM) {
                    if (2 * e >= tail0) acc = acc + wv[u].x * wv[u].x;
                    if (2 * e + 1 >= tail0) acc = acc + wv[u].y * wv[u].y;
                }
            }
        }
        base += step;
        if (base < hi) issue(base);
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {  // odd-length tail element
        const i64 e = n - 1;
        double x = w[e];
        if (MODE != PJ_DOT) {
            x = x - ch * va[e];
            w[e] = x;
        }
        if (MODE == PJ_DOT || MODE == PJ_AXPY_DOT) acc = acc + x * vb[e];
        if (MODE == PJ_AXPY_NORM && e >= tail0) acc = acc + x * x;
    }
    if (MODE != PJ_AXPY) {
        const double s = block_sum(acc, sm);
        if (threadIdx.x == 0) pout[blockIdx.x] = s;
    }
}

// out = w / h, h = sqrt(sum(pin)) (norm2 + scale, gmres_mgsr.f90:362-363,384).
// hslot (optional) receives h.  h == 0 (exact breakdown) writes zeros instead
// of the reference's Inf/NaN.
// hcopy (optional): block 0 also publishes hsrc[0..ncopy) and h to hcopy
// (mapped pinned host memory: the step's Hessenberg column, no extra copy).
// pin_norm: pin[0] is h itself (a norm taken in the reference's order, k_norm2_seq).
__global__ __launch_bounds__(TPB) void k_scale(double *__restrict__ out, const double *__restrict__ w,
                                               const double *__restrict__ pin, int npin,
                                               double *__restrict__ hslot, i64 n,
                                               double *__restrict__ hcopy = nullptr,
                                               const double *__restrict__ hsrc = nullptr, int ncopy = 0,
                                               int pin_norm = 0) {
    __shared__ double sm[WAVES];
    const double h = pin_norm ? pin[0] : sqrt(reduce_slab(pin, npin, sm));
    if (hslot != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *hslot = h;
    if (hcopy != nullptr && blockIdx.x == 0) {
        for (int k = threadIdx.x; k < ncopy; k += TPB) hcopy[k] = hsrc[k];
        if (threadIdx.x == 0) hcopy[ncopy] = h;
    }
    const i64 n2 = n >> 1;
    const double2 *__restrict__ W2 = reinterpret_cast<const double2 *>(w);
    double2 *__restrict__ O2 = reinterpret_cast<double2 *>(out);
    const i64 stride = (i64)gridDim.x * TPB;
    if (h != 0.0) {
        for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n2; e += stride) {
            double2 v = W2[e];
            v.x = v.x / h;
            v.y = v.y / h;
            O2[e] = v;
        }
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) out[n - 1] = w[n - 1] / h;
    } else {
        for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n2; e += stride) O2[e] = double2{0.0, 0.0};
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) out[n - 1] = 0.0;
    }
}

// out[0] = NORM2(x(0:n)) as flang-rt computes it (Norm2Accumulator<8>: a running
// max m and a scaled sum s, result m sqrt(1 + s); the tests check it against the CPU restatement) --
// the reference's serial norm2 of gmres_hh.f90:251-253,307,315, in its order.  One
// workgroup: chunks of TPB elements staged through LDS, thread 0 folds each in order
// (GK_TUNE_HH_NORM_ORDER, single rank; ~2 us per 256 elements).
__global__ __launch_bounds__(TPB) void k_norm2_seq(const double *__restrict__ x, i64 n, double *__restrict__ out) {
    __shared__ double buf[TPB];
    double mx = 0.0, s = 0.0;
    for (i64 c0 = 0; c0 < n; c0 += TPB) {
        const i64 e = c0 + threadIdx.x;
        buf[threadIdx.x] = e < n ? x[e] : 0.0;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int cnt = n - c0 < TPB ? (int)(n - c0) : TPB;
            for (int k = 0; k < cnt; ++k) {
                const double a = fabs(buf[k]);
                if (mx == 0.0) {
                    mx = a;
                } else if (a > mx) {
                    const double t = mx / a;
                    const double tsq = t * t;
                    s = s * tsq;
                    s = s + tsq;
                    mx = a;
                } else {
                    const double t = a / mx;
                    s = s + t * t;
                }
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = mx * sqrt(1.0 + s);
}

// out[0] = sqrt(sum(pin)) or sum(pin).
__global__ __launch_bounds__(TPB) void k_finalize(const double *__restrict__ pin, int npin,
                                                  double *__restrict__ out, int take_sqrt) {
    __shared__ double sm[WAVES];
    const double s = reduce_slab(pin, npin, sm);
    if (threadIdx.x == 0) out[0] = take_sqrt ? sqrt(s) : s;
}

// x[e] += sum_k V[k*ld + e] * y[k]  (gmres_mgsr.f90:400-406: the reference's
// row-wise dot_product(V(idx,1:n_out), y) with idx on the lane, k sequential).
__global__ __launch_bounds__(TPB) void k_update_x(double *__restrict__ x, const double *__restrict__ V,
                                                  i64 ld, const double *__restrict__ y, int nout, i64 n) {
    const i64 n2 = n >> 1;
    const i64 stride = (i64)gridDim.x * TPB;
    double2 *__restrict__ X2 = reinterpret_cast<double2 *>(x);
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n2; e += stride) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll 8
        for (int k = 0; k < nout; ++k) {
            const double2 v = reinterpret_cast<const double2 *>(V + (i64)k * ld)[e];
            const double yk = y[k];
            s0 = s0 + v.x * yk;
            s1 = s1 + v.y * yk;
        }
        double2 xv = X2[e];
        xv.x = xv.x + s0;
        xv.y = xv.y + s1;
        X2[e] = xv;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        double s = 0.0;
        for (int k = 0; k < nout; ++k) s = s + V[(i64)k * ld + n - 1] * y[k];
        x[n - 1] = x[n - 1] + s;
    }
}

// x = x + w  (gmres_hh.f90:374-378)
__global__ __launch_bounds__(TPB) void k_add(double *__restrict__ x, const double *__restrict__ w, i64 n) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) x[e] = x[e] + w[e];
}

// y = y + a x  (host scalar a)
__global__ __launch_bounds__(TPB) void k_axpy_host(double *__restrict__ y, double a, const double *__restrict__ x,
                                                   i64 n) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) y[e] = y[e] + a * x[e];
}

// x[e] = deterministic pseudo-random value of the GLOBAL index g0+e in [-1,1)
// (splitmix64), identical for any slab decomposition.
__global__ __launch_bounds__(TPB) void k_fill_hash(double *__restrict__ x, i64 n, i64 g0, unsigned long long seed) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) {
        unsigned long long z = (unsigned long long)(g0 + e) + seed * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        x[e] = (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
    }
}

// Linear combinations of the short-recurrence solvers, in the reference's
// expression order (src/cg.f90:205-231, src/bicgstab.f90:131-180).
enum { LC_COPY = 0, LC_AXPY = 1, LC_AXPY2 = 2, LC_XPAYMZ = 3, LC_ZERO = 4 };
__global__ __launch_bounds__(TPB) void k_lincomb(int form, double *out, const double *a, const double *b,
                                                 const double *c, double s1, double s2, i64 n) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) {
        double v;
        switch (form) {
            case LC_COPY: v = a[e]; break;
            case LC_AXPY: v = a[e] + s1 * b[e]; break;                  // a + s1 b
            case LC_AXPY2: v = a[e] + s1 * b[e] + s2 * c[e]; break;      // (a + s1 b) + s2 c
            case LC_XPAYMZ: v = a[e] + s1 * (b[e] - s2 * c[e]); break;   // a + s1 (b - s2 c)
            default: v = 0.0; break;
        }
        out[e] = v;
    }
}

__global__ __launch_bounds__(TPB) void k_fill(double *__restrict__ x, double v, i64 n) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) x[e] = v;
}

// x = 0 except x[gk - g0] = vals[k] for global indices gk = k in [0, nvals)
// (v_j = e_j, gmres_hh.f90:257-265; w(1:n_out) = y, :356-357).
__global__ __launch_bounds__(TPB) void k_set_prefix(double *__restrict__ x, i64 n, i64 g0,
                                                    const double *__restrict__ vals, int first,
                                                    int nvals) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) {
        const i64 g = g0 + e;
        x[e] = (g >= first && g < first + nvals) ? vals[g - first] : 0.0;
    }
}

// x = e_g (global index g): zero everywhere, `value` at global index g.
__global__ __launch_bounds__(TPB) void k_set_unit(double *__restrict__ x, i64 n, i64 g0, i64 g, double value) {
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) x[e] = (g0 + e == g) ? value : 0.0;
}

// Householder reflector fix-up (gmres_hh.f90:39-41, :305-318): zero global
// indices < zero_below; at global index fix_idx add delta[0]; accumulate
// sum w^2 of the result into pout.
__global__ __launch_bounds__(TPB) void k_hh_fix(double *__restrict__ w, i64 n, i64 g0, i64 zero_below,
                                                i64 fix_idx, const double *__restrict__ delta,
                                                double *__restrict__ pout) {
    __shared__ double sm[WAVES];
    const i64 stride = (i64)gridDim.x * TPB;
    const double dl = delta[0];
    double acc = 0.0;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) {
        const i64 g = g0 + e;
        double v = w[e];
        if (g < zero_below) {
            v = 0.0;
            w[e] = v;
        } else if (g == fix_idx) {
            v = v + dl;
            w[e] = v;
        }
        acc = acc + v * v;
    }
    const double s = block_sum(acc, sm);
    if (threadIdx.x == 0) pout[blockIdx.x] = s;
}

// Householder pivot bookkeeping, one workgroup.  hb[0..j] = w(1:j+1) broadcast
// from the owning rank; pin = sum of squares of the tail.
//  start (j == 0): beta = sqrt(sum w^2); g1 = -sign(beta,w1); delta = sign(beta,w1)
//                  -> res[0] = g1, delta[0] = sign(beta, w1)          (:250-252)
//  step  (j >= 1): tmp = sqrt(tail); H(j+1,j) = w(j+1) > 0 ? -tmp : tmp
//                  -> hcol[0..j-1] = w(1:j), hcol[j] = H(j+1,j), delta = -H (:306-316)
// pin_norm: pin[0] is the norm itself (k_norm2_seq) instead of a partial slab of squares.
__global__ void k_hh_pivot(const double *__restrict__ hb, const double *__restrict__ pin, int npin,
                           int j, double *__restrict__ hcol, double *__restrict__ delta,
                           double *__restrict__ hcopy = nullptr, int pin_norm = 0) {
    __shared__ double sm[WAVES];
    const double s = pin_norm ? pin[0] : sqrt(reduce_slab(pin, npin, sm));
    if (j == 0) {
        if (threadIdx.x == 0) {
            const double w1 = hb[0];
            const double sg = copysign(fabs(s), w1);
            hcol[0] = -sg;
            delta[0] = sg;
        }
        return;
    }
    for (int k = threadIdx.x; k < j; k += blockDim.x) {
        hcol[k] = hb[k];
        if (hcopy != nullptr) hcopy[k] = hb[k];
    }
    if (threadIdx.x == 0) {
        const double H = (hb[j] > 0.0) ? -s : s;
        hcol[j] = H;
        if (hcopy != nullptr) hcopy[j] = H;
        delta[0] = -H;
    }
}

// --------------------------------------------------------------------------
// Poisson-5 stencil sweep with fused preconditioner epilogues
// (src/problems/poisson.f90:33-77, src/preconds/chebyshev.f90:27-37).
//
// A workgroup owns TPB*VEC consecutive points of the fast index i and marches
// over JT grid lines j, keeping lines j-1, j, j+1 of the operand in registers:
// every operand element is read from HBM once (plus one halo line per JT),
// the W/E neighbours come from the adjacent lanes by __shfl (wave64; lanes 0
// and 63 read their outer neighbour through L1).  Missing neighbours at the
// physical boundary are zeros: x + 0 is exact, so the sum ((W+E)+S)+N is
// bit-identical to the reference's separate edge / corner statements.
// Lines -1 and nlines come from the halo buffers (RCCL halo exchange on N
// GPUs) or are zero at the physical boundary.
// --------------------------------------------------------------------------
enum {
    OP_PLAIN = 0,      // y = A x
    OP_RESID = 1,      // y = b - A x                                (gmres_mgsr.f90:314-319)
    OP_CBPR2 = 2,      // x = z: zp = z/d, y = zp + alpha*(z - A zp) (chebyshev.f90:27-37)
    OP_CHEB_FIRST = 3, // x = r: d0 = r/theta; first Chebyshev iteration
    OP_CHEB_ITER = 4,  // x = d: next Chebyshev iteration
};

struct StArgs {
    const double *x;    // operand, nlines*N
    const double *hlo;  // line -1 (nullptr: physical boundary)
    const double *hhi;  // line nlines (nullptr: physical boundary)
    const double *in1;  // RESID: b ; CHEB_ITER: residual r_k
    const double *in2;  // CHEB_ITER: running sum z_k
    double *y;          // main output
    double *o_res;      // CHEB: r_{k+1} (nullptr on the last iteration)
    double *o_d;        // CHEB: d_{k+1} (nullptr on the last iteration)
    const double *vdot; // ACC_DOT partner vector
    double *part;       // partial slab (ACC != NONE)
    double s1, s2, s3;  // CBPR2: d, alpha ; CHEB: theta(first)/unused, c1, c2
    int N, nlines, JT;
};

template <int VEC>
__device__ __forceinline__ void ld_vec(const double *p, bool ok, double (&v)[VEC]) {
    if (ok) {
        if constexpr (VEC == 2) {
            const double2 t = *reinterpret_cast<const double2 *>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = p[0];
        }
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) v[k] = 0.0;
    }
}

template <int VEC>
__device__ __forceinline__ void st_vec(double *p, const double (&v)[VEC]) {
    if constexpr (VEC == 2) {
        *reinterpret_cast<double2 *>(p) = double2{v[0], v[1]};
    } else {
        p[0] = v[0];
    }
}

template <int VEC, int OP, int ACC>
__global__ __launch_bounds__(TPB) void k_stencil(StArgs a) {
    __shared__ double sm[WAVES];
    const int N = a.N;
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPB * VEC) + (i64)VEC * threadIdx.x;
    const bool act = i0 < N;
    const int j0 = blockIdx.y * a.JT;
    const int j1 = min(j0 + a.JT, a.nlines);
    // operand transform at load (CBPR2: /d ; CHEB_FIRST: /theta)
    constexpr bool XF = (OP == OP_CBPR2 || OP == OP_CHEB_FIRST);
    const double dv = a.s1;
    double acc = 0.0;

    auto line_ptr = [&](int jj) -> const double * {
        if (jj < 0) return a.hlo;
        if (jj >= a.nlines) return a.hhi;
        return a.x + (i64)jj * N;
    };
    auto load_line = [&](int jj, double (&raw)[VEC], double (&t)[VEC]) {
        const double *p = line_ptr(jj);
        ld_vec<VEC>(p != nullptr ? p + i0 : nullptr, act && p != nullptr, raw);
#pragma unroll
        for (int k = 0; k < VEC; ++k) t[k] = XF ? raw[k] / dv : raw[k];
    };

    if (j0 < a.nlines) {
        // lines j-1, j, j+1 in registers and line j+2 in flight while line j is computed
        double rm[VEC], rc[VEC], rp[VEC], tm[VEC], tc[VEC], tp[VEC], rn[VEC], tn[VEC];
        load_line(j0 - 1, rm, tm);
        load_line(j0, rc, tc);
        load_line(j0 + 1, rp, tp);
#pragma unroll
        for (int k = 0; k < VEC; ++k) rn[k] = tn[k] = 0.0;
        for (int j = j0; j < j1; ++j) {
            if (j + 2 <= j1) load_line(j + 2, rn, tn);
            const i64 row = (i64)j * N;
            // W/E neighbours of the lane's first / last point
            double left = __shfl_up(tc[VEC - 1], 1, 64);  // previous lane's last point
            double right = __shfl_down(tc[0], 1, 64);      // next lane's first point
            if (lane == 0 && act) left = (i0 > 0) ? a.x[row + i0 - 1] : 0.0;
            if (lane == 63 && act) right = (i0 + VEC < N) ? a.x[row + i0 + VEC] : 0.0;
            if (XF && lane == 0) left = left / dv;
            if (XF && lane == 63) right = right / dv;
            if (i0 == 0) left = 0.0;
            if (i0 + VEC >= N) right = 0.0;
            double yv[VEC];
            double in1v[VEC], in2v[VEC];
            if (OP == OP_RESID || OP == OP_CHEB_ITER) ld_vec<VEC>(a.in1 + row + i0, act, in1v);
            if (OP == OP_CHEB_ITER) ld_vec<VEC>(a.in2 + row + i0, act, in2v);
            // the dot operand is issued with the line loads, not after the store
            double vd[VEC];
            if (ACC == ACC_DOT) ld_vec<VEC>(a.vdot + row + i0, act, vd);
            double resv[VEC], dnv[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const double W = (k == 0) ? left : tc[k - 1];
                const double E = (k == VEC - 1) ? right : tc[k + 1];
                const double s = ((W + E) + tp[k]) + tm[k];
                const double ax = 4.0 * tc[k] - 1.0 * s;
                if (OP == OP_PLAIN) {
                    yv[k] = ax;
                } else if (OP == OP_RESID) {
                    yv[k] = in1v[k] - ax;
                } else if (OP == OP_CBPR2) {
                    yv[k] = tc[k] + a.s2 * (rc[k] - ax);
                } else if (OP == OP_CHEB_FIRST) {
                    // res = r - A d0 ; d1 = c1*d0 + c2*res ; z = d0 + d1
                    const double res = rc[k] - ax;
                    const double dn = a.s2 * tc[k] + a.s3 * res;
                    resv[k] = res;
                    dnv[k] = dn;
                    yv[k] = tc[k] + dn;
                } else {  // OP_CHEB_ITER
                    const double res = in1v[k] - ax;
                    const double dn = a.s2 * tc[k] + a.s3 * res;
                    resv[k] = res;
                    dnv[k] = dn;
                    yv[k] = in2v[k] + dn;
                }
            }
            if (act) {
                st_vec<VEC>(a.y + row + i0, yv);
                if (OP == OP_CHEB_FIRST || OP == OP_CHEB_ITER) {
                    if (a.o_res != nullptr) st_vec<VEC>(a.o_res + row + i0, resv);
                    if (a.o_d != nullptr) st_vec<VEC>(a.o_d + row + i0, dnv);
                }
                if (ACC == ACC_DOT) {
#pragma unroll
                    for (int k = 0; k < VEC; ++k) acc = acc + yv[k] * vd[k];
                } else if (ACC == ACC_NORM) {
#pragma unroll
                    for (int k = 0; k < VEC; ++k) acc = acc + yv[k] * yv[k];
                }
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                rm[k] = rc[k];
                tm[k] = tc[k];
                rc[k] = rp[k];
                tc[k] = tp[k];
                rp[k] = rn[k];
                tp[k] = tn[k];
            }
        }
    }
    if (ACC != ACC_NONE) {
        const double s = block_sum(acc, sm);
        if (threadIdx.x == 0) a.part[(i64)blockIdx.y * gridDim.x + blockIdx.x] = s;
    }
}

// --------------------------------------------------------------------------
// Gram matrix of columns 0..c-1 of V (the v_err diagnostics,
// gmres_mgsr.f90:414-420, gmres_hh.f90:587-591).  Off the Arnoldi metric.
// Each workgroup stages GROWS rows x c columns in LDS and accumulates the
// c(c+1)/2 pairs it owns; slab[blk*npairs + p]; then k_gram_reduce sums the
// slab over workgroups in a fixed order.
// --------------------------------------------------------------------------
constexpr int GROWS = 32;
constexpr int GCMAX = 128;
constexpr int GPPT = (GCMAX * (GCMAX + 1) / 2 + TPB - 1) / TPB;  // pairs per thread

__global__ __launch_bounds__(TPB) void k_gram(const double *__restrict__ V, i64 ld, int c, i64 n,
                                              const short2 *__restrict__ pairs, int npairs,
                                              double *__restrict__ slab) {
    __shared__ double tile[GROWS][GCMAX + 1];
    double acc[GPPT];
#pragma unroll
    for (int q = 0; q < GPPT; ++q) acc[q] = 0.0;
    const i64 nchunks = (n + GROWS - 1) / GROWS;
    for (i64 ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
        const i64 r0 = ch * GROWS;
        for (int t = threadIdx.x; t < GROWS * c; t += TPB) {
            const int col = t / GROWS, r = t % GROWS;
            const i64 e = r0 + r;
            tile[r][col] = (e < n) ? V[(i64)col * ld + e] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < GPPT; ++q) {
            const int p = threadIdx.x + q * TPB;
            if (p < npairs) {
                const short2 ab = pairs[p];
                double s = 0.0;
#pragma unroll 8
                for (int r = 0; r < GROWS; ++r) s = s + tile[r][ab.x] * tile[r][ab.y];
                acc[q] = acc[q] + s;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < GPPT; ++q) {
        const int p = threadIdx.x + q * TPB;
        if (p < npairs) slab[(i64)blockIdx.x * npairs + p] = acc[q];
    }
}

__global__ __launch_bounds__(TPB) void k_gram_reduce(const double *__restrict__ slab, int nblk, int npairs,
                                                     double *__restrict__ out) {
    const int p = blockIdx.x * TPB + threadIdx.x;
    if (p >= npairs) return;
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s = s + slab[(i64)b * npairs + p];
    out[p] = s;
}

// --------------------------------------------------------------------------
// Reference-order dots for the orthogonality diagnostics (gmres_mgsr.f90:414-420,
// gmres_hh.f90:568-593).  Fortran dot_product is ONE running sum
// h = h + a(k)*b(k), k = 1..n.  Both diagnostics measure rounding noise, and
// the reference's figure is dominated by that running sum's own rounding, so
// the device evaluates them the same way: one lane per dot, k in order,
// multiply then add (-ffp-contract=off) -- bit-identical to the reference's
// formula on the same basis.  n dependent adds per lane: slow by design, run
// once per solve (the tree-reduced k_gram is the fast alternative).
// --------------------------------------------------------------------------
constexpr int SQ_B = 8;  // double2 per column in flight per lane

__device__ __forceinline__ double seq_dot(const double *__restrict__ a, const double *__restrict__ b, i64 n) {
    const double2 *a2 = reinterpret_cast<const double2 *>(a), *b2 = reinterpret_cast<const double2 *>(b);
    const i64 n2 = n >> 1;
    double h = 0.0;
    i64 e = 0;
    for (; e + SQ_B <= n2; e += SQ_B) {
        double2 x[SQ_B], y[SQ_B];
#pragma unroll
        for (int u = 0; u < SQ_B; ++u) {
            x[u] = a2[e + u];
            y[u] = b2[e + u];
        }
#pragma unroll
        for (int u = 0; u < SQ_B; ++u) {
            h = h + x[u].x * y[u].x;
            h = h + x[u].y * y[u].y;
        }
    }
    for (i64 k = 2 * e; k < n; ++k) h = h + a[k] * b[k];
    return h;
}

// out[p] = dot_product(V(:,pairs[p].x+1), V(:,pairs[p].y+1)), one lane per pair.
__global__ __launch_bounds__(64) void k_seqdot_pairs(const double *__restrict__ V, i64 ld, i64 n,
                                                     const short2 *__restrict__ pairs, int npairs,
                                                     double *__restrict__ out) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= npairs) return;
    const short2 ab = pairs[p];
    out[p] = seq_dot(V + (i64)ab.x * ld, V + (i64)ab.y * ld, n);
}

// calculate_verr's rebuild V(:,i) = P_1..P_i e_i, level s of the reflection
// order (:581-585: for chain i, j = i, i-1, .., 1): chain i >= s applies
// reflector j = i - s.  k_hh_rebuild_dot: d[i] = dot_product(V(:,i), P(:,j));
// k_hh_rebuild_upd: V(:,i) = V(:,i) - 2.0*P(:,j)*d[i] (blockIdx.y = j).
__global__ __launch_bounds__(64) void k_hh_rebuild_dot(const double *__restrict__ Vb, const double *__restrict__ P,
                                                       i64 ld, i64 n, int s, int n_out, double *__restrict__ d) {
    const int i = s + blockIdx.x * 64 + threadIdx.x;
    if (i >= n_out) return;
    d[i] = seq_dot(Vb + (i64)i * ld, P + (i64)(i - s) * ld, n);
}

__global__ __launch_bounds__(TPB) void k_hh_rebuild_upd(double *__restrict__ Vb, const double *__restrict__ P,
                                                        i64 ld, i64 n, int s, const double *__restrict__ d) {
    const int j = blockIdx.y, i = s + j;
    double *__restrict__ v = Vb + (i64)i * ld;
    const double *__restrict__ p = P + (i64)j * ld;
    const double dd = d[i];
    const i64 stride = (i64)gridDim.x * TPB;
    for (i64 e = (i64)blockIdx.x * TPB + threadIdx.x; e < n; e += stride) v[e] = v[e] - 2.0 * p[e] * dd;
}

}  // namespace gk

namespace gk {

// All-reduce / broadcast of a short vector, one workgroup per rank.
//   XS_SLAB : buf[0..count) is a partial slab; each rank reduces its own slab in a
//             fixed order, the ranks' totals are summed in rank order, and the
//             slab becomes {total, 0, ..., 0} (its consumer re-reduces it).
//   XS_VEC  : element-wise sum over ranks in rank order, count <= XS_MAXV.
//   XS_BCAST: buf = root's buf, count <= XS_MAXV.
// The rank-order sum is the same instruction sequence on every rank, so the
// replicated host loops see bit-identical scalars.
// seqbase != nullptr (a launch replayed from a captured graph): the sequence
// number is *seqbase + seq, the host having set *seqbase on the stream before the
// replay -- a graph's kernel arguments are fixed, an exchange's number is not.
template <int MODE>
__global__ __launch_bounds__(TPB) void k_xchg(double *__restrict__ buf, int count, XsPeers peers, int nranks,
                                               int rank, unsigned seq_arg, const unsigned *seqbase, int root,
                                               int *err, u64 timeout) {
    const unsigned seq = seqbase != nullptr ? *seqbase + seq_arg : seq_arg;
    __shared__ double sm[WAVES];
    __shared__ double pay[XS_MAXV];
    __shared__ unsigned rv[XS_MAXR * XS_MAXV * 2];
    __shared__ int bad;
    const int plen = MODE == XS_SLAB ? 1 : count;
    if (threadIdx.x == 0) bad = xs_flag(err);
    if (MODE == XS_SLAB) {
        const double s = reduce_slab(buf, count, sm);  // synchronises the block
        if (threadIdx.x == 0) pay[0] = s;
    } else {
        for (int k = threadIdx.x; k < plen; k += TPB) pay[k] = buf[k];
    }
    __syncthreads();
    const unsigned par = seq & 1u;
    const int tot = nranks * plen * 2;
    if (!bad) {
        for (int t = threadIdx.x; t < tot; t += TPB) {
            const int half = t & 1, k = (t >> 1) % plen, dst = (t >> 1) / plen;
            const u64 bits = (u64)__double_as_longlong(pay[k]);
            xs_put(peers.p[dst] + (((i64)par * XS_MAXR + rank) * XS_MAXV + k) * 2 + half, seq,
                   half ? (unsigned)(bits >> 32) : (unsigned)bits);
        }
        const u64 deadline = wall_clock64() + timeout;
        const u64 *mine = peers.p[rank];
        bool ok = true;
        for (int t = threadIdx.x; t < tot && ok; t += TPB) {
            const int half = t & 1, k = (t >> 1) % plen, src = (t >> 1) / plen;
            unsigned d = 0;
            const int g = xs_get(mine + (((i64)par * XS_MAXR + src) * XS_MAXV + k) * 2 + half, seq, deadline, &d, err);
            ok = g == XG_OK;
            rv[(src * XS_MAXV + k) * 2 + half] = d;
            if (g == XG_LATE) xs_fail(err, MODE == XS_BCAST ? XSE_BCAST : XSE_XCHG, src);
        }
        if (!ok) bad = 1;
    }
    __syncthreads();
    if (bad) {
        for (int k = threadIdx.x; k < count; k += TPB) buf[k] = __builtin_nan("");
        return;
    }
    auto val = [&](int r, int k) {
        const u64 lo = rv[(r * XS_MAXV + k) * 2], hi = rv[(r * XS_MAXV + k) * 2 + 1];
        return __longlong_as_double((long long)((hi << 32) | lo));
    };
    for (int k = threadIdx.x; k < count; k += TPB) {
        if (MODE == XS_SLAB && k > 0) {
            buf[k] = 0.0;
            continue;
        }
        double s;
        if (MODE == XS_BCAST) {
            s = val(root, k);
        } else {
            s = val(0, k);
            for (int r = 1; r < nranks; ++r) s = s + val(r, k);
        }
        buf[k] = s;
    }
}

// Halo lines through the same regions: my first grid line goes to rank-1
// (its side 1), my last to rank+1 (its side 0); then wait for mine and decode
// them into hlo / hhi, the buffers the stencil reads.  One thread per point.
constexpr int XS_HALO_LINES = CF_HMAX;  // deepest halo (the temporal-blocked Chebyshev passes)

__global__ __launch_bounds__(TPB) void k_xhalo(const double *__restrict__ vec, int N, int nlines, int nl,
                                               XsPeers peers, int nranks, int rank, unsigned seq,
                                               double *__restrict__ hlo, double *__restrict__ hhi, int *err,
                                               u64 timeout) {
    // nl grid lines each way: my first nl lines go to rank-1, my last nl to rank+1
    const i64 e = (i64)blockIdx.x * TPB + threadIdx.x;
    if (e >= (i64)nl * N) return;
    const bool lo = rank > 0, hi = rank < nranks - 1;
    const unsigned par = seq & 1u;
    auto slot = [&](u64 *base, int side) {
        return base + gk::XS_RED_WORDS + (((i64)par * 2 + side) * ((i64)XS_HALO_LINES * N) + e) * 2;
    };
    if (xs_flag(err)) {
        if (lo) hlo[e] = __builtin_nan("");
        if (hi) hhi[e] = __builtin_nan("");
        return;
    }
    if (lo) {
        const u64 bits = (u64)__double_as_longlong(vec[e]);
        u64 *q = slot(peers.p[rank - 1], 1);
        xs_put(q, seq, (unsigned)bits);
        xs_put(q + 1, seq, (unsigned)(bits >> 32));
    }
    if (hi) {
        const u64 bits = (u64)__double_as_longlong(vec[(i64)(nlines - nl) * N + e]);
        u64 *q = slot(peers.p[rank + 1], 0);
        xs_put(q, seq, (unsigned)bits);
        xs_put(q + 1, seq, (unsigned)(bits >> 32));
    }
    const u64 deadline = wall_clock64() + timeout;
    u64 *mine = peers.p[rank];
    for (int side = 0; side < 2; ++side) {
        if (side == 0 ? !lo : !hi) continue;
        const u64 *q = slot(mine, side);
        unsigned a = 0, b = 0;
        double v = __builtin_nan("");
        int g = xs_get(q, seq, deadline, &a, err);
        if (g == XG_OK) g = xs_get(q + 1, seq, deadline, &b, err);
        if (g == XG_OK)
            v = __longlong_as_double((long long)(((u64)b << 32) | a));
        else if (g == XG_LATE)
            xs_fail(err, XSE_HALO, side == 0 ? rank - 1 : rank + 1);
        (side == 0 ? hlo : hhi)[e] = v;
    }
}

// R2: register-resident double2 per data thread (w, and the running column);
// L2: LDS-resident double2 of w per data thread (its two columns stream);
// PF: the next column is loaded into a third register array before the wait;
// CW: wave 0 holds no data and only runs the exchange, so its polls never wait
//     behind prefetch loads (vmcnt retires in issue order).
template <int R2, int L2, bool PF, bool NT, bool CW, int MODE>
__global__ __launch_bounds__(RT, 2) void k_mgs_res(ResArgs a) {
    extern __shared__ double2 lw[];  // L2 > 0: [L2][DT] LDS-resident part of w
    __shared__ double sm[RWAVES];
    __shared__ double bc[1];
    __shared__ int okf;
    __shared__ double hsh[RHMAX + 1];
    constexpr int RB = PF ? R2 : 1;
    constexpr int DT = CW ? RT - 64 : RT;  // data threads per workgroup
    const int t = threadIdx.x;
    const bool data = !CW || t >= 64;
    const int td = CW ? t - 64 : t;
    constexpr int mode = MODE;
    const int j = a.j, np = res_np(mode, j);
    const i64 n2 = a.n >> 1, ld2 = a.ld >> 1;
    const i64 tail0 = mode == RES_HH_UP ? a.tail0 : 0;
    // Resident layout in chunks of DT double2 (data thread td holds element td
    // of each): registers hold chunks b*R2 + k (k < R2), LDS chunks G*R2 + b*L2
    // + k (k < L2); a chunk is resident when it lies below nres2 (a multiple of
    // DT), so the test is uniform and every address is a uniform base + td*16.
    // [nres2, n2) streams through w in HBM as in k_proj.
    const i64 nch = a.nres2 / DT;
    const i64 c0 = (i64)blockIdx.x * a.r2e, cend = c0 + a.r2e < nch ? c0 + a.r2e : nch;
    const i64 l0 = (i64)gridDim.x * a.r2e + (i64)blockIdx.x * a.l2e, lend = l0 + a.l2e < nch ? l0 + a.l2e : nch;
    const double2 *__restrict__ V2 = reinterpret_cast<const double2 *>(a.V);
    double2 *__restrict__ W2 = reinterpret_cast<double2 *>(a.w);
    auto colchunk = [&](int col, i64 c) { return V2 + (i64)col * ld2 + c * DT; };
    double2 wr[R2], xa[R2], xb[RB];
#pragma unroll
    for (int k = 0; k < R2; ++k) {  // zeros past nres2: they add exact zeros to every dot
        wr[k] = xa[k] = double2{0.0, 0.0};
        if constexpr (PF) xb[k] = double2{0.0, 0.0};
        if (data && c0 + k < cend) {
            wr[k] = W2[(c0 + k) * DT + td];
            xa[k] = colchunk(res_col(mode, j, 0), c0 + k)[td];              // AXPY partner of projection 0
            if constexpr (PF) xb[k] = colchunk(res_col(mode, j, 1), c0 + k)[td];  // its dot partner
        }
    }
    if constexpr (L2 > 0) {
        for (int k = 0; k < L2; ++k)
            if (data && l0 + k < lend) lw[k * DT + td] = W2[(l0 + k) * DT + td];
    }
    const i64 sstride = (i64)gridDim.x * DT;
    const i64 sbase = a.nres2 + (i64)res_stream_wg() * DT + td;
    ResClock clk;
    clk.start(a.stamps);
    int xi = 0;  // exchange index
    double h;
    bool ok = true;
    if (mode == RES_HH_DOWN) {  // the pre-dot <v, V_col(0)> (xa holds V_col(0))
        const int q = res_col(mode, j, 0);
        const double2 *__restrict__ B2 = V2 + (i64)q * ld2;
        double acc = 0.0;
        if (a.unit_known) {  // <e_u, P_q> = P_q(u): the one nonzero product, as the full sum gives it
            if (blockIdx.x == 0 && t == 0 && a.unit_e >= 0) acc = a.V[(i64)q * a.ld + a.unit_e];
        } else if (data) {
#pragma unroll
            for (int k = 0; k < R2; ++k) {
                acc = acc + wr[k].x * xa[k].x;
                acc = acc + wr[k].y * xa[k].y;
            }
            if constexpr (L2 > 0) {
                for (int k = 0; k < L2; ++k)
                    if (l0 + k < lend) {
                        const double2 wv = lw[k * DT + td], bv = ldv<NT>(B2 + (l0 + k) * DT + td);
                        acc = acc + wv.x * bv.x;
                        acc = acc + wv.y * bv.y;
                    }
            }
            for (i64 e = sbase; e < n2; e += sstride) {
                const double2 wv = W2[e], bv = ldv<NT>(B2 + e);
                acc = acc + wv.x * bv.x;
                acc = acc + wv.y * bv.y;
            }
            if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && td == 0) acc = acc + a.w[a.n - 1] * a.V[(i64)q * a.ld + a.n - 1];
        }
        acc = wave_sum(acc);
        if ((t & 63) == 0) sm[t >> 6] = acc;
        __syncthreads();
        if (t < 64) res_exchange<RWAVES, MODE == RES_MGS, RES_POLL_SLEEP_SMALL>(a, xi, sm, bc, &okf);
        __syncthreads();
        ++xi;
        h = bc[0];
        ok = okf != 0;
    } else {
        double s = 0.0;
        for (int k = t; k < a.npin; k += RT) s += a.pin[k];
        h = block_sum_rt(s, sm);
        ok = res_pin_fold(a, h, bc, &okf);
    }
    // Projection p: i = p mod j, AXPY w -= h V_i (h = the dot of p), then the
    // dot of projection p+1 with V_q, q = (p+1) mod j -- or ||w||^2 after the
    // last one.  X holds V_i; PF: Y holds V_q (prefetched), and X <- the dot
    // partner of p+1 is loaded before the wait.
    auto proj = [&](int p, auto &X, auto &Y) -> bool {
        const int i = res_col(mode, j, p);
        const bool last = p == np - 1;
        const int q = res_col(mode, j, p + 1);
        const int kind = !last ? RK_DOT : (mode == RES_HH_DOWN ? RK_NONE : RK_NORM);
        if (mode == RES_MGS && blockIdx.x == 0 && t == 0) hsh[i] = (p < j ? 0.0 : hsh[i]) + h;  // H(i,j) (+)= h
        const double ch = mode == RES_MGS ? h : a.coef * h;
        double acc = 0.0;
        if (data) {
#pragma unroll
            for (int k = 0; k < R2; ++k) {
                wr[k].x = wr[k].x - ch * X[k].x;
                wr[k].y = wr[k].y - ch * X[k].y;
            }
            if (kind == RK_NONE) {
            } else if (last) {
#pragma unroll
                for (int k = 0; k < R2; ++k)
                    sq_acc(acc, wr[k], (c0 + k) * DT + td, tail0, mode == RES_HH_UP && c0 + k == 0);
            } else if constexpr (PF) {
#pragma unroll
                for (int k = 0; k < R2; ++k) {
                    acc = acc + wr[k].x * Y[k].x;
                    acc = acc + wr[k].y * Y[k].y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < R2; ++k)
                    if (c0 + k < cend) X[k] = ldv<NT>(colchunk(q, c0 + k) + td);
#pragma unroll
                for (int k = 0; k < R2; ++k) {
                    acc = acc + wr[k].x * X[k].x;
                    acc = acc + wr[k].y * X[k].y;
                }
            }
            const double2 *__restrict__ A2 = V2 + (i64)i * ld2;
            const double2 *__restrict__ B2 = V2 + (i64)q * ld2;
            if constexpr (L2 > 0) {  // w in LDS, its two columns stream: 16 B/unknown
                for (int k = 0; k < L2; k += 2) {
                    double2 wv[2], av[2], bv[2];
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const i64 c = l0 + k + u;
                        if (k + u < L2 && c < lend) {
                            wv[u] = lw[(k + u) * DT + td];
                            av[u] = ldv<NT>(A2 + c * DT + td);
                            if (!last) bv[u] = a.qdef ? ldv<false>(B2 + c * DT + td) : ldv<NT>(B2 + c * DT + td);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const i64 c = l0 + k + u;
                        if (k + u < L2 && c < lend) {
                            wv[u].x = wv[u].x - ch * av[u].x;
                            wv[u].y = wv[u].y - ch * av[u].y;
                            lw[(k + u) * DT + td] = wv[u];
                            if (kind == RK_NONE) {
                            } else if (last) {
                                sq_acc(acc, wv[u], c * DT + td, tail0, mode == RES_HH_UP && c == 0);
                            } else {
                                acc = acc + wv[u].x * bv[u].x;
                                acc = acc + wv[u].y * bv[u].y;
                            }
                        }
                    }
                }
            }
            for (i64 e0 = sbase; e0 < n2; e0 += 2 * sstride) {  // streamed part: 32 B/unknown
                double2 wv[2], av[2], bv[2];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const i64 e = e0 + u * sstride;
                    if (e < n2) {
                        wv[u] = W2[e];
                        av[u] = ldv<NT>(A2 + e);
                        if (!last) bv[u] = a.qdef ? ldv<false>(B2 + e) : ldv<NT>(B2 + e);
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const i64 e = e0 + u * sstride;
                    if (e < n2) {
                        wv[u].x = wv[u].x - ch * av[u].x;
                        wv[u].y = wv[u].y - ch * av[u].y;
                        W2[e] = wv[u];
                        if (kind == RK_NONE) {
                        } else if (last) {
                            sq_acc(acc, wv[u], e, tail0, mode == RES_HH_UP && 2 * a.nres2 < tail0);
                        } else {
                            acc = acc + wv[u].x * bv[u].x;
                            acc = acc + wv[u].y * bv[u].y;
                        }
                    }
                }
            }
            if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && td == 0) {  // odd-length tail element
                const i64 e = a.n - 1;
                const double x = a.w[e] - ch * a.V[(i64)i * a.ld + e];
                a.w[e] = x;
                if (kind == RK_DOT) acc = acc + x * a.V[(i64)q * a.ld + e];
                if (kind == RK_NORM && e >= tail0) acc = acc + x * x;
            }
        }
        if (kind == RK_NONE) return true;
        clk.passed(a.stamps);
        acc = wave_sum(acc);
        if ((t & 63) == 0) sm[t >> 6] = acc;
        __syncthreads();
        if constexpr (PF) {
            if (data && p + 2 < np) {  // the dot partner of projection p+1, in flight during the exchange
                const int q2 = res_col(mode, j, p + 2);
#pragma unroll
                for (int k = 0; k < R2; ++k)
                    if (c0 + k < cend) X[k] = ldv<NT>(colchunk(q2, c0 + k) + td);
            }
        }
        if (t < 64) res_exchange<RWAVES, MODE == RES_MGS, RES_POLL_SLEEP_SMALL>(a, xi, sm, bc, &okf);
        __syncthreads();
        ++xi;
        h = bc[0];
        clk.waited(a.stamps);
        return okf != 0;
    };
    if constexpr (PF) {
        for (int p = 0; p < np && ok; p += 2) {
            ok = proj(p, xa, xb);
            if (ok && p + 1 < np) ok = proj(p + 1, xb, xa);
        }
    } else {
        for (int p = 0; p < np && ok; ++p) ok = proj(p, xa, xb);
    }
    if (!ok) return;  // uniform per workgroup; *err is set
    if (mode != RES_MGS) {  // reflections: the resident part of w back to HBM
        if (data) {
#pragma unroll
            for (int k = 0; k < R2; ++k)
                if (c0 + k < cend) W2[(c0 + k) * DT + td] = wr[k];
            if constexpr (L2 > 0) {
                for (int k = 0; k < L2; ++k)
                    if (l0 + k < lend) W2[(l0 + k) * DT + td] = lw[k * DT + td];
            }
        }
        if (mode == RES_HH_UP && blockIdx.x == 0 && t == 0) a.hs[0] = h;  // ||w(j+1:n)||^2
        clk.finish(a.stamps, mode);
        return;
    }
    // h = ||w|| ; V(:,j+1) = w / h  (h == 0: zeros, as k_scale)
    const double hn = sqrt(h);
    double2 *__restrict__ O2 = reinterpret_cast<double2 *>(a.vout);
    if (data) {
#pragma unroll
        for (int k = 0; k < R2; ++k)
            if (c0 + k < cend)
                O2[(c0 + k) * DT + td] = hn != 0.0 ? double2{wr[k].x / hn, wr[k].y / hn} : double2{0.0, 0.0};
        if constexpr (L2 > 0) {
            for (int k = 0; k < L2; ++k)
                if (l0 + k < lend) {
                    const double2 v = lw[k * DT + td];
                    O2[(l0 + k) * DT + td] = hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0};
                }
        }
        for (i64 e = sbase; e < n2; e += sstride) {
            const double2 v = W2[e];
            O2[e] = hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0};
        }
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && td == 0) a.vout[a.n - 1] = hn != 0.0 ? a.w[a.n - 1] / hn : 0.0;
    }
    clk.finish(a.stamps, mode);
    if (blockIdx.x == 0) {  // H(1:j+1, j) to the device column and the mapped host mirror
        __syncthreads();
        for (int k = t; k < j; k += RT) {
            a.hs[k] = hsh[k];
            a.hcopy[k] = hsh[k];
        }
        if (t == 0) {
            a.hs[j] = hn;
            a.hcopy[j] = hn;
        }
    }
}

// --------------------------------------------------------------------------
// Resident MGS-R step, w-only variant for large slabs: ONE wave per SIMD
// (256-thread workgroups, one per CU) so each lane can hold ~400 registers
// (VGPRs + AGPRs of the unified file), and they hold w only -- RW double2 per
// thread in registers and LW more in LDS.  Per projection a resident unknown
// moves 16 B (its two Krylov columns) instead of 32; the running column V_q is
// loaded with the default policy, so it is still in the Infinity Cache when
// it is read again as V_i by the next projection (V_i itself non-temporal).
// Same exchange, same arithmetic as k_mgs_res.
// --------------------------------------------------------------------------
constexpr int WT = 256;  // threads per workgroup (4 waves, one per SIMD)
#ifndef GK_RES_WB
#define GK_RES_WB 8
#endif
constexpr int WB = GK_RES_WB;        // double2 per column per batch in flight per thread
#ifndef GK_RES_WB_HH
#define GK_RES_WB_HH 6
#endif
constexpr int WB_HH = GK_RES_WB_HH;  // the reflection chains' batch (their RW is larger)
// (Round 5 removed measured-slower A/B paths from this kernel: XPF -- the next
// pass's first batch loaded before the exchange wait, 42.4 -> 46.9 us per projection
// at RW 80; ROT -- every workgroup's chunk range moved to its neighbour's, the even
// XCDs lagged as before (profiles/r02/res_trace_rotation.jsonl); REV -- the LDS part
// walked in alternating halves, 40.89 -> 44.05 us (profiles/r04/ab_rev_wb_r04i.jsonl);
// STEN -- the stencil formed in the prologue, 245.9 -> 236.2 it/s
// (profiles/r03/ab_res_sten_r03k.jsonl).  DESIGN.md 3.1 keeps the numbers.)
// TOUCH: while wave 0 runs a pass's all-gather, waves 1..3 pull the first
// TOUCH chunks (4 KiB each) of the NEXT pass's dot column -- the one that
// comes from HBM -- into L2 with one dword load per 128-B line into a sink
// register, so the memory pipe works through the wait.  0 = off; A/B at
// 4096^2 with one granule array (profiles/r02/ab_touch*.jsonl): 8 +-0, 16 -1.5 %,
// 32 -2.2 % per projection (MGS-R 42.4 -> 41.7 us, HH 43.2 -> 42.2 us), 48 / 64
// slower (the touched lines outgrow the 128 KiB per-CU share of L2); the depths
// now in use are below.
#ifndef GK_RES_TOUCH
#define GK_RES_TOUCH 24
#endif
constexpr int TOUCH = GK_RES_TOUCH;
#ifndef GK_RES_TOUCH_MGS
#define GK_RES_TOUCH_MGS 28
#endif
// Touched chunks per workgroup: MGS-R launches (paced touches) TOUCH_MGS, the
// reflection chains (burst) TOUCH.  A/B at 4096^2 after the granule replicas and the
// pacing (profiles/r02/ab_touch_depth_paced.jsonl, ab_touch_depth_mode.jsonl): MGS-R
// 16 / 20 / 24 / 28 / 32 / 40 / 48 -> 41.47 / 41.08 / 41.04 / 40.78 / 41.17 / 42.7 / 43.6
// us per projection (two boxes); Householder 24 vs 32: 40.76 vs 41.96 us per reflection.
constexpr int TOUCH_MGS = GK_RES_TOUCH_MGS;
// Load policy of the dot column V_q of a pass (A/B knob): 0 = default, so the
// column is still in the Infinity Cache when the next pass reads it as its
// AXPY column V_i; 1 = non-temporal like V_i (every column comes from HBM).
#ifndef GK_RES_QNT
#define GK_RES_QNT 0
#endif
constexpr bool RES_QNT = GK_RES_QNT != 0;
#ifndef GK_RES_TOUCH_PACE
#define GK_RES_TOUCH_PACE 24
#endif
// TOUCH_PACE > 0 (MGS-R step launches): the touch loads go out one per lane per
// round, s_sleep TOUCH_PACE between rounds, and stop once wave 0 holds the
// exchange's total -- a late workgroup (short wait) then has few touches left to
// drain before its next pass (the trace: a workgroup late at exchange p ran its
// next pass 0.5 us longer).  A/B at 4096^2 (profiles/r02/ab_touch_pace.jsonl):
// MGS-R 41.55 -> 41.28 us per projection at 24 (8: 41.37); the reflection chains
// run slower with it (pace 8: 41.9 -> 42.7 us), so they keep the all-at-once touch.
// 0: all issued at once (drained after the exchange).  Interleaving the resident
// chunks over the grid (chunk b + kG instead of a contiguous range per workgroup)
// was measured too: 41.5 -> 48.0 us (DRAM row locality lost).
constexpr int TOUCH_PACE = GK_RES_TOUCH_PACE;
#ifndef GK_RES_TOUCH_PACE_HH
#define GK_RES_TOUCH_PACE_HH 0
#endif
// the reflection chains' pacing (0 = burst); re-measured after the depth / residency
// re-tune (profiles/r02/ab_pace_retune.jsonl): 8 / 24 -> 41.06 / 41.1 vs 40.57 us burst
constexpr int TOUCH_PACE_HH = GK_RES_TOUCH_PACE_HH;

template <int RW, int LW, int MODE, int WBT = WB>
__global__ __launch_bounds__(WT, 1) void k_mgs_wres(ResArgs a) {
    extern __shared__ double2 lw[];  // [LW][WT]
    __shared__ double sm[WT / 64];
    __shared__ double bc[1];
    __shared__ int okf;
    __shared__ int xdone;  // PACE: the exchange in progress has completed
    // H(1:j, j): WO_HMAX entries, not RHMAX + 1 -- the MGS step's 39 LDS chunks of w leave
    // 4,048 bytes of the CU's 160 KiB (res_plan keeps m + 1 <= WO_HMAX on this kernel)
    __shared__ double hsh[MODE == RES_MGS ? WO_HMAX : 1];
    const int t = threadIdx.x;
    constexpr int mode = MODE;
    constexpr int PACE = MODE == RES_MGS ? TOUCH_PACE : TOUCH_PACE_HH;
    constexpr int TCH = MODE == RES_MGS ? TOUCH_MGS : TOUCH;  // touched chunks per workgroup
    const int j = a.j, np = res_np(mode, j);
    const i64 n2 = a.n >> 1, ld2 = a.ld >> 1;
    const i64 nch = a.nres2 / WT;
    const i64 bq = blockIdx.x;  // chunk range of this workgroup
    const i64 c0 = bq * a.r2e, cend = c0 + a.r2e < nch ? c0 + a.r2e : nch;
    const i64 l0 = (i64)gridDim.x * a.r2e + bq * a.l2e, lend = l0 + a.l2e < nch ? l0 + a.l2e : nch;
    const i64 tail0 = mode == RES_HH_UP ? a.tail0 : 0;
    const double2 *__restrict__ V2 = reinterpret_cast<const double2 *>(a.V);
    double2 *__restrict__ W2 = reinterpret_cast<double2 *>(a.w);
    ResClock clk;
    clk.start(a.stamps);
    int touch_sink = 0;
    const i64 sstride = (i64)gridDim.x * WT;
    const i64 sbase = a.nres2 + (i64)res_stream_wg() * WT + t;
    double2 wr[RW];
    if (mode == RES_HH_DOWN && a.unit_init) {
        // w = e_u built in place (gmres_hh.f90:257-264): no k_set_unit launch, no read
        // of w; the streamed part is written by the thread that streams it later
        const i64 u = a.unit_e;  // local index of the 1.0, -1 on other ranks
        auto unit2 = [&](i64 e2) { return double2{2 * e2 == u ? 1.0 : 0.0, 2 * e2 + 1 == u ? 1.0 : 0.0}; };
#pragma unroll
        for (int k = 0; k < RW; ++k) wr[k] = (c0 + k < cend) ? unit2((c0 + k) * WT + t) : double2{0.0, 0.0};
        for (int k = 0; k < LW; ++k)
            if (l0 + k < lend) lw[k * WT + t] = unit2((l0 + k) * WT + t);
        for (i64 e = sbase; e < n2; e += sstride) W2[e] = unit2(e);
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) a.w[a.n - 1] = (a.n - 1 == u) ? 1.0 : 0.0;
    } else {
#pragma unroll
        for (int k = 0; k < RW; ++k) wr[k] = (c0 + k < cend) ? W2[(c0 + k) * WT + t] : double2{0.0, 0.0};
        for (int k = 0; k < LW; ++k)
            if (l0 + k < lend) lw[k * WT + t] = W2[(l0 + k) * WT + t];
    }
    // acc += the closing reduction of element pair e2 (local double2 index)
    auto red = [&](double &acc, const double2 &v, const double2 &b, int kind, i64 e2, bool chk) {
        if (kind == RK_DOT) {
            acc = acc + v.x * b.x;
            acc = acc + v.y * b.y;
        } else if (kind == RK_NORM) {
            sq_acc(acc, v, e2, tail0, chk);
        }
    };
    // One pass over the slab: w -= ch V_i, then the reduction `kind`
    // (<w, V_q>, ||w(tail0:)||^2, or none).  Returns this thread's partial.
    auto pass = [&](double ch, int i, int q, int kind) -> double {
        const double2 *__restrict__ A2 = V2 + (i64)i * ld2;
        const double2 *__restrict__ B2 = V2 + (i64)q * ld2;
        const bool dot = kind == RK_DOT;
        double acc = 0.0;
        // registers: batches of WBT chunks, both columns in flight (k0 a constant once unrolled)
        auto rbatch = [&](const int k0) {
            double2 av[WBT], bv[WBT];
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const i64 c = c0 + k0 + u;
                if (k0 + u < RW && c < cend) {
                    av[u] = ldv<true>(A2 + c * WT + t);
                    if (dot) bv[u] = ldv<RES_QNT>(B2 + c * WT + t);
                }
            }
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                if (k < RW && c0 + k < cend) {
                    wr[k].x = wr[k].x - ch * av[u].x;
                    wr[k].y = wr[k].y - ch * av[u].y;
                    red(acc, wr[k], bv[u], kind, (c0 + k) * WT + t, mode == RES_HH_UP && c0 + k == 0);
                }
            }
        };
        // LDS: the same, w from / to LDS
        auto lbatch = [&](const int k0, const int kend) {
            double2 av[WBT], bv[WBT];
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const i64 c = l0 + k0 + u;
                if (k0 + u < kend && c < lend) {
                    av[u] = ldv<true>(A2 + c * WT + t);
                    if (dot) bv[u] = ldv<RES_QNT>(B2 + c * WT + t);
                }
            }
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                if (k < kend && l0 + k < lend) {
                    double2 wv = lw[k * WT + t];
                    wv.x = wv.x - ch * av[u].x;
                    wv.y = wv.y - ch * av[u].y;
                    lw[k * WT + t] = wv;
                    red(acc, wv, bv[u], kind, (l0 + k) * WT + t, mode == RES_HH_UP && l0 + k == 0);
                }
            }
        };
#pragma unroll
        for (int k0 = 0; k0 < RW; k0 += WBT) rbatch(k0);
        for (int k0 = 0; k0 < LW; k0 += WBT) lbatch(k0, LW);
        for (i64 e0 = sbase; e0 < n2; e0 += 2 * sstride) {  // streamed part: 32 B/unknown
            double2 wv[2], av[2], bv[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const i64 e = e0 + u * sstride;
                if (e < n2) {
                    wv[u] = W2[e];
                    av[u] = ldv<true>(A2 + e);
                    if (dot) bv[u] = ldv<RES_QNT>(B2 + e);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const i64 e = e0 + u * sstride;
                if (e < n2) {
                    wv[u].x = wv[u].x - ch * av[u].x;
                    wv[u].y = wv[u].y - ch * av[u].y;
                    W2[e] = wv[u];
                    red(acc, wv[u], bv[u], kind, e, mode == RES_HH_UP && 2 * a.nres2 < tail0);
                }
            }
        }
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) {  // odd-length tail element
            const i64 e = a.n - 1;
            const double x = a.w[e] - ch * a.V[(i64)i * a.ld + e];
            a.w[e] = x;
            if (kind == RK_DOT) acc = acc + x * a.V[(i64)q * a.ld + e];
            if (kind == RK_NORM && e >= tail0) acc = acc + x * x;
        }
        return acc;
    };
    // all-gather of the partials: the same h in every workgroup (and rank)
    int xi = 0;
    auto reduce = [&](double acc, double &h, int touch_col) -> bool {
        clk.passed(a.stamps);
        acc = wave_sum(acc);
        if ((t & 63) == 0) sm[t >> 6] = acc;
        if (PACE > 0 && t == 0) xdone = 0;
        __syncthreads();
        if (t < 64) {
            res_exchange<WT / 64, MODE == RES_MGS, RES_POLL_SLEEP>(a, xi, sm, bc, &okf);
            if (PACE > 0 && t == 0) *(volatile int *)&xdone = 1;
        } else if constexpr (TCH > 0) {
            if (touch_col >= 0) {
                // lines [0, 32*TCH) of the workgroup's register-resident part of
                // the column (contiguous from chunk c0); all loads land in one sink
                // register, drained below before anything can reuse it
                const i64 r0 = c0, r1 = cend;
                const i64 lines = (i64)32 * (r1 - r0 < TCH ? (r1 - r0 > 0 ? r1 - r0 : 0) : TCH);
                const char *base = reinterpret_cast<const char *>(V2 + (i64)touch_col * ld2 + r0 * WT);
                for (i64 l = t - 64; l < lines; l += WT - 64) {
                    if constexpr (PACE > 0) {
                        if (*(volatile int *)&xdone) break;  // wave-uniform: one LDS word
                    }
                    const char *ptr = base + l * 128;
                    asm volatile("global_load_dword %0, %1, off" : "+v"(touch_sink) : "v"(ptr) : "memory");
                    if constexpr (PACE > 0) __builtin_amdgcn_s_sleep(PACE);
                }
            }
        }
        __syncthreads();
        if constexpr (TCH > 0) asm volatile("s_waitcnt vmcnt(0)" : : "v"(touch_sink) : "memory");
        ++xi;
        h = bc[0];
        clk.waited(a.stamps);
        return okf != 0;
    };
    // The last pass of a reflection chain reduces nothing: RES_HH_UP's closing
    // ||w(j+1:n)||^2 is taken after the loop, from the registers w is written
    // back from, so the pass code of all three modes is the same (the tail test
    // inside the unrolled loop made the UP pass 28 % slower: 45.9 vs 35.7 us).
    auto kind_of = [&](int p) { return p < np - 1 ? RK_DOT : (mode == RES_MGS ? RK_NORM : RK_NONE); };
    double h;
    bool ok = true;
    if (mode == RES_HH_DOWN) {
        // the pre-dot as an AXPY pass with h = 0 (w - 0 V = w): a dot-only copy of the
        // unrolled register loop would not fit the register file
        const int q = res_col(mode, j, 0);
        double acc = 0.0;
        if (a.unit_known) {  // <e_u, P_q> = P_q(u): the one nonzero product, as the full sum gives it
            if (blockIdx.x == 0 && t == 0 && a.unit_e >= 0) acc = a.V[(i64)q * a.ld + a.unit_e];
        } else {
            acc = pass(0.0, q, q, RK_DOT);
        }
        ok = reduce(acc, h, kind_of(0) == RK_DOT ? res_col(mode, j, 1) : -1);
    } else {
        double s = 0.0;
        for (int k = t; k < a.npin; k += WT) s += a.pin[k];
        s = wave_sum(s);
        if ((t & 63) == 0) sm[t >> 6] = s;
        __syncthreads();
        h = sm[0];
#pragma unroll
        for (int w = 1; w < WT / 64; ++w) h += sm[w];
        __syncthreads();
        ok = res_pin_fold(a, h, bc, &okf);
    }
    for (int p = 0; p < np && ok; ++p) {
        const int i = res_col(mode, j, p);
        const int kind = kind_of(p);
        if (mode == RES_MGS && blockIdx.x == 0 && t == 0) hsh[i] = (p < j ? 0.0 : hsh[i]) + h;  // H(i,j) (+)= h
        const double acc = pass(mode == RES_MGS ? h : a.coef * h, i, res_col(mode, j, p + 1), kind);
        if (kind != RK_NONE)
            ok = reduce(acc, h, p + 1 < np && kind_of(p + 1) == RK_DOT ? res_col(mode, j, p + 2) : -1);
    }
    if (!ok) return;  // uniform per workgroup; *err is set
    const bool close = mode == RES_HH_UP && a.close_hh;
    if (mode != RES_MGS) {  // reflections: the resident part of w back to HBM (not when close)
        double acc = 0.0;  // RES_HH_UP: ||w(j+1:n)||^2, local indices >= tail0
        const bool up = mode == RES_HH_UP;
#pragma unroll
        for (int k = 0; k < RW; ++k)
            if (c0 + k < cend) {
                if (!close) W2[(c0 + k) * WT + t] = wr[k];
                if (up) sq_acc(acc, wr[k], (c0 + k) * WT + t, tail0, c0 + k == 0);
            }
        for (int k = 0; k < LW; ++k)
            if (l0 + k < lend) {
                const double2 v = lw[k * WT + t];
                if (!close) W2[(l0 + k) * WT + t] = v;
                if (up) sq_acc(acc, v, (l0 + k) * WT + t, tail0, l0 + k == 0);
            }
        if (up) {
            for (i64 e = sbase; e < n2; e += sstride) sq_acc(acc, W2[e], e, tail0, 2 * e < tail0 + 2);
            if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0 && a.n - 1 >= tail0) {
                const double x = a.w[a.n - 1];
                acc = acc + x * x;
            }
            ok = reduce(acc, h, -1);
            if (!ok) return;
            if (blockIdx.x == 0 && t == 0) a.hs[0] = h;  // ||w(j+1:n)||^2
        }
        if (!close) {
            clk.finish(a.stamps, mode);
            return;
        }
        // Next reflector in the same launch (gmres_hh.f90:306-318; k_hh_pivot + k_hh_fix +
        // k_scale of the launch path, the same element arithmetic): on the rank owning
        // w(j+1) (local index f = tail0 >= 0) H(j+1,j) = w(j+1) > 0 ? -tmp : tmp with tmp =
        // sqrt(h), w(1:j) = 0, w(j+1) = w(j+1) - H; then P(:,j+1) = w / ||w||.  w(1:j+1)
        // before the fix goes to hb for the pivot kernel (the H column).  The indices <= f
        // lie in chunks 0 and 1 (f <= RHMAX): the per-element test runs there only.
        const double s = sqrt(h);
        const i64 f = tail0;
        auto fix1 = [&](double &x, i64 g) {
            if (g < f) {
                a.hb[g] = x;
                x = 0.0;
            } else if (g == f) {
                a.hb[g] = x;
                const double dl = (x > 0.0) ? s : -s;  // delta = -H
                x = x + dl;
            }
        };
        auto fix_sq = [&](double &acc2, double2 &v, i64 e2, bool chk) {
            if (chk) {
                fix1(v.x, 2 * e2);
                fix1(v.y, 2 * e2 + 1);
            }
            acc2 = acc2 + v.x * v.x;
            acc2 = acc2 + v.y * v.y;
        };
        const i64 cfix = f >= 0 ? f / (2 * WT) : -1;  // last chunk holding an index <= f
        double acc2 = 0.0;
#pragma unroll
        for (int k = 0; k < RW; ++k)
            if (c0 + k < cend) fix_sq(acc2, wr[k], (c0 + k) * WT + t, c0 + k <= cfix);
        for (int k = 0; k < LW; ++k)
            if (l0 + k < lend) {
                double2 v = lw[k * WT + t];
                const bool chk = l0 + k <= cfix;
                fix_sq(acc2, v, (l0 + k) * WT + t, chk);
                if (chk) lw[k * WT + t] = v;
            }
        for (i64 e = sbase; e < n2; e += sstride) {
            double2 v = W2[e];
            const bool chk = 2 * e <= f;
            fix_sq(acc2, v, e, chk);
            if (chk) W2[e] = v;
        }
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) {
            double x = a.w[a.n - 1];
            if (a.n - 1 <= f) {
                fix1(x, a.n - 1);
                a.w[a.n - 1] = x;
            }
            acc2 = acc2 + x * x;
        }
        ok = reduce(acc2, h, -1);
        if (!ok) return;
    }
    const double hn = sqrt(h);
    double2 *__restrict__ O2 = reinterpret_cast<double2 *>(a.vout);
#pragma unroll
    for (int k = 0; k < RW; ++k)
        if (c0 + k < cend)
            O2[(c0 + k) * WT + t] = hn != 0.0 ? double2{wr[k].x / hn, wr[k].y / hn} : double2{0.0, 0.0};
    for (int k = 0; k < LW; ++k)
        if (l0 + k < lend) {
            const double2 v = lw[k * WT + t];
            O2[(l0 + k) * WT + t] = hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0};
        }
    for (i64 e = sbase; e < n2; e += sstride) {
        const double2 v = W2[e];
        O2[e] = hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0};
    }
    if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) a.vout[a.n - 1] = hn != 0.0 ? a.w[a.n - 1] / hn : 0.0;
    clk.finish(a.stamps, mode);
    if (mode == RES_MGS && blockIdx.x == 0) {
        __syncthreads();
        for (int k = t; k < j; k += WT) {
            a.hs[k] = hsh[k];
            a.hcopy[k] = hsh[k];
        }
        if (t == 0) {
            a.hs[j] = hn;
            a.hcopy[j] = hn;
        }
    }
}


// --------------------------------------------------------------------------
// Resident MGS-R step, column-cache variant (k_mgs_wres's structure, NT-thread
// workgroups, one per CU: NT = 256 one wave per SIMD, 512 two -- the second wave
// keeps a batch of loads in flight while the first consumes its own, at half
// the registers per thread): w wholly in registers (RW
// double2 per thread) and the running Krylov column cached on chip -- RX
// double2 per thread in registers, LX more in LDS.  A pass reads only its dot
// column V_q (its AXPY column V_i is the previous pass's V_q, still cached):
// 8 B per unknown per projection, against 16 B for the w-only kernel and for
// k_mgs_res's LDS-held w.  For slabs of up to RW chunks per thread -- the slab
// of one GPU of 4096^2 / 2 and of 8192^2 / 8 is 64 (RX + LX = 62 cached), of
// 4096^2 / 4 is 32.  Chunks past RX + LX (not cached) read V_i too (16 B),
// chunks past RW stream (32 B).  Same exchange, same element arithmetic as
// k_mgs_res / k_mgs_wres; only the dot summation order within a thread
// differs.  Columns non-temporal (nothing is re-read through the caches).
// --------------------------------------------------------------------------
template <int RW, int RX, int LX, int MODE, int WBT = 8, int TCHP = 0, int NT = WT>
__global__ __launch_bounds__(NT, 1) void k_mgs_wpc(ResArgs a) {
    static_assert(RX <= RW && RX + LX <= RW, "the column cache covers register chunks of w only");
    extern __shared__ double2 lx[];  // [LX][NT]: cached column of chunks RX .. RX + LX - 1
    __shared__ int xdone;            // the exchange in progress has completed (stops the touches)
    __shared__ double sm[NT / 64];
    __shared__ double bc[1];
    __shared__ int okf;
    __shared__ double hsh[RHMAX + 1];
    const int t = threadIdx.x;
    constexpr int mode = MODE;
    const int j = a.j, np = res_np(mode, j);
    const i64 n2 = a.n >> 1, ld2 = a.ld >> 1;
    const i64 nch = a.nres2 / NT;
    const i64 c0 = (i64)blockIdx.x * a.r2e, cend = c0 + a.r2e < nch ? c0 + a.r2e : nch;
    const i64 tail0 = mode == RES_HH_UP ? a.tail0 : 0;
    const double2 *__restrict__ V2 = reinterpret_cast<const double2 *>(a.V);
    double2 *__restrict__ W2 = reinterpret_cast<double2 *>(a.w);
    ResClock clk;
    clk.start(a.stamps);
    const i64 sstride = (i64)gridDim.x * NT;
    const i64 sbase = a.nres2 + (i64)res_stream_wg() * NT + t;
    double2 wr[RW], xc[RX > 0 ? RX : 1];
    {  // w, and the AXPY column of pass 0 into the cache
        const double2 *__restrict__ C2 = V2 + (i64)res_col(mode, j, 0) * ld2;
#pragma unroll
        for (int k = 0; k < RW; ++k) wr[k] = (c0 + k < cend) ? W2[(c0 + k) * NT + t] : double2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < RX; ++k) xc[k] = (c0 + k < cend) ? ldv<true>(C2 + (c0 + k) * NT + t) : double2{0.0, 0.0};
        for (int k = 0; k < LX; ++k)
            if (c0 + RX + k < cend) lx[k * NT + t] = ldv<true>(C2 + (c0 + RX + k) * NT + t);
    }
    // One pass: w -= ch V_i (the cached column; V_i from HBM past the cache), then
    // the reduction `kind`; with a dot, V_q replaces the cached column.  Batches of
    // WBT chunks (A/B, profiles/r04/ab_wpc_r04d.jsonl: software-pipelining the
    // batches -- batch b + 1 issued before b is consumed -- was slower, 17.5 ->
    // 18.3 us per projection at 2896^2, and so were 4- and 16-chunk batches).
    auto pass = [&](double ch, int i, int q, int kind) -> double {
        const double2 *__restrict__ A2 = V2 + (i64)i * ld2;
        const double2 *__restrict__ B2 = V2 + (i64)q * ld2;
        const bool dot = kind == RK_DOT;
        double acc = 0.0;
#pragma unroll
        for (int k0 = 0; k0 < RW; k0 += WBT) {
            double2 av[WBT], bv[WBT];
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                const i64 c = c0 + k;
                if (k < RW && c < cend) {
                    if (dot) bv[u] = ldv<true>(B2 + c * NT + t);
                    if (k >= RX + LX) av[u] = ldv<true>(A2 + c * NT + t);  // not cached
                }
            }
#pragma unroll
            for (int u = 0; u < WBT; ++u) {
                const int k = k0 + u;
                if (k < RW && c0 + k < cend) {
                    double2 x;
                    if (k < RX)
                        x = xc[k < RX ? k : 0];
                    else if (k < RX + LX)
                        x = lx[(k - RX) * NT + t];
                    else
                        x = av[u];
                    wr[k].x = wr[k].x - ch * x.x;
                    wr[k].y = wr[k].y - ch * x.y;
                    if (dot) {
                        acc = acc + wr[k].x * bv[u].x;
                        acc = acc + wr[k].y * bv[u].y;
                        if (k < RX)
                            xc[k < RX ? k : 0] = bv[u];
                        else if (k < RX + LX)
                            lx[(k - RX) * NT + t] = bv[u];
                    } else if (kind == RK_NORM) {
                        sq_acc(acc, wr[k], (c0 + k) * NT + t, tail0, mode == RES_HH_UP && c0 + k == 0);
                    }
                }
            }
        }
        for (i64 e0 = sbase; e0 < n2; e0 += 2 * sstride) {  // streamed part: 32 B/unknown
            double2 wv[2], av[2], bv[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const i64 e = e0 + u * sstride;
                if (e < n2) {
                    wv[u] = W2[e];
                    av[u] = ldv<true>(A2 + e);
                    if (dot) bv[u] = ldv<true>(B2 + e);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const i64 e = e0 + u * sstride;
                if (e < n2) {
                    wv[u].x = wv[u].x - ch * av[u].x;
                    wv[u].y = wv[u].y - ch * av[u].y;
                    W2[e] = wv[u];
                    if (dot) {
                        acc = acc + wv[u].x * bv[u].x;
                        acc = acc + wv[u].y * bv[u].y;
                    } else if (kind == RK_NORM) {
                        sq_acc(acc, wv[u], e, tail0, mode == RES_HH_UP && 2 * a.nres2 < tail0);
                    }
                }
            }
        }
        if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) {  // odd-length tail element
            const i64 e = a.n - 1;
            const double x = a.w[e] - ch * a.V[(i64)i * a.ld + e];
            a.w[e] = x;
            if (dot) acc = acc + x * a.V[(i64)q * a.ld + e];
            if (kind == RK_NORM && e >= tail0) acc = acc + x * x;
        }
        return acc;
    };
    // The all-gather; meanwhile waves 1..3 touch the first TCHP chunks of the NEXT
    // pass's dot column (one dword per 128-B line into a sink register, paced, up
    // to the moment wave 0 holds the total), so that pass starts on lines already
    // in L2 instead of paying the stream's ramp-up after every exchange (the pass
    // time was ~3.3 us + bytes / 5.7 TB/s over 1448^2..2896^2, r04d).
    int xi = 0;
    int touch_sink = 0;
    auto reduce = [&](double acc, double &h, int touch_col) -> bool {
        clk.passed(a.stamps);
        acc = wave_sum(acc);
        if ((t & 63) == 0) sm[t >> 6] = acc;
        if (t == 0) xdone = 0;
        __syncthreads();
        if (t < 64) {
            res_exchange<NT / 64, MODE == RES_MGS, RES_POLL_SLEEP_PC>(a, xi, sm, bc, &okf);
            if (t == 0) *(volatile int *)&xdone = 1;
        } else if constexpr (TCHP > 0) {
            if (touch_col >= 0) {
                const char *base = reinterpret_cast<const char *>(V2 + (i64)touch_col * ld2 + c0 * NT);
                const i64 nc = cend - c0 < TCHP ? (cend - c0 > 0 ? cend - c0 : 0) : TCHP;
                for (i64 l = t - 64; l < 32 * nc; l += NT - 64) {
                    if (*(volatile int *)&xdone) break;  // wave-uniform: one LDS word
                    asm volatile("global_load_dword %0, %1, off" : "+v"(touch_sink) : "v"(base + l * 128) : "memory");
                    __builtin_amdgcn_s_sleep(TOUCH_PACE);
                }
            }
        }
        __syncthreads();
        if constexpr (TCHP > 0) asm volatile("s_waitcnt vmcnt(0)" : : "v"(touch_sink) : "memory");
        ++xi;
        h = bc[0];
        clk.waited(a.stamps);
        return okf != 0;
    };
    auto kind_of = [&](int p) { return p < np - 1 ? RK_DOT : (mode == RES_HH_DOWN ? RK_NONE : RK_NORM); };
    auto next_dot_col = [&](int p) { return p + 1 < np && kind_of(p + 1) == RK_DOT ? res_col(mode, j, p + 2) : -1; };
    double h;
    bool ok = true;
    if (mode == RES_HH_DOWN) {
        // the pre-dot <v, V_col(0)> as a pass with h = 0 (w - 0 V = w; the cache is
        // refilled with the same column)
        const int q = res_col(mode, j, 0);
        double acc = 0.0;
        if (a.unit_known) {  // <e_u, P_q> = P_q(u): the one nonzero product, as the full sum gives it
            if (blockIdx.x == 0 && t == 0 && a.unit_e >= 0) acc = a.V[(i64)q * a.ld + a.unit_e];
        } else {
            acc = pass(0.0, q, q, RK_DOT);
        }
        ok = reduce(acc, h, kind_of(0) == RK_DOT ? res_col(mode, j, 1) : -1);
    } else {
        double s = 0.0;
        for (int k = t; k < a.npin; k += NT) s += a.pin[k];
        s = wave_sum(s);
        if ((t & 63) == 0) sm[t >> 6] = s;
        __syncthreads();
        h = sm[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) h += sm[w];
        __syncthreads();
        ok = res_pin_fold(a, h, bc, &okf);
    }
    for (int p = 0; p < np && ok; ++p) {
        const int i = res_col(mode, j, p);
        const int kind = kind_of(p);
        if (mode == RES_MGS && blockIdx.x == 0 && t == 0) hsh[i] = (p < j ? 0.0 : hsh[i]) + h;  // H(i,j) (+)= h
        const double acc = pass(mode == RES_MGS ? h : a.coef * h, i, res_col(mode, j, p + 1), kind);
        if (kind != RK_NONE) ok = reduce(acc, h, next_dot_col(p));
    }
    if (!ok) return;  // uniform per workgroup; *err is set
    if (mode != RES_MGS) {  // reflections: w back to HBM (RES_HH_UP: h = ||w(j+1:n)||^2)
#pragma unroll
        for (int k = 0; k < RW; ++k)
            if (c0 + k < cend) W2[(c0 + k) * NT + t] = wr[k];
        if (mode == RES_HH_UP && blockIdx.x == 0 && t == 0) a.hs[0] = h;
        clk.finish(a.stamps, mode);
        return;
    }
    const double hn = sqrt(h);
    double2 *__restrict__ O2 = reinterpret_cast<double2 *>(a.vout);
#pragma unroll
    for (int k = 0; k < RW; ++k)
        if (c0 + k < cend)
            O2[(c0 + k) * NT + t] = hn != 0.0 ? double2{wr[k].x / hn, wr[k].y / hn} : double2{0.0, 0.0};
    for (i64 e = sbase; e < n2; e += sstride) {
        const double2 v = W2[e];
        O2[e] = hn != 0.0 ? double2{v.x / hn, v.y / hn} : double2{0.0, 0.0};
    }
    if ((a.n & 1) && blockIdx.x == gridDim.x - 1 && t == 0) a.vout[a.n - 1] = hn != 0.0 ? a.w[a.n - 1] / hn : 0.0;
    clk.finish(a.stamps, mode);
    if (blockIdx.x == 0) {
        __syncthreads();
        for (int k = t; k < j; k += NT) {
            a.hs[k] = hsh[k];
            a.hcopy[k] = hsh[k];
        }
        if (t == 0) {
            a.hs[j] = hn;
            a.hcopy[j] = hn;
        }
    }
}

}  // namespace gk
