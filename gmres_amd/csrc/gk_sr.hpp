// gk_sr.hpp -- fused device passes of the short-recurrence solvers that share
// the GMRES operator / preconditioner seam: pcg_omp (src/cg.f90:154-234) and
// pbicgstab_omp (src/bicgstab.f90:91-182).
//
// The reference runs every BLAS-1 operation as its own OpenMP loop and keeps
// the scalars (alpha, beta, omega, the residual) in `single` blocks.  Here one
// iteration is two (PCG) or three (BiCGSTAB) passes over HBM:
//
//   * k_sr_march: a Poisson-5 line march (k_stencil's register scheme: lines
//     j-1, j, j+1 in registers, W/E neighbours by __shfl) whose OPERAND is
//     formed on load from up to three vectors -- p = z + beta p, p = r +
//     beta (p - omega ap), s = r - alpha ap -- so the vector update that
//     precedes a stencil in the reference costs no pass of its own, and whose
//     epilogue carries the element-wise updates and dots that follow it;
//   * k_sr_march2 (cbpr2, one rank): two-level marches -- the preconditioner
//     and the operator next to it in one pass, level 1 one line ahead of
//     level 2 (PCG: r update + z = cbpr2(r); BiCGSTAB: z = cbpr2(p), A z);
//   * k_sr_vec: the element-wise passes (BiCGSTAB's x / r update with its two
//     dots), double2 streams.
//
// Scalars never leave the device.  Every pass writes one partial per
// workgroup; the LAST workgroup to finish (a completion ticket, one atomic per
// workgroup) sums the slab in a fixed order and computes the next scalar
// (alpha = rz / <Ap, p>, ...) into SrDev, which the next pass reads.  On N
// ranks the slab is all-reduced first and k_sr_fin does the same on one
// workgroup.  The per-iteration residual goes to a device history and a
// mapped host mirror; once it drops below tol every later pass returns at
// entry -- the reference's `if (converged) cycle` -- so the host may queue
// iterations ahead without reading anything back per iteration.
//
// Element-wise expressions keep the reference's association order (compiled
// with -ffp-contract=off); only the dot-product summation order differs.
#pragma once
#include "gk_kernels.hpp"  // ld_vec, st_vec

namespace gk {

// Device-resident scalars of one short-recurrence solve.
struct SrDev {
    double rz;      // PCG: <r, z> of the current iteration; BiCGSTAB: rr0 = <r, r0>
    double alpha, beta, omega;
    double res;     // residual of the last executed iteration
    double tol;
    int it;         // iterations executed
    int done;       // first iteration with res < tol (0: none)
    unsigned ticket;  // completion ticket of the running pass (0 between passes)
    int maxit;      // length of the history
};

// Mapped host copy, written by the residual finaliser of every iteration.
struct SrMirror {
    int it, done;
    double res;
};

// Fused line-march passes.  Operand u per point; t = u / d for the cbpr2
// passes (chebyshev.f90:27-31), else t = u; ax = A t.
enum {
    SRK_CG_P = 0,  // u = z + beta p (cg.f90:227-231); ou = u; dot <A u, u> (:196-199)
    SRK_CG_X = 1,  // u = p; x += alpha u; r -= alpha A u; dot <r, r> (:206-211)
    SRK_CG_Z = 2,  // u = r; oy = z = cbpr2(r) (chebyshev.f90:27-37); dot <r, z> (cg.f90:213-217)
    SRK_BI_P = 3,  // u = r + beta (p - omega ap) (bicgstab.f90:176-180); ou = u; oy = ap = A u; dot <ap, r0>
    SRK_BI_PC = 4, // u as BI_P; ou = u; oy = z1 = cbpr2(u)
    SRK_BI_S = 5,  // u = s = r - alpha ap (:131-135); ou = s; oy = as = A s; dots <as, s>, <as, as> (:139-144)
    SRK_BI_SC = 6, // u as BI_S; ou = s; oy = z2 = cbpr2(s)
    SRK_ST1 = 7,   // u = in0; oy = A u; dot <A u, vd>        (cbpr2 BiCGSTAB: ap = A z1, <ap, r0>)
    SRK_ST2 = 8,   // u = in0; oy = A u; dots <A u, vd>, <A u, A u>  (as = A z2, <as, s>, <as, as>)
};

// Element-wise passes.
enum {
    SRV_BI_X = 0,   // x = (x + alpha z1) + omega z2; r = s - omega as; dots <r, r>, <r, r0> (:148-171)
    SRV_BI_PE = 1,  // ou = r + beta (p - omega ap)          (generic preconditioner)
    SRV_BI_SE = 2,  // ou = r - alpha ap                     (generic preconditioner)
    SRV_DOT = 3,    // dot <in0, in1>                         (solve start)
    SRV_BI_XS = 4,  // SRV_BI_X with z2 = s (identity M: in1 == in2): one load serves both operands
};

// What the last workgroup computes from the pass's partial slab(s).
enum {
    FIN_NONE = 0,
    FIN_CG_INIT = 1,   // rz = <r, z>; beta = 0 (p = z + 0 * 0 on the first iteration)
    FIN_CG_ALPHA = 2,  // alpha = rz / <Ap, p>                          (cg.f90:200-202)
    FIN_CG_RES_ID = 3, // identity M: res = sqrt(<r,r>); beta = <r,r> / rz; rz = <r,r>  (:218-226)
    FIN_CG_RES = 4,    // res = sqrt(<r,r>) (beta from FIN_CG_BETA)
    FIN_CG_BETA = 5,   // beta = <r, z> / rz; rz = <r, z>
    FIN_BI_INIT = 6,   // rr0 = <r, r0>; beta = 0; omega = 1
    FIN_BI_ALPHA = 7,  // alpha = rr0 / <ap, r0>                        (:127-129)
    FIN_BI_OMEGA = 8,  // omega = <as, s> / <as, as>                   (:145-147)
    FIN_BI_RES = 9,    // res = sqrt(<r,r>); beta = (<r,r0> / rr0) (alpha / omega); rr0 = <r,r0>  (:159-175)
    FIN_CG_RES_BETA = 10,  // FIN_CG_RES then FIN_CG_BETA from the second slab (k_sr_march2 SR2_CG_XZ)
};

struct SrArgs {
    const double *in0, *in1, *in2;  // operand inputs (k_sr_march) / element-wise inputs (k_sr_vec)
    const double *lo[3], *hi[3];    // halo line of each operand input (nullptr: physical boundary)
    const double *zl;               // N zeros: the line beyond a physical boundary
    double *ou;                     // the operand u itself (p, s)
    double *oy;                     // the stencil output (ap, as, z, z1, z2); k_sr_march2: the level-1 output
    double *oz;                     // k_sr_march2: the level-2 output (z, ap, as)
    double *x, *r;                  // updated in place (CG_X; BI_X)
    const double *e0;               // BI_X: as
    const double *vd;               // dot partner (r0, s)
    double *part0, *part1;          // partial slabs (one entry per workgroup)
    SrDev *sd;
    double *hist;                   // device history [maxit]
    SrMirror *mir;                  // mapped host mirror
    double cd, ca;                  // cbpr2: d, alpha (chebyshev.f90:19-25)
    int N, nlines, JT, fin;
};

// Partials cross workgroups (and XCDs, whose L2s are not coherent) inside one
// launch: written and read as agent-scope relaxed atomics, which go to the
// coherence point, so no L2 write-back fence is needed.  (A release on the
// ticket writes back the XCD's whole L2: with acq_rel tickets the dot-carrying
// passes ran at 0.26-0.33 of HBM, measured r06c.)
__device__ __forceinline__ void sr_put(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double sr_get(const double *p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long *>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Fixed-order sum of a slab written by sr_put (k_sr_fin: any partial slab).
__device__ __forceinline__ double sr_slab_sum(const double *p, int np, double *sm) {
    double s = 0.0;
    for (int k = threadIdx.x; k < np; k += TPB) s += sr_get(p + k);
    return block_sum(s, sm);
}

// The finaliser: one workgroup (all TPB threads) after every partial of the
// pass is visible.
__device__ __forceinline__ void sr_fin(int mode, SrDev *sd, const double *p0, const double *p1, int np,
                                       double *hist, SrMirror *mir, double *sm) {
    const double s0 = sr_slab_sum(p0, np, sm);
    const double s1 =
        (mode == FIN_BI_OMEGA || mode == FIN_BI_RES || mode == FIN_CG_RES_BETA) ? sr_slab_sum(p1, np, sm) : 0.0;
    if (threadIdx.x != 0) return;
    switch (mode) {
        case FIN_CG_INIT:
            sd->rz = s0;
            sd->beta = 0.0;
            break;
        case FIN_CG_ALPHA: sd->alpha = sd->rz / s0; break;
        case FIN_CG_BETA:
            sd->beta = s0 / sd->rz;
            sd->rz = s0;
            break;
        case FIN_BI_INIT:
            sd->rz = s0;
            sd->beta = 0.0;
            sd->omega = 1.0;
            break;
        case FIN_BI_ALPHA: sd->alpha = sd->rz / s0; break;
        case FIN_BI_OMEGA: sd->omega = s0 / s1; break;
        default: {  // the residual of an iteration
            const double res = sqrt(s0);
            const int it = sd->it + 1;
            sd->it = it;
            sd->res = res;
            if (it <= sd->maxit) hist[it - 1] = res;
            if (res < sd->tol && sd->done == 0) sd->done = it;
            if (mode == FIN_CG_RES_ID) {
                sd->beta = s0 / sd->rz;
                sd->rz = s0;
            } else if (mode == FIN_BI_RES) {
                sd->beta = (s1 / sd->rz) * (sd->alpha / sd->omega);
                sd->rz = s1;
            } else if (mode == FIN_CG_RES_BETA) {
                sd->beta = s1 / sd->rz;
                sd->rz = s1;
            }
            mir->res = res;
            mir->done = sd->done;
            mir->it = it;
            break;
        }
    }
}

// Publish this workgroup's partial(s); the last workgroup of the grid runs
// the finaliser (fin != FIN_NONE: single rank).  Each partial is stored at the
// coherence point (sr_put) and acknowledged (vmcnt(0)) before the workgroup
// takes its ticket, so the workgroup that takes the last ticket finds every
// partial there (sr_get).
template <int NACC>
__device__ __forceinline__ void sr_publish(const SrArgs &a, double acc0, double acc1, int bid, int nblk,
                                           double *sm, int *last) {
    const double s0 = block_sum(acc0, sm);
    const double s1 = NACC > 1 ? block_sum(acc1, sm) : 0.0;
    if (threadIdx.x == 0) {
        sr_put(a.part0 + bid, s0);
        if (NACC > 1) sr_put(a.part1 + bid, s1);
    }
    if (a.fin == FIN_NONE) return;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial stores are acknowledged
        const unsigned t = __hip_atomic_fetch_add(&a.sd->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = (t == (unsigned)nblk - 1u) ? 1 : 0;
    }
    __syncthreads();
    if (*last == 0) return;
    sr_fin(a.fin, a.sd, a.part0, a.part1, nblk, a.hist, a.mir, sm);
    if (threadIdx.x == 0) a.sd->ticket = 0u;
}

template <int K>
__device__ __forceinline__ double sr_operand(double v0, double v1, double v2, double al, double be, double om) {
    if constexpr (K == SRK_CG_P) return v0 + be * v1;
    else if constexpr (K == SRK_BI_P || K == SRK_BI_PC) return v0 + be * (v1 - om * v2);
    else if constexpr (K == SRK_BI_S || K == SRK_BI_SC) return v0 - al * v1;
    else return v0;
}

template <int K>
constexpr int sr_nin() {
    return (K == SRK_BI_P || K == SRK_BI_PC) ? 3 : (K == SRK_CG_P || K == SRK_BI_S || K == SRK_BI_SC) ? 2 : 1;
}

template <int K>
constexpr int sr_nacc() {
    return (K == SRK_BI_S || K == SRK_ST2) ? 2 : (K == SRK_BI_PC || K == SRK_BI_SC) ? 0 : 1;
}

// One line of loads in flight ahead of use (A/B r06j at 4096^2: 0 / 1 / 2 extra lines ->
// PCG 4,684 / 4,614 / 4,523 it/s, BiCGSTAB 2,133 / 2,085 / 2,052; the deeper rings were
// removed).

// Cache policy of the streamed operands (each read or written once per pass):
// bit 0 non-temporal loads of the march operands, bit 1 non-temporal stores,
// bit 2 non-temporal loads in the element-wise passes, bit 3 non-temporal loads
// of the march epilogue operands (x, r, the dot partner), bit 4 non-temporal
// loads of the march operands read for the last time in the iteration (the
// previous p / ap), bit 5 the same in the two-level marches and for r in
// BiCGSTAB's s pass.  The W/E edge loads keep the default policy.  Default 62
// (A/B r06y / r06z / r06ax / r06az at 4096^2: 14 over 0 +7-13 % on every leg; 30
// over 14 +1-5 %; 62 over 30 +1 % on BiCGSTAB cbpr2; bit 0 -- every operand
// non-temporal -- loses 2-14 %).
#ifndef GK_SR_NT
#define GK_SR_NT 62
#endif
typedef double sr_d2v __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 sr_ld2(const double *p) {
    if constexpr (NT) {
        const sr_d2v t = __builtin_nontemporal_load(reinterpret_cast<const sr_d2v *>(p));
        return double2{t.x, t.y};
    } else {
        return *reinterpret_cast<const double2 *>(p);
    }
}
template <bool NT>
__device__ __forceinline__ double sr_ld1(const double *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
__device__ __forceinline__ void sr_st2(double *p, double2 v) {
    if constexpr (GK_SR_NT & 2) __builtin_nontemporal_store(sr_d2v{v.x, v.y}, reinterpret_cast<sr_d2v *>(p));
    else *reinterpret_cast<double2 *>(p) = v;
}
template <int VEC>
__device__ __forceinline__ void sr_stv(double *p, const double (&v)[VEC]) {
    if constexpr (VEC == 2) sr_st2(p, double2{v[0], v[1]});
    else if constexpr (GK_SR_NT & 2) __builtin_nontemporal_store(v[0], p);
    else p[0] = v[0];
}

template <int VEC, int K>
__global__ __launch_bounds__(TPB) void k_sr_march(SrArgs a) {
    __shared__ double sm[WAVES];
    __shared__ int last;
    if (a.sd->done) return;  // converged: the reference's `if (converged) cycle`
    constexpr bool CB = (K == SRK_CG_Z || K == SRK_BI_PC || K == SRK_BI_SC);
    constexpr int NIN = sr_nin<K>();
    constexpr int NACC = sr_nacc<K>();
    constexpr bool WU = (K == SRK_CG_P || K == SRK_BI_P || K == SRK_BI_PC || K == SRK_BI_S || K == SRK_BI_SC);
    constexpr bool WY = (K != SRK_CG_P && K != SRK_CG_X);
    constexpr bool VD = (K == SRK_BI_P || K == SRK_ST1 || K == SRK_ST2);
    const double al = a.sd->alpha, be = a.sd->beta, om = a.sd->omega;
    const double dv = a.cd, ca = a.ca;
    const int N = a.N;
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPB * VEC) + (i64)VEC * threadIdx.x;
    const bool act = i0 < N;
    const int j0 = blockIdx.y * a.JT;
    const int j1 = min(j0 + a.JT, a.nlines);
    double acc0 = 0.0, acc1 = 0.0;

    auto in_ptr = [&](int v) -> const double * { return v == 0 ? a.in0 : v == 1 ? a.in1 : a.in2; };
    // Software pipeline: the raw operand inputs of line j+2 and the epilogue and
    // edge-lane inputs of line j+1 are issued at the top of step j and consumed in
    // step j+1.  Every load is unconditional (addresses clamped to valid memory,
    // out-of-range values replaced by selects afterwards), so the compiler can wait
    // for exactly the loads a step consumes instead of draining the pipeline at a
    // branch merge.
    const i64 il = act ? i0 : 0;  // the load column (a lane past N loads column 0, then writes nothing)
    auto ldr = [&](const double *p, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 1) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 1) != 0>(p);
        }
    };
    auto lde = [&](const double *p, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 8) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 8) != 0>(p);
        }
    };
    // line jj of input q: own line, halo line, or the zero line past a physical
    // boundary (the operand of zero inputs is +0 in every formula: no select).
    // The halo choice is made once, outside the march.
    const double *lo_[3], *hi_[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        lo_[q] = a.lo[q] != nullptr ? a.lo[q] : a.zl;
        hi_[q] = a.hi[q] != nullptr ? a.hi[q] : a.zl;
    }
    auto src = [&](int q, int jj) -> const double * {
        return jj < 0 ? lo_[q] : (jj < a.nlines ? in_ptr(q) + (i64)jj * N : (jj == a.nlines ? hi_[q] : a.zl));
    };
    // operand inputs read here for the last time in the iteration (p, ap of the previous
    // iteration: CG_P in1, BI_P in1 / in2) may load non-temporally (GK_SR_NT bit 4)
    auto ldlast = [&](const double *p, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 16) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 16) != 0>(p);
        }
    };
    auto raw_line = [&](int jj, double (&v)[3][VEC]) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            // last use in the iteration: the previous p / ap (CG_P, BI_P in1 / in2); with bit 5
            // also r in BiCGSTAB's s pass (BI_S in0: bi_x then overwrites it)
            const bool last = (q > 0 && (K == SRK_CG_P || K == SRK_BI_P)) ||
                                  ((GK_SR_NT & 32) != 0 && q == 0 && K == SRK_BI_S);
            if (q < NIN && last) {
                ldlast(src(q, jj) + il, v[q]);
            } else if (q < NIN) {
                ldr(src(q, jj) + il, v[q]);
            } else {
#pragma unroll
                for (int k = 0; k < VEC; ++k) v[q][k] = 0.0;
            }
        }
    };
    auto form = [&](const double (&v)[3][VEC], double (&u)[VEC], double (&t)[VEC]) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double x = sr_operand<K>(v[0][k], v[1][k], v[2][k], al, be, om);
            u[k] = act ? x : 0.0;
            t[k] = CB ? u[k] / dv : u[k];
        }
    };
    auto edge_t = [&](const double (&e)[3]) -> double {  // t of an edge lane's W/E neighbour
        const double u = sr_operand<K>(e[0], e[1], e[2], al, be, om);
        return CB ? u / dv : u;
    };
    // edge inputs of own line jj: lane 0 the point left of the window, lane 63 the
    // one right of it; the other lanes load lane 0's point (lanes 1..31) or lane
    // 63's (32..62), so the wave's edge load touches two cache lines and never
    // re-reads the lanes' own points through L2 (A/B r06ap: +3-5 % over every lane
    // reloading its own point)
    const i64 wb0 = i0 - (i64)VEC * lane;  // the wave's first point
    i64 ei = lane < 32 ? wb0 - 1 : wb0 + 64 * VEC;
    ei = ei < 0 ? 0 : (ei >= N ? N - 1 : ei);
    auto edge_ld = [&](int jj, double (&e)[3]) {
        const i64 off = (i64)jj * N + ei;
#pragma unroll
        for (int q = 0; q < 3; ++q) e[q] = q < NIN ? in_ptr(q)[off] : 0.0;
    };
    auto epi_ld = [&](int jj, double (&xv)[VEC], double (&rv)[VEC], double (&vd)[VEC]) {
        const i64 off = (i64)jj * N + il;
        if (K == SRK_CG_X) {
            lde(a.x + off, xv);
            lde(a.r + off, rv);
        }
        if (VD) lde(a.vd + off, vd);
    };

    if (j0 < a.nlines) {
        double uc[VEC], up[VEC], tm[VEC], tc[VEC], tp[VEC], scratch[VEC];
        {
            double v[3][VEC];
            raw_line(j0 - 1, v);
            form(v, scratch, tm);
            raw_line(j0, v);
            form(v, uc, tc);
            raw_line(j0 + 1, v);
            form(v, up, tp);
        }
        // in flight: operand inputs of line j+2, epilogue operands of line j+1
        double rw[3][VEC];
        double xq[VEC] = {}, rq[VEC] = {}, vq[VEC] = {};
        double xc[VEC] = {}, rc[VEC] = {}, vc[VEC] = {}, ec[3] = {};
        epi_ld(j0, xc, rc, vc);
        edge_ld(j0, ec);
        for (int j = j0; j < j1; ++j) {
            // issue: operand inputs of line j+2 (unused past the block's last line),
            // epilogue and edge inputs of line j+1 (line j stands in past the last)
            const int jn = j + 1 < j1 ? j + 1 : j;
            raw_line(j + 2, rw);
            epi_ld(jn, xq, rq, vq);
            double en[3] = {};
            edge_ld(jn, en);
            const i64 row = (i64)j * N;
            double left = __shfl_up(tc[VEC - 1], 1, 64);
            double right = __shfl_down(tc[0], 1, 64);
            const double et = edge_t(ec);
            left = lane == 0 ? et : left;
            right = lane == 63 ? et : right;
            left = i0 == 0 ? 0.0 : left;
            right = i0 + VEC >= N ? 0.0 : right;
            double yv[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const double W = (k == 0) ? left : tc[k - 1];
                const double E = (k == VEC - 1) ? right : tc[k + 1];
                const double s = ((W + E) + tp[k]) + tm[k];
                const double ax = 4.0 * tc[k] - 1.0 * s;
                if constexpr (CB) {
                    yv[k] = tc[k] + ca * (uc[k] - ax);
                } else {
                    yv[k] = ax;
                }
                if constexpr (K == SRK_CG_X) {
                    xc[k] = xc[k] + al * uc[k];
                    rc[k] = rc[k] - al * ax;
                }
            }
            if (act) {
                if (WU) sr_stv<VEC>(a.ou + row + i0, uc);
                if (WY) sr_stv<VEC>(a.oy + row + i0, yv);
                if (K == SRK_CG_X) {
                    sr_stv<VEC>(a.x + row + i0, xc);
                    sr_stv<VEC>(a.r + row + i0, rc);
                }
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {  // a lane past N contributes exact zeros (u = 0)
                if constexpr (K == SRK_CG_P) acc0 = acc0 + yv[k] * uc[k];
                else if constexpr (K == SRK_CG_X) acc0 = act ? acc0 + rc[k] * rc[k] : acc0;
                else if constexpr (K == SRK_CG_Z) acc0 = act ? acc0 + uc[k] * yv[k] : acc0;
                else if constexpr (K == SRK_BI_P || K == SRK_ST1) acc0 = act ? acc0 + yv[k] * vc[k] : acc0;
                else if constexpr (K == SRK_BI_S) {
                    acc0 = act ? acc0 + yv[k] * uc[k] : acc0;
                    acc1 = act ? acc1 + yv[k] * yv[k] : acc1;
                } else if constexpr (K == SRK_ST2) {
                    acc0 = act ? acc0 + yv[k] * vc[k] : acc0;
                    acc1 = act ? acc1 + yv[k] * yv[k] : acc1;
                }
            }
            // line j+2's operand, formed now that line j is done; the rings advance
            double un[VEC], tn[VEC];
            form(rw, un, tn);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                tm[k] = tc[k];
                uc[k] = up[k];
                tc[k] = tp[k];
                up[k] = un[k];
                tp[k] = tn[k];
                xc[k] = xq[k];
                rc[k] = rq[k];
                vc[k] = vq[k];
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) ec[q] = en[q];
        }
    }
    if constexpr (NACC > 0)
        sr_publish<NACC>(a, acc0, acc1, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, sm, &last);
}

// Two-level marches (single rank, gk_sr_* with cbpr2): the preconditioner and
// the operator next to it in ONE pass.  Level 1 is computed one line ahead of
// level 2 (line j+1 at step j), so level 2 finds its three lines in registers;
// the W/E neighbours across windows come from the edge lanes, which compute the
// level-1 value of the point beyond their window themselves (two edge columns:
// ea next to the window, eb one further).  Every element-wise expression, the
// stencil's association order and the per-workgroup dot order are those of the
// one-level passes it replaces, on the same grid: the results are bit-identical
// to SRK_CG_X + SRK_CG_Z, SRK_BI_PC + SRK_ST1, SRK_BI_SC + SRK_ST2.  Halo lines
// of other ranks are not supported (the level-1 value of a halo line needs two
// lines of the neighbour's inputs): N ranks keep the one-level passes.
enum {
    SR2_CG_XZ = 0,  // u = p; x += alpha u; v1 = r - alpha A u -> oy (next r); v2 = cbpr2(v1) -> oz (z);
                    // dots <v1, v1>, <v1, v2>        (cg.f90:206-217; chebyshev.f90:27-37)
    SR2_BI_P = 1,   // u = r + beta (p - omega ap) -> ou; v1 = cbpr2(u) -> oy (z1); v2 = A v1 -> oz (ap);
                    // dot <v2, r0>                   (bicgstab.f90:121-129, 176-180)
    SR2_BI_S = 2,   // u = r - alpha ap -> ou (s); v1 = cbpr2(u) -> oy (z2); v2 = A v1 -> oz (as);
                    // dots <v2, u>, <v2, v2>         (bicgstab.f90:131-147)
};

template <int K2>
constexpr int sr2_nin() {
    return K2 == SR2_BI_P ? 3 : K2 == SR2_BI_S ? 2 : 1;
}

// A t at one point, k_stencil's order: 4 tc - (((W + E) + N) + S)   (poisson.f90:42)
__device__ __forceinline__ double sr_ax(double tc, double W, double E, double tN, double tS) {
    const double s = ((W + E) + tN) + tS;
    return 4.0 * tc - 1.0 * s;
}

template <int VEC, int K2>
__global__ __launch_bounds__(TPB) void k_sr_march2(SrArgs a) {
    __shared__ double sm[WAVES];
    __shared__ int last;
    if (a.sd->done) return;
    constexpr int NIN = sr2_nin<K2>();
    constexpr bool CG = K2 == SR2_CG_XZ;
    constexpr int OPK = K2 == SR2_BI_P ? SRK_BI_P : K2 == SR2_BI_S ? SRK_BI_S : SRK_CG_X;  // operand formula
    const double al = a.sd->alpha, be = a.sd->beta, om = a.sd->omega;
    const double dv = a.cd, ca = a.ca;
    const int N = a.N, nl = a.nlines;
    const int lane = threadIdx.x & 63;
    const i64 i0 = (i64)blockIdx.x * (TPB * VEC) + (i64)VEC * threadIdx.x;
    const bool act = i0 < N;
    const int j0 = blockIdx.y * a.JT;
    const int j1 = min(j0 + a.JT, nl);
    const i64 il = act ? i0 : 0;
    // edge columns: ea next to the window (lane 0: left, lane 63: right), eb one further
    const bool e0l = lane == 0, e63 = lane == 63;
    const i64 wb0 = i0 - (i64)VEC * lane;  // the wave's first point (edge loads grouped as in k_sr_march)
    i64 ea = lane < 32 ? wb0 - 1 : wb0 + 64 * VEC;
    i64 eb = lane < 32 ? wb0 - 2 : wb0 + 64 * VEC + 1;
    const bool eb_ok = e0l ? (i0 - 2 >= 0) : (e63 ? (i0 + VEC + 1 < N) : true);
    ea = ea < 0 ? 0 : (ea >= N ? N - 1 : ea);
    eb = eb < 0 ? 0 : (eb >= N ? N - 1 : eb);
    const double *in[3] = {a.in0, a.in1, a.in2};
    auto src = [&](const double *b, int jj) -> const double * {
        return (jj >= 0 && jj < nl) ? b + (i64)jj * N : a.zl;
    };
    auto ld = [&](const double *p, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 1) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 1) != 0>(p);
        }
    };
    auto lde = [&](const double *p, double (&v)[VEC]) {
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 8) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 8) != 0>(p);
        }
    };
    // raw operand inputs of one line: own points, ea, eb
    struct Raw {
        double v[3][VEC], a[3], b[3];
    };
    auto ldl = [&](const double *p, double (&v)[VEC]) {  // last-use inputs (GK_SR_NT bit 5)
        if constexpr (VEC == 2) {
            const double2 t = sr_ld2<(GK_SR_NT & 32) != 0>(p);
            v[0] = t.x;
            v[1] = t.y;
        } else {
            v[0] = sr_ld1<(GK_SR_NT & 32) != 0>(p);
        }
    };
    auto raw = [&](int jj, Raw &w) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            // last use in the iteration: the previous p / ap (BI_P in1 / in2), r in the s pass (BI_S in0)
            const bool last = (K2 == SR2_BI_P && q > 0) || (K2 == SR2_BI_S && q == 0);
            if (q < NIN) {
                const double *l = src(in[q], jj);
                if (last)
                    ldl(l + il, w.v[q]);
                else
                    ld(l + il, w.v[q]);
                w.a[q] = l[ea];
                w.b[q] = l[eb];
            } else {
#pragma unroll
                for (int k = 0; k < VEC; ++k) w.v[q][k] = 0.0;
                w.a[q] = w.b[q] = 0.0;
            }
        }
    };
    // level-0 line: operand u and its stencil argument t (= u / d for cbpr2 at level 1)
    struct Ul {
        double u[VEC], t[VEC], ua, ta, tb;
    };
    auto form = [&](const Raw &w, Ul &o) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double x = sr_operand<OPK>(w.v[0][k], w.v[1][k], w.v[2][k], al, be, om);
            o.u[k] = act ? x : 0.0;
            o.t[k] = CG ? o.u[k] : o.u[k] / dv;
        }
        o.ua = sr_operand<OPK>(w.a[0], w.a[1], w.a[2], al, be, om);
        o.ta = CG ? o.ua : o.ua / dv;
        const double ub = sr_operand<OPK>(w.b[0], w.b[1], w.b[2], al, be, om);
        o.tb = eb_ok ? (CG ? ub : ub / dv) : 0.0;
    };
    // level-1 line: v1 and its stencil argument t2 (= v1 / d for cbpr2 at level 2)
    struct Vl {
        double v[VEC], t[VEC], va, ta;
    };
    // CG: r of one line (own points and ea) for v1 = r - alpha A p
    struct Rl {
        double v[VEC], a;
    };
    auto rld = [&](int jj, Rl &o) {
        if constexpr (CG) {
            const double *l = src(a.r, jj);
            lde(l + il, o.v);
            o.a = l[ea];
        } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) o.v[k] = 0.0;
            o.a = 0.0;
        }
    };
    // level 1 at line jj (centre c, neighbours s = jj-1, n = jj+1)
    auto lev1 = [&](int jj, const Ul &us, const Ul &uc, const Ul &un, const Rl &rr, Vl &o) {
        double left = __shfl_up(uc.t[VEC - 1], 1, 64);
        double right = __shfl_down(uc.t[0], 1, 64);
        left = e0l ? uc.ta : left;
        right = e63 ? uc.ta : right;
        left = i0 == 0 ? 0.0 : left;
        right = i0 + VEC >= N ? 0.0 : right;
        const bool lv = jj >= 0 && jj < nl;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const double W = (k == 0) ? left : uc.t[k - 1];
            const double E = (k == VEC - 1) ? right : uc.t[k + 1];
            const double ax = sr_ax(uc.t[k], W, E, un.t[k], us.t[k]);
            const double v = CG ? rr.v[k] - al * ax : uc.t[k] + ca * (uc.u[k] - ax);
            o.v[k] = (lv && act) ? v : 0.0;
            o.t[k] = CG ? o.v[k] / dv : o.v[k];
        }
        // the edge point ea: lane 0 -> W = eb, E = own point 0; lane 63 -> W = own point VEC-1, E = eb
        const double Wa = e0l ? uc.tb : uc.t[VEC - 1];
        const double Ea = e0l ? uc.t[0] : uc.tb;
        const double axa = sr_ax(uc.ta, Wa, Ea, un.ta, us.ta);
        const double va = CG ? rr.a - al * axa : uc.ta + ca * (uc.ua - axa);
        o.va = lv ? va : 0.0;
        o.ta = CG ? o.va / dv : o.va;
    };
    double acc0 = 0.0, acc1 = 0.0;
    if (j0 < nl) {
        Ul u0, u1, u2;  // lines j, j+1, j+2
        Vl vm, vc;      // level 1 at lines j-1, j
        Rl rc;          // CG: r of line j+1
        {
            Raw w0, w1, w2, w3, w4;
            Rl ra, rb;
            raw(j0 - 2, w0);
            raw(j0 - 1, w1);
            raw(j0, w2);
            raw(j0 + 1, w3);
            raw(j0 + 2, w4);
            rld(j0 - 1, ra);
            rld(j0, rb);
            rld(j0 + 1, rc);
            Ul um2, um1;
            form(w0, um2);
            form(w1, um1);
            form(w2, u0);
            form(w3, u1);
            form(w4, u2);
            lev1(j0 - 1, um2, um1, u0, ra, vm);
            lev1(j0, um1, u0, u1, rb, vc);
        }
        double xc[VEC] = {}, dc[VEC] = {};
        auto epi = [&](int jj, double (&xv)[VEC], double (&dd)[VEC]) {
            const i64 off = (i64)jj * N + il;
            if constexpr (CG) lde(a.x + off, xv);
            if constexpr (K2 == SR2_BI_P) lde(a.vd + off, dd);
        };
        epi(j0, xc, dc);
        for (int j = j0; j < j1; ++j) {
            // issue: raw inputs of line j+3, r of line j+2, epilogue of line j+1 (line j stands in past the last)
            Raw wn;
            raw(j + 3, wn);
            Rl rn;
            rld(j + 2, rn);
            double xn[VEC] = {}, dn[VEC] = {};
            epi(j + 1 < j1 ? j + 1 : j, xn, dn);
            Vl vp;  // level 1 at line j+1
            lev1(j + 1, u0, u1, u2, rc, vp);
            // level 2 at line j
            double left = __shfl_up(vc.t[VEC - 1], 1, 64);
            double right = __shfl_down(vc.t[0], 1, 64);
            left = e0l ? vc.ta : left;
            right = e63 ? vc.ta : right;
            left = i0 == 0 ? 0.0 : left;
            right = i0 + VEC >= N ? 0.0 : right;
            double y[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const double W = (k == 0) ? left : vc.t[k - 1];
                const double E = (k == VEC - 1) ? right : vc.t[k + 1];
                const double ax = sr_ax(vc.t[k], W, E, vp.t[k], vm.t[k]);
                y[k] = CG ? vc.t[k] + ca * (vc.v[k] - ax) : ax;
                if constexpr (CG) xc[k] = xc[k] + al * u0.u[k];
            }
            const i64 row = (i64)j * N;
            if (act) {
                if constexpr (!CG) sr_stv<VEC>(a.ou + row + i0, u0.u);
                sr_stv<VEC>(a.oy + row + i0, vc.v);
                sr_stv<VEC>(a.oz + row + i0, y);
                if constexpr (CG) sr_stv<VEC>(a.x + row + i0, xc);
            }
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                if constexpr (CG) {  // cg_x's <r, r> then cg_z's <r, z>
                    acc0 = act ? acc0 + vc.v[k] * vc.v[k] : acc0;
                    acc1 = act ? acc1 + vc.v[k] * y[k] : acc1;
                } else if constexpr (K2 == SR2_BI_P) {  // st1: <ap, r0>
                    acc0 = act ? acc0 + y[k] * dc[k] : acc0;
                } else {  // st2: <as, s>, <as, as>
                    acc0 = act ? acc0 + y[k] * u0.u[k] : acc0;
                    acc1 = act ? acc1 + y[k] * y[k] : acc1;
                }
            }
            // advance: line j+3 formed now that line j is done
            u0 = u1;
            u1 = u2;
            form(wn, u2);
            vm = vc;
            vc = vp;
            rc = rn;
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                xc[k] = xn[k];
                dc[k] = dn[k];
            }
        }
    }
    constexpr int NACC = K2 == SR2_BI_P ? 1 : 2;
    sr_publish<NACC>(a, acc0, acc1, blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y, sm, &last);
}

// Element-wise passes: grid-stride over double2 chunks, U in flight per thread.
template <int K, int U>
__global__ __launch_bounds__(TPB) void k_sr_vec(SrArgs a, i64 n) {
    __shared__ double sm[WAVES];
    __shared__ int last;
    if (a.sd->done) return;
    constexpr bool BX = K == SRV_BI_X || K == SRV_BI_XS;
    constexpr int NACC = BX ? 2 : K == SRV_DOT ? 1 : 0;
    const double al = a.sd->alpha, be = a.sd->beta, om = a.sd->omega;
    const i64 n2 = n >> 1;
    const i64 step = (i64)gridDim.x * TPB * U;
    double acc0 = 0.0, acc1 = 0.0;
    auto L = [](const double *p, i64 e) { return sr_ld2<(GK_SR_NT & 4) != 0>(p + 2 * e); };
    for (i64 b = (i64)blockIdx.x * TPB * U + threadIdx.x; b < n2; b += step) {
        double2 v0[U], v1[U], v2[U], v3[U], v4[U], v5[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = b + (i64)u * TPB;
            if (e < n2) {
                if (BX) {
                    v0[u] = L(a.x, e);
                    v1[u] = L(a.in0, e);  // z1
                    v3[u] = L(a.in2, e);  // s
                    v2[u] = K == SRV_BI_XS ? v3[u] : L(a.in1, e);  // z2
                    v4[u] = L(a.e0, e);   // as
                    v5[u] = L(a.vd, e);   // r0
                } else if (K == SRV_BI_PE) {
                    v0[u] = L(a.in0, e);
                    v1[u] = L(a.in1, e);
                    v2[u] = L(a.in2, e);
                } else {
                    v0[u] = L(a.in0, e);
                    v1[u] = L(a.in1, e);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const i64 e = b + (i64)u * TPB;
            if (e >= n2) continue;
            if constexpr (BX) {
                double2 xn, rn;
                xn.x = v0[u].x + al * v1[u].x + om * v2[u].x;
                xn.y = v0[u].y + al * v1[u].y + om * v2[u].y;
                rn.x = v3[u].x - om * v4[u].x;
                rn.y = v3[u].y - om * v4[u].y;
                sr_st2(a.x + 2 * e, xn);
                sr_st2(a.r + 2 * e, rn);
                acc0 = acc0 + rn.x * rn.x;
                acc0 = acc0 + rn.y * rn.y;
                acc1 = acc1 + rn.x * v5[u].x;
                acc1 = acc1 + rn.y * v5[u].y;
            } else if constexpr (K == SRV_BI_PE) {
                double2 o;
                o.x = v0[u].x + be * (v1[u].x - om * v2[u].x);
                o.y = v0[u].y + be * (v1[u].y - om * v2[u].y);
                sr_st2(a.ou + 2 * e, o);
            } else if constexpr (K == SRV_BI_SE) {
                double2 o;
                o.x = v0[u].x - al * v1[u].x;
                o.y = v0[u].y - al * v1[u].y;
                sr_st2(a.ou + 2 * e, o);
            } else {
                acc0 = acc0 + v0[u].x * v1[u].x;
                acc0 = acc0 + v0[u].y * v1[u].y;
            }
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {  // odd-length tail element
        const i64 e = n - 1;
        if constexpr (BX) {
            a.x[e] = a.x[e] + al * a.in0[e] + om * a.in1[e];
            const double rn = a.in2[e] - om * a.e0[e];
            a.r[e] = rn;
            acc0 = acc0 + rn * rn;
            acc1 = acc1 + rn * a.vd[e];
        } else if constexpr (K == SRV_BI_PE) {
            a.ou[e] = a.in0[e] + be * (a.in1[e] - om * a.in2[e]);
        } else if constexpr (K == SRV_BI_SE) {
            a.ou[e] = a.in0[e] - al * a.in1[e];
        } else {
            acc0 = acc0 + a.in0[e] * a.in1[e];
        }
    }
    if constexpr (NACC > 0) sr_publish<NACC>(a, acc0, acc1, blockIdx.x, gridDim.x, sm, &last);
}

// The finaliser as its own launch (N ranks: after the slab all-reduce; or
// after a generic preconditioner pass), one workgroup.
__global__ __launch_bounds__(TPB) void k_sr_fin(int mode, SrDev *sd, const double *p0, const double *p1, int np,
                                                double *hist, SrMirror *mir) {
    __shared__ double sm[WAVES];
    if (sd->done) return;
    sr_fin(mode, sd, p0, p1, np, hist, mir, sm);
}

}  // namespace gk
