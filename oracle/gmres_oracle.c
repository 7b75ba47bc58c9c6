/*
 * gmres_oracle.c -- CPU restatement of the reference GMRES(m) hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gmres_amd/, the C-ABI
 * library, the Fortran host) links, calls or loads this file.  It is used by
 * tests/ (as the checker), __graft_entry__.smoke() (as the checker) and
 * bench.py's cpu_baseline leg (as the reported CPU baseline, kind "port").
 *
 * It restates, loop for loop and in the same floating-point operation order,
 * the Fortran reference "Krylov Lab" (AlexanderGSC/gmres):
 *   - stvec            src/problems/poisson.f90:33-77
 *   - cbpr2            src/preconds/chebyshev.f90:8-38
 *   - gmres_mgsr_mf    src/gmres_mgsr.f90:98-199   (variant OR_MGSR_MF)
 *   - gmres_mgsr_omp   src/gmres_mgsr.f90:277-421  (variant OR_MGSR_OMP)
 *   - gmres_hh_omp     src/gmres_hh.f90:211-385    (midcycle_exit = 0)
 *   - gmres_hh_prec_omp src/gmres_hh.f90:388-566   (midcycle_exit = 1)
 *   - calculate_verr   src/gmres_hh.f90:568-593
 *   - pcg_omp          src/cg.f90:154-234
 *   - pbicgstab_omp    src/bicgstab.f90:91-182
 * plus two things the reference does not have:
 *   - an identity preconditioner (config 1 "no precond");
 *   - Chebyshev(k), the build-defined degree-k polynomial preconditioner of
 *     BASELINE config 3: k steps of the Chebyshev
 *     semi-iteration for A z = r from z = 0 on the interval given by params.
 *
 * Fortran intrinsics are restated as amdflang 22 (ROCm 7.2) implements them:
 *   dot_product -> sequential left-to-right sum of products (inlined loop);
 *   norm2       -> flang runtime Norm2Accumulator<8>: running max m and a
 *                  scaled sum s, result m*sqrt(1+s) (verified by disassembling
 *                  _FortranANorm2_8 / DoTotalReduction<double,Norm2Accumulator<8>>
 *                  in libflang_rt.runtime.a of this image);
 *   hypot       -> libm hypot;  sign(a,b) -> copysign(|a|, b).
 * Compile with -ffp-contract=off so that a*b+c is two roundings, as the
 * reference's x86-64 baseline build (no FMA) does.
 *
 * Vector layout: Fortran column-major grid, idx = i + j*N (0-based), i fastest.
 * With nthreads == 1 every reduction is sequential (the deterministic serial
 * oracle); with nthreads > 1 the dot/AXPY loops are OpenMP
 * work-shared like the *_omp reference (reduction order then unpinned).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define OR_PREC_IDENTITY 0
#define OR_PREC_CBPR2 1
#define OR_PREC_CHEB 2

#define OR_MGSR_MF 0
#define OR_MGSR_OMP 1

typedef long long i64;

static int g_nt = 1; /* OpenMP threads for the vector loops */

void or_set_threads(int nt) { g_nt = nt < 1 ? 1 : nt; }

/* ---------------------------------------------------------------- intrinsics */

/* flang norm2: src semantic of Fortran NORM2 as flang-rt computes it. */
double or_norm2(const double *x, i64 n) {
    double mx = 0.0, s = 0.0;
    for (i64 k = 0; k < n; ++k) {
        double a = fabs(x[k]);
        if (mx == 0.0) {
            mx = a;
        } else if (a > mx) {
            double t = mx / a;
            double tsq = t * t;
            s = s * tsq;
            s = s + tsq;
            mx = a;
        } else {
            double t = a / mx;
            s = s + t * t;
        }
    }
    return mx * sqrt(1.0 + s);
}

/* dot_product(a, b): sequential, or OpenMP reduction when g_nt > 1. */
double or_dot(const double *a, const double *b, i64 n) {
    double h = 0.0;
    if (g_nt > 1) {
#pragma omp parallel for num_threads(g_nt) reduction(+ : h) schedule(static)
        for (i64 k = 0; k < n; ++k) h = h + a[k] * b[k];
    } else {
        for (i64 k = 0; k < n; ++k) h = h + a[k] * b[k];
    }
    return h;
}

/* w = w - h*v   (gmres_mgsr.f90:354-358) */
static void axpy_minus(double *w, double h, const double *v, i64 n) {
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
    for (i64 k = 0; k < n; ++k) w[k] = w[k] - h * v[k];
}

/* w = w - 2*P*dot  (gmres_hh.f90:280, :301; written 2.0d0*P(idx,i)*dot) */
static void reflect_minus(double *w, double dot, const double *p, i64 n) {
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
    for (i64 k = 0; k < n; ++k) w[k] = w[k] - 2.0 * p[k] * dot;
}

static void div_into(double *dst, const double *src, double s, i64 n) {
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
    for (i64 k = 0; k < n; ++k) dst[k] = src[k] / s;
}

/* ------------------------------------------------------------------ operator */

/* y = A x, 2D Dirichlet 5-point Laplacian on an N x N grid
 * (src/problems/poisson.f90:33-77).  Sum order: ((W+E)+S)+Nn with missing
 * neighbours dropped, exactly as the interior/edge/corner statements of the
 * reference (:42, :48, :53, :58, :64, :70-76).  S = idx+N, Nn = idx-N. */
void or_stvec(const double *x, double *y, int N) {
    const i64 n = N;
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
    for (i64 j = 1; j < n - 1; ++j) {
        for (i64 i = 1; i < n - 1; ++i) {
            i64 idx = i + j * n;
            y[idx] = 4.0 * x[idx] - 1.0 * (x[idx - 1] + x[idx + 1] + x[idx + n] + x[idx - n]);
        }
    }
    for (i64 i = 1; i < n - 1; ++i) { /* col = 1 */
        y[i] = 4.0 * x[i] - 1.0 * (x[i - 1] + x[i + 1] + x[i + n]);
    }
    for (i64 i = 1; i < n - 1; ++i) { /* col = n */
        i64 idx = n * n - n + i;
        y[idx] = 4.0 * x[idx] - 1.0 * (x[idx - 1] + x[idx + 1] + x[idx - n]);
    }
    for (i64 j = 1; j < n - 1; ++j) { /* row = 1 */
        i64 idx = j * n;
        y[idx] = 4.0 * x[idx] - 1.0 * (x[idx + 1] + x[idx + n] + x[idx - n]);
    }
    for (i64 j = 1; j < n - 1; ++j) { /* row = n */
        i64 idx = j * n + n - 1;
        y[idx] = 4.0 * x[idx] - 1.0 * (x[idx - 1] + x[idx + n] + x[idx - n]);
    }
    /* corners (:69-76) */
    y[0] = 4.0 * x[0] - 1.0 * (x[1] + x[n]);
    y[n - 1] = 4.0 * x[n - 1] - 1.0 * (x[n - 2] + x[2 * n - 1]);
    {
        i64 idx = n * (n - 1);
        y[idx] = 4.0 * x[idx] - 1.0 * (x[idx + 1] + x[idx - n]);
        idx = n * (n - 1) + n - 1;
        y[idx] = 4.0 * x[idx] - 1.0 * (x[idx - 1] + x[idx - n]);
    }
}

/* --------------------------------------------------------- preconditioners */

/* cbpr2 coefficients (chebyshev.f90:19-26). */
void or_cbpr2_coeffs(const double *params, double *d_out, double *alpha_out) {
    double eigen_min = params[0], eigen_max = params[1];
    double c = (eigen_max - eigen_min) / 2.0;
    double d = (eigen_max + eigen_min) / 2.0;
    double alpha = 1.0 / d;
    double beta = (c * alpha / 2.0);
    beta = beta * beta;
    alpha = 1.0 / (d - beta);
    *d_out = d;
    *alpha_out = alpha;
}

/* Chebyshev(k) scalars: theta = (a+b)/2, delta = |b-a|/2, sigma = theta/delta. */
void or_cheb_coeffs(const double *params, double *theta, double *delta) {
    double a = params[0], b = params[1];
    *theta = (a + b) / 2.0;
    *delta = fabs(b - a) / 2.0;
}

/* z = M^-1 r.  aux, aux2: caller scratch of length N*N (aux2 only for CHEB). */
void or_precond(int kind, const double *r, double *z, double *aux, double *aux2,
                const double *params, int degree, int N) {
    const i64 n = (i64)N * N;
    if (kind == OR_PREC_IDENTITY) {
        memcpy(z, r, sizeof(double) * n);
        return;
    }
    if (kind == OR_PREC_CBPR2) { /* chebyshev.f90:27-37 */
        double d, alpha;
        or_cbpr2_coeffs(params, &d, &alpha);
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
        for (i64 k = 0; k < n; ++k) z[k] = r[k] / d;
        or_stvec(z, aux, N);
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
        for (i64 k = 0; k < n; ++k) z[k] = z[k] + alpha * (r[k] - aux[k]);
        return;
    }
    /* OR_PREC_CHEB: Chebyshev semi-iteration, `degree` applications of A.
     *   res = r; d = res/theta; z = d; rho0 = delta/theta
     *   repeat degree times:
     *     res = res - A d
     *     rho1 = 1/(2 sigma - rho0)
     *     d = (rho1*rho0)*d + (2 rho1/delta)*res
     *     z = z + d;  rho0 = rho1
     * aux = res (working residual), aux2 = A d. */
    {
        double theta, delta;
        or_cheb_coeffs(params, &theta, &delta);
        double sigma = theta / delta;
        double rho0 = delta / theta;
        double *res = aux, *ad = aux2;
        double *dv = (double *)malloc(sizeof(double) * n);
        for (i64 k = 0; k < n; ++k) {
            res[k] = r[k];
            dv[k] = r[k] / theta;
            z[k] = dv[k];
        }
        for (int it = 0; it < degree; ++it) {
            double rho1 = 1.0 / (2.0 * sigma - rho0);
            double c1 = rho1 * rho0, c2 = 2.0 * rho1 / delta;
            or_stvec(dv, ad, N);
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
            for (i64 k = 0; k < n; ++k) {
                double rr = res[k] - ad[k];
                double dd = c1 * dv[k] + c2 * rr;
                res[k] = rr;
                dv[k] = dd;
                z[k] = z[k] + dd;
            }
            rho0 = rho1;
        }
        free(dv);
    }
}

/* ------------------------------------------------------- Givens & backsolve */

/* Column j (0-based) of H (ld = m+1): apply old rotations, make a new one,
 * rotate g  (gmres_mgsr.f90:364-383). */
static void givens_step(double *H, int ld, double *cs, double *sn, double *g, int j) {
    double *h = H + (i64)j * ld;
    for (int i = 0; i < j; ++i) {
        double tmp = h[i];
        h[i] = cs[i] * tmp + sn[i] * h[i + 1];
        h[i + 1] = -sn[i] * tmp + cs[i] * h[i + 1];
    }
    double ds = hypot(h[j + 1], h[j]);
    cs[j] = h[j] / ds;
    sn[j] = h[j + 1] / ds;
    h[j] = cs[j] * h[j] + sn[j] * h[j + 1];
    h[j + 1] = 0.0;
    double tmp = g[j];
    g[j] = cs[j] * tmp + sn[j] * g[j + 1];
    g[j + 1] = -sn[j] * tmp + cs[j] * g[j + 1];
}

/* y(n_out) = g/H; y(i) = (g(i) - dot_product(H(i,i+1:n_out), y(i+1:n_out)))/H(i,i) */
static void back_solve(const double *H, int ld, const double *g, double *y, int m, int n_out) {
    for (int i = 0; i < m; ++i) y[i] = 0.0;
    y[n_out - 1] = g[n_out - 1] / H[(i64)(n_out - 1) * ld + (n_out - 1)];
    for (int i = n_out - 2; i >= 0; --i) {
        double s = 0.0;
        for (int k = i + 1; k < n_out; ++k) s = s + H[(i64)k * ld + i] * y[k];
        y[i] = (g[i] - s) / H[(i64)i * ld + i];
    }
}

static double true_rel_residual(const double *b, const double *x, double *tmp, int N, double bnorm) {
    const i64 n = (i64)N * N;
    or_stvec(x, tmp, N);
    for (i64 k = 0; k < n; ++k) tmp[k] = b[k] - tmp[k];
    return or_norm2(tmp, n) / bnorm;
}

/* ------------------------------------------------------------- GMRES MGS-R */

/*
 * Restarted left-preconditioned GMRES(m) with MGS + one re-orthogonalisation.
 * variant OR_MGSR_MF  = gmres_mgsr_mf  (gmres_mgsr.f90:98-199)
 * variant OR_MGSR_OMP = gmres_mgsr_omp (gmres_mgsr.f90:277-421): no in-loop
 *   exit, V(:,j+1) always written, `converged` latch (:335, :385-389).
 * Outputs: x (n), final_err (m, last cycle), v_err (m+1), n_out, restart_out.
 * Optional histories (may be NULL): hist_res[c] = ||b - A x_c||/||b|| after
 * cycle c; hist_ferr[c*m + j] = final_err(j) of cycle c.  *n_cycles = cycles run.
 * step_limit > 0 stops after that many Arnoldi steps in total (bounded CPU
 * baseline sample); step_times (may be NULL) receives omp_get_wtime() after
 * each step.  Returns 0, or 1 if step_limit cut the run short.
 */
int or_gmres_mgsr(const double *b, int N, int m, double tol, int prec, const double *params,
                  int degree, int variant, int max_restarts, double *x, double *final_err,
                  double *v_err, int *n_out_p, int *restart_out, double *hist_res,
                  double *hist_ferr, int *n_cycles, int step_limit, double *step_times) {
    const i64 n = (i64)N * N;
    const int ld = m + 1;
    double *V = (double *)calloc((size_t)n * (m + 1), sizeof(double));
    double *H = (double *)calloc((size_t)(m + 1) * m, sizeof(double));
    double *w = (double *)malloc(sizeof(double) * n);
    double *z = (double *)malloc(sizeof(double) * n);
    double *aux = (double *)malloc(sizeof(double) * n);
    double *aux2 = (double *)malloc(sizeof(double) * n);
    double *g = (double *)calloc(m + 1, sizeof(double));
    double *y = (double *)calloc(m, sizeof(double));
    double *cs = (double *)calloc(m, sizeof(double));
    double *sn = (double *)calloc(m, sizeof(double));
    int n_out = 0, converged = 0, cut = 0, steps = 0, st;
    double h_val = 0.0;
    for (int k = 0; k < m; ++k) final_err[k] = 0.0;
    for (int k = 0; k <= m; ++k) v_err[k] = 0.0;
    for (i64 k = 0; k < n; ++k) x[k] = 0.0;
    *restart_out = 0;
    double beta0 = or_norm2(b, n);
    for (st = 1; st <= max_restarts; ++st) {
        memset(g, 0, sizeof(double) * (m + 1));
        memset(H, 0, sizeof(double) * (m + 1) * m);
        if (variant == OR_MGSR_MF) memset(V, 0, sizeof(double) * n * (m + 1));
        or_stvec(x, w, N);
        for (i64 k = 0; k < n; ++k) z[k] = b[k] - w[k];
        or_precond(prec, z, w, aux, aux2, params, degree, N);
        double beta = or_norm2(w, n);
        g[0] = beta;
        div_into(V, w, beta, n);
        for (int j = 0; j < m; ++j) {
            if (converged) break; /* `if (converged) cycle` (:335) */
            n_out = j + 1;
            or_stvec(V + (i64)j * n, z, N);
            or_precond(prec, z, w, aux, aux2, params, degree, N);
            double *Hj = H + (i64)j * ld;
            for (int k = 0; k < 2; ++k) {
                for (int i = 0; i <= j; ++i) {
                    double h_tmp = or_dot(w, V + (i64)i * n, n);
                    Hj[i] = Hj[i] + h_tmp;
                    axpy_minus(w, h_tmp, V + (i64)i * n, n);
                }
            }
            h_val = or_norm2(w, n);
            Hj[j + 1] = h_val;
            givens_step(H, ld, cs, sn, g, j);
            final_err[j] = fabs(g[j + 1]) / beta0;
            if (hist_ferr) hist_ferr[(i64)(st - 1) * m + j] = final_err[j];
            ++steps;
            if (step_times) step_times[steps - 1] = omp_get_wtime();
            if (variant == OR_MGSR_MF) {
                if (h_val < tol || final_err[j] < tol) {
                    n_out = j + 1;
                    break;
                }
                div_into(V + (i64)(j + 1) * n, w, h_val, n);
            } else {
                div_into(V + (i64)(j + 1) * n, w, h_val, n);
                if (final_err[j] < tol) {
                    *restart_out = st;
                    converged = 1;
                }
            }
            if (step_limit > 0 && steps >= step_limit) {
                cut = 1;
                break;
            }
        }
        if (cut) break;
        back_solve(H, ld, g, y, m, n_out);
        /* x(idx) = x(idx) + dot_product(V(idx,1:n_out), y(1:n_out))  (:400-406) */
#pragma omp parallel for num_threads(g_nt) if (g_nt > 1) schedule(static)
        for (i64 e = 0; e < n; ++e) {
            double s = 0.0;
            for (int k = 0; k < n_out; ++k) s = s + V[(i64)k * n + e] * y[k];
            x[e] = x[e] + s;
        }
        if (hist_res) hist_res[st - 1] = true_rel_residual(b, x, aux, N, beta0);
        if (n_cycles) *n_cycles = st;
        if (h_val < tol || final_err[n_out - 1] < tol) {
            *restart_out = st;
            break;
        }
    }
    if (!cut) {
        if (st > max_restarts) *restart_out = max_restarts;
        /* v_err epilogue (:414-420) */
        for (int j = 1; j <= n_out; ++j) {
            const double *vj1 = V + (i64)j * n;
            for (int i = 1; i <= j; ++i) {
                double d = or_dot(V + (i64)(i - 1) * n, vj1, n);
                v_err[j] = v_err[j] + 2.0 * (d * d);
            }
            double dd = or_dot(vj1, vj1, n) - 1.0;
            v_err[j] = v_err[j] + dd * dd;
            v_err[j] = sqrt(v_err[j - 1] * v_err[j - 1] + v_err[j]);
        }
    }
    *n_out_p = n_out;
    free(V); free(H); free(w); free(z); free(aux); free(aux2);
    free(g); free(y); free(cs); free(sn);
    return cut;
}

/* ----------------------------------------------------------- GMRES Householder */

/* calculate_verr (gmres_hh.f90:568-593): rebuild V = P_1..P_i e_i, then
 * v_err(i) += sum_{j<i} 2 (V_i . V_j)^2 (squared, not cumulative);
 * x = V y. */
static void calculate_verr(const double *P, double *x, const double *y, double *v_err,
                           int n_iter, i64 n) {
    double *V = (double *)calloc((size_t)n * n_iter, sizeof(double));
    for (int i = 0; i < n_iter; ++i) V[(i64)i * n + i] = 1.0;
    for (int i = 0; i < n_iter; ++i) {
        double *vi = V + (i64)i * n;
        for (int j = i; j >= 0; --j) {
            double d = or_dot(vi, P + (i64)j * n, n);
            reflect_minus(vi, d, P + (i64)j * n, n);
        }
    }
    for (int i = 1; i < n_iter; ++i) {
        for (int j = 0; j < i; ++j) {
            double d = or_dot(V + (i64)i * n, V + (i64)j * n, n);
            v_err[i] = v_err[i] + 2.0 * (d * d);
        }
    }
    for (i64 e = 0; e < n; ++e) {
        double s = 0.0;
        for (int k = 0; k < n_iter; ++k) s = s + V[(i64)k * n + e] * y[k];
        x[e] = s;
    }
    free(V);
}

/*
 * Householder GMRES(m) (Walker '88 style), matrix-free.
 * midcycle_exit = 0: gmres_hh_omp (gmres_hh.f90:211-385) -- no preconditioner
 *   application at cycle start (w = b - A x directly, :243-253), every cycle runs
 *   the full m steps (exit commented out, :340-344); pass prec = IDENTITY.
 * midcycle_exit = 1: gmres_hh_prec_omp (:388-566) -- z = b - A x, w = M^-1 z,
 *   `converged` latch skips the rest of the cycle (:439, :521-525).
 * Histories as in or_gmres_mgsr.
 */
int or_gmres_hh(const double *b, int N, int m, double tol, int prec, const double *params,
                int degree, int midcycle_exit, int max_stages, double *x, double *final_err,
                double *v_err, int *n_out_p, int *stages_out, double *hist_res,
                double *hist_ferr, int *n_cycles, int step_limit, double *step_times) {
    const i64 n = (i64)N * N;
    const int ld = m + 1;
    double *P = (double *)calloc((size_t)n * (m + 1), sizeof(double));
    double *H = (double *)calloc((size_t)(m + 1) * m, sizeof(double));
    double *w = (double *)malloc(sizeof(double) * n);
    double *z = (double *)malloc(sizeof(double) * n);
    double *vj = (double *)malloc(sizeof(double) * n);
    double *aux = (double *)malloc(sizeof(double) * n);
    double *aux2 = (double *)malloc(sizeof(double) * n);
    double *g = (double *)calloc(m + 1, sizeof(double));
    double *y = (double *)calloc(m, sizeof(double));
    double *cs = (double *)calloc(m, sizeof(double));
    double *sn = (double *)calloc(m, sizeof(double));
    int n_out = 0, converged = 0, cut = 0, steps = 0;
    double h_val = 0.0;
    for (int k = 0; k < m; ++k) final_err[k] = 0.0;
    for (int k = 0; k <= m; ++k) v_err[k] = 0.0;
    for (i64 k = 0; k < n; ++k) x[k] = 0.0;
    *stages_out = 0;
    double beta0 = or_norm2(b, n);
    for (int k = 1; k <= max_stages; ++k) {
        memset(g, 0, sizeof(double) * (m + 1));
        memset(P, 0, sizeof(double) * n * (m + 1));
        memset(H, 0, sizeof(double) * (m + 1) * m);
        or_stvec(x, w, N);
        if (midcycle_exit) {
            for (i64 e = 0; e < n; ++e) z[e] = b[e] - w[e];
            or_precond(prec, z, w, aux, aux2, params, degree, N);
        } else {
            for (i64 e = 0; e < n; ++e) w[e] = b[e] - w[e];
        }
        double beta = or_norm2(w, n);
        g[0] = -copysign(fabs(beta), w[0]);
        w[0] = copysign(fabs(beta), w[0]) + w[0];
        div_into(P, w, or_norm2(w, n), n);
        for (int j = 0; j < m; ++j) {
            if (converged) break;
            for (i64 e = 0; e < n; ++e) vj[e] = 0.0;
            n_out = j + 1;
            vj[j] = 1.0;
            for (int i = j; i >= 0; --i) {
                double d = or_dot(vj, P + (i64)i * n, n);
                reflect_minus(vj, d, P + (i64)i * n, n);
            }
            if (midcycle_exit) {
                or_stvec(vj, z, N);
                or_precond(prec, z, w, aux, aux2, params, degree, N);
            } else {
                or_stvec(vj, w, N);
            }
            for (int i = 0; i <= j; ++i) {
                double d = or_dot(w, P + (i64)i * n, n);
                reflect_minus(w, d, P + (i64)i * n, n);
            }
            double *Hj = H + (i64)j * ld;
            for (int i = 0; i <= j; ++i) Hj[i] = w[i];
            if (j + 1 < n) {
                double tmp = or_norm2(w + j + 1, n - j - 1);
                Hj[j + 1] = (w[j + 1] > 0.0) ? -tmp : tmp;
                h_val = fabs(Hj[j + 1]);
                for (int i = 0; i <= j; ++i) w[i] = 0.0;
                w[j + 1] = w[j + 1] - Hj[j + 1];
                double nw = or_norm2(w, n);
                div_into(w, w, nw, n);
                memcpy(P + (i64)(j + 1) * n, w, sizeof(double) * n);
            } else {
                Hj[j + 1] = 0.0;
            }
            givens_step(H, ld, cs, sn, g, j);
            final_err[j] = fabs(g[j + 1]) / beta0;
            if (hist_ferr) hist_ferr[(i64)(k - 1) * m + j] = final_err[j];
            ++steps;
            if (step_times) step_times[steps - 1] = omp_get_wtime();
            if (midcycle_exit && final_err[j] < tol) {
                n_out = j + 1;
                *stages_out = k;
                converged = 1;
            }
            if (step_limit > 0 && steps >= step_limit) {
                cut = 1;
                break;
            }
        }
        if (cut) break;
        back_solve(H, ld, g, y, m, n_out);
        for (i64 e = 0; e < n; ++e) w[e] = 0.0;
        for (int i = 0; i < n_out; ++i) w[i] = y[i];
        for (int i = n_out - 1; i >= 0; --i) {
            double d = or_dot(w, P + (i64)i * n, n);
            reflect_minus(w, d, P + (i64)i * n, n);
        }
        for (i64 e = 0; e < n; ++e) x[e] = x[e] + w[e];
        if (hist_res) hist_res[k - 1] = true_rel_residual(b, x, aux, N, beta0);
        if (n_cycles) *n_cycles = k;
        *stages_out = k;
        if (final_err[n_out - 1] < tol) break;
    }
    if (!cut) calculate_verr(P, w, y, v_err, n_out, n);
    (void)h_val;
    *n_out_p = n_out;
    free(P); free(H); free(w); free(z); free(vj); free(aux); free(aux2);
    free(g); free(y); free(cs); free(sn);
    return cut;
}

/* -------------------------------------------------------- CG / BiCGSTAB ---- */

/* pcg_omp (src/cg.f90:154-234): x0 = 0, r = b, z = M^-1 r, p = z; per
 * iteration rr = <r,z>, alpha = rr/<Ap,p>; x += alpha p; r -= alpha Ap;
 * res = sqrt(<r,r>); z = M^-1 r; beta = <r,z>/rr; p = z + beta p.
 * *iter in: max iterations, out: first i with res < tol (unchanged if never).
 * hist_res[i-1] = res of iteration i (may be NULL). */
void or_pcg(const double *b, int N, double tol, int *iter, double *res_out, int prec, const double *params,
            int degree, double *x, double *hist_res) {
    const i64 n = (i64)N * N;
    double *ax = (double *)malloc(sizeof(double) * n), *p = (double *)malloc(sizeof(double) * n);
    double *r = (double *)calloc((size_t)n, sizeof(double)), *z = (double *)malloc(sizeof(double) * n);
    double *aux = (double *)malloc(sizeof(double) * n), *aux2 = (double *)malloc(sizeof(double) * n);
    int maxit = *iter, converged = 0;
    double res = 0.0;
    for (i64 j = 0; j < n; ++j) {
        x[j] = 0.0;
        r[j] = b[j];
    }
    or_precond(prec, r, z, aux, aux2, params, degree, N);
    for (i64 j = 0; j < n; ++j) p[j] = z[j];
    for (int i = 1; i <= maxit; ++i) {
        if (converged) break;
        or_stvec(p, ax, N);
        double rr = 0.0, alpha = 0.0, beta = 0.0;
        res = 0.0;
        for (i64 j = 0; j < n; ++j) {
            rr = rr + r[j] * z[j];
            alpha = alpha + ax[j] * p[j];
        }
        alpha = rr / alpha;
        for (i64 j = 0; j < n; ++j) {
            x[j] = x[j] + alpha * p[j];
            r[j] = r[j] - alpha * ax[j];
            res = res + r[j] * r[j];
        }
        or_precond(prec, r, z, aux, aux2, params, degree, N);
        for (i64 j = 0; j < n; ++j) beta = beta + r[j] * z[j];
        res = sqrt(res);
        beta = beta / rr;
        if (hist_res) hist_res[i - 1] = res;
        if (res < tol) {
            converged = 1;
            *iter = i;
        }
        for (i64 j = 0; j < n; ++j) p[j] = z[j] + beta * p[j];
    }
    *res_out = res;
    free(ax); free(p); free(r); free(z); free(aux); free(aux2);
}

/* pbicgstab_omp (src/bicgstab.f90:91-182); the reference leaves its dot
 * accumulators uninitialised before the first iteration (:102, :123-126):
 * they start at 0 here. */
void or_pbicgstab(const double *b, int N, double tol, int *max_iter, double *res_out, int prec,
                  const double *params, int degree, double *x, double *hist_res) {
    const i64 n = (i64)N * N;
    double *r = (double *)malloc(sizeof(double) * n), *r0 = (double *)malloc(sizeof(double) * n);
    double *ap = (double *)malloc(sizeof(double) * n), *s = (double *)malloc(sizeof(double) * n);
    double *as = (double *)malloc(sizeof(double) * n), *p = (double *)malloc(sizeof(double) * n);
    double *z1 = (double *)malloc(sizeof(double) * n), *z2 = (double *)malloc(sizeof(double) * n);
    double *aux = (double *)malloc(sizeof(double) * n), *aux2 = (double *)malloc(sizeof(double) * n);
    int converged = 0, iters = *max_iter;
    double rr0 = 0.0, ap_r0 = 0.0, as_s = 0.0, as_as = 0.0, r_r0_new = 0.0, res = 0.0;
    for (i64 j = 0; j < n; ++j) {
        x[j] = 0.0;
        r[j] = b[j];
        r0[j] = r[j];
        p[j] = r0[j];
    }
    for (int i = 1; i <= *max_iter; ++i) {
        if (converged) break;
        or_precond(prec, p, z1, aux, aux2, params, degree, N);
        or_stvec(z1, ap, N);
        for (i64 j = 0; j < n; ++j) {
            rr0 = rr0 + r[j] * r0[j];
            ap_r0 = ap_r0 + ap[j] * r0[j];
        }
        double alpha = rr0 / ap_r0;
        for (i64 j = 0; j < n; ++j) s[j] = r[j] - alpha * ap[j];
        or_precond(prec, s, z2, aux, aux2, params, degree, N);
        or_stvec(z2, as, N);
        for (i64 j = 0; j < n; ++j) {
            as_s = as_s + as[j] * s[j];
            as_as = as_as + as[j] * as[j];
        }
        double omega = as_s / as_as;
        for (i64 j = 0; j < n; ++j) {
            x[j] = x[j] + alpha * z1[j] + omega * z2[j];
            r[j] = s[j] - omega * as[j];
        }
        res = or_norm2(r, n);
        if (hist_res) hist_res[i - 1] = res;
        if (res < tol) {
            iters = i;
            converged = 1;
        }
        for (i64 j = 0; j < n; ++j) r_r0_new = r_r0_new + r[j] * r0[j];
        double beta = (r_r0_new / rr0) * (alpha / omega);
        r_r0_new = 0.0;
        as_s = 0.0;
        as_as = 0.0;
        rr0 = 0.0;
        ap_r0 = 0.0;
        for (i64 j = 0; j < n; ++j) p[j] = r[j] + beta * (p[j] - omega * ap[j]);
    }
    *max_iter = iters;
    *res_out = res;
    free(r); free(r0); free(ap); free(s); free(as); free(p); free(z1); free(z2); free(aux); free(aux2);
}
