/*
 * gmres_hip.h -- C-ABI of libgmres_hip.so, the MI355X (gfx950) device side of
 * the restarted GMRES(m) inner cycle for the 2D Poisson 5-point operator.
 *
 * Drop-in boundary.  The reference (AlexanderGSC/gmres, Fortran) plugs its
 * operator and preconditioner into the solvers through two abstract
 * interfaces (src/interfaces.f90:13-17 `stencil_vector(x,y,n)` and
 * :20-27 `precond(A_x,r,z,aux,params,n)`), and the solvers
 * (src/gmres_mgsr.f90:277-421 gmres_mgsr_omp, :98-199 gmres_mgsr_mf,
 * src/gmres_hh.f90:211-385 gmres_hh_omp, :388-566 gmres_hh_prec_omp) run the
 * Arnoldi cycle on host arrays.  This library replaces the vector work of
 * those solvers with HIP kernels on device-resident data; the small
 * Hessenberg / Givens / back-solve work stays on the host (Fortran module
 * gmres_amd/fortran/gmres_hip.f90 binds these symbols with ISO_C_BINDING).
 *
 * Conventions
 *   - Every function returns int status: GK_OK (0) or a negative GK_ERR_*;
 *     gk_last_error() returns a message for the calling thread's last error.
 *   - Grid: N x N ("nside"), Fortran column-major, idx = i + (j-1)*N with i
 *     fastest.  A context owns the slab of grid lines j in [line0, line0+nlines)
 *     (0-based line0); nloc = N*nlines local unknowns.  Single GPU:
 *     line0 = 0, nlines = N.
 *   - Host arrays are plain double* of the local length; device pointers in
 *     the stateless kernel API are plain device addresses (16-byte aligned).
 *   - `j` arguments are 1-based Arnoldi step numbers as in the reference.
 *   - A context is single-host-thread, stream-ordered, not re-entrant.
 */
#ifndef GMRES_HIP_H
#define GMRES_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define GK_OK 0
#define GK_ERR_ARG (-1)   /* bad argument (shape, range, alignment, order) */
#define GK_ERR_HIP (-2)   /* HIP runtime error */
#define GK_ERR_RCCL (-3)  /* RCCL error */
#define GK_ERR_STATE (-4) /* call out of order (e.g. step before cycle start) */
#define GK_ERR_NOMEM (-5) /* device allocation failed */
#define GK_ERR_COMM (-6)  /* device exchange: a peer missed its deadline (see gk_comm_init_xgmi) */

/* Preconditioner kinds (the reference's `precond` plug-ins). */
#define GK_PREC_IDENTITY 0 /* z = r ; config 1 "no precond"  */
#define GK_PREC_CBPR2 1    /* src/preconds/chebyshev.f90:8-38, params(1:2) */
#define GK_PREC_CHEB 2     /* Chebyshev(k) semi-iteration, build-defined (BASELINE config 3) */

/* Kernel ids for gk_profile_read(). */
#define GK_KID_PROJ 0    /* fused MGS-R / Householder projection (axpy_i + dot_{i+1}) */
#define GK_KID_STENCIL 1 /* Poisson-5 stencil sweeps incl. fused preconditioner sweeps */
#define GK_KID_SCALE 2   /* normalisation V(:,j+1) = w / h */
#define GK_KID_UPDATE 3  /* x += V y */
#define GK_KID_COMM 4    /* all-reduce / broadcast (RCCL, local group or device exchange) */
#define GK_KID_OTHER 5
#define GK_KID_RES 6     /* resident MGS-R step: whole cascade + norm + scale in one launch */
#define GK_KID_PREC 7    /* temporal-blocked Chebyshev(k) passes (k_cheb_fused) */
#define GK_KID_HALO 8    /* halo lines with the slab neighbours (RCCL send/recv, local group or device exchange) */
#define GK_KID_GRAPH 9   /* one launch-path MGS-R step replayed as a hipGraph (its 2j projections, all-reduces, scale) */
/* short-recurrence passes (gk_sr_*): GK_KID_SR + the pass kind of gk_sr.hpp --
 * 0 cg_p, 1 cg_x, 2 cg_z, 3 bi_p, 4 bi_pc, 5 bi_s, 6 bi_sc, 7 st1, 8 st2 (line
 * marches), 9 bi_x, 10 bi_pe, 11 bi_se, 12 dot (element-wise), 13 cg_xz, 14 bi_pz,
 * 15 bi_sz (two-level marches: cbpr2 and the operator in one pass) */
#define GK_KID_SR 10
#define GK_NKID 26

typedef struct gk_ctx gk_ctx;
typedef struct gk_group gk_group;

const char *gk_last_error(void);
int gk_version(void);
/* Which runtime this library is running on (bench.py / smoke() report it):
 * hipRuntimeGetVersion, hipDriverGetVersion, ncclGetVersion, and the files the
 * process mapped for libamdhip64 and librccl (dladdr of one of their symbols),
 * NUL-terminated into hip_path / rccl_path (capacity `len` bytes each). */
int gk_runtime_info(int *hip_runtime, int *hip_driver, int *rccl, char *hip_path, char *rccl_path, int len);

/* ------------------------------------------------------------ context ---- */
/* Create a context on HIP device `device` for an N x N grid, owning lines
 * [line0, line0+nlines), Krylov dimension m (restart length).  Allocates
 * V (n x (m+1)), the work vectors and the reduction slabs in HBM. */
int gk_create(int device, int nside, int line0, int nlines, int m, gk_ctx **out);
int gk_destroy(gk_ctx *ctx);
/* Multi-GPU: rank 0 calls gk_comm_unique_id, the 128 bytes are shared out of
 * band, then every rank calls gk_comm_init.  Ranks own consecutive slabs
 * (rank r-1 below rank r).  `max_lines` = the largest nlines of any rank. */
int gk_comm_unique_id(unsigned char id[128]);
int gk_comm_init(gk_ctx *ctx, int nranks, int rank, int max_lines, const unsigned char id[128]);
/* In-process communicator with the same message pattern as RCCL: nranks
 * contexts of ONE process (any devices, e.g. all on one GPU for testing the
 * slab decomposition), each driven by its own host thread. */
int gk_group_create(int nranks, gk_group **out);
int gk_group_destroy(gk_group *g);
int gk_comm_init_local(gk_ctx *ctx, gk_group *g, int rank, int max_lines);
/* Device exchange ("xgmi" back-end, SURVEY 8e "custom xGMI flag-based
 * all-reduce"): the per-projection all-reduces, the Householder broadcast and
 * the halo lines are moved by the GPUs themselves -- each rank stores tagged
 * 8-byte granules straight into every peer's receive region over xGMI, and
 * the consumer polls its own region -- instead of one RCCL call per
 * reduction.  Same results on every rank (rank-order sums).
 *   gk_comm_init_xgmi   decomposition without RCCL (ranks on distinct GPUs,
 *                       or several processes on one GPU);
 *   gk_xchg_handle      this rank's IPC handle (64 bytes) to share out of band;
 *   gk_xchg_open        map every rank's region (handles: nranks x 64 bytes,
 *                       rank order) and route collectives through it;
 *   gk_xchg_local       the same for a gk_group (in-process, after every
 *                       member's gk_comm_init_local); GK_ERR_STATE at once
 *                       when the members on this device, plus one stream
 *                       (the null stream), exceed the process's hardware
 *                       queues (GPU_MAX_HW_QUEUES, HIP's default 4): streams
 *                       would share a queue, and a spinning exchange kernel
 *                       could sit in front of its peer's kernel until the
 *                       deadline;
 *   gk_xchg_enable      0: back to RCCL / the local group, 1: device exchange;
 *   gk_xchg_selftest    collective check of the reduction and halo paths with
 *                       a deadline; GK_ERR_COMM if any granule is missing or
 *                       wrong.  Also usable after gk_comm_init (RCCL present):
 *                       a failed test leaves the exchange disabled.  (Tests:
 *                       env GK_DEBUG_SELFTEST_FAIL=<rank> makes that rank fail
 *                       at once without taking part; its peers then miss
 *                       their deadline.)
 * Usable together with gk_comm_init (then RCCL remains the fallback).
 * A missed deadline during a solve (GK_ERR_COMM, naming the late rank or
 * workgroup) retires the exchange of that context: its later exchanges fail at
 * once and gk_xchg_enable(1) refuses.  It does NOT switch back to RCCL by
 * itself -- the caller does, on EVERY rank together, with gk_xchg_enable(0)
 * (switching only the rank that saw the miss would desynchronise the ranks). */
int gk_comm_init_xgmi(gk_ctx *ctx, int nranks, int rank, int max_lines);
int gk_xchg_handle(gk_ctx *ctx, unsigned char handle[64]);
int gk_xchg_open(gk_ctx *ctx, const unsigned char *handles);
int gk_xchg_local(gk_ctx *ctx);
int gk_xchg_enable(gk_ctx *ctx, int on);
int gk_xchg_selftest(gk_ctx *ctx, int timeout_ms);
int gk_local_size(gk_ctx *ctx, long long *nloc);
/* What this context's collectives actually run on: kind = GK_COMM_NONE (single
 * rank), GK_COMM_RCCL, GK_COMM_LOCAL (gk_group) or GK_COMM_XGMI (device
 * exchange on); nranks_seen = the communicator's own rank count (ncclCommCount
 * for RCCL, the mapped exchange regions for the device exchange). */
#define GK_COMM_NONE 0
#define GK_COMM_RCCL 1
#define GK_COMM_LOCAL 2
#define GK_COMM_XGMI 3
int gk_comm_info(gk_ctx *ctx, int *kind, int *nranks_seen);
/* First contact between two devices of the node (no context needed): whether
 * `device` can map `peer`'s memory (hipDeviceCanAccessPeer) and the link type
 * and hop count between them (hipExtGetLinkTypeAndHopCount; link_type as HIP's
 * HSA_AMD_LINK_INFO_TYPE: 4 = xGMI, 2 = PCIe).  bench.py logs it for every rank
 * pair of an N-GPU line.  device == peer: can_access 1, hops 0. */
int gk_peer_info(int device, int peer, int *can_access, int *link_type, int *hops);
/* Collective, every rank together: the mean cost (us, HIP events on the
 * context stream) of one all-reduce of a projection's partial slab and of one
 * halo exchange (one grid line with each neighbour) through the collective in
 * use (device exchange, RCCL or the local group), over `iters` back-to-back
 * calls.  Diagnostic (bench.py reports it beside a multi-GPU line); leaves
 * the reduction slots and halo buffers overwritten. */
int gk_comm_latency(gk_ctx *ctx, int iters, double *allreduce_us, double *halo_us);

/* Preconditioner: kind GK_PREC_*, params (cbpr2: params[0..1] as
 * chebyshev.f90:19-25; CHEB: interval ends params[0..1]), degree (CHEB only). */
int gk_set_precond(gk_ctx *ctx, int kind, const double *params, int nparams, int degree);
/* Right-hand side b (local part, host) or b = A*1 built on device
 * (the manufactured RHS of every reference driver, test_poisson_mf.f90:39-40). */
int gk_set_rhs(gk_ctx *ctx, const double *b_local);
int gk_set_rhs_ones(gk_ctx *ctx);
/* beta0 = ||b||_2 (global). */
int gk_rhs_norm(gk_ctx *ctx, double *beta0);
/* x = 0 (x0 is always 0 in the reference, gmres_mgsr.f90:304). */
int gk_zero_x(gk_ctx *ctx);
int gk_get_x(gk_ctx *ctx, double *x_local);
/* Copy column col (0-based) of a device basis to the host (nloc doubles):
 * which = 0: V(:,col+1) -- the MGS-R Krylov basis, or the Householder
 * reflectors P(:,col+1) (gmres_hh.f90 keeps P in the same array);
 * which = 1: the Householder basis rebuilt by gk_hh_verr (calculate_verr's V).
 * Diagnostic only (the orthogonality tests evaluate the reference's formula on
 * the device basis). */
int gk_get_basis(gk_ctx *ctx, int which, int col, double *out);
int gk_set_x(gk_ctx *ctx, const double *x_local);
/* Host-array operator application on this context's slab (clobbers the
 * work vectors; not between cycle start and update):  what = 0: out = A in
 * (stencil_vector, poisson.f90:33-77); what = 1: out = M^-1 in (precond). */
int gk_apply(gk_ctx *ctx, int what, const double *in, double *out);
/* ||b - A x|| / ||b|| (global, true unpreconditioned residual). */
int gk_true_residual(gk_ctx *ctx, double *rel);

/* -------------------------------------------- MGS-R cycle (gmres_mgsr.f90) */
/* w = M^-1 (b - A x); beta = ||w||; V(:,1) = w / beta   (:314-329).
 * Returns beta (= g(1)). */
int gk_mgs_cycle_start(gk_ctx *ctx, double *beta);
/* Arnoldi step j (1 <= j <= m): z = A V(:,j); w = M^-1 z; two MGS passes
 * over V(:,1:j) accumulating H(1:j,j); h = ||w||; V(:,j+1) = w / h
 * (:336-363, :384).  hcol[0..j] = H(1:j+1, j) before any Givens rotation. */
int gk_mgs_step(gk_ctx *ctx, int j, double *hcol);
/* The same step split in two so the host can run the Givens rotation of
 * step j while the GPU already works on step j+1: gk_mgs_step_async enqueues
 * step j and returns; gk_mgs_step_wait(j) blocks until its Hessenberg column
 * is available.  Enqueueing step j+1 before step j's convergence test is
 * harmless: a step only writes w and V(:,j+1) and its own column slot. */
int gk_mgs_step_async(gk_ctx *ctx, int j);
int gk_mgs_step_wait(gk_ctx *ctx, int j, double *hcol);
/* x += V(:,1:n_out) y  (:400-406). */
int gk_update_x(gk_ctx *ctx, const double *y, int n_out);
/* Orthogonality diagnostic v_err(1:n_out+1) (:414-420) from the Gram matrix
 * of V(:,1:n_out+1) computed on device.  zero_last != 0 treats V(:,n_out+1)
 * as the zero column gmres_mgsr_mf leaves after an in-cycle exit (:172-176). */
int gk_mgs_verr(gk_ctx *ctx, int n_out, int zero_last, double *v_err);

/* -------------------------------------- Householder cycle (gmres_hh.f90) */
/* Cycle start.  precondition = 0: w = b - A x (gmres_hh_omp :243-253);
 * 1: w = M^-1 (b - A x) (gmres_hh_prec_omp :425-436).  Builds reflector
 * P(:,1); returns g1 = g(1) = -sign(beta, w(1)). */
int gk_hh_cycle_start(gk_ctx *ctx, int precondition, double *g1);
/* Step j: v = P_1..P_j e_j; w = A v (M^-1 if precondition); w = P_j..P_1 w;
 * hcol[0..j] = H(1:j+1,j) (H(j+1,j) = -sign(||w(j+1:n)||, w(j+1)));
 * builds P(:,j+1)  (:255-321 / :438-502). */
int gk_hh_step(gk_ctx *ctx, int j, int precondition, double *hcol);
/* Split form of gk_hh_step (see gk_mgs_step_async). */
int gk_hh_step_async(gk_ctx *ctx, int j, int precondition);
int gk_hh_step_wait(gk_ctx *ctx, int j, double *hcol);
/* x += P_1..P_n_out [y;0]  (:350-378). */
int gk_hh_update_x(gk_ctx *ctx, const double *y, int n_out);
/* calculate_verr (:568-593): v_err(i) = sum_{j<i} 2 (V_i.V_j)^2, V rebuilt
 * from the reflectors on device (extra n x n_out buffer). */
int gk_hh_verr(gk_ctx *ctx, int n_out, double *v_err);

/* ------------------------------------------------ spectrum estimate ---- */
/* k Lanczos steps on A from a deterministic pseudo-random start vector (the
 * same for any slab decomposition); returns the extreme Ritz values of the
 * k x k tridiagonal (Sturm bisection on the host).  The README-promised
 * eigenvalue estimate for the Chebyshev parameters (README.md:11; the
 * reference hard-codes params, chebyshev.f90:20).  Clobbers work vectors. */
int gk_lanczos_bounds(gk_ctx *ctx, int k, double *lmin, double *lmax);

/* ------------------------------------------- device vector primitives ---- */
/* For the short-recurrence solvers that share the operator / preconditioner
 * seam (pcg_omp src/cg.f90:154-234, pbicgstab_omp src/bicgstab.f90:91-182):
 * context-resident vectors by id: GK_VEC_X = x, GK_VEC_B = b, 2 .. m+2 =
 * scratch (the Krylov columns).  Scalars come back to the host, as the
 * reference computes them in `single` blocks. */
#define GK_VEC_X 0
#define GK_VEC_B 1
#define GK_LC_COPY 0   /* out = a                  */
#define GK_LC_AXPY 1   /* out = a + s1*b           */
#define GK_LC_AXPY2 2  /* out = (a + s1*b) + s2*c  */
#define GK_LC_XPAYMZ 3 /* out = a + s1*(b - s2*c)  */
#define GK_LC_ZERO 4   /* out = 0                  */
int gk_vec_count(gk_ctx *ctx, int *count);
/* what = 0: out = A in; what = 1: out = M^-1 in (in != out). */
int gk_vec_apply(gk_ctx *ctx, int what, int in, int out);
/* result = <a, b> over all ranks (synchronous). */
int gk_vec_dot(gk_ctx *ctx, int a, int b, double *result);
int gk_vec_lincomb(gk_ctx *ctx, int form, int out, int a, int b, int c, double s1, double s2);

/* ------------------------------------- fused short-recurrence solvers ---- */
/* pcg_omp (src/cg.f90:154-234) and pbicgstab_omp (src/bicgstab.f90:91-182)
 * with every scalar on the device: one iteration is 2 (PCG) or 3 (BiCGSTAB)
 * fused passes (gmres_amd/csrc/gk_sr.hpp; with cbpr2 on one rank the
 * preconditioner runs inside two-level marches; N ranks or
 * GK_TUNE_SR_TWO_LEVEL 0: 3 / 5 passes), no host round trip per dot.  They replace the call sequence the reference's solvers make
 * through the operator / preconditioner seam (interfaces.f90:13-27): the
 * Fortran drivers pcg_drive / bicgstab_drive queue iterations in chunks and
 * read one status per chunk.  Vectors: the context's Krylov columns 0..7
 * and its w / vj work vectors (needs m >= 7); x stays in HBM (gk_get_x).
 *
 * gk_sr_start: x = 0, r = b; PCG: z = M^-1 r, p = z (cg.f90:174-187);
 *   BiCGSTAB: r0 = p = r (bicgstab.f90:112-118).  max_iter bounds the total
 *   number of iterations gk_sr_iterate may queue (the history's length).
 * gk_sr_iterate: queue k more iterations, no host wait.  Iterations after the
 *   first with res < tol return at entry on the device (`if (converged) cycle`).
 * gk_sr_status: wait = 0: for the oldest queued chunk; 1: for everything
 *   queued.  *executed = iterations run, *done = the first iteration with
 *   res < tol (0: none), *res = residual of the last executed iteration.
 * gk_sr_history: hist[0..n) = res after iterations 1..n (n <= *executed).
 * gk_set_precond / gk_set_rhs(_ones) / gk_set_x / gk_mgs_cycle_start /
 * gk_hh_cycle_start end a running solve (they change its data or reuse its
 * vectors): gk_sr_iterate / status / history then return GK_ERR_STATE until
 * the next gk_sr_start. */
#define GK_SR_PCG 0
#define GK_SR_BICGSTAB 1
int gk_sr_start(gk_ctx *ctx, int solver, double tol, int max_iter);
int gk_sr_iterate(gk_ctx *ctx, int k);
int gk_sr_status(gk_ctx *ctx, int wait, int *executed, int *done, double *res);
int gk_sr_history(gk_ctx *ctx, double *hist, int n);

/* ---------------------------------------------------------- profiling ---- */
/* enable = 1: every launch is bracketed by HIP events on the context stream;
 * enable = S > 1: only the launches of MGS-R steps with j % S == 0 (launch
 * durations do not depend on j, so the per-launch average is unbiased while
 * the event overhead drops S-fold).  gk_profile_read returns the summed
 * device time (ms) and launch count per kernel id since the last reset. */
int gk_profile_enable(gk_ctx *ctx, int enable);
int gk_profile_reset(gk_ctx *ctx);
int gk_profile_read(gk_ctx *ctx, int kid, double *total_ms, long long *launches);
/* Time split of the resident launches, measured inside them (wall clock of
 * thread 0 of every workgroup): mode 1 enables and zeroes, 2 zeroes, 0
 * disables, -1 only reads.  For the launches of kind `which` (0 MGS-R step,
 * 1 Householder UP chain, 2 Householder DOWN chain) since the last reset:
 * the mean over workgroups of the time streaming passes, the time waiting in
 * the in-launch all-gathers, and the launch total, summed over launches (out
 * pointers may be NULL to skip reading). */
int gk_profile_res_split(gk_ctx *ctx, int mode, int which, double *pass_ms, double *wait_ms, double *total_ms,
                         long long *launches);
/* The same split per workgroup (blockIdx order, summed over launches): the
 * arrival skew of the in-launch all-gathers shows as the spread of pass_ms. */
int gk_profile_res_wg(gk_ctx *ctx, int which, double *pass_ms, double *wait_ms, int maxwg, int *nwg);
/* All-gather trace of one resident launch: for every workgroup and in-launch exchange, the
 * wall-clock ticks at which its partial was published and at which it held the grid total
 * (tools/res_trace.py: arrival skew vs propagation).  arm 1: trace the MGS-R step launches
 * of Arnoldi step j from now on (mode must be 0; each overwrites the last); 0: off; -1: read
 * the last traced launch into out[nwg][nx][2]. */
int gk_profile_res_trace(gk_ctx *ctx, int arm, int j, int mode, unsigned long long *out, int maxwg, int maxx,
                         int *nwg, int *nx, double *tick_per_ms);
int gk_sync(gk_ctx *ctx);

/* ------------------------------------------- resident-step variant plan ---- */
/* Which resident kernel an Arnoldi step (and a Householder chain) runs on.
 * Selection is by the slab's local length and the workgroups available
 * (compute units / contexts sharing the device), so a 2- / 4- / 8-GPU split
 * of one grid selects a different variant than the single-GPU run does:
 *   GK_RES_NONE       no resident launch (one launch per projection);
 *   GK_RES_PREFETCH   k_mgs_res<R2 in 2,4,8, PF, control wave>: small slabs;
 *   GK_RES_PAIRS      k_mgs_res<12, 0>: w and the running column in registers;
 *   GK_RES_PAIRS_LDS  k_mgs_res<12, 18>: the same plus w of 18 chunks per
 *                     workgroup in LDS, the rest streamed;
 *   GK_RES_WONLY      k_mgs_wres: w only, in registers + LDS (large slabs);
 *   GK_RES_WCOL       k_mgs_wpc: w in registers and the running Krylov column cached
 *                     (registers + LDS) -- 8 B per unknown per projection for slabs of
 *                     up to 64 x 256 double2 per workgroup (one GPU of 4096^2 / 2 and
 *                     of 8192^2 / 8), in 512-thread workgroups (two waves per SIMD); slabs
 *                     of <= 16 chunks per thread (4096^2 / 4) keep the whole column in
 *                     registers (r2 = 16, l2 = 0);
 *   GK_RES_BLOCKED    k_mgs_blk (gmres_amd/csrc/gk_blk.hpp): the blocked-projection MGS-R
 *                     step of GK_TUNE_RES_BLOCK > 1 -- one all-gather per block of S
 *                     projections; r2 / l2 = cached column chunks per block slot in
 *                     registers / LDS, blk = S.
 * info[GK_RES_INFO_LEN]: variant, workgroups G, R2, L2, prefetch, control
 * wave, w-only, non-temporal column loads, register / LDS chunks per
 * workgroup in use, dynamic LDS bytes, resident double2 of the slab, and
 * (unused, 0),
 * (gk_res_info only) whether the Arnoldi step's Chebyshev(k) pass forms z = A v in its own
 * stage 0 (1 / 0; -1 on a multi-rank context whose smallest slab is not known
 * until its first solve), the threads per workgroup (= double2 per chunk), and the
 * projection block S (1: strict MGS-R).
 * gk_res_plan_query: pure host computation for a slab of nloc unknowns on a
 * device with `cus` compute units shared by `share` contexts; hh != 0 the
 * reflection chains' plan; nt: -1 auto (from nloc), 0 / 1 forced; block: the
 * GK_TUNE_RES_BLOCK value (1, 2 or 4) of the MGS step's plan.  No device
 * is touched (the CPU tests pin every production split with it).
 * gk_res_info: the plan this context uses now (its tuning, communicator and
 * sharing applied); variant GK_RES_NONE when steps run launch by launch. */
#define GK_RES_NONE 0
#define GK_RES_PREFETCH 1
#define GK_RES_PAIRS 2
#define GK_RES_PAIRS_LDS 3
#define GK_RES_WONLY 4
#define GK_RES_WCOL 5
#define GK_RES_BLOCKED 6
#define GK_RES_INFO_LEN 16
int gk_res_plan_query(long long nloc, int cus, int share, int hh, int nt, int block, long long *info);
int gk_res_info(gk_ctx *ctx, int hh, long long *info);

/* Launch-policy knobs (defaults are the tuned values; for A/B measurement).
 *   GK_TUNE_PROJ_NT        1: non-temporal loads of the Krylov columns in the
 *                          projection kernel (keeps w resident in the 256 MB
 *                          Infinity Cache); 0: plain loads; -1: auto (default:
 *                          non-temporal when a vector exceeds 48 MiB)
 *   GK_TUNE_PROJ_BLOCKS    workgroups of the projection kernel (0 = auto)
 *   GK_TUNE_STENCIL_BLOCKS target workgroups of the stencil sweeps (0 = auto)
 *   (keys 3, 17 and 26 -- the reversed projection walk, the w-only step's stencil
 *   prologue and the look-ahead blocked step -- were measured slower and removed in
 *   round 5; DESIGN.md 3.1 / 3.1c / 3.4 keep the numbers; they are unknown keys now)
 *   GK_TUNE_PROJ_BLOCKED   1: contiguous range per workgroup; 0: grid-stride
 *   GK_TUNE_PROJ_UNROLL    double2 loads in flight per thread and array: 2, 4, 8; 0 = auto
 *   GK_TUNE_CHEB_FUSED     1 (default): Chebyshev(k <= 8) as temporal-blocked passes of up to
 *                          4 sweeps each (single slab, even N); 0: one launch per sweep
 *   GK_TUNE_XCHG_TIMEOUT_MS deadline of one device-exchange wait (default 20000)
 *   GK_TUNE_RES            resident MGS-R step (one persistent launch per Arnoldi step, w and the
 *                          running Krylov column held in registers, dots all-gathered inside the
 *                          launch): -1 auto (default: on for a single rank or the device exchange,
 *                          m <= 512, one context per device), 1 also with several contexts on one
 *                          device (their streams must then run concurrently), 0 off (one launch
 *                          per projection)
 *   GK_TUNE_RES_R2         cap of register-resident double2 per thread and array: 0 auto, 2/4/8/12
 *   GK_TUNE_RES_SHARE      contexts sharing this device (resident launches use CUs / share
 *                          workgroups; gk_comm_init_local sets it to the group size)
 *   GK_TUNE_RES_TIMEOUT_MS deadline of one in-launch wait (default 20000); a miss fails the step
 *                          with GK_ERR_COMM and switches the context to the launch path
 *   GK_TUNE_RES_LDS        1 (default): when the slab exceeds the register-resident part, keep w
 *                          of 144 KiB more per workgroup in LDS (16 B/unknown per projection
 *                          instead of 32); 0: stream it
 *   GK_TUNE_RES_WONLY      large slabs: -1 (default) pick by the modelled bytes per projection,
 *                          1 always, 0 never the w-only variant (one wave per SIMD, ~490 registers
 *                          per lane: w in registers + LDS, both columns streamed)
 *   GK_TUNE_VERR_ORDER     1 (default): the v_err diagnostics (gk_mgs_verr, gk_hh_verr) use the
 *                          reference's dot_product order, one running sum per dot (bit-identical
 *                          to the reference's formula on the same basis; single rank); 0: tree
 *                          reduction (fast; N ranks always use it)
 *   GK_TUNE_HH_FUSE        1 (default): with the w-only resident variant a Householder step folds
 *                          its small launches into the reflection chains -- the DOWN chain builds
 *                          e_j itself, the UP chain ends with the reflector fix-up and
 *                          P(:,j+1) = w/||w|| (gmres_hh.f90:306-318); 0: separate k_set_unit,
 *                          k_hh_fix and k_scale launches
 *   GK_TUNE_CHEB_STEN      1 (default): the Arnoldi step's Chebyshev(k <= 8) pass forms z = A v
 *                          itself in a stage ahead of its levels (no stencil launch, no z vector;
 *                          N >= 128, slabs of at least k + 1 lines); 0: stencil launch + pass
 *   GK_TUNE_GRAPH          1 (default): a launch-path MGS-R step (RCCL ranks, device-exchange ranks
 *                          with the resident step off, or one rank with it off) is captured once
 *                          per step index j as a hipGraph -- its 2j projection launches, 2j + 1
 *                          all-reduces (ncclAllReduce / k_xchg captured as graph nodes; a replayed
 *                          k_xchg takes its sequence number from a device base set before each
 *                          replay) and the normalisation -- and replayed in later cycles;
 *                          0: launched call by call.  A capture that fails switches it off for
 *                          the context (gk_last_error keeps the reason).
 *   GK_TUNE_RES_QDEF       k_mgs_res with non-temporal columns (pairs / pairs+lds): 1 = the LDS-held
 *                          and streamed parts read each pass's dot column V_q with the default
 *                          policy, so the next pass's AXPY column (the same V_q) is an
 *                          Infinity-Cache hit (the w-only kernel's policy); 0 = both
 *                          non-temporal; -1 (default) = the measured choice
 *   GK_TUNE_RES_FOLD       1 (default): N ranks on the device exchange -- the MGS step's first dot
 *                          <w, V(:,1)> (Householder: <w, P_1>) is summed across ranks inside the
 *                          resident launch (its rank-total hop) instead of by a k_xchg launch
 *                          before it; 0: the launch
 *   GK_TUNE_RES_PC         column-cache variant (GK_RES_WCOL): -1 (default) where its modelled
 *                          bytes per projection are fewer than both the pairs and the w-only
 *                          variants' (two-wave build; a one-wave build, GK_RES_PC_NT=256,
 *                          needs at most 2/3 of them); 0 never; 1 wherever the slab fits
 *   GK_TUNE_RES_BLOCK      1 (default): the strict MGS-R step (gmres_mgsr.f90:341-360), one
 *                          in-launch all-gather per projection; 2 or 4 (opt-in): the blocked
 *                          step k_mgs_blk -- the projections of each sweep in blocks of S
 *                          columns, ONE all-gather per block carrying its S dots and the Gram
 *                          terms of its newest column, the h formed by MGS's exact-arithmetic
 *                          recurrence h_k = <w,V_k> - sum_{l<k} h_l <V_l,V_k> (the two sweeps
 *                          stay separate, so the reorthogonalisation still sees w after the
 *                          whole first sweep): 2 (1 + ceil((j-1)/S)) all-gathers per step
 *                          instead of 2j.  Not bit-identical to the strict step (within the
 *                          residual-history tolerance of DESIGN.md 4.3).  MGS-R resident
 *                          steps only; Householder and the launch path stay strict.
 *   GK_TUNE_RES_PF         the STRICT MGS-R step on the blocked kernel with blocks of 1
 *                          (k_mgs_blk<S = 1>: the reference's projection order, one all-gather
 *                          per projection) whose next dot column is prefetched into LDS during
 *                          each all-gather; gk_res_info reports variant blocked, blk 1.  0
 *                          (default): the strict kernels; 1: for every slab up to 32 chunks of
 *                          512 double2 per workgroup (faster on one GPU at 16 chunks only;
 *                          DESIGN.md 3.1c)
 *   GK_TUNE_WATCHDOG_MS    limit of every host wait on the context's stream (gk_sync, the step
 *                          waits, gk_update_x ...); 0 (default) = twice the longest device
 *                          deadline plus a minute.  Past it the wait returns GK_ERR_COMM (a
 *                          kernel of the context was never scheduled) and the context is
 *                          BROKEN: every later call returns GK_ERR_STATE; gk_destroy frees it
 *                          once its stream drains (bounded by the same limit; else it is kept)
 *   GK_TUNE_HH_NORM_ORDER  0 (default): the Householder reflector norms (gmres_hh.f90:251-253,
 *                          307, 315) tree-reduced in the resident chains; 1 (one rank): taken
 *                          in the reference's own order -- flang-rt's NORM2, a running max and
 *                          scaled sum over the vector (k_norm2_seq) -- so the device basis
 *                          carries the reference's normalisation rounding (the v_err band of
 *                          DESIGN.md 4.3 becomes two-sided); the step runs unfused.  A
 *                          diagnostic mode: one sequential pass per norm (~0.1 ms per 16 K)
 *   GK_TUNE_SR_BLOCKS      target workgroups of the short-recurrence line marches (gk_sr_*; 0 =
 *                          auto, 512: each marches JT = lines x windows / 512 grid lines, up to
 *                          256 -- long marches re-read fewer neighbour lines)
 *   GK_TUNE_SR_TWO_LEVEL   1 (default): with the cbpr2 preconditioner on one rank the
 *                          short-recurrence solvers run the preconditioner and the operator
 *                          next to it in one two-level march (PCG 2 passes per iteration,
 *                          BiCGSTAB 3); 0: one pass each (3 / 5).  Bit-identical results;
 *                          read by gk_sr_start
 *   GK_TUNE_SPIN_WAIT      1 (default): gk_mgs_step_wait / gk_hh_step_wait spin on the step's
 *                          event; 0: hipEventSynchronize (may sleep in the driver per step) */
#define GK_TUNE_PROJ_NT 0
#define GK_TUNE_PROJ_BLOCKS 1
#define GK_TUNE_STENCIL_BLOCKS 2
#define GK_TUNE_PROJ_BLOCKED 4
#define GK_TUNE_PROJ_UNROLL 5
#define GK_TUNE_CHEB_FUSED 6
#define GK_TUNE_XCHG_TIMEOUT_MS 7
#define GK_TUNE_RES 8
#define GK_TUNE_RES_R2 9
#define GK_TUNE_RES_SHARE 10
#define GK_TUNE_RES_TIMEOUT_MS 11
#define GK_TUNE_RES_LDS 12
#define GK_TUNE_RES_WONLY 13
#define GK_TUNE_VERR_ORDER 14
#define GK_TUNE_HH_FUSE 15
#define GK_TUNE_CHEB_STEN 16
#define GK_TUNE_SPIN_WAIT 18
#define GK_TUNE_GRAPH 19
#define GK_TUNE_RES_QDEF 20
#define GK_TUNE_RES_PC 21
#define GK_TUNE_RES_FOLD 22
#define GK_TUNE_RES_BLOCK 23
#define GK_TUNE_WATCHDOG_MS 24
#define GK_TUNE_HH_NORM_ORDER 25
#define GK_TUNE_RES_PF 27
#define GK_TUNE_SR_BLOCKS 28
#define GK_TUNE_SR_TWO_LEVEL 29
int gk_set_tuning(gk_ctx *ctx, int key, int value);
/* Test hook: hold = 1 enqueues on the context's stream a wait for a mapped host
 * word that only hold = 0 writes (hipStreamWaitValue32) -- every later kernel of
 * the context then stays unscheduled until the release, as with a hardware queue
 * that is never mapped; it exercises the host watchdog (GK_TUNE_WATCHDOG_MS). */
int gk_debug_hold_stream(gk_ctx *ctx, int hold);

/* ------------------------- stateless kernel API (caller device memory) ---- */
/* y = A x on lines [0,nlines) of an N-wide slab; halo_lo / halo_hi are the
 * grid lines just below / above the slab (NULL at the physical boundary)
 * -- stencil_vector, src/problems/poisson.f90:33-77.  stream: hipStream_t. */
int gk_poisson5(int nside, int nlines, const double *x, const double *halo_lo,
                const double *halo_hi, double *y, void *stream);
/* z = M^-1 r for the single-slab case (precond, src/interfaces.f90:20-27);
 * scratch: 3 vectors of N*N doubles. */
int gk_precond_apply(int nside, int kind, const double *params, int degree, const double *r,
                     double *z, double *scratch, void *stream);
/* Fused MGS projection (gmres_mgsr.f90:343-358): h = <w,va>;
 * w -= h*va; result[0] = h (device). */
int gk_mgs_project(long long n, double *w, const double *va, double *result, void *stream);
/* result[0] = <a,b> (device). */
int gk_dot(long long n, const double *a, const double *b, double *result, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GMRES_HIP_H */
