!! gmres_hip.f90 -- Fortran host side of the MI355X GMRES(m) inner cycle.
!!
!! The reference (AlexanderGSC/gmres) keeps its solvers in Fortran and plugs
!! the operator / preconditioner in through procedure arguments
!! (src/interfaces.f90:13-27).  This file keeps that host language and that
!! plug-in shape: the restart loop, the Hessenberg Givens rotations, the
!! back-solve and the convergence tests run here, on the host, exactly as in
!! src/gmres_mgsr.f90 / src/gmres_hh.f90; every O(n) vector operation runs on
!! the GPU through the C-ABI of libgmres_hip.so (include/gmres_hip.h), bound
!! below with ISO_C_BINDING.  Only the (j+1)-long Hessenberg column of each
!! Arnoldi step crosses PCIe.
!!
!! Modules
!!   gmres_hip_c           ISO_C_BINDING interfaces to include/gmres_hip.h
!!   gmres_hip_interfaces  the reference's two abstract plug-in interfaces
!!   gmres_hip             device-backed plug-ins (hip_poisson5, hip_identity,
!!                         hip_cbpr2, hip_chebyshev), drop-in solvers
!!                         gmres_mgsr_hip / gmres_hh_hip / gmres_hh_prec_hip,
!!                         and bind(C) drivers for harnesses that already hold
!!                         a device context (gmres_mgsr_hip_run, gmres_hh_hip_run).

module gmres_hip_c
    use, intrinsic :: iso_c_binding
    implicit none
    integer(c_int), parameter :: GK_OK = 0
    integer(c_int), parameter :: GK_PREC_IDENTITY = 0, GK_PREC_CBPR2 = 1, GK_PREC_CHEB = 2
    integer(c_int), parameter :: GK_VEC_X = 0, GK_VEC_B = 1
    integer(c_int), parameter :: GK_SR_PCG = 0, GK_SR_BICGSTAB = 1
    integer(c_int), parameter :: GK_LC_COPY = 0, GK_LC_AXPY = 1, GK_LC_AXPY2 = 2, GK_LC_XPAYMZ = 3, GK_LC_ZERO = 4
    interface
        function gk_last_error() result(p) bind(C, name='gk_last_error')
            import :: c_ptr
            type(c_ptr) :: p
        end function
        integer(c_int) function gk_create(device, nside, line0, nlines, m, ctx) bind(C, name='gk_create')
            import :: c_int, c_ptr
            integer(c_int), value :: device, nside, line0, nlines, m
            type(c_ptr), intent(out) :: ctx
        end function
        integer(c_int) function gk_destroy(ctx) bind(C, name='gk_destroy')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function gk_local_size(ctx, nloc) bind(C, name='gk_local_size')
            import :: c_int, c_ptr, c_long_long
            type(c_ptr), value :: ctx
            integer(c_long_long), intent(out) :: nloc
        end function
        integer(c_int) function gk_set_precond(ctx, kind, params, nparams, degree) bind(C, name='gk_set_precond')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: kind, nparams, degree
            real(c_double), intent(in) :: params(*)
        end function
        integer(c_int) function gk_set_rhs(ctx, b) bind(C, name='gk_set_rhs')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(in) :: b(*)
        end function
        integer(c_int) function gk_rhs_norm(ctx, beta0) bind(C, name='gk_rhs_norm')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(out) :: beta0
        end function
        integer(c_int) function gk_zero_x(ctx) bind(C, name='gk_zero_x')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function gk_get_x(ctx, x) bind(C, name='gk_get_x')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(out) :: x(*)
        end function
        integer(c_int) function gk_apply(ctx, what, xin, xout) bind(C, name='gk_apply')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: what
            real(c_double), intent(in) :: xin(*)
            real(c_double), intent(out) :: xout(*)
        end function
        integer(c_int) function gk_true_residual(ctx, rel) bind(C, name='gk_true_residual')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(out) :: rel
        end function
        integer(c_int) function gk_mgs_cycle_start(ctx, beta) bind(C, name='gk_mgs_cycle_start')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(out) :: beta
        end function
        integer(c_int) function gk_mgs_step(ctx, j, hcol) bind(C, name='gk_mgs_step')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: j
            real(c_double), intent(out) :: hcol(*)
        end function
        integer(c_int) function gk_mgs_step_async(ctx, j) bind(C, name='gk_mgs_step_async')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: j
        end function
        integer(c_int) function gk_mgs_step_wait(ctx, j, hcol) bind(C, name='gk_mgs_step_wait')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: j
            real(c_double), intent(out) :: hcol(*)
        end function
        integer(c_int) function gk_update_x(ctx, y, n_out) bind(C, name='gk_update_x')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(in) :: y(*)
            integer(c_int), value :: n_out
        end function
        integer(c_int) function gk_mgs_verr(ctx, n_out, zero_last, v_err) bind(C, name='gk_mgs_verr')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: n_out, zero_last
            real(c_double), intent(out) :: v_err(*)
        end function
        integer(c_int) function gk_hh_cycle_start(ctx, precondition, g1) bind(C, name='gk_hh_cycle_start')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: precondition
            real(c_double), intent(out) :: g1
        end function
        integer(c_int) function gk_hh_step(ctx, j, precondition, hcol) bind(C, name='gk_hh_step')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: j, precondition
            real(c_double), intent(out) :: hcol(*)
        end function
        integer(c_int) function gk_hh_step_async(ctx, j, precondition) bind(C, name='gk_hh_step_async')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: j, precondition
        end function
        integer(c_int) function gk_hh_step_wait(ctx, j, hcol) bind(C, name='gk_hh_step_wait')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: j
            real(c_double), intent(out) :: hcol(*)
        end function
        integer(c_int) function gk_hh_update_x(ctx, y, n_out) bind(C, name='gk_hh_update_x')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(in) :: y(*)
            integer(c_int), value :: n_out
        end function
        integer(c_int) function gk_hh_verr(ctx, n_out, v_err) bind(C, name='gk_hh_verr')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: n_out
            real(c_double), intent(out) :: v_err(*)
        end function
        integer(c_int) function gk_vec_apply(ctx, what, vin, vout) bind(C, name='gk_vec_apply')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: what, vin, vout
        end function
        integer(c_int) function gk_vec_dot(ctx, a, b, res) bind(C, name='gk_vec_dot')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: a, b
            real(c_double), intent(out) :: res
        end function
        integer(c_int) function gk_vec_lincomb(ctx, form, vout, a, b, c, s1, s2) bind(C, name='gk_vec_lincomb')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: form, vout, a, b, c
            real(c_double), value :: s1, s2
        end function
        integer(c_int) function gk_sr_start(ctx, solver, tol, max_iter) bind(C, name='gk_sr_start')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: solver, max_iter
            real(c_double), value :: tol
        end function
        integer(c_int) function gk_sr_iterate(ctx, k) bind(C, name='gk_sr_iterate')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: k
        end function
        integer(c_int) function gk_sr_status(ctx, wait, executed, done, res) bind(C, name='gk_sr_status')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            integer(c_int), value :: wait
            integer(c_int), intent(out) :: executed, done
            real(c_double), intent(out) :: res
        end function
        integer(c_int) function gk_sr_history(ctx, hist, n) bind(C, name='gk_sr_history')
            import :: c_int, c_ptr, c_double
            type(c_ptr), value :: ctx
            real(c_double), intent(out) :: hist(*)
            integer(c_int), value :: n
        end function
        integer(c_size_t) function c_strlen(p) bind(C, name='strlen')
            import :: c_ptr, c_size_t
            type(c_ptr), value :: p
        end function
    end interface
contains
    !> Message of the calling thread's last libgmres_hip error.
    function gk_error_message() result(s)
        character(len=:), allocatable :: s
        type(c_ptr) :: p
        character(kind=c_char), pointer :: a(:)
        integer :: k, n
        p = gk_last_error()
        n = int(c_strlen(p))
        call c_f_pointer(p, a, [n])
        allocate (character(len=n) :: s)
        do k = 1, n
            s(k:k) = a(k)
        end do
    end function

    !> error stop with the library's message when status /= GK_OK.
    subroutine gk_require(status, what)
        integer(c_int), intent(in) :: status
        character(len=*), intent(in) :: what
        if (status /= GK_OK) then
            write (*, '(A,A,A,I0,A,A)') 'gmres_hip: ', what, ' failed (status ', status, '): ', gk_error_message()
            error stop 2
        end if
    end subroutine
end module gmres_hip_c

!> The reference's plug-in interfaces (src/interfaces.f90:13-27), restated so a
!> driver written against them compiles unchanged against gmres_hip.
module gmres_hip_interfaces
    implicit none
    abstract interface
        subroutine stencil_vector(x, y, n)
            real(8), intent(in) :: x(:)
            real(8), intent(out) :: y(:)
            integer, intent(in) :: n     ! grid side N (not the vector length)
        end subroutine stencil_vector
    end interface
    abstract interface
        subroutine precond(A_x, r, z, aux, params, n)
            import :: stencil_vector
            procedure(stencil_vector) :: A_x
            real(8), intent(in) :: r(:)
            real(8), intent(out) :: z(:)
            real(8), intent(out) :: aux(:)
            real(8), intent(in) :: params(:)
            integer, intent(in) :: n
        end subroutine precond
    end interface
end module gmres_hip_interfaces

!> Table output in the reference's column layout (src/utils/utils.f90:37-51:
!> print_header / print_line), so sweep tables diff 1:1 against the
!> reference drivers' output (tests/strong_scaling.f90, tests/weak_scaling.f90).
module gmres_hip_report
    implicit none
    private
    public :: report_header, report_line
contains
    subroutine report_header(title)
        character(len=*), intent(in) :: title
        print *, title
        write (*, '(A3, A10, A10, A10, A10, A14, A14, A14, A14, A14, A10, A15)') "#", "Vars", "Iters", &
            "Restarts", "gmres(n)", "Tol.", "L2 Norm", "L_inf Norm", "Residual", "||I-V.t*V||", "Time", "Info"
        write (*, '(150("-"))')
    end subroutine report_header

    subroutine report_line(test, nvars, seconds, iterations, restarts, m, tol, resid, verr, l2, linf, info)
        integer, intent(in) :: test, nvars, iterations, restarts, m
        real(8), intent(in) :: seconds, resid, verr, l2, linf, tol
        character(len=*), intent(in) :: info
        character(len=30) :: desc
        desc = info
        write (*, '(I3, I10, I10, I10, I10, ES14.2, ES14.4, ES14.4, ES14.4, ES14.4, F10.4, A20)') test, nvars, &
            iterations, restarts, m, tol, l2, linf, resid, verr, seconds, desc
    end subroutine report_line
end module gmres_hip_report

module gmres_hip
    use, intrinsic :: iso_c_binding
    use gmres_hip_c
    use gmres_hip_interfaces
    implicit none
    private
    !> restart cap, as gmres_mgsr.f90:6 max_restarts / gmres_hh.f90:8 stages
    integer, public :: hip_max_restarts = 1000
    !> HIP device used by the drop-in solvers and the host-array plug-ins
    integer, public :: hip_device = 0
    !> Chebyshev(k) degree used by hip_chebyshev when params(3) is absent
    integer, public :: hip_cheb_degree = 8
    integer, parameter, public :: MGSR_OMP = 1, MGSR_MF = 0

    public :: stencil_vector, precond
    public :: hip_poisson5, hip_identity, hip_cbpr2, hip_chebyshev
    public :: gmres_mgsr_hip, gmres_hh_hip, gmres_hh_prec_hip, hip_release
    public :: pcg_hip, pbicgstab_hip, pcg_drive, bicgstab_drive, pcg_drive_seq, bicgstab_drive_seq
    !> iterations queued per chunk by the fused short-recurrence drivers
    integer, public :: hip_sr_chunk = 32
    public :: mgsr_drive, hh_drive, givens_column, back_solve

    type(c_ptr) :: opctx = c_null_ptr   ! context of the host-array plug-ins
    integer :: opctx_n = -1
contains

    ! ------------------------------------------------------------- helpers --

    !> Apply the previous rotations to column j of H, build rotation j, rotate g
    !> (gmres_mgsr.f90:364-383; identical in gmres_hh.f90:322-337).
    subroutine givens_column(H, cs, sn, g, j)
        real(8), intent(inout) :: H(:, :), cs(:), sn(:), g(:)
        integer, intent(in) :: j
        real(8) :: tmp, ds
        integer :: i
        do i = 1, j - 1
            tmp = H(i, j)
            H(i, j) = cs(i)*tmp + sn(i)*H(i + 1, j)
            H(i + 1, j) = -sn(i)*tmp + cs(i)*H(i + 1, j)
        end do
        ds = hypot(H(j + 1, j), H(j, j))
        cs(j) = H(j, j)/ds
        sn(j) = H(j + 1, j)/ds
        H(j, j) = cs(j)*H(j, j) + sn(j)*H(j + 1, j)
        H(j + 1, j) = 0.0d0
        tmp = g(j)
        g(j) = cs(j)*tmp + sn(j)*g(j + 1)
        g(j + 1) = -sn(j)*tmp + cs(j)*g(j + 1)
    end subroutine givens_column

    !> y from the upper-triangular H y = g (gmres_mgsr.f90:394-398).
    subroutine back_solve(H, g, y, n_out)
        real(8), intent(in) :: H(:, :), g(:)
        real(8), intent(out) :: y(:)
        integer, intent(in) :: n_out
        integer :: i
        y = 0.0d0
        y(n_out) = g(n_out)/H(n_out, n_out)
        do i = n_out - 1, 1, -1
            y(i) = (g(i) - dot_product(H(i, i + 1:n_out), y(i + 1:n_out)))/H(i, i)
        end do
    end subroutine back_solve

    integer function grid_side(nvec) result(ns)
        integer, intent(in) :: nvec
        ns = nint(sqrt(dble(nvec)))
        if (ns*ns /= nvec) then
            write (*, '(A,I0)') 'gmres_hip: vector length is not a square grid: ', nvec
            error stop 2
        end if
    end function grid_side

    ! ------------------------------------------------------------ drivers --

    !> Restarted MGS-R GMRES(m) on a device context whose RHS and preconditioner
    !> are set.  variant = MGSR_OMP: gmres_mgsr_omp semantics
    !> (gmres_mgsr.f90:277-421: `converged` latch, V(:,j+1) always formed);
    !> MGSR_MF: gmres_mgsr_mf (:98-199: exit inside the j loop).
    !> hist_res(c) = true residual after cycle c, hist_ferr(j,c) = final_err(j)
    !> of cycle c (written only when want_hist).  Returns a GK status.
    integer function mgsr_drive(ctx, m, tol, beta0, variant, max_cyc, x, final_err, v_err, n_out, &
                                restart_out, want_verr, want_hist, hist_res, hist_ferr, n_cycles, keep_x) &
        result(st)
        type(c_ptr), intent(in) :: ctx
        integer, intent(in) :: m, variant, max_cyc
        real(8), intent(in) :: tol, beta0
        real(8), intent(out) :: x(*), final_err(m), v_err(m + 1)
        integer, intent(out) :: n_out, restart_out, n_cycles
        logical, intent(in) :: want_verr, want_hist
        real(8), intent(inout) :: hist_res(*), hist_ferr(m, *)
        logical, intent(in), optional :: keep_x  ! .true.: x stays in HBM (gk_get_x later)
        real(8), allocatable :: H(:, :), g(:), y(:), cs(:), sn(:), hcol(:)
        real(8) :: beta, h_val
        integer :: cyc, j, zero_last
        logical :: converged, exited
        allocate (H(m + 1, m), g(m + 1), y(m), cs(m), sn(m), hcol(m + 1))
        final_err = 0.0d0; v_err = 0.0d0; cs = 0.0d0; sn = 0.0d0
        n_out = 0; restart_out = 0; n_cycles = 0; h_val = 0.0d0
        converged = .false.; exited = .false.
        st = gk_zero_x(ctx); if (st /= GK_OK) return     ! x0 = 0 (gmres_mgsr.f90:304)
        do cyc = 1, max_cyc
            g = 0.0d0; H = 0.0d0
            st = gk_mgs_cycle_start(ctx, beta); if (st /= GK_OK) return
            g(1) = beta
            exited = .false.
            ! Pipelined: step j+1 is enqueued on the GPU before the host waits for
            ! step j's Hessenberg column, so the Givens work below overlaps it.
            if (.not. converged) then
                st = gk_mgs_step_async(ctx, 1); if (st /= GK_OK) return
            end if
            do j = 1, m
                if (converged) exit
                n_out = j
                if (j < m) then
                    st = gk_mgs_step_async(ctx, j + 1); if (st /= GK_OK) return
                end if
                st = gk_mgs_step_wait(ctx, j, hcol); if (st /= GK_OK) return
                H(1:j + 1, j) = hcol(1:j + 1)
                h_val = hcol(j + 1)
                call givens_column(H, cs, sn, g, j)
                final_err(j) = abs(g(j + 1))/beta0
                if (want_hist) hist_ferr(j, cyc) = final_err(j)
                if (variant == MGSR_MF) then
                    if (h_val < tol .or. final_err(j) < tol) then
                        n_out = j
                        exited = .true.
                        exit
                    end if
                else if (final_err(j) < tol) then
                    restart_out = cyc
                    converged = .true.
                end if
            end do
            call back_solve(H, g, y, n_out)
            st = gk_update_x(ctx, y, n_out); if (st /= GK_OK) return
            n_cycles = cyc
            if (want_hist) then
                st = gk_true_residual(ctx, hist_res(cyc)); if (st /= GK_OK) return
            end if
            if (h_val < tol .or. final_err(n_out) < tol) then
                restart_out = cyc
                exit
            end if
        end do
        if (restart_out == 0) restart_out = n_cycles
        if (want_verr) then
            zero_last = merge(1, 0, exited)
            st = gk_mgs_verr(ctx, n_out, zero_last, v_err); if (st /= GK_OK) return
        end if
        if (present(keep_x)) then
            if (keep_x) return
        end if
        st = gk_get_x(ctx, x)
    end function mgsr_drive

    !> Householder GMRES(m) on a device context.  midcycle_exit = .false.:
    !> gmres_hh_omp (gmres_hh.f90:211-385, always full cycles, no preconditioner
    !> at cycle start when precondition = 0); .true.: gmres_hh_prec_omp
    !> (:388-566, `converged` latch).
    integer function hh_drive(ctx, m, tol, beta0, precondition, midcycle_exit, max_cyc, x, final_err, &
                              v_err, n_out, stages_out, want_verr, want_hist, hist_res, hist_ferr, &
                              n_cycles, keep_x) result(st)
        type(c_ptr), intent(in) :: ctx
        integer, intent(in) :: m, max_cyc, precondition
        logical, intent(in) :: midcycle_exit
        real(8), intent(in) :: tol, beta0
        real(8), intent(out) :: x(*), final_err(m), v_err(m + 1)
        integer, intent(out) :: n_out, stages_out, n_cycles
        logical, intent(in) :: want_verr, want_hist
        real(8), intent(inout) :: hist_res(*), hist_ferr(m, *)
        logical, intent(in), optional :: keep_x  ! .true.: x stays in HBM (gk_get_x later)
        real(8), allocatable :: H(:, :), g(:), y(:), cs(:), sn(:), hcol(:)
        real(8) :: g1
        integer :: k, j
        logical :: converged
        allocate (H(m + 1, m), g(m + 1), y(m), cs(m), sn(m), hcol(m + 1))
        final_err = 0.0d0; v_err = 0.0d0; cs = 0.0d0; sn = 0.0d0
        n_out = 0; stages_out = 0; n_cycles = 0
        converged = .false.
        st = gk_zero_x(ctx); if (st /= GK_OK) return
        do k = 1, max_cyc
            g = 0.0d0; H = 0.0d0
            st = gk_hh_cycle_start(ctx, precondition, g1); if (st /= GK_OK) return
            g(1) = g1
            if (.not. converged) then
                st = gk_hh_step_async(ctx, 1, precondition); if (st /= GK_OK) return
            end if
            do j = 1, m
                if (converged) exit
                n_out = j
                if (j < m) then  ! pipelined as in mgsr_drive
                    st = gk_hh_step_async(ctx, j + 1, precondition); if (st /= GK_OK) return
                end if
                st = gk_hh_step_wait(ctx, j, hcol); if (st /= GK_OK) return
                H(1:j + 1, j) = hcol(1:j + 1)
                call givens_column(H, cs, sn, g, j)
                final_err(j) = abs(g(j + 1))/beta0
                if (want_hist) hist_ferr(j, k) = final_err(j)
                if (midcycle_exit .and. final_err(j) < tol) then
                    n_out = j
                    stages_out = k
                    converged = .true.
                end if
            end do
            call back_solve(H, g, y, n_out)
            st = gk_hh_update_x(ctx, y, n_out); if (st /= GK_OK) return
            n_cycles = k
            stages_out = k
            if (want_hist) then
                st = gk_true_residual(ctx, hist_res(k)); if (st /= GK_OK) return
            end if
            if (final_err(n_out) < tol) exit
        end do
        if (want_verr) then
            st = gk_hh_verr(ctx, n_out, v_err); if (st /= GK_OK) return
        end if
        if (present(keep_x)) then
            if (keep_x) return
        end if
        st = gk_get_x(ctx, x)
    end function hh_drive

    !> The fused short-recurrence solve (gk_sr_*): every scalar stays on the
    !> device, the iterations are queued in chunks of hip_sr_chunk and chunk k+1
    !> is queued before the host waits for chunk k; one status read per chunk.
    !> Iterations after convergence are no-ops on the device (the reference's
    !> `if (converged) cycle`).  iter: in = max iterations, out = the first i with
    !> res < tol (unchanged when none), as pcg_omp / pbicgstab_omp return it.
    integer function sr_drive(ctx, solver, tol, iter, res, want_hist, hist) result(st)
        type(c_ptr), intent(in) :: ctx
        integer(c_int), intent(in) :: solver
        real(8), intent(in) :: tol
        integer, intent(inout) :: iter
        real(8), intent(out) :: res
        logical, intent(in) :: want_hist
        real(8), intent(inout) :: hist(*)
        integer(c_int) :: executed, done, k, queued, maxit, wait
        maxit = int(max(iter, 0), c_int)
        res = 0.0d0
        st = gk_sr_start(ctx, solver, tol, maxit); if (st /= GK_OK) return
        k = int(min(hip_sr_chunk, maxit), c_int)
        st = gk_sr_iterate(ctx, k); if (st /= GK_OK) return
        queued = k
        do
            if (queued < maxit) then
                k = int(min(hip_sr_chunk, maxit - queued), c_int)
                st = gk_sr_iterate(ctx, k); if (st /= GK_OK) return
                queued = queued + k
            end if
            wait = merge(1_c_int, 0_c_int, queued >= maxit)
            st = gk_sr_status(ctx, wait, executed, done, res); if (st /= GK_OK) return
            if (done > 0 .or. wait == 1) exit
        end do
        st = gk_sr_status(ctx, 1_c_int, executed, done, res); if (st /= GK_OK) return
        if (done > 0) iter = done
        if (want_hist .and. executed > 0) st = gk_sr_history(ctx, hist, executed)
    end function sr_drive

    !> pcg_omp (src/cg.f90:154-234) on the fused device passes.
    integer function pcg_drive(ctx, tol, iter, res, want_hist, hist) result(st)
        type(c_ptr), intent(in) :: ctx
        real(8), intent(in) :: tol
        integer, intent(inout) :: iter
        real(8), intent(out) :: res
        logical, intent(in) :: want_hist
        real(8), intent(inout) :: hist(*)
        st = sr_drive(ctx, GK_SR_PCG, tol, iter, res, want_hist, hist)
    end function pcg_drive

    !> pbicgstab_omp (src/bicgstab.f90:91-182) on the fused device passes.
    integer function bicgstab_drive(ctx, tol, max_iter, res, want_hist, hist) result(st)
        type(c_ptr), intent(in) :: ctx
        real(8), intent(in) :: tol
        integer, intent(inout) :: max_iter
        real(8), intent(out) :: res
        logical, intent(in) :: want_hist
        real(8), intent(inout) :: hist(*)
        st = sr_drive(ctx, GK_SR_BICGSTAB, tol, max_iter, res, want_hist, hist)
    end function bicgstab_drive

    !> Preconditioned CG as the reference sequences it: pcg_omp
    !> (src/cg.f90:154-234) one BLAS-1 operation per device call, its scalars on
    !> the host (the A/B baseline of the fused pcg_drive, and its cross-check).
    !> iter: in = max iterations, out = first i with res < tol.
    integer function pcg_drive_seq(ctx, tol, iter, res, want_hist, hist) result(st)
        type(c_ptr), intent(in) :: ctx
        real(8), intent(in) :: tol
        integer, intent(inout) :: iter
        real(8), intent(out) :: res
        logical, intent(in) :: want_hist
        real(8), intent(inout) :: hist(*)
        integer(c_int), parameter :: VR = 2, VZ = 3, VP = 4, VAX = 5
        real(8) :: rr, pap, alpha, beta, rsq
        integer :: i, maxit
        logical :: converged
        converged = .false.
        maxit = iter
        res = 0.0d0
        st = gk_vec_lincomb(ctx, GK_LC_ZERO, GK_VEC_X, GK_VEC_X, GK_VEC_X, GK_VEC_X, 0.0d0, 0.0d0)
        if (st /= GK_OK) return
        st = gk_vec_lincomb(ctx, GK_LC_COPY, VR, GK_VEC_B, GK_VEC_B, GK_VEC_B, 0.0d0, 0.0d0); if (st /= GK_OK) return
        st = gk_vec_apply(ctx, 1_c_int, VR, VZ); if (st /= GK_OK) return              ! z = M^-1 r
        st = gk_vec_lincomb(ctx, GK_LC_COPY, VP, VZ, VZ, VZ, 0.0d0, 0.0d0); if (st /= GK_OK) return
        do i = 1, maxit
            if (converged) exit
            st = gk_vec_apply(ctx, 0_c_int, VP, VAX); if (st /= GK_OK) return       ! ax = A p
            st = gk_vec_dot(ctx, VR, VZ, rr); if (st /= GK_OK) return
            st = gk_vec_dot(ctx, VAX, VP, pap); if (st /= GK_OK) return
            alpha = rr/pap
            st = gk_vec_lincomb(ctx, GK_LC_AXPY, GK_VEC_X, GK_VEC_X, VP, VP, alpha, 0.0d0); if (st /= GK_OK) return
            st = gk_vec_lincomb(ctx, GK_LC_AXPY, VR, VR, VAX, VAX, -alpha, 0.0d0); if (st /= GK_OK) return
            st = gk_vec_dot(ctx, VR, VR, rsq); if (st /= GK_OK) return
            st = gk_vec_apply(ctx, 1_c_int, VR, VZ); if (st /= GK_OK) return        ! z = M^-1 r
            st = gk_vec_dot(ctx, VR, VZ, beta); if (st /= GK_OK) return
            res = sqrt(rsq)
            beta = beta/rr
            if (want_hist) hist(i) = res
            if (res < tol) then
                converged = .true.
                iter = i
            end if
            st = gk_vec_lincomb(ctx, GK_LC_AXPY, VP, VZ, VP, VP, beta, 0.0d0); if (st /= GK_OK) return  ! p = z + beta p
        end do
    end function pcg_drive_seq

    !> Preconditioned BiCGSTAB as the reference sequences it: pbicgstab_omp
    !> (src/bicgstab.f90:91-182), one operation per device call; the
    !> reference's uninitialised first-iteration accumulators are taken as 0.
    integer function bicgstab_drive_seq(ctx, tol, max_iter, res, want_hist, hist) result(st)
        type(c_ptr), intent(in) :: ctx
        real(8), intent(in) :: tol
        integer, intent(inout) :: max_iter
        real(8), intent(out) :: res
        logical, intent(in) :: want_hist
        real(8), intent(inout) :: hist(*)
        integer(c_int), parameter :: VR = 2, VR0 = 3, VAP = 4, VS = 5, VAS = 6, VP = 7, VZ1 = 8, VZ2 = 9
        real(8) :: rr0, ap_r0, as_s, as_as, r_r0_new, alpha, omega, beta, rsq
        integer :: i, iters
        logical :: converged
        converged = .false.
        iters = max_iter
        res = 0.0d0
        st = gk_vec_lincomb(ctx, GK_LC_ZERO, GK_VEC_X, GK_VEC_X, GK_VEC_X, GK_VEC_X, 0.0d0, 0.0d0)
        if (st /= GK_OK) return
        st = gk_vec_lincomb(ctx, GK_LC_COPY, VR, GK_VEC_B, GK_VEC_B, GK_VEC_B, 0.0d0, 0.0d0); if (st /= GK_OK) return
        st = gk_vec_lincomb(ctx, GK_LC_COPY, VR0, VR, VR, VR, 0.0d0, 0.0d0); if (st /= GK_OK) return
        st = gk_vec_lincomb(ctx, GK_LC_COPY, VP, VR0, VR0, VR0, 0.0d0, 0.0d0); if (st /= GK_OK) return
        do i = 1, max_iter
            if (converged) exit
            st = gk_vec_apply(ctx, 1_c_int, VP, VZ1); if (st /= GK_OK) return      ! z1 = M^-1 p
            st = gk_vec_apply(ctx, 0_c_int, VZ1, VAP); if (st /= GK_OK) return     ! ap = A z1
            st = gk_vec_dot(ctx, VR, VR0, rr0); if (st /= GK_OK) return
            st = gk_vec_dot(ctx, VAP, VR0, ap_r0); if (st /= GK_OK) return
            alpha = rr0/ap_r0
            st = gk_vec_lincomb(ctx, GK_LC_AXPY, VS, VR, VAP, VAP, -alpha, 0.0d0); if (st /= GK_OK) return
            st = gk_vec_apply(ctx, 1_c_int, VS, VZ2); if (st /= GK_OK) return      ! z2 = M^-1 s
            st = gk_vec_apply(ctx, 0_c_int, VZ2, VAS); if (st /= GK_OK) return     ! as = A z2
            st = gk_vec_dot(ctx, VAS, VS, as_s); if (st /= GK_OK) return
            st = gk_vec_dot(ctx, VAS, VAS, as_as); if (st /= GK_OK) return
            omega = as_s/as_as
            st = gk_vec_lincomb(ctx, GK_LC_AXPY2, GK_VEC_X, GK_VEC_X, VZ1, VZ2, alpha, omega); if (st /= GK_OK) return
            st = gk_vec_lincomb(ctx, GK_LC_AXPY, VR, VS, VAS, VAS, -omega, 0.0d0); if (st /= GK_OK) return
            st = gk_vec_dot(ctx, VR, VR, rsq); if (st /= GK_OK) return
            res = sqrt(rsq)
            if (want_hist) hist(i) = res
            if (res < tol) then
                iters = i
                converged = .true.
            end if
            st = gk_vec_dot(ctx, VR, VR0, r_r0_new); if (st /= GK_OK) return
            beta = (r_r0_new/rr0)*(alpha/omega)
            st = gk_vec_lincomb(ctx, GK_LC_XPAYMZ, VP, VR, VP, VAP, beta, omega); if (st /= GK_OK) return
        end do
        max_iter = iters
    end function bicgstab_drive_seq

    !> Drop-in for pcg_omp (src/cg.f90:154-162).
    subroutine pcg_hip(Ax_op, b, x, tol, iter, res, M_inv, params)
        procedure(stencil_vector) :: Ax_op
        real(8), intent(in) :: b(:)
        real(8), allocatable, intent(out) :: x(:)
        real(8), intent(in) :: tol
        integer, intent(inout) :: iter
        real(8), intent(out) :: res
        procedure(precond) :: M_inv
        real(8), intent(in) :: params(:)
        type(c_ptr) :: ctx
        integer(c_int) :: kind, degree
        real(8) :: dummy(1)
        call require_device_op(Ax_op, 'pcg_hip')
        call prec_kind(M_inv, params, kind, degree)
        allocate (x(size(b)))
        ctx = solver_ctx(b, 8, kind, degree, params)
        call gk_require(pcg_drive(ctx, tol, iter, res, .false., dummy), 'pcg_hip')
        call gk_require(gk_get_x(ctx, x), 'gk_get_x')
        call gk_require(gk_destroy(ctx), 'gk_destroy')
    end subroutine pcg_hip

    !> Drop-in for pbicgstab_omp (src/bicgstab.f90:91-99).
    subroutine pbicgstab_hip(ax_op, b, x, tol, max_iter, res, m_inv, params)
        procedure(stencil_vector) :: ax_op
        real(8), intent(in) :: b(:)
        real(8), allocatable, intent(out) :: x(:)
        real(8), intent(in) :: tol
        integer, intent(inout) :: max_iter
        real(8), intent(out) :: res
        procedure(precond) :: m_inv
        real(8), intent(in) :: params(:)
        type(c_ptr) :: ctx
        integer(c_int) :: kind, degree
        real(8) :: dummy(1)
        call require_device_op(ax_op, 'pbicgstab_hip')
        call prec_kind(m_inv, params, kind, degree)
        allocate (x(size(b)))
        ctx = solver_ctx(b, 8, kind, degree, params)
        call gk_require(bicgstab_drive(ctx, tol, max_iter, res, .false., dummy), 'pbicgstab_hip')
        call gk_require(gk_get_x(ctx, x), 'gk_get_x')
        call gk_require(gk_destroy(ctx), 'gk_destroy')
    end subroutine pbicgstab_hip

    ! ------------------------------------------------ host-array plug-ins --

    subroutine ensure_opctx(n)
        integer, intent(in) :: n
        if (opctx_n == n) return
        if (c_associated(opctx)) call gk_require(gk_destroy(opctx), 'gk_destroy')
        call gk_require(gk_create(int(hip_device, c_int), int(n, c_int), 0_c_int, int(n, c_int), 1_c_int, opctx), &
                        'gk_create')
        opctx_n = n
    end subroutine ensure_opctx

    !> Free the plug-ins' device context.
    subroutine hip_release()
        if (c_associated(opctx)) call gk_require(gk_destroy(opctx), 'gk_destroy')
        opctx = c_null_ptr
        opctx_n = -1
    end subroutine hip_release

    !> y = A x on the GPU; conforms to stencil_vector (replaces stvec,
    !> src/problems/poisson.f90:33-77).  As an Ax_vec argument it selects the
    !> device 5-point operator of the solvers below.
    subroutine hip_poisson5(x, y, n)
        real(8), intent(in) :: x(:)
        real(8), intent(out) :: y(:)
        integer, intent(in) :: n
        call ensure_opctx(n)
        call gk_require(gk_apply(opctx, 0_c_int, x, y), 'hip_poisson5')
    end subroutine hip_poisson5

    subroutine apply_prec(kind, params, degree, r, z, n)
        integer(c_int), intent(in) :: kind, degree
        real(8), intent(in) :: params(:), r(:)
        real(8), intent(out) :: z(:)
        integer, intent(in) :: n
        real(8) :: p(2)
        p = 0.0d0
        if (size(params) >= 2) p = params(1:2)
        call ensure_opctx(n)
        call gk_require(gk_set_precond(opctx, kind, p, 2_c_int, degree), 'gk_set_precond')
        call gk_require(gk_apply(opctx, 1_c_int, r, z), 'preconditioner')
    end subroutine apply_prec

    subroutine require_device_op(A_x, who)
        procedure(stencil_vector) :: A_x
        character(len=*), intent(in) :: who
        if (.not. c_associated(c_funloc(A_x), c_funloc(hip_poisson5))) then
            write (*, '(A,A)') who, ': the operator must be hip_poisson5 (device-resident 5-point stencil)'
            error stop 2
        end if
    end subroutine require_device_op

    !> z = r; conforms to precond (config 1 "no preconditioner").
    subroutine hip_identity(A_x, r, z, aux, params, n)
        procedure(stencil_vector) :: A_x
        real(8), intent(in) :: r(:)
        real(8), intent(out) :: z(:), aux(:)
        real(8), intent(in) :: params(:)
        integer, intent(in) :: n
        call require_device_op(A_x, 'hip_identity')
        call apply_prec(GK_PREC_IDENTITY, params, 1_c_int, r, z, n)
        aux = 0.0d0
    end subroutine hip_identity

    !> Two-term Chebyshev preconditioner of src/preconds/chebyshev.f90:8-38 on
    !> the GPU (one fused stencil sweep); conforms to precond.
    subroutine hip_cbpr2(A_x, r, z, aux, params, n)
        procedure(stencil_vector) :: A_x
        real(8), intent(in) :: r(:)
        real(8), intent(out) :: z(:), aux(:)
        real(8), intent(in) :: params(:)
        integer, intent(in) :: n
        call require_device_op(A_x, 'hip_cbpr2')
        call apply_prec(GK_PREC_CBPR2, params, 1_c_int, r, z, n)
        aux = 0.0d0
    end subroutine hip_cbpr2

    !> Chebyshev(k) polynomial preconditioner (build-defined, BASELINE config 3):
    !> k semi-iteration sweeps on [params(1), params(2)]; k = params(3) if given.
    subroutine hip_chebyshev(A_x, r, z, aux, params, n)
        procedure(stencil_vector) :: A_x
        real(8), intent(in) :: r(:)
        real(8), intent(out) :: z(:), aux(:)
        real(8), intent(in) :: params(:)
        integer, intent(in) :: n
        call require_device_op(A_x, 'hip_chebyshev')
        call apply_prec(GK_PREC_CHEB, params, int(cheb_degree(params), c_int), r, z, n)
        aux = 0.0d0
    end subroutine hip_chebyshev

    integer function cheb_degree(params) result(k)
        real(8), intent(in) :: params(:)
        k = hip_cheb_degree
        if (size(params) >= 3) k = nint(params(3))
    end function cheb_degree

    subroutine prec_kind(M_inv, params, kind, degree)
        procedure(precond) :: M_inv
        real(8), intent(in) :: params(:)
        integer(c_int), intent(out) :: kind, degree
        degree = 1
        if (c_associated(c_funloc(M_inv), c_funloc(hip_identity))) then
            kind = GK_PREC_IDENTITY
        else if (c_associated(c_funloc(M_inv), c_funloc(hip_cbpr2))) then
            kind = GK_PREC_CBPR2
        else if (c_associated(c_funloc(M_inv), c_funloc(hip_chebyshev))) then
            kind = GK_PREC_CHEB
            degree = int(cheb_degree(params), c_int)
        else
            write (*, '(A)') 'gmres_hip: M_inv must be hip_identity, hip_cbpr2 or hip_chebyshev'
            error stop 2
        end if
    end subroutine prec_kind

    type(c_ptr) function solver_ctx(b, m, kind, degree, params) result(ctx)
        real(8), intent(in) :: b(:), params(:)
        integer, intent(in) :: m
        integer(c_int), intent(in) :: kind, degree
        integer :: nsize
        real(8) :: p(2)
        nsize = grid_side(size(b))
        p = 0.0d0
        if (size(params) >= 2) p = params(1:2)
        call gk_require(gk_create(int(hip_device, c_int), int(nsize, c_int), 0_c_int, int(nsize, c_int), &
                                  int(m, c_int), ctx), 'gk_create')
        call gk_require(gk_set_precond(ctx, kind, p, 2_c_int, degree), 'gk_set_precond')
        call gk_require(gk_set_rhs(ctx, b), 'gk_set_rhs')
    end function solver_ctx

    ! ------------------------------------------------- drop-in solvers ------

    !> Drop-in for gmres_mgsr_omp (src/gmres_mgsr.f90:277-288), same argument
    !> list; Ax_vec must be hip_poisson5 and M_inv one of the hip_* plug-ins.
    !> Optional variant = MGSR_MF reproduces gmres_mgsr_mf (:98-109).
    subroutine gmres_mgsr_hip(Ax_vec, b, x, m, tol, final_err, v_err, n_out, restart_out, M_inv, params, variant)
        procedure(stencil_vector) :: Ax_vec
        real(8), intent(in) :: b(:)
        real(8), allocatable, intent(out) :: x(:)
        integer, intent(in) :: m
        real(8), intent(in) :: tol
        real(8), allocatable, intent(out) :: final_err(:), v_err(:)
        integer, intent(out) :: n_out, restart_out
        procedure(precond) :: M_inv
        real(8), intent(in) :: params(:)
        integer, intent(in), optional :: variant
        type(c_ptr) :: ctx
        integer(c_int) :: kind, degree
        integer :: var, ncyc
        real(8) :: dummy_h(1), dummy_f(1, 1)
        call require_device_op(Ax_vec, 'gmres_mgsr_hip')
        call prec_kind(M_inv, params, kind, degree)
        var = MGSR_OMP
        if (present(variant)) var = variant
        allocate (x(size(b)), final_err(m), v_err(m + 1))
        ctx = solver_ctx(b, m, kind, degree, params)
        call gk_require(mgsr_drive(ctx, m, tol, norm2(b), var, hip_max_restarts, x, final_err, v_err, n_out, &
                                   restart_out, .true., .false., dummy_h, dummy_f, ncyc), 'gmres_mgsr_hip')
        call gk_require(gk_destroy(ctx), 'gk_destroy')
    end subroutine gmres_mgsr_hip

    !> Drop-in for gmres_hh_omp (src/gmres_hh.f90:211-219): no preconditioner,
    !> full cycles.
    subroutine gmres_hh_hip(Ax_vec, b, x, m, tol, final_err, v_err, n_out, stages_out)
        procedure(stencil_vector) :: Ax_vec
        real(8), intent(in) :: b(:)
        real(8), allocatable, intent(out) :: x(:)
        integer, intent(in) :: m
        real(8), intent(in) :: tol
        real(8), allocatable, intent(out) :: final_err(:), v_err(:)
        integer, intent(out) :: n_out, stages_out
        type(c_ptr) :: ctx
        integer :: ncyc
        real(8) :: dummy_h(1), dummy_f(1, 1), p(2)
        call require_device_op(Ax_vec, 'gmres_hh_hip')
        allocate (x(size(b)), final_err(m), v_err(m + 1))
        p = 0.0d0
        ctx = solver_ctx(b, m, GK_PREC_IDENTITY, 1_c_int, p)
        call gk_require(hh_drive(ctx, m, tol, norm2(b), 0, .false., hip_max_restarts, x, final_err, v_err, &
                                 n_out, stages_out, .true., .false., dummy_h, dummy_f, ncyc), 'gmres_hh_hip')
        call gk_require(gk_destroy(ctx), 'gk_destroy')
    end subroutine gmres_hh_hip

    !> Drop-in for gmres_hh_prec_omp (src/gmres_hh.f90:388-398).
    subroutine gmres_hh_prec_hip(Ax_vec, b, x, m, tol, final_err, v_err, n_out, stages_out, m_inv, params)
        procedure(stencil_vector) :: Ax_vec
        real(8), intent(in) :: b(:)
        real(8), allocatable, intent(out) :: x(:)
        integer, intent(in) :: m
        real(8), intent(in) :: tol
        real(8), allocatable, intent(out) :: final_err(:), v_err(:)
        integer, intent(out) :: n_out, stages_out
        procedure(precond) :: m_inv
        real(8), intent(in) :: params(:)
        type(c_ptr) :: ctx
        integer(c_int) :: kind, degree
        integer :: ncyc
        real(8) :: dummy_h(1), dummy_f(1, 1)
        call require_device_op(Ax_vec, 'gmres_hh_prec_hip')
        call prec_kind(m_inv, params, kind, degree)
        allocate (x(size(b)), final_err(m), v_err(m + 1))
        ctx = solver_ctx(b, m, kind, degree, params)
        call gk_require(hh_drive(ctx, m, tol, norm2(b), 1, .true., hip_max_restarts, x, final_err, v_err, &
                                 n_out, stages_out, .true., .false., dummy_h, dummy_f, ncyc), 'gmres_hh_prec_hip')
        call gk_require(gk_destroy(ctx), 'gk_destroy')
    end subroutine gmres_hh_prec_hip

end module gmres_hip

! ----------------------------------------------------------------------------
! bind(C) drivers for a harness that already holds a device context (the
! Python bench / tests, or any C/C++ host).  Arrays are the local slab;
! keep_x /= 0 leaves the solution in HBM (x is not written: read it later with
! gk_get_x), so a timed solve moves nothing over PCIe.
! ----------------------------------------------------------------------------

integer(c_int) function gmres_mgsr_hip_run(ctx, m, tol, variant, max_cyc, x, final_err, v_err, n_out, &
                                           restart_out, want_verr, want_hist, hist_res, hist_ferr, n_cycles, &
                                           keep_x) bind(C, name='gmres_mgsr_hip_run')
    use, intrinsic :: iso_c_binding
    use gmres_hip_c
    use gmres_hip, only: mgsr_drive
    implicit none
    type(c_ptr), value :: ctx
    integer(c_int), value :: m, variant, max_cyc, want_verr, want_hist, keep_x
    real(c_double), value :: tol
    real(c_double), intent(out) :: x(*), final_err(*), v_err(*)
    real(c_double), intent(inout) :: hist_res(*), hist_ferr(*)
    integer(c_int), intent(out) :: n_out, restart_out, n_cycles
    real(8) :: beta0
    integer :: no, ro, nc
    gmres_mgsr_hip_run = gk_rhs_norm(ctx, beta0)
    if (gmres_mgsr_hip_run /= GK_OK) return
    gmres_mgsr_hip_run = mgsr_drive(ctx, int(m), tol, beta0, int(variant), int(max_cyc), x, final_err, v_err, &
                                    no, ro, want_verr /= 0, want_hist /= 0, hist_res, hist_ferr, nc, keep_x /= 0)
    n_out = no; restart_out = ro; n_cycles = nc
end function gmres_mgsr_hip_run

integer(c_int) function gmres_hh_hip_run(ctx, m, tol, precondition, midcycle_exit, max_cyc, x, final_err, &
                                         v_err, n_out, stages_out, want_verr, want_hist, hist_res, hist_ferr, &
                                         n_cycles, keep_x) bind(C, name='gmres_hh_hip_run')
    use, intrinsic :: iso_c_binding
    use gmres_hip_c
    use gmres_hip, only: hh_drive
    implicit none
    type(c_ptr), value :: ctx
    integer(c_int), value :: m, precondition, midcycle_exit, max_cyc, want_verr, want_hist, keep_x
    real(c_double), value :: tol
    real(c_double), intent(out) :: x(*), final_err(*), v_err(*)
    real(c_double), intent(inout) :: hist_res(*), hist_ferr(*)
    integer(c_int), intent(out) :: n_out, stages_out, n_cycles
    real(8) :: beta0
    integer :: no, so, nc
    gmres_hh_hip_run = gk_rhs_norm(ctx, beta0)
    if (gmres_hh_hip_run /= GK_OK) return
    gmres_hh_hip_run = hh_drive(ctx, int(m), tol, beta0, int(precondition), midcycle_exit /= 0, int(max_cyc), &
                                x, final_err, v_err, no, so, want_verr /= 0, want_hist /= 0, hist_res, &
                                hist_ferr, nc, keep_x /= 0)
    n_out = no; stages_out = so; n_cycles = nc
end function gmres_hh_hip_run

integer(c_int) function pcg_hip_run(ctx, tol, iter, res, want_hist, hist) bind(C, name='pcg_hip_run')
    use, intrinsic :: iso_c_binding
    use gmres_hip, only: pcg_drive
    implicit none
    type(c_ptr), value :: ctx
    real(c_double), value :: tol
    integer(c_int), intent(inout) :: iter
    real(c_double), intent(out) :: res
    integer(c_int), value :: want_hist
    real(c_double), intent(inout) :: hist(*)
    integer :: it
    it = iter
    pcg_hip_run = pcg_drive(ctx, tol, it, res, want_hist /= 0, hist)
    iter = it
end function pcg_hip_run

integer(c_int) function pbicgstab_hip_run(ctx, tol, max_iter, res, want_hist, hist) bind(C, name='pbicgstab_hip_run')
    use, intrinsic :: iso_c_binding
    use gmres_hip, only: bicgstab_drive
    implicit none
    type(c_ptr), value :: ctx
    real(c_double), value :: tol
    integer(c_int), intent(inout) :: max_iter
    real(c_double), intent(out) :: res
    integer(c_int), value :: want_hist
    real(c_double), intent(inout) :: hist(*)
    integer :: it
    it = max_iter
    pbicgstab_hip_run = bicgstab_drive(ctx, tol, it, res, want_hist /= 0, hist)
    max_iter = it
end function pbicgstab_hip_run

!> The as-written sequence (one device call per BLAS-1 operation, scalars on
!> the host): solver 0 = pcg_drive_seq, 1 = bicgstab_drive_seq.
integer(c_int) function sr_hip_run_seq(ctx, solver, tol, iter, res, want_hist, hist) bind(C, name='sr_hip_run_seq')
    use, intrinsic :: iso_c_binding
    use gmres_hip, only: pcg_drive_seq, bicgstab_drive_seq
    implicit none
    type(c_ptr), value :: ctx
    integer(c_int), value :: solver
    real(c_double), value :: tol
    integer(c_int), intent(inout) :: iter
    real(c_double), intent(out) :: res
    integer(c_int), value :: want_hist
    real(c_double), intent(inout) :: hist(*)
    integer :: it
    it = iter
    if (solver == 0) then
        sr_hip_run_seq = pcg_drive_seq(ctx, tol, it, res, want_hist /= 0, hist)
    else
        sr_hip_run_seq = bicgstab_drive_seq(ctx, tol, it, res, want_hist /= 0, hist)
    end if
    iter = it
end function sr_hip_run_seq
