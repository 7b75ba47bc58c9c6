!! ref_driver -- TEST INFRASTRUCTURE (oracle/_ref): runs the REFERENCE's own
!! solver modules, compiled from /root/reference/src by oracle/Makefile.ref,
!! through their operator seam (src/interfaces.f90:13-27).  It is the checker
!! and the CPU baseline, never part of the product path (gmres_amd/).
!!
!! This file is ours: a driver in the shape of tests/test_poisson_mf.f90 and
!! tests/strong_scaling.f90 (b = A*1, x0 = 0, params (8.2, 0.2)) that wraps
!! the reference's stvec (src/problems/poisson.f90:33-77) in an instrumented
!! operator `op` (SURVEY 8c step 5): every call is counted once per team; the
!! call that opens restart cycle k sees x_{k-1}, so it logs the TRUE relative
!! residual ||b - A x_{k-1}|| / ||b||; the call that opens Arnoldi step j of
!! cycle 1 logs an omp_get_wtime stamp (step timing for the CPU baseline).
!! MAXCYC / STEPLIM end the run after K cycles / S steps of cycle 1 (the
!! reference has no such knob: it runs up to 1000 restarts).
!!
!! usage: ref_driver <solver> <N> <m> <prec> <max_cycles> <step_limit> [xfile]
!!   solver: mgsr_mf | mgsr_omp | hh_omp | hh_prec_omp | pcg_omp | pbicgstab_omp
!!   prec:   identity | cbpr2        threads: OMP_NUM_THREADS
!!   max_cycles = 0 / step_limit = 0: no cap.  xfile: x written as raw fp64.
!!   env REF_TIME_CAP=<s>: also end the run at the first step of cycle 1 that
!!   opens after <s> seconds (bounded CPU-baseline samples).
!!   env REF_TOL=<tol>: the GMRES tol (default 1e-15).  A tol between cycle 1's
!!   final_err(m-1) and final_err(m) ends the solve normally after exactly one
!!   full cycle, so final_err(1:m) and x of cycle 1 are printed.
!! Output: one "KEY values..." record per line (parsed by oracle/refrun.py).
module ref_seam
    use interfaces, only: stencil_vector
    use poisson, only: stvec
    use omp_lib
    use iso_c_binding
    implicit none
    real(8), allocatable :: b_ref(:)
    real(8) :: bnorm = 1.0d0, t_over = 0.0d0, t0 = 0.0d0, t_cap = 0.0d0
    integer :: ncall = 0, per = 1, mm = 1, max_cyc = 0, step_lim = 0
    logical :: counting = .false.
    interface
        subroutine c_exit(status) bind(C, name="_exit")
            import :: c_int
            integer(c_int), value :: status
        end subroutine
    end interface
contains
    subroutine op(x, y, n)  ! conforms to stencil_vector (src/interfaces.f90:13-17)
        real(8), intent(in) :: x(:)
        real(8), intent(out) :: y(:)
        integer, intent(in) :: n
        integer :: c, k, j
        real(8) :: s, ta, tb
        call stvec(x, y, n)
        !$omp single
        if (counting) then
            ta = omp_get_wtime()
            ncall = ncall + 1
            c = ncall - 1
            if (mod(c, per*(mm+1)) == 0) then          ! cycle k = c/(per(m+1)) + 1 opens
                k = c / (per*(mm+1)) + 1
                s = norm2(b_ref - y)   ! the intrinsic the solvers use (flang-rt scaled sum)
                write(*, '(A, I6, 2ES26.17)') 'CYC ', k, s / bnorm, ta - t0 - t_over
                if (max_cyc > 0 .and. k > max_cyc) call finish_cut()
            else if (k_of(c) == 1 .and. mod(c, per) == 0) then   ! Arnoldi step j of cycle 1 opens
                j = c / per
                write(*, '(A, I6, ES26.17)') 'STEP ', j, ta - t0 - t_over
                if (step_lim > 0 .and. j > step_lim) call finish_cut()
                if (t_cap > 0.0d0 .and. ta - t0 - t_over > t_cap) call finish_cut()
            end if
            tb = omp_get_wtime()
            t_over = t_over + (tb - ta)
        end if
        !$omp end single
    end subroutine op

    integer function k_of(c)
        integer, intent(in) :: c
        k_of = c / (per*(mm+1)) + 1
    end function

    subroutine finish_cut()
        write(*, '(A)') 'CUT'
        flush(6)
        call c_exit(0_c_int)   ! inside a parallel region: leave without tearing the team down
    end subroutine

    subroutine identity(A_x, r, z, aux, params, n)  ! conforms to precond (interfaces.f90:20-27)
        procedure(stencil_vector) :: A_x
        real(8), intent(in) :: r(:)
        real(8), intent(out) :: z(:), aux(:)
        real(8), intent(in) :: params(:)
        integer, intent(in) :: n
        integer :: i
        !$omp do
        do i = 1, size(r)
            z(i) = r(i)
        end do
        !$omp end do
    end subroutine identity
end module ref_seam

program ref_driver
    use ref_seam
    use poisson, only: stvec
    use chebyshev_precond, only: cbpr2
    use gmres_mgsr_mod, only: gmres_mgsr_mf, gmres_mgsr_omp
    use gmres_hh_mod, only: gmres_hh_omp, gmres_hh_prec_omp
    use conjugate_gradient, only: pcg_omp
    use bicgstab_mod, only: pbicgstab_omp
    use omp_lib
    implicit none
    character(len=32) :: solver, prec, arg
    character(len=512) :: xfile
    integer :: N, m, n_out, cyc_out, iters, i, nthr, u
    real(8), allocatable :: b(:), x(:), ones(:), fe(:), ve(:), params(:)
    real(8) :: tol, res, s, t1

    if (command_argument_count() < 6) then
        print *, 'usage: ref_driver <solver> <N> <m> <prec> <max_cycles> <step_limit> [xfile]'
        stop 2
    end if
    call get_command_argument(1, solver)
    call get_command_argument(2, arg); read(arg, *) N
    call get_command_argument(3, arg); read(arg, *) m
    call get_command_argument(4, prec)
    call get_command_argument(5, arg); read(arg, *) max_cyc
    call get_command_argument(6, arg); read(arg, *) step_lim
    xfile = ''
    if (command_argument_count() >= 7) call get_command_argument(7, xfile)
    call get_environment_variable('REF_TIME_CAP', arg, status=i)
    if (i == 0) read(arg, *) t_cap

    allocate(b(N*N), ones(N*N), params(2))
    params(1) = 8.2d0; params(2) = 0.2d0                 ! tests/test_poisson_mf.f90:38
    ones = 1.0d0
    call stvec(ones, b, N)                               ! b = A*1 (test_poisson_mf.f90:39-40)
    allocate(b_ref(N*N)); b_ref = b
    bnorm = norm2(b)
    mm = m
    per = 1
    if (trim(prec) == 'cbpr2') per = 2
    !$omp parallel
    !$omp masked
    nthr = omp_get_num_threads()
    !$omp end masked
    !$omp end parallel
    write(*, '(A, A, A, A, 3I8)') 'RUN ', trim(solver), ' ', trim(prec), N, m, nthr
    tol = 1.0d-15
    call get_environment_variable('REF_TOL', arg, status=i)
    if (i == 0) read(arg, *) tol
    counting = .true.
    t0 = omp_get_wtime()
    select case (trim(solver))
    case ('mgsr_mf')
        if (per == 2) then
            call gmres_mgsr_mf(op, b, x, m, tol, fe, ve, n_out, cyc_out, cbpr2, params)
        else
            call gmres_mgsr_mf(op, b, x, m, tol, fe, ve, n_out, cyc_out, identity, params)
        end if
    case ('mgsr_omp')
        if (per == 2) then
            call gmres_mgsr_omp(op, b, x, m, tol, fe, ve, n_out, cyc_out, cbpr2, params)
        else
            call gmres_mgsr_omp(op, b, x, m, tol, fe, ve, n_out, cyc_out, identity, params)
        end if
    case ('hh_omp')
        call gmres_hh_omp(op, b, x, m, tol, fe, ve, n_out, cyc_out)
    case ('hh_prec_omp')
        if (per == 2) then
            call gmres_hh_prec_omp(op, b, x, m, tol, fe, ve, n_out, cyc_out, cbpr2, params)
        else
            call gmres_hh_prec_omp(op, b, x, m, tol, fe, ve, n_out, cyc_out, identity, params)
        end if
    case ('pcg_omp', 'pbicgstab_omp')
        counting = .false.
        tol = 1.0d-9                                     ! tests/test_cg.f90:20
        iters = m
        if (trim(solver) == 'pcg_omp') then
            if (per == 2) then
                call pcg_omp(stvec, b, x, tol, iters, res, cbpr2, params)
            else
                call pcg_omp(stvec, b, x, tol, iters, res, identity, params)
            end if
        else
            if (per == 2) then
                call pbicgstab_omp(stvec, b, x, tol, iters, res, cbpr2, params)
            else
                call pbicgstab_omp(stvec, b, x, tol, iters, res, identity, params)
            end if
        end if
        t1 = omp_get_wtime()
        write(*, '(A, I8, ES26.17)') 'KRYLOV ', iters, res
        call write_x()
        write(*, '(A, ES26.17)') 'TIME ', t1 - t0
        write(*, '(A)') 'DONE'
        stop
    case default
        print *, 'unknown solver ', trim(solver)
        stop 2
    end select
    t1 = omp_get_wtime()
    counting = .false.
    write(*, '(A, ES26.17)') 'TIME ', t1 - t0 - t_over
    write(*, '(A, 2I8)') 'OUT ', n_out, cyc_out
    call stvec(x, ones, N)
    write(*, '(A, ES26.17)') 'FINALRES ', norm2(b - ones) / bnorm
    write(*, '(A, I6)', advance='no') 'FERR ', n_out
    do i = 1, n_out
        write(*, '(ES26.17)', advance='no') fe(i)
    end do
    write(*, *)
    write(*, '(A, I6)', advance='no') 'VERR ', size(ve)
    do i = 1, size(ve)
        write(*, '(ES26.17)', advance='no') ve(i)
    end do
    write(*, *)
    call write_x()
    write(*, '(A)') 'DONE'
contains
    subroutine write_x()
        s = 0.0d0
        do i = 1, N*N
            s = s + (x(i) - 1.0d0)**2
        end do
        write(*, '(A, 2ES26.17)') 'XERR ', sqrt(s), maxval(abs(x - 1.0d0))
        if (len_trim(xfile) > 0) then
            open(newunit=u, file=trim(xfile), access='stream', form='unformatted', status='replace')
            write(u) x
            close(u)
        end if
    end subroutine write_x
end program ref_driver
