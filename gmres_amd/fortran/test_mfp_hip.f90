!! test_mfp_hip -- `test_mfp` (tests/test_poisson_mf.f90) on the GPU.
!! Same CLI (<grid size> <iterations per restart>), same manufactured problem
!! (b = A*1, tol = 1e-15, Chebyshev params (8.2, 0.2)) and the same printed
!! lines; the only source change a reference user makes is the call names:
!!   stvec -> hip_poisson5, cbpr2 -> hip_cbpr2,
!!   gmres_hh_prec_omp -> gmres_hh_prec_hip, gmres_mgsr_omp -> gmres_mgsr_hip.
program test_mfp_hip
    use gmres_hip
    implicit none
    integer :: nsize, max_iter, n_args
    character(len=32) :: arg_str
    n_args = command_argument_count()
    if (n_args < 2) then
        print *, "usage ./test_mfp_hip <grid size> <iterations per restart>"
        stop
    end if
    call get_command_argument(1, arg_str)
    read (arg_str, *) nsize
    call get_command_argument(2, arg_str)
    read (arg_str, *) max_iter
    write (*, '(60("-"))')
    call run(nsize, max_iter, .true.)
    write (*, '(60("-"))')
    call run(nsize, max_iter, .false.)
    write (*, '(60("-"))')
    call hip_release()
contains
    subroutine run(nsize, max_iter, householder)
        integer, intent(in) :: nsize, max_iter
        logical, intent(in) :: householder
        real(8), allocatable :: b(:), x(:), errn(:), verr(:), params(:)
        real(8) :: tol
        integer :: n_iter, n_stages, c0, c1, crate
        tol = 1.d-15
        allocate (b(nsize*nsize), x(nsize*nsize), params(2))
        params(1) = 8.2d0; params(2) = 0.2d0
        x = 1.0d0
        call hip_poisson5(x, b, nsize)   ! b = A*1: every solution entry must be 1.0
        if (householder) then
            write (*, '(A)') 'GMRES Poisson 2D Test Matrix Free (Householder Chebyshev, MI355X)'
        else
            write (*, '(A)') 'GMRES Poisson 2D Test Matrix Free (MGSR Chebyshev, MI355X)'
        end if
        write (*, '(A,I8,A18,I5,A8,ES10.2)') "N VARS=", nsize*nsize, " MAX ITERS/STAGE=", max_iter, " TOL=", tol
        call system_clock(c0, crate)
        if (householder) then
            call gmres_hh_prec_hip(hip_poisson5, b, x, max_iter, tol, errn, verr, n_iter, n_stages, hip_cbpr2, params)
        else
            call gmres_mgsr_hip(hip_poisson5, b, x, max_iter, tol, errn, verr, n_iter, n_stages, hip_cbpr2, params)
        end if
        call system_clock(c1)
        write (*, '(A30, I8, A10, I4)') 'Iterations until convergence:', (n_stages - 1)*max_iter + n_iter, &
            ' Stages=', n_stages
        write (*, '(A30, ES12.4)') "Final ||I - V.t * V||:", verr(n_iter)
        write (*, '(A30, ES12.4)') 'Final residual:', errn(n_iter)
        write (*, '(A30, ES12.4)') 'Max error L_max:', maxval(abs(x - 1.0d0))
        write (*, '(A30, ES12.4)') 'L2 norm:', norm2(x - 1.0d0)
        write (*, '(A30, 10F10.4)') 'First 10 solution elements', x(1:10)
        write (*, '(A30, F12.4, A)') 'Elapsed time:', dble(c1 - c0)/dble(crate), ' secs.'
    end subroutine run
end program test_mfp_hip
