!! sweep_hip -- the reference's sweep drivers on the GPU, printing their table
!! layout (gmres_hip_report = utils.f90 print_header/print_line columns):
!!   sweep_hip m     <N> <ntests>   restart-length sweep m = 20, 25, ...
!!                                  (tests/weak_scaling.f90: HH + cbpr2)
!!   sweep_hip grid  <N0> <ntests>  grid sweep N = N0, N0+30, ... at m = 90
!!                                  (tests/test1.f90: MGS-R + cbpr2)
!!   sweep_hip prec  <N> <m>        one MGS-R solve per preconditioner
!! The Info column names the device instead of an OpenMP thread count.
program sweep_hip
    use gmres_hip
    use gmres_hip_report
    implicit none
    character(len=32) :: mode, arg
    integer :: nsize, ntests, i, m
    if (command_argument_count() < 3) then
        print *, "usage ./sweep_hip <m|grid|prec> <grid size> <num tests | m>"
        stop
    end if
    call get_command_argument(1, mode)
    call get_command_argument(2, arg)
    read (arg, *) nsize
    call get_command_argument(3, arg)
    read (arg, *) ntests
    select case (trim(mode))
    case ('m')
        call report_header('GMRES restart sweep (Householder with Chebyshev precond, MI355X)')
        do i = 1, ntests
            m = 20 + 5*(i - 1)
            call run(i, nsize, m, 'hh', 'cbpr2')
        end do
    case ('grid')
        call report_header('GMRES grid sweep (MGSR with Chebyshev precond, MI355X)')
        do i = 1, ntests
            call run(i, nsize + 30*(i - 1), 90, 'mgsr', 'cbpr2')
        end do
    case ('prec')
        call report_header('GMRES preconditioner comparison (MGSR, MI355X)')
        call run(1, nsize, ntests, 'mgsr', 'identity')
        call run(2, nsize, ntests, 'mgsr', 'cbpr2')
        call run(3, nsize, ntests, 'mgsr', 'cheb')
    case default
        print *, "unknown mode ", trim(mode)
        stop 1
    end select
    write (*, '(150("-"))')
    call hip_release()
contains
    subroutine run(test, n, m, method, prec)
        integer, intent(in) :: test, n, m
        character(len=*), intent(in) :: method, prec
        real(8), allocatable :: b(:), x(:), errn(:), verr(:), params(:)
        integer :: n_iter, n_stages, c0, c1, crate
        real(8) :: tol
        tol = 1.d-15
        allocate (b(n*n), x(n*n), params(3))
        params = [8.2d0, 0.2d0, 8.0d0]
        x = 1.0d0
        call hip_poisson5(x, b, n)
        call system_clock(c0, crate)
        if (method == 'hh') then
            call gmres_hh_prec_hip(hip_poisson5, b, x, m, tol, errn, verr, n_iter, n_stages, hip_cbpr2, params)
        else if (prec == 'identity') then
            call gmres_mgsr_hip(hip_poisson5, b, x, m, tol, errn, verr, n_iter, n_stages, hip_identity, params)
        else if (prec == 'cheb') then
            call gmres_mgsr_hip(hip_poisson5, b, x, m, tol, errn, verr, n_iter, n_stages, hip_chebyshev, params)
        else
            call gmres_mgsr_hip(hip_poisson5, b, x, m, tol, errn, verr, n_iter, n_stages, hip_cbpr2, params)
        end if
        call system_clock(c1)
        call report_line(test, n*n, dble(c1 - c0)/dble(crate), (n_stages - 1)*m + n_iter, n_stages, m, tol, &
                         errn(n_iter), verr(n_iter), norm2(x - 1.0d0), maxval(abs(x - 1.0d0)), &
                         trim(method)//'+'//trim(prec))
    end subroutine run
end program sweep_hip
