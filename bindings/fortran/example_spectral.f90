! example_spectral.f90 — the reference's spectral unit test (test/optical_props/
! test_opticalprops.f90:81-142) through the binding: the same tables, spectral(...) then 10^4
! updates, each checked against the test's bounds. Host-side sampling only (no GPU needed).
! usage: example_spectral OUT  ->  prints "spectral OK" or the failed check; OUT holds the
! first 100 samples (wavelength, mus, mua, hgg, n; stream access, real64) for comparison.
program example_spectral
    use smcrt_mod
    use smcrt_glue
    implicit none
    real(c_double), allocatable :: flux(:, :), mua_a(:, :), hgg_a(:, :), n_a(:, :), mus_a(:, :)
    type(smcrt_optprop) :: o
    real(c_double) :: wave
    integer(c_int64_t) :: draw
    integer(c_int64_t), parameter :: seed = 1234569
    character(len=512) :: out
    integer :: i, u

    call get_command_argument(1, out)
    allocate(mua_a(10, 2))
    mua_a(:, 1) = [100, 200, 300, 400, 500, 600, 700, 800, 900, 1000]
    mua_a(:, 2) = [0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1]
    allocate(flux(10, 2))
    flux(:, 1) = [100, 200, 300, 400, 500, 600, 700, 800, 900, 1000]
    flux(:, 2) = [1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0]
    allocate(n_a(10, 2))
    n_a(:, 1) = [100, 200, 300, 400, 500, 600, 700, 800, 900, 1000]
    n_a(:, 2) = [1.0, 1.5, 1.5, 1.0, 1.5, 1.8, 1.9, 2.0, 2.1, 2.2]
    allocate(mus_a(10, 2))
    mus_a(:, 1) = [100, 200, 300, 400, 500, 600, 700, 800, 900, 1000]
    mus_a(:, 2) = [0.0, 1.0, 2.0, 3.0, 4.0, 3.0, 2.0, 1.0, 0.5, 0.0]
    allocate(hgg_a(3, 2))
    hgg_a(:, 1) = [100, 450, 900]
    hgg_a(:, 2) = [0.9, 0.9, 0.9]

    draw = 0
    o = smcrt_spectral_props(mus_a, mua_a, hgg_a, n_a, flux, seed, draw)   ! spectral(...)
    open(newunit=u, file=trim(out), access="stream", form="unformatted", status="replace")
    do i = 1, 10000                                                         ! optProp%update(wave)
        o = smcrt_spectral_props(mus_a, mua_a, hgg_a, n_a, flux, seed, draw, SMCRT_SPECTRAL_UPDATE, wave)
        if (i <= 100) write(u) wave, o%mus, o%mua, o%hgg, o%n
        if (wave < 100 .or. wave > 1000) call fail("Expected a wavelength between [100, 1000]!")
        if (abs(o%hgg - 0.9_c_double) > 0.05_c_double) call fail("hgg")
        if (abs(o%mua - 0.1_c_double) > 0.05_c_double) call fail("mua")
        if (o%n < 1.0 .or. o%n > 2.2) call fail("Expected a refractive between [1, 2.2]!")
        if (o%mus < 0.0 .or. o%mus > 4.0) call fail("Expected mus between [0.0, 4.0]!")
        if (o%flags /= SMCRT_NODE_ALBEDO_UNGUARDED) call fail("updateSpectral's albedo rule")
    end do
    close(u)
    print '(a)', "spectral OK"
contains
    subroutine fail(msg)
        character(len=*), intent(in) :: msg
        print '(a)', "Spectral check failed! "//msg
        error stop 1
    end subroutine fail
end program example_spectral
