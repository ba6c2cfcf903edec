! example_scat_test.f90 — the reference's end-to-end scatter KAT (test/end_to_end/test_scat.f90:
! 33-38, res/scat_test.toml via test_kernel) driven from Fortran through smcrt_mod.
! Usage: example_scat_test [nphotons [n_gpus]]; prints "nscatt/photon = <value>" (KAT: 57.5 +- 0.5).
! n_gpus > 0 runs the photons through smcrt_multi_run on devices 0 .. n_gpus-1 (run_MCRT's
! n_gpus setting, INTEGRATION.md §2.1) instead of smcrt_run on device 0; the counters it prints
! are the same either way.
program example_scat_test
    use smcrt_mod
    implicit none

    type(smcrt_sdf_node)   :: nodes(2)
    integer(c_int32_t)     :: top(2)
    type(smcrt_grid)       :: grid
    type(smcrt_detector)   :: dets(1)
    type(smcrt_source)     :: src
    type(smcrt_run_config) :: cfg
    type(smcrt_tallies)    :: io
    type(c_ptr)            :: scene, multi
    integer(c_int32_t)     :: n_gpus
    real(c_float), allocatable, target :: jmean(:, :, :)
    real(c_double), target     :: nscatt
    integer(c_int64_t), target :: counters(SMCRT_NCOUNTERS)
    real(c_double) :: ident(16)
    integer :: ierr, nargs, i
    character(len=32) :: arg
    integer(c_int64_t) :: nphotons

    nphotons = 100000_c_int64_t
    nargs = command_argument_count()
    if (nargs >= 1) then
        call get_command_argument(1, arg)
        read(arg, *) nphotons
    end if
    n_gpus = 0
    if (nargs >= 2) then
        call get_command_argument(2, arg)
        read(arg, *) n_gpus
    end if

    ident = 0._c_double
    ident(1) = 1._c_double; ident(6) = 1._c_double; ident(11) = 1._c_double; ident(16) = 1._c_double

    ! setup_scat_test, setupGeometry.f90:409-435: sphere r=1 (mus=tau=10, g=0), box 2^3 (mus=0)
    nodes(1)%kind = SMCRT_SDF_SPHERE; nodes(1)%layer = 1; nodes(1)%transform = ident
    nodes(1)%param(1) = 1._c_double
    nodes(1)%mus = 10._c_double; nodes(1)%mua = 0._c_double; nodes(1)%hgg = 0._c_double; nodes(1)%n = 1._c_double
    nodes(2)%kind = SMCRT_SDF_BOX; nodes(2)%layer = 2; nodes(2)%transform = ident
    nodes(2)%param(1:3) = 1._c_double   ! half lengths of the 2x2x2 box
    nodes(2)%mus = 0._c_double; nodes(2)%mua = 0._c_double; nodes(2)%hgg = 0._c_double; nodes(2)%n = 1._c_double
    top = [0_c_int32_t, 1_c_int32_t]

    grid = smcrt_grid(nx=200, ny=200, nz=200, xmax=1._c_double, ymax=1._c_double, zmax=1._c_double)
    allocate(jmean(grid%nx, grid%ny, grid%nz))
    jmean = 0._c_float

    if (n_gpus > 0) then
        ierr = smcrt_multi_create(nodes, 2_c_int32_t, top, 2_c_int32_t, grid, dets, 0_c_int32_t, c_null_ptr, &
                                  n_gpus, multi)
    else
        ierr = smcrt_scene_create(nodes, 2_c_int32_t, top, 2_c_int32_t, grid, dets, 0_c_int32_t, 0_c_int32_t, scene)
    end if
    if (ierr /= SMCRT_OK) then
        print *, "scene upload failed: ", smcrt_error_message()
        error stop 1
    end if

    src%kind = SMCRT_SRC_POINT
    src%pos = 0._c_double
    cfg = smcrt_run_config(n_photons=nphotons, seed=123456789_c_int64_t, &
                           flags=ior(SMCRT_FLAG_PATHLENGTH, SMCRT_FLAG_TEST_KERNEL))
    nscatt = 0._c_double
    counters = 0
    io%jmean = c_loc(jmean)
    io%nscatt = c_loc(nscatt)
    io%counters = c_loc(counters)
    if (n_gpus > 0) then
        ierr = smcrt_multi_run(multi, src, cfg, io)
    else
        ierr = smcrt_run(scene, src, cfg, io)
    end if
    if (ierr /= SMCRT_OK) then
        print *, "run failed: ", smcrt_error_message()
        error stop 1
    end if
    ierr = smcrt_normalise_fluence(jmean, grid, nphotons)
    print '(a,f10.5)', "nscatt/photon = ", nscatt / real(nphotons, c_double)
    print '(a,i0)', "photons = ", counters(1)
    print '(a,es24.16)', "sum(jmean normalised) = ", sum(real(jmean, c_double))
    print '(a,es24.16)', "nscatt = ", nscatt
    do i = 1, SMCRT_NCOUNTERS
        print '(a,i0,a,i0)', "counter ", i - 1, " = ", counters(i)
    end do
    if (n_gpus > 0) then
        call smcrt_multi_destroy(multi)
    else
        call smcrt_scene_destroy(scene)
    end if
end program example_scat_test
