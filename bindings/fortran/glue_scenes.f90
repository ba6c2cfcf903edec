! glue_scenes.f90 — builds reference scenes with smcrt_glue the way setupGeometry.f90,
! parse_detectors.f90 and parse_source.f90 build them from res/<name>.toml, and writes each
! as the flat tables smcrt_scene_create receives. tests/test_fortran_binding.py compares them
! field by field with the C++ TOML front end (smcrt_job_scene) on the same files.
! usage: glue_scenes OUTDIR [VESSELDIR]  ->  OUTDIR/<name>.bin for scat_test, aptran,
! validation1, omg, test_dects, egg_test, and vessels (get_vessels on VESSELDIR's edges.dat,
! nodes.dat, radii.dat; res/vessels.toml's uniform source) when VESSELDIR is given
program glue_scenes
    use smcrt_mod
    use smcrt_glue
    implicit none
    character(len=512) :: outdir, vdir
    type(smcrt_sdf), allocatable :: a(:), kids(:)
    type(smcrt_detector), allocatable :: d(:)
    type(smcrt_source) :: src
    type(smcrt_optprop) :: zero
    real(c_double), parameter :: corner1(3) = [-1._c_double, -1._c_double, 1._c_double], &
        corner2(3) = [2._c_double, 0._c_double, 0._c_double], corner3(3) = [0._c_double, 2._c_double, 0._c_double]
    real(c_double) :: seg(6, 9)
    integer :: i, ierr

    call get_command_argument(1, outdir)
    vdir = ""
    if (command_argument_count() >= 2) call get_command_argument(2, vdir)
    zero = smcrt_mono(0._c_double, 0._c_double, 0._c_double, 1._c_double)

    ! res/scat_test.toml: setup_scat_test (setupGeometry.f90:409-435), tau = 10; point source
    allocate(a(2), d(0))
    a(1) = smcrt_sphere(1._c_double, smcrt_mono(10._c_double, 0._c_double, 0._c_double, 1._c_double), 1)
    a(2) = smcrt_box([2._c_double, 2._c_double, 2._c_double], zero, 2)
    ierr = smcrt_source_from("point", [0._c_double, 0._c_double, 0._c_double], [0._c_double, 0._c_double, 0._c_double], &
                             corner1, corner2, corner3, src)
    call emit("scat_test", a, d, src, ierr)
    deallocate(a, d)

    ! res/aptran.toml: setup_tran_and_jacques (:335-363); uniform source, vector direction
    allocate(a(3), d(0))
    a(2) = smcrt_box([2._c_double, 2._c_double, 2._c_double], smcrt_mono(0._c_double, 1.e-17_c_double, 0._c_double, &
                     1._c_double), 2)
    a(3) = smcrt_box([2.01_c_double, 2.01_c_double, 2.01_c_double], smcrt_mono(0._c_double, 10000000._c_double, &
                     0._c_double, 1._c_double), 3)
    a(1) = smcrt_sphere(0.5_c_double, smcrt_mono(0._c_double, 1.e-17_c_double, 0._c_double, 1.33_c_double), 1, &
                        transform=smcrt_invert(smcrt_translate([0._c_double, 0._c_double, 0._c_double])))
    ierr = smcrt_source_from("uniform", [0._c_double, 0._c_double, 0._c_double], [0._c_double, 0._c_double, -1._c_double], &
                             [-0.25_c_double, 0._c_double, 0.99999_c_double], [0.5_c_double, 0._c_double, 0._c_double], &
                             [0._c_double, 0._c_double, 0._c_double], src)
    call emit("aptran", a, d, src, ierr)
    deallocate(a, d)

    ! res/validation1.toml: setup_box (:73-147) and two circle detectors; pencil source along z
    allocate(a(2), d(2))
    a(1) = smcrt_box([100._c_double, 100._c_double, 0.02_c_double], smcrt_mono(90._c_double, 10._c_double, 0.75_c_double, &
                     1._c_double), 1, transform=smcrt_invert(smcrt_translate([0._c_double, 0._c_double, 0._c_double])))
    a(2) = smcrt_box([100._c_double, 100._c_double, 0.03_c_double], zero, 2)
    d(1) = smcrt_circle_dect([0._c_double, 0._c_double, -0.01_c_double], [0._c_double, 0._c_double, -1._c_double], 1, &
                             20._c_double, 100)
    d(2) = smcrt_circle_dect([0._c_double, 0._c_double, 0.01_c_double], [0._c_double, 0._c_double, 1._c_double], 1, &
                             20._c_double, 100)
    ierr = smcrt_source_from("pencil", [0._c_double, 0._c_double, -0.01_c_double], [0._c_double, 0._c_double, 1._c_double], &
                             corner1, corner2, corner3, src)
    call emit("validation1", a, d, src, ierr)
    deallocate(a, d)

    ! res/omg.toml: setup_omg_sdf (:466-549), a smooth-union model of a torus and nine
    ! cylinders, inside a box
    allocate(a(2), d(0), kids(10))
    seg = reshape([-.25_c_double, 0._c_double, -.25_c_double, -.25_c_double, 0._c_double, .25_c_double, &
                   -.25_c_double, 0._c_double, -.25_c_double, .25_c_double, 0._c_double, 0._c_double, &
                   .25_c_double, 0._c_double, 0._c_double, -.25_c_double, 0._c_double, .25_c_double, &
                   -.25_c_double, 0._c_double, .25_c_double, .25_c_double, 0._c_double, .25_c_double, &
                   -.25_c_double, 0._c_double, .5_c_double, .25_c_double, 0._c_double, .5_c_double, &
                   -.25_c_double, 0._c_double, .5_c_double, -.25_c_double, 0._c_double, .75_c_double, &
                   .25_c_double, 0._c_double, .5_c_double, .25_c_double, 0._c_double, .75_c_double, &
                   .25_c_double, 0._c_double, .75_c_double, 0._c_double, 0._c_double, .75_c_double, &
                   0._c_double, 0._c_double, .625_c_double, 0._c_double, 0._c_double, .75_c_double], [6, 9])
    kids(1) = smcrt_torus(0.2_c_double, 0.05_c_double, smcrt_mono(10._c_double, 0.16_c_double, 0._c_double, 2.65_c_double), &
                          1, transform=smcrt_invert(smcrt_translate([0._c_double, 0._c_double, -0.7_c_double])))
    do i = 1, 9
        if (i == 1) then
            kids(i + 1) = smcrt_cylinder(seg(1:3, i), seg(4:6, i), 0.05_c_double, &
                                         smcrt_mono(10._c_double, 0.16_c_double, 0._c_double, 2.65_c_double), 1, &
                                         transform=smcrt_invert(smcrt_rotate_y(90._c_double)))
        else
            kids(i + 1) = smcrt_cylinder(seg(1:3, i), seg(4:6, i), 0.05_c_double, &
                                         smcrt_mono(10._c_double, 0.16_c_double, 0._c_double, 2.65_c_double), 1)
        end if
    end do
    a(1) = smcrt_model(kids, SMCRT_OP_SMOOTH_UNION, 0.09_c_double)
    a(2) = smcrt_box([2._c_double, 2._c_double, 2._c_double], zero, 2)
    ierr = smcrt_source_from("uniform", [0._c_double, 0._c_double, 0._c_double], [0._c_double, -1._c_double, 0._c_double], &
                             [-1._c_double, 0.99999_c_double, -1._c_double], [2._c_double, 0._c_double, 0._c_double], &
                             [0._c_double, 0._c_double, 2._c_double], src)
    call emit("omg", a, d, src, ierr)
    deallocate(a, d, kids)

    ! res/test_dects.toml: scat_test geometry with a circle, an annulus and a camera
    allocate(a(2), d(3))
    a(1) = smcrt_sphere(1._c_double, smcrt_mono(10._c_double, 0._c_double, 0._c_double, 1._c_double), 1)
    a(2) = smcrt_box([2._c_double, 2._c_double, 2._c_double], zero, 2)
    d(1) = smcrt_circle_dect([-1._c_double, 0._c_double, 0._c_double], [-1._c_double, 0._c_double, 0._c_double], 4, &
                             0.5_c_double, 10)
    d(2) = smcrt_annulus_dect([-1._c_double, 0._c_double, 0._c_double], [-1._c_double, 0._c_double, 0._c_double], 3, &
                              0.5_c_double, 1._c_double, 10)
    d(3) = smcrt_camera([-1._c_double, -1._c_double, -1._c_double], [0._c_double, 2._c_double, 0._c_double], &
                        [0._c_double, 0._c_double, 2._c_double], 2, 10, 5000._c_double)
    ierr = smcrt_source_from("point", [0._c_double, 0._c_double, 0._c_double], [0._c_double, 0._c_double, 0._c_double], &
                             corner1, corner2, corner3, src)
    call emit("test_dects", a, d, src, ierr)
    deallocate(a, d)

    ! res/egg_test.toml: setup_egg (:149-248), numOptProp = 3 with the parser's defaults (mus 1,
    ! mua 0, hgg 0, n 1); the albumen and shell are Moss eggs revolved about y
    allocate(a(4), d(0))
    a(1) = smcrt_sphere(1._c_double, smcrt_mono(1._c_double, 0._c_double, 0._c_double, 1._c_double), 1, &
                        transform=smcrt_invert(smcrt_translate([0._c_double, 0._c_double, 0._c_double])))
    a(2) = smcrt_revolution(smcrt_egg(2._c_double * (1 - 0.02_c_double), 1.5_c_double * (1 - 0.02_c_double), &
                                      1.4_c_double * (1 - 0.02_c_double), &
                                      smcrt_mono(1._c_double, 0._c_double, 0._c_double, 1._c_double), 3), &
                            0._c_double, center=[0._c_double, 0._c_double, 0._c_double])
    a(3) = smcrt_revolution(smcrt_egg(2._c_double, 1.5_c_double, 1.4_c_double, &
                                      smcrt_mono(1._c_double, 0._c_double, 0._c_double, 1._c_double), 2), &
                            0._c_double, center=[0._c_double, 0._c_double, 0._c_double])
    a(4) = smcrt_box([5._c_double, 5._c_double, 5._c_double], zero, 4)
    ierr = smcrt_source_from("point", [0._c_double, 0._c_double, 0._c_double], [0._c_double, 0._c_double, 0._c_double], &
                             corner1, corner2, corner3, src)
    call emit("egg_test", a, d, src, ierr)
    deallocate(a, d)

    ! res/vessels.toml: get_vessels (:552-652) on the data set in VESSELDIR; uniform source on
    ! the top face with the vector direction applied (DESIGN.md §2)
    if (len_trim(vdir) > 0) then
        allocate(d(0))
        call smcrt_get_vessels(trim(vdir), a, ierr)
        if (ierr /= SMCRT_OK) error stop "smcrt_get_vessels failed"
        ierr = smcrt_source_from("uniform", [0._c_double, 0._c_double, 0._c_double], [0._c_double, 0._c_double, &
                                 -1._c_double], [-0.16_c_double, -0.09_c_double, 0.129999_c_double], &
                                 [0.32_c_double, 0._c_double, 0._c_double], [0._c_double, 0.18_c_double, 0._c_double], src)
        call emit("vessels", a, d, src, ierr)
        deallocate(a, d)
    end if

contains

    subroutine emit(name, array, dets, s, status)
        character(len=*), intent(in) :: name
        type(smcrt_sdf), intent(in) :: array(:)
        type(smcrt_detector), intent(in) :: dets(:)
        type(smcrt_source), intent(in) :: s
        integer, intent(in) :: status
        type(smcrt_sdf_node), allocatable :: nodes(:)
        integer(c_int32_t), allocatable :: top(:)
        integer :: u
        if (status /= SMCRT_OK) error stop "smcrt_source_from failed"
        call smcrt_flatten(array, nodes, top)
        open(newunit=u, file=trim(outdir)//"/"//name//".bin", access="stream", form="unformatted", status="replace")
        write(u) int(size(nodes), c_int32_t), int(size(top), c_int32_t), int(size(dets), c_int32_t)
        write(u) nodes, top
        if (size(dets) > 0) write(u) dets
        ! the source's value fields (its spectrum pointer stays null: the constant 500 nm)
        write(u) s%kind, s%beam, s%pos, s%dir, s%p1, s%p2, s%p3, s%radius, s%beam_size, s%focal_length, s%rlo, &
                 s%rhi, s%sigma, s%rotation
        close(u)
    end subroutine emit

end program glue_scenes
