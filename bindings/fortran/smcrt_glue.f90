! smcrt_glue.f90 — the reference-side conversion code of INTEGRATION.md §2.2-2.4 as a module.
!
! run_MCRT's replacement body (INTEGRATION.md §2.1) has to turn signedMCRT's own objects into
! the flat tables of include/smcrt.h: the SDF tree array(:) into smcrt_sdf_node + top,
! dects(:) into smcrt_detector, and the [source] dictionary into smcrt_source. This module is
! that conversion. Its constructors take the arguments of the reference's constructors
! (sdfs.f90:158-492, sdf_base.f90:101-144, detectors.f90:103-445, photon.f90 via
! parse_source.f90) and keep what the engine needs, so a maintainer's adapter is one call per
! reference object:
!
!     select type (v => array(i)%value)
!     type is (sphere); g(i) = smcrt_sphere(v%radius, op(v), v%layer, v%transform)
!     ...
!     call smcrt_flatten(g, nodes, top)
!
! tests/test_fortran_binding.py builds res/scat_test, aptran, validation1, omg, test_dects and
! egg_test (revolution modifiers) with it
! (bindings/fortran/glue_scenes.f90) and checks every field against the C++ TOML front end.
module smcrt_glue
    use iso_c_binding
    use smcrt_mod
    implicit none
    private

    public :: smcrt_optprop, smcrt_mono, smcrt_spectral_props, smcrt_sdf
    public :: smcrt_sphere, smcrt_box, smcrt_torus, smcrt_cylinder, smcrt_triprism, smcrt_segment, &
              smcrt_capsule, smcrt_cone, smcrt_egg, smcrt_plane, smcrt_model
    public :: smcrt_revolution, smcrt_extrude, smcrt_onion, smcrt_twist, smcrt_bend, smcrt_elongate, &
              smcrt_displacement_sine
    public :: smcrt_count_nodes, smcrt_flatten, smcrt_get_vessels
    public :: smcrt_circle_dect, smcrt_annulus_dect, smcrt_camera, smcrt_fibre_dect
    public :: smcrt_source_from
    public :: smcrt_identity, smcrt_translate, smcrt_rotate_y, smcrt_invert

    !> init_mono's inputs (opticalProperties.f90:107-125); the engine derives kappa and the
    !> albedo exactly as init_mono does.
    !> flags: SMCRT_NODE_ALBEDO_UNGUARDED for properties from updateSpectral.
    type :: smcrt_optprop
        real(c_double) :: mus = 0._c_double, mua = 0._c_double, hgg = 0._c_double, n = 1._c_double
        integer(c_int32_t) :: flags = 0
    end type smcrt_optprop

    !> One element of the reference's array(:) (sdf_base.f90:27-52): a primitive, or a model
    !> whose children are SDFs again.
    type :: smcrt_sdf
        type(smcrt_sdf_node) :: node
        type(smcrt_sdf), allocatable :: children(:)
    end type smcrt_sdf

contains

    function smcrt_mono(mus, mua, hgg, n) result(o)
        real(c_double), intent(in) :: mus, mua, hgg, n
        type(smcrt_optprop) :: o
        o = smcrt_optprop(mus=mus, mua=mua, hgg=hgg, n=n)
    end function smcrt_mono

    !> spectral(mus, mua, hgg, n, flux) (opticalProperties.f90:127-156) and updateSpectral
    !> (:171-201): each argument an array(n, 2) as the reference takes them. mode is one of
    !> SMCRT_SPECTRAL_* (default SMCRT_SPECTRAL_INIT); draw is the position in the seed's host
    !> stream (include/smcrt.h), advanced by the draws taken; wavelength returns the sample.
    function smcrt_spectral_props(mus, mua, hgg, n, flux, seed, draw, mode, wavelength) result(o)
        real(c_double), target, intent(in) :: mus(:, :), mua(:, :), hgg(:, :), n(:, :), flux(:, :)
        integer(c_int64_t), intent(in) :: seed
        integer(c_int64_t), intent(inout) :: draw
        integer(c_int32_t), optional, intent(in) :: mode
        real(c_double), optional, intent(out) :: wavelength
        type(smcrt_optprop) :: o
        type(smcrt_spectral) :: sp
        type(smcrt_optprops) :: p
        real(c_double), allocatable, target :: a(:, :), b(:, :), c(:, :), d(:, :), e(:, :)
        integer(c_int32_t) :: m
        m = SMCRT_SPECTRAL_INIT
        if (present(mode)) m = mode
        a = mus; b = mua; c = hgg; d = n; e = flux   ! contiguous copies
        sp%n_mus = size(a, 1); sp%n_mua = size(b, 1); sp%n_hgg = size(c, 1); sp%n_n = size(d, 1)
        sp%n_flux = size(e, 1)
        sp%mus = c_loc(a); sp%mua = c_loc(b); sp%hgg = c_loc(c); sp%n = c_loc(d); sp%flux = c_loc(e)
        if (smcrt_spectral_sample(sp, m, seed, draw, p) /= 0) error stop "smcrt_spectral_sample failed"
        o = smcrt_optprop(mus=p%mus, mua=p%mua, hgg=p%hgg, n=p%n, flags=p%node_flags)
        if (present(wavelength)) wavelength = p%wavelength
    end function smcrt_spectral_props

    ! ------------------------------------------------------------ transforms ---------------
    function smcrt_identity() result(t)
        real(c_double) :: t(4, 4)
        integer :: i
        t = 0._c_double
        do i = 1, 4
            t(i, i) = 1._c_double
        end do
    end function smcrt_identity

    function smcrt_translate(o) result(t)  ! sdfHelpers.f90:169-182: row 4 holds the offset
        real(c_double), intent(in) :: o(3)
        real(c_double) :: t(4, 4)
        t(:, 1) = [1._c_double, 0._c_double, 0._c_double, o(1)]
        t(:, 2) = [0._c_double, 1._c_double, 0._c_double, o(2)]
        t(:, 3) = [0._c_double, 0._c_double, 1._c_double, o(3)]
        t(:, 4) = [0._c_double, 0._c_double, 0._c_double, 1._c_double]
    end function smcrt_translate

    function smcrt_rotate_y(angle) result(t)  ! sdfHelpers.f90:33-50 (angle in degrees)
        real(c_double), intent(in) :: angle
        real(c_double) :: t(4, 4), r, c, s
        r = angle * 3.14159265358979323846264338327950288_c_double / 180._c_double
        c = cos(r)
        s = sin(r)
        t(:, 1) = [c, 0._c_double, s, 0._c_double]
        t(:, 2) = [0._c_double, 1._c_double, 0._c_double, 0._c_double]
        t(:, 3) = [-s, 0._c_double, c, 0._c_double]
        t(:, 4) = [0._c_double, 0._c_double, 0._c_double, 1._c_double]
    end function smcrt_rotate_y

    function smcrt_invert(a) result(b)  ! mat_class.f90:154-207, term for term
        real(c_double), intent(in) :: a(4, 4)
        real(c_double) :: b(4, 4), detinv
        detinv = 1._c_double / (a(1,1)*(a(2,2)*(a(3,3)*a(4,4)-a(3,4)*a(4,3))+a(2,3)*(a(3,4)*a(4,2)-a(3,2)*a(4,4)) &
                 + a(2,4)*(a(3,2)*a(4,3)-a(3,3)*a(4,2))) &
                 - a(1,2)*(a(2,1)*(a(3,3)*a(4,4)-a(3,4)*a(4,3))+a(2,3)*(a(3,4)*a(4,1)-a(3,1)*a(4,4)) &
                 + a(2,4)*(a(3,1)*a(4,3)-a(3,3)*a(4,1))) &
                 + a(1,3)*(a(2,1)*(a(3,2)*a(4,4)-a(3,4)*a(4,2))+a(2,2)*(a(3,4)*a(4,1)-a(3,1)*a(4,4)) &
                 + a(2,4)*(a(3,1)*a(4,2)-a(3,2)*a(4,1))) &
                 - a(1,4)*(a(2,1)*(a(3,2)*a(4,3)-a(3,3)*a(4,2))+a(2,2)*(a(3,3)*a(4,1)-a(3,1)*a(4,3)) &
                 + a(2,3)*(a(3,1)*a(4,2)-a(3,2)*a(4,1))))
        b(1,1) = detinv*(a(2,2)*(a(3,3)*a(4,4)-a(3,4)*a(4,3))+a(2,3)*(a(3,4)*a(4,2)-a(3,2)*a(4,4)) &
                 + a(2,4)*(a(3,2)*a(4,3)-a(3,3)*a(4,2)))
        b(2,1) = detinv*(a(2,1)*(a(3,4)*a(4,3)-a(3,3)*a(4,4))+a(2,3)*(a(3,1)*a(4,4)-a(3,4)*a(4,1)) &
                 + a(2,4)*(a(3,3)*a(4,1)-a(3,1)*a(4,3)))
        b(3,1) = detinv*(a(2,1)*(a(3,2)*a(4,4)-a(3,4)*a(4,2))+a(2,2)*(a(3,4)*a(4,1)-a(3,1)*a(4,4)) &
                 + a(2,4)*(a(3,1)*a(4,2)-a(3,2)*a(4,1)))
        b(4,1) = detinv*(a(2,1)*(a(3,3)*a(4,2)-a(3,2)*a(4,3))+a(2,2)*(a(3,1)*a(4,3)-a(3,3)*a(4,1)) &
                 + a(2,3)*(a(3,2)*a(4,1)-a(3,1)*a(4,2)))
        b(1,2) = detinv*(a(1,2)*(a(3,4)*a(4,3)-a(3,3)*a(4,4))+a(1,3)*(a(3,2)*a(4,4)-a(3,4)*a(4,2)) &
                 + a(1,4)*(a(3,3)*a(4,2)-a(3,2)*a(4,3)))
        b(2,2) = detinv*(a(1,1)*(a(3,3)*a(4,4)-a(3,4)*a(4,3))+a(1,3)*(a(3,4)*a(4,1)-a(3,1)*a(4,4)) &
                 + a(1,4)*(a(3,1)*a(4,3)-a(3,3)*a(4,1)))
        b(3,2) = detinv*(a(1,1)*(a(3,4)*a(4,2)-a(3,2)*a(4,4))+a(1,2)*(a(3,1)*a(4,4)-a(3,4)*a(4,1)) &
                 + a(1,4)*(a(3,2)*a(4,1)-a(3,1)*a(4,2)))
        b(4,2) = detinv*(a(1,1)*(a(3,2)*a(4,3)-a(3,3)*a(4,2))+a(1,2)*(a(3,3)*a(4,1)-a(3,1)*a(4,3)) &
                 + a(1,3)*(a(3,1)*a(4,2)-a(3,2)*a(4,1)))
        b(1,3) = detinv*(a(1,2)*(a(2,3)*a(4,4)-a(2,4)*a(4,3))+a(1,3)*(a(2,4)*a(4,2)-a(2,2)*a(4,4)) &
                 + a(1,4)*(a(2,2)*a(4,3)-a(2,3)*a(4,2)))
        b(2,3) = detinv*(a(1,1)*(a(2,4)*a(4,3)-a(2,3)*a(4,4))+a(1,3)*(a(2,1)*a(4,4)-a(2,4)*a(4,1)) &
                 + a(1,4)*(a(2,3)*a(4,1)-a(2,1)*a(4,3)))
        b(3,3) = detinv*(a(1,1)*(a(2,2)*a(4,4)-a(2,4)*a(4,2))+a(1,2)*(a(2,4)*a(4,1)-a(2,1)*a(4,4)) &
                 + a(1,4)*(a(2,1)*a(4,2)-a(2,2)*a(4,1)))
        b(4,3) = detinv*(a(1,1)*(a(2,3)*a(4,2)-a(2,2)*a(4,3))+a(1,2)*(a(2,1)*a(4,3)-a(2,3)*a(4,1)) &
                 + a(1,3)*(a(2,2)*a(4,1)-a(2,1)*a(4,2)))
        b(1,4) = detinv*(a(1,2)*(a(2,4)*a(3,3)-a(2,3)*a(3,4))+a(1,3)*(a(2,2)*a(3,4)-a(2,4)*a(3,2)) &
                 + a(1,4)*(a(2,3)*a(3,2)-a(2,2)*a(3,3)))
        b(2,4) = detinv*(a(1,1)*(a(2,3)*a(3,4)-a(2,4)*a(3,3))+a(1,3)*(a(2,4)*a(3,1)-a(2,1)*a(3,4)) &
                 + a(1,4)*(a(2,1)*a(3,3)-a(2,3)*a(3,1)))
        b(3,4) = detinv*(a(1,1)*(a(2,4)*a(3,2)-a(2,2)*a(3,4))+a(1,2)*(a(2,1)*a(3,4)-a(2,4)*a(3,1)) &
                 + a(1,4)*(a(2,2)*a(3,1)-a(2,1)*a(3,2)))
        b(4,4) = detinv*(a(1,1)*(a(2,2)*a(3,3)-a(2,3)*a(3,2))+a(1,2)*(a(2,3)*a(3,1)-a(2,1)*a(3,3)) &
                 + a(1,3)*(a(2,1)*a(3,2)-a(2,2)*a(3,1)))
    end function smcrt_invert

    ! ------------------------------------------------------------ SDF constructors ---------
    ! Each takes the arguments of the reference constructor of the same name (sdfs.f90), with
    ! the optical properties as smcrt_optprop; a missing transform is the identity.
    function prim(kind, param, op, layer, transform) result(s)
        integer(c_int32_t), intent(in) :: kind
        real(c_double), intent(in) :: param(:)
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        real(c_double) :: t(4, 4)
        if (present(transform)) then
            t = transform
        else
            t = smcrt_identity()
        end if
        s%node%kind = kind
        s%node%layer = int(layer, c_int32_t)
        s%node%transform = reshape(t, [16])   ! column-major, as sdf_base.f90:21
        s%node%param(1:size(param)) = param
        s%node%mus = op%mus; s%node%mua = op%mua; s%node%hgg = op%hgg; s%node%n = op%n
        s%node%flags = op%flags
    end function prim

    function smcrt_sphere(radius, op, layer, transform) result(s)  ! sphere_init :463-492
        real(c_double), intent(in) :: radius
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_SPHERE, [radius], op, layer, transform)
    end function smcrt_sphere

    function smcrt_box(lengths, op, layer, transform) result(s)  ! box_init :433-461
        real(c_double), intent(in) :: lengths(3)
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_BOX, .5_c_double * lengths, op, layer, transform)  ! half lengths, :455
    end function smcrt_box

    function smcrt_torus(oradius, iradius, op, layer, transform) result(s)  ! torus_init :401-431
        real(c_double), intent(in) :: oradius, iradius
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_TORUS, [oradius, iradius], op, layer, transform)
    end function smcrt_torus

    function smcrt_cylinder(a, b, radius, op, layer, transform) result(s)  ! cylinder_init :365-399
        real(c_double), intent(in) :: a(3), b(3), radius
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_CYLINDER, [a, b, radius], op, layer, transform)
    end function smcrt_cylinder

    function smcrt_triprism(h1, h2, op, layer, transform) result(s)  ! triprism_init :295-325
        real(c_double), intent(in) :: h1, h2
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_TRIPRISM, [h1, h2], op, layer, transform)
    end function smcrt_triprism

    function smcrt_segment(a, b, op, layer, transform) result(s)  ! segment_init :158-191
        real(c_double), intent(in) :: a(3), b(3)
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_SEGMENT, [a, b], op, layer, transform)
    end function smcrt_segment

    function smcrt_capsule(a, b, r, op, layer, transform) result(s)  ! capsule_init :259-293
        real(c_double), intent(in) :: a(3), b(3), r
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_CAPSULE, [a, b, r], op, layer, transform)
    end function smcrt_capsule

    function smcrt_cone(a, b, ra, rb, op, layer, transform) result(s)  ! cone_init :327-363
        real(c_double), intent(in) :: a(3), b(3), ra, rb
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_CONE, [a, b, ra, rb], op, layer, transform)
    end function smcrt_cone

    function smcrt_egg(r1, r2, h, op, layer, transform) result(s)  ! egg_init :193-227
        real(c_double), intent(in) :: r1, r2, h
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_EGG, [r1, r2, h], op, layer, transform)
    end function smcrt_egg

    function smcrt_plane(a, op, layer, transform) result(s)  ! plane_init :229-257
        real(c_double), intent(in) :: a(3)
        type(smcrt_optprop), intent(in) :: op
        integer, intent(in) :: layer
        real(c_double), optional, intent(in) :: transform(4, 4)
        type(smcrt_sdf) :: s
        s = prim(SMCRT_SDF_PLANE, a, op, layer, transform)
    end function smcrt_plane

    !> model_init (sdf_base.f90:101-144): a CSG fold over `array`. `op` is the engine's code
    !> for the model's procedure pointer (SMCRT_OP_UNION, _SMOOTH_UNION, _SUBTRACTION,
    !> _INTERSECTION: the adapter maps associated(m%func, union) etc.). The model has no layer
    !> or optics of its own: it reports those of array(1), as the reference's getters do.
    function smcrt_model(array, op, k) result(s)
        type(smcrt_sdf), intent(in) :: array(:)
        integer(c_int32_t), intent(in) :: op
        real(c_double), optional, intent(in) :: k
        type(smcrt_sdf) :: s
        if (size(array) < 1) error stop "smcrt_model: a model needs at least one SDF"
        ! (a child may be a model again, as in the reference; smcrt_scene_create accepts 32
        ! levels of models)
        s%node%kind = SMCRT_SDF_MODEL
        s%node%op = op
        s%node%transform = reshape(smcrt_identity(), [16])
        if (present(k)) s%node%k = k
        s%node%layer = array(1)%node%layer
        s%node%mus = array(1)%node%mus; s%node%mua = array(1)%node%mua
        s%node%hgg = array(1)%node%hgg; s%node%n = array(1)%node%n
        s%node%flags = array(1)%node%flags
        s%node%n_children = int(size(array), c_int32_t)
        allocate(s%children, source=array)
    end function smcrt_model

    ! ------------------------------------------------------------ modifiers ----------------
    ! sdfModifiers.f90's *_init: the modifier wraps `prim` (a primitive, model or modifier), takes
    ! its layer and optics, and keeps the identity transform it never applies.
    function modifier(kind, prim_sdf, param) result(s)
        integer(c_int32_t), intent(in) :: kind
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: param(:)
        type(smcrt_sdf) :: s
        s%node%kind = kind
        s%node%transform = reshape(smcrt_identity(), [16])
        s%node%param(1:size(param)) = param
        s%node%layer = prim_sdf%node%layer
        s%node%mus = prim_sdf%node%mus; s%node%mua = prim_sdf%node%mua
        s%node%hgg = prim_sdf%node%hgg; s%node%n = prim_sdf%node%n
        s%node%flags = prim_sdf%node%flags
        s%node%n_children = 1
        allocate(s%children(1))
        s%children(1) = prim_sdf
    end function modifier

    function smcrt_revolution(prim_sdf, o, center) result(s)  ! revolution_init :238-266
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: o
        real(c_double), optional, intent(in) :: center(3)
        type(smcrt_sdf) :: s
        real(c_double) :: c(3)
        c = 0._c_double
        if (present(center)) c = center
        s = modifier(SMCRT_SDF_REVOLUTION, prim_sdf, [o, c])
    end function smcrt_revolution

    function smcrt_extrude(prim_sdf, h) result(s)  ! extrude_init :143-159
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: h
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_EXTRUDE, prim_sdf, [h])
    end function smcrt_extrude

    function smcrt_onion(prim_sdf, thickness) result(s)  ! onion_init :268-284
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: thickness
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_ONION, prim_sdf, [thickness])
    end function smcrt_onion

    function smcrt_twist(prim_sdf, k) result(s)  ! twist_init :126-141 (k is a default real there)
        type(smcrt_sdf), intent(in) :: prim_sdf
        real, intent(in) :: k
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_TWIST, prim_sdf, [real(k, c_double)])
    end function smcrt_twist

    function smcrt_bend(prim_sdf, k) result(s)  ! bend_init :196-212
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: k
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_BEND, prim_sdf, [k])
    end function smcrt_bend

    function smcrt_elongate(prim_sdf, size3) result(s)  ! elongate_init :161-176
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: size3(3)
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_ELONGATE, prim_sdf, size3)
    end function smcrt_elongate

    !> displacement_init (:178-194) with the engine's built-in f(p) = a sin(fx x) sin(fy y) sin(fz z)
    !> (the reference takes any procedure(primitive); device code cannot call a host pointer)
    function smcrt_displacement_sine(prim_sdf, amplitude, freq) result(s)
        type(smcrt_sdf), intent(in) :: prim_sdf
        real(c_double), intent(in) :: amplitude, freq(3)
        type(smcrt_sdf) :: s
        s = modifier(SMCRT_SDF_DISPLACEMENT, prim_sdf, [real(SMCRT_DISP_SINE, c_double), amplitude, freq])
    end function smcrt_displacement_sine

    ! ------------------------------------------------------------ scene builders ------------
    !> get_vessels (setupGeometry.f90:552-652) for a host that builds the vessel net itself:
    !> reads dir/edges.dat, dir/nodes.dat and dir/radii.dat with list-directed reads, counts
    !> as the reference does (successful reads until the first failure, :585-602), reads the
    !> nodes with the edge count as the loop bound (:615), rescales (:629-639, res = 0.001) and
    !> returns one capsule per edge plus the dermis box. Rows of nodes that the :615 bound
    !> leaves unread are 0 here (the reference leaves them undefined), as in the C++ front end.
    !> status: SMCRT_OK, or SMCRT_ERR_INVALID_ARG for a missing file, no edge, an edge naming a
    !> node outside 1..N, or an axis whose max|coordinate| is 0.
    subroutine smcrt_get_vessels(dir, array, status)
        character(len=*), intent(in) :: dir
        type(smcrt_sdf), allocatable, intent(out) :: array(:)
        integer, intent(out) :: status
        real(c_double), allocatable :: xyz(:, :), rad(:)
        integer, allocatable :: ends(:, :)
        integer :: u, ios, ne, nn, i, j1, j2
        real(c_double) :: v3(3), mx(3), scale
        integer :: e2(2)
        type(smcrt_optprop) :: vessel, dermis

        status = SMCRT_ERR_INVALID_ARG
        vessel = smcrt_mono(94._c_double, 231._c_double, 0.9_c_double, 1.37_c_double)
        dermis = smcrt_mono(357._c_double, 0.458_c_double, 0.9_c_double, 1.37_c_double)
        scale = 0.001_c_double

        open(newunit=u, file=dir//"/edges.dat", status="old", action="read", iostat=ios)
        if (ios /= 0) return
        ne = 0
        do
            read(u, *, iostat=ios) e2
            if (ios /= 0) exit
            ne = ne + 1
        end do
        close(u)
        open(newunit=u, file=dir//"/nodes.dat", status="old", action="read", iostat=ios)
        if (ios /= 0) return
        nn = 0
        do
            read(u, *, iostat=ios) v3
            if (ios /= 0) exit
            nn = nn + 1
        end do
        close(u)
        if (ne == 0) return
        allocate(ends(ne, 2), xyz(nn, 3), rad(nn))
        ends = 0
        xyz = 0._c_double
        rad = 0._c_double

        open(newunit=u, file=dir//"/edges.dat", status="old", action="read")
        do i = 1, ne
            read(u, *, iostat=ios) ends(i, :)
            if (ios /= 0) exit
        end do
        close(u)
        open(newunit=u, file=dir//"/nodes.dat", status="old", action="read")
        do i = 1, min(ne, nn)        ! the reference's bound is the edge count (:615)
            read(u, *, iostat=ios) xyz(i, :)
            if (ios /= 0) exit
        end do
        close(u)
        open(newunit=u, file=dir//"/radii.dat", status="old", action="read", iostat=ios)
        if (ios /= 0) return
        do i = 1, nn
            read(u, *, iostat=ios) rad(i)
            if (ios /= 0) exit
        end do
        close(u)

        do i = 1, 3
            mx(i) = maxval(abs(xyz(:, i)))
            if (.not. (mx(i) > 0._c_double)) return
            xyz(:, i) = xyz(:, i) / mx(i) - 0.5_c_double
            xyz(:, i) = xyz(:, i) * mx(i) * scale
        end do

        allocate(array(ne + 1))
        do i = 1, ne
            j1 = ends(i, 1)
            j2 = ends(i, 2)
            if (j1 < 1 .or. j1 > nn .or. j2 < 1 .or. j2 > nn) then
                deallocate(array)
                return
            end if
            array(i) = smcrt_capsule(xyz(j1, :), xyz(j2, :), rad(j1) * scale, vessel, 1)
        end do
        array(ne + 1) = smcrt_box([.32_c_double, .18_c_double, .26_c_double], dermis, 2)
        status = SMCRT_OK
    end subroutine smcrt_get_vessels

    ! ------------------------------------------------------------ flattening ---------------
    recursive integer function smcrt_count_nodes(array) result(n)
        type(smcrt_sdf), intent(in) :: array(:)
        integer :: i
        n = size(array)
        do i = 1, size(array)
            if (allocated(array(i)%children)) n = n + smcrt_count_nodes(array(i)%children)
        end do
    end function smcrt_count_nodes

    !> The SDF array as smcrt_scene_create wants it: the top-level SDFs first, in array order
    !> (top(i) = i-1), then each model's children in a contiguous run after them
    !> (first_child, 0-based), a nested model's children after its own run. For models of
    !> primitives this is the order the C++ front end and rsmcrt_amd.scene use.
    subroutine smcrt_flatten(array, nodes, top)
        type(smcrt_sdf), intent(in) :: array(:)
        type(smcrt_sdf_node), allocatable, intent(out) :: nodes(:)
        integer(c_int32_t), allocatable, intent(out) :: top(:)
        integer :: i, k
        allocate(nodes(smcrt_count_nodes(array)), top(size(array)))
        do i = 1, size(array)
            top(i) = int(i - 1, c_int32_t)
        end do
        k = size(array)  ! next free slot, 0-based
        call place(array, 0)
    contains
        recursive subroutine place(a, base)
            type(smcrt_sdf), intent(in) :: a(:)
            integer, intent(in) :: base  ! 0-based slot of a(1)
            integer :: j, first
            do j = 1, size(a)
                nodes(base + j) = a(j)%node
            end do
            do j = 1, size(a)
                if (allocated(a(j)%children)) then  ! a model or a modifier
                    first = k
                    nodes(base + j)%first_child = int(first, c_int32_t)
                    nodes(base + j)%n_children = int(size(a(j)%children), c_int32_t)
                    k = k + size(a(j)%children)
                    call place(a(j)%children, first)
                end if
            end do
        end subroutine place
    end subroutine smcrt_flatten

    ! ------------------------------------------------------------ detectors ----------------
    ! The reference's detector constructors (detectors.f90). nbins is the constructor's
    ! argument; the data arrays hold nbins + 1 bins (:116). The direction is taken as given:
    ! parse_detectors.f90 normalises circle and fibre directions before the call (:159, :249).
    function smcrt_circle_dect(pos, dir, layer, radius, nbins) result(d)  ! init_circle_dect :103-145
        real(c_double), intent(in) :: pos(3), dir(3), radius
        integer, intent(in) :: layer, nbins
        type(smcrt_detector) :: d
        d%kind = SMCRT_DET_CIRCLE
        d%pos = pos; d%dir = dir; d%layer = int(layer, c_int32_t)
        d%radius = radius
        d%nbins = int(nbins + 1, c_int32_t)
        if (nbins == 0) then
            d%bin_wid = 1._c_double
        else
            d%bin_wid = radius / real(nbins, c_double)
        end if
    end function smcrt_circle_dect

    function smcrt_annulus_dect(pos, dir, layer, r1, r2, nbins) result(d)  ! init_annulus_dect :166-200
        real(c_double), intent(in) :: pos(3), dir(3), r1, r2
        integer, intent(in) :: layer, nbins
        type(smcrt_detector) :: d
        d%kind = SMCRT_DET_ANNULUS
        d%pos = pos; d%dir = dir; d%layer = int(layer, c_int32_t)
        d%r1 = r1; d%r2 = r2
        d%nbins = int(nbins + 1, c_int32_t)
        if (nbins == 0) then
            d%bin_wid = 1._c_double
        else
            d%bin_wid = (r2 - r1) / real(nbins, c_double)
        end if
    end function smcrt_annulus_dect

    function smcrt_camera(p1, p2, p3, layer, nbins, maxval) result(d)  ! init_camera :395-445
        real(c_double), intent(in) :: p1(3), p2(3), p3(3), maxval
        integer, intent(in) :: layer, nbins
        type(smcrt_detector) :: d
        real(c_double) :: n(3), e1(3), e2(3), ln
        e1 = p2 - p1
        e2 = p3 - p1
        n = [e2(2)*e1(3) - e2(3)*e1(2), -e2(1)*e1(3) + e2(3)*e1(1), e2(1)*e1(2) - e2(2)*e1(1)]  ! e2 .cross. e1
        ln = sqrt(n(1)*n(1) + n(2)*n(2) + n(3)*n(3))
        d%kind = SMCRT_DET_CAMERA
        d%pos = p1; d%e1 = e1; d%e2 = e2; d%dir = n / ln
        d%width = sqrt(e1(1)*e1(1) + e1(2)*e1(2) + e1(3)*e1(3))
        d%height = sqrt(e2(1)*e2(1) + e2(2)*e2(2) + e2(3)*e2(3))
        d%layer = int(layer, c_int32_t)
        d%nbins = int(nbins + 1, c_int32_t)
        if (nbins == 0) then
            d%bin_wid = 1._c_double
            d%bin_wid_y = 1._c_double
        else
            d%bin_wid = maxval / real(nbins + 1, c_double)
            d%bin_wid_y = maxval / real(nbins + 1, c_double)
        end if
    end function smcrt_camera

    function smcrt_fibre_dect(pos, dir, layer, nbins, focalLength1, focalLength2, f1Aperture, f2Aperture, &
                              frontOffset, backOffset, frontToPinSep, pinToBackSep, pinAperture, acceptAngle, &
                              coreDiameter) result(d)  ! init_fibre_dect :246-329
        real(c_double), intent(in) :: pos(3), dir(3)
        integer, intent(in) :: layer, nbins
        real(c_double), intent(in) :: focalLength1, focalLength2, f1Aperture, f2Aperture, frontOffset, backOffset, &
                                      frontToPinSep, pinToBackSep, pinAperture, acceptAngle, coreDiameter
        type(smcrt_detector) :: d
        d%kind = SMCRT_DET_FIBRE
        d%pos = pos; d%dir = dir; d%layer = int(layer, c_int32_t)
        d%fibre = [focalLength1, focalLength2, f1Aperture, f2Aperture, frontOffset, backOffset, frontToPinSep, &
                   pinToBackSep, pinAperture, acceptAngle, coreDiameter]
        d%nbins = int(nbins + 1, c_int32_t)
        if (nbins == 0) then
            d%bin_wid = 1._c_double
        else
            d%bin_wid = coreDiameter / 2._c_double / real(nbins, c_double)
        end if
    end function smcrt_fibre_dect

    ! ------------------------------------------------------------ sources ------------------
    !> The [source] dictionary as smcrt_source (photon.f90:311-1043 via parse_source.f90): the
    !> emitter name, its position and direction, the three corner vectors pos1..pos3 of the
    !> uniform emitter and the beam parameters (the dictionary's keys of the same names).
    !> Names as init_source (photon.f90:127-156). Returns SMCRT_OK, or 1 for an unknown
    !> emitter or beam type.
    integer function smcrt_source_from(name, pos, dir, pos1, pos2, pos3, src, radius, focalLength, beam_type, &
                                       beam_size, rlo, rhi, sigma, rotation) result(ierr)
        character(len=*), intent(in) :: name
        real(c_double), intent(in) :: pos(3), dir(3), pos1(3), pos2(3), pos3(3)
        type(smcrt_source), intent(out) :: src
        real(c_double), optional, intent(in) :: radius, focalLength, beam_size, rlo, rhi, sigma, rotation(3)
        character(len=*), optional, intent(in) :: beam_type
        character(len=:), allocatable :: beam
        ierr = SMCRT_OK
        src%kind = 0
        select case (name)
        case ("point");    src%kind = SMCRT_SRC_POINT
        case ("uniform");  src%kind = SMCRT_SRC_UNIFORM
        case ("pencil");   src%kind = SMCRT_SRC_PENCIL
        case ("circular"); src%kind = SMCRT_SRC_CIRCULAR
        case ("focus");    src%kind = SMCRT_SRC_FOCUS
        case ("annulus");  src%kind = SMCRT_SRC_ANNULUS
        case ("slm");      src%kind = SMCRT_SRC_SLM
        case ("dslit");    src%kind = SMCRT_SRC_DSLIT
        case ("aperture"); src%kind = SMCRT_SRC_APERTURE
        case default
            ierr = 1
            return
        end select
        src%pos = pos; src%dir = dir
        src%p1 = pos1; src%p2 = pos2; src%p3 = pos3
        if (present(radius)) src%radius = radius
        if (present(focalLength)) src%focal_length = focalLength
        if (present(beam_size)) src%beam_size = beam_size
        if (present(rlo)) src%rlo = rlo
        if (present(rhi)) src%rhi = rhi
        if (present(sigma)) src%sigma = sigma
        if (present(rotation)) src%rotation = rotation
        beam = "gaussian"
        if (present(beam_type)) beam = beam_type
        if (src%kind == SMCRT_SRC_FOCUS) then  ! focus_type, photon.f90:415-427
            select case (beam)
            case ("gaussian"); src%beam = SMCRT_BEAM_GAUSSIAN
            case ("square");   src%beam = SMCRT_BEAM_SQUARE
            case ("circle");   src%beam = SMCRT_BEAM_CIRCLE
            case default; ierr = 1
            end select
        else if (src%kind == SMCRT_SRC_ANNULUS) then  ! annulus_type, photon.f90:880-892
            select case (beam)
            case ("gaussian");      src%beam = SMCRT_BEAM_GAUSSIAN
            case ("tophat");        src%beam = SMCRT_BEAM_TOPHAT
            case ("besselAnnulus"); src%beam = SMCRT_BEAM_BESSEL
            case default; ierr = 1
            end select
        end if
    end function smcrt_source_from

end module smcrt_glue
