! smcrt_mod.f90 — ISO_C_BINDING interface to the MI355X engine (include/smcrt.h).
!
! The module a signedMCRT maintainer adds next to src/kernelsMod.f90 so that run_MCRT
! (kernelsMod.f90:1790-1898) can hand its photon loop to the GPU. Every type below is
! bind(C) and matches the C struct of the same name field for field; every interface binds
! one entry point of include/smcrt.h. See INTEGRATION.md for the run_MCRT body that uses it.
module smcrt_mod
    use iso_c_binding
    implicit none

    integer(c_int), parameter :: SMCRT_OK = 0
    ! smcrt_status (include/smcrt.h)
    integer(c_int), parameter :: SMCRT_ERR_INVALID_ARG = -1, SMCRT_ERR_HIP = -2, SMCRT_ERR_RCCL = -3, &
        SMCRT_ERR_DEVICE_FAULT = -4, SMCRT_ERR_NO_DEVICE = -5, SMCRT_ERR_OOM = -6, SMCRT_ERR_UNSUPPORTED = -7
    ! smcrt_sdf_kind
    integer(c_int32_t), parameter :: SMCRT_SDF_SPHERE = 1, SMCRT_SDF_BOX = 2, SMCRT_SDF_TORUS = 3, &
        SMCRT_SDF_CYLINDER = 4, SMCRT_SDF_TRIPRISM = 5, SMCRT_SDF_SEGMENT = 6, SMCRT_SDF_CAPSULE = 7, &
        SMCRT_SDF_CONE = 8, SMCRT_SDF_EGG = 9, SMCRT_SDF_PLANE = 10, SMCRT_SDF_MODEL = 11
    ! the modifiers of sdfModifiers.f90 (ABI 4): each wraps one node
    integer(c_int32_t), parameter :: SMCRT_SDF_REVOLUTION = 12, SMCRT_SDF_EXTRUDE = 13, SMCRT_SDF_ONION = 14, &
        SMCRT_SDF_TWIST = 15, SMCRT_SDF_BEND = 16, SMCRT_SDF_ELONGATE = 17, SMCRT_SDF_DISPLACEMENT = 18
    integer(c_int32_t), parameter :: SMCRT_DISP_SINE = 1
    integer(c_int), parameter :: SMCRT_MOD_ABI_VERSION = 5  ! compare with smcrt_abi_version()
    ! smcrt_csg_op
    integer(c_int32_t), parameter :: SMCRT_OP_UNION = 0, SMCRT_OP_SMOOTH_UNION = 1, &
        SMCRT_OP_SUBTRACTION = 2, SMCRT_OP_INTERSECTION = 3
    ! smcrt_source_kind (photon.f90 emitters)
    integer(c_int32_t), parameter :: SMCRT_SRC_POINT = 1, SMCRT_SRC_UNIFORM = 2, SMCRT_SRC_PENCIL = 3, &
        SMCRT_SRC_CIRCULAR = 4, SMCRT_SRC_FOCUS = 5, SMCRT_SRC_ANNULUS = 6, SMCRT_SRC_SLM = 7, &
        SMCRT_SRC_DSLIT = 8, SMCRT_SRC_APERTURE = 9
    ! smcrt_beam_kind (focus_type / annulus_type)
    integer(c_int32_t), parameter :: SMCRT_BEAM_GAUSSIAN = 0, SMCRT_BEAM_SQUARE = 1, SMCRT_BEAM_CIRCLE = 2, &
        SMCRT_BEAM_TOPHAT = 3, SMCRT_BEAM_BESSEL = 4
    ! smcrt_spectrum_kind (piecewise.f90)
    integer(c_int32_t), parameter :: SMCRT_SPEC_CONSTANT = 0, SMCRT_SPEC_1D = 1, SMCRT_SPEC_2D = 2
    ! smcrt_detector_kind
    integer(c_int32_t), parameter :: SMCRT_DET_CIRCLE = 1, SMCRT_DET_ANNULUS = 2, SMCRT_DET_CAMERA = 3, &
        SMCRT_DET_FIBRE = 4
    ! run flags
    integer(c_int32_t), parameter :: SMCRT_FLAG_PATHLENGTH = 1, SMCRT_FLAG_SURVIVAL_BIAS = 2, &
        SMCRT_FLAG_RENDER_SOURCE = 4, SMCRT_FLAG_TEST_KERNEL = 8, SMCRT_FLAG_END_EARLY = 16, &
        SMCRT_FLAG_RECORD_PHOTONS = 32, SMCRT_FLAG_ASYNC_FOLD = 64, SMCRT_FLAG_OVERLAP = 128
    integer, parameter :: SMCRT_NCOUNTERS = 16
    ! multi-GPU: packed-tally fields (smcrt_pack_layout%fields), all visible devices
    integer(c_int32_t), parameter :: SMCRT_PACK_JMEAN = 1, SMCRT_PACK_ABSORB = 2, SMCRT_PACK_EMISSION = 4, &
        SMCRT_PACK_DET_BINS = 8
    integer(c_int32_t), parameter :: SMCRT_ALL_DEVICES = -1
    integer, parameter :: SMCRT_UNIQUE_ID_BYTES = 128
    ! smcrt_symmetry (escape function, kernelsMod.f90:85-1460)
    integer(c_int32_t), parameter :: SMCRT_SYM_NONE = 0, SMCRT_SYM_PRISM = 1, SMCRT_SYM_FLIPPED = 2, &
        SMCRT_SYM_UNIFORM_SLAB = 3, SMCRT_SYM_NONE_ROTATIONAL = 4, SMCRT_SYM_ROTATIONAL_360 = 5
    ! inverse MCRT flags (kernelsMod.f90:1462-1787)
    integer(c_int32_t), parameter :: SMCRT_INVERSE_FIND_MUS = 1, SMCRT_INVERSE_FIND_MUA = 2, &
        SMCRT_INVERSE_FIND_G = 4, SMCRT_INVERSE_FIND_N = 8, SMCRT_INVERSE_APPLY_TRIAL = 16

    type, bind(C) :: smcrt_sdf_node
        integer(c_int32_t) :: kind = 0, layer = 0, op = 0, first_child = 0, n_children = 0
        integer(c_int32_t) :: flags = 0       ! SMCRT_NODE_* (ABI 5)
        integer(c_int32_t) :: reserved(2) = 0
        real(c_double)     :: transform(16) = 0._c_double   ! = reshape(sdf%transform, [16])
        real(c_double)     :: param(12) = 0._c_double
        real(c_double)     :: k = 0._c_double
        real(c_double)     :: mus = 0._c_double, mua = 0._c_double, hgg = 0._c_double, n = 1._c_double
    end type smcrt_sdf_node

    type, bind(C) :: smcrt_grid
        integer(c_int32_t) :: nx, ny, nz, reserved = 0
        real(c_double)     :: xmax, ymax, zmax
    end type smcrt_grid

    type, bind(C) :: smcrt_spectrum
        integer(c_int32_t) :: kind = 0, reserved = 0
        real(c_double)     :: wavelength = 500._c_double
        integer(c_int64_t) :: n = 0
        type(c_ptr)        :: array = c_null_ptr      ! c_loc(array(1,1)) of an (n,2) real(c_double) array
        integer(c_int32_t) :: width = 0, height = 0
        type(c_ptr)        :: image = c_null_ptr      ! c_loc(image(1,1)) of image(width,height)
        real(c_double)     :: cell_width = 0._c_double, cell_height = 0._c_double
    end type smcrt_spectrum

    type, bind(C) :: smcrt_source
        integer(c_int32_t) :: kind, reserved = 0
        real(c_double)     :: pos(3) = 0._c_double, dir(3) = 0._c_double
        real(c_double)     :: p1(3) = 0._c_double, p2(3) = 0._c_double, p3(3) = 0._c_double
        integer(c_int32_t) :: beam = 0, reserved2 = 0
        real(c_double)     :: radius = 0.5_c_double, beam_size = 0.5_c_double, focal_length = 1._c_double
        real(c_double)     :: rlo = 0.5_c_double, rhi = 0.6_c_double, sigma = 0.04_c_double
        real(c_double)     :: rotation(3) = 0._c_double
        type(c_ptr)        :: spectrum = c_null_ptr  ! c_loc of a target smcrt_spectrum, or null (constant 500)
    end type smcrt_source

    type, bind(C) :: smcrt_detector
        integer(c_int32_t) :: kind = 0, nbins = 0, layer = 0, reserved = 0
        real(c_double)     :: pos(3) = 0._c_double, dir(3) = 0._c_double
        real(c_double)     :: e1(3) = 0._c_double, e2(3) = 0._c_double
        real(c_double)     :: radius = 0._c_double, r1 = 0._c_double, r2 = 0._c_double
        real(c_double)     :: width = 0._c_double, height = 0._c_double
        real(c_double)     :: bin_wid = 0._c_double, bin_wid_y = 0._c_double
        real(c_double)     :: fibre(11) = 0._c_double
    end type smcrt_detector

    type, bind(C) :: smcrt_run_config
        integer(c_int64_t) :: n_photons, first_photon = 0, seed
        integer(c_int32_t) :: flags, reserved = 0
    end type smcrt_run_config

    type, bind(C) :: smcrt_tallies
        type(c_ptr) :: jmean = c_null_ptr, absorb = c_null_ptr, emission = c_null_ptr
        type(c_ptr) :: jmean_f64 = c_null_ptr, absorb_f64 = c_null_ptr, emission_f64 = c_null_ptr
        type(c_ptr) :: det_bins = c_null_ptr, nscatt = c_null_ptr, moments = c_null_ptr
        type(c_ptr) :: counters = c_null_ptr, records = c_null_ptr
    end type smcrt_tallies

    type, bind(C) :: smcrt_device_tallies
        type(c_ptr) :: jmean = c_null_ptr, absorb = c_null_ptr, emission = c_null_ptr
        type(c_ptr) :: det_bins = c_null_ptr, nscatt = c_null_ptr, moments = c_null_ptr
        type(c_ptr) :: counters = c_null_ptr, records = c_null_ptr
    end type smcrt_device_tallies

    type, bind(C) :: smcrt_escape_config          ! the [symmetry] table
        integer(c_int32_t) :: symmetry = 0, n(3) = 10
        real(c_double)     :: max(3) = 1._c_double, pos(3) = 0._c_double
        real(c_double)     :: dir(3) = [0._c_double, 0._c_double, 1._c_double], rotation = 0._c_double
    end type smcrt_escape_config

    ! ABI 5: spectral optical properties (opticalProperties.f90:127-201)
    integer(c_int32_t), parameter :: SMCRT_NODE_ALBEDO_UNGUARDED = 1
    integer(c_int32_t), parameter :: SMCRT_SPECTRAL_INIT = 0, SMCRT_SPECTRAL_UPDATE = 1, &
        SMCRT_SPECTRAL_INIT_AS_WRITTEN = 2

    type, bind(C) :: smcrt_spectral               ! five piecewise1D array(n, 2) tables
        integer(c_int64_t) :: n_mus = 0, n_mua = 0, n_hgg = 0, n_n = 0, n_flux = 0
        type(c_ptr)        :: mus = c_null_ptr, mua = c_null_ptr, hgg = c_null_ptr, n = c_null_ptr, &
                              flux = c_null_ptr
    end type smcrt_spectral

    type, bind(C) :: smcrt_optprops               ! opticalProp_base's fields + the wavelength
        real(c_double)     :: mus = 0, mua = 0, hgg = 0, g2 = 0, n = 0, kappa = 0, albedo = 0, wavelength = 0
        integer(c_int32_t) :: node_flags = 0, reserved = 0
    end type smcrt_optprops

    type, bind(C) :: smcrt_inverse_config         ! the [inverse] table
        integer(c_int32_t) :: layer, flags, max_steps = 1000, reserved = 0
        real(c_double)     :: max_step_size = 1._c_double, grad_step_size = 1e-4_c_double, accuracy = 0.01_c_double
        integer(c_int64_t) :: seed = 123456789
    end type smcrt_inverse_config

    type, bind(C) :: smcrt_pack_layout            ! the packed buffer of the multi-GPU reduction
        integer(c_int64_t) :: n_voxels = 0, n_det_bins = 0
        integer(c_int32_t) :: fields = 0, reserved = 0
    end type smcrt_pack_layout

    type, bind(C) :: smcrt_kernel_times
        real(c_double)     :: transport_ms = 0._c_double, deposit_ms = 0._c_double
        integer(c_int64_t) :: launches = 0, lean_launches = 0, far_steps = 0
        real(c_double)     :: fold_cu_ms = 0._c_double
        integer(c_int64_t) :: lean_hazards = 0  ! ABI 4
    end type smcrt_kernel_times

    interface
        integer(c_int) function smcrt_abi_version() bind(C, name="smcrt_abi_version")
            import :: c_int
        end function smcrt_abi_version

        integer(c_int) function smcrt_device_count(count) bind(C, name="smcrt_device_count")
            import :: c_int, c_int32_t
            integer(c_int32_t), intent(out) :: count
        end function smcrt_device_count

        type(c_ptr) function smcrt_last_error() bind(C, name="smcrt_last_error")
            import :: c_ptr
        end function smcrt_last_error

        integer(c_int) function smcrt_scene_create(nodes, n_nodes, top, n_top, grid, dets, n_dets, &
                                                   device, scene) bind(C, name="smcrt_scene_create")
            import :: c_int, c_int32_t, c_ptr, smcrt_sdf_node, smcrt_grid, smcrt_detector
            type(smcrt_sdf_node), intent(in)  :: nodes(*)
            integer(c_int32_t), value         :: n_nodes
            integer(c_int32_t), intent(in)    :: top(*)
            integer(c_int32_t), value         :: n_top
            type(smcrt_grid), intent(in)      :: grid
            type(smcrt_detector), intent(in)  :: dets(*)
            integer(c_int32_t), value         :: n_dets, device
            type(c_ptr), intent(out)          :: scene
        end function smcrt_scene_create

        subroutine smcrt_scene_destroy(scene) bind(C, name="smcrt_scene_destroy")
            import :: c_ptr
            type(c_ptr), value :: scene
        end subroutine smcrt_scene_destroy

        integer(c_int) function smcrt_scene_det_bins(scene, n) bind(C, name="smcrt_scene_det_bins")
            import :: c_int, c_int64_t, c_ptr
            type(c_ptr), value              :: scene
            integer(c_int64_t), intent(out) :: n
        end function smcrt_scene_det_bins

        integer(c_int) function smcrt_scene_set_optprops(scene, top_index, mus, mua, hgg, n) &
                bind(C, name="smcrt_scene_set_optprops")
            import :: c_int, c_int32_t, c_double, c_ptr
            type(c_ptr), value        :: scene
            integer(c_int32_t), value :: top_index
            real(c_double), value     :: mus, mua, hgg, n
        end function smcrt_scene_set_optprops

        integer(c_int) function smcrt_scene_check(scene) bind(C, name="smcrt_scene_check")
            import :: c_int, c_ptr
            type(c_ptr), value :: scene
        end function smcrt_scene_check

        integer(c_int) function smcrt_spectral_sample(sp, mode, seed, draw, out) &
                bind(C, name="smcrt_spectral_sample")
            import :: c_int, c_int32_t, c_int64_t, smcrt_spectral, smcrt_optprops
            type(smcrt_spectral), intent(in)  :: sp
            integer(c_int32_t), value         :: mode
            integer(c_int64_t), value         :: seed
            integer(c_int64_t), intent(inout) :: draw
            type(smcrt_optprops), intent(out) :: out
        end function smcrt_spectral_sample

        integer(c_int) function smcrt_scene_set_spectral(scene, top_index, sp, mode, seed, draw, out) &
                bind(C, name="smcrt_scene_set_spectral")
            import :: c_int, c_int32_t, c_int64_t, c_ptr, smcrt_spectral, smcrt_optprops
            type(c_ptr), value                :: scene
            integer(c_int32_t), value         :: top_index
            type(smcrt_spectral), intent(in)  :: sp
            integer(c_int32_t), value         :: mode
            integer(c_int64_t), value         :: seed
            integer(c_int64_t), intent(inout) :: draw
            type(smcrt_optprops), intent(out) :: out
        end function smcrt_scene_set_spectral

        integer(c_int) function smcrt_run(scene, src, cfg, io) bind(C, name="smcrt_run")
            import :: c_int, c_ptr, smcrt_source, smcrt_run_config, smcrt_tallies
            type(c_ptr), value                 :: scene
            type(smcrt_source), intent(in)     :: src
            type(smcrt_run_config), intent(in) :: cfg
            type(smcrt_tallies), intent(inout) :: io
        end function smcrt_run

        ! the escape function's batched launch cells (kernelsMod.f90:533-642): one launch for
        ! every origin; det_totals(n_dets, n_origins) accumulates total_dect per origin
        integer(c_int) function smcrt_run_origins(scene, src, origins, n_origins, cfg, det_totals, io) &
                bind(C, name="smcrt_run_origins")
            import :: c_int, c_ptr, c_double, c_int64_t, smcrt_source, smcrt_run_config, smcrt_tallies
            type(c_ptr), value                 :: scene
            type(smcrt_source), intent(in)     :: src
            real(c_double), intent(in)         :: origins(3, *)
            integer(c_int64_t), value          :: n_origins
            type(smcrt_run_config), intent(in) :: cfg
            real(c_double), intent(inout)      :: det_totals(*)
            type(smcrt_tallies), intent(inout) :: io
        end function smcrt_run_origins

        integer(c_int) function smcrt_scene_classify(scene, points, n, layer, kappa) bind(C, name="smcrt_scene_classify")
            import :: c_int, c_ptr, c_double, c_int64_t, c_int32_t
            type(c_ptr), value             :: scene
            real(c_double), intent(in)     :: points(3, *)
            integer(c_int64_t), value      :: n
            integer(c_int32_t), intent(out) :: layer(*)
            real(c_double), intent(out)    :: kappa(*)
        end function smcrt_scene_classify

        ! escape_Function (kernelsMod.f90:85-530): escape_sym(n_dets, n0, n1, n2) and
        ! escape(n_dets, nxg, nyg, nzg), real(sp) as iarray.f90:18
        integer(c_int) function smcrt_escape_run(scene, src, cfg, run, escape_sym, escape, io) &
                bind(C, name="smcrt_escape_run")
            import :: c_int, c_ptr, c_float, smcrt_source, smcrt_escape_config, smcrt_run_config, smcrt_tallies
            type(c_ptr), value                    :: scene
            type(smcrt_source), intent(in)        :: src
            type(smcrt_escape_config), intent(in) :: cfg
            type(smcrt_run_config), intent(in)    :: run
            real(c_float), intent(out)            :: escape_sym(*), escape(*)
            type(smcrt_tallies), intent(inout)    :: io
        end function smcrt_escape_run

        ! inverse_MCRT (kernelsMod.f90:1462-1751): steps = gradDescentData(max_steps, 5)
        integer(c_int) function smcrt_inverse_run(scene, src, cfg, run, targets, steps, io) &
                bind(C, name="smcrt_inverse_run")
            import :: c_int, c_ptr, c_double, smcrt_source, smcrt_inverse_config, smcrt_run_config
            type(c_ptr), value                     :: scene
            type(smcrt_source), intent(in)         :: src
            type(smcrt_inverse_config), intent(in) :: cfg
            type(smcrt_run_config), intent(in)     :: run
            real(c_double), intent(in)             :: targets(*)
            real(c_double), intent(out)            :: steps(*)
            type(c_ptr), value                     :: io
        end function smcrt_inverse_run

        integer(c_int) function smcrt_run_device(scene, src, cfg, dev, stream) bind(C, name="smcrt_run_device")
            import :: c_int, c_ptr, smcrt_source, smcrt_run_config, smcrt_device_tallies
            type(c_ptr), value                 :: scene
            type(smcrt_source), intent(in)     :: src
            type(smcrt_run_config), intent(in) :: cfg
            type(smcrt_device_tallies), intent(inout) :: dev
            type(c_ptr), value                 :: stream
        end function smcrt_run_device

        integer(c_int) function smcrt_scene_set_timing(scene, enable) bind(C, name="smcrt_scene_set_timing")
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value        :: scene
            integer(c_int32_t), value :: enable
        end function smcrt_scene_set_timing

        integer(c_int) function smcrt_scene_kernel_times(scene, times) bind(C, name="smcrt_scene_kernel_times")
            import :: c_int, c_ptr, smcrt_kernel_times
            type(c_ptr), value                    :: scene
            type(smcrt_kernel_times), intent(out) :: times
        end function smcrt_scene_kernel_times

        integer(c_int) function smcrt_write_data_f32(filename, array, nx, ny, nz, metadata, dect_id, overwrite, &
                                                     written_path, path_cap) bind(C, name="smcrt_write_data_f32")
            import :: c_int, c_int32_t, c_char, c_float, c_ptr
            character(kind=c_char), intent(in) :: filename(*)
            real(c_float), intent(in)          :: array(*)
            integer(c_int32_t), value          :: nx, ny, nz
            type(c_ptr), value                 :: metadata, dect_id   ! C strings or c_null_ptr
            integer(c_int32_t), value          :: overwrite
            type(c_ptr), value                 :: written_path
            integer(c_int32_t), value          :: path_cap
        end function smcrt_write_data_f32

        integer(c_int) function smcrt_write_detector(filename, d, data, id, nphotons) &
                bind(C, name="smcrt_write_detector")
            import :: c_int, c_int64_t, c_char, c_double, smcrt_detector
            character(kind=c_char), intent(in) :: filename(*)
            type(smcrt_detector), intent(in)   :: d
            real(c_double), intent(in)         :: data(*)
            character(kind=c_char), intent(in) :: id(*)
            integer(c_int64_t), value          :: nphotons
        end function smcrt_write_detector

        integer(c_int) function smcrt_write_checkpoint(filename, toml_filename, photons_run, jmean, grid, &
                                                       overwrite, written_path, path_cap) &
                bind(C, name="smcrt_write_checkpoint")
            import :: c_int, c_int32_t, c_int64_t, c_char, c_float, c_ptr, smcrt_grid
            character(kind=c_char), intent(in) :: filename(*), toml_filename(*)
            integer(c_int64_t), value          :: photons_run
            real(c_float), intent(in)          :: jmean(*)
            type(smcrt_grid), intent(in)       :: grid
            integer(c_int32_t), value          :: overwrite
            type(c_ptr), value                 :: written_path
            integer(c_int32_t), value          :: path_cap
        end function smcrt_write_checkpoint

        ! ---- multi-GPU (SURVEY §8(b) n_gpus, §8(e)): the OpenMP team of run_MCRT
        ! (kernelsMod.f90:1833-1861) and its intended mpi_reduce (:2351-2357) ----
        ! one process, several GPUs: `devices` is c_loc of an integer(c_int32_t) array of device
        ! ordinals, or c_null_ptr for devices 0 .. n_devices-1 (n_devices <= 0: every visible GPU)
        integer(c_int) function smcrt_multi_create(nodes, n_nodes, top, n_top, grid, dets, n_dets, &
                devices, n_devices, multi) bind(C, name="smcrt_multi_create")
            import :: c_int, c_int32_t, c_ptr, smcrt_sdf_node, smcrt_grid, smcrt_detector
            type(smcrt_sdf_node), intent(in) :: nodes(*)
            integer(c_int32_t), value        :: n_nodes
            integer(c_int32_t), intent(in)   :: top(*)
            integer(c_int32_t), value        :: n_top
            type(smcrt_grid), intent(in)     :: grid
            type(smcrt_detector), intent(in) :: dets(*)
            integer(c_int32_t), value        :: n_dets
            type(c_ptr), value               :: devices
            integer(c_int32_t), value        :: n_devices
            type(c_ptr), intent(out)         :: multi
        end function smcrt_multi_create

        integer(c_int) function smcrt_multi_info(multi, n_devices) bind(C, name="smcrt_multi_info")
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value              :: multi
            integer(c_int32_t), intent(out) :: n_devices
        end function smcrt_multi_info

        type(c_ptr) function smcrt_multi_scene(multi, i) bind(C, name="smcrt_multi_scene")
            import :: c_int32_t, c_ptr
            type(c_ptr), value        :: multi
            integer(c_int32_t), value :: i
        end function smcrt_multi_scene

        ! smcrt_run over the devices: accumulate + collect
        integer(c_int) function smcrt_multi_run(multi, src, cfg, io) bind(C, name="smcrt_multi_run")
            import :: c_int, c_ptr, smcrt_source, smcrt_run_config, smcrt_tallies
            type(c_ptr), value                 :: multi
            type(smcrt_source), intent(in)     :: src
            type(smcrt_run_config), intent(in) :: cfg
            type(smcrt_tallies), intent(in)    :: io
        end function smcrt_multi_run

        ! photons handed to the devices in chunks, accumulated on the devices (no collective)
        integer(c_int) function smcrt_multi_accumulate(multi, src, cfg) bind(C, name="smcrt_multi_accumulate")
            import :: c_int, c_ptr, smcrt_source, smcrt_run_config
            type(c_ptr), value                 :: multi
            type(smcrt_source), intent(in)     :: src
            type(smcrt_run_config), intent(in) :: cfg
        end function smcrt_multi_accumulate

        ! ONE packed RCCL reduce of every device's accumulators, added into io
        integer(c_int) function smcrt_multi_collect(multi, io) bind(C, name="smcrt_multi_collect")
            import :: c_int, c_ptr, smcrt_tallies
            type(c_ptr), value              :: multi
            type(smcrt_tallies), intent(in) :: io
        end function smcrt_multi_collect

        integer(c_int) function smcrt_multi_device_photons(multi, photons) bind(C, name="smcrt_multi_device_photons")
            import :: c_int, c_int64_t, c_ptr
            type(c_ptr), value              :: multi
            integer(c_int64_t), intent(out) :: photons(*)
        end function smcrt_multi_device_photons

        subroutine smcrt_multi_destroy(multi) bind(C, name="smcrt_multi_destroy")
            import :: c_ptr
            type(c_ptr), value :: multi
        end subroutine smcrt_multi_destroy

        ! one process per GPU (mpirun): rank 0 makes the id and broadcasts its bytes (e.g. with
        ! MPI_Bcast), every rank joins on its device, runs smcrt_run_device into device buffers
        ! and sums them with ONE packed collective (root < 0: all-reduce; else reduce to root)
        integer(c_int) function smcrt_comm_unique_id(id) bind(C, name="smcrt_comm_unique_id")
            import :: c_int, c_int8_t
            integer(c_int8_t), intent(out) :: id(*)
        end function smcrt_comm_unique_id

        integer(c_int) function smcrt_comm_init_rank(id, n_ranks, rank, device, comm) &
                bind(C, name="smcrt_comm_init_rank")
            import :: c_int, c_int8_t, c_int32_t, c_ptr
            integer(c_int8_t), intent(in) :: id(*)
            integer(c_int32_t), value     :: n_ranks, rank, device
            type(c_ptr), intent(out)      :: comm
        end function smcrt_comm_init_rank

        subroutine smcrt_comm_destroy(comm) bind(C, name="smcrt_comm_destroy")
            import :: c_ptr
            type(c_ptr), value :: comm
        end subroutine smcrt_comm_destroy

        integer(c_int) function smcrt_comm_info(comm, n_ranks, rank, device) bind(C, name="smcrt_comm_info")
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value         :: comm
            integer(c_int32_t), intent(out) :: n_ranks, rank, device
        end function smcrt_comm_info

        integer(c_int) function smcrt_reduce_device_tallies(scene, comm, dev, root, stream) &
                bind(C, name="smcrt_reduce_device_tallies")
            import :: c_int, c_int32_t, c_ptr, smcrt_device_tallies
            type(c_ptr), value                     :: scene, comm
            type(smcrt_device_tallies), intent(in) :: dev
            integer(c_int32_t), value              :: root
            type(c_ptr), value                     :: stream
        end function smcrt_reduce_device_tallies

        integer(c_int) function smcrt_scene_fence(scene, stream) bind(C, name="smcrt_scene_fence")
            import :: c_int, c_ptr
            type(c_ptr), value :: scene, stream
        end function smcrt_scene_fence

        ! the packed layout on the host (to move a rank's tallies through MPI instead of RCCL)
        integer(c_int) function smcrt_pack_size(layout, n) bind(C, name="smcrt_pack_size")
            import :: c_int, c_int64_t, smcrt_pack_layout
            type(smcrt_pack_layout), intent(in) :: layout
            integer(c_int64_t), intent(out)     :: n
        end function smcrt_pack_size

        integer(c_int) function smcrt_pack_host(layout, t, buf) bind(C, name="smcrt_pack_host")
            import :: c_int, c_double, smcrt_pack_layout, smcrt_tallies
            type(smcrt_pack_layout), intent(in) :: layout
            type(smcrt_tallies), intent(in)     :: t
            real(c_double), intent(out)         :: buf(*)
        end function smcrt_pack_host

        integer(c_int) function smcrt_unpack_host(layout, buf, t) bind(C, name="smcrt_unpack_host")
            import :: c_int, c_double, smcrt_pack_layout, smcrt_tallies
            type(smcrt_pack_layout), intent(in) :: layout
            real(c_double), intent(in)          :: buf(*)
            type(smcrt_tallies), intent(in)     :: t
        end function smcrt_unpack_host

        integer(c_int) function smcrt_normalise_fluence(grid_data, grid, nphotons) &
                bind(C, name="smcrt_normalise_fluence")
            import :: c_int, c_int64_t, c_float, smcrt_grid
            real(c_float), intent(inout) :: grid_data(*)
            type(smcrt_grid), intent(in) :: grid
            integer(c_int64_t), value    :: nphotons
        end function smcrt_normalise_fluence
    end interface

contains

    function smcrt_error_message() result(msg)
        !! Copy smcrt_last_error() into a Fortran string.
        character(len=:), allocatable :: msg
        character(kind=c_char), pointer :: p(:)
        integer :: i, n
        type(c_ptr) :: cp
        cp = smcrt_last_error()
        call c_f_pointer(cp, p, [4096])
        n = 0
        do i = 1, 4096
            if (p(i) == c_null_char) exit
            n = i
        end do
        allocate(character(len=n) :: msg)
        do i = 1, n
            msg(i:i) = p(i)
        end do
    end function smcrt_error_message

end module smcrt_mod
