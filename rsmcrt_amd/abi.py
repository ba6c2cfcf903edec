"""ctypes mirror of include/smcrt.h (the C ABI of the engine).

Field order and sizes must match the header exactly; tests/test_abi.py checks the sizes
against the library's own view of them.
"""
import ctypes as C

SMCRT_ABI_VERSION = 5

# smcrt_status
OK = 0
ERR_INVALID_ARG = -1
ERR_HIP = -2
ERR_RCCL = -3
ERR_DEVICE_FAULT = -4
ERR_NO_DEVICE = -5
ERR_OOM = -6
ERR_UNSUPPORTED = -7

STATUS_NAMES = {
    OK: "OK", ERR_INVALID_ARG: "INVALID_ARG", ERR_HIP: "HIP_ERROR", ERR_RCCL: "RCCL_ERROR",
    ERR_DEVICE_FAULT: "DEVICE_FAULT", ERR_NO_DEVICE: "NO_DEVICE", ERR_OOM: "OUT_OF_MEMORY",
    ERR_UNSUPPORTED: "UNSUPPORTED",
}

# smcrt_sdf_kind (reference src/sdfs/sdfs.f90)
SDF_SPHERE, SDF_BOX, SDF_TORUS, SDF_CYLINDER, SDF_TRIPRISM = 1, 2, 3, 4, 5
SDF_SEGMENT, SDF_CAPSULE, SDF_CONE, SDF_EGG, SDF_PLANE, SDF_MODEL = 6, 7, 8, 9, 10, 11
# the modifiers of src/sdfs/sdfModifiers.f90 (ABI 4): each wraps one node
SDF_REVOLUTION, SDF_EXTRUDE, SDF_ONION, SDF_TWIST, SDF_BEND, SDF_ELONGATE, SDF_DISPLACEMENT = 12, 13, 14, 15, 16, 17, 18
DISP_SINE = 1  # smcrt_displacement_fn

# smcrt_csg_op (src/sdfs/sdfModifiers.f90:428-491)
OP_UNION, OP_SMOOTH_UNION, OP_SUBTRACTION, OP_INTERSECTION = 0, 1, 2, 3

# smcrt_source_kind (reference src/photon.f90 emitters)
SRC_POINT, SRC_UNIFORM, SRC_PENCIL = 1, 2, 3
SRC_CIRCULAR, SRC_FOCUS, SRC_ANNULUS, SRC_SLM, SRC_DSLIT, SRC_APERTURE = 4, 5, 6, 7, 8, 9
SOURCE_KINDS = {"point": SRC_POINT, "uniform": SRC_UNIFORM, "pencil": SRC_PENCIL, "circular": SRC_CIRCULAR,
                "focus": SRC_FOCUS, "annulus": SRC_ANNULUS, "slm": SRC_SLM, "dslit": SRC_DSLIT,
                "aperture": SRC_APERTURE}

# smcrt_beam_kind: focus_type / annulus_type
BEAM_GAUSSIAN, BEAM_SQUARE, BEAM_CIRCLE, BEAM_TOPHAT, BEAM_BESSEL = 0, 1, 2, 3, 4
BEAM_KINDS = {"gaussian": BEAM_GAUSSIAN, "square": BEAM_SQUARE, "circle": BEAM_CIRCLE, "tophat": BEAM_TOPHAT,
              "besselAnnulus": BEAM_BESSEL}

# smcrt_spectrum_kind (src/opticalProps/piecewise.f90)
SPEC_CONSTANT, SPEC_1D, SPEC_2D = 0, 1, 2

# smcrt_detector_kind
DET_CIRCLE, DET_ANNULUS, DET_CAMERA, DET_FIBRE = 1, 2, 3, 4

# run flags
FLAG_PATHLENGTH = 1 << 0
FLAG_SURVIVAL_BIAS = 1 << 1
FLAG_RENDER_SOURCE = 1 << 2
FLAG_TEST_KERNEL = 1 << 3
FLAG_END_EARLY = 1 << 4
FLAG_RECORD_PHOTONS = 1 << 5
FLAG_ASYNC_FOLD = 1 << 6
FLAG_OVERLAP = 1 << 7

# counters
COUNTER_NAMES = [
    "photons", "emit_retries", "scatters", "absorbed", "sdf_evals", "deposits",
    "grid_updates", "tauint", "fresnel", "reflections", "bounce_aborts", "faults",
    "rng_draws", "detector_hits", "escaped", "wave_iters",
]
NCOUNTERS = 16
CTR = {name: i for i, name in enumerate(COUNTER_NAMES)}
# counters that describe the engine, not the photons: excluded from parity comparisons
ENGINE_COUNTERS = ("wave_iters",)


class SdfNode(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("layer", C.c_int32), ("op", C.c_int32),
        ("first_child", C.c_int32), ("n_children", C.c_int32), ("flags", C.c_int32), ("reserved", C.c_int32 * 2),
        ("transform", C.c_double * 16), ("param", C.c_double * 12), ("k", C.c_double),
        ("mus", C.c_double), ("mua", C.c_double), ("hgg", C.c_double), ("n", C.c_double),
    ]


# smcrt_sdf_node.flags (ABI 5)
NODE_ALBEDO_UNGUARDED = 1

# smcrt_spectral_mode (ABI 5)
SPECTRAL_INIT = 0
SPECTRAL_UPDATE = 1
SPECTRAL_INIT_AS_WRITTEN = 2


class Spectral(C.Structure):
    """smcrt_spectral: five piecewise1D tables, each a Fortran array(n, 2)."""
    _fields_ = [("n_mus", C.c_int64), ("n_mua", C.c_int64), ("n_hgg", C.c_int64), ("n_n", C.c_int64),
                ("n_flux", C.c_int64), ("mus", C.POINTER(C.c_double)), ("mua", C.POINTER(C.c_double)),
                ("hgg", C.POINTER(C.c_double)), ("n", C.POINTER(C.c_double)), ("flux", C.POINTER(C.c_double))]


class OptProps(C.Structure):
    _fields_ = [("mus", C.c_double), ("mua", C.c_double), ("hgg", C.c_double), ("g2", C.c_double),
                ("n", C.c_double), ("kappa", C.c_double), ("albedo", C.c_double), ("wavelength", C.c_double),
                ("node_flags", C.c_int32), ("reserved", C.c_int32)]


class Grid(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ny", C.c_int32), ("nz", C.c_int32), ("reserved", C.c_int32),
                ("xmax", C.c_double), ("ymax", C.c_double), ("zmax", C.c_double)]


class Spectrum(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("wavelength", C.c_double),
                ("n", C.c_int64), ("array", C.POINTER(C.c_double)),
                ("width", C.c_int32), ("height", C.c_int32), ("image", C.POINTER(C.c_double)),
                ("cell_width", C.c_double), ("cell_height", C.c_double)]


class Source(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32),
                ("pos", C.c_double * 3), ("dir", C.c_double * 3),
                ("p1", C.c_double * 3), ("p2", C.c_double * 3), ("p3", C.c_double * 3),
                ("beam", C.c_int32), ("reserved2", C.c_int32),
                ("radius", C.c_double), ("beam_size", C.c_double), ("focal_length", C.c_double),
                ("rlo", C.c_double), ("rhi", C.c_double), ("sigma", C.c_double),
                ("rotation", C.c_double * 3), ("spectrum", C.POINTER(Spectrum))]


class Detector(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("nbins", C.c_int32), ("layer", C.c_int32), ("reserved", C.c_int32),
        ("pos", C.c_double * 3), ("dir", C.c_double * 3), ("e1", C.c_double * 3), ("e2", C.c_double * 3),
        ("radius", C.c_double), ("r1", C.c_double), ("r2", C.c_double),
        ("width", C.c_double), ("height", C.c_double),
        ("bin_wid", C.c_double), ("bin_wid_y", C.c_double), ("fibre", C.c_double * 11),
    ]


class RunConfig(C.Structure):
    _fields_ = [("n_photons", C.c_uint64), ("first_photon", C.c_uint64), ("seed", C.c_uint64),
                ("flags", C.c_uint32), ("reserved", C.c_int32)]


class PhotonRecord(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("dir", C.c_double * 3), ("weight", C.c_double),
                ("cell", C.c_int32 * 3), ("layer", C.c_int32), ("nscatt", C.c_uint32),
                ("bounces", C.c_uint32), ("draws", C.c_uint32), ("status", C.c_uint32)]


class Tallies(C.Structure):
    _fields_ = [
        ("jmean", C.POINTER(C.c_float)), ("absorb", C.POINTER(C.c_float)),
        ("emission", C.POINTER(C.c_float)),
        ("jmean_f64", C.POINTER(C.c_double)), ("absorb_f64", C.POINTER(C.c_double)),
        ("emission_f64", C.POINTER(C.c_double)),
        ("det_bins", C.POINTER(C.c_double)), ("nscatt", C.POINTER(C.c_double)),
        ("moments", C.POINTER(C.c_double)), ("counters", C.POINTER(C.c_uint64)),
        ("records", C.POINTER(PhotonRecord)),
    ]


class DeviceTallies(C.Structure):
    _fields_ = [
        ("jmean", C.c_void_p), ("absorb", C.c_void_p), ("emission", C.c_void_p),
        ("det_bins", C.c_void_p), ("nscatt", C.c_void_p), ("moments", C.c_void_p),
        ("counters", C.c_void_p), ("records", C.c_void_p),
    ]


# photon record as a numpy dtype (same layout)
def record_dtype():
    import numpy as np
    return np.dtype([("pos", "<f8", 3), ("dir", "<f8", 3), ("weight", "<f8"), ("cell", "<i4", 3),
                     ("layer", "<i4"), ("nscatt", "<u4"), ("bounces", "<u4"), ("draws", "<u4"),
                     ("status", "<u4")])


# smcrt_symmetry (escape function, kernelsMod.f90:85-1460)
SYM_NONE, SYM_PRISM, SYM_FLIPPED, SYM_UNIFORM_SLAB, SYM_NONE_ROTATIONAL, SYM_ROTATIONAL_360 = 0, 1, 2, 3, 4, 5
SYMMETRY_KINDS = {"none": SYM_NONE, "prism": SYM_PRISM, "flipped": SYM_FLIPPED, "uniformSlab": SYM_UNIFORM_SLAB,
                  "noneRotational": SYM_NONE_ROTATIONAL, "360rotational": SYM_ROTATIONAL_360}


class EscapeConfig(C.Structure):
    _fields_ = [("symmetry", C.c_int32), ("n", C.c_int32 * 3), ("max", C.c_double * 3), ("pos", C.c_double * 3),
                ("dir", C.c_double * 3), ("rotation", C.c_double)]


# inverse MCRT flags (kernelsMod.f90:1462-1787)
INVERSE_FIND_MUS, INVERSE_FIND_MUA, INVERSE_FIND_G, INVERSE_FIND_N, INVERSE_APPLY_TRIAL = 1, 2, 4, 8, 16


class InverseConfig(C.Structure):
    _fields_ = [("layer", C.c_int32), ("flags", C.c_int32), ("max_steps", C.c_int32), ("reserved", C.c_int32),
                ("max_step_size", C.c_double), ("grad_step_size", C.c_double), ("accuracy", C.c_double),
                ("seed", C.c_uint64)]


# job modes (the reference's build variants)
JOB_DEFAULT, JOB_ESCAPE, JOB_INVERSE = 0, 1, 2


class JobDesc(C.Structure):
    _fields_ = [("n_photons", C.c_int64), ("seed", C.c_int64), ("flags", C.c_int32), ("n_nodes", C.c_int32),
                ("n_top", C.c_int32), ("n_dets", C.c_int32), ("overwrite", C.c_int32), ("grid", Grid),
                ("source", Source), ("experiment", C.c_char * 64), ("source_name", C.c_char * 32)]


# packed tally layout of the multi-GPU reduction (include/smcrt.h)
PACK_JMEAN, PACK_ABSORB, PACK_EMISSION, PACK_DET_BINS = 1, 2, 4, 8
UNIQUE_ID_BYTES = 128
ALL_DEVICES = -1


class PackLayout(C.Structure):
    _fields_ = [("n_voxels", C.c_int64), ("n_det_bins", C.c_int64), ("fields", C.c_uint32), ("reserved", C.c_int32)]


class KernelTimes(C.Structure):
    _fields_ = [("transport_ms", C.c_double), ("deposit_ms", C.c_double), ("launches", C.c_int64),
                ("lean_launches", C.c_int64), ("far_steps", C.c_int64), ("fold_cu_ms", C.c_double),
                ("lean_hazards", C.c_int64)]


EXPORTED_SYMBOLS = [
    "smcrt_abi_version", "smcrt_device_count", "smcrt_last_error", "smcrt_scene_create",
    "smcrt_scene_destroy", "smcrt_scene_det_bins", "smcrt_scene_set_optprops", "smcrt_run",
    "smcrt_run_device", "smcrt_normalise_fluence", "smcrt_scene_set_timing", "smcrt_scene_kernel_times",
    "smcrt_write_data_f32", "smcrt_write_data_f64", "smcrt_write_detector", "smcrt_write_checkpoint",
    "smcrt_job_load", "smcrt_job_destroy", "smcrt_job_info", "smcrt_job_scene", "smcrt_job_metadata", "smcrt_job_run",
    "smcrt_scene_info", "smcrt_run_origins", "smcrt_scene_classify", "smcrt_escape_sym_dims", "smcrt_escape_cells",
    "smcrt_escape_map", "smcrt_escape_run", "smcrt_scene_get_optprops", "smcrt_inverse_run", "smcrt_job_load_mode",
    "smcrt_job_escape_config", "smcrt_job_inverse_config", "smcrt_job_targets", "smcrt_job_run_escape",
    "smcrt_job_run_inverse", "smcrt_scene_fence",
    "smcrt_pack_size", "smcrt_pack_host", "smcrt_unpack_host", "smcrt_comm_unique_id", "smcrt_comm_init_rank",
    "smcrt_comm_info", "smcrt_comm_destroy", "smcrt_reduce_device_tallies", "smcrt_multi_create", "smcrt_multi_info",
    "smcrt_multi_scene", "smcrt_multi_run", "smcrt_multi_accumulate", "smcrt_multi_collect",
    "smcrt_multi_device_photons", "smcrt_multi_destroy", "smcrt_job_run_devices",
    "smcrt_spectral_sample", "smcrt_scene_set_spectral", "smcrt_scene_check",
]
