/*
 * smcrt.h — C ABI of the MI355X photon-packet engine (rsmcrt_amd).
 *
 * Drop-in boundary for signedMCRT's per-photon hot path. The reference seam is
 *   subroutine run_MCRT(input_file, history, packet, dict, distances, image, dects, array,
 *                       nscatt, start, tev, spectrum)          /root/reference/src/kernelsMod.f90:1790-1898
 * whose results are side effects on the module globals jmean/absorb/emission
 * (src/iarray.f90:10-18), on nscatt (intent inout) and on dects(i)%p%data. Per-photon
 * tauint2 calls (src/inttau2.f90:15) are not FFI-viable, so the whole photon loop
 * (noBiasPropagation kernelsMod.f90:1901-1976 / survivalBiasPropagation :1979-2067) crosses
 * this boundary at once.
 *
 * Everything here is plain C: POD structs, pointers and sizes; no HIP or torch types.
 * A Fortran ISO_C_BINDING module that binds these entry points is given in INTEGRATION.md.
 *
 * Conventions
 *  - All geometry is fp64 (reference constants.f90:18, wp = real64).
 *  - Grids are (nx, ny, nz) with x fastest (Fortran column-major jmean(i,j,k), iarray.f90:12).
 *  - Tallies are ACCUMULATED INTO (never overwritten), so checkpoint/resume and multi-run
 *    accumulation work (kernelsMod.f90:52-72).
 *  - Photon j of a run uses the counter-based Philox4x32-10 stream keyed by
 *    (seed, first_photon + j): results do not depend on how photons are split across
 *    launches or GPUs (replaces init_rng/ran2, random_mod.f90:44-90).
 *  - Every entry point returns 0 on success or a negative smcrt_status; none aborts.
 *    The reference's `error stop` paths inside the photon loop (inttau2.f90:276,515,572)
 *    terminate only the offending photon and are counted in SMCRT_CTR_FAULTS.
 */
#ifndef SMCRT_H
#define SMCRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMCRT_ABI_VERSION 5

typedef enum smcrt_status {
  SMCRT_OK = 0,
  SMCRT_ERR_INVALID_ARG = -1,
  SMCRT_ERR_HIP = -2,
  SMCRT_ERR_RCCL = -3,
  SMCRT_ERR_DEVICE_FAULT = -4,
  SMCRT_ERR_NO_DEVICE = -5,
  SMCRT_ERR_OOM = -6,
  SMCRT_ERR_UNSUPPORTED = -7
} smcrt_status;

/* ---------------------------------------------------------------- SDF scene ---- */
/* Primitive kinds: reference src/sdfs/sdfs.f90 evaluate_* (494-735). */
typedef enum smcrt_sdf_kind {
  SMCRT_SDF_SPHERE = 1,   /* param[0]=radius                                   sdfs.f90:494-508 */
  SMCRT_SDF_BOX = 2,      /* param[0..2]=HALF lengths (ctor halves, :455)      sdfs.f90:510-525 */
  SMCRT_SDF_TORUS = 3,    /* param[0]=oradius param[1]=iradius                 sdfs.f90:527-542 */
  SMCRT_SDF_CYLINDER = 4, /* param[0..2]=a param[3..5]=b param[6]=radius       sdfs.f90:544-581 */
  SMCRT_SDF_TRIPRISM = 5, /* param[0]=h1 param[1]=h2                           sdfs.f90:583-597 */
  SMCRT_SDF_SEGMENT = 6,  /* param[0..2]=a param[3..5]=b                       sdfs.f90:599-626 */
  SMCRT_SDF_CAPSULE = 7,  /* param[0..2]=a param[3..5]=b param[6]=r            sdfs.f90:628-648 */
  SMCRT_SDF_CONE = 8,     /* param[0..2]=a param[3..5]=b param[6]=ra param[7]=rb sdfs.f90:650-686 */
  SMCRT_SDF_EGG = 9,      /* param[0]=r1 param[1]=r2 param[2]=h                sdfs.f90:688-718 */
  SMCRT_SDF_PLANE = 10,   /* param[0..2]=a (unit normal)                       sdfs.f90:720-735 */
  SMCRT_SDF_MODEL = 11,   /* CSG fold over children       sdf_base.f90:146-161, sdfModifiers.f90:428-491 */
  /* ---- ABI 4: the domain modifiers of sdfModifiers.f90. Each wraps ONE node
     (first_child, n_children = 1), which may be a primitive, a model or another modifier; it
     takes the layer and optical properties of that node (the *_init functions copy
     prim%optProps and prim%layer) and ignores its own transform (the reference sets it to the
     identity and never applies it). Models and modifiers nest at most 32 levels deep. */
  SMCRT_SDF_REVOLUTION = 12, /* param[0]=o, param[1..3]=center: q = (|(p-c).xz| - o, (p-c).y, 0)   :303-321 */
  SMCRT_SDF_EXTRUDE = 13,    /* param[0]=h: w = (d(p), |p.z| - h); min(max(w),0) + |max(w,0)|    :286-301 */
  SMCRT_SDF_ONION = 14,      /* param[0]=thickness: |d(p)| - thickness                          :323-333 */
  SMCRT_SDF_TWIST = 15,      /* param[0]=k: d of p rotated by k*p.z in the xy plane              :353-371
                                (twist_init takes k as default real: pass real(k_sp, wp))      */
  SMCRT_SDF_BEND = 16,       /* param[0]=k: d of p rotated by k*p.x in the xy plane              :373-391 */
  SMCRT_SDF_ELONGATE = 17,   /* param[0..2]=size: q = |p| - size; d(max(q,0)) + min(max(q),0)     :335-351 */
  SMCRT_SDF_DISPLACEMENT = 18 /* d(p) + f(p) with a built-in f (param[0] = smcrt_displacement_fn):  :393-408
                                the reference takes any pure function of pos and ships none    */
} smcrt_sdf_kind;

/* Built-in displacement functions f(p) of SMCRT_SDF_DISPLACEMENT (param[0]); the reference's
 * displacement_init takes an arbitrary procedure(primitive) pointer, which cannot cross to
 * device code. The `repeat` modifier is not provided: its evaluate is an `error stop "Not
 * implmented"` in the reference (sdfModifiers.f90:410-426). */
typedef enum smcrt_displacement_fn {
  SMCRT_DISP_SINE = 1 /* param[1]=amplitude a, param[2..4]=frequencies (fx, fy, fz):
                         f(p) = ((a * sin(fx*p.x)) * sin(fy*p.y)) * sin(fz*p.z) */
} smcrt_displacement_fn;

/* CSG operators of a MODEL node (sdfModifiers.f90:428-491). */
typedef enum smcrt_csg_op {
  SMCRT_OP_UNION = 0,        /* min(d1,d2)                                   */
  SMCRT_OP_SMOOTH_UNION = 1, /* min(d1,d2) - h^3 k/6, h=max(k-|d1-d2|,0)/k   */
  SMCRT_OP_SUBTRACTION = 2,  /* max(-d1,d2)                                  */
  SMCRT_OP_INTERSECTION = 3  /* max(d1,d2)                                   */
} smcrt_csg_op;

/* One SDF node. The scene is a node table; `top` lists the top-level SDFs in the
 * reference's sdfs_array order (their index+1 is the reference "layer" index used by
 * tauint2's maxloc). A MODEL node folds its children nodes[first_child ..
 * first_child+n_children-1] left to right with `op` (eval_model, sdf_base.f90:146-161).
 * Optical properties are the reference `mono` inputs (opticalProperties.f90:107-125);
 * kappa/albedo/g2 are derived by the library exactly as init_mono does. For a MODEL the
 * reference uses its first child's properties (model_init, sdf_base.f90:133-134); the
 * builder is expected to copy them into the model node. */
typedef struct smcrt_sdf_node {
  int32_t kind;        /* smcrt_sdf_kind */
  int32_t layer;       /* sdf_base%layer: the reference ID (render/detector), not the array index */
  int32_t op;          /* smcrt_csg_op, MODEL only */
  int32_t first_child; /* MODEL only */
  int32_t n_children;  /* MODEL only */
  int32_t flags;       /* SMCRT_NODE_* (ABI 5; was reserved, 0 keeps init_mono's rules) */
  int32_t reserved[2];
  double transform[16]; /* Fortran t(4,4), column-major: transform[(c-1)*4+(r-1)] = t(r,c).
                           p = pos .dot. t (vector_class.f90:292-304) */
  double param[12];
  double k;            /* MODEL smoothing parameter */
  double mus, mua, hgg, n;
} smcrt_sdf_node;

/* smcrt_sdf_node.flags (ABI 5). */
#define SMCRT_NODE_ALBEDO_UNGUARDED 1 /* albedo = mus / kappa without init_mono's "albedo = 1 when
                                         mua < 1e-9" (updateSpectral, opticalProperties.f90:197-199) */

/* ----------------------------------------------------------------- grid ---------- */
/* cart_grid (grid.f90:14-25, init_grid_cart :119-159): voxel faces at (i-1)*2*max/n. */
typedef struct smcrt_grid {
  int32_t nx, ny, nz, reserved;
  double xmax, ymax, zmax; /* HALF extents */
} smcrt_grid;

/* ----------------------------------------------------------------- source -------- */
typedef enum smcrt_source_kind {
  SMCRT_SRC_POINT = 1,    /* isotropic point       photon.f90:311-359 (2 draws)          */
  SMCRT_SRC_UNIFORM = 2,  /* uniform parallelogram photon.f90:566-649 (2 draws)          */
  SMCRT_SRC_PENCIL = 3,   /* pencil beam           photon.f90:652-710 (0 draws)          */
  SMCRT_SRC_CIRCULAR = 4, /* uniform disc          photon.f90:214-308 (2 draws)          */
  SMCRT_SRC_FOCUS = 5,    /* focused beam          photon.f90:361-563 (2 draws)          */
  SMCRT_SRC_ANNULUS = 6,  /* annular beam          photon.f90:850-1043 (2, gaussian 2k+1) */
  SMCRT_SRC_SLM = 7,      /* image source          photon.f90:159-212 (2-D spectrum)     */
  SMCRT_SRC_DSLIT = 8,    /* double slit           photon.f90:712-780 (5 draws)          */
  SMCRT_SRC_APERTURE = 9  /* square aperture       photon.f90:782-848 (4 draws)          */
} smcrt_source_kind;

/* Beam profiles: focus_type (photon.f90:394-428) and annulus_type (:878-891). */
typedef enum smcrt_beam_kind {
  SMCRT_BEAM_GAUSSIAN = 0, /* focus: radius = beam_size*sqrt(-log(1-ran2)); annulus: rang(mid, sigma) */
  SMCRT_BEAM_SQUARE = 1,   /* focus only: x, y = ranu(-beam_size, beam_size)                          */
  SMCRT_BEAM_CIRCLE = 2,   /* focus only: radius = beam_size*sqrt(ran2)                               */
  SMCRT_BEAM_TOPHAT = 3,   /* annulus only: radius = sqrt(rlo^2 + (rhi^2-rlo^2)*ran2)                 */
  SMCRT_BEAM_BESSEL = 4    /* annulus only ("besselAnnulus"): radius = rlo + (rhi-rlo)*ran2           */
} smcrt_beam_kind;

/* Spectrum of a source (piecewise.f90, parse_spectrum.f90:52-117). Every source samples it
 * once per emission (`spectrum%p%sample`): a constant draws nothing, a 1-D spectrum one
 * ran2 (inverse CDF, trapezoid weights), a 2-D one (an image, sampled in Morton order) three.
 * The sampled wavelength only changes the geometry of the dslit and aperture sources; the
 * slm source takes its (x, y) from a 2-D spectrum. Arrays are host memory, read during
 * smcrt_run only. */
typedef enum smcrt_spectrum_kind {
  SMCRT_SPEC_CONSTANT = 0, /* piecewise.f90:93-107  (getValue)   */
  SMCRT_SPEC_1D = 1,       /* piecewise.f90:109-168 (sample1D)   */
  SMCRT_SPEC_2D = 2        /* piecewise.f90:171-236 (sample2D)   */
} smcrt_spectrum_kind;

typedef struct smcrt_spectrum {
  int32_t kind, reserved;
  double wavelength;         /* constant value (parse default 500.0) */
  int64_t n;                 /* 1-D: rows of array(n, 2) */
  const double* array;       /* 1-D: Fortran array(n,2): x = array[0..n), y = array[n..2n) */
  int32_t width, height;     /* 2-D: image(width, height), Fortran order (x fastest) */
  const double* image;
  double cell_width, cell_height; /* 2-D: piecewise2D cell_width / cell_height */
} smcrt_spectrum;

typedef struct smcrt_source {
  int32_t kind, reserved;
  double pos[3];  /* photon_origin%pos (point, pencil, circular, focus, annulus, slm) */
  double dir[3];  /* photon_origin%n{x,y,z}p (uniform, pencil, circular, slm) */
  double p1[3], p2[3], p3[3]; /* uniform: pos1 + r1*pos2 + r2*pos3 (photon.f90:596-612) */
  /* ---- ABI 2: the remaining sources of photon.f90 and the source spectrum ---- */
  int32_t beam;               /* smcrt_beam_kind: focus_type / annulus_type */
  int32_t reserved2;
  double radius;              /* circular */
  double beam_size;           /* focus */
  double focal_length;        /* focus, annulus: focalLength */
  double rlo, rhi, sigma;     /* annulus */
  double rotation[3];         /* focus, annulus: the [source] rotation vector (normalised by the emitter) */
  const smcrt_spectrum* spectrum; /* NULL: constant 500.0 (no draws) */
} smcrt_source;

/* ----------------------------------------------------------------- detectors ----- */
typedef enum smcrt_detector_kind {
  SMCRT_DET_CIRCLE = 1,  /* detectors.f90:147-164  */
  SMCRT_DET_ANNULUS = 2, /* detectors.f90:212-244  */
  SMCRT_DET_CAMERA = 3,  /* detectors.f90:401-469  */
  SMCRT_DET_FIBRE = 4    /* detectors.f90:246-393  */
} smcrt_detector_kind;

/* A constructed detector object (the fields the reference init_* functions set).
 * 1-D detectors own nbins doubles (nbins already includes the reference's extra bin,
 * init_circle_dect: out%nbins = nbins + 1); the camera owns nbins*nbins doubles laid
 * out data(idx, idy) -> idx-1 + nbins*(idy-1). */
typedef struct smcrt_detector {
  int32_t kind;
  int32_t nbins;       /* stored bin count (TOML nbins + 1) */
  int32_t layer;
  int32_t reserved;
  double pos[3];       /* circle/annulus/fibre: centre; camera: p1 (first corner) */
  double dir[3];       /* circle/annulus/fibre: surface normal; camera: n = normalised e2 x e1 */
  double e1[3], e2[3]; /* camera edge vectors */
  double radius;       /* circle */
  double r1, r2;       /* annulus */
  double width, height;/* camera */
  double bin_wid;      /* 1-D bin width (camera: bin_wid_x) */
  double bin_wid_y;    /* camera */
  double fibre[11];    /* focalLength1, focalLength2, f1Aperture, f2Aperture, frontOffset,
                          backOffset, frontToPinSep, pinToBackSep, pinAperture, acceptAngle,
                          coreDiameter */
} smcrt_detector;

/* ----------------------------------------------------------------- run ----------- */
enum {
  SMCRT_FLAG_PATHLENGTH = 1u << 0,    /* -Dpathlength: path-length jmean deposition (inttau2.f90:408-445) */
  SMCRT_FLAG_SURVIVAL_BIAS = 1u << 1, /* -DsurvivalBias: kernelsMod.f90:1979-2067 */
  SMCRT_FLAG_RENDER_SOURCE = 1u << 2, /* state%render_source: emission tally (kernelsMod.f90:1945) */
  SMCRT_FLAG_TEST_KERNEL = 1u << 3,   /* test_kernel semantics (kernelsMod.f90:2069-2182): no re-emission,
                                         initial layer mask ds<=0, scatter-order moments */
  SMCRT_FLAG_END_EARLY = 1u << 4,     /* test_kernel end_early: stop after the 4th scatter */
  SMCRT_FLAG_RECORD_PHOTONS = 1u << 5, /* fill smcrt_tallies.records (debug/parity) */
  SMCRT_FLAG_ASYNC_FOLD = 1u << 6,     /* smcrt_run_device: the jmean fold may finish after later work
                                          on the stream; jmean is complete after smcrt_scene_fence */
  SMCRT_FLAG_OVERLAP = 1u << 7         /* smcrt_run_device: launches rotate over up to four internal
                                          streams of the scene (two with SMCRT_SLOTS=2 or record pools
                                          above 24 GiB), each after the caller's earlier work, so launch k+1
                                          fills the GPU while launch k's slowest photons finish; every
                                          tally is complete in `stream` order only after
                                          smcrt_scene_fence (implies SMCRT_FLAG_ASYNC_FOLD) */
};

typedef struct smcrt_run_config {
  uint64_t n_photons;    /* photons in this call (int64: no int32 overflow, sim_state.f90:12) */
  uint64_t first_photon; /* global index of the first photon (multi-GPU shards, resume) */
  uint64_t seed;         /* state%iseed */
  uint32_t flags;        /* SMCRT_FLAG_* */
  int32_t reserved;
} smcrt_run_config;

/* Counter slots (uint64). Integer outputs: bit-exact between the HIP path and the CPU
 * restatement for the same seed. */
enum {
  SMCRT_CTR_PHOTONS = 0,      /* photons completed */
  SMCRT_CTR_EMIT_RETRIES,     /* re-emissions because the start cell was outside the grid */
  SMCRT_CTR_SCATTERS,         /* == nscatt */
  SMCRT_CTR_ABSORBED,         /* albedo roulette absorptions */
  SMCRT_CTR_SDF_EVALS,        /* packet%cnts equivalent (top-level SDF evaluations) */
  SMCRT_CTR_DEPOSITS,         /* jmean deposits (voxel crossings) */
  SMCRT_CTR_GRID_UPDATES,     /* update_grids calls */
  SMCRT_CTR_TAUINT,           /* tauint2 calls */
  SMCRT_CTR_FRESNEL,          /* reflect_refract calls */
  SMCRT_CTR_REFLECTIONS,      /* Fresnel reflections */
  SMCRT_CTR_BOUNCE_ABORTS,    /* bounces > 1000 early returns (inttau2.f90:313-315) */
  SMCRT_CTR_FAULTS,           /* would-be `error stop` events; photon terminated */
  SMCRT_CTR_RNG_DRAWS,        /* ran2() calls */
  SMCRT_CTR_DETECTOR_HITS,    /* detector bin increments */
  SMCRT_CTR_ESCAPED,          /* photons terminated by leaving the grid/geometry */
  SMCRT_CTR_WAVE_ITERS,       /* engine diagnostic: scheduler iterations summed over waves
                                 (no reference counterpart; launch-geometry dependent) */
  SMCRT_NCOUNTERS = 16
};

/* Per-photon record (SMCRT_FLAG_RECORD_PHOTONS), for trajectory-level parity checks. */
typedef struct smcrt_photon_record {
  double pos[3];   /* final packet%pos */
  double dir[3];   /* final direction */
  double weight;
  int32_t cell[3]; /* final packet%{x,y,z}cell (1-based, -1 outside) */
  int32_t layer;
  uint32_t nscatt;
  uint32_t bounces;
  uint32_t draws;  /* RNG draws consumed */
  uint32_t status; /* 1 absorbed, 2 escaped, 3 fault, 4 end_early */
} smcrt_photon_record;

/* Host tallies. Every pointer may be NULL (that tally is skipped). All accumulate.
 * fp32 grids keep the reference layout/type (iarray.f90:12-16); the engine sums in fp64
 * internally and adds the run's total into the float arrays once, at the end of the call.
 * The optional fp64 grids receive the same totals without the final rounding. */
typedef struct smcrt_tallies {
  float* jmean;      /* nx*ny*nz */
  float* absorb;     /* nx*ny*nz */
  float* emission;   /* nx*ny*nz */
  double* jmean_f64; /* nx*ny*nz */
  double* absorb_f64;
  double* emission_f64;
  double* det_bins;  /* concatenated detector data, in detector order */
  double* nscatt;    /* scalar */
  double* moments;   /* 24 doubles: [order 1..4][x,y,z] sums of pos, then of pos**2 (test_kernel) */
  uint64_t* counters;/* SMCRT_NCOUNTERS */
  smcrt_photon_record* records; /* n_photons entries, with SMCRT_FLAG_RECORD_PHOTONS */
} smcrt_tallies;

typedef struct smcrt_scene smcrt_scene;

/* ABI version of the loaded library (== SMCRT_ABI_VERSION it was built with). */
int smcrt_abi_version(void);
/* Number of visible HIP devices (0 is a valid answer; a negative status on error). */
int smcrt_device_count(int32_t* count);
/* Message for the last error on this thread ("" when none). */
const char* smcrt_last_error(void);

/* Upload a scene (SDF table, grid, detectors) to HIP device `device`. The scene stays
 * resident across smcrt_run calls (escape/inverse drivers reuse it, kernelsMod.f90:617,1642). */
int smcrt_scene_create(const smcrt_sdf_node* nodes, int32_t n_nodes,
                       const int32_t* top, int32_t n_top,
                       const smcrt_grid* grid,
                       const smcrt_detector* dets, int32_t n_dets,
                       int32_t device, smcrt_scene** out);
void smcrt_scene_destroy(smcrt_scene* scene);

/* The scene's fluence grid, number of top-level SDFs and of detectors (any may be NULL). */
int smcrt_scene_info(const smcrt_scene* scene, smcrt_grid* grid, int32_t* n_top, int32_t* n_dets);

/* Total doubles of detector data the scene's detectors own (size of det_bins). */
int smcrt_scene_det_bins(const smcrt_scene* scene, int64_t* n_doubles);

/* Replace the optical properties of top-level SDF `top_index` (updateOptProp,
 * sdf_base.f90:255-263; used by inverse MCRT). */
int smcrt_scene_set_optprops(smcrt_scene* scene, int32_t top_index,
                             double mus, double mua, double hgg, double n);

/* ---- ABI 5: spectral optical properties (opticalProperties.f90:127-201) -------------------
 * The reference's `spectral` type holds five piecewise1D tables (init_piecewise1D,
 * piecewise.f90:142-168; array(n, 2): x = wavelength, y = value) and derives mono-equivalent
 * properties from them: init_spectral when it is constructed, updateSpectral on each update.
 * No reference input file selects it and its run_MCRT never calls update, so a spectral layer
 * is a host-side sampler whose result is written into one top-level SDF's properties between
 * runs (smcrt_scene_set_spectral); the transport kernels see an ordinary layer.
 * Draws come from a host Philox4x32-10 stream keyed by `seed` (the reference's global ran2
 * stream cannot be reproduced): draw d is the (d & 1) half of block (d >> 1, 2, 0, 0xFFFFFFFF).
 * `*draw` is the caller's position in that stream; each sampled table takes one draw and
 * advances it, so successive updates continue the stream. */
typedef struct smcrt_spectral {
  int64_t n_mus, n_mua, n_hgg, n_n, n_flux; /* rows of each array(n, 2); every n >= 2 */
  const double* mus;  /* Fortran array(n, 2): x = a[0 .. n), y = a[n .. 2n) */
  const double* mua;
  const double* hgg;
  const double* n;
  const double* flux; /* the wavelength pdf */
} smcrt_spectral;

typedef enum smcrt_spectral_mode {
  /* init_spectral as documented (:141-155): a wavelength from the flux CDF (one draw), then
   * mus, mua, hgg and n interpolated at it (sample1D with value, piecewise.f90:132-137);
   * kappa = mus + mua, albedo = 1 when mua < 1e-9. */
  SMCRT_SPECTRAL_INIT = 0,
  /* updateSpectral (:171-201): the same draw and interpolation; albedo = mus / kappa with no
   * guard (out->node_flags = SMCRT_NODE_ALBEDO_UNGUARDED). */
  SMCRT_SPECTRAL_UPDATE = 1,
  /* init_spectral as compiled (:142-148): the properties are sampled with sample(x, y), i.e.
   * without a value, so each is an inverse-CDF draw of its own table's x axis (a wavelength),
   * one draw each after the flux's (five draws); `wave` is only passed as the unused y. */
  SMCRT_SPECTRAL_INIT_AS_WRITTEN = 2
} smcrt_spectral_mode;

typedef struct smcrt_optprops {
  double mus, mua, hgg, g2, n, kappa, albedo; /* opticalProp_base's fields */
  double wavelength;  /* the flux-sampled wavelength (updateSpectral's intent(out)) */
  int32_t node_flags; /* SMCRT_NODE_* that make a node derive kappa/albedo as above */
  int32_t reserved;
} smcrt_optprops;

/* Sample a spectral layer's properties. INVALID_ARG for a NULL table, n < 2 or a bad mode. */
int smcrt_spectral_sample(const smcrt_spectral* sp, int32_t mode, uint64_t seed, uint64_t* draw,
                          smcrt_optprops* out);

/* smcrt_spectral_sample, then write the result into top-level SDF `top_index` (mus, mua, hgg,
 * n and the node flags; like smcrt_scene_set_optprops). `out` may be NULL. */
int smcrt_scene_set_spectral(smcrt_scene* scene, int32_t top_index, const smcrt_spectral* sp, int32_t mode,
                             uint64_t seed, uint64_t* draw, smcrt_optprops* out);

/* Run cfg->n_photons photons (the body of run_MCRT) and accumulate into `io`.
 * Synchronous: returns when the tallies are in host memory. */
int smcrt_run(smcrt_scene* scene, const smcrt_source* src, const smcrt_run_config* cfg,
              smcrt_tallies* io);

/* Device-resident variant for multi-GPU and benchmarking: launches on `stream`
 * (a hipStream_t; NULL = the legacy default stream) and accumulates into caller-owned
 * DEVICE buffers (fp64 grids of nx*ny*nz, det bins, nscatt/moments/counters as in
 * smcrt_tallies; any may be NULL). Asynchronous: nothing is copied to the host.
 * The caller sums these buffers across ranks (one RCCL all-reduce per buffer). */
typedef struct smcrt_device_tallies {
  double* jmean;
  double* absorb;
  double* emission;
  double* det_bins;
  double* nscatt;
  double* moments;
  uint64_t* counters;
  smcrt_photon_record* records;
} smcrt_device_tallies;

int smcrt_run_device(smcrt_scene* scene, const smcrt_source* src, const smcrt_run_config* cfg,
                     smcrt_device_tallies* dev, void* stream);

/* Batched point sources: the inner loop of the escape function, which calls run_MCRT once
 * per launch cell with packet = photon("point") placed at the cell centre
 * (kernelsMod.f90:533-642, 959-1071). Photons [first_photon, first_photon + n_photons) of
 * EACH of the n_origins isotropic point sources at origins[3k..3k+2] run in one batched
 * launch; photon i of every origin uses Philox counter i, as every reference run_MCRT
 * restarts its streams from iseed (kernelsMod.f90:1850). `src` supplies the spectrum only
 * (NULL: constant). det_totals[k * n_dets + d] accumulates total_dect of detector d over
 * origin k's photons (detector_base.f90 total_1D/total_2D); io accumulates the tallies of
 * all origins (its det_bins are not written). SMCRT_FLAG_RECORD_PHOTONS is refused. */
int smcrt_run_origins(smcrt_scene* scene, const smcrt_source* src, const double* origins, int64_t n_origins,
                      const smcrt_run_config* cfg, double* det_totals, smcrt_tallies* io);

/* The top-level SDF holding each point, maxloc(ds, mask=ds<0) (0: outside every SDF), and
 * its kappa (0 when outside), evaluated on the scene's device: the launch-cell test of the
 * escape function (kernelsMod.f90:589-603). `kappa` may be NULL. */
int smcrt_scene_classify(smcrt_scene* scene, const double* points, int64_t n, int32_t* layer, double* kappa);

/* Make `stream` wait for every deposit fold in flight (SMCRT_FLAG_ASYNC_FOLD launches) and
 * every launch in flight on the internal streams (SMCRT_FLAG_OVERLAP): all tallies are
 * complete in `stream` order after this call. The fold of one launch then runs beside the
 * next launch's transport kernel (two record-log slots). */
int smcrt_scene_fence(smcrt_scene* scene, void* stream);

/* ABI 5: wait for every launch and fold of the scene (smcrt_run_device's asynchronous work) and
 * report the watchdog. Every cross-wave wait inside the kernels (a photon lane waiting for its
 * event, synchronous segment or slot; a producer waiting for a ring or event-queue word; a
 * deposit waiting for a bucket claim) is bounded by SMCRT_WATCHDOG_MS of wall clock (default
 * 2000; 0 = unbounded). A wait past it -- a lost wake-up, which would otherwise hang the GPU --
 * makes its block leave its loops and the grid drain; this call (and smcrt_run, which checks by
 * itself) then returns SMCRT_ERR_DEVICE_FAULT with the wait site and block in
 * smcrt_last_error(). The tallies of such a run are incomplete. */
int smcrt_scene_check(smcrt_scene* scene);

/* Per-kernel device time (ms) of the launches made since the previous query, from HIP
 * events recorded on the launch stream around each kernel group while timing is enabled
 * (off by default; no reference counterpart: it is the measurement hook of bench.py).
 * smcrt_scene_kernel_times waits for those launches to finish, then resets the sums. */
typedef struct smcrt_kernel_times {
  double transport_ms;  /* transport_kernel */
  double deposit_ms;    /* binned jmean fold: bin_hist .. bin_reduce */
  int64_t launches;     /* transport launches timed */
  int64_t lean_launches; /* of all launches since the last query (timed or not), those that ran
                            the lean path (ws_kernel: scenes of few tops without detectors or
                            survival bias) */
  int64_t far_steps;     /* march steps taken by the far-field march (long sphere-tracing runs with
                            only the nearest SDF re-evaluated) since the last query */
  double fold_cu_ms;     /* the deposit fold's own work since the last query: the sum of its reduce
                            workgroups' run times divided by the CU count (one workgroup fills a CU),
                            i.e. the whole-chip time it took, without the time it queued behind
                            transport launches (which deposit_ms includes) */
  /* ---- ABI 4 (the struct grew from 48 to 56 bytes) ---- */
  int64_t lean_hazards;  /* deferred lean-path voxel walks that ended in tflag or an
                            error stop since the last query. Each is also counted in SMCRT_CTR_FAULTS: the
                            photon went on as if the walk had stayed inside the grid, so it no longer
                            follows the reference. Expected 0; only the debug knob
                            SMCRT_DEBUG_LEAN_MARGIN=0|all (tests) provokes them. */
} smcrt_kernel_times;

int smcrt_scene_set_timing(smcrt_scene* scene, int32_t enable);
int smcrt_scene_kernel_times(smcrt_scene* scene, smcrt_kernel_times* out);

/* Normalisation of writer.f90:25-52 (normalise_fluence): grid *= nx*ny*nz / nphotons,
 * i.e. (8*xmax*ymax*zmax)/(nphotons*dx*dy*dz). Host-side helper on an fp32 grid. */
int smcrt_normalise_fluence(float* grid, const smcrt_grid* g, uint64_t nphotons);

/* ---- escape function (kernelsMod.f90:85-1460, the -DescapeFunction build) --------------
 * The reference runs run_MCRT once per launch cell of a symmetry grid (escapenphotons
 * photons from a point source at the cell centre), stores escapeSymmetry(d, cell) =
 * total_dect(d) / nphotons, fills the cells the symmetry implies, then interpolates onto
 * the fluence grid (escape(d, i, j, k)). Here every launch cell runs in ONE batched launch
 * on the resident scene (smcrt_run_origins). Both arrays are fp32 (iarray.f90:18), in
 * Fortran order with the detector index fastest. */
typedef enum smcrt_symmetry {
  SMCRT_SYM_NONE = 0,            /* every cell of the Cartesian symmetry grid        :177-213 */
  SMCRT_SYM_PRISM = 1,           /* the z layer holding (0,0,0), copied to all z     :215-265 */
  SMCRT_SYM_FLIPPED = 2,         /* z cells 1..nz/2+1, mirrored in z                 :267-316 */
  SMCRT_SYM_UNIFORM_SLAB = 3,    /* the column holding (0,0,0), copied to all x, y   :318-363 */
  SMCRT_SYM_NONE_ROTATIONAL = 4, /* every (r, theta, z) cell of the cylindrical grid :365-411 */
  SMCRT_SYM_ROTATIONAL_360 = 5   /* theta cell 1 only, copied to every theta         :413-453 */
} smcrt_symmetry;

typedef struct smcrt_escape_config {  /* [symmetry] table, parse.f90:188-340 */
  int32_t symmetry;  /* smcrt_symmetry (symmetryType) */
  int32_t n[3];      /* GridSize: nx, ny, nz (Cartesian) or nr, ntheta, nz (cylindrical) */
  double max[3];     /* maxValues: xmax, ymax, zmax, or rmax, (unused: tmax = 2 pi), zmax */
  double pos[3];     /* position: the symmetry grid's centre (symGridPos) */
  double dir[3];     /* direction: its z axis (symGridDir), normalised by the callee */
  double rotation;   /* rotation about that axis in degrees, [0, 360) (symGridRot) */
} smcrt_escape_config;

/* Symmetry-grid dimensions (n0, n1, n2) of escapeSymmetry. Host only. */
int smcrt_escape_sym_dims(const smcrt_escape_config* cfg, int32_t dims[3]);

/* Launch cells in the reference's loop order: 1-based symmetry-grid indices (3 per cell) and
 * emission positions (the cell centre taken off the symmetry grid: rotate about z, align z
 * with `dir`, shift by `pos`; kernelsMod.f90:566-577, 1004-1021). Either output may be NULL
 * (n_cells is always set). Host only. */
int smcrt_escape_cells(const smcrt_escape_config* cfg, int64_t* n_cells, int32_t* cells, double* positions);

/* escapeSymmetry -> escape on `grid` (cart_map_escape_sym :644-957 / cyl_map_escape_sym
 * :1073-1460: tri/bi/linear interpolation, area weights in cylindrical cells, -1 outside the
 * symmetry grid). escape_sym: n_dets*n0*n1*n2, escape: n_dets*nx*ny*nz. Host only. */
int smcrt_escape_map(const smcrt_escape_config* cfg, const smcrt_grid* grid, int32_t n_dets, const float* escape_sym,
                     float* escape);

/* The escape function on a resident scene: cells -> smcrt_scene_classify (cells outside
 * every SDF or in a kappa = 0 layer keep 0 and are not run) -> one smcrt_run_origins with
 * run->n_photons per cell -> escapeSymmetry = total / n_photons -> symmetry fill ->
 * smcrt_escape_map. io accumulates the tallies of every cell's photons, as the reference's
 * jmean does over its run_MCRT calls. Either output array may be NULL. */
int smcrt_escape_run(smcrt_scene* scene, const smcrt_source* src, const smcrt_escape_config* cfg,
                     const smcrt_run_config* run, float* escape_sym, float* escape, smcrt_tallies* io);

/* ---- inverse MCRT (kernelsMod.f90:1462-1787, the -DinverseMCRT build) ------------------
 * The reference draws maxNumSteps random guesses of the searched optical properties of one
 * layer (AdaLIPO's explore stage; the exploit branch is unreachable, :1620), runs run_MCRT
 * for each and scores it with inverse_evaluate (:1753-1787): -mean |total_dect/nphotons -
 * inverseTarget| over the detectors with a target (/= -1). Here the scene stays resident on
 * the GPU across the steps. */
enum {
  SMCRT_INVERSE_FIND_MUS = 1u << 0,  /* Findmus */
  SMCRT_INVERSE_FIND_MUA = 1u << 1,  /* Findmua */
  SMCRT_INVERSE_FIND_G = 1u << 2,    /* Findg   */
  SMCRT_INVERSE_FIND_N = 1u << 3,    /* Findn   */
  /* Apply each guess to the layer before its run. The reference builds the trial property
   * from the layer's ORIGINAL values (mono(mus, mua, hgg, n), :1630-1631), so every step
   * reruns the same scene; without this flag that behaviour is kept. */
  SMCRT_INVERSE_APPLY_TRIAL = 1u << 4
};

typedef struct smcrt_inverse_config {  /* [inverse] table, parse.f90:343-413 */
  int32_t layer;      /* layer: the first top-level SDF with this layer id is searched */
  int32_t flags;      /* SMCRT_INVERSE_* */
  int32_t max_steps;  /* maxNumSteps */
  int32_t reserved;
  double max_step_size, grad_step_size, accuracy;  /* parsed; unused by the reference's search */
  uint64_t seed;      /* stream of the guesses (the reference draws them from its global ran2) */
} smcrt_inverse_config;

/* The top-level SDF's layer id and optical properties as the reference's getters return
 * them (sdf_base.f90:192-269; mus = getKappa() - getMua()). Any output may be NULL. */
int smcrt_scene_get_optprops(const smcrt_scene* scene, int32_t top_index, int32_t* layer, double* mus, double* mua,
                             double* hgg, double* n);

/* inverse_MCRT on a resident scene. targets[d] = inverseTarget of detector d (-1: none).
 * steps: max_steps*5 doubles, gradDescentData(maxNumSteps, 5) in Fortran order: guesses of
 * mus, mua, g, n then the error of step i at steps[(c-1)*max_steps + (i-1)]. run->n_photons
 * photons per step, each step from photon first_photon (the reference reseeds every
 * run_MCRT). The layer's original properties are restored at the end. A step whose
 * properties repeat an earlier step's bits reuses that step's error (runs are deterministic),
 * so the reference's mode costs two runs when io is NULL. With io (may be NULL) every step
 * runs and io accumulates all max_steps runs, as the reference's jmean does. */
int smcrt_inverse_run(smcrt_scene* scene, const smcrt_source* src, const smcrt_inverse_config* cfg,
                      const smcrt_run_config* run, const double* targets, double* steps, smcrt_tallies* io);

/* ---- multi-GPU: photon shards + ONE packed RCCL reduction (SURVEY §8(b) n_gpus, §8(e)) --
 * The reference splits `do j = 1, nphotons` statically over OpenMP threads
 * (kernelsMod.f90:1859) and means to sum the tallies onto the root with mpi_reduce
 * (kernelsMod.f90:2351-2357). Here photon index ranges are split over GPUs; since a photon's
 * Philox stream is keyed by its global index, N GPUs compute exactly the photons one GPU
 * would. The only exchange is one reduction of a packed fp64 buffer per run, over RCCL
 * (xGMI between the GPUs of a node). RCCL (librccl.so.1) is loaded on first use; without it
 * these calls return SMCRT_ERR_RCCL.
 *
 * Packed layout (fp64 elements, in this order; a grid or the detector block is present only
 * when its bit is set in `fields`, the scalar block always):
 *   jmean[n_voxels] | absorb[n_voxels] | emission[n_voxels] | det_bins[n_det_bins] |
 *   nscatt | moments[24] | counters[SMCRT_NCOUNTERS]
 * Counters travel as doubles: exact while every total stays below 2^53. */
enum {
  SMCRT_PACK_JMEAN = 1u << 0,
  SMCRT_PACK_ABSORB = 1u << 1,
  SMCRT_PACK_EMISSION = 1u << 2,
  SMCRT_PACK_DET_BINS = 1u << 3
};
typedef struct smcrt_pack_layout {
  int64_t n_voxels;    /* nx*ny*nz */
  int64_t n_det_bins;  /* smcrt_scene_det_bins */
  uint32_t fields;     /* SMCRT_PACK_* */
  int32_t reserved;
} smcrt_pack_layout;

/* Doubles in a packed buffer of this layout. Host only. */
int smcrt_pack_size(const smcrt_pack_layout* layout, int64_t* n_doubles);
/* Host tallies -> packed buffer (grids from the fp64 arrays when given, else from the fp32
 * ones; a NULL tally packs zeros). Host only. */
int smcrt_pack_host(const smcrt_pack_layout* layout, const smcrt_tallies* t, double* buf);
/* Packed buffer -> host tallies, ACCUMULATED like smcrt_run's (fp32 grids get
 * (float)((double)old + value)). Host only. */
int smcrt_unpack_host(const smcrt_pack_layout* layout, const double* buf, smcrt_tallies* t);

/* One process per GPU (torchrun / mpirun): rank 0 makes an id and hands it to every rank
 * (out of band); each rank then joins on its device. */
#define SMCRT_UNIQUE_ID_BYTES 128
typedef struct smcrt_comm smcrt_comm;
int smcrt_comm_unique_id(uint8_t* id /* SMCRT_UNIQUE_ID_BYTES */);
int smcrt_comm_init_rank(const uint8_t* id, int32_t n_ranks, int32_t rank, int32_t device, smcrt_comm** out);
void smcrt_comm_destroy(smcrt_comm* comm);
/* ABI 4: the communicator's rank count and this rank as RCCL reports them (ncclCommCount,
 * ncclCommUserRank), and its device (any output may be NULL). */
int smcrt_comm_info(const smcrt_comm* comm, int32_t* n_ranks, int32_t* rank, int32_t* device);
/* Sum every rank's device tallies (smcrt_run_device's buffers) over `comm` with ONE packed
 * collective on `stream`: an all-reduce when root < 0 (every rank gets the sums), else a
 * reduce onto rank `root` (the mpi_reduce of kernelsMod.f90:2353-2357; the other ranks'
 * buffers are left as they were). The fields are the non-NULL pointers of `dev` (records are
 * not reduced); every rank must pass the same set. Asynchronous on `stream`. */
int smcrt_reduce_device_tallies(smcrt_scene* scene, smcrt_comm* comm, smcrt_device_tallies* dev, int32_t root,
                                void* stream);

/* One process, several GPUs: smcrt_run with n_gpus. smcrt_multi_create
 * uploads the scene to each of `devices` (NULL: devices 0 .. n_devices-1; n_devices <= 0:
 * every visible device) and gives each device resident fp64 accumulators.
 * smcrt_multi_accumulate runs photons [first, first + N) in chunks handed to whichever device
 * has a free launch slot (overlapped launches, nothing waited for); smcrt_multi_collect sums
 * every device's accumulators onto the first device with ONE packed RCCL reduce, adds them
 * into `io` as smcrt_run does and zeroes the accumulators. A job split into batches therefore
 * pays one collective when it collects (per checkpoint, or once), not one per batch.
 * If a launch fails inside smcrt_multi_accumulate, everything accumulated since the last
 * collect is discarded (the devices are fenced, the accumulators zeroed) and the error is
 * returned, so a later collect never sums partial tallies; smcrt_multi_device_photons tells
 * how many photons the accumulators hold.
 * smcrt_multi_run = accumulate + collect. Results do not depend on the number of devices or
 * on which device ran which chunk (up to the fp64 summation order of jmean); counters and
 * integer tallies are exact. Photon records are refused (use smcrt_run). */
typedef struct smcrt_multi smcrt_multi;
int smcrt_multi_create(const smcrt_sdf_node* nodes, int32_t n_nodes, const int32_t* top, int32_t n_top,
                       const smcrt_grid* grid, const smcrt_detector* dets, int32_t n_dets,
                       const int32_t* devices, int32_t n_devices, smcrt_multi** out);
int smcrt_multi_info(const smcrt_multi* multi, int32_t* n_devices);
/* The scene on device slot i (0 <= i < n_devices), e.g. for smcrt_scene_set_optprops. */
smcrt_scene* smcrt_multi_scene(smcrt_multi* multi, int32_t i);
int smcrt_multi_run(smcrt_multi* multi, const smcrt_source* src, const smcrt_run_config* cfg, smcrt_tallies* io);
int smcrt_multi_accumulate(smcrt_multi* multi, const smcrt_source* src, const smcrt_run_config* cfg);
int smcrt_multi_collect(smcrt_multi* multi, smcrt_tallies* io);
/* Photons each device ran since the last collect (n_devices entries; load-balance diagnostic). */
int smcrt_multi_device_photons(const smcrt_multi* multi, uint64_t* photons);
void smcrt_multi_destroy(smcrt_multi* multi);

/* ---- output formats (src/writer.f90), host-side, no GPU needed ------------------------
 * Written byte for byte as the reference writes them, so its readers
 * (tools/read_nrrd_class.py, tools/plotDetectorsClass.py) load them unchanged. If the
 * target exists and `overwrite` is 0, " (i)" is inserted before the extension
 * (get_new_file_name, writer.f90:273-291); the name used is copied to `written_path`
 * (may be NULL) when it fits in `path_cap` bytes. */

/* write_data (writer.f90:162-226) for an fp32 / fp64 volume of nx*ny*nz values in Fortran
 * order, chosen by extension:
 *   .nrrd: NRRD0004 header (write_hdr :300-327; "sizes: nz ny nx"), the optional `metadata`
 *          text (the reference's toml_dump of its dict), a blank line, then the raw data;
 *   .raw / .dat: the raw data only (write_3d_r4_raw / _r8_raw :228-271);
 *   anything else: SMCRT_ERR_UNSUPPORTED ("File type not supported!").
 * `dect_id` (may be NULL) adds the "dector: <ID>" line of the escape-function files. */
int smcrt_write_data_f32(const char* filename, const float* array, int32_t nx, int32_t ny, int32_t nz,
                         const char* metadata, const char* dect_id, int32_t overwrite,
                         char* written_path, int32_t path_cap);
int smcrt_write_data_f64(const char* filename, const double* array, int32_t nx, int32_t ny, int32_t nz,
                         const char* metadata, const char* dect_id, int32_t overwrite,
                         char* written_path, int32_t path_cap);

/* write_detected_photons (writer.f90:55-138) for one detector: an fp64 stream of type
 * (1 circle, 2 fibre, 3 annulus), len(ID), the ID characters, nphotons, the geometry, then
 * (bin centre, value) for each of d->nbins bins. A camera gives an empty file, as in the
 * reference. The file is replaced if it exists (status='REPLACE'). */
int smcrt_write_detector(const char* filename, const smcrt_detector* d, const double* data,
                         const char* id, int64_t nphotons);

/* checkpoint (writer.f90:419-455): "tomlfile=<toml_filename>", "photons_run=<n>", then
 * jmean (fp32, nx*ny*nz, Fortran order) raw. */
int smcrt_write_checkpoint(const char* filename, const char* toml_filename, int64_t photons_run,
                           const float* jmean, const smcrt_grid* g, int32_t overwrite,
                           char* written_path, int32_t path_cap);

/* ---- TOML front end (src/parse/parse*.f90, src/setup.f90, src/setupGeometry.f90) --------
 * smcrt_job_load reads a res/<name>.toml file with the reference's keys, defaults and error
 * messages. It builds the scene the way setup_simulation does and keeps the output and
 * simulation settings.
 *   Geometries: sphere, box, test_box, scat_test, scat_test2, aptran, sphere_scene, exp, omg,
 *     egg (ABI 4: revolution modifiers), vessels (get_vessels, setupGeometry.f90:552-652:
 *     edges.dat, nodes.dat and radii.dat are read from the input file's directory, the
 *     reference's res/; a missing file is SMCRT_ERR_INVALID_ARG naming it). logo (the
 *     reference stops on it, setupGeometry.f90:326-328) returns SMCRT_ERR_UNSUPPORTED.
 *   Sources: point, uniform, pencil; a constant spectrum.
 *   Detectors: circle, annulus, camera, grouped by type as parse_detectors does.
 * Build-defined: sphere_scene's sphere list, which the reference draws from an unseeded
 * compiler RNG (setupGeometry.f90:285-292). Here draw d is Philox4x32-10 of counter
 * (d, 0x5350, 0, 0) under key iseed. */
typedef struct smcrt_job smcrt_job;

typedef struct smcrt_job_desc {
  int64_t n_photons;  /* [source] nphotons */
  int64_t seed;       /* [simulation] iseed */
  int32_t flags;      /* SMCRT_FLAG_PATHLENGTH | RENDER_SOURCE as configured */
  int32_t n_nodes, n_top, n_dets;
  int32_t overwrite;  /* [output] overwrite */
  smcrt_grid grid;
  smcrt_source source;
  char experiment[64];  /* geom_name */
  char source_name[32];
} smcrt_job_desc;

int smcrt_job_load(const char* toml_path, smcrt_job** out);
/* The reference's build variants parse one more table (parse.f90:64-70): SMCRT_JOB_ESCAPE
 * reads [symmetry] (its escapenphotons replaces nphotons; symmetryType joins the metadata),
 * SMCRT_JOB_INVERSE reads [inverse] (an error if absent). smcrt_job_load = DEFAULT. */
enum { SMCRT_JOB_DEFAULT = 0, SMCRT_JOB_ESCAPE = 1, SMCRT_JOB_INVERSE = 2 };
int smcrt_job_load_mode(const char* toml_path, int32_t mode, smcrt_job** out);
void smcrt_job_destroy(smcrt_job* job);
int smcrt_job_info(const smcrt_job* job, smcrt_job_desc* desc);
/* Copies the flattened scene (desc.n_nodes nodes, desc.n_top top-level indices) and the
 * detectors (desc.n_dets) into caller arrays. */
int smcrt_job_scene(const smcrt_job* job, smcrt_sdf_node* nodes, int32_t* top, smcrt_detector* dets);
/* The metadata dict (the values parse_* and finalise set) as TOML text, for NRRD headers. */
int smcrt_job_metadata(const smcrt_job* job, char* buf, int32_t cap);
/* default_MCRT (kernelsMod.f90:14-82): run_MCRT on `device` (SMCRT_ALL_DEVICES: every
 * visible GPU through smcrt_multi_run), then finalise (:2321-2416).
 * Photons run in batches of checkpoint_every_n; after each, <checkpoint_file> is rewritten
 * with the tally of the photons done so far (writer.f90:426-457). With load_checkpoint,
 * <checkpoint_file> is read back, and its input file (next to this one) is run for its
 * remaining photons with iseed*101 from zeroed tallies, as the reference's second setup()
 * leaves it. A relative <checkpoint_file> is taken relative to outdir for both the write
 * and the read (the reference uses one CWD-relative name for both, kernelsMod.f90:54,1863).
 * Writes, under outdir (the reference's fileplace):
 *   jmean/<fluence>, normalised;
 *   emission/<render_source_name>, normalised;
 *   absorb/absorb.nrrd;
 *   detectors/detector_<i>.dat.
 * `nscatt` (may be NULL) receives the total scatter count. */
#define SMCRT_ALL_DEVICES (-1)
int smcrt_job_run(smcrt_job* job, int32_t device, const char* outdir, double* nscatt);
/* smcrt_job_run over an explicit list of GPUs (photon shards + one RCCL reduce per batch). */
int smcrt_job_run_devices(smcrt_job* job, const int32_t* devices, int32_t n_devices, const char* outdir,
                          double* nscatt);

/* The parsed [symmetry] / [inverse] tables and the detectors' inverseTarget values
 * (parse_detectors.f90:102, -1 when absent; desc.n_dets of them). */
int smcrt_job_escape_config(const smcrt_job* job, smcrt_escape_config* out);
int smcrt_job_inverse_config(const smcrt_job* job, smcrt_inverse_config* out);
int smcrt_job_targets(const smcrt_job* job, double* targets);
/* escape_Function (kernelsMod.f90:85-530): smcrt_escape_run, then write_escape
 * (writer.f90:136-166: escape/dectID_<ID>__escape<i>.nrrd on the fluence grid and
 * __escapeSym<i>.nrrd on the symmetry grid, with a "dector: <ID>" header line), then
 * finalise as smcrt_job_run (detector files hold zero bins: the reference's mapping resets
 * the detectors). */
int smcrt_job_run_escape(smcrt_job* job, int32_t device, const char* outdir);
/* inverse_MCRT (kernelsMod.f90:1462-1751) on `device`: steps = gradDescentData(maxNumSteps, 5)
 * (see smcrt_inverse_run). Writes no files, as the reference. */
int smcrt_job_run_inverse(smcrt_job* job, int32_t device, int32_t apply_trial, double* steps);

#ifdef __cplusplus
}
#endif
#endif /* SMCRT_H */
