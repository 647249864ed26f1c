/*
 * mph_gpu.h -- C ABI of the MI355X-native MPH explicit hot path (libmph_gpu.so).
 *
 * Drop-in boundary for the reference solver Ryo1011gd/ParticleMethod_FSI (src/main.cpp).
 * The reference has no plugin/FFI layer: its hot path is a set of `static void calculateX(void)`
 * functions over file-scope globals (main.cpp:200-241) called in a fixed order by main()
 * (main.cpp:581-688).  This header replaces that whole layer with a context object:
 *
 *   reference                                              | this ABI
 *   -------------------------------------------------------+--------------------------------------
 *   readDataFile          main.cpp:729-786                 | mph_read_data_file
 *   readGridFile          main.cpp:788-955                 | mph_read_grid_header/_particles
 *   initializeWeight/Fluid/Wall/Domain main.cpp:534-537,    | mph_create  (derives every constant,
 *     1191-1469; acc update device main.cpp:549-560;       |   uploads, builds the structure
 *     calculateInitialNeighbor/Neighbor/DensityA/          |   Lagrangian lists and normalizer,
 *     GravityCenter/DensityP/Lamesconstant/Normalizer      |   runs the init sums)
 *     main.cpp:564-570                                     |
 *   one iteration of the time loop main.cpp:597-686       | mph_step(ctx, 1)
 *   acc update host main.cpp:987-989 + array reads         | mph_get
 *   writeProfFile main.cpp:957-982                         | mph_write_prof
 *   writeVtkFile  main.cpp:984-1189                        | mph_write_vtk
 *   err_malloc/err_fopen exit(1) errorfunc.cpp:8-31        | negative MphStatus + mph_last_error
 *
 * Data at the boundary is the reference's own layout (vec3T.hpp:31-34 / main.cpp:105-197):
 * AoS double[n][3] for vectors, row-major double[n][3][3] for tensors, int[n] for ints, always in
 * the ORIGINAL particle order of the .grid file.  Internally the device keeps a cell-sorted
 * struct-of-arrays copy and a permutation; nothing of that leaks through this header.
 *
 * Threading: one host thread per context; several contexts may coexist (no global state).
 * mph_step is stream-ordered; mph_get/mph_write_* synchronise.
 */
#ifndef MPH_GPU_H_INCLUDED
#define MPH_GPU_H_INCLUDED

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPH_TYPE_COUNT 6            /* main.cpp:68 */
#define MPH_MAX_NEIGHBOR_COUNT 512  /* main.cpp:100 (semantic limit; overflow is an error here) */
/* Bumped on every incompatible change of a declaration below (3: mph_slab_bounds/_owner/_window
 * take `cuts`; mph_dist_info slot 0/2 meaning); bindings compare mph_abi_version() with it.     */
#define MPH_ABI_VERSION 4

/* Compile-time case modules of the reference (main.cpp:54-59) as a runtime switch.  The module
 * selects the clamp rule of updateElasticPosition (main.cpp:1918-2044).                        */
typedef enum MphModule {
    MPH_MODULE_BAR = 0,          /* Bar_Module: x0.x < 0.001 clamped, force zeroed   (1918-1943) */
    MPH_MODULE_DAM = 1,          /* DAM_Module: x0.y < 0.002 clamped, force zeroed   (1967-1992) */
    MPH_MODULE_TUREK_HRON = 2,   /* Turek_Hron: x0.x < 0.205 clamped                 (1944-1966) */
    MPH_MODULE_ROLLING1 = 3,     /* Rolling1:   x0.y < 0.003 clamped, force zeroed   (1993-2018) */
    MPH_MODULE_HYDROELASTIC = 4, /* Hydroelastic: x0.x<0.01||>1.99, force zeroed     (2019-2044) */
    MPH_MODULE_NONE = 5          /* no clamp (only the unconditional drift of 2070-2079)          */
} MphModule;

/* calculateWall (main.cpp:2963-3072): the shipped rigid motion (the `#else` branch 3031-3071:
 * rotation WallRotation + translation WallVelocity while Time < 0.2) or the compile-time
 * `Rolling` branch (2974-3030: every step the walls turn about z through WallCenter by
 * dtheta = MAX_ANGLE [sin(w t) - sin(w (t - Dt))], w = 2 pi / ROLLING_PERIOD, main.cpp:2959-2960). */
typedef enum MphWallMotion {
    MPH_WALL_RIGID = 0,
    MPH_WALL_ROLLING = 1
} MphWallMotion;

typedef enum MphStatus {
    MPH_OK = 0,
    MPH_ERR_ARG = -1,
    MPH_ERR_IO = -2,
    MPH_ERR_NEIGHBOR_OVERFLOW = -3,  /* a particle found >= 512 neighbours (main.cpp:1766-1768) */
    MPH_ERR_DEVICE_OOM = -4,
    MPH_ERR_HIP = -5,
    MPH_ERR_RCCL = -6,
    MPH_ERR_DOMAIN = -7,             /* domain too small for the cell stencil        */
    MPH_ERR_UNSUPPORTED = -8,
    MPH_ERR_NONFINITE = -9,
    MPH_ERR_TRANSPORT = -10,         /* slab mode: host exchange callback failed                  */
    MPH_ERR_CAPACITY = -11           /* slab mode: local arrays full, or a particle jumped a slab */
} MphStatus;

/* Everything the reference reads from its .data file (main.cpp:743-767) and .grid header
 * (main.cpp:797-804), plus the two compile-time switches.  All derived constants (radii, kernel
 * normalisations, N0a/N0p, CofA, cell grid, wall rotations ...) are computed inside mph_create
 * exactly as initializeWeight/Fluid/Wall/Domain do.                                             */
typedef struct MphConfig {
    int    dim;                       /* 2 or 3: TWO_DIMENSIONAL main.cpp:50 */
    int    module;                    /* MphModule */
    double dt;                        /* Dt */
    double elastic_dt;                /* ElasticDt */
    double output_interval;           /* OutputInterval */
    double vtk_output_interval;       /* VtkOutputInterval */
    double end_time;                  /* EndTime */
    double radius_ratio_a;            /* RadiusRatioA (RadiusRatioG = RadiusRatioA, main.cpp:1193) */
    double radius_ratio_p;            /* RadiusRatioP */
    double radius_ratio_v;            /* RadiusRatioV */
    double density[MPH_TYPE_COUNT];
    double bulk_modulus[MPH_TYPE_COUNT];
    double bulk_viscosity[MPH_TYPE_COUNT];
    double shear_viscosity[MPH_TYPE_COUNT];
    double surface_tension[MPH_TYPE_COUNT];   /* .data gives types 0,1,4,5 (main.cpp:756) */
    double young_modulus[MPH_TYPE_COUNT];     /* .data gives types 2..5     (main.cpp:757) */
    double poisson_ratio[MPH_TYPE_COUNT];     /* .data gives types 2..5     (main.cpp:758) */
    double interaction_ratio[MPH_TYPE_COUNT][MPH_TYPE_COUNT];
    double gravity[3];
    double wall_center[MPH_TYPE_COUNT][3];    /* only Wall6/Wall7 -> types 4/5 are parsed (766-767) */
    double wall_velocity[MPH_TYPE_COUNT][3];
    double wall_omega[MPH_TYPE_COUNT][3];
    double time;                      /* .grid line 1 (restart time) */
    double particle_spacing;          /* .grid line 2 */
    double domain_min[3];
    double domain_max[3];
    int    wall_motion;               /* MphWallMotion (compile-time `Rolling`, main.cpp:58) */
} MphConfig;

/* sizeof(MphConfig) as compiled into the library (FFI bindings check their mirror against it). */
int mph_config_sizeof(void);
/* MPH_ABI_VERSION as compiled into the library.                                              */
int mph_abi_version(void);

/* Per-particle arrays readable with mph_get (original particle order). */
typedef enum MphField {
    MPH_FIELD_POSITION = 0,           /* double[n][3] */
    MPH_FIELD_INITIAL_POSITION = 1,   /* double[n][3] */
    MPH_FIELD_VELOCITY = 2,           /* double[n][3] */
    MPH_FIELD_FORCE = 3,              /* double[n][3] */
    MPH_FIELD_ACCELERATION = 4,       /* double[n][3] */
    MPH_FIELD_GRAVITY_CENTER = 5,     /* double[n][3] */
    MPH_FIELD_PRESSURE_P = 6,         /* double[n] */
    MPH_FIELD_PRESSURE_A = 7,         /* double[n] */
    MPH_FIELD_DENSITY_A = 8,          /* double[n] */
    MPH_FIELD_VOL_STRAIN_P = 9,       /* double[n] */
    MPH_FIELD_DIVERGENCE_P = 10,      /* double[n] */
    MPH_FIELD_MASS = 11,              /* double[n] */
    MPH_FIELD_KAPPA = 12,             /* double[n] */
    MPH_FIELD_LAMBDA = 13,            /* double[n] */
    MPH_FIELD_MU = 14,                /* double[n] */
    MPH_FIELD_NEIGHBOR_COUNT = 15,    /* int[n] */
    MPH_FIELD_INITIAL_STRUCTURE_NEIGHBOR_COUNT = 16, /* int[n] */
    MPH_FIELD_PROPERTY = 17,          /* int[n] */
    MPH_FIELD_DEFORM_GRADIENT = 18,   /* double[n][3][3] */
    MPH_FIELD_STRAIN = 19,            /* double[n][3][3] */
    MPH_FIELD_STRESS = 20,            /* double[n][3][3] */
    MPH_FIELD_NORMALIZER = 21,        /* double[n][3][3] */
    MPH_FIELD_LAMBDA_LAMES = 22,      /* double[n] */
    MPH_FIELD_MU_LAMES = 23,          /* double[n] */
    MPH_FIELD_VIRIAL_STRESS = 24,     /* double[n][3][3], VirialStressAtParticle (mph_compute_virial) */
    MPH_FIELD_VIRIAL_PRESSURE = 25,   /* double[n], VirialPressureAtParticle (mph_compute_virial) */
    MPH_FIELD_COUNT = 26
} MphField;

typedef struct MphCtx MphCtx;

/* ---- host-side file formats (no device needed) ------------------------------------------- */

/* Fill cfg with the reference's static defaults (zeros, Dt=ElasticDt=1e100) for dim/module. */
int mph_config_default(MphConfig* cfg, int dim, int module);
/* .data keyword file, main.cpp:729-786.  Unknown lines are ignored like the reference.      */
int mph_read_data_file(const char* path, MphConfig* cfg);
/* .grid / .prof header (Time; N dx xmin xmax ymin ymax zmin zmax), main.cpp:796-804.
 * Both readers also accept the binary grid of mph_write_grid_binary (detected by its magic).  */
int mph_read_grid_header(const char* path, MphConfig* cfg, int* n);
/* .grid / .prof body: n lines "type x y z x0 y0 z0 vx vy vz", main.cpp:896-904.             */
int mph_read_grid_particles(const char* path, int n, int* property, double* pos, double* pos0,
                            double* vel);
/* Binary grid (the input-path variant of SURVEY 8f: the ASCII .grid of a 16M-particle case is
 * 2 GB and takes the generator 33 s): magic "MPHGRIDB", int32 version 1, int32 n, double time,
 * dx, domain_min[3], domain_max[3], then int32 property[n] (zero-padded to 8 bytes) and
 * double position[n][3], initial_position[n][3], velocity[n][3], little endian.  The values
 * are stored exactly (no %e rounding).                                                        */
int mph_write_grid_binary(const char* path, const MphConfig* cfg, int n, const int* property,
                          const double* pos, const double* pos0, const double* vel);
/* .prof writer with the reference's exact format, main.cpp:957-982.                          */
int mph_write_prof_arrays(const char* path, const MphConfig* cfg, double time, int n,
                          const int* property, const double* pos, const double* pos0,
                          const double* vel);
/* legacy-ASCII .vtk writer with the reference's exact format, main.cpp:984-1189.            */
int mph_write_vtk_arrays(const char* path, int n, const int* property, const double* pos,
                         const double* pos0, const double* vel, const double* accel,
                         const double* force, const double* stress, const double* strain,
                         const int* initial_structure_neighbor_count, const int* neighbor_count);

/* Binary VTK XML (.vtu) alternative to the ASCII writer: the same point fields as
 * mph_write_vtk_arrays, Float32/Int32 in raw appended data (UInt64 headers), stress and strain as
 * 9-component tensors, one VTK_VERTEX cell per particle.                                       */
int mph_write_vtu_arrays(const char* path, int n, const int* property, const double* pos,
                         const double* pos0, const double* vel, const double* accel,
                         const double* force, const double* stress, const double* strain,
                         const int* initial_structure_neighbor_count, const int* neighbor_count);

/* setInitialVelocityProfile (main.cpp:395-441) on host arrays (original order; vel is updated in
 * place).  Bar_Module: the beam's first bending mode on the structure particles, v = (0,
 * 0.01 c0 f(x0)/f(L), 0) with c0 = sqrt(3.25e6/Density) and f of main.cpp:387-392 (the
 * reference's only call, main.cpp:571, is commented out: an explicit option).  Turek_Hron: the
 * parabolic inlet on fluid particles with x <= 0.01 and, while time < 0.7, x > 1.5 -- the
 * reference calls it every step before calculateWall (main.cpp:592-594), which mph_step does on
 * the device by itself for MPH_MODULE_TUREK_HRON.  Other modules: no change.                   */
int mph_velocity_profile_arrays(const MphConfig* cfg, double time, int n, const int* property,
                                const double* pos, const double* pos0, double* vel);

/* Every constant the reference derives before its time loop (initializeWeight/Fluid/Wall/Domain,
 * main.cpp:1191-1469), without a device: 36 doubles in the slot order of mph_get_scalars.      */
int mph_derive_scalars(const MphConfig* cfg, double* out36);
/* Host-side initialisation of the elastic solid that mph_create performs: the fixed Lagrangian
 * neighbour lists (calculateInitialNeighbor, main.cpp:1497-1658), calculateLamesconstant
 * (2526-2540) and calculateNormalizer (2544-2653).  Outputs are per particle, original order,
 * zero for non-structure particles: isnc int[n], normalizer double[n][3][3], lame_l/lame_m
 * double[n].  Any output pointer may be NULL.                                                   */
int mph_structure_init(const MphConfig* cfg, int n, const int* property, const double* pos0,
                       int* isnc, double* normalizer, double* lame_l, double* lame_m);

/* ---- device context ------------------------------------------------------------------------ */

/* Create a context on HIP device `device`, upload the particles, derive all constants and run
 * the reference's initialisation sums (main.cpp:534-570).                                    */
int mph_create(MphCtx** ctx, const MphConfig* cfg, int n, const int* property,
               const double* pos, const double* pos0, const double* vel, int device);
/* Advance nsteps time steps (main.cpp:597-686 each).  Steps are replayed from captured
 * hipGraphs of 8 and 1 steps; returns MPH_ERR_NEIGHBOR_OVERFLOW if any particle reached 512
 * neighbours.  The output-only fields (Force, Acceleration, DensityA, VolStrainP, DivergenceP,
 * and GravityCenter/PressureA without surface tension) are stored by the last step of each
 * replayed batch, so after a successful mph_step they hold that step's values; after an error
 * they are undefined (the state itself -- Position, Velocity -- is the failing step's).        */
int mph_step(MphCtx* ctx, int nsteps);
/* Step batching for the drop-in loop that calls mph_step(ctx, 1) once per iteration
 * (INTEGRATION.md section 2); single contexts only (slab mode: MPH_ERR_ARG for on != 0).
 * With it on, mph_step only counts the steps and launches them 8 at a time from the 8-step
 * graph, with the output-only stores on each batch's last step -- the cost of one
 * mph_step(ctx, 8) instead of eight synchronised single steps.  Time (mph_time) advances per call.
 * Steps still pending run, and the error flags of everything launched are read, at the next
 * flush point: mph_synchronize, mph_get, mph_set, every writer, mph_compute_virial,
 * mph_neighbor_stats, mph_profile_steps, mph_phase_timing, turning batching off, mph_destroy; so
 * every field read after a step is that step's, bit for bit as without batching.  A launched
 * batch's error is also reported by a later mph_step once its flags have landed (no wait).
 * Errors therefore surface up to two batches late, or at the next flush point.  Off by default. */
int mph_set_step_batching(MphCtx* ctx, int on);
/* Wait for all work the context enqueued (slab mode: both of its streams); with step batching,
 * launches the pending steps first and returns their status. */
int mph_synchronize(MphCtx* ctx);
/* Copy a field to host, AoS, original particle order.                                      */
int mph_get(MphCtx* ctx, int field, void* host_out);
/* Overwrite Position or Velocity (original order) -- the reference's `acc update device`.    */
int mph_set(MphCtx* ctx, int field, const void* host_in);
/* setInitialVelocityProfile() (main.cpp:395-441) applied once to the current state, as the
 * reference's commented call after the initialisation sums would (main.cpp:571); see
 * mph_velocity_profile_arrays.                                                                */
int mph_set_initial_velocity_profile(MphCtx* ctx);
int mph_particle_count(const MphCtx* ctx);
double mph_time(const MphCtx* ctx);
/* Derived scalar constants, same slots as oracle/ref_harness.inc ref_scalars (36 doubles).  */
int mph_get_scalars(const MphCtx* ctx, double* out36);
/* The output files of the whole problem.  Slab mode: collective calls (every rank at the same
 * step); each rank's owned particles are gathered on rank 0 (RCCL: one receive per rank; host
 * transport: along the ring of neighbour exchanges), which writes `path` -- the same bytes as a
 * single context holding the same state; the other ranks write nothing.                        */
int mph_write_prof(MphCtx* ctx, const char* path);
int mph_write_vtk(MphCtx* ctx, const char* path);
int mph_write_vtu(MphCtx* ctx, const char* path);   /* mph_write_vtu_arrays of the current state */
/* writeVtkFile (main.cpp:984-1189) off the time loop's critical path: the fields are copied to
 * host memory now (one D2H per field) and formatted and written by a background thread while
 * the following steps run.  At most one file is in flight; mph_output_wait joins it and
 * returns its status (also called by the next mph_write_vtk_async and by mph_destroy).
 * The bytes are those of mph_write_vtk.                                                        */
int mph_write_vtk_async(MphCtx* ctx, const char* path);
int mph_output_wait(MphCtx* ctx);
/* Message of the last failure on ctx; with ctx == NULL, of the last failed mph_create* on the
 * calling thread (the context is destroyed on failure).                                        */
const char* mph_last_error(const MphCtx* ctx);
void mph_destroy(MphCtx* ctx);

/* calculateVirialStressAtParticle (main.cpp:3077-3318), which the reference runs after the
 * physics of every VTK output step (main.cpp:672-673): per-particle virial stress of the
 * pressure (PressureP, PressureA), viscous and diffuse-interface pair forces over the step's
 * neighbour list at the post-step positions and velocities, and VirialPressureAtParticle
 * = -tr/dim.  Results are read with mph_get(MPH_FIELD_VIRIAL_STRESS / _PRESSURE); zeros until
 * the first call.  Slab mode: collective; every rank computes its owned particles, after one halo
 * exchange of the ghosts' post-step positions and velocities.                               */
int mph_compute_virial(MphCtx* ctx);

/* ---- measurement ---------------------------------------------------------------------------- */

/* Run nsteps with a HIP event pair around every kernel launch (direct launches on the
 * context's stream, no graph) and report per-kernel-kind average duration in milliseconds.
 * names: MPH_PROFILE_MAX slots of 32 chars; returns the number of entries.  The last entry is
 * "gpu_busy": the union of all kernel intervals per step (launches = nsteps), which is less than
 * their sum where kernels of two streams overlap (slab mode).                                  */
#define MPH_PROFILE_MAX 24
int mph_profile_steps(MphCtx* ctx, int nsteps, double* avg_ms, int* launches, char* names32);
/* The list kernels as the timed steps run them (direct launches of mph_profile_steps take 3-8 %
 * longer): the search (with the XCD split), pass A and pass B, each captured `reps` (1..64) times
 * into a graph of its own and replayed between two HIP events on the context's stream; avg_ms3 =
 * milliseconds per launch (-1: not measured -- pass B with elastic slots).  Each replay recomputes
 * the last step's results bit for bit, so the state is unchanged (slab contexts: on the rank's
 * own set, no exchange, pass B as one launch).  After at least one step (else MPH_ERR_ARG).     */
int mph_profile_graphs(MphCtx* ctx, int reps, double* avg_ms3);
/* Phase timing: the reference's clock() buckets of its step loop (main.cpp:695-700) from HIP
 * events.  With on != 0 mph_step launches the kernels of its step batches directly instead of
 * replaying the captured graphs (HIP does not time events recorded inside a graph), with three
 * events per step -- before the cell sort, after the neighbour search, after the elastic
 * substeps -- read after every batch (mph_step returns after its steps have run anyway);
 * mph_compute_virial is bracketed too.  mph_phase_times adds up, in milliseconds of GPU time since the context was
 * created: [0] neighbour search (calculateNeighbor with its cell sort: k_prep .. k_neighbors),
 * [1] explicit calculation (the pass-A/pass-B sums, integration and elastic substeps), [2] the
 * virial.  Single contexts only (slab mode: MPH_ERR_ARG for on != 0).                          */
int mph_phase_timing(MphCtx* ctx, int on);
int mph_phase_times(const MphCtx* ctx, double* out3);
/* Mean/max neighbour count of the last step (for algorithmic byte/flop accounting).         */
int mph_neighbor_stats(MphCtx* ctx, double* mean, int* max);

/* ---- multi-GPU slab decomposition (one process per GPU, RCCL over xGMI) ------------------ */

/* The reference runs one process over all particles (OpenMP/OpenACC, main.cpp:597-686); it has
 * no domain decomposition.  These entry points add one: the periodic domain is cut into
 * `nranks` slabs along `axis` (equal widths, or the caller's cuts: MphSlabOptions.cuts); each rank
 * owns the particles inside its slab, mirrors the
 * ones within one cutoff of a face to that neighbour as ghosts, and hands particles that crossed
 * a face to the neighbour at the start of the next step.  Per step: one exchange of
 * (x, v, type, id) for migrants + ghosts before the cell sort, one of the pass-A values
 * (PressureP [, GravityCenter, PressureA]) of the ghosts before the force pass.
 * Elastic-solid particles (types 2, 3) are owned for good by the slab of their InitialPosition;
 * their fixed Lagrangian lists reach into static ghost slots of the two neighbours, refreshed
 * before each half of every elastic substep (displacements, then first Piola-Kirchhoff stress).
 *
 * mph_get in slab mode fills only the entries of the particles this rank owns (indexed by the
 * original particle index, arrays of mph_particle_count() = the global count); the other
 * entries are left untouched, so a caller can merge the ranks' arrays.                        */

/* 128-byte RCCL unique id generated on rank 0 and shared out of band by the caller.          */
int mph_dist_unique_id(char* out128);
/* Same as mph_create, but this rank owns only the particles whose slab (along `axis`) is
 * `rank` of `nranks`; all ranks pass the full particle set.  Transport: RCCL (ncclSend/Recv
 * with the two periodic neighbours, on the context's stream).  Every size of a step is kept on
 * the device and messages travel with fixed capacities of 1.25 c + 4096 particles for a count c
 * (checked every 32 steps, also inside one mph_step call, and grown when a count passed 90 %), so
 * the steps are replayed from captured hipGraphs with no host round trip in between
 * (MPH_SLAB_GRAPHS=0: direct launches).                                                       */
int mph_create_dist(MphCtx** ctx, const MphConfig* cfg, int n, const int* property,
                    const double* pos, const double* pos0, const double* vel, int device,
                    int rank, int nranks, const char* unique_id128, int axis);
/* Host-staged transport for the same protocol: the context copies each message to pinned host
 * memory and calls `fn`, which must deliver send_l to the left neighbour (received there as
 * its recv_r) and send_r to the right neighbour (its recv_l), with the byte counts given.
 * Used to run several ranks on one GPU (tests) or where RCCL is unavailable.  Returns 0 on
 * success.                                                                                     */
typedef int (*mph_host_exchange_fn)(void* user, const void* send_l, size_t bytes_send_l,
                                    const void* send_r, size_t bytes_send_r, void* recv_l,
                                    size_t bytes_recv_l, void* recv_r, size_t bytes_recv_r);
int mph_create_dist_host(MphCtx** ctx, const MphConfig* cfg, int n, const int* property,
                         const double* pos, const double* pos0, const double* vel, int device,
                         int rank, int nranks, int axis, mph_host_exchange_fn fn, void* user);
/* General slab-mode constructor: the transport (RCCL unique id, or a host exchange callback) and,
 * with n_glob > 0, slab-local creation -- the arrays hold only the n particles this rank needs,
 * with their original indices ids[n] (ascending) among n_glob: every particle whose coordinate
 * along the axis (Position; InitialPosition for elastic particles) lies within the window of
 * mph_slab_window.  Others are not needed (ghosts arrive from the neighbours).  In slab-local mode
 * mph_get returns the static inputs (Property, InitialPosition, Mass, ...) for the particles this
 * rank was created with, and the state for the particles it owns.                             */
typedef struct MphSlabOptions {
    int rank, nranks, axis;
    const char* unique_id128;          /* RCCL transport, or NULL and host_fn:                  */
    mph_host_exchange_fn host_fn;      /* host-staged transport                                  */
    void* host_user;
    int n_glob;                        /* 0: the arrays hold every particle (n == n_glob)       */
    const int* ids;
    /* NULL: nranks equal slabs; else the nranks - 1 interior boundaries along the axis, strictly
     * ascending inside the domain (slab r = [cuts[r-1], cuts[r]), the first and last reaching
     * the domain faces), the same array on every rank -- e.g. particle-count quantiles, so that
     * the ranks hold equal shares (balanced_cuts in particlemethod_fsi_amd/dist.py)           */
    const double* cuts;
} MphSlabOptions;
int mph_create_slab(MphCtx** ctx, const MphConfig* cfg, int n, const int* property, const double* pos,
                    const double* pos0, const double* vel, int device, const MphSlabOptions* opt);
/* Host-only: the periodic window [lo, hi) (out2) along `axis` that rank `rank` of `nranks` needs
 * at slab-local creation: its slab widened by two halo widths on each side.  cuts: as in
 * MphSlabOptions (NULL: equal slabs).                                                         */
int mph_slab_window(const MphConfig* cfg, int rank, int nranks, int axis, const double* cuts, double* out2);
/* One-rank RCCL communicator on `device` whose two neighbours are itself: checks that the
 * exchange delivers each message to the right buffer (the per-peer ordering nranks == 2 relies
 * on) without a second GPU.  Returns 0 on success.                                            */
int mph_dist_selftest(int device);
/* Slab-mode facts for reports: out8 = {slab ranks of the decomposition (1 without slabs), rank,
 * size of the RCCL communicator (ncclCommCount; 0 under the host-staged transport), steps
 * replayed from captured graphs,
 * local array capacity, largest send / receive message capacity (particles), particles held
 * (owned + ghosts)}.                                                                          */
int mph_dist_info(const MphCtx* ctx, int* out8);
/* Pass-B mode of a slab context (out5; all -1 without slabs): {overlap on (1) / off (0), how it
 * was set: 1 / 0 forced by MPH_SLAB_OVERLAP, -1 chosen at creation by the ranks together, then
 * the creation probe's maxima over ranks in ms -- halo exchange, redistribution exchange (both at
 * their message capacities), the cost of pass B split into interior and face launches over one
 * launch (-1: not probed)}.  Overlap is chosen when the two exchanges take longer than the split. */
int mph_dist_overlap(const MphCtx* ctx, double* out5);
/* Mean/max length of the stored neighbour lists of the last search (what the passes walk: the
 * pairs within the passes' largest radius; with MPH_LIST_FULL=1 at creation every
 * neighbour, = mph_neighbor_stats): entries, not rows (the gap rows of the aligned lists do not
 * count).  ABI 4 (round 6): replaces mph_list_formats, which reported the compact 16-bit list
 * format removed from the product.                                                            */
int mph_list_stats(MphCtx* ctx, double* mean, int* max);
/* The neighbour lists of calculateNeighbor themselves (main.cpp:1764-1772: Neighbor[i][k] = j for
 * k < 512), for verification: the sets of the `count` particles [first, first + count) (original
 * order) from the last search, each row as ascending original indices (the reference's rows are in
 * its cell-scan order; the sets are what both define).  counts[count] receives each particle's
 * NeighborCount; ids the rows back to back (row k starts at the sum of min(counts, 512) before
 * it), ids_cap its capacity in ints.  Returns the number of ids written, or a negative MphStatus
 * (MPH_ERR_ARG when ids_cap is too small).  Single contexts with the reference's whole lists only
 * (created with MPH_LIST_FULL=1 in the environment: by default the lists keep only the pairs
 * within the largest radius of the passes' sums, NeighborCount still counts every neighbour;
 * MPH_ERR_UNSUPPORTED in slab mode or without MPH_LIST_FULL=1).  The gap rows of the aligned
 * lists are skipped.                                                          */
int mph_neighbor_rows(MphCtx* ctx, int first, int count, int* counts, int* ids, long long ids_cap);
/* Particles currently owned by this rank (after the last migration); their original indices.  */
int mph_owned_count(const MphCtx* ctx);
int mph_owned_ids(MphCtx* ctx, int* out_ids);
/* Host-only: the slab bounds [lo, hi) of `rank` and the halo width along `axis` that a slab
 * context would use (out3 = {lo, hi, h}), and which rank owns coordinate c.  cuts: as in
 * MphSlabOptions (NULL: equal slabs).                                                         */
int mph_slab_bounds(const MphConfig* cfg, int rank, int nranks, int axis, const double* cuts, double* out3);
int mph_slab_owner(const MphConfig* cfg, int nranks, int axis, const double* cuts, double c);

#ifdef __cplusplus
}
#endif
#endif /* MPH_GPU_H_INCLUDED */
