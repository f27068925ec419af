/*
 * ikgrasp — MI355X-native batched dual-arm grasp-pose inverse kinematics.
 *
 * C-ABI of libikgrasp.so (plain pointers and sizes; no C++ or torch types).
 * It replaces the per-call Pinocchio loop of the reference:
 *
 *   computeqgrasppose(robot, qcurrent, cube, cubetarget, viz=None)
 *       /root/reference/inverse_geometry.py:17-100
 *
 * whose Python->C++ crossings (pin.framesForwardKinematics :58,
 * pin.computeJointJacobians :59, pin.log :66-67, pin.computeFrameJacobian
 * :75-76, np.linalg.pinv :83, pin.integrate :86, projecttojointlimits :89 ->
 * tools.py:21-22) are fused into one HIP kernel launch over a batch.
 * The ctypes binding a maintainer adds on the reference side is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *   - SE(3) placements are 12 scalars: R row-major (9) then t (3).
 *   - Motion vectors are [linear; angular] (Pinocchio convention).
 *   - Float arrays use the dtype selected by `dtype` (IKG_F64 / IKG_F32).
 *   - All buffers are owned by the caller.  They are device pointers unless
 *     IKG_FLAG_HOST_POINTERS is set, in which case the library stages them
 *     through device scratch and synchronises the stream before returning.
 *   - Float inputs must be finite.  With IKG_FLAG_HOST_POINTERS the solve
 *     entry points check targets, q0 and seeds and return IKG_EINVAL for a
 *     NaN/inf; device-pointer callers own the check (the kernels are built
 *     with finite-math assumptions, so a non-finite input gives unspecified
 *     values for that problem's outputs).
 *   - Return 0 on success, a negative IKG_E* code on failure; the message of
 *     the last failure on the calling thread is ikg_last_error().  Nothing
 *     throws or exits across this boundary.
 *   - Calls are re-entrant per (model, stream).
 *   - Results are deterministic: no answer depends on the order in which a
 *     launch's waves run, on the batch size or on a problem's position, with
 *     the exceptions below.  With the collision term, a problem that
 *     converges into collision runs on in the batch kernel itself, which
 *     writes a checkpoint of its loop state per 32-update window into the
 *     problem's own fixed slot; the scan proves windows colliding with a
 *     certificate, and a window it cannot prove is regenerated from its
 *     checkpoint by the same loop compiled as the resume kernel.  Which path
 *     a problem takes is a function of that problem alone, so its answer is
 *     the same in any batch, chunking (a batch whose checkpoints exceed their
 *     budget, IKG_CK_BUDGET_MB, runs as equal launches in the whole batch's
 *     layout) or records round (IKG_REC_BUDGET_MB); the regenerated iterates
 *     agree with the batch loop's to rounding (the two instantiations
 *     contract a few products into FMAs differently: flags and update counts
 *     equal, q <= 1e-12 fp64 on the tests' batches).  Those kernels recompute
 *     the carried joint trig exactly at every window start (every 32 updates
 *     in fp64, 128 without the collision term), so a problem that never
 *     collides gets the same answer as without the term to rounding, not bit
 *     for bit.  (Models the batch
 *     kernel does not record for -- generic or run-time-compiled kernels,
 *     lambda > 0, the QUAD layout -- run on in the trajectory kernel, which
 *     agrees with the batch loop to rounding, q <= 1e-9.)  And in
 *     fp64 a broadcast q0
 *     (q0_stride = 0) and per-problem q0 rows (and multi-start seeds)
 *     advance the joint sin/cos by different rules for steps of
 *     0.025..0.25 rad (exact sincos / a longer series), so when such steps
 *     occur -- random seeds, not the reference's q0 = 0 on its sampler's
 *     targets -- the two agree to rounding (q <= 1e-10, end effectors
 *     <= 1e-12 over 150 updates), not bit for bit.  fp32 takes the longer
 *     series for every q0 layout: its answer does not depend on how q0 is
 *     passed.  A multi-start's seed equals a per-row solve of that seed bit
 *     for bit.  fp32 results also depend on the kernel layout (PAIR /
 *     PACKED), which AUTO picks by batch size.
 *
 * Graphs
 *   - Device-pointer solves are stream-ordered and may be captured into a
 *     hipGraph (no host synchronisation, no blocking allocation).  Scratch a
 *     captured solve needs (records, multi-start and continuation workspaces)
 *     is allocated at capture time and owned by the captured graph (a graph
 *     user object).  When the graph and all its executable instantiations
 *     are destroyed the buffer goes on the model's pending list: a later
 *     capture on the model reuses it if it is large enough (so recapturing
 *     every cycle holds a bounded number of buffers), and the model's next
 *     uncaptured solve, ikg_model_trim or ikg_model_destroy frees it.
 *   - All instantiations of one captured graph share that scratch: do not
 *     launch two of them concurrently (on different streams).
 *   - Destroy graphs before the model: they also reference its device tables.
 *
 * Scratch memory
 *   - Uncaptured solves take their scratch from a stream-ordered pool the
 *     model owns (one per device it solves on).  The pool keeps up to
 *     1.25 GiB of freed memory reserved for the next solve (environment
 *     IKG_WS_KEEP_MB overrides the amount) and releases the rest at the next
 *     synchronisation.  A collision solve holds, while it runs, its window
 *     checkpoints (17 KB per fp64 problem, 8.7 KB fp32, at max_iters 1,000)
 *     and the records of the problems its scan regenerates, up to the
 *     records budget (1 GiB).  ikg_model_trim synchronises each such device and
 *     releases everything the pools hold unused; ikg_model_destroy
 *     synchronises and destroys the pools.  Released memory goes back to the
 *     HIP runtime, which keeps it mapped for later pools and allocations of
 *     the process (the device's free-memory figure does not rise; a second
 *     model reuses it without taking more of the device), and a destroyed
 *     model leaves that figure where it was before the model existed
 *     (tests/test_gpu_memory.py).  IKG_WS_POOL=0 in the environment
 *     selects the device's default pool.
 */
#ifndef IKGRASP_H
#define IKGRASP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IKG_MAX_NQ 32
#define IKG_ARM_DOF 6
#define IKG_MAX_GEOMS 64
#define IKG_MAX_PAIRS 1024

enum ikg_dtype { IKG_F64 = 0, IKG_F32 = 1 };

enum ikg_status {
  IKG_OK = 0,
  IKG_EINVAL = -1,      /* bad argument / unsupported model structure */
  IKG_EHIP = -2,        /* HIP runtime error */
  IKG_ENOMEM = -3,      /* device allocation failed */
  IKG_ENODEV = -4       /* no such device */
};

/* flags */
#define IKG_FLAG_HOST_POINTERS 1u

/* kernel variant selector (ikg_params.variant) */
enum ikg_variant {
  IKG_VARIANT_AUTO = 0,   /* ikg_solve_batch: PACKED where it applies and B > 4 pair waves
                             per CU, else PAIR (QUAD measured no faster: explicit only);
                             ikg_solve_multistart: PAIR */
  IKG_VARIANT_PAIR = 1,   /* two lanes per problem (one arm per lane), 32 problems / wave */
  IKG_VARIANT_PACKED = 2, /* fp32, Nextage-class models, lambda = 0: one lane per problem with
                             both arms packed in 2-vectors (v_pk_*_f32), 64 problems / wave */
  IKG_VARIANT_QUAD = 3    /* Nextage-class models, lambda = 0: four lanes per arm (rows of the
                             kinematic chain split over them), 8 problems / wave */
};

/* Robot + grasp-object description (produced by the model compiler,
 * ikgrasp/model.py, from the URDFs — setup_pinocchio.py:73-83). */
typedef struct ikg_model_desc {
  int32_t nq;                        /* configuration size (15 for Nextage) */
  int32_t parent[IKG_MAX_NQ];        /* parent joint (q index), -1 = universe */
  int32_t axis[IKG_MAX_NQ];          /* 0/1/2 = revolute about +X/+Y/+Z */
  double placement[IKG_MAX_NQ][12];  /* joint placement in parent frame (R row-major, t) */
  double lower[IKG_MAX_NQ];          /* joint limits (projecttojointlimits, tools.py:21-22) */
  double upper[IKG_MAX_NQ];
  int32_t root_q;                    /* shared joint feeding both arms (chest) */
  int32_t arm_q[2][IKG_ARM_DOF];     /* left/right arm joints, proximal -> distal */
  double hand[2][12];                /* LARM_EFF / RARM_EFF frame in last arm joint frame */
  double hook[2][12];                /* LARM_HOOK / RARM_HOOK in the cube frame (cube_small.urdf:34-47) */
} ikg_model_desc;

/* Loop hyper-parameters; defaults equal the reference
 * (EPSILON config.py:22, DT and max_iters inverse_geometry.py:53-54). */
typedef struct ikg_params {
  double eps;          /* stop when |log6 err| < eps for both hands (1e-3) */
  double dt;           /* q <- clip(q + dt * dq) (1e-2) */
  int32_t max_iters;   /* joint updates before giving up (1000) */
  int32_t variant;     /* enum ikg_variant */
  double lambda;       /* damping of (J J^T + lambda I); 0 = pinv semantics (reference) */
  int32_t problems_per_wave; /* 1..32 problems per 64-lane wave; 0 = auto (32) */
  int32_t check_collision;   /* 1: reference `success` = converged AND collision-free, iterating on while
                                converged-but-colliding (inverse_geometry.py:70, :97-98); needs
                                ikg_model_set_collision.  0: convergence only (default). */
} ikg_params;

/* Collision scene (tools.py:25-35 collision(); pairs built in
 * setup_pinocchio.py:53-60), produced by ikgrasp/collision.py. */
enum ikg_geom_kind {
  IKG_GEOM_SPHERE = 0,    /* dims: radius */
  IKG_GEOM_BOX = 1,       /* dims: half extents */
  IKG_GEOM_CYLINDER = 2,  /* dims: radius, half length (local z) */
  IKG_GEOM_MESHBOX = 3    /* convex hull of a box mesh (the cube): half extents */
};
typedef struct ikg_collision_desc {
  int32_t n_geoms;
  int32_t kind[IKG_MAX_GEOMS];
  int32_t joint[IKG_MAX_GEOMS];          /* q index of the parent joint, -1 = world-fixed */
  double placement[IKG_MAX_GEOMS][12];   /* in the parent joint frame (world if joint = -1) */
  double dims[IKG_MAX_GEOMS][3];
  int32_t target_geom;                   /* geometry placed at each solve's cube target, -1 none */
  int32_t n_pairs;
  int32_t pairs[IKG_MAX_PAIRS][2];
} ikg_collision_desc;

typedef struct ikg_model ikg_model;

/* Build a device-ready model (tables are uploaded to every device lazily). */
int ikg_model_create(const ikg_model_desc* desc, ikg_model** out);
void ikg_model_destroy(ikg_model* model);

/* Return the scratch memory the model's pools keep for later solves (and the
 * buffers of destroyed captured graphs) to the driver; the model stays usable.
 * Synchronises every device the model has solved on.  No reference
 * counterpart (the reference allocates nothing on a device). */
int ikg_model_trim(ikg_model* model);

/* Attach (or replace) the collision scene of a model. */
int ikg_model_set_collision(ikg_model* model, const ikg_collision_desc* desc);

/*
 * Compile the pair-layout kernels against this model's tables (hipRTC, gfx950)
 * and use them for later ikg_solve_batch / ikg_solve_multistart calls of
 * `dtype` on `device` that run the pair layout (not PACKED / QUAD).  Joint
 * axes, identity placements, zero offsets and limits become compile-time
 * constants; results match the prebuilt kernels' (same flags and update
 * counts, q to rounding: folded exact 0 / 1 terms).  The first call per
 * model and dtype compiles (about 0.5 s), later devices only load.  `flags`: 0,
 * or IKG_SPECIALIZE_IF_GENERIC to do nothing (and return IKG_OK) for a model the
 * prebuilt library already specialises (Nextage class).  Do not call
 * concurrently with a solve on the same model.  With the environment variable
 * IKG_JIT_CACHE_DIR set, code objects are cached there (keyed by the generated
 * source, the embedded device headers and the compile options).  No reference
 * counterpart: inverse_geometry.py has one Python-level model
 * (setup_pinocchio.py:73-83); this is the per-model code generation the batched
 * library adds.
 */
#define IKG_SPECIALIZE_IF_GENERIC 1u
int ikg_model_specialize(ikg_model* model, int device, int dtype, uint32_t flags);
/* 1 if ikg_model_specialize succeeded for (device, dtype), else 0. */
int ikg_model_is_specialized(const ikg_model* model, int device, int dtype);

/* Fill `p` with the reference defaults. */
void ikg_params_default(ikg_params* p);

/*
 * Batched computeqgrasppose (inverse_geometry.py:17-100).  With
 * params->check_collision = 1 (needs ikg_model_set_collision) the stop test is
 * the reference's `errors pass and not collision(q)` (:70) and a final
 * colliding q is a failure (:97-98); with 0 it is the error test only.
 *   targets   [B,12]  cube placements (cubetarget); hooks are applied inside
 *   q0        [B,nq] (q0_stride = nq) or [nq] broadcast (q0_stride = 0)
 *   q_out     [B,nq]  first iterate with both errors < eps, else the iterate
 *                     after max_iters updates (same as the reference)
 *   converged [B]     1 if the stop test passed (the reference `success`
 *                     when check_collision = 1)
 *   iters     [B]     joint updates performed (may be NULL)
 *   err_out   [B,2]   |log6| of left/right hand at q_out (may be NULL)
 */
int ikg_solve_batch(const ikg_model* model, int device, int dtype,
                    const void* targets, const void* q0, int64_t q0_stride, int64_t B,
                    const ikg_params* params,
                    void* q_out, uint8_t* converged, int32_t* iters, void* err_out,
                    void* stream, uint32_t flags);

/*
 * Multi-start: every target is solved from every seed (S seeds x T targets);
 * per target the best seed is kept: lowest max(|eL|,|eR|) among converged
 * seeds, else lowest overall (ties -> lowest seed index).
 *   seeds [S,nq]; outputs per target: q_out [T,nq], converged [T], iters [T],
 *   err_out [T,2], best_seed [T] (any output but q_out may be NULL).
 */
int ikg_solve_multistart(const ikg_model* model, int device, int dtype,
                         const void* targets, int64_t T, const void* seeds, int64_t S,
                         const ikg_params* params,
                         void* q_out, uint8_t* converged, int32_t* iters, void* err_out,
                         int32_t* best_seed, void* stream, uint32_t flags);

/*
 * Batched effector forward kinematics (pin.framesForwardKinematics +
 * data.oMf[LARM_EFF/RARM_EFF], inverse_geometry.py:58-63).
 *   q [B,nq] -> hands [B,2,12]
 */
int ikg_fk_batch(const ikg_model* model, int device, int dtype,
                 const void* q, int64_t B, void* hands, void* stream, uint32_t flags);

/*
 * Batched SE(3) logarithm, pin.log6 (the pose error of
 * inverse_geometry.py:66-67): M [B,12] -> out [B,6] = [v; w].
 */
int ikg_log6_batch(int device, int dtype, const void* M, int64_t B, void* out, void* stream, uint32_t flags);

/*
 * Batched collision query, tools.collision(robot, q) (tools.py:25-35) with the
 * cube placed at each target (setcubeplacement, tools.py:62-68):
 *   q [B,nq], targets [B,12] -> in_collision [B] (1 = some active pair intersects)
 */
int ikg_collision_batch(const ikg_model* model, int device, int dtype, const void* q, const void* targets,
                        int64_t B, uint8_t* in_collision, void* stream, uint32_t flags);

/*
 * Batched distance query, tools.distanceToObstacle(robot, q) (tools.py:37-51):
 * the minimum over the active pairs listed in pair_idx (indices into the
 * scene's pair list; the reference takes the pairs whose second geometry is
 * the table or the obstacle) of the pair distance (hpp-fcl
 * computeDistance().min_distance; <= 0 when the pair intersects):
 *   q [B,nq], targets [B,12] -> dist [B].  pair_idx is a host array.
 */
int ikg_distance_batch(const ikg_model* model, int device, int dtype, const void* q, const void* targets,
                       int64_t B, const int32_t* pair_idx, int32_t n_pairs, void* dist, void* stream,
                       uint32_t flags);

/*
 * Batched cube-placement check of the planner's sampler / path projection
 * (path.py:51-52, :136-138: pin.computeCollisions on the cube's own collision
 * model, setup_pinocchio.py:62-70): the scene's target geometry placed at each
 * targets[i] against the world-fixed geometries listed in geoms (host array):
 *   targets [B,12] -> in_collision [B].
 */
int ikg_target_env_batch(const ikg_model* model, int device, int dtype, const void* targets, int64_t B,
                         const int32_t* geoms, int32_t n_geoms, uint8_t* in_collision, void* stream,
                         uint32_t flags);

/*
 * Controller kinematics: the kinematic terms of the
 * task-space controller, control.py:284-345, for a batch of states.
 * Replaces, per state and per hand (LARM_EFF, RARM_EFF):
 *   pin.computeAllTerms + updateFramePlacements -> data.oMf     (control.py:284-287, :305)
 *   pin.getFrameVelocity(model, data, fid, rf)                  (:310-313)
 *   pin.computeFrameJacobian(model, data, q, fid, rf)           (:341-342)
 *   pin.getFrameJacobianTimeVariation(model, data, fid, rf)     (:343-344)
 *   J_dot @ vq                                                  (:345)
 *   the desired-state FK (:292-294) and the PD errors (:314-333)
 * rf: enum ikg_reference_frame (the controller uses LOCAL_WORLD_ALIGNED).
 *   q, v [B,nq] (v may be NULL = zero velocity); q_des, v_des [B,nq] are only
 *   read for err/derr (v_des NULL = 0).  Every output is optional (NULL):
 *   placement [B,2,12]   oMf of LARM_EFF, RARM_EFF
 *   velocity  [B,2,6]    frame velocity in rf
 *   J, dJ     [B,12,nq]  rows 0-5 LARM_EFF, 6-11 RARM_EFF (np.vstack, :369), in rf;
 *                        dJ = d/dt J along q' = v
 *   dJv       [B,12]     dJ v
 *   err       [B,12]     per hand [x_des - x; log3(R_des R^T)]     (:326-327)
 *   derr      [B,12]     per hand v_des - v, LOCAL_WORLD_ALIGNED   (:330-331)
 */
enum ikg_reference_frame { IKG_WORLD = 0, IKG_LOCAL = 1, IKG_LOCAL_WORLD_ALIGNED = 2 };
typedef struct ikg_frame_kin_out {
  void* placement;
  void* velocity;
  void* J;
  void* dJ;
  void* dJv;
  void* err;
  void* derr;
} ikg_frame_kin_out;
int ikg_frame_kinematics_batch(const ikg_model* model, int device, int dtype, const void* q, const void* v,
                               const void* q_des, const void* v_des, int64_t B, int rf,
                               const ikg_frame_kin_out* out, void* stream, uint32_t flags);

/* Thread-local message of the last failure ("" if none). */
const char* ikg_last_error(void);

/* Library version string. */
const char* ikg_version(void);

#ifdef __cplusplus
}
#endif

#endif /* IKGRASP_H */
