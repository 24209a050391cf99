/*
 * rbe_planner.h — C-ABI of librbe_mi355x.so, the MI355X-native replacement for the
 * state-validity / plan path of sgajera12/RBE550_final_project.
 *
 * What each entry point replaces in the reference (paths relative to /root/reference):
 *
 *   rp_create / rp_destroy      PlannerInterface.__init__ + _ensure_adapter      code/planning.py:14-30
 *   rp_set_scene(_rot, _poses)  the Genesis scene the collider sees (plane, boxes
 *                               at their poses, upright or toppled, raised robot
 *                               base)                                             code/scenes.py:29-34,49-85,
 *                                                                                 code/planning.py:211
 *   rp_set_attached             self.attached_object + the exemption of
 *                               collision_with_attached_object                    code/planning.py:153,221-230
 *   rp_check_states(_device)    _is_ompl_state_valid: set_qpos (FK) +
 *                               detect_collision + pair filter, for N states      code/planning.py:209-219,238-242
 *   rp_state_contacts           diagnose_valid_violation (which links collide)    code/planning.py:43-57
 *   rp_check_edges(_device)     OMPL DiscreteMotionValidator::checkMotion, run
 *                               inside ss.solve / simplifySolution                code/planning.py:190,196
 *   rp_plan                     plan_path body from the space setup to the
 *                               interpolated path: RealVectorStateSpace bounds,
 *                               RRTConnect solve, simplifySolution,
 *                               path.interpolate(num_waypoints)                   code/planning.py:139-200
 *   rp_plan_async / rp_plan_wait rp_plan on the context's planner thread, so the
 *                               caller's tensor-list conversion and qpos restore
 *                               overlap the query                                 code/planning.py:200-205,232-242
 *   rp_reserve                  (new) workspace sizing ahead of the first query
 *   rp_ik                       robot.inverse_kinematics(link=hand, pos, quat) that
 *                               makes plan_path's goals (Genesis, batched restarts)  code/motion_primitives.py:131-134
 *   rp_group_*                  (new) data-parallel sharding of each RRT-Connect
 *                               iteration across ranks with an all-gather;
 *                               the reference is single-process                   code/planning.py:121-122
 *   rp_get_stats / rp_last_error counters and error text (the reference prints /
 *                               logs: planning.py:199, 202)
 *
 * ABI rules: plain C types only; 0 = ok, <0 = error (text via rp_last_error);
 * no C++ exception crosses the boundary; every output buffer is caller-allocated;
 * one host thread per context at a time. There is NO CPU execution path in this
 * library: rp_create fails if no MI355X (gfx950) device is present.
 *
 * State layout: the 9-D Franka qpos (7 arm joints, 2 fingers) in the order of
 * robot.n_qs (code/planning.py:143-150). Batched states are row-major N x 9.
 */
#ifndef RBE_PLANNER_H
#define RBE_PLANNER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RP_NQ 9                 /* planning dimension: 7 revolute + 2 prismatic  */
#define RP_MAX_CAPSULES 32
#define RP_MAX_SELF_PAIRS 64
#define RP_MAX_BOXES 64

/* Link indices of the Franka chain; names match the Genesis/MJCF links the
 * reference looks up (planning.py:222). */
enum {
    RP_LINK0 = 0, RP_LINK1, RP_LINK2, RP_LINK3, RP_LINK4, RP_LINK5, RP_LINK6, RP_LINK7,
    RP_HAND = 8, RP_LEFT_FINGER = 9, RP_RIGHT_FINGER = 10, RP_NUM_LINKS = 11
};

/* Return codes */
enum {
    RP_OK = 0,
    RP_ERR_ARG = -1,        /* bad argument (null pointer, size out of range)       */
    RP_ERR_DEVICE = -2,     /* no gfx950 device / HIP runtime error                 */
    RP_ERR_STATE = -3,      /* call out of order (e.g. rp_plan before rp_set_scene) */
    RP_ERR_CAPACITY = -4,   /* tree / path capacity exceeded                        */
    RP_ERR_EXCHANGE = -5    /* group all-gather (callback or RCCL) failed            */
};

/* Plan status (OMPL PlannerStatus analogue; planning.py:190-202 treats EXACT and
 * APPROXIMATE as "solved"). */
enum {
    RP_STATUS_NONE = 0,
    RP_STATUS_EXACT = 1,
    RP_STATUS_APPROXIMATE = 2,
    RP_STATUS_TIMEOUT = 3,        /* no solution and no approximate path            */
    RP_STATUS_INVALID_START = 4,  /* start out of bounds or in collision            */
    RP_STATUS_INVALID_GOAL = 5    /* goal out of bounds or in collision             */
};

/* One collision capsule rigidly attached to a link: segment a-b in the link frame. */
typedef struct rp_capsule {
    int32_t link;        /* RP_LINK*                                  */
    float a[3];
    float b[3];
    float radius;
} rp_capsule;

/* Robot collision model (kinematics are the fixed Franka Panda chain). */
typedef struct rp_robot_desc {
    int32_t n_capsules;                        /* <= RP_MAX_CAPSULES          */
    rp_capsule capsules[RP_MAX_CAPSULES];
    int32_t n_self_pairs;                      /* <= RP_MAX_SELF_PAIRS        */
    int32_t self_pairs[RP_MAX_SELF_PAIRS][2];  /* capsule index pairs         */
} rp_robot_desc;

/* Box obstacle: centre, half extents, rotation about world z (yaw, radians).
 * Genesis gs.morphs.Box(size=s, pos=c) has half = s/2 (scenes.py:59-62). */
typedef struct rp_box {
    float center[3];
    float half[3];
    float yaw;
} rp_box;

/* Box obstacle with a full orientation: quaternion (w, x, y, z), the order of
 * Genesis entity.get_quat(). A block that toppled or leans (goal3's "Stack
 * collapsed! ... TAMP will re-plan", code/goal3_tallest.py:257) is tilted; x = y = 0
 * is an upright box of yaw atan2(2(wz + xy), 1 - 2(y^2 + z^2)). */
typedef struct rp_box_rot {
    float center[3];
    float half[3];
    double quat[4];
} rp_box_rot;

/* rp_plan parameters. Zero / negative fields take the default shown. */
typedef struct rp_plan_params {
    uint64_t seed;          /* Philox key; the reference is unseeded (scenes.py:9)          */
    int64_t batch;          /* max samples per RRT-Connect iteration (global), 4096         */
    int64_t batch_min;      /* samples in iteration 0; iteration k draws
                               min(batch, batch_min << k). Default min(batch, 64): easy
                               queries solve in the first, cheap iteration (pick / place
                               queries: 0.083 -> 0.072 ms vs 256, tools/plan_sweep.py)   */
    double range;           /* steering distance, default 0.2 * maxExtent (OMPL RRTConnect) */
    double resolution;      /* edge resolution, default 0.01 * maxExtent (OMPL default)     */
    double timeout_s;       /* wall-clock budget of the solve, default 5.0 (planning.py:63);
                               checked once per iteration, so a plan can overrun it by its
                               last iteration. Rank groups: an iteration that opens
                               replicated (see group_repl) only learns of a timeout at the
                               next vote, up to RP_GROUP_VOTE_EVERY - 1 iterations later
                               (the oracle applies the same rule)                          */
    int64_t max_iters;      /* iteration cap (deterministic tests), default unlimited        */
    int32_t n_waypoints;    /* path.interpolate(n) (planning.py:198), default 100; 0 = none */
    int32_t simplify;       /* smooth_path (planning.py:195-196): 0 = off; 1 = simplifyMax
                               structure (shortcuts + B-spline rounds);
                               2 = vertex shortcuts only                                */
    int64_t tree_capacity;  /* nodes per tree, default 1<<22                                */
    int32_t straight_first; /* 0 (default) = with simplification on, check the straight edge
                               start -> goal first and return it when valid (the path the
                               shortcut stage would reduce any solution to); < 0 = always
                               run RRT-Connect; ignored when simplify == 0               */
    int32_t chunk;          /* execution only, never the result: an iteration runs as ordered
                               sub-batches — chunk samples, then each next one 4x the last
                               but at least a quarter of what is left — and ends after the
                               sub-batch holding the first REACHED sample (the trees keep
                               the appends up to that sample, DESIGN.md §4 step 5, whatever
                               the sub-batching); on trees of >= 4,096 nodes the first
                               sub-batch is at least a quarter of the iteration. 0 =
                               default 64; < 0 = the whole iteration as one batch        */
    int64_t group_repl;     /* rank groups (rp_group_init*): sub-batches (see chunk) of at
                               most this many samples run replicated — every rank computes
                               the whole sub-batch, nothing is exchanged (same trees: the
                               planner is deterministic); larger ones are sharded with one
                               record all-gather each. Timeout vote: an iteration whose
                               first sub-batch is sharded votes through that exchange; one
                               that opens replicated first exchanges the ranks' timeout
                               flags alone when k % RP_GROUP_VOTE_EVERY ==
                               RP_GROUP_VOTE_EVERY - 1 (all stop if any timed out).
                               0 = RP_GROUP_REPL_DEFAULT; < 0 = always shard            */
} rp_plan_params;

#define RP_GROUP_REPL_DEFAULT 4096
#define RP_GROUP_VOTE_EVERY 8

/* rp_ik parameters (defaults follow Genesis inverse_kinematics). Zero / negative
 * fields take the default shown. */
typedef struct rp_ik_params {
    uint64_t seed;          /* Philox key of the random restarts                          */
    int32_t n_seeds;        /* restarts per target, restart 0 = init (max_samples), 256   */
    int32_t iters;          /* damped-least-squares steps per restart, 64                  */
    double damping;         /* 0.01                                                        */
    double pos_tol;         /* position tolerance, 5e-4 m                                  */
    double rot_tol;         /* orientation tolerance, 5e-3                                 */
} rp_ik_params;

/* rp_ik per-target status */
enum { RP_IK_OK = 0, RP_IK_COLLIDING = 1, RP_IK_NOT_CONVERGED = 2 };

/* Counters of the last call (per rank). */
typedef struct rp_stats {
    int64_t states_checked;     /* validity evaluations actually executed             */
    int64_t edges_checked;
    int64_t samples;            /* samples drawn (global)                             */
    int64_t iterations;
    int64_t start_tree_size;
    int64_t goal_tree_size;
    int64_t path_states_raw;    /* before simplify / interpolate                     */
    int64_t path_states_simplified;
    double solve_ms;            /* wall time of the solve loop                       */
    double simplify_ms;
    double total_ms;            /* wall time of the whole rp_plan call               */
    double exchange_ms;         /* group all-gather time (RCCL: stream events; host
                                   transport: the callback)                          */
} rp_stats;

/* Kernel profile of the last rp_plan (rp_set_profiling on): HIP events around every
 * nearest-node launch and every edge-validity launch, on the planner stream. The
 * work counts are algorithmic: nn_pairs = (query, tree node) distance evaluations;
 * edge_states = validity evaluations executed by the edge launches. */
typedef struct rp_profile {
    int64_t nn_launches;
    double nn_ms;
    double nn_pairs;
    int64_t edge_launches;
    double edge_ms;
    int64_t edge_states;
} rp_profile;

typedef struct rp_ctx rp_ctx;

/* Host-transport all-gather used by a rank group (rp_group_init): gather
 * `bytes_per_rank` bytes of every rank's `send` into `recv` (rank-major). Both are
 * pinned host buffers owned by the library, valid for the duration of the call.
 * Return 0 on success. */
typedef int (*rp_allgather_fn)(void* user, const void* send, void* recv, int64_t bytes_per_rank);

#define RP_RCCL_ID_BYTES 128    /* ncclUniqueId */

/* Library identity: returns a static string ("librbe_mi355x <version> gfx950"). */
const char* rp_version(void);

/* Layout version of the structs above (rp_plan_params, rp_box_rot, rp_stats, ...):
 * bumped whenever one of them changes size or meaning (the structs carry no size
 * field). A client checks rp_abi_version() == RP_ABI_VERSION once, before passing
 * any struct (native.py load() does); a mismatch means the header and the library
 * disagree and no call may be made. Version 5: rp_box_rot / rp_set_scene_rot;
 * 6: rp_selftest_f64 writes six values per input; 7: rp_query / rp_plan_many. */
#define RP_ABI_VERSION 7
int rp_abi_version(void);

/* Fill `out` with the built-in Franka Panda capsule model (spec/franka_capsules.json). */
int rp_default_robot(rp_robot_desc* out);

/* Create a context on HIP device `device` (>= 0). `robot` may be NULL (default model).
 * The capsule geometry is compiled into the kernels (spec/franka_capsules.json, the
 * constants fold into the instruction stream), so a non-NULL `robot` must equal
 * rp_default_robot()'s description field for field; any other model is RP_ERR_ARG.
 * The parameter lets a caller assert the model it was built against. */
int rp_create(rp_ctx** out, int device, const rp_robot_desc* robot);
void rp_destroy(rp_ctx* ctx);

/* Obstacles: boxes + ground plane at z = plane_z; robot base translation (the
 * reference raises it by 1 cm, scenes.py:29-34). Replaces any previous scene and
 * clears the attached box. */
int rp_set_scene(rp_ctx* ctx, const rp_box* boxes, int32_t n_boxes, float plane_z,
                 const float base_pos[3]);

/* rp_set_scene with full box orientations (the Genesis collider sees every box at
 * its simulated pose, code/planning.py:211). An upright box, |x|, |y| <= 1e-7 |quat|
 * (a rotation about z to within simulation noise; a quaternion whose norm is not 1 is
 * normalised first), gets exactly the record rp_set_scene makes for its yaw
 * atan2(2(wz + xy), 1 - 2(y^2 + z^2)); any other box is tilted: the quaternion
 * is normalised and turned into a rotation matrix in double, rounded to float once,
 * and the collider tests the capsules against the rotated box (world AABB padded by
 * 1e-6 m). RP_ERR_ARG for a zero quaternion. */
int rp_set_scene_rot(rp_ctx* ctx, const rp_box_rot* boxes, int32_t n_boxes, float plane_z,
                     const float base_pos[3]);

/* Attached object (planning.py:221-230): contacts between box `box_index` and the
 * links set in `exempt_link_mask` (bit = 1 << RP_LINK*) are ignored.
 * box_index = -1 clears. The reference exempts hand | left_finger | right_finger. */
int rp_set_attached(rp_ctx* ctx, int32_t box_index, uint32_t exempt_link_mask);

/* rp_set_scene_rot + rp_set_attached from the simulator's poses in one call (the
 * drop-in planning.py's per-query scene ingestion): box j at position
 * poses[7j .. 7j+2] (rounded to float) with orientation quaternion (w, x, y, z) =
 * poses[7j+3 .. 7j+6] (upright or tilted, as rp_set_scene_rot), half extents
 * halves[3j .. 3j+2]. base_pos: the robot base (double). */
int rp_set_scene_poses(rp_ctx* ctx, const double* poses, const float* halves, int32_t n_boxes,
                       float plane_z, const double base_pos[3], int32_t attached_box,
                       uint32_t exempt_link_mask);

/* Validity of N states (row-major N x 9 float32, host memory). flags_out[i] = 1 if
 * valid (collision free), 0 otherwise. */
int rp_check_states(rp_ctx* ctx, const float* q, int64_t n, uint8_t* flags_out);

/* Same on device-resident buffers (e.g. torch tensors' data_ptr), asynchronous: the
 * kernel is launched on `stream` (a hipStream_t) or, when `stream` is NULL, on the
 * context's own non-blocking stream. NULL therefore does NOT mean the legacy
 * default stream; pass an explicit stream to order against other work. */
int rp_check_states_device(rp_ctx* ctx, const float* q_dev, int64_t n, uint8_t* flags_dev,
                           void* stream);

/* Motion validity of N edges qa[i] -> qb[i] (row-major N x 9 float64), with OMPL's
 * DiscreteMotionValidator semantics: qb and the interior states
 * qa + (qb - qa) * j / nd, j = 1..nd-1, nd = ceil(|qb - qa| / resolution) are checked
 * (qa is assumed valid). out[i] = 1 if the motion is valid. */
int rp_check_edges(rp_ctx* ctx, const double* qa, const double* qb, int64_t n,
                   double resolution, uint8_t* out);
/* Device-buffer variant, fully asynchronous on `stream` (NULL: the context stream):
 * no host read-back; it uses the context's edge scratch, so calls in flight on
 * different streams must be ordered by the caller. */
int rp_check_edges_device(rp_ctx* ctx, const double* qa_dev, const double* qb_dev, int64_t n,
                          double resolution, uint8_t* out_dev, void* stream);

/* Collision report for one state (diagnostics, planning.py:43-57): up to `cap`
 * (link, obstacle) pairs; obstacle >= 0 is a box index, -1 the plane, -2 - k a
 * self contact with link k. Returns the number of pairs found (may exceed cap). */
int rp_state_contacts(rp_ctx* ctx, const double q[RP_NQ], int32_t* pairs_out, int32_t cap);

/* Full query: bounds + start/goal checks, batched RRT-Connect, simplification and
 * interpolation. path_out receives *n_out states (row-major, float64). */
int rp_plan(rp_ctx* ctx, const double start[RP_NQ], const double goal[RP_NQ],
            const double lo[RP_NQ], const double hi[RP_NQ], const rp_plan_params* params,
            double* path_out, int32_t path_cap, int32_t* n_out, int32_t* status_out);

/* rp_plan split in two (same arguments, same results): rp_plan_async copies the
 * inputs and hands the query to the context's planner thread, which runs rp_plan;
 * it returns at once, so the caller's own per-query work (planning.py builds the
 * waypoint tensors, code/planning.py:232-242, and restores qpos, :205) overlaps the
 * GPU's. path_out, n_out and status_out must stay valid until rp_plan_wait, which
 * blocks until the query is done and returns rp_plan's code. Every other call on the
 * context while a query is in flight is RP_ERR_STATE. */
int rp_plan_async(rp_ctx* ctx, const double start[RP_NQ], const double goal[RP_NQ],
                  const double lo[RP_NQ], const double hi[RP_NQ], const rp_plan_params* params,
                  double* path_out, int32_t path_cap, int32_t* n_out, int32_t* status_out);
int rp_plan_wait(rp_ctx* ctx);

/* One query of rp_plan_many: its scene (rp_set_scene's boxes, plane and base), its
 * attached box (rp_set_attached with the reference's exemption, hand | left_finger |
 * right_finger; -1 = none), start, goal and parameters. */
typedef struct rp_query {
    const rp_box* boxes;
    int32_t n_boxes;
    float plane_z;
    float base_pos[3];
    int32_t attached_box;
    double start[RP_NQ];
    double goal[RP_NQ];
    rp_plan_params params;
} rp_query;

/* Many independent queries kept in flight on several contexts of this process
 * (BASELINE config 3: goal3's ~20 RRT queries "pipelined";
 * code/goal3_tallest.py:63-283 -> code/motion_primitives.py:144): query i runs on
 * ctxs[i % n_ctx] through that context's planner thread (rp_plan_async), after the
 * context's previous query; every context has its own stream, so the queries'
 * dependent small kernels overlap. Each result is the one rp_plan gives for that
 * query alone: path i goes to path_out + i * path_cap * 9 (n_out[i] states),
 * status_out[i], rc_out[i] = that query's rp_plan code. Returns RP_OK when every
 * query succeeded, else the first failing query's code (the others still ran).
 * The contexts must be idle; they are idle again on return, each holding its last
 * query's scene and stats. */
int rp_plan_many(rp_ctx* const* ctxs, int32_t n_ctx, const rp_query* queries, int32_t n,
                 const double lo[RP_NQ], const double hi[RP_NQ], double* path_out, int32_t path_cap,
                 int32_t* n_out, int32_t* status_out, int32_t* rc_out);

/* Size the planner's device workspace for queries of up to `batch` samples per
 * iteration on trees of `tree_capacity` nodes (0: the rp_plan_params defaults), so
 * that the first such query allocates nothing (hipMalloc / hipFree synchronise the
 * device: milliseconds inside the query otherwise). Buffers only grow; rp_plan
 * grows them itself for anything larger. */
int rp_reserve(rp_ctx* ctx, int64_t batch, int64_t tree_capacity);

/* Batched IK of the hand link: for each of n_targets poses (pos[3], quat[4] as
 * w, x, y, z; world frame, robot base from rp_set_scene) run n_seeds damped-least-
 * squares restarts on the 7 arm joints at once (restart 0 from init[t], the others
 * from seeded samples; fingers stay at init[t]), check the converged ones against
 * the current scene, and return per target the collision-free converged solution
 * closest to init[t] (status RP_IK_OK), else the closest converged one
 * (RP_IK_COLLIDING), else the restart with the smallest pose error
 * (RP_IK_NOT_CONVERGED). q_out: n_targets x 9. */
int rp_ik(rp_ctx* ctx, int32_t n_targets, const double* pos, const double* quat, const double* init,
          const double lo[RP_NQ], const double hi[RP_NQ], const rp_ik_params* params, double* q_out,
          int32_t* status_out);

/* Data-parallel rank group (DESIGN.md §4 "Multi-GPU"; the reference is one process,
 * code/planning.py:121-122). Each rank (one process per GPU) owns one context. Every
 * RRT-Connect iteration then shards its samples across the group: each rank runs the
 * nearest-node searches, steering and edge checks of its slice and packs one
 * 12-byte record per sample; ONE all-gather of the records per iteration lets every
 * rank append the same nodes, so the trees (and the plan) are identical for every
 * world size and equal to the single-rank result.
 *
 * rp_group_init_rccl: the all-gather is an RCCL ncclAllGather on the context stream
 * (xGMI between the GPUs of a node), no host synchronisation besides the
 * iteration's status wait. `id` comes from rp_group_rccl_unique_id on rank 0,
 * broadcast by the caller; every rank must call it (it is collective). Ranks must
 * be on distinct GPUs.
 * rp_group_init: host transport: the records go through library-owned pinned host
 * buffers and `fn` (e.g. torch.distributed gloo); for ranks sharing a GPU and CPU
 * rehearsals. world = 1 (fn may be NULL) returns the context to single-rank
 * planning. */
int rp_group_init(rp_ctx* ctx, int32_t rank, int32_t world, rp_allgather_fn fn, void* user);
/* rp_group_init_shm: shared-memory transport for ranks of ONE node (they may share a
 * GPU): `base` / `bytes` is a host segment every rank has mapped (POSIX shared
 * memory, zero-filled when created); the library registers it with HIP, the pack
 * kernel writes this rank's records into it in place, the ranks meet at a spin
 * barrier on per-rank sequence words in the segment, and the accept kernels read
 * every rank's records from it (no copies, no callback). */
int rp_group_init_shm(rp_ctx* ctx, int32_t rank, int32_t world, void* base, int64_t bytes);
int rp_group_rccl_unique_id(uint8_t id_out[RP_RCCL_ID_BYTES]);
/* rp_group_init_local: a rank group of `world` contexts of ONE process (the drop-in
 * PlannerInterface with planning.configure(devices=[...]): the reference drives one
 * planner from one process, code/motion_primitives.py:38, planning.py:121-122).
 * ctxs[r] becomes rank r. transport RP_TRANSPORT_RCCL: one communicator per context
 * from ncclCommInitAll over their devices (must be distinct; xGMI between the GPUs);
 * RP_TRANSPORT_SHM: a pinned host segment of `bytes` bytes (0: 64 MiB) that the
 * library allocates and every context reads and writes in place (contexts may share
 * a device); RP_TRANSPORT_NONE: RCCL when the devices are distinct, else SHM.
 * Each context plans from its own thread (rp_plan_async on every rank, then
 * rp_plan_wait on every rank); world 1 returns the context to single-rank planning.
 * The segment is freed when the last context leaves the group. */
int rp_group_init_local(rp_ctx* const* ctxs, int32_t world, int32_t transport, int64_t bytes);
int rp_group_init_rccl(rp_ctx* ctx, int32_t rank, int32_t world, const uint8_t id[RP_RCCL_ID_BYTES]);

/* What the context's rank group is, as its transport sees it: for RCCL the
 * communicator's own ncclCommUserRank / ncclCommCount (so a measurement at N GPUs can
 * show that RCCL saw N ranks); otherwise the rank / world given at initialisation.
 * transport: RP_TRANSPORT_*; a context outside any group reports rank 0 of 1, NONE. */
enum { RP_TRANSPORT_NONE = 0, RP_TRANSPORT_HOST = 1, RP_TRANSPORT_RCCL = 2, RP_TRANSPORT_SHM = 3 };
int rp_group_info(rp_ctx* ctx, int32_t* rank_out, int32_t* world_out, int32_t* transport_out);

int rp_get_stats(rp_ctx* ctx, rp_stats* out);

/* Per-kernel-class timing of rp_plan (measurement runs; off by default: the events
 * cost a few microseconds per iteration). rp_get_profile returns the last plan's. */
int rp_set_profiling(rp_ctx* ctx, int32_t on);
int rp_get_profile(rp_ctx* ctx, rp_profile* out);

/* Last error text for this context (or for a failed rp_create when ctx is NULL). */
const char* rp_last_error(rp_ctx* ctx);

/* The context's own HIP stream (hipStream_t; non-blocking). Callers record events on
 * it (e.g. torch.cuda.ExternalStream) to time or order work against the planner's
 * launches without opening another hardware queue. */
int rp_get_stream(rp_ctx* ctx, void** stream_out);

/* Kernel-level timing of the last timed call made with profiling on
 * (rp_set_profiling), measured with HIP events on the launch's stream (ms):
 * rp_check_states_device (the validity kernel), rp_check_edges (the edge launch, no
 * copies), rp_selftest_nn (the search, no copies). RP_ERR_ARG if no such call was
 * made. */
int rp_last_kernel_ms(rp_ctx* ctx, double* ms);

/* Numerics self-test (used by the parity tests): device sqrt(|x|), 0.13037 / x,
 * ceil(7x), (double)(float)x and the forward kinematics' joint sin / cos of
 * (float)x for each x[i] -> out[6*i .. 6*i+5]. The planner's steering and segment
 * counts rely on the first four being IEEE correctly rounded; the last two must
 * equal the oracle's ro_sincos bit for bit. */
int rp_selftest_f64(rp_ctx* ctx, const double* x, int64_t n, double* out);

/* Nearest-node self-test (used by the parity tests): out[i] = the index of the tree
 * state nearest to query i (n x 9 and T x 9 float64, host memory; lowest index among
 * equal squared distances, the oracle's strict-< scan), by the planner's large-tree
 * search with the filter constants of bounds [lo, hi]. mode 0: packed-f32 filter;
 * 1 / 4 / 8: matrix-core filter with 1 / 4 / 8 row blocks of 16 queries per wave. */
int rp_selftest_nn(rp_ctx* ctx, const double* q, int64_t n, const double* tree, int64_t T,
                   const double lo[RP_NQ], const double hi[RP_NQ], int32_t mode, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* RBE_PLANNER_H */
