/*
 * rbe_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's state-validity / plan path, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
 * It is never linked into, loaded by, or called from the product library
 * (librbe_mi355x.so) or rbe550_final_project_amd/ — the product has no CPU path.
 *
 * What it restates (reference file:line):
 *   ro_state_valid   _is_ompl_state_valid + collision_with_attached_object
 *                    code/planning.py:209-230 (Genesis FK + collider [EXT-GS],
 *                    capsule model of spec/franka_capsules.json)
 *   ro_check_edge    OMPL DiscreteMotionValidator::checkMotion used inside
 *                    ss.solve (code/planning.py:190) [EXT-OMPL, SURVEY App. B.2]
 *   ro_plan          plan_path (code/planning.py:139-200): RRTConnect
 *                    [EXT-OMPL, App. B.3] in the batched form of DESIGN.md §4,
 *                    simplifySolution (greedy vertex reduction),
 *                    PathGeometric::interpolate [EXT-OMPL, App. B.4]
 *
 * Parity status: OMPL and Genesis are absent here and the reference ships no
 * golden vectors for this arithmetic, so parity with the reference's numbers is
 * UNPINNED; the oracle is pinned by (a) the FK known answers of SURVEY.md A.3,
 * (b) Random123 Philox4x32-10 known answers, (c) the exemption truth table
 * produced by running the reference's own planning.py with stubbed genesis/ompl
 * (tests/golden/make_reference_fixtures.py).
 */
#ifndef RBE_ORACLE_H
#define RBE_ORACLE_H
#include <stdint.h>
#include "../include/rbe_planner.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ro_scene ro_scene;

ro_scene* ro_scene_create(const rp_robot_desc* robot);
void ro_scene_destroy(ro_scene* s);
int ro_scene_set(ro_scene* s, const rp_box* boxes, int32_t n_boxes, float plane_z,
                 const float base_pos[3]);
int ro_scene_set_rot(ro_scene* s, const rp_box_rot* boxes, int32_t n_boxes, float plane_z,
                     const float base_pos[3]);
int ro_scene_set_attached(ro_scene* s, int32_t box_index, uint32_t exempt_link_mask);

/* 1 = valid (collision free). */
int ro_state_valid(const ro_scene* s, const float q[RP_NQ]);
/* n states row-major; returns number of states evaluated. threads <= 0: all cores. */
int64_t ro_check_states(const ro_scene* s, const float* q, int64_t n, uint8_t* flags, int threads);
/* world capsule endpoints (12 x 6 floats) for FK tests */
void ro_fk_capsules(const ro_scene* s, const float q[RP_NQ], float* out72);
/* sin/cos of the shared polynomial */
void ro_sincos(float x, float* s, float* c);
/* Philox4x32-10 */
void ro_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* checkMotion(qa -> qb) (qb + interior checked). Returns 1 if valid. *states counts. */
int ro_check_edge(const ro_scene* s, const double* qa, const double* qb, double resolution,
                  int64_t* states);
int64_t ro_check_edges(const ro_scene* s, const double* qa, const double* qb, int64_t n,
                       double resolution, uint8_t* out);

/* Contacts for diagnostics (same encoding as rp_state_contacts). */
int ro_state_contacts(const ro_scene* s, const double q[RP_NQ], int32_t* pairs_out, int32_t cap);

/* Rank-group all-gather over host buffers (see rp_group_init). */
typedef int (*ro_allgather_fn)(void* user, const void* send, void* recv, int64_t bytes_per_rank);

int ro_plan(const ro_scene* s, const double start[RP_NQ], const double goal[RP_NQ],
            const double lo[RP_NQ], const double hi[RP_NQ], const rp_plan_params* p,
            int32_t rank, int32_t world, ro_allgather_fn fn, void* user,
            double* path_out, int32_t path_cap, int32_t* n_out, int32_t* status_out,
            rp_stats* stats);

/* geometry primitives (unit tests) */
/* batched hand-link IK, the algorithm of rp_ik (rbe550_final_project_amd/csrc/rp_ik.h) */
int ro_ik(const ro_scene* s, int32_t n_targets, const double* pos, const double* quat, const double* init,
          const double lo[RP_NQ], const double hi[RP_NQ], const rp_ik_params* params, double* q_out,
          int32_t* status_out);
/* hand pose of an arm configuration: R (row-major 3x3), p (3) */
void ro_hand_pose(const ro_scene* s, const double q[RP_NQ], double R[9], double p[3]);
/* float64 polynomial sin / cos of the IK */
void ro_sincos64(double x, double* s, double* c);

float ro_seg_box_d2(const float a[3], const float b[3], const float h[3]);
float ro_seg_seg_d2(const float a1[3], const float b1[3], const float a2[3], const float b2[3]);

/* PathGeometric::interpolate(count) on a path (in place into out, cap states). */
int ro_interpolate(const double* path, int32_t n, int32_t count, double* out, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif
