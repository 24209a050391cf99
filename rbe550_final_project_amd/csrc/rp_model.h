// rp_model.h — compile-time structure of the Franka Panda collision model
// (capsule -> link assignment and self-collision pairs). The numeric geometry
// (endpoints, radii) is runtime data (rp_robot_desc, spec/franka_capsules.json);
// the structure is baked into the kernels so every capsule lives in registers
// with compile-time indices (a runtime-indexed per-thread array would go to
// scratch memory on gfx950). rp_create rejects a descriptor whose structure
// differs from this one.
#pragma once
#include <hip/hip_runtime.h>

namespace rp {

// Work-item / workgroup ids straight from the hardware registers. HIP's threadIdx /
// blockIdx / blockDim / gridDim are device-library calls (__ockl_get_local_id ...),
// and device-library functions are not inlined into code built with
// -mno-amdgpu-ieee (their attributes differ): every use was an s_swappc call (2,400
// call sites in the library, two at the top of every k_validity wave).
__device__ __forceinline__ unsigned rp_tid() { return __builtin_amdgcn_workitem_id_x(); }
__device__ __forceinline__ unsigned rp_bid() { return __builtin_amdgcn_workgroup_id_x(); }
__device__ __forceinline__ unsigned rp_bid_y() { return __builtin_amdgcn_workgroup_id_y(); }
// Block size and workgroup count from the hidden kernel arguments (code object v5:
// hidden_block_count_x at offset 0, hidden_group_size_x at 12 — what HIP's gridDim /
// blockDim read), NOT from the dispatch packet: the packet lives in the AQL queue in
// host memory, so every wave reading it paid a PCIe round trip (the latency kernels'
// grid-stride loops: k_edges_ml<16> 11 -> 24 us per launch, C3 RRT-forced plans
// 0.040 -> 0.065 ms; tools/plan_trace.py A/B, profiles/r03/ids_ab.txt).
__device__ __forceinline__ unsigned rp_bdim() {
    return ((const unsigned short*)__builtin_amdgcn_implicitarg_ptr())[6];
}
__device__ __forceinline__ unsigned rp_gdim() {
    return ((const unsigned*)__builtin_amdgcn_implicitarg_ptr())[0];
}

constexpr int NQ = 9;       // 7 arm joints + 2 fingers (code/planning.py:143-150)
constexpr int NCAP = 12;
constexpr int NLINK = 11;
// link of each capsule: link0..link4, link5 (x2), link6, link7, hand, fingers
constexpr int CAP_LINK[NCAP] = {0, 1, 2, 3, 4, 5, 5, 6, 7, 8, 9, 10};

enum : int {
    C_LINK0 = 0, C_LINK1, C_LINK2, C_LINK3, C_LINK4, C_LINK5A, C_LINK5B,
    C_LINK6, C_LINK7, C_HAND, C_LFINGER, C_RFINGER
};

constexpr int NPAIR = 35;
constexpr int PAIRS[NPAIR][2] = {
    {C_LINK0, C_LINK5B}, {C_LINK0, C_LINK6}, {C_LINK0, C_LINK7}, {C_LINK0, C_HAND},
    {C_LINK0, C_LFINGER}, {C_LINK0, C_RFINGER},
    {C_LINK1, C_LINK5A}, {C_LINK1, C_LINK5B}, {C_LINK1, C_LINK6}, {C_LINK1, C_LINK7},
    {C_LINK1, C_HAND}, {C_LINK1, C_LFINGER}, {C_LINK1, C_RFINGER},
    {C_LINK2, C_LINK5A}, {C_LINK2, C_LINK5B}, {C_LINK2, C_LINK6}, {C_LINK2, C_LINK7},
    {C_LINK2, C_HAND}, {C_LINK2, C_LFINGER}, {C_LINK2, C_RFINGER},
    {C_LINK3, C_LINK6}, {C_LINK3, C_LINK7}, {C_LINK3, C_HAND}, {C_LINK3, C_LFINGER},
    {C_LINK3, C_RFINGER},
    {C_LINK4, C_LINK7}, {C_LINK4, C_HAND}, {C_LINK4, C_LFINGER}, {C_LINK4, C_RFINGER},
    {C_LINK5A, C_HAND}, {C_LINK5A, C_LFINGER}, {C_LINK5A, C_RFINGER},
    {C_LINK5B, C_HAND}, {C_LINK5B, C_LFINGER}, {C_LINK5B, C_RFINGER},
};

// Joint limits as float32 (model.py Q_LO / Q_HI: Genesis keeps q_limit in float32).
constexpr float Q_LO_F[NQ] = {-2.8973f, -1.7628f, -2.8973f, -3.0718f, -2.8973f, -0.0175f, -2.8973f, 0.0f, 0.0f};
constexpr float Q_HI_F[NQ] = {2.8973f, 1.7628f, 2.8973f, -0.0698f, 2.8973f, 3.7525f, 2.8973f, 0.04f, 0.04f};

// Self pairs proven never to touch while every joint is inside [Q_LO_F, Q_HI_F]
// (tools/prove_pairs.py: exact segment distance on a joint grid minus a Lipschitz
// bound exceeds r_I + r_J + 1e-4 m; tests/golden/never_pairs_proof.json). A wave
// whose states are all inside the limits skips them; any other wave tests them.
constexpr int NEVER_PAIRS[][2] = {
    {C_LINK2, C_LINK5A}, {C_LINK3, C_LINK6}, {C_LINK3, C_LINK7}, {C_LINK4, C_LINK7}, {C_LINK4, C_HAND},
    {C_LINK4, C_LFINGER}, {C_LINK4, C_RFINGER}, {C_LINK5B, C_HAND}, {C_LINK5B, C_LFINGER}, {C_LINK5B, C_RFINGER},
};
constexpr bool pair_never(int p) {
    for (const auto& n : NEVER_PAIRS)
        if (n[0] == PAIRS[p][0] && n[1] == PAIRS[p][1]) return true;
    return false;
}

// Reach of each capsule while every joint is inside [Q_LO_F, Q_HI_F] (tools/
// prove_reach.py, tests/golden/reach_proof.json): every point of capsule C lies
// within REACH[C] metres of the robot base (C = 0, a fixed capsule) or of the
// shoulder, base + (0, 0, 0.333) (every other capsule: on joint 1's axis, so q0
// moves no point towards or away from it). Grid maximum + Lipschitz slack for the
// capsules moved by <= 4 joints, the chain sum for the others; radius included;
// rounded up to float.
constexpr float REACH[NCAP] = {0.168167f, 0.253000f, 0.120006f, 0.306792f, 0.398614f, 0.681955f,
                               0.802594f, 0.911263f, 0.999263f, 1.090294f, 1.136424f, 1.136424f};
constexpr float SHOULDER_Z = 0.333f;

// Capsule geometry (spec/franka_capsules.json): a(3), b(3), radius, in the link
// frame. Compiled into the kernels (zero terms of the link->world transform fold
// away, no scalar loads); rp_create rejects a descriptor with other numbers.
constexpr float CAP_GEOM[NCAP][7] = {
    {-0.09f, 0.0f, 0.06f, -0.06f, 0.0f, 0.06f, 0.06f},       // link0
    {0.0f, 0.0f, -0.193f, 0.0f, 0.0f, -0.05f, 0.06f},        // link1
    {0.0f, 0.0f, -0.06f, 0.0f, 0.0f, 0.06f, 0.06f},          // link2
    {0.0f, 0.0f, -0.22f, 0.0f, 0.0f, -0.07f, 0.06f},         // link3
    {0.0f, 0.0f, -0.06f, 0.0f, 0.0f, 0.06f, 0.06f},          // link4
    {0.0f, 0.0f, -0.31f, 0.0f, 0.0f, -0.21f, 0.06f},         // link5a
    {0.0f, 0.08f, -0.20f, 0.0f, 0.08f, -0.06f, 0.025f},      // link5b
    {0.0f, 0.0f, -0.07f, 0.0f, 0.0f, 0.01f, 0.05f},          // link6
    {0.0f, 0.0f, -0.06f, 0.0f, 0.0f, 0.08f, 0.04f},          // link7
    {0.0f, -0.05f, 0.04f, 0.0f, 0.05f, 0.04f, 0.04f},        // hand
    {0.0f, 0.012f, 0.012f, 0.0f, 0.012f, 0.040f, 0.010f},    // left finger
    {0.0f, 0.012f, 0.012f, 0.0f, 0.012f, 0.040f, 0.010f},    // right finger
};

constexpr int MAX_BOXES = 64;
constexpr int GRID_MIN_BOXES = 16;   // scenes with more boxes use the axis-grid broad phase
constexpr int CLUSTER = 8;                       // boxes per broad-phase cluster
constexpr int MAX_CLUSTERS = MAX_BOXES / CLUSTER;

// Device scene record (one constant buffer, read by wave-uniform scalar loads).
// Box record: 16 floats so one s_load_dwordx16 fetches it.
//   [0..2] centre  [3..5] half extents  [6] cos(yaw) [7] sin(yaw)
//   [8..10] world AABB lo  [11..13] world AABB hi  [14] exempt-capsule bits (bits
//   0..NCAP-1) | BOX_TILTED  [15] index of the box in the caller's order (boxes are
//   stored cluster-sorted)
// A tilted box (rp_set_scene_rot with a rotation that moves the z axis: a toppled
// or leaning block) has BOX_TILTED set and its world -> box rotation in rot[slot]:
// rows of R^T (row i = box axis i in world coordinates), 9 floats; [6], [7] unused.
// Upright boxes keep the yaw transform (no extra loads or VALU in the hot path).
constexpr unsigned BOX_TILTED = 0x80000000u;
// Cluster record: [0..2] AABB lo, [4..6] AABB hi (union of its boxes' AABBs),
//   [3] first box, [7] box count (as int bits).
// Axis grid (many-box scenes, `grid` = 1): per axis, GRID_CELLS cells over the
//   boxes' extent; grid_lo[a][c] = boxes whose AABB-lo cell is <= c (widened by
//   one cell), grid_hi[a][c] = boxes whose AABB-hi cell is >= c (widened). For a
//   capsule AABB [u, v], grid_lo[a][cell(v)] & grid_hi[a][cell(u)] over the three
//   axes is a superset of the boxes whose AABB overlaps it (cell() is monotone;
//   the widening absorbs any host/device rounding difference), so the exact AABB
//   test on that superset finds exactly the boxes the full scan would.
constexpr int GRID_CELLS = 64;
constexpr int ML_UNITS_PAD = (NPAIR + NCAP * MAX_BOXES + 7) / 8 * 8;   // 808: whole 16-B words
struct DevScene {
    float box[MAX_BOXES][16];
    float rot[MAX_BOXES][12];    // tilted boxes: R^T rows (9 floats), pad
    float cluster[MAX_CLUSTERS][8];
    float base[4];               // robot base translation (scenes.py:29-34), pad
    float plane_z;
    int n_boxes;
    int n_clusters;
    int grid;                    // 1: broad phase through the axis grid
    unsigned env_far;            // bit C: capsule C can reach no box (REACH; rp_lib.hip env_far_mask)
    float grid_o[4];             // per-axis origin, pad
    float grid_s[4];             // per-axis cells per metre, pad
    unsigned long long grid_lo[3][GRID_CELLS];
    unsigned long long grid_hi[3][GRID_CELLS];
    // test units of the lane-group kernels (rp_math.h state_collides_ml) for waves
    // whose states are all inside the joint limits: the self pairs that are not never
    // pairs, then capsule x box for the capsules that can reach a box (env_far clear);
    // unit u < NPAIR is self pair u, else capsule (u - NPAIR) / n_boxes vs box
    // (u - NPAIR) % n_boxes (rp_lib.hip upload_scene)
    int ml_n;
    alignas(16) unsigned short ml_unit[ML_UNITS_PAD];
};

// cell of coordinate v on an axis with origin o and scale s (cells per metre),
// clamped to [0, GRID_CELLS - 1]; monotone in v. Shared by host and device.
__host__ __device__ inline int grid_cell(float v, float o, float s) {
    float t = (v - o) * s;
    t = t < 0.0f ? 0.0f : t;
    t = t > (float)(GRID_CELLS - 1) ? (float)(GRID_CELLS - 1) : t;
    return (int)t;
}

}  // namespace rp
