// rp_math.h — device arithmetic of the state-validity hot path (gfx950).
//
// Replaces what one reference validity callback triggers (code/planning.py:209-230):
//   robot.set_qpos(q)         -> Genesis FK kernel            => fk_capsules()
//   robot.detect_collision()  -> Genesis broad+narrow phase   => state_collides()
//   collision_with_attached_object()                          => per-box exempt bits
//
// Numerics contract: float32; every operation written out in a fixed
// order with explicit fused multiply-adds (fmaf, one rounding) and otherwise plain
// IEEE ops; compiled with -ffp-contract=off so the compiler adds no other fusion.
// The CPU oracle (oracle/rbe_oracle.c) restates the same sequence with C99 fmaf, so
// flags are bit-identical. sin/cos come from rp_sincos() (polynomial), never libm.
//
// Code shape: FK and the broad phases are straight-line code; the two narrow phases
// (segment-box, segment-segment) are single out-of-line functions: they run only
// for overlapping AABBs, and inlining them at 12 + 35 call sites made a 12k-
// instruction kernel that thrashed the instruction cache.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rp_model.h"

namespace rp {

struct V3 { float x, y, z; };

#ifdef RP_STAMPS
// in-kernel timestamps (diagnostic builds only): lane 0 of each k_validity wave
// writes s_memtime at fixed points into g_stamps[wave][k] (vector store)
constexpr int STAMP_WAVES = 65536, STAMP_K = 8;
__device__ unsigned long long g_stamps[STAMP_WAVES * STAMP_K];
__device__ __forceinline__ void stamp(int k) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    const unsigned w = rp_bid();
    if (w < STAMP_WAVES && __lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) g_stamps[w * STAMP_K + k] = t;
}
#define RP_STAMP(k) stamp(k)
// single-block kernels of the plan path: lane 0 of the block records
// s_memrealtime (100 MHz) at point k of kernel slot `kid` (g_tstamps[kid][k])
constexpr int TSTAMP_K = 16;
__device__ unsigned long long g_tstamps[8 * TSTAMP_K];
__device__ __forceinline__ void tstamp(int kid, int k) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (rp_tid() == 0 && rp_bid() == 0) g_tstamps[kid * TSTAMP_K + k] = t;
}
#define RP_TSTAMP(kid, k) tstamp(kid, k)
// per-block stamps of a multi-block plan kernel (k_edges_ml: one wave per block)
constexpr int ESTAMP_BLOCKS = 4096, ESTAMP_K = 16;
__device__ unsigned long long g_estamps[ESTAMP_BLOCKS * ESTAMP_K];
__device__ __forceinline__ void estamp(int k) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    if (rp_tid() == 0 && rp_bid() < ESTAMP_BLOCKS) g_estamps[rp_bid() * ESTAMP_K + k] = t;
}
#define RP_ESTAMP(k) estamp(k)
#else
#define RP_STAMP(k)
#define RP_TSTAMP(kid, k)
#define RP_ESTAMP(k)
#endif

// min / max / clamp as single instructions (v_min_f32, v_max_f32, v_med3_f32). The
// oracle writes them as compares; for the finite operands here the two agree except
// possibly in the sign of a zero result, which no later comparison or square sees.
__device__ __forceinline__ float fminr(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float fmaxr(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ float clampr(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ float clamp01(float x) { return clampr(x, 0.0f, 1.0f); }
__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
// (u . v) = fma(uz, vz, fma(uy, vy, ux * vx))
__device__ __forceinline__ float dot3(V3 u, V3 v) { return fma_(u.z, v.z, fma_(u.y, v.y, u.x * v.x)); }

// sin and cos of x, |x| < ~100: quadrant reduction with a 3-part pi/2 (FMA
// Cody-Waite), then minimax polynomials on [-pi/4, pi/4].
__device__ __forceinline__ void rp_sincos(float x, float* sn, float* cs) {
    const float k = floorf(x * 0.636619772f + 0.5f);
    float r = fma_(-k, 1.5703125f, x);
    r = fma_(-k, 4.837512969970703125e-4f, r);
    r = fma_(-k, 7.54978995489188216e-8f, r);
    const float z = r * r;
    const float ps = fma_(fma_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sr = fma_(r * z, ps, r);
    const float pc = fma_(fma_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    const float cr = fma_(z * z, pc, fma_(-0.5f, z, 1.0f));
    // The quadrant is read from the bits of this same rounded k (k + 1.5 x 2^23 holds
    // k's two's-complement low bits, |k| < 2^22), not converted: the compiler folds
    // (int)floorf(y + 0.5f) into v_cvt_rpi_i32_f32(y), which rounds y + 0.5 exactly
    // instead of to f32 — at x = 0.785398126 (the float just below pi/4) the f32 sum is
    // 1.0 but the exact one is below 1, so the reduction used k = 1 with the quadrant of
    // k = 0 and sin came out negated (-0.7071; the oracle: k = 1 throughout). Found by an
    // edge-parity seed; it also changed flags of the bench's own uniform states. An empty
    // asm barrier on k fixed it too but cost 14 % of k_validity; this form costs nothing
    // (profiles/r05/sincos_fix_ab.txt; tests/test_gpu_parity.py::test_sincos_quadrant_bounds).
    const int qd = __float_as_int(k + 12582912.0f) & 3;
    // quadrant by bits: odd quadrants swap sin and cos, quadrants 2 and 3 negate sin,
    // 1 and 2 negate cos (the oracle's case analysis, the same values; as selects and
    // sign-bit XORs instead of a branchy case analysis: -63 SALU, -35 VALU per wave,
    // +4 % goal3)
    const bool odd = qd & 1;
    const float s0 = odd ? cr : sr, c0 = odd ? sr : cr;
    *sn = __uint_as_float(__float_as_uint(s0) ^ ((unsigned)(qd & 2) << 30));
    *cs = __uint_as_float(__float_as_uint(c0) ^ ((unsigned)((qd + 1) & 2) << 30));
}

// A rigid frame: rotation columns c0, c1, c2 and origin p (world).
struct Frame { V3 c0, c1, c2, p; };

// R <- R * Rz(angle) given (s, c): n0 = c*c0 + s*c1, n1 = c*c1 - s*c0
__device__ __forceinline__ void rot_sc(Frame& f, float s, float c) {
    V3 n0, n1;
    n0.x = fma_(c, f.c0.x, s * f.c1.x);
    n0.y = fma_(c, f.c0.y, s * f.c1.y);
    n0.z = fma_(c, f.c0.z, s * f.c1.z);
    n1.x = fma_(c, f.c1.x, -(s * f.c0.x));
    n1.y = fma_(c, f.c1.y, -(s * f.c0.y));
    n1.z = fma_(c, f.c1.z, -(s * f.c0.z));
    f.c0 = n0;
    f.c1 = n1;
}
__device__ __forceinline__ void rot_z(Frame& f, float q) {
    float s, c;
    rp_sincos(q, &s, &c);
    rot_sc(f, s, c);
}
// R <- R * Rx(+90deg): [c0, c2, -c1]
__device__ __forceinline__ void rot_xp(Frame& f) {
    V3 t = f.c1;
    f.c1 = f.c2;
    f.c2.x = -t.x; f.c2.y = -t.y; f.c2.z = -t.z;
}
// R <- R * Rx(-90deg): [c0, -c2, c1]
__device__ __forceinline__ void rot_xm(Frame& f) {
    V3 t = f.c2;
    f.c2 = f.c1;
    f.c1.x = -t.x; f.c1.y = -t.y; f.c1.z = -t.z;
}
// p <- p + k * col
__device__ __forceinline__ void shift(V3& p, float k, V3 col) {
    p.x = fma_(k, col.x, p.x);
    p.y = fma_(k, col.y, p.y);
    p.z = fma_(k, col.z, p.z);
}
// world point of link-frame point (a0, a1, a2)
__device__ __forceinline__ V3 xform(const Frame& f, float a0, float a1, float a2) {
    V3 w;
    w.x = fma_(a2, f.c2.x, fma_(a1, f.c1.x, fma_(a0, f.c0.x, f.p.x)));
    w.y = fma_(a2, f.c2.y, fma_(a1, f.c1.y, fma_(a0, f.c0.y, f.p.y)));
    w.z = fma_(a2, f.c2.z, fma_(a1, f.c1.z, fma_(a0, f.c0.z, f.p.z)));
    return w;
}

// a, b: segment endpoints (world); m = a + b (twice the centre: the self-pair
// sphere prefilter's operand, made once per capsule instead of once per pair)
struct Capsules { V3 a[NCAP]; V3 b[NCAP]; V3 m[NCAP]; };

// fma(a2, c2, fma(a1, c1, fma(a0, c0, p))) with compile-time a: a zero term is
// skipped (fma(0, x, p) == p for finite x, up to the sign of a zero result, which
// no later comparison can observe).
template <int C, int O>
__device__ __forceinline__ V3 xform_c(const Frame& f) {
    constexpr float a0 = CAP_GEOM[C][O], a1 = CAP_GEOM[C][O + 1], a2 = CAP_GEOM[C][O + 2];
    V3 w = f.p;
    if constexpr (a0 != 0.0f) { w.x = fma_(a0, f.c0.x, w.x); w.y = fma_(a0, f.c0.y, w.y); w.z = fma_(a0, f.c0.z, w.z); }
    if constexpr (a1 != 0.0f) { w.x = fma_(a1, f.c1.x, w.x); w.y = fma_(a1, f.c1.y, w.y); w.z = fma_(a1, f.c1.z, w.z); }
    if constexpr (a2 != 0.0f) { w.x = fma_(a2, f.c2.x, w.x); w.y = fma_(a2, f.c2.y, w.y); w.z = fma_(a2, f.c2.z, w.z); }
    return w;
}

template <int C>
__device__ __forceinline__ void place(Capsules& k, const Frame& f) {
    k.a[C] = xform_c<C, 0>(f);
    k.b[C] = xform_c<C, 3>(f);
    k.m[C] = {k.a[C].x + k.b[C].x, k.a[C].y + k.b[C].y, k.a[C].z + k.b[C].z};   // (dead unless a sphere uses it)
}
// Franka Panda forward kinematics (MJCF bodies of
// panda.xml that Genesis loads at code/scenes.py:85) -> world capsule endpoints.
// After each capsule is placed, v.template at<C>(k) runs; a true return stops the
// walk (a collision found: the rest of the chain is not needed). Capsules whose
// last use has passed are dead, so their registers are reused.
// BF (base fixed): the robot base is the reference's (0, 0, 0.01) (scenes.py:29-34),
// a compile-time constant, so everything that depends on the base alone (link0 and
// link1's capsules, the shoulder position) folds into literals and takes no
// registers; the values are the ones the runtime base gives
constexpr float BASE_FIXED[3] = {0.0f, 0.0f, 0.01f};
// joint angle source of the walk: sin / cos of joint i from q (rp_sincos), or
// precomputed values (the low-latency kernels compute the 7 in parallel lanes;
// the same function of q, so the same bits)
struct JointsQ {
    const float* q;
    __device__ __forceinline__ void rot(Frame& f, int i) const { rot_z(f, q[i]); }
};
struct JointsSC {
    float s[7], c[7];
    __device__ __forceinline__ void rot(Frame& f, int i) const { rot_sc(f, s[i], c[i]); }
};
template <class Visit, bool BF = false, class J = JointsQ>
__device__ __forceinline__ bool fk_walk_j(const float q[NQ], const J& jt, const float* base, Capsules& k,
                                          Visit& v) {
    Frame f;
    f.c0 = {1.0f, 0.0f, 0.0f};
    f.c1 = {0.0f, 1.0f, 0.0f};
    f.c2 = {0.0f, 0.0f, 1.0f};
    if constexpr (BF) f.p = {BASE_FIXED[0], BASE_FIXED[1], BASE_FIXED[2]};
    else f.p = {base[0], base[1], base[2]};
    place<C_LINK0>(k, f);
    if (v.template at<C_LINK0>(k)) return true;
    shift(f.p, 0.333f, f.c2);               // link1: pos (0,0,0.333), joint 1
    jt.rot(f, 0);
    place<C_LINK1>(k, f);
    if (v.template at<C_LINK1>(k)) return true;
    rot_xm(f);                              // link2: quat (1,-1,0,0) = Rx(-90), joint 2
    jt.rot(f, 1);
    place<C_LINK2>(k, f);
    if (v.template at<C_LINK2>(k)) return true;
    shift(f.p, -0.316f, f.c1);              // link3: pos (0,-0.316,0), Rx(+90), joint 3
    rot_xp(f);
    jt.rot(f, 2);
    place<C_LINK3>(k, f);
    if (v.template at<C_LINK3>(k)) return true;
    shift(f.p, 0.0825f, f.c0);              // link4: pos (0.0825,0,0), Rx(+90), joint 4
    rot_xp(f);
    jt.rot(f, 3);
    place<C_LINK4>(k, f);
    if (v.template at<C_LINK4>(k)) return true;
    shift(f.p, -0.0825f, f.c0);             // link5: pos (-0.0825,0.384,0), Rx(-90), joint 5
    shift(f.p, 0.384f, f.c1);
    rot_xm(f);
    jt.rot(f, 4);
    place<C_LINK5A>(k, f);
    if (v.template at<C_LINK5A>(k)) return true;
    place<C_LINK5B>(k, f);
    if (v.template at<C_LINK5B>(k)) return true;
    rot_xp(f);                              // link6: Rx(+90), joint 6
    jt.rot(f, 5);
    place<C_LINK6>(k, f);
    if (v.template at<C_LINK6>(k)) return true;
    shift(f.p, 0.088f, f.c0);               // link7: pos (0.088,0,0), Rx(+90), joint 7
    rot_xp(f);
    jt.rot(f, 6);
    place<C_LINK7>(k, f);
    if (v.template at<C_LINK7>(k)) return true;
    shift(f.p, 0.107f, f.c2);               // hand: pos (0,0,0.107), Rz(-45deg)
    rot_sc(f, -0.70710677f, 0.70710677f);
    place<C_HAND>(k, f);
    if (v.template at<C_HAND>(k)) return true;
    shift(f.p, 0.0584f, f.c2);              // fingers: (0,0,0.0584), prismatic +-hand y
    {
        Frame l = f;
        shift(l.p, q[7], f.c1);
        place<C_LFINGER>(k, l);
        if (v.template at<C_LFINGER>(k)) return true;
        Frame r = f;
        shift(r.p, -q[8], f.c1);
        r.c0.x = -f.c0.x; r.c0.y = -f.c0.y; r.c0.z = -f.c0.z;  // Rz(180)
        r.c1.x = -f.c1.x; r.c1.y = -f.c1.y; r.c1.z = -f.c1.z;
        place<C_RFINGER>(k, r);
        if (v.template at<C_RFINGER>(k)) return true;
    }
    return false;
}
template <class Visit, bool BF = false, class SC = DevScene>
__device__ __forceinline__ bool fk_walk(const float q[NQ], const SC* __restrict__ sc, Capsules& k,
                                        Visit& v) {
    const JointsQ jt{q};
    return fk_walk_j<Visit, BF>(q, jt, sc->base, k, v);
}

struct NoVisit {
    template <int C>
    __device__ __forceinline__ bool at(const Capsules&) { return false; }
};

template <class SC = DevScene>
__device__ __forceinline__ void fk_capsules(const float q[NQ], const SC* __restrict__ sc, Capsules& k) {
    NoVisit v;
    fk_walk<NoVisit, false, SC>(q, sc, k, v);
}

// Capsule AABB expanded by its radius.
struct Aabb { V3 lo, hi; };
__device__ __forceinline__ Aabb capsule_aabb(V3 a, V3 b, float r) {
    Aabb o;
    o.lo.x = fminr(a.x, b.x) - r; o.hi.x = fmaxr(a.x, b.x) + r;
    o.lo.y = fminr(a.y, b.y) - r; o.hi.y = fmaxr(a.y, b.y) + r;
    o.lo.z = fminr(a.z, b.z) - r; o.hi.z = fmaxr(a.z, b.z) + r;
    return o;
}
// separation of capsule AABB u from box [lo, hi]: > 0 iff disjoint (max of the six
// interval differences; see aabb_disjoint)
__device__ __forceinline__ float aabb_sep(const Aabb& u, const float* lo, const float* hi) {
    const float a = fmaxr(fmaxr(u.lo.x - hi[0], lo[0] - u.hi.x), fmaxr(u.lo.y - hi[1], lo[1] - u.hi.y));
    return fmaxr(a, fmaxr(u.lo.z - hi[2], lo[2] - u.hi.z));
}
// The six interval tests as one max of differences: for finite (or infinite, never
// NaN) operands with subnormals kept, x - y > 0 <=> x > y (x != y => x - y != 0), so
// the result is the same bool. One compare instead of six compares whose lane masks
// are ORed by scalar instructions (each VALU -> SGPR -> SALU hop waits in a lone
// wave's chain): A/B +3 % goal3 4M states, +1.6 % clutter64, +10 % at 64k states
// (-DRP_AABB_CMP builds the compare form).
__device__ __forceinline__ bool aabb_disjoint(const Aabb& u, const float* lo, const float* hi) {
    const float a = fmaxr(fmaxr(u.lo.x - hi[0], lo[0] - u.hi.x), fmaxr(u.lo.y - hi[1], lo[1] - u.hi.y));
    const float b = fmaxr(u.lo.z - hi[2], lo[2] - u.hi.z);
    return fmaxr(a, b) > 0.0f;
}
__device__ __forceinline__ bool aabb_disjoint2(const Aabb& u, const Aabb& v) {
    const float a = fmaxr(fmaxr(u.lo.x - v.hi.x, v.lo.x - u.hi.x), fmaxr(u.lo.y - v.hi.y, v.lo.y - u.hi.y));
    const float b = fmaxr(u.lo.z - v.hi.z, v.lo.z - u.hi.z);
    return fmaxr(a, b) > 0.0f;
}

// g(t) = q(t) . d with q the excess of a + t d over the box [-h, h]; also |q|^2.
__device__ __forceinline__ float excess_dot(V3 a, V3 d, V3 h, float t, float* f2) {
    const float px = fma_(t, d.x, a.x), py = fma_(t, d.y, a.y), pz = fma_(t, d.z, a.z);
    const float cx = clampr(px, -h.x, h.x);
    const float cy = clampr(py, -h.y, h.y);
    const float cz = clampr(pz, -h.z, h.z);
    const V3 qv = {px - cx, py - cy, pz - cz};
    *f2 = dot3(qv, qv);
    return dot3(qv, d);
}

// Segment a-b (box frame) vs box [-h, h]: the squared distance is a convex piecewise
// quadratic in t with C^1 joins; its derivative g is piecewise linear and
// nondecreasing with breakpoints where a coordinate crosses +-h. Locate the root of
// g between the sorted breakpoints and interpolate linearly inside that piece.
__device__ __forceinline__ float segment_box_dist2_body(V3 a, V3 b, V3 h) {
    const V3 d = {b.x - a.x, b.y - a.y, b.z - a.z};
    float T[6];
    {
        float u = 0.0f, v = 0.0f;
        if (d.x != 0.0f) { const float inv = 1.0f / d.x; u = (-h.x - a.x) * inv; v = (h.x - a.x) * inv; }
        T[0] = clamp01(u); T[1] = clamp01(v);
        u = 0.0f; v = 0.0f;
        if (d.y != 0.0f) { const float inv = 1.0f / d.y; u = (-h.y - a.y) * inv; v = (h.y - a.y) * inv; }
        T[2] = clamp01(u); T[3] = clamp01(v);
        u = 0.0f; v = 0.0f;
        if (d.z != 0.0f) { const float inv = 1.0f / d.z; u = (-h.z - a.z) * inv; v = (h.z - a.z) * inv; }
        T[4] = clamp01(u); T[5] = clamp01(v);
    }
    // sorting network (12 exchanges) — the sorted multiset is order independent
#define RP_CX(i, j) { const float lo_ = fminr(T[i], T[j]); const float hi_ = fmaxr(T[i], T[j]); T[i] = lo_; T[j] = hi_; }
    RP_CX(0, 1) RP_CX(2, 3) RP_CX(4, 5) RP_CX(0, 2) RP_CX(3, 5) RP_CX(1, 4)
    RP_CX(0, 1) RP_CX(2, 3) RP_CX(4, 5) RP_CX(1, 2) RP_CX(3, 4) RP_CX(2, 3)
#undef RP_CX
    float f2;
    const float g0 = excess_dot(a, d, h, 0.0f, &f2);
    if (g0 >= 0.0f) return f2;
    float f2e;
    const float g7 = excess_dot(a, d, h, 1.0f, &f2e);
    if (g7 <= 0.0f) return f2e;
    float tl = 0.0f, gl = g0, tk = 1.0f, gk = g7;
    bool found = false;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        float fi;
        const float gi = excess_dot(a, d, h, T[i], &fi);
        if (!found) {
            if (gi >= 0.0f) { found = true; tk = T[i]; gk = gi; }
            else { tl = T[i]; gl = gi; }
        }
    }
    const float ts = fma_(tk - tl, (-gl) / (gk - gl), tl);
    excess_dot(a, d, h, ts, &f2);
    return f2;
}

// Closest distance^2 between segments a1-b1 and a2-b2.
__device__ __forceinline__ float segment_segment_dist2_body(V3 a1, V3 b1, V3 a2, V3 b2) {
    const V3 d1 = {b1.x - a1.x, b1.y - a1.y, b1.z - a1.z};
    const V3 d2 = {b2.x - a2.x, b2.y - a2.y, b2.z - a2.z};
    const V3 w = {a1.x - a2.x, a1.y - a2.y, a1.z - a2.z};
    const float A = dot3(d1, d1), E = dot3(d2, d2), F = dot3(d2, w);
    float s, t;
    if (A <= 1e-12f) {
        s = 0.0f;
        t = (E <= 1e-12f) ? 0.0f : clamp01(F / E);
    } else {
        const float C = dot3(d1, w);
        if (E <= 1e-12f) {
            t = 0.0f;
            s = clamp01(-C / A);
        } else {
            const float B = dot3(d1, d2);
            const float den = fma_(A, E, -(B * B));
            s = den > 0.0f ? clamp01(fma_(B, F, -(C * E)) / den) : 0.0f;
            const float tn = fma_(B, s, F);
            if (tn < 0.0f) { t = 0.0f; s = clamp01(-C / A); }
            else if (tn > E) { t = 1.0f; s = clamp01((B - C) / A); }
            else { t = tn / E; }
        }
    }
    const V3 p1 = {fma_(d1.x, s, a1.x), fma_(d1.y, s, a1.y), fma_(d1.z, s, a1.z)};
    const V3 p2 = {fma_(d2.x, t, a2.x), fma_(d2.y, t, a2.y), fma_(d2.z, t, a2.z)};
    const V3 dd = {p1.x - p2.x, p1.y - p2.y, p1.z - p2.z};
    return dot3(dd, dd);
}

// The throughput kernels call the narrow phases as functions (one copy each instead
// of one per call site: 35 pair sites in k_validity); the lane-group kernels, with
// a couple of sites, inline them (a call there costs more than the code size saves).
__device__ __attribute__((noinline)) float segment_box_dist2(V3 a, V3 b, V3 h) {
    return segment_box_dist2_body(a, b, h);
}
__device__ __attribute__((noinline)) float segment_segment_dist2(V3 a1, V3 b1, V3 a2, V3 b2) {
    return segment_segment_dist2_body(a1, b1, a2, b2);
}

// World point p in the frame of box record bx. Upright box: rotation by -yaw about
// z (cos / sin in bx[6], bx[7]). Tilted box (BOX_TILTED in bx[14]): the rows of R^T
// in rt (DevScene::rot of the box's slot), p'_i = fma(rt_i2, dz, fma(rt_i1, dy,
// rt_i0 * dx)). The oracle (oracle/rbe_oracle.c box_frame) writes the same sequence.
__device__ __forceinline__ V3 box_frame_yaw(V3 p, const float* __restrict__ bx) {
    const float cs = bx[6], sn = bx[7];
    const float dx = p.x - bx[0], dy = p.y - bx[1], dz = p.z - bx[2];
    return {fma_(cs, dx, sn * dy), fma_(cs, dy, -(sn * dx)), dz};
}
__device__ __forceinline__ V3 box_frame_rot(V3 p, const float* __restrict__ bx, const float* __restrict__ rt) {
    const float dx = p.x - bx[0], dy = p.y - bx[1], dz = p.z - bx[2];
    return {fma_(rt[2], dz, fma_(rt[1], dy, rt[0] * dx)), fma_(rt[5], dz, fma_(rt[4], dy, rt[3] * dx)),
            fma_(rt[8], dz, fma_(rt[7], dy, rt[6] * dx))};
}
__device__ __forceinline__ bool box_tilted(const float* __restrict__ bx) {
    return (__float_as_uint(bx[14]) & BOX_TILTED) != 0u;
}

// narrow phase of capsule (a, b, r) against box record bx (rt: its rotation rows
// when tilted)
template <bool INL = false>
__device__ __forceinline__ bool capsule_box_narrow(V3 a, V3 b, float r, const float* __restrict__ bx,
                                                   const float* __restrict__ rt) {
    V3 pa, pb;
    if (box_tilted(bx)) {
        pa = box_frame_rot(a, bx, rt);
        pb = box_frame_rot(b, bx, rt);
    } else {
        pa = box_frame_yaw(a, bx);
        pb = box_frame_yaw(b, bx);
    }
    const V3 h = {bx[3], bx[4], bx[5]};
    return (INL ? segment_box_dist2_body(pa, pb, h) : segment_box_dist2(pa, pb, h)) <= r * r;
}

// Capsule C vs the plane and every box of the scene (skipping exempt pairs). The
// cluster AABB tests are an exact reject (a box AABB lies inside its cluster's), so
// they change no result, only how much broad-phase work a lane does.
template <int C>
__device__ __forceinline__ bool capsule_hits_env(const Capsules& k, const DevScene* __restrict__ sc) {
    constexpr float r = CAP_GEOM[C][6];
    const Aabb u = capsule_aabb(k.a[C], k.b[C], r);
    if (u.lo.z <= sc->plane_z) return true;  // capsule vs ground plane
    const int ncl = sc->n_clusters;
    for (int cl = 0; cl < ncl; ++cl) {
        const float* cr = sc->cluster[cl];
        if (aabb_disjoint(u, cr, cr + 4)) continue;
        const int j0 = __float_as_int(cr[3]), nj = __float_as_int(cr[7]);
        for (int j = j0; j < j0 + nj; ++j) {
            const float* bx = sc->box[j];
            if ((__float_as_uint(bx[14]) >> C) & 1u) continue;
            if (aabb_disjoint(u, bx + 8, bx + 11)) continue;
            if (capsule_box_narrow(k.a[C], k.b[C], r, bx, sc->rot[j])) return true;
        }
    }
    return false;
}

template <int P>
__device__ __forceinline__ bool pair_hits(const Capsules& k) {
    constexpr int I = PAIRS[P][0], J = PAIRS[P][1];
    constexpr float ri = CAP_GEOM[I][6], rj = CAP_GEOM[J][6];
    const Aabb u = capsule_aabb(k.a[I], k.b[I], ri);
    const Aabb v = capsule_aabb(k.a[J], k.b[J], rj);
    if (aabb_disjoint2(u, v)) return false;
    constexpr float rr = ri + rj;
    return segment_segment_dist2(k.a[I], k.b[I], k.a[J], k.b[J]) <= rr * rr;
}

// every self pair whose second capsule is J (all first capsules precede J in the
// chain, so the pair is complete as soon as J is placed)
template <int J, int P = 0>
__device__ __forceinline__ bool pairs_ending_at(const Capsules& k) {
    if constexpr (P == NPAIR) {
        return false;
    } else {
        if constexpr (PAIRS[P][1] == J) {
            static_assert(PAIRS[P][0] < J, "self pair out of chain order");
            if (pair_hits<P>(k)) return true;
        }
        return pairs_ending_at<J, P + 1>(k);
    }
}

// ---------------------------------------------------------------------------
// Axis-grid scenes staged in LDS (round 6)
// ---------------------------------------------------------------------------
// On an axis-grid scene (> 16 boxes) the broad phase gathers per lane: each lane's
// candidate boxes differ, so the grid masks and the 64-B box records are vector loads
// from global memory (L2), one dependent round trip per candidate round, and the
// grid-scene kernels waited on memory ~60 % of their wave cycles (profiles/r06
// edges_pmc_*.txt: SQ_WAIT_ANY). SceneGrid holds exactly the fields the grid path
// reads, with DevScene's names (state_collides is templated on the scene type), and a
// block of several waves stages it once in its LDS (~10 KB, shared by the block's
// waves: four one-wave queues + one copy keep 4 blocks of 4 waves on a CU, the grid
// kernels' register-bound occupancy). Same values, same arithmetic: same flags.
struct SceneGrid {
    alignas(16) float box[MAX_BOXES][16];
    alignas(16) float rot[MAX_BOXES][12];
    alignas(16) unsigned long long grid_lo[3][GRID_CELLS];
    alignas(16) unsigned long long grid_hi[3][GRID_CELLS];
    alignas(16) float grid_o[4];
    float grid_s[4];
    float base[4];
    float plane_z;
    unsigned env_far;
};
// every thread of the block (nt of them) copies its share; the caller synchronises
__device__ __forceinline__ void scene_grid_stage(const DevScene* __restrict__ sc, SceneGrid& L, int tid, int nt) {
    // (DevScene's box / rot arrays start 16-byte aligned, its grid masks 8-byte aligned)
    constexpr int NB4 = MAX_BOXES * 16 / 4, NR4 = MAX_BOXES * 12 / 4, NG = 3 * GRID_CELLS;
    const float4* b = reinterpret_cast<const float4*>(&sc->box[0][0]);
    const float4* r = reinterpret_cast<const float4*>(&sc->rot[0][0]);
    for (int i = tid; i < NB4; i += nt) reinterpret_cast<float4*>(&L.box[0][0])[i] = b[i];
    for (int i = tid; i < NR4; i += nt) reinterpret_cast<float4*>(&L.rot[0][0])[i] = r[i];
    for (int i = tid; i < NG; i += nt) {
        (&L.grid_lo[0][0])[i] = (&sc->grid_lo[0][0])[i];
        (&L.grid_hi[0][0])[i] = (&sc->grid_hi[0][0])[i];
    }
    if (tid < 4) {
        L.grid_o[tid] = sc->grid_o[tid];
        L.grid_s[tid] = sc->grid_s[tid];
        L.base[tid] = sc->base[tid];
    }
    if (tid == 0) {
        L.plane_z = sc->plane_z;
        L.env_far = sc->env_far;
    }
}

// ---------------------------------------------------------------------------
// Wave-compacted narrow phases
// ---------------------------------------------------------------------------
// A narrow phase in SIMT code costs the whole wave whenever ANY of its 64 lanes
// needs it: with ~35 self pairs and per-lane candidate rates of 0.1-7 %, a wave
// ran ~11 narrow phases although a lane needs ~0.4 on average. Instead, a lane
// whose broad phase passes appends the candidate (endpoints already in the box /
// world frame) to a per-wave LDS queue; when the next batch would overflow it, the
// active lanes pop one full pass of items (one per lane), and at the end of the
// chain they drain the rest.
// The set of tests and their arithmetic are unchanged, so results are identical.
// All queue operations sit in wave-uniform control flow (ballot + mbcnt).
// 64 items: WaveQ = 64 x 104 B + 256 B = 6912 B. A batch has at most 64 items (one
// per active lane) and a full-queue pop frees min(pending, active lanes) slots, so
// QCAP >= 64 is what makes "pop one pass, then enqueue" never overflow: with
// pending < active lanes the pop empties the queue and the batch can hold up to 64.
// Measured residency of one-wave workgroups (tools/occupancy_probe.hip, wave start /
// end stamps + HW_ID): at most 18 waves per CU with 8,192 B of LDS each, 21 at
// 6,656-7,680 B, 25 at 5,632-6,144 B; the register budget (5 waves per SIMD = 20
// per CU) binds at 6,912 B, not LDS.
constexpr int QSS = 15, QSB = 11;
constexpr int QCAP = 64;   // items per queue
static_assert(QCAP >= 64, "a batch of one item per lane must fit after one pop pass");

struct WaveQ {
    alignas(16) float ss[QCAP][QSS];   // self pair: a1 b1 a2 b2 (12), owner lane | pair << 8, r_i, r_j
    alignas(16) float sb[QCAP][QSB];   // capsule-box: pa pb (box frame) h (9), r^2, owner lane
    int hit[64];                       // per-lane collision found by a drained item
};
static_assert(sizeof(WaveQ) <= 7680, "WaveQ must let 20 one-wave workgroups share a CU");

__device__ __forceinline__ int rank_in(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Cluster AABBs of the scene, hoisted into (scalar) registers once per state: the
// kernels are instantiated for NCL = 0, 1, 2, 4, 8 clusters; unused slots hold an
// empty box (lo = +inf) that no capsule overlaps.
constexpr int NCL_GRID = -1;   // broad-phase instantiation for axis-grid scenes

template <int NCL>
struct ClusterRegs {
    float c[NCL > 0 ? NCL : 1][8];
    template <class SC>
    __device__ __forceinline__ void load(const SC* __restrict__ sc) {
        if constexpr (NCL > 0) {
#pragma unroll
            for (int i = 0; i < NCL; ++i)
#pragma unroll
                for (int w = 0; w < 8; ++w) c[i][w] = sc->cluster[i][w];
        }
    }
};

template <int NCL>
struct QueueState {
    WaveQ* Q;
    int nss, nsb;     // wave-uniform item counts
    bool in_limits;   // every state of the wave inside the joint limits (skip never pairs)
    int lane;
    float plane_z;
    unsigned env_far;   // DevScene::env_far if the wave is inside the joint limits, else 0
    ClusterRegs<NCL> cl;
};

#ifdef RP_PAIR_STATS
// diagnostic builds (tools/val_lab.hip): per self pair [P][0] sphere passes, [P][1]
// AABB passes, [P][2] narrow-phase hits; [NPAIR][0] lanes walked
__device__ unsigned long long g_pairstats[NPAIR + 1][3];
#define RP_PSTAT(p, i, v) do { if (v) atomicAdd(&g_pairstats[p][i], (unsigned long long)(v)); } while (0)
#else
#define RP_PSTAT(p, i, v) do { } while (0)
#endif

// Drains pop: a queue is drained only when the next enqueue would overflow it, and
// then by exactly one pass over its top items (one per active lane), so mid-walk
// passes run full; the walk's end pops until empty. Room is guaranteed: a batch has
// at most as many items as there are active lanes. (Draining whenever more than
// QCAP - 64 items were pending ran more, emptier passes and needed a larger queue.)
template <class S>
__device__ __forceinline__ void pop_ss(S& s) {
    const unsigned long long act = __ballot(1);
    const int nact = __popcll(act), r = rank_in(act);
    const int take = s.nss < nact ? s.nss : nact;
    __builtin_amdgcn_wave_barrier();
    if (r < take) {
        const float* it = s.Q->ss[s.nss - 1 - r];
        const V3 a1 = {it[0], it[1], it[2]}, b1 = {it[3], it[4], it[5]};
        const V3 a2 = {it[6], it[7], it[8]}, b2 = {it[9], it[10], it[11]};
        const int tag = __float_as_int(it[12]);
        const float ri = it[13], rj = it[14];
        const Aabb u = capsule_aabb(a1, b1, ri);
        const Aabb v = capsule_aabb(a2, b2, rj);
        if (!aabb_disjoint2(u, v)) {
            const float rr = ri + rj;
            // an LDS OR (ds_or_b32) from every popping lane instead of a store under a
            // per-lane branch: no exec-mask save / restore (+2.9 % goal3 A/B)
#ifdef RP_PAIR_STATS
            const bool h = segment_segment_dist2(a1, b1, a2, b2) <= rr * rr;
            RP_PSTAT(tag >> 8, 1, 1);
            RP_PSTAT(tag >> 8, 2, h ? 1 : 0);
            atomicOr(&s.Q->hit[tag & 63], (int)h);
#else
            atomicOr(&s.Q->hit[tag & 63], (int)(segment_segment_dist2(a1, b1, a2, b2) <= rr * rr));
#endif
        }
    }
    __builtin_amdgcn_wave_barrier();
    s.nss -= take;
}
template <class S>
__device__ __forceinline__ void pop_sb(S& s) {
    const unsigned long long act = __ballot(1);
    const int nact = __popcll(act), r = rank_in(act);
    const int take = s.nsb < nact ? s.nsb : nact;
    __builtin_amdgcn_wave_barrier();
    if (r < take) {
        const float* it = s.Q->sb[s.nsb - 1 - r];
        const V3 pa = {it[0], it[1], it[2]}, pb = {it[3], it[4], it[5]}, h = {it[6], it[7], it[8]};
        atomicOr(&s.Q->hit[__float_as_int(it[10])], (int)(segment_box_dist2(pa, pb, h) <= it[9]));
    }
    __builtin_amdgcn_wave_barrier();
    s.nsb -= take;
}
// make room for a batch of c items (wave-uniform)
template <class S>
__device__ __forceinline__ void room_ss(S& s, int c) {
    if (s.nss + c > QCAP) pop_ss(s);
}
template <class S>
__device__ __forceinline__ void room_sb(S& s, int c) {
    if (s.nsb + c > QCAP) pop_sb(s);
}

// queue item of capsule C vs box record bx (box frame segment, half extents, r^2);
// rt: the box's rotation rows, read only when the box is tilted (a wave-uniform
// branch in the cluster scenes, whose records sit in scalar registers)
template <int C, class S>
__device__ __forceinline__ void enqueue_sb(const Capsules& k, const float* bx, const float* __restrict__ rt,
                                           float r, S& s, unsigned long long m) {
    float* it = s.Q->sb[s.nsb + rank_in(m)];
    if (box_tilted(bx)) {
        const V3 pa = box_frame_rot(k.a[C], bx, rt), pb = box_frame_rot(k.b[C], bx, rt);
        it[0] = pa.x; it[1] = pa.y; it[2] = pa.z;
        it[3] = pb.x; it[4] = pb.y; it[5] = pb.z;
    } else {
        const float cs = bx[6], sn = bx[7];
        float dx = k.a[C].x - bx[0], dy = k.a[C].y - bx[1];
        it[0] = fma_(cs, dx, sn * dy); it[1] = fma_(cs, dy, -(sn * dx)); it[2] = k.a[C].z - bx[2];
        dx = k.b[C].x - bx[0]; dy = k.b[C].y - bx[1];
        it[3] = fma_(cs, dx, sn * dy); it[4] = fma_(cs, dy, -(sn * dx)); it[5] = k.b[C].z - bx[2];
    }
    it[6] = bx[3]; it[7] = bx[4]; it[8] = bx[5];
    it[9] = r * r;
    it[10] = __int_as_float(s.lane);
}

// capsule C vs plane (immediate) and boxes (queued)
template <int C, int NCL, class SC>
__device__ __forceinline__ bool env_queued(const Capsules& k, const SC* __restrict__ sc,
                                           QueueState<NCL>& s) {
    constexpr float r = CAP_GEOM[C][6];
    const Aabb u = capsule_aabb(k.a[C], k.b[C], r);
    if (u.lo.z <= s.plane_z) return true;  // capsule vs ground plane
    if ((s.env_far >> C) & 1u) return false;   // no box within the capsule's reach (wave-uniform)
    if constexpr (NCL == NCL_GRID) {
        // superset of the AABB-overlapping boxes from the axis grid (per-lane
        // gathers), then the exact AABB test on each candidate, one per lane per
        // round: rounds = the largest candidate count in the wave
        unsigned long long m = ~0ull;
        const float ulo[3] = {u.lo.x, u.lo.y, u.lo.z}, uhi[3] = {u.hi.x, u.hi.y, u.hi.z};
#pragma unroll
        for (int a = 0; a < 3; ++a)
            m &= sc->grid_lo[a][grid_cell(uhi[a], sc->grid_o[a], sc->grid_s[a])] &
                 sc->grid_hi[a][grid_cell(ulo[a], sc->grid_o[a], sc->grid_s[a])];
        while (__any(m != 0)) {
            bool cand = false;
            const float* bx = sc->box[0];
            const float* rt = sc->rot[0];
            if (m) {
                const int jb = __builtin_ctzll(m);
                bx = sc->box[jb];
                rt = sc->rot[jb];
                m &= m - 1;
                // exempt bit and box test as one separation value (one lane mask;
                // A/B clutter64 +9.7 %; -DRP_GRID_CMP builds the mask form)
                const float ex = ((__float_as_uint(bx[14]) >> C) & 1u) ? __builtin_inff() : -__builtin_inff();
                cand = fmaxr(ex, aabb_sep(u, bx + 8, bx + 11)) <= 0.0f;
            }
            const unsigned long long bm = __ballot(cand);
            if (!bm) continue;
            room_sb(s, __popcll(bm));
            if (cand) enqueue_sb<C>(k, bx, rt, r, s, bm);
            s.nsb += __popcll(bm);
        }
        return false;
    }
#pragma unroll
    for (int cl = 0; cl < NCL; ++cl) {
        const float* cr = s.cl.c[cl];
        // cluster test, box test and exempt bit folded into one separation value:
        // candidate iff max(cluster sep, box sep, exempt ? inf : -inf) <= 0 (one lane
        // mask per box instead of three combined by scalar ops: A/B +1.9 % goal3 4M,
        // +1.6 % at 64k; -DRP_ENV_CMP builds the mask form)
        const float csep = aabb_sep(u, cr, cr + 4);
        if (!__any(csep <= 0.0f)) continue;
        const int j0 = __float_as_int(cr[3]), nj = __float_as_int(cr[7]);
        for (int j = j0; j < j0 + nj; ++j) {
            // the whole 64-B record in one scalar load; branch-free candidate test
            struct Rec { float v[16]; };
            const Rec rec = *reinterpret_cast<const Rec*>(sc->box[j]);
            const float* bx = rec.v;
            const float ex = ((__float_as_uint(bx[14]) >> C) & 1u) ? __builtin_inff() : -__builtin_inff();
            const bool cand = fmaxr(fmaxr(csep, ex), aabb_sep(u, bx + 8, bx + 11)) <= 0.0f;
            const unsigned long long m = __ballot(cand);
            if (!m) continue;
            room_sb(s, __popcll(m));
            if (cand) enqueue_sb<C>(k, bx, sc->rot[j], r, s, m);
            s.nsb += __popcll(m);
        }
    }
    return false;
}

// Bounding-sphere radius of capsule C: radius + half its length + 1e-4 m. The
// margin dwarfs float rounding (~1e-7 m here), so two disjoint spheres prove the
// capsules are farther apart than any rounding could hide: the prefilter can never
// drop a pair that the exact test (AABB + narrow phase, as in the oracle) would
// report, i.e. it changes no result.
constexpr double csqrt(double x) {
    double r = x > 1.0 ? x : 1.0;
    for (int i = 0; i < 64; ++i) r = 0.5 * (r + x / r);
    return r;
}
template <int C>
constexpr float sphere_radius() {
    constexpr double dx = (double)CAP_GEOM[C][3] - CAP_GEOM[C][0];
    constexpr double dy = (double)CAP_GEOM[C][4] - CAP_GEOM[C][1];
    constexpr double dz = (double)CAP_GEOM[C][5] - CAP_GEOM[C][2];
    return (float)((double)CAP_GEOM[C][6] + 0.5 * csqrt(dx * dx + dy * dy + dz * dz) + 1e-4);
}

// sphere prefilter of self pair P (exact reject, see sphere_radius)
template <int P>
__device__ __forceinline__ bool pair_sphere(const Capsules& k) {
    constexpr int I = PAIRS[P][0], J = PAIRS[P][1];
    constexpr float RS = sphere_radius<I>() + sphere_radius<J>();
    // the centres' sums made once per capsule (place): -6 VALU per pair, 25 pairs per
    // state; the same values (the same two adds), so the same bools
    const V3 d = {k.m[I].x - k.m[J].x, k.m[I].y - k.m[J].y, k.m[I].z - k.m[J].z};
    // |centre_I - centre_J| <= RS  <=>  |2 centre_I - 2 centre_J|^2 <= (2 RS)^2
    return dot3(d, d) <= (2.0f * RS) * (2.0f * RS);
}

// queue the candidates of pair P (wave-uniform call)
template <int P, class S>
__device__ __forceinline__ void pair_enqueue(const Capsules& k, S& s, bool cand, unsigned long long m) {
    constexpr int I = PAIRS[P][0], J = PAIRS[P][1];
    if ((__lane_id() & 63) == 0) RP_PSTAT(P, 0, __popcll(m));
    if (!m) return;
    room_ss(s, __popcll(m));
    if (cand) {
        float* it = s.Q->ss[s.nss + rank_in(m)];
        it[0] = k.a[I].x; it[1] = k.a[I].y; it[2] = k.a[I].z;
        it[3] = k.b[I].x; it[4] = k.b[I].y; it[5] = k.b[I].z;
        it[6] = k.a[J].x; it[7] = k.a[J].y; it[8] = k.a[J].z;
        it[9] = k.b[J].x; it[10] = k.b[J].y; it[11] = k.b[J].z;
        it[12] = __int_as_float(s.lane | (P << 8));
        it[13] = CAP_GEOM[I][6];
        it[14] = CAP_GEOM[J][6];
    }
    s.nss += __popcll(m);
}

constexpr bool pairs_in_chain_order() {
    for (int P = 0; P < NPAIR; ++P)
        if (PAIRS[P][0] >= PAIRS[P][1]) return false;
    return true;
}
// a pair is complete (both capsules placed) when its second capsule is
static_assert(pairs_in_chain_order(), "self pair out of chain order");

// the self pairs whose second capsule is J, in PAIRS order
struct PairList { int n; int p[NPAIR]; };
template <int J>
constexpr PairList pairs_ending() {
    PairList l{};
    for (int P = 0; P < NPAIR; ++P)
        if (PAIRS[P][1] == J) l.p[l.n++] = P;
    return l;
}

template <int J, int T, class S>
__device__ __forceinline__ void pairs_each(const Capsules& k, S& s) {
    constexpr PairList L = pairs_ending<J>();
    if constexpr (T < L.n) {
        // never pairs are left out of the walk (their first capsule then dies early,
        // which lowers the register peak); waves with a state outside the joint
        // limits test them afterwards (never_pairs_outside_limits)
        if constexpr (!pair_never(L.p[T])) {
            constexpr int P = L.p[T], I = PAIRS[P][0];
            {
                const bool cand = pair_sphere<P>(k);
                pair_enqueue<P>(k, s, cand, __ballot(cand));
            }
            (void)I;
        }
        pairs_each<J, T + 1, S>(k, s);
    }
}

template <int J, class S>
__device__ __forceinline__ void pairs_queued(const Capsules& k, S& s) {
    constexpr PairList L = pairs_ending<J>();
    if constexpr (L.n > 0) {
        pairs_each<J, 0, S>(k, s);
    }
}

// Work roles of a state check (k_validity_split: two or three waves share each
// state), a bit set: ROLE_ENV the plane and box tests of every capsule, ROLE_PA the
// self pairs completed before capsule SPLIT_J, ROLE_PB the self pairs completed at
// SPLIT_J or later and the never pairs of waves outside the joint limits. The sets
// partition ROLE_ALL's tests, so OR-ing the roles' results gives its result.
enum { ROLE_ENV = 1, ROLE_PA = 2, ROLE_PB = 4, ROLE_ALL = 7 };
#ifndef RP_SPLIT_J
#define RP_SPLIT_J C_LINK6
#endif
constexpr int SPLIT_J = RP_SPLIT_J;

template <int NCL, int ROLE = ROLE_ALL, class SC = DevScene>
struct QueuedVisit {
    const SC* __restrict__ sc;
    QueueState<NCL> s;
    template <int C>
    __device__ __forceinline__ bool at(const Capsules& k) {
        if constexpr (C == C_LINK4) RP_STAMP(2);
        if constexpr (C == C_LINK6) RP_STAMP(3);
        if constexpr (C == C_HAND) RP_STAMP(4);
        if constexpr ((ROLE & ROLE_ENV) != 0) {
            if (env_queued<C>(k, sc, s)) return true;
        }
        if constexpr (((ROLE & ROLE_PA) != 0 && C < SPLIT_J) || ((ROLE & ROLE_PB) != 0 && C >= SPLIT_J))
            pairs_queued<C>(k, s);
        return false;
    }
};

// the never pairs (rp_model.h NEVER_PAIRS) of a wave with a state outside the joint
// limits, where their proof does not hold: the capsules are placed again (a second
// FK walk, rare) and the pairs queued as in the walk
template <int P = 0, class S>
__device__ __forceinline__ void never_pairs_each(const Capsules& k, S& s) {
    if constexpr (P < NPAIR) {
        if constexpr (pair_never(P)) {
            const bool cand = pair_sphere<P>(k);
            pair_enqueue<P>(k, s, cand, __ballot(cand));
        }
        never_pairs_each<P + 1>(k, s);
    }
}
template <class S, class SC>
__device__ __forceinline__ void never_pairs_outside_limits(const float q[NQ], const SC* __restrict__ sc,
                                                                     S& s) {
    Capsules k;
    fk_capsules<SC>(q, sc, k);
    never_pairs_each(k, s);
}

// true if the state collides with the plane, a (non-exempt) box, or itself: the OR
// over every test. Plane tests decide at once (a colliding lane stops walking);
// box and self narrow phases are queued and drained wave-compacted. Every lane of
// the wave that is still running must call this at the same point. NCL >= the
// scene's cluster count (rp_lib.hip picks the instantiation).
template <int NCL, bool BF = false, int ROLE = ROLE_ALL, class SC = DevScene>
__device__ __forceinline__ bool state_collides(const float q[NQ], const SC* __restrict__ sc, WaveQ& Q) {
    Capsules k;
    QueuedVisit<NCL, ROLE, SC> v;
    v.sc = sc;
    v.s.Q = &Q;
    v.s.nss = 0;
    v.s.nsb = 0;
    v.s.lane = (int)__lane_id();
    {
        // q_j in [lo_j, hi_j] for all j <=> max_j max(lo_j - q_j, q_j - hi_j) <= 0 (the
        // aabb_disjoint argument; one lane mask instead of 18 ANDed: +1.9 % goal3 A/B)
        float ex = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < NQ; ++j) ex = fmaxr(ex, fmaxr(Q_LO_F[j] - q[j], q[j] - Q_HI_F[j]));
        const bool in = ex <= 0.0f;
        v.s.in_limits = !__any(!in);
    }
    v.s.plane_z = sc->plane_z;
    v.s.env_far = v.s.in_limits ? sc->env_far : 0u;
    if constexpr ((ROLE & ROLE_ENV) != 0) v.s.cl.load(sc);
    Q.hit[v.s.lane] = 0;
    __builtin_amdgcn_wave_barrier();
    // the 7 joint sin / cos first: independent chains, interleaved, instead of one
    // exposed polynomial chain per link (the same function of q: the same bits;
    // A/B +5 % goal3 4M states, +1.5 % at 64k, clutter64 +-0; -DRP_SC_WALK builds
    // the per-link form)
    JointsSC jt;
#pragma unroll
    for (int i = 0; i < 7; ++i) rp_sincos(q[i], &jt.s[i], &jt.c[i]);
    if (fk_walk_j<QueuedVisit<NCL, ROLE, SC>, BF>(q, jt, sc->base, k, v)) return true;
    if constexpr ((ROLE & ROLE_PB) != 0)
        if (!v.s.in_limits) never_pairs_outside_limits(q, sc, v.s);
    RP_STAMP(5);
    while (v.s.nsb > 0) pop_sb(v.s);
    RP_STAMP(6);
    while (v.s.nss > 0) pop_ss(v.s);
    RP_STAMP(7);
    return Q.hit[v.s.lane] != 0;
}

// ---------------------------------------------------------------------------
// Low-latency state check: GL lanes per state (DESIGN.md §5 "latency kernels")
// ---------------------------------------------------------------------------
// A launch too small to fill the chip (a straight edge; the few thousand edges of a
// small RRT iteration; the simplification's candidate edges) is as slow as one
// wave's dependency chain when one lane owns a state (~20k cycles, FK + 12 capsule
// walks + 35 pairs in sequence). Here a group of GL lanes shares a state: the 7
// joint sin/cos are computed by 7 lanes at once and exchanged, every lane then walks
// the (short) FK chain, lane 0 of the group stores the 12 capsules in LDS, and the
// group's lanes split the tests — unit u < NPAIR is self pair u, unit NPAIR + c*nb + j
// is capsule c vs box j — with the oracle's test arithmetic (plain per-box AABB, no
// cluster / grid / sphere prefilters, every self pair): the state collides iff the
// plane test or any unit hits (group OR). Same flags as state_collides.
__constant__ int ML_PAIR_I[NPAIR] = {
#define RP_PI(p) PAIRS[p][0]
    RP_PI(0), RP_PI(1), RP_PI(2), RP_PI(3), RP_PI(4), RP_PI(5), RP_PI(6), RP_PI(7), RP_PI(8), RP_PI(9),
    RP_PI(10), RP_PI(11), RP_PI(12), RP_PI(13), RP_PI(14), RP_PI(15), RP_PI(16), RP_PI(17), RP_PI(18), RP_PI(19),
    RP_PI(20), RP_PI(21), RP_PI(22), RP_PI(23), RP_PI(24), RP_PI(25), RP_PI(26), RP_PI(27), RP_PI(28), RP_PI(29),
    RP_PI(30), RP_PI(31), RP_PI(32), RP_PI(33), RP_PI(34)
#undef RP_PI
};
__constant__ int ML_PAIR_J[NPAIR] = {
#define RP_PJ(p) PAIRS[p][1]
    RP_PJ(0), RP_PJ(1), RP_PJ(2), RP_PJ(3), RP_PJ(4), RP_PJ(5), RP_PJ(6), RP_PJ(7), RP_PJ(8), RP_PJ(9),
    RP_PJ(10), RP_PJ(11), RP_PJ(12), RP_PJ(13), RP_PJ(14), RP_PJ(15), RP_PJ(16), RP_PJ(17), RP_PJ(18), RP_PJ(19),
    RP_PJ(20), RP_PJ(21), RP_PJ(22), RP_PJ(23), RP_PJ(24), RP_PJ(25), RP_PJ(26), RP_PJ(27), RP_PJ(28), RP_PJ(29),
    RP_PJ(30), RP_PJ(31), RP_PJ(32), RP_PJ(33), RP_PJ(34)
#undef RP_PJ
};
__constant__ float ML_RADIUS[NCAP] = {CAP_GEOM[0][6], CAP_GEOM[1][6], CAP_GEOM[2][6], CAP_GEOM[3][6],
                                      CAP_GEOM[4][6], CAP_GEOM[5][6], CAP_GEOM[6][6], CAP_GEOM[7][6],
                                      CAP_GEOM[8][6], CAP_GEOM[9][6], CAP_GEOM[10][6], CAP_GEOM[11][6]};

struct CapsLds { float v[NCAP][6]; };   // a.xyz, b.xyz of each capsule (world)

// The scene and the test tables in LDS: in these latency-bound kernels every
// dependent global load is a round trip to another XCD's L2 or HBM (~1-2 us), so
// the block loads all of it at once at its start (overlapping the FK chain) and
// the test loop reads only LDS.
struct SceneLds {
    float box[MAX_BOXES][16];
    float rot[MAX_BOXES][12];
    int pi[NPAIR], pj[NPAIR];
    float rad[NCAP];
    float plane_z, base[3];
    int nb, un;
    alignas(16) unsigned short ul[ML_UNITS_PAD];   // DevScene::ml_unit (un of them)
};
// all 64 lanes of the (one-wave) block; no wait (state_collides_ml waits)
__device__ __forceinline__ void scene_to_lds(const DevScene* __restrict__ sc, SceneLds& L) {
    const int t = (int)rp_tid();
    const float4* src = reinterpret_cast<const float4*>(&sc->box[0][0]);
    float4* dst = reinterpret_cast<float4*>(&L.box[0][0]);
#pragma unroll
    for (int k = 0; k < MAX_BOXES * 4 / 64; ++k) dst[t + 64 * k] = src[t + 64 * k];
    {
        const float4* rs = reinterpret_cast<const float4*>(&sc->rot[0][0]);
        float4* rd = reinterpret_cast<float4*>(&L.rot[0][0]);
#pragma unroll
        for (int k = 0; k < MAX_BOXES * 3 / 64; ++k) rd[t + 64 * k] = rs[t + 64 * k];
    }
    if (t < NPAIR) {
        L.pi[t] = ML_PAIR_I[t];
        L.pj[t] = ML_PAIR_J[t];
    }
    if (t < NCAP) L.rad[t] = ML_RADIUS[t];
    {
        const uint4* us = reinterpret_cast<const uint4*>(sc->ml_unit);
        uint4* ud = reinterpret_cast<uint4*>(L.ul);
        for (int k = t; k < ML_UNITS_PAD / 8; k += 64) ud[k] = us[k];
    }
    if (t == 0) {
        L.plane_z = sc->plane_z;
        L.nb = sc->n_boxes;
        L.un = sc->ml_n;
    }
    if (t < 3) L.base[t] = sc->base[t];
}
struct NoVisitPlane {   // plane test only, in the walk (every lane, registers)
    float plane_z;
    template <int C>
    __device__ __forceinline__ bool at(const Capsules& k) {
        constexpr float r = CAP_GEOM[C][6];
        return fminr(k.a[C].z, k.b[C].z) - r <= plane_z;   // capsule_aabb(...).lo.z <= plane
    }
};

// Every lane of the wave calls it (wave-uniform control flow); `run`: this lane's
// group has a state. Returns the group's verdict on every lane of the group.
template <int GL, bool BF = false>
__device__ __forceinline__ bool state_collides_ml(const float q[NQ], bool run, const SceneLds& sc,
                                                  CapsLds* caps) {
    static_assert(GL >= 8 && GL <= 64 && (GL & (GL - 1)) == 0, "group of 8..64 lanes");
    const int lane = (int)__lane_id();
    const int gl = lane & (GL - 1), base = lane & ~(GL - 1);
    CapsLds& cs = caps[lane / GL];
    // joint sin / cos: lane gl < 7 of the group computes joint gl's
    float sj, cj;
    rp_sincos(q[gl < 7 ? gl : 0], &sj, &cj);
    JointsSC jt;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        jt.s[i] = __shfl(sj, base + i, 64);
        jt.c[i] = __shfl(cj, base + i, 64);
    }
    if constexpr (GL == 16) RP_ESTAMP(8);
    __syncthreads();   // the block's SceneLds (scene_to_lds, issued before the caller's state setup)
    if constexpr (GL == 16) RP_ESTAMP(9);
    Capsules k;
    NoVisitPlane pv{sc.plane_z};
    bool hit = run && fk_walk_j<NoVisitPlane, BF>(q, jt, sc.base, k, pv);
    if constexpr (GL == 16) RP_ESTAMP(10);
    if (!__any(run && !hit)) return hit;   // every state decided by the plane (or idle)
    if (gl == 0) {
#pragma unroll
        for (int c = 0; c < NCAP; ++c) {
            cs.v[c][0] = k.a[c].x; cs.v[c][1] = k.a[c].y; cs.v[c][2] = k.a[c].z;
            cs.v[c][3] = k.b[c].x; cs.v[c][4] = k.b[c].y; cs.v[c][5] = k.b[c].z;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if constexpr (GL == 16) RP_ESTAMP(11);
    const int nb = sc.nb;
    const bool active = run && !hit;   // uniform within the group
    // every running state of the wave inside the joint limits: the scene's reduced
    // unit list (no never pairs, no box tests of capsules that reach no box: both
    // proven for such states, DevScene::ml_unit), else every unit
    bool reduced;
    {
        float ex = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < NQ; ++j) ex = fmaxr(ex, fmaxr(Q_LO_F[j] - q[j], q[j] - Q_HI_F[j]));
        reduced = !__any(active && !(ex <= 0.0f));
    }
    const int units = reduced ? sc.un : NPAIR + NCAP * nb;
    for (int u0 = 0; u0 < units; u0 += GL) {
        const int u = reduced ? (int)sc.ul[u0 + gl < units ? u0 + gl : 0] : u0 + gl;
        bool h = false;
        if (active && u0 + gl < units) {
            if (u < NPAIR) {
                const int i = sc.pi[u], j = sc.pj[u];
                const float* pi = cs.v[i];
                const float* pj = cs.v[j];
                const V3 a1 = {pi[0], pi[1], pi[2]}, b1 = {pi[3], pi[4], pi[5]};
                const V3 a2 = {pj[0], pj[1], pj[2]}, b2 = {pj[3], pj[4], pj[5]};
                const float ri = sc.rad[i], rj = sc.rad[j];
                if (!aabb_disjoint2(capsule_aabb(a1, b1, ri), capsule_aabb(a2, b2, rj))) {
                    const float rr = ri + rj;
                    h = segment_segment_dist2_body(a1, b1, a2, b2) <= rr * rr;
                }
            } else {
                const int w = u - NPAIR;
                const int c = w / nb, j = w - c * nb;
                const float* bx = sc.box[j];
                if (!((__float_as_uint(bx[14]) >> c) & 1u)) {
                    const float* pc = cs.v[c];
                    const V3 a = {pc[0], pc[1], pc[2]}, b = {pc[3], pc[4], pc[5]};
                    const float r = sc.rad[c];
                    if (!aabb_disjoint(capsule_aabb(a, b, r), bx + 8, bx + 11))
                        h = capsule_box_narrow<true>(a, b, r, bx, sc.rot[j]);
                }
            }
        }
        constexpr unsigned long long GMASK = GL == 64 ? ~0ull : ((1ull << (GL & 63)) - 1);
        const unsigned long long m = __ballot(h);
        hit = hit || ((m >> base) & GMASK) != 0;
        if (!__any(active && !hit)) break;   // every group decided
    }
    if constexpr (GL == 16) RP_ESTAMP(12);
    __builtin_amdgcn_wave_barrier();   // the LDS capsules are reused by the next state
    return hit;
}

}  // namespace rp
