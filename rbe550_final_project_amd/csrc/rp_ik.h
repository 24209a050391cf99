// rp_ik.h — batched inverse kinematics of the Franka hand link (gfx950).
//
// Replaces Genesis robot.inverse_kinematics(link=hand, pos, quat) as called by
// code/motion_primitives.py:131-134 (_ik_for_pose) to turn grasp / place poses
// into goal configurations for plan_path [EXT-GS]. Genesis runs damped least
// squares from the current qpos and restarts from random samples when it fails
// (max_samples); here every (target, restart) pair is one lane, all restarts run
// at once, and the result is validity-filtered with the collision kernel.
//
// Float64 throughout, written to the numerics contract (fixed
// operation order, no FMA contraction, polynomial sin/cos) so oracle/rbe_oracle.c
// ro_ik reproduces every lane bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rp_plan_math.h"

namespace rp {

constexpr uint32_t IK_TAG = 0x524B494Bu;   // Philox counter tag of IK restarts

// sin / cos for |x| < 1e5: Cody-Waite reduction by pi/2, fdlibm kernel polynomials
__device__ __forceinline__ void sincos64(double x, double* s, double* c) {
    const double kd = rint(x * 6.36619772367581382433e-01);
    const double r = (x - kd * 1.57079632673412561417e+00) - kd * 6.07710050650619224932e-11;
    const double w = r * r;
    double ps = 1.58969099521155010221e-10;
    ps = -2.50507602534068634195e-08 + w * ps;
    ps = 2.75573137070700676789e-06 + w * ps;
    ps = -1.98412698298579493134e-04 + w * ps;
    ps = 8.33333333332248946124e-03 + w * ps;
    ps = -1.66666666666666324348e-01 + w * ps;
    const double sn = r + r * w * ps;
    double pc = -1.13596475577881948265e-11;
    pc = 2.08757232129817482790e-09 + w * pc;
    pc = -2.75573143513906633035e-07 + w * pc;
    pc = 2.48015872894767294178e-05 + w * pc;
    pc = -1.38888888888741095749e-03 + w * pc;
    pc = 4.16666666666666019037e-02 + w * pc;
    const double cs = 1.0 - 0.5 * w + w * w * pc;
    switch ((int)kd & 3) {
        case 0: *s = sn; *c = cs; break;
        case 1: *s = cs; *c = -sn; break;
        case 2: *s = -sn; *c = -cs; break;
        default: *s = -cs; *c = sn; break;
    }
}

// joint offsets (link frame translation before the joint) and the +-90 deg
// x-rotation of each joint frame
constexpr double IK_T[7][3] = {{0.0, 0.0, 0.333}, {0.0, 0.0, 0.0},   {0.0, -0.316, 0.0}, {0.0825, 0.0, 0.0},
                                     {-0.0825, 0.384, 0.0}, {0.0, 0.0, 0.0}, {0.088, 0.0, 0.0}};
constexpr int IK_RX[7] = {0, -1, 1, 1, -1, 1, 1};
constexpr double IK_FLANGE = 0.107;                       // link7 -> hand along z
constexpr double IK_C45 = 0.70710678118654757;            // cos(-pi/4) = -sin(-pi/4)

// Hand frame (columns R[0..2], origin p) and every joint's world axis z[j] and
// origin o[j] for the arm joints q[0..6], robot base at `base`.
struct HandFk {
    double R[3][3];
    double p[3];
    double z[7][3];
    double o[7][3];
};

__device__ __forceinline__ void hand_fk(const double* q, const double base[3], HandFk& f) {
    double c0[3] = {1.0, 0.0, 0.0}, c1[3] = {0.0, 1.0, 0.0}, c2[3] = {0.0, 0.0, 1.0};
    double p[3] = {base[0], base[1], base[2]};
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const double* t = IK_T[j];
#pragma unroll
        for (int i = 0; i < 3; ++i) p[i] = p[i] + (c0[i] * t[0] + c1[i] * t[1] + c2[i] * t[2]);
        if (IK_RX[j] > 0) {
#pragma unroll
            for (int i = 0; i < 3; ++i) { const double a = c1[i]; c1[i] = c2[i]; c2[i] = -a; }
        } else if (IK_RX[j] < 0) {
#pragma unroll
            for (int i = 0; i < 3; ++i) { const double a = c1[i]; c1[i] = -c2[i]; c2[i] = a; }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) { f.z[j][i] = c2[i]; f.o[j][i] = p[i]; }
        double s, c;
        sincos64(q[j], &s, &c);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double a = c0[i], b = c1[i];
            c0[i] = c * a + s * b;
            c1[i] = c * b - s * a;
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = p[i] + IK_FLANGE * c2[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {   // Rz(-pi/4): c = IK_C45, s = -IK_C45
        const double a = c0[i], b = c1[i];
        c0[i] = IK_C45 * a + -IK_C45 * b;
        c1[i] = IK_C45 * b - -IK_C45 * a;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) { f.R[0][i] = c0[i]; f.R[1][i] = c1[i]; f.R[2][i] = c2[i]; f.p[i] = p[i]; }
}

__device__ __forceinline__ void cross3(const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// rotation matrix columns of a (w, x, y, z) quaternion, normalised first
__device__ __forceinline__ void quat_columns(const double* qt, double T[3][3]) {
    const double n = sqrt(qt[0] * qt[0] + qt[1] * qt[1] + qt[2] * qt[2] + qt[3] * qt[3]);
    const double w = qt[0] / n, x = qt[1] / n, y = qt[2] / n, z = qt[3] / n;
    T[0][0] = 1.0 - 2.0 * (y * y + z * z); T[0][1] = 2.0 * (x * y + w * z); T[0][2] = 2.0 * (x * z - w * y);
    T[1][0] = 2.0 * (x * y - w * z); T[1][1] = 1.0 - 2.0 * (x * x + z * z); T[1][2] = 2.0 * (y * z + w * x);
    T[2][0] = 2.0 * (x * z + w * y); T[2][1] = 2.0 * (y * z - w * x); T[2][2] = 1.0 - 2.0 * (x * x + y * y);
}

// pose error: position pt - p and orientation 0.5 * sum_k R_k x T_k (zero when the
// frames agree); squared norms in e2[0] (position), e2[1] (orientation)
__device__ __forceinline__ void pose_error(const HandFk& f, const double* pt, const double T[3][3], double e[6],
                                           double e2[2]) {
    double x0[3], x1[3], x2[3];
    cross3(f.R[0], T[0], x0);
    cross3(f.R[1], T[1], x1);
    cross3(f.R[2], T[2], x2);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        e[i] = pt[i] - f.p[i];
        e[3 + i] = 0.5 * (x0[i] + x1[i] + x2[i]);
    }
    e2[0] = e[0] * e[0] + e[1] * e[1] + e[2] * e[2];
    e2[1] = e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
}

struct IkArgs {
    const double* pos;     // n_targets x 3
    const double* quat;    // n_targets x 4 (w, x, y, z)
    const double* init;    // n_targets x 9
    double lo[NQ], hi[NQ];
    double base[3];
    uint64_t seed;
    int n_targets, n_seeds, iters;
    double damping, pos_tol, rot_tol;
};

// lane (target t, restart k): k = 0 starts from init[t], k > 0 from a Philox sample
// of the arm joints (fingers from init). Damped least squares on the hand pose:
// dq = J^T (J J^T + damping^2 I)^-1 e, clamped to the bounds, `iters` steps (early
// stop below 1% of both tolerances). out: q (9), errors (2), converged flag.
__global__ __launch_bounds__(64) void k_ik(IkArgs a, double* __restrict__ q_out, double* __restrict__ err_out,
                                           uint8_t* __restrict__ conv, float* __restrict__ q32) {
    const int64_t g = (int64_t)rp_bid() * rp_bdim() + rp_tid();
    if (g >= (int64_t)a.n_targets * a.n_seeds) return;
    const int t = (int)(g / a.n_seeds), k = (int)(g - (int64_t)t * a.n_seeds);
    double q[NQ];
    const double* qi = a.init + (int64_t)t * NQ;
    if (k == 0) {
#pragma unroll
        for (int i = 0; i < NQ; ++i) q[i] = qi[i];
    } else {
        sample_state(a.seed, (uint64_t)g, a.lo, a.hi, q, IK_TAG);
        q[7] = qi[7];
        q[8] = qi[8];
    }
    double T[3][3];
    quat_columns(a.quat + (int64_t)t * 4, T);
    const double* pt = a.pos + (int64_t)t * 3;
    const double lam2 = a.damping * a.damping;
    const double stop_p = (0.01 * a.pos_tol) * (0.01 * a.pos_tol), stop_r = (0.01 * a.rot_tol) * (0.01 * a.rot_tol);
    HandFk f;
    double e[6], e2[2];
    for (int it = 0; it < a.iters; ++it) {
        hand_fk(q, a.base, f);
        pose_error(f, pt, T, e, e2);
        if (e2[0] <= stop_p && e2[1] <= stop_r) break;
        double J[6][7];
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const double d[3] = {f.p[0] - f.o[j][0], f.p[1] - f.o[j][1], f.p[2] - f.o[j][2]};
            double v[3];
            cross3(f.z[j], d, v);
#pragma unroll
            for (int i = 0; i < 3; ++i) { J[i][j] = v[i]; J[3 + i][j] = f.z[j][i]; }
        }
        double L[6][6];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
#pragma unroll
            for (int cidx = 0; cidx <= r; ++cidx) {
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < 7; ++j) s = s + J[r][j] * J[cidx][j];
                if (r == cidx) s = s + lam2;
#pragma unroll
                for (int m = 0; m < cidx; ++m) s = s - L[r][m] * L[cidx][m];
                L[r][cidx] = (r == cidx) ? sqrt(s) : s / L[cidx][cidx];
            }
        }
        double y[6], x[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            double s = e[r];
#pragma unroll
            for (int m = 0; m < r; ++m) s = s - L[r][m] * y[m];
            y[r] = s / L[r][r];
        }
#pragma unroll
        for (int r = 5; r >= 0; --r) {
            double s = y[r];
#pragma unroll
            for (int m = r + 1; m < 6; ++m) s = s - L[m][r] * x[m];
            x[r] = s / L[r][r];
        }
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            double dq = 0.0;
#pragma unroll
            for (int r = 0; r < 6; ++r) dq = dq + J[r][j] * x[r];
            double v = q[j] + dq;
            if (v < a.lo[j]) v = a.lo[j];
            if (v > a.hi[j]) v = a.hi[j];
            q[j] = v;
        }
    }
    hand_fk(q, a.base, f);
    pose_error(f, pt, T, e, e2);
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        q_out[g * NQ + i] = q[i];
        q32[g * NQ + i] = (float)q[i];
    }
    err_out[2 * g] = e2[0];
    err_out[2 * g + 1] = e2[1];
    conv[g] = (e2[0] <= a.pos_tol * a.pos_tol && e2[1] <= a.rot_tol * a.rot_tol) ? 1 : 0;
}

// per target (one lane): the restart to return. Class 0 = converged and collision
// free, 1 = converged but colliding, 2 = not converged; within class 0 / 1 the
// smallest joint-space distance to init, within class 2 the smallest pose error;
// ties -> lowest restart index. status = the class.
__global__ void k_ik_select(IkArgs a, const double* __restrict__ q, const double* __restrict__ err,
                            const uint8_t* __restrict__ conv, const uint8_t* __restrict__ valid,
                            double* __restrict__ q_best, int32_t* __restrict__ status) {
    const int t = rp_bid() * rp_bdim() + rp_tid();
    if (t >= a.n_targets) return;
    const double* qi = a.init + (int64_t)t * NQ;
    int best_k = 0, best_c = 3;
    double best_v = 0.0;
    for (int k = 0; k < a.n_seeds; ++k) {
        const int64_t g = (int64_t)t * a.n_seeds + k;
        const int cls = conv[g] ? (valid[g] ? 0 : 1) : 2;
        const double v = cls < 2 ? dist2(q + g * NQ, qi) : err[2 * g] + err[2 * g + 1];
        if (cls < best_c || (cls == best_c && v < best_v)) {
            best_c = cls;
            best_v = v;
            best_k = k;
        }
    }
    const int64_t g = (int64_t)t * a.n_seeds + best_k;
    for (int i = 0; i < NQ; ++i) q_best[(int64_t)t * NQ + i] = q[g * NQ + i];
    status[t] = best_c;
}

}  // namespace rp
