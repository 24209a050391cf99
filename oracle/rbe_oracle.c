/*
 * rbe_oracle.c — CPU ORACLE (test infrastructure only; see rbe_oracle.h).
 *
 * Plain C restatement of the hot path, written to the numerics contract of
 * float32 collision arithmetic and float64 planner arithmetic, every
 * operation in a fixed order, built with -ffp-contract=off, so that the HIP
 * kernels of librbe_mi355x.so (which follow the same contract) must produce
 * bit-identical validity flags, trees and paths. Reference anchors per function.
 */
#include "rbe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NQ RP_NQ
#define NCAPMAX RP_MAX_CAPSULES

typedef struct { float x, y, z; } v3;

struct ro_scene {
    int ncap;
    int cap_link[NCAPMAX];
    float cap_a[NCAPMAX][3], cap_b[NCAPMAX][3], cap_r[NCAPMAX];
    int npair;
    int pair[RP_MAX_SELF_PAIRS][2];
    int nbox;
    float box_c[RP_MAX_BOXES][3], box_h[RP_MAX_BOXES][3], box_cs[RP_MAX_BOXES], box_sn[RP_MAX_BOXES];
    float box_lo[RP_MAX_BOXES][3], box_hi[RP_MAX_BOXES][3];
    int box_tilt[RP_MAX_BOXES];          /* 1: box_rt holds R^T rows (rp_set_scene_rot) */
    float box_rt[RP_MAX_BOXES][9];
    uint32_t box_exempt[RP_MAX_BOXES];   /* capsule bits */
    float plane_z;
    float base[3];
};

/* ------------------------------------------------------------------------- */
/* scene                                                                     */
/* ------------------------------------------------------------------------- */

ro_scene* ro_scene_create(const rp_robot_desc* r) {
    if (!r || r->n_capsules <= 0 || r->n_capsules > NCAPMAX || r->n_self_pairs < 0 ||
        r->n_self_pairs > RP_MAX_SELF_PAIRS)
        return NULL;
    ro_scene* s = (ro_scene*)calloc(1, sizeof(ro_scene));
    s->ncap = r->n_capsules;
    for (int c = 0; c < s->ncap; ++c) {
        s->cap_link[c] = r->capsules[c].link;
        for (int k = 0; k < 3; ++k) {
            s->cap_a[c][k] = r->capsules[c].a[k];
            s->cap_b[c][k] = r->capsules[c].b[k];
        }
        s->cap_r[c] = r->capsules[c].radius;
    }
    s->npair = r->n_self_pairs;
    for (int i = 0; i < s->npair; ++i) {
        s->pair[i][0] = r->self_pairs[i][0];
        s->pair[i][1] = r->self_pairs[i][1];
    }
    s->base[2] = 0.01f;
    return s;
}

void ro_scene_destroy(ro_scene* s) { free(s); }

int ro_scene_set(ro_scene* s, const rp_box* boxes, int32_t n, float plane_z, const float base[3]) {
    if (!s || n < 0 || n > RP_MAX_BOXES || (n > 0 && !boxes)) return RP_ERR_ARG;
    s->nbox = n;
    for (int j = 0; j < n; ++j) {
        const rp_box* b = &boxes[j];
        /* yaw -> cos/sin once, in double, rounded to float (same as the product host) */
        const float cs = (float)cos((double)b->yaw);
        const float sn = (float)sin((double)b->yaw);
        const float acs = cs < 0.0f ? -cs : cs, asn = sn < 0.0f ? -sn : sn;
        float ext[3];
        ext[0] = acs * b->half[0] + asn * b->half[1];
        ext[1] = asn * b->half[0] + acs * b->half[1];
        ext[2] = b->half[2];
        for (int k = 0; k < 3; ++k) {
            s->box_c[j][k] = b->center[k];
            s->box_h[j][k] = b->half[k];
            s->box_lo[j][k] = b->center[k] - ext[k];
            s->box_hi[j][k] = b->center[k] + ext[k];
        }
        s->box_cs[j] = cs;
        s->box_sn[j] = sn;
        s->box_tilt[j] = 0;
        s->box_exempt[j] = 0;
    }
    s->plane_z = plane_z;
    if (base) {
        s->base[0] = base[0];
        s->base[1] = base[1];
        s->base[2] = base[2];
    }
    return RP_OK;
}

/* Boxes with orientation quaternions (w, x, y, z): the product's rp_set_scene_rot
 * restated. |x|, |y| <= 1e-7 |q| (quat_upright) is an upright box of yaw
 * atan2(2(wz + xy), 1 - 2(y^2 + z^2)) (q normalised first when its norm is not 1);
 * any other box is tilted: the normalised quaternion's rotation matrix R (world =
 * R * box) in double, rounded to float once; the box frame of a world point p is
 * R^T (p - c); world AABB half extents |R_k0| h0 + |R_k1| h1 + |R_k2| h2 + 1e-6. A
 * toppled block is what goal3's collapse check re-plans around
 * (code/goal3_tallest.py:257); Genesis' collider sees every box at its pose
 * (code/planning.py:211). */
/* upright to simulation noise: |x|, |y| <= 1e-7 |q| (rp_lib.hip quat_upright) */
static int quat_upright(double x, double y, double n2) {
    const double t = 1e-7 * sqrt(n2);
    return fabs(x) <= t && fabs(y) <= t;
}

int ro_scene_set_rot(ro_scene* s, const rp_box_rot* boxes, int32_t n, float plane_z, const float base[3]) {
    if (!s || n < 0 || n > RP_MAX_BOXES || (n > 0 && !boxes)) return RP_ERR_ARG;
    rp_box up[RP_MAX_BOXES];
    memset(up, 0, sizeof up);
    for (int j = 0; j < n; ++j) {
        const rp_box_rot* b = &boxes[j];
        for (int k = 0; k < 3; ++k) { up[j].center[k] = b->center[k]; up[j].half[k] = b->half[k]; }
        double w = b->quat[0], x = b->quat[1], y = b->quat[2], z = b->quat[3];
        const double n2 = w * w + x * x + y * y + z * z;
        if (n2 == 0.0) return RP_ERR_ARG;
        if (quat_upright(x, y, n2) && fabs(n2 - 1.0) > 1e-12) {   /* non-unit upright: normalised */
            const double nr = sqrt(n2);
            w /= nr; x /= nr; y /= nr; z /= nr;
        }
        up[j].yaw = (float)atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z));
    }
    int rc = ro_scene_set(s, up, n, plane_z, base);
    if (rc) return rc;
    for (int j = 0; j < n; ++j) {
        const rp_box_rot* b = &boxes[j];
        double w = b->quat[0], x = b->quat[1], y = b->quat[2], z = b->quat[3];
        if (quat_upright(x, y, w * w + x * x + y * y + z * z)) continue;
        double nrm = sqrt(w * w + x * x + y * y + z * z);
        w /= nrm; x /= nrm; y /= nrm; z /= nrm;
        double R[3][3] = {{1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - w * z), 2.0 * (x * z + w * y)},
                          {2.0 * (x * y + w * z), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - w * x)},
                          {2.0 * (x * z - w * y), 2.0 * (y * z + w * x), 1.0 - 2.0 * (x * x + y * y)}};
        float Rf[3][3];
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) Rf[r][k] = (float)R[r][k];
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) s->box_rt[j][3 * i + k] = Rf[k][i];
        for (int k = 0; k < 3; ++k) {
            float ext = fabsf(Rf[k][0]) * b->half[0] + fabsf(Rf[k][1]) * b->half[1] + fabsf(Rf[k][2]) * b->half[2] +
                        1e-6f;
            s->box_lo[j][k] = b->center[k] - ext;
            s->box_hi[j][k] = b->center[k] + ext;
        }
        s->box_cs[j] = 0.0f;
        s->box_sn[j] = 0.0f;
        s->box_tilt[j] = 1;
    }
    return RP_OK;
}

int ro_scene_set_attached(ro_scene* s, int32_t box, uint32_t link_mask) {
    if (!s || box >= s->nbox) return RP_ERR_ARG;
    for (int j = 0; j < s->nbox; ++j) s->box_exempt[j] = 0;
    if (box < 0) return RP_OK;
    uint32_t bits = 0;
    for (int c = 0; c < s->ncap; ++c)
        if ((link_mask >> s->cap_link[c]) & 1u) bits |= 1u << c;
    s->box_exempt[box] = bits;
    return RP_OK;
}

/* ------------------------------------------------------------------------- */
/* float32 kinematics + collision (planning.py:209-230 restated)             */
/* ------------------------------------------------------------------------- */

static float mn(float a, float b) { return a < b ? a : b; }
static float mx(float a, float b) { return a > b ? a : b; }
static float c01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }
static float dot(v3 u, v3 v) { return fmaf(u.z, v.z, fmaf(u.y, v.y, u.x * v.x)); }

void ro_sincos(float x, float* sn, float* cs) {
    float k = floorf(x * 0.636619772f + 0.5f);
    float r = fmaf(-k, 1.5703125f, x);
    r = fmaf(-k, 4.837512969970703125e-4f, r);
    r = fmaf(-k, 7.54978995489188216e-8f, r);
    float z = r * r;
    float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float sr = fmaf(r * z, ps, r);
    float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float cr = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    switch (((int)k) & 3) {
        case 0: *sn = sr; *cs = cr; break;
        case 1: *sn = cr; *cs = -sr; break;
        case 2: *sn = -sr; *cs = -cr; break;
        default: *sn = -cr; *cs = sr; break;
    }
}

/* rotation columns R[0..2] (each a 3-vector) and origin P */
typedef struct { float R[3][3]; float P[3]; } frame;

/* R <- R * Rz: n0 = c*c0 + s*c1, n1 = c*c1 - s*c0 (fused as in rp_math.h) */
static void f_rot(frame* f, float s, float c) {
    float n0[3], n1[3];
    for (int k = 0; k < 3; ++k) {
        n0[k] = fmaf(c, f->R[0][k], s * f->R[1][k]);
        n1[k] = fmaf(c, f->R[1][k], -(s * f->R[0][k]));
    }
    for (int k = 0; k < 3; ++k) { f->R[0][k] = n0[k]; f->R[1][k] = n1[k]; }
}
static void f_rz(frame* f, float q) {
    float s, c;
    ro_sincos(q, &s, &c);
    f_rot(f, s, c);
}
/* R * Rx(+90) = [c0, c2, -c1]; R * Rx(-90) = [c0, -c2, c1] */
static void f_rx(frame* f, int plus) {
    float c1[3], c2[3];
    for (int k = 0; k < 3; ++k) { c1[k] = f->R[1][k]; c2[k] = f->R[2][k]; }
    for (int k = 0; k < 3; ++k) {
        if (plus) { f->R[1][k] = c2[k]; f->R[2][k] = -c1[k]; }
        else { f->R[1][k] = -c2[k]; f->R[2][k] = c1[k]; }
    }
}
static void f_shift(float P[3], float k, const float col[3]) {
    for (int i = 0; i < 3; ++i) P[i] = fmaf(k, col[i], P[i]);
}

/* world frames of the 11 links (panda.xml, scenes.py:85) */
static void link_frames(const ro_scene* s, const float q[NQ], frame F[RP_NUM_LINKS]) {
    frame f;
    memset(&f, 0, sizeof f);
    f.R[0][0] = 1.0f; f.R[1][1] = 1.0f; f.R[2][2] = 1.0f;
    f.P[0] = s->base[0]; f.P[1] = s->base[1]; f.P[2] = s->base[2];
    F[0] = f;
    f_shift(f.P, 0.333f, f.R[2]); f_rz(&f, q[0]); F[1] = f;
    f_rx(&f, 0); f_rz(&f, q[1]); F[2] = f;
    f_shift(f.P, -0.316f, f.R[1]); f_rx(&f, 1); f_rz(&f, q[2]); F[3] = f;
    f_shift(f.P, 0.0825f, f.R[0]); f_rx(&f, 1); f_rz(&f, q[3]); F[4] = f;
    f_shift(f.P, -0.0825f, f.R[0]); f_shift(f.P, 0.384f, f.R[1]); f_rx(&f, 0); f_rz(&f, q[4]); F[5] = f;
    f_rx(&f, 1); f_rz(&f, q[5]); F[6] = f;
    f_shift(f.P, 0.088f, f.R[0]); f_rx(&f, 1); f_rz(&f, q[6]); F[7] = f;
    /* hand: flange +0.107 z, Rz(-45deg) with the rounded constants */
    f_shift(f.P, 0.107f, f.R[2]);
    f_rot(&f, -0.70710677f, 0.70710677f);
    F[8] = f;
    f_shift(f.P, 0.0584f, f.R[2]);
    frame l = f;
    f_shift(l.P, q[7], f.R[1]);
    F[9] = l;
    frame r = f;
    f_shift(r.P, -q[8], f.R[1]);
    for (int k = 0; k < 3; ++k) { r.R[0][k] = -f.R[0][k]; r.R[1][k] = -f.R[1][k]; }
    F[10] = r;
}

static v3 to_world(const frame* f, const float a[3]) {
    v3 w;
    w.x = fmaf(a[2], f->R[2][0], fmaf(a[1], f->R[1][0], fmaf(a[0], f->R[0][0], f->P[0])));
    w.y = fmaf(a[2], f->R[2][1], fmaf(a[1], f->R[1][1], fmaf(a[0], f->R[0][1], f->P[1])));
    w.z = fmaf(a[2], f->R[2][2], fmaf(a[1], f->R[1][2], fmaf(a[0], f->R[0][2], f->P[2])));
    return w;
}

static void capsules_world(const ro_scene* s, const float q[NQ], v3* A, v3* B) {
    frame F[RP_NUM_LINKS];
    link_frames(s, q, F);
    for (int c = 0; c < s->ncap; ++c) {
        A[c] = to_world(&F[s->cap_link[c]], s->cap_a[c]);
        B[c] = to_world(&F[s->cap_link[c]], s->cap_b[c]);
    }
}

void ro_fk_capsules(const ro_scene* s, const float q[NQ], float* out) {
    v3 A[NCAPMAX], B[NCAPMAX];
    capsules_world(s, q, A, B);
    for (int c = 0; c < s->ncap; ++c) {
        out[6 * c + 0] = A[c].x; out[6 * c + 1] = A[c].y; out[6 * c + 2] = A[c].z;
        out[6 * c + 3] = B[c].x; out[6 * c + 4] = B[c].y; out[6 * c + 5] = B[c].z;
    }
}

typedef struct { float lo[3], hi[3]; } aabb;

static aabb cap_box(v3 a, v3 b, float r) {
    aabb o;
    o.lo[0] = mn(a.x, b.x) - r; o.hi[0] = mx(a.x, b.x) + r;
    o.lo[1] = mn(a.y, b.y) - r; o.hi[1] = mx(a.y, b.y) + r;
    o.lo[2] = mn(a.z, b.z) - r; o.hi[2] = mx(a.z, b.z) + r;
    return o;
}
static int disjoint(const aabb* u, const float lo[3], const float hi[3]) {
    for (int k = 0; k < 3; ++k)
        if (u->lo[k] > hi[k] || u->hi[k] < lo[k]) return 1;
    return 0;
}

/* derivative g(t) = q(t).d of the squared excess; writes |q(t)|^2 */
static float g_of(const float a[3], const float d[3], const float h[3], float t, float* f2) {
    float qv[3];
    for (int k = 0; k < 3; ++k) {
        float p = fmaf(t, d[k], a[k]);
        float cl = p < -h[k] ? -h[k] : (p > h[k] ? h[k] : p);
        qv[k] = p - cl;
    }
    *f2 = fmaf(qv[2], qv[2], fmaf(qv[1], qv[1], qv[0] * qv[0]));
    return fmaf(qv[2], d[2], fmaf(qv[1], d[1], qv[0] * d[0]));
}

/* squared distance segment a-b to box [-h,h] (box frame); DESIGN.md §3.3 */
static float seg_box_d2(const float a[3], const float b[3], const float h[3]) {
    float d[3], T[6];
    for (int k = 0; k < 3; ++k) d[k] = b[k] - a[k];
    for (int k = 0; k < 3; ++k) {
        float u = 0.0f, v = 0.0f;
        if (d[k] != 0.0f) {
            float inv = 1.0f / d[k];
            u = (-h[k] - a[k]) * inv;
            v = (h[k] - a[k]) * inv;
        }
        T[2 * k] = c01(u);
        T[2 * k + 1] = c01(v);
    }
    /* insertion sort: the sorted multiset is what matters */
    for (int i = 1; i < 6; ++i) {
        float x = T[i];
        int j = i - 1;
        while (j >= 0 && T[j] > x) { T[j + 1] = T[j]; --j; }
        T[j + 1] = x;
    }
    float f2, f2e;
    float g0 = g_of(a, d, h, 0.0f, &f2);
    if (g0 >= 0.0f) return f2;
    float g7 = g_of(a, d, h, 1.0f, &f2e);
    if (g7 <= 0.0f) return f2e;
    float tl = 0.0f, gl = g0, tk = 1.0f, gk = g7;
    for (int i = 0; i < 6; ++i) {
        float fi, gi = g_of(a, d, h, T[i], &fi);
        if (gi >= 0.0f) { tk = T[i]; gk = gi; break; }
        tl = T[i];
        gl = gi;
    }
    float ts = fmaf(tk - tl, (-gl) / (gk - gl), tl);
    g_of(a, d, h, ts, &f2);
    return f2;
}

static float seg_seg_d2(v3 a1, v3 b1, v3 a2, v3 b2) {
    v3 d1 = {b1.x - a1.x, b1.y - a1.y, b1.z - a1.z};
    v3 d2 = {b2.x - a2.x, b2.y - a2.y, b2.z - a2.z};
    v3 w = {a1.x - a2.x, a1.y - a2.y, a1.z - a2.z};
    float A = dot(d1, d1), E = dot(d2, d2), F = dot(d2, w);
    float s, t;
    if (A <= 1e-12f) {
        s = 0.0f;
        t = (E <= 1e-12f) ? 0.0f : c01(F / E);
    } else {
        float C = dot(d1, w);
        if (E <= 1e-12f) {
            t = 0.0f;
            s = c01(-C / A);
        } else {
            float Bd = dot(d1, d2);
            float den = fmaf(A, E, -(Bd * Bd));
            s = den > 0.0f ? c01(fmaf(Bd, F, -(C * E)) / den) : 0.0f;
            float tn = fmaf(Bd, s, F);
            if (tn < 0.0f) { t = 0.0f; s = c01(-C / A); }
            else if (tn > E) { t = 1.0f; s = c01((Bd - C) / A); }
            else t = tn / E;
        }
    }
    v3 p1 = {fmaf(d1.x, s, a1.x), fmaf(d1.y, s, a1.y), fmaf(d1.z, s, a1.z)};
    v3 p2 = {fmaf(d2.x, t, a2.x), fmaf(d2.y, t, a2.y), fmaf(d2.z, t, a2.z)};
    v3 dd = {p1.x - p2.x, p1.y - p2.y, p1.z - p2.z};
    return dot(dd, dd);
}

/* world point P in the frame of box j: rotation by -yaw about z (upright), or
 * R^T (P - c) with rows rt (tilted): o_i = fma(rt_i2, dz, fma(rt_i1, dy, rt_i0 dx)) */
static void box_frame(const ro_scene* s, int j, v3 P, float o[3]) {
    const float dx = P.x - s->box_c[j][0], dy = P.y - s->box_c[j][1], dz = P.z - s->box_c[j][2];
    if (s->box_tilt[j]) {
        const float* rt = s->box_rt[j];
        for (int i = 0; i < 3; ++i) o[i] = fmaf(rt[3 * i + 2], dz, fmaf(rt[3 * i + 1], dy, rt[3 * i] * dx));
    } else {
        const float cs = s->box_cs[j], sn = s->box_sn[j];
        o[0] = fmaf(cs, dx, sn * dy);
        o[1] = fmaf(cs, dy, -(sn * dx));
        o[2] = dz;
    }
}

static int cap_vs_box(const ro_scene* s, int c, v3 A, v3 B, const aabb* u, int j) {
    if ((s->box_exempt[j] >> c) & 1u) return 0;
    if (disjoint(u, s->box_lo[j], s->box_hi[j])) return 0;
    float pa[3], pb[3];
    box_frame(s, j, A, pa);
    box_frame(s, j, B, pb);
    const float r = s->cap_r[c];
    return seg_box_d2(pa, pb, s->box_h[j]) <= r * r;
}

static int pair_hit(const ro_scene* s, int p, const v3* A, const v3* B) {
    int i = s->pair[p][0], j = s->pair[p][1];
    aabb u = cap_box(A[i], B[i], s->cap_r[i]);
    aabb v = cap_box(A[j], B[j], s->cap_r[j]);
    if (disjoint(&u, v.lo, v.hi)) return 0;
    float rr = s->cap_r[i] + s->cap_r[j];
    return seg_seg_d2(A[i], B[i], A[j], B[j]) <= rr * rr;
}

int ro_state_valid(const ro_scene* s, const float q[NQ]) {
    v3 A[NCAPMAX], B[NCAPMAX];
    capsules_world(s, q, A, B);
    for (int c = 0; c < s->ncap; ++c) {
        aabb u = cap_box(A[c], B[c], s->cap_r[c]);
        if (u.lo[2] <= s->plane_z) return 0;
        for (int j = 0; j < s->nbox; ++j)
            if (cap_vs_box(s, c, A[c], B[c], &u, j)) return 0;
    }
    for (int p = 0; p < s->npair; ++p)
        if (pair_hit(s, p, A, B)) return 0;
    return 1;
}

int ro_state_contacts(const ro_scene* s, const double qd[NQ], int32_t* out, int32_t cap) {
    float q[NQ];
    for (int i = 0; i < NQ; ++i) q[i] = (float)qd[i];
    v3 A[NCAPMAX], B[NCAPMAX];
    capsules_world(s, q, A, B);
    int n = 0;
#define PUSH(l, o) do { if (n < cap && out) { out[2 * n] = (l); out[2 * n + 1] = (o); } ++n; } while (0)
    for (int c = 0; c < s->ncap; ++c) {
        aabb u = cap_box(A[c], B[c], s->cap_r[c]);
        if (u.lo[2] <= s->plane_z) PUSH(s->cap_link[c], -1);
        for (int j = 0; j < s->nbox; ++j)
            if (cap_vs_box(s, c, A[c], B[c], &u, j)) PUSH(s->cap_link[c], j);
    }
    for (int p = 0; p < s->npair; ++p)
        if (pair_hit(s, p, A, B)) PUSH(s->cap_link[s->pair[p][0]], -2 - s->cap_link[s->pair[p][1]]);
#undef PUSH
    return n;
}

int64_t ro_check_states(const ro_scene* s, const float* q, int64_t n, uint8_t* flags, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < n; ++i) flags[i] = (uint8_t)ro_state_valid(s, q + NQ * i);
    (void)threads;
    return n;
}

/* ------------------------------------------------------------------------- */
/* Philox4x32-10 (Salmon et al. 2011; Random123)                             */
/* ------------------------------------------------------------------------- */

void ro_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#define SAMPLE_TAG 0x52425035u

/* uniform sample g in [lo, hi] */
static void sample_state_tag(uint64_t seed, uint64_t g, const double* lo, const double* hi, double* q,
                             uint32_t tag) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t u[12];
    for (uint32_t j = 0; j < 3; ++j) {
        uint32_t ctr[4] = {(uint32_t)g, (uint32_t)(g >> 32), j, tag};
        ro_philox(ctr, key, u + 4 * j);
    }
    for (int i = 0; i < NQ; ++i) {
        double x = (double)u[i] * 2.3283064365386962890625e-10;
        q[i] = lo[i] + (hi[i] - lo[i]) * x;
    }
}
static void sample_state(uint64_t seed, uint64_t g, const double* lo, const double* hi, double* q) {
    sample_state_tag(seed, g, lo, hi, q, SAMPLE_TAG);
}

/* ------------------------------------------------------------------------- */
/* float64 state space (OMPL RealVectorStateSpace semantics)                 */
/* ------------------------------------------------------------------------- */

static double dist2(const double* a, const double* b) {
    double s = 0.0;
    for (int i = 0; i < NQ; ++i) {
        double d = a[i] - b[i];
        s = s + d * d;
    }
    return s;
}
static void interp(const double* a, const double* b, double t, double* out) {
    for (int i = 0; i < NQ; ++i) out[i] = a[i] + (b[i] - a[i]) * t;
}
static int valid_d(const ro_scene* s, const double* q) {
    float f[NQ];
    for (int i = 0; i < NQ; ++i) f[i] = (float)q[i];
    return ro_state_valid(s, f);
}

/* checkMotion with the endpoint chosen by mode (0: `to`, 1: `from`) — OMPL
 * DiscreteMotionValidator::checkMotion [EXT-OMPL] visits the interior in bisection
 * order; the validity result does not depend on the order. */
static int edge_valid(const ro_scene* s, const double* from, const double* to, int mode, double res,
                      int64_t* states) {
    double d = sqrt(dist2(from, to));
    int nd = (int)ceil(d / res);
    ++*states;
    if (!valid_d(s, mode ? from : to)) return 0;
    if (nd >= 2) {
        /* FIFO of intervals (1, nd-1) */
        int qa[512], qb[512], head = 0, tail = 0;
        int* big_a = NULL;
        int* big_b = NULL;
        int capq = 512;
        int* A = qa;
        int* B = qb;
        if (nd > 500) {
            capq = nd + 8;
            big_a = (int*)malloc(sizeof(int) * capq);
            big_b = (int*)malloc(sizeof(int) * capq);
            A = big_a;
            B = big_b;
        }
        A[tail] = 1; B[tail] = nd - 1; ++tail;
        int ok = 1;
        double st[NQ];
        while (head < tail) {
            int a = A[head], b = B[head];
            ++head;
            int mid = (a + b) / 2;
            interp(from, to, (double)mid / (double)nd, st);
            ++*states;
            if (!valid_d(s, st)) { ok = 0; break; }
            if (a < mid) { A[tail] = a; B[tail] = mid - 1; ++tail; }
            if (mid < b) { A[tail] = mid + 1; B[tail] = b; ++tail; }
        }
        free(big_a);
        free(big_b);
        return ok;
    }
    return 1;
}

int ro_check_edge(const ro_scene* s, const double* qa, const double* qb, double res, int64_t* states) {
    int64_t dummy = 0;
    return edge_valid(s, qa, qb, 0, res, states ? states : &dummy);
}

int64_t ro_check_edges(const ro_scene* s, const double* qa, const double* qb, int64_t n, double res,
                       uint8_t* out) {
    int64_t states = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : states)
#endif
    for (int64_t i = 0; i < n; ++i) {
        int64_t st = 0;
        out[i] = (uint8_t)edge_valid(s, qa + NQ * i, qb + NQ * i, 0, res, &st);
        states += st;
    }
    return states;
}

/* ------------------------------------------------------------------------- */
/* trees                                                                     */
/* ------------------------------------------------------------------------- */

/* Exact nearest-node index for the sequential (batch 1) CPU baseline: an
 * insert-only bucket kd-tree over a tree's nodes. OMPL's RRTConnect searches a
 * GNAT [EXT-OMPL, planning.py:156], not a linear scan, so the CPU planner the GPU
 * is timed against gets a sublinear exact search too. The answer is the linear
 * scan's bit for bit: the same dist2, the lexicographic (distance, index) minimum
 * (= the strict-< scan's lowest index among ties), and a subtree is skipped only
 * if fl(fl(split - x)^2) > best, a lower bound of every dist2 in it (rounding is
 * monotone, the sum's terms are non-negative), so no tie is ever pruned. */
#define KD_LEAF 16
typedef struct {
    int dim;          /* < 0: leaf */
    double split;     /* internal: left = coordinate < split, right = >= split */
    int32_t child[2];
    int32_t* idx;     /* leaf: node indices */
    int32_t cnt, cap;
} kd_node;
typedef struct {
    kd_node* nodes;
    int32_t n, cap;
} kd_tree;

static int32_t kd_new_leaf(kd_tree* k) {
    if (k->n == k->cap) {
        k->cap = k->cap ? 2 * k->cap : 256;
        k->nodes = (kd_node*)realloc(k->nodes, sizeof(kd_node) * k->cap);
    }
    kd_node* nd = &k->nodes[k->n];
    nd->dim = -1;
    nd->split = 0.0;
    nd->child[0] = nd->child[1] = -1;
    nd->cap = KD_LEAF;
    nd->cnt = 0;
    nd->idx = (int32_t*)malloc(sizeof(int32_t) * KD_LEAF);
    return k->n++;
}
static void kd_free(kd_tree* k) {
    for (int32_t i = 0; i < k->n; ++i) free(k->nodes[i].idx);
    free(k->nodes);
    k->nodes = NULL;
    k->n = k->cap = 0;
}
static int cmp_double(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}
/* add node `id` (state q, pts = the tree's states) */
static void kd_insert(kd_tree* k, const double* pts, int32_t id) {
    if (k->n == 0) kd_new_leaf(k);
    const double* q = pts + NQ * (int64_t)id;
    int32_t v = 0;
    while (k->nodes[v].dim >= 0) v = k->nodes[v].child[q[k->nodes[v].dim] >= k->nodes[v].split];
    kd_node* L = &k->nodes[v];
    if (L->cnt == L->cap) {
        /* split at the median of the widest dimension; identical points stay in a
         * growing leaf */
        int dim = -1;
        double spread = 0.0;
        for (int d = 0; d < NQ; ++d) {
            double lo = INFINITY, hi = -INFINITY;
            for (int i = 0; i < L->cnt; ++i) {
                const double c = pts[NQ * (int64_t)L->idx[i] + d];
                lo = c < lo ? c : lo;
                hi = c > hi ? c : hi;
            }
            if (hi - lo > spread) { spread = hi - lo; dim = d; }
        }
        if (dim >= 0) {
            /* (a leaf that grew past KD_LEAF while its points were identical splits
             * too, as soon as they are not: searches stay logarithmic) */
            double* cs = (double*)malloc(sizeof(double) * L->cnt);
            for (int i = 0; i < L->cnt; ++i) cs[i] = pts[NQ * (int64_t)L->idx[i] + dim];
            qsort(cs, L->cnt, sizeof(double), cmp_double);
            double split = cs[L->cnt / 2];
            if (!(split > cs[0])) split = cs[L->cnt - 1];   /* both sides non-empty */
            free(cs);
            const int32_t a = kd_new_leaf(k), b = kd_new_leaf(k);
            L = &k->nodes[v];   /* (realloc) */
            for (int i = 0; i < L->cnt; ++i) {
                const int32_t j = L->idx[i];
                kd_node* C = &k->nodes[pts[NQ * (int64_t)j + dim] >= split ? b : a];
                if (C->cnt == C->cap) {
                    C->cap *= 2;
                    C->idx = (int32_t*)realloc(C->idx, sizeof(int32_t) * C->cap);
                }
                C->idx[C->cnt++] = j;
            }
            free(L->idx);
            L->idx = NULL;
            L->cnt = L->cap = 0;
            L->dim = dim;
            L->split = split;
            L->child[0] = a;
            L->child[1] = b;
            kd_insert(k, pts, id);
            return;
        }
        L->cap *= 2;
        L->idx = (int32_t*)realloc(L->idx, sizeof(int32_t) * L->cap);
    }
    L->idx[L->cnt++] = id;
}
static void kd_search(const kd_tree* k, int32_t v, const double* pts, const double* x, double* best, int32_t* bi) {
    const kd_node* nd = &k->nodes[v];
    if (nd->dim < 0) {
        for (int i = 0; i < nd->cnt; ++i) {
            const int32_t j = nd->idx[i];
            const double d = dist2(pts + NQ * (int64_t)j, x);
            if (d < *best || (d == *best && j < *bi)) { *best = d; *bi = j; }
        }
        return;
    }
    const int side = x[nd->dim] >= nd->split;
    kd_search(k, nd->child[side], pts, x, best, bi);
    const double g = side ? x[nd->dim] - nd->split : nd->split - x[nd->dim];
    if (g * g <= *best) kd_search(k, nd->child[!side], pts, x, best, bi);
}

typedef struct {
    double* q;
    int32_t* parent;
    uint8_t* cand;   /* start tree: extension node whose connect did not reach */
    int64_t n, cap;
    kd_tree* kd;     /* sequential baseline: exact index over all n nodes (else NULL) */
    int kd_want;     /* build the index once the tree outgrows a linear scan */
} tree_t;

static int tree_init(tree_t* t, int64_t cap) {
    t->q = (double*)malloc(sizeof(double) * NQ * cap);
    t->parent = (int32_t*)malloc(sizeof(int32_t) * cap);
    t->cand = (uint8_t*)calloc(cap, 1);
    t->n = 0;
    t->cap = cap;
    t->kd = NULL;
    t->kd_want = 0;
    return t->q && t->parent && t->cand;
}
static void tree_free(tree_t* t) {
    free(t->q);
    free(t->parent);
    free(t->cand);
    if (t->kd) {
        kd_free(t->kd);
        free(t->kd);
    }
}
static int64_t tree_add(tree_t* t, const double* q, int32_t parent) {
    memcpy(t->q + NQ * t->n, q, sizeof(double) * NQ);
    t->parent[t->n] = parent;
    t->cand[t->n] = 0;
    if (t->kd) kd_insert(t->kd, t->q, (int32_t)t->n);
    return t->n++;
}
/* nearest node among the first n (ties -> lowest index); the kd index (which holds
 * exactly the tree's nodes) when the tree has one and n is all of them. The index is
 * built when a tree that wants one passes KD_MIN nodes (a linear scan is faster
 * below), then kept up to date by tree_add. */
#define KD_MIN 256
static int32_t nearest(tree_t* t, int64_t n, const double* x) {
    double best = INFINITY;
    int32_t idx = -1;
    if (t->kd_want && !t->kd && t->n > KD_MIN) {
        t->kd = (kd_tree*)calloc(1, sizeof(kd_tree));
        for (int64_t j = 0; j < t->n; ++j) kd_insert(t->kd, t->q, (int32_t)j);
    }
    if (t->kd && n == t->n && t->kd->n > 0) {
        kd_search(t->kd, 0, t->q, x, &best, &idx);
        return idx;
    }
    for (int64_t j = 0; j < n; ++j) {
        double d = dist2(t->q + NQ * j, x);
        if (d < best) { best = d; idx = (int32_t)j; }
    }
    return idx;
}

static void steer(const double* near, const double* target, double range, double* out, int* reach) {
    double d = sqrt(dist2(near, target));
    if (d > range) {
        interp(near, target, range / d, out);
        *reach = 0;
    } else {
        memcpy(out, target, sizeof(double) * NQ);
        *reach = 1;
    }
}

/* connect chain from node state y toward x: up to cmax steps of `range`
 * (cmax = ceil(maxExtent / range) + 1 covers any pair of in-bounds states).
 * Returns step count m; *reach = whether step m lands on x. */
static int build_chain(const double* y, const double* x, double range, double (*chain)[NQ], int cmax,
                       int* reach) {
    const double* cur = y;
    *reach = 0;
    for (int m = 0; m < cmax; ++m) {
        int r;
        steer(cur, x, range, chain[m], &r);
        if (r) { *reach = 1; return m + 1; }
        cur = chain[m];
    }
    return cmax;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int out_of_bounds(const double* q, const double* lo, const double* hi) {
    const double eps = 2.220446049250313e-16; /* OMPL satisfiesBounds tolerance */
    for (int i = 0; i < NQ; ++i)
        if (q[i] - eps > hi[i] || q[i] + eps < lo[i]) return 1;
    return 0;
}

/* PathGeometric::interpolate(count) [EXT-OMPL, SURVEY App. B.4] */
int ro_interpolate(const double* path, int32_t n, int32_t count, double* out, int32_t cap) {
    if (count < n || n < 2) {
        if (n > cap) return -1;
        memcpy(out, path, sizeof(double) * NQ * n);
        return n;
    }
    if (count > cap) return -1;
    double remaining = 0.0;
    for (int i = 0; i + 1 < n; ++i) remaining += sqrt(dist2(path + NQ * i, path + NQ * (i + 1)));
    int m = 0;
    int cnt = count;
    const int n1 = n - 1;
    for (int i = 0; i < n1; ++i) {
        const double* s1 = path + NQ * i;
        const double* s2 = path + NQ * (i + 1);
        memcpy(out + NQ * m++, s1, sizeof(double) * NQ);
        int maxN = cnt + i - n;
        if (maxN > 0) {
            double seg = sqrt(dist2(s1, s2));
            int ns = (i + 1 == n1) ? maxN + 2 : (int)floor(0.5 + (double)cnt * seg / remaining) + 1;
            if (ns > 2) {
                ns -= 2;
                if (ns > maxN) ns = maxN;
                for (int j = 1; j <= ns; ++j) interp(s1, s2, (double)j / (double)(ns + 1), out + NQ * m++);
            } else {
                ns = 0;
            }
            cnt -= ns + 1;
            remaining -= seg;
        } else {
            cnt--;
        }
    }
    memcpy(out + NQ * m++, path + NQ * n1, sizeof(double) * NQ);
    return m;
}

/* walk a tree from node to its root (inclusive) */
static int walk(const tree_t* t, int32_t node, double* out, int cap) {
    int n = 0;
    while (node >= 0) {
        if (n >= cap) return -1;
        memcpy(out + NQ * n++, t->q + NQ * node, sizeof(double) * NQ);
        node = t->parent[node];
    }
    return n;
}

/* Path simplification: a deterministic restatement of the
 * structure of OMPL PathSimplifier::simplifyMax [EXT-OMPL] (planning.py:195-196):
 * reduceVertices + collapseCloseVertices -> a greedy farthest-valid shortcut over
 * all vertex pairs; smoothBSpline(path, 3, length / 100) restated exactly (it is
 * deterministic in OMPL); its subdivision midpoints then give the next reduction
 * the segment-interior shortcut points of shortcutPath. Rounds repeat while the
 * path gets shorter. Level 1 = all of it, level 2 = the shortcut only. */
#define SIMPLIFY_MAXN 1024
/* batched RRT loops run OpenMP over samples / targets from this many on (the
 * sequential B = 1 CPU baseline stays single-threaded) */
#define OMP_MIN_ITEMS 512
#define SIMPLIFY_ROUNDS 2
#define SMOOTH_STEPS 3
#define SMOOTH_MAX 256   /* a smoothing round runs only if 8n - 7 <= SMOOTH_MAX */

static double path_length(const double* P, int n) {
    double L = 0.0;
    for (int i = 0; i + 1 < n; ++i) L = L + sqrt(dist2(P + NQ * i, P + NQ * (i + 1)));
    return L;
}

/* greedy vertex reduction: from each kept vertex jump to the farthest later
 * vertex with a valid straight edge */
static int reduce_vertices(const ro_scene* s, double* path, int n, double res, int64_t* states) {
    if (n < 3 || n > SIMPLIFY_MAXN) return n;
    double* out = (double*)malloc(sizeof(double) * NQ * n);
    int m = 0, i = 0;
    memcpy(out, path, sizeof(double) * NQ);
    m = 1;
    while (i < n - 1) {
        int j = n - 1;
        while (j > i + 1 && !edge_valid(s, path + NQ * i, path + NQ * j, 0, res, states)) --j;
        memcpy(out + NQ * m++, path + NQ * j, sizeof(double) * NQ);
        i = j;
    }
    memcpy(path, out, sizeof(double) * NQ * m);
    free(out);
    return m;
}

/* OMPL PathSimplifier::smoothBSpline(path, steps, min_change) [EXT-OMPL]; P has
 * room for 2^steps (n - 1) + 1 states */
static int smooth_bspline(const ro_scene* s, double* P, int n, int steps, double min_change, double res,
                          int64_t* states) {
    if (n < 3) return n;
    double* Q = (double*)malloc(sizeof(double) * NQ * (2 * n));
    for (int step = 0; step < steps; ++step) {
        /* PathGeometric::subdivide: a midpoint between every pair of states */
        memcpy(Q, P, sizeof(double) * NQ);
        for (int k = 1; k < n; ++k) {
            interp(P + NQ * (k - 1), P + NQ * k, 0.5, Q + NQ * (2 * k - 1));
            memcpy(Q + NQ * (2 * k), P + NQ * k, sizeof(double) * NQ);
        }
        n = 2 * n - 1;
        memcpy(P, Q, sizeof(double) * NQ * n);
        Q = (double*)realloc(Q, sizeof(double) * NQ * (2 * n));
        int u = 0;
        for (int i = 2; i < n - 1; i += 2) {
            double t1[NQ], t2[NQ];
            const double* a = P + NQ * (i - 1);
            const double* b = P + NQ * (i + 1);
            ++*states;
            if (!valid_d(s, a)) continue;
            interp(a, P + NQ * i, 0.5, t1);
            interp(P + NQ * i, b, 0.5, t2);
            interp(t1, t2, 0.5, t1);
            if (edge_valid(s, a, t1, 0, res, states) && edge_valid(s, t1, b, 0, res, states)) {
                if (sqrt(dist2(P + NQ * i, t1)) > min_change) {
                    memcpy(P + NQ * i, t1, sizeof(double) * NQ);
                    ++u;
                }
            }
        }
        if (u == 0) break;
    }
    free(Q);
    return n;
}

/* level 1: reduce, then rounds of smooth + reduce while the length decreases;
 * level 2: reduce only. path has room for max(n, SMOOTH_MAX) states. */
static int simplify_path(const ro_scene* s, double* path, int n, int level, double res, int64_t* states) {
    if (n < 3 || n > SIMPLIFY_MAXN || level <= 0) return n;
    n = reduce_vertices(s, path, n, res, states);
    if (level == 2) return n;
    double* Q = (double*)malloc(sizeof(double) * NQ * SMOOTH_MAX);
    for (int r = 0; r < SIMPLIFY_ROUNDS; ++r) {
        if (n < 3 || 8 * n - 7 > SMOOTH_MAX) break;
        const double L0 = path_length(path, n);
        memcpy(Q, path, sizeof(double) * NQ * n);
        int m = smooth_bspline(s, Q, n, SMOOTH_STEPS, L0 / 100.0, res, states);
        m = reduce_vertices(s, Q, m, res, states);
        if (!(path_length(Q, m) < L0)) break;
        memcpy(path, Q, sizeof(double) * NQ * m);
        n = m;
    }
    free(Q);
    return n;
}

int ro_plan(const ro_scene* s, const double start[NQ], const double goal[NQ], const double lo[NQ],
            const double hi[NQ], const rp_plan_params* pp, int32_t rank, int32_t world,
            ro_allgather_fn fn, void* user, double* path_out, int32_t path_cap, int32_t* n_out,
            int32_t* status_out, rp_stats* stats) {
    const double t_begin = now_s();
    rp_stats st;
    memset(&st, 0, sizeof st);
    *n_out = 0;
    *status_out = RP_STATUS_NONE;
    if (world < 1) world = 1;
    if (rank < 0 || rank >= world) return RP_ERR_ARG;
    if (world > 1 && !fn) return RP_ERR_ARG;

    double ext2 = 0.0;
    for (int i = 0; i < NQ; ++i) ext2 += (hi[i] - lo[i]) * (hi[i] - lo[i]);
    const double max_extent = sqrt(ext2);
    rp_plan_params p = *pp;
    if (p.batch <= 0) p.batch = 4096;
    if (p.range <= 0) p.range = 0.2 * max_extent;
    if (p.resolution <= 0) p.resolution = 0.01 * max_extent;
    if (p.timeout_s <= 0) p.timeout_s = 5.0;
    if (p.max_iters <= 0) p.max_iters = INT64_MAX;
    if (p.tree_capacity <= 0) p.tree_capacity = 1 << 22;
    if (p.batch % world) return RP_ERR_ARG;
    /* batch schedule: iteration k draws min(batch, batch_min << k) samples; the
     * global sample counter keeps running, so the schedule is part of the
     * algorithm's definition (same on every rank and on the GPU) */
    if (p.batch_min <= 0) p.batch_min = p.batch < 64 ? p.batch : 64;
    if (p.batch_min > p.batch) p.batch_min = p.batch;
    p.batch_min = ((p.batch_min + world - 1) / world) * world;
    const int cmax = (int)ceil(max_extent / p.range) + 1;
    /* rank groups (include/rbe_planner.h group_repl): iterations of at most `repl`
     * samples are replicated here (every rank computes all of it, no exchange), larger
     * ones sharded. rp_lib.hip decides per sub-batch instead (an execution detail:
     * the trees are the same); what both share is the timeout vote, which follows the
     * GPU's first sub-batch of the iteration (chunk0 = rp_plan_params.chunk, default
     * 64; at least a quarter of the iteration on trees of >= 4,096 nodes): when it is
     * sharded the vote rides on the iteration's first exchange, when it is replicated
     * the group exchanges the flags alone every RP_GROUP_VOTE_EVERY iterations */
    int64_t repl = p.group_repl > 0 ? p.group_repl : p.group_repl < 0 ? 0 : RP_GROUP_REPL_DEFAULT;
    if (world == 1) repl = 0;
    int64_t chunk0 = p.chunk > 0 ? p.chunk : p.chunk < 0 ? INT64_MAX : 64;
    if (chunk0 != INT64_MAX) chunk0 = ((chunk0 + world - 1) / world) * world;

    /* PlannerInputStates: invalid start / goal are skipped -> status */
    if (out_of_bounds(start, lo, hi) || !valid_d(s, start)) {
        *status_out = RP_STATUS_INVALID_START;
        st.states_checked += 1;
        if (stats) *stats = st;
        return RP_OK;
    }
    if (out_of_bounds(goal, lo, hi) || !valid_d(s, goal)) {
        *status_out = RP_STATUS_INVALID_GOAL;
        st.states_checked += 2;
        if (stats) *stats = st;
        return RP_OK;
    }
    st.states_checked += 2;

    /* straight-first (rp_plan_params.straight_first, rp_lib.hip plan_impl): with
     * simplification on, a valid straight edge start -> goal is the path REDUCE's
     * greedy farthest-valid walk would shorten any solution to, so it is checked
     * first and returned when valid */
    if (p.simplify > 0 && p.straight_first >= 0) {
        st.edges_checked++;
        if (edge_valid(s, start, goal, 0, p.resolution, &st.states_checked)) {
            double raw2[2 * NQ];
            memcpy(raw2, start, sizeof(double) * NQ);
            memcpy(raw2 + NQ, goal, sizeof(double) * NQ);
            int m = (p.n_waypoints > 0) ? ro_interpolate(raw2, 2, p.n_waypoints, path_out, path_cap)
                                        : (2 <= path_cap ? (memcpy(path_out, raw2, sizeof raw2), 2) : -1);
            st.start_tree_size = st.goal_tree_size = 1;
            st.path_states_raw = st.path_states_simplified = 2;
            st.total_ms = 1e3 * (now_s() - t_begin);
            if (stats) *stats = st;
            if (m < 0) return RP_ERR_CAPACITY;
            *n_out = m;
            *status_out = RP_STATUS_EXACT;
            return RP_OK;
        }
    }

    tree_t T[2];
    if (!tree_init(&T[0], p.tree_capacity) || !tree_init(&T[1], p.tree_capacity)) return RP_ERR_CAPACITY;
    /* the sequential loop (one sample per iteration, one rank): exact kd-tree
     * nearest-node searches (RBE_ORACLE_KD=0: the linear scan, same answers) */
    {
        const char* e = getenv("RBE_ORACLE_KD");
        if (p.batch == 1 && world == 1 && !(e && *e == '0')) T[0].kd_want = T[1].kd_want = 1;
    }
    tree_add(&T[0], start, -1);
    tree_add(&T[1], goal, -1);

    const int64_t BMAX = p.batch;
    int64_t B = p.batch_min;
    uint64_t gbase = 0;
    int32_t* res = (int32_t*)malloc(sizeof(int32_t) * BMAX);
    int32_t* mine = (int32_t*)malloc(sizeof(int32_t) * (BMAX + 1));
    int32_t* rbuf = (int32_t*)malloc(sizeof(int32_t) * (BMAX / world + 1) * world);
    int64_t* tnode = (int64_t*)malloc(sizeof(int64_t) * BMAX);
    int32_t* trec = (int32_t*)malloc(sizeof(int32_t) * 2 * (BMAX + world));
    int32_t* tmine = (int32_t*)malloc(sizeof(int32_t) * 2 * (BMAX + world));
    double (*chain)[NQ] = (double(*)[NQ])malloc(sizeof(double) * NQ * cmax);

    int solved = 0;
    int32_t s_node = -1, g_node = -1; /* solution join nodes (start tree, goal tree) */
    const double t_solve = now_s();
    int64_t iter = 0;
    for (; iter < p.max_iters; ++iter) {
        /* timeout: in a group every rank votes through the first exchange so that
         * all ranks leave the loop at the same iteration */
        const int tflag = (now_s() - t_solve) >= p.timeout_s;
        if (world == 1 && tflag) break;
        const int repl_it = world > 1 && B <= repl;
        const int a_start = (iter % 2) == 0;
        tree_t* A = a_start ? &T[0] : &T[1];
        tree_t* Bt = a_start ? &T[1] : &T[0];
        if (A->n + B > A->cap || Bt->n + B * cmax > Bt->cap) break;
        const int64_t TA = A->n, TB = Bt->n;
        /* the timeout vote (rp_lib.hip plan_impl, group_vote) */
        int64_t c_first = B < chunk0 ? B : chunk0;
        if (TA + TB >= 4096) {
            const int64_t quarter = ((B / 4 + world - 1) / world) * world;
            if (quarter > c_first) c_first = quarter;
            if (c_first > B) c_first = B;
        }
        const int vote_first = world > 1 && c_first > repl;
        if (world > 1 && !vote_first && iter % RP_GROUP_VOTE_EVERY == RP_GROUP_VOTE_EVERY - 1) {
            double te = now_s();
            mine[0] = tflag;
            if (fn(user, mine, rbuf, (int64_t)sizeof(int32_t))) { solved = -1; break; }
            st.exchange_ms += 1e3 * (now_s() - te);
            int any = 0;
            for (int r = 0; r < world; ++r) any |= rbuf[r];
            if (any) break;
        }
        const uint64_t g0 = gbase;
        const int64_t per = repl_it ? B : B / world;
        const int64_t off = repl_it ? 0 : rank * per;
        /* extension: my slice of the batch (samples are independent: OpenMP over
         * them for large batches, same results as the serial loop) */
        int64_t ext_states = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : ext_states) if (per >= OMP_MIN_ITEMS)
        for (int64_t k = 0; k < per; ++k) {
            const int64_t i = off + k;
            double qr[NQ], qn[NQ];
            int reach;
            sample_state(p.seed, g0 + (uint64_t)i, lo, hi, qr);
            int32_t nn = nearest(A, TA, qr);
            steer(A->q + NQ * nn, qr, p.range, qn, &reach);
            int ok = a_start ? edge_valid(s, A->q + NQ * nn, qn, 0, p.resolution, &ext_states)
                             : edge_valid(s, qn, A->q + NQ * nn, 1, p.resolution, &ext_states);
            mine[k] = ok ? nn : -1;
        }
        st.states_checked += ext_states;
        st.edges_checked += per;
        if (world > 1 && !repl_it) {
            double te = now_s();
            mine[per] = vote_first ? tflag : 0;
            if (fn(user, mine, rbuf, (int64_t)(sizeof(int32_t) * (per + 1)))) { solved = -1; break; }
            st.exchange_ms += 1e3 * (now_s() - te);
            int any = 0;
            for (int r = 0; r < world; ++r) {
                memcpy(res + r * per, rbuf + r * (per + 1), sizeof(int32_t) * per);
                any |= rbuf[r * (per + 1) + per];
            }
            if (any) break;
        } else {
            memcpy(res, mine, sizeof(int32_t) * per);
        }
        /* append accepted extension nodes in global sample order */
        int64_t nacc = 0;
        for (int64_t i = 0; i < B; ++i) {
            if (res[i] < 0) continue;
            double qr[NQ], qn[NQ];
            int reach;
            sample_state(p.seed, g0 + (uint64_t)i, lo, hi, qr);
            steer(A->q + NQ * res[i], qr, p.range, qn, &reach);
            tnode[nacc++] = tree_add(A, qn, res[i]);
        }
        st.samples += B;
        /* connect: my slice of the accepted targets (independent: OpenMP) */
        const int64_t pt = repl_it ? nacc : (nacc + world - 1) / world;
        const int64_t toff = repl_it ? 0 : rank * pt;
        int64_t con_states = 0, con_edges = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : con_states, con_edges) if (pt >= OMP_MIN_ITEMS)
        for (int64_t k = 0; k < pt; ++k) {
            const int64_t t = toff + k;
            tmine[2 * k] = -1;
            tmine[2 * k + 1] = 0;
            if (t >= nacc) continue;
            double (*ch)[NQ] = (double(*)[NQ])malloc(sizeof(double) * NQ * cmax);
            const double* x = A->q + NQ * tnode[t];
            int32_t y = nearest(Bt, TB, x);
            int reach;
            int m = build_chain(Bt->q + NQ * y, x, p.range, ch, cmax, &reach);
            int L = 0;
            for (int c = 0; c < m; ++c) {
                const double* from = c == 0 ? Bt->q + NQ * y : ch[c - 1];
                int ok = a_start ? edge_valid(s, ch[c], from, 1, p.resolution, &con_states)
                                 : edge_valid(s, from, ch[c], 0, p.resolution, &con_states);
                con_edges++;
                if (!ok) break;
                ++L;
            }
            free(ch);
            tmine[2 * k] = y;
            tmine[2 * k + 1] = L;
        }
        st.states_checked += con_states;
        st.edges_checked += con_edges;
        if (world > 1 && !repl_it) {
            double te = now_s();
            if (fn(user, tmine, trec, (int64_t)(sizeof(int32_t) * 2 * pt))) { solved = -1; break; }
            st.exchange_ms += 1e3 * (now_s() - te);
        } else {
            memcpy(trec, tmine, sizeof(int32_t) * 2 * pt);
        }
        /* append connect chains in target order; the first REACHED target wins and
         * ends the iteration: the trees keep the appends of the samples up to and
         * including the winning one, none after it (rp_lib.hip plan_impl runs an
         * iteration as ordered sub-batches and stops after the one that solves; the
         * path only depends on the iteration's snapshot and the winning sample, so
         * this truncation is what makes the result independent of the sub-batching) */
        for (int64_t t = 0; t < nacc; ++t) {
            const int32_t y = trec[2 * t];
            const int L = trec[2 * t + 1];
            const double* x = A->q + NQ * tnode[t];
            int reach;
            int m = build_chain(Bt->q + NQ * y, x, p.range, chain, cmax, &reach);
            int32_t par = y;
            for (int c = 0; c < L; ++c) par = (int32_t)tree_add(Bt, chain[c], par);
            const int reached = (L == m) && reach;
            if (reached) {
                solved = 1;
                if (a_start) {       /* x in start tree, chain end in goal tree */
                    s_node = A->parent[tnode[t]];
                    g_node = par;
                } else {             /* chain end in start tree, x in goal tree */
                    s_node = Bt->parent[par];
                    g_node = (int32_t)tnode[t];
                }
                A->n = tnode[t] + 1;   /* drop the later samples' extension nodes */
                break;
            }
            if (a_start) A->cand[tnode[t]] = 1;
        }
        gbase += (uint64_t)B;
        B = 2 * B < BMAX ? 2 * B : BMAX;
        if (solved) { ++iter; break; }
    }
    st.iterations = iter;
    st.solve_ms = 1e3 * (now_s() - t_solve);
    st.start_tree_size = T[0].n;
    st.goal_tree_size = T[1].n;

    int rc = RP_OK;
    int64_t cap = T[0].n + T[1].n + 2;
    if (cap < SMOOTH_MAX) cap = SMOOTH_MAX;   /* simplification may return more states than it got */
    double* raw = (double*)malloc(sizeof(double) * NQ * cap);
    int n_raw = 0;
    if (solved == 1) {
        int ns = walk(&T[0], s_node, raw, (int)cap);
        for (int i = 0; i < ns / 2; ++i)
            for (int k = 0; k < NQ; ++k) {
                double tmp = raw[NQ * i + k];
                raw[NQ * i + k] = raw[NQ * (ns - 1 - i) + k];
                raw[NQ * (ns - 1 - i) + k] = tmp;
            }
        int ng = walk(&T[1], g_node, raw + NQ * ns, (int)(cap - ns));
        n_raw = ns + ng;
        *status_out = RP_STATUS_EXACT;
    } else if (solved == 0) {
        /* approximate: start-tree extension node closest to the goal */
        double best = INFINITY;
        int32_t bi = -1;
        for (int64_t j = 0; j < T[0].n; ++j) {
            if (!T[0].cand[j]) continue;
            double d = dist2(T[0].q + NQ * j, goal);
            if (d < best) { best = d; bi = (int32_t)j; }
        }
        if (bi >= 0) {
            int ns = walk(&T[0], bi, raw, (int)cap);
            for (int i = 0; i < ns / 2; ++i)
                for (int k = 0; k < NQ; ++k) {
                    double tmp = raw[NQ * i + k];
                    raw[NQ * i + k] = raw[NQ * (ns - 1 - i) + k];
                    raw[NQ * (ns - 1 - i) + k] = tmp;
                }
            n_raw = ns;
            *status_out = RP_STATUS_APPROXIMATE;
        } else {
            *status_out = RP_STATUS_TIMEOUT;
        }
    } else {
        rc = RP_ERR_EXCHANGE;
    }
    st.path_states_raw = n_raw;
    if (n_raw > 0) {
        double t0 = now_s();
        if (p.simplify) n_raw = simplify_path(s, raw, n_raw, p.simplify, p.resolution, &st.states_checked);
        st.simplify_ms = 1e3 * (now_s() - t0);
        st.path_states_simplified = n_raw;
        int m = (p.n_waypoints > 0) ? ro_interpolate(raw, n_raw, p.n_waypoints, path_out, path_cap)
                                    : (n_raw <= path_cap ? (memcpy(path_out, raw, sizeof(double) * NQ * n_raw), n_raw) : -1);
        if (m < 0) rc = RP_ERR_CAPACITY;
        else *n_out = m;
    }
    free(raw);
    free(res); free(mine); free(rbuf); free(tnode); free(trec); free(tmine); free(chain);
    tree_free(&T[0]);
    tree_free(&T[1]);
    st.total_ms = 1e3 * (now_s() - t_begin);
    if (stats) *stats = st;
    return rc;
}

/* geometry primitives exported for the unit tests */
float ro_seg_box_d2(const float a[3], const float b[3], const float h[3]) { return seg_box_d2(a, b, h); }
float ro_seg_seg_d2(const float a1[3], const float b1[3], const float a2[3], const float b2[3]) {
    v3 p = {a1[0], a1[1], a1[2]}, q = {b1[0], b1[1], b1[2]}, r = {a2[0], a2[1], a2[2]}, s = {b2[0], b2[1], b2[2]};
    return seg_seg_d2(p, q, r, s);
}

/* ------------------------------------------------------------------------- */
/* hand-link inverse kinematics (rp_ik; Genesis robot.inverse_kinematics as    */
/* called by code/motion_primitives.py:131-134 [EXT-GS])                       */
/* ------------------------------------------------------------------------- */
/* Damped least squares on the hand pose from n_seeds restarts per target
 * (restart 0 = init, the others Philox samples with tag IK_TAG), float64 in a
 * fixed operation order so the GPU lanes are reproduced bit for bit. */
#define IK_TAG 0x524B494Bu

/* sin / cos: Cody-Waite reduction by pi/2 and the fdlibm kernel polynomials */
void ro_sincos64(double x, double* s, double* c) {
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

/* translation of each joint frame in its parent, then the
 * x-rotation (+-90 deg) of the frame before the joint's z rotation */
static const double IKT[7][3] = {{0.0, 0.0, 0.333}, {0.0, 0.0, 0.0}, {0.0, -0.316, 0.0}, {0.0825, 0.0, 0.0},
                                 {-0.0825, 0.384, 0.0}, {0.0, 0.0, 0.0}, {0.088, 0.0, 0.0}};
static const int IKRX[7] = {0, -1, 1, 1, -1, 1, 1};
#define IK_FLANGE 0.107
#define IK_C45 0.70710678118654757

typedef struct { double R[3][3]; double p[3]; double z[7][3]; double o[7][3]; } hand_fk_t;

static void hand_fk(const double* q, const double base[3], hand_fk_t* f) {
    double c0[3] = {1.0, 0.0, 0.0}, c1[3] = {0.0, 1.0, 0.0}, c2[3] = {0.0, 0.0, 1.0};
    double p[3] = {base[0], base[1], base[2]};
    for (int j = 0; j < 7; ++j) {
        const double* t = IKT[j];
        for (int i = 0; i < 3; ++i) p[i] = p[i] + (c0[i] * t[0] + c1[i] * t[1] + c2[i] * t[2]);
        for (int i = 0; i < 3; ++i) {
            const double a = c1[i];
            if (IKRX[j] > 0) { c1[i] = c2[i]; c2[i] = -a; }
            else if (IKRX[j] < 0) { c1[i] = -c2[i]; c2[i] = a; }
        }
        for (int i = 0; i < 3; ++i) { f->z[j][i] = c2[i]; f->o[j][i] = p[i]; }
        double sn, cs;
        ro_sincos64(q[j], &sn, &cs);
        for (int i = 0; i < 3; ++i) {
            const double a = c0[i], b = c1[i];
            c0[i] = cs * a + sn * b;
            c1[i] = cs * b - sn * a;
        }
    }
    for (int i = 0; i < 3; ++i) p[i] = p[i] + IK_FLANGE * c2[i];
    for (int i = 0; i < 3; ++i) {
        const double a = c0[i], b = c1[i];
        c0[i] = IK_C45 * a + -IK_C45 * b;
        c1[i] = IK_C45 * b - -IK_C45 * a;
    }
    for (int i = 0; i < 3; ++i) { f->R[0][i] = c0[i]; f->R[1][i] = c1[i]; f->R[2][i] = c2[i]; f->p[i] = p[i]; }
}

static void cross3(const double* a, const double* b, double* o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

static void quat_columns(const double* qt, double T[3][3]) {
    const double n = sqrt(qt[0] * qt[0] + qt[1] * qt[1] + qt[2] * qt[2] + qt[3] * qt[3]);
    const double w = qt[0] / n, x = qt[1] / n, y = qt[2] / n, z = qt[3] / n;
    T[0][0] = 1.0 - 2.0 * (y * y + z * z); T[0][1] = 2.0 * (x * y + w * z); T[0][2] = 2.0 * (x * z - w * y);
    T[1][0] = 2.0 * (x * y - w * z); T[1][1] = 1.0 - 2.0 * (x * x + z * z); T[1][2] = 2.0 * (y * z + w * x);
    T[2][0] = 2.0 * (x * z + w * y); T[2][1] = 2.0 * (y * z - w * x); T[2][2] = 1.0 - 2.0 * (x * x + y * y);
}

static void pose_error(const hand_fk_t* f, const double* pt, double T[3][3], double e[6], double e2[2]) {
    double x0[3], x1[3], x2[3];
    cross3(f->R[0], T[0], x0);
    cross3(f->R[1], T[1], x1);
    cross3(f->R[2], T[2], x2);
    for (int i = 0; i < 3; ++i) {
        e[i] = pt[i] - f->p[i];
        e[3 + i] = 0.5 * (x0[i] + x1[i] + x2[i]);
    }
    e2[0] = e[0] * e[0] + e[1] * e[1] + e[2] * e[2];
    e2[1] = e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
}

void ro_hand_pose(const ro_scene* s, const double q[NQ], double R[9], double p[3]) {
    const double base[3] = {s->base[0], s->base[1], s->base[2]};
    hand_fk_t f;
    hand_fk(q, base, &f);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] = f.R[c][r];
    for (int i = 0; i < 3; ++i) p[i] = f.p[i];
}

/* one restart: q (in/out, 9), squared pose errors e2; returns converged */
static int ik_solve(const double* pt, double T[3][3], const double base[3], const double* lo, const double* hi,
                    int iters, double damping, double pos_tol, double rot_tol, double* q, double e2[2]) {
    const double lam2 = damping * damping;
    const double stop_p = (0.01 * pos_tol) * (0.01 * pos_tol), stop_r = (0.01 * rot_tol) * (0.01 * rot_tol);
    hand_fk_t f;
    double e[6];
    for (int it = 0; it < iters; ++it) {
        hand_fk(q, base, &f);
        pose_error(&f, pt, T, e, e2);
        if (e2[0] <= stop_p && e2[1] <= stop_r) break;
        double J[6][7];
        for (int j = 0; j < 7; ++j) {
            const double d[3] = {f.p[0] - f.o[j][0], f.p[1] - f.o[j][1], f.p[2] - f.o[j][2]};
            double v[3];
            cross3(f.z[j], d, v);
            for (int i = 0; i < 3; ++i) { J[i][j] = v[i]; J[3 + i][j] = f.z[j][i]; }
        }
        double L[6][6];
        for (int r = 0; r < 6; ++r)
            for (int c = 0; c <= r; ++c) {
                double sum = 0.0;
                for (int j = 0; j < 7; ++j) sum = sum + J[r][j] * J[c][j];
                if (r == c) sum = sum + lam2;
                for (int m = 0; m < c; ++m) sum = sum - L[r][m] * L[c][m];
                L[r][c] = (r == c) ? sqrt(sum) : sum / L[c][c];
            }
        double y[6], x[6];
        for (int r = 0; r < 6; ++r) {
            double sum = e[r];
            for (int m = 0; m < r; ++m) sum = sum - L[r][m] * y[m];
            y[r] = sum / L[r][r];
        }
        for (int r = 5; r >= 0; --r) {
            double sum = y[r];
            for (int m = r + 1; m < 6; ++m) sum = sum - L[m][r] * x[m];
            x[r] = sum / L[r][r];
        }
        for (int j = 0; j < 7; ++j) {
            double dq = 0.0;
            for (int r = 0; r < 6; ++r) dq = dq + J[r][j] * x[r];
            double v = q[j] + dq;
            if (v < lo[j]) v = lo[j];
            if (v > hi[j]) v = hi[j];
            q[j] = v;
        }
    }
    hand_fk(q, base, &f);
    pose_error(&f, pt, T, e, e2);
    return e2[0] <= pos_tol * pos_tol && e2[1] <= rot_tol * rot_tol;
}

int ro_ik(const ro_scene* s, int32_t n_targets, const double* pos, const double* quat, const double* init,
          const double lo[NQ], const double hi[NQ], const rp_ik_params* pp, double* q_out, int32_t* status_out) {
    if (!s || n_targets < 0 || !pp || (n_targets > 0 && (!pos || !quat || !init || !q_out || !status_out)))
        return RP_ERR_ARG;
    rp_ik_params p = *pp;
    if (p.n_seeds <= 0) p.n_seeds = 256;
    if (p.iters <= 0) p.iters = 64;
    if (p.damping <= 0) p.damping = 0.01;
    if (p.pos_tol <= 0) p.pos_tol = 5e-4;
    if (p.rot_tol <= 0) p.rot_tol = 5e-3;
    const double base[3] = {s->base[0], s->base[1], s->base[2]};
    for (int t = 0; t < n_targets; ++t) {
        double T[3][3];
        quat_columns(quat + 4 * t, T);
        const double* qi = init + NQ * t;
        int best_c = 3, best_k = 0;
        double best_v = 0.0, best_q[NQ];
        for (int k = 0; k < p.n_seeds; ++k) {
            const uint64_t g = (uint64_t)t * (uint64_t)p.n_seeds + (uint64_t)k;
            double q[NQ], e2[2];
            if (k == 0) {
                memcpy(q, qi, sizeof q);
            } else {
                sample_state_tag(p.seed, g, lo, hi, q, IK_TAG);
                q[7] = qi[7];
                q[8] = qi[8];
            }
            const int conv = ik_solve(pos + 3 * t, T, base, lo, hi, p.iters, p.damping, p.pos_tol, p.rot_tol, q, e2);
            int cls = 2;
            if (conv) {
                float f[NQ];
                for (int i = 0; i < NQ; ++i) f[i] = (float)q[i];
                cls = ro_state_valid(s, f) ? 0 : 1;
            }
            const double v = cls < 2 ? dist2(q, qi) : e2[0] + e2[1];
            if (cls < best_c || (cls == best_c && v < best_v)) {
                best_c = cls;
                best_v = v;
                best_k = k;
                memcpy(best_q, q, sizeof q);
            }
        }
        (void)best_k;
        memcpy(q_out + NQ * t, best_q, sizeof best_q);
        status_out[t] = best_c;
    }
    return RP_OK;
}
