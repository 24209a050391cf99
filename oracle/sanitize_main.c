/*
 * sanitize_main.c — host sanitizer driver of the CPU oracle (TEST INFRASTRUCTURE).
 *
 * Built with -fsanitize=address,undefined together with rbe_oracle.c (oracle/Makefile
 * target `asan`) and run by tests/test_oracle_sanitize.py. It drives every oracle
 * entry point the parity tests use — state and edge checks, contacts, single- and
 * two-rank plans (ranks as threads with a barrier all-gather), interpolate, IK — on
 * the scene in the input file, and cross-checks the batched calls against the
 * per-state ones, so an out-of-bounds access or undefined operation anywhere on
 * the checker's paths aborts the run.
 *
 * Input (binary, written by the test): rp_robot_desc; int32 n_boxes; rp_box[n_boxes];
 * int32 attached; double start[9], goal[9], lo[9], hi[9].
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rbe_oracle.h"

static int fail(const char* what) {
    fprintf(stderr, "sanitize_main: %s\n", what);
    return 1;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static double urand(void) {  /* xorshift64*: a fixed stream, test inputs only */
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (double)((rng_state * 0x2545F4914F6CDD1Dull) >> 11) * (1.0 / 9007199254740992.0);
}

typedef struct {
    const ro_scene* s;
    const double *start, *goal, *lo, *hi;
    rp_plan_params p;
    int rank;
    double path[4096 * RP_NQ];
    int32_t n, status;
    int rc;
} rank_job;

static pthread_barrier_t g_bar;
static unsigned char g_slots[2][1 << 20];

/* two ranks in one process: each writes its slot, the barrier orders the copies */
static int gather2(void* user, const void* send, void* recv, int64_t bytes) {
    const int rank = *(const int*)user;
    if (bytes > (int64_t)sizeof g_slots[0]) return 1;
    memcpy(g_slots[rank], send, (size_t)bytes);
    pthread_barrier_wait(&g_bar);
    memcpy(recv, g_slots[0], (size_t)bytes);
    memcpy((unsigned char*)recv + bytes, g_slots[1], (size_t)bytes);
    pthread_barrier_wait(&g_bar);
    return 0;
}

static void* run_rank(void* arg) {
    rank_job* j = (rank_job*)arg;
    rp_stats st;
    j->rc = ro_plan(j->s, j->start, j->goal, j->lo, j->hi, &j->p, j->rank, 2, gather2, &j->rank, j->path, 4096,
                    &j->n, &j->status, &st);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc != 2) return fail("usage: sanitize_main <input.bin>");
    FILE* f = fopen(argv[1], "rb");
    if (!f) return fail("cannot open input");
    rp_robot_desc desc;
    int32_t nb = 0, att = -1;
    rp_box boxes[RP_MAX_BOXES];
    double start[RP_NQ], goal[RP_NQ], lo[RP_NQ], hi[RP_NQ];
    int ok = fread(&desc, sizeof desc, 1, f) == 1 && fread(&nb, 4, 1, f) == 1 && nb >= 0 && nb <= RP_MAX_BOXES &&
             fread(boxes, sizeof(rp_box), (size_t)nb, f) == (size_t)nb && fread(&att, 4, 1, f) == 1 &&
             fread(start, 8, RP_NQ, f) == RP_NQ && fread(goal, 8, RP_NQ, f) == RP_NQ &&
             fread(lo, 8, RP_NQ, f) == RP_NQ && fread(hi, 8, RP_NQ, f) == RP_NQ;
    fclose(f);
    if (!ok) return fail("short input");

    ro_scene* s = ro_scene_create(&desc);
    if (!s) return fail("ro_scene_create");
    const float base[3] = {0.0f, 0.0f, 0.01f};
    if (ro_scene_set(s, boxes, nb, 0.0f, base) || ro_scene_set_attached(s, att, 0x700u)) return fail("scene");

    /* states: batched (2 threads) == one by one */
    enum { NS = 20000 };
    float* q = (float*)malloc(sizeof(float) * NS * RP_NQ);
    uint8_t* fl = (uint8_t*)malloc(NS);
    for (int i = 0; i < NS * RP_NQ; ++i) q[i] = (float)(lo[i % RP_NQ] + (hi[i % RP_NQ] - lo[i % RP_NQ]) * urand());
    if (ro_check_states(s, q, NS, fl, 2) != NS) return fail("ro_check_states count");
    int n_valid = 0;
    for (int i = 0; i < NS; ++i) {
        if (fl[i] != ro_state_valid(s, q + (size_t)i * RP_NQ)) return fail("batched flag != single flag");
        n_valid += fl[i];
    }
    float caps[RP_MAX_CAPSULES * 6];
    ro_fk_capsules(s, q, caps);

    /* contacts of a few invalid states */
    int32_t pairs[2 * 64];
    for (int i = 0, seen = 0; i < NS && seen < 50; ++i) {
        if (fl[i]) continue;
        double qd[RP_NQ];
        for (int k = 0; k < RP_NQ; ++k) qd[k] = q[(size_t)i * RP_NQ + k];
        if (ro_state_contacts(s, qd, pairs, 64) <= 0) return fail("invalid state without contacts");
        ++seen;
    }

    /* edges: batched == one by one */
    enum { NE = 400 };
    double* ea = (double*)malloc(sizeof(double) * NE * RP_NQ);
    double* eb = (double*)malloc(sizeof(double) * NE * RP_NQ);
    uint8_t eo[NE];
    for (int i = 0; i < NE * RP_NQ; ++i) {
        const int k = i % RP_NQ;
        ea[i] = lo[k] + (hi[k] - lo[k]) * urand();
        eb[i] = ea[i] + 0.3 * (urand() - 0.5);
        if (eb[i] < lo[k]) eb[i] = lo[k];
        if (eb[i] > hi[k]) eb[i] = hi[k];
    }
    ro_check_edges(s, ea, eb, NE, 0.13037, eo);
    for (int i = 0; i < NE; ++i) {
        int64_t cnt = 0;
        if (eo[i] != ro_check_edge(s, ea + (size_t)i * RP_NQ, eb + (size_t)i * RP_NQ, 0.13037, &cnt))
            return fail("batched edge != single edge");
    }

    /* plans: sequential (batch 1), batched, each simplification level */
    static double path[4096 * RP_NQ];
    int32_t n = 0, status = 0;
    rp_stats st;
    const int64_t batches[3] = {1, 256, 1024};
    for (int bi = 0; bi < 3; ++bi)
        for (int level = 0; level <= 2; ++level) {
            rp_plan_params p;
            memset(&p, 0, sizeof p);
            p.seed = 7 + (uint64_t)bi;
            p.batch = batches[bi];
            p.timeout_s = 30.0;
            p.n_waypoints = 150;
            p.simplify = level;
            p.straight_first = -1;
            if (ro_plan(s, start, goal, lo, hi, &p, 0, 1, NULL, NULL, path, 4096, &n, &status, &st))
                return fail("ro_plan");
            if (status != RP_STATUS_EXACT && status != RP_STATUS_APPROXIMATE) return fail("plan not solved");
            if (n != 150) return fail("plan waypoints != 150");
        }

    /* two ranks (threads) == one rank */
    rp_plan_params p2;
    memset(&p2, 0, sizeof p2);
    p2.seed = 11;
    p2.batch = 256;
    p2.timeout_s = 30.0;
    p2.n_waypoints = 150;
    p2.simplify = 1;
    p2.straight_first = -1;
    p2.max_iters = 64;
    if (ro_plan(s, start, goal, lo, hi, &p2, 0, 1, NULL, NULL, path, 4096, &n, &status, &st)) return fail("ro_plan w1");
    static rank_job jobs[2];
    pthread_barrier_init(&g_bar, NULL, 2);
    pthread_t th[2];
    for (int r = 0; r < 2; ++r) {
        jobs[r].s = s;
        jobs[r].start = start;
        jobs[r].goal = goal;
        jobs[r].lo = lo;
        jobs[r].hi = hi;
        jobs[r].p = p2;
        jobs[r].rank = r;
        pthread_create(&th[r], NULL, run_rank, &jobs[r]);
    }
    for (int r = 0; r < 2; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&g_bar);
    for (int r = 0; r < 2; ++r) {
        if (jobs[r].rc || jobs[r].status != status || jobs[r].n != n) return fail("two-rank plan differs");
        if (memcmp(jobs[r].path, path, sizeof(double) * (size_t)n * RP_NQ)) return fail("two-rank path differs");
    }

    /* interpolate */
    static double ip[1000 * RP_NQ];
    if (ro_interpolate(path, n, 600, ip, 1000) != 600) return fail("ro_interpolate");

    /* IK: hand poses of a few valid states as targets */
    enum { NT = 4 };
    double pos[NT * 3], quat[NT * 4], init[NT * RP_NQ], qo[NT * RP_NQ];
    int32_t ist[NT];
    for (int t = 0, i = 0; t < NT && i < NS; ++i) {
        if (!fl[i]) continue;
        double qd[RP_NQ], R[9], pp[3];
        for (int k = 0; k < RP_NQ; ++k) qd[k] = q[(size_t)i * RP_NQ + k];
        ro_hand_pose(s, qd, R, pp);
        const double w = 0.5 * sqrt(fmax(0.0, 1.0 + R[0] + R[4] + R[8]));
        if (w < 0.1) continue;
        memcpy(pos + 3 * t, pp, sizeof pp);
        quat[4 * t] = w;
        quat[4 * t + 1] = (R[7] - R[5]) / (4 * w);
        quat[4 * t + 2] = (R[2] - R[6]) / (4 * w);
        quat[4 * t + 3] = (R[3] - R[1]) / (4 * w);
        memcpy(init + RP_NQ * t, start, sizeof start);
        ++t;
    }
    rp_ik_params ikp;
    memset(&ikp, 0, sizeof ikp);
    ikp.seed = 3;
    ikp.n_seeds = 32;
    if (ro_ik(s, NT, pos, quat, init, lo, hi, &ikp, qo, ist)) return fail("ro_ik");
    double s64, c64;
    ro_sincos64(1.25, &s64, &c64);

    printf("sanitize ok: %d/%d valid states, %d edges, 9 plans + a two-rank plan (%d waypoints), IK status %d %d %d %d\n",
           n_valid, NS, NE, n, ist[0], ist[1], ist[2], ist[3]);
    free(q);
    free(fl);
    free(ea);
    free(eb);
    ro_scene_destroy(s);
    return 0;
}
