// rp_nn.h — nearest tree node for many queries on the matrix cores (gfx950 MFMA).
//
// RRTConnect's nearest-neighbour query (OMPL NearestNeighbors, code/planning.py:156,
// 190) over trees of 10^5 nodes is n x T squared distances, a distance matrix:
// |x - y|^2 = |x|^2 + |y|^2 - 2 x.y is a GEMM of the queries against the nodes plus
// rank-1 terms. Here v_mfma_f32_16x16x32_f16 computes, for a tile of 16 queries x 16
// nodes, the whole FILTER VALUE
//
//     Q = S^2 x~.y~  -  S^2 |y'|^2 / 2  +  S^2 (thr - |x'|^2) / 2      (x' = x - c)
//
// in ONE instruction: the K = 32 slots hold the 9 coordinates as f16 hi / lo parts
// (x_hi y_hi + x_lo y_hi + x_hi y_lo: 27 slots), the node's half norm as a hi / lo
// pair against -2^G, and the query's threshold term as a hi / lo pair against 2^H.
// Q >= 0 <=> (approximately) |x - y|^2 <= thr. The approximation error is bounded
// (DESIGN.md §5.2): every node whose exact f64 distance is <= the query's exact
// best so far has Q >= 0 when thr = best + e0 + e1 best, so the filter never drops a
// node that could be the answer. A node that passes gets the oracle's exact f64
// dist2 (same operands, same order) and the lexicographic (distance, index) update,
// so the result is bit for bit the linear strict-< scan's: the nearest node, lowest
// index among equal distances. Large trees only (rp_lib.hip nn_split): the ranges of
// the tree go to grid.y, k_nn_reduce merges them as for k_nn_part.
#pragma once
#include "rp_plan_math.h"

namespace rp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

// per-plan constants of the filter (host: nn_mfma_params in rp_lib.hip)
struct NnMfma {
    double c[NQ];   // centre of the bounds (coordinates x' = x - c, |x'| <= R0)
    double S;       // coordinate scale, a power of two (S R0 <= 16384: f16 range)
    double G2;      // 2^G: the node half-norm slots (A: -2^G, B: g / 2^G, hi / lo)
    double H2;      // 2^H: the threshold slots (A: h / 2^H, hi / lo; B: 2^H)
    double e0, e1;  // thr = best + e0 + e1 * best
    double thr0;    // threshold while a query has no exact best (every node passes)
    double iG2, iH2;   // 2^-G, 2^-H (exact: a product by them is the division by 2^G, 2^H)
};

// B fragments through a buffer descriptor (k_nn_mfma; 0: flat loads, A/B)
#ifndef RP_NN_BUF
#define RP_NN_BUF 1
#endif

// waves per block (template W): each with its own queries and tree stream
constexpr int NNM_SEEDS = 8;    // nodes per range evaluated exactly before the scan (threshold seeds)

// v = hi + lo to ~2^-22 |v|: through f32 (hardware conversions; an f64 -> f16
// conversion has no instruction and compiles to a ~60-instruction correctly rounded
// sequence): |v - vf| <= 2^-24 |v|, vf - hi is exact in f32, |vf - hi - lo| <= 2^-11
// |vf - hi| <= 2^-22 |vf| (or half an f16 subnormal step) — the representation error
// the filter's margin is sized for (rp_lib.hip nn_mfma_params)
__device__ __forceinline__ void split16(double v, _Float16& hi, _Float16& lo) {
    const float vf = (float)v;
    hi = (_Float16)vf;
    lo = (_Float16)(vf - (float)hi);
}

// rank of this lane among the set lanes of m (ballot + mbcnt)
__device__ __forceinline__ int rank_lanes(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// LDS ordering between the lanes of one wave (stores, then other lanes' loads)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// threshold slots (f16 hi / lo of h / 2^H) of a query with exact best b
__device__ __forceinline__ void thr_slots(const NnMfma& P, double b, double na, _Float16& hh, _Float16& hl) {
    const double thr = b < 1e300 ? b + (P.e0 + P.e1 * b) : P.thr0;
    split16((P.S * P.S) * (thr - na) * 0.5 * P.iH2, hh, hl);
}

// A fragment of a query (row), k chunk `ch` (lane >> 4) of 8 slots
__device__ __forceinline__ h8 a_frag(const NnMfma& P, const double* x, bool live, int ch, double* na_out,
                                     _Float16* hh_out, _Float16* hl_out) {
    _Float16 xh[NQ], xl[NQ];
    double na = 0.0;
#pragma unroll
    for (int d = 0; d < NQ; ++d) {
        const double xd = x[d] - P.c[d];
        na += xd * xd;
        split16(P.S * xd, xh[d], xl[d]);
    }
    _Float16 hh, hl;
    thr_slots(P, __builtin_inf(), na, hh, hl);
    const _Float16 z = (_Float16)0.0f, mg = (_Float16)(-P.G2);
    h8 a;
    if (!live) {   // no query: Q = -2^G |y'|^2 S^2 / 2 - 65504 * 2^H < 0 for every node (dead pads too)
        a = h8{z, z, z, z, z, z, z, z};
        if (ch == 3) {
            a[3] = mg;
            a[4] = mg;
            a[5] = (_Float16)(-65504.0f);
        }
    } else if (ch == 0) {
        a = h8{xh[0], xh[1], xh[2], xh[3], xh[4], xh[5], xh[6], xh[7]};
    } else if (ch == 1) {
        a = h8{xh[8], xl[0], xl[1], xl[2], xl[3], xl[4], xl[5], xl[6]};
    } else if (ch == 2) {
        a = h8{xl[7], xl[8], xh[0], xh[1], xh[2], xh[3], xh[4], xh[5]};
    } else {
        a = h8{xh[6], xh[7], xh[8], mg, mg, hh, hl, z};
    }
    *na_out = na;
    *hh_out = hh;
    *hl_out = hl;
    return a;
}

// B image chunk of a node: its 8 slots of k chunk `ch`
__device__ __forceinline__ h8 b_frag(const NnMfma& P, const double* y, int ch) {
    _Float16 yh[NQ], yl[NQ];
    double nb = 0.0;
#pragma unroll
    for (int d = 0; d < NQ; ++d) {
        const double yd = y[d] - P.c[d];
        nb += yd * yd;
        split16(P.S * yd, yh[d], yl[d]);
    }
    _Float16 gh, gl;
    split16((P.S * P.S) * nb * 0.5 * P.iG2, gh, gl);
    const _Float16 z = (_Float16)0.0f, h2 = (_Float16)P.H2;
    if (ch == 0) return h8{yh[0], yh[1], yh[2], yh[3], yh[4], yh[5], yh[6], yh[7]};
    if (ch == 1) return h8{yh[8], yh[0], yh[1], yh[2], yh[3], yh[4], yh[5], yh[6]};
    if (ch == 2) return h8{yh[7], yh[8], yl[0], yl[1], yl[2], yl[3], yl[4], yl[5]};
    return h8{yl[6], yl[7], yl[8], gh, gl, h2, h2, z};
}

// B operand images of tree nodes [t0, t1): img[node][32] f16 (64 B), made once per
// node and plan (the searches read them; rp_lib.hip keeps a per-tree count). The
// slots [t1, round_up(t1, NNM_PAD)) get a dead image that no query passes (norm slots
// 65504 against -2^G, no threshold slots: Q = -2^(G+1) 65504 < 0), so the search's
// tiles need no bounds test; the buffer holds NNM_PAD spare nodes.
constexpr int NNM_PAD = 64;
__global__ void k_nn_image(const double* __restrict__ tree, int64_t t0, int64_t t1, NnMfma P, h8* __restrict__ img) {
    const int64_t i = (int64_t)rp_bid() * rp_bdim() + rp_tid();
    const int64_t node = t0 + (i >> 2);
    const int ch = (int)(i & 3);
    const int64_t tpad = (t1 + NNM_PAD - 1) / NNM_PAD * NNM_PAD;
    if (node >= tpad) return;
    if (node >= t1) {
        const _Float16 z = (_Float16)0.0f, big = (_Float16)65504.0f;
        img[node * 4 + ch] = ch == 3 ? h8{z, z, z, big, big, z, z, z} : h8{z, z, z, z, z, z, z, z};
        return;
    }
    double y[NQ];
#pragma unroll
    for (int d = 0; d < NQ; ++d) y[d] = tree[node * NQ + d];
    img[node * 4 + ch] = b_frag(P, y, ch);
}

// Nearest node of each query over tree range [y * chunk, (y + 1) * chunk) ->
// part[y * n + q] (exact distance, index; index -1: no node). Queries: qx (n x 9
// f64); status (NNQ_ROWS): n = min(n, status[0] - t0), and with devgeom the
// geometry (qblocks, chunk, ranges) is nn_geom's for that n within the grid (the
// host's chunk / qblocks are ignored; devgeom bit 1: nn_geom's fit off). RB row
// blocks of 16 queries per wave.
// Grid: 1-D, qblocks x (tree ranges) blocks. Blocks are remapped so that each group
// of blocks sharing an XCD (blockIdx % 8 labels them, cdna_hip_programming.md T1,
// the bijective form) takes a contiguous run of (range, query block) pairs: the
// blocks of one tree range sit on one XCD and its L2 holds that range (the tree's
// 72 B/node are re-read by every query block).
// nwg: the blocks in use (the first nwg of the grid; the rest return)
__device__ __forceinline__ void nn_block_coords(int64_t qblocks, int64_t nwg, int64_t* qb, int64_t* y) {
    const int64_t lid = (int64_t)rp_bid();
    const int64_t q = nwg / 8, r = nwg % 8, xcd = lid % 8;
    const int64_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + lid / 8;
    *y = wgid / qblocks;
    *qb = wgid - *y * qblocks;
}
__device__ __forceinline__ void nn_block_coords(int64_t qblocks, int64_t* qb, int64_t* y) {
    nn_block_coords(qblocks, (int64_t)rp_gdim(), qb, y);
}

// Geometry of a split search: n queries in blocks of per_block, the T nodes in S
// ranges of `chunk` (a multiple of 64, >= 32 x 64 = 2,048 nodes: a range's first
// stages hold most of its threshold updates, which a longer range amortises), about
// >= 1,024 blocks in all; maxblocks > 0 caps qblocks x S. A search whose query count
// is on the device (NNQ_ROWS: the accepted extensions) has its grid sized on the host
// for the largest count and takes the geometry of the actual count in the kernel, so
// a few thousand queries against a large tree still get ~1,024 blocks (the host
// geometry of the largest count would give them qblocks_max x 2 blocks, most idle).
struct NnGeom {
    int64_t qblocks, chunk;
    int S;
};
// fit: the ranges per query block are rounded DOWN, so qblocks x S stays within
// `target` (the blocks resident at once: 1,024 = 256 CUs x 4 one-wave-per-SIMD blocks
// at 4 waves per SIMD) whenever qblocks <= target. Rounded up (fit = false, round 5's
// geometry) a 98,304-query search took 192 x 6 = 1,152 blocks: a second round of 128
// blocks after the first 1,024.
__host__ __device__ inline NnGeom nn_geom(int64_t n, int64_t T, int64_t per_block, int64_t maxblocks,
                                          int64_t target = 1024, bool fit = true) {
    NnGeom g;
    g.qblocks = (n + per_block - 1) / per_block;
    const int64_t qb = g.qblocks > 0 ? g.qblocks : 1;
    const int64_t stages = (T + 63) / 64;
    int64_t S0 = fit ? target / qb : (target + qb - 1) / qb;
    if (S0 > stages / 32) S0 = stages / 32;
    if (maxblocks > 0 && S0 > maxblocks / qb) S0 = maxblocks / qb;
    if (S0 < 1) S0 = 1;
    g.chunk = ((stages + S0 - 1) / S0) * 64;
    g.S = (int)((T + g.chunk - 1) / g.chunk);
    return g;
}

#ifdef RP_NN_COUNT
// diagnostic builds: [0] column tiles scanned (per wave), [1] tiles that took the
// exact path, [2] exact-path rounds, [3] passing (row, node) elements
__device__ unsigned long long g_nncount[4];
#define RP_NNC(i, v) do { if (lane == 0) atomicAdd(&g_nncount[i], (unsigned long long)(v)); } while (0)
#else
#define RP_NNC(i, v) do { } while (0)
#endif

// Exact path: the (row, node) pairs that pass the filter are
// appended to a per-wave LDS list (a ballot and a prefix count per round, no
// barrier); the list is evaluated 64 pairs at a time (one per lane: the exact f64
// distance and the lexicographic (distance, index) update of the row, three wave
// LDS syncs per 64 pairs) when it holds NNM_FLUSH pairs and at the end of the range,
// and only then are the rows' threshold slots tightened. The deferred tightening
// lets a few more nodes through; the result does not depend on the order in which
// a row's candidates are evaluated (the range's lexicographic minimum).
#ifndef RP_NNM_FLUSH
#define RP_NNM_FLUSH 64
#endif
constexpr int NNM_FLUSH = RP_NNM_FLUSH;
constexpr int NNM_CAND = NNM_FLUSH + 64;   // a round appends at most one pair per lane

// (4 waves per SIMD at every RB: the register budget of 128 VGPRs)
template <int RB, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4))) void k_nn_mfma(const double* __restrict__ qx, int64_t n,
                                                          const int* status, int64_t t0,
                                                          const double* __restrict__ tree, const h8* __restrict__ img,
                                                          int64_t T, int64_t chunk, int64_t qblocks, NnMfma P,
                                                          DI2* __restrict__ part, int devgeom, int tstride,
                                                          const DI2* __restrict__ init, int init_S,
                                                          const int* __restrict__ gate,
                                                          unsigned long long* __restrict__ gbest) {
    constexpr int QW = 16 * RB;   // queries per wave
    // gate: a pipelined sub-batch's search (rp_lib.hip plan_impl) does nothing once the
    // previous sub-batch's first REACHED word is set (its result is then never read)
    if (gate && *gate != 0x7fffffff) return;
    __shared__ unsigned long long s_best[W][QW];            // exact best distance (f64 bits; >= 0)
    __shared__ int s_bi[W][QW];                             // its node (lowest index among equal)
    __shared__ int s_ti[W][QW];                             // a round's lowest node at the new best
    __shared__ int2 s_cand[W][NNM_CAND];                    // passing (row, node) pairs, not yet evaluated
    __shared__ double s_na[W][QW];                          // |x'|^2 of each row (threshold slots)
    __shared__ unsigned long long s_gb[W][QW];              // the query's bound over every range (gbest)
    int64_t nwg = (int64_t)rp_gdim();
    if (status) {
        n = min(n, (int64_t)status[0] - t0);
        if (n <= 0) return;
        if (devgeom) {
            const NnGeom g = nn_geom(n, T, (int64_t)W * QW, nwg, 1024, (devgeom & 2) == 0);
            qblocks = g.qblocks;
            chunk = g.chunk;
            nwg = g.qblocks * g.S;
            if ((int64_t)rp_bid() >= nwg) return;
        }
    }
    int64_t qb, yr;
    nn_block_coords(qblocks, nwg, &qb, &yr);
    const int64_t qb0 = qb * W * QW;
    if (qb0 >= n) return;   // whole block idle (uniform)
    // (w wave-uniform in an SGPR: the per-wave LDS bases need no VGPRs)
    const int w = __builtin_amdgcn_readfirstlane((int)(rp_tid() >> 6)), lane = (int)(rp_tid() & 63), ch = lane >> 4;
    const int64_t t_lo = yr * chunk, t_hi = min(T, t_lo + chunk);
    const int64_t qw0 = qb0 + (int64_t)w * QW;
    // a row's query state, read from global memory (L1 / L2) where the exact path needs
    // it: staging the wave's 64 states in LDS cost more than it saved (rows past n
    // read the last query; their results are never written)
    auto qrow = [&](int r) -> const double* { return qx + min<int64_t>(qw0 + r, n - 1) * NQ; };
    // seed every query's exact best with NNM_SEEDS nodes spread over the range (the
    // exact f64 distance, lexicographic (distance, index) minimum): the filter then
    // starts from a typical distance instead of letting every node of the first stage
    // through to the exact path. Order does not matter: the result is the range's
    // lexicographic minimum whatever order its nodes are evaluated in.
    // With a pilot (init: each query's nearest node over a strided subset of the whole
    // tree, an upper bound d1 on its answer), every range starts from d1 instead and
    // no node yet (index sentinel INT_MAX): the range returns its lexicographic minimum
    // over the nodes at distance <= d1, or none — the pilot's node itself is in some
    // range and passes the filter there (distance d1 <= the threshold), so the minimum
    // over the ranges is the answer.
    for (int r = lane; r < QW; r += 64) {
        unsigned long long bb = 0x7FF0000000000000ull;   // +inf
        int bi = -1;
        if (init && qw0 + r < n) {   // (the pilot's ranges: their minimum distance)
            for (int y = 0; y < init_S; ++y) {
                const DI2 v = init[(int64_t)y * n + qw0 + r];
                const unsigned long long db = (unsigned long long)__double_as_longlong(v.d);
                if (v.i >= 0 && db < bb) {
                    bb = db;
                    bi = 0x7fffffff;
                }
            }
        }
        if (bi < 0 && qw0 + r < n) {
            const int64_t R = t_hi - t_lo;
#pragma unroll 1
            for (int k = 0; k < NNM_SEEDS; ++k) {
                const int64_t j = t_lo + (R * k) / NNM_SEEDS;
                if (k > 0 && j == t_lo + (R * (k - 1)) / NNM_SEEDS) continue;
                const unsigned long long db =
                    (unsigned long long)__double_as_longlong(dist2(tree + j * NQ, qrow(r)));
                if (db < bb || (db == bb && (int)j < bi)) {
                    bb = db;
                    bi = (int)j;
                }
            }
        }
        s_best[w][r] = bb;
        s_bi[w][r] = bi;
        s_gb[w][r] = bb;
    }
    wave_lds_sync();
    // A fragments (row lane & 15 of each row block; k chunk ch); the threshold slots
    // (chunk 3, elements 5 / 6) follow each row's exact best. The rows' |x'|^2 wait in
    // LDS for the threshold updates (registers: RB = 8 fits 4 waves per SIMD)
    h8 a[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int r = rb * 16 + (lane & 15);
        _Float16 hh, hl;
        double na;
        a[rb] = a_frag(P, qrow(r), qw0 + r < n, ch, &na, &hh, &hl);
        if (ch == 0) s_na[w][r] = na;
        const double b0 = __longlong_as_double((long long)s_best[w][r]);
        if (ch == 3 && qw0 + r < n && b0 < 1e300) {   // the seeded threshold
            thr_slots(P, b0, na, hh, hl);
            a[rb][5] = hh;
            a[rb][6] = hl;
        }
    }
    wave_lds_sync();
    int ncand = 0;   // wave-uniform
    // evaluate the listed pairs, then tighten the rows' threshold slots
    auto flush = [&]() {
        wave_lds_sync();   // the list's writes
        for (int b0 = 0; b0 < ncand; b0 += 64) {
            RP_NNC(2, 1);
            const int k = b0 + lane;
            const bool has = k < ncand;
            int row = 0, node = 0;
            unsigned long long prev = 0, db = 0;
            if (has) {
                const int2 cnd = s_cand[w][k];
                row = cnd.x;
                node = cnd.y;
                prev = s_best[w][row];
                s_ti[w][row] = 0x7fffffff;
                db = (unsigned long long)__double_as_longlong(dist2(tree + (int64_t)node * NQ, qrow(row)));
            }
            wave_lds_sync();
            if (has) atomicMin(&s_best[w][row], db);
            wave_lds_sync();
            const unsigned long long cur = has ? s_best[w][row] : 0ull;
            if (has && db == cur) atomicMin(&s_ti[w][row], node);
            wave_lds_sync();
            if (has && db == cur && s_ti[w][row] == node) {   // the row's lowest node at its new best
                if (cur < prev) s_bi[w][row] = node;
                else if (node < s_bi[w][row]) s_bi[w][row] = node;
            }
            wave_lds_sync();
        }
        ncand = 0;
        if (gbest) {
            // the ranges of a query run at once in other blocks: each publishes its
            // exact best (atomicMin on the f64 bits, non-negative: ordered as integers)
            // and takes the minimum over all of them so far as its filter bound. Only
            // the threshold follows it: s_best / s_bi stay this range's own exactly
            // evaluated minimum, and any node at distance <= the final answer still
            // passes (the bound is >= the answer), so the reduce over the ranges is
            // unchanged
            for (int r = lane; r < QW; r += 64) {
                const unsigned long long mine = s_best[w][r];
                const unsigned long long old = qw0 + r < n ? atomicMin(gbest + qw0 + r, mine) : mine;
                s_gb[w][r] = old < mine ? old : mine;
            }
            wave_lds_sync();
        }
        if (ch == 3) {   // (the same slots again where a row's best did not move)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                const int r = rb * 16 + (lane & 15);
                // (s_gb <= s_best once shared: one word per row, as without sharing)
                const double bnow = __longlong_as_double((long long)(gbest ? s_gb[w][r] : s_best[w][r]));
                if (bnow < 1e300) {
                    _Float16 hh, hl;
                    thr_slots(P, bnow, s_na[w][r], hh, hl);
                    a[rb][5] = hh;
                    a[rb][6] = hl;
                }
            }
        }
    };
    // Each wave streams its range's node images itself, B fragments straight from
    // global memory (L2: the XCD-grouped blocks of a range read the same lines),
    // PF column tiles ahead: every load lands in a fixed register that the MFMAs of
    // its tile read PF tiles later (no register rotation, which made the compiler
    // wait for each tile's freshly issued load), and loads past the range re-read its
    // last tile (unconditional: static vmcnt waits). Tiles need no bounds test: the
    // image's pad slots and dead query rows never pass (k_nn_image, a_frag).
    // (3 tiles ahead — RB 8 with 4 held 3 VGPRs over the 128 of 4 waves per SIMD in
    // scratch, RB 4 with 4 and the shared bounds 5; tests/test_isa_guard.py)
#ifndef RP_NN_PF8
#define RP_NN_PF8 3
#endif
    constexpr int PF = RB >= 8 ? RP_NN_PF8 : 3;
    // tiles of the range: every tstride-th (a pilot search), else all
    const int64_t ntiles = ((t_hi - t_lo + 15) / 16 + tstride - 1) / tstride;
    const int col = lane & 15;   // this lane's column of every tile
    // tile t: the wave-uniform base + t x tstride KiB plus this lane's 16-byte slot
    const uint32_t loff = (uint32_t)((col * 4 + ch) * 16);
    const int64_t tbytes = (int64_t)tstride * 1024, tnodes = (int64_t)tstride * 16;
#if RP_NN_BUF
    // through a buffer descriptor of the range's images: the tile's byte offset in an
    // SGPR (soffset), the lane's slot in voffset, so a tile costs no VALU address
    // arithmetic (the flat form kept a 64-bit base + slot pair and paid a 64-bit
    // multiply-add per tile on the vector pipe, whose issue the MFMAs already crowd).
    // Every load is inside the descriptor (tiles past the range re-read its last one).
    const uint64_t ubv = (uint64_t)(img + t_lo * 4);
    const uint32_t ub_lo = __builtin_amdgcn_readfirstlane((uint32_t)ubv);
    const uint32_t ub_hi = __builtin_amdgcn_readfirstlane((uint32_t)(ubv >> 32));
    const int nbytes = (int)__builtin_amdgcn_readfirstlane((uint32_t)(ntiles * tbytes));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(((uint64_t)ub_hi << 32) | ub_lo), (short)0, nbytes, 0x00020000);
    auto tile_b = [&](int64_t t) {
        const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(t * tbytes));
        return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rs, loff, so, 0));
    };
#else
    const char* ub = (const char*)(img + t_lo * 4);
    auto tile_b = [&](int64_t t) { return *(const h8*)(ub + t * tbytes + loff); };
#endif
    h8 bq[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) bq[u] = tile_b(min<int64_t>(u, ntiles - 1));
    const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    auto tile_step = [&](int64_t tile, const h8& b) {
        f4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rb], b, zero, 0, 0, 0);
        // this lane's column: acc[rb][e] = row rb * 16 + 4 ch + e; mr[rb]: its max
        float mr[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) mr[rb] = fmaxf(fmaxf(acc[rb][0], acc[rb][1]), fmaxf(acc[rb][2], acc[rb][3]));
        float m = mr[0];
#pragma unroll
        for (int rb = 1; rb < RB; ++rb) m = fmaxf(m, mr[rb]);
        RP_NNC(0, 1);
        if (!__any(m >= 0.0f)) return;
        RP_NNC(1, 1);
        // the passing elements as a bit mask (bit rb * 4 + e), built only for the row
        // blocks with any; then appended one per lane and round
        unsigned pm = 0;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
            if (__any(mr[rb] >= 0.0f)) {
#pragma unroll
                for (int e = 0; e < 4; ++e) pm |= (acc[rb][e] >= 0.0f ? 1u : 0u) << (rb * 4 + e);
            }
        const int node = (int)(t_lo + tile * tnodes + col);
#ifdef RP_NN_COUNT
        {
            unsigned tot = __popc(pm);
            for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
            RP_NNC(3, tot);
        }
#endif
        while (__any(pm != 0)) {
            const bool has = pm != 0;
            const int e = has ? __builtin_ctz(pm) : 0;
            pm &= pm - 1;
            const unsigned long long bm = __ballot(has);
            if (has) s_cand[w][ncand + rank_lanes(bm)] = int2{(e >> 2) * 16 + ch * 4 + (e & 3), node};
            ncand += __popcll(bm);
            if (ncand >= NNM_FLUSH) flush();
        }
    };
    int64_t tb = 0;
    for (; tb + 2 * PF <= ntiles; tb += PF) {   // (every prefetch in range)
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            bq[u] = tile_b(tb + PF + u);
        }
    }
    for (; tb + PF <= ntiles; tb += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            bq[u] = tile_b(min<int64_t>(tb + u + PF, ntiles - 1));
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (tb + u < ntiles) tile_step(tb + u, bq[u]);
    if (ncand > 0) flush();
    wave_lds_sync();
    // the lane id recomputed (mbcnt) rather than kept live across the scan: at RB 8 the
    // values the results' addresses derive from were held in scratch (2 dwords)
    const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    for (int r = ln; r < QW; r += 64) {
        const int64_t q = qw0 + r;
        if (q < n)
            part[yr * n + q] = DI2{__longlong_as_double((long long)s_best[w][r]),
                                   s_bi[w][r] == 0x7fffffff ? -1 : s_bi[w][r], 0};
    }
}

// k_nn_reduce of a k_nn_mfma search: with devgeom and a status-bounded count, the
// ranges are nn_geom's for the actual count (per_block queries per block, the grid's
// maxblocks), else the host's S
__global__ void k_nn_reduce_g(const DI2* __restrict__ part, int64_t n, int S, const int* status, int64_t t0,
                              int32_t* __restrict__ out, int64_t T, int64_t per_block, int64_t maxblocks,
                              int devgeom) {
    const int64_t k = (int64_t)rp_bid() * rp_bdim() + rp_tid();
    if (status) {
        n = min(n, (int64_t)status[0] - t0);
        if (devgeom && n > 0) S = nn_geom(n, T, per_block, maxblocks, 1024, (devgeom & 2) == 0).S;
    }
    if (k >= n) return;
    double bd = __builtin_inf();
    int bi = -1;
    for (int s = 0; s < S; ++s) {
        const DI2 v = part[(int64_t)s * n + k];
        if (v.i >= 0 && (v.d < bd || (v.d == bd && v.i < bi))) { bd = v.d; bi = v.i; }
    }
    out[k] = bi;
}

// the queries of a split search as f64 states (NNQ_SAMPLE / NNQ_STEER: Philox samples,
// steered; nn_query of rp_kernels.h)
// gbest (the ranges' shared bounds, k_nn_mfma): reset to +inf here, in the launch every
// sample / steer search makes right before its ranges run (no memset launch)
__global__ void k_nn_queries(NnQuery Q, int64_t n, double* __restrict__ qx,
                             unsigned long long* __restrict__ gbest) {
    const int64_t k = (int64_t)rp_bid() * rp_bdim() + rp_tid();
    if (k >= n) return;
    if (gbest) gbest[k] = ~0ull;
    double x[NQ];
    nn_query(Q, k, x);
#pragma unroll
    for (int d = 0; d < NQ; ++d) qx[k * NQ + d] = x[d];
}

}  // namespace rp
