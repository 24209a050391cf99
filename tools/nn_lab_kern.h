// nn_lab_kern.h — experimental variants of rp_nn.h k_nn_mfma for tools/nn_lab.hip
// (diagnostic; not the product). k_nnv<RB, W, V, PF>: V = 0 the product's code, V = 1
// the fast path only (no exact path: wrong answers, a speed bound), V = 3 the fast
// path on the same B fragments over and over (no loads: the MFMA + VALU bound); PF
// tiles prefetched.
#pragma once
namespace rp {
template <int RB, int W, int V, int PF = 4, bool GQ = false, int WPE = 1>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void k_nnv(const double* __restrict__ qx, int64_t n,
                                                          const int* status, int64_t t0,
                                                          const double* __restrict__ tree, const h8* __restrict__ img,
                                                          int64_t T, int64_t chunk, int64_t qblocks, NnMfma P,
                                                          DI2* __restrict__ part) {
    constexpr int QW = 16 * RB;   // queries per wave
    __shared__ double s_q[GQ ? 1 : W][GQ ? 1 : QW][NQ];     // query states (exact path; GQ: from global)
    __shared__ unsigned long long s_best[W][QW];            // exact best distance (f64 bits; >= 0)
    __shared__ int s_bi[W][QW];                             // its node (lowest index among equal)
    __shared__ int s_ti[W][QW];                             // a round's lowest node at the new best
    __shared__ int2 s_cand[W][NNM_CAND];                    // passing (row, node) pairs, not yet evaluated
    if (status) n = min(n, (int64_t)status[0] - t0);
    int64_t qb, yr;
    nn_block_coords(qblocks, &qb, &yr);
    const int64_t qb0 = qb * W * QW;
    if (qb0 >= n) return;   // whole block idle (uniform)
    const int w = (int)(rp_tid() >> 6), lane = (int)(rp_tid() & 63), ch = lane >> 4;
    const int64_t t_lo = yr * chunk, t_hi = min(T, t_lo + chunk);
    const int64_t qw0 = qb0 + (int64_t)w * QW;

    auto qrow = [&](int r) -> const double* {
        if constexpr (GQ) return qx + min<int64_t>(qw0 + r, n - 1) * NQ;
        else return &s_q[w][r][0];
    };
    if constexpr (!GQ) {
        for (int i = lane; i < QW * NQ; i += 64) {
            const int r = i / NQ, d = i - r * NQ;
            const int64_t q = qw0 + r;
            s_q[w][r][d] = q < n ? qx[q * NQ + d] : 0.0;
        }
        wave_lds_sync();
    }
    // seed every query's exact best with NNM_SEEDS nodes spread over the range (the
    // exact f64 distance, lexicographic (distance, index) minimum): the filter then
    // starts from a typical distance instead of letting every node of the first stage
    // through to the exact path. Order does not matter: the result is the range's
    // lexicographic minimum whatever order its nodes are evaluated in.
    for (int r = lane; r < QW; r += 64) {
        unsigned long long bb = 0x7FF0000000000000ull;   // +inf
        int bi = -1;
        if (qw0 + r < n) {
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
    }
    wave_lds_sync();
    // A fragments (row lane & 15 of each row block; k chunk ch); the threshold slots
    // (chunk 3, elements 5 / 6) follow each row's exact best
    h8 a[RB];
    double na[RB], curb[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int r = rb * 16 + (lane & 15);
        _Float16 hh, hl;
        a[rb] = a_frag(P, qrow(r), qw0 + r < n, ch, &na[rb], &hh, &hl);
        curb[rb] = __builtin_inf();
        const double b0 = __longlong_as_double((long long)s_best[w][r]);
        if (ch == 3 && qw0 + r < n && b0 < 1e300) {   // the seeded threshold
            curb[rb] = b0;
            thr_slots(P, b0, na[rb], hh, hl);
            a[rb][5] = hh;
            a[rb][6] = hl;
        }
    }
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
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int r = rb * 16 + (lane & 15);
            const double bnow = __longlong_as_double((long long)s_best[w][r]);
            if (ch == 3 && bnow != curb[rb]) {
                curb[rb] = bnow;
                _Float16 hh, hl;
                thr_slots(P, bnow, na[rb], hh, hl);
                a[rb][5] = hh;
                a[rb][6] = hl;
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
    const int64_t ntiles = (t_hi - t_lo + 15) / 16;
    const int col = lane & 15;   // this lane's column of every tile
    const h8* ib = img + (t_lo + col) * 4 + ch;   // tile t: ib[t * 64]
    h8 bq[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) bq[u] = ib[min<int64_t>(u, ntiles - 1) * 64];
    const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    float sink = -1e30f;
    auto tile_step = [&](int64_t tile, const h8& b) {
        f4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rb], b, zero, 0, 0, 0);
        // this lane's column: acc[rb][e] = row rb * 16 + 4 ch + e
        float m = fmaxf(fmaxf(acc[0][0], acc[0][1]), fmaxf(acc[0][2], acc[0][3]));
#pragma unroll
        for (int rb = 1; rb < RB; ++rb) m = fmaxf(m, fmaxf(fmaxf(acc[rb][0], acc[rb][1]), fmaxf(acc[rb][2], acc[rb][3])));
        RP_NNC(0, 1);
        if constexpr (V == 1 || V == 3) {   // (the max feeds an output, so the MFMAs stay)
            sink = fmaxf(sink, m);
            return;
        }
        if (!__any(m >= 0.0f)) return;
        RP_NNC(1, 1);
        unsigned pm = 0;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int e = 0; e < 4; ++e) pm |= (acc[rb][e] >= 0.0f ? 1u : 0u) << (rb * 4 + e);
        const int node = (int)(t_lo + tile * 16 + col);
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
    const h8* nx = ib + PF * 64;   // the next group's first tile
    for (; tb + 2 * PF <= ntiles; tb += PF, nx += PF * 64) {   // (every prefetch in range)
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            if constexpr (V == 3) asm volatile("" : "+v"(bq[u]));
            else bq[u] = nx[u * 64];
        }
    }
    for (; tb + PF <= ntiles; tb += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            bq[u] = ib[min<int64_t>(tb + u + PF, ntiles - 1) * 64];
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (tb + u < ntiles) tile_step(tb + u, bq[u]);
    if (ncand > 0) flush();
    wave_lds_sync();
    for (int r = lane; r < QW; r += 64) {
        const int64_t q = qw0 + r;
        if (q < n)
            part[yr * n + q] =
                DI2{__longlong_as_double((long long)s_best[w][r]), s_bi[w][r], V != 0 ? (int)(sink > 0.0f) : 0};
    }
}



// ---------------------------------------------------------------------------
// V2: approximate tightening, deferred exact evaluation.
// A passing (row, node) element's filter value Q gives the node's distance to
// within eps: d~2 = thr_r - 2 Q / S^2, |d~2 - d2| <= eps_r = 2e-5 R0^2 + 3e-6 thr_r
// (the filter's error bound E(thr) <= 1.8e-5 R0^2 + 2.3e-6 thr plus the f32
// rounding of thr_r and of d~2). So u = d~2 + eps >= d2 >= the range's exact best:
// U[r] = min u is an upper bound on it, and the row's threshold follows U
// (thr = U + e0 + e1 U: every node with d2 <= best <= U still passes). Every
// node that could be the answer (d2 <= best_final <= U_final) passed the filter at
// its tile (U only decreases) and has l = d~2 - eps <= d2 <= U_final: candidates
// with l > U_final are dropped, the rest (a few per row) get the oracle's exact f64
// dist2 and the lexicographic (distance, index) update at the range's end. No
// global load, f64 arithmetic or LDS atomic chain per candidate inside the scan.
constexpr int NNC2 = 256;   // candidate list per wave

__device__ __forceinline__ float f32_up(double b) {   // smallest float >= b (b >= 0)
    float f = (float)b;
    if ((double)f < b) f = __uint_as_float(__float_as_uint(f) + 1u);   // (b >= 0, finite)
    return f;
}

template <int RB, int W, int REFRESH>
__global__ __launch_bounds__(64 * W) void k_nnv2(const double* __restrict__ qx, int64_t n, const int* status,
                                                 int64_t t0, const double* __restrict__ tree,
                                                 const h8* __restrict__ img, int64_t T, int64_t chunk,
                                                 int64_t qblocks, NnMfma P, DI2* __restrict__ part) {
    constexpr int QW = 16 * RB;
    __shared__ double s_q[W][QW][NQ];
    __shared__ unsigned long long s_best[W][QW];   // exact best (f64 bits) of the evaluated nodes
    __shared__ int s_bi[W][QW];
    __shared__ int s_ti[W][QW];
    __shared__ unsigned s_U[W][QW];                // upper bound on the range's best (f32 bits, >= 0)
    __shared__ float s_thr[W][QW];                 // the threshold the row's slots encode
    __shared__ unsigned s_cn[W][NNC2];             // candidate: node | row << 24
    __shared__ float s_cl[W][NNC2];                // its lower bound l on d2
    if (status) n = min(n, (int64_t)status[0] - t0);
    int64_t qb, yr;
    nn_block_coords(qblocks, &qb, &yr);
    const int64_t qb0 = qb * W * QW;
    if (qb0 >= n) return;
    const int w = (int)(rp_tid() >> 6), lane = (int)(rp_tid() & 63), ch = lane >> 4;
    const int64_t t_lo = yr * chunk, t_hi = min(T, t_lo + chunk);
    const int64_t qw0 = qb0 + (int64_t)w * QW;
    const double R02 = (P.thr0 - P.e0) / 4.04;   // R0^2 (nn_mfma_params: thr0 = 4.04 R0^2 + e0)
    const float eps0 = (float)(2e-5 * R02), eps1 = 3e-6f;
    const float kq = (float)(2.0 / (P.S * P.S));  // exact (S a power of two)

    for (int i = lane; i < QW * NQ; i += 64) {
        const int r = i / NQ, d = i - r * NQ;
        const int64_t q = qw0 + r;
        s_q[w][r][d] = q < n ? qx[q * NQ + d] : 0.0;
    }
    wave_lds_sync();
    for (int r = lane; r < QW; r += 64) {
        unsigned long long bb = 0x7FF0000000000000ull;
        int bi = -1;
        if (qw0 + r < n) {
            const int64_t R = t_hi - t_lo;
#pragma unroll 1
            for (int k = 0; k < NNM_SEEDS; ++k) {
                const int64_t j = t_lo + (R * k) / NNM_SEEDS;
                if (k > 0 && j == t_lo + (R * (k - 1)) / NNM_SEEDS) continue;
                const unsigned long long db =
                    (unsigned long long)__double_as_longlong(dist2(tree + j * NQ, &s_q[w][r][0]));
                if (db < bb || (db == bb && (int)j < bi)) {
                    bb = db;
                    bi = (int)j;
                }
            }
        }
        s_best[w][r] = bb;
        s_bi[w][r] = bi;
        const double b = __longlong_as_double((long long)bb);
        s_U[w][r] = __float_as_uint(b < 1e300 ? f32_up(b) : __builtin_inff());
    }
    wave_lds_sync();
    h8 a[RB];
    double na[RB];
    unsigned curU[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int r = rb * 16 + (lane & 15);
        _Float16 hh, hl;
        a[rb] = a_frag(P, &s_q[w][r][0], qw0 + r < n, ch, &na[rb], &hh, &hl);
        curU[rb] = s_U[w][r];
        const float U = __uint_as_float(curU[rb]);
        const double thr = U < 1e30f ? (double)U + (P.e0 + P.e1 * (double)U) : P.thr0;
        if (ch == 3) {
            thr_slots(P, U < 1e30f ? (double)U : 1e301, na[rb], hh, hl);
            if (qw0 + r < n) {
                a[rb][5] = hh;
                a[rb][6] = hl;
            }
            s_thr[w][r] = (float)thr;
        }
    }
    wave_lds_sync();
    int ncand = 0, pend = 0;   // wave-uniform
    // drop the candidates whose lower bound exceeds their row's U (in place)
    auto prune = [&]() {
        wave_lds_sync();
        int kept = 0;
        for (int b0 = 0; b0 < ncand; b0 += 64) {
            const int k = b0 + lane;
            unsigned cn = 0;
            float cl = 0.0f;
            bool keep = false;
            if (k < ncand) {
                cn = s_cn[w][k];
                cl = s_cl[w][k];
                keep = cl <= __uint_as_float(s_U[w][cn >> 24]);
            }
            const unsigned long long bm = __ballot(keep);
            wave_lds_sync();
            if (keep) {
                const int dst = kept + rank_lanes(bm);
                s_cn[w][dst] = cn;
                s_cl[w][dst] = cl;
            }
            kept += __popcll(bm);
            wave_lds_sync();
        }
        ncand = kept;
    };
    // exact f64 evaluation of the listed candidates (the oracle's dist2, lexicographic
    // (distance, index) update of the row), then U = the exact best rounded up
    auto evaluate = [&]() {
        wave_lds_sync();
        for (int b0 = 0; b0 < ncand; b0 += 64) {
            const int k = b0 + lane;
            const bool has = k < ncand;
            int row = 0, node = 0;
            unsigned long long prev = 0, db = 0;
            if (has) {
                const unsigned cn = s_cn[w][k];
                row = (int)(cn >> 24);
                node = (int)(cn & 0xFFFFFFu);
                prev = s_best[w][row];
                s_ti[w][row] = 0x7fffffff;
                db = (unsigned long long)__double_as_longlong(dist2(tree + (int64_t)node * NQ, &s_q[w][row][0]));
            }
            wave_lds_sync();
            if (has) atomicMin(&s_best[w][row], db);
            wave_lds_sync();
            const unsigned long long cur = has ? s_best[w][row] : 0ull;
            if (has && db == cur) atomicMin(&s_ti[w][row], node);
            wave_lds_sync();
            if (has && db == cur && s_ti[w][row] == node) {
                if (cur < prev) s_bi[w][row] = node;
                else if (node < s_bi[w][row]) s_bi[w][row] = node;
            }
            wave_lds_sync();
        }
        ncand = 0;
        for (int r = lane; r < QW; r += 64) {
            const double b = __longlong_as_double((long long)s_best[w][r]);
            if (b < 1e300) atomicMin(&s_U[w][r], __float_as_uint(f32_up(b)));
        }
        wave_lds_sync();
    };
    // rows whose U fell: new threshold slots (ch 3 lanes) and s_thr
    auto refresh = [&]() {
        wave_lds_sync();
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int r = rb * 16 + (lane & 15);
            const unsigned u = s_U[w][r];
            if (ch == 3 && u != curU[rb] && qw0 + r < n) {
                curU[rb] = u;
                const double U = (double)__uint_as_float(u);
                _Float16 hh, hl;
                thr_slots(P, U, na[rb], hh, hl);
                a[rb][5] = hh;
                a[rb][6] = hl;
                s_thr[w][r] = (float)(U + (P.e0 + P.e1 * U));
            }
        }
        wave_lds_sync();
    };
    constexpr int PF = 4;
    const int64_t ntiles = (t_hi - t_lo + 15) / 16;
    const int col = lane & 15;
    const h8* ib = img + (t_lo + col) * 4 + ch;
    h8 bq[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) bq[u] = ib[min<int64_t>(u, ntiles - 1) * 64];
    const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
    auto tile_step = [&](int64_t tile, const h8& b) {
        f4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rb], b, zero, 0, 0, 0);
        float m = fmaxf(fmaxf(acc[0][0], acc[0][1]), fmaxf(acc[0][2], acc[0][3]));
#pragma unroll
        for (int rb = 1; rb < RB; ++rb) m = fmaxf(m, fmaxf(fmaxf(acc[rb][0], acc[rb][1]), fmaxf(acc[rb][2], acc[rb][3])));
        if (!__any(m >= 0.0f)) return;
        // sign bits -> the passing elements (Q >= 0: a required node has Q > 0)
        unsigned neg = 0;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int e = 0; e < 4; ++e) neg |= (__float_as_uint(acc[rb][e]) >> 31) << (rb * 4 + e);
        unsigned pm = ~neg & (RB >= 8 ? 0xFFFFFFFFu : ((1u << (4 * RB)) - 1u));
        const unsigned node = (unsigned)(t_lo + tile * 16 + col);
        while (__any(pm != 0)) {
            const bool has = pm != 0;
            const int e = has ? __builtin_ctz(pm) : 0;
            pm &= pm - 1;
            const unsigned long long bm = __ballot(has);
            if (ncand + __popcll(bm) > NNC2) {   // (wave-uniform) full list: prune, then evaluate
                prune();
                if (ncand + 64 > NNC2) evaluate();
            }
            if (has) {
                const int row = (e >> 2) * 16 + ch * 4 + (e & 3);
                float q = 0.0f;
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (rb * 4 + k == e) q = acc[rb][k];
                const float thr = s_thr[w][row];
                const float dt = __builtin_fmaf(-q, kq, thr);
                const float eps = __builtin_fmaf(eps1, thr, eps0);
                const float u = fmaxf(dt + eps, 0.0f);
                atomicMin(&s_U[w][row], __float_as_uint(u));
                const int dst = ncand + rank_lanes(bm);
                s_cn[w][dst] = node | ((unsigned)row << 24);
                s_cl[w][dst] = dt - eps;
            }
            ncand += __popcll(bm);
        }
        if (REFRESH > 0 && ++pend >= REFRESH) {
            pend = 0;
            refresh();
        }
    };
    int64_t tb = 0;
    const h8* nx = ib + PF * 64;
    for (; tb + 2 * PF <= ntiles; tb += PF, nx += PF * 64) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            bq[u] = nx[u * 64];
        }
    }
    for (; tb + PF <= ntiles; tb += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            tile_step(tb + u, bq[u]);
            bq[u] = ib[min<int64_t>(tb + u + PF, ntiles - 1) * 64];
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (tb + u < ntiles) tile_step(tb + u, bq[u]);
    if (ncand > 0) {
        prune();
        evaluate();
    }
    wave_lds_sync();
    for (int r = lane; r < QW; r += 64) {
        const int64_t q = qw0 + r;
        if (q < n) part[yr * n + q] = DI2{__longlong_as_double((long long)s_best[w][r]), s_bi[w][r], 0};
    }
}

}  // namespace rp

template <class Run>
void nn_lab_variants(Run& run, int32_t* out0, int32_t* out1) {
    using namespace rp;
    run(k_nnv<4, 4, 0>, 4, out1, "v0 (product copy)", false, out0);
    run(k_nnv<8, 4, 0>, 8, out1, "v0 RB8 (product code)", false, out0);
    run(k_nnv<4, 4, 1>, 4, out1, "v1 fast path only", false, out0);
    run(k_nnv<8, 4, 1>, 8, out1, "v1 RB8 fast path only", false, out0);
    run(k_nnv<4, 4, 3>, 4, out1, "v3 RB4 no loads", false, out0);
    run(k_nnv<8, 4, 3>, 8, out1, "v3 RB8 no loads", false, out0);
    run(k_nnv<8, 4, 1, 2>, 8, out1, "v1 RB8 PF2", false, out0);
    run(k_nnv<8, 4, 1, 8>, 8, out1, "v1 RB8 PF8", false, out0);
    run(k_nnv<8, 4, 0, 8>, 8, out1, "v0 RB8 PF8", false, out0);
    run(k_nnv<4, 4, 0, 4, true>, 4, out1, "v0 RB4 global queries", false, out0);
    run(k_nnv<8, 4, 0, 4, true>, 8, out1, "v0 RB8 global queries", false, out0);
    run(k_nnv<8, 4, 1, 4, true>, 8, out1, "v1 RB8 global queries", false, out0);
    run(k_nnv<8, 4, 0, 4, true, 4>, 8, out1, "v0 RB8 global q, 4 waves/SIMD", false, out0);
    run(k_nnv<4, 4, 0, 4, true, 5>, 4, out1, "v0 RB4 global q, 5 waves/SIMD", false, out0);
    run(1, 4, out1, "product again", false, out0);
    run(1, 8, out1, "product RB8", false, out0);
    run(16, 4, out1, "product RB4 pilot 16", false, out0);
    run(16, 8, out1, "product RB8 pilot 16", false, out0);
    run(8, 4, out1, "product RB4 pilot 8", false, out0);
    run(32, 4, out1, "product RB4 pilot 32", false, out0);
    run(k_nnv<4, 4, 0, 4, true>, 4, out1, "v0 RB4 global queries again", false, out0);
}
