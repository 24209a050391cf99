// nn_lab.hip — standalone A/B harness for the nearest-node matrix-core kernel
// (diagnostic tool, not the product): builds in seconds instead of the library's
// minutes. Generates n uniform queries and an RRT-like tree of T nodes (random-walk
// branches, as tools/nn_bench.py), makes the node images (k_nn_image), runs the
// product kernel rp::k_nn_mfma<RB, 4> and the experimental variants of
// tools/nn_lab_kern.h, reduces over the ranges (k_nn_reduce), checks every variant's
// indices against the product's and the product's against a CPU brute force on a
// sample of queries, and prints the kernel times (HIP events, median of reps).
//
//   hipcc (library flags) -o tools/lab/nn_lab tools/nn_lab.hip   (tools/lab/build.sh)
//   tools/lab/nn_lab [n] [T] [reps]
#include "../rbe550_final_project_amd/csrc/rp_kernels.h"
#include "../rbe550_final_project_amd/csrc/rp_nn.h"
#include "nn_lab_kern.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <type_traits>
#include <vector>

using namespace rp;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static const double QLO[NQ] = {-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973, 0.0, 0.0};
static const double QHI[NQ] = {2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973, 0.04, 0.04};

// rp_lib.hip nn_mfma_params (the same constants)
static bool params(const double* lo, const double* hi, NnMfma* P) {
    double r2 = 0.0;
    for (int i = 0; i < NQ; ++i) {
        P->c[i] = 0.5 * (lo[i] + hi[i]);
        const double h = 0.5 * (hi[i] - lo[i]);
        r2 += h * h;
    }
    const double R0 = std::sqrt(r2) * (1.0 + 1e-9) + 1e-12;
    P->S = std::ldexp(1.0, (int)std::floor(std::log2(16384.0 / R0)));
    const double s2r2 = P->S * P->S * R0 * R0;
    const int H = (int)std::ceil(std::log2(2.2 * s2r2 / 65504.0));
    const int G = (int)std::ceil(std::log2(0.55 * s2r2 / 65504.0));
    P->H2 = std::ldexp(1.0, H);
    P->G2 = std::ldexp(1.0, G);
    P->iH2 = std::ldexp(1.0, -H);
    P->iG2 = std::ldexp(1.0, -G);
    P->e0 = 8e-5 * R0 * R0 + 1e-12;
    P->e1 = 2e-5;
    P->thr0 = 4.04 * R0 * R0 + P->e0;
    return true;
}

struct Geom {
    int64_t qblocks, chunk;
    int S;
};
static Geom geom(int64_t n, int64_t T, int RB, int W) {
    const int64_t per_block = (int64_t)W * 16 * RB;
    Geom g;
    g.qblocks = (n + per_block - 1) / per_block;
    const int64_t stages = (T + 63) / 64;
    const int64_t want = std::max<int64_t>(1, (1024 + g.qblocks - 1) / g.qblocks);
    const int64_t S0 = std::max<int64_t>(1, std::min<int64_t>(want, stages / 32));
    g.chunk = ((stages + S0 - 1) / S0) * 64;
    g.S = (int)((T + g.chunk - 1) / g.chunk);
    return g;
}

template <class F>
static float timed(F launch, int reps, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, s));
        launch();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float m = 0;
        CK(hipEventElapsedTime(&m, a, b));
        ms.push_back(m);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 131072;
    const int64_t T = argc > 2 ? atoll(argv[2]) : 300000;
    const int reps = argc > 3 ? atoi(argv[3]) : 7;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> N(0.0, 1.0);
    std::vector<double> q(n * NQ), tree(T * NQ);
    for (int64_t i = 0; i < n; ++i)
        for (int d = 0; d < NQ; ++d) q[i * NQ + d] = QLO[d] + (QHI[d] - QLO[d]) * U(rng);
    double span = 0;
    for (int d = 0; d < NQ; ++d) span = std::max(span, QHI[d] - QLO[d]);
    for (int d = 0; d < NQ; ++d) tree[d] = QLO[d] + (QHI[d] - QLO[d]) * U(rng);
    for (int64_t i = 1; i < T; ++i) {   // random-walk branches (tools/nn_bench.py walk_tree)
        const int64_t par = (int64_t)(U(rng) * (double)i);
        double dv[NQ], nn = 0;
        for (int d = 0; d < NQ; ++d) nn += (dv[d] = N(rng)) * dv[d];
        const double st = 0.2 * span / 6.0 / std::sqrt(nn);
        for (int d = 0; d < NQ; ++d)
            tree[i * NQ + d] = std::min(QHI[d], std::max(QLO[d], tree[par * NQ + d] + dv[d] * st));
    }
    NnMfma P;
    params(QLO, QHI, &P);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    double *dq, *dt;
    h8* dimg;
    DI2 *part, *pilot;
    int32_t *out0, *out1;
    CK(hipMalloc(&dq, sizeof(double) * n * NQ));
    CK(hipMalloc(&dt, sizeof(double) * T * NQ));
    CK(hipMalloc(&dimg, sizeof(h8) * (T + NNM_PAD) * 4));
    CK(hipMalloc(&part, sizeof(DI2) * n * 64));
    CK(hipMalloc(&pilot, sizeof(DI2) * n * 16));
    CK(hipMalloc(&out0, sizeof(int32_t) * n));
    CK(hipMalloc(&out1, sizeof(int32_t) * n));
    CK(hipMemcpy(dq, q.data(), sizeof(double) * n * NQ, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, tree.data(), sizeof(double) * T * NQ, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_nn_image, dim3((unsigned)(((T + NNM_PAD) * 4 + 255) / 256)), dim3(256), 0, s,
                       (const double*)dt, (int64_t)0, T, P, dimg);
    CK(hipStreamSynchronize(s));

    auto run = [&](auto kern, int RB, int32_t* out, const char* name, bool check, const int32_t* ref) {
        const Geom g = geom(n, T, RB, 4);
        auto launch = [&]() {
            if constexpr (std::is_same_v<decltype(kern), int>) {   // the product: kern = pilot stride
                int S1 = 0;
                if (kern > 1) {   // the pilot over every kern-th tile (rp_lib.hip launch_nn_mfma_w)
                    const int64_t qb1 = (n + 255) / 256;
                    const int64_t sub = ((T + 15) / 16 + kern - 1) / kern;
                    int64_t s1 = std::max<int64_t>(1, std::min<int64_t>({(1024 + qb1 - 1) / qb1, sub / 8, 16}));
                    const int64_t chunk1 = (sub + s1 - 1) / s1 * kern * 16;
                    S1 = (int)((T + chunk1 - 1) / chunk1);
                    hipLaunchKernelGGL((k_nn_mfma<4, 4>), dim3((unsigned)(qb1 * S1)), dim3(256), 0, s,
                                       (const double*)dq, n, (const int*)nullptr, (int64_t)0, (const double*)dt,
                                       (const h8*)dimg, T, chunk1, qb1, P, pilot, 0, kern, (const DI2*)nullptr, 0, (const int*)nullptr, (unsigned long long*)nullptr);
                }
                if (RB == 8)
                    hipLaunchKernelGGL((k_nn_mfma<8, 4>), dim3((unsigned)(g.qblocks * g.S)), dim3(256), 0, s,
                                       (const double*)dq, n, (const int*)nullptr, (int64_t)0, (const double*)dt,
                                       (const h8*)dimg, T, g.chunk, g.qblocks, P, part, 0, 1,
                                       kern > 1 ? (const DI2*)pilot : nullptr, S1, (const int*)nullptr, (unsigned long long*)nullptr);
                else
                    hipLaunchKernelGGL((k_nn_mfma<4, 4>), dim3((unsigned)(g.qblocks * g.S)), dim3(256), 0, s,
                                       (const double*)dq, n, (const int*)nullptr, (int64_t)0, (const double*)dt,
                                       (const h8*)dimg, T, g.chunk, g.qblocks, P, part, 0, 1,
                                       kern > 1 ? (const DI2*)pilot : nullptr, S1, (const int*)nullptr, (unsigned long long*)nullptr);
            } else {
                hipLaunchKernelGGL(kern, dim3((unsigned)(g.qblocks * g.S)), dim3(256), 0, s, (const double*)dq, n,
                                   (const int*)nullptr, (int64_t)0, (const double*)dt, (const h8*)dimg, T, g.chunk,
                                   g.qblocks, P, part);
            }
        };
        launch();
        CK(hipGetLastError());
        const float ms = timed(launch, reps, s);
        hipLaunchKernelGGL(k_nn_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const DI2*)part, n, g.S,
                           (const int*)nullptr, (int64_t)0, out);
        CK(hipStreamSynchronize(s));
        std::vector<int32_t> h(n), r(ref ? n : 0);
        CK(hipMemcpy(h.data(), out, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        if (ref) {
            CK(hipMemcpy(r.data(), ref, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < n; ++i) bad += h[i] != r[i];
        }
        if (check) {   // CPU brute force on 512 queries (strict-< scan: lowest index on ties)
            for (int64_t i = 0; i < n; i += n / 512) {
                double bd = INFINITY;
                int bi = -1;
                for (int64_t j = 0; j < T; ++j) {
                    double d2 = 0;
                    for (int d = 0; d < NQ; ++d) {
                        const double e = tree[j * NQ + d] - q[i * NQ + d];
                        d2 += e * e;
                    }
                    if (d2 < bd) { bd = d2; bi = (int)j; }
                }
                (void)bd;
                bad += h[i] != bi;
            }
        }
        const double pairs = (double)n * (double)T;
        printf("%-28s RB %d  %8.3f ms  %6.2f e12 pairs/s  %5.3f of f16 MFMA peak  mismatches %lld\n", name, RB, ms,
               pairs / (ms * 1e-3) / 1e12, pairs * 64 / (ms * 1e-3) / 2.5e15, (long long)bad);
        fflush(stdout);
    };
    run(1, 4, out0, "product k_nn_mfma", true, nullptr);   // (int kern: the product, pilot stride)
    nn_lab_variants(run, out0, out1);
    return 0;
}
