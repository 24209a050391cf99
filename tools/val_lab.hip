// val_lab.hip — standalone A/B harness for the state-validity kernel (diagnostic
// tool, not the product). The k_validity compiled into this binary from the tree's
// current headers (rp_math.h / rp_kernels.h: the variant under test) runs beside the
// one inside a librbe_mi355x.so build (dlopen, RBE_LIB_PATH: the baseline), on the
// same HBM-resident uniform states and the same scene record (rp_debug_scene), with
// HIP events on one stream, interleaved; flags must be bit-identical.
//
//   tools/lab/build.sh val_lab && tools/lab/val_lab [states] [reps] [scene: goal3|pentagon|toppled]
#include "../rbe550_final_project_amd/csrc/rp_kernels.h"
#include "../include/rbe_planner.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <dlfcn.h>

// the baseline library, loaded at run time (RBE_LIB_PATH, default the in-tree build)
struct Lib {
    int (*create)(rp_ctx**, int, const rp_robot_desc*);
    int (*set_scene)(rp_ctx*, const rp_box*, int32_t, float, const float*);
    int (*set_scene_rot)(rp_ctx*, const rp_box_rot*, int32_t, float, const float*);
    int (*debug_scene)(rp_ctx*, void*, int64_t);
    int (*check_dev)(rp_ctx*, const float*, int64_t, uint8_t*, void*);
    int (*get_stream)(rp_ctx*, void**);
    void (*destroy)(rp_ctx*);
};
static Lib load_lib() {
    const char* path = getenv("RBE_LIB_PATH");
    if (!path || !*path) path = "rbe550_final_project_amd/librbe_mi355x.so";
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(1); }
    Lib L;
    L.create = (decltype(L.create))dlsym(h, "rp_create");
    L.set_scene = (decltype(L.set_scene))dlsym(h, "rp_set_scene");
    L.set_scene_rot = (decltype(L.set_scene_rot))dlsym(h, "rp_set_scene_rot");
    L.debug_scene = (decltype(L.debug_scene))dlsym(h, "rp_debug_scene");
    L.check_dev = (decltype(L.check_dev))dlsym(h, "rp_check_states_device");
    L.get_stream = (decltype(L.get_stream))dlsym(h, "rp_get_stream");
    L.destroy = (decltype(L.destroy))dlsym(h, "rp_destroy");
    if (!L.create || !L.debug_scene || !L.check_dev) { fprintf(stderr, "%s lacks rp_debug_scene\n", path); exit(1); }
    return L;
}

using namespace rp;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ void k_uniform(float* q, int64_t n, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int d = 0; d < NQ; ++d) {
        uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull + (uint64_t)d * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
        q[i * NQ + d] = Q_LO_F[d] + (Q_HI_F[d] - Q_LO_F[d]) * u;
    }
}

template <int NCL>
void launch(const float* q, int64_t n, uint8_t* f, const DevScene* sc, hipStream_t s) {
    hipLaunchKernelGGL((k_validity<NCL, true>), dim3((unsigned)((n + VTHREADS - 1) / VTHREADS)), dim3(VTHREADS), 0, s,
                       q, n, f, sc);
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : (1 << 24);
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const char* scene = argc > 3 ? argv[3] : "goal3";
    std::vector<rp_box> boxes;
    std::vector<rp_box_rot> rboxes;
    const double xs[2] = {0.45, 0.65}, ys[5] = {-0.40, -0.20, 0.0, 0.20, 0.40};
    for (double x : xs)
        for (double y : ys) boxes.push_back(rp_box{{(float)x, (float)y, 0.02f}, {0.02f, 0.02f, 0.02f}, 0.0f});
    if (!strcmp(scene, "pentagon"))
        for (size_t k = 0; k < boxes.size(); ++k) boxes[k].yaw = (float)(0.6283 * k);
    const Lib L = load_lib();
    rp_ctx* ctx = nullptr;
    if (L.create(&ctx, 0, nullptr) != 0) { fprintf(stderr, "rp_create failed\n"); return 1; }
    const float base[3] = {0.0f, 0.0f, 0.01f};
    if (!strcmp(scene, "toppled")) {
        for (size_t k = 0; k < boxes.size(); ++k) {
            rp_box_rot b{};
            std::memcpy(b.center, boxes[k].center, sizeof b.center);
            std::memcpy(b.half, boxes[k].half, sizeof b.half);
            const double a = 0.3 * (double)k;   // a tilt about an oblique axis per block
            b.quat[0] = std::cos(a / 2); b.quat[1] = 0.6 * std::sin(a / 2); b.quat[2] = 0.8 * std::sin(a / 2);
            rboxes.push_back(b);
        }
        L.set_scene_rot(ctx, rboxes.data(), (int)rboxes.size(), 0.0f, base);
    } else {
        L.set_scene(ctx, boxes.data(), (int)boxes.size(), 0.0f, base);
    }
    DevScene hs;
    if (L.debug_scene(ctx, &hs, sizeof hs) != 0) { fprintf(stderr, "rp_debug_scene: layout mismatch\n"); return 1; }
    DevScene* ds;
    float* q;
    uint8_t *fa, *fb;
    CK(hipMalloc(&ds, sizeof hs));
    CK(hipMemcpy(ds, &hs, sizeof hs, hipMemcpyHostToDevice));
    CK(hipMalloc(&q, sizeof(float) * NQ * n));
    CK(hipMalloc(&fa, n));
    CK(hipMalloc(&fb, n));
    hipStream_t s;
    void* vs = nullptr;
    L.get_stream(ctx, &vs);
    s = (hipStream_t)vs;
    hipLaunchKernelGGL(k_uniform, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, n, 1234ull);
    CK(hipStreamSynchronize(s));
    const int ncl = hs.grid ? NCL_GRID : hs.n_clusters <= 0 ? 0 : hs.n_clusters == 1 ? 1 : hs.n_clusters == 2 ? 2
                                                             : hs.n_clusters <= 4 ? 4 : 8;
    auto lab = [&]() {
        switch (ncl) {
            case 0: launch<0>(q, n, fb, ds, s); break;
            case 1: launch<1>(q, n, fb, ds, s); break;
            case 2: launch<2>(q, n, fb, ds, s); break;
            case 4: launch<4>(q, n, fb, ds, s); break;
            default: launch<8>(q, n, fb, ds, s); break;
        }
    };
    auto lib = [&]() { L.check_dev(ctx, q, n, fa, s); };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time1 = [&](auto f) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 5; ++k) f();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms / 5;
    };
    lib();
    lab();
    CK(hipStreamSynchronize(s));
    std::vector<float> ta, tb;
    for (int r = 0; r < reps; ++r) {
        ta.push_back(time1(lib));
        tb.push_back(time1(lab));
    }
    std::sort(ta.begin(), ta.end());
    std::sort(tb.begin(), tb.end());
    std::vector<uint8_t> ha(n), hb(n);
    CK(hipMemcpy(ha.data(), fa, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), fb, n, hipMemcpyDeviceToHost));
    int64_t diff = 0, valid = 0;
    for (int64_t i = 0; i < n; ++i) {
        diff += ha[i] != hb[i];
        valid += ha[i];
    }
    const double ma = ta[ta.size() / 2], mb = tb[tb.size() / 2];
    printf("%s n=%lld ncl=%d: library %.4f ms (%.2f G/s)  tree headers %.4f ms (%.2f G/s)  ratio %.4f  "
           "min %.4f / %.4f  flags differ %lld  valid %.4f\n",
           scene, (long long)n, ncl, ma, n / (ma * 1e-3) / 1e9, mb, n / (mb * 1e-3) / 1e9, ma / mb, ta[0], tb[0],
           (long long)diff, (double)valid / n);
#ifdef RP_PAIR_STATS
    {   // per self pair: sphere passes, AABB passes, narrow-phase hits per state (one lab launch)
        unsigned long long z[NPAIR + 1][3] = {};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_pairstats), z, sizeof z));
        lab();
        CK(hipStreamSynchronize(s));
        unsigned long long h[NPAIR + 1][3];
        CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pairstats), sizeof h));
        double ts = 0, ta = 0, th = 0;
        for (int p = 0; p < NPAIR; ++p) {
            if (!h[p][0]) continue;
            printf("pair %2d (%2d,%2d): sphere %.4f  aabb %.4f  hit %.4f per state\n", p, PAIRS[p][0], PAIRS[p][1],
                   (double)h[p][0] / n, (double)h[p][1] / n, (double)h[p][2] / n);
            ts += h[p][0]; ta += h[p][1]; th += h[p][2];
        }
        printf("all pairs: sphere %.3f  aabb %.3f  hit %.3f per state\n", ts / n, ta / n, th / n);
    }
#endif
    L.destroy(ctx);
    return diff != 0;
}
