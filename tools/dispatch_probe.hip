// dispatch_probe.hip — how fast the chip retires one-wave workgroups that do (almost)
// nothing: the floor of an edge pass-1 launch whose grid (groups x kmax rounds) is
// mostly rounds past every group's items. Variants: no work; one scalar load then exit;
// two dependent vector loads + a wave scan (k_edges' layout scan) then exit. Each with
// the k_edges LDS footprint (~7 KB) or none. Prints microseconds per launch (HIP events,
// median of 20) and workgroups per microsecond.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lab/dispatch_probe tools/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int LDSW>
__global__ __launch_bounds__(1024) void k_empty(int* out) {
    __shared__ float lds[LDSW > 0 ? LDSW : 1];
    if (LDSW > 0 && threadIdx.x == 999) { lds[threadIdx.x] = 1.0f; out[0] = (int)lds[threadIdx.x ^ 1]; }
}

template <int LDSW>
__global__ __launch_bounds__(64, 5) void k_scalar(const int* __restrict__ rounds, int kk, int* out) {
    __shared__ float lds[LDSW > 0 ? LDSW : 1];
    const int g = blockIdx.x / kk, r = blockIdx.x - g * kk;
    if (r >= rounds[g]) return;   // (rounds = 0: every wave exits here)
    lds[threadIdx.x] = (float)r;
    __builtin_amdgcn_wave_barrier();
    out[blockIdx.x] = (int)lds[threadIdx.x ^ 1];
}

template <int LDSW>
__global__ __launch_bounds__(64, 5) void k_scan(const int* __restrict__ nd, const int* __restrict__ cntv, int kk,
                                                int* out) {
    __shared__ float lds[LDSW > 0 ? LDSW : 1];
    const int g = blockIdx.x / kk, r = blockIdx.x - g * kk;
    const int lane = threadIdx.x;
    const int d = nd[g * 64 + lane];
    int c = d >= 0 ? cntv[g * 64 + lane] : 0;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(c, o, 64);
        if (lane >= o) c += v;
    }
    const int total = __builtin_amdgcn_readlane(c, 63);
    if (r * 64 >= total) return;
    lds[lane] = (float)c;
    __builtin_amdgcn_wave_barrier();
    out[blockIdx.x] = (int)lds[lane ^ 1];
}

template <class F>
float time_it(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> v;
    for (int i = 0; i < 25; ++i) {
        hipEventRecord(a, 0);
        f();
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (i >= 5) v.push_back(ms * 1e3f);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const int kk = 38;
    const int blocks[] = {9216, 58368, 175104};
    const int maxg = 175104 / kk + 1;
    int *rounds, *nd, *cntv, *out;
    CK(hipMalloc(&rounds, maxg * sizeof(int)));
    CK(hipMalloc(&nd, maxg * 64 * sizeof(int)));
    CK(hipMalloc(&cntv, maxg * 64 * sizeof(int)));
    CK(hipMalloc(&out, 175104 * sizeof(int)));
    CK(hipMemset(rounds, 0, maxg * sizeof(int)));
    CK(hipMemset(nd, 0, maxg * 64 * sizeof(int)));
    CK(hipMemset(cntv, 0, maxg * 64 * sizeof(int)));   // no items anywhere: every wave is dead
    for (int wpb : {4, 16}) {   // waves per workgroup, same wave count as the one-wave grids
        for (int nb : blocks) {
            const float t = time_it([&] { hipLaunchKernelGGL(k_empty<0>, dim3(nb / wpb), dim3(64 * wpb), 0, 0, out); });
            const float tl = time_it([&] { hipLaunchKernelGGL(k_empty<1760 * 4>, dim3(nb / wpb), dim3(64 * wpb), 0, 0, out); });
            printf("waves %6d as %d-wave WGs: empty %6.1f us (%5.0f waves/us) | +28 KB LDS %6.1f (%5.0f)\n", nb, wpb, t, nb / t,
                   tl, nb / tl);
        }
    }
    for (int nb : blocks) {
        const float t0 = time_it([&] { hipLaunchKernelGGL(k_empty<0>, dim3(nb), dim3(64), 0, 0, out); });
        const float t1 = time_it([&] { hipLaunchKernelGGL(k_empty<1760>, dim3(nb), dim3(64), 0, 0, out); });
        const float t2 = time_it([&] { hipLaunchKernelGGL(k_scalar<1760>, dim3(nb), dim3(64), 0, 0, rounds, kk, out); });
        const float t3 = time_it([&] { hipLaunchKernelGGL(k_scan<1760>, dim3(nb), dim3(64), 0, 0, nd, cntv, kk, out); });
        const float t4 = time_it([&] { hipLaunchKernelGGL(k_scalar<0>, dim3(nb), dim3(64), 0, 0, rounds, kk, out); });
        printf("blocks %6d: empty %6.1f us (%5.0f WG/us) | empty+7KB LDS %6.1f (%5.0f) | scalar-load exit %6.1f (%5.0f) | "
               "scalar no LDS %6.1f (%5.0f) | scan exit %6.1f (%5.0f)\n",
               nb, t0, nb / t0, t1, nb / t1, t2, nb / t2, t4, nb / t4, t3, nb / t3);
    }
    return 0;
}
