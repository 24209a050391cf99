// Occupancy probe: how many waves of a kernel with W-wave workgroups and L bytes of
// LDS per workgroup are resident per CU / per SIMD at once on this GPU. Each wave
// sleeps, and lane 0 records its start / end time (s_memrealtime) and its hardware
// position (HW_ID: SIMD, CU, SH, SE; XCC_ID); the host counts the largest number of
// overlapping waves per CU and per SIMD.
//   hipcc --offload-arch=gfx950 -O2 -o occupancy_probe tools/occupancy_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

struct Rec { unsigned long long t0, t1; unsigned hw, xcc; };

__global__ void k_sleep(int reps, Rec* out) {
    extern __shared__ int lds[];
    unsigned long long t0, t1;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int r = 0; r < reps; ++r) __builtin_amdgcn_s_sleep(127);
    lds[threadIdx.x] = reps;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) out[w] = Rec{t0, t1 + (lds[threadIdx.x] < 0), hw, xcc};
}

static int max_overlap(std::vector<std::pair<unsigned long long, int>>& ev) {
    std::sort(ev.begin(), ev.end());
    int cur = 0, best = 0;
    for (auto& e : ev) { cur += e.second; best = std::max(best, cur); }
    return best;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int max_waves = cus * 32 * 2;
    Rec* d;
    hipMalloc(&d, sizeof(Rec) * max_waves);
    std::vector<Rec> h(max_waves);
    printf("CUs %d\n", cus);
    const int threads[] = {64, 128, 256};
    for (int B : threads) {
        for (int L = 0; L <= 10240; L += (L < 4096 ? 4096 : 512)) {
            const int wpb = B / 64;
            const size_t lds = std::max<size_t>((size_t)L * wpb, (size_t)B * 4);
            const int blocks = max_waves / wpb;
            hipLaunchKernelGGL(k_sleep, dim3(blocks), dim3(B), lds, 0, 40, d);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            hipMemcpy(h.data(), d, sizeof(Rec) * max_waves, hipMemcpyDeviceToHost);
            // CU key: XCC, SE, SH, CU (HW_ID bits 8..15); SIMD: bits 4..5
            std::map<unsigned, std::vector<std::pair<unsigned long long, int>>> cu, simd;
            for (int w = 0; w < blocks * wpb; ++w) {
                const unsigned key = ((h[w].xcc & 0xf) << 8) | ((h[w].hw >> 8) & 0xff);
                cu[key].push_back({h[w].t0, +1});
                cu[key].push_back({h[w].t1, -1});
                const unsigned skey = (key << 2) | ((h[w].hw >> 4) & 3);
                simd[skey].push_back({h[w].t0, +1});
                simd[skey].push_back({h[w].t1, -1});
            }
            int cmax = 0, smax = 0;
            for (auto& kv : cu) cmax = std::max(cmax, max_overlap(kv.second));
            for (auto& kv : simd) smax = std::max(smax, max_overlap(kv.second));
            printf("block %3d threads, LDS %6zu B/block (%5d B/wave): %zu CUs seen, max %2d waves/CU, max %d waves/SIMD\n",
                   B, lds, L, cu.size(), cmax, smax);
        }
    }
    return 0;
}
