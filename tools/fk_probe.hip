// fk_probe.hip — the device's joint sin / cos and capsule endpoints of one state
// (diagnostic: compare with oracle.OracleScene.fk_capsules / oracle.sincos).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//     -Xarch_device -fno-honor-nans -Xarch_device -mno-amdgpu-ieee -o tools/lab/fk_probe tools/fk_probe.hip
//   tools/lab/fk_probe q0 ... q8
#include "../rbe550_final_project_amd/csrc/rp_kernels.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void k_fk(const float* q, const rp::DevScene* sc, float* out) {
    float qq[rp::NQ];
    for (int i = 0; i < rp::NQ; ++i) qq[i] = q[i];
    for (int i = 0; i < 7; ++i) {
        rp::rp_sincos(qq[i], &out[2 * i], &out[2 * i + 1]);
        out[200 + i] = floorf(qq[i] * 0.636619772f + 0.5f);
    }
    rp::Capsules k;
    rp::fk_capsules(qq, sc, k);
    for (int c = 0; c < rp::NCAP; ++c) {
        out[14 + 6 * c + 0] = k.a[c].x; out[14 + 6 * c + 1] = k.a[c].y; out[14 + 6 * c + 2] = k.a[c].z;
        out[14 + 6 * c + 3] = k.b[c].x; out[14 + 6 * c + 4] = k.b[c].y; out[14 + 6 * c + 5] = k.b[c].z;
    }
}

// sin / cos of n values (the sweep mode: tools/lab/fk_probe --sweep < values)
__global__ void k_sc(const float* x, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rp::rp_sincos(x[i], &out[2 * i], &out[2 * i + 1]);
}

int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "--sweep")) {
        std::vector<float> xs;
        float v;
        while (scanf("%f", &v) == 1) xs.push_back(v);
        const int n = (int)xs.size();
        float *dx, *dy;
        (void)hipMalloc(&dx, n * sizeof(float));
        (void)hipMalloc(&dy, 2 * n * sizeof(float));
        (void)hipMemcpy(dx, xs.data(), n * sizeof(float), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_sc, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, dy);
        std::vector<float> y(2 * n);
        (void)hipMemcpy(y.data(), dy, 2 * n * sizeof(float), hipMemcpyDeviceToHost);
        for (int i = 0; i < n; ++i) printf("%.9g %.9g %.9g\n", xs[i], y[2 * i], y[2 * i + 1]);
        return 0;
    }
    float q[9] = {0};
    for (int i = 0; i < 9 && i + 1 < argc; ++i) q[i] = strtof(argv[i + 1], nullptr);
    rp::DevScene h;
    memset(&h, 0, sizeof(h));
    h.base[2] = 0.01f;
    float *dq, *dout;
    rp::DevScene* ds;
    (void)hipMalloc(&dq, sizeof(q));
    (void)hipMalloc(&dout, 256 * sizeof(float));
    (void)hipMalloc(&ds, sizeof(h));
    (void)hipMemcpy(dq, q, sizeof(q), hipMemcpyHostToDevice);
    (void)hipMemcpy(ds, &h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_fk, dim3(1), dim3(1), 0, 0, dq, ds, dout);
    float o[256];
    (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    for (int i = 0; i < 7; ++i) printf("joint %d q %.9g k %g sin %.9g cos %.9g\n", i, q[i], o[200 + i], o[2 * i], o[2 * i + 1]);
    for (int c = 0; c < rp::NCAP; ++c)
        printf("cap %2d a %.9g %.9g %.9g b %.9g %.9g %.9g\n", c, o[14 + 6 * c], o[15 + 6 * c], o[16 + 6 * c], o[17 + 6 * c],
               o[18 + 6 * c], o[19 + 6 * c]);
    return 0;
}
