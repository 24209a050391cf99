// rp_plan_math.h — float64 state-space arithmetic of the planner (device side).
//
// OMPL RealVectorStateSpace semantics used by RRTConnect inside ss.solve
// (code/planning.py:143-156, 190) [EXT-OMPL, SURVEY.md App. B.1]: Euclidean
// distance over the 9 dims, interpolation from + (to - from) * t, uniform sampling
// lo + (hi - lo) * u. Written to the numerics contract so the CPU
// oracle's trees are bit-identical: fixed summation order, no FMA contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rp_model.h"

namespace rp {

constexpr uint32_t SAMPLE_TAG = 0x52425035u;

// (a 64-bit product, not __umulhi: the device-library call is not inlined into
// kernels built with -mno-amdgpu-ieee, whose attributes differ; this is one
// v_mul_hi_u32)
__device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        const uint32_t hi0 = mulhi32(0xD2511F53u, c[0]);
        const uint32_t lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c[2]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0;
        const uint32_t n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    }
}

// Global sample g of the query (counter-based: independent of batch split / rank).
__device__ __forceinline__ void sample_state(uint64_t seed, uint64_t g, const double* lo,
                                             const double* hi, double q[NQ], uint32_t tag = SAMPLE_TAG) {
    uint32_t u[12];
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        uint32_t c[4] = {(uint32_t)g, (uint32_t)(g >> 32), j, tag};
        philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        u[4 * j + 0] = c[0]; u[4 * j + 1] = c[1]; u[4 * j + 2] = c[2]; u[4 * j + 3] = c[3];
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const double x = (double)u[i] * 2.3283064365386962890625e-10;
        q[i] = lo[i] + (hi[i] - lo[i]) * x;
    }
}

__device__ __forceinline__ double dist2(const double* a, const double* b) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const double d = a[i] - b[i];
        s = s + d * d;
    }
    return s;
}

__device__ __forceinline__ void interp(const double* a, const double* b, double t, double* out) {
#pragma unroll
    for (int i = 0; i < NQ; ++i) out[i] = a[i] + (b[i] - a[i]) * t;
}

// RRTConnect::growTree steering: move at most `range` from near toward target.
__device__ __forceinline__ int steer(const double* near, const double* target, double range,
                                     double* out) {
    const double d = sqrt(dist2(near, target));
    if (d > range) {
        interp(near, target, range / d, out);
        return 0;
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) out[i] = target[i];
    return 1;
}

// validSegmentCount: ceil(|b - a| / resolution)
__device__ __forceinline__ int segment_count(const double* a, const double* b, double res) {
    return (int)ceil(sqrt(dist2(a, b)) / res);
}

}  // namespace rp
