// synth_pairs.hip — on-device generator of the C4 batched-replay pairs ("pairs are generated on
// device from the seed so PCIe time is not counted").  BENCH INFRASTRUCTURE, not part of the NDT product surface
// (include/ndt_hip.h): built into its own libndt_synth.so, called by bench.py before the timed region.
//
// A pair restates xchu_slam_amd/synth.py's World on the device: the localmap samples every surface of a seeded world
// (undulating ground stratified per 1 m cell, building facades and poles by area) in a pseudo-random order; the scan is
// a LiDAR-like sample (density ~ 1/r up to max_range) of the same surfaces around a sensor pose, in the sensor frame.
// The small per-pair world (buildings, poles, pose) comes from the host (synth.make_world + a numpy pose); every point
// is a pure function of (seed, index) through a counter-based hash, so pair i is the same bits on any GPU / rank.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "ndt_synth.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// uniform [0,1) with 24 bits, and a second independent one from the same 64-bit draw
__device__ __forceinline__ float u_hi(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float u_lo(uint64_t h) { return (float)((h >> 8) & 0xffffffull) * (1.0f / 16777216.0f); }

__device__ __forceinline__ uint64_t draw(uint64_t seed, uint64_t idx, uint32_t k) {
    return mix64(mix64(seed * 0x100000001b3ull + k) ^ idx);
}

// standard normal pair (Box-Muller)
__device__ __forceinline__ void gauss2(uint64_t h, float* a, float* b) {
    const float u1 = 1.0f - u_hi(h);  // (0, 1]
    const float u2 = u_lo(h);
    const float r = sqrtf(-2.0f * logf(u1));
    float s, c;
    sincospif(2.0f * u2, &s, &c);
    *a = r * c;
    *b = r * s;
}

__device__ __forceinline__ float ground_z(float x, float y) { return 0.2f * sinf(x / 15.0f) * cosf(y / 11.0f); }

__device__ int pick_cdf(const float* cdf, int n, float u) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// a point on the facade of building k (synth.World._walls): perimeter parameter s, height fraction v
__device__ float3 wall_point(const float* b, float s01, float v01) {
    const float cx = b[0], cy = b[1], w = b[2], d = b[3], h = b[4], yaw = b[5];
    const float s = s01 * 2.0f * (w + d);
    float u, v;
    if (s < w) { u = s - w / 2; v = -d / 2; }
    else if (s < w + d) { u = w / 2; v = -d / 2 + (s - w); }
    else if (s < 2 * w + d) { u = w / 2 - (s - w - d); v = d / 2; }
    else { u = -w / 2; v = d / 2 - (s - 2 * w - d); }
    float sn, c;
    sincosf(yaw, &sn, &c);
    return make_float3(cx + c * u - sn * v, cy + sn * u + c * v, v01 * h);
}

__device__ float3 pole_point(const float* p, float th01, float v01) {
    float s, c;
    sincospif(2.0f * th01, &s, &c);
    return make_float3(p[0] + p[2] * c, p[1] + p[2] * s, v01 * p[3]);
}

// Feistel bijection on [0, 2^(2*hb)), cycle-walked into [0, M): the localmap's point order
__device__ uint64_t feistel(uint64_t x, int hb, uint64_t key) {
    const uint64_t mask = (1ull << hb) - 1;
    uint64_t l = x >> hb, r = x & mask;
    for (int k = 0; k < 4; ++k) {
        const uint64_t f = mix64(r ^ (key + (uint64_t)k * 0x632be59bd9b4e019ull)) & mask;
        const uint64_t t = l ^ f;
        l = r;
        r = t;
    }
    return (l << hb) | r;
}

__global__ void k_synth_target(SynthPairDesc d, const float* __restrict__ world, float4* __restrict__ out) {
    const long long M = d.n_ground + d.n_walls + d.n_poles;
    const float* bld = world;
    const float* bcdf = world + 6 * d.nb;
    const float* poles = world + 6 * d.nb + 2 * d.nb;
    const uint64_t key = mix64(d.seed_target ^ 0x5bd1e995ull);
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < M; q += (long long)gridDim.x * blockDim.x) {
        uint64_t j = (uint64_t)q;
        do { j = feistel(j, d.perm_half_bits, key); } while (j >= (uint64_t)M);
        const uint64_t h0 = draw(d.seed_target, j, 0);
        float3 p;
        if ((long long)j < d.n_ground) {
            const long long cell = (long long)j / d.per_cell;
            const int ii = (int)(cell / d.cells_side), jj = (int)(cell % d.cells_side);
            const float x = (float)ii - d.half + u_hi(h0), y = (float)jj - d.half + u_lo(h0);
            p = make_float3(x, y, ground_z(x, y));
        } else if ((long long)j < d.n_ground + d.n_walls) {
            const int k = pick_cdf(bcdf, d.nb, u_hi(h0));
            const uint64_t h1 = draw(d.seed_target, j, 1);
            p = wall_point(bld + 6 * k, u_hi(h1), u_lo(h1));
        } else {
            const int k = min(d.np - 1, (int)(u_hi(h0) * d.np));
            const uint64_t h1 = draw(d.seed_target, j, 1);
            p = pole_point(poles + 4 * k, u_hi(h1), u_lo(h1));
        }
        float n0, n1, n2, n3;
        gauss2(draw(d.seed_target, j, 2), &n0, &n1);
        gauss2(draw(d.seed_target, j, 3), &n2, &n3);
        out[q] = make_float4(p.x + d.noise * n0, p.y + d.noise * n1, p.z + d.noise * n2, 1.0f);
    }
}

__global__ void k_synth_source(SynthPairDesc d, const float* __restrict__ world, float4* __restrict__ out) {
    const float* bld = world;
    const float* poles = world + 6 * d.nb + 2 * d.nb;
    const float* near_b = world + 6 * d.nb + d.nb;            // near-building cdf (nb entries)
    const float* near_p = world + 6 * d.nb + 2 * d.nb + 4 * d.np;  // near-pole cdf (np entries)
    const float R = d.max_range;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < d.n_source; q += gridDim.x * blockDim.x) {
        float3 p = make_float3(d.cx + 2.0f, d.cy, 0.0f);
        for (uint32_t a = 0; a < 512; ++a) {
            const uint64_t h0 = draw(d.seed_source, (uint64_t)q, 4 * a);
            const uint64_t h1 = draw(d.seed_source, (uint64_t)q, 4 * a + 1);
            const float cls = u_hi(h0);
            float3 c;
            if (cls < 0.55f || (cls < 0.95f && d.nb_near == 0) || (cls >= 0.95f && d.np_near == 0)) {
                const float rr = 1.0f + u_lo(h0) * (R - 1.0f);
                float s, co;
                sincospif(2.0f * u_hi(h1), &s, &co);
                const float x = d.cx + rr * co, y = d.cy + rr * s;
                c = make_float3(x, y, ground_z(x, y));
            } else if (cls < 0.95f) {
                const int k = pick_cdf(near_b, d.nb, u_lo(h0));
                c = wall_point(bld + 6 * k, u_hi(h1), u_lo(h1));
            } else {
                const int k = pick_cdf(near_p, d.np, u_lo(h0));
                c = pole_point(poles + 4 * k, u_hi(h1), u_lo(h1));
            }
            const float r = hypotf(c.x - d.cx, c.y - d.cy);
            const float thin = u_hi(draw(d.seed_source, (uint64_t)q, 4 * a + 2));
            p = c;
            if (r > 1.0f && r < R && fabsf(c.x) < d.half && fabsf(c.y) < d.half && thin < fminf(1.0f, 15.0f / fmaxf(r, 1.0f))) break;
        }
        float n0, n1, n2, n3;
        gauss2(draw(d.seed_source, (uint64_t)q, 4000), &n0, &n1);
        gauss2(draw(d.seed_source, (uint64_t)q, 4001), &n2, &n3);
        const double x = (double)(p.x + d.noise * n0), y = (double)(p.y + d.noise * n1), z = (double)(p.z + d.noise * n2);
        const double* m = d.world_to_sensor;
        out[q] = make_float4((float)(m[0] * x + m[1] * y + m[2] * z + m[3]), (float)(m[4] * x + m[5] * y + m[6] * z + m[7]),
                             (float)(m[8] * x + m[9] * y + m[10] * z + m[11]), 1.0f);
    }
}

}  // namespace

extern "C" int ndt_synth_world_floats(int nb, int np) { return 6 * nb + 2 * nb + 4 * np + np; }

extern "C" int ndt_synth_pair_device(const SynthPairDesc* desc, const float* h_world, float* d_world, void* d_target,
                                     void* d_source) {
    if (!desc || !h_world || !d_world || !d_target || !d_source || desc->nb <= 0 || desc->np <= 0 || desc->n_source < 0)
        return 1;
    if (hipSetDevice(desc->device) != hipSuccess) return 5;
    const size_t wbytes = sizeof(float) * (size_t)ndt_synth_world_floats(desc->nb, desc->np);
    if (hipMemcpy(d_world, h_world, wbytes, hipMemcpyHostToDevice) != hipSuccess) return 5;
    const long long M = desc->n_ground + desc->n_walls + desc->n_poles;
    if (M > 0) hipLaunchKernelGGL(k_synth_target, dim3(4096), dim3(256), 0, nullptr, *desc, d_world, (float4*)d_target);
    if (desc->n_source > 0)
        hipLaunchKernelGGL(k_synth_source, dim3((desc->n_source + 255) / 256), dim3(256), 0, nullptr, *desc, d_world,
                           (float4*)d_source);
    if (hipGetLastError() != hipSuccess) return 5;
    return hipDeviceSynchronize() == hipSuccess ? 0 : 5;
}
