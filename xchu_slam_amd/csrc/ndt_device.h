// ndt_device.h — device helpers shared by the build, pass and control kernels.
#pragma once
#include <hip/hip_runtime.h>
#include "ndt_types.h"
#include "ndt_linalg.h"

namespace ndt {

__device__ __forceinline__ unsigned hash_slot(int key, unsigned log2cap) {
    return ((unsigned)key * 0x9E3779B1u) >> (32u - log2cap);
}

// Open-addressing lookup: returns the stored value (cloud index, possibly with kRejectBit) or -1.
__device__ __forceinline__ int hash_find(const int2* __restrict__ table, unsigned log2cap, int key) {
    const unsigned mask = (1u << log2cap) - 1u;
    unsigned h = hash_slot(key, log2cap);
    for (;;) {
        const int2 e = table[h];
        if (e.x == key) return e.y;
        if (e.x == kEmptyKey) return -1;
        h = (h + 1u) & mask;
    }
}

// Voxel key -> cloud index (| kRejectBit) or -1: dense cell index grid when the grid fits its allocation,
// open-addressing hash otherwise (GridHeader::dense decides, per build).
__device__ __forceinline__ int voxel_lookup(bool dense, const int* __restrict__ grid, const int2* __restrict__ table,
                                            unsigned log2cap, int key) {
    return dense ? grid[key] : hash_find(table, log2cap, key);
}

// Block-wide exclusive scan of one int per thread (kBlock threads); *total = sum.  Two barriers.
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds /*[4]*/, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds[w] = x;
    __syncthreads();
    int wofs = 0;
    for (int q = 0; q < w; ++q) wofs += lds[q];
    const int tot = lds[0] + lds[1] + lds[2] + lds[3];
    __syncthreads();
    *total = tot;
    return wofs + x - v;
}

// exp evaluated in double and rounded once: the correctly rounded expf in all but double-rounding ties
// (glibc's expf, used by the reference at ndt_omp_impl.hpp:507, is correctly rounded to 0.502 ulp).
__device__ __forceinline__ float exp_f(float x) { return (float)exp((double)x); }

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    return __shfl_xor(v, m, 64);
}

// Deterministic workgroup reduction of NV (<= 64) doubles per thread; thread v < NV of the block receives
// sum v.  Inside each wave a reduce-scatter butterfly: at the step with lane mask m every lane keeps half of
// the values it carries and adds the partner's copy of that half, so the wave needs 32+16+8+4+2+1 = 63
// shuffles (not 6*NV) and lane l ends with the wave total of value l.  Waves are then summed in index order.
template <int NV>
__device__ __forceinline__ void block_reduce_store(double (&acc)[NV], double* red /*LDS [4][NV]*/, double* out, int stride) {
    static_assert(NV <= 64, "reduce-scatter carries at most 64 values");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[64];
#pragma unroll
    for (int v = 0; v < 64; ++v) a[v] = v < NV ? acc[v] : 0.0;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const bool hi = (lane & m) != 0;
#pragma unroll
        for (int i = 0; i < m; ++i) {
            const double keep = hi ? a[i + m] : a[i];
            const double send = hi ? a[i] : a[i + m];
            a[i] = keep + shfl_xor_d(send, m);
        }
    }
    // lane l now holds the wave sum of value l in a[0]
    if (lane < NV) red[w * NV + lane] = a[0];
    __syncthreads();
    if ((int)threadIdx.x < NV) {
        const int v = threadIdx.x;
        double s = red[v];
        s += red[NV + v];
        s += red[2 * NV + v];
        s += red[3 * NV + v];
        out[(size_t)v * stride] = s;
    }
}

}  // namespace ndt
