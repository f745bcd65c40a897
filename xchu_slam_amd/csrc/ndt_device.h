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

// exp evaluated in double and rounded once: the correctly rounded expf in all but double-rounding ties
// (glibc's expf, used by the reference at ndt_omp_impl.hpp:507, is correctly rounded to 0.502 ulp).
__device__ __forceinline__ float exp_f(float x) { return (float)exp((double)x); }

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    return __shfl_xor(v, m, 64);
}

// Deterministic workgroup reduction of NV doubles per thread; thread v < NV of the block receives sum v.
// Fixed butterfly inside each wave, then waves summed in index order.
template <int NV>
__device__ __forceinline__ void block_reduce_store(double (&acc)[NV], double* red /*LDS [4][NV]*/, double* out, int stride) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double x = acc[v];
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) x += shfl_xor_d(x, m);
        if (lane == 0) red[w * NV + v] = x;
    }
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
