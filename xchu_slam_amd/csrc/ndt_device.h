// ndt_device.h — device helpers shared by the build, pass and control kernels.
#pragma once
#include <hip/hip_runtime.h>
#include "ndt_types.h"
#include "ndt_linalg.h"
#include "ndt_pair.h"

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
// Workgroup barrier that orders LDS only: it does not wait for this wave's outstanding global loads/stores
// (HIP's __syncthreads() is a fence on every address space, i.e. also an s_waitcnt vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int NW = kBlock / 64>
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds /*[NW]*/, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds[w] = x;
    lds_barrier();
    int wofs = 0;
    for (int q = 0; q < w; ++q) wofs += lds[q];
    int tot = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) tot += lds[q];
    lds_barrier();
    *total = tot;
    return wofs + x - v;
}


// Profiling build only (-DNDT_BODY_STAMPS, `make VARIANT=dbg`): per-workgroup phase stamps of the first
// kBlkPasses passes, plain stores into private slots (no contention), read back by ndt_dbg_read_blk.
#ifdef NDT_BODY_STAMPS
constexpr int kBlkPasses = 64, kBlkMax = 1024, kBlkSlots = 8;
static __device__ unsigned long long g_blk_ts[kBlkPasses * kBlkMax * kBlkSlots];
// per-tile phase sums of one workgroup (probe, compaction, pairs), stored into slots 5..7 at the end of the body
#define NDT_TILE_ACC(acc, mark, k)                                        \
    do {                                                                  \
        __syncthreads();                                                  \
        const unsigned long long _n = __builtin_amdgcn_s_memrealtime();   \
        (acc)[k] += _n - (mark);                                          \
        (mark) = _n;                                                      \
    } while (0)
#define NDT_TILE_ACC_STORE(pass, acc)                                                                          \
    do {                                                                                                       \
        if (threadIdx.x == 0 && (pass) >= 0 && (pass) < kBlkPasses && blockIdx.x < kBlkMax)                     \
            for (int _k = 0; _k < 3; ++_k) g_blk_ts[((size_t)(pass) * kBlkMax + blockIdx.x) * kBlkSlots + 5 + _k] = (acc)[_k]; \
    } while (0)
#define NDT_BLK_STAMP(pass, slot)                                                                            \
    do {                                                                                                     \
        __syncthreads();                                                                                     \
        if (threadIdx.x == 0 && (pass) >= 0 && (pass) < kBlkPasses && blockIdx.x < kBlkMax)                   \
            g_blk_ts[((size_t)(pass) * kBlkMax + blockIdx.x) * kBlkSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
// the last workgroup's tail of pass p stamps into the unused workgroup row kBlkMax-1 of pass p
static __device__ unsigned long long* g_tail_ts;
static __device__ unsigned g_tail_wg;  // the workgroup whose tail stamps g_tail_ts (leading-tail kernels: workgroup 0)
#define NDT_TAIL_STAMP(slot)                                                  \
    do {                                                                      \
        if (g_tail_ts && g_tail_wg == blockIdx.x) g_tail_ts[(slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define NDT_BLK_STAMP(pass, slot) do { } while (0)
#define NDT_TAIL_STAMP(slot) do { } while (0)
#endif

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
    return __shfl_xor(v, m, 64);
}

// Cross-lane exchanges of the reduce-scatter below, all register-to-register (no LDS round trip):
//   swap32: v_permlane32_swap  — lanes 32..63 of A trade places with lanes 0..31 of B;
//   swap16: v_permlane16_swap  — odd 16-lane rows of A trade places with even rows of B;
//   dpp<C>: v_mov_b32_dpp      — row_ror:8 / row_half_mirror / quad_perm partner reads (m = 8, 4, 2, 1).
__device__ __forceinline__ void split_d(double v, unsigned& lo, unsigned& hi) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    lo = (unsigned)u;
    hi = (unsigned)(u >> 32);
}
__device__ __forceinline__ double join_d(unsigned lo, unsigned hi) {
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
template <int M>
__device__ __forceinline__ double swap_add_d(double A, double B) {
    unsigned al, ah, bl, bh;
    split_d(A, al, ah);
    split_d(B, bl, bh);
    if (M == 32) {
        const auto l = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
        return join_d(l[0], h[0]) + join_d(l[1], h[1]);
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
        return join_d(l[0], h[0]) + join_d(l[1], h[1]);
    }
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    unsigned lo, hi;
    split_d(v, lo, hi);
    lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, 0xf, 0xf, false);
    hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, 0xf, 0xf, false);
    return join_d(lo, hi);
}
template <int M>
__device__ __forceinline__ double partner_d(double v) {
    // the partner differs from this lane in bit log2(M) and agrees in every higher bit
    if (M == 8) return dpp_d<0x128>(v);   // row_ror:8
    if (M == 4) return dpp_d<0x141>(v);   // row_half_mirror
    if (M == 2) return dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
    return dpp_d<0xB1>(v);                // quad_perm [1,0,3,2]
}

template <int M>
__device__ __forceinline__ void rs_step(double* a, int lane) {
    if (M >= 16) {
        // lanes with bit M clear keep a[i] + partner's a[i]; lanes with it set keep a[i+M] + partner's a[i+M]
#pragma unroll
        for (int i = 0; i < M; ++i) a[i] = swap_add_d<M>(a[i], a[i + M]);
    } else {
        const bool hi = (lane & M) != 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const double keep = hi ? a[i + M] : a[i];
            const double send = hi ? a[i] : a[i + M];
            a[i] = keep + partner_d<M>(send);
        }
    }
}

// Deterministic workgroup reduction of NV (<= 64) doubles per thread; thread v < NV of the block receives
// sum v.  Inside each wave a reduce-scatter: at the step for lane bit m every lane keeps half of the values
// it carries and adds its partner's copy of that half, so the wave needs 32+16+8+4+2+1 = 63 exchanges (not
// 6*NV) and lane l ends with the wave total of value l.  Waves are then summed in index order.
template <int NV, int NW = kBlock / 64>
__device__ __forceinline__ void block_reduce_store(double (&acc)[NV], double* red /*LDS [NW][NV]*/, double* out, int stride) {
    static_assert(NV <= 64, "reduce-scatter carries at most 64 values");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[64];
#pragma unroll
    for (int v = 0; v < 64; ++v) a[v] = v < NV ? acc[v] : 0.0;
    rs_step<32>(a, lane);
    rs_step<16>(a, lane);
    rs_step<8>(a, lane);
    rs_step<4>(a, lane);
    rs_step<2>(a, lane);
    rs_step<1>(a, lane);
    // lane l now holds the wave sum of value l in a[0]
    if (lane < NV) red[w * NV + lane] = a[0];
    lds_barrier();
    if ((int)threadIdx.x < NV) {
        const int v = threadIdx.x;
        double s = red[v];
#pragma unroll
        for (int q = 1; q < NW; ++q) s += red[q * NV + v];
        // write-through (sc1) store: visible at agent scope once drained, no L2 write-back fence needed
        __hip_atomic_store(out + (size_t)v * stride, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Split accumulation (NDT_SPLIT_ACC, derivatives.hip): lanes 0-31 of a wave hold the sums of the 22 "low" terms of every
// pair (score, g0..g2, H columns 0..2), lanes 32-63 the 22 "high" ones (g3..g5, the pair count, H columns 3..5): each pair's
// terms are exchanged across the half-waves (v_permlane32_swap) as they are produced, so that a lane keeps 22 f64 sums
// instead of 44.  Value k of the low / high set -> index of the 44 reduced values:
__host__ __device__ constexpr int split_lo_term(int k) { return k < 4 ? k : 7 + 6 * ((k - 4) / 3) + (k - 4) % 3; }
__host__ __device__ constexpr int split_hi_term(int k) { return k < 3 ? 4 + k : (k == 3 ? 43 : 10 + 6 * ((k - 4) / 3) + (k - 4) % 3); }
constexpr int kSplitAcc = 22;

// block_reduce_store for split sums: the state after the reduce-scatter's first (lane bit 32) step of block_reduce_store,
// which the per-pair exchange already did; the remaining steps, then value -> term.
template <int NW = kBlock / 64>
__device__ __forceinline__ void block_reduce_store_split(double (&acc)[kSplitAcc], double* red /*LDS [NW][kNumAcc]*/, double* out,
                                                         int stride) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double a[32];
#pragma unroll
    for (int v = 0; v < 32; ++v) a[v] = v < kSplitAcc ? acc[v] : 0.0;
    rs_step<16>(a, lane);
    rs_step<8>(a, lane);
    rs_step<4>(a, lane);
    rs_step<2>(a, lane);
    rs_step<1>(a, lane);
    // lane l holds the wave sum of value l: low value l (l < 32) or high value l - 32
    const int k = lane & 31;
    if (k < kSplitAcc) red[w * kNumAcc + (lane < 32 ? split_lo_term(k) : split_hi_term(k))] = a[0];
    lds_barrier();
    if ((int)threadIdx.x < kNumAcc) {
        const int v = threadIdx.x;
        double s = red[v];
#pragma unroll
        for (int q = 1; q < NW; ++q) s += red[q * kNumAcc + v];
        __hip_atomic_store(out + (size_t)v * stride, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace ndt
