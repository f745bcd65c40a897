// solver.hip — small helper kernels around the align chain: the aligned output cloud (k_transform / k_transform_mat),
// the rare JacobiSVD fallback of a degenerate Newton system (k_svd_resume), the align's state upload (k_align_init) and
// its end-of-round read-back into pinned host memory (k_readback).  The Newton / More-Thuente driver itself
// (computeTransformation, ndt_omp_impl.hpp:73-164; computeStepLengthMT :760-916) lives in ndt_control.h and runs inside
// the derivative-pass kernels (derivatives.hip): in the last workgroup of a pass, or at the start of the next pass's
// kernel (leading-tail chains).
#include "ndt_control.h"

namespace ndt {

// Aligned output cloud: source transformed by final_transformation_ (pcl::transformPointCloud).
__global__ __launch_bounds__(kBlock) void k_transform(const float4* __restrict__ src, int n, const AlignState* __restrict__ st,
                                                      float4* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* T = st->T;
    const float4 p = src[i];
    float4 o;
    o.x = T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12];
    o.y = T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13];
    o.z = T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14];
    o.w = 1.0f;
    out[i] = o;
}

// pcl::transformPointCloud(in, out, T) for a caller-given f32 transform (odom_node.cpp:220, 290): x,y,z
// transformed in the same operation order as k_transform, the 4th lane (intensity) carried through.
__global__ __launch_bounds__(kBlock) void k_transform_mat(const float4* __restrict__ src, int n, Mat4f T, float4* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 p = src[i];
    float4 o;
    o.x = T.m[0] * p.x + T.m[4] * p.y + T.m[8] * p.z + T.m[12];
    o.y = T.m[1] * p.x + T.m[5] * p.y + T.m[9] * p.z + T.m[13];
    o.z = T.m[2] * p.x + T.m[6] * p.y + T.m[10] * p.z + T.m[14];
    o.w = p.w;
    out[i] = o;
}

// Device-to-device copy of 16-byte words for the C-ABI's copies (setInputSource, the odom driver's localmap snapshot):
// a plain kernel follows the previous kernel on the stream with no gap, where a runtime blit copy costs a launch of its
// own and ~6 us of idle queue before it (rocprofv3, C2 step: 4.4 us copy + 6.2 us gap)
__global__ __launch_bounds__(kBlock) void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) dst[i] = src[i];
}

// Rare path: the Newton system was degenerate for LU; solve it with Eigen's JacobiSVD semantics (rank
// truncation) and resume the optimiser exactly where control_step paused.
__global__ __launch_bounds__(kBlock) void k_svd_resume(AlignState* st) {
    __shared__ AlignState s_st;
    constexpr int kWords = sizeof(AlignState) / 8;
    unsigned long long* gw = reinterpret_cast<unsigned long long*>(st);
    unsigned long long* lw = reinterpret_cast<unsigned long long*>(&s_st);
    for (int k = threadIdx.x; k < kWords; k += kBlock) lw[k] = gw[k];
    __syncthreads();
    if (threadIdx.x == 0 && s_st.needs_svd && !s_st.done) {
        double mg[6];
        for (int k = 0; k < 6; ++k) mg[k] = -s_st.g[k];
        svd_solve6_rowmajor(s_st.H, mg, s_st.svd_dp);
        s_st.svd_ready = 1;
        s_st.needs_svd = 0;
        newton_request(&s_st);
    }
    solve_loop(&s_st);
    if (s_st.needs_tables) prepare_pass_parallel(&s_st);
    for (int k = threadIdx.x; k < kWords; k += kBlock) gw[k] = lw[k];
}

// Start of an align in one launch (instead of a state upload, a ticket-counter memset and a stamp memset + init):
// the host-built state arrives as the kernel argument, the pass ticket counters are zeroed, and (profiling) the
// stamp rows are reset — slot 0 of each row to ~0 (a min), the others to 0.
static_assert(sizeof(AlignState) <= 3072, "AlignState travels as a kernel argument (4 KB limit)");
__global__ void k_align_init(const AlignState st, AlignState* __restrict__ d_state, unsigned* __restrict__ counter,
                             unsigned long long* __restrict__ ts, int ts_words, unsigned long long* __restrict__ clk,
                             const GridHeader* __restrict__ hdr, unsigned long long seq, const uint4* __restrict__ cp_src,
                             uint4* __restrict__ cp_dst, long long cp_words) {
    constexpr int kWords = sizeof(AlignState) / 8;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    // the source copy ndt_set_source_device deferred to this align (16-byte words, grid-stride)
    for (long long k = i; k < cp_words; k += (long long)gridDim.x * kBlock) cp_dst[k] = cp_src[k];
    if (blockIdx.x == 0) {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&st);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(d_state);
        for (int k = threadIdx.x; k < kWords; k += kBlock) dst[k] = src[k];
        for (int k = threadIdx.x; k < kPassCounterWords; k += kBlock) counter[k] = 0u;  // pass tickets (incl. group tickets)
        if (threadIdx.x == 0) {
            clk[0] = __builtin_amdgcn_s_memrealtime();  // the align's device clock span starts here
            clk[2] = seq;  // the sequence number the first round's read-back (captured in the chain's graph) releases
        }
        // the look-back error flag of the target build queued ahead of this align is latched into the align's own state
        // (a later setInputTarget rewrites the shared header before this align is waited for)
        __syncthreads();
        if (threadIdx.x == 0) {
            d_state->build_error = hdr ? hdr->pad[0] : 0;
            d_state->grid_cells = hdr ? hdr->cells : 0;
        }
    }
    if (ts)
        for (int k = i; k < ts_words; k += gridDim.x * kBlock) ts[k] = (k % kTsStride) == 0 ? ~0ull : 0ull;
}

// End-of-round read-back into pinned host memory by one workgroup: the optimiser state and, when profiling, the stamps
// and pass records of this round — replaces up to three blit copies and the launch gaps between them — and the target
// header's build error bits.  Then the
// align's device clock span (clk[0] = k_align_init's start stamp) and, last, the round's sequence number, released at
// system scope after every thread's stores: the host spins on it instead of waking from a stream synchronisation.
__global__ __launch_bounds__(kBlock) void k_readback(const unsigned long long* __restrict__ st, unsigned long long* h_st, int st_words,
                                                     const unsigned long long* __restrict__ ts, unsigned long long* h_ts, int ts_words,
                                                     const unsigned long long* __restrict__ hist, unsigned long long* h_hist,
                                                     int hist_words, const unsigned long long* __restrict__ clk, unsigned long long* h_clk,
                                                     unsigned long long* h_seq, unsigned long long seq,
                                                     unsigned long long* __restrict__ d_mirror, const GridHeader* __restrict__ hdr) {
    // seq == 0: the round's sequence number is clk[2] (k_align_init wrote it), so that the launch can sit in a graph
    if (seq == 0) seq = clk[2];
    const int i = threadIdx.x;
    for (int k = i; k < st_words; k += kBlock) {
        const unsigned long long w = st[k];
        h_st[k] = w;
        if (d_mirror) d_mirror[k] = w;  // leading-tail chains: the final state also into the primary state buffer
    }
    for (int k = i; k < ts_words; k += kBlock) h_ts[k] = ts[k];
    for (int k = i; k < hist_words; k += kBlock) h_hist[k] = hist[k];
    if (i == 0) {
        h_clk[0] = clk[0];
        h_clk[1] = __builtin_amdgcn_s_memrealtime();
        h_clk[2] = clk[3];  // the start stamp of the last target build (k_minmax)
        // the target header's build error bits at the end of the round (incl. the align's own source-order sort)
        h_clk[3] = hdr ? (unsigned long long)(unsigned)hdr->pad[0] : 0ull;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this thread's stores reach host memory first
    __syncthreads();
    if (i == 0) __hip_atomic_store(h_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace ndt
