// Micro-benchmark for a counting-sort target build (tools only, not product code): on N random cell keys in [0, D)
//   1. atomicAdd-with-return into a zeroed int[D] (the rank of each point in its cell),
//   2. a full pass over int[D] (read + write, the cell scan's traffic),
//   3. a random 16-byte scatter of N float4 to their ranked slots,
//   4. a random 16-byte gather of N float4 (the finalize's point reads today).
// Build: hipcc --offload-arch=gfx950 -O3 -o count_bench count_bench.hip ; run: ./count_bench N D
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_count(const int* __restrict__ key, int n, int* __restrict__ cnt, int* __restrict__ rank) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) rank[i] = atomicAdd(&cnt[key[i]], 1);
}
__global__ void k_pass(int* __restrict__ a, long long d, int* __restrict__ b) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < d; i += (long long)gridDim.x * blockDim.x) {
        const int v = a[i];
        b[i] = v ? (int)i : -1;
        if (v) a[i] = 0;
    }
}
__global__ void k_scatter(const float4* __restrict__ p, const int* __restrict__ key, const int* __restrict__ rank, int n,
                          const int* __restrict__ off, float4* __restrict__ out, int m) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int pos = (int)(((unsigned)off[key[i] % m] + (unsigned)rank[i]) % (unsigned)n);
        out[pos] = p[i];
    }
}
__global__ void k_gather(const float4* __restrict__ p, const int* __restrict__ idx, int n, float4* __restrict__ out) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = p[idx[i]];
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1840000;
    const long long d = argc > 2 ? atoll(argv[2]) : 5600000;
    std::vector<int> hk(n), hi(n);
    unsigned long long s = 88172645463325252ull;
    const long long vox = n / 9 + 1;  // ~9 points per occupied cell, cells spread over [0, d)
    std::vector<long long> cell(vox);
    for (long long v = 0; v < vox; ++v) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; cell[v] = (long long)(s % (unsigned long long)d); }
    for (int i = 0; i < n; ++i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hk[i] = (int)cell[s % vox]; }
    for (int i = 0; i < n; ++i) hi[i] = i;
    for (int i = n - 1; i > 0; --i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; const int j = (int)(s % (unsigned)(i + 1)); std::swap(hi[i], hi[j]); }
    int *key, *rank, *cnt, *b, *idx;
    float4 *p, *out;
    CK(hipMalloc(&key, n * 4)); CK(hipMalloc(&rank, n * 4)); CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&cnt, d * 4)); CK(hipMalloc(&b, d * 4));
    CK(hipMalloc(&p, n * 16)); CK(hipMalloc(&out, n * 16));
    CK(hipMemcpy(key, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(idx, hi.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(cnt, 0, d * 4)); CK(hipMemset(p, 0, n * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char* what, auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s %9.2f us per launch\n", what, 1000.f * ms / reps);
    };
    const int nb = 2048;
    timeit("count: atomicAdd with return", [&] { hipLaunchKernelGGL(k_count, dim3(nb), dim3(256), 0, 0, key, n, cnt, rank); hipLaunchKernelGGL(k_pass, dim3(nb), dim3(256), 0, 0, cnt, d, b); });
    timeit("cell pass alone (read D, write D)", [&] { hipLaunchKernelGGL(k_pass, dim3(nb), dim3(256), 0, 0, cnt, d, b); });
    timeit("scatter float4 (random write)", [&] { hipLaunchKernelGGL(k_scatter, dim3(nb), dim3(256), 0, 0, p, key, rank, n, b, out, (int)d); });
    timeit("gather float4 (random read)", [&] { hipLaunchKernelGGL(k_gather, dim3(nb), dim3(256), 0, 0, p, idx, n, out); });
    timeit("empty-ish launch", [&] { hipLaunchKernelGGL(k_count, dim3(1), dim3(64), 0, 0, key, 0, cnt, rank); });
    printf("n %d d %lld\n", n, d);
    return 0;
}
