// front_end.hip — filter_node's scan front end on the device: the cloud odom_node receives on
// /filtered_points.
//
// Reference: xchu_mapping/src/filter_node.cpp:218-273 (CloudFilter::Run):
//   pcl::removeNaNFromPointCloud -> keep 1.0 < sqrt(pow(x,2.0) + pow(y,2.0)) < 60 (:238-247, double)
//   -> pcl::VoxelGrid<PointXYZI> leaf 0.5 (:33-34, 249-251; voxel_build.hip + k_downsample_finalize)
//   -> pcl::StatisticalOutlierRemoval<PointXYZI> mean_k 30, stddev_mul 1.0 (:253-263).
// StatisticalOutlierRemoval::applyFilterIndices (PCL 1.7, third-party, not vendored): for every point the k+1
// nearest neighbours (KdTreeFLANN, exact, L2_Simple float squared distances, ascending, the point itself first);
// distance = (float)(sum_{j=1..k} sqrt(d_j) / k) in double; mean / variance over all distances in double
// (sq_sum adds the float square); keep the points with distance <= mean + stddev_mul * stddev, in input order.
//
// MI355X mapping: crop + compaction (flags, single-pass scan, scatter: input order kept); the exact k-NN search
// runs one 16-lane team per query over the block-major nearest-neighbour index (the getFitnessScore index of
// voxel_build.hip), each lane keeping the k+1 smallest squared distances it saw in registers (branch-free min/max
// insertion), merged in ascending order at the end;
// the threshold statistics are one fixed-order f64 reduction (deterministic).  Integer / gather work, no MFMA.
#include "ndt_device.h"

namespace ndt {

// removeNaNFromPointCloud + range crop: flag per point (input order)
__global__ __launch_bounds__(kBlock) void k_crop_flags(const float4* __restrict__ in, int n, double r_min, double r_max,
                                                       int* __restrict__ flags) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 p = in[i];
        bool keep = isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
        if (keep) {
            // std::sqrt(pow(x, 2.0) + pow(y, 2.0)): the squares of floats are exact in double
            const double r = sqrt((double)p.x * (double)p.x + (double)p.y * (double)p.y);
            keep = r_min < r && r < r_max;
        }
        flags[i] = keep ? 1 : 0;
    }
}

// order-preserving compaction: out[idx[i]] = in[i] for the flagged points
__global__ __launch_bounds__(kBlock) void k_compact4(const float4* __restrict__ in, const int* __restrict__ flags,
                                                     const int* __restrict__ idx, int n, float4* __restrict__ out) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock)
        if (flags[i]) out[idx[i]] = in[i];
}

__device__ __forceinline__ float sq_l2_simple(const float4 t, const float q[3]) {
    float d = 0.f, u;
    u = t.x - q[0]; d += u * u;
    u = t.y - q[1]; d += u * u;
    u = t.z - q[2]; d += u * u;
    return d;
}

// The C smallest squared distances one lane has seen, ascending (registers; the insertion is a branch-free min/max
// cascade, taken only when the candidate beats the largest kept value).
template <int C>
struct TopK {
    float v[C];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] = INFINITY;
    }
    __device__ __forceinline__ void insert(float d) {
        if (!(d < v[C - 1])) return;
#pragma unroll
        for (int j = 0; j < C; ++j) {
            const float lo = fminf(v[j], d);
            d = fmaxf(v[j], d);
            v[j] = lo;
        }
    }
    __device__ __forceinline__ int count_le(float b) const {
        int n = 0;
#pragma unroll
        for (int j = 0; j < C; ++j) n += v[j] <= b ? 1 : 0;
        return n;
    }
    __device__ __forceinline__ void pop() {
#pragma unroll
        for (int j = 0; j < C - 1; ++j) v[j] = v[j + 1];
        v[C - 1] = INFINITY;
    }
};

constexpr int kKnnTeam = 16;
__device__ __forceinline__ int team_sum_i(int v) {
    for (int m = kKnnTeam / 2; m > 0; m >>= 1) v += __shfl_xor(v, m, kKnnTeam);
    return v;
}

// StatisticalOutlierRemoval distances: one 16-lane team per query point of `pts` (which is also the indexed cloud);
// every lane keeps the C smallest squared distances of the candidates IT visited, so the team's k+1 smallest are
// among the union of the lane lists.  Search: the 3x3x3 cells around the query cell, then Chebyshev ring 2, cells
// split over the lanes; it stops once k+1 visited candidates lie within the ring's lower bound (every unvisited point
// is at least that far, as in k_fitness); otherwise square shells of 8x8x8-cell blocks from the query's own block
// outwards (fresh lists: every point of every visited block exactly once), each block's points split over the lanes.
// The k+1 smallest are then merged in ascending order (team argmin, ties to the lower lane) and summed as FLANN's
// sorted result: distance = (float)(sum_{j=1..k} sqrt(d_j) / k).
// six waves per SIMD (80 VGPRs, 8 B/lane of scratch instead of 88 VGPRs at five): the team search is latency bound
// (fe workload: 476.9 -> 458.8 us per launch, profiles/r02_s4/sor_waves_ab.txt)
template <int C>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) void k_sor_knn(const float4* __restrict__ pts, int n, int mean_k, const GridHeader* __restrict__ h,
                                                    const int* __restrict__ block_table, const int* __restrict__ cell_off,
                                                    const float4* __restrict__ ix_pts, float* __restrict__ dist_out) {
    const int k1 = mean_k + 1;
    const int db[3] = {h->div_b[0], h->div_b[1], h->div_b[2]};
    const int nbk[3] = {h->nblk[0], h->nblk[1], h->nblk[2]};
    const float cell = h->leaf[0];
    const int t = threadIdx.x % kKnnTeam;
    const int teams = kBlock / kKnnTeam;
    for (int i = blockIdx.x * teams + threadIdx.x / kKnnTeam; i < n; i += gridDim.x * teams) {
        const float4 p = pts[i];
        const float q[3] = {p.x, p.y, p.z};
        TopK<C> top;
        top.init();
        int c[3];
        for (int a = 0; a < 3; ++a) c[a] = (int)(floorf(q[a] * h->inv_leaf[a]) - (float)h->min_b[a]);
        const float slack = 1e-4f * cell + 4e-7f * (fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]));
        int rmax = 0;
        for (int a = 0; a < 3; ++a) rmax = max(rmax, max(c[a], db[a] - 1 - c[a]));
        bool done = false;
        for (int ring = 1; ring <= 2 && !done; ++ring) {
            const int side = 2 * ring + 1, total = side * side * side;
            for (int k = t; k < total; k += kKnnTeam) {
                const int dx = k % side - ring, dy = (k / side) % side - ring, dz = k / (side * side) - ring;
                if (ring == 2 && abs(dx) < 2 && abs(dy) < 2 && abs(dz) < 2) continue;
                const int x = c[0] + dx, y = c[1] + dy, z = c[2] + dz;
                if (x < 0 || y < 0 || z < 0 || x >= db[0] || y >= db[1] || z >= db[2]) continue;
                const int occ = block_table[(((z >> 3) * nbk[1] + (y >> 3)) * nbk[0]) + (x >> 3)];
                if (occ < 0) continue;
                const int l = ((z & 7) << 6) | ((y & 7) << 3) | (x & 7);
                const int* off = cell_off + (size_t)occ * (kFitBlockCells + 1);
                const int e = off[l + 1];
                for (int j = off[l]; j < e; ++j) top.insert(sq_l2_simple(ix_pts[j], q));
            }
            const float bound = fmaxf(0.f, (float)ring * cell - slack);
            done = team_sum_i(top.count_le(bound * bound)) >= k1 || ring >= rmax;
        }
        if (!done) {
            int cb[3], bmax = 0;
            for (int a = 0; a < 3; ++a) {
                cb[a] = c[a] >> 3;
                bmax = max(bmax, max(cb[a], nbk[a] - 1 - cb[a]));
            }
            top.init();
            for (int r = 0; r <= bmax; ++r) {
                const int lo2 = max(cb[2] - r, 0), hi2 = min(cb[2] + r, nbk[2] - 1);
                const int lo1 = max(cb[1] - r, 0), hi1 = min(cb[1] + r, nbk[1] - 1);
                const int lo0 = max(cb[0] - r, 0), hi0 = min(cb[0] + r, nbk[0] - 1);
                for (int z = lo2; z <= hi2; ++z)
                    for (int y = lo1; y <= hi1; ++y)
                        for (int x = lo0; x <= hi0; ++x) {
                            if (abs(z - cb[2]) != r && abs(y - cb[1]) != r && abs(x - cb[0]) != r) continue;
                            const int occ = block_table[((z * nbk[1] + y) * nbk[0]) + x];
                            if (occ < 0) continue;
                            const int* off = cell_off + (size_t)occ * (kFitBlockCells + 1);
                            const int e = off[kFitBlockCells];
                            for (int j = off[0] + t; j < e; j += kKnnTeam) top.insert(sq_l2_simple(ix_pts[j], q));
                        }
                const float bound = fmaxf(0.f, (float)(8 * r) * cell - slack);
                if (team_sum_i(top.count_le(bound * bound)) >= k1) break;
            }
        }
        // merge: k+1 rounds of team argmin over the lane heads, ascending
        double dist_sum = 0.0;
        for (int r = 0; r < k1; ++r) {
            float m = top.v[0];
            int ml = t;
            for (int off = kKnnTeam / 2; off > 0; off >>= 1) {
                const float om = __shfl_xor(m, off, kKnnTeam);
                const int ol = __shfl_xor(ml, off, kKnnTeam);
                if (om < m || (om == m && ol < ml)) { m = om; ml = ol; }
            }
            if (r >= 1) dist_sum += sqrt((double)m);
            if (t == ml) top.pop();
        }
        if (t == 0) dist_out[i] = (float)(dist_sum / (double)mean_k);
    }
}

// RadiusOutlierRemoval (filter_node.cpp:265-272, PCL 1.7 applyFilterIndices): radiusSearch(point, radius) over the
// cloud itself (FLANN: squared distance < (float)(radius*radius), the point itself included); keep the point when it
// has at least min_neighbors.  One 16-lane team per query, the cells whose points can lie within the radius split over
// the lanes.
__global__ __launch_bounds__(kBlock) void k_ror_keep(const float4* __restrict__ pts, int n, double radius, int min_nb,
                                                     const GridHeader* __restrict__ h, const int* __restrict__ block_table,
                                                     const int* __restrict__ cell_off, const float4* __restrict__ ix_pts,
                                                     int* __restrict__ flags) {
    const int db[3] = {h->div_b[0], h->div_b[1], h->div_b[2]};
    const int nbk[3] = {h->nblk[0], h->nblk[1], h->nblk[2]};
    const float cell = h->leaf[0];
    const float r2 = (float)(radius * radius);
    const int t = threadIdx.x % kKnnTeam;
    const int teams = kBlock / kKnnTeam;
    for (int i = blockIdx.x * teams + threadIdx.x / kKnnTeam; i < n; i += gridDim.x * teams) {
        const float4 p = pts[i];
        const float q[3] = {p.x, p.y, p.z};
        int c[3];
        for (int a = 0; a < 3; ++a) c[a] = (int)(floorf(q[a] * h->inv_leaf[a]) - (float)h->min_b[a]);
        const float slack = 1e-4f * cell + 4e-7f * (fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]));
        // every point within the radius lies in a cell at most ext cells away along each axis
        const int ext = max(1, (int)ceilf(((float)radius + slack) / cell));
        const int side = 2 * ext + 1, total = side * side * side;
        int cnt = 0;
        for (int k = t; k < total; k += kKnnTeam) {
            const int x = c[0] + k % side - ext, y = c[1] + (k / side) % side - ext, z = c[2] + k / (side * side) - ext;
            if (x < 0 || y < 0 || z < 0 || x >= db[0] || y >= db[1] || z >= db[2]) continue;
            const int occ = block_table[(((z >> 3) * nbk[1] + (y >> 3)) * nbk[0]) + (x >> 3)];
            if (occ < 0) continue;
            const int l = ((z & 7) << 6) | ((y & 7) << 3) | (x & 7);
            const int* off = cell_off + (size_t)occ * (kFitBlockCells + 1);
            const int e = off[l + 1];
            for (int j = off[l]; j < e; ++j) cnt += sq_l2_simple(ix_pts[j], q) < r2 ? 1 : 0;
        }
        cnt = team_sum_i(cnt);
        if (t == 0) flags[i] = cnt >= min_nb ? 1 : 0;
    }
}

template __global__ void k_sor_knn<32>(const float4*, int, int, const GridHeader*, const int*, const int*, const float4*, float*);
template __global__ void k_sor_knn<64>(const float4*, int, int, const GridHeader*, const int*, const int*, const float4*, float*);

// mean / variance of the distances (one workgroup, fixed order: thread t sums a contiguous chunk, then a fixed
// tree), threshold = mean + stddev_mul * stddev (applyFilterIndices); thr[0] = threshold, thr[1] = mean, thr[2] = stddev
__global__ __launch_bounds__(kBlock) void k_sor_stats(const float* __restrict__ dist, int n, double stddev_mul, double* __restrict__ thr) {
    const int per = (n + kBlock - 1) / kBlock;
    const int b = threadIdx.x * per, e = min(n, b + per);
    double sum = 0.0, sq = 0.0;
    for (int i = b; i < e; ++i) {
        const float d = dist[i];
        sum += d;
        sq += d * d;  // float square, as distances[i] * distances[i] with float operands
    }
    __shared__ double s_sum[kBlock], s_sq[kBlock];
    s_sum[threadIdx.x] = sum;
    s_sq[threadIdx.x] = sq;
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) { s_sum[threadIdx.x] += s_sum[threadIdx.x + off]; s_sq[threadIdx.x] += s_sq[threadIdx.x + off]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double nv = (double)n;
        const double mean = s_sum[0] / nv;
        const double variance = (s_sq[0] - s_sum[0] * s_sum[0] / nv) / (nv - 1);
        const double stddev = sqrt(variance);
        thr[0] = mean + stddev_mul * stddev;
        thr[1] = mean;
        thr[2] = stddev;
    }
}

// keep distances <= threshold (negative_ = false)
__global__ __launch_bounds__(kBlock) void k_sor_keep(const float* __restrict__ dist, int n, const double* __restrict__ thr,
                                                     int* __restrict__ flags) {
    const double t = thr[0];
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) flags[i] = ((double)dist[i] > t) ? 0 : 1;
}

}  // namespace ndt
