// voxel_build.hip — target voxel grid (pclomp::VoxelGridCovariance::applyFilter) on the device.
//
// Reference: voxel_grid_covariance_omp_impl.hpp:48-370 (min/max, overflow guard, binning with
// floor(x*inv_leaf) - (float)min_b, f64 moments per leaf starting from cov_ = Identity, (n-1)/n scaling,
// SelfAdjointEigenSolver + eigenvalue inflation, inverse, rejection), voxel_grid_covariance_omp.h:285-297.
//
// MI355X pipeline (all device-resident, no host sync, capturable in a hipGraph):
//   minmax -> header -> voxel key per point -> stable LSD radix sort (key, point index), 8-bit digits,
//   only as many passes as the key needs -> segment heads + scan -> per-voxel finalize (one thread per voxel,
//   points summed in input order = the reference's std::map insertion order, f64) -> compaction of the
//   voxels with >= min points (the reference's KD cloud) in ascending key order -> open-addressing hash.
// HBM-bound integer/byte work: coalesced tiles of 4096 keys per workgroup, LDS digit counters, wave ballots
// for stable in-wave ranks; no atomics on data (counts only), so the result is bitwise deterministic.
#include "ndt_device.h"

namespace ndt {

constexpr int kTileItems = 16;                  // items per thread per tile
constexpr int kTile = kBlock * kTileItems;      // 4096 keys per workgroup
constexpr int kRadixAux = kRadixAuxWords;         // digit histograms of the 4 passes (copies) + 4 tile tickets

// ---------------------------------------------------------------- min / max (pcl::getMinMax3D)
// Workgroup 0 also clears the digit histograms k_keys adds into (radix_aux = [copies][4 digit positions][256] + [4] tile
// tickets), so that k_keys needs no separate header kernel before it.
// clk_start (target builds): the build's start stamp (100 MHz device clock), for ndt_last_timings without stream events
// (an event recorded between two kernels costs the stream ~6 us of idle, rocprofv3)
// hdr_save (a merge-extended target, k_merge_append): workgroup 0 also keeps the current target header in hdr_save before
// k_keys replaces it (k_keys folds the saved box into the new one, k_merge_append reads the old key layout from it).
// copy_to (a merge-extended target whose new points the caller left elsewhere): the points are also stored there.
__global__ __launch_bounds__(kBlock) void k_minmax(const float4* __restrict__ pts, int n, int is_dense, float* __restrict__ part,
                                                   int* __restrict__ radix_aux, unsigned long long* __restrict__ clk_start,
                                                   const GridHeader* __restrict__ hdr_cur, GridHeader* __restrict__ hdr_save,
                                                   float4* __restrict__ copy_to) {
    if (clk_start && blockIdx.x == 0 && threadIdx.x == 0) *clk_start = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < kRadixAux; i += kBlock) radix_aux[i] = 0;
        if (hdr_save) {
            static_assert(sizeof(GridHeader) % 4 == 0 && sizeof(GridHeader) / 4 <= kBlock, "header copy: one word per thread");
            if (threadIdx.x < sizeof(GridHeader) / 4)
                reinterpret_cast<int*>(hdr_save)[threadIdx.x] = reinterpret_cast<const int*>(hdr_cur)[threadIdx.x];
        }
    }
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int cnt = 0;
    // four points per thread per round, all loads issued before any is consumed
    const int stride = gridDim.x * kBlock;
    for (int i0 = blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += 4 * stride) {
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = i0 + u * stride < n ? pts[i0 + u * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
        if (copy_to) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * stride < n) copy_to[i0 + u * stride] = q[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 p = q[u];
            if (i0 + u * stride >= n) break;
            if (!is_dense && !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) continue;
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            ++cnt;
        }
    }
    __shared__ float s[kBlock][7];
    s[threadIdx.x][0] = mn[0]; s[threadIdx.x][1] = mn[1]; s[threadIdx.x][2] = mn[2];
    s[threadIdx.x][3] = mx[0]; s[threadIdx.x][4] = mx[1]; s[threadIdx.x][5] = mx[2];
    s[threadIdx.x][6] = __int_as_float(cnt);
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            const int o = threadIdx.x + off;
            for (int a = 0; a < 3; ++a) s[threadIdx.x][a] = fminf(s[threadIdx.x][a], s[o][a]);
            for (int a = 3; a < 6; ++a) s[threadIdx.x][a] = fmaxf(s[threadIdx.x][a], s[o][a]);
            s[threadIdx.x][6] = __int_as_float(__float_as_int(s[threadIdx.x][6]) + __float_as_int(s[o][6]));
        }
        __syncthreads();
    }
    if (threadIdx.x < 7) part[blockIdx.x * 7 + threadIdx.x] = s[0][threadIdx.x];
}

// ---------------------------------------------------------------- grid header
// From the nb min/max partials, by one workgroup (parallel reduction, order independent); thread 0 stores the header to
// *h (LDS here: every k_keys workgroup derives it itself, workgroup 0 also stores it for the later kernels).
// fold (a merge-extended target): the current target's box and point count join the new points' (pcl::getMinMax3D over
// old + new points, order independent)
__device__ __forceinline__ void header_body(const float* __restrict__ part, int nb, GridHeader* h, float leaf, int min_pts, double eig_mult,
                                            int is_dense, int layout, int binning, float (*s)[7],
                                            const GridHeader* __restrict__ fold = nullptr) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int cnt = 0;
    if (fold && threadIdx.x == 0) {
        for (int a = 0; a < 3; ++a) { mn[a] = fold->minp[a]; mx[a] = fold->maxp[a]; }
        cnt = fold->n_points;
    }
    for (int b = threadIdx.x; b < nb; b += kBlock) {
        for (int a = 0; a < 3; ++a) { mn[a] = fminf(mn[a], part[b * 7 + a]); mx[a] = fmaxf(mx[a], part[b * 7 + 3 + a]); }
        cnt += __float_as_int(part[b * 7 + 6]);
    }
    for (int a = 0; a < 3; ++a) { s[threadIdx.x][a] = mn[a]; s[threadIdx.x][3 + a] = mx[a]; }
    s[threadIdx.x][6] = __int_as_float(cnt);
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) {
            const int o = threadIdx.x + off;
            for (int a = 0; a < 3; ++a) s[threadIdx.x][a] = fminf(s[threadIdx.x][a], s[o][a]);
            for (int a = 3; a < 6; ++a) s[threadIdx.x][a] = fmaxf(s[threadIdx.x][a], s[o][a]);
            s[threadIdx.x][6] = __int_as_float(__float_as_int(s[threadIdx.x][6]) + __float_as_int(s[o][6]));
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    for (int a = 0; a < 3; ++a) { mn[a] = s[0][a]; mx[a] = s[0][3 + a]; }
    cnt = __float_as_int(s[0][6]);
    GridHeader g;
    for (int a = 0; a < 4; ++a) { g.min_b[a] = g.max_b[a] = g.div_b[a] = g.divb_mul[a] = 0; }
    for (int a = 0; a < 3; ++a) { g.leaf[a] = leaf; g.inv_leaf[a] = 1.0f / leaf; g.minp[a] = mn[a]; g.maxp[a] = mx[a]; }
    g.leaf[3] = 1.f; g.inv_leaf[3] = 1.f; g.minp[3] = g.maxp[3] = 0.f;
    g.n_points = cnt;
    g.n_leaves = g.n_cloud = g.n_valid = 0;
    g.overflow = 0;
    g.empty = 0;
    g.key_bits = 0;
    g.sentinel = 0;
    g.log2cap = 6;
    g.min_points = min_pts;
    g.min_eig_mult = eig_mult;
    g.cells = 0;
    g.dense = 0;
    g.pad[0] = g.pad[1] = 0;
    g.binning = binning;
    g.layout = layout;
    g.n_blocks_occ = 0;
    g.nblk[0] = g.nblk[1] = g.nblk[2] = g.nblk[3] = 0;
    g.flip = 0;
    g.pad2 = 0;
    if (cnt == 0) {
        g.empty = 1;
    } else if (layout == 1) {
        // nearest-neighbour index: cell = leaf, doubled until the block-major key range fits kFitMaxKeys (the
        // search is exact for any cell size; the cell only trades table size against points per cell)
        float cell = leaf;
        long long R = 0;
        for (int it = 0; it < 64; ++it) {
            const float inv = 1.0f / cell;
            long long nbk[3];
            for (int a = 0; a < 3; ++a) {
                g.min_b[a] = (int)floorf(mn[a] * inv);
                g.max_b[a] = (int)floorf(mx[a] * inv);
                g.div_b[a] = g.max_b[a] - g.min_b[a] + 1;
                nbk[a] = ((long long)g.div_b[a] + 7) >> 3;
            }
            R = nbk[0] * nbk[1] * nbk[2] * kFitBlockCells;
            if (R <= kFitMaxKeys && g.div_b[0] > 0 && g.div_b[1] > 0 && g.div_b[2] > 0) {
                for (int a = 0; a < 3; ++a) g.nblk[a] = (int)nbk[a];
                break;
            }
            cell *= 2.0f;
        }
        for (int a = 0; a < 3; ++a) { g.leaf[a] = cell; g.inv_leaf[a] = 1.0f / cell; }
        g.divb_mul[0] = 1;
        g.divb_mul[1] = g.div_b[0];
        g.divb_mul[2] = g.div_b[0] * g.div_b[1];
        g.cells = R;
        int bits = 0;
        const long long top = is_dense ? (R - 1) : R;
        while (bits < 31 && (top >> bits) != 0) ++bits;
        g.key_bits = bits;
        g.sentinel = is_dense ? 0x7fffffff : (int)((1LL << bits) - 1);
    } else {
        const long long dx = (long long)((mx[0] - mn[0]) * g.inv_leaf[0]) + 1;
        const long long dy = (long long)((mx[1] - mn[1]) * g.inv_leaf[1]) + 1;
        const long long dz = (long long)((mx[2] - mn[2]) * g.inv_leaf[2]) + 1;
        if (dx * dy * dz > 2147483647LL) {
            g.overflow = 1;
            g.empty = 1;
        } else {
            for (int a = 0; a < 3; ++a) {
                // ndt_cpu VoxelGrid::findBoundaries: floor(max_x_ / voxel_x_) (division); VGC: floor(min * inverse_leaf)
                g.min_b[a] = binning ? (int)floorf(mn[a] / leaf) : (int)floorf(mn[a] * g.inv_leaf[a]);
                g.max_b[a] = binning ? (int)floorf(mx[a] / leaf) : (int)floorf(mx[a] * g.inv_leaf[a]);
                g.div_b[a] = g.max_b[a] - g.min_b[a] + 1;
            }
            g.divb_mul[0] = 1;
            g.divb_mul[1] = g.div_b[0];
            g.divb_mul[2] = g.div_b[0] * g.div_b[1];
            const long long D = (long long)g.div_b[0] * g.div_b[1] * g.div_b[2];
            g.cells = D;
            if (D > 2147483646LL) {
                g.overflow = 1;
                g.empty = 1;
            } else {
                // sentinel (> every valid key) for skipped points of non-dense clouds
                int bits = 0;
                long long top = is_dense ? (D - 1) : D;
                while (bits < 31 && (top >> bits) != 0) ++bits;
                g.key_bits = bits;
                g.sentinel = is_dense ? 0x7fffffff : (int)((1LL << bits) - 1);
            }
        }
    }
    *h = g;
}

// ---------------------------------------------------------------- voxel key per point (binning, :218-223)
// Grid-stride over the points: key + index per point, the digit histograms of every radix pass the key needs
// (LDS counters, then one global add per non-zero counter), and the look-back status words of the sort
// cleared for the onesweep passes.
__device__ __forceinline__ int voxel_key(const float4 p, int is_dense, const GridHeader* __restrict__ h) {
    if (!is_dense && !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) return h->sentinel;
    int ijk0, ijk1, ijk2;
    if (h->binning) {
        // ndt_cpu VoxelGrid::voxelId: floorf(p / voxel) - min_b (integer subtraction)
        ijk0 = (int)floorf(p.x / h->leaf[0]) - h->min_b[0];
        ijk1 = (int)floorf(p.y / h->leaf[1]) - h->min_b[1];
        ijk2 = (int)floorf(p.z / h->leaf[2]) - h->min_b[2];
    } else {
        ijk0 = (int)(floorf(p.x * h->inv_leaf[0]) - (float)h->min_b[0]);
        ijk1 = (int)(floorf(p.y * h->inv_leaf[1]) - (float)h->min_b[1]);
        ijk2 = (int)(floorf(p.z * h->inv_leaf[2]) - (float)h->min_b[2]);
    }
    if (h->layout == 1)
        return ((((ijk2 >> 3) * h->nblk[1] + (ijk1 >> 3)) * h->nblk[0] + (ijk0 >> 3)) << 9) | ((ijk2 & 7) << 6) | ((ijk1 & 7) << 3) |
               (ijk0 & 7);
    return ijk0 * h->divb_mul[0] + ijk1 * h->divb_mul[1] + ijk2 * h->divb_mul[2];
}

// Every workgroup first derives the grid header from k_minmax's partials (a few KB of L2 reads; one launch fewer per sort
// than a separate header kernel), workgroup 0 stores it for the kernels after this one.
// Target builds (grid != nullptr) also choose the lookup structure here — the dense cell grid when the box's cells fit
// its allocation, else the hash table — and clear it (grid-stride over every workgroup), so that no separate set-up
// kernel runs between the scans and the finalize (one launch ~4.7 us, rocprofv3); the hash capacity follows from the
// cloud count in k_cloud_scan.
__global__ __launch_bounds__(kBlock) void k_keys(const float4* __restrict__ pts, int n, int is_dense, const float* __restrict__ part, int nb_mm,
                                                 GridHeader* __restrict__ hout, float leaf, int min_pts, double eig_mult, int layout,
                                                 int binning, int* __restrict__ keys, int* __restrict__ vals,
                                                 int* __restrict__ radix_aux, unsigned* __restrict__ status, int status_words,
                                                 int* __restrict__ grid, long long grid_cap, int2* __restrict__ table, long long table_slots,
                                                 const GridHeader* __restrict__ fold, int val_base) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < status_words; i += gridDim.x * kBlock) status[i] = 0u;
    __shared__ GridHeader s_h;
    __shared__ float s_red[kBlock][7];
    header_body(part, nb_mm, &s_h, leaf, min_pts, eig_mult, is_dense, layout, binning, s_red, fold);
    __syncthreads();
    const bool lookup = grid != nullptr && !s_h.empty;
    const bool dense = lookup && s_h.cells > 0 && s_h.cells <= grid_cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        GridHeader g = s_h;
        g.dense = dense ? 1 : 0;
        *hout = g;
    }
    const GridHeader* h = &s_h;
    if (h->empty) return;
    if (lookup) {
        // 16-byte stores (4 cells / 2 hash slots each): C5's 139 M-cell grid is 557 MB
        const long long words = dense ? s_h.cells : 2 * table_slots;
        const int4 fill = dense ? make_int4(-1, -1, -1, -1) : make_int4(kEmptyKey, 0, kEmptyKey, 0);
        int4* dst = dense ? reinterpret_cast<int4*>(grid) : reinterpret_cast<int4*>(table);
        const long long m4 = words / 4;
        for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < m4; i += (long long)gridDim.x * kBlock) dst[i] = fill;
        if (blockIdx.x == 0 && threadIdx.x < (int)(words - 4 * m4)) {
            int* w = dense ? grid : reinterpret_cast<int*>(table);
            w[4 * m4 + threadIdx.x] = (threadIdx.x & 1) && !dense ? 0 : -1;
        }
    }
    const int passes = (h->key_bits + 7) / 8;
    __shared__ int cnt[4][256];
    for (int q = 0; q < 4; ++q) cnt[q][threadIdx.x] = 0;
    __syncthreads();
    const int stride = gridDim.x * kBlock;
    for (int i0 = blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += 4 * stride) {
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) p[u] = i0 + u * stride < n ? pts[i0 + u * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u * stride;
            if (i >= n) break;
            const int key = voxel_key(p[u], is_dense, h);
            keys[i] = key;
            vals[i] = val_base + i;
            for (int q = 0; q < passes; ++q) atomicAdd(&cnt[q][(key >> (8 * q)) & 255], 1);
        }
    }
    __syncthreads();
    for (int q = 0; q < passes; ++q) {
        const int c = cnt[q][threadIdx.x];
        if (c) atomicAdd(&radix_aux[(blockIdx.x % kRadixCopies) * 1024 + q * 256 + threadIdx.x], c);
    }
}

// ---------------------------------------------------------------- LSD radix sort, 8-bit digits, onesweep
__device__ __forceinline__ bool radix_pass_active(const GridHeader* h, int pass) { return !h->empty && 8 * pass < h->key_bits; }

// Look-back status word of (tile, digit): flag in the top two bits, count below.
constexpr unsigned kStAgg = 1u << 30;   // tile's own count published
constexpr unsigned kStPre = 2u << 30;   // inclusive prefix over tiles 0..tile published
constexpr unsigned kStCnt = (1u << 30) - 1u;
// bounded wait: a lost predecessor ends the pass instead of hanging.  A poll is one agent-scope load (~1 us from MALL) plus
// s_sleep, so 2^15 polls bound a stuck tile to ~30 ms against look-backs that resolve in microseconds; at 2^22 each of the
// four time-outs of C4's 16-queue x 8-stream run waited ~2 s (profiles/r06/c4_queues)
constexpr int kSpinLimit = 1 << 15;

// One pass = one kernel.  Tiles (ITEMS * kBlock keys: 4096 for large sorts, 6144 from 4 M keys, 1024 when the sort has fewer tiles
// than CUs, so that a small sort's per-tile latency is short) are indexed by blockIdx.x (see kScanAgg below for why
// that drains in practice), or by an atomic ticket when `tickets` is set (the build a timed-out look-back re-runs: a
// tile then waits only on tiles that started before it).  Each wave owns ITEMS * 64
// consecutive keys of its tile and ranks them stably with no workgroup barrier: item by item (index order), the
// lanes of one digit find each other with 8 ballots, read the wave's running count of that digit in LDS and the
// group's first lane advances it.  One barrier later, thread = digit turns the per-wave counts into per-wave
// offsets and the tile's count, publishes the count (decoupled look-back status), resolves its exclusive prefix by
// walking back over earlier tiles and adds the global digit base from the histogram of k_keys.  Large tiles are
// first placed in digit order in LDS and leave as one contiguous run of stores per digit; small tiles (~4 keys per
// digit) scatter straight from the ranks.  Output is the same as a hist/scan/scatter pass: bitwise deterministic.
template <int ITEMS>
__global__ __launch_bounds__(kBlock) void k_radix_onesweep(int* __restrict__ k0, int* __restrict__ v0, int* __restrict__ k1,
                                                           int* __restrict__ v1, int n, int pass, const GridHeader* h,
                                                           int* __restrict__ radix_aux, unsigned* __restrict__ status, int nb,
                                                           GridHeader* __restrict__ herr, int last_pass, int tickets) {
    static_assert(kBlock == 256, "thread = digit");
    // the host launches as many passes as it predicts the key needs (the previous grid's width): the last
    // launched pass flags a key that needs more, and the build is re-run with all four (ndt_api.hip align_finish)
    if (pass == last_pass && pass < 3 && blockIdx.x == 0 && threadIdx.x == 0 && radix_pass_active(h, pass + 1))
        atomicOr(&herr->pad[0], kBuildErrPasses);
    if (!radix_pass_active(h, pass)) return;
    const int* kin = (pass & 1) ? k1 : k0;
    const int* vin = (pass & 1) ? v1 : v0;
    int* kout = (pass & 1) ? k0 : k1;
    int* vout = (pass & 1) ? v0 : v1;
    constexpr int NW = kBlock / 64;
    constexpr int TILE = ITEMS * kBlock;
    constexpr bool kStage = ITEMS >= 16;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int shift = 8 * pass;
    __shared__ int s_tile;
    __shared__ int wcnt[NW][256];   // per-wave running digit counts, then per-wave exclusive offsets
    __shared__ int dpos[256];       // per digit: tile-local start (staged) or global position of the tile's first key
    __shared__ int lds_scan[NW];
    __shared__ int s_key[kStage ? TILE : 1];
    __shared__ int s_val[kStage ? TILE : 1];
    if (tid == 0) s_tile = tickets ? atomicAdd(&radix_aux[kRadixCopies * 1024 + pass], 1) : (int)blockIdx.x;
#pragma unroll
    for (int q = 0; q < NW; ++q) wcnt[q][tid] = 0;
    __syncthreads();
    const int tile = s_tile;
    const int base = tile * TILE;
    const int wbase = base + w * (ITEMS * 64);
    int key[ITEMS], val[ITEMS], rk[ITEMS];
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const int i = wbase + r * 64 + lane;
        key[r] = i < n ? kin[i] : 0;
        val[r] = i < n ? vin[i] : 0;
    }
    // A: rank among the wave's earlier keys of the same digit (wave-synchronous LDS: a wave's LDS operations complete
    // in order, the fences only keep the compiler from reordering them)
    const unsigned long long lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
#pragma unroll
    for (int r = 0; r < ITEMS; ++r) {
        const bool valid = wbase + r * 64 + lane < n;
        const int digit = (key[r] >> shift) & 255;
        unsigned long long m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (digit >> b) & 1;
            const unsigned long long bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        const int before = wcnt[w][digit];
        const int below = __popcll(m & lt);
        rk[r] = before + below;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        if (valid && below == 0) wcnt[w][digit] = before + __popcll(m);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
    __syncthreads();
    // B: thread = digit: per-wave exclusive offsets, the tile's count published at once (later tiles' look-back sums it)
    int agg_i = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        const int c = wcnt[q][tid];
        wcnt[q][tid] = agg_i;
        agg_i += c;
    }
    unsigned* st = status + (size_t)pass * nb * 256;
    const unsigned agg = (unsigned)agg_i;
    __hip_atomic_store(&st[(size_t)tile * 256 + tid], (tile == 0 ? kStPre : kStAgg) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int lstart = 0;
    if constexpr (kStage) {
        int ltot;
        lstart = block_exclusive_scan(agg_i, lds_scan, &ltot);  // its barriers also publish the offsets above
        dpos[tid] = lstart;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r)
            if (wbase + r * 64 + lane < n) {
                const int digit = (key[r] >> shift) & 255;
                const int pos = dpos[digit] + wcnt[w][digit] + rk[r];
                s_key[pos] = key[r];
                s_val[pos] = val[r];
            }
    }
    // look back over earlier tiles (stops at the first inclusive prefix), publish the inclusive prefix.  Status words
    // are agent-scope atomics: the per-XCD L2s are not coherent.
    unsigned excl = 0;
    if (tile > 0) {
        // walk back over earlier tiles kLookBack at a time (their status loads in flight together), summing
        // aggregates until the first inclusive prefix; a window stops at the first tile not yet published and is
        // re-read from there
#ifndef NDT_LOOKBACK
#define NDT_LOOKBACK 8
#endif
        constexpr int kLookBack = NDT_LOOKBACK;
        int t = tile - 1;
        int spin = 0;
        for (;;) {
            unsigned wd[kLookBack];
#pragma unroll
            for (int u = 0; u < kLookBack; ++u)
                wd[u] = (t - u >= 0) ? __hip_atomic_load(&st[(size_t)(t - u) * 256 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : kStPre;
            // branch-free over the window (fully unrolled: wd stays in registers): take words while they are published
            // and no inclusive prefix has been taken yet
            bool stop = false, go = true;
            int used = 0;
#pragma unroll
            for (int u = 0; u < kLookBack; ++u) {
                const unsigned f = wd[u] & ~kStCnt;
                const bool take = go && f != 0u;
                excl += take ? (wd[u] & kStCnt) : 0u;
                used += take ? 1 : 0;
                const bool last = take && (f == kStPre || t - u == 0);
                stop = stop || last;
                go = take && !last;
            }
            if (stop) break;
            t -= used;
            if (used < kLookBack) {
                if (++spin > kSpinLimit) { atomicOr(&herr->pad[0], kBuildErrLookback); break; }  // sort_error
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __hip_atomic_store(&st[(size_t)tile * 256 + tid], kStPre | ((excl + agg) & kStCnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // global base of this digit = exclusive scan of the pass histogram
    int tot;
    int dcount = 0;
#pragma unroll
    for (int q = 0; q < kRadixCopies; ++q) dcount += radix_aux[q * 1024 + pass * 256 + tid];
    const int dbase = block_exclusive_scan(dcount, lds_scan, &tot);
    if constexpr (kStage) {
        dpos[tid] = dbase + (int)excl - lstart;
        __syncthreads();
        const int m_tile = min(TILE, n - base);
        for (int j = tid; j < m_tile; j += kBlock) {
            const int k = s_key[j];
            const int pos = dpos[(k >> shift) & 255] + j;
            kout[pos] = k;
            vout[pos] = s_val[j];
        }
    } else {
        dpos[tid] = dbase + (int)excl;
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ITEMS; ++r)
            if (wbase + r * 64 + lane < n) {
                const int digit = (key[r] >> shift) & 255;
                const int pos = dpos[digit] + wcnt[w][digit] + rk[r];
                kout[pos] = key[r];
                vout[pos] = val[r];
            }
    }
}

template __global__ void k_radix_onesweep<4>(int*, int*, int*, int*, int, int, const GridHeader*, int*, unsigned*, int, GridHeader*,
                                                  int, int);
template __global__ void k_radix_onesweep<16>(int*, int*, int*, int*, int, int, const GridHeader*, int*, unsigned*, int, GridHeader*,
                                                  int, int);
template __global__ void k_radix_onesweep<24>(int*, int*, int*, int*, int, int, const GridHeader*, int*, unsigned*, int, GridHeader*,
                                                  int, int);

// n is either the host count or *n_dev when n_dev != nullptr.
__device__ __forceinline__ int scan_n(int n, const int* n_dev) { return n_dev ? *n_dev : n; }

// sorted key / value buffer after the radix passes the key needed (ping-pong); a merged target (h->flip) sits in the
// other one.  sorted_buf_nominal: the radix parity alone (a sort that borrows the target header's key width)
__device__ __forceinline__ const int* sorted_buf_nominal(const GridHeader* h, const int* b0, const int* b1) {
    const int passes = (h->key_bits + 7) / 8;
    return (passes & 1) ? b1 : b0;
}
__device__ __forceinline__ const int* sorted_buf(const GridHeader* h, const int* b0, const int* b1) {
    const int passes = (h->key_bits + 7) / 8;
    return ((passes + h->flip) & 1) ? b1 : b0;
}

// ---------------------------------------------------------------- exclusive scan (int), single pass
// Tile = blockIdx.x.  The command processor hands workgroups to the XCDs round-robin and each XCD dispatches its
// share in increasing ID order, so the lowest unfinished tile is always resident (every lower ID on its XCD has
// finished and freed its slot) and the look-back chain drains; an atomic ticket per tile (sc.tickets, the build a timed-out
// look-back re-runs: a never-reset 64-bit counter, the host passes its value at launch) serialised 4.5k tiles on one
// address and cost C5 ~100 us per build (profiles/r02_s3).  Decoupled look-back over 64-bit status words tagged with a per-launch epoch (so the status array is
// never cleared): [63:32] epoch, [31:30] flag (1 = tile aggregate, 2 = inclusive prefix), [29:0] value.
// The look-back is wave-parallel: lane k reads tile (t-1-k); the window stops at the nearest inclusive prefix.
constexpr unsigned long long kScanAgg = 1ull << 30, kScanPre = 2ull << 30, kScanVal = (1ull << 30) - 1;

// One wave of a tile: publish the tile total, walk back over earlier tiles (lane k reads tile t-1-k; the window
// stops at the nearest inclusive prefix), publish the inclusive prefix.  Returns the exclusive prefix (uniform
// over the wave).  A lost predecessor ends the wait after kSpinLimit polls and raises the header's error flag.
__device__ long long scan_lookback(unsigned long long* __restrict__ status, int tile, int tot, unsigned epoch,
                                   GridHeader* __restrict__ herr) {
    const int lane = threadIdx.x & 63;  // any one wave of the workgroup
    const unsigned long long tag = (unsigned long long)epoch << 32;
    if (lane == 0)
        __hip_atomic_store(&status[tile], tag | (tile == 0 ? kScanPre : kScanAgg) | (unsigned long long)tot, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    long long excl = 0;
    int t = tile - 1;
    int spin = 0;
    while (t >= 0) {
        const int tt = t - lane;
        unsigned long long wd = 0;
        bool ready = true;
        if (tt >= 0) {
            wd = __hip_atomic_load(&status[tt], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = (wd >> 32) == epoch && (wd & (kScanAgg | kScanPre)) != 0;
        }
        const bool pre = tt >= 0 && ready && (wd & kScanPre);
        const unsigned long long pre_mask = __ballot(pre);
        // lanes up to (and including) the first prefix, or the whole window, must be published
        const int stop = pre_mask ? (__ffsll((long long)pre_mask) - 1) : 63;
        const unsigned long long need = (stop == 63) ? ~0ull : ((2ull << stop) - 1);
        const unsigned long long not_ready = __ballot(!ready) & need;
        if (not_ready) {
            if (++spin > kSpinLimit) { if (lane == 0) atomicOr(&herr->pad[0], kBuildErrLookback); break; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        long long v = (tt >= 0 && lane <= stop) ? (long long)(wd & kScanVal) : 0;
        for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
        excl += v;
        if (pre_mask) break;
        t -= 64;
    }
    if (lane == 0 && tile > 0)
        __hip_atomic_store(&status[tile], tag | kScanPre | ((unsigned long long)(excl + tot) & kScanVal), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// tile ticket + block scan + look-back: returns this thread's exclusive prefix of `sum`; *tile_out, *total (last tile)
__device__ __forceinline__ int tile_scan(const ScanCtx& sc, int sum, GridHeader* herr, int* s_tile, int* s_excl, int* lds, int tile,
                                         int* total) {
    int tot;
    const int ex = block_exclusive_scan(sum, lds, &tot);
    if (threadIdx.x < 64) {
        const long long excl = scan_lookback(sc.status, tile, tot, sc.epoch, herr);
        if (threadIdx.x == 0) *s_excl = (int)excl;
    }
    __syncthreads();
    *total = *s_excl + tot;
    return ex + *s_excl;
}

__device__ __forceinline__ int take_ticket(const ScanCtx& sc, int* s_tile) {
    if (threadIdx.x == 0) *s_tile = sc.tickets ? (int)(atomicAdd(sc.ticket, 1ull) - sc.ticket_base) : (int)blockIdx.x;
    __syncthreads();
    return *s_tile;
}

// A tile's ints (plus EXTRA after it) staged through LDS with coalesced loads (consecutive lanes, consecutive words)
// so that each thread can then walk its kTileItems consecutive items from LDS; one pad word per 32 keeps the
// per-thread rows on distinct banks.  first: global index of staged word 0 (may be -1: filled).
constexpr int kStageWords = kTile + 2 + (kTile + 2) / 32 + 1;
__host__ __device__ constexpr int st_idx(int p) { return p + (p >> 5); }
template <int EXTRA>
__device__ __forceinline__ void stage_tile(const int* __restrict__ in, long long first, int n, int fill, int* s) {
    // every load of the thread is issued before the first LDS store (one round trip per tile, not one per word)
    constexpr int R = (kTile + EXTRA + kBlock - 1) / kBlock;
    int v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int p = threadIdx.x + r * kBlock;
        const long long i = first + p;
        v[r] = (p < kTile + EXTRA && i >= 0 && i < n) ? in[i] : fill;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int p = threadIdx.x + r * kBlock;
        if (p < kTile + EXTRA) s[st_idx(p)] = v[r];
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBlock) void k_scan_onepass(const int* __restrict__ in, int n, const int* n_dev, int* __restrict__ out,
                                                         int* __restrict__ total_out, ScanCtx sc, GridHeader* __restrict__ herr) {
    __shared__ int s_tile, s_excl, lds[4];
    __shared__ int s_in[kStageWords];
    const int tile = take_ticket(sc, &s_tile);
    const int nn = scan_n(n, n_dev);
    const int base = tile * kTile + threadIdx.x * kTileItems;
    stage_tile<0>(in, (long long)tile * kTile, nn, 0, s_in);
    int loc[kTileItems];
    int sum = 0;
#pragma unroll
    for (int k = 0; k < kTileItems; ++k) {
        loc[k] = s_in[st_idx(threadIdx.x * kTileItems + k)];
        sum += loc[k];
    }
    int total;
    int ex = tile_scan(sc, sum, herr, &s_tile, &s_excl, lds, tile, &total);
    if (tile == sc.nb - 1 && threadIdx.x == 0 && total_out) *total_out = total;
#pragma unroll
    for (int k = 0; k < kTileItems; ++k) {
        if (base + k < nn) out[base + k] = ex;
        ex += loc[k];
    }
}

// ---------------------------------------------------------------- merge-extended target (odom_node's localmap)
// odom_node sets as target the localmap as it stood before each keyframe's append (odom_node.cpp:233, 349): between two
// localmap resets every target is the previous one plus the points appended since.  Its stable sort by voxel key is then
// the previous target's stable sort — keys re-expressed in the grown box, an order-preserving map of cells — merged with
// the stable sort of the new points alone, old points first on equal keys (their indices are smaller): bitwise the
// radix sort of all points, so the segment scan, cloud scan and finalize that follow give the same grid.  Merge path:
// each workgroup finds where its 2048 outputs start and end in the two sequences (64-way search by one wave per end,
// three rounds for ~10^5 keys), stages both slices in LDS, and each thread merges 8 outputs after a binary search in
// LDS.  Output goes to the ping-pong buffer the previous sort does not occupy (h_new->flip records the swap).
constexpr int kMergeTile = kMergeTileKeys;
constexpr int kMergeItems = kMergeTile / kBlock;

struct KeyRemap {
    int mo1, mo2;          // old layout: key = ix + mo1 * iy + mo2 * iz
    int off[3];            // old min_b - new min_b
    int mn1, mn2;          // new layout
    bool exact;            // both layouts' f32 cell arithmetic exact (|cell| < 2^23): integer remap, else from the point
};

__device__ __forceinline__ int remap_key(const KeyRemap& r, int k, int v, const float4* __restrict__ pts, const GridHeader* __restrict__ hn) {
    if (!r.exact) return voxel_key(pts[v], 1, hn);
    const int iz = k / r.mo2;
    const int rem = k - iz * r.mo2;
    const int iy = rem / r.mo1;
    const int ix = rem - iy * r.mo1;
    return (ix + r.off[0]) + r.mn1 * (iy + r.off[1]) + r.mn2 * (iz + r.off[2]);
}

__global__ __launch_bounds__(kBlock) void k_merge_append(int* __restrict__ k0, int* __restrict__ v0, int* __restrict__ k1,
                                                         int* __restrict__ v1, const GridHeader* __restrict__ ho, int n_old,
                                                         const int* __restrict__ qk0, const int* __restrict__ qv0,
                                                         const int* __restrict__ qk1, const int* __restrict__ qv1, int n_new,
                                                         GridHeader* __restrict__ hn, const float4* __restrict__ pts) {
    if (hn->empty) return;
    const int n = n_old + n_new;
    const int d0 = blockIdx.x * kMergeTile;
    if (d0 >= n) return;
    const int d1 = min(d0 + kMergeTile, n);
    // the previous sort's buffers (after its own merge swap, if any) and the other pair for the output
    const int po = ((ho->key_bits + 7) / 8 + ho->flip) & 1;
    const int* ok = po ? k1 : k0;
    const int* ov = po ? v1 : v0;
    int* wk = po ? k0 : k1;
    int* wv = po ? v0 : v1;
    const int pn = ((hn->key_bits + 7) / 8) & 1;
    const int* qk = pn ? qk1 : qk0;  // the new points' radix sort, nominal parity
    const int* qv = pn ? qv1 : qv0;
    if (blockIdx.x == 0 && threadIdx.x == 0) hn->flip = (po == 0 ? 1 : 0) != pn ? 1 : 0;
    KeyRemap r;
    r.mo1 = ho->divb_mul[1]; r.mo2 = ho->divb_mul[2];
    r.mn1 = hn->divb_mul[1]; r.mn2 = hn->divb_mul[2];
    bool exact = true;
    for (int a = 0; a < 3; ++a) {
        r.off[a] = ho->min_b[a] - hn->min_b[a];
        exact = exact && abs(hn->min_b[a]) < (1 << 23) && abs(hn->max_b[a]) < (1 << 23);
    }
    r.exact = exact;
    // beyond 2^23 the old points' keys are recomputed from the points, and f32 rounding may map two old cells to one new
    // cell out of order: the merge is then not the fresh sort, so the build is flagged and re-run from scratch
    if (!exact && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&hn->pad[0], kBuildErrMerge);
    __shared__ int s_split[2];
    __shared__ int s_k[kMergeTile], s_v[kMergeTile];
    // split of diagonal d: the number of old keys among the first d outputs (old first on ties)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < 2) {
        const int d = w == 0 ? d0 : d1;
        int lo = max(0, d - n_new), hi = min(d, n_old);
        while (lo < hi) {
            const int step = (hi - lo + 63) / 64;
            const int m = lo + lane * step;
            bool t = false;  // old[m] precedes new[d-1-m]
            if (m < hi) t = remap_key(r, ok[m], ov[m], pts, hn) <= qk[d - 1 - m];
            const unsigned long long probed = __ballot(m < hi);
            const unsigned long long fls = __ballot(m < hi && !t);
            if (fls == 0ull) {
                lo = lo + (63 - __clzll((long long)probed)) * step + 1;  // past the last probe
            } else {
                const int f = __ffsll((long long)fls) - 1;
                const int nlo = f == 0 ? lo : lo + (f - 1) * step + 1;
                hi = lo + f * step;
                lo = nlo;
            }
        }
        if (lane == 0) s_split[w] = lo;
    }
    __syncthreads();
    const int a0 = s_split[0], a1 = s_split[1];
    const int la = a1 - a0, b0 = d0 - a0, lb = (d1 - d0) - la;
    for (int i = threadIdx.x; i < la; i += kBlock) {
        const int v = ov[a0 + i];
        s_k[i] = remap_key(r, ok[a0 + i], v, pts, hn);
        s_v[i] = v;
    }
    for (int i = threadIdx.x; i < lb; i += kBlock) {
        s_k[la + i] = qk[b0 + i];
        s_v[la + i] = qv[b0 + i];
    }
    __syncthreads();
    const int dl = threadIdx.x * kMergeItems;
    const int tn = d1 - d0;
    if (dl >= tn) return;
    int lo = max(0, dl - lb), hi = min(dl, la);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_k[mid] <= s_k[la + dl - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int ai = lo, bi = dl - lo;
#pragma unroll
    for (int k = 0; k < kMergeItems; ++k) {
        if (dl + k >= tn) break;
        const bool take_a = ai < la && (bi >= lb || s_k[ai] <= s_k[la + bi]);
        const int src = take_a ? ai : la + bi;
        wk[d0 + dl + k] = s_k[src];
        wv[d0 + dl + k] = s_v[src];
        ai += take_a ? 1 : 0;
        bi += take_a ? 0 : 1;
    }
}

// Segments of the sorted keys (one per occupied voxel) in one pass: head flags from neighbouring keys, their scan,
// seg_start[s] = first sorted position of voxel s, seg_start[n_leaves] = number of binned points; n_leaves -> h.
__global__ __launch_bounds__(kBlock) void k_seg_scan(const int* __restrict__ k0, const int* __restrict__ k1, int n,
                                                     GridHeader* __restrict__ h, int* __restrict__ seg_start, ScanCtx sc) {
    __shared__ int s_tile, s_excl, lds[4];
    __shared__ int s_k[kStageWords];
    const int tile = take_ticket(sc, &s_tile);
    const bool empty = h->empty != 0;
    const int* k = sorted_buf(h, k0, k1);
    const int sentinel = h->sentinel;
    const int base = tile * kTile + threadIdx.x * kTileItems;
    unsigned heads = 0;
    int sum = 0;
    if (!empty) {
        // staged word p = sorted key (tile start - 1 + p): each item's predecessor is the word before it
        stage_tile<1>(k, (long long)tile * kTile - 1, n, 0, s_k);
        int prev = s_k[st_idx(threadIdx.x * kTileItems)];
#pragma unroll
        for (int q = 0; q < kTileItems; ++q) {
            const int i = base + q;
            if (i >= n) break;
            const int key = s_k[st_idx(threadIdx.x * kTileItems + q + 1)];
            if (key != sentinel && (i == 0 || prev != key)) { heads |= 1u << q; ++sum; }
            prev = key;
        }
    }
    int total;
    int ex = tile_scan(sc, sum, h, &s_tile, &s_excl, lds, tile, &total);
#pragma unroll
    for (int q = 0; q < kTileItems; ++q)
        if (heads & (1u << q)) seg_start[ex++] = base + q;
    if (tile == sc.nb - 1 && threadIdx.x == 0) {
        h->n_leaves = total;
        seg_start[total] = empty ? 0 : h->n_points;
    }
}

// Leaves with >= min points (the reference's KD cloud) in ascending key order: flags from the segment sizes, their
// scan, cloud_span[c] = (first, end) sorted position of cloud voxel c (its segment, so that the finalize's first load
// is its point range, not a leaf number to look up); n_cloud -> h.  n = upper bound of the leaf count (host).
// The last tile also completes the header: the hash capacity (next pow2 >= 4 * n_cloud, load <= 1/4, clamped to the
// allocation) and empty when no voxel qualifies.
__global__ __launch_bounds__(kBlock) void k_cloud_scan(const int* __restrict__ seg_start, int n, GridHeader* __restrict__ h,
                                                       int2* __restrict__ cloud_span, ScanCtx sc, unsigned max_log2cap) {
    __shared__ int s_tile, s_excl, lds[4];
    __shared__ int s_seg[kStageWords];
    const int tile = take_ticket(sc, &s_tile);
    const int nl = h->empty ? 0 : h->n_leaves;
    // the grid is sized for the host's upper bound (one leaf per point); tiles past the one holding leaf nl have no
    // leaves and no successor that needs their look-back word: they leave at once.  `last` is the tile of leaf nl - 1
    // (tile 0 when there are none): with one leaf per point and nl a multiple of kTile, nl / kTile is past the grid
    const int last = nl > 0 ? (nl - 1) / kTile : 0;
    if (tile > last) return;
    const int base = tile * kTile + threadIdx.x * kTileItems;
    const int minp = h->min_points;
    unsigned fl = 0;
    int sum = 0;
    stage_tile<1>(seg_start, (long long)tile * kTile, nl + 1, 0, s_seg);
#pragma unroll
    for (int q = 0; q < kTileItems; ++q) {
        const int s = base + q;
        if (s >= nl) break;
        const int p = threadIdx.x * kTileItems + q;
        if (s_seg[st_idx(p + 1)] - s_seg[st_idx(p)] >= minp) { fl |= 1u << q; ++sum; }
    }
    int total;
    int ex = tile_scan(sc, sum, h, &s_tile, &s_excl, lds, tile, &total);
#pragma unroll
    for (int q = 0; q < kTileItems; ++q)
        if (fl & (1u << q)) {
            const int p = threadIdx.x * kTileItems + q;
            cloud_span[ex++] = make_int2(s_seg[st_idx(p)], s_seg[st_idx(p + 1)]);
        }
    if (tile == last && threadIdx.x == 0) {
        h->n_cloud = total;
        unsigned l = 6;
        while (l < max_log2cap && (1LL << l) < 4LL * (long long)total) ++l;
        h->log2cap = l;
        if (total == 0) h->empty = 1;
    }
}

// ---------------------------------------------------------------- segments (one per occupied voxel)





// Per-voxel statistics of one cloud voxel (applyFilter second pass, :282-367) from its point indices idx[b, e)
// in input order.  Points are gathered kGather at a time (all loads in flight, the next chunk's indices loading
// behind them: one round trip per chunk) and accumulated one by one, so every f64 sum has the reference's operation
// order.  Measured: C5 finalize 547 -> 424 us, C2 64 -> 59 us against an index round trip per chunk; 16-point chunks
// or a second chunk of points in flight do not help (more registers, same round trips).  Writes the voxel's records at cloud index ci.
constexpr int kGather = 8;
__device__ __forceinline__ bool leaf_stats(const float4* __restrict__ pts, const int* __restrict__ idx, int b, int e, int ci, int key,
                                           const GridHeader* __restrict__ h, VoxelRec* __restrict__ recs, float4* __restrict__ cent,
                                           double* __restrict__ icovd, int* __restrict__ cloud_key, double* __restrict__ evals_out) {
    const int n = e - b;
    double sum[3] = {0.0, 0.0, 0.0};
    double cov[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};  // Leaf(): cov_ = Identity
    float cen[3] = {0.f, 0.f, 0.f};
    // the next chunk's indices are loaded while this chunk's points are in flight: one round trip per chunk
    int ix[kGather];
#pragma unroll
    for (int k = 0; k < kGather; ++k) ix[k] = (b + k < e) ? idx[b + k] : -1;
    for (int j0 = b; j0 < e; j0 += kGather) {
        float4 q[kGather];
#pragma unroll
        for (int k = 0; k < kGather; ++k) q[k] = ix[k] >= 0 ? pts[ix[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < kGather; ++k) ix[k] = (j0 + kGather + k < e) ? idx[j0 + kGather + k] : -1;
#pragma unroll
        for (int k = 0; k < kGather; ++k) {
            if (j0 + k >= e) break;
            const float4 p = q[k];
            const double pd[3] = {(double)p.x, (double)p.y, (double)p.z};
            sum[0] += pd[0]; sum[1] += pd[1]; sum[2] += pd[2];
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) cov[r + 3 * c] += pd[r] * pd[c];
            cen[0] += p.x; cen[1] += p.y; cen[2] += p.z;
        }
    }
    const float nf = (float)n;
    for (int a = 0; a < 3; ++a) cen[a] /= nf;
    const double nd = (double)n;
    double mean[3];
    for (int a = 0; a < 3; ++a) mean[a] = sum[a] / nd;
    if (h->binning)  // ndt_cpu keeps no float centroid: the exported centroid is the f64 one, narrowed
        for (int a = 0; a < 3; ++a) cen[a] = (float)mean[a];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) cov[r + 3 * c] = (cov[r + 3 * c] - 2 * (sum[r] * mean[c])) / nd + mean[r] * mean[c];
    const double f = (n - 1.0) / n;
    for (int k = 0; k < 9; ++k) cov[k] *= f;
    double ev[3], V[9];
    if (h->binning) aw_sym_eigen3(cov, ev, V);  // ndt_cpu: cpu::SymmetricEigensolver3x3
    else sym_eigen3(cov, ev, V);
    double icov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool rejected = false;
    if (ev[0] < 0 || ev[1] < 0 || ev[2] <= 0) {
        rejected = true;
        ev[0] = ev[1] = ev[2] = 0.0;
    } else {
        const double mce = h->min_eig_mult * ev[2];
        if (ev[0] < mce) {
            ev[0] = mce;
            if (ev[1] < mce) ev[1] = mce;
            double Vi[9];
            inverse3<double>(V, Vi);
            double VD[9];
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) VD[r + 3 * c] = V[r + 3 * c] * ev[c];
            for (int c = 0; c < 3; ++c)
                for (int r = 0; r < 3; ++r) {
                    double acc = VD[r + 0] * Vi[0 + 3 * c];
                    acc += VD[r + 3] * Vi[1 + 3 * c];
                    acc += VD[r + 6] * Vi[2 + 3 * c];
                    cov[r + 3 * c] = acc;
                }
        }
        inverse3<double>(cov, icov);
        // VGC rejects an infinite inverse (voxel_grid_covariance_omp_impl.hpp:359-364); ndt_cpu keeps it
        double mxv = -HUGE_VAL, mnv = HUGE_VAL;
        for (int k = 0; k < 9; ++k) { mxv = fmax(mxv, icov[k]); mnv = fmin(mnv, icov[k]); }
        if (!h->binning && (mxv == HUGE_VAL || mnv == -HUGE_VAL)) rejected = true;
    }
    VoxelRec rec;
    for (int a = 0; a < 3; ++a) rec.mean[a] = mean[a];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) rec.icov[r * 3 + c] = (float)icov[r + 3 * c];
    rec.npts = rejected ? -1 : n;
    recs[ci] = rec;
    cent[ci] = make_float4(cen[0], cen[1], cen[2], 0.f);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) icovd[(size_t)ci * 9 + r * 3 + c] = icov[r + 3 * c];
    cloud_key[ci] = key;
    for (int a = 0; a < 3; ++a) evals_out[(size_t)ci * 3 + a] = ev[a];
    return rejected;
}

// radix-path finalize: one thread per cloud voxel, points = the voxel's segment of the stable sort; the voxel then
// enters the lookup structure (dense cell grid or open-addressing hash, as k_keys chose).  The random read of
// the points in input order is the floor: gathering them into sorted order first (k_sorted_gather, 4 loads in flight
// per thread) costs 430 us alone on C5's 18.7 M points against 534 us for this whole kernel.
// WAVES: the occupancy the register allocation is held to (2: 182 VGPRs; 3: 168 VGPRs + 60 B/lane of scratch).  Measured
// (round 2): C2's 195 k voxels 60.1 -> 55.3 us at 3, C5's 1.8 M voxels 424 -> 442 us; the host picks by target size.
template <int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void k_leaf_finalize(const float4* __restrict__ pts, const int* __restrict__ k0,
                                                          const int* __restrict__ k1, const int* __restrict__ v0,
                                                          const int* __restrict__ v1, const int2* __restrict__ cloud_span,
                                                          GridHeader* __restrict__ h,
                                                          VoxelRec* __restrict__ recs, float4* __restrict__ cent,
                                                          double* __restrict__ icovd, int* __restrict__ cloud_key,
                                                          double* __restrict__ evals_out, int* __restrict__ grid,
                                                          int2* __restrict__ table, int* __restrict__ valid_part) {
    const int ci = blockIdx.x * kBlock + threadIdx.x;
    // the span load is not behind the count test (the buffer holds the whole grid's threads): both in one round trip
    const int2 be = cloud_span[ci];
    if (ci >= h->n_cloud) return;
    const int* keys = sorted_buf(h, k0, k1);
    const int* vals = sorted_buf(h, v0, v1);
    const int b = be.x, e = be.y;
    const int key = keys[b];
    const bool rejected = leaf_stats(pts, vals, b, e, ci, key, h, recs, cent, icovd, cloud_key, evals_out);
    // usable voxels per wave (lane 0 holds the wave's smallest index, active whenever the wave is): no atomics on one
    // counter (3k serialized atomics cost ~35 us); ndt_grid_info sums the ceil(n_cloud/64) wave counts
    const unsigned long long ok = __ballot(!rejected);
    if ((threadIdx.x & 63) == 0) valid_part[ci >> 6] = (int)__popcll(ok);
    const int val = ci | (rejected ? kRejectBit : 0);
    if (h->dense) {
        if (key >= 0 && (long long)key < h->cells) grid[key] = val;
        return;
    }
    const unsigned log2cap = h->log2cap;
    const unsigned mask = (1u << log2cap) - 1u;
    unsigned slot = hash_slot(key, log2cap);
    const unsigned long long empty = (unsigned long long)(unsigned)kEmptyKey;  // (x = -1, y = 0)
    const unsigned long long mine = ((unsigned long long)(unsigned)val << 32) | (unsigned)key;
    unsigned long long* t = reinterpret_cast<unsigned long long*>(table);
    for (;;) {
        const unsigned long long prev = atomicCAS(&t[slot], empty, mine);
        if (prev == empty) return;
        slot = (slot + 1u) & mask;
    }
}






// pcl::VoxelGrid<PointXYZI>::applyFilter second half: per-voxel mean of x,y,z,intensity (downsample_all_data_),
// output ordered by ascending voxel index (odom_node.cpp:334-335).  Points of a voxel are summed in input order.
// Two kernels: the points are first gathered into sorted order (parallel, coalesced writes) so that each voxel's
// serial sum streams one contiguous range instead of chasing indices (dense voxels near the sensor hold hundreds).
__global__ __launch_bounds__(kBlock) void k_sorted_gather(const float4* __restrict__ pts, const int* __restrict__ v0,
                                                          const int* __restrict__ v1, const GridHeader* __restrict__ h,
                                                          float4* __restrict__ sorted, int n) {
    if (h->empty) return;
    const int* vals = sorted_buf(h, v0, v1);
    const int m = min(n, h->n_points);
    // 4 points per thread per round: the index loads, then the 4 independent random point loads, then the stores
    constexpr int U = 4;
    for (int i0 = blockIdx.x * (kBlock * U) + threadIdx.x; i0 < m; i0 += gridDim.x * (kBlock * U)) {
        int v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * kBlock < m ? vals[i0 + u * kBlock] : -1;
        float4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = v[u] >= 0 ? pts[v[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (v[u] >= 0) sorted[i0 + u * kBlock] = q[u];
    }
}

#define NDT_FIN_INST(W)                                                                                                   \
    template __global__ void k_leaf_finalize<W>(const float4*, const int*, const int*, const int*, const int*, const int2*, \
                                                GridHeader*, VoxelRec*, float4*, double*, int*, double*, int*, int2*, int*);
NDT_FIN_INST(2)
NDT_FIN_INST(3)
#undef NDT_FIN_INST

// ---------------------------------------------------------------- source order of an align
// The derivative passes visit the source in the order of the target cells its points fall into under the align's
// initial transform (cells clamped to the grid box): the 7 probes and the voxel records of neighbouring lanes
// then share cache lines.  Per-point arithmetic is unchanged; only the order of the f64 partial sums moves (as
// the reference's OpenMP partition moves it run to run).  Keys + digit histograms here, the radix passes of the
// target build reused (same header: key_bits of the target grid), then k_src_gather.
__global__ __launch_bounds__(kBlock) void k_src_keys(const float4* __restrict__ src, int n, Mat4f Tm, const GridHeader* __restrict__ h,
                                                     int* __restrict__ keys, int* __restrict__ vals, int* __restrict__ radix_aux,
                                                     unsigned* __restrict__ status, int status_words) {
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < status_words; i += gridDim.x * kBlock) status[i] = 0u;
    if (h->empty) return;
    const int passes = (h->key_bits + 7) / 8;
    const float* T = Tm.m;
    __shared__ int cnt[4][256];
    for (int q = 0; q < 4; ++q) cnt[q][threadIdx.x] = 0;
    __syncthreads();
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 p = src[i];
        const float x[3] = {T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12], T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13],
                            T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14]};
        int key = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float f = floorf(x[a] * h->inv_leaf[a]) - (float)h->min_b[a];
            const int c = isfinite(f) ? (int)fminf(fmaxf(f, 0.f), (float)(h->div_b[a] - 1)) : 0;
            key += c * h->divb_mul[a];
        }
        keys[i] = key;
        vals[i] = i;
        for (int q = 0; q < passes; ++q) atomicAdd(&cnt[q][(key >> (8 * q)) & 255], 1);
    }
    __syncthreads();
    for (int q = 0; q < passes; ++q) {
        const int c = cnt[q][threadIdx.x];
        if (c) atomicAdd(&radix_aux[(blockIdx.x % kRadixCopies) * 1024 + q * 256 + threadIdx.x], c);
    }
}

__global__ __launch_bounds__(kBlock) void k_src_gather(const float4* __restrict__ src, const int* __restrict__ v0, const int* __restrict__ v1,
                                                       const GridHeader* __restrict__ h, float4* __restrict__ out, int n) {
    const int* vals = h->empty ? nullptr : sorted_buf_nominal(h, v0, v1);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) out[i] = src[vals ? vals[i] : i];
}

__global__ __launch_bounds__(kBlock) void k_downsample_finalize(const float4* __restrict__ sorted, const int* __restrict__ seg_start,
                                                                const GridHeader* __restrict__ h, float4* __restrict__ out) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (h->empty || s >= h->n_leaves) return;
    const int b = seg_start[s], e = seg_start[s + 1];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int j = b;
    for (; j + 4 <= e; j += 4) {
        const float4 p0 = sorted[j], p1 = sorted[j + 1], p2 = sorted[j + 2], p3 = sorted[j + 3];
        a0 += p0.x; a1 += p0.y; a2 += p0.z; a3 += p0.w;
        a0 += p1.x; a1 += p1.y; a2 += p1.z; a3 += p1.w;
        a0 += p2.x; a1 += p2.y; a2 += p2.z; a3 += p2.w;
        a0 += p3.x; a1 += p3.y; a2 += p3.z; a3 += p3.w;
    }
    for (; j < e; ++j) {
        const float4 p = sorted[j];
        a0 += p.x; a1 += p.y; a2 += p.z; a3 += p.w;
    }
    const float cnt = (float)(e - b);
    out[s] = make_float4(a0 / cnt, a1 / cnt, a2 / cnt, a3 / cnt);
}

// odom_node keyframe insertion (odom_node.cpp:333-338): the VoxelGrid output (or, when the leaf overflowed the
// index range, the transformed input itself, as pcl::VoxelGrid does) appended to two device clouds.
__global__ __launch_bounds__(kBlock) void k_append2(const float4* __restrict__ ds, const float4* __restrict__ raw, int n,
                                                    const GridHeader* __restrict__ h, float4* __restrict__ dst_a, float4* __restrict__ dst_b) {
    const bool overflow = h->overflow != 0;
    const int cnt = overflow ? n : (h->empty ? 0 : h->n_leaves);
    const float4* srcp = overflow ? raw : ds;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < cnt; i += gridDim.x * kBlock) {
        const float4 v = srcp[i];
        dst_a[i] = v;
        dst_b[i] = v;
    }
}

// ================================================================ nearest-neighbour index (getFitnessScore)
// pcl::Registration::getFitnessScore searches a KD tree over ALL target points.  The device index is the
// target binned at the grid resolution (same stable sort as the voxel build): points gathered into leaf
// order, plus the ascending leaf keys and their start offsets.
__global__ __launch_bounds__(kBlock) void k_fit_gather(const float4* __restrict__ pts, const int* __restrict__ k0,
                                                       const int* __restrict__ k1, const int* __restrict__ v0,
                                                       const int* __restrict__ v1, const int* __restrict__ seg_start, int n,
                                                       const GridHeader* __restrict__ h, float4* __restrict__ fit_pts,
                                                       int* __restrict__ fit_keys, int* __restrict__ fit_start) {
    if (h->empty) return;
    const int* keys = sorted_buf(h, k0, k1);
    const int* vals = sorted_buf(h, v0, v1);
    const int nl = h->n_leaves;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        if (i < h->n_points) fit_pts[i] = pts[vals[i]];
        if (i < nl) {
            fit_start[i] = seg_start[i];
            fit_keys[i] = keys[seg_start[i]];
        }
        if (i == 0) fit_start[nl] = seg_start[nl];
    }
}

// Block tables of the index (layout 1): block_table[block] = occupied-block ordinal or -1, and per occupied block
// 513 offsets into the sorted points, one per local cell (z%8, y%8, x%8) plus the block end — so a cell lookup is
// two dependent loads and a block's points are one contiguous range.
__global__ __launch_bounds__(kBlock) void k_fit_block_flags(const int* __restrict__ fit_keys, const GridHeader* __restrict__ h,
                                                            int* __restrict__ flags) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (h->empty || s >= h->n_leaves) return;
    flags[s] = (s == 0 || (fit_keys[s] >> 9) != (fit_keys[s - 1] >> 9)) ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void k_fit_block_clear(int* __restrict__ block_table, const GridHeader* __restrict__ h) {
    const int nb = h->empty ? 0 : (int)(h->cells >> 9);
    for (int b = blockIdx.x * kBlock + threadIdx.x; b < nb; b += gridDim.x * kBlock) block_table[b] = -1;
}

__global__ __launch_bounds__(kBlock) void k_fit_tables(const int* __restrict__ fit_keys, const int* __restrict__ fit_start,
                                                       const int* __restrict__ flags, const int* __restrict__ blk_ex,
                                                       const GridHeader* __restrict__ h, int* __restrict__ block_table,
                                                       int* __restrict__ cell_off) {
    const int s = blockIdx.x * kBlock + threadIdx.x;
    const int nl = h->empty ? 0 : h->n_leaves;
    if (s >= nl) return;
    const int key = fit_keys[s];
    const int occ = blk_ex[s] + flags[s] - 1;
    const int l = key & 511;
    int* off = cell_off + (size_t)occ * (kFitBlockCells + 1);
    if (flags[s]) block_table[key >> 9] = occ;
    const int prev = flags[s] ? -1 : (fit_keys[s - 1] & 511);
    for (int j = prev + 1; j <= l; ++j) off[j] = fit_start[s];
    const bool last = (s + 1 == nl) || flags[s + 1];
    if (last)
        for (int j = l + 1; j <= kFitBlockCells; ++j) off[j] = fit_start[s + 1];
}

// Exact nearest neighbour of each transformed source point (pcl::transformPointCloud in f32) over all target
// points, one 16-lane team per query.  The index is block-major (8x8x8-cell blocks, cells x-fastest inside a block),
// so the cells of an x-row inside one block hold one contiguous range of points: a row of up to 5 cells is at most two
// ranges, found with one block-table load and two offset loads per block.  Search order:
//   phase 1: the 3x3x3 cube around the query cell as 9 x-rows (one per lane), then the 5x5x5 cube as 25 x-rows (its
//     inner cells scanned again: the minimum is idempotent); after the cube of radius r every unvisited point lies in
//     a cell at Chebyshev distance >= r+1, i.e. at least r cells away along some axis (a small slack covers binning
//     round-off), so the team stops once its best squared distance is below that;
//   phase 2 (no point that close): square shells of 8x8x8-cell blocks; each occupied block whose lower bound
//     beats the best is scanned as one contiguous range split over the lanes; after block shell r every unvisited
//     point is at least 8r cells away along some axis.
// Distances are FLANN's L2_Simple in float ((dx^2 + dy^2) + dz^2); the minimum does not depend on the visiting
// order or on the lane split.
#ifndef NDT_FIT_RANGE_U
#define NDT_FIT_RANGE_U 8
#endif
constexpr int kFitTeam = NDT_FIT_TEAM;  // lanes per query (ndt_types.h)
constexpr int kFitBlock = NDT_FIT_BLOCK;  // threads per k_fitness workgroup (ndt_types.h)
constexpr int kFitP2 = 8;  // block-scan loads in flight per lane

__device__ __forceinline__ float team_min(float v) {
    for (int m = kFitTeam / 2; m > 0; m >>= 1) v = fminf(v, __shfl_xor(v, m, kFitTeam));
    return v;
}

__device__ __forceinline__ float l2_simple(const float4 t, const float q[3]) {
    float d = 0.f, u;
    u = t.x - q[0]; d += u * u;
    u = t.y - q[1]; d += u * u;
    u = t.z - q[2]; d += u * u;
    return d;
}

// min over the points [b, e) of the index, four loads in flight (the last point repeated past e: harmless for a
// minimum) instead of one round trip per point (a localmap cell holds one point per keyframe that saw it)
__device__ __forceinline__ float range_min(const float4* __restrict__ pts, int b, int e, const float q[3], float best) {
    constexpr int U = NDT_FIT_RANGE_U;
    for (int j = b; j < e; j += U) {
        float4 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = pts[min(j + u, e - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) best = fminf(best, l2_simple(p[u], q));
    }
    return best;
}

// min over the points of the cells (xa..xb, y, z), 0 <= xa <= xb < xa + 8 inside the grid: at most two blocks
__device__ __forceinline__ float row_min(int xa, int xb, int y, int z, const int nbk[3], const int* __restrict__ block_table,
                                         const int* __restrict__ cell_off, const float4* __restrict__ pts, const float q[3], float best) {
    const int lyz = ((z & 7) << 6) | ((y & 7) << 3);
    const int base = ((z >> 3) * nbk[1] + (y >> 3)) * nbk[0];
    const int bxa = xa >> 3, bxb = xb >> 3;
    const int occ_a = block_table[base + bxa];
    const int occ_b = bxb != bxa ? block_table[base + bxb] : -1;
    int b0 = 0, e0 = 0, b1 = 0, e1 = 0;
    if (occ_a >= 0) {
        const int* off = cell_off + (size_t)occ_a * (kFitBlockCells + 1);
        b0 = off[lyz | (xa & 7)];
        e0 = off[(lyz | (bxb != bxa ? 7 : (xb & 7))) + 1];
    }
    if (occ_b >= 0) {
        const int* off = cell_off + (size_t)occ_b * (kFitBlockCells + 1);
        b1 = off[lyz];
        e1 = off[(lyz | (xb & 7)) + 1];
    }
    best = range_min(pts, b0, e0, q, best);
    return range_min(pts, b1, e1, q, best);
}

// min over up to kFitCells cells of a ring cube (cell k0, k0 + kFitTeam, ...: one lane's share), each level of loads
// (block table, cell offsets, points) issued for all of them before any is consumed
#ifndef NDT_FIT_CELLS
#define NDT_FIT_CELLS 2
#endif
constexpr int kFitCells = NDT_FIT_CELLS;
__device__ __forceinline__ float cells_min(int k0, int ncell, int side, int ring, const int c[3], const int db[3], const int nbk[3],
                                           const int* __restrict__ block_table, const int* __restrict__ cell_off,
                                           const float4* __restrict__ pts, const float q[3], float best) {
    int occ[kFitCells], lc[kFitCells], b[kFitCells], n[kFitCells];
#pragma unroll
    for (int i = 0; i < kFitCells; ++i) {
        const int k = k0 + i * kFitTeam;
        const int x = c[0] + k % side - ring, y = c[1] + (k / side) % side - ring, z = c[2] + k / (side * side) - ring;
        const bool in = k < ncell && x >= 0 && y >= 0 && z >= 0 && x < db[0] && y < db[1] && z < db[2];
        lc[i] = ((z & 7) << 6) | ((y & 7) << 3) | (x & 7);
        occ[i] = in ? block_table[((z >> 3) * nbk[1] + (y >> 3)) * nbk[0] + (x >> 3)] : -1;
    }
    int tot = 0;
#pragma unroll
    for (int i = 0; i < kFitCells; ++i) {
        b[i] = 0;
        n[i] = 0;
        if (occ[i] >= 0) {
            const int* off = cell_off + (size_t)occ[i] * (kFitBlockCells + 1);
            b[i] = off[lc[i]];
            n[i] = off[lc[i] + 1] - b[i];
        }
        tot += n[i];
    }
    // the cells' point ranges walked as one sequence, NDT_FIT_RANGE_U loads in flight (the last point repeated past the end)
    constexpr int U = NDT_FIT_RANGE_U;
    for (int j = 0; j < tot; j += U) {
        float4 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int v = min(j + u, tot - 1);
            int idx = 0;
#pragma unroll
            for (int i = 0; i < kFitCells; ++i) {
                if (v >= 0 && v < n[i]) idx = b[i] + v;
                v -= n[i];
            }
            p[u] = pts[idx];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) best = fminf(best, l2_simple(p[u], q));
    }
    return best;
}

// The per-workgroup (sum, count) partials are summed by the last workgroup to finish (ticket), in a fixed order
// (thread-strided, then a fixed tree), and written straight to the caller's pinned result slots.
// Six waves per SIMD: the search is latency bound (a wave's 4 queries wait on dependent gathers 70 % of the time) and
// 80 VGPRs still need no scratch (C3: 82.8 vs 87.8 us at the default 5 waves; 8 waves spill 76 B/lane, 93 us).
#ifndef NDT_FIT_WAVES
#define NDT_FIT_WAVES 6
#endif
__global__ __launch_bounds__(kFitBlock) __attribute__((amdgpu_waves_per_eu(NDT_FIT_WAVES))) void k_fitness(const float4* __restrict__ src, int n, Mat4f Tm, const GridHeader* __restrict__ h,
                                                    const int* __restrict__ block_table, const int* __restrict__ cell_off,
                                                    const float4* __restrict__ fit_pts, double max_range, float* __restrict__ nn_d2,
                                                    double* __restrict__ part_sum, int* __restrict__ part_cnt,
                                                    unsigned* __restrict__ ticket, double* __restrict__ out_sum,
                                                    long long* __restrict__ out_cnt) {
    const float* T = Tm.m;
    double sum = 0.0;
    int cnt = 0;
    const bool empty = h->empty != 0 || h->n_leaves == 0;
    const int db[3] = {h->div_b[0], h->div_b[1], h->div_b[2]};
    const int nbk[3] = {h->nblk[0], h->nblk[1], h->nblk[2]};
    const float cell = h->leaf[0];
    const int t = threadIdx.x % kFitTeam;
    const int teams = kFitBlock / kFitTeam;
    for (int i = blockIdx.x * teams + threadIdx.x / kFitTeam; i < n; i += gridDim.x * teams) {
        const float4 p = src[i];
        float q[3];
        q[0] = T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12];
        q[1] = T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13];
        q[2] = T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14];
        float best = INFINITY;
        if (!empty) {
            int c[3];
            for (int a = 0; a < 3; ++a) c[a] = (int)(floorf(q[a] * h->inv_leaf[a]) - (float)h->min_b[a]);
            const float slack = 1e-4f * cell + 4e-7f * (fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]));
            int r0 = 0, rmax = 0;
            for (int a = 0; a < 3; ++a) {
                const int out = c[a] < 0 ? -c[a] : (c[a] >= db[a] ? c[a] - db[a] + 1 : 0);
                r0 = max(r0, out);
                rmax = max(rmax, max(c[a], db[a] - 1 - c[a]));
            }
            rmax = max(rmax, r0);
            // distance from the query to the nearest face of its own cell
            float face = cell;
            for (int a = 0; a < 3; ++a) {
                const float lo = (float)(c[a] + h->min_b[a]) * h->leaf[a];
                face = fminf(face, fminf(fmaxf(q[a] - lo, 0.f), fmaxf(lo + h->leaf[a] - q[a], 0.f)));
            }
            bool done = false;
            // ---- phase 1: the cubes of radius 1 (9 x-rows) and 2 (25 x-rows)
            if (r0 <= 2) {
                for (int ring = 1; ring <= 2 && !done; ++ring) {
                    const int side = 2 * ring + 1;
                    // one cell per lane of the team per step (x-rows per lane measured slower: 111 vs 95 us on C3), a
                    // lane's cells NDT_FIT_CELLS at a time: their table, offset and point loads issued together
                    const int ncell = side * side * side;
                    for (int k0 = t; k0 < ncell; k0 += kFitCells * kFitTeam)
                        best = cells_min(k0, ncell, side, ring, c, db, nbk, block_table, cell_off, fit_pts, q, best);
                    best = team_min(best);
                    // every unvisited point lies outside the cube of radius `ring` around the query cell: at least the
                    // query's distance to the nearest cube face away (binning round-off inside the slack)
                    const float bound = fmaxf(0.f, face + (float)ring * cell - slack);
                    done = best <= bound * bound || ring >= rmax;
                }
            }
            // ---- phase 2: block shells, each candidate block's points split over the team
            if (!done) {
                int cb[3], b0 = 0, bmax = 0;
                for (int a = 0; a < 3; ++a) {
                    cb[a] = c[a] >> 3;  // arithmetic shift: floor for cells left of the grid
                    const int out = cb[a] < 0 ? -cb[a] : (cb[a] >= nbk[a] ? cb[a] - nbk[a] + 1 : 0);
                    b0 = max(b0, out);
                    bmax = max(bmax, max(cb[a], nbk[a] - 1 - cb[a]));
                }
                bmax = max(bmax, b0);
                auto visit_block = [&](int x, int y, int z) {
                    const int occ = block_table[((z * nbk[1] + y) * nbk[0]) + x];
                    if (occ < 0) return;
                    // lower bound: per-axis cell gap between the query cell and the block's cells
                    const int bx[3] = {x, y, z};
                    float lb = 0.f;
                    for (int a = 0; a < 3; ++a) {
                        const int lo = bx[a] * 8, hi = lo + 7;
                        const int gap = c[a] < lo ? lo - c[a] - 1 : (c[a] > hi ? c[a] - hi - 1 : 0);
                        const float g = fmaxf(0.f, (float)gap * cell - slack);
                        lb += g * g;
                    }
                    if (lb >= best) return;  // best is team-uniform here
                    const int* off = cell_off + (size_t)occ * (kFitBlockCells + 1);
                    const int e = off[kFitBlockCells];
                    // a block holds up to hundreds of points: eight loads in flight per lane (clamped repeats are
                    // harmless for a minimum), not one round trip per point
                    for (int j = off[0] + t; j < e; j += kFitP2 * kFitTeam) {
                        float4 p[kFitP2];
#pragma unroll
                        for (int u = 0; u < kFitP2; ++u) p[u] = fit_pts[min(j + u * kFitTeam, e - 1)];
#pragma unroll
                        for (int u = 0; u < kFitP2; ++u) best = fminf(best, l2_simple(p[u], q));
                    }
                    best = team_min(best);
                };
                for (int r = b0; r <= bmax; ++r) {
                    const int lo2 = max(cb[2] - r, 0), hi2 = min(cb[2] + r, nbk[2] - 1);
                    const int lo1 = max(cb[1] - r, 0), hi1 = min(cb[1] + r, nbk[1] - 1);
                    const int lo0 = max(cb[0] - r, 0), hi0 = min(cb[0] + r, nbk[0] - 1);
                    for (int z = lo2; z <= hi2; ++z)
                        for (int y = lo1; y <= hi1; ++y) {
                            if (abs(z - cb[2]) == r || abs(y - cb[1]) == r) {
                                for (int x = lo0; x <= hi0; ++x) visit_block(x, y, z);
                            } else {
                                if (cb[0] - r >= 0) visit_block(cb[0] - r, y, z);
                                if (r > 0 && cb[0] + r <= nbk[0] - 1) visit_block(cb[0] + r, y, z);
                            }
                        }
                    const float bound = fmaxf(0.f, (float)(8 * r) * cell - slack);
                    if (best <= bound * bound) break;
                }
            }
        }
        if (t == 0) {
            nn_d2[i] = best;
            if (best != INFINITY && (double)best <= max_range) { sum += (double)best; ++cnt; }
        }
    }
    // (sum, count): workgroup tree -> per-workgroup partial; the last workgroup of each group of kFitGroup sums its
    // group's partials (one load per thread, fixed tree) into a group partial; the last group's reducer sums the
    // group partials (fixed tree) into the caller's pinned result slots.  Hand-offs as in the pass epilogue (recipe
    // R1): partials stored write-through (sc1) and drained before the ticket, the ticket taker acquires — an
    // agent-scope release fence would write back the L2 in each of thousands of workgroups.  One counter per group
    // (own cache line): thousands of increments of one word serialise at its L2 channel.
    __shared__ double s_sum[kFitBlock];
    __shared__ long long s_cnt[kFitBlock];
    __shared__ int s_role;
    auto tree = [&](double v, long long k) {
        s_sum[threadIdx.x] = v;
        s_cnt[threadIdx.x] = k;
        __syncthreads();
        for (int off = kFitBlock / 2; off > 0; off >>= 1) {
            if ((int)threadIdx.x < off) { s_sum[threadIdx.x] += s_sum[threadIdx.x + off]; s_cnt[threadIdx.x] += s_cnt[threadIdx.x + off]; }
            __syncthreads();
        }
    };
    tree(sum, cnt);
    const int nb = gridDim.x;
    const int g = blockIdx.x / kFitGroup, ng = (nb + kFitGroup - 1) / kFitGroup;
    const int g0 = g * kFitGroup, gsize = min(kFitGroup, nb - g0);
    if (threadIdx.x == 0) {
        __hip_atomic_store(part_sum + blockIdx.x, s_sum[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part_cnt + blockIdx.x, (int)s_cnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_role = __hip_atomic_fetch_add(&ticket[kFitTicketStride * (1 + g)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned)gsize - 1;
    }
    __syncthreads();
    if (!s_role) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    {
        const int t = threadIdx.x;
        tree(t < gsize ? part_sum[g0 + t] : 0.0, t < gsize ? (long long)part_cnt[g0 + t] : 0ll);
    }
    if (threadIdx.x == 0) {
        ticket[kFitTicketStride * (1 + g)] = 0u;
        __hip_atomic_store(part_sum + nb + g, s_sum[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part_cnt + nb + g, (int)s_cnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_role = __hip_atomic_fetch_add(&ticket[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)ng - 1 ? 2 : 0;
    }
    __syncthreads();
    if (s_role != 2) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    {
        // more groups than threads: each thread first sums its strided share in ascending order (fixed order)
        double v = 0.0;
        long long k = 0;
        for (int t = threadIdx.x; t < ng; t += kFitBlock) { v += part_sum[nb + t]; k += part_cnt[nb + t]; }
        tree(v, k);
    }
    if (threadIdx.x == 0) {
        // pinned host slots: system-scope stores; a count of -1 reports an index whose sort hit the look-back time limit
        // (the header's error flag: the decoupled look-backs rely on each XCD dispatching its workgroups in order)
        __hip_atomic_store(out_sum, s_sum[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(out_cnt, h->pad[0] ? -1ll : (long long)s_cnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ticket[0] = 0u;
    }
}


}  // namespace ndt
