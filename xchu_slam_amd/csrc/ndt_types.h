// ndt_types.h — device-resident data layouts of the MI355X NDT path.
//
// HBM layout (one ndt_ctx):
//   source      : float4 xyzw  [N]                         (coalesced 16 B/lane loads)
//   target      : float4 xyzw  [M]                         (build input)
//   GridHeader  : 1 record                                 (VGC scalars: min_b/max_b/div_b/divb_mul ...)
//   VoxelRec    : [n_cloud] 64 B, ascending voxel key      (hot record of the derivative pass)
//   cloud_cent  : float4 [n_cloud]                         (float centroid for radius search)
//   cloud_icovd : double[9] [n_cloud]                      (f64 inverse covariance, pcl_ndt / computeHessian)
//   hash table  : int2 (key, cloud index | reject bit)     (open addressing, load <= 1/4)
//   AlignState  : 1 record                                 (device-side Newton / More-Thuente state)
//   partials    : double [44][nblocks]                     (per-workgroup score/g/H/pairs)
#pragma once
#include <stdint.h>

namespace ndt {

constexpr int kBlock = 256;          // threads per workgroup (4 waves of 64)
// derivative-pass workgroups.  The leading-tail chain (k_pass_lead: every workgroup first redoes the previous pass's
// reduction and Newton step) runs one 512-thread workgroup per CU, so that the redundant tails stay one per CU; the
// last-workgroup-tail kernel (k_pass_direct: large clouds, More-Thuente / radius chains, batched replay) runs two
// 256-thread workgroups per CU, whose tile phases (probes, compaction barriers, pair math) drift apart instead of
// running in lockstep (C5 single pass 80.7 -> 73.9 us, tools/pass_micro.py; C2 unchanged).  DIRECT26 keeps one
// 4-wave workgroup per CU (its 26-candidate pair list fills the LDS).
constexpr int kLeadBlock = 512;
// one-tile leading-tail passes (every workgroup's points fit one tile): 768 threads, 12 waves per CU = three per SIMD; with
// split sums and no tile loop the kernel fits 168 VGPRs
constexpr int kLeadBlock1 = 768;
// 1: split sums in the pass kernels (derivatives.hip SplitSink: 22 f64 sums per lane instead of 44)
#ifndef NDT_SPLIT_ACC
#define NDT_SPLIT_ACC 1
#endif
// the one-tile kernel's three-wave register budget needs the split sums
#ifndef NDT_LEAD_ONE_TILE
#define NDT_LEAD_ONE_TILE NDT_SPLIT_ACC
#endif
// 1: last-workgroup-tail passes whose geometry has one tile per workgroup run the one-tile kernel (three waves per SIMD)
#ifndef NDT_DIRECT_ONE_TILE
#define NDT_DIRECT_ONE_TILE 0
#endif
constexpr int kDirectBlock = 256;
// 1: the direct passes' pair arithmetic issued as packed f32 pairs (pair_pk, ndt_pair.h; bitwise the same results)
#ifndef NDT_PACKED_PAIR
#define NDT_PACKED_PAIR 1
#endif
// 1: DIRECT7 passes over a dense grid load the centre row's three cells (0, +x, -x) with one dwordx3 load
#ifndef NDT_ROW_TRIPLE
#define NDT_ROW_TRIPLE 1
#endif
// 1: DIRECT7 passes keep each source point's cell and probe results across the passes of an align (neighbour cache)
#ifndef NDT_NBR_CACHE
#define NDT_NBR_CACHE 1
#endif
__host__ __device__ constexpr int pass_block(int search, bool lead, bool one_tile = false) {
    return search == 1 /*DIRECT26*/ ? kBlock : (lead ? (one_tile ? kLeadBlock1 : kLeadBlock) : kDirectBlock);
}
// waves per SIMD the register allocation of one-point-per-thread k_pass_direct (DIRECT7 / DIRECT1) is held to: 2, or 3
// with split accumulation (its tile state spills around the pair loop, the pair loop itself stays in registers); the
// two-points-per-thread tiles hold 77 KB of LDS, two workgroups per CU, and stay at 2
#ifndef NDT_PASS_WAVES
#define NDT_PASS_WAVES 2
#endif
// one_tile: a one-point-per-thread geometry with one tile per workgroup (no tile loop: the split sums are not live across
// the probes) runs three waves per SIMD
__host__ __device__ constexpr int pass_waves(int search, int ppt, bool one_tile = false) {
    return search == 1 ? 1 : (ppt == 2 ? 2 : (one_tile ? 3 : NDT_PASS_WAVES));
}
// k_pass_direct workgroups (4 waves) per CU: one per wave slot of a SIMD
__host__ __device__ constexpr int pass_wgs_per_cu(int search, bool lead, int ppt, bool one_tile = false) {
    return (search == 1 || lead) ? 1 : pass_waves(search, ppt, one_tile);
}
constexpr int kNumAcc = 44;          // score + g[6] + H[36] + pairs
constexpr int kEmptyKey = -1;        // empty hash slot
constexpr int kRejectBit = 0x40000000;  // cloud leaf rejected by eigen/inf tests (nr_points = -1)
// per-pass partials are [kNumAcc][partial_stride(nblocks)] doubles: rows 16-byte aligned for paired loads
__host__ __device__ constexpr int partial_stride(int nb) { return (nb + 1) & ~1; }
constexpr int kMaxHistory = 4096;
// pass tickets (re-armed by the last workgroup; reset at every align start): word 0 the pass's ticket, then the group
// tickets of the two-level hand-off (grids of more than kTwoLevelMinBlocks workgroups: kMaxGroups groups, one ticket per
// kGroupTicketStride words, i.e. its own 128-byte line)
constexpr int kMaxGroups = 64;
constexpr int kGroupTicketStride = 32;
constexpr int kGroupTicketBase = 16;
constexpr int kPassCounterWords = kGroupTicketBase + kMaxGroups * kGroupTicketStride;
constexpr int kTwoLevelMinBlocks = 1024;
// group partials of the two-level hand-off: [kNumAcc][kMaxGroups] doubles after the [kNumAcc][partial_stride(nb)] ones
__host__ __device__ constexpr int group_size(int nb) { return nb / kMaxGroups >= 64 ? (nb + kMaxGroups - 1) / kMaxGroups : 64; }
// profiling stamps per pass (s_memrealtime, 100 MHz): [0] start(min), [1] end(max), [2] last body done(max),
// [3] tail acquired, [4] tail reduced, [6] state staged in LDS, [7] control step done, [5] next pass prepared
constexpr int kTsStride = 16;
// radix sort auxiliaries: kRadixCopies copies of the [4 digit positions][256] global digit counts (workgroup b of the key
// kernel adds into copy b % kRadixCopies, so that fewer workgroups contend for one counter; the passes sum the copies)
// + 4 tile tickets (ticket-ordered passes)
constexpr int kRadixCopies = 8;
constexpr int kRadixAuxWords = kRadixCopies * 4 * 256 + 4;

enum PassKind { PASS_FULL = 0, PASS_GRAD = 1, PASS_HESS = 2 };
enum SearchMode { S_KDTREE = 0, S_DIRECT26 = 1, S_DIRECT7 = 2, S_DIRECT1 = 3 };

// a 4x4 f32 transform (column-major, as Eigen::Matrix4f) passed to kernels by value
struct Mat4f {
    float m[16];
};

struct GridHeader {
    int min_b[4], max_b[4], div_b[4], divb_mul[4];
    float leaf[4], inv_leaf[4];
    float minp[4], maxp[4];
    int n_points;       // points binned (finite)
    int n_leaves;       // occupied voxels (std::map size)
    int n_cloud;        // leaves with >= min points (KD cloud)
    int n_valid;        // leaves usable by DIRECT search
    int overflow;       // dx*dy*dz > INT32_MAX  -> empty grid
    int empty;          // no usable grid
    int key_bits;       // significant bits of the voxel key (radix passes)
    int sentinel;       // key of skipped (non-finite) points
    unsigned log2cap;   // hash capacity = 1 << log2cap
    int min_points;
    double min_eig_mult;
    long long cells;    // div_b[0]*div_b[1]*div_b[2]
    int dense;          // 1: dense cell grid lookup (cells <= grid allocation), 0: hash lookup
    int pad[2];         // pad[0]: build error bits (kBuildErr*), pad[1]: the front end's kept count
    int binning;        // 0: pclomp VGC (ijk = floor(x * inv_leaf) - min_b); 1: ndt_cpu VoxelGrid (floorf(x / leaf) - min_b)
    // nearest-neighbour index layout (getFitnessScore): 0 = row-major voxel key (voxel grid, VoxelGrid filter);
    // 1 = block-major key ((block index) << 9 | z%8 << 6 | y%8 << 3 | x%8) over 8x8x8-cell blocks, so that every
    // block's points are contiguous after the sort
    int layout;
    int n_blocks_occ;   // layout 1: occupied blocks
    int nblk[4];        // layout 1: blocks per axis
    // 1: the sorted keys / indices sit in the other ping-pong buffer than the radix passes' parity says (a target grid
    // extended by merge, k_merge_append); 0 for every header header_body makes
    int flip;
    int pad2;
};
// GridHeader::pad[0] bits: the build ran but its sort may be wrong, and is re-run (ndt_api.hip align_finish)
constexpr int kBuildErrLookback = 1;  // a decoupled look-back timed out (a predecessor tile not resident): re-run with tickets
constexpr int kBuildErrPasses = 2;    // the key needs more radix passes than were launched: re-run with all four
constexpr int kBuildErrMerge = 4;     // a merge-extended build beyond the exact cell remap (|cell| >= 2^23): re-run fresh
constexpr int kMergeTileKeys = 2048;                   // outputs per workgroup of k_merge_append
constexpr int kFitBlockCells = 512;                    // 8 x 8 x 8 cells per block
// threads per k_fitness workgroup (a workgroup ends with its slowest query: one wave keeps a far query from holding three)
#ifndef NDT_FIT_BLOCK
#define NDT_FIT_BLOCK 64
#endif
// lanes per getFitnessScore query (k_fitness team)
#ifndef NDT_FIT_TEAM
#define NDT_FIT_TEAM 16
#endif
static_assert(NDT_FIT_BLOCK >= 64, "k_fitness: a group's partials are reduced one per thread");
constexpr int kFitGroup = 64;                          // k_fitness workgroups per first-level ticket
constexpr int kFitTicketStride = 64;                   // words between ticket counters (own cache lines / channels)
constexpr long long kFitMaxKeys = 1LL << 25;           // key range cap of layout 1 (cells doubled until it fits)
constexpr int kFitMaxBlocks = (int)(kFitMaxKeys / kFitBlockCells);

// Hot per-voxel record: f64 mean (x' = float(x_trans - mean) exactly as ndt_omp_impl.hpp:260,500)
// and the f32 inverse covariance (c_inv.cast<float>(), :502), full 3x3 row-major.
struct __attribute__((aligned(16))) VoxelRec {
    double mean[3];
    float icov[9];
    int npts;
};
static_assert(sizeof(VoxelRec) == 64, "VoxelRec must be 64 B");

// single-pass scan launch context (voxel_build.hip): look-back words, the monotone tile ticket and its value at
// launch, the launch's epoch tag, the tile count
struct ScanCtx {
    unsigned long long* status;
    unsigned long long* ticket;
    unsigned long long ticket_base;
    unsigned epoch;
    int nb;
    int tickets;   // 1: tiles taken by the atomic ticket instead of blockIdx.x (a build re-run after a look-back timeout)
};

struct PassRecordDev {
    int kind, newton_iter;
    double x[6];
    double score;
    double g[6];
    double H[36];
    long long pairs;
};

struct AlignState {
    // ---- constants of this align ----
    double gauss_d1, gauss_d2, gauss_d3;
    double step_max, step_min, trans_eps;
    int max_iter, n_src, search, precision;
    int mt_possible;   // step_max <= step_min: More-Thuente inner loop may run (ndt_omp_impl.hpp:807)
    float radius;      // radiusSearch radius = resolution_ (ndt_omp_impl.hpp:233,583)
    // ---- Newton state (computeTransformation) ----
    double p[6];
    double score, g[6], H[36];
    int nr_iterations, converged, done, phase;  // phase 0 = initial pass pending
    // ---- More-Thuente state (computeStepLengthMT) ----
    double dir[6], x_t[6];
    double phi_0, d_phi_0;
    double a_l, f_l, g_l, a_u, f_u, g_u, a_t;
    double phi_t, d_phi_t, psi_t, d_psi_t;
    int open_interval, interval_converged, step_iterations;
    int want_solve;    // a Newton solve of H dp = -g is requested (run wave-parallel by the control workgroup)
    // ---- next pass ----
    int pending, pass_kind, solver_fallbacks, needs_tables;
    int needs_svd, svd_ready;          // degenerate Newton system: the chain pauses for k_svd_resume
    int partials_pending;              // leading-tail chain: the previous kernel left a pass's partials to consume
    int build_error;                   // the target build this align runs against raised its look-back error flag (k_align_init)
    double svd_dp[6];
    float T[16];        // final_transformation_ (col-major) = transform of the next / last pass
    float jang[8][4];   // computeAngleDerivatives f32 tables (ndt_omp.h:470, :483)
    float hang[16][4];
    double jang_d[8][3];
    double hang_d[15][3];
    double x_eval[6];   // parameters of the next pass (for the history)
    // ---- outputs ----
    double trans_probability;
    int n_passes, hist_count;
    long long pairs_total;
    long long grid_cells;   // cells of the target grid this align ran against (k_align_init): sizes later dense grids
};

}  // namespace ndt
