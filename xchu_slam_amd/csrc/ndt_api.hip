// ndt_api.hip — C-ABI (include/ndt_hip.h) of the MI355X NDT library.
//
// Host-side mirror of pclomp::NormalDistributionsTransform's registration surface
// (ndt_omp.h:70-497 + pcl::Registration::align): setInputTarget -> device voxel build,
// setInputSource -> device copy, align -> device-resident Newton chain captured in a hipGraph.
// The host only prepares the initial state (guess -> p0, exactly ndt_omp_impl.hpp:89-104 in f32),
// launches, and reads back one small result record: one synchronisation per align.
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include <cstring>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cmath>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <shared_mutex>
#include <thread>

#include "../../include/ndt_hip.h"
#include "ndt_types.h"
#include "ndt_linalg.h"

namespace ndt {
// kernels (defined in the other translation units)
__global__ void k_minmax(const float4*, int, int, float*, int*, unsigned long long*, const GridHeader*, GridHeader*, float4*);
__global__ void k_keys(const float4*, int, int, const float*, int, GridHeader*, float, int, double, int, int, int*, int*, int*, unsigned*, int,
                       int*, long long, int2*, long long, const GridHeader*, int);
__global__ void k_merge_append(int*, int*, int*, int*, const GridHeader*, int, const int*, const int*, const int*, const int*, int,
                               GridHeader*, const float4*);
template <int ITEMS>
__global__ void k_radix_onesweep(int*, int*, int*, int*, int, int, const GridHeader*, int*, unsigned*, int, GridHeader*, int, int);
__global__ void k_scan_onepass(const int*, int, const int*, int*, int*, ScanCtx, GridHeader*);
__global__ void k_seg_scan(const int*, const int*, int, GridHeader*, int*, ScanCtx);
__global__ void k_cloud_scan(const int*, int, GridHeader*, int2*, ScanCtx, unsigned);

template <int WAVES>
__global__ void k_leaf_finalize(const float4*, const int*, const int*, const int*, const int*, const int2*, GridHeader*,
                                VoxelRec*, float4*, double*, int*, double*, int*, int2*, int*);
__global__ void k_sorted_gather(const float4*, const int*, const int*, const GridHeader*, float4*, int);
__global__ void k_src_keys(const float4*, int, Mat4f, const GridHeader*, int*, int*, int*, unsigned*, int);
__global__ void k_src_gather(const float4*, const int*, const int*, const GridHeader*, float4*, int);
__global__ void k_crop_flags(const float4*, int, double, double, int*);
__global__ void k_compact4(const float4*, const int*, const int*, int, float4*);
template <int C>
__global__ void k_sor_knn(const float4*, int, int, const GridHeader*, const int*, const int*, const float4*, float*);
__global__ void k_sor_stats(const float*, int, double, double*);
__global__ void k_sor_keep(const float*, int, const double*, int*);
__global__ void k_ror_keep(const float4*, int, double, int, const GridHeader*, const int*, const int*, const float4*, int*);
__global__ void k_downsample_finalize(const float4*, const int*, const GridHeader*, float4*);
__global__ void k_fit_gather(const float4*, const int*, const int*, const int*, const int*, const int*, int, const GridHeader*, float4*,
                             int*, int*);
__global__ void k_fit_block_flags(const int*, const GridHeader*, int*);
__global__ void k_append2(const float4*, const float4*, int, const GridHeader*, float4*, float4*);
__global__ void k_fit_block_clear(int*, const GridHeader*);
__global__ void k_fit_tables(const int*, const int*, const int*, const int*, const GridHeader*, int*, int*);
__global__ void k_fitness(const float4*, int, Mat4f, const GridHeader*, const int*, const int*, const float4*, double, float*, double*,
                          int*, unsigned*, double*, long long*);
__global__ void k_score_radius(const float4*, int, Mat4f, const GridHeader*, const int2*, const int*, const VoxelRec*, const float4*,
                               const double*, double, double, double, float, double*);
template <int SEARCH, int PPT, bool ONE_TILE>
__global__ void k_pass_direct(const float4*, int, int, const GridHeader*, const int2*, const int*, const VoxelRec*, const AlignState*,
                              AlignState*, double*, unsigned*, double*, PassRecordDev*, int, int, unsigned long long*, int4*);
__global__ void k_pass_radius(const float4*, int, const GridHeader*, const int2*, const int*, const VoxelRec*, const float4*,
                              const double*, const AlignState*, AlignState*, double*, unsigned*, double*, PassRecordDev*, int, int,
                              unsigned long long*);
__global__ void k_transform(const float4*, int, const AlignState*, float4*);
__global__ void k_transform_mat(const float4*, int, Mat4f, float4*);
__global__ void k_align_init(const AlignState, AlignState*, unsigned*, unsigned long long*, int, unsigned long long*, const GridHeader*,
                             unsigned long long, const uint4*, uint4*, long long);
__global__ void k_copy16(const uint4*, uint4*, size_t);
__global__ void k_readback(const unsigned long long*, unsigned long long*, int, const unsigned long long*, unsigned long long*, int,
                           const unsigned long long*, unsigned long long*, int, const unsigned long long*, unsigned long long*,
                           unsigned long long*, unsigned long long, unsigned long long*, const GridHeader*);
hipError_t dbg_read_blk(unsigned long long* host, size_t count);
__global__ void k_svd_resume(AlignState*);
template <int SEARCH, bool ONE_TILE>
__global__ void k_pass_lead(const float4*, int, int, const GridHeader*, const int2*, const int*, const VoxelRec*, const AlignState*,
                            AlignState*, const double*, double*, PassRecordDev*, int, unsigned long long*, int4*);
}  // namespace ndt

using namespace ndt;

namespace {

constexpr int kTileKeys = kBlock * 16;

template <typename T> struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;
};

struct Scratch {
    DevBuf<int> k0, v0, k1, v1, radix_aux, seg_start, flags, cloud_idx;
    DevBuf<int2> cloud_span;
    DevBuf<unsigned> radix_status;
    DevBuf<float> mm;
    DevBuf<float4> sorted_pts;   // points gathered into voxel order (VoxelGrid filter)
    DevBuf<unsigned long long> scan_status;   // single-pass scan look-back words (epoch-tagged, never cleared)
    DevBuf<unsigned long long> scan_ticket;   // monotone tile ticket of the single-pass scan
    unsigned long long scan_tickets = 0;      // host copy of the ticket counter
    unsigned scan_epoch = 0;
};

// Where a sort / scan runs: a stream and the scratch its kernels own (radix buffers, look-back words).  The ctx's
// main stream owns ndt_ctx::s; getFitnessScore (index build + query) and the keyframe insertion run on side lanes with
// scratch of their own, so that odom_node's per-scan tail overlaps the main stream's target build and align (C3).
struct Lane {
    hipStream_t st;
    Scratch& s;
};

// On a side lane's host thread: where fail() puts the error text (the ctx's error string belongs to the caller's thread)
thread_local std::string* tl_err = nullptr;

// The host thread of a side lane: the lane's launches (a sort is ~13 kernels, ~4 us of host time each) are issued from
// it in FIFO order, so the caller only records a main-stream marker and posts the job.  A job's failure is kept until
// the lane's result call (take_error).
struct LaneWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv_job, cv_idle;
    std::deque<std::function<ndt_status()>> jobs;
    int pending = 0;
    bool stop = false;
    ndt_status st = NDT_OK;  // first failure not yet taken
    std::string msg;
    int device = 0;
    std::shared_mutex* capture_mu;  // the ctx's align-graph capture lock, held shared while a job runs (see ndt_ctx::capture_mu)

    LaneWorker(int dev, std::shared_mutex* cap) : device(dev), capture_mu(cap) { th = std::thread([this] { run(); }); }
    ~LaneWorker() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv_job.notify_one();
        th.join();
    }
    void post(std::function<ndt_status()> f) {
        {
            std::lock_guard<std::mutex> g(mu);
            jobs.push_back(std::move(f));
            ++pending;
        }
        cv_job.notify_one();
    }
    // waits until every posted job has been issued; returns the pending failure (kept)
    ndt_status drain(std::string* err) {
        std::unique_lock<std::mutex> g(mu);
        cv_idle.wait(g, [this] { return pending == 0; });
        if (st != NDT_OK && err) *err = msg;
        return st;
    }
    // a job failed and its failure has not been taken yet (non-blocking)
    bool failed() {
        std::lock_guard<std::mutex> g(mu);
        return st != NDT_OK;
    }
    ndt_status take_error(std::string* err) {
        const ndt_status s = drain(err);
        std::lock_guard<std::mutex> g(mu);
        st = NDT_OK;
        return s;
    }
    void run() {
        (void)hipSetDevice(device);
        std::string local;
        tl_err = &local;
        for (;;) {
            std::function<ndt_status()> f;
            bool skip;
            {
                std::unique_lock<std::mutex> g(mu);
                cv_job.wait(g, [this] { return stop || !jobs.empty(); });
                if (jobs.empty()) return;  // stopped, nothing left
                f = std::move(jobs.front());
                jobs.pop_front();
                // after a failure the jobs queued behind it are dropped until take_error: they would launch on buffers the
                // failed job left unbuilt (e.g. a getFitnessScore query on an index whose allocation failed)
                skip = st != NDT_OK;
            }
            local.clear();
            ndt_status s = NDT_OK;
            if (!skip) {
                std::shared_lock<std::shared_mutex> g(*capture_mu);
                s = f();
            }
            {
                std::lock_guard<std::mutex> g(mu);
                if (s != NDT_OK && st == NDT_OK) {
                    st = s;
                    msg = local;
                }
                --pending;
            }
            cv_idle.notify_all();
        }
    }
};

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }



}  // namespace

// Exact nearest-neighbour index over a cloud (block-major binning, layout 1 of k_header): the points sorted into
// 8x8x8-cell blocks, a block table and per-occupied-block cell offsets.
struct NNIndex {
    GridHeader* hdr = nullptr;          // binning (device)
    DevBuf<float4> pts;                 // points in (block, cell) order
    DevBuf<int> keys, start;            // per occupied cell: key, first point
    DevBuf<int> blk, off;               // block table + per-occupied-block cell offsets
};

struct ndt_ctx {
    ndt_params prm{};
    int device = 0;
    int n_cu = 256;  // compute units the main stream's passes spread over (direct-pass grid)
    // CU partition (NDT_LANE_CUS, A/B): the side lanes run on lane_mask's CUs, the main stream on the others
    std::vector<uint32_t> lane_mask;
    hipStream_t stream = nullptr;
    std::string err;
    // target grid
    DevBuf<float4> target;            // owned copy for host-provided targets
    const float4* target_ptr = nullptr;  // points the build reads (owned copy or the caller's device buffer)
    int M = 0;
    int target_dense = 1;
    bool has_target = false;
    bool grid_valid = false;
    float grid_res = 0.f;
    GridHeader* d_hdr = nullptr;
    GridHeader* d_hdr_ds = nullptr;
    GridHeader* d_hdr_fe = nullptr;  // the filter's compaction scans: pad[0] look-back timeout flag, pad[1] kept count
    NNIndex fit_ix;                     // nearest-neighbour index over the target (getFitnessScore)
    NNIndex sor_ix;                     // nearest-neighbour index over a filtered scan (StatisticalOutlierRemoval)
    DevBuf<int> fit_cnt;
    DevBuf<unsigned> fit_ticket;        // last-workgroup ticket of k_fitness (re-armed by that workgroup)
    // asynchronous getFitnessScore / keyframe insertion: results land in pinned memory, an event marks them
    struct AsyncOut {
        double fit_sum;
        long long fit_cnt;
        GridHeader ins_hdr;
        int fe_words[4];  // ndt_filter_scan_device: [0] scan flag, [1] scan count, [2] outlier index sort flag
    };
    AsyncOut* d_async = nullptr;
    AsyncOut* h_async = nullptr;        // pinned
    hipEvent_t ev_fit = nullptr, ev_ins = nullptr;
    bool fit_pending = false, ins_pending = false;
    // side lanes (created on first use): fit_stream runs getFitnessScore's index build and query, ins_stream the
    // keyframe insertion, each issued by its own host thread.  ev_tgt marks (main stream) the current target's points in
    // place — recorded ahead of each build, the index build waits on it, not on the voxel build; ev_main_* are the
    // main-stream markers a side-lane job waits on; ev_fit_src / ev_fit_tgt mark (fit_stream) the end of the last query
    // that read the ctx's source / of the last index build that read the ctx's target points (main waits on them
    // before it rewrites what the index or query read)
    hipStream_t fit_stream = nullptr, ins_stream = nullptr;
    LaneWorker* fit_worker = nullptr;   // host threads issuing the side lanes' launches
    LaneWorker* ins_worker = nullptr;
    Scratch s_fit, s_ins;
    GridHeader* d_hdr_ins = nullptr;    // keyframe insertion's VoxelGrid binning
    hipEvent_t ev_tgt = nullptr, ev_main_fit = nullptr, ev_main_ins = nullptr, ev_fit_src = nullptr, ev_fit_tgt = nullptr;
    int lanes_marked = 0;  // ndt_side_lanes_mark: bit 0 the next fitness query, bit 1 the next insertion use ev_main_fit as is
    bool fit_src_used = false, fit_tgt_used = false;
    // held exclusively while the main stream captures an align graph and shared while a lane thread runs a job: a stream
    // wait issued by a lane thread during the capture is rejected by the runtime ("dependency created on uncaptured
    // work"), and the lanes' allocations (hipMalloc / hipFree on growth) stay out of it too; the two lanes issue side by
    // side
    std::shared_mutex capture_mu;
    int fit_n = 0;                      // source points of the last query
    size_t ins_n_in = 0;
    DevBuf<float4> ins_tr, ins_ds;      // keyframe insertion scratch (transformed scan, VoxelGrid output)
    DevBuf<double> fit_sum;
    DevBuf<float> fit_d2;
    bool fit_valid = false;             // index matches the current target
    GridHeader* h_hdr = nullptr;  // pinned
    bool tgt_ev_valid = false;  // ev_tgt marks the current target (recorded by build_target once the fit lane is in use)
    Scratch s;
    // merge-extended targets (ndt_set_target_append_device): the new points' sort scratch, the previous header, and whether
    // s's sorted keys / indices and d_hdr still describe the current target (no other main-stream sort since its build)
    Scratch s_inc;
    GridHeader* d_hdr_prev = nullptr;
    bool inc_ok = false;
    // target-build robustness (GridHeader::pad[0] bits, checked by the align read-back or settle_build): radix passes
    // launched = the key width of the last grid read back, +1 bit of margin (radix_pred; 4 until a grid was seen);
    // radix_force (ndt_set_build_options test hook) fixes the count; tile_tickets (sticky once a look-back timed out, or
    // set by the hook) takes every sort's tiles by atomic ticket; counters for ndt_build_stats
    int radix_pred = 4, radix_force = 0;
    bool tile_tickets = false;
    bool build_unchecked = false;   // a target build queued whose error bits no align / settle_build has read yet
    bool rerun_full = false;        // a re-run build: all four radix passes whatever the prediction or the hook says
    float al_guess[16] = {0};       // the guess of the align in flight (re-run after a flagged build)
    int al_berr = 0;                // build error bits the align's read-back found (align_finish_once)
    long long n_builds_full = 0, n_builds_merge = 0, n_builds_rerun = 0, n_rerun_lookback = 0;
    // target generations (one per setInputTarget): of the current target, of the one the fit index was last queued
    // for, and of the one the last align result belongs to (ndt_fitness_score_async_aligned)
    unsigned long long tgt_gen = 0, fit_ix_gen = ~0ull, align_tgt_gen = ~0ull;
    DevBuf<VoxelRec> recs;
    DevBuf<float4> cent;
    DevBuf<double> icovd, evals;
    DevBuf<int> cloud_key;
    DevBuf<int> valid_part;             // usable-voxel count per finalize wave (summed by ndt_grid_info)
    DevBuf<int2> table;
    unsigned max_log2cap = 6;
    DevBuf<int> grid;                   // dense cell -> cloud index grid (used when the bbox fits)
    long long grid_cells_seen = 0;      // largest target cell count read back (align, single pass, grid info): sizes the grid
    // source
    DevBuf<float4> source;
    int N = 0;
    bool has_source = false;
    const float4* src_pend = nullptr;   // ndt_set_source_device's copy, deferred to the next align (its k_align_init) or flush_source
    // source in target-cell order for the passes of an align (k_src_keys): the cloud the pass kernels read
    DevBuf<float4> source_ord;
    DevBuf<int> ord_k0, ord_v0, ord_k1, ord_v1;
    const float4* pass_src = nullptr;
    bool order_source = true;
    // pass-chain options (ndt_set_pass_options): leading-tail chains where an align is latency-bound, two points per
    // thread in large last-workgroup-tail passes
    bool opt_lead_tail = true;
    int opt_ppt = 2;
    // filter_node front end (ndt_filter_scan): scratch + the last call's SOR statistics
    DevBuf<int> fe_flags, fe_idx;
    DevBuf<float4> fe_in, fe_crop, fe_ds, fe_out;
    DevBuf<float> fe_dist;
    DevBuf<double> fe_thr;
    size_t fe_nvox = 0;
    // align
    AlignState* d_state = nullptr;
    // leading-tail chains (k_pass_lead): the second state / partials buffer of the ping-pong and the parity of the next
    // kernel of the align in flight (kernel j reads state j & 1, writes state (j + 1) & 1, writes partials j & 1)
    AlignState* d_state2 = nullptr;
    int lead = 0, lead_par = 0;
    bool no_lead = false;  // batched replay: several aligns in flight share the CUs, the redundant tails would cost CU time
    AlignState* h_state = nullptr;  // pinned (coherent), written by k_readback
    // read-back words (pinned, coherent): [0] sequence number of the last finished round, [1..2] device clock of the
    // align's start / that round's end (100 MHz); d_clk[0]: the start stamp k_align_init takes
    unsigned long long* h_rb = nullptr;
    unsigned long long* d_clk = nullptr;
    unsigned long long rb_seq = 0, al_seq = 0;
    DevBuf<double> partials;
    DevBuf<double> partials2;  // leading-tail chains: the other partials buffer
    DevBuf<int4> nbr;                   // DIRECT7 neighbour cache of the align's source points (2 x int4 per point)
    DevBuf<double> score_part;          // calculateScore per-workgroup partial sums
    // gauss_d1_/d2_/d3_ as the reference holds them: set by the constructor for resolution 1.0 / outlier 0.55
    // (ndt_omp_impl.hpp:46-63) and recomputed at the start of every align (:80-87); calculateScore reads them
    double gauss_cur[3] = {0.0, 0.0, 0.0};
    DevBuf<double> reduce_out;
    DevBuf<unsigned> counter;           // last-workgroup ticket of the pass epilogue (re-armed by the last workgroup)
    PassRecordDev* d_hist = nullptr;
    int hist_cap = kMaxHistory;
    DevBuf<float4> out_cloud;
    DevBuf<unsigned long long> ts;      // per-pass kTsStride s_memrealtime stamps (profiling)
    double prof_phase_sum[7] = {0, 0, 0, 0, 0, 0, 0};
    int prof_phase_count = 0;
    double prof_body_sum[5] = {0, 0, 0, 0, 0};
    int prof_body_count = 0;
    double prof_tail_sum[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    int prof_tail_count = 0;
    unsigned long long* h_ts = nullptr;  // pinned copies, filled by k_readback before the align's sync
    PassRecordDev* h_hist = nullptr;
    int h_prof_cap = 0;
    bool have_result = false;
    // graph cache: a few captured chains (different slot counts / buffers), round-robin replacement
    static constexpr int kGraphKey = 23;
    static constexpr int kGraphCache = 64;
    struct GraphEntry {
        hipGraphExec_t exec = nullptr;
        long long key[kGraphKey] = {0};
    };
    GraphEntry graphs[kGraphCache];  // scans of a few neighbouring size buckets (geom_points) x both lead parities
    int graph_next = 0;
    int last_passes = 0;                // passes of the previous align: sizes the first graph round of the next
    // timing
    bool built_since_align = false;  // ms_build: a target build was queued since the last align
    std::vector<hipEvent_t> pass_ev;
    bool profiling = false;
    double ms_build = 0, ms_align = 0, ms_pass_avg = 0, pass_bytes_avg = 0;
    double prof_ms_sum = 0, prof_bytes_sum = 0;
    long long prof_count = 0;
    std::vector<PassRecordDev> last_hist;
    // align in flight (align_enqueue -> align_finish)
    bool al_inflight = false, al_mt = false;
    int al_full = 0, al_slots = 0;
    // helper contexts of the batched replay (one stream each), created on first use
    std::vector<ndt_ctx*> helpers;
};

namespace {

ndt_status fail(ndt_ctx* c, ndt_status st, const std::string& msg) {
    if (tl_err) *tl_err = msg;  // a side lane's host thread: reported by the lane's result call
    else if (c) c->err = msg;
    return st;
}

Lane main_lane(ndt_ctx* c) { return Lane{c->stream, c->s}; }

#define HIPCHK(ctx, expr)                                                                       \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return fail(ctx, NDT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

template <typename T> ndt_status ensure(ndt_ctx* c, DevBuf<T>& b, size_t n) {
    if (n == 0) n = 1;
    if (b.cap >= n) return NDT_OK;
    const size_t want = std::max(n, b.cap + b.cap / 2);
    if (b.p) HIPCHK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
    if (hipMalloc(&b.p, want * sizeof(T)) != hipSuccess) {
        b.p = nullptr;
        return fail(c, NDT_ENOMEM, "hipMalloc failed");
    }
    b.cap = want;
    return NDT_OK;
}

template <typename T> void release(DevBuf<T>& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
}

#define TRY(expr)                          \
    do {                                   \
        ndt_status _s = (expr);            \
        if (_s != NDT_OK) return _s;       \
    } while (0)

// the side lanes (fit_stream / ins_stream), created on the first side-lane call, at the lowest stream priority (the
// main stream, whose target build and align are the scan loop's critical path, has the highest)
ndt_status side_lanes(ndt_ctx* c) {
    if (c->fit_stream) return NDT_OK;
    int least = 0, greatest = 0;
    HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
    if (!c->lane_mask.empty()) {
        HIPCHK(c, hipExtStreamCreateWithCUMask(&c->fit_stream, (uint32_t)c->lane_mask.size() * 32, c->lane_mask.data()));
        HIPCHK(c, hipExtStreamCreateWithCUMask(&c->ins_stream, (uint32_t)c->lane_mask.size() * 32, c->lane_mask.data()));
    } else {
        HIPCHK(c, hipStreamCreateWithPriority(&c->fit_stream, hipStreamNonBlocking, least));
        HIPCHK(c, hipStreamCreateWithPriority(&c->ins_stream, hipStreamNonBlocking, least));
    }
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_main_fit, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_main_ins, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fit_src, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_fit_tgt, hipEventDisableTiming));
    if (hipMalloc(&c->d_hdr_ins, sizeof(GridHeader)) != hipSuccess) return fail(c, NDT_ENOMEM, "hipMalloc failed");
    c->fit_worker = new LaneWorker(c->device, &c->capture_mu);
    c->ins_worker = new LaneWorker(c->device, &c->capture_mu);
    return NDT_OK;
}

// the main stream continues after the fit-lane work that reads what it is about to rewrite: the last query that read the
// ctx's source (source = true) or the last index build that read the ctx's target points (source = false)
// Device copy on `stream` by k_copy16 when both pointers and the size are 16-byte aligned, else a runtime copy
ndt_status copy16(ndt_ctx* c, hipStream_t stream, void* dst, const void* src, size_t bytes) {
    if (!bytes) return NDT_OK;
    if (((uintptr_t)dst | (uintptr_t)src | bytes) & 15) {
        HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream));
        return NDT_OK;
    }
    const size_t n = bytes / 16;
    const int nb = (int)std::min<size_t>(std::max<size_t>(1, (n + kBlock - 1) / kBlock), 1024);
    hipLaunchKernelGGL(k_copy16, dim3(nb), dim3(kBlock), 0, stream, reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n);
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

// The deferred source copy (ndt_set_source_device), issued now on the ctx stream for a reader other than an align
ndt_status flush_source(ndt_ctx* c) {
    if (!c->src_pend) return NDT_OK;
    const float4* p = c->src_pend;
    c->src_pend = nullptr;
    if (c->N) TRY(copy16(c, c->stream, c->source.p, p, (size_t)c->N * sizeof(float4)));
    return NDT_OK;
}

ndt_status main_after_fit(ndt_ctx* c, bool source) {
    if (!(source ? c->fit_src_used : c->fit_tgt_used)) return NDT_OK;
    std::string msg;
    // every queued fit-lane launch issued; a failure is reported here and cleared (it would otherwise block every later
    // target / source change), and the index it may have left unbuilt is dropped
    const ndt_status st = c->fit_worker->take_error(&msg);
    if (st != NDT_OK) {
        c->fit_valid = false;
        c->fit_pending = false;
        return fail(c, st, "getFitnessScore: " + msg);
    }
    HIPCHK(c, hipStreamWaitEvent(c->stream, source ? c->ev_fit_src : c->ev_fit_tgt, 0));
    return NDT_OK;
}

bool valid_params(const ndt_params* p) {
    return p && p->resolution > 0.f && std::isfinite(p->resolution) && p->max_iter >= 0 && p->search >= 0 && p->search <= 3 &&
           p->min_points_per_voxel >= 1 && p->precision_mode >= 0 && p->precision_mode <= 2;
}

// Drops every cached chain; a chain may still be in flight on the stream, so the stream is waited for first (see build_graph)
void invalidate_graph(ndt_ctx* c) {
    bool any = false;
    for (auto& g : c->graphs) any = any || g.exec;
    if (any && c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& g : c->graphs) {
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
        g.exec = nullptr;
    }
}

// launch context of one single-pass scan over nb tiles (look-back words grown and zeroed on demand; the epoch tag
// makes words of earlier launches stale, so they are never cleared again)
ndt_status scan_ctx(ndt_ctx* c, Lane L, int nb, ScanCtx* sc) {
    sc->tickets = c->tile_tickets ? 1 : 0;
    if ((size_t)nb > L.s.scan_status.cap) {
        TRY(ensure(c, L.s.scan_status, (size_t)nb));
        HIPCHK(c, hipMemsetAsync(L.s.scan_status.p, 0, L.s.scan_status.cap * sizeof(unsigned long long), L.st));
    }
    if (!L.s.scan_ticket.p) {
        TRY(ensure(c, L.s.scan_ticket, 1));
        HIPCHK(c, hipMemsetAsync(L.s.scan_ticket.p, 0, sizeof(unsigned long long), L.st));
        L.s.scan_tickets = 0;
    }
    sc->status = L.s.scan_status.p;
    sc->ticket = L.s.scan_ticket.p;
    sc->ticket_base = L.s.scan_tickets;
    sc->epoch = ++L.s.scan_epoch;
    sc->nb = nb;
    // the device counter advances only in ticket mode (each of the nb tiles takes one): the host copy must follow it
    // exactly, or a ctx switched to tickets after a look-back timeout computes negative tiles from a stale base
    if (sc->tickets) L.s.scan_tickets += (unsigned long long)nb;
    return NDT_OK;
}

// exclusive scan of n ints (n_dev optional device count), total written to total_out (device, optional):
// one single-pass kernel (decoupled look-back; a timed-out look-back raises herr's error flag)
ndt_status enqueue_scan(ndt_ctx* c, Lane L, const int* in, int n_host, const int* n_dev, int* out, int* total_out, GridHeader* herr) {
    const int nb = std::max(1, ceil_div(n_host, kTileKeys));
    ScanCtx sc;
    TRY(scan_ctx(c, L, nb, &sc));
    hipLaunchKernelGGL(k_scan_onepass, dim3(nb), dim3(kBlock), 0, L.st, in, n_host, n_dev, out, total_out, sc, herr);
    return NDT_OK;
}

// Radix tile size (keys per thread) for a sort of n keys: 16 (4096-key tiles) when there are at least as many tiles
// as CUs, else 4 (1024-key tiles: 4x the workgroups for a small sort); 24 (6144-key tiles, 24 keys per digit run of the
// staged scatter instead of 16) from 4 M keys: C5's 18.7 M-key target sort 117 -> 111 us per pass, while C2's ~2 M-key
// sorts lose 2 % with it (32: 256 VGPRs, one wave per SIMD, 156 us).
constexpr int kRadixWideKeys = 4 << 20;
int radix_items(const ndt_ctx* c, int n) {
    return ceil_div(n, kTileKeys) < c->n_cu ? 4 : (n >= kRadixWideKeys ? 24 : 16);
}
void launch_radix_pass(const ndt_ctx* c, Lane L, int items, int nb, int* k0, int* v0, int* k1, int* v1, int n, int pass,
                       const GridHeader* h, GridHeader* herr, int last_pass = 3) {
    auto* kern = items == 4 ? k_radix_onesweep<4> : items == 16 ? k_radix_onesweep<16> : k_radix_onesweep<24>;
    hipLaunchKernelGGL(kern, dim3(nb), dim3(kBlock), 0, L.st, k0, v0, k1, v1, n, pass, h, L.s.radix_aux.p, L.s.radix_status.p, nb,
                       herr, last_pass, c->tile_tickets ? 1 : 0);
}

// Radix passes a main-stream sort against the target grid launches (target build, merge-extended build, source order):
// a key of b bits needs ceil(b / 8); the host does not know b before the build ran (the box is reduced on the device), so
// it launches what the last grid read back needed with one bit of margin (radix_pred) — the fourth pass of C2's 23-bit
// keys was an empty launch (~5.5 us per build).  A key wider than predicted is flagged by the last launched pass and the
// build re-run with four (align_finish / settle_build).
int radix_launch_passes(const ndt_ctx* c) {
    if (c->rerun_full) return 4;
    return c->radix_force > 0 ? std::min(c->radix_force, 4) : c->radix_pred;
}
void note_grid_width(ndt_ctx* c, long long cells, int dense) {
    if (cells <= 0) return;
    const long long top = dense ? cells - 1 : cells;
    int bits = 0;
    while (bits < 31 && (top >> bits) != 0) ++bits;
    c->radix_pred = std::min(4, std::max(1, (bits + 1 + 7) / 8));
}

// keys -> stable sort -> segments on header h; leaves h->n_leaves, seg_start, sorted buffers
// cloud_span (target build): the cloud voxels' (>= min points) point ranges in ascending key order as well (k_cloud_scan)
// cloud_span != nullptr: the target build (lookup structure chosen and cleared by k_keys, header completed by k_cloud_scan)
ndt_status enqueue_bin_and_sort(ndt_ctx* c, Lane L, const float4* pts, int n, int dense, GridHeader* h, float leaf, int layout = 0,
                                int binning = 0, int2* cloud_span = nullptr, int passes = 4) {
    if (&L.s == &c->s && !cloud_span) c->inc_ok = false;  // another main-stream sort overwrites the target's sorted keys
    const int nb_mm = std::max(1, std::min(ceil_div(n, 4 * kBlock), 1024));  // k_minmax: four points per thread per round
    TRY(ensure(c, L.s.mm, (size_t)nb_mm * 7));
    // small sorts (fewer 4096-key tiles than CUs) use 1024-key tiles: 4x the workgroups, a quarter of the latency
    const int items = radix_items(c, n);
    const int nb_sort = std::max(1, ceil_div(n, kBlock * items));
    // a target's sorted keys / indices get a quarter of headroom: a merge-extended target (enqueue_target_append) reads the
    // previous sort in place and needs room for the grown one
    const size_t n_kv = cloud_span ? (size_t)n + (size_t)n / 4 : (size_t)n;
    TRY(ensure(c, L.s.k0, n_kv)); TRY(ensure(c, L.s.v0, n_kv)); TRY(ensure(c, L.s.k1, n_kv)); TRY(ensure(c, L.s.v1, n_kv));
    TRY(ensure(c, L.s.radix_aux, kRadixAuxWords));
    TRY(ensure(c, L.s.radix_status, (size_t)4 * 256 * nb_sort));
    TRY(ensure(c, L.s.seg_start, (size_t)n + 1));
    // min/max partials (and the digit histograms cleared), then keys: every keys workgroup derives the header itself
    hipLaunchKernelGGL(k_minmax, dim3(nb_mm), dim3(kBlock), 0, L.st, pts, n, dense, L.s.mm.p, L.s.radix_aux.p,
                       cloud_span ? c->d_clk + 3 : nullptr, nullptr, nullptr, nullptr);
    const int nb_keys = std::max(1, std::min(ceil_div(n, 4 * kBlock), 512));
    hipLaunchKernelGGL(k_keys, dim3(nb_keys), dim3(kBlock), 0, L.st, pts, n, dense, L.s.mm.p, nb_mm, h, leaf, c->prm.min_points_per_voxel,
                       c->prm.min_covar_eigvalue_mult, layout, binning, L.s.k0.p, L.s.v0.p, L.s.radix_aux.p, L.s.radix_status.p,
                       4 * 256 * nb_sort, cloud_span ? c->grid.p : nullptr, (long long)c->grid.cap, cloud_span ? c->table.p : nullptr,
                       1LL << c->max_log2cap, nullptr, 0);
    for (int pass = 0; pass < passes; ++pass)
        launch_radix_pass(c, L, items, nb_sort, L.s.k0.p, L.s.v0.p, L.s.k1.p, L.s.v1.p, n, pass, h, h, passes - 1);
    const int nb_seg = std::max(1, ceil_div(n, kTileKeys));
    ScanCtx sc;
    TRY(scan_ctx(c, L, nb_seg, &sc));
    hipLaunchKernelGGL(k_seg_scan, dim3(nb_seg), dim3(kBlock), 0, L.st, L.s.k0.p, L.s.k1.p, n, h, L.s.seg_start.p, sc);
    if (cloud_span) {
        ScanCtx sc2;
        TRY(scan_ctx(c, L, nb_seg, &sc2));
        hipLaunchKernelGGL(k_cloud_scan, dim3(nb_seg), dim3(kBlock), 0, L.st, L.s.seg_start.p, n, h, cloud_span, sc2, c->max_log2cap);
    }
    return NDT_OK;
}

// VoxelGrid means of the points binned on h: gather into voxel order, then one serial sum per voxel
ndt_status enqueue_downsample_finalize(ndt_ctx* c, Lane L, const GridHeader* h, const float4* in, int n, float4* out) {
    TRY(ensure(c, L.s.sorted_pts, std::max(n, 1)));
    const int nb = std::max(1, std::min(ceil_div(n, 4 * kBlock), 2048));  // four points per thread per round
    hipLaunchKernelGGL(k_sorted_gather, dim3(nb), dim3(kBlock), 0, L.st, in, L.s.v0.p, L.s.v1.p, h, L.s.sorted_pts.p, n);
    hipLaunchKernelGGL(k_downsample_finalize, dim3(std::max(1, ceil_div(n, kBlock))), dim3(kBlock), 0, L.st, L.s.sorted_pts.p,
                       L.s.seg_start.p, h, out);
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

// dense grid: grown lazily to twice the largest cell count seen (capped at 1 Gi cells = 4 GiB)
ndt_status grow_grid(ndt_ctx* c) {
    const long long want_cells = std::min<long long>(std::max<long long>(2 * c->grid_cells_seen, 16ll << 20), 1ll << 30);
    if ((long long)c->grid.cap < want_cells) TRY(ensure(c, c->grid, (size_t)want_cells));
    return NDT_OK;
}

ndt_status alloc_cloud_buffers(ndt_ctx* c, size_t max_cloud) {
    TRY(ensure(c, c->recs, max_cloud)); TRY(ensure(c, c->cent, max_cloud)); TRY(ensure(c, c->icovd, max_cloud * 9));
    TRY(ensure(c, c->evals, max_cloud * 3)); TRY(ensure(c, c->cloud_key, max_cloud));
    return NDT_OK;
}

constexpr int kFinalize3WavesMaxPoints = 4 << 20;

// Target buffers for M points: records, lookup structure, cloud spans; returns the finalize's workgroup count.
ndt_status prepare_target_buffers(ndt_ctx* c, int M, int* nb_cloud) {
    TRY(grow_grid(c));
    const size_t max_cloud = std::max(1, M / std::max(1, c->prm.min_points_per_voxel) + 1);
    TRY(alloc_cloud_buffers(c, max_cloud));
    unsigned l = 6;
    while (l < 30 && (1ull << l) < 4ull * max_cloud) ++l;
    c->max_log2cap = l;
    TRY(ensure(c, c->table, (size_t)1 << l));
    *nb_cloud = std::max(1, ceil_div((long long)max_cloud, kBlock));
    TRY(ensure(c, c->s.cloud_span, (size_t)*nb_cloud * kBlock));  // every finalize thread loads its entry
    TRY(ensure(c, c->valid_part, max_cloud / 64 + 1));
    return NDT_OK;
}

// one thread per cloud voxel: moments, eigen inflation, inverse, and its lookup entry
ndt_status launch_finalize(ndt_ctx* c, int M, int nb_cloud) {
    // three waves per SIMD below ~4 M target points (C2 / C3 localmaps), two above (C5: the larger register file wins)
    auto* fin = M < kFinalize3WavesMaxPoints ? k_leaf_finalize<3> : k_leaf_finalize<2>;
    hipLaunchKernelGGL(fin, dim3(nb_cloud), dim3(kBlock), 0, c->stream, c->target_ptr, c->s.k0.p, c->s.k1.p, c->s.v0.p,
                       c->s.v1.p, c->s.cloud_span.p, c->d_hdr, c->recs.p, c->cent.p, c->icovd.p, c->cloud_key.p,
                       c->evals.p, c->grid.p, c->table.p, c->valid_part.p);
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

ndt_status enqueue_target_build(ndt_ctx* c) {
    c->inc_ok = false;
    ++c->n_builds_full;
    const int M = c->M;
    int nb_cloud = 0;
    TRY(prepare_target_buffers(c, M, &nb_cloud));
    // precision_mode 2 (ndt_cpu) bins like cpu::VoxelGrid (division), the others like pclomp's VGC (multiplication)
    // keys, sort, segments and the cloud voxels (>= min points) in key order; then the lookup structure chosen and
    // cleared, then the finalize
    TRY(enqueue_bin_and_sort(c, main_lane(c), c->target_ptr, M, c->target_dense, c->d_hdr, c->prm.resolution, 0, c->prm.precision_mode == 2 ? 1 : 0,
                             c->s.cloud_span.p, radix_launch_passes(c)));
    TRY(launch_finalize(c, M, nb_cloud));
    // a pclomp grid over a dense cloud can be extended by merge (its sorted keys / indices stay in c->s)
    c->inc_ok = c->prm.precision_mode != 2 && c->target_dense == 1 && M > 0;
    return NDT_OK;
}

// The target grown by n_new points appended after its n_old (k_merge_append): the new points' min/max (the current
// header saved and its box folded in), their keys in the grown box and their radix sort (own scratch), the merge with
// the current sort, then the same segment scan, cloud scan and finalize as a full build.  Bitwise the grid of
// enqueue_target_build over the n_old + n_new points.
ndt_status enqueue_target_append(ndt_ctx* c, int n_old, int n_new, const float4* new_src) {
    const int M = n_old + n_new;
    int nb_cloud = 0;
    TRY(prepare_target_buffers(c, M, &nb_cloud));
    Lane Q{c->stream, c->s_inc};
    // new_src: the new points are read there and stored after the old ones by k_minmax (no separate copy launch)
    float4* copy_to = new_src ? const_cast<float4*>(c->target_ptr) + n_old : nullptr;
    const float4* pts_new = new_src ? new_src : c->target_ptr + n_old;
    const int nq = std::max(n_new, 1);
    const int nb_mm = std::max(1, std::min(ceil_div(nq, 4 * kBlock), 1024));
    TRY(ensure(c, Q.s.mm, (size_t)nb_mm * 7));
    const int items = radix_items(c, nq);
    const int nb_sort = std::max(1, ceil_div(nq, kBlock * items));
    TRY(ensure(c, Q.s.k0, nq)); TRY(ensure(c, Q.s.v0, nq)); TRY(ensure(c, Q.s.k1, nq)); TRY(ensure(c, Q.s.v1, nq));
    TRY(ensure(c, Q.s.radix_aux, kRadixAuxWords));
    TRY(ensure(c, Q.s.radix_status, (size_t)4 * 256 * nb_sort));
    TRY(ensure(c, c->s.seg_start, (size_t)M + 1));
    hipLaunchKernelGGL(k_minmax, dim3(nb_mm), dim3(kBlock), 0, c->stream, pts_new, n_new, 1, Q.s.mm.p, Q.s.radix_aux.p, c->d_clk + 3,
                       c->d_hdr, c->d_hdr_prev, copy_to);
    // the target's points are all in place now: getFitnessScore's index (fit lane) may start beside the rest
    if (c->tgt_ev_valid) HIPCHK(c, hipEventRecord(c->ev_tgt, c->stream));
    // k_keys also clears the grown target's lookup structure (its whole dense grid or hash table): sized for that as well
    // as for the new points, capped as in a full build
    const long long clear_words = std::max<long long>((long long)c->grid.cap, 2LL << c->max_log2cap) / 4;
    const int nb_keys = std::max(1, (int)std::min<long long>(std::max<long long>(ceil_div(nq, 4 * kBlock), ceil_div(clear_words, 4LL * kBlock)), 512));
    hipLaunchKernelGGL(k_keys, dim3(nb_keys), dim3(kBlock), 0, c->stream, pts_new, n_new, 1, Q.s.mm.p, nb_mm, c->d_hdr, c->prm.resolution,
                       c->prm.min_points_per_voxel, c->prm.min_covar_eigvalue_mult, 0, 0, Q.s.k0.p, Q.s.v0.p, Q.s.radix_aux.p,
                       Q.s.radix_status.p, 4 * 256 * nb_sort, c->grid.p, (long long)c->grid.cap, c->table.p, 1LL << c->max_log2cap,
                       c->d_hdr_prev, n_old);
    const int passes = radix_launch_passes(c);
    for (int pass = 0; pass < passes; ++pass)
        launch_radix_pass(c, Q, items, nb_sort, Q.s.k0.p, Q.s.v0.p, Q.s.k1.p, Q.s.v1.p, n_new, pass, c->d_hdr, c->d_hdr, passes - 1);
    hipLaunchKernelGGL(k_merge_append, dim3(std::max(1, ceil_div(M, kMergeTileKeys))), dim3(kBlock), 0, c->stream, c->s.k0.p, c->s.v0.p,
                       c->s.k1.p, c->s.v1.p, c->d_hdr_prev, n_old, Q.s.k0.p, Q.s.v0.p, Q.s.k1.p, Q.s.v1.p, n_new, c->d_hdr,
                       c->target_ptr);
    const Lane L = main_lane(c);
    const int nb_seg = std::max(1, ceil_div(M, kTileKeys));
    ScanCtx sc, sc2;
    TRY(scan_ctx(c, L, nb_seg, &sc));
    hipLaunchKernelGGL(k_seg_scan, dim3(nb_seg), dim3(kBlock), 0, c->stream, c->s.k0.p, c->s.k1.p, M, c->d_hdr, c->s.seg_start.p, sc);
    TRY(scan_ctx(c, L, nb_seg, &sc2));
    hipLaunchKernelGGL(k_cloud_scan, dim3(nb_seg), dim3(kBlock), 0, c->stream, c->s.seg_start.p, M, c->d_hdr, c->s.cloud_span.p, sc2,
                       c->max_log2cap);
    TRY(launch_finalize(c, M, nb_cloud));
    return NDT_OK;
}

// No stream events around the build unless getFitnessScore's index uses them: an event recorded between two kernels leaves
// the stream idle ~6 us (rocprofv3, C2 step).  The build's time comes from device stamps (k_minmax's start .. the align's
// k_align_init, read back with the align), the largest grid seen from the align state (grid_cells).
ndt_status build_target(ndt_ctx* c) {
    ++c->tgt_gen;
    // the target's points are in place: getFitnessScore's index (fit lane) may start beside the build
    c->tgt_ev_valid = c->fit_tgt_used;
    if (c->tgt_ev_valid) HIPCHK(c, hipEventRecord(c->ev_tgt, c->stream));
    TRY(enqueue_target_build(c));
    c->build_unchecked = true;
    c->built_since_align = true;
    c->grid_valid = true;
    c->fit_valid = false;
    c->grid_res = c->prm.resolution;
    c->have_result = false;
    return NDT_OK;
}

int pass_blocks(int n) { return std::max(1, std::min(ceil_div(n, kBlock), 2048)); }

// The point count a pass chain's launch geometry is built for: the scan's size rounded up to 1/64 of its power of two
// (<= ~1.6 % more points per workgroup), at least a multiple of 256.  The pass kernels take the real count from the align state, so one
// captured chain serves every scan of the bucket: odom_node's filtered scans change size every frame, and a chain
// re-captured per align cost ~50 us (4 k points, 11 passes: 0.226 vs 0.178 ms per align).  Source buffers hold at least
// this many points (the kernels prefetch up to it).
int geom_points(int n) {
    if (n <= 4096) return std::max(256, ceil_div(n, 256) * 256);
    int p = 1;
    while (p * 2 <= n) p *= 2;
    const int step = p / 64;
    return ceil_div(n, step) * step;
}

// Direct-pass geometry: one workgroup per CU (fewer for small clouds), each taking `rounds` tiles of ppb points
// (ppb <= the workgroup size) so every CU carries the same share of the scan.
struct PassGeom {
    int nb, ppb, block;
};
PassGeom direct_geom(const ndt_ctx* c, bool lead);
bool pass_ppt2(const ndt_ctx* c);
bool lead_one_tile(const ndt_ctx* c);
bool direct_one_tile(const ndt_ctx* c);
bool grid_one_tile(const ndt_ctx* c);

bool needs_direct(const ndt_params& p) { return p.precision_mode == 0 && p.search != NDT_KDTREE; }
bool needs_radius(const ndt_params& p, bool mt_possible) { return !needs_direct(p) || mt_possible; }

// The neighbour cache the direct passes of an align read and write (DIRECT7 only; sized by ensure_align_buffers); the
// single-pass test hook (mode 1) runs without it
// one tile per workgroup only (C2 / C3 / C4 scans): its entries are read at kernel start beside the points; where
// workgroups walk several tiles (C5) the later tiles' entry loads and the registers they hold cost more than the
// probes they save (C5 88.6 vs 81.3 us per pass, C2 20.6 vs 21.1 us)
bool nbr_single_tile(const ndt_ctx* c, bool lead) {
    const int n = geom_points(std::max(1, c->N));
    const PassGeom g = direct_geom(c, lead);
    const int per_tile = g.block * ((!lead && pass_ppt2(c)) ? 2 : 1);
    return ceil_div(n, g.nb * per_tile) <= 1;
}
// allocation: whichever chain (leading tail or not) the next align picks
bool nbr_cache_wanted(const ndt_ctx* c) {
    if (c->prm.search != NDT_DIRECT7 || !NDT_NBR_CACHE) return false;
    return nbr_single_tile(c, true) || nbr_single_tile(c, false);
}
int4* nbr_cache(ndt_ctx* c, int mode) {
    if (mode != 0 || c->prm.search != NDT_DIRECT7 || !NDT_NBR_CACHE || !nbr_single_tile(c, c->lead != 0)) return nullptr;
    return c->nbr.cap >= 2 * (size_t)geom_points(std::max(1, c->N)) ? c->nbr.p : nullptr;
}

void launch_pass(ndt_ctx* c, int mode) {
    const ndt_params& p = c->prm;
    if (!needs_direct(p)) return;
    const PassGeom g = direct_geom(c, false);
    const bool ppt2 = pass_ppt2(c), one = direct_one_tile(c) || grid_one_tile(c);
    auto* kern = p.search == NDT_DIRECT26 ? k_pass_direct<S_DIRECT26, 1, false>
                 : p.search == NDT_DIRECT1
                     ? (ppt2 ? k_pass_direct<S_DIRECT1, 2, false> : (one ? k_pass_direct<S_DIRECT1, 1, true> : k_pass_direct<S_DIRECT1, 1, false>))
                     : (ppt2 ? k_pass_direct<S_DIRECT7, 2, false> : (one ? k_pass_direct<S_DIRECT7, 1, true> : k_pass_direct<S_DIRECT7, 1, false>));
    hipLaunchKernelGGL(kern, dim3(g.nb), dim3(g.block), 0, c->stream, c->pass_src, geom_points(c->N), g.ppb, c->d_hdr,
                       c->table.p, c->grid.p, c->recs.p, c->d_state, c->d_state, c->partials.p, c->counter.p, c->reduce_out.p,
                       c->d_hist, c->hist_cap, mode, c->profiling ? c->ts.p : nullptr, nbr_cache(c, mode));
}

void launch_radius(ndt_ctx* c, int mode) {
    const int nb = pass_blocks(geom_points(c->N));
    hipLaunchKernelGGL(k_pass_radius, dim3(nb), dim3(kBlock), 0, c->stream, c->pass_src, geom_points(c->N), c->d_hdr, c->table.p, c->grid.p, c->recs.p,
                       c->cent.p, c->icovd.p, c->d_state, c->d_state, c->partials.p, c->counter.p, c->reduce_out.p, c->d_hist,
                       c->hist_cap, mode,
                       c->profiling ? c->ts.p : nullptr);
}

// One leading-tail pass kernel (k_pass_lead) as kernel j = c->lead_par of the align's chain (see ndt_ctx::lead); the
// one-tile kernel (768 threads, three waves per SIMD) wherever the scan's point bucket fits one tile per workgroup.
void launch_lead(ndt_ctx* c, int j) {
    const PassGeom g = direct_geom(c, true);
    const bool one = lead_one_tile(c);
    AlignState* st[2] = {c->d_state, c->d_state2};
    double* pp[2] = {c->partials.p, c->partials2.p};
    const AlignState* sin = st[j & 1];
    AlignState* sout = st[(j + 1) & 1];
    const double* pin = pp[(j + 1) & 1];
    double* pout = pp[j & 1];
    unsigned long long* ts = c->profiling ? c->ts.p : nullptr;
    switch (c->prm.search) {
        case NDT_DIRECT26:
            hipLaunchKernelGGL((k_pass_lead<S_DIRECT26, false>), dim3(g.nb), dim3(g.block), 0, c->stream, c->pass_src, geom_points(c->N), g.ppb, c->d_hdr,
                               c->table.p, c->grid.p, c->recs.p, sin, sout, pin, pout, c->d_hist, c->hist_cap, ts, nbr_cache(c, 0));
            break;
        case NDT_DIRECT1:
            hipLaunchKernelGGL((one ? k_pass_lead<S_DIRECT1, true> : k_pass_lead<S_DIRECT1, false>), dim3(g.nb), dim3(g.block), 0, c->stream, c->pass_src, geom_points(c->N), g.ppb, c->d_hdr,
                               c->table.p, c->grid.p, c->recs.p, sin, sout, pin, pout, c->d_hist, c->hist_cap, ts, nbr_cache(c, 0));
            break;
        default:
            hipLaunchKernelGGL((one ? k_pass_lead<S_DIRECT7, true> : k_pass_lead<S_DIRECT7, false>), dim3(g.nb), dim3(g.block), 0, c->stream, c->pass_src, geom_points(c->N), g.ppb, c->d_hdr,
                               c->table.p, c->grid.p, c->recs.p, sin, sout, pin, pout, c->d_hist, c->hist_cap, ts, nbr_cache(c, 0));
            break;
    }
}

// Workgroups of at most one per CU (of this ctx's share) x the pass's workgroups per CU, and at least ~64 points each
int direct_blocks(const ndt_ctx* c, bool lead, int n, int ppt, bool one_tile = false) {
    return std::max(1, std::min(c->n_cu * pass_wgs_per_cu(c->prm.search, lead, ppt, one_tile), ceil_div(n, 64)));
}

// Last-workgroup-tail passes of one point per thread whose point bucket fits one tile per workgroup at three workgroups
// per CU (C4's 120 k-point pairs): k_pass_direct<S, 1, true>, three waves per SIMD
bool direct_one_tile(const ndt_ctx* c) {
    if (!NDT_DIRECT_ONE_TILE || c->prm.search == NDT_DIRECT26 || pass_ppt2(c)) return false;
    const int n = geom_points(std::max(1, c->N));
    return (long long)n <= (long long)direct_blocks(c, false, n, 1, true) * pass_block(c->prm.search, false);
}

// Last-workgroup-tail passes (k_pass_direct) of DIRECT7 / DIRECT1 hold two points per thread in a tile (half the
// tiles, the pair list packed into one word) once a workgroup walks >= 4 tiles of one point per thread (C5's 1 M-point
// scans: pass 87 -> 81 us; at C4's 3 tiles the halved tile count loses, 27.4 -> 28.8 us).  Every cloud index must then
// fit 22 bits.  ndt_set_pass_options(points_per_thread = 1) keeps one point per thread.
bool pass_ppt2(const ndt_ctx* c) {
    if (c->opt_ppt != 2 || c->prm.search == NDT_DIRECT26 || grid_one_tile(c)) return false;
    const long long max_cloud = (long long)c->M / std::max(1, c->prm.min_points_per_voxel) + 1;
    const int n = geom_points(std::max(1, c->N));
    const int rounds1 = ceil_div(n, direct_blocks(c, false, n, 1) * pass_block(c->prm.search, false));
    return max_cloud < (1ll << 22) && rounds1 >= 4;
}

// leading-tail passes in one tile per workgroup (k_pass_lead<S, true>): DIRECT7 / DIRECT1 whose point bucket fits one
// 768-point tile per CU
bool lead_one_tile(const ndt_ctx* c) {
    return NDT_LEAD_ONE_TILE && c->prm.search != NDT_DIRECT26 && (long long)geom_points(std::max(1, c->N)) <= (long long)c->n_cu * kLeadBlock1;
}

// Last-workgroup-tail passes of large clouds as a grid of one-tile workgroups (k_pass_direct<S, 1, true>: no tile loop,
// three waves per SIMD, as many 256-point workgroups as the scan needs — C5's 1 M points: 3 907) whose partials are
// summed by the two-level hand-off (pass_handoff); the alternative to the two-points-per-thread tile loop (pass_ppt2).
// ndt_set_pass_options(points_per_thread = 3) selects it (A/B; off by default).
bool grid_one_tile(const ndt_ctx* c) {
    if (c->opt_ppt != 3 || c->prm.search == NDT_DIRECT26) return false;
    return geom_points(std::max(1, c->N)) > c->n_cu * kLeadBlock1;
}

PassGeom direct_geom(const ndt_ctx* c, bool lead) {
    PassGeom g;
    g.block = pass_block(c->prm.search, lead, lead && lead_one_tile(c));
    const int n = geom_points(std::max(1, c->N));
    if (!lead && grid_one_tile(c)) {
        g.nb = ceil_div(n, g.block);
        g.ppb = g.block;
        return g;
    }
    const int ppt = (!lead && pass_ppt2(c)) ? 2 : 1;
    g.nb = direct_blocks(c, lead, n, ppt, !lead && direct_one_tile(c));
    const int per_tile = g.block * ppt;
    const int rounds = ceil_div(n, g.nb * per_tile);
    g.ppb = ceil_div(n, g.nb * rounds);
    return g;
}

// enqueue `slots` (pass, control) pairs; pass events optional
ndt_status enqueue_chain(ndt_ctx* c, int slots, bool mt_possible, bool with_events) {
    for (int s = 0; s < slots; ++s) {
        if (with_events) HIPCHK(c, hipEventRecord(c->pass_ev[2 * s], c->stream));
        if (c->lead) {
            launch_lead(c, c->lead_par + s);
        } else {
            launch_pass(c, 0);
            if (needs_radius(c->prm, mt_possible)) launch_radius(c, 0);
        }
        if (with_events) HIPCHK(c, hipEventRecord(c->pass_ev[2 * s + 1], c->stream));
    }
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

void init_state(ndt_ctx* c, const float guess[16], AlignState* st) {
    std::memset(st, 0, sizeof(AlignState));
    const ndt_params& p = c->prm;
    gauss_constants(p.outlier_ratio, p.resolution, &st->gauss_d1, &st->gauss_d2, &st->gauss_d3);
    c->gauss_cur[0] = st->gauss_d1;
    c->gauss_cur[1] = st->gauss_d2;
    c->gauss_cur[2] = st->gauss_d3;
    st->step_max = p.step_size;
    st->step_min = p.trans_eps / 2;
    st->trans_eps = p.trans_eps;
    st->max_iter = p.max_iter;
    st->n_src = c->N;
    st->search = p.search;
    st->precision = p.precision_mode;
    st->mt_possible = (st->step_max - st->step_min) > 0 ? 0 : 1;
    st->radius = p.resolution;
    // pcl::Registration::align: final = I; computeTransformation: guess != I -> final = guess, output = guess * input
    bool ident = true;
    for (int k = 0; k < 16; ++k)
        if (guess[k] != ((k % 5 == 0) ? 1.f : 0.f)) ident = false;
    float F[16];
    for (int k = 0; k < 16; ++k) F[k] = ident ? ((k % 5 == 0) ? 1.f : 0.f) : guess[k];
    for (int k = 0; k < 16; ++k) st->T[k] = F[k];
    // p = [translation, rotation().eulerAngles(0,1,2)] in f32 (ndt_omp_impl.hpp:96-104)
    float L[9], R[9], eul[3];
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) L[i + 3 * j] = F[i + 4 * j];
    polar_rotation_f(L, R);
    euler012_f(R, eul);
    st->p[0] = F[12]; st->p[1] = F[13]; st->p[2] = F[14];
    st->p[3] = eul[0]; st->p[4] = eul[1]; st->p[5] = eul[2];
    for (int k = 0; k < 6; ++k) { st->x_eval[k] = st->p[k]; st->x_t[k] = st->p[k]; }
    angle_tables(st->p, st->jang, st->hang, st->jang_d, st->hang_d);
    st->phase = 0;
    st->pending = 1;
    st->pass_kind = PASS_FULL;
}

ndt_status ensure_align_buffers(ndt_ctx* c) {
    const int nb = pass_blocks(geom_points(c->N));
    const int nbd = std::max(nb, std::max(direct_geom(c, false).nb, direct_geom(c, true).nb));
    // + the group partials of the two-level hand-off (grids of more than kTwoLevelMinBlocks workgroups)
    TRY(ensure(c, c->partials, (size_t)kNumAcc * (partial_stride(nbd) + kMaxGroups)));
    TRY(ensure(c, c->partials2, (size_t)kNumAcc * (partial_stride(nbd) + kMaxGroups)));
    TRY(ensure(c, c->reduce_out, kNumAcc));
    TRY(ensure(c, c->counter, kPassCounterWords));
    // the neighbour cache only where the passes read it (32 B per point; a multi-tile geometry such as C5's never does)
    if (nbr_cache_wanted(c)) TRY(ensure(c, c->nbr, 2 * (size_t)geom_points(c->N)));
    else if (c->nbr.p) release(c->nbr);
    return NDT_OK;
}

ndt_status ensure_pass_events(ndt_ctx* c, int slots) {
    if ((int)c->pass_ev.size() < 2 * slots) {
        size_t old = c->pass_ev.size();
        c->pass_ev.resize(2 * slots);
        for (size_t k = old; k < c->pass_ev.size(); ++k) HIPCHK(c, hipEventCreate(&c->pass_ev[k]));
        invalidate_graph(c);
    }
    return NDT_OK;
}

AlignState* lead_state(ndt_ctx* c, int ahead);
ndt_status prepare_readback(ndt_ctx* c, int from, int to);
void launch_readback(ndt_ctx* c, int from, int to, const AlignState* d_src, unsigned long long seq);

// with_readback: the round's k_readback is captured as the graph's last node (the first round of an align: from 0 to
// the round's passes, its sequence number read from d_clk[2]) — a kernel queued behind a graph launch starts ~8.7 us after
// the graph's last kernel (rocprofv3, C2 step), inside the graph it follows at once
ndt_status build_graph(ndt_ctx* c, int slots, bool mt_possible, hipGraphExec_t* out, bool with_readback) {
    constexpr int kGraphKey = ndt_ctx::kGraphKey;
    // every pointer / size baked into the captured kernels
    // (one slot per captured pointer: a combined key could collide after a reallocation and replay freed buffers)
    const long long key[kGraphKey] = {geom_points(c->N), (long long)(uintptr_t)c->pass_src, (long long)(uintptr_t)c->table.p, c->prm.search,
                                      c->prm.precision_mode,
                                      mt_possible | (c->profiling ? 2 : 0) | (c->lead ? 4 : 0) | ((c->lead_par & 1) ? 8 : 0) |
                                          (pass_ppt2(c) ? 16 : 0), slots,
                                      (long long)(uintptr_t)c->recs.p, (long long)(uintptr_t)c->partials.p,
                                      (long long)(uintptr_t)c->grid.p, (long long)(uintptr_t)c->reduce_out.p,
                                      (long long)(uintptr_t)c->counter.p, (long long)(uintptr_t)c->cent.p,
                                      (long long)(uintptr_t)c->icovd.p, (long long)(uintptr_t)c->ts.p,
                                      (long long)(uintptr_t)c->d_hdr, (long long)(uintptr_t)c->d_state,
                                      (long long)(uintptr_t)c->d_hist, (long long)(uintptr_t)c->partials2.p,
                                      (long long)(uintptr_t)nbr_cache(c, 0), with_readback ? 1 : 0,
                                      (long long)(uintptr_t)c->h_ts, (long long)(uintptr_t)c->h_hist};
    for (auto& g : c->graphs)
        if (g.exec && std::memcmp(key, g.key, sizeof(key)) == 0) {
            *out = g.exec;
            return NDT_OK;
        }
    ndt_ctx::GraphEntry& slot = c->graphs[c->graph_next];
    c->graph_next = (c->graph_next + 1) % ndt_ctx::kGraphCache;
    if (slot.exec) {
        // the evicted chain may still run on the stream (an earlier align of this ctx, an async align whose wait has not
        // come): its executable owns the kernel arguments of its nodes, so it is destroyed only once the stream is past it
        HIPCHK(c, hipStreamSynchronize(c->stream));
        (void)hipGraphExecDestroy(slot.exec);
    }
    slot.exec = nullptr;
    if (c->profiling) TRY(ensure(c, c->ts, kTsStride * (size_t)c->hist_cap));
    const int rb_to = slots * (mt_possible ? 4 : 1);
    if (with_readback) TRY(prepare_readback(c, 0, rb_to));
    hipGraph_t g;
    std::unique_lock<std::shared_mutex> capture(c->capture_mu);
    HIPCHK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    ndt_status st = enqueue_chain(c, slots, mt_possible, false);
    if (st == NDT_OK && with_readback) launch_readback(c, 0, rb_to, lead_state(c, slots), 0ull);
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    capture.unlock();
    if (st != NDT_OK) return st;
    if (e != hipSuccess) return fail(c, NDT_EDEVICE, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
    e = hipGraphInstantiate(&slot.exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) { slot.exec = nullptr; return fail(c, NDT_EDEVICE, std::string("hipGraphInstantiate: ") + hipGetErrorString(e)); }
    std::memcpy(slot.key, key, sizeof(key));
    *out = slot.exec;
    return NDT_OK;
}


// The pass chain of one round: the captured graph (one hipGraphLaunch per round).
ndt_status launch_chain(ndt_ctx* c, int slots, bool mt, bool with_readback = false) {
    hipGraphExec_t gx = nullptr;
    TRY(build_graph(c, slots, mt, &gx, with_readback));
    HIPCHK(c, hipGraphLaunch(gx, c->stream));
    return NDT_OK;
}

// The device state after `ahead` more kernels of the chain: the only state buffer without leading-tail chains, else
// the ping-pong buffer kernel lead_par + ahead reads.
AlignState* lead_state(ndt_ctx* c, int ahead) {
    if (!c->lead) return c->d_state;
    return ((c->lead_par + ahead) & 1) ? c->d_state2 : c->d_state;
}

// End-of-round read-back, queued on the stream before the align's own synchronisation (no extra round trip): the
// optimiser state and, when profiling, the stamps and pass records of passes [from, to), all by one k_readback launch
// straight into pinned host memory (blit copies would cost a launch + gap each), then the round's sequence number.
ndt_status prepare_readback(ndt_ctx* c, int from, int to) {
    to = std::min(to, c->hist_cap);
    const bool prof = c->profiling && to > from;
    if (prof && c->h_prof_cap < c->hist_cap) {
        if (c->h_ts) (void)hipHostFree(c->h_ts);
        if (c->h_hist) (void)hipHostFree(c->h_hist);
        c->h_ts = nullptr;
        c->h_hist = nullptr;
        c->h_prof_cap = 0;
        if (hipHostMalloc(&c->h_ts, kTsStride * (size_t)c->hist_cap * sizeof(unsigned long long), hipHostMallocCoherent) != hipSuccess ||
            hipHostMalloc(&c->h_hist, (size_t)c->hist_cap * sizeof(PassRecordDev), hipHostMallocCoherent) != hipSuccess)
            return fail(c, NDT_ENOMEM, "hipHostMalloc failed");
        c->h_prof_cap = c->hist_cap;
    }
    return NDT_OK;
}

// seq: the round's sequence number, or 0 for the one k_align_init stored in d_clk[2] (the launch is then graph-capturable)
void launch_readback(ndt_ctx* c, int from, int to, const AlignState* d_src, unsigned long long seq) {
    to = std::min(to, c->hist_cap);
    const bool prof = c->profiling && to > from;
    static_assert(sizeof(PassRecordDev) % 8 == 0, "pass records copied as 8-byte words");
    using u64 = unsigned long long;
    const int ts_words = prof ? kTsStride * (to - from) : 0;
    const int hist_words = prof ? (int)((to - from) * sizeof(PassRecordDev) / 8) : 0;
    const u64* ts = prof ? c->ts.p + kTsStride * (size_t)from : nullptr;
    u64* h_ts = prof ? c->h_ts + kTsStride * (size_t)from : nullptr;
    const u64* hist = prof ? reinterpret_cast<const u64*>(c->d_hist + from) : nullptr;
    u64* h_hist = prof ? reinterpret_cast<u64*>(c->h_hist + from) : nullptr;
    hipLaunchKernelGGL(k_readback, dim3(1), dim3(kBlock), 0, c->stream, reinterpret_cast<const u64*>(d_src),
                       reinterpret_cast<u64*>(c->h_state), (int)(sizeof(AlignState) / 8), ts, h_ts, ts_words, hist, h_hist, hist_words,
                       c->d_clk, c->h_rb + 1, c->h_rb, seq,
                       d_src != c->d_state ? reinterpret_cast<u64*>(c->d_state) : nullptr, c->d_hdr);
}

// A continuation round's read-back, queued behind its graph
ndt_status enqueue_readback(ndt_ctx* c, int from, int to, const AlignState* d_src) {
    TRY(prepare_readback(c, from, to));
    c->al_seq = ++c->rb_seq;
    launch_readback(c, from, to, d_src, c->al_seq);
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

// per-pass kernel time from the in-kernel stamps (first workgroup start .. last workgroup end, 100 MHz clock)
ndt_status collect_pass_times(ndt_ctx* c, int hist_before) {
    const int total = std::min(c->h_state->hist_count, c->hist_cap);
    const int ran = total - hist_before;
    if (ran <= 0 || !c->h_ts) return NDT_OK;
    const PassRecordDev* hist = c->h_hist + hist_before;
    double sum = 0, bytes = 0;
    int cnt = 0;
    for (int k = 0; k < ran; ++k) {
        const unsigned long long* t = &c->h_ts[kTsStride * (size_t)(hist_before + k)];
        if (t[1] <= t[0] || t[0] == ~0ull) continue;
        sum += (double)(t[1] - t[0]) * 1e-5;  // 100 MHz ticks -> ms
        bytes += 16.0 * c->N + 36.0 * (double)hist[k].pairs;  // B_pass = 16 N + 36 P
        ++cnt;
        // phases: blocks' bodies, hand-off, partials reduce, control step, state write-back / drain
        if (t[2] >= t[0] && t[3] >= t[2] && t[4] >= t[3] && t[6] >= t[4] && t[7] >= t[6] && t[5] >= t[7] && t[1] >= t[5]) {
            const unsigned long long e[8] = {t[0], t[2], t[3], t[4], t[6], t[7], t[5], t[1]};
            for (int q = 0; q < 7; ++q) c->prof_phase_sum[q] += (double)(e[q + 1] - e[q]) * 1e-5;
            ++c->prof_phase_count;
        }
    }
    // profiling build: mean per-workgroup phases of this align's passes (private per-block stamps)
    constexpr int kBP = 64, kBM = 1024, kBS = 8;
    static const bool have_blk = dbg_read_blk(nullptr, 0) == hipSuccess;
    std::vector<unsigned long long> blk;
    if (have_blk) blk.resize((size_t)kBP * kBM * kBS);
    if (have_blk && dbg_read_blk(blk.data(), blk.size()) == hipSuccess) {
        const int nbk = std::min(direct_geom(c, c->lead != 0).nb, kBM);
        for (int k = 0; k < ran && hist_before + k < kBP; ++k) {
            const int pidx = hist_before + k;
            const unsigned long long t0 = c->h_ts[kTsStride * (size_t)pidx];
            double ph[5] = {0, 0, 0, 0, 0};
            bool ok = true;
            int nb_used = 0;
            for (int b = 0; b < nbk && ok; ++b) {
                const unsigned long long* e = &blk[((size_t)pidx * kBM + b) * kBS];
                if (e[1] == 0) continue;  // a workgroup past the scan's points (the geometry covers its size bucket)
                if (e[1] < e[0] || e[2] < e[1] || e[3] < e[2] || e[4] < e[3]) { ok = false; break; }
                ++nb_used;
                // entry: from workgroup 0's pass stamp (a leading-tail kernel: after the state staging) to the body
                ph[0] += e[0] > t0 ? (double)(e[0] - t0) : 0.0;
                // probe / compaction / pairs: the body's per-tile sums (slots 5..7); block reduction: last tile end .. epilogue
                for (int q = 0; q < 3; ++q) ph[1 + q] += (double)e[5 + q];
                ph[4] += (double)(e[4] - e[3]);
            }
            if (!ok || nb_used == 0) continue;
            // NDT_BLK_DUMP=file: every workgroup's body end (from the pass stamp) and per-phase ticks of pass 10
            // (NDT_BLK_DUMP_PASS), appended
            // (the spread of the workgroups' finish times behind the means)
            static const char* dump = getenv("NDT_BLK_DUMP");
            static const int dump_pass = getenv("NDT_BLK_DUMP_PASS") ? atoi(getenv("NDT_BLK_DUMP_PASS")) : 10;
            if (dump && pidx == dump_pass) {
                if (FILE* f = fopen(dump, "a")) {
                    for (int b = 0; b < nbk; ++b) {
                        const unsigned long long* e = &blk[((size_t)pidx * kBM + b) * kBS];
                        if (e[1] == 0 || e[4] < t0) continue;
                        fprintf(f, "%d %llu %llu %llu %llu %llu\n", b, e[0] > t0 ? e[0] - t0 : 0ull, e[4] - t0, e[5], e[6], e[7]);
                    }
                    fclose(f);
                }
            }
            for (int q = 0; q < 5; ++q) c->prof_body_sum[q] += ph[q] / nb_used * 1e-5;
            ++c->prof_body_count;
            if (c->lead) {
                // leading-tail kernels: workgroup 0's prologue (staging, partial reduction, control step + tables) in the
                // tail slots record / machine / solve_setup
                const unsigned long long* r = &blk[((size_t)pidx * kBM + kBM - 2) * kBS];
                // the consumed pass's control-step stamps (tail_control, workgroup 0): [4] record done, [5] state machine
                // done, [0]/[1] the step, [2] sin/cos, [3] tables
                const unsigned long long* tl = pidx >= 1 ? &blk[((size_t)(pidx - 1) * kBM + kBM - 1) * kBS] : nullptr;
                if (r[1] >= r[0] && r[2] >= r[1] && r[3] >= r[2] && r[0] > 0 && tl && tl[4] >= r[2] && tl[5] >= tl[4] &&
                    tl[1] >= tl[5] && tl[2] >= tl[1] && tl[3] >= tl[2] && r[3] >= tl[3]) {
                    c->prof_tail_sum[0] += (double)(r[1] - r[0]) * 1e-5;    // record    <- staging
                    c->prof_tail_sum[1] += (double)(r[2] - r[1]) * 1e-5;    // machine   <- partial reduction
                    c->prof_tail_sum[2] += (double)(tl[4] - r[2]) * 1e-5;   // solve_setup <- pass record
                    c->prof_tail_sum[3] += (double)(tl[5] - tl[4]) * 1e-5;  // solve     <- state machine
                    c->prof_tail_sum[4] += (double)(tl[1] - tl[5]) * 1e-5;  // post_solve <- to the step
                    c->prof_tail_sum[5] += (double)(tl[2] - tl[1]) * 1e-5;  // sincos    <- step + sin/cos + barrier
                    c->prof_tail_sum[6] += (double)(tl[3] - tl[2]) * 1e-5;  // rows      <- T + tables
                    c->prof_tail_sum[7] += (double)(r[3] - tl[3]) * 1e-5;   // writeback <- to the body
                    ++c->prof_tail_count;
                }
                continue;
            }
            // tail: [0] before / [1] after the Newton LU solve, [2] sin/cos ready, [3] tables written
            const unsigned long long* tl = &blk[((size_t)pidx * kBM + kBM - 1) * kBS];
            const unsigned long long* t = &c->h_ts[kTsStride * (size_t)pidx];
            if (tl[4] >= t[6] && tl[5] >= tl[4] && tl[0] >= tl[5] && tl[1] >= tl[0] && t[7] >= tl[1] && tl[2] >= t[7] &&
                tl[3] >= tl[2] && t[5] >= tl[3]) {
                const unsigned long long e[9] = {t[6], tl[4], tl[5], tl[0], tl[1], t[7], tl[2], tl[3], t[5]};
                for (int q = 0; q < 8; ++q) c->prof_tail_sum[q] += (double)(e[q + 1] - e[q]) * 1e-5;
                // the speculative Newton solve on wave 0: its start after staging, its duration
                if (tl[6] >= t[6] && tl[7] >= tl[6]) {
                    c->prof_tail_sum[8] += (double)(tl[6] - t[6]) * 1e-5;
                    c->prof_tail_sum[9] += (double)(tl[7] - tl[6]) * 1e-5;
                }
                ++c->prof_tail_count;
            }
        }
    }
    c->prof_ms_sum += sum;
    c->prof_bytes_sum += bytes;
    c->prof_count += cnt;
    if (c->prof_count) { c->ms_pass_avg = c->prof_ms_sum / c->prof_count; c->pass_bytes_avg = c->prof_bytes_sum / c->prof_count; }
    return NDT_OK;
}

// Source order of this align (k_src_keys): points sorted by the target cell they fall into under the initial
// transform, so that neighbouring lanes of a pass probe and gather neighbouring cells.  Clouds below 256 Ki points keep
// their order: there the sort (~35 us) costs about what it saves (C2: 1.5 us per pass over 33 passes; C3: 2-4 passes).
#ifndef NDT_ORDER_MIN_POINTS
#define NDT_ORDER_MIN_POINTS 262144
#endif
constexpr int kOrderMinPoints = NDT_ORDER_MIN_POINTS;
constexpr int kLeadMaxPoints = 262144;  // leading-tail chains below this many source points (align_enqueue)
ndt_status enqueue_source_order(ndt_ctx* c, const float T[16]) {
    c->pass_src = c->source.p;
    const int n = c->N;
    if (!c->order_source || n < kOrderMinPoints) return NDT_OK;
    TRY(ensure(c, c->source_ord, geom_points(n)));
    TRY(ensure(c, c->ord_k0, n)); TRY(ensure(c, c->ord_v0, n)); TRY(ensure(c, c->ord_k1, n)); TRY(ensure(c, c->ord_v1, n));
    const int items = radix_items(c, n);
    const int nb_sort = std::max(1, ceil_div(n, kBlock * items));
    TRY(ensure(c, c->s.radix_aux, kRadixAuxWords));
    TRY(ensure(c, c->s.radix_status, (size_t)4 * 256 * nb_sort));
    Mat4f Tm;
    std::memcpy(Tm.m, T, sizeof(Tm.m));
    HIPCHK(c, hipMemsetAsync(c->s.radix_aux.p, 0, kRadixAuxWords * sizeof(int), c->stream));
    const int nb_keys = std::max(1, std::min(ceil_div(n, kBlock), 1024));
    hipLaunchKernelGGL(k_src_keys, dim3(nb_keys), dim3(kBlock), 0, c->stream, c->source.p, n, Tm, c->d_hdr, c->ord_k0.p, c->ord_v0.p,
                       c->s.radix_aux.p, c->s.radix_status.p, 4 * 256 * nb_sort);
    const int passes = radix_launch_passes(c);
    for (int pass = 0; pass < passes; ++pass)
        launch_radix_pass(c, main_lane(c), items, nb_sort, c->ord_k0.p, c->ord_v0.p, c->ord_k1.p, c->ord_v1.p, n, pass, c->d_hdr, c->d_hdr,
                          passes - 1);
    hipLaunchKernelGGL(k_src_gather, dim3(std::max(1, std::min(ceil_div(n, kBlock), 2048))), dim3(kBlock), 0, c->stream, c->source.p,
                       c->ord_v0.p, c->ord_v1.p, c->d_hdr, c->source_ord.p, n);
    HIPCHK(c, hipGetLastError());
    c->pass_src = c->source_ord.p;
    return NDT_OK;
}

// Waits for the read-back of round `seq`: spins on the sequence word k_readback releases last (a stream
// synchronisation sleeps on the completion interrupt and wakes tens of microseconds after the GPU is done); a device
// error still surfaces through the periodic stream query.  NDT_SPIN_WAIT=0 synchronises the stream instead (A/B).
ndt_status wait_readback(ndt_ctx* c, unsigned long long seq) {
    const volatile unsigned long long* w = c->h_rb;
    for (unsigned it = 1;; ++it) {
        if (*w == seq) break;
        if ((it & 1023u) == 0) {
            const hipError_t e = hipStreamQuery(c->stream);
            if (e == hipSuccess) {
                if (*w == seq) break;
                return fail(c, NDT_EDEVICE, "align read-back missing after the stream finished");
            }
            if (e != hipErrorNotReady) return fail(c, NDT_EDEVICE, std::string("align: ") + hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return NDT_OK;
}

// An align in two halves: align_enqueue queues the initial state and the first round of the pass chain (a graph of
// last_passes+1 passes, which normally covers the whole align) with the read-back of the final state, without waiting;
// align_finish waits, runs any further rounds (slow convergence, SVD fallback) synchronously and records timings.
// ndt_align = both back to back; ndt_align_async / ndt_align_wait and the batched replay keep several contexts
// (streams) in flight.
ndt_status align_enqueue(ndt_ctx* c, const float guess[16]) {
    TRY(ensure_align_buffers(c));
    std::memcpy(c->al_guess, guess, sizeof(c->al_guess));
    init_state(c, guess, c->h_state);
    const bool mt = c->h_state->mt_possible != 0;
    // Newton-only chains: the first round covers the previous align's pass count + 1 (scan-to-scan replay converges
    // in a similar number of iterations), continuation rounds 8 passes; passes queued after convergence exit at
    // once but still cost a launch each.  More-Thuente chains (4 passes per slot possible) keep 16-slot rounds.
    // leading-tail chain (ndt_set_pass_options(lead_tail = 0): last-workgroup tails) whenever the align runs direct passes only
    // Used where the align is latency-bound: one registration at a time (not the batched replay, where the other
    // streams' bodies fill the CUs a last-workgroup tail leaves idle: C4 1437 vs 1156 pairs/s) and below kLeadMaxPoints
    // source points (C5's 1 M-point passes are body-bound: 227.7 vs 225.3 scans/s); C2 954 -> 1022, C3 2219 -> 2334.
    // ndt_set_pass_options(lead_tail = 0) forces last-workgroup tails (tests/test_gpu_lead.py compares the two chains)
    c->lead = (c->opt_lead_tail && !c->no_lead && c->N < kLeadMaxPoints && needs_direct(c->prm) && !needs_radius(c->prm, mt)) ? 1 : 0;
    c->lead_par = 0;
    // a leading-tail chain needs one kernel more than it has passes (the last pass's step runs in the next kernel)
    const int full = mt ? 16 : c->prm.max_iter + 3 + c->lead;
    int slots = full;
    if (!mt && c->last_passes > 0) slots = std::min(full, std::max(3, c->last_passes + 1 + c->lead));
    if (c->profiling) TRY(ensure(c, c->ts, kTsStride * (size_t)c->hist_cap));
    {
        // state upload + ticket reset (+ stamp reset) + the align's start stamp as one launch; the state is passed by
        // value (kernel argument)
        const int ts_words = c->profiling ? kTsStride * c->hist_cap : 0;
        // + the source copy ndt_set_source_device deferred (four 16-byte words per thread and round; a source that is not
        // 16-byte aligned is copied by copy16 first)
        if (c->src_pend && (reinterpret_cast<uintptr_t>(c->src_pend) & 15)) TRY(flush_source(c));
        const long long cp_words = c->src_pend ? (long long)c->N : 0;
        const int nb = std::max({1, std::min(256, ceil_div(ts_words, kBlock)), (int)std::min<long long>(1024, ceil_div(cp_words, 4LL * kBlock))});
        const uint4* cp_src = reinterpret_cast<const uint4*>(c->src_pend);
        c->src_pend = nullptr;
        c->al_seq = ++c->rb_seq;
        c->lanes_marked = 0;  // a side-lane mark not taken before this align is dropped
        hipLaunchKernelGGL(k_align_init, dim3(nb), dim3(kBlock), 0, c->stream, *c->h_state, c->d_state, c->counter.p,
                           c->profiling ? c->ts.p : nullptr, ts_words, c->d_clk, c->grid_valid ? c->d_hdr : nullptr, c->al_seq,
                           cp_src, reinterpret_cast<uint4*>(c->source.p), cp_words);
        HIPCHK(c, hipGetLastError());
    }
    TRY(enqueue_source_order(c, c->h_state->T));
    TRY(launch_chain(c, slots, mt, true));  // the round's read-back is the graph's last node
    c->lead_par += slots;
    c->al_inflight = true;
    c->al_mt = mt;
    c->al_full = full;
    c->al_slots = slots;
    return NDT_OK;
}

ndt_status align_finish_once(ndt_ctx* c) {
    if (!c->al_inflight) return fail(c, NDT_EINVAL, "no align in flight");
    c->al_inflight = false;
    const bool mt = c->al_mt;
    const int full = c->al_full;
    int slots = c->al_slots;
    int hist_before = 0;
    int rounds = 0;
    const int max_rounds = 1 + (c->prm.max_iter + 3) * 12 / 3 + 4 + 64;
    for (;;) {
        TRY(wait_readback(c, c->al_seq));
        ++rounds;
        if (c->profiling) TRY(collect_pass_times(c, hist_before));
        if (c->h_state->done || rounds >= max_rounds) break;
        if (!mt) slots = std::min(full, 8);
        if (c->h_state->needs_svd) {
            hipLaunchKernelGGL(k_svd_resume, dim3(1), dim3(kBlock), 0, c->stream, lead_state(c, 0));
            HIPCHK(c, hipGetLastError());
        }
        hist_before = std::min(c->h_state->hist_count, c->hist_cap);
        TRY(launch_chain(c, slots, mt));
        TRY(enqueue_readback(c, hist_before, hist_before + slots * (mt ? 4 : 1), lead_state(c, slots)));
        c->lead_par += slots;
    }
    c->ms_align = (double)(c->h_rb[2] - c->h_rb[1]) * 1e-5;  // 100 MHz device clock: k_align_init .. last read-back
    // a build queued since the previous align: its start (k_minmax) .. this align's start (100 MHz device clock)
    if (c->built_since_align && c->h_rb[1] > c->h_rb[3]) c->ms_build = (double)(c->h_rb[1] - c->h_rb[3]) * 1e-5;
    c->built_since_align = false;
    c->grid_cells_seen = std::max(c->grid_cells_seen, c->h_state->grid_cells);
    c->have_result = true;
    c->align_tgt_gen = c->tgt_gen;
    c->last_passes = c->h_state->n_passes;
    if (!c->h_state->done) return fail(c, NDT_EDEVICE, "align did not finish within the slot budget");
    // the target build's error bits (GridHeader::pad[0]): latched by k_align_init for the build queued ahead of the align,
    // and read again by the last read-back (the align's own source-order sort reports into the same header)
    c->al_berr = c->h_state->build_error | (int)c->h_rb[4];
    if (!c->al_berr) {
        c->build_unchecked = false;
        note_grid_width(c, c->h_state->grid_cells, c->target_dense);
    }
    return NDT_OK;
}

// A target build whose sort flagged an error (GridHeader::pad[0]) is queued again from scratch: all four radix passes,
// tiles by atomic ticket from now on if a look-back timed out (the blockIdx.x tile order relies on each XCD dispatching
// its workgroups in increasing order, observed but not guaranteed when other streams' kernels hold the CUs; a ticket
// tile waits only on tiles that started before it), a fresh sort where a merge could not be exact.  Same grid as a
// first build that had not failed.
ndt_status rerun_build(ndt_ctx* c, int berr) {
    ++c->n_builds_rerun;
    if (berr & kBuildErrLookback) {
        c->tile_tickets = true;
        ++c->n_rerun_lookback;
    }
    c->inc_ok = false;
    c->rerun_full = true;
    const ndt_status st = build_target(c);
    c->rerun_full = false;
    return st;
}

// align_finish_once, and after a flagged target build: the build re-run and the align with it (same guess, same source)
ndt_status align_finish(ndt_ctx* c) {
    TRY(align_finish_once(c));
    if (!c->al_berr) return NDT_OK;
    const int berr = c->al_berr;
    TRY(rerun_build(c, berr));
    TRY(align_enqueue(c, c->al_guess));
    TRY(align_finish_once(c));
    if (c->al_berr)
        return fail(c, NDT_EDEVICE, std::string("target build failed twice (error bits ") + std::to_string(berr) + ", " +
                                        std::to_string(c->al_berr) + ")");
    return NDT_OK;
}

// The synchronous readers of the target grid other than an align (grid inspection, single passes, calculateScore): the
// error bits of a build no align has checked yet, read back now; a flagged build is re-run.
ndt_status settle_build(ndt_ctx* c) {
    if (!c->build_unchecked || !c->grid_valid) return NDT_OK;
    for (int attempt = 0;; ++attempt) {
        HIPCHK(c, hipMemcpyAsync(c->h_hdr, c->d_hdr, sizeof(GridHeader), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const int berr = c->h_hdr->pad[0];
        if (!berr) break;
        if (attempt > 0) return fail(c, NDT_EDEVICE, "target build failed twice (error bits " + std::to_string(berr) + ")");
        TRY(rerun_build(c, berr));
    }
    c->build_unchecked = false;
    note_grid_width(c, c->h_hdr->cells, c->target_dense);
    return NDT_OK;
}

ndt_status run_align(ndt_ctx* c, const float guess[16]) {
    TRY(align_enqueue(c, guess));
    return align_finish(c);
}

void fill_result(ndt_ctx* c, ndt_result* out) {
    const AlignState* st = c->h_state;
    for (int k = 0; k < 16; ++k) out->final_tf[k] = st->T[k];
    out->nr_iterations = st->nr_iterations;
    out->converged = st->converged;
    out->trans_probability = st->trans_probability;
    out->score = st->score;
    out->n_passes = st->n_passes;
    out->n_pairs = st->pairs_total;
    out->solver_fallbacks = st->solver_fallbacks;
}

ndt_status upload_points(ndt_ctx* c, DevBuf<float4>& dst, const float* xyz, size_t n, size_t stride_bytes) {
    TRY(ensure(c, dst, n));
    std::vector<float4> tmp(n);
    const char* base = reinterpret_cast<const char*>(xyz);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        tmp[i] = make_float4(f[0], f[1], f[2], 1.0f);
    }
    if (n) HIPCHK(c, hipMemcpyAsync(dst.p, tmp.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return NDT_OK;
}

ndt_status set_dev(ndt_ctx* c) {
    HIPCHK(c, hipSetDevice(c->device));
    return NDT_OK;
}

}  // namespace

// =====================================================================================================
extern "C" {

ndt_status ndt_default_params(ndt_params* out) {
    if (!out) return NDT_EINVAL;
    out->resolution = 1.0f;
    out->step_size = 0.1;
    out->trans_eps = 0.1;
    out->outlier_ratio = 0.55;
    out->max_iter = 35;
    out->search = NDT_DIRECT7;
    out->min_points_per_voxel = 6;
    out->min_covar_eigvalue_mult = 0.01;
    out->precision_mode = 0;
    out->device = 0;
    return NDT_OK;
}

ndt_status ndt_create(const ndt_params* params, ndt_ctx** out) {
    if (!out) return NDT_EINVAL;
    *out = nullptr;
    ndt_params p;
    if (params) p = *params; else ndt_default_params(&p);
    if (!valid_params(&p)) return NDT_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return NDT_EDEVICE;
    if (p.device < 0 || p.device >= ndev) return NDT_EINVAL;
    ndt_ctx* c = new ndt_ctx();
    c->prm = p;
    c->device = p.device;
    // the main stream (target build, align: a scan loop's critical path) at the highest priority, the side lanes
    // (getFitnessScore, keyframe insertion) at the lowest
    int prio_least = 0, prio_greatest = 0;
    if (hipSetDevice(c->device) != hipSuccess || hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_greatest) != hipSuccess) {
        delete c;
        return NDT_EDEVICE;
    }
    int n_cu = 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess && n_cu > 0) c->n_cu = n_cu;
    // A/B: NDT_LANE_CUS = k side-lane CUs (NDT_LANE_CU_MODE 0: every (n_cu / k)-th CU, 1: the first k), the main stream
    // on the rest (its pass grids sized for them)
    if (const char* e = std::getenv("NDT_LANE_CUS")) {
        const int k = std::atoi(e);
        const int mode = std::getenv("NDT_LANE_CU_MODE") ? std::atoi(std::getenv("NDT_LANE_CU_MODE")) : 0;
        if (k > 0 && k < c->n_cu) {
            const int words = (c->n_cu + 31) / 32, stride = c->n_cu / k;
            std::vector<uint32_t> main_mask(words, 0u);
            c->lane_mask.assign(words, 0u);
            int taken = 0;
            for (int i = 0; i < c->n_cu; ++i) {
                const bool lane = mode == 1 ? i < k : (i % stride == stride - 1 && taken < k);
                if (lane) ++taken;
                (lane ? c->lane_mask : main_mask)[i / 32] |= 1u << (i % 32);
            }
            hipStream_t ms = nullptr;
            if (hipExtStreamCreateWithCUMask(&ms, (uint32_t)words * 32, main_mask.data()) == hipSuccess) {
                (void)hipStreamDestroy(c->stream);
                c->stream = ms;
                c->n_cu -= taken;
            } else {
                c->lane_mask.clear();
            }
        }
    }
    if (const char* e = std::getenv("NDT_PPT")) c->opt_ppt = std::max(1, std::min(3, std::atoi(e)));  // A/B runs (pass geometry)
    gauss_constants(0.55, 1.0f, &c->gauss_cur[0], &c->gauss_cur[1], &c->gauss_cur[2]);
    bool ok = hipMalloc(&c->d_hdr, sizeof(GridHeader)) == hipSuccess && hipMalloc(&c->d_hdr_ds, sizeof(GridHeader)) == hipSuccess &&
              hipMalloc(&c->d_hdr_prev, sizeof(GridHeader)) == hipSuccess &&
              hipMalloc(&c->d_hdr_fe, sizeof(GridHeader)) == hipSuccess && hipMemset(c->d_hdr_fe, 0, sizeof(GridHeader)) == hipSuccess &&
              hipMalloc(&c->fit_ix.hdr, sizeof(GridHeader)) == hipSuccess &&
              hipMalloc(&c->sor_ix.hdr, sizeof(GridHeader)) == hipSuccess &&
              hipHostMalloc(&c->h_hdr, sizeof(GridHeader), hipHostMallocDefault) == hipSuccess &&

              hipMalloc(&c->d_state, sizeof(AlignState)) == hipSuccess && hipMalloc(&c->d_state2, sizeof(AlignState)) == hipSuccess &&
              hipHostMalloc(&c->h_state, sizeof(AlignState), hipHostMallocCoherent) == hipSuccess &&
              hipHostMalloc(&c->h_rb, 8 * sizeof(unsigned long long), hipHostMallocCoherent) == hipSuccess &&
              hipMalloc(&c->d_clk, 4 * sizeof(unsigned long long)) == hipSuccess &&
              hipMalloc(&c->d_hist, sizeof(PassRecordDev) * c->hist_cap) == hipSuccess &&

              hipMalloc(&c->d_async, sizeof(ndt_ctx::AsyncOut)) == hipSuccess &&
              hipHostMalloc(&c->h_async, sizeof(ndt_ctx::AsyncOut), hipHostMallocDefault) == hipSuccess &&
              hipEventCreateWithFlags(&c->ev_fit, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->ev_ins, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->ev_tgt, hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        ndt_destroy(c);
        return NDT_ENOMEM;
    }
    std::memset(c->h_state, 0, sizeof(AlignState));
    std::memset(c->h_rb, 0, 8 * sizeof(unsigned long long));
    *out = c;
    return NDT_OK;
}

ndt_status ndt_set_params(ndt_ctx* c, const ndt_params* p) {
    if (!c || !valid_params(p)) return fail(c, NDT_EINVAL, "invalid params");
    if (p->device != c->device) return fail(c, NDT_EINVAL, "device cannot change on an existing ctx");
    // pclomp::setResolution (ndt_omp.h:127-137): re-init the grid only when the resolution changed AND a
    // source is set; otherwise the grid keeps its leaf size until the next setInputTarget.
    const bool res_changed = p->resolution != c->prm.resolution;
    // the ndt_cpu backend (precision_mode 2) keeps its own cpu::VoxelGrid (division binning, its eigen solver): a
    // change between it and the pclomp/pcl grids rebuilds the target as a fresh setInputTarget would
    const bool grid_kind_changed = (p->precision_mode == 2) != (c->prm.precision_mode == 2);
    c->prm = *p;
    c->inc_ok = false;  // the next target is built from scratch under the new parameters
    invalidate_graph(c);
    if (c->has_target && ((res_changed && c->has_source) || grid_kind_changed)) {
        TRY(set_dev(c));
        TRY(build_target(c));
    }
    return NDT_OK;
}

ndt_status ndt_set_target(ndt_ctx* c, const float* xyz, size_t n, size_t stride_bytes, int is_dense) {
    if (!c || (n && !xyz) || stride_bytes < 12 || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad target");
    TRY(set_dev(c));
    TRY(main_after_fit(c, false));  // the fit lane may still read the owned copy
    TRY(upload_points(c, c->target, xyz, n, stride_bytes));
    c->target_ptr = c->target.p;
    c->M = (int)n;
    c->target_dense = is_dense ? 1 : 0;
    c->has_target = true;
    return build_target(c);
}

ndt_status ndt_set_target_device(ndt_ctx* c, const float* d_xyz4, size_t n, int is_dense) {
    if (!c || (n && !d_xyz4) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad target");
    TRY(set_dev(c));
    // like pcl::Registration::setInputTarget the cloud is referenced, not copied: the caller keeps the
    // device buffer alive and unmodified while this ctx uses it (until the next set_target)
    c->target_ptr = reinterpret_cast<const float4*>(d_xyz4);
    c->M = (int)n;
    c->target_dense = is_dense ? 1 : 0;
    c->has_target = true;
    return build_target(c);
}

// setInputTarget of a cloud that extends the current target: its first n_old points are the current target's (same
// values, same order) and n_new follow (odom_node.cpp:233 / 349 between localmap resets: pc_target_ is the localmap,
// which only grows by appends).  The grid is the one ndt_set_target_device builds; when the current sort can be reused
// it is built by merging the new points' sort into it (enqueue_target_append), otherwise from scratch.
ndt_status ndt_set_target_append_device(ndt_ctx* c, float* d_xyz4, size_t n_old, size_t n_new, int is_dense,
                                        const float* d_new4) {
    if (!c || ((n_old + n_new) && !d_xyz4) || n_old + n_new > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad target");
    TRY(set_dev(c));
    const float4* new_src = reinterpret_cast<const float4*>(d_new4);
    if (new_src == reinterpret_cast<const float4*>(d_xyz4) + n_old) new_src = nullptr;  // already in place
    const size_t m = n_old + n_new;
    const bool disabled = std::getenv("NDT_NO_TARGET_MERGE") != nullptr;  // A/B runs and tests
    const bool merge = !disabled && c->inc_ok && c->has_target && c->grid_valid && is_dense && c->target_dense == 1 &&
                       (size_t)c->M == n_old && n_old > 0 && c->grid_res == c->prm.resolution && c->prm.precision_mode != 2 &&
                       c->s.k0.cap >= m && c->s.v0.cap >= m && c->s.k1.cap >= m && c->s.v1.cap >= m;
    c->target_ptr = reinterpret_cast<const float4*>(d_xyz4);
    c->M = (int)m;
    c->target_dense = is_dense ? 1 : 0;
    c->has_target = true;
    if (!merge) {
        if (new_src && n_new)
            TRY(ndt_memcpy_d2d(c, d_xyz4 + 4 * n_old, d_new4, n_new * sizeof(float4)));
        return build_target(c);
    }
    ++c->tgt_gen;
    c->tgt_ev_valid = c->fit_tgt_used;
    if (c->tgt_ev_valid && !new_src) HIPCHK(c, hipEventRecord(c->ev_tgt, c->stream));
    const ndt_status st = enqueue_target_append(c, (int)n_old, (int)n_new, new_src);
    if (st != NDT_OK) {
        c->inc_ok = false;
        return st;
    }
    ++c->n_builds_merge;
    c->build_unchecked = true;
    c->built_since_align = true;
    c->grid_valid = true;
    c->fit_valid = false;
    c->grid_res = c->prm.resolution;
    c->have_result = false;
    return NDT_OK;
}

// cpu::NormalDistributionsTransform::updateVoxelGrid (ndt_cpu/NormalDistributionsTransform.h:39, driven at
// odom_node.cpp:344-345 when incremental voxel update is on): the new points join the target after the old ones.  The
// cpu::VoxelGrid keeps per-voxel sums that the new points extend in input order, so every voxel's statistics equal those
// of a grid built over old + new points in that order; the device appends the points to its owned target copy and
// rebuilds the grid (one sort of the whole target, ~0.2 ms for 2 M points).  Known difference: ndt_cpu's incremental
// path leaves a voxel that was rejected (points_per_voxel = -1) and then receives points with a count of -1 + k, which
// hides it from radiusSearch; the rebuild counts it afresh.
static ndt_status append_target(ndt_ctx* c, const float4* d_new, const float* h_new, size_t n, size_t stride_bytes) {
    TRY(set_dev(c));
    TRY(main_after_fit(c, false));  // the fit lane may still read the owned copy
    if (n == 0) return NDT_OK;
    const size_t m0 = c->has_target ? (size_t)c->M : 0, m = m0 + n;
    if (m > 0x7fffffffULL) return fail(c, NDT_EINVAL, "target too large");
    if (c->target_ptr != c->target.p || c->target.cap < m) {
        // a larger owned buffer (or the first owned copy of a caller-referenced target), old points first
        DevBuf<float4> nb;
        TRY(ensure(c, nb, std::max(m, m0 + m0 / 2)));
        if (m0) HIPCHK(c, hipMemcpyAsync(nb.p, c->target_ptr, m0 * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        release(c->target);
        c->target = nb;
        nb.p = nullptr;
        nb.cap = 0;
    }
    if (d_new) {
        HIPCHK(c, hipMemcpyAsync(c->target.p + m0, d_new, n * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
    } else {
        std::vector<float4> tmp(n);
        const char* base = reinterpret_cast<const char*>(h_new);
        for (size_t i = 0; i < n; ++i) {
            const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
            tmp[i] = make_float4(f[0], f[1], f[2], 1.0f);
        }
        HIPCHK(c, hipMemcpyAsync(c->target.p + m0, tmp.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    c->target_ptr = c->target.p;
    c->M = (int)m;
    if (!c->has_target) c->target_dense = 1;
    c->has_target = true;
    return build_target(c);
}

ndt_status ndt_update_target(ndt_ctx* c, const float* xyz, size_t n, size_t stride_bytes) {
    if (!c || (n && !xyz) || stride_bytes < 12 || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad target update");
    return append_target(c, nullptr, xyz, n, stride_bytes);
}

ndt_status ndt_update_target_device(ndt_ctx* c, const float* d_xyz4, size_t n) {
    if (!c || (n && !d_xyz4) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad target update");
    return append_target(c, reinterpret_cast<const float4*>(d_xyz4), nullptr, n, 16);
}

ndt_status ndt_set_source(ndt_ctx* c, const float* xyz, size_t n, size_t stride_bytes) {
    if (!c || (n && !xyz) || stride_bytes < 12 || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad source");
    TRY(set_dev(c));
    const float4* old = c->source.p;
    TRY(main_after_fit(c, true));  // a fitness query may still read the source
    TRY(ensure(c, c->source, geom_points((int)n)));
    c->src_pend = nullptr;  // replaced before it was copied
    TRY(upload_points(c, c->source, xyz, n, stride_bytes));
    if (c->source.p != old) invalidate_graph(c);  // a new size alone keeps the chains (geom_points)
    c->N = (int)n;
    c->has_source = true;
    c->have_result = false;
    return NDT_OK;
}

ndt_status ndt_set_source_device(ndt_ctx* c, const float* d_xyz4, size_t n) {
    if (!c || (n && !d_xyz4) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad source");
    TRY(set_dev(c));
    const float4* old = c->source.p;
    TRY(main_after_fit(c, true));  // a fitness query may still read the source
    TRY(ensure(c, c->source, geom_points((int)n)));
    if (c->source.p != old) invalidate_graph(c);  // a new size alone keeps the chains (geom_points)
    // the copy is deferred: the next align does it in its k_align_init (one launch less), any other reader of the source
    // first (flush_source); stream order is unchanged (nothing between reads the ctx source)
#ifndef NDT_DEFER_SOURCE
#define NDT_DEFER_SOURCE 1
#endif
    c->src_pend = n ? reinterpret_cast<const float4*>(d_xyz4) : nullptr;
    c->N = (int)n;
    if (!NDT_DEFER_SOURCE) TRY(flush_source(c));
    c->has_source = true;
    c->have_result = false;
    return NDT_OK;
}

ndt_status ndt_align(ndt_ctx* c, const float guess[16], ndt_result* out) {
    if (!c || !guess || !out) return fail(c, NDT_EINVAL, "null argument");
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (!c->has_source || c->N == 0) return fail(c, NDT_ENOSOURCE, "no input source");
    if (c->al_inflight) return fail(c, NDT_EINVAL, "an asynchronous align is in flight (ndt_align_wait first)");
    TRY(set_dev(c));
    if (!c->grid_valid) TRY(build_target(c));
    TRY(run_align(c, guess));
    fill_result(c, out);
    return NDT_OK;
}

ndt_status ndt_get_output(ndt_ctx* c, float* xyz, size_t stride_bytes) {
    if (!c || !xyz || stride_bytes < 12) return fail(c, NDT_EINVAL, "bad output");
    if (!c->have_result) return fail(c, NDT_EINVAL, "no align result");
    TRY(set_dev(c));
    TRY(flush_source(c));
    TRY(ensure(c, c->out_cloud, c->N));
    hipLaunchKernelGGL(k_transform, dim3(std::max(1, ceil_div(c->N, kBlock))), dim3(kBlock), 0, c->stream, c->source.p, c->N, c->d_state,
                       c->out_cloud.p);
    std::vector<float4> tmp(c->N);
    if (c->N) HIPCHK(c, hipMemcpyAsync(tmp.data(), c->out_cloud.p, c->N * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    char* base = reinterpret_cast<char*>(xyz);
    for (int i = 0; i < c->N; ++i) {
        float* f = reinterpret_cast<float*>(base + (size_t)i * stride_bytes);
        f[0] = tmp[i].x; f[1] = tmp[i].y; f[2] = tmp[i].z;
    }
    return NDT_OK;
}

ndt_status ndt_get_history(ndt_ctx* c, ndt_pass_record* out, int cap, int* n_out) {
    if (!c || !n_out || (cap > 0 && !out)) return fail(c, NDT_EINVAL, "bad history args");
    TRY(set_dev(c));
    const int n = std::min(std::min(c->h_state->hist_count, c->hist_cap), std::max(cap, 0));
    std::vector<PassRecordDev> tmp(n);
    if (n) HIPCHK(c, hipMemcpy(tmp.data(), c->d_hist, n * sizeof(PassRecordDev), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        out[i].kind = tmp[i].kind;
        out[i].newton_iter = tmp[i].newton_iter;
        for (int k = 0; k < 6; ++k) { out[i].x[k] = tmp[i].x[k]; out[i].g[k] = tmp[i].g[k]; }
        out[i].score = tmp[i].score;
        for (int k = 0; k < 36; ++k) out[i].H[k] = tmp[i].H[k];
        out[i].pairs = tmp[i].pairs;
    }
    *n_out = std::min(c->h_state->hist_count, c->hist_cap);
    return NDT_OK;
}


static ndt_status single_pass(ndt_ctx* c, const double p[6], const float T[16], int kind, bool force_radius, double* res44) {
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (!c->has_source || c->N == 0) return fail(c, NDT_ENOSOURCE, "no input source");
    TRY(set_dev(c));
    if (!c->grid_valid) TRY(build_target(c));
    TRY(settle_build(c));
    TRY(flush_source(c));
    TRY(ensure_align_buffers(c));
    TRY(ensure(c, c->reduce_out, kNumAcc));
    c->pass_src = c->source.p;
    AlignState* st = c->h_state;
    init_state(c, T, st);
    for (int k = 0; k < 16; ++k) st->T[k] = T[k];
    for (int k = 0; k < 6; ++k) { st->p[k] = p[k]; st->x_eval[k] = p[k]; st->x_t[k] = p[k]; }
    angle_tables(p, st->jang, st->hang, st->jang_d, st->hang_d);
    st->pass_kind = kind;
    st->pending = 1;
    HIPCHK(c, hipMemcpyAsync(c->d_state, st, sizeof(AlignState), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->counter.p, 0, kPassCounterWords * sizeof(unsigned), c->stream));
    if (kind == PASS_HESS || force_radius || !needs_direct(c->prm)) launch_radius(c, 1);
    else launch_pass(c, 1);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(res44, c->reduce_out.p, kNumAcc * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    // the target's cell count sizes the next dense grid, as an align's read-back does (align_finish)
    long long cells = 0;
    HIPCHK(c, hipMemcpyAsync(&cells, &c->d_hdr->cells, sizeof(cells), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->grid_cells_seen = std::max(c->grid_cells_seen, cells);
    c->have_result = false;
    return NDT_OK;
}

ndt_status ndt_derivatives(ndt_ctx* c, const double p[6], const float T[16], int compute_hessian, double* score, double g[6], double H[36],
                           long long* pairs) {
    if (!c || !p || !T) return fail(c, NDT_EINVAL, "null argument");
    double r[kNumAcc];
    TRY(single_pass(c, p, T, compute_hessian ? PASS_FULL : PASS_GRAD, false, r));
    if (score) *score = r[0];
    if (g) for (int k = 0; k < 6; ++k) g[k] = r[1 + k];
    if (H) for (int k = 0; k < 36; ++k) H[k] = r[7 + k];
    if (pairs) *pairs = (long long)r[43];
    return NDT_OK;
}

ndt_status ndt_hessian_radius(ndt_ctx* c, const double p[6], const float T[16], double H[36], long long* pairs) {
    if (!c || !p || !T) return fail(c, NDT_EINVAL, "null argument");
    double r[kNumAcc];
    TRY(single_pass(c, p, T, PASS_HESS, true, r));
    if (H) for (int k = 0; k < 36; ++k) H[k] = r[7 + k];
    if (pairs) *pairs = (long long)r[43];
    return NDT_OK;
}

ndt_status ndt_calculate_score(ndt_ctx* c, const float T[16], double* out) {
    if (!c || !T || !out) return fail(c, NDT_EINVAL, "null argument");
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (!c->has_source || c->N == 0) return fail(c, NDT_ENOSOURCE, "no input source");
    TRY(set_dev(c));
    if (!c->grid_valid) TRY(build_target(c));
    TRY(settle_build(c));
    TRY(flush_source(c));
    const int nb = std::max(1, std::min(ceil_div(c->N, kBlock), 1024));
    TRY(ensure(c, c->score_part, nb));
    Mat4f Tm;
    for (int k = 0; k < 16; ++k) Tm.m[k] = T[k];
    const double d1 = c->gauss_cur[0], d2 = c->gauss_cur[1], d3 = c->gauss_cur[2];
    hipLaunchKernelGGL(k_score_radius, dim3(nb), dim3(kBlock), 0, c->stream, c->source.p, c->N, Tm, c->d_hdr, c->table.p, c->grid.p,
                       c->recs.p, c->cent.p, c->icovd.p, d1, d2, d3, c->prm.resolution, c->score_part.p);
    HIPCHK(c, hipGetLastError());
    std::vector<double> part(nb);
    HIPCHK(c, hipMemcpyAsync(part.data(), c->score_part.p, nb * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double score = 0.0;
    for (int b = 0; b < nb; ++b) score += part[b];
    *out = score / (double)c->N;
    return NDT_OK;
}

// nearest-neighbour index over all target points (built on the first fitness query after a target change)
// Builds an NNIndex over n device points (cell = base cell size, doubled by k_header until the block-major key range
// fits).  Uses the ctx's sort scratch; stream-ordered.
ndt_status enqueue_nn_index(ndt_ctx* c, Lane L, const float4* pts, int n, int dense, float cell, NNIndex& ix) {
    TRY(enqueue_bin_and_sort(c, L, pts, n, dense, ix.hdr, cell, 1));
    TRY(ensure(c, ix.pts, std::max(n, 1))); TRY(ensure(c, ix.keys, std::max(n, 1))); TRY(ensure(c, ix.start, (size_t)n + 1));
    const int nb = std::max(1, std::min(ceil_div(n, kBlock), 4096));
    hipLaunchKernelGGL(k_fit_gather, dim3(nb), dim3(kBlock), 0, L.st, pts, L.s.k0.p, L.s.k1.p, L.s.v0.p, L.s.v1.p,
                       L.s.seg_start.p, n, ix.hdr, ix.pts.p, ix.keys.p, ix.start.p);
    // occupied blocks: flags -> exclusive scan -> block table + 513 cell offsets per occupied block
    const size_t max_occ = (size_t)std::max(1, std::min(n, kFitMaxBlocks));
    TRY(ensure(c, L.s.flags, std::max(n, 1))); TRY(ensure(c, L.s.cloud_idx, std::max(n, 1)));
    TRY(ensure(c, ix.blk, (size_t)kFitMaxBlocks)); TRY(ensure(c, ix.off, max_occ * (kFitBlockCells + 1)));
    const int nb_pts = std::max(1, ceil_div(n, kBlock));
    hipLaunchKernelGGL(k_fit_block_flags, dim3(nb_pts), dim3(kBlock), 0, L.st, ix.keys.p, ix.hdr, L.s.flags.p);
    TRY(enqueue_scan(c, L, L.s.flags.p, std::max(n, 1), &ix.hdr->n_leaves, L.s.cloud_idx.p, &ix.hdr->n_blocks_occ, ix.hdr));
    hipLaunchKernelGGL(k_fit_block_clear, dim3(std::max(1, std::min(kFitMaxBlocks / kBlock, 256))), dim3(kBlock), 0, L.st,
                       ix.blk.p, ix.hdr);
    hipLaunchKernelGGL(k_fit_tables, dim3(nb_pts), dim3(kBlock), 0, L.st, ix.keys.p, ix.start.p, L.s.flags.p,
                       L.s.cloud_idx.p, ix.hdr, ix.blk.p, ix.off.p);
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

// getFitnessScore's index over the current target, queued on the fit lane behind the target's points (ev_tgt, recorded
// ahead of the voxel build, so the two builds run side by side); issued by the lane's host thread
ndt_status ensure_fit_index(ndt_ctx* c) {
    TRY(side_lanes(c));
    if (c->fit_worker->failed()) {
        // a fit-lane job failed (possibly this index's build): report it now instead of querying a half-built index
        std::string msg;
        const ndt_status st = c->fit_worker->take_error(&msg);
        c->fit_valid = false;
        c->fit_pending = false;
        return fail(c, st, "getFitnessScore: " + msg);
    }
    if (c->fit_valid) return NDT_OK;
    const float4* pts = c->target_ptr;
    const int M = c->M, dense = c->target_dense;
    const float res = c->prm.resolution;
    if (!c->tgt_ev_valid) {  // the first index of this ctx: behind everything queued so far (the build included)
        HIPCHK(c, hipEventRecord(c->ev_tgt, c->stream));
        c->tgt_ev_valid = true;
    }
    c->fit_ix_gen = c->tgt_gen;
    c->fit_worker->post([c, pts, M, dense, res]() -> ndt_status {
        HIPCHK(c, hipStreamWaitEvent(c->fit_stream, c->ev_tgt, 0));
        // target points binned in 8x8x8-cell blocks (block-major keys, same stable radix sort as the voxel build)
        TRY(enqueue_nn_index(c, Lane{c->fit_stream, c->s_fit}, pts, M, dense, res, c->fit_ix));
        HIPCHK(c, hipEventRecord(c->ev_fit_tgt, c->fit_stream));
        return NDT_OK;
    });
    c->fit_tgt_used = true;
    c->fit_valid = true;
    return NDT_OK;
}

void release_nn_index(NNIndex& ix) {
    release(ix.pts); release(ix.keys); release(ix.start); release(ix.blk); release(ix.off);
    if (ix.hdr) (void)hipFree(ix.hdr);
    ix.hdr = nullptr;
}

// getFitnessScore of N device points src (the ctx's source, or a caller cloud that stays valid until the result call)
static ndt_status fitness_enqueue(ndt_ctx* c, const float* T, double max_range, const float4* src, int N, bool ctx_source,
                                  bool index_ready = false) {
    TRY(set_dev(c));
    if (!index_ready) TRY(ensure_fit_index(c));
    // getFitnessScore uses final_transformation_: the last align's result (identity before any align)
    Mat4f Tm;
    for (int k = 0; k < 16; ++k) Tm.m[k] = T ? T[k] : (c->have_result ? c->h_state->T[k] : (k % 5 == 0 ? 1.f : 0.f));
    // the query runs on the fit lane behind the main stream's work so far (the source copy, the align whose transform
    // it applies: the marker is recorded here, on the caller's thread) and beside whatever the main stream queues next
    if (c->lanes_marked & 1) c->lanes_marked &= ~1;  // the caller's mark (ndt_side_lanes_mark)
    else HIPCHK(c, hipEventRecord(c->ev_main_fit, c->stream));
    c->fit_worker->post([c, Tm, src, N, max_range, ctx_source]() -> ndt_status {
        HIPCHK(c, hipStreamWaitEvent(c->fit_stream, c->ev_main_fit, 0));
        // 16-lane team per query; the grid capped at 32 Ki workgroups (measured caps 8192 / 2048 / 1024 / 512 of 256-thread
        // workgroups: 89.4 / 85.9 / 90.7 / 128.9 us on C3)
        static const int grid_cap = [] {
            const char* e = std::getenv("NDT_FIT_GRID");  // A/B runs
            return e ? std::max(1, std::atoi(e)) : 8192 * (256 / NDT_FIT_BLOCK);
        }();
        const int nb = std::max(1, std::min(ceil_div(N, NDT_FIT_BLOCK / NDT_FIT_TEAM), grid_cap));
        const int ngrp = ceil_div(nb, kFitGroup);
        TRY(ensure(c, c->fit_sum, nb + ngrp)); TRY(ensure(c, c->fit_cnt, nb + ngrp)); TRY(ensure(c, c->fit_d2, N));
        const size_t n_ticket = (size_t)kFitTicketStride * (1 + ngrp);
        if (c->fit_ticket.cap < n_ticket) {
            TRY(ensure(c, c->fit_ticket, n_ticket));
            HIPCHK(c, hipMemsetAsync(c->fit_ticket.p, 0, c->fit_ticket.cap * sizeof(unsigned), c->fit_stream));
        }
        // the last workgroup sums the partials and writes (sum, count) straight into the pinned result slots
        hipLaunchKernelGGL(k_fitness, dim3(nb), dim3(NDT_FIT_BLOCK), 0, c->fit_stream, src, N, Tm, c->fit_ix.hdr, c->fit_ix.blk.p,
                           c->fit_ix.off.p, c->fit_ix.pts.p, max_range, c->fit_d2.p, c->fit_sum.p, c->fit_cnt.p, c->fit_ticket.p,
                           &c->h_async->fit_sum, &c->h_async->fit_cnt);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipEventRecord(c->ev_fit, c->fit_stream));
        if (ctx_source) HIPCHK(c, hipEventRecord(c->ev_fit_src, c->fit_stream));
        return NDT_OK;
    });
    if (ctx_source) c->fit_src_used = true;
    c->fit_pending = true;
    c->fit_n = N;
    return NDT_OK;
}

ndt_status ndt_fitness_score_async(ndt_ctx* c, const float* T, double max_range) {
    if (!c) return NDT_EINVAL;
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (!c->has_source || c->N == 0) return fail(c, NDT_ENOSOURCE, "no input source");
    TRY(set_dev(c));
    TRY(flush_source(c));  // the query reads the ctx source on the fit lane, behind the main stream's work so far
    return fitness_enqueue(c, T, max_range, c->source.p, c->N, true);
}

ndt_status ndt_fitness_score_async_cloud(ndt_ctx* c, const float* T, double max_range, const float* d_src4, size_t n) {
    if (!c || (n && !d_src4) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad fitness cloud");
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (n == 0) return fail(c, NDT_ENOSOURCE, "empty fitness cloud");
    return fitness_enqueue(c, T, max_range, reinterpret_cast<const float4*>(d_src4), (int)n, false);
}

// getFitnessScore of the last align against the target it aligned to, callable after setInputTarget has replaced that
// target (odom_node.cpp:280 runs before :349; queuing the query after the new target's build lets the build's first
// kernels start before the query fills the CUs).  Needs that target's index queued (ndt_fitness_index_async after its
// setInputTarget); the query is queued ahead of the new target's index build on the fit lane (FIFO).
ndt_status ndt_fitness_score_async_aligned(ndt_ctx* c, double max_range, const float* d_src4, size_t n) {
    if (!c || (n && !d_src4) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad fitness cloud");
    if (n == 0) return fail(c, NDT_ENOSOURCE, "empty fitness cloud");
    if (c->align_tgt_gen == ~0ull) return fail(c, NDT_EINVAL, "no align result");
    TRY(set_dev(c));
    if (c->align_tgt_gen == c->tgt_gen) {  // the target has not changed since the align
        float T[16];
        for (int k = 0; k < 16; ++k) T[k] = c->h_state->T[k];
        return fitness_enqueue(c, T, max_range, reinterpret_cast<const float4*>(d_src4), (int)n, false);
    }
    if (c->fit_ix_gen != c->align_tgt_gen || !c->fit_worker || c->fit_worker->failed())
        return fail(c, NDT_EINVAL, "getFitnessScore: the aligned target's index was not queued before setInputTarget");
    float T[16];
    for (int k = 0; k < 16; ++k) T[k] = c->h_state->T[k];
    return fitness_enqueue(c, T, max_range, reinterpret_cast<const float4*>(d_src4), (int)n, false, true);
}

ndt_status ndt_fitness_index_async(ndt_ctx* c) {
    if (!c) return NDT_EINVAL;
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    TRY(set_dev(c));
    return ensure_fit_index(c);
}

ndt_status ndt_fitness_score_result(ndt_ctx* c, double* out) {
    if (!c || !out) return fail(c, NDT_EINVAL, "null argument");
    std::string msg;
    // a failed fit-lane job is taken (and cleared) even when no query is pending, so that it cannot stay stuck
    const ndt_status st = c->fit_worker ? c->fit_worker->take_error(&msg) : NDT_OK;  // every fit-lane job issued
    if (st == NDT_OK && !c->fit_pending) return fail(c, NDT_EINVAL, "no fitness score enqueued");
    TRY(set_dev(c));
    if (st != NDT_OK) {
        c->fit_pending = false;
        c->fit_valid = false;  // the index may not have been built
        return fail(c, st, "getFitnessScore: " + msg);
    }
    HIPCHK(c, hipEventSynchronize(c->ev_fit));
    const double sum = c->h_async->fit_sum;
    const long long cnt = c->h_async->fit_cnt;
    if (cnt < 0) {
        c->fit_valid = false;
        return fail(c, NDT_EDEVICE, "getFitnessScore: nearest-neighbour index sort: radix look-back timed out");
    }
    // Registration::getFitnessScore: mean of the squared distances <= max_range, DBL_MAX when none qualifies
    *out = cnt > 0 ? sum / (double)cnt : DBL_MAX;
    return NDT_OK;
}

ndt_status ndt_fitness_score(ndt_ctx* c, const float T[16], double max_range, double* out, float* nn_d2) {
    if (!c || !out) return fail(c, NDT_EINVAL, "null argument");
    TRY(ndt_fitness_score_async(c, T, max_range));
    if (nn_d2) {
        std::string msg;
        const ndt_status st = c->fit_worker->drain(&msg);  // the query has been issued (its failure is reported below)
        if (st == NDT_OK) {
            HIPCHK(c, hipMemcpyAsync(nn_d2, c->fit_d2.p, (size_t)c->fit_n * sizeof(float), hipMemcpyDeviceToHost, c->fit_stream));
            HIPCHK(c, hipStreamSynchronize(c->fit_stream));
        }
    }
    return ndt_fitness_score_result(c, out);
}

ndt_status ndt_keyframe_insert_async(ndt_ctx* c, const float T[16], const float* d_scan4, size_t n, float leaf, float* d_map_a, size_t n_a,
                                     float* d_map_b, size_t n_b) {
    if (!c || !T || (n && (!d_scan4 || !d_map_a || !d_map_b)) || !(leaf > 0.f) || n > 0x7fffffffULL)
        return fail(c, NDT_EINVAL, "bad keyframe insert args");
    TRY(set_dev(c));
    TRY(side_lanes(c));
    c->ins_n_in = n;
    c->ins_pending = true;
    // the insertion lane: behind the main stream's work so far (whatever wrote the scan or grew the maps; the marker is
    // recorded here, on the caller's thread), beside what the main stream queues next; its own binning header and sort
    // scratch, its launches issued by the lane's host thread
    hipEvent_t ev_main = c->ev_main_ins;
    if (c->lanes_marked & 2) {  // the caller's mark (ndt_side_lanes_mark)
        c->lanes_marked &= ~2;
        ev_main = c->ev_main_fit;
    } else {
        HIPCHK(c, hipEventRecord(c->ev_main_ins, c->stream));
    }
    Mat4f Tm;
    for (int k = 0; k < 16; ++k) Tm.m[k] = T[k];
    const float4* scan = reinterpret_cast<const float4*>(d_scan4);
    float4* dst_a = reinterpret_cast<float4*>(d_map_a) + n_a;
    float4* dst_b = reinterpret_cast<float4*>(d_map_b) + n_b;
    c->ins_worker->post([c, Tm, scan, n, leaf, dst_a, dst_b, ev_main]() -> ndt_status {
        if (n == 0) {
            HIPCHK(c, hipStreamSynchronize(c->ins_stream));  // no earlier insertion still writes the pinned header
            std::memset(&c->h_async->ins_hdr, 0, sizeof(GridHeader));
            c->h_async->ins_hdr.empty = 1;
            HIPCHK(c, hipEventRecord(c->ev_ins, c->ins_stream));
            return NDT_OK;
        }
        const Lane L{c->ins_stream, c->s_ins};
        HIPCHK(c, hipStreamWaitEvent(L.st, ev_main, 0));
        TRY(ensure(c, c->ins_tr, n)); TRY(ensure(c, c->ins_ds, n));
        hipLaunchKernelGGL(k_transform_mat, dim3(ceil_div((long long)n, kBlock)), dim3(kBlock), 0, L.st, scan, (int)n, Tm, c->ins_tr.p);
        TRY(enqueue_bin_and_sort(c, L, c->ins_tr.p, (int)n, 1, c->d_hdr_ins, leaf));
        TRY(enqueue_downsample_finalize(c, L, c->d_hdr_ins, c->ins_tr.p, (int)n, c->ins_ds.p));
        hipLaunchKernelGGL(k_append2, dim3(std::max(1, std::min(ceil_div((long long)n, kBlock), 1024))), dim3(kBlock), 0, L.st,
                           c->ins_ds.p, c->ins_tr.p, (int)n, c->d_hdr_ins, dst_a, dst_b);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(&c->h_async->ins_hdr, c->d_hdr_ins, sizeof(GridHeader), hipMemcpyDeviceToHost, L.st));
        HIPCHK(c, hipEventRecord(c->ev_ins, L.st));
        return NDT_OK;
    });
    return NDT_OK;
}

ndt_status ndt_side_lanes_mark(ndt_ctx* c) {
    if (!c) return NDT_EINVAL;
    TRY(set_dev(c));
    TRY(side_lanes(c));
    HIPCHK(c, hipEventRecord(c->ev_main_fit, c->stream));
    c->lanes_marked = 3;
    return NDT_OK;
}

ndt_status ndt_keyframe_insert_result(ndt_ctx* c, size_t* n_inserted) {
    if (!c || !n_inserted) return fail(c, NDT_EINVAL, "null argument");
    if (!c->ins_pending) return fail(c, NDT_EINVAL, "no keyframe insertion enqueued");
    TRY(set_dev(c));
    std::string msg;
    const ndt_status st = c->ins_worker->take_error(&msg);  // the insertion has been issued
    if (st != NDT_OK) {
        c->ins_pending = false;
        return fail(c, st, "keyframe insertion: " + msg);
    }
    HIPCHK(c, hipEventSynchronize(c->ev_ins));
    const GridHeader& h = c->h_async->ins_hdr;
    if (h.pad[0]) return fail(c, NDT_EDEVICE, "keyframe insertion: VoxelGrid sort: radix look-back timed out");
    *n_inserted = h.overflow ? c->ins_n_in : (h.empty ? 0 : (size_t)h.n_leaves);
    return h.overflow ? NDT_EOVERFLOW : NDT_OK;
}

ndt_status ndt_grid_info(ndt_ctx* c, int header[16]) {
    if (!c || !header) return fail(c, NDT_EINVAL, "null argument");
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    TRY(set_dev(c));
    if (!c->grid_valid) TRY(build_target(c));
    TRY(settle_build(c));
    HIPCHK(c, hipMemcpyAsync(c->h_hdr, c->d_hdr, sizeof(GridHeader), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const GridHeader& h = *c->h_hdr;
    c->grid_cells_seen = std::max(c->grid_cells_seen, h.cells);
    for (int a = 0; a < 3; ++a) { header[a] = h.min_b[a]; header[3 + a] = h.max_b[a]; header[6 + a] = h.div_b[a]; header[9 + a] = h.divb_mul[a]; }
    header[12] = h.n_leaves;
    header[13] = h.n_cloud;
    header[14] = h.overflow;
    // usable voxels: the finalize's per-wave counts
    long long nv = 0;
    if (h.n_cloud > 0 && !h.empty) {
        std::vector<int> part((size_t)(h.n_cloud + 63) / 64);
        HIPCHK(c, hipMemcpy(part.data(), c->valid_part.p, part.size() * sizeof(int), hipMemcpyDeviceToHost));
        for (int v : part) nv += v;
    }
    header[15] = (int)nv;
    return NDT_OK;
}

ndt_status ndt_grid_leaves(ndt_ctx* c, int* keys, int* npts, double* mean, double* icov9, float* centroid3, int cap, int* n_out) {
    int hdr[16];
    TRY(ndt_grid_info(c, hdr));
    const int n = std::min(hdr[13], std::max(cap, 0));
    *n_out = hdr[13];
    if (n == 0) return NDT_OK;
    std::vector<VoxelRec> r(n);
    std::vector<float4> ce(n);
    std::vector<int> k(n);
    std::vector<double> ic((size_t)n * 9);
    HIPCHK(c, hipMemcpy(r.data(), c->recs.p, n * sizeof(VoxelRec), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(ce.data(), c->cent.p, n * sizeof(float4), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(k.data(), c->cloud_key.p, n * sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(ic.data(), c->icovd.p, (size_t)n * 9 * sizeof(double), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        if (keys) keys[i] = k[i];
        if (npts) npts[i] = r[i].npts;
        if (mean) for (int a = 0; a < 3; ++a) mean[3 * i + a] = r[i].mean[a];
        if (icov9) for (int a = 0; a < 9; ++a) icov9[9 * i + a] = ic[(size_t)9 * i + a];
        if (centroid3) { centroid3[3 * i] = ce[i].x; centroid3[3 * i + 1] = ce[i].y; centroid3[3 * i + 2] = ce[i].z; }
    }
    return NDT_OK;
}

ndt_status ndt_align_async(ndt_ctx* c, const float guess[16]) {
    if (!c || !guess) return fail(c, NDT_EINVAL, "null argument");
    if (!c->has_target) return fail(c, NDT_ENOTARGET, "no input target");
    if (!c->has_source || c->N == 0) return fail(c, NDT_ENOSOURCE, "no input source");
    if (c->al_inflight) return fail(c, NDT_EINVAL, "an align is already in flight on this context");
    TRY(set_dev(c));
    if (!c->grid_valid) TRY(build_target(c));
    return align_enqueue(c, guess);
}

ndt_status ndt_align_wait(ndt_ctx* c, ndt_result* out) {
    if (!c || !out) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    TRY(align_finish(c));
    fill_result(c, out);
    return NDT_OK;
}

// Batched offline replay on this device: pairs round-robin over the context and its helper contexts (one HIP stream
// each, three in flight), every context keeping one registration in flight, so that one pair's target
// build and pass-kernel tails overlap another pair's passes.  Each pair runs exactly the code of a single align:
// results are bit-identical to registering the pairs one by one.
ndt_status ndt_align_batch(ndt_ctx* c, const ndt_pair_desc* pairs, int n_pairs, ndt_result* out) {
    if (!c || (n_pairs > 0 && (!pairs || !out))) return fail(c, NDT_EINVAL, "bad batch");
    TRY(set_dev(c));
    // three registrations in flight (measured on C4 pairs: 2 streams 1257, 3 streams 1385, 4 streams 1193 pairs/s — the
    // 4th stream competes for the process's 4 hardware queues and the pass bodies already fill every CU)
    int streams = 3;
    if (const char* e = std::getenv("NDT_BATCH_STREAMS")) streams = std::max(1, std::min(16, std::atoi(e)));  // A/B runs
    streams = std::max(1, std::min(streams, n_pairs));
    while ((int)c->helpers.size() < streams - 1) {
        ndt_ctx* h = nullptr;
        ndt_params p = c->prm;
        p.device = c->device;
        TRY(ndt_create(&p, &h));
        c->helpers.push_back(h);
    }
    std::vector<ndt_ctx*> ctxs(1, c);
    for (int k = 0; k < streams - 1; ++k) {
        ndt_ctx* h = c->helpers[k];
        h->prm = c->prm;
        h->profiling = c->profiling;
        // the ctx's pass / build options (a helper created after ndt_set_pass_options / ndt_set_build_options gets them too)
        h->opt_lead_tail = c->opt_lead_tail;
        h->opt_ppt = c->opt_ppt;
        h->order_source = c->order_source;
        h->radix_force = c->radix_force;
        h->tile_tickets = h->tile_tickets || c->tile_tickets;
        ctxs.push_back(h);
    }
    // every registration in flight spreads its passes over all CUs (spreading each over n_cu / streams CUs was
    // measured neutral) and keeps last-workgroup tails (the other streams' bodies fill the CUs a tail leaves idle)
    // (A/B: NDT_BATCH_LEAD=1 lets them run leading-tail chains)
    static const bool batch_lead = std::getenv("NDT_BATCH_LEAD") != nullptr;
    for (ndt_ctx* x : ctxs) x->no_lead = streams > 1 && !batch_lead;
    std::vector<int> slot_pair(streams, -1);
    ndt_status rs = NDT_OK;
    auto drain = [&](int k) -> ndt_status {
        if (slot_pair[k] < 0) return NDT_OK;
        ndt_status st = ndt_align_wait(ctxs[k], &out[slot_pair[k]]);
        if (st != NDT_OK && ctxs[k] != c) c->err = ctxs[k]->err;
        slot_pair[k] = -1;
        return st;
    };
    for (int i = 0; i < n_pairs && rs == NDT_OK; ++i) {
        const int k = i % streams;
        if ((rs = drain(k)) != NDT_OK) break;
        ndt_ctx* x = ctxs[k];
        if ((rs = ndt_set_target_device(x, pairs[i].d_target_xyz4, pairs[i].n_target, 1)) == NDT_OK &&
            (rs = ndt_set_source_device(x, pairs[i].d_source_xyz4, pairs[i].n_source)) == NDT_OK &&
            (rs = ndt_align_async(x, pairs[i].guess)) == NDT_OK)
            slot_pair[k] = i;
        if (rs != NDT_OK && x != c) c->err = x->err;
    }
    for (int k = 0; k < streams; ++k) {
        const ndt_status st = drain(k);
        if (rs == NDT_OK) rs = st;
    }
    c->no_lead = false;
    return rs;
}

ndt_status ndt_voxel_downsample(ndt_ctx* c, const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset, float leaf, float* out4,
                                size_t cap, size_t* n_out) {
    if (!c || (n && !xyzi) || !n_out || stride_bytes < 16 || !(leaf > 0.f) || intensity_offset < 3 ||
        (size_t)intensity_offset * 4 + 4 > stride_bytes || n > 0x7fffffffULL)
        return fail(c, NDT_EINVAL, "bad downsample args");
    TRY(set_dev(c));
    *n_out = 0;
    if (n == 0) return NDT_OK;
    DevBuf<float4> in, outb;
    std::vector<float4> tmp(n);
    const char* base = reinterpret_cast<const char*>(xyzi);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        tmp[i] = make_float4(f[0], f[1], f[2], f[intensity_offset]);
    }
    ndt_status st = ensure(c, in, n);
    if (st == NDT_OK) st = ensure(c, outb, n);
    if (st != NDT_OK) { release(in); release(outb); return st; }
    ndt_status rs = NDT_OK;
    do {
        if (hipMemcpyAsync(in.p, tmp.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream) != hipSuccess) { rs = fail(c, NDT_EDEVICE, "copy"); break; }
        const bool saved_grid = c->grid_valid;
        rs = enqueue_bin_and_sort(c, main_lane(c), in.p, (int)n, 1, c->d_hdr_ds, leaf);
        c->grid_valid = saved_grid;
        if (rs != NDT_OK) break;
        if ((rs = enqueue_downsample_finalize(c, main_lane(c), c->d_hdr_ds, in.p, (int)n, outb.p)) != NDT_OK) break;
        if (hipMemcpyAsync(c->h_hdr, c->d_hdr_ds, sizeof(GridHeader), hipMemcpyDeviceToHost, c->stream) != hipSuccess) { rs = fail(c, NDT_EDEVICE, "copy"); break; }
        if (hipStreamSynchronize(c->stream) != hipSuccess) { rs = fail(c, NDT_EDEVICE, "sync"); break; }
        const GridHeader h = *c->h_hdr;
        if (h.pad[0]) { rs = fail(c, NDT_EDEVICE, "voxel downsample: radix look-back timed out"); break; }
        if (h.overflow) {
            // pcl::VoxelGrid: "Leaf size is too small" -> output = input copy
            const size_t m = std::min(cap, n);
            for (size_t i = 0; i < m; ++i) { out4[4 * i] = tmp[i].x; out4[4 * i + 1] = tmp[i].y; out4[4 * i + 2] = tmp[i].z; out4[4 * i + 3] = tmp[i].w; }
            *n_out = n;
            rs = NDT_EOVERFLOW;
            c->err = "voxel downsample: leaf size too small, output = input";
            break;
        }
        const size_t m = std::min(cap, (size_t)h.n_leaves);
        std::vector<float4> o(m);
        if (m && hipMemcpy(o.data(), outb.p, m * sizeof(float4), hipMemcpyDeviceToHost) != hipSuccess) { rs = fail(c, NDT_EDEVICE, "copy"); break; }
        for (size_t i = 0; i < m; ++i) { out4[4 * i] = o[i].x; out4[4 * i + 1] = o[i].y; out4[4 * i + 2] = o[i].z; out4[4 * i + 3] = o[i].w; }
        *n_out = (size_t)h.n_leaves;
    } while (0);
    release(in);
    release(outb);
    return rs;
}

ndt_status ndt_transform_device(ndt_ctx* c, const float T[16], const float* d_in4, size_t n, float* d_out4) {
    if (!c || !T || (n && (!d_in4 || !d_out4)) || n > 0x7fffffffULL) return fail(c, NDT_EINVAL, "bad transform args");
    TRY(set_dev(c));
    if (n == 0) return NDT_OK;
    Mat4f Tm;
    for (int k = 0; k < 16; ++k) Tm.m[k] = T[k];
    hipLaunchKernelGGL(k_transform_mat, dim3(ceil_div((long long)n, kBlock)), dim3(kBlock), 0, c->stream,
                       reinterpret_cast<const float4*>(d_in4), (int)n, Tm, reinterpret_cast<float4*>(d_out4));
    HIPCHK(c, hipGetLastError());
    return NDT_OK;
}

ndt_status ndt_voxel_downsample_device(ndt_ctx* c, const float* d_in4, size_t n, float leaf, float* d_out4, size_t* n_out) {
    if (!c || !n_out || (n && (!d_in4 || !d_out4)) || !(leaf > 0.f) || n > 0x7fffffffULL)
        return fail(c, NDT_EINVAL, "bad downsample args");
    TRY(set_dev(c));
    *n_out = 0;
    if (n == 0) return NDT_OK;
    const float4* in = reinterpret_cast<const float4*>(d_in4);
    const bool saved_grid = c->grid_valid;
    ndt_status rs = enqueue_bin_and_sort(c, main_lane(c), in, (int)n, 1, c->d_hdr_ds, leaf);
    c->grid_valid = saved_grid;
    if (rs != NDT_OK) return rs;
    TRY(enqueue_downsample_finalize(c, main_lane(c), c->d_hdr_ds, in, (int)n, reinterpret_cast<float4*>(d_out4)));
    HIPCHK(c, hipMemcpyAsync(c->h_hdr, c->d_hdr_ds, sizeof(GridHeader), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->h_hdr->pad[0]) return fail(c, NDT_EDEVICE, "voxel downsample: radix look-back timed out");
    if (c->h_hdr->overflow) {
        // pcl::VoxelGrid: "Leaf size is too small for the input dataset" -> output = input copy
        HIPCHK(c, hipMemcpyAsync(d_out4, d_in4, n * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
        *n_out = n;
        c->err = "voxel downsample: leaf size too small, output = input";
        return NDT_EOVERFLOW;
    }
    *n_out = (size_t)c->h_hdr->n_leaves;
    return NDT_OK;
}


// ---------------------------------------------------------------- filter_node front end
ndt_status ndt_filter_default_params(ndt_filter_params* out) {
    if (!out) return NDT_EINVAL;
    out->leaf = 0.5f;
    out->r_min = 1.0;
    out->r_max = 60.0;
    out->mean_k = 30;
    out->stddev_mul = 1.0;
    out->outlier_method = 0;
    out->ror_radius = 0.8;
    out->ror_min_neighbors = 5;
    return NDT_OK;
}

ndt_status ndt_filter_scan_device(ndt_ctx* c, const ndt_filter_params* prm, const float* d_in4, size_t n, float* d_out4, size_t* n_out) {
    if (!c || !prm || !n_out || (n && (!d_in4 || !d_out4 || d_in4 == d_out4)) || n > 0x7fffffffULL || !(prm->leaf > 0.f) ||
        prm->mean_k < 1 || prm->mean_k > 63 || !(prm->r_min < prm->r_max) || prm->outlier_method < 0 || prm->outlier_method > 1 ||
        (prm->outlier_method == 1 && !(prm->ror_radius > 0.0)))
        return fail(c, NDT_EINVAL, "bad filter args");
    TRY(set_dev(c));
    *n_out = 0;
    c->fe_nvox = 0;
    if (n == 0) return NDT_OK;
    const int N = (int)n;
    const float4* in = reinterpret_cast<const float4*>(d_in4);
    float4* out = reinterpret_cast<float4*>(d_out4);
    TRY(ensure(c, c->fe_flags, n)); TRY(ensure(c, c->fe_idx, n)); TRY(ensure(c, c->fe_crop, n));
    TRY(ensure(c, c->fe_ds, n)); TRY(ensure(c, c->fe_dist, n)); TRY(ensure(c, c->fe_thr, 4));
    const int nb = std::max(1, std::min(ceil_div(N, kBlock), 2048));
    // the compaction scans write their count to d_hdr_fe->pad[1] and raise a look-back timeout in d_hdr_fe->pad[0] (its own
    // header: the VoxelGrid build rewrites d_hdr_ds); both come back in one copy into pinned memory.  The flag is cleared
    // only after it was raised.
    int* fw = c->h_async->fe_words;
    auto scan_failed = [&](const char* what) -> ndt_status {
        (void)hipMemsetAsync(&c->d_hdr_fe->pad[0], 0, sizeof(int), c->stream);
        return fail(c, NDT_EDEVICE, std::string("filter: ") + what + " compaction scan: look-back timed out");
    };
    // 1. removeNaNFromPointCloud + range crop (filter_node.cpp:236-247), input order kept
    hipLaunchKernelGGL(k_crop_flags, dim3(nb), dim3(kBlock), 0, c->stream, in, N, prm->r_min, prm->r_max, c->fe_flags.p);
    TRY(enqueue_scan(c, main_lane(c), c->fe_flags.p, N, nullptr, c->fe_idx.p, &c->d_hdr_fe->pad[1], c->d_hdr_fe));
    hipLaunchKernelGGL(k_compact4, dim3(nb), dim3(kBlock), 0, c->stream, in, c->fe_flags.p, c->fe_idx.p, N, c->fe_crop.p);
    HIPCHK(c, hipMemcpyAsync(fw, &c->d_hdr_fe->pad[0], 2 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (fw[0]) return scan_failed("crop");
    const int m = fw[1];
    if (m == 0) return NDT_OK;
    // 2. VoxelGrid (filter_node.cpp:249-251)
    const bool saved_grid = c->grid_valid;
    ndt_status rs = enqueue_bin_and_sort(c, main_lane(c), c->fe_crop.p, m, 1, c->d_hdr_ds, prm->leaf);
    c->grid_valid = saved_grid;
    if (rs != NDT_OK) return rs;
    TRY(enqueue_downsample_finalize(c, main_lane(c), c->d_hdr_ds, c->fe_crop.p, m, c->fe_ds.p));
    HIPCHK(c, hipMemcpyAsync(c->h_hdr, c->d_hdr_ds, sizeof(GridHeader), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->h_hdr->pad[0]) return fail(c, NDT_EDEVICE, "filter: VoxelGrid sort: radix look-back timed out");
    int nv = c->h_hdr->n_leaves;
    if (c->h_hdr->overflow) {  // pcl::VoxelGrid: leaf too small -> output = input copy
        HIPCHK(c, hipMemcpyAsync(c->fe_ds.p, c->fe_crop.p, (size_t)m * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
        nv = m;
    }
    c->fe_nvox = (size_t)nv;
    const int nbq = std::max(1, std::min(ceil_div(nv, kBlock / 16), 16384));  // 16-lane team per query
    if (prm->outlier_method == 1) {
        // 3'. RadiusOutlierRemoval (filter_node.cpp:265-272): index cell just above the radius (one ring of cells)
        TRY(enqueue_nn_index(c, main_lane(c), c->fe_ds.p, nv, 1, (float)(1.01 * prm->ror_radius), c->sor_ix));
        hipLaunchKernelGGL(k_ror_keep, dim3(nbq), dim3(kBlock), 0, c->stream, c->fe_ds.p, nv, prm->ror_radius, prm->ror_min_neighbors,
                           c->sor_ix.hdr, c->sor_ix.blk.p, c->sor_ix.off.p, c->sor_ix.pts.p, c->fe_flags.p);
    } else {
        // 3. StatisticalOutlierRemoval (filter_node.cpp:253-263)
        if (nv <= prm->mean_k) {
            HIPCHK(c, hipMemcpyAsync(out, c->fe_ds.p, (size_t)nv * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            *n_out = (size_t)nv;
            return NDT_OK;
        }
        // k-NN index over the voxel-filtered cloud: base cell 3 leaves (the mean_k = 30 neighbours of a surface point lie
        // within the 3x3x3 cells around it on a 0.5 m grid)
        TRY(enqueue_nn_index(c, main_lane(c), c->fe_ds.p, nv, 1, 3.0f * prm->leaf, c->sor_ix));
        if (prm->mean_k + 1 <= 32)
            hipLaunchKernelGGL(k_sor_knn<32>, dim3(nbq), dim3(kBlock), 0, c->stream, c->fe_ds.p, nv, prm->mean_k, c->sor_ix.hdr,
                               c->sor_ix.blk.p, c->sor_ix.off.p, c->sor_ix.pts.p, c->fe_dist.p);
        else
            hipLaunchKernelGGL(k_sor_knn<64>, dim3(nbq), dim3(kBlock), 0, c->stream, c->fe_ds.p, nv, prm->mean_k, c->sor_ix.hdr,
                               c->sor_ix.blk.p, c->sor_ix.off.p, c->sor_ix.pts.p, c->fe_dist.p);
        hipLaunchKernelGGL(k_sor_stats, dim3(1), dim3(kBlock), 0, c->stream, c->fe_dist.p, nv, prm->stddev_mul, c->fe_thr.p);
        const int nbk = std::max(1, std::min(ceil_div(nv, kBlock), 2048));
        hipLaunchKernelGGL(k_sor_keep, dim3(nbk), dim3(kBlock), 0, c->stream, c->fe_dist.p, nv, c->fe_thr.p, c->fe_flags.p);
    }
    const int nbv = std::max(1, std::min(ceil_div(nv, kBlock), 2048));
    TRY(enqueue_scan(c, main_lane(c), c->fe_flags.p, nv, nullptr, c->fe_idx.p, &c->d_hdr_fe->pad[1], c->d_hdr_fe));
    hipLaunchKernelGGL(k_compact4, dim3(nbv), dim3(kBlock), 0, c->stream, c->fe_ds.p, c->fe_flags.p, c->fe_idx.p, nv, out);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(fw, &c->d_hdr_fe->pad[0], 2 * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    // the outlier filter's neighbour index (enqueue_nn_index: its own sort, header rewritten per build) flags its
    // look-back timeouts in sor_ix.hdr
    HIPCHK(c, hipMemcpyAsync(&fw[2], &c->sor_ix.hdr->pad[0], sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (fw[2]) {
        // a compaction-scan flag raised beside it is cleared too, or the next call would report a stale timeout
        if (fw[0]) (void)hipMemsetAsync(&c->d_hdr_fe->pad[0], 0, sizeof(int), c->stream);
        return fail(c, NDT_EDEVICE, "filter: outlier neighbour index sort: radix look-back timed out");
    }
    if (fw[0]) return scan_failed("outlier");
    *n_out = (size_t)fw[1];
    return NDT_OK;
}

ndt_status ndt_filter_scan(ndt_ctx* c, const ndt_filter_params* prm, const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset,
                           float* out4, size_t cap, size_t* n_out) {
    if (!c || !prm || !n_out || (n && (!xyzi || !out4)) || stride_bytes < 16 || intensity_offset < 3 ||
        (size_t)intensity_offset * 4 + 4 > stride_bytes || n > 0x7fffffffULL)
        return fail(c, NDT_EINVAL, "bad filter args");
    TRY(set_dev(c));
    *n_out = 0;
    if (n == 0) return ndt_filter_scan_device(c, prm, nullptr, 0, nullptr, n_out);
    std::vector<float4> tmp(n);
    const char* base = reinterpret_cast<const char*>(xyzi);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        tmp[i] = make_float4(f[0], f[1], f[2], f[intensity_offset]);
    }
    TRY(ensure(c, c->fe_in, n)); TRY(ensure(c, c->fe_out, n));
    HIPCHK(c, hipMemcpyAsync(c->fe_in.p, tmp.data(), n * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    TRY(ndt_filter_scan_device(c, prm, reinterpret_cast<const float*>(c->fe_in.p), n, reinterpret_cast<float*>(c->fe_out.p), n_out));
    const size_t k = std::min(cap, *n_out);
    if (k) {
        std::vector<float4> o(k);
        HIPCHK(c, hipMemcpy(o.data(), c->fe_out.p, k * sizeof(float4), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < k; ++i) { out4[4 * i] = o[i].x; out4[4 * i + 1] = o[i].y; out4[4 * i + 2] = o[i].z; out4[4 * i + 3] = o[i].w; }
    }
    return NDT_OK;
}

ndt_status ndt_filter_last_stats(ndt_ctx* c, float* dist, size_t cap, size_t* n_voxel, double thr[3]) {
    if (!c || !n_voxel) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    *n_voxel = c->fe_nvox;
    const size_t k = std::min(cap, c->fe_nvox);
    if (dist && k) HIPCHK(c, hipMemcpy(dist, c->fe_dist.p, k * sizeof(float), hipMemcpyDeviceToHost));
    if (thr) {
        if (c->fe_thr.p) HIPCHK(c, hipMemcpy(thr, c->fe_thr.p, 3 * sizeof(double), hipMemcpyDeviceToHost));
        else thr[0] = thr[1] = thr[2] = 0.0;
    }
    return NDT_OK;
}

ndt_status ndt_memcpy_d2d(ndt_ctx* c, void* d_dst, const void* d_src, size_t bytes) {
    if (!c || (bytes && (!d_dst || !d_src))) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    if (bytes) TRY(copy16(c, c->stream, d_dst, d_src, bytes));
    return NDT_OK;
}

ndt_status ndt_device_alloc(ndt_ctx* c, size_t bytes, void** d_ptr) {
    if (!c || !d_ptr) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    if (hipMalloc(d_ptr, bytes ? bytes : 1) != hipSuccess) return fail(c, NDT_ENOMEM, "hipMalloc failed");
    return NDT_OK;
}

ndt_status ndt_device_free(ndt_ctx* c, void* d_ptr) {
    if (!c) return NDT_EINVAL;
    TRY(set_dev(c));
    if (d_ptr) HIPCHK(c, hipFree(d_ptr));
    return NDT_OK;
}

ndt_status ndt_memcpy_h2d(ndt_ctx* c, void* d_dst, const void* h_src, size_t bytes) {
    if (!c || (bytes && (!d_dst || !h_src))) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    if (bytes) HIPCHK(c, hipMemcpy(d_dst, h_src, bytes, hipMemcpyHostToDevice));
    return NDT_OK;
}

ndt_status ndt_memcpy_d2h(ndt_ctx* c, void* h_dst, const void* d_src, size_t bytes) {
    if (!c || (bytes && (!h_dst || !d_src))) return fail(c, NDT_EINVAL, "null argument");
    TRY(set_dev(c));
    if (bytes) HIPCHK(c, hipMemcpy(h_dst, d_src, bytes, hipMemcpyDeviceToHost));
    return NDT_OK;
}

ndt_status ndt_synchronize(ndt_ctx* c) {
    if (!c) return NDT_EINVAL;
    TRY(set_dev(c));
    TRY(flush_source(c));  // after a synchronize the caller may reuse the buffer it set as source
    // the side lanes' host threads first (every posted job issued; a job's failure stays for its result call)
    for (LaneWorker* w : {c->fit_worker, c->ins_worker}) if (w) (void)w->drain(nullptr);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->fit_stream) HIPCHK(c, hipStreamSynchronize(c->fit_stream));
    if (c->ins_stream) HIPCHK(c, hipStreamSynchronize(c->ins_stream));
    return NDT_OK;
}

ndt_status ndt_last_timings(ndt_ctx* c, double* ms_build, double* ms_align, double* ms_pass_avg, double* pass_bytes_avg) {
    if (!c) return NDT_EINVAL;
    if (ms_build) *ms_build = c->ms_build;
    if (ms_align) *ms_align = c->ms_align;
    // pass statistics over this ctx and the helper contexts of ndt_align_batch (the batch's other streams)
    double ms = c->prof_ms_sum, bytes = c->prof_bytes_sum;
    long long cnt = c->prof_count;
    for (const ndt_ctx* h : c->helpers) {
        ms += h->prof_ms_sum;
        bytes += h->prof_bytes_sum;
        cnt += h->prof_count;
    }
    if (ms_pass_avg) *ms_pass_avg = cnt ? ms / cnt : 0.0;
    if (pass_bytes_avg) *pass_bytes_avg = cnt ? bytes / cnt : 0.0;
    return NDT_OK;
}

ndt_status ndt_pass_phases(ndt_ctx* c, double ms[22]) {
    if (!c || !ms) return NDT_EINVAL;
    for (int q = 0; q < 7; ++q) ms[q] = c->prof_phase_count ? c->prof_phase_sum[q] / c->prof_phase_count : 0.0;
    for (int q = 0; q < 5; ++q) ms[7 + q] = c->prof_body_count ? c->prof_body_sum[q] / c->prof_body_count : 0.0;
    for (int q = 0; q < 10; ++q) ms[12 + q] = c->prof_tail_count ? c->prof_tail_sum[q] / c->prof_tail_count : 0.0;
    return NDT_OK;
}

ndt_status ndt_set_pass_options(ndt_ctx* c, int lead_tail, int points_per_thread, int source_order) {
    if (!c || lead_tail < 0 || lead_tail > 1 || points_per_thread < 1 || points_per_thread > 3 || source_order < 0 ||
        source_order > 1)
        return fail(c, NDT_EINVAL, "bad pass options");
    if (c->al_inflight) return fail(c, NDT_EINVAL, "an asynchronous align is in flight (ndt_align_wait first)");
    c->opt_lead_tail = lead_tail != 0;
    c->opt_ppt = points_per_thread;
    c->order_source = source_order != 0;
    for (ndt_ctx* h : c->helpers) TRY(ndt_set_pass_options(h, lead_tail, points_per_thread, source_order));
    return NDT_OK;
}

ndt_status ndt_set_build_options(ndt_ctx* c, int tile_tickets, int radix_passes) {
    if (!c || tile_tickets < 0 || tile_tickets > 1 || radix_passes < 0 || radix_passes > 4) return fail(c, NDT_EINVAL, "bad build options");
    if (c->al_inflight) return fail(c, NDT_EINVAL, "an asynchronous align is in flight (ndt_align_wait first)");
    c->tile_tickets = tile_tickets != 0;
    c->radix_force = radix_passes;
    for (ndt_ctx* h : c->helpers) TRY(ndt_set_build_options(h, tile_tickets, radix_passes));
    return NDT_OK;
}

ndt_status ndt_build_stats(ndt_ctx* c, long long out[6]) {
    if (!c || !out) return fail(c, NDT_EINVAL, "null argument");
    out[0] = c->n_builds_full;
    out[1] = c->n_builds_merge;
    out[2] = c->n_builds_rerun;
    out[3] = c->n_rerun_lookback;
    out[4] = c->tile_tickets ? 1 : 0;
    out[5] = radix_launch_passes(c);
    for (const ndt_ctx* h : c->helpers) {  // ndt_align_batch's helper contexts (their own streams and builds)
        out[0] += h->n_builds_full;
        out[1] += h->n_builds_merge;
        out[2] += h->n_builds_rerun;
        out[3] += h->n_rerun_lookback;
        out[4] += h->tile_tickets ? 1 : 0;
    }
    return NDT_OK;
}

ndt_status ndt_set_profiling(ndt_ctx* c, int enable) {
    if (!c) return NDT_EINVAL;
    for (ndt_ctx* h : c->helpers) TRY(ndt_set_profiling(h, enable));
    c->profiling = enable != 0;
    c->prof_ms_sum = c->prof_bytes_sum = 0;
    for (double& v : c->prof_phase_sum) v = 0;
    for (double& v : c->prof_body_sum) v = 0;
    for (double& v : c->prof_tail_sum) v = 0;
    c->prof_phase_count = c->prof_body_count = c->prof_tail_count = 0;
    c->prof_count = 0;
    c->ms_pass_avg = c->pass_bytes_avg = 0;
    // no graph invalidation: the profiling flag and the stamp buffer are part of every graph's cache key, so a call
    // that only resets the statistics keeps the captured chains
    return NDT_OK;
}

const char* ndt_last_error(const ndt_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int ndt_abi_version(void) { return NDT_HIP_ABI_VERSION; }

void ndt_destroy(ndt_ctx* c) {
    if (!c) return;
    for (ndt_ctx* h : c->helpers) ndt_destroy(h);
    c->helpers.clear();
    (void)hipSetDevice(c->device);
    delete c->fit_worker;  // joins the side lanes' host threads after their queued jobs
    delete c->ins_worker;
    c->fit_worker = c->ins_worker = nullptr;
    for (hipStream_t st : {c->stream, c->fit_stream, c->ins_stream}) if (st) (void)hipStreamSynchronize(st);
    invalidate_graph(c);
    release(c->target); release(c->source); release(c->recs); release(c->cent); release(c->icovd); release(c->evals);
    release(c->cloud_key); release(c->valid_part); release(c->table); release(c->grid); release(c->partials); release(c->partials2); release(c->nbr); release(c->score_part); release_nn_index(c->fit_ix); release_nn_index(c->sor_ix); release(c->ins_tr); release(c->ins_ds); release(c->fit_cnt); release(c->fit_ticket);release(c->fit_sum); release(c->fit_d2); release(c->reduce_out); release(c->counter); release(c->out_cloud); release(c->ts);
    for (Scratch* sp : {&c->s, &c->s_fit, &c->s_ins, &c->s_inc}) {
        Scratch& s = *sp;
        release(s.k0); release(s.v0); release(s.k1); release(s.v1); release(s.radix_aux); release(s.radix_status);
        release(s.seg_start); release(s.flags); release(s.cloud_idx); release(s.cloud_span); release(s.mm); release(s.sorted_pts);
        release(s.scan_status); release(s.scan_ticket);
    }
    release(c->fe_flags); release(c->fe_idx); release(c->fe_in); release(c->fe_crop); release(c->fe_ds);
    release(c->fe_out); release(c->fe_dist); release(c->fe_thr);
    release(c->source_ord); release(c->ord_k0); release(c->ord_v0); release(c->ord_k1); release(c->ord_v1);
    if (c->d_hdr) (void)hipFree(c->d_hdr);
    if (c->d_hdr_ds) (void)hipFree(c->d_hdr_ds);
    if (c->d_hdr_prev) (void)hipFree(c->d_hdr_prev);
    if (c->d_hdr_fe) (void)hipFree(c->d_hdr_fe);
    if (c->d_hdr_ins) (void)hipFree(c->d_hdr_ins);
    if (c->h_hdr) (void)hipHostFree(c->h_hdr);
    if (c->d_async) (void)hipFree(c->d_async);
    if (c->h_async) (void)hipHostFree(c->h_async);
    if (c->ev_fit) (void)hipEventDestroy(c->ev_fit);
    if (c->ev_ins) (void)hipEventDestroy(c->ev_ins);
    if (c->h_ts) (void)hipHostFree(c->h_ts);
    if (c->h_hist) (void)hipHostFree(c->h_hist);
    if (c->d_state) (void)hipFree(c->d_state);
    if (c->d_state2) (void)hipFree(c->d_state2);
    if (c->h_state) (void)hipHostFree(c->h_state);
    if (c->h_rb) (void)hipHostFree(c->h_rb);
    if (c->d_clk) (void)hipFree(c->d_clk);
    if (c->d_hist) (void)hipFree(c->d_hist);
    for (auto e : {c->ev_tgt, c->ev_main_fit, c->ev_main_ins, c->ev_fit_src, c->ev_fit_tgt}) if (e) (void)hipEventDestroy(e);
    for (auto e : c->pass_ev) (void)hipEventDestroy(e);
    for (hipStream_t st : {c->stream, c->fit_stream, c->ins_stream}) if (st) (void)hipStreamDestroy(st);
    delete c;
}

}  // extern "C"
