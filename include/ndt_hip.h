/* ndt_hip.h — C-ABI of the MI355X-native NDT scan-matching library (libndt_hip.so).
 *
 * Drop-in boundary for the reference's registration object
 *   pclomp::NormalDistributionsTransform<pcl::PointXYZI, pcl::PointXYZI>
 * (reference: /root/reference/xchu_mapping/include/pclomp/ndt_omp.h:70-497) as used by
 * odom_node (xchu_mapping/src/odom_node.cpp:69-80, 227-228, 277-283, 348-349).
 * Plain C: opaque handle, plain pointers and sizes, status codes — no C++/torch types.
 * One ctx = one HIP device + one HIP stream; a ctx is not thread-safe (same as the reference,
 * which is driven from odom_node's single main thread).
 *
 * Each entry point names the reference interface it replaces.
 */
#ifndef NDT_HIP_H_
#define NDT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Layout version of the structs below and of the buffers the library writes through caller pointers
 * (ndt_result, ndt_pass_record, ndt_pair_desc, ndt_filter_params, ndt_pass_phases' 22 doubles).  History: 1 = round 1;
 * 2 = ndt_result.solver_fallbacks appended, ndt_pass_phases 20 -> 22 doubles.  A caller built against this header
 * checks ndt_abi_version() == NDT_HIP_ABI_VERSION before its first call. */
#define NDT_HIP_ABI_VERSION 2

typedef struct ndt_ctx ndt_ctx;

typedef enum {
    NDT_OK = 0,
    NDT_EINVAL = 1,      /* bad argument                                                         */
    NDT_ENOTARGET = 2,   /* align before setInputTarget (PCL: initCompute fails, align is a no-op) */
    NDT_ENOSOURCE = 3,   /* align before setInputSource                                          */
    NDT_EOVERFLOW = 4,   /* voxel index overflow: grid left empty (VGC applyFilter :79-84 warns)  */
    NDT_EDEVICE = 5,     /* HIP runtime error / no device                                        */
    NDT_ENOMEM = 6
} ndt_status;

/* = pclomp::NeighborSearchMethod order (ndt_omp.h:52-57) */
typedef enum { NDT_KDTREE = 0, NDT_DIRECT26 = 1, NDT_DIRECT7 = 2, NDT_DIRECT1 = 3 } ndt_search;

typedef struct {
    float resolution;                /* setResolution            (ndt_omp.h:127-137)   default 1.0   */
    double step_size;                /* setStepSize              (ndt_omp.h:160-164)   default 0.1   */
    double trans_eps;                /* setTransformationEpsilon (pcl::Registration)   default 0.1   */
    double outlier_ratio;            /* setOulierRatio           (ndt_omp.h:178-182)   default 0.55  */
    int max_iter;                    /* setMaximumIterations     (pcl::Registration)   default 35    */
    int search;                      /* setNeighborhoodSearchMethod (ndt_omp.h:184)    default DIRECT7 */
    int min_points_per_voxel;        /* VGC::setMinPointPerVoxel (voxel_grid_covariance_omp.h:135) default 6 */
    double min_covar_eigvalue_mult;  /* VGC::setCovEigValueInflationRatio (:155)       default 0.01  */
    int precision_mode;              /* 0 = ndt_omp (f32 per pair), 1 = pcl_ndt (f64 per pair, radius),
                                        2 = ndt_cpu (cpu::NormalDistributionsTransform: its own cpu::VoxelGrid
                                        and radius search, f64 per pair; odom_node.cpp:57-68, launch default) */
    int device;                      /* HIP device ordinal                                           */
} ndt_params;

typedef struct {
    float final_tf[16];              /* getFinalTransformation(), column-major (Eigen::Matrix4f)      */
    int nr_iterations;               /* getFinalNumIteration()   (ndt_omp.h:200-204)                 */
    int converged;                   /* hasConverged()                                               */
    double trans_probability;        /* getTransformationProbability() (ndt_omp.h:191-195)           */
    double score;                    /* last computeDerivatives score                                */
    int n_passes;                    /* derivative evaluations performed                             */
    long long n_pairs;               /* total (point, voxel) pairs evaluated over all passes (P)     */
    int solver_fallbacks;            /* Newton solves that took JacobiSVD semantics (degenerate / ill-conditioned H:
                                        kappa_1(H) > 6.25e13 or a zero pivot; ndt_omp_impl.hpp:118-124)   */
} ndt_result;

/* One derivative evaluation: kind 0 = computeDerivatives with Hessian (ndt_omp_impl.hpp:175),
 * 1 = gradient-only MT trial (:869), 2 = computeHessian radius pass (:550). */
typedef struct {
    int kind;
    int newton_iter;
    double x[6];
    double score;
    double g[6];
    double H[36];
    long long pairs;
} ndt_pass_record;

/* Batched offline replay: one independent scan->localmap pair (device-resident float4 xyzw). */
typedef struct {
    const float* d_target_xyz4;
    size_t n_target;
    const float* d_source_xyz4;
    size_t n_source;
    float guess[16];
} ndt_pair_desc;

/* Defaults of the pclomp ctor (ndt_omp_impl.hpp:46-69) + VGC ctor (voxel_grid_covariance_omp.h:202-217). */
ndt_status ndt_default_params(ndt_params* out);

/* new pclomp::NormalDistributionsTransform (odom_node.cpp:71-72) */
ndt_status ndt_create(const ndt_params* params, ndt_ctx** out);
/* setResolution/setStepSize/setTransformationEpsilon/setMaximumIterations/setNeighborhoodSearchMethod
 * (odom_node.cpp:73-78).  Does not rebuild the grid (see ndt_set_target). */
ndt_status ndt_set_params(ndt_ctx* ctx, const ndt_params* params);

/* setInputTarget (ndt_omp.h:117-122 -> init() :271-278 -> VGC::filter(true) :285-297).
 * Copies n points (x,y,z float at the start of each stride_bytes record; 32 = pcl::PointXYZI)
 * and rebuilds the voxel grid on the device.  is_dense = PointCloud::is_dense. */
ndt_status ndt_set_target(ndt_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes, int is_dense);
/* Same, from a device-resident float4 array (no PCIe transfer). */
ndt_status ndt_set_target_device(ndt_ctx* ctx, const float* d_xyz4, size_t n, int is_dense);
/* setInputTarget of n_old + n_new device points whose first n_old are the current target's points (same values, same
 * order) — odom_node's pc_target_ = localmap between localmap resets (odom_node.cpp:233, 349), which only grows by
 * appends.  Same grid as ndt_set_target_device(d_xyz4, n_old + n_new, is_dense) bit for bit; when the current grid's
 * sort is still held (pclomp grid, dense cloud, no other sort on the main stream since, same parameters) it is built by
 * merging the sort of the n_new points into it, otherwise from scratch.  The buffer is referenced like
 * ndt_set_target_device's.  d_new4 (may be NULL): the n_new points are read there and stored at d_xyz4 + 4 * n_old by
 * the build itself, on the ctx stream (the caller's snapshot of a growing map needs no separate copy). */
ndt_status ndt_set_target_append_device(ndt_ctx* ctx, float* d_xyz4, size_t n_old, size_t n_new, int is_dense,
                                        const float* d_new4);

/* cpu::NormalDistributionsTransform::updateVoxelGrid(new_cloud) (ndt_cpu/NormalDistributionsTransform.h:39;
 * odom_node.cpp:344-345): append points to the target (after the existing ones) and update the voxel grid, as if the
 * target had been set to old + new.  Host points (stride as ndt_set_target) or device float4 points (copied). */
ndt_status ndt_update_target(ndt_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
ndt_status ndt_update_target_device(ndt_ctx* ctx, const float* d_xyz4, size_t n);

/* setInputSource (pcl::Registration, odom_node.cpp:278). Copies: the host version at once; the device version on the
 * ctx stream with the next align (inside its first kernel) or the next other call that reads the source, whichever
 * comes first — d_xyz4 stays unmodified until then (pcl::Registration keeps the caller's cloud the same way), or until
 * ndt_synchronize. */
ndt_status ndt_set_source(ndt_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
ndt_status ndt_set_source_device(ndt_ctx* ctx, const float* d_xyz4, size_t n);

/* align(output, guess) (pcl::Registration::align -> computeTransformation, ndt_omp_impl.hpp:73-164;
 * odom_node.cpp:279).  guess: column-major 4x4.  Synchronous; fills out. */
ndt_status ndt_align(ndt_ctx* ctx, const float guess[16], ndt_result* out);
/* The aligned `output` cloud of align(): source transformed by final_tf, written as x,y,z at each stride. */
ndt_status ndt_get_output(ndt_ctx* ctx, float* xyz, size_t stride_bytes);
/* Per-pass trace of the last align (history of computeDerivatives results). */
ndt_status ndt_get_history(ndt_ctx* ctx, ndt_pass_record* out, int cap, int* n_out);

/* Test hooks: one computeDerivatives pass (ndt_omp_impl.hpp:175) at parameters p with point transform T. */
ndt_status ndt_derivatives(ndt_ctx* ctx, const double p[6], const float T[16], int compute_hessian,
                           double* score, double g[6], double H[36], long long* pairs);
/* computeHessian (radius neighbours, f64; ndt_omp_impl.hpp:550-607) at p with transform T. */
ndt_status ndt_hessian_radius(ndt_ctx* ctx, const double p[6], const float T[16], double H[36], long long* pairs);
/* calculateScore (ndt_omp_impl.hpp:919-952) of the source transformed by T (uses the Gaussian constants the
 * object holds: the constructor's until an align recomputes them, as the reference's members). */
ndt_status ndt_calculate_score(ndt_ctx* ctx, const float T[16], double* out);
/* pcl::Registration::getFitnessScore(max_range) (called by odom_node.cpp:280 after every align): mean of the
 * squared nearest-neighbour distances from the source transformed by T (NULL = the last align's final
 * transformation, identity before any align) to ALL target points, over the distances <= max_range (PCL
 * compares the squared distance); DBL_MAX when none qualifies.  nn_d2 (optional, N floats) receives every
 * point's squared distance. */
ndt_status ndt_fitness_score(ndt_ctx* ctx, const float* T, double max_range, double* out, float* nn_d2);

/* getFitnessScore, asynchronous: enqueued on the ctx's fitness side stream behind everything queued on the ctx
 * stream so far (source, align), so that it runs beside what the caller queues next (a target build, a keyframe
 * insertion); ndt_fitness_score_result waits for it and returns the score (same semantics as ndt_fitness_score). */
ndt_status ndt_fitness_score_async(ndt_ctx* ctx, const float* T, double max_range);
ndt_status ndt_fitness_score_result(ndt_ctx* ctx, double* out);
/* getFitnessScore of an explicit device cloud (float4, n points: normally the source the last align registered) instead
 * of the ctx's source, asynchronous like ndt_fitness_score_async: the cloud is read on the side stream, so the ctx's
 * source may be replaced (the next scan's setInputSource) while the query is in flight; d_src4 stays unmodified until
 * ndt_fitness_score_result. */
ndt_status ndt_fitness_score_async_cloud(ndt_ctx* ctx, const float* T, double max_range, const float* d_src4, size_t n);
/* getFitnessScore of the last align (its final transformation, its target) over a device cloud, asynchronous like
 * ndt_fitness_score_async_cloud, and callable after setInputTarget has replaced the target that align used (odom_node
 * queries at :280 and sets the next target at :349; queuing the query after the new target's build is queued lets that
 * build start first).  The replaced target's index must have been queued (ndt_fitness_index_async after its
 * setInputTarget); NDT_EINVAL otherwise. */
ndt_status ndt_fitness_score_async_aligned(ndt_ctx* ctx, double max_range, const float* d_src4, size_t n);
/* getFitnessScore's nearest-neighbour index over the current target, queued now on the fitness side stream behind the
 * target's points (beside the voxel build and the next align) instead of at the first query after setInputTarget.
 * A scan loop that queries every scan (odom_node.cpp:280) calls it after each setInputTarget.  The index build reads
 * the target cloud: a caller-referenced device target stays unmodified until the next ndt_fitness_score_result or
 * ndt_synchronize. */
ndt_status ndt_fitness_index_async(ndt_ctx* ctx);

/* Voxel grid inspection: header = min_b[3], max_b[3], div_b[3], divb_mul[3], n_leaves, n_cloud, overflow,
 * n_valid (16 ints).  Leaves with >= min points (the reference's KD cloud) in ascending key order. */
ndt_status ndt_grid_info(ndt_ctx* ctx, int header[16]);
ndt_status ndt_grid_leaves(ndt_ctx* ctx, int* keys, int* npts, double* mean, double* icov9, float* centroid3,
                           int cap, int* n_out);

/* Pass-chain options, tuning and test hooks (defaults = the measured best; the results of every combination agree with
 * the oracle within the parity bars): lead_tail 1 runs an align whose passes are latency-bound (direct search, no
 * More-Thuente loop, < 256 Ki source points, not inside ndt_align_batch) as a leading-tail chain — each pass's Newton
 * step at the start of the next pass kernel — and 0 keeps last-workgroup tails everywhere (bitwise the same records;
 * tests/test_gpu_lead.py); points_per_thread 2 lets large last-workgroup-tail passes hold two points per thread per tile,
 * 1 keeps one (another fixed f64 summation order), 3 runs them as a grid of one-tile workgroups (one 256-point tile
 * each, three waves per SIMD, partials summed in two levels: another fixed order); source_order 1 visits clouds of >= 256 Ki points in
 * target-cell order during an align, 0 keeps the caller's order (another fixed f64 summation order).  Applies to the
 * ctx and its batch helper contexts; no align may be in flight. */
ndt_status ndt_set_pass_options(ndt_ctx* ctx, int lead_tail, int points_per_thread, int source_order);

/* Target-build robustness hooks (no reference counterpart).  A target sort whose decoupled look-back timed
 * out (a predecessor tile never became resident: blockIdx.x tile order relies on each XCD dispatching its workgroups in
 * order, which heavy concurrent work on other streams can defeat), whose key needed more radix passes than were
 * launched (the count is predicted from the previous grid), or whose merge-extended sort could not be exact, is flagged
 * on the device and re-run from scratch by the align (or the next synchronous grid reader) — with tiles taken by atomic
 * ticket from then on after a timeout.  ndt_set_build_options (test hook): tile_tickets 1 = tiles by atomic ticket
 * always, 0 = by workgroup index (default); radix_passes 1..4 = launch exactly that many radix passes per target sort
 * (too few is flagged and re-run with four), 0 = predicted (default).  ndt_build_stats: out[0] full builds, out[1]
 * merge-extended builds, out[2] builds re-run after a flag, out[3] of those the look-back timeouts, out[4] contexts whose
 * tiles are taken by ticket, out[5] radix passes the next target sort launches; [0..4] include ndt_align_batch's helper
 * contexts. */
ndt_status ndt_set_build_options(ndt_ctx* ctx, int tile_tickets, int radix_passes);
ndt_status ndt_build_stats(ndt_ctx* ctx, long long out[6]);

/* align split in two: ndt_align_async queues the registration on the ctx stream and returns; ndt_align_wait waits for it
 * and fills out (same result as ndt_align).  One align in flight per ctx; several ctxs (streams) run concurrently. */
ndt_status ndt_align_async(ndt_ctx* ctx, const float guess[16]);
ndt_status ndt_align_wait(ndt_ctx* ctx, ndt_result* out);

/* Batched offline alignment of independent pairs on this ctx's device: pairs round-robin over three
 * streams (this ctx and two helper ctxs, created on first use), one registration in flight per stream; per-pair results
 * bit-identical to one-by-one aligns. */
ndt_status ndt_align_batch(ndt_ctx* ctx, const ndt_pair_desc* pairs, int n_pairs, ndt_result* out);

/* pcl::VoxelGrid<PointXYZI> downsample (odom_node.cpp:96-99, 334-335): per-voxel mean of x,y,z,intensity,
 * output ordered by ascending voxel index.  out4 receives x,y,z,intensity per output point. */
ndt_status ndt_voxel_downsample(ndt_ctx* ctx, const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset,
                                float leaf, float* out4, size_t cap, size_t* n_out);

/* filter_node front end (xchu_mapping/src/filter_node.cpp:218-273): the cloud odom_node receives on
 * /filtered_points.  removeNaNFromPointCloud (non-finite points dropped) -> keep r_min < sqrt(x^2+y^2) < r_max (double)
 * -> pcl::VoxelGrid<PointXYZI>(leaf) -> pcl::StatisticalOutlierRemoval(mean_k, stddev_mul) (use_outlier_removal_method,
 * filter_node.h:71).  Output x,y,z,intensity in the reference's order (voxel index order, outliers removed). */
typedef struct {
    float leaf;          /* downSizeFilterKeyFrames leaf size   (filter_node.cpp:33-34)  default 0.5  */
    double r_min, r_max; /* range crop on sqrt(x^2+y^2)          (:239-247)               default 1, 60 */
    int mean_k;          /* StatisticalOutlierRemoval::setMeanK  (:256-259)               default 30 (<= 63) */
    double stddev_mul;   /* setStddevMulThresh                   (:257-260)               default 1.0  */
    int outlier_method;  /* use_outlier_removal_method (filter_node.h:71): 0 = StatisticalOutlierRemoval (default),
                            1 = RadiusOutlierRemoval (:265-272)                                             */
    double ror_radius;   /* RadiusOutlierRemoval::setRadiusSearch          default 0.8              */
    int ror_min_neighbors; /* setMinNeighborsInRadius (neighbours counted with the point itself) default 5 */
} ndt_filter_params;
ndt_status ndt_filter_default_params(ndt_filter_params* out);
/* host cloud: x,y,z at the start of each stride_bytes record, intensity at float index intensity_offset; out4 receives
 * up to cap points (x,y,z,i); *n_out = the filtered size.  A cloud left with <= mean_k points after the voxel filter is
 * returned without outlier removal (PCL reads past its neighbour list there). */
ndt_status ndt_filter_scan(ndt_ctx* ctx, const ndt_filter_params* prm, const float* xyzi, size_t n, size_t stride_bytes,
                           int intensity_offset, float* out4, size_t cap, size_t* n_out);
/* device float4 (x,y,z,i) in and out (d_out4 capacity n, must not alias d_in4); synchronises. */
ndt_status ndt_filter_scan_device(ndt_ctx* ctx, const ndt_filter_params* prm, const float* d_in4, size_t n, float* d_out4, size_t* n_out);
/* per-point SOR distances and threshold of the last filter_scan (test hook): dist[0..n_voxel) in voxel order,
 * thr = {threshold, mean, stddev}; *n_voxel = points after the voxel filter. */
ndt_status ndt_filter_last_stats(ndt_ctx* ctx, float* dist, size_t cap, size_t* n_voxel, double thr[3]);

/* Device-resident variants used by the odom_node replay driver (include/ndt_odom.h), all ordered on the ctx's
 * stream.  d_in4/d_out4 are float4 x,y,z,intensity arrays.
 * pcl::transformPointCloud(in, out, T) (odom_node.cpp:220, 290): out may equal in; asynchronous. */
ndt_status ndt_transform_device(ndt_ctx* ctx, const float T[16], const float* d_in4, size_t n, float* d_out4);
/* pcl::VoxelGrid<PointXYZI>::filter (odom_node.cpp:334-335) of a device cloud: d_out4 (capacity n, must not
 * alias d_in4) receives the voxel means in ascending voxel order; *n_out their count (synchronises). */
ndt_status ndt_voxel_downsample_device(ndt_ctx* ctx, const float* d_in4, size_t n, float leaf, float* d_out4, size_t* n_out);
/* odom_node keyframe insertion (odom_node.cpp:290, 333-338), asynchronous: transformPointCloud(scan, T) ->
 * VoxelGrid(leaf) -> the voxel means appended at d_map_a + n_a and d_map_b + n_b (localmap and tmp_map; float4
 * clouds with room for n more points each), queued on the ctx's insertion side stream behind everything queued on
 * the ctx stream so far (it runs beside what the caller queues next, e.g. the next target build); the scan and the two
 * appended ranges stay untouched until ndt_keyframe_insert_result, which waits and returns how many points were
 * appended (NDT_EOVERFLOW when the leaf overflowed the index range: the transformed scan itself was appended, as
 * pcl::VoxelGrid outputs its input then). */
ndt_status ndt_keyframe_insert_async(ndt_ctx* ctx, const float T[16], const float* d_scan4, size_t n, float leaf, float* d_map_a,
                                     size_t n_a, float* d_map_b, size_t n_b);
ndt_status ndt_keyframe_insert_result(ndt_ctx* ctx, size_t* n_inserted);
/* Marks the point on the ctx stream that the next ndt_fitness_score_async[_cloud] and the next
 * ndt_keyframe_insert_async queue behind (instead of "everything queued so far" at their own calls), so that a scan
 * loop can queue its target copy and build on the ctx stream first and post the side-lane jobs after them, beside
 * them.  A mark not taken by the next align is dropped. */
ndt_status ndt_side_lanes_mark(ndt_ctx* ctx);
/* Device-to-device copy, asynchronous on the ctx stream. */
ndt_status ndt_memcpy_d2d(ndt_ctx* ctx, void* d_dst, const void* d_src, size_t bytes);

/* Device memory helpers (callers without their own GPU runtime binding, e.g. the bench). */
ndt_status ndt_device_alloc(ndt_ctx* ctx, size_t bytes, void** d_ptr);
ndt_status ndt_device_free(ndt_ctx* ctx, void* d_ptr);
ndt_status ndt_memcpy_h2d(ndt_ctx* ctx, void* d_dst, const void* h_src, size_t bytes);
ndt_status ndt_memcpy_d2h(ndt_ctx* ctx, void* h_dst, const void* d_src, size_t bytes);
/* Waits for the ctx stream and its side streams (getFitnessScore, keyframe insertion). */
ndt_status ndt_synchronize(ndt_ctx* ctx);

/* Timing of the last set_target / align on the device (HIP events, ms) and the dominant kernel's
 * average duration (derivative pass, ms) with its algorithmic bytes per launch. */
ndt_status ndt_last_timings(ndt_ctx* ctx, double* ms_build, double* ms_align, double* ms_pass_avg, double* pass_bytes_avg);
/* Profiling breakdown of the average derivative pass (ms), from in-kernel stamps: [0] workgroup bodies
 * (first start .. last workgroup's partials stored), [1] hand-off (ticket + acquire), [2] last workgroup's
 * fixed-order partials reduction, [3] AlignState staged into LDS, [4] Newton/More-Thuente control step,
 * [5] next transform + angle tables, [6] state write-back and drain; [7..11] (profiling build
 * libndt_hip_dbg.so only, else 0) mean workgroup entry after the first, probes, pair compaction, pair math,
 * block reduction; [12..19] (profiling build) history record + state copy, state machine, solve set-up,
 * the 6x6 solve, after it, sin/cos of the next angles, transform + table rows, table write-back; [20..21]
 * (profiling build) start of the speculative Newton solve after staging, its duration.
 * Profiling aid, no reference counterpart. */
ndt_status ndt_pass_phases(ndt_ctx* ctx, double ms[22]);
/* Enable/disable the in-kernel per-pass timing stamps (s_memrealtime). */
ndt_status ndt_set_profiling(ndt_ctx* ctx, int enable);

const char* ndt_last_error(const ndt_ctx* ctx);
/* NDT_HIP_ABI_VERSION the library was built with */
int ndt_abi_version(void);
void ndt_destroy(ndt_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* NDT_HIP_H_ */
