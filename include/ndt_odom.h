/* ndt_odom.h — C-ABI of the odom_node scan-loop replay driver (in libndt_hip.so).
 *
 * Restates LidarOdom::OdomEstimate (reference: xchu_mapping/src/odom_node.cpp:208-356, parameters :42-99,
 * pose helpers xchu_mapping/include/xchu_mapping/common.h:38-71) without ROS, for the "use_omp" backend
 * (odom_node.cpp:69-80) with no IMU / wheel odometry (launch default use_imu=false, use_odom=false):
 *   - constant-velocity guess: previous_pose + diff_pose with roll/pitch held (:234-236), Pose6D2Matrix (Z*Y*X);
 *   - setInputSource + align + getFitnessScore (:277-283) on the MI355X registration (include/ndt_hip.h);
 *   - keyframe gate: shift_dis = |dxy| >= min_add_scan_shift -> the scan, transformed by t_localizer and
 *     VoxelGrid-downsampled, is appended to localmap and tmp_map, and the target is rebuilt from pc_target_,
 *     the copy of localmap taken BEFORE this scan's append (one-scan lag, :233, 329-346);
 *   - localmap reset: localmap_size >= max_submap_size -> localmap = tmp_map, tmp_map cleared (:352-356).
 * localmap / tmp_map / pc_target_ live in HBM; a scan is handed over as host x,y,z(,i) or a device float4 array.
 */
#ifndef NDT_ODOM_H_
#define NDT_ODOM_H_

#include "ndt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ndt_odom ndt_odom;

/* LidarOdom::ParamInitial (odom_node.cpp:42-99) */
typedef struct {
    float ndt_resolution;       /* "ndt_resolution"      default 2.0  (:43)                        */
    double ndt_step_size;       /* "ndt_step_size"       default 0.1  (:44)                        */
    double ndt_trans_eps;       /* "ndt_trans_eps"       default 0.01 (:45)                        */
    int ndt_max_iter;           /* "ndt_max_iter"        default 30   (:46)                        */
    double min_add_scan_shift;  /* "min_add_scan_shift"  default 0.5  (:47)                        */
    double max_submap_size;     /* "max_submap_size"     default 5    (:49)                        */
    double init_pose[6];        /* init_x, init_y, init_z, init_roll, init_pitch, init_yaw (:86-94), default 0 */
    float localmap_leaf;        /* downSizeFilterLocalmap leaf = 2 * 0.5 (:96-98)                   */
    int search;                 /* setNeighborhoodSearchMethod(DIRECT7) (:73)                     */
    int compute_fitness;        /* getFitnessScore() after every align (:280); 1                  */
    int device;                 /* HIP device ordinal                                           */
    int method_type;            /* "ndt_method_type" (:55-69): 0 pcl_ndt, 1 ndt_cpu (launch default), 3 ndt_omp;
                                   default 3 here (the bench's replay path)                       */
    int incremental_voxel_update; /* "incremental_voxel_update" (:53, launch: false): ndt_cpu keyframes call
                                   updateVoxelGrid(transformed scan) instead of setInputTarget (:343-347) */
} ndt_odom_params;

/* common.h Pose6D: x, y, z, roll, pitch, yaw */
typedef struct {
    double x, y, z, roll, pitch, yaw;
} ndt_pose6d;

typedef struct {
    float init_guess[16];       /* Pose6D2Matrix(guess_pose).cast<float>() (:254), column-major             */
    float t_localizer[16];      /* getFinalTransformation() (:281)                                        */
    float t_base_link[16];      /* t_localizer * tf_l2b (:289)                                            */
    ndt_pose6d guess_pose;      /* (:234-236)                                                            */
    ndt_pose6d localizer_pose;  /* Matrix2Pose6D(t_localizer) (:291)                                      */
    ndt_pose6d current_pose;    /* = ndt_pose = Matrix2Pose6D(t_base_link) (:292-296)                      */
    ndt_pose6d diff_pose;       /* current - previous (:311)                                             */
    double fitness_score;       /* getFitnessScore() (:280); 0 when compute_fitness = 0                   */
    double shift_dis;           /* (:324)                                                                */
    double localmap_size;       /* after this scan (:330, :355)                                          */
    int has_converged;
    int final_num_iteration;
    int keyframe;               /* shift_dis >= min_add_scan_shift: appended + target rebuilt (:329-346)   */
    int localmap_reset;         /* localmap = tmp_map this scan (:352-356)                                */
    long long n_localmap;       /* points in localmap / tmp_map / the registration target after this scan   */
    long long n_tmp_map;
    long long n_target;
    long long n_appended;       /* points the downsampled scan added (0 when not a keyframe)                */
    int n_passes;               /* derivative passes of this align                                        */
    long long n_pairs;
    /* host wall clock (ms): setInputSource+align (includes waiting for a pending target build); the wait for the
     * fitness score and for the keyframe insertion count once the keyframe work is queued (in a batch: after the next
     * scan's align); the scan's two stages together */
    double ms_align, ms_fitness, ms_map, ms_total;
} ndt_odom_result;

ndt_status ndt_odom_default_params(ndt_odom_params* out);
ndt_status ndt_odom_create(const ndt_odom_params* params, ndt_odom** out);
/* OdomEstimate(filtered_scan_ptr, current_scan_time) (:208-356) for a host scan: x,y,z float at the start of each
 * stride_bytes record (32 = pcl::PointXYZI, intensity at byte offset 16 carried into the localmap when
 * stride_bytes >= 20, else 0).  An empty scan is rejected as the reference does (:211-214): NDT_EINVAL, state
 * unchanged. */
ndt_status ndt_odom_process(ndt_odom* o, const float* xyz, size_t n, size_t stride_bytes, double stamp, ndt_odom_result* out);
/* Same for a device-resident float4 x,y,z,intensity scan (read during the call only). */
ndt_status ndt_odom_process_device(ndt_odom* o, const float* d_xyz4, size_t n, double stamp, ndt_odom_result* out);
/* OdomEstimate over `count` device scans in order (an offline replay of a recorded sequence): the same per-scan work and
 * records as `count` ndt_odom_process_device calls, pipelined — each scan's getFitnessScore and keyframe insertion are
 * collected after the NEXT scan's align instead of before its record is returned, so they run beside that align and
 * the target build.  The scans stay unmodified until the call returns; on a failure the records before the failing scan
 * are complete. */
ndt_status ndt_odom_process_batch_device(ndt_odom* o, const float* const* d_scans, const size_t* n, const double* stamps, int count,
                                         ndt_odom_result* out);
/* The registration object the driver owns (timings, history, grid inspection through include/ndt_hip.h). */
ndt_ctx* ndt_odom_registration(ndt_odom* o);
/* Copies of the current localmap (which = 0), tmp_map (1) or registration target pc_target_ (2) as x,y,z,i
 * float4; *n_out receives the full size even when cap is smaller. */
ndt_status ndt_odom_get_cloud(ndt_odom* o, int which, float* out4, size_t cap, size_t* n_out);
const char* ndt_odom_last_error(const ndt_odom* o);
void ndt_odom_destroy(ndt_odom* o);

#ifdef __cplusplus
}
#endif
#endif /* NDT_ODOM_H_ */
