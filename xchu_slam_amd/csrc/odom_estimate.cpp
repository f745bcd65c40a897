// odom_estimate.cpp — the odom_node scan loop (LidarOdom::OdomEstimate) over the MI355X registration.
//
// Plain host C++ written against the public surface only (include/ndt_hip.hpp over include/ndt_hip.h): it is the
// caller odom_node is, not part of the device library.  Reference: xchu_mapping/src/odom_node.cpp:208-356
// (scan loop), :42-99 (parameters), xchu_mapping/include/xchu_mapping/common.h:38-71 (Pose6D helpers).
// localmap, tmp_map and the registration target (pc_target_) are device float4 clouds; per scan the host
// does the pose arithmetic (a few hundred flops) and issues: set_source, align (one sync), getFitnessScore (side
// stream), and on keyframes transform -> VoxelGrid -> appends (side stream) and the target rebuild + its fitness index;
// then waits for the score and the appended count.  ndt_odom_process_batch_device runs the same steps pipelined: a
// scan's score and count are collected after the NEXT scan's align (they overlap it and the target build).
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ndt_hip.hpp"
#include "../../include/ndt_odom.h"

namespace {

struct Pose6D {
    double x = 0, y = 0, z = 0, roll = 0, pitch = 0, yaw = 0;
};

// common.h:38-44
Pose6D operator+(const Pose6D& a, const Pose6D& b) {
    return Pose6D{a.x + b.x, a.y + b.y, a.z + b.z, a.roll + b.roll, a.pitch + b.pitch, a.yaw + b.yaw};
}
Pose6D operator-(const Pose6D& a, const Pose6D& b) {
    return Pose6D{a.x - b.x, a.y - b.y, a.z - b.z, a.roll - b.roll, a.pitch - b.pitch, a.yaw - b.yaw};
}

using M3 = double[3][3];

// Eigen::AngleAxisd(angle, unit axis e_k).toRotationMatrix() (Eigen 3.3 AngleAxis.h): the diagonal entry of the
// axis is (1 - c) * 1 + c, the other two are 0 * 0 + c; off-diagonals are 0 * 0 -/+ s.
void axis_rotation(double angle, int axis, M3 R) {
    const double s = std::sin(angle), c = std::cos(angle);
    const double ax[3] = {axis == 0 ? 1.0 : 0.0, axis == 1 ? 1.0 : 0.0, axis == 2 ? 1.0 : 0.0};
    const double sa[3] = {s * ax[0], s * ax[1], s * ax[2]};
    const double ca[3] = {(1.0 - c) * ax[0], (1.0 - c) * ax[1], (1.0 - c) * ax[2]};
    double t = ca[0] * ax[1];
    R[0][1] = t - sa[2]; R[1][0] = t + sa[2];
    t = ca[0] * ax[2];
    R[0][2] = t + sa[1]; R[2][0] = t - sa[1];
    t = ca[1] * ax[2];
    R[1][2] = t - sa[0]; R[2][1] = t + sa[0];
    for (int k = 0; k < 3; ++k) R[k][k] = ca[k] * ax[k] + c;
}

// fixed-size 3x3 lazy product: each coefficient is the unrolled redux a0*b0 + (a1*b1 + a2*b2)
void mul3(const M3 A, const M3 B, M3 C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + (A[i][1] * B[1][j] + A[i][2] * B[2][j]);
}

// Pose6D2Matrix (common.h:64-71): (Translation3d * AngleAxisd(yaw, Z) * AngleAxisd(pitch, Y) * AngleAxisd(roll, X))
// in double, then .cast<float>() as odom_node does (:254, :93).  Column-major out.
ndt_hip::Matrix4f pose_to_matrix(const Pose6D& p) {
    M3 Rz, Ry, Rx, Rzy, R;
    axis_rotation(p.yaw, 2, Rz);
    axis_rotation(p.pitch, 1, Ry);
    axis_rotation(p.roll, 0, Rx);
    mul3(Rz, Ry, Rzy);
    mul3(Rzy, Rx, R);
    ndt_hip::Matrix4f m{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i + 4 * j] = (float)R[i][j];
    m[12] = (float)p.x; m[13] = (float)p.y; m[14] = (float)p.z; m[15] = 1.0f;
    return m;
}

// Matrix2Pose6D (common.h:51-63) of a float matrix cast to double: Eigen::Quaterniond(rot) (Eigen 3.3
// quaternionbase_assign_impl, trace branch / largest-diagonal branch), then tf::Matrix3x3(q).getRPY
// (ROS tf LinearMath Matrix3x3::setRotation + getEulerYPR, solution 1).  tf is a third-party dependency of the
// reference, restated from its published source.
Pose6D matrix_to_pose(const ndt_hip::Matrix4f& mf) {
    double m[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i][j] = (double)mf[i + 4 * j];
    double q[4];  // x, y, z, w
    double t = m[0][0] + (m[1][1] + m[2][2]);
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[2][1] - m[1][2]) * t;
        q[1] = (m[0][2] - m[2][0]) * t;
        q[2] = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[k][j] - m[j][k]) * t;
        q[j] = (m[j][i] + m[i][j]) * t;
        q[k] = (m[k][i] + m[i][k]) * t;
    }
    // tf::Matrix3x3::setRotation
    const double d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    const double s = 2.0 / d;
    const double xs = q[0] * s, ys = q[1] * s, zs = q[2] * s;
    const double wx = q[3] * xs, wy = q[3] * ys, wz = q[3] * zs;
    const double xx = q[0] * xs, xy = q[0] * ys, xz = q[0] * zs;
    const double yy = q[1] * ys, yz = q[1] * zs, zz = q[2] * zs;
    const double r00 = 1.0 - (yy + zz), r10 = xy + wz;
    const double r20 = xz - wy, r21 = yz + wx, r22 = 1.0 - (xx + yy);
    Pose6D p;
    p.x = (double)mf[12]; p.y = (double)mf[13]; p.z = (double)mf[14];
    // tf::Matrix3x3::getEulerYPR(yaw, pitch, roll, 1)
    if (std::fabs(r20) >= 1.0) {
        p.yaw = 0.0;
        const double delta = std::atan2(r21, r22);
        p.pitch = r20 < 0.0 ? M_PI / 2.0 : -M_PI / 2.0;
        p.roll = delta;
    } else {
        p.pitch = -std::asin(r20);
        const double cp = std::cos(p.pitch);
        p.roll = std::atan2(r21 / cp, r22 / cp);
        p.yaw = std::atan2(r10 / cp, r00 / cp);
    }
    return p;
}

// Matrix4f * Matrix4f (column j = ((A.c0 * b0j + A.c1 * b1j) + A.c2 * b2j) + A.c3 * b3j)
ndt_hip::Matrix4f mul4(const ndt_hip::Matrix4f& A, const ndt_hip::Matrix4f& B) {
    ndt_hip::Matrix4f C{};
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i)
            C[i + 4 * j] = ((A[i] * B[4 * j] + A[i + 4] * B[1 + 4 * j]) + A[i + 8] * B[2 + 4 * j]) + A[i + 12] * B[3 + 4 * j];
    return C;
}

// Matrix4f::inverse() of the rigid tf_b2l (odom_node.cpp:94), via cofactors in double.  Exact for the default
// identity; for other init poses it may differ from Eigen's SSE 4x4 inverse in the last bit.
ndt_hip::Matrix4f inverse4(const ndt_hip::Matrix4f& mf) {
    double a[16], inv[16];
    for (int k = 0; k < 16; ++k) a[k] = mf[k];
    inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] + a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
    inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] - a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
    inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] + a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
    inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] - a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
    inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] - a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
    inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] + a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
    inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] - a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
    inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] + a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
    inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] + a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
    inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] - a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
    inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] + a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
    inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] - a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
    inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] - a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
    inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] + a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
    inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] - a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
    inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] + a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
    const double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
    ndt_hip::Matrix4f out{};
    for (int k = 0; k < 16; ++k) out[k] = (float)(inv[k] / det);
    return out;
}

#ifdef NDT_ODOM_PROF
// host time per call site of the scan loop (profiling build only; printed by ndt_odom_destroy)
struct HostProf {
    double ms[10] = {};
    long long n[10] = {};
    ~HostProf() {
        static const char* names[10] = {"finish", "fit_async", "ins_async", "memcpy", "set_target", "fit_index", "set_source",
                                        "align", "finish_in_begin", "other"};
        for (int k = 0; k < 10; ++k)
            if (n[k]) fprintf(stderr, "odom host %-16s %8.2f us x %lld\n", names[k], 1000.0 * ms[k] / (double)n[k], n[k]);
    }
};
static HostProf g_hp;
#define HP_BEGIN(k) const auto _hp##k = std::chrono::steady_clock::now()
#define HP_END(k) (g_hp.ms[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - _hp##k).count(), ++g_hp.n[k])
#else
#define HP_BEGIN(k) do { } while (0)
#define HP_END(k) do { } while (0)
#endif

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

ndt_pose6d to_c(const Pose6D& p) { return ndt_pose6d{p.x, p.y, p.z, p.roll, p.pitch, p.yaw}; }

}  // namespace

// a growable device float4 cloud allocated through the registration's ctx
struct DevCloud {
    float* p = nullptr;
    size_t n = 0, cap = 0;
};

struct ndt_odom {
    ndt_odom_params prm{};
    ndt_hip::NormalDistributionsTransform* reg = nullptr;
    std::string err;
    DevCloud localmap, tmp_map, target[2], scan, transformed, ds;
    int target_cur = -1;            // which target buffer the registration references
    // the target is a snapshot of localmap's first tgt_prefix_n points and localmap has only grown since (no reset):
    // the next snapshot extends it (ndt_set_target_append_device)
    bool tgt_is_prefix = false;
    size_t tgt_prefix_n = 0;
    bool initial_scan_loaded = false;
    long long n_keyframes = 0;      // cloud_keyframes_.size()
    Pose6D previous_pose, diff_pose, current_pose;
    double previous_scan_time = 0.0;
    double localmap_size = 0.0, odom_size = 0.0;
    double velocity[3] = {0, 0, 0};
    ndt_hip::Matrix4f tf_b2l{}, tf_l2b{};
    // the scan whose getFitnessScore / keyframe insertion are still in flight (odom_begin -> odom_finish)
    ndt_odom_result* pend = nullptr;
    bool pend_keyframe = false, pend_reset = false;
    double pend_ms = 0.0;
};

namespace {

ndt_status odom_fail(ndt_odom* o, ndt_status s, const std::string& msg) {
    if (o) o->err = msg;
    return s;
}

#define OTRY(expr)                                                                          \
    do {                                                                                    \
        ndt_status _s = (expr);                                                             \
        if (_s != NDT_OK) return odom_fail(o, _s, std::string(#expr) + ": " + ndt_last_error(o->reg->handle())); \
    } while (0)

ndt_status reserve(ndt_odom* o, DevCloud& c, size_t n, bool keep) {
    if (n <= c.cap) return NDT_OK;
    size_t cap = std::max<size_t>(n, c.cap + c.cap / 2);
    cap = std::max<size_t>(cap, 1 << 16);
    void* p = nullptr;
    ndt_ctx* ctx = o->reg->handle();
    OTRY(ndt_device_alloc(ctx, cap * 16, &p));
    if (keep && c.n) OTRY(ndt_memcpy_d2d(ctx, p, c.p, c.n * 16));
    if (c.p) OTRY(ndt_device_free(ctx, c.p));
    c.p = static_cast<float*>(p);
    c.cap = cap;
    return NDT_OK;
}

// setInputTarget(pc_target_) where pc_target_ is the current localmap: snapshot into the buffer the registration
// does not reference, then point the registration at it (the build reads it on the stream, in order)
ndt_status set_target_from_localmap(ndt_odom* o) {
    const int nxt = o->target_cur == 0 ? 1 : 0;
    DevCloud& t = o->target[nxt];
    OTRY(reserve(o, t, o->localmap.n, false));
    if (o->localmap.n) OTRY(ndt_memcpy_d2d(o->reg->handle(), t.p, o->localmap.p, o->localmap.n * 16));
    t.n = o->localmap.n;
    OTRY(ndt_set_target_device(o->reg->handle(), t.p, t.n, 1));
    o->target_cur = nxt;
    o->tgt_is_prefix = true;
    o->tgt_prefix_n = t.n;
    // getFitnessScore (:280) queries this target every scan: its index is built now, beside the voxel build and the align
    if (o->prm.compute_fitness) OTRY(ndt_fitness_index_async(o->reg->handle()));
    return NDT_OK;
}

bool incremental(const ndt_odom* o) { return o->prm.method_type == 1 && o->prm.incremental_voxel_update != 0; }

// OdomEstimate (odom_node.cpp:208-356), second half: the pending scan's getFitnessScore and appended count collected,
// then the map bookkeeping (:337-338, the localmap reset :352-356 decided in odom_begin) and its record completed.
ndt_status odom_finish(ndt_odom* o) {
    ndt_odom_result* out = o->pend;
    if (!out) return NDT_OK;
    o->pend = nullptr;
    ndt_ctx* ctx = o->reg->handle();
    auto t0 = std::chrono::steady_clock::now();
    // a getFitnessScore failure is reported only after the keyframe insertion has been collected and counted into the
    // maps, so that the map bookkeeping stays complete whichever lane failed
    ndt_status st_fit = NDT_OK;
    std::string err_fit;
    if (o->prm.compute_fitness) {
        st_fit = ndt_fitness_score_result(ctx, &out->fitness_score);
        if (st_fit != NDT_OK) err_fit = std::string("ndt_fitness_score_result: ") + ndt_last_error(ctx);
    }
    out->ms_fitness = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    size_t appended = 0;
    if (o->pend_keyframe) {
        const ndt_status st = ndt_keyframe_insert_result(ctx, &appended);
        if (st != NDT_OK && st != NDT_EOVERFLOW) return odom_fail(o, st, std::string("keyframe insert: ") + ndt_last_error(ctx));
        const size_t base = o->localmap.n;
        o->localmap.n += appended;
        o->tmp_map.n += appended;
        // :343-345 ndt_cpu with incremental_voxel_update: updateVoxelGrid(transformed_scan_ptr) — the downsampled
        // keyframe just appended to localmap — instead of setInputTarget(pc_target_)
        if (incremental(o) && appended) {
            OTRY(ndt_update_target_device(ctx, o->localmap.p + 4 * base, appended));
            if (o->prm.compute_fitness) OTRY(ndt_fitness_index_async(ctx));
        }
    }
    out->ms_map = ms_since(t0);
    // :352-356
    if (o->pend_reset) {
        std::swap(o->localmap, o->tmp_map);
        o->tmp_map.n = 0;
        o->tgt_is_prefix = false;  // localmap is now the points since the last reset, not a growth of the target
    }
    out->n_localmap = (long long)o->localmap.n;
    out->n_tmp_map = (long long)o->tmp_map.n;
    out->n_target = o->target_cur >= 0 ? (long long)o->target[o->target_cur].n : 0;
    out->n_appended = (long long)appended;
    out->ms_total = o->pend_ms + out->ms_fitness + out->ms_map;
    if (st_fit != NDT_OK) return odom_fail(o, st_fit, err_fit);
    return NDT_OK;
}

// OdomEstimate (odom_node.cpp:208-356), first half, on a device scan of n float4 points: the align (one sync), the pose
// arithmetic and the keyframe decision; the previous scan's results collected (odom_finish) if still pending; then this
// scan's getFitnessScore and keyframe work queued and the scan left pending.  d_scan stays unmodified until its
// odom_finish.
ndt_status odom_begin(ndt_odom* o, const float* d_scan, size_t n, double stamp, ndt_odom_result* out) {
    ndt_ctx* ctx = o->reg->handle();
    std::memset(out, 0, sizeof(*out));
    const auto t_call = std::chrono::steady_clock::now();
    if (!o->initial_scan_loaded || o->n_keyframes == 0) {
        OTRY(odom_finish(o));
        // :218-231 — the first scan, moved into the body frame, seeds localmap and the target
        OTRY(reserve(o, o->localmap, o->localmap.n + n, true));
        OTRY(ndt_transform_device(ctx, o->tf_l2b.data(), d_scan, n, o->localmap.p + 4 * o->localmap.n));
        o->localmap.n += n;
        OTRY(set_target_from_localmap(o));  // pc_target_ (empty) += transformed == localmap here
        o->initial_scan_loaded = true;
    }
    // :233 pc_target_ = copy of localmap — materialised at the keyframe below, before this scan's append

    // :234-236 constant-velocity guess, roll/pitch held
    Pose6D guess = o->previous_pose + o->diff_pose;
    guess.pitch = o->previous_pose.pitch;
    guess.roll = o->previous_pose.roll;
    const ndt_hip::Matrix4f init_guess = pose_to_matrix(guess);  // :254

    // :277-283 (the target this align needs was queued on the device stream by the previous scan)
    auto t0 = std::chrono::steady_clock::now();
    HP_BEGIN(6);
    OTRY(ndt_set_source_device(ctx, d_scan, n));
    HP_END(6);
    HP_BEGIN(7);
    o->reg->align(init_guess);
    HP_END(7);
    const ndt_result& r = o->reg->result();
    out->ms_align = ms_since(t0);
    const ndt_hip::Matrix4f t_localizer = o->reg->getFinalTransformation();

    // :289-300
    const ndt_hip::Matrix4f t_base_link = mul4(t_localizer, o->tf_l2b);
    const Pose6D localizer_pose = matrix_to_pose(t_localizer);
    const Pose6D ndt_pose = matrix_to_pose(t_base_link);
    o->current_pose = ndt_pose;
    ++o->n_keyframes;  // cloud_keyframes_.push_back (:299)

    // :303-327
    const double secs = stamp - o->previous_scan_time;
    o->diff_pose = o->current_pose - o->previous_pose;
    o->velocity[0] = o->diff_pose.x / secs;
    o->velocity[1] = o->diff_pose.y / secs;
    o->velocity[2] = o->diff_pose.z / secs;
    const double shift_dis = std::sqrt(std::pow(o->current_pose.x - o->previous_pose.x, 2.0) +
                                       std::pow(o->current_pose.y - o->previous_pose.y, 2.0));
    o->previous_pose = o->current_pose;
    o->previous_scan_time = stamp;

    // the previous scan's score and appended count (its keyframe work ran beside this align), before this scan's
    // fitness query reuses the result slot and its keyframe work reads the map sizes
    HP_BEGIN(8);
    OTRY(odom_finish(o));
    HP_END(8);

    const bool keyframe = shift_dis >= o->prm.min_add_scan_shift;
    if (keyframe) {
        // :329-346 transformed scan (:290) -> VoxelGrid(1.0) -> localmap += , tmp_map += , setInputTarget(pc_target_);
        // pc_target_ is the localmap as it was before this append
        o->localmap_size += shift_dis;
        o->odom_size += shift_dis;
        OTRY(reserve(o, o->localmap, o->localmap.n + n, true));
        OTRY(reserve(o, o->tmp_map, o->tmp_map.n + n, true));
        // pc_target_ between resets = the current target plus the keyframes appended since: the current snapshot is
        // extended in place (the build stores the new points; the old ones, which the fit lane may still be indexing,
        // are not touched) when its buffer has room, else a full snapshot goes to the other buffer
        const int cur = o->target_cur;
        const bool grow = !incremental(o) && o->tgt_is_prefix && cur >= 0 && o->localmap.n >= o->tgt_prefix_n &&
                          o->target[cur].n == o->tgt_prefix_n;
        const bool in_place = grow && o->target[cur].cap >= o->localmap.n;
        const int nxt = in_place ? cur : (cur == 0 ? 1 : 0);
        DevCloud& t = o->target[nxt];
        if (!in_place) OTRY(reserve(o, t, o->localmap.n, false));
        // the side lanes (getFitnessScore :280, the insertion) queue behind this mark — the align and the map growth —
        // and beside what the main stream queues next; the insertion job is posted after the pc_target_ copy and the
        // target build are queued (the next align waits for those, not for the insertion).  It appends behind the
        // points the copy reads.
        OTRY(ndt_side_lanes_mark(ctx));
        // getFitnessScore (:280) against the target this scan was aligned to: queued before setInputTarget replaces it,
        // or (fit_late) after the new target's build is queued, against the aligned target's index
        const bool fit_late = std::getenv("NDT_ODOM_FIT_LATE") != nullptr;
        const bool late = fit_late && o->prm.compute_fitness && !incremental(o);
        HP_BEGIN(1);
        if (o->prm.compute_fitness && !late) OTRY(ndt_fitness_score_async_cloud(ctx, nullptr, DBL_MAX, d_scan, n));
        HP_END(1);
        HP_BEGIN(3);
        if (!in_place && o->localmap.n) OTRY(ndt_memcpy_d2d(ctx, t.p, o->localmap.p, o->localmap.n * 16));
        HP_END(3);
        const size_t n_old = o->tgt_prefix_n;
        t.n = o->localmap.n;
        if (!incremental(o)) {
            HP_BEGIN(4);
            // a grown target's grid extends the current one by merge (the same grid as a fresh setInputTarget)
            if (in_place)
                OTRY(ndt_set_target_append_device(ctx, t.p, n_old, t.n - n_old, 1, o->localmap.p + 4 * n_old));
            else if (grow)
                OTRY(ndt_set_target_append_device(ctx, t.p, n_old, t.n - n_old, 1, nullptr));
            else
                OTRY(ndt_set_target_device(ctx, t.p, t.n, 1));
            o->tgt_is_prefix = true;
            o->tgt_prefix_n = t.n;
            HP_END(4);
        }
        if (late) OTRY(ndt_fitness_score_async_aligned(ctx, DBL_MAX, d_scan, n));
        HP_BEGIN(2);
        OTRY(ndt_keyframe_insert_async(ctx, t_localizer.data(), d_scan, n, o->prm.localmap_leaf, o->localmap.p, o->localmap.n,
                                       o->tmp_map.p, o->tmp_map.n));
        HP_END(2);
        if (!incremental(o)) {
            o->target_cur = nxt;
            HP_BEGIN(5);
            if (o->prm.compute_fitness) OTRY(ndt_fitness_index_async(ctx));
            HP_END(5);
        }
    } else {
        // getFitnessScore (:280): queued on the registration's side stream over this scan's points
        HP_BEGIN(1);
        if (o->prm.compute_fitness) OTRY(ndt_fitness_score_async_cloud(ctx, nullptr, DBL_MAX, d_scan, n));
        HP_END(1);
    }
    // :352-356 decided now, applied with the appended count (odom_finish)
    const bool reset = o->localmap_size >= o->prm.max_submap_size;
    if (reset) o->localmap_size = 0.0;

    for (int k = 0; k < 16; ++k) {
        out->init_guess[k] = init_guess[k];
        out->t_localizer[k] = t_localizer[k];
        out->t_base_link[k] = t_base_link[k];
    }
    out->guess_pose = to_c(guess);
    out->localizer_pose = to_c(localizer_pose);
    out->current_pose = to_c(o->current_pose);
    out->diff_pose = to_c(o->diff_pose);
    out->shift_dis = shift_dis;
    out->localmap_size = o->localmap_size;
    out->has_converged = r.converged;
    out->final_num_iteration = r.nr_iterations;
    out->keyframe = keyframe ? 1 : 0;
    out->localmap_reset = reset ? 1 : 0;
    out->n_passes = r.n_passes;
    out->n_pairs = r.n_pairs;
    o->pend = out;
    o->pend_keyframe = keyframe;
    o->pend_reset = reset;
    o->pend_ms = ms_since(t_call);
    // updateVoxelGrid (ndt_cpu, incremental) changes the target the next align uses: nothing may pend past it
    if (incremental(o) && keyframe) return odom_finish(o);
    return NDT_OK;
}

// After a failed call: the scan left pending by the previous odom_begin (its record lives in the caller's array, which
// the caller may free once this call returns) is completed now — its getFitnessScore and keyframe insertion collected,
// its appended points counted into the maps — so that no pointer into the caller's records survives the call and the
// records before the failing scan are complete.  The first error's message is kept.
void settle_pending(ndt_odom* o) {
    if (!o->pend) return;
    const std::string first = o->err;
    try {
        (void)odom_finish(o);
    } catch (const ndt_hip::Error&) {
    }
    o->pend = nullptr;
    o->err = first;
}

void free_cloud(ndt_odom* o, DevCloud& c) {
    if (c.p) (void)ndt_device_free(o->reg->handle(), c.p);
    c = DevCloud{};
}

}  // namespace

extern "C" {

ndt_status ndt_odom_default_params(ndt_odom_params* p) {
    if (!p) return NDT_EINVAL;
    std::memset(p, 0, sizeof(*p));
    p->ndt_resolution = 2.0f;
    p->ndt_step_size = 0.1;
    p->ndt_trans_eps = 0.01;
    p->ndt_max_iter = 30;
    p->min_add_scan_shift = 0.5;
    p->max_submap_size = 5.0;
    p->localmap_leaf = 1.0f;
    p->search = NDT_DIRECT7;
    p->compute_fitness = 1;
    p->device = 0;
    p->method_type = 3;
    p->incremental_voxel_update = 0;
    return NDT_OK;
}

ndt_status ndt_odom_create(const ndt_odom_params* params, ndt_odom** out) {
    if (!out) return NDT_EINVAL;
    *out = nullptr;
    ndt_odom_params p;
    if (params) p = *params; else ndt_odom_default_params(&p);
    if (!(p.ndt_resolution > 0.f) || !(p.localmap_leaf > 0.f) || p.ndt_max_iter < 0 || p.search < 0 || p.search > 3 ||
        !(p.method_type == 0 || p.method_type == 1 || p.method_type == 3))
        return NDT_EINVAL;
    ndt_odom* o = new ndt_odom();
    o->prm = p;
    try {
        o->reg = new ndt_hip::NormalDistributionsTransform(p.device);
        // odom_node.cpp:71-78
        o->reg->setNeighborhoodSearchMethod(static_cast<ndt_hip::NeighborSearchMethod>(p.search));
        // MethodType (:55-69): use_pcl -> pcl::NormalDistributionsTransform, use_cpu -> cpu:: (ndt_cpu), use_omp -> pclomp
        o->reg->setPrecisionMode(p.method_type == 0 ? 1 : (p.method_type == 1 ? 2 : 0));
        o->reg->setTransformationEpsilon(p.ndt_trans_eps);
        o->reg->setStepSize(p.ndt_step_size);
        o->reg->setResolution(p.ndt_resolution);
        o->reg->setMaximumIterations(p.ndt_max_iter);
    } catch (const ndt_hip::Error& e) {
        const ndt_status s = e.status;
        delete o->reg;
        delete o;
        return s;
    }
    // :92-94
    Pose6D tl{p.init_pose[0], p.init_pose[1], p.init_pose[2], p.init_pose[3], p.init_pose[4], p.init_pose[5]};
    o->tf_b2l = pose_to_matrix(tl);
    o->tf_l2b = inverse4(o->tf_b2l);
    *out = o;
    return NDT_OK;
}

ndt_status ndt_odom_process_device(ndt_odom* o, const float* d_xyz4, size_t n, double stamp, ndt_odom_result* out) {
    if (!o || !out) return NDT_EINVAL;
    if (n == 0 || !d_xyz4) return odom_fail(o, NDT_EINVAL, "check your cloud...");  // :211-214
    ndt_status st = NDT_OK;
    try {
        st = odom_finish(o);  // a batch's last scan is complete already; nothing pends between calls
        if (st == NDT_OK) st = odom_begin(o, d_xyz4, n, stamp, out);
        if (st == NDT_OK) st = odom_finish(o);
    } catch (const ndt_hip::Error& e) {
        st = odom_fail(o, e.status, e.what());
    }
    if (st != NDT_OK) settle_pending(o);
    return st;
}

ndt_status ndt_odom_process_batch_device(ndt_odom* o, const float* const* d_scans, const size_t* n, const double* stamps, int count,
                                         ndt_odom_result* out) {
    if (!o || count < 0 || (count && (!d_scans || !n || !stamps || !out))) return o ? odom_fail(o, NDT_EINVAL, "bad batch") : NDT_EINVAL;
    for (int k = 0; k < count; ++k)
        if (n[k] == 0 || !d_scans[k]) return odom_fail(o, NDT_EINVAL, "check your cloud...");  // :211-214, before any scan runs
    ndt_status st = NDT_OK;
    try {
        for (int k = 0; k < count && st == NDT_OK; ++k) st = odom_begin(o, d_scans[k], n[k], stamps[k], &out[k]);
        if (st == NDT_OK) st = odom_finish(o);
    } catch (const ndt_hip::Error& e) {
        st = odom_fail(o, e.status, e.what());
    }
    // a failure leaves no scan pending: the records before the failing scan are complete (ndt_odom.h)
    if (st != NDT_OK) settle_pending(o);
    return st;
}

ndt_status ndt_odom_process(ndt_odom* o, const float* xyz, size_t n, size_t stride_bytes, double stamp, ndt_odom_result* out) {
    if (!o || !out || stride_bytes < 12) return o ? odom_fail(o, NDT_EINVAL, "bad scan") : NDT_EINVAL;
    if (n == 0 || !xyz) return odom_fail(o, NDT_EINVAL, "check your cloud...");
    std::vector<float> tmp(4 * n);
    const char* base = reinterpret_cast<const char*>(xyz);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        tmp[4 * i] = f[0]; tmp[4 * i + 1] = f[1]; tmp[4 * i + 2] = f[2];
        tmp[4 * i + 3] = stride_bytes >= 20 ? f[4] : 0.0f;
    }
    OTRY(reserve(o, o->scan, n, false));
    OTRY(ndt_memcpy_h2d(o->reg->handle(), o->scan.p, tmp.data(), n * 16));
    o->scan.n = n;
    return ndt_odom_process_device(o, o->scan.p, n, stamp, out);
}

ndt_ctx* ndt_odom_registration(ndt_odom* o) { return o && o->reg ? o->reg->handle() : nullptr; }

ndt_status ndt_odom_get_cloud(ndt_odom* o, int which, float* out4, size_t cap, size_t* n_out) {
    if (!o || !n_out || which < 0 || which > 2 || (cap && !out4)) return NDT_EINVAL;
    const DevCloud* c = which == 0 ? &o->localmap : which == 1 ? &o->tmp_map : (o->target_cur >= 0 ? &o->target[o->target_cur] : nullptr);
    *n_out = c ? c->n : 0;
    if (!c) return NDT_OK;
    const size_t m = std::min(cap, c->n);
    ndt_ctx* ctx = o->reg->handle();
    OTRY(ndt_synchronize(ctx));
    if (m) OTRY(ndt_memcpy_d2h(ctx, out4, c->p, m * 16));
    return NDT_OK;
}

const char* ndt_odom_last_error(const ndt_odom* o) { return o ? o->err.c_str() : "null odom"; }

void ndt_odom_destroy(ndt_odom* o) {
    if (!o) return;
    if (o->reg) {
        (void)ndt_synchronize(o->reg->handle());
        for (DevCloud* c : {&o->localmap, &o->tmp_map, &o->target[0], &o->target[1], &o->scan, &o->transformed, &o->ds}) free_cloud(o, *c);
        delete o->reg;
    }
    delete o;
}

}  // extern "C"
