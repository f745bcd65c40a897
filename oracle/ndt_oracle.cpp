// oracle/ndt_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// Clean-room CPU restatement of the reference NDT scan-matching path
// (pclomp::NormalDistributionsTransform + pclomp::VoxelGridCovariance as called
// by odom_node, lowmee/xchu_slam).  Used ONLY by tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg, as the checker / CPU baseline.  Never linked
// into or called by the product library (xchu_slam_amd/libndt_hip.so).
//
// PARITY STATUS: UNPINNED.  The reference ships no tests, fixtures or golden
// vectors for this path; its sources need Eigen/PCL/Boost/
// FLANN which are absent here, so it cannot be compiled (no oracle/_ref); its
// prebuilt .so files are never loaded (task rules).  This restatement follows
// the reference text line by line (citations below) and is checked against
// analytic known-answer tests (finite differences, rigid-transform recovery,
// closed-form voxel statistics) in tests/test_oracle.py.
//
// Followed reference files (paths relative to /root/reference/xchu_mapping/):
//   include/pclomp/ndt_omp_impl.hpp        :46-69 ctor, :73-164 computeTransformation,
//       :175-283 computeDerivatives, :286-398 computeAngleDerivatives,
//       :401-488 computePointDerivatives, :491-548 updateDerivatives,
//       :550-641 computeHessian/updateHessian, :643-916 More-Thuente,
//       :919-952 calculateScore
//   include/pclomp/ndt_omp.h               :117-137 setInputTarget/setResolution,
//       :210-229 convertTransform, :271-278 init, :425-442 MT auxiliary functions
//   include/pclomp/voxel_grid_covariance_omp_impl.hpp :48-370 applyFilter,
//       :373-442 getNeighborhoodAtPoint{,7,1}
//   include/pclomp/voxel_grid_covariance_omp.h :92-187 Leaf (cov_ starts at Identity!),
//       :202-217 defaults, :470-499 radiusSearch
// Third-party semantics restated (not vendored, versions inferred):
//   PCL ~1.7: Registration::align, transformPointCloud (dense path), getMinMax3D,
//             VoxelGrid::setLeafSize, getAllNeighborCellIndices, KdTreeFLANN radius
//             search (exact, strict '<' on squared float distance, sorted ascending);
//             pcl::NormalDistributionsTransform (precision_mode 1 = "pcl_ndt").
//   Eigen 3.3: see eigen33_restate.h.
//   FLANN: L2_Simple float distance, RadiusResultSet (dist < r^2).
#include "eigen33_restate.h"

#include <cstdint>
#include <cstring>
#include <cstdio>
#include <map>
#include <tuple>
#include <cmath>
#include <vector>
#include <algorithm>
#include <limits>
#include <chrono>
#include <unordered_map>
#include <cmath>
#ifdef _OPENMP
#include <omp.h>
#endif

using e33::Mat;
typedef Mat<float, 3> M3f;
typedef Mat<double, 3> M3d;
typedef Mat<double, 6> M6d;

namespace orc {

enum Search { KDTREE = 0, DIRECT26 = 1, DIRECT7 = 2, DIRECT1 = 3 };

struct Pt { float x, y, z, w; };

struct Leaf {
    int nr_points = 0;
    double mean[3] = {0, 0, 0};
    float centroid[4] = {0, 0, 0, 0};
    M3d cov = M3d::identity();   // NOTE: Leaf() initialises cov_ to Identity (voxel_grid_covariance_omp.h:50)
    M3d icov = M3d::zero();
    M3d evecs = M3d::identity();
    double evals[3] = {0, 0, 0};
    int ppv = 0;                 // ndt_cpu: points_per_voxel_ (radiusSearch validity; -1 once rejected)
};

// ndt_cpu (Autoware cpu::VoxelGrid) raw per-voxel sums, kept across updateVoxelGrid calls
struct AwCell {
    double sum[3] = {0, 0, 0};
    M3d cov = M3d::identity();   // scatterPointsToVoxelGrid: tmp_cov_ starts at Identity (libndt_cpu.so, checked as text)
    int n = 0;
    int ppv = 0;
};

// cpu::SymmetricEigensolver3x3::compute (ndt_cpu/SymmetricEigenSolver.h:55-273) — its arithmetic, quirks included:
// the d_k "norms" multiply where they should add (:172-174), imax can never become 2 (:179-180), a diagonal input keeps
// its unsorted diagonal (:128-133).  Returns ascending-by-construction eigenvalues, eigenvectors as columns of V.
static void aw_cross3(const double u[3], const double v[3], double o[3]) {
    o[0] = u[1] * v[2] - u[2] * v[1];
    o[1] = u[2] * v[0] - u[0] * v[2];
    o[2] = u[0] * v[1] - u[1] * v[0];
}
static void aw_eigen3(const M3d& A, double ev[3], M3d& V) {
    double a00 = A(0, 0), a01 = A(0, 1), a02 = A(0, 2), a11 = A(1, 1), a12 = A(1, 2), a22 = A(2, 2);
    double m0 = std::fabs(a00) > std::fabs(a01) ? std::fabs(a00) : std::fabs(a01);
    double m1 = std::fabs(a02) > std::fabs(a11) ? std::fabs(a02) : std::fabs(a11);
    double m2 = std::fabs(a12) > std::fabs(a22) ? std::fabs(a12) : std::fabs(a22);
    double big = m0 > m1 ? m0 : m1;
    big = big > m2 ? big : m2;
    V = M3d::identity();
    if (big == 0.0) { ev[0] = ev[1] = ev[2] = 0.0; return; }
    const double s = 1.0 / big;
    a00 *= s; a01 *= s; a02 *= s; a11 *= s; a12 *= s; a22 *= s;
    const double off = a01 * a01 + a02 * a02 + a12 * a12;
    if (!(off > 0.0)) {
        ev[0] = a00 * big; ev[1] = a11 * big; ev[2] = a22 * big;
        return;
    }
    const double tr3 = (a00 + a11 + a22) / 3.0;
    const double b00 = a00 - tr3, b11 = a11 - tr3, b22 = a22 - tr3;
    const double den = std::sqrt((b00 * b00 + b11 * b11 + b22 * b22 + off * 2.0) / 6.0);
    const double c00 = b11 * b22 - a12 * a12, c01 = a01 * b22 - a12 * a02, c02 = a01 * a12 - b11 * a02;
    double hd = (b00 * c00 - a01 * c01 + a02 * c02) / (den * den * den) * 0.5;
    hd = hd > -1.0 ? hd : -1.0;
    hd = hd < 1.0 ? hd : 1.0;
    const double ang = std::acos(hd) / 3.0;
    const double be2 = std::cos(ang) * 2.0;
    const double be0 = std::cos(ang + M_PI * 2.0 / 3.0) * 2.0;
    const double be1 = -(be0 + be2);
    double e[3] = {tr3 + den * be0, tr3 + den * be1, tr3 + den * be2};
    const int j1 = 1, j0 = hd >= 0.0 ? 2 : 0, j2 = hd >= 0.0 ? 0 : 2;
    // first eigenvector: the best of three row cross products of (A - e_j0 I)
    const double R[3][3] = {{a00 - e[j0], a01, a02}, {a01, a11 - e[j0], a12}, {a02, a12, a22 - e[j0]}};
    double X[3][3];
    aw_cross3(R[0], R[1], X[0]);
    aw_cross3(R[0], R[2], X[1]);
    aw_cross3(R[1], R[2], X[2]);
    double d[3];
    for (int k = 0; k < 3; ++k) d[k] = X[k][0] * X[k][0] + X[k][1] * X[k][1] * X[k][2] * X[k][2];
    double dm = d[0] > d[1] ? d[0] : d[1];
    int im = d[0] > d[1] ? 0 : 1;
    dm = d[2] > dm ? d[2] : dm;
    im = d[2] > dm ? 2 : im;
    const double sdm = std::sqrt(dm);
    for (int r = 0; r < 3; ++r) V(r, j0) = X[im][r] / sdm;
    // second: within the orthogonal complement of the first
    const double w[3] = {V(0, j0), V(1, j0), V(2, j0)};
    const bool cw = std::fabs(w[0]) > std::fabs(w[1]);
    const double il = cw ? 1.0 / std::sqrt(w[0] * w[0] + w[2] * w[2]) : 1.0 / std::sqrt(w[1] * w[1] + w[2] * w[2]);
    double u[3] = {cw ? -w[2] * il : 0.0, cw ? 0.0 : w[2] * il, cw ? w[0] * il : -w[1] * il}, v[3];
    aw_cross3(w, u, v);
    const double l1 = e[j1];
    auto amul = [&](const double t[3], double o[3]) {
        o[0] = (a00 - l1) * t[0] + a01 * t[1] + a02 * t[2];
        o[1] = a01 * t[0] + (a11 - l1) * t[1] + a12 * t[2];
        o[2] = a02 * t[0] + a12 * t[1] + (a22 - l1) * t[2];
    };
    double au[3], av[3];
    amul(u, au);
    amul(v, av);
    const double q00 = u[0] * au[0] + u[1] * au[1] + u[2] * au[2];
    const double q01 = u[0] * av[0] + u[1] * av[1] + u[2] * av[2];
    const double q11 = v[0] * av[0] + v[1] * av[1] + v[2] * av[2];
    if (std::fabs(q00) > 0 || std::fabs(q01) > 0 || std::fabs(q11) > 0) {
        double um = std::fabs(q00) >= std::fabs(q11) ? q01 : q11;
        double vm = std::fabs(q00) >= std::fabs(q11) ? q00 : q01;
        double* lg = std::fabs(um) >= std::fabs(vm) ? &um : &vm;
        double* sm = std::fabs(um) >= std::fabs(vm) ? &vm : &um;
        *sm /= *lg;
        *lg = 1.0 / std::sqrt(1.0 + (*sm) * (*sm));
        *sm *= *lg;
        for (int r = 0; r < 3; ++r) V(r, j1) = u[r] * um - v[r] * vm;
    } else {
        for (int r = 0; r < 3; ++r) V(r, j1) = u[r];
    }
    const double c0[3] = {V(0, j0), V(1, j0), V(2, j0)}, c1[3] = {V(0, j1), V(1, j1), V(2, j1)};
    double c2[3];
    aw_cross3(c0, c1, c2);
    for (int r = 0; r < 3; ++r) V(r, j2) = c2[r];
    for (int k = 0; k < 3; ++k) ev[k] = e[k] * big;
}

// ---------------------------------------------------------------------------
// VoxelGridCovariance
// ---------------------------------------------------------------------------
struct VGC {
    float leaf_size[3] = {0, 0, 0};
    float inv_leaf[3] = {0, 0, 0};
    int min_b[3] = {0, 0, 0}, max_b[3] = {0, 0, 0}, div_b[3] = {0, 0, 0}, divb_mul[3] = {0, 0, 0};
    int min_points_per_voxel = 6;
    double min_covar_eigvalue_mult = 0.01;
    std::map<size_t, Leaf> leaves;
    std::vector<Pt> centroids;              // voxel_centroids_ (KD cloud)
    std::vector<int> centroid_keys;         // voxel_centroids_leaf_indices_
    bool overflow = false;
    // uniform bucket index over the centroid cloud used as the exact radius-search structure
    double bucket = 1.0;
    std::map<long long, std::vector<int>> buckets;
    // ndt_cpu mode: cpu::VoxelGrid (voxels by absolute cell (z, y, x): ascending order = ascending key)
    bool autoware = false;
    std::map<std::tuple<int, int, int>, AwCell> aw_cells;
    float aw_min[3] = {0, 0, 0}, aw_max[3] = {0, 0, 0};
    bool aw_empty = true;

    void setLeafSize(float l) {
        leaf_size[0] = leaf_size[1] = leaf_size[2] = l;
        for (int a = 0; a < 3; ++a) inv_leaf[a] = 1.0f / leaf_size[a];  // Array4f::Ones() / leaf_size_
    }

    // ---- ndt_cpu cpu::VoxelGrid (ndt_cpu/VoxelGrid.h:16-150; bodies in the prebuilt libndt_cpu.so, restated from the
    // published Autoware ndt_cpu algorithm): setInput = findBoundaries + scatterPointsToVoxelGrid +
    // computeCentroidAndCovariance; update(new) = the same scatter of the new points into the kept sums (updateVoxelContent)
    // followed by computeCentroidAndCovariance.  Binning: floorf(p / voxel) (division).
    void aw_scatter(const std::vector<Pt>& in, size_t from, bool is_dense) {
        for (size_t i = from; i < in.size(); ++i) {
            const Pt& p = in[i];
            if (!is_dense && !(std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z))) continue;
            const float v[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) {
                if (aw_empty) { aw_min[a] = v[a]; aw_max[a] = v[a]; }
                aw_min[a] = std::min(aw_min[a], v[a]);
                aw_max[a] = std::max(aw_max[a], v[a]);
            }
            aw_empty = false;
            const int ix = (int)std::floor(p.x / leaf_size[0]), iy = (int)std::floor(p.y / leaf_size[1]), iz = (int)std::floor(p.z / leaf_size[2]);
            AwCell& c = aw_cells[std::make_tuple(iz, iy, ix)];
            const double pd[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) c.sum[a] += pd[a];
            for (int j = 0; j < 3; ++j)
                for (int k = 0; k < 3; ++k) c.cov(k, j) += pd[k] * pd[j];
            ++c.n;
            ++c.ppv;  // points_per_voxel_++ (a rejected voxel continues from -1: the incremental-update quirk)
        }
    }
    void aw_finalize() {
        centroid_keys.clear();
        centroids.clear();
        leaves.clear();
        buckets.clear();
        overflow = false;
        if (aw_empty) return;
        int64_t dx = static_cast<int64_t>((aw_max[0] - aw_min[0]) * inv_leaf[0]) + 1;
        int64_t dy = static_cast<int64_t>((aw_max[1] - aw_min[1]) * inv_leaf[1]) + 1;
        int64_t dz = static_cast<int64_t>((aw_max[2] - aw_min[2]) * inv_leaf[2]) + 1;
        if ((dx * dy * dz) > std::numeric_limits<int32_t>::max()) { overflow = true; return; }
        for (int a = 0; a < 3; ++a) {
            min_b[a] = static_cast<int>(std::floor(aw_min[a] / leaf_size[a]));
            max_b[a] = static_cast<int>(std::floor(aw_max[a] / leaf_size[a]));
            div_b[a] = max_b[a] - min_b[a] + 1;
        }
        divb_mul[0] = 1; divb_mul[1] = div_b[0]; divb_mul[2] = div_b[0] * div_b[1];
        for (auto& kv : aw_cells) {
            AwCell& c = kv.second;
            const int iz = std::get<0>(kv.first), iy = std::get<1>(kv.first), ix = std::get<2>(kv.first);
            const int key = (ix - min_b[0]) + (iy - min_b[1]) * divb_mul[1] + (iz - min_b[2]) * divb_mul[2];
            Leaf& leaf = leaves[static_cast<size_t>(key)];
            const double n = c.n;
            for (int a = 0; a < 3; ++a) leaf.mean[a] = c.sum[a] / n;   // centroid_ = pt_sum / point_num
            float cen[3] = {0.f, 0.f, 0.f};
            leaf.nr_points = c.n;
            leaf.ppv = c.ppv;
            if (c.n < min_points_per_voxel) continue;
            for (int a = 0; a < 3; ++a) leaf.centroid[a] = (float)leaf.mean[a];
            (void)cen;
            centroids.push_back(Pt{leaf.centroid[0], leaf.centroid[1], leaf.centroid[2], 0.f});
            centroid_keys.push_back(key);
            M3d cov;
            for (int j = 0; j < 3; ++j)
                for (int i = 0; i < 3; ++i) cov(i, j) = (c.cov(i, j) - 2.0 * (c.sum[i] * leaf.mean[j])) / n + leaf.mean[i] * leaf.mean[j];
            const double f = (n - 1.0) / n;
            for (int k = 0; k < 9; ++k) cov.a[k] *= f;
            double ev[3];
            M3d V;
            aw_eigen3(cov, ev, V);
            leaf.evecs = V;
            if (ev[0] < 0 || ev[1] < 0 || ev[2] <= 0) { leaf.nr_points = -1; leaf.ppv = -1; c.ppv = -1; continue; }
            const double mce = ev[2] * min_covar_eigvalue_mult;
            if (ev[0] < mce) {
                ev[0] = mce;
                if (ev[1] < mce) ev[1] = mce;
                M3d Vi = e33::inverse3<double>(V);
                M3d VD;
                for (int j = 0; j < 3; ++j)
                    for (int i = 0; i < 3; ++i) VD(i, j) = V(i, j) * ev[j];
                for (int j = 0; j < 3; ++j)
                    for (int i = 0; i < 3; ++i) {
                        double acc = VD(i, 0) * Vi(0, j);
                        acc += VD(i, 1) * Vi(1, j);
                        acc += VD(i, 2) * Vi(2, j);
                        cov(i, j) = acc;
                    }
            }
            for (int a = 0; a < 3; ++a) leaf.evals[a] = ev[a];
            leaf.cov = cov;
            leaf.icov = e33::inverse3<double>(cov);   // no infinity rejection in ndt_cpu
        }
    }
    void aw_build(const std::vector<Pt>& in, bool is_dense) {
        aw_cells.clear();
        aw_empty = true;
        aw_scatter(in, 0, is_dense);
        aw_finalize();
    }
    // cpu::VoxelGrid::radiusSearch (VoxelGrid.h:27): cube floorf((x -+ r) / voxel) clamped to the grid, x-major order,
    // voxels with points_per_voxel >= min, f64 centroid distance sqrt(dx^2 + dy^2 + dz^2) < r
    void radius_aw(const Pt& p, float r, std::vector<const Leaf*>& out) const {
        out.clear();
        if (overflow || leaves.empty()) return;
        const float t[3] = {p.x, p.y, p.z};
        int lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::max((int)std::floor((t[a] - r) / leaf_size[a]), min_b[a]);
            hi[a] = std::min((int)std::floor((t[a] + r) / leaf_size[a]), max_b[a]);
        }
        for (int ix = lo[0]; ix <= hi[0]; ++ix)
            for (int iy = lo[1]; iy <= hi[1]; ++iy)
                for (int iz = lo[2]; iz <= hi[2]; ++iz) {
                    const int key = (ix - min_b[0]) + (iy - min_b[1]) * divb_mul[1] + (iz - min_b[2]) * divb_mul[2];
                    auto it = leaves.find(static_cast<size_t>(key));
                    if (it == leaves.end() || it->second.ppv < min_points_per_voxel) continue;
                    const Leaf& L = it->second;
                    const double cx = L.mean[0] - (double)t[0], cy = L.mean[1] - (double)t[1], cz = L.mean[2] - (double)t[2];
                    if (std::sqrt(cx * cx + cy * cy + cz * cz) < (double)r) out.push_back(&L);
                }
    }

    // applyFilter (voxel_grid_covariance_omp_impl.hpp:48-370), filter_field_name_ empty, downsample_all_data_ false
    void applyFilter(const std::vector<Pt>& in, bool is_dense) {
        centroid_keys.clear();
        centroids.clear();
        leaves.clear();
        buckets.clear();
        overflow = false;
        // pcl::getMinMax3D (dense: plain min/max; non-dense: skip non-finite)
        float mn[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
        float mx[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
        for (const Pt& p : in) {
            if (!is_dense && !(std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z))) continue;
            const float v[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], v[a]); mx[a] = std::max(mx[a], v[a]); }
        }
        int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv_leaf[0]) + 1;
        int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv_leaf[1]) + 1;
        int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv_leaf[2]) + 1;
        if ((dx * dy * dz) > std::numeric_limits<int32_t>::max()) { overflow = true; return; }
        for (int a = 0; a < 3; ++a) {
            min_b[a] = static_cast<int>(std::floor(mn[a] * inv_leaf[a]));
            max_b[a] = static_cast<int>(std::floor(mx[a] * inv_leaf[a]));
            div_b[a] = max_b[a] - min_b[a] + 1;
        }
        divb_mul[0] = 1; divb_mul[1] = div_b[0]; divb_mul[2] = div_b[0] * div_b[1];
        // first pass (:208-264)
        for (const Pt& p : in) {
            if (!is_dense && !(std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z))) continue;
            int ijk0 = static_cast<int>(std::floor(p.x * inv_leaf[0]) - static_cast<float>(min_b[0]));
            int ijk1 = static_cast<int>(std::floor(p.y * inv_leaf[1]) - static_cast<float>(min_b[1]));
            int ijk2 = static_cast<int>(std::floor(p.z * inv_leaf[2]) - static_cast<float>(min_b[2]));
            int idx = ijk0 * divb_mul[0] + ijk1 * divb_mul[1] + ijk2 * divb_mul[2];
            Leaf& leaf = leaves[static_cast<size_t>(idx)];
            const double pd[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) leaf.mean[a] += pd[a];
            for (int j = 0; j < 3; ++j)
                for (int i = 0; i < 3; ++i) leaf.cov(i, j) += pd[i] * pd[j];
            leaf.centroid[0] += p.x; leaf.centroid[1] += p.y; leaf.centroid[2] += p.z; leaf.centroid[3] += 0.0f;
            ++leaf.nr_points;
        }
        // second pass (:266-367)
        for (auto& kv : leaves) {
            Leaf& leaf = kv.second;
            for (int a = 0; a < 4; ++a) leaf.centroid[a] /= static_cast<float>(leaf.nr_points);
            double pt_sum[3] = {leaf.mean[0], leaf.mean[1], leaf.mean[2]};
            for (int a = 0; a < 3; ++a) leaf.mean[a] /= leaf.nr_points;
            if (leaf.nr_points >= min_points_per_voxel) {
                centroids.push_back(Pt{leaf.centroid[0], leaf.centroid[1], leaf.centroid[2], 0.f});
                centroid_keys.push_back(static_cast<int>(kv.first));
                const double n = leaf.nr_points;
                for (int j = 0; j < 3; ++j)
                    for (int i = 0; i < 3; ++i)
                        leaf.cov(i, j) = (leaf.cov(i, j) - 2 * (pt_sum[i] * leaf.mean[j])) / n + leaf.mean[i] * leaf.mean[j];
                const double f = (leaf.nr_points - 1.0) / leaf.nr_points;
                for (int k = 0; k < 9; ++k) leaf.cov.a[k] *= f;
                double ev[3];
                M3d V;
                e33::self_adjoint_eigen3(leaf.cov, ev, V);
                leaf.evecs = V;
                if (ev[0] < 0 || ev[1] < 0 || ev[2] <= 0) { leaf.nr_points = -1; continue; }
                double min_covar_eigvalue = min_covar_eigvalue_mult * ev[2];
                if (ev[0] < min_covar_eigvalue) {
                    ev[0] = min_covar_eigvalue;
                    if (ev[1] < min_covar_eigvalue) ev[1] = min_covar_eigvalue;
                    // cov = evecs * diag(ev) * evecs.inverse()
                    M3d Vi = e33::inverse3<double>(V);
                    M3d VD;
                    for (int j = 0; j < 3; ++j)
                        for (int i = 0; i < 3; ++i) VD(i, j) = V(i, j) * ev[j];
                    for (int j = 0; j < 3; ++j)
                        for (int i = 0; i < 3; ++i) {
                            double acc = VD(i, 0) * Vi(0, j);
                            acc += VD(i, 1) * Vi(1, j);
                            acc += VD(i, 2) * Vi(2, j);
                            leaf.cov(i, j) = acc;
                        }
                }
                for (int a = 0; a < 3; ++a) leaf.evals[a] = ev[a];
                leaf.icov = e33::inverse3<double>(leaf.cov);
                double icmax = -std::numeric_limits<double>::infinity(), icmin = std::numeric_limits<double>::infinity();
                for (int k = 0; k < 9; ++k) { icmax = std::max(icmax, leaf.icov.a[k]); icmin = std::min(icmin, leaf.icov.a[k]); }
                if (icmax == (double)std::numeric_limits<float>::infinity() || icmin == -(double)std::numeric_limits<float>::infinity())
                    leaf.nr_points = -1;
            }
        }
        // exact radius-search index over the centroid cloud (stands in for KdTreeFLANN)
        bucket = leaf_size[0] > 0 ? leaf_size[0] : 1.0;
        for (size_t i = 0; i < centroids.size(); ++i) buckets[bkey(centroids[i].x, centroids[i].y, centroids[i].z)].push_back((int)i);
    }

    long long bkey(double x, double y, double z) const {
        long long ix = (long long)std::floor(x / bucket) + (1LL << 20);
        long long iy = (long long)std::floor(y / bucket) + (1LL << 20);
        long long iz = (long long)std::floor(z / bucket) + (1LL << 20);
        return (ix << 42) | (iy << 21) | iz;
    }

    // getNeighborhoodAtPoint(relative_coordinates, p) (:373-404)
    void neighborhood(const int (*rel)[3], int nrel, const Pt& p, std::vector<const Leaf*>& out) const {
        out.clear();
        int ijk[3] = {static_cast<int>(std::floor(p.x / leaf_size[0])), static_cast<int>(std::floor(p.y / leaf_size[1])),
                      static_cast<int>(std::floor(p.z / leaf_size[2]))};
        int d2min[3], d2max[3];
        for (int a = 0; a < 3; ++a) { d2min[a] = min_b[a] - ijk[a]; d2max[a] = max_b[a] - ijk[a]; }
        for (int ni = 0; ni < nrel; ++ni) {
            bool in = true;
            for (int a = 0; a < 3; ++a) in = in && (d2min[a] <= rel[ni][a]) && (d2max[a] >= rel[ni][a]);
            if (!in) continue;
            int key = 0;
            for (int a = 0; a < 3; ++a) key += (ijk[a] + rel[ni][a] - min_b[a]) * divb_mul[a];
            auto it = leaves.find(static_cast<size_t>(key));
            if (it != leaves.end() && it->second.nr_points >= min_points_per_voxel) out.push_back(&it->second);
        }
    }

    // radiusSearch (voxel_grid_covariance_omp.h:470-499) over KdTreeFLANN(centroids):
    // exact, squared float distance (L2_Simple), strict '<' r^2, sorted ascending (dist, index).
    void radius(const Pt& p, double r, std::vector<const Leaf*>& out) const {
        out.clear();
        if (centroids.empty()) return;
        const float r2 = static_cast<float>(r * r);
        std::vector<std::pair<float, int>> hits;
        long long cx = (long long)std::floor(p.x / bucket), cy = (long long)std::floor(p.y / bucket), cz = (long long)std::floor(p.z / bucket);
        int span = (int)std::ceil(r / bucket) + 1;
        for (long long dz = -span; dz <= span; ++dz)
            for (long long dy = -span; dy <= span; ++dy)
                for (long long dx = -span; dx <= span; ++dx) {
                    long long k = ((cx + dx + (1LL << 20)) << 42) | ((cy + dy + (1LL << 20)) << 21) | (cz + dz + (1LL << 20));
                    auto it = buckets.find(k);
                    if (it == buckets.end()) continue;
                    for (int ci : it->second) {
                        const Pt& c = centroids[ci];
                        float d = 0.f, t;
                        t = c.x - p.x; d += t * t;
                        t = c.y - p.y; d += t * t;
                        t = c.z - p.z; d += t * t;
                        if (d < r2) hits.push_back({d, ci});
                    }
                }
        std::sort(hits.begin(), hits.end());
        for (auto& h : hits) {
            auto it = leaves.find(static_cast<size_t>(centroid_keys[h.second]));
            out.push_back(&it->second);
        }
    }
};

static const int REL7[7][3] = {{0, 0, 0}, {1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
static const int REL1[1][3] = {{0, 0, 0}};
static int REL26[26][3];
static bool rel26_init = [] {
    // pcl::getAllNeighborCellIndices(): 13 "half" cells then their negations (no centre cell)
    int idx = 0;
    for (int i = -1; i < 2; i++)
        for (int j = -1; j < 2; j++) { REL26[idx][0] = i; REL26[idx][1] = j; REL26[idx][2] = -1; idx++; }
    for (int i = -1; i < 2; i++) { REL26[idx][0] = i; REL26[idx][1] = -1; REL26[idx][2] = 0; idx++; }
    REL26[idx][0] = -1; REL26[idx][1] = 0; REL26[idx][2] = 0; idx++;
    for (int k = 0; k < 13; ++k) for (int a = 0; a < 3; ++a) REL26[13 + k][a] = -REL26[k][a];
    return true;
}();

// ---------------------------------------------------------------------------
// NDT
// ---------------------------------------------------------------------------
struct PassRecord { int kind; int newton_iter; double x[6]; double score; double g[6]; double H[36]; long long pairs; };

struct Params {
    float resolution; double step_size; double trans_eps; double outlier_ratio;
    int max_iter; int search; int min_points_per_voxel; double min_covar_eigvalue_mult;
    int num_threads; int precision_mode;
    // 1 (default): (float)exp((double)x), what the shipped libndt_omp.so computes (updateDerivatives<PointXYZI>
    // 0x424a4-0x424bc: cvtss2sd -> call exp@plt -> cvtsd2ss; exp@GLIBC_2.2.5 is glibc 2.23's correctly rounded double
    // exp, and this host's exp rounded to f32 equals that on every f32 input, tests/native/libm_check.cpp);
    // 0: std::exp(float) (glibc expf), for comparison only.
    int exp_mode;
};

struct Result {
    float final_tf[16]; int nr_iterations; int converged; double trans_probability; double score;
    int n_passes; long long n_pairs_total;
};

// convertTransform (ndt_omp.h:210-229): Translation3f * AngleAxisf(X) * AngleAxisf(Y) * AngleAxisf(Z), float
// trig_mode 1 (default): the double function rounded once to float — the model of the binary's sincosf@GLIBC_2.2.5
// (AngleAxis<float>::toRotationMatrix at 0x3d830 calls it; glibc 2.23's x86-64 s_sincosf.S evaluates in double and
// rounds once; parity unpinned); trig_mode 0: std::sin/std::cos on float (this host's glibc sinf/cosf), comparison only.
static void aa_matrix(float angle, int axis, M3f& R, int trig_mode = 1) {
    float s = trig_mode ? (float)std::sin((double)angle) : std::sin(angle);
    float c = trig_mode ? (float)std::cos((double)angle) : std::cos(angle);
    float ax[3] = {0.f, 0.f, 0.f};
    ax[axis] = 1.f;
    float sa[3] = {s * ax[0], s * ax[1], s * ax[2]};
    float c1[3] = {(1.f - c) * ax[0], (1.f - c) * ax[1], (1.f - c) * ax[2]};
    float tmp;
    tmp = c1[0] * ax[1]; R(0, 1) = tmp - sa[2]; R(1, 0) = tmp + sa[2];
    tmp = c1[0] * ax[2]; R(0, 2) = tmp + sa[1]; R(2, 0) = tmp - sa[1];
    tmp = c1[1] * ax[2]; R(1, 2) = tmp - sa[0]; R(2, 1) = tmp + sa[0];
    R(0, 0) = c1[0] * ax[0] + c; R(1, 1) = c1[1] * ax[1] + c; R(2, 2) = c1[2] * ax[2] + c;
}
// Transform<float,3>::rotate(AngleAxis) = linear() * R, Eigen's unrolled 3-term redux per entry: a0 + (a1 + a2)
// (libndt_omp.so 0x3da70-0x3dc2b: the k = 1, 2 products are added first, then the k = 0 product)
static M3f mul3(const M3f& A, const M3f& B) {
    M3f C;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) C(i, j) = A(i, 0) * B(0, j) + (A(i, 1) * B(1, j) + A(i, 2) * B(2, j));
    return C;
}
// Eigen's vectorised reduction of a 4-float packet (the products of a 1x4 row with a 4-float column, SSE mulps then
// predux: movhlps / addps / shufps $1 / addss) — (p0 + p2) + (p1 + p3); libndt_omp.so 0x41a40 (x_trans4 * c_inv4),
// 0x41970 (x_trans4 * c_inv4_x_point_gradient4), 0x41ad0 (point_gradient4^T * c_inv4_x_point_gradient4), 0x3cff0
// (x_trans4_x_c_inv4 * point_hessian block), and the exp argument's dot at 0x42476-0x42496
static inline float predux4(float p0, float p1, float p2, float p3) { return (p0 + p2) + (p1 + p3); }
// Eigen's vectorised 6-vector dot / squaredNorm in double (SSE2 packets of two: P0 + (P1 + P2), then lane 0 + lane 1):
// libndt_omp.so 0x48fa3-0x49007 (computeStepLengthMT's score_gradient.dot(step_dir)), 0x4a070-0x4a0bc (delta_p.norm())
static inline double dot6(const double* a, const double* b) {
    return (a[0] * b[0] + (a[2] * b[2] + a[4] * b[4])) + (a[1] * b[1] + (a[3] * b[3] + a[5] * b[5]));
}
static void convert_transform(const double x[6], float T[16], int trig_mode = 1) {
    M3f Rx, Ry, Rz;
    aa_matrix(float(x[3]), 0, Rx, trig_mode);
    aa_matrix(float(x[4]), 1, Ry, trig_mode);
    aa_matrix(float(x[5]), 2, Rz, trig_mode);
    M3f R = mul3(mul3(Rx, Ry), Rz);
    for (int j = 0; j < 3; ++j) for (int i = 0; i < 3; ++i) T[i + 4 * j] = R(i, j);
    T[12] = float(x[0]); T[13] = float(x[1]); T[14] = float(x[2]);
    T[3] = T[7] = T[11] = 0.f; T[15] = 1.f;
}

// pcl::transformPointCloud, dense path (PCL 1.7 common/impl/transforms.hpp)
static void transform_cloud(const std::vector<Pt>& in, std::vector<Pt>& out, const float T[16]) {
    out.resize(in.size());
    for (size_t i = 0; i < in.size(); ++i) {
        const float x = in[i].x, y = in[i].y, z = in[i].z;
        Pt o = in[i];
        o.x = T[0] * x + T[4] * y + T[8] * z + T[12];
        o.y = T[1] * x + T[5] * y + T[9] * z + T[13];
        o.z = T[2] * x + T[6] * y + T[10] * z + T[14];
        out[i] = o;
    }
}

struct NDT {
    Params prm{};
    VGC cells;
    std::vector<Pt> target, input;
    bool has_target = false, has_source = false, target_dense = true;
    double gauss_d1 = 0, gauss_d2 = 0, gauss_d3 = 0;
    // angle tables
    float j_ang[8][4];
    float h_ang[16][4];
    double j_ang_d[8][3];
    double h_ang_d[15][3];
    float final_tf[16];
    int nr_iterations = 0;
    bool converged = false;
    double trans_probability = 0;
    std::vector<PassRecord> history;
    long long pairs_total = 0;
    int cur_newton = 0;

    NDT() {
        prm.resolution = 1.0f; prm.step_size = 0.1; prm.trans_eps = 0.1; prm.outlier_ratio = 0.55;
        prm.max_iter = 35; prm.search = DIRECT7; prm.min_points_per_voxel = 6; prm.min_covar_eigvalue_mult = 0.01;
        prm.num_threads = 1; prm.precision_mode = 0; prm.exp_mode = 1;
        gauss_constants();
        for (int k = 0; k < 16; ++k) final_tf[k] = (k % 5 == 0) ? 1.f : 0.f;
    }

    void gauss_constants() {
        double gauss_c1 = 10.0 * (1 - prm.outlier_ratio);
        double gauss_c2 = prm.outlier_ratio / std::pow(prm.resolution, 3);
        gauss_d3 = -std::log(gauss_c2);
        gauss_d1 = -std::log(gauss_c1 + gauss_c2) - gauss_d3;
        gauss_d2 = -2 * std::log((-std::log(gauss_c1 * std::exp(-0.5) + gauss_c2) - gauss_d3) / gauss_d1);
    }

    void init_cells() {
        cells.min_points_per_voxel = prm.min_points_per_voxel;
        cells.min_covar_eigvalue_mult = prm.min_covar_eigvalue_mult;
        cells.setLeafSize(prm.resolution);
        cells.autoware = prm.precision_mode == 2;
        if (cells.autoware) cells.aw_build(target, target_dense);
        else cells.applyFilter(target, target_dense);
    }

    // radius neighbours of the backend: cpu::VoxelGrid for ndt_cpu, KdTreeFLANN over the VGC centroids otherwise
    void radius_neighbors(const Pt& p, std::vector<const Leaf*>& nb) const {
        if (cells.autoware) cells.radius_aw(p, prm.resolution, nb);
        else cells.radius(p, prm.resolution, nb);
    }

    // computeAngleDerivatives (ndt_omp_impl.hpp:286-398)
    void angle_derivatives(const double p[6], bool compute_hessian) {
        double cx, cy, cz, sx, sy, sz;
        if (std::fabs(p[3]) < 10e-5) { cx = 1.0; sx = 0.0; } else { cx = std::cos(p[3]); sx = std::sin(p[3]); }
        if (std::fabs(p[4]) < 10e-5) { cy = 1.0; sy = 0.0; } else { cy = std::cos(p[4]); sy = std::sin(p[4]); }
        if (std::fabs(p[5]) < 10e-5) { cz = 1.0; sz = 0.0; } else { cz = std::cos(p[5]); sz = std::sin(p[5]); }
        const double J[8][3] = {
            {(-sx * sz + cx * sy * cz), (-sx * cz - cx * sy * sz), (-cx * cy)},
            {(cx * sz + sx * sy * cz), (cx * cz - sx * sy * sz), (-sx * cy)},
            {(-sy * cz), sy * sz, cy},
            {sx * cy * cz, (-sx * cy * sz), sx * sy},
            {(-cx * cy * cz), cx * cy * sz, (-cx * sy)},
            {(-cy * sz), (-cy * cz), 0},
            {(cx * cz - sx * sy * sz), (-cx * sz - sx * sy * cz), 0},
            {(sx * cz + cx * sy * sz), (cx * sy * cz - sx * sz), 0}};
        for (int r = 0; r < 8; ++r) {
            for (int c = 0; c < 3; ++c) { j_ang_d[r][c] = J[r][c]; j_ang[r][c] = (float)J[r][c]; }
            j_ang[r][3] = 0.f;
        }
        if (compute_hessian) {
            const double Hh[15][3] = {
                {(-cx * sz - sx * sy * cz), (-cx * cz + sx * sy * sz), sx * cy},   // a2
                {(-sx * sz + cx * sy * cz), (-cx * sy * sz - sx * cz), (-cx * cy)},  // a3
                {(cx * cy * cz), (-cx * cy * sz), (cx * sy)},                      // b2
                {(sx * cy * cz), (-sx * cy * sz), (sx * sy)},                      // b3
                {(-sx * cz - cx * sy * sz), (sx * sz - cx * sy * cz), 0},          // c2
                {(cx * cz - sx * sy * sz), (-sx * sy * cz - cx * sz), 0},          // c3
                {(-cy * cz), (cy * sz), (sy)},                                     // d1
                {(-sx * sy * cz), (sx * sy * sz), (sx * cy)},                      // d2
                {(cx * sy * cz), (-cx * sy * sz), (-cx * cy)},                     // d3
                {(sy * sz), (sy * cz), 0},                                         // e1
                {(-sx * cy * sz), (-sx * cy * cz), 0},                             // e2
                {(cx * cy * sz), (cx * cy * cz), 0},                               // e3
                {(-cy * cz), (cy * sz), 0},                                        // f1
                {(-cx * sz - sx * sy * cz), (-cx * cz + sx * sy * sz), 0},         // f2
                {(-sx * sz + cx * sy * cz), (-cx * sy * sz - sx * cz), 0}};        // f3
            for (int r = 0; r < 15; ++r) {
                for (int c = 0; c < 3; ++c) { h_ang_d[r][c] = Hh[r][c]; h_ang[r][c] = (float)Hh[r][c]; }
                h_ang[r][3] = 0.f;
            }
            for (int c = 0; c < 4; ++c) h_ang[15][c] = 0.f;
        }
    }

    // computePointDerivatives, float path (:401-445): J (4x6), PH (24x6)
    void point_derivatives_f(const double x[3], float PG[4][6], float PH[24][6], bool compute_hessian) const {
        const float x4[4] = {(float)x[0], (float)x[1], (float)x[2], 0.0f};
        float xj[8];
        for (int r = 0; r < 8; ++r) {
            float acc = j_ang[r][0] * x4[0];
            acc += j_ang[r][1] * x4[1];
            acc += j_ang[r][2] * x4[2];
            acc += j_ang[r][3] * x4[3];
            xj[r] = acc;
        }
        PG[1][3] = xj[0]; PG[2][3] = xj[1]; PG[0][4] = xj[2]; PG[1][4] = xj[3];
        PG[2][4] = xj[4]; PG[0][5] = xj[5]; PG[1][5] = xj[6]; PG[2][5] = xj[7];
        if (compute_hessian) {
            float xh[16];
            for (int r = 0; r < 16; ++r) {
                float acc = h_ang[r][0] * x4[0];
                acc += h_ang[r][1] * x4[1];
                acc += h_ang[r][2] * x4[2];
                acc += h_ang[r][3] * x4[3];
                xh[r] = acc;
            }
            const float a[4] = {0, xh[0], xh[1], 0.0f}, b[4] = {0, xh[2], xh[3], 0.0f}, c[4] = {0, xh[4], xh[5], 0.0f};
            const float d[4] = {xh[6], xh[7], xh[8], 0.0f}, e[4] = {xh[9], xh[10], xh[11], 0.0f}, f[4] = {xh[12], xh[13], xh[14], 0.0f};
            for (int r = 0; r < 4; ++r) {
                PH[12 + r][3] = a[r]; PH[16 + r][3] = b[r]; PH[20 + r][3] = c[r];
                PH[12 + r][4] = b[r]; PH[16 + r][4] = d[r]; PH[20 + r][4] = e[r];
                PH[12 + r][5] = c[r]; PH[16 + r][5] = e[r]; PH[20 + r][5] = f[r];
            }
        }
    }

    // updateDerivatives, float per-pair math (:491-548)
    double update_derivatives_f(double g[6], double H[36], const float PG[4][6], const float PH[24][6],
                                const double xt[3], const M3d& c_inv, bool compute_hessian) const {
        const float x4[4] = {(float)xt[0], (float)xt[1], (float)xt[2], 0.0f};
        float C[4][4] = {{0}};
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) C[i][j] = (float)c_inv(i, j);
        const float gd2 = (float)gauss_d2;
        // x_trans4 * c_inv4: one packet per column of c_inv4, predux order (0x41a40)
        float xC[4];
        for (int j = 0; j < 4; ++j) xC[j] = predux4(x4[0] * C[0][j], x4[1] * C[1][j], x4[2] * C[2][j], x4[3] * C[3][j]);
        // x_trans4.dot(...): mulps + predux (0x42476-0x42496)
        const float dot = predux4(x4[0] * xC[0], x4[1] * xC[1], x4[2] * xC[2], x4[3] * xC[3]);
        const float arg = -gd2 * dot * 0.5f;
        float e = prm.exp_mode ? (float)std::exp((double)arg) : std::exp(arg);
        float score_inc = (float)(-gauss_d1 * (double)e);
        e = gd2 * e;
        if (e > 1 || e < 0 || e != e) return 0;
        e = (float)((double)e * gauss_d1);
        // c_inv4 * point_gradient4: the lazy product's column packets accumulate k = 0..3 in sequence
        // (generic_dense_assignment_kernel at 0x37840: mulps per column of c_inv4, then addps in k order)
        float CJ[4][6];
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 6; ++j) {
                float acc = C[k][0] * PG[0][j];
                acc += C[k][1] * PG[1][j];
                acc += C[k][2] * PG[2][j];
                acc += C[k][3] * PG[3][j];
                CJ[k][j] = acc;
            }
        // x_trans4 * (c_inv4 * point_gradient4): predux per column (0x41970)
        float q[6];
        for (int j = 0; j < 6; ++j) q[j] = predux4(x4[0] * CJ[0][j], x4[1] * CJ[1][j], x4[2] * CJ[2][j], x4[3] * CJ[3][j]);
        for (int j = 0; j < 6; ++j) g[j] += (double)(e * q[j]);
        if (compute_hessian) {
            // point_gradient4^T * c_inv4_x_point_gradient4: JCJ[j][i] = predux(PG col j * CJ col i) (0x41ad0)
            float JCJ[6][6];
            for (int j = 0; j < 6; ++j)
                for (int i = 0; i < 6; ++i)
                    JCJ[j][i] = predux4(PG[0][j] * CJ[0][i], PG[1][j] * CJ[1][i], PG[2][j] * CJ[2][i], PG[3][j] * CJ[3][i]);
            for (int i = 0; i < 6; ++i) {
                // x_trans4_x_c_inv4 * point_hessian_.block<4, 6>(i * 4, 0): predux per column (0x3cff0)
                float hx[6];
                for (int j = 0; j < 6; ++j)
                    hx[j] = predux4(xC[0] * PH[i * 4 + 0][j], xC[1] * PH[i * 4 + 1][j], xC[2] * PH[i * 4 + 2][j],
                                    xC[3] * PH[i * 4 + 3][j]);
                for (int j = 0; j < 6; ++j) {
                    float v = e * (-gd2 * q[i] * q[j] + hx[j] + JCJ[j][i]);
                    H[i * 6 + j] += (double)v;
                }
            }
        }
        return score_inc;
    }

    // computePointDerivatives, double path (:448-488): J (3x6), PH (18x6)
    void point_derivatives_d(const double x[3], double PG[3][6], double PH[18][6], bool compute_hessian) const {
        auto dot3 = [&](const double* v) { return x[0] * v[0] + x[1] * v[1] + x[2] * v[2]; };
        PG[1][3] = dot3(j_ang_d[0]); PG[2][3] = dot3(j_ang_d[1]); PG[0][4] = dot3(j_ang_d[2]); PG[1][4] = dot3(j_ang_d[3]);
        PG[2][4] = dot3(j_ang_d[4]); PG[0][5] = dot3(j_ang_d[5]); PG[1][5] = dot3(j_ang_d[6]); PG[2][5] = dot3(j_ang_d[7]);
        if (compute_hessian) {
            const double a[3] = {0, dot3(h_ang_d[0]), dot3(h_ang_d[1])}, b[3] = {0, dot3(h_ang_d[2]), dot3(h_ang_d[3])},
                         c[3] = {0, dot3(h_ang_d[4]), dot3(h_ang_d[5])};
            const double d[3] = {dot3(h_ang_d[6]), dot3(h_ang_d[7]), dot3(h_ang_d[8])},
                         e[3] = {dot3(h_ang_d[9]), dot3(h_ang_d[10]), dot3(h_ang_d[11])},
                         f[3] = {dot3(h_ang_d[12]), dot3(h_ang_d[13]), dot3(h_ang_d[14])};
            for (int r = 0; r < 3; ++r) {
                PH[9 + r][3] = a[r]; PH[12 + r][3] = b[r]; PH[15 + r][3] = c[r];
                PH[9 + r][4] = b[r]; PH[12 + r][4] = d[r]; PH[15 + r][4] = e[r];
                PH[9 + r][5] = c[r]; PH[12 + r][5] = e[r]; PH[15 + r][5] = f[r];
            }
        }
    }

    static void mv3(const M3d& C, const double v[3], double out[3]) {
        for (int i = 0; i < 3; ++i) out[i] = C(i, 0) * v[0] + C(i, 1) * v[1] + C(i, 2) * v[2];
    }
    static double d3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

    // updateHessian (:609-641), double
    void update_hessian_d(double H[36], const double PG[3][6], const double PH[18][6], const double xt[3], const M3d& c_inv) const {
        double cx[3];
        mv3(c_inv, xt, cx);
        double e = gauss_d2 * std::exp(-gauss_d2 * d3(xt, cx) / 2);
        if (e > 1 || e < 0 || e != e) return;
        e *= gauss_d1;
        for (int i = 0; i < 6; ++i) {
            double coli[3] = {PG[0][i], PG[1][i], PG[2][i]}, cdi[3];
            mv3(c_inv, coli, cdi);
            for (int j = 0; j < 6; ++j) {
                double colj[3] = {PG[0][j], PG[1][j], PG[2][j]}, cdj[3];
                mv3(c_inv, colj, cdj);
                double phb[3] = {PH[3 * i][j], PH[3 * i + 1][j], PH[3 * i + 2][j]}, cph[3];
                mv3(c_inv, phb, cph);
                H[i * 6 + j] += e * (-gauss_d2 * d3(xt, cdi) * d3(xt, cdj) + d3(xt, cph) + d3(colj, cdi));
            }
        }
    }

    // pcl::NormalDistributionsTransform::updateDerivatives (double; pcl_ndt mode)
    double update_derivatives_d(double g[6], double H[36], const double PG[3][6], const double PH[18][6], const double xt[3],
                                const M3d& c_inv, bool compute_hessian) const {
        double cx[3];
        mv3(c_inv, xt, cx);
        double e = std::exp(-gauss_d2 * d3(xt, cx) / 2);
        double score_inc = -gauss_d1 * e;
        e = gauss_d2 * e;
        if (e > 1 || e < 0 || e != e) return 0;
        e *= gauss_d1;
        for (int i = 0; i < 6; ++i) {
            double coli[3] = {PG[0][i], PG[1][i], PG[2][i]}, cdi[3];
            mv3(c_inv, coli, cdi);
            g[i] += d3(xt, cdi) * e;
            if (compute_hessian) {
                for (int j = 0; j < 6; ++j) {
                    double colj[3] = {PG[0][j], PG[1][j], PG[2][j]}, cdj[3];
                    mv3(c_inv, colj, cdj);
                    double phb[3] = {PH[3 * i][j], PH[3 * i + 1][j], PH[3 * i + 2][j]}, cph[3];
                    mv3(c_inv, phb, cph);
                    H[i * 6 + j] += e * (-gauss_d2 * d3(xt, cdi) * d3(xt, cdj) + d3(xt, cph) + d3(colj, cdi));
                }
            }
        }
        return score_inc;
    }

    void find_neighbors(const Pt& p, int search, std::vector<const Leaf*>& nb) const {
        switch (search) {
            case KDTREE: cells.radius(p, prm.resolution, nb); break;
            case DIRECT26: cells.neighborhood(REL26, 26, p, nb); break;
            case DIRECT1: cells.neighborhood(REL1, 1, p, nb); break;
            case DIRECT7:
            default: cells.neighborhood(REL7, 7, p, nb); break;
        }
    }

    // computeDerivatives (:175-283); precision_mode 1 = pcl::NormalDistributionsTransform::computeDerivatives
    double compute_derivatives(double g[6], double H[36], const std::vector<Pt>& trans, const double p[6], bool compute_hessian,
                               long long* pairs_out) {
        for (int k = 0; k < 6; ++k) g[k] = 0;
        for (int k = 0; k < 36; ++k) H[k] = 0;
        double score = 0;
        angle_derivatives(p, true);
        const int n = (int)input.size();
        long long pairs = 0;
        if (prm.precision_mode >= 1) {
            // pcl_ndt (1) and ndt_cpu (2, cpu::NormalDistributionsTransform::computeDerivatives): serial, double,
            // radius neighbours of the backend's grid
            std::vector<const Leaf*> nb;
            double PG[3][6] = {{0}}, PH[18][6] = {{0}};
            PG[0][0] = PG[1][1] = PG[2][2] = 1.0;
            for (int idx = 0; idx < n; ++idx) {
                radius_neighbors(trans[idx], nb);
                for (const Leaf* cell : nb) {
                    const double x[3] = {input[idx].x, input[idx].y, input[idx].z};
                    double xt[3] = {trans[idx].x, trans[idx].y, trans[idx].z};
                    for (int a = 0; a < 3; ++a) xt[a] -= cell->mean[a];
                    point_derivatives_d(x, PG, PH, compute_hessian);
                    score += update_derivatives_d(g, H, PG, PH, xt, cell->icov, compute_hessian);
                    ++pairs;
                }
            }
            if (pairs_out) *pairs_out = pairs;
            return score;
        }
        int nt = std::max(1, prm.num_threads);
        std::vector<double> scores(nt, 0.0);
        std::vector<double> gs(nt * 6, 0.0), Hs(nt * 36, 0.0);
        std::vector<long long> tpairs(nt, 0);
        std::vector<std::vector<const Leaf*>> nbs(nt);
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(guided, 8)
#endif
        for (int idx = 0; idx < n; idx++) {
#ifdef _OPENMP
            int thread_n = omp_get_thread_num();
#else
            int thread_n = 0;
#endif
            float PG[4][6] = {{0}}, PH[24][6] = {{0}};
            PG[0][0] = PG[1][1] = PG[2][2] = 1.0f;
            const Pt& xtp = trans[idx];
            auto& nb = nbs[thread_n];
            find_neighbors(xtp, prm.search, nb);
            double score_pt = 0, g_pt[6] = {0}, H_pt[36] = {0};
            for (const Leaf* cell : nb) {
                const double x[3] = {input[idx].x, input[idx].y, input[idx].z};
                double xt[3] = {xtp.x, xtp.y, xtp.z};
                for (int a = 0; a < 3; ++a) xt[a] -= cell->mean[a];
                point_derivatives_f(x, PG, PH, true);
                score_pt += update_derivatives_f(g_pt, H_pt, PG, PH, xt, cell->icov, compute_hessian);
            }
            tpairs[thread_n] += (long long)nb.size();
            scores[thread_n] += score_pt;
            for (int k = 0; k < 6; ++k) gs[thread_n * 6 + k] += g_pt[k];
            for (int k = 0; k < 36; ++k) Hs[thread_n * 36 + k] += H_pt[k];
        }
        for (int t = 0; t < nt; ++t) {
            score += scores[t];
            for (int k = 0; k < 6; ++k) g[k] += gs[t * 6 + k];
            for (int k = 0; k < 36; ++k) H[k] += Hs[t * 36 + k];
            pairs += tpairs[t];
        }
        if (pairs_out) *pairs_out = pairs;
        return score;
    }

    // computeHessian (:550-607): serial, double, radius neighbours
    void compute_hessian(double H[36], const std::vector<Pt>& trans, long long* pairs_out) {
        for (int k = 0; k < 36; ++k) H[k] = 0;
        double PG[3][6] = {{0}}, PH[18][6] = {{0}};
        PG[0][0] = PG[1][1] = PG[2][2] = 1.0;
        std::vector<const Leaf*> nb;
        long long pairs = 0;
        for (size_t idx = 0; idx < input.size(); idx++) {
            radius_neighbors(trans[idx], nb);
            for (const Leaf* cell : nb) {
                const double x[3] = {input[idx].x, input[idx].y, input[idx].z};
                double xt[3] = {trans[idx].x, trans[idx].y, trans[idx].z};
                for (int a = 0; a < 3; ++a) xt[a] -= cell->mean[a];
                point_derivatives_d(x, PG, PH, true);
                update_hessian_d(H, PG, PH, xt, cell->icov);
                ++pairs;
            }
        }
        if (pairs_out) *pairs_out = pairs;
    }

    void record(int kind, const double x[6], double score, const double g[6], const double H[36], long long pairs) {
        PassRecord r;
        r.kind = kind; r.newton_iter = cur_newton; r.score = score; r.pairs = pairs;
        for (int k = 0; k < 6; ++k) { r.x[k] = x[k]; r.g[k] = g[k]; }
        for (int k = 0; k < 36; ++k) r.H[k] = H[k];
        history.push_back(r);
        pairs_total += pairs;
    }

    // More-Thuente (:643-757)
    static bool update_interval(double& a_l, double& f_l, double& g_l, double& a_u, double& f_u, double& g_u, double a_t, double f_t, double g_t) {
        if (f_t > f_l) { a_u = a_t; f_u = f_t; g_u = g_t; return false; }
        else if (g_t * (a_l - a_t) > 0) { a_l = a_t; f_l = f_t; g_l = g_t; return false; }
        else if (g_t * (a_l - a_t) < 0) { a_u = a_l; f_u = f_l; g_u = g_l; a_l = a_t; f_l = f_t; g_l = g_t; return false; }
        else return true;
    }
    static double trial_value(double a_l, double f_l, double g_l, double a_u, double f_u, double g_u, double a_t, double f_t, double g_t) {
        if (f_t > f_l) {
            double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
            double w = std::sqrt(z * z - g_t * g_l);
            double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
            double a_q = a_l - 0.5 * (a_l - a_t) * g_l / (g_l - (f_l - f_t) / (a_l - a_t));
            if (std::fabs(a_c - a_l) < std::fabs(a_q - a_l)) return a_c;
            else return 0.5 * (a_q + a_c);
        } else if (g_t * g_l < 0) {
            double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
            double w = std::sqrt(z * z - g_t * g_l);
            double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
            double a_s = a_l - (a_l - a_t) / (g_l - g_t) * g_l;
            if (std::fabs(a_c - a_t) >= std::fabs(a_s - a_t)) return a_c;
            else return a_s;
        } else if (std::fabs(g_t) <= std::fabs(g_l)) {
            double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
            double w = std::sqrt(z * z - g_t * g_l);
            double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
            double a_s = a_l - (a_l - a_t) / (g_l - g_t) * g_l;
            double a_t_next;
            if (std::fabs(a_c - a_t) < std::fabs(a_s - a_t)) a_t_next = a_c;
            else a_t_next = a_s;
            if (a_t > a_l) return std::min(a_t + 0.66 * (a_u - a_t), a_t_next);
            else return std::max(a_t + 0.66 * (a_u - a_t), a_t_next);
        } else {
            double z = 3 * (f_t - f_u) / (a_t - a_u) - g_t - g_u;
            double w = std::sqrt(z * z - g_t * g_u);
            return a_u + (a_t - a_u) * (w - g_u - z) / (g_t - g_u + 2 * w);
        }
    }

    double step_length_mt(const double x[6], double step_dir[6], double step_init, double step_max, double step_min,
                          double& score, double g[6], double H[36], std::vector<Pt>& trans) {
        double phi_0 = -score;
        double d_phi_0 = 0;
        d_phi_0 = dot6(g, step_dir);
        d_phi_0 = -d_phi_0;
        double x_t[6];
        if (d_phi_0 >= 0) {
            if (d_phi_0 == 0) return 0;
            d_phi_0 *= -1;
            for (int k = 0; k < 6; ++k) step_dir[k] *= -1;
        }
        const int max_step_iterations = 10;
        int step_iterations = 0;
        const double mu = 1.e-4, nu = 0.9;
        double a_l = 0, a_u = 0;
        auto psi = [&](double a, double f_a) { return f_a - phi_0 - mu * d_phi_0 * a; };
        auto dpsi = [&](double g_a) { return g_a - mu * d_phi_0; };
        double f_l = psi(a_l, phi_0), g_l = dpsi(d_phi_0);
        double f_u = psi(a_u, phi_0), g_u = dpsi(d_phi_0);
        // NOTE: reference bug kept verbatim (ndt_omp_impl.hpp:807): the inner loop below is skipped whenever step_max > step_min
        bool interval_converged = (step_max - step_min) > 0, open_interval = true;
        double a_t = step_init;
        a_t = std::min(a_t, step_max);
        a_t = std::max(a_t, step_min);
        for (int k = 0; k < 6; ++k) x_t[k] = x[k] + step_dir[k] * a_t;
        convert_transform(x_t, final_tf);
        transform_cloud(input, trans, final_tf);
        long long pairs = 0;
        score = compute_derivatives(g, H, trans, x_t, true, &pairs);
        record(0, x_t, score, g, H, pairs);
        double phi_t = -score;
        double d_phi_t = 0;
        d_phi_t = dot6(g, step_dir);
        d_phi_t = -d_phi_t;
        double psi_t = psi(a_t, phi_t);
        double d_psi_t = dpsi(d_phi_t);
        while (!interval_converged && step_iterations < max_step_iterations && !(psi_t <= 0 && d_phi_t <= -nu * d_phi_0)) {
            if (open_interval) a_t = trial_value(a_l, f_l, g_l, a_u, f_u, g_u, a_t, psi_t, d_psi_t);
            else a_t = trial_value(a_l, f_l, g_l, a_u, f_u, g_u, a_t, phi_t, d_phi_t);
            a_t = std::min(a_t, step_max);
            a_t = std::max(a_t, step_min);
            for (int k = 0; k < 6; ++k) x_t[k] = x[k] + step_dir[k] * a_t;
            convert_transform(x_t, final_tf);
            transform_cloud(input, trans, final_tf);
            score = compute_derivatives(g, H, trans, x_t, false, &pairs);
            record(1, x_t, score, g, H, pairs);
            phi_t = -score;
            d_phi_t = 0;
            d_phi_t = dot6(g, step_dir);
            d_phi_t = -d_phi_t;
            psi_t = psi(a_t, phi_t);
            d_psi_t = dpsi(d_phi_t);
            if (open_interval && (psi_t <= 0 && d_psi_t >= 0)) {
                open_interval = false;
                f_l = f_l + phi_0 - mu * d_phi_0 * a_l;
                g_l = g_l + mu * d_phi_0;
                f_u = f_u + phi_0 - mu * d_phi_0 * a_u;
                g_u = g_u + mu * d_phi_0;
            }
            if (open_interval) interval_converged = update_interval(a_l, f_l, g_l, a_u, f_u, g_u, a_t, psi_t, d_psi_t);
            else interval_converged = update_interval(a_l, f_l, g_l, a_u, f_u, g_u, a_t, phi_t, d_phi_t);
            step_iterations++;
        }
        if (step_iterations) {
            compute_hessian(H, trans, &pairs);
            record(2, x_t, score, g, H, pairs);
        }
        return a_t;
    }

    // pcl::Registration::align + computeTransformation (:73-164)
    int align(const float guess[16], Result* res, std::vector<Pt>* output) {
        if (!has_target || !has_source) return -1;
        history.clear();
        pairs_total = 0;
        cur_newton = 0;
        // align(): output = copy(input), data[3] = 1, final = transformation = previous = I
        std::vector<Pt> out = input;
        for (auto& p : out) p.w = 1.0f;
        for (int k = 0; k < 16; ++k) final_tf[k] = (k % 5 == 0) ? 1.f : 0.f;
        nr_iterations = 0;
        converged = false;
        gauss_constants();
        bool is_identity = true;
        for (int k = 0; k < 16; ++k) if (guess[k] != ((k % 5 == 0) ? 1.f : 0.f)) is_identity = false;
        if (!is_identity) {
            for (int k = 0; k < 16; ++k) final_tf[k] = guess[k];
            std::vector<Pt> tmp;
            transform_cloud(out, tmp, guess);
            out.swap(tmp);
        }
        M3f L;
        for (int j = 0; j < 3; ++j) for (int i = 0; i < 3; ++i) L(i, j) = final_tf[i + 4 * j];
        M3f R = e33::rotation_of(L);
        float eul[3];
        e33::euler_angles_012(R, eul);
        double p[6] = {final_tf[12], final_tf[13], final_tf[14], eul[0], eul[1], eul[2]};
        double g[6], H[36], delta_p[6];
        long long pairs = 0;
        double score = compute_derivatives(g, H, out, p, true, &pairs);
        record(0, p, score, g, H, pairs);
        while (!converged) {
            M6d Hm;
            for (int i = 0; i < 6; ++i) for (int j = 0; j < 6; ++j) Hm(i, j) = H[i * 6 + j];
            e33::SVD<double, 6> sv = e33::jacobi_svd<double, 6>(Hm);
            double mg[6];
            for (int k = 0; k < 6; ++k) mg[k] = -g[k];
            e33::svd_solve<double, 6>(sv, mg, delta_p);
            const double nrm2 = dot6(delta_p, delta_p);
            double delta_p_norm = std::sqrt(nrm2);
            if (delta_p_norm == 0 || delta_p_norm != delta_p_norm) {
                trans_probability = score / static_cast<double>(input.size());
                converged = delta_p_norm == delta_p_norm;
                break;
            }
            if (nrm2 > 0) { double s = std::sqrt(nrm2); for (int k = 0; k < 6; ++k) delta_p[k] /= s; }  // normalize()
            cur_newton = nr_iterations + 1;
            delta_p_norm = step_length_mt(p, delta_p, delta_p_norm, prm.step_size, prm.trans_eps / 2, score, g, H, out);
            for (int k = 0; k < 6; ++k) delta_p[k] *= delta_p_norm;
            for (int k = 0; k < 6; ++k) p[k] = p[k] + delta_p[k];
            if (nr_iterations > prm.max_iter || (nr_iterations && (std::fabs(delta_p_norm) < prm.trans_eps))) converged = true;
            nr_iterations++;
        }
        trans_probability = score / static_cast<double>(input.size());
        if (res) {
            for (int k = 0; k < 16; ++k) res->final_tf[k] = final_tf[k];
            res->nr_iterations = nr_iterations;
            res->converged = converged ? 1 : 0;
            res->trans_probability = trans_probability;
            res->score = score;
            res->n_passes = (int)history.size();
            res->n_pairs_total = pairs_total;
        }
        if (output) *output = out;
        return 0;
    }

    // calculateScore (:919-952)
    double calculate_score(const std::vector<Pt>& trans) const {
        double score = 0;
        std::vector<const Leaf*> nb;
        for (size_t idx = 0; idx < trans.size(); idx++) {
            cells.radius(trans[idx], prm.resolution, nb);
            for (const Leaf* cell : nb) {
                double xt[3] = {trans[idx].x, trans[idx].y, trans[idx].z};
                for (int a = 0; a < 3; ++a) xt[a] -= cell->mean[a];
                double cx[3];
                mv3(cell->icov, xt, cx);
                double e = std::exp(-gauss_d2 * d3(xt, cx) / 2);
                double score_inc = -gauss_d1 * e - gauss_d3;
                score += score_inc / nb.size();
            }
        }
        return score / static_cast<double>(trans.size());
    }
};

static std::vector<Pt> load_points(const float* xyz, size_t n, size_t stride_bytes) {
    std::vector<Pt> v(n);
    const char* base = reinterpret_cast<const char*>(xyz);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        v[i] = Pt{f[0], f[1], f[2], 1.0f};
    }
    return v;
}

}  // namespace orc

// ---------------------------------------------------------------------------
// C ABI for ctypes (tests / bench cpu_baseline only)
// ---------------------------------------------------------------------------
extern "C" {

typedef orc::Params orc_params;
typedef orc::Result orc_result;
typedef orc::PassRecord orc_pass_record;

void* orc_create(void) { return new orc::NDT(); }
void orc_destroy(void* h) { delete static_cast<orc::NDT*>(h); }

void orc_default_params(orc_params* p) { orc::NDT t; *p = t.prm; }

void orc_set_params(void* h, const orc_params* p) {
    orc::NDT* n = static_cast<orc::NDT*>(h);
    const bool res_changed = n->prm.resolution != p->resolution;
    const bool kind_changed = (n->prm.precision_mode == 2) != (p->precision_mode == 2);
    n->prm = *p;
    // setResolution re-inits the grid only if a source is set (ndt_omp.h:127-137); switching to / from the ndt_cpu
    // backend means another grid type (cpu::VoxelGrid): built afresh like the product does
    if (n->has_target && ((res_changed && n->has_source) || kind_changed)) n->init_cells();
}

// cpu::SymmetricEigensolver3x3 restatement (column-major A and V), exposed for the known-answer tests
void orc_aw_eigen3(const double A[9], double ev[3], double V[9]) {
    M3d m, v;
    for (int k = 0; k < 9; ++k) m.a[k] = A[k];
    orc::aw_eigen3(m, ev, v);
    for (int k = 0; k < 9; ++k) V[k] = v.a[k];
}

// cpu::NormalDistributionsTransform::updateVoxelGrid (ndt_cpu/NormalDistributionsTransform.h:39, odom_node.cpp:344-345):
// ndt_cpu scatters the new points into its kept per-voxel sums (VoxelGrid::update -> updateVoxelContent) and recomputes
// the voxels; the other backends have no incremental path and are rebuilt over old + new.
int orc_update_target(void* h, const float* xyz, size_t n, size_t stride_bytes) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    std::vector<orc::Pt> add = orc::load_points(xyz, n, stride_bytes);
    const size_t old = o->target.size();
    o->target.insert(o->target.end(), add.begin(), add.end());
    if (!o->has_target) { o->has_target = true; o->target_dense = true; o->init_cells(); return o->cells.overflow ? 4 : 0; }
    o->has_target = true;
    if (o->cells.autoware) {
        o->cells.aw_scatter(o->target, old, o->target_dense);
        o->cells.aw_finalize();
    } else {
        o->init_cells();
    }
    return o->cells.overflow ? 4 : 0;
}

int orc_set_target(void* h, const float* xyz, size_t n, size_t stride_bytes, int is_dense) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    o->target = orc::load_points(xyz, n, stride_bytes);
    o->target_dense = is_dense != 0;
    o->has_target = true;
    o->init_cells();
    return o->cells.overflow ? 4 : 0;
}

int orc_set_source(void* h, const float* xyz, size_t n, size_t stride_bytes) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    o->input = orc::load_points(xyz, n, stride_bytes);
    o->has_source = true;
    return 0;
}

int orc_align(void* h, const float guess[16], orc_result* res, float* out_xyz4) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    std::vector<orc::Pt> out;
    int rc = o->align(guess, res, out_xyz4 ? &out : nullptr);
    if (rc == 0 && out_xyz4)
        for (size_t i = 0; i < out.size(); ++i) { out_xyz4[4 * i] = out[i].x; out_xyz4[4 * i + 1] = out[i].y; out_xyz4[4 * i + 2] = out[i].z; out_xyz4[4 * i + 3] = out[i].w; }
    return rc;
}

int orc_history_size(void* h) { return (int)static_cast<orc::NDT*>(h)->history.size(); }
int orc_history(void* h, orc_pass_record* out, int cap) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    int n = std::min(cap, (int)o->history.size());
    for (int i = 0; i < n; ++i) out[i] = o->history[i];
    return n;
}

// One derivative pass at pose parameters p with point transform T (col-major 4x4).
double orc_derivatives(void* h, const double p[6], const float T[16], int compute_hessian, double g[6], double H[36], long long* pairs) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    o->gauss_constants();
    std::vector<orc::Pt> trans;
    orc::transform_cloud(o->input, trans, T);
    return o->compute_derivatives(g, H, trans, p, compute_hessian != 0, pairs);
}

void orc_hessian_radius(void* h, const double p[6], const float T[16], double H[36], long long* pairs) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    o->gauss_constants();
    o->angle_derivatives(p, true);
    std::vector<orc::Pt> trans;
    orc::transform_cloud(o->input, trans, T);
    o->compute_hessian(H, trans, pairs);
}

double orc_calculate_score(void* h, const float T[16]) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    std::vector<orc::Pt> trans;
    orc::transform_cloud(o->input, trans, T);
    return o->calculate_score(trans);
}

void orc_convert_transform(const double x[6], float T[16]) { orc::convert_transform(x, T); }
void orc_convert_transform_mode(const double x[6], float T[16], int trig_mode) { orc::convert_transform(x, T, trig_mode); }

void orc_initial_p(const float guess[16], double p[6]) {
    M3f L;
    for (int j = 0; j < 3; ++j) for (int i = 0; i < 3; ++i) L(i, j) = guess[i + 4 * j];
    M3f R = e33::rotation_of(L);
    float eul[3];
    e33::euler_angles_012(R, eul);
    p[0] = guess[12]; p[1] = guess[13]; p[2] = guess[14]; p[3] = eul[0]; p[4] = eul[1]; p[5] = eul[2];
}

void orc_gauss_constants(void* h, double out[3]) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    o->gauss_constants();
    out[0] = o->gauss_d1; out[1] = o->gauss_d2; out[2] = o->gauss_d3;
}

// Grid export: header ints [min_b3, max_b3, div_b3, divb_mul3, n_leaves, n_cloud, overflow]
void orc_grid_header(void* h, int out[15]) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    for (int a = 0; a < 3; ++a) { out[a] = o->cells.min_b[a]; out[3 + a] = o->cells.max_b[a]; out[6 + a] = o->cells.div_b[a]; out[9 + a] = o->cells.divb_mul[a]; }
    out[12] = (int)o->cells.leaves.size();
    out[13] = (int)o->cells.centroids.size();
    out[14] = o->cells.overflow ? 1 : 0;
}

// Leaves in ascending key order: key, nr_points (after rejection), mean[3], icov[9] (row-major), centroid[3], evals[3]
int orc_grid_leaves(void* h, int* keys, int* npts, double* mean, double* icov, float* centroid, double* evals, int cap) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    int i = 0;
    for (auto& kv : o->cells.leaves) {
        if (i >= cap) break;
        const orc::Leaf& L = kv.second;
        keys[i] = (int)kv.first;
        npts[i] = L.nr_points;
        for (int a = 0; a < 3; ++a) { mean[3 * i + a] = L.mean[a]; centroid[3 * i + a] = L.centroid[a]; evals[3 * i + a] = L.evals[a]; }
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) icov[9 * i + 3 * r + c] = L.icov(r, c);
        ++i;
    }
    return i;
}

// Per-point neighbour lists (keys) for the given transformed cloud (xyz4), search mode, max 32 per point.
int orc_neighbors(void* h, const float* xyz4, int n, int search, int* out_keys, int* out_count) {
    orc::NDT* o = static_cast<orc::NDT*>(h);
    std::vector<const orc::Leaf*> nb;
    std::map<const orc::Leaf*, int> rev;
    for (auto& kv : o->cells.leaves) rev[&kv.second] = (int)kv.first;
    long long total = 0;
    for (int i = 0; i < n; ++i) {
        orc::Pt p{xyz4[4 * i], xyz4[4 * i + 1], xyz4[4 * i + 2], 1.f};
        o->find_neighbors(p, search, nb);
        int c = std::min<int>(32, (int)nb.size());
        out_count[i] = (int)nb.size();
        for (int k = 0; k < c; ++k) out_keys[32 * i + k] = rev[nb[k]];
        total += nb.size();
    }
    return (int)total;
}

// PCL VoxelGrid<PointXYZI>::applyFilter (downsample_all_data_ = true, min points 0) — next-row a16.
// Output centroids (x,y,z,intensity) ordered by ascending voxel index.  Within-voxel order follows input
// order (PCL's std::sort is not stable, so its float sums are implementation-defined; parity to tolerance).
int orc_voxel_downsample(const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset, float leaf, float* out4, int cap) {
    const char* base = reinterpret_cast<const char*>(xyzi);
    float inv = 1.0f / leaf;
    float mn[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
    float mx[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], f[a]); mx[a] = std::max(mx[a], f[a]); }
    }
    int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
    int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
    int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
    if ((dx * dy * dz) > static_cast<int64_t>(std::numeric_limits<int32_t>::max())) {
        // PCL: warn and output = input copy
        int m = (int)std::min<size_t>(n, (size_t)cap);
        for (int i = 0; i < m; ++i) { const float* f = reinterpret_cast<const float*>(base + i * stride_bytes); for (int a = 0; a < 4; ++a) out4[4 * i + a] = f[a == 3 ? intensity_offset : a]; }
        return -(int)n;
    }
    int minb[3], maxb[3], divb[3];
    for (int a = 0; a < 3; ++a) { minb[a] = (int)std::floor(mn[a] * inv); maxb[a] = (int)std::floor(mx[a] * inv); divb[a] = maxb[a] - minb[a] + 1; }
    int mul[3] = {1, divb[0], divb[0] * divb[1]};
    std::vector<std::pair<unsigned int, unsigned int>> idx(n);
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        int ijk0 = static_cast<int>(std::floor(f[0] * inv) - static_cast<float>(minb[0]));
        int ijk1 = static_cast<int>(std::floor(f[1] * inv) - static_cast<float>(minb[1]));
        int ijk2 = static_cast<int>(std::floor(f[2] * inv) - static_cast<float>(minb[2]));
        idx[i] = {(unsigned)(ijk0 * mul[0] + ijk1 * mul[1] + ijk2 * mul[2]), (unsigned)i};
    }
    std::stable_sort(idx.begin(), idx.end(), [](const std::pair<unsigned, unsigned>& a, const std::pair<unsigned, unsigned>& b) { return a.first < b.first; });
    int outn = 0;
    size_t i = 0;
    while (i < n) {
        size_t j = i;
        float s[4] = {0, 0, 0, 0};
        while (j < n && idx[j].first == idx[i].first) {
            const float* f = reinterpret_cast<const float*>(base + idx[j].second * stride_bytes);
            s[0] += f[0]; s[1] += f[1]; s[2] += f[2]; s[3] += f[intensity_offset];
            ++j;
        }
        float cnt = (float)(j - i);
        if (outn < cap) for (int a = 0; a < 4; ++a) out4[4 * outn + a] = s[a] / cnt;
        ++outn;
        i = j;
    }
    return outn;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// filter_node front end, restated from xchu_mapping/src/filter_node.cpp:218-273 and the PCL 1.7
// filters it calls (third-party, not vendored; algorithm as published in pcl/filters/impl/filter.hpp
// removeNaNFromPointCloud, voxel_grid.hpp, statistical_outlier_removal.hpp applyFilterIndices):
//   removeNaNFromPointCloud (only when !is_dense) -> keep 1 < sqrt(pow(x,2.0)+pow(y,2.0)) < 60 -> VoxelGrid(leaf)
//   -> StatisticalOutlierRemoval(mean_k, stddev_mul): per point the k+1 nearest (exact kd-tree, FLANN L2_Simple float
//   squared distances, ascending, itself first), distance = (float)(sum_{j=1..k} sqrt(d_j) / k) (double sum; PCL's
//   unqualified sqrt on a float resolves to ::sqrt(double)), sum / sq_sum over all points in input order (sq_sum adds
//   the float square), threshold = mean + mul * sqrt((sq_sum - sum^2/n)/(n-1)), keep distance <= threshold.
// k-NN here: exact, by a hash grid with ring search (or brute force when brute != 0, to check the grid search).
// ---------------------------------------------------------------------------
namespace orc {

static inline float l2_simple3(const float* a, const float* b) {
    float d = 0.f, u;
    u = a[0] - b[0]; d += u * u;
    u = a[1] - b[1]; d += u * u;
    u = a[2] - b[2]; d += u * u;
    return d;
}

// the k1 smallest squared distances from point i to all points (itself included), ascending
static void knn_sq(const std::vector<float>& P, int n, int i, int k1, bool brute, float cell,
                   const std::unordered_map<long long, std::vector<int>>& grid, int ext[3][2], std::vector<float>& out) {
    out.clear();
    const float* q = &P[4 * (size_t)i];
    if (brute) {
        std::vector<float> d(n);
        for (int j = 0; j < n; ++j) d[j] = l2_simple3(&P[4 * (size_t)j], q);
        const int k = std::min(k1, n);
        std::partial_sort(d.begin(), d.begin() + k, d.end());
        out.assign(d.begin(), d.begin() + k);
        return;
    }
    auto key = [](long long x, long long y, long long z) { return ((x & 0x1FFFFF) << 42) | ((y & 0x1FFFFF) << 21) | (z & 0x1FFFFF); };
    long long c[3];
    for (int a = 0; a < 3; ++a) c[a] = (long long)std::floor(q[a] / cell);
    std::vector<float> best;
    long long rmax = 0;
    for (int a = 0; a < 3; ++a) rmax = std::max(rmax, std::max(c[a] - ext[a][0], ext[a][1] - c[a]));
    for (long long r = 0; r <= rmax; ++r) {
        for (long long dz = -r; dz <= r; ++dz)
            for (long long dy = -r; dy <= r; ++dy)
                for (long long dx = -r; dx <= r; ++dx) {
                    if (std::max(std::llabs(dx), std::max(std::llabs(dy), std::llabs(dz))) != r) continue;
                    auto it = grid.find(key(c[0] + dx, c[1] + dy, c[2] + dz));
                    if (it == grid.end()) continue;
                    for (int j : it->second) best.push_back(l2_simple3(&P[4 * (size_t)j], q));
                }
        if ((int)best.size() >= k1) {
            std::nth_element(best.begin(), best.begin() + (k1 - 1), best.end());
            const float kth = best[k1 - 1];
            // every unvisited point lies in a cell at Chebyshev distance >= r+1: at least r*cell away along an axis
            const double bound = std::max(0.0, (double)r * cell * (1.0 - 1e-6));
            if ((double)kth <= bound * bound) break;
        }
    }
    const int k = std::min(k1, (int)best.size());
    std::partial_sort(best.begin(), best.begin() + k, best.end());
    out.assign(best.begin(), best.begin() + k);
}

}  // namespace orc

extern "C" int orc_filter_scan(const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset, int is_dense, float leaf, double r_min,
                               double r_max, int mean_k, double stddev_mul, int brute, float* out4, int cap, float* dist_out, int dist_cap,
                               double* thr_out, int* n_voxel_out, int outlier_method, double ror_radius, int ror_min_neighbors);

int orc_filter_scan(const float* xyzi, size_t n, size_t stride_bytes, int intensity_offset, int is_dense, float leaf, double r_min,
                    double r_max, int mean_k, double stddev_mul, int brute, float* out4, int cap, float* dist_out, int dist_cap,
                    double* thr_out, int* n_voxel_out, int outlier_method, double ror_radius, int ror_min_neighbors) {
    const char* base = reinterpret_cast<const char*>(xyzi);
    std::vector<float> crop;  // x,y,z,i
    for (size_t i = 0; i < n; ++i) {
        const float* f = reinterpret_cast<const float*>(base + i * stride_bytes);
        if (!is_dense && !(std::isfinite(f[0]) && std::isfinite(f[1]) && std::isfinite(f[2]))) continue;
        const double r = std::sqrt(std::pow(f[0], 2.0) + std::pow(f[1], 2.0));
        if (r_min < r && r < r_max) { crop.push_back(f[0]); crop.push_back(f[1]); crop.push_back(f[2]); crop.push_back(f[intensity_offset]); }
    }
    const int m = (int)(crop.size() / 4);
    if (thr_out) thr_out[0] = thr_out[1] = thr_out[2] = 0.0;
    if (n_voxel_out) *n_voxel_out = 0;
    if (m == 0) return 0;
    std::vector<float> ds((size_t)m * 4);
    int nv = orc_voxel_downsample(crop.data(), (size_t)m, 16, 3, leaf, ds.data(), m);
    if (nv < 0) nv = -nv;  // overflow: output = input copy
    ds.resize((size_t)nv * 4);
    if (n_voxel_out) *n_voxel_out = nv;
    if (outlier_method == 1) {
        // RadiusOutlierRemoval (filter_node.cpp:265-272; PCL 1.7 applyFilterIndices): radiusSearch counts the points
        // with squared distance < (float)(radius*radius), the point itself included; keep when count >= min_neighbors
        const float r2 = static_cast<float>(ror_radius * ror_radius);
        int k = 0;
        for (int i = 0; i < nv; ++i) {
            int cnt = 0;
            for (int j = 0; j < nv; ++j) cnt += orc::l2_simple3(&ds[4 * (size_t)j], &ds[4 * (size_t)i]) < r2 ? 1 : 0;
            if (cnt < ror_min_neighbors) continue;
            if (k < cap) std::memcpy(out4 + 4 * (size_t)k, &ds[4 * (size_t)i], 4 * sizeof(float));
            ++k;
        }
        return k;
    }
    if (nv <= mean_k) {
        const int k = std::min(nv, cap);
        std::memcpy(out4, ds.data(), (size_t)k * 4 * sizeof(float));
        return nv;
    }
    const float cell = 3.0f * leaf;
    std::unordered_map<long long, std::vector<int>> grid;
    int ext[3][2] = {{1 << 30, -(1 << 30)}, {1 << 30, -(1 << 30)}, {1 << 30, -(1 << 30)}};
    auto key = [](long long x, long long y, long long z) { return ((x & 0x1FFFFF) << 42) | ((y & 0x1FFFFF) << 21) | (z & 0x1FFFFF); };
    if (!brute)
        for (int i = 0; i < nv; ++i) {
            long long c[3];
            for (int a = 0; a < 3; ++a) {
                c[a] = (long long)std::floor(ds[4 * (size_t)i + a] / cell);
                ext[a][0] = std::min<long long>(ext[a][0], c[a]);
                ext[a][1] = std::max<long long>(ext[a][1], c[a]);
            }
            grid[key(c[0], c[1], c[2])].push_back(i);
        }
    std::vector<float> distances(nv);
    std::vector<float> nn;
    for (int i = 0; i < nv; ++i) {
        orc::knn_sq(ds, nv, i, mean_k + 1, brute != 0, cell, grid, ext, nn);
        double dist_sum = 0.0;
        for (int k = 1; k < mean_k + 1; ++k) dist_sum += std::sqrt((double)nn[k]);
        distances[i] = static_cast<float>(dist_sum / mean_k);
    }
    double sum = 0, sq_sum = 0;
    for (int i = 0; i < nv; ++i) {
        sum += distances[i];
        sq_sum += distances[i] * distances[i];
    }
    const double mean = sum / static_cast<double>(nv);
    const double variance = (sq_sum - sum * sum / static_cast<double>(nv)) / (static_cast<double>(nv) - 1);
    const double stddev = std::sqrt(variance);
    const double thr = mean + stddev_mul * stddev;
    if (thr_out) { thr_out[0] = thr; thr_out[1] = mean; thr_out[2] = stddev; }
    if (dist_out) std::memcpy(dist_out, distances.data(), (size_t)std::min(nv, dist_cap) * sizeof(float));
    int k = 0;
    for (int i = 0; i < nv; ++i) {
        if (distances[i] > thr) continue;
        if (k < cap) std::memcpy(out4 + 4 * (size_t)k, &ds[4 * (size_t)i], 4 * sizeof(float));
        ++k;
    }
    return k;
}

extern "C" {
double orc_now(void) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // extern "C"
