// ndt_hip.hpp — C++ face of libndt_hip.so, shaped like the class it replaces:
//   pclomp::NormalDistributionsTransform<PointSource, PointTarget>
//   (reference: xchu_mapping/include/pclomp/ndt_omp.h:70-497, driven by odom_node.cpp:69-80, 227-283, 338-349).
// Header-only RAII wrapper over the C-ABI of include/ndt_hip.h: same method names, same argument meaning; clouds are
// plain x,y,z(,intensity) float arrays (host, with a byte stride; or device float4) instead of pcl::PointCloud, and
// 4x4 transforms are column-major float[16] (Eigen::Matrix4f storage).  Errors throw ndt_hip::Error (the reference
// prints PCL warnings and returns; a C++ caller that wants the PCL behaviour catches).
#ifndef NDT_HIP_HPP_
#define NDT_HIP_HPP_

#include <array>
#include <cfloat>
#include <stdexcept>
#include <string>

#include "ndt_hip.h"

namespace ndt_hip {

using Matrix4f = std::array<float, 16>;  // column-major, as Eigen::Matrix4f::data()

inline Matrix4f identity4() { return Matrix4f{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}; }

class Error : public std::runtime_error {
public:
    Error(ndt_status s, const std::string& what) : std::runtime_error(what), status(s) {}
    ndt_status status;
};

// = pclomp::NeighborSearchMethod (ndt_omp.h:52-57)
enum NeighborSearchMethod { KDTREE = NDT_KDTREE, DIRECT26 = NDT_DIRECT26, DIRECT7 = NDT_DIRECT7, DIRECT1 = NDT_DIRECT1 };

class NormalDistributionsTransform {
public:
    explicit NormalDistributionsTransform(int device = 0) {
        ndt_default_params(&prm_);
        prm_.device = device;
        check(ndt_create(&prm_, &ctx_), "ndt_create");
    }
    ~NormalDistributionsTransform() { ndt_destroy(ctx_); }
    NormalDistributionsTransform(const NormalDistributionsTransform&) = delete;
    NormalDistributionsTransform& operator=(const NormalDistributionsTransform&) = delete;

    // ---- parameters (ndt_omp.h:127-204, pcl::Registration)
    void setResolution(float r) { prm_.resolution = r; push(); }
    float getResolution() const { return prm_.resolution; }
    void setStepSize(double s) { prm_.step_size = s; push(); }
    double getStepSize() const { return prm_.step_size; }
    void setOulierRatio(double o) { prm_.outlier_ratio = o; push(); }
    double getOulierRatio() const { return prm_.outlier_ratio; }
    void setTransformationEpsilon(double e) { prm_.trans_eps = e; push(); }
    void setMaximumIterations(int n) { prm_.max_iter = n; push(); }
    int getMaximumIterations() const { return prm_.max_iter; }
    void setNeighborhoodSearchMethod(NeighborSearchMethod m) { prm_.search = m; push(); }
    // backend: 0 = pclomp ndt_omp, 1 = pcl::NormalDistributionsTransform, 2 = cpu::NormalDistributionsTransform (ndt_cpu)
    void setPrecisionMode(int mode) { prm_.precision_mode = mode; push(); }
    // cpu::NormalDistributionsTransform::updateVoxelGrid (ndt_cpu/NormalDistributionsTransform.h:39)
    void updateVoxelGridDevice(const float* d_xyz4, size_t n) { check(ndt_update_target_device(ctx_, d_xyz4, n), "updateVoxelGrid"); }
    void setNumThreads(int) {}  // OpenMP thread count of the CPU reference: the device sizes its own grid

    // ---- clouds (pcl::Registration::setInputTarget / setInputSource)
    void setInputTarget(const float* xyz, size_t n, size_t stride_bytes = 32, bool is_dense = true) {
        check(ndt_set_target(ctx_, xyz, n, stride_bytes, is_dense ? 1 : 0), "setInputTarget");
    }
    // device float4 cloud, referenced (kept alive and unmodified by the caller until the next setInputTarget)
    void setInputTargetDevice(const float* d_xyz4, size_t n, bool is_dense = true) {
        check(ndt_set_target_device(ctx_, d_xyz4, n, is_dense ? 1 : 0), "setInputTarget");
    }
    void setInputSource(const float* xyz, size_t n, size_t stride_bytes = 32) {
        check(ndt_set_source(ctx_, xyz, n, stride_bytes), "setInputSource");
    }
    void setInputSourceDevice(const float* d_xyz4, size_t n) { check(ndt_set_source_device(ctx_, d_xyz4, n), "setInputSource"); }

    // ---- registration (pcl::Registration::align -> computeTransformation, ndt_omp_impl.hpp:73-164)
    void align(const Matrix4f& guess) { check(ndt_align(ctx_, guess.data(), &res_), "align"); }
    // align(output, guess): also writes the transformed source (x,y,z at each stride)
    void align(float* output_xyz, size_t stride_bytes, const Matrix4f& guess) {
        align(guess);
        check(ndt_get_output(ctx_, output_xyz, stride_bytes), "align output");
    }
    Matrix4f getFinalTransformation() const {
        Matrix4f m;
        for (int k = 0; k < 16; ++k) m[k] = res_.final_tf[k];
        return m;
    }
    bool hasConverged() const { return res_.converged != 0; }
    int getFinalNumIteration() const { return res_.nr_iterations; }
    double getTransformationProbability() const { return res_.trans_probability; }
    const ndt_result& result() const { return res_; }

    // pcl::Registration::getFitnessScore(max_range) over the last align's final transformation
    double getFitnessScore(double max_range = DBL_MAX) {
        double f = 0.0;
        check(ndt_fitness_score(ctx_, nullptr, max_range, &f, nullptr), "getFitnessScore");
        return f;
    }
    // calculateScore(trans_cloud) of the source under T (ndt_omp_impl.hpp:919-952)
    double calculateScore(const Matrix4f& T) {
        double s = 0.0;
        check(ndt_calculate_score(ctx_, T.data(), &s), "calculateScore");
        return s;
    }

    ndt_ctx* handle() const { return ctx_; }
    void check(ndt_status s, const char* what) const {
        if (s != NDT_OK) throw Error(s, std::string(what) + ": " + ndt_last_error(ctx_));
    }

private:
    void push() { check(ndt_set_params(ctx_, &prm_), "set params"); }
    ndt_params prm_{};
    ndt_ctx* ctx_ = nullptr;
    ndt_result res_{};
};

}  // namespace ndt_hip

#endif  // NDT_HIP_HPP_
