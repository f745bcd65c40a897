// oracle/eigen33_restate.h — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Clean-room restatement of the Eigen 3.3 numerical routines that the reference
// NDT path (xchu_mapping/include/pclomp/*) calls.  Eigen is NOT vendored under
// /root/reference and is absent from this image; the version is inferred as
// Eigen 3.3.x (SVDBase<JacobiSVD<...>> symbols and the ±π branch
// of eulerAngles in the reference's prebuilt libndt_omp.so).  The algorithms
// below restate Eigen 3.3's published source semantics:
//   * JacobiSVD<Matrix<T,N,N>>  (two-sided Jacobi, real_2x2_jacobi_svd, makeJacobi,
//     sort descending, SVDBase::_solve_impl rank truncation at N*eps*sigma_max)
//     — used at ndt_omp_impl.hpp:119-121 (6x6 double) and by
//     Transform::rotation() (3x3 float polar decomposition) at ndt_omp_impl.hpp:102.
//   * MatrixBase::eulerAngles(0,1,2) (float)           — ndt_omp_impl.hpp:102.
//   * SelfAdjointEigenSolver<Matrix3d>::compute        — voxel_grid_covariance_omp_impl.hpp:333.
//     (scaling, 3x3 tridiagonalization_inplace, implicit symmetric QR with
//      Wilkinson shift, ascending sort)
//   * Matrix3d::inverse() via cofactors                — voxel_grid_covariance_omp_impl.hpp:355,359.
// Summation orders are the natural sequential ones; Eigen's SSE reductions may
// associate some dot products differently (ulp-level), which is below the
// reference's own OpenMP-partition nondeterminism (ndt_omp_impl.hpp:205,276-280).
#pragma once
#include <cmath>
#include <limits>
#include <algorithm>

namespace e33 {

// column-major N x N
template <typename T, int N> struct Mat {
    T a[N * N];
    T& operator()(int i, int j) { return a[i + N * j]; }
    const T& operator()(int i, int j) const { return a[i + N * j]; }
    static Mat identity() { Mat m; for (int j = 0; j < N; ++j) for (int i = 0; i < N; ++i) m(i, j) = (i == j) ? T(1) : T(0); return m; }
    static Mat zero() { Mat m; for (int k = 0; k < N * N; ++k) m.a[k] = T(0); return m; }
};

template <typename T> struct Rot { T c, s; };

// apply_rotation_in_the_plane(x, y, j): x' = c x + s y ; y' = -s x + c y
template <typename T, int N> inline void apply_left(Mat<T, N>& m, int p, int q, Rot<T> j) {
    for (int k = 0; k < N; ++k) {
        T xi = m(p, k), yi = m(q, k);
        m(p, k) = j.c * xi + j.s * yi;
        m(q, k) = -j.s * xi + j.c * yi;
    }
}
// applyOnTheRight uses j.transpose() = (c, -s)
template <typename T, int N> inline void apply_right(Mat<T, N>& m, int p, int q, Rot<T> j) {
    const T c = j.c, s = -j.s;
    for (int k = 0; k < N; ++k) {
        T xi = m(k, p), yi = m(k, q);
        m(k, p) = c * xi + s * yi;
        m(k, q) = -s * xi + c * yi;
    }
}

// JacobiRotation::makeJacobi(x, y, z) (real)
template <typename T> inline Rot<T> make_jacobi(T x, T y, T z) {
    Rot<T> r;
    T deno = T(2) * std::fabs(y);
    if (deno < std::numeric_limits<T>::min()) { r.c = T(1); r.s = T(0); return r; }
    T tau = (x - z) / deno;
    T w = std::sqrt(tau * tau + T(1));
    T t;
    if (tau > T(0)) t = T(1) / (tau + w);
    else t = T(1) / (tau - w);
    T sign_t = t > T(0) ? T(1) : T(-1);
    T n = T(1) / std::sqrt(t * t + T(1));
    r.s = -sign_t * (y / std::fabs(y)) * std::fabs(t) * n;
    r.c = n;
    return r;
}

// internal::real_2x2_jacobi_svd
template <typename T, int N>
inline void real_2x2_jacobi_svd(const Mat<T, N>& mat, int p, int q, Rot<T>* jl, Rot<T>* jr) {
    Mat<T, 2> m;
    m(0, 0) = mat(p, p); m(0, 1) = mat(p, q);
    m(1, 0) = mat(q, p); m(1, 1) = mat(q, q);
    Rot<T> rot1;
    T t = m(0, 0) + m(1, 1);
    T d = m(1, 0) - m(0, 1);
    if (std::fabs(d) < std::numeric_limits<T>::min()) { rot1.s = T(0); rot1.c = T(1); }
    else {
        T u = t / d;
        T tmp = std::sqrt(T(1) + u * u);
        rot1.s = T(1) / tmp;
        rot1.c = u / tmp;
    }
    apply_left<T, 2>(m, 0, 1, rot1);
    *jr = make_jacobi<T>(m(0, 0), m(0, 1), m(1, 1));
    // *j_left = rot1 * j_right->transpose()
    Rot<T> o{jr->c, -jr->s};
    jl->c = rot1.c * o.c - rot1.s * o.s;
    jl->s = rot1.c * o.s + rot1.s * o.c;
}

template <typename T, int N> struct SVD {
    Mat<T, N> U, V;
    T sv[N];
    int nonzero;
};

// JacobiSVD<Matrix<T,N,N>>(A, ComputeFullU|ComputeFullV)
template <typename T, int N> inline SVD<T, N> jacobi_svd(const Mat<T, N>& A) {
    SVD<T, N> r;
    T scale = T(0);
    for (int k = 0; k < N * N; ++k) scale = std::max(scale, std::fabs(A.a[k]));
    if (scale == T(0)) scale = T(1);
    Mat<T, N> w;
    for (int k = 0; k < N * N; ++k) w.a[k] = A.a[k] / scale;
    r.U = Mat<T, N>::identity();
    r.V = Mat<T, N>::identity();
    const T considerAsZero = std::numeric_limits<T>::min();
    const T precision = T(2) * std::numeric_limits<T>::epsilon();
    T maxDiagEntry = T(0);
    for (int i = 0; i < N; ++i) maxDiagEntry = std::max(maxDiagEntry, std::fabs(w(i, i)));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 1000) {
        finished = true;
        ++sweeps;
        for (int p = 1; p < N; ++p) {
            for (int q = 0; q < p; ++q) {
                T threshold = std::max(considerAsZero, precision * maxDiagEntry);
                if (std::fabs(w(p, q)) > threshold || std::fabs(w(q, p)) > threshold) {
                    finished = false;
                    Rot<T> jl, jr;
                    real_2x2_jacobi_svd<T, N>(w, p, q, &jl, &jr);
                    apply_left<T, N>(w, p, q, jl);
                    apply_right<T, N>(r.U, p, q, Rot<T>{jl.c, -jl.s});  // U.applyOnTheRight(p,q,j_left.transpose())
                    apply_right<T, N>(w, p, q, jr);
                    apply_right<T, N>(r.V, p, q, jr);
                    maxDiagEntry = std::max(maxDiagEntry, std::max(std::fabs(w(p, p)), std::fabs(w(q, q))));
                }
            }
        }
    }
    for (int i = 0; i < N; ++i) {
        T a = w(i, i);
        r.sv[i] = std::fabs(a);
        if (a < T(0))
            for (int k = 0; k < N; ++k) r.U(k, i) = -r.U(k, i);
    }
    for (int i = 0; i < N; ++i) r.sv[i] *= scale;
    r.nonzero = N;
    for (int i = 0; i < N; i++) {
        int pos = i;
        T mx = r.sv[i];
        for (int k = i + 1; k < N; ++k)
            if (r.sv[k] > mx) { mx = r.sv[k]; pos = k; }
        if (mx == T(0)) { r.nonzero = i; break; }
        if (pos != i) {
            std::swap(r.sv[i], r.sv[pos]);
            for (int k = 0; k < N; ++k) { std::swap(r.U(k, pos), r.U(k, i)); std::swap(r.V(k, pos), r.V(k, i)); }
        }
    }
    return r;
}

// SVDBase::_solve_impl with default threshold (diagSize * epsilon)
template <typename T, int N> inline void svd_solve(const SVD<T, N>& s, const T* rhs, T* dst) {
    int rank = 0;
    if (N > 0) {
        T thr = std::max(s.sv[0] * (T(N) * std::numeric_limits<T>::epsilon()), std::numeric_limits<T>::min());
        int i = s.nonzero - 1;
        while (i >= 0 && s.sv[i] < thr) --i;
        rank = i + 1;
    }
    T tmp[N];
    for (int k = 0; k < rank; ++k) {
        T acc = T(0);
        for (int i = 0; i < N; ++i) acc += s.U(i, k) * rhs[i];
        tmp[k] = acc;
    }
    for (int k = 0; k < rank; ++k) tmp[k] = (T(1) / s.sv[k]) * tmp[k];
    for (int i = 0; i < N; ++i) {
        T acc = T(0);
        for (int k = 0; k < rank; ++k) acc += s.V(i, k) * tmp[k];
        dst[i] = acc;
    }
}

// 3x3 determinant (Eigen determinant_impl<3>)
template <typename T> inline T det3(const Mat<T, 3>& m) {
    auto h = [&](int a, int b, int c) { return m(0, a) * (m(1, b) * m(2, c) - m(1, c) * m(2, b)); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// Transform<float,3,Affine>::rotation() -> computeRotationScaling (polar decomposition)
inline Mat<float, 3> rotation_of(const Mat<float, 3>& L) {
    SVD<float, 3> s = jacobi_svd<float, 3>(L);
    // x = (U * V^T).determinant(); the 3x3 lazy product's entries as a0 + (a1 + a2) (libndt_omp.so 0x46190)
    Mat<float, 3> UVt;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) UVt(i, j) = s.U(i, 0) * s.V(j, 0) + (s.U(i, 1) * s.V(j, 1) + s.U(i, 2) * s.V(j, 2));
    float x = det3<float>(UVt);
    Mat<float, 3> m = s.U;
    for (int i = 0; i < 3; ++i) m(i, 0) /= x;
    Mat<float, 3> R;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R(i, j) = m(i, 0) * s.V(j, 0) + (m(i, 1) * s.V(j, 1) + m(i, 2) * s.V(j, 2));
    return R;
}

// MatrixBase<Matrix3f>::eulerAngles(0, 1, 2)  (Eigen 3.3)
inline void euler_angles_012(const Mat<float, 3>& m, float res[3]) {
    const int i = 0, j = 1, k = 2;
    res[0] = std::atan2(m(j, k), m(k, k));
    float c2 = std::sqrt(m(i, i) * m(i, i) + m(i, j) * m(i, j));
    if (res[0] > 0.f) {
        res[0] -= float(3.14159265358979323846);
        res[1] = std::atan2(-m(i, k), -c2);
    } else {
        res[1] = std::atan2(-m(i, k), c2);
    }
    // sincosf (0x3b4e1), modelled as the double functions rounded once (see convert_transform's trig_mode)
    float s1 = (float)std::sin((double)res[0]);
    float c1 = (float)std::cos((double)res[0]);
    res[2] = std::atan2(s1 * m(k, i) - c1 * m(j, i), c1 * m(j, j) - s1 * m(k, j));
    res[0] = -res[0]; res[1] = -res[1]; res[2] = -res[2];
}

// ---- SelfAdjointEigenSolver<Matrix3d>::compute (Eigen 3.3) ------------------
inline double positive_real_hypot(double x, double y) {
    double p = std::max(x, y);
    if (p == 0.0) return 0.0;
    double qp = std::min(y, x) / p;
    return p * std::sqrt(1.0 + qp * qp);
}
inline Rot<double> make_givens(double p, double q) {
    Rot<double> r;
    if (q == 0.0) { r.c = p < 0.0 ? -1.0 : 1.0; r.s = 0.0; }
    else if (p == 0.0) { r.c = 0.0; r.s = q < 0.0 ? 1.0 : -1.0; }
    else if (std::fabs(p) > std::fabs(q)) {
        double t = q / p; double u = std::sqrt(1.0 + t * t); if (p < 0.0) u = -u;
        r.c = 1.0 / u; r.s = -t * r.c;
    } else {
        double t = p / q; double u = std::sqrt(1.0 + t * t); if (q < 0.0) u = -u;
        r.s = -1.0 / u; r.c = -t * r.s;
    }
    return r;
}

inline bool self_adjoint_eigen3(const Mat<double, 3>& A, double evals[3], Mat<double, 3>& evecs) {
    Mat<double, 3> mat = Mat<double, 3>::zero();
    for (int j = 0; j < 3; ++j) for (int i = j; i < 3; ++i) mat(i, j) = A(i, j);  // lower triangle
    double scale = 0.0;
    for (int k = 0; k < 9; ++k) scale = std::max(scale, std::fabs(mat.a[k]));
    if (scale == 0.0) scale = 1.0;
    for (int j = 0; j < 3; ++j) for (int i = j; i < 3; ++i) mat(i, j) /= scale;
    double diag[3], sub[2];
    // tridiagonalization_inplace_selector<MatrixType,3,false>
    {
        const double tol = std::numeric_limits<double>::min();
        diag[0] = mat(0, 0);
        double v1norm2 = mat(2, 0) * mat(2, 0);
        if (v1norm2 <= tol) {
            diag[1] = mat(1, 1); diag[2] = mat(2, 2);
            sub[0] = mat(1, 0); sub[1] = mat(2, 1);
            mat = Mat<double, 3>::identity();
        } else {
            double beta = std::sqrt(mat(1, 0) * mat(1, 0) + v1norm2);
            double invBeta = 1.0 / beta;
            double m01 = mat(1, 0) * invBeta;
            double m02 = mat(2, 0) * invBeta;
            double q = 2.0 * m01 * mat(2, 1) + m02 * (mat(2, 2) - mat(1, 1));
            diag[1] = mat(1, 1) + m02 * q;
            diag[2] = mat(2, 2) - m02 * q;
            sub[0] = beta;
            sub[1] = mat(2, 1) - m01 * q;
            mat(0, 0) = 1; mat(0, 1) = 0; mat(0, 2) = 0;
            mat(1, 0) = 0; mat(1, 1) = m01; mat(1, 2) = m02;
            mat(2, 0) = 0; mat(2, 1) = m02; mat(2, 2) = -m01;
        }
    }
    // computeFromTridiagonal_impl
    const int n = 3, maxIterations = 30;
    int end = n - 1, start = 0, iter = 0;
    const double considerAsZero = std::numeric_limits<double>::min();
    const double precision = 2.0 * std::numeric_limits<double>::epsilon();
    while (end > 0) {
        for (int i = start; i < end; ++i)
            if (std::fabs(sub[i]) <= (std::fabs(diag[i]) + std::fabs(diag[i + 1])) * precision || std::fabs(sub[i]) <= considerAsZero)
                sub[i] = 0.0;
        while (end > 0 && sub[end - 1] == 0.0) end--;
        if (end <= 0) break;
        iter++;
        if (iter > maxIterations * n) break;
        start = end - 1;
        while (start > 0 && sub[start - 1] != 0.0) start--;
        // tridiagonal_qr_step
        double td = (diag[end - 1] - diag[end]) * 0.5;
        double e = sub[end - 1];
        double mu = diag[end];
        if (td == 0.0) mu -= std::fabs(e);
        else {
            double e2 = e * e;
            double h = positive_real_hypot(std::fabs(td), std::fabs(e));
            if (e2 == 0.0) mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
            else mu -= e2 / (td + (td > 0.0 ? h : -h));
        }
        double x = diag[start] - mu;
        double z = sub[start];
        for (int k = start; k < end; ++k) {
            Rot<double> rot = make_givens(x, z);
            double sdk = rot.s * diag[k] + rot.c * sub[k];
            double dkp1 = rot.s * sub[k] + rot.c * diag[k + 1];
            diag[k] = rot.c * (rot.c * diag[k] - rot.s * sub[k]) - rot.s * (rot.c * sub[k] - rot.s * diag[k + 1]);
            diag[k + 1] = rot.s * sdk + rot.c * dkp1;
            sub[k] = rot.c * sdk - rot.s * dkp1;
            if (k > start) sub[k - 1] = rot.c * sub[k - 1] - rot.s * z;
            x = sub[k];
            if (k < end - 1) {
                z = -rot.s * sub[k + 1];
                sub[k + 1] = rot.c * sub[k + 1];
            }
            apply_right<double, 3>(mat, k, k + 1, rot);  // q.applyOnTheRight(k,k+1,rot)
        }
    }
    bool ok = iter <= maxIterations * n;
    if (ok) {
        for (int i = 0; i < n - 1; ++i) {
            int kk = 0;
            double mn = diag[i];
            for (int t = 1; t < n - i; ++t)
                if (diag[i + t] < mn) { mn = diag[i + t]; kk = t; }
            if (kk > 0) {
                std::swap(diag[i], diag[kk + i]);
                for (int r = 0; r < 3; ++r) std::swap(mat(r, i), mat(r, kk + i));
            }
        }
    }
    for (int i = 0; i < 3; ++i) evals[i] = diag[i] * scale;
    evecs = mat;
    return ok;
}

// Matrix3d::inverse() (compute_inverse<MatrixType,ResultType,3>)
template <typename T> inline Mat<T, 3> inverse3(const Mat<T, 3>& m) {
    auto cof = [&](int i, int j) {
        int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return m(i1, j1) * m(i2, j2) - m(i1, j2) * m(i2, j1);
    };
    T c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    T det = c0 * m(0, 0) + c1 * m(1, 0) + c2 * m(2, 0);
    T invdet = T(1) / det;
    Mat<T, 3> r;
    r(0, 0) = c0 * invdet; r(0, 1) = c1 * invdet; r(0, 2) = c2 * invdet;
    r(1, 0) = cof(0, 1) * invdet; r(1, 1) = cof(1, 1) * invdet; r(1, 2) = cof(2, 1) * invdet;
    r(2, 0) = cof(0, 2) * invdet; r(2, 1) = cof(1, 2) * invdet; r(2, 2) = cof(2, 2) * invdet;
    return r;
}

}  // namespace e33
