// ndt_linalg.h — small fixed-size linear algebra for the NDT path, callable on host and device.
//
// Semantics follow the Eigen 3.3 routines the reference calls (Eigen is a third-party dependency of
// /root/reference/xchu_mapping, not vendored; version inferred 3.3.x):
//   * SelfAdjointEigenSolver<Matrix3d> + Matrix3d::inverse  (voxel_grid_covariance_omp_impl.hpp:333-364)
//   * Transform<float,3,Affine>::rotation() polar decomposition + eulerAngles(0,1,2)  (ndt_omp_impl.hpp:96-104)
//   * AngleAxis composition of convertTransform (ndt_omp.h:210-229, ndt_omp_impl.hpp:138-143, 815-819)
//   * JacobiSVD<Matrix<double,6,6>>::solve (ndt_omp_impl.hpp:119-121): the device solver uses an LU (same solution
//     up to cond*eps; ndt_control.h lu6_solve_rows) whenever a condition bound proves Eigen's rank truncation
//     (sigma_i < 6*eps*sigma_max treated as zero) cannot apply (kCondLU below), else the two-sided Jacobi SVD here.
// All arithmetic is compiled with -ffp-contract=off so host and device round identically.
#pragma once
#include <math.h>
#include <float.h>
#include "ndt_libm.h"

#if defined(__HIPCC__)
#define NDT_HD __host__ __device__ inline
#else
#define NDT_HD inline
#endif

namespace ndt {

template <typename T> NDT_HD T tmax(T a, T b) { return a < b ? b : a; }
template <typename T> NDT_HD T tmin(T a, T b) { return b < a ? b : a; }
template <typename T> NDT_HD void tswap(T& a, T& b) { T t = a; a = b; b = t; }

template <typename T> struct Limits;
template <> struct Limits<float> {
    NDT_HD static float min() { return FLT_MIN; }
    NDT_HD static float eps() { return FLT_EPSILON; }
};
template <> struct Limits<double> {
    NDT_HD static double min() { return DBL_MIN; }
    NDT_HD static double eps() { return DBL_EPSILON; }
};

// ------------------------------------------------------------------------------------------------
// Two-sided Jacobi SVD of a square N x N matrix (column-major a[i + N*j]).
// ------------------------------------------------------------------------------------------------
template <typename T> struct JRot { T c, s; };

template <typename T, int N> NDT_HD void rot_rows(T* m, int p, int q, T c, T s) {
    for (int k = 0; k < N; ++k) {
        T xi = m[p + N * k], yi = m[q + N * k];
        m[p + N * k] = c * xi + s * yi;
        m[q + N * k] = -s * xi + c * yi;
    }
}
template <typename T, int N> NDT_HD void rot_cols(T* m, int p, int q, T c, T s) {
    // applyOnTheRight(p,q,j) rotates with j^T = (c, -s)
    const T st = -s;
    for (int k = 0; k < N; ++k) {
        T xi = m[k + N * p], yi = m[k + N * q];
        m[k + N * p] = c * xi + st * yi;
        m[k + N * q] = -st * xi + c * yi;
    }
}

template <typename T> NDT_HD JRot<T> jacobi_rotation(T x, T y, T z) {
    JRot<T> r;
    T deno = T(2) * fabs(y);
    if (deno < Limits<T>::min()) { r.c = T(1); r.s = T(0); return r; }
    T tau = (x - z) / deno;
    T w = sqrt(tau * tau + T(1));
    T t = (tau > T(0)) ? T(1) / (tau + w) : T(1) / (tau - w);
    T sign_t = t > T(0) ? T(1) : T(-1);
    T n = T(1) / sqrt(t * t + T(1));
    r.s = -sign_t * (y / fabs(y)) * fabs(t) * n;
    r.c = n;
    return r;
}

template <typename T, int N>
NDT_HD void svd_jacobi(const T* A, T* U, T* V, T* sv, int* nonzero) {
    T w[N * N];
    T scale = T(0);
    for (int k = 0; k < N * N; ++k) scale = tmax(scale, (T)fabs(A[k]));
    if (scale == T(0)) scale = T(1);
    for (int k = 0; k < N * N; ++k) w[k] = A[k] / scale;
    for (int k = 0; k < N * N; ++k) { U[k] = (k % (N + 1) == 0) ? T(1) : T(0); V[k] = U[k]; }
    const T tiny = Limits<T>::min();
    const T precision = T(2) * Limits<T>::eps();
    T maxDiag = T(0);
    for (int i = 0; i < N; ++i) maxDiag = tmax(maxDiag, (T)fabs(w[i + N * i]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
        finished = true;
        for (int p = 1; p < N; ++p)
            for (int q = 0; q < p; ++q) {
                T thr = tmax(tiny, precision * maxDiag);
                if (fabs(w[p + N * q]) > thr || fabs(w[q + N * p]) > thr) {
                    finished = false;
                    // real_2x2_jacobi_svd
                    T m00 = w[p + N * p], m01 = w[p + N * q], m10 = w[q + N * p], m11 = w[q + N * q];
                    T t = m00 + m11, d = m10 - m01;
                    JRot<T> r1;
                    if (fabs(d) < tiny) { r1.s = T(0); r1.c = T(1); }
                    else { T u = t / d; T tmp = sqrt(T(1) + u * u); r1.s = T(1) / tmp; r1.c = u / tmp; }
                    T n00 = r1.c * m00 + r1.s * m10, n01 = r1.c * m01 + r1.s * m11;
                    T n11 = -r1.s * m01 + r1.c * m11;
                    JRot<T> jr = jacobi_rotation<T>(n00, n01, n11);
                    const T oc = jr.c, os = -jr.s;
                    JRot<T> jl;
                    jl.c = r1.c * oc - r1.s * os;
                    jl.s = r1.c * os + r1.s * oc;
                    rot_rows<T, N>(w, p, q, jl.c, jl.s);
                    rot_cols<T, N>(U, p, q, jl.c, -jl.s);
                    rot_cols<T, N>(w, p, q, jr.c, jr.s);
                    rot_cols<T, N>(V, p, q, jr.c, jr.s);
                    maxDiag = tmax(maxDiag, tmax((T)fabs(w[p + N * p]), (T)fabs(w[q + N * q])));
                }
            }
    }
    for (int i = 0; i < N; ++i) {
        T a = w[i + N * i];
        sv[i] = fabs(a);
        if (a < T(0))
            for (int k = 0; k < N; ++k) U[k + N * i] = -U[k + N * i];
    }
    for (int i = 0; i < N; ++i) sv[i] *= scale;
    *nonzero = N;
    for (int i = 0; i < N; ++i) {
        int pos = i;
        T mx = sv[i];
        for (int k = i + 1; k < N; ++k)
            if (sv[k] > mx) { mx = sv[k]; pos = k; }
        if (mx == T(0)) { *nonzero = i; break; }
        if (pos != i) {
            tswap(sv[i], sv[pos]);
            for (int k = 0; k < N; ++k) { tswap(U[k + N * pos], U[k + N * i]); tswap(V[k + N * pos], V[k + N * i]); }
        }
    }
}

// JacobiSVD::solve with the default threshold
template <int N> NDT_HD void svd_solve(const double* A, const double* b, double* x) {
    double U[N * N], V[N * N], sv[N];
    int nz;
    svd_jacobi<double, N>(A, U, V, sv, &nz);
    double thr = tmax(sv[0] * (double(N) * DBL_EPSILON), DBL_MIN);
    int i = nz - 1;
    while (i >= 0 && sv[i] < thr) --i;
    int rank = i + 1;
    double tmp[N];
    for (int k = 0; k < rank; ++k) {
        double acc = 0.0;
        for (int r = 0; r < N; ++r) acc += U[r + N * k] * b[r];
        tmp[k] = (1.0 / sv[k]) * acc;
    }
    for (int r = 0; r < N; ++r) {
        double acc = 0.0;
        for (int k = 0; k < rank; ++k) acc += V[r + N * k] * tmp[k];
        x[r] = acc;
    }
}

// JacobiSVD's rank truncation (singular values < 6*eps*sigma_max treated as zero, Appendix A.8) can only change the
// Newton direction when cond_2(H) > 1/(6 eps) = 7.5e14.  kappa_1 = ||H||_1 ||H^-1||_1 bounds it: cond_2 <= 6 kappa_1.
// Below kCondLU (half of 7.5e14 / 6, margin for the rounding of the computed factors) the LU solution is the full-rank
// solution JacobiSVD computes too (same system, up to cond * eps); above it the solve goes to the Eigen-semantics SVD.
constexpr double kCondLU = 6.25e13;

// JacobiSVD<Matrix<double,6,6>>(H).solve(b) for an H stored row-major
NDT_HD void svd_solve6_rowmajor(const double* Hrow, const double* b, double* x) {
    double colmajor[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) colmajor[i + 6 * j] = Hrow[i * 6 + j];
    svd_solve<6>(colmajor, b, x);
}

// ------------------------------------------------------------------------------------------------
// cpu::SymmetricEigensolver3x3::compute (ndt_cpu backend, /root/reference/xchu_mapping/include/ndt_cpu/
// SymmetricEigenSolver.h:55-273, used by ndt_cpu's VoxelGrid::computeCentroidAndCovariance): closed-form eigenvalues of
// the max-scaled matrix (acos/cos of the half determinant), eigenvectors from cross products — restated operation for
// operation, including the header's quirks: d_k = r_k0^2 + r_k1^2 * r_k2^2 (a product where a sum is meant, :172-174),
// imax never becomes 2 (the second selection compares against the already updated maximum, :179-180), and a
// diagonal input returns its diagonal unsorted (:128-133).  A column-major, ev ascending unless diagonal, V column-major.
NDT_HD void aw_cross(const double* u, const double* v, double* o) {
    o[0] = u[1] * v[2] - u[2] * v[1];
    o[1] = u[2] * v[0] - u[0] * v[2];
    o[2] = u[0] * v[1] - u[1] * v[0];
}
NDT_HD void aw_sym_eigen3(const double* A, double* ev, double* V) {
    double a00 = A[0], a01 = A[3], a02 = A[6], a11 = A[4], a12 = A[7], a22 = A[8];
    const double max0 = (fabs(a00) > fabs(a01)) ? fabs(a00) : fabs(a01);
    const double max1 = (fabs(a02) > fabs(a11)) ? fabs(a02) : fabs(a11);
    const double max2 = (fabs(a12) > fabs(a22)) ? fabs(a12) : fabs(a22);
    double mabs = (max0 > max1) ? max0 : max1;
    mabs = (mabs > max2) ? mabs : max2;
    for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0 : 0.0;
    if (mabs == 0.0) {
        ev[0] = ev[1] = ev[2] = 0.0;
        return;
    }
    const double inv = 1.0 / mabs;
    a00 *= inv; a01 *= inv; a02 *= inv; a11 *= inv; a12 *= inv; a22 *= inv;
    const double norm = a01 * a01 + a02 * a02 + a12 * a12;
    if (norm > 0.0) {
        const double t3 = (a00 + a11 + a22) / 3.0;
        const double b00 = a00 - t3, b11 = a11 - t3, b22 = a22 - t3;
        const double denom = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2.0) / 6.0);
        const double c00 = b11 * b22 - a12 * a12;
        const double c01 = a01 * b22 - a12 * a02;
        const double c02 = a01 * a12 - b11 * a02;
        const double det = (b00 * c00 - a01 * c01 + a02 * c02) / (denom * denom * denom);
        double half = det * 0.5;
        half = (half > -1.0) ? half : -1.0;
        half = (half < 1.0) ? half : 1.0;
        const double angle = acos(half) / 3.0;
        const double beta2 = cos(angle) * 2.0;
        const double beta0 = cos(angle + 3.14159265358979323846 * 2.0 / 3.0) * 2.0;
        const double beta1 = -(beta0 + beta2);
        ev[0] = t3 + denom * beta0;
        ev[1] = t3 + denom * beta1;
        ev[2] = t3 + denom * beta2;
        const int i1 = 1;
        const int i0 = half >= 0.0 ? 2 : 0, i2 = half >= 0.0 ? 0 : 2;
        // computeEigenvector0 (:149-183)
        {
            const double e0 = ev[i0];
            const double r0[3] = {a00 - e0, a01, a02}, r1[3] = {a01, a11 - e0, a12}, r2[3] = {a02, a12, a22 - e0};
            double x0[3], x1[3], x2[3];
            aw_cross(r0, r1, x0);
            aw_cross(r0, r2, x1);
            aw_cross(r1, r2, x2);
            const double d0 = x0[0] * x0[0] + x0[1] * x0[1] * x0[2] * x0[2];
            const double d1 = x1[0] * x1[0] + x1[1] * x1[1] * x1[2] * x1[2];
            const double d2 = x2[0] * x2[0] + x2[1] * x2[1] * x2[2] * x2[2];
            double dmax = (d0 > d1) ? d0 : d1;
            int imax = (d0 > d1) ? 0 : 1;
            dmax = (d2 > dmax) ? d2 : dmax;
            imax = (d2 > dmax) ? 2 : imax;
            const double* xr = imax == 0 ? x0 : (imax == 1 ? x1 : x2);
            const double sq = sqrt(dmax);
            for (int r = 0; r < 3; ++r) V[r + 3 * i0] = xr[r] / sq;
        }
        // computeEigenvector1 (:185-239) with computeOrthogonalComplement (:253-264)
        {
            const double w[3] = {V[0 + 3 * i0], V[1 + 3 * i0], V[2 + 3 * i0]};
            const bool c = fabs(w[0]) > fabs(w[1]);
            const double il = c ? (1.0 / sqrt(w[0] * w[0] + w[2] * w[2])) : (1.0 / sqrt(w[1] * w[1] + w[2] * w[2]));
            double u[3] = {c ? -w[2] * il : 0.0, c ? 0.0 : w[2] * il, c ? w[0] * il : -w[1] * il};
            double v[3];
            aw_cross(w, u, v);
            const double e1 = ev[i1];
            const double au[3] = {(a00 - e1) * u[0] + a01 * u[1] + a02 * u[2], a01 * u[0] + (a11 - e1) * u[1] + a12 * u[2],
                                  a02 * u[0] + a12 * u[1] + (a22 - e1) * u[2]};
            const double av[3] = {(a00 - e1) * v[0] + a01 * v[1] + a02 * v[2], a01 * v[0] + (a11 - e1) * v[1] + a12 * v[2],
                                  a02 * v[0] + a12 * v[1] + (a22 - e1) * v[2]};
            const double m00 = u[0] * au[0] + u[1] * au[1] + u[2] * au[2];
            const double m01 = u[0] * av[0] + u[1] * av[1] + u[2] * av[2];
            const double m11 = v[0] * av[0] + v[1] * av[1] + v[2] * av[2];
            if (fabs(m00) > 0 || fabs(m01) > 0 || fabs(m11) > 0) {
                double um = (fabs(m00) >= fabs(m11)) ? m01 : m11;
                double vm = (fabs(m00) >= fabs(m11)) ? m00 : m01;
                const bool res = fabs(um) >= fabs(vm);
                double& large = res ? um : vm;
                double& small = res ? vm : um;
                small /= large;
                large = 1.0 / sqrt(1.0 + small * small);
                small *= large;
                for (int r = 0; r < 3; ++r) V[r + 3 * i1] = u[r] * um - v[r] * vm;
            } else {
                for (int r = 0; r < 3; ++r) V[r + 3 * i1] = u[r];
            }
        }
        // computeEigenvector2 (:266-273)
        {
            const double e0v[3] = {V[0 + 3 * i0], V[1 + 3 * i0], V[2 + 3 * i0]};
            const double e1v[3] = {V[0 + 3 * i1], V[1 + 3 * i1], V[2 + 3 * i1]};
            double o[3];
            aw_cross(e0v, e1v, o);
            for (int r = 0; r < 3; ++r) V[r + 3 * i2] = o[r];
        }
    } else {
        ev[0] = a00;
        ev[1] = a11;
        ev[2] = a22;
    }
    for (int k = 0; k < 3; ++k) ev[k] *= mabs;
}

// ------------------------------------------------------------------------------------------------
// SelfAdjointEigenSolver<Matrix3d>::compute (scaled, 3x3 tridiagonalisation, implicit QR, ascending)
// A column-major 3x3 (only the lower triangle is read).  evecs column-major.
// ------------------------------------------------------------------------------------------------
NDT_HD double pos_hypot(double x, double y) {
    double p = tmax(x, y);
    if (p == 0.0) return 0.0;
    double qp = tmin(y, x) / p;
    return p * sqrt(1.0 + qp * qp);
}

NDT_HD void givens(double p, double q, double* c, double* s) {
    if (q == 0.0) { *c = p < 0.0 ? -1.0 : 1.0; *s = 0.0; }
    else if (p == 0.0) { *c = 0.0; *s = q < 0.0 ? 1.0 : -1.0; }
    else if (fabs(p) > fabs(q)) {
        double t = q / p; double u = sqrt(1.0 + t * t); if (p < 0.0) u = -u;
        *c = 1.0 / u; *s = -t * (*c);
    } else {
        double t = p / q; double u = sqrt(1.0 + t * t); if (q < 0.0) u = -u;
        *s = -1.0 / u; *c = -t * (*s);
    }
}

// One implicit symmetric QR sweep (Wilkinson shift mu) over the window [S, E] of the 3x3 tridiagonal
// (d diagonal, e sub-diagonal) accumulating the rotations into Q, as Eigen's tridiagonal_qr_step.
template <int S, int E>
NDT_HD void qr_sweep3(double* d, double* e, double* Q, double mu) {
    double x = d[S] - mu, z = e[S];
#pragma unroll
    for (int k = S; k < E; ++k) {
        double c, s;
        givens(x, z, &c, &s);
        double sdk = s * d[k] + c * e[k];
        double dkp1 = s * e[k] + c * d[k + 1];
        d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
        d[k + 1] = s * sdk + c * dkp1;
        e[k] = c * sdk - s * dkp1;
        if (k > S) e[k - 1] = c * e[k - 1] - s * z;
        x = e[k];
        if (k < E - 1) { z = -s * e[k + 1]; e[k + 1] = c * e[k + 1]; }
        // Q.applyOnTheRight(k, k+1, rot): columns k, k+1 with (c, -s)
        for (int r = 0; r < 3; ++r) {
            double xi = Q[r + 3 * k], yi = Q[r + 3 * (k + 1)];
            Q[r + 3 * k] = c * xi + (-s) * yi;
            Q[r + 3 * (k + 1)] = -(-s) * xi + c * yi;
        }
    }
}

NDT_HD bool sym_eigen3(const double* A, double* ev, double* Q) {
    double m[9];
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) m[i + 3 * j] = (i >= j) ? A[i + 3 * j] : 0.0;
    double scale = 0.0;
    for (int k = 0; k < 9; ++k) scale = tmax(scale, fabs(m[k]));
    if (scale == 0.0) scale = 1.0;
    for (int j = 0; j < 3; ++j)
        for (int i = j; i < 3; ++i) m[i + 3 * j] /= scale;
    double d[3], e[2];
    d[0] = m[0];
    const double v1norm2 = m[2] * m[2];
    if (v1norm2 <= DBL_MIN) {
        d[1] = m[4]; d[2] = m[8]; e[0] = m[1]; e[1] = m[5];
        for (int k = 0; k < 9; ++k) Q[k] = (k % 4 == 0) ? 1.0 : 0.0;
    } else {
        double beta = sqrt(m[1] * m[1] + v1norm2);
        double invBeta = 1.0 / beta;
        double m01 = m[1] * invBeta, m02 = m[2] * invBeta;
        double q = 2.0 * m01 * m[5] + m02 * (m[8] - m[4]);
        d[1] = m[4] + m02 * q;
        d[2] = m[8] - m02 * q;
        e[0] = beta;
        e[1] = m[5] - m01 * q;
        Q[0] = 1; Q[3] = 0; Q[6] = 0;
        Q[1] = 0; Q[4] = m01; Q[7] = m02;
        Q[2] = 0; Q[5] = m02; Q[8] = -m01;
    }
    const int n = 3, maxIt = 30;
    int end = n - 1, start = 0, iter = 0;
    const double precision = 2.0 * DBL_EPSILON;
    // Every index below is a compile-time constant: the active window (start, end) of a 3x3 tridiagonal is
    // one of (0,2), (1,2), (0,1), and each has its own fully unrolled QR sweep (qr_sweep3), so the device code
    // has no dynamically indexed register arrays.  The operations are exactly those of the generic loop.
    while (end > 0) {
        if (start <= 0 && 0 < end)
            if (fabs(e[0]) <= (fabs(d[0]) + fabs(d[1])) * precision || fabs(e[0]) <= DBL_MIN) e[0] = 0.0;
        if (start <= 1 && 1 < end)
            if (fabs(e[1]) <= (fabs(d[1]) + fabs(d[2])) * precision || fabs(e[1]) <= DBL_MIN) e[1] = 0.0;
        if (end == 2 && e[1] == 0.0) end = 1;
        if (end == 1 && e[0] == 0.0) end = 0;
        if (end <= 0) break;
        iter++;
        if (iter > maxIt * n) break;
        start = (end == 2 && e[0] != 0.0) ? 0 : end - 1;
        const double dE1 = end == 2 ? d[1] : d[0], dE = end == 2 ? d[2] : d[1], eE1 = end == 2 ? e[1] : e[0];
        double td = (dE1 - dE) * 0.5;
        double ee = eE1;
        double mu = dE;
        if (td == 0.0) mu -= fabs(ee);
        else {
            double e2 = ee * ee;
            double h = pos_hypot(fabs(td), fabs(ee));
            if (e2 == 0.0) mu -= (ee / (td + (td > 0.0 ? 1.0 : -1.0))) * (ee / h);
            else mu -= e2 / (td + (td > 0.0 ? h : -h));
        }
        if (end == 2) {
            if (start == 0) qr_sweep3<0, 2>(d, e, Q, mu);
            else qr_sweep3<1, 2>(d, e, Q, mu);
        } else {
            qr_sweep3<0, 1>(d, e, Q, mu);
        }
    }
    bool ok = iter <= maxIt * n;
    if (ok) {
        // selection sort of the eigenvalues (ascending), swapping eigenvector columns; static indices
#pragma unroll
        for (int i = 0; i < n - 1; ++i) {
            int kk = 0;
            double mn = d[i];
#pragma unroll
            for (int t = 1; t < n - i; ++t)
                if (d[i + t] < mn) { mn = d[i + t]; kk = t; }
#pragma unroll
            for (int t = 1; t < n - i; ++t) {
                if (kk == t) {
                    tswap(d[i], d[t + i]);
                    for (int r = 0; r < 3; ++r) tswap(Q[r + 3 * i], Q[r + 3 * (t + i)]);
                }
            }
        }
    }
    for (int i = 0; i < 3; ++i) ev[i] = d[i] * scale;
    return ok;
}

// Matrix3::inverse() by cofactors (column-major in/out)
template <typename T> NDT_HD void inverse3(const T* m, T* r) {
#define NDT_M(i, j) m[(i) + 3 * (j)]
#define NDT_COF(i, j) (NDT_M(((i) + 1) % 3, ((j) + 1) % 3) * NDT_M(((i) + 2) % 3, ((j) + 2) % 3) - NDT_M(((i) + 1) % 3, ((j) + 2) % 3) * NDT_M(((i) + 2) % 3, ((j) + 1) % 3))
    T c0 = NDT_COF(0, 0), c1 = NDT_COF(1, 0), c2 = NDT_COF(2, 0);
    T det = c0 * NDT_M(0, 0) + c1 * NDT_M(1, 0) + c2 * NDT_M(2, 0);
    T invdet = T(1) / det;
    r[0 + 3 * 0] = c0 * invdet; r[0 + 3 * 1] = c1 * invdet; r[0 + 3 * 2] = c2 * invdet;
    r[1 + 3 * 0] = NDT_COF(0, 1) * invdet; r[1 + 3 * 1] = NDT_COF(1, 1) * invdet; r[1 + 3 * 2] = NDT_COF(2, 1) * invdet;
    r[2 + 3 * 0] = NDT_COF(0, 2) * invdet; r[2 + 3 * 1] = NDT_COF(1, 2) * invdet; r[2 + 3 * 2] = NDT_COF(2, 2) * invdet;
#undef NDT_COF
#undef NDT_M
}

// ------------------------------------------------------------------------------------------------
// Pose parameterisation
// ------------------------------------------------------------------------------------------------
// AngleAxis<float>(angle, unit axis a).toRotationMatrix(), column-major (libndt_omp.so 0x3d830).  sin / cos: the binary's
// sincosf, modelled as the correctly rounded f32 values (sinf_dr / cosf_dr, ndt_libm.h).
NDT_HD void angle_axis_sc(float s, float c, int a, float* R) {
    float ax[3] = {0.f, 0.f, 0.f};
    ax[a] = 1.f;
    const float sa0 = s * ax[0], sa1 = s * ax[1], sa2 = s * ax[2];
    const float c10 = (1.f - c) * ax[0], c11 = (1.f - c) * ax[1], c12 = (1.f - c) * ax[2];
    float t;
    t = c10 * ax[1]; R[0 + 3 * 1] = t - sa2; R[1 + 3 * 0] = t + sa2;
    t = c10 * ax[2]; R[0 + 3 * 2] = t + sa1; R[2 + 3 * 0] = t - sa1;
    t = c11 * ax[2]; R[1 + 3 * 2] = t - sa0; R[2 + 3 * 1] = t + sa0;
    R[0] = c10 * ax[0] + c; R[4] = c11 * ax[1] + c; R[8] = c12 * ax[2] + c;
}

NDT_HD void angle_axis_f(float angle, int a, float* R) { angle_axis_sc(ndt::sinf_dr(angle), ndt::cosf_dr(angle), a, R); }

// C = A * B (3x3 f32, column-major) as Transform::rotate evaluates it: Eigen's unrolled 3-term redux, a0 + (a1 + a2)
// (libndt_omp.so 0x3da70-0x3dc2b)
NDT_HD void mat3_mul_f(const float* A, const float* B, float* C) {
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i)
            C[i + 3 * j] = A[i + 0] * B[0 + 3 * j] + (A[i + 3] * B[1 + 3 * j] + A[i + 6] * B[2 + 3 * j]);
}

// convertTransform (ndt_omp.h:210-229): T = Translation3f(x) * AA(roll,X) * AA(pitch,Y) * AA(yaw,Z)
NDT_HD void convert_transform(const double* x, float* T) {
    float Rx[9], Ry[9], Rz[9], Rxy[9], R[9];
    angle_axis_f((float)x[3], 0, Rx);
    angle_axis_f((float)x[4], 1, Ry);
    angle_axis_f((float)x[5], 2, Rz);
    mat3_mul_f(Rx, Ry, Rxy);
    mat3_mul_f(Rxy, Rz, R);
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) T[i + 4 * j] = R[i + 3 * j];
    T[3] = 0.f; T[7] = 0.f; T[11] = 0.f;
    T[12] = (float)x[0]; T[13] = (float)x[1]; T[14] = (float)x[2]; T[15] = 1.f;
}

// computeAngleDerivatives (ndt_omp_impl.hpp:286-398): f32 tables narrowed from f64 expressions, and
// the f64 vectors of the double path.
NDT_HD void angle_tables(const double* p, float (*jang)[4], float (*hang)[4], double (*jd)[3], double (*hd)[3]) {
    double cx, cy, cz, sx, sy, sz;
    if (fabs(p[3]) < 10e-5) { cx = 1.0; sx = 0.0; } else { sincos(p[3], &sx, &cx); }
    if (fabs(p[4]) < 10e-5) { cy = 1.0; sy = 0.0; } else { sincos(p[4], &sy, &cy); }
    if (fabs(p[5]) < 10e-5) { cz = 1.0; sz = 0.0; } else { sincos(p[5], &sz, &cz); }
    const double J[8][3] = {
        {(-sx * sz + cx * sy * cz), (-sx * cz - cx * sy * sz), (-cx * cy)},
        {(cx * sz + sx * sy * cz), (cx * cz - sx * sy * sz), (-sx * cy)},
        {(-sy * cz), sy * sz, cy},
        {sx * cy * cz, (-sx * cy * sz), sx * sy},
        {(-cx * cy * cz), cx * cy * sz, (-cx * sy)},
        {(-cy * sz), (-cy * cz), 0},
        {(cx * cz - sx * sy * sz), (-cx * sz - sx * sy * cz), 0},
        {(sx * cz + cx * sy * sz), (cx * sy * cz - sx * sz), 0}};
    const double Hh[15][3] = {
        {(-cx * sz - sx * sy * cz), (-cx * cz + sx * sy * sz), sx * cy},
        {(-sx * sz + cx * sy * cz), (-cx * sy * sz - sx * cz), (-cx * cy)},
        {(cx * cy * cz), (-cx * cy * sz), (cx * sy)},
        {(sx * cy * cz), (-sx * cy * sz), (sx * sy)},
        {(-sx * cz - cx * sy * sz), (sx * sz - cx * sy * cz), 0},
        {(cx * cz - sx * sy * sz), (-sx * sy * cz - cx * sz), 0},
        {(-cy * cz), (cy * sz), (sy)},
        {(-sx * sy * cz), (sx * sy * sz), (sx * cy)},
        {(cx * sy * cz), (-cx * sy * sz), (-cx * cy)},
        {(sy * sz), (sy * cz), 0},
        {(-sx * cy * sz), (-sx * cy * cz), 0},
        {(cx * cy * sz), (cx * cy * cz), 0},
        {(-cy * cz), (cy * sz), 0},
        {(-cx * sz - sx * sy * cz), (-cx * cz + sx * sy * sz), 0},
        {(-sx * sz + cx * sy * cz), (-cx * sy * sz - sx * cz), 0}};
    for (int r = 0; r < 8; ++r) {
        for (int c = 0; c < 3; ++c) { jang[r][c] = (float)J[r][c]; jd[r][c] = J[r][c]; }
        jang[r][3] = 0.f;
    }
    for (int r = 0; r < 15; ++r) {
        for (int c = 0; c < 3; ++c) { hang[r][c] = (float)Hh[r][c]; hd[r][c] = Hh[r][c]; }
        hang[r][3] = 0.f;
    }
    for (int c = 0; c < 4; ++c) hang[15][c] = 0.f;
}

// One row of the angle tables: rows 0-7 = j_ang a..h (eq. 6.19), rows 8-22 = h_ang a2..f3 (eq. 6.21).
NDT_HD void angle_table_row(int r, double cx, double sx, double cy, double sy, double cz, double sz, double* o) {
    switch (r) {
        case 0: o[0] = (-sx * sz + cx * sy * cz); o[1] = (-sx * cz - cx * sy * sz); o[2] = (-cx * cy); break;
        case 1: o[0] = (cx * sz + sx * sy * cz); o[1] = (cx * cz - sx * sy * sz); o[2] = (-sx * cy); break;
        case 2: o[0] = (-sy * cz); o[1] = sy * sz; o[2] = cy; break;
        case 3: o[0] = sx * cy * cz; o[1] = (-sx * cy * sz); o[2] = sx * sy; break;
        case 4: o[0] = (-cx * cy * cz); o[1] = cx * cy * sz; o[2] = (-cx * sy); break;
        case 5: o[0] = (-cy * sz); o[1] = (-cy * cz); o[2] = 0; break;
        case 6: o[0] = (cx * cz - sx * sy * sz); o[1] = (-cx * sz - sx * sy * cz); o[2] = 0; break;
        case 7: o[0] = (sx * cz + cx * sy * sz); o[1] = (cx * sy * cz - sx * sz); o[2] = 0; break;
        case 8: o[0] = (-cx * sz - sx * sy * cz); o[1] = (-cx * cz + sx * sy * sz); o[2] = sx * cy; break;
        case 9: o[0] = (-sx * sz + cx * sy * cz); o[1] = (-cx * sy * sz - sx * cz); o[2] = (-cx * cy); break;
        case 10: o[0] = (cx * cy * cz); o[1] = (-cx * cy * sz); o[2] = (cx * sy); break;
        case 11: o[0] = (sx * cy * cz); o[1] = (-sx * cy * sz); o[2] = (sx * sy); break;
        case 12: o[0] = (-sx * cz - cx * sy * sz); o[1] = (sx * sz - cx * sy * cz); o[2] = 0; break;
        case 13: o[0] = (cx * cz - sx * sy * sz); o[1] = (-sx * sy * cz - cx * sz); o[2] = 0; break;
        case 14: o[0] = (-cy * cz); o[1] = (cy * sz); o[2] = (sy); break;
        case 15: o[0] = (-sx * sy * cz); o[1] = (sx * sy * sz); o[2] = (sx * cy); break;
        case 16: o[0] = (cx * sy * cz); o[1] = (-cx * sy * sz); o[2] = (-cx * cy); break;
        case 17: o[0] = (sy * sz); o[1] = (sy * cz); o[2] = 0; break;
        case 18: o[0] = (-sx * cy * sz); o[1] = (-sx * cy * cz); o[2] = 0; break;
        case 19: o[0] = (cx * cy * sz); o[1] = (cx * cy * cz); o[2] = 0; break;
        case 20: o[0] = (-cy * cz); o[1] = (cy * sz); o[2] = 0; break;
        case 21: o[0] = (-cx * sz - sx * sy * cz); o[1] = (-cx * cz + sx * sy * sz); o[2] = 0; break;
        default: o[0] = (-sx * sz + cx * sy * cz); o[1] = (-cx * sy * sz - sx * cz); o[2] = 0; break;
    }
}

// The 69 entries of angle_table_row (rows 0..22 x 3) as data, so that every entry can be evaluated by its own
// lane without divergence.  Each entry is ((s1*v[a])*v[b])*v[c] [+ ((s2*v[d])*v[e])*v[f]] over
// v = {1, sx, cx, sy, cy, sz, cz, 0}: exactly the operations and association order of the expressions above
// (x*1 is exact, a - b*c*d == a + ((-b)*c)*d, (-a)*b == -(a*b) in round-to-nearest).
// Packed as bits: [2:0] a, [5:3] b, [8:6] c, [9] s1 negative, [12:10] d, [15:13] e, [18:16] f, [19] s2 negative,
// [20] second product present.
enum : unsigned char { TV_1 = 0, TV_SX = 1, TV_CX = 2, TV_SY = 3, TV_CY = 4, TV_SZ = 5, TV_CZ = 6, TV_0 = 7 };
#define NDT_TE1(n1, a, b, c) ((unsigned)(a) | ((unsigned)(b) << 3) | ((unsigned)(c) << 6) | ((unsigned)(n1) << 9))
#define NDT_TE2(n1, a, b, c, n2, d, e, f) \
    (NDT_TE1(n1, a, b, c) | ((unsigned)(d) << 10) | ((unsigned)(e) << 13) | ((unsigned)(f) << 16) | ((unsigned)(n2) << 19) | (1u << 20))
#define NDT_ANGLE_TABLE_CODE                                                                                                         \
    {NDT_TE2(1, TV_SX, TV_SZ, TV_1, 0, TV_CX, TV_SY, TV_CZ), NDT_TE2(1, TV_SX, TV_CZ, TV_1, 1, TV_CX, TV_SY, TV_SZ),                  \
     NDT_TE1(1, TV_CX, TV_CY, TV_1),                                                                                                 \
     NDT_TE2(0, TV_CX, TV_SZ, TV_1, 0, TV_SX, TV_SY, TV_CZ), NDT_TE2(0, TV_CX, TV_CZ, TV_1, 1, TV_SX, TV_SY, TV_SZ),                  \
     NDT_TE1(1, TV_SX, TV_CY, TV_1),                                                                                                 \
     NDT_TE1(1, TV_SY, TV_CZ, TV_1), NDT_TE1(0, TV_SY, TV_SZ, TV_1), NDT_TE1(0, TV_CY, TV_1, TV_1),                                   \
     NDT_TE1(0, TV_SX, TV_CY, TV_CZ), NDT_TE1(1, TV_SX, TV_CY, TV_SZ), NDT_TE1(0, TV_SX, TV_SY, TV_1),                               \
     NDT_TE1(1, TV_CX, TV_CY, TV_CZ), NDT_TE1(0, TV_CX, TV_CY, TV_SZ), NDT_TE1(1, TV_CX, TV_SY, TV_1),                               \
     NDT_TE1(1, TV_CY, TV_SZ, TV_1), NDT_TE1(1, TV_CY, TV_CZ, TV_1), NDT_TE1(0, TV_0, TV_1, TV_1),                                   \
     NDT_TE2(0, TV_CX, TV_CZ, TV_1, 1, TV_SX, TV_SY, TV_SZ), NDT_TE2(1, TV_CX, TV_SZ, TV_1, 1, TV_SX, TV_SY, TV_CZ),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1),                                                                                                   \
     NDT_TE2(0, TV_SX, TV_CZ, TV_1, 0, TV_CX, TV_SY, TV_SZ), NDT_TE2(0, TV_CX, TV_SY, TV_CZ, 1, TV_SX, TV_SZ, TV_1),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1),                                                                                                   \
     NDT_TE2(1, TV_CX, TV_SZ, TV_1, 1, TV_SX, TV_SY, TV_CZ), NDT_TE2(1, TV_CX, TV_CZ, TV_1, 0, TV_SX, TV_SY, TV_SZ),                  \
     NDT_TE1(0, TV_SX, TV_CY, TV_1),                                                                                                 \
     NDT_TE2(1, TV_SX, TV_SZ, TV_1, 0, TV_CX, TV_SY, TV_CZ), NDT_TE2(1, TV_CX, TV_SY, TV_SZ, 1, TV_SX, TV_CZ, TV_1),                  \
     NDT_TE1(1, TV_CX, TV_CY, TV_1),                                                                                                 \
     NDT_TE1(0, TV_CX, TV_CY, TV_CZ), NDT_TE1(1, TV_CX, TV_CY, TV_SZ), NDT_TE1(0, TV_CX, TV_SY, TV_1),                               \
     NDT_TE1(0, TV_SX, TV_CY, TV_CZ), NDT_TE1(1, TV_SX, TV_CY, TV_SZ), NDT_TE1(0, TV_SX, TV_SY, TV_1),                               \
     NDT_TE2(1, TV_SX, TV_CZ, TV_1, 1, TV_CX, TV_SY, TV_SZ), NDT_TE2(0, TV_SX, TV_SZ, TV_1, 1, TV_CX, TV_SY, TV_CZ),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1),                                                                                                   \
     NDT_TE2(0, TV_CX, TV_CZ, TV_1, 1, TV_SX, TV_SY, TV_SZ), NDT_TE2(1, TV_SX, TV_SY, TV_CZ, 1, TV_CX, TV_SZ, TV_1),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1),                                                                                                   \
     NDT_TE1(1, TV_CY, TV_CZ, TV_1), NDT_TE1(0, TV_CY, TV_SZ, TV_1), NDT_TE1(0, TV_SY, TV_1, TV_1),                                   \
     NDT_TE1(1, TV_SX, TV_SY, TV_CZ), NDT_TE1(0, TV_SX, TV_SY, TV_SZ), NDT_TE1(0, TV_SX, TV_CY, TV_1),                               \
     NDT_TE1(0, TV_CX, TV_SY, TV_CZ), NDT_TE1(1, TV_CX, TV_SY, TV_SZ), NDT_TE1(1, TV_CX, TV_CY, TV_1),                               \
     NDT_TE1(0, TV_SY, TV_SZ, TV_1), NDT_TE1(0, TV_SY, TV_CZ, TV_1), NDT_TE1(0, TV_0, TV_1, TV_1),                                   \
     NDT_TE1(1, TV_SX, TV_CY, TV_SZ), NDT_TE1(1, TV_SX, TV_CY, TV_CZ), NDT_TE1(0, TV_0, TV_1, TV_1),                                 \
     NDT_TE1(0, TV_CX, TV_CY, TV_SZ), NDT_TE1(0, TV_CX, TV_CY, TV_CZ), NDT_TE1(0, TV_0, TV_1, TV_1),                                 \
     NDT_TE1(1, TV_CY, TV_CZ, TV_1), NDT_TE1(0, TV_CY, TV_SZ, TV_1), NDT_TE1(0, TV_0, TV_1, TV_1),                                   \
     NDT_TE2(1, TV_CX, TV_SZ, TV_1, 1, TV_SX, TV_SY, TV_CZ), NDT_TE2(1, TV_CX, TV_CZ, TV_1, 0, TV_SX, TV_SY, TV_SZ),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1),                                                                                                   \
     NDT_TE2(1, TV_SX, TV_SZ, TV_1, 0, TV_CX, TV_SY, TV_CZ), NDT_TE2(1, TV_CX, TV_SY, TV_SZ, 1, TV_SX, TV_CZ, TV_1),                  \
     NDT_TE1(0, TV_0, TV_1, TV_1)}

// Entry k (= row*3 + col) of the angle tables from its code word.
NDT_HD double angle_table_entry(unsigned code, double sx, double cx, double sy, double cy, double sz, double cz) {
    const double v[8] = {1.0, sx, cx, sy, cy, sz, cz, 0.0};
    double a = v[code & 7];
    if (code & (1u << 9)) a = -a;
    double r = (a * v[(code >> 3) & 7]) * v[(code >> 6) & 7];
    if (code & (1u << 20)) {
        double d = v[(code >> 10) & 7];
        if (code & (1u << 19)) d = -d;
        r = r + (d * v[(code >> 13) & 7]) * v[(code >> 16) & 7];
    }
    return r;
}

// Transform<float,3,Affine>::rotation() (polar decomposition via JacobiSVD<Matrix3f>), column-major
NDT_HD void polar_rotation_f(const float* L, float* R) {
    float U[9], V[9], sv[3];
    int nz;
    svd_jacobi<float, 3>(L, U, V, sv, &nz);
    // U * V^T: entries a0 + (a1 + a2) (libndt_omp.so 0x46190)
    float UVt[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) UVt[i + 3 * j] = U[i] * V[j] + (U[i + 3] * V[j + 3] + U[i + 6] * V[j + 6]);
#define NDT_H(a, b, c) (UVt[0 + 3 * (a)] * (UVt[1 + 3 * (b)] * UVt[2 + 3 * (c)] - UVt[1 + 3 * (c)] * UVt[2 + 3 * (b)]))
    float x = NDT_H(0, 1, 2) - NDT_H(1, 0, 2) + NDT_H(2, 0, 1);
#undef NDT_H
    for (int i = 0; i < 3; ++i) U[i] /= x;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i + 3 * j] = U[i] * V[j] + (U[i + 3] * V[j + 3] + U[i + 6] * V[j + 6]);
}

// MatrixBase<Matrix3f>::eulerAngles(0,1,2) (Eigen 3.3, includes the +-pi branch on the first angle)
NDT_HD void euler012_f(const float* m, float* res) {
#define NDT_C(i, j) m[(i) + 3 * (j)]
    res[0] = atan2f(NDT_C(1, 2), NDT_C(2, 2));
    float c2 = sqrtf(NDT_C(0, 0) * NDT_C(0, 0) + NDT_C(0, 1) * NDT_C(0, 1));
    if (res[0] > 0.f) {
        res[0] -= 3.14159265358979323846f;
        res[1] = atan2f(-NDT_C(0, 2), -c2);
    } else {
        res[1] = atan2f(-NDT_C(0, 2), c2);
    }
    float s1 = ndt::sinf_dr(res[0]), c1 = ndt::cosf_dr(res[0]);  // sincosf at 0x3b4e1 (model: ndt_libm.h)
    res[2] = atan2f(s1 * NDT_C(2, 0) - c1 * NDT_C(1, 0), c1 * NDT_C(1, 1) - s1 * NDT_C(2, 1));
    res[0] = -res[0]; res[1] = -res[1]; res[2] = -res[2];
#undef NDT_C
}

// Gaussian fitting constants (eq. 6.8; ndt_omp_impl.hpp:80-87)
NDT_HD void gauss_constants(double outlier_ratio, float resolution, double* d1, double* d2, double* d3) {
    double c1 = 10.0 * (1 - outlier_ratio);
    double c2 = outlier_ratio / pow((double)resolution, 3);
    *d3 = -log(c2);
    *d1 = -log(c1 + c2) - *d3;
    *d2 = -2 * log((-log(c1 * exp(-0.5) + c2) - *d3) / *d1);
}

}  // namespace ndt
