// Host check: the f32 evaluation orders restated in ndt_pair.h / ndt_linalg.h against a transcription of the shipped
// libndt_omp.so's own instruction sequences (read as text with objdump -d, never run) into SSE intrinsics:
//   updateDerivatives<PointXYZI> 0x422a0-0x42968 with its callees
//     0x41a40 x_trans4 * c_inv4            (per column: mulps, then movhlps / addps / shufps $1 / addss)
//     0x42471 x_trans4.dot(x_trans4 * c_inv4)   (mulps + the same reduction)
//     0x37840 c_inv4 * point_gradient4     (per column: broadcast, mulps per c_inv4 column, addps in k order)
//     0x41970 x_trans4 * (c_inv4 * point_gradient4)
//     0x41ad0 point_gradient4^T * (c_inv4 * point_gradient4)
//     0x3cff0 x_trans4_x_c_inv4 * point_hessian_.block<4, 6>(4 i, 0)
//     exp: cvtss2sd, exp@plt, cvtsd2ss (0x424a4-0x424bc); the reject test, e_x_cov_x *= gauss_d1_ in double, the
//     gradient / Hessian updates as scalar mulss / addss / cvtss2sd / addsd (0x42620-0x42962)
//   computePointDerivatives<PointXYZI> 0x4b650 (j_ang * x4) and 0x4a650 (h_ang * x4 packets)
//   Transform::rotate<AngleAxisf> 0x3da70 (3x3 product, scalar mulss / addss)
// compared with pair_f32 and pair_pk (the device's pair arithmetic) and mat3_mul_f — every accumulated value equal
// (==: only the sign of an exact zero may differ) on random pairs, with and without the Hessian.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -msse2
#include <xmmintrin.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include "../../xchu_slam_amd/csrc/ndt_pair.h"
#include "../../xchu_slam_amd/csrc/ndt_linalg.h"

static const unsigned long long kTabBits[ndt::kExpTabLen] = {NDT_EXP2_64_TAB};
static double tab_d[ndt::kExpTabLen];

// movaps v -> t; movhlps v, t; addps t, v; movaps v -> t; shufps $1, v, t; addss t, v
static float predux(__m128 v) {
    __m128 t = _mm_movehl_ps(v, v);
    v = _mm_add_ps(v, t);
    t = _mm_shuffle_ps(v, v, 1);
    return _mm_cvtss_f32(_mm_add_ss(v, t));
}

struct Ref {  // the binary's operands, Eigen layouts (column-major)
    alignas(16) float x4[4];
    alignas(16) float c4[16];   // c_inv4
    alignas(16) float pg[24];   // point_gradient4 4x6
    alignas(16) float ph[144];  // point_hessian_ 24x6
};

// updateDerivatives as the binary evaluates it; g[6], H[36] (row-major (i, j)) accumulate, returns score_inc
static double update_derivatives_sse(const Ref& R, float gd2f, double d1, bool hess, double* g, double* H) {
    const __m128 x = _mm_load_ps(R.x4);
    alignas(16) float tmp[4];
    for (int j = 0; j < 4; ++j) tmp[j] = predux(_mm_mul_ps(_mm_load_ps(R.c4 + 4 * j), x));                   // 0x41a40
    const float dot = predux(_mm_mul_ps(_mm_load_ps(tmp), x));                                                  // 0x42471
    const float neg = -gd2f;
    const float arg = (dot * neg) * 0.5f;
    const float e = (float)std::exp((double)arg);                                                               // 0x424a4
    const float ed2 = gd2f * e;
    if (!(ed2 <= 1.f) || 0.f > ed2 || ed2 != ed2) return 0.0;
    const float e2 = (float)((double)ed2 * d1);
    alignas(16) float cpg[24];
    for (int c = 0; c < 6; ++c) {                                                                               // 0x37840
        __m128 a0 = _mm_mul_ps(_mm_load_ps(R.c4 + 0), _mm_set1_ps(R.pg[4 * c + 0]));
        __m128 a1 = _mm_mul_ps(_mm_load_ps(R.c4 + 4), _mm_set1_ps(R.pg[4 * c + 1]));
        __m128 a2 = _mm_mul_ps(_mm_load_ps(R.c4 + 8), _mm_set1_ps(R.pg[4 * c + 2]));
        __m128 a3 = _mm_mul_ps(_mm_load_ps(R.c4 + 12), _mm_set1_ps(R.pg[4 * c + 3]));
        _mm_store_ps(cpg + 4 * c, _mm_add_ps(a3, _mm_add_ps(a2, _mm_add_ps(a1, a0))));
    }
    float v[6];
    for (int j = 0; j < 6; ++j) v[j] = predux(_mm_mul_ps(_mm_load_ps(cpg + 4 * j), x));                       // 0x41970
    for (int j = 0; j < 6; ++j) g[j] += (double)(v[j] * e2);
    if (hess) {
        float Rm[36];  // Rm[row + 6 col] = pg col row . cpg col col (0x41ad0)
        for (int c = 0; c < 6; ++c)
            for (int r = 0; r < 6; ++r) Rm[r + 6 * c] = predux(_mm_mul_ps(_mm_load_ps(cpg + 4 * c), _mm_load_ps(R.pg + 4 * r)));
        const __m128 xc = _mm_load_ps(tmp);
        for (int i = 0; i < 6; ++i) {
            float ext[6];
            for (int j = 0; j < 6; ++j) ext[j] = predux(_mm_mul_ps(_mm_loadu_ps(R.ph + 24 * j + 4 * i), xc));  // 0x3cff0
            const float nv = neg * v[i];
            for (int j = 0; j < 6; ++j) {
                float t = v[j] * nv;
                t = t + ext[j];
                t = t + Rm[j + 6 * i];
                H[i * 6 + j] += (double)(t * e2);
            }
        }
    }
    return (double)(float)(-d1 * (double)e);
}

struct Pt {
    float xt[3], xj[8], xh[15];
};
struct Rec {
    double mean[3];
    float icov[9];
};

int main() {
    for (int i = 0; i < ndt::kExpTabLen; ++i) std::memcpy(&tab_d[i], &kTabBits[i], 8);
    std::mt19937_64 rng(17);
    std::normal_distribution<double> N(0.0, 1.0);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long bad = 0, accepted = 0;
    const int n = 300000;
    for (int s = 0; s < n; ++s) {
        // angle tables (computeAngleDerivatives: f64 entries narrowed to f32) and a point
        double p[6];
        for (double& a : p) a = U(rng) * ((s % 3 == 0) ? 3.1 : 0.3);
        const double cx = std::cos(p[3]), sx = std::sin(p[3]), cy = std::cos(p[4]), sy = std::sin(p[4]), cz = std::cos(p[5]),
                     sz = std::sin(p[5]);
        float jang[8][4] = {}, hang[16][4] = {};
        for (int r = 0; r < 23; ++r) {
            double o[3];
            ndt::angle_table_row(r, cx, sx, cy, sy, cz, sz, o);
            for (int c = 0; c < 3; ++c) (r < 8 ? jang[r][c] : hang[r - 8][c]) = (float)o[c];
        }
        const double scale = (s % 7 == 0) ? 1e-3 : ((s % 11 == 0) ? 300.0 : 60.0);
        const float x4[4] = {(float)(U(rng) * scale), (float)(U(rng) * scale), (float)(U(rng) * scale), 0.f};
        // the binary's point derivatives: j_ang * x4 (0x4b6bc) and h_ang * x4 (0x4a650), packets summed in k order
        float xj[8], xh[16];
        for (int r = 0; r < 8; ++r) xj[r] = ((jang[r][0] * x4[0] + jang[r][1] * x4[1]) + jang[r][2] * x4[2]) + jang[r][3] * x4[3];
        for (int r = 0; r < 16; ++r) xh[r] = ((hang[r][0] * x4[0] + hang[r][1] * x4[1]) + hang[r][2] * x4[2]) + hang[r][3] * x4[3];
        // the device's point_deriv (derivatives.hip): the same three products in the same order
        Pt t;
        for (int r = 0; r < 8; ++r) {
            float acc = jang[r][0] * x4[0];
            acc += jang[r][1] * x4[1];
            acc += jang[r][2] * x4[2];
            t.xj[r] = acc;
        }
        for (int r = 0; r < 15; ++r) {
            float acc = hang[r][0] * x4[0];
            acc += hang[r][1] * x4[1];
            acc += hang[r][2] * x4[2];
            t.xh[r] = acc;
        }
        // a voxel: mean near the transformed point, f32 inverse covariance (not exactly symmetric when s % 3 == 0)
        Rec rec;
        float xt3[3];
        for (int a = 0; a < 3; ++a) {
            xt3[a] = (float)(U(rng) * scale);
            rec.mean[a] = (double)xt3[a] + N(rng) * ((s % 5 == 0) ? 2.0 : 0.4);
            t.xt[a] = xt3[a];
        }
        double A[9], Cv[9];
        for (double& a : A) a = N(rng) * 0.3;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double acc = (i == j) ? 0.01 : 0.0;
                for (int k = 0; k < 3; ++k) acc += A[i * 3 + k] * A[j * 3 + k];
                Cv[i * 3 + j] = acc;
            }
        const double det = Cv[0] * (Cv[4] * Cv[8] - Cv[5] * Cv[7]) - Cv[1] * (Cv[3] * Cv[8] - Cv[5] * Cv[6]) + Cv[2] * (Cv[3] * Cv[7] - Cv[4] * Cv[6]);
        const double inv[9] = {(Cv[4] * Cv[8] - Cv[5] * Cv[7]) / det, (Cv[2] * Cv[7] - Cv[1] * Cv[8]) / det, (Cv[1] * Cv[5] - Cv[2] * Cv[4]) / det,
                               (Cv[5] * Cv[6] - Cv[3] * Cv[8]) / det, (Cv[0] * Cv[8] - Cv[2] * Cv[6]) / det, (Cv[2] * Cv[3] - Cv[0] * Cv[5]) / det,
                               (Cv[3] * Cv[7] - Cv[4] * Cv[6]) / det, (Cv[1] * Cv[6] - Cv[0] * Cv[7]) / det, (Cv[0] * Cv[4] - Cv[1] * Cv[3]) / det};
        for (int k = 0; k < 9; ++k) rec.icov[k] = (float)(inv[k] * ((s % 3 == 0) ? (1.0 + 1e-6 * U(rng)) : 1.0));
        // the binary's operands
        Ref R;
        std::memset(&R, 0, sizeof(R));
        for (int a = 0; a < 3; ++a) R.x4[a] = (float)((double)t.xt[a] - rec.mean[a]);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R.c4[i + 4 * j] = rec.icov[i * 3 + j];
        for (int a = 0; a < 3; ++a) R.pg[a + 4 * a] = 1.f;
        R.pg[1 + 4 * 3] = xj[0]; R.pg[2 + 4 * 3] = xj[1]; R.pg[0 + 4 * 4] = xj[2]; R.pg[1 + 4 * 4] = xj[3];
        R.pg[2 + 4 * 4] = xj[4]; R.pg[0 + 4 * 5] = xj[5]; R.pg[1 + 4 * 5] = xj[6]; R.pg[2 + 4 * 5] = xj[7];
        const bool hess = (s % 4) != 0;
        if (hess) {
            const float a[4] = {0, xh[0], xh[1], 0}, b[4] = {0, xh[2], xh[3], 0}, c[4] = {0, xh[4], xh[5], 0};
            const float d[4] = {xh[6], xh[7], xh[8], 0}, e[4] = {xh[9], xh[10], xh[11], 0}, f[4] = {xh[12], xh[13], xh[14], 0};
            for (int r = 0; r < 4; ++r) {
                R.ph[12 + r + 24 * 3] = a[r]; R.ph[16 + r + 24 * 3] = b[r]; R.ph[20 + r + 24 * 3] = c[r];
                R.ph[12 + r + 24 * 4] = b[r]; R.ph[16 + r + 24 * 4] = d[r]; R.ph[20 + r + 24 * 4] = e[r];
                R.ph[12 + r + 24 * 5] = c[r]; R.ph[16 + r + 24 * 5] = e[r]; R.ph[20 + r + 24 * 5] = f[r];
            }
        }
        const float gd2 = (s % 2) ? 0.4331230047f : 0.7563627303f;
        const double d1 = (s % 2) ? -2.2172252440 : -0.7044467358;
        const double init = (s % 9 == 0) ? 1.5 : 0.0;
        double ref[44], a[44], b[44];
        for (int k = 0; k < 44; ++k) ref[k] = a[k] = b[k] = init;
        ref[0] += update_derivatives_sse(R, gd2, d1, hess, ref + 1, ref + 7);
        for (int r = 0; r < 8; ++r)
            if (std::memcmp(&xj[r], &t.xj[r], 4) != 0 && !(xj[r] == t.xj[r])) ++bad;
        for (int r = 0; r < 15; ++r)
            if (!(xh[r] == t.xh[r])) ++bad;
        float pd[ndt::kPkTerms] __attribute__((aligned(8)));
        ndt::pk_terms(t.xj, t.xh, pd);
        ndt::pair_f32(t, rec, gd2, d1, hess, a, tab_d);
        ndt::pair_pk(t.xt, pd, rec, gd2, d1, hess, b, tab_d);
        if (a[0] != init) ++accepted;
        for (int k = 0; k < 43; ++k) {
            const bool same_a = (a[k] == ref[k]) || (std::isnan(a[k]) && std::isnan(ref[k]));
            const bool same_b = (b[k] == ref[k]) || (std::isnan(b[k]) && std::isnan(ref[k]));
            if (!same_a || !same_b) {
                if (bad < 8) std::printf("pair %d value %d: binary %.17g pair_f32 %.17g pair_pk %.17g\n", s, k, ref[k], a[k], b[k]);
                ++bad;
            }
        }
        // convertTransform's rotation: Transform::rotate (0x3da70) vs mat3_mul_f
        if (s % 8 == 0) {
            float M[9], B[9], C1[9], C2[9];
            for (int k = 0; k < 9; ++k) { M[k] = (float)U(rng); B[k] = (float)U(rng); }
            ndt::mat3_mul_f(M, B, C1);
            for (int j = 0; j < 3; ++j)
                for (int i = 0; i < 3; ++i) {
                    float t12 = M[i + 3] * B[1 + 3 * j];
                    const float t2 = M[i + 6] * B[2 + 3 * j];
                    t12 = t12 + t2;
                    const float t0 = M[i] * B[3 * j];
                    C2[i + 3 * j] = t0 + t12;
                }
            for (int k = 0; k < 9; ++k)
                if (!(C1[k] == C2[k])) ++bad;
        }
    }
    std::printf("pairs %d accepted %ld mismatched: %ld\n", n, accepted, bad);
    return bad ? 1 : 0;
}
