// Host check: pair_pk (the pair arithmetic issued as packed f32 pairs) against pair_f32 (one f32 operation per reference
// operation, ndt_omp_impl.hpp:491-548) — every accumulated value equal (==; only the sign of an exact zero may differ),
// on random pairs with and without the Hessian.  Build: g++ -O2 -std=c++17 -ffp-contract=off.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include "../../xchu_slam_amd/csrc/ndt_pair.h"

struct Pt {
    float xt[3], xj[8], xh[15];
};
struct Rec {
    double mean[3];
    float icov[9];
};

static const unsigned long long kTabBits[ndt::kExpTabLen] = {NDT_EXP2_64_TAB};
static double kTab[ndt::kExpTabLen];

int main() {
    for (int i = 0; i < ndt::kExpTabLen; ++i) std::memcpy(&kTab[i], &kTabBits[i], 8);
    std::mt19937_64 rng(11);
    std::normal_distribution<double> N(0.0, 1.0);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    long bad = 0, accepted = 0;
    const int n = 400000;
    for (int s = 0; s < n; ++s) {
        Pt t;
        Rec r;
        const double scale = (s % 7 == 0) ? 1e-3 : ((s % 11 == 0) ? 300.0 : 60.0);
        for (int a = 0; a < 3; ++a) {
            t.xt[a] = (float)(U(rng) * scale);
            r.mean[a] = (double)t.xt[a] + N(rng) * ((s % 5 == 0) ? 2.0 : 0.4);
        }
        // icov: inverse of an SPD covariance (row-major, f32; not exactly symmetric when s % 3 == 0)
        double A[9];
        for (double& x : A) x = N(rng) * 0.3;
        double Cv[9];
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
        for (int k = 0; k < 9; ++k) r.icov[k] = (float)(inv[k] * ((s % 3 == 0) ? (1.0 + 1e-6 * U(rng)) : 1.0));
        for (float& x : t.xj) x = (float)(U(rng) * scale);
        for (float& x : t.xh) x = (float)(U(rng) * scale);
        if (s % 13 == 0) t.xh[3] = 0.f;
        const bool hess = (s % 4) != 0;
        float pd[ndt::kPkTerms] __attribute__((aligned(8)));
        ndt::pk_terms(t.xj, t.xh, pd);
        const float gd2 = (s % 2) ? 0.4331230047f : 0.7563627303f;
        const double d1 = (s % 2) ? -2.2172252440 : -0.7044467358;
        double a[44], b[44];
        for (int k = 0; k < 44; ++k) a[k] = b[k] = (s % 9 == 0) ? 1.5 : 0.0;
        ndt::pair_f32(t, r, gd2, d1, hess, a, kTab);
        ndt::pair_pk(t.xt, pd, r, gd2, d1, hess, b, kTab);
        if (a[0] != ((s % 9 == 0) ? 1.5 : 0.0)) ++accepted;
        for (int k = 0; k < 44; ++k) {
            const bool same = (a[k] == b[k]) || (std::isnan(a[k]) && std::isnan(b[k]));
            if (!same) {
                if (bad < 8) std::printf("pair %d value %d: %.17g vs %.17g\n", s, k, a[k], b[k]);
                ++bad;
            }
        }
    }
    std::printf("pairs %d accepted %ld mismatched: %ld\n", n, accepted, bad);
    return bad ? 1 : 0;
}
