// Host check: the data-driven angle-table evaluator (angle_table_entry, one lane per entry on the device) against
// angle_table_row (computeAngleDerivatives, ndt_omp_impl.hpp:286-398), bit for bit, on random angles.
#include <cstdio>
#include <cstring>
#include <cmath>
#include <random>
#include "../../xchu_slam_amd/csrc/ndt_linalg.h"

int main() {
    using namespace ndt;
    static const unsigned code[69] = NDT_ANGLE_TABLE_CODE;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-3.2, 3.2);
    long bad = 0;
    for (int s = 0; s < 200000; ++s) {
        double a[3];
        for (int k = 0; k < 3; ++k) a[k] = (s % 5 == 0) ? 0.0 : U(rng) * ((s % 3) ? 1.0 : 1e-3);
        double sx = std::sin(a[0]), cx = std::cos(a[0]), sy = std::sin(a[1]), cy = std::cos(a[1]), sz = std::sin(a[2]), cz = std::cos(a[2]);
        for (int r = 0; r < 23; ++r) {
            double o[3];
            ndt::angle_table_row(r, cx, sx, cy, sy, cz, sz, o);
            for (int c = 0; c < 3; ++c) {
                const double e = ndt::angle_table_entry(code[r * 3 + c], sx, cx, sy, cy, sz, cz);
                if (std::memcmp(&e, &o[c], sizeof(double)) != 0) {
                    if (bad < 5) std::printf("row %d col %d: %.17g vs %.17g\n", r, c, e, o[c]);
                    ++bad;
                }
            }
        }
    }
    std::printf("angle table entries mismatched: %ld\n", bad);
    return bad ? 1 : 0;
}
