// Host check: the device's restatements of glibc's libm (xchu_slam_amd/csrc/ndt_libm.h) against this host's glibc —
// the functions the reference calls: expf (std::exp(float), ndt_omp_impl.hpp:507) and sinf / cosf (Eigen::AngleAxisf in
// convertTransform, ndt_omp.h:210-229) — bit for bit on every STRIDE-th f32 bit pattern (argument; 1 = all 2^32, run once:
// 0 of 4,278,190,082 non-NaN inputs differ for expf, 0 of 2,246,049,792 with |x| < 120 for sinf and cosf), plus every
// pattern of [-2, 0] for expf (the pass's range) and of [-0.1, 0.1] for sinf / cosf (the angles of a Newton step).
// Build: g++ -O2 -std=c++17 -ffp-contract=off -fopenmp.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include "../../xchu_slam_amd/csrc/ndt_libm.h"

static const unsigned long long kTab[ndt::kExp2fTabLen] = {NDT_EXP2F_TAB};

template <typename F>
static long check(const char* name, unsigned long long lo, unsigned long long hi, unsigned long long stride, F accept, long* n_out) {
    long bad = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(static)
    for (long long u = (long long)lo; u < (long long)hi; u += (long long)stride) {
        const unsigned b = (unsigned)u;
        float x;
        std::memcpy(&x, &b, 4);
        if (x != x || !accept(x)) continue;
        ++n;
        float g, v;
        if (name[0] == 'e') { g = expf(x); v = ndt::exp_f(x, kTab); }
        else if (name[0] == 's') { g = sinf(x); v = ndt::sinf_r(x); }
        else { g = cosf(x); v = ndt::cosf_r(x); }
        if (std::memcmp(&g, &v, 4) != 0) {
            ++bad;
            if (bad < 4) std::printf("%s x=%a glibc %a restated %a\n", name, x, g, v);
        }
    }
    *n_out += n;
    return bad;
}

int main(int argc, char** argv) {
    const unsigned long long stride = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 7;
    auto all = [](float) { return true; };
    auto trig = [](float x) { return std::fabs(x) < 120.f; };
    long n = 0, bad = 0;
    bad += check("expf", 0, 1ull << 32, stride, all, &n);
    bad += check("expf", 0x80000000ull, 0xc0000001ull, 1, all, &n);  // [-2, -0]
    for (const char* f : {"sinf", "cosf"}) {
        bad += check(f, 0, 1ull << 32, stride, trig, &n);
        bad += check(f, 0, 0x3dcccccdull, 1, trig, &n);               // [0, 0.1]
        bad += check(f, 0x80000000ull, 0xbdcccccdull, 1, trig, &n);   // [-0.1, -0]
    }
    std::printf("inputs %ld mismatched: %ld\n", n, bad);
    return bad ? 1 : 0;
}
