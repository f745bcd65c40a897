// Host check of ndt_libm.h against the semantics of the shipped libndt_omp.so (read as text, never run):
//   exp_dr(x)  == RN_f32(RN_f64(e^x))  — updateDerivatives' (float)exp((double)x) (0x424a4-0x424bc) with glibc 2.23's
//                 correctly rounded double exp;
//   sinf_dr / cosf_dr == RN_f32(sin x) / RN_f32(cos x) for |x| < 120 — the model of the binary's sincosf (unpinned);
//   sincosf_dr2 (both at once) == sinf_dr / cosf_dr bit for bit.
// Truth: this host's glibc double function G (error < 1 ulp) decides wherever every double within 3 ulp of G rounds to
// the same f32; otherwise libquadmath (expq / sinq / cosq, 113-bit) rounded to double, then to f32.  Also reports how
// often the oracle's own expression ((float)std::exp((double)x), tests' oracle exp_mode 1) differs from the truth.
// Argument: STRIDE over the 2^32 f32 bit patterns (1 = exhaustive), plus every 7th pattern of [-2, 0] (exp) and of
// [-0.1, 0.1] (sin / cos), the ranges the pass and a Newton step live in.
// Build: g++ -O2 -std=c++17 -ffp-contract=off -fopenmp libm_check.cpp -lquadmath
#include <quadmath.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../xchu_slam_amd/csrc/ndt_libm.h"

static const unsigned long long kTabBits[ndt::kExpTabLen] = {NDT_EXP2_64_TAB};

static double up(double d, int k) { for (int i = 0; i < k; ++i) d = std::nextafter(d, INFINITY); return d; }
static double dn(double d, int k) { for (int i = 0; i < k; ++i) d = std::nextafter(d, -INFINITY); return d; }

// fn: 0 exp, 1 sin, 2 cos
static float truth(int fn, float x, long* slow) {
    const double xd = x;
    const double g = fn == 0 ? std::exp(xd) : (fn == 1 ? std::sin(xd) : std::cos(xd));
    if (std::isfinite(g)) {
        const float a = (float)dn(g, 3), b = (float)up(g, 3);
        if (a == b) return (float)g;  // (== : the bracket around an exact 0 spans -0 .. +0)
    } else if (std::isinf(g) && fn == 0) {
        return (float)g;  // e^x > DBL_MAX: +inf either way
    }
    ++*slow;
    const __float128 q = fn == 0 ? expq((__float128)xd) : (fn == 1 ? sinq((__float128)xd) : cosq((__float128)xd));
    return (float)(double)q;
}

static double tab_d[ndt::kExpTabLen];

static long check(int fn, unsigned long long lo, unsigned long long hi, unsigned long long stride, long* n_out, long* slow_out,
                  long* oracle_bad) {
    long bad = 0, n = 0, slow = 0, obad = 0;
#pragma omp parallel for reduction(+ : bad, n, slow, obad) schedule(dynamic, 65536)
    for (long long u = (long long)lo; u < (long long)hi; u += (long long)stride) {
        const unsigned b = (unsigned)u;
        float x;
        std::memcpy(&x, &b, 4);
        if (x != x) continue;
        if (fn != 0 && !(std::fabs(x) < 120.f)) continue;
        ++n;
        const float t = truth(fn, x, &slow);
        float v = fn == 0 ? ndt::exp_dr(x, tab_d) : ndt::sincosf_dr(x, fn == 2);
        if (fn != 0) {
            // the joint evaluation (sincosf_dr2, the align tail's) must give the bits of the single calls
            float js, jc;
            ndt::sincosf_dr2(x, &js, &jc);
            const float j = fn == 1 ? js : jc;
            if (std::memcmp(&j, &v, 4) != 0) v = -v * 3.f + 1.f;  // counted as a mismatch below
        }
        const double xd = x;
        const float o = (float)(fn == 0 ? std::exp(xd) : (fn == 1 ? std::sin(xd) : std::cos(xd)));
        if (std::memcmp(&t, &v, 4) != 0) {
            ++bad;
            if (bad < 6) std::printf("fn %d x=%a truth %a restated %a\n", fn, x, t, v);
        }
        if (std::memcmp(&t, &o, 4) != 0) ++obad;
    }
    *n_out += n;
    *slow_out += slow;
    *oracle_bad += obad;
    return bad;
}

int main(int argc, char** argv) {
    for (int i = 0; i < ndt::kExpTabLen; ++i) std::memcpy(&tab_d[i], &kTabBits[i], 8);
    const unsigned long long stride = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 61;
    const char* names[3] = {"exp", "sin", "cos"};
    long total_bad = 0;
    for (int fn = 0; fn < 3; ++fn) {
        long n = 0, slow = 0, obad = 0, bad = 0;
        bad += check(fn, 0, 1ull << 32, stride, &n, &slow, &obad);
        if (fn == 0) {
            bad += check(fn, 0x80000000ull, 0xc0000001ull, 7, &n, &slow, &obad);  // [-2, -0]
        } else {
            bad += check(fn, 0, 0x3dcccccdull, 7, &n, &slow, &obad);              // [0, 0.1]
            bad += check(fn, 0x80000000ull, 0xbdcccccdull, 7, &n, &slow, &obad);  // [-0.1, -0]
        }
        std::printf("%s: inputs %ld quad-resolved %ld host-libm-rounded differs %ld restated mismatched %ld\n", names[fn], n, slow,
                    obad, bad);
        total_bad += bad;
    }
    std::printf("mismatched: %ld\n", total_bad);
    return total_bad ? 1 : 0;
}
