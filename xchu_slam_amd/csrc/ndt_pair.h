// ndt_pair.h — the per-pair arithmetic of updateDerivatives (ndt_omp_impl.hpp:491-548), f32 per pair, accumulated in f64:
//   pair_f32: one f32 operation per reference operation, in the order the shipped libndt_omp.so evaluates them (read as
//             text with objdump -d; tests/native/sse_order_check.cpp re-evaluates the binary's SSE sequences):
//             * every 1x4-row-times-4-column product (x'C 0x41a40, the exp argument's dot 0x42476, q = x'(CJ) 0x41970,
//               J^T(CJ) 0x41ad0, (x'C) H_E 0x3cff0) is an SSE packet reduction (p0 + p2) + (p1 + p3); the fourth lane is
//               an exact zero (x4[3], row 3 of J and H_E), so a three-term one reads (p0 + p2) + p1;
//             * C * J (0x37840) accumulates k = 0, 1, 2 in sequence; the point derivatives (j_ang * x4, h_ang * x4,
//               0x4b6bc / 0x4a650) too;
//             * exp is (float)exp((double)x) (0x424a4-0x424bc, exp_dr);
//   pair_pk : the SAME f32 operations issued two at a time as packed f32 (v_pk_mul_f32 / v_pk_add_f32 on gfx950), each
//             lane of a packed instruction an independent IEEE f32 operation on exactly the operands and in exactly the
//             association of pair_f32 — results bit for bit identical (tests/native/pair_pk_check.cpp), except that a
//             few sums start from an exact +0 term (0 + x = x; only the sign of an exact zero can differ, which never
//             changes a sum).  A wave alone issues one VALU instruction per ~5.5 cycles (tools/native/valu_rates.hip:
//             two waves per SIMD reach 2.7 cycles per scalar f32 op, 2.0 per op packed), so the pass kernels, which run
//             two to three waves per SIMD, are issue-bound on the f32 part; packing halves its issue slots.
// Host and device code (the host check compiles it with g++ -ffp-contract=off).
#pragma once
#include <math.h>
#include "ndt_libm.h"

#if defined(__HIPCC__)
#define NDT_PAIR_FN __host__ __device__ __attribute__((always_inline)) inline
#else
#define NDT_PAIR_FN __attribute__((always_inline)) inline
#endif

namespace ndt {

typedef float pf2 __attribute__((vector_size(8)));

NDT_PAIR_FN pf2 pk(float a, float b) { return pf2{a, b}; }
NDT_PAIR_FN pf2 splat(float a) { return pf2{a, a}; }

NDT_PAIR_FN float red3(float p0, float p1, float p2) { return (p0 + p2) + p1; }  // predux of (p0, p1, p2, +-0)

// One (point, voxel) pair of updateDerivatives (f32), accumulated into acc[0]=score, acc[1..6]=g, acc[7..42]=H.
// t: xt[3] (transformed point), xj[8] (j_ang * x, eq. 6.19), xh[15] (h_ang * x, eq. 6.21); v: mean[3] (f64), icov[9] (f32,
// row-major).  etab: the exp_dr table (ndt_libm.h).

template <typename PT, typename RT>
NDT_PAIR_FN void pair_f32(const PT& t, const RT& v, float gd2, double d1, bool hess, double* acc, const double* etab) {
    float xp[3];
    for (int a = 0; a < 3; ++a) xp[a] = (float)((double)t.xt[a] - v.mean[a]);
    const float* C = v.icov;  // row-major C[i*3+j]
    float xC[3];
    for (int j = 0; j < 3; ++j) xC[j] = red3(xp[0] * C[0 * 3 + j], xp[1] * C[1 * 3 + j], xp[2] * C[2 * 3 + j]);
    const float dot = red3(xp[0] * xC[0], xp[1] * xC[1], xp[2] * xC[2]);
    float e = exp_dr(-gd2 * dot * 0.5f, etab);
    const float score_inc = (float)(-d1 * (double)e);
    e = gd2 * e;
    if (e > 1.f || e < 0.f || e != e) return;
    e = (float)((double)e * d1);
    acc[0] += (double)score_inc;
    // CJ (rows 0..2): columns 0..2 are C itself, columns 3..5 are C * J_col
    float CJ[3][6];
    for (int k = 0; k < 3; ++k) {
        CJ[k][0] = C[k * 3 + 0]; CJ[k][1] = C[k * 3 + 1]; CJ[k][2] = C[k * 3 + 2];
        float a3 = C[k * 3 + 1] * t.xj[0];
        a3 += C[k * 3 + 2] * t.xj[1];
        CJ[k][3] = a3;
        float a4 = C[k * 3 + 0] * t.xj[2];
        a4 += C[k * 3 + 1] * t.xj[3];
        a4 += C[k * 3 + 2] * t.xj[4];
        CJ[k][4] = a4;
        float a5 = C[k * 3 + 0] * t.xj[5];
        a5 += C[k * 3 + 1] * t.xj[6];
        a5 += C[k * 3 + 2] * t.xj[7];
        CJ[k][5] = a5;
    }
    float q[6];
    for (int j = 0; j < 6; ++j) q[j] = red3(xp[0] * CJ[0][j], xp[1] * CJ[1][j], xp[2] * CJ[2][j]);
    for (int j = 0; j < 6; ++j) acc[1 + j] += (double)(e * q[j]);
    if (!hess) return;
    // x' C * H_E blocks (a..f of eq. 6.21); a, b, c have a zero x component
    const float ha = xC[1] * t.xh[0] + xC[2] * t.xh[1];
    const float hb = xC[1] * t.xh[2] + xC[2] * t.xh[3];
    const float hc = xC[1] * t.xh[4] + xC[2] * t.xh[5];
    const float hd = red3(xC[0] * t.xh[6], xC[1] * t.xh[7], xC[2] * t.xh[8]);
    const float he = red3(xC[0] * t.xh[9], xC[1] * t.xh[10], xC[2] * t.xh[11]);
    const float hf = red3(xC[0] * t.xh[12], xC[1] * t.xh[13], xC[2] * t.xh[14]);
    const float ng = -gd2;
    for (int i = 0; i < 6; ++i) {
        const float ngq = ng * q[i];
        for (int j = 0; j < 6; ++j) {
            // JCJ(j,i) = J_col_j . CJ_col_i
            float jcj;
            if (j < 3) jcj = CJ[j][i];
            else if (j == 3) { jcj = t.xj[0] * CJ[1][i]; jcj += t.xj[1] * CJ[2][i]; }
            else if (j == 4) jcj = red3(t.xj[2] * CJ[0][i], t.xj[3] * CJ[1][i], t.xj[4] * CJ[2][i]);
            else jcj = red3(t.xj[5] * CJ[0][i], t.xj[6] * CJ[1][i], t.xj[7] * CJ[2][i]);
            float v0 = ngq * q[j];
            if (i >= 3 && j >= 3) {
                float hx;
                if (i == 3) hx = (j == 3) ? ha : (j == 4 ? hb : hc);
                else if (i == 4) hx = (j == 3) ? hb : (j == 4 ? hd : he);
                else hx = (j == 3) ? hc : (j == 4 ? he : hf);
                v0 = v0 + hx;
            }
            v0 = v0 + jcj;
            acc[7 + i * 6 + j] += (double)(e * v0);
        }
    }
}

// The point's derivative terms in the order pair_pk reads them as f32 pairs (24 floats):
//   [0..7]   xj0 xj1 | xj2 xj5 | xj3 xj6 | xj4 xj7
//   [8..23]  xh0 xh2 | xh1 xh3 | 0 xh6 | xh4 xh7 | xh5 xh8 | xh9 xh12 | xh10 xh13 | xh11 xh14
constexpr int kPkTerms = 24;
NDT_PAIR_FN void pk_terms(const float* xj, const float* xh, float* o) {
    o[0] = xj[0]; o[1] = xj[1]; o[2] = xj[2]; o[3] = xj[5]; o[4] = xj[3]; o[5] = xj[6]; o[6] = xj[4]; o[7] = xj[7];
    o[8] = xh[0]; o[9] = xh[2]; o[10] = xh[1]; o[11] = xh[3]; o[12] = 0.f; o[13] = xh[6]; o[14] = xh[4]; o[15] = xh[7];
    o[16] = xh[5]; o[17] = xh[8]; o[18] = xh[9]; o[19] = xh[12]; o[20] = xh[10]; o[21] = xh[13]; o[22] = xh[11]; o[23] = xh[14];
}

// The 43 accumulated terms of a pair, handed to a sink as they are produced: grad(score
// increment, (g0, g1), (g2, g3), (g4, g5)), then row(i, (H_i0, H_i1), (H_i2, H_i3), (H_i4, H_i5)) for i = 0..5 when hess.
// AccSink adds them to the 43 f64 sums of one lane.
struct AccSink {
    double* acc;
    NDT_PAIR_FN void grad(float score_inc, pf2 G01, pf2 G23, pf2 G45) {
        acc[0] += (double)score_inc;
        acc[1] += (double)G01[0]; acc[2] += (double)G01[1];
        acc[3] += (double)G23[0]; acc[4] += (double)G23[1];
        acc[5] += (double)G45[0]; acc[6] += (double)G45[1];
    }
    NDT_PAIR_FN void row(int i, pf2 T01, pf2 T23, pf2 T45) {
        double* h = acc + 7 + i * 6;
        h[0] += (double)T01[0]; h[1] += (double)T01[1];
        h[2] += (double)T23[0]; h[3] += (double)T23[1];
        h[4] += (double)T45[0]; h[5] += (double)T45[1];
    }
};

// pair_f32 with its f32 operations issued in pairs.  xt: transformed point; pd: the point's pk_terms (8-byte aligned).
// PRED: no early return for a rejected pair (every lane reaches every sink call: a sink that exchanges terms between lanes
// needs them all); a pair that does not count hands over zeros.
template <bool PRED, typename RT, typename Sink>
NDT_PAIR_FN void pair_pk_terms(const float* xt, const float* pd, const RT& v, float gd2, double d1, bool hess, const double* etab,
                               Sink& sink, bool valid = true) {
    float xp[3];
    for (int a = 0; a < 3; ++a) xp[a] = (float)((double)xt[a] - v.mean[a]);
    const float* C = v.icov;
    // x'C: columns 0, 1 packed, column 2 alone (each (xp0 C0j + xp2 C2j) + xp1 C1j, as pair_f32)
    pf2 xC01 = splat(xp[0]) * pk(C[0], C[1]);
    xC01 = xC01 + splat(xp[2]) * pk(C[6], C[7]);
    xC01 = xC01 + splat(xp[1]) * pk(C[3], C[4]);
    const float xC2 = red3(xp[0] * C[2], xp[1] * C[5], xp[2] * C[8]);
    const pf2 xp01 = pk(xp[0], xp[1]);
    const pf2 d01 = xp01 * xC01;
    const float dot = (d01[0] + xp[2] * xC2) + d01[1];
    float e = exp_dr(-gd2 * dot * 0.5f, etab);
    const float score_inc = (float)(-d1 * (double)e);
    e = gd2 * e;
    const bool ok = !(e > 1.f || e < 0.f || e != e);
    if (!PRED && !ok) return;
    // predicated: a rejected pair (or a lane past the tile's pairs) contributes E * V with E = +0 and a score of +0, i.e.
    // signed zeros (V is finite for finite records); adding a zero leaves an f64 sum that starts at +0 unchanged bit for bit
    float si = score_inc;
    if (PRED) {
        const bool use = ok && valid;
        e = use ? e : 0.f;
        si = use ? si : 0.f;
    }
    e = (float)((double)e * d1);
    const pf2* pj = reinterpret_cast<const pf2*>(pd);
    const pf2 X01 = pj[0], X25 = pj[1], X36 = pj[2], X47 = pj[3];
    // C * J columns 3..5: rows 0, 1 packed (P3, P4, P5; the C column pairs Cc0..Cc2), row 2 alone (r3) / packed (R45)
    const pf2 Cc0 = pk(C[0], C[3]), Cc1 = pk(C[1], C[4]), Cc2 = pk(C[2], C[5]);
    pf2 P3 = Cc1 * splat(X01[0]);
    P3 = P3 + Cc2 * splat(X01[1]);
    pf2 P4 = Cc0 * splat(X25[0]);
    P4 = P4 + Cc1 * splat(X36[0]);
    P4 = P4 + Cc2 * splat(X47[0]);
    pf2 P5 = Cc0 * splat(X25[1]);
    P5 = P5 + Cc1 * splat(X36[1]);
    P5 = P5 + Cc2 * splat(X47[1]);
    float r3 = C[7] * X01[0];
    r3 += C[8] * X01[1];
    pf2 R45 = splat(C[6]) * X25;
    R45 = R45 + splat(C[7]) * X36;
    R45 = R45 + splat(C[8]) * X47;
    // q = x'^T C J (columns 0..2 = x'C), each (xp0 CJ0j + xp2 CJ2j) + xp1 CJ1j
    const pf2 t3 = xp01 * P3, t4 = xp01 * P4, t5 = xp01 * P5;
    const float q3 = (t3[0] + xp[2] * r3) + t3[1];
    const pf2 q45 = (pk(t4[0], t5[0]) + splat(xp[2]) * R45) + pk(t4[1], t5[1]);
    const float q4 = q45[0], q5 = q45[1];
    const pf2 Q01 = xC01, Q23 = pk(xC2, q3), Q45 = pk(q4, q5);
    sink.grad(si, splat(e) * Q01, splat(e) * Q23, splat(e) * Q45);
    if (!hess) return;
    const pf2* ph = pj + 4;
    // (ha, hb), (hc, hd), (he, hf), each (xC0 h0 + xC2 h2) + xC1 h1; hc as (xC0 * 0 + xC2 xh5) + xC1 xh4
    pf2 HAB = splat(xC01[1]) * ph[0];
    HAB = HAB + splat(xC2) * ph[1];
    pf2 HCD = splat(xC01[0]) * ph[2];
    HCD = HCD + splat(xC2) * ph[4];
    HCD = HCD + splat(xC01[1]) * ph[3];
    pf2 HEF = splat(xC01[0]) * ph[5];
    HEF = HEF + splat(xC2) * ph[7];
    HEF = HEF + splat(xC01[1]) * ph[6];
    const float qv[6] = {Q01[0], Q01[1], xC2, q3, q4, q5};
    const float ng = -gd2;
    const pf2 E = splat(e);
    for (int i = 0; i < 6; ++i) {
        // CJ column i: rows 0, 1 (J01) and row 2 (c2)
        pf2 J01;
        float c2;
        if (i == 0) { J01 = Cc0; c2 = C[6]; }
        else if (i == 1) { J01 = Cc1; c2 = C[7]; }
        else if (i == 2) { J01 = Cc2; c2 = C[8]; }
        else if (i == 3) { J01 = P3; c2 = r3; }
        else if (i == 4) { J01 = P4; c2 = R45[0]; }
        else { J01 = P5; c2 = R45[1]; }
        const float ngq = ng * qv[i];
        // JCJ(3, i) = xj0 CJ1i + xj1 CJ2i; JCJ(4..5, i) packed, (xj CJ0i + xj' CJ2i) + xj'' CJ1i
        float j3 = X01[0] * J01[1];
        j3 += X01[1] * c2;
        pf2 J45 = X25 * splat(J01[0]);
        J45 = J45 + X47 * splat(c2);
        J45 = J45 + X36 * splat(J01[1]);
        pf2 V01 = splat(ngq) * Q01;
        pf2 V23 = splat(ngq) * Q23;
        pf2 V45 = splat(ngq) * Q45;
        if (i == 3) { V23[1] = V23[1] + HAB[0]; V45 = V45 + pk(HAB[1], HCD[0]); }
        if (i == 4) { V23[1] = V23[1] + HAB[1]; V45 = V45 + pk(HCD[1], HEF[0]); }
        if (i == 5) { V23[1] = V23[1] + HCD[0]; V45 = V45 + HEF; }
        V01 = V01 + J01;
        V23[0] = V23[0] + c2;
        V23[1] = V23[1] + j3;
        V45 = V45 + J45;
        sink.row(i, E * V01, E * V23, E * V45);
    }
}

template <typename RT>
NDT_PAIR_FN void pair_pk(const float* xt, const float* pd, const RT& v, float gd2, double d1, bool hess, double* acc,
                         const double* etab) {
    AccSink s{acc};
    pair_pk_terms<false>(xt, pd, v, gd2, d1, hess, etab, s);
}

}  // namespace ndt
