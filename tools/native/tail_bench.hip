// Micro-benchmark (tools only, not product code): the latency of the pass tail's pieces (ndt_control.h) in one
// 768-thread workgroup, the shape of the one-tile leading-tail kernel, on a synthetic Newton state (SPD Hessian, a
// More-Thuente interval that is closed: the default path).  Each piece runs R times back to back from a pristine LDS copy
// of the state; s_memtime (shader clock) brackets it on thread 0 after a barrier.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I../../xchu_slam_amd/csrc -o tail_bench tail_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include "ndt_control.h"

using namespace ndt;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int B = 768, NW = B / 64;
constexpr int kPieces = 9;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }

// An instrumented copy of tail_control's fast path 3 (ndt_control.h): s_memtime stamps per wave into ts[]
// [0] start, wave 0: [1] LU done [2] step regs [3] sincos [4] state stored [5] T; wave 1: [6] record [7] state machine
// [8] step regs [9] sincos [10] entries; [11] after the closing barrier
__device__ __noinline__ void fast3_stamped(AlignState& s_st, const double* red, PassRecordDev* hist, unsigned long long* tsl) {
    __shared__ double s_spec_dp[6];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) tsl[0] = now();
    double x_lu[6];
    if (wv == 0) {
        (void)lu6_solve_rows(red + 7, red + 1, s_spec_dp, true, x_lu);
        if (lane == 0) tsl[1] = now();
    } else if (wv == 1) {
        control_record_wave(&s_st, red, hist, 0);
        if (lane == 0) tsl[6] = now();
        control_step_wave(&s_st, red);
        if (lane == 0) tsl[7] = now();
    }
    const unsigned code0 = (wv == 1) ? c_angle_code[lane] : 0u;
    const unsigned code1 = (wv == 1 && lane < 5) ? c_angle_code[64 + lane] : 0u;
    lds_barrier();
    if (wv <= 1) {
        StepRegs o;
        double dpi[6];
        for (int k = 0; k < 6; ++k) dpi[k] = wv == 0 ? x_lu[k] : s_spec_dp[k];
        const bool ok = after_solve_regs(s_st, dpi, o);
        if (lane == 0) tsl[wv == 0 ? 2 : 8] = now();
        double xa = 0.0;
        for (int k = 0; k < 3; ++k)
            if (lane == k) xa = o.xt[3 + k];
        if (wv == 0) {
            float sn = 0.f, cs = 1.f;
            if (ok && lane < 3) sincosf_dr2((float)xa, &sn, &cs);
            float sa[3], ca[3];
            for (int a = 0; a < 3; ++a) {
                sa[a] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sn), a));
                ca[a] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cs), a));
            }
            if (lane == 0) tsl[3] = now();
            after_solve_store(s_st, o, 0);
            if (lane == 0) tsl[4] = now();
            if (lane == 0) {
                float R3[3][9];
                for (int a = 0; a < 3; ++a) angle_axis_sc(sa[a], ca[a], a, R3[a]);
                float Rxy[9], R[9];
                mat3_mul_f(R3[0], R3[1], Rxy);
                mat3_mul_f(Rxy, R3[2], R);
                for (int j = 0; j < 3; ++j)
                    for (int i = 0; i < 3; ++i) s_st.T[i + 4 * j] = R[i + 3 * j];
                tsl[5] = now();
            }
        } else {
            __shared__ double s_fv3[8];
            double sn = 0.0, cs = 1.0;
            if (ok && lane < 3 && !(fabs(xa) < 10e-5)) sincos(xa, &sn, &cs);
            if (lane < 3) { s_fv3[1 + 2 * lane] = sn; s_fv3[2 + 2 * lane] = cs; } else if (lane == 3) { s_fv3[0] = 1.0; s_fv3[7] = 0.0; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            if (lane == 0) tsl[9] = now();
            for (int h = 0; h < 2; ++h) {
                const int t = h * 64 + lane;
                if (t < 69) {
                    const unsigned code = h ? code1 : code0;
                    double a = s_fv3[code & 7];
                    if (code & (1u << 9)) a = -a;
                    double v = (a * s_fv3[(code >> 3) & 7]) * s_fv3[(code >> 6) & 7];
                    if (code & (1u << 20)) {
                        double d = s_fv3[(code >> 10) & 7];
                        if (code & (1u << 19)) d = -d;
                        v = v + (d * s_fv3[(code >> 13) & 7]) * s_fv3[(code >> 16) & 7];
                    }
                    const int r = t / 3, c = t - 3 * r;
                    if (r < 8) { s_st.jang[r][c] = (float)v; s_st.jang_d[r][c] = v; }
                    else { s_st.hang[r - 8][c] = (float)v; s_st.hang_d[r - 8][c] = v; }
                }
            }
            if (lane == 0) tsl[10] = now();
        }
    }
    lds_barrier();
    if (threadIdx.x == 0) tsl[11] = now();
}

__global__ __launch_bounds__(B) void k_tail_bench(const AlignState* __restrict__ st0, const double* __restrict__ red0, int reps,
                                                  unsigned long long* __restrict__ out, double* __restrict__ sink, PassRecordDev* hist,
                                                  AlignState* __restrict__ st_out) {
    __shared__ AlignState s_st;
    __shared__ double red[kNumAcc];
    __shared__ double s_dp[6];
    __shared__ double s_sc[12];
    const int t = threadIdx.x, wv = t >> 6;
    unsigned long long acc[kPieces] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    __shared__ unsigned long long tsl[12];
    unsigned long long tacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    constexpr int kWords = sizeof(AlignState) / 8;
    for (int r = 0; r < reps; ++r) {
        for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&s_st)[k] = reinterpret_cast<const unsigned long long*>(st0)[k];
        if (t < kNumAcc) red[t] = red0[t];
        lds_barrier();
        // [0] the speculative LU solve (wave 0)
        unsigned long long t0 = now();
        if (wv == 0) {
            const int f = lu6_solve_rows(red + 7, red + 1, s_dp, true);
            if (t == 0 && f) sink[0] += 1.0;
        }
        lds_barrier();
        unsigned long long t1 = now();
        acc[0] += t1 - t0;
        // [1] the pass record + copy (wave 1), [2] the state machine (wave 1 lane 0)
        t0 = now();
        if (wv == 1) control_record_wave(&s_st, red, hist, 0);
        lds_barrier();
        t1 = now();
        acc[1] += t1 - t0;
        t0 = now();
        if (t == 64) control_step(&s_st, red);
        lds_barrier();
        t1 = now();
        acc[2] += t1 - t0;
        // [3] newton_after_solve (lane 0)
        t0 = now();
        if (t == 0) newton_after_solve(&s_st, s_dp, 0);
        lds_barrier();
        t1 = now();
        acc[3] += t1 - t0;
        // [4] the sin / cos wave (wave 0)
        t0 = now();
        if (wv == 0) pass_sincos_wave(&s_st, s_sc);
        lds_barrier();
        t1 = now();
        acc[4] += t1 - t0;
        // [5] T + tables
        t0 = now();
        pass_tables<NW>(&s_st, s_sc);
        t1 = now();
        acc[5] += t1 - t0;

        // [6] the whole tail_control (as the kernels run it), from the pristine state again
        for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&s_st)[k] = reinterpret_cast<const unsigned long long*>(st0)[k];
        lds_barrier();
        t0 = now();
        tail_control<NW, 1>(s_st, red, hist, 0, nullptr);
        lds_barrier();
        t1 = now();
        acc[6] += t1 - t0;
        if (r == reps - 1)
            for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&st_out[0])[k] = reinterpret_cast<unsigned long long*>(&s_st)[k];
        // [8] tail_control with fast path 3
        for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&s_st)[k] = reinterpret_cast<const unsigned long long*>(st0)[k];
        lds_barrier();
        t0 = now();
        tail_control<NW, 3>(s_st, red, hist, 0, nullptr);
        lds_barrier();
        t1 = now();
        acc[8] += t1 - t0;
        if (r == reps - 1)
            for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&st_out[1])[k] = reinterpret_cast<unsigned long long*>(&s_st)[k];
        // the instrumented fast path 3
        for (int k = t; k < kWords; k += B) reinterpret_cast<unsigned long long*>(&s_st)[k] = reinterpret_cast<const unsigned long long*>(st0)[k];
        lds_barrier();
        fast3_stamped(s_st, red, hist, tsl);
        lds_barrier();
        if (t == 0)
            for (int k = 1; k < 12; ++k) tacc[k] += tsl[k] - tsl[0];
        // [7] an empty barrier pair (the measurement's own overhead)
        t0 = now();
        lds_barrier();
        lds_barrier();
        t1 = now();
        acc[7] += t1 - t0;
        if (t == 0) sink[1] += s_st.x_t[0] + s_st.T[0] + s_st.jang[1][1];
    }
    if (t == 0) {
        for (int k = 0; k < kPieces; ++k) out[k] = acc[k];
        for (int k = 1; k < 12; ++k) out[kPieces + k] = tacc[k];
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
    // synthetic state: first Newton pass consumed (phase 1), full pass, closed interval, no inner trial
    AlignState st;
    std::memset(&st, 0, sizeof(st));
    st.gauss_d1 = -2.2172252440; st.gauss_d2 = 0.4331230047; st.gauss_d3 = 0.5978370008;
    st.step_max = 0.1; st.step_min = 0.0; st.trans_eps = 0.0;
    st.max_iter = 30; st.n_src = 120000; st.search = 2; st.precision = 0; st.mt_possible = 0; st.radius = 1.0f;
    const double p[6] = {10.3, -4.2, 0.8, 0.01, -0.02, 0.3};
    const double dir[6] = {0.6, -0.3, 0.1, 0.002, -0.001, 0.74};
    double nd = 0;
    for (double d : dir) nd += d * d;
    for (int k = 0; k < 6; ++k) { st.p[k] = p[k]; st.dir[k] = dir[k] / std::sqrt(nd); st.x_t[k] = p[k]; st.x_eval[k] = p[k]; }
    st.a_t = 0.05;
    st.phase = 1; st.pass_kind = PASS_FULL; st.pending = 0; st.interval_converged = 1; st.step_iterations = 0; st.nr_iterations = 3;
    st.score = -150000.0;
    // reduced pass: score, g, H (SPD: A A^T + diag), pairs
    double red[kNumAcc];
    red[0] = -151000.0;
    srand(7);
    double A[36];
    for (double& a : A) a = (rand() / (double)RAND_MAX - 0.5) * 2000.0;
    for (int i = 0; i < 6; ++i) red[1 + i] = (rand() / (double)RAND_MAX - 0.5) * 500.0;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = 0;
            for (int k = 0; k < 6; ++k) s += A[i * 6 + k] * A[j * 6 + k];
            red[7 + i * 6 + j] = s + (i == j ? 5e4 : 0.0);
        }
    red[43] = 380000.0;
    AlignState* d_st; AlignState* d_st_out; double* d_red; unsigned long long* d_out; double* d_sink; PassRecordDev* d_hist;
    CK(hipMalloc(&d_st, sizeof(st))); CK(hipMalloc(&d_red, sizeof(red))); CK(hipMalloc(&d_out, (kPieces + 12) * 8));
    CK(hipMalloc(&d_sink, 16)); CK(hipMalloc(&d_hist, sizeof(PassRecordDev))); CK(hipMalloc(&d_st_out, 2 * sizeof(AlignState)));
    CK(hipMemcpy(d_st, &st, sizeof(st), hipMemcpyHostToDevice)); CK(hipMemcpy(d_red, red, sizeof(red), hipMemcpyHostToDevice));
    CK(hipMemset(d_sink, 0, 16));
    hipLaunchKernelGGL(k_tail_bench, dim3(1), dim3(B), 0, 0, d_st, d_red, 4, d_out, d_sink, d_hist, d_st_out);  // warm-up
    hipLaunchKernelGGL(k_tail_bench, dim3(1), dim3(B), 0, 0, d_st, d_red, reps, d_out, d_sink, d_hist, d_st_out);
    CK(hipDeviceSynchronize());
    unsigned long long out[kPieces + 12];
    CK(hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const char* names[kPieces] = {"lu6_solve_rows", "control_record_wave", "control_step", "newton_after_solve", "pass_sincos_wave",
                                  "pass_tables", "tail_control (whole)", "two empty barriers", "tail_control fast 3"};
    printf("shader clock %d MHz, %d reps; cycles (us at that clock) per call incl. one barrier:\n", clk_khz / 1000, reps);
    for (int k = 0; k < kPieces; ++k)
        printf("  %-22s %8.0f cycles %7.3f us\n", names[k], (double)out[k] / reps, (double)out[k] / reps / (clk_khz / 1000.0));
    const char* tn[12] = {"", "w0 LU done", "w0 step regs", "w0 sincos", "w0 state stored", "w0 T", "w1 record", "w1 state machine",
                          "w1 step regs", "w1 sincos", "w1 entries", "closing barrier"};
    printf("instrumented fast path 3 (cycles from its start):\n");
    for (int k = 1; k < 12; ++k) printf("  %-18s %8.0f\n", tn[k], (double)out[kPieces + k] / reps);
    double sk[2];
    CK(hipMemcpy(sk, d_sink, 16, hipMemcpyDeviceToHost));
    printf("sink %.1f\n", sk[0]);
    AlignState so[2];
    CK(hipMemcpy(so, d_st_out, sizeof(so), hipMemcpyDeviceToHost));
    const bool same = std::memcmp(&so[0], &so[1], sizeof(AlignState)) == 0;
    printf("fast 1 and fast 3 leave %s states (pending %d/%d, x_t[5] %.17g / %.17g, T[0] %.9g / %.9g)\n", same ? "bitwise identical" : "DIFFERENT",
           so[0].pending, so[1].pending, so[0].x_t[5], so[1].x_t[5], so[0].T[0], so[1].T[0]);
    return same ? 0 : 1;
}
