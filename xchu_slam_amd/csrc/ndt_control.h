// ndt_control.h — device-side Newton / More-Thuente driver (computeTransformation, ndt_omp_impl.hpp:73-164,
// computeStepLengthMT :760-916, updateIntervalMT :646-677, trialValueSelectionMT :682-757).
//
// control_step() runs on ONE lane with the optimiser state staged in LDS; it consumes the reduced results of
// the pass that just finished and decides the next pass (kind + parameters x_t).  prepare_pass_parallel()
// then builds the next transform and angle tables with the six sin/cos evaluations spread over lanes.
#pragma once
#include "ndt_device.h"

namespace ndt {

__device__ __forceinline__ double dot6(const double* a, const double* b) {
    double s = a[0] * b[0];
    for (int k = 1; k < 6; ++k) s += a[k] * b[k];
    return s;
}

// Marks the next pass; the transform / tables for x_t are built afterwards by prepare_pass_parallel().
__device__ void prepare_pass(AlignState* st, int kind) {
    for (int k = 0; k < 6; ++k) st->x_eval[k] = st->x_t[k];
    st->pass_kind = kind;
    st->pending = 1;
    st->needs_tables = 1;
}

__device__ void finish(AlignState* st) {
    st->trans_probability = st->score / (double)st->n_src;
    st->done = 1;
    st->pending = 0;
}

__device__ bool update_interval(double& a_l, double& f_l, double& g_l, double& a_u, double& f_u, double& g_u, double a_t,
                                double f_t, double g_t) {
    if (f_t > f_l) { a_u = a_t; f_u = f_t; g_u = g_t; return false; }
    else if (g_t * (a_l - a_t) > 0) { a_l = a_t; f_l = f_t; g_l = g_t; return false; }
    else if (g_t * (a_l - a_t) < 0) { a_u = a_l; f_u = f_l; g_u = g_l; a_l = a_t; f_l = f_t; g_l = g_t; return false; }
    return true;
}

__device__ double trial_value(double a_l, double f_l, double g_l, double a_u, double f_u, double g_u, double a_t, double f_t,
                              double g_t) {
    if (f_t > f_l) {
        double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
        double w = sqrt(z * z - g_t * g_l);
        double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
        double a_q = a_l - 0.5 * (a_l - a_t) * g_l / (g_l - (f_l - f_t) / (a_l - a_t));
        return (fabs(a_c - a_l) < fabs(a_q - a_l)) ? a_c : 0.5 * (a_q + a_c);
    } else if (g_t * g_l < 0) {
        double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
        double w = sqrt(z * z - g_t * g_l);
        double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
        double a_s = a_l - (a_l - a_t) / (g_l - g_t) * g_l;
        return (fabs(a_c - a_t) >= fabs(a_s - a_t)) ? a_c : a_s;
    } else if (fabs(g_t) <= fabs(g_l)) {
        double z = 3 * (f_t - f_l) / (a_t - a_l) - g_t - g_l;
        double w = sqrt(z * z - g_t * g_l);
        double a_c = a_l + (a_t - a_l) * (w - g_l - z) / (g_t - g_l + 2 * w);
        double a_s = a_l - (a_l - a_t) / (g_l - g_t) * g_l;
        double a_t_next = (fabs(a_c - a_t) < fabs(a_s - a_t)) ? a_c : a_s;
        if (a_t > a_l) return fmin(a_t + 0.66 * (a_u - a_t), a_t_next);
        return fmax(a_t + 0.66 * (a_u - a_t), a_t_next);
    } else {
        double z = 3 * (f_t - f_u) / (a_t - a_u) - g_t - g_u;
        double w = sqrt(z * z - g_t * g_u);
        return a_u + (a_t - a_u) * (w - g_u - z) / (g_t - g_u + 2 * w);
    }
}

// std::min / std::max semantics (return the first argument unless the second compares less / greater)
__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }

// tail of the Newton iteration after the line search returned step a (ndt_omp_impl.hpp:135-157)
__device__ bool newton_tail(AlignState* st, double a) {
    for (int k = 0; k < 6; ++k) st->p[k] = st->p[k] + st->dir[k] * a;
    const int nr = st->nr_iterations;
    bool conv = nr > st->max_iter || (nr && (fabs(a) < st->trans_eps));
    st->nr_iterations = nr + 1;
    if (conv) { st->converged = 1; finish(st); return true; }
    return false;
}

// Newton direction + start of computeStepLengthMT; loops only through zero-slope directions.
__device__ void newton_step(AlignState* st) {
    for (int guard = 0; guard < 1000000; ++guard) {
        double mg[6], dp[6];
        for (int k = 0; k < 6; ++k) mg[k] = -st->g[k];
        if (lu_solve6(st->H, mg, dp)) {
            // degenerate pivot: JacobiSVD semantics needed; pause the chain for k_svd_resume (rare path)
            if (!st->svd_ready) {
                st->needs_svd = 1;
                st->pending = 0;
                return;
            }
            for (int k = 0; k < 6; ++k) dp[k] = st->svd_dp[k];
            st->solver_fallbacks += 1;
        }
        st->svd_ready = 0;
        double nrm2 = 0.0;
        for (int k = 0; k < 6; ++k) nrm2 += dp[k] * dp[k];
        const double norm = sqrt(nrm2);
        if (norm == 0 || norm != norm) {
            st->converged = (norm == norm) ? 1 : 0;
            finish(st);
            return;
        }
        if (nrm2 > 0) { const double s = sqrt(nrm2); for (int k = 0; k < 6; ++k) dp[k] /= s; }
        for (int k = 0; k < 6; ++k) st->dir[k] = dp[k];
        // computeStepLengthMT
        st->phi_0 = -st->score;
        st->d_phi_0 = -dot6(st->g, st->dir);
        if (st->d_phi_0 >= 0) {
            if (st->d_phi_0 == 0) {
                if (newton_tail(st, 0.0)) return;
                continue;
            }
            st->d_phi_0 *= -1;
            for (int k = 0; k < 6; ++k) st->dir[k] *= -1;
        }
        const double mu = 1.e-4;
        st->a_l = 0; st->a_u = 0;
        st->f_l = st->phi_0 - st->phi_0 - mu * st->d_phi_0 * st->a_l;
        st->g_l = st->d_phi_0 - mu * st->d_phi_0;
        st->f_u = st->phi_0 - st->phi_0 - mu * st->d_phi_0 * st->a_u;
        st->g_u = st->d_phi_0 - mu * st->d_phi_0;
        st->interval_converged = (st->step_max - st->step_min) > 0;   // reference quirk kept (:807)
        st->open_interval = 1;
        st->step_iterations = 0;
        double a_t = norm;
        a_t = smin(a_t, st->step_max);
        a_t = smax(a_t, st->step_min);
        st->a_t = a_t;
        for (int k = 0; k < 6; ++k) st->x_t[k] = st->p[k] + st->dir[k] * a_t;
        prepare_pass(st, PASS_FULL);
        return;
    }
}

__device__ void mt_loop_check(AlignState* st) {
    const double nu = 0.9;
    if (!st->interval_converged && st->step_iterations < 10 && !(st->psi_t <= 0 && st->d_phi_t <= -nu * st->d_phi_0)) {
        double a_t;
        if (st->open_interval) a_t = trial_value(st->a_l, st->f_l, st->g_l, st->a_u, st->f_u, st->g_u, st->a_t, st->psi_t, st->d_psi_t);
        else a_t = trial_value(st->a_l, st->f_l, st->g_l, st->a_u, st->f_u, st->g_u, st->a_t, st->phi_t, st->d_phi_t);
        a_t = smin(a_t, st->step_max);
        a_t = smax(a_t, st->step_min);
        st->a_t = a_t;
        for (int k = 0; k < 6; ++k) st->x_t[k] = st->p[k] + st->dir[k] * a_t;
        prepare_pass(st, PASS_GRAD);
        return;
    }
    if (st->step_iterations) {
        // computeHessian at x_t (radius neighbours, f64); T and tables are those of x_t already
        for (int k = 0; k < 6; ++k) st->x_eval[k] = st->x_t[k];
        st->pass_kind = PASS_HESS;
        st->pending = 1;
        return;
    }
    if (!newton_tail(st, st->a_t)) newton_step(st);
}

__device__ void eval_trial(AlignState* st) {
    const double mu = 1.e-4;
    st->phi_t = -st->score;
    st->d_phi_t = -dot6(st->g, st->dir);
    st->psi_t = st->phi_t - st->phi_0 - mu * st->d_phi_0 * st->a_t;
    st->d_psi_t = st->d_phi_t - mu * st->d_phi_0;
}

__device__ void control_step(AlignState* st, const double* r, PassRecordDev* hist, int hist_cap) {
    const int kind = st->pass_kind;
    const long long pairs = (long long)r[43];
    if (st->hist_count < hist_cap) {
        PassRecordDev& h = hist[st->hist_count];
        h.kind = kind;
        h.newton_iter = st->phase == 0 ? 0 : st->nr_iterations + 1;
        // a Hessian-only pass (computeHessian, ndt_omp_impl.hpp:550) carries the line search's score / gradient
        const bool hess_only = kind == PASS_HESS;
        for (int k = 0; k < 6; ++k) { h.x[k] = st->x_eval[k]; h.g[k] = hess_only ? st->g[k] : r[1 + k]; }
        h.score = hess_only ? st->score : r[0];
        for (int k = 0; k < 36; ++k) h.H[k] = r[7 + k];
        h.pairs = pairs;
    }
    st->hist_count++;
    st->n_passes++;
    st->pairs_total += pairs;
    st->pending = 0;
    if (st->phase == 0) {
        st->phase = 1;
        st->score = r[0];
        for (int k = 0; k < 6; ++k) st->g[k] = r[1 + k];
        for (int k = 0; k < 36; ++k) st->H[k] = r[7 + k];
        newton_step(st);
        return;
    }
    if (kind == PASS_FULL) {
        st->score = r[0];
        for (int k = 0; k < 6; ++k) st->g[k] = r[1 + k];
        for (int k = 0; k < 36; ++k) st->H[k] = r[7 + k];
        eval_trial(st);
        mt_loop_check(st);
    } else if (kind == PASS_GRAD) {
        const double mu = 1.e-4;
        st->score = r[0];
        for (int k = 0; k < 6; ++k) st->g[k] = r[1 + k];
        for (int k = 0; k < 36; ++k) st->H[k] = 0.0;
        eval_trial(st);
        if (st->open_interval && (st->psi_t <= 0 && st->d_psi_t >= 0)) {
            st->open_interval = 0;
            st->f_l = st->f_l + st->phi_0 - mu * st->d_phi_0 * st->a_l;
            st->g_l = st->g_l + mu * st->d_phi_0;
            st->f_u = st->f_u + st->phi_0 - mu * st->d_phi_0 * st->a_u;
            st->g_u = st->g_u + mu * st->d_phi_0;
        }
        if (st->open_interval)
            st->interval_converged = update_interval(st->a_l, st->f_l, st->g_l, st->a_u, st->f_u, st->g_u, st->a_t, st->psi_t, st->d_psi_t);
        else
            st->interval_converged = update_interval(st->a_l, st->f_l, st->g_l, st->a_u, st->f_u, st->g_u, st->a_t, st->phi_t, st->d_phi_t);
        st->step_iterations++;
        mt_loop_check(st);
    } else {
        for (int k = 0; k < 36; ++k) st->H[k] = r[7 + k];
        if (!newton_tail(st, st->a_t)) newton_step(st);
    }
}

// convertTransform(x_t) -> T and computeAngleDerivatives(x_t) -> tables, for a workgroup: lanes 0-2 evaluate
// the f32 AngleAxis sin/cos, lanes 3-5 the f64 angle-derivative sin/cos, then lane 0 assembles T and lanes
// 0-22 one table row each.  Same arithmetic as convert_transform / angle_tables in ndt_linalg.h.
__device__ void prepare_pass_parallel(AlignState* st) {
    __shared__ double s_sc[12];
    const int t = threadIdx.x;
    if (t < 3) {
        double s, c;
        sincos((double)(float)st->x_t[3 + t], &s, &c);
        s_sc[2 * t] = s;
        s_sc[2 * t + 1] = c;
    } else if (t < 6) {
        const double a = st->x_t[t];
        double s = 0.0, c = 1.0;
        if (!(fabs(a) < 10e-5)) sincos(a, &s, &c);
        s_sc[2 * t] = s;
        s_sc[2 * t + 1] = c;
    }
    __syncthreads();
    if (t == 0) {
        float R3[3][9];
        for (int a = 0; a < 3; ++a) angle_axis_sc((float)s_sc[2 * a], (float)s_sc[2 * a + 1], a, R3[a]);
        float Rxy[9], R[9];
        mat3_mul_f(R3[0], R3[1], Rxy);
        mat3_mul_f(Rxy, R3[2], R);
        for (int j = 0; j < 3; ++j)
            for (int i = 0; i < 3; ++i) st->T[i + 4 * j] = R[i + 3 * j];
        st->T[3] = 0.f; st->T[7] = 0.f; st->T[11] = 0.f;
        st->T[12] = (float)st->x_t[0]; st->T[13] = (float)st->x_t[1]; st->T[14] = (float)st->x_t[2]; st->T[15] = 1.f;
    }
    if (t < 23) {
        const double sx = s_sc[6], cx = s_sc[7], sy = s_sc[8], cy = s_sc[9], sz = s_sc[10], cz = s_sc[11];
        double row[3];
        angle_table_row(t, cx, sx, cy, sy, cz, sz, row);
        if (t < 8) {
            for (int c = 0; c < 3; ++c) { st->jang[t][c] = (float)row[c]; st->jang_d[t][c] = row[c]; }
            st->jang[t][3] = 0.f;
        } else {
            const int r = t - 8;
            for (int c = 0; c < 3; ++c) { st->hang[r][c] = (float)row[c]; st->hang_d[r][c] = row[c]; }
            st->hang[r][3] = 0.f;
        }
    }
    if (t < 4) st->hang[15][t] = 0.f;
    if (t == 0) st->needs_tables = 0;
    __syncthreads();
}

// Sum of x over the 64 lanes of the wave, identical on every lane (register exchanges only; each step adds
// the two halves in the same order on both sides, so all lanes hold the same bits).
__device__ __forceinline__ double wave_allreduce_d(double x) {
    x = swap_add_d<32>(x, x);
    x = swap_add_d<16>(x, x);
    x += partner_d<8>(x);
    x += partner_d<4>(x);
    x += partner_d<2>(x);
    x += partner_d<1>(x);
    return x;
}

// Deterministic reduction of a pass's partials [kNumAcc][partial_stride(nb)] by ONE workgroup into LDS
// red[kNumAcc].  Wave w owns values v = w, w+4, ...; lane l sums the 16-byte pairs (2l, 2l+1) + 128k of each
// of its rows.  All of a lane's loads (11 rows x 4 pairs for nb <= 512) are issued before any is consumed,
// so the reduction costs one memory round trip, not one per value.
__device__ __forceinline__ void reduce_partials_block(const double* __restrict__ partials, int nb, double* red) {
    constexpr int Q = (kNumAcc + 3) / 4;
    constexpr int K = 4;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ps = partial_stride(nb);
    double s[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) s[q] = 0.0;
    for (int c0 = 0; c0 < nb; c0 += 128 * K) {
        double2 x[Q][K];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int v = w + 4 * q;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int b = c0 + 2 * lane + 128 * k;
                x[q][k] = (v < kNumAcc && b < nb) ? *reinterpret_cast<const double2*>(partials + (size_t)v * ps + b)
                                                  : make_double2(0.0, 0.0);
                if (b + 1 >= nb) x[q][k].y = 0.0;  // row padding is never written
            }
        }
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int k = 0; k < K; ++k) {
                s[q] += x[q][k].x;
                s[q] += x[q][k].y;
            }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int v = w + 4 * q;
        const double t = wave_allreduce_d(s[q]);
        if (v < kNumAcc && lane == 0) red[v] = t;
    }
    __syncthreads();
}

static_assert(sizeof(AlignState) % 8 == 0, "AlignState is copied as 8-byte words");

// Epilogue of every derivative pass (all threads of every workgroup call it).
//  1. workgroup partials -> partials[v][block] (reduce-scatter block reduction);
//  2. hand-off (Guideline 16): every storing wave drains (vmcnt 0), workgroup barrier, one lane releases at
//     agent scope and takes a ticket on `counter`; the workgroup that draws the last ticket acquires;
//  3. that last workgroup reduces all partials in a fixed order and either publishes them (mode 1: test hook)
//     or runs the Newton / More-Thuente control step on the LDS-staged state and prepares the next pass
//     (mode 0), then re-arms the ticket counter for the next launch.
// The align is therefore one kernel per derivative pass with no host round trip and no separate reduce /
// control launches; results are bitwise deterministic (no float atomics, fixed orders).
__device__ __forceinline__ void pass_epilogue(double (&acc)[kNumAcc], double* red4, AlignState* st, double* partials,
                                              unsigned* counter, double* red_out, PassRecordDev* hist, int hist_cap, int mode,
                                              unsigned long long* ts) {
    block_reduce_store<kNumAcc>(acc, red4, partials + blockIdx.x, partial_stride(gridDim.x));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ts && threadIdx.x == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        atomicMax(&ts[2], now);
    }
#ifdef NDT_BODY_STAMPS
    NDT_BLK_STAMP(st->n_passes, 4);
#endif
    __shared__ unsigned s_ticket;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_ticket = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_ticket != gridDim.x - 1) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ts) ts[3] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    __shared__ double red[kNumAcc];
    reduce_partials_block(partials, gridDim.x, red);
    if (ts && threadIdx.x == 0) ts[4] = __builtin_amdgcn_s_memrealtime();
    if (mode == 1) {
        if (threadIdx.x < kNumAcc) red_out[threadIdx.x] = red[threadIdx.x];
        if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __shared__ AlignState s_st;
    constexpr int kWords = sizeof(AlignState) / 8;
    unsigned long long* gw = reinterpret_cast<unsigned long long*>(st);
    unsigned long long* lw = reinterpret_cast<unsigned long long*>(&s_st);
    for (int k = threadIdx.x; k < kWords; k += kBlock) lw[k] = gw[k];
    __syncthreads();
    if (ts && threadIdx.x == 0) ts[6] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) control_step(&s_st, red, hist, hist_cap);
    __syncthreads();
    if (ts && threadIdx.x == 0) ts[7] = __builtin_amdgcn_s_memrealtime();
    if (s_st.needs_tables) prepare_pass_parallel(&s_st);
    if (ts && threadIdx.x == 0) ts[5] = __builtin_amdgcn_s_memrealtime();
    for (int k = threadIdx.x; k < kWords; k += kBlock) gw[k] = lw[k];
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ndt
