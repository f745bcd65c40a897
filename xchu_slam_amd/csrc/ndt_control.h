// ndt_control.h — device-side Newton / More-Thuente driver (computeTransformation, ndt_omp_impl.hpp:73-164,
// computeStepLengthMT :760-916, updateIntervalMT :646-677, trialValueSelectionMT :682-757).
//
// control_step() runs on ONE lane with the optimiser state staged in LDS; it consumes the reduced results of
// the pass that just finished and decides the next pass (kind + parameters x_t).  prepare_pass_parallel()
// then builds the next transform and angle tables with the six sin/cos evaluations spread over lanes.
#pragma once
#include "ndt_device.h"

namespace ndt {

// Eigen's vectorised 6-vector dot / squaredNorm (SSE2, three packets of two doubles): packet sum P0 + (P1 + P2), then
// lane 0 + lane 1 — libndt_omp.so 0x48fa3-0x49007 (score_gradient.dot(step_dir) in computeStepLengthMT) and
// 0x4a070-0x4a0bc (delta_p.norm() in computeTransformation)
__device__ __forceinline__ double dot6(const double* a, const double* b) {
    return (a[0] * b[0] + (a[2] * b[2] + a[4] * b[4])) + (a[1] * b[1] + (a[3] * b[3] + a[5] * b[5]));
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    unsigned lo, hi;
    split_d(v, lo, hi);
    lo = (unsigned)__builtin_amdgcn_readlane((int)lo, l);
    hi = (unsigned)__builtin_amdgcn_readlane((int)hi, l);
    return join_d(lo, hi);
}

// Marks the next pass; the transform / tables for x_t are built afterwards by prepare_pass_parallel().
__device__ __forceinline__ void prepare_pass(AlignState* st, int kind) {
    for (int k = 0; k < 6; ++k) st->x_eval[k] = st->x_t[k];
    st->pass_kind = kind;
    st->pending = 1;
    st->needs_tables = 1;
}

__device__ __forceinline__ void finish(AlignState* st) {
    st->trans_probability = st->score / (double)st->n_src;
    st->done = 1;
    st->pending = 0;
}

// std::min / std::max semantics (return the first argument unless the second compares less / greater)
__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }

__device__ __forceinline__ bool update_interval(double& a_l, double& f_l, double& g_l, double& a_u, double& f_u, double& g_u, double a_t,
                                double f_t, double g_t) {
    if (f_t > f_l) { a_u = a_t; f_u = f_t; g_u = g_t; return false; }
    else if (g_t * (a_l - a_t) > 0) { a_l = a_t; f_l = f_t; g_l = g_t; return false; }
    else if (g_t * (a_l - a_t) < 0) { a_u = a_l; f_u = f_l; g_u = g_l; a_l = a_t; f_l = f_t; g_l = g_t; return false; }
    return true;
}

__device__ __forceinline__ double trial_value(double a_l, double f_l, double g_l, double a_u, double f_u, double g_u, double a_t, double f_t,
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
        // std::min / std::max (ndt_omp_impl.hpp:742-745), not fmin / fmax: they differ on NaN and signed zeros
        if (a_t > a_l) return smin(a_t + 0.66 * (a_u - a_t), a_t_next);
        return smax(a_t + 0.66 * (a_u - a_t), a_t_next);
    } else {
        double z = 3 * (f_t - f_u) / (a_t - a_u) - g_t - g_u;
        double w = sqrt(z * z - g_t * g_u);
        return a_u + (a_t - a_u) * (w - g_u - z) / (g_t - g_u + 2 * w);
    }
}

// tail of the Newton iteration after the line search returned step a (ndt_omp_impl.hpp:135-157)
__device__ __forceinline__ bool newton_tail(AlignState* st, double a) {
    for (int k = 0; k < 6; ++k) st->p[k] = st->p[k] + st->dir[k] * a;
    const int nr = st->nr_iterations;
    bool conv = nr > st->max_iter || (nr && (fabs(a) < st->trans_eps));
    st->nr_iterations = nr + 1;
    if (conv) { st->converged = 1; finish(st); return true; }
    return false;
}

// Newton direction (ndt_omp_impl.hpp:118-124, JacobiSVD solve of H dp = -g) is requested here and solved by
// the first wave (lu6_solve_rows); newton_after_solve() then runs the rest of the iteration.
__device__ __forceinline__ void newton_request(AlignState* st) { st->want_solve = 1; }

// After the solve: normalise the direction and start computeStepLengthMT.  A zero-slope direction takes a
// zero step and asks for another solve (the reference's loop through newton iterations with step 0).
__device__ __forceinline__ void newton_after_solve(AlignState* st, const double* dp_in, int lu_fail) {
    st->want_solve = 0;
    double dp[6];
    for (int k = 0; k < 6; ++k) dp[k] = dp_in[k];
    if (lu_fail) {
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
    const double nrm2 = dot6(dp, dp);
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
            if (!newton_tail(st, 0.0)) newton_request(st);
            return;
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
}

__device__ __forceinline__ void mt_loop_check(AlignState* st) {
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
    if (!newton_tail(st, st->a_t)) newton_request(st);
}

__device__ __forceinline__ void eval_trial(AlignState* st) {
    const double mu = 1.e-4;
    st->phi_t = -st->score;
    st->d_phi_t = -dot6(st->g, st->dir);
    st->psi_t = st->phi_t - st->phi_0 - mu * st->d_phi_0 * st->a_t;
    st->d_psi_t = st->d_phi_t - mu * st->d_phi_0;
}

// Consumption of a finished pass by ONE wave (lanes 0..48): the history record and the copy of score / gradient /
// Hessian into the optimiser state (which of them depends on the pass kind, as the reference's computeDerivatives /
// computeHessian callers overwrite them).  No workgroup barrier: within a wave the LDS reads of the old
// state are issued before the writes that overwrite them (program order, in-order LDS), so another wave can run
// the speculative Newton solve meanwhile (pass_epilogue).
__device__ __forceinline__ void control_record_wave(AlignState* st, const double* r, PassRecordDev* hist, int hist_cap) {
    const int t = threadIdx.x & 63;
    const int kind = st->pass_kind;
    const bool hess_only = kind == PASS_HESS;
    const int hc = st->hist_count;
    if (hc < hist_cap) {
        PassRecordDev& h = hist[hc];
        if (t < 36) h.H[t] = r[7 + t];
        else if (t < 42) h.g[t - 36] = hess_only ? st->g[t - 36] : r[1 + (t - 36)];
        else if (t < 48) h.x[t - 42] = st->x_eval[t - 42];
        else if (t == 48) {
            h.kind = kind;
            h.newton_iter = st->phase == 0 ? 0 : st->nr_iterations + 1;
            h.score = hess_only ? st->score : r[0];
            h.pairs = (long long)r[43];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const bool full = st->phase == 0 || kind == PASS_FULL;
    if (full || kind == PASS_GRAD) {
        if (t < 36) st->H[t] = full ? r[7 + t] : 0.0;
        else if (t < 42) st->g[t - 36] = r[1 + (t - 36)];
        else if (t == 42) st->score = r[0];
    } else if (t < 36) {
        st->H[t] = r[7 + t];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// One lane: the Newton / More-Thuente state machine for the pass just recorded (score/g/H already copied).
__device__ __forceinline__ void control_step(AlignState* st, const double* r) {
    const int kind = st->pass_kind;
    const long long pairs = (long long)r[43];
    st->hist_count++;
    st->n_passes++;
    st->pairs_total += pairs;
    st->pending = 0;
    if (st->phase == 0) {
        st->phase = 1;
        newton_request(st);
        return;
    }
    if (kind == PASS_FULL) {
        eval_trial(st);
        mt_loop_check(st);
    } else if (kind == PASS_GRAD) {
        const double mu = 1.e-4;
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
        if (!newton_tail(st, st->a_t)) newton_request(st);
    }
}

// control_step by a whole wave for the initial pass and the default Newton path (a full pass, More-Thuente interval
// closed, no inner trial: eval_trial + newton_tail + newton_request), the state read into registers and written one
// field per lane — the same expressions in the same order as control_step; any other case runs control_step on lane 0.
// Called by every lane of the wave after control_record_wave.
__device__ __forceinline__ void control_step_wave(AlignState* st, const double* r) {
    const int lane = threadIdx.x & 63;
    const int kind = st->pass_kind, phase = st->phase;
    const bool common = phase == 1 && kind == PASS_FULL && st->interval_converged && st->step_iterations == 0;
    if (!common) {
        if (lane == 0) control_step(st, r);
        return;
    }
    const long long pairs = (long long)r[43];
    const int hc = st->hist_count, np = st->n_passes, nr = st->nr_iterations, max_iter = st->max_iter, n_src = st->n_src;
    const long long pt = st->pairs_total;
    const double score = st->score, phi_0 = st->phi_0, d_phi_0 = st->d_phi_0, a_t = st->a_t, trans_eps = st->trans_eps;
    double g[6], dir[6], p[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) { g[k] = st->g[k]; dir[k] = st->dir[k]; p[k] = st->p[k]; }
    const double mu = 1.e-4;
    const double phi_t = -score;
    const double d_phi_t = -dot6(g, dir);
    const double psi_t = phi_t - phi_0 - mu * d_phi_0 * a_t;
    const double d_psi_t = d_phi_t - mu * d_phi_0;
    const bool conv = nr > max_iter || (nr && (fabs(a_t) < trans_eps));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    if (lane == 0) {
        st->hist_count = hc + 1;
        st->n_passes = np + 1;
        st->pairs_total = pt + pairs;
        st->pending = 0;
        st->nr_iterations = nr + 1;
        if (conv) {
            st->converged = 1;
            st->trans_probability = score / (double)n_src;
            st->done = 1;
        } else {
            st->want_solve = 1;
        }
    } else if (lane == 1) {
        st->phi_t = phi_t;
        st->d_phi_t = d_phi_t;
        st->psi_t = psi_t;
        st->d_psi_t = d_psi_t;
    } else if (lane < 8) {
        double pk = 0.0, dk = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (lane - 2 == k) { pk = p[k]; dk = dir[k]; }
        st->p[lane - 2] = pk + dk * a_t;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}


// Newton direction H dx = b (b negated when neg_b) by one whole wave (all 64 lanes call it, uniform control flow): LU
// without pivoting (the Hessian of an NDT score near its optimum is symmetric positive definite up to rounding), lane
// i < 6 holds row i, each elimination step broadcasts the pivot row and the pivot with readlanes and every lane forms
// the pivot reciprocal (v_rcp + a Newton step) itself; the substitutions run row by row with the solved components
// broadcast, in ascending-column order (bitwise the former single-lane solve, at 120 instead of 290 f64 instructions).
// Returns 1 (on every lane) when the LU answer may differ from the reference's JacobiSVD<6d>::solve
// (ndt_omp_impl.hpp:118-124): a pivot below 1e-12 max|H| (or non-finite), or a condition bound above kCondLU
// (ndt_linalg.h) — the caller then takes the Eigen-semantics SVD (k_svd_resume).  The bound: with H = LU,
// ||H^-1|| <= ||U^-1|| ||L^-1|| and, for a triangular T, ||T^-1||_inf <= ||M(T)^-1 e||_inf (M(T): |diagonal|,
// -|off-diagonal|; Higham, Accuracy and Stability of Numerical Algorithms, Thm 8.12), so
// kappa_inf(H) <= ||H||_inf max(z) max(y) with M(U) z = e and M(L) y = e — two extra substitutions; cond_2 <= 6 kappa_inf.
// Growth without pivoting only raises the bound (the SVD then decides), it can never let a system through that JacobiSVD
// would truncate.  x_out written by lane 0.
__device__ __forceinline__ int lu6_solve_rows(const double* Hrow, const double* b, double* x_out, bool neg_b, double* x_all = nullptr) {
    const int lane = threadIdx.x & 63;
    const int i = lane < 6 ? lane : 5;
    double a[6];
    double amax_l = 0.0, rs = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        a[j] = Hrow[i * 6 + j];
        amax_l = tmax(amax_l, fabs(a[j]));
        rs += fabs(a[j]);
    }
    double r = neg_b ? -b[i] : b[i];
    // maxima over the six rows as a tree (max is exact: any order gives the same value)
    double am[6], hr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) { am[k] = readlane_d(amax_l, k); hr[k] = readlane_d(rs, k); }
    const double amax = tmax(tmax(tmax(0.0, am[0]), tmax(am[1], am[2])), tmax(am[3], tmax(am[4], am[5])));
    const double hinf = tmax(tmax(tmax(0.0, hr[0]), tmax(hr[1], hr[2])), tmax(hr[3], tmax(hr[4], hr[5])));
    bool bad = !(amax > 0.0) || !(amax < HUGE_VAL);
    const double tol = 1e-12 * amax;
    double inv_piv[6];
    // y (the bound's forward substitution with M(L), unit diagonal) rides along the elimination: once column c is
    // eliminated, lane c's sum 1 + sum_j<c |l_cj| y_j is complete (the same adds in the same order as a separate pass)
    double y[6], x[6], z[6];
    double yacc = 1.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const double piv = readlane_d(a[c], c);
        bad = bad || !(fabs(piv) > tol);
        double inv = __builtin_amdgcn_rcp(piv);
        inv = fma(fma(-piv, inv, 1.0), inv, inv);
        inv_piv[c] = inv;
        double prow[6];
#pragma unroll
        for (int j = c + 1; j < 6; ++j) prow[j] = readlane_d(a[j], c);
        const double rc = readlane_d(r, c);
        y[c] = readlane_d(yacc, c);
        if (lane > c && lane < 6) {
            const double f = a[c] * inv;
#pragma unroll
            for (int j = c + 1; j < 6; ++j) a[j] -= f * prow[j];
            r -= f * rc;
            a[c] = f;
            yacc += fabs(f) * y[c];
        }
    }
    // x and z (backward, U): row i is finished on lane i and broadcast (a progressive form — every lane subtracting
    // its term as soon as a component is broadcast — measured 0.5% slower on C2)
#pragma unroll
    for (int k = 5; k >= 0; --k) {
        double acc = r, zacc = 1.0;
#pragma unroll
        for (int j = k + 1; j < 6; ++j) {
            acc -= a[j] * x[j];
            zacc += fabs(a[j]) * z[j];
        }
        x[k] = readlane_d(acc * inv_piv[k], k);
        z[k] = readlane_d(zacc * fabs(inv_piv[k]), k);
    }
    const double zmax = tmax(tmax(tmax(0.0, z[0]), tmax(z[1], z[2])), tmax(z[3], tmax(z[4], z[5])));
    const double ymax = tmax(tmax(tmax(0.0, y[0]), tmax(y[1], y[2])), tmax(y[3], tmax(y[4], y[5])));
    bad = bad || !(hinf * zmax * ymax <= kCondLU);
    if (x_all)
#pragma unroll
        for (int k = 0; k < 6; ++k) x_all[k] = x[k];  // uniform over the wave (every component was broadcast)
    if (bad) return 1;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) x_out[k] = x[k];
    return 0;
}

// Runs every Newton solve the state machine requested (all threads of the workgroup; normally one).  spec_dp:
// the solve of H dp = -g already computed (speculatively, during the control step) for the H and g this loop
// solves with — they do not change inside the loop — so it is taken instead of solving again.
__device__ __forceinline__ void solve_loop(AlignState* st, const double* spec_dp = nullptr, const int* spec_fail = nullptr) {
    __shared__ double s_dp[6];
    __shared__ double s_mg[6];
    __shared__ int s_fail;
    for (int guard = 0; guard < (1 << 20); ++guard) {
        lds_barrier();
        if (!st->want_solve) break;
        if (spec_dp) {
            if (threadIdx.x == 0) {
                NDT_TAIL_STAMP(0);
                NDT_TAIL_STAMP(1);
                newton_after_solve(st, spec_dp, *spec_fail);
            }
            continue;
        }
        if (threadIdx.x < 6) s_mg[threadIdx.x] = -st->g[threadIdx.x];
        lds_barrier();
        if (threadIdx.x == 0) NDT_TAIL_STAMP(0);
        if (threadIdx.x < 64) {
            const int f = lu6_solve_rows(st->H, s_mg, s_dp, false);
            if (threadIdx.x == 0) s_fail = f;
        }
        lds_barrier();
        if (threadIdx.x == 0) {
            NDT_TAIL_STAMP(1);
            newton_after_solve(st, s_dp, s_fail);
        }
    }
    lds_barrier();
}

__constant__ unsigned c_angle_code[69] = NDT_ANGLE_TABLE_CODE;

// For the tail's fast path: the sin/cos of x_t's angles by ONE wave (lanes 0-2: the f32 AngleAxis sin/cos, lanes 3-5:
// the f64 angle-derivative sin/cos); pass_tables, after a workgroup barrier: T and the tables from them (also the
// second half of prepare_pass_parallel)
__device__ __forceinline__ void pass_sincos_wave(const AlignState* st, double* sc) {
    const int lane = threadIdx.x & 63;
    if (lane < 3) {
        // sin and cos of one angle side by side (sincosf_dr2: the bits of sinf_dr / cosf_dr, two independent chains)
        float sn, cs;
        sincosf_dr2((float)st->x_t[3 + lane], &sn, &cs);
        sc[2 * lane] = (double)sn;
        sc[2 * lane + 1] = (double)cs;
    } else if (lane < 6) {
        const int k = lane - 3;
        const double a = st->x_t[3 + k];
        double sn = 0.0, cs = 1.0;
        if (!(fabs(a) < 10e-5)) sincos(a, &sn, &cs);
        sc[6 + 2 * k] = sn;
        sc[6 + 2 * k + 1] = cs;
    }
}
template <int NW>
__device__ void pass_tables(AlignState* st, const double* s_sc) {
    static_assert(NW >= 4, "T is assembled by wave 3");
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (w == 3 && lane == 0) {
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
    if (t < 69) {
        const double v = angle_table_entry(c_angle_code[t], s_sc[6], s_sc[7], s_sc[8], s_sc[9], s_sc[10], s_sc[11]);
        const int r = t / 3, c = t - 3 * r;
        if (r < 8) { st->jang[r][c] = (float)v; st->jang_d[r][c] = v; }
        else { st->hang[r - 8][c] = (float)v; st->hang_d[r - 8][c] = v; }
    } else if (t >= 96 && t < 104) {
        st->jang[t - 96][3] = 0.f;
    } else if (t >= 104 && t < 120) {
        st->hang[t - 104][3] = 0.f;
    } else if (t >= 120 && t < 123) {
        st->hang[15][t - 120] = 0.f;
    }
    if (t == 0) st->needs_tables = 0;
    lds_barrier();
    if (t == 0) NDT_TAIL_STAMP(3);
}

// convertTransform(x_t) -> T and computeAngleDerivatives(x_t) -> tables, for a workgroup: wave 0 lanes 0-2
// evaluate the f32 AngleAxis sin/cos (the correctly rounded model of the binary's sincosf, ndt_libm.h) while wave 1
// lanes 0-2 evaluate the f64
// angle-derivative sin/cos; then
// wave 3 lane 0 assembles T while threads 0..68 evaluate one table entry each (angle_table_entry: the
// operations of angle_table_row, bit for bit; tests/native/angle_table_check.cpp).
// Same arithmetic as convert_transform / angle_tables in ndt_linalg.h.
template <int NW = kBlock / 64>
__device__ void prepare_pass_parallel(AlignState* st) {
    __shared__ double s_sc[12];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (w == 0 && lane < 3) {
        float sn, cs;
        sincosf_dr2((float)st->x_t[3 + lane], &sn, &cs);
        s_sc[2 * lane] = (double)sn;
        s_sc[2 * lane + 1] = (double)cs;
    } else if (w == 1 && lane < 3) {
        const double a = st->x_t[3 + lane];
        double s = 0.0, c = 1.0;
        if (!(fabs(a) < 10e-5)) sincos(a, &s, &c);
        s_sc[6 + 2 * lane] = s;
        s_sc[6 + 2 * lane + 1] = c;
    }
    lds_barrier();
    if (t == 0) NDT_TAIL_STAMP(2);
    pass_tables<NW>(st, s_sc);
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
// stride: doubles between two values' rows (default: the partials layout of an nb-workgroup grid); partials (+ the
// first column) and stride even
template <int NW = kBlock / 64, int K = 4>
__device__ __forceinline__ void reduce_partials_block(const double* __restrict__ partials, int nb, double* red, int stride = -1) {
    constexpr int Q = (kNumAcc + NW - 1) / NW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ps = stride > 0 ? stride : partial_stride(nb);
    double s[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) s[q] = 0.0;
    for (int c0 = 0; c0 < nb; c0 += 128 * K) {
        double2 x[Q][K];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int v = w + NW * q;
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
        const int v = w + NW * q;
        const double t = wave_allreduce_d(s[q]);
        if (v < kNumAcc && lane == 0) red[v] = t;
    }
    lds_barrier();
}

// reduce_partials_block with the first K0 column pairs' loads issued earlier (partials_preload, beside a leading-tail
// kernel's state staging), summed here in the same order
template <int NW, int K0>
struct PartialsPre {
    double2 x[(kNumAcc + NW - 1) / NW][K0];
};
template <int NW, int K0>
__device__ __forceinline__ void partials_preload(const double* __restrict__ partials, int nb, PartialsPre<NW, K0>& pre) {
    constexpr int Q = (kNumAcc + NW - 1) / NW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ps = partial_stride(nb);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int v = w + NW * q;
#pragma unroll
        for (int k = 0; k < K0; ++k) {
            // unconditional loads from clamped addresses (no branch, so no join resolved by waiting); the entries outside
            // the partials are masked where they are summed
            const int b = min(2 * lane + 128 * k, ps - 2);
            pre.x[q][k] = *reinterpret_cast<const double2*>(partials + (size_t)min(v, kNumAcc - 1) * ps + b);
        }
    }
}
template <int NW, int K, int K0>
__device__ __forceinline__ void reduce_partials_pre(const double* __restrict__ partials, int nb, const PartialsPre<NW, K0>& pre,
                                                    double* red) {
    constexpr int Q = (kNumAcc + NW - 1) / NW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ps = partial_stride(nb);
    double s[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        s[q] = 0.0;
#pragma unroll
        for (int k = 0; k < K0; ++k) {
            const int v = w + NW * q, b = 2 * lane + 128 * k;
            const bool in = v < kNumAcc && b < nb;
            s[q] += in ? pre.x[q][k].x : 0.0;
            s[q] += (in && b + 1 < nb) ? pre.x[q][k].y : 0.0;  // row padding is never written
        }
    }
    for (int c0 = 128 * K0; c0 < nb; c0 += 128 * K) {
        double2 x[Q][K];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int v = w + NW * q;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int b = c0 + 2 * lane + 128 * k;
                x[q][k] = (v < kNumAcc && b < nb) ? *reinterpret_cast<const double2*>(partials + (size_t)v * ps + b)
                                                  : make_double2(0.0, 0.0);
                if (b + 1 >= nb) x[q][k].y = 0.0;
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
        const int v = w + NW * q;
        const double t = wave_allreduce_d(s[q]);
        if (v < kNumAcc && lane == 0) red[v] = t;
    }
    lds_barrier();
}

static_assert(sizeof(AlignState) % 8 == 0, "AlignState is copied as 8-byte words");

// Control part of a pass's tail (the last workgroup, all its threads), on the LDS-staged state: the pass record, the
// Newton / More-Thuente step and the next pass's transform + angle tables.  Initial and full passes hand this pass's H
// and g straight to the Newton solve (control_record_wave copies them; the state machine then asks for the solve unless
// the align ends): wave 0 solves H dp = -g from the reduced values while wave 1 records the pass and runs the state
// machine.
// newton_after_solve (lu_fail = 0) for the step's common outcome, in registers, by every lane of a wave (uniform values):
// the same expressions on the same inputs, so the same bits.  Returns false where the general function takes another
// branch (a zero / NaN step, a zero slope); xt, dir, phi_0, d_phi_0, a_t are then not set.  The six divisions of the
// normalisation run one per lane (an f64 division's scale / fmas pair goes through VCC, so six in one lane serialise)
// and are broadcast back.
struct StepRegs {
    double xt[6], dir[6], phi_0, d_phi_0, a_t;
};
__device__ __forceinline__ bool after_solve_regs(const AlignState& st, const double* dp_in, StepRegs& o) {
    const int lane = threadIdx.x & 63;
    double dp[6], p[6], g[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) { dp[k] = dp_in[k]; p[k] = st.p[k]; g[k] = st.g[k]; }
    const double score = st.score, step_max = st.step_max, step_min = st.step_min;
    const double nrm2 = dot6(dp, dp);
    const double norm = sqrt(nrm2);
    if (norm == 0 || norm != norm) return false;
    if (nrm2 > 0) {
        const double sq = sqrt(nrm2);
        double mine = dp[0];
#pragma unroll
        for (int k = 1; k < 6; ++k)
            if (lane == k) mine = dp[k];
        const double q = mine / sq;
#pragma unroll
        for (int k = 0; k < 6; ++k) dp[k] = readlane_d(q, k);
    }
    o.phi_0 = -score;
    double d_phi_0 = -dot6(g, dp);
    if (d_phi_0 >= 0) {
        if (d_phi_0 == 0) return false;
        d_phi_0 *= -1;
#pragma unroll
        for (int k = 0; k < 6; ++k) dp[k] *= -1;
    }
    o.d_phi_0 = d_phi_0;
    double a_t = norm;
    a_t = smin(a_t, step_max);
    a_t = smax(a_t, step_min);
    o.a_t = a_t;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        o.dir[k] = dp[k];
        o.xt[k] = p[k] + dp[k] * a_t;
    }
    return true;
}
// ... and its state writes (+ prepare_pass(PASS_FULL)), one field per lane of the calling wave
__device__ __forceinline__ void after_solve_store(AlignState& st, const StepRegs& o, int needs_tables) {
    const int lane = threadIdx.x & 63;
    const double mu = 1.e-4;
    const double phi_0 = o.phi_0, d_phi_0 = o.d_phi_0;
    // the interval's ends, uniform (computed before the per-lane stores, as newton_after_solve's expressions)
    const double a_l = 0, a_u = 0;
    const double f_l = phi_0 - phi_0 - mu * d_phi_0 * a_l, g_l = d_phi_0 - mu * d_phi_0;
    const double f_u = phi_0 - phi_0 - mu * d_phi_0 * a_u, g_u = d_phi_0 - mu * d_phi_0;
    const int ic = (st.step_max - st.step_min) > 0;
    if (lane < 6) {
        double d = 0.0, x = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (lane == k) { d = o.dir[k]; x = o.xt[k]; }
        st.dir[lane] = d;
        st.x_t[lane] = x;
        st.x_eval[lane] = x;
    } else if (lane == 6) {
        st.phi_0 = phi_0;
        st.d_phi_0 = d_phi_0;
    } else if (lane == 7) {
        st.a_l = a_l;
        st.f_l = f_l;
        st.g_l = g_l;
    } else if (lane == 8) {
        st.a_u = a_u;
        st.f_u = f_u;
        st.g_u = g_u;
    } else if (lane == 9) {
        st.interval_converged = ic;
        st.open_interval = 1;
        st.step_iterations = 0;
        st.a_t = o.a_t;
    } else if (lane == 10) {
        st.want_solve = 0;
        st.svd_ready = 0;
        st.pass_kind = PASS_FULL;
        st.pending = 1;
        st.needs_tables = needs_tables;
    }
}

// tail_control's fast paths (see there): 1 = the step on one lane, then the sin / cos on one wave; 3 = the step in
// registers on waves 0 and 1, the f32 and the f64 sin / cos on one wave each
#ifndef NDT_TAIL_FAST
#define NDT_TAIL_FAST 3
#endif
template <int NW, int FAST = NDT_TAIL_FAST>
__device__ __forceinline__ void tail_control(AlignState& s_st, const double* red, PassRecordDev* hist, int hist_cap,
                                             unsigned long long* ts) {
    __shared__ double s_spec_dp[6];
    __shared__ int s_spec_fail;
    const bool spec = s_st.phase == 0 || s_st.pass_kind == PASS_FULL;
    const int wv = threadIdx.x >> 6;
    double x_lu[6];
    if (wv == 0) {
        if (spec) {
            if (threadIdx.x == 0) NDT_TAIL_STAMP(6);
            const int f = lu6_solve_rows(red + 7, red + 1, s_spec_dp, true, x_lu);
            if (threadIdx.x == 0) {
                s_spec_fail = f;
                NDT_TAIL_STAMP(7);
            }
        }
    } else if (wv == 1) {
        control_record_wave(&s_st, red, hist, hist_cap);
        if ((threadIdx.x & 63) == 0) NDT_TAIL_STAMP(4);
        if (FAST == 3) {
            control_step_wave(&s_st, red);
        } else if ((threadIdx.x & 63) == 0) {
            control_step(&s_st, red);
        }
        if ((threadIdx.x & 63) == 0) NDT_TAIL_STAMP(5);
    }
    bool tables_done = false;
    if (FAST == 3) {
        // fast path 3 (the Newton step after a speculatively solved direction, nearly every pass): after the state
        // machine asked for the solve, waves 0, 1 and 2 each take the step in registers (wave 0 from its LU registers,
        // the others from the LDS copy: the same bits); wave 0 builds T (the f32 AngleAxis sin / cos on lanes 0-2), wave 1
        // the angle tables (the f64 sin / cos on lanes 0-2, one entry per lane), wave 2 writes the state one field per
        // lane, side by side; one barrier ends the tail.  Anything else continues as solve_loop / prepare_pass_parallel.
        // the angle-table codes of wave 1's entries (t = lane, 64 + lane), loaded now, used after the state machine
        const int lane = threadIdx.x & 63;
        const unsigned code0 = (wv == 1) ? c_angle_code[lane] : 0u;
        const unsigned code1 = (wv == 1 && lane < 5) ? c_angle_code[64 + lane] : 0u;
        __shared__ int s_go3;
        __shared__ double s_fv3[8];
        lds_barrier();
        if (spec && s_st.want_solve && !s_spec_fail) {  // uniform
            if (wv <= 2) {
                StepRegs o;
                double dpi[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) dpi[k] = wv == 0 ? x_lu[k] : s_spec_dp[k];
                const bool ok = after_solve_regs(s_st, dpi, o);
                double xa = 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (lane == k) xa = o.xt[3 + k];
                if (wv == 0) {
                    // convertTransform(x_t): the f32 AngleAxis sin / cos on lanes 0-2, broadcast, T on lane 0 (the
                    // operations of pass_tables' T), the constant table columns; then the state writes
                    float sn = 0.f, cs = 1.f;
                    if (ok && lane < 3) sincosf_dr2((float)xa, &sn, &cs);
                    float sa[3], ca[3];
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        sa[a] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sn), a));
                        ca[a] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cs), a));
                    }
                    if (ok) {
                        if (lane == 0) {
                            float R3[3][9];
                            for (int a = 0; a < 3; ++a) angle_axis_sc(sa[a], ca[a], a, R3[a]);
                            float Rxy[9], R[9];
                            mat3_mul_f(R3[0], R3[1], Rxy);
                            mat3_mul_f(Rxy, R3[2], R);
                            for (int j = 0; j < 3; ++j)
                                for (int i = 0; i < 3; ++i) s_st.T[i + 4 * j] = R[i + 3 * j];
                            s_st.T[3] = 0.f; s_st.T[7] = 0.f; s_st.T[11] = 0.f;
                            s_st.T[12] = (float)o.xt[0]; s_st.T[13] = (float)o.xt[1]; s_st.T[14] = (float)o.xt[2]; s_st.T[15] = 1.f;
                        } else if (lane >= 32 && lane < 40) {
                            s_st.jang[lane - 32][3] = 0.f;
                        } else if (lane >= 40 && lane < 56) {
                            s_st.hang[lane - 40][3] = 0.f;
                        } else if (lane >= 56 && lane < 59) {
                            s_st.hang[15][lane - 56] = 0.f;
                        }
                    }
                    if (threadIdx.x == 0) s_go3 = ok ? 1 : 0;
                } else if (wv == 2) {
                    // the state writes, one field per lane, beside waves 0 and 1 (p, g, score and the step bounds it
                    // read are written by no one here)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                    if (ok) after_solve_store(s_st, o, 0);
                } else {
                    // computeAngleDerivatives(x_t): the f64 sin / cos on lanes 0-2, the eight factors {1, sx, cx, sy,
                    // cy, sz, cz, 0} through LDS, entry t = lane (and 64 + lane) on every lane: angle_table_entry's
                    // operations with its factor lookups as indexed LDS reads
                    double sn = 0.0, cs = 1.0;
                    if (ok && lane < 3 && !(fabs(xa) < 10e-5)) sincos(xa, &sn, &cs);
                    if (lane < 3) {
                        s_fv3[1 + 2 * lane] = sn;
                        s_fv3[2 + 2 * lane] = cs;
                    } else if (lane == 3) {
                        s_fv3[0] = 1.0;
                        s_fv3[7] = 0.0;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
                    if (ok) {
#pragma unroll
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
                    }
                }
            }
            lds_barrier();
            if (s_go3) {
                if (ts && threadIdx.x == 0) ts[7] = __builtin_amdgcn_s_memrealtime();
                if (threadIdx.x == 0) { NDT_TAIL_STAMP(0); NDT_TAIL_STAMP(1); NDT_TAIL_STAMP(2); NDT_TAIL_STAMP(3); }
                tables_done = true;
            }
        }
    }
    if (FAST == 1) {
    // fast path (the Newton step after a speculatively solved direction, nearly every pass): wave 0 takes the step
    // (lane 0) and, without a workgroup barrier, the sin/cos of the new angles (lanes 0-5); one barrier, then T and the
    // tables.  Any other case (a second solve request, a paused chain) continues as solve_loop / prepare_pass_parallel.
    __shared__ double s_sc[12];
    lds_barrier();
    if (spec && s_st.want_solve) {
        if (wv == 0) {
            if (threadIdx.x == 0) {
                NDT_TAIL_STAMP(0);
                NDT_TAIL_STAMP(1);
                newton_after_solve(&s_st, s_spec_dp, s_spec_fail);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            if (!s_st.want_solve && s_st.needs_tables) pass_sincos_wave(&s_st, s_sc);
        }
        lds_barrier();
        if (!s_st.want_solve) {
            if (ts && threadIdx.x == 0) ts[7] = __builtin_amdgcn_s_memrealtime();
            if (threadIdx.x == 0) NDT_TAIL_STAMP(2);
            if (s_st.needs_tables) pass_tables<NW>(&s_st, s_sc);
            tables_done = true;
        }
    }
    }
    if (!tables_done) {
        solve_loop(&s_st, spec ? s_spec_dp : nullptr, &s_spec_fail);
        if (ts && threadIdx.x == 0) ts[7] = __builtin_amdgcn_s_memrealtime();
        if (s_st.needs_tables) prepare_pass_parallel<NW>(&s_st);
    }
    if (ts && threadIdx.x == 0) ts[5] = __builtin_amdgcn_s_memrealtime();
}

// Epilogue of every derivative pass (all threads of every workgroup call it); returns true in the workgroup that ran
// the tail.
//  1. workgroup partials -> partials[v][block] (reduce-scatter block reduction);
//  2. hand-off (Guideline 16, recipe R1): partials stored write-through (sc1), every storing wave drains
//     (vmcnt 0), workgroup barrier, one lane takes a ticket on `counter`; the workgroup that draws the last
//     ticket acquires (agent scope) and reads them with plain loads;
//  3. that last workgroup reduces all partials in a fixed order and either publishes them (mode 1: test hook)
//     or runs the Newton / More-Thuente control step on the LDS-staged state and prepares the next pass
//     (mode 0), then re-arms the ticket counter for the next launch.
// The align is therefore one kernel per derivative pass with no host round trip and no separate reduce /
// control launches; results are bitwise deterministic (no float atomics, fixed orders).
// pass_handoff: steps 2-3 above, after the workgroup's partials were stored write-through (step 1).
// K: the partial reduction's column pairs per lane and round trip (reduce_partials_block)
template <int NW = kBlock / 64, int K = 4>
__device__ __forceinline__ bool pass_handoff(AlignState* st, double* partials, unsigned* counter, double* red_out, PassRecordDev* hist,
                                             int hist_cap, int mode, unsigned long long* ts) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // profiling stamps are single plain stores (no atomics on shared words): the pass start by workgroup 0 (dispatched
    // first), everything else by the last workgroup (the last body to finish draws the last ticket)
    const unsigned long long t_body = ts ? __builtin_amdgcn_s_memrealtime() : 0ull;
#ifdef NDT_BODY_STAMPS
    NDT_BLK_STAMP(st->n_passes, 4);
#endif
    __shared__ unsigned s_ticket;
    __shared__ double red[kNumAcc];
    // two-level hand-off (grids of more than kTwoLevelMinBlocks workgroups, e.g. one 256-point tile per workgroup over a
    // 1 M-point scan): the last workgroup of each group of G consecutive workgroups sums the group's columns in index
    // order into the group partials, and the last group's closer sums those — the final tail reads ~64 columns instead
    // of thousands, and the group sums run beside the other groups' bodies.  Fixed orders: deterministic.
    const int nb = gridDim.x;
    const bool two = nb > kTwoLevelMinBlocks;
    const int G = group_size(nb), ng = (nb + G - 1) / G;
    const int ps = partial_stride(nb);
    double* gpart = partials + (size_t)kNumAcc * ps;
    if (two) {
        const int g = blockIdx.x / G, members = min(G, nb - g * G);
        unsigned* gt = counter + kGroupTicketBase + kGroupTicketStride * g;
        if (threadIdx.x == 0) s_ticket = __hip_atomic_fetch_add(gt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (s_ticket != (unsigned)members - 1) return false;
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(gt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next launch
        }
        __syncthreads();
        reduce_partials_block<NW, K>(partials + (size_t)g * G, members, red, ps);
        if ((int)threadIdx.x < kNumAcc)
            __hip_atomic_store(gpart + (size_t)threadIdx.x * kMaxGroups + g, red[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        // the partials were stored write-through (sc1) and drained by the storing wave before the barrier above,
        // so the ticket needs no release fence (no L2 write-back); the last workgroup still acquires below
        s_ticket = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_ticket != (two ? (unsigned)ng : gridDim.x) - 1) return false;
    if (ts && threadIdx.x == 0) ts[2] = t_body;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (ts) ts[3] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    // the optimiser state is fetched together with the partials (one memory round trip for both)
    constexpr int B = 64 * NW;
    static_assert(sizeof(AlignState) / 8 <= 2 * B, "AlignState staging assumes <= 2 words per thread");
    constexpr int kWords = sizeof(AlignState) / 8;
    unsigned long long* gw = reinterpret_cast<unsigned long long*>(st);
    unsigned long long sv0 = 0, sv1 = 0;
    if (mode == 0) {
        if ((int)threadIdx.x < kWords) sv0 = gw[threadIdx.x];
        if ((int)threadIdx.x + B < kWords) sv1 = gw[threadIdx.x + B];
    }
#ifdef NDT_BODY_STAMPS
    if (threadIdx.x == 0) {
        const int p = st->n_passes;
        g_tail_ts = p < kBlkPasses ? &g_blk_ts[((size_t)p * kBlkMax + kBlkMax - 1) * kBlkSlots] : nullptr;
        g_tail_wg = blockIdx.x;
    }
#endif
    if (two) reduce_partials_block<NW, K>(gpart, ng, red, kMaxGroups);
    else reduce_partials_block<NW, K>(partials, gridDim.x, red);
    if (ts && threadIdx.x == 0) ts[4] = __builtin_amdgcn_s_memrealtime();
    if (mode == 1) {
        if (threadIdx.x < kNumAcc) red_out[threadIdx.x] = red[threadIdx.x];
        if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
    }
    __shared__ AlignState s_st;
    unsigned long long* lw = reinterpret_cast<unsigned long long*>(&s_st);
    if ((int)threadIdx.x < kWords) lw[threadIdx.x] = sv0;
    if ((int)threadIdx.x + B < kWords) lw[threadIdx.x + B] = sv1;
    lds_barrier();
    if (ts && threadIdx.x == 0) ts[6] = __builtin_amdgcn_s_memrealtime();
    tail_control<NW>(s_st, red, hist, hist_cap, ts);
    for (int k = threadIdx.x; k < kWords; k += B) gw[k] = lw[k];
    if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

template <int NW = kBlock / 64>
__device__ __forceinline__ bool pass_epilogue(double (&acc)[kNumAcc], double* redw, AlignState* st, double* partials,
                                              unsigned* counter, double* red_out, PassRecordDev* hist, int hist_cap, int mode,
                                              unsigned long long* ts) {
    block_reduce_store<kNumAcc, NW>(acc, redw, partials + blockIdx.x, partial_stride(gridDim.x));
    return pass_handoff<NW>(st, partials, counter, red_out, hist, hist_cap, mode, ts);
}

}  // namespace ndt
