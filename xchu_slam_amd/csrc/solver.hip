// solver.hip — device-side Newton / More-Thuente driver (computeTransformation, ndt_omp_impl.hpp:73-164,
// computeStepLengthMT :760-916, updateIntervalMT :646-677, trialValueSelectionMT :682-757).
//
// One tiny workgroup per derivative pass: reduces the per-workgroup partials of the pass in a fixed order
// (deterministic f64), records the pass in the history, then advances the optimiser state machine and
// prepares the transform + angle tables of the next pass.  The whole align therefore runs as a chain of
// (pass, control) kernel pairs without a host round trip; the chain is captured once in a hipGraph.
#include "ndt_device.h"

namespace ndt {

__device__ __forceinline__ double dot6(const double* a, const double* b) {
    double s = a[0] * b[0];
    for (int k = 1; k < 6; ++k) s += a[k] * b[k];
    return s;
}

__device__ void prepare_pass(AlignState* st, int kind) {
    convert_transform(st->x_t, st->T);
    angle_tables(st->x_t, st->jang, st->hang, st->jang_d, st->hang_d);
    for (int k = 0; k < 6; ++k) st->x_eval[k] = st->x_t[k];
    st->pass_kind = kind;
    st->pending = 1;
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
        st->solver_fallbacks += solve6(st->H, mg, dp);
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
        for (int k = 0; k < 6; ++k) { h.x[k] = st->x_eval[k]; h.g[k] = r[1 + k]; }
        h.score = r[0];
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

// Deterministic reduction of one pass's partials [kNumAcc][nb] -> red[kNumAcc]: one workgroup per value
// (44 workgroups spread the 8*44*nb bytes over many CUs); each thread sums a fixed strided subset, then a
// fixed wave butterfly and the four waves in index order.
__global__ __launch_bounds__(kBlock) void k_reduce_partials(const AlignState* __restrict__ st, const double* __restrict__ partials,
                                                            int nb, double* __restrict__ red_out, int force) {
    if (!force && (st->done || !st->pending)) return;
    const int v = blockIdx.x;
    const double* col = partials + (size_t)v * nb;
    double s = 0.0;
    for (int b0 = threadIdx.x; b0 < nb; b0 += kBlock * 4) {
        double x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) { const int b = b0 + kBlock * k; x[k] = b < nb ? col[b] : 0.0; }
#pragma unroll
        for (int k = 0; k < 4; ++k) s += x[k];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += shfl_xor_d(s, m);
    __shared__ double w4[4];
    if ((threadIdx.x & 63) == 0) w4[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = w4[0];
        t += w4[1];
        t += w4[2];
        t += w4[3];
        red_out[v] = t;
    }
}

static_assert(sizeof(AlignState) % 8 == 0, "AlignState is copied as 8-byte words");

// One control step per pass: the optimiser state is staged in LDS (one coalesced read and write per
// launch) so that the single-lane Newton / More-Thuente logic runs on LDS latency, not HBM latency.
__global__ __launch_bounds__(kBlock) void k_control(AlignState* __restrict__ st, const double* __restrict__ red_in,
                                                    PassRecordDev* __restrict__ hist, int hist_cap) {
    if (st->done || !st->pending) return;
    __shared__ AlignState s_st;
    __shared__ double red[kNumAcc];
    constexpr int kWords = sizeof(AlignState) / 8;
    unsigned long long* gw = reinterpret_cast<unsigned long long*>(st);
    unsigned long long* lw = reinterpret_cast<unsigned long long*>(&s_st);
    for (int k = threadIdx.x; k < kWords; k += kBlock) lw[k] = gw[k];
    if (threadIdx.x < kNumAcc) red[threadIdx.x] = red_in[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) control_step(&s_st, red, hist, hist_cap);
    __syncthreads();
    for (int k = threadIdx.x; k < kWords; k += kBlock) gw[k] = lw[k];
}

// Aligned output cloud: source transformed by final_transformation_ (pcl::transformPointCloud).
__global__ __launch_bounds__(kBlock) void k_transform(const float4* __restrict__ src, int n, const AlignState* __restrict__ st,
                                                      float4* __restrict__ out) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float* T = st->T;
    const float4 p = src[i];
    float4 o;
    o.x = T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12];
    o.y = T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13];
    o.z = T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14];
    o.w = 1.0f;
    out[i] = o;
}

__global__ void k_ts_init(unsigned long long* ts, int n) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) ts[2 * i] = ~0ull;
}

}  // namespace ndt
