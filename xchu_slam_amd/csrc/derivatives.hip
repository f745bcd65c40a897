// derivatives.hip — the NDT derivative pass (score, gradient, Hessian over all source points).
//
// Reference: pclomp::NormalDistributionsTransform::computeDerivatives (ndt_omp_impl.hpp:175-283),
// computePointDerivatives (:401-445), updateDerivatives (:491-548), and for the radius paths
// computeHessian/updateHessian (:550-641) + pcl::NormalDistributionsTransform (pcl_ndt mode).
//
// MI355X mapping: one thread per source point (grid-stride over a fixed grid => fixed summation order),
// the point is transformed on the fly from the original cloud (no transformed-cloud round trip through
// HBM), voxel neighbours come from an open-addressing hash probe, each (point, voxel) pair reads one
// 64 B VoxelRec, per-pair math is f32 exactly as the reference (its dense 4x6/24x6 products restated
// sparsely: the skipped terms are exact zeros), and the 43 sums are accumulated in f64 per thread,
// reduced by a fixed wave butterfly + LDS into per-workgroup partials.  No atomics => bitwise
// run-to-run determinism.  Memory-bound gather + reduction, no MFMA.
#include "ndt_control.h"

namespace ndt {

// exp_dr's 2^(i/64) double-double table (ndt_libm.h), staged into LDS by every kernel that evaluates pairs: exp_dr looks up
// one 16-byte (hi, lo) entry per lane
__constant__ unsigned long long c_exp_tab[kExpTabLen] = {NDT_EXP2_64_TAB};
__device__ __forceinline__ void stage_exp_tab(double* s_exp) {
    if (threadIdx.x < kExpTabLen) s_exp[threadIdx.x] = __longlong_as_double((long long)c_exp_tab[threadIdx.x]);
}

// Split accumulation (ndt_device.h): a lane keeps 22 f64 sums instead of 44 (88 -> 44 VGPRs), every pair's terms exchanged
// across the half-waves as they are produced (22 v_permlane32_swap per pair); NDT_SPLIT_ACC=0 (ndt_types.h): every lane
// keeps all 44 sums.
constexpr int kBodyAcc = NDT_SPLIT_ACC ? kSplitAcc : kNumAcc;
// record register sets of the pair loop: 2 (one gather in flight behind a pair's math) or 3 (two)
#ifndef NDT_REC_SETS
#define NDT_REC_SETS 2
#endif

// The pair sink of split accumulation.  put(k, lo, hi): this lane's low term k and high term k; after the swap lanes 0-31
// hold the low term k of their own pair and of lane + 32's, lanes 32-63 the high term k of lane - 32's pair and of their
// own.  A pair that does not count (rejected, or a lane past the tile's pairs) hands over zeros (pair_pk_terms<true>), so
// the sums are plain adds, no branch.
struct SplitSink {
    double* acc;
    __device__ __forceinline__ void put(int k, float lo, float hi) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
        acc[k] += (double)__uint_as_float(r[0]);
        acc[k] += (double)__uint_as_float(r[1]);
    }
    // (g0, g1), (g2, g3), (g4, g5): low score, g0, g1, g2 / high g3, g4, g5 and the pair-count slot (0 here)
    __device__ __forceinline__ void grad(float score_inc, pf2 G01, pf2 G23, pf2 G45) {
        put(0, score_inc, G23[1]);
        put(1, G01[0], G45[0]);
        put(2, G01[1], G45[1]);
        put(3, G23[0], 0.f);
    }
    // row i: low H_i0..H_i2, high H_i3..H_i5
    __device__ __forceinline__ void row(int i, pf2 T01, pf2 T23, pf2 T45) {
        put(4 + 3 * i, T01[0], T23[1]);
        put(5 + 3 * i, T01[1], T45[0]);
        put(6 + 3 * i, T23[0], T45[1]);
    }
};

// DIRECT7 offsets (centre, then +-x, +-y, +-z) as a compile-time function: the unrolled probes take them as immediates
// (a __constant__ table is read with scalar loads in every pass's probe phase)
__host__ __device__ constexpr int rel7(int r, int a) { return r == 0 ? 0 : (a == (r - 1) / 2 ? ((r & 1) ? 1 : -1) : 0); }
static_assert(rel7(0, 0) == 0 && rel7(1, 0) == 1 && rel7(2, 0) == -1 && rel7(3, 1) == 1 && rel7(4, 1) == -1 && rel7(5, 2) == 1 &&
                  rel7(6, 2) == -1 && rel7(3, 0) == 0 && rel7(6, 1) == 0,
              "DIRECT7 order: centre, +x, -x, +y, -y, +z, -z");
// pcl::getAllNeighborCellIndices(): 13 "half" offsets then their negations (the centre cell is NOT included)
__constant__ int c_rel26[26][3] = {
    {-1, -1, -1}, {-1, 0, -1}, {-1, 1, -1}, {0, -1, -1}, {0, 0, -1}, {0, 1, -1}, {1, -1, -1}, {1, 0, -1}, {1, 1, -1},
    {-1, -1, 0}, {0, -1, 0}, {1, -1, 0}, {-1, 0, 0},
    {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, 1, 1}, {0, 0, 1}, {0, -1, 1}, {-1, 1, 1}, {-1, 0, 1}, {-1, -1, 1},
    {1, 1, 0}, {0, 1, 0}, {-1, 1, 0}, {1, 0, 0}};

struct PointTerms {
    float x[3];      // original point (computePointDerivatives uses the untransformed point)
    float xt[3];     // transformed point
    float xj[8];     // j_ang * x   (eq. 6.19)
    float xh[15];    // h_ang * x   (eq. 6.21)
};

__device__ __forceinline__ void load_point_terms(const float4 p, const AlignState* __restrict__ st, PointTerms& t, bool hess) {
    const float* T = st->T;
    t.x[0] = p.x; t.x[1] = p.y; t.x[2] = p.z;
    // pcl::transformPointCloud: ((m0*x + m1*y) + m2*z) + m3, f32
    t.xt[0] = T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12];
    t.xt[1] = T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13];
    t.xt[2] = T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        float acc = st->jang[r][0] * p.x;
        acc += st->jang[r][1] * p.y;
        acc += st->jang[r][2] * p.z;
        t.xj[r] = acc;
    }
    if (hess) {
#pragma unroll
        for (int r = 0; r < 15; ++r) {
            float acc = st->hang[r][0] * p.x;
            acc += st->hang[r][1] * p.y;
            acc += st->hang[r][2] * p.z;
            t.xh[r] = acc;
        }
    }
}

// computePointDerivatives terms of one source point (ndt_omp_impl.hpp:448-488, f32): the reference evaluates
// them for every (point, voxel) pair; they depend on the point only, so the pass computes them once per point
// into LDS and every pair of the point reads the same values.
// Stored in the order the pair math reads it: natural (xj[8], xh[15], pad) for pair_f32, or pk_terms' f32 pairs for
// pair_pk (NDT_PACKED_PAIR, ndt_pair.h).
struct __align__(16) PointDeriv {
    float v[24];
};
static_assert(sizeof(PointDeriv) == 96, "PointDeriv is six float4");
static_assert(kPkTerms == 24, "pk_terms fill a PointDeriv");

// tab: the f32 angle tables of the pass, j_ang (8 x 4) followed by h_ang (16 x 4) as in AlignState, read from LDS
// (k_pass_lead's staged state, k_pass_direct's staged copy): uniform-address broadcasts instead of a chain of scalar
// loads per tile
template <bool PACKED>
__device__ __forceinline__ void point_deriv(const float4 p, const float* __restrict__ tab, PointDeriv& d, bool hess) {
    float xj[8], xh[15];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        float acc = tab[4 * r + 0] * p.x;
        acc += tab[4 * r + 1] * p.y;
        acc += tab[4 * r + 2] * p.z;
        xj[r] = acc;
    }
#pragma unroll
    for (int r = 0; r < 15; ++r) {
        float acc = 0.f;
        if (hess) {
            acc = tab[32 + 4 * r + 0] * p.x;
            acc += tab[32 + 4 * r + 1] * p.y;
            acc += tab[32 + 4 * r + 2] * p.z;
        }
        xh[r] = acc;
    }
    if (PACKED) {
        pk_terms(xj, xh, d.v);
    } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) d.v[r] = xj[r];
#pragma unroll
        for (int r = 0; r < 15; ++r) d.v[8 + r] = xh[r];
        d.v[23] = 0.f;
    }
}
static_assert(offsetof(AlignState, hang) == offsetof(AlignState, jang) + 32 * sizeof(float), "h_ang follows j_ang");

// A VoxelRec gathered as four 16-byte words (one dwordx4 load each, straight into the registers the pair math
// reads), and its field view.
struct RecRaw {
    uint4 a, b, c, d;
};
__device__ __forceinline__ RecRaw load_rec(const VoxelRec* __restrict__ recs, int idx) {
    const uint4* p = reinterpret_cast<const uint4*>(recs + idx);
    // npts (the last word) is not read by the pair math: 15 dwords, one register fewer per record in flight
    const uint3 d = *reinterpret_cast<const uint3*>(p + 3);
    return RecRaw{p[0], p[1], p[2], make_uint4(d.x, d.y, d.z, 0u)};
}
struct RecView {
    double mean[3];
    float icov[9];
};
__device__ __forceinline__ RecView rec_view(const RecRaw& r) {
    RecView v;
    v.mean[0] = join_d(r.a.x, r.a.y);
    v.mean[1] = join_d(r.a.z, r.a.w);
    v.mean[2] = join_d(r.b.x, r.b.y);
    v.icov[0] = __uint_as_float(r.b.z); v.icov[1] = __uint_as_float(r.b.w);
    v.icov[2] = __uint_as_float(r.c.x); v.icov[3] = __uint_as_float(r.c.y); v.icov[4] = __uint_as_float(r.c.z);
    v.icov[5] = __uint_as_float(r.c.w);
    v.icov[6] = __uint_as_float(r.d.x); v.icov[7] = __uint_as_float(r.d.y); v.icov[8] = __uint_as_float(r.d.z);
    return v;
}
static_assert(offsetof(VoxelRec, icov) == 24 && offsetof(VoxelRec, npts) == 60, "RecRaw decode assumes the VoxelRec layout");

// pair_f32 operand view: transformed point + the point's derivative record (both from LDS)
struct PairPoint {
    float xt[3];
    const float* xj;
    const float* xh;
};

// A (point, voxel) pair of a tile in LDS: int2 (tile-local point, cloud index), or packed into one word (cloud index << 10
// | tile-local point) where a tile holds two points per thread — the pair list then takes half the LDS, so that two
// workgroups still fit a CU (the host packs only when every cloud index is below 2^22).
template <int PPT> struct PairSlot;
template <> struct PairSlot<1> {
    using T = int2;
    __device__ static T pack(int pt, int vox) { return make_int2(pt, vox); }
    __device__ static int point(T s) { return s.x; }
    __device__ static int voxel(T s) { return s.y; }
};
template <> struct PairSlot<2> {
    using T = unsigned;
    __device__ static T pack(int pt, int vox) { return ((unsigned)vox << 10) | (unsigned)pt; }
    __device__ static int point(T s) { return (int)(s & 1023u); }
    __device__ static int voxel(T s) { return (int)(s >> 10); }
};

#ifndef NDT_OWN_FIRST
#define NDT_OWN_FIRST 1
#endif
// a wave-uniform double moved to SGPRs (its two halves read from the first active lane)
__device__ __forceinline__ double uniform_d(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Direct-neighbourhood pass (DIRECT7 / DIRECT26 / DIRECT1).  Per tile of up to PPT * B points (PPT per thread):
//   1. probe: every thread transforms its points and issues all PPT * NREL voxel lookups independently
//      (dense cell grid: one 4 B load per probe, +-x neighbours on the same cache line);
//   2. compact: a block exclusive scan of the per-thread hit counts lays the (point, voxel) pairs out
//      in LDS in (thread, point, neighbour-order) order — deterministic, no atomics;
//   3. pair math: threads take pairs round-robin, gather the 64 B voxel record and run updateDerivatives.
// Pair math is therefore dense (no divergence on misses) and memory latency is exposed once per phase; two points per
// thread halve the tiles of a workgroup and with them the per-tile latency chains (probe round trip, scan barriers,
// first record gather).
// ONE_TILE: the geometry gives every workgroup one tile (no tile loop, no next tile's points): the sums are then not live
// across the probe phase, which keeps the kernel within three waves' registers.
// EPRE: the first tile's neighbour cache entries arrive in e_first (loaded at kernel start); false: loaded here like
// every later tile's (the leading-tail kernel's hash-grid instantiation: e_first stays live into one body only, which
// keeps the one-tile kernel free of scratch)
template <int SEARCH, bool DENSE, int B, int PPT = 1, bool ONE_TILE = false, bool EPRE = true, bool PPRE = EPRE>
__device__ __forceinline__ void direct_pass_body(const float4* __restrict__ src, int n, int ppb, const GridHeader* __restrict__ hdr,
                                                 const int2* __restrict__ table, const int* __restrict__ grid,
                                                 const VoxelRec* __restrict__ recs, const AlignState* __restrict__ st, double* acc,
                                                 long long& pairs, int pidx, const float4 (&p_first)[PPT],
                                                 const int4 (&e_first)[PPT][2], float4* s_xt, PointDeriv* s_pd,
                                                 typename PairSlot<PPT>::T* s_pair, int* s_scan, const float* __restrict__ tab,
                                                 const double* __restrict__ etab, int4* __restrict__ nbr) {
    using PS = PairSlot<PPT>;
    constexpr int NREL = SEARCH == S_DIRECT26 ? 26 : (SEARCH == S_DIRECT1 ? 1 : 7);
    constexpr bool kOwn = NDT_OWN_FIRST && PPT == 1 && NDT_SPLIT_ACC && NDT_REC_SETS != 3;
    const bool hess = st->pass_kind == PASS_FULL;
    // the Gaussian constants are uniform: held in SGPRs through the pair loop (LDS-staged state reads land in VGPRs)
    const float gd2 = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int((float)st->gauss_d2)));
    const double d1 = uniform_d(st->gauss_d1);
    const bool empty = hdr->empty != 0;
    const float leaf0 = hdr->leaf[0], leaf1 = hdr->leaf[1], leaf2 = hdr->leaf[2];
    const int mb0 = hdr->min_b[0], mb1 = hdr->min_b[1], mb2 = hdr->min_b[2];
    const int xb0 = hdr->max_b[0], xb1 = hdr->max_b[1], xb2 = hdr->max_b[2];
    const int dm1 = hdr->divb_mul[1], dm2 = hdr->divb_mul[2];
    const unsigned log2cap = hdr->log2cap;
    const long long cells = hdr->cells;
    const float* T = st->T;
    // Neighbour cache (DIRECT7): per source point of this align, the halo cell its transformed point fell in and that
    // cell's seven probe results, 32 B.  The neighbour set of a point is a function of its cell alone (the grid does
    // not change during an align), so a point whose cell is unchanged since the previous direct pass reuses it instead
    // of issuing seven scattered grid loads; the first pass of an align writes every entry.  Halo cell: the cell
    // shifted by one so that the one-cell border around the grid, whose points still reach grid cells, is indexed too;
    // cells further out have no neighbours at all (key -1, no loads).
    constexpr bool kNC = NREL == 7;
    const int hd0 = hdr->div_b[0] + 2, hd1 = hdr->div_b[1] + 2, hd2 = hdr->div_b[2] + 2;
    const bool nc_on = kNC && nbr != nullptr && (long long)hd0 * hd1 * hd2 < 0x7fffffffLL;
    const bool nc_read = nc_on && pidx > 0;
    const int hm1 = hd0, hm2 = hd0 * hd1;
    // tiles of ppb (<= PPT * B) points: tile t of this workgroup covers [(blockIdx + t*grid) * ppb, +ppb); thread k holds
    // tile-local points k, k + B, ...  The next tile's points are loaded at the top of each tile (one HBM round trip
    // hidden behind this tile's work).
    // PPRE false (k_pass_direct's second body instantiation, a hash grid): the first tile's points are loaded here, not
    // taken from the caller's registers — the dense / hash dispatch is structured as then-block, flow, else-block, so a
    // value the else-body reads is live through the whole then-body (C5's kernel: 256 VGPRs + 8 B of scratch -> 253, none;
    // C4 1980 -> 1998 pairs/s).  The leading-tail kernel keeps its points (C2 1261 vs 1247 scans/s the other way).
    float4 p_cur[PPT];
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
        if (PPRE) {
            p_cur[q] = p_first[q];
        } else {
            const int li = (int)threadIdx.x + q * B, i0 = blockIdx.x * ppb + li;
            p_cur[q] = (li < ppb && i0 < n) ? src[i0] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
#ifdef NDT_BODY_STAMPS
    unsigned long long t_mark = 0, t_acc[3] = {0ull, 0ull, 0ull};
#endif
    for (int base = blockIdx.x * ppb; base < n; base += gridDim.x * ppb) {
#ifdef NDT_BODY_STAMPS
        __syncthreads();
        t_mark = __builtin_amdgcn_s_memrealtime();
#endif
        float4 p[PPT];
        bool on[PPT];
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
            const int li = (int)threadIdx.x + q * B;
            p[q] = p_cur[q];
            on[q] = li < ppb && base + li < n;
        }
        // this tile's neighbour cache entries (the first tile's were loaded at kernel start; later tiles' are coalesced
        // loads in flight during the transform)
        int4 ent[PPT][2];
        const bool first_tile = base == (int)blockIdx.x * ppb;
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
            ent[q][0] = e_first[q][0];
            ent[q][1] = e_first[q][1];
            if (nc_read && on[q] && (!first_tile || !EPRE)) {
                const int4* e = nbr + 2 * (size_t)(base + (int)threadIdx.x + q * B);
                ent[q][0] = e[0];
                ent[q][1] = e[1];
            }
        }
        int v[PPT][NREL];
        float4 xt[PPT];
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
            // pcl::transformPointCloud: ((m0*x + m1*y) + m2*z) + m3, f32
            xt[q].x = T[0] * p[q].x + T[4] * p[q].y + T[8] * p[q].z + T[12];
            xt[q].y = T[1] * p[q].x + T[5] * p[q].y + T[9] * p[q].z + T[13];
            xt[q].z = T[2] * p[q].x + T[6] * p[q].y + T[10] * p[q].z + T[14];
            xt[q].w = 0.f;
            // getNeighborhoodAtPoint: ijk = floor(p / leaf_size) (float division), bounds vs min_b/max_b
            const int i0 = (int)floorf(xt[q].x / leaf0), i1 = (int)floorf(xt[q].y / leaf1), i2 = (int)floorf(xt[q].z / leaf2);
            int ck = -1;
            bool settled = false;  // neighbours known without probing (far from the grid, or a cache hit)
            if (nc_on) {
                const int h0 = i0 - mb0 + 1, h1 = i1 - mb1 + 1, h2 = i2 - mb2 + 1;
                const bool far = !on[q] || empty || h0 < 0 || h0 >= hd0 || h1 < 0 || h1 >= hd1 || h2 < 0 || h2 >= hd2;
                ck = far ? -1 : h0 + h1 * hm1 + h2 * hm2;
                const bool hit = nc_read && on[q] && ent[q][0].x == ck;
                settled = far || hit;
                if (settled) {
                    v[q][0] = hit ? ent[q][0].y : -1; v[q][1] = hit ? ent[q][0].z : -1; v[q][2] = hit ? ent[q][0].w : -1;
                    v[q][3] = hit ? ent[q][1].x : -1; v[q][4] = hit ? ent[q][1].y : -1; v[q][5] = hit ? ent[q][1].z : -1;
                    v[q][6] = hit ? ent[q][1].w : -1;
                }
            }
            if (!settled) {
            constexpr bool kTriple = NDT_ROW_TRIPLE && DENSE && SEARCH == S_DIRECT7;
            if (kTriple) {
                // DIRECT7 offsets 0, +x, -x are three consecutive cells of one grid row: one dwordx3 load for the three
                // (a point whose row triple would leave the grid allocation loads them one by one)
                const int kc = (i0 - mb0) + (i1 - mb1) * dm1 + (i2 - mb2) * dm2;
                const bool tri_ok = kc >= 1 && (long long)kc + 1 < cells;
                const uint3 t3 = *reinterpret_cast<const uint3*>(grid + (tri_ok ? kc - 1 : 0));
                int g[3] = {(int)t3.y, (int)t3.z, (int)t3.x};
                bool in3[3];
                int key3[3];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const int c0 = i0 + rel7(r, 0);
                    in3[r] = on[q] && !empty && !(c0 < mb0 || c0 > xb0 || i1 < mb1 || i1 > xb1 || i2 < mb2 || i2 > xb2);
                    key3[r] = kc + rel7(r, 0);
                }
                if (!tri_ok) {
#pragma unroll
                    for (int r = 0; r < 3; ++r) g[r] = grid[in3[r] ? key3[r] : 0];
                }
#pragma unroll
                for (int r = 0; r < 3; ++r) v[q][r] = in3[r] ? g[r] : -1;
            }
#pragma unroll
            for (int r = kTriple ? 3 : 0; r < NREL; ++r) {
                int d0, d1i, d2;
                if (SEARCH == S_DIRECT26) { d0 = c_rel26[r][0]; d1i = c_rel26[r][1]; d2 = c_rel26[r][2]; }
                else if (SEARCH == S_DIRECT1) { d0 = 0; d1i = 0; d2 = 0; }
                else { d0 = rel7(r, 0); d1i = rel7(r, 1); d2 = rel7(r, 2); }
                const int c0 = i0 + d0, c1 = i1 + d1i, c2 = i2 + d2;
                const bool in = on[q] && !empty && !(c0 < mb0 || c0 > xb0 || c1 < mb1 || c1 > xb1 || c2 < mb2 || c2 > xb2);
                const int key = (c0 - mb0) + (c1 - mb1) * dm1 + (c2 - mb2) * dm2;
                if (DENSE) {
                    // branch-free: every probe's load is issued before any is consumed
                    const int g = grid[in ? key : 0];
                    v[q][r] = in ? g : -1;
                } else {
                    v[q][r] = in ? hash_find(table, log2cap, key) : -1;
                }
            }
            }
            // an entry is (re)written after its point probed, and for every point in an align's first pass (entries left
            // by an earlier align must never match: its grid was another)
            if (nc_on && on[q] && (!settled || !nc_read)) {
                int4* e = nbr + 2 * (size_t)(base + (int)threadIdx.x + q * B);
                e[0] = make_int4(ck, v[q][0], v[q][1], v[q][2]);
                e[1] = make_int4(v[q][3], v[q][4], v[q][5], v[q][6]);
            }
        }
        // the next tile's points are loaded behind this tile's probes (loads complete in issue order; issued before the
        // probes they would hold up the results the compaction waits for — measured neutral at C5 / C2, 81.4 vs 82.0 us)
#pragma unroll
        for (int q = 0; q < PPT && !ONE_TILE; ++q) {
            const int li = (int)threadIdx.x + q * B, inext = base + li + gridDim.x * ppb;
            p_cur[q] = (li < ppb && inext < n) ? src[inext] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        // the per-point derivative terms are computed while the probe loads are in flight
        int c = 0;
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
            if (!on[q]) continue;
            const int li = (int)threadIdx.x + q * B;
            s_xt[li] = xt[q];
            PointDeriv pd;
            point_deriv<NDT_PACKED_PAIR != 0>(p[q], tab, pd, hess);
            s_pd[li] = pd;
        }
        // own first pair (kOwn): a point's first neighbour in probe order stays with its thread — its record gather is
        // issued here, as soon as the probes are back, and runs behind the compaction's scan and barriers; the point's
        // other pairs are compacted and dealt round robin as before.  (Lanes without one gather the tile's first
        // record slot-clamped to voxel 0 and hand over zeros.)
        bool own = false;
        int own_vox = 0;
        if (kOwn) {
#pragma unroll
            for (int r = 0; r < NREL; ++r)
                if (!own && v[0][r] >= 0 && !(v[0][r] & kRejectBit)) {
                    own = true;
                    own_vox = v[0][r];
                    v[0][r] = -1;
                }
        }
        // unconditional (recs holds at least one record once a target is set; an empty grid gives no own pair, so the
        // record is then never used): a load joined with another value at a branch is copied, i.e. waited for, at once
        const RecRaw own_rec = kOwn ? load_rec(recs, own_vox) : RecRaw{};
#pragma unroll
        for (int q = 0; q < PPT; ++q)
#pragma unroll
            for (int r = 0; r < NREL; ++r) c += (v[q][r] >= 0 && !(v[q][r] & kRejectBit)) ? 1 : 0;
        NDT_BLK_STAMP(pidx, 1);
#ifdef NDT_BODY_STAMPS
        NDT_TILE_ACC(t_acc, t_mark, 0);
#endif
        int tot, own_tot = 0;
        int ofs;
        if (kOwn) {
            // one scan for both counts: the compacted pairs in the low 20 bits, the own pairs above
            int packed;
            ofs = block_exclusive_scan<B / 64>(c + (own ? 1 << 20 : 0), s_scan, &packed);
            ofs &= (1 << 20) - 1;
            packed = __builtin_amdgcn_readfirstlane(packed);
            tot = packed & ((1 << 20) - 1);
            own_tot = packed >> 20;
        } else {
            ofs = block_exclusive_scan<B / 64>(c, s_scan, &tot);
            tot = __builtin_amdgcn_readfirstlane(tot);  // the block total (uniform): the pair loop's bound and count in SGPRs
        }
        if (c) {
#pragma unroll
            for (int q = 0; q < PPT; ++q)
#pragma unroll
                for (int r = 0; r < NREL; ++r)
                    if (v[q][r] >= 0 && !(v[q][r] & kRejectBit)) s_pair[ofs++] = PS::pack((int)threadIdx.x + q * B, v[q][r]);
        }
        lds_barrier();
        NDT_BLK_STAMP(pidx, 2);
#ifdef NDT_BODY_STAMPS
        NDT_TILE_ACC(t_acc, t_mark, 1);
#endif
        pairs += tot + own_tot;
        // pair math, the next pair's record gather in flight during this pair's math.  The prefetch index is clamped
        // (unconditional load: no join of a loaded value with an undefined one right behind the load, which would
        // make the compiler copy - and therefore wait for - the record at once)
        auto pair_at = [&](const typename PS::T pr, const RecRaw& raw, bool valid) {
            const int pt = PS::point(pr);
            const float4 x = s_xt[pt];
#if NDT_SPLIT_ACC
            const float xt3[3] = {x.x, x.y, x.z};
            SplitSink sink{acc};
            pair_pk_terms<true>(xt3, s_pd[pt].v, rec_view(raw), gd2, d1, hess, etab, sink, valid);
#elif NDT_PACKED_PAIR
            (void)valid;
            const float xt3[3] = {x.x, x.y, x.z};
            pair_pk(xt3, s_pd[pt].v, rec_view(raw), gd2, d1, hess, acc, etab);
#else
            PairPoint t;
            t.xt[0] = x.x; t.xt[1] = x.y; t.xt[2] = x.z;
            t.xj = s_pd[pt].v;
            t.xh = s_pd[pt].v + 8;
            (void)valid;
            pair_f32(t, rec_view(raw), gd2, d1, hess, acc, etab);
#endif
        };
        // two register sets A / B: A's reload is issued right after A's math, B's load right before it, so one
        // record gather is always in flight behind the current pair's math and no record is ever copied.  Split
        // accumulation exchanges terms between lanes, so every lane of a wave runs every iteration its first lane runs
        // (lanes past the tile's pairs compute a clamped pair and mask it out); otherwise each lane stops at its last pair.
        constexpr bool kWaveLoop = NDT_SPLIT_ACC != 0;
        int j = threadIdx.x;
        const int jw0 = kWaveLoop ? (int)(threadIdx.x & ~63u) : j;  // the loop's exit test: wave-uniform with split sums
#if NDT_REC_SETS == 3
        // three sets A / B / C: two record gathers in flight behind the current pair's math
        if (jw0 < tot) {
            auto pA = s_pair[min(j, tot - 1)];
            RecRaw A = load_rec(recs, PS::voxel(pA));
            auto pB = s_pair[min(j + B, tot - 1)];
            RecRaw Bv = load_rec(recs, PS::voxel(pB));
            for (int jw = jw0;;) {
                const auto pC = s_pair[min(j + 2 * B, tot - 1)];
                const RecRaw Cv = load_rec(recs, PS::voxel(pC));
                pair_at(pA, A, j < tot);
                if (jw + B >= tot) break;
                pA = s_pair[min(j + 3 * B, tot - 1)];
                A = load_rec(recs, PS::voxel(pA));
                pair_at(pB, Bv, j + B < tot);
                if (jw + 2 * B >= tot) break;
                pB = s_pair[min(j + 4 * B, tot - 1)];
                Bv = load_rec(recs, PS::voxel(pB));
                pair_at(pC, Cv, j + 2 * B < tot);
                if (jw + 3 * B >= tot) break;
                j += 3 * B;
                jw += 3 * B;
            }
        }
#else
        // the own pair's math (wave-uniform: a wave with no own pair skips it), behind the first compacted gather
        const bool wave_own = kOwn && __ballot(own) != 0;
        const auto own_slot = PS::pack(own ? (int)threadIdx.x : 0, 0);
        if (jw0 < tot) {
            auto pA = s_pair[min(j, tot - 1)];
            RecRaw A = load_rec(recs, PS::voxel(pA));
            if (wave_own) pair_at(own_slot, own_rec, own);
            for (int jw = jw0;;) {
                const int j1 = j + B;
                const auto pB = s_pair[min(j1, tot - 1)];
                const RecRaw Bv = load_rec(recs, PS::voxel(pB));
                pair_at(pA, A, j < tot);
                if (jw + B >= tot) break;
                const int j2 = j1 + B;
                pA = s_pair[min(j2, tot - 1)];
                A = load_rec(recs, PS::voxel(pA));
                pair_at(pB, Bv, j1 < tot);
                if (jw + 2 * B >= tot) break;
                j = j2;
                jw += 2 * B;
            }
        } else if (wave_own) {
            pair_at(own_slot, own_rec, own);
        }
#endif
        lds_barrier();
        NDT_BLK_STAMP(pidx, 3);
#ifdef NDT_BODY_STAMPS
        NDT_TILE_ACC(t_acc, t_mark, 2);
#endif
        if (ONE_TILE) break;
    }
#ifdef NDT_BODY_STAMPS
    NDT_TILE_ACC_STORE(pidx, t_acc);
#endif
}

// The last-workgroup-tail pass of one registration (k_pass_direct).
template <int SEARCH, int PPT, bool ONE_TILE>
__device__ __forceinline__ void pass_direct_impl(const float4* __restrict__ src, int n, int ppb, const GridHeader* __restrict__ hdr,
                                                 const int2* __restrict__ table, const int* __restrict__ grid,
                                                 const VoxelRec* __restrict__ recs, const AlignState* __restrict__ st,
                                                 AlignState* st_mut, double* __restrict__ partials, unsigned* counter, double* red_out,
                                                 PassRecordDev* hist, int hist_cap, int mode, unsigned long long* __restrict__ ts,
                                                 int4* __restrict__ nbr) {
    // the first tile's point load is issued before the state is inspected (independent round trips overlap)
    constexpr int B = pass_block(SEARCH, false);
    constexpr int NW = B / 64;
    // the kernel's start is stamped before anything else, so that the stamp window is the launch's (rocprofv3) duration
    const bool stamp0 = ts && blockIdx.x == 0 && threadIdx.x == 0;
    const unsigned long long t_entry = stamp0 ? __builtin_amdgcn_s_memrealtime() : 0ull;
    float4 p_first[PPT];
    int4 e_first[PPT][2];
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
        const int li = (int)threadIdx.x + q * B, i_first = blockIdx.x * ppb + li;
        const bool on_first = li < ppb && i_first < n;
        p_first[q] = on_first ? src[i_first] : make_float4(0.f, 0.f, 0.f, 0.f);
        e_first[q][0] = make_int4(-2, 0, 0, 0);
        e_first[q][1] = make_int4(0, 0, 0, 0);
        if (nbr && on_first) {
            // the first tile's neighbour cache entries, read beside its points (used only from an align's second pass on)
            e_first[q][0] = nbr[2 * (size_t)i_first];
            e_first[q][1] = nbr[2 * (size_t)i_first + 1];
        }
    }
    // the angle-table and expf-table words are loaded beside the state and the first points, not behind the state check
    // (C5 81.2 / 81.5 vs 81.6 / 81.5 us, C4 1929 vs 1906 pairs/s, same box)
    const float tab_w = threadIdx.x < 96 ? (&st->jang[0][0])[threadIdx.x] : 0.f;
    const unsigned long long exp_w = threadIdx.x < kExpTabLen ? c_exp_tab[threadIdx.x] : 0ull;
    if (!st->pending || st->pass_kind == PASS_HESS) return;
    const int pass_idx = st->n_passes;
    if (pass_idx >= kMaxHistory) ts = nullptr;
    if (ts && stamp0) ts[kTsStride * pass_idx] = t_entry;
    __shared__ double red[NW * kNumAcc];
    double acc[kBodyAcc];
#pragma unroll
    for (int v = 0; v < kBodyAcc; ++v) acc[v] = 0.0;
    long long pairs = 0;
    NDT_BLK_STAMP(pass_idx, 0);
    // one set of LDS tiles shared by both grid flavours of the body
    constexpr int NREL = SEARCH == S_DIRECT26 ? 26 : (SEARCH == S_DIRECT1 ? 1 : 7);
    __shared__ float4 s_xt[B * PPT];
    __shared__ PointDeriv s_pd[B * PPT];
    __shared__ typename PairSlot<PPT>::T s_pair[B * PPT * NREL];
    __shared__ int s_scan[NW];
    __shared__ float s_tab[96];
    __shared__ __align__(16) double s_exp[kExpTabLen];
    if (threadIdx.x < 96) s_tab[threadIdx.x] = tab_w;
    if (threadIdx.x < kExpTabLen) s_exp[threadIdx.x] = __longlong_as_double((long long)exp_w);
    lds_barrier();
    const int n_pts = min(n, st->n_src);  // the geometry (grid, ppb) covers a point bucket >= the scan's points
    if (hdr->dense)
        direct_pass_body<SEARCH, true, B, PPT, ONE_TILE>(src, n_pts, ppb, hdr, table, grid, recs, st, acc, pairs, pass_idx, p_first, e_first, s_xt,
                                               s_pd, s_pair, s_scan, s_tab, s_exp, nbr);
    else
        direct_pass_body<SEARCH, false, B, PPT, ONE_TILE, false>(src, n_pts, ppb, hdr, table, grid, recs, st, acc, pairs, pass_idx, p_first, e_first,
                                                s_xt, s_pd, s_pair, s_scan, s_tab, s_exp, nbr);
    // the body only reads the state through the const view; only the last workgroup writes it (st_mut)
#if NDT_SPLIT_ACC
    if (threadIdx.x == 32) acc[3] += (double)pairs;  // the high set's pair-count slot (split_hi_term(3) = 43)
    block_reduce_store_split<NW>(acc, red, partials + blockIdx.x, partial_stride(gridDim.x));
    // three-wave (one-tile) kernels reduce the partials two column pairs per lane and round trip: the four-pair loads do
    // not fit their registers
    const bool tail = pass_handoff<NW, ONE_TILE ? 2 : 4>(st_mut, partials, counter, red_out, hist, hist_cap, mode,
                                                          ts ? ts + kTsStride * pass_idx : nullptr);
#else
    acc[43] = threadIdx.x == 0 ? (double)pairs : 0.0;
    const bool tail = pass_epilogue<NW>(acc, red, st_mut, partials, counter, red_out, hist, hist_cap, mode,
                                         ts ? ts + kTsStride * pass_idx : nullptr);
#endif
    if (ts && tail) {
        __syncthreads();
        if (threadIdx.x == 0) ts[kTsStride * pass_idx + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

template <int SEARCH, int PPT, bool ONE_TILE>
__global__ __launch_bounds__(pass_block(SEARCH, false)) __attribute__((amdgpu_waves_per_eu(pass_waves(SEARCH, PPT, ONE_TILE))))
void k_pass_direct(const float4* __restrict__ src, int n, int ppb, const GridHeader* __restrict__ hdr, const int2* __restrict__ table,
                   const int* __restrict__ grid, const VoxelRec* __restrict__ recs, const AlignState* __restrict__ st,
                   AlignState* st_mut, double* __restrict__ partials, unsigned* counter, double* red_out, PassRecordDev* hist,
                   int hist_cap, int mode, unsigned long long* __restrict__ ts, int4* __restrict__ nbr) {
    pass_direct_impl<SEARCH, PPT, ONE_TILE>(src, n, ppb, hdr, table, grid, recs, st, st_mut, partials, counter, red_out, hist, hist_cap, mode, ts,
                                  nbr);
}


// ---------------------------------------------------------------------------------------------------
// Leading-tail pass (chains without radius passes): every workgroup of pass k+1 first reduces pass k's partials and
// runs the Newton / More-Thuente step itself on an LDS copy of the state (the same bits in every workgroup: same
// inputs, fixed orders), then runs pass k+1's body from that LDS state.  No ticket, no last-workgroup hand-off and no
// state round trip between the control step and the body: the tail's inputs (partials, state) are read at kernel
// start next to the first points.  State and partials ping-pong between two buffers by chain slot (the host picks the
// parity), workgroup 0 writes the new state (and the pass record); a kernel whose state says "no body" only copies it.
template <int SEARCH, bool ONE_TILE>
__global__ __launch_bounds__(pass_block(SEARCH, true, ONE_TILE)) __attribute__((amdgpu_waves_per_eu(ONE_TILE ? 3 : 1))) void k_pass_lead(const float4* __restrict__ src, int n, int ppb,
                                                      const GridHeader* __restrict__ hdr, const int2* __restrict__ table,
                                                      const int* __restrict__ grid, const VoxelRec* __restrict__ recs,
                                                      const AlignState* __restrict__ st_in, AlignState* __restrict__ st_out,
                                                      const double* __restrict__ part_in, double* __restrict__ part_out,
                                                      PassRecordDev* hist, int hist_cap, unsigned long long* __restrict__ ts,
                                                      int4* __restrict__ nbr) {
    constexpr int B = pass_block(SEARCH, true, ONE_TILE);
    constexpr int NW = B / 64;
    constexpr int kWords = sizeof(AlignState) / 8;
    static_assert(kWords <= 2 * B, "AlignState staging assumes <= 2 words per thread");
#ifdef NDT_BODY_STAMPS
    const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
#endif
    const int i_first = blockIdx.x * ppb + threadIdx.x;
    const bool on_first = (int)threadIdx.x < ppb && i_first < n;
    const float4 p_first[1] = {on_first ? src[i_first] : make_float4(0.f, 0.f, 0.f, 0.f)};
    // the neighbour cache entries of this workgroup's points, read next to them (ahead of the Newton step)
    int4 e_first[1][2] = {{make_int4(-2, 0, 0, 0), make_int4(0, 0, 0, 0)}};
    if (nbr && on_first) {
        e_first[0][0] = nbr[2 * (size_t)i_first];
        e_first[0][1] = nbr[2 * (size_t)i_first + 1];
    }
    __shared__ AlignState s_st;
    __shared__ __align__(16) double s_exp[kExpTabLen];
#ifndef NDT_LEAD_PRELOAD
#define NDT_LEAD_PRELOAD 1
#endif
#ifndef NDT_LEAD_HASH_PPRE
#define NDT_LEAD_HASH_PPRE 0
#endif
    PartialsPre<NW, 2> pre;
    {
        // the exp table's and the state's words loaded together from clamped addresses (no branch around a load: a load
        // and its LDS store in one conditional block are a round trip each, one after the other), then stored
        const int t = threadIdx.x;
        const unsigned long long* gw = reinterpret_cast<const unsigned long long*>(st_in);
        unsigned long long* lw = reinterpret_cast<unsigned long long*>(&s_st);
        const unsigned long long ew = c_exp_tab[t < kExpTabLen ? t : 0];
        const unsigned long long a = gw[t < kWords ? t : 0];
        const unsigned long long b = gw[t + B < kWords ? t + B : 0];
        // the previous pass's first 256 partial columns, loaded behind the state (in flight while it is stored and
        // inspected; a kernel that consumes none discards them)
        if (NDT_LEAD_PRELOAD) partials_preload<NW, 2>(part_in, gridDim.x, pre);
        if (t < kExpTabLen) s_exp[t] = __longlong_as_double((long long)ew);
        if (t < kWords) lw[t] = a;
        if (t + B < kWords) lw[t + B] = b;
    }
    lds_barrier();
    // profiling: this kernel's start is the start of its body's pass and the end of the pass whose partials it consumes
    const unsigned long long t_start = (ts && blockIdx.x == 0 && threadIdx.x == 0) ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const bool consumed = s_st.partials_pending != 0;
    __shared__ double red[kNumAcc];
#ifdef NDT_BODY_STAMPS
    const unsigned long long t_staged = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_reduced = t_staged;
    // the tail stamps of workgroup 0's control step (row kBlkMax - 1 of the consumed pass)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const int pc = s_st.n_passes;
        g_tail_ts = pc < kBlkPasses ? &g_blk_ts[((size_t)pc * kBlkMax + kBlkMax - 1) * kBlkSlots] : nullptr;
        g_tail_wg = 0;
    }
    __syncthreads();
#endif
    if (s_st.partials_pending) {
        // two column pairs per lane and row: one round trip covers the 256 partial columns of a one-workgroup-per-CU
        // grid (four left half the loads predicated off; the non-zero terms are added in the same order either way):
        // C2 20.77 vs 21.10 us per pass, 1105 / 1107 vs 1089 / 1095 scans/s (same-box A/B)
        if (NDT_LEAD_PRELOAD) reduce_partials_pre<NW, 2, 2>(part_in, gridDim.x, pre, red);
        else reduce_partials_block<NW, 2>(part_in, gridDim.x, red);
#ifdef NDT_BODY_STAMPS
        t_reduced = __builtin_amdgcn_s_memrealtime();
#endif
        tail_control<NW>(s_st, red, hist, blockIdx.x == 0 ? hist_cap : 0, nullptr);
        if (threadIdx.x == 0) s_st.partials_pending = 0;
        lds_barrier();
    }
#ifdef NDT_BODY_STAMPS
    // profiling build: workgroup 0's prologue (entry, staged, reduced, controlled) in row kBlkMax - 2 of its body's pass
    if (blockIdx.x == 0 && threadIdx.x == 0 && s_st.n_passes < kBlkPasses) {
        unsigned long long* r = &g_blk_ts[((size_t)s_st.n_passes * kBlkMax + kBlkMax - 2) * kBlkSlots];
        r[0] = t_entry; r[1] = t_staged; r[2] = t_reduced; r[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const bool body = s_st.pending && s_st.pass_kind != PASS_HESS;
    if (ts && blockIdx.x == 0 && threadIdx.x == 0) {
        const int k = s_st.n_passes;  // index of this kernel's body (the consumed pass was k - 1)
        if (consumed && k - 1 >= 0 && k - 1 < kMaxHistory) ts[kTsStride * (k - 1) + 1] = t_start;
        if (body && k < kMaxHistory) ts[kTsStride * k] = t_start;
    }
    if (threadIdx.x == 0 && body) s_st.partials_pending = 1;
    lds_barrier();
    if (blockIdx.x == 0) {
        const unsigned long long* lw = reinterpret_cast<const unsigned long long*>(&s_st);
        unsigned long long* gw = reinterpret_cast<unsigned long long*>(st_out);
        for (int k = threadIdx.x; k < kWords; k += B) gw[k] = lw[k];
    }
    if (!body) return;
    __shared__ double redw[NW * kNumAcc];
    double acc[kBodyAcc];
#pragma unroll
    for (int v = 0; v < kBodyAcc; ++v) acc[v] = 0.0;
    long long pairs = 0;
    constexpr int NREL = SEARCH == S_DIRECT26 ? 26 : (SEARCH == S_DIRECT1 ? 1 : 7);
    __shared__ float4 s_xt[B];
    __shared__ PointDeriv s_pd[B];
    __shared__ int2 s_pair[B * NREL];
    __shared__ int s_scan[NW];
    const int pidx = s_st.n_passes;
    const int n_pts = min(n, s_st.n_src);  // the geometry (grid, ppb) covers a point bucket >= the scan's points
    NDT_BLK_STAMP(pidx, 0);
    if (hdr->dense)
        direct_pass_body<SEARCH, true, B, 1, ONE_TILE>(src, n_pts, ppb, hdr, table, grid, recs, &s_st, acc, pairs, pidx, p_first, e_first, s_xt,
                                          s_pd, s_pair, s_scan, &s_st.jang[0][0], s_exp, nbr);
    else {
        const int4 e_none[1][2] = {{make_int4(-2, 0, 0, 0), make_int4(0, 0, 0, 0)}};
        direct_pass_body<SEARCH, false, B, 1, ONE_TILE, false, NDT_LEAD_HASH_PPRE != 0>(src, n_pts, ppb, hdr, table, grid, recs, &s_st, acc, pairs, pidx, p_first,
                                                               e_none, s_xt, s_pd, s_pair, s_scan, &s_st.jang[0][0], s_exp, nbr);
    }
#if NDT_SPLIT_ACC
    if (threadIdx.x == 32) acc[3] += (double)pairs;
    block_reduce_store_split<NW>(acc, redw, part_out + blockIdx.x, partial_stride(gridDim.x));
    NDT_BLK_STAMP(pidx, 4);
#else
    acc[43] = threadIdx.x == 0 ? (double)pairs : 0.0;
    block_reduce_store<kNumAcc, NW>(acc, redw, part_out + blockIdx.x, partial_stride(gridDim.x));
#endif
}
#define NDT_LEAD_INST(S, ONE)                                                                                                   \
    template __global__ void k_pass_lead<S, ONE>(const float4*, int, int, const GridHeader*, const int2*, const int*, const VoxelRec*, \
                                                 const AlignState*, AlignState*, const double*, double*, PassRecordDev*, int,         \
                                                 unsigned long long*, int4*);
NDT_LEAD_INST(S_DIRECT7, false)
NDT_LEAD_INST(S_DIRECT7, true)
NDT_LEAD_INST(S_DIRECT1, false)
NDT_LEAD_INST(S_DIRECT1, true)
NDT_LEAD_INST(S_DIRECT26, false)
#undef NDT_LEAD_INST

// ---------------------------------------------------------------------------------------------------
// Radius-neighbour pass: KdTreeFLANN::radiusSearch over the voxel-centroid cloud (voxel_grid_covariance_omp.h
// :470-499) restated as a voxel-stencil probe + exact float distance test (strict < r^2, L2_Simple order),
// neighbours visited in ascending (distance, cloud index) order.  Serves KDTREE search (f32 math),
// pcl_ndt mode (f64 math) and computeHessian (f64, PASS_HESS).
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ void pair_f64(const double* x /*orig*/, const double* xt /*x' */, const double* Cd /*row-major*/,
                                         const AlignState* __restrict__ st, int mode /*0 grad+score,1 +hess,2 hess only*/,
                                         double* acc) {
    const double gd2 = st->gauss_d2, gd1 = st->gauss_d1;
    auto mv = [&](const double* v, double* o) {
        for (int i = 0; i < 3; ++i) o[i] = Cd[i * 3 + 0] * v[0] + Cd[i * 3 + 1] * v[1] + Cd[i * 3 + 2] * v[2];
    };
    auto d3 = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    // computePointDerivatives, double path (ndt_omp_impl.hpp:448-488)
    double PG[3][6] = {{1, 0, 0, 0, 0, 0}, {0, 1, 0, 0, 0, 0}, {0, 0, 1, 0, 0, 0}};
    auto dx = [&](const double* v) { return x[0] * v[0] + x[1] * v[1] + x[2] * v[2]; };
    PG[1][3] = dx(st->jang_d[0]); PG[2][3] = dx(st->jang_d[1]); PG[0][4] = dx(st->jang_d[2]); PG[1][4] = dx(st->jang_d[3]);
    PG[2][4] = dx(st->jang_d[4]); PG[0][5] = dx(st->jang_d[5]); PG[1][5] = dx(st->jang_d[6]); PG[2][5] = dx(st->jang_d[7]);
    double Hb[6][3];  // a..f
    Hb[0][0] = 0; Hb[0][1] = dx(st->hang_d[0]); Hb[0][2] = dx(st->hang_d[1]);
    Hb[1][0] = 0; Hb[1][1] = dx(st->hang_d[2]); Hb[1][2] = dx(st->hang_d[3]);
    Hb[2][0] = 0; Hb[2][1] = dx(st->hang_d[4]); Hb[2][2] = dx(st->hang_d[5]);
    for (int r = 0; r < 3; ++r) { Hb[3][r] = dx(st->hang_d[6 + r]); Hb[4][r] = dx(st->hang_d[9 + r]); Hb[5][r] = dx(st->hang_d[12 + r]); }
    // block (i,j) of H_E for i,j in 3..5 -> index into Hb
    const int blk[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
    double cx[3];
    mv(xt, cx);
    double e;
    if (mode == 2) {
        e = gd2 * exp(-gd2 * d3(xt, cx) / 2);  // updateHessian (:619)
        if (e > 1 || e < 0 || e != e) return;
    } else {
        e = exp(-gd2 * d3(xt, cx) / 2);        // pcl updateDerivatives
        const double score_inc = -gd1 * e;
        e = gd2 * e;
        if (e > 1 || e < 0 || e != e) return;
        acc[0] += score_inc;
    }
    e *= gd1;
    for (int i = 0; i < 6; ++i) {
        double ci[3] = {PG[0][i], PG[1][i], PG[2][i]}, cdi[3];
        mv(ci, cdi);
        if (mode != 2) acc[1 + i] += d3(xt, cdi) * e;
        if (mode == 0) continue;
        for (int j = 0; j < 6; ++j) {
            double cj[3] = {PG[0][j], PG[1][j], PG[2][j]}, cdj[3];
            mv(cj, cdj);
            double ph[3] = {0, 0, 0};
            if (i >= 3 && j >= 3) { const double* b = Hb[blk[i - 3][j - 3]]; ph[0] = b[0]; ph[1] = b[1]; ph[2] = b[2]; }
            double cph[3];
            mv(ph, cph);
            acc[7 + i * 6 + j] += e * (-gd2 * d3(xt, cdi) * d3(xt, cdj) + d3(xt, cph) + d3(cj, cdi));
        }
    }
}

// VoxelGridCovariance::radiusSearch (voxel_grid_covariance_omp.h:470-499: KdTreeFLANN over the KD cloud of
// voxel centroids, radius = resolution) restated on the voxel grid: every cell whose centroid can lie within
// the radius is visited, the exact float distance test (strict < r^2, FLANN L2_Simple order) selects, and the
// neighbours come out in ascending (distance, cloud index) order, as FLANN's sorted result.
struct RadiusGrid {
    bool dense;
    float inv[3];
    int mb[3], db[3];
    int dm1, dm2;
    unsigned log2cap;
    float r2;
    int ext;
};
constexpr int kMaxCand = 48;

__device__ __forceinline__ RadiusGrid radius_grid(const GridHeader* __restrict__ hdr, float radius) {
    RadiusGrid g;
    g.dense = hdr->dense != 0;
    for (int a = 0; a < 3; ++a) { g.inv[a] = hdr->inv_leaf[a]; g.mb[a] = hdr->min_b[a]; g.db[a] = hdr->div_b[a]; }
    g.dm1 = hdr->divb_mul[1];
    g.dm2 = hdr->divb_mul[2];
    g.log2cap = hdr->log2cap;
    // KdTreeFLANN radius search: PCL passes radius*radius (double) narrowed to float
    g.r2 = (float)((double)radius * (double)radius);
    g.ext = max(1, (int)ceilf(radius * g.inv[0]));
    return g;
}

// Visits every voxel centroid within the radius (exact float test, strict < r^2) in stencil order: fn(cloud index, d2).
template <typename F>
__device__ __forceinline__ void radius_walk(const RadiusGrid& g, const float* xt, const int* __restrict__ grid,
                                            const int2* __restrict__ table, const float4* __restrict__ cent, F&& fn) {
    // stencil centre in binning coordinates; extend by one cell where the point is within float noise of a face
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        const float s = xt[a] * g.inv[a];
        const float fl = floorf(s);
        const int u = (int)(fl - (float)g.mb[a]);
        const float fr = s - fl;
        const float tol = 1e-4f + 16.f * fabsf(s) * FLT_EPSILON;
        lo[a] = u - g.ext - (fr < tol ? 1 : 0);
        hi[a] = u + g.ext + (fr > 1.f - tol ? 1 : 0);
        lo[a] = max(lo[a], 0);
        hi[a] = min(hi[a], g.db[a] - 1);
    }
    for (int c2 = lo[2]; c2 <= hi[2]; ++c2)
        for (int c1 = lo[1]; c1 <= hi[1]; ++c1)
            for (int c0 = lo[0]; c0 <= hi[0]; ++c0) {
                const int key = c0 + c1 * g.dm1 + c2 * g.dm2;
                const int v = voxel_lookup(g.dense, grid, table, g.log2cap, key);
                if (v < 0) continue;
                const int idx = v & ~kRejectBit;
                const float4 c = cent[idx];
                float d = 0.f, tt;
                tt = c.x - xt[0]; d += tt * tt;
                tt = c.y - xt[1]; d += tt * tt;
                tt = c.z - xt[2]; d += tt * tt;
                if (d < g.r2) fn(idx, d);
            }
}

// The neighbours sorted as FLANN returns them (ascending distance, then cloud index).  A radius of one leaf reaches at
// most 3 x 3 x 3 cells (<= 27 centroids, always within kMaxCand); a larger radius (setResolution after setInputTarget
// without a source keeps the old leaf, ndt_omp.h:127-137) can exceed the list: the count is then returned
// (> kMaxCand) with the list incomplete, and the caller visits the neighbours with radius_walk instead — same pairs,
// stencil order (the f64 sums differ from FLANN's order by rounding only), never a truncated neighbour set.
__device__ __forceinline__ int radius_candidates(const RadiusGrid& g, const float* xt, const int* __restrict__ grid,
                                                 const int2* __restrict__ table, const float4* __restrict__ cent, float* cd, int* ci) {
    int nc = 0;
    radius_walk(g, xt, grid, table, cent, [&](int idx, float d) {
        if (nc < kMaxCand) {
            // insertion into the sorted candidate list (distance, cloud index)
            int k = nc;
            while (k > 0 && (cd[k - 1] > d || (cd[k - 1] == d && ci[k - 1] > idx))) { cd[k] = cd[k - 1]; ci[k] = ci[k - 1]; --k; }
            cd[k] = d; ci[k] = idx;
        }
        ++nc;
    });
    return nc;
}

// cpu::VoxelGrid::radiusSearch (ndt_cpu backend; the method is declared at ndt_cpu/VoxelGrid.h:27, its body ships only
// in the prebuilt libndt_cpu.so and is restated from the published Autoware ndt_cpu algorithm, cross-checked against the
// binary's code as text): the cells of the cube floorf((x -+ r) / leaf) clamped to the grid, visited x-major (x outer,
// z inner); a voxel with >= min points (not rejected) is a neighbour when the f64 distance from its f64 centroid,
// sqrt(dx^2 + dy^2 + dz^2), is below the radius.  fn(cloud index) in visiting order.
template <typename F>
__device__ __forceinline__ void radius_walk_aw(const GridHeader* __restrict__ hdr, const float* xt, float radius,
                                               const int* __restrict__ grid, const int2* __restrict__ table,
                                               const VoxelRec* __restrict__ recs, F&& fn) {
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = max((int)floorf((xt[a] - radius) / hdr->leaf[a]), hdr->min_b[a]);
        hi[a] = min((int)floorf((xt[a] + radius) / hdr->leaf[a]), hdr->max_b[a]);
    }
    const bool dense = hdr->dense != 0;
    const int dm1 = hdr->divb_mul[1], dm2 = hdr->divb_mul[2];
    const double r = (double)radius;
    for (int ix = lo[0]; ix <= hi[0]; ++ix)
        for (int iy = lo[1]; iy <= hi[1]; ++iy)
            for (int iz = lo[2]; iz <= hi[2]; ++iz) {
                const int key = (ix - hdr->min_b[0]) + (iy - hdr->min_b[1]) * dm1 + (iz - hdr->min_b[2]) * dm2;
                const int v = voxel_lookup(dense, grid, table, hdr->log2cap, key);
                if (v < 0 || (v & kRejectBit)) continue;
                const double* m = recs[v].mean;
                const double cx = m[0] - (double)xt[0], cy = m[1] - (double)xt[1], cz = m[2] - (double)xt[2];
                if (sqrt(cx * cx + cy * cy + cz * cz) < r) fn(v);
            }
}

__global__ __launch_bounds__(kBlock) void k_pass_radius(const float4* __restrict__ src, int n,
                                                        const GridHeader* __restrict__ hdr,
                                                        const int2* __restrict__ table,
                                                        const int* __restrict__ grid,
                                                        const VoxelRec* __restrict__ recs,
                                                        const float4* __restrict__ cent,
                                                        const double* __restrict__ icovd,
                                                        const AlignState* __restrict__ st,
                                                        AlignState* st_mut,
                                                        double* __restrict__ partials,
                                                        unsigned* counter, double* red_out,
                                                        PassRecordDev* hist, int hist_cap, int mode,
                                                        unsigned long long* __restrict__ ts) {
    if (!st->pending) return;
    const int kind = st->pass_kind;
    // KDTREE search, pcl_ndt (precision 1) and ndt_cpu (precision 2, cpu::VoxelGrid neighbours) evaluate every pass here
    const bool radius_search = st->search == S_KDTREE || st->precision >= 1;
    if (kind != PASS_HESS && !radius_search) return;
    const int pass_idx = st->n_passes;
    if (pass_idx >= kMaxHistory) ts = nullptr;
    if (ts && blockIdx.x == 0 && threadIdx.x == 0) ts[kTsStride * pass_idx] = __builtin_amdgcn_s_memrealtime();
    __shared__ double red[4 * kNumAcc];
    __shared__ __align__(16) double s_exp[kExpTabLen];
    stage_exp_tab(s_exp);
    __syncthreads();
    const bool f64 = st->precision >= 1 || kind == PASS_HESS;
    const int mode64 = kind == PASS_HESS ? 2 : (kind == PASS_FULL ? 1 : 0);
    const float gd2 = (float)st->gauss_d2;
    const double d1 = st->gauss_d1;
    double acc[kNumAcc];
#pragma unroll
    for (int v = 0; v < kNumAcc; ++v) acc[v] = 0.0;
    const bool empty = hdr->empty != 0 || hdr->n_cloud == 0;
    const RadiusGrid rg = radius_grid(hdr, st->radius);
    const bool aw = hdr->binning != 0;  // a cpu::VoxelGrid target (ndt_cpu): its own radius search
    const int stride = gridDim.x * kBlock;
    int pairs = 0;
    const int n_pts = min(n, st->n_src);  // the launch geometry covers a point bucket (a captured chain serves many scan sizes)
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n_pts; i += stride) {
        PointTerms t;
        const float4 p = src[i];
        load_point_terms(p, st, t, kind == PASS_FULL);
        if (empty) continue;
        float cd[kMaxCand];
        int ci[kMaxCand];
        const int nc = aw ? 0 : radius_candidates(rg, t.xt, grid, table, cent, cd, ci);
        const double xo[3] = {p.x, p.y, p.z};
        auto pair = [&](int idx) {
            ++pairs;
            if (!f64) {
                const VoxelRec rec = recs[idx];
                pair_f32(t, rec, gd2, d1, kind == PASS_FULL, acc, s_exp);
            } else {
                const VoxelRec rec = recs[idx];
                double xt[3] = {(double)t.xt[0] - rec.mean[0], (double)t.xt[1] - rec.mean[1], (double)t.xt[2] - rec.mean[2]};
                pair_f64(xo, xt, icovd + (size_t)idx * 9, st, mode64, acc);
            }
        };
        if (aw) {
            radius_walk_aw(hdr, t.xt, st->radius, grid, table, recs, pair);
        } else if (nc <= kMaxCand) {
            for (int k = 0; k < nc; ++k) pair(ci[k]);
        } else {
            radius_walk(rg, t.xt, grid, table, cent, [&](int idx, float) { pair(idx); });
        }
    }
    acc[43] = (double)pairs;
    // the body only reads the state through the const view; only the last workgroup writes it (st_mut)
    const bool tail = pass_epilogue(acc, red, st_mut, partials, counter, red_out, hist, hist_cap, mode,
                                    ts ? ts + kTsStride * pass_idx : nullptr);
    if (ts && tail) {
        __syncthreads();
        if (threadIdx.x == 0) ts[kTsStride * pass_idx + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// NormalDistributionsTransform::calculateScore (ndt_omp_impl.hpp:919-952) of the source transformed by T
// (pcl::transformPointCloud, f32): f64 score over the radius neighbours, each term divided by the point's
// neighbour count.  One partial sum per workgroup (fixed order), summed in order by the host.
__global__ __launch_bounds__(kBlock) void k_score_radius(const float4* __restrict__ src, int n, Mat4f Tm,
                                                         const GridHeader* __restrict__ hdr, const int2* __restrict__ table,
                                                         const int* __restrict__ grid, const VoxelRec* __restrict__ recs,
                                                         const float4* __restrict__ cent, const double* __restrict__ icovd,
                                                         double gd1, double gd2, double gd3, float radius,
                                                         double* __restrict__ partials) {
    const float* T = Tm.m;
    double score = 0.0;
    const bool empty = hdr->empty != 0 || hdr->n_cloud == 0;
    const RadiusGrid rg = radius_grid(hdr, radius);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n && !empty; i += gridDim.x * kBlock) {
        const float4 p = src[i];
        float xt[3];
        xt[0] = T[0] * p.x + T[4] * p.y + T[8] * p.z + T[12];
        xt[1] = T[1] * p.x + T[5] * p.y + T[9] * p.z + T[13];
        xt[2] = T[2] * p.x + T[6] * p.y + T[10] * p.z + T[14];
        float cd[kMaxCand];
        int ci[kMaxCand];
        const int nc = radius_candidates(rg, xt, grid, table, cent, cd, ci);
        auto term = [&](int idx) {
            const double* C = icovd + (size_t)idx * 9;
            const VoxelRec& rec = recs[idx];
            const double x[3] = {(double)xt[0] - rec.mean[0], (double)xt[1] - rec.mean[1], (double)xt[2] - rec.mean[2]};
            double cx[3];
            for (int r = 0; r < 3; ++r) cx[r] = C[r * 3 + 0] * x[0] + C[r * 3 + 1] * x[1] + C[r * 3 + 2] * x[2];
            const double e = exp(-gd2 * (x[0] * cx[0] + x[1] * cx[1] + x[2] * cx[2]) / 2);
            const double score_inc = -gd1 * e - gd3;
            score += score_inc / (double)nc;
        };
        if (nc <= kMaxCand) {
            for (int k = 0; k < nc; ++k) term(ci[k]);
        } else {
            radius_walk(rg, xt, grid, table, cent, [&](int idx, float) { term(idx); });
        }
    }
    // fixed-order workgroup sum
    __shared__ double s_part[kBlock];
    s_part[threadIdx.x] = score;
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) s_part[threadIdx.x] += s_part[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = s_part[0];
}

#define NDT_INST(S, P, O) template __global__ void k_pass_direct<S, P, O>(const float4*, int, int, const GridHeader*, const int2*,   \
                                                                         const int*, const VoxelRec*, const AlignState*, AlignState*, \
                                                                         double*, unsigned*, double*,                                 \
                                                                         PassRecordDev*, int, int, unsigned long long*, int4*);
NDT_INST(S_DIRECT7, 1, false)
NDT_INST(S_DIRECT7, 1, true)
NDT_INST(S_DIRECT7, 2, false)
NDT_INST(S_DIRECT26, 1, false)
NDT_INST(S_DIRECT1, 1, false)
NDT_INST(S_DIRECT1, 1, true)
NDT_INST(S_DIRECT1, 2, false)
#undef NDT_INST


}  // namespace ndt

namespace ndt {
// host side of the profiling build's per-workgroup stamps (hipErrorNotSupported in the product build)
hipError_t dbg_read_blk(unsigned long long* host, size_t count) {
#ifdef NDT_BODY_STAMPS
    if (!host) return hipSuccess;
    const size_t n = std::min(count, (size_t)kBlkPasses * kBlkMax * kBlkSlots);
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_blk_ts), n * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost);
#else
    (void)host;
    (void)count;
    return hipErrorNotSupported;
#endif
}
}  // namespace ndt
