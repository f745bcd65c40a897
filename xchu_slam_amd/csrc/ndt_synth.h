/* ndt_synth.h — C-ABI of libndt_synth.so: the on-device generator of the C4 batched-replay pairs.
 * BENCH INFRASTRUCTURE ONLY (bench.py --workload c4); not part of the NDT drop-in surface declared in include/. */
#ifndef NDT_SYNTH_H_
#define NDT_SYNTH_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    unsigned long long seed_target;  /* localmap points (SURVEY: 1000 + i)                                   */
    unsigned long long seed_source;  /* scan points     (SURVEY: 5000 + i)                                   */
    int device;
    int nb, np;                      /* buildings / poles of the world (host arrays, see world layout below) */
    int nb_near, np_near;            /* how many of them lie within the scan's range (cdf weight > 0)        */
    int cells_side;                  /* ground cells per side (= int(2 half))                                */
    int per_cell;                    /* ground points per 1 m cell (= round(density))                         */
    int perm_half_bits;              /* Feistel half width: 4^perm_half_bits >= n_target                     */
    long long n_ground, n_walls, n_poles;  /* localmap = n_ground + n_walls + n_poles points                 */
    int n_source;
    float half, noise, max_range;
    float cx, cy;                    /* sensor position (world frame)                                         */
    double world_to_sensor[12];      /* row-major 3x4: inverse of the true sensor pose                       */
} SynthPairDesc;

/* world layout (floats): buildings nb x (cx, cy, w, d, h, yaw) | facade-area cdf [nb] | near-facade cdf [nb]
 *                        | poles np x (x, y, r, h) | near-pole cdf [np] */
int ndt_synth_world_floats(int nb, int np);

/* Fill d_target (n_ground + n_walls + n_poles float4) and d_source (n_source float4, sensor frame); d_world holds
 * ndt_synth_world_floats() floats of device scratch.  Synchronous.  0 = ok, 1 = bad argument, 5 = HIP error. */
int ndt_synth_pair_device(const SynthPairDesc* desc, const float* h_world, float* d_world, void* d_target, void* d_source);

#ifdef __cplusplus
}
#endif
#endif
