/* synth.h -- seeded synthetic sliding windows (test and bench input generator, not part of
 * the hot path).  See synth.cpp. */
#ifndef LDSO_AMD_SYNTH_H_
#define LDSO_AMD_SYNTH_H_

#include <stdint.h>

#include "../../include/ldso_ba.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ldso_synth_params {
    int32_t n_frames;
    int32_t n_points;
    int32_t width;
    int32_t height;
    uint64_t seed;
    float outlier_frac;     /* fraction of points with a grossly wrong idepth        */
    float idepth_noise;     /* relative gaussian noise on inlier idepths             */
    float newest_perturb;   /* pose perturbation of the newest frame's state (rad/m) */
    float baseline;         /* camera travel per keyframe along x (m)                */
    /* appended in round 6 (all zero = the round-1..5 window) */
    int32_t motion;         /* 0: sideways (x) travel, EuRoC-style intrinsics fx = 0.6w, fy = 0.9h;
                             * 1: forward (+z) travel of U(fwd_min, fwd_max) m per keyframe towards a
                             *    plane plane_depth m ahead, as a KITTI car drives                   */
    float fx, fy, cx, cy;   /* pinhole intrinsics of the output images (fx <= 0: motion's default)   */
    float fwd_min, fwd_max; /* forward travel per keyframe (m), motion 1                              */
    float plane_depth;      /* far facade's distance from the first keyframe (m), motion 1            */
    float edge_frac;        /* fraction of points drawn in the 4..9-px band along the image border   */
} ldso_synth_params;

/* Fills a synthetic window.  Output sizes:
 *   frames[N], dI[N*h*w*3], calib[4], frame_energy_th[N], point_host[P],
 *   point_data[P*LDSO_BA_POINT_STRIDE], point_res_begin[P+1], res_target[R], res_state[R],
 *   res_energy[R], res_flags[R] with R = P*(N-1).  Returns 0 on success. */
int ldso_synth_fill(const ldso_synth_params *prm, ldso_ba_frame_state *frames, float *dI, float *calib,
                    float *frame_energy_th, int32_t *point_host, float *point_data, int32_t *point_res_begin,
                    int32_t *res_target, int8_t *res_state, float *res_energy, uint8_t *res_flags);

#ifdef __cplusplus
}
#endif

#endif
