// ldso_ba_internal.h -- constants of the hot path (include/Settings.h, src/Setting.cc) and
// host-side helpers shared by the C ABI translation units.
#pragma once
#include <string>

#include "../../include/ldso_ba.h"

#if defined(__HIP__)
#define LDSO_HD __host__ __device__
#else
#define LDSO_HD
#endif

namespace ldso_ba {

// include/Settings.h:28-35
constexpr float kScaleIdepth = 1.0f;
constexpr float kScaleF = 50.0f;
constexpr float kScaleC = 50.0f;
// src/Setting.cc
constexpr float kOutlierTHSumComponent = 50.0f * 50.0f;  // :41
constexpr float kHuberTH = 9.0f;                           // :76
constexpr float kFrameEnergyTHN = 0.7f;                    // :79
constexpr float kFrameEnergyTHConstWeight = 0.5f;          // :77
constexpr float kFrameEnergyTHFacMedian = 1.5f;            // :81
constexpr float kOverallEnergyTHWeight = 1.0f;             // :82
constexpr float kInitialCalibHessian = 5e9f;               // :22
constexpr float kInitialRotPrior = 1e11f;                  // :18
constexpr float kInitialTransPrior = 1e10f;                // :19
constexpr float kInitialAffBPrior = 1e14f;                 // :20
constexpr float kInitialAffAPrior = 1e14f;                 // :21
constexpr double kSolverModeDelta = 0.00001;               // :24
constexpr float kIdepthFixPriorMargFac = 600.0f * 600.0f;   // :17
constexpr float kMargWeightFac = 0.5f * 0.5f;               // :45

// Fast path of the nullspace projection (EnergyFunctional::orthogonalize, EnergyFunctional.cc:809-841)
// for 7 nullspaces: when the Gram matrix G = N^T N of the normalised nullspaces is so well
// conditioned that no singular value of N can fall under kSolverModeDelta * max (checked with
// lambda_min >= 1 / |G^-1|_F and lambda_max <= trace G, with a factor 2 margin), the
// pseudo-inverse is the inverse: coef = G^-1 N^T x via Cholesky.  Returns false (coef untouched)
// otherwise, and the caller runs the Jacobi eigen-decomposition.  One definition for the host
// solver and k_solve, so both produce the same bits.
LDSO_HD inline bool gram_pinv7(const double (&G)[7][7], double (&Gi)[7][7]) {
#pragma clang fp contract(off)
    double L[7][7], Li[7][7];
    for (int j = 0; j < 7; j++) {
        double s = G[j][j];
        for (int p = 0; p < j; p++) s -= L[j][p] * L[j][p];
        if (!(s > 0)) return false;
        L[j][j] = sqrt(s);
        for (int i = j + 1; i < 7; i++) {
            double t = G[i][j];
            for (int p = 0; p < j; p++) t -= L[i][p] * L[j][p];
            L[i][j] = t / L[j][j];
        }
        for (int i = 0; i < j; i++) L[i][j] = 0;
    }
    for (int c = 0; c < 7; c++)  // L^-1, column by column (forward substitution on e_c)
        for (int i = 0; i < 7; i++) {
            if (i < c) {
                Li[i][c] = 0;
                continue;
            }
            double t = i == c ? 1.0 : 0.0;
            for (int p = c; p < i; p++) t -= L[i][p] * Li[p][c];
            Li[i][c] = t / L[i][i];
        }
    double f2 = 0, tr = 0;
    for (int a = 0; a < 7; a++) {
        tr += G[a][a];
        for (int b = 0; b < 7; b++) {
            double t = 0;
            for (int i = (a > b ? a : b); i < 7; i++) t += Li[i][a] * Li[i][b];
            Gi[a][b] = t;
            f2 += t * t;
        }
    }
    return kSolverModeDelta * kSolverModeDelta * tr * sqrt(f2) < 0.5;
}
// coef = G^-1 ntx, row by row (the second half of the fast path)
LDSO_HD inline double gram_apply7_row(const double *Gi_row, const double *ntx) {
#pragma clang fp contract(off)
    double t = 0;
    for (int b = 0; b < 7; b++) t += Gi_row[b] * ntx[b];
    return t;
}
LDSO_HD inline bool gram_inverse_coef7(const double (&G)[7][7], const double (&ntx)[7], double (&coef)[7]) {
    double Gi[7][7];
    if (!gram_pinv7(G, Gi)) return false;
    for (int a = 0; a < 7; a++) coef[a] = gram_apply7_row(Gi[a], ntx);
    return true;
}

// the ldso_ba_last_error() message of this thread; returns code
int set_error(int code, const std::string &msg);

int frame_precalc(int N, const ldso_ba_frame_state *fr, const float calib[4], float *out);
int set_adjoints(int N, const ldso_ba_frame_state *fr, double *adH, double *adT, double *cPrior);
int frame_take_data(int N, const ldso_ba_frame_state *fr, float mode_a, float mode_b, double *prior, double *delta,
                    double *delta_prior);
int nullspaces(int N, const ldso_ba_frame_state *fr, double *out);
int solve_system(int N, int iteration, double lambda, const double *HA, const double *bA, const double *HL,
                 const double *bL, const double *HM, const double *bM, const double *Hsc, const double *bsc,
                 const double *ns, int n_null, double *x_out);
int ad_ht_delta(int N, const double *delta, const double *adH, const double *adT, float *out);
double calc_m_energy(int N, const double *HM, const double *bM, const float *c_delta, const double *frame_delta);
double calc_l_energy(int N, const double *frame_prior, const double *frame_delta_prior, const double *c_prior,
                     const float *c_delta, int n_points, const float *deltaF, const float *priorF);
int marginalize_frame(int N, int idx, const double *HM, const double *bM, const double *prior,
                      const double *delta_prior, double *HM_out, double *bM_out);

}  // namespace ldso_ba
