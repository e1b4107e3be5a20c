// ldso_ba_internal.h -- constants of the hot path (include/Settings.h, src/Setting.cc) and
// host-side helpers shared by the C ABI translation units.
#pragma once
#include "../../include/ldso_ba.h"

namespace ldso_ba {

// include/Settings.h:28-35
constexpr float kScaleIdepth = 1.0f;
constexpr float kScaleF = 50.0f;
constexpr float kScaleC = 50.0f;
// src/Setting.cc
constexpr float kOutlierTHSumComponent = 50.0f * 50.0f;  // :41
constexpr float kHuberTH = 9.0f;                           // :76
constexpr float kAffineOptModeA = 1e12f;                   // :65
constexpr float kAffineOptModeB = 1e8f;                    // :66
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

int frame_precalc(int N, const ldso_ba_frame_state *fr, const float calib[4], float *out);
int set_adjoints(int N, const ldso_ba_frame_state *fr, double *adH, double *adT, double *cPrior);
int frame_take_data(int N, const ldso_ba_frame_state *fr, double *prior, double *delta, double *delta_prior);
int nullspaces(int N, const ldso_ba_frame_state *fr, double *out);
int solve_system(int N, int iteration, double lambda, const double *HA, const double *bA, const double *HL,
                 const double *bL, const double *HM, const double *bM, const double *Hsc, const double *bsc,
                 const double *ns, int n_null, double *x_out);

}  // namespace ldso_ba
