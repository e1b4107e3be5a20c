// host_math.cpp -- host-side (double precision) pieces of the hot path that run once per
// iteration on a handful of numbers: FrameFramePrecalc::Set, EnergyFunctional::setAdjointsF,
// FrameHessian::takeData, getNullspaces and the solve of EnergyFunctional::solveSystemF.
// They are O(N^2) or O((8N+4)^3) with N <= 16 and stay on the CPU next to the caller.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/ldso_ba.h"
#include "ldso_ba_internal.h"
#include "se3.h"

namespace ldso_ba {

// FrameFramePrecalc::Set (src/internal/FrameFramePrecalc.cc:6-35) for all (h,t)
int frame_precalc(int N, const ldso_ba_frame_state *fr, const float calib[4], float *out) {
    std::vector<Pose> ev(N), cur(N);
    for (int f = 0; f < N; f++) {
        ev[f] = eval_pose(fr[f]);
        cur[f] = current_pose(fr[f]);
    }
    for (int h = 0; h < N; h++) {
        const Pose evInvH = ev[h].inverse(), curInvH = cur[h].inverse();
        for (int t = 0; t < N; t++)
            pair_precalc(ev[t], evInvH, cur[t], curInvH, calib, fr[h], fr[t],
                         out + (size_t)(h + N * t) * LDSO_BA_PRECALC_STRIDE);
    }
    return 0;
}

// EnergyFunctional::setAdjointsF (EnergyFunctional.cc:551-609)
int set_adjoints(int N, const ldso_ba_frame_state *fr, double *adH, double *adT, double *cPrior) {
    std::vector<Pose> ev(N);
    for (int f = 0; f < N; f++) ev[f] = eval_pose(fr[f]);
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            double adj[36];
            (ev[t] * ev[h].inverse()).adjoint(adj);
            double *AH = adH + (size_t)(h + t * N) * 64, *AT = adT + (size_t)(h + t * N) * 64;
            std::memset(AH, 0, 64 * sizeof(double));
            std::memset(AT, 0, 64 * sizeof(double));
            for (int i = 0; i < 8; i++) AH[i * 9] = AT[i * 9] = 1;
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 6; c++) AH[r * 8 + c] = -adj[c * 6 + r];  // -Adj^T
            float a, b;
            affine_from_to((float)fr[h].ab_exposure, (float)fr[t].ab_exposure, (float)(fr[h].state_zero[6] * kScaleA),
                           (float)(fr[h].state_zero[7] * kScaleB), (float)(fr[t].state_zero[6] * kScaleA),
                           (float)(fr[t].state_zero[7] * kScaleB), a, b);
            (void)b;
            AT[6 * 8 + 6] = -a;
            AH[6 * 8 + 6] = a;
            AT[7 * 8 + 7] = -1;
            AH[7 * 8 + 7] = a;
            const double rs[8] = {kScaleXiTrans, kScaleXiTrans, kScaleXiTrans, kScaleXiRot, kScaleXiRot, kScaleXiRot, kScaleA, kScaleB};
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) {
                    AH[r * 8 + c] *= rs[r];
                    AT[r * 8 + c] *= rs[r];
                }
        }
    if (cPrior)
        for (int i = 0; i < 4; i++) cPrior[i] = kInitialCalibHessian;
    return 0;
}

// FrameHessian::takeData / getPrior / get_state_minus_stateZero (FrameHessian.h:59-70,142-174)
int frame_take_data(int N, const ldso_ba_frame_state *fr, float mode_a, float mode_b, double *prior, double *delta,
                    double *delta_prior) {
    for (int f = 0; f < N; f++)
        frame_take_data_one(fr[f], mode_a, mode_b, prior ? prior + 8 * f : nullptr, delta ? delta + 8 * f : nullptr,
                            delta_prior ? delta_prior + 8 * f : nullptr);
    return 0;
}

// FrameHessian::setStateZero nullspaces (FrameHessian.cc:26-57) + FullSystem::getNullspaces
// (FullSystem.cc:2027-2076): out[7][8N+4] = pose x6 then scale, as orthogonalize() stacks them
int nullspaces(int N, const ldso_ba_frame_state *fr, double *out) {
    const int n = 8 * N + 4;
    std::memset(out, 0, sizeof(double) * 7 * n);
    const double unscale[6] = {1.0 / (double)0.5f, 1.0 / (double)0.5f, 1.0 / (double)0.5f, 1, 1, 1};
    for (int f = 0; f < N; f++) {
        Pose E = eval_pose(fr[f]), Ei = E.inverse();
        for (int i = 0; i < 6; i++) {
            double ep[6] = {0, 0, 0, 0, 0, 0}, em[6] = {0, 0, 0, 0, 0, 0}, lp[6], lm[6];
            ep[i] = 1e-3;
            em[i] = -1e-3;
            ((E * Pose::exp(ep)) * Ei).log(lp);
            ((E * Pose::exp(em)) * Ei).log(lm);
            for (int k = 0; k < 6; k++) out[(size_t)i * n + 4 + 8 * f + k] = (lp[k] - lm[k]) / 2e-3 * unscale[k];
        }
        Pose P = E, M = E;
        for (int k = 0; k < 3; k++) {
            P.t[k] *= 1.00001;
            M.t[k] /= 1.00001;
        }
        double lp[6], lm[6];
        (P * Ei).log(lp);
        (M * Ei).log(lm);
        for (int k = 0; k < 6; k++) out[(size_t)6 * n + 4 + 8 * f + k] = (lp[k] - lm[k]) / 2e-3 * unscale[k];
    }
    return 0;
}

namespace {
// In-place LDL^T with symmetric diagonal pivoting (Eigen::LDLT's strategy), then solve.  Only
// the lower triangle is kept: a symmetric swap of k < p touches (k,j)<->(p,j) for j < k,
// (i,k)<->(p,i) for k < i < p, (i,k)<->(i,p) for i > p and the two diagonals; every element
// sees the same operations as with a full symmetric matrix.
void ldlt_solve(int n, std::vector<double> &A, std::vector<double> &b) {
    std::vector<int> perm(n);
    std::vector<double> col(n, 0.0);
    for (int i = 0; i < n; i++) perm[i] = i;
    double *a = A.data();
    auto at = [a, n](int r, int c) -> double & { return a[(size_t)r * n + c]; };
    for (int k = 0; k < n; k++) {
        int piv = k;
        for (int i = k + 1; i < n; i++)
            if (std::fabs(at(i, i)) > std::fabs(at(piv, piv))) piv = i;
        if (piv != k) {
            std::swap(perm[k], perm[piv]);
            for (int j = 0; j < k; j++) std::swap(at(k, j), at(piv, j));
            for (int i = k + 1; i < piv; i++) std::swap(at(i, k), at(piv, i));
            for (int i = piv + 1; i < n; i++) std::swap(at(i, k), at(i, piv));
            std::swap(at(k, k), at(piv, piv));
        }
        const double d = at(k, k);
        // trailing update with the unscaled column c = A(., k): A(i,j) = fma(-(c_i c_j), 1/d,
        // A(i,j)) -- symmetric in i and j, so the device kernels may update either triangle --
        // then L(i,k) = c_i / d
        const double rd = d != 0 ? 1.0 / d : 0.0;
        for (int i = k + 1; i < n; i++) col[i] = at(i, k);
        for (int i = k + 1; i < n; i++) {
            const double ci = col[i];
            double *row = &at(i, 0);
            for (int j = k + 1; j <= i; j++) row[j] = std::fma(-(ci * col[j]), rd, row[j]);
            row[k] = d != 0 ? ci / d : 0.0;
        }
    }
    std::vector<double> y(n);
    for (int i = 0; i < n; i++) y[i] = b[perm[i]];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) y[i] = std::fma(-at(i, j), y[j], y[i]);
    for (int i = 0; i < n; i++) y[i] = at(i, i) != 0 ? y[i] / at(i, i) : 0.0;
    // back substitution column by column (j descending), the order k_solve uses on the GPU
    for (int j = n - 1; j >= 0; j--)
        for (int i = 0; i < j; i++) y[i] = std::fma(-at(j, i), y[j], y[i]);
    for (int i = 0; i < n; i++) b[perm[i]] = y[i];
}

// x -= N (N^T N)^+ N^T x with columns normalised and singular values below
// setting_solverModeDelta * max cut (EnergyFunctional::orthogonalize, EnergyFunctional.cc:809-841)
void project_out(int n, const double *ns, int k, std::vector<double> &x) {
    std::vector<double> Nm((size_t)n * k);
    for (int c = 0; c < k; c++) {
        double s = 0;
        for (int i = 0; i < n; i++) s += ns[(size_t)c * n + i] * ns[(size_t)c * n + i];
        s = std::sqrt(s);
        for (int i = 0; i < n; i++) Nm[(size_t)i * k + c] = ns[(size_t)c * n + i] / s;
    }
    std::vector<double> G((size_t)k * k, 0.0), V((size_t)k * k, 0.0);
    for (int a = 0; a < k; a++)
        for (int c = 0; c < k; c++)
            for (int i = 0; i < n; i++) G[(size_t)a * k + c] += Nm[(size_t)i * k + a] * Nm[(size_t)i * k + c];
    for (int i = 0; i < k; i++) V[(size_t)i * k + i] = 1;
    std::vector<double> ntx(k, 0.0), coef(k, 0.0);
    for (int a = 0; a < k; a++)
        for (int i = 0; i < n; i++) ntx[a] += Nm[(size_t)i * k + a] * x[i];
    bool fast = false;
    if (k == 7) {
        double g7[7][7], n7[7], c7[7];
        for (int a = 0; a < 7; a++) {
            n7[a] = ntx[a];
            for (int c = 0; c < 7; c++) g7[a][c] = G[(size_t)a * 7 + c];
        }
        fast = gram_inverse_coef7(g7, n7, c7);
        if (fast)
            for (int a = 0; a < 7; a++) coef[a] = c7[a];
    }
    // Jacobi sweeps in round-robin order (circle method): 7 rounds of 3 disjoint rotations; in a
    // round all angles come from the round's starting G, then every column update, then every row
    // update (disjoint pairs make both phases order-free).  k_solve runs the same rounds.
    if (!fast) {
        static constexpr int kRounds[7][3][2] = {
            {{1, 6}, {2, 5}, {3, 4}}, {{0, 2}, {3, 6}, {4, 5}}, {{1, 3}, {0, 4}, {5, 6}}, {{2, 4}, {1, 5}, {0, 6}},
            {{3, 5}, {2, 6}, {0, 1}}, {{4, 6}, {0, 3}, {1, 2}}, {{0, 5}, {1, 4}, {2, 3}}};
        for (int sweep = 0; sweep < 64; sweep++) {
            double off = 0;
            for (int p = 0; p < k; p++)
                for (int q = p + 1; q < k; q++) off += G[(size_t)p * k + q] * G[(size_t)p * k + q];
            if (off < 1e-30) break;
            for (int rd = 0; rd < 7; rd++) {
                double c[3], s[3];
                bool on[3];
                for (int e = 0; e < 3; e++) {
                    const int p = kRounds[rd][e][0], q = kRounds[rd][e][1];
                    on[e] = q < k && G[(size_t)p * k + q] != 0;
                    if (!on[e]) continue;
                    const double apq = G[(size_t)p * k + q];
                    const double th = (G[(size_t)q * k + q] - G[(size_t)p * k + p]) / (2 * apq);
                    const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1));
                    c[e] = 1 / std::sqrt(t * t + 1);
                    s[e] = t * c[e];
                }
                for (int e = 0; e < 3; e++) {
                    if (!on[e]) continue;
                    const int p = kRounds[rd][e][0], q = kRounds[rd][e][1];
                    for (int r = 0; r < k; r++) {
                        const double gp = G[(size_t)r * k + p], gq = G[(size_t)r * k + q];
                        G[(size_t)r * k + p] = c[e] * gp - s[e] * gq;
                        G[(size_t)r * k + q] = s[e] * gp + c[e] * gq;
                    }
                }
                for (int e = 0; e < 3; e++) {
                    if (!on[e]) continue;
                    const int p = kRounds[rd][e][0], q = kRounds[rd][e][1];
                    for (int r = 0; r < k; r++) {
                        const double gp = G[(size_t)p * k + r], gq = G[(size_t)q * k + r];
                        G[(size_t)p * k + r] = c[e] * gp - s[e] * gq;
                        G[(size_t)q * k + r] = s[e] * gp + c[e] * gq;
                        const double vp = V[(size_t)r * k + p], vq = V[(size_t)r * k + q];
                        V[(size_t)r * k + p] = c[e] * vp - s[e] * vq;
                        V[(size_t)r * k + q] = s[e] * vp + c[e] * vq;
                    }
                }
            }
        }
        double smax = 0;
        for (int e = 0; e < k; e++) smax = std::max(smax, std::sqrt(std::max(0.0, G[(size_t)e * k + e])));
        for (int e = 0; e < k; e++) {
            const double ev = G[(size_t)e * k + e];
            if (!(std::sqrt(std::max(0.0, ev)) > kSolverModeDelta * smax)) continue;
            double proj = 0;
            for (int a = 0; a < k; a++) proj += V[(size_t)a * k + e] * ntx[a];
            for (int a = 0; a < k; a++) coef[a] += V[(size_t)a * k + e] * proj / ev;
        }
    }
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int a = 0; a < k; a++) s += Nm[(size_t)i * k + a] * coef[a];
        x[i] -= s;
    }
}
}  // namespace

// EnergyFunctional::solveSystemF, non-VI / FIX_LAMBDA / ORTHOGONALIZE_X_LATER branch
// (EnergyFunctional.cc:282-283, 310, 342-378, 413-432)
int solve_system(int N, int iteration, double lambda, const double *HA, const double *bA, const double *HL,
                 const double *bL, const double *HM, const double *bM, const double *Hsc, const double *bsc,
                 const double *ns, int n_null, double *x_out) {
    const int n = 8 * N + 4;
    (void)lambda;
    lambda = 1e-5;  // SOLVER_FIX_LAMBDA
    std::vector<double> H((size_t)n * n), b(n);
    for (int i = 0; i < n; i++) {
        for (int j = i; j < n; j++) {
            const size_t q = (size_t)i * n + j;
            H[q] = HL[q] + (HM ? HM[q] : 0.0) + HA[q];
        }
        b[i] = bL[i] + (bM ? bM[i] : 0.0) + bA[i] - bsc[i] / (1 + lambda);
    }
    for (int i = 0; i < n; i++) H[(size_t)i * n + i] *= (1 + lambda);
    const double sc = 1.0f / (1 + lambda);
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) H[(size_t)i * n + j] -= Hsc[(size_t)i * n + j] * sc;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) H[(size_t)i * n + j] = H[(size_t)j * n + i];
    std::vector<double> s(n);
    for (int i = 0; i < n; i++) s[i] = 1.0 / std::sqrt(H[(size_t)i * n + i] + 10);
    for (int i = 0; i < n; i++) {
        b[i] *= s[i];
        for (int j = 0; j < n; j++) H[(size_t)i * n + j] *= s[i] * s[j];
    }
    ldlt_solve(n, H, b);
    std::vector<double> x(n);
    for (int i = 0; i < n; i++) x[i] = s[i] * b[i];
    if (iteration >= 2 && ns && n_null > 0) project_out(n, ns, n_null, x);
    std::memcpy(x_out, x.data(), n * sizeof(double));
    return 0;
}

namespace {
// util::MatrixInverter::invertPosDef, non-fast branch (src/util/MatrixInverter.cc:25-51): Jacobi
// scaling, pseudo-inverse of the scaled symmetric matrix (the SVD of a symmetric matrix has
// V diag(1/sigma) U^T = sum over non-zero eigenvalues of q q^T / lambda), scaling undone.
// M is read as selfadjointView<Upper>; the full symmetric inverse is returned.
void invert_pos_def(int n, const double *M, double *out) {
    std::vector<double> s(n), A((size_t)n * n), V((size_t)n * n, 0.0);
    for (int i = 0; i < n; i++) s[i] = 1.0 / std::sqrt(std::fabs(M[(size_t)i * n + i]) + 10);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const double m = i <= j ? M[(size_t)i * n + j] : M[(size_t)j * n + i];
            A[(size_t)i * n + j] = s[i] * m * s[j];
        }
    for (int i = 0; i < n; i++) V[(size_t)i * n + i] = 1;
    for (int sweep = 0; sweep < 100; sweep++) {  // cyclic Jacobi
        double off = 0, diag = 0;
        for (int p = 0; p < n; p++) {
            diag += A[(size_t)p * n + p] * A[(size_t)p * n + p];
            for (int q = p + 1; q < n; q++) off += A[(size_t)p * n + q] * A[(size_t)p * n + q];
        }
        if (off <= 1e-32 * diag) break;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[(size_t)p * n + q];
                if (apq == 0) continue;
                const double th = (A[(size_t)q * n + q] - A[(size_t)p * n + p]) / (2 * apq);
                const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1));
                const double c = 1 / std::sqrt(t * t + 1), sn = t * c;
                for (int k = 0; k < n; k++) {
                    const double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
                    A[(size_t)k * n + p] = c * akp - sn * akq;
                    A[(size_t)k * n + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    const double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
                    A[(size_t)p * n + k] = c * apk - sn * aqk;
                    A[(size_t)q * n + k] = sn * apk + c * aqk;
                    const double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
                    V[(size_t)k * n + p] = c * vkp - sn * vkq;
                    V[(size_t)k * n + q] = sn * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double acc = 0;
            for (int e = 0; e < n; e++) {
                const double lam = A[(size_t)e * n + e];
                if (lam != 0) acc += V[(size_t)i * n + e] * V[(size_t)j * n + e] / lam;
            }
            out[(size_t)i * n + j] = s[i] * acc * s[j];
        }
}
}  // namespace

// EnergyFunctional::marginalizeFrame (EnergyFunctional.cc:109-191), HM / bM part
int marginalize_frame(int N, int idx, const double *HM, const double *bM, const double *prior,
                      const double *delta_prior, double *HM_out, double *bM_out) {
    const int odim = 8 * N + 4, ndim = odim - 8;
    std::vector<double> H(HM, HM + (size_t)odim * odim), b(bM, bM + odim);
    if (idx != N - 1) {  // move frame idx's rows and columns to the end, :120-139
        const int io = idx * 8 + 4;
        std::vector<int> order;  // new position -> old index
        for (int i = 0; i < io; i++) order.push_back(i);
        for (int i = io + 8; i < odim; i++) order.push_back(i);
        for (int i = io; i < io + 8; i++) order.push_back(i);
        std::vector<double> H2((size_t)odim * odim), b2(odim);
        for (int i = 0; i < odim; i++) {
            b2[i] = b[order[i]];
            for (int j = 0; j < odim; j++) H2[(size_t)i * odim + j] = H[(size_t)order[i] * odim + order[j]];
        }
        H.swap(H2);
        b.swap(b2);
    }
    for (int i = 0; i < 8; i++) {  // the frame's prior, :143-144
        H[(size_t)(ndim + i) * odim + ndim + i] += prior[i];
        b[ndim + i] += prior[i] * delta_prior[i];
    }
    std::vector<double> sv(odim), svi(odim);
    for (int i = 0; i < odim; i++) {
        sv[i] = std::sqrt(std::fabs(H[(size_t)i * odim + i]) + 10);
        svi[i] = 1.0 / sv[i];
    }
    for (int i = 0; i < odim; i++) {
        b[i] *= svi[i];
        for (int j = 0; j < odim; j++) H[(size_t)i * odim + j] *= svi[i] * svi[j];
    }
    double hp[64], hpi[64];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) hp[i * 8 + j] = H[(size_t)(ndim + i) * odim + ndim + j];
    invert_pos_def(8, hp, hpi);
    // bli = H(bottom, 0:ndim)^T hpi; H(0:ndim, 0:ndim) -= bli H(bottom, 0:ndim); b -= bli b_tail
    std::vector<double> bli((size_t)ndim * 8);
    for (int i = 0; i < ndim; i++)
        for (int k = 0; k < 8; k++) {
            double acc = 0;
            for (int m = 0; m < 8; m++) acc += H[(size_t)(ndim + m) * odim + i] * hpi[m * 8 + k];
            bli[(size_t)i * 8 + k] = acc;
        }
    for (int i = 0; i < ndim; i++) {
        for (int j = 0; j < ndim; j++) {
            double acc = 0;
            for (int k = 0; k < 8; k++) acc += bli[(size_t)i * 8 + k] * H[(size_t)(ndim + k) * odim + j];
            H[(size_t)i * odim + j] -= acc;
        }
        double acc = 0;
        for (int k = 0; k < 8; k++) acc += bli[(size_t)i * 8 + k] * b[ndim + k];
        b[i] -= acc;
    }
    for (int i = 0; i < ndim; i++) {  // unscale and symmetrise, :166-171
        bM_out[i] = sv[i] * b[i];
        for (int j = 0; j < ndim; j++) H[(size_t)i * odim + j] *= sv[i] * sv[j];
    }
    for (int i = 0; i < ndim; i++)
        for (int j = 0; j < ndim; j++)
            HM_out[(size_t)i * ndim + j] = 0.5 * (H[(size_t)i * odim + j] + H[(size_t)j * odim + i]);
    return 0;
}

}  // namespace ldso_ba

namespace ldso_ba {

// EnergyFunctional::setDeltaF's adHTdeltaF (EnergyFunctional.cc:523-533): for every (h, t),
// delta_h^T adHostF + delta_t^T adTargetF in float (Mat18f = Vec8f^T * Mat88f), index h + N t.
int ad_ht_delta(int N, const double *delta, const double *adH, const double *adT, float *out) {
    for (int h = 0; h < N; h++)
        for (int t = 0; t < N; t++) {
            const int idx = h + t * N;
            float dh[8], dt[8];
            for (int k = 0; k < 8; k++) {
                dh[k] = (float)delta[8 * h + k];
                dt[k] = (float)delta[8 * t + k];
            }
            for (int j = 0; j < 8; j++) {
                float a = 0.f, b = 0.f;
                for (int k = 0; k < 8; k++) {
                    a += dh[k] * (float)adH[(size_t)idx * 64 + k * 8 + j];
                    b += dt[k] * (float)adT[(size_t)idx * 64 + k * 8 + j];
                }
                out[(size_t)idx * 8 + j] = a + b;
            }
        }
    return 0;
}

// EnergyFunctional::calcMEnergyF (EnergyFunctional.cc:473-479): delta^T (2 bM + HM delta) with
// delta = getStitchedDeltaF() = [cDeltaF; frames' delta] (EnergyFunctional.h:192-198).
double calc_m_energy(int N, const double *HM, const double *bM, const float *c_delta, const double *frame_delta) {
    const int n = 8 * N + 4;
    std::vector<double> d(n);
    for (int i = 0; i < 4; i++) d[i] = (double)c_delta[i];
    for (int i = 0; i < 8 * N; i++) d[4 + i] = frame_delta[i];
    double e = 0;
    for (int r = 0; r < n; r++) {
        double hd = 0;
        for (int c = 0; c < n; c++) hd += HM[(size_t)r * n + c] * d[c];
        e += d[r] * (2 * bM[r] + hd);
    }
    return e;
}

// EnergyFunctional::calcLEnergyF_MT (EnergyFunctional.cc:481-498) with calcLEnergyPt
// (:751-806): the frame priors in double, the calibration prior in float, and per point the
// Accumulator11 float sums (MatrixAccumulators.h:68-123) over IndexThreadReduce chunks of 50
// points, each chunk's float total added to the double stats in chunk order.  The
// linearised-residual term (2 res_toZeroF + J delta) J delta is empty: residuals are only ever
// linearised inside marginalizePointsF, which removes their points in the same call
// (ldso_ba_marginalize_points), exactly as FullSystem::flagPointsForRemoval + marginalizePointsF.
double calc_l_energy(int N, const double *frame_prior, const double *frame_delta_prior, const double *c_prior,
                     const float *c_delta, int n_points, const float *deltaF, const float *priorF) {
    double E = 0;
    for (int f = 0; f < N; f++) {
        double s = 0;
        for (int k = 0; k < 8; k++)
            s += frame_delta_prior[8 * f + k] * frame_prior[8 * f + k] * frame_delta_prior[8 * f + k];
        E += s;
    }
    float sc = 0.f;
    for (int k = 0; k < 4; k++) sc += c_delta[k] * (float)c_prior[k] * c_delta[k];
    E += sc;
    double stats = 0;
    for (int c0 = 0; c0 < n_points; c0 += 50) {
        float acc = 0.f;  // Accumulator11::SSEData[0]; finish() moves it through the 1k / 1m stages
        for (int q = c0; q < n_points && q < c0 + 50; q++) acc += deltaF[q] * deltaF[q] * priorF[q];
        float a1k = 0.f, a1m = 0.f;
        a1k += acc;
        a1m += a1k;
        stats += (double)(((a1m + 0.f) + 0.f) + 0.f);
    }
    return E + stats;
}

}  // namespace ldso_ba
