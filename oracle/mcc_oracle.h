/*
 * mcc_oracle.h -- CPU restatement of the reference bundle-adjustment hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product (multi_camera_calibration_amd/csrc).  Only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
 * The product never links, calls or falls back to it.
 *
 * Restates (file:line under the reference yulong314/multi_camera_calibration):
 *   optimizeExtrinsics ............... src/multicalib.cpp:462-514
 *   sparseSolver / conjungate (CG) ... src/multicalib.cpp:565-592  (Eigen 3 ConjugateGradient,
 *                                      DiagonalPreconditioner, tol = DBL_EPSILON, maxIter = 2P)
 *   MultiCameraCalibration::computeJacobianExtrinsic / computePhotoCameraJacobian (omni)
 *                                      src/multicalib.cpp:593-703, 717-824
 *   MyMultiCameraCalibration::computeJacobianExtrinsic / computePhotoCameraJacobian (pinhole)
 *                                      src/mymulticalib.cpp:468-614, 668-818
 *   DoubleSideCalibration::computeJacobianExtrinsic / computePhotoCameraJacobian
 *                                      src/doubleSide.cpp:288-430, 434-581
 *   computeProjectError .............. src/multicalib.cpp:895-1006, src/mymulticalib.cpp:820-939,
 *                                      src/doubleSide.cpp:640-769
 *   compose_motion ................... src/multicalib.cpp:1008-1056
 *   cv::omnidir::projectPoints ....... src/omnidir.cpp:84-245
 *   OpenCV 4.x calib3d cv::Rodrigues / cv::projectPoints / cv::matMulDeriv and core small-matrix
 *   gemm (third-party, NOT vendored in the reference, version unpinned: README.md:14) restated
 *   from their published formulas -- see SURVEY.md Appendix A.  Parity of that arithmetic is
 *   "unpinned" (no OpenCV in this image); it is pinned instead by finite differences, Rodrigues
 *   identities and the camodocal PinholeCamera known-answer tests (camodocal/PinholeCamera_test.cc).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: the reference's OpenCV builds use the SSE
 * baseline, i.e. no fused multiply-add).
 */
#ifndef MCC_ORACLE_H
#define MCC_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

enum { ORA_PINHOLE = 0, ORA_OMNI = 1, ORA_DOUBLESIDE = 2 };
enum { ORA_FRONT = 0, ORA_BACK = 1 };
enum { ORA_SOLVER_CG = 0, ORA_SOLVER_SCHUR = 1, ORA_SOLVER_DENSE_J = 2 };

typedef struct ora_problem {
    int model;              /* ORA_PINHOLE (MyMulti), ORA_OMNI (base class), ORA_DOUBLESIDE   */
    int n_cams;             /* C: camera vertices 0..C-1 (camera 0 = identity, not optimised) */
    int n_photos;           /* V: photo vertices C..C+V-1 (stored as photo index 0..V-1)      */
    int n_edges;            /* E: (camera, photo) observations, in reference edge order       */
    const int *edge_cam;    /* [E] camera vertex                                              */
    const int *edge_photo;  /* [E] photo index (vertex - C)                                   */
    const int *edge_side;   /* [E] ORA_FRONT / ORA_BACK                                       */
    const int *edge_off;    /* [E] first corner                                               */
    const int *edge_n;      /* [E] corner count                                               */
    const float *obj;       /* [3 * corners] object points (x,y,z), CV_32F as stored by ref   */
    const float *img;       /* [2 * corners] observed corners (u,v), CV_32F                   */
    int nd;                 /* distortion coefficients per camera (pinhole 4/5/8/12, omni 4)  */
    const float *K;         /* [9 * C] row-major camera matrices, CV_32F                      */
    const float *D;         /* [nd * C] distortion, CV_32F                                    */
    const float *xi;        /* [C] Mei xi (omni only)                                         */
    const double *ds_pose;  /* [16] MyMulti doubleSideTransform (CV_64F 4x4), BACK edges only */
    const float *cam_pose;  /* [16 * C] DoubleSide fixed camera poses (CV_32F 4x4)            */
} ora_problem;

int ora_nparams(const ora_problem *p);
int ora_param_col_photo(const ora_problem *p, int photo);   /* first column of a photo */
int ora_param_col_cam(const ora_problem *p, int cam);       /* -1 for fixed cameras    */

/* OpenCV cvRodrigues2 semantics.  v2m: J is 3x9 (row = r_i, col = R row-major).
 * m2v: R is orthonormalised (polar factor = U*Vt of the SVD), J is 9x3. */
void ora_rodrigues_v2m(const double r[3], double R[9], double J[27]);
void ora_rodrigues_m2v(const double R[9], double r[3], double J[27]);

/* compose_motion, src/multicalib.cpp:1008-1056.  d[k] (3x3 row-major) in the reference's
 * output order: dom3dom1, dom3dT1, dom3dom2, dom3dT2, dT3dom1, dT3dT1, dT3dom2, dT3dT2. */
void ora_compose_motion(const double om1[3], const double T1[3], const double om2[3],
                        const double T2[3], double om3[3], double T3[3], double d[8][9]);

/* computeTiltProjectionMatrix: the tilted sensor's matTilt (3 x 3 row-major) for tau_x, tau_y */
void ora_tilt_matrix(double tauX, double tauY, double M[9]);

/* cv::projectPoints (pinhole, CV_32F object points -> CV_32F image points; nd 4, 5, 8, 12 or 14, the
 * last with the tilted-sensor projection).
 * jac (optional): 2n x 6 row-major, columns [d/drvec(3), d/dtvec(3)], rows u0,v0,u1,v1,... */
int ora_project_pinhole(int n, const float *obj, const float rvec[3], const float tvec[3],
                        const float K[9], const float *D, int nd, float *img, double *jac);

/* cv::omnidir::projectPoints, src/omnidir.cpp:84-245.  jac (optional): 2n x 6 (om, T). */
void ora_project_omni(int n, const float *obj, const float rvec[3], const float tvec[3],
                      const float K[9], double xi, const float D[4], float *img, double *jac);

/* Per-edge linearisation: the 2N x 6 Jacobian blocks of the global/camera vertex (jc, or the
 * double-side block for ORA_DOUBLESIDE) and of the photo vertex (jp), the 2N residual
 * E = fl32(obs - proj) as double, and the projected float pixels (proj, optional). */
int ora_edge_linearize(const ora_problem *p, const float *x, int e,
                       double *jc, double *jp, double *E, float *proj);

/* Dense faithful normal equations (J is (2*corners) x P, as src/mymulticalib.cpp:683). */
int ora_normal_dense(const ora_problem *p, const float *x, double *JTJ, double *JTE);

/* The same normal equations the way the reference forms them: a materialised dense J
 * ((2*corners) x P, zero-filled) and the dense products J^T J, J^T E (src/mymulticalib.cpp:683,
 * 802-803), single-threaded -- the ref-faithful CPU baseline's cost model. */
int ora_normal_dense_j(const ora_problem *p, const float *x, double *JTJ, double *JTE);

/* Eigen ConjugateGradient<Lower|Upper, DiagonalPreconditioner>, tol = eps, maxIter = 2P,
 * solve() called twice as in src/multicalib.cpp:571-577. Returns iterations of last solve. */
int ora_cg(int P, const double *A, const double *b, double *x);

/* One linearisation + solve (the computeJacobianExtrinsic seam).  solver ORA_SOLVER_CG is the
 * faithful dense path (dense J^T J accumulated per edge + CG x2), ORA_SOLVER_DENSE_J the same with
 * the materialised dense J and gemm products, ORA_SOLVER_SCHUR the exact block-sparse
 * Schur/Cholesky solve. */
int ora_linearize_solve(const ora_problem *p, const float *x, int solver,
                        double *delta, double *jte);

/* Block-sparse pieces (for tests / multi-rank decomposition checks).  Photo subset
 * [photo_lo, photo_hi) restricts the accumulation to those photos' edges.  The packed global
 * system has m = global block size; S is m x m (full), r is m. */
int ora_global_dim(const ora_problem *p);
int ora_schur_partial(const ora_problem *p, const float *x, int photo_lo, int photo_hi,
                      double *S, double *r);

/* Back-substitution of the photo blocks [lo, hi) for a given global step dg[m]:
 * dphoto[6 * (hi - lo)] (the rank-local half of a photo-sharded step). */
int ora_photo_backsub(const ora_problem *p, const float *x, int lo, int hi, const double *dg,
                      double *dphoto);

/* The optimizeExtrinsics loop.  crit_type: 1 COUNT, 2 EPS, 3 COUNT+EPS.  Returns the
 * computeProjectError mean (or a negative value on failure). */
double ora_optimize(const ora_problem *p, int crit_type, int max_count, double eps, int solver,
                    float *x, int *iters, double *last_change);

/* computeProjectError: per-edge mean L2 error (float) and the reference's mean
 * ((double)float-total / totalNPoints, with totalNPoints = 2N pinhole / N omni). */
int ora_project_error(const ora_problem *p, const float *x, float *edge_err, double *mean);

/* ---- cv::omnidir::calibrate, mcc_oracle_omnicalib.c.  Parameters in the
 * reference's encodeParameters layout: [om_i(3), T_i(3)] x n, fx, fy, s, cx, cy, xi, k1, k2, p1, p2
 * (P = 6n + 10), CV_64F.  Views are [off[i], off[i+1]) ranges of obj (xyz) / img (uv). */
/* projectPoints with the 2x16 Jacobian (JacobianRow order); kin = fx, fy, s, cx, cy */
void ora_omni_project_full(int n, const double *obj, const double om[3], const double T[3],
                           const double kin[5], double xi, const double D[4], double *img, double *jac);
void ora_omni_flags2idx(int flags, int n, int *idx);
/* computeJacobian: JTE before subMatrix (P), and/or (JTJ + epsilon)^-1 and JTE after it (n_free) */
int ora_omni_jacobian(int n, const int *off, const double *obj, const double *img, const double *para,
                      int flags, double epsilon, double *JTJ_inv, double *JTE_full, double *JTE_sub, int *n_free);
/* G of the loop at iteration iter (alpha_smooth2, epsilon, fillFixed), P long */
int ora_omni_step(int n, const int *off, const double *obj, const double *img, const double *para,
                  int flags, int iter, double *G);
int ora_omni_optimize(int n, const int *off, const double *obj, const double *img, double *para, int flags,
                      int crit_type, int max_count, double eps, int *iters, double *last_change);
double ora_omni_rms(int n, const int *off, const double *obj, const double *img, const double *para);
int ora_omni_init(int n_img, const int *off, const double *obj, const double *img, int width, int height,
                  double *om_out, double *t_out, double *K, double *xi, int *idx, int *n_idx);
double ora_omni_calibrate(int n_img, const int *off, const double *obj, const double *img, int width, int height,
                          int flags, int crit_type, int max_count, double eps, double *K, double *xi, double *D,
                          double *om, double *t, int *idx, int *n_idx, int *iters);

/* OpenMP threads the oracle uses (1 if built without OpenMP). */
int ora_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
