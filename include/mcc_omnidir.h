/*
 * mcc_omnidir.h -- C ABI of the MI355X per-camera intrinsic calibration of the Mei omnidirectional
 * model (libmcc.so): cv::omnidir::calibrate, SURVEY.md 8(f) row 4.
 *
 * The reference calls it once per camera from MultiCameraCalibration::loadImages
 * (src/multicalib.cpp:273-278, TermCriteria(COUNT + EPS, 300, 1e-7)) before the extrinsic
 * bundle adjustment of mcc.h, and the omnidir tutorial calls it directly
 * (tutorials/omnidir_tutorial.markdown:45-49).  Entry points and the reference code each replaces:
 *
 *   mcc_omnidir_calibrate ....... cv::omnidir::calibrate (include/opencv2/ccalib/omnidir.hpp,
 *                                 src/omnidir.cpp:1067-1211): initialise, then the loop, then the
 *                                 rms of estimateUncertainties.
 *   mcc_omnidir_initialize ...... cv::omnidir::internal::initializeCalibration
 *                                 (src/omnidir.cpp:551-748); host code, no GPU.
 *   mcc_omnicalib_create ........ the per-view point lists calibrate converts to CV_64F
 *                                 (src/omnidir.cpp:1083-1094), deep-copied to the device.
 *   mcc_omnicalib_jacobian ...... cv::omnidir::internal::computeJacobian (src/omnidir.cpp:851-935)
 *                                 and one G of the loop (src/omnidir.cpp:1134-1142).
 *   mcc_omnicalib_optimize ...... the loop of calibrate (src/omnidir.cpp:1126-1149), on the device.
 *   mcc_omnicalib_rms ........... estimateUncertainties' rms (src/omnidir.cpp:1791-1803).
 *
 * Parameters use the reference's encodeParameters layout (src/omnidir.cpp:1541-1568), CV_64F:
 *   x = [om_0(3), T_0(3), ..., om_{n-1}, T_{n-1}, fx, fy, s, cx, cy, xi, k1, k2, p1, p2], P = 6n + 10.
 * The reference's JTJ + epsilon adds epsilon to EVERY entry of the (flag-reduced) dense normal
 * matrix; the device solves it exactly as a block-arrow Schur system plus a Sherman-Morrison
 * correction for the rank-one epsilon * 1 1^T term -- never a dense P x P matrix.
 *
 * Conventions as mcc.h: 0 = OK, negative MCC_E* on error, message in mcc_last_error().
 */
#ifndef MCC_OMNIDIR_H
#define MCC_OMNIDIR_H

#include "mcc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cv::omnidir flags (include/opencv2/ccalib/omnidir.hpp:56-66) */
#define MCC_OMNI_CALIB_USE_GUESS 1
#define MCC_OMNI_CALIB_FIX_SKEW 2
#define MCC_OMNI_CALIB_FIX_K1 4
#define MCC_OMNI_CALIB_FIX_K2 8
#define MCC_OMNI_CALIB_FIX_P1 16
#define MCC_OMNI_CALIB_FIX_P2 32
#define MCC_OMNI_CALIB_FIX_XI 64
#define MCC_OMNI_CALIB_FIX_GAMMA 128
#define MCC_OMNI_CALIB_FIX_CENTER 256

typedef struct mcc_omnicalib mcc_omnicalib;

typedef struct mcc_omnicalib_desc {
    int n_views;
    const int *view_off;   /* [n_views + 1] corner ranges                        */
    const double *obj;     /* [3 * corners] pattern points (x, y, z)             */
    const double *img;     /* [2 * corners] image points (u, v)                  */
    int flags;             /* MCC_OMNI_CALIB_FIX_* (flags2idx semantics)         */
    int device;            /* HIP device ordinal                                 */
} mcc_omnicalib_desc;

int mcc_omnicalib_create(mcc_omnicalib **out, const mcc_omnicalib_desc *desc);
void mcc_omnicalib_destroy(mcc_omnicalib *h);
int mcc_omnicalib_nparams(const mcc_omnicalib *h);

/* computeJacobian at params (P) for loop iteration iter: jte[P] = J^T E before the flag
 * reduction, G[P] = alpha_smooth2 (JTJ + epsilon)^-1 JTE with fixed entries 0 (fillFixed).
 * Either output may be NULL. */
int mcc_omnicalib_jacobian(mcc_omnicalib *h, const double *params, int iter, double *jte, double *G);

/* calibrate's loop from params_inout (P): crit_type MCC_CRIT_COUNT / EPS / COUNT_EPS. */
int mcc_omnicalib_optimize(mcc_omnicalib *h, int crit_type, int max_count, double eps, double *params_inout,
                           int *iters, double *last_change);

/* rms reprojection error at params (estimateUncertainties) */
int mcc_omnicalib_rms(mcc_omnicalib *h, const double *params, double *rms);

/* measurement: n_steps unconditional loop steps (no stop test; iterations 0..n_steps-1 of the
 * alpha / epsilon schedules) from params, graph-launched; ms_per_step = device time per step
 * (one kernel launch) from two HIP events on the handle's stream.  params are not modified. */
int mcc_omnicalib_time_steps(mcc_omnicalib *h, const double *params, int n_steps, double *ms_per_step);

/* initializeCalibration (host): om / t [3 * n_views] of the kept views in idx order, K[9]
 * (row-major), xi, idx[n_views] kept view indices, n_idx. */
int mcc_omnidir_initialize(int n_views, const int *view_off, const double *obj, const double *img, int width,
                           int height, double *om, double *t, double *K, double *xi, int *idx, int *n_idx);

/* cv::omnidir::calibrate: K[9], xi, D[4], om / t [3 * n_views] (kept views), idx, n_idx, rms,
 * iterations (may be NULL). */
int mcc_omnidir_calibrate(int n_views, const int *view_off, const double *obj, const double *img, int width,
                          int height, int flags, int crit_type, int max_count, double eps, int device, double *K,
                          double *xi, double *D, double *om, double *t, int *idx, int *n_idx, double *rms,
                          int *iters);

#ifdef __cplusplus
}
#endif
#endif
