// mcc_omnicalib_internal.h -- device state and kernel arguments of the omnidir intrinsic
// calibration (cv::omnidir::calibrate, src/omnidir.cpp:1067-1211), shared by mcc_omnicalib.hip
// and mcc_omnicalib_api.cpp.  Not part of the public ABI (include/mcc_omnidir.h).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mcc_omnidir.h"

namespace mcc {

// packed per-view contribution (and group / total sums) of one loop step
constexpr int kOcS = 0;      // [55] S_v = V_v - W_v^T U_v^-1 W_v, upper triangle of 10 x 10, row-major
constexpr int kOcRb = 55;    // [10] rc_v - W_v^T U_v^-1 rp_v            (reduced rhs of JTE)
constexpr int kOcWu = 65;    // [10] W_v^T U_v^-1 1                      (reduced rhs of the ones vector)
constexpr int kOcJc = 75;    // [10] rc_v = JIn^T E                      (the intrinsic JTE)
constexpr int kOcAb = 85;    //      1^T U_v^-1 rp_v
constexpr int kOcAu = 86;    //      1^T U_v^-1 1
constexpr int kOcNg = 87;    //      |G_pose|^2 of the update applied in phase 0
constexpr int kOcNx = 88;    //      |x_pose|^2 before it
constexpr int kOcLc = 89;

constexpr int kOcMaxCorners = 512;   // per view (LDS staging of the 2N x 16 Jacobian strip)

// Device-resident loop state (calibrate, src/omnidir.cpp:1126-1149).
struct OcState {
    int iter;          // completed updates k
    int done;          // stop test fired
    int crit_type;     // 0 = never stop (measurement), 1 COUNT, 2 EPS, 3 COUNT+EPS
    int max_count;
    double eps;
    double change;     // |G| / |x| of the last update
    double normG2_c, normX2_c;   // intrinsic parts of the last update
    double alpha2, coef;         // alpha_smooth2 and the Sherman-Morrison factor of the pending update
    int pending;       // a pose update waits for the next step's phase 0
    int error;         // bit 0: a view's 6 x 6 block is not PD, bit 1: the reduced 10 x 10 system
};

struct OcArgs {
    OcState* st;
    const int* view_off;                       // [n+1]
    const double* ox; const double* oy; const double* oz;   // [corners] SoA pattern points
    const double* iu; const double* iv;        // [corners] image points
    double* x;                                 // [6n + 10] parameters (encodeParameters layout)
    const double* mask;                        // [10] 1 = free intrinsic, 0 = fixed (flags2idx)
    double* Yv;                                // [60 n] Y_v = U_v^-1 W_v (next step's pose update)
    double* zb; double* zu;                    // [6n] U_v^-1 rp_v, U_v^-1 1
    double* yc;                                // [10] intrinsic part of the pending solution
    double* jte;                               // [6n + 10] J^T E of the last linearisation
    double* G;                                 // [6n + 10] G of the last update
    double* contrib;                           // [n * kOcLc]
    double* gsum;                              // [n_groups * kOcLc]
    int* cnt;                                  // [n_groups + 1] tickets, zero between launches
    int n, group_size, n_groups, max_np;
};

struct OcErrArgs {
    const int* view_off;
    const double* ox; const double* oy; const double* oz;
    const double* iu; const double* iv;
    const double* x;
    double* view_sq;                           // [n] sum of squared errors per view
    int n;
};

}  // namespace mcc

size_t mcc_oc_shmem(int max_np);
hipError_t mcc_oc_set_attrs(int max_np);
hipError_t mcc_launch_oc_step(const mcc::OcArgs& a, hipStream_t s);
hipError_t mcc_launch_oc_err(const mcc::OcErrArgs& a, hipStream_t s);
extern "C" __attribute__((visibility("hidden"))) int mcc_internal_fail(int code, const char* msg);
// cvRodrigues2 matrix -> vector with the orthonormalisation of its SVD (host, mcc_api.cpp)
extern "C" __attribute__((visibility("hidden"))) void mcc_internal_rodrigues_m2v(const double* R, double* r);
