// mcc_omnicalib_api.cpp -- host side of the omnidir intrinsic calibration C ABI
// (include/mcc_omnidir.h; cv::omnidir::calibrate, src/omnidir.cpp:1067-1211).
//
// mcc_omnicalib_* keep the per-view corners (CV_64F, as calibrate converts them, :1083-1094) in
// HBM as structure-of-arrays and run calibrate's loop on the device: one k_oc_step launch per
// iteration, graph-launched 8 at a time, the stop test on the device.  initializeCalibration
// (:551-748) is host code here as in the reference (a 6-column SVD and a 3-column least-squares
// fit per view, O(corners)).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mcc_omnidir.h"
#include "mcc_omnicalib_internal.h"

using mcc::OcState;

namespace {

int oc_fail(int code, const std::string& msg) { return mcc_internal_fail(code, msg.c_str()); }

#define OCCHK(expr)                                                                          \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) return oc_fail(MCC_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

template <typename T>
struct DBuf {
    T* p = nullptr;
    hipError_t alloc(size_t n) { return hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T)); }
    hipError_t upload(const T* h, size_t n) {
        hipError_t e = alloc(n);
        if (e == hipSuccess && n) e = hipMemcpy(p, h, n * sizeof(T), hipMemcpyHostToDevice);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
};

// flags2idx (src/omnidir.cpp:2031-2076) for the 10 intrinsics: 1 = free, 0 = fixed.  The cascade
// of >= tests is the reference's (CALIB_USE_GUESS is not handled there either).
void intrinsic_mask(int flags, double* m) {
    for (int i = 0; i < 10; ++i) m[i] = 1.0;
    int f = flags;
    if (f >= MCC_OMNI_CALIB_FIX_CENTER) { m[3] = m[4] = 0; f -= MCC_OMNI_CALIB_FIX_CENTER; }
    if (f >= MCC_OMNI_CALIB_FIX_GAMMA) { m[0] = m[1] = 0; f -= MCC_OMNI_CALIB_FIX_GAMMA; }
    if (f >= MCC_OMNI_CALIB_FIX_XI) { m[5] = 0; f -= MCC_OMNI_CALIB_FIX_XI; }
    if (f >= MCC_OMNI_CALIB_FIX_P2) { m[9] = 0; f -= MCC_OMNI_CALIB_FIX_P2; }
    if (f >= MCC_OMNI_CALIB_FIX_P1) { m[8] = 0; f -= MCC_OMNI_CALIB_FIX_P1; }
    if (f >= MCC_OMNI_CALIB_FIX_K2) { m[7] = 0; f -= MCC_OMNI_CALIB_FIX_K2; }
    if (f >= MCC_OMNI_CALIB_FIX_K1) { m[6] = 0; f -= MCC_OMNI_CALIB_FIX_K1; }
    if (f >= MCC_OMNI_CALIB_FIX_SKEW) m[2] = 0;
}

}  // namespace

struct mcc_omnicalib {
    int n = 0, P = 0, flags = 0, device = 0, max_np = 1, group_size = 1, n_groups = 1;
    long long corners = 0;
    std::vector<int> off;
    hipStream_t stream = nullptr;
    DBuf<double> ox, oy, oz, iu, iv, x, mask, Yv, zb, zu, yc, jte, G, contrib, gsum, view_sq;
    DBuf<int> view_off, cnt;
    DBuf<OcState> st;
    OcState* h_st = nullptr;
    static constexpr int kGraphSteps = 8;
    hipGraphExec_t gexec[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};

    mcc::OcArgs args() const {
        return mcc::OcArgs{st.p, view_off.p, ox.p, oy.p, oz.p, iu.p, iv.p, x.p, mask.p, Yv.p, zb.p, zu.p, yc.p,
                           jte.p, G.p, contrib.p, gsum.p, cnt.p, n, group_size, n_groups, max_np};
    }
};

namespace {

int oc_set_state(mcc_omnicalib* h, int iter, int crit, int max_count, double eps) {
    OCCHK(hipStreamSynchronize(h->stream));
    OcState s{};
    s.iter = iter;
    s.crit_type = crit;
    s.max_count = max_count;
    s.eps = eps;
    s.change = 1.0;
    *h->h_st = s;
    OCCHK(hipMemcpyAsync(h->st.p, h->h_st, sizeof(OcState), hipMemcpyHostToDevice, h->stream));
    OCCHK(hipStreamSynchronize(h->stream));
    return MCC_OK;
}

int oc_read_state(mcc_omnicalib* h) {
    OCCHK(hipMemcpyAsync(h->h_st, h->st.p, sizeof(OcState), hipMemcpyDeviceToHost, h->stream));
    OCCHK(hipStreamSynchronize(h->stream));
    if (h->h_st->error & 1) return oc_fail(MCC_ENOTPD, "omnidir calibrate: a view's 6x6 pose block J^T J is not positive definite");
    if (h->h_st->error & 2) return oc_fail(MCC_ENOTPD, "omnidir calibrate: the reduced intrinsic system is not positive definite");
    return MCC_OK;
}

int oc_upload_params(mcc_omnicalib* h, const double* params) {
    OCCHK(hipMemcpyAsync(h->x.p, params, sizeof(double) * h->P, hipMemcpyHostToDevice, h->stream));
    return MCC_OK;
}

int oc_build_graphs(mcc_omnicalib* h) {
    if (h->gexec[0]) return MCC_OK;
    const int counts[2] = {1, mcc_omnicalib::kGraphSteps};
    const mcc::OcArgs a = h->args();
    for (int g = 0; g < 2; ++g) {
        hipGraph_t graph;
        OCCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        hipError_t le = hipSuccess;
        for (int s = 0; s < counts[g] && le == hipSuccess; ++s) le = mcc_launch_oc_step(a, h->stream);
        hipError_t ee = hipStreamEndCapture(h->stream, &graph);
        if (le != hipSuccess) return oc_fail(MCC_EHIP, std::string("k_oc_step launch: ") + hipGetErrorString(le));
        if (ee != hipSuccess) return oc_fail(MCC_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ee));
        OCCHK(hipGraphInstantiate(&h->gexec[g], graph, nullptr, nullptr, 0));
        OCCHK(hipGraphDestroy(graph));
    }
    return MCC_OK;
}

int oc_launch_steps(mcc_omnicalib* h, int n) {
    int rc = oc_build_graphs(h);
    if (rc) return rc;
    while (n >= mcc_omnicalib::kGraphSteps) {
        OCCHK(hipGraphLaunch(h->gexec[1], h->stream));
        n -= mcc_omnicalib::kGraphSteps;
    }
    while (n-- > 0) OCCHK(hipGraphLaunch(h->gexec[0], h->stream));
    return MCC_OK;
}

// ---------------------------------------------------------------- initializeCalibration (host)

// One-sided (Hestenes) Jacobi SVD of A (m x k, row-major, overwritten by U * diag(sv)).
void svd_jacobi(std::vector<double>& A, int m, int k, double* V, double* sv) {
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) V[i * k + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double worst = 0;
        for (int p = 0; p < k - 1; ++p)
            for (int q = p + 1; q < k; ++q) {
                double app = 0, aqq = 0, apq = 0;
                for (int r = 0; r < m; ++r) {
                    const double xp = A[(size_t)r * k + p], xq = A[(size_t)r * k + q];
                    app += xp * xp;
                    aqq += xq * xq;
                    apq += xp * xq;
                }
                if (app == 0 || aqq == 0) continue;
                const double rel = std::fabs(apq) / std::sqrt(app * aqq);
                worst = std::max(worst, rel);
                if (rel < 1e-15) continue;
                const double zeta = (aqq - app) / (2 * apq);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
                const double c = 1 / std::sqrt(1 + t * t), s = c * t;
                for (int r = 0; r < m; ++r) {
                    double& xp = A[(size_t)r * k + p];
                    double& xq = A[(size_t)r * k + q];
                    const double a0 = xp, a1 = xq;
                    xp = c * a0 - s * a1;
                    xq = s * a0 + c * a1;
                }
                for (int r = 0; r < k; ++r) {
                    const double a0 = V[r * k + p], a1 = V[r * k + q];
                    V[r * k + p] = c * a0 - s * a1;
                    V[r * k + q] = s * a0 + c * a1;
                }
            }
        if (worst < 1e-15) break;
    }
    for (int j = 0; j < k; ++j) {
        double s = 0;
        for (int r = 0; r < m; ++r) s += A[(size_t)r * k + j] * A[(size_t)r * k + j];
        sv[j] = std::sqrt(s);
    }
}

// omnidir::projectPoints without distortion (D = 0) for xi and K = [g 0 u0; 0 g v0] (init only)
void project_nodist(int np, const double* obj, const double* om, const double* t, double g, double u0, double v0,
                    double xi, double* out) {
    const double th = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (th >= 2.220446049250313e-16) {
        const double c = std::cos(th), s = std::sin(th), c1 = 1 - c;
        const double x = om[0] / th, y = om[1] / th, z = om[2] / th;
        const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
        const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
        for (int k = 0; k < 9; ++k) R[k] = c * ((k % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[k] + s * rx[k];
    }
    for (int i = 0; i < np; ++i) {
        const double* X = obj + 3 * (size_t)i;
        double Xc[3];
        for (int a = 0; a < 3; ++a) Xc[a] = R[a * 3] * X[0] + R[a * 3 + 1] * X[1] + R[a * 3 + 2] * X[2] + t[a];
        const double nr = std::sqrt(Xc[0] * Xc[0] + Xc[1] * Xc[1] + Xc[2] * Xc[2]);
        const double zs = Xc[2] / nr + xi;
        out[2 * i] = g * (Xc[0] / nr / zs) + u0;
        out[2 * i + 1] = g * (Xc[1] / nr / zs) + v0;
    }
}

double mean_l2(int np, const double* img, const double* proj) {   // computeMeanReproErr (:1892-1934)
    double e = 0;
    for (int j = 0; j < np; ++j) {
        const double dx = img[2 * j] - proj[2 * j], dy = img[2 * j + 1] - proj[2 * j + 1];
        e += std::sqrt(dx * dx + dy * dy);
    }
    return e / np;
}

}  // namespace

extern "C" {

int mcc_omnicalib_create(mcc_omnicalib** out, const mcc_omnicalib_desc* d) {
    if (!out || !d) return oc_fail(MCC_EINVAL, "null argument");
    *out = nullptr;
    if (d->n_views < 1 || !d->view_off || !d->obj || !d->img)
        return oc_fail(MCC_EINVAL, "omnidir calibrate needs at least one view with points");
    const int n = d->n_views;
    int max_np = 1;
    for (int i = 0; i < n; ++i) {
        const int np = d->view_off[i + 1] - d->view_off[i];
        if (np < 3) return oc_fail(MCC_EINVAL, "every view needs at least 3 points");
        if (np > mcc::kOcMaxCorners)
            return oc_fail(MCC_EINVAL, "a view holds more than " + std::to_string(mcc::kOcMaxCorners) + " points");
        max_np = std::max(max_np, np);
    }
    if (d->view_off[0] != 0) return oc_fail(MCC_EINVAL, "view_off[0] must be 0");
    auto* h = new mcc_omnicalib();
    h->n = n;
    h->P = 6 * n + 10;
    h->flags = d->flags;
    h->device = d->device;
    h->max_np = max_np;
    h->off.assign(d->view_off, d->view_off + n + 1);
    h->corners = h->off[n];
    h->group_size = std::max(1, (int)std::ceil(std::sqrt((double)n)));
    h->n_groups = (n + h->group_size - 1) / h->group_size;
    auto bail = [&](int rc) {
        mcc_omnicalib_destroy(h);
        return rc;
    };
#define OCCHK_H(expr)                                                                        \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess) return bail(oc_fail(MCC_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e))); \
    } while (0)
    OCCHK_H(hipSetDevice(d->device));
    OCCHK_H(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    const size_t C = (size_t)h->corners;
    std::vector<double> soa[5];
    for (auto& s : soa) s.resize(C);
    for (size_t c = 0; c < C; ++c) {
        soa[0][c] = d->obj[3 * c];
        soa[1][c] = d->obj[3 * c + 1];
        soa[2][c] = d->obj[3 * c + 2];
        soa[3][c] = d->img[2 * c];
        soa[4][c] = d->img[2 * c + 1];
    }
    OCCHK_H(h->ox.upload(soa[0].data(), C));
    OCCHK_H(h->oy.upload(soa[1].data(), C));
    OCCHK_H(h->oz.upload(soa[2].data(), C));
    OCCHK_H(h->iu.upload(soa[3].data(), C));
    OCCHK_H(h->iv.upload(soa[4].data(), C));
    OCCHK_H(h->view_off.upload(h->off.data(), n + 1));
    double m[10];
    intrinsic_mask(d->flags, m);
    OCCHK_H(h->mask.upload(m, 10));
    OCCHK_H(h->x.alloc(h->P));
    OCCHK_H(h->Yv.alloc(60 * (size_t)n));
    OCCHK_H(h->zb.alloc(6 * (size_t)n));
    OCCHK_H(h->zu.alloc(6 * (size_t)n));
    OCCHK_H(h->yc.alloc(10));
    OCCHK_H(h->jte.alloc(h->P));
    OCCHK_H(h->G.alloc(h->P));
    OCCHK_H(h->contrib.alloc((size_t)n * mcc::kOcLc));
    OCCHK_H(h->gsum.alloc((size_t)h->n_groups * mcc::kOcLc));
    OCCHK_H(h->view_sq.alloc(n));
    OCCHK_H(h->cnt.alloc(h->n_groups + 1));
    OCCHK_H(hipMemset(h->cnt.p, 0, sizeof(int) * (h->n_groups + 1)));
    OCCHK_H(hipMemset(h->G.p, 0, sizeof(double) * h->P));
    OCCHK_H(hipMemset(h->jte.p, 0, sizeof(double) * h->P));
    OCCHK_H(h->st.alloc(1));
    OCCHK_H(hipHostMalloc((void**)&h->h_st, sizeof(OcState), hipHostMallocDefault));
    OCCHK_H(mcc_oc_set_attrs(max_np));
    OCCHK_H(hipEventCreate(&h->ev[0]));
    OCCHK_H(hipEventCreate(&h->ev[1]));
#undef OCCHK_H
    *out = h;
    return MCC_OK;
}

void mcc_omnicalib_destroy(mcc_omnicalib* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto& g : h->gexec)
        if (g) (void)hipGraphExecDestroy(g);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (DBuf<double>* b : {&h->ox, &h->oy, &h->oz, &h->iu, &h->iv, &h->x, &h->mask, &h->Yv, &h->zb, &h->zu, &h->yc,
                            &h->jte, &h->G, &h->contrib, &h->gsum, &h->view_sq})
        b->release();
    h->view_off.release();
    h->cnt.release();
    h->st.release();
    if (h->h_st) (void)hipHostFree(h->h_st);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int mcc_omnicalib_nparams(const mcc_omnicalib* h) { return h ? h->P : MCC_EINVAL; }

int mcc_omnicalib_jacobian(mcc_omnicalib* h, const double* params, int iter, double* jte, double* G) {
    if (!h || !params || iter < 0) return oc_fail(MCC_EINVAL, "bad argument");
    OCCHK(hipSetDevice(h->device));
    int rc = oc_set_state(h, iter, MCC_CRIT_COUNT, iter + 1, 0.0);
    if (rc) return rc;
    if ((rc = oc_upload_params(h, params))) return rc;
    // step 1 linearises and solves iteration `iter` (the intrinsic part of G), step 2 applies the
    // pending pose update (the pose part of G) and stops (iter + 1 >= max_count)
    // (step 2 linearises again at the updated point: JTE is read between the two)
    const mcc::OcArgs a = h->args();
    OCCHK(mcc_launch_oc_step(a, h->stream));
    if ((rc = oc_read_state(h))) return rc;
    if (jte) OCCHK(hipMemcpy(jte, h->jte.p, sizeof(double) * h->P, hipMemcpyDeviceToHost));
    OCCHK(mcc_launch_oc_step(a, h->stream));
    if ((rc = oc_read_state(h))) return rc;
    if (G) OCCHK(hipMemcpy(G, h->G.p, sizeof(double) * h->P, hipMemcpyDeviceToHost));
    return MCC_OK;
}

int mcc_omnicalib_optimize(mcc_omnicalib* h, int crit_type, int max_count, double eps, double* params_inout,
                           int* iters, double* last_change) {
    if (!h || !params_inout) return oc_fail(MCC_EINVAL, "null argument");
    if (crit_type < 1 || crit_type > 3) return oc_fail(MCC_EINVAL, "crit_type must be 1, 2 or 3");
    OCCHK(hipSetDevice(h->device));
    int rc = oc_set_state(h, 0, crit_type, max_count, eps);
    if (rc) return rc;
    if ((rc = oc_upload_params(h, params_inout))) return rc;
    const long long cap = crit_type == MCC_CRIT_EPS ? 1000000LL : (long long)max_count + 1;
    long long launched = 0;
    while (true) {
        if ((rc = oc_launch_steps(h, mcc_omnicalib::kGraphSteps))) return rc;
        launched += mcc_omnicalib::kGraphSteps;
        if ((rc = oc_read_state(h))) return rc;
        if (h->h_st->done) break;
        if (launched > cap + mcc_omnicalib::kGraphSteps) return oc_fail(MCC_EINVAL, "omnidir calibrate did not terminate");
    }
    if (iters) *iters = h->h_st->iter;
    if (last_change) *last_change = h->h_st->change;
    OCCHK(hipMemcpy(params_inout, h->x.p, sizeof(double) * h->P, hipMemcpyDeviceToHost));
    return MCC_OK;
}

int mcc_omnicalib_rms(mcc_omnicalib* h, const double* params, double* rms) {
    if (!h || !params || !rms) return oc_fail(MCC_EINVAL, "null argument");
    OCCHK(hipSetDevice(h->device));
    OCCHK(hipStreamSynchronize(h->stream));
    int rc = oc_upload_params(h, params);
    if (rc) return rc;
    const mcc::OcErrArgs a{h->view_off.p, h->ox.p, h->oy.p, h->oz.p, h->iu.p, h->iv.p, h->x.p, h->view_sq.p, h->n};
    OCCHK(mcc_launch_oc_err(a, h->stream));
    std::vector<double> sq(h->n);
    OCCHK(hipMemcpyAsync(sq.data(), h->view_sq.p, sizeof(double) * h->n, hipMemcpyDeviceToHost, h->stream));
    OCCHK(hipStreamSynchronize(h->stream));
    double s = 0;
    for (int v = 0; v < h->n; ++v) s += sq[v];   // view order
    *rms = std::sqrt(s / (double)h->corners);
    return MCC_OK;
}

int mcc_omnicalib_time_steps(mcc_omnicalib* h, const double* params, int n_steps, double* ms_per_step) {
    if (!h || !params || n_steps < 1 || !ms_per_step) return oc_fail(MCC_EINVAL, "bad argument");
    OCCHK(hipSetDevice(h->device));
    int rc = oc_set_state(h, 0, 0, 0, 0.0);
    if (rc) return rc;
    if ((rc = oc_upload_params(h, params))) return rc;
    if ((rc = oc_launch_steps(h, 2))) return rc;   // graph instantiation + first touch
    OCCHK(hipEventRecord(h->ev[0], h->stream));
    if ((rc = oc_launch_steps(h, n_steps))) return rc;
    OCCHK(hipEventRecord(h->ev[1], h->stream));
    OCCHK(hipEventSynchronize(h->ev[1]));
    if ((rc = oc_read_state(h))) return rc;
    float ms = 0.f;
    OCCHK(hipEventElapsedTime(&ms, h->ev[0], h->ev[1]));
    *ms_per_step = (double)ms / n_steps;
    return MCC_OK;
}

int mcc_omnidir_initialize(int n_img, const int* off, const double* obj, const double* img, int width, int height,
                           double* om_out, double* t_out, double* K, double* xi, int* idx, int* n_idx) {
    // initializeCalibration, src/omnidir.cpp:551-748 (Li et al., IROS 2013, section III)
    if (n_img < 1 || !off || !obj || !img || !om_out || !t_out || !K || !xi || !idx || !n_idx)
        return oc_fail(MCC_EINVAL, "bad argument");
    const double u0 = width / 2, v0 = height / 2;   // Size::width / 2: integer division
    std::vector<double> omA(3 * (size_t)n_img, 0.0), tA(3 * (size_t)n_img, 0.0), gammaAll(n_img, 0.0);
    std::vector<double> proj;
    for (int im = 0; im < n_img; ++im) {
        const int np = off[im + 1] - off[im];
        if (np < 3) return oc_fail(MCC_EINVAL, "every view needs at least 3 points");
        const double* ob = obj + 3 * (size_t)off[im];
        const double* ip = img + 2 * (size_t)off[im];
        proj.resize(2 * (size_t)np);
        // extrinsic part: the null vector of M = [-v x, -v y, u x, u y, -v, u] (V column 5 of the SVD)
        std::vector<double> M(6 * (size_t)np);
        for (int j = 0; j < np; ++j) {
            const double x = ob[3 * j], y = ob[3 * j + 1], u = ip[2 * j] - u0, v = ip[2 * j + 1] - v0;
            double* r = &M[6 * (size_t)j];
            r[0] = -v * x; r[1] = -v * y; r[2] = u * x; r[3] = u * y; r[4] = -v; r[5] = u;
        }
        double V[36], sv[6];
        svd_jacobi(M, np, 6, V, sv);
        const int jm = (int)(std::min_element(sv, sv + 6) - sv);
        double best = 1e5;
        for (int coef = 1; coef >= -1; coef -= 2) {
            const double r11 = V[0 * 6 + jm] * coef, r12 = V[1 * 6 + jm] * coef, r21 = V[2 * 6 + jm] * coef;
            const double r22 = V[3 * 6 + jm] * coef, t1 = V[4 * 6 + jm] * coef, t2 = V[5 * 6 + jm] * coef;
            // r31^2 solves z^2 + b z + c = 0 with c <= 0; the reference keeps its positive root
            const double q = r11 * r12 + r21 * r22;
            const double b = r11 * r11 + r21 * r21 - r12 * r12 - r22 * r22, c = -q * q;
            const double disc = std::sqrt(b * b - 4 * c);
            const double z = b > 0 ? (-2 * c) / (b + disc) : (-b + disc) / 2;
            const double r31s = std::sqrt(z);
            for (int coef2 = 1; coef2 >= -1; coef2 -= 2) {
                const double r31 = r31s * coef2, r32 = -q / r31;
                double r1[3] = {r11, r21, r31}, r2[3] = {r12, r22, r32}, t[3] = {t1, t2, 0};
                const double scale = 1 / std::sqrt(r1[0] * r1[0] + r1[1] * r1[1] + r1[2] * r1[2]);
                for (int k = 0; k < 3; ++k) { r1[k] *= scale; r2[k] *= scale; t[k] *= scale; }
                // intrinsic part (Scaramuzza's equations): A [gamma^2-ish, 1/gamma^2-ish, t3] = B
                std::vector<double> A(6 * (size_t)np), B(2 * (size_t)np);
                for (int j = 0; j < np; ++j) {
                    const double x = ob[3 * j], y = ob[3 * j + 1], u = ip[2 * j] - u0, v = ip[2 * j + 1] - v0;
                    const double rho2 = u * u + v * v;
                    const double a0 = (r1[1] * x + r2[1] * y + t[1]) / 2, a1 = (r1[0] * x + r2[0] * y + t[0]) / 2;
                    double* ra = &A[3 * (size_t)j];
                    double* rb = &A[3 * (size_t)(np + j)];
                    ra[0] = a0; ra[1] = -a0 * rho2; ra[2] = -v;
                    rb[0] = a1; rb[1] = -a1 * rho2; rb[2] = -u;
                    B[j] = v * (r1[2] * x + r2[2] * y);
                    B[np + j] = u * (r1[2] * x + r2[2] * y);
                }
                double maxA[3] = {0, 0, 0};
                for (int r = 0; r < 2 * np; ++r)
                    for (int cc = 0; cc < 3; ++cc) maxA[cc] = std::max(maxA[cc], std::fabs(A[3 * (size_t)r + cc]));
                for (int r = 0; r < 2 * np; ++r)
                    for (int cc = 0; cc < 3; ++cc) A[3 * (size_t)r + cc] /= maxA[cc];
                // A.inv(DECOMP_SVD) * B: minimum-norm least squares through the SVD of A
                double Va[9], sa[3];
                svd_jacobi(A, 2 * np, 3, Va, sa);
                const double smax = std::max(sa[0], std::max(sa[1], sa[2]));
                double res[3] = {0, 0, 0};
                for (int cc = 0; cc < 3; ++cc) {
                    if (!(sa[cc] > smax * 2.220446049250313e-16 * 2 * np)) continue;
                    double ub = 0;
                    for (int r = 0; r < 2 * np; ++r) ub += A[3 * (size_t)r + cc] * B[r];
                    ub /= sa[cc] * sa[cc];
                    for (int k = 0; k < 3; ++k) res[k] += Va[k * 3 + cc] * ub;
                }
                for (int k = 0; k < 3; ++k) res[k] *= 1 / maxA[k];
                const double gamma = std::sqrt(res[0] / res[1]);
                t[2] = res[2];
                const double r3[3] = {r1[1] * r2[2] - r1[2] * r2[1], r1[2] * r2[0] - r1[0] * r2[2],
                                      r1[0] * r2[1] - r1[1] * r2[0]};
                const double R[9] = {r1[0], r2[0], r3[0], r1[1], r2[1], r3[1], r1[2], r2[2], r3[2]};
                double om[3];
                mcc_internal_rodrigues_m2v(R, om);
                project_nodist(np, ob, om, t, gamma, u0, v0, 1.0, proj.data());
                const double err = mean_l2(np, ip, proj.data());
                if (err < best) {   // NaN never wins, as in the reference
                    best = err;
                    std::copy(om, om + 3, &omA[3 * (size_t)im]);
                    std::copy(t, t + 3, &tA[3 * (size_t)im]);
                    gammaAll[im] = gamma;
                }
            }
        }
    }
    std::vector<double> g = gammaAll;
    std::nth_element(g.begin(), g.begin() + n_img / 2, g.end());
    const double gammaFinal = g[n_img / 2];
    const double Kf[9] = {gammaFinal, 0, u0, 0, gammaFinal, v0, 0, 0, 1};
    std::copy(Kf, Kf + 9, K);
    int nk = 0;
    for (int i = 0; i < n_img; ++i) {   // keep views whose re-projection with the median gamma is < 100 px
        const int np = off[i + 1] - off[i];
        proj.resize(2 * (size_t)np);
        project_nodist(np, obj + 3 * (size_t)off[i], &omA[3 * (size_t)i], &tA[3 * (size_t)i], gammaFinal, u0, v0, 1.0,
                       proj.data());
        if (mean_l2(np, img + 2 * (size_t)off[i], proj.data()) < 100) {
            idx[nk] = i;
            std::copy(&omA[3 * (size_t)i], &omA[3 * (size_t)i] + 3, om_out + 3 * (size_t)nk);
            std::copy(&tA[3 * (size_t)i], &tA[3 * (size_t)i] + 3, t_out + 3 * (size_t)nk);
            ++nk;
        }
    }
    *n_idx = nk;
    *xi = 1;
    return MCC_OK;
}

int mcc_omnidir_calibrate(int n_img, const int* off, const double* obj, const double* img, int width, int height,
                          int flags, int crit_type, int max_count, double eps, int device, double* K, double* xi,
                          double* D, double* om, double* t, int* idx, int* n_idx, double* rms, int* iters) {
    // src/omnidir.cpp:1067-1211: initialise, keep the idx views, encodeParameters(K, om, t, D = 0,
    // xi), the loop, decodeParameters, estimateUncertainties' rms
    if (!K || !xi || !D || !om || !t || !idx || !n_idx || !rms) return oc_fail(MCC_EINVAL, "null argument");
    std::vector<double> om0(3 * (size_t)std::max(n_img, 1)), t0(om0.size());
    double K0[9], xi0 = 1;
    int nk = 0;
    int rc = mcc_omnidir_initialize(n_img, off, obj, img, width, height, om0.data(), t0.data(), K0, &xi0, idx, &nk);
    if (rc) return rc;
    if (nk < 1) return oc_fail(MCC_EINVAL, "omnidir calibrate: no view survived the initialisation");
    std::vector<int> o2(nk + 1, 0);
    for (int i = 0; i < nk; ++i) o2[i + 1] = o2[i] + off[idx[i] + 1] - off[idx[i]];
    std::vector<double> ob2(3 * (size_t)o2[nk]), im2(2 * (size_t)o2[nk]);
    for (int i = 0; i < nk; ++i) {
        const int np = o2[i + 1] - o2[i];
        std::copy(obj + 3 * (size_t)off[idx[i]], obj + 3 * (size_t)(off[idx[i]] + np), &ob2[3 * (size_t)o2[i]]);
        std::copy(img + 2 * (size_t)off[idx[i]], img + 2 * (size_t)(off[idx[i]] + np), &im2[2 * (size_t)o2[i]]);
    }
    const int P = 6 * nk + 10;
    std::vector<double> para(P);
    for (int i = 0; i < nk; ++i)
        for (int k = 0; k < 3; ++k) {
            para[6 * i + k] = om0[3 * i + k];
            para[6 * i + 3 + k] = t0[3 * i + k];
        }
    double* q = &para[6 * (size_t)nk];
    q[0] = K0[0]; q[1] = K0[4]; q[2] = K0[1]; q[3] = K0[2]; q[4] = K0[5]; q[5] = xi0;
    q[6] = q[7] = q[8] = q[9] = 0;
    mcc_omnicalib_desc d{nk, o2.data(), ob2.data(), im2.data(), flags, device};
    mcc_omnicalib* h = nullptr;
    if ((rc = mcc_omnicalib_create(&h, &d))) return rc;
    int it = 0;
    rc = mcc_omnicalib_optimize(h, crit_type, max_count, eps, para.data(), &it, nullptr);
    if (!rc) rc = mcc_omnicalib_rms(h, para.data(), rms);
    mcc_omnicalib_destroy(h);
    if (rc) return rc;
    const double Kd[9] = {q[0], q[2], q[3], 0, q[1], q[4], 0, 0, 1};
    std::copy(Kd, Kd + 9, K);
    *xi = q[5];
    std::copy(q + 6, q + 10, D);
    for (int i = 0; i < nk; ++i)
        for (int k = 0; k < 3; ++k) {
            om[3 * i + k] = para[6 * i + k];
            t[3 * i + k] = para[6 * i + 3 + k];
        }
    *n_idx = nk;
    if (iters) *iters = it;
    return MCC_OK;
}

}  // extern "C"
