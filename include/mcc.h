/*
 * mcc.h -- C ABI of the MI355X multi-camera bundle-adjustment hot path (libmcc.so).
 *
 * Drop-in boundary for MultiCameraCalibration::optimizeExtrinsics and its per-iteration
 * linearisation seam in the reference (yulong314/multi_camera_calibration):
 *
 *   mcc_create ........... replaces the problem state the reference keeps in _edgeList /
 *                          _vertexList / _objectPointsForEachCamera / _imagePointsForEachCamera /
 *                          _cameraMatrix / _distortCoeffs / _xi (include/opencv2/ccalib/
 *                          multicalib.hpp:207-214, mymulticalib.hpp:122-126, doubleSide.hpp:128-130)
 *                          once loadImages()+initialize() have built it.
 *   mcc_linearize_solve .. replaces the virtual computeJacobianExtrinsic(x, JTJ_inv, JTE, deltaX)
 *                          (multicalib.hpp:176 -> src/multicalib.cpp:593-703,
 *                          mymulticalib.hpp:164 -> src/mymulticalib.cpp:668-818,
 *                          doubleSide.hpp:133 -> src/doubleSide.cpp:434-581): one linearisation and
 *                          the normal-equation solve; JTJ_inv is never materialised.
 *   mcc_optimize ......... replaces the loop of optimizeExtrinsics (multicalib.hpp:155 ->
 *                          src/multicalib.cpp:462-507): undamped Gauss-Newton with the
 *                          0.95^(k+1) step factor and float32 state, driven on the device.
 *   mcc_project_error .... replaces the virtual computeProjectError(x) (multicalib.hpp:188 ->
 *                          src/multicalib.cpp:895-1006, src/mymulticalib.cpp:820-939,
 *                          src/doubleSide.cpp:640-769): per-edge float32 error sums in reference
 *                          order and the reference's meanReProjError.
 *   mcc_comm_* ........... multi-GPU: photo vertices sharded over ranks, one RCCL all-reduce of the
 *                          reduced camera system per Gauss-Newton step (no reference counterpart).
 *
 * Conventions: every function returns 0 on success or a negative MCC_E* code; the message is
 * in mcc_last_error() (thread-local).  Nothing throws across the ABI.  Inputs are deep-copied
 * to the device by mcc_create; output pointers are caller-allocated host memory.  One
 * mcc_problem per host thread; calls on one problem are serialised by the caller (the
 * reference is single-threaded and non-reentrant, src/multicalib.cpp:120).
 */
#ifndef MCC_H
#define MCC_H

#ifdef __cplusplus
extern "C" {
#endif

#define MCC_OK 0
#define MCC_EINVAL (-1)     /* bad argument / unsupported configuration          */
#define MCC_EHIP (-2)       /* HIP runtime error                                 */
#define MCC_ENOTPD (-3)     /* a normal-equation block is not positive definite  */
#define MCC_ECOMM (-4)      /* RCCL error                                        */
#define MCC_ENOMEM (-5)
#define MCC_ETIMEOUT (-6)   /* a device-side wait timed out (the m > 30 warm-solve helper)     */

/* Camera model / class semantics the linearisation follows. */
#define MCC_MODEL_PINHOLE 0     /* MyMultiCameraCalibration, cv::projectPoints (k1..k6,p1,p2,s1..s4) */
#define MCC_MODEL_OMNI 1        /* MultiCameraCalibration base class, cv::omnidir::projectPoints    */
#define MCC_MODEL_DOUBLESIDE 2  /* DoubleSideCalibration (pinhole), fixed cameras + ds transform    */

#define MCC_FRONT 0             /* MultiCameraCalibration::FRONT_PATTERN (multicalib.hpp:82) */
#define MCC_BACK 1              /* MultiCameraCalibration::BACK_PATTERN                      */

/* TermCriteria types as the reference tests them (src/multicalib.cpp:475-477). */
#define MCC_CRIT_COUNT 1
#define MCC_CRIT_EPS 2
#define MCC_CRIT_COUNT_EPS 3

typedef struct mcc_problem mcc_problem;

/* Problem description in the reference's layout.  Camera vertices 0..n_cams-1 (camera 0 is the
 * identity and is not optimised), photo vertices n_cams.. are given as photo indices
 * 0..n_photos-1.  Edges are in reference order (_edgeList).  Parameters follow buildParas
 * (src/multicalib.cpp:422-440): [cam1..cam(C-1), photo0..] x (rvec, tvec), or for DOUBLESIDE
 * (src/doubleSide.cpp:233-261): [ds, photo0..].  n_photos >= 1 and n_edges >= 1 (MCC_EINVAL
 * otherwise: the reference's mean error is 0/0 without observations).  A camera without
 * observations is accepted (a photo shard of a multi-GPU problem may lack one); if the whole
 * problem leaves one unobserved the solve reports MCC_ENOTPD.  At most 22 cameras
 * (global block m <= 128, the reduced solve's LDS-resident matrix) and 1024 corners per edge. */
typedef struct mcc_desc {
    int model;
    int n_cams, n_photos, n_edges;
    const int *edge_cam;     /* [E] camera vertex                                  */
    const int *edge_photo;   /* [E] photo index                                    */
    const int *edge_side;    /* [E] MCC_FRONT / MCC_BACK (NULL = all front)        */
    const int *edge_off;     /* [E] first corner of the edge in obj/img            */
    const int *edge_n;       /* [E] corners of the edge                            */
    const float *obj;        /* [3*corners] object points, float32                 */
    const float *img;        /* [2*corners] observed corners, float32              */
    int nd;                  /* distortion coefficients per camera: pinhole 4/5/8/12, omni 4 */
    const float *K;          /* [9*n_cams] camera matrices (row-major), float32     */
    const float *D;          /* [nd*n_cams] distortion, float32                    */
    const float *xi;         /* [n_cams] Mei xi (OMNI), else NULL                  */
    const double *ds_pose;   /* [16] PINHOLE: doubleSideTransform (CV_64F 4x4), used by BACK edges */
    const float *cam_pose;   /* [16*n_cams] DOUBLESIDE: fixed camera poses (CV_32F 4x4)            */
    int device;              /* HIP device ordinal                                 */
} mcc_desc;

int mcc_create(mcc_problem **out, const mcc_desc *desc);
void mcc_destroy(mcc_problem *p);
const char *mcc_last_error(void);

int mcc_nparams(const mcc_problem *p);            /* P of this (local) problem              */
int mcc_global_dim(const mcc_problem *p);         /* m: 6(C-1), or 6 for DOUBLESIDE         */

int mcc_set_params(mcc_problem *p, const float *x, int n);
int mcc_get_params(mcc_problem *p, float *x, int n);

/* One linearisation + normal-equation solve at the current parameters (no update).
 * delta[P], jte[P] (either may be NULL): the reference's deltaX and JTE. */
int mcc_linearize_solve(mcc_problem *p, double *delta, double *jte);

/* optimizeExtrinsics' loop (without the final computeProjectError).  x_inout[P] holds the
 * initial float32 parameters and receives the result.  iters / last_change may be NULL. */
int mcc_optimize(mcc_problem *p, int crit_type, int max_count, double eps, float *x_inout,
                 int *iters, double *last_change);

/* n unconditional Gauss-Newton iterations on the device-resident parameters, enqueued
 * asynchronously (bench / throughput path).  Use mcc_synchronize to wait.  The first call after
 * any other entry point switches the device state to free-running (one host round trip);
 * back-to-back calls only enqueue. */
int mcc_step(mcc_problem *p, int n);
int mcc_synchronize(mcc_problem *p);
/* Wait for the enqueued steps, then report a device-side failure they hit (MCC_ECOMM: a peer
 * exchange timed out; MCC_ENOTPD: a normal-equation block was not positive definite).  A
 * failing step sets the device loop's stop flag (the final solve of the step does, or the peer
 * exchange on a timeout), so the free-running steps after it are no-ops; a throughput caller
 * checks this once after its timed window (outside it: one small device-to-host copy).  The
 * error stays in the device state until an entry point rewrites it (mcc_set_params,
 * mcc_optimize, mcc_linearize_solve); after mcc_check has reported it, the next mcc_step also
 * rewrites it and continues from the current parameters. */
int mcc_check(mcc_problem *p);

/* computeProjectError(x): edge_err[E] (reference edge order, may be NULL), mean. */
int mcc_project_error(mcc_problem *p, const float *x, float *edge_err, double *mean);
/* the same with the quantities the reference prints (src/mymulticalib.cpp:898-937): each corner's
 * float32 L2 error corner_err[corners] (reference corner order: errorsVector, for the standard
 * deviation), totalError (the float32 sum of the per-edge sums in edge order) and totalNPoints
 * (2N per pinhole edge, N per omnidirectional one); every output may be NULL. */
int mcc_project_error_detail(mcc_problem *p, const float *x, float *edge_err, float *corner_err,
                             float *total_error, long long *total_points, double *mean);

/* ---- multi-GPU (RCCL over xGMI).  All ranks hold the same cameras and disjoint photo sets;
 * x of a rank is [global block, its photos].  The global block stays identical on all ranks. */
#define MCC_UNIQUE_ID_BYTES 128
int mcc_comm_unique_id(unsigned char *id /* [128] */);
int mcc_comm_init(mcc_problem *p, const unsigned char *id, int nranks, int rank);
/* greedy balance of photos over ranks by corner count (descending); rank_of_photo[n_photos] */
int mcc_partition_photos(int n_photos, int n_edges, const int *edge_photo, const int *edge_n,
                         int nranks, int *rank_of_photo);
/* collective helpers on the problem's communicator (device-side, blocking); over the peer
 * transport when it is on or when there is no RCCL communicator */
int mcc_comm_allreduce_max(mcc_problem *p, double *v);
int mcc_comm_barrier(mcc_problem *p);

/* ---- peer transport: the step's only exchange without RCCL.  The final arriving workgroup of
 * every rank writes its packed reduced camera system into every peer's inbox (device memory
 * mapped by IPC, over xGMI) in LL words (32 data bits + 32-bit epoch per 8-B store) and sums all
 * ranks' systems in rank order, so every rank solves identical bits in the same kernel; no
 * all-reduce launch and no k_solve launch per step.  Collective, in this order on every rank:
 *   mcc_peer_handle(p, h)            -> this rank's inbox handle; exchange them (file, MPI, ...)
 *   mcc_peer_init(p, all, n, rank)   -> maps the peers, runs a two-round handshake (all ranks
 *                                       agree: MCC_OK on every rank, or MCC_ECOMM on every rank)
 * after which the steps use it (mcc_peer_enable(p, 0) falls back to the RCCL communicator).
 * Works across devices and for several ranks on one device (no RCCL needed).  A rank that does
 * not deliver within MCC_PEER_TIMEOUT_MS (default 30000) fails the step with MCC_ECOMM. */
#define MCC_PEER_HANDLE_BYTES 64
#define MCC_PEER_MAX_RANKS 64
int mcc_peer_handle(mcc_problem *p, unsigned char *handle /* [64] */);
int mcc_peer_init(mcc_problem *p, const unsigned char *handles /* [64 * nranks], rank order */, int nranks,
                  int rank);
int mcc_peer_enable(mcc_problem *p, int on);

/* ---- diagnostics / measurement */
/* the warm solves since mcc_create: out[5] = {solves by refinement with the previous system's inverse,
 * refinement corrections in them, refinements that did not converge (the direct elimination ran
 * instead), direct solves for want of an inverse (an optimisation's first step(s), or the previous
 * system was not positive definite), steps that had to wait for the inverse's producer}.
 * m > 30 split step: k_solve refines with the inverse a resident helper kernel computes while the step
 * linearises; it waits for the helper as long as needed, up to MCC_WARM_TIMEOUT_MS (default 10000),
 * after which the step fails with MCC_ETIMEOUT.  m <= 30 (MCC_SMALL_WARM, default on; single GPU or the
 * peer transport): a spare workgroup of the step's linearisation launch inverts the previous system,
 * and the final solve refines with it (the fused step: with the previous launch's, two updates stale);
 * the last field counts fused steps whose final arriver waited for the spare to acknowledge its inputs,
 * with the same MCC_WARM_TIMEOUT_MS bound; the m <= 30 counters run only with MCC_SOLVE_STATS=1 at
 * mcc_create (their atomics cost ~0.5 us per fused step).  All zero when the problem takes the direct
 * elimination only
 * (m > 96, MCC_WARM=0, MCC_SMALL_WARM=0, RCCL on the fused step).  Which solve a step takes depends on
 * the systems only, never on timing. */
int mcc_solve_stats(mcc_problem *p, long long *out);
/* the last mcc_optimize as its caller saw it: host_ms[4] = {setup (parameters in, state reset), steps
 * (graph launches of kGraphSteps = 8 steps and the host's stop-test poll after each), finish (the
 * pending photo update flushed, parameters out), the whole call} in wall milliseconds; *device_ms =
 * HIP events from before the first step launch to after the last launched step; *launched = steps
 * launched (the ones after the stop test fired return at once); *iters = updates made; *polls = host
 * round trips to the stop test. */
int mcc_optimize_profile(mcc_problem *p, double *host_ms, double *device_ms, int *launched, int *iters,
                         int *polls);
/* per-corner float32 residuals fl32(obs - proj) at x, reference corner order [2*corners] */
int mcc_debug_residuals(mcc_problem *p, const float *x, float *res);
/* test only: the warm solves' injected delays and wait bound, as MCC_SPARE_DELAY_US / MCC_WARM_DELAY_US /
 * MCC_WARM_TIMEOUT_MS set them at mcc_create (a negative argument keeps the current value); the captured
 * step graphs are rebuilt.  Lets a test fail a step by a timeout and then run the same handle again. */
int mcc_debug_delays(mcc_problem *p, double spare_delay_us, double warm_delay_us, double warm_timeout_ms);
/* test / measurement: the m > 30 dense solve alone (k_solve's elimination), x = S^-1 r for a
 * packed SPD system [S upper triangle row-major, m(m+1)/2 | r, m] on `device`; with reps > 0 the
 * average device time of `reps` back-to-back launches (one workgroup each) in *us_per_solve; with
 * stamps (64 entries) the elimination's per-phase s_memtime stamps of the first launch. */
int mcc_debug_solve(int device, int m, const double *packed, double *x, int reps, double *us_per_solve,
                    long long *stamps);
/* average device time (ms) per launch of the linearisation kernel over the last
 * mcc_timing_begin/mcc_timing_end window (HIP events on the problem's stream), and launches.
 * Fused single-GPU problems (m <= 30 and at most two photos per CU: one kernel per step) time
 * the whole window of graph-launched steps with two events; split-step problems record an event
 * pair around the linearisation kernels (k_group, or k_prep + k_edge + k_photo) of every step and
 * one around the whole step, launched eagerly behind a ~5 ms device-side delay kernel, so that the
 * whole window is queued before the GPU reaches it and runs back to back (no host launch latency
 * between the kernels inside the event pairs). */
int mcc_timing_begin(mcc_problem *p);
int mcc_timing_end(mcc_problem *p, double *lin_ms_per_launch, double *step_ms, int *launches);
/* per-step time distribution: n_windows windows of `steps` free-running steps each, enqueued back to
 * back (graph-launched as mcc_step launches them) with a HIP event between windows; ms_per_window[i]
 * is window i's device time (a leading window, which would include the idle gap before the first
 * launch, is run and dropped).  *graph_launched = 1 when the steps ran as graphs. */
int mcc_timing_windows(mcc_problem *p, int n_windows, int steps, double *ms_per_window, int *graph_launched);
/* split-step problems: average device time (ms) per launch of the linearisation kernels alone
 * (k_group, or k_prep + k_edge + k_photo), `launches` of them in ONE captured graph bracketed by two
 * HIP events on the problem's stream -- the kernels back to back as the step graphs run them, with
 * no event between them (events recorded inside a captured graph carry no timestamps on HIP).  Each
 * launch re-applies the pending photo update and rewrites its operands (Y', z'), so the parameters and
 * those operands are restored after the window: the next step continues the trajectory it would have
 * taken without the probe (the Schur slots and photo sums the probe leaves are outputs the next step
 * rewrites before reading).  MCC_EINVAL for a fused-step problem. */
int mcc_timing_linearize(mcc_problem *p, int launches, double *ms_per_launch);
/* average time (ms) of the step's data-path exchange over the same window, and the exchanges:
 * RCCL all-reduces by HIP event pairs around each ncclAllReduce, the peer transport by the
 * device's own s_memrealtime ticks from the first send to the rank-ordered sums (in-kernel, so
 * it includes waiting for the slowest rank).  0 exchanges on a single rank. */
int mcc_timing_exchange(mcc_problem *p, double *ms_per_exchange, int *exchanges);
/* diagnostic build only (libmcc_diag.so, -DMCC_DIAG): first call arms per-phase s_memtime
 * stamps (k_linearize; split step: k_photo per group, k_prep, k_edge rows), later calls copy
 * [32 * n_photos] stamps (then k_schur's [8 * grid]) out
 * (others: MCC_EINVAL) */
int mcc_debug_stamps(mcc_problem *p, long long *out, int n);
/* static facts about the problem for roofline accounting */
int mcc_problem_stats(const mcc_problem *p, long long *corners, long long *edges,
                      long long *photos, long long *alg_bytes_per_step);
/* which step the problem runs: *split_step = 0 for the fused single-kernel step (m <= 30 and at
 * most two photo workgroups per CU, or MCC_FUSED=1), 2 for the split step with its linearisation
 * as one group kernel (k_group, k_schur, [k_solve]), 3 for that group kernel with the reduction and
 * the m <= 30 solve folded into its launch (one k_group launch per step; MCC_GFOLD=0 gives 2), 1 for
 * the split step's three-kernel form
 * (k_prep, k_edge, k_photo, k_schur, [k_solve]; MCC_GROUP=0); *photo_groups = the groups'
 * workgroups (split step).  The choice
 * depends on the device's CU count (fused iff m <= 30 and n_photos <= 2 x CUs: 512 on MI355X), and
 * the two paths sum the normal equations in different orders, so the last FP64 bits of a step (and
 * in rare cases a float32 ulp of the state) depend on the device model; MCC_FUSED pins it. */
int mcc_problem_path(const mcc_problem *p, int *split_step, int *photo_groups);

#ifdef __cplusplus
}
#endif
#endif
