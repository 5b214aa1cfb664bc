// mcc_api.cpp -- host side of libmcc.so: the extern "C" ABI of include/mcc.h.
//
// mcc_create turns the reference's problem (edge list + per-edge corner Mats + intrinsics, as
// MyMultiCameraCalibration::loadImages/initialize leave them, src/mymulticalib.cpp:348-405,
// 615-667) into a photo-major, structure-of-arrays layout in HBM, precomputes the Schur pair
// lists, and drives the Gauss-Newton loop of optimizeExtrinsics (src/multicalib.cpp:462-514)
// on one HIP stream, captured as hipGraphs.  Multi-GPU: one process per GPU, photo vertices
// sharded, one RCCL all-reduce of the packed reduced camera system per step.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/mcc.h"
#include "mcc_internal.h"

using mcc::State;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return fail(MCC_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
    } while (0)

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t alloc(size_t count) {
        n = count;
        return hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T));
    }
    hipError_t upload(const T* h, size_t count) {
        hipError_t e = alloc(count);
        if (e != hipSuccess) return e;
        if (count) e = hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
};

// Idle non-blocking streams per device, kept for the next problem: hipStreamDestroy costs ~2 ms
// (most of an mcc_destroy) and creating one more than that.  A stream is returned only after it
// has drained and its graphs and events are gone.
// high: the warm solve's helper stream, at the highest stream priority, so that it never shares a
// hardware queue with a step stream (streams are multiplexed onto a few queues per priority; a
// resident helper kernel in a step stream's queue would hold that queue's later kernels back)
struct StreamPool {
    std::mutex mu;
    std::vector<std::pair<int, hipStream_t>> idle;   // (device * 2 + high, stream)
    hipError_t take(int device, hipStream_t* s, bool high = false) {
        const int key = device * 2 + (high ? 1 : 0);
        {
            std::lock_guard<std::mutex> lk(mu);
            for (size_t i = 0; i < idle.size(); ++i)
                if (idle[i].first == key) {
                    *s = idle[i].second;
                    idle.erase(idle.begin() + (long)i);
                    return hipSuccess;
                }
        }
        if (!high) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
        int least = 0, greatest = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e != hipSuccess) return e;
        return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
    }
    void give(int device, hipStream_t s, bool high = false) {
        std::lock_guard<std::mutex> lk(mu);
        idle.emplace_back(device * 2 + (high ? 1 : 0), s);
    }
};
StreamPool& stream_pool() {
    static StreamPool* pool = new StreamPool();   // never destroyed: streams outlive static teardown
    return *pool;
}

// Host restatement of cvRodrigues2 matrix -> vector (with the polar re-orthonormalisation)
// used once per problem for fixed transforms (doubleSideTransform2vec,
// src/mymulticalib.cpp:105-117; cameraPose2vec, src/doubleSide.cpp:262-275).
void host_rodrigues_m2v(const double* Rin, double* r) {
    double R[9];
    std::memcpy(R, Rin, sizeof(R));
    for (int it = 0; it < 40; ++it) {
        double cof[9] = {R[4] * R[8] - R[5] * R[7], -(R[3] * R[8] - R[5] * R[6]), R[3] * R[7] - R[4] * R[6],
                         -(R[1] * R[8] - R[2] * R[7]), R[0] * R[8] - R[2] * R[6], -(R[0] * R[7] - R[1] * R[6]),
                         R[1] * R[5] - R[2] * R[4], -(R[0] * R[5] - R[2] * R[3]), R[0] * R[4] - R[1] * R[3]};
        double d = R[0] * cof[0] + R[1] * cof[1] + R[2] * cof[2], delta = 0;
        if (!(std::fabs(d) > 1e-300)) break;
        for (int k = 0; k < 9; ++k) {
            double v = 0.5 * (R[k] + cof[k] / d);
            delta = std::max(delta, std::fabs(v - R[k]));
            R[k] = v;
        }
        if (delta < 1e-15) break;
    }
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t;
            t = (R[0] + 1) * 0.5; rx = std::sqrt(std::max(t, 0.));
            t = (R[4] + 1) * 0.5; ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5; rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta; ry *= theta; rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s) * theta;
        rx *= vth; ry *= vth; rz *= vth;
    }
    r[0] = rx; r[1] = ry; r[2] = rz;
}

// computeTiltProjectionMatrix (OpenCV calib3d, distortion_model.hpp) for the tilted-sensor model of
// cv::projectPoints with 14 coefficients, which src/mymulticalib.cpp:566 reaches with whatever
// Distortion the camera XML holds (:118-132): matTilt = matProjZ * (matRotY * matRotX), row-major,
// Matx products summed left to right from 0
void tilt_matrix(double tx, double ty, double M[9]) {
    const double cx = std::cos(tx), sx = std::sin(tx), cy = std::cos(ty), sy = std::sin(ty);
    const double rx[9] = {1, 0, 0, 0, cx, sx, 0, -sx, cx};
    const double ry[9] = {cy, 0, -sy, 0, 1, 0, sy, 0, cy};
    double rxy[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += ry[3 * i + k] * rx[3 * k + j];
            rxy[3 * i + j] = s;
        }
    const double pz[9] = {rxy[8], 0, -rxy[2], 0, rxy[8], -rxy[5], 0, 0, 1};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += pz[3 * i + k] * rxy[3 * k + j];
            M[3 * i + j] = s;
        }
}

}  // namespace

struct mcc_problem {
    int model = 0, C = 0, V = 0, E = 0, nd = 0, m = 0, P = 0, device = 0;
    long long corners = 0;
    bool rational = false;
    int prism = 0;   // 1: thin prism s1..s4, 2: + the tilted sensor (nd = 14, tau != 0)
    int has_back = 0;
    int max_epp = 1, nblk = 0, n_items = 0, n_pairs = 0, n_norm_chunks = 0;
    size_t n_pair_doubles = 0;   // Schur pair-product slots (36 or 48 doubles each)
    // split step's k_photo groups (consecutive photos) and their pair / contribution lists
    int n_pgroups = 0, max_gpairs = 0, max_gcon = 0, max_gedges = 0;
    size_t photo_shmem = 0;
    // split step as ONE fused kernel per group (k_group: photo update, edge prologues, sweep, chain,
    // photo Schur work) instead of k_prep -> k_edge -> k_photo; MCC_GROUP=0 selects the three
    int use_group = 1;
    size_t group_shmem = 0;
    int group_lanes = 32;   // k_group's lanes per edge (32: 512-thread workgroups; 16: 256)
    // fused single-kernel step (m <= kFusedMaxM): photo contributions + two-level reduction
    static constexpr int kFusedMaxM = 30;
    int fused = 0, group_size = 1, n_groups = 1;
    // m > 30 (or MCC_FUSED=0): the split step k_prep -> k_edge -> k_photo -> k_schur -> k_solve
    int max_cpp = 1;   // most corners of one photo
    hipStream_t stream = nullptr;

    // host-side maps
    std::vector<int> dev2ref_edge;      // device edge -> reference edge
    std::vector<long long> dev2ref_corner;
    std::vector<int> edge_n_dev;

    // device buffers
    DevBuf<float> obj_x, obj_y, obj_z, img_u, img_v, x, xerr, K, D, xi, cam_rt, cam_pose, resid, edge_sum, corner_err;
    DevBuf<long long> stamps;
    DevBuf<double> ds_rt, Y, pairprod, zp, gp_tot, item_out, packed, dg, delta, photo_norm, alpha, contrib, gsum, W;
    DevBuf<double> erec, echain, eh;   // split step (m > 30): per-edge records
    DevBuf<double> tilt;               // [C][9] matTilt (prism == 2)
    DevBuf<double> ssinv;              // m <= 30 warm solve: the previous system's inverse [m x m]
    DevBuf<int> ssinv_ok;
    DevBuf<int> photo_ptr, photo_corner, edge_gblock, block_items, edge_photo, counter, cnt, cnt_blk;
    DevBuf<int> pgrp_ptr, pgrp_edge, gpair_ptr, gcon_ptr;
    DevBuf<int> prep_ptr, prep_edge;   // k_prep4's groups (three-kernel split step)
    // MCC_POISON_HANDOFF=1 (test): every buffer handed between workgroups inside one launch or
    // between the step's kernels is filled with NaN (all-ones bytes) before each step, so that a
    // read of a word its producer has not yet stored this step shows up in the result
    bool poison = false;
    int poison_level = 0;
    bool peer_push = true;   // m > 30 with the peer transport: k_peer_push sends from many workgroups
    int schur_one_level = 0; // k_schur's single hand-off level (m <= 30; MCC_SCHUR_ONE_LEVEL=0 restores two)
    int n_prep = 0, prep_lanes = 1;   // MCC_PREP_LANES=4: k_prep4 (measured slower at configs 3 and 5)
    // warm solve (m > 30 split step, MCC_WARM=0 turns it off): a resident helper kernel on a side
    // stream (one per batch of update steps) inverts each step's reduced system while the next step
    // linearises; the next k_solve refines with it (WarmCtx, mcc_internal.h)
    bool warm = false;
    hipStream_t side = nullptr;      // the helper's stream
    double* sinv = nullptr;          // [M x M] the helper's S^-1 (ordinary memory)
    double* prev2 = nullptr;         // uncached: [2][prev_stride] k_schur's copies of [S | r] (iteration parity)
    int prev_stride = 0;
    unsigned* wsync = nullptr;       // uncached: [8] epochs, stop, the helper's PD flag; its refined epoch, status, corrections
    double* xsol = nullptr;          // uncached: [128] the helper's solution (helper_refine)
    bool helper_refine = false;      // single GPU, m > 30: the helper refines too (MCC_HELPER_REFINE)
    // k_schur publishes the system at its start and the helper polls prev2's words as the blocks land
    // (config3, three-kernel step: 108.4-109.1 -> 107.4-107.6 us per step), else at its end and the helper
    // stages in one batch (k_group's step: config3's 8-rank shard, whose step the helper's cycle bounds,
    // was 0.9 us slower polled); MCC_HELPER_POLL=0/1 forces either
    int helper_early = 0;
    int inv_la = 0;                  // the helper's look-ahead inversion (WarmCtx::inv_la): the k_group path
    DevBuf<long long> warm_stats;    // [5] (mcc_solve_stats)
    int warm_poison = 0;             // MCC_WARM_POISON=1 (test): the helper publishes NaN inverses
    // k_solve's bound on the wait for the helper (MCC_WARM_TIMEOUT_MS, default 10 s; a step that hits
    // it fails with MCC_ETIMEOUT), the helper's idle exit (the wait bound plus the peer timeout: a
    // k_solve may sit in a peer exchange before it publishes), the test delay (MCC_WARM_DELAY_US)
    long long warm_wait_ticks = 1000000000LL, warm_idle_ticks = 4000000000LL, warm_delay_ticks = 0;
    long long spare_delay_ticks = 0;  // MCC_SPARE_DELAY_US (test): the fused step's spare starts this late
    bool small_stats = false;         // MCC_SOLVE_STATS=1: count the m <= 30 warm solves (SolveCtx::sstats)
    // k_group's step with k_schur's reduction and the solve folded into the same launch (LinArgs::fold;
    // MCC_GFOLD=0 keeps k_group -> k_schur): fnorm [4V] and fiv [m^2 + 1] hand-off words, kFoldEmpty
    // between launches like the slots and the item partials
    bool gfold = false;
    int fold_direct = 0;   // the final workgroup sums where the words land (LinArgs::fold_direct)
    int fold_dyn = 0;      // the groups take the reduction's tasks as they finish (LinArgs::fold_dyn)
    int fold_first = 0;    // MCC_FOLD_CONSUMERS_FIRST=1 (test): LinArgs::fold_first
    DevBuf<int> fold_ticket;
    int max_item_slots = 0;
    DevBuf<double> fnorm, fiv;
    int fault_photo = -1;            // MCC_FAULT_PHOTO (test): LinArgs::fault_photo
    DevBuf<unsigned char> edge_lphoto;
    DevBuf<unsigned> gcon;
    DevBuf<int4> edge_info, items, gpairs;
    DevBuf<State> state;
    State* h_state = nullptr;   // pinned staging
    float* h_x = nullptr;       // [P] pinned staging of mcc_optimize's parameters (allocated on first use)
    int packed_len = 0, ntri = 0;

    // graphs: gexec[k] = 2^k update steps (k < kGraphSizes), built on first use; a run of n steps
    // is launched as the binary decomposition of n (20 steps: two launches, 16 + 4).
    // mcc_optimize polls the device stop test every kGraphSteps steps.
    static constexpr int kGraphSteps = 8;
    static constexpr int kGraphSizes = 7;   // up to 64 steps per launch
    hipGraphExec_t gexec[kGraphSizes] = {};
    // mcc_timing_linearize: a graph of lin_graph_n launches of the split step's linearisation kernels
    hipGraphExec_t lin_graph = nullptr;
    int lin_graph_n = 0;
    // x, and the pending photo update's operands Y' and z', across that window: each launch applies the
    // pending update again and rewrites Y' and z' at the drifted parameters
    DevBuf<float> xsave;
    DevBuf<double> ysave, zpsave;
    int graph_sizes = kGraphSizes;   // MCC_GRAPH_SIZES (A/B of the launch granularity)
    bool use_graph = true;
    // the device State is in free-running mode (crit_type 0) since the last mcc_step: later
    // mcc_step calls enqueue without a host round trip (set_state clears it)
    bool stepping = false;

    // RCCL
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    // peer transport (mcc_peer_*): LL inbox in uncached device memory, peers' inboxes via IPC
    static constexpr int kPeerMaxRanks = MCC_PEER_MAX_RANKS;
    unsigned long long* inbox = nullptr;
    std::vector<void*> peer_mapped;          // IPC mappings to close
    unsigned long long** peers_dev = nullptr;
    double* peer_scratch = nullptr;          // [4] handshake / max
    int peer_n = 0;                          // ranks of an initialised transport
    bool peer_on = false;
    long long peer_timeout = 0;              // s_memrealtime ticks

    // timing window
    bool timing = false;
    std::vector<hipEvent_t> ev_marks;        // mcc_timing_windows
    std::vector<hipEvent_t> ev_lin, ev_step;
    int ev_used = 0;
    // fused single-kernel step: the window is timed by two events around graph-launched steps
    bool timing_window = false;
    hipEvent_t ev_win[2] = {nullptr, nullptr};
    long long win_steps = 0;
    // exchange time over the window: RCCL all-reduces by event pairs (eager window), the peer
    // exchange by the device's own tick sum (State::xchg_ticks, in-kernel) against its value and
    // the epoch at mcc_timing_begin
    std::vector<hipEvent_t> ev_x;
    int ev_x_used = 0;
    long long xchg_ticks0 = 0;
    unsigned xchg_epoch0 = 0;
    // the last mcc_optimize, as its caller sees it (mcc_optimize_profile): host phases, the device time
    // from the first step launch to the end of the last, the steps launched, the host's stop-test polls
    hipEvent_t ev_opt[2] = {nullptr, nullptr};
    double opt_host_ms[4] = {0, 0, 0, 0};   // setup (parameters in, state), steps (launch + stop polls), finish, call
    double opt_dev_ms = 0.0;
    int opt_launched = 0, opt_iters = 0, opt_polls = 0;

};

namespace {

mcc::SolveCtx solve_ctx(mcc_problem* p, int do_update) {
    mcc::SolveCtx c{p->state.p, p->alpha.p, (int)p->alpha.n, p->x.p, p->dg.p, p->delta.p, p->m, do_update};
    c.sstats = p->ssinv.p && p->small_stats ? p->warm_stats.p : nullptr;   // the m <= 30 warm solve's statistics
    return c;
}

mcc::WarmCtx warm_ctx(mcc_problem* p) {
    const int copy_prev = (p->comm || p->peer_on) ? 1 : 0;   // sharded: k_solve copies the summed system
    return mcc::WarmCtx{p->sinv, reinterpret_cast<int*>(p->wsync + 3), p->prev2, p->prev_stride, copy_prev, p->wsync, p->warm_stats.p,
                        p->warm_poison, p->warm_wait_ticks, p->warm_idle_ticks, p->warm_delay_ticks,
                        p->helper_refine && !copy_prev ? 1 : 0, p->xsol, p->helper_early,
                        p->stamps.p ? p->stamps.p + p->stamps.n - 64 : nullptr, p->inv_la};
}

mcc::PeerCtx peer_ctx(mcc_problem* p, bool on) {
    mcc::PeerCtx pc{};
    if (!on) return pc;
    pc.inbox = p->inbox;
    pc.peers = p->peers_dev;
    pc.nranks = p->peer_n;
    pc.rank = p->rank;
    pc.Lc = p->packed_len;
    pc.timeout = p->peer_timeout;
    return pc;
}

// every captured graph of the problem (they hold kernel arguments: buffers, transport, stamps)
void drop_graphs(mcc_problem* p) {
    for (auto& g : p->gexec)
        if (g) { (void)hipGraphExecDestroy(g); g = nullptr; }
    if (p->lin_graph) { (void)hipGraphExecDestroy(p->lin_graph); p->lin_graph = nullptr; }
}

// lin_only (mcc_timing_linearize): the split step's linearisation kernels alone
int enqueue_step(mcc_problem* p, int do_update, float* resid_dev, bool lin_only = false) {
    using namespace mcc;
    const bool tim = p->timing && p->ev_used + 2 <= (int)p->ev_lin.size();
    // the m <= 30 warm solve (a spare workgroup of k_group / k_linearize inverts the previous step's
    // system; k_schur's or the next k_linearize's final arriver refines with it): single GPU or the
    // peer transport (with RCCL, k_solve solves)
    const bool swarm = p->ssinv.p && (p->peer_on || !p->comm);
    if (p->poison) {
        // (with the warm solve the packed system carries the previous step's system into the next
        // step, like dg: it is an input of the step, not a hand-off inside it, and stays unpoisoned;
        // on the fused step so does the inverse, which the next launch reads)
        for (auto* b : {&p->contrib, &p->gsum, &p->item_out, &p->pairprod, &p->packed, &p->ssinv})
            if (b->p && b->n && !(swarm && b == &p->packed) && !(p->fused && b == &p->ssinv))
                HIPCHK(hipMemsetAsync(b->p, 0xFF, sizeof(double) * b->n, p->stream));
        if (swarm && !p->fused) HIPCHK(hipMemsetAsync(p->ssinv_ok.p, 0xFF, 2 * sizeof(int), p->stream));
        for (auto* b : {&p->erec, &p->echain, &p->eh})
            if (b->p && b->n) HIPCHK(hipMemsetAsync(b->p, 0xFF, sizeof(double) * b->n, p->stream));
        // 2: the negative control -- dg carries the previous solve into this step's photo update,
        // so poisoning it must reach the parameters (the test checks that it does)
        if (p->poison_level > 1 && p->dg.p) HIPCHK(hipMemsetAsync(p->dg.p, 0xFF, sizeof(double) * p->dg.n, p->stream));
    }
    if (tim) HIPCHK(hipEventRecord(p->ev_step[p->ev_used], p->stream));
    if (tim) HIPCHK(hipEventRecord(p->ev_lin[p->ev_used], p->stream));
    LinArgs la{};
    la.state = p->state.p;
    la.photo_ptr = p->photo_ptr.p;
    la.photo_corner = p->photo_corner.p;
    la.max_cpp = p->max_cpp;
    la.edge_info = p->edge_info.p;
    la.obj_x = p->obj_x.p; la.obj_y = p->obj_y.p; la.obj_z = p->obj_z.p;
    la.img_u = p->img_u.p; la.img_v = p->img_v.p;
    la.x = p->x.p;
    la.K = p->K.p; la.D = p->D.p; la.xi = p->xi.p; la.tilt = p->tilt.p;
    la.cam_rt = p->cam_rt.p; la.ds_rt = p->ds_rt.p;
    la.nd = p->nd; la.global_dim = p->m;
    la.n_cams = p->C; la.has_back = p->has_back;
    la.Y = p->Y.p; la.zp = p->zp.p;
    la.pgrp_ptr = p->pgrp_ptr.p; la.pgrp_edge = p->pgrp_edge.p; la.edge_lphoto = p->edge_lphoto.p; la.gpair_ptr = p->gpair_ptr.p; la.gpairs = p->gpairs.p;
    la.gcon_ptr = p->gcon_ptr.p; la.gcon = p->gcon.p; la.pairprod = p->pairprod.p;
    la.prep_ptr = p->prep_ptr.p; la.prep_edge = p->prep_edge.p; la.n_prep = p->n_prep; la.prep_lanes = p->prep_lanes;
    la.n_pgroups = p->n_pgroups; la.max_gpairs = p->max_gpairs; la.max_gcon = p->max_gcon; la.max_gedges = p->max_gedges;
    la.gp_tot = p->gp_tot.p;
    la.resid = resid_dev;
    la.gblock = p->edge_gblock.p;
    la.dg = p->dg.p;
    la.photo_norm = p->photo_norm.p;
    la.stamps = p->stamps.p;
    la.fault_photo = p->fault_photo;
    // (the fused step: update launches only -- the spare's acknowledgement is the launch's iteration + 1,
    // distinct for the update launches of one optimisation, and a linearisation-only launch keeps the
    // iteration; it solves by the direct elimination)
    const bool lwarm = swarm && (do_update || !p->fused);
    la.ssinv = lwarm ? p->ssinv.p : nullptr;
    la.ssinv_ok = lwarm ? p->ssinv_ok.p : nullptr;
    la.spare_wait = p->warm_wait_ticks;
    la.spare_delay = p->spare_delay_ticks;
    // any RCCL communicator (also 1 rank: the GPU tests exercise this path on one device) takes the
    // split path: the packed system is summed by RCCL and solved by k_solve.  The peer transport
    // keeps one kernel per step: the final arriver exchanges with the peers and solves.
    const bool peer = p->peer_on;
    const bool rccl = p->comm != nullptr && !peer;
    la.fused = p->fused;
    la.group_size = p->group_size; la.n_groups = p->n_groups;
    la.rank = p->rank; la.fuse_solve = rccl ? 0 : 1;
    la.peer = peer_ctx(p, peer && p->fused);
    la.contrib = p->contrib.p; la.gsum = p->gsum.p; la.cnt = p->cnt.p; la.packed = p->packed.p; la.W = p->W.p;
    la.solve = solve_ctx(p, do_update);
    la.solve.stamps = nullptr;
    la.n_edges = p->E; la.n_photos = p->V;
    la.erec = p->erec.p; la.echain = p->echain.p; la.eh = p->eh.p;
    SchurArgs sa{};
    // m > 30: the register-tiled elimination runs in its own kernel (k_solve); with RCCL the
    // all-reduce sits between the reduction and k_solve; with the peer transport and m <= 30, the
    // reduction's final workgroup exchanges and solves (no k_peer_push / k_solve launches)
    const bool split = rccl || p->m > 30;
    if (!p->fused) {
        sa.state = p->state.p;
        sa.items = p->items.p;
        sa.pairprod = p->pairprod.p;
        sa.item_out = p->item_out.p;
        sa.n_items = p->n_items;
        sa.photo_norm = p->photo_norm.p; sa.n_photos = p->V;
        sa.counter = p->counter.p;
        sa.cnt_blk = p->cnt_blk.p;
        sa.nblk = p->nblk;
        sa.block_items = p->block_items.p;
        sa.packed = p->packed.p;
        sa.m = p->m; sa.rank = p->rank; sa.fuse_solve = split ? 0 : 1;
        sa.one_level = p->schur_one_level;
        sa.prev2 = p->warm && do_update && !p->comm && !p->peer_on ? p->prev2 : nullptr;   // single GPU
        sa.prev_stride = p->prev_stride;
        sa.wpub = sa.prev2 && p->helper_refine ? p->wsync : nullptr;   // (single GPU: prev2 set)
        sa.wpub_early = p->helper_early;
        sa.ssinv = swarm ? p->ssinv.p : nullptr;
        sa.ssinv_ok = swarm ? p->ssinv_ok.p : nullptr;
        sa.peer = peer_ctx(p, peer && !split);
        sa.solve = solve_ctx(p, do_update);
        sa.stamps = p->stamps.p ? p->stamps.p + mcc::kStampStride * (size_t)std::max(p->V, 1) : nullptr;
    }
    // k_group's step as one launch (LinArgs::fold): the reduction's workgroups follow the groups; the
    // timing probe's linearisation-only launches run k_group alone and empty the slots after it
    const bool fold = p->gfold && !lin_only;
    if (fold) {
        la.fold = 1;
        la.fold_parts = p->n_items + p->n_norm_chunks;
        la.fold_direct = p->fold_direct;
        la.fold_dyn = p->fold_dyn;
        la.fold_ticket = p->fold_ticket.p;
        la.fold_first = p->fold_first;
        la.fsa = sa;
        la.fsa.ssinv = la.ssinv ? p->fiv.p : nullptr;   // this launch's spare -> the final workgroup
        la.fsa.ssinv_ok = nullptr;
        la.fnorm = p->fnorm.p;
        la.fiv = p->fiv.p;
    }
    if (p->V > 0) {
        if (!p->fused && p->use_group)
            HIPCHK(mcc_launch_group(la, p->model, p->rational, p->prism, p->group_lanes, p->group_shmem, p->stream));
        else if (!p->fused)
            HIPCHK(mcc_launch_split(la, p->model, p->rational, p->prism, p->photo_shmem, p->stream));
        else
            HIPCHK(mcc_launch_linearize(la, p->model, p->V, p->max_epp, p->rational, p->prism, p->stream));
    }
    if (lin_only) return MCC_OK;
    if (tim) HIPCHK(hipEventRecord(p->ev_lin[p->ev_used + 1], p->stream));
    if (p->fused) {
        if (rccl) {
            const bool tx = tim && p->ev_x_used + 2 <= (int)p->ev_x.size();
            if (tx) HIPCHK(hipEventRecord(p->ev_x[p->ev_x_used], p->stream));
            ncclResult_t r = ncclAllReduce(p->packed.p, p->packed.p, (size_t)p->packed_len, ncclDouble, ncclSum,
                                           p->comm, p->stream);
            if (r != ncclSuccess) return fail(MCC_ECOMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
            if (tx) {
                HIPCHK(hipEventRecord(p->ev_x[p->ev_x_used + 1], p->stream));
                p->ev_x_used += 2;
            }
            SolveArgs so{solve_ctx(p, do_update), p->packed.p, peer_ctx(p, false), 0, {}};
            HIPCHK(mcc_launch_solve(so, p->stream));
        }
        if (tim) {
            HIPCHK(hipEventRecord(p->ev_step[p->ev_used + 1], p->stream));
            p->ev_used += 2;
        }
        return MCC_OK;
    }

    if (!fold) HIPCHK(mcc_launch_schur(sa, p->n_items + p->n_norm_chunks, p->stream));
    if (rccl) {
        const bool tx = tim && p->ev_x_used + 2 <= (int)p->ev_x.size();
        if (tx) HIPCHK(hipEventRecord(p->ev_x[p->ev_x_used], p->stream));
        ncclResult_t r = ncclAllReduce(p->packed.p, p->packed.p, (size_t)p->packed_len, ncclDouble, ncclSum,
                                       p->comm, p->stream);
        if (r != ncclSuccess) return fail(MCC_ECOMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        if (tx) {
            HIPCHK(hipEventRecord(p->ev_x[p->ev_x_used + 1], p->stream));
            p->ev_x_used += 2;
        }
    }
    if (split) {
        SolveArgs so{solve_ctx(p, do_update), p->packed.p, peer_ctx(p, peer), 0, {}};
        // MCC_DIAG: k_solve's phase stamps after k_schur's rows
        so.ctx.stamps = p->stamps.p ? p->stamps.p + mcc::kStampStride * (size_t)std::max(p->V, 1) +
                                          mcc::kSchurStampStride * (size_t)(p->n_items + p->n_norm_chunks)
                                    : nullptr;
        if (p->warm && do_update) so.warm = warm_ctx(p);
        if (peer && p->peer_push) {   // MCC_PEER_PUSH=0: k_solve's one workgroup sends too
            HIPCHK(mcc_launch_peer_push(so.peer, p->state.p, p->packed.p, p->stream));
            so.pushed = 1;
        }
        HIPCHK(mcc_launch_solve(so, p->stream));
    }
    if (tim) {
        HIPCHK(hipEventRecord(p->ev_step[p->ev_used + 1], p->stream));
        p->ev_used += 2;
    }
    return MCC_OK;
}

// standalone photo back-substitution: deltaX of the photos (do_update = 0) or a flush of the
// pending update (do_update = 1)
int enqueue_backsub(mcc_problem* p, int do_update) {
    mcc::BacksubArgs ba{p->state.p, p->photo_ptr.p, p->edge_gblock.p, p->Y.p, p->zp.p, p->dg.p,
                        p->fused ? p->W.p : nullptr, p->x.p, p->delta.p, p->photo_norm.p, p->V, p->m, do_update};
    HIPCHK(mcc_launch_backsub(ba, p->stream));
    return MCC_OK;
}

int build_graph(mcc_problem* p, int k) {
    if (p->gexec[k]) return MCC_OK;
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal));
    int rc = MCC_OK;
    for (int s = 0; s < (1 << k) && rc == MCC_OK; ++s) rc = enqueue_step(p, 1, nullptr);
    hipError_t ee = hipStreamEndCapture(p->stream, &graph);
    if (rc != MCC_OK) return rc;
    if (ee != hipSuccess) return fail(MCC_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ee));
    HIPCHK(hipGraphInstantiate(&p->gexec[k], graph, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(graph));
    return MCC_OK;
}
int launch_update_steps(mcc_problem* p, int n) {
    if (p->timing_window) p->win_steps += n;
    // the split step's timing window runs eagerly (an event pair around the linearisation kernels of
    // every step; HIP events recorded inside a captured graph carry no timestamps) behind k_delay,
    // which keeps the GPU busy while the host enqueues the window, so the GPU then runs the steps
    // back to back as it runs a graph's, without waiting for launches between kernels
    const bool eager = !p->use_graph || p->timing;
    if (!eager) {
        // every graph of this batch exists before the batch's helper starts: instantiating a 64-step
        // graph takes milliseconds, which the helper would otherwise spend polling for the first system
        for (int k = p->graph_sizes - 1, r = n; k >= 0; --k)
            if (r >= (1 << k)) {
                int rc = build_graph(p, k);
                if (rc) return rc;
                r -= (r >> k) << k;
            }
    }
    if (p->warm && n > 0) {
        // the batch's helper: after the previous one (side-stream order), with the stop flag cleared
        HIPCHK(hipMemsetAsync(p->wsync + 2, 0, sizeof(unsigned), p->side));
        HIPCHK(mcc_launch_sinv_helper(warm_ctx(p), p->m, n, p->side));
    }
    int rc = MCC_OK;
    if (eager) {
        for (int i = 0; i < n && rc == MCC_OK; ++i) rc = enqueue_step(p, 1, nullptr);
    } else {
        for (int k = p->graph_sizes - 1; k >= 0 && rc == MCC_OK; --k)
            while (n >= (1 << k) && rc == MCC_OK) {
                hipError_t e = hipGraphLaunch(p->gexec[k], p->stream);
                if (e != hipSuccess) rc = fail(MCC_EHIP, std::string("hipGraphLaunch: ") + hipGetErrorString(e));
                n -= 1 << k;
            }
    }
    if (rc != MCC_OK && p->warm) {
        // the steps that would have fed the helper were not enqueued: release it (uncached flag)
        const unsigned one = 1;
        (void)hipMemcpy(p->wsync + 2, &one, sizeof(one), hipMemcpyHostToDevice);
    }
    return rc;
}

int read_state(mcc_problem* p);

// prev2 (the m > 30 warm solve's copies of [S | r], WarmCtx::refine): every word kFoldEmpty until the
// step's k_schur writes it, the pad word of an odd packed length 0 for good; the helper empties the
// words it has consumed.  Reset whenever the host re-enters (no launch in flight, the helper has exited:
// a loop that stopped or failed may leave an unconsumed system behind)
// (stream-ordered on the step stream: k_schur's writes follow it, and the helper reads a buffer only
// after k_schur's publication; `pad_too` also sets the pad words, once at mcc_create)
int reset_prev2(mcc_problem* p, bool pad_too = false) {
    if (!p->prev2) return MCC_OK;
    const int n = p->ntri + p->m;   // the words k_schur writes; the pad word after them stays 0
    for (int b = 0; b < 2; ++b)
        HIPCHK(hipMemsetAsync(p->prev2 + (size_t)b * p->prev_stride, 0xFF, (size_t)n * sizeof(double), p->stream));
    if (pad_too && p->prev_stride > n) {
        HIPCHK(hipStreamSynchronize(p->stream));
        const double zero[1] = {0.0};
        for (int b = 0; b < 2; ++b)
            HIPCHK(hipMemcpy(p->prev2 + (size_t)b * p->prev_stride + n, zero, sizeof(double), hipMemcpyHostToDevice));
    }
    return MCC_OK;
}

int set_state(mcc_problem* p, int reset_iter, int crit_type, int max_count, double eps) {
    p->stepping = false;
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(p->h_state, p->state.p, sizeof(State), hipMemcpyDeviceToHost));
    if (p->gfold && p->h_state->error) {
        // a folded launch that failed (a consumer's poll bound, a peer timeout) may have left words
        // behind: slots its items cleared before a late producer wrote them, partials its final never
        // read, a late spare's inverse and status.  Every launch of the stream has ended (synchronised
        // above), so all of them go back to kFoldEmpty, as mcc_create leaves them.
        for (auto* b : {&p->pairprod, &p->item_out, &p->fnorm, &p->fiv})
            if (b->p) HIPCHK(hipMemset(b->p, 0xFF, sizeof(double) * std::max<size_t>(b->n, 1)));
    }
    if (reset_iter && p->warm) {
        // a new optimisation starts without a previous inverse (its first solve is the direct
        // elimination), so its result does not depend on what the problem solved before.  The last
        // batch's helper has exited or will after inverting the last published system: wait for it.
        HIPCHK(hipStreamSynchronize(p->side));
        HIPCHK(hipMemset(p->wsync, 0, 2 * sizeof(unsigned)));
        HIPCHK(hipMemset(p->wsync + 4, 0, 3 * sizeof(unsigned)));   // the helper's refined epoch, status, corrections
    }
    if (p->warm && p->helper_refine) {
        HIPCHK(hipStreamSynchronize(p->side));
        int rc = reset_prev2(p);
        if (rc) return rc;
        if (!reset_iter) {
            // a system the last batch's helper did not consume (the loop stopped in k_solve after k_schur
            // published it) is withdrawn with its words: the next helper waits for the next publication
            unsigned inv = 0;
            HIPCHK(hipMemcpy(&inv, p->wsync + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(p->wsync, &inv, sizeof(unsigned), hipMemcpyHostToDevice));
        }
    }
    if (reset_iter) {
        p->h_state->iter = 0;
        p->h_state->change = 1.0;
        p->h_state->cam_normG2 = p->h_state->cam_normX2 = 0.0;
    }
    p->h_state->done = 0;
    p->h_state->crit_type = crit_type;
    p->h_state->max_count = max_count;
    p->h_state->eps = eps;
    p->h_state->error = 0;
    // the fused step's spare protocol restarts (the stream is idle: no spare of an earlier launch runs)
    p->h_state->spare_ack = 0;
    HIPCHK(hipMemcpy(p->state.p, p->h_state, sizeof(State), hipMemcpyHostToDevice));
    // the folded reduction's task ticket (a failed launch's groups may not all have drawn)
    if (p->fold_ticket.p) HIPCHK(hipMemset(p->fold_ticket.p, 0, sizeof(int)));
    return MCC_OK;
}

// mcc_optimize's start: mcc_set_params + set_state(reset) with one host round trip (the state read
// that tells a failed previous launch and keeps the device-monotonic words); the parameters and the
// new state go in as copies ordered before the first step on the stream (round 6: the setup took
// ~8 synchronous copies, ~75 us of a config4 call)
int begin_optimize(mcc_problem* p, const float* x, int crit_type, int max_count, double eps) {
    p->stepping = false;
    if (!p->h_x) HIPCHK(hipHostMalloc((void**)&p->h_x, sizeof(float) * std::max(p->P, 1), hipHostMallocDefault));
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(p->h_state, p->state.p, sizeof(State), hipMemcpyDeviceToHost));
    if (p->gfold && p->h_state->error)   // (set_state: what a failed folded launch leaves)
        for (auto* b : {&p->pairprod, &p->item_out, &p->fnorm, &p->fiv})
            if (b->p) HIPCHK(hipMemset(b->p, 0xFF, sizeof(double) * std::max<size_t>(b->n, 1)));
    if (p->warm) {   // (set_state: no previous inverse; the last batch's helper has exited)
        HIPCHK(hipStreamSynchronize(p->side));
        HIPCHK(hipMemset(p->wsync, 0, 2 * sizeof(unsigned)));
        HIPCHK(hipMemset(p->wsync + 4, 0, 3 * sizeof(unsigned)));
        if (p->helper_refine) {
            int rc = reset_prev2(p);
            if (rc) return rc;
        }
    }
    State* h = p->h_state;
    h->iter = 0;
    h->change = 1.0;
    h->cam_normG2 = h->cam_normX2 = 0.0;
    h->done = 0;
    h->crit_type = crit_type;
    h->max_count = max_count;
    h->eps = eps;
    h->error = 0;
    h->spare_ack = 0;
    h->pending = 0;   // new parameters: no pending photo update
    std::memcpy(p->h_x, x, sizeof(float) * p->P);
    HIPCHK(hipMemcpyAsync(p->x.p, p->h_x, sizeof(float) * p->P, hipMemcpyHostToDevice, p->stream));
    HIPCHK(hipMemcpyAsync(p->state.p, h, sizeof(State), hipMemcpyHostToDevice, p->stream));
    if (p->fold_ticket.p) HIPCHK(hipMemsetAsync(p->fold_ticket.p, 0, sizeof(int), p->stream));
    return MCC_OK;
}

int flush_pending(mcc_problem* p) {
    int rc = read_state(p);
    if (rc) return rc;
    if (!p->h_state->pending) return MCC_OK;
    if ((rc = enqueue_backsub(p, 1))) return rc;
    HIPCHK(hipStreamSynchronize(p->stream));
    p->h_state->pending = 0;
    HIPCHK(hipMemcpy(&p->state.p->pending, &p->h_state->pending, sizeof(int), hipMemcpyHostToDevice));
    return MCC_OK;
}

int read_state(mcc_problem* p) {
    HIPCHK(hipMemcpyAsync(p->h_state, p->state.p, sizeof(State), hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    return MCC_OK;
}

int check_state_error(mcc_problem* p) {
    const int e = p->h_state->error;
    if (e & mcc::kErrPeerTimeout) return fail(MCC_ECOMM, "peer exchange timed out (a rank did not deliver)");
    if (e & mcc::kErrWarmTimeout)
        return fail(MCC_ETIMEOUT, "the warm-solve helper did not deliver the previous step's inverse in time");
    if (e & mcc::kErrCameraNotPD) return fail(MCC_ENOTPD, "reduced camera system is not positive definite");
    if (e & mcc::kErrPhotoNotPD)
        return fail(MCC_ENOTPD, "a photo normal-equation block is not positive definite (on this or another rank)");
    return MCC_OK;
}

}  // namespace

extern "C" {

const char* mcc_last_error(void) { return g_err.c_str(); }

// the other C-ABI translation units (mcc_omnicalib_api.cpp) report through the same message slot
__attribute__((visibility("hidden"))) int mcc_internal_fail(int code, const char* msg) { return fail(code, msg); }
__attribute__((visibility("hidden"))) void mcc_internal_rodrigues_m2v(const double* R, double* r) {
    host_rodrigues_m2v(R, r);
}

int mcc_nparams(const mcc_problem* p) { return p ? p->P : 0; }
int mcc_global_dim(const mcc_problem* p) { return p ? p->m : 0; }

int mcc_create(mcc_problem** out, const mcc_desc* d) {
    if (!out || !d) return fail(MCC_EINVAL, "null argument");
    *out = nullptr;
    if (d->model < 0 || d->model > 2) return fail(MCC_EINVAL, "unknown model");
    if (d->n_cams < 1 || d->n_photos < 0 || d->n_edges < 0) return fail(MCC_EINVAL, "bad sizes");
    // the reference's meanReProjError is 0 / 0 without observations (src/multicalib.cpp:989), and
    // a photo vertex exists only through an edge (getPhotoVertex, :323-346); a rank of a sharded
    // problem needs photos of its own to take part in the per-step exchange
    if (d->n_photos < 1 || d->n_edges < 1) return fail(MCC_EINVAL, "no photo vertices / observations");
    if (d->model != MCC_MODEL_DOUBLESIDE && d->n_cams < 2) return fail(MCC_EINVAL, "need >= 2 cameras");
    if (d->model == MCC_MODEL_OMNI && (d->nd != 4 || !d->xi)) return fail(MCC_EINVAL, "omni needs nd == 4 and xi");
    if (d->model != MCC_MODEL_OMNI && !(d->nd == 4 || d->nd == 5 || d->nd == 8 || d->nd == 12 || d->nd == 14))
        return fail(MCC_EINVAL, "pinhole nd must be 4, 5, 8, 12 or 14");
    if (d->model == MCC_MODEL_DOUBLESIDE && !d->cam_pose) return fail(MCC_EINVAL, "DOUBLESIDE needs cam_pose");
    const int C = d->n_cams, V = d->n_photos, E = d->n_edges;
    for (int e = 0; e < E; ++e) {
        if (d->edge_cam[e] < 0 || d->edge_cam[e] >= C || d->edge_photo[e] < 0 || d->edge_photo[e] >= V ||
            d->edge_n[e] < 1 || d->edge_off[e] < 0)
            return fail(MCC_EINVAL, "edge " + std::to_string(e) + " out of range");
        if (d->edge_n[e] > 1024) return fail(MCC_EINVAL, "more than 1024 corners in an edge");
        int side = d->edge_side ? d->edge_side[e] : MCC_FRONT;
        if (side == MCC_BACK && d->model == MCC_MODEL_PINHOLE && !d->ds_pose)
            return fail(MCC_EINVAL, "BACK edge without doubleSideTransform (the reference dereferences an empty Mat)");
        if (side == MCC_BACK && d->model == MCC_MODEL_OMNI) return fail(MCC_EINVAL, "BACK edges are pinhole only");
    }

    mcc_problem* p = new mcc_problem();
    p->model = d->model; p->C = C; p->V = V; p->E = E; p->nd = d->nd; p->device = d->device;
    p->m = d->model == MCC_MODEL_DOUBLESIDE ? 6 : 6 * (C - 1);
    p->P = p->m + 6 * V;
    int rc = MCC_OK;
    auto bail = [&](int code) { mcc_destroy(p); return code; };
#define HIPC(expr)                                                                          \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return bail(fail(MCC_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e))); \
    } while (0)
    HIPC(hipSetDevice(d->device));
    HIPC(stream_pool().take(d->device, &p->stream));
    if (const char* g = std::getenv("MCC_GRAPH")) p->use_graph = std::atoi(g) != 0;
    if (const char* g = std::getenv("MCC_GRAPH_SIZES"))
        p->graph_sizes = std::min(mcc_problem::kGraphSizes, std::max(1, std::atoi(g)));

    // distortion specialisation (zero coefficients are exact no-ops in OpenCV's formula)
    if (d->model != MCC_MODEL_OMNI) {
        for (int c = 0; c < C; ++c)
            for (int q = 5; q < std::min(d->nd, 12); ++q) {
                const float v = d->D[d->nd * c + q];
                if (v != 0.f) {
                    if (q < 8) p->rational = true;
                    else p->prism = 1;
                }
            }
        // the tilted sensor (tau_x, tau_y: D[12], D[13] of 14): matTilt per camera in FP64, as
        // cvProjectPoints2Internal forms it from the CV_32F coefficients (identity where tau = 0, which
        // the projection then applies exactly: vecTilt = (xd0, yd0, 1), invProj = 1)
        bool tilt = false;
        for (int c = 0; c < C && d->nd == 14; ++c)
            tilt = tilt || d->D[14 * c + 12] != 0.f || d->D[14 * c + 13] != 0.f;
        if (tilt) {
            p->rational = true;   // zero k4..k6 / s1..s4 are exact no-ops in the 14-term formula
            p->prism = 2;
            std::vector<double> mt(9 * (size_t)C);
            for (int c = 0; c < C; ++c) tilt_matrix(d->D[14 * c + 12], d->D[14 * c + 13], mt.data() + 9 * c);
            HIPC(p->tilt.upload(mt.data(), mt.size()));
        }
    }

    // ---- photo-major edge order (stable within a photo: reference edge order)
    std::vector<int> order(E);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return d->edge_photo[a] < d->edge_photo[b]; });
    p->dev2ref_edge = order;
    std::vector<int> photo_ptr(V + 1, 0);
    for (int e = 0; e < E; ++e) photo_ptr[d->edge_photo[e] + 1]++;
    for (int v = 0; v < V; ++v) {
        p->max_epp = std::max(p->max_epp, photo_ptr[v + 1]);
        photo_ptr[v + 1] += photo_ptr[v];
    }
    long long ncorner = 0;
    for (int e = 0; e < E; ++e) ncorner += d->edge_n[e];
    p->corners = ncorner;
    std::vector<float> ox(ncorner), oy(ncorner), oz(ncorner), iu(ncorner), iv(ncorner);
    std::vector<int4> info(E);
    std::vector<int> gblock(E), ephoto(E);
    p->dev2ref_corner.resize(ncorner);
    p->edge_n_dev.resize(E);
    long long off = 0;
    for (int de = 0; de < E; ++de) {
        const int e = order[de], n = d->edge_n[e];
        const int side = d->edge_side ? d->edge_side[e] : MCC_FRONT;
        for (int i = 0; i < n; ++i) {
            const long long s = (long long)d->edge_off[e] + i;
            ox[off + i] = d->obj[3 * s]; oy[off + i] = d->obj[3 * s + 1]; oz[off + i] = d->obj[3 * s + 2];
            iu[off + i] = d->img[2 * s]; iv[off + i] = d->img[2 * s + 1];
            p->dev2ref_corner[off + i] = s;
        }
        info[de] = make_int4(d->edge_cam[e], side, (int)off, n);
        if (side == MCC_BACK) p->has_back = 1;
        ephoto[de] = d->edge_photo[e];
        p->edge_n_dev[de] = n;
        if (d->model == MCC_MODEL_DOUBLESIDE) gblock[de] = side == MCC_BACK ? 0 : -1;
        else gblock[de] = d->edge_cam[e] - 1;
        off += n;
    }
    std::vector<int> photo_corner(V + 1, 0);
    for (int v = 0; v < V; ++v) {
        photo_corner[v + 1] = photo_corner[v];
        for (int de = photo_ptr[v]; de < photo_ptr[v + 1]; ++de) photo_corner[v + 1] += info[de].w;
        p->max_cpp = std::max(p->max_cpp, photo_corner[v + 1] - photo_corner[v]);
    }

    // small camera blocks and at most two photo workgroups per CU (the fused kernel's occupancy):
    // one kernel per Gauss-Newton step.  More photos than that run the fused kernel's serial
    // per-photo chain in several rounds, and the split step is faster (config4, 1000 views:
    // 43.3 vs 47.4 us; config2, 500 views: 38.2 vs 25.9 us).  MCC_FUSED=1 / 0 forces either.
    int n_cu = 256;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess || n_cu <= 0)
        n_cu = 256;
    const int n_cu_dev = n_cu;   // the device's own (the folded step's progress rule below)
    if (const char* f = std::getenv("MCC_CUS")) n_cu = std::max(1, std::atoi(f));   // test: the path rules at another CU count
    // (the tilted sensor takes the split step: the fused kernel's PRISM variants already hold 256 VGPRs,
    // and the tilt's per-corner 3 x 3 map and 2 x 2 chain spill there; k_group / k_edge have room)
    const bool fusable = p->m <= mcc_problem::kFusedMaxM && V > 0 && p->max_epp <= 64 && p->prism != 2;
    p->fused = fusable && V <= 2 * n_cu;

    // ---- Schur pair lists.  The split step's photo work (k_group / k_photo) takes groups of
    // consecutive photos (at most kPhotoGroup photos and the cap's edges) and sums the group's pair
    // products per camera-pair block: one slot per (group, block), block-major over the groups,
    // k_schur sums a block's slots in order.  A contribution is one ordered edge pair (e1, e2) of a
    // photo with gblock(e1) <= gblock(e2) (both orders within one block), in photo then edge order.
    const int nb = p->m / 6;
    p->nblk = nb * (nb + 1) / 2;
    auto blk_index = [nb](int b1, int b2) { return b1 * nb - b1 * (b1 - 1) / 2 + (b2 - b1); };
    auto make_groups = [&](int cap) {
        std::vector<int> g(1, 0);
        for (int v = 0; v < V;) {
            int w = v, edges = 0;
            while (w < V && w - v < mcc::kPhotoGroup &&
                   (w == v || edges + (photo_ptr[w + 1] - photo_ptr[w]) <= cap)) {
                edges += photo_ptr[w + 1] - photo_ptr[w];
                ++w;
            }
            g.push_back(w);
            v = w;
        }
        return g;
    };
    // k_group takes groups of at most kGroupRound edges (one 16-edge round per workgroup; config4's
    // 1 000 photos -> 250 workgroups, one per CU); k_photo's groups sum more photos (<= 64 edges).
    // k_group (two workgroups per CU) wins while its groups fit the CUs in one wave of workgroups
    // (config4: 32.3 vs 36.9 us per step); with more groups the three-kernel form's higher
    // occupancy wins (config5: 67.3 vs 61.0, config3: 185.5 vs 120.5).  MCC_GROUP=1 / 0 forces.
    int group_cap = mcc::kGroupRound;   // MCC_GROUP_EDGES: k_group's edges per group (A/B; > 16: several rounds)
    const char* gcap_env = std::getenv("MCC_GROUP_EDGES");
    if (gcap_env) group_cap = std::max(1, std::min(4 * mcc::kGroupRound, std::atoi(gcap_env)));
    std::vector<int> pgrp_ptr = make_groups(group_cap);
    // More 16-edge groups than CUs: wider groups (up to two 16-edge rounds each) while that brings them
    // within one wave of workgroups -- a second wave of groups costs a whole group chain, a second
    // round inside a group only its edge phases (config3's 8-rank shard, 625 views / 4 871 edges:
    // 313 groups of 16 -> 244 of <= 24 edges, 58.4 -> 47.4 us per step against the three kernels;
    // at 64 edges config5's 2 000 views take 65.0 vs 60.2 us, so the widening stops at 32)
    for (int cap = mcc::kGroupRound + 8; !gcap_env && (int)pgrp_ptr.size() - 1 > n_cu && cap <= 2 * mcc::kGroupRound;
         cap += 8) {
        std::vector<int> g = make_groups(cap);
        if ((int)g.size() - 1 <= n_cu) {
            pgrp_ptr = std::move(g);
            group_cap = cap;
        }
    }
    // The fused kernel runs a photo's edges one per wave on its four waves, so photos with more than
    // four edges take it through several dependent rounds; k_group spreads a group's 16 edges over its
    // eight waves in one.  With more than four edges per photo and k_group's groups within the CUs the
    // split step wins (config5's 500-view shard, 8 edges per photo: 28.9 vs 32.5 us per step).
    if (p->fused && p->max_epp > 4 && (int)pgrp_ptr.size() - 1 <= n_cu) p->fused = false;
    if (const char* f = std::getenv("MCC_FUSED")) p->fused = fusable && std::atoi(f) != 0;
    if (!p->fused && p->max_epp > 64)
        return bail(fail(MCC_EINVAL, "more than 64 edges (camera observations) of one photo vertex"));
    p->use_group = !p->fused && (int)pgrp_ptr.size() - 1 <= n_cu;
    if (const char* f = std::getenv("MCC_GROUP")) p->use_group = !p->fused && std::atoi(f) != 0;
    if (!p->use_group) pgrp_ptr = make_groups(mcc::kPhotoGroupEdges);
    if (const char* f = std::getenv("MCC_GROUP_LANES")) p->group_lanes = std::atoi(f) == 16 ? 16 : 32;
    if (const char* f = std::getenv("MCC_PEER_PUSH")) p->peer_push = std::atoi(f) != 0;
    if (const char* f = std::getenv("MCC_POISON_HANDOFF")) {
        p->poison_level = std::atoi(f);
        p->poison = p->poison_level != 0;
    }
    const int NG = (int)pgrp_ptr.size() - 1;
    std::vector<int4> gpairs;                           // {first contribution, count, diagonal << 1, slot}
    std::vector<unsigned> gcon;
    std::vector<int> gpair_ptr(NG + 1, 0), gcon_ptr(NG + 1, 0);
    std::vector<std::vector<int>> blk_src(p->nblk);   // each block's gpairs, group order
    std::vector<std::vector<unsigned>> per_blk(p->nblk);
    for (int g = 0; g < NG; ++g) {
        const int ge0 = photo_ptr[pgrp_ptr[g]];
        std::vector<int> used;
        for (int v = pgrp_ptr[g]; v < pgrp_ptr[g + 1]; ++v)
            for (int e1 = photo_ptr[v]; e1 < photo_ptr[v + 1]; ++e1) {
                if (gblock[e1] < 0) continue;
                for (int e2 = photo_ptr[v]; e2 < photo_ptr[v + 1]; ++e2) {
                    if (gblock[e2] < 0 || gblock[e1] > gblock[e2]) continue;
                    const int b = blk_index(gblock[e1], gblock[e2]);
                    if (per_blk[b].empty()) used.push_back(b);
                    per_blk[b].push_back((unsigned)(e1 - ge0) | ((unsigned)(e2 - ge0) << 8) |
                                         ((e1 == e2 ? 1u : 0u) << 16) | ((unsigned)(v - pgrp_ptr[g]) << 17));
                }
            }
        // the group's block pairs by contribution count, largest first: k_photo's pair tasks of a
        // wave step through their contributions in lock-step, so each wave should hold pairs of
        // similar counts (config3: 15.5 -> 10.8 iterations on a group's busiest wave).  Outputs
        // are unchanged: a pair's slot offset travels with it.
        std::sort(used.begin(), used.end(), [&](int x, int y) {
            return per_blk[x].size() != per_blk[y].size() ? per_blk[x].size() > per_blk[y].size() : x < y;
        });
        const int cbase = (int)gcon.size();
        for (int b : used) {
            blk_src[b].push_back((int)gpairs.size());
            const int b1 = [&] { int r = 0; while (r + 1 < nb && blk_index(r + 1, r + 1) <= b) ++r; return r; }();
            gpairs.push_back(make_int4((int)gcon.size() - cbase, (int)per_blk[b].size(), blk_index(b1, b1) == b ? 2 : 0, -1));
            gcon.insert(gcon.end(), per_blk[b].begin(), per_blk[b].end());
            per_blk[b].clear();
        }
        gpair_ptr[g + 1] = (int)gpairs.size();
        gcon_ptr[g + 1] = (int)gcon.size();
        p->max_gpairs = std::max(p->max_gpairs, gpair_ptr[g + 1] - gpair_ptr[g]);
        p->max_gcon = std::max(p->max_gcon, gcon_ptr[g + 1] - gcon_ptr[g]);
        p->max_gedges = std::max(p->max_gedges, photo_ptr[pgrp_ptr[g + 1]] - ge0);
    }
    p->n_pgroups = NG;
    p->photo_shmem = mcc::photo_lds_bytes(p->max_gedges, p->max_gpairs, p->max_gcon);
    p->group_shmem = mcc::group_lds_bytes(p->max_gedges, C, p->max_gpairs, p->max_gcon);
    std::vector<int4> items;
    std::vector<int> block_items(p->nblk + 1, 0);
    // slot sizes: 48 doubles on a diagonal camera-pair block (S entries, r, JTE), 36 off the
    // diagonal (no self pair there, so r and JTE would be zeros); pair .w = the slot's offset in
    // doubles; item = {block, first slot's offset, slots, slot size}
    int n_slots = 0;
    size_t n_doubles = 0;
    // m <= 30 with several camera-pair blocks (one hand-off level: the final arriver loads every
    // item's partial in one batch, so more items cost it little): 64 slots per item, four items per
    // 250-slot block at config4 -- 28.4-28.6 vs 29.1-29.2 us per step with 320 (interleaved, round 4;
    // 32: 28.7-28.8, 16: 30.7).  config5's single block (DoubleSide, m = 6) keeps 320 (60.5-60.7 vs
    // 60.8-60.9 at 64)
    int min_slots = p->m <= 30 && p->nblk > 1 ? 64 : 320;
    if (const char* f = std::getenv("MCC_ITEM_SLOTS")) min_slots = std::max(1, std::atoi(f));
    for (int b = 0; b < p->nblk; ++b) {
        int b1 = 0;
        while (b1 + 1 < nb && blk_index(b1 + 1, b1 + 1) <= b) ++b1;
        const int stride = blk_index(b1, b1) == b ? 48 : 36;
        const int begin = n_slots;
        const size_t base = n_doubles;
        for (int src : blk_src[b]) {
            gpairs[src].w = (int)n_doubles;
            n_doubles += stride;
            ++n_slots;
        }
        if (n_doubles > (size_t)INT32_MAX) return bail(fail(MCC_EINVAL, "too many Schur pairs"));
        const int end = n_slots;
        // <= 24 work items per block keeps the last-arriver assembly short; >= min_slots slots per
        // item (MCC_ITEM_SLOTS, default 320) amortises an item's fixed latency (one load round trip, the
        // write-through hand-off and ticket) over more slots (config3, interleaved: 160 -> 320 slots
        // 120.8 -> 119.6 us per step, 640 122.3; configs 4 and 5 within noise)
        // A block of at most min_slots slots is one item, which writes the block's packed entries
        // itself (slot size | kItemSingle): no item hand-off level (config4: every block, k_schur
        // 9.2 -> 8.7 us).  Larger blocks keep >= min_slots per item: config5's one block of 250
        // slots as a single item took 10.7 us against 9.3 as two items and the hand-off.
        // Blocks of (single_max, min_slots] slots take two items (config5's 250-slot block: k_schur
        // 10.5 us as one item vs 9.8 as two under rocprofv3)
        const int nsl = end - begin, single_max = std::min(min_slots, 160);
        int per_item = std::max(min_slots, (nsl + 23) / 24);
        if (nsl > single_max && nsl <= per_item) per_item = (nsl + 1) / 2;
        const int single = (nsl <= per_item) ? mcc::kItemSingle : 0;
        for (int s = begin; s < end; s += per_item) {
            items.push_back(make_int4(b, (int)(base + (size_t)(s - begin) * stride), std::min(end, s + per_item) - s,
                                      stride | single));
            p->max_item_slots = std::max(p->max_item_slots, items.back().z);
        }
        // a block no photo couples gets one empty item: it writes the block's zeros (every packed
        // entry is rewritten each step; the all-reduce leaves sums there)
        if (begin == end) items.push_back(make_int4(b, (int)base, 0, stride | mcc::kItemSingle));
        block_items[b + 1] = (int)items.size();
    }
    p->n_pair_doubles = n_doubles;
    // A camera block without an observation here is accepted: a rank of a photo-sharded problem
    // may hold no photo of some camera while the summed system is fine.  If the whole problem
    // leaves a camera unobserved, the reduced system is singular and the step fails with
    // MCC_ENOTPD (the device positive-definiteness check of the solve).
    p->n_items = (int)items.size();
    p->n_pairs = n_slots;
    p->n_norm_chunks = (V + 255) / 256;
    // one hand-off level (m <= 30) while the final arriver loads everything in one batch
    const bool one_fits = p->m <= 30 && 48 * (p->n_items + p->n_norm_chunks) + p->m * p->m <= mcc::kSchurOneLevelLoads * 256;
    p->schur_one_level = one_fits ? 1 : 0;
    if (const char* f = std::getenv("MCC_SCHUR_ONE_LEVEL")) p->schur_one_level = one_fits && std::atoi(f) != 0;
    if (p->m > 128) return bail(fail(MCC_EINVAL, "global block larger than 128 parameters (22 cameras)"));
    p->group_size = std::max(1, (int)std::ceil(std::sqrt((double)std::max(V, 1))));
    p->n_groups = (std::max(V, 1) + p->group_size - 1) / p->group_size;

    // ---- fixed transforms
    std::vector<float> cam_rt(6 * C, 0.f);
    if (d->model == MCC_MODEL_DOUBLESIDE) {
        for (int c = 0; c < C; ++c) {
            double R[9], r[3];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R[i * 3 + j] = d->cam_pose[16 * c + i * 4 + j];
            host_rodrigues_m2v(R, r);
            for (int i = 0; i < 3; ++i) { cam_rt[6 * c + i] = (float)r[i]; cam_rt[6 * c + 3 + i] = d->cam_pose[16 * c + i * 4 + 3]; }
        }
    }
    double ds_rt[6] = {0, 0, 0, 0, 0, 0};
    if (d->ds_pose && d->model == MCC_MODEL_PINHOLE) {
        double R[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[i * 3 + j] = d->ds_pose[i * 4 + j];
        host_rodrigues_m2v(R, ds_rt);
        for (int i = 0; i < 3; ++i) ds_rt[3 + i] = d->ds_pose[i * 4 + 3];
    }
    std::vector<double> alpha(4096);
    for (size_t k = 0; k < alpha.size(); ++k) alpha[k] = std::pow(0.95, (double)k + 1.0);   // src/multicalib.cpp:483

    // ---- uploads
    HIPC(p->obj_x.upload(ox.data(), ncorner)); HIPC(p->obj_y.upload(oy.data(), ncorner));
    HIPC(p->obj_z.upload(oz.data(), ncorner));
    HIPC(p->img_u.upload(iu.data(), ncorner)); HIPC(p->img_v.upload(iv.data(), ncorner));
    HIPC(p->edge_info.upload(info.data(), E));
    HIPC(p->edge_gblock.upload(gblock.data(), E));
    HIPC(p->edge_photo.upload(ephoto.data(), E));
    HIPC(p->photo_ptr.upload(photo_ptr.data(), V + 1));
    HIPC(p->photo_corner.upload(photo_corner.data(), V + 1));
    HIPC(p->K.upload(d->K, 9 * C));
    HIPC(p->D.upload(d->D, (size_t)d->nd * C));
    std::vector<float> xi(C, 0.f);
    if (d->xi) std::copy(d->xi, d->xi + C, xi.begin());
    HIPC(p->xi.upload(xi.data(), C));
    HIPC(p->cam_rt.upload(cam_rt.data(), 6 * C));
    std::vector<float> cp(16 * C, 0.f);
    if (d->cam_pose) std::copy(d->cam_pose, d->cam_pose + 16 * C, cp.begin());
    HIPC(p->cam_pose.upload(cp.data(), 16 * C));
    HIPC(p->ds_rt.upload(ds_rt, 6));
    HIPC(p->alpha.upload(alpha.data(), alpha.size()));
    HIPC(p->pgrp_ptr.upload(pgrp_ptr.data(), pgrp_ptr.size()));
    {
        std::vector<int> pgrp_edge(pgrp_ptr.size());
        for (size_t g = 0; g < pgrp_ptr.size(); ++g) pgrp_edge[g] = photo_ptr[pgrp_ptr[g]];
        HIPC(p->pgrp_edge.upload(pgrp_edge.data(), pgrp_edge.size()));
        std::vector<unsigned char> lph(std::max(E, 1), 0);
        for (size_t g = 0; g + 1 < pgrp_ptr.size(); ++g)
            for (int v = pgrp_ptr[g]; v < pgrp_ptr[g + 1]; ++v)
                for (int e = photo_ptr[v]; e < photo_ptr[v + 1]; ++e) lph[e] = (unsigned char)(v - pgrp_ptr[g]);
        HIPC(p->edge_lphoto.upload(lph.data(), lph.size()));
    }
    if (!p->fused && !p->use_group) {
        // k_prep4's groups: consecutive photos, <= kPrepPhotos of them and kPrepEdges edges (or one photo)
        if (const char* f = std::getenv("MCC_PREP_LANES")) p->prep_lanes = std::atoi(f) == 4 ? 4 : 1;
        std::vector<int> pp(1, 0);
        for (int v = 0; v < V;) {
            int w = v, edges = 0;
            while (w < V && w - v < mcc::kPrepPhotos &&
                   (w == v || edges + (photo_ptr[w + 1] - photo_ptr[w]) <= mcc::kPrepEdges)) {
                edges += photo_ptr[w + 1] - photo_ptr[w];
                ++w;
            }
            pp.push_back(w);
            v = w;
        }
        std::vector<int> pe(pp.size());
        for (size_t g = 0; g < pp.size(); ++g) pe[g] = photo_ptr[pp[g]];
        p->n_prep = (int)pp.size() - 1;
        HIPC(p->prep_ptr.upload(pp.data(), pp.size()));
        HIPC(p->prep_edge.upload(pe.data(), pe.size()));
    }
    HIPC(p->gpair_ptr.upload(gpair_ptr.data(), gpair_ptr.size()));
    HIPC(p->gpairs.upload(gpairs.data(), gpairs.size()));
    HIPC(p->gcon_ptr.upload(gcon_ptr.data(), gcon_ptr.size()));
    HIPC(p->gcon.upload(gcon.data(), gcon.size()));
    HIPC(p->items.upload(items.data(), items.size()));
    HIPC(p->block_items.upload(block_items.data(), block_items.size()));
    HIPC(p->x.alloc(p->P)); HIPC(p->xerr.alloc(p->P));
    HIPC(p->Y.alloc(36 * (size_t)E));
    HIPC(p->pairprod.alloc(p->fused ? 0 : p->n_pair_doubles));
    const bool use_split = !p->fused && !p->use_group;   // k_prep -> k_edge -> k_photo records
    HIPC(p->erec.alloc(use_split ? 12 * (size_t)E : 0));
    HIPC(p->echain.alloc(use_split ? 54 * (size_t)E : 0));
    HIPC(p->eh.alloc(use_split ? 90 * (size_t)E : 0));
    HIPC(p->zp.alloc(6 * (size_t)V));
    HIPC(p->gp_tot.alloc(6 * (size_t)V));
    // + 24 zeroed items of padding: the assembly loads a fixed 24 items per block unconditionally
    HIPC(p->item_out.alloc(48 * (size_t)(items.size() + p->n_norm_chunks + 24)));
    HIPC(hipMemset(p->item_out.p, 0, sizeof(double) * p->item_out.n));
    HIPC(p->counter.alloc(1));
    HIPC(hipMemset(p->counter.p, 0, sizeof(int)));
    HIPC(p->cnt_blk.alloc(p->nblk));
    HIPC(hipMemset(p->cnt_blk.p, 0, sizeof(int) * std::max(p->nblk, 1)));
    p->ntri = p->m * (p->m + 1) / 2;
    p->packed_len = p->ntri + 2 * p->m + 2;
    HIPC(p->packed.alloc(p->packed_len));
    HIPC(p->dg.alloc(p->m)); HIPC(p->delta.alloc(p->P));
    HIPC(p->photo_norm.alloc(2 * (size_t)V));
    if (p->fused) {
        // rows padded to an even count: 16-B write-through stores (k_linearize's hand-off)
        const size_t lcp = (size_t)((p->packed_len + 1) & ~1);
        HIPC(p->contrib.alloc(lcp * std::max(V, 1)));
        HIPC(p->gsum.alloc(lcp * p->n_groups));
        HIPC(p->W.alloc((size_t)6 * p->m * std::max(V, 1)));
        HIPC(p->cnt.alloc(p->n_groups + 1));
        HIPC(hipMemset(p->cnt.p, 0, sizeof(int) * (p->n_groups + 1)));
    }
    HIPC(hipMemset(p->photo_norm.p, 0, sizeof(double) * 2 * std::max(V, 1)));
    HIPC(p->edge_sum.alloc(E));
    HIPC(p->state.alloc(1));
    HIPC(hipHostMalloc((void**)&p->h_state, sizeof(State), hipHostMallocDefault));
    std::memset(p->h_state, 0, sizeof(State));
    p->h_state->change = 1.0;
    HIPC(hipMemcpy(p->state.p, p->h_state, sizeof(State), hipMemcpyHostToDevice));
    if (C > 63) return bail(fail(MCC_EINVAL, "more than 63 cameras"));
    if (p->fused && mcc_lin_shmem(p->max_epp, C, p->m, p->max_cpp) > 160 * 1024)
        return bail(fail(MCC_EINVAL, "too many edges / corners per photo for the LDS staging"));
    if (!p->fused && !p->use_group && p->photo_shmem > 160 * 1024)
        return bail(fail(MCC_EINVAL, "too many Schur pairs of one photo for k_photo's LDS"));
    if (!p->fused && p->use_group && p->group_shmem > 160 * 1024)
        return bail(fail(MCC_EINVAL, "too many edges / Schur pairs of one photo group for k_group's LDS"));
    HIPC(mcc_set_kernel_attrs(p->max_epp, C, p->m, p->max_cpp, p->photo_shmem, p->use_group ? p->group_shmem : 0));
    // m <= 30 on k_group -> k_schur (config4): the previous system's inverse from a spare k_group
    // workgroup, refinement in k_schur's final solve (MCC_SMALL_WARM=0: the register Gauss-Jordan
    // only).  With S and the inverse in registers the refinement takes ~1.7 us at m = 18 against the
    // elimination's ~2.6 (config4, interleaved: 28.9 vs 29.4 us per step); round 4's first form, reading
    // them from LDS per product, took ~3 us and lost
    // The fused step (config2) refines with the inverse its previous launch's spare workgroup formed
    // (two updates stale: the spare and the final arriver of one launch run at the same time); its
    // LDS holds the spare's [S | I] and the final arriver's S, r and inverse (mcc_lin_shmem).
    // Two buffers by iteration parity, each tagged with the iteration that made it.
    {
        bool sw = (!p->fused && p->use_group && p->schur_one_level &&
                   p->group_shmem >= (size_t)2 * p->m * p->m * sizeof(double)) ||   // the spare's [S | I] in LDS
                  (p->fused && p->m <= 30);
        if (const char* f = std::getenv("MCC_SMALL_WARM")) sw = sw && std::atoi(f) != 0;
        if (sw) {
            HIPC(p->ssinv.alloc(2 * (size_t)p->m * p->m));
            HIPC(p->ssinv_ok.alloc(2));
            HIPC(hipMemset(p->ssinv_ok.p, 0, 2 * sizeof(int)));
            HIPC(p->warm_stats.alloc(5));   // mcc_solve_stats
            HIPC(hipMemset(p->warm_stats.p, 0, 5 * sizeof(long long)));
        }
    }
    // the folded reduction: k_group's one-level m <= 30 step with items of at most kSub x kFoldSlots
    // slots (every m <= 30 rig with several camera-pair blocks takes 64; a one-block rig 320: no fold)
    p->gfold = !p->fused && p->use_group && p->schur_one_level && p->max_item_slots <= 5 * 13 &&
               48 * (p->n_items + p->n_norm_chunks) + p->m * p->m + 1 <= mcc::kSchurOneLevelLoads * 256;
    // Progress of the folded launch does not rest on dispatch order.  Its producers (the groups, the
    // spare) never wait; its consumers (items, norm chunks, the final workgroup) spin until their words
    // land.  Whatever order the dispatcher picks, the launch completes as long as the spinning
    // consumers cannot hold every workgroup slot a producer needs: with at least one slot left over,
    // some producer is always resident or dispatchable, runs to its end and frees its slot.  k_group
    // fits at least one workgroup per CU, so the fold is taken only when the consumers fill at most
    // half of the CUs (the other half stays for producers even when another kernel shares the device);
    // otherwise the step is k_group -> k_schur.  MCC_FOLD_CONSUMERS_FIRST=1 (tests) lays the grid out
    // with the consumers at the lowest indices to exercise exactly that.
    const int fold_spin = p->n_items + p->n_norm_chunks + 1;
    p->gfold = p->gfold && 2 * fold_spin <= n_cu_dev;
    if (const char* f = std::getenv("MCC_GFOLD")) p->gfold = p->gfold && std::atoi(f) != 0;
    if (const char* f = std::getenv("MCC_FOLD_CONSUMERS_FIRST"))   // (a test instantiation, omnidir rigs)
        p->fold_first = p->gfold && p->model == MCC_MODEL_OMNI && std::atoi(f) != 0;
    if (p->gfold) {
        // the final workgroup's LDS (k_schur's one-level layout) within k_group's
        const size_t fs = mcc::schur_lds_bytes(p->m, 1, 1, 1, p->n_items + p->n_norm_chunks, p->nblk);
        if (fs > p->group_shmem) {
            p->group_shmem = fs;
            HIPC(mcc_set_kernel_attrs(p->max_epp, C, p->m, p->max_cpp, p->photo_shmem, p->group_shmem));
        }
        HIPC(p->fnorm.alloc(4 * (size_t)std::max(V, 1)));
        HIPC(p->fiv.alloc((size_t)p->m * p->m + 1));
        int max_bi = 0;
        for (int b = 0; b < p->nblk; ++b) max_bi = std::max(max_bi, block_items[b + 1] - block_items[b]);
        const int ivt = 512 - 48 * p->nblk - 2;   // the inverse's threads
        p->fold_direct = p->group_lanes == 32 && max_bi <= 8 && p->n_norm_chunks <= 4 && ivt > 0 &&
                         p->m * p->m <= 8 * ivt;
        if (const char* f = std::getenv("MCC_FOLD_DIRECT")) p->fold_direct = p->fold_direct && std::atoi(f) != 0;
        // MCC_FOLD_DYN=1: the groups themselves take the items, norm chunks and the final task by ticket
        // once their own work is done, instead of trailing workgroups that wait for a CU the groups free
        // (config5's 500-view shard: the trailing items started 1.5 us after the last group ended).
        // Measured, not the default: config4 26.55 vs 26.41 us per step, config5's shard 29.3 vs 29.5
        // (interleaved, gpurun_out/r05u) -- the last group's slots, not the items' start, set the tail.
        // With fold_dyn a finished group spins on slots of groups that may not have started, so the
        // whole grid must be resident at once: the groups and the spare within one workgroup per CU.
        const char* fd = std::getenv("MCC_FOLD_DYN");
        p->fold_dyn = fd && std::atoi(fd) != 0 && p->n_pgroups >= 2 * (p->n_items + p->n_norm_chunks + 1) &&
                      p->prism != 2 && p->n_pgroups + 1 <= n_cu_dev;
        if (p->fold_dyn) {
            HIPC(p->fold_ticket.alloc(1));
            HIPC(hipMemset(p->fold_ticket.p, 0, sizeof(int)));
        }
        for (auto* b : {&p->pairprod, &p->item_out, &p->fnorm, &p->fiv})
            if (b->p) HIPC(hipMemset(b->p, 0xFF, sizeof(double) * std::max<size_t>(b->n, 1)));
    }
    p->warm = !p->fused && p->m > 30;
    if (const char* f = std::getenv("MCC_WARM")) p->warm = p->warm && std::atoi(f) != 0;
    p->helper_refine = p->warm && p->m <= 96;   // (single GPU only: warm_ctx, enqueue_step; the warm path's M <= 96)
    if (const char* f = std::getenv("MCC_HELPER_REFINE")) p->helper_refine = p->helper_refine && std::atoi(f) != 0;
    p->helper_early = p->helper_refine && !p->use_group;
    if (const char* f = std::getenv("MCC_HELPER_POLL")) p->helper_early = p->helper_refine && std::atoi(f) != 0;
    p->inv_la = p->use_group;   // (mcc_kernels.hip gj_inverse_blocked: where the helper's cycle bounds the step)
    if (const char* f = std::getenv("MCC_INV_LA")) p->inv_la = std::atoi(f) != 0;
    if (const char* f = std::getenv("MCC_WARM_POISON")) p->warm_poison = std::atoi(f);
    if (const char* f = std::getenv("MCC_WARM_TIMEOUT_MS")) p->warm_wait_ticks = (long long)(std::max(1.0, std::atof(f)) * 1e5);
    if (const char* f = std::getenv("MCC_WARM_DELAY_US")) p->warm_delay_ticks = (long long)(std::max(0.0, std::atof(f)) * 1e2);
    if (const char* f = std::getenv("MCC_SPARE_DELAY_US")) p->spare_delay_ticks = (long long)(std::max(0.0, std::atof(f)) * 1e2);
    if (const char* f = std::getenv("MCC_SOLVE_STATS")) p->small_stats = std::atoi(f) != 0;
    if (const char* f = std::getenv("MCC_FAULT_PHOTO")) p->fault_photo = std::atoi(f);
    {
        double peer_ms = 30000.0;   // the helper outlives a k_solve's longest wait at a peer exchange
        if (const char* t = std::getenv("MCC_PEER_TIMEOUT_MS")) peer_ms = std::max(1.0, std::atof(t));
        p->warm_idle_ticks = p->warm_wait_ticks + (long long)(peer_ms * 1e5) + 100000000LL;
    }
    p->warm = p->warm && p->m <= 96;   // the staged system and inverse fit k_solve's LDS up to M = 96
    if (p->warm) {
        const size_t M = 16 * (size_t)((p->m + 15) / 16);
        HIPC(hipMalloc((void**)&p->sinv, M * M * sizeof(double)));   // cached: the helper releases it, k_solve reads it in a later launch
        p->prev_stride = (p->ntri + p->m + 1) & ~1;
        HIPC(hipExtMallocWithFlags((void**)&p->prev2, 2 * (size_t)p->prev_stride * sizeof(double), hipDeviceMallocUncached));
        if (int r = reset_prev2(p, true)) return bail(r);
        HIPC(hipExtMallocWithFlags((void**)&p->wsync, 8 * sizeof(unsigned), hipDeviceMallocUncached));
        HIPC(hipMemset(p->wsync, 0, 8 * sizeof(unsigned)));
        HIPC(hipExtMallocWithFlags((void**)&p->xsol, 128 * sizeof(double), hipDeviceMallocUncached));
        HIPC(hipMemset(p->xsol, 0, 128 * sizeof(double)));
        if (!p->warm_stats.p) HIPC(p->warm_stats.alloc(5));
        HIPC(hipMemset(p->warm_stats.p, 0, 5 * sizeof(long long)));
        HIPC(stream_pool().take(d->device, &p->side, true));
    }
#undef HIPC
    (void)rc;
    *out = p;
    return MCC_OK;
}

void mcc_destroy(mcc_problem* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    const bool side_drained = p->side && hipStreamSynchronize(p->side) == hipSuccess;
    const bool drained = p->stream && hipStreamSynchronize(p->stream) == hipSuccess;
    if (p->sinv) (void)hipFree(p->sinv);
    if (p->prev2) (void)hipFree(p->prev2);
    if (p->wsync) (void)hipFree(p->wsync);
    if (p->xsol) (void)hipFree(p->xsol);
    p->warm_stats.release();
    drop_graphs(p);
    p->xsave.release(); p->ysave.release(); p->zpsave.release();
    for (auto e : p->ev_lin) (void)hipEventDestroy(e);
    for (auto e : p->ev_step) (void)hipEventDestroy(e);
    for (auto e : p->ev_opt) if (e) (void)hipEventDestroy(e);
    for (auto e : p->ev_x) (void)hipEventDestroy(e);
    for (auto e : p->ev_marks) (void)hipEventDestroy(e);
    for (auto e : p->ev_win) if (e) (void)hipEventDestroy(e);
    if (p->comm) (void)ncclCommDestroy(p->comm);
    for (void* m : p->peer_mapped) (void)hipIpcCloseMemHandle(m);
    if (p->peers_dev) (void)hipFree(p->peers_dev);
    if (p->peer_scratch) (void)hipFree(p->peer_scratch);
    if (p->inbox) (void)hipFree(p->inbox);
    p->obj_x.release(); p->obj_y.release(); p->obj_z.release(); p->img_u.release(); p->img_v.release();
    p->x.release(); p->xerr.release(); p->K.release(); p->D.release(); p->xi.release(); p->cam_rt.release();
    p->cam_pose.release(); p->resid.release(); p->edge_sum.release(); p->corner_err.release(); p->stamps.release();
    p->contrib.release(); p->gsum.release(); p->cnt.release(); p->W.release();
    p->ds_rt.release(); p->Y.release(); p->pairprod.release(); p->zp.release();
    p->erec.release(); p->echain.release(); p->eh.release(); p->tilt.release(); p->fnorm.release(); p->fiv.release();
    p->fold_ticket.release(); p->ssinv.release(); p->ssinv_ok.release();
    p->gp_tot.release(); p->item_out.release(); p->packed.release(); p->dg.release(); p->delta.release();
    p->photo_norm.release(); p->alpha.release();
    p->photo_ptr.release(); p->photo_corner.release(); p->edge_gblock.release(); p->block_items.release(); p->counter.release(); p->cnt_blk.release();
    p->edge_photo.release(); p->edge_info.release(); p->items.release(); p->gpairs.release();
    p->prep_ptr.release(); p->prep_edge.release();
    p->pgrp_ptr.release(); p->pgrp_edge.release(); p->edge_lphoto.release(); p->gpair_ptr.release(); p->gcon_ptr.release(); p->gcon.release();
    p->state.release();
    if (p->h_state) (void)hipHostFree(p->h_state);
    if (p->h_x) (void)hipHostFree(p->h_x);
    if (drained) stream_pool().give(p->device, p->stream);   // a stream that faulted is not reused
    else if (p->stream) (void)hipStreamDestroy(p->stream);
    if (side_drained) stream_pool().give(p->device, p->side, true);
    else if (p->side) (void)hipStreamDestroy(p->side);
    delete p;
}

int mcc_set_params(mcc_problem* p, const float* x, int n) {
    if (!p || !x || n != p->P) return fail(MCC_EINVAL, "mcc_set_params: size mismatch");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(p->x.p, x, sizeof(float) * n, hipMemcpyHostToDevice));
    // new parameters start a new optimisation: iteration 0 (alpha = 0.95^1), no pending update
    int rc = set_state(p, 1, 0, 0, 0.0);
    if (rc) return rc;
    const int zero = 0;
    HIPCHK(hipMemcpy(&p->state.p->pending, &zero, sizeof(int), hipMemcpyHostToDevice));
    return MCC_OK;
}

int mcc_get_params(mcc_problem* p, float* x, int n) {
    if (!p || !x || n != p->P) return fail(MCC_EINVAL, "mcc_get_params: size mismatch");
    HIPCHK(hipSetDevice(p->device));
    int rc = flush_pending(p);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(x, p->x.p, sizeof(float) * n, hipMemcpyDeviceToHost));
    return MCC_OK;
}

int mcc_linearize_solve(mcc_problem* p, double* delta, double* jte) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipSetDevice(p->device));
    int rc = flush_pending(p);
    if (rc) return rc;
    if ((rc = set_state(p, 0, 0, 0, 0.0))) return rc;
    if ((rc = enqueue_step(p, 0, nullptr))) return rc;
    if ((rc = enqueue_backsub(p, 0))) return rc;
    if ((rc = read_state(p))) return rc;
    if ((rc = check_state_error(p))) return rc;
    if (delta) HIPCHK(hipMemcpy(delta, p->delta.p, sizeof(double) * p->P, hipMemcpyDeviceToHost));
    if (jte) {
        std::vector<double> pk(p->packed_len), gp(6 * (size_t)p->V);
        HIPCHK(hipMemcpy(pk.data(), p->packed.p, sizeof(double) * p->packed_len, hipMemcpyDeviceToHost));
        if (p->V) HIPCHK(hipMemcpy(gp.data(), p->gp_tot.p, sizeof(double) * 6 * p->V, hipMemcpyDeviceToHost));
        for (int i = 0; i < p->m; ++i) jte[i] = pk[p->ntri + p->m + i];
        for (int i = 0; i < 6 * p->V; ++i) jte[p->m + i] = gp[i];
    }
    return MCC_OK;
}

int mcc_optimize(mcc_problem* p, int crit_type, int max_count, double eps, float* x_inout, int* iters,
                 double* last_change) {
    if (!p || !x_inout) return fail(MCC_EINVAL, "null argument");
    if (crit_type < 1 || crit_type > 3) return fail(MCC_EINVAL, "crit_type must be 1, 2 or 3");
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    HIPCHK(hipSetDevice(p->device));
    int rc = begin_optimize(p, x_inout, crit_type, max_count, eps);
    if (rc) return rc;
    if (!p->ev_opt[0]) {
        HIPCHK(hipEventCreate(&p->ev_opt[0]));
        HIPCHK(hipEventCreate(&p->ev_opt[1]));
    }
    const auto t1 = clk::now();
    HIPCHK(hipEventRecord(p->ev_opt[0], p->stream));
    const long long cap = crit_type == MCC_CRIT_EPS ? 1000000LL : (long long)max_count + 1;
    long long launched = 0;
    int polls = 0;
    while (true) {
        const int chunk = mcc_problem::kGraphSteps;
        if ((rc = launch_update_steps(p, chunk))) return rc;
        HIPCHK(hipEventRecord(p->ev_opt[1], p->stream));
        launched += chunk;
        ++polls;
        if ((rc = read_state(p))) return rc;
        if ((rc = check_state_error(p))) return rc;
        if (p->h_state->done) break;
        if (launched > cap + chunk) return fail(MCC_EINVAL, "optimize did not terminate");
    }
    const auto t2 = clk::now();
    if (iters) *iters = p->h_state->iter;
    if (last_change) *last_change = p->h_state->change;
    p->opt_iters = p->h_state->iter;
    // the finish: the pending photo update flushed (the state was read by the last poll), the
    // parameters out -- one synchronisation
    if (p->h_state->pending) {
        if ((rc = enqueue_backsub(p, 1))) return rc;
        p->h_state->pending = 0;
        HIPCHK(hipMemsetAsync(&p->state.p->pending, 0, sizeof(int), p->stream));
    }
    HIPCHK(hipMemcpyAsync(p->h_x, p->x.p, sizeof(float) * p->P, hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    std::memcpy(x_inout, p->h_x, sizeof(float) * p->P);
    const auto t3 = clk::now();
    float dev = 0.f;
    if (hipEventElapsedTime(&dev, p->ev_opt[0], p->ev_opt[1]) != hipSuccess) dev = -1.f;
    p->opt_dev_ms = dev;
    p->opt_host_ms[0] = ms(t0, t1);
    p->opt_host_ms[1] = ms(t1, t2);
    p->opt_host_ms[2] = ms(t2, t3);
    p->opt_host_ms[3] = ms(t0, t3);
    p->opt_launched = (int)launched;
    p->opt_polls = polls;
    return rc;
}

int mcc_optimize_profile(mcc_problem* p, double* host_ms, double* device_ms, int* launched, int* iters,
                         int* polls) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    if (host_ms) std::memcpy(host_ms, p->opt_host_ms, sizeof(p->opt_host_ms));
    if (device_ms) *device_ms = p->opt_dev_ms;
    if (launched) *launched = p->opt_launched;
    if (iters) *iters = p->opt_iters;
    if (polls) *polls = p->opt_polls;
    return MCC_OK;
}

int mcc_step(mcc_problem* p, int n) {
    if (!p || n < 0) return fail(MCC_EINVAL, "bad argument");
    HIPCHK(hipSetDevice(p->device));
    // crit_type 0: every step updates (no stop test), iteration counter keeps running.  Only the
    // first call after another entry point touched the state syncs and rewrites it; back-to-back
    // calls just enqueue (no host round trip inside a timed window of steps)
    if (!p->stepping) {
        int rc = set_state(p, 0, 0, 0, 0.0);
        if (rc) return rc;
        p->stepping = true;
    }
    return launch_update_steps(p, n);
}

int mcc_synchronize(mcc_problem* p) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipStreamSynchronize(p->stream));
    return MCC_OK;
}

int mcc_check(mcc_problem* p) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipSetDevice(p->device));
    int rc = read_state(p);
    if (rc) return rc;
    rc = check_state_error(p);
    // a failed step left `done` set: the next mcc_step must rewrite the state (set_state), not
    // enqueue onto a stopped loop
    if (rc) p->stepping = false;
    return rc;
}

int mcc_project_error_detail(mcc_problem* p, const float* x, float* edge_err, float* corner_err, float* total_error,
                             long long* total_points, double* mean) {
    if (!p || !x) return fail(MCC_EINVAL, "null argument");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(p->xerr.p, x, sizeof(float) * p->P, hipMemcpyHostToDevice));
    if (corner_err && !p->corner_err.p) HIPCHK(p->corner_err.alloc(std::max<long long>(p->corners, 1)));
    mcc::ErrArgs a{p->edge_info.p, p->edge_photo.p, p->obj_x.p, p->obj_y.p, p->obj_z.p, p->img_u.p, p->img_v.p,
                   p->xerr.p, p->K.p, p->D.p, p->xi.p, p->tilt.p, p->cam_pose.p, p->edge_sum.p,
                   corner_err ? p->corner_err.p : nullptr, p->nd, p->m};
    if (p->E) HIPCHK(mcc_launch_project_error(a, p->model, p->E, p->rational, p->prism, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    std::vector<float> sums(p->E);
    if (p->E) HIPCHK(hipMemcpy(sums.data(), p->edge_sum.p, sizeof(float) * p->E, hipMemcpyDeviceToHost));
    if (corner_err && p->corners) {
        std::vector<float> ce(p->corners);
        HIPCHK(hipMemcpy(ce.data(), p->corner_err.p, sizeof(float) * p->corners, hipMemcpyDeviceToHost));
        for (long long c = 0; c < p->corners; ++c) corner_err[p->dev2ref_corner[c]] = ce[c];
    }
    std::vector<float> by_ref(p->E);
    std::vector<int> n_ref(p->E);
    for (int de = 0; de < p->E; ++de) {
        by_ref[p->dev2ref_edge[de]] = sums[de];
        n_ref[p->dev2ref_edge[de]] = p->edge_n_dev[de];
    }
    // totals in reference edge order, float32 (src/mymulticalib.cpp:913-923, hazard H6)
    float total = 0.f;
    long long npts = 0;
    for (int e = 0; e < p->E; ++e) {
        if (edge_err) edge_err[e] = by_ref[e] / n_ref[e];
        total += by_ref[e];
        npts += p->model == MCC_MODEL_OMNI ? n_ref[e] : 2LL * n_ref[e];   // error.total() (H2)
    }
    if (total_error) *total_error = total;
    if (total_points) *total_points = npts;
    if (mean) *mean = npts ? (double)total / (double)npts : 0.0;
    return MCC_OK;
}

int mcc_project_error(mcc_problem* p, const float* x, float* edge_err, double* mean) {
    return mcc_project_error_detail(p, x, edge_err, nullptr, nullptr, nullptr, mean);
}

int mcc_debug_solve(int device, int m, const double* packed, double* x, int reps, double* us_per_solve,
                    long long* stamps) {
    if (m <= 30 || m > 128 || !packed || !x) return fail(MCC_EINVAL, "mcc_debug_solve: 30 < m <= 128, non-null buffers");
    HIPCHK(hipSetDevice(device));
    const size_t n = (size_t)m * (m + 1) / 2 + (size_t)m;
    struct Bufs {
        double* pk = nullptr;
        double* xd = nullptr;
        int* err = nullptr;
        long long* st = nullptr;
        hipStream_t s = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        ~Bufs() {
            (void)hipFree(pk); (void)hipFree(xd); (void)hipFree(err); (void)hipFree(st);
            if (e0) (void)hipEventDestroy(e0);
            if (e1) (void)hipEventDestroy(e1);
            if (s) (void)hipStreamDestroy(s);
        }
    } b;
    HIPCHK(hipMalloc(&b.pk, n * sizeof(double)));
    HIPCHK(hipMalloc(&b.xd, (size_t)m * sizeof(double)));
    HIPCHK(hipMalloc(&b.err, sizeof(int)));
    HIPCHK(hipMalloc(&b.st, 64 * sizeof(long long)));
    HIPCHK(hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking));
    HIPCHK(hipMemcpy(b.pk, packed, n * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemset(b.err, 0, sizeof(int)));
    HIPCHK(hipMemset(b.st, 0, 64 * sizeof(long long)));
    HIPCHK(mcc_launch_debug_solve(b.pk, b.xd, m, b.err, stamps ? b.st : nullptr, b.s));
    HIPCHK(hipStreamSynchronize(b.s));
    int err = 0;
    HIPCHK(hipMemcpy(x, b.xd, (size_t)m * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&err, b.err, sizeof(int), hipMemcpyDeviceToHost));
    if (stamps) HIPCHK(hipMemcpy(stamps, b.st, 64 * sizeof(long long), hipMemcpyDeviceToHost));
    if (reps > 0 && us_per_solve) {
        HIPCHK(hipEventCreate(&b.e0));
        HIPCHK(hipEventCreate(&b.e1));
        HIPCHK(hipEventRecord(b.e0, b.s));
        for (int r = 0; r < reps; ++r) HIPCHK(mcc_launch_debug_solve(b.pk, b.xd, m, b.err, nullptr, b.s));
        HIPCHK(hipEventRecord(b.e1, b.s));
        HIPCHK(hipEventSynchronize(b.e1));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, b.e0, b.e1));
        *us_per_solve = 1e3 * (double)ms / reps;
    }
    return err ? fail(MCC_ENOTPD, "mcc_debug_solve: not positive definite") : MCC_OK;
}

int mcc_solve_stats(mcc_problem* p, long long* out) {
    if (!p || !out) return fail(MCC_EINVAL, "null argument");
    HIPCHK(hipSetDevice(p->device));
    std::memset(out, 0, 5 * sizeof(long long));
    if (!p->warm_stats.p) return MCC_OK;
    HIPCHK(hipStreamSynchronize(p->stream));
    if (p->side) HIPCHK(hipStreamSynchronize(p->side));
    HIPCHK(hipMemcpy(out, p->warm_stats.p, 5 * sizeof(long long), hipMemcpyDeviceToHost));
    return MCC_OK;
}

int mcc_debug_delays(mcc_problem* p, double spare_delay_us, double warm_delay_us, double warm_timeout_ms) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipStreamSynchronize(p->stream));
    if (p->side) HIPCHK(hipStreamSynchronize(p->side));
    if (spare_delay_us >= 0.0) p->spare_delay_ticks = (long long)(spare_delay_us * 1e2);
    if (warm_delay_us >= 0.0) p->warm_delay_ticks = (long long)(warm_delay_us * 1e2);
    if (warm_timeout_ms >= 0.0) {
        const long long w = (long long)(std::max(1.0, warm_timeout_ms) * 1e5);
        p->warm_idle_ticks += w - p->warm_wait_ticks;   // (the idle exit keeps its margin over the bound)
        p->warm_wait_ticks = w;
    }
    drop_graphs(p);   // (the delays and the bound are kernel arguments)
    return MCC_OK;
}

int mcc_debug_residuals(mcc_problem* p, const float* x, float* res) {
    if (!p || !x || !res) return fail(MCC_EINVAL, "null argument");
    int rc = mcc_set_params(p, x, p->P);
    if (rc) return rc;
    if (!p->resid.p) HIPCHK(p->resid.alloc(2 * (size_t)std::max<long long>(p->corners, 1)));
    if ((rc = set_state(p, 0, 0, 0, 0.0))) return rc;
    if ((rc = enqueue_step(p, 0, p->resid.p))) return rc;
    HIPCHK(hipStreamSynchronize(p->stream));
    std::vector<float> r(2 * (size_t)p->corners);
    if (p->corners) HIPCHK(hipMemcpy(r.data(), p->resid.p, sizeof(float) * r.size(), hipMemcpyDeviceToHost));
    for (long long c = 0; c < p->corners; ++c) {
        res[2 * p->dev2ref_corner[c]] = r[2 * c];
        res[2 * p->dev2ref_corner[c] + 1] = r[2 * c + 1];
    }
    return MCC_OK;
}

int mcc_debug_stamps(mcc_problem* p, long long* out, int n) {
#ifdef MCC_DIAG
    if (!p || !out) return fail(MCC_EINVAL, "null argument");
    HIPCHK(hipSetDevice(p->device));
    if (!p->stamps.p) {
        const size_t n_st = mcc::kStampStride * (size_t)std::max(p->V, 1) + mcc::kSchurStampStride * (size_t)(p->n_items + p->n_norm_chunks) + 16 + 64;   // (+ the helper's)
        HIPCHK(p->stamps.alloc(n_st));
        HIPCHK(hipMemset(p->stamps.p, 0, sizeof(long long) * n_st));
        HIPCHK(hipMemset(p->stamps.p + n_st - 64, 0xFF, sizeof(long long) * 64));   // the helper's: -1 until written
        drop_graphs(p);   // graphs captured the old pointer
        return MCC_OK;   // armed: the next steps record
    }
    HIPCHK(hipStreamSynchronize(p->stream));
    const int cnt = std::min(n, (int)p->stamps.n);
    HIPCHK(hipMemcpy(out, p->stamps.p, sizeof(long long) * cnt, hipMemcpyDeviceToHost));
    return MCC_OK;
#else
    (void)p; (void)out; (void)n;
    return fail(MCC_EINVAL, "mcc_debug_stamps needs the MCC_DIAG build (libmcc_diag.so)");
#endif
}

int mcc_timing_begin(mcc_problem* p) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipSetDevice(p->device));
    if (p->ev_lin.empty()) {
        p->ev_lin.resize(512);
        p->ev_step.resize(512);
        for (auto& e : p->ev_lin) HIPCHK(hipEventCreate(&e));
        for (auto& e : p->ev_step) HIPCHK(hipEventCreate(&e));
    }
    p->ev_used = 0;
    p->ev_x_used = 0;
    if (p->ev_x.empty()) {
        p->ev_x.resize(512);
        for (auto& e : p->ev_x) HIPCHK(hipEventCreate(&e));
    }
    {
        int rc = read_state(p);
        if (rc) return rc;
        p->xchg_ticks0 = p->h_state->xchg_ticks;
        p->xchg_epoch0 = p->h_state->epoch;
    }
    if (p->fused && (!p->comm || p->peer_on)) {   // one kernel per step: time the launch window itself (graphs stay on)
        if (!p->ev_win[0]) {
            HIPCHK(hipEventCreate(&p->ev_win[0]));
            HIPCHK(hipEventCreate(&p->ev_win[1]));
        }
        p->win_steps = 0;
        p->timing_window = true;
        HIPCHK(hipEventRecord(p->ev_win[0], p->stream));
        return MCC_OK;
    }
    p->timing = true;
    // the GPU busy for ~5 ms (s_memrealtime) while the host enqueues the window's steps (a window of
    // 100 split steps is ~600 API calls, ~2 ms)
    HIPCHK(mcc_launch_delay(500000LL, p->stream));
    return MCC_OK;
}

int mcc_timing_end(mcc_problem* p, double* lin_ms, double* step_ms, int* launches) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    if (p->timing_window) {
        HIPCHK(hipEventRecord(p->ev_win[1], p->stream));
        HIPCHK(hipEventSynchronize(p->ev_win[1]));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p->ev_win[0], p->ev_win[1]));
        p->timing_window = false;
        const double per = p->win_steps ? ms / (double)p->win_steps : 0.0;
        if (lin_ms) *lin_ms = per;
        if (step_ms) *step_ms = per;
        if (launches) *launches = (int)p->win_steps;
        return MCC_OK;
    }
    HIPCHK(hipStreamSynchronize(p->stream));
    double lin = 0, st = 0;
    const int n = p->ev_used / 2;
    for (int i = 0; i < n; ++i) {
        float a = 0, b = 0;
        HIPCHK(hipEventElapsedTime(&a, p->ev_lin[2 * i], p->ev_lin[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&b, p->ev_step[2 * i], p->ev_step[2 * i + 1]));
        lin += a;
        st += b;
    }
    p->timing = false;
    if (lin_ms) *lin_ms = n ? lin / n : 0.0;
    if (step_ms) *step_ms = n ? st / n : 0.0;
    if (launches) *launches = n;
    return MCC_OK;
}

int mcc_timing_windows(mcc_problem* p, int n_windows, int steps, double* ms_per_window, int* graph_launched) {
    if (!p || n_windows < 1 || steps < 1 || !ms_per_window) return fail(MCC_EINVAL, "bad timing-window arguments");
    HIPCHK(hipSetDevice(p->device));
    if (p->timing || p->timing_window) return fail(MCC_EINVAL, "mcc_timing_windows inside a timing window");
    if (!p->stepping) {
        int rc = set_state(p, 0, 0, 0, 0.0);
        if (rc) return rc;
        p->stepping = true;
    }
    if ((int)p->ev_marks.size() < n_windows + 2) {
        const size_t old = p->ev_marks.size();
        p->ev_marks.resize(n_windows + 2);
        for (size_t i = old; i < p->ev_marks.size(); ++i) HIPCHK(hipEventCreate(&p->ev_marks[i]));
    }
    // n_windows + 1 windows back to back, each bracketed by an event on the step stream, enqueued
    // before any wait: the GPU runs them without a gap, and the first one (which would include the
    // idle time before the first graph arrives) is dropped
    for (int w = 0; w <= n_windows; ++w) {
        HIPCHK(hipEventRecord(p->ev_marks[w], p->stream));
        int rc = launch_update_steps(p, steps);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(p->ev_marks[n_windows + 1], p->stream));
    HIPCHK(hipEventSynchronize(p->ev_marks[n_windows + 1]));
    for (int w = 1; w <= n_windows; ++w) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, p->ev_marks[w], p->ev_marks[w + 1]));
        ms_per_window[w - 1] = ms;
    }
    if (graph_launched) *graph_launched = p->use_graph ? 1 : 0;
    return MCC_OK;
}

int mcc_timing_linearize(mcc_problem* p, int launches, double* ms_per_launch) {
    if (!p || launches < 1 || !ms_per_launch) return fail(MCC_EINVAL, "bad arguments");
    HIPCHK(hipSetDevice(p->device));
    if (p->fused) return fail(MCC_EINVAL, "mcc_timing_linearize: the fused step is one kernel (mcc_timing_begin / end)");
    if (p->timing || p->timing_window) return fail(MCC_EINVAL, "mcc_timing_linearize inside a timing window");
    if (!p->stepping) {
        int rc = set_state(p, 0, 0, 0, 0.0);
        if (rc) return rc;
        p->stepping = true;
    }
    if (!p->lin_graph || p->lin_graph_n != launches) {
        if (p->lin_graph) { (void)hipGraphExecDestroy(p->lin_graph); p->lin_graph = nullptr; }
        hipGraph_t graph;
        HIPCHK(hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal));
        int rc = MCC_OK;
        for (int i = 0; i < launches && rc == MCC_OK; ++i) rc = enqueue_step(p, 1, nullptr, true);
        hipError_t ee = hipStreamEndCapture(p->stream, &graph);
        if (rc != MCC_OK) return rc;
        if (ee != hipSuccess) return fail(MCC_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ee));
        HIPCHK(hipGraphInstantiate(&p->lin_graph, graph, nullptr, nullptr, 0));
        HIPCHK(hipGraphDestroy(graph));
        p->lin_graph_n = launches;
    }
    if (!p->ev_win[0]) {
        HIPCHK(hipEventCreate(&p->ev_win[0]));
        HIPCHK(hipEventCreate(&p->ev_win[1]));
    }
    if (!p->xsave.p) HIPCHK(p->xsave.alloc(p->P));
    if (!p->ysave.p) HIPCHK(p->ysave.alloc(p->Y.n));
    if (!p->zpsave.p) HIPCHK(p->zpsave.alloc(p->zp.n));
    HIPCHK(hipMemcpyAsync(p->xsave.p, p->x.p, sizeof(float) * p->P, hipMemcpyDeviceToDevice, p->stream));
    HIPCHK(hipMemcpyAsync(p->ysave.p, p->Y.p, sizeof(double) * p->Y.n, hipMemcpyDeviceToDevice, p->stream));
    HIPCHK(hipMemcpyAsync(p->zpsave.p, p->zp.p, sizeof(double) * p->zp.n, hipMemcpyDeviceToDevice, p->stream));
    HIPCHK(hipEventRecord(p->ev_win[0], p->stream));
    HIPCHK(hipGraphLaunch(p->lin_graph, p->stream));
    HIPCHK(hipEventRecord(p->ev_win[1], p->stream));
    // the parameters and the pending update's operands as before the window (each launch re-applied
    // the pending photo update and rewrote Y', z'), so the next step continues the trajectory; the
    // state (pending, alpha, dg) is untouched by the linearisation kernels
    HIPCHK(hipMemcpyAsync(p->x.p, p->xsave.p, sizeof(float) * p->P, hipMemcpyDeviceToDevice, p->stream));
    HIPCHK(hipMemcpyAsync(p->Y.p, p->ysave.p, sizeof(double) * p->Y.n, hipMemcpyDeviceToDevice, p->stream));
    HIPCHK(hipMemcpyAsync(p->zp.p, p->zpsave.p, sizeof(double) * p->zp.n, hipMemcpyDeviceToDevice, p->stream));
    // the folded step's slots are empty between launches (LinArgs::fold): the probe's k_group alone
    // wrote them with nothing to consume them
    if (p->gfold) HIPCHK(hipMemsetAsync(p->pairprod.p, 0xFF, sizeof(double) * p->pairprod.n, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, p->ev_win[0], p->ev_win[1]));
    *ms_per_launch = ms / launches;
    return MCC_OK;
}

int mcc_timing_exchange(mcc_problem* p, double* ms_per_exchange, int* exchanges) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    HIPCHK(hipSetDevice(p->device));
    int rc = read_state(p);
    if (rc) return rc;
    double ms = 0.0;
    int n = 0;
    if (p->peer_on) {
        n = (int)(p->h_state->epoch - p->xchg_epoch0);
        ms = (double)(p->h_state->xchg_ticks - p->xchg_ticks0) * 1e-5;   // 100 MHz ticks -> ms
    } else {
        n = p->ev_x_used / 2;
        for (int i = 0; i < n; ++i) {
            float a = 0;
            HIPCHK(hipEventElapsedTime(&a, p->ev_x[2 * i], p->ev_x[2 * i + 1]));
            ms += a;
        }
    }
    if (ms_per_exchange) *ms_per_exchange = n ? ms / n : 0.0;
    if (exchanges) *exchanges = n;
    return MCC_OK;
}

int mcc_problem_path(const mcc_problem* p, int* split_step, int* photo_groups) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    if (split_step) *split_step = p->fused ? 0 : (p->use_group ? (p->gfold ? 3 : 2) : 1);
    if (photo_groups) *photo_groups = p->fused ? 0 : p->n_pgroups;
    return MCC_OK;
}

int mcc_problem_stats(const mcc_problem* p, long long* corners, long long* edges, long long* photos,
                      long long* alg_bytes) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    if (corners) *corners = p->corners;
    if (edges) *edges = p->E;
    if (photos) *photos = p->V;
    // 20 B per corner (float32 obj xyz + img uv) + 280 B per edge
    if (alg_bytes) *alg_bytes = 20LL * p->corners + 280LL * p->E;
    return MCC_OK;
}

// ---------------------------------------------------------------- multi-GPU
int mcc_comm_unique_id(unsigned char* id) {
    if (!id) return fail(MCC_EINVAL, "null id");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(MCC_ECOMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    static_assert(sizeof(u.internal) == MCC_UNIQUE_ID_BYTES, "nccl id size");
    std::memcpy(id, u.internal, MCC_UNIQUE_ID_BYTES);
    return MCC_OK;
}

int mcc_comm_init(mcc_problem* p, const unsigned char* id, int nranks, int rank) {
    if (!p || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(MCC_EINVAL, "bad comm arguments");
    HIPCHK(hipSetDevice(p->device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, MCC_UNIQUE_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&p->comm, nranks, u, rank);
    if (r != ncclSuccess) return fail(MCC_ECOMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    p->nranks = nranks;
    p->rank = rank;
    drop_graphs(p);
    return MCC_OK;
}

int mcc_comm_allreduce_max(mcc_problem* p, double* v) {
    if (!p || !v) return fail(MCC_EINVAL, "null argument");
    if (p->peer_n > 1 && (p->peer_on || !p->comm)) {   // over the peer transport
        HIPCHK(hipSetDevice(p->device));
        HIPCHK(hipMemcpyAsync(p->peer_scratch, v, sizeof(double), hipMemcpyHostToDevice, p->stream));
        HIPCHK(mcc_launch_peer_max(peer_ctx(p, true), p->state.p, p->peer_scratch, p->stream));
        HIPCHK(hipMemcpyAsync(v, p->peer_scratch, sizeof(double), hipMemcpyDeviceToHost, p->stream));
        int rc = read_state(p);
        if (rc) return rc;
        return check_state_error(p);
    }
    if (!p->comm || p->nranks == 1) return MCC_OK;
    HIPCHK(hipSetDevice(p->device));
    double* dv;
    HIPCHK(hipMalloc((void**)&dv, sizeof(double)));
    HIPCHK(hipMemcpy(dv, v, sizeof(double), hipMemcpyHostToDevice));
    ncclResult_t r = ncclAllReduce(dv, dv, 1, ncclDouble, ncclMax, p->comm, p->stream);
    if (r != ncclSuccess) { (void)hipFree(dv); return fail(MCC_ECOMM, ncclGetErrorString(r)); }
    HIPCHK(hipStreamSynchronize(p->stream));
    HIPCHK(hipMemcpy(v, dv, sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipFree(dv));
    return MCC_OK;
}

int mcc_comm_barrier(mcc_problem* p) {
    double v = 0.0;
    int rc = mcc_comm_allreduce_max(p, &v);
    if (rc) return rc;
    HIPCHK(hipDeviceSynchronize());
    return MCC_OK;
}

int mcc_peer_handle(mcc_problem* p, unsigned char* handle) {
    if (!p || !handle) return fail(MCC_EINVAL, "null argument");
    HIPCHK(hipSetDevice(p->device));
    if (!p->inbox) {
        const size_t words = (size_t)2 * mcc_problem::kPeerMaxRanks * 2 * (size_t)p->packed_len;
        HIPCHK(hipExtMallocWithFlags((void**)&p->inbox, words * sizeof(unsigned long long), hipDeviceMallocUncached));
        HIPCHK(hipMemset(p->inbox, 0, words * sizeof(unsigned long long)));   // epoch 0 is never sent
        HIPCHK(hipMalloc((void**)&p->peer_scratch, 4 * sizeof(double)));
        HIPCHK(hipDeviceSynchronize());
    }
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, p->inbox));
    static_assert(sizeof(h) == MCC_PEER_HANDLE_BYTES, "IPC handle size");
    std::memcpy(handle, &h, MCC_PEER_HANDLE_BYTES);
    return MCC_OK;
}

int mcc_peer_init(mcc_problem* p, const unsigned char* handles, int nranks, int rank) {
    if (!p || !handles || nranks < 1 || nranks > mcc_problem::kPeerMaxRanks || rank < 0 || rank >= nranks)
        return fail(MCC_EINVAL, "bad peer arguments");
    if (!p->inbox) return fail(MCC_EINVAL, "mcc_peer_handle must be called first");
    if (p->V == 0) return fail(MCC_EINVAL, "a rank of the peer transport needs photos");
    if (p->peer_n) return fail(MCC_EINVAL, "peer transport already initialised");
    if (p->comm && (p->rank != rank || p->nranks != nranks)) return fail(MCC_EINVAL, "rank differs from the RCCL one");
    HIPCHK(hipSetDevice(p->device));
    std::vector<unsigned long long*> ptrs(nranks, nullptr);
    for (int q = 0; q < nranks; ++q) {
        if (q == rank) { ptrs[q] = p->inbox; continue; }
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)q * MCC_PEER_HANDLE_BYTES, MCC_PEER_HANDLE_BYTES);
        void* m = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&m, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(MCC_ECOMM, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
        p->peer_mapped.push_back(m);
        ptrs[q] = (unsigned long long*)m;
    }
    if (!p->peers_dev) HIPCHK(hipMalloc((void**)&p->peers_dev, mcc_problem::kPeerMaxRanks * sizeof(void*)));
    HIPCHK(hipMemcpy(p->peers_dev, ptrs.data(), nranks * sizeof(void*), hipMemcpyHostToDevice));
    double ms = 30000.0;
    if (const char* t = std::getenv("MCC_PEER_TIMEOUT_MS")) ms = std::max(1.0, std::atof(t));
    p->peer_timeout = (long long)(ms * 1e5);   // s_memrealtime: 100 MHz
    p->peer_n = nranks;
    p->rank = rank;
    p->nranks = nranks;
    HIPCHK(mcc_launch_peer_handshake(peer_ctx(p, true), p->state.p, p->peer_scratch, p->stream));
    double out[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(out, p->peer_scratch, sizeof(out), hipMemcpyDeviceToHost, p->stream));
    HIPCHK(hipStreamSynchronize(p->stream));
    if (out[0] != 1.0) {
        p->peer_n = 0;
        return fail(MCC_ECOMM, "peer handshake failed: mismatches " + std::to_string((long long)out[1]) +
                                   ", round-1 timeout " + std::to_string((int)out[2]) + ", round-2 timeout " +
                                   std::to_string((int)out[3]));
    }
    p->peer_on = true;
    drop_graphs(p);
    return MCC_OK;
}

int mcc_peer_enable(mcc_problem* p, int on) {
    if (!p) return fail(MCC_EINVAL, "null problem");
    if (on && !p->peer_n) return fail(MCC_EINVAL, "peer transport not initialised");
    if (!on && !p->comm && p->peer_n > 1) return fail(MCC_EINVAL, "no RCCL communicator to fall back to");
    if (p->peer_on != (on != 0)) {
        HIPCHK(hipStreamSynchronize(p->stream));
        drop_graphs(p);
    }
    p->peer_on = on != 0;
    return MCC_OK;
}

int mcc_partition_photos(int n_photos, int n_edges, const int* edge_photo, const int* edge_n, int nranks,
                         int* rank_of_photo) {
    if (n_photos < 0 || nranks < 1 || !rank_of_photo || (n_edges && (!edge_photo || !edge_n)))
        return fail(MCC_EINVAL, "bad partition arguments");
    std::vector<long long> w(n_photos, 0);
    for (int e = 0; e < n_edges; ++e) {
        if (edge_photo[e] < 0 || edge_photo[e] >= n_photos) return fail(MCC_EINVAL, "edge_photo out of range");
        w[edge_photo[e]] += edge_n[e];
    }
    std::vector<int> ord(n_photos);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return w[a] > w[b]; });
    std::vector<long long> load(nranks, 0);
    for (int v : ord) {
        int best = 0;
        for (int r = 1; r < nranks; ++r)
            if (load[r] < load[best]) best = r;
        rank_of_photo[v] = best;
        load[best] += w[v];
    }
    return MCC_OK;
}

}  // extern "C"
