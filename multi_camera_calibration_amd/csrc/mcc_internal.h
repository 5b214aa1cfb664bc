// mcc_internal.h -- device state and kernel argument blocks shared by mcc_kernels.hip and
// mcc_api.cpp.  Not part of the public ABI (include/mcc.h).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mcc.h"

namespace mcc {

constexpr int kStampStride = 32;   // MCC_DIAG: s_memtime / s_memrealtime slots per k_linearize workgroup
constexpr int kSchurStampStride = 16;   // MCC_DIAG: slots per k_schur workgroup (after k_linearize's rows)

// Device-resident loop state of optimizeExtrinsics (src/multicalib.cpp:468-507).
struct State {
    int iter;         // completed updates k
    int done;         // stop test fired
    int crit_type;    // 0 = never stop (bench / linearize-only), 1 COUNT, 2 EPS, 3 COUNT+EPS
    int max_count;
    double eps;
    double change;    // ||G|| / ||x|| of the last update
    double alpha;     // 0.95^(k+1) of the running step
    double cam_normG2, cam_normX2;   // global-block partials of the last update
    int error;        // kErr* bits below
    int pending;      // a solved photo update waits to be applied by the next k_linearize
    unsigned int epoch;   // peer exchanges completed (monotonic over the problem's life)
    long long xchg_ticks; // s_memrealtime ticks (100 MHz) inside peer exchanges, summed (monotonic)
    // the fused step's m <= 30 warm solve (k_linearize's spare workgroup, small_inverse): the spare's
    // acknowledgement of an update launch -- iter + 1 once it holds the launch's inputs (state words,
    // the packed system) in LDS; the launch's final arriver writes neither the packed system nor the
    // state before it has seen it.  Update launches of one optimisation have distinct iter, and
    // set_state clears the word (no launch in flight), so an acknowledgement is never a stale one.
    unsigned int spare_ack;
};
// State::error bits
constexpr int kErrPhotoNotPD = 1;    // a photo's 6 x 6 block (any rank: summed through the exchange)
constexpr int kErrCameraNotPD = 2;   // the reduced camera system
constexpr int kErrPeerTimeout = 4;   // a peer did not deliver its system
constexpr int kErrWarmTimeout = 8;   // the warm-solve helper did not deliver the previous inverse, or
                                     // the fused step's spare did not acknowledge its inputs

// Peer transport (multi-GPU without RCCL in the step): every rank's final arriver writes its packed
// reduced system straight into every peer's inbox over xGMI, then sums all ranks' systems in rank
// order.  LL format (the RCCL low-latency protocol's idea): each 8-B word carries 32 data bits and
// the 32-bit epoch of the exchange, so a reader needs no cross-device ordering or fence, only the
// 8-B single-copy atomicity of an aligned store.  Inbox: [2 slots (epoch parity)][nranks][2 Lc]
// words in uncached device memory; peers[q] is rank q's inbox mapped into this process (IPC).
struct PeerCtx {
    unsigned long long* inbox;
    unsigned long long* const* peers;   // [nranks] device array (peers[rank] == inbox)
    int nranks;                         // 0: transport off
    int rank, Lc;
    long long timeout;                  // s_memrealtime ticks (100 MHz)
};

struct SolveCtx {
    State* state;
    const double* alpha; int n_alpha;
    float* x;
    double* dg;       // [m]
    double* delta;    // [P]
    int m, do_update;
    long long* stamps;   // MCC_DIAG: solve phase stamps (set by k_schur's last arriver)
    // m <= 30 warm-solve statistics (mcc_solve_stats, the m > 30 helper's layout): refinements tried,
    // corrections, refinements that fell back to the elimination, eliminations without an inverse,
    // fused steps whose final arriver waited for the spare.  Null unless MCC_SOLVE_STATS=1: the
    // counters' atomics at the end of the solving workgroup cost ~0.5 us per config2 step
    long long* sstats;
};

struct SchurArgs {
    State* state;
    const int4* items;   // {camera-pair block, first slot's offset in doubles, slot count, slot size 48 | 36}
    const double* pairprod;   // 48 (diagonal block) or 36 doubles per slot, written by k_photo, block-major
    double* item_out;    // [48 * (items + norm chunks)]
    int n_items;
    const double* photo_norm; int n_photos;
    int* counter;        // level-2 ticket over blocks + norm chunks (zero between launches)
    int* cnt_blk;        // [nblk] level-1 tickets: the last item of a camera-pair block sums it
    int nblk;
    const int* block_items;   // [nblk + 1]
    double* packed;
    int m, rank, fuse_solve;
    int one_level;       // m <= 30: one hand-off level (schur_one_level) instead of items -> blocks -> norms
    const double* ssinv; // m <= 30 warm solve: [2][m x m], this step's in buffer iteration & 1 (k_group's spare)
    const int* ssinv_ok; // [2] tags (iteration + 1)
    SolveCtx solve;
    long long* stamps;   // MCC_DIAG builds: [8 * grid]
    PeerCtx peer;        // nranks > 0 (m <= 30, peer transport): the final arriver exchanges, then solves
    double* prev2;       // m > 30 warm solve: [2][prev_stride] copy of [S | r] for the helper (null: off)
    int prev_stride;
    unsigned* wpub;      // m > 30, the helper refines (WarmCtx::refine): k_schur publishes the system
                         // (sync[0] = iteration + 1) when it starts and empties the other prev2 buffer
    int wpub_early;      // (the helper polls prev2's words as they land: the three-kernel step), or with 0
                         // its final arriver once prev2 is complete (k_group's step: mcc_create)
};

struct LinArgs {
    State* state;
    const int* photo_ptr;     // [V+1] photo-major edge ranges
    const int* photo_corner;  // [V+1] photo-major corner ranges (corners of a photo are contiguous)
    int max_cpp;              // most corners of one photo (LDS staging)
    const int4* edge_info;    // [E] {cam, side, corner_off, n}
    const float* obj_x; const float* obj_y; const float* obj_z;   // [corners] photo-major
    const float* img_u; const float* img_v;
    float* x;                 // [P] float32 parameters [global m | photos] (photo part updated in place)
    const float* K; const float* D; const float* xi;
    const double* tilt;       // [C][9] the tilted-sensor matTilt (nd = 14, tau != 0; null otherwise)
    const float* cam_rt;      // DOUBLESIDE fixed cameras (rvec, tvec) [6C]
    const double* ds_rt;      // PINHOLE doubleSideTransform (rvec, tvec) [6]
    int nd, global_dim, n_cams, has_back;
    // outputs
    double* Y;        // [36E] Schur factors Y'_e = Hgp_e Hpp^-1
    // split step: k_photo runs over groups of consecutive photos (<= kPhotoGroup photos and
    // <= kPhotoGroupEdges edges); each group sums its photos' Schur pair products per camera-pair
    // block and writes them at that block's slot (block-major over the groups; k_schur sums them)
    const int* pgrp_ptr;     // [n_pgroups + 1] first photo of each group
    const int* pgrp_edge;    // [n_pgroups + 1] first edge of each group (photo_ptr[pgrp_ptr[g]])
    const unsigned char* edge_lphoto;   // [E] an edge's photo within its group (0 .. kPhotoGroup - 1)
    const int* gpair_ptr;    // [n_pgroups + 1] ranges of gpairs
    const int4* gpairs;      // {first contribution (group-relative), count, diagonal block << 1, slot offset}
    const int* gcon_ptr;     // [n_pgroups + 1] ranges of gcon
    const unsigned* gcon;    // contribution: edge a | edge b << 8 | self << 16 | photo << 17 (group-local)
    double* pairprod;        // per slot {S_ab entries (36), [diagonal block] r_a (6), JTE_a (6)}
    int n_pgroups, max_gpairs, max_gcon, max_gedges;
    double* zp;       // [6V] z' = Hpp^-1 gp
    double* gp_tot;   // [6V] photo JTE
    float* resid;     // optional [2*corners] float32 residuals (debug)
    // pending update of the previous step (fused back-substitution)
    const int* gblock;       // [E] global block of an edge or -1
    const double* dg;        // [m] global-block delta of the previous solve
    double* photo_norm;      // [2V] ||G||^2, ||x||^2 partials of the applied update
    long long* stamps;       // MCC_DIAG builds: [16V] s_memtime per phase
    // fused single-kernel step (m <= 30): every photo writes its packed contribution
    // [S upper | r | jte_g | normG2 | normX2], a fixed-order two-level last-arriver reduction sums
    // them (groups of group_size consecutive photos, then the groups), and the final arriver
    // solves (fuse_solve) or leaves the packed system for the all-reduce + k_solve
    int fused, group_size, n_groups, rank, fuse_solve;
    double* contrib;         // [V * Lc]
    double* gsum;            // [n_groups * Lc]
    int* cnt;                // [n_groups + 1] tickets, zero between launches
    double* packed;          // [Lc]
    double* W;               // [V * 6m] per-photo pending-update matrix (next step's phase 0)
    SolveCtx solve;
    PeerCtx peer;            // nranks > 0: the final arriver exchanges with the peers and solves
    // split step (m > 30): k_prep -> k_edge -> k_photo
    int n_edges, n_photos;
    double* erec;            // [12E] R (9), T (3) of the float32 composed pose (k_prep -> k_edge)
    double* echain;          // [54E] chain-map blocks Gp11, Gp21, Gp22, Gg11, Gg21, Gg22 (k_prep -> k_edge)
    double* eh;              // [90E] Hpp upper (21), Hgg upper (21), Hgp (36), gp (6), gg (6) (k_edge -> k_photo)
    // k_prep4: groups of consecutive photos (<= kPrepPhotos photos and kPrepEdges edges, or one photo)
    const int* prep_ptr;     // [n_prep + 1] first photo of each group
    const int* prep_edge;    // [n_prep + 1] first edge of each group
    int n_prep, prep_lanes;  // prep_lanes: 4 (k_prep4) or 1 (k_prep, one lane per edge)
    int fault_photo;         // test (MCC_FAULT_PHOTO): this local photo's 6 x 6 block is reported not
                             // positive definite (its factor stays finite); -1 off
    // m <= 30 warm solve: k_group's spare workgroup inverts the previous step's packed system
    int fold_first;          // test layout (MCC_FOLD_CONSUMERS_FIRST=1): the spare and the folded reduction's
                             // workgroups take the LOWEST grid indices, the groups the rest -- the
                             // progress invariant must not rest on dispatch order (mcc_create); (placed
                             // in fault_photo's padding: a shifted LinArgs tail cost k_group SGPR spills)
    double* ssinv;           // [2][m x m] by iteration parity (null: off)
    int* ssinv_ok;           // [2] the iteration + 1 whose spare workgroup formed the buffer (0: none)
    // the fused step's spare: its wait bound at the final arriver (s_memrealtime ticks; past it the
    // step fails with kErrWarmTimeout), and a test delay before it reads anything (MCC_SPARE_DELAY_US)
    long long spare_wait, spare_delay;
    // k_group with the step's reduction and solve folded into the same launch (gfold: m <= 30, one
    // hand-off level): after the groups (and the spare) the grid holds fsa.n_items item workgroups,
    // the norm chunks (fold_parts in all) and one final workgroup.  The hand-off words are their own
    // flags: every slot, norm partial, item partial and the spare's inverse holds kFoldEmpty (all-ones,
    // a NaN no arithmetic produces) until its producer's sc1 store lands, and its consumer puts
    // kFoldEmpty back after reading it -- no store drain, ticket or fence on either side.
    int fold, fold_parts;
    int fold_direct;          // the final workgroup sums where the words land (fold_final_direct)
    int fold_dyn;             // the groups take the reduction's tasks by ticket as they finish (no
                              // trailing workgroups: those waited for a CU until the groups ended)
    int* fold_ticket;         // fold_dyn: the tasks' ticket (the last of the n_pgroups takers resets it)
    SchurArgs fsa;            // the reduction (k_schur's arguments: items, slots, partials, packed, solve)
    double* fnorm;            // [4V] per photo ||G||^2, ||x||^2, not-PD flag, pad (the norm chunks' input)
    double* fiv;              // [m^2 + 1] the spare's inverse and its status, +-(iteration + 1) as a double
};
constexpr long long kFoldEmpty = -1LL;

constexpr int kItemSingle = 256;   // k_schur item flag (in .w, over the slot size): the block's only item
constexpr int kPhotoGroup = 8;        // photos per k_photo workgroup, at most
constexpr int kPhotoGroupEdges = 64;  // edges per k_photo workgroup, at most
constexpr int kGroupRound = 16;       // edges per k_group round (4 waves x 4 edges x 16 lanes); its groups' cap
// k_photo's LDS (doubles, then ints): per edge [Hgg upper 21 | pad | U 36 | gg 6] (64), per photo the
// Hpp / gp sums [28], Hpp's inverse Cholesky factor Li [36] and v [6]; then per edge gblock and
// photo (ints), the group's pairs (int4) and contributions (unsigned)
__host__ __device__ inline size_t photo_lds_doubles(int gne) {
    return (size_t)64 * gne + (size_t)70 * kPhotoGroup;
}
__host__ __device__ inline size_t photo_lds_bytes(int gne, int npairs, int ncon) {
    return photo_lds_doubles(gne) * 8 + 4 * (size_t)((2 * gne + 3) & ~3) + 16 * (size_t)npairs + 4 * (size_t)ncon;
}

// k_group (mcc_group.hpp): the fused split step's per-group LDS
constexpr int kGChunk = 96;       // corners of one edge staged in LDS at a time
constexpr int kGIntr = 28;        // k_group's LDS intrinsics row: fx fy cx cy skew xi k[12] matTilt[9] pad
constexpr int kGRecP = 40;        // k_group's per-edge sweep record: R 9 | T 3 | 6 intrinsics | k[12] | matTilt[9] | pad
constexpr int kGRec = 92;         // doubles per group edge: sE (64: Hgg upper 21 | pad | U 36 | gg 6)
                                  // + Hpp upper 21 | gp 6 | pad; the edge's prologue scratch meanwhile

// LDS layout of k_group (offsets in doubles; host and device share it)
struct GroupLayout {
    int rec, s27, sLi, sv, sph, sxn, spart, sdg, ctab, ktab, sds, sP, sGb, sU, ndoubles;
    int iInfo, iGb, iEq, iPh, iPq, iCn, nints;   // int offsets after the doubles
};
__host__ __device__ inline GroupLayout group_layout(int gne, int C, int nq, int nc) {
    GroupLayout L;
    L.rec = 0;
    L.s27 = L.rec + kGRec * gne;                // [8][28] per-photo Hpp upper 21 | gp 6 sums
    L.sLi = L.s27 + 28 * kPhotoGroup;           // [8][36] Li = L^-1 (Hpp = L L^T)
    L.sv = L.sLi + 36 * kPhotoGroup;            // [8][6]  v = Li gp
    L.sph = L.sv + 6 * kPhotoGroup;             // [8][24] R1 | Jr1 | T1 of the updated photo
    L.sxn = L.sph + 24 * kPhotoGroup;           // [8][16] x (6) | pad | G (6) | pad
    L.spart = L.sxn + 16 * kPhotoGroup;         // [gne][6] Y'_e^T dg partials of the photo update
    L.sdg = L.spart + 6 * gne;                  // [128] the previous solve's global-block delta
    L.ctab = L.sdg + 128;                       // [C][24] camera R | Jl | T
    L.ktab = L.ctab + 24 * C;                   // [C][kGIntr] fx fy cx cy skew xi k[12] matTilt[9]
    L.sds = L.ktab + kGIntr * C;                // [32] double-side transform Rds | Jrds | dst
    L.sP = L.sds + 32;                          // [16][kGRecP] sweep record: R | T | fx fy cx cy skew xi | k[12] | matTilt[9]
    L.sGb = L.sP + kGRecP * kGroupRound;        // [16][56] chain-map blocks [photo 27 | pad | global 27 | pad]
    L.sU = L.sGb + 56 * kGroupRound;            // per wave: corners [5][96][4] floats | chain {A 36, B 8, X 96} x 4
    L.ndoubles = L.sU + 4 * (5 * kGChunk * 4 / 2);
    L.ndoubles = (L.ndoubles + 1) & ~1;         // 16-B aligned int4 area
    L.iInfo = 0;                                // int4 [gne] {cam, side, corner offset, n}
    L.iGb = L.iInfo + 4 * gne;                  // [gne] global block
    L.iEq = L.iGb + gne;                        // [gne] group-local photo
    L.iPh = L.iEq + gne;                        // [kPhotoGroup + 1] group-relative first edge of each photo
    L.iPq = (L.iPh + kPhotoGroup + 1 + 3) & ~3; // int4 [nq] pair tasks
    L.iCn = L.iPq + 4 * nq;                     // [nc] contributions
    L.nints = L.iCn + nc;
    return L;
}
__host__ __device__ inline size_t group_lds_bytes(int gne, int C, int nq, int nc) {
    const GroupLayout L = group_layout(gne, C, nq, nc);
    return (size_t)L.ndoubles * 8 + (size_t)L.nints * 4;
}

// k_prep4 (mcc_group.hpp): one wave per group of consecutive photos, 4 lanes per edge prologue
constexpr int kPrepEdges = 16;            // edges per round (64 lanes / 4); the groups' edge cap
constexpr int kPrepPhotos = kPhotoGroup;  // photos per group, at most
struct PrepLayout {
    int tab, S, sdg, sxn, scam, ndoubles;   // doubles
    int iInfo, iGb, iPh, nints;             // ints after the doubles
};
// tab: Rodrigues tables (R 9, J 9, T 3, pad) of the photos [kPrepPhotos], cameras [C] and the
// double-side transform; S: per edge slot the prologue's scratch (84 doubles with back-side
// edges, else 42), aliased by the photo update's partial sums (<= 64 edges x 6)
__host__ __device__ inline PrepLayout prep_layout(int C, bool back) {
    PrepLayout L;
    int o = 0;
    L.tab = o; o += 24 * (kPrepPhotos + C + 1);
    L.S = o; o += kPrepEdges * (back ? 84 : 42);
    L.sdg = o; o += 128;
    L.sxn = o; o += 16 * kPrepPhotos;
    L.scam = o; o += 6 * C + 6;
    L.ndoubles = (o + 1) & ~1;
    int n = 0;
    L.iInfo = n; n += 4 * 64;
    L.iGb = n; n += 64;
    L.iPh = n; n += kPrepPhotos + 1;
    L.nints = n;
    return L;
}
__host__ __device__ inline size_t prep_lds_bytes(int C, bool back) {
    const PrepLayout L = prep_layout(C, back);
    return (size_t)L.ndoubles * 8 + (size_t)L.nints * 4;
}

// k_schur's dynamic LDS (doubles): the final arriver's S (m x m) and r (m) when the launch solves
// (fuse_solve), the m <= 30 warm solve's inverse (m x m, ssinv), and with one hand-off level the copy
// of every workgroup's partials (48 per item or norm chunk, grid) followed by the block ranges (nblk + 1
// ints) -- all of them loaded in one round trip
__host__ __device__ inline size_t schur_items_offset(int m, int fuse, int ssinv) {
    return fuse ? (size_t)m * m + m + (ssinv ? (size_t)m * m : 0) : 0;
}
__host__ __device__ inline size_t schur_lds_bytes(int m, int fuse, int ssinv, int one_level, int grid, int nblk) {
    size_t d = schur_items_offset(m, fuse, ssinv);
    if (one_level) d += 48 * (size_t)grid + (nblk + 2) / 2;
    return d * sizeof(double);
}
// one hand-off level only while the final arriver's copy is one batch of loads: 48 grid + m^2 <=
// kSchurOneLevelLoads x 256 (k_schur's threads)
constexpr int kSchurOneLevelLoads = 16;



// The m > 30 solve with the previous step's inverse (the "warm" solve, solve_large in
// mcc_kernels.hip): a resident helper kernel on a side stream (k_sinv_helper) inverts each update
// step's reduced system while the next step linearises; the next k_solve solves its own system by
// iterative refinement preconditioned with that inverse and falls back to the direct elimination
// when the refinement does not converge within kWarmMaxIters corrections.  sinv_ok_sys, sprev and
// sync are uncached device memory (the helper and the k_solve launches hand them over while both
// run); sinv is ordinary memory, written back by the helper (agent release) before its epoch.
// The system itself reaches the helper through prev2: k_schur writes [S | r] to prev2[iter & 1] beside
// the packed system (one more write-through store per entry, spread over the block workgroups), and
// k_solve publishes the epoch e + 1 (iteration e solved) as soon as it holds S_t^-1 in LDS -- no copy
// or store drain of its own.  The double buffer is safe: the step that writes prev2[iter & 1] again
// starts after the next k_solve, which waited for the helper to invert (and so to read) this one.
// Which algorithm a step takes depends only on the systems (the epoch count, the helper's PD flag,
// the refinement's convergence), never on timing: k_solve always waits for the previous system's
// inverse, and a helper that does not deliver within wait_ticks fails the step (error bit 3,
// MCC_ETIMEOUT) instead of switching to the direct elimination.
struct WarmCtx {
    double* sinv;            // [M x M] (M = 16 ceil(m / 16), row-major) the helper's inverse
    int* sinv_ok_sys;        // the helper's elimination found the system positive definite
    double* prev2;           // [2][prev_stride] uncached: the copy of [S | r] per iteration parity
    int prev_stride;         // packed [S | r] rounded up to even
    int copy_prev;           // 1: k_solve writes the copy (sharded: the rank-summed system exists only
                             // after the exchange); 0: k_schur wrote it (single GPU)
    unsigned* sync;          // [8] epochs: systems published (k_solve; refine: k_schur), systems inverted by the
                             // helper; stop; PD; refine: the epoch the helper refined, its status (0 no
                             // inverse, 1 converged, 2 not), its corrections
    long long* stats;        // [5] warm solves, corrections, fallbacks, direct (no inverse yet), waited for the helper
    int poison;              // test (MCC_WARM_POISON=1): the helper publishes a NaN inverse, so every
                             // warm solve must fall back to the direct elimination
    long long wait_ticks;    // k_solve's bound on the wait for the helper (s_memrealtime, 100 MHz)
    long long idle_ticks;    // the helper exits after this long without a new system (a safety net: the
                             // batch's k_solves publish or raise the stop flag, and the host launches the
                             // helper only after the batch's graphs exist)
    long long delay_ticks;   // test (MCC_WARM_DELAY_US): the helper holds each inverse back this long
    int refine;              // single GPU (MCC_HELPER_REFINE): the helper refines with the inverse it holds in
                             // LDS and publishes x (xsol); k_solve only waits for it (or eliminates)
    double* xsol;            // refine: [kWarmN] uncached, the helper's solution of the published system
    int poll;                // refine: k_schur publishes at its start and the helper polls prev2's words
                             // (SchurArgs::wpub_early), else one batch once the system is complete
    long long* hst;          // MCC_DIAG builds: the helper's phase stamps, [4 systems][16] (null otherwise)
    int inv_la;              // the helper inverts with the look-ahead schedule (gj_inverse_blocked<true>)
};
constexpr int kWarmMaxIters = 4;

struct SolveArgs {
    SolveCtx ctx;
    double* packed;
    PeerCtx peer;            // nranks > 0: exchange the packed system with the peers first
    int pushed;              // k_peer_push already sent this rank's system (k_solve only receives)
    WarmCtx warm;            // m > 30: sync == null -> the direct elimination
};

struct BacksubArgs {
    const State* state;
    const int* photo_ptr;
    const int* gblock;
    const double* Y; const double* zp; const double* dg;
    const double* W;         // fused path: per-photo pending-update matrix (else nullptr: Y)
    float* x;
    double* delta;
    double* photo_norm;
    int n_photos, m, do_update;
};

struct ErrArgs {
    const int4* edge_info;
    const int* edge_photo;
    const float* obj_x; const float* obj_y; const float* obj_z;
    const float* img_u; const float* img_v;
    const float* x;
    const float* K; const float* D; const float* xi;
    const double* tilt;      // [C][9] matTilt (null: no tilt)
    const float* cam_pose;   // DOUBLESIDE [16C]
    float* edge_sum;         // [E] device order
    float* corner_err;       // optional [corners] device order: each corner's float32 L2 error
    int nd, m;
};

}  // namespace mcc

// launch wrappers (mcc_kernels.hip)
size_t mcc_lin_shmem(int max_edges_per_photo, int n_cams, int m, int max_cpp);
size_t mcc_solve_shmem(int m);
hipError_t mcc_set_kernel_attrs(int max_epp, int n_cams, int m, int max_cpp, size_t photo_shmem, size_t group_shmem);
hipError_t mcc_launch_group(const mcc::LinArgs& a, int model, bool rational, int prism, int lanes,
                            size_t group_shmem, hipStream_t s);
hipError_t mcc_launch_split(const mcc::LinArgs& a, int model, bool rational, int prism, size_t photo_shmem,
                            hipStream_t s);
hipError_t mcc_launch_linearize(const mcc::LinArgs& a, int model, int n_photos, int max_epp, bool rational, int prism, hipStream_t s);
hipError_t mcc_launch_schur(const mcc::SchurArgs& a, int grid, hipStream_t s);
hipError_t mcc_launch_solve(const mcc::SolveArgs& a, hipStream_t s);
hipError_t mcc_launch_peer_push(const mcc::PeerCtx& pc, const mcc::State* st, const double* vals, hipStream_t s);
hipError_t mcc_launch_debug_solve(const double* packed, double* x, int m, int* err, long long* stamps, hipStream_t s);
hipError_t mcc_launch_sinv_helper(const mcc::WarmCtx& w, int m, int n_systems, hipStream_t s);
hipError_t mcc_launch_backsub(const mcc::BacksubArgs& a, hipStream_t s);
hipError_t mcc_launch_delay(long long ticks, hipStream_t s);
hipError_t mcc_launch_peer_handshake(const mcc::PeerCtx& pc, mcc::State* st, double* out, hipStream_t s);
hipError_t mcc_launch_peer_max(const mcc::PeerCtx& pc, mcc::State* st, double* v, hipStream_t s);
hipError_t mcc_launch_project_error(const mcc::ErrArgs& a, int model, int n_edges, bool rational, int prism, hipStream_t s);
