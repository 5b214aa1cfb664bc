// mcc_group.hpp -- the fused split step k_group (included by mcc_kernels.hip, namespace mcc).
//
// One 256-thread workgroup per group of consecutive photo vertices (host-built: at most kPhotoGroup
// photos and kGroupRound edges, or one photo with more edges), doing in ONE launch what k_prep,
// k_edge and k_photo do in three (src/mymulticalib.cpp:468-614, 668-818; src/multicalib.cpp:593-824;
// src/doubleSide.cpp:288-581):
//   phase 0  loads of the group (one round trip: edge records, Schur pair lists, the previous step's
//            Y', z', dg, the cameras, the first round's corners); the pending photo update
//            x = fl32(x + fl32(alpha (z' - sum_e Y'_e^T dg))) (k_prep's, group-cooperative), the
//            cameras' Rodrigues tables (one lane per camera), the photos' Rodrigues (one lane per
//            photo);
//   phase A  per round of 16 edges (4 waves x 4 edges x 16 lanes, k_edge's strided lane map): the
//            edge prologue by the edge's 16 lanes (compose_motion, float32 composed pose, chain maps;
//            lanes own matrix entries), the corner sweep and the 16-lane butterfly of the 27
//            normal-equation sums (k_edge's), and the chain H = G^T A' G, g = G^T b' into the group's
//            LDS -- nothing per edge goes through HBM (k_prep -> k_edge -> k_photo wrote and re-read
//            erec / echain / eh: 66 + 90 doubles per edge);
//   phase B  k_photo's per-photo Cholesky, z', U / Y', and the group's Schur pair products written
//            once per (group, camera-pair block) slot for k_schur.
// Every reduction keeps the split step's fixed order (edge order within a photo, the pair lists'
// contribution order), so a run is bitwise reproducible.

// kGroupRound, kGChunk, kGRec and the LDS layout (group_layout) are in mcc_internal.h (host + device).

// The edge prologue by the edge's 16 lanes (sub = 0..15): prep_edge's chain (compose_motion of
// photo and camera, src/multicalib.cpp:1008-1056, called at src/mymulticalib.cpp:498-500; BACK:
// compose_motion(ds, photofront), :503-518 / src/doubleSide.cpp:320-328; the float32 composed pose,
// src/mymulticalib.cpp:546-553; the chain maps), with lanes owning the entries of each 3x3
// product.  S: 84 doubles of scratch.  Outputs: P[0..11] = R, T of the float32 pose; Gb = the
// chain maps' nonzero blocks [Gp11, Gp21, Gp22 | pad | Gg11, Gg21, Gg22 | pad].
template <int MODEL, bool BACK, int L, int GW = 28>
__device__ __forceinline__ void group_prologue(const double* ph, const double* ct, const double* sds, int side,
                                               int sub, double* S, double* P, double* Gb) {
    const double* R1 = ph;
    const double* Jr1 = ph + 9;
    const double* T1 = ph + 18;
    const double* R2 = ct;
    const double* Jl2 = ct + 9;
    const double* T2 = ct + 18;
    double* X = S;        // R3 [0..8], T3 [9..11], q [12..14]
    double* W = S + 15;   // A1 [0..8], A2 [9..17], B2 [18..26]
    // ---- compose_motion(photo, camera): R3 = R2 R1, q = R2 T1, T3 = q + T2 (OpenCV order)
    for (int e = sub; e < 12; e += L) {
        if (e < 9) {
            const int i = e / 3, j = e % 3;
            X[e] = dot3_nc(R2[i * 3], R1[j], R2[i * 3 + 1], R1[3 + j], R2[i * 3 + 2], R1[6 + j]);
        } else {
            const int i = e - 9;
            const double q = dot3_nc(R2[i * 3], T1[0], R2[i * 3 + 1], T1[1], R2[i * 3 + 2], T1[2]);
            X[12 + i] = q;
            X[9 + i] = add_nc(q, T2[i]);
        }
    }
    wave_sync_lds();
    double om[3], th, sn, cs;
    int jz;
    {
        double R3[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) R3[k] = X[k];
        rodrigues_m2v(R3, om, th, sn, cs, jz);
    }
    // ---- A1 = Jr^-1(om3) Jr(om1), A2 = Jl^-1(om3) Jl(om2), B2 = -[q]x Jl(om2)
    for (int e = sub; e < 27; e += L) {
        const int blk = e / 9, ee = e % 9, i = ee / 3, j = ee % 3;
        double row[3];
        if (blk < 2) {
            so3_poly_row(om, blk == 0 ? 0.5 : -0.5, jinv_coef(th, sn, cs), i, row);
        } else {
            const double q[3] = {X[12], X[13], X[14]};
            negskew_row(q, i, row);
        }
        const double* B = blk == 0 ? Jr1 : Jl2;
        const double v = row[0] * B[j] + row[1] * B[3 + j] + row[2] * B[6 + j];
        W[e] = BACK && blk < 2 && rot_jzero(sn, cs) ? 0.0 : v;
    }
    // cvRodrigues2's theta ~ pi branch: A1 = A2 = 0 (rot_jzero).  A cold loop where there is no BACK chain
    // (a select on every entry cost config4 ~0.4 us per step); a select in the BACK variants (the loop
    // spilled the tilted ones, at 256 VGPRs)
#if defined(MCC_NO_JZERO)   // (A/B builds only)
    if (false)
#elif !defined(MCC_JZ_SELECT)
    if (!BACK && __builtin_expect(jz, 0))
#else
    if (!BACK && __builtin_expect(rot_jzero(sn, cs), 0))
#endif
        for (int e = sub; e < 18; e += L) W[e] = 0.0;
    wave_sync_lds();
    if (!BACK || side != MCC_BACK) {
        // float32 composed pose, its Rodrigues (for the projection) and Jl
        double rf[3], Tf[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)om[k]; Tf[k] = (double)(float)X[9 + k]; }
        Rot rp;
        rodrigues_near(rf, th, sn, cs, rp);
        double ja, jb;
        jac_coef(rp.th, rp.s, rp.c, ja, jb);
        if (sub == 0) {
#pragma unroll
            for (int k = 0; k < 9; ++k) P[k] = rp.R[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) P[9 + k] = Tf[k];
        }
        // Gp = [[Jl A1, 0], [0, R2]];  Gg = [[Jl A2, 0], [B2, I]] (DoubleSide front: 0,
        // src/doubleSide.cpp:335-336)
        for (int t = sub; t < 54; t += L) {
            const int w = t / 27, blk = (t % 27) / 9, ee = t % 9, i = ee / 3, j = ee % 3;
            double v;
            if (w == 1 && MODEL == MCC_MODEL_DOUBLESIDE) {
                v = 0.0;
            } else if (blk == 0) {
                double row[3];
                so3_poly_row(rf, ja, jb, i, row);
                const double* M = w == 0 ? W : W + 9;
                v = row[0] * M[j] + row[1] * M[3 + j] + row[2] * M[6 + j];
            } else if (blk == 1) {
                v = w == 0 ? 0.0 : W[18 + ee];
            } else {
                v = w == 0 ? R2[ee] : (i == j ? 1.0 : 0.0);
            }
            Gb[GW * w + 9 * blk + ee] = v;
        }
        return;
    }
    // ---- BACK: compose_motion(ds, photofront); R(om_front) is the FP64 composed rotation R3
    double fa, fb;
    jac_coef(th, sn, cs, fa, fb);   // Jlf = Jl(om_front) = I + fa [om]x + fb [om]x^2
    double* Xb = S + 42;   // Rb [0..8], Tb [9..11], qb [12..14]
    double* Wb = S + 57;   // A1b [0..8], A2b [9..17], B2b [18..26]
    const double* Rds = sds;
    const double* Jrds = sds + 9;
    const double* dst = sds + 18;
    for (int e = sub; e < 12; e += L) {
        if (e < 9) {
            const int i = e / 3, j = e % 3;
            Xb[e] = dot3_nc(X[i * 3], Rds[j], X[i * 3 + 1], Rds[3 + j], X[i * 3 + 2], Rds[6 + j]);
        } else {
            const int i = e - 9;
            const double q = dot3_nc(X[i * 3], dst[0], X[i * 3 + 1], dst[1], X[i * 3 + 2], dst[2]);
            Xb[12 + i] = q;
            Xb[9 + i] = add_nc(q, X[9 + i]);
        }
    }
    wave_sync_lds();
    double omb[3], thb, snb, csb;
    {
        double Rb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) Rb[k] = Xb[k];
        rodrigues_m2v(Rb, omb, thb, snb, csb);
    }
    // A1b = Jr^-1(omb) Jr(ds), A2b = Jl^-1(omb) Jlf, B2b = -[qb]x Jlf
    for (int e = sub; e < 27; e += L) {
        const int blk = e / 9, ee = e % 9, i = ee / 3, j = ee % 3;
        double row[3], bc[3];
        if (blk < 2) {
            so3_poly_row(omb, blk == 0 ? 0.5 : -0.5, jinv_coef(thb, snb, csb), i, row);
        } else {
            const double q[3] = {Xb[12], Xb[13], Xb[14]};
            negskew_row(q, i, row);
        }
        if (blk == 0) {
            bc[0] = Jrds[j]; bc[1] = Jrds[3 + j]; bc[2] = Jrds[6 + j];
        } else {
            so3_poly_col(om, fa, fb, j, bc);   // column j of Jlf (registers: no private array)
        }
        // (rot_jzero: A1b = A2b = 0; a select here -- the cold loop of the front chain spilled the tilted
        // BACK variants, at 256 VGPRs)
        Wb[e] = blk < 2 && rot_jzero(snb, csb) ? 0.0 : row[0] * bc[0] + row[1] * bc[1] + row[2] * bc[2];
    }
    wave_sync_lds();
    double rf[3], Tf[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { rf[k] = (double)(float)omb[k]; Tf[k] = (double)(float)Xb[9 + k]; }
    Rot rp;
    rodrigues_near(rf, thb, snb, csb, rp);
    double ja, jb;
    jac_coef(rp.th, rp.s, rp.c, ja, jb);
    if (sub == 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) P[k] = rp.R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) P[9 + k] = Tf[k];
    }
    // Gp = [[Jl A2b A1, 0], [B2b A1, R2]] (:509-512); Gg (MyMulti, hazard A12: :514-517 omit
    // dTt/dTf dTf/dRc) = [[Jl A2b A2, 0], [B2b A2, I]]; Gg (DoubleSide ds, doubleSide.cpp:398-399)
    // = [[Jl A1b, 0], [0, R_front]]
    for (int t = sub; t < 54; t += L) {
        const int w = t / 27, blk = (t % 27) / 9, ee = t % 9, i = ee / 3, j = ee % 3;
        const bool ds = w == 1 && MODEL == MCC_MODEL_DOUBLESIDE;
        const double* M = w == 0 ? W : W + 9;   // A1 (photo) / A2 (camera)
        double v;
        if (blk == 0) {
            double row[3];
            so3_poly_row(rf, ja, jb, i, row);
            if (ds) {
                v = row[0] * Wb[j] + row[1] * Wb[3 + j] + row[2] * Wb[6 + j];
            } else {
                double t9[3];   // column j of A2b M
#pragma unroll
                for (int k = 0; k < 3; ++k) t9[k] = Wb[9 + k * 3] * M[j] + Wb[9 + k * 3 + 1] * M[3 + j] + Wb[9 + k * 3 + 2] * M[6 + j];
                v = row[0] * t9[0] + row[1] * t9[1] + row[2] * t9[2];
            }
        } else if (blk == 1) {
            v = ds ? 0.0 : Wb[18 + i * 3] * M[j] + Wb[18 + i * 3 + 1] * M[3 + j] + Wb[18 + i * 3 + 2] * M[6 + j];
        } else {
            v = w == 0 ? R2[ee] : (ds ? X[ee] : (i == j ? 1.0 : 0.0));
        }
        Gb[GW * w + 9 * blk + ee] = v;
    }
}

// The chain of one edge from LDS (k_edge's edge_chain_xh with the chain-map blocks read from Gb
// and H written into the edge's group record): X_w = A' G_w (X_p with b' as a seventh column),
// then [Hpp | gp] = Gp^T [Xp | b'], [Hgp | gg] = Gg^T [Xp | b'], Hgg = Gg^T Xg.  Record layout:
// rec[0..20] Hgg upper, rec[22..57] Hgp (U after k_photo's step), rec[58..63] gg,
// rec[64..84] Hpp upper, rec[85..90] gp.  Every lane of the wave calls it (wave-level syncs).
struct GroupChain {
    double A[36], B[8];
    double X[2][6][8];
};
__device__ __forceinline__ void group_chain(GroupChain& CH, const double* Gbe, int sq, bool valid, double* rec) {
    if (sq < 12) {
        const int w = sq / 6, i = sq % 6;
        double ar[6], gm[28], xr[8];
        const double2* A2 = reinterpret_cast<const double2*>(CH.A + 6 * i);
        const double2* G2 = reinterpret_cast<const double2*>(Gbe + 28 * w);
#pragma unroll
        for (int q = 0; q < 3; ++q) { const double2 v = A2[q]; ar[2 * q] = v.x; ar[2 * q + 1] = v.y; }
#pragma unroll
        for (int q = 0; q < 14; ++q) { const double2 v = G2[q]; gm[2 * q] = v.x; gm[2 * q + 1] = v.y; }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double s2 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s2 += ar[k] * gm[k * 3 + j];            // G11
#pragma unroll
            for (int k = 0; k < 3; ++k) s2 += ar[3 + k] * gm[9 + k * 3 + j];   // G21
            xr[j] = s2;
            double s3 = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s3 += ar[3 + k] * gm[18 + k * 3 + j];  // G22
            xr[3 + j] = s3;
        }
        xr[6] = w == 0 ? CH.B[i] : 0.0;
        xr[7] = 0.0;
        double2* X2 = reinterpret_cast<double2*>(CH.X[w][i]);
#pragma unroll
        for (int q = 0; q < 4; ++q) X2[q] = make_double2(xr[2 * q], xr[2 * q + 1]);
    }
    wave_sync_lds();
    if (sq < 9 && valid) {
        const int T = sq / 3, i = sq % 3;
        const double* Gl = Gbe + 28 * (T == 0 ? 0 : 1);
        const double2* X2 = reinterpret_cast<const double2*>(CH.X[T == 2 ? 1 : 0][0]);
        double c11[3], c21[3], c22[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            c11[k] = Gl[k * 3 + i];
            c21[k] = Gl[9 + k * 3 + i];
            c22[k] = Gl[18 + k * 3 + i];
        }
        double h[7], h2[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) { h[j] = 0.0; h2[j] = 0.0; }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double xk[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) { const double2 v = X2[4 * k + q]; xk[2 * q] = v.x; xk[2 * q + 1] = v.y; }
            const double c = k < 3 ? c11[k] : c21[k - 3];
#pragma unroll
            for (int j = 0; j < 7; ++j) h[j] += c * xk[j];
            if (k >= 3) {
#pragma unroll
                for (int j = 0; j < 7; ++j) h2[j] += c22[k - 3] * xk[j];
            }
        }
        // T = 0: Hpp (upper, rows i, i + 3) and gp; T = 1: Hgp (rows i, i + 3) and gg; T = 2: Hgg
        const int i2 = i + 3;
        if (T == 1) {
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                rec[22 + 6 * i + j] = h[j];
                rec[22 + 6 * i2 + j] = h2[j];
            }
            rec[58 + i] = h[6];
            rec[58 + i2] = h2[6];
        } else {
            double* base = rec + (T == 0 ? 64 : 0);
            double* o1 = base + 6 * i - i * (i - 1) / 2 - i;
            double* o2 = base + 6 * i2 - i2 * (i2 - 1) / 2 - i2;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                if (j >= i) o1[j] = h[j];
                if (j >= i2) o2[j] = h2[j];
            }
            if (T == 0) {
                rec[85 + i] = h[6];
                rec[85 + i2] = h2[6];
            }
        }
    }
}

// ---------------------------------------------------------------- the folded reduction (gfold)
// k_group's step with k_schur's one-level reduction and the m <= 30 solve in the SAME launch
// (LinArgs::fold): after the groups (and the spare) the grid holds one item
// workgroup per k_schur item, one per norm chunk, and a final workgroup.  Nothing signals: every
// handed-off word is its own flag (kFoldEmpty until the producer's 8-byte sc1 store lands; 8-byte
// aligned halves of a store are single-copy atomic), each consumer polls the words it needs with sc1
// loads and writes kFoldEmpty back once it has read them, so the words are empty again before the next
// launch's producers (after the kernel boundary).  Progress needs no dispatch order and no
// co-residency of the whole grid: producers (groups, spare) never wait, and mcc_create takes the fold
// only while the spinning consumers fill at most half of the CUs (one k_group workgroup fits per CU),
// so in any dispatch order a slot stays free for some producer, which runs to its end
// (MCC_FOLD_CONSUMERS_FIRST=1 puts the consumers at the lowest grid indices to test exactly that).
// fold_dyn is the exception: a finished group spins on groups that may not have started, so it needs
// the whole grid resident (mcc_create: groups + spare <= CUs).  The sums are k_schur's,
// in its order (kSub sub-chunks per item entry, chunks in photo order, items in item order), so the
// bits are the k_group -> k_schur step's.  Where k_schur's boundary and item phase followed the last
// group (~4 us at config4), the items here have summed most slots by then.
__device__ __forceinline__ bool fold_valid(double v) { return __double_as_longlong(v) != kFoldEmpty; }
__device__ __forceinline__ void fold_empty(double* p) { st_sc1(p, __longlong_as_double(kFoldEmpty)); }
// a poll that outlives LinArgs::spare_wait: the step fails (MCC_ETIMEOUT) and the loop stops
__device__ __forceinline__ bool fold_timed_out(const LinArgs& a, long long t0) {
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 < a.spare_wait) return false;
    atomicOr(&a.state->error, kErrWarmTimeout);
    a.state->done = 1;
    return true;
}

// item workgroup: the item's slots (sub-chunk sub sums slots sub, sub + kSub, ... of entry q, k_schur's
// order), each thread loading all of its slots in one batch and adding the valid prefix in order; the
// item's 48-entry partial -> fsa.item_out (sc1)
constexpr int kFoldSlots = 13;   // slots per thread: items of <= 64 slots (mcc_create) over kSub sub-chunks
// (The batch is re-issued back to back while slots are missing.  Round 6 measured the polls' cost: a
// sleeping single-slot pre-wait for items dispatched while the groups run left the step's memory-side
// traffic at 12.94 MB against 13.04 (config4), and its extra round trip for items that start late cost
// +0.5 us per step)
__device__ __forceinline__ void fold_item(const LinArgs& la, int item) {
    const SchurArgs& a = la.fsa;
    const int tid = threadIdx.x;
    const int4 it = a.items[item];   // {block, first slot's offset (doubles), slots, slot size 48 | 36}
    const int q = tid % 48, sub = tid / 48, sz = it.w & (kItemSingle - 1);
    __shared__ double part[kSub][48];
    __shared__ int fail;
    long long* srow = a.stamps ? a.stamps + kSchurStampStride * (size_t)item : nullptr;   // MCC_DIAG
    SSTAMP(srow, 0, 0);
    if (tid == 0) fail = 0;
    double s = 0.0;
    const int ns = sub < kSub ? (it.z - sub + kSub - 1) / kSub : 0;   // this thread's slots
    if (ns > 0 && q < sz) {
        const double* pp = a.pairprod + (size_t)it.y + q;
        int next = 0;
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (;;) {
            // the slots not summed yet (the summed ones re-read at the first slot's address instead)
            double v[kFoldSlots];
#pragma unroll
            for (int u = 0; u < kFoldSlots; ++u)
                v[u] = ld_sc1(pp + (size_t)sz * (sub + kSub * (u < next ? 0 : min(u, ns - 1))));
#pragma unroll
            for (int u = 0; u < kFoldSlots; ++u)
                if (u == next && u < ns && fold_valid(v[u])) {
                    s += v[u];
                    ++next;
                }
            if (next >= ns) break;
            if (fold_timed_out(la, t0)) { fail = 1; break; }
        }
        s += 0.0;   // (k_schur adds its batch's zero padding: -0.0 becomes +0.0 there too)
    }
    if (sub < kSub) part[sub][q] = s;
    __syncthreads();
    if (tid < 48 && !fail) {
        double t = part[0][tid];
        for (int c = 1; c < kSub; ++c) t += part[c][tid];
        st_sc1(a.item_out + 48 * (size_t)item + tid, t);
    }
    SSTAMP(srow, 1, 0);
    // the slots back to kFoldEmpty, after the partial (ahead of it these stores held its store up)
    if (ns > 0 && q < sz) {
        double* pp = const_cast<double*>(a.pairprod) + (size_t)it.y + q;
        for (int u = 0; u < ns; ++u) fold_empty(pp + (size_t)sz * (sub + kSub * u));
    }
}

// norm-chunk workgroup c: 256 photos' ||G||^2, ||x||^2 (k_schur's norm chunk: a fixed butterfly per
// wave, the four waves in order) and their not-PD flags (the final workgroup's photo error)
__device__ __forceinline__ void fold_chunk(const LinArgs& la, int c) {
    const SchurArgs& a = la.fsa;
    const int tid = threadIdx.x;
    __shared__ double wred[3][kSchurThreads / 64];
    __shared__ int fail;
    long long* srow = a.stamps ? a.stamps + kSchurStampStride * (size_t)(a.n_items + c) : nullptr;   // MCC_DIAG
    SSTAMP(srow, 0, 0);
    if (tid == 0) fail = 0;
    if (tid < kSchurThreads) {   // waves 0..3
        const int p = c * kSchurThreads + tid;
        double g = 0.0, x = 0.0, bad = 0.0;
        if (p < a.n_photos) {
            const double* fp = la.fnorm + 4 * (size_t)p;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            for (;;) {
                const double w0 = ld_sc1(fp), w1 = ld_sc1(fp + 1), w2 = ld_sc1(fp + 2);
                if (fold_valid(w0) && fold_valid(w1) && fold_valid(w2)) {
                    g = w0; x = w1; bad = w2;
                    break;
                }
                if (fold_timed_out(la, t0)) { fail = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        g = wave_sum(g);
        x = wave_sum(x);
        bad = wave_sum(bad);
        if ((tid & 63) == 0) {
            wred[0][tid >> 6] = g;
            wred[1][tid >> 6] = x;
            wred[2][tid >> 6] = bad;
        }
    }
    __syncthreads();
    if (tid < 3 && !fail) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kSchurThreads / 64; ++w) v += wred[tid][w];
        st_sc1(a.item_out + 48 * (size_t)(a.n_items + c) + tid, v);
    }
    SSTAMP(srow, 1, 0);
    const int p = c * kSchurThreads + tid;
    if (tid < kSchurThreads && p < a.n_photos) {   // back to kFoldEmpty, after the partial
        double* fw = la.fnorm + 4 * (size_t)p;
        fold_empty(fw); fold_empty(fw + 1); fold_empty(fw + 2);
    }
}

// the final workgroup: every partial (48 per item / chunk) and the spare's inverse with its status into
// LDS by polling (each thread a fixed set of words, re-read until valid; the inverse's words only when
// the status says there is one), then kFoldEmpty back into all of them, and k_schur's one-level finish
// (sums in item order, placement, the refinement or elimination, the camera update)
template <int U>
__device__ __forceinline__ void fold_final_u(const LinArgs& la) {
    const SchurArgs& a = la.fsa;
    State* st = a.state;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int m = a.m, np = la.fold_parts;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const bool useiv = a.ssinv != nullptr && a.fuse_solve;   // (a.ssinv is la.fiv here)
    double* Iv = sm + m * m + m;
    double* itm = sm + schur_items_offset(m, a.fuse_solve, a.ssinv != nullptr);   // [np][48]
    int* sbi = reinterpret_cast<int*>(itm + 48 * (size_t)np);                       // [nblk + 1]
    __shared__ double s_status;
    __shared__ int s_fail;
    long long* srow = a.stamps ? a.stamps + kSchurStampStride * (size_t)np : nullptr;   // MCC_DIAG: after the parts
    SSTAMP(srow, 10, 0);   // (slots 0..2 are the solve's)
    const int bi = a.block_items[tid < a.nblk ? tid : a.nblk];
    const int iter = st->iter;
    const double cn0 = st->cam_normG2, cn1 = st->cam_normX2;
    const int nI = 48 * np, nV = useiv ? m * m + 1 : 0, n = nI + nV;
    if (tid == 0) {
        s_status = useiv ? 0.0 : -1.0;   // 0: not seen yet; no inverse buffer: none
        s_fail = 0;
    }
    __syncthreads();
    unsigned have = 0;   // words of this thread already in LDS
    // (a norm chunk's partial carries 3 words: ||G||^2, ||x||^2, the not-PD count; an item's all 48)
    auto due = [&](int t) { return t >= nI || t < 48 * a.n_items || t % 48 < 3; };
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int t = u * nt + tid;
            t = t < n ? t : n - 1;
            v[u] = ld_sc1(t < nI ? a.item_out + t : la.fiv + (t - nI));
        }
        // (every thread reads the status itself: its inverse words are due unless it says "none")
        const double stt = useiv ? ld_sc1(la.fiv + m * m) : -1.0;
        int pend = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = u * nt + tid;
            if (t >= n || ((have >> u) & 1) || !due(t)) continue;
            if (!fold_valid(v[u])) {
                // partials and the status are always due; the inverse unless the status says "none"
                if (t < nI || t == nI + m * m || !fold_valid(stt) || stt > 0.0) ++pend;
                continue;
            }
            have |= 1u << u;
            if (t < nI) itm[t] = v[u];
            else if (t < nI + m * m) Iv[t - nI] = v[u];
            else s_status = v[u];
        }
        if (!__syncthreads_or(pend)) break;
        // the poll bound, decided by one thread for all (the loop's barriers stay matched)
        if (tid == 0 && (long long)__builtin_amdgcn_s_memrealtime() - t0 >= la.spare_wait) {
            atomicOr(&st->error, kErrWarmTimeout);
            st->done = 1;
            s_fail = 1;
        }
        __syncthreads();
        if (s_fail) return;
    }
    // every word back to kFoldEmpty for the next launch's producers (this launch's have all landed)
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = u * nt + tid;
        if (t < n && ((have >> u) & 1)) fold_empty(t < nI ? a.item_out + t : la.fiv + (t - nI));
    }
    if (tid <= a.nblk) sbi[tid] = bi;
    // a photo block that is not positive definite (any chunk's flag sum, entry 2)
    int err_now = 0;
    for (int k = a.n_items; k < np; ++k) err_now |= itm[48 * k + 2] != 0.0 ? kErrPhotoNotPD : 0;
    __syncthreads();
    SSTAMP(srow, 8, 0);   // the partials landed in LDS
    // (the inverse only with this launch's tag: fold_final_direct)
    schur_finish(a, np, iter, cn0, cn1, err_now, useiv && s_status == (double)(iter + 1), srow);
}
// The final workgroup with the sums formed where the words land (LinArgs::fold_direct: 512 threads,
// <= 8 items per camera-pair block, <= 4 norm chunks -- config4): thread t < 48 nblk owns entry t of
// the packed system and polls its block's item words straight into registers, adding them in item
// order (k_schur's order, so the same bits); threads 48 nblk, +1 own ||G||^2, ||x||^2 (each with the
// chunks' not-PD counts), the rest the spare's inverse.  Nothing passes through an LDS copy of the
// partials: the copy, a barrier and the runtime-bounded LDS sums (~1.8 us from the landed batch to the
// placed sums at config4) leave the tail.
constexpr int kFoldKI = 8;   // words per thread
__device__ __forceinline__ void fold_final_reset(const LinArgs& la, const double* const* src, unsigned have, bool useiv) {
#pragma unroll
    for (int q = 0; q < kFoldKI; ++q)
        if ((have >> q) & 1) fold_empty(const_cast<double*>(src[q]));
    if (threadIdx.x == 0 && useiv) fold_empty(la.fiv + la.fsa.m * la.fsa.m);
}
__device__ __forceinline__ void fold_final_direct(const LinArgs& la) {
    const SchurArgs& a = la.fsa;
    State* st = a.state;
    const int tid = threadIdx.x, nt = blockDim.x;
    const int m = a.m, nb = m / 6, ntri = m * (m + 1) / 2, np = la.fold_parts, nc = np - a.n_items;
    extern __shared__ __attribute__((aligned(16))) double sm[];
    double* S = sm;
    double* r = sm + m * m;
    double* Iv = sm + m * m + m;
    __shared__ double norms[2];
    __shared__ int s_fail;
    const bool useiv = a.ssinv != nullptr && a.fuse_solve;
    const bool lds = a.fuse_solve && a.peer.nranks == 0;
    long long* srow = a.stamps ? a.stamps + kSchurStampStride * (size_t)np : nullptr;   // MCC_DIAG
    SSTAMP(srow, 10, 0);
    const int nent = a.nblk * 48, ivt0 = nent + 2, nivt = nt - ivt0;
    // this thread's words
    const double* src[kFoldKI];
    int cnt = 0, kind = 0;   // kind 1: an entry, 2: a norm (+ not-PD counts), 3: inverse words
    int blk = 0, e = 0;
    if (tid < nent) {
        blk = tid / 48;
        e = tid % 48;
        const int k0 = a.block_items[blk], nk = a.block_items[blk + 1] - k0;
        int b1 = 0;
#pragma unroll
        for (int b = 1; b < 5; ++b)
            if (b < nb && b * nb - b * (b - 1) / 2 <= blk) b1 = b;
        const int b2 = b1 + (blk - (b1 * nb - b1 * (b1 - 1) / 2));
        kind = 1;
        cnt = e >= 36 && b1 != b2 ? 0 : nk;   // (off-diagonal blocks: 36 entries)
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) src[q] = a.item_out + 48 * (size_t)(k0 + (q < nk ? q : 0)) + e;
    } else if (tid < ivt0) {
        const int w = tid - nent;
        kind = 2;
        cnt = 2 * nc;   // chunk words w, then the chunks' not-PD counts (entry 2)
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) {
            const int c = q < nc ? q : (q - nc < nc ? q - nc : 0);
            src[q] = a.item_out + 48 * (size_t)(a.n_items + c) + (q < nc ? w : 2);
        }
    } else {
        kind = 3;
        const int j0 = tid - ivt0;
        cnt = 0;
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) {
            const int j = j0 + q * nivt;
            if (useiv && j < m * m) cnt = q + 1;
            src[q] = la.fiv + (useiv && j < m * m ? j : 0);
        }
    }
    // the state words, read ahead of the poll (their loads overlap it)
    const int iter = st->iter;
    const double cn = kind == 2 && a.rank == 0 ? (tid - nent ? st->cam_normX2 : st->cam_normG2) : 0.0;
    if (tid == 0) s_fail = 0;
    __syncthreads();
    double kv[kFoldKI];
    unsigned have = 0;
    double stt = -1.0;
    // each thread polls its own words until they have all landed (one memory round trip per pass, no
    // barrier per pass), then one barrier; words already in registers are re-read at the status word's
    // address (one request per wave) instead of their own
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (;;) {
        double v[kFoldKI];
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) v[q] = ld_sc1(((have >> q) & 1) ? la.fiv + m * m : src[q]);
        if (useiv) stt = ld_sc1(la.fiv + m * m);
        int pend = tid == 0 && useiv && !fold_valid(stt) ? 1 : 0;
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) {
            if (q >= cnt || ((have >> q) & 1)) continue;
            if (fold_valid(v[q])) {
                kv[q] = v[q];
                have |= 1u << q;
            } else if (kind != 3 || !fold_valid(stt) || stt > 0.0) {
                ++pend;   // the inverse's words are due unless the status says "none"
            }
        }
        if (!pend) break;
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 >= la.spare_wait) {
            s_fail = 1;
            break;
        }
    }
    __shared__ double s_stt;
    if (tid == 0) s_stt = stt;   // (thread 0 waited for the status; a thread whose own words landed
                                 // first may have read it empty)
    __syncthreads();
    if (s_fail) {
        if (tid == 0) {
            atomicOr(&st->error, kErrWarmTimeout);
            st->done = 1;
        }
        return;
    }
    SSTAMP(srow, 8, 0);   // every word landed
    // the inverse only with this launch's tag, +(iteration + 1) (the spare's status is +-(iteration + 1));
    // a status another launch left would read as landed, and its inverse is not this system's: the
    // step then eliminates directly (set_state empties every word after a failed launch, so this is a
    // guard, not a path)
    const bool ivok = useiv && s_stt == (double)(iter + 1);
    if (kind == 1 && cnt > 0) {
        double v = 0.0;
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q)
            if (q < cnt) v += kv[q];   // item order (k_schur's level-1 sums)
        int b1 = 0;
#pragma unroll
        for (int b = 1; b < 5; ++b)
            if (b < nb && b * nb - b * (b - 1) / 2 <= blk) b1 = b;
        const int b2 = b1 + (blk - (b1 * nb - b1 * (b1 - 1) / 2));
        if (e < 36) {
            const int ii = e / 6, jj = e % 6, i = 6 * b1 + ii, j = 6 * b2 + jj;
            if (b1 != b2 || ii <= jj) {
                a.packed[packed_index(i, j, m)] = v;
                if (lds) {
                    S[i * m + j] = v;
                    S[j * m + i] = v;
                }
            }
        } else {
            const int w = (e - 36) / 6, i = 6 * b1 + (e - 36) % 6;
            a.packed[ntri + w * m + i] = v;   // r (w = 0), JTE of the global block (w = 1)
            if (lds && w == 0) r[i] = v;
        }
    } else if (kind == 2) {
        const int w = tid - nent;
        double nrm = 0.0, bad = 0.0;
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q) {
            if (q < nc) nrm += kv[q];                  // chunk order
            else if (q < 2 * nc) bad += kv[q];
        }
        if (a.rank == 0) nrm += cn;
        if (iter <= 0) nrm = 0.0;
        nrm = photo_flag_norm(bad != 0.0 ? kErrPhotoNotPD : 0, w, nrm);
        norms[w] = nrm;
        a.packed[ntri + 2 * m + w] = nrm;
    } else if (kind == 3 && ivok) {
        const int j0 = tid - ivt0;
#pragma unroll
        for (int q = 0; q < kFoldKI; ++q)
            if (q < cnt) Iv[j0 + q * nivt] = kv[q];
    }
    SSTAMP(srow, 9, 0);   // sums placed (thread 0)
    if (!a.fuse_solve) {
        fold_final_reset(la, src, have, useiv);
        return;
    }
    __syncthreads();   // S, r, the inverse and the norms in LDS
    if (a.peer.nranks > 0) {
        if (!peer_exchange(a.peer, st, a.packed)) {
            fold_final_reset(la, src, have, useiv);
            return;
        }
        for (int t = tid; t < ntri + m; t += nt) {
            const double v = a.packed[t];
            if (t < ntri) {
                int i, j;
                packed_ij(t, m, i, j);
                S[i * m + j] = v;
                S[j * m + i] = v;
            } else {
                r[t - ntri] = v;
            }
        }
        if (tid < 2) norms[tid] = a.packed[ntri + 2 * m + tid];
        __syncthreads();
    }
    SSTAMP(srow, 3, 0);
    SolveCtx sc = a.solve;
    sc.stamps = srow;
    solve_global<false>(sc, S, r, norms[0], norms[1], nullptr, ivok ? Iv : nullptr);
    SSTAMP(srow, 7, 0);
    // every word back to kFoldEmpty for the next launch's producers (after the solve: ahead of it these
    // 4 000 write-through stores held up the placement's)
    fold_final_reset(la, src, have, useiv);
}
// (one batch width per k_group shape: the host keeps 48 parts + m^2 + 1 within k_schur's one-level
// bound, kSchurOneLevelLoads x 256 words)
template <int NT>
__device__ __forceinline__ void fold_final(const LinArgs& la) {
    if (NT == 512 && la.fold_direct) {
        fold_final_direct(la);
        return;
    }
    constexpr int UM = kSchurOneLevelLoads * 256 / NT;
    const int n = 48 * la.fold_parts + (la.fsa.ssinv != nullptr ? la.fsa.m * la.fsa.m + 1 : 0);
    if (n <= UM / 2 * NT) fold_final_u<UM / 2>(la);
    else fold_final_u<UM>(la);
}

#ifndef MCC_GROUP_PAIR_THREADS
#define MCC_GROUP_PAIR_THREADS 256   // threads the pair tasks may spread over (config4, 32 lanes: 256 29.0 vs 512 29.8 us per step)
#endif
#ifndef MCC_GROUP_OCC
#define MCC_GROUP_OCC 2   // k_group workgroups per CU the register budget allows (LDS: ~64 KB each)
#endif
// The group's work (phases 0, A, B above); false when the loop has stopped (nothing done).
template <int MODEL, bool RATIONAL, int PRISM, bool BACK, int L>
__device__ __forceinline__ bool group_body(const LinArgs& a, const int grp) {
    constexpr int NT = kGroupRound * L, EPW = 64 / L;   // threads; edges per wave
    State* st = a.state;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // ---- round trip 1: the state and the group's ranges (the stop test after the loads are issued)
    const int done = st->done, pending = st->pending;
    const double alpha_prev = st->alpha;   // step factor of the pending update
    const int p0 = a.pgrp_ptr[grp], np = a.pgrp_ptr[grp + 1] - p0;
    const int ge0 = a.pgrp_edge[grp], gne = a.pgrp_edge[grp + 1] - ge0;   // the group's edges are contiguous
    const int q0 = a.gpair_ptr[grp], nq = a.gpair_ptr[grp + 1] - q0;
    const int c0 = a.gcon_ptr[grp], nc = a.gcon_ptr[grp + 1] - c0;
    if (done) return false;
    long long* stp = a.stamps ? a.stamps + kStampStride * (size_t)grp : nullptr;   // MCC_DIAG: slots 0..11
    SSTAMP(stp, 0, 0);
    const int C = a.n_cams, m = a.global_dim;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const GroupLayout GL = group_layout(gne, C, nq, nc);
    double* rec = smem + GL.rec;
    double* s27 = smem + GL.s27;
    double* sLi = smem + GL.sLi;
    double* sv = smem + GL.sv;
    double* sph = smem + GL.sph;
    double* sxn = smem + GL.sxn;
    double* spart = smem + GL.spart;
    double* sdg = smem + GL.sdg;
    double* ctab = smem + GL.ctab;
    double* ktab = smem + GL.ktab;
    double* sds = smem + GL.sds;
    double* sP = smem + GL.sP;
    double* sGb = smem + GL.sGb;
    int* ibase = reinterpret_cast<int*>(smem + GL.ndoubles);
    int4* sInfo = reinterpret_cast<int4*>(ibase + GL.iInfo);
    int* sgb = ibase + GL.iGb;
    int* seq = ibase + GL.iEq;
    int* sph0 = ibase + GL.iPh;
    int4* spq = reinterpret_cast<int4*>(ibase + GL.iPq);
    unsigned* scn = reinterpret_cast<unsigned*>(ibase + GL.iCn);
    // this wave's corner staging [5][kGChunk][4] (union with its chain records after the sweep)
    float(*sC)[kGChunk][EPW] = reinterpret_cast<float(*)[kGChunk][EPW]>(smem + GL.sU + wave * (5 * kGChunk * EPW / 2));
    GroupChain* sCH = reinterpret_cast<GroupChain*>(smem + GL.sU + wave * (5 * kGChunk * EPW / 2));
    static_assert(EPW * sizeof(GroupChain) <= 5 * kGChunk * EPW * sizeof(float), "k_group chain union");

    const int g = lane % EPW, sub = lane / EPW;   // edge slot of the wave, lane within the edge
    // corners of an edge -> this wave's staging (every load of the chunk issued before the first store)
    auto stage = [&](int eoff, int cc0, int cn) {
        constexpr int PER = kGChunk / L;
        float v[PER][5];
        int sb = sub;
        asm volatile("" : "+v"(sb));
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = sb + L * u;
            const unsigned c = (unsigned)(eoff + cc0 + (i < cn ? i : 0));
            v[u][0] = a.obj_x[c];
            v[u][1] = a.obj_y[c];
            v[u][2] = a.obj_z[c];
            v[u][3] = a.img_u[c];
            v[u][4] = a.img_v[c];
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int i = sb + L * u;
            if (i < cn) {
#pragma unroll
                for (int f = 0; f < 5; ++f) sC[f][i][g] = v[u][f];
            }
        }
    };

    // the cameras' (and the double-side transform's) Rodrigues tables are formed by threads outside
    // the photo tasks' wave while those update the photos (k_linearize's wave-1 code)
    constexpr int CAM0 = NT / 2, DST = CAM0 + 63;
    double om2[3] = {0.0, 0.0, 0.0}, T2[3] = {0.0, 0.0, 0.0};
    // ---- phase 0: every load of the group in one round trip
    {
        // the first round's corners (issued first: the longest stream)
        {
            const int le = wave * EPW + g;
            const int4 info = le < gne ? a.edge_info[ge0 + le] : make_int4(0, 0, 0, 0);
            if (le < gne) stage(info.z, 0, min(info.w, kGChunk));
        }
        // edge records, the group's pair lists
        for (int t = tid; t < gne; t += NT) {
            sInfo[t] = a.edge_info[ge0 + t];
            sgb[t] = a.gblock[ge0 + t];
            seq[t] = a.edge_lphoto[ge0 + t];
        }
        if (tid <= np) sph0[tid] = a.photo_ptr[p0 + tid] - ge0;
        for (int t = tid; t < nq; t += NT) spq[t] = a.gpairs[q0 + t];
        for (int t = tid; t < nc; t += NT) scn[t] = a.gcon[c0 + t];
        for (int t = tid; t < m; t += NT) sdg[t] = a.dg[t];
        if (tid >= CAM0 && tid < CAM0 + C) {   // camera tables: loads here, Rodrigues after the partials
            const int c = tid - CAM0;
            if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.cam_rt[6 * c + k]; T2[k] = a.cam_rt[6 * c + 3 + k]; }
            } else if (c == 0) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = 0.0; T2[k] = 0.0; }   // src/mymulticalib.cpp:721-725
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.x[6 * (c - 1) + k]; T2[k] = a.x[6 * (c - 1) + 3 + k]; }
            }
            double* kt = ktab + kGIntr * c;
            const float* Kc = a.K + 9 * c;
            kt[0] = Kc[0]; kt[1] = Kc[4]; kt[2] = Kc[2]; kt[3] = Kc[5]; kt[4] = Kc[1];
            kt[5] = MODEL == MCC_MODEL_OMNI ? (double)a.xi[c] : 0.0;
            const int nd = a.nd;
#pragma unroll
            for (int q = 0; q < 12; ++q) kt[6 + q] = q < nd ? (double)a.D[nd * c + q] : 0.0;
            if (PRISM == 2)
#pragma unroll
                for (int q = 0; q < 9; ++q) kt[18 + q] = a.tilt[9 * c + q];
        } else if (BACK && tid == DST) {   // the double-side transform (BACK edges; DoubleSide's global block)
            if (MODEL == MCC_MODEL_DOUBLESIDE) {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.x[k]; T2[k] = a.x[3 + k]; }
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k) { om2[k] = a.ds_rt[k]; T2[k] = a.ds_rt[3 + k]; }
            }
        }
    }
    // the pending update's operands: thread (le, k) < 6 gne forms sum_i Y'_e[i][k] dg_g(e)[i]
    // (k_prep's order; its first task's Y' column and global block loaded in this round trip);
    // thread 192 + 6q + k < 192 + 6 np: photo q's x_k and z'_k
    float xo = 0.f;
    double zk = 0.0;
    const int pq = (tid - 192) / 6, pk = (tid - 192) % 6;
    const bool ptask = tid >= 192 && pq < np;
    double2 pn0 = make_double2(0.0, 0.0);   // the fold without a pending update: the norms k_backsub left
    if (ptask) {
        xo = a.x[m + 6 * (size_t)(p0 + pq) + pk];
        if (pending) zk = a.zp[6 * (size_t)(p0 + pq) + pk];
        else if (a.fold && pk == 0) pn0 = *reinterpret_cast<const double2*>(a.photo_norm + 2 * (size_t)(p0 + pq));
    }
    double y0[6];
    int gb0 = -1;
    if (pending && tid < 6 * gne) {
        const int le = tid / 6, k = tid % 6;
        gb0 = a.gblock[ge0 + le];
        const double* Ye = a.Y + 36 * (size_t)(ge0 + le);
#pragma unroll
        for (int i = 0; i < 6; ++i) y0[i] = Ye[6 * i + k];
    }
    __syncthreads();
    SSTAMP(stp, 1, 0);
    if (pending) {
        for (int t = tid; t < 6 * gne; t += NT) {
            const int le = t / 6, k = t % 6;
            int gbl = gb0;
            double y[6];
            if (t == tid) {
#pragma unroll
                for (int i = 0; i < 6; ++i) y[i] = y0[i];
            } else {
                gbl = sgb[le];
                const double* Ye = a.Y + 36 * (size_t)(ge0 + le);
#pragma unroll
                for (int i = 0; i < 6; ++i) y[i] = Ye[6 * i + k];
            }
            const double* d = sdg + 6 * (gbl < 0 ? 0 : gbl);
            double sk = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) sk += y[i] * d[i];
            spart[6 * le + k] = gbl < 0 ? 0.0 : sk;
        }
    }
    __syncthreads();
    if (tid >= CAM0 && tid < CAM0 + C) {
        const int c = tid - CAM0;
        Rot r2;
        rodrigues_v2m(om2, r2);
        double J[9];
        so3_jac(om2, r2, +1.0, J);
        double* ct = ctab + 24 * c;
#pragma unroll
        for (int k = 0; k < 9; ++k) { ct[k] = r2.R[k]; ct[9 + k] = J[k]; }
#pragma unroll
        for (int k = 0; k < 3; ++k) ct[18 + k] = T2[k];
    } else if (BACK && tid == DST) {
        Rot rd;
        rodrigues_v2m(om2, rd);
        double J[9];
        so3_jac(om2, rd, -1.0, J);
#pragma unroll
        for (int k = 0; k < 9; ++k) { sds[k] = rd.R[k]; sds[9 + k] = J[k]; }
#pragma unroll
        for (int k = 0; k < 3; ++k) sds[18 + k] = T2[k];
    }
    // the photo update x = fl32(x + fl32(alpha (z' - sum_e Y'_e^T dg))) (k_prep's; src/multicalib.cpp:482-501)
    if (ptask) {
        float xn = xo;
        double Gk = 0.0;
        if (pending) {
            double t = zk;
            for (int le = sph0[pq]; le < sph0[pq + 1]; ++le) t -= spart[6 * le + pk];
            const float G = (float)(alpha_prev * t);   // G = alpha*delta -> CV_32F (:491-496)
            xn = xo + G;                                // x = x + G (:501)
            a.x[m + 6 * (size_t)(p0 + pq) + pk] = xn;
            Gk = (double)G;
        }
        sxn[16 * pq + pk] = (double)xn;
        sxn[16 * pq + 8 + pk] = Gk;
    }
    wave_sync_lds();   // the photo tasks are all in wave 3
    if (ptask && pk == 0) {   // ||G||^2, ||x||^2 partials (stop test); the photo's Rodrigues
        const double* xs = sxn + 16 * pq;
        if (pending) {
            double g2 = 0.0, x2 = 0.0;
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                g2 += xs[8 + q] * xs[8 + q];
                x2 += xs[q] * xs[q];
            }
            a.photo_norm[2 * (size_t)(p0 + pq)] = g2;
            a.photo_norm[2 * (size_t)(p0 + pq) + 1] = x2;
            pn0 = make_double2(g2, x2);
        }
        if (a.fold) {   // (sxn's pad words) the folded norm chunk's input, written after the Cholesky
            sxn[16 * pq + 6] = pn0.x;
            sxn[16 * pq + 7] = pn0.y;
        }
        const double om1[3] = {xs[0], xs[1], xs[2]};
        Rot r1;
        rodrigues_v2m(om1, r1);
        double* ph = sph + 24 * pq;
        so3_jac(om1, r1, -1.0, ph + 9);
#pragma unroll
        for (int k = 0; k < 9; ++k) ph[k] = r1.R[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) ph[18 + k] = xs[3 + k];
    }
    __syncthreads();
    SSTAMP(stp, 2, 0);

    // ---- phase A: rounds of 16 edges
    for (int rb = 0; rb < gne; rb += kGroupRound) {
        const int es = wave * EPW + g, le = rb + es;
        const bool ev = le < gne;
        const int4 info = ev ? sInfo[le] : make_int4(0, 0, 0, 0);
        const int cam = info.x;
        double* P = sP + kGRecP * es;
        double* Gbe = sGb + 56 * es;
        if (rb > 0 && ev) stage(info.z, 0, min(info.w, kGChunk));
        if (ev) {
            group_prologue<MODEL, BACK, L>(sph + 24 * seq[le], ctab + 24 * cam, sds, info.y, sub, rec + kGRec * le, P, Gbe);
            const double* kt = ktab + kGIntr * cam;
            for (int k = sub; k < (PRISM == 2 ? 27 : 18); k += L) P[12 + k] = kt[k];
        }
        wave_sync_lds();
        if (rb == 0) SSTAMP(stp, 3, 0);
        // ---- the sweep (k_edge's): FP64 projection + 2 x 6 J' rows, float32 residual, 27 sums
        double acc[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) acc[q] = 0.0;
        const int nn = info.w;
        for (int cc0 = 0;; cc0 += kGChunk) {
            if (cc0 >= nn) break;
            const int cn = min(nn - cc0, kGChunk);
            if (cc0 > 0) {
                wave_sync_lds();   // the previous chunk is consumed
                stage(info.z, cc0, cn);
                wave_sync_lds();
            }
#pragma unroll 1
            for (int i = sub; i < cn; i += L) {
                int po = 0;
                asm volatile("" : "+v"(po));
                const double* Pq = P + po;
                double R[9], T[3], kd[12];
#pragma unroll
                for (int q = 0; q < 9; ++q) R[q] = Pq[q];
#pragma unroll
                for (int q = 0; q < 3; ++q) T[q] = Pq[9 + q];
#pragma unroll
                for (int q = 0; q < 12; ++q) kd[q] = Pq[18 + q];
                const double fx = Pq[12], fy = Pq[13], cx = Pq[14], cy = Pq[15], sk = Pq[16], xi = Pq[17];
                const double X = sC[0][i][g], Y = sC[1][i][g], Z = sC[2][i][g];
                const float ou = sC[3][i][g], ov = sC[4][i][g];
                double Yr[3], D[6];
                float u, v;
                if (MODEL == MCC_MODEL_OMNI)
                    omni_corner(R, T, kd, fx, fy, cx, cy, sk, xi, X, Y, Z, Yr, u, v, D);
                else
                    pinhole_corner<RATIONAL, PRISM>(R, T, kd, fx, fy, cx, cy, X, Y, Z, Yr, u, v, D, Pq + 30);
                const float euf = ou - u, evf = ov - v;   // fl32(imagePoints - imagePoints2)
                if (a.resid) {
                    const size_t c = (size_t)info.z + cc0 + i;
                    a.resid[2 * c] = euf;
                    a.resid[2 * c + 1] = evf;
                }
                const double eu = euf, ev2 = evf;
                double ju[6], jv[6];   // J' rows: [Y x d, d]
                ju[0] = Yr[1] * D[2] - Yr[2] * D[1];
                ju[1] = Yr[2] * D[0] - Yr[0] * D[2];
                ju[2] = Yr[0] * D[1] - Yr[1] * D[0];
                ju[3] = D[0]; ju[4] = D[1]; ju[5] = D[2];
                jv[0] = Yr[1] * D[5] - Yr[2] * D[4];
                jv[1] = Yr[2] * D[3] - Yr[0] * D[5];
                jv[2] = Yr[0] * D[4] - Yr[1] * D[3];
                jv[3] = D[3]; jv[4] = D[4]; jv[5] = D[5];
                int q = 0;
#pragma unroll
                for (int r = 0; r < 6; ++r)
#pragma unroll
                    for (int s2 = r; s2 < 6; ++s2, ++q) acc[q] = fma(jv[r], jv[s2], fma(ju[r], ju[s2], acc[q]));
#pragma unroll
                for (int r = 0; r < 6; ++r) acc[21 + r] = fma(jv[r], ev2, fma(ju[r], eu, acc[21 + r]));
            }
        }
        // ---- butterfly (k_edge's strided reduce-scatter over the edge's 16 lanes), then the chain
        if (rb == 0) SSTAMP(stp, 4, 0);
        int tq = lane;
        asm volatile("" : "+v"(tq));
        strided_reduce_scatter<L>(acc, tq);
        const int gq = tq % EPW, sq = tq / EPW;
        const int base = strided_rs_base<L>(tq);
        wave_sync_lds();   // the corners are consumed: the chain records overwrite them
        {
            GroupChain& CW = sCH[gq];
#pragma unroll
            for (int q = 0; q < 32 / L; ++q) {
                const int idx = base + q;
                if (idx < 21) {
                    int r, s2;
                    tri6(idx, r, s2);
                    CW.A[r * 6 + s2] = acc[q];
                    CW.A[s2 * 6 + r] = acc[q];
                } else if (idx < 27) {
                    CW.B[idx - 21] = acc[q];
                }
            }
        }
        wave_sync_lds();
        {
            const int eq = rb + wave * EPW + gq;
            group_chain(sCH[gq], sGb + 56 * (wave * EPW + gq), sq, eq < gne, rec + kGRec * (eq < gne ? eq : 0));
        }
        wave_sync_lds();   // this wave's chain records are consumed before the next round's corners
        if (rb == 0) SSTAMP(stp, 5, 0);
    }
#ifdef MCC_DIAG
    if (stp && lane == 0 && wave < 16) {   // per wave: the rounds done (slots 16 + wave)
        __builtin_amdgcn_sched_barrier(0);
        stp[16 + wave] = (long long)MCC_DIAG_CLOCK();
        __builtin_amdgcn_sched_barrier(0);
    }
#endif
    __syncthreads();
    SSTAMP(stp, 6, 0);

    // ---- phase B: k_photo's photo work on the group's LDS records
    constexpr int ES = kGRec;
    double* sE = rec;
    // photo q's Hpp / gp column sums in edge order
    if (tid < 27 * np) {
        const int q = tid / 27, col27 = tid % 27;
        double s = 0.0;
        for (int le = sph0[q]; le < sph0[q + 1]; ++le) s += rec[kGRec * le + 64 + col27];
        s27[28 * q + col27] = s;
    }
    __syncthreads();
    SSTAMP(stp, 7, 0);
    if (tid < np) {   // one lane per photo: Cholesky Hpp = L L^T, Li = L^-1, v = Li gp, z' = Li^T v
        const int q = tid, photo = p0 + q;
        double A[21], gs[6], Lm[6][6], Li[6][6];
        const double2* S2 = reinterpret_cast<const double2*>(s27 + 28 * q);
#pragma unroll
        for (int k = 0; k < 14; ++k) {
            const double2 w = S2[k];
            if (2 * k < 21) A[2 * k] = w.x; else gs[2 * k - 21] = w.x;
            if (2 * k + 1 < 21) A[2 * k + 1] = w.y; else if (2 * k + 1 < 27) gs[2 * k + 1 - 21] = w.y;
        }
        bool bad = false;
        double idg[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double d = A[6 * j - j * (j - 1) / 2];
#pragma unroll
            for (int k = 0; k < j; ++k) d -= Lm[j][k] * Lm[j][k];
            bad |= !(d > 0.0);
            const double sd = sqrt(d > 0.0 ? d : 1.0);
            const double is = 1.0 / sd;
            Lm[j][j] = sd;
            idg[j] = is;
#pragma unroll
            for (int i = j + 1; i < 6; ++i) {
                double t = A[6 * j - j * (j - 1) / 2 + (i - j)];   // Hpp(j, i) = Hpp(i, j)
#pragma unroll
                for (int k = 0; k < j; ++k) t -= Lm[i][k] * Lm[j][k];
                Lm[i][j] = t * is;
            }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // column j of Li: forward substitution of L x = e_j
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (i < j) { Li[i][j] = 0.0; continue; }
                double t = i == j ? 1.0 : 0.0;
#pragma unroll
                for (int k = j; k < i; ++k) t -= Lm[i][k] * Li[k][j];
                Li[i][j] = t * idg[i];
            }
        }
        double vv[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k <= i; ++k) t += Li[i][k] * gs[k];
            vv[i] = t;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            double t = 0.0;
#pragma unroll
            for (int i = j; i < 6; ++i) t += Li[i][j] * vv[i];
            a.zp[6 * (size_t)photo + j] = t;
            a.gp_tot[6 * (size_t)photo + j] = gs[j];
            sv[6 * q + j] = vv[j];
        }
        double2* L2 = reinterpret_cast<double2*>(sLi + 36 * q);
#pragma unroll
        for (int k = 0; k < 18; ++k) L2[k] = make_double2(Li[(2 * k) / 6][(2 * k) % 6], Li[(2 * k + 1) / 6][(2 * k + 1) % 6]);
        if (bad || photo == a.fault_photo) atomicOr(&st->error, kErrPhotoNotPD);
        if (a.fold) {   // the norm chunk's input: ||G||^2, ||x||^2 and the not-PD flag (sc1, each word its flag)
            double* fw = a.fnorm + 4 * (size_t)photo;
            st_sc1_x2(fw, sxn[16 * q + 6], sxn[16 * q + 7]);
            st_sc1(fw + 2, bad || photo == a.fault_photo ? 1.0 : 0.0);
        }
    }
    __syncthreads();
    SSTAMP(stp, 8, 0);
    for (int t = tid; t < 6 * gne; t += NT) {   // task (edge, row i): U row i in place of Hgp row i, Y' row i
        const int le = t / 6, i = t % 6;
        double h[6], li[36], u[6], y[6];
        double2* H2 = reinterpret_cast<double2*>(sE + ES * le + 22 + 6 * i);
        const double2* I2 = reinterpret_cast<const double2*>(sLi + 36 * seq[le]);
#pragma unroll
        for (int q = 0; q < 3; ++q) { const double2 w = H2[q]; h[2 * q] = w.x; h[2 * q + 1] = w.y; }
#pragma unroll
        for (int q = 0; q < 18; ++q) { const double2 w = I2[q]; li[2 * q] = w.x; li[2 * q + 1] = w.y; }
        const bool gl = sgb[le] >= 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // U[i][j] = sum_{k <= j} Hgp[i][k] Li[j][k]
            double w = 0.0;
#pragma unroll
            for (int k = 0; k <= j; ++k) w += h[k] * li[6 * j + k];
            u[j] = gl ? w : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {   // Y'[i][j] = sum_{k >= j} U[i][k] Li[k][j]
            double w = 0.0;
#pragma unroll
            for (int k = j; k < 6; ++k) w += u[k] * li[6 * k + j];
            y[j] = w;
        }
        double2* G2 = reinterpret_cast<double2*>(a.Y + 36 * (size_t)(ge0 + le) + 6 * i);
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            H2[q] = make_double2(u[2 * q], u[2 * q + 1]);
            G2[q] = make_double2(y[2 * q], y[2 * q + 1]);
        }
    }
    __syncthreads();
    SSTAMP(stp, 9, 0);
    // the group's Schur pair products per camera-pair block -> its slot (k_photo's pair tasks)
    int H = 1;
    while (H < 32 && 6 * nq * 2 * H <= (NT < MCC_GROUP_PAIR_THREADS ? NT : MCC_GROUP_PAIR_THREADS)) H *= 2;
    for (int t = tid; t < 6 * nq * H; t += NT) {
        const int h = t % H, k = t / H / 6, i0 = (t / H) % 6;
        const int4 pqv = spq[k];   // {first contribution, count, diagonal block << 1, slot offset}
        const bool diag = (pqv.z & 2) != 0;
        double acc[6], racc = 0.0, jacc = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[j] = 0.0;
#pragma unroll 1
        for (int c = pqv.x + h; c < pqv.x + pqv.y; c += H) {
            const unsigned w = scn[c];
            const int ea = w & 255, eb = (w >> 8) & 255, q = w >> 17;
            const bool self = (w >> 16) & 1;
            const double2* Y2 = reinterpret_cast<const double2*>(sE + ES * ea + 22 + 6 * i0);
            const double2* B2 = reinterpret_cast<const double2*>(sE + ES * eb + 22);
            double y[6];
#pragma unroll
            for (int qq = 0; qq < 3; ++qq) { const double2 v = Y2[qq]; y[2 * qq] = v.x; y[2 * qq + 1] = v.y; }
            const double* Hgg = sE + ES * ea;
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double hb[6];
#pragma unroll
                for (int qq = 0; qq < 3; ++qq) { const double2 v = B2[3 * j + qq]; hb[2 * qq] = v.x; hb[2 * qq + 1] = v.y; }
                double d = 0.0;
#pragma unroll
                for (int kk = 0; kk < 6; ++kk) d += y[kk] * hb[kk];
                double hv = 0.0;
                if (self) {
                    const int rr = i0 < j ? i0 : j, cc = i0 < j ? j : i0;
                    hv = Hgg[rr * 6 - rr * (rr - 1) / 2 + (cc - rr)];
                }
                acc[j] += self ? hv - d : -d;
            }
            if (diag && self) {
                double d = 0.0;
#pragma unroll
                for (int kk = 0; kk < 6; ++kk) d += y[kk] * sv[6 * q + kk];
                const double gg = sE[ES * ea + 58 + i0];
                racc += gg - d;
                jacc += gg;
            }
        }
        for (int o = 1; o < H; o <<= 1) {   // the H parts are lanes t - h .. t - h + H - 1 (H | 64)
#pragma unroll
            for (int j = 0; j < 6; ++j) acc[j] += __shfl_xor(acc[j], o);
            racc += __shfl_xor(racc, o);
            jacc += __shfl_xor(jacc, o);
        }
        if (h == 0) {   // write-through (sc1): the folded items poll these words in this launch
            double* out = a.pairprod + (size_t)pqv.w;
#ifdef MCC_SLOT_PLAIN   // (A/B builds only)
#pragma unroll
            for (int j = 0; j < 6; ++j) out[i0 * 6 + j] = acc[j];
            if (diag) {
                out[36 + i0] = racc;
                out[42 + i0] = jacc;
            }
#else
#pragma unroll
            for (int j = 0; j < 6; j += 2) st_sc1_x2(out + i0 * 6 + j, acc[j], acc[j + 1]);
            if (diag) {
                st_sc1(out + 36 + i0, racc);
                st_sc1(out + 42 + i0, jacc);
            }
#endif
        }
    }
#ifdef MCC_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    SSTAMP(stp, 10, 0);
#endif
    return true;
}

// FIRST (a test instantiation, omnidir only: LinArgs::fold_first): the trailing workgroups (spare,
// items, norm chunks, final) take the lowest grid indices and the groups the rest.  A separate
// instantiation: remapping the index in the product kernel cost its register allocation ~230 more
// SGPR-spill reloads and config4 ~0.2-0.4 us per step.
template <int MODEL, bool RATIONAL, int PRISM, bool BACK, int L, bool FIRST = false>
__global__ __launch_bounds__(kGroupRound * L, MCC_GROUP_OCC * 16 / L) void k_group(LinArgs a) {
    constexpr int NT = kGroupRound * L;
    static_assert(L == 16 || L == 32, "k_group: 16 or 32 lanes per edge");
    State* st = a.state;
    const int tid = threadIdx.x;
    int grp = blockIdx.x;
    if (FIRST) {   // (test layout: the trailing workgroups first, then the groups)
        const int nlead = (int)gridDim.x - a.n_pgroups;
        grp = grp < nlead ? a.n_pgroups + grp : grp - nlead;
    }
    if (a.ssinv && grp == a.n_pgroups) {   // the spare workgroup: the previous system's inverse (m <= 30 warm solve)
        extern __shared__ __attribute__((aligned(16))) double smem_spare[];
        small_inverse(a, smem_spare, false);
        return;
    }
    // the folded reduction's task (item, norm chunk, the final): a trailing workgroup's by its index, or
    // (fold_dyn) a group's next by ticket once its own work is done -- ONE call site of the task code
    // per kernel (two made k_group half as large again and config4 1 us slower per step).  (Not in the
    // tilted sensor's variants: at 256 VGPRs the ticket tail tipped their sweep into a spill; the host
    // keeps the trailing task workgroups there.)
    int task;
    if (a.fold && grp > a.n_pgroups - (a.ssinv ? 0 : 1)) {
        if (st->done) return;
        task = grp - a.n_pgroups - (a.ssinv ? 1 : 0);
    } else {
        if (!group_body<MODEL, RATIONAL, PRISM, BACK, L>(a, grp) || PRISM == 2 || !a.fold_dyn) return;
        __shared__ int s_task;
        __syncthreads();   // the group's LDS is free
        if (tid == 0) {
            const int t = __hip_atomic_fetch_add(a.fold_ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the last taker resets the ticket for the next launch (every other taker has drawn)
            if (t == a.n_pgroups - 1) __hip_atomic_store(a.fold_ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_task = t;
        }
        __syncthreads();
        task = s_task;
    }
    if (task < a.fsa.n_items) fold_item(a, task);
    else if (task < a.fold_parts) fold_chunk(a, task - a.fsa.n_items);
    else if (task == a.fold_parts) fold_final<NT>(a);
}

// ---------------------------------------------------------------- k_prep4
// The three-kernel split step's first kernel (k_prep -> k_edge -> k_photo) with the edge prologue
// spread over 4 lanes: one wave per group of consecutive photos (at most kPrepPhotos photos and
// kPrepEdges edges, or one photo with more, in rounds of 16 edges), doing
//   - every load in one round trip after the group's ranges (k_group's phase 0: dg, the cameras,
//     the photos' x and z', the edge records, the first Y' column of each (edge, k) task);
//   - the pending photo update x = fl32(x + fl32(alpha (z' - sum_e Y'_e^T dg))) in edge order
//     (k_prep's; src/multicalib.cpp:482-501) and the stop test's norm partials;
//   - one Rodrigues pass over the photos, the cameras and the double-side transform (lanes
//     running the same code on different poses);
//   - group_prologue by 4 lanes per edge (lanes own entries of the 3 x 3 products; the scalar
//     chain -- m2v, the float32 pose's Rodrigues, the Jacobian coefficients -- per lane), writing
//     erec (R, T) and echain (the chain maps' nonzero blocks) for k_edge.
// One lane per edge (k_prep, prep_lanes = 1) leaves the matrix work of an edge on one lane; four
// lanes cut each wave's instruction stream and write each record 4 doubles per edge at a time.
#ifndef MCC_PREP4_WAVES
#define MCC_PREP4_WAVES 2
#endif
template <int MODEL, bool BACK>
__global__ __launch_bounds__(64, MCC_PREP4_WAVES) void k_prep4(LinArgs a) {
    const State* st = a.state;
    const int tid = threadIdx.x, grp = blockIdx.x;
    const int done = st->done, pending = st->pending;
    const double alpha_prev = st->alpha;   // step factor of the pending update
    const int p0 = a.prep_ptr[grp], np = a.prep_ptr[grp + 1] - p0;
    const int ge0 = a.prep_edge[grp], gne = a.prep_edge[grp + 1] - ge0;
    if (done) return;
    long long* stp = a.stamps ? a.stamps + kStampStride * (size_t)grp + 8 : nullptr;   // MCC_DIAG: slots 8..11
    SSTAMP(stp, 0, 0);
    const int C = a.n_cams, m = a.global_dim;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const PrepLayout PL = prep_layout(C, BACK);
    double* tab = smem + PL.tab;     // photos [0, kPrepPhotos), cameras, the double-side transform
    double* S = smem + PL.S;
    double* spart = S;               // the update's partial sums (consumed before the prologues)
    double* sdg = smem + PL.sdg;
    double* sxn = smem + PL.sxn;
    double* scam = smem + PL.scam;   // camera (rvec, tvec) [6C], the double-side transform [6]
    int* ib = reinterpret_cast<int*>(smem + PL.ndoubles);
    int4* sInfo = reinterpret_cast<int4*>(ib + PL.iInfo);
    int* sgb = ib + PL.iGb;
    int* sph0 = ib + PL.iPh;
    constexpr int SW = BACK ? 84 : 42;
    // ---- phase 0: one round trip
    for (int t = tid; t < m; t += 64) sdg[t] = a.dg[t];
    for (int t = tid; t < 6 * C; t += 64) {
        const int c = t / 6, k = t % 6;
        scam[t] = MODEL == MCC_MODEL_DOUBLESIDE ? (double)a.cam_rt[t]
                                                : (c == 0 ? 0.0 : (double)a.x[6 * (c - 1) + k]);   // src/mymulticalib.cpp:721-725
    }
    if (BACK && tid < 6) scam[6 * C + tid] = MODEL == MCC_MODEL_DOUBLESIDE ? (double)a.x[tid] : a.ds_rt[tid];
    if (tid <= np) sph0[tid] = a.photo_ptr[p0 + tid] - ge0;
    for (int t = tid; t < gne; t += 64) {
        sInfo[t] = a.edge_info[ge0 + t];
        sgb[t] = a.gblock[ge0 + t];
    }
    const int pq = tid / 6, pk = tid % 6;
    const bool ptask = pq < np;
    float xo = 0.f;
    double zk = 0.0;
    double2 pn0 = make_double2(0.0, 0.0);   // the fold without a pending update: the norms k_backsub left
    if (ptask) {
        xo = a.x[m + 6 * (size_t)(p0 + pq) + pk];
        if (pending) zk = a.zp[6 * (size_t)(p0 + pq) + pk];
        else if (a.fold && pk == 0) pn0 = *reinterpret_cast<const double2*>(a.photo_norm + 2 * (size_t)(p0 + pq));
    }
    double y0[6];
    int gb0 = -1;
    if (pending && tid < 6 * gne) {
        const int le = tid / 6, k = tid % 6;
        gb0 = a.gblock[ge0 + le];
        const double* Ye = a.Y + 36 * (size_t)(ge0 + le);
#pragma unroll
        for (int i = 0; i < 6; ++i) y0[i] = Ye[6 * i + k];
    }
    wave_sync_lds();
    // ---- the pending update: (edge, k) partials, then photo q's component k in edge order
    if (pending) {
        for (int t = tid; t < 6 * gne; t += 64) {
            const int le = t / 6, k = t % 6;
            int gbl = gb0;
            double y[6];
            if (t == tid) {
#pragma unroll
                for (int i = 0; i < 6; ++i) y[i] = y0[i];
            } else {
                gbl = sgb[le];
                const double* Ye = a.Y + 36 * (size_t)(ge0 + le);
#pragma unroll
                for (int i = 0; i < 6; ++i) y[i] = Ye[6 * i + k];
            }
            const double* d = sdg + 6 * (gbl < 0 ? 0 : gbl);
            double sk = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) sk += y[i] * d[i];
            spart[6 * le + k] = gbl < 0 ? 0.0 : sk;
        }
    }
    wave_sync_lds();
    if (ptask) {
        float xn = xo;
        double Gk = 0.0;
        if (pending) {
            double t = zk;
            for (int le = sph0[pq]; le < sph0[pq + 1]; ++le) t -= spart[6 * le + pk];
            const float G = (float)(alpha_prev * t);   // G = alpha*delta -> CV_32F (:491-496)
            xn = xo + G;                                // x = x + G (:501)
            a.x[m + 6 * (size_t)(p0 + pq) + pk] = xn;
            Gk = (double)G;
        }
        sxn[16 * pq + pk] = (double)xn;
        sxn[16 * pq + 8 + pk] = Gk;
    }
    wave_sync_lds();
    SSTAMP(stp, 1, 0);
    if (pending && ptask && pk == 0) {   // ||G||^2, ||x||^2 partials of the applied update (stop test)
        const double* xs = sxn + 16 * pq;
        double g2 = 0.0, x2 = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            g2 += xs[8 + q] * xs[8 + q];
            x2 += xs[q] * xs[q];
        }
        a.photo_norm[2 * (size_t)(p0 + pq)] = g2;
        a.photo_norm[2 * (size_t)(p0 + pq) + 1] = x2;
    }
    // ---- one Rodrigues pass: photos (Jr), cameras (Jl), the double-side transform (Jr)
    for (int t = tid; t < np + C + (BACK ? 1 : 0); t += 64) {
        const double* src;
        double* out;
        double sgn;
        if (t < np) {
            src = sxn + 16 * t; out = tab + 24 * t; sgn = -1.0;
        } else if (t < np + C) {
            src = scam + 6 * (t - np); out = tab + 24 * (kPrepPhotos + t - np); sgn = 1.0;
        } else {
            src = scam + 6 * C; out = tab + 24 * (kPrepPhotos + C); sgn = -1.0;
        }
        const double om[3] = {src[0], src[1], src[2]};
        Rot r;
        rodrigues_v2m(om, r);
        double J[9];
        so3_jac(om, r, sgn, J);
#pragma unroll
        for (int k = 0; k < 9; ++k) { out[k] = r.R[k]; out[9 + k] = J[k]; }
#pragma unroll
        for (int k = 0; k < 3; ++k) out[18 + k] = src[3 + k];
    }
    wave_sync_lds();
    SSTAMP(stp, 2, 0);
    // ---- the edge prologues: rounds of 16 edges, 4 lanes each -> erec, echain
    const int es = tid >> 2, sub = tid & 3;
    for (int rb = 0; rb < gne; rb += kPrepEdges) {
        const int le = rb + es;
        if (le < gne) {
            const int4 info = sInfo[le];
            int q = 0;
            while (q + 1 < np && sph0[q + 1] <= le) ++q;
            const size_t e = (size_t)ge0 + le;
            group_prologue<MODEL, BACK, 4, 27>(tab + 24 * q, tab + 24 * (kPrepPhotos + info.x), tab + 24 * (kPrepPhotos + C),
                                               info.y, sub, S + SW * es, a.erec + 12 * e, a.echain + 54 * e);
        }
        wave_sync_lds();   // this round's scratch is consumed before the next round's
    }
#ifdef MCC_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    SSTAMP(stp, 3, 0);
}
