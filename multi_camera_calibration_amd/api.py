"""Python binding of libmcc.so (include/mcc.h) -- the MI355X hot path behind the reference's
optimiser seam.

Mirrors the reference's operator interface for this path (cv::multicalib, include/opencv2/ccalib/
multicalib.hpp:155-188):

    BundleAdjuster.optimize_extrinsics(...)       -> MultiCameraCalibration::optimizeExtrinsics
    BundleAdjuster.compute_jacobian_extrinsic(x)  -> computeJacobianExtrinsic(x, JTJ_inv, JTE, deltaX)
    BundleAdjuster.compute_project_error(x)       -> computeProjectError(x)

There is no CPU fallback: if libmcc.so is missing or the device is unusable the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np

from . import rig as _rig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MCC_LIB") or os.path.join(_HERE, "libmcc.so")   # MCC_LIB: libmcc_diag.so for stamps
HEADER = os.path.join(os.path.dirname(_HERE), "include", "mcc.h")
HEADERS = [HEADER, os.path.join(os.path.dirname(_HERE), "include", "mcc_omnidir.h")]   # the C ABI of libmcc.so

_i32p = ctypes.POINTER(ctypes.c_int)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)

MCC_CRIT_COUNT, MCC_CRIT_EPS, MCC_CRIT_COUNT_EPS = 1, 2, 3


class MccError(RuntimeError):
    pass


class _Desc(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int), ("n_cams", ctypes.c_int), ("n_photos", ctypes.c_int),
                ("n_edges", ctypes.c_int), ("edge_cam", _i32p), ("edge_photo", _i32p),
                ("edge_side", _i32p), ("edge_off", _i32p), ("edge_n", _i32p),
                ("obj", _f32p), ("img", _f32p), ("nd", ctypes.c_int), ("K", _f32p),
                ("D", _f32p), ("xi", _f32p), ("ds_pose", _f64p), ("cam_pose", _f32p),
                ("device", ctypes.c_int)]


class _OmniDesc(ctypes.Structure):
    _fields_ = [("n_views", ctypes.c_int), ("view_off", _i32p), ("obj", _f64p), ("img", _f64p),
                ("flags", ctypes.c_int), ("device", ctypes.c_int)]


_LIB = None


HOST_LIB_PATH = os.path.join(_HERE, "libmcc_host.so")
SAMPLE_PATH = os.path.join(_HERE, "build", "multi_cameras_calibration")
OMNI_SAMPLE_PATH = os.path.join(_HERE, "build", "omni_calibration")
# the reference's samples/multi_cameras_calibration.cpp compiled unchanged against
# include/opencv2/ccalib/*.hpp (built only where the reference tree exists; the binary travels)
REF_SAMPLE_SRC = "/root/reference/samples/multi_cameras_calibration.cpp"
REF_SAMPLE_PATH = os.path.join(_HERE, "build", "ref_multi_cameras_calibration")


def build(force: bool = False) -> str:
    """Compile libmcc.so in-tree for gfx950 (hipcc cross-compiles without a GPU), and the host
    side of the sample flow (libmcc_host.so, build/multi_cameras_calibration) with g++."""
    inc = os.path.dirname(HEADER)
    srcs = [os.path.join(_HERE, d, f) for d in ("csrc", "host", "samples") for f in os.listdir(os.path.join(_HERE, d))]
    srcs += [os.path.join(inc, f) for f in os.listdir(inc)]
    outs = [LIB_PATH, HOST_LIB_PATH, SAMPLE_PATH, OMNI_SAMPLE_PATH]
    stale = any(not os.path.exists(o) for o in outs) or any(
        os.path.getmtime(s) > min(os.path.getmtime(o) for o in outs) for s in srcs)
    if force or stale:
        subprocess.run(["make", "-s", "--no-print-directory", "-C", _HERE, "-j8", "all"], check=True)
    if os.path.exists(REF_SAMPLE_SRC):
        # optional: the reference's sample compiled against the compatibility headers (the test
        # that needs it, tests/test_reference_sample.py, builds it itself and reports a failure);
        # a drifted header must not keep libmcc.so from loading
        r = subprocess.run(["make", "-s", "--no-print-directory", "-C", _HERE, "ref_sample"],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            import warnings
            warnings.warn(f"reference sample build failed (libmcc.so is unaffected):\n{r.stdout[-2000:]}")
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise MccError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        L.mcc_last_error.restype = ctypes.c_char_p
        L.mcc_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(_Desc)]
        for name in ("mcc_nparams", "mcc_global_dim"):
            getattr(L, name).argtypes = [ctypes.c_void_p]
        L.mcc_destroy.argtypes = [ctypes.c_void_p]
        L.mcc_destroy.restype = None
        L.mcc_set_params.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int]
        L.mcc_get_params.argtypes = [ctypes.c_void_p, _f32p, ctypes.c_int]
        L.mcc_linearize_solve.argtypes = [ctypes.c_void_p, _f64p, _f64p]
        L.mcc_optimize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, _f32p,
                                   _i32p, _f64p]
        L.mcc_step.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.mcc_synchronize.argtypes = [ctypes.c_void_p]
        L.mcc_check.argtypes = [ctypes.c_void_p]
        L.mcc_project_error.argtypes = [ctypes.c_void_p, _f32p, _f32p, _f64p]
        L.mcc_debug_residuals.argtypes = [ctypes.c_void_p, _f32p, _f32p]
        # (round-6 entry points: absent from an older build loaded through MCC_LIB for an A/B)
        if hasattr(L, "mcc_optimize_profile"):
            L.mcc_optimize_profile.argtypes = [ctypes.c_void_p, _f64p, _f64p, _i32p, _i32p, _i32p]
        if hasattr(L, "mcc_debug_delays"):
            L.mcc_debug_delays.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L.mcc_timing_begin.argtypes = [ctypes.c_void_p]
        L.mcc_timing_end.argtypes = [ctypes.c_void_p, _f64p, _f64p, _i32p]
        L.mcc_timing_exchange.argtypes = [ctypes.c_void_p, _f64p, _i32p]
        L.mcc_timing_windows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _f64p, _i32p]
        L.mcc_timing_linearize.argtypes = [ctypes.c_void_p, ctypes.c_int, _f64p]
        L.mcc_project_error_detail.argtypes = [ctypes.c_void_p, _f32p, _f32p, _f32p, _f32p,
                                               ctypes.POINTER(ctypes.c_longlong), _f64p]
        L.mcc_problem_stats.argtypes = [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_longlong)] * 4
        L.mcc_solve_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]
        L.mcc_problem_path.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.mcc_comm_unique_id.argtypes = [ctypes.c_char_p]
        L.mcc_comm_init.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.mcc_comm_allreduce_max.argtypes = [ctypes.c_void_p, _f64p]
        L.mcc_comm_barrier.argtypes = [ctypes.c_void_p]
        L.mcc_partition_photos.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, _i32p, ctypes.c_int, _i32p]
        L.mcc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
        L.mcc_debug_solve.argtypes = [ctypes.c_int, ctypes.c_int, _f64p, _f64p, ctypes.c_int, _f64p,
                                      ctypes.POINTER(ctypes.c_longlong)]
        L.mcc_peer_handle.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.mcc_peer_init.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.mcc_peer_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
        # include/mcc_omnidir.h
        L.mcc_omnicalib_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(_OmniDesc)]
        L.mcc_omnicalib_destroy.argtypes = [ctypes.c_void_p]
        L.mcc_omnicalib_destroy.restype = None
        L.mcc_omnicalib_nparams.argtypes = [ctypes.c_void_p]
        L.mcc_omnicalib_jacobian.argtypes = [ctypes.c_void_p, _f64p, ctypes.c_int, _f64p, _f64p]
        L.mcc_omnicalib_optimize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, _f64p,
                                             _i32p, _f64p]
        L.mcc_omnicalib_rms.argtypes = [ctypes.c_void_p, _f64p, _f64p]
        L.mcc_omnicalib_time_steps.argtypes = [ctypes.c_void_p, _f64p, ctypes.c_int, _f64p]
        L.mcc_omnidir_initialize.argtypes = [ctypes.c_int, _i32p, _f64p, _f64p, ctypes.c_int, ctypes.c_int, _f64p,
                                             _f64p, _f64p, _f64p, _i32p, _i32p]
        L.mcc_omnidir_calibrate.argtypes = [ctypes.c_int, _i32p, _f64p, _f64p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                            _f64p, _f64p, _f64p, _f64p, _f64p, _i32p, _i32p, _f64p, _i32p]
        _LIB = L
    return _LIB


def debug_solve(S, r, reps=0, stamps=False, device=0):
    """k_solve's m > 30 elimination alone on the SPD system S x = r (mcc_debug_solve): returns x,
    the average device microseconds per solve over `reps` launches (None without reps) and, with
    stamps, the first launch's 64 per-phase s_memtime stamps."""
    S = np.asarray(S, np.float64)
    m = S.shape[0]
    iu = np.triu_indices(m)
    packed = np.ascontiguousarray(np.concatenate([S[iu], np.asarray(r, np.float64)]))
    x = np.zeros(m, np.float64)
    us = np.zeros(1, np.float64)
    st = np.zeros(64, np.int64)
    _check(lib().mcc_debug_solve(device, m, _ptr(packed, _f64p), _ptr(x, _f64p), int(reps), _ptr(us, _f64p),
                                 st.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)) if stamps else None),
           "mcc_debug_solve")
    return x, (float(us[0]) if reps else None), (st if stamps else None)


def declared_symbols():
    """Every function the C-ABI headers of libmcc.so (include/mcc.h, include/mcc_omnidir.h) declare."""
    txt = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(mcc_[a-z_]+)\s*\(", txt, re.M)))


def _check(rc, what):
    if rc != 0:
        raise MccError(f"{what} failed ({rc}): {lib().mcc_last_error().decode()}")


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def partition_photos(prob, nranks):
    """Greedy corner-count balance of photo vertices over ranks (mcc_partition_photos)."""
    out = np.zeros(prob.n_photos, np.int32)
    ep = np.ascontiguousarray(prob.edge_photo, np.int32)
    en = np.ascontiguousarray(prob.edge_n, np.int32)
    _check(lib().mcc_partition_photos(prob.n_photos, prob.n_edges, _ptr(ep, _i32p), _ptr(en, _i32p),
                                      nranks, _ptr(out, _i32p)), "mcc_partition_photos")
    return out


def file_allgather(directory: str, rank: int, world: int, payload: bytes, timeout: float = 300.0) -> list:
    """All-gather of small byte strings among the processes of one node through files in
    `directory` (RCCL unique id and peer inbox handles; no torch, no RCCL needed)."""
    import time
    os.makedirs(directory, exist_ok=True)
    tmp = os.path.join(directory, f".r{rank}.tmp")
    with open(tmp, "wb") as f:
        f.write(payload)
    os.replace(tmp, os.path.join(directory, f"r{rank}"))
    out, t0 = [None] * world, time.time()
    while any(v is None for v in out):
        for q in range(world):
            fn = os.path.join(directory, f"r{q}")
            if out[q] is None and os.path.exists(fn):
                with open(fn, "rb") as f:
                    out[q] = f.read()
        if time.time() - t0 > timeout:
            raise MccError(f"timed out waiting for {world} ranks in {directory}")
        time.sleep(0.02)
    return out


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(lib().mcc_comm_unique_id(buf), "mcc_comm_unique_id")
    return buf.raw


class BundleAdjuster:
    """One mcc_problem: the reference's BA state for one (local) set of photo vertices."""

    def __init__(self, prob: "_rig.Problem", device: int = 0):
        self.prob = prob
        self._keep = []

        def arr(a, dt):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dt)
            self._keep.append(a)
            return a
        d = _Desc()
        d.model, d.n_cams, d.n_photos, d.n_edges = prob.model, prob.n_cams, prob.n_photos, prob.n_edges
        d.edge_cam = _ptr(arr(prob.edge_cam, np.int32), _i32p)
        d.edge_photo = _ptr(arr(prob.edge_photo, np.int32), _i32p)
        d.edge_side = _ptr(arr(prob.edge_side, np.int32), _i32p)
        d.edge_off = _ptr(arr(prob.edge_off, np.int32), _i32p)
        d.edge_n = _ptr(arr(prob.edge_n, np.int32), _i32p)
        d.obj = _ptr(arr(prob.obj, np.float32), _f32p)
        d.img = _ptr(arr(prob.img, np.float32), _f32p)
        d.nd = prob.nd
        d.K = _ptr(arr(prob.K, np.float32), _f32p)
        d.D = _ptr(arr(prob.D, np.float32), _f32p)
        d.xi = _ptr(arr(prob.xi, np.float32), _f32p) if prob.model == _rig.OMNI else None
        d.ds_pose = _ptr(arr(prob.ds_pose, np.float64), _f64p) if prob.ds_pose is not None else None
        d.cam_pose = _ptr(arr(prob.cam_pose, np.float32), _f32p) if prob.cam_pose is not None else None
        d.device = device
        h = ctypes.c_void_p()
        _check(lib().mcc_create(ctypes.byref(h), ctypes.byref(d)), "mcc_create")
        self.h = h
        self.P = lib().mcc_nparams(h)
        self.m = lib().mcc_global_dim(h)

    def close(self):
        if getattr(self, "h", None):
            lib().mcc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- state
    def set_params(self, x):
        x = np.ascontiguousarray(x, np.float32)
        _check(lib().mcc_set_params(self.h, _ptr(x, _f32p), x.size), "mcc_set_params")

    def get_params(self):
        x = np.zeros(self.P, np.float32)
        _check(lib().mcc_get_params(self.h, _ptr(x, _f32p), self.P), "mcc_get_params")
        return x

    # -- the reference seam
    def compute_jacobian_extrinsic(self, x):
        """(deltaX, JTE) of one linearisation at x (computeJacobianExtrinsic)."""
        self.set_params(x)
        delta = np.zeros(self.P)
        jte = np.zeros(self.P)
        _check(lib().mcc_linearize_solve(self.h, _ptr(delta, _f64p), _ptr(jte, _f64p)), "mcc_linearize_solve")
        return delta, jte

    def optimize_extrinsics(self, x0, crit_type=MCC_CRIT_COUNT_EPS, max_count=200, eps=1e-7):
        """optimizeExtrinsics: returns (x, meanReProjError, iterations, last change)."""
        x = np.array(x0, np.float32, copy=True)
        it = ctypes.c_int(0)
        ch = ctypes.c_double(0)
        _check(lib().mcc_optimize(self.h, crit_type, max_count, eps, _ptr(x, _f32p), ctypes.byref(it),
                                  ctypes.byref(ch)), "mcc_optimize")
        _, mean = self.compute_project_error(x)
        return x, mean, it.value, ch.value

    def compute_project_error(self, x):
        x = np.ascontiguousarray(x, np.float32)
        err = np.zeros(self.prob.n_edges, np.float32)
        mean = ctypes.c_double(0)
        _check(lib().mcc_project_error(self.h, _ptr(x, _f32p), _ptr(err, _f32p), ctypes.byref(mean)),
               "mcc_project_error")
        return err, mean.value

    # -- throughput path
    def step(self, n):
        _check(lib().mcc_step(self.h, n), "mcc_step")

    def synchronize(self):
        _check(lib().mcc_synchronize(self.h), "mcc_synchronize")

    def check(self):
        """Raise if an enqueued step failed on the device (peer timeout, not positive definite)."""
        _check(lib().mcc_check(self.h), "mcc_check")

    def residuals(self, x):
        x = np.ascontiguousarray(x, np.float32)
        r = np.zeros(2 * self.prob.n_corners, np.float32)
        _check(lib().mcc_debug_residuals(self.h, _ptr(x, _f32p), _ptr(r, _f32p)), "mcc_debug_residuals")
        return r

    def optimize_profile(self):
        """The last optimize_extrinsics as the caller saw it (mcc_optimize_profile): host phases (ms),
        device ms from the first step launch to the end of the last, steps launched, updates, polls."""
        hm = np.zeros(4, np.float64)
        dev = ctypes.c_double(0)
        n, it, polls = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
        _check(lib().mcc_optimize_profile(self.h, _ptr(hm, _f64p), ctypes.byref(dev), ctypes.byref(n),
                                          ctypes.byref(it), ctypes.byref(polls)), "mcc_optimize_profile")
        return {"host_setup_ms": hm[0], "host_steps_ms": hm[1], "host_finish_ms": hm[2], "host_call_ms": hm[3],
                "device_ms": dev.value, "steps_launched": n.value, "iters": it.value, "stop_polls": polls.value}

    def debug_delays(self, spare_delay_us=-1.0, warm_delay_us=-1.0, warm_timeout_ms=-1.0):
        """test only: change the injected warm-solve delays / wait bound of this handle (-1 keeps one)"""
        _check(lib().mcc_debug_delays(self.h, float(spare_delay_us), float(warm_delay_us), float(warm_timeout_ms)),
               "mcc_debug_delays")

    def timing_begin(self):
        _check(lib().mcc_timing_begin(self.h), "mcc_timing_begin")

    def timing_end(self):
        lin = ctypes.c_double(0)
        st = ctypes.c_double(0)
        n = ctypes.c_int(0)
        _check(lib().mcc_timing_end(self.h, ctypes.byref(lin), ctypes.byref(st), ctypes.byref(n)), "mcc_timing_end")
        return lin.value, st.value, n.value

    def timing_windows(self, n_windows, steps):
        """Device time (ms) of each of n_windows back-to-back windows of `steps` free-running steps
        (mcc_timing_windows), and whether they ran graph-launched."""
        out = np.zeros(n_windows)
        g = ctypes.c_int(0)
        _check(lib().mcc_timing_windows(self.h, n_windows, steps, _ptr(out, _f64p), ctypes.byref(g)), "mcc_timing_windows")
        return out, bool(g.value)

    def project_error_detail(self, x):
        """(edge errors, per-corner L2 errors in reference order, totalError, totalNPoints, mean)."""
        x = np.ascontiguousarray(x, np.float32)
        err = np.zeros(self.prob.n_edges, np.float32)
        cerr = np.zeros(self.prob.n_corners, np.float32)
        tot = ctypes.c_float(0)
        npts = ctypes.c_longlong(0)
        mean = ctypes.c_double(0)
        _check(lib().mcc_project_error_detail(self.h, _ptr(x, _f32p), _ptr(err, _f32p), _ptr(cerr, _f32p),
                                              ctypes.byref(tot), ctypes.byref(npts), ctypes.byref(mean)),
               "mcc_project_error_detail")
        return err, cerr, tot.value, npts.value, mean.value

    def timing_linearize(self, launches: int) -> float:
        """Split step: ms per launch of the linearisation kernels alone, `launches` of them in one
        captured graph between two HIP events (mcc_timing_linearize)."""
        ms = ctypes.c_double()
        _check(lib().mcc_timing_linearize(self.h, launches, ctypes.byref(ms)), "mcc_timing_linearize")
        return ms.value

    def timing_exchange(self):
        """(ms per data-path exchange, exchanges) over the last timing window (mcc_timing_exchange)."""
        ms = ctypes.c_double(0)
        n = ctypes.c_int(0)
        _check(lib().mcc_timing_exchange(self.h, ctypes.byref(ms), ctypes.byref(n)), "mcc_timing_exchange")
        return ms.value, n.value

    def stats(self):
        v = [ctypes.c_longlong(0) for _ in range(4)]
        _check(lib().mcc_problem_stats(self.h, *[ctypes.byref(t) for t in v]), "mcc_problem_stats")
        return dict(corners=v[0].value, edges=v[1].value, photos=v[2].value, alg_bytes=v[3].value)

    def solve_stats(self):
        """The warm solves (mcc_solve_stats; m > 30: the helper kernel's inverse, m <= 30: the spare
        workgroup's): solves by refinement with the previous system's inverse, their refinement
        corrections, refinements that fell back to the direct elimination, direct solves for want of an
        inverse, steps that waited for the inverse's producer (the choice of solve never depends on the
        wait; all zero on the direct-only paths)."""
        v = (ctypes.c_longlong * 5)()
        _check(lib().mcc_solve_stats(self.h, v), "mcc_solve_stats")
        return dict(warm=v[0], corrections=v[1], fallbacks=v[2], direct=v[3], waited=v[4])

    def path(self):
        """'fused' (one kernel per step) or 'split' (k_prep, k_edge, k_photo, k_schur, k_solve)."""
        sp = ctypes.c_int(0)
        ng = ctypes.c_int(0)
        _check(lib().mcc_problem_path(self.h, ctypes.byref(sp), ctypes.byref(ng)), "mcc_problem_path")
        return "split" if sp.value else "fused"

    def step_kernels(self):
        """The kernels of one step's linearisation: 'k_linearize' (fused), 'k_group' (the split step's
        fused group kernel) or 'k_prep+k_edge+k_photo' (MCC_GROUP=0)."""
        sp = ctypes.c_int(0)
        ng = ctypes.c_int(0)
        _check(lib().mcc_problem_path(self.h, ctypes.byref(sp), ctypes.byref(ng)), "mcc_problem_path")
        return {0: "k_linearize", 1: "k_prep+k_edge+k_photo", 2: "k_group", 3: "k_group"}[sp.value]

    def photo_groups(self):
        """The split step's photo-group workgroups (mcc_problem_path; 0 on the fused step)."""
        sp = ctypes.c_int(0)
        ng = ctypes.c_int(0)
        _check(lib().mcc_problem_path(self.h, ctypes.byref(sp), ctypes.byref(ng)), "mcc_problem_path")
        return ng.value

    def folded(self):
        """True when a step is ONE k_group launch: the Schur reduction and the m <= 30 solve folded
        into the group kernel's grid (mcc_problem_path 3; MCC_GFOLD=0 turns it off)."""
        sp = ctypes.c_int(0)
        _check(lib().mcc_problem_path(self.h, ctypes.byref(sp), None), "mcc_problem_path")
        return sp.value == 3

    def stamps(self):
        """libmcc_diag.so only: first call arms, later calls return [n_photos, 32] s_memtime stamps
        followed by k_schur's [workgroups, 8]."""
        out = np.zeros(32 * max(self.prob.n_photos, 1) + 8 * 65536, np.int64)
        _check(lib().mcc_debug_stamps(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), out.size),
               "mcc_debug_stamps")
        return out

    # -- multi-GPU
    def comm_init(self, uid: bytes, nranks: int, rank: int):
        _check(lib().mcc_comm_init(self.h, uid, nranks, rank), "mcc_comm_init")

    def allreduce_max(self, v: float) -> float:
        d = ctypes.c_double(v)
        _check(lib().mcc_comm_allreduce_max(self.h, ctypes.byref(d)), "mcc_comm_allreduce_max")
        return d.value

    def barrier(self):
        _check(lib().mcc_comm_barrier(self.h), "mcc_comm_barrier")

    def peer_handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        _check(lib().mcc_peer_handle(self.h, buf), "mcc_peer_handle")
        return buf.raw

    def peer_init(self, handles, nranks: int, rank: int):
        """Collective: map the peers' inboxes and handshake (raises MccError on every rank if the
        transport does not work)."""
        blob = b"".join(handles)
        _check(lib().mcc_peer_init(self.h, blob, nranks, rank), "mcc_peer_init")

    def peer_enable(self, on: bool):
        _check(lib().mcc_peer_enable(self.h, int(bool(on))), "mcc_peer_enable")


# ---------------------------------------------------------------- cv::omnidir::calibrate
# include/mcc_omnidir.h; the reference's names: cv::omnidir::calibrate (src/omnidir.cpp:1067-1211),
# internal::initializeCalibration (:551-748), internal::computeJacobian (:851-935).
CALIB_USE_GUESS, CALIB_FIX_SKEW, CALIB_FIX_K1, CALIB_FIX_K2 = 1, 2, 4, 8
CALIB_FIX_P1, CALIB_FIX_P2, CALIB_FIX_XI, CALIB_FIX_GAMMA, CALIB_FIX_CENTER = 16, 32, 64, 128, 256


def _views(off, obj, img):
    off = np.ascontiguousarray(off, np.int32)
    obj = np.ascontiguousarray(obj, np.float64).reshape(-1, 3)
    img = np.ascontiguousarray(img, np.float64).reshape(-1, 2)
    if off.ndim != 1 or off.size < 2 or off[0] != 0 or off[-1] != obj.shape[0] or obj.shape[0] != img.shape[0]:
        raise MccError("view offsets / points mismatch")
    return off, obj, img


class OmniCalibrator:
    """The device-resident state of cv::omnidir::calibrate's loop for one camera's views
    (CV_64F pattern / image points, parameters in encodeParameters layout, P = 6n + 10)."""

    def __init__(self, off, obj, img, flags: int = 0, device: int = 0):
        self.off, self.obj, self.img = _views(off, obj, img)
        d = _OmniDesc()
        d.n_views = self.off.size - 1
        d.view_off = _ptr(self.off, _i32p)
        d.obj = _ptr(self.obj, _f64p)
        d.img = _ptr(self.img, _f64p)
        d.flags, d.device = flags, device
        h = ctypes.c_void_p()
        _check(lib().mcc_omnicalib_create(ctypes.byref(h), ctypes.byref(d)), "mcc_omnicalib_create")
        self.h = h
        self.P = lib().mcc_omnicalib_nparams(h)

    def close(self):
        if getattr(self, "h", None):
            lib().mcc_omnicalib_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compute_jacobian(self, params, it=0):
        """(JTE before the flag reduction, G of loop iteration `it`) at params (computeJacobian)."""
        p = np.ascontiguousarray(params, np.float64)
        jte, G = np.zeros(self.P), np.zeros(self.P)
        _check(lib().mcc_omnicalib_jacobian(self.h, _ptr(p, _f64p), it, _ptr(jte, _f64p), _ptr(G, _f64p)),
               "mcc_omnicalib_jacobian")
        return jte, G

    def optimize(self, params, crit_type=MCC_CRIT_COUNT_EPS, max_count=200, eps=1e-4):
        """calibrate's loop: (params, iterations, last change)."""
        p = np.array(params, np.float64, copy=True)
        it, ch = ctypes.c_int(0), ctypes.c_double(0)
        _check(lib().mcc_omnicalib_optimize(self.h, crit_type, max_count, eps, _ptr(p, _f64p), ctypes.byref(it),
                                            ctypes.byref(ch)), "mcc_omnicalib_optimize")
        return p, it.value, ch.value

    def rms(self, params):
        p = np.ascontiguousarray(params, np.float64)
        r = ctypes.c_double(0)
        _check(lib().mcc_omnicalib_rms(self.h, _ptr(p, _f64p), ctypes.byref(r)), "mcc_omnicalib_rms")
        return r.value

    def time_steps(self, params, n_steps):
        p = np.ascontiguousarray(params, np.float64)
        ms = ctypes.c_double(0)
        _check(lib().mcc_omnicalib_time_steps(self.h, _ptr(p, _f64p), n_steps, ctypes.byref(ms)),
               "mcc_omnicalib_time_steps")
        return ms.value


def omnidir_initialize(off, obj, img, image_size):
    """initializeCalibration: (om[k, 3], t[k, 3], K 3x3, xi, idx[k]) -- host code, no GPU."""
    off, obj, img = _views(off, obj, img)
    n = off.size - 1
    om, t, K = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(9)
    xi, nk = ctypes.c_double(0), ctypes.c_int(0)
    idx = np.zeros(n, np.int32)
    _check(lib().mcc_omnidir_initialize(n, _ptr(off, _i32p), _ptr(obj, _f64p), _ptr(img, _f64p), int(image_size[0]),
                                        int(image_size[1]), _ptr(om, _f64p), _ptr(t, _f64p), _ptr(K, _f64p),
                                        ctypes.byref(xi), _ptr(idx, _i32p), ctypes.byref(nk)),
           "mcc_omnidir_initialize")
    k = nk.value
    return om[:k], t[:k], K.reshape(3, 3), xi.value, idx[:k].copy()


def omnidir_calibrate(off, obj, img, image_size, flags=0, crit_type=MCC_CRIT_COUNT_EPS, max_count=200, eps=1e-4,
                      device=0):
    """cv::omnidir::calibrate: (rms, K, xi, D, om[k, 3], t[k, 3], idx[k], iterations)."""
    off, obj, img = _views(off, obj, img)
    n = off.size - 1
    K, D = np.zeros(9), np.zeros(4)
    om, t = np.zeros((n, 3)), np.zeros((n, 3))
    xi, rms, nk, it = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_int(0), ctypes.c_int(0)
    idx = np.zeros(n, np.int32)
    _check(lib().mcc_omnidir_calibrate(n, _ptr(off, _i32p), _ptr(obj, _f64p), _ptr(img, _f64p), int(image_size[0]),
                                       int(image_size[1]), flags, crit_type, max_count, eps, device, _ptr(K, _f64p),
                                       ctypes.byref(xi), _ptr(D, _f64p), _ptr(om, _f64p), _ptr(t, _f64p),
                                       _ptr(idx, _i32p), ctypes.byref(nk), ctypes.byref(rms), ctypes.byref(it)),
           "mcc_omnidir_calibrate")
    k = nk.value
    return rms.value, K.reshape(3, 3), xi.value, D, om[:k], t[:k], idx[:k].copy(), it.value
