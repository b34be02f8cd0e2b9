"""ctypes binding of libf110qp.so (include/f110qp.h).

This is the Python-side binding a maintainer would write over the C ABI; the product's
compute path is the HIP kernel behind it. There is no CPU fallback: if the library is
missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# F110QP_LIB selects a diagnostic build (e.g. lib_stamps/); default is the in-tree product library
LIB_PATH = os.environ.get("F110QP_LIB", os.path.join(PKG_ROOT, "lib", "libf110qp.so"))
# the test / measurement build (same kernels; f110qp_create also reads the F110QP_* knobs that force
# kernel variants). Solvers use it while USE_TEST_BUILD is true (the tests' `knob` fixture sets it).
TEST_LIB_PATH = os.environ.get("F110QP_TEST_LIB", os.path.join(PKG_ROOT, "lib_test", "libf110qp.so"))
USE_TEST_BUILD = False

OK = 0
ERR_INVALID = -1
ERR_HIP = -2
ERR_ALLOC = -3
SOLVED = 1
SOLVED_INACCURATE = 2
MAX_ITER = -2
PRIMAL_INFEASIBLE = -3
NUMERICAL = -10
GAP_INACTIVE = 0
GAP_ACTIVE = 1
BACKEND_AUTO = 0
BACKEND_WAVE = 1
BACKEND_LANE = 2
LANE_MIN_BATCH = 1024
LANE_MIN_BATCH_WIDE = 1
LANE_MIN_BATCH_GROUPED = LANE_MIN_BATCH
LANE_MIN_BATCH_GROUPED_WIDE = LANE_MIN_BATCH_WIDE
LANE_MAX_SMALL_BATCH = 8
GAP_SCREEN_MIN_BATCH = 1024


def auto_backend(horizon: int, batch: int, gap: bool, grouped: bool = False) -> int:
    """The back end BACKEND_AUTO resolves to (mirrors resolve_backend() in f110qp_api.cpp)."""
    if grouped:
        min_b = LANE_MIN_BATCH_GROUPED if horizon <= 32 else LANE_MIN_BATCH_GROUPED_WIDE
    else:
        min_b = LANE_MIN_BATCH if horizon <= 32 else LANE_MIN_BATCH_WIDE
    small = not grouped and horizon <= 32 and batch <= LANE_MAX_SMALL_BATCH
    return BACKEND_LANE if (not gap and (batch >= min_b or small)) else BACKEND_WAVE


def auto_gap_screen(batch: int, grouped: bool = False, warm_start: bool = False) -> bool:
    """Whether AUTO takes the box screen for a gap-row call (mirrors gap_screen() in f110qp_api.cpp)."""
    return not grouped and not warm_start and batch >= GAP_SCREEN_MIN_BATCH


MAX_HORIZON = 48

# every symbol include/f110qp.h declares
EXPORTED = (
    "f110qp_version",
    "f110qp_last_error",
    "f110qp_default_config",
    "f110qp_create",
    "f110qp_destroy",
    "f110qp_solve_batch",
    "f110qp_solve_batch_dev",
    "f110qp_solve_batch_dev_sync",
    "f110qp_solve_grouped",
    "f110qp_solve_grouped_dev",
    "f110qp_condense_debug_dev",
    "f110qp_qp_dims",
    "f110qp_assemble_debug_dev",
    "f110qp_warm_reset",
    "f110qp_find_half_spaces",
    "f110qp_find_half_spaces_dev",
    "f110qp_default_plan_config",
    "f110qp_traj_table",
    "f110qp_parse_waypoints",
    "f110qp_plan_batch_dev",
    "f110qp_plan_batch",
    "f110qp_solve_batch_ex",
    "f110qp_solve_batch_ex_dev",
    "f110qp_solve_grouped_ex",
    "f110qp_solve_grouped_ex_dev",
    "f110qp_select_dev",
    "f110qp_backend_info",
    "f110qp_lane_segments",
    "f110qp_gap_screen",
    "f110qp_last_recheck_count",
    "f110qp_lane_starts",
    "f110qp_warm_hits",
    "f110qp_sync_signals",
    "f110qp_test_build",
)
SCRATCH_NAMES = {0: "none (wave back end)", 1: "LDS fp64", 2: "LDS fp32", 3: "HBM fp64", 4: "HBM fp32"}


class Config(C.Structure):
    _fields_ = [
        ("horizon", C.c_int),
        ("dt", C.c_float),
        ("q", C.c_double * 3),
        ("r", C.c_double * 2),
        ("u_des", C.c_double * 2),
        ("u_min", C.c_float * 2),
        ("u_max", C.c_float * 2),
        ("gap_mode", C.c_int),
        ("max_iter", C.c_int),
        ("device", C.c_int),
        ("warm_start", C.c_int),
        ("backend", C.c_int),
        ("x_ref_points", C.c_int),
    ]


class PlanConfig(C.Structure):
    _fields_ = [
        ("size", C.c_int),
        ("discrete", C.c_float),
        ("dilation", C.c_float),
        ("lookahead", C.c_float),
        ("speed_max", C.c_double),
        ("steer_max", C.c_double),
        ("steer_discrete", C.c_int),
        ("traj_discrete", C.c_int),
        ("dt", C.c_double),
    ]


class F110QPError(RuntimeError):
    pass


_libs = {}


def load(test: bool = False):
    """Load libf110qp.so (raises if it is missing: there is no fallback path). test=True: the
    test / measurement build lib_test/libf110qp.so."""
    path = TEST_LIB_PATH if test else LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise F110QPError(f"{path} not built: run `make -C {PKG_ROOT}` (hipcc, gfx950)")
    L = C.CDLL(path)
    fp = C.c_void_p
    L.f110qp_version.restype = C.c_int
    L.f110qp_last_error.restype = C.c_char_p
    L.f110qp_default_config.argtypes = [C.POINTER(Config), C.c_int]
    L.f110qp_create.argtypes = [C.POINTER(C.c_void_p), C.POINTER(Config)]
    L.f110qp_destroy.argtypes = [C.c_void_p]
    L.f110qp_solve_batch.argtypes = [C.c_void_p, C.c_int] + [fp] * 8
    L.f110qp_solve_batch_dev.argtypes = [C.c_void_p, C.c_int] + [fp] * 9
    L.f110qp_solve_batch_dev_sync.argtypes = [C.c_void_p, C.c_int] + [fp] * 9
    L.f110qp_solve_grouped.argtypes = [C.c_void_p, C.c_int] + [fp] * 5 + [C.c_int] + [fp] * 4
    L.f110qp_solve_grouped_dev.argtypes = [C.c_void_p, C.c_int] + [fp] * 5 + [C.c_int] + [fp] * 5
    L.f110qp_solve_batch_ex.argtypes = [C.c_void_p, C.c_int] + [fp] * 10
    L.f110qp_solve_batch_ex_dev.argtypes = [C.c_void_p, C.c_int] + [fp] * 11
    L.f110qp_solve_grouped_ex.argtypes = [C.c_void_p, C.c_int] + [fp] * 5 + [C.c_int] + [fp] * 6
    L.f110qp_solve_grouped_ex_dev.argtypes = [C.c_void_p, C.c_int] + [fp] * 5 + [C.c_int] + [fp] * 7
    L.f110qp_select_dev.argtypes = [C.c_int, fp, C.c_int, fp, fp, fp, fp, fp]
    L.f110qp_backend_info.argtypes = [C.c_void_p, C.c_int, C.c_int] + [C.POINTER(C.c_int)] * 3
    L.f110qp_lane_segments.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.f110qp_gap_screen.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.f110qp_last_recheck_count.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    L.f110qp_lane_starts.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.f110qp_warm_hits.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.f110qp_sync_signals.argtypes = [C.c_void_p, C.POINTER(C.c_uint)]
    L.f110qp_test_build.restype = C.c_int
    L.f110qp_condense_debug_dev.argtypes = [C.c_void_p, C.c_int] + [fp] * 6
    L.f110qp_warm_reset.argtypes = [C.c_void_p]
    L.f110qp_qp_dims.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 4
    L.f110qp_assemble_debug_dev.argtypes = [C.c_void_p] + [fp] * 14
    L.f110qp_find_half_spaces.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_float), C.c_int,
                                          C.c_float, C.c_float, C.c_float, C.c_float, C.c_float,
                                          C.c_float, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.f110qp_find_half_spaces_dev.argtypes = [C.c_int, fp, fp, C.c_int, C.c_float, C.c_float, C.c_float,
                                              C.c_float, C.c_float, C.c_float, fp, fp, fp, fp]
    L.f110qp_default_plan_config.argtypes = [C.POINTER(PlanConfig)]
    L.f110qp_traj_table.argtypes = [C.POINTER(PlanConfig), fp]
    L.f110qp_parse_waypoints.argtypes = [C.c_char_p, fp, C.c_int, C.POINTER(C.c_int)]
    L.f110qp_plan_batch_dev.argtypes = [C.POINTER(PlanConfig), C.c_int, fp, fp, C.c_int, C.c_float, C.c_float,
                                        C.c_float, fp, fp, C.c_int, fp, fp, fp, fp, fp, fp, fp, fp]
    _libs[path] = L
    return L


def last_error(lib=None) -> str:
    return (lib or load()).f110qp_last_error().decode()


def _check(rc: int, what: str, lib=None):
    if rc != OK:
        raise F110QPError(f"{what} failed ({rc}): {last_error(lib)}")


def default_config(horizon: int, **over) -> Config:
    c = Config()
    load().f110qp_default_config(C.byref(c), horizon)
    for k, v in over.items():
        if k in ("q", "r", "u_des", "u_min", "u_max"):
            arr = getattr(c, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(c, k, v)
    return c


def qp_dims(horizon: int):
    """(n, m, nnz_P, nnz_A) of the reference's OSQP problem (f110qp_qp_dims)."""
    v = [C.c_int() for _ in range(4)]
    _check(load().f110qp_qp_dims(horizon, *[C.byref(x) for x in v]), "f110qp_qp_dims")
    return tuple(x.value for x in v)


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _tp(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _dev(t, dtype: str, n: int, name: str, optional: bool = False, where: bool = False):
    """Check a device tensor before its raw pointer crosses the C ABI: a contiguous CUDA (HIP)
    tensor of the ABI's element type with at least n elements (the kernels write / read exactly
    that many; a float32 tensor where the ABI wants float64, or an int64 one where it wants int32,
    would be an out-of-bounds write or a silent misread)."""
    if t is None:
        if optional:
            return
        raise F110QPError(f"{name} is required")
    import torch

    want = {"f32": torch.float32, "f64": torch.float64, "i32": torch.int32, "u8": torch.uint8}[dtype]
    if not isinstance(t, torch.Tensor):
        raise F110QPError(f"{name} must be a torch tensor on the device, got {type(t).__name__}")
    if t.dtype != want:
        raise F110QPError(f"{name} must be {want}, got {t.dtype}")
    if not t.is_contiguous():
        raise F110QPError(f"{name} must be contiguous")
    if t.numel() < n:
        raise F110QPError(f"{name} holds {t.numel()} elements, the call needs {n}")
    if where and t.device.type != "cuda":
        raise F110QPError(f"{name} must be a device (cuda/HIP) tensor, got {t.device}")


def _devs(*specs):
    """_dev over several (tensor, dtype, n, name[, optional]) specs: every type / size check
    first, then the placement of each (so a host-side test sees the type errors)."""
    for sp in specs:
        _dev(*sp)
    for sp in specs:
        _dev(*sp[:4], *(sp[4:] or (False,)), where=True)


class Solver:
    """One f110qp context (device workspace). Mirrors the reference's OsqpEigen::Solver
    member of MPC (include/f110-mpc/mpc.h:63) for B instances at once."""

    def __init__(self, config: Config, test_build: bool | None = None):
        self.lib = load(USE_TEST_BUILD if test_build is None else test_build)
        self.config = config
        h = C.c_void_p()
        self._chk = lambda rc, what: _check(rc, what, self.lib)
        self._chk(self.lib.f110qp_create(C.byref(h), C.byref(config)), "f110qp_create")
        self._h = h

    @property
    def horizon(self) -> int:
        return self.config.horizon

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.f110qp_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def backend_info(self, batch: int, grouped: bool = False):
        """(backend, qps_per_wave, scratch) of a solve call of `batch` QPs (f110qp_backend_info)."""
        v = [C.c_int() for _ in range(3)]
        self._chk(self.lib.f110qp_backend_info(self._h, int(batch), int(grouped), *[C.byref(x) for x in v]),
               "f110qp_backend_info")
        return tuple(x.value for x in v)

    def lane_segments(self, batch: int) -> int:
        """Horizon segments per QP of a solve call of `batch` QPs (f110qp_lane_segments): 1, or
        2 / 4 / 8 when the lane back end runs the partitioned Riccati (lane_seg_kernel.h)."""
        v = C.c_int()
        self._chk(self.lib.f110qp_lane_segments(self._h, int(batch), C.byref(v)), "f110qp_lane_segments")
        return v.value

    def lane_starts(self, batch: int) -> int:
        """PDAS starts per QP of a solve call of `batch` QPs (f110qp_lane_starts): 2 with the
        partitioned-horizon kernel's twin start, else 1."""
        v = C.c_int()
        self._chk(self.lib.f110qp_lane_starts(self._h, int(batch), C.byref(v)), "f110qp_lane_starts")
        return v.value

    def last_recheck_count(self) -> int:
        """QPs the last gap-row call sent to the fp64 re-check (f110qp_last_recheck_count;
        synchronises with that call)."""
        v = C.c_int()
        self._chk(self.lib.f110qp_last_recheck_count(self._h, C.byref(v)), "f110qp_last_recheck_count")
        return v.value

    def warm_hits(self):
        """(traffic_calls, hits) since the previous warm_hits (f110qp_warm_hits)."""
        t, h = C.c_int(), C.c_int()
        self._chk(self.lib.f110qp_warm_hits(self._h, C.byref(t), C.byref(h)), "f110qp_warm_hits")
        return t.value, h.value

    def sync_signals(self) -> int:
        """Synchronous calls on this solver that waited on the kernel's completion word instead of
        synchronising the stream (f110qp_sync_signals)."""
        n = C.c_uint()
        self._chk(self.lib.f110qp_sync_signals(self._h, C.byref(n)), "f110qp_sync_signals")
        return n.value

    @property
    def test_build(self) -> bool:
        return bool(self.lib.f110qp_test_build())

    def gap_screen(self, batch: int) -> bool:
        """Does a gap-row solve call of `batch` QPs take the box screen on the lane back end before
        the wave kernel's GI (f110qp_gap_screen)?"""
        v = C.c_int()
        self._chk(self.lib.f110qp_gap_screen(self._h, int(batch), C.byref(v)), "f110qp_gap_screen")
        return bool(v.value)

    def solve(self, x0, u_lin, x_ref, halfspace=None, objective=False):
        """Host arrays in, host arrays out (synchronous). Returns (u[B,N,2], x[B,N+1,3],
        status[B], iters[B]) and, with objective=True, also (obj[B], cost[B]) float64
        (f110qp_solve_batch_ex)."""
        N = self.horizon
        x0 = np.ascontiguousarray(x0, np.float32).reshape(-1, 3)
        B = x0.shape[0]
        ul = np.ascontiguousarray(u_lin, np.float32).reshape(B, 2)
        S = self.config.x_ref_points or N
        xr = np.ascontiguousarray(x_ref, np.float32).reshape(B, S, 3)
        hs = None if halfspace is None else np.ascontiguousarray(halfspace, np.float32).reshape(B, 6)
        u = np.empty((B, N, 2), np.float32)
        x = np.empty((B, N + 1, 3), np.float32)
        st = np.empty(B, np.int32)
        it = np.empty(B, np.int32)
        if objective:
            ob = np.empty(B, np.float64)
            co = np.empty(B, np.float64)
            self._chk(self.lib.f110qp_solve_batch_ex(self._h, B, _p(x0), _p(ul), _p(xr), _p(hs), _p(u), _p(x),
                                                  _p(st), _p(it), _p(ob), _p(co)), "f110qp_solve_batch_ex")
            return u, x, st, it, ob, co
        self._chk(self.lib.f110qp_solve_batch(self._h, B, _p(x0), _p(ul), _p(xr), _p(hs), _p(u), _p(x),
                                           _p(st), _p(it)), "f110qp_solve_batch")
        return u, x, st, it

    def _check_dev(self, x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters=None, obj=None, cost=None,
                   group=None):
        """Shapes, element types and placement of a device call's tensors (see _dev)."""
        B = int(x0.shape[0])
        N = self.horizon
        S = self.config.x_ref_points or N
        specs = [(x0, "f32", 3 * B, "x0"), (u_lin, "f32", 2 * B, "u_lin"), (x_ref, "f32", 3 * S * B, "x_ref"),
                 (halfspace, "f32", 6 * B, "halfspace", self.config.gap_mode == GAP_INACTIVE),
                 (u_out, "f32", 2 * N * B, "u_out"), (x_out, "f32", 3 * (N + 1) * B, "x_out"),
                 (status, "i32", B, "status"), (iters, "i32", B, "iters", True), (obj, "f64", B, "obj", True),
                 (cost, "f64", B, "cost", True)]
        if group is not None:
            specs.append((group, "i32", B, "group"))
        _devs(*specs)
        return B

    def solve_dev(self, x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters=None, stream=None,
                  obj=None, cost=None):
        """Device (torch) tensors in/out, enqueued on `stream` (torch.cuda stream or None =
        current stream). Asynchronous. obj / cost: optional float64 [B] device tensors
        (f110qp_solve_batch_ex_dev)."""
        import torch

        B = self._check_dev(x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters, obj, cost)
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        if obj is not None or cost is not None:
            self._chk(self.lib.f110qp_solve_batch_ex_dev(self._h, B, _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace),
                                                      _tp(u_out), _tp(x_out), _tp(status), _tp(iters), _tp(obj),
                                                      _tp(cost), C.c_void_p(stream.cuda_stream)),
                   "f110qp_solve_batch_ex_dev")
            return
        self._chk(self.lib.f110qp_solve_batch_dev(self._h, B, _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace),
                                               _tp(u_out), _tp(x_out), _tp(status), _tp(iters),
                                               C.c_void_p(stream.cuda_stream)), "f110qp_solve_batch_dev")

    def prepare_dev(self, x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters=None, stream=None,
                    sync=False):
        """A launcher for repeated f110qp_solve_batch_dev calls on the same device buffers: the
        ctypes arguments are converted once, each call is one C call (what a C++ caller of the ABI
        pays; bench.py's timed steps use it so Python argument marshalling is not the step).
        sync=True: f110qp_solve_batch_dev_sync (returns with the results in device memory)."""
        import torch

        self._check_dev(x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters)
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        fn = self.lib.f110qp_solve_batch_dev_sync if sync else self.lib.f110qp_solve_batch_dev
        args = (self._h, x0.shape[0], _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace), _tp(u_out), _tp(x_out),
                _tp(status), _tp(iters), C.c_void_p(stream.cuda_stream))

        def launch():
            rc = fn(*args)
            if rc != OK:
                _check(rc, "f110qp_solve_batch_dev", self.lib)
        return launch

    def prepare_grouped_dev(self, x0, u_lin, x_ref, halfspace, group, num_groups, u_out, x_out, status,
                            iters=None, stream=None):
        """prepare_dev for f110qp_solve_grouped_dev."""
        import torch

        self._check_dev(x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters, group=group)
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        fn = self.lib.f110qp_solve_grouped_dev
        args = (self._h, x0.shape[0], _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace), _tp(group), int(num_groups),
                _tp(u_out), _tp(x_out), _tp(status), _tp(iters), C.c_void_p(stream.cuda_stream))

        def launch():
            rc = fn(*args)
            if rc != OK:
                _check(rc, "f110qp_solve_grouped_dev", self.lib)
        return launch

    def assemble_debug(self, x0, u_lin, x_ref, halfspace=None):
        """f110qp_assemble_debug_dev for one instance (host arrays in; the device computes; host
        dict of the CSC arrays out, the oracle.assemble layout)."""
        import torch

        N = self.horizon
        n, m, nzp, nza = qp_dims(N)
        dev = torch.device("cuda", self.config.device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32).reshape(-1)).to(dev)  # noqa: E731
        x0d, uld, xrd = t(x0), t(u_lin), t(x_ref)
        hsd = None if halfspace is None else t(halfspace)
        out = {"P_colptr": torch.empty(n + 1, dtype=torch.int32, device=dev),
               "P_rowind": torch.empty(nzp, dtype=torch.int32, device=dev),
               "P_val": torch.empty(nzp, dtype=torch.float64, device=dev),
               "q": torch.empty(n, dtype=torch.float64, device=dev),
               "A_colptr": torch.empty(n + 1, dtype=torch.int32, device=dev),
               "A_rowind": torch.empty(nza, dtype=torch.int32, device=dev),
               "A_val": torch.empty(nza, dtype=torch.float64, device=dev),
               "l": torch.empty(m, dtype=torch.float64, device=dev),
               "u": torch.empty(m, dtype=torch.float64, device=dev)}
        stream = torch.cuda.current_stream(dev)
        o = out
        self._chk(self.lib.f110qp_assemble_debug_dev(self._h, _tp(x0d), _tp(uld), _tp(xrd), _tp(hsd), _tp(o["P_colptr"]),
                                                  _tp(o["P_rowind"]), _tp(o["P_val"]), _tp(o["q"]), _tp(o["A_colptr"]),
                                                  _tp(o["A_rowind"]), _tp(o["A_val"]), _tp(o["l"]), _tp(o["u"]),
                                                  C.c_void_p(stream.cuda_stream)), "f110qp_assemble_debug_dev")
        torch.cuda.synchronize(dev)
        return {k: v.cpu().numpy() for k, v in out.items()}

    def solve_grouped(self, x0, u_lin, x_ref, group, num_groups=None, halfspace=None, objective=False):
        """Grouped solve on host arrays (f110qp_solve_grouped): group [B] int scenario ids.
        objective=True also returns (obj[B], cost[B]) (f110qp_solve_grouped_ex)."""
        N = self.horizon
        x0 = np.ascontiguousarray(x0, np.float32).reshape(-1, 3)
        B = x0.shape[0]
        ul = np.ascontiguousarray(u_lin, np.float32).reshape(B, 2)
        S = self.config.x_ref_points or N
        xr = np.ascontiguousarray(x_ref, np.float32).reshape(B, S, 3)
        hs = None if halfspace is None else np.ascontiguousarray(halfspace, np.float32).reshape(B, 6)
        g = np.ascontiguousarray(group, np.int32).reshape(B)
        G = int(g.max()) + 1 if num_groups is None else int(num_groups)
        u = np.empty((B, N, 2), np.float32)
        x = np.empty((B, N + 1, 3), np.float32)
        st = np.empty(B, np.int32)
        it = np.empty(B, np.int32)
        if objective:
            ob = np.empty(B, np.float64)
            co = np.empty(B, np.float64)
            self._chk(self.lib.f110qp_solve_grouped_ex(self._h, B, _p(x0), _p(ul), _p(xr), _p(hs), _p(g), G, _p(u),
                                                    _p(x), _p(st), _p(it), _p(ob), _p(co)), "f110qp_solve_grouped_ex")
            return u, x, st, it, ob, co
        self._chk(self.lib.f110qp_solve_grouped(self._h, B, _p(x0), _p(ul), _p(xr), _p(hs), _p(g), G, _p(u), _p(x),
                                             _p(st), _p(it)), "f110qp_solve_grouped")
        return u, x, st, it

    def solve_grouped_dev(self, x0, u_lin, x_ref, halfspace, group, num_groups, u_out, x_out, status, iters=None,
                          stream=None, obj=None, cost=None):
        """Grouped solve on device (torch) tensors; group [B] int32 on the device; obj / cost
        optional float64 [B] (f110qp_solve_grouped_ex_dev)."""
        import torch

        B = self._check_dev(x0, u_lin, x_ref, halfspace, u_out, x_out, status, iters, obj, cost, group=group)
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        if obj is not None or cost is not None:
            self._chk(self.lib.f110qp_solve_grouped_ex_dev(self._h, B, _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace),
                                                        _tp(group), int(num_groups), _tp(u_out), _tp(x_out),
                                                        _tp(status), _tp(iters), _tp(obj), _tp(cost),
                                                        C.c_void_p(stream.cuda_stream)), "f110qp_solve_grouped_ex_dev")
            return
        self._chk(self.lib.f110qp_solve_grouped_dev(self._h, B, _tp(x0), _tp(u_lin), _tp(x_ref), _tp(halfspace),
                                                 _tp(group), int(num_groups), _tp(u_out), _tp(x_out), _tp(status),
                                                 _tp(iters), C.c_void_p(stream.cuda_stream)),
               "f110qp_solve_grouped_dev")

    def warm_reset(self):
        self._chk(self.lib.f110qp_warm_reset(self._h), "f110qp_warm_reset")

    def condense_debug_dev(self, x0, u_lin, x_ref, H_out, g_out, stream=None):
        import torch

        B = x0.shape[0]
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        self._chk(self.lib.f110qp_condense_debug_dev(self._h, B, _tp(x0), _tp(u_lin), _tp(x_ref), _tp(H_out),
                                                  _tp(g_out), C.c_void_p(stream.cuda_stream)),
               "f110qp_condense_debug_dev")


def select_dev(group, num_groups, cost, status, winner, best_cost, stream=None):
    """Per-scenario argmin on the device (f110qp_select_dev): group [B] i32, cost [B] f64,
    status [B] i32 -> winner [G] i32 (-1: no solved candidate), best_cost [G] f64."""
    import torch

    B = int(group.shape[0])
    _devs((group, "i32", B, "group"), (cost, "f64", B, "cost"), (status, "i32", B, "status"),
          (winner, "i32", int(num_groups), "winner"), (best_cost, "f64", int(num_groups), "best_cost"))
    if stream is None:
        stream = torch.cuda.current_stream(cost.device)
    _check(load().f110qp_select_dev(int(group.shape[0]), _tp(group), int(num_groups), _tp(cost), _tp(status),
                                    _tp(winner), _tp(best_cost), C.c_void_p(stream.cuda_stream)),
           "f110qp_select_dev")


def find_half_spaces(state, ranges, angle_min, angle_inc, angle_max, thresh=3.0, divider=1.5, buffer=3.0):
    """Constraints::FindHalfSpaces for one scan (host). Returns (l1, l2) or raises when the
    scan has no gap."""
    L = load()
    s = np.ascontiguousarray(state, np.float64)
    r = np.ascontiguousarray(ranges, np.float32)
    l1 = np.zeros(3)
    l2 = np.zeros(3)
    rc = L.f110qp_find_half_spaces(s.ctypes.data_as(C.POINTER(C.c_double)), r.ctypes.data_as(C.POINTER(C.c_float)),
                                   len(r), float(angle_min), float(angle_inc), float(angle_max), float(thresh),
                                   float(divider), float(buffer), l1.ctypes.data_as(C.POINTER(C.c_double)),
                                   l2.ctypes.data_as(C.POINTER(C.c_double)))
    _check(rc, "f110qp_find_half_spaces")
    return l1, l2


def find_half_spaces_dev(states, ranges, angle_min, angle_inc, angle_max, hs_out, gap_lo=None, gap_hi=None,
                         thresh=3.0, divider=1.5, buffer=3.0, stream=None):
    """Batched FindHalfSpaces on torch device tensors: states [B,3] f32, ranges [B,R] f32 ->
    hs_out [B,2,3] f32."""
    import torch

    L = load()
    if stream is None:
        stream = torch.cuda.current_stream(states.device)
    B, R = ranges.shape
    _devs((states, "f32", 3 * B, "states"), (ranges, "f32", B * R, "ranges"), (hs_out, "f32", 6 * B, "hs_out"),
          (gap_lo, "i32", B, "gap_lo", True), (gap_hi, "i32", B, "gap_hi", True))
    _check(L.f110qp_find_half_spaces_dev(B, _tp(states), _tp(ranges), R, float(angle_min), float(angle_inc),
                                         float(angle_max), float(thresh), float(divider), float(buffer),
                                         _tp(hs_out), _tp(gap_lo), _tp(gap_hi), C.c_void_p(stream.cuda_stream)),
           "f110qp_find_half_spaces_dev")


# ---- planning stage (plan_kernels.hip) ---------------------------------------------------------

def default_plan_config(**over) -> PlanConfig:
    c = PlanConfig()
    load().f110qp_default_plan_config(C.byref(c))
    for k, v in over.items():
        setattr(c, k, v)
    return c


def traj_table(cfg: PlanConfig) -> np.ndarray:
    """Traj_Plan::generate_traj_table (host): [T, P, 3] float64, car frame."""
    t = np.zeros((cfg.steer_discrete + 1, cfg.traj_discrete, 3), np.float64)
    rc = load().f110qp_traj_table(C.byref(cfg), _p(t))
    if rc < 0:
        _check(rc, "f110qp_traj_table")
    return t


def parse_waypoints(text: str, max_n: int = 100000) -> np.ndarray:
    """Trajectory::ReadCSV on CSV text: [n, 3] (x, y, ori)."""
    wp = np.zeros((max_n, 3), np.float64)
    n = C.c_int(0)
    _check(load().f110qp_parse_waypoints(text.encode(), _p(wp), max_n, C.byref(n)), "f110qp_parse_waypoints")
    return wp[: n.value].copy()


def grid_blocks(cfg: PlanConfig) -> int:
    return int(np.float32(cfg.size) / np.float32(cfg.discrete))


def plan_batch_dev(cfg: PlanConfig, pose, ranges, angle_min, angle_inc, angle_max, table, waypoints, x_ref, x0,
                   best_traj, best_global, status, valid=None, grid=None, stream=None):
    """Batched planning stage on torch device tensors: pose [B,4] f64, ranges [B,R] f32, table
    [T,P,3] f64, waypoints [W,2] f64 -> x_ref [B,P,3] f32, x0 [B,3] f32, best_traj / best_global
    / status [B] i32 (valid [B,T] u8 and grid [B,G,G] u8 optional)."""
    import torch

    B = pose.shape[0]
    if stream is None:
        stream = torch.cuda.current_stream(pose.device)
    _check(load().f110qp_plan_batch_dev(C.byref(cfg), B, _tp(pose), _tp(ranges), ranges.shape[1], float(angle_min),
                                        float(angle_inc), float(angle_max), _tp(table), _tp(waypoints),
                                        waypoints.shape[0], _tp(grid), _tp(valid), _tp(best_global), _tp(best_traj),
                                        _tp(x_ref), _tp(x0), _tp(status), C.c_void_p(stream.cuda_stream)),
           "f110qp_plan_batch_dev")
