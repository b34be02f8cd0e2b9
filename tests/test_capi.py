"""The C ABI library on the CPU: it loads, exports every symbol include/f110qp.h declares,
mirrors the reference defaults and validates its arguments (no compute call needs a GPU)."""
import ctypes as C
import os
import re

import numpy as np
import pytest
from conftest import ROOT


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "f110qp.h")).read()
    return sorted(set(re.findall(r"\b(f110qp_[a-z_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol(capi):
    syms = declared_symbols()
    assert len(syms) >= 10
    assert set(syms) == set(capi.EXPORTED)
    lib = C.CDLL(capi.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s


def test_product_library_reads_no_environment(capi):
    """The product library (what bench.py times and MPC::Update links) carries no F110QP_* knob:
    its behaviour is the config alone, as the reference's fixed OSQP settings (src/mpc.cpp:98-99).
    The knobs live in the test build only (lib_test/libf110qp.so, -DF110QP_TEST_HOOKS)."""
    data = open(capi.LIB_PATH, "rb").read()
    assert b"F110QP_" not in data
    assert b"getenv" not in data
    assert capi.load().f110qp_test_build() == 0
    t = capi.load(test=True)
    assert t.f110qp_test_build() == 1
    assert b"F110QP_RECHECK_ALL" in open(capi.TEST_LIB_PATH, "rb").read()
    for sym in declared_symbols():
        assert hasattr(C.CDLL(capi.TEST_LIB_PATH), sym), sym


def test_diagnostic_queries_without_a_call(capi):
    """f110qp_last_recheck_count and f110qp_warm_hits before any solve call: zero, no HIP call."""
    s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))
    assert s.last_recheck_count() == 0
    assert s.warm_hits() == (0, 0)
    s.close()
    w = capi.Solver(capi.default_config(20, warm_start=1))
    assert w.warm_hits() == (0, 0) and w.last_recheck_count() == 0
    L = capi.load()
    assert L.f110qp_last_recheck_count(None, None) == capi.ERR_INVALID
    assert L.f110qp_warm_hits(w._h, None, None) == capi.ERR_INVALID
    w.close()


@pytest.mark.parametrize("lang,cc", [("c", "gcc"), ("c++", "g++")])
def test_header_compiles_as_c_and_cpp(lang, cc):
    """include/f110qp.h is the drop-in boundary: plain C, usable from the reference's C++."""
    import shutil
    import subprocess

    if shutil.which(cc) is None:
        pytest.skip(f"{cc} not installed")
    hdr = os.path.join(ROOT, "include", "f110qp.h")
    subprocess.run([cc, "-fsyntax-only", "-Wall", "-Werror", "-x", lang, hdr], check=True)


def test_library_is_gfx950_code_object(capi):
    data = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data  # the offload bundle targets MI355X


def test_version_and_defaults(capi):
    L = capi.load()
    assert L.f110qp_version() == 6
    c = capi.default_config(20)
    # params.yaml:1-13,42-47 and constraints.cpp:19,21
    assert c.horizon == 20 and c.dt == np.float32(0.01)
    assert list(c.q) == [10.0, 10.0, 0.0] and list(c.r) == [0.1, 5.0]
    assert list(c.u_des) == [4.5, 0.0]
    assert list(c.u_min) == [3.0, float(np.float32(-0.43))]
    assert list(c.u_max) == [4.5, float(np.float32(0.43))]
    assert c.gap_mode == capi.GAP_INACTIVE and c.backend == capi.BACKEND_AUTO


@pytest.mark.parametrize("over,msg", [
    (dict(horizon=0), "horizon"),
    (dict(horizon=49), "horizon"),
    (dict(backend=3), "backend"),
    (dict(x_ref_points=19), "x_ref_points"),
    (dict(r=[0.0, 5.0]), "R must be > 0"),
    (dict(q=[-1.0, 10.0, 0.0]), "Q must be"),
    (dict(u_min=[5.0, -0.43]), "u_min > u_max"),
    (dict(gap_mode=7), "gap_mode"),
    (dict(dt=0.0), "dt"),
    (dict(max_iter=-1), "max_iter"),
])
def test_create_rejects_bad_config(capi, over, msg):
    c = capi.default_config(20)
    for k, v in over.items():
        if k in ("q", "r", "u_min", "u_max"):
            for i, x in enumerate(v):
                getattr(c, k)[i] = x
        else:
            setattr(c, k, v)
    with pytest.raises(capi.F110QPError, match=msg):
        capi.Solver(c)


def test_solve_argument_validation_without_gpu(capi):
    s = capi.Solver(capi.default_config(20))
    L = capi.load()
    # batch 0 is a no-op, negative batch / NULL buffers are rejected before any HIP call
    assert L.f110qp_solve_batch_dev(s._h, 0, None, None, None, None, None, None, None, None, None) == capi.OK
    assert L.f110qp_solve_batch_dev(s._h, -1, None, None, None, None, None, None, None, None, None) == capi.ERR_INVALID
    assert L.f110qp_solve_batch_dev(s._h, 4, None, None, None, None, None, None, None, None, None) == capi.ERR_INVALID
    assert "non-NULL" in capi.last_error()
    assert L.f110qp_solve_batch_dev(None, 4, None, None, None, None, None, None, None, None, None) == capi.ERR_INVALID
    g = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))
    buf = np.zeros(1024, np.float32)
    p = C.c_void_p(buf.ctypes.data)
    assert L.f110qp_solve_batch_dev(g._h, 4, p, p, p, None, p, p, p, None, None) == capi.ERR_INVALID
    assert "halfspace" in capi.last_error()
    s.close()
    g.close()
    capi.Solver(capi.default_config(20)).close()  # create/destroy never touches the device


def test_device_tensor_checks_before_the_abi(capi):
    """The binding refuses tensors whose raw pointer would be misread or overrun by the kernels
    (float32 obj/cost, int64 status/group/winner, short or strided buffers)."""
    import torch

    N, B = 20, 8
    s = capi.Solver(capi.default_config(N))
    f = lambda *sh: torch.zeros(*sh, dtype=torch.float32)  # noqa: E731
    i = lambda *sh: torch.zeros(*sh, dtype=torch.int32)  # noqa: E731
    args = [f(B, 3), f(B, 2), f(B, N, 3), None, f(B, N, 2), f(B, N + 1, 3), i(B)]
    with pytest.raises(capi.F110QPError, match="obj must be torch.float64"):
        s.solve_dev(*args, obj=f(B))
    with pytest.raises(capi.F110QPError, match="status must be torch.int32"):
        s.solve_dev(*args[:6], torch.zeros(B, dtype=torch.int64))
    with pytest.raises(capi.F110QPError, match="u_out holds"):
        s.solve_dev(*args[:4], f(B - 1, N, 2), *args[5:])
    with pytest.raises(capi.F110QPError, match="x_ref must be contiguous"):
        s.solve_dev(args[0], args[1], f(B, 3, N).transpose(1, 2), *args[3:])
    with pytest.raises(capi.F110QPError, match="device"):
        s.solve_dev(*args)  # host tensors
    with pytest.raises(capi.F110QPError, match="group must be torch.int32"):
        s.prepare_grouped_dev(*args[:4], torch.zeros(B, dtype=torch.int64), 2, *args[4:])
    with pytest.raises(capi.F110QPError, match="best_cost must be torch.float64"):
        capi.select_dev(i(B), 2, torch.zeros(B, dtype=torch.float64), i(B), i(2), f(2))
    with pytest.raises(capi.F110QPError, match="winner holds"):
        capi.select_dev(i(B), 4, torch.zeros(B, dtype=torch.float64), i(B), i(2), torch.zeros(4, dtype=torch.float64))
    g = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE))
    with pytest.raises(capi.F110QPError, match="halfspace is required"):
        g.solve_dev(*args)
    s.close()
    g.close()


def test_find_half_spaces_no_gap_is_an_error(capi):
    r = np.full(1080, 1.0, np.float32)
    with pytest.raises(capi.F110QPError, match="no gap"):
        capi.find_half_spaces([0, 0, 0], r, -np.pi, 2 * np.pi / 1080, np.pi)


def test_product_does_not_import_the_oracle():
    """The shipped path never routes through the checker (no CPU fallback)."""
    pkg = os.path.join(ROOT, "f110-mpc_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".hpp")) or f == "Makefile":
                txt = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "import oracle" not in txt and "liboracle" not in txt and "f110_oracle" not in txt, f


def test_capi_raises_when_library_missing(monkeypatch):
    from f110qp import capi

    monkeypatch.setattr(capi, "_libs", {})
    monkeypatch.setattr(capi, "LIB_PATH", "/nonexistent/libf110qp.so")
    with pytest.raises(capi.F110QPError, match="not built"):
        capi.load()


def test_auto_backend_policy(capi):
    """BACKEND_AUTO: the wave kernel for mid-size box batches and for gap rows, the lane kernel
    from the measured crossover (1,024 QPs at N <= 32; every batch at N > 32) and for the single
    QP of MPC::Update (up to 8 QPs at N <= 32: the partitioned horizon beats one QP's wave chain),
    mirrored by the library's own resolution (f110qp_backend_info)."""
    for B in (1, 4, 8):
        assert capi.auto_backend(20, B, False) == capi.BACKEND_LANE
    assert capi.auto_backend(20, 9, False) == capi.BACKEND_WAVE
    s = capi.Solver(capi.default_config(20))
    for B in (1, 8, 9, 512, 1023, 1024, 4096):
        assert s.backend_info(B)[0] == capi.auto_backend(20, B, False), B
    assert s.lane_segments(1) == 4
    s.close()
    assert capi.auto_backend(20, 512, False) == capi.BACKEND_WAVE
    assert capi.auto_backend(20, 1023, False) == capi.BACKEND_WAVE
    assert capi.auto_backend(20, 1024, False) == capi.BACKEND_LANE
    assert capi.auto_backend(20, 4096, False) == capi.BACKEND_LANE
    assert capi.auto_backend(20, 65536, True) == capi.BACKEND_WAVE
    assert capi.auto_backend(40, 1, False) == capi.BACKEND_LANE
    assert capi.auto_backend(40, 768, True) == capi.BACKEND_WAVE


def test_auto_backend_grouped_policy(capi):
    """Grouped calls follow the ungrouped thresholds: the C4 shard (8,192 x N = 40) and the full
    C4 batch run on the lane kernel (grouped wave measured 1,041 vs 240 us at the shard)."""
    assert capi.auto_backend(40, 8192, False, grouped=True) == capi.BACKEND_LANE
    assert capi.auto_backend(40, 65536, False, grouped=True) == capi.BACKEND_LANE
    assert capi.auto_backend(40, 1, False, grouped=True) == capi.BACKEND_LANE
    assert capi.auto_backend(20, 1023, False, grouped=True) == capi.BACKEND_WAVE
    assert capi.auto_backend(20, 1, False, grouped=True) == capi.BACKEND_WAVE  # grouped: thresholds only


def test_gap_screen_policy(capi):
    """Gap rows under AUTO take the box screen on the lane back end from F110QP_GAP_SCREEN_MIN_BATCH
    QPs (ungrouped, no warm start); an explicit LANE back end at every batch size (no warm start),
    an explicit WAVE back end never. Mirrored by capi.auto_gap_screen."""
    sg = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))
    for B in (1, 512, 1023, 1024, 4096, 65536):
        assert sg.gap_screen(B) == capi.auto_gap_screen(B) == (B >= capi.GAP_SCREEN_MIN_BATCH), B
    sg.close()
    for over in (dict(backend=capi.BACKEND_WAVE), dict(warm_start=1),
                 dict(backend=capi.BACKEND_LANE, warm_start=1)):
        s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE, **over))
        assert not s.gap_screen(4096), over
        s.close()
    s = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
    assert all(s.gap_screen(B) for B in (1, 64, 4096, 65536))
    s.close()
    s = capi.Solver(capi.default_config(20))  # box rows: nothing to screen
    assert not s.gap_screen(4096)
    s.close()


def test_qp_dims_match_reference_sizes(capi, oracle):
    """f110qp_qp_dims: the reference's n = 5N+3, m = 7N+5 (src/mpc.cpp:26-29) and the stored
    nonzeros of P and A, equal to the oracle's assembly for every horizon."""
    for N in (1, 20, 30, 40, 48):
        assert capi.qp_dims(N) == oracle.dims(N)


def test_backend_info_resolves_auto_and_scratch(capi):
    """f110qp_backend_info (host only, no device needed): AUTO resolves to the lane back end at
    the measured thresholds (F110QP_LANE_MIN_BATCH[_WIDE]), gap rows to the wave back end (an
    explicit F110QP_BACKEND_LANE reports the box screen's lane solve);
    the lane QPs-per-wave fill <= 256 waves; the scratch sits in LDS (fp64 when it fits) while the
    grid's waves are resident with it and in HBM (fp32) at the C4 size."""
    s20 = capi.Solver(capi.default_config(20))
    assert s20.backend_info(512) == (capi.BACKEND_WAVE, 1, 0)
    assert s20.backend_info(1024) == (capi.BACKEND_LANE, 16, 1)  # C2: segmented, S = 4
    assert s20.backend_info(capi.LANE_MIN_BATCH)[0] == capi.BACKEND_LANE
    assert s20.backend_info(4096) == (capi.BACKEND_LANE, 16, 1)
    assert s20.backend_info(65536) == (capi.BACKEND_LANE, 64, 4)
    s40 = capi.Solver(capi.default_config(40))
    assert s40.backend_info(1)[0] == capi.BACKEND_LANE
    # small batches split every QP's horizon over S lanes (lane_seg_kernel.h): 64 / S QPs per wave
    assert s40.backend_info(8192, grouped=True) == (capi.BACKEND_LANE, 8, 1)
    assert s40.lane_segments(8192) == 8 and s20.lane_segments(4096) == 4
    assert s20.lane_segments(65536) == 1 and s20.lane_segments(1024) == 4 and s20.lane_segments(512) == 1
    # horizons S does not divide: segments of floor(N / S) or one more stage (the reference's
    # default N = 30 and odd N)
    s30, s25 = capi.Solver(capi.default_config(30)), capi.Solver(capi.default_config(25))
    assert s30.lane_segments(4096) == 8 and s25.lane_segments(4096) == 8
    # fp64 scratch at 16,384 x N = 30 would need 222 KB of LDS per CU: float scratch, S = 4
    assert s30.lane_segments(16384) == 4 and s30.backend_info(16384)[2] == 2
    # the middle of the C4 curve (65,536 over 4 / 2 GPUs): 16,384 x N = 40 on fp32 LDS scratch at
    # S = 4 in one dispatch round, 32,768 at S = 4 in two (four of its eight waves per CU fit the
    # LDS at once), 65,536 keeps the HBM-scratch sequential kernel
    assert s40.lane_segments(16384) == 4 and s40.backend_info(16384) == (capi.BACKEND_LANE, 16, 2)
    assert s40.lane_segments(32768) == 4 and s40.backend_info(32768)[2] == 2
    assert s40.lane_segments(65536) == 1 and s40.backend_info(65536)[2] == 4
    s30.close()
    s25.close()
    assert s40.backend_info(65536, grouped=True) == (capi.BACKEND_LANE, 64, 4)
    sg = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE))
    assert sg.backend_info(65536)[0] == capi.BACKEND_WAVE and sg.backend_info(4096)[0] == capi.BACKEND_WAVE
    sl = capi.Solver(capi.default_config(20, gap_mode=capi.GAP_ACTIVE, backend=capi.BACKEND_LANE))
    assert sl.backend_info(4096) == (capi.BACKEND_LANE, 16, 1) and sl.lane_segments(4096) == 4
    assert sl.backend_info(65536) == (capi.BACKEND_LANE, 64, 4)  # the box solve's sequential kernel
    sl.close()
    for s in (s20, s40, sg):
        s.close()
