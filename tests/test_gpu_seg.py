"""Parity of the partitioned-horizon lane kernel (csrc/lane_seg_kernel.h: each QP's horizon split
over S = 2 / 4 / 8 lanes, a Riccati recursion over the segment ends) with the exact optimum of the
CPU oracle, through the C ABI. F110QP_LANE_SEG forces S (1 = the sequential lane_kernel.h).
Tolerance: the north star's 1e-4 relative; observed at the fp32 output rounding (~1e-7)."""
import numpy as np
import pytest

from f110qp import workload

from test_gpu_parity import TOL, check, rel_err

pytestmark = pytest.mark.gpu


def _lane(capi, N, **cfg):
    return capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE, **cfg))


@pytest.mark.parametrize("S,N", [(2, 2), (2, 10), (4, 20), (2, 30), (8, 40), (4, 40), (2, 40), (8, 48), (4, 4),
                                 (8, 16), (4, 30), (8, 30), (8, 20), (4, 17), (2, 25), (8, 47), (4, 9), (2, 3)])
def test_segments_horizons(oracle, capi, knob, monkeypatch, S, N):
    """Every segment count on horizons it divides and on horizons it does not (segments of
    floor(N / S) or one more stage, 2 .. 24), many active bounds on both faces, batch not a
    multiple of the QPs per wave; N / S < 2 keeps the sequential kernel."""
    knob("F110QP_LANE_SEG", str(S))
    w = workload.make_batch(1000, N, seed=9100 + 10 * S + N, heading="true", lateral=1.5, steer_range=1.0)
    s = _lane(capi, N)
    assert s.lane_segments(1000) == (S if N // S >= 2 else 1)
    s.close()
    u, x, st, it = check(oracle, capi, N, w, backend=capi.BACKEND_LANE)
    assert (st == capi.SOLVED).all()


@pytest.mark.parametrize("rot", ["0", "1"])
@pytest.mark.parametrize("S", ["2", "4"])
def test_segments_general_frame_far_origin(oracle, capi, knob, monkeypatch, rot, S):
    """Heading frame (q0 == q1) and general frame (F110QP_LANE_ROT=0), headings all round the
    circle, 1 km from the origin."""
    knob("F110QP_LANE_SEG", S)
    knob("F110QP_LANE_ROT", rot)
    N, B = 20, 1500
    w = workload.make_batch(B, N, seed=6161, heading="true", lateral=1.5, steer_range=1.0)
    w["x0"][:, 2] = np.random.default_rng(5).uniform(-np.pi, np.pi, B).astype(np.float32)
    w["x0"][:, :2] += np.float32(1000.0)
    w["x_ref"][:, :, :2] += np.float32(1000.0)
    check(oracle, capi, N, w, backend=capi.BACKEND_LANE)


def test_segments_custom_weights(oracle, capi, knob, monkeypatch):
    """q0 != q1 (general frame), other R, u_des inside the box, narrow bounds."""
    knob("F110QP_LANE_SEG", "4")
    N = 20
    over = dict(q=[3.0, 7.0, 2.0], r=[0.5, 1.5], u_des=[3.7, 0.05], u_min=[3.5, -0.2], u_max=[4.0, 0.2])
    w = workload.make_batch(640, N, seed=882, lateral=0.7)
    check(oracle, capi, N, w, backend=capi.BACKEND_LANE, **over)


@pytest.mark.parametrize("kmax,S,N", [("0", "4", 20), ("1", "4", 20), ("0", "8", 40), ("2", "2", 40)])
def test_segments_single_flip(oracle, capi, knob, monkeypatch, kmax, S, N):
    """Past kmax PDAS passes a QP flips only its first violation over the WHOLE horizon (the min
    over its segment lanes; the other segments undo theirs): exact results, more passes."""
    knob("F110QP_LANE_SEG", S)
    knob("F110QP_LANE_KMAX", kmax)
    knob("F110QP_LANE_TWIN", "0")  # one start: the iterates are the sequential kernel's
    w = workload.make_batch(1200, N, seed=992 + N, heading="true", lateral=1.5, steer_range=1.0)
    u, x, st, it = check(oracle, capi, N, w, backend=capi.BACKEND_LANE)
    knob("F110QP_LANE_SEG", "1")
    s = _lane(capi, N)
    _, _, _, it_seq = s.solve(w["x0"], w["u_lin"], w["x_ref"])
    s.close()
    # the same single-flip iterates as the sequential kernel (pass counts agree)
    assert np.abs(it.astype(int) - it_seq.astype(int)).max() <= 1
    monkeypatch.delenv("F110QP_LANE_KMAX")
    knob("F110QP_LANE_SEG", S)
    s = _lane(capi, N)
    _, _, _, it_pdas = s.solve(w["x0"], w["u_lin"], w["x_ref"])
    s.close()
    assert it.max() > it_pdas.max()


@pytest.mark.parametrize("S", ["2", "4", "8"])
def test_segments_agree_with_sequential(capi, knob, monkeypatch, S):
    """Same PDAS iterates as lane_kernel.h (pass counts equal on all but rounding ties), same
    status, solutions within 1e-7."""
    N, B = 40, 2048
    w = workload.make_batch(B, N, seed=2222, heading="true", lateral=1.2, steer_range=0.8)
    knob("F110QP_LANE_TWIN", "0")  # one start: the iterates are the sequential kernel's
    out = {}
    for seg in ("1", S):
        knob("F110QP_LANE_SEG", seg)
        s = _lane(capi, N)
        out[seg] = s.solve(w["x0"], w["u_lin"], w["x_ref"], objective=True)
        s.close()
    a, b = out["1"], out[S]
    np.testing.assert_array_equal(a[2], b[2])
    assert (a[3] != b[3]).mean() < 0.01
    assert rel_err(b[0], a[0].astype(np.float64)).max() <= 1e-6
    assert rel_err(b[1], a[1].astype(np.float64)).max() <= 1e-6
    np.testing.assert_allclose(b[4], a[4], rtol=1e-9, atol=1e-9 * np.abs(a[4]).max())
    np.testing.assert_allclose(b[5], a[5], rtol=1e-9, atol=1e-12)


def test_segments_objective(oracle, capi, knob, monkeypatch):
    """obj / cost outputs (the segment lanes' partial sums reduced across the QP) against the
    oracle's objective of its exact optimum."""
    knob("F110QP_LANE_SEG", "4")
    N, B = 40, 500
    w = workload.make_batch(B, N, seed=1717, heading="true", lateral=1.0, steer_range=0.6)
    s = _lane(capi, N)
    u, x, st, it, obj, cost = s.solve(w["x0"], w["u_lin"], w["x_ref"], objective=True)
    s.close()
    prm = oracle.params(N)
    ur, xr, sr, obr = oracle.solve_batch(prm, w["x0"], w["u_lin"], w["x_ref"], objective=True)
    np.testing.assert_array_equal(st, sr)
    np.testing.assert_allclose(obj, obr, rtol=1e-6, atol=1e-6)
    cr = oracle.tracking_cost(prm, ur, xr, w["x_ref"])
    assert (np.abs(cost - cr) <= 1e-6 * np.maximum(1.0, cr)).all(), np.abs(cost - cr).max()
    assert np.isfinite(obj).all() and (cost >= 0).all()


def test_segments_warm_closed_loop(oracle, capi, monkeypatch):
    """C5 as a closed loop on the segmented kernel (auto picks S = 4 at 4,096 x N = 20): every tick
    at the exact optimum, warm passes no more than cold on average."""
    N, B, T = 20, 4096, 6
    prm = oracle.params(N)
    ref = []

    def solve(x0, ul, xr):
        u, x, st = oracle.solve_batch(prm, x0, ul, xr)
        ref.append((u, x, st))
        return u

    ticks = workload.closed_loop_stream(solve, B, N, T, seed=56)
    warm = _lane(capi, N, warm_start=1)
    assert warm.lane_segments(B) == 4
    for t, w in enumerate(ticks):
        u, x, st, it = warm.solve(w["x0"], w["u_lin"], w["x_ref"])
        ur, xr, sr = ref[t]
        np.testing.assert_array_equal(st, sr)
        assert rel_err(u, ur).max() <= TOL and rel_err(x, xr).max() <= TOL, t
    warm.close()


def test_segments_non_finite(oracle, capi, knob, monkeypatch):
    """NaN / inf inputs: NUMERICAL and NaN outputs on every segment of those QPs only."""
    knob("F110QP_LANE_SEG", "4")
    N, B = 20, 777
    w = workload.make_batch(B, N, seed=1414)
    bad = {3: ("x_ref", (3, 17, 0), np.nan), 70: ("x0", (70, 2), np.inf), 130: ("u_lin", (130, 1), np.nan),
           776: ("x_ref", (776, N - 1, 2), np.nan)}
    for b, (k, idx, v) in bad.items():
        w[k][idx] = v
    s = _lane(capi, N)
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"])
    s.close()
    badi = np.array(sorted(bad))
    assert (st[badi] == capi.NUMERICAL).all()
    assert np.isnan(u[badi]).all() and np.isnan(x[badi]).all()
    good = np.setdiff1d(np.arange(B), badi)[::7]
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][good], w["u_lin"][good], w["x_ref"][good])
    assert (st[good] == capi.SOLVED).all()
    assert rel_err(u[good], ur).max() <= TOL and rel_err(x[good], xr).max() <= TOL


def test_segments_degenerate_bound(oracle, capi, knob, monkeypatch):
    """u_des on the speed bound with Q = 0: zero multipliers; the flip tolerances hold on the
    segmented kernel too."""
    knob("F110QP_LANE_SEG", "4")
    N = 20
    for q in ([0.0, 0.0, 0.0], [1e-9, 1e-9, 0.0]):
        w = workload.make_batch(700, N, seed=4500, heading="true", lateral=0.0, steer_range=0.0)
        u, x, st, it = check(oracle, capi, N, w, backend=capi.BACKEND_LANE, tol=2e-6, q=q)
        assert (st == capi.SOLVED).all()


@pytest.mark.parametrize("S,N", [("4", 20), ("8", 40), ("2", 30)])
def test_segments_refresh_and_stored_gains_agree(oracle, capi, knob, monkeypatch, S, N):
    """The two ways the segmented kernel applies the segment-end multiplier lam_j to the
    feed-forward: the lam-gains F_i kept in the scratch (where the LDS holds 14 doubles per stage)
    and the refresh sweep (F110QP_LANE_DREF=0 forces it): same status, solutions within 1e-6, both
    at the exact optimum."""
    knob("F110QP_LANE_SEG", S)
    w = workload.make_batch(900, N, seed=7300 + N, heading="true", lateral=1.2, steer_range=0.8)
    out = {}
    for dref in ("1", "0"):
        knob("F110QP_LANE_DREF", dref)
        out[dref] = check(oracle, capi, N, w, backend=capi.BACKEND_LANE)
    np.testing.assert_array_equal(out["0"][2], out["1"][2])
    assert rel_err(out["1"][0], out["0"][0].astype(np.float64)).max() <= 1e-6


@pytest.mark.parametrize("S,N", [(2, 20), (4, 20), (8, 40), (4, 40), (2, 40), (4, 30)])
def test_segments_fp32_scratch(oracle, capi, knob, monkeypatch, S, N):
    """Float references and Riccati scratch (F110QP_LANE_SEG_F32=1; AUTO takes them where fp64
    does not fit, e.g. 16,384 x N = 40): many active bounds on both faces, the exact optimum within
    the fp32-gain tolerance of test_lane_backend_scratch_modes."""
    knob("F110QP_LANE_SEG", str(S))
    knob("F110QP_LANE_SEG_F32", "1")
    w = workload.make_batch(1000, N, seed=9300 + 10 * S + N, heading="true", lateral=1.5, steer_range=1.0)
    s = _lane(capi, N)
    assert s.lane_segments(1000) == S
    assert s.backend_info(1000)[2] == 2  # LDS fp32
    s.close()
    u, x, st, it = check(oracle, capi, N, w, backend=capi.BACKEND_LANE, tol=2e-6)
    assert (st == capi.SOLVED).all()
    assert (u >= np.float32([3.0, -0.43])).all() and (u <= np.float32([4.5, 0.43])).all()


@pytest.mark.parametrize("kmax", ["16", "0"])
def test_segments_fp32_degenerate_bound(oracle, capi, knob, monkeypatch, kmax):
    """des_vel = umax with Q = 0 / tiny Q (a zero-multiplier active bound) on fp32 scratch: the
    single-flip passes' fp32 tolerance settles it (lane_kernel.h's HBM-fp32 rule)."""
    knob("F110QP_LANE_SEG", "4")
    knob("F110QP_LANE_SEG_F32", "1")
    knob("F110QP_LANE_KMAX", kmax)
    N = 20
    for q in ([0.0, 0.0, 0.0], [1e-9, 1e-9, 0.0], [1e-3, 1e-3, 0.0]):
        w = workload.make_batch(700, N, seed=4500, heading="true", lateral=0.0, steer_range=0.0)
        u, x, st, it = check(oracle, capi, N, w, backend=capi.BACKEND_LANE, tol=1e-5, q=q)
        assert (st == capi.SOLVED).all(), (q, np.unique(st, return_counts=True))


def test_c4_32768_per_gpu_two_rounds(oracle, capi):
    """65,536 over 2 GPUs: 32,768 x N = 40 per GPU on the segmented kernel at S = 4 with fp32
    scratch in two dispatch rounds (2,048 waves, four resident per CU by LDS). Parity on a
    strided sample that covers both rounds plus the scenario at the round boundary."""
    N, B = 40, 32768
    g = workload.make_grouped_batch(274, N, seed=4044)
    w = {k: np.ascontiguousarray(g[k][:B]) for k in ("x0", "u_lin", "x_ref")}
    s = capi.Solver(capi.default_config(N))
    assert s.lane_segments(B) == 4 and s.backend_info(B)[2] == 2
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"])
    s.close()
    assert (st == capi.SOLVED).all()
    idx = np.concatenate([np.arange(0, B, 41), np.arange(16320, 16440)])
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][idx], w["u_lin"][idx], w["x_ref"][idx])
    assert (sr == oracle.SOLVED).all()
    assert rel_err(u[idx], ur).max() <= 2e-6 and rel_err(x[idx], xr).max() <= 2e-6


def test_c4_16384_per_gpu_auto(oracle, capi):
    """The middle of the C4 strong-scaling curve: 16,384 x N = 40 QPs per GPU (65,536 over 4
    GPUs). AUTO runs the segmented kernel at S = 4 on fp32 scratch (fp64 does not fit four waves
    per CU); parity on a strided sample plus two whole scenarios."""
    N, B = 40, 16384
    g = workload.make_grouped_batch(137, N, seed=4043)
    w = {k: np.ascontiguousarray(g[k][:B]) for k in ("x0", "u_lin", "x_ref")}
    s = capi.Solver(capi.default_config(N))
    assert s.lane_segments(B) == 4 and s.backend_info(B)[2] == 2
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"])
    s.close()
    assert (st == capi.SOLVED).all()
    idx = np.concatenate([np.arange(0, B, 23), np.arange(600, 840)])
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][idx], w["u_lin"][idx], w["x_ref"][idx])
    assert (sr == oracle.SOLVED).all()
    assert rel_err(u[idx], ur).max() <= 2e-6 and rel_err(x[idx], xr).max() <= 2e-6


@pytest.mark.parametrize("N,B", [(20, 1024), (20, 2048), (20, 4096), (20, 8192), (30, 1000), (40, 512), (20, 1)])
def test_twin_starts_match_one_start(oracle, capi, knob, N, B):
    """Twin starts (f110qp_lane_starts = 2: every QP also solved from the speed bound u_des sits on
    held over the first half of the horizon, the first start to converge answers): the same statuses
    and optimum as one start (F110QP_LANE_TWIN=0), never more passes, fewer on the QPs whose cold PDAS
    walks that prefix a few stages per pass; the objective outputs from the winning start. The pass
    counts equal the numpy model's min over the two starts (DESIGN.md 2b')."""
    w = workload.make_batch(B, N, seed=8100 + N + B, heading="true", lateral=1.0, steer_range=0.6)
    out = {}
    for twin in ("1", "0"):
        knob("F110QP_LANE_TWIN", twin)
        s = _lane(capi, N)
        out[twin] = (s.lane_starts(B), s.lane_segments(B)) + tuple(s.solve(w["x0"], w["u_lin"], w["x_ref"],
                                                                           objective=True))
        s.close()
    (n2, S2, u2, x2, s2, it2, ob2, co2), (n1, S1, u1, x1, s1, it1, ob1, co1) = out["1"], out["0"]
    # twin where the doubled grid is at most two waves per CU and their lam-gain scratch fits the CU's
    # LDS (lane_seg_kernel.h seg_twin: 512 waves, 14 fp64 + 3 fp64 + 1 int per stage and lane, and two
    # 1 KiB state-code tables per wave)
    waves2 = -(-2 * B * S1 // 64)
    fits = -(-waves2 // 256) * (-(-N // max(S1, 1)) * 64 * (3 * 8 + 4 + 14 * 8) + 2048) <= 160 * 1024
    assert n1 == 1 and S2 == S1 and (n2 == 2) == (S1 > 1 and waves2 <= 512 and fits), (n1, n2, S1, S2)
    np.testing.assert_array_equal(s2, s1)
    assert (s2 == capi.SOLVED).all()
    assert rel_err(u2, u1.astype(np.float64)).max() <= 1e-6 and rel_err(x2, x1.astype(np.float64)).max() <= 1e-6
    np.testing.assert_allclose(ob2, ob1, rtol=1e-9, atol=1e-9 * np.abs(ob1).max())
    assert (it2 <= it1).all()
    if n2 == 2 and B >= 1024:
        assert it2.max() < it1.max() or it2.mean() < it1.mean()
    ur, xr, sr = oracle.solve_batch(oracle.params(N), w["x0"][::7], w["u_lin"][::7], w["x_ref"][::7])
    assert rel_err(u2[::7], ur).max() <= TOL and rel_err(x2[::7], xr).max() <= TOL
