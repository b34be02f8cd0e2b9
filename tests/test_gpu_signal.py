"""Completion word of the synchronous calls (f110qp_api.cpp arm_signal / wait_done, signal_call_done
in f110qp_kernels.h): f110qp_solve_batch_dev_sync and the zero-copy host-pointer calls (<= 64 QPs)
return when the call's last kernel has published the call's number to a pinned host word, not
after hipStreamSynchronize. The outputs must then be complete:
read back on ANOTHER stream with no dependency on the solve's, and equal, bit for bit, to the
same calls waiting on the stream (the test build's F110QP_SIG_POLL=0) and to the asynchronous entry
point. Every ungrouped call whose last kernel (lane, wave or the gap rows' fp64 re-check) has at
most 256 workgroups is armed; larger grids, grouped calls and staged host calls (> 64 QPs)
synchronise the stream."""
import numpy as np
import pytest

from f110qp import workload

pytestmark = pytest.mark.gpu

N = 20


def _dev_inputs(torch, w):
    return {k: torch.from_numpy(np.ascontiguousarray(w[k])).cuda() for k in ("x0", "u_lin", "x_ref")}


def _dev_outputs(torch, B, N):
    return (torch.full((B, N, 2), -7.0, dtype=torch.float32, device="cuda"),
            torch.full((B, N + 1, 3), -7.0, dtype=torch.float32, device="cuda"),
            torch.full((B,), -7, dtype=torch.int32, device="cuda"),
            torch.full((B,), -7, dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("B,lane", [(1, False), (8, False), (64, True), (1024, False), (4096, False)])
def test_dev_sync_outputs_complete_on_return(capi, knob, B, lane):
    """20 calls with fresh inputs in the same device buffers: after each dev_sync returns, the
    outputs read on the default stream (no dependency on the solve's side stream) equal the
    stream-synchronised solver's and the asynchronous call's; the poll answered every call up to
    256 waves. (64 QPs
    at N = 20 go to the wave back end under AUTO: forced onto the lane back end here.)"""
    import torch
    cfg = dict(backend=capi.BACKEND_LANE) if lane else {}
    sig = capi.Solver(capi.default_config(N, **cfg))
    knob("F110QP_SIG_POLL", 0)
    ref = capi.Solver(capi.default_config(N, **cfg))
    assert sig.test_build and ref.test_build
    assert sig.backend_info(B)[0] == capi.BACKEND_LANE and sig.lane_segments(B) > 1
    side = torch.cuda.Stream()
    w = workload.make_batch(B, N, seed=300 + B)
    d = _dev_inputs(torch, w)
    outs = {k: _dev_outputs(torch, B, N) for k in ("sig", "ref", "async")}
    launch = {
        "sig": sig.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, *outs["sig"], stream=side, sync=True),
        "ref": ref.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, *outs["ref"], stream=side, sync=True),
        "async": ref.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, *outs["async"], stream=side),
    }
    for call in range(20):
        w = workload.make_batch(B, N, seed=1000 * B + call)
        with torch.cuda.stream(side):
            for k in d:
                d[k].copy_(torch.from_numpy(np.ascontiguousarray(w[k])))
        got = {}
        for k in ("sig", "ref", "async"):
            for t in outs[k]:
                t.fill_(-7)  # on the default stream
            torch.cuda.current_stream().synchronize()
            launch[k]()
            if k == "async":
                side.synchronize()
            # read back on the default stream: no ordering with `side` but the call's own wait
            got[k] = [t.cpu().numpy() for t in outs[k]]
        for a, b, c in zip(got["sig"], got["ref"], got["async"]):
            np.testing.assert_array_equal(a, b)
            np.testing.assert_array_equal(a, c)
        assert (got["sig"][2] == capi.SOLVED).all(), call
    # armed up to 256 waves in the last kernel (f110qp_kernels.hip kSignalMaxGrid): 4,096 QPs with
    # twin starts are 512 waves and synchronise the stream
    assert sig.sync_signals() == (20 if B <= 1024 else 0)
    assert ref.sync_signals() == 0
    sig.close()
    ref.close()


@pytest.mark.parametrize("B,lane", [(1, False), (7, False), (64, True), (65, True)])
def test_host_calls_poll_the_completion_word(capi, knob, B, lane):
    """The host-pointer entry point: up to 64 QPs the kernel stores the outputs straight into the
    pinned staging buffer and the call waits on the completion word; 65 QPs stage through device
    memory and wait for the D2H copy on the stream. Either way the answers equal the
    stream-synchronised solver's on every call, objectives included."""
    cfg = dict(backend=capi.BACKEND_LANE) if lane else {}
    sig = capi.Solver(capi.default_config(N, **cfg))
    knob("F110QP_SIG_POLL", 0)
    ref = capi.Solver(capi.default_config(N, **cfg))
    assert sig.backend_info(B)[0] == capi.BACKEND_LANE and sig.lane_segments(B) > 1
    for call in range(20):
        w = workload.make_batch(B, N, seed=7000 + 100 * B + call)
        a = sig.solve(w["x0"], w["u_lin"], w["x_ref"], objective=True)
        b = ref.solve(w["x0"], w["u_lin"], w["x_ref"], objective=True)
        for p, q in zip(a, b):
            np.testing.assert_array_equal(p, q)
    assert sig.sync_signals() == (20 if B <= 64 else 0)
    assert ref.sync_signals() == 0
    sig.close()
    ref.close()


def test_signal_across_streams_and_entry_points(capi):
    """One solver whose calls alternate between dev_sync on two streams, asynchronous calls, and
    host-pointer calls, with the warm start on (lane back end): the arrival count the kernel re-zeroes and the call
    number stay consistent, every answer equals a fresh solver's."""
    import torch
    B = 256
    s = capi.Solver(capi.default_config(N, warm_start=1, backend=capi.BACKEND_LANE))
    fresh = capi.Solver(capi.default_config(N, warm_start=1, backend=capi.BACKEND_LANE))
    assert s.lane_segments(B) > 1
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    armed = 0
    for call in range(24):
        w = workload.make_batch(B, N, seed=500 + (call % 5))  # repeats: the warm keys hit
        want = fresh.solve(w["x0"], w["u_lin"], w["x_ref"])
        kind = call % 4
        if kind == 3:
            got = s.solve(w["x0"], w["u_lin"], w["x_ref"])  # 256 QPs: staged, stream-synchronised
        else:
            d = _dev_inputs(torch, w)
            o = _dev_outputs(torch, B, N)
            torch.cuda.current_stream().synchronize()
            st = streams[call % 2]
            s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, *o, stream=st, sync=kind != 2)()
            if kind == 2:
                st.synchronize()
            else:
                armed += 1
            got = [t.cpu().numpy() for t in o]
        for p, q in zip(got, want):
            np.testing.assert_array_equal(p, q)
    assert s.sync_signals() == armed
    s.close()
    fresh.close()


@pytest.mark.parametrize("backend", ["seq", "wave", "gap"])
def test_every_ungrouped_call_signals_from_its_last_kernel(capi, knob, backend):
    """The sequential lane kernel (F110QP_LANE_SEG=1), the wave kernel's box path and a gap-row call
    (lane screen or not, GI, then the fp64 re-check: the last kernel signals from its last
    workgroup) all answer synchronous calls through the completion word; the answers equal the
    asynchronous entry point's, on the device and through host pointers."""
    import torch
    B = 64
    if backend == "seq":
        knob("F110QP_LANE_SEG", 1)
        s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_LANE))
        assert s.lane_segments(B) == 1
    elif backend == "wave":
        s = capi.Solver(capi.default_config(N, backend=capi.BACKEND_WAVE))
    else:
        s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE))
    w = workload.make_batch(B, N, seed=41)
    hs = np.zeros((B, 2, 3), np.float32)
    hs[:, :, 2] = 1.0  # 0 x + 0 y >= -1: rows that never bind
    d = _dev_inputs(torch, w)
    h = torch.from_numpy(hs).cuda() if backend == "gap" else None
    o1, o2 = _dev_outputs(torch, B, N), _dev_outputs(torch, B, N)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], h, *o1, stream=side, sync=True)()
    r1 = [t.cpu().numpy() for t in o1]  # read on the default stream
    s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], h, *o2)()
    torch.cuda.synchronize()
    r2 = [t.cpu().numpy() for t in o2]
    for p, q in zip(r1, r2):
        np.testing.assert_array_equal(p, q)
    assert (r1[2] == capi.SOLVED).all()
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs if h is not None else None)
    np.testing.assert_array_equal(u, r1[0])
    assert s.sync_signals() == 2
    s.close()


@pytest.mark.parametrize("screen", ["0", "1"])
def test_gap_call_signal_with_rechecked_qps(capi, knob, screen):
    """A synchronous gap-row call whose re-check list is not empty (the N = 48 stiff golden fixture:
    GI leaves QPs uncertified), with and without the box screen: the completion word comes from the
    re-check's last workgroup after every listed QP is rewritten; the outputs equal the
    stream-synchronised call's (F110QP_SIG_POLL=0) bit for bit."""
    import json
    import os
    from conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "stiff_gap_n48_dt005.npz"))
    src = str(d["source"])
    knob("F110QP_GAP_SCREEN", screen)
    over = json.loads(str(d["params"]))
    import torch
    N2, B = int(d["horizon"]), d["x0"].shape[0]
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k])).cuda() for k in ("x0", "u_lin", "x_ref", "halfspace")}
    res = {}
    for poll in ("1", "0"):
        knob("F110QP_SIG_POLL", poll)
        s = capi.Solver(capi.default_config(N2, gap_mode=capi.GAP_ACTIVE, **over))
        o = _dev_outputs(torch, B, N2)
        torch.cuda.synchronize()
        s.prepare_dev(t["x0"], t["u_lin"], t["x_ref"], t["halfspace"], *o, stream=torch.cuda.Stream(), sync=True)()
        res[poll] = [v.cpu().numpy() for v in o]  # read on the default stream
        res[poll + "n"] = (s.sync_signals(), s.last_recheck_count())
        s.close()
    for p, q in zip(res["1"], res["0"]):
        np.testing.assert_array_equal(p, q)
    np.testing.assert_array_equal(res["1"][2], d["status"])
    assert res["1n"][0] == 1 and res["0n"][0] == 0 and res["1n"][1] > 0, (res["1n"], res["0n"], src)


def test_destroy_right_after_a_polled_call(capi):
    """f110qp_destroy right after a call that returned on its completion word (the kernel may still
    be retiring): the context waits for the device before it frees the word and the count; 30
    create / solve / destroy cycles with the answers checked against a long-lived solver."""
    import torch
    N, B = 20, 8
    w = workload.make_batch(B, N, seed=77)
    d = _dev_inputs(torch, w)
    ref = capi.Solver(capi.default_config(N))
    want = ref.solve(w["x0"], w["u_lin"], w["x_ref"])
    for k in range(30):
        s = capi.Solver(capi.default_config(N))
        o = _dev_outputs(torch, B, N)
        torch.cuda.current_stream().synchronize()
        s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, *o, sync=True)()
        assert s.sync_signals() == 1
        s.close()
        got = [t.cpu().numpy() for t in o]
        for p, q in zip(got, want):
            np.testing.assert_array_equal(p, q)
    ref.close()
