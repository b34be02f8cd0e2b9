"""Single-QP synchronous call latency: the completion word (f110qp_api.cpp wait_done) against the
stream synchronisation (test build, F110QP_SIG_POLL=0), back to back and from an idle GPU
(the stream drained outside the timed region). Prints one JSON line per variant.

    python tools/sync_probe.py [--reps 400] [--batch 1] [--horizon 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--null-stream", action="store_true", help="launch on the legacy default stream")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--pool", type=int, default=64, help="make_batch size the QP is taken from")
    ap.add_argument("--poll", type=int, default=-1, help="1 / 0: only the completion word / only the stream")
    ap.add_argument("--host", action="store_true",
                    help="host-pointer calls instead (zero-copy staging), completion word against stream sync")
    a = ap.parse_args()
    import torch

    from f110qp import capi, workload

    N, B = a.horizon, a.batch
    w = workload.make_batch(a.pool, N, seed=a.seed)
    d = {k: torch.from_numpy(np.ascontiguousarray(w[k][:B])).cuda() for k in ("x0", "u_lin", "x_ref")}
    uo = torch.empty((B, N, 2), dtype=torch.float32, device="cuda")
    xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device="cuda")
    st = torch.empty((B,), dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream() if a.null_stream else torch.cuda.Stream()

    def pct(v):
        v = np.sort(np.asarray(v) * 1e6)
        return {"p50_us": round(float(np.percentile(v, 50)), 2), "p99_us": round(float(np.percentile(v, 99)), 2),
                "min_us": round(float(v[0]), 2)}

    if a.host:
        hx = {k: np.ascontiguousarray(w[k][:B]) for k in ("x0", "u_lin", "x_ref")}
        for poll in (1, 0):
            os.environ["F110QP_SIG_POLL"] = str(poll)
            s = capi.Solver(capi.default_config(N), test_build=True)
            for _ in range(50):
                s.solve(hx["x0"], hx["u_lin"], hx["x_ref"])
            back = []
            for i in range(a.reps):
                t0 = time.perf_counter()
                s.solve(hx["x0"], hx["u_lin"], hx["x_ref"])
                back.append(time.perf_counter() - t0)
            print(json.dumps({"host": True, "poll": poll, "signals": s.sync_signals(), "back_to_back": pct(back)}))
            s.close()
        return
    for poll in ((1, 0) if a.poll < 0 else (a.poll,)):
        os.environ["F110QP_SIG_POLL"] = str(poll)
        s = capi.Solver(capi.default_config(N), test_build=(poll == 0))  # the knob needs the test build
        f = s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, uo, xo, st, stream=stream, sync=True)
        g = s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], None, uo, xo, st, stream=stream)
        for _ in range(50):
            f()
        back, idle, spin = [], [], []
        for i in range(a.reps):
            t0 = time.perf_counter()
            f()
            back.append(time.perf_counter() - t0)
        for i in range(a.reps):
            stream.synchronize()
            time.sleep(50e-6)
            t0 = time.perf_counter()
            f()
            idle.append(time.perf_counter() - t0)
        # asynchronous launch + torch stream synchronize, idle start
        for i in range(a.reps):
            stream.synchronize()
            time.sleep(50e-6)
            t0 = time.perf_counter()
            g()
            stream.synchronize()
            spin.append(time.perf_counter() - t0)
        # launch alone (the asynchronous call's host cost)
        la = []
        for i in range(a.reps):
            stream.synchronize()
            t0 = time.perf_counter()
            g()
            la.append(time.perf_counter() - t0)
        stream.synchronize()
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ea.record(stream)
        for _ in range(50):
            g()
        eb.record(stream)
        torch.cuda.synchronize()
        print(json.dumps({"poll": poll, "null_stream": a.null_stream, "seed": a.seed, "signals": s.sync_signals(), "kernel_us": round(ea.elapsed_time(eb) * 20.0, 2),
                          "back_to_back": pct(back),
                          "idle_start": pct(idle), "async_then_sync_idle": pct(spin), "launch_only": pct(la)}))
        s.close()


if __name__ == "__main__":
    main()
