"""HIP launch + stream-sync floor on this box: wall time per call of a one-element torch kernel
(fill_) followed by a stream synchronize, against the single-QP solve through the prepared
launcher (the bench's single_qp_device). Prints one JSON line.

usage: python tools/launch_floor.py [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
from f110qp import capi, workload  # noqa: E402


def wall(fn, stream, reps):
    for _ in range(50):
        fn()
    stream.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        stream.synchronize()
        t.append(time.perf_counter() - t0)
    t = np.sort(np.array(t) * 1e6)
    return dict(p50_us=round(float(np.percentile(t, 50)), 2), p99_us=round(float(np.percentile(t, 99)), 2),
                min_us=round(float(t[0]), 2))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    one = torch.zeros(1, device=dev)
    out = {"empty_fill_sync": wall(lambda: one.fill_(1.0), stream, reps)}
    N = 20
    w = workload.make_batch(1, N, seed=3)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    s = capi.Solver(capi.default_config(N))
    u = torch.empty(1, N, 2, device=dev)
    x = torch.empty(1, N + 1, 3, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    launch = s.prepare_dev(T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), None, u, x, st, stream=stream)
    out["single_qp_solve_sync"] = wall(launch, stream, reps)
    s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
