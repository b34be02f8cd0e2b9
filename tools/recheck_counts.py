"""How many QPs each gap-row case sends to the fp64 re-check (f110qp_last_recheck_count, product
library), and what the whole solve call costs with those QPs in it (call_us: HIP events around 5
device calls after a warm-up, inputs resident): the screen fuzz corners of tests/test_gpu_screen.py
(AUTO path), the committed gap-row fixtures and the bench's C3 batch. One JSON line (DESIGN.md 2g;
round-5 ADVICE: a timed record of stiff batches that fill the re-check list). Needs the oracle only
for the half-spaces (the checker's FindHalfSpaces, as the tests)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("f110-mpc_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: E402  (torch's HIP runtime first, as the tests)

torch.cuda.is_available()
import oracle  # noqa: E402
from f110qp import capi, workload  # noqa: E402
from fuzz_cases import screen_fuzz_case  # noqa: E402


def hs_of(x0, ranges, geom):
    hs = np.zeros((x0.shape[0], 2, 3), np.float32)
    for b in range(x0.shape[0]):
        rc, l1, l2, _, _ = oracle.find_half_spaces(x0[b].astype(np.float64), ranges[b], *geom)
        hs[b] = l1, l2
    return hs


def count(N, w, hs, **over):
    s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE, **over))
    u, x, st, it = s.solve(w["x0"], w["u_lin"], w["x_ref"], hs)
    n = s.last_recheck_count()
    B = int(w["x0"].shape[0])
    d = {k: torch.from_numpy(np.ascontiguousarray(w[k])).cuda() for k in ("x0", "u_lin", "x_ref")}
    dh = torch.from_numpy(np.ascontiguousarray(hs)).cuda()
    o = (torch.empty((B, N, 2), device="cuda"), torch.empty((B, N + 1, 3), device="cuda"),
         torch.empty((B,), dtype=torch.int32, device="cuda"))
    f = s.prepare_dev(d["x0"], d["u_lin"], d["x_ref"], dh, *o)
    f()
    ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ea.record()
    for _ in range(5):
        f()
    eb.record()
    torch.cuda.synchronize()
    s.close()
    return dict(B=B, rechecked=n, solved=int((st == capi.SOLVED).sum()),
                inaccurate=int((st == capi.SOLVED_INACCURATE).sum()),
                infeasible=int((st == capi.PRIMAL_INFEASIBLE).sum()),
                call_us=round(ea.elapsed_time(eb) * 1000.0 / 5, 1))


def main():
    oracle.build()
    out = {}
    for seed in range(3):
        for case in range(2):
            N, dt, B, over, w, ranges, geom = screen_fuzz_case(seed, case)
            out[f"fuzz_{seed}_{case}"] = dict(N=N, dt=dt, **count(N, w, hs_of(w["x0"], ranges, geom), dt=dt, **over))
    for name in ("c3_gap_n20", "stiff_gap_n33_dt005", "stiff_gap_n48_dt005"):
        d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
        over = json.loads(str(d["params"])) if "params" in d.files else {}
        w = {k: d[k] for k in ("x0", "u_lin", "x_ref")}
        out[name] = count(int(d["horizon"]), w, d["halfspace"], **over)
    w = workload.make_batch(4096, 20, seed=1000)
    ranges, *geom = workload.make_scans(4096, seed=2000)
    out["c3_bench_batch"] = count(20, w, hs_of(w["x0"], ranges, geom))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
