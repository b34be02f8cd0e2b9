"""Per-QP status / iteration difference of the bench's C3 batch between two builds of the library
(F110QP_LIB selects one per process): run once per build, then compare the two .npz files.
Test infrastructure for A/B runs. usage: python tools/c3_status_diff.py out.npz  |  --cmp a.npz b.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    d = np.nonzero((a["st"] != b["st"]) | (np.abs(a["it"] - b["it"]) > 3))[0]
    print("QPs differing:", len(d))
    for i in d[:20]:
        print(i, "st", a["st"][i], b["st"][i], "it", a["it"][i], b["it"][i],
              "du", float(np.abs(a["u"][i] - b["u"][i]).max()))
    sys.exit(0)

import torch  # noqa: E402
from f110qp import capi, workload  # noqa: E402

B, N = 4096, 20
dev = torch.device("cuda", 0)
w = workload.make_batch(B, N, seed=1000)
ranges, amin, ainc, amax = workload.make_scans(B, seed=2000)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
x0, ul, xr, rng = T(w["x0"]), T(w["u_lin"]), T(w["x_ref"]), T(ranges)
hs = torch.empty((B, 2, 3), dtype=torch.float32, device=dev)
capi.find_half_spaces_dev(x0, rng, amin, ainc, amax, hs)
s = capi.Solver(capi.default_config(N, gap_mode=capi.GAP_ACTIVE))
uo = torch.empty((B, N, 2), dtype=torch.float32, device=dev)
xo = torch.empty((B, N + 1, 3), dtype=torch.float32, device=dev)
st = torch.empty((B,), dtype=torch.int32, device=dev)
it = torch.empty((B,), dtype=torch.int32, device=dev)
s.solve_dev(x0, ul, xr, hs, uo, xo, st, it)
torch.cuda.synchronize()
np.savez(sys.argv[1], st=st.cpu().numpy(), it=it.cpu().numpy(), u=uo.cpu().numpy())
print("saved", sys.argv[1], np.bincount(st.cpu().numpy()))
