"""Per-phase cycle breakdown of the planning kernel from the -DF110QP_STAMPS build.
Run:  F110QP_LIB=f110-mpc_amd/lib_stamps/libf110qp.so python tools/plan_stamps.py [B]
The scenes are bench.py's `tick` workload (workload.make_scenes). Cycles are per workgroup
(s_memtime on thread 0, cumulative from kernel entry)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
from f110qp import capi, workload  # noqa: E402

L = capi.load()
assert hasattr(L, "f110qp_read_plan_stamps"), "not a stamps build"
dev = torch.device("cuda", 0)
sc = workload.make_scenes(B, seed=3000)
cfg = capi.default_plan_config()
tab = torch.from_numpy(capi.traj_table(cfg)).to(dev)
pose = torch.from_numpy(sc["pose"]).to(dev)
rng = torch.from_numpy(sc["ranges"]).to(dev)
wp = torch.from_numpy(np.ascontiguousarray(sc["waypoints"][:, :2])).to(dev)
P = cfg.traj_discrete
xr = torch.empty((B, P, 3), dtype=torch.float32, device=dev)
x0 = torch.empty((B, 3), dtype=torch.float32, device=dev)
bt, bg, st = (torch.empty(B, dtype=torch.int32, device=dev) for _ in range(3))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for _ in range(5):
    ev[0].record()
    capi.plan_batch_dev(cfg, pose, rng, sc["angle_min"], sc["angle_inc"], sc["angle_max"], tab, wp, xr, x0, bt, bg,
                        st)
    ev[1].record()
torch.cuda.synchronize()
n = min(B, 4096)
buf = np.zeros((n, 8), np.uint64)
L.f110qp_read_plan_stamps.argtypes = [C.c_void_p, C.c_int]
L.f110qp_read_plan_stamps(C.c_void_p(buf.ctypes.data), n)
b = buf.astype(float)
print(f"B={B} W={wp.shape[0]} beams={rng.shape[1]} kernel {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us (event, last launch)")
names = ["clear grid / flags", "fill grid (beams x dilation)", "collision check", "waypoint pass 1",
         "waypoint passes 2-3", "end-point selection", "outputs"]
prev = np.zeros(n)
for i, nm in enumerate(names):
    d = b[:, i] - prev
    prev = b[:, i]
    print(f"{nm:30s} mean {d.mean():9.0f}  max {d.max():9.0f}  (cum mean {b[:, i].mean():9.0f})")
