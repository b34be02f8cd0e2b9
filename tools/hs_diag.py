"""Which cos/sin does the device FindHalfSpaces kernel match bit for bit? Emulates the reference
geometry (constraints.cpp:179-264) in numpy with fp64 cos/sin and with fp32 cos/sin and counts
bit-equal rows against the device on the adversarial scans."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f110-mpc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from f110qp import capi  # noqa: E402
from halfspace_cases import adversarial_scans, scan_geometry  # noqa: E402

f = np.float32
nr, B = 1080, 512
amin, ainc, amax = scan_geometry(nr)
r = adversarial_scans(B, nr, 11)
rng = np.random.default_rng(11)
st = np.column_stack([rng.uniform(-30, 30, B), rng.uniform(-30, 30, B), rng.uniform(-3, 3, B)]).astype(np.float32)
dev = torch.device("cuda", 0)
hs = torch.empty((B, 2, 3), dtype=torch.float32, device=dev)
lo = torch.empty(B, dtype=torch.int32, device=dev)
hi = torch.empty(B, dtype=torch.int32, device=dev)
capi.find_half_spaces_dev(torch.from_numpy(st).to(dev), torch.from_numpy(r).to(dev), amin, ainc, amax, hs, lo, hi)
torch.cuda.synchronize()
hs, lo, hi = hs.cpu().numpy(), lo.cpu().numpy(), hi.cpu().numpy()


def emulate(b, trig):
    l, h = int(lo[b]), int(hi[b])
    a1 = f(f(amin + f(f(l) * ainc)) + st[b, 2])
    a2 = f(f(amin + f(f(h) * ainc)) + st[b, 2])
    c1, s1, c2, s2 = trig(a1), trig(a2, sin=True), trig(a2), trig(a1, sin=True)
    X, Y = np.float64(st[b, 0]), np.float64(st[b, 1])
    p1x = f(np.float64(r[b, l]) * c1 + X); p1y = f(np.float64(r[b, l]) * s2 + Y)
    p2x = f(np.float64(r[b, h]) * c2 + X); p2y = f(np.float64(r[b, h]) * s1 + Y)
    return p1x, p1y, p2x, p2y


def t64(a, sin=False):
    return np.sin(np.float64(a)) if sin else np.cos(np.float64(a))


def t32(a, sin=False):
    return np.float64(np.sin(f(a)) if sin else np.cos(f(a)))


ok = (lo >= 0) & (hi >= 0) & (lo < nr) & (hi < nr)
for name, trig in (("fp64 cos/sin", t64), ("fp32 cos/sin", t32)):
    eq = tot = 0
    for b in np.nonzero(ok)[0]:
        p1x, p1y, p2x, p2y = emulate(b, trig)
        if not np.isfinite([p1x, p1y, p2x, p2y]).all():
            continue
        px, py = f(st[b, 0]), f(st[b, 1])
        a1, b1 = f(py - p1y), f(p1x - px)
        tot += 1
        eq += int(abs(hs[b, 0, 0]) == abs(a1) and abs(hs[b, 0, 1]) == abs(b1))
    print(f"{name}: a1/b1 bit-equal on {eq}/{tot} scans")
shown = 0
for b in np.nonzero(ok)[0]:
    p1x, p1y, p2x, p2y = emulate(b, t64)
    if not np.isfinite([p1x, p1y, p2x, p2y]).all():
        continue
    px, py = f(st[b, 0]), f(st[b, 1])
    a1, b1 = f(py - p1y), f(p1x - px)
    if not (abs(hs[b, 0, 0]) == abs(a1) and abs(hs[b, 0, 1]) == abs(b1)) and shown < 6:
        shown += 1
        print(b, b % 8, int(lo[b]), int(hi[b]), "dev", hs[b, 0], "emu a1 b1", a1, b1, "p1", p1x, p1y, "r", r[b, lo[b]], r[b, hi[b]])
