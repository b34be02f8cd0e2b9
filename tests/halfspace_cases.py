"""Adversarial LaserScans for FindHalfSpaces (reference src/constraints.cpp:116-177): many short
runs, single-beam gaps (never recorded: the stale `hi`), equal longest runs (the first wins), runs
across the kernel's 64-beam blocks, windows that open on a short or a long beam, all-open and
all-closed scans, NaN / inf / exactly-threshold ranges. Shared by the CPU closed-form check and the
GPU kernel parity test."""
import numpy as np


def scan_geometry(nr):
    """angle_min/inc/max of an nr-beam 270-degree scan (float32, as sensor_msgs/LaserScan)."""
    amin = np.float32(-2.35619449)
    ainc = np.float32(4.71238898 / (nr - 1))
    amax = np.float32(amin + ainc * np.float32(nr - 1))
    return amin, ainc, amax


def adversarial_scans(B, nr, seed):
    rng = np.random.default_rng(seed)
    r = np.empty((B, nr), np.float32)
    for b in range(B):
        kind = b % 8
        if kind == 0:    # Bernoulli open flags: many short runs and ties
            o = rng.random(nr) < rng.choice([0.3, 0.5, 0.7, 0.85])
        elif kind == 1:  # single-beam gaps only
            o = np.zeros(nr, bool)
            o[rng.integers(0, 2) :: 2] = True
        elif kind == 2:  # two equal longest runs, plus shorter ones
            o = np.zeros(nr, bool)
            L = int(rng.integers(2, max(3, min(40, nr // 10))))
            cand = np.arange(0, nr - L, L + 2)
            starts = np.sort(rng.choice(cand, min(4, len(cand)), replace=False))
            for i, s in enumerate(starts):
                o[s : s + (L if i < 2 else int(rng.integers(1, L)))] = True
        elif kind == 3:  # long runs crossing 64-beam block boundaries
            o = np.zeros(nr, bool)
            for s in range(int(rng.integers(40, 70)), nr, 150):
                o[s : s + int(rng.integers(60, 140))] = True
        elif kind == 4:  # all open / all closed
            o = np.full(nr, bool(rng.integers(0, 2)))
        elif kind == 5:  # sparse: at most one run of length >= 2 somewhere
            o = rng.random(nr) < 0.05
        else:            # smooth arcs (realistic) with noise
            o = rng.random(nr) < 0.1
            c = int(rng.integers(0, nr))
            o[max(0, c - 80) : c + 80] = rng.random(min(nr, c + 80) - max(0, c - 80)) < 0.95
        v = np.where(o, rng.uniform(3.0001, 9.0, nr), rng.uniform(0.2, 3.0, nr)).astype(np.float32)
        # edge values: exactly the threshold (not open), NaN (not open), +inf (open)
        m = rng.random(nr)
        v[(m < 0.01) & ~o] = np.float32(3.0)
        v[(m > 0.995) & ~o] = np.nan
        v[(m > 0.995) & o] = np.inf
        r[b] = v
    return r


def closed_form(ranges, amin, ainc, amax, thresh=3.0, divider=1.5):
    """The run characterisation the device kernel implements (halfspace_kernels.hip header):
    first longest run of >= 2 open in-window beams -> (start, end); else (-1, -1) when the
    window's first beam is closed; else (0, 0). Before the buffer shrink."""
    nr = ranges.shape[0]
    f = np.float32
    num = int(f(f(f(amax) - f(amin)) / f(ainc)) + f(1.0))
    num = min(num, nr)
    lim = f(f(1.571) / f(divider))
    best, blo, bhi = 0, None, None
    w0 = None
    start = None
    for p in range(num):
        ang = f(f(amin) + f(f(p) * f(ainc)))
        if not (ang > -lim and ang < lim):
            start = None
            continue
        op = bool(ranges[p] > f(thresh))
        if w0 is None:
            w0 = (p, op)
        if op:
            if start is None:
                start = p
            elif p - start > best:
                best, blo, bhi = p - start, start, p
        else:
            start = None
    if blo is not None:
        return blo, bhi
    if w0 is not None and not w0[1]:
        return -1, -1
    return 0, 0
