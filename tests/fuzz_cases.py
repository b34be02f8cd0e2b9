"""The screen-size fuzz cases of tests/test_gpu_screen.py::test_screen_fuzz_configs_against_oracle
(AUTO gap calls of 1,024..1,600 QPs over random corners of the ABI's parameter space), generated
in one place for the test, tools/screen_case_probe.py and tests/golden/make_golden.py (the
stiff-corner fixtures). Test infrastructure."""
import numpy as np

from f110qp import workload


def screen_fuzz_case(seed: int, case: int):
    """(N, dt, B, over, w, ranges, (amin, ainc, amax)) of case `case` of seed `seed`; over holds
    the f110qp_config / oracle.params overrides (q, r, u_des, u_min, u_max)."""
    rng = np.random.default_rng(7100 + seed)
    for c in range(case + 1):
        N = int(rng.choice([5, 13, 20, 27, 33, 40, 48]))
        lo0, lo1 = float(rng.uniform(1.0, 3.5)), float(rng.uniform(-0.6, -0.1))
        hi0, hi1 = lo0 + float(rng.uniform(0.3, 2.0)), -lo1 * float(rng.uniform(0.5, 1.5))
        ud = [float(rng.choice([hi0, lo0, 0.5 * (lo0 + hi0)])), float(rng.choice([0.0, hi1, lo1]))]
        q01 = float(rng.choice([0.0, 1.0, 10.0, 40.0]))
        over = dict(q=[q01, q01 if rng.random() < 0.5 else float(rng.uniform(0.5, 20.0)),
                       float(rng.choice([0.0, 0.5, 3.0]))],
                    r=[float(rng.uniform(0.05, 2.0)), float(rng.uniform(0.5, 10.0))], u_des=ud,
                    u_min=[lo0, lo1], u_max=[hi0, hi1])
        dt = float(np.float32(rng.choice([0.005, 0.01, 0.02, 0.05])))
        B = int(rng.integers(1024, 1600))
        w = workload.make_batch(B, N, seed=int(rng.integers(1 << 30)), heading="true",
                                lateral=float(rng.uniform(0.0, 1.5)), steer_range=float(rng.uniform(0.0, 0.8)))
        ranges, amin, ainc, amax = workload.make_scans(B, seed=int(rng.integers(1 << 30)))
        if c == case:
            return N, dt, B, over, w, ranges, (amin, ainc, amax)
