"""FindHalfSpaces gap search: the closed form the device kernel evaluates in parallel
(tests/halfspace_cases.py::closed_form) equals the reference's sequential state machine
(oracle/f110_oracle.c, constraints.cpp:116-177) on adversarial scans. CPU only."""
import numpy as np
import pytest
from halfspace_cases import adversarial_scans, closed_form, scan_geometry


@pytest.mark.parametrize("nr,seed", [(1080, 1), (1081, 2), (200, 3), (64, 4), (130, 5)])
def test_closed_form_matches_reference_machine(oracle, nr, seed):
    amin, ainc, amax = scan_geometry(nr)
    r = adversarial_scans(96, nr, seed)
    state = np.array([1.0, -2.0, 0.3])
    buffer = np.float32(3.0)
    for b in range(r.shape[0]):
        lo, hi = closed_form(r[b], amin, ainc, amax)
        # the reference's buffer shrink (constraints.cpp:173-177)
        if np.float32(hi - lo) > np.float32(2.0) * buffer:
            hi, lo = int(np.float32(hi) - buffer), int(np.float32(lo) + buffer)
        _, _, _, rlo, rhi = oracle.find_half_spaces(state, r[b], amin, ainc, amax)
        assert (lo, hi) == (rlo, rhi), (b, b % 8)
