"""BASELINE.json configs C2/C3 at full size, bit-exact against the oracle
(which needs ~2 s single-threaded), plus size-independent properties."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, status_state

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_full_size_bit_exact(built, cfg):
    eb, ch = (10_000_000, 1) if cfg == "C2" else (5_000_000, 2)
    xa = synth.stream(eb, 8, ch, "A", seed=0)
    ref, st_ref, _, _ = oracle.decode(xa, eb, 8, ch)
    got, st = dev_decode(xa, eb, 8, ch, want_status=True)
    assert np.array_equal(got, ref)
    assert status_state(st)[:2 * ch] == st_ref[:2 * ch]


def test_worst_case_mix_full_size(built):
    """Profile mix W (gain 4 only: slowest resync) on C3."""
    eb = 5_000_000
    xa = synth.stream(eb, 8, 2, "W", seed=1)
    ref, _, _, _ = oracle.decode(xa, eb, 8, 2)
    got, st = dev_decode(xa, eb, 8, 2, want_status=True)
    assert np.array_equal(got, ref)
    assert st[3] > 0      # the repair pass did real work on this mix
