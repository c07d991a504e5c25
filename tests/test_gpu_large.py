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


@pytest.mark.parametrize("bits,ch", [(8, 2), (8, 1), (4, 2), (6, 1)])
def test_auto_plan_short_warmup(built, bits, ch):
    """The automatic plan on a ragged stream with a cut last block and a
    2-eblock warm-up, so many chunks need repair: each wave of the decode
    kernel repairs its own chunks, inside the wave and at the boundary with
    the wave before it (its exit record)."""
    eb = 2_500_003
    frames = eb * 32 - 7
    xa = synth.stream(eb, bits, ch, "A", seed=5)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, (1, -2, 3, -4), frames)
    got, st = dev_decode(xa, eb, bits, ch, frames=frames, state=(1, -2, 3, -4),
                         warmup=2, want_status=True)
    assert np.array_equal(got, ref)
    assert st[3] > 0
    assert status_state(st)[:2 * ch] == st_ref[:2 * ch]


@pytest.mark.parametrize("bits,ch", [(8, 2), (6, 1)])
def test_auto_plan_ragged(built, bits, ch):
    """The automatic (uniform) plan on the same ragged stream."""
    eb = 2_500_003
    frames = eb * 32 - 7
    xa = synth.stream(eb, bits, ch, "A", seed=6)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, (5, 6, -7, 8), frames)
    got, st = dev_decode(xa, eb, bits, ch, frames=frames, state=(5, 6, -7, 8),
                         want_status=True)
    assert np.array_equal(got, ref)
    q = 8 // ch                       # chunk quantum, eblocks (XA_CHUNK_Q)
    c = -(-(-(-eb // 131072)) // q) * q
    assert st[6] == c and st[5] == -(-eb // c)
    assert status_state(st)[:2 * ch] == st_ref[:2 * ch]

