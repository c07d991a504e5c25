"""The region kernel (K1r, bjxa_amd/csrc/xa_region.hip, opt-in through
VARIANT_REGION): contiguous per-wave regions, warm-up from the neighbour's
chunk in LDS, in-wave verification and repair, K2 over region boundaries.
Bit-exact against the oracle in every format, with ragged lengths, cut
last blocks, a caller state, bad profiles and the worst-case mix."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, status_state

pytestmark = pytest.mark.gpu

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)]


@pytest.mark.parametrize("bits,ch", FORMATS)
@pytest.mark.parametrize("mix", ["A", "W", "F"])
def test_region_random(built, bits, ch, mix):
    eb = 300_007 if ch == 2 else 500_009
    frames = eb * 32 - 5
    state = (3, -9, 12, -1)
    xa = synth.stream(eb, bits, ch, mix, seed=17)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    got, st = dev_decode(xa, eb, bits, ch, frames=frames, state=state, want_status=True,
                         variant=bjxa_amd.VARIANT_REGION)
    assert np.array_equal(got, ref)
    assert status_state(st)[:2 * ch] == st_ref[:2 * ch]
    assert st[6] == (8 if ch == 2 else 16) and st[7] == 8


@pytest.mark.parametrize("eb", [1, 7, 64 * 8 - 1, 64 * 8 + 1, 3 * 512 + 13])
def test_region_small_and_edges(built, eb):
    """One partial region, exact region multiples +-1 (stereo 512 eblocks
    per region)."""
    xa = synth.stream(eb, 8, 2, "A", seed=eb)
    ref, _, _, _ = oracle.decode(xa, eb, 8, 2)
    assert np.array_equal(dev_decode(xa, eb, 8, 2, variant=bjxa_amd.VARIANT_REGION), ref)


@pytest.mark.parametrize("at,chan", [(0, 0), (511, 1), (512, 0), (100_000, 1)])
def test_region_bad_profile(built, at, chan):
    eb = 200_000
    xa = synth.stream(eb, 8, 2, "A", seed=5)
    xa[(at * 2 + chan) * 33] = 0x5D
    ref, st_ref, done, badc = oracle.decode(xa, eb, 8, 2)
    got, st = dev_decode(xa, eb, 8, 2, want_status=True, variant=bjxa_amd.VARIANT_REGION)
    assert int(st[0]) == at * 2 + chan and (done, badc) == (at, chan)
    n = done * 64
    assert np.array_equal(got[:n], ref[:n])
