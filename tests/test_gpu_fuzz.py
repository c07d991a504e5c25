"""Seeded fuzz of the device decode against the oracle: random formats,
lengths (1 to ~300k eblocks), cut last blocks, entry states (the
reference's befL/befR, src/libbjxa.c:417-420), profile mixes, and chunk /
warm-up tunings that the host rounds to whole chunk quanta.  Every case is
bit-exact or, for streams with a gain >= 5 profile, exact up to the first
bad channel block with the reference's error position
(src/libbjxa.c:547-550)."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, status_state
from test_gpu_batch import check, run_batch

pytestmark = pytest.mark.gpu

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)]


def case(rng, i):
    bits, ch = FORMATS[int(rng.integers(0, 6))]
    eb = int(np.exp(rng.uniform(0, np.log(300_000))))
    mix = "AFWZ"[int(rng.integers(0, 4))]
    xa = synth.stream(eb, bits, ch, mix, seed=5000 + i)
    if rng.random() < 0.15:
        # one protocol error somewhere (gain nibble 5..15)
        k = int(rng.integers(0, eb * ch))
        xa[k * (bits * 4 + 1)] = int(rng.integers(0x50, 0x100))
    cut = int(rng.integers(0, 32)) if rng.random() < 0.5 else 0
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4))
    return xa, eb, bits, ch, eb * 32 - cut, state


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_single_stream(built, seed):
    rng = np.random.default_rng(100 + seed)
    for i in range(12):
        xa, eb, bits, ch, frames, state = case(rng, seed * 100 + i)
        chunk = int(rng.choice([0, 0, 1, 5, 12, 33, 64]))
        warm = int(rng.choice([-1, -1, 0, 3, 8, 17]))
        pcm, st = dev_decode(xa, eb, bits, ch, frames=frames, state=state,
                             chunk=chunk, warmup=warm, want_status=True)
        ref, st_ref, done, bad = oracle.decode(xa, eb, bits, ch, state, frames)
        what = (seed, i, bits, ch, eb, frames, chunk, warm)
        if bad < 0:
            assert st[0] == bjxa_amd.NO_ERROR, what
            assert np.array_equal(pcm, ref), what
            assert status_state(st)[:2 * ch] == st_ref[:2 * ch], what
        else:
            assert st[0] == done * ch + bad, what
            n = done * 32 * ch
            assert np.array_equal(pcm[:n], ref[:n]), what


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_batch(built, seed):
    rng = np.random.default_rng(200 + seed)
    specs = [case(rng, 1000 + seed * 100 + i) for i in range(int(rng.integers(1, 40)))]
    chunk = int(rng.choice([0, 0, 7, 40]))
    warm = int(rng.choice([-1, 0, 5, 12]))
    pcms, st = run_batch(specs, chunk=chunk, warmup=warm)
    check(specs, pcms, st)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_host_api(built, seed):
    """The unchanged bjxa_decode() on host buffers with random call sizes
    (small-call path and bulk path, src/libbjxa.c:602-661 per call), the
    state carried across calls, against one single-pass oracle decode."""
    rng = np.random.default_rng(300 + seed)
    bits, ch = FORMATS[seed % 6]
    eb = int(rng.integers(1, 60_000))
    frames = eb * 32 - int(rng.integers(0, 32))
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4))
    xa = synth.stream(eb, bits, ch, "AFWZ"[seed % 4], seed=7000 + seed)
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    bx = (bits * 4 + 1) * ch
    out = bytearray()
    with bjxa_amd.Decoder() as d:
        d.parse_header(bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state))
        pos, left = 0, frames * ch * 2
        while pos < eb:
            n = min(int(np.exp(rng.uniform(0, np.log(20_000)))), eb - pos)
            dst = np.zeros(n * 64 * ch, np.uint8)
            assert d.decode(dst, xa[pos * bx:(pos + n) * bx].copy()) == n
            take = min(n * 64 * ch, left)
            out += dst[:take].tobytes()
            left -= take
            pos += n
    assert bytes(out) == ref.tobytes()


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_encode(built, seed):
    """Device encode of random PCM lengths in every format against the
    oracle's restatement of bjxa_encode (src/libbjxa.c:759-819)."""
    from gpu_util import dev_encode
    rng = np.random.default_rng(400 + seed)
    for i in range(6):
        bits, ch = FORMATS[int(rng.integers(0, 6))]
        frames = int(np.exp(rng.uniform(0, np.log(2_000_000))))
        pcm = synth.pcm(frames, ch, seed=seed * 10 + i)
        assert np.array_equal(dev_encode(pcm, frames, bits, ch),
                              oracle.encode(pcm, frames, bits, ch)), (seed, i, bits, ch, frames)
