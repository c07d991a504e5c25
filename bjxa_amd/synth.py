"""Synthetic XA stream generator for benchmarks and parity tests.

Streams are raw XA block data (no header): `eblocks` effective blocks, each
`channels` channel blocks of `bits*4+1` bytes (profile byte, then packed
codes), the layout bjxa_decode consumes (src/libbjxa.c:629-646).

Reference-encoder output always carries profile 0 (src/libbjxa.c:679) and so
never exercises the predictor; decode workloads therefore draw profiles from
one of the mixes of SURVEY.md §8(d):

  A  gain uniform 0-4, range uniform 0-12        (default)
  F  fixture-like: gain 0 p=.949, 1 .0066, 2 .0445, 3 .00005; ranges as in
     test/square-*.xa
  W  worst case for speculation: gain 4 only, range 12-15
  Z  all profiles 0 (reference-encoder shape)

Data bytes are uniform.  Everything is a deterministic function of `seed`.
"""
import numpy as np

_F_GAIN = ([0, 1, 2, 3], [0.949, 0.0066, 0.0445, 0.00005])
# range histogram of test/square-mono-*.xa
_F_RANGE = ([0, 1, 2, 3, 4, 6], [8790, 6891, 3447, 487, 137, 920])


def profiles(n, mix, rng):
    if mix == "A":
        g = rng.integers(0, 5, n)
        r = rng.integers(0, 13, n)
    elif mix == "F":
        gv, gp = _F_GAIN
        gp = np.array(gp) / np.sum(gp)
        g = rng.choice(gv, n, p=gp)
        rv, rp = _F_RANGE
        rp = np.array(rp, dtype=np.float64)
        r = rng.choice(rv, n, p=rp / rp.sum())
    elif mix == "W":
        g = np.full(n, 4)
        r = rng.integers(12, 16, n)
    elif mix == "Z":
        g = np.zeros(n, dtype=np.int64)
        r = np.zeros(n, dtype=np.int64)
    else:
        raise ValueError("unknown profile mix %r" % (mix,))
    return ((g << 4) | r).astype(np.uint8)


def stream(eblocks, bits=8, channels=2, mix="A", seed=0):
    """Return a uint8 array of eblocks*channels*(bits*4+1) bytes."""
    bsz = bits * 4 + 1
    n = eblocks * channels
    rng = np.random.Generator(np.random.PCG64(0xB1A5000000000000 + seed))
    buf = rng.integers(0, 256, n * bsz, dtype=np.uint8)
    buf.reshape(n, bsz)[:, 0] = profiles(n, mix, rng)
    return buf


def pcm(frames, channels=2, seed=0):
    """Uniform int16 PCM (encode workloads)."""
    rng = np.random.Generator(np.random.PCG64(0xB1A5100000000000 + seed))
    return rng.integers(-32768, 32768, frames * channels, dtype=np.int16)
