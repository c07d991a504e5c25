"""GPU encode parity: byte-exact XA against the oracle, the round-trip
identity that pins the reference's encode, and the survey's
encoder SHA-1s as a regression check."""
import hashlib

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, dev_encode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("wav", ["square-mono.wav", "square-stereo.wav"])
@pytest.mark.parametrize("bits", [4, 6, 8])
def test_encode_fixture_sha1(built, wav, bits, manifest, golden):
    """`bjxa encode --bits N` output, through the drop-in C API."""
    xa = bjxa_amd.encode_wav(golden(wav), bits)
    assert hashlib.sha1(xa).hexdigest() == manifest["encode"][wav][str(bits)]


@pytest.mark.parametrize("bits", [4, 6, 8])
@pytest.mark.parametrize("ch", [1, 2])
@pytest.mark.parametrize("frames", [1, 31, 32, 33, 127, 128, 129, 100003])
def test_encode_random(built, bits, ch, frames):
    pcm = synth.pcm(frames, ch, seed=frames + bits)
    assert np.array_equal(dev_encode(pcm, frames, bits, ch), oracle.encode(pcm, frames, bits, ch))


@pytest.mark.parametrize("bits", [4, 6, 8])
@pytest.mark.parametrize("ch", [1, 2])
def test_round_trip(built, bits, ch):
    """The reference's encode pins itself: every profile byte is 0
    (src/libbjxa.c:679) and each code is the top `bits` bits of its sample
    (:349-391), so decode(encode(x)) == x with the low 16-bits bits cleared,
    exactly -- an identity that fixes every code byte."""
    frames = 300001
    pcm = synth.pcm(frames, ch, seed=bits + ch)
    xa = dev_encode(pcm, frames, bits, ch)
    eb = (frames + 31) // 32
    assert (xa.reshape(eb * ch, bits * 4 + 1)[:, 0] == 0).all()
    back = dev_decode(xa, eb, bits, ch, frames=frames)
    assert np.array_equal(back, pcm & np.int16(~((1 << (16 - bits)) - 1)))


def test_encode_incremental(built):
    """One bjxa_encode per block, as bjxa(1)'s default loop does
    (src/bjxa_encode.c:108-167)."""
    frames = 32 * 50 + 7
    pcm = synth.pcm(frames, 2, seed=3)
    e = bjxa_amd.Encoder()
    fmt = e.init({"data_len_pcm": frames * 4, "blocks": 0, "block_size_pcm": 0,
                  "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                  "channels": 2}, 4)
    out = bytearray()
    raw = pcm.tobytes()
    pos = 0
    for _ in range(fmt["blocks"]):
        chunk = np.frombuffer(raw[pos:pos + 128].ljust(128, b"\0"), np.uint8).copy()
        dst = np.zeros(fmt["block_size_xa"], np.uint8)
        assert e.encode(dst, chunk) == 1
        out += dst.tobytes()
        pos += 128
    e.close()
    assert bytes(out) == oracle.encode(pcm, frames, 4, 2).tobytes()
