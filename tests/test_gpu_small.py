"""The host API's GPU paths for small calls (<= 32 eblocks per
bjxa_decode/bjxa_encode, bjxa_amd/csrc/xa_small.hip, reached with the
offload threshold at 0) and the bulk path, and the default routing that
sends calls below the offload threshold to the CPU core and larger ones to
the GPU: every format, call sizes on both sides of each threshold, state
carried across calls, the reference's error semantics."""
import errno

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth

pytestmark = pytest.mark.gpu

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)]


@pytest.mark.parametrize("bits,ch", FORMATS)
def test_small_calls_chain(built, bits, ch):
    """A stream decoded through calls of 1..40 eblocks (small and bulk path
    interleaved) equals the single-pass oracle, incl. bef state and a cut
    last block."""
    rng = np.random.default_rng(bits * 10 + ch)
    eb = 700
    frames = eb * 32 - 11
    state = (1234, -2345, -3456, 4567)
    xa = synth.stream(eb, bits, ch, "A", seed=bits + ch)
    hdr = bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state)
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    bx = (bits * 4 + 1) * ch
    out = bytearray()
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        pos, left = 0, frames * ch * 2
        while pos < eb:
            n = min(int(rng.integers(1, 41)), eb - pos)
            dst = np.zeros(n * 64 * ch, np.uint8)
            assert d.decode(dst, xa[pos * bx:(pos + n) * bx].copy()) == n
            take = min(n * 64 * ch, left)
            out += dst[:take].tobytes()
            left -= take
            pos += n
    assert bytes(out) == ref.tobytes()


@pytest.mark.parametrize("n", [1, 2, 17, 32])
@pytest.mark.parametrize("ch,bad", [(1, 0), (2, 0), (2, 1)])
def test_small_call_invalid_profile(built, n, ch, bad):
    """EPROTO inside a small call: earlier eblocks are returned, and the
    carried state is the reference's partial update (a bad right block has
    advanced the left channel), as on the bulk path."""
    j = n - 1
    xa = synth.stream(n, 6, ch, "A", seed=n + ch).reshape(n * ch, 25)
    xa[j * ch + bad, 0] = 0x5F
    hdr = bjxa_amd.xa_header(xa.size, n * 32, 44100, 6, ch)
    ref, st_ref, done, badc = oracle.decode(xa.reshape(-1), n, 6, ch)
    assert done == j and badc == bad
    fixed = xa.copy()
    fixed[j * ch + bad, 0] = 0x00
    ref2, _, _, _ = oracle.decode(fixed.reshape(-1)[j * ch * 25:], 1, 6, ch, st_ref)
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        dst = np.full(n * 64 * ch, 0x11, np.uint8)
        with pytest.raises(bjxa_amd.BjxaError) as ei:
            d.decode(dst, xa.reshape(-1).copy())
        assert ei.value.errno == errno.EPROTO
        assert np.array_equal(dst[:j * 64 * ch].view(np.int16), ref[:j * 32 * ch])
        assert (dst[j * 64 * ch:] == 0x11).all()
        dst2 = np.zeros(64 * ch, np.uint8)
        assert d.decode(dst2, fixed.reshape(-1)[j * ch * 25:].copy()) == 1
        assert np.array_equal(dst2.view(np.int16), ref2)


@pytest.mark.parametrize("bits,ch", FORMATS)
def test_small_encode_calls(built, bits, ch):
    """Encode through calls of 1..40 blocks equals the single-pass oracle."""
    rng = np.random.default_rng(100 + bits * 10 + ch)
    frames = 32 * 300 + 9
    pcm = synth.pcm(frames, ch, seed=bits + ch)
    e = bjxa_amd.Encoder()
    fmt = e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                  "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                  "channels": ch}, bits)
    raw = pcm.tobytes()
    bp, bx = fmt["block_size_pcm"], fmt["block_size_xa"]
    out, pos = bytearray(), 0
    while pos < fmt["blocks"]:
        n = min(int(rng.integers(1, 41)), fmt["blocks"] - pos)
        chunk = np.frombuffer(raw[pos * bp:(pos + n) * bp].ljust(n * bp, b"\0"),
                              np.uint8).copy()
        dst = np.zeros(n * bx, np.uint8)
        assert e.encode(dst, chunk) == n
        out += dst.tobytes()
        pos += n
    e.close()
    assert bytes(out) == oracle.encode(pcm, frames, bits, ch).tobytes()


@pytest.mark.routing
@pytest.mark.parametrize("bits,ch", FORMATS)
def test_default_routing_chain(built, bits, ch):
    """Default routing: calls below the decode offload threshold run on the
    CPU core, larger ones on the GPU, through one decoder; the chained
    output equals the single-pass oracle (state handed back and forth)."""
    thr = bjxa_amd.offload_threshold(bjxa_amd.OFFLOAD_DECODE)
    assert 0 < thr < 1 << 20
    rng = np.random.default_rng(300 + bits * 10 + ch)
    sizes = [int(v) for v in rng.integers(1, 3 * thr, 24)] + [1, 2, thr - 1, thr]
    eb = sum(sizes)
    frames = eb * 32 - 5
    state = (-1, 2, -3, 4)
    xa = synth.stream(eb, bits, ch, "W", seed=bits * 3 + ch)
    hdr = bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state)
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    bx = (bits * 4 + 1) * ch
    out = bytearray()
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        pos, left = 0, frames * ch * 2
        for n in sizes:
            dst = np.zeros(n * 64 * ch, np.uint8)
            assert d.decode(dst, xa[pos * bx:(pos + n) * bx].copy()) == n
            take = min(n * 64 * ch, left)
            out += dst[:take].tobytes()
            left -= take
            pos += n
    assert bytes(out) == ref.tobytes()


@pytest.mark.routing
@pytest.mark.parametrize("bits,ch", FORMATS)
def test_default_routing_encode(built, bits, ch):
    """Encode calls on both sides of the encode offload threshold."""
    thr = bjxa_amd.offload_threshold(bjxa_amd.OFFLOAD_ENCODE)
    rng = np.random.default_rng(400 + bits * 10 + ch)
    sizes = [int(v) for v in rng.integers(1, 2 * thr, 10)] + [thr - 1, thr]
    blocks = sum(sizes)
    frames = blocks * 32 - 3
    pcm = synth.pcm(frames, ch, seed=bits + 5 * ch)
    e = bjxa_amd.Encoder()
    fmt = e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                  "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                  "channels": ch}, bits)
    raw = pcm.tobytes()
    bp, bx = fmt["block_size_pcm"], fmt["block_size_xa"]
    out, pos = bytearray(), 0
    for n in sizes:
        chunk = np.frombuffer(raw[pos * bp:(pos + n) * bp].ljust(n * bp, b"\0"),
                              np.uint8).copy()
        dst = np.zeros(n * bx, np.uint8)
        assert e.encode(dst, chunk) == n
        out += dst.tobytes()
        pos += n
    e.close()
    assert bytes(out) == oracle.encode(pcm, frames, bits, ch).tobytes()
