"""The library's CPU core (bjxa_amd/csrc/xa_cpu.c) through the unchanged
bjxa_decode()/bjxa_encode() host API, against the oracle: every format,
profile mixes including clamp-heavy and worst-case, entry state, cut last
blocks, calls of random sizes chained through one decoder (the reference
CLI's incremental shape, src/bjxa_decode.c:102-155), and the reference's
EPROTO semantics (src/libbjxa.c:547-550, :633-646).  Routing is pinned to
the CPU (offload threshold at its maximum), so these run without a GPU."""
import errno

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)]


@pytest.fixture(autouse=True)
def cpu_only(built):
    with bjxa_amd.offload(None):
        yield


def chained_decode(xa, eb, bits, ch, frames, state, sizes):
    hdr = bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state)
    bx = (bits * 4 + 1) * ch
    out = bytearray()
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        pos, left = 0, frames * ch * 2
        for n in sizes:
            if pos >= eb:
                break
            n = min(n, eb - pos)
            dst = np.zeros(n * 64 * ch, np.uint8)
            assert d.decode(dst, xa[pos * bx:(pos + n) * bx].copy()) == n
            take = min(n * 64 * ch, left)
            out += dst[:take].tobytes()
            left -= take
            pos += n
        assert pos == eb
        with pytest.raises(bjxa_amd.BjxaError) as ei:
            d.decode(np.zeros(64 * ch, np.uint8), np.zeros(bx, np.uint8))
        assert ei.value.errno == errno.EPROTO       # past the end
    return bytes(out)


@pytest.mark.parametrize("bits,ch", FORMATS)
@pytest.mark.parametrize("mix", ["A", "W", "F"])
def test_chained_calls(bits, ch, mix):
    rng = np.random.default_rng(bits * 100 + ch * 10 + ord(mix))
    eb = 3000
    frames = eb * 32 - int(rng.integers(0, 32))
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4))
    xa = synth.stream(eb, bits, ch, mix, seed=bits * 7 + ch)
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    sizes = [int(v) for v in rng.integers(1, 300, 200)] + [eb]
    assert chained_decode(xa, eb, bits, ch, frames, state, sizes) == ref.tobytes()
    # one call per block, and one call for the whole stream
    assert chained_decode(xa, eb, bits, ch, frames, state, [1] * eb) == ref.tobytes()
    assert chained_decode(xa, eb, bits, ch, frames, state, [eb]) == ref.tobytes()


@pytest.mark.parametrize("bits,ch", FORMATS)
def test_clamp_heavy(bits, ch):
    """Range 0 with extreme codes and gain 4 drive both int16 bounds."""
    rng = np.random.default_rng(5)
    eb = 2000
    xa = synth.stream(eb, bits, ch, "A", seed=3).reshape(eb * ch, bits * 4 + 1)
    xa[:, 0] = (4 << 4) | rng.integers(0, 2, eb * ch)
    xa[:, 1:] = rng.choice([0x00, 0x7F, 0x80, 0xFF, 0x77, 0x88], xa[:, 1:].shape)
    xa = xa.reshape(-1)
    ref, st, _, _ = oracle.decode(xa, eb, bits, ch)
    assert (ref == 32767).any() and (ref == -32768).any()
    assert chained_decode(xa, eb, bits, ch, eb * 32, (0, 0, 0, 0), [eb]) == ref.tobytes()


@pytest.mark.parametrize("n", [1, 2, 17, 500])
@pytest.mark.parametrize("ch,bad", [(1, 0), (2, 0), (2, 1)])
def test_invalid_profile(n, ch, bad):
    """EPROTO: earlier eblocks are in dst and counted, nothing of the bad
    eblock is written, and a bad right block has advanced the left channel:
    the retried (fixed) block decodes from that partial state."""
    j = n - 1
    xa = synth.stream(n, 8, ch, "A", seed=n + ch).reshape(n * ch, 33)
    xa[j * ch + bad, 0] = 0x5F + 0x10 * (n % 11 % 10)
    ref, st_ref, done, badc = oracle.decode(xa.reshape(-1), n, 8, ch)
    assert done == j and badc == bad
    # a retry fails again, and a bad right block advances the left channel
    # once more on the way
    _, st_retry, _, _ = oracle.decode(xa.reshape(-1)[j * ch * 33:], 1, 8, ch, st_ref)
    fixed = xa.copy()
    fixed[j * ch + bad, 0] = 0x00
    ref2, _, _, _ = oracle.decode(fixed.reshape(-1)[j * ch * 33:], 1, 8, ch, st_retry)
    with bjxa_amd.Decoder() as d:
        d.parse_header(bjxa_amd.xa_header(xa.size, n * 32, 44100, 8, ch))
        dst = np.full(n * 64 * ch, 0x11, np.uint8)
        with pytest.raises(bjxa_amd.BjxaError) as ei:
            d.decode(dst, xa.reshape(-1).copy())
        assert ei.value.errno == errno.EPROTO
        assert np.array_equal(dst[:j * 64 * ch].view(np.int16), ref[:j * 32 * ch])
        assert (dst[j * 64 * ch:] == 0x11).all()
        with pytest.raises(bjxa_amd.BjxaError):
            d.decode(np.zeros(64 * ch, np.uint8), xa.reshape(-1)[j * ch * 33:].copy())
        dst2 = np.zeros(64 * ch, np.uint8)
        assert d.decode(dst2, fixed.reshape(-1)[j * ch * 33:].copy()) == 1
        assert np.array_equal(dst2.view(np.int16), ref2)


@pytest.mark.parametrize("name", ["square-mono-4.xa", "square-mono-6.xa", "square-mono-8.xa",
                                  "square-stereo-4.xa", "square-stereo-6.xa",
                                  "square-stereo-8.xa"])
def test_fixture_sha1(name, manifest, golden):
    """test/test_decode.sh:24-78 on the CPU core."""
    import hashlib
    wav = bjxa_amd.decode_file(golden(name))
    assert hashlib.sha1(wav).hexdigest() == manifest["fixtures"][name]["wav_sha1"]


def test_saturation_vector(manifest):
    import hashlib
    wav = bjxa_amd.decode_file(bytes.fromhex(manifest["boundary"]["hex"]))
    assert hashlib.sha1(wav).hexdigest() == manifest["boundary"]["wav_sha1"]


@pytest.mark.parametrize("bits,ch", FORMATS)
def test_encode_chained(bits, ch):
    """Encode through calls of random sizes equals the single-pass oracle,
    incl. the zero-padded last block."""
    rng = np.random.default_rng(200 + bits * 10 + ch)
    frames = 32 * 900 + 13
    pcm = synth.pcm(frames, ch, seed=bits + ch)
    e = bjxa_amd.Encoder()
    fmt = e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                  "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                  "channels": ch}, bits)
    raw = pcm.tobytes()
    bp, bx = fmt["block_size_pcm"], fmt["block_size_xa"]
    out, pos = bytearray(), 0
    while pos < fmt["blocks"]:
        n = min(int(rng.integers(1, 200)), fmt["blocks"] - pos)
        chunk = np.frombuffer(raw[pos * bp:(pos + n) * bp].ljust(n * bp, b"\0"),
                              np.uint8).copy()
        dst = np.zeros(n * bx, np.uint8)
        assert e.encode(dst, chunk) == n
        out += dst.tobytes()
        pos += n
    e.close()
    assert bytes(out) == oracle.encode(pcm, frames, bits, ch).tobytes()


@pytest.mark.parametrize("wav", ["square-mono.wav", "square-stereo.wav"])
@pytest.mark.parametrize("bits", [4, 6, 8])
def test_encode_fixture_sha1(wav, bits, manifest, golden):
    import hashlib
    xa = bjxa_amd.encode_wav(golden(wav), bits)
    assert hashlib.sha1(xa).hexdigest() == manifest["encode"][wav][str(bits)]


def test_routing_api(built):
    """bjxa_hip_offload_threshold: set/query per direction, EINVAL else."""
    old = bjxa_amd.offload_threshold(bjxa_amd.OFFLOAD_DECODE, 12345)
    assert bjxa_amd.offload_threshold(bjxa_amd.OFFLOAD_DECODE) == 12345
    assert bjxa_amd.offload_threshold(bjxa_amd.OFFLOAD_DECODE, old) == 12345
    with pytest.raises(bjxa_amd.BjxaError) as ei:
        bjxa_amd.offload_threshold(7)
    assert ei.value.errno == errno.EINVAL
