"""GPU decode parity: the gfx950 kernels against the oracle and the
reference's known answers.  Bit-exact int16 PCM is the only bar."""
import errno
import hashlib

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, status_state

pytestmark = pytest.mark.gpu

FIXTURES = ["square-mono-4.xa", "square-mono-6.xa", "square-mono-8.xa",
            "square-stereo-4.xa", "square-stereo-6.xa", "square-stereo-8.xa"]


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_wav_sha1(built, name, manifest, golden):
    """test/test_decode.sh:24-78 through the drop-in C API, single pass."""
    wav = bjxa_amd.decode_file(golden(name))
    assert hashlib.sha1(wav).hexdigest() == manifest["fixtures"][name]["wav_sha1"]


def test_saturation_vector(built, manifest):
    """test/test_decode.sh:80-122 (the int16 clamp)."""
    wav = bjxa_amd.decode_file(bytes.fromhex(manifest["boundary"]["hex"]))
    assert hashlib.sha1(wav).hexdigest() == manifest["boundary"]["wav_sha1"]


@pytest.mark.parametrize("name", ["square-mono-8.xa", "square-stereo-6.xa"])
def test_fixture_incremental(built, name, golden):
    """The bjxa(1) default loop: one bjxa_decode per block
    (src/bjxa_decode.c:122-152), plus uneven multi-block calls."""
    data = golden(name)
    ref = oracle.decode_file(data)[44:]
    for sizes in ([1] * 40 + [10 ** 9], [7, 1000, 3, 10 ** 9]):
        with bjxa_amd.Decoder() as d:
            d.parse_header(data[:32])
            fmt = d.decode_format()
            bx, bp = fmt["block_size_xa"], fmt["block_size_pcm"]
            xa = np.frombuffer(data, np.uint8, offset=32)
            out, pos, left = bytearray(), 0, fmt["data_len_pcm"]
            for n in sizes:
                if pos >= fmt["blocks"]:
                    break
                n = min(n, fmt["blocks"] - pos)
                dst = np.zeros(n * bp, np.uint8)
                got = d.decode(dst, xa[pos * bx:(pos + n) * bx].copy())
                assert got == n
                take = min(n * bp, left)
                out += dst[:take].tobytes()
                left -= take
                pos += n
            with pytest.raises(bjxa_amd.BjxaError) as ei:
                d.decode(np.zeros(bp, np.uint8), np.zeros(bx, np.uint8))
            assert ei.value.errno == errno.EPROTO     # past the end
        assert bytes(out) == ref


@pytest.mark.parametrize("bits", [4, 6, 8])
@pytest.mark.parametrize("ch", [1, 2])
@pytest.mark.parametrize("mix", ["A", "F", "W", "Z"])
def test_random_streams(built, bits, ch, mix):
    eb = 40000 + 17 * bits + ch
    xa = synth.stream(eb, bits, ch, mix, seed=bits * 10 + ch)
    frames = eb * 32 - 11
    state = (1234, -555, -32768, 32767)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, state, frames=frames)
    got, st = dev_decode(xa, eb, bits, ch, frames=frames, state=state, want_status=True)
    assert np.array_equal(got, ref)
    assert st[0] == bjxa_amd.NO_ERROR
    n = 2 * ch
    assert status_state(st)[:n] == st_ref[:n]


@pytest.mark.parametrize("chunk,warmup", [(2, 0), (4, 0), (8, 2), (16, 4), (64, 0), (4, 64)])
def test_repair_paths(built, chunk, warmup):
    """Short/zero warm-up forces mismatching chunks, repairs that do not
    converge within a chunk, and cascades through the sequential tail."""
    for ch, bits in ((2, 8), (1, 6)):
        eb = 5003
        xa = synth.stream(eb, bits, ch, "W", seed=chunk * 100 + warmup)
        ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch)
        got, st = dev_decode(xa, eb, bits, ch, chunk=chunk, warmup=warmup, want_status=True)
        assert np.array_equal(got, ref)
        assert status_state(st)[:2 * ch] == st_ref[:2 * ch]


@pytest.mark.parametrize("cut", [0, 8, 4, 3])
def test_store_paths(built, cut):
    """Each of K1's three store paths out of the LDS stage (xa_decode.hip
    store_lines, ost_line / ost_piece / ost_quad): a stream whose last wave
    is partial, ending on a whole block (cut 0) or inside its last block on
    a 16-B boundary of the PCM (stereo cut 4 or 8 frames, mono cut 8) --
    the predicated fast path -- or off it (cut 3, mono cut 4: per-piece
    bounds and the 2-byte tail); every format, bit-exact."""
    for bits in (4, 6, 8):
        for ch in (1, 2):
            eb = 64 * 40 * 3 + 40 * 5 + 17      # 3 whole waves, 5 chunks + 17 eblocks
            xa = synth.stream(eb, bits, ch, "A", seed=900 + cut + bits + ch)
            frames = eb * 32 - cut
            ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, frames=frames)
            got, st = dev_decode(xa, eb, bits, ch, frames=frames, chunk=40,
                                 want_status=True)
            assert np.array_equal(got, ref), (bits, ch, cut)
            assert status_state(st)[:2 * ch] == st_ref[:2 * ch]


@pytest.mark.parametrize("eb", [1, 2, 3, 5, 31, 257])
def test_tiny_streams(built, eb):
    for bits in (4, 6, 8):
        for ch in (1, 2):
            xa = synth.stream(eb, bits, ch, "A", seed=eb)
            for frames in {eb * 32, eb * 32 - 31, eb * 32 - 1}:
                ref, _, _, _ = oracle.decode(xa, eb, bits, ch, (5, -7, 9, -11), frames=frames)
                got = dev_decode(xa, eb, bits, ch, frames=frames, state=(5, -7, 9, -11))
                assert np.array_equal(got, ref), (bits, ch, frames)


def test_clamp_heavy(built):
    """Saturating inputs everywhere: gain 4 at range 0 with extreme codes."""
    eb = 20000
    xa = synth.stream(eb, 8, 2, "A", seed=77).reshape(eb * 2, 33)
    xa[:, 0] = np.where(np.arange(eb * 2) % 3 == 0, 0x40, 0x30)
    xa[:, 1:] = np.where(np.arange(32) % 2 == 0, 0x7F, 0x80)
    xa = xa.reshape(-1)
    ref, _, _, _ = oracle.decode(xa, eb, 8, 2)
    assert (ref == 32767).any() and (ref == -32768).any()
    assert np.array_equal(dev_decode(xa, eb, 8, 2), ref)


@pytest.mark.parametrize("ch,bad", [(1, 0), (2, 0), (2, 1)])
def test_invalid_profile(built, ch, bad):
    """test/test_decode_error.sh:221-282 semantics through bjxa_decode:
    blocks before the bad one are decoded and counted, the call fails with
    EPROTO, a bad right block has already advanced the left channel."""
    eb, j = 300, 123
    xa = synth.stream(eb, 8, ch, "A", seed=ch + bad).reshape(eb * ch, 33)
    xa[j * ch + bad, 0] = 0x5F
    hdr = bjxa_amd.xa_header(xa.size, eb * 32, 44100, 8, ch)
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        dst = np.full(eb * 64 * ch, 0x11, np.uint8)
        with pytest.raises(bjxa_amd.BjxaError) as ei:
            d.decode(dst, xa.reshape(-1).copy())
        assert ei.value.errno == errno.EPROTO
        ref, st_ref, done, badc = oracle.decode(xa.reshape(-1), eb, 8, ch)
        assert done == j and badc == bad
        assert np.array_equal(dst[:j * 64 * ch].view(np.int16), ref[:j * 32 * ch])
        assert (dst[j * 64 * ch:] == 0x11).all()
        # only the decoded prefix was accounted for: the next call starts
        # at the bad eblock and fails again
        with pytest.raises(bjxa_amd.BjxaError):
            d.decode(dst, xa.reshape(-1)[j * ch * 33:].copy())
    # the carried state is the reference's partial update (a bad right block
    # leaves the left channel advanced): continuing with a patched profile
    # must equal the oracle continuing from its own partial state
    fixed = xa.copy()
    fixed[j * ch + bad, 0] = 0x00
    ref2, _, _, _ = oracle.decode(fixed.reshape(-1)[j * ch * 33:], eb - j, 8, ch, st_ref)
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        dst = np.zeros(eb * 64 * ch, np.uint8)
        with pytest.raises(bjxa_amd.BjxaError):
            d.decode(dst, xa.reshape(-1).copy())
        dst2 = np.zeros((eb - j) * 64 * ch, np.uint8)
        assert d.decode(dst2, fixed.reshape(-1)[j * ch * 33:].copy()) == eb - j
        assert np.array_equal(dst2.view(np.int16), ref2)


def test_bef_entry_state(built, golden):
    """A header's befL/befR seeds the predictor (src/libbjxa.c:417-420)."""
    xa = synth.stream(1000, 4, 2, "A", seed=5)
    st = (-20000, 30000, 12345, -12345)
    hdr = bjxa_amd.xa_header(xa.size, 1000 * 32 - 5, 22050, 4, 2, st)
    wav = bjxa_amd.decode_file(hdr + xa.tobytes())
    assert wav == oracle.decode_file(hdr + xa.tobytes())


_K = np.array([[0, 0], [240, 0], [460, -208], [392, -220], [488, -240]] +
              [[0, 0]] * 11, dtype=np.int64)


def _big_gain_steps(xa, eb, bits, ch, pcm):
    """Predictor steps whose |p0*K0 + p1*K1| >= 2^24 (src/libbjxa.c:565),
    where the kernels' f32 prediction rounds and only the int16 clamp makes
    it exact."""
    s = pcm.reshape(eb, 32, ch).astype(np.int64)
    prof = xa.reshape(eb, ch, bits * 4 + 1)[:, :, 0].astype(np.int64)
    n = 0
    for c in range(ch):
        x = s[:, :, c].reshape(-1)
        g = (prof[:, c] >> 4).repeat(32)
        p0 = np.concatenate([[0], x[:-1]])
        p1 = np.concatenate([[0, 0], x[:-2]])
        n += int(np.sum(np.abs(p0 * _K[g, 0] + p1 * _K[g, 1]) >= 1 << 24))
    return n


@pytest.mark.parametrize("ch", [1, 2])
def test_f32_rounding_regime(built, ch):
    """The f32 steps (xa_step_lr, xa_step_f) round p0*K0/256 + p1*K1/256 once
    |g| >= 2^24; the stream must reach that regime often and still match
    the oracle bit for bit."""
    eb = 40000
    xa = synth.stream(eb, 8, ch, "A", seed=1234 + ch).reshape(eb * ch, 33)
    # every other channel block at gain 4, range 0 (uniform codes): the
    # state swings across the whole int16 range, and about 1 % of the steps
    # have |g| >= 2^24
    xa[np.arange(eb * ch) % 2 == 0, 0] = 0x40
    xa = xa.reshape(-1)
    ref, _, _, _ = oracle.decode(xa, eb, 8, ch)
    assert _big_gain_steps(xa, eb, 8, ch, ref) > 10000
    assert np.array_equal(dev_decode(xa, eb, 8, ch), ref)


@pytest.mark.parametrize("bits", [4, 6, 8])
@pytest.mark.parametrize("ch", [1, 2])
def test_repair_cut_block_exact_dst(built, bits, ch):
    """Repairs everywhere (warm-up 0, 16-eblock chunks, mix W) on a stream
    whose last block is cut, decoded into a PCM buffer of exactly the
    emitted frames (rounded up to the 16-B alignment) followed by a guard:
    the repair path must emit the cut block exactly and never touch the
    guard (the old end state of the cut block is not read)."""
    torch = pytest.importorskip("torch")
    eb = 4099
    for cut in (1, 17, 31):
        frames = eb * 32 - cut
        xa = synth.stream(eb, bits, ch, "W", seed=bits * 7 + ch + cut)
        ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, (9, -9, 99, -99), frames=frames)
        nbytes = frames * 2 * ch
        alloc = (nbytes + 15) // 16 * 16
        buf = torch.full((alloc + 4096,), 0x5A, dtype=torch.uint8, device="cuda")
        src = torch.from_numpy(xa).cuda()
        ws_len = bjxa_amd.decode_workspace_size(eb, ch, 16, 0)
        ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
        status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        bjxa_amd.workspace_init(ws.data_ptr(), ws_len, s)
        bjxa_amd.decode_device(src.data_ptr(), buf.data_ptr(), eb, frames, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (9, -9, 99, -99),
                               16, 0, s)
        torch.cuda.synchronize()
        out = buf.cpu().numpy()
        st = status.cpu().numpy().view(np.uint32)
        assert st[3] > 0                                    # repairs ran
        assert np.array_equal(out[:nbytes].view(np.int16), ref), cut
        assert (out[nbytes:] == 0x5A).all(), cut
        assert status_state(st)[:2 * ch] == st_ref[:2 * ch]
