"""The verify/repair pass inside the decode kernel (xa_decode.hip
settle_wave) and what it leaves to the sequential tail: cascades, wave
boundaries whose exit record does not come (forced with the tuning knobs
VARIANT_NORECORD / VARIANT_NOWAIT), and a workspace left inconsistent by a
failed launch -- every case bit-exact against the
oracle, which restates src/libbjxa.c:533-578 / :602-661."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import dev_decode, require_gpu, status_state
from test_gpu_batch import FORMATS, check, make, run_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("bits,ch", [(8, 2), (6, 1), (4, 2)])
def test_long_cascades(built, bits, ch):
    """Mix W (gain 4 only, ranges 12-15: the slowest resync), no warm-up,
    16-eblock chunks: nearly every chunk is repaired in the decode kernel
    and repairs that never meet the stored trajectory cascade through the
    tail, across waves."""
    eb = 400_003
    frames = eb * 32 - 3
    xa = synth.stream(eb, bits, ch, "W", seed=11)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, (7, -7, 70, -70), frames)
    got, st = dev_decode(xa, eb, bits, ch, frames=frames, state=(7, -7, 70, -70),
                         chunk=16, warmup=0, want_status=True)
    assert np.array_equal(got, ref)
    assert status_state(st)[:2 * ch] == st_ref[:2 * ch]
    assert st[3] > st[5] // 4          # repairs in the decode kernel
    assert st[4] > 0                   # and cascades in the tail


@pytest.mark.parametrize("variant", [bjxa_amd.VARIANT_NORECORD, bjxa_amd.VARIANT_NOWAIT,
                                     bjxa_amd.VARIANT_NORECORD | bjxa_amd.VARIANT_NOWAIT])
@pytest.mark.parametrize("mix", ["A", "W"])
def test_boundaries_left_to_tail(built, variant, mix):
    """Waves that get no exit record from the wave before them (none
    written, or none waited for) queue their first boundary for the tail,
    which re-checks and repairs it in chunk order."""
    eb = 1_000_000
    xa = synth.stream(eb, 8, 2, mix, seed=12)
    ref, st_ref, _, _ = oracle.decode(xa, eb, 8, 2)
    got, st = dev_decode(xa, eb, 8, 2, want_status=True, variant=variant, warmup=0)
    assert np.array_equal(got, ref)
    assert status_state(st) == st_ref
    if variant & bjxa_amd.VARIANT_NORECORD:
        assert st[4] > 0


def _layout(nchunks):
    """Byte offsets of the single-stream workspace (xa_gpu.hip ws_bytes):
    control words, g, e, queue (2n), exit records (16-B aligned)."""
    g = 256
    e = g + 8 * nchunks
    q = e + 8 * nchunks
    x = (q + 8 * nchunks + 15) // 16 * 16
    return g, e, q, x


@pytest.mark.parametrize("poke", ["full", "stale"])
def test_stale_workspace(built, poke):
    """A workspace as a failed launch could leave it: the queue length at
    (full) or below (stale) capacity with garbage entries, some out of
    range, and garbage exit records.  The next decode on it must still be
    bit-exact -- past the capacity the tail re-checks every boundary, and
    entries outside the stream are skipped -- and leave it clean."""
    torch = require_gpu()
    eb, bits, ch = 600_000, 8, 2
    xa = synth.stream(eb, bits, ch, "W", seed=13)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch)
    src = torch.from_numpy(xa).cuda()
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
    ws_len = bjxa_amd.decode_workspace_size(eb, ch, 0, 0)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    def decode():
        dst.fill_(0x5A)
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0), 0, 0,
                               sh)
        torch.cuda.synchronize()
        return dst.cpu().numpy().view(np.int16), status.cpu().numpy().view(np.uint32).copy()

    got, st = decode()
    assert np.array_equal(got, ref)
    n = int(st[5])
    g, e, q, x = _layout(n)
    assert x + 16 * ((n + 63) // 64) <= ws_len
    rng = np.random.default_rng(14)
    ctl = ws[:256].view(torch.int32)
    ctl[1] = 2 * n if poke == "full" else n // 3          # XA_CTL_NQ
    junk = rng.integers(0, 1 << 32, 2 * n, dtype=np.uint64).astype(np.uint32)
    junk[::7] = rng.integers(1, n, junk[::7].size)        # some in range
    ws[q:q + 8 * n].copy_(torch.from_numpy(junk.view(np.uint8)))
    nx = 16 * ((n + 63) // 64)
    ws[x:x + nx].copy_(torch.from_numpy(rng.integers(0, 256, nx, dtype=np.uint8)))
    got, st = decode()
    assert np.array_equal(got, ref)
    assert status_state(st) == st_ref
    assert int(ctl[1].item()) == 0 and int(ctl[3].item()) == 0   # NQ, OVF reset
    got, st = decode()                                             # and reusable
    assert np.array_equal(got, ref)


def test_smaller_stream_reuses_workspace(built):
    """a smaller stream decoded in a workspace sized for (and
    last used by) a larger one puts its exit records on the larger decode's
    stale g/e/queue words.  Records pass on their launch tag alone, and the
    tag is a small counter, so the worst case is written here: every stale
    word pair in the smaller layout's record region set to the NEXT launch's
    tag with a bogus state beside it.  The library zeroes a record region
    whose layout changed (xa_gpu.hip ws_records_stale); without that, lane
    0 of every wave would repair its chunk from the bogus state."""
    torch = require_gpu()
    big, small, bits, ch = 3_000_000, 900_000, 8, 2
    xa_big = synth.stream(big, bits, ch, "A", seed=17)
    xa_small = synth.stream(small, bits, ch, "W", seed=18)
    ref_big, _, _, _ = oracle.decode(xa_big, big, bits, ch)
    ref_small, st_ref, _, _ = oracle.decode(xa_small, small, bits, ch)
    ws_len = bjxa_amd.decode_workspace_size(big, ch, 0, 0)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    def decode(xa, eb):
        src = torch.from_numpy(xa).cuda()
        dst = torch.full((eb * 64 * ch,), 0x5A, dtype=torch.uint8, device="cuda")
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0),
                               0, 0, sh)
        torch.cuda.synchronize()
        return dst.cpu().numpy().view(np.int16), status.cpu().numpy().view(np.uint32).copy()

    got, st = decode(xa_small, small)          # learn the smaller layout
    assert np.array_equal(got, ref_small)
    n_small = int(st[5])
    got, st = decode(xa_big, big)
    assert np.array_equal(got, ref_big)
    n_big = int(st[5])
    assert n_big > n_small
    xb = _layout(n_big)[3]
    rec = ws[xb:xb + 16].cpu().numpy().view(np.uint32)
    assert rec[1] == rec[3] != 0               # {state, tag} x 2: this launch's tag
    nxt = (int(rec[1]) + 1) & 0xFFFFFFFF or 1
    xs = _layout(n_small)[3]
    nw = (n_small + 63) // 64
    assert xs + 16 * nw <= _layout(n_big)[3]   # inside the big decode's g/e/queue
    words = np.empty((nw, 4), dtype=np.uint32)
    words[:, 0::2] = 0x12345678                # bogus exit state, both channels
    words[:, 1::2] = nxt
    ws[xs:xs + 16 * nw].copy_(torch.from_numpy(words.reshape(-1).view(np.uint8)))
    got, st = decode(xa_small, small)
    assert np.array_equal(got, ref_small)
    assert status_state(st) == st_ref
    rec = ws[xs:xs + 16].cpu().numpy().view(np.uint32)
    assert rec[1] == rec[3] == nxt             # the tag prediction held


def test_larger_stream_after_smaller(built):
    """The other direction of the same hazard: a larger stream after a
    smaller one in the same workspace puts its records where stale words
    lie (here, poisoned with the next launch's tag); the changed layout
    zeroes them first.  Big, small, then big again."""
    torch = require_gpu()
    big, small, bits, ch = 2_500_000, 700_000, 8, 2
    xa_big = synth.stream(big, bits, ch, "W", seed=19)
    xa_small = synth.stream(small, bits, ch, "A", seed=20)
    ref_big, st_ref, _, _ = oracle.decode(xa_big, big, bits, ch)
    ref_small, _, _, _ = oracle.decode(xa_small, small, bits, ch)
    ws_len = bjxa_amd.decode_workspace_size(big, ch, 0, 0)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    def decode(xa, eb):
        src = torch.from_numpy(xa).cuda()
        dst = torch.full((eb * 64 * ch,), 0x5A, dtype=torch.uint8, device="cuda")
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0),
                               0, 0, sh)
        torch.cuda.synchronize()
        return dst.cpu().numpy().view(np.int16), status.cpu().numpy().view(np.uint32).copy()

    got, st = decode(xa_big, big)              # learn the larger layout
    assert np.array_equal(got, ref_big)
    n_big = int(st[5])
    got, st = decode(xa_small, small)
    assert np.array_equal(got, ref_small)
    xs = _layout(int(st[5]))[3]
    rec = ws[xs:xs + 16].cpu().numpy().view(np.uint32)
    assert rec[1] == rec[3] != 0
    nxt = (int(rec[1]) + 1) & 0xFFFFFFFF or 1
    xb = _layout(n_big)[3]
    nw = (n_big + 63) // 64
    words = np.empty((nw, 4), dtype=np.uint32)
    words[:, 0::2] = 0x7FFF8001                # bogus exit state, both channels
    words[:, 1::2] = nxt
    ws[xb:xb + 16 * nw].copy_(torch.from_numpy(words.reshape(-1).view(np.uint8)))
    got, st = decode(xa_big, big)
    assert np.array_equal(got, ref_big)
    assert status_state(st) == st_ref
    rec = ws[xb:xb + 16].cpu().numpy().view(np.uint32)
    assert rec[1] == rec[3] == nxt             # the tag prediction held


@pytest.mark.parametrize("variant", [bjxa_amd.VARIANT_NORECORD, bjxa_amd.VARIANT_NOWAIT])
def test_batch_boundaries_left_to_tail(built, variant):
    """The batch kernel with the same knobs: every format, cascades."""
    specs = [make(40000 + 777 * i, bits, ch, 600 + i, mix="W" if i % 2 else "A",
                  cut=i % 3)
             for i, (bits, ch) in enumerate(FORMATS * 2)]
    pcms, st = run_batch(specs, chunk=16, warmup=0, variant=variant)
    check(specs, pcms, st)
    if variant & bjxa_amd.VARIANT_NORECORD:
        assert st[:, 4].sum() > 0


def test_manual_chunk_capped(built):
    """A manual chunk length whose wave would span more than 4 GiB of XA
    (64 chunks of 2,000,000 8-bit stereo eblocks) is capped by the planner
    (xa_gpu.hip max_chunk), so the repair windows' 32-bit descriptor
    offsets stay in range; the decode is still bit-exact.  Warm-up 0 makes
    the second chunk's entry wrong, so its repair runs through the
    descriptor."""
    eb = 2_100_000
    xa = synth.stream(eb, 8, 2, "W", seed=15)
    ref, st_ref, _, _ = oracle.decode(xa, eb, 8, 2)
    got, st = dev_decode(xa, eb, 8, 2, chunk=2_000_000, warmup=0, want_status=True)
    assert np.array_equal(got, ref)
    assert status_state(st) == st_ref
    cap = ((1 << 32) - (1 << 20)) // (64 * 33 * 2) // 4 * 4
    assert st[6] == cap and st[5] == -(-eb // cap)


def test_pipe2_plan(built):
    """Tuning bit 20 (two decodes in flight): the planner targets half the
    lanes, so the chunks are twice as long; bit-exact, including a ragged
    tail and an entry state."""
    eb = 2_500_003
    frames = eb * 32 - 9
    xa = synth.stream(eb, 8, 2, "A", seed=16)
    ref, st_ref, _, _ = oracle.decode(xa, eb, 8, 2, (3, -3, 30, -30), frames)
    got, st = dev_decode(xa, eb, 8, 2, frames=frames, state=(3, -3, 30, -30),
                         want_status=True, variant=bjxa_amd.VARIANT_PIPE2)
    assert np.array_equal(got, ref)
    assert status_state(st) == st_ref
    c = -(-(-(-eb // 65536)) // 4) * 4     # ceil(eb / (131072 / 2)) to the quantum
    assert st[6] == c
