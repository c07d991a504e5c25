"""Batched decode (bjxa_hip_batch_*): many streams of mixed formats per
launch, each bit-exact against the oracle's single-stream decode
(src/libbjxa.c:602-661 per stream), with per-stream status."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import require_gpu, status_state

pytestmark = pytest.mark.gpu

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)]


def run_batch(specs, chunk=0, warmup=-1, repeat=1, variant=0):
    """specs: list of (xa bytes, eblocks, bits, ch, frames, state).  Returns
    (pcm list, status array [n, 8])."""
    torch = require_gpu()
    srcs, dsts, streams = [], [], []
    for xa, eb, bits, ch, frames, state in specs:
        s = torch.from_numpy(np.ascontiguousarray(xa)).cuda()
        d = torch.full((eb * 64 * ch,), 0x5A, dtype=torch.uint8, device="cuda")
        srcs.append(s)
        dsts.append(d)
        streams.append({"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb,
                        "bits": bits, "channels": ch, "frames": frames, "state": state})
    status = torch.zeros(len(specs) * bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    with bjxa_amd.Batch(streams, chunk, warmup, sh, variant) as b:
        for _ in range(repeat):
            b.decode(status.data_ptr(), sh)
        torch.cuda.synchronize()
    out = []
    for (xa, eb, bits, ch, frames, state), d in zip(specs, dsts):
        raw = d.cpu().numpy()
        assert (raw[frames * ch * 2:] == 0x5A).all()
        out.append(raw.view(np.int16)[:frames * ch].copy())
    return out, status.cpu().numpy().view(np.uint32).reshape(len(specs), -1).copy()


def check(specs, pcms, st):
    for i, ((xa, eb, bits, ch, frames, state), pcm) in enumerate(zip(specs, pcms)):
        ref, st_ref, done, bad = oracle.decode(xa, eb, bits, ch, state, frames)
        if bad < 0:
            assert st[i][0] == bjxa_amd.NO_ERROR, i
            assert np.array_equal(pcm, ref), "stream %d (%d-bit, %dch, %d eblocks)" % (
                i, bits, ch, eb)
            assert status_state(st[i])[:2 * ch] == st_ref[:2 * ch], i
        else:
            # first failing channel block; output before it must match
            assert st[i][0] == done * ch + bad, (i, st[i][0], done, bad)
            n = done * 32 * ch
            assert np.array_equal(pcm[:n], ref[:n]), i


def make(eb, bits, ch, seed, mix="A", cut=0, state=(0, 0, 0, 0)):
    xa = synth.stream(eb, bits, ch, mix, seed=seed)
    return (xa, eb, bits, ch, eb * 32 - cut, state)


@pytest.mark.parametrize("variant", [0, bjxa_amd.VARIANT_DECOR])
def test_batch_mixed_formats(built, variant):
    """Every format, ragged lengths, cut last blocks, entry states; with
    VARIANT_DECOR every stream also gets the packed-layout plan (chunks one
    quantum longer where the stride is on 8 KiB)."""
    rng = np.random.default_rng(3)
    specs = []
    for i in range(48):
        bits, ch = FORMATS[i % 6]
        eb = int(rng.choice([1, 2, 17, 63, 64, 65, 1000, 4097, 20000, 70001]))
        cut = int(rng.integers(0, 32)) if i % 4 == 0 else 0
        state = tuple(int(v) for v in rng.integers(-3000, 3000, 4))
        specs.append(make(eb, bits, ch, 100 + i, cut=cut, state=state))
    pcms, st = run_batch(specs, variant=variant)
    check(specs, pcms, st)


@pytest.mark.parametrize("variant", [0, bjxa_amd.VARIANT_DECOR])
def test_batch_repairs_and_cascades(built, variant):
    """Warm-up 0 and short chunks: nearly every chunk is repaired and
    worst-case profiles cascade through whole chunks (with and without the
    packed-layout plan)."""
    specs = [make(30000, bits, ch, 200 + i, mix="W" if i % 2 else "A")
             for i, (bits, ch) in enumerate(FORMATS)]
    pcms, st = run_batch(specs, chunk=16, warmup=0, variant=variant)
    check(specs, pcms, st)
    assert st[:, 3].sum() > 0


def test_batch_repeat_reuses_workspace(built):
    specs = [make(50000, 8, 2, 300), make(50000, 8, 1, 301, cut=5)]
    pcms, st = run_batch(specs, repeat=3)
    check(specs, pcms, st)


def test_batch_invalid_profiles(built):
    """A gain nibble >= 5 in some streams reports that stream's first failing
    channel block; the other streams are unaffected."""
    specs = []
    for i, (bits, ch) in enumerate(FORMATS):
        xa, eb, b_, c_, frames, state = make(5000, bits, ch, 400 + i)
        if i % 2 == 0:
            bsz = bits * 4 + 1
            blk = 1234 * ch + (ch - 1)          # the R block when stereo
            xa = xa.copy()
            xa[blk * bsz] = 0x5F
        specs.append((xa, eb, b_, c_, frames, state))
    pcms, st = run_batch(specs)
    check(specs, pcms, st)


def test_batch_c5_shape(built):
    """C5-shaped (8-bit stereo, 65,536 eblocks per stream), 32 streams."""
    specs = [make(65536, 8, 2, 500 + i) for i in range(32)]
    pcms, st = run_batch(specs)
    check(specs, pcms, st)
    assert (st[:, 6] == 16).all()      # 32 x 131072 channel blocks over 131072 lanes, / 2


def test_batch_c4_full_size(built):
    """BASELINE config C4 at full size in one launch: 1024 streams, stream i
    with bits (4,6,8)[i%3], channels 1+((i/3)&1), 16,384 eblocks, seeded as
    bench.py seeds them; every stream bit-exact against the oracle (decoded
    on 8 host threads) and its exit state equal."""
    import threading
    torch = require_gpu()
    import bench
    inputs = bench.batch_inputs("C4", 0, 0, 0, 1024)
    assert len(inputs) == 1024
    srcs, dsts, streams = [], [], []
    for i, bits, ch, eb, xa in inputs:
        s = torch.from_numpy(xa).cuda()
        d = torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
        srcs.append(s)
        dsts.append(d)
        streams.append({"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb,
                        "bits": bits, "channels": ch})
    status = torch.zeros(1024 * bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    with bjxa_amd.Batch(streams, stream=sh) as b:
        b.decode(status.data_ptr(), sh)
        torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint32).reshape(1024, -1)
    bad = []

    def work(k):
        for j in range(k, 1024, 8):
            i, bits, ch, eb, xa = inputs[j]
            ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch)
            got = dsts[j].cpu().numpy().view(np.int16)
            if (not np.array_equal(got, ref) or st[j][0] != bjxa_amd.NO_ERROR or
                    status_state(st[j])[:2 * ch] != st_ref[:2 * ch]):
                bad.append(i)
    ths = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not bad, bad[:10]


def test_batch_streams_share_k1_workgroups(built):
    """Streams of one or two waves each, so every K1 workgroup holds waves
    of several streams and formats: its inner-boundary verification must
    check a wave's first chunk against the previous wave only when both are
    the same stream.  Warm-up 0 with chunks of 16 forces repairs and
    cascades inside workgroups and across their boundaries (K2); entry
    states, cut last blocks and an invalid profile ride along."""
    rng = np.random.default_rng(21)
    specs = []
    for i in range(40):
        bits, ch = FORMATS[i % 6]
        eb = int(rng.integers(40, 2048))
        cut = int(rng.integers(1, 32)) if i % 5 == 0 else 0
        state = tuple(int(v) for v in rng.integers(-3000, 3000, 4))
        specs.append(make(eb, bits, ch, 800 + i, mix="W" if i % 3 == 0 else "A",
                          cut=cut, state=state))
    xa, eb, bits, ch, frames, state = specs[7]
    xa = xa.copy()
    xa[(eb // 2) * ch * (bits * 4 + 1)] = 0x5F
    specs[7] = (xa, eb, bits, ch, frames, state)
    pcms, st = run_batch(specs, chunk=16, warmup=0)
    check(specs, pcms, st)
    assert st[:, 3].sum() > 0


class RawBuffers:
    """Device buffers each from a hipMalloc of its own (outside torch's
    caching allocator, which carves mid-size tensors out of shared
    segments), as uint8 tensors; freed on exit."""

    def __init__(self):
        import ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.hip.hipFree.argtypes = [ctypes.c_void_p]
        self.ptrs = []

    def get(self, n, fill=0x5A):
        import ctypes
        torch = require_gpu()
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), n) == 0
        self.ptrs.append(p.value)

        class Iface:
            __cuda_array_interface__ = {"shape": (n,), "typestr": "|u1",
                                        "data": (p.value, False), "version": 2}
        t = torch.as_tensor(Iface(), device="cuda")
        t.fill_(fill)
        return t

    def __enter__(self):
        return self

    def __exit__(self, *a):
        require_gpu().cuda.synchronize()
        for p in self.ptrs:
            self.hip.hipFree(p)


PACKED_SPAN = 64 << 20      # xa_gpu.hip XA_PACKED_SPAN


def run_packed(specs, chunk, layout, variant=0):
    """run_batch with the PCM images laid out as `layout`:
      "packed"  back to back at the start of one allocation of at least
                PACKED_SPAN bytes (a caller's own big buffer)
      "raw"     a hipMalloc of its own each
      "torch"   a torch tensor each (small ones share the caching
                allocator's segments)
      "carved"  a torch tensor each, carved by the caching allocator out of
                one freed block of 128 MiB (so one allocation of >= 64 MiB,
                at offsets the allocator chose)"""
    torch = require_gpu()
    sizes = [eb * 64 * ch for _, eb, _, ch, _, _ in specs]
    with RawBuffers() as raw:
        if layout == "packed":
            big = torch.full((max(sum(sizes), PACKED_SPAN),), 0x5A, dtype=torch.uint8,
                             device="cuda")
            offs = np.cumsum([0] + sizes[:-1])
            dsts = [big[o:o + n] for o, n in zip(offs, sizes)]
        elif layout == "raw":
            dsts = [raw.get(n) for n in sizes]
        elif layout == "carved":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            big = torch.empty((128 << 20,), dtype=torch.uint8, device="cuda")
            del big                     # cached, free: the next tensors split it
            dsts = [torch.full((n,), 0x5A, dtype=torch.uint8, device="cuda") for n in sizes]
        else:
            dsts = [torch.full((n,), 0x5A, dtype=torch.uint8, device="cuda") for n in sizes]
        srcs = [torch.from_numpy(np.ascontiguousarray(xa)).cuda() for xa, *_ in specs]
        streams = [{"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb,
                    "bits": bits, "channels": ch, "frames": frames, "state": state}
                   for s, d, (xa, eb, bits, ch, frames, state) in zip(srcs, dsts, specs)]
        status = torch.zeros(len(specs) * bjxa_amd.STATUS_WORDS, dtype=torch.int32,
                             device="cuda")
        sh = torch.cuda.current_stream().cuda_stream
        with bjxa_amd.Batch(streams, chunk, -1, sh, variant) as b:
            b.decode(status.data_ptr(), sh)
            torch.cuda.synchronize()
        out = [d.cpu().numpy().view(np.int16)[:frames * ch].copy()
               for d, (_, _, _, ch, frames, _) in zip(dsts, specs)]
    return out, status.cpu().numpy().view(np.uint32).reshape(len(specs), -1).copy()


@pytest.mark.parametrize("layout", ["raw", "torch", "packed", "carved"])
def test_batch_packed_layout_plan(built, layout):
    """Streams whose PCM lane stride is a multiple of 8 KiB (here 64 stereo
    eblocks per lane) get chunks one quantum longer only when eight or more
    PCM images share one allocation of at least 64 MiB (a caller's packed
    buffer); in allocations of their own, and in torch tensors that share
    the caching allocator's (smaller) segments, they keep them (DESIGN.md §5
    R4-7, R5-4).  Tensors the caching allocator carves out of one freed
    block of >= 64 MiB share that allocation as a packed buffer does, and R4-11
    measured one allocation to want the longer chunks whatever the offsets
    between its images, so they count as packed.  Bit-exact
    either way, including with the choice forced off and on."""
    eb = 16384 if layout == "carved" else 4096      # 2 MiB PCM: the large pool
    specs = [make(eb, 8, 2, 900 + i, cut=(5 if i == 3 else 0)) for i in range(8)]
    chunk = 128
    pcms, st = run_packed(specs, chunk, layout)
    check(specs, pcms, st)
    assert (st[:, 6] == (68 if layout in ("packed", "carved") else 64)).all()
    for v, c in ((bjxa_amd.VARIANT_NODECOR, 64), (bjxa_amd.VARIANT_DECOR, 68)):
        pcms, st = run_packed(specs, chunk, layout, v)
        check(specs, pcms, st)
        assert (st[:, 6] == c).all()
