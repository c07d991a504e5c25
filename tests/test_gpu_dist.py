"""One stream split over ranks on the GPU path (bjxa_amd.dist with
device_range_decoder): two gloo ranks sharing the box's GPU, each decoding
its range through bjxa_hip_decode_async; the joined PCM must equal the
oracle's single-pass decode."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream(eb, bits, ch, mix, bad):
    from bjxa_amd import synth
    xa = synth.stream(eb, bits, ch, mix, seed=88)
    if bad is not None:
        xa[(bad[0] * ch + bad[1]) * (bits * 4 + 1)] = 0x5C
    return xa


def _worker(rank, world, port, q, eb, bits, ch, mix, warmup, frames, init, bad):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bjxa_amd import dist as bdist
        xa = _stream(eb, bits, ch, mix, bad)
        ebsz = (bits * 4 + 1) * ch
        lo, hi = bdist.split_ranges(eb, world)[rank]
        first = max(lo - warmup, 0)
        src = torch.from_numpy(xa[first * ebsz:hi * ebsz].copy()).cuda()
        dst = torch.zeros((hi - first) * 64 * ch, dtype=torch.uint8, device="cuda")
        dec = bdist.device_range_decoder(src.data_ptr(), dst.data_ptr(), lo, hi, frames,
                                         bits, ch, warmup)
        fin, fbad = bdist.resolve(dec, lo, hi, init, warmup)
        n = (min(frames, hi * 32) - lo * 32) * ch
        pcm = dst.cpu().numpy().view(np.int16)[(lo - first) * 32 * ch:][:n]
        q.put((rank, pcm.tobytes(), fin, fbad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mix,warmup,bad", [
    ("A", 8, None), ("W", 0, None),
    # a bad right block mid-range; one in rank 1's warm-up (rank 0 owns it);
    # one at rank 1's first eblock
    ("A", 8, (100_000, 1)), ("W", 8, (150_000 - 3, 0)), ("A", 8, (150_000, 1)),
    # a bad right block in the last, cut eblock: the carried left state
    # comes from frames 30/31 the cut PCM does not hold (round-2 ADVICE)
    ("A", 8, (300_000, 1))])
def test_split_two_ranks_on_gpu(built, mix, warmup, bad):
    import oracle
    world, eb, bits, ch = 2, 300_001, 8, 2
    frames = eb * 32 - 3
    init = (5, -6, 7, -8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, eb, bits, ch, mix, warmup,
                                                 frames, init, bad)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    xa = _stream(eb, bits, ch, mix, bad)
    ref, st_ref, done, badc = oracle.decode(xa, eb, bits, ch, init, frames)
    joined = b"".join(r[1] for r in res)
    for r in res:
        assert tuple(r[2]) == tuple(st_ref)
    if bad is None:
        assert joined == ref.tobytes()
        assert all(r[3] is None for r in res)
    else:
        assert (done, badc) == bad
        n = done * 32 * ch * 2
        assert joined[:n] == ref.tobytes()[:n]
        assert all(r[3] == bad[0] * ch + bad[1] for r in res)
