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


def _worker(rank, world, port, q, eb, bits, ch, mix, warmup, frames, init):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bjxa_amd import dist as bdist, synth
        xa = synth.stream(eb, bits, ch, mix, seed=88)
        ebsz = (bits * 4 + 1) * ch
        lo, hi = bdist.split_ranges(eb, world)[rank]
        first = max(lo - warmup, 0)
        src = torch.from_numpy(xa[first * ebsz:hi * ebsz].copy()).cuda()
        dst = torch.zeros((hi - first) * 64 * ch, dtype=torch.uint8, device="cuda")
        dec = bdist.device_range_decoder(src.data_ptr(), dst.data_ptr(), lo, hi, frames,
                                         bits, ch, warmup)
        fin = bdist.resolve(dec, lo, hi, init, warmup)
        n = (min(frames, hi * 32) - lo * 32) * ch
        pcm = dst.cpu().numpy().view(np.int16)[(lo - first) * 32 * ch:][:n]
        q.put((rank, pcm.tobytes(), fin))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mix,warmup", [("A", 8), ("W", 0)])
def test_split_two_ranks_on_gpu(built, mix, warmup):
    import oracle
    from bjxa_amd import synth
    world, eb, bits, ch = 2, 300_001, 8, 2
    frames = eb * 32 - 3
    init = (5, -6, 7, -8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, eb, bits, ch, mix, warmup,
                                                 frames, init)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    xa = synth.stream(eb, bits, ch, mix, seed=88)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch, init, frames)
    assert b"".join(r[1] for r in res) == ref.tobytes()
    assert tuple(res[0][2]) == tuple(st_ref)
