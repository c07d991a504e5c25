"""BASELINE config C5 on one GPU, at full size: the 1,024-stream job (8-bit
stereo, 65,536 eblocks per stream, seeded as bench.py seeds it) decoded in
one batch, and as the exact per-rank shares that `bench.py --gpus N` gives
every rank at N = 2, 4 and 8 (bench.shard_range).  Every stream's PCM and
exit state is compared with the oracle (src/libbjxa.c:602-661, once per
stream), decoded on host threads.  The shares are decoded one after another
on the one GPU, each in a batch of its own with fresh per-stream buffers,
as each rank of an N-GPU run decodes its share; the N = 8 share is the C5g
shape whose plan (64-eblock chunks, an 8 KiB lane stride) the placement
rule of xa_gpu.hip packed_pcm() acts on."""
import threading

import numpy as np
import pytest

import bjxa_amd
import oracle
from gpu_util import require_gpu, status_state

pytestmark = pytest.mark.gpu

NSTREAMS, EBLOCKS, BITS, CH = 1024, 65536, 8, 2
PCM_BYTES = EBLOCKS * 64 * CH


def _threads():
    import os
    return max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def c5(built):
    """(inputs, device tensor of every stream's reference PCM [n, PCM_BYTES],
    reference exit states)."""
    torch = require_gpu()
    import bench
    inputs = [None] * NSTREAMS
    states = [None] * NSTREAMS
    ref = torch.empty((NSTREAMS, PCM_BYTES), dtype=torch.uint8, device="cuda")
    nth = _threads()
    lock = threading.Lock()

    def work(k):
        for j in range(k, NSTREAMS, nth):
            (item,) = bench.batch_inputs("C5", 0, 0, j, j + 1)
            i, bits, ch, eb, xa = item
            assert (i, bits, ch, eb) == (j, BITS, CH, EBLOCKS)
            pcm, st, done, bad = oracle.decode(xa, eb, bits, ch)
            assert bad < 0 and done == eb
            inputs[j] = item
            states[j] = tuple(int(v) for v in st)
            with lock:
                ref[j].copy_(torch.from_numpy(pcm.view(np.uint8)))
    ths = [threading.Thread(target=work, args=(k,)) for k in range(nth)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert all(x is not None for x in inputs)
    torch.cuda.synchronize()
    return inputs, ref, states


def _decode_share(c5, lo, hi):
    """One batch over streams lo..hi-1 in per-stream torch buffers; returns
    the list of stream indices whose PCM or exit state differs, and the
    status rows."""
    torch = require_gpu()
    inputs, ref, states = c5
    share = inputs[lo:hi]
    srcs = [torch.from_numpy(xa).cuda() for _, _, _, _, xa in share]
    dsts = [torch.full((PCM_BYTES,), 0x5A, dtype=torch.uint8, device="cuda") for _ in share]
    streams = [{"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": EBLOCKS,
                "bits": BITS, "channels": CH} for s, d in zip(srcs, dsts)]
    n = hi - lo
    status = torch.zeros(n * bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    with bjxa_amd.Batch(streams, stream=sh) as b:
        b.decode(status.data_ptr(), sh)
        torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint32).reshape(n, -1).copy()
    bad = [lo + k for k, d in enumerate(dsts)
           if not torch.equal(d, ref[lo + k]) or st[k][0] != bjxa_amd.NO_ERROR or
           status_state(st[k]) != states[lo + k]]
    del srcs, dsts
    torch.cuda.empty_cache()
    return bad, st


def test_c5_full_job(c5):
    """All 1,024 streams in one launch (bench's C5 at N = 1)."""
    bad, st = _decode_share(c5, 0, NSTREAMS)
    assert not bad, bad[:10]
    assert st[:, 5].sum() > 0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c5_rank_shares(c5, world):
    """Every rank's share at N = world, as bench.shard_range cuts the job;
    the shares together cover every stream once."""
    import bench
    covered = []
    for rank in range(world):
        lo, hi = bench.shard_range(NSTREAMS, rank, world)
        covered.extend(range(lo, hi))
        bad, st = _decode_share(c5, lo, hi)
        assert not bad, (world, rank, bad[:10])
        if world == 8:
            # C5g: 128 x 131072 channel blocks over 131072 lanes -> 128
            # channel blocks per lane, 64 stereo eblocks per chunk; separate
            # torch buffers are not "packed" (xa_gpu.hip packed_pcm)
            assert (st[:, 6] == 64).all(), set(st[:, 6].tolist())
    assert covered == list(range(NSTREAMS))
