"""Decodes in flight on several HIP streams at once ("two
in flight"; bench.py --pipeline): each in-flight decode has its own
workspace, status and PCM buffers, consecutive decodes reuse a slot only
after the previous one on the same stream, and every result must equal the
oracle's.  The kernels of neighbouring decodes overlap on the chip (the
next spec kernel starts in the previous one's tail, a fix kernel runs
beside a spec kernel), which is exactly what these tests exercise."""
import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth
from gpu_util import require_gpu

pytestmark = pytest.mark.gpu

JOBS = [  # (eblocks, bits, channels, mix): mix W forces many repairs
    (300_000, 8, 2, "W"), (250_001, 4, 1, "A"), (180_000, 6, 2, "F"),
    (400_000, 8, 1, "W"), (123_457, 6, 1, "A"), (260_000, 4, 2, "W"),
]


@pytest.mark.parametrize("depth", [2, 3])
def test_single_streams_in_flight(built, depth):
    torch = require_gpu()
    inputs = [synth.stream(eb, bits, ch, mix, seed=700 + i)
              for i, (eb, bits, ch, mix) in enumerate(JOBS)]
    refs = [oracle.decode(xa, eb, bits, ch)[0]
            for xa, (eb, bits, ch, _) in zip(inputs, JOBS)]
    srcs = [torch.from_numpy(xa).cuda() for xa in inputs]
    cap_eb = max(eb for eb, _, _, _ in JOBS)
    ws_len = max(bjxa_amd.decode_workspace_size(eb, ch) for eb, _, ch, _ in JOBS)
    slots = []
    for k in range(depth):
        st = torch.cuda.current_stream() if k == 0 else torch.cuda.Stream()
        ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
        bjxa_amd.workspace_init(ws.data_ptr(), ws_len, st.cuda_stream)
        slots.append({"st": st, "ws": ws,
                      "dst": torch.empty(cap_eb * 128, dtype=torch.uint8, device="cuda"),
                      "status": torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32,
                                            device="cuda")})
    torch.cuda.synchronize()
    # three rounds over the jobs, job j of round r on slot (r * len + j) % depth;
    # a slot's PCM is copied out on its own stream before the slot is reused
    outs = {}
    n = 0
    for rnd in range(3):
        for j, (eb, bits, ch, _) in enumerate(JOBS):
            sl = slots[n % depth]
            n += 1
            bjxa_amd.decode_device(srcs[j].data_ptr(), sl["dst"].data_ptr(), eb, eb * 32, bits,
                                   ch, sl["ws"].data_ptr(), ws_len, sl["status"].data_ptr(),
                                   stream=sl["st"].cuda_stream)
            with torch.cuda.stream(sl["st"]):
                outs[(rnd, j)] = (sl["dst"][:eb * 64 * ch].clone(), sl["status"].clone())
    torch.cuda.synchronize()
    for (rnd, j), (pcm, status) in outs.items():
        eb, bits, ch, _ = JOBS[j]
        got = pcm.cpu().numpy().view(np.int16)
        assert np.array_equal(got, refs[j]), "round %d job %d differs" % (rnd, j)
        assert status.cpu().numpy().view(np.uint32)[0] == 0xFFFFFFFF


def test_batches_in_flight(built):
    """Two batch objects (each with its own workspace) decoding the same
    streams into separate PCM buffers on two HIP streams, four times each."""
    torch = require_gpu()
    specs = [(16_384 + 37 * i, (4, 6, 8)[i % 3], 1 + (i // 3) % 2) for i in range(40)]
    inputs = [synth.stream(eb, bits, ch, "W" if i % 4 == 0 else "A", seed=900 + i)
              for i, (eb, bits, ch) in enumerate(specs)]
    refs = [oracle.decode(xa, eb, bits, ch)[0] for xa, (eb, bits, ch) in zip(inputs, specs)]
    srcs = [torch.from_numpy(xa).cuda() for xa in inputs]
    pairs = []
    for k in range(2):
        st = torch.cuda.current_stream() if k == 0 else torch.cuda.Stream()
        dsts = [torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
                for eb, _, ch in specs]
        desc = [{"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb, "bits": bits,
                 "channels": ch} for s, d, (eb, bits, ch) in zip(srcs, dsts, specs)]
        status = torch.zeros(len(specs) * bjxa_amd.STATUS_WORDS, dtype=torch.int32,
                             device="cuda")
        pairs.append((st, dsts, bjxa_amd.Batch(desc, stream=st.cuda_stream), status))
    torch.cuda.synchronize()
    try:
        for _ in range(4):
            for st, _, batch, status in pairs:
                batch.decode(status.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        for _, dsts, _, status in pairs:
            st_w = status.cpu().numpy().view(np.uint32).reshape(len(specs), -1)
            assert (st_w[:, 0] == 0xFFFFFFFF).all()
            for d, ref in zip(dsts, refs):
                assert np.array_equal(d.cpu().numpy().view(np.int16), ref)
    finally:
        for _, _, batch, _ in pairs:
            batch.close()
