"""Threading contract of the C API (reference bjxa.3.rst.in:278-283): a
codec is not MT-safe, but separate codecs on separate threads are.  Eight
threads each drive their own decoder (and encoder) through calls of mixed
sizes -- small ones on the CPU core, large ones on the GPU under the
default routing, or all on the GPU -- and every stream must equal the
oracle bit for bit."""
import threading

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth

pytestmark = pytest.mark.gpu

FORMATS = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1), (8, 2), (4, 1)]


def decode_job(i, results):
    bits, ch = FORMATS[i % len(FORMATS)]
    rng = np.random.default_rng(1000 + i)
    sizes = [int(v) for v in rng.integers(1, 6000, 12)] + [1, 3, 40000]
    eb = sum(sizes)
    frames = eb * 32 - i
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4))
    xa = synth.stream(eb, bits, ch, "AW"[i & 1], seed=500 + i)
    bx = (bits * 4 + 1) * ch
    out = bytearray()
    with bjxa_amd.Decoder() as d:
        d.parse_header(bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state))
        pos, left = 0, frames * ch * 2
        for n in sizes:
            dst = np.zeros(n * 64 * ch, np.uint8)
            assert d.decode(dst, xa[pos * bx:(pos + n) * bx].copy()) == n
            take = min(n * 64 * ch, left)
            out += dst[:take].tobytes()
            left -= take
            pos += n
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch, state, frames)
    results[i] = bytes(out) == ref.tobytes()


def encode_job(i, results):
    bits, ch = FORMATS[i % len(FORMATS)]
    frames = 32 * 30000 + i
    pcm = synth.pcm(frames, ch, seed=700 + i)
    e = bjxa_amd.Encoder()
    try:
        fmt = e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                      "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                      "channels": ch}, bits)
        raw = pcm.tobytes()
        bp, bx = fmt["block_size_pcm"], fmt["block_size_xa"]
        out, pos = bytearray(), 0
        for n in (1, 7, 20000, 1000, fmt["blocks"]):
            n = min(n, fmt["blocks"] - pos)
            if n == 0:
                break
            chunk = np.frombuffer(raw[pos * bp:(pos + n) * bp].ljust(n * bp, b"\0"),
                                  np.uint8).copy()
            dst = np.zeros(n * bx, np.uint8)
            assert e.encode(dst, chunk) == n
            out += dst.tobytes()
            pos += n
    finally:
        e.close()
    results[100 + i] = bytes(out) == oracle.encode(pcm, frames, bits, ch).tobytes()


def run_threads(n):
    results = {}
    ths = [threading.Thread(target=decode_job, args=(i, results)) for i in range(n)]
    ths += [threading.Thread(target=encode_job, args=(i, results)) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=240)
    return results


@pytest.mark.routing
def test_eight_codecs_default_routing(built):
    res = run_threads(8)
    assert len(res) == 16 and all(res.values()), res


def test_eight_codecs_all_gpu(built):
    res = run_threads(8)
    assert len(res) == 16 and all(res.values()), res
