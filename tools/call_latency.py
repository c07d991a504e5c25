"""Per-call cost of the host API, CPU core against GPU, by call size:
bjxa_decode()/bjxa_encode() with n effective blocks per call, the reference
CLI's default incremental shape being n = 1 (src/bjxa_decode.c:102-155).
The crossover sizes set the default offload thresholds (libbjxa.c,
DESIGN.md §1 "Routing").

usage: python tools/call_latency.py [--quick]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

import bjxa_amd  # noqa: E402
from bjxa_amd import synth  # noqa: E402

SIZES = (1, 4, 16, 64, 256, 512, 1024, 2048, 4096, 8192, 16384, 65536)


def time_decode(n, bits, ch, route):
    calls = max(5, min(2000, 400000 // n))
    eb = n * calls
    bx = (bits * 4 + 1) * ch
    xa = synth.stream(eb, bits, ch, "A", seed=9)
    hdr = bjxa_amd.xa_header(len(xa), eb * 32, 44100, bits, ch)
    dst = np.empty(n * 64 * ch, dtype=np.uint8)
    pieces = [xa[i * n * bx:(i + 1) * n * bx].copy() for i in range(calls)]
    with bjxa_amd.offload(0 if route == "gpu" else None), bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        d.decode(dst, pieces[0])            # first call: device setup
        t = time.perf_counter()
        for p in pieces[1:]:
            d.decode(dst, p)
        return (time.perf_counter() - t) / (calls - 1)


def time_encode(n, bits, ch, route):
    calls = max(5, min(2000, 400000 // n))
    frames = n * 32 * calls
    pcm = synth.pcm(frames, ch, seed=3)
    bp = 64 * ch
    raw = pcm.view(np.uint8)
    pieces = [raw[i * n * bp:(i + 1) * n * bp].copy() for i in range(calls)]
    dst = np.empty(n * (bits * 4 + 1) * ch, dtype=np.uint8)
    with bjxa_amd.offload(0 if route == "gpu" else None):
        e = bjxa_amd.Encoder()
        e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                "block_size_xa": 0, "samples_rate": 8000, "sample_bits": 16,
                "channels": ch}, bits)
        e.encode(dst, pieces[0])
        t = time.perf_counter()
        for p in pieces[1:]:
            e.encode(dst, p)
        dt = (time.perf_counter() - t) / (calls - 1)
        e.close()
    return dt


def main():
    import torch  # noqa: F401  (one HIP runtime with the library)
    sizes = SIZES[::2] if "--quick" in sys.argv else SIZES
    out = {"decode": {}, "encode": {}}
    for what, fn in (("decode", time_decode), ("encode", time_encode)):
        for bits, ch in ((8, 2), (8, 1), (4, 1)):
            key = "%d-bit %s" % (bits, "stereo" if ch == 2 else "mono")
            rows = {}
            for n in sizes:
                row = {}
                for route in ("cpu", "gpu"):
                    dt = fn(n, bits, ch, route)
                    row[route + "_us"] = round(dt * 1e6, 2)
                    row[route + "_MSps"] = round(n * 32 * ch / dt / 1e6, 1)
                rows[str(n)] = row
                print(what, key, n, row, flush=True)
            out[what][key] = rows
    print(json.dumps(out))


if __name__ == "__main__":
    main()
