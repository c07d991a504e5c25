"""Per-call cost of the host API for small calls: bjxa_decode() with
n effective blocks per call (the reference CLI's default incremental shape
is n = 1, src/bjxa_decode.c:102-155), on 8-bit stereo.

usage: python tools/call_latency.py
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


def main():
    out = {}
    for n in (1, 16, 256, 4096, 65536):
        calls = max(20, min(2000, 200000 // n))
        eb = n * calls
        xa = synth.stream(eb, 8, 2, "A", seed=9)
        hdr = bjxa_amd.xa_header(len(xa), eb * 32, 44100, 8, 2)
        dst = np.empty(n * 128, dtype=np.uint8)
        with bjxa_amd.Decoder() as d:
            d.parse_header(hdr)
            d.decode(dst, xa[:n * 66])            # first call: device setup
            t = time.perf_counter()
            for i in range(1, calls):
                d.decode(dst, xa[i * n * 66:(i + 1) * n * 66])
            dt = (time.perf_counter() - t) / (calls - 1)
        out[str(n)] = {"us_per_call": round(dt * 1e6, 1),
                       "MSamples_per_s": round(n * 64 / dt / 1e6, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
