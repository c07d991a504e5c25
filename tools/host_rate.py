"""PCIe-inclusive rate of the unchanged C API: bjxa_decode() on host buffers
(src/libbjxa.c:602-661 call shape, single pass), through libbjxa.so.0.

The stream is the largest one a single XA header can describe
(nDataLen < 2^27): 2,000,000 8-bit stereo eblocks or
4,000,000 8-bit mono blocks.  Reported: MSamples/s and GB/s of host bytes
moved (XA in + PCM out), median of 5 calls after a discarded first, and the
check against the oracle.

usage: python tools/host_rate.py [--ch 2|1]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--ch", type=int, default=2)
    ap.add_argument("--passes", type=int, default=5)
    ap.add_argument("--encode", action="store_true",
                    help="bjxa_encode() of the same stream's PCM instead")
    ap.add_argument("--fresh", action="store_true",
                    help="with --alt-env: a new, untouched output buffer for every call "
                         "(its page faults inside the call, as for a caller that "
                         "allocates per file)")
    ap.add_argument("--alt-env", default=None,
                    help="NAME=V1,V2: alternate this environment variable between "
                         "calls (a knob the library reads per call) and report the "
                         "median per value")
    args = ap.parse_args()
    if args.alt_env and args.encode:
        return alt_encode_rate(args)
    if args.alt_env:
        return alt_rate(args)
    if args.encode:
        return encode_rate(args)
    ch = args.ch
    eb = 2_000_000 if ch == 2 else 4_000_000
    bits = 8
    xa = synth.stream(eb, bits, ch, "A", seed=7)
    hdr = bjxa_amd.xa_header(len(xa), eb * 32, 44100, bits, ch)
    dst = np.empty(eb * 64 * ch, dtype=np.uint8)
    times = []
    with bjxa_amd.Decoder() as d:       # one codec: device buffers persist
        for i in range(args.passes + 1):
            d.parse_header(hdr)
            t = time.perf_counter()
            n = d.decode(dst, xa)
            times.append(time.perf_counter() - t)
            assert n == eb, n
    import oracle
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch)
    ok = bool(np.array_equal(dst.view(np.int16), ref))
    med = float(np.median(times[1:]))
    samples = eb * 32 * ch
    print(json.dumps({"api": "bjxa_decode (host buffers)", "bits": bits, "channels": ch,
                      "eblocks": eb, "ms": round(med * 1e3, 3),
                      "MSamples_per_s": round(samples / med / 1e6, 1),
                      "host_GB_per_s": round((len(xa) + dst.nbytes) / med / 1e9, 2),
                      "first_call_ms": round(times[0] * 1e3, 3), "bit_exact": ok}))


def alt_rate(args):
    """Decode calls alternating a per-call library knob, interleaved in one
    process (box and run drift hit every value alike)."""
    name, vals = args.alt_env.split("=", 1)
    vals = vals.split(",")
    ch = args.ch
    eb = 2_000_000 if ch == 2 else 4_000_000
    bits = 8
    xa = synth.stream(eb, bits, ch, "A", seed=7)
    hdr = bjxa_amd.xa_header(len(xa), eb * 32, 44100, bits, ch)
    import oracle
    ref = oracle.decode(xa, eb, bits, ch)[0]
    dst = np.zeros(eb * 64 * ch, dtype=np.uint8)
    times = {v: [] for v in vals}
    exact = {v: True for v in vals}
    with bjxa_amd.Decoder() as d:
        for i in range(args.passes + 1):
            for v in vals:
                os.environ[name] = v
                if args.fresh:
                    dst = np.empty(eb * 64 * ch, dtype=np.uint8)
                else:
                    dst.fill(0)
                d.parse_header(hdr)
                t = time.perf_counter()
                assert d.decode(dst, xa) == eb
                if i:
                    times[v].append(time.perf_counter() - t)
                exact[v] = exact[v] and bool(np.array_equal(dst.view(np.int16), ref))
    print(json.dumps({"api": "bjxa_decode (host buffers)", "channels": ch, "eblocks": eb,
                      "fresh_output": args.fresh, "knob": name,
                      "ms_median": {v: round(float(np.median(t)) * 1e3, 3)
                                    for v, t in times.items()},
                      "bit_exact": exact,
                      "ms_all": {v: [round(x * 1e3, 3) for x in t] for v, t in times.items()}}))


def alt_encode_rate(args):
    """bjxa_encode() calls alternating a per-call library knob, in one
    process."""
    name, vals = args.alt_env.split("=", 1)
    vals = vals.split(",")
    ch = args.ch
    eb = 2_000_000 if ch == 2 else 4_000_000
    bits, frames = 8, eb * 32
    pcm = synth.pcm(frames, ch, seed=7)
    fmt0 = {"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
            "block_size_xa": 0, "samples_rate": 44100, "sample_bits": 16, "channels": ch}
    dst = np.zeros(eb * ch * (bits * 4 + 1), np.uint8)
    import oracle
    ref = oracle.encode(pcm, frames, bits, ch)
    times = {v: [] for v in vals}
    exact = {v: True for v in vals}
    e = bjxa_amd.Encoder()
    for i in range(args.passes + 1):
        for v in vals:
            os.environ[name] = v
            dst.fill(0)
            e.init(fmt0, bits)
            t = time.perf_counter()
            assert e.encode(dst, pcm.view(np.uint8)) == eb
            if i:
                times[v].append(time.perf_counter() - t)
            exact[v] = exact[v] and bool(np.array_equal(dst, ref))
    e.close()
    print(json.dumps({"api": "bjxa_encode (host buffers)", "channels": ch, "eblocks": eb,
                      "knob": name, "ms_median": {v: round(float(np.median(t)) * 1e3, 3)
                                                  for v, t in times.items()},
                      "byte_exact": exact,
                      "ms_all": {v: [round(x * 1e3, 3) for x in t] for v, t in times.items()}}))


def encode_rate(args):
    """bjxa_encode() on host buffers: the PCM of the same largest stream
    (64M stereo / 128M mono frames) into XA, one call."""
    ch = args.ch
    eb = 2_000_000 if ch == 2 else 4_000_000
    bits, frames = 8, eb * 32
    pcm = synth.pcm(frames, ch, seed=7)
    fmt0 = {"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
            "block_size_xa": 0, "samples_rate": 44100, "sample_bits": 16, "channels": ch}
    dst = np.zeros(eb * ch * (bits * 4 + 1), np.uint8)
    times = []
    e = bjxa_amd.Encoder()         # one codec: device buffers persist
    for i in range(args.passes + 1):
        fmt = e.init(fmt0, bits)
        t = time.perf_counter()
        n = e.encode(dst, pcm.view(np.uint8))
        times.append(time.perf_counter() - t)
        assert n == fmt["blocks"] == eb, n
    e.close()
    import oracle
    ok = bool(np.array_equal(dst, oracle.encode(pcm, frames, bits, ch)))
    med = float(np.median(times[1:]))
    print(json.dumps({"api": "bjxa_encode (host buffers)", "bits": bits, "channels": ch,
                      "eblocks": eb, "ms": round(med * 1e3, 3),
                      "MSamples_per_s": round(frames * ch / med / 1e6, 1),
                      "host_GB_per_s": round((pcm.nbytes + dst.nbytes) / med / 1e9, 2),
                      "first_call_ms": round(times[0] * 1e3, 3), "byte_exact": ok}))


if __name__ == "__main__":
    main()
