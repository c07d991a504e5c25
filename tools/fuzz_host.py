"""Randomised parity soak of the unchanged host API (bjxa.h) against the
oracle, for `--seconds`: bjxa_decode on host buffers with streams of 1 ..
2.5M eblocks (log-uniform, capped where one header's data length must stay
under 2^27; so every route is drawn: the library's CPU core
for small calls, the serial GPU route, the duplex route from 64 MiB of
PCM), any format, header entry state and cut sample count, the stream fed
in 1-4 calls split at random eblocks (state carried between calls, as the
reference's callers do, src/bjxa_decode.c:56-100) and, in one round of
four, an invalid profile byte (EPROTO at that eblock, src/libbjxa.c:550;
nothing written past it); and bjxa_encode of random PCM.  Prints one JSON
line; exit status 1 on any mismatch.

usage: python tools/fuzz_host.py [--seconds 120] [--seed 1]
"""
import argparse
import errno
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def decode_round(rng, stats, max_eb=2_500_000):
    bits = int(rng.choice([4, 6, 8]))
    ch = int(rng.integers(1, 3))
    eb = max(1, int(np.exp(rng.uniform(0, np.log(max_eb)))))
    mix = ["A", "W", "F", "Z"][int(rng.integers(0, 4))]
    bx = (bits * 4 + 1) * ch
    eb = min(eb, ((1 << 27) - 1) // bx)     # one XA header's data_len < 2^27
    xa = synth.stream(eb, bits, ch, mix, seed=int(rng.integers(0, 1 << 30)))
    if rng.random() < 0.25:
        xa = xa.copy()
        j, c = int(rng.integers(0, eb)), int(rng.integers(0, ch))
        xa[j * bx + c * (bits * 4 + 1)] = 0x50 | int(rng.integers(0, 16))
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4)) if rng.random() < 0.5 \
        else (0, 0, 0, 0)
    frames = eb * 32 - (int(rng.integers(0, 32)) if rng.random() < 0.3 else 0)
    ref, _, done, badc = oracle.decode(xa, eb, bits, ch, state, frames)
    k = int(rng.integers(0, 4))
    cuts = sorted(set(int(v) for v in rng.integers(1, eb, k))) if eb > 1 else []
    bounds = [0] + cuts + [eb]
    out = np.full(eb * 64 * ch + 64, 0x3C, np.uint8)
    hdr = bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch, state)
    if os.environ.get("FUZZ_LOG"):
        print("decode bits=%d ch=%d eb=%d mix=%s frames=%d bounds=%s bad=%d" % (
            bits, ch, eb, mix, frames, bounds, badc), file=sys.stderr, flush=True)
    why = None
    failed = False
    with bjxa_amd.Decoder() as d:
        d.parse_header(hdr)
        for e0, e1 in zip(bounds, bounds[1:]):
            try:
                n = d.decode(out[e0 * 64 * ch:e1 * 64 * ch], xa[e0 * bx:e1 * bx].copy())
            except bjxa_amd.BjxaError as e:
                if badc < 0 or e.errno != errno.EPROTO or not e0 <= done < e1:
                    why = "unexpected %r in [%d, %d)" % (e, e0, e1)
                failed = True
                break
            if n != e1 - e0:
                why = "count %d != %d" % (n, e1 - e0)
                break
    if why is None and badc >= 0 and not failed:
        why = "no EPROTO"
    if why is None:
        n = (done if badc >= 0 else eb) * 32 * ch
        n = min(n, frames * ch)
        if not np.array_equal(out[:2 * n].view(np.int16), ref[:n]):
            why = "pcm"
        elif not (out[2 * n:] == 0x3C).all():
            why = "bytes past the output"
    stats["decode_calls"] += len(bounds) - 1
    stats["decode_streams"] += 1
    stats["eblocks"] += eb
    stats["eproto"] += badc >= 0
    route = "cpu" if eb <= 64 else "duplex" if eb * 64 * ch >= (64 << 20) else "gpu"
    stats["by_size"][route] = stats["by_size"].get(route, 0) + 1
    return None if why is None else {"why": why, "bits": bits, "ch": ch, "eb": eb, "mix": mix,
                                     "frames": frames, "bounds": bounds[:6], "bad": badc}


def encode_round(rng, stats, max_frames=64_000_000):
    bits = int(rng.choice([4, 6, 8]))
    ch = int(rng.integers(1, 3))
    # (at least one block of PCM: the reference's bjxa_encode wants a whole
    # block of source, src/libbjxa.c:778, ENOBUFS below it)
    frames = max(32, int(np.exp(rng.uniform(np.log(32), np.log(max_frames // ch)))))
    pcm = synth.pcm(frames, ch, seed=int(rng.integers(0, 1 << 30)))
    if os.environ.get("FUZZ_LOG"):
        print("encode bits=%d ch=%d frames=%d" % (bits, ch, frames), file=sys.stderr,
              flush=True)
    e = bjxa_amd.Encoder()
    try:
        fmt = e.init({"data_len_pcm": frames * 2 * ch, "blocks": 0, "block_size_pcm": 0,
                      "block_size_xa": 0, "samples_rate": 44100, "sample_bits": 16,
                      "channels": ch}, bits)
        n = fmt["blocks"] * fmt["block_size_xa"]
        buf = np.full(n + 64, 0xA5, np.uint8)
        got = e.encode(buf[:n], pcm.view(np.uint8))
    finally:
        e.close()
    stats["encode_streams"] += 1
    why = None
    if got != fmt["blocks"]:
        why = "count"
    elif not np.array_equal(buf[:n], oracle.encode(pcm, frames, bits, ch)):
        why = "xa"
    elif not (buf[n:] == 0xA5).all():
        why = "bytes past the output"
    return None if why is None else {"why": why, "bits": bits, "ch": ch, "frames": frames}


def new_stats():
    return {"decode_streams": 0, "decode_calls": 0, "eblocks": 0, "eproto": 0,
            "encode_streams": 0, "by_size": {}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    stats = new_stats()
    bad = []
    deadline = time.monotonic() + args.seconds
    tick = time.monotonic() + 30
    while time.monotonic() < deadline:
        if time.monotonic() > tick:         # (a progress line every 30 s)
            tick += 30
            print("progress", json.dumps(stats), file=sys.stderr, flush=True)
        r = decode_round(rng, stats) if rng.random() < 0.75 else encode_round(rng, stats)
        if r is not None:
            bad.append(r)
    print(json.dumps({"seconds": args.seconds, "seed": args.seed, **stats,
                      "mismatches": len(bad), "first": bad[:5]}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
