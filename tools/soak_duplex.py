"""Soak of the duplex route from several threads at once: each thread
decodes, through its own codec, streams drawn at random from a few shapes
into outputs placed at random (reused, fresh, 2-B offset, or the thread's
own region of one shared buffer, next to its neighbours' regions within a
page, so calls' registrations overlap), for
`--seconds`; every result is compared with the oracle's PCM (computed once
per stream).  Prints one JSON line; exit status 1 on any mismatch or error.

usage: python tools/soak_duplex.py [--threads 4] [--seconds 60] [--seed 1]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402

SLAB = 16 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    shapes = [(8, 2, 4 * (SLAB // 128) + 17, "A"), (8, 1, 4 * (SLAB // 64) + 3, "W"),
              (4, 2, 5 * (SLAB // 128) + 999, "F"), (6, 1, 4 * (SLAB // 64) + 1, "A")]
    streams = []
    for i, (bits, ch, eb, mix) in enumerate(shapes):
        xa = synth.stream(eb, bits, ch, mix, seed=500 + i)
        frames = eb * 32 - (i % 3)
        ref = oracle.decode(xa, eb, bits, ch, (0, 0, 0, 0), frames)[0]
        streams.append((xa, eb, bits, ch, frames, ref))
    # one shared buffer: thread t's region starts 1,000 B after t-1's ends
    big = max(eb * 64 * ch for _, eb, _, ch, _, _ in streams)
    shared = np.zeros(args.threads * (big + 1000) + 4096, np.uint8)
    lock = threading.Lock()
    stats = {"calls": 0, "bad": [], "errors": [], "by_place": {}}
    deadline = time.monotonic() + args.seconds

    def worker(t):
        rng = np.random.default_rng(args.seed * 100 + t)
        reused = np.zeros(big + 64, np.uint8)
        with bjxa_amd.Decoder() as d:
            while time.monotonic() < deadline:
                k = int(rng.integers(0, len(streams)))
                xa, eb, bits, ch, frames, ref = streams[k]
                n = eb * 64 * ch
                place = ["reused", "fresh", "offset", "shared"][int(rng.integers(0, 4))]
                if place == "reused":
                    dst = reused[:n]
                elif place == "fresh":
                    dst = np.empty(n, np.uint8)
                elif place == "offset":
                    dst = reused[2:2 + n]
                else:
                    o = 1000 + t * (big + 1000)
                    dst = shared[o:o + n]
                try:
                    d.parse_header(bjxa_amd.xa_header(xa.size, frames, 44100, bits, ch))
                    got = d.decode(dst, xa)
                    ok = got == eb and np.array_equal(dst[:frames * 2 * ch].view(np.int16), ref)
                except Exception as e:          # reported below
                    with lock:
                        stats["errors"].append("%d %s %r" % (t, place, e))
                    continue
                with lock:
                    stats["calls"] += 1
                    stats["by_place"][place] = stats["by_place"].get(place, 0) + 1
                    if not ok:
                        stats["bad"].append((t, k, place))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(args.threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    print(json.dumps({"threads": args.threads, "seconds": args.seconds,
                      "calls": stats["calls"], "by_place": stats["by_place"],
                      "mismatches": stats["bad"][:20], "errors": stats["errors"][:10]}))
    return 1 if stats["bad"] or stats["errors"] else 0


if __name__ == "__main__":
    sys.exit(main())
