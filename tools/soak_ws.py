"""Soak of one workspace reused across streams of different sizes (the
layout change of DESIGN.md §5 R6-1): `--iters` decodes through
bjxa_hip_decode_async, each of a stream drawn at random from a few sizes
and mixes, every result compared on the GPU with the oracle's PCM
(computed once per stream) and its exit state checked.

usage: python tools/soak_ws.py [--iters 400] [--seed 1]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    ch, bits = 2, 8
    shapes = [(5_000_000, "A"), (1_300_001, "W"), (700_003, "A"), (2_600_000, "F"),
              (64 * 40 * 3 + 17, "W")]
    streams = []
    for i, (eb, mix) in enumerate(shapes):
        xa = synth.stream(eb, bits, ch, mix, seed=300 + i)
        ref, st, _, _ = oracle.decode(xa, eb, bits, ch)
        streams.append({"eb": eb, "src": torch.from_numpy(xa).cuda(),
                        "ref": torch.from_numpy(ref.view(np.uint8)).cuda(),
                        "state": tuple(int(v) for v in st)})
    big = max(eb for eb, _ in shapes)
    ws_len = bjxa_amd.decode_workspace_size(big, ch, 0, -1)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    dst = torch.empty(big * 64 * ch, dtype=torch.uint8, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)
    bad, counts = [], [0] * len(streams)
    for it in range(args.iters):
        k = int(rng.integers(0, len(streams)))
        s = streams[k]
        counts[k] += 1
        eb = s["eb"]
        bjxa_amd.decode_device(s["src"].data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0), 0, -1,
                               sh)
        same = torch.equal(dst[:eb * 64 * ch], s["ref"])
        st = status.cpu().numpy().view(np.uint32)

        def split(w):
            w = int(w)
            return [int(np.int16(np.uint16(w & 0xFFFF))), int(np.int16(np.uint16(w >> 16)))]
        state = tuple(split(st[1]) + split(st[2]))
        if not same or state != s["state"]:
            bad.append((it, k))
    print(json.dumps({"iters": args.iters, "streams": [s["eb"] for s in streams],
                      "decodes_per_stream": counts, "mismatches": bad[:20],
                      "n_mismatch": len(bad)}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
