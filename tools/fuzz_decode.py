"""Randomised parity soak of the device decode entry points against the
oracle, for `--seconds`: each round is either one stream through
bjxa_hip_decode_async or a batch through bjxa_hip_batch_*, with the
format (4/6/8 bits, mono/stereo), length (1 .. 1.5M eblocks, log-uniform),
profile mix, entry state, cut last block, manual chunk/warm-up tuning and,
in one round of four, an invalid profile byte (gain nibble >= 5) drawn at
random.  Checked per stream: the status's first failing channel block
(the reference's EPROTO point, src/libbjxa.c:550), the PCM before it (all
of it when none fails), and the exit state when none fails.  Prints one
JSON line; exit status 1 on any mismatch.

usage: python tools/fuzz_decode.py [--seconds 120] [--seed 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402

MIXES = ["A", "W", "F", "Z"]


def draw_stream(rng, max_eb):
    bits = int(rng.choice([4, 6, 8]))
    ch = int(rng.integers(1, 3))
    eb = int(np.exp(rng.uniform(0, np.log(max_eb))))
    eb = max(1, eb)
    mix = MIXES[int(rng.integers(0, len(MIXES)))]
    xa = synth.stream(eb, bits, ch, mix, seed=int(rng.integers(0, 1 << 30)))
    bx = bits * 4 + 1
    bad = None
    if rng.random() < 0.25:
        j = int(rng.integers(0, eb))
        c = int(rng.integers(0, ch))
        xa = xa.copy()
        xa[(j * ch + c) * bx] = 0x50 | int(rng.integers(0, 16))
        bad = (j, c)
    state = tuple(int(v) for v in rng.integers(-32768, 32768, 4)) if rng.random() < 0.5 \
        else (0, 0, 0, 0)
    frames = eb * 32 - (int(rng.integers(0, 32)) if rng.random() < 0.3 else 0)
    return {"bits": bits, "ch": ch, "eb": eb, "mix": mix, "xa": xa, "state": state,
            "frames": frames, "bad": bad}


def expect(s):
    ref, st, done, badc = oracle.decode(s["xa"], s["eb"], s["bits"], s["ch"], s["state"],
                                        s["frames"])
    err = 0xFFFFFFFF if badc < 0 else done * s["ch"] + badc
    return ref, st, done, err


def check(s, got_pcm, words, exp):
    ref, st, done, err = exp
    ch = s["ch"]
    if int(words[0]) != err:
        return "err %d != %d" % (int(words[0]), err)
    n = (done * 32 if err != 0xFFFFFFFF else s["frames"]) * ch
    n = min(n, s["frames"] * ch)
    if not np.array_equal(got_pcm[:n], ref[:n]):
        return "pcm"
    if err == 0xFFFFFFFF:
        def split(w):
            return [int(np.int16(np.uint16(w & 0xFFFF))), int(np.int16(np.uint16(w >> 16)))]
        gs = split(int(words[1])) + split(int(words[2]))
        if ch == 1:
            gs = gs[:2] + list(st[2:])
        if tuple(gs) != tuple(st):
            return "state %s != %s" % (gs, st)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    sh = torch.cuda.current_stream().cuda_stream
    W = bjxa_amd.STATUS_WORDS
    stats = {"single": 0, "batch_streams": 0, "batches": 0, "with_bad": 0, "eblocks": 0}
    bad_cases = []
    deadline = time.monotonic() + args.seconds
    tick = time.monotonic() + 30
    while time.monotonic() < deadline:
        if time.monotonic() > tick:         # (a progress line every 30 s)
            tick += 30
            print("progress", json.dumps(stats), file=sys.stderr, flush=True)
        if rng.random() < 0.5:
            s = draw_stream(rng, 1_500_000)
            G = 8 // s["ch"]
            chunk = 0 if rng.random() < 0.6 else int(rng.integers(4, 64)) * G
            warm = -1 if rng.random() < 0.6 else int(rng.choice([0, 4, 8, 16, 24]))
            exp = expect(s)
            src = torch.from_numpy(s["xa"]).cuda()
            dst = torch.zeros(s["eb"] * 64 * s["ch"] + 16, dtype=torch.uint8, device="cuda")
            n = bjxa_amd.decode_workspace_size(s["eb"], s["ch"], chunk, warm)
            ws = torch.zeros(n, dtype=torch.uint8, device="cuda")
            bjxa_amd.workspace_init(ws.data_ptr(), n, sh)
            st = torch.zeros(W, dtype=torch.int32, device="cuda")
            bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), s["eb"], s["frames"],
                                   s["bits"], s["ch"], ws.data_ptr(), n, st.data_ptr(),
                                   s["state"], chunk, warm, sh)
            torch.cuda.synchronize()
            got = dst.cpu().numpy()[:s["frames"] * s["ch"] * 2].view(np.int16)
            why = check(s, got, st.cpu().numpy().view(np.uint32), exp)
            stats["single"] += 1
            stats["eblocks"] += s["eb"]
            stats["with_bad"] += s["bad"] is not None
            if why:
                bad_cases.append({"kind": "single", "why": why, "chunk": chunk, "warm": warm,
                                  **{k: s[k] for k in ("bits", "ch", "eb", "mix", "state",
                                                       "frames", "bad")}})
        else:
            k = int(rng.integers(2, 65))
            ss = [draw_stream(rng, 40_000) for _ in range(k)]
            exps = [expect(s) for s in ss]
            srcs = [torch.from_numpy(s["xa"]).cuda() for s in ss]
            dsts = [torch.zeros(s["eb"] * 64 * s["ch"] + 16, dtype=torch.uint8, device="cuda")
                    for s in ss]
            st = torch.zeros(W * k, dtype=torch.int32, device="cuda")
            with bjxa_amd.Batch([{"d_src": a.data_ptr(), "d_dst": b.data_ptr(),
                                  "eblocks": s["eb"], "bits": s["bits"],
                                  "channels": s["ch"], "frames": s["frames"],
                                  "state": s["state"]}
                                 for a, b, s in zip(srcs, dsts, ss)], stream=sh) as b:
                b.decode(st.data_ptr(), sh)
                torch.cuda.synchronize()
            words = st.cpu().numpy().view(np.uint32).reshape(k, W)
            stats["batches"] += 1
            for i, (s, d, e) in enumerate(zip(ss, dsts, exps)):
                got = d.cpu().numpy()[:s["frames"] * s["ch"] * 2].view(np.int16)
                why = check(s, got, words[i], e)
                stats["batch_streams"] += 1
                stats["eblocks"] += s["eb"]
                stats["with_bad"] += s["bad"] is not None
                if why:
                    bad_cases.append({"kind": "batch", "why": why, "index": i, "of": k,
                                      **{kk: s[kk] for kk in ("bits", "ch", "eb", "mix",
                                                              "state", "frames", "bad")}})
    print(json.dumps({"seconds": args.seconds, "seed": args.seed, **stats,
                      "mismatches": len(bad_cases), "first": bad_cases[:5]}))
    return 1 if bad_cases else 0


if __name__ == "__main__":
    sys.exit(main())
