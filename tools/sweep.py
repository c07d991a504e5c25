"""Tuning sweep for the device decode: for each (chunk, warm-up) pair time the
speculative kernel (hipEvents on the launch stream) and the whole step, and
check bit-exactness against the oracle once per pair.

usage: python tools/sweep.py [--workload C3|C2] [--mix A] [--pairs 26:8,32:8,...]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import bjxa_amd  # noqa: E402
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402
from bench import WORKLOADS, hip_runtime  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--mix", default="A")
    ap.add_argument("--pairs", default="0:-1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--no-events", action="store_true",
                    help="time steps without the per-step hipEvent pair")
    args = ap.parse_args()
    for v in args.variants.split(","):
        run(args, int(v))


def run(args, variant):
    eb, bits, ch, _ = WORKLOADS[args.workload]
    xa = synth.stream(eb, bits, ch, args.mix, seed=0)
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch)
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(xa).to(dev)
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
    status = torch.zeros(8, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    hip = hip_runtime()
    samples = eb * 32 * ch
    alg = eb * ch * (bits * 4 + 1) + eb * 64 * ch
    for pair in args.pairs.split(","):
        chunk, warm = (int(v) for v in pair.split(":"))
        ws_len = bjxa_amd.decode_workspace_size(eb, ch, chunk, warm)
        ws = torch.zeros(ws_len, dtype=torch.uint8, device=dev)
        bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)
        evs = []
        for _ in range(args.steps + 2):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            hip.hipEventCreate(ctypes.byref(a))
            hip.hipEventCreate(ctypes.byref(b))
            evs.append((a.value, b.value))

        def step(i):
            bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                                   ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0),
                                   chunk, warm, sh,
                                   (None, None) if args.no_events else evs[i], variant)
        step(0)
        step(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(2, args.steps + 2):
            step(i)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        ms = []
        for a, b in ([] if args.no_events else evs[2:]):
            f = ctypes.c_float()
            hip.hipEventElapsedTime(ctypes.byref(f), a, b)
            ms.append(f.value)
        spec = float(np.mean(ms)) if ms else float("nan")
        st = status.cpu().numpy().view(np.uint32)
        ok = bool(np.array_equal(dst.cpu().numpy().view(np.int16), ref))
        print(json.dumps({"workload": args.workload, "mix": args.mix, "variant": variant, "chunk": chunk,
                          "warm": warm, "chunks": int(st[5]), "step_ms": round(dt * 1e3, 4),
                          "spec_ms": round(spec, 4),
                          "spec_GBs": round(alg / spec / 1e6, 1),
                          "MSps": round(samples / dt / 1e6, 1),
                          "repaired": int(st[3]), "tail": int(st[4]), "exact": ok}), flush=True)
        for a, b in evs:
            hip.hipEventDestroy(a)
            hip.hipEventDestroy(b)
        del ws


if __name__ == "__main__":
    main()
