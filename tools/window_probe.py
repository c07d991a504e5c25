"""Where does bench.py's timed window lose time against its own calibration?
  One process, the C3 stream of bench.py (same seed,
same buffers, slot 0), and the same 20-step loop timed five ways,
interleaved over --rounds rounds:

  plain    steps back to back, wall time between two synchronizes (what
           choose_depth's depth-1 calibration times)
  ev       the same with a hipEvent pair recorded around every step on the
           stream (what bench.py's timed_region did through round 4)
  evnf     the same with events created hipEventDisableSystemFence
  evspec   the same with the events passed into the decode (around K1
           only, what bench.py's kernel-timing pass does)
  evend    one event pair around the whole loop (no per-step events)

Prints the median ms per step of each mode (wall), and for the event modes
the median of the per-step event spans.

usage: python tools/window_probe.py [--steps 20] [--rounds 8] [--mix A]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
from bjxa_amd import synth  # noqa: E402

HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--mix", default="A")
    ap.add_argument("--eblocks", type=int, default=5_000_000)
    args = ap.parse_args()
    eb, bits, ch = args.eblocks, 8, 2
    dev = torch.device("cuda", 0)
    xa = synth.stream(eb, bits, ch, args.mix, seed=0)
    src = torch.from_numpy(xa).to(dev)
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
    ws_len = bjxa_amd.decode_workspace_size(eb, ch)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device=dev)
    st = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                        ctypes.c_void_p]

    def events(n, flags=0):
        out = []
        for _ in range(n):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            hip.hipEventCreateWithFlags(ctypes.byref(a), flags)
            hip.hipEventCreateWithFlags(ctypes.byref(b), flags)
            out.append((a.value, b.value))
        return out

    def spans(evs):
        out = []
        for a, b in evs:
            f = ctypes.c_float()
            hip.hipEventSynchronize(b)
            hip.hipEventElapsedTime(ctypes.byref(f), a, b)
            out.append(f.value)
        return out

    def step(ev=(None, None)):
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, st.data_ptr(), (0, 0, 0, 0), 0, -1,
                               sh, ev)

    ev_std = events(args.steps)
    ev_nf = events(args.steps, HIP_EVENT_DISABLE_SYSTEM_FENCE)
    ev_end = events(1)

    def run(mode):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if mode == "evend":
            hip.hipEventRecord(ev_end[0][0], sh)
        for i in range(args.steps):
            if mode == "ev":
                hip.hipEventRecord(ev_std[i][0], sh)
                step()
                hip.hipEventRecord(ev_std[i][1], sh)
            elif mode == "evnf":
                hip.hipEventRecord(ev_nf[i][0], sh)
                step()
                hip.hipEventRecord(ev_nf[i][1], sh)
            elif mode == "evspec":
                step(ev_std[i])
            else:
                step()
        if mode == "evend":
            hip.hipEventRecord(ev_end[0][1], sh)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        sp = None
        if mode in ("ev", "evspec"):
            sp = float(np.median(spans(ev_std)))
        elif mode == "evnf":
            sp = float(np.median(spans(ev_nf)))
        elif mode == "evend":
            sp = spans(ev_end)[0] / args.steps
        return wall, sp

    modes = ["plain", "ev", "evnf", "evspec", "evend"]
    for _ in range(5):
        step()
    res = {m: ([], []) for m in modes}
    for r in range(args.rounds):
        order = modes[r % len(modes):] + modes[:r % len(modes)]
        for m in order:
            w, sp = run(m)
            res[m][0].append(w)
            if sp is not None:
                res[m][1].append(sp)
    for m in modes:
        w, sp = res[m]
        print("%-7s wall %.4f ms/step (min %.4f max %.4f)%s" % (
            m, np.median(w), np.min(w), np.max(w),
            "  event span median %.4f" % np.median(sp) if sp else ""), flush=True)


if __name__ == "__main__":
    main()
