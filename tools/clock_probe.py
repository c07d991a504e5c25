"""Is a decode after an idle host pause slower because the GPU clock dropped?
(R5-2's clock-state claim had no clock
reading behind it.)

One process, bench.py's C3 stream (slot 0: same seed, same buffers).  A
one-wave probe kernel (tools/clock_probe.hip) reads the shader clock --
s_memtime against the 100 MHz s_memrealtime over `--ticks` ticks -- on the
decode stream.  Interleaved over --rounds rounds:

  hot        ten decodes back to back, then the probe (the clock right
             after sustained decoding), then one decode timed by hipEvents
             around K1 and by host wall time (call .. synchronize)
  cold       synchronize, sleep --pause ms, the probe (the clock after the
             pause), then one decode timed the same way, then the probe
  cold_bare  synchronize, sleep --pause ms, one decode timed the same way
             with no probe before it (what one bjxa(1) call on an idle GPU
             sees, less the copies)

Prints one JSON object: per mode the median and range of MHz, K1 ms (event)
and step ms (wall).

usage: python tools/clock_probe.py [--rounds 10] [--pause 10] [--ticks 500]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
import bench  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def stats(v):
    v = sorted(v)
    return {"median": round(v[len(v) // 2], 4), "min": round(v[0], 4), "max": round(v[-1], 4),
            "n": len(v)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--pause", type=float, default=10.0, help="idle host pause, ms")
    ap.add_argument("--ticks", type=int, default=500, help="probe length, 100 MHz ticks")
    ap.add_argument("--mix", default="A")
    args = ap.parse_args()
    so = os.path.join(ROOT, "tools", "bin", "clock_probe.so")
    probe = ctypes.CDLL(so)
    probe.clk_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]

    eb, bits, ch = 5_000_000, 8, 2
    dev = torch.device("cuda", 0)
    xa = synth.stream(eb, bits, ch, args.mix, seed=0)
    src = torch.from_numpy(xa).to(dev)
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
    ws_len = bjxa_amd.decode_workspace_size(eb, ch)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device=dev)
    st = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)
    clk = torch.zeros(2 * 64, dtype=torch.int64, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)
    evs = bench.EventPairs(3 * args.rounds)
    ev_it = iter(evs.ev)
    slot = [0]

    def decode(ev=(None, None)):
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, st.data_ptr(), (0, 0, 0, 0), 0, -1, sh,
                               ev)

    def clock():
        k = slot[0]
        slot[0] = (k + 1) % 64
        if probe.clk_launch(clk.data_ptr() + 16 * k, args.ticks, sh) != 0:
            raise RuntimeError("clk_launch")
        return k

    def timed_decode():
        ev = next(ev_it)
        t0 = time.perf_counter()
        decode(ev)
        torch.cuda.synchronize(dev)
        return ev, (time.perf_counter() - t0) * 1e3

    for _ in range(20):
        decode()
    torch.cuda.synchronize(dev)
    rec = {m: {"mhz_before": [], "mhz_after": [], "k1": [], "wall": []}
           for m in ("hot", "cold", "cold_bare")}
    pend = []           # (mode, key, probe slot) read after the loop
    pend_ev = []        # (mode, event pair)
    for _ in range(args.rounds):
        # hot
        for _ in range(10):
            decode()
        pend.append(("hot", "mhz_before", clock()))
        torch.cuda.synchronize(dev)     # (the GPU idles for the sync's ~50 us)
        ev, wall = timed_decode()
        pend_ev.append(("hot", ev))
        rec["hot"]["wall"].append(wall)
        # cold, with probes around the decode
        torch.cuda.synchronize(dev)
        time.sleep(args.pause / 1e3)
        pend.append(("cold", "mhz_before", clock()))
        ev, wall = timed_decode()
        pend_ev.append(("cold", ev))
        rec["cold"]["wall"].append(wall)
        pend.append(("cold", "mhz_after", clock()))
        torch.cuda.synchronize(dev)
        # cold, nothing before the decode
        time.sleep(args.pause / 1e3)
        ev, wall = timed_decode()
        pend_ev.append(("cold_bare", ev))
        rec["cold_bare"]["wall"].append(wall)
        # read the probes of this round before their slots are reused
        c = clk.cpu().numpy().reshape(64, 2)
        for m, key, k in pend:
            rec[m][key].append(float(c[k, 0]) / float(c[k, 1]) * 100.0)
        pend = []
    # the clock through a run of decodes that starts after the pause: probe
    # after every decode (3 runs of 40, median per position)
    traj = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        time.sleep(args.pause / 1e3)
        ks = []
        for _ in range(40):
            decode()
            ks.append(clock())      # (40 of the 64 slots: no reuse in a run)
        torch.cuda.synchronize(dev)
        c = clk.cpu().numpy().reshape(64, 2)
        traj.append([float(c[k, 0]) / float(c[k, 1]) * 100.0 for k in ks])
    torch.cuda.synchronize(dev)
    c = clk.cpu().numpy().reshape(64, 2)
    for m, key, k in pend:
        rec[m][key].append(float(c[k, 0]) / float(c[k, 1]) * 100.0)
    hip = evs.hip
    for m, (a, b) in pend_ev:
        f = ctypes.c_float()
        hip.hipEventElapsedTime(ctypes.byref(f), a, b)
        rec[m]["k1"].append(f.value)
    evs.close()
    out = {"what": "shader clock (s_memtime / s_memrealtime x 100 MHz) around C3 decodes, "
                   "hot vs after an idle host pause", "pause_ms": args.pause,
           "probe_ticks": args.ticks, "rounds": args.rounds, "mix": args.mix}
    for m, r in rec.items():
        out[m] = {k: stats(v) for k, v in r.items() if v}
    out["trajectory_mhz_after_decode_k"] = [round(sorted(col)[1], 1) for col in zip(*traj)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
