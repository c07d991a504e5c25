"""Per-wave timeline of the speculative kernel (K1) on C3 from a
diagnostic build with -DXA_DBG_TIMES: start, end of warm-up and end of
every wave (s_memrealtime, 100 MHz) and its XCD/SE/CU.  Prints the spread
of starts and ends, the warm-up phase, and per-XCD end times: how much of
the kernel is start-up, steady streaming and tail.

usage: make -C bjxa_amd/csrc OUT=$PWD/dbg/times OBJ=$PWD/dbg/times/build EXTRA=-DXA_DBG_TIMES
       BJXA_LIB_PATH=dbg/times/libbjxa.so.0 python tools/wave_times.py [C3|C2] [mix]
           [variant] [tag]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "C3"
    mix = sys.argv[2] if len(sys.argv) > 2 else "A"
    variant = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0
    tag = sys.argv[4] if len(sys.argv) > 4 else ""
    eb, ch = (5_000_000, 2) if wl == "C3" else (10_000_000, 1)
    xa = synth.stream(eb, 8, ch, mix, seed=0)
    src = torch.from_numpy(xa).cuda()
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
    ws_len = bjxa_amd.decode_workspace_size(eb, ch, variant=variant)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    st = torch.zeros(8, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)
    out = []
    for it in range(6):
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, 8, ch,
                               ws.data_ptr(), ws_len, st.data_ptr(), stream=sh,
                               variant=variant)
        torch.cuda.synchronize()
        s = st.cpu().numpy().view(np.uint32)
        nch = int(s[5])
        nw = (nch + 63) // 64
        q0 = 256 + 16 * nch + 4 * nch
        rec = ws[q0:q0 + 16 * nw].cpu().numpy().view(np.uint32).reshape(nw, 4).astype(np.int64)
        t0 = rec[:, 0].min()
        start, warm, end = (rec[:, 0] - t0) / 100.0, (rec[:, 1] - t0) / 100.0, \
            (rec[:, 2] - t0) / 100.0      # microseconds
        xcc = rec[:, 3] >> 16
        if it < 2:
            continue
        np.save(os.path.join(ROOT, "gpurun_out", "wt_%s_%s%s_%d.npy" % (wl, mix, tag, it)), rec)
        r = {"waves": nw, "kernel_us": float(end.max()),
             "start_pct": [float(np.percentile(start, p)) for p in (0, 50, 90, 100)],
             "warm_end_pct": [float(np.percentile(warm, p)) for p in (0, 50, 90, 100)],
             "end_pct": [float(np.percentile(end, p)) for p in (0, 10, 50, 90, 100)],
             "per_xcd_end_max": [float(end[xcc == x].max()) for x in range(8)],
             "per_xcd_end_med": [float(np.median(end[xcc == x])) for x in range(8)],
             "per_xcd_waves": [int((xcc == x).sum()) for x in range(8)],
             "per_xcd_dur_med": [float(np.median((end - start)[xcc == x])) for x in range(8)],
             # dispatch: the XCD that workgroup b lands on, by b % 8
             "xcd_of_block_mod8": [int(np.bincount(xcc[(np.arange(nw) // 4) % 8 == m],
                                                   minlength=8).argmax()) for m in range(8)],
             "block_mod8_match": float(np.mean(xcc == ((np.arange(nw) // 4) % 8))),
             "dur_pct": [float(np.percentile(end - start, p)) for p in (0, 50, 100)]}
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
