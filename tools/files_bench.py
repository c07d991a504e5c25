"""File-to-file throughput of bjxa_hip_decode_files on a C4-shaped set:
1024 XA files in host memory (bits (4,6,8)[i%3], channels 1+((i/3)&1),
16,384 effective blocks each) -> 1024 WAV files in host memory, one call.
PCIe-inclusive by construction.  Median of 5 calls after a discarded first;
every WAV checked against the oracle once.

usage: python tools/files_bench.py [--files N] [--calls K]
           [--libs label=path ...]   (interleaved A/B of library builds:
                                      one call of each per round, in one
                                      process; median per build)
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

import bjxa_amd  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1024)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--libs", nargs="*", default=None)
    args = ap.parse_args()
    files, samples = [], 0
    for i in range(args.files):
        bits, ch, eb = (4, 6, 8)[i % 3], 1 + ((i // 3) & 1), 16384
        xa = synth.stream(eb, bits, ch, "A", seed=1000 + i)
        files.append(bjxa_amd.xa_header(xa.size, eb * 32, 44100, bits, ch) + xa.tobytes())
        samples += eb * 32 * ch
    n = len(files)
    bufs = [ctypes.create_string_buffer(f, len(f)) for f in files]
    outs = [ctypes.create_string_buffer(44 + (len(f) - 32) * 64 //
                                        (bjxa_amd.parse_header_fields(f)["bits"] * 4 + 1))
            for f in files]
    xa_p = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
    xa_l = (ctypes.c_size_t * n)(*[len(f) for f in files])
    wv_p = (ctypes.c_void_p * n)(*[ctypes.addressof(o) for o in outs])
    wv_l = (ctypes.c_size_t * n)(*[len(o) for o in outs])
    st = (ctypes.c_int * n)()
    if args.libs:
        libs = [(lab, ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL))
                for lab, path in (x.split("=", 1) for x in args.libs)]
    else:
        libs = [("new", bjxa_amd.lib())]
    import oracle
    want = [oracle.decode_file(f) for f in files]
    times = {lab: [] for lab, _ in libs}
    ok = {}
    for r in range(args.calls + 1):
        for lab, L in libs:
            for o in outs:
                ctypes.memset(o, 0, len(o))
            t = time.perf_counter()
            done = L.bjxa_hip_decode_files(xa_p, xa_l, wv_p, wv_l, st, n)
            times[lab].append(time.perf_counter() - t)
            assert done == n, (lab, done, list(st)[:8])
            if r == 0:
                ok[lab] = all(o.raw == w for o, w in zip(outs, want))
    moved = sum(len(f) for f in files) + sum(len(o) for o in outs)
    for lab, _ in libs:
        med = float(np.median(times[lab][1:]))
        print(json.dumps({"lib": lab, "files": n, "samples": samples,
                          "ms": round(med * 1e3, 2),
                          "MSamples_per_s": round(samples / med / 1e6, 1),
                          "host_GB_per_s": round(moved / med / 1e9, 2),
                          "first_call_ms": round(times[lab][0] * 1e3, 2),
                          "bit_exact": ok[lab]}))


if __name__ == "__main__":
    main()
