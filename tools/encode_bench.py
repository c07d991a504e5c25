"""Device encode throughput (bjxa_hip_encode_async, the GPU side of
bjxa_encode(), src/libbjxa.c:759-819): C3-shaped PCM (5,000,000 8-bit stereo
eblocks = 320M samples) by default.  Algorithmic bytes: PCM read (2 B per
sample) + XA written ((4*bits+1)/32 B per sample).  Byte-exact against the
oracle's encode.

usage: python tools/encode_bench.py [--bits 8] [--ch 2] [--eblocks N]
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
from bjxa_amd import synth  # noqa: E402
from bench import HBM_PEAK_GBS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--ch", type=int, default=2)
    ap.add_argument("--eblocks", type=int, default=5_000_000)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    frames = args.eblocks * 32
    pcm = synth.pcm(frames, args.ch, seed=3)
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(pcm).to(dev)
    nxa = args.eblocks * args.ch * (args.bits * 4 + 1)
    dst = torch.empty(nxa, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        bjxa_amd.encode_device(src.data_ptr(), frames, args.bits, args.ch, dst.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    s0.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bjxa_amd.encode_device(src.data_ptr(), frames, args.bits, args.ch, dst.data_ptr(), sh)
    s1.record()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / args.steps
    ms = s0.elapsed_time(s1) / args.steps
    import oracle
    ref = oracle.encode(pcm, frames, args.bits, args.ch)
    ok = bool(np.array_equal(dst.cpu().numpy(), np.frombuffer(ref, np.uint8)
                             if isinstance(ref, (bytes, bytearray)) else ref))
    alg = pcm.nbytes + nxa
    samples = frames * args.ch
    print(json.dumps({"bits": args.bits, "channels": args.ch, "eblocks": args.eblocks,
                      "step_ms": round(dt * 1e3, 4), "kernel_ms": round(ms, 4),
                      "MSamples_per_s": round(samples / dt / 1e6, 1),
                      "alg_GBs": round(alg / (ms * 1e-3) / 1e9, 1),
                      "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "byte_exact": ok}))


if __name__ == "__main__":
    main()
