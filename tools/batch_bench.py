"""Batched decode throughput on the SURVEY.md §8(d) batch configs, one GPU.

  C4   1024 streams; stream i: bits (4,6,8)[i%3], channels 1+((i/3)&1),
       16,384 effective blocks each (mixed formats in one launch)
  C5g  one GPU's share of C5 at 8 GPUs: 128 streams of 8-bit stereo,
       65,536 effective blocks each (C5 = 1024 such streams over 8 GPUs)
  C5x  C5's per-GPU share at N GPUs: --streams 1024/N

Streams are seeded synthetic XA (mix A), device-resident; one step = one
bjxa_hip_batch_decode_async over all of them.  Reports MSamples/s, the spec
kernel's hipEvent time and its algorithmic HBM fraction (read + write of
every stream / time / 8 TB/s), and bit-exactness of every stream against the
oracle.

usage: python tools/batch_bench.py [--config C4|C5g] [--streams N] [--steps K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

from bench import run_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4", choices=["C4", "C5g"])
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()
    import torch
    r = run_batch(args.config, args.steps, args.warmup, torch.device("cuda", 0),
                  not args.no_verify, args.streams)
    r["config"] = args.config
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
