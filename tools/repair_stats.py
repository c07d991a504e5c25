"""How much repair work a plan leaves, computed on the CPU with the oracle
(no GPU): for every chunk of a synthetic stream, the speculative decode
(warm-up of W eblocks from state (0,0), as xa_decode.hip's K1 does) against
the true trajectory; a chunk whose entry state is wrong is repaired block by
block until a block-end state meets the speculative one (fix_chunk).
Reports the repaired chunks, the repair lengths in blocks, and per wave (64
chunks, repaired side by side by the wave's lanes) the longest repair --
the serial time a wave adds after its main loop.

usage: python tools/repair_stats.py [--eblocks 5000000] [--chunk 40]
           [--warm 8 6 4] [--mix A W F] [--bits 8] [--ch 2]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402


def block_end_states(pcm, ch):
    """frames 30/31 of every eblock, as one int64 key per eblock"""
    f = pcm.reshape(-1, 32, ch).astype(np.int64) & 0xFFFF
    k = np.zeros(f.shape[0], dtype=np.int64)
    for c in range(ch):
        k = (k << 32) | (f[:, 30, c] << 16) | f[:, 31, c]
    return k


def stats(xa, eb, bits, ch, C, W):
    ebsz = (bits * 4 + 1) * ch
    ref, _, _, _ = oracle.decode(xa, eb, bits, ch)
    true_k = block_end_states(ref, ch)
    n = (eb + C - 1) // C
    lens = np.zeros(n, dtype=np.int64)
    for q in range(1, n):
        b0, b1 = q * C, min(q * C + C, eb)
        w0 = max(0, b0 - W)
        seg = xa[w0 * ebsz:b1 * ebsz]
        pcm, _, _, _ = oracle.decode(seg, b1 - w0, bits, ch)
        k = block_end_states(pcm, ch)[b0 - w0:]
        # entry correct iff the state at the end of block b0-1 matches
        if w0 < b0:
            pk = block_end_states(pcm[:(b0 - w0) * 32 * ch], ch)[-1]
        else:
            pk = 0
        if pk == true_k[b0 - 1]:
            continue
        meet = np.nonzero(k == true_k[b0:b1])[0]
        lens[q] = (meet[0] + 1) if meet.size else (b1 - b0 + 1000)   # +1000: cascades
    rep = lens[lens > 0]
    waves = lens[:(n // 64) * 64].reshape(-1, 64).max(axis=1)
    return {"chunks": n, "repaired": int(rep.size),
            "len_mean": float(rep.mean()) if rep.size else 0.0,
            "len_p50": float(np.median(rep)) if rep.size else 0.0,
            "len_max": int(rep.max()) if rep.size else 0,
            "cascading": int((rep >= 1000).sum()),
            "blocks": int(rep[rep < 1000].sum()),
            "wave_max_mean": float(waves.mean()),
            "wave_max_p90": float(np.percentile(waves, 90)),
            "waves_with_repair": float((waves > 0).mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eblocks", type=int, default=5_000_000)
    ap.add_argument("--chunk", type=int, default=40)
    ap.add_argument("--warm", type=int, nargs="+", default=[8, 6, 4])
    ap.add_argument("--mix", nargs="+", default=["A", "W", "F"])
    ap.add_argument("--bits", type=int, default=8)
    ap.add_argument("--ch", type=int, default=2)
    args = ap.parse_args()
    for mix in args.mix:
        xa = synth.stream(args.eblocks, args.bits, args.ch, mix, seed=0)
        for w in args.warm:
            s = stats(xa, args.eblocks, args.bits, args.ch, args.chunk, w)
            print("mix %s W=%d C=%d: %s" % (mix, w, args.chunk, s), flush=True)


if __name__ == "__main__":
    main()
