"""Localise decode mismatches: per (bits, ch, mix, tuning) report how many
samples differ from the oracle and where the first ones are."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402,F401
import oracle  # noqa: E402
from bjxa_amd import synth  # noqa: E402
from gpu_util import dev_decode  # noqa: E402


def run(bits, ch, mix, eb, chunk, warmup):
    xa = synth.stream(eb, bits, ch, mix, seed=1)
    ref, st_ref, _, _ = oracle.decode(xa, eb, bits, ch)
    got, st = dev_decode(xa, eb, bits, ch, chunk=chunk, warmup=warmup, want_status=True)
    bad = np.nonzero(got != ref)[0]
    msg = "bits=%d ch=%d mix=%s eb=%d C=%d W=%d: mismatches=%d status=%s" % (
        bits, ch, mix, eb, chunk, warmup, bad.size, [hex(int(v)) for v in st[:6]])
    if bad.size:
        i = bad[:8]
        fr = i // ch
        msg += "\n   first idx %s\n   eblock %s frame %s chan %s\n   got %s\n   ref %s" % (
            i.tolist(), (fr // 32).tolist(), (fr % 32).tolist(), (i % ch).tolist(),
            got[i].tolist(), ref[i].tolist())
        eblk = np.unique(bad // ch // 32)
        msg += "\n   bad eblocks: n=%d first %s" % (eblk.size, eblk[:20].tolist())
    print(msg, flush=True)


if __name__ == "__main__":
    for bits in (8, 4, 6):
        for ch in (1, 2):
            run(bits, ch, "Z", 64, 16, 0)
            run(bits, ch, "Z", 4096, 16, 8)
            run(bits, ch, "A", 64, 64, 0)
            run(bits, ch, "A", 4096, 16, 64)
            run(bits, ch, "A", 4096, 16, 8)
