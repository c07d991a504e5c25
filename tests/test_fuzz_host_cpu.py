"""A short, seeded run of tools/fuzz_host.py's rounds in the CPU suite:
without a GPU every host call runs on the library's CPU core, so this is
random shapes (formats, split calls, header states, cut sample counts,
invalid profile bytes, encodes) through the unchanged bjxa.h API against
the oracle.  The GPU box runs the full tool (profiles/r06_fuzz_host.txt)."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location(
        "fuzz_host", os.path.join(ROOT, "tools", "fuzz_host.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_fuzz_host_rounds(built):
    f = _tool()
    rng = np.random.default_rng(2024)
    stats = f.new_stats()
    bad = []
    for i in range(60):
        r = f.decode_round(rng, stats, max_eb=20_000) if i % 4 else \
            f.encode_round(rng, stats, max_frames=400_000)
        if r is not None:
            bad.append(r)
    assert not bad, bad[:3]
    assert stats["eproto"] > 0 and stats["encode_streams"] > 0
