"""K1's output stage is free of LDS bank conflicts (tools/lds_banks.py
restates xa_decode.hip ost_line / ost_piece / ost_quad under the banking
rules of MI355X_MICROARCH.md §LDS), and the tool's formulas are the ones
in the kernel source."""
import os
import re
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lds_banks  # noqa: E402


def test_stage_conflict_free():
    w, r = lds_banks.stage_conflicts(lds_banks.ost_line, lds_banks.ost_piece,
                                     lds_banks.ost_quad)
    assert (w, r) == (0, 0)
    # the earlier layouts, for scale: each conflicts on one side
    assert lds_banks.stage_conflicts(*lds_banks.LAYOUTS["pitch144 (round 4)"]) == (0, 32)


def test_stage_fits_and_lines_disjoint():
    used = set()
    for j in range(64):
        for p in range(8):
            o = lds_banks.ost_line(j) + lds_banks.ost_piece(p)
            for b in range(o, o + 16):
                assert b not in used
                used.add(b)
    assert max(used) < lds_banks.ost_line(64) == 8704


def test_tool_matches_kernel_source():
    src = open(os.path.join(ROOT, "bjxa_amd", "csrc", "xa_decode.hip")).read()
    assert "0xfbae9dc873261540ull" in src
    assert re.search(r"return \(j >> 1\) \* \(2 \* XA_LB \+ 16\) \+ \(j & 1\) \* \(XA_LB / 2\);", src)
    assert "return 16 * (p + (p & 4));" in src
    kern = open(os.path.join(ROOT, "bjxa_amd", "csrc", "xa_kern.h")).read()
    assert "(qq % QL) + (qq % QL & 4)" in kern
