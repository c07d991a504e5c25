"""The drop-in boundary: libbjxa.so.0 exports exactly the reference's
symbols (src/libbjxa.map:16-47) plus the LIBBJXA_HIP_0.1 node, the headers
declare them, bjxa_format_t keeps its layout, and the errno contract holds
(tests/c/test_api.c mirrors test/test_libbjxa_api.c).  No GPU needed."""
import os
import re
import subprocess
import sys

import pytest

from conftest import GOLDEN, ROOT

INC = os.path.join(ROOT, "include")


def exported(path):
    out = subprocess.run(["readelf", "--dyn-syms", "-W", path], check=True,
                         capture_output=True, text=True).stdout
    syms = {}
    for line in out.splitlines():
        m = re.search(r"\bFUNC\s+GLOBAL\s+DEFAULT\s+\d+\s+(\w+)@@?([\w.]+)", line)
        if m:
            syms[m.group(1)] = m.group(2)
    return syms


def test_symbol_versions(built):
    syms = exported(built.LIB_PATH)
    want = {}
    for node, names in list(built.REFERENCE_SYMBOLS.items()) + list(built.EXTENSION_SYMBOLS.items()):
        for n in names:
            want[n] = node
    assert syms == want


def test_soname(built):
    out = subprocess.run(["readelf", "-d", built.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    assert "Library soname: [libbjxa.so.0]" in out


def test_headers_declare_every_export(built):
    text = open(os.path.join(INC, "bjxa.h")).read() + open(os.path.join(INC, "bjxa_hip.h")).read()
    declared = set(re.findall(r"\b(bjxa_\w+)\s*\(", text))
    assert declared == set(exported(built.LIB_PATH))


def test_format_layout(tmp_path):
    """bjxa_format_t: 16 bytes, offsets 0/4/8/9/10/12/13 (src/bjxa.h:24-32)."""
    src = tmp_path / "layout.c"
    src.write_text("""
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <sys/types.h>
#include "bjxa.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(bjxa_format_t),
    offsetof(bjxa_format_t, data_len_pcm), offsetof(bjxa_format_t, blocks),
    offsetof(bjxa_format_t, block_size_pcm), offsetof(bjxa_format_t, block_size_xa),
    offsetof(bjxa_format_t, samples_rate), offsetof(bjxa_format_t, sample_bits),
    offsetof(bjxa_format_t, channels));
  return 0; }""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I" + INC, "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert out == ["16", "0", "4", "8", "9", "10", "12", "13"]


def build_api_test(built, tmp_path):
    exe = tmp_path / "test_api"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I" + INC,
                    "-o", str(exe), os.path.join(ROOT, "tests", "c", "test_api.c"),
                    "-L" + os.path.dirname(built.LIB_PATH), "-l:libbjxa.so.0",
                    "-Wl,-rpath," + os.path.dirname(built.LIB_PATH), "-lz"], check=True)
    return str(exe)


def test_c_api_contract_cpu(built, manifest, tmp_path):
    """Argument/errno checks of test/test_libbjxa_api.c, and the fixture
    decoded one block per call, on a host with no GPU visible: every call
    runs on the library's CPU core."""
    import hashlib
    exe = build_api_test(built, tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    wav = tmp_path / "out.wav"
    r = subprocess.run([exe, GOLDEN, str(wav)], stdin=subprocess.DEVNULL, capture_output=True,
                       text=True, env=env)
    assert r.returncode == 0, r.stderr
    assert "test_api: ok" in r.stdout
    sha = hashlib.sha1(wav.read_bytes()).hexdigest()
    assert sha == manifest["fixtures"]["square-mono-4.xa"]["wav_sha1"]


@pytest.mark.parametrize("case", range(11))
def test_header_error_vectors(built, manifest, case):
    """test/test_decode_error.sh:32-219: every malformed header is refused
    with EPROTO by bjxa_parse_header (block-level cases need the GPU)."""
    import errno
    import bjxa_amd
    vec = manifest["header_errors"][case]
    data = bytes.fromhex(vec["hex"])
    with bjxa_amd.Decoder() as d:
        if vec["fails_in"] == "bjxa_fread_header":
            with pytest.raises(bjxa_amd.BjxaError) as ei:
                d.parse_header(data[:32])
            assert ei.value.errno == errno.EPROTO
        else:
            assert d.parse_header(data[:32]) == 32


def test_header_size_limit(built):
    """nDataLen >= 2^27 overflows 32*data_len (src/libbjxa.c:433-434)."""
    import bjxa_amd
    ok = 4067203 * 33
    with bjxa_amd.Decoder() as d:
        assert d.parse_header(bjxa_amd.xa_header(ok, ok // 33 * 32, 44100, 8, 1)) == 32
        bad = 4067204 * 33
        with pytest.raises(bjxa_amd.BjxaError):
            d.parse_header(bjxa_amd.xa_header(bad, bad // 33 * 32, 44100, 8, 1))


def test_riff_roundtrip(built, golden):
    import bjxa_amd
    wav = golden("square-stereo.wav")
    fmt = bjxa_amd.parse_riff_header(wav[:44])
    assert fmt == {"data_len_pcm": 2646000, "blocks": 0, "block_size_pcm": 0,
                   "block_size_xa": 0, "samples_rate": 44100, "sample_bits": 16,
                   "channels": 2}


BATCH_PROBE = r"""
import errno, sys
sys.path.insert(0, sys.argv[1])
import bjxa_amd
def err(streams):
    try:
        bjxa_amd.Batch(streams)
    except bjxa_amd.BjxaError as e:
        return e.errno
    return 0
ok = {"d_src": 0x10000, "d_dst": 0x20000, "eblocks": 100, "bits": 8, "channels": 2}
res = [err([]), err([dict(ok, bits=5)]), err([dict(ok, channels=3)]),
       err([dict(ok, d_dst=0x20008)]), err([dict(ok, d_src=0x10002)]),
       err([dict(ok, frames=100 * 32 + 1)]), err([dict(ok, frames=99 * 32)]),
       err([ok, dict(ok, eblocks=0)]), err([ok, dict(ok, bits=4, channels=1)])]
print(" ".join(str(r) for r in res))
"""


def test_batch_argument_checks(built):
    """bjxa_hip_batch_new validates every descriptor (EINVAL) before it
    needs the device (ENODEV without one)."""
    import errno
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", BATCH_PROBE, ROOT], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    got = [int(v) for v in r.stdout.split()]
    assert got == [errno.EINVAL] * 8 + [errno.ENODEV], got


def test_workspace_size_covers_shorter_streams(built):
    """bjxa_hip_decode_workspace(eb) is non-decreasing in eb (automatic
    plan), so a workspace sized for a stream also serves every shorter one
    (INTEGRATION.md), although the plan's chunk count is not monotone (C3's
    5,000,000 eblocks plan 125,000 chunks, 2,600,000 plan 130,000).  Host
    arithmetic only, no GPU needed (without one the planner assumes 256
    CUs)."""
    import numpy as np
    rng = np.random.default_rng(5)
    ebs = sorted(set(int(v) for v in rng.integers(1, 60_000_000, 400)) |
                 {1, 16, 17, 2_097_152, 2_097_153, 2_600_000, 5_000_000})
    for ch in (1, 2):
        sizes = [built.decode_workspace_size(eb, ch) for eb in ebs]
        assert all(a <= b for a, b in zip(sizes, sizes[1:])), ch
        assert built.decode_workspace_size(2_600_000, ch) <= \
            built.decode_workspace_size(5_000_000, ch)
