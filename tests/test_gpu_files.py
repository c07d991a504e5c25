"""bjxa_hip_decode_files: many XA files -> WAV files in one batched pass,
each equal to what `bjxa decode` makes of it (the oracle's decode_file),
with per-file status for broken inputs."""
import errno

import numpy as np
import pytest

import bjxa_amd
import oracle
from bjxa_amd import synth

FIXTURES = ["square-mono-4.xa", "square-mono-6.xa", "square-mono-8.xa",
            "square-stereo-4.xa", "square-stereo-6.xa", "square-stereo-8.xa"]


def xa_file(eb, bits, ch, seed, cut=0, state=(0, 0, 0, 0)):
    xa = synth.stream(eb, bits, ch, "A", seed=seed)
    return bjxa_amd.xa_header(xa.size, eb * 32 - cut, 22050, bits, ch, state) + xa.tobytes()


@pytest.mark.gpu
def test_decode_files_batch(built, golden):
    rng = np.random.default_rng(7)
    files = [golden(n) for n in FIXTURES]
    for i in range(30):
        bits, ch = [(8, 2), (6, 2), (4, 2), (8, 1), (6, 1), (4, 1)][i % 6]
        eb = int(rng.choice([1, 31, 33, 1000, 20001]))
        files.append(xa_file(eb, bits, ch, 600 + i, cut=int(rng.integers(0, 32)),
                             state=tuple(int(v) for v in rng.integers(-999, 999, 4))))
    # a block profile with gain 5 in the right channel of eblock 77
    bad = bytearray(xa_file(200, 8, 2, 700))
    bad[32 + (77 * 2 + 1) * 33] = 0x50
    files.append(bytes(bad))
    files.append(b"KWD2" + files[0][4:])                  # wrong magic
    files.append(files[1][:-100])                          # truncated body
    odd = bytearray(xa_file(3, 8, 2, 701))
    odd[4:8] = (3 * 33).to_bytes(4, "little")              # 3 channel blocks, stereo
    files.append(bytes(odd[:32 + 99]))
    res = bjxa_amd.decode_files(files)
    k = len(files) - 4                                     # the bad-profile file
    for f, (wav, st) in zip(files[:k], res[:k]):
        assert st == 0
        assert wav == oracle.decode_file(f)
    wav, st = res[k]
    assert st == errno.EPROTO
    full = oracle.decode(np.frombuffer(files[k], np.uint8, offset=32), 200, 8, 2)
    assert full[2] == 77                                   # eblocks before the bad one
    assert wav[:44] == oracle.decode_file(xa_file(200, 8, 2, 700))[:44]
    assert wav[44:44 + 77 * 128] == full[0][:77 * 64].tobytes()
    assert [s for _, s in res[k + 1:]] == [errno.EPROTO, errno.ENOBUFS, errno.EPROTO]


def test_decode_files_host_checks(built):
    """Without a GPU: files refused by their headers get their errno and no
    device is needed; a batch with a decodable file fails with ENODEV."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    probe = r"""
import errno, sys
sys.path.insert(0, sys.argv[1])
import bjxa_amd
good = bjxa_amd.xa_header(33, 32, 8000, 8, 1) + bytes(33)
bad = b"KWD2" + good[4:]
print([s for _, s in bjxa_amd.decode_files([bad, good[:40]])])
try:
    bjxa_amd.decode_files([good])
    print("no error")
except bjxa_amd.BjxaError as e:
    print(e.errno)
"""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", probe, ROOT], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert lines[0] == str([errno.EPROTO, errno.ENOBUFS])
    assert lines[1] == str(errno.ENODEV)


@pytest.mark.gpu
def test_decode_files_multi_slab(built):
    """A batch whose images span several 64 MiB staging slabs (input ~80 MB,
    output ~160 MB): files of odd sizes straddle the slab cuts, the copy
    pool splits pieces between threads, and a file that stops at a bad
    profile in the middle of a slab keeps exactly its PCM prefix."""
    rng = np.random.default_rng(11)
    files = []
    total = 0
    i = 0
    while total < 80_000_000:
        bits, ch = [(8, 2), (6, 1), (4, 2), (8, 1)][i % 4]
        eb = int(rng.integers(50_000, 400_000)) | 1
        files.append(xa_file(eb, bits, ch, 900 + i, cut=int(rng.integers(0, 32))))
        total += len(files[-1])
        i += 1
    k = len(files) // 2
    bad = bytearray(files[k])
    bits, ch = [(8, 2), (6, 1), (4, 2), (8, 1)][k % 4]
    stop = 12345
    bad[32 + stop * ch * (bits * 4 + 1)] = 0x60
    files[k] = bytes(bad)
    res = bjxa_amd.decode_files(files)
    for j, (f, (wav, st)) in enumerate(zip(files, res)):
        if j == k:
            assert st == errno.EPROTO
            full = oracle.decode(np.frombuffer(f, np.uint8, offset=32),
                                 (len(f) - 32) // (ch * (bits * 4 + 1)), bits, ch)
            assert full[2] == stop
            assert wav[44:44 + stop * 64 * ch] == full[0][:stop * 32 * ch].tobytes()
        else:
            assert st == 0
            assert wav == oracle.decode_file(f), j
