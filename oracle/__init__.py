"""ctypes view of the CPU restatement (oracle/xa_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by bjxa_amd/.  Everything here restates
reference behaviour; the citations point at the reference routine restated.
"""
import ctypes
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libxa_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        L.xo_decode.restype = ctypes.c_uint64
        L.xo_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint,
                                ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
        L.xo_encode.restype = ctypes.c_uint64
        L.xo_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint,
                                ctypes.c_uint, ctypes.c_void_p]
        _lib = L
    return _lib


def decode(xa, eblocks, bits, ch, state=(0, 0, 0, 0), frames=None, out=None):
    """Single-pass decode (bjxa_decode, src/libbjxa.c:602-661).

    Returns (pcm int16[frames*ch], state tuple, blocks_done, bad_chan)."""
    xa = np.ascontiguousarray(np.frombuffer(xa, dtype=np.uint8) if isinstance(xa, (bytes, bytearray)) else xa)
    if frames is None:
        frames = eblocks * 32
    st = np.array(state, dtype=np.int16)
    pcm = out if out is not None else np.empty(frames * ch, dtype=np.int16)
    bad = ctypes.c_int(-1)
    done = lib().xo_decode(xa.ctypes.data, eblocks, bits, ch, st.ctypes.data,
                           pcm.ctypes.data, frames, ctypes.byref(bad))
    return pcm, tuple(int(v) for v in st), int(done), bad.value


def encode(pcm, frames, bits, ch):
    """Single-pass encode (bjxa_encode, src/libbjxa.c:759-819)."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    eblocks = (frames + 31) // 32
    xa = np.empty(eblocks * ch * (bits * 4 + 1), dtype=np.uint8)
    lib().xo_encode(pcm.ctypes.data, frames, bits, ch, xa.ctypes.data)
    return xa


def parse_xa_header(buf):
    """Field split of the 32-byte XA header (src/libbjxa.c:409-421)."""
    magic, data_len, samples, rate, bits, ch, loop, l0, l1, r0, r1, pad = \
        struct.unpack("<4sIIHBBIhhhhI", bytes(buf[:32]))
    return dict(magic=magic, data_len=data_len, samples=samples, rate=rate,
                bits=bits, channels=ch, state=(l0, l1, r0, r1))


def validate_xa_header(buf):
    """bjxa_parse_header's checks (src/libbjxa.c:405-437, in that order,
    uint32 arithmetic) and bjxa_decode_format's block count (:588-597).
    Returns None on EPROTO -- including a stereo payload of an odd number of
    channel blocks, which passes :425-437 and trips the assertion at :597 --
    else the fields of a bjxa_hip_header_t record."""
    h = parse_xa_header(buf)
    dl, ns, bits, ch = h["data_len"], h["samples"], h["bits"], h["channels"]
    if h["magic"] != b"KWD1" or dl == 0 or ns == 0 or h["rate"] == 0:
        return None
    if bits not in (4, 6, 8) or ch not in (1, 2):
        return None
    bs = bits * 4 + 1
    max_samples = ((32 * dl) & 0xffffffff) // (bs * ch)
    if (dl // bs) * bs != dl or max_samples < ns or max_samples - ns >= 32:
        return None
    blocks = dl // (bs * ch)
    if blocks * bs * ch != dl:
        return None
    return dict(data_len=dl, samples=ns, blocks=blocks,
                data_len_pcm=(ns * ch * 2) & 0xffffffff, rate=h["rate"], bits=bits,
                channels=ch, state=h["state"])


def random_xa_headers(rng, n):
    """n 32-byte XA headers, about half valid, the rest broken in one of the
    ways the checks of src/libbjxa.c:405-437 catch (test input generator)."""
    out = np.zeros((n, 32), np.uint8)
    for i in range(n):
        bits = int(rng.choice([4, 6, 8]))
        ch = int(rng.integers(1, 3))
        bs = bits * 4 + 1
        nblk = int(np.exp(rng.uniform(0, np.log(2e8 / bs))))
        if ch == 2 and rng.random() < 0.8:
            nblk += nblk & 1
        dl = nblk * bs
        mx = ((32 * dl) & 0xffffffff) // (bs * ch)
        ns = max(1, mx - int(rng.integers(0, 32)))
        rate = int(rng.choice([22050, 44100, 48000, 1]))
        magic = b"KWD1"
        state = [int(v) for v in rng.integers(-32768, 32768, 4)]
        k = int(rng.integers(0, 14))
        if k == 0:
            magic = b"KWD" + bytes([int(rng.integers(0, 256))])
        elif k == 1:
            dl = 0
        elif k == 2:
            ns = 0
        elif k == 3:
            rate = 0
        elif k == 4:
            bits = int(rng.choice([0, 1, 5, 7, 9, 16, 255]))
        elif k == 5:
            ch = int(rng.choice([0, 3, 4, 255]))
        elif k == 6:
            dl += int(rng.integers(1, bs))
        elif k == 7:
            ns = mx + int(rng.integers(1, 100))
        elif k == 8:
            ns = max(1, mx - int(rng.integers(32, 1000)))
        elif k == 9:
            dl = int(rng.integers(1, 2**32))
            ns = int(rng.integers(1, 2**32))
        out[i] = np.frombuffer(magic + struct.pack("<IIHBBIhhhhI", dl & 0xffffffff,
                               ns & 0xffffffff, rate, bits & 0xff, ch & 0xff,
                               int(rng.integers(0, 2**32)), *state,
                               int(rng.integers(0, 2**32))), np.uint8)
    return out


def riff_header(ch, rate, data_len_pcm):
    """44-byte RIFF/WAVE header (bjxa_dump_riff_header, src/libbjxa.c:898-927)."""
    return (b"RIFF" + struct.pack("<I", 36 + data_len_pcm) + b"WAVEfmt " +
            struct.pack("<IHHIIHH", 16, 1, ch, rate, rate * ch * 2, ch * 2, 16) +
            b"data" + struct.pack("<I", data_len_pcm))


def decode_file(data):
    """XA file bytes -> WAV bytes, as `bjxa decode` produces them."""
    h = parse_xa_header(data)
    bsz = (h["bits"] * 4 + 1) * h["channels"]
    eblocks = h["data_len"] // bsz
    xa = np.frombuffer(data, dtype=np.uint8, offset=32, count=eblocks * bsz)
    pcm, _, done, bad = decode(xa, eblocks, h["bits"], h["channels"], h["state"],
                               frames=h["samples"])
    assert bad < 0 and done == eblocks
    return riff_header(h["channels"], h["rate"], pcm.nbytes) + pcm.tobytes()
