"""bjxa_amd -- MI355X-native libbjxa.

The product is the C library ``bjxa_amd/libbjxa.so.0`` (host C framing plus
hand-written gfx950 HIP kernels), a drop-in for the reference libbjxa
(src/bjxa.h, src/libbjxa.map).  This module is a thin ctypes view of its
C-ABI for the tests and the benchmark:

* :class:`Decoder` / :class:`Encoder` mirror ``bjxa_decoder_t`` /
  ``bjxa_encoder_t`` entry for entry (same names, argument meaning and
  errno behaviour: failures raise :class:`BjxaError` carrying the errno).
* :func:`decode_device` / :func:`encode_device` expose the device-resident
  extension (include/bjxa_hip.h) on raw device pointers.

Host-buffer calls below the offload threshold (and every call on a host
without a GPU) run on the library's CPU core (csrc/xa_cpu.c); the
device-resident entry points always run the HIP kernels and fail with
ENODEV without a GPU.  A missing library raises immediately.

Processes that also use PyTorch must import torch before calling
:func:`lib` so both share one HIP runtime.
"""
import ctypes
import errno as _errno
import os
import struct
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# BJXA_LIB_PATH selects an experimental build (tools/); default is in-tree
LIB_PATH = os.environ.get("BJXA_LIB_PATH") or os.path.join(_HERE, "libbjxa.so.0")
_lib = None

STATUS_WORDS = 8
NO_ERROR = 0xFFFFFFFF


class BjxaError(OSError):
    pass


def build():
    """Compile libbjxa.so.0 in-tree (host C + gfx950 kernels)."""
    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)


class Format(ctypes.Structure):
    """bjxa_format_t (reference src/bjxa.h:24-32)."""
    _fields_ = [("data_len_pcm", ctypes.c_uint32), ("blocks", ctypes.c_uint32),
                ("block_size_pcm", ctypes.c_uint8), ("block_size_xa", ctypes.c_uint8),
                ("samples_rate", ctypes.c_uint16), ("sample_bits", ctypes.c_uint8),
                ("channels", ctypes.c_uint8)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class HipStream(ctypes.Structure):
    """bjxa_hip_stream_t (include/bjxa_hip.h)."""
    _fields_ = [("d_src", ctypes.c_void_p), ("d_dst", ctypes.c_void_p),
                ("frames", ctypes.c_uint64), ("eblocks", ctypes.c_uint32),
                ("bits", ctypes.c_uint8), ("channels", ctypes.c_uint8),
                ("state", ctypes.c_int16 * 4)]


class HipTuning(ctypes.Structure):
    _fields_ = [("chunk", ctypes.c_uint32), ("warmup", ctypes.c_int32),
                ("ev_spec", ctypes.c_void_p * 2), ("variant", ctypes.c_uint32)]


_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_SIGS = {
    # LIBBJXA_0.1
    "bjxa_decoder": (_P, []),
    "bjxa_free_decoder": (ctypes.c_int, [_P]),
    "bjxa_parse_header": (ctypes.c_ssize_t, [_P, _P, _SZ]),
    "bjxa_fread_header": (ctypes.c_ssize_t, [_P, _P]),
    "bjxa_decode_format": (ctypes.c_int, [_P, _P]),
    "bjxa_decode": (ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
    "bjxa_dump_riff_header": (ctypes.c_ssize_t, [_P, _P, _SZ]),
    "bjxa_fwrite_riff_header": (ctypes.c_ssize_t, [_P, _P]),
    "bjxa_dump_pcm": (ctypes.c_int, [_P, _P, _SZ]),
    "bjxa_fwrite_pcm": (ctypes.c_int, [_P, _SZ, _P]),
    # LIBBJXA_0.5
    "bjxa_encoder": (_P, []),
    "bjxa_free_encoder": (ctypes.c_int, [_P]),
    "bjxa_encode_init": (ctypes.c_int, [_P, _P, ctypes.c_uint8]),
    "bjxa_parse_riff_header": (ctypes.c_ssize_t, [_P, _P, _SZ]),
    "bjxa_fread_riff_header": (ctypes.c_ssize_t, [_P, _P]),
    "bjxa_encode_format": (ctypes.c_int, [_P, _P]),
    "bjxa_encode": (ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
    "bjxa_dump_header": (ctypes.c_ssize_t, [_P, _P, _SZ]),
    "bjxa_fwrite_header": (ctypes.c_ssize_t, [_P, _P]),
    # LIBBJXA_HIP_0.1
    "bjxa_hip_decode_workspace": (_SZ, [ctypes.c_uint32, ctypes.c_uint, _P]),
    "bjxa_hip_workspace_init": (ctypes.c_int, [_P, _SZ, _P]),
    "bjxa_hip_decode_async": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P]),
    "bjxa_hip_encode_async": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint,
                                             ctypes.c_uint, _P, _P]),
    "bjxa_hip_version": (ctypes.c_char_p, []),
    "bjxa_hip_batch_new": (ctypes.c_void_p, [_P, ctypes.c_uint32, _P, _P]),
    "bjxa_hip_batch_decode_async": (ctypes.c_int, [_P, _P, _P, _P]),
    "bjxa_hip_batch_free": (None, [_P]),
    "bjxa_hip_decode_files": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_uint32]),
    # LIBBJXA_HIP_0.2
    "bjxa_hip_parse_headers_async": (ctypes.c_int, [_P, _SZ, ctypes.c_uint32, _P, _P]),
    # LIBBJXA_HIP_0.3
    "bjxa_hip_offload_threshold": (ctypes.c_int64, [ctypes.c_int, ctypes.c_int64]),
}
REFERENCE_SYMBOLS = {  # src/libbjxa.map:16-47
    "LIBBJXA_0.1": ["bjxa_decode", "bjxa_decode_format", "bjxa_decoder", "bjxa_dump_pcm",
                    "bjxa_dump_riff_header", "bjxa_fread_header", "bjxa_free_decoder",
                    "bjxa_fwrite_pcm", "bjxa_fwrite_riff_header", "bjxa_parse_header"],
    "LIBBJXA_0.5": ["bjxa_dump_header", "bjxa_encode", "bjxa_encode_format",
                    "bjxa_encode_init", "bjxa_encoder", "bjxa_fread_riff_header",
                    "bjxa_free_encoder", "bjxa_fwrite_header", "bjxa_parse_riff_header"],
}
EXTENSION_SYMBOLS = {"LIBBJXA_HIP_0.1": ["bjxa_hip_batch_decode_async", "bjxa_hip_batch_free",
                                         "bjxa_hip_batch_new", "bjxa_hip_decode_async",
                                         "bjxa_hip_decode_files",
                                         "bjxa_hip_decode_workspace", "bjxa_hip_encode_async",
                                         "bjxa_hip_version", "bjxa_hip_workspace_init"],
                     "LIBBJXA_HIP_0.2": ["bjxa_hip_parse_headers_async"],
                     "LIBBJXA_HIP_0.3": ["bjxa_hip_offload_threshold"]}


def lib():
    """Load libbjxa.so.0 from the package directory (fails loudly)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("bjxa_amd: %s is missing; run bjxa_amd.build() "
                               "(make -C bjxa_amd/csrc)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH, use_errno=True)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(ret, what):
    if ret is None or ret < 0:
        e = ctypes.get_errno()
        raise BjxaError(e, "%s: %s" % (what, os.strerror(e)))
    return ret


def _buf(obj):
    """(pointer, length) of a writable/readonly buffer (numpy, bytearray, bytes)."""
    if isinstance(obj, bytes):
        return ctypes.cast(ctypes.c_char_p(obj), ctypes.c_void_p).value, len(obj)
    if hasattr(obj, "ctypes"):
        return obj.ctypes.data, obj.nbytes
    c = (ctypes.c_char * len(obj)).from_buffer(obj)
    return ctypes.addressof(c), len(obj)


class Decoder:
    """bjxa_decoder_t (reference src/libbjxa.c:217-228, API src/bjxa.h:36-49)."""

    def __init__(self):
        self._p = lib().bjxa_decoder()
        if not self._p:
            _check(-1, "bjxa_decoder")

    def close(self):
        if self._p:
            p = ctypes.c_void_p(self._p)
            _check(lib().bjxa_free_decoder(ctypes.byref(p)), "bjxa_free_decoder")
            self._p = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def parse_header(self, hdr):
        ptr, n = _buf(hdr)
        return _check(lib().bjxa_parse_header(self._p, ptr, n), "bjxa_parse_header")

    def decode_format(self):
        f = Format()
        _check(lib().bjxa_decode_format(self._p, ctypes.byref(f)), "bjxa_decode_format")
        return f.as_dict()

    def decode(self, dst, src, dst_len=None, src_len=None):
        dp, dn = _buf(dst)
        sp, sn = _buf(src)
        return _check(lib().bjxa_decode(self._p, dp, dn if dst_len is None else dst_len,
                                        sp, sn if src_len is None else src_len), "bjxa_decode")

    def dump_riff_header(self):
        out = bytearray(44)
        ptr, n = _buf(out)
        _check(lib().bjxa_dump_riff_header(self._p, ptr, n), "bjxa_dump_riff_header")
        return bytes(out)


class Encoder:
    """bjxa_encoder_t (reference src/libbjxa.c:230-242, API src/bjxa.h:53-65)."""

    def __init__(self):
        self._p = lib().bjxa_encoder()
        if not self._p:
            _check(-1, "bjxa_encoder")

    def close(self):
        if self._p:
            p = ctypes.c_void_p(self._p)
            _check(lib().bjxa_free_encoder(ctypes.byref(p)), "bjxa_free_encoder")
            self._p = None

    __del__ = close

    def init(self, fmt, bits):
        f = Format(**fmt) if isinstance(fmt, dict) else fmt
        _check(lib().bjxa_encode_init(self._p, ctypes.byref(f), bits), "bjxa_encode_init")
        return f.as_dict()

    def encode_format(self):
        f = Format()
        _check(lib().bjxa_encode_format(self._p, ctypes.byref(f)), "bjxa_encode_format")
        return f.as_dict()

    def encode(self, dst, src, dst_len=None, src_len=None):
        dp, dn = _buf(dst)
        sp, sn = _buf(src)
        return _check(lib().bjxa_encode(self._p, dp, dn if dst_len is None else dst_len,
                                        sp, sn if src_len is None else src_len), "bjxa_encode")

    def dump_header(self):
        out = bytearray(32)
        ptr, n = _buf(out)
        _check(lib().bjxa_dump_header(self._p, ptr, n), "bjxa_dump_header")
        return bytes(out)


def parse_riff_header(hdr):
    f = Format()
    ptr, n = _buf(hdr)
    _check(lib().bjxa_parse_riff_header(ctypes.byref(f), ptr, n), "bjxa_parse_riff_header")
    return f.as_dict()


def decode_file(data):
    """XA file bytes -> WAV bytes, the single-pass shape of `bjxa decode`
    (reference src/bjxa_decode.c:56-100)."""
    import numpy as np
    with Decoder() as d:
        d.parse_header(data[:32])
        fmt = d.decode_format()
        riff = d.dump_riff_header()
        xa_len = fmt["block_size_xa"] * fmt["blocks"]
        src = np.frombuffer(data, dtype=np.uint8, offset=32, count=xa_len).copy()
        pcm = np.empty(fmt["data_len_pcm"] // 2, dtype=np.int16)
        n = d.decode(pcm, src)
        if n != fmt["blocks"]:
            raise BjxaError(_errno.EIO, "short decode")
    return riff + pcm.astype("<i2").tobytes()


def encode_wav(data, bits=6):
    """WAV bytes -> XA file bytes, the single-pass shape of `bjxa encode`
    (reference src/bjxa_encode.c:62-106)."""
    import numpy as np
    fmt = parse_riff_header(data[:44])
    e = Encoder()
    try:
        fmt = e.init(fmt, bits)
        hdr = e.dump_header()
        pcm = np.frombuffer(data, dtype="<i2", offset=44,
                            count=fmt["data_len_pcm"] // 2).astype(np.int16)
        out = np.empty(fmt["blocks"] * fmt["block_size_xa"], dtype=np.uint8)
        n = e.encode(out, pcm)
        if n != fmt["blocks"]:
            raise BjxaError(_errno.EIO, "short encode")
    finally:
        e.close()
    return hdr + out.tobytes()


# ---- device-resident extension (include/bjxa_hip.h) ----------------------

VARIANT_PACE_OFF = 15 << 8   # tuning variant bits 8-11: no pacing barriers
VARIANT_NORECORD = 0x40000   # test knob: every wave boundary goes to the sequential tail
VARIANT_NOWAIT = 0x80000     # test knob: waves do not wait for the previous wave's record
VARIANT_PIPE2 = 0x100000     # plan for two decodes in flight (one K1 workgroup per CU)
VARIANT_DECOR = 0x10000      # batches: the longer chunks of packed PCM images, forced
VARIANT_NODECOR = 0x20000    # batches: the same, never


def decode_workspace_size(eblocks, channels, chunk=0, warmup=-1, variant=0):
    """bjxa_hip_decode_workspace: device workspace bytes for one stream
    (pass the same chunk/warmup/variant as the decode)."""
    t = HipTuning(chunk, warmup)
    t.variant = variant
    return lib().bjxa_hip_decode_workspace(eblocks, channels, ctypes.byref(t))


def workspace_init(d_ws, ws_len, stream=0):
    _check(lib().bjxa_hip_workspace_init(d_ws, ws_len, stream), "bjxa_hip_workspace_init")


def decode_device(d_src, d_dst, eblocks, frames, bits, channels, d_ws, ws_len, d_status,
                  state=(0, 0, 0, 0), chunk=0, warmup=-1, stream=0, events=(None, None),
                  variant=0):
    """bjxa_hip_decode_async; `events` = optional hipEvent_t pair recorded
    around the speculative-decode kernel on `stream`."""
    s = HipStream(d_src, d_dst, frames, eblocks, bits, channels, (ctypes.c_int16 * 4)(*state))
    t = HipTuning(chunk, warmup, (ctypes.c_void_p * 2)(*events), variant)
    _check(lib().bjxa_hip_decode_async(ctypes.byref(s), d_ws, ws_len, d_status,
                                       ctypes.byref(t), stream), "bjxa_hip_decode_async")


class Batch:
    """bjxa_hip_batch_*: many device-resident streams decoded per launch.

    `streams` is a list of dicts with d_src, d_dst, eblocks, bits, channels
    and optional frames (default eblocks*32) and state."""

    def __init__(self, streams, chunk=0, warmup=-1, stream=0, variant=0):
        arr = (HipStream * len(streams))()
        for i, d in enumerate(streams):
            arr[i] = HipStream(d["d_src"], d["d_dst"], d.get("frames", d["eblocks"] * 32),
                               d["eblocks"], d["bits"], d["channels"],
                               (ctypes.c_int16 * 4)(*d.get("state", (0, 0, 0, 0))))
        t = HipTuning(chunk, warmup)
        t.variant = variant
        self.n = len(streams)
        self._p = lib().bjxa_hip_batch_new(arr, self.n, ctypes.byref(t), stream)
        if not self._p:
            e = ctypes.get_errno()
            raise BjxaError(e, "bjxa_hip_batch_new: %s" % os.strerror(e))

    def decode(self, d_status, stream=0, events=(None, None)):
        """Decode every stream; d_status holds n * STATUS_WORDS uint32."""
        t = HipTuning(0, -1, (ctypes.c_void_p * 2)(*events), 0)
        _check(lib().bjxa_hip_batch_decode_async(self._p, d_status, ctypes.byref(t), stream),
               "bjxa_hip_batch_decode_async")

    def close(self):
        if self._p:
            lib().bjxa_hip_batch_free(self._p)
            self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def decode_files(files):
    """bjxa_hip_decode_files: XA files (bytes) -> [(WAV bytes, errno)].

    Every WAV buffer is sized from its header (44 + data_len_pcm); a file
    whose header does not parse gets b"" and its errno."""
    n = len(files)
    bufs = [ctypes.create_string_buffer(bytes(f), len(f)) for f in files]
    outs = []
    for f in files:
        size = 44
        h = parse_header_fields(f)
        if h is not None and h["bits"] in (4, 6, 8) and h["channels"] in (1, 2):
            # bounded by what the file can hold, whatever the header says
            data_len = min(h["data_len"], max(len(f) - 32, 0))
            most = 32 * data_len // ((h["bits"] * 4 + 1) * h["channels"])
            size += min(h["samples"], most) * h["channels"] * 2
        outs.append(ctypes.create_string_buffer(size))
    xa = (ctypes.c_void_p * n)(*[ctypes.addressof(b) for b in bufs])
    xl = (ctypes.c_size_t * n)(*[len(f) for f in files])
    wv = (ctypes.c_void_p * n)(*[ctypes.addressof(o) for o in outs])
    wl = (ctypes.c_size_t * n)(*[len(o) for o in outs])
    st = (ctypes.c_int * n)()
    _check(lib().bjxa_hip_decode_files(xa, xl, wv, wl, st, n), "bjxa_hip_decode_files")
    res = []
    for o, f, s in zip(outs, files, st):
        h = parse_header_fields(f)
        res.append((o.raw if h is not None else b"", int(s)))
    return res


def parse_header_fields(data):
    """Raw XA header fields (src/libbjxa.c:409-421), no validation."""
    if len(data) < 32 or bytes(data[:4]) != b"KWD1":
        return None
    data_len, samples, rate, bits, ch = struct.unpack("<IIHBB", bytes(data[4:16]))
    return {"data_len": data_len, "samples": samples, "rate": rate, "bits": bits,
            "channels": ch}


def header_record():
    """numpy dtype of bjxa_hip_header_t (include/bjxa_hip.h), 32 bytes."""
    import numpy as np
    return np.dtype([("data_len", "<u4"), ("samples", "<u4"), ("blocks", "<u4"),
                     ("data_len_pcm", "<u4"), ("rate", "<u2"), ("bits", "u1"),
                     ("channels", "u1"), ("state", "<i2", 4), ("status", "<i4")])


def parse_headers_device(d_src, stride, n, d_out, stream=0):
    """Validate n device-resident XA headers (bjxa_parse_header's checks,
    src/libbjxa.c:395-453) into n header_record() entries at d_out."""
    _check(lib().bjxa_hip_parse_headers_async(d_src, stride, n, d_out, stream),
           "bjxa_hip_parse_headers_async")


def encode_device(d_pcm, frames, bits, channels, d_xa, stream=0):
    _check(lib().bjxa_hip_encode_async(d_pcm, frames, bits, channels, d_xa, stream),
           "bjxa_hip_encode_async")


OFFLOAD_DECODE, OFFLOAD_ENCODE = 0, 1


def offload_threshold(direction, eblocks=-1):
    """bjxa_hip_offload_threshold: set (eblocks >= 0) or query the number
    of effective blocks from which bjxa_decode/bjxa_encode calls run on the
    GPU; returns the previous value."""
    return _check(lib().bjxa_hip_offload_threshold(direction, eblocks),
                  "bjxa_hip_offload_threshold")


class offload:
    """Context manager routing host-API calls: offload(0) sends every call
    to the GPU, offload(None) none (CPU core only)."""

    def __init__(self, eblocks):
        self.v = (1 << 63) - 1 if eblocks is None else eblocks

    def __enter__(self):
        self.old = [offload_threshold(d, self.v) for d in (OFFLOAD_DECODE, OFFLOAD_ENCODE)]
        return self

    def __exit__(self, *a):
        for d, v in zip((OFFLOAD_DECODE, OFFLOAD_ENCODE), self.old):
            offload_threshold(d, v)


def version():
    return lib().bjxa_hip_version().decode()


def xa_header(data_len, samples, rate, bits, channels, state=(0, 0, 0, 0)):
    """32-byte XA header bytes (layout src/libbjxa.c:409-421)."""
    return b"KWD1" + struct.pack("<IIHBBIhhhhI", data_len, samples, rate, bits, channels,
                                 0, *state, 0)
