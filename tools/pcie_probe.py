"""Host<->device copy behaviour behind the host-pointer API (bjxa_decode on
host buffers): pageable vs registered (hipHostRegister) memory, the cost of
registering, and whether H2D and D2H overlap on two streams.  Sizes are the
largest single-header 8-bit stereo stream: 132 MB of XA in, 256 MB of PCM out.

usage: python tools/pcie_probe.py
"""
import ctypes
import json
import time

import numpy as np
import torch

H2D, D2H = 1, 2


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    P = ctypes.c_void_p
    hip.hipMemcpyAsync.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int, P]
    hip.hipStreamSynchronize.argtypes = [P]
    hip.hipHostRegister.argtypes = [P, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [P]
    nin, nout = 132_000_000, 256_000_000
    hin = np.random.default_rng(0).integers(0, 256, nin, dtype=np.uint8)
    hout = np.empty(nout, dtype=np.uint8)
    hout[:] = 1
    din = torch.empty(nin, dtype=torch.uint8, device="cuda")
    dout = torch.empty(nout, dtype=torch.uint8, device="cuda")
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    r = {}

    def t(fn, n=5):
        fn()
        ts = []
        for _ in range(n):
            a = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - a)
        return round(float(np.median(ts)) * 1e3, 3)

    def h2d(stream=s1, n=nin):
        hip.hipMemcpyAsync(din.data_ptr(), hin.ctypes.data, n, H2D, stream.cuda_stream)

    def d2h(stream=s2, n=nout):
        hip.hipMemcpyAsync(hout.ctypes.data, dout.data_ptr(), n, D2H, stream.cuda_stream)

    def sync():
        hip.hipStreamSynchronize(s1.cuda_stream)
        hip.hipStreamSynchronize(s2.cuda_stream)

    r["pageable_h2d_ms"] = t(lambda: (h2d(), sync()))
    r["pageable_d2h_ms"] = t(lambda: (d2h(), sync()))
    r["pageable_both_2streams_ms"] = t(lambda: (h2d(), d2h(), sync()))

    def reg():
        hip.hipHostRegister(hin.ctypes.data, nin, 0)
        hip.hipHostRegister(hout.ctypes.data, nout, 0)

    def unreg():
        hip.hipHostUnregister(hin.ctypes.data)
        hip.hipHostUnregister(hout.ctypes.data)

    r["register_unregister_ms"] = t(lambda: (reg(), unreg()))
    reg()
    r["registered_h2d_ms"] = t(lambda: (h2d(), sync()))
    r["registered_d2h_ms"] = t(lambda: (d2h(), sync()))
    r["registered_both_2streams_ms"] = t(lambda: (h2d(), d2h(), sync()))
    unreg()
    r["in_MB"], r["out_MB"] = nin / 1e6, nout / 1e6
    print(json.dumps(r))


if __name__ == "__main__":
    main()
