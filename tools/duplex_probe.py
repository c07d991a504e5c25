"""Can the host-pointer path move its two directions at once?  (VERDICT r04
item 5)  The largest single-header 8-bit stereo
stream (2,000,000 eblocks: 132 MB of XA in, 256 MB of PCM out), timed five
ways on one GPU, median of --reps:

  dma_serial    pinned XA -> HBM copy, decode, HBM -> pinned PCM copy, one
                stream (what bjxa_decode does, with pinned instead of
                pageable buffers)
  dma_2streams  the two copies alone, issued together on two streams
  zc_both       the decode kernels reading XA from, and writing PCM into,
                pinned host memory directly (device-mapped pointers): the
                PCIe reads and the posted writes at once
  zc_in / zc_out  only the input / only the output in host memory
  *_nc          the same with hipHostMallocNonCoherent buffers

Each zero-copy variant is checked against the HBM decode byte for byte.

usage: python tools/duplex_probe.py [--eblocks 2000000] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bjxa_amd  # noqa: E402
from bjxa_amd import synth  # noqa: E402

H2D, D2H = 1, 2
COHERENT, NONCOHERENT = 0x40000000, 0x80000000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eblocks", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    eb, bits, ch = args.eblocks, 8, 2
    nin, nout = eb * ch * (bits * 4 + 1), eb * 64 * ch
    hip = ctypes.CDLL("libamdhip64.so.7")
    P = ctypes.c_void_p
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(P), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [P]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(P), P, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int, P]
    hip.hipStreamSynchronize.argtypes = [P]

    def host(n, flags):
        p = P()
        assert hip.hipHostMalloc(ctypes.byref(p), n, flags) == 0
        d = P()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), p, 0) == 0
        return p.value, d.value, np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))

    xa = synth.stream(eb, bits, ch, "A", seed=0)
    din = torch.from_numpy(xa).cuda()
    dout = torch.empty(nout, dtype=torch.uint8, device="cuda")
    ws_len = bjxa_amd.decode_workspace_size(eb, ch)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device="cuda")
    st = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    sh = s1.cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    def decode(src, dst):
        bjxa_amd.decode_device(src, dst, eb, eb * 32, bits, ch, ws.data_ptr(), ws_len,
                               st.data_ptr(), (0, 0, 0, 0), 0, -1, sh)

    decode(din.data_ptr(), dout.data_ptr())
    torch.cuda.synchronize()
    ref = dout.cpu().numpy().copy()

    def t(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - a)
        return round(float(np.median(ts)) * 1e3, 3)

    res = {"eblocks": eb, "xa_bytes": nin, "pcm_bytes": nout}
    for tag, flags in (("", COHERENT), ("_nc", NONCOHERENT)):
        hin, hin_d, hin_np = host(nin, flags)
        hout, hout_d, hout_np = host(nout, flags)
        hin_np[:] = xa
        hout_np[:] = 0

        def dma_serial():
            hip.hipMemcpyAsync(din.data_ptr(), hin, nin, H2D, sh)
            decode(din.data_ptr(), dout.data_ptr())
            hip.hipMemcpyAsync(hout, dout.data_ptr(), nout, D2H, sh)

        def dma_2streams():
            hip.hipMemcpyAsync(din.data_ptr(), hin, nin, H2D, sh)
            hip.hipMemcpyAsync(hout, dout.data_ptr(), nout, D2H, s2.cuda_stream)
            hip.hipStreamSynchronize(s2.cuda_stream)

        res["dma_serial" + tag] = t(dma_serial)
        res["dma_2streams" + tag] = t(dma_2streams)
        res["zc_both" + tag] = t(lambda: decode(hin_d, hout_d))
        res["zc_both" + tag + "_exact"] = bool(np.array_equal(hout_np, ref))
        hout_np[:] = 0
        res["zc_in" + tag] = t(lambda: decode(hin_d, dout.data_ptr()))
        res["zc_out" + tag] = t(lambda: decode(din.data_ptr(), hout_d))
        res["zc_out" + tag + "_exact"] = bool(np.array_equal(hout_np, ref))
        torch.cuda.synchronize()
        hip.hipHostFree(hin)
        hip.hipHostFree(hout)
        print(json.dumps(res), flush=True)
    res["hbm_decode"] = t(lambda: decode(din.data_ptr(), dout.data_ptr()))

    # slab pipeline: the input of slab k+1 by DMA (stream A) while slab k
    # decodes with its PCM written straight into host memory (stream B);
    # entry states are not chained here (timing only)
    hin, hin_d, hin_np = host(nin, COHERENT)
    hout, hout_d, hout_np = host(nout, COHERENT)
    hin_np[:] = xa
    hip.hipEventCreate.argtypes = [ctypes.POINTER(P)]
    hip.hipEventRecord.argtypes = [P, P]
    hip.hipStreamWaitEvent.argtypes = [P, P, ctypes.c_uint]
    ebsz = ch * (bits * 4 + 1)
    for nslab in (4, 8, 16):
        evs = []
        for _ in range(nslab):
            e = P()
            hip.hipEventCreate(ctypes.byref(e))
            evs.append(e.value)
        per = (eb + nslab - 1) // nslab
        wsn = bjxa_amd.decode_workspace_size(per, ch)
        wss = [torch.zeros(wsn, dtype=torch.uint8, device="cuda") for _ in range(2)]
        sts = [torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device="cuda")
               for _ in range(2)]
        for w in wss:
            bjxa_amd.workspace_init(w.data_ptr(), wsn, sh)

        def pipe():
            for k in range(nslab):
                lo, hi = k * per, min(eb, (k + 1) * per)
                hip.hipMemcpyAsync(din.data_ptr() + lo * ebsz, hin + lo * ebsz,
                                   (hi - lo) * ebsz, H2D, s2.cuda_stream)
                hip.hipEventRecord(evs[k], s2.cuda_stream)
            for k in range(nslab):
                lo, hi = k * per, min(eb, (k + 1) * per)
                hip.hipStreamWaitEvent(sh, evs[k], 0)
                bjxa_amd.decode_device(din.data_ptr() + lo * ebsz, hout_d + lo * 128,
                                       hi - lo, (hi - lo) * 32, bits, ch,
                                       wss[k % 2].data_ptr(), wsn, sts[k % 2].data_ptr(),
                                       (0, 0, 0, 0), 0, -1, sh)
        res["pipe_dma_in_zc_out_%d" % nslab] = t(pipe)
    hip.hipHostFree(hin)
    hip.hipHostFree(hout)

    # pinning a caller's pageable buffers in place, and posted writes into one
    hip.hipHostRegister.argtypes = [P, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [P]
    user_out = np.ones(nout, dtype=np.uint8)

    def reg():
        assert hip.hipHostRegister(user_out.ctypes.data, nout, 2) == 0
        d = P()
        assert hip.hipHostGetDevicePointer(ctypes.byref(d), user_out.ctypes.data, 0) == 0
        return d.value
    a = time.perf_counter()
    ud = reg()
    res["register_256MB_ms"] = round((time.perf_counter() - a) * 1e3, 3)
    res["zc_out_registered"] = t(lambda: decode(din.data_ptr(), ud))
    res["zc_out_registered_exact"] = bool(np.array_equal(user_out, ref))
    a = time.perf_counter()
    hip.hipHostUnregister(user_out.ctypes.data)
    res["unregister_256MB_ms"] = round((time.perf_counter() - a) * 1e3, 3)

    # host memcpy of the PCM (pinned staging -> a caller's buffer), T threads
    import threading
    src_np = np.ones(nout, dtype=np.uint8)
    for th in (1, 4, 8, 16):
        parts = np.array_split(np.arange(nout, dtype=np.int64)[::1 << 20], th)

        def cp(lo_hi):
            lo, hi = lo_hi
            np.copyto(user_out[lo:hi], src_np[lo:hi])
        step = (nout + th - 1) // th

        def run():
            ts = [threading.Thread(target=cp, args=((i * step, min(nout, (i + 1) * step)),))
                  for i in range(th)]
            for x in ts:
                x.start()
            for x in ts:
                x.join()
        res["host_memcpy_256MB_%dthr_ms" % th] = t(run)
        del parts
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
