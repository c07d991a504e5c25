"""In-process interleaved A/B of library builds on one GPU: every build is
loaded side by side (ctypes, RTLD_LOCAL) and decodes the same
device-resident stream in rotation, so box-to-box and run-to-run drift hit
all variants alike.  Reports per build the median step time (spec + fix,
events around bjxa_hip_decode_async), the median spec-kernel time, and
whether its PCM equals the first build's.

usage: python tools/ab_inproc.py [--wl C3|C2|C4|C5|C5g] [--mix A] [--reps 6]
           [--steps 20] [--layout sep|packed] label=path[:variant[:chunk[:warmup]]] ...
(C4/C5/C5g: the batched decode, bjxa_hip_batch_*, streams seeded as bench.py)
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from bjxa_amd import synth, HipStream, HipTuning  # noqa: E402

WL = {"C3": (5_000_000, 8, 2), "C2": (10_000_000, 8, 1), "C3s": (1_000_000, 8, 2),
      "C5s": (128 * 65536, 8, 2)}   # C5g's eblocks as one stream
BATCH = ("C4", "C5", "C5g")


_HIP = []


def raw_buffer(n, flags=None):
    """A uint8 CUDA tensor over a hipMalloc of exactly n bytes (kept for the
    life of the process); with `flags`, hipExtMallocWithFlags (4 =
    hipDeviceMallocContiguous)."""
    if not _HIP:
        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        h.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                            ctypes.c_uint]
        _HIP.append(h)
    p = ctypes.c_void_p()
    if flags is None:
        assert _HIP[0].hipMalloc(ctypes.byref(p), n) == 0
    else:
        assert _HIP[0].hipExtMallocWithFlags(ctypes.byref(p), n, flags) == 0

    class Iface:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "|u1",
                                    "data": (p.value, False), "version": 2}
    return torch.as_tensor(Iface(), device="cuda")


def load(path):
    L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    L.bjxa_hip_decode_workspace.restype = ctypes.c_size_t
    L.bjxa_hip_decode_workspace.argtypes = [ctypes.c_uint32, ctypes.c_uint, ctypes.c_void_p]
    L.bjxa_hip_workspace_init.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.bjxa_hip_batch_new.restype = ctypes.c_void_p
    L.bjxa_hip_batch_new.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_void_p]
    L.bjxa_hip_batch_decode_async.argtypes = [ctypes.c_void_p] * 4
    L.bjxa_hip_batch_free.argtypes = [ctypes.c_void_p]
    L.bjxa_hip_decode_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wl", default="C3")
    ap.add_argument("--mix", default="A")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--offset", type=int, default=0,
                    help="single-stream workloads: place src/dst this many bytes into "
                         "larger allocations (a multiple of 16)")
    ap.add_argument("--eblocks", type=int, default=0,
                    help="single-stream workloads: override the stream length")
    ap.add_argument("--layout", default="sep",
                    help="batches: one allocation per stream buffer (sep) or all "
                         "streams back to back in one allocation (packed); also gaps, "
                         "gaps2m, skew, pages, packed_src, packed_dst, hipmalloc, and "
                         "rot<b> / pad<b> (PCM only, one allocation: image i shifted by "
                         "(37 i mod 64) << b, or images 2^b bytes apart past their size)")
    ap.add_argument("builds", nargs="+")
    args = ap.parse_args()
    batch = args.wl in BATCH or args.wl.startswith(("C3x", "B"))
    if batch:
        import bench
        if args.wl.startswith("B"):
            # B<n>x<eb>: n separately allocated 8-bit stereo streams of eb eblocks
            n, e = (int(v) for v in args.wl[1:].split("x"))
            inputs = [(i, 8, 2, e, synth.stream(e, 8, 2, args.mix, seed=1000 + i))
                      for i in range(n)]
        elif args.wl.startswith("C3x"):
            # C3's 5M eblocks as n separately allocated streams (C3x<n>)
            n = int(args.wl[3:])
            inputs = [(i, 8, 2, 5_000_000 // n, synth.stream(5_000_000 // n, 8, 2, args.mix,
                                                            seed=1000 + i))
                      for i in range(n)]
        else:
            inputs = bench.batch_inputs(args.wl, 0, 0, 0, len(bench.batch_specs(args.wl)),
                                        mix=args.mix)
        lay = args.layout
        shift = None
        if lay.startswith(("rot", "pad")):
            shift = (lay[:3], int(lay[3:]))
            lay = "packed_dst"
        elif lay in ("contig", "contig_sep"):
            # PCM images back to back in one hipDeviceMallocContiguous
            # allocation, or each in one of its own
            shift = (lay, 0)
            lay = "sep"
        elif lay.startswith(("grp", "own")):
            # grp<g>: PCM images back to back in allocations of g images each;
            # own<m>: each PCM image at the start of an allocation of m MiB
            shift = (lay[:3], int(lay[3:]))
            lay = "sep"
        assert lay in ("sep", "packed", "gaps", "gaps2m", "skew", "pages", "packed_src",
                       "packed_dst", "hipmalloc"), args.layout
        if lay in ("packed", "gaps", "gaps2m", "skew", "pages", "packed_src",
                   "packed_dst"):
            # every stream in one allocation, back to back at 256-B steps
            # (gaps: plus a seeded random gap of 0-255 x 256 B before each;
            # gaps2m: 0-31 x 64 KiB; skew: stream i at +(37 i mod 32) x
            # 64 KiB + (i mod 16) x 4 KiB; pages: each stream on a fresh 2 MiB
            # boundary after 0-3 whole 2 MiB pages left unused)
            rng = np.random.default_rng(7)

            def carve(sizes):
                offs, o = [], 0
                for k, n in enumerate(sizes):
                    if args.layout == "gaps":
                        o += int(rng.integers(0, 256)) * 256
                    elif args.layout == "gaps2m":
                        o += int(rng.integers(0, 32)) * 65536
                    elif args.layout == "pages":
                        o = (o + (1 << 21) - 1) // (1 << 21) * (1 << 21) + \
                            int(rng.integers(0, 4)) * (1 << 21)
                    elif args.layout == "skew":
                        o = (o + (1 << 21) - 1) // (1 << 21) * (1 << 21) + \
                            ((37 * k) % 32) * 65536 + (k % 16) * 4096
                    if shift is not None and shift[0] == "rot":
                        # image k at k whole strides plus (37 k mod 64) << b
                        st = (((n + (64 << shift[1]) - 1) >> (shift[1] + 6)) + 1) << \
                            (shift[1] + 6)
                        o = k * st + (((37 * k) % 64) << shift[1])
                    offs.append(o)
                    o += (n + 255) // 256 * 256
                    if shift is not None and shift[0] == "pad":
                        o += 1 << shift[1]
                big = torch.empty(o, dtype=torch.uint8, device="cuda")
                return [big[a:a + n] for a, n in zip(offs, sizes)]
            # (packed_src / packed_dst: only the XA inputs / only the PCM
            # images back to back in one allocation, the other side separate)
            if lay == "packed_dst":
                srcs = [torch.from_numpy(x).cuda() for *_, x in inputs]
            else:
                srcs = carve([x.size for *_, x in inputs])
                for t_, (*_, x) in zip(srcs, inputs):
                    t_.copy_(torch.from_numpy(x))
            if lay == "packed_src":
                dsts = [torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
                        for _, _, ch, eb, _ in inputs]
            else:
                dsts = carve([eb * 64 * ch for _, _, ch, eb, _ in inputs])
        elif lay == "hipmalloc":
            # every buffer a hipMalloc of its own at its exact size (as a C
            # caller would make them), outside torch's caching allocator
            srcs = [raw_buffer(x.size) for *_, x in inputs]
            for t_, (*_, x) in zip(srcs, inputs):
                t_.copy_(torch.from_numpy(x))
            dsts = [raw_buffer(eb * 64 * ch) for _, _, ch, eb, _ in inputs]
        else:
            srcs = [torch.from_numpy(x).cuda() for *_, x in inputs]
            sizes = [eb * 64 * ch for _, _, ch, eb, _ in inputs]
            if shift is not None and shift[0] == "grp":
                dsts = []
                for i in range(0, len(sizes), shift[1]):
                    part = sizes[i:i + shift[1]]
                    big = torch.empty(sum(part), dtype=torch.uint8, device="cuda")
                    o = 0
                    for n in part:
                        dsts.append(big[o:o + n])
                        o += n
            elif shift is not None and shift[0] == "contig":
                big = raw_buffer(sum(sizes), 4)
                offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
                dsts = [big[int(o):int(o) + n] for o, n in zip(offs, sizes)]
            elif shift is not None and shift[0] == "contig_sep":
                dsts = [raw_buffer(n, 4) for n in sizes]
            elif shift is not None and shift[0] == "own":
                dsts = [torch.empty(max(n, shift[1] << 20), dtype=torch.uint8,
                                    device="cuda")[:n] for n in sizes]
            else:
                dsts = [torch.empty(n, dtype=torch.uint8, device="cuda") for n in sizes]
        arr = (HipStream * len(inputs))()
        for i, ((_, bits, ch, eb, _), s_, d_) in enumerate(zip(inputs, srcs, dsts)):
            arr[i] = HipStream(s_.data_ptr(), d_.data_ptr(), eb * 32, eb, bits, ch,
                               (ctypes.c_int16 * 4)(0, 0, 0, 0))
        dst = dsts[0]
        st = torch.zeros(8 * len(inputs), dtype=torch.int32, device="cuda")
        eb = bits = ch = 0
    else:
        eb, bits, ch = WL[args.wl]
        eb = args.eblocks or eb
        xa = synth.stream(eb, bits, ch, args.mix, seed=0)
        if args.offset:
            # stream buffers placed `offset` bytes into larger allocations
            o = args.offset
            sbig = torch.empty(xa.size + o, dtype=torch.uint8, device="cuda")
            dbig = torch.empty(eb * 64 * ch + o, dtype=torch.uint8, device="cuda")
            src = sbig[o:o + xa.size]
            src.copy_(torch.from_numpy(xa))
            dst = dbig[o:o + eb * 64 * ch]
        else:
            src = torch.from_numpy(xa).cuda()
            dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device="cuda")
        st = torch.zeros(8, dtype=torch.int32, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                        ctypes.c_void_p]
    builds = []
    for spec in args.builds:
        label, rest = spec.split("=", 1)
        parts = rest.split(":")
        path = parts[0]
        var = int(parts[1], 0) if len(parts) > 1 and parts[1] else 0
        chunk = int(parts[2]) if len(parts) > 2 and parts[2] else 0
        warm = int(parts[3]) if len(parts) > 3 and parts[3] else -1
        L = load(path)
        tune = HipTuning(chunk, warm)
        tune.variant = var
        if batch:
            bp = L.bjxa_hip_batch_new(arr, len(inputs), ctypes.byref(tune), sh)
            assert bp, "batch_new failed"
            n, ws = bp, None
        else:
            n = L.bjxa_hip_decode_workspace(eb, ch, ctypes.byref(tune))
            ws = torch.zeros(n, dtype=torch.uint8, device="cuda")
            L.bjxa_hip_workspace_init(ws.data_ptr(), n, sh)
        evs = []
        for _ in range(args.steps):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            hip.hipEventCreate(ctypes.byref(a))
            hip.hipEventCreate(ctypes.byref(b))
            evs.append((a.value, b.value))
        builds.append({"label": label, "L": L, "tune": tune, "ws": ws, "n": n, "evs": evs,
                       "step": [], "spec": [], "sum": None})
    s = None if batch else HipStream(src.data_ptr(), dst.data_ptr(), eb * 32, eb, bits, ch,
                                     (ctypes.c_int16 * 4)(0, 0, 0, 0))

    def run(b, timed):
        t = b["tune"]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(args.steps):
            if timed:
                t.ev_spec[0], t.ev_spec[1] = b["evs"][i]
                e0.record()
            if batch:
                rc = b["L"].bjxa_hip_batch_decode_async(b["n"], st.data_ptr(),
                                                        ctypes.byref(t), sh)
            else:
                rc = b["L"].bjxa_hip_decode_async(ctypes.byref(s), b["ws"].data_ptr(), b["n"],
                                                  st.data_ptr(), ctypes.byref(t), sh)
            assert rc == 0
            if timed:
                e1.record()
                e1.synchronize()
                b["step"].append(e0.elapsed_time(e1))
                f = ctypes.c_float()
                hip.hipEventElapsedTime(ctypes.byref(f), *b["evs"][i])
                b["spec"].append(f.value)
        t.ev_spec[0] = t.ev_spec[1] = None

    for b in builds:
        run(b, False)
    torch.cuda.synchronize()
    for r in range(args.reps):
        order = builds[r % len(builds):] + builds[:r % len(builds)]
        for b in order:
            run(b, True)
            if b["sum"] is None:
                torch.cuda.synchronize()
                b["sum"] = int(dst.view(torch.int16).to(torch.int64).sum().item()) ^ \
                    int(dst[::4093].to(torch.int64).sum().item()) << 40
            dst.fill_(0)
    ref = builds[0]["sum"]
    for b in builds:
        print("%-10s step %.4f ms (p10 %.4f)  spec %.4f ms (p10 %.4f)  same-as-first %s" % (
            b["label"], np.median(b["step"]), np.percentile(b["step"], 10),
            np.median(b["spec"]), np.percentile(b["spec"], 10), b["sum"] == ref), flush=True)


if __name__ == "__main__":
    main()
