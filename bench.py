#!/usr/bin/env python3
"""bench.py -- XA ADPCM decode throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path (bjxa_hip_decode_async: speculative
decode + verify/repair/tail) over one synthetic XA stream already resident
in HBM.  The bench line is BASELINE config C3 -- one 8-bit stereo stream of
5,000,000 effective blocks (320M int16 samples), profile mix A -- the case
north_star quotes its target on; at N=1 the same run also measures C2
(configs[1]: one 8-bit mono stream of 10,000,000 blocks) and the batched
configs C4 (1024 mixed-format streams per launch) and C5g (one GPU's share of
C5 at 8 GPUs), and the encode direction on C3-shaped PCM, reported under
"other_configs" (--no-other skips them).

Multi-GPU (torchrun, one process per GPU): every rank decodes its own
C3-sized stream (independent objects, no data-path collective), so per-GPU
work is fixed: "scaling": "weak".  RCCL carries only the barriers, the max
over ranks of the timed region and the AND of the bit-exact checks.

Reported:
  value       decoded MSamples/s of the whole job (all ranks) over the timed
              steps (barrier + synchronize on both sides, max over ranks)
  roofline    xa_decode_spec, the dominant kernel: algorithmic bytes per
              launch (XA read + PCM written, SURVEY.md §8(d): 3.03125 B per
              8-bit sample) / its mean duration from hipEvents recorded on
              the launch stream (every EV_EVERY-th timed step), against
              8 TB/s; the read-only fraction
              beside it; traffic = HBM bytes per launch from the committed
              rocprofv3 PMC summary (profiles/pmc_latest.json)
  cpu_baseline  the oracle (CPU restatement of libbjxa's decode, 1 thread)
              on the same stream, rank 0 at N=1 only: median of 5 passes
              after a discarded first pass (the bit-exact check)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (eblocks per rank, bits, channels, description)
    "C2": (10_000_000, 8, 1, "C2: 8-bit mono XA stream, 10,000,000 blocks"),
    "C3": (5_000_000, 8, 2, "C3: 8-bit stereo XA stream, 5,000,000 eblocks"),
}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
CPU_PASSES = 5
# hipEvent pairs around the spec kernel are recorded on every EV_EVERY-th
# timed step only: a timing event drains the stream (measured +5.5 us per
# step when recorded on every step)
EV_EVERY = 5


def hip_runtime():
    """The HIP runtime torch already loaded (same soname)."""
    L = ctypes.CDLL("libamdhip64.so.7")
    L.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                      ctypes.c_void_p]
    L.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    L.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return L


def reduce_over_ranks(elapsed, ok, dev):
    """Whole-job view of one rank's result: the max of the timed region over
    ranks and the AND of the bit-exact checks (None = not checked counts as
    passing).  RCCL on the GPU box; the gloo test runs it on CPU tensors."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([1 if ok in (None, True) else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    return float(t.item()), (bool(okt.item()) if ok is not None else None)


def job_value(samples_per_rank, world, steps, elapsed):
    """MSamples/s of the whole job: every rank decodes its own stream."""
    return samples_per_rank * world * steps / elapsed / 1e6


def host_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run_workload(name, args, dev, world, rank, verify, cpu_leg):
    """Decode one seeded stream `args.steps` times (after `args.warmup`
    untimed steps); returns the measurements of this rank."""
    import torch
    import torch.distributed as dist
    import bjxa_amd
    from bjxa_amd import synth

    eb, bits, ch, desc = WORKLOADS[name]
    samples = eb * 32 * ch
    xa_np = synth.stream(eb, bits, ch, args.mix, seed=rank)
    src = torch.from_numpy(xa_np).to(dev)
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
    ws_len = bjxa_amd.decode_workspace_size(eb, ch, args.chunk, args.warm_blocks)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device=dev)
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bjxa_amd.workspace_init(ws.data_ptr(), ws_len, sh)

    hip = hip_runtime()
    nev = args.steps + args.warmup
    evs = []
    for _ in range(nev):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        hip.hipEventCreate(ctypes.byref(a))
        hip.hipEventCreate(ctypes.byref(b))
        evs.append((a.value, b.value))

    def step(i):
        ev = evs[i] if (i - args.warmup) % EV_EVERY == 0 else (None, None)
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0),
                               args.chunk, args.warm_blocks, sh, ev)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.warmup, nev):
        step(i)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0

    spec_ms = []
    for i in range(args.warmup, nev):
        if (i - args.warmup) % EV_EVERY:
            continue
        a, b = evs[i]
        ms = ctypes.c_float()
        hip.hipEventSynchronize(b)
        hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
        spec_ms.append(ms.value)
    for a, b in evs:
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
    st = status.cpu().numpy().view(np.uint32).copy()

    ok, cpu = None, None
    if verify or cpu_leg:
        import oracle
        out = dst.cpu().numpy().view(np.int16)
        ref, _, _, _ = oracle.decode(xa_np, eb, bits, ch)   # also the discarded pass
        ok = bool(np.array_equal(out, ref))
        del out
        if cpu_leg:
            times = []
            for _ in range(CPU_PASSES):
                t = time.perf_counter()
                oracle.decode(xa_np, eb, bits, ch, out=ref)
                times.append(time.perf_counter() - t)
            med = float(np.median(times))
            cpu = {"value": round(samples / med / 1e6, 1), "unit": "MSamples/s", "cores": 1,
                   "kind": "port",
                   "sample": "the full %s stream (%d samples), oracle/xa_oracle.c single-pass "
                             "decode on 1 thread, median of %d passes after a discarded first; "
                             "host CPU: %s" % (name, samples, CPU_PASSES, host_cpu())}
        del ref

    xa_bytes = eb * ch * (bits * 4 + 1)
    return {"name": name, "desc": desc, "eb": eb, "bits": bits, "ch": ch, "samples": samples,
            "elapsed": elapsed, "spec_ms": float(np.mean(spec_ms)), "status": st,
            "xa_bytes": xa_bytes, "alg_bytes": xa_bytes + eb * 64 * ch, "ok": ok, "cpu": cpu}


BATCHES = {
    # C4 = 1024 mixed-format streams; C5 = 1024 8-bit stereo
    # streams of 65,536 eblocks over 8 GPUs -- "C5g" is one GPU's share
    "C4": "C4: 1024 streams, bits (4,6,8)[i%3], channels 1+((i/3)&1), 16,384 eblocks each",
    "C5g": "C5 per-GPU share at 8 GPUs: 128 8-bit stereo streams of 65,536 eblocks",
    "C5": "C5: 1024 8-bit stereo streams of 65,536 eblocks, a contiguous share per rank",
}


def batch_specs(name, nstreams=0):
    if name == "C4":
        n = nstreams or 1024
        return [((4, 6, 8)[i % 3], 1 + ((i // 3) & 1), 16384) for i in range(n)]
    if name == "C5":
        return [(8, 2, 65536)] * (nstreams or 1024)
    return [(8, 2, 65536)] * (nstreams or 128)


def shard_range(n, rank, world):
    """Contiguous share [lo, hi) of n streams for `rank` of `world`."""
    return rank * n // world, (rank + 1) * n // world


def run_batch(name, steps, warmup, dev, verify, nstreams=0, rank=0, world=1):
    """Decode a batch config (bjxa_hip_batch_*: all streams per launch)
    `steps` times after `warmup` untimed steps.  With world > 1 this rank
    takes a contiguous share of the streams (seeded by global index, so the
    job is the same at every N) and the timed region is bracketed by
    barriers."""
    import torch
    import torch.distributed as dist
    import bjxa_amd
    from bjxa_amd import synth
    specs = batch_specs(name, nstreams)
    lo, hi = shard_range(len(specs), rank, world)
    xas, srcs, dsts, streams = [], [], [], []
    samples = alg = 0
    for i in range(lo, hi):
        bits, ch, eb = specs[i]
        xa = synth.stream(eb, bits, ch, "A", seed=1000 + i)
        s = torch.from_numpy(xa).to(dev)
        d = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
        xas.append(xa)
        srcs.append(s)
        dsts.append(d)
        streams.append({"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb,
                        "bits": bits, "channels": ch})
        samples += eb * 32 * ch
        alg += xa.nbytes + eb * 64 * ch
    specs = specs[lo:hi]
    status = torch.zeros(len(specs) * bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    hip = hip_runtime()
    evs = []
    for _ in range(steps + warmup):
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        hip.hipEventCreate(ctypes.byref(a))
        hip.hipEventCreate(ctypes.byref(b))
        evs.append((a.value, b.value))
    with bjxa_amd.Batch(streams, stream=sh) as batch:
        for i in range(warmup):
            batch.decode(status.data_ptr(), sh, evs[i])
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(warmup, warmup + steps):
            batch.decode(status.data_ptr(), sh,
                         evs[i] if (i - warmup) % EV_EVERY == 0 else (None, None))
        torch.cuda.synchronize(dev)
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        dt = elapsed / steps
    spec = []
    for i in range(warmup, warmup + steps):
        if (i - warmup) % EV_EVERY:
            continue
        a, b = evs[i]
        f = ctypes.c_float()
        hip.hipEventElapsedTime(ctypes.byref(f), a, b)
        spec.append(f.value)
    for a, b in evs:
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
    spec_ms = float(np.mean(spec))
    st = status.cpu().numpy().view(np.uint32).reshape(len(specs), -1)
    ok = None
    if verify:
        import oracle
        ok = True
        for (bits, ch, eb), xa, d in zip(specs, xas, dsts):
            ref, _, _, _ = oracle.decode(xa, eb, bits, ch)
            if not np.array_equal(d.cpu().numpy().view(np.int16), ref):
                ok = False
                break
    return {"workload": BATCHES.get(name, name), "streams": len(specs),
            "samples": samples, "elapsed": elapsed,
            "value": round(samples / dt / 1e6, 1), "unit": "MSamples/s",
            "ms_per_step": round(dt * 1e3, 4), "spec_ms": round(spec_ms, 4),
            "frac": round(alg / (spec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "alg_bytes": alg, "repaired": int(st[:, 3].sum()), "tail": int(st[:, 4].sum()),
            "chunks": int(st[:, 5].sum()), "bit_exact": ok}


def run_encode(steps, warmup, dev, verify):
    """bjxa_hip_encode_async on C3-shaped PCM (5,000,000 8-bit stereo
    eblocks = 320M samples), the GPU side of bjxa_encode()."""
    import torch
    import bjxa_amd
    from bjxa_amd import synth
    eb, bits, ch = 5_000_000, 8, 2
    frames = eb * 32
    pcm = synth.pcm(frames, ch, seed=3)
    src = torch.from_numpy(pcm).to(dev)
    nxa = eb * ch * (bits * 4 + 1)
    dst = torch.empty(nxa, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(warmup):
        bjxa_amd.encode_device(src.data_ptr(), frames, bits, ch, dst.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(steps):
        bjxa_amd.encode_device(src.data_ptr(), frames, bits, ch, dst.data_ptr(), sh)
    e1.record()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    ms = e0.elapsed_time(e1) / steps
    ok = None
    if verify:
        import oracle
        ok = bool(np.array_equal(dst.cpu().numpy(), oracle.encode(pcm, frames, bits, ch)))
    alg = pcm.nbytes + nxa
    return {"workload": "encode, C3-shaped: 320M int16 samples (8-bit stereo) -> XA",
            "value": round(frames * ch / dt / 1e6, 1), "unit": "MSamples/s",
            "ms_per_step": round(dt * 1e3, 4), "kernel_ms": round(ms, 4),
            "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes": alg,
            "byte_exact": ok}


def pmc_traffic(workload, mix):
    """HBM bytes per spec launch from the committed PMC summary, if it was
    taken on this workload and mix."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("workload") == workload and d.get("mix") == mix:
        return d.get("hbm_bytes_per_launch"), d.get("source")
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="C3", choices=sorted(WORKLOADS) + ["C5"],
                    help="C3/C2: one stream per rank (weak scaling); C5: 1024 "
                         "streams split over the ranks (strong scaling)")
    ap.add_argument("--mix", default="A", choices=["A", "F", "W", "Z"])
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--warm-blocks", type=int, default=-1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-other", action="store_true",
                    help="skip the C2/C4/C5g lines at N=1")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    if args.workload == "C5":
        return main_c5(args, dev, world, rank)

    cpu_leg = rank == 0 and world == 1 and not args.no_cpu
    r = run_workload(args.workload, args, dev, world, rank, not args.no_verify, cpu_leg)
    elapsed, ok = r["elapsed"], r["ok"]
    if world > 1:
        elapsed, ok = reduce_over_ranks(elapsed, ok, dev)

    other = {}
    if world == 1 and not args.no_other:
        for name in sorted(WORKLOADS):
            if name == args.workload:
                continue
            o = run_workload(name, args, dev, 1, rank, not args.no_verify, False)
            other[name] = {
                "workload": o["desc"], "value": round(job_value(o["samples"], 1, args.steps,
                                                                o["elapsed"]), 1),
                "unit": "MSamples/s", "ms_per_step": round(o["elapsed"] / args.steps * 1e3, 4),
                "spec_ms": round(o["spec_ms"], 4),
                "frac": round(o["alg_bytes"] / (o["spec_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "chunk": int(o["status"][6]), "bit_exact": o["ok"]}
            ok = ok if o["ok"] in (None, True) else False
        for name in sorted(BATCHES):
            o = run_batch(name, args.steps, args.warmup, dev, not args.no_verify)
            other[name] = o
            ok = ok if o["bit_exact"] in (None, True) else False
        o = run_encode(args.steps, args.warmup, dev, not args.no_verify)
        other["encode_C3"] = o
        ok = ok if o["byte_exact"] in (None, True) else False

    st = r["status"]
    achieved = r["alg_bytes"] / (r["spec_ms"] * 1e-3) / 1e9
    read_gbs = r["xa_bytes"] / (r["spec_ms"] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(args.workload, args.mix)
    line = {
        "metric": "decoded PCM MSamples/s (+ achieved HBM GB/s vs roofline), bit-exact vs CPU",
        "value": round(job_value(r["samples"], world, args.steps, elapsed), 1),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32+f32",
        "data": "synthetic (seeded XA stream, profile mix %s, uniform codes)" % args.mix,
        "config": {"workload": r["desc"] + " per rank", "workload_id": args.workload,
                   "bits": r["bits"], "channels": r["ch"],
                   "eblocks_per_rank": r["eb"], "samples_per_rank": r["samples"],
                   "profile_mix": args.mix, "parallelism": "independent streams, 1 per GPU",
                   "chunk": int(st[6]), "warmup_eblocks": int(st[7]),
                   "tuning": "auto" if not args.chunk and args.warm_blocks < 0 else "manual"},
        "roofline": {"bound": "hbm", "kernel": "xa_decode_spec",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "alg_bytes_per_launch": r["alg_bytes"], "traffic_source": traffic_src,
                     "read_only_achieved": round(read_gbs, 1),
                     "read_only_frac": round(read_gbs / HBM_PEAK_GBS, 4),
                     "launch_ms": round(r["spec_ms"], 4)},
        "cpu_baseline": r["cpu"],
        "bit_exact": ok,
        "repaired_chunks": int(st[3]), "tail_repairs": int(st[4]), "chunks": int(st[5]),
    }
    if other:
        line["other_configs"] = other
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok in (None, True) else 1


def main_c5(args, dev, world, rank):
    """C5: the fixed job of 1024 8-bit stereo streams (65,536 eblocks each)
    split over the ranks -- strong scaling, no data-path collective."""
    import torch.distributed as dist
    r = run_batch("C5", args.steps, args.warmup, dev, not args.no_verify, 0, rank, world)
    elapsed, ok = r["elapsed"], r["bit_exact"]
    if world > 1:
        elapsed, ok = reduce_over_ranks(elapsed, ok, dev)
    total = 1024 * 65536 * 64
    line = {
        "metric": "decoded PCM MSamples/s (+ achieved HBM GB/s vs roofline), bit-exact vs CPU",
        "value": round(total * args.steps / elapsed / 1e6, 1), "unit": "MSamples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int32+f32",
        "data": "synthetic (seeded XA streams, profile mix A, uniform codes)",
        "config": {"workload": BATCHES["C5"], "workload_id": "C5",
                   "streams_per_rank": r["streams"],
                   "parallelism": "stream shards, one batched launch per GPU"},
        "roofline": {"bound": "hbm", "kernel": "xa_decode_spec_batch (rank 0)",
                     "achieved": round(r["alg_bytes"] / (r["spec_ms"] * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": r["frac"],
                     "traffic": None, "alg_bytes_per_launch": r["alg_bytes"],
                     "launch_ms": r["spec_ms"]},
        "cpu_baseline": None, "bit_exact": ok,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok in (None, True) else 1


if __name__ == "__main__":
    sys.exit(main())
