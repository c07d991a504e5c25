#!/usr/bin/env python3
"""bench.py -- XA ADPCM decode throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path (bjxa_hip_decode_async: speculative
decode + verify/repair + tail) over one synthetic XA stream already resident
in HBM.  Default workload is BASELINE config C3: one 8-bit stereo stream of
5,000,000 effective blocks (320M int16 samples), profile mix A.

Multi-GPU (torchrun, one process per GPU): every rank decodes its own
C3-sized stream (independent objects, no data-path collective), so per-GPU
work is fixed: "scaling": "weak".  RCCL carries only the barrier and the
max-over-ranks time.

Reported:
  value       decoded MSamples/s of the whole job (all ranks) over the timed
              steps (barrier + synchronize on both sides, max over ranks)
  roofline    xa_decode_spec, the dominant kernel: algorithmic bytes per
              launch (XA read + PCM written, SURVEY.md §8(d): 3.03125 B per
              8-bit sample) / its mean duration from hipEvents recorded on
              the launch stream, against 8 TB/s; traffic from the committed
              rocprofv3 PMC summary (profiles/pmc_latest.json) if present
  cpu_baseline  the oracle (CPU restatement of libbjxa's decode, 1 thread)
              on the same stream, rank 0 at N=1 only; also the bit-exact check
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="C3", choices=sorted(WORKLOADS))
    ap.add_argument("--mix", default="A", choices=["A", "F", "W", "Z"])
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--warm-blocks", type=int, default=-1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-verify", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import bjxa_amd
    from bjxa_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    eb, bits, ch, desc = WORKLOADS[args.workload]
    samples = eb * 32 * ch
    xa_np = synth.stream(eb, bits, ch, args.mix, seed=rank)
    src = torch.from_numpy(xa_np).to(dev)
    dst = torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
    ws_len = bjxa_amd.decode_workspace_size(eb, ch, args.chunk, args.warm_blocks)
    ws = torch.zeros(ws_len, dtype=torch.uint8, device=dev)
    status = torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
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
        bjxa_amd.decode_device(src.data_ptr(), dst.data_ptr(), eb, eb * 32, bits, ch,
                               ws.data_ptr(), ws_len, status.data_ptr(), (0, 0, 0, 0),
                               args.chunk, args.warm_blocks, sh, evs[i])

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
    for a, b in evs[args.warmup:]:
        ms = ctypes.c_float()
        hip.hipEventSynchronize(b)
        hip.hipEventElapsedTime(ctypes.byref(ms), a, b)
        spec_ms.append(ms.value)
    spec_avg_ms = float(np.mean(spec_ms))
    st = status.cpu().numpy().view(np.uint32)

    # bit-exact check of the last step against the oracle
    ok = None
    cpu = None
    if not args.no_verify or (rank == 0 and world == 1 and not args.no_cpu):
        import oracle
        out = dst.cpu().numpy().view(np.int16)
        t = time.perf_counter()
        ref, _, _, _ = oracle.decode(xa_np, eb, bits, ch)
        t_cpu = time.perf_counter() - t
        ok = bool(np.array_equal(out, ref))
        del ref
        if rank == 0 and world == 1 and not args.no_cpu:
            # two more timed single-thread passes; report the best
            times = [t_cpu]
            for _ in range(2):
                t = time.perf_counter()
                oracle.decode(xa_np, eb, bits, ch)
                times.append(time.perf_counter() - t)
            best = min(times)
            cpu = {"value": round(samples / best / 1e6, 1), "unit": "MSamples/s", "cores": 1,
                   "kind": "port",
                   "sample": "the full %s stream (%d samples), oracle/xa_oracle.c "
                             "single-pass decode, 1 thread, best of 3" % (args.workload, samples)}
    if world > 1:
        elapsed, ok = reduce_over_ranks(elapsed, ok, dev)

    xa_bytes = eb * ch * (bits * 4 + 1)
    pcm_bytes = eb * 64 * ch
    alg_bytes = xa_bytes + pcm_bytes
    achieved = alg_bytes / (spec_avg_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                p = json.load(f)
            if p.get("workload") == args.workload and p.get("mix") == args.mix:
                traffic = p.get("hbm_bytes_per_launch")
                traffic_src = p.get("source")
        except (OSError, ValueError):
            traffic = None

    value = job_value(samples, world, args.steps, elapsed)
    line = {
        "metric": "decoded PCM MSamples/s (+ achieved HBM GB/s vs roofline), bit-exact vs CPU",
        "value": round(value, 1),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded XA stream, profile mix %s, uniform codes)" % args.mix,
        "config": {"workload": desc + " per rank", "workload_id": args.workload,
                   "bits": bits, "channels": ch,
                   "eblocks_per_rank": eb, "samples_per_rank": samples,
                   "profile_mix": args.mix, "parallelism": "independent streams, 1 per GPU",
                   "chunk": int(st[6]), "warmup_eblocks": int(st[7]),
                   "tuning": "auto" if not args.chunk and args.warm_blocks < 0 else "manual"},
        "roofline": {"bound": "hbm", "kernel": "xa_decode_spec",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "alg_bytes_per_launch": alg_bytes, "traffic_source": traffic_src,
                     "launch_ms": round(spec_avg_ms, 4)},
        "cpu_baseline": cpu,
        "bit_exact": ok,
        "repaired_chunks": int(st[3]), "tail_repairs": int(st[4]), "chunks": int(st[5]),
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    for a, b in evs:
        hip.hipEventDestroy(a)
        hip.hipEventDestroy(b)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok in (None, True) else 1


if __name__ == "__main__":
    sys.exit(main())
