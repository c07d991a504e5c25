#!/usr/bin/env python3
"""bench.py -- XA ADPCM decode throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one synthetic input already
resident in HBM.

N = 1 (default): BASELINE config C3 -- one 8-bit stereo stream of 5,000,000
effective blocks (320M int16 samples), profile mix A, decoded by
bjxa_hip_decode_async (speculative decode + verify/repair/tail).  The same
run measures, under "other_configs": C2 (one 8-bit mono stream of 10M
blocks), C4 (1024 mixed-format streams per launch), C5 (the whole 1024-stream
job on this GPU: the N = 1 point of the scaling curve), C5g (one GPU's share
of C5 at 8 GPUs) and the encode direction on C3-shaped PCM, each in a child
process of its own started before this one touches the GPU, so every
configuration allocates its buffers in a fresh process as a caller (or one
rank of the N > 1 job) would (in one process the C5g
share landed where it ran 20 % slower).  --no-other skips them.

N > 1 (`--gpus N`): BASELINE config C5 -- 1024 8-bit stereo streams of
65,536 eblocks, a fixed job split into contiguous shares, one rank per GPU,
one batched launch per rank per step: "scaling": "strong".  Without
WORLD_SIZE in the environment, bench.py starts the N ranks itself (a child
`torch.distributed.run`, before anything touches the GPU) and passes its
exit status through; under torchrun it is one of the ranks.  The data path
has no collective (streams are independent); RCCL carries the control plane
of SURVEY.md §5: the barriers, the max over ranks of the timed region,
AllReduce(sum) of the counters, AllReduce(min) of the first failing stream,
and an AllGather of every stream's 64-bit PCM checksum, which rank 0 checks
against the oracle's.  C3 on every rank (weak scaling) is reported under
other_configs.

Reported:
  value       decoded MSamples/s of the whole job over the timed steps
              (barrier + synchronize on both sides, max over ranks); with
              --pipeline D (default 0: 1 or 2 by a calibration run after
              the warm-up) consecutive steps run on D HIP
              streams with their own input copy and output/workspace
              buffers (no slot can hit another's input in a cache), so one
              step's tail overlaps the next step's head; every step is a
              whole decode, and ms_per_step_serial times the same steps one
              at a time
  roofline    the dominant kernel (xa_decode_spec; xa_decode_spec_batch for
              C5): algorithmic bytes per launch (XA read + PCM written,
              SURVEY.md §8(d): 3.03125 B per 8-bit sample) / its median
              duration over >= 20 launches timed with hipEvents recorded on
              the launch stream in a separate pass after the timed region,
              against 8 TB/s; the read-only fraction beside it; traffic =
              HBM bytes per launch from the committed rocprofv3 PMC summary
              (profiles/pmc_latest.json) when it was taken on this workload
  cpu_baseline  rank 0 at N = 1, for every line: the oracle (CPU
              restatement of libbjxa's decode/encode): C2/C3 and the encode on
              1 thread (a stream is serial), C4/C5/C5g on all host cores the
              process may use (its affinity mask; BJXA_CPU_THREADS lowers
              it), one decoder per thread, streams round-robin; median of 5
              passes after a discarded first

CPU rehearsal: BJXA_BENCH_BACKEND=gloo runs the N > 1 path on CPU (gloo,
small job via --streams/--eblocks), decoding each rank's share with the
library's host API on its CPU core; tests/test_dist.py drives it.
BJXA_BENCH_BACKEND=gloo-gpu runs it on a one-GPU box: every rank decodes its
share with the batched kernels on GPU 0 and the control plane runs over
gloo (tests/test_gpu_bench.py drives it at 2 and 3 ranks).
"""
import argparse
import contextlib
import ctypes
import datetime
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (eblocks per rank, bits, channels, description)
    "C2": (10_000_000, 8, 1, "C2: 8-bit mono XA stream, 10,000,000 blocks"),
    "C3": (5_000_000, 8, 2, "C3: 8-bit stereo XA stream, 5,000,000 eblocks"),
}
BATCHES = {
    # C4 = 1024 mixed-format streams; C5 = 1024 8-bit stereo
    # streams of 65,536 eblocks over 1-8 GPUs -- "C5g" is one GPU's share at 8
    "C4": "C4: 1024 streams, bits (4,6,8)[i%3], channels 1+((i/3)&1), 16,384 eblocks each",
    "C5": "C5: 1024 8-bit stereo streams of 65,536 eblocks, a contiguous share per rank",
    "C5g": "C5 per-GPU share at 8 GPUs: 128 8-bit stereo streams of 65,536 eblocks",
}
METRIC = "decoded PCM MSamples/s (+ achieved HBM GB/s vs roofline), bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
CPU_PASSES = 5
EV_SAMPLES = 20         # launches timed with events, after the timed region
NO_ERROR = 0xFFFFFFFF
# every collective (and the rendezvous) of a rank gives up after this long, so
# a stuck rank ends the job with its rank named instead of hanging for
# torch's default 10 minutes
PG_TIMEOUT_S = float(os.environ.get("BJXA_BENCH_PG_TIMEOUT", "180"))
FIRST_ERR_NONE = (1 << 62)


# ---- process plumbing --------------------------------------------------------

def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_pg(backend, **kw):
    """Join the job's process group with PG_TIMEOUT_S on every collective."""
    import torch.distributed as dist
    dist.init_process_group(backend, timeout=datetime.timedelta(seconds=PG_TIMEOUT_S), **kw)


def stall_for_test(rank):
    """tests/test_dist.py: BJXA_BENCH_STALL_RANK=r makes rank r sleep
    BJXA_BENCH_STALL_S seconds before its first collective (a stuck rank)."""
    if os.environ.get("BJXA_BENCH_STALL_RANK", "") == str(rank):
        time.sleep(float(os.environ.get("BJXA_BENCH_STALL_S", "60")))


def launch_ranks(n):
    """Start n ranks of this script under torch.distributed.run (one process
    per GPU) from a parent that has not touched the GPU, and return their
    exit status.  The ranks' stdout (rank 0's JSON line) passes through."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % n, "--master-addr=127.0.0.1",
           "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def hip_runtime():
    """The HIP runtime torch already loaded (same soname)."""
    L = ctypes.CDLL("libamdhip64.so.7")
    L.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    L.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p,
                                      ctypes.c_void_p]
    L.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    L.hipEventDestroy.argtypes = [ctypes.c_void_p]
    return L


class EventPairs:
    """hipEvent pairs recorded around the spec kernel on the launch stream
    (torch.cuda.Event only sees torch's current stream)."""

    def __init__(self, n):
        self.hip = hip_runtime()
        self.hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self.ev = []
        for _ in range(n):
            a, b = ctypes.c_void_p(), ctypes.c_void_p()
            self.hip.hipEventCreate(ctypes.byref(a))
            self.hip.hipEventCreate(ctypes.byref(b))
            self.ev.append((a.value, b.value))

    def ms(self):
        out = []
        for a, b in self.ev:
            f = ctypes.c_float()
            self.hip.hipEventSynchronize(b)
            self.hip.hipEventElapsedTime(ctypes.byref(f), a, b)
            out.append(f.value)
        return out

    def close(self):
        for a, b in self.ev:
            self.hip.hipEventDestroy(a)
            self.hip.hipEventDestroy(b)


def reduce_over_ranks(elapsed, ok, dev):
    """Whole-job view of one rank's result: the max of the timed region over
    ranks and the AND of the bit-exact checks (None = not checked counts as
    passing).  RCCL on the GPU box; the gloo tests run it on CPU tensors."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([1 if ok in (None, True) else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    return float(t.item()), (bool(okt.item()) if ok is not None else None)


def dist_on():
    """True when this rank is in a process group (any world size): the
    control-plane collectives then run through it, RCCL on the GPU box --
    also at world size 1 under --force-pg, so that one GPU executes the
    exact collectives the N > 1 line issues."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def job_value(samples_per_rank, world, steps, elapsed):
    """MSamples/s of a weak-scaling job: every rank decodes its own stream."""
    return samples_per_rank * world * steps / elapsed / 1e6


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cpu.max quota /
    period), or None: a GPU box shows all its cores in the affinity mask
    but may grant only a per-GPU share of their time."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def host_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """Threads for the batch CPU baseline: every core in this process's
    affinity mask (BASELINE.md "all online host cores"), unless
    BJXA_CPU_THREADS lowers it (a shared box's per-GPU share).  Returns
    (threads, cores in the affinity mask, CPUs online)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    n = aff
    cap = os.environ.get("BJXA_CPU_THREADS", "")
    if cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n), aff, os.cpu_count()


# ---- PCM checksums (the AllGather payload) -------------------------------------

def pcm_checksum_np(pcm_i16):
    """64-bit position-weighted checksum of an int16 PCM array (wrapping
    int64 arithmetic, so any summation order gives the same value)."""
    x = pcm_i16.astype(np.int64)
    w = (np.arange(x.size, dtype=np.int64) % 65521) + 1
    with np.errstate(over="ignore"):
        return int(np.sum(x * w, dtype=np.int64))


def pcm_checksum_torch(buf_u8, n):
    """The same checksum of the first n int16 of a device byte buffer."""
    import torch
    x = buf_u8[:2 * n].view(torch.int16).to(torch.int64)
    w = torch.arange(n, dtype=torch.int64, device=x.device) % 65521 + 1
    return int((x * w).sum().item())


# ---- one long stream per rank (C2/C3) ----------------------------------------

def timed_serial(step, steps, dev):
    """The same steps one at a time on slot 0 (no overlap between steps),
    reported beside a pipelined timing; this rank only, no barrier."""
    import torch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(0)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def timed_region(step, steps, depth, slots, dev):
    """The timed region: `steps` steps (consecutive slots when depth > 1,
    else slot 0), bracketed by a barrier (N > 1) and device synchronizes,
    and nothing else on the streams.  Then the same steps once more with a
    hipEvent pair recorded around each on its slot's stream, untimed, for
    the spread of the steps: an event between two steps costs the step
    after it ~4 % on C3 (tools/window_probe.py), which is
    why round 4's timed window, which held them, ran slower than the same
    loop without them.  Returns (wall seconds, per-step event ms)."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize(dev)
    if dist_on():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i if depth > 1 else 0)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist_on():
        dist.barrier()
    evs = EventPairs(steps)
    rec = evs.hip.hipEventRecord
    for i in range(steps):
        k = i if depth > 1 else 0
        sh = slots[k % len(slots)]["sh"]
        rec(evs.ev[i][0], sh)
        step(k)
        rec(evs.ev[i][1], sh)
    ms = evs.ms()
    evs.close()
    torch.cuda.synchronize(dev)
    return elapsed, ms


def spread(ms, depth=1):
    """min / median / max of per-step event times (ms)"""
    if not ms:
        return None
    what = ("hipEvents around each step of a pass of the same steps right after the "
            "timed region (outside it: an event between steps slows the next one), "
            "on its stream")
    if depth > 1:
        what += ("; %d steps in flight, so each span also holds the overlapping steps' "
                 "share of the chip (ms_per_step is the throughput)" % depth)
    return {"min": round(float(np.min(ms)), 4), "median": round(float(np.median(ms)), 4),
            "max": round(float(np.max(ms)), 4), "n": len(ms), "what": what}


PIPE_CAL_STEPS = 20     # steps per calibration run of --pipeline 0
PIPE_CAL_ROUNDS = 4     # interleaved runs per depth
PIPE_CAL_MARGIN = 0.01  # two in flight must win by this much


def py_median(v):
    """Median in plain Python.  Not numpy: the first np.median of a process
    pauses the host ~8 ms (lazy imports), and a GPU left idle that long
    before the timed window ran it 3 % slower on C3 and 15 % on C4 (and
    the one-at-a-time pass after it), reproducibly;
    nothing numpy runs between the calibration and the timed loops."""
    s = sorted(v)
    n = len(s)
    return (s[(n - 1) // 2] + s[n // 2]) / 2.0


def calibration_pass(step, nslots, dev):
    """PIPE_CAL_ROUNDS runs of PIPE_CAL_STEPS steps one at a time and with
    every slot in flight, interleaved; wall seconds of each run per depth."""
    import torch
    t = {1: [], nslots: []}
    for _ in range(PIPE_CAL_ROUNDS):
        for d in (1, nslots):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(PIPE_CAL_STEPS):
                step(i if d > 1 else 0)
            torch.cuda.synchronize(dev)
            t[d].append(time.perf_counter() - t0)
    return t


def choose_depth(step, nslots, dev, want):
    """Steps in flight for the timed region.  want >= 1: that many (up to
    the slots made).  want == 0 (auto, the default): after the warm-up,
    PIPE_CAL_STEPS steps one at a time and the same with every slot in
    flight, PIPE_CAL_ROUNDS times each, interleaved, in two passes of which
    the second decides (the first settles the GPU); steps in flight are
    timed only if every run of them beats every run one at a time by
    PIPE_CAL_MARGIN
    (round 2: two in flight won 4 % on C3 and lost 3-10 % on C4/C5g on the
    driver's box; on C3 the two are often within noise).  Returns (depth,
    median calibration ms per step, or None)."""
    if want >= 1 or nslots == 1:
        return max(1, min(want, nslots)), None
    # the first pass only settles the GPU: a timed window right after a
    # single pass ran 0.5-3 % slower on C3 and 2-8 % on C2, whose second
    # pass also shows two in flight winning
    calibration_pass(step, nslots, dev)
    t = calibration_pass(step, nslots, dev)
    med = {d: py_median(v) for d, v in t.items()}
    # steps in flight only if their slowest run beats the fastest run one at
    # a time: how two in-flight steps interleave depends on host timing, and
    # a config whose runs spread (C4: 0.45-0.51 ms) is
    # timed one at a time
    best = nslots if max(t[nslots]) < min(t[1]) * (1.0 - PIPE_CAL_MARGIN) else 1
    cal = {"depth%d_ms" % d: round(v / PIPE_CAL_STEPS * 1e3, 4) for d, v in med.items()}
    cal["runs_ms"] = {"depth%d" % d: [round(x / PIPE_CAL_STEPS * 1e3, 4) for x in v]
                      for d, v in t.items()}
    return best, cal


def pipeline_slots(depth, dev, make):
    """`depth` independent sets of output/workspace buffers, each with a HIP
    stream of its own (slot 0 on torch's current stream).  Consecutive steps
    go to consecutive slots, so step i+1's spec kernel can take the CUs that
    step i's tail leaves idle and step i's verify/repair kernel runs beside
    it; step i+depth reuses slot i's buffers after step i on the same
    stream.  Every step is still a whole decode of its batch.  make(k)
    builds slot k's buffers (slots k >= 1 copy the input, so no step reads
    another slot's input out of a cache)."""
    import torch
    slots = []
    for k in range(max(1, depth)):
        st = torch.cuda.current_stream(dev) if k == 0 else torch.cuda.Stream(dev)
        sl = make(k)
        sl["stream"] = st
        sl["sh"] = st.cuda_stream
        slots.append(sl)
    return slots


def run_workload(name, args, dev, world, rank, verify, cpu_leg):
    """Decode one seeded stream `args.steps` times (after `args.warmup`
    untimed steps), then time EV_SAMPLES more launches with events;
    returns the measurements of this rank."""
    import torch
    import torch.distributed as dist
    import bjxa_amd
    from bjxa_amd import synth

    eb, bits, ch, desc = WORKLOADS[name]
    samples = eb * 32 * ch
    xa_np = synth.stream(eb, bits, ch, args.mix, seed=rank)
    src = torch.from_numpy(xa_np).to(dev)
    ws_len = bjxa_amd.decode_workspace_size(eb, ch, args.chunk, args.warm_blocks,
                                            args.variant)
    slots = pipeline_slots(args.pipeline or 2, dev, lambda k: {
        "src": src if k == 0 else src.clone(),
        "dst": torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev),
        "ws": torch.zeros(ws_len, dtype=torch.uint8, device=dev),
        "status": torch.zeros(bjxa_amd.STATUS_WORDS, dtype=torch.int32, device=dev)})
    for sl in slots:
        bjxa_amd.workspace_init(sl["ws"].data_ptr(), ws_len, sl["sh"])
    torch.cuda.synchronize(dev)

    def step(i, ev=(None, None)):
        sl = slots[i % len(slots)]
        bjxa_amd.decode_device(sl["src"].data_ptr(), sl["dst"].data_ptr(), eb, eb * 32, bits, ch,
                               sl["ws"].data_ptr(), ws_len, sl["status"].data_ptr(),
                               (0, 0, 0, 0), args.chunk, args.warm_blocks, sl["sh"], ev,
                               args.variant)

    for i in range(args.warmup):
        step(i)
    depth, cal = choose_depth(step, len(slots), dev, args.pipeline)
    elapsed, step_ms = timed_region(step, args.steps, depth, slots, dev)

    serial = timed_serial(step, args.steps, dev) if depth > 1 else elapsed
    # diagnostic (BJXA_BENCH_RECAL=1): the calibration once more after the
    # timed loops, to tell drift over the run from the window itself
    recal = None
    if os.environ.get("BJXA_BENCH_RECAL") == "1":
        # (with one slot there is nothing to calibrate: choose_depth gives None)
        recal = choose_depth(step, len(slots), dev, 0)[1] or {}
        # the timed window's loop and the calibration's, interleaved
        seq = []
        for _ in range(3):
            seq.append(("window", round(timed_region(step, args.steps, depth, slots,
                                                      dev)[0] / args.steps * 1e3, 4)))
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i in range(args.steps):
                step(i if depth > 1 else 0)
            torch.cuda.synchronize(dev)
            seq.append(("loop", round((time.perf_counter() - t0) / args.steps * 1e3, 4)))
        recal["interleaved"] = seq

    # kernel timing: slot 0 alone, one launch at a time (no overlap)
    evs = EventPairs(max(EV_SAMPLES, args.steps))
    for ev in evs.ev:
        step(0, ev)
    spec_ms = evs.ms()
    evs.close()
    torch.cuda.synchronize(dev)
    cold = cold_single(step, dev) if rank == 0 else None
    st = slots[0]["status"].cpu().numpy().view(np.uint32).copy()
    # every slot's PCM and the status words the API defines (first error,
    # exit state, plan) equal slot 0's; the repair counters (words 3, 4)
    # may differ: whether a wave's boundary is repaired inside K1 or by the
    # tail depends on timing when other kernels share the GPU
    st0 = slots[0]["status"].cpu().numpy().view(np.uint32)
    same = all(torch.equal(sl["dst"], slots[0]["dst"]) and
               all(int(a) == int(b) for i, (a, b) in enumerate(zip(
                   sl["status"].cpu().numpy().view(np.uint32), st0)) if i not in (3, 4))
               for sl in slots[1:])

    ok, cpu, exact = None, None, None
    if verify or cpu_leg:
        import oracle
        out = slots[0]["dst"].cpu().numpy().view(np.int16)
        ref, _, _, _ = oracle.decode(xa_np, eb, bits, ch)   # also the discarded pass
        exact = bool(np.array_equal(out, ref))
        ok = exact and same
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
                             "host CPU: %s" % (name, samples, CPU_PASSES, host_cpu()),
                   "why": "libbjxa's CPU path cannot be built here (its autoconf config.h is "
                          "absent), so the baseline is oracle/xa_oracle.c, which restates "
                          "its loop shape for shape (bjxa_decode -> inflate -> "
                          "decode_inflated, src/libbjxa.c:602-661, :286-345, :533-578); "
                          "product_cpu_core is this library's own faster CPU path",
                   "product_cpu_core": product_cpu_core(xa_np, eb, bits, ch)}
        del ref

    xa_bytes = eb * ch * (bits * 4 + 1)
    return {"name": name, "desc": desc, "eb": eb, "bits": bits, "ch": ch, "samples": samples,
            "elapsed": elapsed, "serial": serial, "pipeline": depth, "pipeline_cal": cal,
            "recal": recal,
            "step_ms": spread(step_ms, depth), "spec_ms": float(np.median(spec_ms)),
            "spec_samples": len(spec_ms), "status": st, "xa_bytes": xa_bytes,
            "alg_bytes": xa_bytes + eb * 64 * ch, "ok": ok, "pcm_equal_oracle": exact,
            "slots_agree": same, "cpu": cpu, "cold": cold}


COLD_PAUSE_S = 0.010
COLD_SAMPLES = 7


def cold_single(step, dev):
    """One decode after an idle host pause of COLD_PAUSE_S, as one bjxa(1)
    call on an otherwise idle GPU sees it: the wall
    time from the call to its synchronize (K1 + K2 + launch and sync
    latency) and K1 alone by events; median of COLD_SAMPLES.  After the
    pause the shader clock is at its 2.4 GHz boost; under sustained decoding
    the power manager holds it near 2.0 GHz, dipping to ~1.9 GHz some 15
    decodes in (tools/clock_probe.py), so a cold K1 runs
    slightly faster than a hot one."""
    import torch
    evs = EventPairs(COLD_SAMPLES)
    wall = []
    for ev in evs.ev:
        torch.cuda.synchronize(dev)
        time.sleep(COLD_PAUSE_S)
        t0 = time.perf_counter()
        step(0, ev)
        torch.cuda.synchronize(dev)
        wall.append((time.perf_counter() - t0) * 1e3)
    k1 = evs.ms()
    evs.close()
    return {"wall_ms": round(py_median(wall), 4), "k1_ms": round(py_median(k1), 4),
            "pause_ms": COLD_PAUSE_S * 1e3, "samples": COLD_SAMPLES,
            "what": "one decode (K1 + tail) after an idle host pause: wall = call to "
                    "synchronize; k1 = its spec kernel by hipEvents"}


def product_cpu_core(xa_np, eb, bits, ch, sample_eb=1_000_000):
    """This library's own CPU core (bjxa_decode routed off the GPU,
    bjxa_amd/csrc/xa_cpu.c) on the first `sample_eb` eblocks of the stream,
    1 thread, median of 3 passes after a discarded first."""
    import bjxa_amd
    n = min(eb, sample_eb)
    bsz = (bits * 4 + 1) * ch
    xa = np.ascontiguousarray(xa_np[:n * bsz])
    pcm = np.zeros(n * 32 * ch, np.int16)
    times = []
    with bjxa_amd.offload(None):
        for k in range(4):
            with bjxa_amd.Decoder() as d:
                d.parse_header(bjxa_amd.xa_header(xa.size, n * 32, 44100, bits, ch))
                t = time.perf_counter()
                d.decode(pcm, xa)
                if k:
                    times.append(time.perf_counter() - t)
    med = float(np.median(times))
    return {"value": round(n * 32 * ch / med / 1e6, 1), "unit": "MSamples/s", "cores": 1,
            "sample": "first %d eblocks (%d samples) through bjxa_decode() on the library's "
                      "CPU core (bjxa_amd/csrc/xa_cpu.c), median of 3 passes after a "
                      "discarded first" % (n, n * 32 * ch)}


# ---- batched streams (C4/C5) ------------------------------------------------

def batch_specs(name, nstreams=0, eblocks=0):
    """[(bits, channels, eblocks)] of a batch config."""
    if name == "C4":
        n = nstreams or 1024
        return [((4, 6, 8)[i % 3], 1 + ((i // 3) & 1), eblocks or 16384) for i in range(n)]
    if name == "C5":
        return [(8, 2, eblocks or 65536)] * (nstreams or 1024)
    return [(8, 2, eblocks or 65536)] * (nstreams or 128)


def shard_range(n, rank, world):
    """Contiguous share [lo, hi) of n streams for `rank` of `world`."""
    return rank * n // world, (rank + 1) * n // world


def batch_inputs(name, nstreams, eblocks, lo, hi, bad_stream=-1, mix="A"):
    """Seeded XA of streams lo..hi-1 of a batch job (seed = 1000 + global
    index, so the job is the same at every N); `bad_stream` gets a gain-5
    profile in its middle eblock (first-error collective test)."""
    from bjxa_amd import synth
    specs = batch_specs(name, nstreams, eblocks)
    out = []
    for i in range(lo, hi):
        bits, ch, eb = specs[i]
        xa = synth.stream(eb, bits, ch, mix, seed=1000 + i)
        if i == bad_stream:
            xa[(eb // 2) * ch * (bits * 4 + 1)] = 0x57
        out.append((i, bits, ch, eb, xa))
    return out


def oracle_batch(inputs, threads, outs=None):
    """Oracle decode of a list of streams on `threads` host threads (one
    decoder per thread, streams round-robin); returns {index: pcm} and the
    seconds it took.  `outs` ({index: int16 array}) are output buffers
    allocated and touched beforehand (pre-fault all buffers --
    fresh ones page-fault inside the timed region, and hundreds of threads
    faulting at once serialise in the kernel)."""
    import oracle
    res = {}

    def work(k):
        for j in range(k, len(inputs), threads):
            i, bits, ch, eb, xa = inputs[j]
            res[i] = oracle.decode(xa, eb, bits, ch, out=None if outs is None else outs[i])
    t = time.perf_counter()
    ths = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return res, time.perf_counter() - t


def cpu_batch_baseline(name, inputs):
    """C4/C5 CPU baseline: the oracle on all usable host cores."""
    threads, aff, online = cpu_threads()
    samples = sum(eb * 32 * ch for _, _, ch, eb, _ in inputs)
    outs = {i: np.ones(eb * 32 * ch, np.int16) for i, _, ch, eb, _ in inputs}
    oracle_batch(inputs, threads, outs)                 # discarded first pass
    times = [oracle_batch(inputs, threads, outs)[1] for _ in range(CPU_PASSES)]
    del outs
    med = float(np.median(times))
    return {"value": round(samples / med / 1e6, 1), "unit": "MSamples/s", "cores": threads,
            "cores_affinity": aff, "cpus_online": online, "cpu_quota_cpus": cpu_quota(),
            "kind": "port",
            "sample": "all %d streams of %s (%d samples), oracle/xa_oracle.c single-pass decode "
                      "(libbjxa's block loop restated, src/libbjxa.c:602-661), one decoder per "
                      "thread on %d threads (%d cores in the affinity mask%s), streams "
                      "round-robin, output buffers pre-faulted, median of %d passes after a "
                      "discarded first; host: %s, %s CPUs online%s"
                      % (len(inputs), name, samples, threads, aff,
                         "; BJXA_CPU_THREADS" if threads < aff else "", CPU_PASSES,
                         host_cpu(), online,
                         "" if cpu_quota() is None else
                         ", cgroup quota %.1f CPUs of time" % cpu_quota())}


def run_batch(name, steps, warmup, dev, verify, nstreams=0, rank=0, world=1, eblocks=0,
              cpu_leg=False, bad_stream=-1, pipeline=1, variant=0):
    """Decode (this rank's share of) a batch config with bjxa_hip_batch_* --
    all streams per launch -- `steps` times after `warmup` untimed steps,
    then time EV_SAMPLES more launches with events.  Returns this rank's
    measurements incl. per-stream checksums and first failing stream."""
    import torch
    import torch.distributed as dist
    import bjxa_amd
    specs = batch_specs(name, nstreams, eblocks)
    lo, hi = shard_range(len(specs), rank, world)
    inputs = batch_inputs(name, nstreams, eblocks, lo, hi, bad_stream)
    # every stream in allocations of its own, as separate callers' buffers
    # are: without this the allocator carves them back to back out of the
    # previous config's cached segments, and same-size streams packed at
    # power-of-two spacing decode up to 30 % slower ("Stream
    # placement")
    torch.cuda.empty_cache()
    srcs = [torch.from_numpy(xa).to(dev) for _, _, _, _, xa in inputs]
    samples = sum(eb * 32 * ch for _, _, ch, eb, _ in inputs)
    alg = sum(xa.nbytes + eb * 64 * ch for _, _, ch, eb, xa in inputs)
    n = len(inputs)

    def make_slot(k):
        dsts = [torch.empty(eb * 64 * ch, dtype=torch.uint8, device=dev)
                for _, _, ch, eb, _ in inputs]
        # slot 0 decodes the callers' inputs, every other slot its own copy
        own = srcs if k == 0 else [s.clone() for s in srcs]
        return {"dsts": dsts, "srcs": own,
                "status": torch.zeros(max(n, 1) * bjxa_amd.STATUS_WORDS, dtype=torch.int32,
                                      device=dev)}
    slots = pipeline_slots(pipeline or 2, dev, make_slot)
    elapsed, spec, serial, depth, cal, step_ms = 0.0, [0.0], 0.0, 1, None, []
    if n:
        with contextlib.ExitStack() as stack:
            for sl in slots:
                desc = [{"d_src": s.data_ptr(), "d_dst": d.data_ptr(), "eblocks": eb,
                         "bits": bits, "channels": ch}
                        for s, d, (_, bits, ch, eb, _) in zip(sl["srcs"], sl["dsts"], inputs)]
                sl["batch"] = stack.enter_context(bjxa_amd.Batch(desc, stream=sl["sh"],
                                                                 variant=variant))
            torch.cuda.synchronize(dev)

            def step(i, ev=(None, None)):
                sl = slots[i % len(slots)]
                sl["batch"].decode(sl["status"].data_ptr(), sl["sh"], ev)
            for i in range(warmup):
                step(i)
            depth, cal = choose_depth(step, len(slots), dev, pipeline)
            elapsed, step_ms = timed_region(step, steps, depth, slots, dev)
            serial = timed_serial(step, steps, dev) if depth > 1 else elapsed
            # kernel timing: slot 0 alone, one launch at a time
            evs = EventPairs(max(EV_SAMPLES, steps))
            for ev in evs.ev:
                step(0, ev)
            spec = evs.ms()
            evs.close()
            torch.cuda.synchronize(dev)
    elif dist_on():
        dist.barrier()
        dist.barrier()
    dsts, status = slots[0]["dsts"], slots[0]["status"]
    spec_ms = float(np.median(spec))
    st = status.cpu().numpy().view(np.uint32).reshape(max(n, 1), -1)[:n]
    # a failed stream counts only the PCM before its failing eblock
    valid = [eb * 32 * ch if int(w[0]) == NO_ERROR else int(w[0]) // ch * 32 * ch
             for (_, _, ch, eb, _), w in zip(inputs, st)]

    def agrees(sl):
        """Slot sl's results equal slot 0's where the API defines them: the
        first error, the PCM before it and, for a clean stream, the exit
        state.  The chunk plan (and with it the repair counts, and the PCM
        and state past an error) may differ between slots: the packed-layout
        plan depends on where each slot's buffers sit."""
        s2 = sl["status"].cpu().numpy().view(np.uint32).reshape(max(n, 1), -1)[:n]
        return all(int(a[0]) == int(w[0]) and (int(w[0]) != NO_ERROR or
                                               tuple(a[1:3]) == tuple(w[1:3])) and
                   torch.equal(x[:2 * v], y[:2 * v])
                   for a, w, x, y, v in zip(s2, st, sl["dsts"], dsts, valid))
    same = all(agrees(sl) for sl in slots[1:])
    sums = [pcm_checksum_torch(d, v) for d, v in zip(dsts, valid)]
    first_err = min([i for (i, *_), w in zip(inputs, st) if int(w[0]) != NO_ERROR],
                    default=FIRST_ERR_NONE)
    ok, ref_sums = None, None
    if verify:
        threads = cpu_threads()[0]
        refs, _ = oracle_batch(inputs, max(1, threads // world))
        ok, ref_sums = same, []
        for (i, bits, ch, eb, xa), d, w in zip(inputs, dsts, st):
            pcm, _, done, _ = refs[i]
            ref_sums.append(pcm_checksum_np(pcm[:done * 32 * ch]))
            if int(w[0]) != NO_ERROR:       # compare up to the failing eblock
                m = done * 32 * ch
                ok = ok and bool(np.array_equal(d.cpu().numpy().view(np.int16)[:m], pcm[:m]))
            elif not np.array_equal(d.cpu().numpy().view(np.int16), pcm):
                ok = False
        del refs
    cpu = cpu_batch_baseline(name, inputs) if cpu_leg else None
    return {"workload": BATCHES.get(name, name), "streams": n, "shard": [lo, hi],
            "samples": samples, "elapsed": elapsed,
            "value": round(samples * steps / elapsed / 1e6, 1) if elapsed else 0.0,
            "unit": "MSamples/s",
            "ms_per_step": round(elapsed / steps * 1e3, 4), "step_ms": spread(step_ms, depth),
            "pipeline": depth, "pipeline_cal": cal,
            "ms_per_step_serial": round(serial / steps * 1e3, 4),
            "spec_ms": round(spec_ms, 4), "spec_samples": len(spec),
            "frac": round(alg / (spec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if spec_ms else 0.0,
            "alg_bytes": alg, "repaired": int(st[:, 3].sum()) if n else 0,
            "tail": int(st[:, 4].sum()) if n else 0, "chunks": int(st[:, 5].sum()) if n else 0,
            "bit_exact": ok, "checksums": sums, "ref_checksums": ref_sums,
            "first_error": first_err, "cpu_baseline": cpu}


def run_encode(steps, warmup, dev, verify, cpu_leg=False):
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
    t0 = time.perf_counter()
    for _ in range(steps):
        bjxa_amd.encode_device(src.data_ptr(), frames, bits, ch, dst.data_ptr(), sh)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    # per-launch kernel time: events around each of EV_SAMPLES launches
    # (encode is one kernel, so torch's events on the same stream suffice),
    # each launch after a 512 MiB read that evicts the 256 MiB Infinity
    # Cache, so no launch reads its 640 MB input partly from the cache
    # (round-2 VERDICT: an isolated launch otherwise times below the trace).
    # A read, not a fill: dirty fill lines would be written back during the
    # launch and charge it for traffic that is not its own.
    flush = torch.ones(128 << 20, dtype=torch.int32, device=dev)
    ms = []
    for i in range(max(EV_SAMPLES, steps)):
        flush.sum()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bjxa_amd.encode_device(src.data_ptr(), frames, bits, ch, dst.data_ptr(), sh)
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    del flush
    med = float(np.median(ms))
    ok, cpu = None, None
    if verify or cpu_leg:
        import oracle
        ref = oracle.encode(pcm, frames, bits, ch)      # also the discarded pass
        ok = bool(np.array_equal(dst.cpu().numpy(), ref))
        if cpu_leg:
            times = []
            for _ in range(CPU_PASSES):
                t = time.perf_counter()
                oracle.encode(pcm, frames, bits, ch)
                times.append(time.perf_counter() - t)
            # (its own name: this median once overwrote the kernel's, so
            # round 2's encode kernel_ms was the CPU time in seconds)
            cpu_s = float(np.median(times))
            cpu = {"value": round(frames * ch / cpu_s / 1e6, 1), "unit": "MSamples/s",
                   "cores": 1, "kind": "port",
                   "sample": "the full C3-shaped PCM (%d samples), oracle/xa_oracle.c "
                             "single-pass encode on 1 thread, median of %d passes after a "
                             "discarded first; host CPU: %s" % (frames * ch, CPU_PASSES,
                                                                  host_cpu())}
        del ref
    alg = pcm.nbytes + nxa
    return {"workload": "encode, C3-shaped: 320M int16 samples (8-bit stereo) -> XA",
            "value": round(frames * ch / dt / 1e6, 1), "unit": "MSamples/s",
            "ms_per_step": round(dt * 1e3, 4), "kernel_ms": round(med, 4),
            "kernel_samples": len(ms),
            "kernel_ms_stat": "median of %d launches, each after a 512 MiB cache-evicting "
                              "read" % len(ms),
            "frac": round(alg / (med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "step_frac": round(alg / dt / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes": alg,
            "byte_exact": ok, "cpu_baseline": cpu}


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


# ---- entry ------------------------------------------------------------------

def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS) + ["C5"],
                    help="default: C3 at N=1 (one stream per rank), C5 at N>1 (the "
                         "1024-stream job split over the ranks)")
    ap.add_argument("--mix", default="A", choices=["A", "F", "W", "Z"])
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--warm-blocks", type=int, default=-1)
    ap.add_argument("--variant", type=lambda v: int(v, 0), default=0,
                    help="tuning variant bits of every decode (include/bjxa_hip.h)")
    ap.add_argument("--streams", type=int, default=0, help="C5 streams (default 1024)")
    ap.add_argument("--eblocks", type=int, default=0, help="C5 eblocks per stream (65,536)")
    ap.add_argument("--bad-stream", type=int, default=-1,
                    help="C5: give this stream a gain-5 profile (first-error collective)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="steps in flight: consecutive steps on this many HIP streams, "
                         "each with its own input copy, output and workspace buffers; "
                         "0 (default) = 1 or 2, whichever a short calibration after the "
                         "warm-up finds faster on this workload and box")
    ap.add_argument("--force-pg", action="store_true",
                    help="join an RCCL process group even at --gpus 1 (the rank starts "
                         "under torch.distributed.run), so the control-plane collectives "
                         "of the N > 1 line execute through librccl on one GPU")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-other", action="store_true",
                    help="skip the other_configs lines")
    ap.add_argument("--only-other", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def other_child(name, args):
    """other_configs[name], measured by a child bench.py (--only-other) in a
    process of its own; the parent has not touched the GPU yet."""
    cmd = [sys.executable, os.path.abspath(__file__), "--only-other", name,
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--mix", args.mix,
           "--pipeline", str(args.pipeline)]
    cmd += ["--no-cpu"] if args.no_cpu else []
    cmd += ["--no-verify"] if args.no_verify else []
    p = subprocess.run(cmd, stdout=subprocess.PIPE)
    if p.returncode != 0:
        raise RuntimeError("bench.py --only-other %s: exit status %d" % (name, p.returncode))
    return json.loads(p.stdout.decode().strip().splitlines()[-1])


def other_configs(args, workload):
    """Every other_configs line at N = 1 beside `workload`'s, each from its
    own child process."""
    names = [n for n in sorted(WORKLOADS) if n != workload] + sorted(BATCHES) + ["encode_C3"]
    return {n: other_child(n, args) for n in names}


def only_other(args):
    """Child side of other_child: one other_configs line on GPU 0."""
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    name, cpu_leg, verify = args.only_other, not args.no_cpu, not args.no_verify
    if name in WORKLOADS:
        o = other_stream_line(run_workload(name, args, dev, 1, 0, verify, cpu_leg), args.steps)
    elif name in BATCHES:
        o = run_batch(name, args.steps, args.warmup, dev, verify, cpu_leg=cpu_leg,
                      variant=args.variant,
                      pipeline=args.pipeline)
        for k in ("checksums", "ref_checksums", "shard"):
            o.pop(k)
        if o["first_error"] == FIRST_ERR_NONE:
            o["first_error"] = None
    elif name == "encode_C3":
        o = run_encode(args.steps, args.warmup, dev, verify, cpu_leg)
    else:
        raise ValueError(name)
    print(json.dumps(o), flush=True)
    return 0


def main():
    args = parse_args()
    if (args.gpus > 1 or args.force_pg) and "WORLD_SIZE" not in os.environ:
        # the parent never touches the GPU: it only starts the ranks
        return launch_ranks(args.gpus)

    import torch
    import torch.distributed as dist

    if args.only_other:
        return only_other(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("BJXA_BENCH_BACKEND", "nccl")
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus), file=sys.stderr)
        return 2
    if backend == "gloo":
        dev = torch.device("cpu")
        if world > 1 or args.force_pg:
            init_pg("gloo")
        return main_c5_cpu(args, dev, world, rank)
    if backend == "gloo-gpu":
        # rehearsal of the N > 1 GPU path on a one-GPU box: every rank
        # decodes its share on GPU 0, the control plane runs over gloo
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        if world > 1:
            init_pg("gloo")
        try:
            return main_c5(args, dev, world, rank, cdev=torch.device("cpu"))
        finally:
            if world > 1:
                dist.destroy_process_group()
    workload = args.workload or ("C3" if world == 1 else "C5")
    # the other configurations first, in child processes, while this one
    # has not touched the GPU
    others = other_configs(args, workload) if (world == 1 and not args.force_pg and
                                               workload in WORKLOADS and
                                               not args.no_other) else None
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.force_pg:
        init_pg("nccl", device_id=dev)
    try:
        if workload == "C5":
            return main_c5(args, dev, world, rank)
        return main_stream(args, workload, dev, world, rank, others)
    finally:
        if dist_on():
            dist.destroy_process_group()


def other_stream_line(o, steps, world=1):
    return {"workload": o["desc"] + (" per rank" if world > 1 else ""),
            "value": round(job_value(o["samples"], world, steps, o["elapsed"]), 1),
            "unit": "MSamples/s", "ms_per_step": round(o["elapsed"] / steps * 1e3, 4),
            "pipeline": o["pipeline"], "pipeline_cal": o["pipeline_cal"],
            "ms_per_step_serial": round(o["serial"] / steps * 1e3, 4),
            "step_ms": o["step_ms"],
            "spec_ms": round(o["spec_ms"], 4), "spec_samples": o["spec_samples"],
            "frac": round(o["alg_bytes"] / (o["spec_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "chunk": int(o["status"][6]), "bit_exact": o["ok"],
            "pcm_equal_oracle": o["pcm_equal_oracle"], "slots_agree": o["slots_agree"],
            "cpu_baseline": o["cpu"]}


def main_stream(args, workload, dev, world, rank, others=None):
    """C3 (or C2): one stream per rank, weak scaling; `others`: the
    other_configs lines (other_configs(), measured before this)."""
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu
    r = run_workload(workload, args, dev, world, rank, not args.no_verify, cpu_leg)
    elapsed, ok = r["elapsed"], r["ok"]
    if dist_on():
        elapsed, ok = reduce_over_ranks(elapsed, ok, dev)

    other = others or {}
    for o in other.values():
        exact = o.get("bit_exact", o.get("byte_exact"))
        ok = ok if exact in (None, True) else False

    st = r["status"]
    achieved = r["alg_bytes"] / (r["spec_ms"] * 1e-3) / 1e9
    read_gbs = r["xa_bytes"] / (r["spec_ms"] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(workload, args.mix)
    line = {
        "metric": METRIC,
        "value": round(job_value(r["samples"], world, args.steps, elapsed), 1),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "ms_per_step_serial": round(r["serial"] / args.steps * 1e3, 4),
        "step_ms": r["step_ms"],
        "cold_single_decode": r["cold"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32+f32",
        "data": "synthetic (seeded XA stream, profile mix %s, uniform codes)" % args.mix,
        "config": {"workload": r["desc"] + " per rank", "workload_id": workload,
                   "bits": r["bits"], "channels": r["ch"],
                   "eblocks_per_rank": r["eb"], "samples_per_rank": r["samples"],
                   "profile_mix": args.mix, "parallelism": "independent streams, 1 per GPU",
                   "chunk": int(st[6]), "warmup_eblocks": int(st[7]),
                   "tuning": "auto" if not args.chunk and args.warm_blocks < 0 else "manual",
                   "pipeline": r["pipeline"], "pipeline_cal": r["pipeline_cal"],
                   **({"recal": r["recal"]} if r.get("recal") else {})},
        "roofline": {"bound": "hbm", "kernel": "xa_decode_spec",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "alg_bytes_per_launch": r["alg_bytes"], "traffic_source": traffic_src,
                     "read_only_achieved": round(read_gbs, 1),
                     "read_only_frac": round(read_gbs / HBM_PEAK_GBS, 4),
                     "launch_ms": round(r["spec_ms"], 4),
                     "launch_ms_stat": "median of %d launches" % r["spec_samples"],
                     "step_frac": round(r["alg_bytes"] / (elapsed / args.steps) / 1e9 /
                                        HBM_PEAK_GBS / world, 4)},
        "cpu_baseline": r["cpu"],
        "bit_exact": ok,
        "repaired_chunks": int(st[3]), "tail_repairs": int(st[4]), "chunks": int(st[5]),
    }
    if other:
        line["other_configs"] = other
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok in (None, True) else 1


def c5_control_plane(r, dev, world, nstreams):
    """SURVEY.md §5 collectives of the batched job: AllReduce(sum) of the
    counters, AllReduce(min) of the first failing stream, AllGather of the
    per-stream PCM checksums (padded shares) -- GPU's and oracle's -- which
    rank 0 compares.  Returns the job-wide view."""
    import torch
    import torch.distributed as dist
    cnt = torch.tensor([r["samples"], r["alg_bytes"], r["repaired"], r["tail"], r["chunks"],
                        r["streams"]], dtype=torch.int64, device=dev)
    fe = torch.tensor([r["first_error"]], dtype=torch.int64, device=dev)
    if dist_on():
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
        dist.all_reduce(fe, op=dist.ReduceOp.MIN)
    width = (nstreams + world - 1) // world
    have_ref = r["ref_checksums"] is not None

    def gather(vals):
        t = torch.zeros(width + 1, dtype=torch.int64, device=dev)
        t[0] = len(vals)
        if vals:
            t[1:1 + len(vals)] = torch.tensor(vals, dtype=torch.int64)
        if not dist_on():
            return [t]
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return parts

    def flat(parts):
        return [int(v) for p in parts for v in p[1:1 + int(p[0])].tolist()]
    sums = flat(gather(r["checksums"]))
    refs = flat(gather(r["ref_checksums"] or [])) if have_ref else None
    shards = gather([r["shard"][0], r["shard"][1]])
    c = [int(v) for v in cnt.tolist()]
    return {"samples": c[0], "alg_bytes": c[1], "repaired": c[2], "tail": c[3],
            "chunks": c[4], "streams": c[5], "first_error": int(fe.item()),
            "checksums": sums, "ref_checksums": refs,
            "shards": [[int(p[1]), int(p[2])] for p in shards]}


def checksum_report(job):
    """Digest of the gathered checksum vector and rank 0's comparison."""
    import hashlib
    h = hashlib.sha1(np.array(job["checksums"], dtype=np.int64).tobytes()).hexdigest()
    match = None
    if job["ref_checksums"] is not None:
        match = job["checksums"] == job["ref_checksums"]
    return h, match


def main_c5(args, dev, world, rank, cdev=None):
    """C5: the fixed job of 1024 8-bit stereo streams (65,536 eblocks each)
    split over the ranks -- strong scaling, no data-path collective.  `cdev`:
    the device of the control-plane tensors (the GPU under RCCL, the CPU
    under gloo)."""
    cdev = cdev or dev
    nstreams = args.streams or 1024
    r = run_batch("C5", args.steps, args.warmup, dev, not args.no_verify, nstreams, rank,
                  world, args.eblocks, bad_stream=args.bad_stream, pipeline=args.pipeline)
    elapsed, ok = r["elapsed"], r["bit_exact"]
    if dist_on():
        elapsed, ok = reduce_over_ranks(elapsed, ok, cdev)
    job = c5_control_plane(r, cdev, world, nstreams)
    digest, match = checksum_report(job)
    if match is False:
        ok = False
    # per-rank kernel times for the report
    import torch
    import torch.distributed as dist
    lm = torch.tensor([r["spec_ms"], r["frac"]], dtype=torch.float64, device=cdev)
    parts = [torch.zeros_like(lm) for _ in range(world)]
    if dist_on():
        dist.all_gather(parts, lm)
    else:
        parts = [lm]
    per_rank = [[round(float(p[0]), 4), round(float(p[1]), 4)] for p in parts]

    other = {}
    if not args.no_other and world > 1:
        o = run_workload("C3", args, dev, world, rank, not args.no_verify, False)
        el, ok3 = reduce_over_ranks(o["elapsed"], o["ok"], cdev)
        o["elapsed"] = el
        o["ok"] = ok3
        other["C3_weak"] = other_stream_line(o, args.steps, world)
        ok = ok if ok3 in (None, True) else False

    spec_ms = r["spec_ms"]
    line = {
        "metric": METRIC,
        "value": round(job["samples"] * args.steps / elapsed / 1e6, 1), "unit": "MSamples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "ms_per_step_serial": r["ms_per_step_serial"], "step_ms": r["step_ms"],
        "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "int32+f32",
        "data": "synthetic (seeded XA streams, profile mix A, uniform codes)",
        "config": {"workload": BATCHES["C5"] if not (args.streams or args.eblocks) else
                   "C5-shaped: %d 8-bit stereo streams of %d eblocks, a contiguous share "
                   "per rank" % (nstreams, batch_specs("C5", nstreams, args.eblocks)[0][2]),
                   "workload_id": "C5", "streams": job["streams"],
                   "streams_per_rank": [hi - lo for lo, hi in job["shards"]],
                   "parallelism": "stream shards, one batched launch per GPU, RCCL control "
                                  "plane only", "pipeline": r["pipeline"],
                   "pipeline_cal": r["pipeline_cal"],
                   "scaling_n1_ref": "other_configs.C5 of the N = 1 line (python bench.py): "
                                     "this same job on one GPU, the first point of the "
                                     "strong-scaling curve (the N = 1 headline itself is "
                                     "C3, one stream)"},
        "roofline": {"bound": "hbm", "kernel": "xa_decode_spec_batch (rank 0)",
                     "achieved": round(r["alg_bytes"] / (spec_ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": r["frac"],
                     "traffic": None, "alg_bytes_per_launch": r["alg_bytes"],
                     "launch_ms": spec_ms,
                     "launch_ms_stat": "median of %d launches" % r["spec_samples"],
                     "per_rank_launch_ms_frac": per_rank},
        "cpu_baseline": None, "bit_exact": ok,
        "control_plane": {"shards": job["shards"], "samples": job["samples"],
                          "repaired_chunks": job["repaired"], "tail_repairs": job["tail"],
                          "first_error_stream": None if job["first_error"] >= FIRST_ERR_NONE
                          else job["first_error"],
                          "checksums_sha1": digest, "checksums_match_oracle": match,
                          "backend": dist.get_backend() if dist_on() else None},
    }
    if other:
        line["other_configs"] = other
    if cdev.type != dev.type:
        line["device"] = ("rehearsal: all %d ranks share GPU 0 (control plane over gloo); "
                          "the times are not a scaling measurement" % world)
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok in (None, True) else 1


def main_c5_cpu(args, dev, world, rank):
    """CPU rehearsal of the N > 1 path (gloo): this rank's share of a small
    C5-shaped job decoded with the library's host API (its CPU core), then
    the same control plane as main_c5."""
    import torch.distributed as dist
    import bjxa_amd
    nstreams = args.streams or 16
    eblocks = args.eblocks or 1000
    specs = batch_specs("C5", nstreams, eblocks)
    lo, hi = shard_range(len(specs), rank, world)
    inputs = batch_inputs("C5", nstreams, eblocks, lo, hi, args.bad_stream)
    stall_for_test(rank)
    if dist_on():
        dist.barrier()
    t0 = time.perf_counter()
    first_err, pcms = FIRST_ERR_NONE, {}
    with bjxa_amd.offload(None):
        for _ in range(args.steps):
            for i, bits, ch, eb, xa in inputs:
                pcm = np.zeros(eb * 32 * ch, np.int16)
                with bjxa_amd.Decoder() as d:
                    d.parse_header(bjxa_amd.xa_header(xa.size, eb * 32, 44100, bits, ch))
                    try:
                        d.decode(pcm, xa)
                        pcms[i] = pcm
                    except bjxa_amd.BjxaError:
                        # the PCM before the failing eblock (none past it)
                        first_err = min(first_err, i)
                        bad = next(b for b in range(eb) if any(
                            xa[(b * ch + c) * (bits * 4 + 1)] >= 0x50 for c in range(ch)))
                        pcms[i] = pcm[:bad * 32 * ch]
    elapsed = time.perf_counter() - t0
    sums = [pcm_checksum_np(pcms[i]) for i, *_ in inputs]
    ok, refs = None, None
    if not args.no_verify:
        ref, _ = oracle_batch(inputs, 1)
        refs = [pcm_checksum_np(ref[i][0][:ref[i][2] * 32 * ch]) for i, bits, ch, eb, xa in inputs]
        ok = sums == refs
    if dist_on():
        elapsed, ok = reduce_over_ranks(elapsed, ok, dev)
    samples = sum(eb * 32 * ch for _, _, ch, eb, _ in inputs)
    r = {"samples": samples, "alg_bytes": 0, "repaired": 0, "tail": 0, "chunks": 0,
         "streams": len(inputs), "first_error": first_err, "checksums": sums,
         "ref_checksums": refs, "shard": [lo, hi]}
    job = c5_control_plane(r, dev, world, nstreams)
    digest, match = checksum_report(job)
    if match is False:
        ok = False
    line = {"metric": METRIC, "value": round(job["samples"] * args.steps / elapsed / 1e6, 1),
            "unit": "MSamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "int32", "data": "synthetic (seeded XA streams, profile mix A)",
            "device": "cpu (gloo rehearsal of the RCCL path; library host API on its CPU core)",
            "backend": dist.get_backend() if dist_on() else None,
            "config": {"workload": "C5-shaped: %d streams of %d eblocks" % (nstreams, eblocks),
                       "workload_id": "C5", "streams": job["streams"],
                       "streams_per_rank": [b - a for a, b in job["shards"]]},
            "bit_exact": ok,
            "control_plane": {"shards": job["shards"], "samples": job["samples"],
                              "first_error_stream": None if job["first_error"] >= FIRST_ERR_NONE
                              else job["first_error"],
                              "checksums_sha1": digest, "checksums_match_oracle": match}}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on():
        dist.destroy_process_group()
    return 0 if ok in (None, True) else 1


def main_named():
    """main(), with a failure of this rank (a collective that timed out, a
    peer that died) reported under its rank before the exit status."""
    try:
        return main()
    except Exception as e:  # noqa: BLE001 -- report, then fail the job
        print("bench.py rank %s: %s: %s" % (os.environ.get("RANK", "0"), type(e).__name__, e),
              file=sys.stderr, flush=True)
        return 3


if __name__ == "__main__":
    sys.exit(main_named())
