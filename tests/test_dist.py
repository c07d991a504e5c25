"""The multi-GPU bench path on CPU: world_size 2 over gloo.

bench.py shards by stream (every rank decodes its own seeded stream, no
data-path collective) and reduces only the timed region (max) and the
bit-exact flags (AND) across ranks.  These tests run that reduction and the
per-rank workload derivation in two gloo processes.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from bjxa_amd import synth
        dev = torch.device("cpu")
        # rank r times 1.0 + r seconds; rank 1 fails its check in round 2
        t, ok = bench.reduce_over_ranks(1.0 + rank, True, dev)
        t2, ok2 = bench.reduce_over_ranks(0.5, rank != 1, dev)
        t3, ok3 = bench.reduce_over_ranks(0.25, None, dev)
        # each rank's stream: C3-shaped, seeded by rank
        xa = synth.stream(1000, 8, 2, "A", seed=rank)
        h = int(np.bitwise_xor.reduce(xa.view(np.uint64)))
        ht = torch.tensor([h & 0x7fffffffffffffff], dtype=torch.int64)
        hs = [torch.zeros_like(ht) for _ in range(world)]
        dist.all_gather(hs, ht)
        q.put((rank, t, ok, t2, ok2, t3, ok3, [int(x.item()) for x in hs]))
    finally:
        dist.destroy_process_group()


def test_bench_reduction_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, ok, t2, ok2, t3, ok3, hs in res:
        assert t == 2.0 and ok is True          # max over ranks
        assert t2 == 0.5 and ok2 is False       # one failing rank fails the job
        assert ok3 is None                       # unchecked stays unchecked
        assert hs[0] != hs[1]                   # ranks decode different streams


def test_py_median():
    """bench.py's calibration median (plain Python, so that no numpy call
    runs between the calibration and the timed loops) equals numpy's."""
    import bench
    rng = np.random.default_rng(3)
    for n in (1, 2, 3, 4, 7, 8):
        v = list(rng.random(n))
        assert bench.py_median(v) == pytest.approx(float(np.median(v)))


def test_choose_depth_calls_no_numpy(monkeypatch):
    """choose_depth ends right before the timed window, so it must not call
    numpy (a first numpy call pauses the host and idles the GPU, DESIGN.md
    §5 R5-2): run it on CPU with numpy's reductions made to fail."""
    import bench

    def boom(*a, **k):
        raise AssertionError("numpy called in choose_depth")
    for name in ("median", "mean", "percentile", "min", "max", "sort"):
        monkeypatch.setattr(bench.np, name, boom)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    calls = []
    depth, cal = bench.choose_depth(lambda i: calls.append(i), 2, torch.device("cpu"), 0)
    assert depth in (1, 2) and len(calls) == 2 * bench.PIPE_CAL_ROUNDS * 2 * bench.PIPE_CAL_STEPS
    assert len(cal["runs_ms"]["depth1"]) == bench.PIPE_CAL_ROUNDS


def test_job_value_weak_scaling():
    import bench
    # 2 ranks x 320M samples x 20 steps in 10 ms
    assert bench.job_value(320_000_000, 2, 20, 0.01) == pytest.approx(1.28e6)
    # per-GPU work fixed: doubling ranks at equal time doubles the value
    assert bench.job_value(1, 4, 1, 1.0) == 2 * bench.job_value(1, 2, 1, 1.0)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_c5_shards_cover_the_job(world):
    """bench.py --workload C5: the ranks' contiguous shares of the 1024
    streams are disjoint, cover them all, and differ by at most one."""
    import bench
    n = len(bench.batch_specs("C5"))
    assert n == 1024
    got = [bench.shard_range(n, r, world) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(got, got[1:]))
    sizes = [hi - lo for lo, hi in got]
    assert max(sizes) - min(sizes) <= 1


def _neutral(xa, bits, ch):
    """the stream with every gain nibble >= 5 cleared (what a speculative
    warm-up through a bad block amounts to: the kernels decode it with K = 0)"""
    x = xa.copy().reshape(-1, bits * 4 + 1)
    bad = x[:, 0] >= 0x50
    x[bad, 0] &= 0x0F
    return x.reshape(-1)


def _split_worker(rank, world, port, q, eb, bits, ch, mix, warmup, frames, init, bad):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from bjxa_amd import dist as bdist
        xa = _split_stream(eb, bits, ch, mix, bad)
        ebsz = (bits * 4 + 1) * ch
        lo, hi = bdist.split_ranges(eb, world)[rank]
        out = {}
        calls = []

        def local_decode(first, state):
            calls.append(first)
            st = state
            if first < lo:
                w = _neutral(xa[first * ebsz:lo * ebsz], bits, ch)
                _, st, _, _ = oracle.decode(w, lo - first, bits, ch, state)
            fr = min(frames, hi * 32) - lo * 32
            pcm, ex, done, badc = oracle.decode(xa[lo * ebsz:hi * ebsz].copy(), hi - lo, bits,
                                                ch, st, fr)
            out["pcm"] = pcm
            if done < hi - lo:
                return st, ex, (lo + done) * ch + badc
            return st, ex

        fin, fbad = bdist.resolve(local_decode, lo, hi, init, warmup)
        q.put((rank, out["pcm"].tobytes(), fin, len(calls), fbad))
    finally:
        dist.destroy_process_group()


def _split_stream(eb, bits, ch, mix, bad):
    """seeded stream; `bad` = (eblock, channel) gets gain nibble 5"""
    from bjxa_amd import synth
    xa = synth.stream(eb, bits, ch, mix, seed=77)
    if bad is not None:
        xa[(bad[0] * ch + bad[1]) * (bits * 4 + 1)] = 0x53
    return xa


@pytest.mark.parametrize("world,eb,bits,ch,mix,warmup,bad", [
    (2, 3000, 8, 2, "A", 8, None), (3, 3001, 6, 1, "W", 2, None),
    (3, 4000, 4, 2, "W", 0, None), (3, 10, 8, 2, "A", 8, None),
    (3, 3000, 8, 2, "W", 8, (1500, 1)), (3, 3000, 8, 2, "A", 8, (1000, 0)),
    (2, 3001, 6, 1, "W", 8, (1505, 0)), (2, 3001, 6, 1, "W", 8, (1495, 0)),
    (3, 3000, 4, 2, "A", 8, (2999, 1))])
def test_single_stream_split(world, eb, bits, ch, mix, warmup, bad):
    """bjxa_amd.dist.resolve: a stream split over ranks, each decoding its
    range speculatively (warm-up from (0,0)) and re-decoding when the
    all-gathered chain of states says its entry was wrong, equals the
    single-pass decode; ranges shorter than the warm-up start at eblock 0.
    With a bad profile the result is the reference's first-bad-block
    outcome: its index, the carried state (a bad right block leaves the
    left channel advanced), and the PCM before it -- including a bad block
    at the first eblock of a range or inside the next rank's warm-up."""
    import oracle
    frames = eb * 32 - 5
    init = (11, -22, 33, -44) if ch == 2 else (11, -22, 0, 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q, eb, bits, ch, mix,
                                                       warmup, frames, init, bad))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xa = _split_stream(eb, bits, ch, mix, bad)
    ref, st_ref, done, badc = oracle.decode(xa, eb, bits, ch, init, frames)
    for r in res:
        assert tuple(r[2])[:2 * ch] == tuple(st_ref)[:2 * ch]
    joined = b"".join(r[1] for r in res)
    if bad is None:
        assert joined == ref.tobytes()
        assert all(r[4] is None for r in res)
    else:
        assert done == bad[0] and badc == bad[1]
        n = done * 32 * ch * 2
        assert joined[:n] == ref.tobytes()[:n]
        assert all(r[4] == bad[0] * ch + bad[1] for r in res)
    if mix == "W" and eb > 100 and bad is None:
        assert any(r[3] > 1 for r in res)      # some rank had to re-decode


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(BJXA_BENCH_BACKEND="gloo", HIP_VISIBLE_DEVICES="-1")
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, env=env, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("world,streams", [(2, 7), (3, 8)])
def test_bench_launcher_spawns_ranks(world, streams):
    """`bench.py --gpus N` with no WORLD_SIZE starts N ranks itself (child
    torch.distributed.run, same code path as on the GPU box but over gloo):
    the line reports n_gpus == N, the shards tile the job, and the
    AllGather'ed per-stream checksums match the oracle's on rank 0."""
    rc, line, err = _bench(["--gpus", str(world), "--streams", str(streams), "--eblocks", "300",
                            "--steps", "1", "--warmup", "0"])
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == world and line["scaling"] == "strong"
    cp = line["control_plane"]
    shards = cp["shards"]
    assert len(shards) == world and shards[0][0] == 0 and shards[-1][1] == streams
    assert all(a[1] == b[0] for a, b in zip(shards, shards[1:]))
    assert line["config"]["streams"] == streams
    assert cp["samples"] == streams * 300 * 64
    assert line["bit_exact"] is True and cp["checksums_match_oracle"] is True
    assert cp["first_error_stream"] is None


def test_bench_first_error_collective():
    """AllReduce(min) of the first failing stream: stream 5 of 8 carries a
    gain-5 profile; every stream's checksum (the failed one's up to its
    failing eblock) still matches the oracle's."""
    rc, line, err = _bench(["--gpus", "2", "--streams", "8", "--eblocks", "200",
                            "--steps", "1", "--warmup", "0", "--bad-stream", "5"])
    assert rc == 0, err[-3000:]
    assert line["control_plane"]["first_error_stream"] == 5
    assert line["control_plane"]["checksums_match_oracle"] is True


def test_bench_world_mismatch():
    """A rank whose WORLD_SIZE disagrees with --gpus refuses to report."""
    rc, line, err = _bench(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert rc == 2 and line is None and "WORLD_SIZE=1" in err


def test_bench_stuck_rank_times_out():
    """A rank that stops answering (BJXA_BENCH_STALL_RANK: rank 1 sleeps
    before its first collective) fails the job within the process group's
    timeout (BJXA_BENCH_PG_TIMEOUT, 180 s by default), with the rank that
    gave up named, instead of waiting torch's default 10 minutes."""
    import time
    t = time.time()
    rc, line, err = _bench(["--gpus", "2", "--streams", "4", "--eblocks", "100",
                            "--steps", "1", "--warmup", "0"],
                           {"BJXA_BENCH_PG_TIMEOUT": "5", "BJXA_BENCH_STALL_RANK": "1",
                            "BJXA_BENCH_STALL_S": "90"}, timeout=200)
    assert rc != 0 and line is None
    assert time.time() - t < 80
    assert "bench.py rank 0:" in err


def test_bench_force_pg_one_rank():
    """`--gpus 1 --force-pg` starts one rank under torch.distributed.run and
    joins a process group at world size 1, so the control plane's
    collectives run through the backend (gloo here, RCCL on the GPU box:
    tests/test_gpu_bench.py) instead of being skipped."""
    rc, line, err = _bench(["--gpus", "1", "--force-pg", "--streams", "6", "--eblocks", "250",
                            "--steps", "1", "--warmup", "0", "--bad-stream", "4"])
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 1 and line["backend"] == "gloo"
    cp = line["control_plane"]
    assert cp["shards"] == [[0, 6]] and cp["first_error_stream"] == 4
    assert cp["checksums_match_oracle"] is True and line["bit_exact"] is True
