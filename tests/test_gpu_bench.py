"""bench.py's C5 line on the GPU (the driver's N > 1 headline, here at one
rank): a small C5-shaped job through the batched kernels, the per-stream
checksums compared with the oracle's, and the first-error stream."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def _bench(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, env=env, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_c5_line_one_gpu(built):
    rc, line, err = _bench(["--workload", "C5", "--streams", "24", "--eblocks", "3000",
                            "--steps", "3", "--warmup", "1", "--no-other", "--no-cpu"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    assert line["config"]["workload_id"] == "C5" and line["config"]["streams"] == 24
    assert line["bit_exact"] is True
    cp = line["control_plane"]
    assert cp["checksums_match_oracle"] is True and cp["first_error_stream"] is None
    assert cp["shards"] == [[0, 24]]
    assert line["roofline"]["launch_ms"] > 0 and line["value"] > 0


def test_bench_c5_first_error_one_gpu(built):
    rc, line, err = _bench(["--workload", "C5", "--streams", "12", "--eblocks", "2000",
                            "--steps", "2", "--warmup", "1", "--no-other", "--no-cpu",
                            "--bad-stream", "7"])
    assert rc == 0, err[-2000:]
    assert line["control_plane"]["first_error_stream"] == 7
    assert line["control_plane"]["checksums_match_oracle"] is True
    assert line["bit_exact"] is True


def test_bench_c5_two_ranks_shared_gpu(built):
    """The N > 1 path of bench.py on one GPU: `--gpus 2` starts its own two
    ranks, each decodes its share of the job with the batched kernels on
    GPU 0, and the control plane (gloo here, RCCL on a node) gathers the
    checksums, the first failing stream and the per-rank C3 lines."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BJXA_BENCH_BACKEND"] = "gloo-gpu"
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--workload", "C5", "--streams", "20", "--eblocks", "3000",
                        "--steps", "3", "--warmup", "1", "--no-cpu", "--bad-stream", "13"],
                       capture_output=True, text=True, env=env, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, r.stderr[-3000:]
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert "rehearsal" in line["device"]
    cp = line["control_plane"]
    assert cp["shards"] == [[0, 10], [10, 20]]
    assert cp["first_error_stream"] == 13
    assert cp["checksums_match_oracle"] is True and line["bit_exact"] is True
    c3 = line["other_configs"]["C3_weak"]
    assert c3["bit_exact"] is True and c3["value"] > 0
    assert c3["pcm_equal_oracle"] is True and c3["slots_agree"] is True


def test_bench_c5_three_ranks_shared_gpu(built):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BJXA_BENCH_BACKEND"] = "gloo-gpu"
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "3",
                        "--workload", "C5", "--streams", "17", "--eblocks", "2500",
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--no-other"],
                       capture_output=True, text=True, env=env, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, r.stderr[-3000:]
    line = json.loads(lines[-1])
    assert line["n_gpus"] == 3
    assert line["control_plane"]["shards"] == [[0, 5], [5, 11], [11, 17]]
    assert line["control_plane"]["first_error_stream"] is None
    assert line["control_plane"]["checksums_match_oracle"] is True
    assert line["bit_exact"] is True


def test_bench_default_line_c3(built):
    """The driver's N = 1 headline path (C3, main_stream) end to end: the
    full stream, bit-exact against the oracle, roofline and its fields."""
    rc, line, err = _bench(["--steps", "3", "--warmup", "1", "--no-other", "--no-cpu"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 1 and line["config"]["workload_id"] == "C3"
    assert line["bit_exact"] is True and line["value"] > 0
    rf = line["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["achieved"] > 0
    assert "device" not in line
    # --pipeline 0 (default): the calibration picks one or two in flight
    cfg = line["config"]
    assert cfg["pipeline"] in (1, 2) and line["ms_per_step_serial"] > 0
    cal = cfg["pipeline_cal"]
    assert set(cal) == {"depth1_ms", "depth2_ms", "runs_ms"}
    # two in flight only when every run of them beats every run one at a
    # time by the margin
    runs = cal["runs_ms"]
    assert len(runs["depth1"]) == len(runs["depth2"]) >= 3
    two = max(runs["depth2"]) < min(runs["depth1"]) * (1 - 0.01) - 1e-4
    one = max(runs["depth2"]) > min(runs["depth1"]) * (1 - 0.01) + 1e-4
    assert (cfg["pipeline"] == 2) if two else (cfg["pipeline"] == 1) if one else True


def test_bench_pipeline_slots_agree(built):
    """Three steps in flight on three HIP streams: every slot's PCM and
    status must equal slot 0's, which is checked against the oracle."""
    rc, line, err = _bench(["--workload", "C5", "--streams", "16", "--eblocks", "4000",
                            "--steps", "7", "--warmup", "2", "--no-other", "--no-cpu",
                            "--pipeline", "3"])
    assert rc == 0, err[-2000:]
    assert line["config"]["pipeline"] == 3 and line["bit_exact"] is True
    assert line["control_plane"]["checksums_match_oracle"] is True
    rc, line, err = _bench(["--workload", "C2", "--steps", "5", "--warmup", "1", "--no-other",
                            "--no-cpu", "--pipeline", "3"])
    assert rc == 0, err[-2000:]
    assert line["config"]["pipeline"] == 3 and line["bit_exact"] is True


def test_bench_c5_rccl_one_rank(built):
    """The N > 1 line's control plane through librccl on a one-GPU box:
    `--gpus 1 --force-pg` starts one rank under torch.distributed.run, which
    joins an `nccl` (RCCL) process group bound to its device, so the
    barriers, the AllReduce(max/min/sum) of the timed region, the counters
    and the first failing stream, and the AllGather of the per-stream
    checksums all execute through RCCL on device tensors -- the exact calls
    the driver's 8-GPU run makes first (round-2 VERDICT, missing #1)."""
    rc, line, err = _bench(["--gpus", "1", "--force-pg", "--workload", "C5",
                            "--streams", "24", "--eblocks", "3000", "--steps", "3",
                            "--warmup", "1", "--no-other", "--no-cpu", "--bad-stream", "17"])
    assert rc == 0, err[-3000:]
    assert line["n_gpus"] == 1 and line["scaling"] == "strong"
    cp = line["control_plane"]
    assert cp["backend"] == "nccl"
    assert cp["first_error_stream"] == 17
    assert cp["checksums_match_oracle"] is True and line["bit_exact"] is True
    assert cp["shards"] == [[0, 24]]
    assert "device" not in line


@pytest.mark.parametrize("name", ["C5g", "encode_C3"])
def test_bench_other_config_child(built, name):
    """The child side of other_configs (bench.py --only-other): one line,
    measured in its own process, bit-exact against the oracle."""
    rc, line, err = _bench(["--only-other", name, "--steps", "3", "--warmup", "1",
                            "--no-cpu"])
    assert rc == 0, err[-2000:]
    if name == "C5g":
        assert line["bit_exact"] is True and line["streams"] == 128
        assert line["first_error"] is None and 0 < line["spec_ms"] < line["ms_per_step"] * 2
    else:
        assert line["byte_exact"] is True
