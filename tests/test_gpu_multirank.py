"""bench.py's N-rank path rehearsed on one GPU (the driver's 8-GPU scaling run uses the same code).

Plain `bench.py --gpus 2` (the driver's form) starts a child torch.distributed.run with two ranks
before any GPU call; with more ranks than visible devices they share the GPU and use gloo for the
timing collectives (RCCL needs a device per rank).  Each
rank processes the frames of its own seed; the test then runs each rank's workload alone
(`--seed-rank r`) and requires bit-identical outputs, and checks that the aggregate rate counts
the work of both ranks over the max-over-ranks time.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--points", "8192", "--batch", "4", "--steps", "6", "--warmup", "1", "--rotate", "3", "--no-extras",
        "--no-density", "--no-cpu-baseline", "--no-fp32-mfma-leg", "--no-standalone"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_bench_two_ranks_on_one_gpu(cuda, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", *ARGS, "--dump", str(tmp_path / "w2"),
           "--detail", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["steps"] == 6
    assert line["distributed"]["world_size"] == 2 and len(line["distributed"]["ranks"]) == 2
    assert len(r.stdout.strip().splitlines()[-1]) <= 4096
    # whole-job rate: both ranks' frames over the max-over-ranks window
    per_rank_points = 4 * 8192 * 6
    assert abs(line["value"] - 2 * per_rank_points / (line["ms_per_step"] * 6 / 1e3) / 1e6) <= 1e-6 * line["value"]
    for rank in (0, 1):
        w2 = json.load(open(tmp_path / f"w2.rank{rank}.json"))
        assert w2["world"] == 2 and w2["seed_rank"] == rank
        r1 = subprocess.run([sys.executable, "bench.py", *ARGS, "--seed-rank", str(rank), "--dump",
                             str(tmp_path / f"w1_{rank}")], cwd=REPO, env=env, capture_output=True, text=True,
                            timeout=300)
        assert r1.returncode == 0, r1.stderr[-4000:]
        w1 = json.load(open(tmp_path / f"w1_{rank}.rank0.json"))
        assert w1["world"] == 1 and w1["seed_rank"] == rank
        assert w2["digests"] == w1["digests"], f"rank {rank}: outputs differ from its 1-rank run"
    assert json.load(open(tmp_path / "w2.rank0.json"))["digests"] != json.load(open(tmp_path / "w2.rank1.json"))["digests"]


ARGS_C3 = ["--batch", "32", "--points", "65536", "--steps", "4", "--warmup", "1", "--rotate", "4", "--no-extras",
           "--no-density", "--no-cpu-baseline", "--no-fp32-mfma-leg", "--no-standalone"]


@pytest.mark.timeout(900)
def test_bench_configs3_eight_ranks_on_one_gpu(cuda, tmp_path):
    """BASELINE configs[3] (256 x 65 536-point frames sharded per frame over 8 GPUs, no collectives) at
    its real shape through plain `bench.py --gpus 8`: eight ranks of 32 frames each share the one GPU
    (gloo for the timing collectives).  The line reports world 8 and 256 frames per step over the ranks,
    its value is the whole job's points over the max-over-ranks window, and ranks 0 and 7 compute exactly
    what their own frames give in a 1-rank run (`--seed-rank`).  A rehearsal of the 8-GPU code path, not
    a scaling measurement (the ranks share one GPU)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "8", *ARGS_C3, "--dump", str(tmp_path / "w8"),
           "--detail", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = _last_json(r.stdout)
    steps = 4
    assert line["n_gpus"] == 8 and line["steps"] == steps
    assert line["config"]["global_batch_frames"] == 256 and line["config"]["frames_per_gpu"] == 32
    d = line["distributed"]
    assert d["world_size"] == 8 and sorted(row[0] for row in d["ranks"]) == list(range(8))
    assert sum(row[2] for row in d["ranks"]) == 256 * steps  # every rank's 32 frames per step
    assert abs(line["value"] - 8 * 32 * 65536 * steps / (line["ms_per_step"] * steps / 1e3) / 1e6) \
        <= 1e-6 * line["value"]
    # the window is the max over ranks: no rank's own window is longer
    assert max(row[3] for row in d["ranks"]) <= line["ms_per_step"] * steps * (1 + 1e-3)  # (4 digits in the line)
    for rank in (0, 7):
        w8 = json.load(open(tmp_path / f"w8.rank{rank}.json"))
        assert w8["world"] == 8 and w8["seed_rank"] == rank
        r1 = subprocess.run([sys.executable, "bench.py", *ARGS_C3, "--seed-rank", str(rank), "--dump",
                             str(tmp_path / f"w1_{rank}")], cwd=REPO, env=env, capture_output=True, text=True,
                            timeout=300)
        assert r1.returncode == 0, r1.stderr[-4000:]
        w1 = json.load(open(tmp_path / f"w1_{rank}.rank0.json"))
        assert w1["world"] == 1 and w1["seed_rank"] == rank
        assert w8["digests"] == w1["digests"], f"rank {rank}: outputs differ from its 1-rank run"
    assert json.load(open(tmp_path / "w8.rank0.json"))["digests"] != json.load(open(tmp_path / "w8.rank7.json"))["digests"]


ARGS_C4 = ["--batch", "4", "--points", "8192", "--steps", "3", "--warmup", "1", "--rotate", "2", "--msg-batch", "32",
           "--msg-steps", "3", "--no-density", "--no-cpu-baseline", "--no-fp32-mfma-leg", "--no-standalone",
           "--no-host-feed"]


@pytest.mark.timeout(900)
def test_bench_configs4_eight_ranks_on_one_gpu(cuda, tmp_path):
    """BASELINE configs[4] (the MSG bf16 stack on 131 072-point frames over 8 GPUs) through bench.py's
    8-rank path on the one GPU: its MSG leg runs 32 frames of that shape per rank (the per-GPU share of
    256); ranks 0 and 7 compute exactly what their own frames give in a 1-rank run.  A rehearsal of the
    8-GPU code path (the ranks share one GPU), not a scaling measurement."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "8", *ARGS_C4, "--dump", str(tmp_path / "w8"),
           "--detail", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=800)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 8 and line["distributed"]["world_size"] == 8
    msg = json.load(open(tmp_path / "detail.json"))["other_configs"]["configs[4]_msg_131k_bf16"]
    assert msg["frames_per_gpu"] == 32 and msg["points_per_frame"] == 131072
    key = "configs[4]_msg_131k_bf16"
    for rank in (0, 7):
        w8 = json.load(open(tmp_path / f"w8.rank{rank}.json"))
        assert w8["world"] == 8 and key in w8["digests"]
        r1 = subprocess.run([sys.executable, "bench.py", *ARGS_C4, "--seed-rank", str(rank), "--dump",
                             str(tmp_path / f"w1_{rank}")], cwd=REPO, env=env, capture_output=True, text=True,
                            timeout=400)
        assert r1.returncode == 0, r1.stderr[-4000:]
        w1 = json.load(open(tmp_path / f"w1_{rank}.rank0.json"))
        assert w8["digests"][key] == w1["digests"][key], f"rank {rank}: MSG outputs differ from its 1-rank run"
    assert json.load(open(tmp_path / "w8.rank0.json"))["digests"][key] != \
        json.load(open(tmp_path / "w8.rank7.json"))["digests"][key]
